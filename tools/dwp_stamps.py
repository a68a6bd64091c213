#!/usr/bin/env python3
"""Per-phase cycle stamps of the PPO loss side's kernels (diagnostic; a -DLL_STAMP=1 build as
TRLX_T5_AMD_LIB): one PPOHotPath.policy_loss_from_hidden at the C2 / C3 shape, then the
s_memtime sums the kernels left in g_ll_stamps, per wave per tile:
  forward (16x16 form, ll_fwd16_block): wait + barrier, S loop (+ softmax, DMA), O loop (+ P store)
  dW (k_lmloss_dwp or k_lmloss_dw): wait + barrier, [dW: Sᵀ phase, dS tail,] dW phase

  TRLX_T5_AMD_LIB=stamp/lib_stamp.so python tools/dwp_stamps.py [--config c2] [--tune lmloss_dw=1]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--tune", action="append", default=[])
    args = ap.parse_args()
    import torch
    import __graft_entry__
    from lossside_bench import SHAPES
    P = __graft_entry__.load_package()
    lib = P.load_library()
    for kv in args.tune:
        k, v = kv.split("=")
        P._lib.set_tuning(k, int(v))
    B, T, V, H, masked = SHAPES[args.config]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    f = dict(generator=g, device=dev)
    h = torch.randn(B, T, H, **f).to(torch.bfloat16)
    w = (torch.randn(V, H, **f) * 0.05).to(torch.bfloat16)
    labels = torch.randint(0, V, (B, T), **f)
    old_values = torch.randn(B, T, **f)
    values = old_values + 0.3 * torch.randn(B, T, **f)
    scores = torch.rand(B, **f) * 24 - 12
    lengths = mask = None
    if masked:
        lengths = torch.randint(1, T + 1, (B,), **f)
        mask = (torch.arange(T, device=dev)[None, :] < lengths[:, None]).long()
    hp = P.PPOHotPath(P.PPOConfig(), B, T, V, torch.bfloat16, dev, kl_coef=0.05)
    hp.experience_from_hidden(h, w, h, w, labels, old_values, scores, lengths=lengths, mask=mask, route="fused")
    hp.policy_loss_from_hidden(h, w, labels, values, old_values, mask=mask)
    torch.cuda.synchronize()
    hp.policy_loss_from_hidden(h, w, labels, values, old_values, mask=mask)
    torch.cuda.synchronize()
    buf = np.zeros(1 << 16, dtype=np.uint64)
    lib.trlx_debug_ll_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    assert lib.trlx_debug_ll_stamps(buf.ctypes.data, buf.size) == 0
    out = {"config": args.config, "tune": args.tune}
    for name, reg, cols in (("fwd", buf[:1 << 15], ["wait+barrier", "S_loop", "O_loop+store", "of_which_exchange_barrier"]),
                            ("dw", buf[1 << 15:], ["wait+barrier", "S_phase", "dS_tail", "dW_phase"])):
        m = reg.reshape(-1, 8).astype(np.float64)
        m = m[m[:, 6] > 0]
        if not m.size:
            continue
        per = m[:, :4] / m[:, 6:7]
        out[name] = {"waves": int(m.shape[0]), "tiles_per_wave": round(float(m[:, 6].mean()), 1),
                     "cycles_per_tile": {n: round(float(v), 1) for n, v in zip(cols, per.mean(0)) if v > 0}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
