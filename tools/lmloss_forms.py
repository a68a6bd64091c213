#!/usr/bin/env python3
"""A/B of the fused lm_head loss kernels' forms (csrc/lmhead_loss.hip tunings lmloss_fwd /
lmloss_dw), one process, interleaved rounds, HIP events on the launch stream:

  fwd   trlx_lmhead_logprobs_fwd_saved (forward MFMA launch + restart launch + combine)
  bwd   trlx_lmhead_logprobs_bwd (combine + dW MFMA launch + token-split reduce)

per form, at a config's token count (C2: 6144 x 50257 x 768; C3 live tokens ~6.4k x 32128),
with TFLOP/s on the two MFMA passes each runs.  Also the max relative difference of lp / dW
between the forms (same operands).

  python tools/lmloss_forms.py [--config c2|c3] [--iters 10] [--rounds 5] [--fwd 1,3] [--dw 1,2]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {"c2": (6144, 768, 50257), "c3": (6432, 768, 32128), "h512": (4096, 512, 32128)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(SHAPES))
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--fwd", default="1,3")
    ap.add_argument("--dw", default="1,2")
    args = ap.parse_args()
    import torch
    import __graft_entry__
    P = __graft_entry__.load_package()
    L = P._lib
    L.load()
    N, H, V = SHAPES[args.config]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    h = torch.randn(N, H, generator=g, device=dev).to(torch.bfloat16)
    w = (0.05 * torch.randn(V, H, generator=g, device=dev)).to(torch.bfloat16)
    y = torch.randint(0, V, (N,), generator=g, device=dev)
    gout = torch.randn(N, generator=g, device=dev)
    f32 = dict(dtype=torch.float32, device=dev)
    lp, lse, e = torch.empty(N, **f32), torch.empty(N, **f32), torch.empty((N, H), **f32)
    dh = torch.empty((N, H), dtype=torch.bfloat16, device=dev)
    dw = torch.empty((V, H), dtype=torch.bfloat16, device=dev)
    ws = torch.empty(L.query("trlx_lmhead_loss_workspace_bytes", N, H, V), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream

    def fwd():
        L.call("trlx_lmhead_logprobs_fwd_saved", h.data_ptr(), H, w.data_ptr(), H, N, H, V, y.data_ptr(), 1,
               lp.data_ptr(), L.F32, lse.data_ptr(), e.data_ptr(), ws.data_ptr(), s)

    def bwd():
        L.call("trlx_lmhead_logprobs_bwd", h.data_ptr(), H, w.data_ptr(), H, N, H, V, y.data_ptr(), 1,
               gout.data_ptr(), L.F32, lse.data_ptr(), e.data_ptr(), dh.data_ptr(), H, L.BF16, dw.data_ptr(), L.BF16,
               H, ws.data_ptr(), s)

    def timed(fn, iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters * 1e3

    fwds = [int(x) for x in args.fwd.split(",")]
    dws = [int(x) for x in args.dw.split(",")]
    ref = {}
    for fo in fwds:  # warm up + results per form
        L.set_tuning("lmloss_fwd", fo)
        for _ in range(5):
            fwd()
        torch.cuda.synchronize()
        ref[("fwd", fo)] = (lp.clone(), e.clone())
    L.set_tuning("lmloss_fwd", fwds[0])
    fwd()
    for do in dws:
        L.set_tuning("lmloss_dw", do)
        for _ in range(5):
            bwd()
        torch.cuda.synchronize()
        ref[("dw", do)] = (dh.clone(), dw.clone())
    times = {}
    for r in range(args.rounds):
        order = fwds if r % 2 == 0 else fwds[::-1]
        for fo in order:
            L.set_tuning("lmloss_fwd", fo)
            times.setdefault(f"fwd{fo}", []).append(timed(fwd, args.iters))
        L.set_tuning("lmloss_fwd", fwds[0])
        fwd()
        order = dws if r % 2 == 0 else dws[::-1]
        for do in order:
            L.set_tuning("lmloss_dw", do)
            times.setdefault(f"dw{do}", []).append(timed(bwd, args.iters))
    L.set_tuning("lmloss_fwd", 0)
    L.set_tuning("lmloss_dw", 0)
    flop2 = 2 * 2 * N * V * H
    out = {"config": args.config, "N": N, "H": H, "V": V, "iters": args.iters, "rounds": args.rounds}
    for k, v in times.items():
        med = sorted(v)[len(v) // 2]
        out[k] = {"median_us": round(med, 1), "min_us": round(min(v), 1), "tflops_2pass": round(flop2 / med / 1e6, 1),
                  "rounds_us": [round(x, 1) for x in v]}

    def rel(a, b):
        a, b = a.double(), b.double()
        return float((a - b).norm() / b.norm().clamp_min(1e-30))
    base_f, base_d = ref[("fwd", fwds[0])], ref[("dw", dws[0])]
    out["agree"] = {f"fwd{fo}": {"lp": rel(ref[("fwd", fo)][0], base_f[0]), "E": rel(ref[("fwd", fo)][1], base_f[1])}
                    for fo in fwds}
    out["agree"].update({f"dw{do}": {"dh": rel(ref[("dw", do)][0], base_d[0]), "dW": rel(ref[("dw", do)][1], base_d[1])}
                         for do in dws})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
