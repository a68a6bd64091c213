#!/usr/bin/env python3
"""Price the parts of the fused lm_head loss forward's steady-state step (diagnostic only).

Each library under abl/ is the product built with -DLL_ABLATE=<bits> (csrc/lmhead_loss.hip:
1 softmax, 2 group-sum exchange, 4 next-tile DMA, 8 O product, 16 S product dropped; the
results of such a build are wrong).  One subprocess per library (TRLX_T5_AMD_LIB), each timing
trlx_lmhead_logprobs_fwd_saved (forward + combine) and trlx_lmhead_logprobs_bwd (combine + dW)
at the C2 shape with HIP events, median of --iters.

  python tools/lmloss_ablate.py [--libs base,abl/lib_abl1.so,...] [--iters 20]
  (LL_TUNE=key=value,... sets library tunings in each child; LL_STAMPS=1 with a -DLL_STAMP=1 build)
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(N, H, V, iters):
    sys.path.insert(0, ROOT)
    import torch
    import __graft_entry__
    P = __graft_entry__.load_package()
    L = P._lib
    L.load()
    for kv in filter(None, os.environ.get("LL_TUNE", "").split(",")):  # e.g. LL_TUNE=lmloss_dw_stage=1
        k, v = kv.split("=")
        L.set_tuning(k, int(v))
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    h = torch.randn(N, H, generator=g, device=dev).to(torch.bfloat16)
    w = (torch.randn(V, H, generator=g, device=dev) * 0.05).to(torch.bfloat16)
    y = torch.randint(0, V, (N,), generator=g, device=dev)
    lp = torch.empty(N, device=dev)
    lse = torch.empty(N, device=dev)
    e = torch.empty(N, H, device=dev)
    gin = torch.randn(N, generator=g, device=dev)
    dh = torch.empty(N, H, dtype=torch.bfloat16, device=dev)
    dw = torch.empty(V, H, dtype=torch.bfloat16, device=dev)
    ws = torch.empty(L.query("trlx_lmhead_loss_workspace_bytes", N, H, V), dtype=torch.uint8, device=dev)
    st = L.stream_of(h)

    def fwd():
        L.call("trlx_lmhead_logprobs_fwd_saved", h.data_ptr(), H, w.data_ptr(), H, N, H, V, y.data_ptr(), 1,
               lp.data_ptr(), L.F32, lse.data_ptr(), e.data_ptr(), ws.data_ptr(), st)

    def bwd():
        L.call("trlx_lmhead_logprobs_bwd", h.data_ptr(), H, w.data_ptr(), H, N, H, V, y.data_ptr(), 1,
               gin.data_ptr(), L.F32, lse.data_ptr(), e.data_ptr(), dh.data_ptr(), H, L.BF16, dw.data_ptr(),
               L.BF16, H, ws.data_ptr(), st)

    out = {}
    if os.environ.get("LL_STAMPS"):
        import ctypes
        import numpy as np
        fwd()
        torch.cuda.synchronize()
        bwd()
        torch.cuda.synchronize()
        buf = np.zeros(1 << 16, dtype=np.uint64)
        lib = L.load()
        lib.trlx_debug_ll_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        assert lib.trlx_debug_ll_stamps(buf.ctypes.data, buf.size) == 0
        if os.environ.get("LL_HS"):  # H-sliced engine: [wait+barrier, S part, P part, phases] per wave
            for name, reg in (("fwd_hs", buf[:1 << 15]), ("dw_hs", buf[1 << 15:])):
                m = reg.reshape(-1, 8)
                m = m[m[:, 3] > 0].astype(np.float64)
                if m.size:
                    per = m[:, :3] / m[:, 3:4]
                    out[name + "_stamp_cycles_per_phase"] = {n: round(float(v), 1) for n, v in zip(
                        ["wait_dma+barrier", "S_part(+X)", "P_part"], per.mean(0))}
                    out[name + "_phases_per_wave"] = float(m[:, 3].mean())
            buf[:] = 0
        dm = buf[1 << 15:].reshape(-1, 8)
        dm = dm[dm[:, 6] > 0].astype(np.float64)
        if dm.size:
            dper = dm[:, :4] / dm[:, 6:7]
            out["dw_stamp_cycles_per_step"] = {n: round(float(v), 1) for n, v in zip(
                ["wait_dma+barrier", "S_phase", "dS_tail", "dW_phase"], dper.mean(0))}
        sm = buf[:1 << 15].reshape(-1, 8)
        sm = sm[sm[:, 6] > 0].astype(np.float64)
        per = sm[:, :6] / sm[:, 6:7] if sm.size else np.zeros((1, 6))
        names = ["wait_dma+barrier", "S+softmax", "xwrite+dma_issue", "O_product", "mid_barrier", "xread"]
        out["stamp_cycles_per_step"] = {n: round(float(v), 1) for n, v in zip(names, per.mean(0))}
        out["stamp_waves"] = int(sm.shape[0])
        out["steps_per_wave"] = float(sm[:, 6].mean())
    for name, fn in (("fwd", fwd), ("bwd", bwd)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
        for a, b in ev:
            a.record()
            fn()
            b.record()
        torch.cuda.synchronize()
        out[name + "_us"] = round(statistics.median(a.elapsed_time(b) for a, b in ev) * 1e3, 1)
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="base")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--shape", default="6144,768,50257")
    ap.add_argument("--child", action="store_true")
    args = ap.parse_args()
    N, H, V = (int(x) for x in args.shape.split(","))
    if args.child:
        child(N, H, V, args.iters)
        return
    for lib in args.libs.split(","):
        env = dict(os.environ)
        if lib != "base":
            env["TRLX_T5_AMD_LIB"] = os.path.join(ROOT, lib)
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--iters", str(args.iters),
                            "--shape", args.shape], env=env, capture_output=True, text=True, timeout=300)
        line = r.stdout.strip().splitlines()[-1] if r.returncode == 0 and r.stdout.strip() else r.stderr[-400:]
        print(json.dumps({"lib": lib, "result": line}), flush=True)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
