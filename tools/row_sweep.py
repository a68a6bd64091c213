"""Launch-variant sweep of the vocab-row kernels (C2 shape by default), A/B inside ONE
process so every variant sees the same GPU: each round runs the bench's pair of row
launches back to back (experience forward over policy + ref rows, then the fused PPO
row pass that writes dlogits), with HIP events around each launch; medians over rounds.
GPU-box tool:  [B=.. T=.. V=.. DT=bf16|f32] python tools/row_sweep.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import __graft_entry__  # noqa: E402

P = __graft_entry__.load_package()
from trlx_t5_amd import _lib  # noqa: E402

KEYS = ("row_variant", "resident_threads", "resident_lb512", "stream_threads", "stream_unroll", "row_order")


def main():
    B, T, V = int(os.environ.get("B", 128)), int(os.environ.get("T", 48)), int(os.environ.get("V", 50257))
    dt = torch.bfloat16 if os.environ.get("DT", "bf16") == "bf16" else torch.float32
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    x0 = torch.randn(B, T, V, generator=g, device=dev).to(dt)
    x1 = torch.randn(B, T, V, generator=g, device=dev).to(dt)
    x2 = torch.randn(B, T, V, generator=g, device=dev).to(dt)
    y = torch.randint(0, V, (B, T), generator=g, device=dev)
    lp0, lp1, lp2 = (torch.empty(B, T, device=dev) for _ in range(3))
    adv = torch.randn(B, T, device=dev)
    dx = P.grad_buffer_like(x2)
    s = torch.cuda.current_stream().cuda_stream
    es = x0.element_size()

    def fwd():
        _lib.call("trlx_lsm_gather_fwd", x0.data_ptr(), x1.data_ptr(), _lib.dtype_code(x0), B, T, V, x0.stride(0),
                  x0.stride(1), y.data_ptr(), y.stride(0), y.stride(1), lp0.data_ptr(), lp1.data_ptr(), _lib.F32,
                  None, None, s)

    def ppo():
        _lib.call("trlx_ppo_policy_fused", x2.data_ptr(), _lib.dtype_code(x2), B, T, V, x2.stride(0), x2.stride(1),
                  y.data_ptr(), y.stride(0), y.stride(1), lp0.data_ptr(), _lib.F32, adv.data_ptr(), None, 1, None,
                  None, float(B * T), 0.2, lp2.data_ptr(), dx.data_ptr(), dx.stride(0), dx.stride(1), s)

    variants = [("resident (default)", {}), ("resident wave-major", dict(row_order=1)),
                ("resident lb512", dict(resident_lb512=1))]
    for thr in (640, 1024):
        variants.append((f"resident {thr}", dict(resident_threads=thr)))
    for thr, u in ((256, 4), (256, 8)):
        variants.append((f"stream {thr} u{u}", dict(row_variant=2, stream_threads=thr, stream_unroll=u)))
    extra = os.environ.get("VARIANTS")
    if extra:
        variants = [(n, c) for n, c in variants if any(e in n for e in extra.split(","))]

    def setv(cfg):
        for k in KEYS:
            _lib.set_tuning(k, cfg.get(k, 0))

    ref = {}
    dst = torch.empty_like(x0)
    for name, fn in [("torch copy_ (R+W)", lambda: dst.copy_(x0))]:
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 10 * 1e3
        ref[name] = (us, 2 * x0.numel() * es / us / 1e3)
    res = {v[0]: {"fwd": [], "ppo": []} for v in variants}
    for rnd in range(6):
        for name, cfg in variants:
            setv(cfg)
            fwd()
            ppo()
            evs = []
            for _ in range(4):
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                ev[0].record()
                fwd()
                ev[1].record()
                ppo()
                ev[2].record()
                evs.append(ev)
            torch.cuda.synchronize()
            for ev in evs:
                res[name]["fwd"].append(ev[0].elapsed_time(ev[1]) * 1e3)
                res[name]["ppo"].append(ev[1].elapsed_time(ev[2]) * 1e3)
    setv({})
    print(f"shape {B}x{T}x{V} {dt} (in sequence: fwd over 2 tensors, then the PPO R+W pass)")
    for k, (us, gbs) in ref.items():
        print(f"{k:24s} {us:9.1f} us {gbs:8.1f} GB/s")
    nb = 2 * x0.numel() * es
    for name, _ in variants:
        f = sorted(res[name]["fwd"])[len(res[name]["fwd"]) // 2]
        p = sorted(res[name]["ppo"])[len(res[name]["ppo"]) // 2]
        print(f"{name:24s} fwd {f:8.1f} us {nb / f / 1e3:7.1f} GB/s | ppo(R+W) {p:8.1f} us {nb / p / 1e3:7.1f} GB/s"
              f" | pair {f + p:8.1f} us")
    print(json.dumps({"ref": ref, "res": res}))


if __name__ == "__main__":
    main()
