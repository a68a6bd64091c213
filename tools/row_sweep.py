"""Launch-geometry sweep of the vocab-row kernels on the C2 shape (one process,
interleaved rounds, HIP events on the launch stream).  GPU-box tool; prints a table."""
import os
import sys
import json

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import __graft_entry__  # noqa: E402

P = __graft_entry__.load_package()
from trlx_t5_amd import _lib  # noqa: E402


def main():
    B, T, V = int(os.environ.get("B", 128)), int(os.environ.get("T", 48)), int(os.environ.get("V", 50257))
    dt = torch.bfloat16 if os.environ.get("DT", "bf16") == "bf16" else torch.float32
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    x0 = torch.randn(B, T, V, generator=g, device=dev).to(dt)
    x1 = torch.randn(B, T, V, generator=g, device=dev).to(dt)
    y = torch.randint(0, V, (B, T), generator=g, device=dev)
    lp0 = torch.empty(B, T, device=dev)
    lp1 = torch.empty(B, T, device=dev)
    adv = torch.randn(B, T, device=dev)
    dx = P.grad_buffer_like(x0)
    s = torch.cuda.current_stream().cuda_stream
    es = x0.element_size()

    def fwd():
        _lib.call("trlx_lsm_gather_fwd", x0.data_ptr(), x1.data_ptr(), _lib.dtype_code(x0), B, T, V, x0.stride(0),
                  x0.stride(1), y.data_ptr(), y.stride(0), y.stride(1), lp0.data_ptr(), lp1.data_ptr(), _lib.F32,
                  None, None, s)

    def ppo():
        _lib.call("trlx_ppo_policy_fused", x0.data_ptr(), _lib.dtype_code(x0), B, T, V, x0.stride(0), x0.stride(1),
                  y.data_ptr(), y.stride(0), y.stride(1), lp1.data_ptr(), _lib.F32, adv.data_ptr(), None, 1, None,
                  None, float(B * T), 0.2, lp0.data_ptr(), dx.data_ptr(), dx.stride(0), dx.stride(1), s)

    variants = [("resident auto", dict(row_variant=1)), ("resident 512 nolb", dict(row_variant=1, resident_lb512=0))]
    for thr in (448, 512, 640, 1024):
        variants.append((f"resident {thr}", dict(row_variant=1, resident_threads=thr)))
    for thr, u in ((256, 2), (256, 4), (256, 8), (128, 8)):
        variants.append((f"stream {thr} u{u}", dict(row_variant=2, stream_threads=thr, stream_unroll=u)))

    def setv(cfg):
        for k in ("row_variant", "resident_threads", "stream_threads", "stream_unroll"):
            _lib.set_tuning(k, cfg.get(k, 0))
        _lib.set_tuning("resident_lb512", cfg.get("resident_lb512", 1))

    # copy / read reference points (torch's own kernels)
    ref = {}
    dst = torch.empty_like(x0)
    for name, fn in [("torch copy_ (R+W)", lambda: dst.copy_(x0)), ("torch sum (R)", lambda: x0.sum(dtype=torch.float32))]:
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 10 * 1e3
        nbytes = x0.numel() * es * (2 if "copy" in name else 1)
        ref[name] = (us, nbytes / us / 1e3)
    res = {v[0]: {"fwd": [], "ppo": []} for v in variants}
    for rnd in range(5):
        for name, cfg in variants:
            setv(cfg)
            for kname, fn, nbytes in (("fwd", fwd, 2 * x0.numel() * es), ("ppo", ppo, 2 * x0.numel() * es)):
                fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res[name][kname].append(e0.elapsed_time(e1) / 5 * 1e3)
    setv({})
    print(f"shape {B}x{T}x{V} {dt}")
    for k, (us, gbs) in ref.items():
        print(f"{k:24s} {us:9.1f} us {gbs:8.1f} GB/s")
    for name, _ in variants:
        f = sorted(res[name]["fwd"])[2]
        p = sorted(res[name]["ppo"])[2]
        nb = 2 * x0.numel() * es
        print(f"{name:24s} fwd(2 rows) {f:8.1f} us {nb / f / 1e3:7.1f} GB/s | ppo(R+W) {p:8.1f} us {nb / p / 1e3:7.1f} GB/s")
    print(json.dumps({"ref": ref, "res": res}))


if __name__ == "__main__":
    main()
