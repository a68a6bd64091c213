"""Fused lm_head + logprobs (trlx_lmhead_logprobs) vs the unfused path it replaces
(hipBLASLt GEMM writing bf16 logits + the fused log-softmax-gather row kernel), HIP events,
medians.  GPU-box tool:  python tools/lmhead_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import __graft_entry__  # noqa: E402

P = __graft_entry__.load_package()


def timeit(fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return sorted(ts)[len(ts) // 2]


VARIANTS = tuple(int(v) for v in os.environ.get("LM_VARIANTS", "3,8").split(","))


def main():
    dev = torch.device("cuda:0")
    shapes = [("C2 GPT-2 (128x48 tokens)", 6144, 768, 50257), ("C3 T5-base (256x48)", 12288, 768, 32128),
              ("C4 UL2-20B (128x128)", 16384, 4096, 32128)]
    for name, N, H, V in shapes:
        g = torch.Generator(device=dev).manual_seed(0)
        h = (torch.randn(N, H, generator=g, device=dev) * 0.1).to(torch.bfloat16)
        w = (torch.randn(V, H, generator=g, device=dev) * 0.1).to(torch.bfloat16)
        y = torch.randint(0, V, (N,), generator=g, device=dev)
        res = {}
        for rnd in range(3):  # interleaved rounds (run-to-run drift is several %)
            for var in VARIANTS:
                P._lib.call("trlx_lmhead_set_variant", var)
                res.setdefault(var, []).append(timeit(lambda: P.lm_head_logprobs(h, w, y, out_dtype=torch.float32)))
        res = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
        P._lib.call("trlx_lmhead_set_variant", 0)
        res["auto"] = timeit(lambda: P.lm_head_logprobs(h, w, y, out_dtype=torch.float32))
        fused = res["auto"]
        print("   variants (us):", {k: round(v, 1) for k, v in res.items()})
        gemm = timeit(lambda: h @ w.t())
        logits = h @ w.t()
        rows = timeit(lambda: P.logprobs_from_logits(logits, y))
        flop = 2.0 * N * H * V
        print(f"{name:26s} N={N} H={H} V={V}: fused {fused:8.1f} us ({flop / fused / 1e6:6.1f} TFLOP/s) | "
              f"hipBLASLt GEMM {gemm:8.1f} us + logprob rows {rows:6.1f} us = {gemm + rows:8.1f} us | "
              f"speedup {(gemm + rows) / fused:4.2f}x")


if __name__ == "__main__":
    main()
