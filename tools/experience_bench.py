"""Experience step at the BASELINE shapes: (a) the logits path — policy and reference
lm_head GEMMs by hipBLASLt (torch.matmul, bf16 [N, V] logits written to HBM) + PPOHotPath.
experience (log-softmax-gather rows + GAE tail); (b) PPOHotPath.experience_from_hidden —
the lm_head folded in (two MFMA launches, logits never in HBM) + the same tail.  HIP events,
interleaved medians.  GPU-box tool:  python tools/experience_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import __graft_entry__  # noqa: E402

P = __graft_entry__.load_package()


def timeit(fn, reps=10):
    for _ in range(3):
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


def main():
    dev = torch.device("cuda:0")
    shapes = [("C2 GPT-2 sentiments", 128, 48, 768, 50257), ("C3 T5-base", 256, 48, 768, 32128),
              ("C4 UL2-20B (per GPU)", 128, 128, 4096, 32128)]
    if len(sys.argv) > 1:  # extra shapes "B,T,H,V ..." (route crossover sweeps)
        shapes = [("sweep", *map(int, a.split(","))) for a in sys.argv[1:]]
    for name, B, T, H, V in shapes:
        g = torch.Generator(device=dev).manual_seed(0)
        h = (torch.randn(B, T, H, generator=g, device=dev) * 0.1).to(torch.bfloat16)
        hr = (torch.randn(B, T, H, generator=g, device=dev) * 0.1).to(torch.bfloat16)
        w = (torch.randn(V, H, generator=g, device=dev) * 0.1).to(torch.bfloat16)
        wr = (torch.randn(V, H, generator=g, device=dev) * 0.1).to(torch.bfloat16)
        y = torch.randint(0, V, (B, T), generator=g, device=dev)
        ov = torch.randn(B, T, generator=g, device=dev)
        sc = torch.randn(B, generator=g, device=dev)
        hp = P.PPOHotPath(P.PPOConfig(), B, T, V, torch.bfloat16, dev, kl_coef=0.05)
        logits = torch.empty(B, T, V, dtype=torch.bfloat16, device=dev)
        ref_logits = torch.empty_like(logits)

        def via_logits():
            torch.matmul(h, w.t(), out=logits)
            torch.matmul(hr, wr.t(), out=ref_logits)
            hp.experience(logits, ref_logits, y, ov, sc)

        def via_hidden():
            hp.experience_from_hidden(h, w, hr, wr, y, ov, sc, route="fused")

        def via_auto():  # the default dispatch (gemm route from H >= LM_HEAD_GEMM_MIN_H)
            hp.experience_from_hidden(h, w, hr, wr, y, ov, sc)

        res = {"logits": [], "hidden": [], "auto": []}
        for _ in range(3):
            res["logits"].append(timeit(via_logits))
            res["hidden"].append(timeit(via_hidden))
            res["auto"].append(timeit(via_auto))
        a, b, c = (sorted(v)[1] for v in res.values())
        flop = 2 * 2.0 * B * T * H * V
        print(f"{name:22s} B={B} T={T} H={H} V={V}: GEMMs + rows + tail {a:8.1f} us | lm_head-fused {b:8.1f} us "
              f"({flop / b / 1e6:6.1f} TFLOP/s) | speedup {a / b:4.2f}x | default route {c:8.1f} us ({a / c:4.2f}x)",
              flush=True)


if __name__ == "__main__":
    main()
