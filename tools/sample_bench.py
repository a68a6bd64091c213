"""ILQL sampling step (trlx_ilql_sample) vs the reference's torch ops for the same step
(log_softmax + beta*adv, topk_mask, softmax, multinomial), HIP events, medians.
GPU-box tool:  python tools/sample_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
import __graft_entry__  # noqa: E402

P = __graft_entry__.load_package()
from oracle import ppo_oracle as orc  # noqa: E402


def timeit(fn, reps=20):
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


def torch_step(logits, tqs, vs, beta, k, temp):
    qs = torch.minimum(tqs[0], tqs[1])
    pi_beta = F.log_softmax(logits, -1)
    pi = F.softmax(orc.topk_mask(pi_beta + beta * (qs - vs), k) / temp, -1)
    return torch.multinomial(pi, num_samples=1)


def main():
    dev = torch.device("cuda:0")
    for dt, B in [(torch.float32, b) for b in (8, 32, 128)] + [(torch.bfloat16, b) for b in (8, 128)]:
        V = 50257
        g = torch.Generator(device=dev).manual_seed(0)
        logits = torch.randn(B, V, generator=g, device=dev).to(dt)
        tqs = [torch.randn(B, V, generator=g, device=dev).to(dt) for _ in range(2)]
        vs = torch.randn(B, 1, generator=g, device=dev).to(dt)
        ours = timeit(lambda: P.ilql_sample_step(logits, tqs, vs, beta=4.0, top_k=20, generator=g))
        ref = timeit(lambda: torch_step(logits, tqs, vs, 4.0, 20, 1.0))
        print(f"{str(dt)[6:]:8s} B={B:4d} V={V}: fused sampling step {ours:8.1f} us | torch ops (reference step) {ref:8.1f} us"
              f" | {ref / ours:5.2f}x")


if __name__ == "__main__":
    main()
