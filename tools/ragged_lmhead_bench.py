"""The experience step from hidden states (PPOHotPath.experience_from_hidden, fused lm_head
route) at C3's T5-base shape — 256 rollouts x 48 decoder tokens, H 768, V 32128 — dense vs
with bench.py's ragged decoder lengths (L ~ U{1..48}): the ragged launches gather the valid
tokens' hidden rows and skip the padding's tiles.  HIP events, interleaved medians.

  python tools/ragged_lmhead_bench.py [--B 256] [--T 48] [--H 768] [--V 32128] [--reps 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--B", type=int, default=256)
    p.add_argument("--T", type=int, default=48)
    p.add_argument("--H", type=int, default=768)
    p.add_argument("--V", type=int, default=32128)
    p.add_argument("--reps", type=int, default=20)
    a = p.parse_args()
    import torch
    import __graft_entry__
    P = __graft_entry__.load_package()
    dev = torch.device("cuda", 0)
    B, T, H, V = a.B, a.T, a.H, a.V
    g = torch.Generator(device=dev).manual_seed(0)
    h = (torch.randn(B, T, H, generator=g, device=dev) * 0.2).to(torch.bfloat16)
    hr = (torch.randn(B, T, H, generator=g, device=dev) * 0.2).to(torch.bfloat16)
    w = (torch.randn(V, H, generator=g, device=dev) * 0.2).to(torch.bfloat16)
    wr = (torch.randn(V, H, generator=g, device=dev) * 0.2).to(torch.bfloat16)
    y = torch.randint(0, V, (B, T), generator=g, device=dev)
    ov = torch.randn(B, T, generator=g, device=dev)
    sc = torch.randn(B, generator=g, device=dev)
    L = torch.randint(1, T + 1, (B,), generator=g, device=dev)
    fill = float(L.sum()) / (B * T)
    hp = P.PPOHotPath(P.PPOConfig(), B, T, V, torch.bfloat16, dev, kl_coef=0.05)

    def run(lens):
        hp.experience_from_hidden(h, w, hr, wr, y, ov, sc, lengths=lens, route="fused")

    res = {"dense": [], "ragged": []}
    for _ in range(3):
        run(None)
        run(L)
    torch.cuda.synchronize()
    for _ in range(a.reps):
        for name, lens in (("dense", None), ("ragged", L)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(lens)
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) * 1e3)
    print(f"experience_from_hidden fused, {B}x{T} tokens, H {H}, V {V}, ragged fill {fill:.4f}")
    for name, ts in res.items():
        ts.sort()
        print(f"{name:7s} median {ts[len(ts) // 2]:8.1f} us  (min {ts[0]:.1f})")


if __name__ == "__main__":
    main()
