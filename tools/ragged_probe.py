"""Where a ragged batch's time goes: the C3 step (pipelined, bf16) with the same logits under
different decoder-length patterns, interleaved rounds in one process.
  dense   no lengths / mask (every row read)
  full    lengths = T, mask all ones (the per-row checks run, nothing is skipped)
  random  bench.py's L ~ U{1..T} (about half the rows skipped)
  sorted  the same lengths sorted descending (the skipped rows gather at the end of the grid)
Prints per-launch averages (HIP events) and the step time.

  python tools/ragged_probe.py [--config c3] [--steps 60] [--rounds 3]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="c3")
    p.add_argument("--steps", type=int, default=60)
    p.add_argument("--rounds", type=int, default=3)
    a = p.parse_args()
    import torch
    import torch.distributed as dist
    import __graft_entry__
    import bench
    P = __graft_entry__.load_package()
    P.load_library()
    dev = torch.device("cuda", 0)
    B, T, V, _ = bench.CONFIGS[a.config]
    ns = argparse.Namespace(host_state=False, schedule="pipelined", overlap_tail=False, no_defer_tail=False,
                            loss_norm="rank", split_beta=False, no_gae_fold=False, coef_launch=False, warmup=5,
                            settle_ms=200.0, steps=a.steps, no_timers=False)
    hp, step, x = bench.ppo_setup(torch, P, ns, B, T, V, dev, 0, True, torch.bfloat16)
    L = x["lengths"].clone()
    ar = torch.arange(T, device=dev)[None, :]
    pats = {"dense": (None, None), "full": (torch.full_like(L, T), torch.ones_like(x["mask"])),
            "random": (L, (ar < L[:, None]).long())}
    Ls = torch.sort(L, descending=True).values
    pats["sorted"] = (Ls, (ar < Ls[:, None]).long())
    res = {n: [] for n in pats}
    for rnd in range(a.rounds):
        for key in pats:
            x["lengths"], x["mask"] = pats[key]
            bench.settle_and_warm(step, torch, ns, dev)
            el, km, _ = bench.timed_run(step, hp, torch, dist, ns, dev, 1, {"experience", "loss"})
            res[key].append((el / a.steps * 1e3, km["experience"] * 1e3, km["loss"] * 1e3))
            print(f"round {rnd} {key:12s} step {res[key][-1][0]:.4f} ms  E {res[key][-1][1]:7.2f} us  "
                  f"L {res[key][-1][2]:7.2f} us", flush=True)
    fill = float(L.sum()) / (B * T)
    print(f"{a.config} {B}x{T}x{V}: random fill {fill:.4f}")
    for name, r in res.items():
        r = sorted(r)
        m = r[len(r) // 2]
        print(f"median {name:12s} step {m[0]:.4f} ms  E {m[1]:7.2f} us  L {m[2]:7.2f} us")


if __name__ == "__main__":
    main()
