"""Where a ragged batch's time goes: the C3 step (pipelined, bf16) with the same logits under
different decoder-length patterns, interleaved rounds in one process.
  dense   no lengths / mask (every row read)
  full    lengths = T, mask all ones (the per-row checks run, nothing is skipped)
  random  bench.py's L ~ U{1..T} (about half the rows skipped)
  sorted  the same lengths sorted descending (the skipped rows gather at the end of the grid)
  halfB / altB / halfT  fill 0.5: first half of the rollouts valid / every other rollout / the
          first half of every rollout
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
    p.add_argument("--orders", default="0", help="tuning values to compare (ragged_order / loss_order: 0 valid rows first, 1 natural order)")
    p.add_argument("--key", default="ragged_order", help="the tuning key --orders sets (ragged_order or loss_order)")
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
    # fill 0.5 at three granularities of the padding: whole rollouts (the first half of the
    # batch valid), alternate rollouts, and the second half of every rollout
    half = torch.zeros_like(L)
    half[: B // 2] = T
    alt = torch.zeros_like(L)
    alt[::2] = T
    tail = torch.full_like(L, T // 2)
    for n, l in (("halfB", half), ("altB", alt), ("halfT", tail)):
        pats[n] = (l, (ar < l[:, None]).long())
    from trlx_t5_amd import _lib
    orders = [int(v) for v in a.orders.split(",")]
    runs = [(n, o) for n in pats for o in (orders if n != "dense" else orders[:1])]
    res = {(f"{n} o{o}" if len(orders) > 1 else n): [] for n, o in runs}
    for rnd in range(a.rounds):
        for name, o in runs:
            key = f"{name} o{o}" if len(orders) > 1 else name
            x["lengths"], x["mask"] = pats[name]
            _lib.set_tuning(a.key, o)
            bench.settle_and_warm(step, torch, ns, dev)
            el, km, _ = bench.timed_run(step, hp, torch, dist, ns, dev, 1, {"experience", "loss"})
            res[key].append((el / a.steps * 1e3, km["experience"] * 1e3, km["loss"] * 1e3))
            print(f"round {rnd} {key:12s} step {res[key][-1][0]:.4f} ms  E {res[key][-1][1]:7.2f} us  "
                  f"L {res[key][-1][2]:7.2f} us", flush=True)
    _lib.set_tuning(a.key, 0)
    fill = float(L.sum()) / (B * T)
    print(f"{a.config} {B}x{T}x{V}: random fill {fill:.4f}")
    for name, r in res.items():
        r = sorted(r)
        m = r[len(r) // 2]
        print(f"median {name:12s} step {m[0]:.4f} ms  E {m[1]:7.2f} us  L {m[2]:7.2f} us")


if __name__ == "__main__":
    main()
