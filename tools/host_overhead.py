"""Host-side cost of one PPO hot-path step: the time the Python caller spends enqueueing a
step (argument checks, ctypes calls, events) against the GPU time of the step.  If the
enqueue time approached the GPU time the bench would measure the host, not the kernels.

  python tools/host_overhead.py [--config c2|c4] [--steps 200] [--schedule pipelined|serial]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="c2")
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--schedule", default="pipelined", choices=("pipelined", "serial"))
    args = p.parse_args()
    import torch
    import __graft_entry__
    import bench
    P = __graft_entry__.load_package()
    P.load_library()
    dev = torch.device("cuda", 0)
    B, T, V, _ = bench.CONFIGS[args.config]
    ns = argparse.Namespace(host_state=False, schedule=args.schedule, overlap_tail=False, no_defer_tail=False,
                            loss_norm="rank", split_beta=False, no_gae_fold=False, coef_launch=False)
    hp, step, _ = bench.ppo_setup(torch, P, ns, B, T, V, dev, 0, args.config == "c3", torch.bfloat16)
    for _ in range(20):
        step()
    torch.cuda.synchronize()
    # host enqueue time per step, measured while the GPU still has work queued (not host-bound
    # waits): time N calls, then the drain
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t1 = time.perf_counter()
    hp.wait_stats()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    host_us = (t1 - t0) / args.steps * 1e6
    wall_us = (t2 - t0) / args.steps * 1e6
    print(f"{args.config} {args.schedule}: host enqueue {host_us:.1f} us/step, wall {wall_us:.1f} us/step "
          f"(host / wall = {host_us / wall_us:.2f})")


if __name__ == "__main__":
    main()
