"""World-1 A/B of where the distributed schedules' time goes (bench.py's C2 step, --dist):
serial / pipelined x all-reduces on a side stream joined by fence-free events (product) or
enqueued inline on the step's stream (A/B only: no overlap, no joins).  Prints ms/step of
each variant, interleaved over several rounds."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402


def main():
    sys.argv = ["bench.py", "--cpu-seconds", "0"]
    args = bench.parse()
    import torch
    import torch.distributed as dist
    import __graft_entry__
    P = __graft_entry__.load_package()
    P.load_library()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29542")
    dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
    comm = P.RcclComm.from_process_group(device=dev)
    B, T, V, _ = bench.CONFIGS["c2"]
    variants = {}
    only = os.environ.get("SCHED_PROBE_ONLY")  # e.g. "pipelined/side" (for a profiler run)
    for sched in ("serial", "pipelined"):
        for mode in ("side", "inline"):
            if only and f"{sched}/{mode}" != only:
                continue
            args.schedule = sched
            P.PPOHotPath._comm_timing_events = mode == "side-timing-ev"
            hp, step, x = bench.ppo_setup(torch, P, args, B, T, V, dev, 0, False, torch.bfloat16, 1, comm)
            hp._comm_inline = mode == "inline"
            variants[f"{sched}/{mode}"] = (hp, step)
    res = {k: [] for k in variants}
    for rnd in range(4):
        for k, (hp, step) in variants.items():
            for _ in range(100):
                step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(300):
                step()
            hp.wait_stats()
            torch.cuda.synchronize()
            res[k].append((time.perf_counter() - t0) / 300 * 1e3)
        print(f"round {rnd}: " + "  ".join(f"{k} {v[-1]:.4f}" for k, v in res.items()), flush=True)
    for k, v in res.items():
        print(f"{k}: median {sorted(v)[len(v) // 2]:.4f} ms/step")
    comm.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
