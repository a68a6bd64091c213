"""Cost of the whitening all-reduce through torch.distributed "nccl" (RCCL) at world size 1 on
one MI355X: host time per call, and GPU time of a dependent chain compute -> all_reduce ->
compute with and without the collective.  GPU-box tool:  python tools/rccl_probe.py"""
import os
import time

import torch
import torch.distributed as dist


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29544")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    x = torch.zeros(4, dtype=torch.float64, device=dev)
    y = torch.randn(1 << 20, device=dev)
    for _ in range(20):
        dist.all_reduce(x[:3])
    torch.cuda.synchronize()
    for mode in ("sync", "async+wait", "none"):
        n = 200
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        h = 0.0
        e0.record()
        for _ in range(n):
            y.mul_(1.0000001)  # a small dependent kernel on the compute stream
            t0 = time.perf_counter()
            if mode == "sync":
                dist.all_reduce(x[:3])
            elif mode == "async+wait":
                dist.all_reduce(x[:3], async_op=True).wait()
            h += time.perf_counter() - t0
        e1.record()
        torch.cuda.synchronize()
        print(f"{mode:11s} GPU {e0.elapsed_time(e1) * 1e3 / n:7.1f} us/iter   host all_reduce call {h * 1e6 / n:6.1f} us",
              flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
