"""Can two RCCL ranks share the one GPU of the dev box?  If they can, the world-2 RCCL path
(bench.py's DP schedule over the "nccl" backend) can be exercised here instead of only on the
driver's 8-GPU node.  Spawns two ranks on cuda:0, initialises ProcessGroupNCCL and all-reduces
a small fp64 vector; prints what RCCL says.

  python tools/rccl_same_device_probe.py
"""
import os
import sys

import torch
import torch.multiprocessing as mp


def _rank(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2")
    try:
        import torch.distributed as dist
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", rank=rank, world_size=2, device_id=dev)
        x = torch.full((4,), float(rank + 1), dtype=torch.float64, device=dev)
        dist.all_reduce(x)
        torch.cuda.synchronize()
        q.put((rank, "ok", x.cpu().tolist()))
        dist.destroy_process_group()
    except Exception as e:  # report, do not hang the peer
        q.put((rank, "error", repr(e)[:400]))


def main():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 100
    ps = [ctx.Process(target=_rank, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = []
    try:
        for _ in range(2):
            res.append(q.get(timeout=90))
    except Exception as e:
        res.append(("-", "timeout", repr(e)))
    for p in ps:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    for r in sorted(res, key=str):
        print(r)
    print("exit codes", [p.exitcode for p in ps])
    return 0


if __name__ == "__main__":
    sys.exit(main())
