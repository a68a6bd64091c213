"""Print the C-ABI entry points (and comm all-reduces) one bench step issues, in call order:
python3 tools/call_trace.py [bench flags...], e.g. --dist --schedule serial --comm rccl."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402


def main():
    sys.argv = ["bench.py"] + sys.argv[1:]
    args = bench.parse()
    import torch
    import torch.distributed as dist
    import __graft_entry__
    P = __graft_entry__.load_package()
    P.load_library()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = None
    if args.dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29541")
        dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
        if args.comm == "rccl":
            comm = P.RcclComm.from_process_group(device=dev)
    B, T, V, _ = bench.CONFIGS[args.config]
    hp, step, _ = bench.ppo_setup(torch, P, args, B, T, V, dev, 0, args.config == "c3", torch.bfloat16, 1, comm)
    log = []
    real = P._lib.call

    def call(name, *a):
        log.append(name)
        return real(name, *a)
    P._lib.call = call
    for i in range(3):
        step()
        print(f"step {i}: {' '.join(log)}", flush=True)
        log.clear()
    hp.wait_stats()
    print(f"wait_stats: {' '.join(log)}", flush=True)
    torch.cuda.synchronize()
    if comm is not None:
        comm.close()
    if args.dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
