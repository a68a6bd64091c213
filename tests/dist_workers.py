"""Worker functions for spawned torch.distributed (gloo) test processes.  Importable in
a fresh child: it registers the package itself."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402

__graft_entry__.load_package()

import torch  # noqa: E402

from trlx_t5_amd.modeling import _allreduce_moments, moments_to_mean_var  # noqa: E402


def whiten_stats_worker(rank, world, port, xs, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    shard = xs.chunk(world, dim=0)[rank].double()
    st = torch.stack([shard.sum(), (shard * shard).sum(), torch.tensor(float(shard.numel())),
                      torch.tensor(0.0, dtype=torch.float64)])
    _allreduce_moments(st)  # the product's exchange: ONE all-reduce of {sum, sumsq, n}
    mean, var = moments_to_mean_var(st, unbiased=False)
    q.put((rank, float(mean), float(var), float(st[2])))
    dist.barrier()
    dist.destroy_process_group()
