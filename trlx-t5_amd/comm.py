"""RCCL stats all-reduce helper (SURVEY §8b "Collectives"): one communicator per process for
the hot path's small fp64 SUM all-reduces — the whitening record {Σ A, Σ A², n[, Σmask]}
(the two dist.all_reduce calls of get_global_statistics, trlx/utils/modeling.py:13-14,18-19)
and the score moments of RunningMoments under torch.distributed (modeling.py:85-86).

ProcessGroupNCCL runs each collective on an internal stream joined to the caller's with
default HIP events; on MI355X every such event record is a system-scope release that idles
the compute queue ~20 µs (two per PPO step: +50 µs/step at world size 1, measured,
profiles/r02_rccl_world1.log).  `RcclComm.allreduce_` enqueues ncclAllReduce on the stream
it is given — the step's own stream (no join at all) or a side stream the caller joins with
fence-free events (timing.LaunchEvent).  The communicator is created over the ranks of an
initialised torch.distributed group (the unique id travels by broadcast_object_list) from
the RCCL library PyTorch itself loaded (dlopen of the same file: one RCCL per process).
"""
import ctypes
import os
from typing import Optional

import torch

from . import _lib

__all__ = ["RcclComm", "rccl_library_path"]


def rccl_library_path() -> str:
    """The librccl.so PyTorch runs on (torch/lib), else the system one."""
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p if os.path.exists(p) else "librccl.so.1"


class RcclComm:
    def __init__(self, handle: ctypes.c_void_p, nranks: int, rank: int, device: torch.device):
        self._h = handle
        self.nranks, self.rank, self.device = nranks, rank, device

    @classmethod
    def from_process_group(cls, group=None, device=None) -> "RcclComm":
        """Collective over the ranks of `group` (default: WORLD); call on every rank after
        torch.distributed is initialised and the rank's device is current."""
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("RcclComm.from_process_group needs an initialised torch.distributed group")
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        torch.cuda.set_device(dev)
        _lib.call("trlx_comm_load", rccl_library_path().encode())
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        nb = int(_lib.query("trlx_comm_unique_id_bytes"))
        uid = ctypes.create_string_buffer(nb)
        if rank == 0:
            _lib.call("trlx_comm_unique_id", uid, nb)
        box = [uid.raw]
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast_object_list(box, src=src, group=group)
        uid = ctypes.create_string_buffer(box[0], nb)
        h = ctypes.c_void_p()
        _lib.call("trlx_comm_init", ctypes.byref(h), uid, nb, world, rank)
        return cls(h, world, rank, dev)

    def allreduce_(self, t: torch.Tensor, stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
        """In-place SUM over the ranks of a contiguous fp64 device tensor, enqueued on `stream`
        (default: the current stream)."""
        if t.dtype != torch.float64 or not t.is_contiguous() or t.device != self.device:
            raise ValueError(f"allreduce_ needs a contiguous fp64 tensor on {self.device}")
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _lib.call("trlx_comm_allreduce_sum_f64", self._h, t.data_ptr(), t.numel(), s.cuda_stream)
        return t

    def close(self):
        """ncclCommDestroy (collective in spirit: every rank closes).  Not done from __del__:
        at interpreter shutdown the HIP runtime may already be torn down."""
        if self._h is not None and self._h.value:
            _lib.call("trlx_comm_destroy", self._h)
        self._h = None
