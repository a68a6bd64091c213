"""Device-resident PPO rollout store — a drop-in for
trlx/pipeline/ppo_pipeline.py `PPORolloutStorage` and trlx/data/ppo_types.py.

The reference moves every experience chunk to the host (`.cpu()` of five tensors,
ppo_orchestrator.py:169-173), splits it into per-sample `PPORLElement`s (:177-186) and
re-pads them per training batch with `pad_sequence` in a DataLoader collate
(ppo_pipeline.py:36-66), then copies the batch back to the GPU
(accelerate_ppo_model.py:81-85).  Here the store keeps each field as a padded columnar
buffer in HBM — queries right-aligned (left-padded with pad_token_id), responses
left-aligned (right-padded with pad_token_id), logprobs / values / rewards left-aligned
(right-padded with 0.0) — so pushing a generation batch and collating a training batch are
each ONE launch of `trlx_rows_copy`, and a batch never leaves the device.  The collated
batch equals the reference collate exactly: the rows' own padding is already in place, so
padding a batch to its widest query / response is a column window of the buffers.
"""
import ctypes
from dataclasses import dataclass
from typing import Iterable, List, Optional

import numpy as np
import torch

from . import _lib

__all__ = ["PPORLElement", "PPORLBatch", "PPORolloutStorage", "RolloutLoader"]


@dataclass
class PPORLElement:
    """One rollout (trlx/data/ppo_types.py:6-31)."""
    query_tensor: torch.Tensor
    response_tensor: torch.Tensor
    logprobs: torch.Tensor
    values: torch.Tensor
    rewards: torch.Tensor


@dataclass
class PPORLBatch:
    """A collated batch (trlx/data/ppo_types.py:34-57)."""
    query_tensors: torch.Tensor
    response_tensors: torch.Tensor
    logprobs: torch.Tensor
    values: torch.Tensor
    rewards: torch.Tensor


_FIELDS = ("query", "response", "logprobs", "values", "rewards")


def _rows_copy(fields, rows, src_idx=None, src_row0=0, dst_idx=None, dst_row0=0, stream=None):
    """fields: list of (src, dst, src_col0, dst_col0, cols) with 2-D tensors (row stride =
    stride(0), unit column stride)."""
    n = len(fields)
    srcs = (ctypes.c_void_p * n)(*[f[0].data_ptr() for f in fields])
    dsts = (ctypes.c_void_p * n)(*[f[1].data_ptr() for f in fields])
    sld = (ctypes.c_int64 * n)(*[f[0].stride(0) for f in fields])
    dld = (ctypes.c_int64 * n)(*[f[1].stride(0) for f in fields])
    sc0 = (ctypes.c_int64 * n)(*[f[2] for f in fields])
    dc0 = (ctypes.c_int64 * n)(*[f[3] for f in fields])
    cols = (ctypes.c_int64 * n)(*[f[4] for f in fields])
    es = (ctypes.c_int * n)(*[f[0].element_size() for f in fields])
    for f in fields:
        if f[0].dtype != f[1].dtype or f[0].stride(-1) != 1 or f[1].stride(-1) != 1:
            raise ValueError("rows_copy: matching dtypes and unit column strides required")
    s = stream if stream is not None else _lib.stream_of(fields[0][1])
    _lib.call("trlx_rows_copy", n, ctypes.cast(srcs, ctypes.c_void_p), ctypes.cast(dsts, ctypes.c_void_p),
              ctypes.cast(sld, ctypes.c_void_p), ctypes.cast(dld, ctypes.c_void_p),
              ctypes.cast(sc0, ctypes.c_void_p), ctypes.cast(dc0, ctypes.c_void_p),
              ctypes.cast(cols, ctypes.c_void_p), ctypes.cast(es, ctypes.c_void_p), int(rows),
              _lib.ptr(src_idx), int(src_row0), _lib.ptr(dst_idx), int(dst_row0), s)


class PPORolloutStorage:
    """Rollout storage for PPO training, resident in HBM (ppo_pipeline.py:11-68).

    push(exps) takes the reference's iterable of PPORLElement; push_batch(...) takes a
    generation batch as [n, W] device tensors (the orchestrator's own layout, no split into
    elements).  create_loader(batch_size, shuffle) yields PPORLBatch objects on the device.
    """

    def __init__(self, pad_token_id: int, device=None, capacity: int = 1024):
        self.pad_token_id = int(pad_token_id)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self._cap = max(1, int(capacity))
        self._n = 0
        self._wq = 0  # buffer widths (max over pushed rows)
        self._wr = 0
        self._qw: List[int] = []  # per-row widths (host copies: batch widths need no device sync)
        self._rw: List[int] = []
        self._bufs = None
        self._dtypes = None

    # -------------------------------------------------------------- storage
    def _alloc(self, cap, wq, wr, dtypes):
        q = torch.full((cap, wq), self.pad_token_id, dtype=torch.int64, device=self.device)
        r = torch.full((cap, wr), self.pad_token_id, dtype=torch.int64, device=self.device)
        lp, v, rw = (torch.zeros((cap, wr), dtype=dt, device=self.device) for dt in dtypes)
        return [q, r, lp, v, rw]

    def _ensure(self, extra, wq, wr, dtypes):
        need = self._n + extra
        if self._bufs is not None and need <= self._cap and wq <= self._wq and wr <= self._wr:
            return
        cap = self._cap
        while cap < need:
            cap *= 2
        wq, wr = max(wq, self._wq), max(wr, self._wr)
        new = self._alloc(cap, wq, wr, dtypes)
        if self._bufs is not None and self._n:
            old = self._bufs
            # queries stay right-aligned, the rest left-aligned
            _rows_copy([(old[0], new[0], 0, wq - self._wq, self._wq)]
                       + [(old[i], new[i], 0, 0, self._wr) for i in range(1, 5)], self._n)
        self._bufs, self._cap, self._wq, self._wr = new, cap, wq, wr

    def push_batch(self, query_tensors, response_tensors, logprobs, values, rewards):
        """Append n rollouts given as [n, Wq] / [n, Wr] device tensors (one launch)."""
        ts = [query_tensors, response_tensors, logprobs, values, rewards]
        _lib.require_cuda(*ts)
        n, wq = query_tensors.shape
        wr = response_tensors.shape[1]
        for t in ts[1:]:
            if t.dim() != 2 or t.shape[0] != n or t.shape[1] != wr:
                raise ValueError(f"response-side tensors must be [{n}, {wr}], got {tuple(t.shape)}")
        if self._dtypes is None:
            self._dtypes = tuple(t.dtype for t in ts[2:])
        q = query_tensors.to(device=self.device, dtype=torch.int64).contiguous()
        r = response_tensors.to(device=self.device, dtype=torch.int64).contiguous()
        rest = [t.to(device=self.device, dtype=dt).contiguous() for t, dt in zip(ts[2:], self._dtypes)]
        self._ensure(n, wq, wr, self._dtypes)
        b = self._bufs
        _rows_copy([(q, b[0], 0, self._wq - wq, wq), (r, b[1], 0, 0, wr)]
                   + [(src, b[2 + i], 0, 0, wr) for i, src in enumerate(rest)], n, dst_row0=self._n)
        self._qw.extend([wq] * n)
        self._rw.extend([wr] * n)
        self._n += n

    def push(self, exps: Iterable[PPORLElement]):
        """The reference's push(list of PPORLElement) (ppo_pipeline.py:22-23): runs of
        consecutive elements with equal widths are stacked and pushed as one batch."""
        exps = list(exps)
        i = 0
        while i < len(exps):
            e0 = exps[i]
            j = i + 1
            while (j < len(exps) and exps[j].query_tensor.shape == e0.query_tensor.shape
                   and exps[j].response_tensor.shape == e0.response_tensor.shape):
                j += 1
            grp = exps[i:j]
            dev = self.device
            self.push_batch(*[torch.stack([getattr(e, f).to(dev) for e in grp]) for f in
                              ("query_tensor", "response_tensor", "logprobs", "values", "rewards")])
            i = j

    def clear_history(self):
        self._n = 0
        self._qw, self._rw = [], []
        if self._bufs is not None:  # restore the padding for the next fill
            self._bufs[0].fill_(self.pad_token_id)
            self._bufs[1].fill_(self.pad_token_id)
            for t in self._bufs[2:]:
                t.zero_()

    def __len__(self) -> int:
        return self._n

    def __getitem__(self, index: int) -> PPORLElement:
        if not -self._n <= index < self._n:
            raise IndexError(index)
        i = index % self._n
        b = self._bufs
        wq, wr = self._qw[i], self._rw[i]
        return PPORLElement(b[0][i, self._wq - wq:], b[1][i, :wr], b[2][i, :wr], b[3][i, :wr], b[4][i, :wr])

    # -------------------------------------------------------------- collate
    def collate(self, idx: torch.Tensor, rows: np.ndarray) -> PPORLBatch:
        """Gather rows `idx` (device int64; `rows` = the same indices on the host) into a
        PPORLBatch padded exactly like the reference collate (ppo_pipeline.py:40-66)."""
        n = len(rows)
        qw = np.asarray(self._qw)[rows]
        rw = np.asarray(self._rw)[rows]
        wq, wr = int(qw.max()), int(rw.max())
        b = self._bufs
        out = [torch.empty((n, wq), dtype=torch.int64, device=self.device),
               torch.empty((n, wr), dtype=torch.int64, device=self.device)]
        out += [torch.empty((n, wr), dtype=t.dtype, device=self.device) for t in b[2:]]
        _rows_copy([(b[0], out[0], self._wq - wq, 0, wq)] + [(b[i], out[i], 0, 0, wr) for i in range(1, 5)], n,
                   src_idx=idx)
        return PPORLBatch(*out)

    def create_loader(self, batch_size: int, shuffle: bool, generator: Optional[torch.Generator] = None,
                      drop_last: bool = False) -> "RolloutLoader":
        """Batches of the stored rollouts (ppo_pipeline.py:34-68 / torch DataLoader order:
        sequential, or a torch.randperm permutation when shuffle)."""
        return RolloutLoader(self, batch_size, shuffle, generator, drop_last)


class RolloutLoader:
    """Iterable of device PPORLBatch objects over a PPORolloutStorage snapshot."""

    def __init__(self, store: PPORolloutStorage, batch_size: int, shuffle: bool,
                 generator: Optional[torch.Generator], drop_last: bool):
        self.store, self.batch_size, self.shuffle = store, int(batch_size), bool(shuffle)
        self.generator, self.drop_last = generator, drop_last

    def __len__(self):
        n = len(self.store)
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        n = len(self.store)
        order = torch.randperm(n, generator=self.generator) if self.shuffle else torch.arange(n)
        order_dev = order.to(self.store.device, non_blocking=False)
        host = order.numpy()
        for k in range(len(self)):
            lo, hi = k * self.batch_size, min(n, (k + 1) * self.batch_size)
            yield self.store.collate(order_dev[lo:hi], host[lo:hi])
