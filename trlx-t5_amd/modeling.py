"""Drop-in for trlx/utils/modeling.py (reference file) on MI355X.

Same names, signatures and return conventions as the reference; every tensor
computation is a HIP kernel from libtrlx_t5_amd.so (no CPU path):

  get_global_statistics  modeling.py:9-21   partial moments + RCCL all-reduce of {sum, sumsq, n}
  whiten                 modeling.py:24-34  biased (distributed branch) / unbiased (var_mean)
  logprobs_from_logits   modeling.py:37-41  fused single-pass log-softmax + gather, autograd
  flatten_dict           modeling.py:44-57  host utility
  RunningMoments         modeling.py:72-104 Chan merge of batch moments (device fp64 record)
"""
from collections.abc import MutableMapping
from typing import Tuple

import torch
import torch.distributed as dist

from . import _lib

__all__ = ["get_global_statistics", "whiten", "logprobs_from_logits", "flatten_dict", "RunningMoments",
           "moments", "grad_buffer_like"]


# ------------------------------------------------------------------ moments (A3)
def moments(xs: torch.Tensor) -> torch.Tensor:
    """fp64 [4] device tensor {sum, sum of squares, count, 0} of xs (deterministic)."""
    _lib.require_cuda(xs)
    x = xs.contiguous()
    n = x.numel()
    nblk = _lib.query("trlx_moments_num_blocks", n)
    part = torch.empty(nblk * _lib.MOMENT_SLOTS, dtype=torch.float64, device=x.device)
    st = torch.empty(_lib.MOMENT_SLOTS, dtype=torch.float64, device=x.device)
    s = _lib.stream_of(x)
    _lib.call("trlx_moments_partial", _lib.ptr(x), _lib.dtype_code(x), n, _lib.ptr(part), s)
    _lib.call("trlx_moments_finalize", _lib.ptr(part), nblk, _lib.ptr(st), s)
    return st


def _allreduce_moments(st: torch.Tensor) -> torch.Tensor:
    """SUM {sum, sumsq, count} across ranks (one fp64 RCCL all-reduce, modeling.py:14,19)."""
    if dist.is_available() and dist.is_initialized():
        head = st[:3]
        dist.all_reduce(head, dist.ReduceOp.SUM)
    return st


def moments_to_mean_var(st: torch.Tensor, unbiased: bool):
    """{sum, sumsq, count} -> (mean, var) as fp64 0-d tensors on st's device (no sync).
    Same formula the kernels use (ppo_math.h whiten_coeffs)."""
    total, sumsq, count = st[0], st[1], st[2]
    mean = total / count
    m2 = (sumsq - total * mean).clamp_min(0)
    return mean, m2 / ((count - 1) if unbiased else count)


def get_global_statistics(xs: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Global mean and biased variance of xs across processes (modeling.py:9-21).

    Returns 0-d tensors in xs.dtype like the reference (which builds its all-reduce
    buffer in xs.dtype).  The accumulation itself is fp64 on device and one all-reduce.
    """
    st = _allreduce_moments(moments(xs))
    mean, var = moments_to_mean_var(st, unbiased=False)
    return mean.to(xs.dtype), var.to(xs.dtype), st[2].to(xs.dtype)


def whiten(xs: torch.Tensor, shift_mean=True, distributed=True) -> torch.Tensor:
    """(xs - mean) * rsqrt(var + 1e-8) (+ mean if not shift_mean)  — modeling.py:24-34.

    distributed and torch.distributed initialised -> global biased variance (one
    all-reduce); otherwise torch.var_mean semantics (unbiased).
    """
    use_dist = distributed and dist.is_available() and dist.is_initialized()
    st = moments(xs)
    if use_dist:
        _allreduce_moments(st)
    x = xs.contiguous()
    out = torch.empty_like(x)
    _lib.call("trlx_whiten_apply", _lib.ptr(x), _lib.dtype_code(x), x.numel(), _lib.ptr(st),
              0 if use_dist else 1, 1 if shift_mean else 0, _lib.ptr(out), _lib.dtype_code(out),
              _lib.stream_of(x))
    return out.view_as(xs)


# ------------------------------------------------------------------ logprobs (A1)
def _token_geometry(logits: torch.Tensor, labels: torch.Tensor):
    """Express logits[..., V] / labels[...] as (B, T, V, sb, st) / (lb, lt) strided views."""
    if logits.dim() < 2:
        raise ValueError("logits must have at least 2 dims [..., V]")
    if tuple(labels.shape) != tuple(logits.shape[:-1]):
        raise ValueError(f"labels shape {tuple(labels.shape)} must equal logits.shape[:-1] {tuple(logits.shape[:-1])}")
    if labels.dtype != torch.int64:
        raise TypeError("labels must be int64 (torch.gather index)")
    if logits.stride(-1) != 1:
        logits = logits.contiguous()
    if logits.dim() == 2:
        N, V = logits.shape
        return logits, labels, (N, 1, V, logits.stride(0), 0), (labels.stride(0), 0)
    if logits.dim() > 3:
        lead = logits.shape[:-2]
        logits = logits.reshape(-1, logits.shape[-2], logits.shape[-1])
        labels = labels.reshape(-1, labels.shape[-1])
        del lead
    B, T, V = logits.shape
    return logits, labels, (B, T, V, logits.stride(0), logits.stride(1)), (labels.stride(0), labels.stride(1))


def grad_buffer_like(x: torch.Tensor) -> torch.Tensor:
    """Uninitialised tensor with x's size/strides whose rows have x's 256-byte phase, so the
    kernels write dlogits with the same 16-B vectors, grouped into the same whole 256-B
    spans, that they read logits with (the kernels need the 16-B phase for correctness;
    the 256-B phase keeps the stores line-aligned, common.h line_shift)."""
    es = x.element_size()
    extent = 1 + sum((s - 1) * st for s, st in zip(x.shape, x.stride()) if s > 0)
    pad = 256 // es
    buf = torch.empty(extent + pad, dtype=x.dtype, device=x.device)
    off = ((x.data_ptr() - buf.data_ptr()) % 256) // es
    return buf.as_strided(x.shape, x.stride(), off)


class _LogprobsFromLogits(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        _lib.require_cuda(logits, labels)
        orig_shape = labels.shape
        lg, lb, (B, T, V, sb, st), (l0, l1) = _token_geometry(logits, labels)
        out = torch.empty((B, T), dtype=logits.dtype, device=logits.device)
        lse = torch.empty((B, T), dtype=torch.float32, device=logits.device)
        _lib.call("trlx_lsm_gather_fwd", _lib.ptr(lg), None, _lib.dtype_code(lg), B, T, V, sb, st,
                  _lib.ptr(lb), l0, l1, _lib.ptr(out), None, _lib.dtype_code(out), _lib.ptr(lse), None,
                  _lib.stream_of(lg))
        ctx.save_for_backward(lg, lb, lse)
        ctx.geom = (B, T, V, sb, st, l0, l1)
        ctx.logits_meta = (logits.shape, lg is logits)
        return out.view(orig_shape)

    @staticmethod
    def backward(ctx, grad_out):
        lg, lb, lse = ctx.saved_tensors
        B, T, V, sb, st, l0, l1 = ctx.geom
        g = grad_out.contiguous()
        if g.dtype not in (torch.float32, torch.bfloat16):
            g = g.float()
        dx = grad_buffer_like(lg)
        dsb, dst = (dx.stride(0), dx.stride(1)) if dx.dim() == 3 else (dx.stride(0), 0)
        _lib.call("trlx_lsm_gather_bwd", _lib.ptr(lg), _lib.dtype_code(lg), B, T, V, sb, st, _lib.ptr(lb),
                  l0, l1, _lib.ptr(lse), _lib.ptr(g), _lib.dtype_code(g), _lib.ptr(dx), dsb, dst,
                  _lib.stream_of(lg))
        shape, same = ctx.logits_meta
        return (dx if same else dx.reshape(shape)), None


def logprobs_from_logits(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """log_softmax(logits, -1).gather(-1, labels[..., None]).squeeze(-1) — modeling.py:37-41.

    One HBM pass over each vocab row (the [.., V] log-softmax is never materialised);
    differentiable w.r.t. logits (backward = one read + one write of the row).  Output dtype
    = logits dtype, like the reference.
    """
    return _LogprobsFromLogits.apply(logits, labels)


# ------------------------------------------------------------------ host utilities
def flatten_dict(d, parent_key: str = "", sep: str = "/") -> dict:
    """Nested dict -> flat dict with `sep`-joined keys (modeling.py:44-57)."""
    items = {}
    for k, v in d.items():
        key = f"{parent_key}{sep}{k}" if parent_key else k
        if isinstance(v, MutableMapping):
            items.update(flatten_dict(v, key, sep=sep))
        else:
            items[key] = v
    return items


def merge_moments(mean, var, count, xs_mean, xs_var, xs_count):
    """Chan/parallel merge used by RunningMoments.update (modeling.py:91-102); host floats.

    Returns (new_mean, new_var, new_std(unbiased), new_count)."""
    delta = xs_mean - mean
    tot = count + xs_count
    new_sum = xs_var * xs_count
    old_sum = var * count + delta ** 2 * count * xs_count / tot
    new_mean = mean + delta * xs_count / tot
    new_var = (old_sum + new_sum) / tot
    new_std = (new_var * tot / (tot - 1)) ** 0.5
    return new_mean, new_var, new_std, tot


class RunningMoments:
    """Running mean / std of a scalar stream (modeling.py:72-104), device resident.

    State: one fp64 controller record on the device of the first batch (TRLX_CTL_* slots,
    the layout PPOControlState uses).  update(xs) = the device moments kernel {Σx, Σx², n}
    (all-reduced across ranks when torch.distributed is initialised: get_global_statistics
    semantics, biased variance; torch.var_mean(unbiased=False) otherwise) and the Chan merge
    kernel (trlx_score_moments_merge, term for term modeling.py:91-102, in fp64) — no host
    synchronisation.  Types follow the reference: update returns (batch mean, unbiased batch
    std) as 0-d tensors of xs.dtype on xs.device; after the first update mean / var / std are
    0-d device tensors (xs.dtype), and count is a Python float without a process group (the
    reference's 1e-24 + numel) or a 0-d device tensor with one (its all-reduced count).
    Before the first update they are the reference's initial Python numbers.
    """

    def __init__(self):
        self._st = None       # fp64 [TRLX_CTL_SLOTS] device record, allocated by the first update
        self._dtype = None    # dtype of the last batch (the reference's attribute tensors carry it)
        self._count = 1e-24   # host count (non-distributed updates only)
        self._host_count = True

    def _slot(self, k, init):
        if self._st is None:
            return init
        return self._st[k].to(self._dtype)

    @property
    def mean(self):
        return self._slot(_lib.CTL_MEAN, 0)

    @property
    def var(self):
        return self._slot(_lib.CTL_VAR, 1)

    @property
    def std(self):
        return self._slot(_lib.CTL_STD, 1)

    @property
    def count(self):
        if self._st is None or self._host_count:
            return self._count
        return self._st[_lib.CTL_COUNT].to(self._dtype)

    def update(self, xs: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        _lib.require_cuda(xs)
        s = _lib.stream_of(xs)
        if self._st is None:
            self._st = torch.empty(_lib.CTL_SLOTS, dtype=torch.float64, device=xs.device)
            _lib.call("trlx_ctl_init", _lib.ptr(self._st), 0.0, 0.0, float("nan"), 0, s)
        elif self._st.device != xs.device:
            raise ValueError(f"RunningMoments state lives on {self._st.device}, batch on {xs.device}")
        st = moments(xs)
        use_dist = dist.is_available() and dist.is_initialized()
        if use_dist:
            _allreduce_moments(st)
            self._host_count = False
        else:
            self._count = self._count + xs.numel()
        _lib.call("trlx_score_moments_merge", _lib.ptr(self._st), _lib.ptr(self._st), _lib.ptr(st), s)
        self._dtype = xs.dtype
        return (self._st[_lib.CTL_BATCH_MEAN].to(xs.dtype), self._st[_lib.CTL_BATCH_STD].to(xs.dtype))

    def _update_scaled(self, scores: torch.Tensor, mode: int, clip: float, ref_std=None):
        """update(scores) fused with the orchestrator's scale / clip (ppo.prepare_scores): one
        trlx_score_ctl_update launch on this record (local two-pass fp64 batch moments, or the
        all-reduced ones under a process group).  Returns (scores', batch mean, batch std)."""
        _lib.require_cuda(scores)
        x = scores.to(torch.float32).contiguous()
        if x.numel() == 0:
            raise ValueError("prepare_scores: empty score batch")
        s = _lib.stream_of(x)
        if self._st is None:
            self._st = torch.empty(_lib.CTL_SLOTS, dtype=torch.float64, device=x.device)
            _lib.call("trlx_ctl_init", _lib.ptr(self._st), 0.0, 0.0, float("nan"), 0, s)
        g = None
        if dist.is_available() and dist.is_initialized():
            g = _allreduce_moments(moments(x))
            self._host_count = False
        else:
            self._count = self._count + x.numel()
        if mode == _lib.SCALE_REF:  # the caller's ref_std (ppo_orchestrator.py:96-98 keeps it host side)
            self._st[_lib.CTL_REF_STD].fill_(float(ref_std))
            self._st[_lib.CTL_REF_SET].fill_(1.0)
        out = torch.empty_like(x)
        c = _lib.ScoreCtl(_lib.ptr(self._st), _lib.ptr(self._st), _lib.ptr(g), mode, clip)
        _lib.call("trlx_score_ctl_update", _lib.ptr(x), _lib.F32, x.numel(), c, _lib.ptr(out), _lib.F32, s)
        self._dtype = x.dtype
        return out.view_as(scores), self._st[_lib.CTL_BATCH_MEAN].to(x.dtype), self._st[_lib.CTL_BATCH_STD].to(x.dtype)
