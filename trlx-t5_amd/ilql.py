"""Drop-in for the ILQL loss of trlx/model/nn/ilql_models.py (config 5) on MI355X.

  ILQLConfig        ilql_models.py:37-58  (method config; .loss on HIP kernels)
  ILQLConfig.loss   ilql_models.py:52-116 (CQL / AWAC cross-entropies over V, TD and
                                           expectile V losses, with autograd)
  ILQLBatch         trlx/data/ilql_types.py:30-49
  ilql_sample_step  ilql_models.py:296-316 (one decode step of generate: log_softmax +
                    beta*adv, topk_mask, softmax / temperature, the draw) — §8f rank 3

The loss runs as three launches (include/trlx_t5_amd.h, trlx_ilql_*): every logits row and
every Q-head row is read once and its gradient row written once in the forward; the
autograd backward only scales the stored gradients by grad_output (a no-op for 1).
"""
import ctypes
from dataclasses import dataclass
from typing import Any, Sequence

import torch

from . import _lib
from .modeling import grad_buffer_like
from .timing import make_event

__all__ = ["ILQLConfig", "ILQLBatch", "ILQLHotPath", "ILQL_LOSS_KEYS", "ilql_sample_step"]

# stats keys in the reference's order (its dict comprehension walks locals(): loss_q,
# loss_v, loss_cql, loss_awac, loss — ilql_models.py:109-113)
ILQL_LOSS_KEYS = ("losses/loss_q", "losses/loss_v", "losses/loss_cql", "losses/loss_awac", "losses/loss")
_SLOT = {"losses/loss": 0, "losses/loss_q": 1, "losses/loss_v": 2, "losses/loss_cql": 3, "losses/loss_awac": 4}


@dataclass
class ILQLBatch:
    """Batched ILQL elements (trlx/data/ilql_types.py:30-49)."""
    input_ids: torch.Tensor       # [B, L] int64
    attention_mask: torch.Tensor  # [B, L]
    rewards: torch.Tensor         # [B, A]
    states_ixs: torch.Tensor      # [B, S]
    actions_ixs: torch.Tensor     # [B, A]
    dones: torch.Tensor           # [B, S]


def _row_view(x, name, shape3):
    if x.dim() != 3 or tuple(x.shape) != tuple(shape3):
        raise ValueError(f"{name} must have shape {tuple(shape3)}, got {tuple(x.shape)}")
    if x.stride(-1) != 1:
        x = x.contiguous()
    return x


def _strides(x):
    return x.stride(0), x.stride(1)


class _ILQLLoss(torch.autograd.Function):
    """Forward = trlx_ilql_loss_fused (gradients computed eagerly, closed form); backward
    scales the stored gradients in place by grad_output."""

    @staticmethod
    def forward(ctx, cfg, logits, vs, q0, q1, tq0, tq1, batch):
        dev = logits.device
        B, L, V = logits.shape
        nq = 1 if q1 is None else 2
        A = q0.shape[1]
        S = A + 1
        lg = _row_view(logits, "logits", (B, L, V))
        qs = [_row_view(q, f"qs[{i}]", (B, A, V)) for i, q in enumerate((q0, q1)[:nq])]
        tqs = [_row_view(q, f"target_qs[{i}]", (B, A, V)) for i, q in enumerate((tq0, tq1)[:nq])]
        for t in qs + tqs:
            if t.dtype != lg.dtype:
                raise TypeError("logits, qs and target_qs must share one dtype")
        vflat = vs.reshape(B, S) if vs.numel() == B * S else None
        if vflat is None:
            raise ValueError(f"vs must hold [B, A+1] = [{B}, {S}] values, got {tuple(vs.shape)}")
        vflat = vflat.contiguous()
        if vflat.dtype not in (torch.float32, torch.bfloat16):
            vflat = vflat.float()
        ids = batch.input_ids.to(device=dev, dtype=torch.int64).contiguous()
        attn = batch.attention_mask.to(device=dev, dtype=torch.int64).contiguous()
        aix = batch.actions_ixs.to(device=dev, dtype=torch.int64).contiguous()
        dones = batch.dones.to(device=dev, dtype=torch.int64).contiguous()
        rew = batch.rewards.to(device=dev).contiguous()
        if rew.dtype not in (torch.float32, torch.bfloat16):
            rew = rew.float()
        for name, t, shp in (("input_ids", ids, (B, L)), ("attention_mask", attn, (B, L)),
                             ("actions_ixs", aix, (B, A)), ("dones", dones, (B, S)), ("rewards", rew, (B, A))):
            if tuple(t.shape) != shp:
                raise ValueError(f"batch.{name} must have shape {shp}, got {tuple(t.shape)}")

        dlg = grad_buffer_like(lg)
        dqs = [grad_buffer_like(q) for q in qs]
        dvs = torch.empty((B, S), dtype=torch.float32, device=dev)
        losses = torch.empty(5, dtype=torch.float32, device=dev)
        ws = torch.zeros(_lib.query("trlx_ilql_workspace_bytes", B, L, A, nq), dtype=torch.uint8, device=dev)

        a = _lib.IlqlArgs()
        a.dtype, a.nq, a.B, a.L, a.A, a.V = _lib.dtype_code(lg), nq, B, L, A, V
        a.logits = lg.data_ptr()
        a.logits_sb, a.logits_st = _strides(lg)
        a.dlogits = dlg.data_ptr()
        a.dlogits_sb, a.dlogits_st = _strides(dlg)
        for i in range(nq):
            a.q[i], a.tq[i], a.dq[i] = qs[i].data_ptr(), tqs[i].data_ptr(), dqs[i].data_ptr()
            a.q_sb[i], a.q_st[i] = _strides(qs[i])
            a.tq_sb[i], a.tq_st[i] = _strides(tqs[i])
            a.dq_sb[i], a.dq_st[i] = _strides(dqs[i])
        a.input_ids, a.attention_mask, a.actions_ixs, a.dones = (ids.data_ptr(), attn.data_ptr(), aix.data_ptr(),
                                                                 dones.data_ptr())
        a.rewards, a.rewards_dtype = rew.data_ptr(), _lib.dtype_code(rew)
        a.vs, a.vs_dtype = vflat.data_ptr(), _lib.dtype_code(vflat)
        a.tau, a.gamma, a.cql_scale, a.awac_scale = (float(cfg.tau), float(cfg.gamma), float(cfg.cql_scale),
                                                     float(cfg.awac_scale))
        a.dvs, a.losses, a.workspace = dvs.data_ptr(), losses.data_ptr(), ws.data_ptr()
        _lib.call("trlx_ilql_loss_fused", ctypes.byref(a), _lib.stream_of(lg))

        ctx.grads = [dlg] + dqs
        ctx.dvs = dvs
        ctx.meta = (logits.shape, [q.shape for q in (q0, q1)[:nq]], vs.shape, vs.dtype, nq)
        ctx.mark_non_differentiable(losses)
        return losses[0].clone(), losses

    @staticmethod
    def backward(ctx, grad_loss, grad_stats):
        if ctx.grads is None:
            raise RuntimeError("ILQL loss backward called twice (gradients are scaled in place)")
        grads, ctx.grads = ctx.grads, None
        g = grad_loss.to(torch.float32).reshape(1).contiguous()
        for t in grads:  # whole backing buffer; the kernel returns at once when grad_output == 1
            buf = t if t._base is None else t._base
            _lib.call("trlx_scale_by", _lib.ptr(buf), _lib.ptr(buf), _lib.dtype_code(buf), buf.numel(),
                      _lib.ptr(g), _lib.stream_of(buf))
        dvs = ctx.dvs
        _lib.call("trlx_scale_by", _lib.ptr(dvs), _lib.ptr(dvs), _lib.F32, dvs.numel(), _lib.ptr(g),
                  _lib.stream_of(dvs))
        lshape, qshapes, vshape, vdtype, nq = ctx.meta
        dvs = dvs.view(vshape).to(vdtype)
        dq = grads[1:] + [None] * (2 - nq)
        return None, grads[0], dvs, dq[0], dq[1], None, None, None


@dataclass
class ILQLConfig:
    """ILQL method config (ilql_models.py:37-49) with the loss on MI355X."""

    name: str = "ilqlconfig"
    tau: float = 0.7
    gamma: float = 0.99
    cql_scale: float = 0.1
    awac_scale: float = 1.0
    alpha: float = 0.001
    steps_for_target_q_sync: float = 5
    betas: Sequence[float] = (4,)
    two_qs: bool = True

    @classmethod
    def from_dict(cls, config: dict):
        return cls(**config)

    def loss(self, outputs: Any, labels: ILQLBatch):
        """ILQLConfig.loss (ilql_models.py:52-116): outputs = (logits, (qs, target_qs, vs)).

        Returns (loss, stats) with the reference's stats keys; stats values are 0-d device
        tensors ("losses/loss" is the loss itself).  Gradients reach logits, qs and vs.
        Deviation: with one action per row (A == 1) and B > 1 the reference's
        `vs[:, :-1].squeeze()` drops the action axis and broadcasts [B,1] against [B]
        into a [B,B] loss; that degenerate shape raises ValueError here."""
        logits, (qs, target_qs, vs) = outputs
        qs, target_qs = list(qs), list(target_qs)
        if len(qs) not in (1, 2) or len(target_qs) != len(qs):
            raise ValueError("ILQL needs 1 or 2 Q heads and as many target heads")
        _lib.require_cuda(logits, vs, *qs, *target_qs)
        B, A = qs[0].shape[0], qs[0].shape[1]
        if A == 1 and B > 1:
            raise ValueError("A == 1 with B > 1: the reference's squeeze() broadcasts [B,1] against [B] "
                             "(ilql_models.py:70-72); unsupported")
        q1 = qs[1] if len(qs) > 1 else None
        tq1 = target_qs[1] if len(qs) > 1 else None
        loss, losses = _ILQLLoss.apply(self, logits, vs, qs[0], q1, target_qs[0].detach(),
                                       None if tq1 is None else tq1.detach(), labels)
        stats = {k: (loss if k == "losses/loss" else losses[_SLOT[k]]) for k in ILQL_LOSS_KEYS}
        return loss, stats


class ILQLHotPath:
    """Device-resident ILQL loss step for one data-parallel shard (bench / training loop):
    gradient buffers and workspace allocated once per shape; one `step` is the three
    trlx_ilql_* launches (prep, rows, finalize) and allocates nothing.  The reference's
    ILQL loss has no collective (rank-local loss, DDP averages gradients), so shards are
    independent replicas."""

    def __init__(self, cfg: ILQLConfig, B: int, L: int, V: int, dtype: torch.dtype, device):
        self.cfg = cfg
        self.B, self.L, self.V, self.A = B, L, V, L - 1
        self.nq = 2 if cfg.two_qs else 1
        self.dtype = dtype
        self.device = torch.device(device)
        self.dvs = torch.empty((B, self.A + 1), dtype=torch.float32, device=self.device)
        self.losses = torch.empty(5, dtype=torch.float32, device=self.device)
        nbytes = _lib.query("trlx_ilql_workspace_bytes", B, L, self.A, self.nq)
        self.workspace = torch.zeros(nbytes, dtype=torch.uint8, device=self.device)  # tickets re-armed in-kernel
        self.dlogits = None
        self.dq = None
        self.timers = None  # optional {name: [[start_event, end_event], ...]}
        self.timer_names = None  # optional subset of launch names to instrument (None = all)

    def _timed(self, name, s, fn):
        if self.timers is None or (self.timer_names is not None and name not in self.timer_names):
            return fn()
        e0, e1 = make_event(), make_event()
        e0.record(s)
        fn()
        e1.record(s)
        self.timers.setdefault(name, []).append([e0, e1])

    def step(self, logits, qs, target_qs, vs, batch: ILQLBatch):
        B, L, V, A, nq = self.B, self.L, self.V, self.A, self.nq
        if tuple(logits.shape) != (B, L, V) or logits.dtype != self.dtype or logits.stride(-1) != 1:
            raise ValueError("logits do not match the hot path shape / dtype")
        qs, target_qs = list(qs), list(target_qs)
        if len(qs) != nq or len(target_qs) != nq:
            raise ValueError(f"the hot path was built for {nq} Q head(s) (two_qs={self.cfg.two_qs}); got "
                             f"{len(qs)} Q and {len(target_qs)} target-Q heads")
        for q in qs + target_qs:
            if tuple(q.shape) != (B, A, V) or q.dtype != self.dtype or q.stride(-1) != 1:
                raise ValueError("Q heads must be [B, L-1, V] of the logits dtype")
        _lib.require_cuda(logits, vs, batch.rewards, *qs, *target_qs)
        for name, t, shape in (("vs", vs, (B, A + 1)), ("batch.rewards", batch.rewards, (B, A))):
            ok_shape = tuple(t.shape) in (shape, shape + (1,))
            if not ok_shape or not t.is_contiguous() or t.dtype not in (torch.float32, torch.bfloat16):
                raise ValueError(f"{name} must be a contiguous fp32/bf16 {list(shape)} tensor (got "
                                 f"{tuple(t.shape)}/{t.dtype}, contiguous={t.is_contiguous()})")
        for name, shape in (("input_ids", (B, L)), ("attention_mask", (B, L)), ("actions_ixs", (B, A)),
                            ("dones", (B, A + 1))):
            if tuple(getattr(batch, name).shape) != shape:
                raise ValueError(f"batch.{name} has shape {tuple(getattr(batch, name).shape)}, expected {shape}")
        if self.dlogits is None or self.dlogits.stride() != logits.stride():
            self.dlogits = grad_buffer_like(logits)
            self.dq = [grad_buffer_like(q) for q in qs[:nq]]
        a = _lib.IlqlArgs()
        a.dtype, a.nq, a.B, a.L, a.A, a.V = _lib.dtype_code(logits), nq, B, L, A, V
        a.logits, (a.logits_sb, a.logits_st) = logits.data_ptr(), _strides(logits)
        a.dlogits, (a.dlogits_sb, a.dlogits_st) = self.dlogits.data_ptr(), _strides(self.dlogits)
        for i in range(nq):
            a.q[i], a.tq[i], a.dq[i] = qs[i].data_ptr(), target_qs[i].data_ptr(), self.dq[i].data_ptr()
            a.q_sb[i], a.q_st[i] = _strides(qs[i])
            a.tq_sb[i], a.tq_st[i] = _strides(target_qs[i])
            a.dq_sb[i], a.dq_st[i] = _strides(self.dq[i])
        for name in ("input_ids", "attention_mask", "actions_ixs", "dones"):
            t = getattr(batch, name)
            if t.dtype != torch.int64 or not t.is_contiguous():
                raise ValueError(f"batch.{name} must be contiguous int64")
            setattr(a, name, t.data_ptr())
        a.rewards, a.rewards_dtype = batch.rewards.data_ptr(), _lib.dtype_code(batch.rewards)
        a.vs, a.vs_dtype = vs.data_ptr(), _lib.dtype_code(vs)
        a.tau, a.gamma = float(self.cfg.tau), float(self.cfg.gamma)
        a.cql_scale, a.awac_scale = float(self.cfg.cql_scale), float(self.cfg.awac_scale)
        a.dvs, a.losses, a.workspace = self.dvs.data_ptr(), self.losses.data_ptr(), self.workspace.data_ptr()
        s = torch.cuda.current_stream(self.device)
        ref = ctypes.byref(a)
        self._timed("prep", s, lambda: _lib.call("trlx_ilql_prep", ref, s.cuda_stream))
        self._timed("rows", s, lambda: _lib.call("trlx_ilql_rows", ref, s.cuda_stream))
        self._timed("finalize", s, lambda: _lib.call("trlx_ilql_finalize", ref, s.cuda_stream))
        return self.losses, self.dlogits, self.dq, self.dvs


def ilql_sample_step(logits, target_qs, vs, beta=1.0, top_k=20, temperature=1.0, logit_mask=None,
                     input_ids=None, finished=None, eos_token_id=50256, generator=None):
    """One token of CausalLMWithValueHeads.generate (ilql_models.py:296-316) on MI355X.

    logits [B, V] (the last position), target_qs: one or two [B, V] heads, vs [B] or [B, 1];
    logit_mask: optional bool [V', V] indexed by input_ids[:, -1]; finished: optional int64
    [B] or [B, 1], updated in place.  Returns the sampled ids [B, 1] (int64).  The draw is
    the inverse CDF of pi at uniforms from `generator` (torch.rand on the device) instead of
    torch.multinomial's internal draw: same distribution, different random stream."""
    target_qs = list(target_qs) if isinstance(target_qs, (list, tuple)) else [target_qs]
    if len(target_qs) not in (1, 2):
        raise ValueError("one or two target Q heads")
    _lib.require_cuda(logits, vs, *target_qs)
    if logits.dim() != 2:
        raise ValueError("logits must be [B, V] (the last position)")
    B, V = logits.shape
    for q in target_qs:
        if tuple(q.shape) != (B, V) or q.dtype != logits.dtype:
            raise ValueError("target Q heads must match logits in shape and dtype")
    rows = [t if t.stride(-1) == 1 else t.contiguous() for t in [logits] + target_qs]
    v = vs.reshape(B).to(torch.float32).contiguous()
    dev = logits.device
    u = torch.rand(B, generator=generator, device=dev, dtype=torch.float32)
    out = torch.empty(B, dtype=torch.int64, device=dev)
    fin = None
    if finished is not None:
        fin = finished.reshape(B)
        if fin.dtype != torch.int64 or not fin.is_contiguous() or fin.data_ptr() != finished.data_ptr():
            raise ValueError("finished must be a contiguous int64 tensor (updated in place)")
    mask = prev = None
    if logit_mask is not None:
        if input_ids is None:
            raise ValueError("logit_mask needs input_ids")
        mask = logit_mask.to(device=dev)
        # bool and uint8 share the 1-byte layout: reinterpret instead of converting ([V', V]
        # masks can be vocab x vocab — a per-step conversion would copy the whole table)
        mask = mask.view(torch.uint8) if mask.dtype == torch.bool else mask.to(torch.uint8)
        if mask.stride(-1) != 1:
            mask = mask.contiguous()
        prev = input_ids[:, -1].to(device=dev, dtype=torch.int64).contiguous()
    q1 = rows[2] if len(rows) > 2 else None
    _lib.call("trlx_ilql_sample", rows[0].data_ptr(), rows[0].stride(0), rows[1].data_ptr(), rows[1].stride(0),
              _lib.ptr(q1), 0 if q1 is None else q1.stride(0), _lib.dtype_code(rows[0]), v.data_ptr(),
              _lib.ptr(mask), 0 if mask is None else mask.stride(0), _lib.ptr(prev), B, V, float(beta), int(top_k),
              float(temperature), u.data_ptr(), out.data_ptr(), _lib.ptr(fin), int(eos_token_id),
              _lib.stream_of(logits))
    return out.view(B, 1)
