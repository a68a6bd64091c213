"""The PPO experience + loss hot path for one data-parallel shard, device resident.

One `PPOHotPath.step` is, per response token of the shard:

  experience (ppo_orchestrator.py:154-167)
    K1  trlx_lsm_gather_fwd    policy + reference logits rows -> lp, ref_lp      (2 x V*s read)
  loss side (accelerate_ppo_model.py:88-126 -> ppo_models.py:121-199)
    K2  trlx_gae_scan          KL reward (fused) + GAE reverse scan + whitening moments,
                               last block reduces the moments (fixed order)
        [RCCL all-reduce of {sum A, sum A^2, n} when world > 1 — the only exchange]
    K3  trlx_ppo_policy_fused  new-policy logits rows -> lp_new, PPO policy grad, dlogits
                               (1 x V*s read + 1 x V*s write)
    K4  trlx_ppo_loss_elem     value loss + grads + stats partials; last block -> loss, 13 stats
        [RCCL all-reduce of the stats vector for logging when world > 1]

Buffers are allocated once per shape; the step launches four kernels and allocates
nothing.  Rows (rollouts) are sharded contiguously across ranks by the caller
(accelerate_ppo_model.py:146-148 semantics); reference-exact normalisers stay rank-local.
"""
from typing import Optional

import torch
import torch.distributed as dist

from . import _lib
from .modeling import grad_buffer_like
from .ppo import PPOConfig

__all__ = ["PPOHotPath"]


class PPOHotPath:
    def __init__(self, cfg: PPOConfig, B: int, T: int, V: int, logits_dtype: torch.dtype,
                 device, kl_coef: float, value_dtype: torch.dtype = torch.float32):
        self.cfg = cfg
        self.B, self.T, self.V = B, T, V
        self.dtype = logits_dtype
        self.device = torch.device(device)
        self.kl_coef = float(kl_coef)
        f32 = dict(dtype=torch.float32, device=self.device)
        self.lp_old = torch.empty((B, T), **f32)
        self.ref_lp = torch.empty((B, T), **f32)
        self.rewards = torch.empty((B, T), **f32)
        self.adv_raw = torch.empty((B, T), **f32)
        self.returns = torch.empty((B, T), dtype=value_dtype, device=self.device)
        self.lp_new = torch.empty((B, T), **f32)
        self.dvalues = torch.empty((B, T), **f32)
        self.n_gae = _lib.query("trlx_gae_num_blocks", B, T)
        self.gae_part = torch.empty(self.n_gae * _lib.MOMENT_SLOTS, dtype=torch.float64, device=self.device)
        self.adv_stats = torch.empty(_lib.MOMENT_SLOTS, dtype=torch.float64, device=self.device)
        self.n_loss = _lib.query("trlx_ppo_loss_num_blocks", B * T)
        self.loss_part = torch.empty(self.n_loss * _lib.PPO_PARTIAL_SLOTS, dtype=torch.float64, device=self.device)
        self.loss = torch.empty(1, **f32)
        self.tickets = torch.zeros(2, dtype=torch.int32, device=self.device)  # re-armed by the kernels
        self.stats = torch.empty(_lib.PPO_STATS, **f32)
        self.dlogits = None
        self.timers = None  # optional {name: [(start_event, end_event), ...]}

    # -------------------------------------------------------------- helpers
    def _ev(self, name, s):
        if self.timers is None:
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record(s)
        self.timers.setdefault(name, []).append([e, None])
        return e

    def _ev_end(self, name, s):
        if self.timers is None:
            return
        e = torch.cuda.Event(enable_timing=True)
        e.record(s)
        self.timers[name][-1][1] = e

    def _check(self, logits):
        if tuple(logits.shape) != (self.B, self.T, self.V) or logits.dtype != self.dtype or logits.stride(-1) != 1:
            raise ValueError(f"logits {tuple(logits.shape)}/{logits.dtype} do not match the hot path "
                             f"({self.B},{self.T},{self.V})/{self.dtype}")

    # -------------------------------------------------------------- experience
    def experience(self, logits, ref_logits, labels):
        """K1: lp, ref_lp (fp32) of the policy and reference logits at the response tokens."""
        self._check(logits)
        self._check(ref_logits)
        if logits.stride() != ref_logits.stride():
            raise ValueError("policy and reference logits must share strides")
        s = torch.cuda.current_stream(self.device)
        B, T, V = self.B, self.T, self.V
        self._ev("experience_lsm", s)
        _lib.call("trlx_lsm_gather_fwd", logits.data_ptr(), ref_logits.data_ptr(), _lib.dtype_code(logits),
                  B, T, V, logits.stride(0), logits.stride(1), labels.data_ptr(), labels.stride(0),
                  labels.stride(1), self.lp_old.data_ptr(), self.ref_lp.data_ptr(), _lib.F32, None, None,
                  s.cuda_stream)
        self._ev_end("experience_lsm", s)
        return self.lp_old, self.ref_lp

    # -------------------------------------------------------------- loss side
    def advantages(self, old_values, scores, lengths=None, mask=None, group=None):
        """K2+K3 (+ all-reduce): KL reward, GAE, global whitening moments."""
        s = torch.cuda.current_stream(self.device)
        B, T = self.B, self.T
        self._ev("gae", s)
        _lib.call("trlx_gae_scan", old_values.data_ptr(), None, _lib.dtype_code(old_values), B, T, T,
                  float(self.cfg.gamma), float(self.cfg.lam), self.lp_old.data_ptr(), self.ref_lp.data_ptr(),
                  -self.kl_coef, _lib.ptr(scores), _lib.ptr(lengths), _lib.ptr(mask), self.adv_raw.data_ptr(),
                  self.returns.data_ptr(), _lib.dtype_code(self.returns), self.rewards.data_ptr(), _lib.F32,
                  self.gae_part.data_ptr(), self.adv_stats.data_ptr(), self.tickets[0:1].data_ptr(), s.cuda_stream)
        self._ev_end("gae", s)
        self.distributed = dist.is_available() and dist.is_initialized()
        if self.distributed:
            dist.all_reduce(self.adv_stats[:3], dist.ReduceOp.SUM, group=group)
        return self.adv_raw, self.returns

    def policy_loss(self, new_logits, labels, values, old_values, mask=None):
        """K4-K6: fused logprob + PPO grads + dlogits, then the loss and its stats."""
        self._check(new_logits)
        if self.dlogits is None or self.dlogits.stride() != new_logits.stride():
            self.dlogits = grad_buffer_like(new_logits)
        s = torch.cuda.current_stream(self.device)
        B, T, V = self.B, self.T, self.V
        n = B * T
        unbiased = 0 if self.distributed else 1
        msum = self.adv_stats[3:4]  # rank-local sum of the loss mask (ppo_models.py:162,177)
        dx = self.dlogits
        self._ev("loss_fused", s)
        _lib.call("trlx_ppo_policy_fused", new_logits.data_ptr(), _lib.dtype_code(new_logits), B, T, V,
                  new_logits.stride(0), new_logits.stride(1), labels.data_ptr(), labels.stride(0),
                  labels.stride(1), self.lp_old.data_ptr(), _lib.F32, self.adv_raw.data_ptr(),
                  self.adv_stats.data_ptr(), unbiased, _lib.ptr(mask), msum.data_ptr(), float(n),
                  float(self.cfg.cliprange), self.lp_new.data_ptr(), dx.data_ptr(), dx.stride(0), dx.stride(1),
                  s.cuda_stream)
        self._ev_end("loss_fused", s)
        self._ev("loss_stats", s)
        _lib.call("trlx_ppo_loss_elem", n, self.lp_new.data_ptr(), _lib.F32, values.data_ptr(),
                  _lib.dtype_code(values), self.lp_old.data_ptr(), _lib.F32, old_values.data_ptr(),
                  _lib.dtype_code(old_values), self.adv_raw.data_ptr(), _lib.F32, self.adv_stats.data_ptr(),
                  unbiased, self.returns.data_ptr(), _lib.dtype_code(self.returns), _lib.ptr(mask),
                  msum.data_ptr(), float(n), float(self.cfg.cliprange), float(self.cfg.cliprange_value),
                  float(self.cfg.vf_coef), None, self.dvalues.data_ptr(), _lib.F32, self.loss_part.data_ptr(),
                  self.loss.data_ptr(), self.stats.data_ptr(), self.tickets[1:2].data_ptr(), s.cuda_stream)
        self._ev_end("loss_stats", s)
        return self.loss, self.stats, self.dlogits, self.dvalues

    def step(self, logits, ref_logits, new_logits, labels, old_values, values, scores,
             lengths: Optional[torch.Tensor] = None, mask: Optional[torch.Tensor] = None, group=None,
             reduce_stats: bool = True):
        self.experience(logits, ref_logits, labels)
        self.advantages(old_values, scores, lengths=lengths, mask=mask, group=group)
        out = self.policy_loss(new_logits, labels, values, old_values, mask=mask)
        if reduce_stats and self.distributed:
            dist.all_reduce(self.stats, dist.ReduceOp.SUM, group=group)  # logging: mean over ranks
        return out
