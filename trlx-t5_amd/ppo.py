"""Drop-in for the PPO hot path of trlx/model/nn/ppo_models.py and the orchestrator's
KL-penalised reward step (trlx/orchestrator/ppo_orchestrator.py) on MI355X.

  AdaptiveKLController / FixedKLController   ppo_models.py:26-58   (host scalars)
  PPOConfig.get_advantages_and_returns       ppo_models.py:121-139 (HIP GAE scan + whiten)
  PPOConfig.loss                             ppo_models.py:141-199 (HIP loss + grads, autograd)
  PPOConfig.loss_from_logits                 fused A1+A6: one read + one write of each logits row
  prepare_scores                             ppo_orchestrator.py:96-112
  kl_penalty_rewards                         ppo_orchestrator.py:163-167
"""
from dataclasses import dataclass, field
from typing import Any, Dict, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import _lib
from .lm_head import lm_head_logprobs
from .modeling import (RunningMoments, _allreduce_moments, _token_geometry, flatten_dict,
                       grad_buffer_like, whiten)

__all__ = ["AdaptiveKLController", "FixedKLController", "PPOConfig", "kl_penalty_rewards",
           "prepare_scores", "STATS_KEYS", "stats_dict"]


# ------------------------------------------------------------------ KL controllers (A8)
class AdaptiveKLController:
    """beta_{t+1} = beta_t * (1 + clip(KL/target - 1, +-0.2) * n_steps / horizon)  (ppo_models.py:26-44)."""

    def __init__(self, init_kl_coef: float, target: float, horizon: int):
        self.value = init_kl_coef
        self.target = target
        self.horizon = horizon

    def update(self, current: float, n_steps: int):
        err = np.clip(current / self.target - 1, -0.2, 0.2)
        self.value *= 1 + err * n_steps / self.horizon


class FixedKLController:
    """Constant beta (ppo_models.py:47-58)."""

    def __init__(self, kl_coef):
        self.value = kl_coef

    def update(self, current: float, n_steps: int):
        pass


# ------------------------------------------------------------------ stats layout (A6)
STATS_KEYS = (  # order written by trlx_ppo_loss_finalize (ppo_models.py:182-198, flattened)
    "losses/total_loss", "losses/policy_loss", "losses/value_loss",
    "values/mean_old_values", "values/var_old_values", "values/mean_values", "values/values_error",
    "values/clipfrac", "policy/approx_kl", "policy/clipfrac", "returns/mean", "returns/var", "ratio",
)
_FLOAT_KEYS = {"losses/total_loss", "losses/policy_loss", "losses/value_loss", "policy/approx_kl",
               "policy/clipfrac"}  # the reference .item()s these five (ppo_models.py:184-195)


def stats_dict(stats_dev: torch.Tensor) -> dict:
    """Build the reference's flattened stats dict from the device stats vector: Python
    floats for the five keys the reference .item()s (one D2H copy for all five, instead of
    five syncs), 0-d device tensors for the rest."""
    host = stats_dev.detach().to("cpu", non_blocking=False).tolist()
    out = {}
    for i, k in enumerate(STATS_KEYS):
        out[k] = host[i] if k in _FLOAT_KEYS else stats_dev[i]
    return out


# ------------------------------------------------------------------ A2
def prepare_scores(scores: torch.Tensor, running: RunningMoments, scale_reward, cliprange_reward,
                   ref_std=None):
    """Score scaling / clipping of ppo_orchestrator.py:96-112 in ONE device launch
    (trlx_score_ctl_update on the RunningMoments record: the batch moments, the Chan merge,
    then clip(scores / scale, ±cliprange_reward)); no host synchronisation.

    Returns (scores, batch_mean, batch_std).  `ref_std` is the std of the first rollout's
    scores when scale_reward == "ref" (the caller keeps it, as the orchestrator does).
    Under torch.distributed the batch moments are all-reduced first (RunningMoments.update's
    get_global_statistics branch, modeling.py:85-86).
    """
    mode = {False: _lib.SCALE_NONE, None: _lib.SCALE_NONE, "running": _lib.SCALE_RUNNING,
            "ref": _lib.SCALE_REF}.get(scale_reward)
    if mode is None:
        raise ValueError(f"scale_reward must be False, 'running' or 'ref', got {scale_reward!r}")
    if mode == _lib.SCALE_REF and ref_std is None:
        raise ValueError("scale_reward='ref' needs ref_std (the first rollout's score std)")
    return running._update_scaled(scores, mode, float(cliprange_reward or 0.0), ref_std)


def kl_penalty_rewards(logprobs: torch.Tensor, ref_logprobs: torch.Tensor, kl_coef: float,
                       scores: Optional[torch.Tensor] = None,
                       lengths: Optional[torch.Tensor] = None) -> torch.Tensor:
    """rewards = -kl_coef * (logprobs - ref_logprobs); rewards[:, -1] += scores
    (ppo_orchestrator.py:164-167).  With `lengths`, the score lands on each row's last
    valid column and columns beyond it are zero padding.  Output dtype = logprobs dtype."""
    _lib.require_cuda(logprobs, ref_logprobs)
    lp = logprobs.contiguous()
    rlp = ref_logprobs.to(lp.dtype).contiguous()
    B, T = lp.shape
    sc = None if scores is None else scores.to(device=lp.device, dtype=torch.float32).contiguous()
    ln = None if lengths is None else lengths.to(device=lp.device, dtype=torch.int64).contiguous()
    out = torch.empty_like(lp)
    _lib.call("trlx_kl_penalty_rewards", _lib.ptr(lp), _lib.ptr(rlp), _lib.dtype_code(lp), B, T,
              float(kl_coef), _lib.ptr(sc), _lib.ptr(ln), _lib.ptr(out), _lib.dtype_code(out),
              _lib.stream_of(lp))
    return out


# ------------------------------------------------------------------ A6 autograd
class _PPOLoss(torch.autograd.Function):
    """Forward runs the loss kernels, which also produce d loss/d logprobs and d loss/d values
    (closed form, elementwise); backward scales them by grad_output on device."""

    @staticmethod
    def forward(ctx, logprobs, values, old_logprobs, old_values, advantages, returns, mask, c, cv, vf_coef):
        dev = logprobs.device
        n = logprobs.numel()
        ts = [t.contiguous() for t in (logprobs, values, old_logprobs, old_values, advantages, returns)]
        lp, v, olp, ov, adv, ret = ts
        m = None
        msum_dev = None
        s = _lib.stream_of(lp)
        if mask is not None:
            m = mask.to(device=dev, dtype=torch.int64).contiguous()
            part = torch.empty(_lib.query("trlx_moments_num_blocks", n) * _lib.MOMENT_SLOTS,
                               dtype=torch.float64, device=dev)
            mst = torch.empty(_lib.MOMENT_SLOTS, dtype=torch.float64, device=dev)
            _lib.call("trlx_moments_partial", _lib.ptr(m), _lib.I64, n, _lib.ptr(part), s)
            _lib.call("trlx_moments_finalize", _lib.ptr(part), part.numel() // _lib.MOMENT_SLOTS,
                      _lib.ptr(mst), s)
            msum_dev = mst[0:1]
        gdt = torch.float32
        dlp = torch.empty(lp.shape, dtype=gdt, device=dev)
        dv = torch.empty(v.shape, dtype=gdt, device=dev)
        nblk = _lib.query("trlx_ppo_loss_num_blocks", n)
        part = torch.empty(nblk * _lib.PPO_PARTIAL_SLOTS, dtype=torch.float64, device=dev)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        stats = torch.empty(_lib.PPO_STATS, dtype=torch.float32, device=dev)
        ticket = torch.zeros(1, dtype=torch.int32, device=dev)
        _lib.call("trlx_ppo_loss_elem", n, _lib.ptr(lp), _lib.dtype_code(lp), _lib.ptr(v), _lib.dtype_code(v),
                  _lib.ptr(olp), _lib.dtype_code(olp), _lib.ptr(ov), _lib.dtype_code(ov),
                  _lib.ptr(adv), _lib.dtype_code(adv), None, 0, _lib.ptr(ret), _lib.dtype_code(ret),
                  _lib.ptr(m), _lib.ptr(msum_dev), float(n), float(c), float(cv), float(vf_coef),
                  _lib.ptr(dlp), _lib.ptr(dv), _lib.F32, _lib.ptr(part), _lib.ptr(loss), _lib.ptr(stats),
                  _lib.ptr(ticket), s)
        ctx.save_for_backward(dlp, dv)
        ctx.dtypes = (logprobs.dtype, values.dtype)
        ctx.shapes = (logprobs.shape, values.shape)
        ctx.stats = stats
        ctx.mark_non_differentiable(stats)
        return loss, stats

    @staticmethod
    def backward(ctx, grad_loss, grad_stats):
        dlp, dv = ctx.saved_tensors
        g = grad_loss.to(torch.float32).reshape(1).contiguous()
        outs = []
        for t, dt, shp in ((dlp, ctx.dtypes[0], ctx.shapes[0]), (dv, ctx.dtypes[1], ctx.shapes[1])):
            o = torch.empty_like(t)
            _lib.call("trlx_scale_by", _lib.ptr(t), _lib.ptr(o), _lib.F32, t.numel(), _lib.ptr(g),
                      _lib.stream_of(t))
            outs.append(o.view(shp).to(dt))
        return outs[0], outs[1], None, None, None, None, None, None, None, None


class _PPOLossFromLogits(torch.autograd.Function):
    """Fused loss side: logprob forward + PPO policy gradient + dlogits in ONE pass over
    each logits row (vocab_rows.hip, kPpo), then the [B,T] loss/stats kernels.  Backward
    returns the already-written dlogits (scaled in place by grad_output, a no-op for 1)."""

    @staticmethod
    def forward(ctx, logits, values, labels, old_logprobs, old_values, adv_raw, adv_stats, unbiased,
                returns, mask, c, cv, vf_coef):
        dev = logits.device
        lg, lb, (B, T, V, sb, st), (l0, l1) = _token_geometry(logits, labels)
        n = B * T
        s = _lib.stream_of(lg)
        olp = old_logprobs.contiguous()
        adv = adv_raw.to(torch.float32).contiguous()
        m = None if mask is None else mask.to(device=dev, dtype=torch.int64).contiguous()
        msum_dev = None
        if m is not None:
            part = torch.empty(_lib.query("trlx_moments_num_blocks", n) * _lib.MOMENT_SLOTS,
                               dtype=torch.float64, device=dev)
            mst = torch.empty(_lib.MOMENT_SLOTS, dtype=torch.float64, device=dev)
            _lib.call("trlx_moments_partial", _lib.ptr(m), _lib.I64, n, _lib.ptr(part), s)
            _lib.call("trlx_moments_finalize", _lib.ptr(part), part.numel() // _lib.MOMENT_SLOTS,
                      _lib.ptr(mst), s)
            msum_dev = mst[0:1]
        lp_new = torch.empty((B, T), dtype=torch.float32, device=dev)
        dx = grad_buffer_like(lg)
        dsb, dst = (dx.stride(0), dx.stride(1)) if dx.dim() == 3 else (dx.stride(0), 0)
        _lib.call("trlx_ppo_policy_fused", _lib.ptr(lg), _lib.dtype_code(lg), B, T, V, sb, st, _lib.ptr(lb),
                  l0, l1, _lib.ptr(olp), _lib.dtype_code(olp), _lib.ptr(adv), _lib.ptr(adv_stats),
                  int(unbiased), _lib.ptr(m), _lib.ptr(msum_dev), float(n), float(c), _lib.ptr(lp_new),
                  _lib.ptr(dx), dsb, dst, s)
        v = values.contiguous()
        ov = old_values.contiguous()
        ret = returns.contiguous()
        dv = torch.empty(v.shape, dtype=torch.float32, device=dev)
        nblk = _lib.query("trlx_ppo_loss_num_blocks", n)
        part = torch.empty(nblk * _lib.PPO_PARTIAL_SLOTS, dtype=torch.float64, device=dev)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        stats = torch.empty(_lib.PPO_STATS, dtype=torch.float32, device=dev)
        ticket = torch.zeros(1, dtype=torch.int32, device=dev)
        _lib.call("trlx_ppo_loss_elem", n, _lib.ptr(lp_new), _lib.F32, _lib.ptr(v), _lib.dtype_code(v),
                  _lib.ptr(olp), _lib.dtype_code(olp), _lib.ptr(ov), _lib.dtype_code(ov),
                  _lib.ptr(adv), _lib.F32, _lib.ptr(adv_stats), int(unbiased), _lib.ptr(ret),
                  _lib.dtype_code(ret), _lib.ptr(m), _lib.ptr(msum_dev), float(n), float(c), float(cv),
                  float(vf_coef), None, _lib.ptr(dv), _lib.F32, _lib.ptr(part), _lib.ptr(loss),
                  _lib.ptr(stats), _lib.ptr(ticket), s)
        ctx.save_for_backward(dv)
        ctx.dx = dx
        ctx.shapes = (logits.shape, lg is logits, values.shape, values.dtype)
        ctx.mark_non_differentiable(stats, lp_new)
        return loss, stats, lp_new

    @staticmethod
    def backward(ctx, grad_loss, grad_stats, grad_lp):
        (dv,) = ctx.saved_tensors
        dx = ctx.dx
        if dx is None:
            raise RuntimeError("loss_from_logits backward called twice (dlogits are scaled in place)")
        ctx.dx = None
        g = grad_loss.to(torch.float32).reshape(1).contiguous()
        s = _lib.stream_of(dx)
        # scale the whole backing buffer in place (gaps of a strided view included, harmless);
        # the kernel returns immediately when grad_output == 1
        buf = dx if dx._base is None else dx._base
        _lib.call("trlx_scale_by", _lib.ptr(buf), _lib.ptr(buf), _lib.dtype_code(buf), buf.numel(),
                  _lib.ptr(g), s)
        dvo = torch.empty_like(dv)
        _lib.call("trlx_scale_by", _lib.ptr(dv), _lib.ptr(dvo), _lib.F32, dv.numel(), _lib.ptr(g), s)
        lshape, same, vshape, vdt = ctx.shapes
        dvo = dvo.view(vshape)
        if vdt != torch.float32:
            dvo = dvo.to(vdt)
        return ((dx if same else dx.reshape(lshape)), dvo, None, None, None, None, None, None, None,
                None, None, None, None)


# ------------------------------------------------------------------ PPOConfig (A5, A6)
@dataclass
class PPOConfig:
    """Method config of ppo_models.py:64-119 with the hot-path methods on MI355X."""

    name: str = "ppoconfig"
    ppo_epochs: int = 4
    num_rollouts: int = 128
    chunk_size: int = 128
    init_kl_coef: float = 0.05
    target: Optional[float] = 6
    horizon: int = 10000
    gamma: float = 1.0
    lam: float = 0.95
    cliprange: float = 0.2
    cliprange_value: float = 0.2
    vf_coef: float = 1.0
    scale_reward: Any = False
    ref_mean: Optional[float] = None
    ref_std: Optional[float] = None
    cliprange_reward: float = 10
    gen_kwargs: Dict[str, Any] = field(default_factory=dict)

    @classmethod
    def from_dict(cls, config: Dict[str, Any]):
        return cls(**config)

    # -------------------------------------------------------------- A5
    def gae_raw(self, values: torch.Tensor, rewards: torch.Tensor, response_length: int,
                lengths: Optional[torch.Tensor] = None, mask: Optional[torch.Tensor] = None):
        """Unwhitened GAE on device.  Returns (adv_raw fp32 [B,L], returns [B,L] values.dtype,
        moments fp64 [4] = {sum A, sum A^2, count, sum mask})."""
        _lib.require_cuda(values, rewards)
        v = values.contiguous()
        r = rewards.to(v.dtype).contiguous()
        B, T = v.shape
        L = int(response_length)
        dev = v.device
        s = _lib.stream_of(v)
        adv = torch.empty((B, L), dtype=torch.float32, device=dev)
        ret = torch.empty((B, L), dtype=v.dtype, device=dev)
        nblk = _lib.query("trlx_gae_num_blocks", B, L)
        part = torch.empty(nblk * _lib.MOMENT_SLOTS, dtype=torch.float64, device=dev)
        st = torch.empty(_lib.MOMENT_SLOTS, dtype=torch.float64, device=dev)
        ln = None if lengths is None else lengths.to(device=dev, dtype=torch.int64).contiguous()
        mk = None if mask is None else mask.to(device=dev, dtype=torch.int64).contiguous()
        ticket = torch.zeros(1, dtype=torch.int32, device=dev)
        _lib.call("trlx_gae_scan", _lib.ptr(v), _lib.ptr(r), _lib.dtype_code(v), B, T, L, float(self.gamma),
                  float(self.lam), None, None, 0.0, None, _lib.ptr(ln), _lib.ptr(mk), _lib.ptr(adv),
                  _lib.ptr(ret), _lib.dtype_code(ret), None, _lib.F32, _lib.ptr(part), _lib.ptr(st),
                  _lib.ptr(ticket), s)
        return adv, ret, st

    def get_advantages_and_returns(self, values: torch.Tensor, rewards: torch.Tensor, response_length: int,
                                   use_whitening: Optional[bool] = True) -> Tuple[torch.Tensor, torch.Tensor]:
        """GAE advantages and returns (ppo_models.py:121-139): one reverse-scan launch instead
        of the reference's ~5 launches per time step; whitening from the scan's own moments."""
        adv, ret, st = self.gae_raw(values, rewards, response_length)
        if use_whitening:
            use_dist = dist.is_available() and dist.is_initialized()
            if use_dist:
                _allreduce_moments(st)
            out = torch.empty(adv.shape, dtype=values.dtype, device=adv.device)
            _lib.call("trlx_whiten_apply", _lib.ptr(adv), _lib.F32, adv.numel(), _lib.ptr(st),
                      0 if use_dist else 1, 1, _lib.ptr(out), _lib.dtype_code(out), _lib.stream_of(adv))
            adv = out
        else:
            adv = adv.to(values.dtype)
        return adv.detach(), ret

    # -------------------------------------------------------------- A6
    def loss(self, logprobs, values, old_logprobs, old_values, advantages, returns, mask,
             return_device_stats=False):
        """PPO clipped-surrogate + clipped value loss (ppo_models.py:141-199).

        Returns (loss, stats) with the reference's flattened stats keys and value types (or the
        fp32 device stats vector in STATS_KEYS order when return_device_stats=True: no host
        sync).  Gradients flow to `logprobs` and `values` (closed form, computed in the forward
        kernel, scaled by grad_output in backward)."""
        _lib.require_cuda(logprobs, values, old_logprobs, old_values, advantages, returns)
        loss, stats = _PPOLoss.apply(logprobs, values, old_logprobs, old_values, advantages, returns, mask,
                                     self.cliprange, self.cliprange_value, self.vf_coef)
        return loss, (stats if return_device_stats else stats_dict(stats))

    def loss_from_hidden(self, hidden, weight, values, labels, old_logprobs, old_values, advantages, returns,
                         mask=None, plan="auto", return_device_stats=False):
        """The loss side from the policy's last hidden states:
            self.loss(logprobs_from_logits(hidden @ weight.T, labels), values, ...)
        (accelerate_ppo_model.py:96-118 with the lm_head of ppo_models.py:640 / :274), the
        [.., V] logits and dlogits never in HBM: lm_head_logprobs' differentiable MFMA block
        feeds the PPO loss kernels, and backward() delivers d hidden, d weight (lm_head) and
        d values.  hidden [.., H] / weight [V, H] bf16 (H in lm_head.GRAD_HIDDEN_SIZES: the fused
        backward; other H: hipBLASLt bf16 logits + the row kernels, the reference's structure).
        plan: lm_head_logprobs' dW plan ("auto": the forward's bf16 P kept for the backward — 3
        MFMA passes, 2·N·V bytes held until backward — falling back to recomputing S when that
        buffer cannot be allocated; "saved_p"; "recompute").
        Returns (loss, stats) like loss(); logprobs are kept in fp32 (the reference's bf16
        logits give bf16 logprobs)."""
        # the loss multiplies every lp term by `mask`: the fused lm_head skips the masked tokens
        lp = lm_head_logprobs(hidden, weight, labels, out_dtype=torch.float32, plan=plan, mask=mask)
        return self.loss(lp, values, old_logprobs, old_values, advantages, returns, mask,
                         return_device_stats=return_device_stats)

    def loss_from_logits(self, logits, values, labels, old_logprobs, old_values, advantages, returns,
                         mask=None, adv_stats=None, unbiased=True, return_device_stats=False):
        """Fused loss side: equivalent to
            lp = logprobs_from_logits(logits, labels); self.loss(lp, values, ...)
        but with one HBM read + one write of each logits row.  `advantages` are whitened on
        the fly when adv_stats (fp64 {sum, sumsq, n}) is given (unbiased: var_mean branch).
        Returns (loss, stats_dict, lp_new) — or the fp32 device stats vector when
        return_device_stats=True (no host sync)."""
        _lib.require_cuda(logits, values, labels, old_logprobs, old_values, advantages, returns)
        loss, stats, lp_new = _PPOLossFromLogits.apply(
            logits, values, labels, old_logprobs, old_values, advantages, adv_stats, unbiased, returns, mask,
            self.cliprange, self.cliprange_value, self.vf_coef)
        return loss, (stats if return_device_stats else stats_dict(stats)), lp_new
