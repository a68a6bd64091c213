"""Device-resident controller state of the PPO loop.

The reference keeps the loop's scalar state on the host:

  RunningMoments (mean, var, std, count)         trlx/utils/modeling.py:72-104
  ref_mean / ref_std + score scale / clip        trlx/orchestrator/ppo_orchestrator.py:48-49,96-112
  kl_ctl.value and its update(approx_kl, n)      trlx/model/nn/ppo_models.py:26-58,
                                                 accelerate_ppo_model.py:123,130-131

so every experience chunk and every backward round-trips through Python scalars (the
loss stats' `.item()`, RunningMoments attributes as numbers).  `PPOControlState` keeps all
of it in ONE fp64 record in HBM (layout: TRLX_CTL_* in include/trlx_t5_amd.h) that the
kernels read and advance in-stream:

  * `prepare_scores(scores)` — RunningMoments.update + first-batch ref stats + scale +
    clip, one single-workgroup launch (plus, under torch.distributed, one 32-B all-reduce
    of the score moments: get_global_statistics semantics);
  * `kl_update(approx_kl)` — kl_ctl.update with approx_kl read from device memory;
  * `PPOHotPath(..., ctl=state)` folds both into the fused step's two rollout tails, so the
    step stays four launches and needs no host synchronisation at all.

The record is double-buffered: a launch in which many workgroups read the state (the GAE
tail) writes the advanced copy to the other buffer; `cur` flips on the host (no sync).
Host values are available on demand (`host()`: one device->host copy).
"""
from typing import Optional

import torch
import torch.distributed as dist

from . import _lib

__all__ = ["PPOControlState"]

_SCALE = {False: _lib.SCALE_NONE, None: _lib.SCALE_NONE, "running": _lib.SCALE_RUNNING, "ref": _lib.SCALE_REF}


class PPOControlState:
    def __init__(self, device, init_kl_coef: float = 0.05, target: Optional[float] = 6, horizon: float = 10000,
                 scale_reward=False, cliprange_reward: Optional[float] = 10, ref_mean: Optional[float] = None,
                 ref_std: Optional[float] = None, n_steps: int = 1):
        if scale_reward not in _SCALE:
            raise ValueError(f"scale_reward must be False, 'running' or 'ref', got {scale_reward!r}")
        self.device = torch.device(device)
        self.adaptive = target is not None  # accelerate_ppo_model.py:43-48
        self.target = float(target) if target is not None else 0.0
        self.horizon = float(horizon)
        self.scale_mode = _SCALE[scale_reward]
        self.cliprange_reward = float(cliprange_reward or 0.0)
        self.n_steps = int(n_steps)
        self.buf = torch.empty((2, _lib.CTL_SLOTS), dtype=torch.float64, device=self.device)
        self.moments = torch.zeros(4, dtype=torch.float64, device=self.device)  # {Σx, Σx², n, 0}
        self.cur = 0
        s = torch.cuda.current_stream(self.device).cuda_stream
        # the orchestrator overwrites (ref_mean, ref_std) from the first batch iff ref_mean is None (:96-98)
        ref_set = ref_mean is not None
        _lib.call("trlx_ctl_init", self.buf[0].data_ptr(), float(init_kl_coef),
                  float(ref_mean) if ref_set else 0.0, float(ref_std) if ref_std is not None else float("nan"),
                  int(ref_set), s)

    @classmethod
    def from_config(cls, cfg, device, n_steps: int = 1):
        """From a PPOConfig (ppo_models.py:64-119 fields) and train.batch_size."""
        return cls(device, cfg.init_kl_coef, cfg.target, cfg.horizon, cfg.scale_reward, cfg.cliprange_reward,
                   cfg.ref_mean, cfg.ref_std, n_steps)

    # -------------------------------------------------------------- views (0-d device tensors)
    @property
    def state(self) -> torch.Tensor:
        return self.buf[self.cur]

    def _slot(self, k):
        return self.buf[self.cur, k]

    @property
    def kl_coef(self):
        return self._slot(_lib.CTL_KL_COEF)

    @property
    def mean(self):
        return self._slot(_lib.CTL_MEAN)

    @property
    def std(self):
        return self._slot(_lib.CTL_STD)

    @property
    def var(self):
        return self._slot(_lib.CTL_VAR)

    @property
    def count(self):
        return self._slot(_lib.CTL_COUNT)

    def host(self) -> dict:
        """All slots as Python floats (ONE device->host copy; for logging / checkpoints)."""
        v = self.state.to("cpu").tolist()
        names = ["mean", "var", "std", "count", "ref_mean", "ref_std", "ref_set", "kl_coef", "batch_mean",
                 "batch_std", "kl_updates", "last_kl"]
        return {n: v[i] for i, n in enumerate(names)}

    # -------------------------------------------------------------- C-ABI control blocks
    def _global_moments(self, scores, group=None, async_op=False):
        """Score moments all-reduced over ranks (None when torch.distributed is off)."""
        if not (dist.is_available() and dist.is_initialized()):
            return None, None
        _lib.call("trlx_score_moments", scores.data_ptr(), _lib.F32, scores.numel(), self.moments.data_ptr(),
                  _lib.stream_of(scores))
        work = dist.all_reduce(self.moments[:3], dist.ReduceOp.SUM, group=group, async_op=async_op)
        return self.moments, work

    def score_ctl(self, global_moments: Optional[torch.Tensor]):
        """trlx_score_ctl advancing buf[cur] -> buf[1-cur]; flips `cur`."""
        c = _lib.ScoreCtl(self.buf[self.cur].data_ptr(), self.buf[1 - self.cur].data_ptr(),
                          _lib.ptr(global_moments), self.scale_mode, self.cliprange_reward)
        self.cur = 1 - self.cur
        return c

    def kl_ctl(self):
        return _lib.KlCtl(self.buf[self.cur].data_ptr(), int(self.adaptive), self.target, self.horizon,
                          self.n_steps)

    # -------------------------------------------------------------- standalone entry points
    def prepare_scores(self, scores: torch.Tensor, group=None):
        """ppo_orchestrator.py:96-112 on device: returns (scores', batch_mean, batch_std) with
        scores' = clip(scores / scale, ±cliprange_reward) (fp32) and the RunningMoments.update
        return values as 0-d fp64 device tensors.  No host synchronisation."""
        _lib.require_cuda(scores)
        x = scores.to(torch.float32).contiguous()
        if x.numel() == 0:
            raise ValueError("prepare_scores: empty score batch")
        g, _ = self._global_moments(x, group)
        out = torch.empty_like(x)
        c = _lib.ScoreCtl(self.state.data_ptr(), self.state.data_ptr(), _lib.ptr(g), self.scale_mode,
                          self.cliprange_reward)
        _lib.call("trlx_score_ctl_update", x.data_ptr(), _lib.F32, x.numel(), c, out.data_ptr(), _lib.F32,
                  _lib.stream_of(x))
        return out, self._slot(_lib.CTL_BATCH_MEAN), self._slot(_lib.CTL_BATCH_STD)

    def kl_update(self, approx_kl: torch.Tensor, n_steps: Optional[int] = None):
        """kl_ctl.update(approx_kl, n_steps) (ppo_models.py:38-44) with approx_kl a device fp32
        scalar (e.g. PPOHotPath.stats[8]); in place, no host synchronisation."""
        _lib.require_cuda(approx_kl)
        k = approx_kl.to(torch.float32).reshape(-1)[:1].contiguous()
        kc = self.kl_ctl()
        if n_steps is not None:
            kc.n_steps = int(n_steps)
        _lib.call("trlx_kl_ctl_update", kc, k.data_ptr(), _lib.stream_of(k))
