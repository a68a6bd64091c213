"""The PPO experience + loss hot path for one data-parallel shard, device resident.

One `PPOHotPath.step` is four kernel launches (plus, when world > 1, one 24-byte RCCL
all-reduce between the two halves):

  experience  trlx_lsm_gather_fwd          policy + reference logits rows -> lp, ref_lp
                                           (2 x V*s read / token; ppo_orchestrator.py:154-155)
              trlx_ppo_rollout_gae         one wave per rollout: KL-penalised rewards, GAE
                                           advantages + returns, whitening moments
                                           {Σ A, Σ A², n, Σ mask} (ppo_orchestrator.py:163-167,
                                           ppo_models.py:121-136, modeling.py:24-29)
      [RCCL all-reduce of {Σ A, Σ A², n} when world > 1 -- the only data-path exchange]
  loss        trlx_ppo_loss_rows           new-policy rows -> lp_new, PPO policy gradient,
                                           dlogits (V*s read + V*s write / token), d values,
                                           per-token loss terms (ppo_models.py:141-199)
              trlx_ppo_rollout_loss        fixed-order loss sums -> loss + 13 stats
      [optional RCCL all-reduce of the stats vector for logging (reduce_stats=True)]

With `ctl=PPOControlState(...)` the scores pass through the device
RunningMoments + scale/clip inside the GAE tail and beta is read from / advanced in device
memory by the two tails (kl_ctl.update(approx_kl) after the loss): still four launches, no
host synchronisation; under torch.distributed one more 32-B all-reduce (score moments)
overlaps the experience logits pass.

Buffers (and the zero-filled ticket workspace) are allocated once per shape; a step
allocates nothing.  Rows (rollouts) are sharded contiguously across ranks by the caller
(accelerate_ppo_model.py:146-148 semantics); reference-exact loss normalisers stay
rank-local unless loss_norm="global" (Σmask then rides the whitening all-reduce).
"""
from typing import Optional

import ctypes

import torch
import torch.distributed as dist

from . import _lib
from .modeling import grad_buffer_like
from .control import PPOControlState
from .ppo import PPOConfig
from .comm import RcclComm
from .timing import LaunchEvent, make_event

__all__ = ["PPOHotPath"]


class _StreamJoin:
    """A pending side-stream all-reduce: wait() orders the current stream after it (a no-op
    for one enqueued on the step's own stream).  Mirrors the torch Work.wait() the hot path
    calls for torch.distributed collectives."""

    __slots__ = ("_ev", "_dev", "_joined")

    def __init__(self, ev, device):
        self._ev, self._dev, self._joined = ev, device, None

    def wait(self):
        # a stream wait is a barrier packet that idles the queue ~5 us even when already
        # satisfied: a stream that has joined once is ordered after it for good
        s = torch.cuda.current_stream(self._dev)
        if self._ev is not None and self._joined != s.cuda_stream:
            self._ev.wait(s)
            self._joined = s.cuda_stream


class _Works:
    """Several torch.distributed async works waited together."""

    __slots__ = ("_ws",)

    def __init__(self, ws):
        self._ws = ws

    def wait(self):
        for w in self._ws:
            w.wait()


class PPOHotPath:
    _comm_timing_events = False  # A/B knob: timing-capable events for the comm joins
    _fold_gae = True  # A/B knob: pipeline_step runs GAE(k+1) inside the L rows(k) launch (else its own launch)
    _derive_coef = True  # A/B knob: split loss rows derive the whitening coefficients (else a coefficient launch)
    def __init__(self, cfg: PPOConfig, B: int, T: int, V: int, logits_dtype: torch.dtype,
                 device, kl_coef: float, value_dtype: torch.dtype = torch.float32,
                 ctl: Optional[PPOControlState] = None, overlap_tail: bool = False, loss_norm: str = "rank",
                 defer_tail: bool = False, comm: Optional[RcclComm] = None, split_beta: bool = False):
        self.cfg = cfg
        # split_beta: step() runs the split-beta GAE / loss rows (trlx_ppo_rollout_gae_split,
        # trlx_ppo_loss_rows_split) that pipeline_step always uses: A = A0 - beta*Ak, beta
        # applied by the loss rows.  Same arithmetic as pipeline_step, so the two schedules
        # agree bit for bit; the unsplit kernels differ from it only by fp32 association.
        self.split_beta = bool(split_beta)
        self._sbuf = None  # split-beta buffer sets (two: the pipeline's batches k and k+1)
        self._sidx = 0     # the set the current batch uses
        self._lag = False      # pipelined under DP without running-std scaling: score moments merged one batch late
        self._mom_bufs = None  # lag: per-batch score moments {Σx, Σx², n, 0} (two, by batch parity)
        # comm: the boundary's RCCL helper (comm.RcclComm) for the step's all-reduces instead
        # of torch.distributed — enqueued on the step's stream (blocking schedule) or on a side
        # stream joined with fence-free events (pipelined schedule, score moments)
        self.comm = comm
        self._comm_stream = None
        self._comm_events = [LaunchEvent(timing=self._comm_timing_events) for _ in range(8)] \
            if comm is not None else None
        self._comm_ev_i = 0
        self._comm_inline = False
        self._ar_unissued = None  # pipelined + comm: whitening record waiting for the next _begin_step
        # defer_tail: the loss tail of step k runs as the first workgroups of step k+1's
        # experience rows launch (trlx_lsm_gather_fwd_loss_tail) instead of its own launch on
        # the critical path; loss / stats / beta of the last step are final after wait_stats()
        # (which launches a still-pending tail by itself).
        if defer_tail and overlap_tail:
            raise ValueError("defer_tail and overlap_tail are alternatives")
        self.defer_tail = bool(defer_tail)
        self._tail_pending = None
        # loss_norm: "rank" = the reference's rank-local loss normalisers Σmask
        # (ppo_models.py:162,177; DDP then averages the per-rank gradients); "global" = the
        # whitening all-reduce also carries Σmask and each rank divides by Σmask_global / W, so
        # the DDP-averaged gradient is that of the masked mean over the GLOBAL batch (SURVEY
        # §8e: identical to "rank" with all-ones masks or equal Σmask per rank).
        if loss_norm not in ("rank", "global"):
            raise ValueError(f"loss_norm must be 'rank' or 'global', not {loss_norm!r}")
        self.loss_norm = loss_norm
        self.B, self.T, self.V = B, T, V
        self.dtype = logits_dtype
        self.device = torch.device(device)
        self.kl_coef = float(kl_coef)
        self.ctl = ctl  # device-resident RunningMoments / score clip / KL controller (control.py)
        # overlap_tail: the latency-bound loss tail runs on a side stream, beside the NEXT
        # step's experience rows (it only reads the token records and Σmask, which nothing
        # before the next GAE tail rewrites); loss / stats are ready at `tail_done`.
        self.tail_stream = torch.cuda.Stream(self.device) if overlap_tail else None
        self.tail_done = None
        # fence-free events (timing.LaunchEvent), two of each reused alternately: a default
        # event's system-scope fence on record idles the queue for microseconds
        self._sync_events = [LaunchEvent() for _ in range(4)] if overlap_tail else None
        self._sync_i = 0
        f32 = dict(dtype=torch.float32, device=self.device)
        self.lp_old = torch.empty((B, T), **f32)
        self.ref_lp = torch.empty((B, T), **f32)
        self.rewards = torch.empty((B, T), **f32)
        self.adv_raw = self._adv_raw4 = torch.empty((B, T), **f32)  # split-beta: the set's A0
        self.returns = torch.empty((B, T), dtype=value_dtype, device=self.device)
        self.lp_new = torch.empty((B, T), **f32)
        self.dvalues = torch.empty((B, T), **f32)
        self._stats4 = torch.empty(_lib.MOMENT_SLOTS, dtype=torch.float64, device=self.device)
        self.adv_stats = self._stats4  # the current batch's whitening record (split-beta: its 8-slot set)
        self._split_mode = False  # how the current batch's GAE ran (the loss launch must match)
        self._coef_ready = False  # split: the batch's whitening coefficients were folded into a GAE launch
        self._ar_msum = None      # global loss norm: the Σmask slot of the record in flight
        self.loss = torch.empty(1, **f32)
        self.stats = torch.empty(_lib.PPO_STATS, **f32)
        nbytes = _lib.query("trlx_ppo_workspace_bytes", B, T)
        self.workspace = torch.zeros(nbytes, dtype=torch.uint8, device=self.device)  # tickets re-armed in-kernel
        self.dlogits = None
        self.lm_ws = None  # lm_head partials workspace (experience_from_hidden)
        self.lm_logits = None  # [2, B, T, V] bf16 logits of the GEMM route (experience_from_hidden)
        self.lm_loss_ws = None  # the fused loss side's workspace (policy_loss_from_hidden)
        self.distributed = False  # whether the current whitening record is all-reduced (set per experience)
        self._loss_ws_fallback = False  # plan "auto" fell back to the recompute plan (allocation failed)
        self.timers = None  # optional {name: [(start_event, end_event), ...]} (recorded when set)
        self.timer_names = None  # optional subset of launch names to instrument (None = all)
        self._conv = {}  # int64 buffers for labels / mask / lengths given in another integer dtype
        self._order_ws = None  # a ragged batch's row order (trlx_ragged_order_bytes; trlx_lsm_gather_fwd_ragged)
        self._ar_work = None  # pending whitening all-reduce (pipelined schedule)
        self._ar_group = None
        self._lp_bufs = None  # pipelined schedule: two (lp_old, ref_lp) pairs
        self._pending = None  # pipelined schedule: the loss-side inputs of the previous batch

    # -------------------------------------------------------------- helpers
    def _ev(self, name, s):
        if self.timers is None or (self.timer_names is not None and name not in self.timer_names):
            return None
        e = make_event()
        e.record(s)
        self.timers.setdefault(name, []).append([e, None])
        return e

    def _ev_end(self, name, s):
        if self.timers is None or (self.timer_names is not None and name not in self.timer_names):
            return
        e = make_event()
        e.record(s)
        self.timers[name][-1][1] = e

    def _check(self, logits):
        if tuple(logits.shape) != (self.B, self.T, self.V) or logits.dtype != self.dtype or logits.stride(-1) != 1:
            raise ValueError(f"logits {tuple(logits.shape)}/{logits.dtype} do not match the hot path "
                             f"({self.B},{self.T},{self.V})/{self.dtype}")
        if logits.device != self.device:
            raise ValueError(f"logits on {logits.device}, hot path on {self.device}")

    def _int64(self, t, shape, name, required=True):
        """The kernels read labels / mask / lengths as contiguous int64 on this device.  int64
        inputs pass through; other integer or bool dtypes (a bool or int32 attention mask) are
        converted into a buffer owned by the hot path (allocated once, refilled per call)."""
        if t is None:
            if required:
                raise ValueError(f"{name} is required")
            return None
        if tuple(t.shape) != tuple(shape):
            raise ValueError(f"{name} has shape {tuple(t.shape)}, expected {tuple(shape)}")
        if t.device != self.device:
            raise ValueError(f"{name} on {t.device}, hot path on {self.device}")
        if t.is_floating_point() or t.is_complex():
            raise ValueError(f"{name} must be an integer or bool tensor, not {t.dtype}")
        if t.dtype == torch.int64 and t.is_contiguous():
            return t
        buf = self._conv.get(name)
        if buf is None:
            buf = self._conv[name] = torch.empty(tuple(shape), dtype=torch.int64, device=self.device)
        buf.copy_(t)
        return buf

    def _vec(self, t, shape, name, dtypes=(torch.float32, torch.bfloat16)):
        """[B, T] / [B] float vectors (values, old_values: fp32 or bf16; scores: fp32), contiguous."""
        if t is None and name == "scores" and self.ctl is None:
            return None  # no score term (the KL penalty alone)
        if t is None or tuple(t.shape) != tuple(shape):
            raise ValueError(f"{name} has shape {None if t is None else tuple(t.shape)}, expected {tuple(shape)}")
        if t.device != self.device or not t.is_contiguous() or t.dtype not in dtypes:
            raise ValueError(f"{name} must be a contiguous {'/'.join(str(d)[6:] for d in dtypes)} tensor on "
                             f"{self.device} (got {t.dtype}, contiguous={t.is_contiguous()}, {t.device})")
        return t

    # -------------------------------------------------------------- collectives
    def _begin_step(self, scores, group, s, lag=False):
        """Whether the step is distributed, and the score moments all-reduce (device controller
        state under DP) issued so it overlaps the experience rows: (global moments, work).
        lag (pipelined, no running-std scaling): nothing here — this batch's moments ride the
        side-stream segment issued after its GAE launch (_experience_tail)."""
        self.distributed = self.comm is not None or (dist.is_available() and dist.is_initialized())
        if lag:
            return None, None
        if self.comm is None:
            if self.ctl is None:
                return None, None
            return self.ctl._global_moments(scores, group, async_op=True)
        # RCCL helper: the previous pipelined batch's whitening record (held back by
        # _experience_tail) and these score moments share ONE side-stream segment and join
        ts = [] if self._ar_unissued is None else [self._ar_unissued]
        ready = None
        if self.ctl is not None:
            ready = None if self._comm_inline else self._comm_event()
            if ready is None:
                _lib.call("trlx_score_moments", scores.data_ptr(), _lib.F32, scores.numel(),
                          self.ctl.moments.data_ptr(), s.cuda_stream)
            else:  # the side stream's ordering point rides the moments kernel's dispatch
                _lib.call("trlx_score_moments_signal", scores.data_ptr(), _lib.F32, scores.numel(),
                          self.ctl.moments.data_ptr(), s.cuda_stream, ready.handle)
            ts.append(self.ctl.moments[:3])
        join = self._side_allreduce(ts, s, ready) if ts else None
        if self._ar_unissued is not None:
            self._ar_unissued, self._ar_work = None, join
        return (self.ctl.moments, join) if self.ctl is not None else (None, None)

    def _comm_event(self):
        ev = self._comm_events[self._comm_ev_i]
        self._comm_ev_i = (self._comm_ev_i + 1) % len(self._comm_events)
        return ev

    def _score_moments(self, scores, mom, stream):
        _lib.call("trlx_score_moments", scores.data_ptr(), _lib.F32, scores.numel(), mom.data_ptr(), stream.cuda_stream)

    def _side_allreduce(self, ts, s, ready=None, issued=False):
        """comm.allreduce_ of each tensor in `ts` (each its own collective, the same sizes as
        the blocking schedule's, so every element is summed in the same order) on a side
        stream after what `s` has queued; the returned handle's wait() orders the then-current
        stream after them (ordering-only fence-free events: one join per call)."""
        if self._comm_inline:  # A/B only: on `s` itself (no overlap, no joins)
            for t in ts:
                self.comm.allreduce_(t, s)
            return _StreamJoin(None, self.device)
        if self._comm_stream is None:
            self._comm_stream = torch.cuda.Stream(self.device)
        ev_in, ev_out = ready, self._comm_event()
        if ev_in is None:  # `ready`: already recorded on `s` by the last launch
            ev_in = self._comm_event()
            ev_in.record(s)
        if not issued:  # issued: the side stream already waits on `ready`
            ev_in.wait(self._comm_stream)
        for t in ts:
            self.comm.allreduce_(t, self._comm_stream)
        ev_out.record(self._comm_stream)
        return _StreamJoin(ev_out, self.device)

    def _rollout_inputs(self, labels, lengths, mask, old_values, scores):
        B, T = self.B, self.T
        return (self._int64(labels, (B, T), "labels"), self._int64(lengths, (B,), "lengths", required=False),
                self._int64(mask, (B, T), "mask", required=False), self._vec(old_values, (B, T), "old_values"),
                self._vec(scores, (B,), "scores", (torch.float32,)))

    # -------------------------------------------------------------- K1
    def _no_pipeline_pending(self, what):
        """The serial entry points after pipeline_step: its last batch's loss (and, under the lag
        schedule, that batch's RunningMoments merge) exist only inside the pipeline until
        pipeline_flush(); a serial call would silently drop them."""
        if self._pending is not None or self._lag:
            raise RuntimeError(f"{what}: pipeline_step has a pending batch (its loss"
                               f"{' and score-moments merge' if self._lag else ''} not yet run): "
                               f"call pipeline_flush() first")

    def experience(self, logits, ref_logits, labels, old_values, scores, lengths=None, mask=None, group=None):
        """K1 (+ all-reduce): lp, ref_lp, KL rewards, GAE, global whitening moments."""
        self._no_pipeline_pending("experience")
        self._check(logits)
        self._check(ref_logits)
        if logits.stride() != ref_logits.stride():
            raise ValueError("policy and reference logits must share strides")
        B, T, V = self.B, self.T, self.V
        labels, lengths, mask, old_values, scores = self._rollout_inputs(labels, lengths, mask, old_values, scores)
        s = torch.cuda.current_stream(self.device)
        self._use_split(self.split_beta, 0)
        g_mom, work = self._begin_step(scores, group, s)
        self._experience_rows(logits, ref_logits, labels, s, lengths)
        self._experience_tail(s, labels, old_values, scores, lengths, mask, group, g_mom, work)
        return self.lp_old, self.ref_lp

    def _use_split(self, split, idx):
        """Select the unsplit GAE / loss kernels or the split-beta ones with buffer set `idx`."""
        self._split_mode, self._sidx, self._coef_ready = bool(split), idx, False
        if split and self._sbuf is None:
            f32 = dict(dtype=torch.float32, device=self.device)
            self._sbuf = [dict(adv0=torch.empty((self.B, self.T), **f32), adv_kl=torch.empty((self.B, self.T), **f32),
                               rew_kl=torch.empty((self.B, self.T), **f32),
                               rew_score=torch.empty((self.B, self.T), **f32),
                               stats=torch.zeros(_lib.SPLIT_MOMENT_SLOTS, dtype=torch.float64, device=self.device),
                               coef=torch.zeros(4, **f32)) for _ in range(2)]
        if split:
            sb = self._sbuf[idx]
            self.adv_stats, self.adv_raw = sb["stats"], sb["adv0"]
        else:
            self.adv_stats, self.adv_raw = self._stats4, self._adv_raw4

    def _experience_rows(self, logits, ref_logits, labels, s, lengths=None, b0=0, timed=True):
        """Policy + reference rows of rollouts [b0, b0 + logits.shape[0]) -> lp_old, ref_lp.
        lengths (a ragged batch): rows past each rollout's length are store padding, lp = 0,
        not read (trlx_lsm_gather_fwd_ragged)."""
        B, T, V = logits.shape[0], self.T, self.V
        rows = (logits.data_ptr(), ref_logits.data_ptr(), _lib.dtype_code(logits), B, T, V, logits.stride(0),
                logits.stride(1), labels.data_ptr(), labels.stride(0), labels.stride(1))
        outs = (self.lp_old[b0].data_ptr(), self.ref_lp[b0].data_ptr(), _lib.F32)
        order = self._order_scratch() if lengths is not None else None
        if timed:
            self._ev("experience", s)
        if self._tail_pending is not None:  # the previous step's loss tail rides this launch
            pend, self._tail_pending = self._tail_pending, None
            _lib.call("trlx_lsm_gather_fwd_loss_tail", *rows, _lib.ptr(lengths), order, *outs, *self._tail_args(pend),
                      s.cuda_stream)
        elif lengths is not None:
            _lib.call("trlx_lsm_gather_fwd_ragged", *rows, lengths.data_ptr(), order, *outs, s.cuda_stream)
        else:
            _lib.call("trlx_lsm_gather_fwd", *rows, *outs, None, None, s.cuda_stream)
        if timed:
            self._ev_end("experience", s)

    def _order_scratch(self):
        """Device scratch of a ragged batch's row order (trlx_ragged_order_bytes)."""
        if self._order_ws is None:
            self._order_ws = torch.empty(_lib.query("trlx_ragged_order_bytes", self.B, self.T), dtype=torch.uint8,
                                         device=self.device)
        return self._order_ws.data_ptr()

    def _launch_pending_tail(self, s):
        """Run a deferred loss tail by itself (nothing to fold it into)."""
        if self._tail_pending is None:
            return
        pend, self._tail_pending = self._tail_pending, None
        B, T, st, vf, loss, stats, ws, kl = self._tail_args(pend)
        if kl is not None:
            _lib.call("trlx_ppo_rollout_loss_ctl", B, T, st, vf, loss, stats, ws, kl, s.cuda_stream)
        else:
            _lib.call("trlx_ppo_rollout_loss", B, T, st, vf, loss, stats, ws, s.cuda_stream)

    def _tail_args(self, pend):
        """A deferred loss tail's arguments, its KL-controller record resolved NOW: the tail
        updates beta in the record current when it runs (after any GAE launch that advanced
        the double-buffered state in between — the split-beta pipeline's order)."""
        return pend + ((self.ctl.kl_ctl() if self.ctl is not None else None),)

    # hidden size from which the fused lm_head loses to hipBLASLt + the rows kernel
    # (profiles/r01_lmhead_route_sweep.log: fused 1.00-1.08x at H <= 1024, 0.93-0.95x from
    # H = 1536 up to UL2's 4096)
    LM_HEAD_GEMM_MIN_H = 1280
    # gemm route: logits of at most this many tokens per model exist at a time (a ring of
    # [2, chunk, T, V] bf16, 0.5 GB at V = 32128 instead of [2, B, T, V]); measured at the C4
    # shard (profiles/r03_lmhead_chunk.log): 4096-token chunks 1.006x the full-batch GEMM + rows,
    # 2048 0.979x, 1024 0.904x (hipBLASLt loses efficiency on short M)
    LM_HEAD_CHUNK_TOKENS = 4096

    def experience_from_hidden(self, hidden, weight, ref_hidden, ref_weight, labels, old_values, scores,
                               lengths=None, mask=None, group=None, route="auto"):
        """K1 with the lm_head folded in: lp / ref_lp straight from the policy's
        and the reference model's last hidden states ([B, T, H] bf16) and lm_head weights
        ([V, H] bf16) — `logits = lm_head(h)` (ppo_models.py:640, :274, :588) followed by
        logprobs_from_logits (ppo_orchestrator.py:154-155) without the [B, T, V] logits ever
        reaching HBM (two MFMA launches, trlx_lmhead_logprobs) — then the same GAE tail.

        route: "fused" (above), "gemm" (hipBLASLt writes bf16 logits — the reference's own
        bf16 lm_head output — then the experience rows kernel), or "auto" = "gemm" from
        H >= LM_HEAD_GEMM_MIN_H on a bf16 hot path (long K, where the fused kernel is slower).

        Rounding differs by route: "gemm" rounds every logit to bf16 before the log-softmax, as
        the reference's bf16 lm_head does (ppo_models.py:615,640); "fused" keeps the fp32 MFMA
        accumulator (closer to exact).  lp therefore moves by up to ~1 bf16 ulp of the logits
        between the routes (tests/test_gpu_lmhead.py pins both against fp64 at realistic logit
        scale).  The gemm route keeps a [2, chunk, T, V] bf16 ring (LM_HEAD_CHUNK_TOKENS tokens per
        chunk: the full [2, B, T, V] logits never exist); release_lm_logits() frees it."""
        self._no_pipeline_pending("experience_from_hidden")
        self._check_hidden(hidden, weight, ref_hidden, ref_weight)
        labels, lengths, mask, old_values, scores = self._rollout_inputs(labels, lengths, mask, old_values, scores)
        route = self._lm_route(route, hidden, ref_hidden)
        s = torch.cuda.current_stream(self.device)
        if route == "fused":
            self._launch_pending_tail(s)
        self._use_split(self.split_beta, 0)
        g_mom, work = self._begin_step(scores, group, s)
        self._experience_lmhead(hidden, weight, ref_hidden, ref_weight, labels, lengths, s, route)
        self._experience_tail(s, labels, old_values, scores, lengths, mask, group, g_mom, work)
        return self.lp_old, self.ref_lp

    def _check_hidden(self, hidden, weight, ref_hidden, ref_weight):
        B, T, V = self.B, self.T, self.V
        for h, w in ((hidden, weight), (ref_hidden, ref_weight)):
            if h.dim() != 3 or tuple(h.shape[:2]) != (B, T) or w.dim() != 2 or w.shape[0] != V or \
                    w.shape[1] != h.shape[2] or h.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
                raise ValueError(f"hidden {tuple(h.shape)}/{h.dtype} and weight {tuple(w.shape)}/{w.dtype} do not "
                                 f"match the hot path ({B},{T},H) x ({V},H) bf16")

    def _lm_route(self, route, hidden, ref_hidden):
        if route not in ("auto", "fused", "gemm"):
            raise ValueError(f"route must be auto, fused or gemm, not {route!r}")
        if route == "gemm" and self.dtype != torch.bfloat16:
            raise ValueError("the gemm route writes bf16 logits: it needs a bf16 hot path")
        if route == "auto":
            long_k = min(hidden.shape[2], ref_hidden.shape[2]) >= self.LM_HEAD_GEMM_MIN_H
            route = "gemm" if long_k and self.dtype == torch.bfloat16 else "fused"
        return route

    def _experience_lmhead(self, hidden, weight, ref_hidden, ref_weight, labels, lengths, s, route):
        """The policy and reference lm_heads + logprobs into lp_old / ref_lp (the current
        buffer set): the fused MFMA launches, or hipBLASLt logits over rollout chunks + the
        experience rows (a deferred loss tail riding the first rows launch)."""
        B, T, V = self.B, self.T, self.V
        if route == "gemm":
            # rollout chunks: hipBLASLt writes the chunk's policy and reference logits into the
            # ring, one rows launch reads both (the deferred loss tail rides the first)
            _lib.require_cuda(hidden, weight, ref_hidden, ref_weight)
            cb = max(1, min(B, self.LM_HEAD_CHUNK_TOKENS // T))
            if self.lm_logits is None or self.lm_logits.shape[1] != cb:
                self.lm_logits = torch.empty((2, cb, T, V), dtype=torch.bfloat16, device=self.device)
            self._ev("experience", s)
            for b0 in range(0, B, cb):
                nb = min(cb, B - b0)
                x0, x1 = self.lm_logits[0, :nb], self.lm_logits[1, :nb]
                torch.matmul(hidden[b0:b0 + nb], weight.t(), out=x0)
                torch.matmul(ref_hidden[b0:b0 + nb], ref_weight.t(), out=x1)
                self._experience_rows(x0, x1, labels[b0:b0 + nb], s, None if lengths is None else lengths[b0:b0 + nb],
                                      b0=b0, timed=False)
            self._ev_end("experience", s)
            return
        self._launch_pending_tail(s)
        N = B * T
        nbytes = _lib.query("trlx_lmhead_workspace_bytes", N, V)
        if self.lm_ws is None or self.lm_ws.numel() < nbytes:
            self.lm_ws = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        self._ev("experience", s)
        for h, w, out in ((hidden, weight, self.lp_old), (ref_hidden, ref_weight, self.ref_lp)):
            H = h.shape[2]
            if h.stride(2) != 1 or h.stride(1) % 8 or h.stride(0) != T * h.stride(1) or h.data_ptr() % 16:
                h = h.contiguous()
            if w.stride(1) != 1 or w.stride(0) % 8 or w.data_ptr() % 16:
                w = w.contiguous()
            if lengths is not None:  # ragged: the padding's tokens skip the GEMM tiles (lp = 0)
                _lib.call("trlx_lmhead_logprobs_ragged", h.data_ptr(), h.stride(1), w.data_ptr(), w.stride(0), N, H,
                          V, labels.data_ptr(), 1, lengths.data_ptr(), T, self._order_scratch(), out.data_ptr(),
                          _lib.F32, None, self.lm_ws.data_ptr(), s.cuda_stream)
            else:
                _lib.call("trlx_lmhead_logprobs", h.data_ptr(), h.stride(1), w.data_ptr(), w.stride(0), N, H, V,
                          labels.data_ptr(), 1, out.data_ptr(), _lib.F32, None, self.lm_ws.data_ptr(), s.cuda_stream)
        self._ev_end("experience", s)

    def _experience_tail(self, s, labels, old_values, scores, lengths, mask, group, g_mom, work,
                         defer_allreduce=False, lag=False, launch=True):
        """GAE tail (+ the whitening all-reduce).  Split-beta mode: trlx_ppo_rollout_gae_split
        into the current buffer set.  lag: g_mom holds the PREVIOUS batch's all-reduced score
        moments (merged into RunningMoments by this launch), and this batch's moments +
        whitening record are all-reduced on a side-stream segment that starts at this launch's
        own completion signal and has the next batch's loss and experience rows to hide behind.
        launch=False (split mode, the pipelined schedule): the GAE's arguments are returned
        instead of launched — the caller folds the GAE into the previous batch's loss rows
        launch (trlx_ppo_loss_rows_split_gae) and then calls _gae_done() with them."""
        B, T = self.B, self.T
        if work is not None:
            work.wait()
        if self.tail_done is not None:  # previous loss tail: reads Σmask + token records, updates beta
            self.tail_done.wait(s)
        tail = (B, T, self.lp_old.data_ptr(), self.ref_lp.data_ptr(), old_values.data_ptr(),
                _lib.dtype_code(old_values), _lib.ptr(scores), _lib.ptr(lengths), _lib.ptr(mask))
        if self._split_mode:
            sb = self._sbuf[self._sidx]
            done = self._comm_event() if (lag and self.distributed and self.comm is not None
                                          and not self._comm_inline) else None
            beta_state = self.ctl.state.data_ptr() if self.ctl is not None else None  # the GAE's state_in
            ctl = self.ctl.score_ctl(g_mom) if self.ctl is not None else None
            # {Σ A0, Σ A0², n, Σ Ak, Σ A0·Ak, Σ Ak²} (+ Σmask for the global loss normaliser)
            gd = dict(rec=sb["stats"][:7 if self.loss_norm == "global" else 6], msum=sb["stats"][6:7], done=done,
                      scores=scores, group=group, lag=lag, defer=defer_allreduce, beta_state=beta_state, ctl=ctl)
            if not launch:
                gd["args"] = _lib.GaeSplitArgs(
                    *tail, ctypes.pointer(ctl) if ctl is not None else None, self.kl_coef, float(self.cfg.gamma),
                    float(self.cfg.lam), sb["adv0"].data_ptr(), sb["adv_kl"].data_ptr(), sb["rew_kl"].data_ptr(),
                    sb["rew_score"].data_ptr(), sb["stats"].data_ptr(), int(lag), self.workspace.data_ptr())
                return gd
            self._ev("rollout_gae", s)
            _lib.call("trlx_ppo_rollout_gae_split", *tail, ctl, self.kl_coef, float(self.cfg.gamma),
                      float(self.cfg.lam), sb["adv0"].data_ptr(), sb["adv_kl"].data_ptr(), sb["rew_kl"].data_ptr(),
                      sb["rew_score"].data_ptr(), sb["stats"].data_ptr(), None, None, 0, int(lag),
                      self.workspace.data_ptr(), s.cuda_stream, done.handle if done is not None else None)
            self._ev_end("rollout_gae", s)
        else:
            self._ev("rollout_gae", s)
            outs = (float(self.cfg.gamma), float(self.cfg.lam), self.rewards.data_ptr(), self.adv_raw.data_ptr(),
                    self.returns.data_ptr(), _lib.dtype_code(self.returns), self.adv_stats.data_ptr(),
                    self.workspace.data_ptr(), s.cuda_stream)
            if self.ctl is not None:
                _lib.call("trlx_ppo_rollout_gae_ctl", *tail, self.ctl.score_ctl(g_mom), *outs)
            else:
                _lib.call("trlx_ppo_rollout_gae", *tail, self.kl_coef, *outs)
            self._ev_end("rollout_gae", s)
            # {Σ A, Σ A², n} (+ Σmask for the global loss normaliser): the only data-path exchange
            gd = dict(rec=self.adv_stats[:4 if self.loss_norm == "global" else 3], msum=self.adv_stats[3:4],
                      done=None, scores=scores, group=group, lag=lag, defer=defer_allreduce)
        self._gae_done(gd, s)

    def _gae_done(self, gd, s):
        """After the GAE launch (its own, or the loss rows launch it rode): the whitening
        record's all-reduce — blocking, deferred to the next _begin_step, or (lag) on the
        side-stream segment behind the launch's done event."""
        rec, msum, group = gd["rec"], gd["msum"], gd["group"]
        if gd["lag"] and self.distributed:
            self._ar_group, self._ar_msum = group, msum
            mom = self._mom_bufs[self._sidx]
            scores, done = gd["scores"], gd["done"]
            if self.comm is not None:  # one side-stream segment: moments kernel + both all-reduces
                self._ar_unissued = None
                if self._comm_inline:
                    self._score_moments(scores, mom, s)
                    self._ar_work = self._side_allreduce([rec, mom[:3]], s)
                else:
                    if self._comm_stream is None:
                        self._comm_stream = torch.cuda.Stream(self.device)
                    done.wait(self._comm_stream)
                    # the side stream reads the caller's scores: keep their memory from being
                    # handed to a later allocation until that read has run (the caller
                    # typically drops a batch's scores right after pipeline_step returns)
                    scores.record_stream(self._comm_stream)
                    self._score_moments(scores, mom, self._comm_stream)
                    self._ar_work = self._side_allreduce([rec, mom[:3]], s, ready=done, issued=True)
            else:
                self._score_moments(scores, mom, s)
                self._ar_work = _Works([dist.all_reduce(rec, dist.ReduceOp.SUM, group=group, async_op=True),
                                        dist.all_reduce(mom[:3], dist.ReduceOp.SUM, group=group, async_op=True)])
            return
        if self.distributed:
            self._ar_group, self._ar_msum = group, msum
            if self.comm is not None:
                if gd["defer"]:  # issued with the next batch's score moments (_begin_step)
                    self._ar_unissued, self._ar_work = rec, None
                else:  # on the step's own stream: ordered with no join at all
                    self.comm.allreduce_(rec, s)
                    self._ar_work = _StreamJoin(None, self.device)
            else:
                self._ar_work = dist.all_reduce(rec, dist.ReduceOp.SUM, group=group, async_op=True)
            if not gd["defer"]:
                self._resolve_allreduce()

    def _resolve_allreduce(self):
        """Order the current stream after the pending whitening all-reduce (RCCL: a stream
        wait, no host sync) and finish the global loss normaliser."""
        if self._ar_unissued is not None:  # the last pipelined batch: nothing left to hide it behind
            self.comm.allreduce_(self._ar_unissued, torch.cuda.current_stream(self.device))
            self._ar_unissued, self._ar_work = None, _StreamJoin(None, self.device)
        w, self._ar_work = self._ar_work, None
        if w is None:
            return
        w.wait()
        if self.loss_norm == "global":
            world = self.comm.nranks if self.comm is not None else dist.get_world_size(self._ar_group)
            self._ar_msum.div_(world)

    # -------------------------------------------------------------- K2
    def policy_loss(self, new_logits, labels, values, old_values, mask=None, _fold=None):
        """K2: fused logprob + PPO grads + dlogits, value loss, loss + stats.  (_fold: the
        pipelined schedule's next-batch split GAE, _experience_tail(launch=False), run as the
        first workgroups of this launch; _gae_done() follows.)"""
        self._check(new_logits)
        B, T, V = self.B, self.T, self.V
        labels = self._int64(labels, (B, T), "labels")
        mask = self._int64(mask, (B, T), "mask", required=False)
        values = self._vec(values, (B, T), "values")
        old_values = self._vec(old_values, (B, T), "old_values")
        if self.dlogits is None or self.dlogits.stride() != new_logits.stride():
            self.dlogits = grad_buffer_like(new_logits)
        s = torch.cuda.current_stream(self.device)
        # the previous loss tail still to read the token records / loss / stats this launch
        # rewrites (a second policy_loss per experience, the ppo_epochs pattern): deferred ->
        # run it now; on the side stream -> wait for it
        self._launch_pending_tail(s)
        if self.tail_done is not None:
            self.tail_done.wait(s)
        dx = self.dlogits
        rows = (new_logits.data_ptr(), _lib.dtype_code(new_logits), B, T, V, new_logits.stride(0),
                new_logits.stride(1), labels.data_ptr(), labels.stride(0), labels.stride(1), self.lp_old.data_ptr(),
                _lib.F32)
        grads = (float(self.cfg.cliprange), float(self.cfg.cliprange_value), float(self.cfg.vf_coef),
                 self.lp_new.data_ptr(), dx.data_ptr(), dx.stride(0), dx.stride(1), self.dvalues.data_ptr(),
                 self.workspace.data_ptr())
        if _fold is not None and not (self._split_mode and not self._coef_ready):
            raise RuntimeError("a folded GAE rides the first split-beta loss launch of an experience")
        if self._split_mode:
            sb = self._sbuf[self._sidx]
            split = (sb["adv0"].data_ptr(), sb["adv_kl"].data_ptr(), sb["rew_kl"].data_ptr(),
                     sb["rew_score"].data_ptr())
            vals = (sb["stats"].data_ptr() + 6 * 8, _lib.ptr(mask), values.data_ptr(), _lib.dtype_code(values),
                    old_values.data_ptr(), _lib.dtype_code(old_values), self.rewards.data_ptr(),
                    self.returns.data_ptr(), _lib.dtype_code(self.returns))
            self._ev("loss", s)
            if not self._coef_ready and not self._derive_coef and _fold is None:  # A/B: the coefficient launch
                _lib.call("trlx_ppo_whiten_coef", sb["stats"].data_ptr(), 0 if self.distributed else 1,
                          self.ctl.state.data_ptr() if self.ctl is not None else None, self.kl_coef,
                          sb["coef"].data_ptr(), s.cuda_stream)
                self._coef_ready = True
            if self._coef_ready:  # a second loss on this experience (ppo_epochs): the stored coefficients
                _lib.call("trlx_ppo_loss_rows_split", *rows, *split, sb["coef"].data_ptr(), *vals, *grads,
                          s.cuda_stream)
            else:  # the rows derive the whitening coefficients (beta: the state the GAE read) and store them
                if _fold is not None:
                    beta_state = _fold["beta_state"]
                else:
                    beta_state = self.ctl.state.data_ptr() if self.ctl is not None else None
                done = _fold["done"] if _fold is not None else None
                _lib.call("trlx_ppo_loss_rows_split_gae", *rows, *split, sb["stats"].data_ptr(),
                          0 if self.distributed else 1, beta_state, self.kl_coef, sb["coef"].data_ptr(), *vals,
                          *grads, ctypes.byref(_fold["args"]) if _fold is not None else None, s.cuda_stream,
                          done.handle if done is not None else None)
                self._coef_ready = True
            tail_stats = sb["stats"].data_ptr() + 3 * 8  # the tail reads Σmask at stats[3]
        else:
            self._ev("loss", s)
            _lib.call("trlx_ppo_loss_rows", *rows, self.adv_raw.data_ptr(), self.adv_stats.data_ptr(),
                      0 if self.distributed else 1, _lib.ptr(mask), values.data_ptr(), _lib.dtype_code(values),
                      old_values.data_ptr(), _lib.dtype_code(old_values), self.returns.data_ptr(),
                      _lib.dtype_code(self.returns), *grads, s.cuda_stream)
            tail_stats = self.adv_stats.data_ptr()
        self._ev_end("loss", s)
        self._loss_tail(s, tail_stats)
        return self.loss, self.stats, self.dlogits, self.dvalues

    def _loss_tail(self, s, tail_stats):
        """The loss tail after a loss launch (fixed-order sums of the token records -> loss + 13
        stats, + the KL-controller update): deferred into the next experience launch, on the
        side stream, or its own launch."""
        ts = s
        if self.tail_stream is not None:
            rows_done = self._next_event()
            rows_done.record(s)
            ts = self.tail_stream
            rows_done.wait(ts)
        args = (self.B, self.T, tail_stats, float(self.cfg.vf_coef), self.loss.data_ptr(), self.stats.data_ptr(),
                self.workspace.data_ptr())
        if self.defer_tail:  # runs inside the next experience launch (or wait_stats)
            self._tail_pending = args
            return
        self._ev("rollout_loss", ts)
        if self.ctl is not None:  # + kl_ctl.update(approx_kl) (accelerate_ppo_model.py:123,130-131)
            _lib.call("trlx_ppo_rollout_loss_ctl", *args, self.ctl.kl_ctl(), ts.cuda_stream)
        else:
            _lib.call("trlx_ppo_rollout_loss", *args, ts.cuda_stream)
        self._ev_end("rollout_loss", ts)
        if self.tail_stream is not None:
            self.tail_done = self._next_event()
            self.tail_done.record(ts)

    # -------------------------------------------------------------- K2 from hidden states (§8f-2, loss side)
    LOSS_FROM_HIDDEN_SIZES = (512, 768)

    def _loss_from_hidden_route(self, hidden, weight, grad_dtype, route, plan="auto"):
        """policy_loss_from_hidden's argument checks (shapes, dtypes, route, plan) -> the route it
        will take; run before any launch (pipeline_step_from_hidden: when the batch is submitted)."""
        B, T, V = self.B, self.T, self.V
        if hidden.dim() != 3 or tuple(hidden.shape[:2]) != (B, T) or weight.dim() != 2 or weight.shape[0] != V or \
                weight.shape[1] != hidden.shape[2] or hidden.dtype != torch.bfloat16 or weight.dtype != torch.bfloat16:
            raise ValueError(f"hidden {tuple(hidden.shape)}/{hidden.dtype} and weight {tuple(weight.shape)}/"
                             f"{weight.dtype} do not match the hot path ({B},{T},H) x ({V},H) bf16")
        H = hidden.shape[2]
        if grad_dtype not in (torch.bfloat16, torch.float32):
            raise ValueError("grad_dtype must be bf16 or fp32")
        if route not in ("auto", "fused", "gemm"):
            raise ValueError(f"route must be auto, fused or gemm, not {route!r}")
        if plan not in ("auto", "saved_p", "recompute"):
            raise ValueError(f"plan must be auto, saved_p or recompute, not {plan!r}")
        if route == "auto":
            route = "fused" if H in self.LOSS_FROM_HIDDEN_SIZES else "gemm"
        if route == "fused" and H not in self.LOSS_FROM_HIDDEN_SIZES:
            raise ValueError(f"policy_loss_from_hidden: fused route not built for hidden size {H} "
                             f"{self.LOSS_FROM_HIDDEN_SIZES} (route='gemm' takes any H)")
        return route

    def _loss_workspace(self, N, H, V, plan):
        """The fused loss side's workspace and the byte count to pass (the C side picks the
        saved-P plan when it holds the P tiles).  auto: saved P unless its 2·N·V-byte buffer
        cannot be allocated — then the recompute plan, sticky until release_loss_workspace()."""
        small = _lib.query("trlx_lmhead_loss_workspace_bytes", N, H, V)
        big = _lib.query("trlx_ppo_loss_from_hidden_workspace_bytes", N, H, V)
        want = small if (plan == "recompute" or (plan == "auto" and self._loss_ws_fallback)) else big
        cur = getattr(self, "lm_loss_ws", None)
        if cur is None or cur.numel() < want:
            self.lm_loss_ws = None
            try:
                self.lm_loss_ws = torch.empty(want, dtype=torch.uint8, device=self.device)
            except torch.cuda.OutOfMemoryError:
                if plan != "auto" or want == small:
                    raise
                self._loss_ws_fallback = True
                self.lm_loss_ws = cur if cur is not None and cur.numel() >= small else \
                    torch.empty(small, dtype=torch.uint8, device=self.device)
        return self.lm_loss_ws, (min(small, self.lm_loss_ws.numel()) if want == small else self.lm_loss_ws.numel())

    def policy_loss_from_hidden(self, hidden, weight, labels, values, old_values, mask=None,
                                grad_dtype=torch.bfloat16, route="auto", plan="auto"):
        """K2 with the lm_head folded in (loss side): the policy's last hidden
        states [B, T, H] and lm_head weight [V, H] (bf16, H in LOSS_FROM_HIDDEN_SIZES) replace
        the logits — the reference's policy forward + logprobs_from_logits + PPO loss +
        autograd back through the lm_head (accelerate_ppo_model.py:96-118, ppo_models.py:640 /
        :274) without [B, T, V] logits or dlogits in HBM (trlx_ppo_loss_from_hidden: three MFMA
        launches and a per-token combine; tokens with mask == 0 are compacted out).  Returns
        (loss, stats, dhidden [B, T, H], dweight [V, H], dvalues), gradients in grad_dtype;
        the same loss tail (deferred / side stream) as policy_loss.  After an unsplit GAE (the
        serial step()) the advantages are whitened by the GAE record; in split-beta mode
        (pipeline_step_from_hidden, or split_beta=True) by the split record and beta, and the
        batch's rewards / returns are written here (trlx_ppo_loss_from_hidden_split).
        route: "fused" (the kernels above; H in LOSS_FROM_HIDDEN_SIZES), "gemm" (the
        reference's own structure on the hot path's kernels: hipBLASLt bf16 logits -> the fused
        loss rows (policy_loss) -> hipBLASLt dh = dlogits·W and dW = dlogitsᵀ·h; any H, the
        [B, T, V] logits and dlogits in HBM), "auto" = fused where it is built, else gemm.
        plan (fused route): the dW pass's plan — "saved_p" (the forward's bf16 P tiles kept in
        the workspace, ~2·N·V bytes = the size of bf16 logits, 0.62 GB at C2: 3 MFMA passes),
        "recompute" (no N·V buffer: S recomputed in the dW pass, 4 passes), "auto" = saved_p
        unless that workspace cannot be allocated (then recompute, until
        release_loss_workspace())."""
        B, T, V = self.B, self.T, self.V
        route = self._loss_from_hidden_route(hidden, weight, grad_dtype, route, plan)
        H = hidden.shape[2]
        if route == "gemm":
            return self._policy_loss_from_hidden_gemm(hidden, weight, labels, values, old_values, mask, grad_dtype)
        _lib.require_cuda(hidden, weight)
        labels = self._int64(labels, (B, T), "labels")
        mask = self._int64(mask, (B, T), "mask", required=False)
        values = self._vec(values, (B, T), "values")
        old_values = self._vec(old_values, (B, T), "old_values")
        h = hidden.reshape(B * T, H)
        if h.stride(1) != 1 or h.stride(0) % 8 or h.data_ptr() % 16:
            h = h.contiguous()
        w = weight if (weight.stride(1) == 1 and weight.stride(0) % 8 == 0 and weight.data_ptr() % 16 == 0) \
            else weight.contiguous()
        N = B * T
        if getattr(self, "dhidden", None) is None or self.dhidden.shape != (B, T, H) or self.dhidden.dtype != grad_dtype:
            self.dhidden = torch.empty((B, T, H), dtype=grad_dtype, device=self.device)
            self.dweight = torch.empty((V, H), dtype=grad_dtype, device=self.device)
        # the saved-P plan's workspace (the forward's bf16 P tiles: ~V·N·2 bytes, 0.62 GB at C2)
        # or the recompute plan's; release_loss_workspace() frees it
        lm_ws, lm_bytes = self._loss_workspace(N, H, V, plan)
        s = torch.cuda.current_stream(self.device)
        self._launch_pending_tail(s)
        if self.tail_done is not None:
            self.tail_done.wait(s)
        dh, dw = self.dhidden, self.dweight
        vals = (_lib.ptr(mask), values.data_ptr(), _lib.dtype_code(values), old_values.data_ptr(),
                _lib.dtype_code(old_values))
        outs = (float(self.cfg.cliprange), float(self.cfg.cliprange_value), float(self.cfg.vf_coef),
                self.lp_new.data_ptr(), dh.data_ptr(), H, _lib.dtype_code(dh), dw.data_ptr(), _lib.dtype_code(dw), H,
                self.dvalues.data_ptr(), self.workspace.data_ptr(), lm_ws.data_ptr(), lm_bytes, s.cuda_stream)
        self._ev("loss", s)
        if self._split_mode:
            # split beta (the pipelined DP schedule, or step() with split_beta=True): the
            # whitening coefficients of A = A0 - beta*Ak come from the batch's (all-reduced)
            # split record and the current beta on the first loss of an experience (stored for a
            # later one), and this launch writes the batch's rewards and returns — as
            # trlx_ppo_loss_rows_split_gae does for the logits route
            sb = self._sbuf[self._sidx]
            derive = not self._coef_ready
            _lib.call("trlx_ppo_loss_from_hidden_split", h.data_ptr(), h.stride(0), w.data_ptr(), w.stride(0), B, T,
                      H, V, labels.data_ptr(), self.lp_old.data_ptr(), _lib.F32, sb["adv0"].data_ptr(),
                      sb["adv_kl"].data_ptr(), sb["rew_kl"].data_ptr(), sb["rew_score"].data_ptr(),
                      None if derive else sb["coef"].data_ptr(), sb["stats"].data_ptr() if derive else None,
                      0 if self.distributed else 1, self.ctl.state.data_ptr() if self.ctl is not None else None,
                      self.kl_coef, sb["coef"].data_ptr(), sb["stats"].data_ptr() + 6 * 8, *vals,
                      self.rewards.data_ptr(), self.returns.data_ptr(), _lib.dtype_code(self.returns), *outs)
            self._coef_ready = True
            tail_stats = sb["stats"].data_ptr() + 3 * 8  # the tail reads Σmask at stats[3]
        else:
            _lib.call("trlx_ppo_loss_from_hidden", h.data_ptr(), h.stride(0), w.data_ptr(), w.stride(0), B, T, H, V,
                      labels.data_ptr(), self.lp_old.data_ptr(), _lib.F32, self.adv_raw.data_ptr(),
                      self.adv_stats.data_ptr(), 0 if self.distributed else 1, *vals, self.returns.data_ptr(),
                      _lib.dtype_code(self.returns), *outs)
            tail_stats = self.adv_stats.data_ptr()
        self._ev_end("loss", s)
        self._loss_tail(s, tail_stats)
        return self.loss, self.stats, dh, dw, self.dvalues

    def step_from_hidden(self, hidden, weight, ref_hidden, ref_weight, new_hidden, labels, old_values, values,
                         scores, lengths=None, mask=None, group=None, route="auto", new_weight=None,
                         loss_route="auto", grad_dtype=torch.bfloat16):
        """step() from hidden states on both sides: experience_from_hidden
        (policy + reference lm_head + logprobs, GAE; `route`) then policy_loss_from_hidden on the
        updated policy's hidden states (new_weight: its lm_head, default `weight`; `loss_route`,
        gradients in `grad_dtype`)."""
        self.experience_from_hidden(hidden, weight, ref_hidden, ref_weight, labels, old_values, scores,
                                    lengths=lengths, mask=mask, group=group, route=route)
        return self.policy_loss_from_hidden(new_hidden, weight if new_weight is None else new_weight, labels, values,
                                            old_values, mask=mask, route=loss_route, grad_dtype=grad_dtype)

    def _policy_loss_from_hidden_gemm(self, hidden, weight, labels, values, old_values, mask, grad_dtype):
        """policy_loss_from_hidden's gemm route: hipBLASLt bf16 logits (the reference's lm_head
        output dtype on the T5 path), the fused loss rows, hipBLASLt dh / dW GEMMs."""
        B, T, V = self.B, self.T, self.V
        H = hidden.shape[2]
        N = B * T
        if getattr(self, "loss_logits", None) is None or self.loss_logits.shape != (B, T, V):
            self.loss_logits = torch.empty((B, T, V), dtype=torch.bfloat16, device=self.device)
        torch.matmul(hidden, weight.t(), out=self.loss_logits)
        loss, stats, dl, dv = self.policy_loss(self.loss_logits, labels, values, old_values, mask=mask)
        d2 = dl.reshape(N, V)
        h2 = hidden.reshape(N, H)
        if getattr(self, "dhidden", None) is None or self.dhidden.shape != (B, T, H) or self.dhidden.dtype != grad_dtype:
            self.dhidden = torch.empty((B, T, H), dtype=grad_dtype, device=self.device)
            self.dweight = torch.empty((V, H), dtype=grad_dtype, device=self.device)
        if grad_dtype == torch.bfloat16:
            torch.matmul(d2, weight, out=self.dhidden.view(N, H))
            torch.matmul(d2.t(), h2, out=self.dweight)
        else:  # bf16 operands, fp32 accumulation AND output (as the fused route's fp32 gradients)
            self.dhidden.view(N, H).copy_(torch.mm(d2, weight, out_dtype=torch.float32))
            self.dweight.copy_(torch.mm(d2.t(), h2, out_dtype=torch.float32))
        return loss, stats, self.dhidden, self.dweight, dv

    def release_loss_logits(self):
        """Free the policy_loss_from_hidden gemm route's [B, T, V] logits (re-allocated on next use)."""
        self.loss_logits = None

    def release_loss_workspace(self):
        """Free the fused policy_loss_from_hidden workspace (its saved P tiles; re-allocated on
        next use, when plan "auto" tries the saved-P plan's size again)."""
        self.lm_loss_ws = None
        self._loss_ws_fallback = False

    def release_lm_logits(self):
        """Free the gemm route's [2, chunk, T, V] logits ring (re-allocated on next use)."""
        self.lm_logits = None

    def wait_stats(self, stream=None):
        """Make `stream` (default: the current one) wait for the loss / stats of the last
        step: launches a deferred loss tail on it (defer_tail), or waits for the side-stream
        tail (overlap_tail); a no-op otherwise."""
        s = stream or torch.cuda.current_stream(self.device)
        self._launch_pending_tail(s)
        if self.tail_done is not None:
            self.tail_done.wait(s)

    def _next_event(self):
        ev = self._sync_events[self._sync_i]
        self._sync_i = (self._sync_i + 1) % len(self._sync_events)
        return ev

    # -------------------------------------------------------------- pipelined schedule (DP > 1)
    def pipeline_step(self, logits, ref_logits, new_logits, labels, old_values, values, scores,
                      lengths: Optional[torch.Tensor] = None, mask: Optional[torch.Tensor] = None, group=None):
        """Software-pipelined step (the data-parallel schedule; bit-identical to step() with
        split_beta=True at any world size).  Per call (batch k+1), two launches:

            E rows(k+1) [+ loss tail(k-1)] | [AR(k) in flight beside them]
              -> join AR(k) -> L rows(k) [+ GAE(k+1) as the launch's first workgroups] -> AR(k+1) async
                                         [tail(k) deferred into the next E launch]

        Split beta (trlx_ppo_rollout_gae_split): the reward r = score - beta*kl enters GAE
        linearly, so GAE(k+1) needs neither the KL-controller update of loss tail(k) nor
        anything of L rows(k): it runs as the first workgroups of the L rows(k) launch
        (trlx_ppo_loss_rows_split_gae), whose rows derive batch k's whitening coefficients
        from its all-reduced record and apply beta (A = A0 - beta*Ak, rewards, returns).
        Every loss sees the beta the serial schedule would give it, so losses, stats,
        gradients and controller state are bit-identical to step() with split_beta=True
        (tests/test_gpu_dist.py) and equal to the unsplit step() up to fp32 association.  The
        whitening all-reduce of batch k runs while the experience rows of batch k+1 stream;
        nothing else waits on the network.  Returns the PREVIOUS batch's (loss, stats,
        dlogits, dvalues) — valid until the next call; with defer_tail, loss / stats are final
        after wait_stats() — or None on the first call; pipeline_flush() runs the last pending
        loss.  lp_old / ref_lp and the split buffers are double-buffered.  Under a process group
        without running-std score scaling (lag) the controller's RunningMoments run one batch
        behind until pipeline_flush() merges the last batch's moments.  The serial entry points
        (step / experience / experience_from_hidden) refuse to run while a batch is pending."""
        self._check(logits)
        self._check(ref_logits)
        if logits.stride() != ref_logits.stride():
            raise ValueError("policy and reference logits must share strides")
        self._check(new_logits)

        def experience(labels, lengths, s):
            self._experience_rows(logits, ref_logits, labels, s, lengths)  # + the deferred loss tail(k-1)

        def loss(p, fold):
            return self.policy_loss(p["new_logits"], p["labels"], p["values"], p["old_values"], mask=p["mask"],
                                    _fold=fold)

        return self._pipeline(experience, loss, dict(new_logits=new_logits), labels, old_values, values, scores,
                              lengths, mask, group, fold=self._fold_gae)

    def pipeline_step_from_hidden(self, hidden, weight, ref_hidden, ref_weight, new_hidden, labels, old_values,
                                  values, scores, lengths: Optional[torch.Tensor] = None,
                                  mask: Optional[torch.Tensor] = None, group=None, new_weight=None, route="auto",
                                  loss_route="auto", grad_dtype=torch.bfloat16):
        """pipeline_step from hidden states on both sides (SURVEY §8f-2 under the data-parallel
        schedule, accelerate_ppo_model.py:88-126 under the DDP sharding of :146-148): per call
        (batch k+1)

            E lm_heads(k+1) [loss tail(k-1) first] | [AR(k) in flight beside them]
              -> GAE(k+1) (split, its own launch) -> join AR(k) -> loss from hidden(k) -> AR(k+1) async

        The loss side of batch k derives its whitening coefficients from the all-reduced split
        record and beta (trlx_ppo_loss_from_hidden_split), so the whitening all-reduce of batch
        k hides behind the experience lm_heads of batch k+1 exactly as in pipeline_step, and the
        results are bit-identical to step_from_hidden on a split_beta=True hot path.  Returns
        the PREVIOUS batch's (loss, stats, dhidden, dweight, dvalues) or None on the first call
        (valid until the next call); pipeline_flush() runs the last pending loss.  The GAE keeps
        its own launch: the loss side is ~2 ms of MFMA work, against which a 7-us launch is
        noise, and no launch of it can host the rollout waves."""
        self._check_hidden(hidden, weight, ref_hidden, ref_weight)
        w_new = weight if new_weight is None else new_weight
        # the loss side's checks now, before any launch of this batch (a failure inside the next
        # call's loss would lose this batch after its experience had run)
        loss_route = self._loss_from_hidden_route(new_hidden, w_new, grad_dtype, loss_route)
        route = self._lm_route(route, hidden, ref_hidden)

        def experience(labels, lengths, s):
            self._experience_lmhead(hidden, weight, ref_hidden, ref_weight, labels, lengths, s, route)

        def loss(p, fold):
            # batch k's loss runs in call k+1: its lm_head weight must still be the one it was
            # submitted with (an in-place optimizer.step in between would pair hidden(k) with W(k+1))
            if p["new_weight"]._version != p["weight_version"]:
                raise RuntimeError("pipeline_step_from_hidden: new_weight was modified in place between the call "
                                   "that submitted the batch and the one running its loss; step the optimizer "
                                   "after pipeline_flush(), or pass a copy")
            return self.policy_loss_from_hidden(p["new_hidden"], p["new_weight"], p["labels"], p["values"],
                                                p["old_values"], mask=p["mask"], grad_dtype=p["grad_dtype"],
                                                route=p["loss_route"])

        return self._pipeline(experience, loss, dict(new_hidden=new_hidden, new_weight=w_new, grad_dtype=grad_dtype,
                                                     loss_route=loss_route, weight_version=w_new._version),
                              labels, old_values, values, scores, lengths, mask, group, fold=False)

    def _pipeline(self, experience, loss, payload, labels, old_values, values, scores, lengths, mask, group, fold):
        """The pipelined schedule around an experience launch sequence and a loss (see
        pipeline_step); fold: the next batch's GAE rides the loss launch (the logits route)."""
        B, T = self.B, self.T
        orig = (labels, lengths, mask)
        labels, lengths, mask, old_values, scores = self._rollout_inputs(labels, lengths, mask, old_values, scores)
        values = self._vec(values, (B, T), "values")
        # converted index tensors live in shared buffers the next call refills: keep copies
        labels, lengths, mask = (t if t is None or t is o else t.clone() for t, o in zip((labels, lengths, mask), orig))
        if self._lp_bufs is None:
            self._lp_bufs = [(self.lp_old, self.ref_lp), (torch.empty_like(self.lp_old), torch.empty_like(self.ref_lp))]
        prev = self._pending
        nb = prev["buf"] ^ 1 if prev is not None else 0
        s = torch.cuda.current_stream(self.device)
        self._use_split(True, nb)
        # lag: without running-std scaling the rewards do not need this batch's global score
        # moments, so RunningMoments merges them one batch late and their all-reduce leaves
        # the front of the step (no moments launch, no side-stream hop ahead of the rows)
        distributed = self.comm is not None or (dist.is_available() and dist.is_initialized())
        lag = distributed and self.ctl is not None and self.ctl.scale_mode != _lib.SCALE_RUNNING
        if lag and self._mom_bufs is None:
            self._mom_bufs = torch.zeros((2, 4), dtype=torch.float64, device=self.device)
        self._lag = lag
        g_mom, work = self._begin_step(scores, group, s, lag=lag)  # + AR(k) on the side stream (RCCL, no lag)
        self.lp_old, self.ref_lp = self._lp_bufs[nb]
        experience(labels, lengths, s)
        self._resolve_allreduce()  # AR(k): the loss of batch k derives its whitening coefficients from it
        if lag:  # batch k's all-reduced score moments (none before the first batch)
            g_mom = self._mom_bufs[prev["buf"]] if prev is not None else None
        # GAE(k+1): its own launch on the first call (or without folding), else folded into L rows(k)
        gd = self._experience_tail(s, labels, old_values, scores, lengths, mask, group, g_mom, work,
                                   defer_allreduce=True, lag=lag, launch=prev is None or not fold)
        out = None
        if prev is not None:
            self._use_split(True, prev["buf"])
            self.lp_old, self.ref_lp = self._lp_bufs[prev["buf"]]
            out = prev["loss"](prev, gd if fold else None)
            self._use_split(True, nb)
            self.lp_old, self.ref_lp = self._lp_bufs[nb]
            if fold:
                self._gae_done(gd, s)
        self._pending = dict(payload, buf=nb, loss=loss, labels=labels, values=values, old_values=old_values,
                             mask=mask)
        return out

    def pipeline_flush(self):
        """Run the pending loss of the last pipeline_step(_from_hidden) batch; returns its outputs
        (or None)."""
        prev, self._pending = self._pending, None
        if prev is None:
            return None
        self._use_split(True, prev["buf"])
        self.lp_old, self.ref_lp = self._lp_bufs[prev["buf"]]
        self._resolve_allreduce()  # nothing left to hide it behind
        if self._lag:  # the last batch's score moments: RunningMoments' last merge
            st = self.ctl.state.data_ptr()
            _lib.call("trlx_score_moments_merge", st, st, self._mom_bufs[prev["buf"]].data_ptr(),
                      torch.cuda.current_stream(self.device).cuda_stream)
            self._lag = False
        return prev["loss"](prev, None)

    def step(self, logits, ref_logits, new_logits, labels, old_values, values, scores,
             lengths: Optional[torch.Tensor] = None, mask: Optional[torch.Tensor] = None, group=None,
             reduce_stats: bool = False):
        """One experience + loss pass over this rank's shard.  The loss stats are rank-local
        like the reference's (ppo_models.py:162-198 runs per rank; Accelerate logs rank 0);
        reduce_stats=True averages them over ranks with one extra all-reduce (logging)."""
        self.experience(logits, ref_logits, labels, old_values, scores, lengths=lengths, mask=mask, group=group)
        out = self.policy_loss(new_logits, labels, values, old_values, mask=mask)
        if reduce_stats and self.distributed:
            self.wait_stats()
            dist.all_reduce(self.stats, dist.ReduceOp.SUM, group=group)  # logging: mean over ranks
            self.stats.div_(dist.get_world_size(group))
        return out
