"""trlx_t5_amd — MI355X-native (gfx950) PPO experience-and-loss hot path of trlX-T5.

Drop-in names (reference file:line in danyang-rainbow/trlx-t5):
  logprobs_from_logits, whiten, get_global_statistics, RunningMoments, flatten_dict
      trlx/utils/modeling.py
  PPOConfig (.get_advantages_and_returns, .loss, .loss_from_logits),
  AdaptiveKLController, FixedKLController
      trlx/model/nn/ppo_models.py
  kl_penalty_rewards, prepare_scores
      trlx/orchestrator/ppo_orchestrator.py:96-112,163-167
  ILQLConfig (.loss), ILQLBatch, ilql_sample_step (one decode step of generate)
      trlx/model/nn/ilql_models.py:52-116,296-316, trlx/data/ilql_types.py
  lm_head_logprobs — fused lm_head GEMM (MFMA) + logprobs, logits never in HBM
  PPORolloutStorage, PPORLElement, PPORLBatch
      trlx/pipeline/ppo_pipeline.py, trlx/data/ppo_types.py (device-resident store)
  PPOHotPath — the fused device-resident experience+loss step (bench / DP shard)
  PPOControlState — RunningMoments / score scale+clip / KL controller state in HBM

All tensor math runs in hand-written HIP kernels (libtrlx_t5_amd.so, C ABI in
include/trlx_t5_amd.h).  There is no CPU fallback.
"""
from . import _lib
from .modeling import (RunningMoments, flatten_dict, get_global_statistics, grad_buffer_like,
                       logprobs_from_logits, moments, whiten)
from .ppo import (STATS_KEYS, AdaptiveKLController, FixedKLController, PPOConfig, kl_penalty_rewards,
                  prepare_scores, stats_dict)
from .lm_head import lm_head_logprobs
from .rollout_store import PPORLBatch, PPORLElement, PPORolloutStorage
from .ilql import ILQL_LOSS_KEYS, ILQLBatch, ILQLConfig, ILQLHotPath, ilql_sample_step
from .control import PPOControlState
from .step import PPOHotPath
from .comm import RcclComm
from .model_inputs import get_model_inputs, shift_tokens_right

__all__ = [
    "logprobs_from_logits", "whiten", "get_global_statistics", "RunningMoments", "flatten_dict", "moments",
    "grad_buffer_like", "PPOConfig", "AdaptiveKLController", "FixedKLController", "kl_penalty_rewards",
    "prepare_scores", "stats_dict", "STATS_KEYS", "PPOHotPath", "load_library",
    "ILQLConfig", "ILQLBatch", "ILQLHotPath", "ILQL_LOSS_KEYS", "ilql_sample_step", "PPORolloutStorage",
    "PPORLElement", "PPORLBatch", "lm_head_logprobs", "PPOControlState",
    "RcclComm", "shift_tokens_right", "get_model_inputs",
]


def load_library():
    """Load libtrlx_t5_amd.so now (raises if it is not built)."""
    return _lib.load()
