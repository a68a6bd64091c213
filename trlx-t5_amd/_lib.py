"""ctypes binding of the C ABI in include/trlx_t5_amd.h (libtrlx_t5_amd.so, built in-tree
for gfx950 by `make -C trlx-t5_amd/csrc` / `__graft_entry__.build()`).

There is no fallback: if the shared library is missing or fails to load, every entry
point raises.  torch is imported first so the HIP runtime the library links against
(libamdhip64.so.7) resolves to the one torch already loaded — the library then launches
on torch's streams directly.
"""
import contextlib
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# TRLX_T5_AMD_LIB: another build of the same library (A/B tooling only, e.g. scripts/ab_rows.sh)
LIB_PATH = os.environ.get("TRLX_T5_AMD_LIB") or os.path.join(_HERE, "libtrlx_t5_amd.so")

F32, BF16, I64 = 0, 1, 2
ABI_VERSION = 2
MOMENT_SLOTS = 4
SPLIT_MOMENT_SLOTS = 8  # split-beta record {Σ A0, Σ A0², n, Σ Ak, Σ A0·Ak, Σ Ak², Σ mask, 0}
PPO_STATS = 13
PPO_PARTIAL_SLOTS = 16

_c_vp, _c_i64, _c_int, _c_f, _c_d = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float, ctypes.c_double


class IlqlArgs(ctypes.Structure):
    """Mirror of trlx_ilql_args (include/trlx_t5_amd.h)."""
    _fields_ = [
        ("dtype", _c_int), ("nq", _c_int),
        ("B", _c_i64), ("L", _c_i64), ("A", _c_i64), ("V", _c_i64),
        ("logits", _c_vp), ("logits_sb", _c_i64), ("logits_st", _c_i64),
        ("q", _c_vp * 2), ("q_sb", _c_i64 * 2), ("q_st", _c_i64 * 2),
        ("tq", _c_vp * 2), ("tq_sb", _c_i64 * 2), ("tq_st", _c_i64 * 2),
        ("input_ids", _c_vp), ("attention_mask", _c_vp), ("actions_ixs", _c_vp), ("dones", _c_vp),
        ("rewards", _c_vp), ("rewards_dtype", _c_int),
        ("vs", _c_vp), ("vs_dtype", _c_int),
        ("tau", _c_f), ("gamma", _c_f), ("cql_scale", _c_f), ("awac_scale", _c_f),
        ("dlogits", _c_vp), ("dlogits_sb", _c_i64), ("dlogits_st", _c_i64),
        ("dq", _c_vp * 2), ("dq_sb", _c_i64 * 2), ("dq_st", _c_i64 * 2),
        ("dvs", _c_vp), ("losses", _c_vp), ("workspace", _c_vp),
    ]


_ilql_p = ctypes.POINTER(IlqlArgs)

CTL_SLOTS = 16
(CTL_MEAN, CTL_VAR, CTL_STD, CTL_COUNT, CTL_REF_MEAN, CTL_REF_STD, CTL_REF_SET, CTL_KL_COEF, CTL_BATCH_MEAN,
 CTL_BATCH_STD, CTL_KL_UPDATES, CTL_LAST_KL) = range(12)
SCALE_NONE, SCALE_RUNNING, SCALE_REF = 0, 1, 2


class ScoreCtl(ctypes.Structure):
    """Mirror of trlx_score_ctl (include/trlx_t5_amd.h)."""
    _fields_ = [("state_in", _c_vp), ("state_out", _c_vp), ("global_moments", _c_vp), ("scale_mode", _c_int),
                ("cliprange_reward", _c_f)]


class KlCtl(ctypes.Structure):
    """Mirror of trlx_kl_ctl (include/trlx_t5_amd.h)."""
    _fields_ = [("state", _c_vp), ("adaptive", _c_int), ("target", _c_d), ("horizon", _c_d), ("n_steps", _c_i64)]


class GaeSplitArgs(ctypes.Structure):
    """Mirror of trlx_gae_split_args (include/trlx_t5_amd.h)."""
    _fields_ = [("B", _c_i64), ("T", _c_i64), ("lp", _c_vp), ("ref_lp", _c_vp), ("values", _c_vp), ("v_dtype", _c_int),
                ("scores", _c_vp), ("lengths", _c_vp), ("mask", _c_vp), ("ctl", ctypes.POINTER(ScoreCtl)),
                ("kl_coef", _c_f), ("gamma", _c_f), ("lam", _c_f), ("adv0", _c_vp), ("adv_kl", _c_vp),
                ("rew_kl", _c_vp), ("rew_score", _c_vp), ("stats8", _c_vp), ("mom_lag", _c_int),
                ("workspace", _c_vp)]


_score_ctl_p = ctypes.POINTER(ScoreCtl)
_kl_ctl_p = ctypes.POINTER(KlCtl)
_gae_split_p = ctypes.POINTER(GaeSplitArgs)

# name -> (restype, argtypes)   (must match include/trlx_t5_amd.h exactly)
SIGNATURES = {
    "trlx_abi_version": (_c_int, []),
    "trlx_last_error": (ctypes.c_char_p, []),
    "trlx_set_tuning": (_c_int, [ctypes.c_char_p, _c_i64]),
    "trlx_lsm_gather_fwd": (_c_int, [_c_vp, _c_vp, _c_int, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64,
                                     _c_vp, _c_i64, _c_i64, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_vp]),
    "trlx_ragged_order_bytes": (_c_i64, [_c_i64, _c_i64]),
    "trlx_lsm_gather_fwd_ragged": (_c_int, [_c_vp, _c_vp, _c_int, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64,
                                            _c_vp, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_vp]),
    "trlx_lsm_gather_bwd": (_c_int, [_c_vp, _c_int, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp,
                                     _c_i64, _c_i64, _c_vp, _c_vp, _c_int, _c_vp, _c_i64, _c_i64, _c_vp]),
    "trlx_kl_penalty_rewards": (_c_int, [_c_vp, _c_vp, _c_int, _c_i64, _c_i64, _c_f, _c_vp, _c_vp,
                                         _c_vp, _c_int, _c_vp]),
    "trlx_gae_num_blocks": (_c_i64, [_c_i64, _c_i64]),
    "trlx_gae_scan": (_c_int, [_c_vp, _c_vp, _c_int, _c_i64, _c_i64, _c_i64, _c_f, _c_f, _c_vp, _c_vp,
                               _c_f, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_int, _c_vp,
                               _c_vp, _c_vp, _c_vp]),
    "trlx_moments_num_blocks": (_c_i64, [_c_i64]),
    "trlx_moments_partial": (_c_int, [_c_vp, _c_int, _c_i64, _c_vp, _c_vp]),
    "trlx_moments_finalize": (_c_int, [_c_vp, _c_i64, _c_vp, _c_vp]),
    "trlx_whiten_apply": (_c_int, [_c_vp, _c_int, _c_i64, _c_vp, _c_int, _c_int, _c_vp, _c_int, _c_vp]),
    "trlx_ppo_policy_fused": (_c_int, [_c_vp, _c_int, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp,
                                       _c_i64, _c_i64, _c_vp, _c_int, _c_vp, _c_vp, _c_int, _c_vp, _c_vp,
                                       _c_d, _c_f, _c_vp, _c_vp, _c_i64, _c_i64, _c_vp]),
    "trlx_ppo_loss_num_blocks": (_c_i64, [_c_i64]),
    "trlx_ppo_loss_elem": (_c_int, [_c_i64, _c_vp, _c_int, _c_vp, _c_int, _c_vp, _c_int, _c_vp, _c_int,
                                    _c_vp, _c_int, _c_vp, _c_int, _c_vp, _c_int, _c_vp, _c_vp, _c_d,
                                    _c_f, _c_f, _c_f, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_vp, _c_vp,
                                    _c_vp]),
    "trlx_ppo_loss_finalize": (_c_int, [_c_vp, _c_i64, _c_i64, _c_vp, _c_d, _c_f, _c_vp, _c_vp, _c_vp]),
    "trlx_scale_by": (_c_int, [_c_vp, _c_vp, _c_int, _c_i64, _c_vp, _c_vp]),
    "trlx_ppo_workspace_bytes": (_c_i64, [_c_i64, _c_i64]),
    "trlx_ppo_rollout_gae": (_c_int, [_c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_vp, _c_f, _c_f,
                                      _c_f, _c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_vp]),
    "trlx_ppo_loss_rows": (_c_int, [_c_vp, _c_int, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp, _c_i64, _c_i64,
                                    _c_vp, _c_int, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_int, _c_vp, _c_int,
                                    _c_vp, _c_int, _c_f, _c_f, _c_f, _c_vp, _c_vp, _c_i64, _c_i64, _c_vp, _c_vp,
                                    _c_vp]),
    "trlx_ppo_rollout_loss": (_c_int, [_c_i64, _c_i64, _c_vp, _c_f, _c_vp, _c_vp, _c_vp, _c_vp]),
    "trlx_ppo_experience_fused": (_c_int, [_c_vp, _c_vp, _c_int, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64,
                                           _c_vp, _c_i64, _c_i64, _c_vp, _c_int, _c_vp, _c_vp, _c_vp, _c_f,
                                           _c_f, _c_f, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_vp,
                                           _c_vp, _c_vp]),
    "trlx_ppo_loss_fused": (_c_int, [_c_vp, _c_int, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp, _c_i64,
                                     _c_i64, _c_vp, _c_int, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_int,
                                     _c_vp, _c_int, _c_vp, _c_int, _c_f, _c_f, _c_f, _c_vp, _c_vp, _c_i64,
                                     _c_i64, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp]),
    "trlx_lmhead_workspace_bytes": (_c_i64, [_c_i64, _c_i64]),
    "trlx_lmhead_loss_workspace_bytes": (_c_i64, [_c_i64, _c_i64, _c_i64]),
    "trlx_ppo_loss_from_hidden": (_c_int, [_c_vp, _c_i64, _c_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp, _c_vp,
                                           _c_int, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_int, _c_vp, _c_int, _c_vp,
                                           _c_int, _c_f, _c_f, _c_f, _c_vp, _c_vp, _c_i64, _c_int, _c_vp,
                                           _c_int, _c_i64, _c_vp, _c_vp, _c_vp, _c_i64, _c_vp]),
    "trlx_lmhead_loss_bwd_workspace_bytes": (_c_i64, [_c_i64, _c_i64, _c_i64]),
    "trlx_ppo_loss_from_hidden_workspace_bytes": (_c_i64, [_c_i64, _c_i64, _c_i64]),
    "trlx_ppo_loss_from_hidden_plan": (_c_int, [_c_i64, _c_i64, _c_i64, _c_i64]),
    "trlx_ppo_loss_from_hidden_split": (_c_int, [_c_vp, _c_i64, _c_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp,
                                                 _c_vp, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_vp,
                                                 _c_f, _c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_int, _c_vp, _c_vp,
                                                 _c_int, _c_f, _c_f, _c_f, _c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_int,
                                                 _c_i64, _c_vp, _c_vp, _c_vp, _c_i64, _c_vp]),
    "trlx_lmhead_logprobs_fwd_saved": (_c_int, [_c_vp, _c_i64, _c_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp, _c_i64,
                                                _c_vp, _c_int, _c_vp, _c_vp, _c_vp, _c_vp]),
    "trlx_lmhead_logprobs_bwd": (_c_int, [_c_vp, _c_i64, _c_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp, _c_i64, _c_vp,
                                          _c_int, _c_vp, _c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_int, _c_i64, _c_vp,
                                          _c_vp]),
    "trlx_lmhead_savep_bytes": (_c_i64, [_c_i64, _c_i64, _c_i64]),
    "trlx_lmhead_logprobs_fwd_ex": (_c_int, [_c_vp, _c_i64, _c_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp, _c_i64,
                                             _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp]),
    "trlx_lmhead_logprobs_bwd_ex": (_c_int, [_c_vp, _c_i64, _c_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp, _c_i64,
                                             _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_int,
                                             _c_i64, _c_vp, _c_vp, _c_vp]),
    "trlx_lmhead_set_variant": (_c_int, [_c_int]),
    "trlx_lmhead_logprobs": (_c_int, [_c_vp, _c_i64, _c_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp, _c_i64, _c_vp,
                                      _c_int, _c_vp, _c_vp, _c_vp]),
    "trlx_lmhead_logprobs_ragged": (_c_int, [_c_vp, _c_i64, _c_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp, _c_i64,
                                             _c_vp, _c_i64, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_vp]),
    "trlx_ilql_sample": (_c_int, [_c_vp, _c_i64, _c_vp, _c_i64, _c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_i64, _c_vp,
                                  _c_i64, _c_i64, _c_f, _c_int, _c_f, _c_vp, _c_vp, _c_vp, _c_i64, _c_vp]),
    "trlx_rows_copy": (_c_int, [_c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_vp,
                                _c_i64, _c_vp, _c_i64, _c_vp]),
    "trlx_shift_tokens_right": (_c_int, [_c_vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp, _c_i64, _c_vp]),
    "trlx_ctl_init": (_c_int, [_c_vp, _c_d, _c_d, _c_d, _c_int, _c_vp]),
    "trlx_score_moments": (_c_int, [_c_vp, _c_int, _c_i64, _c_vp, _c_vp]),
    "trlx_score_moments_signal": (_c_int, [_c_vp, _c_int, _c_i64, _c_vp, _c_vp, _c_vp]),
    "trlx_score_ctl_update": (_c_int, [_c_vp, _c_int, _c_i64, _score_ctl_p, _c_vp, _c_int, _c_vp]),
    "trlx_kl_ctl_update": (_c_int, [_kl_ctl_p, _c_vp, _c_vp]),
    "trlx_ppo_rollout_gae_ctl": (_c_int, [_c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_vp,
                                          _score_ctl_p, _c_f, _c_f, _c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_vp,
                                          _c_vp]),
    "trlx_ppo_rollout_loss_ctl": (_c_int, [_c_i64, _c_i64, _c_vp, _c_f, _c_vp, _c_vp, _c_vp, _kl_ctl_p, _c_vp]),
    "trlx_ppo_rollout_gae_split": (_c_int, [_c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_vp,
                                            _score_ctl_p, _c_f, _c_f, _c_f, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp,
                                            _c_vp, _c_vp, _c_int, _c_int, _c_vp, _c_vp, _c_vp]),
    "trlx_score_moments_merge": (_c_int, [_c_vp, _c_vp, _c_vp, _c_vp]),
    "trlx_ppo_whiten_coef": (_c_int, [_c_vp, _c_int, _c_vp, _c_f, _c_vp, _c_vp]),
    "trlx_ppo_loss_rows_split": (_c_int, [_c_vp, _c_int, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp, _c_i64,
                                          _c_i64, _c_vp, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp,
                                          _c_vp, _c_int, _c_vp, _c_int, _c_vp, _c_vp, _c_int, _c_f, _c_f, _c_f,
                                          _c_vp, _c_vp, _c_i64, _c_i64, _c_vp, _c_vp, _c_vp]),
    "trlx_ppo_loss_rows_split_gae": (_c_int, [_c_vp, _c_int, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp, _c_i64,
                                              _c_i64, _c_vp, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_vp,
                                              _c_f, _c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_int, _c_vp, _c_vp,
                                              _c_int, _c_f, _c_f, _c_f, _c_vp, _c_vp, _c_i64, _c_i64, _c_vp, _c_vp,
                                              _gae_split_p, _c_vp, _c_vp]),
    "trlx_comm_load": (_c_int, [ctypes.c_char_p]),
    "trlx_comm_unique_id_bytes": (_c_i64, []),
    "trlx_comm_unique_id": (_c_int, [_c_vp, _c_i64]),
    "trlx_comm_init": (_c_int, [ctypes.POINTER(ctypes.c_void_p), _c_vp, _c_i64, _c_int, _c_int]),
    "trlx_comm_allreduce_sum_f64": (_c_int, [_c_vp, _c_vp, _c_i64, _c_vp]),
    "trlx_comm_destroy": (_c_int, [_c_vp]),
    "trlx_lsm_gather_fwd_loss_tail": (_c_int, [_c_vp, _c_vp, _c_int, _c_i64, _c_i64, _c_i64, _c_i64, _c_i64, _c_vp,
                                               _c_i64, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_i64, _c_i64,
                                               _c_vp, _c_f, _c_vp, _c_vp, _c_vp, _kl_ctl_p, _c_vp]),
    "trlx_ilql_workspace_bytes": (_c_i64, [_c_i64, _c_i64, _c_i64, _c_int]),
    "trlx_ilql_prep": (_c_int, [_ilql_p, _c_vp]),
    "trlx_ilql_rows": (_c_int, [_ilql_p, _c_vp]),
    "trlx_ilql_finalize": (_c_int, [_ilql_p, _c_vp]),
    "trlx_ilql_loss_fused": (_c_int, [_ilql_p, _c_vp]),
}

_lib = None


class TrlxError(RuntimeError):
    pass


def load():
    """Load (once) and return the ctypes handle; raises if the HIP library is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise TrlxError(
            f"{LIB_PATH} not found: the HIP extension is not built (run `python -c 'import "
            f"__graft_entry__ as g; g.build()'` or `make -C trlx-t5_amd/csrc`). There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.trlx_abi_version() != ABI_VERSION:
        raise TrlxError(f"ABI mismatch: library {lib.trlx_abi_version()} vs binding {ABI_VERSION}")
    _lib = lib
    return lib


def call(name, *args):
    """Invoke a status-returning entry point; raise on a non-zero status."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.trlx_last_error().decode(errors="replace")
        err = ValueError if rc in (1, 2, 3, 5) else TrlxError
        raise err(f"{name} failed (status {rc}): {msg}")
    return rc


_TUNED = {}  # the values set through this binding (the library keeps no getter); unset = 0 (auto)


def set_tuning(key: str, value: int):
    """Launch-geometry knob (see trlx_set_tuning in include/trlx_t5_amd.h).  The knobs are
    process-wide (common.h TuneKnob): a value set here reaches every host thread's launches,
    autograd's backward thread included."""
    call("trlx_set_tuning", key.encode(), int(value))
    _TUNED[key] = int(value)


@contextlib.contextmanager
def tuning(**knobs):
    """Set knobs for the duration of a block and restore the values they had before (the ones
    set through set_tuning, else 0 = auto), also when the block raises."""
    prev = {k: _TUNED.get(k, 0) for k in knobs}
    try:
        for k, v in knobs.items():
            set_tuning(k, v)
        yield
    finally:
        for k, v in prev.items():
            set_tuning(k, v)


def query(name, *args):
    return getattr(load(), name)(*args)


# ------------------------------------------------------------------ tensor helpers
def dtype_code(t):
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.bfloat16:
        return BF16
    if t.dtype == torch.int64:
        return I64
    raise TypeError(f"unsupported dtype {t.dtype} (trlx_t5_amd kernels take float32 / bfloat16 / int64)")


def ptr(t):
    return None if t is None else t.data_ptr()


def stream_of(t):
    """hipStream_t (as int) of torch's current stream on t's device."""
    return torch.cuda.current_stream(t.device).cuda_stream


def require_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("trlx_t5_amd: tensors must live on a ROCm (cuda) device; there is no CPU path")
