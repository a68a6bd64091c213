"""Fused lm_head projection + logprobs on MI355X.

  lm_head_logprobs(hidden, weight, labels)
      == logprobs_from_logits(hidden @ weight.T, labels)     (modeling.py:37-41 after the
         lm_head of ppo_models.py:640 / :274 / :588), experience side (no gradient)

The [.., V] logits are never written to HBM: MFMA tiles of 256 tokens x 256 vocab (ping-pong
schedule; 128 x 128 for small N) keep them in registers and reduce each tile to a partial
(max, Σexp) per token (csrc/lmhead_rows.hip).  PPOHotPath.experience_from_hidden runs the
experience step this way.
"""
import torch

from . import _lib

__all__ = ["lm_head_logprobs"]


def lm_head_logprobs(hidden: torch.Tensor, weight: torch.Tensor, labels: torch.Tensor, out_dtype=None,
                     return_lse: bool = False):
    """hidden [..., H] bf16, weight [V, H] bf16 (nn.Linear.weight), labels [...] int64 ->
    logprobs [...] of out_dtype (default: hidden.dtype, the dtype the reference's logits —
    and so its logprobs — have).  Arithmetic: bf16 products, fp32 accumulation and
    softmax statistics; the logits are not rounded to bf16 (the reference rounds them)."""
    _lib.require_cuda(hidden, weight, labels)
    if hidden.dtype != torch.bfloat16 or weight.dtype != torch.bfloat16:
        raise TypeError("lm_head_logprobs takes bf16 hidden states and weight")
    if labels.dtype != torch.int64:
        raise TypeError("labels must be int64")
    H = hidden.shape[-1]
    if weight.dim() != 2 or weight.shape[1] != H:
        raise ValueError(f"weight must be [V, {H}], got {tuple(weight.shape)}")
    if tuple(labels.shape) != tuple(hidden.shape[:-1]):
        raise ValueError("labels must have hidden.shape[:-1]")
    h = hidden.reshape(-1, H)
    if h.stride(-1) != 1 or h.stride(0) % 8 or h.data_ptr() % 16:
        h = h.contiguous()
    w = weight if (weight.stride(-1) == 1 and weight.stride(0) % 8 == 0 and weight.data_ptr() % 16 == 0) \
        else weight.contiguous()
    y = labels.reshape(-1).contiguous()
    N, V = h.shape[0], w.shape[0]
    dt = hidden.dtype if out_dtype is None else out_dtype
    lp = torch.empty(N, dtype=dt, device=h.device)
    lse = torch.empty(N, dtype=torch.float32, device=h.device) if return_lse else None
    ws = torch.empty(_lib.query("trlx_lmhead_workspace_bytes", N, V), dtype=torch.uint8, device=h.device)
    _lib.call("trlx_lmhead_logprobs", h.data_ptr(), h.stride(0), w.data_ptr(), w.stride(0), N, H, V, y.data_ptr(), 1,
              lp.data_ptr(), _lib.dtype_code(lp), _lib.ptr(lse), ws.data_ptr(), _lib.stream_of(h))
    lp = lp.view(labels.shape)
    return (lp, lse.view(labels.shape)) if return_lse else lp
