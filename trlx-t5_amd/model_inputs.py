"""Seq2seq model inputs of a collated PPO batch (SURVEY §8 A9 glue):
`shift_tokens_right` (trlx/model/accelerate_ppo_model.py:18-25) and
`get_model_inputs` (:63-76) — the decoder_input_ids the policy forward of
AcceleratePPOModel.loss consumes beside labels = response_tensors.  One launch of
`trlx_shift_tokens_right` on the batch's device; no host round trip.
"""
import torch

from . import _lib

__all__ = ["shift_tokens_right", "get_model_inputs"]


def shift_tokens_right(input_ids: torch.Tensor, pad_token_id: int = 0, decoder_start_token_id: int = 0):
    """out[:, 0] = decoder_start_token_id, out[:, 1:] = input_ids[:, :-1], then -100 -> pad_token_id.
    Same dtype as input_ids (integer); [B, 0] raises IndexError as the reference does."""
    _lib.require_cuda(input_ids)
    if input_ids.dim() != 2:
        raise IndexError(f"shift_tokens_right: expected [batch, length] ids, got shape {tuple(input_ids.shape)}")
    if input_ids.dtype.is_floating_point or input_ids.dtype == torch.bool:
        raise TypeError(f"shift_tokens_right: integer token ids expected, got {input_ids.dtype}")
    B, T = input_ids.shape
    if T == 0:
        raise IndexError("shift_tokens_right: index 0 is out of bounds for an empty response (T = 0)")
    x = input_ids if input_ids.dtype == torch.int64 and input_ids.stride(1) == 1 else \
        input_ids.to(torch.int64).contiguous()
    out = torch.empty((B, T), dtype=torch.int64, device=x.device)
    if B:
        _lib.call("trlx_shift_tokens_right", x.data_ptr(), B, T, x.stride(0), int(pad_token_id),
                  int(decoder_start_token_id), out.data_ptr(), out.stride(0), _lib.stream_of(x))
    return out if input_ids.dtype == torch.int64 else out.to(input_ids.dtype)


def get_model_inputs(query_tensors: torch.Tensor, response_tensors: torch.Tensor):
    """(input_seq, new_label_ids, decoder_input_ids) = (query, response, shift_tokens_right(response))
    — pad 0 / start 0, T5's ids, as the reference hard-codes them."""
    return query_tensors, response_tensors, shift_tokens_right(response_tensors)
