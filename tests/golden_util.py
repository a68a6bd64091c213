"""Helpers to turn golden .npz entries (bf16 stored as uint16 bits) into torch tensors."""
import numpy as np
import torch


def T(arr, bf16=None):
    a = np.asarray(arr)
    if a.dtype == np.uint16:
        return torch.from_numpy(a.astype(np.int16)).view(torch.bfloat16)
    t = torch.from_numpy(a.copy())
    return t


def is_bf16(arr):
    return np.asarray(arr).dtype == np.uint16


def loss_rows_lp(new_lp, mask):
    """The loss rows' lp_out: the logprob where mask != 0 and 0 at masked tokens (their rows
    are not read: d loss / d lp is 0 there and no output depends on lp)."""
    return new_lp if mask is None else new_lp.masked_fill(mask == 0, 0)
