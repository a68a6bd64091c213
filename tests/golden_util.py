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
