"""shift_tokens_right / get_model_inputs (accelerate_ppo_model.py:18-25,63-76) through
trlx_shift_tokens_right: bit-exact against the reference-generated fixtures
(tests/golden/model_inputs.npz) and the oracle, plus the reference's edge behaviour."""
import pytest
import torch

import trlx_t5_amd as P
from golden_util import T
from oracle import ppo_oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.mark.parametrize("case", ["plain", "ignore", "start_ignored", "width1"])
def test_shift_golden(golden, case):
    z = golden("model_inputs")
    ids = T(z[f"{case}/ids"]).to(DEV)
    out = P.shift_tokens_right(ids, int(z[f"{case}/pad"]), int(z[f"{case}/start"]))
    assert out.dtype == ids.dtype
    assert torch.equal(out.cpu(), T(z[f"{case}/out"]))


def test_get_model_inputs_golden(golden):
    z = golden("model_inputs")
    q, r = T(z["gmi/query"]).to(DEV), T(z["gmi/response"]).to(DEV)
    a, b, c = P.get_model_inputs(q, r)
    assert a is q and b is r
    assert torch.equal(c.cpu(), T(z["gmi/decoder_input_ids"]))


@pytest.mark.parametrize("B,Tn", [(1, 1), (3, 129), (256, 48), (1024, 128), (7, 4097)])
def test_shift_vs_oracle_sizes(B, Tn):
    g = torch.Generator().manual_seed(B * 7 + Tn)
    ids = torch.randint(-100, 32128, (B, Tn), generator=g)
    ids[ids < 0] = -100  # ~0.3 % ignore ids
    out = P.shift_tokens_right(ids.to(DEV), 0, 0)
    assert torch.equal(out.cpu(), orc.shift_tokens_right(ids))


def test_shift_strided_int32_and_empty_batch():
    g = torch.Generator().manual_seed(5)
    base = torch.randint(-100, 500, (6, 20), generator=g)
    view = base.to(DEV)[:, 3:15]  # row stride 20, not contiguous
    assert torch.equal(P.shift_tokens_right(view, 9, 4).cpu(), orc.shift_tokens_right(base[:, 3:15], 9, 4))
    i32 = base.to(torch.int32)
    out = P.shift_tokens_right(i32.to(DEV), 1, 2)
    assert out.dtype == torch.int32
    assert torch.equal(out.cpu(), orc.shift_tokens_right(i32, 1, 2))
    empty = P.shift_tokens_right(torch.zeros(0, 5, dtype=torch.long, device=DEV))
    assert empty.shape == (0, 5)


def test_shift_errors():
    with pytest.raises(IndexError):
        P.shift_tokens_right(torch.zeros(3, 0, dtype=torch.long, device=DEV))
    with pytest.raises(IndexError):
        P.shift_tokens_right(torch.zeros(5, dtype=torch.long, device=DEV))
    with pytest.raises(TypeError):
        P.shift_tokens_right(torch.zeros(2, 3, device=DEV))
    with pytest.raises(ValueError):
        P.shift_tokens_right(torch.zeros(2, 3, dtype=torch.long))  # CPU tensor: no CPU path
