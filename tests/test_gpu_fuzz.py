"""Seeded random sweep over shapes, vocab sizes, dtypes and row strides (GPU vs the CPU
oracle).  Each case draws B in [1, 5], T in [1, 20], V in [1, 70000] (plus fixed edge
values), a row padding that makes the logits rows a strided view of a wider buffer (every
16-B phase), labels including 0 and V - 1, and checks through the drop-in surface:
  * logprobs_from_logits forward and backward (modeling.py:37-41 + autograd)
  * PPOConfig.loss_from_logits (the fused A1 + A6 row pass) loss, stats and both gradients
  * PPOHotPath.step (T up to 70: two GAE scan chunks; half with decoder lengths + mask)
Tolerances as tests/test_gpu_parity.py: fp32 rtol 1e-5; bf16 outputs are one rounding of the
fp32 result (logprobs rtol 8e-3, gradients rtol 1e-2) against the oracle evaluated in fp32
on the same bf16-quantised inputs.
"""
import random

import pytest
import torch

import trlx_t5_amd as P
from oracle import ppo_oracle as orc
from golden_util import loss_rows_lp

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
RT32 = dict(rtol=1e-5, atol=1e-5)


def _case(i):
    rnd = random.Random(1000 + i)
    fixed = [1, 2, 7, 8, 9, 4096, 4097, 8191, 32128, 50257, 65536]
    V = fixed[i] if i < len(fixed) else rnd.randint(1, 70000)
    dt = torch.bfloat16 if i % 2 else torch.float32
    return V, dt, rnd.randint(1, 5), rnd.randint(1, 20), rnd.choice([0, 1, 3, 5, 8])


def _inputs(i):
    V, dt, B, Tn, pad = _case(i)
    g = torch.Generator().manual_seed(i)
    full = (torch.randn(B, Tn, V + pad, generator=g) * (1 + 3 * torch.rand(1, generator=g))).to(dt)
    y = torch.randint(0, V, (B, Tn), generator=g)
    y.view(-1)[0] = 0
    y.view(-1)[-1] = V - 1
    return V, dt, B, Tn, pad, full, y, g


@pytest.mark.parametrize("i", range(24))
def test_fuzz_logprobs_fwd_bwd(i):
    V, dt, B, Tn, pad, full, y, g = _inputs(i)
    x = full[..., :V]
    gout = torch.randn(B, Tn, generator=g)
    xd = full.to(DEV).requires_grad_(True)
    lp = P.logprobs_from_logits(xd[..., :V], y.to(DEV))
    (lp.float() * gout.to(DEV)).sum().backward()
    xf = x.float().requires_grad_(True)
    ref = orc.logprobs_from_logits(xf, y)
    (ref * gout).sum().backward()
    assert lp.dtype == dt and lp.shape == (B, Tn)
    if dt == torch.float32:
        torch.testing.assert_close(lp.detach().cpu(), ref.detach(), **RT32)
        torch.testing.assert_close(xd.grad[..., :V].cpu(), xf.grad, rtol=1e-5, atol=1e-6)
    else:
        torch.testing.assert_close(lp.detach().float().cpu(), ref.detach(), rtol=8e-3, atol=1e-3)
        torch.testing.assert_close(xd.grad[..., :V].float().cpu(), xf.grad, rtol=1e-2, atol=1e-6)
    if pad:  # the padding columns of the wider buffer get no gradient
        assert xd.grad[..., V:].abs().max().item() == 0.0


@pytest.mark.parametrize("i", range(24))
def test_fuzz_loss_from_logits(i):
    V, dt, B, Tn, pad, full, y, g = _inputs(i)
    x = full[..., :V]
    olp = orc.logprobs_from_logits(x.float(), y) + 0.1 * torch.randn(B, Tn, generator=g)
    ov = torch.randn(B, Tn, generator=g)
    v = ov + 0.3 * torch.randn(B, Tn, generator=g)
    adv = torch.randn(B, Tn, generator=g)
    ret = torch.randn(B, Tn, generator=g)
    mask = (torch.rand(B, Tn, generator=g) > 0.2).long()
    mask.view(-1)[0] = 1
    cfg = P.PPOConfig()
    xd = full.to(DEV).requires_grad_(True)
    vd = v.to(DEV).requires_grad_(True)
    loss, stats, lp_new = cfg.loss_from_logits(xd[..., :V], vd, y.to(DEV), olp.to(DEV), ov.to(DEV), adv.to(DEV),
                                               ret.to(DEV), mask=mask.to(DEV))
    loss.backward()
    xf = x.float().requires_grad_(True)
    vf = v.clone().requires_grad_(True)
    lpf = orc.logprobs_from_logits(xf, y)
    rloss, rstats = orc.ppo_loss(lpf, vf, olp, ov, adv, ret, mask)
    rloss.backward()
    torch.testing.assert_close(lp_new.cpu(), loss_rows_lp(lpf.detach(), mask), **RT32)
    torch.testing.assert_close(loss.detach().cpu(), rloss.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(vd.grad.cpu(), vf.grad, rtol=1e-5, atol=1e-7)
    if dt == torch.float32:
        torch.testing.assert_close(xd.grad[..., :V].cpu(), xf.grad, rtol=1e-5, atol=1e-7)
    else:
        torch.testing.assert_close(xd.grad[..., :V].float().cpu(), xf.grad, rtol=1e-2, atol=1e-7)
    for k in P.STATS_KEYS:
        assert float(stats[k]) == pytest.approx(float(rstats[k]), rel=1e-5, abs=1e-6), k


@pytest.mark.parametrize("i", range(10))
def test_fuzz_hot_path_step(i):
    """PPOHotPath.step (experience rows, GAE tail, loss rows, loss tail) with random shapes,
    half of them with decoder lengths + mask, both logits dtypes, vs the oracle's step."""
    rnd = random.Random(77 + i)
    B, Tn, V = rnd.randint(1, 6), rnd.randint(1, 70), rnd.choice([3, 100, 1031, 4099, 32128, 50257, rnd.randint(2, 60000)])
    dt = torch.bfloat16 if i % 2 else torch.float32
    g = torch.Generator().manual_seed(500 + i)
    logits = torch.randn(B, Tn, V, generator=g).to(dt)
    ref_logits = (logits.float() + 0.1 * torch.randn(B, Tn, V, generator=g)).to(dt)
    new_logits = (logits.float() + 0.05 * torch.randn(B, Tn, V, generator=g)).to(dt)
    labels = torch.randint(0, V, (B, Tn), generator=g)
    old_values = torch.randn(B, Tn, generator=g)
    values = old_values + 0.3 * torch.randn(B, Tn, generator=g)
    scores = torch.rand(B, generator=g) * 24 - 12
    L = mask = None
    if i % 4 >= 2:
        L = torch.randint(1, Tn + 1, (B,), generator=g)
        mask = (torch.arange(Tn)[None, :] < L[:, None]).long()
        old_values = old_values.masked_fill(mask == 0, 0)
    hp = P.PPOHotPath(P.PPOConfig(), B, Tn, V, dt, DEV, kl_coef=0.05)
    d = lambda t: None if t is None else t.to(DEV)  # noqa: E731
    loss, stats, dl, dv = hp.step(d(logits), d(ref_logits), d(new_logits), d(labels), d(old_values), d(values),
                                  d(scores), lengths=d(L), mask=d(mask))
    torch.cuda.synchronize()
    ref = orc.ppo_step_reference(logits.float(), ref_logits.float(), new_logits.float(), labels, old_values, values,
                                 scores, kl_coef=0.05, lengths=L, mask=mask)
    torch.testing.assert_close(hp.lp_old.cpu(), ref["lp"], **RT32)
    torch.testing.assert_close(hp.rewards.cpu(), ref["rewards"], **RT32)
    torch.testing.assert_close(hp.returns.cpu(), ref["returns"], **RT32)
    torch.testing.assert_close(loss.cpu().reshape(()), ref["loss"], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dv.cpu(), ref["dvalues"], rtol=1e-5, atol=1e-8)
    tol = dict(rtol=8e-3, atol=1e-9) if dt == torch.bfloat16 else dict(rtol=1e-5, atol=1e-8)
    torch.testing.assert_close(dl.float().cpu(), ref["dlogits"], **tol)
    st = stats.cpu().tolist()
    for k_i, k in enumerate(P.STATS_KEYS):
        assert st[k_i] == pytest.approx(float(ref["stats"][k]), rel=1e-5, abs=1e-6), k
