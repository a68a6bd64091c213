"""Whitening at a large common offset: advantages ~ N(0, 1) + 1e4 / 1e5.

The product's whitening record is single-pass fp64 — {Σx, Σx², n}, and in split-beta form
{Σ A0, Σ A0², n, Σ Ak, Σ A0·Ak, Σ Ak²} — one all-reduce instead of the reference's two-phase
mean then Σ(x − μ)² (modeling.py:9-21).  One-pass variance loses digits in proportion to
(|μ|/σ)²; these cases pin that the loss stays inside the tolerances at |μ|/σ ~ 1e4 and 1e5:
  * whiten / get_global_statistics (the drop-in surface, var_mean branch) vs the oracle;
  * the split-beta whitening coefficients {μ, rstd} the loss rows derive, vs fp64 statistics of
    the advantages the same launch used;
  * the unsplit record vs fp64 sums of its advantages; the world-2 all-reduced record vs fp64
    statistics of the concatenated shards.
Reference-side note: at these offsets an fp32 mean moves by an ulp of the offset (1e-3 at
1e4) with the summation order, and the reference's distributed branch sums in fp32
(global_sum / count), so it is itself several ulps away from the exact mean; the product's
mean is the correctly rounded fp32 value of an fp64 accumulation (ppo_math.h whiten_coeffs)."""
import os

import numpy as np
import pytest
import torch

import trlx_t5_amd as P
from oracle import ppo_oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
OFFSETS = [1e4, 1e5]


def _xs(off, seed=0, shape=(128, 48)):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g) + off


def _exact(x64, unbiased):
    mu = x64.mean()
    m2 = ((x64 - mu) ** 2).sum()
    return mu, m2 / (x64.numel() - (1 if unbiased else 0))


@pytest.mark.parametrize("off", OFFSETS)
def test_whiten_drop_in_large_offset(off):
    xs = _xs(off)
    got = P.whiten(xs.to(DEV)).cpu()
    want = orc.whiten(xs, distributed=False)  # torch.var_mean branch (unbiased)
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-5)
    got2 = P.whiten(xs.to(DEV), shift_mean=False).cpu()
    torch.testing.assert_close(got2, orc.whiten(xs, shift_mean=False, distributed=False), rtol=1e-5, atol=1e-5)
    mean, var, cnt = P.get_global_statistics(xs.to(DEV))  # no group: the local biased statistics
    mu64, var64 = _exact(xs.double(), unbiased=False)
    assert float(mean) == pytest.approx(float(mu64), rel=1e-7)
    assert float(var) == pytest.approx(float(var64), rel=1e-5)
    assert float(cnt) == xs.numel()


def _offset_step_inputs(B, T, V, off, seed):
    """gamma = lam = 1 and old values ~ -off: A_t = Σ_{k>=t} r_k - V_t ~ N(0, σ) + off."""
    g = torch.Generator().manual_seed(seed)
    logits = torch.randn(B, T, V, generator=g).to(torch.bfloat16)
    ref_logits = (logits.float() + 0.1 * torch.randn(B, T, V, generator=g)).to(torch.bfloat16)
    new_logits = (logits.float() + 0.05 * torch.randn(B, T, V, generator=g)).to(torch.bfloat16)
    labels = torch.randint(0, V, (B, T), generator=g)
    old_values = -off + 0.5 * torch.randn(B, T, generator=g)
    values = old_values + 0.3 * torch.randn(B, T, generator=g)
    scores = torch.randn(B, generator=g)
    return [t.to(DEV) for t in (logits, ref_logits, new_logits, labels, old_values, values, scores)]


@pytest.mark.parametrize("off", OFFSETS)
def test_split_beta_coefficients_large_offset(off):
    B, T, V = 64, 48, 1031
    args = _offset_step_inputs(B, T, V, off, 7)
    hp = P.PPOHotPath(P.PPOConfig(gamma=1.0, lam=1.0), B, T, V, torch.bfloat16, DEV, kl_coef=0.05, split_beta=True)
    hp.step(*args)
    hp.wait_stats()
    torch.cuda.synchronize()
    sb = hp._sbuf[hp._sidx]
    mu, rstd, beta = (float(v) for v in sb["coef"][:3].cpu())
    a0, ak = sb["adv0"].cpu().double(), sb["adv_kl"].cpu().double()
    A = a0 - beta * ak
    assert abs(float(A.mean()) - off) < 0.1 * off  # the offset is really there
    mu64, var64 = _exact(A, unbiased=True)  # no process group: torch.var_mean (unbiased)
    assert mu == np.float32(mu64) or abs(mu - float(mu64)) <= np.spacing(np.float32(mu64))
    assert rstd == pytest.approx(float(1.0 / np.sqrt(float(var64) + 1e-8)), rel=1e-5)
    # the loss saw those coefficients: its advantages are (A - mu) * rstd of the same A
    assert np.isfinite(float(hp.loss.cpu()))


@pytest.mark.parametrize("off", OFFSETS)
def test_unsplit_record_large_offset(off):
    B, T, V = 64, 48, 1031
    args = _offset_step_inputs(B, T, V, off, 8)
    hp = P.PPOHotPath(P.PPOConfig(gamma=1.0, lam=1.0), B, T, V, torch.bfloat16, DEV, kl_coef=0.05)
    hp.step(*args)
    hp.wait_stats()
    torch.cuda.synchronize()
    st = hp.adv_stats.cpu()
    a = hp.adv_raw.cpu().double()
    assert float(st[2]) == a.numel()
    assert float(st[0]) == pytest.approx(float(a.sum()), rel=1e-12)
    n = a.numel()
    m2_rec = float(st[1]) - float(st[0]) ** 2 / n
    m2 = float(((a - a.mean()) ** 2).sum())
    assert m2_rec == pytest.approx(m2, rel=1e-5)


@pytest.mark.parametrize("off", OFFSETS)
def test_dp2_record_large_offset(off):
    """World 2 (gloo on one GPU): the all-reduced record of two shards vs fp64 statistics of
    the concatenated advantages (the quantity the reference's two-phase global statistics
    estimate)."""
    import torch.multiprocessing as mp
    import dist_workers
    world, B, T, V = 2, 16, 48, 1031
    g = torch.Generator().manual_seed(int(off) % 97)
    logits = torch.randn(B, T, V, generator=g).to(torch.bfloat16)
    x = dict(logits=logits, ref_logits=(logits.float() + 0.1 * torch.randn(B, T, V, generator=g)).to(torch.bfloat16),
             new_logits=logits.clone(), labels=torch.randint(0, V, (B, T), generator=g),
             old_values=-off + 0.5 * torch.randn(B, T, generator=g), values=torch.randn(B, T, generator=g),
             scores=torch.randn(B, generator=g), lengths=None, mask=None)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + (os.getpid() + int(off) % 89) % 300
    ps = [ctx.Process(target=dist_workers.hot_path_step_worker,
                      args=(r, world, port, x, q, "rank", "step", dict(gamma=1.0, lam=1.0))) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    a = torch.cat([res[r]["adv_raw"] for r in range(world)]).double()
    n = a.numel()
    m2 = float(((a - a.mean()) ** 2).sum())
    for r in range(world):
        st = res[r]["adv_stats"]
        assert float(st[2]) == n
        assert float(st[0]) == pytest.approx(float(a.sum()), rel=1e-12)
        assert float(st[1]) - float(st[0]) ** 2 / n == pytest.approx(m2, rel=1e-5)
