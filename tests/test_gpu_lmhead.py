"""Fused lm_head + logprobs (csrc/lmhead_rows.hip) through the C ABI,
against the oracle path it replaces: logprobs_from_logits(hidden @ weight.T, labels)
(modeling.py:37-41, oracle/ppo_oracle.py) evaluated in fp64 on the same bf16 inputs.

Tolerance: the kernel multiplies bf16 inputs exactly and accumulates in fp32 (MFMA), so the
logits differ from fp64 by summation order only (~1e-7 relative); logprobs are compared at
rtol 1e-5 + atol 1e-4 (fp32 output) and at bf16 resolution (rtol 1e-2) for bf16 output.
Label gathers are exact: out-of-range labels give NaN, never an out-of-bounds read."""
import pytest
import torch

import trlx_t5_amd as P
from oracle import ppo_oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def oracle_lp(h, w, y):
    logits = h.double() @ w.double().t()
    yy = y.clamp(0, w.shape[0] - 1)
    lp = orc.logprobs_from_logits(logits, yy)
    return torch.where((y >= 0) & (y < w.shape[0]), lp, torch.full_like(lp, float("nan")))


def case(N, H, V, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    h = (torch.randn(N, H, generator=g) * scale).to(torch.bfloat16)
    w = (torch.randn(V, H, generator=g) * scale).to(torch.bfloat16)
    y = torch.randint(0, V, (N,), generator=g)
    y[0] = 0
    y[-1] = V - 1
    return h, w, y


@pytest.mark.parametrize("N,H,V,scale", [
    (1, 64, 23, 1.0), (5, 128, 128, 1.0), (130, 64, 129, 1.0), (257, 768, 1031, 0.1), (64, 768, 50257, 0.2),
    (200, 256, 32128, 0.3), (129, 4096, 384, 0.05),
])
def test_lmhead_vs_oracle(N, H, V, scale):
    h, w, y = case(N, H, V, N + H + V, scale)
    lp, lse = P.lm_head_logprobs(h.to(DEV), w.to(DEV), y.to(DEV), out_dtype=torch.float32, return_lse=True)
    want = oracle_lp(h, w, y)
    torch.testing.assert_close(lp.cpu().double(), want, rtol=1e-5, atol=1e-4)
    want_lse = torch.logsumexp(h.double() @ w.double().t(), -1)
    torch.testing.assert_close(lse.cpu().double(), want_lse, rtol=1e-5, atol=1e-4)


def test_lmhead_bf16_out_strided_and_bad_labels():
    """bf16 output (the reference's logits dtype), a [B, T, H] view whose rows are strided
    (a causal hs[:, :-1] slice), and labels outside [0, V) -> NaN."""
    B, T, H, V = 3, 9, 128, 1000
    g = torch.Generator().manual_seed(4)
    full = (torch.randn(B, T + 1, H, generator=g) * 0.3).to(torch.bfloat16)
    w = (torch.randn(V, H, generator=g) * 0.3).to(torch.bfloat16)
    y = torch.randint(0, V, (B, T), generator=g)
    y[1, 2] = V
    y[2, 0] = -1
    hd = full.to(DEV)[:, :-1]
    assert not hd.is_contiguous()
    lp = P.lm_head_logprobs(hd, w.to(DEV), y.to(DEV))
    assert lp.dtype == torch.bfloat16 and lp.shape == (B, T)
    want = oracle_lp(full[:, :-1].reshape(-1, H), w, y.reshape(-1)).view(B, T)
    got = lp.cpu().float().double()
    assert torch.isnan(got[1, 2]) and torch.isnan(got[2, 0])
    ok = ~torch.isnan(want)
    torch.testing.assert_close(got[ok], want[ok], rtol=1e-2, atol=1e-2)


def test_lmhead_c2_shape_rows_and_determinism():
    """The C2 experience shape (6144 tokens, H 768, V 50257): a row sample against the fp64
    oracle, bitwise-identical repeats."""
    N, H, V = 6144, 768, 50257
    g = torch.Generator(device=DEV).manual_seed(7)
    h = (torch.randn(N, H, generator=g, device=DEV) * 0.15).to(torch.bfloat16)
    w = (torch.randn(V, H, generator=g, device=DEV) * 0.15).to(torch.bfloat16)
    y = torch.randint(0, V, (N,), generator=g, device=DEV)
    lp1 = P.lm_head_logprobs(h, w, y, out_dtype=torch.float32)
    lp2 = P.lm_head_logprobs(h, w, y, out_dtype=torch.float32)
    torch.cuda.synchronize()
    assert torch.equal(lp1, lp2)
    rows = torch.tensor([0, 1, 127, 128, 2047, 4096, 6000, 6143])
    want = oracle_lp(h[rows.to(DEV)].cpu(), w.cpu(), y[rows.to(DEV)].cpu())
    torch.testing.assert_close(lp1[rows.to(DEV)].cpu().double(), want, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("variant", [3, 8, 9])
def test_lmhead_every_variant_vs_oracle(variant):
    """Every tile kernel (3 = 128x128 tiles, 8 = 256x256 ping-pong, 9 = 128x256 two per CU) on ragged shapes: N and V
    not multiples of the tile, H = 64 (one K-step: the ping-pong prologue / tail counts),
    H = 4096 (64 K-steps).  Removed variants are rejected."""
    from trlx_t5_amd import _lib
    try:
        _lib.call("trlx_lmhead_set_variant", variant)
        for N, H, V, sc in [(300, 64, 1000, 0.5), (513, 768, 2051, 0.1), (2053, 192, 300, 0.3), (260, 4096, 517, 0.03),
                            (4096, 64, 4100, 0.5), (2304, 128, 7937, 0.3)]:
            h, w, y = case(N, H, V, 17 * variant + N, sc)
            lp = P.lm_head_logprobs(h.to(DEV), w.to(DEV), y.to(DEV), out_dtype=torch.float32)
            torch.testing.assert_close(lp.cpu().double(), oracle_lp(h, w, y), rtol=1e-5, atol=1e-4,
                                       msg=f"variant {variant} N={N} H={H} V={V}")
    finally:
        _lib.call("trlx_lmhead_set_variant", 0)
    with pytest.raises((ValueError, _lib.TrlxError)):
        _lib.call("trlx_lmhead_set_variant", 5)


def test_experience_from_hidden_vs_oracle():
    """PPOHotPath.experience_from_hidden (lm_head folded into the experience step) against the
    oracle experience on fp64 logits = h·Wᵀ: lp / ref_lp / rewards / returns, then the loss
    side runs on top (the GAE moments feed it as in the logits path)."""
    B, T, H, V = 6, 11, 192, 1531
    g = torch.Generator().manual_seed(21)
    h = (torch.randn(B, T, H, generator=g) * 0.3).to(torch.bfloat16)
    hr = (h.float() + 0.05 * torch.randn(B, T, H, generator=g)).to(torch.bfloat16)
    w = (torch.randn(V, H, generator=g) * 0.3).to(torch.bfloat16)
    wr = (w.float() + 0.02 * torch.randn(V, H, generator=g)).to(torch.bfloat16)
    labels = torch.randint(0, V, (B, T), generator=g)
    old_values = torch.randn(B, T, generator=g)
    values = old_values + 0.3 * torch.randn(B, T, generator=g)
    scores = torch.randn(B, generator=g) * 5
    cfg = P.PPOConfig()
    hp = P.PPOHotPath(cfg, B, T, V, torch.bfloat16, DEV, kl_coef=0.05)
    hp.experience_from_hidden(h.to(DEV), w.to(DEV), hr.to(DEV), wr.to(DEV), labels.to(DEV), old_values.to(DEV),
                              scores.to(DEV))
    torch.cuda.synchronize()
    logits = (h.double() @ w.double().t())
    ref_logits = (hr.double() @ wr.double().t())
    lp = orc.logprobs_from_logits(logits, labels)
    ref_lp = orc.logprobs_from_logits(ref_logits, labels)
    torch.testing.assert_close(hp.lp_old.cpu().double(), lp, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(hp.ref_lp.cpu().double(), ref_lp, rtol=1e-5, atol=1e-4)
    rewards = orc.kl_penalty_rewards(lp.float(), ref_lp.float(), 0.05, scores)
    torch.testing.assert_close(hp.rewards.cpu(), rewards, rtol=1e-4, atol=1e-5)
    adv, ret = orc.gae(old_values, rewards, T, 1.0, 0.95, use_whitening=False)
    torch.testing.assert_close(hp.returns.cpu(), ret, rtol=1e-4, atol=1e-4)
    new_logits = (logits + 0.01).to(torch.bfloat16).to(DEV)  # any policy logits for the loss side
    loss, stats, dl, dv = hp.policy_loss(new_logits, labels.to(DEV), values.to(DEV), old_values.to(DEV))
    torch.cuda.synchronize()
    assert torch.isfinite(loss).all() and torch.isfinite(dl.float()).all()


@pytest.mark.parametrize("H,route,chunk", [(192, "gemm", None), (2048, "auto", None), (192, "auto", None),
                                           (192, "gemm", 14), (2048, "auto", 20)])
def test_experience_from_hidden_routes(H, route, chunk):
    """The GEMM route of experience_from_hidden (hipBLASLt bf16 logits + the experience rows
    kernel over rollout chunks of LM_HEAD_CHUNK_TOKENS tokens — `chunk` forces 2-rollout
    chunks with a ragged last one; "auto" picks it from H >= LM_HEAD_GEMM_MIN_H) against the oracle on the
    bf16-rounded logits the reference's bf16 lm_head produces (ppo_models.py:640 then
    modeling.py:37-41), and against the fused route on the same inputs.  Tolerance: the GEMM
    accumulates in fp32 before rounding to bf16, so a logit may land one bf16 ulp away from
    the fp64-rounded one: atol 2e-2 (SURVEY §8c bf16 logprob bound); fused vs GEMM the same."""
    B, T, V = 5, 7, 1031
    g = torch.Generator().manual_seed(31 + H)
    sc = 1.0 / H ** 0.5
    h = (torch.randn(B, T, H, generator=g)).to(torch.bfloat16)
    hr = (h.float() + 0.05 * torch.randn(B, T, H, generator=g)).to(torch.bfloat16)
    w = (torch.randn(V, H, generator=g) * sc).to(torch.bfloat16)
    wr = (w.float() + 0.02 * sc * torch.randn(V, H, generator=g)).to(torch.bfloat16)
    labels = torch.randint(0, V, (B, T), generator=g)
    labels[0, 0], labels[-1, -1] = 0, V - 1
    old_values = torch.randn(B, T, generator=g)
    scores = torch.randn(B, generator=g) * 5
    args = [t.to(DEV) for t in (h, w, hr, wr, labels, old_values, scores)]
    hp = P.PPOHotPath(P.PPOConfig(), B, T, V, torch.bfloat16, DEV, kl_coef=0.05)
    if chunk:
        hp.LM_HEAD_CHUNK_TOKENS = chunk
    hp.experience_from_hidden(*args, route=route)
    torch.cuda.synchronize()
    expect_gemm = route == "gemm" or H >= P.PPOHotPath.LM_HEAD_GEMM_MIN_H
    assert (hp.lm_logits is not None) == expect_gemm
    if expect_gemm:  # the ring holds one chunk of rollouts, never the whole batch
        assert hp.lm_logits.shape == (2, min(B, max(1, (chunk or hp.LM_HEAD_CHUNK_TOKENS) // T)), T, V)
    lp, ref_lp, rew = hp.lp_old.cpu().double(), hp.ref_lp.cpu().double(), hp.rewards.cpu()
    logits = (h.double() @ w.double().t()).to(torch.bfloat16).double()
    ref_logits = (hr.double() @ wr.double().t()).to(torch.bfloat16).double()
    o_lp = orc.logprobs_from_logits(logits, labels)
    o_ref = orc.logprobs_from_logits(ref_logits, labels)
    torch.testing.assert_close(lp, o_lp, rtol=0, atol=2e-2)
    torch.testing.assert_close(ref_lp, o_ref, rtol=0, atol=2e-2)
    torch.testing.assert_close(rew, orc.kl_penalty_rewards(lp.float(), ref_lp.float(), 0.05, scores),
                               rtol=1e-4, atol=1e-5)
    hf = P.PPOHotPath(P.PPOConfig(), B, T, V, torch.bfloat16, DEV, kl_coef=0.05)
    hf.experience_from_hidden(*args, route="fused")
    torch.cuda.synchronize()
    assert hf.lm_logits is None
    torch.testing.assert_close(hf.lp_old.cpu().double(), lp, rtol=0, atol=2e-2)
    torch.testing.assert_close(hf.ref_lp.cpu().double(), ref_lp, rtol=0, atol=2e-2)


@pytest.mark.parametrize("H", [256, 2048])
def test_experience_from_hidden_route_rounding_at_realistic_scale(H):
    """Route-dependent rounding at a realistic logit scale (|logits| ~ 10-40, bf16 ulp
    0.0625-0.25): the fused route keeps fp32 logits and matches the oracle on the
    exact (fp64) logits to fp32 accumulation error; the gemm route rounds each logit to bf16
    like the reference's bf16 lm_head (ppo_models.py:615,640) and matches the oracle on the
    bf16-rounded logits, except where fp32 accumulation lands the other side of a rounding
    boundary (one ulp of that logit: <= 0.25 here, rare); the two routes therefore differ by
    up to one bf16 ulp of the logits, which is the documented route dependence."""
    B, T, V = 4, 9, 4099
    g = torch.Generator().manual_seed(7 + H)
    h = (torch.randn(B, T, H, generator=g) * 4).to(torch.bfloat16)
    w = (torch.randn(V, H, generator=g) * (3.0 / H ** 0.5)).to(torch.bfloat16)  # logits ~ N(0, 12^2)
    labels = torch.randint(0, V, (B, T), generator=g)
    old_values = torch.randn(B, T, generator=g)
    scores = torch.randn(B, generator=g)
    args = [t.to(DEV) for t in (h, w, h, w, labels, old_values, scores)]
    exact = h.double() @ w.double().t()
    assert float(exact.abs().max()) > 30
    out = {}
    for route in ("fused", "gemm"):
        hp = P.PPOHotPath(P.PPOConfig(), B, T, V, torch.bfloat16, DEV, kl_coef=0.05)
        hp.experience_from_hidden(*args, route=route)
        torch.cuda.synchronize()
        out[route] = hp.lp_old.cpu().double()
    o_exact = orc.logprobs_from_logits(exact, labels)
    o_bf16 = orc.logprobs_from_logits(exact.to(torch.bfloat16).double(), labels)
    torch.testing.assert_close(out["fused"], o_exact, rtol=0, atol=2e-3)
    d = (out["gemm"] - o_bf16).abs()
    assert float(d.max()) <= 0.25 and float((d > 2e-3).float().mean()) <= 0.05, (float(d.max()), d)
    ulp = torch.ldexp(torch.ones(()), torch.frexp(exact.abs().amax(-1))[1].to(torch.int32) - 8)  # per row
    assert bool(((out["gemm"] - out["fused"]).abs() <= ulp + 2e-3).all())


def test_experience_from_hidden_route_arguments():
    B, T, V, H = 2, 3, 67, 64
    h = torch.zeros(B, T, H, dtype=torch.bfloat16, device=DEV)
    w = torch.zeros(V, H, dtype=torch.bfloat16, device=DEV)
    y = torch.zeros(B, T, dtype=torch.int64, device=DEV)
    ov = torch.zeros(B, T, device=DEV)
    sc = torch.zeros(B, device=DEV)
    hp = P.PPOHotPath(P.PPOConfig(), B, T, V, torch.bfloat16, DEV, kl_coef=0.05)
    with pytest.raises(ValueError):
        hp.experience_from_hidden(h, w, h, w, y, ov, sc, route="blas")
    h32 = P.PPOHotPath(P.PPOConfig(), B, T, V, torch.float32, DEV, kl_coef=0.05)
    with pytest.raises(ValueError):
        h32.experience_from_hidden(h, w, h, w, y, ov, sc, route="gemm")


def _ragged_lmhead(h, w, y, B, T, L, variant):
    from trlx_t5_amd import _lib
    N, H = h.shape
    V = w.shape[0]
    lp = torch.full((N,), 7.0, device=DEV)
    lse = torch.full((N,), 7.0, device=DEV)
    ws = torch.empty(_lib.query("trlx_lmhead_workspace_bytes", N, V), dtype=torch.uint8, device=DEV)
    order = torch.empty(_lib.query("trlx_ragged_order_bytes", B, T), dtype=torch.uint8, device=DEV)
    _lib.call("trlx_lmhead_set_variant", variant)
    try:
        _lib.call("trlx_lmhead_logprobs_ragged", h.data_ptr(), H, w.data_ptr(), H, N, H, V, y.data_ptr(), 1,
                  L.data_ptr(), T, order.data_ptr(), lp.data_ptr(), _lib.F32, lse.data_ptr(), ws.data_ptr(),
                  torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    finally:
        _lib.call("trlx_lmhead_set_variant", 0)
    return lp.cpu(), lse.cpu()


@pytest.mark.parametrize("variant,B,T,H", [(9, 64, 48, 768), (9, 37, 70, 256), (8, 64, 48, 768), (3, 9, 20, 128)])
def test_lmhead_ragged(variant, B, T, H):
    """trlx_lmhead_logprobs_ragged: tokens past their rollout's decoder length give lp = lse = 0
    (their hidden rows hold NaN: variant 9 gathers only the valid rows and skips the padding's
    tiles; the others compute every token and zero the padding); the valid tokens carry the
    dense launch's exact bits."""
    V = 1031
    g = torch.Generator().manual_seed(B * T + variant)
    h = (torch.randn(B * T, H, generator=g) * 0.2).to(torch.bfloat16)
    w = (torch.randn(V, H, generator=g) * 0.2).to(torch.bfloat16)
    y = torch.randint(0, V, (B * T,), generator=g)
    L = torch.randint(1, T + 1, (B,), generator=g)
    L[0] = T
    pad = (torch.arange(T)[None, :] >= L[:, None]).reshape(-1)
    hd, wd, yd = h.to(DEV), w.to(DEV), y.to(DEV)
    from trlx_t5_amd import _lib
    _lib.call("trlx_lmhead_set_variant", variant)
    try:
        dense, dlse = P.lm_head_logprobs(hd, wd, yd, out_dtype=torch.float32, return_lse=True)
        torch.cuda.synchronize()
    finally:
        _lib.call("trlx_lmhead_set_variant", 0)
    hp = hd.clone()
    if variant == 9:
        hp[pad.to(DEV)] = float("nan")
    lp, lse = _ragged_lmhead(hp, wd, yd, B, T, L.to(DEV), variant)
    assert torch.equal(lp[pad], torch.zeros(int(pad.sum()))) and torch.equal(lse[pad], torch.zeros(int(pad.sum())))
    assert torch.equal(lp[~pad], dense.cpu()[~pad]) and torch.equal(lse[~pad], dlse.cpu()[~pad])
    torch.testing.assert_close(lp[~pad].double(), oracle_lp(h[~pad], w, y[~pad]), rtol=1e-5, atol=1e-4)


def test_experience_from_hidden_ragged():
    """experience_from_hidden (fused route) with decoder lengths: lp / ref_lp 0 past each
    length, equal to the dense route elsewhere; rewards / returns as the oracle's padded store."""
    B, T, H, V = 64, 48, 256, 1031
    g = torch.Generator().manual_seed(5)
    h = (torch.randn(B, T, H, generator=g) * 0.2).to(torch.bfloat16)
    hr = (h.float() + 0.02 * torch.randn(B, T, H, generator=g)).to(torch.bfloat16)
    w = (torch.randn(V, H, generator=g) * 0.2).to(torch.bfloat16)
    y = torch.randint(0, V, (B, T), generator=g)
    ov = torch.randn(B, T, generator=g)
    sc = torch.randn(B, generator=g)
    L = torch.randint(1, T + 1, (B,), generator=g)
    pad = torch.arange(T)[None, :] >= L[:, None]
    ov = ov.masked_fill(pad, 0)
    d = lambda t: t.to(DEV)  # noqa: E731
    outs = []
    for lens in (None, d(L)):
        hp = P.PPOHotPath(P.PPOConfig(), B, T, V, torch.bfloat16, DEV, kl_coef=0.05)
        hp.experience_from_hidden(d(h), d(w), d(hr), d(w), d(y), d(ov), d(sc), lengths=lens, route="fused")
        torch.cuda.synchronize()
        outs.append((hp.lp_old.cpu().clone(), hp.ref_lp.cpu().clone(), hp.rewards.cpu().clone(),
                     hp.returns.cpu().clone()))
    (lp0, rlp0, _, _), (lp1, rlp1, rew1, ret1) = outs
    assert torch.equal(lp1[pad], torch.zeros(int(pad.sum()))) and torch.equal(rlp1[pad], torch.zeros(int(pad.sum())))
    assert torch.equal(lp1[~pad], lp0[~pad]) and torch.equal(rlp1[~pad], rlp0[~pad])
    logits = h.double() @ w.double().t()
    rlogits = hr.double() @ w.double().t()
    ref = orc.ppo_step_reference(logits, rlogits, logits, y, ov, ov, sc, kl_coef=0.05, lengths=L,
                                 mask=(~pad).long())
    torch.testing.assert_close(rew1.double(), ref["rewards"], rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(ret1.double(), ref["returns"].double(), rtol=1e-4, atol=1e-4)
