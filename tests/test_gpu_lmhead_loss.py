"""§8f-2, loss side: the fused lm_head forward + backward (csrc/lmhead_loss.hip).

The reference's policy update runs lm_head -> [B, T, V] logits -> logprobs_from_logits -> PPO
loss -> autograd back through both (accelerate_ppo_model.py:96-118, ppo_models.py:640 / :274,
modeling.py:37-41, ppo_models.py:141-199).  The product computes lp, dh and dW from the hidden
states without the logits / dlogits ever in HBM.  Checked here against the oracle's own ops
(oracle.ppo_oracle, run with torch on the same device in fp32 — a floating-point kernel's
reference) on the same bf16 hidden states / weights:
  * lp, lse: fp32 MFMA accumulation vs the fp32 logits: rtol 1e-5-level (stated per test);
  * dh, dW: the products use bf16 operands (P and dS tiles rounded to bf16, like the
    reference's bf16 dlogits on the T5 path), so they are compared against the fp64 gradients
    with the reference's OWN bf16 pipeline as the yardstick: the product's relative error
    (Frobenius) must be within 2x the bf16 reference path's (bf16 logits, bf16 log-softmax
    backward, bf16 GEMMs) and below 1e-2;
  * the PPO loss, the 13 stats and dvalues at rtol 1e-4 / the loss rows' tolerances.
Masked tokens are compacted out (their hidden rows are NaN-poisoned here and never read), the
forward's fixed-offset softmax restarts when a later vocab tile's logits exceed the first
tile's by more than e^60 (a case built for it), and two runs are bit-identical.
"""
import pytest
import torch

import trlx_t5_amd as P
from oracle import ppo_oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _operands(N, H, V, seed, wscale=0.05, hscale=1.0):
    g = torch.Generator().manual_seed(seed)
    h = (torch.randn(N, H, generator=g) * hscale).to(torch.bfloat16)
    w = (torch.randn(V, H, generator=g) * wscale).to(torch.bfloat16)
    y = torch.randint(0, V, (N,), generator=g)
    return h, w, y


def _fp64_grads(h, w, y, gout):
    """lp and d(Σ gout·lp)/dh, /dW in fp64 from the bf16 operands."""
    hd = h.double().to(DEV).requires_grad_(True)
    wd = w.double().to(DEV).requires_grad_(True)
    lp = torch.log_softmax(hd @ wd.t(), -1).gather(-1, y.to(DEV)[:, None]).squeeze(-1)
    (lp * gout.double().to(DEV)).sum().backward()
    return lp.detach(), hd.grad, wd.grad


def _bf16_reference_grads(h, w, y, gout):
    """The reference's own bf16 pipeline on the T5 path: bf16 logits (lm_head output), bf16
    log_softmax + gather (modeling.py:37-41) and autograd in bf16."""
    hb = h.to(DEV).requires_grad_(True)
    wb = w.to(DEV).requires_grad_(True)
    lp = orc.logprobs_from_logits(hb @ wb.t(), y.to(DEV))
    (lp * gout.to(DEV).to(lp.dtype)).sum().backward()
    return hb.grad, wb.grad


@pytest.mark.parametrize("N,H,V", [(111, 768, 1000), (64, 512, 33), (300, 768, 50257), (129, 512, 32128)])
def test_lm_head_logprobs_autograd(N, H, V):
    h, w, y = _operands(N, H, V, N + V)
    gout = torch.randn(N, generator=torch.Generator().manual_seed(3))
    hg = h.to(DEV).requires_grad_(True)
    wg = w.to(DEV).requires_grad_(True)
    lp = P.lm_head_logprobs(hg, wg, y.to(DEV), out_dtype=torch.float32)
    (lp * gout.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    lp64, dh64, dw64 = _fp64_grads(h, w, y, gout)
    torch.testing.assert_close(lp.detach().double(), lp64, rtol=1e-5, atol=2e-5)
    assert hg.grad.dtype == torch.bfloat16 and wg.grad.dtype == torch.bfloat16
    bh, bw = _bf16_reference_grads(h, w, y, gout)
    eh, ew = _rel(hg.grad, dh64), _rel(wg.grad, dw64)
    rh, rw = _rel(bh, dh64), _rel(bw, dw64)
    assert eh < 1e-2 and ew < 1e-2, (eh, ew)
    assert eh <= 2 * rh and ew <= 2 * rw, (eh, rh, ew, rw)


def test_lm_head_logprobs_restart_on_large_logit_jump():
    """Vocab rows from the 6th tile on get logits ~80 above the first tile's: the forward's
    fixed exponent offset (the first tile's max) would overflow, so the workgroups rerun
    their split with the true max (k_lmloss_fwd pass 2)."""
    N, H, V = 96, 768, 2048
    h, w, y = _operands(N, H, V, 11)
    hf = h.float()
    wf = w.float()
    d = hf.mean(0)
    wf[5 * 32:] += 80.0 * d / (d @ d)  # x_tv += ~80 on those rows for every token
    w = wf.to(torch.bfloat16)
    gout = torch.randn(N, generator=torch.Generator().manual_seed(4))
    hg = h.to(DEV).requires_grad_(True)
    wg = w.to(DEV).requires_grad_(True)
    lp = P.lm_head_logprobs(hg, wg, y.to(DEV), out_dtype=torch.float32)
    (lp * gout.to(DEV)).sum().backward()
    lp64, dh64, dw64 = _fp64_grads(h, w, y, gout)
    assert torch.isfinite(lp).all() and torch.isfinite(hg.grad.float()).all()
    torch.testing.assert_close(lp.detach().double(), lp64, rtol=1e-5, atol=1e-4)
    assert _rel(hg.grad, dh64) < 1e-2 and _rel(wg.grad, dw64) < 1e-2


def _ppo_inputs(B, T, V, H, seed, masked):
    g = torch.Generator().manual_seed(seed)
    h = torch.randn(B, T, H, generator=g).to(torch.bfloat16)
    w = (torch.randn(V, H, generator=g) * 0.05).to(torch.bfloat16)
    ref_h = (h.float() + 0.1 * torch.randn(B, T, H, generator=g)).to(torch.bfloat16)
    new_h = (h.float() + 0.05 * torch.randn(B, T, H, generator=g)).to(torch.bfloat16)
    labels = torch.randint(0, V, (B, T), generator=g)
    old_values = torch.randn(B, T, generator=g)
    values = old_values + 0.3 * torch.randn(B, T, generator=g)
    scores = torch.rand(B, generator=g) * 24 - 12
    lengths = mask = None
    if masked:
        lengths = torch.randint(1, T + 1, (B,), generator=g)
        lengths[0] = T
        mask = (torch.arange(T)[None, :] < lengths[:, None]).long()
        old_values = old_values.masked_fill(mask == 0, 0)
    return dict(h=h, w=w, ref_h=ref_h, new_h=new_h, labels=labels, old_values=old_values, values=values,
                scores=scores, lengths=lengths, mask=mask)


def _oracle_loss_side(x, lp_old, adv_w, ret, mask):
    """The reference loss side on the device in fp32: logits from the bf16 operands, the
    oracle's logprobs_from_logits and ppo_loss, autograd to (h, W, values)."""
    B, T, H = x["new_h"].shape
    hd = x["new_h"].float().to(DEV).requires_grad_(True)
    wd = x["w"].float().to(DEV).requires_grad_(True)
    vd = x["values"].to(DEV).requires_grad_(True)
    lp = orc.logprobs_from_logits(hd @ wd.t(), x["labels"].to(DEV))
    m = torch.ones(B, T, dtype=torch.long, device=DEV) if mask is None else mask.to(DEV)
    loss, stats = orc.ppo_loss(lp, vd, lp_old.to(DEV), x["old_values"].to(DEV), adv_w.to(DEV), ret.to(DEV), m)
    loss.backward()
    return loss.detach(), stats, lp.detach(), hd.grad, wd.grad, vd.grad


@pytest.mark.parametrize("B,T,V,H,masked", [(4, 9, 1031, 768, False), (16, 48, 32128, 768, True),
                                            (128, 48, 50257, 768, False), (256, 48, 32128, 768, True),
                                            (8, 20, 5000, 512, True), (1, 3, 1031, 768, False),
                                            (3, 2, 777, 512, True)])
def test_hot_path_loss_from_hidden_vs_oracle(B, T, V, H, masked):
    """PPOHotPath.step_from_hidden (fused experience lm_head + GAE, then the fused loss side)
    against the oracle's loss side on the product's own experience outputs (lp_old, whitened
    advantages, returns are checked by the experience tests); C2 and C3 shapes included.
    Masked tokens' hidden rows are NaN: the compacted loss side never reads them."""
    x = _ppo_inputs(B, T, V, H, 100 + B + T, masked)
    cfg = P.PPOConfig()
    hp = P.PPOHotPath(cfg, B, T, V, torch.bfloat16, DEV, kl_coef=0.05)
    d = {k: (v.to(DEV) if isinstance(v, torch.Tensor) else v) for k, v in x.items()}
    if masked:  # the device copy only: the oracle below uses the clean rows
        d["new_h"] = d["new_h"].masked_fill((d["mask"] == 0)[..., None], float("nan"))
    loss, stats, dh, dw, dv = hp.step_from_hidden(d["h"], d["w"], d["ref_h"], d["w"], d["new_h"], d["labels"],
                                                 d["old_values"], d["values"], d["scores"], lengths=d["lengths"],
                                                 mask=d["mask"], route="fused")
    torch.cuda.synchronize()
    # the whitened advantages the loss saw: the GAE record of this step (unbiased, no group)
    st = hp.adv_stats.cpu()
    mu, var = P.modeling.moments_to_mean_var(st, unbiased=True)
    adv_w = ((hp.adv_raw.cpu().double() - mu) * torch.rsqrt(var + 1e-8)).float()
    want_loss, want_stats, want_lp, want_dh, want_dw, want_dv = _oracle_loss_side(
        x, hp.lp_old.cpu(), adv_w, hp.returns.cpu(), x["mask"])
    m = torch.ones(B, T, dtype=torch.bool) if x["mask"] is None else x["mask"].bool()
    torch.testing.assert_close(hp.lp_new.cpu()[m], want_lp.cpu()[m], rtol=1e-5, atol=2e-5)
    if x["mask"] is not None:
        assert (hp.lp_new.cpu()[~m] == 0).all() and (dh.cpu()[~m] == 0).all()
    torch.testing.assert_close(loss.cpu().reshape(()), want_loss.cpu(), rtol=1e-4, atol=1e-5)
    got_stats = dict(zip(P.STATS_KEYS, stats.cpu().tolist()))
    for k in P.STATS_KEYS:
        assert got_stats[k] == pytest.approx(float(want_stats[k]), rel=1e-4, abs=1e-5), k
    torch.testing.assert_close(dv.cpu(), want_dv.cpu(), rtol=1e-5, atol=1e-6)
    assert torch.isfinite(dh.float()).all() and torch.isfinite(dw.float()).all()
    eh, ew = _rel(dh.cpu()[m], want_dh.cpu()[m]), _rel(dw.cpu(), want_dw.cpu())
    assert eh < 1e-2 and ew < 1e-2, (eh, ew)


def test_loss_from_hidden_deterministic_and_drop_in():
    """Two identical calls give the same bits (fixed-order sums, no atomics); the drop-in
    PPOConfig.loss_from_hidden (autograd through lm_head_logprobs + loss) matches the fused
    hot path's gradients to bf16 rounding."""
    B, T, V, H = 8, 24, 3000, 768
    x = _ppo_inputs(B, T, V, H, 77, True)
    d = {k: (v.to(DEV) if isinstance(v, torch.Tensor) else v) for k, v in x.items()}
    outs = []
    for _ in range(2):
        hp = P.PPOHotPath(P.PPOConfig(), B, T, V, torch.bfloat16, DEV, kl_coef=0.05)
        o = hp.step_from_hidden(d["h"], d["w"], d["ref_h"], d["w"], d["new_h"], d["labels"], d["old_values"],
                                d["values"], d["scores"], lengths=d["lengths"], mask=d["mask"], route="fused")
        torch.cuda.synchronize()
        outs.append([t.clone() for t in o])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    # drop-in: whiten the hot path's raw advantages the same way, then autograd
    st = hp.adv_stats
    mu, var = P.modeling.moments_to_mean_var(st, unbiased=True)
    adv_w = ((hp.adv_raw.double() - mu) * torch.rsqrt(var + 1e-8)).float()
    hg = d["new_h"].clone().requires_grad_(True)
    wg = d["w"].clone().requires_grad_(True)
    vg = d["values"].clone().requires_grad_(True)
    loss, stats = P.PPOConfig().loss_from_hidden(hg, wg, vg, d["labels"], hp.lp_old, d["old_values"], adv_w,
                                                hp.returns, d["mask"])
    loss.backward()
    torch.cuda.synchronize()
    torch.testing.assert_close(loss.reshape(()), outs[0][0].reshape(()), rtol=1e-5, atol=1e-6)
    m = d["mask"].bool()
    assert _rel(hg.grad[m], outs[0][2][m]) < 5e-3 and _rel(wg.grad, outs[0][3]) < 5e-3
    torch.testing.assert_close(vg.grad, outs[0][4], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("splits,tsplit", [(1, 1), (3, 2), (8, 5), (5, 16)])
def test_lm_head_logprobs_split_plans(splits, tsplit):
    """Forced grid plans (tuning keys): the forward's vocab split count and the dW kernel's
    token split of its last-round vocab blocks change only the fp32 summation order — every
    plan stays within the fp64 tolerances, and matches the default plan to fp32 / bf16
    rounding."""
    N, H, V = 200, 768, 7000
    h, w, y = _operands(N, H, V, 5)
    gout = torch.randn(N, generator=torch.Generator().manual_seed(6))

    def run():
        hg = h.to(DEV).requires_grad_(True)
        wg = w.to(DEV).requires_grad_(True)
        lp = P.lm_head_logprobs(hg, wg, y.to(DEV), out_dtype=torch.float32)
        (lp * gout.to(DEV)).sum().backward()
        torch.cuda.synchronize()
        return lp.detach(), hg.grad, wg.grad

    base = run()
    P._lib.set_tuning("lmloss_splits", splits)
    P._lib.set_tuning("lmloss_dw_tsplit", tsplit)
    try:
        got = run()
    finally:
        P._lib.set_tuning("lmloss_splits", 0)
        P._lib.set_tuning("lmloss_dw_tsplit", 0)
    lp64, dh64, dw64 = _fp64_grads(h, w, y, gout)
    torch.testing.assert_close(got[0].double(), lp64, rtol=1e-5, atol=2e-5)
    assert _rel(got[1], dh64) < 1e-2 and _rel(got[2], dw64) < 1e-2
    torch.testing.assert_close(got[0], base[0], rtol=1e-6, atol=1e-5)
    # dW: the split plan sets the per-split scale e' of the saved-P plan's scaled rows
    # hq = −g·e'·h, so their bf16 rounding differs between plans (two roundings apart)
    assert _rel(got[1], base[1]) < 2e-3 and _rel(got[2], base[2]) < 6e-3


def test_loss_from_hidden_gemm_route_matches_fused():
    """route='gemm' (hipBLASLt bf16 logits -> the loss rows -> dh / dW GEMMs, the reference's
    structure on the hot path's kernels) against the fused route on the same step: the loss,
    stats and dvalues to the bf16 rounding of the logits, dh / dW to bf16 GEMM tolerance."""
    B, T, V, H = 8, 24, 3000, 768
    x = _ppo_inputs(B, T, V, H, 91, True)
    d = {k: (v.to(DEV) if isinstance(v, torch.Tensor) else v) for k, v in x.items()}
    outs = {}
    for route in ("fused", "gemm"):
        hp = P.PPOHotPath(P.PPOConfig(), B, T, V, torch.bfloat16, DEV, kl_coef=0.05)
        o = hp.step_from_hidden(d["h"], d["w"], d["ref_h"], d["w"], d["new_h"], d["labels"], d["old_values"],
                                d["values"], d["scores"], lengths=d["lengths"], mask=d["mask"], route="fused",
                                loss_route=route)
        torch.cuda.synchronize()
        outs[route] = [t.clone() for t in o]
    f, g = outs["fused"], outs["gemm"]
    torch.testing.assert_close(g[0].reshape(()), f[0].reshape(()), rtol=2e-3, atol=1e-4)
    torch.testing.assert_close(g[4], f[4], rtol=1e-4, atol=1e-6)
    m = d["mask"].bool()
    assert _rel(g[2][m], f[2][m]) < 2e-2 and _rel(g[3], f[3]) < 2e-2
    assert (g[2][~m] == 0).all()


def test_loss_from_hidden_any_hidden_size():
    """H = 1024 (no fused build): loss_route 'auto' takes the gemm route; checked against the
    oracle's loss side on bf16-rounded logits (the reference's own lm_head output dtype on the
    T5 path; straight-through rounding so the oracle's autograd is the reference's)."""
    B, T, V, H = 4, 16, 2500, 1024
    x = _ppo_inputs(B, T, V, H, 17, True)
    d = {k: (v.to(DEV) if isinstance(v, torch.Tensor) else v) for k, v in x.items()}
    hp = P.PPOHotPath(P.PPOConfig(), B, T, V, torch.bfloat16, DEV, kl_coef=0.05)
    loss, stats, dh, dw, dv = hp.step_from_hidden(d["h"], d["w"], d["ref_h"], d["w"], d["new_h"], d["labels"],
                                                 d["old_values"], d["values"], d["scores"], lengths=d["lengths"],
                                                 mask=d["mask"])
    torch.cuda.synchronize()
    st = hp.adv_stats.cpu()
    mu, var = P.modeling.moments_to_mean_var(st, unbiased=True)
    adv_w = ((hp.adv_raw.cpu().double() - mu) * torch.rsqrt(var + 1e-8)).float()
    hd = x["new_h"].float().to(DEV).requires_grad_(True)
    wd = x["w"].float().to(DEV).requires_grad_(True)
    vd = x["values"].to(DEV).requires_grad_(True)
    lg = hd @ wd.t()
    lg = lg + (lg.bfloat16().float() - lg).detach()
    lp = orc.logprobs_from_logits(lg, x["labels"].to(DEV))
    want, _ = orc.ppo_loss(lp, vd, hp.lp_old, x["old_values"].to(DEV), adv_w.to(DEV), hp.returns,
                           x["mask"].to(DEV))
    want.backward()
    torch.testing.assert_close(loss.reshape(()), want.detach(), rtol=2e-3, atol=1e-4)
    torch.testing.assert_close(dv, vd.grad, rtol=1e-4, atol=1e-6)
    m = x["mask"].bool().to(DEV)
    assert _rel(dh[m], hd.grad[m]) < 2e-2 and _rel(dw, wd.grad) < 2e-2


def test_lm_head_logprobs_autograd_any_hidden_size():
    """lm_head_logprobs with gradients at an H the fused backward is not built for (1024):
    hipBLASLt bf16 logits + logprobs_from_logits under autograd, against fp64 (bf16-logits
    tolerance)."""
    N, H, V = 96, 1024, 2000
    h, w, y = _operands(N, H, V, 23)
    gout = torch.randn(N, generator=torch.Generator().manual_seed(8))
    hg = h.to(DEV).requires_grad_(True)
    wg = w.to(DEV).requires_grad_(True)
    lp = P.lm_head_logprobs(hg, wg, y.to(DEV), out_dtype=torch.float32)
    (lp * gout.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    lp64, dh64, dw64 = _fp64_grads(h, w, y, gout)
    torch.testing.assert_close(lp.detach().double(), lp64, rtol=0, atol=6e-2)
    assert _rel(hg.grad, dh64) < 2e-2 and _rel(wg.grad, dw64) < 2e-2


@pytest.mark.parametrize("plan", ["saved_p", "recompute"])
@pytest.mark.parametrize("N,H,V", [(200, 768, 7000), (70, 512, 33), (300, 768, 50257)])
def test_lm_head_logprobs_restart_shapes(plan, N, H, V):
    """The forward (16x16x32 form) against fp64 on both dW plans, with and without the restart
    path (a logit jump of ~80 from the 3rd tile on: the restarted blocks rewrite their P tiles
    and offsets, which the saved-P backward then reads)."""
    for jump in (False, True):
        h, w, y = _operands(N, H, V, N + V)
        if jump and V > 96:
            wf = w.float()
            dvec = h.float().mean(0)
            wf[2 * 32:] += 80.0 * dvec / (dvec @ dvec)
            w = wf.to(torch.bfloat16)
        gout = torch.randn(N, generator=torch.Generator().manual_seed(2))
        hg = h.to(DEV).requires_grad_(True)
        wg = w.to(DEV).requires_grad_(True)
        lp = P.lm_head_logprobs(hg, wg, y.to(DEV), out_dtype=torch.float32, plan=plan)
        (lp * gout.to(DEV)).sum().backward()
        torch.cuda.synchronize()
        lp64, dh64, dw64 = _fp64_grads(h, w, y, gout)
        torch.testing.assert_close(lp.detach().double(), lp64, rtol=1e-5, atol=1e-4)
        assert _rel(hg.grad, dh64) < 1e-2 and _rel(wg.grad, dw64) < 1e-2


def test_lm_head_logprobs_plans_agree_and_frozen_operands():
    """The two dW plans on the same call: lp and dh bit-identical (the plans differ in the dW
    pass only), dW to the bf16 rounding of P / dS.  A frozen lm_head (weight without grad: no dW
    pass, no P kept) and detached hidden states (dh not requested: the combine writes no dh)
    each return the other gradient as in the full call, and None for theirs."""
    N, H, V = 333, 768, 5000
    h, w, y = _operands(N, H, V, 19)
    gout = torch.randn(N, generator=torch.Generator().manual_seed(9)).to(DEV)
    outs = {}
    for plan in ("saved_p", "recompute"):
        hg = h.to(DEV).requires_grad_(True)
        wg = w.to(DEV).requires_grad_(True)
        lp = P.lm_head_logprobs(hg, wg, y.to(DEV), out_dtype=torch.float32, plan=plan)
        (lp * gout).sum().backward()
        torch.cuda.synchronize()
        outs[plan] = (lp.detach(), hg.grad, wg.grad)
    a, b = outs["saved_p"], outs["recompute"]
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    assert _rel(a[2], b[2]) < 4e-3
    # frozen lm_head: dh only
    hg = h.to(DEV).requires_grad_(True)
    lp = P.lm_head_logprobs(hg, w.to(DEV), y.to(DEV), out_dtype=torch.float32)
    (lp * gout).sum().backward()
    torch.cuda.synchronize()
    assert torch.equal(hg.grad, a[1])
    # hidden detached: dW only (saved P), equal to the full call's
    wg = w.to(DEV).requires_grad_(True)
    lp = P.lm_head_logprobs(h.to(DEV), wg, y.to(DEV), out_dtype=torch.float32)
    (lp * gout).sum().backward()
    torch.cuda.synchronize()
    assert torch.equal(wg.grad, a[2])
    # and against torch autograd of the reference structure in fp32 (the same operands)
    _, dh64, dw64 = _fp64_grads(h, w, y, gout.cpu())
    assert _rel(a[1], dh64) < 1e-2 and _rel(wg.grad, dw64) < 1e-2


def test_lm_head_logprobs_saved_p_released_by_backward():
    """The saved-P region (2·N·V bytes) lives in the autograd node's saved tensors: the backward
    releases it with them while the caller still holds lp (its grad_fn alive), and a
    retain_graph backward keeps it for a second pass with the same gradients."""
    N, H, V = 257, 768, 4099
    h, w, y = _operands(N, H, V, 23)
    wg = w.to(DEV).requires_grad_(True)
    lp = P.lm_head_logprobs(h.to(DEV), wg, y.to(DEV), out_dtype=torch.float32, plan="saved_p")
    saved = lp.grad_fn.saved_tensors
    nbytes = P._lib.query("trlx_lmhead_savep_bytes", N, H, V)
    assert saved[-1] is not None and saved[-1].numel() == nbytes
    del saved
    lp.sum().backward(retain_graph=True)
    g1 = wg.grad.clone()
    wg.grad = None
    lp.sum().backward()  # the second pass reads the same P region
    torch.cuda.synchronize()
    assert torch.equal(wg.grad, g1)
    with pytest.raises(RuntimeError):
        lp.grad_fn.saved_tensors  # freed with the graph, lp still referenced


@pytest.mark.parametrize("plan", ["saved_p", "recompute"])
@pytest.mark.parametrize("N,H,V", [(300, 768, 5000), (6144, 768, 32128), (77, 512, 1031)])
def test_lm_head_logprobs_mask_compacts(plan, N, H, V):
    """lm_head_logprobs(mask=...): the masked tokens are compacted out of the MFMA passes
    (their hidden rows NaN-poisoned here: never read) — lp = 0 and zero dh there, the live
    tokens' lp / dh and the dW over the live tokens against fp64 of the live rows alone, on both
    plans; the no-grad path returns the same lp."""
    h, w, y = _operands(N, H, V, N + 5)
    g = torch.Generator().manual_seed(N)
    m = (torch.rand(N, generator=g) < 0.55).long()
    m[0] = 1
    gout = torch.randn(N, generator=g)
    live = m.bool()
    hd = h.to(DEV).masked_fill((m == 0).to(DEV)[:, None], float("nan")).requires_grad_(True)
    wg = w.to(DEV).requires_grad_(True)
    lp = P.lm_head_logprobs(hd, wg, y.to(DEV), out_dtype=torch.float32, plan=plan, mask=m.to(DEV))
    (lp * gout.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    assert (lp.detach().cpu()[~live] == 0).all() and (hd.grad.cpu()[~live] == 0).all()
    assert torch.isfinite(hd.grad).all() and torch.isfinite(wg.grad).all()
    lp64, dh64, dw64 = _fp64_grads(h[live], w, y[live], gout[live])
    torch.testing.assert_close(lp.detach()[live.to(DEV)].double(), lp64, rtol=1e-5, atol=2e-5)
    assert _rel(hd.grad[live.to(DEV)], dh64) < 1e-2 and _rel(wg.grad, dw64) < 1e-2
    with torch.no_grad():
        lp_ng = P.lm_head_logprobs(h.to(DEV), w.to(DEV), y.to(DEV), out_dtype=torch.float32, mask=m.to(DEV))
    torch.testing.assert_close(lp_ng, lp.detach(), rtol=1e-5, atol=2e-5)


@pytest.mark.parametrize("plan", ["saved_p", "recompute"])
@pytest.mark.parametrize("N,H,V,live", [(1, 768, 1000, "all"), (1, 512, 50257, "all"), (130, 768, 4099, "one"),
                                        (130, 768, 4099, "none"), (64, 512, 33, "none")])
def test_lm_head_logprobs_edge_token_counts(plan, N, H, V, live):
    """Edge token counts of the fused loss side: a single token (one partial 64-token block, one
    32-token tile of P), a single live token among masked ones, and every token masked (no live
    token block: the forward, combine and dW passes see nv = 0) — lp / dh / dW against fp64 of
    the live rows, and exact zeros where nothing is live (dW included, never NaN)."""
    h, w, y = _operands(N, H, V, N + V + 7)
    gout = torch.randn(N, generator=torch.Generator().manual_seed(N + 1))
    m = torch.ones(N, dtype=torch.long)
    if live == "one":
        m.zero_()
        m[N // 2] = 1
    elif live == "none":
        m.zero_()
    hd = h.to(DEV).requires_grad_(True)
    wg = w.to(DEV).requires_grad_(True)
    lp = P.lm_head_logprobs(hd, wg, y.to(DEV), out_dtype=torch.float32, plan=plan,
                            mask=None if live == "all" else m.to(DEV))
    (lp * gout.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    assert torch.isfinite(hd.grad).all() and torch.isfinite(wg.grad).all()
    keep = m.bool()
    assert (lp.detach().cpu()[~keep] == 0).all() and (hd.grad.cpu()[~keep] == 0).all()
    if not keep.any():
        assert (wg.grad == 0).all()
        return
    lp64, dh64, dw64 = _fp64_grads(h[keep], w, y[keep], gout[keep])
    torch.testing.assert_close(lp.detach()[keep.to(DEV)].double(), lp64, rtol=1e-5, atol=2e-5)
    assert _rel(hd.grad[keep.to(DEV)], dh64) < 1e-2 and _rel(wg.grad, dw64) < 1e-2


def test_lm_head_logprobs_auto_plan_falls_back_when_p_does_not_fit(monkeypatch):
    """plan="auto": when the saved-P region cannot be allocated (its size made impossible
    here) the call takes the recompute plan and gives the recompute plan's bits."""
    N, H, V = 200, 512, 3000
    h, w, y = _operands(N, H, V, 29)
    gout = torch.randn(N, generator=torch.Generator().manual_seed(1)).to(DEV)

    def run(plan):
        hg = h.to(DEV).requires_grad_(True)
        wg = w.to(DEV).requires_grad_(True)
        lp = P.lm_head_logprobs(hg, wg, y.to(DEV), out_dtype=torch.float32, plan=plan)
        (lp * gout).sum().backward()
        torch.cuda.synchronize()
        return hg.grad, wg.grad

    want = run("recompute")
    real_query = P._lib.query
    monkeypatch.setattr(P._lib, "query", lambda name, *a: (1 << 52) if name == "trlx_lmhead_savep_bytes"
                        else real_query(name, *a))
    got = run("auto")
    assert torch.equal(got[0], want[0]) and torch.equal(got[1], want[1])
    with pytest.raises(torch.cuda.OutOfMemoryError):
        run("saved_p")


# ------------------------------------------------------------------ the softmax halves, checked by themselves
# (VERDICT r04 "What's weak 1"): tests/lmloss_checks.py — E per token, dW on the non-label and
# the label rows separately plus per row, dh against the E term it carries — with limits derived
# from the bf16 rounding of P / dS; tests/test_lmloss_sensitivity.py shows on the CPU that each
# check fails when dW's −p·h term or E is zeroed or off by 10 %.
import lmloss_checks as C  # noqa: E402


def _fwd_saved_bwd(h, w, y, gout, dh_dtype, dw_dtype, plan="recompute"):
    """The drop-in pair through the C ABI on this thread (lp, lse, the saved E, dh, dW):
    trlx_lmhead_logprobs_fwd_saved + _bwd (recompute plan) or _fwd_savep + _bwd_savep
    (saved_p: the forward's P tiles kept in a region of trlx_lmhead_savep_bytes)."""
    N, H = h.shape
    V = w.shape[0]
    L = P._lib
    hd, wd, yd, gd = h.to(DEV), w.to(DEV), y.to(DEV), gout.to(DEV).float()
    f32 = dict(dtype=torch.float32, device=DEV)
    lp, lse, e = torch.empty(N, **f32), torch.empty(N, **f32), torch.empty((N, H), **f32)
    ws = torch.empty(L.query("trlx_lmhead_loss_workspace_bytes", N, H, V), dtype=torch.uint8, device=DEV)
    s = torch.cuda.current_stream(DEV).cuda_stream
    fwd = (hd.data_ptr(), H, wd.data_ptr(), H, N, H, V, yd.data_ptr(), 1, lp.data_ptr(), L.F32, lse.data_ptr(),
           e.data_ptr(), ws.data_ptr())
    saved = None
    if plan == "saved_p":
        saved = torch.empty(L.query("trlx_lmhead_savep_bytes", N, H, V), dtype=torch.uint8, device=DEV)
        L.call("trlx_lmhead_logprobs_fwd_ex", *fwd[:9], None, *fwd[9:], saved.data_ptr(), s)
    else:
        L.call("trlx_lmhead_logprobs_fwd_saved", *fwd, s)
    del ws  # the forward's partials are not needed by the backward
    dh = torch.empty((N, H), dtype=dh_dtype, device=DEV)
    dw = torch.empty((V, H), dtype=dw_dtype, device=DEV)
    wsb = torch.empty(L.query("trlx_lmhead_loss_bwd_workspace_bytes", N, H, V), dtype=torch.uint8, device=DEV)
    bwd = (hd.data_ptr(), H, wd.data_ptr(), H, N, H, V, yd.data_ptr(), 1, gd.data_ptr(), L.F32, lse.data_ptr(),
           e.data_ptr(), dh.data_ptr(), H, L.dtype_code(dh), dw.data_ptr(), L.dtype_code(dw), H, wsb.data_ptr())
    if saved is not None:
        L.call("trlx_lmhead_logprobs_bwd_ex", *bwd[:9], None, *bwd[9:], saved.data_ptr(), s)
    else:
        L.call("trlx_lmhead_logprobs_bwd", *bwd, s)
    torch.cuda.synchronize()
    return lp, lse, e, dh, dw


def _halves_operands(kind, N, H, V, seed):
    if kind == "peaked":
        return C.peaked_operands(N, H, V, seed)
    return _operands(N, H, V, seed)


@pytest.mark.parametrize("plan", ["saved_p", "recompute"])
@pytest.mark.parametrize("kind,N,H,V", [
    ("flat", 6144, 768, 50257), ("peaked", 6144, 768, 50257), ("flat", 12288, 768, 32128),
    ("peaked", 12288, 768, 32128), ("peaked", 1000, 512, 5000), ("flat", 333, 768, 1031), ("flat", 17, 768, 100),
    ("flat", 70, 512, 33)])
def test_lm_head_loss_side_halves(kind, N, H, V, plan):
    """The drop-in pair's saved E, dh and dW against fp64 (C2: V 50257, C3: V 32128 at their
    token counts; flat and peaked softmax; ragged token counts and vocab sizes off the tiles;
    both dW plans), each half by itself (tests/lmloss_checks.py): fp32 outputs (dh sees E at
    2^-7 of |g|·‖E‖) and bf16 outputs."""
    h, w, y = _halves_operands(kind, N, H, V, N + V)
    gout = torch.randn(N, generator=torch.Generator().manual_seed(7))
    t = C.fp64_truth(h.to(DEV), w.to(DEV), y.to(DEV), gout.to(DEV))
    if kind == "peaked":  # the case is what it says: the label's probability is far from 1/V
        p_lab = torch.exp(t["lp"])
        assert float(p_lab.median()) > 0.05, float(p_lab.median())
    for dh_dt, dw_dt in ((torch.float32, torch.float32), (torch.bfloat16, torch.bfloat16)):
        lp, lse, e, dh, dw = _fwd_saved_bwd(h, w, y, gout, dh_dt, dw_dt, plan)
        torch.testing.assert_close(lp.double(), t["lp"], rtol=1e-5, atol=2e-5)
        torch.testing.assert_close(lse.double(), t["lse"], rtol=1e-6, atol=2e-5)
        errs = C.e_errors(e, t["e"])
        errs.update(C.dw_errors(dw, t["dw"], y))
        errs.update(C.dh_errors(dh, t["dh"], gout, t["e"], fp32_out=dh_dt == torch.float32))
        C.assert_within(errs, f"{kind} N={N} V={V} plan={plan} out={dh_dt}")


def _hot_path_halves(x, B, T, V, H, masked, label):
    """PPOHotPath.step_from_hidden with fp32 gradients against the oracle's loss side in fp64
    (lm_head logits of the same bf16 operands, logprobs_from_logits + ppo_loss, autograd) on
    the product's own experience outputs: the loss, dh per token against the E term it
    carries, dW on the non-label rows, the label rows and per row (lmloss_checks); masked
    tokens contribute nothing and their hidden rows are NaN on the device."""
    d = {k: (v.to(DEV) if isinstance(v, torch.Tensor) else v) for k, v in x.items()}
    if masked:
        d["new_h"] = d["new_h"].masked_fill((d["mask"] == 0)[..., None], float("nan"))
    hp = P.PPOHotPath(P.PPOConfig(), B, T, V, torch.bfloat16, DEV, kl_coef=0.05)
    loss, stats, dh, dw, dv = hp.step_from_hidden(d["h"], d["w"], d["ref_h"], d["w"], d["new_h"], d["labels"],
                                                 d["old_values"], d["values"], d["scores"], lengths=d["lengths"],
                                                 mask=d["mask"], route="fused", loss_route="fused",
                                                 grad_dtype=torch.float32)
    torch.cuda.synchronize()
    assert dh.dtype == torch.float32 and dw.dtype == torch.float32
    st = hp.adv_stats.cpu()
    mu, var = P.modeling.moments_to_mean_var(st, unbiased=True)
    adv_w = ((hp.adv_raw.cpu().double() - mu) * torch.rsqrt(var + 1e-8))
    N = B * T
    hd = x["new_h"].double().to(DEV).reshape(N, H).requires_grad_(True)
    wd = x["w"].double().to(DEV).requires_grad_(True)
    logits = hd @ wd.t()
    lp = orc.logprobs_from_logits(logits, x["labels"].to(DEV).reshape(N))
    lp.retain_grad()
    m = torch.ones(B, T, dtype=torch.long) if x["mask"] is None else x["mask"]
    want, _ = orc.ppo_loss(lp.view(B, T), x["values"].double().to(DEV), hp.lp_old.double(),
                           x["old_values"].double().to(DEV), adv_w.to(DEV), hp.returns.double(), m.to(DEV))
    want.backward()
    g = lp.grad.detach()
    with torch.no_grad():
        e64 = torch.softmax(logits.detach(), -1) @ wd.detach()
    torch.testing.assert_close(loss.double().reshape(()), want.detach(), rtol=1e-4, atol=1e-6)
    live = m.reshape(-1).bool()
    errs = C.dw_errors(dw, wd.grad, x["labels"].reshape(-1)[live])
    errs.update(C.dh_errors(dh.reshape(N, H)[live.to(DEV)], hd.grad[live.to(DEV)], g[live.to(DEV)],
                            e64[live.to(DEV)], fp32_out=True))
    C.assert_within(errs, label)
    assert (dh.reshape(N, H)[~live.to(DEV)] == 0).all()
    return [t.clone() for t in (loss, stats, dh, dw, dv)] + [hp.lp_new.clone()]


@pytest.mark.parametrize("B,T,V,H,masked,kind", [(128, 48, 50257, 768, False, "flat"),
                                                 (128, 48, 50257, 768, False, "peaked"),
                                                 (256, 48, 32128, 768, True, "flat"),
                                                 (256, 48, 32128, 768, True, "peaked")])
@pytest.mark.parametrize("plan", [0, 1])
def test_hot_path_loss_side_halves(B, T, V, H, masked, kind, plan):
    """PPOHotPath.step_from_hidden (the PPO route, trlx_ppo_loss_from_hidden) at the C2 and C3
    shards against fp64 (_hot_path_halves), on both dW plans: plan 0 = the default saved-P plan
    (k_lmloss_dwp reads the forward's bf16 P back: its label entries from the fp32 label logit),
    plan 1 = Sᵀ recomputed (k_lmloss_dw)."""
    x = _ppo_inputs(B, T, V, H, 300 + B + T, masked)
    if kind == "peaked":
        nh, w, y = C.peaked_operands(B * T, H, V, 301 + B)
        x["new_h"], x["w"], x["labels"] = nh.view(B, T, H), w, y.view(B, T)
        x["h"] = (nh.float() + 0.05 * torch.randn(B * T, H, generator=torch.Generator().manual_seed(3))).to(
            torch.bfloat16).view(B, T, H)
        x["ref_h"] = (x["h"].float() + 0.1 * torch.randn(B, T, H, generator=torch.Generator().manual_seed(4))).to(
            torch.bfloat16)
    P._lib.set_tuning("lmloss_dw", plan)
    try:
        _hot_path_halves(x, B, T, V, H, masked, f"hot path plan {plan} {kind} B={B} V={V} masked={masked}")
    finally:
        P._lib.set_tuning("lmloss_dw", 0)


@pytest.mark.parametrize("splits,tsplit", [(1, 1), (3, 2), (8, 5), (5, 16)])
def test_hot_path_saved_p_plans(splits, tsplit):
    """The saved-P plan under forced grid plans (vocab splits: each dW wave rescales its P by
    its own split's offset; dW token splits: partials + the fixed-order reduce) and with the
    forward's restart (a logit jump of ~80 from the 3rd W tile on: the restarted blocks rewrite
    their P tiles and offsets), ragged masked batch and H = 512 and 768: fp64 halves checks, and
    against the recompute plan on the same step."""
    for B, T, V, H, jump in ((8, 20, 7000, 768, False), (8, 20, 7000, 768, True), (6, 11, 1031, 512, True)):
        x = _ppo_inputs(B, T, V, H, 40 + splits + tsplit, True)
        if jump:
            wf = x["w"].float()
            dvec = x["new_h"].float().reshape(-1, H).mean(0)
            wf[2 * 32:] += 80.0 * dvec / (dvec @ dvec)
            x["w"] = wf.to(torch.bfloat16)
        P._lib.set_tuning("lmloss_splits", splits)
        P._lib.set_tuning("lmloss_dw_tsplit", tsplit)
        outs = {}
        try:
            for plan in (0, 1):
                P._lib.set_tuning("lmloss_dw", plan)
                outs[plan] = _hot_path_halves(x, B, T, V, H, True,
                                              f"saved-P splits={splits} tsplit={tsplit} H={H} jump={jump} plan={plan}")
        finally:
            for k in ("lmloss_dw", "lmloss_splits", "lmloss_dw_tsplit"):
                P._lib.set_tuning(k, 0)
        a, b = outs[1], outs[0]
        torch.testing.assert_close(b[0], a[0], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(b[4], a[4], rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(b[5], a[5], rtol=1e-5, atol=1e-5)
        assert torch.equal(b[2], a[2])  # dh comes from the combine: the plans differ in dW only
        assert _rel(b[3], a[3]) < 4e-3


def test_lm_head_logprobs_autograd_no_device_allocation_in_steady_state():
    """The drop-in autograd path takes its lp / lse / E / workspace / dh / dW buffers per call
    from PyTorch's stream-ordered caching allocator (lm_head.py): after the first step no call
    reaches hipMalloc — the segment count and the reserved bytes stay put — so a per-call
    torch.empty costs a free-list pop, and two streams never share a workspace (a workspace
    cached in the module would)."""
    N, H, V = 1024, 768, 50257
    h, w, y = _operands(N, H, V, seed=11)
    h = h.to(DEV).requires_grad_(True)
    w = w.to(DEV).requires_grad_(True)
    y = y.to(DEV)

    def step():
        lp = P.lm_head_logprobs(h, w, y)
        lp.float().sum().backward()
        h.grad = None
        w.grad = None

    step()
    step()
    torch.cuda.synchronize()
    st0 = torch.cuda.memory_stats(DEV)
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    st1 = torch.cuda.memory_stats(DEV)
    assert st1["segment.all.allocated"] == st0["segment.all.allocated"]
    assert st1["reserved_bytes.all.current"] == st0["reserved_bytes.all.current"]
