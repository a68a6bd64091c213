"""GPU parity: every HIP kernel, called through the C ABI (via the drop-in Python surface
or directly with _lib.call), against (a) the golden fixtures produced by the reference
and (b) the CPU oracle (oracle/ppo_oracle.py, pinned to those fixtures) on the same
seeded inputs.

Tolerances (BASELINE.json north star):
  gather indices / masks / counts       bit-exact
  fp32 quantities                       rtol 1e-5 (+ small atol for near-zero elements)
  bf16 outputs vs the reference's bf16  rtol 2e-2 (logprobs)
  bf16 *inputs*: kernels compute in fp32, so they are compared at rtol 1e-5 against the
  oracle evaluated in fp32 on the same bf16-quantised inputs (SURVEY §8c precision rule).
"""
import numpy as np
import pytest
import torch

import trlx_t5_amd as P
from trlx_t5_amd import _lib
from golden_util import T, is_bf16, loss_rows_lp
from oracle import ppo_oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")

RT32 = dict(rtol=1e-5, atol=1e-5)


def cuda(t):
    return t.to(DEV)


def lp_fp32_via_abi(logits, labels):
    """lsm_gather_fwd with an fp32 output regardless of the logits dtype (C ABI direct)."""
    x = cuda(logits).contiguous()
    y = cuda(labels).contiguous()
    B, Tn, V = x.shape
    out = torch.empty((B, Tn), dtype=torch.float32, device=DEV)
    lse = torch.empty((B, Tn), dtype=torch.float32, device=DEV)
    _lib.call("trlx_lsm_gather_fwd", x.data_ptr(), None, _lib.dtype_code(x), B, Tn, V, x.stride(0), x.stride(1),
              y.data_ptr(), y.stride(0), y.stride(1), out.data_ptr(), None, _lib.F32, lse.data_ptr(), None,
              _lib.stream_of(x))
    return out.cpu(), lse.cpu()


# ------------------------------------------------------------------ A1 logprobs_from_logits
CASES_LSM = ["small_f32", "small_bf16", "peaked_f32", "wide50257_f32", "wide50257_bf16", "wide32128_bf16"]


@pytest.mark.parametrize("case", CASES_LSM)
def test_logprobs_golden(golden, case):
    z = golden("lsm_gather")
    x, y = T(z[f"{case}/logits"]), T(z[f"{case}/labels"])
    want = T(z[f"{case}/lp"])
    got = P.logprobs_from_logits(cuda(x), cuda(y)).cpu()
    assert got.dtype == x.dtype
    if x.dtype == torch.bfloat16:
        torch.testing.assert_close(got.float(), want.float(), rtol=2e-2, atol=2e-2)
    else:
        torch.testing.assert_close(got, want, **RT32)
    # fp32 arithmetic on the (quantised) inputs vs the fp32 oracle
    lp32, lse = lp_fp32_via_abi(x, y)
    torch.testing.assert_close(lp32, orc.logprobs_from_logits(x.float(), y), **RT32)
    torch.testing.assert_close(lse, torch.logsumexp(x.float(), -1), **RT32)


@pytest.mark.parametrize("case", CASES_LSM)
def test_logprobs_backward_golden(golden, case):
    z = golden("lsm_gather")
    x, y, w = T(z[f"{case}/logits"]), T(z[f"{case}/labels"]), T(z[f"{case}/w"])
    xg = cuda(x).requires_grad_(True)
    lp = P.logprobs_from_logits(xg, cuda(y))
    (lp * cuda(w)).sum().backward()
    got = xg.grad.cpu()
    assert got.dtype == x.dtype and got.shape == x.shape
    # fp32 oracle on the quantised inputs (the reference's bf16 autograd rounds its own
    # log-softmax to bf16 first; the fixture is checked with a bf16-ulp tolerance)
    xf = x.float().requires_grad_(True)
    (orc.logprobs_from_logits(xf, y) * w.float()).sum().backward()
    if x.dtype == torch.bfloat16:
        torch.testing.assert_close(got.float(), xf.grad, rtol=1e-2, atol=1e-6)
        torch.testing.assert_close(got.float(), T(z[f"{case}/dlogits"]).float(), rtol=2e-2, atol=2e-4)
    else:
        torch.testing.assert_close(got, xf.grad, **RT32)
        torch.testing.assert_close(got, T(z[f"{case}/dlogits"]), **RT32)


@pytest.mark.parametrize("V", [1, 5, 7, 8, 9, 37, 255, 4097, 32128, 50257])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_logprobs_vocab_edges(V, dt):
    """Head/tail peeling: every row start phase (odd V => rows start at every 2-B offset)."""
    g = torch.Generator().manual_seed(V)
    B, Tn = 3, 5
    x = (torch.randn(B, Tn, V, generator=g) * 3).to(dt)
    y = torch.randint(0, V, (B, Tn), generator=g)
    y[0, 0], y[-1, -1] = 0, V - 1
    lp32, _ = lp_fp32_via_abi(x, y)
    torch.testing.assert_close(lp32, orc.logprobs_from_logits(x.float(), y), **RT32)
    xg = cuda(x).requires_grad_(True)
    P.logprobs_from_logits(xg, cuda(y)).float().sum().backward()
    xf = x.float().requires_grad_(True)
    orc.logprobs_from_logits(xf, y).sum().backward()
    tol = dict(rtol=1e-2, atol=1e-6) if dt == torch.bfloat16 else RT32
    torch.testing.assert_close(xg.grad.float().cpu(), xf.grad, **tol)


def test_logprobs_strided_causal_view():
    """logits[:, :-1] / tokens[:, 1:] (the causal caller pattern) without copies; the grad
    buffer keeps the view's strides and phase."""
    g = torch.Generator().manual_seed(7)
    B, L, V = 3, 6, 1001
    full = torch.randn(B, L, V, generator=g).to(torch.bfloat16)
    tok = torch.randint(0, V, (B, L), generator=g)
    xf = cuda(full).requires_grad_(True)
    lp = P.logprobs_from_logits(xf[:, :-1], cuda(tok)[:, 1:])
    lp.float().sum().backward()
    ref_x = full.float().requires_grad_(True)
    ref = orc.logprobs_from_logits(ref_x[:, :-1], tok[:, 1:])
    ref.sum().backward()
    torch.testing.assert_close(lp.float().cpu(), ref, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(xf.grad.float().cpu(), ref_x.grad, rtol=1e-2, atol=1e-6)
    # 2-D [N, V] input
    lp2 = P.logprobs_from_logits(cuda(full.reshape(-1, V)), cuda(tok.reshape(-1)))
    torch.testing.assert_close(lp2.float().cpu(), orc.logprobs_from_logits(full.float().reshape(-1, V),
                                                                            tok.reshape(-1)), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("pad", [0, 3])
def test_lsm_bwd_split_rows_phase(dt, pad):
    """V 50257 (the split VGPR + LDS residency kernels of both dtypes): logits rows read from
    a wider buffer (row stride V + pad, so row starts drift against the contiguous dx rows:
    the different-phase store path) and from a contiguous one (same phase)."""
    g = torch.Generator().manual_seed(50 + pad)
    B, Tn, V = 2, 7, 50257
    full = (torch.randn(B, Tn, V + pad, generator=g) * 2).to(dt)
    x = full[..., :V]
    y = torch.randint(0, V, (B, Tn), generator=g)
    y[0, 0], y[-1, -1] = 0, V - 1
    gr = torch.randn(B, Tn, generator=g)
    xd, yd, gd = cuda(full)[..., :V], cuda(y), cuda(gr)
    lse = torch.empty((B, Tn), dtype=torch.float32, device=DEV)
    lp = torch.empty((B, Tn), dtype=torch.float32, device=DEV)
    _lib.call("trlx_lsm_gather_fwd", xd.data_ptr(), None, _lib.dtype_code(xd), B, Tn, V, xd.stride(0), xd.stride(1),
              yd.data_ptr(), yd.stride(0), yd.stride(1), lp.data_ptr(), None, _lib.F32, lse.data_ptr(), None,
              _lib.stream_of(xd))
    dx = torch.full((B, Tn, V), 7.0, dtype=dt, device=DEV)
    _lib.call("trlx_lsm_gather_bwd", xd.data_ptr(), _lib.dtype_code(xd), B, Tn, V, xd.stride(0), xd.stride(1),
              yd.data_ptr(), yd.stride(0), yd.stride(1), lse.data_ptr(), gd.data_ptr(), _lib.F32,
              dx.data_ptr(), dx.stride(0), dx.stride(1), _lib.stream_of(xd))
    xf = x.float().requires_grad_(True)
    ref_lp = orc.logprobs_from_logits(xf, y)
    (ref_lp * gr).sum().backward()
    torch.testing.assert_close(lp.cpu(), ref_lp.detach(), **RT32)
    tol = dict(rtol=1e-2, atol=1e-6) if dt == torch.bfloat16 else RT32
    torch.testing.assert_close(dx.float().cpu(), xf.grad, **tol)


def test_logprobs_bad_label_is_nan_not_oob():
    x = torch.randn(1, 3, 100)
    y = torch.tensor([[0, 100, -1]])
    lp32, _ = lp_fp32_via_abi(x, y)
    assert torch.isfinite(lp32[0, 0]) and torch.isnan(lp32[0, 1]) and torch.isnan(lp32[0, 2])


def test_logprobs_empty_and_determinism():
    x = cuda(torch.randn(0, 4, 50))
    y = cuda(torch.zeros(0, 4, dtype=torch.long))
    assert P.logprobs_from_logits(x, y).shape == (0, 4)
    g = torch.Generator().manual_seed(1)
    x = cuda(torch.randn(16, 8, 50257, generator=g).to(torch.bfloat16))
    y = cuda(torch.randint(0, 50257, (16, 8), generator=g))
    a, b = P.logprobs_from_logits(x, y), P.logprobs_from_logits(x, y)
    assert torch.equal(a, b)


# ------------------------------------------------------------------ A2 KL reward
@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_kl_rewards_golden(golden, dt):
    z = golden("kl_reward")
    k = f"{dt}/none"
    lp, rlp = T(z[f"{k}/lp"]), T(z[f"{k}/ref_lp"])
    s = T(z[f"{k}/scores_out"])
    got = P.kl_penalty_rewards(cuda(lp), cuda(rlp), float(z[f"{dt}/beta"]), cuda(s)).cpu()
    want = T(z[f"{k}/rewards"])
    if dt == "bf16":
        # fp32 arithmetic on the same bf16 logprobs, rounded once to bf16
        ref32 = orc.kl_penalty_rewards(lp.float(), rlp.float(), 0.05, s)
        torch.testing.assert_close(got.float(), ref32, rtol=1e-2, atol=1e-4)
    else:
        torch.testing.assert_close(got, want, **RT32)


def test_kl_rewards_lengths():
    g = torch.Generator().manual_seed(3)
    B, Tn = 6, 11
    lp, rlp = torch.randn(B, Tn, generator=g), torch.randn(B, Tn, generator=g)
    s = torch.randn(B, generator=g)
    L = torch.tensor([11, 1, 5, 10, 3, 11])
    got = P.kl_penalty_rewards(cuda(lp), cuda(rlp), 0.05, cuda(s), lengths=cuda(L)).cpu()
    torch.testing.assert_close(got, orc.kl_penalty_rewards(lp, rlp, 0.05, s, L), **RT32)


# ------------------------------------------------------------------ A3/A4 whiten
@pytest.mark.parametrize("name", ["f32", "bf16", "f32_big"])
def test_whiten_golden(golden, name):
    z = golden("whiten")
    xs = T(z[f"{name}/xs"])
    for fn_kwargs, key in [({}, "nodist"), ({"shift_mean": False}, "nodist_noshift"),
                           ({"distributed": False}, "nodist_disabled")]:
        got = P.whiten(cuda(xs), **fn_kwargs).cpu()
        assert got.dtype == xs.dtype
        if xs.dtype == torch.bfloat16:
            ref32 = orc.whiten(xs.float(), **fn_kwargs)
            torch.testing.assert_close(got.float(), ref32, rtol=1e-2, atol=1e-2)
        else:
            torch.testing.assert_close(got, T(z[f"{name}/{key}"]), **RT32)


def test_moments_and_global_statistics_single_process():
    g = torch.Generator().manual_seed(5)
    xs = torch.randn(300, 7, generator=g) * 2 + 1
    st = P.moments(cuda(xs)).cpu()
    assert st[2].item() == xs.numel()
    torch.testing.assert_close(st[0], xs.double().sum(), rtol=1e-12, atol=1e-9)
    torch.testing.assert_close(st[1], (xs.double() ** 2).sum(), rtol=1e-12, atol=1e-9)
    m = torch.randint(0, 2, (300, 7))
    assert P.moments(cuda(m)).cpu()[0].item() == m.sum().item()


def test_running_moments_kat_device(golden):
    z = golden("host_state")
    rm = P.RunningMoments()
    assert (rm.mean, rm.var, rm.std, rm.count) == (0, 1, 1, 1e-24)  # modeling.py:78-81
    n = 0
    for i in range(4):
        a = T(z[f"rm/{i}/in"]).float()
        bm, bs = rm.update(cuda(a))
        n += a.numel()
        # the reference's types (modeling.py:83-104): xs-dtype 0-d tensors on xs's device
        for t in (bm, bs, rm.mean, rm.var, rm.std):
            assert isinstance(t, torch.Tensor) and t.dim() == 0 and t.dtype == a.dtype and t.device == DEV
        assert isinstance(rm.count, float) and rm.count == pytest.approx(1e-24 + n)
        assert float(bm) == pytest.approx(float(z[f"rm/{i}/batch_mean"]), rel=1e-6, abs=1e-6)
        assert float(bs) == pytest.approx(float(z[f"rm/{i}/batch_std"]), rel=1e-6)
        assert float(rm.std) == pytest.approx(float(z[f"rm/{i}/std"]), rel=1e-6)
        assert float(rm.mean) == pytest.approx(float(z[f"rm/{i}/mean"]), rel=1e-6, abs=1e-6)
    b16 = P.RunningMoments()
    bm, bs = b16.update(cuda(T(z["rm/0/in"])).to(torch.bfloat16))
    assert bm.dtype == bs.dtype == b16.std.dtype == torch.bfloat16


def test_prepare_scores_one_launch_no_host_sync(golden):
    """ppo_orchestrator.py:96-112 through trlx_score_ctl_update on the RunningMoments record:
    the scaled / clipped scores and the batch moments against the oracle's ScoreControl."""
    g = torch.Generator().manual_seed(11)
    for mode in (False, "running", "ref"):
        rm = P.RunningMoments()
        osc = orc.ScoreControl(mode, 1.5)
        ref_std = None
        for k in range(3):
            sc = torch.rand(24, generator=g) * 8 - 4
            if mode == "ref" and ref_std is None:
                ref_std = float(sc.std())
                osc.ref_std = torch.tensor(ref_std)
            out, bm, bs = P.prepare_scores(cuda(sc), rm, mode, 1.5, ref_std=ref_std)
            want, wbm, wbs = osc(sc)
            torch.testing.assert_close(out.cpu(), want, rtol=1e-6, atol=1e-6)
            assert float(bm) == pytest.approx(float(wbm), rel=1e-6, abs=1e-6)
            assert float(bs) == pytest.approx(float(wbs), rel=1e-6)


# ------------------------------------------------------------------ A5 GAE
def test_gae_golden_all_cases(golden):
    z = golden("gae")
    keys = sorted({k.split("/")[0] for k in z.files})
    for k in keys:
        v, r = T(z[f"{k}/values"]), T(z[f"{k}/rewards"])
        cfg = P.PPOConfig(gamma=float(z[f"{k}/gamma"]), lam=float(z[f"{k}/lam"]))
        whit = k.endswith("_w1")
        adv, ret = cfg.get_advantages_and_returns(cuda(v), cuda(r), v.shape[1], use_whitening=whit)
        adv, ret = adv.cpu(), ret.cpu()
        assert adv.dtype == v.dtype and ret.dtype == v.dtype
        if v.dtype == torch.float32:
            torch.testing.assert_close(adv, T(z[f"{k}/adv"]), **RT32, msg=k)
            torch.testing.assert_close(ret, T(z[f"{k}/ret"]), **RT32, msg=k)
        else:
            a32, r32 = orc.gae(v.float(), r.float(), v.shape[1], cfg.gamma, cfg.lam, use_whitening=whit)
            torch.testing.assert_close(adv.float(), a32, rtol=1e-2, atol=1e-2, msg=k)
            torch.testing.assert_close(ret.float(), r32, rtol=1e-2, atol=1e-2, msg=k)
            # fp32 raw path (no final rounding): 1e-5
            araw, rraw, _ = cfg.gae_raw(cuda(v), cuda(r), v.shape[1])
            a32n, _ = orc.gae(v.float(), r.float(), v.shape[1], cfg.gamma, cfg.lam, use_whitening=False)
            torch.testing.assert_close(araw.cpu(), a32n, **RT32, msg=k)


@pytest.mark.parametrize("B,Tn", [(1, 1), (3, 1), (130, 48), (1024, 128), (7, 300)])
def test_gae_shapes(B, Tn):
    g = torch.Generator().manual_seed(B * 1000 + Tn)
    v, r = torch.randn(B, Tn, generator=g), torch.randn(B, Tn, generator=g)
    cfg = P.PPOConfig(gamma=0.99)
    adv, ret = cfg.get_advantages_and_returns(cuda(v), cuda(r), Tn, use_whitening=B * Tn > 1)
    a, rr = orc.gae(v, r, Tn, 0.99, 0.95, use_whitening=B * Tn > 1)
    torch.testing.assert_close(ret.cpu(), rr, **RT32)
    torch.testing.assert_close(adv.cpu(), a, rtol=1e-5, atol=1e-4)


# ------------------------------------------------------------------ A6 PPO loss
LOSS_CASES = ["random", "masked", "ties", "wide_ratio", "bf16", "vf_coef"]


@pytest.mark.parametrize("case", LOSS_CASES)
def test_ppo_loss_golden(golden, case):
    z = golden("ppo_loss")
    g = {n: T(z[f"{case}/{n}"]) for n in ("lp", "olp", "v", "ov", "adv", "ret", "mask")}
    cfg = P.PPOConfig(vf_coef=float(z[f"{case}/vf_coef"]))
    lp = cuda(g["lp"]).requires_grad_(True)
    v = cuda(g["v"]).requires_grad_(True)
    loss, stats = cfg.loss(lp, v, cuda(g["olp"]), cuda(g["ov"]), cuda(g["adv"]), cuda(g["ret"]), cuda(g["mask"]))
    loss.backward()
    assert set(stats) == set(P.STATS_KEYS)
    for k in ("losses/total_loss", "losses/policy_loss", "losses/value_loss", "policy/approx_kl",
              "policy/clipfrac"):
        assert isinstance(stats[k], float)
    if g["lp"].dtype == torch.bfloat16:
        # fp32 oracle on the bf16-quantised inputs
        lpf = g["lp"].float().requires_grad_(True)
        vf = g["v"].float().requires_grad_(True)
        rloss, rstats = orc.ppo_loss(lpf, vf, *(g[n].float() for n in ("olp", "ov", "adv", "ret")), g["mask"],
                                     vf_coef=cfg.vf_coef)
        rloss.backward()
        want_loss, want_glp, want_gv = rloss.detach(), lpf.grad, vf.grad
        want_stats = {k: float(val) for k, val in rstats.items()}
        gtol = dict(rtol=1e-2, atol=1e-4)  # grads are returned in bf16 (input dtype)
    else:
        want_loss, want_glp, want_gv = T(z[f"{case}/loss"]), T(z[f"{case}/grad_lp"]), T(z[f"{case}/grad_v"])
        want_stats = {k: float(z[f"{case}/stats/{k}"]) for k in P.STATS_KEYS}
        gtol = RT32
    torch.testing.assert_close(loss.detach().cpu().float(), want_loss.float(), **RT32)
    torch.testing.assert_close(lp.grad.cpu().float(), want_glp.float(), **gtol)
    torch.testing.assert_close(v.grad.cpu().float(), want_gv.float(), **gtol)
    for k in P.STATS_KEYS:
        assert float(stats[k]) == pytest.approx(want_stats[k], rel=1e-5, abs=1e-6), k


@pytest.mark.parametrize("dt", ["float32", "bfloat16"])
def test_loss_from_logits_chain_golden(golden, dt):
    """Fused A1+A6 (one pass over each logits row) == logprobs_from_logits -> loss -> backward."""
    z = golden("ppo_loss")
    k = f"chain_{dt}"
    x, y = T(z[f"{k}/logits"]), T(z[f"{k}/labels"])
    olp, ov, adv, ret, v = (T(z[f"{k}/{n}"]) for n in ("olp", "ov", "adv", "ret", "v"))
    cfg = P.PPOConfig()
    xg = cuda(x).requires_grad_(True)
    vg = cuda(v).requires_grad_(True)
    loss, stats, lp_new = cfg.loss_from_logits(xg, vg, cuda(y), cuda(olp), cuda(ov), cuda(adv), cuda(ret))
    loss.backward()
    # oracle in fp32 on the same (quantised) inputs
    xf = x.float().requires_grad_(True)
    vf = v.float().requires_grad_(True)
    lpf = orc.logprobs_from_logits(xf, y)
    rloss, rstats = orc.ppo_loss(lpf, vf, olp.float(), ov.float(), adv.float(), ret.float(),
                                 torch.ones(y.shape, dtype=torch.long))
    rloss.backward()
    torch.testing.assert_close(lp_new.cpu(), lpf.detach(), **RT32)
    torch.testing.assert_close(loss.detach().cpu(), rloss.detach(), **RT32)
    if x.dtype == torch.float32:
        torch.testing.assert_close(xg.grad.cpu(), xf.grad, **RT32)
        torch.testing.assert_close(xg.grad.cpu(), T(z[f"{k}/dlogits"]), **RT32)
        torch.testing.assert_close(vg.grad.cpu(), T(z[f"{k}/grad_v"]), **RT32)
    else:
        torch.testing.assert_close(xg.grad.cpu().float(), xf.grad, rtol=1e-2, atol=1e-7)
        torch.testing.assert_close(vg.grad.cpu().float(), vf.grad, rtol=1e-2, atol=1e-5)
    for key in P.STATS_KEYS:
        assert float(stats[key]) == pytest.approx(float(rstats[key]), rel=1e-5, abs=1e-6), key


# ------------------------------------------------------------------ the fused step (bench path)
def _step_inputs(B, Tn, V, seed, lengths=False):
    g = torch.Generator().manual_seed(seed)
    logits = torch.randn(B, Tn, V, generator=g).to(torch.bfloat16)
    ref_logits = (logits.float() + 0.1 * torch.randn(B, Tn, V, generator=g)).to(torch.bfloat16)
    new_logits = (logits.float() + 0.05 * torch.randn(B, Tn, V, generator=g)).to(torch.bfloat16)
    labels = torch.randint(0, V, (B, Tn), generator=g)
    old_values = torch.randn(B, Tn, generator=g)
    values = old_values + 0.3 * torch.randn(B, Tn, generator=g)
    scores = torch.rand(B, generator=g) * 24 - 12
    L = mask = None
    if lengths:
        L = torch.randint(1, Tn + 1, (B,), generator=g)
        L[0] = Tn
        mask = (torch.arange(Tn)[None, :] < L[:, None]).long()
        old_values = old_values.masked_fill(mask == 0, 0)
    return logits, ref_logits, new_logits, labels, old_values, values, scores, L, mask


@pytest.mark.parametrize("B,Tn,V,lengths", [(4, 9, 1031, False), (8, 48, 50257, False), (16, 48, 32128, True),
                                            (128, 48, 50257, False)])
def test_hot_path_step_vs_oracle(B, Tn, V, lengths):
    """PPOHotPath.step (K1..K6) vs the oracle's restated step; the last case is the full
    GPT-2 sentiments bench shape (configs[1])."""
    logits, ref_logits, new_logits, labels, old_values, values, scores, L, mask = _step_inputs(B, Tn, V, B + V,
                                                                                               lengths)
    hp = P.PPOHotPath(P.PPOConfig(), B, Tn, V, torch.bfloat16, DEV, kl_coef=0.05)
    loss, stats, dlogits, dvalues = hp.step(cuda(logits), cuda(ref_logits), cuda(new_logits), cuda(labels),
                                            cuda(old_values), cuda(values), cuda(scores),
                                            lengths=None if L is None else cuda(L),
                                            mask=None if mask is None else cuda(mask))
    torch.cuda.synchronize()
    ref = orc.ppo_step_reference(logits.float(), ref_logits.float(), new_logits.float(), labels, old_values,
                                 values, scores, kl_coef=0.05, lengths=L, mask=mask)
    torch.testing.assert_close(hp.lp_old.cpu(), ref["lp"], **RT32)
    torch.testing.assert_close(hp.ref_lp.cpu(), ref["ref_lp"], **RT32)
    torch.testing.assert_close(hp.rewards.cpu(), ref["rewards"], **RT32)
    torch.testing.assert_close(hp.returns.cpu(), ref["returns"], **RT32)
    torch.testing.assert_close(hp.lp_new.cpu(), loss_rows_lp(ref["new_lp"], mask), **RT32)
    torch.testing.assert_close(loss.cpu().reshape(()), ref["loss"], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dvalues.cpu(), ref["dvalues"], rtol=1e-5, atol=1e-9)
    # dlogits are written in the logits dtype (bf16): one rounding of the fp32 value
    torch.testing.assert_close(dlogits.float().cpu(), ref["dlogits"], rtol=8e-3, atol=1e-9)
    st = stats.cpu().tolist()
    for i, k in enumerate(P.STATS_KEYS):
        assert st[i] == pytest.approx(float(ref["stats"][k]), rel=1e-5, abs=1e-6), k
    # size-independent properties at full size: every dlogits row sums to ~0
    row_sum = dlogits.float().sum(-1)
    assert row_sum.abs().max().item() < 1e-3


def test_hot_path_step_is_deterministic_and_rearms():
    """Same inputs -> bitwise-identical outputs, across fresh instances and across repeated
    steps of one instance (the in-kernel arrival tickets re-arm themselves)."""
    args = _step_inputs(32, 48, 50257, 11)
    logits, ref_logits, new_logits, labels, old_values, values, scores, _, _ = args
    d = [cuda(t) for t in (logits, ref_logits, new_logits, labels, old_values, values, scores)]
    outs = []
    hp = P.PPOHotPath(P.PPOConfig(), 32, 48, 50257, torch.bfloat16, DEV, kl_coef=0.05)
    for i in range(4):
        if i == 3:
            hp = P.PPOHotPath(P.PPOConfig(), 32, 48, 50257, torch.bfloat16, DEV, kl_coef=0.05)
        loss, stats, dl, dv = hp.step(*d)
        outs.append((loss.clone(), stats.clone(), dl.clone(), dv.clone(), hp.adv_stats.clone(), hp.returns.clone()))
    for other in outs[1:]:
        for a, b in zip(outs[0], other):
            assert torch.equal(a, b)
    assert int(hp.workspace.view(torch.int32)[:4].abs().sum()) == 0  # arrival tickets re-armed


@pytest.mark.parametrize("T", [1, 63, 64, 65, 130])
def test_fused_experience_tail_chunking(T):
    """The lane-parallel GAE scan in the experience tail across 64-token chunk boundaries."""
    B, V = 6, 257
    logits, ref_logits, new_logits, labels, old_values, values, scores, L, mask = _step_inputs(B, T, V, 77 + T,
                                                                                               lengths=T > 1)
    hp = P.PPOHotPath(P.PPOConfig(gamma=0.99), B, T, V, torch.bfloat16, DEV, kl_coef=0.05)
    hp.step(cuda(logits), cuda(ref_logits), cuda(new_logits), cuda(labels), cuda(old_values), cuda(values),
            cuda(scores), lengths=None if L is None else cuda(L), mask=None if mask is None else cuda(mask))
    torch.cuda.synchronize()
    ref = orc.ppo_step_reference(logits.float(), ref_logits.float(), new_logits.float(), labels, old_values,
                                 values, scores, cfg_kwargs=dict(gamma=0.99), kl_coef=0.05, lengths=L, mask=mask)
    torch.testing.assert_close(hp.rewards.cpu(), ref["rewards"], **RT32)
    torch.testing.assert_close(hp.returns.cpu(), ref["returns"], rtol=1e-5, atol=2e-5)
    if B * T > 1:
        mu = hp.adv_stats[0].item() / hp.adv_stats[2].item()
        torch.testing.assert_close(torch.tensor(mu), (ref["returns"] - (old_values if L is None else
                                   old_values.masked_fill(mask == 0, 0))).mean().double().float(),
                                   rtol=1e-4, atol=1e-5)


def test_hot_path_step_fp32_logits():
    """The GPT path's fp32 logits (the reference's GPT heads are fp32) through the fused step."""
    B, Tn, V = 8, 48, 50257
    g = torch.Generator().manual_seed(31)
    logits = torch.randn(B, Tn, V, generator=g)
    ref_logits = logits + 0.1 * torch.randn(B, Tn, V, generator=g)
    new_logits = logits + 0.05 * torch.randn(B, Tn, V, generator=g)
    labels = torch.randint(0, V, (B, Tn), generator=g)
    old_values = torch.randn(B, Tn, generator=g)
    values = old_values + 0.3 * torch.randn(B, Tn, generator=g)
    scores = torch.rand(B, generator=g) * 24 - 12
    hp = P.PPOHotPath(P.PPOConfig(), B, Tn, V, torch.float32, DEV, kl_coef=0.05)
    loss, stats, dlogits, dvalues = hp.step(cuda(logits), cuda(ref_logits), cuda(new_logits), cuda(labels),
                                            cuda(old_values), cuda(values), cuda(scores))
    torch.cuda.synchronize()
    ref = orc.ppo_step_reference(logits, ref_logits, new_logits, labels, old_values, values, scores, kl_coef=0.05)
    torch.testing.assert_close(hp.lp_old.cpu(), ref["lp"], **RT32)
    torch.testing.assert_close(hp.rewards.cpu(), ref["rewards"], **RT32)
    torch.testing.assert_close(loss.cpu().reshape(()), ref["loss"], rtol=1e-5, atol=1e-6)
    assert dlogits.dtype == torch.float32
    torch.testing.assert_close(dlogits.cpu(), ref["dlogits"], rtol=1e-4, atol=1e-9)
    # dv = vf_coef / Σm · (v - R): near v = R only the returns' rounding is left — a few fp32
    # ulps of |R| ~ 15 (GAE sums ~1e-6 apart) times 1/Σm = 1/384 -> atol 1e-8
    torch.testing.assert_close(dvalues.cpu(), ref["dvalues"], rtol=1e-5, atol=1e-8)


@pytest.mark.parametrize("V,dt", [(50257, torch.bfloat16), (32128, torch.bfloat16), (50257, torch.float32)])
def test_tuning_knobs_do_not_change_results(V, dt):
    """trlx_set_tuning only changes speed: store cache policies give bit-identical rows,
    split residency / vector order change the fp32 summation order only."""
    B, Tn = 3, 7
    logits, ref_logits, new_logits, labels, old_values, values, scores, _, _ = _step_inputs(B, Tn, V, 5)
    args = [cuda(t) for t in (logits.to(dt), ref_logits.to(dt), new_logits.to(dt), labels, old_values, values,
                              scores)]

    def run():
        hp = P.PPOHotPath(P.PPOConfig(), B, Tn, V, dt, DEV, kl_coef=0.05)
        loss, stats, dl, dv = hp.step(*args)
        torch.cuda.synchronize()
        return [hp.lp_old.clone(), hp.ref_lp.clone(), loss.clone(), stats.clone(), dl.clone(), dv.clone()]

    base = run()
    try:
        for key, vals, exact in [("store_policy", [1, 2, 3, 4, 5], True), ("split_lds", [1, 2], False),
                                 ("split_mid", [1, 2, 3], False), ("row_order", [1], False),
                                 ("row_variant", [2], False)]:
            for v in vals:
                _lib.set_tuning(key, v)
                got = run()
                _lib.set_tuning(key, 0)
                for a, b in zip(base, got):
                    if exact:
                        assert torch.equal(a, b), (key, v)
                    else:
                        tol = dict(rtol=8e-3, atol=1e-9) if b.dtype == torch.bfloat16 else dict(rtol=1e-5, atol=1e-6)
                        torch.testing.assert_close(b.float(), a.float(), **tol, msg=f"{key}={v}")
    finally:
        for key in ("store_policy", "split_lds", "split_mid", "row_order", "row_variant"):
            _lib.set_tuning(key, 0)


def _special_rows(V, g):
    """Rows that probe the bf16 raw-bits maximum (csrc/vocab_rows.hip): its fast path holds
    for rows whose maximum is >= +0, the rest take the exact float pass."""
    rows = []
    base = torch.randn(V, generator=g)
    rows.append(base * 3)                                   # ordinary
    rows.append(torch.log_softmax(base * 2, -1))            # log-probs as logits: max < 0 (fallback)
    rows.append(-250.0 - base.abs() * 50)                   # all <= -250: exp underflow if m were off
    r = base.clone(); r[::3] = -float("inf"); rows.append(r)  # masked vocabulary (-inf)
    r = -base.abs() - 1; r[V // 2] = 0.0; rows.append(r)     # max exactly +0
    r = -base.abs() - 1; r[V // 3] = -0.0; rows.append(r)    # max -0.0 (bits 0x8000: fallback)
    rows.append(base * 3e4)                                  # huge magnitudes
    rows.append(-1e4 + base)                                 # all near -1e4
    r = base.clone(); r[7] = float("inf"); rows.append(r)    # +inf -> NaN row (as log_softmax)
    r = base.clone(); r[V - 2] = float("nan"); rows.append(r)  # NaN -> NaN row
    return torch.stack(rows)


@pytest.mark.parametrize("V", [50257, 32128, 1031, 9])
def test_logprobs_special_values_bf16(V):
    """bf16 rows with negative-only maxima, -0.0, +-inf, NaN and huge magnitudes: forward
    logprobs (experience rows), the fused loss rows' new logprobs and the backward all equal
    the oracle's log_softmax semantics on the same bf16 values (NaN where it gives NaN)."""
    g = torch.Generator().manual_seed(77 + V)
    x = _special_rows(V, g).to(torch.bfloat16)
    N = x.shape[0]
    labels = torch.randint(0, V, (N,), generator=g)
    labels[8] = 7  # the +inf element itself
    ref = orc.logprobs_from_logits(x.float(), labels)
    xd = x.to(DEV).requires_grad_(True)
    lp = P.logprobs_from_logits(xd, labels.to(DEV))
    torch.testing.assert_close(lp.float().cpu(), ref.to(torch.bfloat16).float(), rtol=2e-2, atol=1e-2,
                               equal_nan=True)
    # fp32 outputs: the experience kernel's path (trlx_lsm_gather_fwd into fp32)
    out = torch.empty(1, N, dtype=torch.float32, device=DEV)
    xr = x.to(DEV).view(1, N, V)
    _lib.call("trlx_lsm_gather_fwd", xr.data_ptr(), None, _lib.dtype_code(xr), 1, N, V, xr.stride(0), xr.stride(1),
              labels.to(DEV).data_ptr(), 0, 1, out.data_ptr(), None, _lib.F32, None, None,
              torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    torch.testing.assert_close(out.view(N).cpu(), ref, rtol=1e-5, atol=1e-5, equal_nan=True)
    assert torch.isnan(out.view(N)[8]).item() and torch.isnan(out.view(N)[9]).item()
    # backward (lse from the forward) and the fused loss rows' lp_new
    lp.float().sum().backward()
    xo = x.float().clone().requires_grad_(True)
    orc.logprobs_from_logits(xo, labels).sum().backward()
    ok = torch.isfinite(ref)
    torch.testing.assert_close(xd.grad[ok.to(DEV)].float().cpu(), xo.grad[ok], rtol=2e-2, atol=1e-6)
    cfg = P.PPOConfig()
    ones = torch.ones(1, N, device=DEV)
    loss, _, lp_new = cfg.loss_from_logits(xr, ones, labels.to(DEV).view(1, N), out, ones, ones, ones,
                                           return_device_stats=True)
    torch.cuda.synchronize()
    torch.testing.assert_close(lp_new.view(N).cpu(), ref, rtol=1e-5, atol=1e-5, equal_nan=True)
