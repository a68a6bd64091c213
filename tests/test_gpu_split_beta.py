"""Split-beta GAE (trlx_ppo_rollout_gae_split / trlx_ppo_whiten_coef / trlx_ppo_loss_rows_split),
the arithmetic of the pipelined data-parallel schedule.

The KL-penalised reward r = score_t - beta*kl_t (ppo_orchestrator.py:163-167) enters GAE
(ppo_models.py:121-139) linearly: A = A0 - beta*Ak.  The GAE launch computes A0, Ak and the
split whitening record without beta; the loss rows apply beta, whiten (modeling.py:24-34) and
write this batch's rewards and returns.  Pinned here against the oracle (the reference's
sequential arithmetic, rtol 1e-5), against the unsplit kernels, and pipeline_step (one
process, no process group) against step(split_beta=True) bit for bit — the folded
coefficient launch, the deferred tails and the double-buffered controller state included.
"""
import numpy as np
import pytest
import torch

import trlx_t5_amd as P
from oracle import ppo_oracle as orc
from golden_util import loss_rows_lp

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
RT32 = dict(rtol=1e-5, atol=1e-5)


def cuda(t):
    return None if t is None else t.to(DEV)


def _inputs(B, Tn, V, seed, lengths=False):
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
    return dict(logits=logits, ref_logits=ref_logits, new_logits=new_logits, labels=labels, old_values=old_values,
                values=values, scores=scores, lengths=L, mask=mask)


def _args(x):
    return [cuda(x[k]) for k in ("logits", "ref_logits", "new_logits", "labels", "old_values", "values", "scores")]


@pytest.mark.parametrize("B,Tn,V,lengths,gamma", [(4, 9, 1031, False, 1.0), (16, 48, 32128, True, 1.0),
                                                  (6, 65, 257, True, 0.99), (5, 130, 257, False, 0.99),
                                                  (3, 1, 257, False, 1.0), (128, 48, 50257, False, 1.0)])
def test_split_step_vs_oracle(B, Tn, V, lengths, gamma):
    """step(split_beta=True) vs the oracle's restated step (sequential GAE, native order)."""
    x = _inputs(B, Tn, V, 900 + B + Tn, lengths)
    hp = P.PPOHotPath(P.PPOConfig(gamma=gamma), B, Tn, V, torch.bfloat16, DEV, kl_coef=0.05, split_beta=True)
    loss, stats, dlogits, dvalues = hp.step(*_args(x), lengths=cuda(x["lengths"]), mask=cuda(x["mask"]))
    hp.wait_stats()
    torch.cuda.synchronize()
    ref = orc.ppo_step_reference(x["logits"].float(), x["ref_logits"].float(), x["new_logits"].float(), x["labels"],
                                 x["old_values"], x["values"], x["scores"], cfg_kwargs=dict(gamma=gamma),
                                 kl_coef=0.05, lengths=x["lengths"], mask=x["mask"])
    torch.testing.assert_close(hp.rewards.cpu(), ref["rewards"], **RT32)
    torch.testing.assert_close(hp.returns.cpu(), ref["returns"], rtol=1e-5, atol=2e-5)
    torch.testing.assert_close(hp.lp_new.cpu(), loss_rows_lp(ref["new_lp"], x["mask"]), **RT32)
    torch.testing.assert_close(loss.cpu().reshape(()), ref["loss"], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dvalues.cpu(), ref["dvalues"], rtol=1e-5, atol=1e-8)
    torch.testing.assert_close(dlogits.float().cpu(), ref["dlogits"], rtol=8e-3, atol=1e-9)
    st = stats.cpu().tolist()
    for i, k in enumerate(P.STATS_KEYS):
        assert st[i] == pytest.approx(float(ref["stats"][k]), rel=1e-5, abs=1e-6), k
    # the split record: n and Σmask exact; Σ A = Σ A0 - beta Σ Ak is the reference's Σ advantages
    rec = hp.adv_stats.cpu().double()
    assert rec[2].item() == B * Tn and rec[6].item() == (B * Tn if x["mask"] is None else x["mask"].sum().item())
    adv = ref["returns"].double() - x["old_values"].double()
    assert (rec[0] - 0.05 * rec[3]).item() == pytest.approx(adv.sum().item(), rel=1e-5, abs=1e-4)
    assert int(hp.workspace.view(torch.int32)[:4].abs().sum()) == 0  # arrival tickets re-armed


@pytest.mark.parametrize("use_ctl,lengths,defer", [(True, True, True), (False, False, True), (True, False, False)])
def test_pipelined_world1_matches_serial_split(use_ctl, lengths, defer):
    """pipeline_step (GAE(k+1) folding batch k's whitening coefficients, loss tails deferred
    into the next experience launch or run in-stream) vs step(split_beta=True): every
    batch's loss, stats, dlogits, dvalues, rewards and returns, and the final controller
    state, bit-identical; vs the unsplit step(): fp32 association only."""
    B, Tn, V = 8, 21, 1031
    batches = [_inputs(B, Tn, V, 60 + i, lengths) for i in range(4)]
    res = {}
    for mode in ("serial", "pipelined", "unsplit"):
        cfg = P.PPOConfig(scale_reward="running")
        ctl = P.PPOControlState.from_config(cfg, DEV, n_steps=B) if use_ctl else None
        hp = P.PPOHotPath(cfg, B, Tn, V, torch.bfloat16, DEV, kl_coef=0.05, ctl=ctl, defer_tail=defer,
                          split_beta=mode != "unsplit")
        outs = []

        def grab(o):
            hp.wait_stats()
            torch.cuda.synchronize()
            outs.append([t.float().cpu().clone() for t in o] + [hp.rewards.cpu().clone(), hp.returns.cpu().clone()])

        for x in batches:
            kw = dict(lengths=cuda(x["lengths"]), mask=cuda(x["mask"]))
            if mode == "pipelined":
                o = hp.pipeline_step(*_args(x), **kw)
                if o is not None:
                    grab(o)
            else:
                grab(hp.step(*_args(x), **kw))
        if mode == "pipelined":
            grab(hp.pipeline_flush())
        hp.wait_stats()
        torch.cuda.synchronize()
        res[mode] = (outs, ctl.state.cpu().clone() if use_ctl else None)
    (ser, ser_st), (pip, pip_st), (uns, uns_st) = res["serial"], res["pipelined"], res["unsplit"]
    assert len(ser) == len(pip) == len(uns) == len(batches)
    for i, (a, b, c) in enumerate(zip(ser, pip, uns)):
        for j, (u, v, w) in enumerate(zip(a, b, c)):
            assert torch.equal(u, v), f"batch {i} output {j}"
            torch.testing.assert_close(w, u, rtol=2e-2 if j == 2 else 1e-4, atol=1e-5, msg=f"batch {i} output {j}")
    if use_ctl:
        assert torch.equal(ser_st, pip_st)
        torch.testing.assert_close(uns_st, ser_st, rtol=1e-5, atol=0)


def test_split_second_loss_reuses_the_experience_beta():
    """ppo_epochs pattern: one experience, two policy_loss calls on a changing policy.  The
    second loss reuses the batch's coefficients (the rewards were fixed at experience time,
    as the reference's rollout store fixes them), even though the first loss's tail has
    advanced beta — equal to the unsplit kernels up to fp32 association."""
    B, Tn, V = 8, 17, 1031
    x = _inputs(B, Tn, V, 7)
    g = torch.Generator().manual_seed(8)
    new2 = (x["new_logits"].float() + 0.05 * torch.randn(B, Tn, V, generator=g)).to(torch.bfloat16)
    outs = {}
    for split in (True, False):
        cfg = P.PPOConfig()
        ctl = P.PPOControlState.from_config(cfg, DEV, n_steps=B)
        hp = P.PPOHotPath(cfg, B, Tn, V, torch.bfloat16, DEV, kl_coef=0.05, ctl=ctl, defer_tail=True,
                          split_beta=split)
        a = _args(x)
        hp.experience(a[0], a[1], a[3], a[4], a[6])
        r = []
        for nl in (x["new_logits"], new2):
            loss, stats, dl, dv = hp.policy_loss(cuda(nl), a[3], a[5], a[4])
            hp.wait_stats()
            torch.cuda.synchronize()
            r.append([loss.cpu().clone(), stats.cpu().clone(), dl.float().cpu().clone(), dv.cpu().clone()])
        outs[split] = (r, ctl.state.cpu().clone())
    for a, b in zip(outs[True][0], outs[False][0]):
        for j, (u, v) in enumerate(zip(a, b)):
            torch.testing.assert_close(u, v, rtol=2e-2 if j == 2 else 1e-4, atol=1e-5)
    torch.testing.assert_close(outs[True][1], outs[False][1], rtol=1e-5, atol=0)


def test_whiten_coef_matches_fold():
    """The standalone coefficient launch and the one folded into the next GAE launch give
    the same bits (same function, same beta)."""
    B, Tn, V = 6, 13, 257
    x = _inputs(B, Tn, V, 3)
    hp = P.PPOHotPath(P.PPOConfig(), B, Tn, V, torch.bfloat16, DEV, kl_coef=0.05, split_beta=True)
    hp.experience(*[cuda(x[k]) for k in ("logits", "ref_logits", "labels", "old_values", "scores")])
    sb = hp._sbuf[0]
    coef = torch.empty(4, dtype=torch.float32, device=DEV)
    s = torch.cuda.current_stream(DEV).cuda_stream
    P._lib.call("trlx_ppo_whiten_coef", sb["stats"].data_ptr(), 1, None, 0.05, coef.data_ptr(), s)
    # fold: a second GAE launch into set 1 emitting set 0's coefficients
    sb1 = hp._sbuf[1]
    lp, rlp = hp.lp_old, hp.ref_lp
    ov = cuda(x["old_values"])
    P._lib.call("trlx_ppo_rollout_gae_split", B, Tn, lp.data_ptr(), rlp.data_ptr(), ov.data_ptr(), P._lib.F32,
                cuda(x["scores"]).data_ptr(), None, None, None, 0.05, 1.0, 0.95, sb1["adv0"].data_ptr(),
                sb1["adv_kl"].data_ptr(), sb1["rew_kl"].data_ptr(), sb1["rew_score"].data_ptr(),
                sb1["stats"].data_ptr(), sb["stats"].data_ptr(), sb["coef"].data_ptr(), 1, 0, hp.workspace.data_ptr(), s,
                None)
    torch.cuda.synchronize()
    assert torch.equal(coef, sb["coef"])
    assert torch.equal(sb1["stats"], sb["stats"]) and torch.equal(sb1["adv0"], sb["adv0"])
    # mean / rstd of A = A0 - beta*Ak (unbiased: the var_mean branch)
    A = (sb["adv0"] - 0.05 * sb["adv_kl"]).double()
    mu = A.mean().item()
    assert coef[0].item() == pytest.approx(mu, rel=1e-5, abs=1e-6)
    assert coef[1].item() == pytest.approx((A.var(unbiased=True).item() + 1e-8) ** -0.5, rel=1e-5)
    assert coef[2].item() == np.float32(0.05)


def test_serial_entry_points_refuse_a_pending_pipeline_batch():
    """after pipeline_step the last batch's loss exists only inside the pipeline;
    step() / experience() / experience_from_hidden() raise until pipeline_flush() ran it."""
    B, Tn, V = 4, 9, 1031
    x = _inputs(B, Tn, V, 4242)
    hp = P.PPOHotPath(P.PPOConfig(), B, Tn, V, torch.bfloat16, DEV, kl_coef=0.05, defer_tail=True)
    assert hp.pipeline_step(*_args(x)) is None
    a = _args(x)
    with pytest.raises(RuntimeError, match="pipeline_flush"):
        hp.step(*a)
    with pytest.raises(RuntimeError, match="pipeline_flush"):
        hp.experience(a[0], a[1], a[3], a[4], a[6])
    h = torch.zeros(B, Tn, 64, dtype=torch.bfloat16, device=DEV)
    w = torch.zeros(V, 64, dtype=torch.bfloat16, device=DEV)
    with pytest.raises(RuntimeError, match="pipeline_flush"):
        hp.experience_from_hidden(h, w, h, w, a[3], a[4], a[6])
    assert hp.pipeline_flush() is not None
    hp.step(*a)  # fine again
    torch.cuda.synchronize()
