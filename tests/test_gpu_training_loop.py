"""End-to-end parity of the reference's PPO training-loop semantics (A9 glue) through the
drop-in surface, against the oracle running the same sequence with the same permutations.

Reference flow restated (file:line in danyang-rainbow/trlx-t5):
  make_experience per chunk   ppo_orchestrator.py:96-112 (RunningMoments + scale + clip),
                              :154-155 (logprobs_from_logits x2), :163-167 (KL reward),
                              :169-187 (push to the rollout store)
  prepare_learning            accelerate_ppo_model.py:139-148: store.create_loader(
                              train.batch_size, shuffle=True) — batch_size != chunk_size here
  learn                       accelerate_base_model.py:251-265: for epoch, for minibatch,
                              ppo_epochs (= 4) updates on the SAME minibatch
  loss                        accelerate_ppo_model.py:79-126: GAE + whiten per minibatch
                              (:88-90, recomputed on every update), logprobs_from_logits on
                              the new logits with labels = response (no shift, seq2seq),
                              mask = ones_like (:111), PPOConfig.loss
  post_backward_callback      accelerate_ppo_model.py:136-137: kl_ctl.update(approx_kl of the
                              LAST update, n_steps = train.batch_size) once per minibatch
Two chunks with different response widths make the collated minibatches right-padded
(ppo_pipeline.py:47-65), and the all-ones mask keeps the padding in the loss, as the
reference does.  The model is replaced by deterministic functions of (rollout, update):
new logits / values for rollout i at update u.  fp32 logits (the GPT-path dtype) so that
losses, stats, grads and beta can be held at 1e-5.

Two loss-side routes are checked against the same oracle sequence:
  "drop_in"  logprobs_from_logits + PPOConfig.get_advantages_and_returns + PPOConfig.loss
  "fused"    PPOConfig.gae_raw once per minibatch + PPOConfig.loss_from_logits (whitening
             on the fly from the scan's moments, one read + one write of each logits row)
"""
import pytest
import torch

import trlx_t5_amd as P
from oracle import ppo_oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
V = 1031
CHUNKS = ((24, 10, 7), (24, 8, 5))  # (rollouts, response width, query width)
BATCH, PPO_EPOCHS, EPOCHS = 16, 4, 2


def _chunk(c, n, T, Wq):
    g = torch.Generator().manual_seed(100 + c)
    logits = torch.randn(n, T, V, generator=g) * 2
    ref_logits = logits + 0.2 * torch.randn(n, T, V, generator=g)
    response = torch.randint(1, V, (n, T), generator=g)
    query = torch.randint(1, V, (n, Wq), generator=g)
    values = torch.randn(n, T, generator=g)
    scores = torch.rand(n, generator=g) * 30 - 15
    return logits, ref_logits, response, query, values, scores


def _model(rows, T, u, base_logits, base_values):
    """The 'policy forward' at update u for global rollouts `rows`, padded to width T (the
    reference's model sees the padded response as decoder input)."""
    lg = base_logits[rows, :T] * (1.0 + 0.03 * u) + 0.01 * u
    v = base_values[rows, :T] + 0.05 * u
    return lg, v


@pytest.mark.parametrize("route", ["drop_in", "fused"])
def test_training_loop_parity(route):
    cfg = P.PPOConfig(scale_reward="running", cliprange_reward=10)
    kl = P.AdaptiveKLController(cfg.init_kl_coef, cfg.target, cfg.horizon)
    okl = orc.AdaptiveKLController(cfg.init_kl_coef, cfg.target, cfg.horizon)
    running = P.RunningMoments()
    osc = orc.ScoreControl("running", 10)
    store = P.PPORolloutStorage(pad_token_id=0, device=DEV)
    oelems = []
    Tmax = max(T for _, T, _ in CHUNKS)
    n_all = sum(n for n, _, _ in CHUNKS)
    g = torch.Generator().manual_seed(7)
    base_logits = torch.randn(n_all, Tmax, V, generator=g) * 2  # the policy being trained
    base_values = torch.randn(n_all, Tmax, generator=g)

    # ---- make_experience, chunk by chunk (ppo_orchestrator.py:59-196)
    for c, (n, T, Wq) in enumerate(CHUNKS):
        logits, ref_logits, response, query, values, scores = _chunk(c, n, T, Wq)
        s_dev, _, _ = P.prepare_scores(scores.to(DEV), running, "running", 10)
        lp = P.logprobs_from_logits(logits.to(DEV), response.to(DEV))
        ref_lp = P.logprobs_from_logits(ref_logits.to(DEV), response.to(DEV))
        rewards = P.kl_penalty_rewards(lp, ref_lp, kl.value, s_dev)
        store.push_batch(query.to(DEV), response.to(DEV), lp, values.to(DEV), rewards)
        # oracle
        s_o, _, _ = osc(scores)
        olp = orc.logprobs_from_logits(logits, response)
        oref = orc.logprobs_from_logits(ref_logits, response)
        orw = orc.kl_penalty_rewards(olp, oref, okl.value, s_o)
        torch.testing.assert_close(rewards.cpu(), orw, rtol=1e-5, atol=1e-5)
        for i in range(n):
            oelems.append(P.PPORLElement(query[i], response[i], olp[i], values[i], orw[i]))

    # ---- learn (accelerate_base_model.py:251-265)
    u = 0
    for epoch in range(EPOCHS):
        perm_seed = 1000 + epoch
        loader = store.create_loader(BATCH, shuffle=True, generator=torch.Generator().manual_seed(perm_seed))
        order = torch.randperm(n_all, generator=torch.Generator().manual_seed(perm_seed))
        for k, batch in enumerate(loader):
            rows = order[k * BATCH:(k + 1) * BATCH]
            oq, orsp, olp, ov, orw = orc.ppo_collate([oelems[int(i)] for i in rows], 0)
            assert torch.equal(batch.response_tensors.cpu(), orsp) and torch.equal(batch.query_tensors.cpu(), oq)
            T = orsp.shape[1]
            if route == "fused":
                adv_raw, ret, adv_st = cfg.gae_raw(batch.values, batch.rewards, T)
            for _ in range(PPO_EPOCHS):
                lg, vpred = _model(rows, T, u, base_logits, base_values)
                x = lg.to(DEV).requires_grad_(True)
                v = vpred.to(DEV).requires_grad_(True)
                labels = batch.response_tensors
                mask = torch.ones(labels.shape, dtype=torch.long, device=DEV)
                if route == "drop_in":
                    adv, ret = cfg.get_advantages_and_returns(batch.values, batch.rewards, T)
                    lp_new = P.logprobs_from_logits(x, labels)
                    loss, stats = cfg.loss(lp_new, v, batch.logprobs, batch.values, adv, ret, mask)
                else:
                    loss, stats, _ = cfg.loss_from_logits(x, v, labels, batch.logprobs, batch.values, adv_raw, ret,
                                                          mask=mask, adv_stats=adv_st, unbiased=True)
                loss.backward()
                # oracle update u
                oa, oret = orc.gae(ov, orw, T, cfg.gamma, cfg.lam, use_whitening=True)
                xo = lg.clone().requires_grad_(True)
                vo = vpred.clone().requires_grad_(True)
                olp_new = orc.logprobs_from_logits(xo, orsp)
                oloss, ostats = orc.ppo_loss(olp_new, vo, olp, ov, oa, oret, torch.ones_like(orsp))
                oloss.backward()
                torch.testing.assert_close(loss.detach().cpu().reshape(()), oloss.detach(), rtol=1e-5, atol=1e-6,
                                           msg=f"update {u}")
                for key in P.STATS_KEYS:
                    assert float(stats[key]) == pytest.approx(float(ostats[key]), rel=1e-5, abs=1e-6), (u, key)
                # dlogits: the label element g·(1 - p_y) carries the fp32 rounding of lse (|lse| ~ 10,
                # ulp 1e-6, a few ulps apart between any two fp32 evaluation orders) times |g| ~ 6e-3
                torch.testing.assert_close(x.grad.cpu(), xo.grad, rtol=1e-5, atol=5e-8,
                                           msg=lambda m, u=u: f"dlogits {u}: {m}")
                torch.testing.assert_close(v.grad.cpu(), vo.grad, rtol=1e-5, atol=1e-8,
                                           msg=lambda m, u=u: f"dvalues {u}: {m}")
                approx_kl, o_approx_kl = stats["policy/approx_kl"], ostats["policy/approx_kl"]
                u += 1
            kl.update(approx_kl, n_steps=BATCH)  # post_backward_callback: the last update's approx_kl
            okl.update(o_approx_kl, n_steps=BATCH)
            assert kl.value == pytest.approx(okl.value, rel=1e-9)
    assert u == EPOCHS * PPO_EPOCHS * ((n_all + BATCH - 1) // BATCH)
    assert kl.value != cfg.init_kl_coef
