"""configs[3] (UL2-20B rl_ul2 shape) in the GPU suite.

* Per-GPU C4 workload, 128 rollouts x 128 decoder tokens x V 32128, bf16 logits: one
  PPOHotPath.step against the oracle run in fp32 on the same bf16-quantised inputs at FULL
  size (ppo_orchestrator.py:154-167, ppo_models.py:121-199, modeling.py:37-41 at T = 128:
  two 64-token GAE chunks per rollout).  dlogits are compared on a strided subset of rows
  (every 16th rollout) to keep the host comparison short; every other output in full.
* The 1024-rollout strong-scaling shape (C4 on one GPU), where the loss rows
  write 4.2 GB of dlogits and store_policy_for() selects `sc1` stores: property checks —
  finite, deterministic (two steps bit-identical), every dlogits row sums to ~0
  (g * (1 - sum softmax)), the store policy does not change a bit (sc1 vs nt), and lp /
  ref_lp of sampled rows equal the oracle's.
Tolerances as SURVEY §8c: fp32-accumulated outputs rtol 1e-5 vs the fp32 oracle on the
bf16 inputs; dlogits (bf16 output) rtol 2e-2.
"""
import pytest
import torch

import trlx_t5_amd as P
from trlx_t5_amd import _lib
from oracle import ppo_oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _inputs(B, T, V, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    logits = torch.randn(B, T, V, generator=g, device=DEV).to(torch.bfloat16)
    ref_logits = (logits.float() + 0.1 * torch.randn(B, T, V, generator=g, device=DEV)).to(torch.bfloat16)
    new_logits = (logits.float() + 0.05 * torch.randn(B, T, V, generator=g, device=DEV)).to(torch.bfloat16)
    labels = torch.randint(0, V, (B, T), generator=g, device=DEV)
    labels[0, 0], labels[-1, -1] = 0, V - 1
    old_values = torch.randn(B, T, generator=g, device=DEV)
    values = old_values + 0.3 * torch.randn(B, T, generator=g, device=DEV)
    scores = torch.rand(B, generator=g, device=DEV) * 24 - 12
    return logits, ref_logits, new_logits, labels, old_values, values, scores


def test_c4_per_gpu_step_vs_oracle():
    B, T, V = 128, 128, 32128
    x = _inputs(B, T, V, 4)
    hp = P.PPOHotPath(P.PPOConfig(), B, T, V, torch.bfloat16, DEV, kl_coef=0.05)
    loss, stats, dl, dv = hp.step(*x)
    torch.cuda.synchronize()
    c = [t.cpu() for t in x]
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    ref = orc.ppo_step_reference(c[0].float(), c[1].float(), c[2].float(), c[3], c[4], c[5], c[6], kl_coef=0.05)
    rt = dict(rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(hp.lp_old.cpu(), ref["lp"], **rt)
    torch.testing.assert_close(hp.ref_lp.cpu(), ref["ref_lp"], **rt)
    torch.testing.assert_close(hp.rewards.cpu(), ref["rewards"], **rt)
    torch.testing.assert_close(hp.returns.cpu(), ref["returns"], rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(hp.lp_new.cpu(), ref["new_lp"], **rt)
    torch.testing.assert_close(loss.cpu().reshape(()), ref["loss"], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dv.cpu(), ref["dvalues"], rtol=1e-5, atol=1e-9)
    st = stats.cpu().tolist()
    for i, k in enumerate(P.STATS_KEYS):
        assert st[i] == pytest.approx(float(ref["stats"][k]), rel=1e-4, abs=1e-6), k
    rows = slice(0, B, 16)
    torch.testing.assert_close(dl[rows].float().cpu(), ref["dlogits"][rows], rtol=2e-2, atol=1e-9)
    assert int(hp.adv_stats[2]) == B * T


def test_c4_strong_scaling_shape_properties():
    B, T, V = 1024, 128, 32128
    x = _inputs(B, T, V, 41)
    outs = []
    for pol in (0, 5):  # 0 = auto (sc1 stores at 4.2 GB per launch), 5 = nt forced
        _lib.set_tuning("store_policy", pol)
        try:
            hp = P.PPOHotPath(P.PPOConfig(), B, T, V, torch.bfloat16, DEV, kl_coef=0.05)
            for rep in range(2 if pol == 0 else 1):
                loss, stats, dl, dv = hp.step(*x)
                torch.cuda.synchronize()
                outs.append((loss.clone(), stats.clone(), dv.clone(), hp.lp_old.clone(), hp.lp_new.clone(),
                             dl.view(-1, V)[::97].clone(), torch.isfinite(dl).all().item(),
                             dl.float().sum(-1).abs().max().item()))
        finally:
            _lib.set_tuning("store_policy", 0)
    base = outs[0]
    assert base[6], "non-finite dlogits"
    assert base[7] < 1e-3, base[7]  # each row: g * (onehot - softmax) sums to ~0 (bf16 rounding of V terms)
    assert bool(torch.isfinite(base[0]).all()) and bool(torch.isfinite(base[1]).all())
    for o in outs[1:]:  # repeat and the other store policy: bit-identical
        for a, b in zip(base[:6], o[:6]):
            assert torch.equal(a, b)
    # sampled rows against the oracle (per-row quantities: exact inputs, no batch coupling)
    rows = torch.tensor([0, 1, 333, 777, 1023])
    c = [t[rows].cpu() for t in x[:4]]
    torch.testing.assert_close(base[3][rows].cpu(), orc.logprobs_from_logits(c[0].float(), c[3]),
                               rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(base[4][rows].cpu(), orc.logprobs_from_logits(c[2].float(), c[3]),
                               rtol=1e-5, atol=1e-5)
