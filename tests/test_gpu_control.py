"""GPU parity of the device-resident controller state, through the C ABI:
RunningMoments.update (modeling.py:72-104), the orchestrator's ref stats + score scale /
clip (ppo_orchestrator.py:48-49,96-112) and Adaptive/FixedKLController.update
(ppo_models.py:26-58), standalone and folded into PPOHotPath's rollout tails.

Oracles: the reference's own KAT (tests/test_ppo.py:49-66, via tests/golden/host_state.npz),
the golden KL-controller trajectory, and oracle.ScoreControl / AdaptiveKLController (the
reference's code restated, fp32 tensors as the reference runs it).  Tolerances: the device
state is fp64, the reference's running statistics are fp32 tensors -> rel 1e-5 on the
statistics; the KL coefficient is fp64 in both -> bit-exact when fed the same fp32
approx_kl.
"""
import os

import numpy as np
import pytest
import torch

import trlx_t5_amd as P
from trlx_t5_amd import _lib
from golden_util import T
from oracle import ppo_oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
RT32 = dict(rtol=1e-5, atol=1e-5)


def cuda(t):
    return t.to(DEV)


def test_ctl_init_layout():
    c = P.PPOControlState(DEV, init_kl_coef=0.05, ref_mean=1.5, ref_std=2.5)
    h = c.host()
    assert (h["mean"], h["var"], h["std"], h["count"]) == (0.0, 1.0, 1.0, 1e-24)  # RunningMoments.__init__
    assert (h["ref_mean"], h["ref_std"], h["ref_set"], h["kl_coef"]) == (1.5, 2.5, 1.0, 0.05)
    assert c.buf.shape == (2, _lib.CTL_SLOTS)
    c2 = P.PPOControlState(DEV)
    assert c2.host()["ref_set"] == 0.0 and np.isnan(c2.host()["ref_std"])


def test_running_moments_kat_device_state(golden):
    """The reference KAT sequence through the device state (no host merge)."""
    z = golden("host_state")
    c = P.PPOControlState(DEV, scale_reward=False, cliprange_reward=None)
    for i in range(4):
        a = T(z[f"rm/{i}/in"]).float()
        out, bm, bs = c.prepare_scores(cuda(a))
        assert torch.equal(out.cpu(), a)  # no scale, no clip: scores pass through
        assert float(bm) == pytest.approx(float(z[f"rm/{i}/batch_mean"]), rel=1e-6, abs=1e-6)
        assert float(bs) == pytest.approx(float(z[f"rm/{i}/batch_std"]), rel=1e-6)
        h = c.host()
        assert h["mean"] == pytest.approx(float(z[f"rm/{i}/mean"]), rel=1e-6, abs=1e-6)
        assert h["std"] == pytest.approx(float(z[f"rm/{i}/std"]), rel=1e-6)
        assert h["var"] == pytest.approx(float(z[f"rm/{i}/var"]), rel=1e-6)
        assert h["count"] == pytest.approx(float(z[f"rm/{i}/count"]), rel=1e-12)


@pytest.mark.parametrize("scale", [False, "running", "ref"])
@pytest.mark.parametrize("clip", [10, None])
@pytest.mark.parametrize("preset_ref", [False, True])
def test_prepare_scores_vs_oracle(scale, clip, preset_ref):
    g = torch.Generator().manual_seed(3)
    ref_mean, ref_std = (0.5, 3.0) if preset_ref else (None, None)
    oc = orc.ScoreControl(scale, clip, ref_mean, ref_std)
    c = P.PPOControlState(DEV, scale_reward=scale, cliprange_reward=clip, ref_mean=ref_mean, ref_std=ref_std)
    for step, n in enumerate([128, 37, 1000, 2, 513]):
        s = torch.randn(n, generator=g) * (4 + 10 * step) + step
        want, wm, ws = oc(s)
        got, gm, gs = c.prepare_scores(cuda(s))
        torch.testing.assert_close(got.cpu(), want, rtol=1e-5, atol=1e-5, msg=f"step {step}")
        assert float(gm) == pytest.approx(float(wm), rel=1e-5, abs=1e-6)
        assert float(gs) == pytest.approx(float(ws), rel=1e-5)
        h = c.host()
        assert h["mean"] == pytest.approx(float(oc.running.mean), rel=1e-5, abs=1e-6)
        assert h["std"] == pytest.approx(float(oc.running.std), rel=1e-5)
        assert h["ref_std"] == pytest.approx(float(oc.ref_std), rel=1e-5)
        assert h["ref_mean"] == pytest.approx(float(oc.ref_mean), rel=1e-5, abs=1e-6)
        if clip:
            assert got.abs().max().item() <= clip


def test_prepare_scores_single_score_edge():
    """B = 1: unbiased batch std is NaN, the running std divides by (tot - 1) = 0 -> inf
    (the reference does the same in fp32: tot_count = 1e-24 + 1 == 1.0)."""
    oc = orc.ScoreControl("running", 10)
    c = P.PPOControlState(DEV, scale_reward="running", cliprange_reward=10)
    s = torch.tensor([3.0])
    want, _, ws = oc(s)
    got, _, gs = c.prepare_scores(cuda(s))
    assert np.isnan(float(gs)) and np.isnan(float(ws))
    assert np.isinf(c.host()["std"]) and np.isinf(float(oc.running.std))
    torch.testing.assert_close(got.cpu(), want, equal_nan=True)


def test_kl_controller_golden_and_exact():
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "host_state.npz"))
    c = P.PPOControlState(DEV, init_kl_coef=0.05, target=6, horizon=10000, n_steps=12)
    oc = orc.AdaptiveKLController(0.05, 6, 10000)
    for cur, want in zip(z["kl/currents"], z["kl/values"]):
        k32 = torch.tensor([float(cur)], dtype=torch.float32)
        c.kl_update(cuda(k32))
        oc.update(float(k32), n_steps=12)  # the reference sees approx_kl as a float of an fp32 tensor
        beta = c.host()["kl_coef"]
        assert beta == oc.value  # fp64 in both, same operation order: bit-exact
        assert beta == pytest.approx(float(want), rel=1e-6)  # golden trajectory (fp64 currents)
    assert c.host()["kl_updates"] == len(z["kl/currents"])
    f = P.PPOControlState(DEV, init_kl_coef=0.05, target=None)
    f.kl_update(cuda(torch.tensor([3.0])))
    assert f.host()["kl_coef"] == float(z["kl/fixed"])  # FixedKLController
    nan = P.PPOControlState(DEV, init_kl_coef=0.05, target=6)
    nan.kl_update(cuda(torch.tensor([float("nan")])))
    assert np.isnan(nan.host()["kl_coef"])  # np.clip propagates NaN


def _step_inputs(B, Tn, V, seed):
    g = torch.Generator().manual_seed(seed)
    logits = torch.randn(B, Tn, V, generator=g).to(torch.bfloat16)
    ref_logits = (logits.float() + 0.1 * torch.randn(B, Tn, V, generator=g)).to(torch.bfloat16)
    new_logits = (logits.float() + 0.05 * torch.randn(B, Tn, V, generator=g)).to(torch.bfloat16)
    labels = torch.randint(0, V, (B, Tn), generator=g)
    old_values = torch.randn(B, Tn, generator=g)
    values = old_values + 0.3 * torch.randn(B, Tn, generator=g)
    return logits, ref_logits, new_logits, labels, old_values, values


@pytest.mark.parametrize("scale,target", [("running", 6), ("ref", 6), (False, None), (False, 0.001)])
def test_hot_path_with_device_state_vs_oracle(scale, target):
    """Three PPO steps with the state folded into the rollout tails: scores pass through
    RunningMoments + scale + clip inside the GAE tail, beta is read from the state and
    advanced by kl_ctl.update(approx_kl) in the loss tail — vs the orchestrator + loss +
    controller restated on CPU.  (target 0.001 drives the proportional error to +0.2.)"""
    B, Tn, V = 8, 17, 1031
    cfg = P.PPOConfig(target=target, scale_reward=scale, cliprange_reward=10)
    c = P.PPOControlState.from_config(cfg, DEV, n_steps=B)
    hp = P.PPOHotPath(cfg, B, Tn, V, torch.bfloat16, DEV, kl_coef=123.0, ctl=c)  # kl_coef ignored with ctl
    oc = orc.ScoreControl(scale, 10)
    okl = orc.AdaptiveKLController(0.05, target, 10000) if target else orc.FixedKLController(0.05)
    g = torch.Generator().manual_seed(11)
    for step in range(3):
        logits, ref_logits, new_logits, labels, old_values, values = _step_inputs(B, Tn, V, 40 + step)
        scores = torch.randn(B, generator=g) * 15
        beta = okl.value
        loss, stats, _, _ = hp.step(cuda(logits), cuda(ref_logits), cuda(new_logits), cuda(labels),
                                    cuda(old_values), cuda(values), cuda(scores))
        torch.cuda.synchronize()
        s_t, _, _ = oc(scores)
        ref = orc.ppo_step_reference(logits.float(), ref_logits.float(), new_logits.float(), labels, old_values,
                                     values, s_t, kl_coef=beta)
        torch.testing.assert_close(hp.rewards.cpu(), ref["rewards"], **RT32, msg=f"step {step}")
        torch.testing.assert_close(loss.cpu().reshape(()), ref["loss"], rtol=1e-5, atol=1e-6)
        kl_dev = float(stats[8])
        assert kl_dev == pytest.approx(float(ref["stats"]["policy/approx_kl"]), rel=1e-4, abs=1e-7)
        okl.update(kl_dev, n_steps=B)  # the same fp32 approx_kl the device consumed
        h = c.host()
        assert h["kl_coef"] == okl.value, f"step {step}"
        assert h["std"] == pytest.approx(float(oc.running.std), rel=1e-5)
        assert h["last_kl"] == kl_dev
    assert c.cur in (0, 1) and int(hp.workspace.view(torch.int32)[:4].abs().sum()) == 0


def test_hot_path_device_state_needs_no_host_sync():
    """The step with device state issues no device->host copy: it can be captured in a HIP
    graph (capture fails on any synchronising call) and replayed."""
    B, Tn, V = 4, 9, 257
    cfg = P.PPOConfig(scale_reward="running")
    c = P.PPOControlState.from_config(cfg, DEV, n_steps=B)
    hp = P.PPOHotPath(cfg, B, Tn, V, torch.bfloat16, DEV, kl_coef=0.0, ctl=c)
    logits, ref_logits, new_logits, labels, old_values, values = [cuda(t) for t in _step_inputs(B, Tn, V, 5)]
    scores = cuda(torch.linspace(-20, 20, B))
    args = (logits, ref_logits, new_logits, labels, old_values, values, scores)
    hp.step(*args)  # warm-up (allocates dlogits)
    torch.cuda.synchronize()
    c.cur = 0
    side = torch.cuda.Stream(DEV)
    side.wait_stream(torch.cuda.current_stream(DEV))
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(graph, stream=side):
            hp.step(*args)
            hp.step(*args)  # two steps: the double-buffered state returns to buf[0]
    torch.cuda.synchronize()
    assert c.cur == 0
    before = c.host()
    graph.replay()
    torch.cuda.synchronize()
    after = c.host()
    assert after["count"] == pytest.approx(before["count"] + 2 * B)
    assert after["kl_updates"] == before["kl_updates"] + 2


@pytest.mark.parametrize("mode", ["overlap", "defer"])
def test_overlapped_loss_tail_matches_serial(mode):
    """overlap_tail=True (the loss tail on a side stream beside the next step's experience
    rows) and defer_tail=True (the loss tail folded into the next step's experience rows
    launch) give bit-identical losses, stats, gradients and controller state over several
    steps.  No wait between steps: the tail of step k really runs beside / inside step
    k+1's experience rows; the host waits once (wait_stats) before reading the last stats."""
    B, Tn, V = 16, 33, 3001
    outs = {}
    for overlap in (False, True):
        cfg = P.PPOConfig(scale_reward="running")
        c = P.PPOControlState.from_config(cfg, DEV, n_steps=B)
        kw = {"overlap_tail" if mode == "overlap" else "defer_tail": overlap}
        hp = P.PPOHotPath(cfg, B, Tn, V, torch.bfloat16, DEV, kl_coef=0.0, ctl=c, **kw)
        g = torch.Generator().manual_seed(2)
        inputs = [[cuda(t) for t in _step_inputs(B, Tn, V, step)] + [cuda(torch.randn(B, generator=g) * 9)]
                  for step in range(4)]
        torch.cuda.synchronize()
        grads = []
        for x in inputs:
            loss, stats, dl, dv = hp.step(*x)
            grads.append((dl.clone(), dv.clone()))  # main-stream outputs: ordered with the clone
        hp.wait_stats()
        outs[overlap] = (grads, loss.clone(), stats.clone(), c.state.clone())
        torch.cuda.synchronize()
    (ga, la, sa, ca), (gb, lb, sb, cb) = outs[False], outs[True]
    for (x0, y0), (x1, y1) in zip(ga, gb):
        assert torch.equal(x0, x1) and torch.equal(y0, y1)
    assert torch.equal(la, lb) and torch.equal(sa, sb) and torch.equal(ca, cb)


@pytest.mark.parametrize("mode", ["overlap", "defer"])
def test_overlapped_tail_several_losses_per_experience(mode):
    """The ppo_epochs pattern (accelerate_base_model.py:254): one experience, then several
    policy_loss calls on it.  With overlap_tail each policy_loss must wait for the previous
    loss tail (it rewrites the token records that tail reads): losses, stats and controller
    state equal the serial schedule bit for bit."""
    B, Tn, V = 12, 40, 2053
    res = {}
    for overlap in (False, True):
        cfg = P.PPOConfig()
        c = P.PPOControlState.from_config(cfg, DEV, n_steps=B)
        kw = {"overlap_tail" if mode == "overlap" else "defer_tail": overlap}
        hp = P.PPOHotPath(cfg, B, Tn, V, torch.bfloat16, DEV, kl_coef=0.05, ctl=c, **kw)
        logits, ref_logits, _, labels, old_values, values = [cuda(t) for t in _step_inputs(B, Tn, V, 31)]
        news = [cuda(_step_inputs(B, Tn, V, 40 + e)[2]) for e in range(4)]
        scores = cuda(torch.linspace(-12, 12, B))
        hp.experience(logits, ref_logits, labels, old_values, scores)
        rec = []
        for e in range(4):  # no host-side wait between the updates
            loss, stats, dl, dv = hp.policy_loss(news[e], labels, values, old_values)
            rec.append((dl.clone(), dv.clone()))
        hp.wait_stats()
        # every tail advanced beta from its own approx_kl: the state carries all four
        res[overlap] = (rec, loss.clone(), stats.clone(), c.state.clone(), c.host()["kl_updates"])
        torch.cuda.synchronize()
    for a, b in zip(res[False][0], res[True][0]):
        for x, y in zip(a, b):
            assert torch.equal(x, y)
    for x, y in zip(res[False][1:4], res[True][1:4]):
        assert torch.equal(x, y)
    assert res[True][4] == res[False][4]


def test_hot_path_converts_mask_and_label_dtypes():
    """bool / int32 masks and int32 labels / lengths are converted to the int64 the kernels
    read (not reinterpreted): the results equal the int64 inputs' bit for bit.  Float masks,
    wrong shapes and fp64 scores are rejected."""
    B, Tn, V = 6, 17, 509
    g = torch.Generator().manual_seed(5)
    logits, ref_logits, new_logits, labels, old_values, values = [cuda(t) for t in _step_inputs(B, Tn, V, 8)]
    L = torch.randint(1, Tn + 1, (B,), generator=g)
    mask = (torch.arange(Tn)[None, :] < L[:, None]).long()
    old_values = old_values.masked_fill(cuda(mask) == 0, 0)
    scores = cuda(torch.randn(B, generator=g))
    outs = []
    for mdt, idt in ((torch.int64, torch.int64), (torch.bool, torch.int32), (torch.int32, torch.int32)):
        hp = P.PPOHotPath(P.PPOConfig(), B, Tn, V, torch.bfloat16, DEV, kl_coef=0.05)
        loss, stats, dl, dv = hp.step(logits, ref_logits, new_logits, labels.to(idt), old_values, values, scores,
                                      lengths=cuda(L).to(idt), mask=cuda(mask).to(mdt))
        outs.append((loss.clone(), stats.clone(), dl.clone(), dv.clone(), hp.rewards.clone()))
    torch.cuda.synchronize()
    for o in outs[1:]:
        for x, y in zip(outs[0], o):
            assert torch.equal(x, y)
    hp = P.PPOHotPath(P.PPOConfig(), B, Tn, V, torch.bfloat16, DEV, kl_coef=0.05)
    with pytest.raises(ValueError):
        hp.step(logits, ref_logits, new_logits, labels, old_values, values, scores, mask=cuda(mask).float())
    with pytest.raises(ValueError):
        hp.step(logits, ref_logits, new_logits, labels[:, :-1], old_values, values, scores)
    with pytest.raises(ValueError):
        hp.step(logits, ref_logits, new_logits, labels, old_values, values, scores.double())


def test_hot_path_device_state_with_decoder_lengths():
    """C3-style decoder-length masks with the device state: the transformed score lands on
    column L_b - 1, padding stays zero, the loss normalisers use the mask."""
    B, Tn, V = 10, 21, 777
    g = torch.Generator().manual_seed(13)
    logits, ref_logits, new_logits, labels, old_values, values = _step_inputs(B, Tn, V, 77)
    L = torch.randint(1, Tn + 1, (B,), generator=g)
    L[0] = Tn
    mask = (torch.arange(Tn)[None, :] < L[:, None]).long()
    old_values = old_values.masked_fill(mask == 0, 0)
    cfg = P.PPOConfig(scale_reward="running", cliprange_reward=3)
    c = P.PPOControlState.from_config(cfg, DEV, n_steps=B)
    hp = P.PPOHotPath(cfg, B, Tn, V, torch.bfloat16, DEV, kl_coef=0.0, ctl=c)
    oc = orc.ScoreControl("running", 3)
    okl = orc.AdaptiveKLController(0.05, 6, 10000)
    for step in range(2):
        scores = torch.randn(B, generator=g) * 8
        beta = okl.value
        loss, stats, _, _ = hp.step(cuda(logits), cuda(ref_logits), cuda(new_logits), cuda(labels), cuda(old_values),
                                    cuda(values), cuda(scores), lengths=cuda(L), mask=cuda(mask))
        torch.cuda.synchronize()
        s_t, _, _ = oc(scores)
        ref = orc.ppo_step_reference(logits.float(), ref_logits.float(), new_logits.float(), labels, old_values,
                                     values, s_t, kl_coef=beta, lengths=L, mask=mask)
        torch.testing.assert_close(hp.rewards.cpu(), ref["rewards"], **RT32)
        assert torch.all(hp.rewards.cpu()[mask == 0] == 0)
        torch.testing.assert_close(loss.cpu().reshape(()), ref["loss"], rtol=1e-5, atol=1e-6)
        okl.update(float(stats[8]), n_steps=B)
        assert c.host()["kl_coef"] == okl.value


def test_c1_randomwalks_config_vs_oracle():
    """configs[0], the reference's CPU-runnable case (examples/randomwalks/configs/
    ppo_randomwalks.yml): 128 rollouts x 9 response tokens, V 23, fp32 logits, vf_coef 1.2,
    cliprange_reward 1, adaptive KL (target 6, horizon 10000, n_steps = batch_size 100).
    Four steps of the fused hot path with device state vs the restated orchestrator + loss +
    controller."""
    B, Tn, V = 128, 9, 23
    cfg = P.PPOConfig(init_kl_coef=0.05, target=6, horizon=10000, gamma=1, lam=0.95, cliprange=0.2,
                      cliprange_value=0.2, vf_coef=1.2, scale_reward=False, cliprange_reward=1)
    c = P.PPOControlState.from_config(cfg, DEV, n_steps=100)
    hp = P.PPOHotPath(cfg, B, Tn, V, torch.float32, DEV, kl_coef=0.05, ctl=c)
    oc = orc.ScoreControl(False, 1)
    okl = orc.AdaptiveKLController(0.05, 6, 10000)
    g = torch.Generator().manual_seed(23)
    for step in range(4):
        logits, ref_logits, new_logits, labels, old_values, values = _step_inputs(B, Tn, V, 90 + step)
        logits, ref_logits, new_logits = (t.float() * 2 for t in (logits, ref_logits, new_logits))
        scores = torch.rand(B, generator=g) * 4 - 2  # beyond the +-1 clip on both sides
        beta = okl.value
        loss, stats, dl, dv = hp.step(cuda(logits), cuda(ref_logits), cuda(new_logits), cuda(labels),
                                      cuda(old_values), cuda(values), cuda(scores))
        torch.cuda.synchronize()
        s_t, _, _ = oc(scores)
        ref = orc.ppo_step_reference(logits, ref_logits, new_logits, labels, old_values, values, s_t,
                                     cfg_kwargs=dict(vf_coef=1.2), kl_coef=beta)
        torch.testing.assert_close(hp.lp_old.cpu(), ref["lp"], **RT32)
        torch.testing.assert_close(hp.rewards.cpu(), ref["rewards"], **RT32, msg=f"step {step}")
        torch.testing.assert_close(hp.returns.cpu(), ref["returns"], **RT32)
        torch.testing.assert_close(loss.cpu().reshape(()), ref["loss"], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(dl.cpu(), ref["dlogits"], rtol=1e-5, atol=1e-8)
        torch.testing.assert_close(dv.cpu(), ref["dvalues"], rtol=1e-5, atol=1e-9)
        st = stats.cpu().tolist()
        for i, k in enumerate(P.STATS_KEYS):
            assert st[i] == pytest.approx(float(ref["stats"][k]), rel=1e-5, abs=1e-6), k
        okl.update(st[8], n_steps=100)
        h = c.host()
        assert h["kl_coef"] == okl.value, f"step {step}"
        assert h["mean"] == pytest.approx(float(oc.running.mean), rel=1e-5, abs=1e-7)
        assert h["count"] == pytest.approx(float(oc.running.count))


@pytest.mark.parametrize("dtype,V", [(torch.bfloat16, 50257), (torch.float32, 50257), (torch.bfloat16, 1031)])
def test_deferred_tail_fold_every_rows_kernel(dtype, V):
    """defer_tail folds the loss tail into the experience rows launch where the rows kernel
    can host it (register-resident rows: bf16 V = 50257 and 1031) and runs it as its own
    launch first where it cannot (fp32 V = 50257 takes the streaming forward): three steps,
    bit-identical to the undeferred path, including the KL-controller state."""
    B, Tn = 6, 11
    res = []
    for defer in (False, True):
        cfg = P.PPOConfig()
        c = P.PPOControlState.from_config(cfg, DEV, n_steps=B)
        hp = P.PPOHotPath(cfg, B, Tn, V, dtype, DEV, kl_coef=0.05, ctl=c, defer_tail=defer)
        rec = []
        for step in range(3):
            logits, ref_logits, new_logits, labels, old_values, values = [cuda(t) for t in
                                                                          _step_inputs(B, Tn, V, 60 + step)]
            logits, ref_logits, new_logits = (t.to(dtype) for t in (logits, ref_logits, new_logits))
            scores = cuda(torch.linspace(-3, 3, B))
            loss, stats, dl, dv = hp.step(logits, ref_logits, new_logits, labels, old_values, values, scores)
            rec.append((hp.rewards.clone(), dl.clone(), dv.clone()))
        hp.wait_stats()
        torch.cuda.synchronize()
        res.append((rec, loss.clone(), stats.clone(), c.state.clone()))
    for a, b in zip(res[0][0], res[1][0]):
        for x, y in zip(a, b):
            assert torch.equal(x, y)
    for x, y in zip(res[0][1:], res[1][1:]):
        assert torch.equal(x, y)
