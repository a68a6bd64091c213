"""Data-parallel PPO step on the GPU with world size 2 (two processes sharing cuda:0, gloo
process group — the 8-GPU RCCL run is the driver's; this checks the sharded semantics):
every rank streams only its row block, the whitening statistics are the GLOBAL biased
moments (modeling.py:9-21 branch of whiten, one all-reduce of {Σ A, Σ A², n}), and each
rank's loss / gradients match the oracle applied to its shard with the global whitening
(loss normalisers rank-local, ppo_models.py:162,177)."""
import os

import numpy as np
import pytest
import torch

from oracle import ppo_oracle as orc

pytestmark = pytest.mark.gpu


def _inputs(B, T, V, seed, lengths):
    g = torch.Generator().manual_seed(seed)
    logits = torch.randn(B, T, V, generator=g).to(torch.bfloat16)
    ref_logits = (logits.float() + 0.1 * torch.randn(B, T, V, generator=g)).to(torch.bfloat16)
    new_logits = (logits.float() + 0.05 * torch.randn(B, T, V, generator=g)).to(torch.bfloat16)
    labels = torch.randint(0, V, (B, T), generator=g)
    old_values = torch.randn(B, T, generator=g)
    values = old_values + 0.3 * torch.randn(B, T, generator=g)
    scores = torch.rand(B, generator=g) * 24 - 12
    L = mask = None
    if lengths:
        L = torch.randint(1, T + 1, (B,), generator=g)
        mask = (torch.arange(T)[None, :] < L[:, None]).long()
        old_values = old_values.masked_fill(mask == 0, 0)
    return dict(logits=logits, ref_logits=ref_logits, new_logits=new_logits, labels=labels, old_values=old_values,
                values=values, scores=scores, lengths=L, mask=mask)


@pytest.mark.parametrize("lengths,mode", [(False, "step"), (True, "step"), (False, "pipelined"), (True, "pipelined")])
def test_dp2_step_global_whitening(lengths, mode):
    """Two ranks vs the oracle on the concatenated batch: the whitening moments all-reduced
    (modeling.py:9-21), per-rank losses / gradients on each shard.  mode "pipelined": the
    split-beta schedule (pipeline_step), its split record {Σ A0, Σ A0², n, Σ Ak, ...}."""
    import torch.multiprocessing as mp
    import dist_workers
    world, B, T, V = 2, 8, 20, 1031
    x = _inputs(B, T, V, 5 + lengths, lengths)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() + (37 if mode == "pipelined" else 0)) % 300
    ps = [ctx.Process(target=dist_workers.hot_path_step_worker, args=(r, world, port, x, q, "rank", mode))
          for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0

    # oracle: experience per row, GAE per row, whitening with the GLOBAL biased moments
    f = {k: (v.float() if v is not None and v.is_floating_point() else v) for k, v in x.items()}
    lp = orc.store_padded(orc.logprobs_from_logits(f["logits"], x["labels"]), x["lengths"])
    ref_lp = orc.store_padded(orc.logprobs_from_logits(f["ref_logits"], x["labels"]), x["lengths"])
    rewards = orc.kl_penalty_rewards(lp, ref_lp, 0.05, x["scores"], x["lengths"])
    adv, ret = orc.gae(x["old_values"], rewards, T, 1.0, 0.95, use_whitening=False)
    mu = adv.double().mean()
    var = ((adv.double() - mu) ** 2).mean()
    advw = ((adv.double() - mu) * torch.rsqrt(var + 1e-8)).float()
    for r in range(world):
        got = res[r]
        rows = slice(r * B // world, (r + 1) * B // world)
        torch.testing.assert_close(got["lp"], lp[rows], rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(got["rewards"], rewards[rows], rtol=1e-5, atol=1e-5)
        st = got["adv_stats"]
        assert float(st[2]) == B * T  # the all-reduced count covers both shards
        sum_a = st[0] - float(np.float32(0.05)) * st[3] if mode == "pipelined" else st[0]  # split: Σ A0 - beta Σ Ak
        torch.testing.assert_close(sum_a, adv.double().sum(), rtol=1e-5, atol=1e-4)
        torch.testing.assert_close(got["returns"], ret[rows], rtol=1e-5, atol=2e-5)
        xg = f["new_logits"][rows].clone().requires_grad_(True)
        vg = x["values"][rows].clone().requires_grad_(True)
        new_lp = orc.logprobs_from_logits(xg, x["labels"][rows])
        m = torch.ones(B // world, T, dtype=torch.long) if x["mask"] is None else x["mask"][rows]
        loss, _ = orc.ppo_loss(new_lp, vg, lp[rows], x["old_values"][rows], advw[rows], ret[rows], m)
        loss.backward()
        torch.testing.assert_close(got["loss"].reshape(()), loss.detach(), rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(got["dlogits"], xg.grad, rtol=2e-2, atol=1e-6)
        torch.testing.assert_close(got["dvalues"], vg.grad, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("scale", ["running", "ref"])
def test_dp2_device_state(scale):
    """Device RunningMoments across ranks: every rank merges the GLOBAL score moments (one
    all-reduce of {Σx, Σx², n}), so all ranks hold the same running statistics; ref_std is
    each rank's own first-chunk std; beta advances rank-locally from the rank's approx_kl
    (accelerate_ppo_model.py:123,130-131)."""
    import torch.multiprocessing as mp
    import dist_workers
    world, B, T, V = 2, 8, 12, 517
    x = _inputs(B, T, V, 21, False)
    g = torch.Generator().manual_seed(9)
    seq = [torch.randn(B, generator=g) * 12 + 1, torch.randn(B, generator=g) * 3 - 2]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29800 + os.getpid() % 150
    ps = [ctx.Process(target=dist_workers.ctl_step_worker, args=(r, world, port, x, seq, scale, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    f = {k: (v.float() if v is not None and v.is_floating_point() else v) for k, v in x.items()}
    lp = orc.logprobs_from_logits(f["logits"], x["labels"])
    ref_lp = orc.logprobs_from_logits(f["ref_logits"], x["labels"])
    running = orc.RunningMoments()  # single-process over the concatenated batch == the global statistics
    ref_std = [None] * world
    betas = [0.05] * world
    for i, s in enumerate(seq):
        running.update(s.clone())
        for r in range(world):
            rows = slice(r * B // world, (r + 1) * B // world)
            sr = s[rows].clone()
            if ref_std[r] is None:
                ref_std[r] = sr.std()
            sr = sr / (running.std if scale == "running" else ref_std[r])
            sr = torch.clip(sr, -10, 10)
            want = orc.kl_penalty_rewards(lp[rows], ref_lp[rows], betas[r], sr)
            got = res[r][i]
            torch.testing.assert_close(got["rewards"], want, rtol=1e-5, atol=1e-5)
            assert got["state"]["std"] == pytest.approx(float(running.std), rel=1e-5)
            assert got["state"]["count"] == pytest.approx(float(running.count), rel=1e-12)
            assert got["state"]["ref_std"] == pytest.approx(float(ref_std[r]), rel=1e-5)
            kl = orc.AdaptiveKLController(betas[r], 6, 10000)
            kl.update(got["approx_kl"], n_steps=B // world)
            betas[r] = kl.value
            assert got["state"]["kl_coef"] == betas[r]


def test_dp2_step_global_loss_norm():
    """loss_norm="global" with ragged decoder lengths (unequal Σmask per rank): Σmask rides
    the whitening all-reduce and each rank normalises by Σmask_global / W, so the DDP average
    of the per-rank gradients is the gradient of the masked PPO loss over the CONCATENATED
    batch (the oracle on all rows at once), and the mean of the per-rank losses is that loss
    (SURVEY §8e global-normaliser mode; "rank" stays the reference default)."""
    import torch.multiprocessing as mp
    import dist_workers
    world, B, T, V = 2, 8, 20, 1031
    x = _inputs(B, T, V, 17, True)
    m = x["mask"]
    assert m[: B // 2].sum() != m[B // 2:].sum()  # the case where the two modes differ
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() + 150) % 300
    ps = [ctx.Process(target=dist_workers.hot_path_step_worker, args=(r, world, port, x, q, "global"))
          for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0

    f = {k: (v.float() if v is not None and v.is_floating_point() else v) for k, v in x.items()}
    lp = orc.store_padded(orc.logprobs_from_logits(f["logits"], x["labels"]), x["lengths"])
    ref_lp = orc.store_padded(orc.logprobs_from_logits(f["ref_logits"], x["labels"]), x["lengths"])
    rewards = orc.kl_penalty_rewards(lp, ref_lp, 0.05, x["scores"], x["lengths"])
    adv, ret = orc.gae(x["old_values"], rewards, T, 1.0, 0.95, use_whitening=False)
    mu = adv.double().mean()
    var = ((adv.double() - mu) ** 2).mean()
    advw = ((adv.double() - mu) * torch.rsqrt(var + 1e-8)).float()
    xg = f["new_logits"].clone().requires_grad_(True)
    vg = x["values"].clone().requires_grad_(True)
    new_lp = orc.logprobs_from_logits(xg, x["labels"])
    loss, _ = orc.ppo_loss(new_lp, vg, lp, x["old_values"], advw, ret, m)
    loss.backward()
    for r in range(world):
        got = res[r]
        rows = slice(r * B // world, (r + 1) * B // world)
        assert float(got["adv_stats"][3]) == float(m.sum()) / world
        torch.testing.assert_close(got["dlogits"], world * xg.grad[rows], rtol=2e-2, atol=1e-6)
        torch.testing.assert_close(got["dvalues"], world * vg.grad[rows], rtol=1e-5, atol=1e-6)
    mean_loss = sum(res[r]["loss"].reshape(()) for r in range(world)) / world
    torch.testing.assert_close(mean_loss, loss.detach(), rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("use_ctl,overlap,lengths,loss_norm,scale", [
    (True, True, False, "rank", "running"), (False, False, True, "rank", "running"),
    (True, False, True, "global", "running"), (True, False, False, "rank", False), (True, False, True, "rank", "ref")])
def test_dp2_pipelined_schedule_matches_serial(use_ctl, overlap, lengths, loss_norm, scale):
    """PPOHotPath.pipeline_step (the DP schedule that hides the whitening all-reduce behind
    the next batch's experience rows; split-beta GAE) against step(split_beta=True) over three
    batches at world 2: losses, stats, gradients, rewards, returns and the device controller
    state bit-identical per batch; against the unsplit step() equal up to fp32 association.
    With loss_norm="global" the Σmask of the split record rides the all-reduce (slot 6).
    scale False / "ref": RunningMoments merges each batch's score moments one batch late
    inside the pipeline (lag), the final controller state equals the serial one."""
    import torch.multiprocessing as mp
    import dist_workers
    world, B, T, V = 2, 8, 21, 1031
    batches = [_inputs(B, T, V, 40 + i, lengths) for i in range(3)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() + 151) % 300
    ps = [ctx.Process(target=dist_workers.pipeline_worker, args=(r, world, port, batches, q, use_ctl, overlap,
                                                                 loss_norm, scale)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        (ser, ser_state), (pip, pip_state) = res[r]["serial"], res[r]["pipelined"]
        uns, uns_state = res[r]["unsplit"]
        assert len(ser) == len(pip) == len(uns) == len(batches)
        if use_ctl:
            assert np.array_equal(ser_state, pip_state), f"rank {r} controller state"
            np.testing.assert_allclose(uns_state, ser_state, rtol=1e-5)
        for i, (a, b, c) in enumerate(zip(ser, pip, uns)):
            for j, (x, y, z) in enumerate(zip(a, b, c)):
                assert np.array_equal(x, y, equal_nan=True), f"rank {r} batch {i} output {j}"
                # split beta vs the unsplit kernels: fp32 association only (dlogits: bf16)
                np.testing.assert_allclose(z, x, rtol=2e-2 if j == 2 else 1e-4, atol=1e-5,
                                           err_msg=f"rank {r} batch {i} output {j}")
