"""§8f-2 under the data-parallel schedule (VERDICT r04 "Next round" 2): the PPO update from
hidden states with the batch sharded over ranks (accelerate_ppo_model.py:88-126 under the DDP
sharding of :146-148; whitening statistics global, modeling.py:13-20), several processes
sharing cuda:0 over gloo (the RCCL run at N > 1 is the driver's).

  * pipeline_step_from_hidden (the loss side of batch k derives its whitening coefficients
    from the all-reduced split record while the lm_head experience of batch k+1 runs) is
    bit-identical to step_from_hidden on a split_beta=True hot path, batch by batch;
  * both agree with the oracle on the CONCATENATED batch: fp32 lm_head logits of the same
    bf16 operands, reference logprobs / KL rewards / GAE, global whitening (biased moments),
    the masked PPO loss with the global normaliser (loss_norm="global"), autograd into the
    hidden states, the lm_head weight and the values — each rank's dh / dvalues are its rows of
    W·(global gradient), the DDP average of the ranks' dW is the global dW.
"""
import os

import numpy as np
import pytest
import torch

from oracle import ppo_oracle as orc

pytestmark = pytest.mark.gpu


def _inputs(B, T, V, H, seed, ragged):
    g = torch.Generator().manual_seed(seed)
    h = torch.randn(B, T, H, generator=g).to(torch.bfloat16)
    w = (torch.randn(V, H, generator=g) * 0.05).to(torch.bfloat16)
    ref_h = (h.float() + 0.1 * torch.randn(B, T, H, generator=g)).to(torch.bfloat16)
    new_h = (h.float() + 0.05 * torch.randn(B, T, H, generator=g)).to(torch.bfloat16)
    labels = torch.randint(0, V, (B, T), generator=g)
    old_values = torch.randn(B, T, generator=g)
    values = old_values + 0.3 * torch.randn(B, T, generator=g)
    scores = torch.rand(B, generator=g) * 24 - 12
    L = mask = None
    if ragged:  # C3's decoder lengths: ragged per rollout, unequal Σmask per rank
        L = torch.randint(1, T + 1, (B,), generator=g)
        L[0] = T
        mask = (torch.arange(T)[None, :] < L[:, None]).long()
        old_values = old_values.masked_fill(mask == 0, 0)
    return dict(h=h, w=w, ref_h=ref_h, new_h=new_h, labels=labels, old_values=old_values, values=values,
                scores=scores, lengths=L, mask=mask)


def _oracle(x, world):
    """The reference loss side on the concatenated batch (fp32, CPU): global whitening, global
    Σmask normaliser.  Returns rewards, returns, loss, dh·world, dW, dvalues·world."""
    B, T, H = x["h"].shape
    wf = x["w"].float()
    lp = orc.store_padded(orc.logprobs_from_logits(x["h"].float() @ wf.t(), x["labels"]), x["lengths"])
    ref_lp = orc.store_padded(orc.logprobs_from_logits(x["ref_h"].float() @ wf.t(), x["labels"]), x["lengths"])
    rewards = orc.kl_penalty_rewards(lp, ref_lp, 0.05, x["scores"], x["lengths"])
    adv, ret = orc.gae(x["old_values"], rewards, T, 1.0, 0.95, use_whitening=False)
    mu = adv.double().mean()
    var = ((adv.double() - mu) ** 2).mean()  # biased: the distributed branch of whiten
    advw = ((adv.double() - mu) * torch.rsqrt(var + 1e-8)).float()
    hg = x["new_h"].float().clone().requires_grad_(True)
    wg = wf.clone().requires_grad_(True)
    vg = x["values"].clone().requires_grad_(True)
    new_lp = orc.logprobs_from_logits(hg @ wg.t(), x["labels"])
    m = torch.ones(B, T, dtype=torch.long) if x["mask"] is None else x["mask"]
    loss, _ = orc.ppo_loss(new_lp, vg, lp, x["old_values"], advw, ret, m)
    loss.backward()
    return dict(rewards=rewards, returns=ret, loss=loss.detach(), dh=world * hg.grad, dw=wg.grad,
                dv=world * vg.grad, mask=m)


def _run(world, batches, use_ctl, timeout=300):
    import torch.multiprocessing as mp
    import dist_workers
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() + 61 * world + 7 * use_ctl) % 400
    ps = [ctx.Process(target=dist_workers.pipeline_hidden_worker,
                      args=(r, world, port, batches, q, "global", use_ctl)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=timeout) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _rel(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


@pytest.mark.parametrize("world", [2, 4])
def test_dp_from_hidden_pipelined_matches_serial_and_oracle(world):
    """World 2 and 4, ragged decoder lengths (unequal Σmask per rank), loss_norm="global",
    three batches: pipelined == serial bit for bit; both == the oracle on the concatenated
    batch (rewards / returns at rtol 1e-5, loss at 1e-4, dvalues at 1e-5; dh, dW at the fused
    loss side's bf16-operand tolerance: relative Frobenius 2e-2 of fp32, the sum of the ranks'
    dW against W·dW_global)."""
    B, T, V, H = 8, 20, 1031, 768
    batches = [_inputs(B, T, V, H, 70 + 3 * i + world, True) for i in range(3)]
    for b in batches:
        m = b["mask"]
        sums = [int(m[r * B // world:(r + 1) * B // world].sum()) for r in range(world)]
        assert len(set(sums)) > 1, "the case where rank-local and global normalisers differ"
    res = _run(world, batches, use_ctl=False)
    for i, x in enumerate(batches):
        want = _oracle(x, world)
        dw_sum = 0.0
        losses = []
        for r in range(world):
            ser, pip = res[r]["serial"][0][i], res[r]["pipelined"][0][i]
            for j, (a, b) in enumerate(zip(ser, pip)):
                assert np.array_equal(a, b, equal_nan=True), f"world {world} rank {r} batch {i} output {j}"
            loss, stats, dh, dw, dv, rew, ret = pip
            rows = slice(r * B // world, (r + 1) * B // world)
            m = want["mask"][rows].bool().numpy()
            np.testing.assert_allclose(rew, want["rewards"][rows].numpy(), rtol=1e-5, atol=1e-5)
            np.testing.assert_allclose(ret, want["returns"][rows].numpy(), rtol=1e-5, atol=2e-5)
            np.testing.assert_allclose(dv, want["dv"][rows].numpy(), rtol=1e-5, atol=1e-6)
            assert _rel(dh[m], want["dh"][rows].numpy()[m]) < 2e-2
            assert (dh[~m] == 0).all()
            dw_sum = dw_sum + dw.astype(np.float64)
            losses.append(float(loss.reshape(())))
        # DDP averages the ranks' dW: their mean is the global gradient
        assert _rel(dw_sum / world, want["dw"].numpy()) < 2e-2
        np.testing.assert_allclose(np.mean(losses), float(want["loss"]), rtol=1e-4, atol=1e-5)


def test_dp2_from_hidden_pipelined_device_state():
    """World 2 with the device controller state (beta read from and advanced in device memory
    by the loss tails; the score moments merged one batch late inside the pipeline): the
    pipelined from-hidden schedule's outputs and final controller state equal the serial ones
    bit for bit."""
    B, T, V, H = 8, 12, 517, 512
    batches = [_inputs(B, T, V, H, 90 + i, i == 1) for i in range(3)]
    for b in batches:  # one ragged batch among dense ones: the masks vary per step
        if b["mask"] is None:
            b["mask"] = torch.ones(B, T, dtype=torch.long)
    res = _run(2, batches, use_ctl=True)
    for r in range(2):
        (ser, ser_state), (pip, pip_state) = res[r]["serial"], res[r]["pipelined"]
        assert np.array_equal(ser_state, pip_state), f"rank {r} controller state"
        for i, (a, b) in enumerate(zip(ser, pip)):
            for j, (u, v) in enumerate(zip(a, b)):
                assert np.array_equal(u, v, equal_nan=True), f"rank {r} batch {i} output {j}"
