"""The RCCL path itself ("nccl" backend of torch.distributed on ROCm), at world size 1 on the
one GPU of the dev box — RCCL cannot put two ranks on one device, so N > 1 runs only on the
driver's 8-GPU node; this pins everything short of the wire:
  * ProcessGroupNCCL initialised with device_id before any tensor is made (bench.py's order);
  * PPOHotPath.step (blocking whitening all-reduce; split_beta=True, the kernels the pipeline
    uses) and pipeline_step (async all-reduce, the loss side waiting on RCCL's stream) give
    bit-identical losses, stats, gradients, whitening record and controller state over three
    batches, and the unsplit step() the same numbers up to fp32 association;
  * the same two schedules through the boundary's RCCL helper (comm.RcclComm: ncclAllReduce
    enqueued on the step's stream / a side stream joined by fence-free events) are
    bit-identical to the torch.distributed ones;
  * with the group initialised, whitening takes the reference's distributed branch (biased
    variance, modeling.py:9-21): get_global_statistics / whiten match the reference's own
    gloo world-1 fixtures (tests/golden/whiten.npz dist1) through RCCL.
"""
import os

import numpy as np
import pytest
import torch

from golden_util import T

pytestmark = pytest.mark.gpu


def _batch(B, Tn, V, seed):
    g = torch.Generator().manual_seed(seed)
    logits = torch.randn(B, Tn, V, generator=g).to(torch.bfloat16)
    return dict(logits=logits, ref_logits=(logits.float() + 0.1 * torch.randn(B, Tn, V, generator=g)).to(torch.bfloat16),
                new_logits=(logits.float() + 0.05 * torch.randn(B, Tn, V, generator=g)).to(torch.bfloat16),
                labels=torch.randint(0, V, (B, Tn), generator=g), old_values=torch.randn(B, Tn, generator=g),
                values=torch.randn(B, Tn, generator=g), scores=torch.rand(B, generator=g) * 24 - 12)


def test_rccl_world1_hot_path_and_drop_in_surface(golden):
    import torch.multiprocessing as mp
    import dist_workers
    z = golden("whiten")
    xs_all = {k: T(z[f"{k}/xs"]) for k in ("f32", "bf16", "f32_big")}
    batches = [_batch(6, 19, 1031, 70 + i) for i in range(3)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29400 + os.getpid() % 90
    p = ctx.Process(target=dist_workers.rccl_world1_worker, args=(port, batches, xs_all, q))
    p.start()
    res = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert res["backend"] == "nccl"
    assert res["comm_identity"] and res["comm_rejects_f32"]
    ser, ser_st, ser_ctl = res[("serial", "torch")]
    assert len(ser) == 3
    for key in (("pipelined", "torch"), ("serial", "rccl"), ("pipelined", "rccl")):
        outs, st, ctl = res[key]
        assert len(outs) == 3, key
        for a, b in zip(ser, outs):
            for x, y in zip(a, b):
                assert np.array_equal(x, y, equal_nan=True), key
        assert np.array_equal(ser_st, st) and np.array_equal(ser_ctl, ctl), key
    # the unsplit kernels (step() default): the same numbers up to fp32 association
    uns, _, uns_ctl = res[("unsplit", "rccl")]
    for a, b in zip(ser, uns):
        for i, (x, y) in enumerate(zip(a, b)):
            np.testing.assert_allclose(y, x, rtol=2e-2 if i == 2 else 1e-4, atol=1e-5)
    np.testing.assert_allclose(uns_ctl, ser_ctl, rtol=1e-5)
    for k, (mean, var, count, w, w2) in res["surface"].items():
        bf = k == "bf16"
        assert count == float(z[f"{k}/dist1/count"])
        assert mean == pytest.approx(float(z[f"{k}/dist1/mean"]), rel=2 ** -7 if bf else 1e-5, abs=2e-2 if bf else 1e-6)
        assert var == pytest.approx(float(z[f"{k}/dist1/var"]), rel=2 ** -6 if bf else 1e-5)
        tol = dict(rtol=2 ** -7, atol=1e-2) if bf else dict(rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(torch.from_numpy(w), T(z[f"{k}/dist1/whiten"]).float(), **tol)
        torch.testing.assert_close(torch.from_numpy(w2), T(z[f"{k}/dist1/whiten_noshift"]).float(), **tol)


def test_rccl_lag_schedule_scores_freed_after_call():
    """The side-stream score moments of the lag schedule read the caller's scores after
    pipeline_step has returned: dropping them (and reusing their memory on the main stream)
    must not change the RunningMoments merge (scores.record_stream)."""
    import torch.multiprocessing as mp
    import dist_workers
    batches = [_batch(6, 19, 1031, 90 + i) for i in range(4)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 90
    p = ctx.Process(target=dist_workers.rccl_scores_reuse_worker, args=(port, batches, q))
    p.start()
    res = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert np.all(np.isfinite(res["pipelined"]))
    assert np.array_equal(res["serial"], res["pipelined"])
