"""Ragged batches: the rows a ragged batch does not need are not read.

  * experience rows with decoder lengths (trlx_lsm_gather_fwd_ragged and the loss-tail
    launch of the pipelined schedule): rows (b, t >= L_b) are store padding — the padded
    store holds 0.0 logprobs there (ppo_pipeline.py:47-65) — so lp = ref_lp = 0 and the row
    is not read;
  * loss rows of masked tokens (mask == 0): d loss / d lp = 0 (ppo_models.py:165-177 scales
    every lp path by the mask), so the dlogits row is written as zeros without being read and
    lp_out = 0.
"Not read" is proven by filling those rows with NaN: every output must equal the oracle run
on clean logits (the reference itself would turn a NaN masked row into a NaN loss through
NaN * 0 — the documented deviation).  Tolerances as tests/test_gpu_parity.py.
"""
import pytest
import torch

import trlx_t5_amd as P
from trlx_t5_amd import _lib
from golden_util import loss_rows_lp
from oracle import ppo_oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
RT32 = dict(rtol=1e-5, atol=1e-5)


def _ragged(B, Tn, V, seed, dt=torch.bfloat16, random_mask=False):
    g = torch.Generator().manual_seed(seed)
    logits = torch.randn(B, Tn, V, generator=g).to(dt)
    ref_logits = (logits.float() + 0.1 * torch.randn(B, Tn, V, generator=g)).to(dt)
    new_logits = (logits.float() + 0.05 * torch.randn(B, Tn, V, generator=g)).to(dt)
    labels = torch.randint(0, V, (B, Tn), generator=g)
    old_values = torch.randn(B, Tn, generator=g)
    values = old_values + 0.3 * torch.randn(B, Tn, generator=g)
    scores = torch.rand(B, generator=g) * 24 - 12
    L = torch.randint(1, Tn + 1, (B,), generator=g)
    L[0] = Tn
    pad = torch.arange(Tn)[None, :] >= L[:, None]
    mask = (~pad).long()
    if random_mask:  # masked tokens inside the rollouts too (any mask pattern, value 2 = weight)
        mask = mask * (torch.rand(B, Tn, generator=g) > 0.25).long()
        mask[0, 0] = 2
    old_values = old_values.masked_fill(pad, 0)
    return dict(logits=logits, ref_logits=ref_logits, new_logits=new_logits, labels=labels, old_values=old_values,
                values=values, scores=scores, lengths=L, mask=mask, pad=pad)


def _poison(x):
    """Device copies with NaN in every row the kernels must not read."""
    d = {k: v.to(DEV) for k, v in x.items()}
    for k in ("logits", "ref_logits"):
        d[k] = d[k].clone()
        d[k][d["pad"]] = float("nan")
    d["new_logits"] = d["new_logits"].clone()
    d["new_logits"][d["mask"] == 0] = float("nan")
    return d


@pytest.mark.parametrize("V,dt,ordered", [(32128, torch.bfloat16, True), (32128, torch.bfloat16, False),
                                          (50257, torch.bfloat16, True), (1031, torch.float32, True),
                                          (1031, torch.float32, False), (50257, torch.float32, True)])
def test_ragged_experience_rows_not_read(V, dt, ordered):
    """ordered: with the order scratch (valid rows dispatched first), else natural order."""
    x = _ragged(6, 21, V, 3 + V, dt)
    d = _poison(x)
    B, Tn = 6, 21
    lp0 = torch.full((B, Tn), 7.0, device=DEV)
    lp1 = torch.full((B, Tn), 7.0, device=DEV)
    lg = d["logits"]
    nb = _lib.query("trlx_ragged_order_bytes", B, Tn)
    assert nb >= 4 * (B * Tn + 1)
    order = torch.full((nb // 4,), 12345, dtype=torch.int32, device=DEV) if ordered else None
    _lib.call("trlx_lsm_gather_fwd_ragged", lg.data_ptr(), d["ref_logits"].data_ptr(), _lib.dtype_code(lg), B, Tn, V,
              lg.stride(0), lg.stride(1), d["labels"].data_ptr(), Tn, 1, d["lengths"].data_ptr(),
              None if order is None else order.data_ptr(), lp0.data_ptr(), lp1.data_ptr(), _lib.F32,
              torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    if order is not None and V == 32128:  # the resident rows took the order: valid rows first, then ~padding
        L = x["lengths"]
        nvalid = int(L.sum())
        want = [b * Tn + t for b in range(B) for t in range(int(L[b]))]
        want += [~(b * Tn + t) for b in range(B) for t in range(int(L[b]), Tn)]
        got = order.cpu().tolist()
        assert got[:B * Tn] == want and got[B * Tn] == nvalid
    pad = x["pad"]
    for got, src in ((lp0, x["logits"]), (lp1, x["ref_logits"])):
        got = got.cpu()
        assert torch.equal(got[pad], torch.zeros(int(pad.sum())))
        ref = orc.logprobs_from_logits(src.float(), x["labels"])
        torch.testing.assert_close(got[~pad], ref[~pad], **RT32)


@pytest.mark.parametrize("V,dt", [(32128, torch.bfloat16), (20000, torch.float32), (1031, torch.bfloat16)])
def test_ragged_rows_bit_identical_to_dense(V, dt):
    """With every length = T nothing is padding: the ragged launch gives the plain
    trlx_lsm_gather_fwd's bits."""
    B, Tn = 7, 13
    x = _ragged(B, Tn, V, 5 + V, dt)
    lg, rg, y = x["logits"].to(DEV), x["ref_logits"].to(DEV), x["labels"].to(DEV)
    full = torch.full((B,), Tn, dtype=torch.int64, device=DEV)
    outs = []
    for lens in (None, full):
        lp0, lp1 = torch.empty(B, Tn, device=DEV), torch.empty(B, Tn, device=DEV)
        args = (lg.data_ptr(), rg.data_ptr(), _lib.dtype_code(lg), B, Tn, V, lg.stride(0), lg.stride(1), y.data_ptr(),
                Tn, 1)
        s = torch.cuda.current_stream().cuda_stream
        if lens is None:
            _lib.call("trlx_lsm_gather_fwd", *args, lp0.data_ptr(), lp1.data_ptr(), _lib.F32, None, None, s)
        else:
            _lib.call("trlx_lsm_gather_fwd_ragged", *args, lens.data_ptr(), None, lp0.data_ptr(), lp1.data_ptr(),
                      _lib.F32, s)
        outs.append((lp0, lp1))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("V,dt,variant", [(32128, torch.bfloat16, 0), (50257, torch.bfloat16, 0),
                                          (50257, torch.float32, 0), (4099, torch.bfloat16, 2),
                                          (3000, torch.float32, 2)])
def test_masked_loss_rows_not_read(V, dt, variant):
    """loss_from_logits (trlx_ppo_policy_fused) with an arbitrary mask: masked rows hold NaN.
    variant 2 forces the streaming rows kernel."""
    x = _ragged(5, 17, V, 11 + V, dt, random_mask=True)
    d = _poison(x)
    g = torch.Generator().manual_seed(V)
    olp = orc.logprobs_from_logits(x["new_logits"].float(), x["labels"]) + 0.1 * torch.randn(5, 17, generator=g)
    adv, ret = torch.randn(5, 17, generator=g), torch.randn(5, 17, generator=g)
    cfg = P.PPOConfig()
    xd = d["new_logits"].requires_grad_(True)
    vd = d["values"].clone().requires_grad_(True)
    _lib.set_tuning("row_variant", variant)
    try:
        loss, stats, lp_new = cfg.loss_from_logits(xd, vd, d["labels"], olp.to(DEV), d["old_values"], adv.to(DEV),
                                                   ret.to(DEV), mask=d["mask"])
        loss.backward()
        torch.cuda.synchronize()
    finally:
        _lib.set_tuning("row_variant", 0)
    xf = x["new_logits"].float().requires_grad_(True)
    vf = x["values"].clone().requires_grad_(True)
    lpf = orc.logprobs_from_logits(xf, x["labels"])
    rloss, rstats = orc.ppo_loss(lpf, vf, olp, x["old_values"], adv, ret, x["mask"])
    rloss.backward()
    m0 = x["mask"] == 0
    grad = xd.grad.cpu()
    assert torch.equal(grad[m0].float(), torch.zeros_like(grad[m0].float()))  # zero rows, +0 bits
    assert not torch.signbit(grad[m0].float()).any()
    torch.testing.assert_close(lp_new.cpu(), loss_rows_lp(lpf.detach(), x["mask"]), **RT32)
    torch.testing.assert_close(loss.detach().cpu(), rloss.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(vd.grad.cpu(), vf.grad, rtol=1e-5, atol=1e-7)
    tol = dict(rtol=1e-5, atol=1e-7) if dt == torch.float32 else dict(rtol=1e-2, atol=1e-7)
    torch.testing.assert_close(grad.float(), xf.grad, **tol)
    for k in P.STATS_KEYS:
        assert float(stats[k]) == pytest.approx(float(rstats[k]), rel=1e-5, abs=1e-6), k


@pytest.mark.parametrize("B,Tn,V,dt", [(16, 48, 32128, torch.bfloat16), (12, 48, 50257, torch.bfloat16),
                                       (6, 70, 50257, torch.float32), (9, 33, 257, torch.bfloat16)])
def test_ragged_step_vs_oracle(B, Tn, V, dt):
    """PPOHotPath.step (unsplit) and step(split_beta) on a ragged batch whose padded rows hold
    NaN, vs the oracle on the clean batch."""
    x = _ragged(B, Tn, V, 100 + B + V, dt)
    d = _poison(x)
    ref = orc.ppo_step_reference(x["logits"].float(), x["ref_logits"].float(), x["new_logits"].float(), x["labels"],
                                 x["old_values"], x["values"], x["scores"], kl_coef=0.05, lengths=x["lengths"],
                                 mask=x["mask"])
    for split in (False, True):
        hp = P.PPOHotPath(P.PPOConfig(), B, Tn, V, dt, DEV, kl_coef=0.05, split_beta=split)
        loss, stats, dl, dv = hp.step(d["logits"], d["ref_logits"], d["new_logits"], d["labels"], d["old_values"],
                                      d["values"], d["scores"], lengths=d["lengths"], mask=d["mask"])
        hp.wait_stats()
        torch.cuda.synchronize()
        torch.testing.assert_close(hp.lp_old.cpu(), ref["lp"], **RT32)
        torch.testing.assert_close(hp.ref_lp.cpu(), ref["ref_lp"], **RT32)
        torch.testing.assert_close(hp.rewards.cpu(), ref["rewards"], **RT32)
        torch.testing.assert_close(hp.returns.cpu(), ref["returns"], rtol=1e-5, atol=2e-5)
        torch.testing.assert_close(hp.lp_new.cpu(), loss_rows_lp(ref["new_lp"], x["mask"]), **RT32)
        torch.testing.assert_close(loss.cpu().reshape(()), ref["loss"], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(dv.cpu(), ref["dvalues"], rtol=1e-5, atol=1e-8)
        tol = dict(rtol=8e-3, atol=1e-9) if dt == torch.bfloat16 else dict(rtol=1e-5, atol=1e-8)
        torch.testing.assert_close(dl.float().cpu(), ref["dlogits"], **tol)
        assert torch.equal(dl[x["pad"].to(DEV)].float().abs().sum(), torch.zeros((), device=DEV))
        st = stats.cpu().tolist()
        for i, k in enumerate(P.STATS_KEYS):
            assert st[i] == pytest.approx(float(ref["stats"][k]), rel=1e-5, abs=1e-6), (split, k)



@pytest.mark.parametrize("B,Tn,V,ragged", [(256, 48, 32128, True), (128, 48, 50257, False)])
def test_bench_shard_vs_oracle(B, Tn, V, ragged):
    """The bench's shards at full size — C3: 256 rollouts x 48 decoder tokens x V 32128 with
    ragged decoder lengths, the padded rows NaN; C2: 128 x 48 x V 50257 dense — bf16 logits
    through PPOHotPath.step, against the oracle's reference ops run on the GPU in fp32 on the
    clean batch (the C3 path was pinned only at B <= 16)."""
    g = torch.Generator(device=DEV).manual_seed(512)
    f = dict(generator=g, device=DEV)
    logits = torch.randn(B, Tn, V, **f).to(torch.bfloat16)
    ref_logits = (logits.float() + 0.1 * torch.randn(B, Tn, V, **f)).to(torch.bfloat16)
    new_logits = (logits.float() + 0.05 * torch.randn(B, Tn, V, **f)).to(torch.bfloat16)
    labels = torch.randint(0, V, (B, Tn), **f)
    old_values = torch.randn(B, Tn, **f)
    values = old_values + 0.3 * torch.randn(B, Tn, **f)
    scores = torch.rand(B, **f) * 24 - 12
    L = torch.randint(1, Tn + 1, (B,), **f) if ragged else torch.full((B,), Tn, device=DEV)
    L[0] = Tn
    pad = torch.arange(Tn, device=DEV)[None, :] >= L[:, None]
    mask = (~pad).long()
    old_values = old_values.masked_fill(pad, 0)
    if not ragged:
        L = mask = None
    ref = orc.ppo_step_reference(logits.float(), ref_logits.float(), new_logits.float(), labels, old_values, values,
                                 scores, kl_coef=0.05, lengths=L, mask=mask)
    lg, rl, nl = logits.clone(), ref_logits.clone(), new_logits.clone()
    lg[pad] = float("nan")
    rl[pad] = float("nan")
    nl[pad] = float("nan")
    hp = P.PPOHotPath(P.PPOConfig(), B, Tn, V, torch.bfloat16, DEV, kl_coef=0.05)
    loss, stats, dl, dv = hp.step(lg, rl, nl, labels, old_values, values, scores, lengths=L, mask=mask)
    hp.wait_stats()
    torch.cuda.synchronize()
    torch.testing.assert_close(hp.lp_old, ref["lp"], **RT32)
    torch.testing.assert_close(hp.ref_lp, ref["ref_lp"], **RT32)
    torch.testing.assert_close(hp.rewards, ref["rewards"], **RT32)
    torch.testing.assert_close(hp.returns, ref["returns"], rtol=1e-5, atol=2e-5)
    torch.testing.assert_close(hp.lp_new, loss_rows_lp(ref["new_lp"], mask), **RT32)
    torch.testing.assert_close(loss.reshape(()), ref["loss"].detach().reshape(()), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dv, ref["dvalues"], rtol=1e-5, atol=1e-8)
    torch.testing.assert_close(dl.float(), ref["dlogits"], rtol=8e-3, atol=1e-9)
    assert torch.equal(dl[pad].float().abs().sum(), torch.zeros((), device=DEV))
    st = stats.cpu().tolist()
    for i, k in enumerate(P.STATS_KEYS):
        assert st[i] == pytest.approx(float(torch.as_tensor(ref["stats"][k]).detach()), rel=1e-5, abs=1e-6), k


def test_ragged_pipeline_matches_step():
    """The pipelined schedule (ragged experience rows inside the loss-tail launch, masked loss
    rows beside the folded GAE) over three poisoned ragged batches: bit-identical to
    step(split_beta=True) with standalone loss tails."""
    B, Tn, V = 10, 48, 32128
    xs = [_ragged(B, Tn, V, 40 + i) for i in range(3)]
    ds = [_poison(x) for x in xs]
    args = lambda d: (d["logits"], d["ref_logits"], d["new_logits"], d["labels"], d["old_values"],  # noqa: E731
                      d["values"], d["scores"])
    # serial: the loss tail as its own launch; pipelined: folded into the experience launch
    ser = P.PPOHotPath(P.PPOConfig(), B, Tn, V, torch.bfloat16, DEV, kl_coef=0.05, split_beta=True)
    want = []
    for d in ds:
        loss, stats, dl, dv = ser.step(*args(d), lengths=d["lengths"], mask=d["mask"])
        ser.wait_stats()
        want.append((loss.clone(), stats.clone(), dl.clone(), dv.clone()))
    pip = P.PPOHotPath(P.PPOConfig(), B, Tn, V, torch.bfloat16, DEV, kl_coef=0.05, defer_tail=True)
    got = []
    for d in ds:
        o = pip.pipeline_step(*args(d), lengths=d["lengths"], mask=d["mask"])
        if o is not None:
            pip.wait_stats()
            got.append(tuple(t.clone() for t in o))
    o = pip.pipeline_flush()
    pip.wait_stats()
    got.append(tuple(t.clone() for t in o))
    torch.cuda.synchronize()
    assert len(got) == 3
    for w, g in zip(want, got):
        for a, b in zip(w, g):
            assert torch.equal(a, b)
        assert bool(torch.isfinite(g[0]).all()) and bool(torch.isfinite(g[2].float()).all())



def test_fused_abi_ragged_step():
    """The fused C-ABI pair (trlx_ppo_experience_fused with lengths — its experience rows
    ordered valid-first through the workspace — and trlx_ppo_loss_fused with the mask) on a
    poisoned ragged batch vs the oracle on the clean one."""
    B, Tn, V = 12, 40, 32128
    x = _ragged(B, Tn, V, 321)
    d = _poison(x)
    s = torch.cuda.current_stream().cuda_stream
    f32 = dict(dtype=torch.float32, device=DEV)
    lp, rlp, rew, adv, ret = (torch.empty(B, Tn, **f32) for _ in range(5))
    lpn, dv = torch.empty(B, Tn, **f32), torch.empty(B, Tn, **f32)
    stats = torch.zeros(_lib.MOMENT_SLOTS, dtype=torch.float64, device=DEV)
    loss, lstats = torch.empty(1, **f32), torch.empty(_lib.PPO_STATS, **f32)
    ws = torch.zeros(_lib.query("trlx_ppo_workspace_bytes", B, Tn), dtype=torch.uint8, device=DEV)
    dx = torch.empty(B, Tn, V, dtype=torch.bfloat16, device=DEV)
    lg, rg, ng = d["logits"], d["ref_logits"], d["new_logits"]
    y = d["labels"]
    _lib.call("trlx_ppo_experience_fused", lg.data_ptr(), rg.data_ptr(), _lib.BF16, B, Tn, V, Tn * V, V, y.data_ptr(),
              Tn, 1, d["old_values"].data_ptr(), _lib.F32, d["scores"].data_ptr(), d["lengths"].data_ptr(),
              d["mask"].data_ptr(), 0.05, 1.0, 0.95, lp.data_ptr(), rlp.data_ptr(), rew.data_ptr(), adv.data_ptr(),
              ret.data_ptr(), _lib.F32, stats.data_ptr(), ws.data_ptr(), s)
    _lib.call("trlx_ppo_loss_fused", ng.data_ptr(), _lib.BF16, B, Tn, V, Tn * V, V, y.data_ptr(), Tn, 1, lp.data_ptr(),
              _lib.F32, adv.data_ptr(), stats.data_ptr(), 1, d["mask"].data_ptr(), d["values"].data_ptr(), _lib.F32,
              d["old_values"].data_ptr(), _lib.F32, ret.data_ptr(), _lib.F32, 0.2, 0.2, 1.0, lpn.data_ptr(),
              dx.data_ptr(), Tn * V, V, dv.data_ptr(), loss.data_ptr(), lstats.data_ptr(), ws.data_ptr(), s)
    torch.cuda.synchronize()
    ref = orc.ppo_step_reference(x["logits"].float(), x["ref_logits"].float(), x["new_logits"].float(), x["labels"],
                                 x["old_values"], x["values"], x["scores"], kl_coef=0.05, lengths=x["lengths"],
                                 mask=x["mask"])
    torch.testing.assert_close(lp.cpu(), ref["lp"], **RT32)
    torch.testing.assert_close(rlp.cpu(), ref["ref_lp"], **RT32)
    torch.testing.assert_close(rew.cpu(), ref["rewards"], **RT32)
    torch.testing.assert_close(ret.cpu(), ref["returns"], rtol=1e-5, atol=2e-5)
    torch.testing.assert_close(lpn.cpu(), loss_rows_lp(ref["new_lp"], x["mask"]), **RT32)
    torch.testing.assert_close(loss.cpu().reshape(()), ref["loss"], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dv.cpu(), ref["dvalues"], rtol=1e-5, atol=1e-8)
    torch.testing.assert_close(dx.float().cpu(), ref["dlogits"], rtol=8e-3, atol=1e-9)
    st = lstats.cpu().tolist()
    for i, k in enumerate(P.STATS_KEYS):
        assert st[i] == pytest.approx(float(ref["stats"][k]), rel=1e-5, abs=1e-6), k
    assert int(x["lengths"].sum()) < B * Tn  # a ragged batch


@pytest.mark.parametrize("launch", [1, 2])
@pytest.mark.parametrize("B,Tn,V", [(1100, 3, 4099), (2100, 2, 32128), (1500, 1, 32128), (3, 700, 32128),
                                    (37, 61, 32128)])
def test_ragged_order_many_rollouts(B, Tn, V, launch):
    """The ragged order over several workgroups of rows (rollouts straddling them, one row per
    rollout, rollouts longer than a workgroup's rows), in both forms — k_ragged_order's one
    launch and row_order.h's two chunk-count launches (the default past 64 chunks; tuning
    "order_launch"): the list is valid-first in row order, the count follows, and the ordered
    launch gives the natural-order launch's bits (lengths include 0 and values beyond T)."""
    _lib.set_tuning("order_launch", launch)
    try:
        _ragged_order_case(B, Tn, V)
    finally:
        _lib.set_tuning("order_launch", 0)


def _ragged_order_case(B, Tn, V):
    g = torch.Generator().manual_seed(B)
    x = torch.randn(B, Tn, V, generator=g).to(torch.bfloat16).to(DEV)
    y = torch.randint(0, V, (B, Tn), generator=g).to(DEV)
    L = torch.randint(0, Tn + 2, (B,), generator=g)
    Ld = L.to(DEV)
    nb = _lib.query("trlx_ragged_order_bytes", B, Tn)
    order = torch.zeros(nb // 4, dtype=torch.int32, device=DEV)
    outs = []
    for o in (None, order):
        lp0, lp1 = torch.full((B, Tn), 7.0, device=DEV), torch.full((B, Tn), 7.0, device=DEV)
        _lib.call("trlx_lsm_gather_fwd_ragged", x.data_ptr(), x.data_ptr(), _lib.BF16, B, Tn, V, x.stride(0),
                  x.stride(1), y.data_ptr(), Tn, 1, Ld.data_ptr(), None if o is None else o.data_ptr(), lp0.data_ptr(),
                  lp1.data_ptr(), _lib.F32, torch.cuda.current_stream().cuda_stream)
        outs.append((lp0.cpu(), lp1.cpu()))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    if V == 32128:  # the resident rows (and so the order) were used
        Lc = L.clamp(0, Tn)
        want = [b * Tn + t for b in range(B) for t in range(int(Lc[b]))]
        want += [~(b * Tn + t) for b in range(B) for t in range(int(Lc[b]), Tn)]
        got = order.cpu().tolist()
        assert got[:B * Tn] == want and got[B * Tn] == int(Lc.sum())
    pad = torch.arange(Tn)[None, :] >= L[:, None]
    assert torch.equal(outs[1][0][pad], torch.zeros(int(pad.sum())))
