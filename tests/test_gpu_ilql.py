"""GPU parity of the ILQL loss (A10, ilql_models.py:52-116) through the C ABI
(trlx_ilql_*), against the golden fixtures produced by the reference
(tests/golden/make_golden.py make_ilql) and the CPU oracle (oracle/ppo_oracle.py
ilql_loss, pinned bit-exactly to those fixtures by tests/test_oracle_golden.py).

Tolerances: fp32 rtol 1e-5 (atol 1e-6 on gradients, whose near-zero softmax entries carry
absolute rounding); bf16 inputs are compared against the fp32 oracle on the same
bf16-quantised inputs, gradients at bf16 output resolution (rtol 1e-2).
"""
import numpy as np
import pytest
import torch

import trlx_t5_amd as P
from golden_util import T
from oracle import ppo_oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
KEYS = ("loss", "loss_q", "loss_v", "loss_cql", "loss_awac")


def batch_from(z, k):
    return P.ILQLBatch(**{n: T(z[f"{k}/{n}"]) for n in
                          ("input_ids", "attention_mask", "rewards", "states_ixs", "actions_ixs", "dones")})


def run_gpu(cfg, logits, qs, tqs, vs, batch, grad_scale=1.0):
    lg = logits.to(DEV).requires_grad_(True)
    q = [x.to(DEV).requires_grad_(True) for x in qs]
    tq = [x.to(DEV) for x in tqs]
    v = vs.to(DEV).requires_grad_(True)
    b = P.ILQLBatch(*(getattr(batch, f).to(DEV) for f in ("input_ids", "attention_mask", "rewards", "states_ixs",
                                                         "actions_ixs", "dones")))
    loss, stats = cfg.loss((lg, (q, tq, v)), b)
    assert list(stats) == [f"losses/{k}" for k in ("loss_q", "loss_v", "loss_cql", "loss_awac", "loss")]
    (loss * grad_scale).backward()
    torch.cuda.synchronize()
    return (loss.detach().cpu(), {k: stats[f"losses/{k}"].detach().cpu() for k in KEYS}, lg.grad.cpu(),
            [x.grad.cpu() for x in q], v.grad.cpu())


def run_oracle(logits, qs, tqs, vs, batch, grad_scale=1.0, **kw):
    lg = logits.float().requires_grad_(True)
    q = [x.float().requires_grad_(True) for x in qs]
    v = vs.float().requires_grad_(True)
    loss, stats = orc.ilql_loss(lg, q, [x.float() for x in tqs], v, batch.input_ids, batch.attention_mask,
                                batch.rewards, batch.actions_ixs, batch.dones, **kw)
    (loss * grad_scale).backward()
    return (loss.detach(), {k: stats[f"losses/{k}"].detach() for k in KEYS}, lg.grad, [x.grad for x in q],
            v.grad)


def check(got, want, grad_rtol=1e-5, grad_atol=1e-6):
    gl, gs, gdl, gdq, gdv = got
    wl, ws, wdl, wdq, wdv = want
    torch.testing.assert_close(gl, wl.float(), rtol=1e-5, atol=1e-6)
    for k in KEYS:
        torch.testing.assert_close(gs[k], ws[k].float(), rtol=1e-5, atol=1e-6, msg=k)
    torch.testing.assert_close(gdl.float(), wdl, rtol=grad_rtol, atol=grad_atol)
    for a, b in zip(gdq, wdq):
        torch.testing.assert_close(a.float(), b, rtol=grad_rtol, atol=grad_atol)
    torch.testing.assert_close(gdv.float(), wdv, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("k", ["c0", "c1"])
def test_ilql_golden_small(golden, k):
    z = golden("ilql_loss")
    b = batch_from(z, k)
    logits = T(z[f"{k}/logits"])
    qs = [T(z[f"{k}/q{i}"]) for i in range(2)]
    tqs = [T(z[f"{k}/tq{i}"]) for i in range(2)]
    vs = T(z[f"{k}/vs"])
    loss, stats, dl, dq, dv = run_gpu(P.ILQLConfig(), logits, qs, tqs, vs, b)
    torch.testing.assert_close(loss, T(z[f"{k}/loss"]).float(), rtol=1e-5, atol=1e-6)
    for sk in KEYS:
        torch.testing.assert_close(stats[sk], T(z[f"{k}/stats/losses/{sk}"]).float(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dl, T(z[f"{k}/dlogits"]), rtol=1e-5, atol=1e-6)
    for i in range(2):
        torch.testing.assert_close(dq[i], T(z[f"{k}/dq{i}"]), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dv, T(z[f"{k}/dvs"]), rtol=1e-5, atol=1e-6)


def test_ilql_golden_wide(golden):
    """V = 50257 fixture (inputs regenerated from the fixture's seed exactly as
    make_golden.py draws them; the reference's outputs are stored)."""
    z = golden("ilql_loss")
    k = "c2"
    b = batch_from(z, k)
    B, L = b.input_ids.shape
    A, V = L - 1, 50257
    g = torch.Generator().manual_seed(int(z[f"{k}/seed"]))
    ids = torch.randint(0, V, (B, L), generator=g)
    assert torch.equal(ids, b.input_ids)
    rewards = torch.randn(B, A, generator=g)
    assert torch.equal(rewards, b.rewards)
    logits = torch.randn(B, L, V, generator=g)
    qs = [torch.randn(B, A, V, generator=g) for _ in range(2)]
    tqs = [torch.randn(B, A, V, generator=g) for _ in range(2)]
    vs = torch.randn(B, L, 1, generator=g)
    torch.testing.assert_close(vs, T(z[f"{k}/vs"]), rtol=0, atol=0)
    loss, stats, dl, dq, dv = run_gpu(P.ILQLConfig(), logits, qs, tqs, vs, b)
    torch.testing.assert_close(loss, T(z[f"{k}/loss"]).float(), rtol=1e-5, atol=1e-6)
    for sk in KEYS:
        torch.testing.assert_close(stats[sk], T(z[f"{k}/stats/losses/{sk}"]).float(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(float(dl.double().sum()), float(z[f"{k}/dlogits_sum"]), rtol=0, atol=1e-5)
    np.testing.assert_allclose(float(dl.double().abs().sum()), float(z[f"{k}/dlogits_abs_sum"]), rtol=1e-5)
    np.testing.assert_allclose(float(dq[0].double().abs().sum()), float(z[f"{k}/dq0_abs_sum"]), rtol=1e-5)
    torch.testing.assert_close(dv, T(z[f"{k}/dvs"]), rtol=1e-5, atol=1e-6)


def make_case(B, L, V, seed, dtype=torch.float32, prompt=1, ragged=True, nq=2, peaked=False):
    """Synthetic ILQL batch in the offline orchestrator's layout (offline_orchestrator.py:
    28-73): actions_ixs = arange(prompt-1, L-1), states one longer, dones 1 but the last."""
    g = torch.Generator().manual_seed(seed)
    A = L - prompt
    ids = torch.randint(0, V, (B, L), generator=g)
    ids[0, -1] = V - 1
    ids[-1, 1] = 0
    attn = torch.ones(B, L, dtype=torch.long)
    dones = torch.ones(B, A + 1, dtype=torch.long)
    dones[:, -1] = 0
    if ragged and B > 1:  # padded rows (pad_sequence zeros) of different lengths
        for r in range(1, B, 2):
            cut = 1 + (r * 7) % (L - 1)
            attn[r, cut:] = 0
            dones[r, max(0, cut - prompt):] = 0
    aix = torch.arange(prompt - 1, L - 1).repeat(B, 1)
    six = torch.arange(prompt - 1, L).repeat(B, 1)
    rewards = torch.randn(B, A, generator=g)
    sc = 4.0 if peaked else 1.0
    logits = (torch.randn(B, L, V, generator=g) * sc).to(dtype)
    qs = [(torch.randn(B, A, V, generator=g) * sc).to(dtype) for _ in range(nq)]
    tqs = [(torch.randn(B, A, V, generator=g) * sc).to(dtype) for _ in range(nq)]
    vs = torch.randn(B, A + 1, 1, generator=g)
    return logits, qs, tqs, vs, P.ILQLBatch(ids, attn, rewards, six, aix, dones)


@pytest.mark.parametrize("B,L,V,prompt,nq,peaked", [
    (3, 7, 23, 1, 2, False), (4, 12, 1031, 3, 2, True), (2, 9, 32128, 2, 1, False), (5, 6, 4097, 1, 2, False),
    (1, 8, 777, 1, 2, False),  # B == 1: the reference's squeeze() keeps [A]
])
def test_ilql_vs_oracle_f32(B, L, V, prompt, nq, peaked):
    logits, qs, tqs, vs, b = make_case(B, L, V, 100 + V + B, prompt=prompt, nq=nq, peaked=peaked)
    check(run_gpu(P.ILQLConfig(two_qs=nq == 2), logits, qs, tqs, vs, b),
          run_oracle(logits, qs, tqs, vs, b))


@pytest.mark.parametrize("V", [50257, 32128, 1001])
def test_ilql_vs_oracle_bf16(V):
    """bf16 rows: fp32 arithmetic vs the fp32 oracle on the bf16-quantised inputs."""
    logits, qs, tqs, vs, b = make_case(3, 6, V, 7 + V, dtype=torch.bfloat16)
    got = run_gpu(P.ILQLConfig(), logits, qs, tqs, vs, b)
    assert got[2].dtype == torch.bfloat16
    check(got, run_oracle(logits, qs, tqs, vs, b), grad_rtol=1e-2, grad_atol=2e-6)


def test_ilql_hparams_grad_scale_and_strided_views():
    """Non-default tau/gamma/scales, grad_output != 1, logits as a strided view of a
    wider buffer (odd row phase), all-terminal rows and a zero attention row."""
    B, L, V = 4, 7, 3001
    logits, qs, tqs, vs, b = make_case(B, L, V, 5)
    b.dones[2, :] = 0
    wide = torch.randn(B, L, V + 5)
    wide[:, :, 3:V + 3] = logits
    lview = wide[:, :, 3:V + 3]
    cfg = P.ILQLConfig(tau=0.6, gamma=0.9, cql_scale=0.3, awac_scale=0.5)
    lg = wide.to(DEV)[:, :, 3:V + 3].requires_grad_(True)
    assert lg.stride(1) == V + 5
    got = list(run_gpu(cfg, lview, qs, tqs, vs, b, grad_scale=2.5))
    want = run_oracle(logits, qs, tqs, vs, b, grad_scale=2.5, tau=0.6, gamma=0.9, cql_scale=0.3, awac_scale=0.5)
    check(got, want)
    # the strided device view itself (rows of V+5 elements, 3-element offset)
    q = [x.to(DEV).requires_grad_(True) for x in qs]
    v = vs.to(DEV).requires_grad_(True)
    bd = P.ILQLBatch(*(getattr(b, f).to(DEV) for f in ("input_ids", "attention_mask", "rewards", "states_ixs",
                                                      "actions_ixs", "dones")))
    loss, _ = cfg.loss((lg, (q, [x.to(DEV) for x in tqs], v)), bd)
    (loss * 2.5).backward()
    torch.testing.assert_close(lg.grad.cpu(), want[2], rtol=1e-5, atol=1e-6)


def test_ilql_deterministic_and_finite_at_c5_shape():
    """C5 per-GPU shape (128 x 64 tokens, V 50257, fp32, two Q heads): bitwise-identical
    repeat runs; CE gradient rows sum to zero (softmax − onehot), and each Q row sums to
    its TD gradient (size-independent properties of the reference's autograd)."""
    B, L, V = 128, 64, 50257
    A = L - 1
    g = torch.Generator(device=DEV).manual_seed(3)
    logits = torch.randn(B, L, V, generator=g, device=DEV)
    qs = [torch.randn(B, A, V, generator=g, device=DEV).requires_grad_(True) for _ in range(2)]
    tqs = [torch.randn(B, A, V, generator=g, device=DEV) for _ in range(2)]
    vs = torch.randn(B, L, 1, generator=g, device=DEV)
    ids = torch.randint(0, V, (B, L), generator=g, device=DEV)
    dones = torch.ones(B, L, dtype=torch.long, device=DEV)
    dones[:, -1] = 0
    b = P.ILQLBatch(ids, torch.ones(B, L, dtype=torch.long, device=DEV), torch.randn(B, A, generator=g, device=DEV),
                    torch.arange(L, device=DEV).repeat(B, 1), torch.arange(A, device=DEV).repeat(B, 1), dones)
    outs = []
    for _ in range(2):
        lg = logits.clone().requires_grad_(True)
        q = [x.detach().clone().requires_grad_(True) for x in qs]
        loss, stats = P.ILQLConfig().loss((lg, (q, tqs, vs)), b)
        loss.backward()
        outs.append((loss.detach().clone(), lg.grad, q[0].grad))
    torch.cuda.synchronize()
    assert torch.isfinite(outs[0][0])
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert torch.equal(outs[0][2], outs[1][2])
    dl = outs[0][1].double()
    assert float(dl[:, -1].abs().max()) == 0.0
    assert float(dl.sum(-1).abs().max()) < 1e-6
    # Q-row sums = TD gradient 2(Q - Qt)·done²/n (the CE part sums to zero)
    act = ids[:, 1:].gather(1, torch.arange(A, device=DEV).repeat(B, 1))
    Q = qs[0].detach().gather(-1, act[..., None]).squeeze(-1).double()
    Qt = b.rewards.double() + 0.99 * vs[:, 1:, 0].double() * dones[:, 1:].double()
    n = float(dones[:, :-1].sum())
    td = 2 * (Q - Qt) * dones[:, :-1].double() / n
    torch.testing.assert_close(outs[0][2].double().sum(-1), td, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("i", range(12))
def test_ilql_random_sweep(i):
    """Seeded random shapes: B 2..5, L 3..24, prompt 1..L-2, V 2..60000 (plus 50257 /
    32128), one or two Q heads, fp32 / bf16, ragged rows, peaked or flat logits."""
    import random
    rnd = random.Random(300 + i)
    B, L = rnd.randint(2, 5), rnd.randint(3, 24)
    prompt = rnd.randint(1, L - 2)  # A >= 2 (A == 1 with B > 1 raises: documented deviation)
    V = [50257, 32128][i] if i < 2 else rnd.randint(2, 60000)
    nq = 1 + (i % 2)
    dt = torch.bfloat16 if i % 3 == 2 else torch.float32
    logits, qs, tqs, vs, b = make_case(B, L, V, 900 + i, dtype=dt, prompt=prompt, nq=nq, peaked=bool(i % 4 == 1))
    got = run_gpu(P.ILQLConfig(two_qs=nq == 2), logits, qs, tqs, vs, b)
    want = run_oracle(logits, qs, tqs, vs, b)
    if dt == torch.bfloat16:
        check(got, want, grad_rtol=1e-2, grad_atol=2e-6)
    else:
        check(got, want)


@pytest.mark.parametrize("B,L,V,nq,dtype", [(4, 9, 1031, 2, torch.float32), (3, 12, 4097, 1, torch.float32),
                                            (5, 7, 50257, 2, torch.float32), (4, 10, 2053, 2, torch.bfloat16),
                                            (40, 60, 1031, 2, torch.float32), (70, 33, 257, 1, torch.float32)])
def test_ilql_hot_path_vs_oracle(B, L, V, nq, dtype):
    """ILQLHotPath.step (the bench's C5 path: prep, rows, finalize into buffers owned by the
    hot path, eager gradients) against the oracle's loss, stats and autograd gradients, over
    two steps (the buffers are reused).  The offline orchestrator's layout with a 1-token
    prompt (A = L - 1), ragged padding."""
    logits, qs, tqs, vs, b = make_case(B, L, V, 900 + V + nq, dtype=dtype, nq=nq)
    cfg = P.ILQLConfig(two_qs=nq == 2)
    hp = P.ILQLHotPath(cfg, B, L, V, dtype, DEV)
    bd = P.ILQLBatch(*(getattr(b, f).to(DEV) for f in ("input_ids", "attention_mask", "rewards", "states_ixs",
                                                       "actions_ixs", "dones")))
    want = run_oracle(logits, qs, tqs, vs, b)
    for _ in range(2):
        losses, dl, dq, dvs = hp.step(logits.to(DEV), [q.to(DEV) for q in qs], [q.to(DEV) for q in tqs],
                                      vs.to(DEV), bd)
        torch.cuda.synchronize()
        got = losses.cpu()
        wl, ws, wdl, wdq, wdv = want
        stats = [ws[k] for k in ("loss", "loss_q", "loss_v", "loss_cql", "loss_awac")]  # ilql._SLOT order
        torch.testing.assert_close(got, torch.stack(stats).float(), rtol=1e-5, atol=1e-6)
        gr = dict(rtol=1e-2, atol=1e-6) if dtype == torch.bfloat16 else dict(rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(dl.float().cpu(), wdl, **gr)
        for a, w in zip(dq, wdq):
            torch.testing.assert_close(a.float().cpu(), w, **gr)
        torch.testing.assert_close(dvs.cpu(), wdv.reshape(B, L), rtol=1e-5, atol=1e-6)
    # prep / finalize: several workgroups at the larger shapes (7120 rows -> 7 finalize
    # blocks), their arrival tickets re-armed for the next step
    R = B * L + nq * B * (L - 1)
    tick = hp.workspace[(16 + 16 * R + 15) // 16 * 16:][:16].view(torch.int32)
    assert int(tick.abs().sum()) == 0
    with pytest.raises(ValueError):  # head count must match the config
        hp.step(logits.to(DEV), [q.to(DEV) for q in qs[:1]] * (3 - nq), [q.to(DEV) for q in tqs[:1]], vs.to(DEV), bd)


@pytest.mark.parametrize("V,dtype", [(50257, torch.float32), (4097, torch.float32), (32128, torch.bfloat16)])
def test_ilql_zero_weight_rows_not_read(V, dtype):
    """Rows whose loss weights are all zero — logits rows whose next token is padding
    (attention_mask[b, t+1] = 0) or the last position, Q rows of terminal actions
    (dones[b, a] = 0) — have zero gradients and add nothing to the losses: they hold NaN here
    and every output must still equal the oracle on the clean rows."""
    B, L = 5, 11
    logits, qs, tqs, vs, b = make_case(B, L, V, 900 + V, dtype=dtype)
    A = qs[0].shape[1]
    lp, qp = logits.clone(), [q.clone() for q in qs]
    lmask = torch.cat([b.attention_mask[:, 1:] == 0, torch.ones(B, 1, dtype=torch.bool)], dim=1)
    assert lmask[:, :-1].any() and (b.dones[:, :A] == 0).any()
    lp[lmask] = float("nan")
    for q in qp:
        q[b.dones[:, :A] == 0] = float("nan")
    got = run_gpu(P.ILQLConfig(), lp, qp, tqs, vs, b)
    tol = dict(grad_rtol=1e-2, grad_atol=2e-6) if dtype == torch.bfloat16 else {}
    check(got, run_oracle(logits, qs, tqs, vs, b), **tol)
    assert torch.equal(got[2][lmask].float(), torch.zeros_like(got[2][lmask].float()))
