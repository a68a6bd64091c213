"""ILQL generation's sampling step (csrc/ilql_sample.hip) through the C
ABI, against the oracle restatement of ilql_models.py:296-316 (log_softmax + beta * adv,
topk_mask — pinned to the reference's own topk_mask by tests/test_oracle_golden.py — and
softmax / temperature), evaluated in fp64.

Parity: for an explicit uniform u the kernel must return the token whose CDF interval (in
index order, the inverse-CDF draw) holds u, up to fp32 rounding of the CDF (rtol 1e-5 on the
interval ends); every drawn token is inside the top-k set; over many draws the empirical
frequencies match pi (the distribution torch.multinomial samples).  finished / eos
bookkeeping and logit_mask are exact."""
import pytest
import torch

import trlx_t5_amd as P
from trlx_t5_amd import _lib
from oracle import ppo_oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def oracle_pi(logits, tqs, vs, beta, top_k, temperature, mask=None):
    x = logits.double().clone()
    if mask is not None:
        x[mask] = float("-inf")
    qs = tqs[0].double() if len(tqs) == 1 else torch.minimum(tqs[0].double(), tqs[1].double())
    adv = qs - vs.double().reshape(-1, 1)
    score = torch.log_softmax(x, -1) + beta * adv
    return torch.softmax(orc.topk_mask(score, top_k) / temperature, -1), score


def sample_abi(logits, tqs, vs, beta, top_k, temperature, u, mask=None, prev=None, finished=None, eos=0):
    B, V = logits.shape
    lg = logits.to(DEV).contiguous()
    q = [t.to(DEV).contiguous() for t in tqs]
    v = vs.to(DEV, torch.float32).contiguous()
    uu = u.to(DEV, torch.float32).contiguous()
    out = torch.empty(B, dtype=torch.int64, device=DEV)
    m = None if mask is None else mask.to(DEV, torch.uint8).contiguous()
    pv = None if prev is None else prev.to(DEV).contiguous()
    fin = None if finished is None else finished.to(DEV).contiguous()
    q1 = q[1] if len(q) > 1 else None
    _lib.call("trlx_ilql_sample", lg.data_ptr(), lg.stride(0), q[0].data_ptr(), q[0].stride(0), _lib.ptr(q1),
              0 if q1 is None else q1.stride(0), _lib.dtype_code(lg), v.data_ptr(), _lib.ptr(m),
              0 if m is None else m.stride(0), _lib.ptr(pv), B, V, float(beta), int(top_k), float(temperature),
              uu.data_ptr(), out.data_ptr(), _lib.ptr(fin), int(eos), _lib.stream_of(lg))
    torch.cuda.synchronize()
    return out.cpu(), (None if fin is None else fin.cpu())


def check_draws(tok, pi, score, u, top_k):
    cdf = torch.cumsum(pi, -1)
    for b in range(pi.shape[0]):
        j = int(tok[b])
        lo = float(cdf[b, j - 1]) if j > 0 else 0.0
        hi = float(cdf[b, j])
        assert pi[b, j] > 0, (b, j)
        assert lo - 1e-5 <= float(u[b]) <= hi + 1e-5, (b, j, lo, float(u[b]), hi)
        if top_k <= pi.shape[1]:
            kth = torch.topk(score[b], top_k).values[-1]
            assert score[b, j] >= kth - 1e-6


@pytest.mark.parametrize("V,top_k,nq,dtype", [(23, 5, 2, torch.float32), (1031, 20, 2, torch.float32),
                                              (50257, 20, 2, torch.float32), (32128, 1, 1, torch.float32),
                                              (4097, 4097, 2, torch.float32), (50257, 64, 2, torch.bfloat16),
                                              (300, 500, 1, torch.float32)])
def test_sample_inverse_cdf_vs_oracle(V, top_k, nq, dtype):
    B = 16
    g = torch.Generator().manual_seed(V + top_k)
    logits = (torch.randn(B, V, generator=g) * 3).to(dtype)
    tqs = [(torch.randn(B, V, generator=g)).to(dtype) for _ in range(nq)]
    vs = torch.randn(B, generator=g)
    u = torch.rand(B, generator=g)
    u[0], u[1] = 0.0, 0.999999
    tok, _ = sample_abi(logits, tqs, vs, 2.0, top_k, 0.7, u)
    pi, score = oracle_pi(logits.float(), [t.float() for t in tqs], vs, 2.0, top_k, 0.7)
    check_draws(tok, pi, score, u, top_k)


@pytest.mark.parametrize("V,top_k,quant,dtype", [
    (3000, 20, 0.0, torch.float32),     # every score tied: more candidates than the LDS list -> bisection
    (1000, 5, 0.0, torch.float32),      # every score tied, list fits, 1000 kept > one-wave draw cap
    (50257, 600, None, torch.float32),  # k above the 512 threads of the long-row kernel
    (50257, 1000, None, torch.bfloat16),
    (20000, 50, 0.5, torch.float32),    # coarse values: heavy ties at the threshold
    (50257, 20, 1.0, torch.bfloat16)])
def test_sample_fallback_paths(V, top_k, quant, dtype):
    """Rows that defeat the candidate pre-filter (ties, large k) take the block-wide paths;
    every path must give the inverse-CDF token of the oracle's pi."""
    B = 8
    g = torch.Generator().manual_seed(V + top_k)
    if quant == 0.0:
        logits = torch.zeros(B, V)
        tqs = [torch.zeros(B, V) for _ in range(2)]
    else:
        logits = torch.randn(B, V, generator=g) * 3
        tqs = [torch.randn(B, V, generator=g) for _ in range(2)]
        if quant:
            logits, tqs = (logits / quant).round() * quant, [(t / quant).round() * quant for t in tqs]
    logits, tqs = logits.to(dtype), [t.to(dtype) for t in tqs]
    vs = torch.randn(B, generator=g)
    u = torch.rand(B, generator=g)
    u[0], u[1] = 0.0, 0.999999
    tok, _ = sample_abi(logits, tqs, vs, 2.0, top_k, 0.7, u)
    pi, score = oracle_pi(logits.float(), [t.float() for t in tqs], vs, 2.0, top_k, 0.7)
    check_draws(tok, pi, score, u, top_k)


def test_sample_distribution_matches_pi():
    """Many draws of one row: empirical frequencies vs pi (the multinomial it replaces)."""
    V, top_k, n = 40, 8, 20000
    g = torch.Generator().manual_seed(5)
    row = torch.randn(1, V, generator=g) * 2
    tq = [torch.randn(1, V, generator=g) for _ in range(2)]
    vs = torch.randn(1, generator=g)
    logits = row.repeat(n, 1)
    tqs = [t.repeat(n, 1) for t in tq]
    tok, _ = sample_abi(logits, tqs, vs.repeat(n), 1.0, top_k, 1.0, torch.rand(n, generator=g))
    pi, _ = oracle_pi(row, tq, vs, 1.0, top_k, 1.0)
    freq = torch.bincount(tok, minlength=V).double() / n
    assert int((freq > 0).sum()) <= top_k
    assert float((freq - pi[0]).abs().max()) < 0.015


def test_sample_logit_mask_finished_and_eos():
    B, V, eos = 6, 500, 7
    g = torch.Generator().manual_seed(9)
    logits = torch.randn(B, V, generator=g)
    tqs = [torch.randn(B, V, generator=g) for _ in range(2)]
    vs = torch.randn(B, generator=g)
    mask = torch.zeros(V, V, dtype=torch.bool)
    prev = torch.randint(0, V, (B,), generator=g)
    for b in range(B):  # forbid everything but 3 tokens after prev[b]
        mask[prev[b]] = True
        mask[prev[b], (b * 11 + torch.arange(3)) % V] = False
    finished = torch.tensor([0, 1, 0, 0, 1, 0], dtype=torch.int64)
    u = torch.rand(B, generator=g)
    tok, fin = sample_abi(logits, tqs, vs, 1.0, 20, 1.0, u, mask=mask, prev=prev, finished=finished.clone(), eos=eos)
    pi, score = oracle_pi(logits, tqs, vs, 1.0, 20, 1.0, mask=mask[prev])
    for b in range(B):
        if finished[b]:
            assert int(tok[b]) == eos and int(fin[b]) == 1
        else:
            assert int(tok[b]) in ((b * 11 + torch.arange(3)) % V).tolist()
            assert int(fin[b]) == int(int(tok[b]) == eos)
    live = finished == 0
    check_draws(tok[live], pi[live], score[live], u[live], 20)


def test_sample_step_wrapper():
    """ilql_sample_step: the generate-loop form ([B, 1] ids, finished updated in place)."""
    B, V = 4, 1000
    g = torch.Generator(device=DEV).manual_seed(1)
    logits = torch.randn(B, V, generator=g, device=DEV)
    tqs = [torch.randn(B, V, generator=g, device=DEV) for _ in range(2)]
    vs = torch.randn(B, 1, generator=g, device=DEV)
    fin = torch.zeros(B, 1, dtype=torch.int64, device=DEV)
    ids = P.ilql_sample_step(logits, tqs, vs, beta=1.0, top_k=20, finished=fin, eos_token_id=3, generator=g)
    assert ids.shape == (B, 1) and ids.dtype == torch.int64
    assert bool(((ids >= 0) & (ids < V)).all())
