"""Device-resident rollout store on the GPU, through the C ABI
(trlx_rows_copy): push / collate against the reference store's own loader output
(tests/golden/rollout_store.npz, made by importing trlx/pipeline/ppo_pipeline.py) and
against oracle.ppo_collate (pinned to that fixture) for shuffled orders, growth of capacity
and widths, bf16 value fields, element access and clear_history.  Bit-exact throughout
(pure data movement)."""
import types

import pytest
import torch

import trlx_t5_amd as P
from golden_util import T
from oracle import ppo_oracle as orc

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
NAMES = ("query_tensors", "response_tensors", "logprobs", "values", "rewards")


def chunks_from(z):
    return [tuple(T(z[f"chunk{ci}/{n}"]) for n in ("query", "response", "logprobs", "values", "rewards"))
            for ci in range(3)]


def elems_of(chunks):
    out = []
    for q, r, lp, v, rw in chunks:
        out += [types.SimpleNamespace(query_tensor=q[i], response_tensor=r[i], logprobs=lp[i], values=v[i],
                                      rewards=rw[i]) for i in range(q.shape[0])]
    return out


@pytest.mark.parametrize("api", ["push_batch", "push_elements"])
def test_store_matches_reference_loader(golden, api):
    z = golden("rollout_store")
    store = P.PPORolloutStorage(pad_token_id=0, device=DEV, capacity=2)  # forces capacity growth
    for q, r, lp, v, rw in chunks_from(z):
        if api == "push_batch":
            store.push_batch(q.to(DEV), r.to(DEV), lp.to(DEV), v.to(DEV), rw.to(DEV))
        else:
            store.push([P.PPORLElement(q[i], r[i], lp[i], v[i], rw[i]) for i in range(q.shape[0])])
    assert len(store) == 9
    batches = list(store.create_loader(4, shuffle=False))
    assert len(batches) == int(z["n_batches"])
    for bi, b in enumerate(batches):
        for name in NAMES:
            got = getattr(b, name)
            assert got.is_cuda
            assert torch.equal(got.cpu(), T(z[f"batch{bi}/{name}"])), (bi, name)


def test_store_shuffled_vs_oracle_and_getitem(golden):
    z = golden("rollout_store")
    chunks = chunks_from(z)
    store = P.PPORolloutStorage(pad_token_id=0, device=DEV)
    for c in chunks:
        store.push_batch(*(t.to(DEV) for t in c))
    elems = elems_of(chunks)
    g = torch.Generator().manual_seed(3)
    loader = store.create_loader(3, shuffle=True, generator=g)
    order = torch.randperm(9, generator=torch.Generator().manual_seed(3)).tolist()
    for bi, b in enumerate(loader):
        want = orc.ppo_collate([elems[i] for i in order[3 * bi:3 * bi + 3]], 0)
        for name, w in zip(NAMES, want):
            assert torch.equal(getattr(b, name).cpu(), w), (bi, name)
    for i in (0, 4, 8, -1):
        e, w = store[i], elems[i]
        for f in ("query_tensor", "response_tensor", "logprobs", "values", "rewards"):
            assert torch.equal(getattr(e, f).cpu(), getattr(w, f))


def test_store_width_growth_bf16_and_clear():
    """A wider chunk after narrower ones re-aligns the buffers (queries stay right-aligned);
    bf16 value fields; odd widths (2-byte copies); clear_history restores the padding."""
    g = torch.Generator().manual_seed(11)
    pad = 7
    chunks = []
    for n, wq, wr in ((5, 3, 5), (3, 9, 13), (4, 1, 1), (6, 12, 48)):
        q = torch.randint(8, 100, (n, wq), generator=g)
        r = torch.randint(8, 100, (n, wr), generator=g)
        lp = torch.randn(n, wr, generator=g).to(torch.bfloat16)
        v = torch.randn(n, wr, generator=g).to(torch.bfloat16)
        rw = torch.randn(n, wr, generator=g)
        chunks.append((q, r, lp, v, rw))
    for round_ in range(2):
        store = P.PPORolloutStorage(pad_token_id=pad, device=DEV, capacity=4) if round_ == 0 else store
        if round_ == 1:
            store.clear_history()
            assert len(store) == 0
        for c in chunks:
            store.push_batch(*(t.to(DEV) for t in c))
        elems = elems_of(chunks)
        for bs in (1, 5, 18):
            order = list(range(len(elems)))
            for bi, b in enumerate(store.create_loader(bs, shuffle=False)):
                want = orc.ppo_collate([elems[i] for i in order[bs * bi:bs * bi + bs]], pad)
                for name, w in zip(NAMES, want):
                    got = getattr(b, name).cpu()
                    assert got.dtype == w.dtype and torch.equal(got, w), (round_, bs, bi, name)


def test_store_feeds_the_hot_path():
    """A collated batch goes straight into PPOConfig.loss_from_logits-style consumers: the
    device tensors are contiguous with the reference's shapes."""
    store = P.PPORolloutStorage(pad_token_id=0, device=DEV)
    B, Lq, T_ = 8, 6, 10
    store.push_batch(torch.ones(B, Lq, dtype=torch.long, device=DEV), torch.ones(B, T_, dtype=torch.long, device=DEV),
                     torch.zeros(B, T_, device=DEV), torch.zeros(B, T_, device=DEV), torch.zeros(B, T_, device=DEV))
    b = next(iter(store.create_loader(8, shuffle=True)))
    assert b.query_tensors.shape == (B, Lq) and b.response_tensors.shape == (B, T_)
    assert all(getattr(b, n).is_contiguous() for n in NAMES)
