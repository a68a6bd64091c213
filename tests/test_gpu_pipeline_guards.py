"""pipeline_step_from_hidden's submit-time guards: batch k's loss runs inside
call k+1, so
  * a new_hidden / new_weight the loss side cannot take is refused when batch k is SUBMITTED,
    before any launch — the pending batch and the buffers stay as they were, and the next
    good call still returns the earlier batch's results;
  * an in-place update of new_weight between the submitting call and the call running the
    loss (an optimizer.step in between) is refused instead of pairing hidden(k) with W(k+1).
"""
import pytest
import torch

import trlx_t5_amd as P

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _batch(B, T, V, H, seed):
    g = torch.Generator().manual_seed(seed)
    h = torch.randn(B, T, H, generator=g).to(torch.bfloat16).to(DEV)
    w = (torch.randn(V, H, generator=g) * 0.05).to(torch.bfloat16).to(DEV)
    new_h = (h.float() + 0.05 * torch.randn(B, T, H, generator=g).to(DEV)).to(torch.bfloat16)
    labels = torch.randint(0, V, (B, T), generator=g).to(DEV)
    old_values = torch.randn(B, T, generator=g).to(DEV)
    values = old_values + 0.3
    scores = (torch.rand(B, generator=g) * 24 - 12).to(DEV)
    return h, w, new_h, labels, old_values, values, scores


def test_bad_loss_operands_refused_at_submit():
    B, T, V, H = 4, 8, 1031, 512
    h, w, new_h, labels, ov, v, sc = _batch(B, T, V, H, 1)
    hp = P.PPOHotPath(P.PPOConfig(), B, T, V, torch.bfloat16, DEV, kl_coef=0.05)
    assert hp.pipeline_step_from_hidden(h, w, h, w, new_h, labels, ov, v, sc) is None
    pending = hp._pending
    for bad in (new_h.float(), new_h[:, :, :256].contiguous()):
        with pytest.raises(ValueError):
            hp.pipeline_step_from_hidden(h, w, h, w, bad, labels, ov, v, sc)
        assert hp._pending is pending
    with pytest.raises(ValueError):  # a fused loss route at an H it is not built for
        hp.pipeline_step_from_hidden(h, w, h, w, new_h, labels, ov, v, sc,
                                     new_weight=torch.zeros(V, 1024, dtype=torch.bfloat16, device=DEV))
    assert hp._pending is pending
    out = hp.pipeline_step_from_hidden(h, w, h, w, new_h, labels, ov, v, sc)
    torch.cuda.synchronize()
    assert out is not None and torch.isfinite(out[0]).all()
    # the same batch again on a fresh hot path: the refused calls changed nothing
    hp2 = P.PPOHotPath(P.PPOConfig(), B, T, V, torch.bfloat16, DEV, kl_coef=0.05)
    hp2.pipeline_step_from_hidden(h, w, h, w, new_h, labels, ov, v, sc)
    out2 = hp2.pipeline_step_from_hidden(h, w, h, w, new_h, labels, ov, v, sc)
    torch.cuda.synchronize()
    for a, b in zip(out, out2):
        assert torch.equal(a, b)


def test_in_place_weight_update_between_submit_and_loss_refused():
    B, T, V, H = 4, 8, 1031, 512
    h, w, new_h, labels, ov, v, sc = _batch(B, T, V, H, 2)
    hp = P.PPOHotPath(P.PPOConfig(), B, T, V, torch.bfloat16, DEV, kl_coef=0.05)
    wn = w.clone()
    hp.pipeline_step_from_hidden(h, w, h, w, new_h, labels, ov, v, sc, new_weight=wn)
    wn.mul_(1.0)  # an optimizer step in place
    with pytest.raises(RuntimeError, match="modified in place"):
        hp.pipeline_step_from_hidden(h, w, h, w, new_h, labels, ov, v, sc, new_weight=wn)
