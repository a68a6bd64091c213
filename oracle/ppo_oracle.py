"""CPU ORACLE — test infrastructure only, never part of the product path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
It restates, op for op with stock PyTorch CPU ops, the arithmetic of the reference's
hot path (danyang-rainbow/trlx-t5; every function cites the file:line it follows), so
that (a) it reproduces the reference bit-for-bit on the same inputs — pinned against the
golden fixtures in tests/golden/, which were produced by importing the reference itself
(tests/golden/make_golden.py) — and (b) it can run at full bench sizes on the GPU box,
where the reference does not exist, as the parity checker and the timed CPU baseline.
"""
from functools import reduce
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist
import torch.nn.functional as F


# ------------------------------------------------------------------ trlx/utils/modeling.py
def global_statistics(xs):
    """modeling.py:9-21 — two all-reduces; buffer in xs.dtype; biased variance."""
    buf = torch.tensor([xs.sum(), xs.numel()], device=xs.device)
    dist.all_reduce(buf, dist.ReduceOp.SUM)
    total, count = buf
    mean = total / count
    sq = torch.sum((xs - mean) ** 2)
    dist.all_reduce(sq, dist.ReduceOp.SUM)
    return mean, sq / count, count


def whiten(xs, shift_mean=True, distributed=True):
    """modeling.py:24-34."""
    if distributed and dist.is_initialized():
        mean, var, _ = global_statistics(xs)
    else:
        var, mean = torch.var_mean(xs)
    out = (xs - mean) * torch.rsqrt(var + 1e-8)
    if not shift_mean:
        out += mean
    return out


def logprobs_from_logits(logits, labels):
    """modeling.py:37-41 — full log-softmax over V, then gather."""
    lsm = F.log_softmax(logits, dim=-1)
    return torch.gather(lsm, dim=-1, index=labels.unsqueeze(-1)).squeeze(-1)


class RunningMoments:
    """modeling.py:72-104."""

    def __init__(self):
        self.mean, self.std, self.var, self.count = 0, 1, 1, 1e-24

    def update(self, xs):
        if dist.is_initialized():
            xs_mean, xs_var, xs_count = global_statistics(xs)
        else:
            xs_count = xs.numel()
            xs_var, xs_mean = torch.var_mean(xs, unbiased=False)
        delta = xs_mean - self.mean
        tot = self.count + xs_count
        new_sum = xs_var * xs_count
        old_sum = self.var * self.count + delta ** 2 * self.count * xs_count / tot
        self.mean += delta * xs_count / tot
        self.var = (old_sum + new_sum) / tot
        self.std = (self.var * tot / (tot - 1)).sqrt()
        self.count = tot
        return xs_mean, (xs_var * xs_count / (xs_count - 1)).sqrt()


# ------------------------------------------------------------------ trlx/model/nn/ppo_models.py
class AdaptiveKLController:
    """ppo_models.py:26-44."""

    def __init__(self, init_kl_coef, target, horizon):
        self.value, self.target, self.horizon = init_kl_coef, target, horizon

    def update(self, current, n_steps):
        self.value *= 1 + np.clip(current / self.target - 1, -0.2, 0.2) * n_steps / self.horizon


class FixedKLController:
    """ppo_models.py:47-58."""

    def __init__(self, kl_coef):
        self.value = kl_coef

    def update(self, current, n_steps):
        pass


def gae(values, rewards, response_length, gamma=1, lam=0.95, use_whitening=True):
    """ppo_models.py:121-139 — the per-t reverse loop, then whiten(advantages)."""
    last = 0
    rev = []
    for t in reversed(range(response_length)):
        nxt = values[:, t + 1] if t < response_length - 1 else 0.0
        delta = rewards[:, t] + gamma * nxt - values[:, t]
        last = delta + gamma * lam * last
        rev.append(last)
    adv = torch.stack(rev[::-1], dim=1)
    ret = adv + values
    if use_whitening:
        adv = whiten(adv)
    return adv.detach(), ret


def _flatten(d, parent="", sep="/"):
    out = {}
    for k, v in d.items():
        key = parent + sep + k if parent else k
        if isinstance(v, dict):
            out.update(_flatten(v, key, sep))
        else:
            out[key] = v
    return out


def ppo_loss(logprobs, values, old_logprobs, old_values, advantages, returns, mask,
             cliprange=0.2, cliprange_value=0.2, vf_coef=1):
    """ppo_models.py:141-199 (same ops, same order; stats flattened with '/')."""
    vclip = torch.clamp(values, old_values - cliprange_value, old_values + cliprange_value)
    vl1 = (values - returns) ** 2
    vl2 = (vclip - returns) ** 2
    vf_loss = 0.5 * torch.sum(torch.max(vl1, vl2) * mask) / mask.sum()
    vf_clipfrac = torch.mean((vl2 > vl1).float())
    log_ratio = (logprobs - old_logprobs) * mask
    ratio = torch.exp(log_ratio)
    with torch.no_grad():
        approx_kl = torch.mean((ratio - 1) - log_ratio)
    pg1 = -advantages * ratio
    pg2 = -advantages * torch.clamp(ratio, 1.0 - cliprange, 1.0 + cliprange)
    pg_loss = torch.sum(torch.max(pg1, pg2) * mask) / mask.sum()
    pg_clipfrac = torch.mean((pg2 > pg1).float())
    loss = pg_loss + vf_coef * vf_loss
    stats = {
        "losses": {"total_loss": loss.item(), "policy_loss": pg_loss.item(), "value_loss": vf_loss.item()},
        "values": {"mean_old_values": torch.mean(old_values), "var_old_values": torch.var(old_values),
                   "mean_values": torch.mean(values), "values_error": torch.mean((values - returns) ** 2),
                   "clipfrac": vf_clipfrac},
        "policy": {"approx_kl": approx_kl.item(), "clipfrac": pg_clipfrac.item()},
        "returns": {"mean": torch.mean(returns), "var": torch.var(returns)},
        "ratio": (ratio * mask).sum() / mask.sum(),
    }
    return loss, _flatten(stats)


# ------------------------------------------------------------------ trlx/orchestrator/ppo_orchestrator.py
def prepare_scores(scores, running, scale_reward, cliprange_reward, ref_std=None):
    """ppo_orchestrator.py:96-112 (ref_mean/ref_std bookkeeping left to the caller)."""
    m, s = running.update(scores)
    if scale_reward == "running":
        scores /= running.std
    elif scale_reward == "ref":
        scores /= ref_std
    if cliprange_reward:
        scores = torch.clip(scores, -cliprange_reward, cliprange_reward)
    return scores, m, s


class ScoreControl:
    """The orchestrator's score bookkeeping, ppo_orchestrator.py:48-49 (init from the method
    config) and :96-112 (first-batch ref stats, RunningMoments.update, scale, clip)."""

    def __init__(self, scale_reward=False, cliprange_reward=10, ref_mean=None, ref_std=None):
        self.running = RunningMoments()
        self.ref_mean, self.ref_std = ref_mean, ref_std
        self.scale_reward, self.cliprange_reward = scale_reward, cliprange_reward

    def __call__(self, scores):
        scores = scores.clone()
        if self.ref_mean is None:
            self.ref_mean, self.ref_std = scores.mean(), scores.std()
        batch_mean, batch_std = self.running.update(scores)
        if self.scale_reward == "running":
            scores /= self.running.std
        elif self.scale_reward == "ref":
            scores /= self.ref_std
        if self.cliprange_reward:
            scores = torch.clip(scores, -self.cliprange_reward, self.cliprange_reward)
        return scores, batch_mean, batch_std


def store_padded(x, lengths):
    """A per-token [B, T] tensor as the padded store returns it (ppo_pipeline.py:47-65): each
    element covers its own decoder length and the collate pads with 0.0 (lengths None: as is)."""
    if lengths is None:
        return x
    return x.masked_fill(torch.arange(x.shape[1], device=x.device)[None, :] >= lengths[:, None], 0)


def kl_penalty_rewards(logprobs, ref_logprobs, kl_coef, scores=None, lengths=None):
    """ppo_orchestrator.py:164-167.  With `lengths` (build extension for the padded store,
    ppo_pipeline.py:47-65): the score goes to column lengths[b]-1 and later columns are 0."""
    kls = logprobs - ref_logprobs
    rewards = (-kl_coef * kls).clone()
    if lengths is None:
        if scores is not None:
            rewards[:, -1] += scores
        return rewards
    T = rewards.shape[1]
    pad = torch.arange(T, device=rewards.device)[None, :] >= lengths[:, None]
    rewards = rewards.masked_fill(pad, 0)
    if scores is not None:
        rows = torch.arange(rewards.shape[0], device=rewards.device)
        rewards[rows, lengths - 1] += scores
    return rewards


# ------------------------------------------------------------------ the fused step, restated
def ppo_step_reference(logits, ref_logits, new_logits, labels, old_values, values, scores, cfg_kwargs=None,
                       kl_coef=0.05, lengths=None, mask=None, distributed=False):
    """The bench step with the reference's own ops: experience (ppo_orchestrator.py:154-167)
    then the loss side of accelerate_ppo_model.py:88-126 with autograd backward.  Runs in
    the inputs' dtype (fp32 on bf16-quantised inputs = the parity oracle; native bf16 = the
    reference T5/UL2 path, the timed CPU baseline).  old_lp for the loss = experience lp.
    new_lp is returned at every position; the build's loss rows write 0 where mask == 0
    (nothing depends on it there, so those rows are not read)."""
    cfg = dict(gamma=1, lam=0.95, cliprange=0.2, cliprange_value=0.2, vf_coef=1)
    cfg.update(cfg_kwargs or {})
    B, T = labels.shape
    with torch.no_grad():
        lp = logprobs_from_logits(logits, labels)
        ref_lp = logprobs_from_logits(ref_logits, labels)
        ov = old_values
        if lengths is not None:
            # a ragged batch: the padded store's tensors (ppo_pipeline.py:47-65) — each element's
            # logprobs / values cover its own decoder length, the collate pads them with 0.0
            lp, ref_lp, ov = store_padded(lp, lengths), store_padded(ref_lp, lengths), store_padded(ov, lengths)
        rewards = kl_penalty_rewards(lp, ref_lp, kl_coef, scores, lengths)
    if mask is None:
        mask = torch.ones((B, T), dtype=torch.long, device=labels.device)
    adv, ret = gae(ov, rewards, T, cfg["gamma"], cfg["lam"], use_whitening=True)
    x = new_logits.detach().clone().requires_grad_(True)
    v = values.detach().clone().requires_grad_(True)
    new_lp = logprobs_from_logits(x, labels)
    loss, stats = ppo_loss(new_lp, v, lp, ov, adv, ret, mask, cfg["cliprange"], cfg["cliprange_value"],
                           cfg["vf_coef"])
    loss.backward()
    return dict(lp=lp, ref_lp=ref_lp, rewards=rewards, adv=adv, returns=ret, new_lp=new_lp.detach(), loss=loss.detach(),
                stats=stats, dlogits=x.grad, dvalues=v.grad)


# ------------------------------------------------------------------ trlx/model/nn/ilql_models.py
def ilql_loss(logits, qs, target_qs, vs, input_ids, attention_mask, rewards, actions_ixs, dones,
              tau=0.7, gamma=0.99, cql_scale=0.1, awac_scale=1):
    """ilql_models.py:52-116 (ILQLConfig.loss), same ops and order."""
    actions = input_ids[:, 1:].gather(dim=1, index=actions_ixs).unsqueeze(-1)
    bsize, ntokens, dsize = logits.shape
    Q = [q.gather(-1, actions).squeeze(-1) for q in qs]
    tQs = [q.gather(-1, actions).squeeze(-1).detach() for q in target_qs]
    tQ = reduce(torch.minimum, tQs)
    term = dones[:, :-1]
    n_nt = max(1, term.sum())
    V = vs[:, :-1].squeeze()
    Vnext = vs[:, 1:].squeeze() * dones[:, 1:]
    Q_ = rewards + gamma * Vnext.detach()
    loss_q = sum(((Qi - Q_) * term).pow(2).sum() / n_nt for Qi in Q)
    tQ = tQ.detach()
    loss_v = (((tQ >= V).int() * tau * (tQ - V).pow(2) + (tQ < V).int() * (1 - tau) * (tQ - V).pow(2))
              * term).sum() / n_nt
    nact = qs[0].shape[1]

    def cql(q):
        ce = F.cross_entropy(q.reshape(-1, dsize), actions.reshape(-1), reduction="none")
        return (ce.reshape(bsize, nact) * term).sum() / n_nt

    loss_cql = sum(cql(q) for q in qs)
    loss_awac = (F.cross_entropy(logits[:, :-1, :].reshape(-1, dsize), input_ids[:, 1:].reshape(-1),
                                 reduction="none").reshape(bsize, ntokens - 1)
                 * attention_mask[:, 1:]).sum() / attention_mask[:, 1:].sum()
    loss = loss_q + loss_v + cql_scale * loss_cql + awac_scale * loss_awac
    stats = {"losses/loss": loss, "losses/loss_q": loss_q, "losses/loss_v": loss_v,
             "losses/loss_cql": loss_cql, "losses/loss_awac": loss_awac}
    return loss, stats


# ------------------------------------------------------------------ trlx/pipeline/ppo_pipeline.py
def ppo_collate(elems, pad_token_id):
    """ppo_pipeline.py:40-66 — queries left-padded (flip, pad_sequence, flip), the rest
    right-padded (tokens with pad_token_id, floats with 0.0).  elems: objects with
    query_tensor, response_tensor, logprobs, values, rewards."""
    from torch.nn.utils.rnn import pad_sequence
    return (
        pad_sequence([e.query_tensor.flip(0) for e in elems], padding_value=pad_token_id, batch_first=True).flip(1),
        pad_sequence([e.response_tensor for e in elems], padding_value=pad_token_id, batch_first=True),
        pad_sequence([e.logprobs for e in elems], padding_value=0.0, batch_first=True),
        pad_sequence([e.values for e in elems], padding_value=0.0, batch_first=True),
        pad_sequence([e.rewards for e in elems], padding_value=0.0, batch_first=True),
    )


# ------------------------------------------------------------------ ilql_models.py:24-28 (= utils/__init__.py:107-116)
def topk_mask(xs, k):
    """Scores outside each row's top k -> -inf; entries equal to the k-th value are kept."""
    if k > xs.shape[-1]:
        return xs
    mintop = torch.topk(xs, k)[0][:, -1].unsqueeze(-1)
    return torch.where(xs < mintop, -np.inf * torch.ones_like(xs, dtype=xs.dtype), xs)


# ------------------------------------------------------------------ accelerate_ppo_model.py:18-25,63-76
def shift_tokens_right(ids, pad_token_id=0, decoder_start_token_id=0):
    """Decoder inputs of the seq2seq forward: the start id, then the ids moved one column right;
    every -100 (the start id included) becomes pad_token_id.  Empty responses (T = 0) raise
    IndexError like the reference's column-0 assignment."""
    if ids.dim() != 2 or ids.shape[1] == 0:
        raise IndexError("shift_tokens_right needs [B, T >= 1] ids")
    first = torch.full((ids.shape[0], 1), decoder_start_token_id, dtype=ids.dtype)
    out = torch.cat([first, ids[:, :-1]], dim=1)
    return torch.where(out == -100, torch.full_like(out, pad_token_id), out)


def get_model_inputs(query_tensors, response_tensors):
    """(encoder input, labels, decoder inputs) of AcceleratePPOModel.get_model_inputs."""
    return query_tensors, response_tensors, shift_tokens_right(response_tensors)
