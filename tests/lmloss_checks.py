"""Parity checks for the fused lm_head loss side (§8f-2; csrc/lmhead_loss.hip) that can see the
softmax half of the gradients.

With p = softmax(h·Wᵀ), g_t = d loss / d lp_t and E_t = Σ_v p_tv·W_v (modeling.py:37-41 after the
lm_head of ppo_models.py:640 / :274, differentiated as accelerate_ppo_model.py:96-118 does):

    dh_t = g_t·(W[y_t] − E_t)        dW_v = Σ_t g_t·(1[y_t = v] − p_tv)·h_t

A whole-matrix Frobenius norm is dominated by the label rows of dW (the g_t·h_t terms) and by
W[y_t] in dh, so it cannot see the −p·h / E halves at GPT-2 / T5 vocab sizes (dropping dW's
whole −p·h term moves it by ~1 % at V = 50257).  These checks look at each half by itself:

  * E per token, relative to ‖E_t‖ (the forward's saved E, or O / l);
  * dW on the rows that are no token's label (only −g·p·h terms) and on the label rows, each
    as an aggregate relative norm, plus the max over rows of the per-row relative error;
  * dh per token, relative to |g_t|·‖E_t‖ (the E term it carries) plus its output rounding.

Tolerances follow from the arithmetic: the second products take P and dS as bf16 (8 bits of
significand: unit roundoff u = 2^-8, the errors of independent terms add in quadrature to
~u/√3 ≈ 1.6e-3 rms relative), the outputs may be rounded to bf16 once more (another ~1.6e-3),
everything else accumulates in fp32.  So an aggregate or per-token relative error is
~1.6-2.3e-3 and is held to BF16_REL = 2u = 2^-7 (the two roundings at their bound); one row of
H elements scatters around that by ~1/√H more and is held to ROW_REL = 4u = 2^-6.  A 10 %
error of either half is 0.1.  tests/test_lmloss_sensitivity.py shows on the CPU that every check passes a
bf16-rounded emulation of the kernels' arithmetic and fails when dW's −p·h term or E is
zeroed or off by 10 %.  Test infrastructure only.
"""
import torch

BF16_REL = 2.0 ** -7
ROW_REL = 2.0 ** -6


def row_rel(got, want):
    """Per-row ‖got − want‖ / ‖want‖ in fp64 (rows of exactly zero reference norm: absolute)."""
    g, w = got.double(), want.double()
    return (g - w).norm(dim=-1) / w.norm(dim=-1).clamp_min(1e-300)


def e_errors(e_got, e_want):
    """E_t per token: the max of ‖E_t − E64_t‖ / ‖E64_t‖."""
    return {"e_token_max": float(row_rel(e_got, e_want).max())}


def label_rows(labels, V):
    """bool [V]: vocab rows that are some (valid, unmasked) token's label."""
    y = labels.reshape(-1).cpu()
    y = y[(y >= 0) & (y < V)]
    m = torch.zeros(V, dtype=torch.bool)
    m[y] = True
    return m


def dw_errors(dw_got, dw_want, labels):
    """dW split by rows: aggregate relative norm over the non-label rows and over the label
    rows, and the max per-row relative error.  `labels`: the labels of the tokens that
    contribute (masked tokens excluded)."""
    g, w = dw_got.double().cpu(), dw_want.double().cpu()
    lab = label_rows(labels, w.shape[0])
    d = g - w
    out = {"dw_row_max": float(row_rel(g, w).max())}
    out["dw_nonlabel_rel"] = float(d[~lab].norm() / w[~lab].norm().clamp_min(1e-300)) if (~lab).any() else 0.0
    out["dw_label_rel"] = float(d[lab].norm() / w[lab].norm().clamp_min(1e-300)) if lab.any() else 0.0
    return out


def dh_errors(dh_got, dh_want, g, e_want, fp32_out):
    """dh per token: max over tokens with g ≠ 0 of ‖dh_t − dh64_t‖ / (|g_t|·‖E64_t‖ + ρ·‖dh64_t‖).
    The E term's error is what is checked; ρ covers the output rounding: 1 for bf16 outputs
    (their 2^-9 rounding of ‖dh_t‖ can exceed the whole E term of a flat softmax, so only E's
    own check sees E there), 2^-12 for fp32 outputs (the fp32 subtraction W[y] − E is exact
    to ~1e-7 of ‖dh‖), which makes this check see a 10 % error of E at any softmax."""
    gd = g.double().reshape(-1).cpu()
    rho = 2.0 ** -12 if fp32_out else 1.0
    scale = gd.abs() * e_want.double().cpu().norm(dim=-1) + rho * dh_want.double().cpu().norm(dim=-1)
    err = (dh_got.double().cpu() - dh_want.double().cpu()).norm(dim=-1)
    live = gd != 0
    return {"dh_token_max": float((err[live] / scale[live].clamp_min(1e-300)).max()) if live.any() else 0.0}


LIMITS = {"e_token_max": BF16_REL, "dw_nonlabel_rel": BF16_REL, "dw_label_rel": BF16_REL, "dw_row_max": ROW_REL,
          "dh_token_max": BF16_REL}


def failures(errs):
    """The checks of `errs` over their limits (empty = pass)."""
    return {k: v for k, v in errs.items() if not v <= LIMITS[k]}


def assert_within(errs, what=""):
    bad = failures(errs)
    assert not bad, f"{what}: {bad} (limits {LIMITS}; all {errs})"


def fp64_truth(h, w, y, gout):
    """lp, lse, E, dh, dW of Σ_t gout_t·lp_t in fp64 from the (bf16) operands, on their device."""
    hd, wd = h.double(), w.double()
    s = hd @ wd.t()
    lse = torch.logsumexp(s, -1)
    p = torch.exp(s - lse[:, None])
    lp = s.gather(-1, y[:, None]).squeeze(-1) - lse
    e = p @ wd
    gd = gout.double()
    dh = gd[:, None] * (wd[y] - e)
    ds = -gd[:, None] * p
    ds[torch.arange(len(y), device=ds.device), y] += gd
    dw = ds.t() @ hd
    return dict(lp=lp, lse=lse, e=e, dh=dh, dw=dw)


def peaked_operands(N, H, V, seed, wscale=0.12, hscale=1.0, label_boost=None):
    """bf16 (h, W, y) whose softmax is NOT flat: logits of std σ ~ wscale·hscale·√H (~3.3 at
    H = 768) and each token's label logit raised by label_boost (h_t += c·W[y_t]/‖W[y_t]‖²;
    default ln V + σ²/2, the log of the other logits' Σexp, so p_label spreads around 1/2),
    SURVEY §8d's "peaked" variant."""
    import math
    if label_boost is None:
        label_boost = math.log(V) + (wscale * hscale) ** 2 * H / 2
    g = torch.Generator().manual_seed(seed)
    w = (torch.randn(V, H, generator=g) * wscale).to(torch.bfloat16)
    y = torch.randint(0, V, (N,), generator=g)
    h = torch.randn(N, H, generator=g) * hscale
    wy = w.float()[y]
    h = h + label_boost * wy / (wy * wy).sum(-1, keepdim=True)
    return h.to(torch.bfloat16), w, y
