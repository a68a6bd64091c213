"""CPU: the §8f-2 loss-side parity checks (tests/lmloss_checks.py, used by
tests/test_gpu_lmhead_loss.py) can fail.

On flat and peaked operands, in fp64 on the CPU:
  * an emulation of the fused kernels' arithmetic (csrc/lmhead_loss.hip: fp32 logits from the
    bf16 operands, P = exp(S − m) and dS = g·(1[y = v] − p) rounded to bf16 before the second
    products, fp32 accumulation, bf16 or fp32 outputs) passes every check;
  * each mutation a broken kernel could produce fails the checks named for it:
      - dW's −p·h term zeroed or scaled by 0.9 (a bad split partial / reduce / tail block),
      - E = Σ p·W zeroed or scaled by 1.1 / 0.8 (a bad O product or combine),
      - the last, partial 64-row vocab block of dW zeroed (50257 = 785·64 + 17 at GPT-2's V).
No GPU, no oracle: the checks and their limits are what is under test.
"""
import pytest
import torch

import lmloss_checks as C


def _bf(x):
    return x.to(torch.bfloat16).double()


def _emulate(h, w, y, g, mutate=None, out_bf16=True, plan="recompute"):
    """The kernels' arithmetic (fp32 products of bf16 operands, bf16 P / dS), with an optional
    mutation.  Returns (E, dh, dW) in fp64 holding the emulated values.  plan "saved_p": dW as
    k_lmloss_dwp forms it (one vocab split here): the forward's bf16 P = exp(S − m) with each
    token's label entry replaced by bf16(−(1 − p_y)/e'), times the bf16 scaled rows
    hq = −g·e'·h, e' = e^(m − lse)."""
    hf, wf = h.float(), w.float()
    s = hf @ wf.t()                                    # fp32 MFMA accumulation
    m = s.max(-1, keepdim=True).values                  # the forward's exponent offset
    pf = torch.exp(s - m)
    l = pf.sum(-1, keepdim=True)
    o = _bf(pf) @ wf.double()                           # P in bf16 for O += Wᵀ·P
    e = (o / l.double()).float()
    if mutate == "e_zero":
        e = torch.zeros_like(e)
    elif mutate == "e_x1.1":
        e = e * 1.1
    elif mutate == "e_x0.8":
        e = e * 0.8
    dh = g[:, None] * (wf[y] - e)                       # the combine, fp32
    lse = m + torch.log(l)
    p = torch.exp(s - lse)                              # the dW kernel's recomputed p
    k = {"pw_zero": 0.0, "pw_x0.9": 0.9}.get(mutate, 1.0)
    if plan == "saved_p":
        ep = torch.exp(m - lse)                          # e' (one split: m is the split's offset)
        a_op = pf * k
        py = p[torch.arange(len(y)), y]
        a_op[torch.arange(len(y)), y] = -(1.0 - py) / ep[:, 0]
        hq = -g[:, None] * ep * hf
        dw = (_bf(a_op).t() @ _bf(hq)).float()
    else:
        ds = -g[:, None] * p * k
        ds[torch.arange(len(y)), y] += g
        dw = (_bf(ds).t() @ hf.double()).float()
    if mutate == "tail_block_zero":
        V = w.shape[0]
        dw[(V // 64) * 64:] = 0.0
    if out_bf16:
        dh, dw = dh.bfloat16(), dw.bfloat16()
    return e.double(), dh.double(), dw.double()


def _operands(kind, N, H, V, seed):
    if kind == "flat":
        g = torch.Generator().manual_seed(seed)
        h = torch.randn(N, H, generator=g).to(torch.bfloat16)
        w = (torch.randn(V, H, generator=g) * 0.05).to(torch.bfloat16)
        y = torch.randint(0, V, (N,), generator=g)
        return h, w, y
    return C.peaked_operands(N, H, V, seed, wscale=3.3 / H ** 0.5)


def _errors(h, w, y, g, mutate, out_bf16, plan="recompute"):
    t = C.fp64_truth(h, w, y, g)
    e, dh, dw = _emulate(h, w, y, g.float(), mutate, out_bf16, plan)
    errs = C.e_errors(e, t["e"])
    errs.update(C.dw_errors(dw, t["dw"], y))
    errs.update(C.dh_errors(dh, t["dh"], g, t["e"], fp32_out=not out_bf16))
    return errs


CASES = [("flat", 256, 128, 3000), ("peaked", 256, 128, 3000), ("flat", 96, 64, 50257), ("peaked", 96, 64, 50257)]


@pytest.mark.parametrize("kind,N,H,V", CASES)
@pytest.mark.parametrize("out_bf16", [True, False])
@pytest.mark.parametrize("plan", ["recompute", "saved_p"])
def test_checks_pass_the_kernels_arithmetic(kind, N, H, V, out_bf16, plan):
    h, w, y = _operands(kind, N, H, V, N + V)
    g = torch.randn(N, generator=torch.Generator().manual_seed(1))
    errs = _errors(h, w, y, g, None, out_bf16, plan)
    C.assert_within(errs, f"emulated kernels, {kind}")
    # the margin is real: the emulation sits well inside every limit
    assert all(v < 0.6 * C.LIMITS[k] for k, v in errs.items()), errs


# mutation -> the checks that must fail for it (on the operand kinds listed)
MUST_FAIL = {
    "pw_zero": {"flat": ["dw_nonlabel_rel", "dw_row_max"], "peaked": ["dw_nonlabel_rel", "dw_label_rel", "dw_row_max"]},
    "pw_x0.9": {"flat": ["dw_nonlabel_rel", "dw_row_max"], "peaked": ["dw_nonlabel_rel", "dw_label_rel", "dw_row_max"]},
    "tail_block_zero": {"flat": ["dw_row_max"], "peaked": ["dw_row_max"]},
    "e_zero": {"flat": ["e_token_max", "dh_token_max"], "peaked": ["e_token_max", "dh_token_max"]},
    "e_x1.1": {"flat": ["e_token_max"], "peaked": ["e_token_max", "dh_token_max"]},
    "e_x0.8": {"flat": ["e_token_max"], "peaked": ["e_token_max", "dh_token_max"]},
}


@pytest.mark.parametrize("kind,N,H,V", CASES)
@pytest.mark.parametrize("mutate", sorted(MUST_FAIL))
@pytest.mark.parametrize("out_bf16", [True, False])
def test_checks_fail_broken_kernels(kind, N, H, V, mutate, out_bf16):
    h, w, y = _operands(kind, N, H, V, N + V)
    g = torch.randn(N, generator=torch.Generator().manual_seed(1))
    bad = C.failures(_errors(h, w, y, g, mutate, out_bf16))
    want = set(MUST_FAIL[mutate][kind])
    if not out_bf16 and mutate.startswith("e_"):
        want.add("dh_token_max")  # fp32 outputs: dh's own check sees E at any softmax
    assert want <= set(bad), f"{mutate} on {kind} V={V}: failed {sorted(bad)}, expected {sorted(want)}"
