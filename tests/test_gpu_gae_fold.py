"""The split GAE folded into the loss rows launch (trlx_ppo_loss_rows_split_gae), the pipelined
schedule's two-launch step.

The reward r = score - beta*kl enters GAE (ppo_models.py:121-139, ppo_orchestrator.py:163-167)
linearly, so the split GAE of batch k+1 depends on nothing the loss rows of batch k produce:
it runs as the first workgroups of that launch, 256 threads wide in its arithmetic inside the
512-thread row workgroups (same partial sums, same fixed reduction order as its own launch).
The rows derive batch k's whitening coefficients (modeling.py:24-34) from the split record
themselves instead of a coefficient launch.  Everything here is pinned bit for bit against
the separate launches (GAE launch, coefficient launch, loss rows reading the coefficients).
"""
import ctypes

import pytest
import torch

import trlx_t5_amd as P
from oracle import ppo_oracle as orc

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
L = P._lib


def _batch(B, Tn, V, dtype, seed, lengths):
    g = torch.Generator().manual_seed(seed)
    d = dict(
        new_logits=(torch.randn(B, Tn, V, generator=g) * 2).to(dtype),
        labels=torch.randint(0, V, (B, Tn), generator=g),
        lp=-torch.rand(B, Tn, generator=g) * 8,
        ref_lp=-torch.rand(B, Tn, generator=g) * 8,
        old_values=torch.randn(B, Tn, generator=g),
        values=torch.randn(B, Tn, generator=g),
        scores=torch.rand(B, generator=g) * 24 - 12,
        lengths=None, mask=None)
    if lengths:
        Ls = torch.randint(1, Tn + 1, (B,), generator=g)
        d["lengths"] = Ls
        d["mask"] = (torch.arange(Tn)[None, :] < Ls[:, None]).long()
    return {k: (v.to(DEV) if v is not None else None) for k, v in d.items()}


def _split_set(B, Tn):
    f = dict(dtype=torch.float32, device=DEV)
    return dict(adv0=torch.full((B, Tn), 7.0, **f), adv_kl=torch.full((B, Tn), 7.0, **f),
                rew_kl=torch.full((B, Tn), 7.0, **f), rew_score=torch.full((B, Tn), 7.0, **f),
                stats=torch.zeros(8, dtype=torch.float64, device=DEV), coef=torch.zeros(4, **f))


class _Ctl:
    """A double-buffered controller record (control.PPOControlState without the class)."""

    def __init__(self, scale_mode, seed):
        g = torch.Generator().manual_seed(seed)
        st = torch.zeros(L.CTL_SLOTS, dtype=torch.float64)
        st[L.CTL_MEAN], st[L.CTL_VAR], st[L.CTL_STD], st[L.CTL_COUNT] = 0.3, 2.0, 1.4, 17.0
        st[L.CTL_REF_MEAN], st[L.CTL_REF_STD], st[L.CTL_REF_SET] = 0.1, 3.0, float(seed % 2)
        st[L.CTL_KL_COEF] = 0.05 + 0.01 * torch.rand(1, generator=g, dtype=torch.float64).item()
        self.buf = torch.stack([st, torch.zeros_like(st)]).to(DEV)
        self.scale_mode = scale_mode

    def score_ctl(self, gmom=None):
        return L.ScoreCtl(self.buf[0].data_ptr(), self.buf[1].data_ptr(), L.ptr(gmom), self.scale_mode, 10.0)


def _gae_args(x, sb, ctl, ws, lag, gmom):
    B, Tn = x["lp"].shape
    c = ctl.score_ctl(gmom) if ctl is not None else None
    return L.GaeSplitArgs(B, Tn, x["lp"].data_ptr(), x["ref_lp"].data_ptr(), x["old_values"].data_ptr(), L.F32,
                          x["scores"].data_ptr(), L.ptr(x["lengths"]), L.ptr(x["mask"]),
                          ctypes.pointer(c) if c is not None else None, 0.05, 0.99, 0.95,
                          sb["adv0"].data_ptr(), sb["adv_kl"].data_ptr(), sb["rew_kl"].data_ptr(),
                          sb["rew_score"].data_ptr(), sb["stats"].data_ptr(), int(lag), ws.data_ptr()), c


def _gae_launch(x, sb, ctl, ws, lag, gmom, s):
    B, Tn = x["lp"].shape
    c = ctl.score_ctl(gmom) if ctl is not None else None
    L.call("trlx_ppo_rollout_gae_split", B, Tn, x["lp"].data_ptr(), x["ref_lp"].data_ptr(),
           x["old_values"].data_ptr(), L.F32, x["scores"].data_ptr(), L.ptr(x["lengths"]), L.ptr(x["mask"]), c,
           0.05, 0.99, 0.95, sb["adv0"].data_ptr(), sb["adv_kl"].data_ptr(), sb["rew_kl"].data_ptr(),
           sb["rew_score"].data_ptr(), sb["stats"].data_ptr(), None, None, 0, int(lag), ws.data_ptr(), s, None)


class _Loss:
    """Outputs of one loss rows launch of batch x (split set sb, coefficients `coef`)."""

    def __init__(self, x):
        B, Tn, V = x["new_logits"].shape
        f = dict(dtype=torch.float32, device=DEV)
        self.lp_new, self.dvalues = torch.zeros(B, Tn, **f), torch.zeros(B, Tn, **f)
        self.rewards, self.returns = torch.zeros(B, Tn, **f), torch.zeros(B, Tn, **f)
        self.dx = P.grad_buffer_like(x["new_logits"])
        self.ws = torch.zeros(L.query("trlx_ppo_workspace_bytes", B, Tn), dtype=torch.uint8, device=DEV)

    def common(self, x, sb):
        B, Tn, V = x["new_logits"].shape
        nl = x["new_logits"]
        rows = (nl.data_ptr(), L.dtype_code(nl), B, Tn, V, nl.stride(0), nl.stride(1), x["labels"].data_ptr(),
                Tn, 1, x["lp"].data_ptr(), L.F32, sb["adv0"].data_ptr(), sb["adv_kl"].data_ptr(),
                sb["rew_kl"].data_ptr(), sb["rew_score"].data_ptr())
        vals = (sb["stats"].data_ptr() + 6 * 8, L.ptr(x["mask"]), x["values"].data_ptr(), L.F32,
                x["old_values"].data_ptr(), L.F32, self.rewards.data_ptr(), self.returns.data_ptr(), L.F32)
        grads = (0.2, 0.2, 1.0, self.lp_new.data_ptr(), self.dx.data_ptr(), self.dx.stride(0), self.dx.stride(1),
                 self.dvalues.data_ptr(), self.ws.data_ptr())
        return rows, vals, grads

    def outputs(self):
        return [self.lp_new, self.dvalues, self.rewards, self.returns, self.dx, self.ws]


def _snap(ts):
    torch.cuda.synchronize()
    return [t.clone().cpu() for t in ts]


def _assert_same(a, b, what):
    assert len(a) == len(b)
    for i, (u, v) in enumerate(zip(a, b)):
        assert torch.equal(u.view(torch.uint8) if u.dtype == torch.bfloat16 else u,
                           v.view(torch.uint8) if v.dtype == torch.bfloat16 else v), f"{what}: output {i}"


CASES = [  # (B, T, V, dtype): the split-residency row kernels host the GAE; the others run it standalone
    (128, 48, 50257, torch.bfloat16),   # C2: 9 + 4 vectors (long bf16 split)
    (37, 21, 32128, torch.bfloat16),    # T5/UL2 vocab: 6 + 2 (mid split), B % 4 != 0
    (9, 13, 50257, torch.float32),      # fp32 split (21 + 4)
    (6, 130, 1031, torch.bfloat16),     # all-VGPR rows (no split): standalone GAE, T > 64 (two scan chunks)
    (1100, 3, 257, torch.bfloat16),     # 275 GAE blocks: more block records than one reduction pass takes
]


@pytest.mark.parametrize("B,Tn,V,dtype", CASES)
@pytest.mark.parametrize("ctl_mode", [None, L.SCALE_NONE, L.SCALE_RUNNING, L.SCALE_REF, "lag"])
def test_folded_gae_and_derived_coef_match_separate_launches(B, Tn, V, dtype, ctl_mode):
    """Reference sequence: GAE(next) launch, coefficient launch (trlx_ppo_whiten_coef), loss
    rows reading the coefficients.  Folded: ONE trlx_ppo_loss_rows_split_gae launch.  Every
    output bit-identical: the next batch's adv0 / adv_kl / rew_kl / rew_score / split record /
    advanced controller record, and this batch's lp, dlogits, dvalues, rewards, returns,
    token records and the stored coefficients."""
    if (B > 200 or dtype == torch.float32) and ctl_mode not in (None, L.SCALE_RUNNING):
        pytest.skip("ctl variants covered at the other shapes")
    s = torch.cuda.current_stream(DEV).cuda_stream
    lengths = Tn > 1 and B < 200
    xk = _batch(B, Tn, V, dtype, 11 + B, lengths)       # batch k: its loss runs
    xn = _batch(B, Tn, V, dtype, 12 + B, lengths)       # batch k+1: its GAE runs
    sbk = _split_set(B, Tn)
    # batch k's split record (its own GAE, run once; only the record and A0 / Ak matter here)
    _gae_launch(xk, sbk, None, torch.zeros(L.query("trlx_ppo_workspace_bytes", B, Tn), dtype=torch.uint8,
                                           device=DEV), False, None, s)
    lag = ctl_mode == "lag"
    scale = L.SCALE_NONE if lag else ctl_mode
    gmom = torch.tensor([3.0, 40.0, 7.0, 0.0], dtype=torch.float64, device=DEV) if lag else None
    results = []
    for folded in (False, True):
        sbn = _split_set(B, Tn)
        ctl = _Ctl(scale, B) if ctl_mode is not None else None
        sbk["coef"].zero_()
        out = _Loss(xk)
        rows, vals, grads = out.common(xk, sbk)
        beta_state = ctl.buf[0].data_ptr() if ctl is not None else None
        if folded:
            args, _c = _gae_args(xn, sbn, ctl, out.ws, lag, gmom)
            L.call("trlx_ppo_loss_rows_split_gae", *rows, sbk["stats"].data_ptr(), 1, beta_state, 0.05,
                   sbk["coef"].data_ptr(), *vals, *grads, ctypes.byref(args), s, None)
        else:
            _gae_launch(xn, sbn, ctl, out.ws, lag, gmom, s)
            L.call("trlx_ppo_whiten_coef", sbk["stats"].data_ptr(), 1, beta_state, 0.05, sbk["coef"].data_ptr(), s)
            L.call("trlx_ppo_loss_rows_split", *rows, sbk["coef"].data_ptr(), *vals, *grads, s)
        results.append(_snap(out.outputs() + [sbn[k] for k in ("adv0", "adv_kl", "rew_kl", "rew_score", "stats")]
                             + [sbk["coef"]] + ([ctl.buf] if ctl is not None else [])))
    _assert_same(results[0], results[1], f"folded vs separate ({B}x{Tn}x{V} {dtype}, ctl {ctl_mode})")
    ws = results[1][5]
    assert int(ws.view(torch.int32)[:4].abs().sum()) == 0  # the GAE's arrival ticket re-armed
    assert torch.isfinite(results[1][0]).all()


def test_derived_coef_without_fold_and_second_loss():
    """Without a folded GAE the rows still derive and store the coefficients; a second loss
    on the same experience (ppo_epochs) reading them reproduces the first bit for bit."""
    B, Tn, V = 16, 48, 32128
    s = torch.cuda.current_stream(DEV).cuda_stream
    x = _batch(B, Tn, V, torch.bfloat16, 5, True)
    sb = _split_set(B, Tn)
    _gae_launch(x, sb, None, torch.zeros(L.query("trlx_ppo_workspace_bytes", B, Tn), dtype=torch.uint8, device=DEV),
                False, None, s)
    a = _Loss(x)
    rows, vals, grads = a.common(x, sb)
    L.call("trlx_ppo_loss_rows_split_gae", *rows, sb["stats"].data_ptr(), 0, None, 0.05, sb["coef"].data_ptr(),
           *vals, *grads, None, s, None)
    first = _snap(a.outputs())
    coef = sb["coef"].clone()
    ref = torch.zeros(4, dtype=torch.float32, device=DEV)
    L.call("trlx_ppo_whiten_coef", sb["stats"].data_ptr(), 0, None, 0.05, ref.data_ptr(), s)
    torch.cuda.synchronize()
    assert torch.equal(coef, ref)
    b = _Loss(x)
    rows, vals, grads = b.common(x, sb)
    L.call("trlx_ppo_loss_rows_split", *rows, sb["coef"].data_ptr(), *vals, *grads, s)
    _assert_same(first, _snap(b.outputs()), "derived vs stored coefficients")


def test_forced_streaming_rows_run_the_gae_standalone():
    """Row kernels that cannot host the GAE (here the streaming rows, forced by the tuning
    knob) launch it first: same bits as the hosted form."""
    B, Tn, V = 12, 20, 32128
    s = torch.cuda.current_stream(DEV).cuda_stream
    xk, xn = _batch(B, Tn, V, torch.bfloat16, 21, False), _batch(B, Tn, V, torch.bfloat16, 22, False)
    sbk = _split_set(B, Tn)
    _gae_launch(xk, sbk, None, torch.zeros(L.query("trlx_ppo_workspace_bytes", B, Tn), dtype=torch.uint8,
                                           device=DEV), False, None, s)
    res = []
    for variant in (0, 2):
        L.set_tuning("row_variant", variant)
        try:
            sbn = _split_set(B, Tn)
            out = _Loss(xk)
            rows, vals, grads = out.common(xk, sbk)
            args, _ = _gae_args(xn, sbn, None, out.ws, False, None)
            L.call("trlx_ppo_loss_rows_split_gae", *rows, sbk["stats"].data_ptr(), 1, None, 0.05,
                   sbk["coef"].data_ptr(), *vals, *grads, ctypes.byref(args), s, None)
            res.append(_snap([sbn[k] for k in ("adv0", "adv_kl", "stats")] + [out.rewards, out.returns]))
        finally:
            L.set_tuning("row_variant", 0)
    _assert_same(res[0], res[1], "streaming vs hosted GAE")


def test_fold_argument_checks():
    B, Tn, V = 8, 8, 1031
    s = torch.cuda.current_stream(DEV).cuda_stream
    x = _batch(B, Tn, V, torch.bfloat16, 1, False)
    sb = _split_set(B, Tn)
    out = _Loss(x)
    rows, vals, grads = out.common(x, sb)
    # the GAE writing the set these rows read
    args, _ = _gae_args(x, sb, None, out.ws, False, None)
    with pytest.raises(ValueError, match="other split buffer set"):
        L.call("trlx_ppo_loss_rows_split_gae", *rows, sb["stats"].data_ptr(), 1, None, 0.05, sb["coef"].data_ptr(),
               *vals, *grads, ctypes.byref(args), s, None)
    # a GAE of another batch shape sharing the workspace
    x2 = _batch(B + 1, Tn, V, torch.bfloat16, 2, False)
    args, _ = _gae_args(x2, _split_set(B + 1, Tn), None, out.ws, False, None)
    with pytest.raises(ValueError, match="cannot share"):
        L.call("trlx_ppo_loss_rows_split_gae", *rows, sb["stats"].data_ptr(), 1, None, 0.05, sb["coef"].data_ptr(),
               *vals, *grads, ctypes.byref(args), s, None)
    # rows reading beta from the state the GAE writes
    ctl = _Ctl(L.SCALE_NONE, 3)
    args, _ = _gae_args(x, _split_set(B, Tn), ctl, out.ws, False, None)
    with pytest.raises(ValueError, match="state_in"):
        L.call("trlx_ppo_loss_rows_split_gae", *rows, sb["stats"].data_ptr(), 1, ctl.buf[1].data_ptr(), 0.05,
               sb["coef"].data_ptr(), *vals, *grads, ctypes.byref(args), s, None)


@pytest.mark.parametrize("scale", [False, "ref", "running"])
def test_two_launch_pipeline_matches_serial(scale):
    """pipeline_step (GAE(k+1) inside the L rows(k) launch) vs step(split_beta=True), five
    batches with decoder-length masks and the device controller state: losses, stats,
    dlogits, dvalues, rewards, returns, final controller state bit-identical."""
    B, Tn, V = 24, 33, 32128
    g = torch.Generator().manual_seed(4)
    batches = []
    for i in range(5):
        logits = torch.randn(B, Tn, V, generator=g).to(torch.bfloat16)
        Ls = torch.randint(1, Tn + 1, (B,), generator=g)
        mask = (torch.arange(Tn)[None, :] < Ls[:, None]).long()
        ov = torch.randn(B, Tn, generator=g).masked_fill(mask == 0, 0)
        batches.append(dict(logits=logits, ref_logits=(logits.float() + 0.1 * torch.randn(B, Tn, V, generator=g))
                            .to(torch.bfloat16), new_logits=(logits.float() + 0.05 * torch.randn(B, Tn, V, generator=g))
                            .to(torch.bfloat16), labels=torch.randint(0, V, (B, Tn), generator=g), old_values=ov,
                            values=ov + 0.3 * torch.randn(B, Tn, generator=g), scores=torch.rand(B, generator=g) * 24 - 12,
                            lengths=Ls, mask=mask))
    res = {}
    for mode in ("serial", "pipelined"):
        cfg = P.PPOConfig(scale_reward=scale)
        ctl = P.PPOControlState.from_config(cfg, DEV, n_steps=B)
        hp = P.PPOHotPath(cfg, B, Tn, V, torch.bfloat16, DEV, kl_coef=0.05, ctl=ctl, defer_tail=True,
                          split_beta=True)
        outs = []

        def grab(o):
            hp.wait_stats()
            torch.cuda.synchronize()
            outs.append([t.float().cpu().clone() for t in o] + [hp.rewards.cpu().clone(), hp.returns.cpu().clone()])

        for x in batches:
            a = [x[k].to(DEV) for k in ("logits", "ref_logits", "new_logits", "labels", "old_values", "values",
                                        "scores")]
            kw = dict(lengths=x["lengths"].to(DEV), mask=x["mask"].to(DEV))
            if mode == "pipelined":
                o = hp.pipeline_step(*a, **kw)
                if o is not None:
                    grab(o)
            else:
                grab(hp.step(*a, **kw))
        if mode == "pipelined":
            grab(hp.pipeline_flush())
        hp.wait_stats()
        torch.cuda.synchronize()
        res[mode] = (outs, ctl.state.cpu().clone())
    (ser, ser_st), (pip, pip_st) = res["serial"], res["pipelined"]
    assert len(ser) == len(pip) == len(batches)
    for i, (a, b) in enumerate(zip(ser, pip)):
        for j, (u, v) in enumerate(zip(a, b)):
            assert torch.equal(u, v), f"batch {i} output {j}"
    assert torch.equal(ser_st, pip_st)


@pytest.mark.parametrize("i", range(10))
def test_two_launch_pipeline_fuzz(i):
    """Seeded random cases of the two-launch pipelined step vs step(split_beta=True): B in
    [1, 70], T in [1, 140] (one to three GAE scan chunks), V from 2 to 60000 (bf16 / fp32,
    hosting split kernels, all-VGPR and streaming rows alike), decoder lengths or none, every
    controller mode or host beta, global or rank-local loss normaliser (no process group),
    deferred or in-stream loss tails; three batches: every output and the controller record
    bit-identical."""
    import random
    rnd = random.Random(7700 + i)
    B, Tn = rnd.randint(1, 70), rnd.choice([1, 5, 48, 64, 65, 140])
    V = [50257, 32128, 2][i] if i < 3 else rnd.randint(2, 60000)
    B = max(1, min(B, 6_000_000 // (Tn * V)))  # <= 6 M logits per tensor (CPU generation)
    dt = torch.float32 if i % 3 == 2 else torch.bfloat16
    lengths = i % 2 == 1 and Tn > 1
    scale = [None, False, "ref", "running"][i % 4]
    defer = i % 5 != 0
    g = torch.Generator().manual_seed(i)
    batches = []
    for _ in range(3):
        logits = torch.randn(B, Tn, V, generator=g).to(dt)
        Ls = torch.randint(1, Tn + 1, (B,), generator=g) if lengths else None
        mask = (torch.arange(Tn)[None, :] < Ls[:, None]).long() if lengths else None
        ov = torch.randn(B, Tn, generator=g)
        if lengths:
            ov = ov.masked_fill(mask == 0, 0)
        batches.append([logits, (logits.float() + 0.1 * torch.randn(B, Tn, V, generator=g)).to(dt),
                        (logits.float() + 0.05 * torch.randn(B, Tn, V, generator=g)).to(dt),
                        torch.randint(0, V, (B, Tn), generator=g), ov, ov + 0.3 * torch.randn(B, Tn, generator=g),
                        torch.rand(B, generator=g) * 24 - 12, Ls, mask])
    res = {}
    for mode in ("serial", "pipelined"):
        cfg = P.PPOConfig(scale_reward=scale if scale is not None else False)
        ctl = P.PPOControlState.from_config(cfg, DEV, n_steps=B) if scale is not None else None
        hp = P.PPOHotPath(cfg, B, Tn, V, dt, DEV, kl_coef=0.05, ctl=ctl, defer_tail=defer, split_beta=True)
        outs = []

        def grab(o):
            hp.wait_stats()
            torch.cuda.synchronize()
            outs.append([t.float().cpu().clone() for t in o] + [hp.rewards.cpu().clone(), hp.returns.cpu().clone()])

        for x in batches:
            a = [t.to(DEV) for t in x[:7]]
            kw = dict(lengths=x[7].to(DEV) if x[7] is not None else None, mask=x[8].to(DEV) if x[8] is not None else None)
            if mode == "pipelined":
                o = hp.pipeline_step(*a, **kw)
                if o is not None:
                    grab(o)
            else:
                grab(hp.step(*a, **kw))
        if mode == "pipelined":
            grab(hp.pipeline_flush())
        hp.wait_stats()
        torch.cuda.synchronize()
        res[mode] = (outs, ctl.state.cpu().clone() if ctl is not None else None)
    (ser, ser_st), (pip, pip_st) = res["serial"], res["pipelined"]
    assert len(ser) == len(pip) == 3
    for k, (a, b) in enumerate(zip(ser, pip)):
        for j, (u, v) in enumerate(zip(a, b)):
            assert torch.equal(u, v), f"case {i} (B {B} T {Tn} V {V} {dt}): batch {k} output {j}"
    if ser_st is not None:
        assert torch.equal(ser_st, pip_st)
    # the serial split step itself vs the oracle on the first batch (fp32 association only)
    x = batches[0]
    ref = orc.ppo_step_reference(x[0].float(), x[1].float(), x[2].float(), x[3], x[4], x[5], x[6],
                                 kl_coef=0.05, lengths=x[7], mask=x[8]) if scale is None else None
    if ref is not None:
        torch.testing.assert_close(ser[0][0].reshape(()), ref["loss"], rtol=1e-4, atol=1e-5)
