#!/usr/bin/env python3
"""Loss-side A/B: the PPO policy update from the policy's last hidden states.

  gemm   the unfused route the reference takes (accelerate_ppo_model.py:96-118): hipBLASLt
         lm_head -> bf16 logits [N, V]; the fused loss rows (one read of each logits row, one
         dlogits write: PPOHotPath.policy_loss); hipBLASLt dh = dlogits·W and dW = dlogitsᵀ·h
  fused  PPOHotPath.policy_loss_from_hidden: csrc/lmhead_loss.hip (flash-style forward with the
         O = Σ P·W accumulation, per-token combine, dW pass recomputing the logits tiles) — no
         [N, V] tensor in HBM

Both routes run after the same experience step (GAE, whitening record) and write the same
outputs (loss + stats via the loss tail, dvalues, d hidden, d lm_head weight in bf16).
Interleaved rounds; HIP-event time per call (median), TFLOP/s against the 4·N·V·H·2 flops
the fused route executes (the unfused route's 3 GEMMs are 3·N·V·H·2).

  python tools/lossside_bench.py [--config c2|c3] [--iters 20] [--rounds 3] [--routes gemm,fused,fused_recompute]

  (fused = the default saved-P plan: the forward stores its bf16 P tiles, the dW pass reads them
  back; fused_recompute = the dW pass recomputing the logits tiles)
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {"c2": (128, 48, 50257, 768, False), "c3": (256, 48, 32128, 768, True)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(SHAPES))
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--routes", default="gemm,fused")
    ap.add_argument("--tune", action="append", default=[])
    args = ap.parse_args()
    import torch
    import __graft_entry__
    P = __graft_entry__.load_package()
    P.load_library()
    for kv in args.tune:
        k, v = kv.split("=")
        P._lib.set_tuning(k, int(v))
    B, T, V, H, masked = SHAPES[args.config]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    f = dict(generator=g, device=dev)
    h = torch.randn(B, T, H, **f).to(torch.bfloat16)
    w = (torch.randn(V, H, **f) * 0.05).to(torch.bfloat16)
    ref_h = (h.float() + 0.1 * torch.randn(B, T, H, **f)).to(torch.bfloat16)
    new_h = (h.float() + 0.05 * torch.randn(B, T, H, **f)).to(torch.bfloat16)
    labels = torch.randint(0, V, (B, T), **f)
    old_values = torch.randn(B, T, **f)
    values = old_values + 0.3 * torch.randn(B, T, **f)
    scores = torch.rand(B, **f) * 24 - 12
    lengths = mask = None
    if masked:
        lengths = torch.randint(1, T + 1, (B,), **f)
        mask = (torch.arange(T, device=dev)[None, :] < lengths[:, None]).long()
        old_values = old_values.masked_fill(mask == 0, 0)
    N = B * T
    hp = P.PPOHotPath(P.PPOConfig(), B, T, V, torch.bfloat16, dev, kl_coef=0.05)
    hp.experience_from_hidden(h, w, ref_h, w, labels, old_values, scores, lengths=lengths, mask=mask, route="fused")
    torch.cuda.synchronize()
    logits = torch.empty(B, T, V, dtype=torch.bfloat16, device=dev)
    dh_g = torch.empty(N, H, dtype=torch.bfloat16, device=dev)
    dw_g = torch.empty(V, H, dtype=torch.bfloat16, device=dev)
    h2 = new_h.view(N, H)

    def gemm():
        torch.matmul(new_h, w.t(), out=logits)
        _, _, dl, _ = hp.policy_loss(logits, labels, values, old_values, mask=mask)
        d2 = dl.view(N, V)
        torch.matmul(d2, w, out=dh_g)
        torch.matmul(d2.t(), h2, out=dw_g)

    def fused():
        hp.policy_loss_from_hidden(new_h, w, labels, values, old_values, mask=mask)

    def fused_recompute():  # the dW kernel recomputing S^T (k_lmloss_dw) instead of the saved P
        hp.policy_loss_from_hidden(new_h, w, labels, values, old_values, mask=mask, plan="recompute")

    routes = {"gemm": gemm, "fused": fused, "fused_recompute": fused_recompute}
    names = args.routes.split(",")
    for n in names:  # warm up (and hipBLASLt heuristics)
        for _ in range(3):
            routes[n]()
    torch.cuda.synchronize()
    res = {n: [] for n in names}
    for _ in range(args.rounds):
        for n in names:
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(args.iters)]
            for a, b in evs:
                a.record()
                routes[n]()
                b.record()
            torch.cuda.synchronize()
            res[n].append(statistics.median(a.elapsed_time(b) for a, b in evs) * 1e3)
    # one N·V·H multiply-add pass: the fused route over the live (mask != 0) tokens it keeps,
    # the gemm route over every token; the passes each route's plan runs (bench.py's count)
    nv = int(mask.sum().item()) if mask is not None else N
    flop_live, flop_all = 2.0 * nv * V * H, 2.0 * N * V * H
    savep = P._lib.query("trlx_ppo_loss_from_hidden_plan", N, H, V, hp.lm_loss_ws.numel()) == 1
    out = {"config": args.config, "N": N, "live_tokens": nv, "V": V, "H": H, "masked": masked,
           "us_per_call": {n: [round(x, 1) for x in v] for n, v in res.items()}}
    if "gemm" in res:
        out["gemm_tflops_3pass"] = round(3 * flop_all / (min(res["gemm"]) * 1e-6) / 1e12, 1)
    if "fused" in res:
        passes = 3 if savep else 4
        out["fused_plan"] = "saved_p" if savep else "recompute"
        out[f"fused_tflops_{passes}pass"] = round(passes * flop_live / (min(res["fused"]) * 1e-6) / 1e12, 1)
    if "fused_recompute" in res:
        out["fused_recompute_tflops_4pass"] = round(4 * flop_live / (min(res["fused_recompute"]) * 1e-6) / 1e12, 1)
    if "gemm" in res and "fused" in res:
        out["speedup_fused_vs_gemm"] = round(min(res["gemm"]) / min(res["fused"]), 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
