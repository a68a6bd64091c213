#!/usr/bin/env python3
"""A/B of the saved-P dW kernel's forms (tuning lmloss_dwp_form) inside the
PPO update from hidden states (PPOHotPath.policy_loss_from_hidden, fused route), interleaved
rounds on one box, HIP events on the launch stream; checks that forms with the same split
granule give bit-identical gradients."""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SHAPES = {"c2": (128, 48, 50257, 768, False), "c3_shard": (256, 48, 32128, 768, True)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(SHAPES))
    ap.add_argument("--variants", default="2,1", help="forms, comma separated (the round-6 A/B of the dropped forms 3 / 4 "
                    "and of the XCD placement ran at commit before their removal: profiles/r06f_dwp_forms_*)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    import torch
    import __graft_entry__
    P = __graft_entry__.load_package()
    L = P._lib
    dev = torch.device("cuda:0")
    B, T, V, H, masked = SHAPES[args.config]
    g = torch.Generator(device=dev).manual_seed(4242)
    f = dict(generator=g, device=dev)
    h = torch.randn(B, T, H, **f).to(torch.bfloat16)
    w = (0.05 * torch.randn(V, H, **f)).to(torch.bfloat16)
    new_h = (h.float() + 0.05 * torch.randn(B, T, H, **f)).to(torch.bfloat16)
    labels = torch.randint(0, V, (B, T), **f)
    old_values = torch.randn(B, T, **f)
    values = old_values + 0.3 * torch.randn(B, T, **f)
    scores = torch.rand(B, **f) * 24 - 12
    lengths = mask = None
    if masked:
        lengths = torch.randint(1, T + 1, (B,), **f)
        mask = (torch.arange(T, device=dev)[None, :] < lengths[:, None]).long()
    hp = P.PPOHotPath(P.PPOConfig(), B, T, V, torch.bfloat16, dev, kl_coef=0.05, defer_tail=True)
    hp.experience_from_hidden(h, w, h, w, labels, old_values, scores, lengths=lengths, mask=mask, route="fused")
    variants = [int(v) for v in args.variants.split(",")]
    grads, res = {}, {v: [] for v in variants}

    def run(v, n):
        with L.tuning(lmloss_dwp_form=v):
            for _ in range(n):
                out = hp.policy_loss_from_hidden(new_h, w, labels, values, old_values, mask=mask, route="fused")
        return out

    for v in variants:  # warm-up + the gradients of each form
        out = run(v, 3)
        hp.wait_stats()
        torch.cuda.synchronize()
        grads[v] = (out[2].clone(), out[3].clone())
    for r in range(args.rounds):
        for v in variants[r % len(variants):] + variants[:r % len(variants)]:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run(v, args.iters)
            hp.wait_stats()
            e1.record()
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / args.iters * 1e3)
    base = variants[0]
    for v in variants:
        same = torch.equal(grads[v][1], grads[base][1]) and torch.equal(grads[v][0], grads[base][0])
        rel = float((grads[v][1].double() - grads[base][1].double()).norm() / grads[base][1].double().norm())
        print(json.dumps({"config": args.config, "form": v, "us_per_update": [round(x, 1) for x in res[v]],
                          "median": round(statistics.median(res[v]), 1), "dW_equal_to_first": same,
                          "dW_rel_to_first": rel}), flush=True)


if __name__ == "__main__":
    main()
