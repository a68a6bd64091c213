#!/usr/bin/env python3
"""The drop-in PPO update from hidden states at a BASELINE shape, for rocprofv3 traces:
PPOConfig.loss_from_hidden (autograd through lm_head_logprobs + the PPO loss) + backward,
`--iters` times (VERDICT r05 "Next round" 1: the trace must show k_lmloss_dwp, not k_lmloss_dw).

  rocprofv3 --kernel-trace --stats -d gpurun_out/x -- python3 tools/dropin_update.py --config c2
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {"c2": (128, 48, 50257, 768, False), "c3_shard": (256, 48, 32128, 768, True)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=sorted(SHAPES))
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--plan", default="auto", choices=("auto", "saved_p", "recompute"))
    args = ap.parse_args()
    import torch
    import __graft_entry__
    P = __graft_entry__.load_package()
    dev = torch.device("cuda:0")
    B, T, V, H, masked = SHAPES[args.config]
    g = torch.Generator(device=dev).manual_seed(7)
    f = dict(generator=g, device=dev)
    h = torch.randn(B, T, H, **f).to(torch.bfloat16).requires_grad_(True)
    w = (0.05 * torch.randn(V, H, **f)).to(torch.bfloat16).requires_grad_(True)
    v = torch.randn(B, T, **f).requires_grad_(True)
    labels = torch.randint(0, V, (B, T), **f)
    olp, ov, adv, ret = (torch.randn(B, T, **f) for _ in range(4))
    olp = -olp.abs() - 5
    mask = None
    if masked:
        L = torch.randint(1, T + 1, (B,), **f)
        mask = (torch.arange(T, device=dev)[None, :] < L[:, None]).long()
    cfg = P.PPOConfig()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(args.iters + 3):
        if i == 3:
            e0.record()
        h.grad = w.grad = v.grad = None
        loss, _ = cfg.loss_from_hidden(h, w, v, labels, olp, ov, adv, ret, mask, plan=args.plan,
                                       return_device_stats=True)
        loss.backward()
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"config": args.config, "plan": args.plan, "iters": args.iters,
                      "ms_per_update": round(e0.elapsed_time(e1) / args.iters, 4)}), flush=True)


if __name__ == "__main__":
    main()
