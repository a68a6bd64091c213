#!/usr/bin/env python3
"""Accuracy of the loss side's dW / dh / E against fp64 for both dW plans (saved P, recompute),
flat and peaked softmax, at the C2 and C3 token counts: the lmloss_checks error terms and the
plain relative Frobenius error of dW, per plan (tests/lmloss_checks.py holds the limits)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import __graft_entry__
    P = __graft_entry__.load_package()
    import lmloss_checks as C
    dev = torch.device("cuda:0")
    for kind, N, V in (("flat", 6144, 50257), ("peaked", 6144, 50257), ("flat", 12288, 32128),
                       ("peaked", 12288, 32128)):
        H = 768
        if kind == "peaked":
            h, w, y = C.peaked_operands(N, H, V, 5)
        else:
            g = torch.Generator().manual_seed(5)
            h = torch.randn(N, H, generator=g).to(torch.bfloat16)
            w = (torch.randn(V, H, generator=g) * 0.05).to(torch.bfloat16)
            y = torch.randint(0, V, (N,), generator=g)
        gout = torch.randn(N, generator=torch.Generator().manual_seed(7))
        t = C.fp64_truth(h.to(dev), w.to(dev), y.to(dev), gout.to(dev))
        for plan in ("saved_p", "recompute"):
            hg = h.to(dev).requires_grad_(True)
            wg = w.to(dev).requires_grad_(True)
            lp = P.lm_head_logprobs(hg, wg, y.to(dev), out_dtype=torch.float32, plan=plan)
            (lp * gout.to(dev)).sum().backward()
            torch.cuda.synchronize()
            errs = C.dw_errors(wg.grad.float(), t["dw"], y)
            errs["dw_frob_rel"] = float((wg.grad.double() - t["dw"].double()).norm() / t["dw"].double().norm())
            print(json.dumps({"kind": kind, "N": N, "V": V, "plan": plan,
                              **{k: round(v, 6) for k, v in errs.items()}}), flush=True)
            del hg, wg, lp
        del t
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
