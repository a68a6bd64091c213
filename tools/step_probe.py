"""Decompose the bench step on the GPU: each launch of PPOHotPath.step timed alone
(back-to-back repeats of the same launch) and inside the full step (HIP events around every
launch), many repetitions, medians.  GPU-box tool:  python tools/step_probe.py [c2|c3|c4]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
import __graft_entry__  # noqa: E402

P = __graft_entry__.load_package()


def med(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2]


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    B, T, V, _ = bench.CONFIGS[cfg]
    dev = torch.device("cuda:0")
    dt = torch.float32 if os.environ.get("DT") == "fp32" else torch.bfloat16
    x = bench.make_inputs(torch, B, T, V, dev, seed=1, masked=cfg == "c3", dtype=dt)
    hp = P.PPOHotPath(P.PPOConfig(), B, T, V, dt, dev, kl_coef=0.05)

    def step():
        hp.step(x["logits"], x["ref_logits"], x["new_logits"], x["labels"], x["old_values"], x["values"],
                x["scores"], lengths=x["lengths"], mask=x["mask"])

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    # full step, every launch instrumented
    hp.timers = {}
    for _ in range(40):
        step()
    torch.cuda.synchronize()
    inside = {k: med([a.elapsed_time(b) * 1e3 for a, b in v]) for k, v in hp.timers.items()}
    hp.timers = None
    # full step, no events
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(40):
        step()
    e1.record()
    torch.cuda.synchronize()
    step_us = e0.elapsed_time(e1) * 1e3 / 40
    # each launch alone, back to back
    alone = {}
    for name, fn in (("experience", lambda: hp.experience(x["logits"], x["ref_logits"], x["labels"], x["old_values"],
                                                         x["scores"], lengths=x["lengths"], mask=x["mask"])),
                     ("loss", lambda: hp.policy_loss(x["new_logits"], x["labels"], x["values"], x["old_values"],
                                                     mask=x["mask"]))):
        for _ in range(3):
            fn()
        hp.timers = {}
        for _ in range(30):
            fn()
        torch.cuda.synchronize()
        for k, v in hp.timers.items():
            alone[k] = med([a.elapsed_time(b) * 1e3 for a, b in v])
        hp.timers = None
    print(f"{cfg}: step {step_us:.1f} us (no events)")
    for k in inside:
        print(f"  {k:14s} in step {inside[k]:8.1f} us   alone {alone.get(k, float('nan')):8.1f} us")


if __name__ == "__main__":
    main()
