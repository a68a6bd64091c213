"""Does running the experience rows of batch k+1 beside the loss rows of batch k (two HIP
streams) beat the serial E -> GAE -> L order on one MI355X?  GPU-box tool.

  python tools/overlap_probe.py [c2|c3|c4] [steps]

serial      PPOHotPath.step (E, GAE tail, L rows, loss tail on one stream)
concurrent  stream A: experience (E + GAE tail) of one hot path; stream B: policy_loss (L rows
            + loss tail) of another; the streams join once per step — the upper bound of a
            software-pipelined schedule (no beta dependency between the two)
Both after a 200 ms settle; medians of 5 blocks of `steps` steps.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
import __graft_entry__  # noqa: E402

P = __graft_entry__.load_package()


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    B, T, V, _ = bench.CONFIGS[cfg]
    dev = torch.device("cuda:0")
    x = bench.make_inputs(torch, B, T, V, dev, seed=1, masked=cfg == "c3", dtype=torch.bfloat16)
    c = P.PPOConfig()
    hp = P.PPOHotPath(c, B, T, V, torch.bfloat16, dev, kl_coef=0.05)
    he = P.PPOHotPath(c, B, T, V, torch.bfloat16, dev, kl_coef=0.05)
    hl = P.PPOHotPath(c, B, T, V, torch.bfloat16, dev, kl_coef=0.05)
    a, b = torch.cuda.current_stream(dev), torch.cuda.Stream(dev)
    kw = dict(lengths=x["lengths"], mask=x["mask"])

    def serial():
        hp.step(x["logits"], x["ref_logits"], x["new_logits"], x["labels"], x["old_values"], x["values"],
                x["scores"], **kw)

    hl.experience(x["logits"], x["ref_logits"], x["labels"], x["old_values"], x["scores"], **kw)

    def concurrent():
        b.wait_stream(a)
        he.experience(x["logits"], x["ref_logits"], x["labels"], x["old_values"], x["scores"], **kw)
        with torch.cuda.stream(b):
            hl.policy_loss(x["new_logits"], x["labels"], x["values"], x["old_values"], mask=x["mask"])
        a.wait_stream(b)

    res = {}
    for name, fn in (("serial", serial), ("concurrent", concurrent), ("serial2", serial),
                     ("concurrent2", concurrent)):
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.2:
            fn()
            torch.cuda.synchronize()
        blocks = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(n):
                fn()
            e1.record()
            torch.cuda.synchronize()
            blocks.append(e0.elapsed_time(e1) * 1e3 / n)
        res[name] = sorted(blocks)[2]
        print(f"{cfg} {name:12s} {res[name]:8.1f} us/step  blocks {[round(v, 1) for v in blocks]}", flush=True)


if __name__ == "__main__":
    main()
