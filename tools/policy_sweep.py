"""Interleaved A/B of a tuning knob on the full bench step (PPOHotPath.step as bench.py runs
it: device controller state, overlapped loss tail).  GPU-box tool:
    python tools/policy_sweep.py [c2|c3|c4] [knob] [values, comma-separated]
(env: DT=fp32 for fp32 logits, ROWS=<rollouts> to override the config's rows per GPU)"""
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
    knob = sys.argv[2] if len(sys.argv) > 2 else "store_policy"
    vals = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "0,1,2,3,4").split(",")]
    B, T, V, _ = bench.CONFIGS[cfg]
    B = int(os.environ.get("ROWS", B))  # e.g. ROWS=1024 for the C4 strong-scaling shape on one GPU
    dev = torch.device("cuda:0")
    dt = torch.float32 if os.environ.get("DT") == "fp32" else torch.bfloat16
    x = bench.make_inputs(torch, B, T, V, dev, seed=1, masked=cfg == "c3", dtype=dt)
    pc = P.PPOConfig()
    hp = P.PPOHotPath(pc, B, T, V, dt, dev, kl_coef=0.05,
                      ctl=P.PPOControlState.from_config(pc, dev, n_steps=B), overlap_tail=True)

    def step():
        hp.step(x["logits"], x["ref_logits"], x["new_logits"], x["labels"], x["old_values"], x["values"],
                x["scores"], lengths=x["lengths"], mask=x["mask"])

    res = {v: [] for v in vals}
    for rnd in range(5):
        for v in vals:
            P._lib.set_tuning(knob, v)
            for _ in range(5):
                step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(50):
                step()
            torch.cuda.synchronize()
            res[v].append((time.perf_counter() - t0) / 50 * 1e3)
    P._lib.set_tuning(knob, 0)
    for v in vals:
        xs = sorted(res[v])
        print(f"{cfg} {knob}={v}: median {xs[len(xs) // 2]:.4f} ms/step  min {xs[0]:.4f}  all {[round(t, 4) for t in res[v]]}",
              flush=True)


if __name__ == "__main__":
    main()
