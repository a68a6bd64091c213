"""Interleaved A/B of a tuning knob on the ILQL C5 step (ILQLHotPath.step as bench.py runs
it), one process, rounds alternating between the values.  GPU-box tool:
    python tools/ilql_sweep.py [knob] [values, comma-separated]"""
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
    knob = sys.argv[1] if len(sys.argv) > 1 else "split_lds"
    vals = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "0,1").split(",")]
    B, T, V, _ = bench.CONFIGS["c5"]
    dev = torch.device("cuda:0")
    lg, qs, tqs, vs, batch = bench.make_ilql_inputs(torch, P, B, T, V, dev, seed=1)
    hp = P.ILQLHotPath(P.ILQLConfig(), B, T, V, torch.float32, dev)
    res = {v: [] for v in vals}
    for rnd in range(7):
        for v in vals:
            P._lib.set_tuning(knob, v)
            for _ in range(5):
                hp.step(lg, qs, tqs, vs, batch)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(30):
                hp.step(lg, qs, tqs, vs, batch)
            torch.cuda.synchronize()
            res[v].append((time.perf_counter() - t0) / 30 * 1e3)
    P._lib.set_tuning(knob, 0)
    for v in vals:
        xs = sorted(res[v])
        print(f"c5 {knob}={v}: median {xs[len(xs) // 2]:.4f} ms/step  min {xs[0]:.4f}  all {[round(t, 4) for t in res[v]]}",
              flush=True)


if __name__ == "__main__":
    main()
