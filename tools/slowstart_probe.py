"""Where does a fresh process's slow start come from?  GPU-box tool.

  python tools/slowstart_probe.py [bench|heat|idle] [steps]

Builds the bench's C2 step exactly as bench.py does (device controller state, side-stream
loss tail), runs the bench's 5 warm-up steps, then times every step of the next `steps`
with one fence-free HIP event per step boundary (events only BETWEEN steps, never between
the launches of a step) and prints the per-step GPU time, the cumulative GPU-busy time since
the first launch, and the step's host launch time.

  bench  as above
  heat   first ~300 ms of plain HBM copies (torch copy_) before the warm-up: if the slow
         window disappears, it is chip state (clocks / power), not this step's buffers
  idle   after the measured window, sleep 1 s with the GPU idle, then time 60 more steps:
         does an idle gap bring the slow window back?
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
T_START = time.perf_counter()
import torch  # noqa: E402
import bench  # noqa: E402
import __graft_entry__  # noqa: E402

P = __graft_entry__.load_package()
from trlx_t5_amd.timing import LaunchEvent  # noqa: E402


def timed_steps(step, n):
    evs = [LaunchEvent() for _ in range(n + 1)]
    s = torch.cuda.current_stream()
    host = []
    evs[0].record(s)
    for i in range(n):
        h0 = time.perf_counter()
        step()
        host.append((time.perf_counter() - h0) * 1e6)
        evs[i + 1].record(s)
    torch.cuda.synchronize()
    us = [evs[i].elapsed_time(evs[i + 1]) * 1e3 for i in range(n)]
    return us, host


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "bench"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    B, T, V, _ = bench.CONFIGS["c2"]
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    t_cuda = time.perf_counter()
    if mode == "heat":
        a = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
        b = torch.empty_like(a)
        t0 = time.perf_counter()
        k = 0
        while time.perf_counter() - t0 < 0.3:
            b.copy_(a)
            k += 1
            if k % 20 == 0:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        del a, b
    x = bench.make_inputs(torch, B, T, V, dev, seed=1000, masked=False, dtype=torch.bfloat16)
    cfg = P.PPOConfig()
    ctl = P.PPOControlState.from_config(cfg, dev, n_steps=B)
    hp = P.PPOHotPath(cfg, B, T, V, torch.bfloat16, dev, kl_coef=0.05, ctl=ctl, overlap_tail=True)

    def step():
        hp.step(x["logits"], x["ref_logits"], x["new_logits"], x["labels"], x["old_values"], x["values"],
                x["scores"])

    t_inputs = time.perf_counter()
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t_warm = time.perf_counter()
    if mode == "launch":  # events around the two vocab-row launches of every step
        hp.timers, hp.timer_names = {}, {"experience", "loss"}
    us, host = timed_steps(step, n)
    if mode == "launch":
        for k, v in hp.timers.items():
            print(k, [round(a.elapsed_time(b) * 1e3, 1) for a, b in v])
        hp.timers = None
    out = {"mode": mode, "import_s": round(t_cuda - T_START, 3), "inputs_s": round(t_inputs - t_cuda, 3),
           "warmup_s": round(t_warm - t_inputs, 4)}
    cum, rows = 0.0, []
    for i, (u, h) in enumerate(zip(us, host)):
        cum += u
        rows.append((i, round(u, 1), round(cum / 1e3, 2), round(h, 1)))
    out["steps"] = rows
    bins = {}
    for lo, hi in ((0, 20), (20, 40), (40, 60), (60, 100), (100, 150), (150, n)):
        sel = us[lo:hi]
        if sel:
            bins[f"{lo}-{hi}"] = round(sorted(sel)[len(sel) // 2], 1)
    out["median_us_by_window"] = bins
    if mode == "idle":
        time.sleep(1.0)
        us2, _ = timed_steps(step, 60)
        out["after_idle_1s"] = [round(u, 1) for u in us2]
    print(json.dumps(out["median_us_by_window"]))
    print(json.dumps({k: v for k, v in out.items() if k != "steps"}))
    for r in rows:
        print("step %4d  gpu %8.1f us  cum %8.2f ms  host %7.1f us" % r)


if __name__ == "__main__":
    main()
