#!/usr/bin/env python3
"""Per-kernel durations and the idle gaps between consecutive kernels of a rocprofv3 kernel trace.

  python tools/trace_gaps.py <kernel_trace.csv> [--last N]

Prints, for the last N dispatches, name / duration / gap to the previous dispatch's end (µs),
then the totals: busy time, gap time, and the span from the first start to the last end.
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last", type=int, default=40)
    args = ap.parse_args()
    rows = []
    with open(args.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    rows = rows[-args.last:]
    busy = gaps = 0
    prev_end = None
    for s, e, n in rows:
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        busy += (e - s) / 1e3
        gaps += max(gap, 0.0)
        print(f"{(e - s) / 1e3:9.1f} us  gap {gap:7.1f}  {n[:110]}")
        prev_end = e if prev_end is None else max(prev_end, e)
    print(f"busy {busy:.1f} us  gaps {gaps:.1f} us  span {(rows[-1][1] - rows[0][0]) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
