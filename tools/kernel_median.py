#!/usr/bin/env python3
"""Median duration per kernel (µs) from a rocprofv3 kernel_trace.csv, skipping each kernel's
first --skip dispatches (clock ramp / first-touch), for kernels whose name contains --match.

  python tools/kernel_median.py <k_kernel_trace.csv> [--match k_lmloss] [--skip 3]
"""
import argparse
import collections
import csv
import json
import re
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--match", default="k_lmloss")
    ap.add_argument("--skip", type=int, default=3)
    args = ap.parse_args()
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(args.csv)):
        n = r["Kernel_Name"]
        if args.match in n:
            n = re.sub(r"^void |trlx::|\(trlx::LmLossArgs\)$", "", n)[:60]
            d[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(json.dumps({k: {"n": len(v), "median_us": round(statistics.median(v[args.skip:] or v), 1)}
                      for k, v in d.items()}))


if __name__ == "__main__":
    main()
