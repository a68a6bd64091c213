"""Condense a rocprofv3 `--kernel-trace --stats` kernel_stats.csv into a short text table.

  python tools/kernel_stats.py gpurun_out/prof/run_kernel_stats.csv "<command line>" > profiles/rNN_x.txt
"""
import csv
import sys


def main(path, header=""):
    if header:
        print(header)
    with open(path) as f:
        for r in csv.DictReader(f):
            print(f"{r['Name'][:100]:<100} calls={int(r['Calls']):>4} avg_us={float(r['AverageNs']) / 1e3:>9.2f} "
                  f"min_us={float(r['MinNs']) / 1e3:>9.2f} max_us={float(r['MaxNs']) / 1e3:>9.2f}")


if __name__ == "__main__":
    main(*sys.argv[1:])
