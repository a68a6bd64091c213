#!/usr/bin/env python3
"""MFMA busy per SIMD from a rocprofv3 --pmc counter_collection.csv (SQ_VALU_MFMA_BUSY_CYCLES,
SQ_INSTS_MFMA, SQ_WAVE_CYCLES, GRBM_GUI_ACTIVE): per kernel, averaged over its dispatches.
busy/SIMD = MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs); clock = GRBM_GUI_ACTIVE / 8 / duration.

  python tools/mfma_pmc_summary.py <counter_collection.csv> [--match k_lmloss,Cijk]
"""
import argparse
import collections
import csv
import json
import re


def short(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"trlx::", "", name)
    name = re.sub(r"\(trlx::LmLossArgs\)$", "", name)
    return name[:72]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--match", default="k_lmloss_fwd,k_lmloss_dw<,Cijk")
    args = ap.parse_args()
    pats = args.match.split(",")
    disp = collections.defaultdict(dict)
    for r in csv.DictReader(open(args.csv)):
        if not any(p in r["Kernel_Name"] for p in pats):
            continue
        d = disp[(r["Dispatch_Id"], r["Kernel_Name"])]
        d[r["Counter_Name"]] = float(r["Counter_Value"])
        d["dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    per = collections.defaultdict(list)
    for (_, name), d in disp.items():
        per[short(name)].append(d)
    out = {}
    for name, ds in sorted(per.items()):
        n = len(ds)
        g = sum(d.get("GRBM_GUI_ACTIVE", 0) for d in ds) / n / 8
        out[name] = {
            "dispatches": n,
            "avg_us": round(sum(d["dur_ns"] for d in ds) / n / 1e3, 1),
            "clock_ghz": round(g / (sum(d["dur_ns"] for d in ds) / n), 3),
            "mfma_busy_per_simd": round(sum(d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) for d in ds) / n / (g * 1024), 3),
            "mfma_insts": sum(d.get("SQ_INSTS_MFMA", 0) for d in ds) / n,
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
