#!/usr/bin/env python3
"""Per-kernel averages of every counter in rocprofv3 --pmc counter_collection.csv files (one or
more passes), plus the dispatch duration and derived ratios where their counters are present:
  mfma_busy  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
  l2_hit     = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
  clock_ghz  = GRBM_GUI_ACTIVE / 8 / duration
  wait_frac / inst_wait_frac / active_frac = SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES
  lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE

  python tools/pmc_kernels.py a.csv [b.csv ...] [--match k_lmloss]
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
    return name[:80]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--match", default="k_lmloss")
    args = ap.parse_args()
    pats = args.match.split(",")
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in args.csv:
        disp = collections.defaultdict(dict)
        for r in csv.DictReader(open(path)):
            if not any(p in r["Kernel_Name"] for p in pats):
                continue
            d = disp[(r["Dispatch_Id"], r["Kernel_Name"])]
            d[r["Counter_Name"]] = float(r["Counter_Value"])
            d["dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for (_, name), d in disp.items():
            for k, v in d.items():
                agg[short(name)][k].append(v)
    out = {}
    for name, cs in sorted(agg.items()):
        m = {k: sum(v) / len(v) for k, v in cs.items()}
        o = {k: (round(v, 1) if abs(v) < 1e6 else float(f"{v:.4g}")) for k, v in m.items()}
        g = m.get("GRBM_GUI_ACTIVE")
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            o["mfma_busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8 * 1024), 4)
        if g and m.get("dur_ns"):
            o["clock_ghz"] = round(g / 8 / m["dur_ns"], 3)
        if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
            o["l2_hit"] = round(m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"]), 4)
        if m.get("SQ_WAVE_CYCLES"):
            for k, n in (("SQ_WAIT_ANY", "wait_frac"), ("SQ_WAIT_INST_ANY", "inst_wait_frac"),
                         ("SQ_ACTIVE_INST_ANY", "active_frac")):
                if k in m:
                    o[n] = round(m[k] / m["SQ_WAVE_CYCLES"], 4)
        if m.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_BANK_CONFLICT" in m:
            o["lds_conflict"] = round(m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"], 4)
        o["dispatches"] = len(cs["dur_ns"])
        out[name] = o
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
