"""Summarise rocprofv3 PMC runs (FETCH_SIZE and WRITE_SIZE collected in separate passes, as
MI355X_MICROARCH.md §HBM prescribes) into per-kernel HBM bytes per launch.

  python tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write [--config c2] [--out profiles/pmc_traffic.json]
      [--commit <sha>] [--command '<profiled command>']

Corrections (MI355X_MICROARCH.md §HBM, gfx950): FETCH_SIZE / WRITE_SIZE are in KiB;
FETCH_SIZE reads exactly half the bytes of a wide (16 B/lane) coalesced stream -> x2.
WRITE_SIZE is exact for 16-B-per-lane streaming stores.  Keys of the output follow
bench.py's kernel names ("experience" = the vocab-row forward, "loss" = the fused rows).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection csv under {d}")
    per = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            per[(name, r.get("Counter_Name"))].append(float(r.get("Counter_Value", 0.0)))
    return per


def kernel_key(name):
    if "k_vocab_rows<" in name:  # k_vocab_rows<DT, NV, MODE, ...>: MODE 0 = experience, 2 = fused loss rows
        mode = name.split("k_vocab_rows<", 1)[1].split(",")[2].strip()
        return {"0": "experience", "2": "loss"}.get(mode)
    if "k_rollout_gae" in name:
        return "rollout_gae"
    if "k_rollout_loss" in name:
        return "rollout_loss"
    if "k_ilql_rows" in name:
        return "rows"
    if "k_ilql_prep" in name:
        return "prep"
    if "k_ilql_finalize" in name:
        return "finalize"
    return None


def main():
    args = sys.argv[1:]
    fetch_dir, write_dir = args[0], args[1]
    cfg = "c2"
    out = None
    if "--config" in args:
        cfg = args[args.index("--config") + 1]
    if "--out" in args:
        out = args[args.index("--out") + 1]
    meta = {}
    for key in ("--commit", "--command"):
        if key in args:
            meta[key[2:]] = args[args.index(key) + 1]
    f = load(fetch_dir)
    w = load(write_dir)
    res = {}
    for (name, counter), vals in list(f.items()) + list(w.items()):
        k = kernel_key(name)
        if k is None:
            continue
        avg = sum(vals) / len(vals)
        d = res.setdefault(k, {"kernel": name[:120]})
        if counter == "FETCH_SIZE":
            d["fetch_kib_raw"] = avg
            d["fetch_bytes"] = avg * 1024 * 2  # gfx950: FETCH_SIZE counts half of wide streaming reads
        elif counter == "WRITE_SIZE":
            d["write_bytes"] = avg * 1024
        d["launches"] = len(vals)
    summary = {}
    for k, d in res.items():
        d["hbm_bytes"] = d.get("fetch_bytes", 0.0) + d.get("write_bytes", 0.0)
        summary[k] = d["hbm_bytes"]
    print(json.dumps(res, indent=1))
    if out:
        prev = json.load(open(out)) if os.path.exists(out) else {}
        prev[cfg] = summary
        prev.setdefault("_detail", {})[cfg] = res
        if meta:
            prev.setdefault("_meta", {})[cfg] = meta
        json.dump(prev, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
