"""Per-kernel duration summary of a rocprofv3 SQLite result (rocpd `kernels` view):
name (truncated), calls, average / min / max us.  python tools/rocpd_stats.py <results.db> [filter]"""
import sqlite3
import sys
from collections import defaultdict


def main():
    c = sqlite3.connect(sys.argv[1])
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    per = defaultdict(list)
    for name, dur in c.execute("select name, duration from kernels"):
        if flt in name:
            per[name].append(dur / 1e3)
    rows = sorted(per.items(), key=lambda kv: -sum(kv[1]))
    for name, d in rows:
        short = name.replace("void ", "").split("(")[0][:90]
        print(f"{short:90s} {len(d):5d} {sum(d) / len(d):10.1f} {min(d):10.1f} {max(d):10.1f}")


if __name__ == "__main__":
    main()
