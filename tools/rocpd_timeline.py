"""Kernel timeline from a rocprofv3 rocpd database (run_results.db): the last N dispatches
before the final `skip`, with queue, idle gap before each kernel and duration.
python3 tools/rocpd_timeline.py gpurun_out/<dir>/run_results.db [N] [skip]"""
import sqlite3
import sys


def main(path, n=20, skip=40):
    c = sqlite3.connect(path)
    rows = c.execute("select start, end, queue_id, name from kernels order by start").fetchall()
    sel = rows[len(rows) - skip - n:len(rows) - skip]
    prev = None
    for s, e, q, name in sel:
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        print(f"q{q} gap {gap:7.2f} dur {(e - s) / 1e3:8.2f}  {name[:70]}")
        prev = e


if __name__ == "__main__":
    main(sys.argv[1], *(int(a) for a in sys.argv[2:]))
