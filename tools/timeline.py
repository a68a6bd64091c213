"""Per-step timeline of the bench step from a rocprofv3 --kernel-trace csv: the median
duration of each hot-path kernel and the median idle gap before it (the previous
dispatch's end to this one's start, same queue).  python tools/timeline.py <kernel_trace.csv> [first_n_skip]"""
import csv
import sys


def short(name):
    if "k_vocab_rows<" in name:  # <DT, NV, MODE, ...>: MODE 0 the experience (forward) rows, 2 the loss rows
        mode = name.split("k_vocab_rows<", 1)[1].split(",")[2].strip()
        return {"0": "E rows", "2": "L rows"}.get(mode, "rows(other)")
    for key, lab in (("k_vocab_rows<trlx::BF16T, 13, 0", "E rows"), ("k_vocab_rows<trlx::BF16T, 9, 2", "L rows"),
                     ("k_vocab_rows", "rows(other)"), ("k_rollout_gae", "GAE tail"), ("k_ragged_order", "ragged order"), ("k_rollout_loss", "loss tail"),
                     ("k_ilql_rows", "ILQL rows"), ("k_ilql_prep", "ILQL prep"), ("k_ilql_finalize", "ILQL finalize"),
                     ("k_score_moments", "score moments"), ("k_whiten_coef", "whiten coef"), ("nccl", "RCCL (side)")):
        if key in name:
            return lab
    return None


def main(path, skip=50):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ev = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    ev = [e for e in ev if e[0]][skip:]
    dur, gap = {}, {}
    last_end = None  # the step's own stream: side-stream RCCL kernels are listed, not chained
    for n, s, e in ev:
        dur.setdefault(n, []).append((e - s) / 1e3)
        if n.endswith("(side)"):
            continue
        if last_end is not None:
            gap.setdefault(n, []).append((s - last_end) / 1e3)
        last_end = e
    med = lambda xs: sorted(xs)[len(xs) // 2]
    tot = 0.0
    for n in dur:
        d, g = med(dur[n]), med(gap.get(n, [0.0]))
        tot += d + g
        print(f"{n:12s} n={len(dur[n]):5d}  median {d:8.2f} us   idle gap before {g:6.2f} us")
    print(f"sum of medians (one of each): {tot:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 50)
