#!/usr/bin/env python3
"""rocprofv3 kernel-trace average of a kernel over bench.py's TIMED window.

bench.py runs W warm-up calls then K timed calls of each workload; rocprofv3 --stats averages every
dispatch, warm-up (clock ramp) included.  This prints, per matching kernel, the average over all
dispatches and over dispatches [skip, skip + count) -- the ones bench.py's hipEvents timed.
    python tools/trace_window.py <run_kernel_trace.csv> <kernel-substring> <skip> <count>
"""
import csv
import sys


def main():
    path, pat, skip, count = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    rows = [r for r in csv.DictReader(open(path)) if pat in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    win = d[skip:skip + count]
    print(f"{pat}: {len(d)} dispatches, average {sum(d) / len(d):.4f} ms; "
          f"dispatches {skip}..{skip + len(win) - 1} (bench's timed window) average {sum(win) / max(1, len(win)):.4f} ms, "
          f"window min {min(win):.4f}, max {max(win):.4f} (all dispatches: min {min(d):.4f}, max {max(d):.4f})")


if __name__ == "__main__":
    main()
