#!/usr/bin/env python3
"""Frames in flight, from a rocprofv3 kernel trace (--kernel-trace CSV):

  rocprofv3 --kernel-trace -d D -o run --output-format csv -- \\
      python3 bench.py --cpu-baseline off --steps 20 --inflight 2
  python tools/overlap_trace.py D/**/run_kernel_trace.csv [--steps 20]

For the render_kernel dispatches of the timed region (the `steps` dispatches
after the warm-up ones, found as the longest run of back-to-back
dispatches), prints each one's start / end relative to the first, its
duration, how long it overlapped the previous one, and the period between
consecutive ends.  With two frames in flight the next frame's dispatch starts
while the previous frame's tail still runs, so the per-step period (what
bench.py's ms_per_step measures) is below the per-dispatch duration
(rocprof's average, which also counts the time a dispatch waits for CUs)."""
from __future__ import annotations

import csv
import glob
import json
import statistics
import sys


def main():
    args = sys.argv[1:]
    steps = None
    if "--steps" in args:
        i = args.index("--steps")
        steps = int(args[i + 1])
        del args[i:i + 2]
    paths = [p for a in args for p in glob.glob(a, recursive=True)]
    rows = []
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                if "render_kernel" in r["Kernel_Name"]:
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    if not rows:
        raise SystemExit("no render_kernel dispatches")
    # the timed region: the longest run of dispatches whose starts are < 3 ms
    # apart from the previous end (bench.py issues them back to back)
    runs, cur = [], [rows[0]]
    for a, b in zip(rows, rows[1:]):
        if b[0] - a[1] < 3_000_000:
            cur.append(b)
        else:
            runs.append(cur)
            cur = [b]
    runs.append(cur)
    run = max(runs, key=len)
    if steps:
        run = run[-steps:]
    t0 = run[0][0]
    disp = []
    for k, (s, e, _) in enumerate(run):
        prev_end = run[k - 1][1] if k else None
        disp.append(dict(k=k, start_ms=round((s - t0) / 1e6, 3), end_ms=round((e - t0) / 1e6, 3),
                         dur_ms=round((e - s) / 1e6, 3),
                         overlap_prev_ms=round(max(0, prev_end - s) / 1e6, 3) if prev_end else None,
                         period_ms=round((e - prev_end) / 1e6, 3) if prev_end else None))
    periods = [d["period_ms"] for d in disp[1:]]
    durs = [d["dur_ms"] for d in disp]
    out = dict(dispatches=len(run), kernel=run[0][2][:60],
               mean_dispatch_ms=round(statistics.mean(durs), 3),
               median_dispatch_ms=round(statistics.median(durs), 3),
               mean_period_ms=round((run[-1][1] - run[0][1]) / 1e6 / (len(run) - 1), 3) if len(run) > 1 else None,
               median_period_ms=round(statistics.median(periods), 3) if periods else None,
               overlapped_dispatches=sum(1 for d in disp[1:] if d["overlap_prev_ms"] > 0),
               mean_overlap_ms=round(statistics.mean(d["overlap_prev_ms"] for d in disp[1:]), 3) if periods else None,
               dispatch=disp)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
