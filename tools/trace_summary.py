"""Summarise a rocprofv3 --kernel-trace csv: the dispatch sequence split at the GAN step's first kernel, per-step
busy time, idle gaps, and the device copies (name, size proxy = duration) with their neighbours.
    python tools/trace_summary.py <rocprof -d dir>"""
import collections
import csv
import glob
import os
import sys

files = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)
rows = []
for f in files:
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].replace("void ", "").split("(")[0][:60]))
rows.sort()
print(f"{len(rows)} dispatches")
names = collections.Counter(n for _s, _e, n in rows)
# the step boundary: the schedule kernel of AdamW_G / the first generator conv after it; use adamw_hparams launches
marks = [i for i, (_s, _e, n) in enumerate(rows) if "adamw_hparams" in n]
print("adamw_hparams at dispatch", marks[:40])
# per segment between consecutive hparams launches of the same optimizer (every other one): busy vs wall
for a, b in zip(marks[::2], marks[2::2]):
    seg = rows[a:b]
    wall = seg[-1][1] - seg[0][0]
    busy = sum(e - s for s, e, _n in seg)
    cps = [(n, e - s) for s, e, n in seg if "copy" in n.lower() or "fill" in n.lower()]
    print(f"step [{a},{b}): {len(seg)} dispatches, wall {wall / 1e6:.3f} ms, kernel busy {busy / 1e6:.3f} ms, copies/fills {len(cps)} "
          f"{sum(d for _n, d in cps) / 1e6:.3f} ms")
    gaps = sorted(((seg[i + 1][0] - seg[i][1]), seg[i][2], seg[i + 1][2]) for i in range(len(seg) - 1))[::-1][:8]
    for gap, n0, n1 in gaps:
        print(f"    gap {gap / 1e3:8.1f} us  {n0} -> {n1}")
print("copies / fills anywhere:")
for i, (s, e, n) in enumerate(rows):
    if "copy" in n.lower():
        prev = rows[i - 1][2] if i else ""
        nxt = rows[i + 1][2] if i + 1 < len(rows) else ""
        print(f"  #{i} {n} {(e - s) / 1e3:.1f} us  after {prev} before {nxt}")
