"""Per-kernel SQ counter summary of rocprofv3 --pmc passes (per launch averages; cycles per wave).
    python tools/sq_summary.py gpurun_out/sq1 gpurun_out/sq2 ..."""
import collections
import csv
import glob
import os
import sys

tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("void ", "").split("(")[0][:44]
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(k, d)].add(r["Dispatch_Id"])
rows = []
for k, c in tot.items():
    n = max(len(disp[(k, d)]) for d in sys.argv[1:])
    w = c.get("SQ_WAVES", 0) or 1
    wc = c.get("SQ_WAVE_CYCLES", 0)
    rows.append((wc, k, n, c, w))
rows.sort(reverse=True)
print(f"{'kernel':44s} {'disp':>5s} {'waves/l':>8s} {'wcyc/wave':>9s} {'act%':>5s} {'winst%':>6s} {'wait%':>5s} {'lds%':>5s} {'bankc%':>6s} {'mfma%':>6s} {'valu/w':>7s} {'salu/w':>7s} {'lds/w':>6s}")
for wc, k, n, c, w in rows[:22]:
    g = lambda x: c.get(x, 0)
    busy = g("SQ_BUSY_CYCLES") or 1
    print(f"{k:44s} {n:5d} {w / n:8.0f} {4 * wc / w:9.0f} {100 * g('SQ_ACTIVE_INST_ANY') / max(wc, 1):5.0f} "
          f"{100 * g('SQ_WAIT_INST_ANY') / max(wc, 1):6.0f} {100 * g('SQ_WAIT_ANY') / max(wc, 1):5.0f} "
          f"{100 * g('SQ_WAIT_INST_LDS') / max(wc, 1):5.0f} {100 * g('SQ_LDS_BANK_CONFLICT') / max(g('SQ_LDS_IDX_ACTIVE'), 1):6.0f} "
          f"{100 * g('SQ_VALU_MFMA_BUSY_CYCLES') / max(4 * busy * 256, 1):6.1f} {g('SQ_INSTS_VALU') / w:7.0f} {g('SQ_INSTS_SALU') / w:7.0f} "
          f"{g('SQ_INSTS_LDS') / w:6.0f}")
