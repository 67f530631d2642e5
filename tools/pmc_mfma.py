"""MFMA-utilisation counters per kernel of a short bench run (rocprofv3 --pmc, separate passes).

    python tools/pmc_mfma.py <out_prefix> "<title>" -- <bench args...>

Runs `rocprofv3 -L` once (the counters this box exposes), then one `--pmc` pass per counter group (each within
gfx950's per-pass slots: <= 8 SQ, 2 GRBM; /opt/skills/guides/MI355X_MICROARCH.md "rocprofv3 PMC slots"), each as its own
child process under `timeout -s KILL`, and summarises per kernel:

  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024)
      (MFMA busy cycles summed over the chip's 1024 SIMDs, over the SIMD-cycles of the dispatch; GRBM_GUI_ACTIVE sums
      the 8 XCDs' GPU-busy cycles, so / 8 is the dispatch's duration in cycles: the guide's DVFS item)
  clock_ghz = GRBM_GUI_ACTIVE / 8 / kernel duration (from the same pass's kernel trace)
  plus wave-cycle shares (active / issue-stall / parked), LDS bank-conflict share and VALU / SALU / LDS / MFMA
  instructions per wave.

The driver itself never touches the GPU (every GPU process is a rocprofv3 child).  Writes <out_prefix>.json / .md.
"""
import collections
import csv
import glob
import json
import os
import re
import subprocess
import sys

PASSES = [
    ["SQ_WAVES", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
     "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"],
    ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_MFMA", "SQ_LDS_BANK_CONFLICT",
     "SQ_LDS_IDX_ACTIVE", "GRBM_GUI_ACTIVE"],
]


def available():
    out = subprocess.run(["rocprofv3", "-L"], capture_output=True, text=True, timeout=120)
    return out.stdout + out.stderr


def run_pass(i, counters, bench, outdir):
    d = os.path.join(outdir, f"pass{i}")
    cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", "--kernel-trace", "--pmc", *counters, "-d", d, "-o", "run",
           "--output-format", "csv", "--", sys.executable, "-u", "bench.py", *bench]
    print("[pmc_mfma]", " ".join(cmd), flush=True)
    with open(os.path.join(outdir, f"pass{i}.log"), "w") as log:
        rc = subprocess.call(cmd, stdout=log, stderr=subprocess.STDOUT)
    if rc != 0:
        raise SystemExit(f"pass {i} failed with exit code {rc} (see {outdir}/pass{i}.log)")
    return d


def short(name):
    return name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]


def load(d):
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    dur = collections.defaultdict(float)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[short(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return vals, {k: len(v) for k, v in disp.items()}, dur


def main():
    sep = sys.argv.index("--")
    out, title = sys.argv[1], sys.argv[2]
    bench = sys.argv[sep + 1:]
    outdir = os.path.dirname(out) or "."
    os.makedirs(outdir, exist_ok=True)
    lst = available()
    open(out + "_counters.txt", "w").write(lst)
    names = set(re.findall(r"\b[A-Z][A-Z0-9_]+\b", lst))
    passes = [[c for c in p if c in names] for p in PASSES]
    for p, want in zip(passes, PASSES):
        missing = sorted(set(want) - set(p))
        if missing:
            print("[pmc_mfma] not exposed on this box:", missing, flush=True)
    data = [load(run_pass(i, p, bench, outdir)) for i, p in enumerate(passes)]
    kernels = {}
    for vals, nd, dur in data:
        for k, c in vals.items():
            rec = kernels.setdefault(k, {"launches": nd[k], "counters": {}, "trace_s": 0.0})
            rec["launches"] = max(rec["launches"], nd[k])
            for name, v in c.items():
                if name == "GRBM_GUI_ACTIVE" and "GRBM_GUI_ACTIVE" in rec["counters"]:
                    continue  # the first pass's (it carries the MFMA counter); passes differ by DVFS
                rec["counters"][name] = v
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                rec["trace_s"] = dur.get(k, 0.0)
    rows = {}
    for k, rec in kernels.items():
        c = rec["counters"]
        g = lambda n: c.get(n, 0.0)  # noqa: E731
        cyc = g("GRBM_GUI_ACTIVE") / 8.0
        waves = g("SQ_WAVES") or 1.0
        wc = g("SQ_WAVE_CYCLES") or 1.0
        row = {"launches": rec["launches"],
               "us_per_launch": round(rec["trace_s"] / max(rec["launches"], 1) * 1e6, 2) if rec["trace_s"] else None,
               "mfma_busy": round(g("SQ_VALU_MFMA_BUSY_CYCLES") / (cyc * 1024.0), 4) if cyc else None,
               "clock_ghz": round(cyc / rec["trace_s"] / 1e9, 3) if rec["trace_s"] and cyc else None,
               "active_inst_share": round(g("SQ_ACTIVE_INST_ANY") / wc, 3), "issue_stall_share": round(g("SQ_WAIT_INST_ANY") / wc, 3),
               "parked_share": round(g("SQ_WAIT_ANY") / wc, 3),
               "lds_bank_conflict_share": round(g("SQ_LDS_BANK_CONFLICT") / max(g("SQ_LDS_IDX_ACTIVE"), 1.0), 3),
               "valu_per_wave": round(g("SQ_INSTS_VALU") / waves, 1), "salu_per_wave": round(g("SQ_INSTS_SALU") / waves, 1),
               "lds_per_wave": round(g("SQ_INSTS_LDS") / waves, 1), "mfma_per_wave": round(g("SQ_INSTS_MFMA") / waves, 1),
               "waves_per_launch": round(waves / max(rec["launches"], 1), 1), "raw": c}
        rows[k] = row
    order = sorted(rows, key=lambda k: -(rows[k]["us_per_launch"] or 0) * rows[k]["launches"])
    src = (f"rocprofv3 --kernel-trace --pmc, {len(passes)} separate passes of `bench.py {' '.join(bench)}`: {title}. "
           "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs); per-launch averages over every launch "
           "of the kernel in the run (eager warm-up + graph replays).")
    json.dump({"source": src, "passes": passes, "kernels": {k: rows[k] for k in order}}, open(out + ".json", "w"), indent=1)
    with open(out + ".md", "w") as f:
        f.write(f"# {title}\n\n{src}\n\n| kernel | launches | us/launch | MFMA busy | clock GHz | active | issue-stall | parked | "
                "LDS conflicts | MFMA/wave | VALU/wave | SALU/wave | LDS/wave |\n|---|---|---|---|---|---|---|---|---|---|---|---|---|\n")
        for k in order[:30]:
            r = rows[k]
            f.write(f"| {k[:90]} | {r['launches']} | {r['us_per_launch']} | {r['mfma_busy']} | {r['clock_ghz']} | "
                    f"{r['active_inst_share']} | {r['issue_stall_share']} | {r['parked_share']} | {r['lds_bank_conflict_share']} | "
                    f"{r['mfma_per_wave']} | {r['valu_per_wave']} | {r['salu_per_wave']} | {r['lds_per_wave']} |\n")
    print(open(out + ".md").read())


if __name__ == "__main__":
    main()
