"""DESIGN.md section 3's kernel table from a round's records: the bench line's per-kernel HIP-event totals (one GAN step,
eager) and the PMC traffic summary of the same library.
    python tools/kernel_table.py profiles/<tag>_gan_bench.json profiles/<tag>_gan_pmc_traffic.json [rows]"""
import json
import sys

PEAK_TF, PEAK_GBS = 2500.0, 8000.0


def main():
    bench = json.loads(open(sys.argv[1]).readline())
    pmc = json.load(open(sys.argv[2])) if len(sys.argv) > 2 else {"kernels": {}}
    rows = int(sys.argv[3]) if len(sys.argv) > 3 else 24
    kern = bench["kernels"]
    step = bench["ms_per_step"]
    print(f"| kernel | launches / step | ms / step | µs / launch | rate (algorithmic) | of peak | PMC MB / launch (fetch + write) |")
    print("|---|---|---|---|---|---|---|")
    for name, v in sorted(kern.items(), key=lambda kv: -kv[1]["ms_total"])[:rows]:
        us = v["ms_total"] / v["launches"] * 1e3
        if v.get("tflops"):
            rate, frac = f"{v['tflops']:.0f} TF/s", v["tflops"] / PEAK_TF
        elif v.get("gbs"):
            rate, frac = f"{v['gbs'] / 1e3:.2f} TB/s", v["gbs"] / PEAK_GBS
        else:
            rate, frac = "—", None
        rec = pmc.get("kernels", {}).get(name)
        traffic = f"{rec['hbm_bytes_per_launch'] / 1e6:.1f}" if rec else "—"
        print(f"| `{name}` | {v['launches']} | {v['ms_total']:.3f} | {us:.1f} | {rate} | {'' if frac is None else f'{frac:.2f}'} | {traffic} |")
    print(f"\nStep {step:.3f} ms; the rows above sum to {sum(v['ms_total'] for v in kern.values()):.2f} ms of eager per-launch time.")


if __name__ == "__main__":
    main()
