#!/usr/bin/env python3
"""Per-library PMC summary of a tools/gpu_pmc_libs.sh directory (kernel-name filter, averages over
the launches): LDS bank-conflict share, VALU issue, waits, effective clock.
  python tools/pmc_libs_cmp.py DIR LIB [LIB ...] [--kernel SUBSTR]"""
import collections
import csv
import os
import sys


def load(d, lib, kern):
    acc, n = collections.defaultdict(float), collections.Counter()
    for p in ("p1", "p2"):
        f = os.path.join(d, f"{lib}_{p}", "run_counter_collection.csv")
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
                n[r["Counter_Name"]] += 1
    dur = []
    for p in ("p1", "p2"):
        f = os.path.join(d, f"{lib}_{p}", "run_kernel_trace.csv")
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    return {k: acc[k] / n[k] for k in acc}, sorted(dur)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    kern = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else "fs_kernel"
    if "--kernel" in sys.argv:
        args.remove(kern)
    d, libs = args[0], args[1:]
    for lib in libs:
        c, dur = load(d, lib, kern)
        us = dur[len(dur) // 2]
        clk = c["GRBM_GUI_ACTIVE"] / 8 / us * 1e-3  # GHz: GRBM counts per XCD, summed over 8
        print(f"{lib:10s} kernel {us:7.1f} us  LDS conflicts {c['SQ_LDS_BANK_CONFLICT'] / c['SQ_LDS_IDX_ACTIVE'] * 100:5.1f} % "
              f"of LDS-active  LDS-active/wave-cyc {c['SQ_LDS_IDX_ACTIVE'] / c['SQ_WAVE_CYCLES']:.3f}  "
              f"VALU insts {c['SQ_INSTS_VALU'] / 1e6:6.2f} M  wait_any/wave-cyc {c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']:.3f}  "
              f"wait_inst_lds/wave-cyc {c['SQ_WAIT_INST_LDS'] / c['SQ_WAVE_CYCLES']:.3f}  eff clock {clk:.2f} GHz")


if __name__ == "__main__":
    main()
