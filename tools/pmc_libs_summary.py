#!/usr/bin/env python3
"""Summarise a tools/gpu_pmc_libs.sh run: per library, the dominant r2iq_ kernel's counters
(median over dispatches) and the derived stall / LDS ratios.
  python tools/pmc_libs_summary.py gpurun_out/TAG lib1 lib2 ..."""
import collections
import csv
import os
import statistics
import sys


def passes(run, lib):
    out, kern = {}, None
    for p in ("p1", "p2"):
        per, names = collections.defaultdict(lambda: collections.defaultdict(float)), {}
        for row in csv.DictReader(open(os.path.join(run, f"{lib}_{p}", "run_counter_collection.csv"))):
            if "r2iq_" not in row["Kernel_Name"]:
                continue
            names[row["Dispatch_Id"]] = row["Kernel_Name"]
            per[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
        kern = collections.Counter(names.values()).most_common(1)[0][0]
        keep = [c for d, c in per.items() if names[d] == kern]
        for k in {k for c in keep for k in c}:
            out[k] = statistics.median(c[k] for c in keep)
    return out, kern


def main():
    run, libs = sys.argv[1], sys.argv[2:]
    for lib in libs:
        m, kern = passes(run, lib)
        print(f"{lib:10s} LDS conflict / LDS active {m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']:.4f}  "
              f"conflict cycles {m['SQ_LDS_BANK_CONFLICT']:.4g}  wait LDS / wave {m['SQ_WAIT_INST_LDS'] / m['SQ_WAVE_CYCLES']:.4f}  "
              f"VALU insts {m['SQ_INSTS_VALU']:.4g}  LDS insts {m['SQ_INSTS_LDS']:.4g}  wave cycles {m['SQ_WAVE_CYCLES']:.4g}  "
              f"({kern[:60]})")


if __name__ == "__main__":
    main()
