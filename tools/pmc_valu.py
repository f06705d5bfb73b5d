#!/usr/bin/env python3
"""Build profiles/pmc_valu.json (read by bench.py for roofline.compute) from the VALU pass of
tools/gpu_evidence.sh: median per dispatch of the headline kernel's SQ counters.

  python tools/pmc_valu.py gpurun_out/r02a/pmc_valu profiles/r02/evidence
"""
from __future__ import annotations

import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "r2iq_persistent_kernel<0, false, false, false>"   # the headline launch (d = 0)


def main():
    run, evidence = sys.argv[1], sys.argv[2]
    per = {}
    for row in csv.DictReader(open(os.path.join(run, "run_counter_collection.csv"))):
        if KERNEL not in row["Kernel_Name"]:
            continue
        d = per.setdefault(row["Dispatch_Id"], {})
        d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    names = sorted({k for d in per.values() for k in d})
    med = {k: statistics.median(d[k] for d in per.values() if k in d) for k in names}
    valu = med["SQ_INSTS_VALU"]
    frames = 2048 * 11
    out = {"single d=0 nblk=2048": {
        "valu_insts_per_launch": valu,
        "valu_insts_per_wave_frame": valu / (frames * 4),
        "median_per_dispatch": med, "dispatches": len(per),
        "source": f"{evidence}/ (rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU ..., one pass, median over dispatches "
                  "of r2iq_persistent_kernel<0,...>; bench.py --steps 5 --warmup 2 --warmup-ms 0)"}}
    json.dump(out, open(os.path.join(ROOT, "profiles", "pmc_valu.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
