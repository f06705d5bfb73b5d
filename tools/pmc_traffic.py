#!/usr/bin/env python3
"""Build profiles/pmc_traffic.json (read by bench.py for roofline.traffic) from a
tools/gpu_round.sh run: median FETCH_SIZE / WRITE_SIZE over the headline kernel's dispatches,
corrected by the same counters on tools/pmc_calib.hip, which moves known bytes with the
kernel's access widths (MI355X_MICROARCH.md, HBM section: calibrate the counters' units).

  python tools/pmc_traffic.py gpurun_out/final2 profiles/r01/final
"""
from __future__ import annotations

import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "r2iq_persistent_kernel<0, false, false, false>"   # the headline launch (d = 0), not the sweep


def per_dispatch(path, counter, kernel):
    sums = {}
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter or kernel not in row["Kernel_Name"]:
            continue
        sums[row["Dispatch_Id"]] = sums.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
    return statistics.median(sums.values())


def main():
    run, evidence = sys.argv[1], sys.argv[2]
    nblk = 2048
    alg_read, alg_write = nblk * 65536 * 2, nblk * 32768 * 8
    fetch = per_dispatch(f"{run}/pmc_FETCH_SIZE/run_counter_collection.csv", "FETCH_SIZE", KERNEL)
    write = per_dispatch(f"{run}/pmc_WRITE_SIZE/run_counter_collection.csv", "WRITE_SIZE", KERNEL)
    cf = per_dispatch(f"{run}/calib_FETCH_SIZE/run_counter_collection.csv", "FETCH_SIZE", "calib")
    cw = per_dispatch(f"{run}/calib_WRITE_SIZE/run_counter_collection.csv", "WRITE_SIZE", "calib")
    known_r, known_w = 268435456, 536870912          # tools/pmc_calib.hip
    rf, wf = known_r / (cf * 1024), known_w / (cw * 1024)
    rd, wr = fetch * 1024 * rf, write * 1024 * wf
    out = {"single d=0 nblk=2048": {
        "hbm_bytes_per_launch": rd + wr, "read_bytes_corrected": rd, "write_bytes": wr,
        "fetch_size_kb": fetch, "write_size_kb": write,
        "algorithmic_read_bytes": alg_read, "algorithmic_write_bytes": alg_write,
        "calibration": {"kernel": "tools/pmc_calib.hip (4 B/lane buffer loads, 8 B/lane buffer stores, persistent grid)",
                        "known_read_bytes": known_r, "fetch_size_kb": cf, "read_factor": rf,
                        "known_write_bytes": known_w, "write_size_kb": cw, "write_factor": wf},
        "source": f"{evidence}/ (rocprofv3 --kernel-trace --pmc FETCH_SIZE / WRITE_SIZE, separate passes, median over "
                  "dispatches; MI355X_MICROARCH.md 'HBM': calibrate uncalibrated widths on known bytes)"}}
    json.dump(out, open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
