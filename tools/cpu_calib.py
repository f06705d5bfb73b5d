#!/usr/bin/env python3
"""CPU calibration: time the library's AVX2 CPU backend and the oracle's
float32 port on one core of THIS container for d = 0..4 and relate them to the reference's own
r2iq timed on the same container type by the survey probe (forced-AVX2 worker,
1 core, 2048 blocks).  The reference itself cannot be built here (it needs <fftw3.h>), so the
probe numbers are quoted, not re-measured.  Writes profiles/cpu_calibration.json; bench.py
scales its on-box CPU-backend timing by these ratios to state a reference-equivalent rate.

    python tools/cpu_calib.py [--seconds 5]
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PROBE_REF_MSPS = {0: 418.0, 1: 560.0, 2: 667.0, 3: 773.0, 4: 847.0}   # BASELINE.md §2, forced AVX2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=5.0)
    args = ap.parse_args()
    from oracle import oracle as O
    from extio_sddc_amd.synth import make_stream
    nblk = 16
    x = make_stream(nblk, "mix")
    H = O.filter_bank(1.0, np.float32)
    cpu = "unknown"
    for line in subprocess.run(["lscpu"], capture_output=True, text=True).stdout.splitlines():
        if line.startswith("Model name"):
            cpu = line.split(":", 1)[1].strip()
    import bench
    out = {"container_cpu": cpu, "host": platform.node(), "avx2_backend": {}, "port": {},
           "reference_probe": PROBE_REF_MSPS, "ratio_reference_over_avx2_backend": {},
           "ratio_reference_over_port": {},
           "note": "avx2_backend = the library's CPU backend (extio_sddc_amd/csrc/cpu, a handle on "
                   "SDDC_DDC_DEVICE_CPU), 1 thread, 16-block sample; port = oracle/ddc_oracle.c float32 "
                   "path, 1 thread; reference = survey probe of Core/fft_mt_r2iq (AVX2 worker, MKL FFTW3 "
                   "wrapper) on this container type"}
    for d in range(5):
        v, _, _ = bench.cpu_backend_rate(d, 1024, x, nblk, args.seconds)
        out["avx2_backend"][d] = v
        out["ratio_reference_over_avx2_backend"][d] = PROBE_REF_MSPS[d] / v
        print(f"d={d} avx2 backend {v:.1f} MS/s, reference probe {PROBE_REF_MSPS[d]:.0f} -> ratio "
              f"{PROBE_REF_MSPS[d] / v:.2f}")
        O.r2iq(x, 1, d, 1024, dtype=np.float32, H=H)
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < args.seconds:
            O.r2iq(x, nblk, d, 1024, dtype=np.float32, H=H)
            done += nblk
        v = done * 65536 / (time.perf_counter() - t0) / 1e6
        out["port"][d] = v
        out["ratio_reference_over_port"][d] = PROBE_REF_MSPS[d] / v
        print(f"d={d} port {v:.1f} MS/s, reference probe {PROBE_REF_MSPS[d]:.0f} -> ratio {PROBE_REF_MSPS[d] / v:.2f}")
    with open(os.path.join(ROOT, "profiles", "cpu_calibration.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
