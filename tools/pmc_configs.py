#!/usr/bin/env python3
"""Build profiles/pmc_traffic.json and profiles/pmc_valu.json (read by bench.py: the headline's
roofline.traffic / roofline.compute and every sweep line's traffic / compute) from a
tools/gpu_pmc_configs.sh run.  Per config: the dominant r2iq_ kernel's counters summed per
dispatch, median over dispatches; HBM bytes corrected by the calibration kernel
(MI355X_MICROARCH.md 'rocprofv3 PMC' / HBM: calibrate uncalibrated widths on known bytes); the
effective clock GRBM_GUI_ACTIVE / 8 / dispatch time (MICROARCH 'DVFS give-back').

  python tools/pmc_configs.py gpurun_out/pmc_cfg profiles/r03/pmc_cfg
"""
from __future__ import annotations

import collections
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BLOCK = 65536
# name in bench.py -> (run dir prefix, d, nblk, channels)
CONFIGS = {
    "single d=0 nblk=2048": ("d0", 0, 2048, 1),
    "C3 decim 4": ("d1", 1, 2048, 1),
    "C3 decim 8": ("d2", 2, 2048, 1),
    "C3 decim 16": ("d3", 3, 2048, 1),
    "C3 decim 32": ("d4", 4, 2048, 1),
    "C4 VHF decim 4, sideband invert, rand": ("c4", 1, 2048, 1),
    "C5 1024 channels d=4 nblk=256": ("c5", 4, 256, 1024),
}
CLOCK_MAX_HZ = 2.4e9
SIMDS = 1024
FP32_PEAK = 157.3e12            # MI355X_MICROARCH.md: peak FP32 (vector), at 2.4 GHz
HBM_PEAK = 8.0e12


def read_pass(d):
    """{dispatch: {counter: value}} and {dispatch: kernel} of the dominant r2iq_ kernel."""
    per, names = {}, {}
    for row in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        k = row["Kernel_Name"]
        if "r2iq_" not in k or "build_" in k:
            continue
        disp = row["Dispatch_Id"]
        names[disp] = k
        c = per.setdefault(disp, {})
        c[row["Counter_Name"]] = c.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    top = collections.Counter(names.values()).most_common(1)[0][0]
    keep = {disp: c for disp, c in per.items() if names[disp] == top}
    return keep, top


def durations(d, kernel):
    ts = []
    p = os.path.join(d, "run_kernel_trace.csv")
    for row in csv.DictReader(open(p)):
        if row["Kernel_Name"] == kernel:
            ts.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    return ts


def med(per, name):
    v = [c[name] for c in per.values() if name in c]
    return statistics.median(v) if v else None


def calib(run):
    out = {}
    for c, known in (("FETCH_SIZE", 268435456), ("WRITE_SIZE", 536870912)):
        vals = collections.defaultdict(float)
        for row in csv.DictReader(open(os.path.join(run, f"calib_{c}", "run_counter_collection.csv"))):
            if row["Counter_Name"] == c and "calib" in row["Kernel_Name"]:
                vals[row["Dispatch_Id"]] += float(row["Counter_Value"])
        kb = statistics.median(vals.values())
        out[c] = {"known_bytes": known, "counter_kb": kb, "factor": known / (kb * 1024)}
    return out


def alg_bytes(d, nblk, nch):
    from bench import algorithmic_bytes_per_sample
    return nblk * BLOCK * algorithmic_bytes_per_sample(d, nch, 8)


def main():
    run, evidence = sys.argv[1], sys.argv[2]
    cal = calib(run)
    traffic, valu = {}, {}
    for name, (pre, d, nblk, nch) in CONFIGS.items():
        pf, kern = read_pass(os.path.join(run, f"{pre}_fetch"))
        pw, _ = read_pass(os.path.join(run, f"{pre}_write"))
        rd = med(pf, "FETCH_SIZE") * 1024 * cal["FETCH_SIZE"]["factor"]
        wr = med(pw, "WRITE_SIZE") * 1024 * cal["WRITE_SIZE"]["factor"]
        alg = alg_bytes(d, nblk, nch)
        traffic[name] = {"kernel": kern, "hbm_bytes_per_launch": rd + wr, "read_bytes_corrected": rd,
                         "write_bytes_corrected": wr, "algorithmic_bytes_per_launch": alg,
                         "traffic_over_algorithmic": (rd + wr) / alg,
                         "source": f"{evidence}/{pre}_fetch, {pre}_write (rocprofv3 --kernel-trace --pmc FETCH_SIZE / "
                                   "WRITE_SIZE, separate passes, median over dispatches; calibrated on "
                                   "tools/pmc_calib.hip)"}
        pv, _ = read_pass(os.path.join(run, f"{pre}_valu"))
        ps, _ = read_pass(os.path.join(run, f"{pre}_stall"))
        t_valu = statistics.median(durations(os.path.join(run, f"{pre}_valu"), kern))
        insts = med(pv, "SQ_INSTS_VALU")
        gui = med(pv, "GRBM_GUI_ACTIVE")
        f_eff = gui / 8 / t_valu
        wave_cyc = med(ps, "SQ_WAVE_CYCLES")
        v = {"kernel": kern, "valu_insts_per_launch": insts, "dispatch_s_profiled": t_valu,
             "effective_clock_hz": f_eff,
             "valu_issue_frac_at_2p4GHz": insts / (t_valu * SIMDS * CLOCK_MAX_HZ / 2),
             "valu_issue_frac_at_effective_clock": insts / (t_valu * SIMDS * f_eff / 2),
             "salu_insts_per_launch": med(pv, "SQ_INSTS_SALU"),
             "valu_active_over_wave_cycles": med(pv, "SQ_ACTIVE_INST_VALU") / med(pv, "SQ_WAVE_CYCLES"),
             "stalls": {"wait_any_over_wave_cycles": med(ps, "SQ_WAIT_ANY") / wave_cyc,
                        "wait_inst_any_over_wave_cycles": med(ps, "SQ_WAIT_INST_ANY") / wave_cyc,
                        "active_inst_any_over_wave_cycles": med(ps, "SQ_ACTIVE_INST_ANY") / wave_cyc,
                        "wait_inst_lds_over_wave_cycles": med(ps, "SQ_WAIT_INST_LDS") / wave_cyc,
                        "active_inst_lds_over_wave_cycles": med(ps, "SQ_ACTIVE_INST_LDS") / wave_cyc,
                        "lds_bank_conflict_over_lds_active": med(ps, "SQ_LDS_BANK_CONFLICT")
                        / max(med(ps, "SQ_LDS_IDX_ACTIVE"), 1.0)},
             "counters_valu_pass": {k: med(pv, k) for k in sorted({k for c in pv.values() for k in c})},
             "counters_stall_pass": {k: med(ps, k) for k in sorted({k for c in ps.values() for k in c})}}
        fd = os.path.join(run, f"{pre}_flop")
        if os.path.isdir(fd):
            pfl, _ = read_pass(fd)
            t_fl = statistics.median(durations(fd, kern))
            f_fl = med(pfl, "GRBM_GUI_ACTIVE") / 8 / t_fl
            flops = 64 * (med(pfl, "SQ_INSTS_VALU_ADD_F32") + med(pfl, "SQ_INSTS_VALU_MUL_F32")) \
                + 128 * med(pfl, "SQ_INSTS_VALU_FMA_F32")
            v["fp32_flops_per_launch"] = flops
            v["fp32_flop_frac_at_2p4GHz"] = flops / t_fl / FP32_PEAK
            v["fp32_flop_frac_at_effective_clock"] = flops / t_fl / (FP32_PEAK * f_fl / CLOCK_MAX_HZ)
            v["flop_pass_effective_clock_hz"] = f_fl
            v["arithmetic_intensity_flop_per_byte"] = flops / traffic[name]["algorithmic_bytes_per_launch"]
            v["counters_flop_pass"] = {k: med(pfl, k) for k in sorted({k for c in pfl.values() for k in c})}
        v["source"] = (f"{evidence}/{pre}_valu, {pre}_stall" + (f", {pre}_flop" if os.path.isdir(fd) else "")
                       + " (rocprofv3 --kernel-trace --pmc, one counter group per run, tools/run_lib.py on the "
                       "product library; median over dispatches)")
        valu[name] = v
    json.dump(traffic, open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w"), indent=1)
    json.dump(valu, open(os.path.join(ROOT, "profiles", "pmc_valu.json"), "w"), indent=1)
    for name in CONFIGS:
        t, v = traffic[name], valu[name]
        print(f"{name:40s} {t['kernel'][:40]:40s} traffic/alg {t['traffic_over_algorithmic']:.3f}  "
              f"clk {v['effective_clock_hz'] / 1e9:.2f} GHz  VALU {v['valu_issue_frac_at_effective_clock']:.3f} "
              f"(2.4: {v['valu_issue_frac_at_2p4GHz']:.3f})  "
              + (f"FP32 {v['fp32_flop_frac_at_effective_clock']:.3f} (2.4: {v['fp32_flop_frac_at_2p4GHz']:.3f})"
                 if "fp32_flops_per_launch" in v else ""))


if __name__ == "__main__":
    main()
