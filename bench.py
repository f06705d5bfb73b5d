#!/usr/bin/env python3
"""Benchmark of the MI355X r2iq DDC hot path (BASELINE.json metric).

metric : input MSamples/s at decim=2 (d=0) + achieved % HBM roofline, 1 GPU; IQ max-rel-err
config : configs[1] "single-channel DDC, 128 MS/s int16 in, decim=2, 1xMI355X"
step   : one pass of the fused frame kernel over one batch of --nblk blocks
         (default 2048 x 65536 int16 = 256 MiB, resident in HBM before timing)

  python bench.py [--gpus N --steps K --warmup W] [--d 0] [--mode single|channels]

N > 1 (launched by torch.distributed.run, one rank per GPU):
  single   : weak scaling — each rank owns its own time segment of the stream
             (independent blocks + their 4096-sample halo; no data-path collective)
  channels : config C5 — one 128 MS/s stream, 1024 tune bins sharded over the
             ranks, the int16 batch broadcast from rank 0 over xGMI (RCCL) every step
Rank 0 prints ONE JSON line.
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

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
BLOCK = 65536
HALF = 4096


def algorithmic_bytes_per_sample(d: int, nch: int = 1, out_bytes: int = 8) -> float:
    """B(d) = 2 B int16 read + one output complex (8 B CF32, 4 B CS16) per 2^(d+1) input
    samples, per channel; the 4/3 frame overlap and the tables are not counted."""
    return 2.0 + nch * float(out_bytes) / (1 << (d + 1))


def make_input(torch, nblk: int, seed: int, device, first_block: int = 0) -> "torch.Tensor":
    """Synthetic 128 MS/s-labelled tone mix + noise (SURVEY.md §8(d) source (i)), int16 in HBM:
    blocks [first_block, first_block + nblk) of ONE global stream, preceded by its real 4096-sample
    history (zeros at the stream start).  The noise is a counter-based function of the global
    sample index, so rank r's segment and its halo are exactly the samples of the one stream that
    rank r - 1's segment ends with (the time-segment hand-off of SURVEY.md §8(e))."""
    s0 = first_block * BLOCK - HALF                      # global index of the buffer's first sample
    t = torch.arange(s0, s0 + HALF + nblk * BLOCK, dtype=torch.float64, device=device)
    x = 9000 * torch.sin(2 * np.pi * 0.0713 * t) + 3000 * torch.sin(2 * np.pi * 0.191 * t)
    # two uniforms per sample from a hash of (index, seed), then Box-Muller: N(0, 300)
    u1 = torch.frac(torch.sin(t * 12.9898 + seed * 78.233) * 43758.5453).abs().clamp_(1e-12, 1.0)
    u2 = torch.frac(torch.sin(t * 39.3468 + seed * 11.135) * 24634.6345).abs()
    x += 300 * torch.sqrt(-2 * torch.log(u1)) * torch.cos(2 * np.pi * u2)
    del u1, u2
    out = x.round().clamp_(-32768, 32767).to(torch.int16)
    out[t < 0] = 0                                        # before the stream start: zero history
    del x, t
    return out


def segment_check(torch, ddc, d: int, nblk: int, rank: int, dev, stream, d_out) -> dict:
    """Time-segment self-check: this rank's launch output d_out (blocks
    [rank nblk, (rank + 1) nblk) of the one stream, with its 4096-sample halo from the previous
    rank's segment) against an independent launch of the same kernel over a 2-block window that
    starts one block earlier.  The window's second block must equal the segment's block bit for
    bit: its history then comes from the window's own first block, i.e. the previous rank's data
    for the segment's first block (rank > 0), so a wrong halo shows.  Checked: the segment's first
    block (rank > 0) and its middle block (every rank).  GPU against GPU (the oracle stays in the
    cpu_baseline leg)."""
    from extio_sddc_amd import output_samples
    per = output_samples(d, 1) * 2                      # floats of one block's output
    first = rank * nblk
    blocks = ([first] if rank > 0 else []) + [first + nblk // 2]
    worst, identical = 0.0, True
    for b in blocks:
        win = make_input(torch, 2, 0x5DDC, dev, first_block=b - 1)
        wout = torch.empty(2 * per, dtype=d_out.dtype, device=dev)
        ddc.process_device(win, 2, wout, stream)
        torch.cuda.synchronize()
        seg = d_out[(b - first) * per:(b - first + 1) * per].double()
        ref = wout[per:].double()
        worst = max(worst, ((seg - ref).abs().max() / ref.abs().max()).item())
        identical = identical and bool(torch.equal(d_out[(b - first) * per:(b - first + 1) * per], wout[per:]))
        del win, wout
    return {"blocks_checked": blocks, "max_rel_err": worst, "bit_identical": identical}


def _cpu_model() -> str:
    try:
        for line in subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout.splitlines():
            if line.startswith("Model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return "unknown"


def cpu_backend_rate(d: int, tunebin: int, sample_in: np.ndarray, nblk_sample: int, budget_s: float):
    """The library's CPU backend (a handle on DEVICE_CPU: the AVX2 restatement of the reference's
    Core/fft_mt_r2iq_avx2.cpp worker, extio_sddc_amd/csrc/cpu/) on this thread, over a bounded
    sample: (input MS/s, seconds timed, its output on the sample)."""
    from extio_sddc_amd import DEVICE_CPU, R2iq, output_samples
    blocks = np.ascontiguousarray(sample_in[HALF: HALF + nblk_sample * BLOCK])
    out = np.empty((output_samples(d, nblk_sample), 2), np.float32)
    with R2iq(gain=1.0, device=DEVICE_CPU) as r:
        assert r.backend == "cpu"
        r.setDecimate(d)
        r.setTuneBin(tunebin)
        L, h = r._L, r._h
        L.sddc_ddc_process_host(h, blocks.ctypes.data, nblk_sample, out.ctypes.data)   # warm tables, pages
        done, t0 = 0, time.perf_counter()
        while True:
            L.sddc_ddc_process_host(h, blocks.ctypes.data, nblk_sample, out.ctypes.data)
            done += nblk_sample
            if time.perf_counter() - t0 >= budget_s:
                break
        dt = time.perf_counter() - t0
        r.TurnOn()   # zero history: the output of the sample from the stream start
        y = r.process(blocks)
    return done * BLOCK / dt / 1e6, dt, y


def cpu_baseline(d: int, tunebin: int, gpu_sample_out, sample_in: np.ndarray, nblk_sample: int,
                 budget_s: float, oracle_port_s: float = 3.0) -> dict:
    """cpu_baseline (1 core): the library's AVX2 CPU backend, timed on this host's core over a
    bounded sample of the same workload; the oracle's scalar float32 port (oracle/ddc_oracle.c)
    is timed next to it for reference.  Also checks the GPU's and the CPU backend's output on
    the sample against the f64 oracle."""
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    v, dt, ycpu = cpu_backend_rate(d, tunebin, sample_in, nblk_sample, budget_s)
    H32 = O.filter_bank(1.0, np.float32)
    O.r2iq(sample_in, 1, d, tunebin, dtype=np.float32, H=H32)      # warm tables
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < oracle_port_s:
        O.r2iq(sample_in, nblk_sample, d, tunebin, dtype=np.float32, H=H32)
        done += nblk_sample
    port = done * BLOCK / (time.perf_counter() - t0) / 1e6
    ref = O.r2iq(sample_in, nblk_sample, d, tunebin)                # f64 checker
    return {
        "value": v, "unit": "input MSamples/s", "cores": 1, "kind": "port",
        "sample": f"{nblk_sample} blocks x 65536 int16 (tone mix), repeated for {dt:.1f} s, d={d}, "
                  f"tunebin={tunebin}: the library's AVX2 CPU backend (restatement of "
                  f"Core/fft_mt_r2iq_avx2.cpp without FFTW), 1 thread",
        "cpu_model": _cpu_model(), "host_nproc": os.cpu_count(),
        "oracle_f32_port_1core_MSps": port,
        "iq_max_rel_err_cpu_backend_vs_oracle_f64": O.max_rel_err(ycpu, ref),
        "iq_max_rel_err_gpu_vs_oracle_f64": O.max_rel_err(gpu_sample_out, ref),
        "iq_rms_rel_err_gpu_vs_oracle_f64": O.rms_rel_err(gpu_sample_out, ref),
    }


# one CPU-backend instance, pinned to one CPU; ctypes only (no torch, never touches a GPU)
_CPU_WORKER = r"""
import ctypes, os, sys, time, numpy as np
lib_path, x_path, nblk, d, tb, budget, cpu = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), float(sys.argv[6]), int(sys.argv[7])
os.sched_setaffinity(0, {cpu})
L = ctypes.CDLL(lib_path)
P = ctypes.c_void_p
L.sddc_ddc_create.argtypes = [ctypes.c_float, ctypes.c_int, ctypes.POINTER(P)]
for f in ("sddc_ddc_set_decimation", "sddc_ddc_set_tunebin"): getattr(L, f).argtypes = [P, ctypes.c_int]
L.sddc_ddc_process_host.argtypes = [P, P, ctypes.c_int, P]
h = P()
assert L.sddc_ddc_create(1.0, -1, ctypes.byref(h)) == 0
assert L.sddc_ddc_set_decimation(h, d) == 0 and L.sddc_ddc_set_tunebin(h, tb) == 0
x = np.ascontiguousarray(np.load(x_path)[4096:4096 + nblk * 65536])
out = np.empty(nblk * (32768 >> d) * 2, np.float32)
L.sddc_ddc_process_host(h, x.ctypes.data, nblk, out.ctypes.data)
done, t0 = 0, time.perf_counter()
while time.perf_counter() - t0 < budget:
    assert L.sddc_ddc_process_host(h, x.ctypes.data, nblk, out.ctypes.data) == 0; done += nblk
print(done, time.perf_counter() - t0)
"""


def _cgroup_cpu_quota():
    """CPUs this process may keep busy by its cgroup (v2 cpu.max, v1 cfs quota), or None if unlimited."""
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", None)):
        try:
            with open(path) as f:
                txt = f.read().strip()
        except OSError:
            continue
        if parse:
            q, per = parse(txt)
            if q == "max":
                return None
            return max(1, int(int(q) // int(per)))
        q = int(txt)
        if q <= 0:
            return None
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            return max(1, q // int(f.read().strip()))
    return None


def _distinct_core_cpus():
    """CPUs of this process's affinity set, one per physical core (SMT siblings skipped), capped
    by the cgroup CPU quota when one is set: (cpus, affinity size, quota or None)."""
    try:
        aff = sorted(os.sched_getaffinity(0))
    except AttributeError:
        aff = list(range(os.cpu_count() or 1))
    quota = _cgroup_cpu_quota()
    picked, seen = [], set()
    for c in aff:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/core_id") as f:
                core = f.read().strip()
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id") as f:
                pkg = f.read().strip()
            key = (pkg, core)
        except OSError:
            key = c
        if key in seen:
            continue
        seen.add(key)
        picked.append(c)
    if quota is not None:
        picked = picked[:quota]
    return picked, len(aff), quota


def cpu_baseline_all_cores(d: int, tunebin: int, sample_in: np.ndarray, nblk_sample: int, budget_s: float) -> dict:
    """one independent CPU-backend instance per physical core of this
    process's affinity set (capped by the cgroup CPU quota, which the line states), each a child
    process pinned to its own core that never touches the GPU; aggregate input MS/s."""
    import tempfile
    from extio_sddc_amd._lib import LIB_PATH
    cpus, naff, quota = _distinct_core_cpus()
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        path = os.path.join(td, "sample.npy")
        np.save(path, sample_in)
        env = dict(os.environ, OMP_NUM_THREADS="1")
        ps = [subprocess.Popen([sys.executable, "-c", _CPU_WORKER, LIB_PATH, path, str(nblk_sample), str(d),
                                str(tunebin), str(budget_s), str(c)], stdout=subprocess.PIPE, text=True, env=env)
              for c in cpus]
        total = 0.0
        for p in ps:
            out, _ = p.communicate(timeout=budget_s * 4 + 60)
            done, dt = out.split()
            total += int(done) * BLOCK / float(dt)
    return {"value": total / 1e6, "unit": "input MSamples/s", "cores": len(cpus), "kind": "port",
            "cpus": cpus, "affinity_cpus": naff, "cgroup_cpu_quota": quota,
            "core_budget": ("every physical core of the affinity set" if quota is None else
                            f"the cgroup CPU quota ({quota} CPUs), one per physical core"),
            "sample": f"{len(cpus)} independent CPU-backend processes, one per physical core (pinned), "
                      f"x the 1-core sample, {budget_s:.1f} s each"}


def reference_equivalent(backend_msps: float, d: int):
    """Scale an on-box CPU-backend timing by the committed backend-vs-reference ratio
    (profiles/cpu_calibration.json, tools/cpu_calib.py): an estimate, labelled as such."""
    try:
        with open(os.path.join(ROOT, "profiles", "cpu_calibration.json")) as f:
            r = json.load(f)["ratio_reference_over_avx2_backend"][str(d)]
        return {"value": backend_msps * r, "ratio": r, "kind": "cross-CPU estimate",
                "basis": "reference AVX2 r2iq (survey probe) / this library's AVX2 backend, both measured on 1 core "
                         "of the survey's Xeon container (tools/cpu_calib.py), applied to this host's CPU: an "
                         "estimate across CPU types, not a measurement of the reference here (the reference "
                         "r2iq needs <fftw3.h>, absent from the image); the measured baseline is `value`"}
    except Exception:
        return None


def load_traffic(workload: str):
    """Per-launch HBM bytes measured with rocprofv3 --pmc (profiles/pmc_traffic.json), if present."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            return json.load(f).get(workload)
    except Exception:
        return None


# VALU issue ceiling: 4 SIMDs x 256 CUs, one wave64 VALU instruction per SIMD every 2 cycles
# (MI355X_MICROARCH.md "Wave scheduling"), at the 2400 MHz max clock
VALU_SIMDS = 1024
VALU_CYCLES_PER_INST = 2.0
CLOCK_HZ = 2.4e9
VALU_PEAK_INST_PER_S = VALU_SIMDS * CLOCK_HZ / VALU_CYCLES_PER_INST
FP32_PEAK = 157.3e12   # FLOP/s, vector FP32 at 2.4 GHz (MI355X_MICROARCH.md)


def load_valu(workload: str):
    """Per-launch VALU wave-instructions counted with rocprofv3 --pmc SQ_INSTS_VALU
    (profiles/pmc_valu.json, tools/pmc_valu.py), if present."""
    p = os.path.join(ROOT, "profiles", "pmc_valu.json")
    try:
        with open(p) as f:
            return json.load(f).get(workload)
    except Exception:
        return None


def compute_roofline(workload: str, kern_ms: float):
    """The compute-side bounds of a launch, from the per-config counters of
    profiles/pmc_valu.json (tools/gpu_pmc_configs.sh + tools/pmc_configs.py): VALU issue =
    counted VALU wave-instructions per launch / this run's HIP-event time, against the chip's
    wave-instruction issue rate at the 2.4 GHz maximum clock and at the effective clock the
    counters' pass measured (GRBM_GUI_ACTIVE / 8 / dispatch time, MI355X_MICROARCH.md 'DVFS
    give-back'); and, where counted, FP32 FLOP/s against the 157.3 TF vector peak, scaled the
    same way.  None when the workload has no committed count."""
    v = load_valu(workload)
    if not v:
        return None
    n = float(v["valu_insts_per_launch"])
    t = kern_ms * 1e-3
    ach = n / t
    f_eff = v.get("effective_clock_hz")
    out = {"bound": "valu-issue", "achieved": ach, "peak": VALU_PEAK_INST_PER_S, "unit": "wave-instructions/s",
           "frac": ach / VALU_PEAK_INST_PER_S, "valu_insts_per_launch": n,
           "peak_basis": f"{VALU_SIMDS} SIMDs x {CLOCK_HZ / 1e9:.1f} GHz / {VALU_CYCLES_PER_INST:g} cycles per "
                         "wave64 VALU instruction",
           "source": v.get("source")}
    if f_eff:
        peak_eff = VALU_SIMDS * f_eff / VALU_CYCLES_PER_INST
        out.update({"effective_clock_hz": f_eff, "peak_at_effective_clock": peak_eff,
                    "frac_at_effective_clock": ach / peak_eff})
    if v.get("fp32_flops_per_launch"):
        fl = float(v["fp32_flops_per_launch"])
        out["fp32"] = {"flops_per_launch": fl, "achieved_tflops": fl / t / 1e12, "peak_tflops": FP32_PEAK / 1e12,
                       "frac": fl / t / FP32_PEAK,
                       "frac_at_effective_clock": fl / t / (FP32_PEAK * f_eff / CLOCK_HZ) if f_eff else None,
                       "flop_per_algorithmic_byte": v.get("arithmetic_intensity_flop_per_byte"),
                       "basis": "64 x (ADD_F32 + MUL_F32) + 128 x FMA_F32 wave-instructions (SQ_INSTS_VALU_*_F32)"}
    if v.get("stalls"):
        out["stalls"] = v["stalls"]
    return out


def sweep_counters(name: str, kern_ms: float) -> dict:
    """traffic + compute of one sweep config (profiles/pmc_*.json keys = the config names)."""
    key = "single d=0 nblk=2048" if name == "C3 decim 2" else name
    t = load_traffic(key)
    return {"traffic": t["hbm_bytes_per_launch"] if t else None,
            "traffic_over_algorithmic": t.get("traffic_over_algorithmic") if t else None,
            "compute": compute_roofline(key, kern_ms)}


class ChannelRun:
    """C5 on this rank: channels [lo, hi) of `nch` tune bins 0, 4, ..., 4 (nch - 1) over one shared
    int16 stream.  N > 1: rank 0 holds the batch and every step sends it to all ranks
    (shard.broadcast_samples, scatter + all-gather by default), batch i + 1's transfer running
    while batch i is processed (double-buffered input, shard.pipelined_batches)."""

    def __init__(self, torch, ddc, nch, nblk, d, out_dtype, dev, stream, world, rank, method):
        from extio_sddc_amd import output_samples
        from extio_sddc_amd.shard import channel_shard
        self.torch, self.ddc, self.nblk, self.stream, self.method = torch, ddc, nblk, stream, method
        self.world, self.dev = world, dev
        lo, hi = channel_shard(nch, world, rank)
        self.tbs = [4 * c for c in range(nch)][lo:hi]
        self.nch_local = len(self.tbs)
        self.d_in = make_input(torch, nblk, 0x5DDC, dev) if rank == 0 else \
            torch.empty(HALF + nblk * BLOCK, dtype=torch.int16, device=dev)
        self.d_out = torch.empty((self.nch_local, output_samples(d, nblk) * 2), dtype=out_dtype, device=dev)
        self.batches = None
        self.bcast_check = None
        if world > 1:
            self.bcast_check = self.check_broadcast()
            from extio_sddc_amd.shard import pipelined_batches
            self.d_in2 = self.d_in.clone()
            self.batches = pipelined_batches([self.d_in, self.d_in2], None, src=0, method=method)   # closed after timing

    def check_broadcast(self) -> dict:
        """One broadcast of the real batch with the chosen method, then the batch's checksum on
        every rank against rank 0's (int64 sum of the int32 view and of its squares' low bits):
        a method that delivers wrong bytes on this backend falls back to the plain broadcast."""
        import torch.distributed as dist
        from extio_sddc_amd.shard import broadcast_samples
        torch = self.torch

        def checksum():
            v = self.d_in.view(torch.int32).to(torch.int64)
            return torch.stack([v.sum(), (v * v).remainder(1 << 31).sum()])
        ref = checksum() if dist.get_rank() == 0 else torch.zeros(2, dtype=torch.int64, device=self.d_in.device)
        broadcast_samples(self.d_in, src=0, method=self.method)
        got = checksum()
        dev = self.d_in.device if dist.get_backend() == "nccl" else "cpu"
        ref = ref.to(dev)
        dist.broadcast(ref, src=0)
        bad = torch.tensor([0 if torch.equal(got.to(dev), ref) else 1], dtype=torch.int32, device=dev)
        dist.all_reduce(bad, op=dist.ReduceOp.MAX)
        ok = bad.item() == 0
        out = {"method": self.method, "checksum_equal_on_all_ranks": ok}
        if not ok and self.method != "bcast":
            self.method = "bcast"
            broadcast_samples(self.d_in, src=0, method="bcast")
            out["fallback"] = "bcast"
        return out

    def step(self):
        src = next(self.batches) if self.batches is not None else self.d_in
        self.ddc.process_channels_device(src, self.nblk, self.tbs, self.d_out, self.stream)

    def close(self):
        if self.batches is not None:
            self.batches.close()   # waits for the prefetched broadcast on every rank
            self.batches = None

    def broadcast_and_compute_alone(self, backend: str, reps: int = 10) -> dict:
        """The collective and the compute, each timed alone between barriers (max over ranks), so
        the line shows which of the two bounds the pipelined step."""
        import torch.distributed as dist
        from extio_sddc_amd.shard import broadcast_samples
        torch = self.torch
        res = []
        for phase in ("broadcast", "compute"):
            dist.barrier()
            torch.cuda.synchronize()
            tb0 = time.perf_counter()
            for _ in range(reps):
                if phase == "broadcast":
                    broadcast_samples(self.d_in, src=0, method=self.method)
                else:
                    self.ddc.process_channels_device(self.d_in, self.nblk, self.tbs, self.d_out, self.stream)
            torch.cuda.synchronize()
            res.append((time.perf_counter() - tb0) / reps)
        tt = torch.tensor(res, dtype=torch.float64, device=self.dev if backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        b_s, c_s = tt.tolist()
        batch_bytes = self.d_in.numel() * 2
        return {"method": self.method, "bytes_per_batch": batch_bytes, "ms": b_s * 1e3,
                "GBps_inbound_per_rank": batch_bytes / b_s / 1e9,
                "compute_ms_per_rank": c_s * 1e3, "reps": reps,
                "note": "each timed alone between barriers, max over ranks; the timed steps overlap "
                        "batch i + 1's broadcast with batch i's compute"}


def c5_leg(torch, dist, args, dev, stream, world: int, rank: int, backend: str) -> dict:
    """Config C5 (BASELINE.json configs[4]) beside the headline: 1024 channels at d = 4 (decim 32)
    from one stream, channels sharded over the world's ranks (strong scaling: the stream's rate
    is fixed, each rank computes 1024 / N channels), the int16 batch sent to every rank each step.
    Warm-up to a time floor the ranks agree on, then --c5-steps batches between barrier +
    synchronize, max over ranks."""
    from extio_sddc_amd import R2iq
    d5, nblk5, steps = 4, args.c5_nblk, args.c5_steps
    ddc5 = R2iq(gain=1.0, device=dev.index)
    ddc5.setDecimate(d5)
    ch = ChannelRun(torch, ddc5, 1024, nblk5, d5, torch.float32, dev, stream, world, rank, args.bcast)
    tw0 = time.perf_counter()
    while True:
        for _ in range(5):
            ch.step()
        torch.cuda.synchronize()
        done = (time.perf_counter() - tw0) >= 0.1
        if world > 1:
            flag = torch.tensor([1 if done else 0], dtype=torch.int32, device=dev if backend == "nccl" else "cpu")
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            done = bool(flag.item())
        if done:
            break
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ch.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ch.close()
    info = ch.broadcast_and_compute_alone(backend) if world > 1 else None
    t = torch.tensor([wall], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall = t.item()
    ms = wall * 1e3 / steps
    in_msps = nblk5 * BLOCK * steps / wall / 1e6
    # per rank: the whole int16 batch in + its channels' CF32 outputs
    bytes_rank = nblk5 * BLOCK * algorithmic_bytes_per_sample(d5, ch.nch_local, 8)
    out = {"config": "C5 1024-channel DDC from one stream, channels sharded over the ranks",
           "d": d5, "decim": 2 << d5, "channels": 1024, "channels_per_rank": ch.nch_local, "n_gpus": world,
           "blocks_per_batch": nblk5, "steps": steps, "ms_per_step": ms,
           "input_MSps": in_msps, "channel_MSps": in_msps * 1024,
           "scaling": "strong (fixed stream, 1024 / N channels per rank)",
           "roofline_frac_per_rank": bytes_rank / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
           "bytes_per_rank_per_batch": bytes_rank,
           "broadcast": info or ("none (one rank)" if world == 1 else None),
           "broadcast_check": ch.bcast_check}
    if world == 1 and nblk5 == 256:   # the profiled launch (tools/gpu_pmc_configs.sh): one rank, all channels
        out.update(sweep_counters("C5 1024 channels d=4 nblk=256", ms))
    del ch, ddc5
    torch.cuda.empty_cache()
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults reach the power-managed steady state: the first ~10 ms of back-to-back
    # launches run ~20 % slower; 50 + 100 steps of 2048 blocks take ~50 ms
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--warmup-ms", type=float, default=250.0,
                    help="after --warmup steps, keep launching untimed steps until this much wall time "
                         "has passed, so the timed steps run at steady-state clocks (DESIGN.md §5)")
    ap.add_argument("--d", "--decim-index", dest="d", type=int, default=0,
                    help="decimation index (0 = decim 2); use --decim-index under torchrun")
    ap.add_argument("--tunebin", type=int, default=1024)
    ap.add_argument("--nblk", type=int, default=2048, help="blocks of 65536 per step per GPU")
    ap.add_argument("--mode", choices=["single", "channels"], default="single")
    ap.add_argument("--streams", type=int, default=1,
                    help="single mode: consecutive batches alternate over this many HIP streams (each with its "
                         "own output buffer), so one batch's launch tail overlaps the next batch's start; the "
                         "roofline then comes from a separate single-stream run of the same steps.  Default 1 "
                         "since round 5: with the static split two streams measured slower (DESIGN.md §5)")
    ap.add_argument("--channels", type=int, default=1024)
    ap.add_argument("--bcast", choices=["sag", "bcast"], default="sag",
                    help="C5 input broadcast for N > 1: scatter + all-gather over all links (sag) or one "
                         "broadcast collective (shard.broadcast_samples)")
    ap.add_argument("--no-c5", action="store_true",
                    help="skip the same-run C5 leg (1024 channels at d = 4, sharded over the ranks)")
    ap.add_argument("--c5-nblk", type=int, default=256, help="C5 leg: blocks of 65536 per batch")
    ap.add_argument("--c5-steps", type=int, default=20, help="C5 leg: timed batches")
    ap.add_argument("--c5-timeout", type=float, default=120.0, help="C5 leg watchdog, seconds")
    ap.add_argument("--cpu-budget", type=float, default=10.0, help="seconds of CPU-baseline work")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sweep", action="store_true",
                    help="skip the same-run C3 decim sweep / C4 VHF lines (BASELINE.md §3)")
    ap.add_argument("--cs16", type=float, default=0.0,
                    help="CS16 output with this scale (int16 = rint(x * scale)); 0 = CF32")
    ap.add_argument("--fine-tune", type=float, default=0.0,
                    help="fused fine-tune NCO frequency (fraction of the output rate); 0 = off")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from extio_sddc_amd import R2iq, output_samples

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    # one rank per GPU; SDDC_BENCH_BACKEND=gloo lets a rehearsal put several ranks on one GPU
    # (RCCL refuses two ranks on one device); the driver's runs use the default, RCCL
    backend = os.environ.get("SDDC_BENCH_BACKEND", "nccl")
    ngpu = torch.cuda.device_count()
    gpu = local % ngpu if backend == "gloo" else local
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    d, nblk = args.d, args.nblk
    ddc = R2iq(gain=1.0, device=gpu)
    ddc.setDecimate(d)
    ddc.setTuneBin(args.tunebin)
    if args.fine_tune:
        if args.mode != "single":
            raise SystemExit("--fine-tune is single-channel only")
        ddc.setFineTune(args.fine_tune)
        args.no_cpu_baseline = True   # the CPU leg is the plain DDC
    out_bytes = 8
    out_dtype = torch.float32
    if args.cs16:
        ddc.setOutputFormat("CS16", args.cs16)
        out_bytes, out_dtype = 4, torch.int16
        args.no_cpu_baseline = True   # the CPU leg compares CF32
    stream = torch.cuda.current_stream()

    if args.mode == "single":
        # weak scaling: rank r owns segment r of one stream (its own blocks + the real halo)
        d_in = make_input(torch, nblk, 0x5DDC, dev, first_block=rank * nblk)
        d_out = torch.empty(output_samples(d, nblk) * 2, dtype=out_dtype, device=dev)
        nch_local = 1
        nstreams = max(1, args.streams)
        # pipelined batches: step i on stream i % S into output S (the streams start behind `stream`
        # and `stream` waits for all of them at the end of the timed region)
        pstreams = [stream] + [torch.cuda.Stream(device=dev) for _ in range(nstreams - 1)]
        pouts = [d_out] + [torch.empty_like(d_out) for _ in range(nstreams - 1)]
        step_i = [0]

        def step():
            i = step_i[0] % nstreams
            step_i[0] += 1
            ddc.process_device(d_in, nblk, pouts[i], pstreams[i])

        def fork():   # the other streams start after the work queued on `stream`
            ev = torch.cuda.Event()
            ev.record(stream)
            for ps in pstreams[1:]:
                ps.wait_event(ev)

        def join():   # `stream` waits for the other streams
            for ps in pstreams[1:]:
                ev = torch.cuda.Event()
                ev.record(ps)
                stream.wait_event(ev)
        samples_per_step_all = nblk * BLOCK * world
        workload = f"single d={d} nblk={nblk}" + (f" fine_tune={args.fine_tune}" if args.fine_tune else "") \
            + (" cs16" if args.cs16 else "")
    else:
        ch = ChannelRun(torch, ddc, args.channels, nblk, d, out_dtype, dev, stream, world, rank, args.bcast)
        d_in, d_out, tbs, nch_local, step = ch.d_in, ch.d_out, ch.tbs, ch.nch_local, ch.step
        samples_per_step_all = nblk * BLOCK          # one shared stream
        nstreams = 1

        def fork():
            pass

        def join():
            pass
        workload = f"channels d={d} nblk={nblk} nch={args.channels}" + (" cs16" if args.cs16 else "")

    tw0 = time.perf_counter()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # time floor on the warm-up: the first ~10 ms of back-to-back launches run ~20 % slower
    # while the clocks ramp, so a short --warmup alone would time the ramp, not the kernel
    # (every rank runs the same number of extra steps: the ranks agree on stopping, so the
    # channel mode's collectives stay matched)
    extra = 0
    while True:
        done = (time.perf_counter() - tw0) * 1e3 >= args.warmup_ms
        if world > 1:
            flag = torch.tensor([1 if done else 0], dtype=torch.int32, device=dev if backend == "nccl" else "cpu")
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            done = bool(flag.item())
        if done:
            break
        for _ in range(10):
            step()
        extra += 10
        torch.cuda.synchronize()
    warmup_ms = (time.perf_counter() - tw0) * 1e3
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    fork()
    for _ in range(args.steps):
        step()
    join()
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps          # per step on the launch stream(s)
    if args.mode == "channels":
        ch.close()                                        # waits for the prefetched broadcast
    t = torch.tensor([wall, kern_ms], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall, kern_ms = t.tolist()

    # pipelined batches: the kernel's own launch duration (roofline, rocprof) from the same steps
    # launched back to back on one stream, timed the same way (max over ranks)
    single = None
    if nstreams > 1:
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t1 = time.perf_counter()
        e0.record(stream)
        for _ in range(args.steps):
            ddc.process_device(d_in, nblk, d_out, stream)
        e1.record(stream)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        tt = torch.tensor([time.perf_counter() - t1, e0.elapsed_time(e1) / args.steps], dtype=torch.float64,
                          device=dev if backend == "nccl" else "cpu")
        if world > 1:
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        wall1, kern1 = tt.tolist()
        single = {"streams": nstreams, "ms_per_step_single_stream": wall1 * 1e3 / args.steps,
                  "value_single_stream": samples_per_step_all * args.steps / wall1 / 1e6,
                  "kernel_ms_single_stream": kern1,
                  "note": "value: consecutive batches alternate over the streams (each its own output buffer), "
                          "so one launch's tail overlaps the next one's start; roofline: the kernel's own "
                          "launch duration, from the same steps on one stream"}
        kern_ms = kern1

    # N > 1 channels: the collective and the compute, each timed alone (max over ranks), so the
    # line shows which of the two bounds the pipelined step
    bcast_info = None
    if args.mode == "channels" and world > 1:
        bcast_info = ch.broadcast_and_compute_alone(backend)


    # BASELINE.md §3 / SURVEY §8(d) C3 + C4 in the same run, while the clocks are at their
    # steady state: GPU rate and roofline per config (the headline value stays the d=0 line)
    sweep = []
    if rank == 0 and world == 1 and args.mode == "single" and not args.no_sweep and not (args.cs16 or args.fine_tune):
        for dd, lsb, rnd, name in [(0, 0, 0, "C3 decim 2"), (1, 0, 0, "C3 decim 4"), (2, 0, 0, "C3 decim 8"),
                                   (3, 0, 0, "C3 decim 16"), (4, 0, 0, "C3 decim 32"),
                                   (1, 1, 1, "C4 VHF decim 4, sideband invert, rand")]:
            ddc.setDecimate(dd)
            ddc.setSideband(bool(lsb))
            ddc.updateRand(bool(rnd))
            for _ in range(30):
                ddc.process_device(d_in, nblk, d_out, stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(50):
                ddc.process_device(d_in, nblk, d_out, stream)
            e1.record(stream)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 50
            sweep.append(dict({"config": name, "d": dd, "lsb": lsb, "rand": rnd, "gpu_input_MSps": nblk * BLOCK / ms / 1e3,
                               "roofline_frac": nblk * BLOCK * algorithmic_bytes_per_sample(dd) / (ms * 1e-3) / 1e9
                               / HBM_PEAK_GBS, "kernel_ms": ms}, **(sweep_counters(name, ms) if nblk == 2048 else {})))
        ddc.setDecimate(d)
        ddc.setSideband(False)
        ddc.updateRand(False)
        ddc.process_device(d_in, nblk, d_out, stream)   # d_out holds the headline config again
        torch.cuda.synchronize()

    # single mode: every rank checks its segment (the halo'd first block, a middle block) against
    # a separate launch over a window starting a block earlier; max error / all identical over ranks.
    # After the sweep: its host round trips idle the GPU, and the sweep's first config (d = 0) would
    # then run on a clock still ramping back up
    seg_check = None
    if args.mode == "single" and not (args.cs16 or args.fine_tune):
        seg_check = segment_check(torch, ddc, d, nblk, rank, dev, stream, d_out)
        if world > 1:
            tt = torch.tensor([seg_check["max_rel_err"], 0.0 if seg_check["bit_identical"] else 1.0],
                              dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            seg_check = {"ranks": world, "blocks_checked_rank0": seg_check["blocks_checked"],
                         "max_rel_err_over_ranks": tt[0].item(), "bit_identical_all_ranks": tt[1].item() == 0.0}

    value = samples_per_step_all * args.steps / wall / 1e6
    # roofline of the dominant kernel on THIS rank's launch
    alg_bytes = nblk * BLOCK * algorithmic_bytes_per_sample(d, nch_local, out_bytes)
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    traffic = load_traffic(workload)

    result = {
        "metric": "input MSamples/s at decim=2 + achieved % HBM roofline, 1 GPU; IQ max-rel-err",
        "value": value, "unit": "input MSamples/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "warmup_ms": warmup_ms, "warmup_extra_steps": extra,
        "ms_per_step": wall * 1e3 / args.steps, "higher_is_better": True,
        "scaling": "weak" if args.mode == "single" else "strong",
        "vs_baseline": None, "dtype": "f32 (int16 in, " + ("int16 IQ out)" if args.cs16 else "complex64 out)"), "data": "synthetic",
        "config": {"workload": "single-channel DDC, 128 MS/s int16 in, decim=2, 1xMI355X"
                   if (args.mode == "single" and d == 0 and not args.fine_tune and not args.cs16) else workload,
                   "decim": 2 << d, "d": d, "tunebin": args.tunebin, "blocks_per_step_per_gpu": nblk,
                   "block_samples": BLOCK, "mode": args.mode,
                   "channels": args.channels if args.mode == "channels" else 1,
                   "parallelism": f"time-segments x{world}" if args.mode == "single" else f"channels x{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic["hbm_bytes_per_launch"] if traffic else None,
                     "traffic_unit": "bytes per launch (rocprofv3 FETCH_SIZE/WRITE_SIZE, calibrated)",
                     "traffic_detail": traffic,
                     "kernel": ((traffic or {}).get("kernel") or ("r2iq_fs_kernel" if d == 0 else "r2iq_persistent_kernel"))
                               if args.mode == "single" else "r2iq_channels_kernel",
                     "kernel_ms_per_launch": kern_ms,
                     "algorithmic_bytes_per_launch": alg_bytes,
                     "bytes_per_input_sample": algorithmic_bytes_per_sample(d, nch_local, out_bytes),
                     "compute": compute_roofline(workload, kern_ms)},
    }

    if single:
        result["pipelining"] = single
    if bcast_info:
        result["broadcast"] = bcast_info
    if args.mode == "channels" and world > 1:
        result["broadcast_check"] = ch.bcast_check
    if seg_check:
        result["segment_check"] = seg_check
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        ns = 16
        sample = d_in[: HALF + ns * BLOCK].cpu().numpy()
        if args.mode == "single":
            gout = d_out[: output_samples(d, ns) * 2].cpu().numpy().view(np.complex64)
            tb = args.tunebin
        else:
            gout = d_out[0, : output_samples(d, ns) * 2].cpu().numpy().view(np.complex64)
            tb = tbs[0]
        # d_out holds the whole batch; its first ns blocks depend only on the first ns blocks
        cb = cpu_baseline(d, tb, gout, sample, ns, args.cpu_budget)
        try:
            cb["all_cores"] = cpu_baseline_all_cores(d, tb, sample, ns, args.cpu_budget)
        except Exception as e:   # the 1-core figure stands on its own
            cb["all_cores"] = {"error": str(e)}
        cb["reference_equivalent_cross_cpu_estimate"] = reference_equivalent(cb["value"], d)
        result["cpu_baseline"] = cb
        result["gpu_over_cpu_backend_1core"] = value / cb["value"]
        result["iq_max_rel_err"] = cb.pop("iq_max_rel_err_gpu_vs_oracle_f64")
        result["iq_rms_rel_err"] = cb.pop("iq_rms_rel_err_gpu_vs_oracle_f64")
    if sweep:
        for line in sweep:
            if not args.no_cpu_baseline and not (line["lsb"] or line["rand"]):
                dd, ns = line["d"], 16
                ddc.setDecimate(dd)
                ddc.process_device(d_in, ns, d_out, stream)
                torch.cuda.synchronize()
                gout = d_out[: output_samples(dd, ns) * 2].cpu().numpy().view(np.complex64)
                cbd = cpu_baseline(dd, args.tunebin, gout, d_in[: HALF + ns * BLOCK].cpu().numpy(), ns, 2.0, 1.0)
                line["cpu_backend_1core_MSps"] = cbd["value"]
                line["cpu_oracle_port_1core_MSps"] = cbd["oracle_f32_port_1core_MSps"]
                line["cpu_reference_equivalent_cross_cpu_estimate_MSps"] = (reference_equivalent(cbd["value"], dd) or {}).get("value")
                line["iq_max_rel_err"] = cbd["iq_max_rel_err_gpu_vs_oracle_f64"]
        result["sweep"] = sweep
    if rank == 0:
        result["host"] = platform.node()
    # C5 in the same run (BASELINE.json configs[4]): 1024 channels at d = 4
    # from one shared stream, sharded over the ranks with the int16 batch sent to every rank
    # (scatter + all-gather), so the driver's 1/2/4/8-GPU runs measure the sharded C5 path too.
    # Reported beside the headline, which it does not change.  It runs after the headline is
    # complete, under a watchdog: should its collectives stall, rank 0 still prints the line
    # (with the C5 error) and every rank exits.
    if args.mode == "single" and not (args.no_c5 or args.cs16 or args.fine_tune):
        import threading

        def stalled():
            # the headline stands; the stall is reported and the process exits non-zero (3) so the
            # driver and torchrun see the C5 leg's collective hang
            if rank == 0:
                print(json.dumps(dict(result, c5={"error": f"stalled: no result within {args.c5_timeout:.0f} s",
                                                  "exit_code": 3})), flush=True)
            print(f"bench.py rank {rank}: C5 leg stalled after {args.c5_timeout:.0f} s, exiting 3",
                  file=sys.stderr, flush=True)
            os._exit(3)
        dog = threading.Timer(args.c5_timeout, stalled)
        dog.daemon = True
        dog.start()
        try:
            result["c5"] = c5_leg(torch, dist, args, dev, stream, world, rank, backend)
        except Exception as e:   # the headline stands on its own
            result["c5"] = {"error": f"{type(e).__name__}: {e}"}
        dog.cancel()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
