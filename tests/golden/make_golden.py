"""Regenerate the committed fixtures in tests/golden/ (run in the build container).

kaiser_taps.json
    Outputs of the REFERENCE's own KaiserWindow (Core/fir.cpp:48-105), compiled
    unmodified from /root/reference into oracle/_ref/libref_fir.so by
    `make -C oracle ref`.  Float32 bit patterns (hex) of the 1025 taps for every
    decimation index (the call at Core/fft_mt_r2iq.cpp:191), the tap-count
    estimates (Coef = nullptr, the NDEBUG-off printout at fft_mt_r2iq.cpp:51-67)
    and a few extra parameter sets (clamped counts, Beta branches).

iq_golden.json
    IQ from the f64 oracle (oracle/ddc_oracle.c) on seeded synthetic streams:
    per config the first/last 64 output samples and float64 checksums.  These
    freeze the oracle (they are NOT reference-binary outputs: the reference's
    r2iq is unbuildable here) so the GPU box can check the HIP
    path against fixed vectors as well as against the live oracle.

nco_golden.json
    Outputs of the REFERENCE's own fine-tune mixer, pf_mixer's ALGO H
    (shift_limited_unroll_C_sse_{init,inp_c}, Core/pffft/pf_mixer.cpp:750-856),
    compiled unmodified into oracle/_ref/libref_mixer.so by `make -C oracle ref`:
    float32 bit patterns for seeded inputs fed in chunks (the state carries over),
    and long-run probes of a unit input over 64 buffers of 32768 (phase drift).

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from extio_sddc_amd.synth import make_stream  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))

KAISER_EXTRA = [
    # (ntaps, astop, fpass, fstop)
    (101, 60.0, 0.1, 0.15),
    (64, 40.0, 0.2, 0.3),
    (33, 20.0, 0.05, 0.2),
    (-50, 120.0, 0.01, 0.02),     # estimate clamped to 50
    (0, 80.0, 0.1, 0.12),         # estimate only
]

IQ_CONFIGS = [
    # (d, tunebin, lsb, rand, source)
    (0, 1024, 0, 0, "mix"),
    (1, 1024, 1, 1, "uniform"),
    (2, 284, 0, 0, "bench"),
    (3, 3888, 0, 1, "mix"),
    (4, 0, 1, 0, "mix"),
    (5, 4092, 0, 0, "uniform"),
    (6, 2048, 0, 1, "mix"),
]
IQ_NBLK = 2


def f32hex(a: np.ndarray) -> list:
    return [format(int(v), "08x") for v in np.asarray(a, np.float32).view(np.uint32)]


def kaiser_fixture() -> dict:
    if not O.ref_fir_available():
        raise SystemExit("oracle/_ref/libref_fir.so missing: run `make -C oracle ref` where /root/reference exists")
    out = {"source": "reference Core/fir.cpp KaiserWindow, built by oracle/Makefile `ref`", "per_d": [], "extra": []}
    for d in range(O.NDEC):
        bw = np.float32(64.0) / np.float32(1 << d)
        fp = np.float32(np.float32(0.85) * bw) / np.float32(128.0)
        fs = np.float32(np.float32(1.1) * bw) / np.float32(128.0)
        taps = O.ref_kaiser(O.NTAPS, 120.0, float(fp), float(fs))
        est = O.ref_kaiser(0, 120.0, float(fp), float(fs))
        out["per_d"].append({"d": d, "fpass": float(fp), "fstop": float(fs), "estimate": int(est),
                             "taps_f32_hex": f32hex(taps)})
    for (n, a, fp, fs) in KAISER_EXTRA:
        if n <= 0:
            out["extra"].append({"args": [n, a, fp, fs], "estimate": int(O.ref_kaiser(n, a, fp, fs))})
            n_eff = O.ref_kaiser(n, a, fp, fs) if n < 0 else None
            if n_eff is not None:
                out["extra"][-1]["note"] = "tap count clamp"
        else:
            out["extra"].append({"args": [n, a, fp, fs], "taps_f32_hex": f32hex(O.ref_kaiser(n, a, fp, fs))})
    return out


def iq_fixture() -> dict:
    out = {"source": "f64 oracle (oracle/ddc_oracle.c) on extio_sddc_amd.synth streams, gain 1.0",
           "nblk": IQ_NBLK, "cases": []}
    H = O.filter_bank(1.0)
    for (d, tb, lsb, rand, src) in IQ_CONFIGS:
        x = make_stream(IQ_NBLK, src)
        y = O.r2iq(x, IQ_NBLK, d, tb, lsb, rand, H=H)
        out["cases"].append({
            "d": d, "tunebin": tb, "lsb": lsb, "rand": rand, "source": src, "n": int(y.size),
            "head": [[float(v.real), float(v.imag)] for v in y[:64]],
            "tail": [[float(v.real), float(v.imag)] for v in y[-64:]],
            "sum_abs": float(np.sum(np.abs(y))), "sum": [float(y.sum().real), float(y.sum().imag)],
            "max_abs": float(np.max(np.abs(y))),
        })
    return out


NCO_CASES = [
    # (fc, seed, chunk sizes in complex samples; multiples of 128 like the 32768 buffers)
    (0.0123, 11, [512, 384]),
    (-0.271, 12, [256, 128, 512]),
    (0.4999, 13, [640]),
    (1.0e-4, 14, [384, 256]),
]
NCO_LONG = [0.0123, -0.271]
NCO_LONG_BUFFERS = 64
NCO_BUFFER = 32768


def nco_input(seed: int, n: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    return (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64) * np.float32(1000.0)


def nco_probe_index() -> np.ndarray:
    return np.arange(NCO_LONG_BUFFERS) * NCO_BUFFER + (np.arange(NCO_LONG_BUFFERS) * 997) % NCO_BUFFER


def nco_fixture() -> dict:
    if not O.ref_mixer_available():
        raise SystemExit("oracle/_ref/libref_mixer.so missing: run `make -C oracle ref` where /root/reference exists")
    out = {"source": "reference Core/pffft/pf_mixer.cpp shift_limited_unroll_C_sse_{init,inp_c}, "
                     "built by oracle/Makefile `ref`; phase_start 0", "cases": [], "long": []}
    for fc, seed, chunks in NCO_CASES:
        x = nco_input(seed, sum(chunks))
        m = O.RefMixer(fc)
        y, o = [], 0
        for c in chunks:
            y.append(m.apply(x[o:o + c]))
            o += c
        y = np.concatenate(y)
        out["cases"].append({"fc": fc, "seed": seed, "chunks": chunks,
                             "out_f32_hex": f32hex(y.view(np.float32))})
    idx = nco_probe_index()
    for fc in NCO_LONG:
        m = O.RefMixer(fc)
        ones = np.ones(NCO_BUFFER, np.complex64)
        probes = []
        for b in range(NCO_LONG_BUFFERS):
            yb = m.apply(ones)
            probes.append(yb[idx[b] - b * NCO_BUFFER])
        out["long"].append({"fc": fc, "buffers": NCO_LONG_BUFFERS, "buffer": NCO_BUFFER,
                            "probe_f32_hex": f32hex(np.array(probes, np.complex64).view(np.float32))})
    return out


if __name__ == "__main__":
    if "--nco-only" in sys.argv:
        with open(os.path.join(HERE, "nco_golden.json"), "w") as f:
            json.dump(nco_fixture(), f, indent=0)
        raise SystemExit(0)
    with open(os.path.join(HERE, "kaiser_taps.json"), "w") as f:
        json.dump(kaiser_fixture(), f, indent=0)
    with open(os.path.join(HERE, "iq_golden.json"), "w") as f:
        json.dump(iq_fixture(), f, indent=0)
    with open(os.path.join(HERE, "nco_golden.json"), "w") as f:
        json.dump(nco_fixture(), f, indent=0)
    print("wrote", os.listdir(HERE))
