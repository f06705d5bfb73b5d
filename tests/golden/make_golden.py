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


if __name__ == "__main__":
    with open(os.path.join(HERE, "kaiser_taps.json"), "w") as f:
        json.dump(kaiser_fixture(), f, indent=0)
    with open(os.path.join(HERE, "iq_golden.json"), "w") as f:
        json.dump(iq_fixture(), f, indent=0)
    print("wrote", os.listdir(HERE))
