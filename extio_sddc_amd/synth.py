"""Synthetic int16 ADC streams (no USB; the reference's tests fake the producer too).

Sources, all seeded (default seed 0x5DDC, numpy PCG64):
  "mix"   round(9000 sin(2 pi 0.0713 n) + 3000 sin(2 pi 0.191 n) + N(0, 300)), clipped
  "bench" 16384 sin(2 pi n / 64)   — unittest/benchmark_test.cpp:80-84 fake producer
  "uniform" uniform int16          — exercises the RAND de-randomiser (50 % odd LSBs)
  "zeros" all zero                 — signal_integrity_test.cpp zero-input case
  "oob"   strong out-of-band tone + weak in-band tone (accuracy stress)
A stream is [4096 history | nblk * 65536] samples; the history is zero, the
reference's state after TurnOn (SURVEY.md §7 "History at start").
"""
from __future__ import annotations

import numpy as np

HALF_FFT = 4096
BLOCK = 65536
SEED = 0x5DDC


def make_stream(nblk: int, source: str = "mix", seed: int = SEED, history: bool = True) -> np.ndarray:
    n = nblk * BLOCK
    rng = np.random.default_rng(seed)
    t = np.arange(n, dtype=np.float64)
    if source == "mix":
        x = 9000 * np.sin(2 * np.pi * 0.0713 * t) + 3000 * np.sin(2 * np.pi * 0.191 * t) + rng.normal(0, 300, n)
    elif source == "bench":
        x = 16384 * np.sin(2 * np.pi * t / 64)
    elif source == "uniform":
        x = rng.integers(-32768, 32768, n).astype(np.float64)
    elif source == "zeros":
        x = np.zeros(n)
    elif source == "oob":
        # 30000-unit tone far outside a narrow channel + a 3-unit tone inside it
        x = 30000 * np.sin(2 * np.pi * 0.37 * t) + 3 * np.sin(2 * np.pi * 0.1253 * t) + rng.normal(0, 1, n)
    else:
        raise ValueError(source)
    x = np.clip(np.round(x), -32768, 32767).astype(np.int16)
    if history:
        return np.concatenate([np.zeros(HALF_FFT, np.int16), x])
    return x
