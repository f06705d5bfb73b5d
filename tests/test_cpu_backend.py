"""The C ABI's CPU backend (handles created on SDDC_DDC_DEVICE_CPU: the AVX2 r2iq in
extio_sddc_amd/csrc/cpu/, the reference's Core/fft_mt_r2iq_avx2.cpp worker restated without
FFTW).  Runs without a GPU.

Bars, as for the GPU path: IQ max-rel-err <= 1e-5 against the f64 oracle (leakage-aware for
leakage-only channels, see tests/test_gpu_sweep.py); the NCO and CS16 output stages
bit-exact against their restatements applied to the CF32 output of the same handle."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

from extio_sddc_amd.synth import make_stream

TOL = 1e-5
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def H(oracle):
    return oracle.filter_bank(1.0)


def _cpu(d, tb, lsb=False, rand=False, gain=1.0):
    from extio_sddc_amd import DEVICE_CPU, R2iq
    r = R2iq(gain=gain, device=DEVICE_CPU)
    assert r.backend == "cpu"
    r.setDecimate(d)
    r.setTuneBin(tb)
    r.setSideband(lsb)
    r.updateRand(rand)
    return r


CASES = [
    (0, 1024, 0, 0, "mix"), (0, 0, 0, 0, "mix"), (0, 4092, 1, 1, "uniform"), (0, 2048, 0, 0, "bench"),
    (0, 1024, 0, 0, "oob"), (1, 1024, 1, 1, "mix"), (1, 1024, 1, 1, "oob"), (1, 284, 0, 0, "oob"),
    (2, 1228, 0, 1, "uniform"), (2, 3684, 1, 0, "mix"), (2, 1024, 0, 0, "oob"), (3, 512, 0, 0, "mix"),
    (3, 3888, 0, 1, "bench"), (3, 1024, 0, 0, "oob"), (4, 1024, 0, 0, "mix"), (4, 0, 1, 0, "oob"),
    (4, 4092, 0, 0, "uniform"), (4, 1024, 0, 0, "oob"), (5, 2048, 0, 1, "mix"), (6, 1024, 1, 0, "mix"),
    (6, 4, 0, 0, "uniform"),
]


@pytest.mark.parametrize("d,tb,lsb,rand,src", CASES)
def test_cpu_parity(oracle, H, d, tb, lsb, rand, src):
    nblk = 4
    x = make_stream(nblk, src)
    with _cpu(d, tb, bool(lsb), bool(rand)) as r:
        y = r.process(x[4096:])
    ref = oracle.r2iq(x, nblk, d, tb, lsb, rand, H=H)
    assert y.size == ref.size
    assert oracle.max_rel_err(y, ref) <= TOL


def _sweep_cases():
    from test_gpu_sweep import _cases
    return _cases()


@pytest.mark.parametrize("d,tb,lsb,rand,src,nblk,seed", _sweep_cases())
def test_cpu_random_sweep(oracle, H, d, tb, lsb, rand, src, nblk, seed):
    from test_gpu_sweep import leak_aware_err
    x = make_stream(nblk, src, seed=seed)
    with _cpu(d, tb, bool(lsb), bool(rand)) as r:
        y = r.process(x[4096:])
    err, leak = leak_aware_err(y, oracle.r2iq(x, nblk, d, tb, lsb, rand, H=H), x)
    assert err <= TOL, f"{'leakage-aware' if leak else 'max-rel'} err {err:.3e}"


def test_cpu_golden_fixture():
    with open(os.path.join(HERE, "golden", "iq_golden.json")) as f:
        g = json.load(f)
    for c in g["cases"]:
        x = make_stream(g["nblk"], c["source"])
        with _cpu(c["d"], c["tunebin"], bool(c["lsb"]), bool(c["rand"])) as r:
            y = r.process(x[4096:])
        assert y.size == c["n"]
        head = np.array([complex(*v) for v in c["head"]])
        tail = np.array([complex(*v) for v in c["tail"]])
        assert np.max(np.abs(y[:64] - head)) / c["max_abs"] <= TOL
        assert np.max(np.abs(y[-64:] - tail)) / c["max_abs"] <= TOL


def test_cpu_history_across_calls_reset_and_set_history(oracle, H):
    """process() keeps the 4096-sample history across calls (impl.hpp:32); TurnOn() zeroes it;
    setHistory() restarts a stream mid-way on a fresh handle."""
    nblk, d, tb = 6, 1, 1024
    x = make_stream(nblk, "mix")
    ref = oracle.r2iq(x, nblk, d, tb, H=H)
    with _cpu(d, tb) as r:
        parts = [r.process(x[4096:4096 + 2 * 65536]), r.process(x[4096 + 2 * 65536:4096 + 3 * 65536]),
                 r.process(x[4096 + 3 * 65536:])]
        y = np.concatenate(parts)
        assert oracle.max_rel_err(y, ref) <= TOL
        r.TurnOn()
        np.testing.assert_array_equal(r.process(x[4096:4096 + 65536]), y[:32768 >> d])
    with _cpu(d, tb) as r2:   # blocks 3.. on a new handle, history = the tail of block 2
        r2.setHistory(x[3 * 65536: 3 * 65536 + 4096])
        np.testing.assert_array_equal(r2.process(x[4096 + 3 * 65536:]), y[3 * (32768 >> d):])


def test_cpu_process_blocks_scattered(oracle, H):
    nblk, d, tb = 5, 2, 2048
    x = make_stream(nblk, "uniform")
    blocks = [x[4096 + b * 65536: 4096 + (b + 1) * 65536].copy() for b in range(nblk)]
    with _cpu(d, tb, rand=True) as r:
        y = r.process_blocks(blocks[::-1][::-1])
    assert oracle.max_rel_err(y, oracle.r2iq(x, nblk, d, tb, False, True, H=H)) <= TOL


@pytest.mark.parametrize("d,fc", [(0, 0.0123), (2, -0.21), (4, 0.4)])
def test_cpu_fine_tune_nco_bit_exact(oracle, d, fc):
    """The fused NCO on the CPU backend equals the oracle mixer (itself bit-exact to the
    reference's pf_mixer, tests/golden/nco_golden.json) applied to the plain output, bit for
    bit, with the phase carried across calls."""
    nblk, tb = 4, 1024
    x = make_stream(nblk, "mix")
    with _cpu(d, tb) as r:
        plain = r.process(x[4096:])
    with _cpu(d, tb) as r:
        r.setFineTune(fc)
        mixed = np.concatenate([r.process(x[4096:4096 + 65536]), r.process(x[4096 + 65536:])])
    ref = oracle.Nco(fc).apply(plain)
    np.testing.assert_array_equal(mixed.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("d", [0, 3, 6])
def test_cpu_cs16_bit_exact(d):
    nblk, tb = 3, 1228
    x = make_stream(nblk, "mix")
    with _cpu(d, tb, lsb=True) as r:
        y = r.process(x[4096:])
        scale = 30000.0 / float(np.max(np.abs(y.view(np.float32))))
        r.TurnOn()
        r.setOutputFormat("CS16", scale)
        c = r.process(x[4096:])
    f = y.view(np.float32).reshape(-1, 2)
    np.testing.assert_array_equal(c, np.clip(np.rint(f * np.float32(scale)), -32768, 32767).astype(np.int16))


def test_cpu_handle_has_no_device_path():
    from extio_sddc_amd import DDCError
    from extio_sddc_amd._lib import check
    with _cpu(0, 1024) as r:
        with pytest.raises(DDCError, match="SDDC_ERR_STATE"):
            check(r._L.sddc_ddc_process_device(r._h, 4, 1, 8, None))
