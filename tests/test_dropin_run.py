"""The drop-in boundary: fft_mt_r2iq driven through r2iqControlClass, on each backend.

1. build/bin/r2iq_harness — the class driven exactly as RadioHandler drives it, over the
   standalone ring (include/sddc_compat), checked against the f64 oracle.
2. oracle/_ref/radiohandler_harness — the REFERENCE's unchanged RadioHandlerClass
   (Core/RadioHandler.cpp, built by `make -C oracle radiohandler` where the reference is
   mounted) with a mock USB producer, running our class end to end; output taken from the
   user callback (RadioHandler.cpp:51).  Skipped when that binary was not built.

Every case runs with SDDC_DDC_BACKEND=hip (the MI355X, marked gpu) and =cpu (the library's
AVX2 backend, runs anywhere); the GPU-only failover case runs =auto with an injected failure.
"""
from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

from extio_sddc_amd.synth import make_stream

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "build", "bin", "r2iq_harness")
RH_HARNESS = os.path.join(ROOT, "oracle", "_ref", "radiohandler_harness")
TOL = 1e-5
BBRF103_GAINFACTOR = np.float32(7.8e-8)   # DummyRadio's gain (Core/RadioHandler.h:143, config.h:57)


BACKENDS = [pytest.param("hip", marks=pytest.mark.gpu), "cpu"]


@pytest.fixture(params=BACKENDS)
def backend(request):
    return request.param


def _run(cmd, backend, timeout=120, env=None, stderr=False):
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout,
                       env=dict(os.environ, SDDC_DDC_BACKEND=backend, **(env or {})))
    assert p.returncode == 0, f"{cmd[0]} rc={p.returncode}\n{p.stdout}\n{p.stderr}"
    if backend != "auto":   # an explicit backend never switches
        assert "continuing on the CPU" not in p.stderr and "using the CPU backend" not in p.stderr, p.stderr
    return (p.stdout, p.stderr) if stderr else p.stdout


@pytest.mark.parametrize("d,tb,lsb,rand,src,nblk", [
    (0, 1024, 0, 0, "mix", 6),
    (1, 1024, 1, 1, "mix", 8),      # C4: decim 4, sideband invert, rand
    (2, 284, 0, 0, "uniform", 8),
    (4, 3888, 1, 0, "mix", 32),     # 2^4 input blocks per output block
])
def test_dropin_class(tmp_path, oracle, backend, d, tb, lsb, rand, src, nblk):
    assert os.path.exists(HARNESS), "build/bin/r2iq_harness missing (make -C extio_sddc_amd/csrc)"
    x = make_stream(nblk, src)
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    x[4096:].tofile(fin)
    _run([HARNESS, str(fin), str(nblk), str(d), str(tb), str(lsb), str(rand), "1.0", str(fout)], backend)
    y = np.fromfile(fout, np.float32).view(np.complex64)
    ref = oracle.r2iq(x, nblk, d, tb, lsb, rand)
    assert y.size == ref.size == nblk * (32768 >> d)
    assert oracle.max_rel_err(y, ref) <= TOL


@pytest.mark.skipif(not os.path.exists(RH_HARNESS), reason="reference RadioHandler harness not built here")
@pytest.mark.parametrize("srate_idx,tune_hz,rand", [(4, 8_000_000, 0), (3, 5_000_000, 1), (0, 8_000_000, 0)])
def test_reference_radiohandler_runs_dropin(tmp_path, oracle, backend, srate_idx, tune_hz, rand):
    d = 4 - srate_idx                        # RadioHandler.cpp:152 (adc 64 MHz)
    nblk = max(4, 2 << d)
    x = make_stream(nblk, "mix")
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    x[4096:].tofile(fin)
    _run([RH_HARNESS, str(fin), str(nblk), str(srate_idx), str(tune_hz), str(rand), str(fout)], backend)
    y = np.fromfile(fout, np.float32).view(np.complex64)
    tb, fc = oracle.set_freq_offset(np.float32(tune_hz / 32e6), d)
    assert fc == 0.0                         # exact tune: no fine-tune NCO in OnDataPacket
    ref = oracle.r2iq(x, nblk, d, tb, False, rand, gain=float(BBRF103_GAINFACTOR))
    assert y.size == ref.size                # every callback carries 32768 samples (core_test.cpp:167)
    assert oracle.max_rel_err(y, ref) <= TOL


@pytest.mark.skipif(not os.path.exists(RH_HARNESS), reason="reference RadioHandler harness not built here")
@pytest.mark.parametrize("srate_idx,tune_hz,rand", [(4, 7_777_777, 0), (2, 5_003_000, 1)])
def test_reference_radiohandler_fine_tune(tmp_path, oracle, backend, srate_idx, tune_hz, rand):
    """A tune between 4-bin steps: RadioHandler::TuneLO gets a non-zero residual fc from our
    setFreqOffset and its own CPU mixer (pf_mixer ALGO H, RadioHandler.cpp:33-37) runs on our
    output.  Expected: oracle DDC at tb, then the oracle mixer (bit-exact to pf_mixer)."""
    d = 4 - srate_idx
    nblk = max(4, 2 << d)
    x = make_stream(nblk, "mix")
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    x[4096:].tofile(fin)
    _run([RH_HARNESS, str(fin), str(nblk), str(srate_idx), str(tune_hz), str(rand), str(fout)], backend)
    y = np.fromfile(fout, np.float32).view(np.complex64)
    # RadioHandler.cpp:289: offset / (getSampleRate() / 2.0f), all in float.  The harness tunes
    # before Start() sets the decimation, so setFreqOffset scales the residual by getRatio() of
    # d = 0 (r2iq.h:24, mratio[0] = 1): the reference's behaviour for this call order.
    tb, fc = oracle.set_freq_offset(np.float32(np.float32(tune_hz) / np.float32(32e6)), 0)
    assert fc != 0.0
    plain = oracle.r2iq(x, nblk, d, tb, False, rand, gain=float(BBRF103_GAINFACTOR)).astype(np.complex64)
    ref = oracle.Nco(fc).apply(plain)
    assert y.size == ref.size
    assert oracle.max_rel_err(y, ref) <= TOL


def test_dropin_start_stop_cycles(tmp_path, oracle, backend):
    """20 TurnOn/TurnOff cycles on one object and one pair of rings (the Start/Stop cycling of
    unittest/stability_test.cpp:255-301): every cycle restarts from a zero history
    (TurnOn, fft_mt_r2iq.cpp:111-129), so each cycle's IQ equals the oracle's."""
    d, tb, nblk, cycles = 1, 1024, 8, 20
    x = make_stream(nblk, "mix")
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    x[4096:].tofile(fin)
    out = _run([HARNESS, str(fin), str(nblk), str(d), str(tb), "0", "0", "1.0", str(fout), str(cycles)], backend)
    assert out.count("output blocks 4 of 4") == cycles, out
    y = np.fromfile(fout, np.float32).view(np.complex64).reshape(cycles, -1)
    ref = oracle.r2iq(x, nblk, d, tb)
    for c in range(cycles):
        assert oracle.max_rel_err(y[c], ref) <= TOL
        np.testing.assert_array_equal(y[c].view(np.uint32), y[0].view(np.uint32))


@pytest.mark.parametrize("d,nblk,sched", [
    (1, 8, [(3, 2048, 1), (6, 284, 0)]),            # tune and rand change mid-stream
    (0, 9, [(1, 3888, 0), (2, 3888, 1), (5, 0, 1)]),   # rand alone, then tune alone, edge bins
    (2, 12, [(4, 512, 0)]),                         # inside one output block (4 inputs per output)
])
def test_dropin_per_block_tune_and_rand(tmp_path, oracle, backend, d, nblk, sched):
    """setFreqOffset / updateRand between two known input blocks: the reference reads the tune
    bin and rand once per block (Core/fft_mt_r2iq_impl.hpp:20, 40), so every block's IQ must be
    the oracle's at THAT block's (tunebin, rand), even though the drop-in batches queued blocks
    into one GPU call (a batch is cut where either value changes)."""
    tb0, rand0 = 1024, 0
    x = make_stream(nblk, "mix")
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    x[4096:].tofile(fin)
    spec = ",".join(f"{k}:{tb}:{r}" for k, tb, r in sched)
    _run([HARNESS, str(fin), str(nblk), str(d), str(tb0), "0", str(rand0), "1.0", str(fout)], backend,
         env={"R2IQ_SCHEDULE": spec})
    y = np.fromfile(fout, np.float32).view(np.complex64)
    per = 32768 >> d
    assert y.size == nblk * per
    bounds = [(0, tb0, rand0)] + list(sched) + [(nblk, None, None)]
    for (a, tb, r), (b, _, _) in zip(bounds[:-1], bounds[1:]):
        seg = x[a * 65536: 4096 + b * 65536]          # blocks a..b-1 with their history
        ref = oracle.r2iq(seg, b - a, d, tb, False, r)
        assert oracle.max_rel_err(y[a * per: b * per], ref) <= TOL, (a, b, tb, r)


@pytest.mark.gpu
@pytest.mark.parametrize("d,nblk,fail_after,sched", [(0, 12, 1, [(4, 1228, 1), (8, 1228, 0)]),
                                                      (2, 16, 2, [(5, 1228, 1), (10, 1228, 0)])])
def test_dropin_auto_failover_mid_stream(tmp_path, oracle, d, nblk, fail_after, sched):
    """SDDC_DDC_BACKEND=auto: the GPU handle's (fail_after+1)-th call fails (injected,
    SDDC_DDC_INJECT_FAIL); the worker announces the switch, redoes that batch on a CPU handle
    from the same ring slots and the last block's tail as history, and the output stream is
    continuous: every block equals the oracle's, across the switch.  The rand changes of the
    schedule cut the stream into at least len(sched) + 1 calls, so the failure lands mid-stream."""
    tb = 1228
    x = make_stream(nblk, "mix")
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    x[4096:].tofile(fin)
    spec = ",".join(f"{k}:{t}:{r}" for k, t, r in sched)
    out, err = _run([HARNESS, str(fin), str(nblk), str(d), str(tb), "0", "0", "1.0", str(fout)], "auto",
                    env={"SDDC_DDC_INJECT_FAIL": str(fail_after), "R2IQ_SCHEDULE": spec}, stderr=True)
    assert "continuing on the CPU" in err, err
    y = np.fromfile(fout, np.float32).view(np.complex64)
    per = 32768 >> d
    assert y.size == nblk * per
    bounds = [(0, tb, 0)] + list(sched) + [(nblk, None, None)]
    for (a, t, r), (b, _, _) in zip(bounds[:-1], bounds[1:]):
        ref = oracle.r2iq(x[a * 65536: 4096 + b * 65536], b - a, d, t, False, r)
        assert oracle.max_rel_err(y[a * per: b * per], ref) <= TOL, (a, b)


@pytest.mark.gpu
def test_dropin_auto_failover_with_device_work_in_flight(tmp_path, oracle):
    """As above, but the failing call errors after its first chunk's kernel and D2H were issued
    (SDDC_DDC_INJECT_FAIL_AFTER_D2H): the output stage is partly written and device work is in
    flight when the worker destroys the failed GPU handle (which must neither block nor abort)
    and redoes the batch on the CPU, overwriting the stage.  The stream stays continuous."""
    d, tb, nblk = 1, 1228, 12
    sched = [(4, 1228, 1), (8, 1228, 0)]
    x = make_stream(nblk, "mix")
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    x[4096:].tofile(fin)
    spec = ",".join(f"{k}:{t}:{r}" for k, t, r in sched)
    out, err = _run([HARNESS, str(fin), str(nblk), str(d), str(tb), "0", "0", "1.0", str(fout)], "auto",
                    env={"SDDC_DDC_INJECT_FAIL_AFTER_D2H": "1", "R2IQ_SCHEDULE": spec}, stderr=True)
    assert "continuing on the CPU" in err and "after the first chunk's D2H" in err, err
    y = np.fromfile(fout, np.float32).view(np.complex64)
    per = 32768 >> d
    assert y.size == nblk * per
    bounds = [(0, tb, 0)] + list(sched) + [(nblk, None, None)]
    for (a, t, r), (b, _, _) in zip(bounds[:-1], bounds[1:]):
        ref = oracle.r2iq(x[a * 65536: 4096 + b * 65536], b - a, d, t, False, r)
        assert oracle.max_rel_err(y[a * per: b * per], ref) <= TOL, (a, b)


def test_dropin_auto_without_gpu_uses_cpu(tmp_path, oracle):
    """SDDC_DDC_BACKEND=auto where Init finds no usable GPU (forced here with an invalid
    SDDC_DDC_DEVICE): announced on stderr, then the CPU backend produces the stream."""
    d, tb, nblk = 1, 1024, 6
    x = make_stream(nblk, "mix")
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    x[4096:].tofile(fin)
    out, err = _run([HARNESS, str(fin), str(nblk), str(d), str(tb), "0", "0", "1.0", str(fout)], "auto",
                    env={"SDDC_DDC_DEVICE": "4096"}, stderr=True)
    assert "using the CPU backend" in err, err
    y = np.fromfile(fout, np.float32).view(np.complex64)
    assert oracle.max_rel_err(y, oracle.r2iq(x, nblk, d, tb)) <= TOL


def test_dropin_hip_without_gpu_fails_loudly(tmp_path):
    """SDDC_DDC_BACKEND=hip (the default) never runs on the CPU: without a usable device the
    class reports the error and stays off."""
    x = make_stream(2, "mix")
    fin = tmp_path / "in.bin"
    x[4096:].tofile(fin)
    p = subprocess.run([HARNESS, str(fin), "2", "0", "1024", "0", "0", "1.0", "-"], capture_output=True, text=True,
                       timeout=60, env=dict(os.environ, SDDC_DDC_BACKEND="hip", SDDC_DDC_DEVICE="4096"))
    assert p.returncode == 3 and "sddc_ddc_create" in p.stderr, (p.returncode, p.stderr)
