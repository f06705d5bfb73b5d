"""Batched FFTs and the HIP FFTBackend on the GPU (pytest -m gpu).

Bar: max|y - r| / max|r| <= 1e-5 against numpy's float64 FFT (pocketfft) with FFTW's
conventions (unnormalised; forward e^{-2 pi i nk/n}; r2c keeps n/2+1 bins), the
conventions of Core/fft_backend_fftw.cpp.  The FFTBackend is driven only through its
API (tests/harness/fft_backend_harness.cpp), with GPU-mapped buffers from alloc() and
with plain malloc() buffers (staged); both must agree bit-exactly.  The reference's
own Core/fft_benchmark.cpp, linked with this backend (oracle Makefile `fftbench`),
must run to completion."""
from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOL = 1e-5


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch


@pytest.fixture(scope="module")
def L(torch_dev):
    from extio_sddc_amd._lib import load
    return load()


def rel(y, r):
    return float(np.max(np.abs(y - r)) / np.max(np.abs(r)))


@pytest.mark.parametrize("n", [64, 128, 256, 512, 1024, 2048, 4096])
@pytest.mark.parametrize("direction", [-1, 1])
def test_c2c_batched(torch_dev, L, n, direction):
    torch = torch_dev
    rng = np.random.default_rng(n)
    batch = 5
    x = (rng.standard_normal((batch, n)) + 1j * rng.standard_normal((batch, n))).astype(np.complex64)
    d_in = torch.from_numpy(x.view(np.float32).copy()).cuda()
    d_out = torch.full_like(d_in, float("nan"))
    s = torch.cuda.current_stream().cuda_stream
    assert L.sddc_fft_c2c(d_in.data_ptr(), d_out.data_ptr(), n, batch, direction, s) == 0
    torch.cuda.synchronize()
    y = d_out.cpu().numpy().view(np.complex64).reshape(batch, n)
    xr = x.astype(np.complex128)
    ref = np.fft.fft(xr, axis=1) if direction < 0 else np.fft.ifft(xr, axis=1) * n
    assert rel(y, ref) <= TOL
    # in place gives the same answer
    assert L.sddc_fft_c2c(d_in.data_ptr(), d_in.data_ptr(), n, batch, direction, s) == 0
    torch.cuda.synchronize()
    assert torch.equal(d_in, d_out)


@pytest.mark.parametrize("n", [128, 256, 512, 1024, 2048, 4096, 8192])
def test_r2c_batched(torch_dev, L, n):
    torch = torch_dev
    rng = np.random.default_rng(n + 1)
    batch = 3
    x = rng.standard_normal((batch, n)).astype(np.float32)
    d_in = torch.from_numpy(x.copy()).cuda()
    d_out = torch.full((batch, 2 * (n // 2 + 1)), float("nan"), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    assert L.sddc_fft_r2c(d_in.data_ptr(), d_out.data_ptr(), n, batch, s) == 0
    torch.cuda.synchronize()
    y = d_out.cpu().numpy().view(np.complex64).reshape(batch, n // 2 + 1)
    assert rel(y, np.fft.rfft(x.astype(np.float64), axis=1)) <= TOL


def test_unsupported_sizes(L, torch_dev):
    assert L.sddc_fft_supported(0, 32) == 0 and L.sddc_fft_supported(0, 8192) == 0
    assert L.sddc_fft_supported(1, 8192) == 1 and L.sddc_fft_supported(1, 3000) == 0
    assert L.sddc_fft_c2c(1, 1, 100, 1, -1, None) != 0


def test_fft_backend_api_dump(tmp_path):
    exe = os.path.join(ROOT, "build", "bin", "fft_backend_harness")
    path = str(tmp_path / "fft.bin")
    r = subprocess.run([exe, "dump", path], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    data = open(path, "rb").read()
    off, cases = 0, 0
    while off < len(data):
        kind, n, direction = np.frombuffer(data, np.int32, 3, off)
        off += 12
        nin = n if kind else 2 * n
        nout = 2 * (n // 2 + 1) if kind else 2 * n
        x = np.frombuffer(data, np.float32, nin, off); off += 4 * nin
        y = np.frombuffer(data, np.float32, nout, off); off += 4 * nout
        y2 = np.frombuffer(data, np.float32, nout, off); off += 4 * nout
        if kind:
            ref = np.fft.rfft(x.astype(np.float64))
        else:
            xc = x.view(np.complex64).astype(np.complex128)
            ref = np.fft.fft(xc) if direction < 0 else np.fft.ifft(xc) * n
        assert rel(y.view(np.complex64), ref) <= TOL, (kind, n, direction)
        np.testing.assert_array_equal(y, y2)          # staged malloc() buffers: same result
        cases += 1
    assert cases == 7 * 2 + 7


def test_reference_fft_benchmark_runs_on_hip_backend():
    exe = os.path.join(ROOT, "oracle", "_ref", "fft_benchmark_hip")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref/fft_benchmark_hip not built (needs /root/reference at build time)")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "HIP (gfx950)" in r.stdout
    rows = [l for l in r.stdout.splitlines() if l.strip().split("|")[0].strip().isdigit()]
    assert len(rows) == 6, r.stdout
