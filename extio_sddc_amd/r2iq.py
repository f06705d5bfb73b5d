"""Host-side mirror of the reference's r2iq operator interface over the C ABI.

``R2iq`` exposes the method names and argument meanings of
``r2iqControlClass`` / ``fft_mt_r2iq`` (Core/r2iq.h:16-48,
Core/fft_mt_r2iq.h:21-31) so the parity tests read like the reference's own
tests; the work is done by the gfx950 kernels behind include/sddc_ddc.h.

Reference interface              -> here
  Init(gain, in, out)  .cpp:147  -> R2iq(gain, device)
  setDecimate(d)       r2iq.h:31 -> setDecimate(d)
  updateRand(v)        r2iq.h:25 -> updateRand(v) / getRand()
  setSideband(lsb)     r2iq.h:28 -> setSideband(lsb) / getSideband()
  getRatio()           r2iq.h:21 -> getRatio()
  setFreqOffset(off)   .cpp:101  -> setFreqOffset(off) -> fine-tune residual
  TurnOn()             .cpp:111  -> TurnOn()  (stream reset: zero history)
  worker body  impl.hpp:15-152   -> process(blocks) (host) / process_device(...) (HBM)
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import DDCError, check

FMT_CF32 = 0   # SDDC_DDC_FMT_CF32
FMT_CS16 = 1   # SDDC_DDC_FMT_CS16

HALF_FFT = 4096        # fft_mt_r2iq.h:18
BLOCK = 65536          # config.h:80-81 transferSamples
FRAMES = 11            # fft_mt_r2iq.h:19 fftPerBuf
NDEC = 7               # r2iq.h:5 NDECIDX
OUT_BLOCK = 32768      # config.h:62 EXT_BLOCKLEN
NTAPS = 1025
BBRF103_GAINFACTOR = 7.8e-8   # config.h:57; DummyRadio's gain in the reference tests


def output_samples(d: int, nblk: int) -> int:
    return nblk * (OUT_BLOCK >> d)


def kaiser(ntaps: int, astop: float, fpass: float, fstop: float):
    """KaiserWindow (Core/fir.cpp:48-105); ntaps <= 0 returns the tap estimate."""
    L = _lib.load()
    if ntaps <= 0:
        return L.sddc_ddc_kaiser(ntaps, astop, fpass, fstop, None)
    out = np.zeros(ntaps, np.float32)
    n = L.sddc_ddc_kaiser(ntaps, astop, fpass, fstop, out.ctypes.data)
    return out[:n]


def filter_taps(d: int) -> np.ndarray:
    out = np.zeros(NTAPS, np.float32)
    check(_lib.load().sddc_ddc_filter_taps(d, out.ctypes.data))
    return out


def filter_response(gain: float, d: int) -> np.ndarray:
    out = np.zeros((HALF_FFT, 2), np.float32)
    check(_lib.load().sddc_ddc_filter_response(gain, d, out.ctypes.data))
    return out[:, 0] + 1j * out[:, 1]


def device_count() -> int:
    return _lib.load().sddc_ddc_device_count()


class R2iq:
    """The DDC for one stream on one GPU (one handle = one r2iq worker).
    ``device=DEVICE_CPU`` (-1) selects the library's AVX2 CPU backend instead (host path only)."""

    def __init__(self, gain: float = 1.0, device: int = 0):
        self._L = _lib.load()
        h = ctypes.c_void_p()
        check(self._L.sddc_ddc_create(gain, device, ctypes.byref(h)))
        self._h = h
        self.gain = gain
        self.device = device
        self._d = 0
        self._rand = False
        self._lsb = False
        self._fmt = FMT_CF32

    # -- lifecycle --------------------------------------------------------
    @property
    def backend(self) -> str:
        """"hip" or "cpu": which backend this handle runs (sddc_ddc_backend)."""
        rc = self._L.sddc_ddc_backend(self._h)
        if rc < 0:
            check(rc)
        return "cpu" if rc == _lib.BACKEND_CPU else "hip"

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            self._L.sddc_ddc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- r2iqControlClass -------------------------------------------------
    def setDecimate(self, d: int) -> None:
        check(self._L.sddc_ddc_set_decimation(self._h, d))
        self._d = d

    def getDecimate(self) -> int:
        return self._d

    def getRatio(self) -> int:
        return 1 << self._d          # mratio[mdecimation], fft_mt_r2iq.cpp:32-36

    def updateRand(self, v: bool) -> None:
        check(self._L.sddc_ddc_set_rand(self._h, int(bool(v))))
        self._rand = bool(v)

    def getRand(self) -> bool:
        return self._rand

    def setSideband(self, lsb: bool) -> None:
        check(self._L.sddc_ddc_set_sideband(self._h, int(bool(lsb))))
        self._lsb = bool(lsb)

    def getSideband(self) -> bool:
        return self._lsb

    def setFreqOffset(self, offset: float) -> float:
        return float(self._L.sddc_ddc_set_freq_offset(self._h, offset))

    def setFineTune(self, fc: float) -> None:
        """Fused fine-tune NCO (the mixer RadioHandler applies after the r2iq, pf_mixer.cpp:
        750-856 via RadioHandler.cpp:33-37); fc = the residual from setFreqOffset, 0 = off.
        A new fc restarts the phase at 0, the same fc keeps it (RadioHandler.cpp:291-296)."""
        check(self._L.sddc_ddc_set_fine_tune(self._h, float(fc)))

    def setTuneBin(self, tunebin: int) -> None:
        check(self._L.sddc_ddc_set_tunebin(self._h, tunebin))

    def getTuneBin(self) -> int:
        return self._L.sddc_ddc_get_tunebin(self._h)

    def TurnOn(self) -> None:
        check(self._L.sddc_ddc_reset(self._h))

    def setHistory(self, last4096: np.ndarray) -> None:
        """The next host-path call starts from these 4096 samples as its history."""
        h = np.ascontiguousarray(last4096, np.int16).reshape(-1)
        if h.size != HALF_FFT:
            raise DDCError(-1, f"history must hold {HALF_FFT} samples")
        check(self._L.sddc_ddc_set_history(self._h, h.ctypes.data))

    # -- the hot loop -----------------------------------------------------
    def setOutputFormat(self, fmt: str = "CF32", scale: float = 1.0) -> None:
        """"CF32" (default, the reference's format) or "CS16": int16 (I, Q) =
        saturate(rint(x * scale)) written by the kernels' output stage."""
        code = {"CF32": FMT_CF32, "CS16": FMT_CS16}[fmt.upper()]
        check(self._L.sddc_ddc_set_output_format(self._h, code, float(scale)))
        self._fmt = code

    def _out_dtype(self):
        return np.int16 if self._fmt == FMT_CS16 else np.float32

    def process(self, blocks: np.ndarray) -> np.ndarray:
        """Stateful host path: nblk blocks (int16) -> nblk*(32768>>d) complex64
        (CS16: an int16 array [n, 2])."""
        blocks = np.ascontiguousarray(blocks, np.int16).reshape(-1)
        if blocks.size % BLOCK:
            raise DDCError(-1, f"input length {blocks.size} is not a multiple of {BLOCK}")
        nblk = blocks.size // BLOCK
        out = np.empty((output_samples(self._d, nblk), 2), self._out_dtype())
        check(self._L.sddc_ddc_process_host(self._h, blocks.ctypes.data, nblk, out.ctypes.data))
        if self._fmt == FMT_CS16:
            return out
        return out.view(np.complex64).reshape(-1)

    def process_blocks(self, blocks) -> np.ndarray:
        """Host path over blocks scattered in memory (ring slots): a list of int16 arrays of
        65536 samples each; same output and history semantics as process()."""
        arrs = [np.ascontiguousarray(b, np.int16).reshape(-1) for b in blocks]
        if any(a.size != BLOCK for a in arrs):
            raise DDCError(-1, f"every block must hold {BLOCK} samples")
        ptrs = (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
        out = np.empty((output_samples(self._d, len(arrs)), 2), self._out_dtype())
        check(self._L.sddc_ddc_process_blocks(self._h, ptrs, len(arrs), out.ctypes.data))
        if self._fmt == FMT_CS16:
            return out
        return out.view(np.complex64).reshape(-1)

    def register_host(self, arr: np.ndarray) -> None:
        """Pin a host array for direct DMA on the host path (unregister before freeing it)."""
        check(self._L.sddc_ddc_register_host(self._h, arr.ctypes.data, arr.nbytes))

    def unregister_host(self, arr: np.ndarray) -> None:
        check(self._L.sddc_ddc_unregister_host(self._h, arr.ctypes.data))

    def process_device(self, d_in, nblk: int, d_out, stream=None) -> None:
        """Stateless HBM path.  d_in: int16 device tensor [4096 + nblk*65536];
        d_out: float32 (CS16: int16) device tensor [>= nblk*(32768>>d)*2].  Enqueued on
        `stream` (a torch.cuda.Stream or raw handle; default: torch's current stream)."""
        _check_device_buffers(d_in, nblk, d_out, output_samples(self._d, nblk) * 2, self._fmt)
        check(self._L.sddc_ddc_process_device(self._h, d_in.data_ptr(), nblk, d_out.data_ptr(),
                                              _stream_handle(stream)))

    def process_channels_device(self, d_in, nblk: int, tunebins, d_out, stream=None) -> None:
        """Many-channel path: d_out float32 (CS16: int16) [nch, nblk*(32768>>d)*2]."""
        tb = np.ascontiguousarray(np.asarray(tunebins, np.int32))
        nch = tb.size
        per = output_samples(self._d, nblk) * 2
        _check_device_buffers(d_in, nblk, d_out, per * nch, self._fmt)
        stride = d_out.stride(0) if d_out.dim() > 1 else per
        check(self._L.sddc_ddc_process_channels_device(self._h, d_in.data_ptr(), nblk, tb.ctypes.data, nch,
                                                       d_out.data_ptr(), stride, _stream_handle(stream)))


def _check_device_buffers(d_in, nblk, d_out, out_floats, fmt=0):
    import torch
    if not (d_in.is_cuda and d_out.is_cuda):
        raise DDCError(-1, "device path needs device tensors")
    want = torch.int16 if fmt == FMT_CS16 else torch.float32
    if d_in.dtype != torch.int16 or d_out.dtype != want:
        raise DDCError(-1, f"d_in must be int16 and d_out {want}")
    if not (d_in.is_contiguous() and d_out.is_contiguous()):
        raise DDCError(-1, "tensors must be contiguous")
    if d_in.numel() < HALF_FFT + nblk * BLOCK:
        raise DDCError(-1, f"d_in has {d_in.numel()} samples, need {HALF_FFT + nblk * BLOCK}")
    if d_out.numel() < out_floats:
        raise DDCError(-1, f"d_out has {d_out.numel()} floats, need {out_floats}")


def _stream_handle(stream):
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream
