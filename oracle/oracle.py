"""ORACLE — test infrastructure only (ctypes front for oracle/libddc_oracle.so).

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may
import this module.  The product package (extio_sddc_amd) never does.

Wraps the C restatement in ddc_oracle.c (see its header for the reference
file:line each function restates and for what pins it).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libddc_oracle.so")
REF_FIR_PATH = os.path.join(HERE, "_ref", "libref_fir.so")
REF_MIXER_PATH = os.path.join(HERE, "_ref", "libref_mixer.so")

HALF_FFT = 4096      # fft_mt_r2iq.h:18
BLOCK = 65536        # config.h:80-81 transferSamples
FRAMES = 11          # fft_mt_r2iq.h:19 fftPerBuf
NDEC = 7             # r2iq.h:5
NTAPS = 1025         # fft_mt_r2iq.cpp:181

_lib = None


def build() -> None:
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        L.oracle_init.argtypes = []
        L.oracle_kaiser.argtypes = [ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_float, P]
        L.oracle_kaiser.restype = ctypes.c_int
        L.oracle_filter_taps.argtypes = [ctypes.c_int, P]
        L.oracle_filter_bank_f64.argtypes = [ctypes.c_float, P]
        L.oracle_filter_bank_f32.argtypes = [ctypes.c_float, P]
        L.oracle_fft_c64.argtypes = [P, ctypes.c_int, ctypes.c_int]
        L.oracle_set_freq_offset.argtypes = [ctypes.c_float, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L.oracle_set_freq_offset.restype = ctypes.c_float
        for name in ("oracle_r2iq_f64", "oracle_r2iq_f32"):
            fn = getattr(L, name)
            fn.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, ctypes.c_int, P]
            fn.restype = ctypes.c_int
        L.oracle_forward_r2c_f64.argtypes = [P, ctypes.c_int, P]
        L.oracle_nco_init.argtypes = [ctypes.c_float, ctypes.c_float, P]
        L.oracle_nco_apply.argtypes = [P, ctypes.c_int, P]
        L.oracle_nco_state_size.restype = ctypes.c_int
        L.oracle_init()
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def kaiser(ntaps: int, astop: float, fpass: float, fstop: float):
    """ntaps > 0: the taps.  ntaps <= 0: the tap-count estimate (Coef = nullptr)."""
    if ntaps <= 0:
        return lib().oracle_kaiser(ntaps, astop, fpass, fstop, None)
    out = np.zeros(ntaps, np.float32)
    n = lib().oracle_kaiser(ntaps, astop, fpass, fstop, _ptr(out))
    return out[:n]


def filter_taps(d: int) -> np.ndarray:
    out = np.zeros(NTAPS, np.float32)
    lib().oracle_filter_taps(d, _ptr(out))
    return out


def filter_bank(gain: float, dtype=np.float64) -> np.ndarray:
    """H[d][4096] complex (fft_mt_r2iq.cpp:163-208)."""
    if dtype == np.float64:
        h = np.zeros((NDEC, HALF_FFT, 2), np.float64)
        lib().oracle_filter_bank_f64(gain, _ptr(h))
        return h[..., 0] + 1j * h[..., 1]
    h = np.zeros((NDEC, HALF_FFT, 2), np.float32)
    lib().oracle_filter_bank_f32(gain, _ptr(h))
    return (h[..., 0] + 1j * h[..., 1]).astype(np.complex64)


def fft(x: np.ndarray, sign: int) -> np.ndarray:
    a = np.ascontiguousarray(np.stack([x.real, x.imag], -1).astype(np.float64))
    lib().oracle_fft_c64(_ptr(a), len(x), sign)
    return a[..., 0] + 1j * a[..., 1]


def set_freq_offset(offset: float, d: int):
    tb = ctypes.c_int(0)
    fc = lib().oracle_set_freq_offset(offset, d, ctypes.byref(tb))
    return tb.value, fc


def forward_r2c(frame: np.ndarray, rand: bool = False) -> np.ndarray:
    frame = np.ascontiguousarray(frame, np.int16)
    assert frame.size == 2 * HALF_FFT
    X = np.zeros((HALF_FFT + 1, 2), np.float64)
    lib().oracle_forward_r2c_f64(_ptr(frame), int(rand), _ptr(X))
    return X[:, 0] + 1j * X[:, 1]


def r2iq(stream: np.ndarray, nblk: int, d: int, tunebin: int, lsb: bool = False,
         rand: bool = False, gain: float = 1.0, dtype=np.float64, H=None) -> np.ndarray:
    """Reference-equivalent DDC of ``nblk`` blocks.

    ``stream`` holds 4096 history samples followed by nblk*65536 samples.
    Returns nblk*8*mfft complex samples (complex128 for f64, complex64 for f32).
    """
    stream = np.ascontiguousarray(stream, np.int16)
    assert stream.size >= HALF_FFT + nblk * BLOCK
    mfft = HALF_FFT >> d
    if dtype == np.float64:
        if H is None:
            H = filter_bank(gain, np.float64)
        Hd = np.ascontiguousarray(np.stack([H[d].real, H[d].imag], -1), np.float64)
        out = np.zeros((nblk * 8 * mfft, 2), np.float64)
        rc = lib().oracle_r2iq_f64(_ptr(Hd), d, tunebin, int(lsb), int(rand), _ptr(stream), nblk, _ptr(out))
        assert rc == 0
        return out[:, 0] + 1j * out[:, 1]
    if H is None:
        H = filter_bank(gain, np.float32)
    Hd = np.ascontiguousarray(np.stack([H[d].real, H[d].imag], -1), np.float32)
    out = np.zeros((nblk * 8 * mfft, 2), np.float32)
    rc = lib().oracle_r2iq_f32(_ptr(Hd), d, tunebin, int(lsb), int(rand), _ptr(stream), nblk, _ptr(out))
    assert rc == 0
    return (out[:, 0] + 1j * out[:, 1]).astype(np.complex64)


def ref_fir_available() -> bool:
    return os.path.exists(REF_FIR_PATH)


def ref_kaiser(ntaps: int, astop: float, fpass: float, fstop: float) -> np.ndarray:
    """The reference's own KaiserWindow (Core/fir.cpp:48), compiled into oracle/_ref."""
    L = ctypes.CDLL(REF_FIR_PATH)
    fn = L._Z12KaiserWindowifffPf
    fn.argtypes = [ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_void_p]
    fn.restype = ctypes.c_int
    if ntaps <= 0:
        return fn(ntaps, astop, fpass, fstop, None)
    out = np.zeros(ntaps, np.float32)
    n = fn(ntaps, astop, fpass, fstop, out.ctypes.data)
    return out[:n]


class Nco:
    """Fine-tune NCO restatement (pf_mixer.cpp:750-856, ALGO H); stateful across apply()."""

    def __init__(self, relative_freq: float, phase_start: float = 0.0):
        L = lib()
        self._st = ctypes.create_string_buffer(L.oracle_nco_state_size())
        L.oracle_nco_init(relative_freq, phase_start, self._st)

    def apply(self, iq: np.ndarray) -> np.ndarray:
        """iq: complex64 (n multiple of 4); returns the mixed copy."""
        buf = np.ascontiguousarray(iq, dtype=np.complex64).copy()
        assert buf.size % 4 == 0
        lib().oracle_nco_apply(buf.ctypes.data, buf.size, self._st)
        return buf


def ref_mixer_available() -> bool:
    return os.path.exists(REF_MIXER_PATH)


class RefMixer:
    """The reference's own shift_limited_unroll_C_sse_{init,inp_c} (pf_mixer.cpp:750-856),
    compiled into oracle/_ref by `make -C oracle ref` (build container only)."""

    # shift_limited_unroll_C_sse_data_t (pf_mixer.h:204-216): 264 + 4 + 4 + 3 floats
    class _State(ctypes.Structure):
        _fields_ = [("dinterl_trig", ctypes.c_float * 264), ("phase_state_i", ctypes.c_float * 4),
                    ("phase_state_q", ctypes.c_float * 4), ("dcos_blk", ctypes.c_float),
                    ("dsin_blk", ctypes.c_float), ("phase_increment", ctypes.c_float)]

    def __init__(self, relative_freq: float, phase_start: float = 0.0):
        L = ctypes.CDLL(REF_MIXER_PATH)
        L.shift_limited_unroll_C_sse_init.argtypes = [ctypes.c_float, ctypes.c_float]
        L.shift_limited_unroll_C_sse_init.restype = RefMixer._State
        L.shift_limited_unroll_C_sse_inp_c.argtypes = [ctypes.c_void_p, ctypes.c_int,
                                                       ctypes.POINTER(RefMixer._State)]
        self._L = L
        self._st = L.shift_limited_unroll_C_sse_init(relative_freq, phase_start)

    def apply(self, iq: np.ndarray) -> np.ndarray:
        buf = np.ascontiguousarray(iq, dtype=np.complex64).copy()
        self._L.shift_limited_unroll_C_sse_inp_c(buf.ctypes.data, buf.size, ctypes.byref(self._st))
        return buf


def max_rel_err(y: np.ndarray, ref: np.ndarray) -> float:
    """IQ max-rel-err = max|y - r| / max|r| over the whole stream."""
    return float(np.max(np.abs(y - ref)) / np.max(np.abs(ref)))


def rms_rel_err(y: np.ndarray, ref: np.ndarray) -> float:
    return float(np.sqrt(np.mean(np.abs(y - ref) ** 2) / np.mean(np.abs(ref) ** 2)))
