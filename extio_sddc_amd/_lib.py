"""ctypes binding of the C ABI declared in include/sddc_ddc.h.

The library is the in-tree ``extio_sddc_amd/lib/libsddc_ddc.so`` (built for
gfx950 by ``make -C extio_sddc_amd/csrc``).  There is no fallback: if it is
missing or cannot be loaded, every compute entry point raises.  Its CPU backend
(device ``DEVICE_CPU``) lives in the same library and is only used when a handle
is created on it explicitly.

torch is imported (when installed) BEFORE the library is loaded: PyTorch-ROCm
ships its own ``libamdhip64.so`` with the same soname (libamdhip64.so.7), and
loading torch first makes the dynamic linker bind this library to that one
runtime, so torch device pointers and streams are valid here.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "lib", "libsddc_ddc.so")
CSRC_DIR = os.path.join(PKG_DIR, "csrc")

# Every symbol include/sddc_ddc.h declares: (name, restype, argtypes)
_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_SZ = ctypes.c_size_t
SIGNATURES = {
    "sddc_ddc_abi_version": (_I, []),
    "sddc_ddc_last_error": (ctypes.c_char_p, []),
    "sddc_ddc_device_count": (_I, []),
    "sddc_ddc_kaiser": (_I, [_I, _F, _F, _F, _P]),
    "sddc_ddc_filter_taps": (_I, [_I, _P]),
    "sddc_ddc_filter_response": (_I, [_F, _I, _P]),
    "sddc_ddc_create": (_I, [_F, _I, ctypes.POINTER(_P)]),
    "sddc_ddc_destroy": (_I, [_P]),
    "sddc_ddc_backend": (_I, [_P]),
    "sddc_ddc_set_history": (_I, [_P, _P]),
    "sddc_ddc_set_decimation": (_I, [_P, _I]),
    "sddc_ddc_set_sideband": (_I, [_P, _I]),
    "sddc_ddc_set_rand": (_I, [_P, _I]),
    "sddc_ddc_set_tunebin": (_I, [_P, _I]),
    "sddc_ddc_get_tunebin": (_I, [_P]),
    "sddc_ddc_set_freq_offset": (_F, [_P, _F]),
    "sddc_ddc_reset": (_I, [_P]),
    "sddc_ddc_set_fine_tune": (_I, [_P, _F]),
    "sddc_ddc_set_output_format": (_I, [_P, _I, _F]),
    "sddc_ddc_output_samples": (_SZ, [_I, _I]),
    "sddc_ddc_process_device": (_I, [_P, _P, _I, _P, _P]),
    "sddc_ddc_process_channels_device": (_I, [_P, _P, _I, _P, _I, _P, _SZ, _P]),
    "sddc_ddc_process_host": (_I, [_P, _P, _I, _P]),
    "sddc_ddc_process_blocks": (_I, [_P, _P, _I, _P]),
    "sddc_ddc_register_host": (_I, [_P, _P, _SZ]),
    "sddc_ddc_unregister_host": (_I, [_P, _P]),
    # include/sddc_fft.h
    "sddc_fft_supported": (_I, [_I, _I]),
    "sddc_fft_c2c": (_I, [_P, _P, _I, _I, _I, _P]),
    "sddc_fft_r2c": (_I, [_P, _P, _I, _I, _P]),
}

DEVICE_CPU = -1      # SDDC_DDC_DEVICE_CPU
BACKEND_HIP, BACKEND_CPU = 0, 1

ERRORS = {0: "SDDC_OK", -1: "SDDC_ERR_ARG", -2: "SDDC_ERR_HIP", -3: "SDDC_ERR_NODEV",
          -4: "SDDC_ERR_STATE", -5: "SDDC_ERR_NOMEM"}

_lib = None


class DDCError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


def build(force: bool = False) -> str:
    """Compile the HIP library in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", CSRC_DIR, "-j8"])
    return LIB_PATH


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    try:  # share torch's HIP runtime (see module docstring)
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise DDCError(-3, f"{LIB_PATH} is missing: build it with `make -C {CSRC_DIR}` "
                           "(there is no CPU fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int) -> int:
    if rc != 0:
        raise DDCError(rc, load().sddc_ddc_last_error().decode(errors="replace"))
    return rc
