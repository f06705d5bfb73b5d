"""extio_sddc_amd — MI355X-native real-to-IQ DDC (drop-in for ExtIO_sddc's fft_mt_r2iq).

The product is the gfx950 library behind include/sddc_ddc.h and the drop-in C++
class in include/fft_mt_r2iq.h; this package is its Python host mirror (ctypes).
"""
from ._lib import BACKEND_CPU, BACKEND_HIP, DEVICE_CPU, DDCError, build, load  # noqa: F401
from .r2iq import (BBRF103_GAINFACTOR, BLOCK, FRAMES, HALF_FFT, NDEC, OUT_BLOCK,  # noqa: F401
                   R2iq, device_count, filter_response, filter_taps, kaiser, output_samples)

__all__ = ["R2iq", "DDCError", "DEVICE_CPU", "BACKEND_CPU", "BACKEND_HIP", "build", "load", "kaiser", "filter_taps", "filter_response",
           "device_count", "output_samples", "HALF_FFT", "BLOCK", "FRAMES", "NDEC", "OUT_BLOCK",
           "BBRF103_GAINFACTOR"]
