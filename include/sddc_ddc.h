/*
 * sddc_ddc.h — C ABI of the MI355X-native real-to-IQ down-converter.
 *
 * This is the thin C boundary UNDER the drop-in C++ class `fft_mt_r2iq`
 * (include/fft_mt_r2iq.h), which keeps the reference's r2iqControlClass
 * interface (Core/r2iq.h:16-48) so RadioHandler / libsddc / ExtIO / SoapySDDC
 * load it unchanged.  Plain pointers and sizes only; no C++ or torch types.
 * Every entry point names the reference interface it replaces (file:line,
 * relative to the ExtIO_sddc tree).
 *
 * Conventions (pinned to the reference):
 *   block      = 65536 int16 real ADC samples           (config.h:80-81 transferSamples)
 *   history    = the 4096 samples preceding a block      (fft_mt_r2iq_impl.hpp:32)
 *   d          = decimation index 0..6, mfft = 4096>>d   (r2iq.h:5,39; fft_mt_r2iq.cpp:44-48)
 *   output     = 8*mfft = 32768>>d complex float32 (I,Q interleaved) per input block
 *                (fft_mt_r2iq_impl.hpp:117-138); 2^d blocks fill one 32768-sample
 *                EXT_BLOCKLEN output block (config.h:62)
 *   tunebin    = forward-FFT bin moved to DC, multiple of 4 in [0,4096)
 *                (fft_mt_r2iq.cpp:101-109)
 *
 * Errors: every int-returning call returns SDDC_OK (0) or a negative SDDC_ERR_*;
 * sddc_ddc_last_error() gives a thread-local message.  Nothing throws across this
 * boundary (the reference's r2iq methods are void/bool/float).
 *
 * Backends.  A handle created on a device index >= 0 runs the gfx950 kernels; without a
 * usable gfx950 device sddc_ddc_create() fails with SDDC_ERR_NODEV, and a HIP error fails
 * the call — a GPU handle never falls back to the CPU.  A handle created on
 * SDDC_DDC_DEVICE_CPU runs the library's AVX2 r2iq (the reference's fft_mt_r2iq_avx2.cpp
 * worker, restated without FFTW) on the calling thread: the host path (process_host /
 * process_blocks) with the same controls, output formats, fine-tune NCO and history
 * semantics; its device-path calls return SDDC_ERR_STATE.  Choosing it is the caller's
 * explicit decision (the drop-in class: SDDC_DDC_BACKEND=cpu|auto).
 */
#ifndef SDDC_DDC_H
#define SDDC_DDC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDDC_DDC_ABI_VERSION 3   /* 2: + set_fine_tune, set_output_format, process_blocks, register_host;
                                    3: + CPU handles (SDDC_DDC_DEVICE_CPU), backend, set_history */

#define SDDC_DDC_HALF_FFT   4096    /* halfFft               fft_mt_r2iq.h:18 */
#define SDDC_DDC_FFTN       8192    /* FFTN_R_ADC            config.h:49 */
#define SDDC_DDC_HOP        6144    /* 3*halfFft/2           fft_mt_r2iq_impl.hpp:88 */
#define SDDC_DDC_BLOCK      65536   /* transferSamples       config.h:80-81 */
#define SDDC_DDC_FRAMES     11      /* fftPerBuf             fft_mt_r2iq.h:19 */
#define SDDC_DDC_NDEC       7       /* NDECIDX               r2iq.h:5 */
#define SDDC_DDC_NTAPS      1025    /* halfFft/4+1 taps      fft_mt_r2iq.cpp:181 */
#define SDDC_DDC_OUT_BLOCK  32768   /* EXT_BLOCKLEN          config.h:62 */
#define SDDC_DDC_MAX_CHANNELS 1024  /* 1024 legal tune bins (tunebin = 4c) */
#define SDDC_DDC_MAX_BLOCKS 32768   /* blocks per process_* call (2^31 input samples, 4 GiB) */

enum {
    SDDC_OK = 0,
    SDDC_ERR_ARG = -1,     /* bad argument (range, null, alignment)           */
    SDDC_ERR_HIP = -2,     /* a HIP runtime call or kernel launch failed       */
    SDDC_ERR_NODEV = -3,   /* no usable gfx950 device                          */
    SDDC_ERR_STATE = -4,   /* call not valid in the handle's current state     */
    SDDC_ERR_NOMEM = -5    /* host or device allocation failed                 */
};

typedef struct sddc_ddc sddc_ddc_t;

#define SDDC_DDC_DEVICE_CPU   (-1)  /* sddc_ddc_create(): the host AVX2 backend */
#define SDDC_DDC_BACKEND_HIP  0
#define SDDC_DDC_BACKEND_CPU  1

/* ---- library ------------------------------------------------------------ */
int         sddc_ddc_abi_version(void);
const char *sddc_ddc_last_error(void);
/* Number of visible HIP devices (0 if none / runtime unusable). */
int         sddc_ddc_device_count(void);

/* ---- filter design (host; Core/fir.cpp, fft_mt_r2iq.cpp:163-208) ---------- */
/* KaiserWindow(num_taps, Astop, normFpass, normFstop, Coef)   fir.cpp:48-105.
 * Bit-identical float arithmetic.  coef == NULL with ntaps <= 0 returns the
 * tap-count estimate, exactly like the reference. */
int sddc_ddc_kaiser(int ntaps, float astop, float fpass, float fstop, float *coef);
/* The 1025 taps for decimation index d (fft_mt_r2iq.cpp:189-191). */
int sddc_ddc_filter_taps(int d, float *taps /* [1025] */);
/* H_d = FFT4096(time-reversed gain*2048/8192*taps)  (fft_mt_r2iq.cpp:193-205),
 * evaluated in double and rounded once to float. */
int sddc_ddc_filter_response(float gain, int d, float *H /* [4096][2] */);

/* ---- lifecycle: fft_mt_r2iq::Init (fft_mt_r2iq.cpp:147-227), dtor (:71-98) - */
/* Builds the 7 filter banks for `gain` (hardware->getGain(), RadioHandler.cpp:142)
 * and uploads them with the FFT twiddle tables to `device`. */
int sddc_ddc_create(float gain, int device, sddc_ddc_t **out);
int sddc_ddc_destroy(sddc_ddc_t *h);
/* SDDC_DDC_BACKEND_HIP or SDDC_DDC_BACKEND_CPU (negative on a null handle). */
int sddc_ddc_backend(const sddc_ddc_t *h);

/* ---- control: r2iqControlClass (r2iq.h:23-31) and fft_mt_r2iq -------------- */
int   sddc_ddc_set_decimation(sddc_ddc_t *h, int d);        /* setDecimate   r2iq.h:31 */
int   sddc_ddc_set_sideband(sddc_ddc_t *h, int lsb);        /* setSideband   r2iq.h:28 */
int   sddc_ddc_set_rand(sddc_ddc_t *h, int rand);           /* updateRand    r2iq.h:25 */
int   sddc_ddc_set_tunebin(sddc_ddc_t *h, int tunebin);     /* mtunebin      fft_mt_r2iq.h:97 */
int   sddc_ddc_get_tunebin(const sddc_ddc_t *h);
/* setFreqOffset(offset)  fft_mt_r2iq.cpp:101-109: tunebin = int(offset*1024)*4,
 * returns the fine-tune residual (tunebin/4096 - offset) * 2^d.  Valid domain
 * 0 <= offset < 1 (fraction of Fs/2); outside it the tune bin is clamped into
 * [0, 4092] (the reference would read out of range, impl.hpp:76-79). */
float sddc_ddc_set_freq_offset(sddc_ddc_t *h, float offset);
/* TurnOn() stream reset (fft_mt_r2iq.cpp:111-129): zero history, seq = 0.  The
 * fine-tune NCO keeps its phase (the reference's mixer state lives in RadioHandler). */
int   sddc_ddc_reset(sddc_ddc_t *h);
/* Host path: the next process_host/process_blocks call starts from these 4096 samples as
 * its history instead of the kept one (the reference's peekReadPtr(-1) tail,
 * fft_mt_r2iq_impl.hpp:32) — e.g. to continue a stream on another handle. */
int   sddc_ddc_set_history(sddc_ddc_t *h, const int16_t *last4096);

/* Fused fine-tune NCO: mixes the output with the reference's
 * fine-tune mixer, pf_mixer's shift_limited_unroll_C_sse (Core/pffft/pf_mixer.cpp:
 * 750-856), as RadioHandlerClass::OnDataPacket does after the r2iq when fc != 0
 * (Core/RadioHandler.cpp:33-37).  relative_freq = fc, the residual returned by
 * sddc_ddc_set_freq_offset; a new fc restarts the phase at 0 like
 * shift_limited_unroll_C_sse_init(fc, 0) (RadioHandler.cpp:291-296), the same fc keeps
 * it; 0 turns the mixer off.  While on, process_device / process_host advance the
 * mixer phase by their output length (stream order), and the single-channel path
 * only: process_channels_device returns SDDC_ERR_STATE.  Not for the drop-in class,
 * whose caller (RadioHandler) still mixes on the CPU. */
int   sddc_ddc_set_fine_tune(sddc_ddc_t *h, float relative_freq);

/* Complex samples produced per nblk input blocks at decimation d: nblk*(32768>>d). */
size_t sddc_ddc_output_samples(int d, int nblk);

/* ---- output format ---------------------------------- */
/* CF32 (default): (I,Q) float pairs, the reference's output (RadioHandler / Soapy
 * CF32, SoapySDDC/Streaming.cpp:12-50).  CS16: (I,Q) int16 pairs written by the
 * kernels' output stage, value = saturate_int16(rint(x * cs16_scale)) with
 * round-half-even; 4 bytes per complex sample instead of 8.  Applies to every
 * process_* call (the NCO, if on, mixes first).  CS16 scale must be > 0. */
#define SDDC_DDC_FMT_CF32 0
#define SDDC_DDC_FMT_CS16 1
int sddc_ddc_set_output_format(sddc_ddc_t *h, int format, float cs16_scale);

/* ---- the hot loop (fft_mt_r2iq_impl.hpp:15-152) ---------------------------- */
/* Device-resident; stateless apart from the fine-tune NCO phase.  d_in: device
 * int16 [4096 + nblk*65536] = the 4096-sample history followed by nblk blocks
 * (4-byte aligned start required).  d_out: device buffer of nblk*(32768>>d)
 * complex samples in the output format (CF32: float (I,Q), 8-byte aligned;
 * CS16: int16 (I,Q), 4-byte aligned), in stream order.  Uses the handle's
 * d / sideband / rand / tunebin.  Enqueued on `hip_stream` (a hipStream_t;
 * NULL = default stream); returns after launch. */
int sddc_ddc_process_device(sddc_ddc_t *h, const int16_t *d_in, int nblk,
                            void *d_out, void *hip_stream);

/* Many-channel DDC: one forward transform per
 * frame, shared by `nch` channels with their own tune bins (host array, each a
 * multiple of 4 in [0,4096)).  Channel c's stream starts `c*out_stride`
 * components (floats for CF32, int16 for CS16; 2 per complex sample) into
 * d_out.  All channels use the handle's d/sideband/rand/output format. */
int sddc_ddc_process_channels_device(sddc_ddc_t *h, const int16_t *d_in, int nblk,
                                     const int *tunebins, int nch,
                                     void *d_out, size_t out_stride,
                                     void *hip_stream);

/* Stateful, host buffers: the r2iq worker body.  Consumes nblk consecutive
 * blocks from `in` (host int16 [nblk*65536]), keeps the 4096-sample history
 * across calls (zero after create/reset), writes nblk*(32768>>d) complex
 * samples to `out` (host, in the output format).  Synchronous. */
int sddc_ddc_process_host(sddc_ddc_t *h, const int16_t *in, int nblk, void *out);

/* The same for blocks scattered in host memory (e.g. ring-buffer slots,
 * Core/dsp/ringbuffer.h): block i is blocks[i] (65536 int16). */
int sddc_ddc_process_blocks(sddc_ddc_t *h, const int16_t *const *blocks, int nblk,
                            void *out);

/* ---- ingest ---------------------------------------
 * Pin a caller-owned host region (hipHostRegister) so the host path DMAs blocks
 * from it and output into it directly instead of staging through the library's
 * pinned buffers.  Regions must not overlap; unregister before freeing them.
 * The host path runs chunks of 32 blocks through a two-slot pipeline (H2D,
 * kernel and D2H on separate streams), whichever memory is used. */
int sddc_ddc_register_host(sddc_ddc_t *h, void *ptr, size_t bytes);
int sddc_ddc_unregister_host(sddc_ddc_t *h, void *ptr);

#ifdef __cplusplus
}
#endif

#endif /* SDDC_DDC_H */
