/*
 * fft_mt_r2iq.h — drop-in replacement for ExtIO_sddc's Core/fft_mt_r2iq.h.
 *
 * Same class name, base class, constructor and virtual interface as the reference
 * (Core/fft_mt_r2iq.h:21-31), so RadioHandler (`new fft_mt_r2iq()`,
 * Core/RadioHandler.cpp:94-95), libsddc, the ExtIO DLL and SoapySDDC build and run
 * against it unchanged.  The DSP runs on an MI355X through the C ABI in sddc_ddc.h;
 * FFTW/MKL/Accelerate and the AVX/AVX2/AVX-512/NEON worker variants are gone.
 *
 * Behaviour kept from the reference:
 *   - Init(gain, in, out) designs the 7 filter banks (fft_mt_r2iq.cpp:147-227);
 *   - TurnOn() latches decimation and sideband, starts both rings and one worker
 *     (fft_mt_r2iq.cpp:111-129, impl.hpp:3-7); the history starts at zero;
 *   - updateRand() and setFreqOffset() take effect at the next input block the worker
 *     takes (impl.hpp:20,40): both are read per block, and a batch is cut where they change;
 *   - each input block yields 32768>>d complex floats; one output ring block
 *     (EXT_BLOCKLEN = 32768 complex) is released every 2^d input blocks
 *     (impl.hpp:100-148);
 *   - TurnOff() stops both rings and joins the worker (fft_mt_r2iq.cpp:131-143).
 * Different by design: the worker may hand several already-queued input blocks to
 * the GPU in one launch (never waiting for more than the first).
 *
 * Backend (environment SDDC_DDC_BACKEND, read by Init):
 *   hip  (default) the MI355X; no gfx950 device or a HIP error is reported on stderr and
 *        through lastError(), and the worker stops — never a silent CPU run;
 *   cpu  the library's AVX2 r2iq on the worker thread (the reference's
 *        fft_mt_r2iq_avx2.cpp worker, restated without FFTW);
 *   auto the MI355X, switching to the CPU backend — announced on stderr — when Init finds
 *        no usable device or a GPU call fails mid-stream (the failed batch is redone on the
 *        CPU from the same ring slots and history, so the output stream stays continuous).
 * SDDC_DDC_DEVICE selects the GPU (default 0).
 */
#pragma once

#include <atomic>
#include <cstdint>
#include <string>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "r2iq.h"

/* Core/fft_mt_r2iq.h:18-19 (values of config.h:49,80 — FFTN_R_ADC 8192, transferSize 131072) */
static const int halfFft = 4096;
static const int fftPerBuf = 11;

struct sddc_ddc;

class fft_mt_r2iq : public r2iqControlClass {
public:
    fft_mt_r2iq();
    virtual ~fft_mt_r2iq();

    float setFreqOffset(float offset);

    void Init(float gain, ringbuffer<int16_t> *buffers, ringbuffer<float> *obuffers);
    void TurnOn();
    void TurnOff(void);
    bool IsOn(void);

    /* additions (not part of r2iqControlClass) */
    const char *lastError() const { return last_error_.c_str(); }
    uint64_t blocksProcessed() const { return blocks_done_.load(); }
    /* "hip", "cpu" or "none" (no handle): the backend the worker runs on */
    const char *backendName() const;

private:
    void worker();
    void fail(const char *what);
    bool create_handle(int device);
    bool on() const;                  /* r2iqOn, read/written atomically */
    void set_on(bool v);
    bool switch_to_cpu(uint64_t consumed);

    ringbuffer<int16_t> *inputbuffer = nullptr;
    ringbuffer<float> *outputbuffer = nullptr;
    float GainScale = 0.0f;
    int mfftdim[NDECIDX];
    std::atomic<int> mtunebin;

    sddc_ddc *ddc_ = nullptr;         /* DDC handle (C ABI) */
    int device_ = 0;
    enum class Backend { hip, cpu, autoselect } mode_ = Backend::hip;
    std::atomic<int> backend_{-1};    /* SDDC_DDC_BACKEND_* of ddc_, -1 = none */
    std::thread worker_;
    void writer();

    /* batch IQ, double-buffered between the worker (GPU calls) and the writer thread
     * (copies into the output ring, getWritePtr/WriteDone); registered with the library */
    std::vector<float> out_stage_[2];
    int stage_n_[2] = {0, 0};         /* blocks in a filled stage, 0 = free */
    std::mutex stage_mu_;
    std::condition_variable stage_cv_;
    std::thread writer_;
    void *in_region_ = nullptr;       /* input ring storage registered for direct DMA */
    std::atomic<uint64_t> blocks_done_{0};
    int wc_base_ = 0;                 /* input ring write count at TurnOn */
    uint64_t consumed_ = 0;           /* input blocks taken since TurnOn */
    std::string last_error_;
};
