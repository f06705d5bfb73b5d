// ddc_runtime.cpp — implementation of the C ABI in include/sddc_ddc.h.
//
// Owns the per-handle device state that the reference keeps in fft_mt_r2iq
// (Core/fft_mt_r2iq.h:86-117): the filter bank (filterHw), the FFT "plans"
// (here: twiddle tables), the tune bin and the stream history.  A GPU handle's compute
// calls go to the gfx950 kernels only (no fallback); a handle created on
// SDDC_DDC_DEVICE_CPU holds the AVX2 backend (cpu/r2iq_cpu.h) instead and never calls HIP.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "cpu/r2iq_cpu.h"
#include "ddc_kernels.h"
#include "filterbank.h"
#include "fine_tune.h"
#include "sddc_fft.h"
#include "sddc_ddc.h"
#include "sddc_ddc_internal.h"

namespace {

thread_local std::string g_last_error;

int fail(int code, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define HIP_TRY(expr)                                                                         \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return fail(SDDC_ERR_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),  \
                        __FILE__, __LINE__);                                                  \
    } while (0)

// Restores the caller's current device on scope exit (torch and other users of
// the same process keep their own current device).
struct DeviceGuard {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) err = hipSetDevice(dev);
    }
    ~DeviceGuard()
    {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

constexpr int kHistory = SDDC_DDC_HALF_FFT;
constexpr int kBlock = SDDC_DDC_BLOCK;
constexpr int kHostChunk = 32;   // blocks per pipeline chunk on the host path
constexpr size_t kOutBlockMax = (size_t)SDDC_DDC_OUT_BLOCK * 2 * sizeof(float);   // bytes, CF32 d = 0

// The streams whose launches read a per-handle device table (the (P, Q) coefficients, the NCO
// staging buffer, the channel tune bins, the channel scratch rows).  The C ABI accepts any
// stream per call, so before a table is rewritten the writing stream waits for the last launch
// of EVERY stream that may still read it, not only the most recent one.
struct Readers {
    std::vector<std::pair<hipStream_t, hipEvent_t>> v;

    // after a launch on s that reads the tables
    hipError_t record(hipStream_t s)
    {
        for (auto &p : v)
            if (p.first == s) return hipEventRecord(p.second, s);
        if (v.size() >= 16) {   // bound the set: wait for all, forget them
            hipError_t e = sync();
            if (e != hipSuccess) return e;
            clear();
        }
        hipEvent_t ev = nullptr;
        hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        if (e != hipSuccess) return e;
        v.emplace_back(s, ev);
        return hipEventRecord(ev, s);
    }
    // stream s (about to rewrite a table) waits for every other reader's last launch
    hipError_t order_before(hipStream_t s) const
    {
        for (const auto &p : v)
            if (p.first != s) {
                hipError_t e = hipStreamWaitEvent(s, p.second, 0);
                if (e != hipSuccess) return e;
            }
        return hipSuccess;
    }
    // stream s waits for the last recorded launch on stream `other` (nothing to do when other is
    // s, or when `other` has no entry: entries are dropped only after a host sync of all of them)
    hipError_t order_after(hipStream_t other, hipStream_t s) const
    {
        if (other == s) return hipSuccess;
        for (const auto &p : v)
            if (p.first == other) return hipStreamWaitEvent(s, p.second, 0);
        return hipSuccess;
    }
    // the host waits for every reader (before a synchronous copy or a free)
    hipError_t sync() const
    {
        for (const auto &p : v) {
            hipError_t e = hipEventSynchronize(p.second);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    void clear()
    {
        for (auto &p : v) (void)hipEventDestroy(p.second);
        v.clear();
    }
};

}  // namespace

struct sddc_ddc {
    int device = 0;
    float gain = 0.f;
    int d = 0, lsb = 0, rand = 0, tunebin = SDDC_DDC_HALF_FFT / 4;   // ctor: mtunebin = halfFft/4
    int out_fmt = SDDC_DDC_FMT_CF32;       // output stage format
    float cs16_scale = 1.f;
    sddc::KernelTables tables;
    sddc::LaunchCache launch_cache;        // per-kernel resident workgroups and CUs of this device
    float2 *d_tables = nullptr;

    mutable std::mutex mu;                 // serialises the host path and buffer growth
    hipStream_t stream = nullptr;          // host path: compute stream

    // host path pipeline (process_host / process_blocks): two chunk slots; H2D on s_in,
    // kernel on `stream`, D2H on s_out, ordered by events.  The stream history (last 4096
    // input samples) stays on the device: the tail of the newest slot's input.
    struct HostSlot {
        int16_t *d_in = nullptr;           // [history | kHostChunk blocks]
        void *d_out = nullptr;
        int16_t *h_in = nullptr;           // pinned staging, used for unregistered callers
        void *h_out = nullptr;
        hipEvent_t e_h2d = nullptr, e_k = nullptr, e_d2h = nullptr;
    } hs[2];
    hipStream_t s_in = nullptr, s_out = nullptr;
    bool host_ready = false;
    int last_slot = -1, last_n = 0;        // where the history lives; -1 = zeros (create/reset)
    std::vector<std::pair<const char *, size_t>> regions;   // sddc_ddc_register_host

    int *d_tunebins = nullptr;             // channel tune bins (device)
    std::vector<int> tunebins_cached;
    int2 *d_windows = nullptr;             // per-chunk compact forward-bin windows (channels v2)
    int windows_d = -1;                    // d they were computed for; -2 = do not fit
    float2 *d_chscratch = nullptr;         // channels v2: per-workgroup split-spectrum rows
    int chscratch_rows = 0;
    Readers ch_readers;                    // streams of many-channel launches (tune bins, windows, scratch)

    // split x filter coefficients of the current (d, tunebin), rebuilt on device when either
    // changes; readers = the streams of single-channel launches that read them (and d_nco)
    // Each table set remembers the stream its last rebuild ran on (pq_s, fs_s): a launch
    // on another stream first waits for that stream's last recorded launch (Readers::order_after),
    // which is behind the rebuild (a rebuild is recorded like a launch).
    float4 *d_pq = nullptr;
    int pq_d = -1, pq_tb = -1;
    hipStream_t pq_s = nullptr;
    // the d = 0 wave kernel's per-tunebin tables: pqW (4096 float4) then twI (4096 float2)
    // the d = 0 fused-split kernel's per-tunebin tables: pqf (4096 float4) then fsl (768 float2)
    float4 *d_fs = nullptr;
    int fs_tb = -1;
    hipStream_t fs_s = nullptr;
    // the single-channel kernels' dynamic frame queues: a ring of kQueueSlots slots, one per launch
    // in turn.  A slot is zero when its launch starts and its last workgroup zeroes it again, so
    // the slot's next launch must start after that launch has finished: on the same stream that
    // is stream order; on another stream it waits for the slot's stream (q_s).  A slot whose
    // launch failed, or every slot after a HIP error, is zeroed stream-ordered before its next use.
    static constexpr int kQueueSlots = 64;
    unsigned *d_queue = nullptr;
    int queue_slot = 0;
    int slot_weights = sddc::kSlotWeighting;    // the persistent kernel's slot-weighted split (ddc_queue.hpp)
    sddc::FsSched fs_sched;                    // the d = 0 kernel's frame schedule (ddc_kernels.h)
    hipStream_t q_s[kQueueSlots] = {};
    bool q_used[kQueueSlots] = {};
    bool q_dirty[kQueueSlots] = {};
    Readers readers;

    // fused fine-tune NCO: host chain + per-launch [T | lane starts] staged through a
    // pinned 3-slot ring into d_nco (stream-ordered copy before each launch)
    float nco_fc = 0.f;
    sddc::FineTune nco;
    static constexpr int kNcoSlots = 3;
    float2 *h_nco[kNcoSlots] = {};
    hipEvent_t nco_ev[kNcoSlots] = {};
    size_t h_nco_cap = 0;                  // float2 per slot
    int nco_slot = 0;
    float2 *d_nco = nullptr;
    size_t d_nco_cap = 0;

    // history to start the next host-path call from (sddc_ddc_set_history)
    std::vector<int16_t> hist_override;

    // CPU handle (device SDDC_DDC_DEVICE_CPU): the AVX2 backend; no HIP object above exists
    std::unique_ptr<sddc::cpu::R2iq> cpu;

    // fault injection for failover tests (GPU handles): environment SDDC_DDC_INJECT_FAIL=N
    // makes the (N+1)-th process_* call fail with SDDC_ERR_HIP before any device work
    long inject_fail = -1;
    long inject_late = -1;   // SDDC_DDC_INJECT_FAIL_AFTER_D2H
};

static bool injected_failure(sddc_ddc_t *h)
{
    if (h->inject_fail < 0) return false;
    return h->inject_fail-- == 0;
}
// SDDC_DDC_INJECT_FAIL_AFTER_D2H=N: the (N+1)-th host call fails after its first chunk's kernel and
// D2H were issued, i.e. with device work in flight and the output partly written (a mid-stream
// HIP error as the drop-in's failover meets it)
static bool injected_late_failure(sddc_ddc_t *h)
{
    if (h->inject_late < 0) return false;
    return h->inject_late-- == 0;
}

extern "C" {

int sddc_ddc_abi_version(void) { return SDDC_DDC_ABI_VERSION; }

const char *sddc_ddc_last_error(void) { return g_last_error.c_str(); }

int sddc_ddc_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int sddc_ddc_kaiser(int ntaps, float astop, float fpass, float fstop, float *coef)
{
    return sddc::kaiser_window(ntaps, astop, fpass, fstop, coef);
}

int sddc_ddc_filter_taps(int d, float *taps)
{
    if (d < 0 || d >= SDDC_DDC_NDEC || !taps) return fail(SDDC_ERR_ARG, "filter_taps: bad d=%d or null", d);
    sddc::filter_taps(d, taps);
    return SDDC_OK;
}

int sddc_ddc_filter_response(float gain, int d, float *H)
{
    if (d < 0 || d >= SDDC_DDC_NDEC || !H) return fail(SDDC_ERR_ARG, "filter_response: bad d=%d or null", d);
    std::vector<std::complex<double>> h(SDDC_DDC_HALF_FFT);
    sddc::filter_response(gain, d, h.data());
    for (int i = 0; i < SDDC_DDC_HALF_FFT; i++) {
        H[2 * i] = (float)h[i].real();
        H[2 * i + 1] = (float)h[i].imag();
    }
    return SDDC_OK;
}

size_t sddc_ddc_output_samples(int d, int nblk)
{
    if (d < 0 || d >= SDDC_DDC_NDEC || nblk < 0) return 0;
    return (size_t)nblk * (size_t)(SDDC_DDC_OUT_BLOCK >> d);
}

int sddc_ddc_create(float gain, int device, sddc_ddc_t **out)
{
    if (!out) return fail(SDDC_ERR_ARG, "create: null out");
    *out = nullptr;
    if (device == SDDC_DDC_DEVICE_CPU) {
        if (!sddc::cpu::supported()) return fail(SDDC_ERR_NODEV, "create: the CPU backend needs AVX2 and FMA");
        auto *h = new (std::nothrow) sddc_ddc();
        if (!h) return fail(SDDC_ERR_NOMEM, "create: out of host memory");
        h->device = SDDC_DDC_DEVICE_CPU;
        h->gain = gain;
        try {
            std::vector<std::complex<double>> H((size_t)SDDC_DDC_NDEC * SDDC_DDC_HALF_FFT);
            for (int d = 0; d < SDDC_DDC_NDEC; d++) sddc::filter_response(gain, d, H.data() + (size_t)d * SDDC_DDC_HALF_FFT);
            h->cpu.reset(new sddc::cpu::R2iq(H.data()));
        } catch (const std::exception &ex) {
            delete h;
            return fail(SDDC_ERR_NOMEM, "create: %s", ex.what());
        }
        *out = h;
        return SDDC_OK;
    }
    if (device < 0) return fail(SDDC_ERR_ARG, "create: device %d (>= 0, or SDDC_DDC_DEVICE_CPU)", device);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(SDDC_ERR_NODEV, "create: no HIP device visible");
    if (device < 0 || device >= ndev) return fail(SDDC_ERR_NODEV, "create: device %d of %d", device, ndev);
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(SDDC_ERR_NODEV, "create: device %d is %s, the kernels are built for gfx950", device,
                    prop.gcnArchName);

    DeviceGuard g(device);
    HIP_TRY(g.err);

    auto *h = new (std::nothrow) sddc_ddc();
    if (!h) return fail(SDDC_ERR_NOMEM, "create: out of host memory");
    h->device = device;
    h->gain = gain;
    if (const char *inj = std::getenv("SDDC_DDC_INJECT_FAIL")) h->inject_fail = std::atol(inj);
    if (const char *inj = std::getenv("SDDC_DDC_INJECT_FAIL_AFTER_D2H")) h->inject_late = std::atol(inj);

    // ---- constant tables (one device allocation) ----
    auto W = [](double num, double den) {   // e^{-2 pi i num/den}, double -> float once
        const double a = -2.0 * M_PI * num / den;
        return make_float2((float)std::cos(a), (float)std::sin(a));
    };
    std::vector<float2> host;
    auto put = [&](size_t n) { size_t o = host.size(); host.resize(o + n, make_float2(0.f, 0.f)); return o; };
    const size_t o_tw4096 = put(4096), o_post = put(8192), o_p1 = put(15 * 16), o_recf = put(2 * 256);
    for (int k = 0; k < 4096; k++) host[o_tw4096 + k] = W(k, 4096);
    for (int k = 0; k < 8192; k++) host[o_post + k] = W(k, 8192);
    for (int r = 1; r < 16; r++)
        for (int s = 0; s < 16; s++) host[o_p1 + (r - 1) * 16 + s] = W((double)s * r, 256);
    for (int j = 0; j < 256; j++) {
        host[o_recf + j] = W(j, 4096);
        host[o_recf + 256 + j] = W(4.0 * j, 4096);
    }
    size_t o_hsel[SDDC_DDC_NDEC], o_q1[SDDC_DDC_NDEC], o_reci[SDDC_DDC_NDEC];
    std::vector<std::complex<double>> H(SDDC_DDC_HALF_FFT);
    for (int d = 0; d < SDDC_DDC_NDEC; d++) {
        const int mfft = SDDC_DDC_HALF_FFT >> d;
        sddc::filter_response(gain, d, H.data());
        o_hsel[d] = put(mfft);
        for (int m = 0; m < mfft; m++) {
            // inverse-input position m: H[m] (m < mfft/2), H[4096 - mfft + m] otherwise
            // (impl.hpp:90,94 with filter2 = filter + halfFft - mfft/2, impl.hpp:7)
            const std::complex<double> v = H[m < mfft / 2 ? m : SDDC_DDC_HALF_FFT - mfft + m];
            host[o_hsel[d] + m] = make_float2((float)(0.5 * v.real()), (float)(0.5 * v.imag()));
        }
        // inverse pass-1 table W_{16S}^{s r}, S = mfft/256 (mfft >= 512) or mfft/16
        const int S = mfft >= 512 ? mfft / 256 : mfft / 16;
        o_q1[d] = put(15 * (size_t)S);
        for (int r = 1; r < 16; r++)
            for (int s = 0; s < S; s++) host[o_q1[d] + (r - 1) * S + s] = W((double)s * r, 16.0 * S);
        // inverse pass-2 recurrence bases W_N^j, W_N^{4j}, j < N/16 (mfft >= 512)
        o_reci[d] = put(2 * 256);
        if (mfft >= 512) {
            for (int j = 0; j < mfft / 16; j++) {
                host[o_reci[d] + j] = W(j, mfft);
                host[o_reci[d] + 256 + j] = W(4.0 * j, mfft);
            }
        }
    }
    const size_t ntab = host.size();
    hipError_t e = hipMalloc(&h->d_tables, ntab * sizeof(float2));
    if (e == hipSuccess) e = hipMemcpy(h->d_tables, host.data(), ntab * sizeof(float2), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&h->d_pq, SDDC_DDC_HALF_FFT * sizeof(float4));
    if (e == hipSuccess) e = hipMalloc(&h->d_fs, 4096 * sizeof(float4) + 768 * sizeof(float2));
    if (e == hipSuccess)
        e = hipMalloc(&h->d_queue, (size_t)sddc_ddc::kQueueSlots * sddc::kFsQueueWords * sizeof(unsigned));
    if (e == hipSuccess)   // zeroed on the handle's stream and waited for: the first launch may be on any stream
        e = hipMemsetAsync(h->d_queue, 0, (size_t)sddc_ddc::kQueueSlots * sddc::kFsQueueWords * sizeof(unsigned),
                           h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) {
        sddc_ddc_destroy(h);
        return fail(SDDC_ERR_HIP, "create: %s", hipGetErrorString(e));
    }
    const float2 *T = h->d_tables;
    h->tables.tw4096 = T + o_tw4096;
    h->tables.post8192 = T + o_post;
    h->tables.tw_p1 = T + o_p1;
    h->tables.rec_f = T + o_recf;
    h->tables.lc = &h->launch_cache;
    for (int d = 0; d < SDDC_DDC_NDEC; d++) {
        h->tables.hsel[d] = T + o_hsel[d];
        h->tables.tw_q1[d] = T + o_q1[d];
        h->tables.rec_i[d] = T + o_reci[d];
    }
    *out = h;
    return SDDC_OK;
}

int sddc_ddc_backend(const sddc_ddc_t *h)
{
    if (!h) return fail(SDDC_ERR_ARG, "null handle");
    return h->cpu ? SDDC_DDC_BACKEND_CPU : SDDC_DDC_BACKEND_HIP;
}

int sddc_ddc_destroy(sddc_ddc_t *h)
{
    if (!h) return SDDC_OK;
    if (h->cpu) {
        delete h;
        return SDDC_OK;
    }
    {
        DeviceGuard g(h->device);
        if (h->stream) (void)hipStreamSynchronize(h->stream);
        // copies a failed call left in flight (host_pipeline returns on the first error) finish
        // before their buffers and registrations go
        if (h->s_in) (void)hipStreamSynchronize(h->s_in);
        if (h->s_out) (void)hipStreamSynchronize(h->s_out);
        // launches on the callers' streams may still read the tables below: wait for them first
        (void)h->readers.sync();
        (void)h->ch_readers.sync();
        if (h->d_tables) (void)hipFree(h->d_tables);
        for (auto &sl : h->hs) {
            if (sl.d_in) (void)hipFree(sl.d_in);
            if (sl.d_out) (void)hipFree(sl.d_out);
            if (sl.h_in) (void)hipHostFree(sl.h_in);
            if (sl.h_out) (void)hipHostFree(sl.h_out);
            for (hipEvent_t ev : {sl.e_h2d, sl.e_k, sl.e_d2h})
                if (ev) (void)hipEventDestroy(ev);
        }
        if (h->s_in) (void)hipStreamDestroy(h->s_in);
        if (h->s_out) (void)hipStreamDestroy(h->s_out);
        for (auto &r : h->regions) (void)hipHostUnregister(const_cast<char *>(r.first));
        if (h->d_tunebins) (void)hipFree(h->d_tunebins);
        if (h->d_windows) (void)hipFree(h->d_windows);
        if (h->d_chscratch) (void)hipFree(h->d_chscratch);
        if (h->d_pq) (void)hipFree(h->d_pq);
        if (h->d_fs) (void)hipFree(h->d_fs);
        if (h->d_queue) (void)hipFree(h->d_queue);
        h->readers.clear();
        h->ch_readers.clear();
        for (int i = 0; i < sddc_ddc::kNcoSlots; i++) {
            if (h->h_nco[i]) (void)hipHostFree(h->h_nco[i]);
            if (h->nco_ev[i]) (void)hipEventDestroy(h->nco_ev[i]);
        }
        if (h->d_nco) (void)hipFree(h->d_nco);
        if (h->stream) (void)hipStreamDestroy(h->stream);
    }
    delete h;
    return SDDC_OK;
}

int sddc_ddc_set_decimation(sddc_ddc_t *h, int d)
{
    if (!h) return fail(SDDC_ERR_ARG, "null handle");
    if (d < 0 || d >= SDDC_DDC_NDEC) return fail(SDDC_ERR_ARG, "decimation index %d outside 0..6", d);
    std::lock_guard<std::mutex> lk(h->mu);
    h->d = d;
    return SDDC_OK;
}

int sddc_ddc_set_sideband(sddc_ddc_t *h, int lsb)
{
    if (!h) return fail(SDDC_ERR_ARG, "null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    h->lsb = lsb ? 1 : 0;
    return SDDC_OK;
}

int sddc_ddc_set_rand(sddc_ddc_t *h, int rand)
{
    if (!h) return fail(SDDC_ERR_ARG, "null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    h->rand = rand ? 1 : 0;
    return SDDC_OK;
}

int sddc_ddc_set_tunebin(sddc_ddc_t *h, int tunebin)
{
    if (!h) return fail(SDDC_ERR_ARG, "null handle");
    if (tunebin < 0 || tunebin >= SDDC_DDC_HALF_FFT)
        return fail(SDDC_ERR_ARG, "tune bin %d outside [0,4096)", tunebin);
    std::lock_guard<std::mutex> lk(h->mu);
    h->tunebin = tunebin;
    return SDDC_OK;
}

int sddc_ddc_get_tunebin(const sddc_ddc_t *h)
{
    if (!h) return -1;
    std::lock_guard<std::mutex> lk(h->mu);
    return h->tunebin;
}

float sddc_ddc_set_freq_offset(sddc_ddc_t *h, float offset)
{
    if (!h) {
        fail(SDDC_ERR_ARG, "null handle");
        return 0.f;
    }
    // fft_mt_r2iq.cpp:104-106
    int tb = (int)(offset * SDDC_DDC_HALF_FFT / 4) * 4;
    const float delta = ((float)tb / SDDC_DDC_HALF_FFT) - offset;
    tb = std::min(std::max(tb, 0), SDDC_DDC_HALF_FFT - 4);
    std::lock_guard<std::mutex> lk(h->mu);
    const float ret = delta * (float)(1 << h->d);
    h->tunebin = tb;
    return ret;
}

int sddc_ddc_reset(sddc_ddc_t *h)
{
    if (!h) return fail(SDDC_ERR_ARG, "null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    h->last_slot = -1;   // the next host-path chunk starts from a zero history
    h->hist_override.clear();
    if (h->cpu) h->cpu->reset();
    return SDDC_OK;
}

int sddc_ddc_set_history(sddc_ddc_t *h, const int16_t *last4096)
{
    if (!h || !last4096) return fail(SDDC_ERR_ARG, "set_history: null handle or samples");
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->cpu) {
        h->cpu->set_history(last4096);
        return SDDC_OK;
    }
    h->hist_override.assign(last4096, last4096 + kHistory);
    return SDDC_OK;
}

// Stage [T | lane starts of this launch's 128-sample blocks] for the fused NCO.
static hipError_t stage_nco(sddc_ddc_t *h, int nblk, hipStream_t s)
{
    using sddc::FineTune;
    const long nb = (long)nblk * (SDDC_DDC_BLOCK / 2 >> h->d) / FineTune::kBlock;
    const size_t n = FineTune::kTable + (size_t)nb * FineTune::kLanes;
    hipError_t e;
    if (n > h->h_nco_cap) {
        for (int i = 0; i < sddc_ddc::kNcoSlots; i++) {
            if (h->nco_ev[i] && (e = hipEventSynchronize(h->nco_ev[i])) != hipSuccess) return e;
            if (h->h_nco[i]) (void)hipHostFree(h->h_nco[i]);
            h->h_nco[i] = nullptr;
        }
        h->h_nco_cap = 0;
        for (int i = 0; i < sddc_ddc::kNcoSlots; i++) {
            if ((e = hipHostMalloc(&h->h_nco[i], n * sizeof(float2), hipHostMallocDefault)) != hipSuccess) return e;
            if (!h->nco_ev[i] && (e = hipEventCreateWithFlags(&h->nco_ev[i], hipEventDisableTiming)) != hipSuccess)
                return e;
        }
        h->h_nco_cap = n;
    }
    if (n > h->d_nco_cap) {   // the previous launches may still read the old buffer
        if ((e = h->readers.sync()) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        if (h->d_nco) (void)hipFree(h->d_nco);
        h->d_nco = nullptr;
        h->d_nco_cap = 0;
        if ((e = hipMalloc(&h->d_nco, n * sizeof(float2))) != hipSuccess) return e;
        h->d_nco_cap = n;
    } else if ((e = h->readers.order_before(s)) != hipSuccess) {   // launches on other streams may still read d_nco
        return e;
    }
    const int slot = h->nco_slot;
    h->nco_slot = (slot + 1) % sddc_ddc::kNcoSlots;
    if ((e = hipEventSynchronize(h->nco_ev[slot])) != hipSuccess) return e;   // its last copy is done
    float2 *buf = h->h_nco[slot];
    std::memcpy(buf, h->nco.table(), FineTune::kTable * sizeof(float2));
    h->nco.starts(nb, buf + FineTune::kTable);
    if ((e = hipMemcpyAsync(h->d_nco, buf, n * sizeof(float2), hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    return hipEventRecord(h->nco_ev[slot], s);
}

// The next slot of the handle's dynamic-frame-queue ring for a launch on s (under h->mu, like
// every launch): ordered after the slot's previous launch, or zeroed first if that launch failed.
// *slot receives its index for queue_slot_launched.
static hipError_t next_queue_slot(sddc_ddc_t *h, hipStream_t s, unsigned **wq, int *slot)
{
    const int i = h->queue_slot;
    h->queue_slot = (i + 1) % sddc_ddc::kQueueSlots;
    *slot = i;
    *wq = h->d_queue + (size_t)i * sddc::kFsQueueWords;
    hipError_t e = hipSuccess;
    if (h->q_dirty[i]) {
        if (h->q_used[i]) e = h->readers.order_after(h->q_s[i], s);   // the failed launch may still run
        if (e == hipSuccess) e = hipMemsetAsync(*wq, 0, sddc::kFsQueueWords * sizeof(unsigned), s);
        if (e == hipSuccess) h->q_dirty[i] = false;
    } else if (h->q_used[i]) {
        e = h->readers.order_after(h->q_s[i], s);
    }
    return e;
}

// after the launch that took slot i: on success the slot's last user is s (the launch is recorded
// in readers right after); on failure the slot is zeroed before its next use, on a stream ordered
// after an event recorded on s here: hipGetLastError may report a sticky or earlier error for a
// kernel that was enqueued and still runs (readers.record of the success path is skipped then)
static void queue_slot_launched(sddc_ddc_t *h, int i, hipStream_t s, hipError_t e)
{
    h->q_s[i] = s;
    h->q_used[i] = true;
    if (e != hipSuccess) {
        h->q_dirty[i] = true;
        (void)h->readers.record(s);
    }
}

// a HIP error on a launch path: the state of every in-flight launch is unknown, so every queue
// slot is zeroed (stream-ordered) before its next use
static void queue_mark_all_dirty(sddc_ddc_t *h)
{
    for (int i = 0; i < sddc_ddc::kQueueSlots; i++) h->q_dirty[i] = true;
}

// a launch on s reads a table set last rebuilt on `built`: wait for that rebuild
static hipError_t order_after_build(sddc_ddc_t *h, hipStream_t built, hipStream_t s)
{
    return h->readers.order_after(built, s);
}

static hipError_t launch_single_impl(sddc_ddc_t *h, const int16_t *d_in, int nblk, void *d_out, hipStream_t s);

static hipError_t launch_single(sddc_ddc_t *h, const int16_t *d_in, int nblk, void *d_out, hipStream_t s)
{
    const hipError_t e = launch_single_impl(h, d_in, nblk, d_out, s);
    if (e != hipSuccess) queue_mark_all_dirty(h);
    return e;
}

static hipError_t launch_single_impl(sddc_ddc_t *h, const int16_t *d_in, int nblk, void *d_out, hipStream_t s)
{
    const bool nco = h->nco_fc != 0.f;
    if (nco) {
        hipError_t e = stage_nco(h, nblk, s);
        if (e != hipSuccess) return e;
    }
    const float2 *nco_starts = nco ? h->d_nco + sddc::FineTune::kTable : nullptr, *nco_trig = nco ? h->d_nco : nullptr;
    if (sddc::fs_path(h->d, h->tunebin)) {
        // d = 0 fused-split kernel: its (P, Q) by bin and output-modulation lane factors
        float4 *pqf = h->d_fs;
        float2 *fsl = reinterpret_cast<float2 *>(h->d_fs + 4096);
        if (h->fs_tb != h->tunebin) {
            hipError_t e = h->readers.order_before(s);   // launches on other streams may still read them
            if (e != hipSuccess) return e;
            h->fs_tb = -1;   // a failed rebuild leaves the tables unknown
            e = sddc::launch_build_fs_tables(h->tables, h->tunebin, pqf, fsl, s);
            if (e == hipSuccess) e = h->readers.record(s);
            if (e != hipSuccess) return e;
            h->fs_tb = h->tunebin;
            h->fs_s = s;
        } else if (hipError_t e = order_after_build(h, h->fs_s, s); e != hipSuccess) {
            return e;
        }
        // the default static schedule uses no queue slot; the queue and stealing schedules (A/B)
        // take one of the ring's slots per launch
        unsigned *wq = nullptr;
        int qi = -1;
        hipError_t e = hipSuccess;
        if (h->fs_sched.sched != 0 && (e = next_queue_slot(h, s, &wq, &qi)) != hipSuccess) return e;
        e = sddc::launch_frames_fs(h->tables, d_in, nblk, d_out, pqf, fsl, h->tunebin, h->lsb, h->rand,
                                   h->out_fmt == SDDC_DDC_FMT_CS16, h->cs16_scale, nco_starts, nco_trig, wq,
                                   h->fs_sched, h->device, s);
        if (qi >= 0) queue_slot_launched(h, qi, s, e);
        if (e != hipSuccess) return e;
        return h->readers.record(s);
    }
    if (h->pq_d != h->d || h->pq_tb != h->tunebin) {
        hipError_t e = h->readers.order_before(s);   // launches on other streams may still read d_pq
        if (e != hipSuccess) return e;
        h->pq_d = h->pq_tb = -1;
        e = sddc::launch_build_split_filter(h->tables, h->d, h->tunebin, h->d_pq, s);
        if (e == hipSuccess) e = h->readers.record(s);
        if (e != hipSuccess) return e;
        h->pq_d = h->d;
        h->pq_tb = h->tunebin;
        h->pq_s = s;
    } else if (hipError_t e = order_after_build(h, h->pq_s, s); e != hipSuccess) {
        return e;
    }
    hipError_t e = sddc::launch_frames_persistent(h->tables, h->d, d_in, nblk, d_out, h->d_pq, h->tunebin, h->lsb, h->rand,
                                         h->out_fmt == SDDC_DDC_FMT_CS16, h->cs16_scale, nco_starts, nco_trig,
                                         h->slot_weights, h->device, s);
    if (e != hipSuccess) return e;
    return h->readers.record(s);
}

int sddc_ddc_set_output_format(sddc_ddc_t *h, int format, float cs16_scale)
{
    if (!h) return fail(SDDC_ERR_ARG, "null handle");
    if (format != SDDC_DDC_FMT_CF32 && format != SDDC_DDC_FMT_CS16)
        return fail(SDDC_ERR_ARG, "unknown output format %d", format);
    if (format == SDDC_DDC_FMT_CS16 && !(std::isfinite(cs16_scale) && cs16_scale > 0.f))
        return fail(SDDC_ERR_ARG, "CS16 scale must be finite and > 0");
    std::lock_guard<std::mutex> lk(h->mu);
    h->out_fmt = format;
    h->cs16_scale = format == SDDC_DDC_FMT_CS16 ? cs16_scale : 1.f;
    return SDDC_OK;
}

int sddc_ddc_set_fine_tune(sddc_ddc_t *h, float relative_freq)
{
    if (!h) return fail(SDDC_ERR_ARG, "null handle");
    if (!std::isfinite(relative_freq)) return fail(SDDC_ERR_ARG, "fine tune: non-finite frequency");
    std::lock_guard<std::mutex> lk(h->mu);
    if (relative_freq != h->nco_fc) {   // RadioHandler.cpp:291-296: re-init only on change
        h->nco_fc = relative_freq;
        if (relative_freq != 0.f) h->nco.init(relative_freq, 0.0f);
    }
    return SDDC_OK;
}

/* internal (sddc_ddc_internal.h): a tuning parameter of the kernels, for A/B timing */
int sddc_ddc_internal_set_param(sddc_ddc_t *h, int param, int value)
{
    if (!h) return fail(SDDC_ERR_ARG, "null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    switch (param) {
    case SDDC_DDC_PARAM_SLOT_WEIGHTS:
        h->slot_weights = value != 0;
        return SDDC_OK;
    case SDDC_DDC_PARAM_FS_STATIC_PCT:
        if (value < 0 || value > 100) return fail(SDDC_ERR_ARG, "static share %d outside 0..100", value);
        h->fs_sched.static_pct = value;
        return SDDC_OK;
    case SDDC_DDC_PARAM_FS_FRAMES_PER_WG:
        if (value < 0 || value > 1024) return fail(SDDC_ERR_ARG, "frames per workgroup %d outside 0..1024", value);
        h->fs_sched.fpw = value;
        return SDDC_OK;
    case SDDC_DDC_PARAM_FS_SCHEDULE:
        if (value < 0 || value > 2) return fail(SDDC_ERR_ARG, "FS schedule %d outside 0..2", value);
        h->fs_sched.sched = value;
        return SDDC_OK;
    case SDDC_DDC_PARAM_FS_STEAL_MINREM:
        if (value < 0 || value > 64) return fail(SDDC_ERR_ARG, "steal threshold %d outside 0..64", value);
        h->fs_sched.minrem = value;
        return SDDC_OK;
    case SDDC_DDC_PARAM_FS_ZERO_ROWS:
        h->fs_sched.zr = value != 0;
        return SDDC_OK;
    case SDDC_DDC_PARAM_FS_SLOT_WEIGHTS: {
        for (int k = 0; k < 4 && value != 0; k++) {
            const int wk = (value >> (8 * k)) & 0xff;
            if (wk < 1 || wk > 127) return fail(SDDC_ERR_ARG, "slot weight %d of slot %d outside 1..127", wk, k);
        }
        h->fs_sched.slotw = (unsigned)value;
        return SDDC_OK;
    }
    case SDDC_DDC_PARAM_FS_STEAL_PUBLIC:
        if (value < 0 || value > 1024) return fail(SDDC_ERR_ARG, "public frames %d outside 0..1024", value);
        h->fs_sched.pub = value;
        return SDDC_OK;
    default:
        return fail(SDDC_ERR_ARG, "unknown parameter %d", param);
    }
}

static int check_process_args(sddc_ddc_t *h, const int16_t *in, int nblk, const void *out)
{
    if (!h) return fail(SDDC_ERR_ARG, "null handle");
    if (nblk <= 0 || nblk > SDDC_DDC_MAX_BLOCKS)
        return fail(SDDC_ERR_ARG, "nblk must be in 1..%d (got %d)", SDDC_DDC_MAX_BLOCKS, nblk);
    if (!in || !out) return fail(SDDC_ERR_ARG, "null buffer");
    if (((uintptr_t)in & 3) != 0) return fail(SDDC_ERR_ARG, "input must be 4-byte aligned");
    const unsigned oal = h->out_fmt == SDDC_DDC_FMT_CS16 ? 4 : 8;
    if (((uintptr_t)out & (oal - 1)) != 0) return fail(SDDC_ERR_ARG, "output must be %u-byte aligned", oal);
    return SDDC_OK;
}

int sddc_ddc_process_device(sddc_ddc_t *h, const int16_t *d_in, int nblk, void *d_out, void *hip_stream)
{
    if (!h) return fail(SDDC_ERR_ARG, "null handle");
    std::lock_guard<std::mutex> lk(h->mu);   // the call reads d, format, tune bin: one consistent set
    if (h->cpu) return fail(SDDC_ERR_STATE, "process_device: a CPU handle has no device path");
    int rc = check_process_args(h, d_in, nblk, d_out);
    if (rc) return rc;
    if (injected_failure(h)) return fail(SDDC_ERR_HIP, "injected failure (SDDC_DDC_INJECT_FAIL)");
    DeviceGuard g(h->device);
    HIP_TRY(g.err);
    HIP_TRY(launch_single(h, d_in, nblk, d_out, (hipStream_t)hip_stream));
    return SDDC_OK;
}

int sddc_ddc_process_channels_device(sddc_ddc_t *h, const int16_t *d_in, int nblk, const int *tunebins,
                                     int nch, void *d_out, size_t out_stride, void *hip_stream)
{
    if (!h) return fail(SDDC_ERR_ARG, "null handle");
    std::lock_guard<std::mutex> lk(h->mu);   // d, format and NCO state are read below
    if (h->cpu) return fail(SDDC_ERR_STATE, "process_channels_device: a CPU handle has no device path");
    int rc = check_process_args(h, d_in, nblk, d_out);
    if (rc) return rc;
    if (!tunebins || nch <= 0 || nch > SDDC_DDC_MAX_CHANNELS)
        return fail(SDDC_ERR_ARG, "channel count %d outside 1..%d", nch, SDDC_DDC_MAX_CHANNELS);
    for (int c = 0; c < nch; c++)
        if (tunebins[c] < 0 || tunebins[c] >= SDDC_DDC_HALF_FFT)
            return fail(SDDC_ERR_ARG, "channel %d tune bin %d outside [0,4096)", c, tunebins[c]);
    if (h->nco_fc != 0.f) return fail(SDDC_ERR_STATE, "fine-tune NCO is single-channel; set it to 0 first");
    const size_t need = (size_t)nblk * (size_t)(SDDC_DDC_OUT_BLOCK >> h->d) * 2;
    if (nch > 1 && out_stride < need)
        return fail(SDDC_ERR_ARG, "out_stride %zu < %zu components per channel", out_stride, need);
    if (nch > 1 && (out_stride & 1))   // channels start on whole complex samples
        return fail(SDDC_ERR_ARG, "out_stride %zu must be even (components, 2 per complex sample)", out_stride);
    const int cs16 = h->out_fmt == SDDC_DDC_FMT_CS16;
    DeviceGuard g(h->device);
    HIP_TRY(g.err);
    hipStream_t s = (hipStream_t)hip_stream;
    const bool v2 = h->d >= 4;
    const bool changed = h->tunebins_cached.size() != (size_t)nch ||
                         !std::equal(h->tunebins_cached.begin(), h->tunebins_cached.end(), tunebins);
    if (changed || (v2 && h->windows_d != h->d && h->windows_d != -2 - 8 * h->d)) {
        // earlier launches, on any stream, may still read the device copies
        HIP_TRY(h->ch_readers.sync());
        HIP_TRY(hipStreamSynchronize(s));
    }
    if (changed) {
        if (!h->d_tunebins) HIP_TRY(hipMalloc(&h->d_tunebins, SDDC_DDC_MAX_CHANNELS * sizeof(int)));
        h->tunebins_cached.assign(tunebins, tunebins + nch);
        h->windows_d = -1;
        // synchronous: the host array may go away after we return
        HIP_TRY(hipMemcpy(h->d_tunebins, tunebins, nch * sizeof(int), hipMemcpyHostToDevice));
    }
    const int2 *windows = nullptr;
    if (v2) {
        if (h->windows_d != h->d && h->windows_d != -2 - 8 * h->d) {
            std::vector<int2> w((SDDC_DDC_MAX_CHANNELS + 127) / 128);
            if (sddc::channel_windows(h->d, tunebins, nch, w.data())) {
                if (!h->d_windows) HIP_TRY(hipMalloc(&h->d_windows, w.size() * sizeof(int2)));
                HIP_TRY(hipMemcpy(h->d_windows, w.data(), w.size() * sizeof(int2), hipMemcpyHostToDevice));
                h->windows_d = h->d;
            } else {
                h->windows_d = -2 - 8 * h->d;   // spread-out tune bins: the full-spectrum form
            }
        }
        if (h->windows_d == h->d) windows = h->d_windows;
    }
    if (((v2 && windows && nch > 128) || !v2) && !h->d_chscratch) {
        // one 4096-bin row per resident workgroup (<= 4 per CU), 32 KB each
        int cus = 0;
        HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device));
        HIP_TRY(hipMalloc(&h->d_chscratch, (size_t)cus * 4 * SDDC_DDC_HALF_FFT * sizeof(float2)));
        h->chscratch_rows = cus * 4;
    }
    // the scratch rows are per handle: a launch must not overlap one on another stream
    if (h->d_chscratch) HIP_TRY(h->ch_readers.order_before(s));
    if (v2)
        HIP_TRY(sddc::launch_channels_v2(h->tables, h->d, d_in, nblk, h->d_tunebins, nch, d_out, out_stride,
                                         h->lsb, h->rand, cs16, h->cs16_scale, windows, h->d_chscratch,
                                         h->chscratch_rows, h->device, s));
    else
        HIP_TRY(sddc::launch_channels_p(h->tables, h->d, d_in, nblk, h->d_tunebins, nch, d_out, out_stride,
                                        h->lsb, h->rand, cs16, h->cs16_scale, h->d_chscratch, h->chscratch_rows,
                                        h->device, s));
    HIP_TRY(h->ch_readers.record(s));
    return SDDC_OK;
}

// ---- host path: pipelined chunks ------------------------------------------------------
extern "C++" {

static hipError_t host_setup(sddc_ddc_t *h)
{
    if (h->host_ready) return hipSuccess;
    hipError_t e;
    const size_t in_bytes = (kHistory + (size_t)kHostChunk * kBlock) * sizeof(int16_t);
    const size_t out_bytes = (size_t)kHostChunk * kOutBlockMax;
    for (auto &sl : h->hs) {
        if ((e = hipMalloc(&sl.d_in, in_bytes)) != hipSuccess) return e;
        if ((e = hipMalloc(&sl.d_out, out_bytes)) != hipSuccess) return e;
        if ((e = hipHostMalloc(&sl.h_in, in_bytes, hipHostMallocDefault)) != hipSuccess) return e;
        if ((e = hipHostMalloc(&sl.h_out, out_bytes, hipHostMallocDefault)) != hipSuccess) return e;
        for (hipEvent_t *ev : {&sl.e_h2d, &sl.e_k, &sl.e_d2h})
            if ((e = hipEventCreateWithFlags(ev, hipEventDisableTiming)) != hipSuccess) return e;
    }
    if ((e = hipStreamCreateWithFlags(&h->s_in, hipStreamNonBlocking)) != hipSuccess) return e;
    if ((e = hipStreamCreateWithFlags(&h->s_out, hipStreamNonBlocking)) != hipSuccess) return e;
    h->host_ready = true;
    return hipSuccess;
}

// true if [p, p + bytes) lies in memory registered through sddc_ddc_register_host
static bool host_registered(const sddc_ddc_t *h, const void *p, size_t bytes)
{
    const char *c = static_cast<const char *>(p);
    for (const auto &r : h->regions)
        if (c >= r.first && c + bytes <= r.first + r.second) return true;
    return false;
}

// nblk input blocks, block i at src(i) (host), output written contiguously to out.
// Chunk k of kHostChunk blocks goes through slot k % 2:
//   s_in   : wait e_k (kernel k-2 done with d_in) -> history D2D from the newest slot
//            -> H2D of the blocks (direct from registered memory, else via h_in) -> e_h2d
//   stream : wait e_h2d, e_d2h (D2H k-2 done with d_out) -> kernel -> e_k
//   s_out  : wait e_k -> D2H (direct into registered memory, else into h_out) -> e_d2h
// The host copies staged output of chunk k-1 while chunk k is in flight.
template <class Src>
static int host_pipeline(sddc_ddc_t *h, int nblk, Src src, void *out)
{
    HIP_TRY(host_setup(h));
    // one chunk: nothing to overlap, so skip the cross-stream event hops
    hipStream_t s_in = nblk <= kHostChunk ? h->stream : h->s_in;
    hipStream_t s_out = nblk <= kHostChunk ? h->stream : h->s_out;
    const size_t per_out = (size_t)(SDDC_DDC_OUT_BLOCK >> h->d) * (h->out_fmt == SDDC_DDC_FMT_CS16 ? 4 : 8);
    const size_t blk_bytes = (size_t)kBlock * sizeof(int16_t);
    char *outb = static_cast<char *>(out);
    const bool out_direct = host_registered(h, out, (size_t)nblk * per_out);
    int pend_slot = -1, pend_n = 0;        // staged output not yet copied to the caller
    size_t pend_off = 0;
    auto drain = [&]() -> int {
        if (pend_slot < 0) return SDDC_OK;
        HIP_TRY(hipEventSynchronize(h->hs[pend_slot].e_d2h));
        std::memcpy(outb + pend_off, h->hs[pend_slot].h_out, (size_t)pend_n * per_out);
        pend_slot = -1;
        return SDDC_OK;
    };
    int slot = h->last_slot < 0 ? 0 : 1 - h->last_slot;
    for (int done = 0; done < nblk; done += kHostChunk, slot ^= 1) {
        const int n = std::min(kHostChunk, nblk - done);
        auto &sl = h->hs[slot];
        // ---- input: history, then the blocks ----
        HIP_TRY(hipStreamWaitEvent(s_in, sl.e_k, 0));
        if (!h->hist_override.empty()) {   // sddc_ddc_set_history (pageable source: staged copy)
            HIP_TRY(hipMemcpyAsync(sl.d_in, h->hist_override.data(), kHistory * sizeof(int16_t),
                                   hipMemcpyHostToDevice, s_in));
            HIP_TRY(hipStreamSynchronize(s_in));   // the vector is cleared below
            h->hist_override.clear();
        } else if (h->last_slot < 0) {
            HIP_TRY(hipMemsetAsync(sl.d_in, 0, kHistory * sizeof(int16_t), s_in));
        } else {
            const auto &prev = h->hs[h->last_slot];
            HIP_TRY(hipMemcpyAsync(sl.d_in, prev.d_in + (size_t)h->last_n * kBlock, kHistory * sizeof(int16_t),
                                   hipMemcpyDeviceToDevice, s_in));
        }
        bool staged_in = false;
        for (int i = 0; i < n;) {
            const int16_t *p = src(done + i);
            int run = 1;   // merge blocks that are contiguous in host memory
            while (i + run < n && src(done + i + run) == p + (size_t)run * kBlock) run++;
            int16_t *dst = sl.d_in + kHistory + (size_t)i * kBlock;
            if (host_registered(h, p, run * blk_bytes)) {
                HIP_TRY(hipMemcpyAsync(dst, p, run * blk_bytes, hipMemcpyHostToDevice, s_in));
            } else {
                if (!staged_in) HIP_TRY(hipEventSynchronize(sl.e_h2d));   // h_in free again
                staged_in = true;
                std::memcpy(sl.h_in + (size_t)i * kBlock, p, run * blk_bytes);
                HIP_TRY(hipMemcpyAsync(dst, sl.h_in + (size_t)i * kBlock, run * blk_bytes, hipMemcpyHostToDevice,
                                       s_in));
            }
            i += run;
        }
        HIP_TRY(hipEventRecord(sl.e_h2d, s_in));
        h->last_slot = slot;
        h->last_n = n;
        // ---- kernel ----
        HIP_TRY(hipStreamWaitEvent(h->stream, sl.e_h2d, 0));
        HIP_TRY(hipStreamWaitEvent(h->stream, sl.e_d2h, 0));
        HIP_TRY(launch_single(h, sl.d_in, n, sl.d_out, h->stream));
        HIP_TRY(hipEventRecord(sl.e_k, h->stream));
        // ---- output ----
        if (int rc = drain()) return rc;   // chunk k-1's staged output (its slot is reused next)
        HIP_TRY(hipStreamWaitEvent(s_out, sl.e_k, 0));
        if (out_direct) {
            HIP_TRY(hipMemcpyAsync(outb + (size_t)done * per_out, sl.d_out, (size_t)n * per_out,
                                   hipMemcpyDeviceToHost, s_out));
        } else {
            HIP_TRY(hipMemcpyAsync(sl.h_out, sl.d_out, (size_t)n * per_out, hipMemcpyDeviceToHost, s_out));
            pend_slot = slot;
            pend_n = n;
            pend_off = (size_t)done * per_out;
        }
        HIP_TRY(hipEventRecord(sl.e_d2h, s_out));
        if (done == 0 && injected_late_failure(h))
            return fail(SDDC_ERR_HIP, "injected failure after the first chunk's D2H (SDDC_DDC_INJECT_FAIL_AFTER_D2H)");
    }
    if (int rc = drain()) return rc;
    HIP_TRY(hipStreamSynchronize(s_out));
    HIP_TRY(hipStreamSynchronize(s_in));   // callers may reuse their input buffers
    return SDDC_OK;
}
}  // extern "C++"

// CPU handle: the whole call on the calling thread (cpu/r2iq_cpu.h)
static int cpu_process(sddc_ddc_t *h, const int16_t *const *blocks, int nblk, void *out)
{
    sddc::cpu::Params p;
    p.d = h->d;
    p.tunebin = h->tunebin;
    p.lsb = h->lsb != 0;
    p.rand = h->rand != 0;
    p.cs16 = h->out_fmt == SDDC_DDC_FMT_CS16;
    p.scale = h->cs16_scale;
    std::vector<float2> starts;
    if (h->nco_fc != 0.f) {
        const long nb = (long)nblk * (SDDC_DDC_OUT_BLOCK >> h->d) / sddc::FineTune::kBlock;
        starts.resize((size_t)nb * sddc::FineTune::kLanes);
        h->nco.starts(nb, starts.data());
        p.nco_trig = reinterpret_cast<const float *>(h->nco.table());
        p.nco_starts = reinterpret_cast<const float *>(starts.data());
    }
    try {
        h->cpu->process(blocks, nblk, out, p);
    } catch (const std::exception &ex) {
        return fail(SDDC_ERR_NOMEM, "cpu backend: %s", ex.what());
    }
    return SDDC_OK;
}

int sddc_ddc_process_host(sddc_ddc_t *h, const int16_t *in, int nblk, void *out)
{
    if (!h) return fail(SDDC_ERR_ARG, "null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    int rc = check_process_args(h, in, nblk, out);
    if (rc) return rc;
    if (h->cpu) {
        std::vector<const int16_t *> blocks((size_t)nblk);
        for (int i = 0; i < nblk; i++) blocks[i] = in + (size_t)i * kBlock;
        return cpu_process(h, blocks.data(), nblk, out);
    }
    if (injected_failure(h)) return fail(SDDC_ERR_HIP, "injected failure (SDDC_DDC_INJECT_FAIL)");
    DeviceGuard g(h->device);
    HIP_TRY(g.err);
    return host_pipeline(h, nblk, [in](int i) { return in + (size_t)i * kBlock; }, out);
}

int sddc_ddc_process_blocks(sddc_ddc_t *h, const int16_t *const *blocks, int nblk, void *out)
{
    if (!h) return fail(SDDC_ERR_ARG, "null handle");
    if (!blocks) return fail(SDDC_ERR_ARG, "null block list");
    std::lock_guard<std::mutex> lk(h->mu);
    int rc = check_process_args(h, nblk > 0 ? blocks[0] : nullptr, nblk, out);
    if (rc) return rc;
    for (int i = 0; i < nblk; i++)
        if (!blocks[i] || ((uintptr_t)blocks[i] & 3)) return fail(SDDC_ERR_ARG, "block %d null or unaligned", i);
    if (h->cpu) return cpu_process(h, blocks, nblk, out);
    if (injected_failure(h)) return fail(SDDC_ERR_HIP, "injected failure (SDDC_DDC_INJECT_FAIL)");
    DeviceGuard g(h->device);
    HIP_TRY(g.err);
    return host_pipeline(h, nblk, [blocks](int i) { return blocks[i]; }, out);
}

int sddc_ddc_register_host(sddc_ddc_t *h, void *ptr, size_t bytes)
{
    if (!h || !ptr || !bytes) return fail(SDDC_ERR_ARG, "register_host: null handle/pointer or zero size");
    std::lock_guard<std::mutex> lk(h->mu);
    for (const auto &r : h->regions)
        if (static_cast<char *>(ptr) < r.first + r.second && r.first < static_cast<char *>(ptr) + bytes)
            return fail(SDDC_ERR_ARG, "register_host: overlaps a registered region");
    if (!h->cpu) {   // a CPU handle reads host memory directly: bookkeeping only
        DeviceGuard g(h->device);
        HIP_TRY(g.err);
        HIP_TRY(hipHostRegister(ptr, bytes, hipHostRegisterDefault));
    }
    h->regions.emplace_back(static_cast<const char *>(ptr), bytes);
    return SDDC_OK;
}

int sddc_ddc_unregister_host(sddc_ddc_t *h, void *ptr)
{
    if (!h || !ptr) return fail(SDDC_ERR_ARG, "unregister_host: null handle/pointer");
    std::lock_guard<std::mutex> lk(h->mu);
    for (size_t i = 0; i < h->regions.size(); i++) {
        if (h->regions[i].first == ptr) {
            // in-flight host-path copies finished when process_* returned (synchronous)
            if (!h->cpu) {
                DeviceGuard g(h->device);
                HIP_TRY(g.err);
                HIP_TRY(hipHostUnregister(ptr));
            }
            h->regions.erase(h->regions.begin() + (long)i);
            return SDDC_OK;
        }
    }
    return fail(SDDC_ERR_ARG, "unregister_host: %p was not registered", ptr);
}

/* ---- batched FFTs (include/sddc_fft.h) ------------------------------------ */
int sddc_fft_supported(int kind, int n)
{
    const bool pow2 = n > 0 && (n & (n - 1)) == 0;
    if (!pow2) return 0;
    if (kind == 0) return n >= 64 && n <= 4096;
    if (kind == 1) return n >= 128 && n <= 8192;
    return 0;
}

int sddc_fft_c2c(const void *in, void *out, int n, int batch, int direction, void *hip_stream)
{
    if (!sddc_fft_supported(0, n)) return fail(SDDC_ERR_ARG, "c2c size %d unsupported (64..4096, power of 2)", n);
    if (batch <= 0 || !in || !out) return fail(SDDC_ERR_ARG, "c2c: batch %d / null buffer", batch);
    if (direction != SDDC_FFT_FORWARD && direction != SDDC_FFT_BACKWARD)
        return fail(SDDC_ERR_ARG, "c2c: direction must be -1 or +1");
    hipStream_t s = (hipStream_t)hip_stream;
    HIP_TRY(sddc::fft_prepare(s));
    HIP_TRY(sddc::fft_c2c(in, out, n, batch, direction, s));
    return SDDC_OK;
}

int sddc_fft_r2c(const float *in, void *out, int n, int batch, void *hip_stream)
{
    if (!sddc_fft_supported(1, n)) return fail(SDDC_ERR_ARG, "r2c size %d unsupported (128..8192, power of 2)", n);
    if (batch <= 0 || !in || !out) return fail(SDDC_ERR_ARG, "r2c: batch %d / null buffer", batch);
    if (in == out) return fail(SDDC_ERR_ARG, "r2c: in place is not supported");
    hipStream_t s = (hipStream_t)hip_stream;
    HIP_TRY(sddc::fft_prepare(s));
    HIP_TRY(sddc::fft_r2c(in, out, n, batch, s));
    return SDDC_OK;
}

}  // extern "C"
