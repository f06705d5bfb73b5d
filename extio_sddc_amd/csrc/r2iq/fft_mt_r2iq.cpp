// fft_mt_r2iq.cpp — the drop-in r2iq class (include/fft_mt_r2iq.h) over the C ABI.
//
// Replaces Core/fft_mt_r2iq.cpp + fft_mt_r2iq_{def,avx,avx2,avx512,neon}.cpp +
// fft_mt_r2iq_impl.hpp.  The worker keeps the reference's ring protocol
// (impl.hpp:15-152): one getReadPtr/ReadDone per input block, getWritePtr when the
// output slot position (seq & (2^d-1)) is 0, WriteDone when it is 2^d-1.  The DSP
// itself (convert, r2c, shift x filter, inverse, overlap-discard) is one GPU call per
// batch of queued blocks through sddc_ddc_process_blocks(), which DMAs the blocks
// straight out of the input ring's slots (the ring storage is registered with the
// library at TurnOn) into a pinned batch buffer of IQ.
#include "fft_mt_r2iq.h"

#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "batching.h"
#include "sddc_ddc.h"

// ---- ABI guard: the base class must be byte-identical to Core/r2iq.h ----------------
#pragma GCC diagnostic push
#pragma GCC diagnostic ignored "-Winvalid-offsetof"
namespace {
struct LayoutProbe : r2iqControlClass {
    static constexpr size_t dec();
    static constexpr size_t on();
    static constexpr size_t ratio();
};
constexpr size_t LayoutProbe::dec() { return offsetof(LayoutProbe, mdecimation); }
constexpr size_t LayoutProbe::on() { return offsetof(LayoutProbe, r2iqOn); }
constexpr size_t LayoutProbe::ratio() { return offsetof(LayoutProbe, mratio); }
}  // namespace
static_assert(sizeof(r2iqControlClass) == 48, "r2iqControlClass layout differs from Core/r2iq.h");
static_assert(LayoutProbe::dec() == 8 && LayoutProbe::on() == 12 && LayoutProbe::ratio() == 16,
              "r2iqControlClass field offsets differ from Core/r2iq.h");
#pragma GCC diagnostic pop

static constexpr int kBlock = 65536;     // transferSamples, config.h:80-81

// r2iqOn is a plain bool of the ABI-fixed base class (Core/r2iq.h), written by TurnOn/TurnOff
// on the caller's thread and polled by the worker and writer threads.  Every access here is an
// atomic one on that same byte (acquire/release), so the layout stays and the accesses do not
// race (the reference reads it unsynchronised, impl.hpp:15; found by the TSan build).
bool fft_mt_r2iq::on() const { return __atomic_load_n(&r2iqOn, __ATOMIC_ACQUIRE); }
void fft_mt_r2iq::set_on(bool v) { __atomic_store_n(&r2iqOn, v, __ATOMIC_RELEASE); }
// input blocks per GPU call: the blocks already queued in the 32-transfer ring (config.h:46), up
// to 28, leaving the producer 4 free slots while the batch is copied.  At real-time rates the
// queue holds a block or two and batches stay small; in the saturated benchmark_test procedure
// 28 runs +21-27 % faster than 16 at decimate 0 (6.47 vs 5.09 GS/s input at 64 MHz,
// profiles/r04/e2e/benchmark_test_maxbatch*.jsonl)
static constexpr int kMaxBatch = 28;

// The contiguous storage behind a ring's slots (ringbuffer::setBlockSize allocates all
// slots in one array, Core/dsp/ringbuffer.h:150-165): walk peekReadPtr over one period.
template <class T>
static bool ring_region(ringbuffer<T> *rb, void **base, size_t *bytes)
{
    T *p0 = rb->peekReadPtr(0);
    if (!p0 || rb->getBlockSize() <= 0) return false;
    T *lo = p0, *hi = p0;
    for (int k = 1; k <= 4096; k++) {
        T *p = rb->peekReadPtr(k);
        if (p == p0) {
            *base = lo;
            *bytes = (size_t)(hi - lo + rb->getBlockSize()) * sizeof(T);
            return true;
        }
        lo = p < lo ? p : lo;
        hi = p > hi ? p : hi;
    }
    return false;
}

// The base-class constructor lives in the r2iq implementation (Core/fft_mt_r2iq.cpp:26-37).
r2iqControlClass::r2iqControlClass()
{
    r2iqOn = false;
    randADC = false;
    sideband = false;
    mdecimation = 0;
    for (int i = 0; i < NDECIDX; i++) mratio[i] = 1 << i;
}

fft_mt_r2iq::fft_mt_r2iq() : r2iqControlClass()
{
    mtunebin.store(halfFft / 4);                        // fft_mt_r2iq.cpp:43
    for (int i = 0; i < NDECIDX; i++) mfftdim[i] = halfFft >> i;   // :44-48
    const char *dev = std::getenv("SDDC_DDC_DEVICE");
    device_ = dev ? std::atoi(dev) : 0;
}

const char *fft_mt_r2iq::backendName() const
{
    const int b = backend_.load();
    return b == SDDC_DDC_BACKEND_CPU ? "cpu" : b == SDDC_DDC_BACKEND_HIP ? "hip" : "none";
}

// A fresh handle on `device` (or SDDC_DDC_DEVICE_CPU) with the output stages registered.
bool fft_mt_r2iq::create_handle(int device)
{
    if (ddc_) {
        sddc_ddc_destroy(ddc_);
        ddc_ = nullptr;
        backend_.store(-1);
    }
    if (sddc_ddc_create(GainScale, device, &ddc_) != SDDC_OK) {
        ddc_ = nullptr;
        return false;
    }
    backend_.store(sddc_ddc_backend(ddc_));
    for (auto &st : out_stage_)   // pinned for direct D2H; on failure the library stages through its own buffers
        (void)sddc_ddc_register_host(ddc_, st.data(), st.size() * sizeof(float));
    return true;
}

// SDDC_DDC_BACKEND=auto after a GPU failure in the worker: continue on a CPU handle from the
// same stream position.  The history is the tail of the last block taken (still readable at
// peekReadPtr(-1), Core/dsp/ringbuffer.h; the reference reads it there, impl.hpp:32).
bool fft_mt_r2iq::switch_to_cpu(uint64_t consumed)
{
    std::fprintf(stderr, "[fft_mt_r2iq] GPU backend failed (%s); SDDC_DDC_BACKEND=auto: continuing on the CPU\n",
                 last_error_.c_str());
    if (in_region_) {   // the GPU handle's registration goes with it
        (void)sddc_ddc_unregister_host(ddc_, in_region_);
        in_region_ = nullptr;
    }
    if (!create_handle(SDDC_DDC_DEVICE_CPU)) return false;
    if (sddc_ddc_set_decimation(ddc_, mdecimation) || sddc_ddc_set_sideband(ddc_, getSideband()) ||
        sddc_ddc_reset(ddc_))
        return false;
    if (consumed > 0 && sddc_ddc_set_history(ddc_, inputbuffer->peekReadPtr(-1) + kBlock - halfFft))
        return false;
    return true;
}

fft_mt_r2iq::~fft_mt_r2iq()
{
    if (worker_.joinable()) TurnOff();
    if (ddc_) sddc_ddc_destroy(ddc_);
}

void fft_mt_r2iq::fail(const char *what)
{
    last_error_ = std::string(what) + ": " + sddc_ddc_last_error();
    std::fprintf(stderr, "[fft_mt_r2iq] %s\n", last_error_.c_str());
}

float fft_mt_r2iq::setFreqOffset(float offset)
{
    // fft_mt_r2iq.cpp:101-109: align to 4 bins, return the residual for the fine-tune NCO.
    int tb = (int)(offset * halfFft / 4) * 4;
    const float delta = ((float)tb / halfFft) - offset;
    const float ret = delta * getRatio();
    if (tb < 0) tb = 0;                                  // the reference would read out of range
    if (tb > halfFft - 4) tb = halfFft - 4;
    mtunebin.store(tb);
    return ret;
}

void fft_mt_r2iq::Init(float gain, ringbuffer<int16_t> *input, ringbuffer<float> *obuffers)
{
    inputbuffer = input;
    outputbuffer = obuffers;
    GainScale = gain;
    const char *be = std::getenv("SDDC_DDC_BACKEND");
    mode_ = !be || !std::strcmp(be, "hip") ? Backend::hip
          : !std::strcmp(be, "cpu")        ? Backend::cpu
          : !std::strcmp(be, "auto")       ? Backend::autoselect
                                           : Backend::hip;
    if (be && mode_ == Backend::hip && std::strcmp(be, "hip"))
        std::fprintf(stderr, "[fft_mt_r2iq] SDDC_DDC_BACKEND=%s unknown (hip|cpu|auto): using hip\n", be);
    for (auto &st : out_stage_) st.assign((size_t)kMaxBatch * 8 * halfFft * 2, 0.f);
    if (create_handle(mode_ == Backend::cpu ? SDDC_DDC_DEVICE_CPU : device_)) return;
    fail("Init: sddc_ddc_create");
    if (mode_ != Backend::autoselect) return;
    std::fprintf(stderr, "[fft_mt_r2iq] SDDC_DDC_BACKEND=auto: no usable GPU, using the CPU backend\n");
    if (!create_handle(SDDC_DDC_DEVICE_CPU)) fail("Init: CPU backend");
}

void fft_mt_r2iq::TurnOn()
{
    if (!ddc_ || !inputbuffer || !outputbuffer) {
        last_error_ = "TurnOn without a successful Init";
        std::fprintf(stderr, "[fft_mt_r2iq] %s\n", last_error_.c_str());
        return;
    }
    set_on(true);
    inputbuffer->Start();
    outputbuffer->Start();
    void *base = nullptr;
    size_t bytes = 0;
    if (ring_region(inputbuffer, &base, &bytes) && sddc_ddc_register_host(ddc_, base, bytes) == SDDC_OK)
        in_region_ = base;   // else process_blocks stages the slots (still correct)
    wc_base_ = inputbuffer->getWriteCount();
    consumed_ = 0;
    stage_n_[0] = stage_n_[1] = 0;
    worker_ = std::thread([this] { worker(); });
    writer_ = std::thread([this] { writer(); });
}

void fft_mt_r2iq::TurnOff(void)
{
    set_on(false);
    if (inputbuffer) inputbuffer->Stop();
    if (outputbuffer) outputbuffer->Stop();
    {
        std::lock_guard<std::mutex> lk(stage_mu_);
        stage_cv_.notify_all();
    }
    if (worker_.joinable()) worker_.join();
    if (writer_.joinable()) writer_.join();
    if (in_region_) {
        (void)sddc_ddc_unregister_host(ddc_, in_region_);
        in_region_ = nullptr;
    }
}

bool fft_mt_r2iq::IsOn(void) { return on(); }

// Worker: input ring -> GPU -> out_stage_[k % 2].  Writer: out_stage_ -> output ring, so
// the ring copy of batch k overlaps the GPU round trip of batch k + 1.
void fft_mt_r2iq::worker()
{
    // latched for the whole run, as impl.hpp:3-7
    const int d = mdecimation;
    const bool lsb = getSideband();
    if (sddc_ddc_set_decimation(ddc_, d) || sddc_ddc_set_sideband(ddc_, lsb) || sddc_ddc_reset(ddc_)) {
        fail("worker: configure");
        set_on(false);
        std::lock_guard<std::mutex> lk(stage_mu_);
        stage_cv_.notify_all();
        return;
    }
    int stage = 0;
    while (on()) {
        {
            std::unique_lock<std::mutex> lk(stage_mu_);
            stage_cv_.wait(lk, [&] { return stage_n_[stage] == 0 || !on(); });
        }
        if (!on()) break;
        const int16_t *blocks[kMaxBatch];
        blocks[0] = inputbuffer->getReadPtr();           // blocks while empty
        if (!on()) break;
        // Tune bin and rand of each block are read as the worker takes that block, as the
        // reference reads them once per block (impl.hpp:20, 40).  One GPU call runs one
        // (tunebin, rand) pair, so a block whose values differ from the batch head's starts
        // the next batch instead of joining this one.
        const int tb = mtunebin.load();
        const bool rnd = getRand();
        int n = 1;
        // take more blocks only if they are already queued (never wait for them); they stay
        // in the ring, read in place, until the GPU has copied them
        while (n < kMaxBatch && sddc_r2iq::queued_blocks(inputbuffer->getWriteCount(), wc_base_, consumed_) > (uint32_t)n) {
            if (mtunebin.load() != tb || getRand() != rnd) break;
            blocks[n] = inputbuffer->peekReadPtr(n);
            n++;
        }
        int rc = sddc_ddc_set_tunebin(ddc_, tb) || sddc_ddc_set_rand(ddc_, rnd) ||
                 sddc_ddc_process_blocks(ddc_, blocks, n, out_stage_[stage].data());
        if (rc && mode_ == Backend::autoselect && backend_.load() == SDDC_DDC_BACKEND_HIP) {
            fail("worker: process");
            rc = !switch_to_cpu(consumed_) || sddc_ddc_set_tunebin(ddc_, tb) || sddc_ddc_set_rand(ddc_, rnd) ||
                 sddc_ddc_process_blocks(ddc_, blocks, n, out_stage_[stage].data());
        }
        if (rc) {
            fail("worker: process");
            set_on(false);
            break;
        }
        if (!on()) break;                              // TurnOff reset the ring meanwhile
        for (int i = 0; i < n; i++) inputbuffer->ReadDone();
        consumed_ += (uint64_t)n;
        {
            std::lock_guard<std::mutex> lk(stage_mu_);
            stage_n_[stage] = n;
            stage_cv_.notify_all();
        }
        stage ^= 1;
    }
    std::lock_guard<std::mutex> lk(stage_mu_);
    stage_cv_.notify_all();
}

void fft_mt_r2iq::writer()
{
    const int d = mdecimation;
    const size_t per_blk = (size_t)8 * mfftdim[d] * 2;    // floats of IQ per input block
    const uint64_t mask = (1u << d) - 1;
    uint64_t seq = 0;
    float *pout = nullptr;
    int stage = 0;
    for (;;) {
        int n;
        {
            std::unique_lock<std::mutex> lk(stage_mu_);
            stage_cv_.wait(lk, [&] { return stage_n_[stage] > 0 || !on(); });
            n = stage_n_[stage];
        }
        if (n == 0) break;                               // stopped with nothing pending
        const float *src = out_stage_[stage].data();
        for (int i = 0; i < n; i++) {
            const uint64_t slot = seq & mask;
            if (slot == 0) pout = outputbuffer->getWritePtr();   // impl.hpp:111-114
            if (!on()) return;
            std::memcpy(pout + slot * per_blk, src + (size_t)i * per_blk, per_blk * sizeof(float));
            if (slot == mask) outputbuffer->WriteDone();          // impl.hpp:141-145
            seq++;
        }
        blocks_done_ += (uint64_t)n;
        {
            std::lock_guard<std::mutex> lk(stage_mu_);
            stage_n_[stage] = 0;
            stage_cv_.notify_all();
        }
        stage ^= 1;
    }
}
