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
static constexpr int kMaxBatch = 16;     // input blocks per GPU call (<= half the 32-transfer queue)

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
    if (ddc_) {
        sddc_ddc_destroy(ddc_);
        ddc_ = nullptr;
    }
    if (sddc_ddc_create(gain, device_, &ddc_) != SDDC_OK) {
        ddc_ = nullptr;
        fail("Init: sddc_ddc_create");
        return;
    }
    for (auto &st : out_stage_) {
        st.assign((size_t)kMaxBatch * 8 * halfFft * 2, 0.f);
        // pinned for direct D2H; on failure the library stages through its own buffers
        (void)sddc_ddc_register_host(ddc_, st.data(), st.size() * sizeof(float));
    }
}

void fft_mt_r2iq::TurnOn()
{
    if (!ddc_ || !inputbuffer || !outputbuffer) {
        last_error_ = "TurnOn without a successful Init";
        std::fprintf(stderr, "[fft_mt_r2iq] %s\n", last_error_.c_str());
        return;
    }
    r2iqOn = true;
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
    r2iqOn = false;
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

bool fft_mt_r2iq::IsOn(void) { return r2iqOn; }

// Worker: input ring -> GPU -> out_stage_[k % 2].  Writer: out_stage_ -> output ring, so
// the ring copy of batch k overlaps the GPU round trip of batch k + 1.
void fft_mt_r2iq::worker()
{
    // latched for the whole run, as impl.hpp:3-7
    const int d = mdecimation;
    const bool lsb = getSideband();
    if (sddc_ddc_set_decimation(ddc_, d) || sddc_ddc_set_sideband(ddc_, lsb) || sddc_ddc_reset(ddc_)) {
        fail("worker: configure");
        r2iqOn = false;
        std::lock_guard<std::mutex> lk(stage_mu_);
        stage_cv_.notify_all();
        return;
    }
    int stage = 0;
    while (r2iqOn) {
        {
            std::unique_lock<std::mutex> lk(stage_mu_);
            stage_cv_.wait(lk, [&] { return stage_n_[stage] == 0 || !r2iqOn; });
        }
        if (!r2iqOn) break;
        const int16_t *blocks[kMaxBatch];
        blocks[0] = inputbuffer->getReadPtr();           // blocks while empty
        if (!r2iqOn) break;
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
        if (sddc_ddc_set_tunebin(ddc_, tb) || sddc_ddc_set_rand(ddc_, rnd) ||
            sddc_ddc_process_blocks(ddc_, blocks, n, out_stage_[stage].data())) {
            fail("worker: process");
            r2iqOn = false;
            break;
        }
        if (!r2iqOn) break;                              // TurnOff reset the ring meanwhile
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
            stage_cv_.wait(lk, [&] { return stage_n_[stage] > 0 || !r2iqOn; });
            n = stage_n_[stage];
        }
        if (n == 0) break;                               // stopped with nothing pending
        const float *src = out_stage_[stage].data();
        for (int i = 0; i < n; i++) {
            const uint64_t slot = seq & mask;
            if (slot == 0) pout = outputbuffer->getWritePtr();   // impl.hpp:111-114
            if (!r2iqOn) return;
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
