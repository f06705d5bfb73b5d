// fft_mt_r2iq.cpp — the drop-in r2iq class (include/fft_mt_r2iq.h) over the C ABI.
//
// Replaces Core/fft_mt_r2iq.cpp + fft_mt_r2iq_{def,avx,avx2,avx512,neon}.cpp +
// fft_mt_r2iq_impl.hpp.  The worker keeps the reference's ring protocol
// (impl.hpp:15-152): one getReadPtr/ReadDone per input block, getWritePtr when the
// output slot position (seq & (2^d-1)) is 0, WriteDone when it is 2^d-1.  The DSP
// itself (convert, r2c, shift x filter, inverse, overlap-discard) is one GPU call per
// batch of queued blocks through sddc_ddc_process_host().
#include "fft_mt_r2iq.h"

#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>

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
    in_stage_.assign((size_t)kMaxBatch * kBlock, 0);
    out_stage_.assign((size_t)kMaxBatch * 8 * halfFft * 2, 0.f);
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
    wc_base_ = inputbuffer->getWriteCount();
    consumed_ = 0;
    worker_ = std::thread([this] { worker(); });
}

void fft_mt_r2iq::TurnOff(void)
{
    r2iqOn = false;
    if (inputbuffer) inputbuffer->Stop();
    if (outputbuffer) outputbuffer->Stop();
    if (worker_.joinable()) worker_.join();
}

bool fft_mt_r2iq::IsOn(void) { return r2iqOn; }

void fft_mt_r2iq::worker()
{
    // latched for the whole run, as impl.hpp:3-7
    const int d = mdecimation;
    const bool lsb = getSideband();
    const int mfft = mfftdim[d];
    const size_t per_blk = (size_t)8 * mfft * 2;        // floats of IQ per input block
    const uint64_t mask = (1u << d) - 1;
    if (sddc_ddc_set_decimation(ddc_, d) || sddc_ddc_set_sideband(ddc_, lsb) || sddc_ddc_reset(ddc_)) {
        fail("worker: configure");
        r2iqOn = false;
        return;
    }
    uint64_t seq = 0;
    float *pout = nullptr;
    while (r2iqOn) {
        const int tb = mtunebin.load();                  // per block, impl.hpp:20
        const bool rnd = getRand();                      // per block, impl.hpp:40
        const int16_t *blk = inputbuffer->getReadPtr();  // blocks while empty
        if (!r2iqOn) break;
        std::memcpy(in_stage_.data(), blk, kBlock * sizeof(int16_t));
        inputbuffer->ReadDone();
        consumed_++;
        int n = 1;
        // take more blocks only if they are already queued (never wait for them)
        while (n < kMaxBatch && (uint64_t)(inputbuffer->getWriteCount() - wc_base_) > consumed_) {
            blk = inputbuffer->getReadPtr();
            if (!r2iqOn) break;
            std::memcpy(in_stage_.data() + (size_t)n * kBlock, blk, kBlock * sizeof(int16_t));
            inputbuffer->ReadDone();
            consumed_++;
            n++;
        }
        if (!r2iqOn) break;
        if (sddc_ddc_set_tunebin(ddc_, tb) || sddc_ddc_set_rand(ddc_, rnd) ||
            sddc_ddc_process_host(ddc_, in_stage_.data(), n, out_stage_.data())) {
            fail("worker: process");
            r2iqOn = false;
            break;
        }
        for (int i = 0; i < n; i++) {
            const uint64_t slot = seq & mask;
            if (slot == 0) pout = outputbuffer->getWritePtr();   // impl.hpp:111-114
            if (!r2iqOn) return;
            std::memcpy(pout + slot * per_blk, out_stage_.data() + (size_t)i * per_blk, per_blk * sizeof(float));
            if (slot == mask) outputbuffer->WriteDone();          // impl.hpp:141-145
            seq++;
        }
        blocks_done_ += (uint64_t)n;
    }
}
