// radiohandler_harness.cpp — integration driver: the reference's UNCHANGED RadioHandlerClass
// (Core/RadioHandler.cpp) running the MI355X drop-in fft_mt_r2iq (include/fft_mt_r2iq.h).
//
// Built only where the reference tree exists, by `make -C oracle radiohandler` (outputs
// into oracle/_ref/, git-ignored).  Like the reference's own unit tests (core_test.cpp
// MockFx3Handler, benchmark_test.cpp fx3handler_benchmark) it fakes the USB producer:
// MockFx3 reports hardware model 0 (-> DummyRadio) and its StartStream thread copies
// int16 blocks from a file into the input ring.  The output callback appends the IQ
// to a file.
//
//   radiohandler_harness IN.bin NBLK SRATE_IDX TUNE_HZ RAND OUT.bin
//   radiohandler_harness --benchmark SECONDS [ADC_HZ [SRATE_LO SRATE_HI]]
//
// --benchmark follows the reference's own ThroughputBenchmark (unittest/benchmark_test.cpp):
// the producer fills every transfer with 16384 sin(2 pi i / 64) (:80-84), writes 100 warm-up
// transfers (:87-91), then feeds the input ring as fast as the ring accepts (:98-106; the
// ring's getWritePtr blocks while it is full, so the feed runs at the DDC's pace).  For each
// srate_idx the radio runs SECONDS (3 in the reference, :31) and the output rate is
// output samples / 1e6 / elapsed (:285-290), elapsed measured around Start .. Stop (:267-281).
// One JSON line per srate_idx on stdout.  The backend is the drop-in's (SDDC_DDC_BACKEND).
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "FX3Class.h"
#include "RadioHandler.h"

namespace {

struct MockFx3 : fx3class {
    std::vector<int16_t> data;
    int nblk = 0;
    std::thread producer;
    std::atomic<bool> run{false};

    bool Open() override { return true; }
    bool Control(FX3Command, uint8_t) override { return true; }
    bool Control(FX3Command, uint32_t) override { return true; }
    bool Control(FX3Command, uint64_t) override { return true; }
    bool SetArgument(uint16_t, uint16_t) override { return true; }
    bool GetHardwareInfo(uint32_t *d) override
    {
        *d = 0;   // model 0 -> DummyRadio (RadioHandler.cpp Init)
        return true;
    }
    bool ReadDebugTrace(uint8_t *, uint8_t) override { return false; }
    bool Enumerate(unsigned char &, char *) override { return true; }
    void StartStream(ringbuffer<int16_t> &input, int) override
    {
        input.setBlockSize(65536);
        run = true;
        producer = std::thread([this, &input] {
            for (int b = 0; b < nblk && run; b++) {
                int16_t *p = input.getWritePtr();
                if (!run) break;
                std::memcpy(p, data.data() + (size_t)b * 65536, 65536 * sizeof(int16_t));
                input.WriteDone();
            }
        });
    }
    void StopStream() override
    {
        run = false;
        if (producer.joinable()) producer.join();
    }
};

struct Sink {
    FILE *f = nullptr;
    std::atomic<int> blocks{0};
};

void on_iq(void *ctx, const float *buf, uint32_t len)
{
    auto *s = static_cast<Sink *>(ctx);
    fwrite(buf, sizeof(float), 2 * (size_t)len, s->f);
    s->blocks++;
}

// benchmark_test.cpp's fx3handler_benchmark: pattern, warm-up, free-running feed
struct BenchFx3 : MockFx3 {
    static constexpr int kWarmup = 100;
    std::atomic<long> nxfers{0};
    std::atomic<bool> started{false};
    std::chrono::steady_clock::time_point first_input;

    void StartStream(ringbuffer<int16_t> &input, int) override
    {
        input.setBlockSize(65536);
        run = true;
        nxfers = 0;
        started = false;
        producer = std::thread([this, &input] {
            std::vector<int16_t> pattern(65536);
            for (int i = 0; i < 65536; i++)
                pattern[i] = (int16_t)(16384 * std::sin(2.0 * M_PI * i / 64.0));
            for (int i = 0; i < kWarmup && run; i++) {
                int16_t *p = input.getWritePtr();
                std::memcpy(p, pattern.data(), pattern.size() * sizeof(int16_t));
                input.WriteDone();
            }
            first_input = std::chrono::steady_clock::now();
            started = true;
            while (run) {
                int16_t *p = input.getWritePtr();
                if (!run) break;
                std::memcpy(p, pattern.data(), pattern.size() * sizeof(int16_t));
                input.WriteDone();
                ++nxfers;
            }
        });
    }
};

struct Counter {
    std::atomic<uint64_t> calls{0}, samples{0};
};

void on_count(void *ctx, const float *, uint32_t len)
{
    auto *c = static_cast<Counter *>(ctx);
    c->calls++;
    c->samples += len;
}

int benchmark(double seconds, uint32_t adc_hz, int lo, int hi)
{
    using clk = std::chrono::steady_clock;
    BenchFx3 fx3;
    Counter cnt;
    adcnominalfreq = adc_hz;
    RadioHandlerClass radio;
    if (!radio.Init(&fx3, on_count, nullptr, &cnt)) return 3;
    radio.UpdateSampleRate(adc_hz);
    const char *be = std::getenv("SDDC_DDC_BACKEND");
    int rc = 0;
    for (int idx = lo; idx <= hi; idx++) {
        cnt.calls = 0;
        cnt.samples = 0;
        int d = (adc_hz > N2_BANDSWITCH ? 5 : 4) - idx;   // RadioHandler.cpp:152-154
        if (d < 0) d = 0;
        const auto t0 = clk::now();
        radio.Start(idx);
        while (!fx3.started) std::this_thread::sleep_for(std::chrono::milliseconds(1));
        std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
        const long fed = fx3.nxfers.load();
        const auto t_in = clk::now();
        radio.Stop();
        const auto t1 = clk::now();
        const double el = std::chrono::duration<double>(t1 - t0).count();
        const double el_in = std::chrono::duration<double>(t_in - fx3.first_input).count();
        const double out_msps = cnt.samples / 1e6 / el;
        const double expected = (adc_hz / 2.0) / (double)(1 << d);
        std::printf("{\"srate_idx\": %d, \"decimate\": %d, \"backend\": \"%s\", \"seconds\": %.3f, "
                    "\"callbacks\": %llu, \"output_samples\": %llu, \"output_msps\": %.2f, "
                    "\"realtime_pct\": %.1f, \"input_transfers\": %ld, \"input_msps\": %.1f}\n",
                    idx, d, be ? be : "hip", el, (unsigned long long)cnt.calls.load(),
                    (unsigned long long)cnt.samples.load(), out_msps, 100.0 * cnt.samples / (expected * el), fed,
                    fed * 65536.0 / 1e6 / el_in);
        std::fflush(stdout);
        if (cnt.calls == 0) rc = 4;   // benchmark_test.cpp:383-386
        std::this_thread::sleep_for(std::chrono::milliseconds(100));
    }
    return rc;
}

}  // namespace

int main(int argc, char **argv)
{
    if (argc >= 3 && !std::strcmp(argv[1], "--benchmark"))
        return benchmark(std::atof(argv[2]), argc > 3 ? (uint32_t)std::strtoul(argv[3], nullptr, 10) : 64000000u,
                         argc > 5 ? std::atoi(argv[4]) : 0, argc > 5 ? std::atoi(argv[5]) : 4);
    if (argc != 7) {
        std::fprintf(stderr, "usage: %s IN.bin NBLK SRATE_IDX TUNE_HZ RAND OUT.bin\n", argv[0]);
        return 2;
    }
    MockFx3 fx3;
    fx3.nblk = std::atoi(argv[2]);
    const int srate_idx = std::atoi(argv[3]);
    const uint64_t tune = std::strtoull(argv[4], nullptr, 10);
    const bool rnd = std::atoi(argv[5]) != 0;
    fx3.data.resize((size_t)fx3.nblk * 65536);
    FILE *in = std::fopen(argv[1], "rb");
    if (!in || fread(fx3.data.data(), sizeof(int16_t), fx3.data.size(), in) != fx3.data.size()) {
        std::fprintf(stderr, "cannot read %d blocks from %s\n", fx3.nblk, argv[1]);
        return 2;
    }
    std::fclose(in);
    Sink sink;
    sink.f = std::fopen(argv[6], "wb");
    if (!sink.f) return 2;

    RadioHandlerClass radio;
    if (!radio.Init(&fx3, on_iq, nullptr, &sink)) return 3;   // nullptr -> new fft_mt_r2iq()
    const int d = 4 - srate_idx;                                // RadioHandler.cpp:152
    radio.TuneLO(tune);       // DummyRadio LO = 0 below 32 MHz -> setFreqOffset(tune / 32 MHz)
    radio.UptRand(rnd);
    radio.Start(srate_idx);
    const int want = fx3.nblk >> d;
    for (int ms = 0; ms < 60000 && sink.blocks < want; ms += 10)
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
    radio.Stop();
    std::fclose(sink.f);
    std::printf("output blocks %d of %d\n", sink.blocks.load(), want);
    return sink.blocks >= want ? 0 : 4;
}
