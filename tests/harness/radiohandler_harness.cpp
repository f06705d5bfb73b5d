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
#include <atomic>
#include <chrono>
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

}  // namespace

int main(int argc, char **argv)
{
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
