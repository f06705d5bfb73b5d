// r2iq_harness.cpp — drives the drop-in fft_mt_r2iq through its r2iqControlClass interface
// exactly as RadioHandler does (Init -> setDecimate/setSideband/updateRand/setFreqOffset ->
// TurnOn -> ring traffic -> TurnOff), with the standalone ring (include/sddc_compat).
// A producer thread writes int16 blocks read from a file into the input ring; the main
// thread collects the 32768-sample output blocks into a file.  Also probes the base-class
// byte layout of the private fields (randADC @44, sideband @45, Core/r2iq.h).
//
//   r2iq_harness IN.bin NBLK D TUNEBIN LSB RAND GAIN OUT.bin [CYCLES]
// OUT.bin "-" discards the IQ and reports the end-to-end input rate (PCIe + host copies
// included); IN.bin may hold fewer blocks than NBLK, it is then cycled.  CYCLES > 1 repeats
// TurnOn -> NBLK blocks -> TurnOff on the same object and rings (the Start/Stop cycling of
// unittest/stability_test.cpp:255-301); each cycle's IQ is appended to OUT.bin.
// Env R2IQ_SCHEDULE="K:TUNEBIN:RAND[,K:TUNEBIN:RAND...]" (first cycle): before writing input
// block K the producer waits until the class has processed blocks 0..K-1, then calls
// setFreqOffset(TUNEBIN/4096) and updateRand(RAND), so block K is the first to run with them
// (the reference reads both once per block, Core/fft_mt_r2iq_impl.hpp:20,40).
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "fft_mt_r2iq.h"

int main(int argc, char **argv)
{
    if (argc != 9 && argc != 10) {
        std::fprintf(stderr, "usage: %s IN.bin NBLK D TUNEBIN LSB RAND GAIN OUT.bin [CYCLES]\n", argv[0]);
        return 2;
    }
    const int cycles = argc == 10 ? std::atoi(argv[9]) : 1;
    const int nblk = std::atoi(argv[2]), d = std::atoi(argv[3]), tb = std::atoi(argv[4]);
    const bool lsb = std::atoi(argv[5]) != 0, rnd = std::atoi(argv[6]) != 0;
    const float gain = (float)std::atof(argv[7]);
    FILE *in = std::fopen(argv[1], "rb");
    if (!in) return 2;
    std::fseek(in, 0, SEEK_END);
    const long bytes = std::ftell(in);
    std::fseek(in, 0, SEEK_SET);
    const int have = (int)(bytes / (65536 * 2));
    if (have < 1) return 2;
    std::vector<int16_t> data((size_t)have * 65536);
    if (fread(data.data(), sizeof(int16_t), data.size(), in) != data.size()) return 2;
    std::fclose(in);
    const bool discard = std::strcmp(argv[8], "-") == 0;
    struct Change { int k, tb, rand; };
    std::vector<Change> sched;
    if (const char *e = std::getenv("R2IQ_SCHEDULE")) {
        for (const char *p = e; *p;) {
            Change c{};
            int used = 0;
            if (std::sscanf(p, "%d:%d:%d%n", &c.k, &c.tb, &c.rand, &used) != 3) {
                std::fprintf(stderr, "bad R2IQ_SCHEDULE at '%s'\n", p);
                return 2;
            }
            sched.push_back(c);
            p += used;
            if (*p == ',') p++;
        }
    }

    ringbuffer<int16_t> inbuf;           // 64 slots, like RadioHandlerClass::inputbuffer
    ringbuffer<float> outbuf;
    inbuf.setBlockSize(65536);
    outbuf.setBlockSize(32768 * 2 * sizeof(float));   // RadioHandler.cpp:166 (EXT_BLOCKLEN*2*sizeof(float))

    fft_mt_r2iq r;
    r2iqControlClass *base = &r;
    base->Init(gain, &inbuf, &outbuf);
    base->setDecimate(d);
    base->setSideband(lsb);
    base->updateRand(rnd);
    const unsigned char *raw = reinterpret_cast<const unsigned char *>(base);
    if (raw[44] != (unsigned char)rnd || raw[45] != (unsigned char)lsb) {
        std::fprintf(stderr, "ABI: randADC/sideband not at bytes 44/45\n");
        return 5;
    }
    const float fc = base->setFreqOffset((float)tb / 4096.0f);
    FILE *out = discard ? nullptr : std::fopen(argv[8], "wb");
    const int want = nblk >> d;
    int got = 0;
    for (int cyc = 0; cyc < cycles; cyc++) {
        base->TurnOn();
        if (!base->IsOn()) {
            std::fprintf(stderr, "TurnOn failed: %s\n", r.lastError());
            return 3;
        }
        std::thread producer([&] {
            for (int b = 0; b < nblk; b++) {
                for (const Change &c : sched) {
                    if (cyc != 0 || c.k != b) continue;
                    while (r.blocksProcessed() < (uint64_t)b && base->IsOn())
                        std::this_thread::sleep_for(std::chrono::microseconds(200));
                    base->setFreqOffset((float)c.tb / 4096.0f);
                    base->updateRand(c.rand != 0);
                }
                int16_t *p = inbuf.getWritePtr();
                if (!base->IsOn()) return;
                std::memcpy(p, data.data() + (size_t)(b % have) * 65536, 65536 * sizeof(int16_t));
                inbuf.WriteDone();
            }
        });
        got = 0;
        const auto t0 = std::chrono::steady_clock::now();
        for (; got < want; got++) {
            const float *p = outbuf.getReadPtr();
            if (!base->IsOn()) break;
            if (out) fwrite(p, sizeof(float), 65536, out);
            outbuf.ReadDone();
        }
        const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (discard)
            std::printf("end-to-end: %d blocks in %.3f s = %.1f input MS/s\n", nblk, secs,
                        nblk * 65536.0 / secs / 1e6);
        base->TurnOff();
        producer.join();
        std::printf("cycle %d: output blocks %d of %d, residual fc %g, gpu blocks %llu\n", cyc, got, want, fc,
                    (unsigned long long)r.blocksProcessed());
        if (got != want) break;
    }
    if (out) std::fclose(out);
    return got == want ? 0 : 4;
}
