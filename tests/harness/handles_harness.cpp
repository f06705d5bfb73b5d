// handles_harness.cpp — several threads creating, using and destroying DDC handles at once, and
// sharing one more, through the C ABI (include/sddc_ddc.h).  Built with -fsanitize=thread (the
// HIP kernel objects with their host side instrumented too) by `make -C extio_sddc_amd/csrc
// sanitize`; run by tests/test_sanitizers.py on the CPU backend (DEVICE -1) and, on a GPU box, on
// device 0, where the launch path (launch geometry cache, queue-slot ring, table builds, stream
// hand-off) runs from every thread.  Each private handle's output must equal the reference computed
// serially before the threads start; the shared handle's calls only have to succeed (their
// settings race by design, serialised by the handle's lock).
//
//   handles_harness DEVICE THREADS ITERS
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "sddc_ddc.h"

namespace {

constexpr int kBlocks = 2;
constexpr int kDs = 3;   // d = 0, 1, 2 (d = 0 at tune bin 1024 takes the fused-split kernel)

int run(sddc_ddc_t *h, const std::vector<int16_t> &in, int d, std::vector<float> &out)
{
    if (sddc_ddc_set_decimation(h, d) || sddc_ddc_set_tunebin(h, 1024) || sddc_ddc_reset(h)) return -1;
    out.assign(2 * sddc_ddc_output_samples(d, kBlocks), 0.f);
    return sddc_ddc_process_host(h, in.data(), kBlocks, out.data());
}

}  // namespace

int main(int argc, char **argv)
{
    if (argc != 4) {
        std::fprintf(stderr, "usage: %s DEVICE THREADS ITERS\n", argv[0]);
        return 2;
    }
    const int dev = std::atoi(argv[1]), nthr = std::atoi(argv[2]), iters = std::atoi(argv[3]);
    std::vector<int16_t> in((size_t)kBlocks * 65536);
    uint32_t s = 0x5DDCu;
    for (auto &v : in) {
        s = s * 1664525u + 1013904223u;
        v = (int16_t)(s >> 16);
    }
    std::vector<std::vector<float>> ref(kDs);
    {
        sddc_ddc_t *h = nullptr;
        if (sddc_ddc_create(1.0f, dev, &h)) {
            std::fprintf(stderr, "create: %s\n", sddc_ddc_last_error());
            return 3;
        }
        for (int d = 0; d < kDs; d++)
            if (run(h, in, d, ref[d])) {
                std::fprintf(stderr, "reference d=%d: %s\n", d, sddc_ddc_last_error());
                return 3;
            }
        sddc_ddc_destroy(h);
    }
    sddc_ddc_t *shared = nullptr;
    if (sddc_ddc_create(1.0f, dev, &shared)) return 3;
    std::atomic<int> bad{0}, calls{0};
    std::vector<std::thread> th;
    for (int i = 0; i < nthr; i++)
        th.emplace_back([&, i] {
            for (int it = 0; it < iters; it++) {
                const int d = (i + it) % kDs;
                sddc_ddc_t *h = nullptr;
                std::vector<float> o;
                if (sddc_ddc_create(1.0f, dev, &h) || run(h, in, d, o) || o != ref[d]) {
                    std::fprintf(stderr, "thread %d iter %d d=%d: private handle failed or differs (%s)\n", i, it,
                                 d, sddc_ddc_last_error());
                    bad++;
                }
                if (h) sddc_ddc_destroy(h);
                // the shared handle: output sized for d = 0, the largest, whatever d the call sees
                std::vector<float> o2(2 * sddc_ddc_output_samples(0, kBlocks));
                if (sddc_ddc_set_decimation(shared, d) || sddc_ddc_process_host(shared, in.data(), kBlocks, o2.data())) {
                    std::fprintf(stderr, "thread %d iter %d: shared handle failed (%s)\n", i, it, sddc_ddc_last_error());
                    bad++;
                }
                calls += 2;
            }
        });
    for (auto &t : th) t.join();
    sddc_ddc_destroy(shared);
    std::printf("handles_harness device %d: %d threads x %d iterations, %d calls, %d failures\n", dev, nthr, iters,
                calls.load(), bad.load());
    return bad ? 1 : 0;
}
