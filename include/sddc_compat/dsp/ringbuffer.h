/*
 * sddc_compat/dsp/ringbuffer.h — standalone stand-in for ExtIO_sddc's block ring
 * (Core/dsp/ringbuffer.h), used ONLY when building without the ExtIO_sddc tree.
 * Same public API and blocking semantics: a fixed number of equally sized slots, one
 * producer and one consumer; getReadPtr() blocks while empty, getWritePtr() while full;
 * Stop() releases both sides; peekReadPtr(-1) is the slot read last.
 * The integration build uses the reference's own header instead.
 */
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <vector>

class ringbufferbase {
public:
    explicit ringbufferbase(int count) : slots(count) {}

    int getFullCount() const { return full_waits; }
    int getEmptyCount() const { return empty_waits; }
    int getWriteCount() const { return writes; }

    void ReadDone()
    {
        std::lock_guard<std::mutex> lk(mu);
        rd = (rd + 1) % slots;
        cv.notify_all();
    }
    void WriteDone()
    {
        std::lock_guard<std::mutex> lk(mu);
        wr = (wr + 1) % slots;
        writes++;
        cv.notify_all();
    }
    void Start()
    {
        std::lock_guard<std::mutex> lk(mu);
        rd = wr = 0;
        stopped = false;
    }
    void Stop()
    {
        std::lock_guard<std::mutex> lk(mu);
        rd = 0;
        wr = slots / 2;     /* neither empty nor full: blocked callers return */
        stopped = true;
        cv.notify_all();
    }

protected:
    void WaitUntilNotEmpty()
    {
        std::unique_lock<std::mutex> lk(mu);
        if (stopped || rd != wr) return;
        empty_waits++;
        cv.wait(lk, [this] { return stopped || rd != wr; });
    }
    void WaitUntilNotFull()
    {
        std::unique_lock<std::mutex> lk(mu);
        if (stopped || (wr + 1) % slots != rd) return;
        full_waits++;
        cv.wait(lk, [this] { return stopped || (wr + 1) % slots != rd; });
    }

    int slots;
    // read without the lock by peekReadPtr/peekWritePtr and the counters' getters: atomics
    std::atomic<int> rd{0}, wr{0};

private:
    std::atomic<int> empty_waits{0}, full_waits{0}, writes{0};
    bool stopped = false;
    std::mutex mu;
    std::condition_variable cv;
};

template <typename T>
class ringbuffer : public ringbufferbase {
public:
    explicit ringbuffer(int count = 64) : ringbufferbase(count), ptrs(count, nullptr) {}

    void setBlockSize(int size)
    {
        if (size == block) return;
        block = size;
        const int stride = (size + 7) & ~7;
        storage.assign((size_t)slots * stride, T());
        for (int i = 0; i < slots; i++) ptrs[i] = storage.data() + (size_t)i * stride;
    }
    int getBlockSize() const { return block; }

    T *peekWritePtr(int offset) { return ptrs[(wr + slots + offset) % slots]; }
    T *peekReadPtr(int offset) { return ptrs[(rd + slots + offset) % slots]; }
    T *getWritePtr()
    {
        WaitUntilNotFull();
        return ptrs[wr % slots];
    }
    const T *getReadPtr()
    {
        WaitUntilNotEmpty();
        return ptrs[rd];
    }

private:
    int block = 0;
    std::vector<T> storage;
    std::vector<T *> ptrs;
};
