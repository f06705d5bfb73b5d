// batching.h — the drop-in worker's count of input blocks it may take without waiting.
#pragma once

#include <cstdint>

namespace sddc_r2iq {

// Blocks written into the input ring since TurnOn and not yet taken by the worker.
// write_count is the ring's int writeCount (Core/dsp/ringbuffer.h: incremented once per
// WriteDone, never reset); write_count_at_turnon its value at TurnOn; consumed the blocks the
// worker has taken since.  Counted modulo 2^32: writeCount may wrap past INT_MAX (2^31 blocks
// = 12.7 days at 128 MS/s), and unsigned differences stay exact across the wrap.
inline uint32_t queued_blocks(int write_count, int write_count_at_turnon, uint64_t consumed)
{
    return (uint32_t)write_count - (uint32_t)write_count_at_turnon - (uint32_t)consumed;
}

}  // namespace sddc_r2iq
