"""Host-path ingest on the GPU (pytest -m gpu): the two-slot
pipelined host path, gathering blocks scattered in memory (ring slots), and direct DMA
from/to registered caller memory.  Every variant must equal the plain host path
bit-exactly, and the stream history must carry across chunks and calls (impl.hpp:32)."""
from __future__ import annotations

import numpy as np
import pytest

from extio_sddc_amd.synth import make_stream

pytestmark = pytest.mark.gpu
BLOCK = 65536


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch


def _ddc(d, tb=1024):
    from extio_sddc_amd import R2iq
    r = R2iq(gain=1.0)
    r.setDecimate(d)
    r.setTuneBin(tb)
    return r


def test_multi_chunk_calls_match_oracle(torch_dev, oracle):
    """100 blocks (4 pipeline chunks) in uneven calls == one call == the oracle."""
    d, nblk = 1, 100
    x = make_stream(nblk, "mix")
    with _ddc(d) as r:
        one = r.process(x[4096:])
        r.TurnOn()
        parts = [r.process(x[4096:4096 + 37 * BLOCK]), r.process(x[4096 + 37 * BLOCK:4096 + 38 * BLOCK]),
                 r.process(x[4096 + 38 * BLOCK:])]
    np.testing.assert_array_equal(one.view(np.uint32), np.concatenate(parts).view(np.uint32))
    ref = oracle.r2iq(x, nblk, d, 1024, H=oracle.filter_bank(1.0))
    assert oracle.max_rel_err(one, ref) <= 1e-5


def test_process_blocks_scattered(torch_dev):
    d, nblk = 0, 40
    x = make_stream(nblk, "uniform")
    blocks = [x[4096 + i * BLOCK:4096 + (i + 1) * BLOCK].copy() for i in range(nblk)]
    order = list(range(nblk))
    # scatter: each block in its own allocation, some adjacent pairs contiguous
    pool = np.empty((nblk + 8) * BLOCK, np.int16)
    views = []
    for i in order:
        pos = i + (i // 5)                  # holes every 5 blocks
        pool[pos * BLOCK:(pos + 1) * BLOCK] = blocks[i]
        views.append(pool[pos * BLOCK:(pos + 1) * BLOCK])
    with _ddc(d) as r:
        ref = r.process(x[4096:])
        r.TurnOn()
        y = r.process_blocks(views)
    np.testing.assert_array_equal(y.view(np.uint32), ref.view(np.uint32))


def test_registered_direct_dma(torch_dev):
    d, nblk = 2, 70
    x = make_stream(nblk, "mix")
    inp = np.ascontiguousarray(x[4096:])
    with _ddc(d) as r:
        ref = r.process(inp)
        out = np.empty((ref.size, 2), np.float32)
        r.register_host(inp)
        r.register_host(out)
        r.TurnOn()
        from extio_sddc_amd._lib import check
        check(r._L.sddc_ddc_process_host(r._h, inp.ctypes.data, nblk, out.ctypes.data))
        np.testing.assert_array_equal(out.view(np.complex64).reshape(-1).view(np.uint32), ref.view(np.uint32))
        # partial overlap with a registered region is refused; double unregister too
        from extio_sddc_amd import DDCError
        with pytest.raises(DDCError):
            r.register_host(inp[:BLOCK])
        r.unregister_host(inp)
        r.unregister_host(out)
        with pytest.raises(DDCError):
            r.unregister_host(out)
        r.TurnOn()
        y = r.process(inp)                  # staged again after unregistering
    np.testing.assert_array_equal(y.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("d,split", [(0, 3), (2, 40)])
def test_set_history_continues_stream_on_new_handle(torch_dev, d, split):
    """sddc_ddc_set_history (the drop-in's failover uses it): a fresh handle given the tail of
    block split-1 as history continues the stream bit-exactly, whether the first call is one
    chunk or spans several pipeline chunks; and a GPU handle continues a CPU handle's stream
    within the parity bar."""
    from extio_sddc_amd import DEVICE_CPU, R2iq
    nblk = split + 5
    x = make_stream(nblk, "mix")
    with _ddc(d) as r:
        whole = r.process(x[4096:])
    per = 32768 >> d
    with _ddc(d) as r2:
        r2.setHistory(x[split * BLOCK: split * BLOCK + 4096])
        tail = r2.process(x[4096 + split * BLOCK:])
    np.testing.assert_array_equal(tail.view(np.uint32), whole[split * per:].view(np.uint32))
    with R2iq(gain=1.0, device=DEVICE_CPU) as c:
        c.setDecimate(d)
        c.setTuneBin(1024)
        head = c.process(x[4096:4096 + split * BLOCK])
    with _ddc(d) as r3:
        r3.setHistory(x[split * BLOCK: split * BLOCK + 4096])
        rest = r3.process(x[4096 + split * BLOCK:])
    y = np.concatenate([head, rest])
    assert np.max(np.abs(y - whole)) / np.max(np.abs(whole)) <= 1e-5
