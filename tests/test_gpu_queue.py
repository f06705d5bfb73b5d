"""The headline-size frame schedules against the oracle (pytest -m gpu).

A launch has frames = 11 * nblk against CUs x 4 = 1024 resident workgroups.  Since round 4 both
single-channel kernels split a full-residency launch's frames statically, each workgroup a
contiguous range sized by its CU slot's speed (ddc_queue.hpp slot_split), and the FS kernel can
still hand out the rest of its frames from the device-scope queue (SDDC_DDC_PARAM_FS_STATIC_PCT
< 100: tickets, shard hops, the dry-shard scan).  The small-batch parity tests
(test_gpu_parity.py, 1-5 blocks) never reach either: there every workgroup has one frame.
Here the launches are 256 and 2048 blocks (the BASELINE C2 batch) into NaN-filled outputs, and
the HIP output is compared with the f64 oracle (fft_mt_r2iq_impl.hpp:84-138):
  - every block of the 256-block launches and of the 2048-block d = 0 launch (the headline);
  - at 2048 blocks for d = 1, 2, 4: 2-block windows at the first, middle and last frame of each
    of 8 equal stretches of the stream, the last block and random blocks, each window fed its
    real 4096-sample history from the stream;
  - every schedule computes each frame the same way, so the queue-fed FS launches (static share
    0 % and 40 %) and the equal split must match the default bit for bit.
Plus the queue ring's reuse across streams (more than kQueueSlots = 64 launches over three
streams, one of them backed up) and a table rebuild on one stream read by a launch on another.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 1e-5
BLOCK = 65536
HIST = 4096
FRAMES = 11


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch


@pytest.fixture(scope="module")
def ddc(torch_dev):
    from extio_sddc_amd import R2iq
    r = R2iq(gain=1.0, device=0)
    yield r
    r.close()


@pytest.fixture(scope="module")
def H(oracle):
    return oracle.filter_bank(1.0)


def device_stream(torch, nblk, seed):
    """[4096 zero history | nblk blocks] int16 on the GPU: two tones (one strong) + Gaussian noise,
    the synth 'mix' recipe evaluated on the device (phases in float64)."""
    n = nblk * BLOCK
    g = torch.Generator(device="cuda").manual_seed(seed)
    t = torch.arange(n, dtype=torch.float64, device="cuda")
    x = 9000 * torch.sin(2 * np.pi * torch.frac(0.0713 * t)) + 3000 * torch.sin(2 * np.pi * torch.frac(0.191 * t))
    x += 300 * torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
    del t
    x = torch.clamp(torch.round(x), -32768, 32767).to(torch.int16)
    return torch.cat([torch.zeros(HIST, dtype=torch.int16, device="cuda"), x])


def run(torch, ddc, d_in, nblk, d, tb, stream=None, lsb=0, rand=0):
    from extio_sddc_amd import output_samples
    ddc.setDecimate(d)
    ddc.setTuneBin(tb)
    ddc.setSideband(bool(lsb))
    ddc.updateRand(bool(rand))
    d_out = torch.full((output_samples(d, nblk) * 2,), float("nan"), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ddc.process_device(d_in, nblk, d_out, stream=stream)
    torch.cuda.synchronize()
    return d_out


def shard_windows(nblk, extra_seed):
    """Start blocks of 2-block windows: each of the 8 queue shards' first, middle and last frame
    (ddc_queue.hpp fs_shard_lo), the last block, and four random blocks."""
    nframes = FRAMES * nblk
    starts = set()
    for s in range(8):
        lo, hi = (nframes * s) >> 3, (nframes * (s + 1)) >> 3
        for f in (lo, (lo + hi) // 2, hi - 1):
            starts.add(min(max(f // FRAMES, 0), nblk - 2))
    starts.add(nblk - 2)
    rng = np.random.default_rng(extra_seed)
    starts.update(int(b) for b in rng.integers(0, nblk - 1, 4))
    return sorted(starts)


# CU-slot weights of the slot-weighted split (ddc_kernels.h kFsSlotWeights / kSlotWeights)
SLOT_WEIGHTS = {0: (31, 26, 18, 13), 1: (31, 26, 18, 13), 2: (31, 26, 18, 13), 3: (29, 25, 20, 15),
                4: (29, 25, 20, 15), 5: (29, 25, 20, 15), 6: (29, 25, 20, 15)}


def quarter_windows(nblk, d):
    """Start blocks of 2-block windows at the first, middle and last frame of each workgroup
    quarter's share of a full-residency launch (ddc_queue.hpp slot_split: quarter q takes the
    frames [ns W_q / W, ns W_{q+1} / W) with W_q the cumulative slot weight)."""
    nframes = FRAMES * nblk
    w = np.cumsum((0,) + SLOT_WEIGHTS[d])
    starts = set()
    for q in range(4):
        lo, hi = nframes * w[q] // w[4], nframes * w[q + 1] // w[4]
        for f in (lo, (lo + hi) // 2, hi - 1):
            starts.add(min(max(f // FRAMES - (1 if f % FRAMES == 0 else 0), 0), nblk - 2))
    return sorted(starts)


def check_windows(oracle, H, x, y, nblk, d, tb, starts, lsb=0, rand=0):
    per = 32768 >> d
    worst = 0.0
    for b in starts:
        seg = x[BLOCK * b: HIST + BLOCK * (b + 2)]   # the window's real history + 2 blocks
        r = oracle.r2iq(seg, 2, d, tb, lsb, rand, H=H)
        yw = y[b * per:(b + 2) * per]
        err = oracle.max_rel_err(yw, r)
        worst = max(worst, err)
        assert err <= TOL, f"d={d} window at block {b}: max-rel-err {err:.3e}"
    return worst


@pytest.mark.parametrize("d", [0, 1, 2, 4])
def test_queue_path_every_block_256(torch_dev, ddc, oracle, H, d):
    """256 blocks = 2816 frames: every workgroup takes tickets.  Every output sample vs oracle."""
    torch = torch_dev
    nblk, tb = 256, 1024
    d_in = device_stream(torch, nblk, 0x5DDC + d)
    y = run(torch, ddc, d_in, nblk, d, tb).cpu().numpy().view(np.complex64)
    assert np.all(np.isfinite(y)), f"{np.count_nonzero(~np.isfinite(y))} samples never written"
    x = d_in.cpu().numpy()
    r = oracle.r2iq(x, nblk, d, tb, H=H)
    err = oracle.max_rel_err(y, r)
    assert err <= TOL, f"max-rel-err {err:.3e}"


def test_queue_path_headline_every_block(torch_dev, ddc, oracle, H):
    """The headline launch itself (C2: d = 0, tb 1024, 2048 blocks, 22528 frames in one
    launch): every frame written, every output sample within 1e-5 of the f64 oracle."""
    torch = torch_dev
    nblk, d, tb = 2048, 0, 1024
    d_in = device_stream(torch, nblk, 0x5DDC)
    d_out = run(torch, ddc, d_in, nblk, d, tb)
    assert bool(torch.isfinite(d_out).all()), "frames left unwritten"
    y = d_out.cpu().numpy().view(np.complex64)
    del d_out
    x = d_in.cpu().numpy()
    del d_in
    # the oracle in 256-block pieces, each with its real history (bounded host memory)
    step = 256
    per = 32768 >> d
    num = den = 0.0
    for b0 in range(0, nblk, step):
        r = oracle.r2iq(x[BLOCK * b0: HIST + BLOCK * (b0 + step)], step, d, tb, H=H)
        yw = y[b0 * per:(b0 + step) * per]
        num = max(num, float(np.max(np.abs(yw - r))))
        den = max(den, float(np.max(np.abs(r))))
    assert num / den <= TOL, f"max-rel-err {num / den:.3e}"


@pytest.mark.parametrize("d,lsb,rand", [(1, 0, 0), (2, 0, 0), (4, 0, 0),
                                        (1, 1, 1),   # C4: decim 4, sideband inversion + rand (RAND/LSB instances)
                                        (3, 0, 0),   # C3 decim 16
                                        (5, 0, 0), (6, 0, 0),
                                        (0, 1, 1)])  # the FS kernel's RAND/LSB instance
def test_headline_size_windows_2048(torch_dev, ddc, oracle, H, d, lsb, rand):
    """2048-block launches (every workgroup carries ~22 frames: input prefetch, LDS reuse across
    frames, the slot-weighted ranges) into NaN-filled outputs: 2-block windows at the first,
    middle and last frame of every workgroup quarter's share and of 8 equal stretches, the last
    block and random blocks, each with its real history, against the f64 oracle at 1e-5
    (fft_mt_r2iq_impl.hpp:76-138)."""
    torch = torch_dev
    nblk, tb = 2048, 1024
    d_in = device_stream(torch, nblk, 0x5DDC + 16 * d + 4 * lsb + 2 * rand)
    d_out = run(torch, ddc, d_in, nblk, d, tb, lsb=lsb, rand=rand)
    assert bool(torch.isfinite(d_out).all()), "frames left unwritten"
    y = d_out.cpu().numpy().view(np.complex64)
    del d_out
    x = d_in.cpu().numpy()
    del d_in
    starts = sorted(set(shard_windows(nblk, d)) | set(quarter_windows(nblk, d)))
    check_windows(oracle, H, x, y, nblk, d, tb, starts, lsb, rand)


@pytest.mark.parametrize("d,sched", [(0, 1), (0, 2), (0, 0), (1, 0)])
def test_queue_ring_reuse_across_streams(torch_dev, d, sched):
    """More launches than queue slots (72 > 64), round-robin over three streams, the first one
    backed up behind a 2048-block launch, each into its own NaN-filled output: every output
    equals the same launch run alone on one stream, bit for bit (no frame dropped or doubled).
    sched: the FS kernel's schedule (1 the queue and 2 work stealing take a ring slot per launch;
    0, the default static split, and the persistent kernel at d = 1 take none)."""
    torch = torch_dev
    from extio_sddc_amd import R2iq, output_samples
    ddc = R2iq(gain=1.0, device=0)
    _set_param(ddc, P_FS_SCHEDULE, sched)
    if sched == 1:
        _set_param(ddc, P_FS_STATIC_PCT, 40)
    nblk, nlaunch, noff = 48, 72, 8
    d_in = device_stream(torch, 2048, 0x5DDC + 100 + d)
    ddc.setDecimate(d)
    ddc.setTuneBin(1024)
    ddc.setSideband(False)
    ddc.updateRand(False)
    n = output_samples(d, nblk) * 2
    refs = []
    for o in range(noff):
        out = torch.full((n,), float("nan"), dtype=torch.float32, device="cuda")
        ddc.process_device(d_in[o * 3 * BLOCK:], nblk, out)
        refs.append(out)
    big = torch.empty(output_samples(d, 2048) * 2, dtype=torch.float32, device="cuda")
    outs = [torch.full((n,), float("nan"), dtype=torch.float32, device="cuda") for _ in range(nlaunch)]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in range(3)]
    ddc.process_device(d_in, 2048, big, stream=streams[0])   # stream 0 backs up
    for i in range(nlaunch):
        o = i % noff
        ddc.process_device(d_in[o * 3 * BLOCK:], nblk, outs[i], stream=streams[i % 3])
    torch.cuda.synchronize()
    for i in range(nlaunch):
        assert bool(torch.isfinite(outs[i]).all()), f"launch {i}: frames left unwritten"
        assert torch.equal(outs[i], refs[i % noff]), f"launch {i} differs from the single-stream run"
    # and the handle still works on its default stream afterwards
    again = torch.full((n,), float("nan"), dtype=torch.float32, device="cuda")
    ddc.process_device(d_in, nblk, again)
    torch.cuda.synchronize()
    assert torch.equal(again, refs[0])
    ddc.close()


@pytest.mark.parametrize("d,tb0,tb1", [(0, 1024, 2048), (1, 1024, 2048)])
def test_table_rebuild_seen_by_other_stream(torch_dev, ddc, oracle, H, d, tb0, tb1):
    """The per-tunebin tables are rebuilt on stream A behind a long launch; a launch on stream B
    with the same tune bin (no rebuild of its own) must wait for that rebuild, not read the old
    tables (ddc_runtime.cpp order_after_build)."""
    torch = torch_dev
    from extio_sddc_amd import output_samples
    nblk = 4
    d_in = device_stream(torch, 2048, 0x5DDC + 200 + d)
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    ddc.setDecimate(d)
    ddc.setSideband(False)
    ddc.updateRand(False)
    ddc.setTuneBin(tb0)
    n = output_samples(d, nblk) * 2
    big = torch.empty(output_samples(d, 2048) * 2, dtype=torch.float32, device="cuda")
    ya = torch.full((n,), float("nan"), dtype=torch.float32, device="cuda")
    yb = torch.full((n,), float("nan"), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ddc.process_device(d_in, 2048, big, stream=a)        # A busy, tables of tb0
    ddc.setTuneBin(tb1)
    ddc.process_device(d_in, nblk, ya, stream=a)         # rebuild for tb1, queued on A behind the long launch
    ddc.process_device(d_in, nblk, yb, stream=b)         # same tb1: no rebuild; must see A's
    torch.cuda.synchronize()
    x = d_in[:HIST + nblk * BLOCK].cpu().numpy()
    r = oracle.r2iq(x, nblk, d, tb1, H=H)
    for y in (ya, yb):
        yy = y.cpu().numpy().view(np.complex64)
        assert oracle.max_rel_err(yy, r) <= TOL
    assert torch.equal(ya, yb)


# sddc_ddc_internal.h SDDC_DDC_PARAM_*
P_FS_STATIC_PCT, P_SLOT_WEIGHTS, P_FS_FRAMES_PER_WG, P_FS_SCHEDULE, P_FS_MINREM, P_FS_PUBLIC, P_FS_ZERO_ROWS = \
    1, 2, 3, 4, 5, 6, 7


def _set_param(r, param, value):
    import ctypes
    from extio_sddc_amd import _lib
    f = r._L.sddc_ddc_internal_set_param
    f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    f.restype = ctypes.c_int
    _lib.check(f(r._h, param, value))


SCHEDULES = {
    # d = 0 (FS kernel): the static split (default), the queue at static shares 100 / 40 / 0 %,
    # work stealing (every frame open / the last 4 of each range, steal threshold 2 / disabled),
    # the zero rows computed instead of skipped, and non-persistent grids (16 frames per
    # workgroup: 1408 workgroups, XCD-mapped ranges) with the static split and with work stealing
    # (the steal slots indexed by the mapped range, ddc_queue.hpp StealSchedule::self)
    0: [(), ((P_FS_SCHEDULE, 1), (P_FS_STATIC_PCT, 100)), ((P_FS_SCHEDULE, 1), (P_FS_STATIC_PCT, 40)),
        ((P_FS_SCHEDULE, 1), (P_FS_STATIC_PCT, 0)), ((P_FS_SCHEDULE, 2),),
        ((P_FS_SCHEDULE, 2), (P_FS_PUBLIC, 4), (P_FS_MINREM, 2)), ((P_FS_SCHEDULE, 2), (P_FS_MINREM, 0)),
        ((P_FS_ZERO_ROWS, 0),), ((P_FS_FRAMES_PER_WG, 16),),
        ((P_FS_SCHEDULE, 2), (P_FS_FRAMES_PER_WG, 16), (P_FS_MINREM, 2))],
    # persistent kernel: slot-weighted vs equal contiguous split
    1: [(), ((P_SLOT_WEIGHTS, 0),)],
    4: [(), ((P_SLOT_WEIGHTS, 0),)],
}


@pytest.mark.parametrize("d", [0, 1, 4])
def test_schedules_bit_identical(torch_dev, d):
    """Every schedule computes each frame the same way: the FS kernel's queue (static shares
    100 / 40 / 0 %), work stealing in its forms, the zero rows computed, and the equal split
    instead of the slot-weighted one, each against the default, 2048 blocks, NaN-filled"""
    torch = torch_dev
    from extio_sddc_amd import R2iq, output_samples
    nblk = 2048
    g = torch.Generator(device="cuda").manual_seed(0x5DDC + d)
    d_in = torch.randint(-32768, 32767, (HIST + nblk * BLOCK,), dtype=torch.int16, device="cuda", generator=g)
    outs = []
    for settings in SCHEDULES[d]:
        with R2iq(gain=1.0, device=0) as r:
            r.setDecimate(d)
            r.setTuneBin(1024)
            for param, v in settings:
                _set_param(r, param, v)
            out = torch.full((output_samples(d, nblk) * 2,), float("nan"), dtype=torch.float32, device="cuda")
            r.process_device(d_in, nblk, out)
            torch.cuda.synchronize()
            outs.append(out.view(torch.int32).cpu().numpy())
    assert not np.any(np.isnan(outs[0].view(np.float32))), "frames left unwritten"
    for o, settings in zip(outs[1:], SCHEDULES[d][1:]):
        assert not np.any(np.isnan(o.view(np.float32))), f"{settings}: frames left unwritten"
        np.testing.assert_array_equal(o, outs[0], err_msg=str(settings))


def fs_zero_rows(tb):
    """ddc_fs.hip fs_zero_rows: the whole zero rows of the d = 0 inverse input that the FS kernel
    skips for tune bin tb (> 0 at the top, < 0 at the bottom; a single zero row is computed)"""
    top = 16 - (tb + 2048 + 255) // 256
    bot = (tb - 2048) // 256 if tb > 2048 else 0
    z = top if top > 0 else -bot if bot > 0 else 0
    z = max(-8, min(8, z))
    return 0 if abs(z) == 1 else z


# d = 0 tune bins by the inverse input's whole zero rows (the reference's zero fill,
# impl.hpp:91-96): (tb, rows zero at the top (bins >= tb + 2048), rows zero at the bottom
# (bins < tb - 2048)).  The FS kernel is instantiated per count (ddc_fs.hip launch_fs_v: 2..8 at
# the top, 2..7 at the bottom for CF32 output without the NCO; 4 or none for the NCO / CS16
# outputs), so every count it can select has a tune bin here, most of them two.
ZERO_ROW_BINS = [(2048, 0, 0), (1792, 1, 0), (1536, 2, 0), (1284, 2, 0), (1028, 3, 0), (1024, 4, 0),
                 (768, 5, 0), (724, 5, 0), (512, 6, 0), (260, 6, 0), (256, 7, 0), (0, 8, 0),
                 (2304, 0, 1), (2560, 0, 2), (2812, 0, 2), (3068, 0, 3), (3072, 0, 4), (3328, 0, 5),
                 (3580, 0, 5), (3584, 0, 6), (3836, 0, 6), (3840, 0, 7), (4092, 0, 7)]


def _zero_rows_case(torch, oracle, H, tb, lsb=0, rand=0):
    """4 blocks of each source against the f64 oracle, then 64 blocks with the zero rows skipped
    against the same launch with them computed (NaN-filled outputs, bit-identical)"""
    from extio_sddc_amd import R2iq, output_samples
    from extio_sddc_amd.synth import make_stream

    def launch(r, d_in, nblk):
        r.setDecimate(0)
        r.setTuneBin(tb)
        r.setSideband(bool(lsb))
        r.updateRand(bool(rand))
        out = torch.full((output_samples(0, nblk) * 2,), float("nan"), dtype=torch.float32, device="cuda")
        r.process_device(d_in, nblk, out)
        torch.cuda.synchronize()
        return out.cpu().numpy()

    for src in ("mix", "oob"):
        x = make_stream(4, src)
        with R2iq(gain=1.0, device=0) as r:
            y = launch(r, torch.from_numpy(x).to("cuda"), 4).view(np.complex64)
        err = oracle.max_rel_err(y, oracle.r2iq(x, 4, 0, tb, lsb, rand, H=H))
        assert err <= TOL, f"{src}: max-rel-err {err:.3e}"
    nblk = 64
    d_in = device_stream(torch, nblk, 0x5DDC + tb)
    outs = []
    for zr in (1, 0):
        with R2iq(gain=1.0, device=0) as r:
            _set_param(r, P_FS_ZERO_ROWS, zr)
            outs.append(launch(r, d_in, nblk))
    assert np.all(np.isfinite(outs[0]))
    np.testing.assert_array_equal(outs[0], outs[1])


@pytest.mark.parametrize("tb,ztop,zbot", ZERO_ROW_BINS)
def test_fs_zero_rows(torch_dev, oracle, H, tb, ztop, zbot):
    """The zero-row skip at tune bins giving 0 to 8 zero rows at the top and 0 to 7 at the bottom
    (every instance the plain CF32 output can select): within 1e-5 of the f64 oracle (4 blocks,
    strong out-of-band + weak in-band tone and a mix), and equal to the same launch with the zero
    rows computed (64 blocks, NaN-filled)"""
    assert (2048 - tb) // 256 == ztop if tb <= 2048 else (tb - 2048) // 256 == zbot
    _zero_rows_case(torch_dev, oracle, H, tb)


# the RAND and LSB instances at every count they are built for (ddc_fs.hip launch_fs_v: the same
# counts as the plain output), each count once, both options on; ZR = 4 (tb = 1024) is in the
# C4-style cases of test_gpu_parity.py too
ZERO_ROW_BINS_RL = [(1536, 2), (1028, 3), (1024, 4), (768, 5), (512, 6), (256, 7), (0, 8),
                    (2560, -2), (3068, -3), (3072, -4), (3328, -5), (3584, -6), (3840, -7)]


@pytest.mark.parametrize("tb,zr", ZERO_ROW_BINS_RL)
def test_fs_zero_rows_rand_lsb(torch_dev, oracle, H, tb, zr):
    """The RAND + LSB kernel instances of every zero-row count: 1e-5 vs the f64 oracle with
    de-randomisation and sideband inversion on, and skip on = skip off bit for bit"""
    assert fs_zero_rows(tb) == zr
    _zero_rows_case(torch_dev, oracle, H, tb, lsb=1, rand=1)


def test_fs_zero_row_counts_covered():
    """CPU-side: the tune-bin lists reach every zero-row count launch_fs_v instantiates"""
    counts = {fs_zero_rows(tb) for tb, _, _ in ZERO_ROW_BINS}
    assert counts >= {0, 2, 3, 4, 5, 6, 7, 8, -2, -3, -4, -5, -6, -7}
    assert {zr for _, zr in ZERO_ROW_BINS_RL} == {2, 3, 4, 5, 6, 7, 8, -2, -3, -4, -5, -6, -7}
    assert all(fs_zero_rows(tb) != -8 for tb in range(0, 4096, 4))   # ZR = -8 is never selected
