"""C5 (1024-channel DDC, BASELINE.json configs[4]) at the bench size on a real MI355X.

The bench's C5 step is 256 blocks x all 1024 legal tune bins (tunebin = 4c) at d = 4
(SURVEY.md §8(d)).  Checks, all through the C ABI (sddc_ddc_process_channels_device):
  - full size, CF32: every one of the 1024 channels within 1e-5 (max-rel) of the
    single-channel kernel on the same 256-block stream (the size-independent property:
    a channel of the many-channel DDC IS the single-channel DDC at that tune bin);
  - full size, CS16: every channel bit-exact to saturate(rint(x * scale)) of its CF32 output;
  - small size: every 32nd channel (and the last) of a 1024-channel launch over 3 blocks
    within 1e-5 (max-rel) of the f64 oracle (oracle/ddc_oracle.c, which restates
    Core/fft_mt_r2iq_impl.hpp:76-138), CF32; CS16 within 1 LSB of the oracle.
The sharded 8-GPU form computes the same channels, 128 per rank (extio_sddc_amd/shard.py);
its rank-local launch is this launch restricted to [128 g, 128 g + 128), checked by
test_channel_shards_concatenate below.
"""
from __future__ import annotations

import numpy as np
import pytest

from extio_sddc_amd.synth import make_stream

pytestmark = pytest.mark.gpu

TOL = 1e-5
D = 4
NCH = 1024
TBS = [4 * c for c in range(NCH)]


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    return torch


@pytest.fixture(scope="module")
def ddc(torch_dev):
    from extio_sddc_amd import R2iq
    r = R2iq(gain=1.0, device=0)
    r.setDecimate(D)
    r.setSideband(False)
    r.updateRand(False)
    yield r
    r.close()


@pytest.fixture(scope="module")
def full_stream(torch_dev):
    torch = torch_dev
    nblk = 256
    g = torch.Generator(device="cuda").manual_seed(0x5DDC + 5)
    x = torch.randint(-32768, 32768, (4096 + nblk * 65536,), dtype=torch.int16, device="cuda", generator=g)
    x[:4096] = 0
    return nblk, x


def _cs16_ref(torch, y, scale):
    s = torch.tensor(scale, dtype=torch.float32, device=y.device)
    return torch.clamp(torch.round(y * s), -32768, 32767).to(torch.int16)


def test_c5_full_size_cf32_and_cs16(torch_dev, ddc, full_stream):
    torch = torch_dev
    from extio_sddc_amd import output_samples
    nblk, x = full_stream
    per = output_samples(D, nblk) * 2
    ddc.setOutputFormat("CF32")
    out = torch.full((NCH, per), float("nan"), dtype=torch.float32, device="cuda")
    ddc.process_channels_device(x, nblk, TBS, out)
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    single = torch.empty(per, dtype=torch.float32, device="cuda")
    errs = torch.empty(NCH, dtype=torch.float32, device="cuda")
    for c in range(NCH):
        ddc.setTuneBin(TBS[c])
        ddc.process_device(x, nblk, single)
        errs[c] = (out[c] - single).abs().max() / single.abs().max()
    worst = errs.max().item()
    assert worst <= TOL, f"channel {int(errs.argmax())}: {worst:.3e} vs the single-channel kernel"

    # CS16 of the same launch: bit-exact to the numpy/torch restatement of the output stage
    scale = 30000.0 / out.abs().max().item()
    ddc.setOutputFormat("CS16", scale)
    try:
        c16 = torch.full((NCH, per), -12345, dtype=torch.int16, device="cuda")
        ddc.process_channels_device(x, nblk, TBS, c16)
        torch.cuda.synchronize()
    finally:
        ddc.setOutputFormat("CF32")
    for c in range(0, NCH, 64):   # chunks of rows bound the temporary
        assert torch.equal(c16[c:c + 64], _cs16_ref(torch, out[c:c + 64], scale)), f"CS16 rows {c}..{c + 63}"
    assert c16.abs().max().item() > 20000
    del out, c16
    torch.cuda.empty_cache()


@pytest.mark.parametrize("fmt", ["CF32", "CS16"])
def test_c5_every_32nd_channel_vs_oracle(torch_dev, ddc, oracle, fmt):
    torch = torch_dev
    from extio_sddc_amd import output_samples
    nblk = 3
    x = make_stream(nblk, "mix")
    H = oracle.filter_bank(1.0)
    checked = list(range(0, NCH, 32)) + [NCH - 1]
    refs = {c: oracle.r2iq(x, nblk, D, TBS[c], H=H) for c in checked}
    per = output_samples(D, nblk) * 2
    d_in = torch.from_numpy(x).to("cuda")
    if fmt == "CF32":
        ddc.setOutputFormat("CF32")
        out = torch.full((NCH, per), float("nan"), dtype=torch.float32, device="cuda")
        ddc.process_channels_device(d_in, nblk, TBS, out)
        torch.cuda.synchronize()
        y = out.cpu().numpy()
        for c in checked:
            err = oracle.max_rel_err(y[c].view(np.complex64), refs[c])
            assert err <= TOL, f"channel {c} (tb {TBS[c]}): max-rel-err {err:.3e}"
        return
    scale = 30000.0 / max(float(np.max(np.abs(np.concatenate([r.real, r.imag])))) for r in refs.values())
    ddc.setOutputFormat("CS16", scale)
    try:
        out = torch.full((NCH, per), -12345, dtype=torch.int16, device="cuda")
        ddc.process_channels_device(d_in, nblk, TBS, out)
        torch.cuda.synchronize()
    finally:
        ddc.setOutputFormat("CF32")
    y = out.cpu().numpy()
    for c in checked:
        exact = np.stack([refs[c].real, refs[c].imag], 1) * scale
        assert np.max(np.abs(y[c].reshape(-1, 2) - np.rint(exact))) <= 1, f"channel {c}"


def test_channel_shards_concatenate(torch_dev, ddc, full_stream):
    """The 8-rank C5 split (shard.channel_shard): each rank's 128-channel launch equals the
    matching rows of the 1024-channel launch, bit for bit (same kernel, same chunking)."""
    torch = torch_dev
    from extio_sddc_amd import output_samples
    from extio_sddc_amd.shard import channel_shard
    nblk, x = full_stream
    nblk = 16
    per = output_samples(D, nblk) * 2
    ddc.setOutputFormat("CF32")
    whole = torch.empty((NCH, per), dtype=torch.float32, device="cuda")
    ddc.process_channels_device(x, nblk, TBS, whole)
    part = torch.empty((NCH, per), dtype=torch.float32, device="cuda")
    for rank in range(8):
        lo, hi = channel_shard(NCH, 8, rank)
        ddc.process_channels_device(x, nblk, TBS[lo:hi], part[lo:hi])
    torch.cuda.synchronize()
    assert torch.equal(whole, part)
