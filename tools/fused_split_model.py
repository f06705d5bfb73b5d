"""Index model of the d >= 4 fused split measured in round 4 and not kept (the FUSE path of
profiles/r04/ab/fused_split_d4_6.patch; python -m pytest tools/fused_split_model.py): forward pass 2 on column
c = kFsPerm[lane], the band bin each lane owns and the register its quad partner sends for the
mirror, checked for every tune bin against the bins' plain definitions (the reference's split:
bin tb + m - (m >= N/2 ? N : 0) and its mirror 4096 - bin, Core/fft_mt_r2iq_impl.hpp:84-96)."""
import os
import re

import numpy as np
import pytest

HALF = 4096
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def fs_perm():
    txt = open(os.path.join(ROOT, "extio_sddc_amd", "csrc", "ddc_fs_perm.h")).read()
    body = txt[txt.index("{") + 1:txt.index("}")]
    return np.array([int(x) for x in re.findall(r"\d+", body)])


@pytest.mark.parametrize("d", [4, 5, 6])
def test_fused_split_indices(d):
    N = HALF >> d
    perm = fs_perm()
    assert sorted(perm) == list(range(256))
    lanes = np.arange(256)
    col = perm[lanes]
    partner = lanes ^ 1
    assert np.all((col[partner] == (256 - col) % 256) | (col == 0) | (col == 128))
    for tb in range(HALF):
        s0 = (tb - N // 2) % HALF
        r0 = s0 >> 8
        mrel = ((((1 - s0 - N) % HALF) >> 8) - r0) % 16
        fj = (col - s0) % 256
        valid = fj < N
        fm = np.where(fj < N // 2, fj + N // 2, fj - N // 2)
        fra = ((s0 % 256) + fj) >= 256
        fself = (col == 0) | (col == 128)
        frap = ((s0 % 256) + ((256 - col - s0) % 256)) >= 256
        fidx = (15 - 2 * r0 + (col == 0) - np.where(fself, fra, frap)) % 16
        # register r of lane l holds bin col[l] + 256 ((r + r0) mod 16)
        band = (col + 256 * ((r0 + fra) % 16)) % HALF
        # the band bin is the reference's bin of inverse input fm
        ref_bin = (tb + fm - np.where(fm >= N // 2, N, 0)) % HALF
        assert np.all(band[valid] == ref_bin[valid]), tb
        assert sorted(fm[valid]) == list(range(N)), tb
        # what lane l receives: its partner's (or its own) register fidx of that lane
        src = np.where(fself, lanes, partner)
        got = (col[src] + 256 * ((fidx[src] + r0) % 16)) % HALF
        assert np.all(got[valid] == (HALF - band[valid]) % HALF), tb
        # ... and that register is one the pruned pass 2 computes (groups 0, 1, mrel, mrel + 1)
        groups = {0, 1, mrel % 4, (mrel + 1) % 4}
        assert all((int(fidx[s]) % 4) in groups for s in src[valid]), tb
