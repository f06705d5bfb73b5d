"""The d = 0 fused-split kernel's algorithm (ddc_persistent.hip, r2iq_fs_kernel), modelled step
by step in numpy (tools/fs_model.py), against the f64 oracle: the lane-paired split (mirror
from lane ^ 1, register 15 - k), the inverse on absolute bins and the tune shift as the output
modulation (lane factor g_t + quarter turns).  Also checks the committed lane permutation."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import fs_model as M  # noqa: E402
import fs_perm as P  # noqa: E402
from oracle import oracle as O  # noqa: E402
from extio_sddc_amd.synth import make_stream  # noqa: E402


def test_perm_header_is_a_lane_paired_permutation():
    cols = P.read_header()
    assert P.valid(cols)
    wr, rd = P.conflicts(cols)
    assert (wr, rd) == (0, 0)   # inverse pass-0 stores and forward pass-2 reads conflict-free


@pytest.mark.parametrize("tb", [0, 4, 284, 1024, 1228, 2048, 3888, 4092])
def test_fs_model_matches_oracle(tb):
    perm = np.array(P.read_header())
    H = O.filter_bank(1.0)[0]
    x = make_stream(1, "mix")
    y = M.r2iq_fs(x, 1, tb, H, perm)
    assert O.max_rel_err(y, O.r2iq(x, 1, 0, tb)) < 1e-12
