"""The many-channel v2 kernel's channel-slice layout (ddc_channels.hip, kg): pass A stores and
pass B loads are LDS-bank-conflict-free at d = 4..6 (tools/channel_banks.py), where the unkeyed
layout had a 2-way conflict on every pass-B load of config C5 (d = 4)."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import channel_banks as CB  # noqa: E402


@pytest.mark.parametrize("D", [4, 5, 6])
def test_keyed_slices_conflict_free(D):
    assert CB.slice_conflicts(D) == (0, 0)
    assert CB.slice_conflicts(D, keyed=False) != (0, 0)


@pytest.mark.parametrize("D", [4, 5, 6])
def test_key_stays_inside_the_slice(D):
    N = 4096 >> D
    TPC = N // 16
    for g in range(256 // TPC):
        assert 0 <= CB.key(g, TPC) < N   # an XOR on the element index inside the slice
