"""Drop-in boundary checks that need no GPU.

- include/fft_mt_r2iq.h + extio_sddc_amd/csrc/r2iq/fft_mt_r2iq.cpp compile against the
  REFERENCE's own Core/r2iq.h and dsp/ringbuffer.h (where mounted) and against the
  standalone compat headers; the class's static_asserts pin the base-class layout of
  Core/r2iq.h (sizeof 48, mdecimation @8, r2iqOn @12, mratio @16).
- The exported symbol set matches what the reference's callers link to
  (fft_mt_r2iq::{ctor, dtor, Init, TurnOn, TurnOff, IsOn,
  setFreqOffset} and r2iqControlClass::r2iqControlClass()).
"""
from __future__ import annotations

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "extio_sddc_amd", "csrc", "r2iq", "fft_mt_r2iq.cpp")
REF = "/root/reference"

REQUIRED = [
    "fft_mt_r2iq::fft_mt_r2iq()", "fft_mt_r2iq::~fft_mt_r2iq()",
    "fft_mt_r2iq::Init(float, ringbuffer<short>*, ringbuffer<float>*)",
    "fft_mt_r2iq::TurnOn()", "fft_mt_r2iq::TurnOff()", "fft_mt_r2iq::IsOn()",
    "fft_mt_r2iq::setFreqOffset(float)", "r2iqControlClass::r2iqControlClass()",
]


def _compile(tmp_path, incs):
    obj = tmp_path / "r2iq.o"
    cmd = ["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-c", SRC, "-o", str(obj)] + sum([["-I", i] for i in incs], [])
    p = subprocess.run(cmd, capture_output=True, text=True)
    assert p.returncode == 0, p.stderr
    syms = subprocess.run(["nm", "-C", "--defined-only", str(obj)], capture_output=True, text=True).stdout
    return syms


def test_compiles_against_compat_headers(tmp_path):
    syms = _compile(tmp_path, [os.path.join(ROOT, "include"), os.path.join(ROOT, "include", "sddc_compat")])
    for s in REQUIRED:
        assert s in syms, s


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "Core")), reason="reference tree not mounted")
def test_compiles_against_reference_headers(tmp_path):
    # our include/ first so our fft_mt_r2iq.h wins; r2iq.h and dsp/ringbuffer.h are the reference's
    syms = _compile(tmp_path, [os.path.join(ROOT, "include"), os.path.join(REF, "Core"), REF])
    for s in REQUIRED:
        assert s in syms, s


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "Core")), reason="reference tree not mounted")
def test_reference_radiohandler_links_against_dropin():
    # builds oracle/_ref/radiohandler_harness: the unchanged Core/RadioHandler.cpp + radio models
    # + pf_mixer + our class + libsddc_ddc.so (see oracle/Makefile `radiohandler`)
    p = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "radiohandler"],
                       capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-4000:]
    assert os.path.exists(os.path.join(ROOT, "oracle", "_ref", "radiohandler_harness"))


def test_standalone_harness_built():
    assert os.path.exists(os.path.join(ROOT, "build", "bin", "r2iq_harness")), \
        "run make -C extio_sddc_amd/csrc (or __graft_entry__.build())"


def test_queued_blocks_survives_write_count_wrap(tmp_path):
    """The worker's batching count (csrc/r2iq/batching.h) stays exact when the ring's int
    writeCount (Core/dsp/ringbuffer.h, never reset) passes INT_MAX after 2^31 blocks."""
    src = tmp_path / "t.cpp"
    src.write_text(r'''
#include <climits>
#include <cstdio>
#include <initializer_list>
#include "batching.h"
using sddc_r2iq::queued_blocks;
static int wrap(long long v) { return (int)(unsigned)(v & 0xffffffffLL); }   // two's complement int
int main() {
    int bad = 0;
    for (long long base : {0LL, (long long)INT_MAX - 5, (long long)INT_MAX, 4294967290LL}) {
        for (long long consumed = 0; consumed < 40; consumed += 3)
            for (long long queued = 0; queued < 20; queued++) {
                const long long wc = base + consumed + queued;
                if (queued_blocks(wrap(wc), wrap(base), (unsigned long long)consumed) != (unsigned)queued) bad++;
            }
    }
    std::printf("%d\n", bad);
    return bad != 0;
}
''')
    exe = tmp_path / "t"
    p = subprocess.run(["g++", "-std=c++17", "-O2", "-fwrapv", "-I", os.path.join(ROOT, "extio_sddc_amd", "csrc", "r2iq"),
                        str(src), "-o", str(exe)], capture_output=True, text=True)
    assert p.returncode == 0, p.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.strip() == "0", r.stdout
