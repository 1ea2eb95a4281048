"""The header swap INTEGRATION.md §2 documents, checked against the reference's own callers.

A maintainer replaces seven reference headers (FEC_Encoder.h, FEC_Decoder.h, Memory_Allocator.h,
FEC_Message.h, Encoder.h, Decoder.h, Decoder_Symbol_Wise.h) with one-line forwarders to
include/fec_amd_dropin.h (Decoder_Symbol_Wise.h keeps its FEC_Macro.h include), and drops
src/Decoder_Symbol_Wise.cpp from the build (the drop-in library defines siphon::Decoder_Symbol_Wise).  This test
does exactly that in a temporary copy of the reference's include/ (nothing of the reference is kept
or committed), stubs only what the image lacks (Boost posix_time, Intel ISA-L's header), and runs
`g++ -fsyntax-only` on the reference's callers of the coding path.  It is skipped where
/root/reference is absent (the GPU box).
"""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

REF = "/root/reference"
SWAPPED = ["FEC_Encoder.h", "FEC_Decoder.h", "Memory_Allocator.h", "FEC_Message.h", "Encoder.h",
           "Decoder.h", "Decoder_Symbol_Wise.h"]
FORWARDER = {"Decoder_Symbol_Wise.h": '#pragma once\n#include "FEC_Macro.h"\n#include "fec_amd_dropin.h"\n'}
CALLERS = ["Variable_Rate_FEC_Encoder.cpp", "Variable_Rate_FEC_Decoder.cpp", "Application_Layer_Sender.cpp",
           "Application_Layer_Receiver.cpp"]
# compiled only against the original headers (the swap removes it from the build)
ORIGINAL_ONLY = ["Decoder_Symbol_Wise.cpp"]

# Boost is absent from the image; the reference uses three posix_time names
# (Variable_Rate_FEC_Decoder.h:19,174; Payload_Simulator.h:20,46).  Real Boost brings <string> and
# <cstring> with it (Variable_Rate_FEC_Decoder.cpp calls memcpy on the strength of that), so the stub
# does too; it brings no <cmath>, <fstream> or <random>: those must come from the drop-in header.
BOOST_STUB = """#pragma once
#include <cstdint>
#include <cstring>
#include <string>
namespace boost { namespace posix_time {
struct time_duration { long long us = 0;
  long long total_milliseconds() const { return us / 1000; }
  long long total_microseconds() const { return us; } };
struct ptime { long long us = 0;
  time_duration operator-(const ptime& o) const { return time_duration{us - o.us}; } };
struct microsec_clock { static ptime universal_time() { return ptime{}; }
                        static ptime local_time() { return ptime{}; } };
struct second_clock { static ptime universal_time() { return ptime{}; }
                      static ptime local_time() { return ptime{}; } };
} }
"""
ISAL_STUB = """#pragma once
extern "C" {
unsigned char gf_mul(unsigned char a, unsigned char b);
unsigned char gf_inv(unsigned char a);
int gf_invert_matrix(unsigned char* in, unsigned char* out, const int n);
void gf_gen_cauchy1_matrix(unsigned char* a, int m, int k);
void gf_gen_rs_matrix(unsigned char* a, int m, int k);
}
"""

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "include")) or
                                shutil.which("g++") is None,
                                reason="needs the reference checkout and g++ (not on the GPU box)")


def _overlay(tmp_path, swap: bool):
    inc = tmp_path / ("swapped" if swap else "original")
    shutil.copytree(os.path.join(REF, "include"), inc)
    if swap:
        for h in SWAPPED:
            (inc / h).write_text(FORWARDER.get(h, '#pragma once\n#include "fec_amd_dropin.h"\n'))
    stub = tmp_path / "stubs"
    (stub / "boost" / "date_time" / "posix_time").mkdir(parents=True, exist_ok=True)
    (stub / "boost" / "date_time" / "posix_time" / "posix_time.hpp").write_text(BOOST_STUB)
    (stub / "isa-l.h").write_text(ISAL_STUB)
    return [f"-I{inc}", f"-I{stub}", f"-I{os.path.join(ROOT, 'include')}"]


def _syntax(flags, src):
    return subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-w"] + flags +
                          [os.path.join(REF, "src", src)], capture_output=True, text=True, timeout=120)


@pytest.mark.parametrize("src", CALLERS)
def test_reference_caller_compiles_against_dropin(tmp_path, src):
    r = _syntax(_overlay(tmp_path, swap=True), src)
    assert r.returncode == 0, f"{src} does not compile under the header swap:\n{r.stderr[-3000:]}"


def test_stubs_alone_compile_the_original_headers(tmp_path):
    """Control: the same stubs with the reference's original headers compile the same callers, so a
    failure above is the drop-in header's, not the stubs'."""
    flags = _overlay(tmp_path, swap=False)
    for src in CALLERS + ORIGINAL_ONLY:
        r = _syntax(flags, src)
        assert r.returncode == 0, f"{src}:\n{r.stderr[-2000:]}"
