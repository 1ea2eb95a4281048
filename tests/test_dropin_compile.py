"""The header swap INTEGRATION.md §2 documents, checked against the reference's own callers.

A maintainer replaces nine reference headers (FEC_Encoder.h, FEC_Decoder.h, Memory_Allocator.h,
FEC_Message.h, Encoder.h, Decoder.h, Decoder_Symbol_Wise.h -> include/fec_amd_dropin.h;
basicOperations.h, codingOperations.h -> include/fec_amd_refops.h) with one-line forwarders
(Decoder_Symbol_Wise.h and basicOperations.h keep their FEC_Macro.h include), and drops every coding
source from the build (FEC_Encoder/Decoder, Memory_Allocator, FEC_Message, Encoder*, Decoder*,
Decoder_Symbol_Wise, basicOperations, codingOperations).  This test does exactly that in a temporary
copy of the reference's include/ (nothing of the reference is kept or committed), stubs only Boost
posix_time (absent from the image; ISA-L's header only for the control build of the original headers),
runs `g++ -fsyntax-only` on the reference's callers of the coding path, and links the remaining
sources with -Wl,--no-undefined against libfec_amd.so.  It is skipped where /root/reference is absent
(the GPU box).
"""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

REF = "/root/reference"
SWAPPED = ["FEC_Encoder.h", "FEC_Decoder.h", "Memory_Allocator.h", "FEC_Message.h", "Encoder.h",
           "Decoder.h", "Decoder_Symbol_Wise.h", "basicOperations.h", "codingOperations.h"]
FORWARDER = {"Decoder_Symbol_Wise.h": '#pragma once\n#include "FEC_Macro.h"\n#include "fec_amd_dropin.h"\n',
             "basicOperations.h": '#pragma once\n#include "FEC_Macro.h"\n#include "fec_amd_refops.h"\n',
             "codingOperations.h": '#pragma once\n#include "fec_amd_refops.h"\n'}
# the globals the reference's drivers define (FEC_Macro.h:24-83, application_local_simulation.cpp:45-51)
GLOBALS_STUB = """int RELAYING_TYPE = 0;
int N_INITIAL = -1;
int N_INITIAL_2 = -1;
int var_header_size = 0;
int fixed_header_size = 0;
float EPSILON = 0.0001f;
"""
CALLERS = ["Variable_Rate_FEC_Encoder.cpp", "Variable_Rate_FEC_Decoder.cpp", "Application_Layer_Sender.cpp",
           "Application_Layer_Receiver.cpp"]
# compiled only against the original headers (the swap removes it from the build)
ORIGINAL_ONLY = ["Decoder_Symbol_Wise.cpp"]
# the rest of the reference's sources that a build keeps (the application layers and simulators);
# under the swap they link against libfec_amd.so alone
LINKED = CALLERS + ["Parameter_Estimator.cpp", "Payload_Simulator.cpp", "Erasure_Simulator.cpp",
                    "Erasure_File_Generator.cpp", "ConnectionManager.cpp"]

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
    stub = tmp_path / ("stubs_swapped" if swap else "stubs")
    (stub / "boost" / "date_time" / "posix_time").mkdir(parents=True, exist_ok=True)
    (stub / "boost" / "date_time" / "posix_time" / "posix_time.hpp").write_text(BOOST_STUB)
    if not swap:  # under the swap nothing may include ISA-L any more
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


def test_swapped_reference_links_without_isal(tmp_path):
    """The reference's application layers and simulators (LINKED), compiled under the full swap --
    basicOperations.h and codingOperations.h included, so neither basicOperations.cpp,
    codingOperations.cpp nor any ISA-L header or library takes part -- link into a shared object
    with -Wl,--no-undefined against libfec_amd.so alone; the only other object is a stub defining
    the drivers' globals."""
    import fec_erasure_code_unit_test_relay_amd as fec
    if not os.path.exists(fec.LIB_PATH):
        pytest.skip("needs the built libfec_amd.so")
    flags = _overlay(tmp_path, swap=True)
    objs = []
    for src in LINKED:
        o = tmp_path / (src + ".o")
        r = subprocess.run(["g++", "-std=c++17", "-c", "-fPIC", "-O0", "-w"] + flags +
                           [os.path.join(REF, "src", src), "-o", str(o)], capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, f"{src}:\n{r.stderr[-3000:]}"
        objs.append(str(o))
    g = tmp_path / "globals.cpp"
    g.write_text(GLOBALS_STUB)
    libdir = os.path.dirname(fec.LIB_PATH)
    out = tmp_path / "libreference_swapped.so"
    r = subprocess.run(["g++", "-shared", "-fPIC", "-o", str(out), str(g)] + objs +
                       ["-L", libdir, "-lfec_amd", "-lpthread", "-Wl,--no-undefined"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, f"link under the swap failed:\n{r.stderr[-4000:]}"
    nm = subprocess.run(["nm", "-D", "--undefined-only", str(out)], capture_output=True, text=True)
    assert "gf_mul" not in nm.stdout and "gf_inv" not in nm.stdout  # no ISA-L symbol anywhere


def test_reference_signature_functions_equal_oracle(tmp_path):
    """tests/cpp/refops_test.cpp: the library's gf256_* / init_at_sender / encodeBlock / decodeBlock
    (fec_amd_refops.h, host code over the library's field) against the oracle's restatements of
    basicOperations.cpp / codingOperations.cpp on random matrices and erasure patterns."""
    import fec_erasure_code_unit_test_relay_amd as fec
    if not os.path.exists(fec.LIB_PATH):
        pytest.skip("needs the built libfec_amd.so")
    libdir = os.path.dirname(fec.LIB_PATH)
    exe = tmp_path / "refops_test"
    r = subprocess.run(["g++", "-O2", "-x", "c++", "-std=c++17", os.path.join(ROOT, "tests", "cpp", "refops_test.cpp"),
                        "-x", "c", os.path.join(ROOT, "oracle", "fec_oracle.c"), "-x", "none",
                        "-I", os.path.join(ROOT, "include"), "-L", libdir, "-lfec_amd", f"-Wl,-rpath,{libdir}",
                        "-o", str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "REFOPS OK" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]
