"""Calibration of the CPU baseline: the oracle's reference-structured
restatement timed on the workloads of SURVEY §6's anchors, on one core, in the survey's kind of
container, and the ratio restatement / reference per workload.

Anchors (the reference itself with the ISA-L restatement, g++ -O2, 1 core):
  FEC_Encoder::onTransmit (10,3,3), 1M packets              14.37 us/packet
  FEC_Decoder (10,3,3) on bin/erasure.bin, 360k packets      77.66 us/packet
  FEC_Encoder (10,5,2), 360k packets                         21.39 us/packet
  FEC_Decoder (10,5,2) on bin/erasure.bin, 360k packets     131.12 us/packet
The decode time is the run_stream time (encode + channel + decode) minus the encode-only time of
the same packets.
  python tools/cpu_calibrate.py [--packets 360000] > profiles/r03/cpu_calibration.json"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
from fec_erasure_code_unit_test_relay_amd.streams import load_pattern  # noqa: E402

ANCHORS = {(10, 3, 3): (14.37, 77.66), (10, 5, 2): (21.39, 131.12)}
ap = argparse.ArgumentParser()
ap.add_argument("--packets", type=int, default=360000)
args = ap.parse_args()
P, L = args.packets, 300
pat = load_pattern("bin_erasure")[:P + 10]
res = {"packets": P, "pattern": "bin/erasure.bin (first P+T packets)", "cores": 1, "workloads": {}}
for (T, B, N), (a_enc, a_dec) in ANCHORS.items():
    t0 = time.perf_counter()
    oracle.encode_stream(L, T, B, N, 0, P + T, want_codewords=False)
    enc = (time.perf_counter() - t0) / (P + T) * 1e6
    t0 = time.perf_counter()
    r = oracle.run_stream(L, T, B, N, P, pat, loss_only=False)
    both = (time.perf_counter() - t0) / (P + T) * 1e6
    dec = both - enc
    res["workloads"][f"({T},{B},{N})"] = {
        "encode_us_per_packet": round(enc, 3), "decode_us_per_packet": round(dec, 3),
        "lost": r["lost"],
        "reference_encode_us_per_packet": a_enc, "reference_decode_us_per_packet": a_dec,
        "ratio_encode": round(enc / a_enc, 3), "ratio_decode": round(dec / a_dec, 3),
        "ratio_encode_plus_decode": round((enc + dec) / (a_enc + a_dec), 3)}
    print(json.dumps({f"({T},{B},{N})": res["workloads"][f"({T},{B},{N})"]}), file=sys.stderr, flush=True)
print(json.dumps(res, indent=1))
