"""Writes tests/golden/relay_session_360k.json: the two-hop adaptive relay session (RELAYING_TYPE 2
and 3, application_local_simulation.cpp:71-593 with FLAG_FOR_CONSTANT_TRANS = 1) over
bin/erasure.bin (hop 1) and bin/erasure2.bin (hop 2), Q = 360 020 seqs (the reference's loop
runs until seq NUMBER_OF_ITERATIONS + T + T2 - 1 = 360 019), as the oracle's reference-structured
loop (or_relay_session_run) computes it: per block of 100 seqs the CRC-32 of the hop-1 and hop-2
packets (crc) and of the destination's outputs (crc2), and the totals.  Parity unpinned: the
reference ships no relay output, so this file pins the product to the oracle's restatement.

    python tests/golden/make_relay_session_golden.py
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
import oracle  # noqa: E402
from conftest import load_pattern  # noqa: E402

Q = 360020


def main():
    e1, e2 = load_pattern("bin_erasure"), load_pattern("bin_erasure2")
    res = {"Q": Q, "hop1": "bin/erasure.bin", "hop2": "bin/erasure2.bin", "seed": 0x5EED, "max_payload": 300,
           "block": oracle.SESSION_BLOCK, "source": "oracle/fec_oracle.c or_relay_session_run", "types": {}}
    for R in (2, 3):
        t0 = time.time()
        r = oracle.relay_session_run(R, Q, e1, e2, want_out=True)
        res["types"][str(R)] = {
            "lost": int(r["lost"]), "src_switches": int(r["src_switches"]), "relay_switches": int(r["relay_switches"]),
            "dest_switches": int(r["dest_switches"]), "dest_flags": int(r["dest_flags"]),
            "rate1_sum": float(r["rate1"]), "rate1_n": int(r["rate1_n"]), "rate2_sum": float(r["rate2"]),
            "rate2_n": int(r["rate2_n"]), "processed": int(r["dest_proc"].sum()),
            "hop1_bytes": int(r["hop1_len"].sum()), "relay_bytes": int(r["relay_len"].sum()),
            "crc": [int(x) for x in r["crc"]], "crc2": [int(x) for x in r["crc2"]],
            "oracle_seconds": round(time.time() - t0, 1)}
        print(R, {k: v for k, v in res["types"][str(R)].items() if not k.startswith("crc")}, flush=True)
    json.dump(res, open(os.path.join(HERE, "relay_session_360k.json"), "w"))


if __name__ == "__main__":
    main()
