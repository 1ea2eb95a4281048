"""The two-hop adaptive relay session on the GPU (fec_relay_session_*, RelaySession) against the
oracle's reference-structured loop (or_relay_session_run): per seq the source's packets, the
relay's packets, the destination's outputs and loss verdicts at a few thousand seqs, and the whole
360 000-seq session on bin/erasure.bin / bin/erasure2.bin against the committed digests
(tests/golden/relay_session_360k.json, from the same oracle: parity unpinned, the reference ships
no relay output).  The host control plane alone is checked on the CPU in test_session_control_*."""
import json
import os
import zlib

import numpy as np
import pytest

import oracle
from conftest import GOLDEN, load_pattern

from fec_erasure_code_unit_test_relay_amd.relay import RelaySession

SEED = 0x5EED


def _patterns():
    return load_pattern("bin_erasure"), load_pattern("bin_erasure2")


@pytest.mark.parametrize("R", [2, 3])
def test_session_control_plane_equals_oracle(R):
    """CPU: the symbolic control plane's schedule (hop-1 headers, relay packet sizes, the
    destination's processed seqs and flags, switches, rate sums) equals the oracle loop's."""
    e1, e2 = _patterns()
    Q = 6000
    s = RelaySession(R, Q, e1, e2)
    r = oracle.relay_session_run(R, Q, e1, e2, want_out=True)
    assert np.array_equal(s.hop1_hdr, r["hop1_hdr"])
    assert np.array_equal(np.diff(s.relay_off), r["relay_len"])
    assert np.array_equal(s.proc, r["dest_proc"]) and np.array_equal(s.flag, r["dest_flag"])
    st = s.stats
    assert (st["src_switches"], st["relay_switches"], st["dest_switches"]) == \
        (r["src_switches"], r["relay_switches"], r["dest_switches"])
    assert st["rate1"] == r["rate1"] and st["rate2"] == r["rate2"] and st["min_rate"] == r["min_rate"]


def test_session_control_plane_360k_totals():
    """CPU: the control plane over the whole session equals the committed oracle totals."""
    g = json.load(open(os.path.join(GOLDEN, "relay_session_360k.json")))
    e1, e2 = _patterns()
    for R in (2, 3):
        s = RelaySession(R, g["Q"], e1, e2)
        ref = g["types"][str(R)]
        st = s.stats
        assert st["src_switches"] == ref["src_switches"] and st["relay_switches"] == ref["relay_switches"]
        assert st["dest_switches"] == ref["dest_switches"] and st["relay_bytes"] == ref["relay_bytes"]
        assert st["processed"] == ref["processed"] and int(s.flag.sum()) == ref["dest_flags"]
        assert st["rate1"] == ref["rate1_sum"] and st["rate2"] == ref["rate2_sum"]


def _gpu_run(R, Q, e1, e2):
    import torch
    from fec_erasure_code_unit_test_relay_amd import fill_payload
    s = RelaySession(R, Q, e1, e2)
    pay = fill_payload(0, Q, 300, SEED)
    relay, out, lost, count = s.run(pay)
    torch.cuda.synchronize()
    return s, pay, relay, out, lost, count


@pytest.mark.gpu
@pytest.mark.parametrize("R", [2, 3])
def test_gpu_session_equals_oracle_per_seq(R):
    import torch
    e1, e2 = _patterns()
    Q = 4000
    s, pay, relay, out, lost, count = _gpu_run(R, Q, e1, e2)
    stride1 = 8192
    hop1, hop1_len = s.hop1_packets(stride1)
    torch.cuda.synchronize()
    r = oracle.relay_session_run(R, Q, e1, e2, want_out=True, hop1_stride=stride1, relay_stride=8192)
    # the source's packets (16-byte header + [size BE16][cur][old])
    assert np.array_equal(hop1_len.cpu().numpy(), r["hop1_len"])
    h1 = hop1.cpu().numpy()
    bad = np.nonzero((h1 != r["hop1_pkts"]).any(axis=1))[0]
    assert bad.size == 0, f"hop-1 packet {bad[:5]} differs"
    # the relay's packets
    rl = relay.cpu().numpy()
    off = s.relay_off
    for t in range(Q):
        got = rl[off[t]:off[t + 1]]
        exp = r["relay_pkts"][t, :r["relay_len"][t]]
        assert np.array_equal(got, exp), f"relay packet {t} differs ({np.nonzero(got != exp)[0][:8]})"
    # the destination's outputs and verdicts
    o = out.cpu().numpy()
    bad = np.nonzero((o != r["dest_out"]).any(axis=1))[0]
    assert bad.size == 0, f"destination output {bad[:5]} differs"
    assert np.array_equal(lost.cpu().numpy(), r["dest_lost"])
    assert int(count.item()) == r["lost"]


@pytest.mark.gpu
@pytest.mark.parametrize("R", [2, 3])
def test_gpu_session_360k_equals_golden(R):
    """The whole session (Q = 360 020 seqs): per block of 100 seqs the CRC-32 of the hop-1 and
    relay packets and of the destination's outputs equal the oracle's committed digests."""
    import torch
    g = json.load(open(os.path.join(GOLDEN, "relay_session_360k.json")))
    ref = g["types"][str(R)]
    e1, e2 = _patterns()
    Q = g["Q"]
    s, pay, relay, out, lost, count = _gpu_run(R, Q, e1, e2)
    assert int(count.item()) == ref["lost"]
    hop1, hop1_len = s.hop1_packets(6720)
    torch.cuda.synchronize()
    h1 = hop1.cpu().numpy()
    hl = hop1_len.cpu().numpy()
    rl = relay.cpu().numpy()
    off = s.relay_off
    o = out.cpu().numpy()
    ls = lost.cpu().numpy()
    B = g["block"]
    crc, crc2 = [], []
    for b0 in range(0, Q, B):
        c = c2 = 0
        for t in range(b0, min(Q, b0 + B)):
            n1 = int(hl[t])
            c = zlib.crc32(n1.to_bytes(4, "little"), c)
            c = zlib.crc32(h1[t, :n1].tobytes(), c)
            n2 = int(off[t + 1] - off[t])
            c = zlib.crc32(n2.to_bytes(4, "little"), c)
            c = zlib.crc32(rl[off[t]:off[t + 1]].tobytes(), c)
            c2 = zlib.crc32(bytes([int(s.proc[t]), int(s.flag[t]), int(ls[t])]), c2)
            c2 = zlib.crc32(o[t].tobytes(), c2)
        crc.append(c)
        crc2.append(c2)
    bad = [i for i in range(len(crc)) if crc[i] != ref["crc"][i]]
    assert not bad, f"packet digest blocks {bad[:5]} differ"
    bad = [i for i in range(len(crc2)) if crc2[i] != ref["crc2"][i]]
    assert not bad, f"destination digest blocks {bad[:5]} differ"
