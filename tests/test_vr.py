"""Variable-rate (adaptive) coding, BASELINE config 4 (fec_vr.cpp).

The control plane is pinned by the reference's own runs recorded in SURVEY.md §8(d)/(c): on
bin/erasure.bin with P = 360000 the adaptive P2P loop loses 2982 packets, switches (T,B,N) 1933 times
("Start double coding at the source") at a final coding rate of 0.822 using the tuples (10,b,b),
b in {0,1,2,5..10}; the fixed-rate full stack loses 4662 packets at (10,3,3) and 565 at (10,5,2),
the same as the FEC-level decoder.  The GPU test runs the schedule's byte work and checks every
reported packet against its source."""
import numpy as np
import pytest

from conftest import load_pattern
from fec_erasure_code_unit_test_relay_amd import plan_host
from fec_erasure_code_unit_test_relay_amd.vr import VrPlan


@pytest.fixture(scope="module")
def adaptive():
    return VrPlan(load_pattern("bin_erasure"), 360000)


def test_adaptive_matches_reference_run(adaptive):
    v = adaptive
    assert v.lost == 2982
    assert v.switches == 1933
    assert round(v.coding_rate, 3) == 0.822
    assert v.tuples() == {(10, b, b) for b in (0, 1, 2, 5, 6, 7, 8, 9, 10)}
    assert int((v.fate == 3).sum()) == v.lost and v.fate.min() >= 1  # every packet reported once
    assert v.sent == 360010


def test_schedule_structure(adaptive):
    v = adaptive
    enc, dec, fr = v.encoders, v.decoders, v.frames
    # encoder instances: current over [first, role_switch), old over [role_switch, end), T packets
    assert (enc[1:, 3] == enc[:-1, 4]).all() and enc[0, 3] == 0
    assert ((enc[:-1, 5] - enc[:-1, 4]) == 10).all()
    s = np.arange(v.sent)
    cur = fr[:, 4]
    assert ((enc[cur, 3] <= s) & (s < enc[cur, 4])).all()
    has_old = fr[:, 5] >= 0
    old = fr[has_old, 5]
    assert ((enc[old, 4] <= s[has_old]) & (s[has_old] < enc[old, 5])).all()
    assert (fr[has_old, 3] < 10).all() and (fr[:, :3] == enc[cur, :3]).all()
    # decoder instances follow the encoders one for one here, and report [first, role_switch)
    assert len(dec) == len(enc) and (dec[:, :3] == enc[:, :3]).all()
    for j in (0, 1, 17, len(dec) - 1):
        lo, hi = dec[j, 3], min(dec[j, 4], v.P)
        assert (v.fate_decoder[lo:hi] == j).all()


@pytest.mark.parametrize("tbn,lost", [((10, 3, 3), 4662), ((10, 5, 2), 565)])
def test_fixed_rate_full_stack_equals_fec_level(tbn, lost):
    pat = load_pattern("bin_erasure")
    v = VrPlan(pat, 360000, T=tbn[0], B=tbn[1], N=tbn[2])
    assert v.lost == lost and v.switches == 0 and len(v.encoders) == 1
    # the FEC-level symbolic decoder on the same pattern gives the same lost set
    fate = plan_host(300, *tbn, pat[:360010])
    assert (np.flatnonzero(fate[:360000] == 3) == np.flatnonzero(v.fate == 3)).all()


def test_adaptive_mds_mode_and_iid():
    pat = load_pattern("bin_erasure")
    v = VrPlan(pat[:50010], 50000, adaptive_mode_MDS=True)
    assert all(b == n for _, b, n in v.tuples())
    assert v.lost < 2982 and v.fate.min() >= 1


@pytest.mark.gpu
def test_gpu_adaptive_schedule_round_trip(adaptive):
    import torch
    from fec_erasure_code_unit_test_relay_amd import fill_payload
    torch.cuda.set_device(0)
    v = adaptive
    payload = fill_payload(0, v.sent, 300, 0x5EED)
    cw_cur, len_cur, cw_old, len_old = v.encode(payload)
    has_old = torch.from_numpy(v.frames[:, 5] >= 0).cuda()
    assert bool((len_old[~has_old] == 0).all()) and bool((len_old[has_old] > 0).all())
    out, out_len = v.decode(cw_cur, cw_old)
    torch.cuda.synchronize()
    fate = torch.from_numpy(v.fate).cuda()
    ok = fate != 3
    assert int((out_len == 0).sum()) == v.lost
    assert bool((out_len[ok] == 300).all())
    assert bool((out[ok] == payload[:v.P][ok]).all())
    assert bool((out[~ok] == 0).all())


@pytest.mark.gpu
def test_gpu_adaptive_codewords_match_fixed_encoders(adaptive):
    """Each instance's codewords equal a fresh fixed-rate encoder fed the same packets from its
    creation (X before creation = 0), via the single-configuration batched path."""
    import torch
    from fec_erasure_code_unit_test_relay_amd import Codec, fill_payload
    torch.cuda.set_device(0)
    v = adaptive
    payload = fill_payload(0, v.sent, 300, 0x5EED)
    cw_cur, len_cur, cw_old, len_old = v.encode(payload)
    for j in (0, 5, 100, len(v.encoders) - 1):
        T, B, N, first, sw, end = (int(x) for x in v.encoders[j])
        c = Codec(300, T, B, N)
        ref, ref_len = c.encode(payload[first:end].contiguous())
        n1 = sw - first
        assert bool((cw_cur[first:sw, :c.CW] == ref[:n1]).all()) and bool((len_cur[first:sw] == ref_len[:n1]).all())
        assert bool((cw_old[sw:end, :c.CW] == ref[n1:]).all()) and bool((len_old[sw:end] == ref_len[n1:]).all())


@pytest.mark.gpu
@pytest.mark.parametrize("pattern,mds", [("bin_erasure2", False), ("bin_erasure", True), ("erasure50", False)])
def test_gpu_schedule_round_trip_other_patterns(pattern, mds):
    """Other shipped patterns and the MDS estimator mode: every packet the plan reports received or
    recovered comes back bit-exact, the others come back empty."""
    import torch
    from fec_erasure_code_unit_test_relay_amd import fill_payload
    torch.cuda.set_device(0)
    pat = load_pattern(pattern)
    P = min(120000, pat.size - 20)
    v = VrPlan(pat, P, adaptive_mode_MDS=mds)
    assert v.fate.min() >= 1 and int((v.fate == 3).sum()) == v.lost
    payload = fill_payload(0, v.sent, 300, 0x5EED)
    cw_cur, _, cw_old, _ = v.encode(payload)
    out, out_len = v.decode(cw_cur, cw_old)
    torch.cuda.synchronize()
    ok = torch.from_numpy(v.fate != 3).cuda()
    assert int((out_len == 0).sum()) == v.lost
    assert bool((out[ok] == payload[:P][ok]).all()) and bool((out_len[ok] == 300).all())
