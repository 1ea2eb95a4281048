"""Block mode (fec_block.hip): batched encodeBlock(t = k-1) / decodeBlock(T = n-1, t = 0), the
relay's per-code-block calls (src/Decoder_Symbol_Wise.cpp:322-328, 532-533, 573-575, 610, 643),
against the oracle's reference-structured encode_block / decode_block (oracle/fec_oracle.c, RREF
per call) on the same blocks: every erasure mask of a small code, random masks of larger ones,
garbage in the erased symbols."""
import numpy as np
import pytest

import oracle

TBNS = [(10, 3, 3), (10, 5, 2), (10, 0, 0), (10, 10, 10), (10, 9, 9), (6, 4, 2), (10, 8, 4), (11, 5, 4)]


@pytest.mark.gpu
@pytest.mark.parametrize("tbn", TBNS)
def test_block_encode_matches_oracle(tbn):
    import torch
    from fec_erasure_code_unit_test_relay_amd import Codec
    torch.cuda.set_device(0)
    c = Codec(300, *tbn)
    G = oracle.gen_G(*tbn)
    rng = np.random.default_rng(7)
    for nblk in (1, 255, 256, 1000, 70001):
        data = rng.integers(0, 256, (nblk, c.k), dtype=np.uint8)
        got = c.encode_blocks(torch.from_numpy(data).cuda()).cpu().numpy()
        for b in rng.choice(nblk, size=min(nblk, 300), replace=False):
            cw = np.zeros(c.n, dtype=np.uint8)
            cw[:c.k] = data[b]  # the relay pre-fills the codeword with the data
            oracle.encode_block(data[b], G, cw, c.k - 1)
            assert (got[b] == cw).all(), (tbn, nblk, b)


@pytest.mark.gpu
@pytest.mark.parametrize("tbn", TBNS)
def test_block_decode_matches_oracle(tbn):
    import torch
    from fec_erasure_code_unit_test_relay_amd import Codec
    torch.cuda.set_device(0)
    c = Codec(300, *tbn)
    k, n = c.k, c.n
    G = oracle.gen_G(*tbn)
    rng = np.random.default_rng(11)
    if n <= 11:
        masks = np.arange(1 << n, dtype=np.int64)  # every erasure pattern
    else:
        masks = rng.integers(0, 1 << n, 4096)
    data = rng.integers(0, 256, (masks.size, k), dtype=np.uint8)
    cw = c.encode_blocks(torch.from_numpy(data).cuda()).cpu().numpy()
    er = ((masks[:, None] >> np.arange(n)) & 1).astype(np.uint8)
    noisy = cw.copy()
    noisy[er == 1] = rng.integers(0, 256, int(er.sum()), dtype=np.uint8)  # erased symbols: garbage
    out, er_out = c.decode_blocks(torch.from_numpy(noisy).cuda(), torch.from_numpy(er).cuda())
    out, er_out = out.cpu().numpy(), er_out.cpu().numpy()
    for b in range(masks.size):
        ref, ref_er = oracle.decode_block(noisy[b], G, er[b], n - 1, 0)
        assert (out[b] == ref).all() and (er_out[b] == ref_er).all(), (tbn, int(masks[b]))
        rec = (er[b, :k] == 1) & (er_out[b, :k] == 0)
        assert (out[b, :k][rec] == data[b][rec]).all()  # a recovered symbol is the source symbol
    # MDS code, at most n-k erasures: everything comes back
    if tbn[1] == tbn[2]:
        few = er.sum(1) <= n - k
        assert (er_out[few, :k] == 0).all()
