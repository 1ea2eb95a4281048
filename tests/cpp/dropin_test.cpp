// Drop-in check: a host program written against the reference's class names (FEC_Encoder,
// FEC_Decoder, Memory_Allocator; include/fec_amd_dropin.h) driving the MI355X library, compared
// packet by packet with the oracle restatement (oracle/fec_oracle.h, linked as the checker).
#include <cstdio>
#include <cstring>
#include <vector>

#include "fec_amd_dropin.h"
#include "../../oracle/fec_oracle.h"

static int run(int T, int B, int N, int P) {
    const int L = 300;
    Memory_Allocator mem_tx(300), mem_rx(300);
    FEC_Encoder enc(L, T, B, N, &mem_tx);
    FEC_Decoder dec(L, T, B, N, &mem_rx);
    or_encoder* oe = or_encoder_new(L, T, B, N);
    or_decoder* od = or_decoder_new(L, T, B, N, 0);
    int k, n, S, CW;
    or_geometry(L, T, B, N, &k, &n, &S, &CW);
    std::vector<unsigned char> payload(L), ocw(CW), oout(L);
    int lost = 0, bad = 0;
    unsigned state = 12345u;
    for (int t = 0; t < P; ++t) {
        or_fill_payload(payload.data(), t, 1, L, 0x5EED);
        const int plen = (t % 37 == 5) ? (t % 300) : L;
        int size = 0;
        unsigned char* wire = enc.onTransmit(payload.data(), plen, t, &size);
        const int osize = or_encoder_transmit(oe, payload.data(), plen, t, ocw.data());
        if (size != osize || std::memcmp(wire, ocw.data(), size) != 0) {
            std::printf("encode mismatch at %d\n", t);
            return 1;
        }
        state = state * 1103515245u + 12345u;
        const bool erased = ((state >> 16) % 100) < 4 || (t % 211 >= 50 && t % 211 < 53);
        int got = 0;
        unsigned char* out = dec.onReceive(erased ? nullptr : wire, erased ? 0 : size, t, &got, erased);
        const int ogot = or_decoder_receive(od, erased ? nullptr : ocw.data(), osize, t, erased, oout.data());
        if (got != ogot || std::memcmp(out, oout.data(), got < L ? (got > 0 ? got : 0) : L) != 0) {
            std::printf("decode mismatch at %d: %d vs %d\n", t, got, ogot);
            ++bad;
        }
        if (t >= T && got == 0) ++lost;
    }
    or_encoder_free(oe);
    or_decoder_free(od);
    unsigned char* G = enc.encoder->getG();
    if (G[0] != 1) return 1;
    std::printf("(T,B,N)=(%d,%d,%d) packets=%d lost=%d mismatches=%d\n", T, B, N, P, lost, bad);
    return bad ? 1 : 0;
}

int main() {
    int rc = 0;
    rc |= run(10, 3, 3, 1500);
    rc |= run(10, 5, 2, 1500);
    rc |= run(10, 10, 10, 400);
    if (rc == 0) std::printf("DROPIN OK\n");
    return rc;
}
