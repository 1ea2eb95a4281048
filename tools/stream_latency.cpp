// Per-call latency of the streaming C ABI (FEC_Encoder::onTransmit / FEC_Decoder::onReceive
// equivalents) from C++, no Python in the loop: (10,3,3), 300-byte packets, every 7th packet erased
// in bursts.  Checks each output packet against its source.
//   g++ -O2 -std=c++17 -I include tools/stream_latency.cpp -L fec_erasure_code_unit_test_relay_amd \
//       -lfec_amd -Wl,-rpath,'$ORIGIN/../fec_erasure_code_unit_test_relay_amd' -o tools/stream_latency
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "fec_amd.h"

int main(int argc, char** argv) {
    const int P = argc > 1 ? std::atoi(argv[1]) : 5000;
    const int L = 300, T = 10, B = 3, N = 3;
    fec_encoder* enc = nullptr;
    fec_decoder* dec = nullptr;
    if (fec_encoder_create(L, T, B, N, &enc) || fec_decoder_create(L, T, B, N, &dec)) {
        std::fprintf(stderr, "create failed\n");
        return 1;
    }
    std::vector<uint8_t> data(static_cast<size_t>(P) * L);
    uint64_t z = 12345;
    for (auto& b : data) {
        z = z * 6364136223846793005ull + 1442695040888963407ull;
        b = static_cast<uint8_t>(z >> 56);
    }
    std::vector<uint8_t> wire(static_cast<size_t>(P) * 2048);
    std::vector<int> wsize(P);
    // warm-up coders (not timed)
    {
        fec_encoder* e2 = nullptr;
        fec_encoder_create(L, T, B, N, &e2);
        for (int s = 0; s < 200; ++s) fec_encoder_transmit(e2, data.data(), L, s, wire.data(), &wsize[0]);
        fec_encoder_destroy(e2);
    }
    auto t0 = std::chrono::steady_clock::now();
    for (int s = 0; s < P; ++s)
        if (int st = fec_encoder_transmit(enc, data.data() + static_cast<size_t>(s) * L, L, s,
                                          wire.data() + static_cast<size_t>(s) * 2048, &wsize[s])) {
            std::fprintf(stderr, "transmit %d: %s\n", s, fec_strerror(st));
            return 1;
        }
    auto t1 = std::chrono::steady_clock::now();
    std::vector<uint8_t> out(L + 64);
    int lost = 0, bad = 0, erased = 0;
    for (int s = 0; s < P; ++s) {
        const bool er = (s % 97) >= 94;  // bursts of 3 every 97 packets
        erased += er;
        int pl = 0;
        if (int st = fec_decoder_receive(dec, er ? nullptr : wire.data() + static_cast<size_t>(s) * 2048, wsize[s],
                                         s, er ? 1 : 0, out.data(), &pl)) {
            std::fprintf(stderr, "receive %d: %s\n", s, fec_strerror(st));
            return 1;
        }
        if (s >= T) {
            if (pl == 0)
                ++lost;
            else if (pl != L || std::memcmp(out.data(), data.data() + static_cast<size_t>(s - T) * L, L) != 0)
                ++bad;
        }
    }
    auto t2 = std::chrono::steady_clock::now();
    const double us_tx = std::chrono::duration<double, std::micro>(t1 - t0).count() / P;
    const double us_rx = std::chrono::duration<double, std::micro>(t2 - t1).count() / P;
    std::printf("C ABI: fec_encoder_transmit %.2f us/call, fec_decoder_receive %.2f us/call (%d packets, %d erased, "
                "%d lost, %d wrong)\n", us_tx, us_rx, P, erased, lost, bad);
    fec_encoder_destroy(enc);
    fec_decoder_destroy(dec);
    return bad ? 1 : 0;
}
