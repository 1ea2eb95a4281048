// Per-call latency of the streaming C ABI (FEC_Encoder::onTransmit / FEC_Decoder::onReceive
// equivalents) from C++, no Python in the loop: (10,3,3), 300-byte packets, every 7th packet erased
// in bursts.  Checks each output packet against its source.
//   g++ -O2 -std=c++17 -I include tools/stream_latency.cpp -L fec_erasure_code_unit_test_relay_amd \
//       -lfec_amd -Wl,-rpath,'$ORIGIN/../fec_erasure_code_unit_test_relay_amd' -o tools/stream_latency
#include <algorithm>
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
    // per-call durations by what the call outputs: packet s-T received (a systematic copy) or
    // erased (a recovery on the GPU, or nothing when lost)
    std::vector<double> us_copy, us_rec;
    for (int s = 0; s < P; ++s) {
        const bool er = (s % 97) >= 94;  // bursts of 3 every 97 packets
        erased += er;
        int pl = 0;
        const auto c0 = std::chrono::steady_clock::now();
        if (int st = fec_decoder_receive(dec, er ? nullptr : wire.data() + static_cast<size_t>(s) * 2048, wsize[s],
                                         s, er ? 1 : 0, out.data(), &pl)) {
            std::fprintf(stderr, "receive %d: %s\n", s, fec_strerror(st));
            return 1;
        }
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - c0).count();
        if (s >= T) {
            const bool out_erased = ((s - T) % 97) >= 94;
            (out_erased ? us_rec : us_copy).push_back(us);
            if (pl == 0)
                ++lost;
            else if (pl != L || std::memcmp(out.data(), data.data() + static_cast<size_t>(s - T) * L, L) != 0)
                ++bad;
        }
    }
    auto t2 = std::chrono::steady_clock::now();
    const double us_tx = std::chrono::duration<double, std::micro>(t1 - t0).count() / P;
    const double us_rx = std::chrono::duration<double, std::micro>(t2 - t1).count() / P;
    auto stats = [](std::vector<double> v, double* mean, double* p50, double* p99, double* mx) {
        if (v.empty()) {
            *mean = *p50 = *p99 = *mx = 0;
            return;
        }
        double sum = 0;
        for (double x : v) sum += x;
        std::sort(v.begin(), v.end());
        *mean = sum / v.size();
        *p50 = v[v.size() / 2];
        *p99 = v[std::min(v.size() - 1, v.size() * 99 / 100)];
        *mx = v.back();
    };
    double cm, c50, c99, cmx, rm, r50, r99, rmx;
    stats(us_copy, &cm, &c50, &c99, &cmx);
    stats(us_rec, &rm, &r50, &r99, &rmx);
    std::printf("C ABI: fec_encoder_transmit %.2f us/call, fec_decoder_receive %.2f us/call (%d packets, %d erased, "
                "%d lost, %d wrong)\n", us_tx, us_rx, P, erased, lost, bad);
    std::printf("  receive, output received (systematic copy): %zu calls, mean %.2f p50 %.2f p99 %.2f max %.1f us\n",
                us_copy.size(), cm, c50, c99, cmx);
    std::printf("  receive, output erased (recovery): %zu calls, mean %.2f p50 %.2f p99 %.2f max %.1f us\n",
                us_rec.size(), rm, r50, r99, rmx);
    fec_encoder_destroy(enc);
    fec_decoder_destroy(dec);
    return bad ? 1 : 0;
}
