// Host-only timing of the config 4 plan (fec::VrPlan::run): control loop and decoder phases.
//   g++ -O2 -std=c++17 -pthread -I fec_erasure_code_unit_test_relay_amd/csrc -I include -I/opt/rocm/include \
//       -D__HIP_PLATFORM_AMD__ tools/vr_plan_bench.cpp -o tools/ubench/vr_plan_bench \
//       -L fec_erasure_code_unit_test_relay_amd -lfec_amd -Wl,-rpath,'$ORIGIN/../../fec_erasure_code_unit_test_relay_amd'
//   ./tools/ubench/vr_plan_bench pattern.bin [reps]   (FEC_VR_DEBUG=1: phase split on stderr)
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "fec_vr.h"

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<uint8_t> pat(1 << 20);
    pat.resize(std::fread(pat.data(), 1, pat.size(), f));
    std::fclose(f);
    const int reps = argc > 2 ? std::atoi(argv[2]) : 10;
    double best = 1e30, c_best = 1e30, d_best = 1e30;
    fec::VrPlan p;
    for (int r = 0; r < reps; ++r) {
        const auto t0 = std::chrono::steady_clock::now();
        p.run(300, 10, -1, -1, false, pat.data(), static_cast<int64_t>(pat.size()), 360000);
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        best = std::min(best, ms);
        c_best = std::min(c_best, p.control_ms);
        d_best = std::min(d_best, p.decoders_ms);
    }
    std::printf("plan %.3f ms (control %.3f, decoders %.3f); lost %lld switches %lld steady %lld of %lld, enc %zu dec %zu\n",
                best, c_best, d_best, static_cast<long long>(p.lost), static_cast<long long>(p.switches),
                static_cast<long long>(p.steady_packets), static_cast<long long>(p.sent), p.enc.size(), p.dec.size());
    return 0;
}
