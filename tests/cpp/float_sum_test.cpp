// fec::float_add_repeated (fec_vr.cpp) against the loop it replaces: `count` sequential float adds
// of one rate (Variable_Rate_FEC_Encoder.cpp:176-190's final_sum_coding_rate), bit for bit, over
// the coding rates of every (T,B,N) with T <= 10 in both forms (single and double coding), random
// rates, exact halves and powers of two (ties at every binade), starting sums from 0 to 2^22, and
// whole run sequences like a plan's.  Prints "FLOAT SUM OK" and exits 0 on success.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

namespace fec {
float float_add_repeated(float s, float r, int64_t count);
}

static float seq(float s, float r, int64_t count) {
    for (int64_t i = 0; i < count; ++i) s += r;
    return s;
}

static uint32_t bits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

int main() {
    std::vector<float> rates;
    for (int T = 0; T <= 10; ++T)
        for (int N = 0; N <= T; ++N)
            for (int B = N; B <= T; ++B) {
                const int k = T - N + 1;
                rates.push_back(static_cast<float>(k) / (k + B));
                for (int No = 0; No <= T; ++No)
                    rates.push_back(static_cast<float>(k) / ((k + B) + (T - No + 1) + (T - No + 1 + B)));
            }
    for (float r : {0.5f, 0.25f, 0.75f, 1.0f, 0.125f, 0.375f, 1.5f, 3.0f, 0.0625f}) rates.push_back(r);
    std::mt19937_64 g(12345);
    std::uniform_real_distribution<float> u01(0.0f, 1.0f);
    for (int i = 0; i < 200; ++i) rates.push_back(u01(g));
    int64_t cases = 0, bad = 0;
    const float starts[] = {0.0f, 1e-6f, 0.3f, 1.0f, 7.5f, 1000.25f, 65535.0f, 131072.0f, 262143.9f, 300000.0f, 4194304.0f};
    std::uniform_int_distribution<int64_t> ucount(0, 400000);
    for (float r : rates)
        for (float s0 : starts)
            for (int64_t c : {int64_t(0), int64_t(1), int64_t(2), int64_t(3), int64_t(17), int64_t(1000), ucount(g)}) {
                ++cases;
                const float a = seq(s0, r, c), b = fec::float_add_repeated(s0, r, c);
                if (bits(a) != bits(b)) {
                    if (++bad <= 10)
                        std::printf("s0 %.9g r %.9g count %lld: loop %.9g (%08x) fast %.9g (%08x)\n", s0, r,
                                    static_cast<long long>(c), a, bits(a), b, bits(b));
                }
            }
    // run sequences as a plan makes them: runs of 1..2000 packets of rates from the table
    for (int t = 0; t < 50; ++t) {
        std::uniform_int_distribution<size_t> ur(0, rates.size() - 1);
        std::uniform_int_distribution<int64_t> ul(1, 2000);
        float a = 0, b = 0;
        int64_t total = 0;
        while (total < 360000) {
            const float r = rates[ur(g)];
            const int64_t c = ul(g);
            a = seq(a, r, c);
            b = fec::float_add_repeated(b, r, c);
            total += c;
        }
        ++cases;
        if (bits(a) != bits(b) && ++bad <= 10) std::printf("sequence %d: loop %.9g fast %.9g\n", t, a, b);
    }
    std::printf("%lld cases, %lld differ\n", static_cast<long long>(cases), static_cast<long long>(bad));
    if (bad) return 1;
    std::printf("FLOAT SUM OK\n");
    return 0;
}
