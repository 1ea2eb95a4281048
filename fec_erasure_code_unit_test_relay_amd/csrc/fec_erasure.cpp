// fec_erasure.cpp -- erasure-pattern generators (the inputs of the decode path), restating
// Erasure_File_Generator (src/Erasure_File_Generator.cpp:25-297) byte for byte.
//
// The reference draws every sample as std::uniform_real_distribution<double>(0, 1) over
// std::mt19937.  libstdc++ implements that draw as generate_canonical<double, 53>: two 32-bit
// engine outputs g1, g2, u = (double(g1) + double(g2) * 2^32) / 2^64, and u = nextafter(1, 0) if
// the rounding reached 1.  It is restated explicitly below (canonical()), so the patterns do not
// depend on the standard library the host code is built with.  The probabilities stay `float`,
// as in the reference's signatures; `dist(gen) < p` then compares in double.
//
// The reference writes one byte per packet to a .bin file (1 = erased) plus text side files;
// here the bytes go to a caller buffer (the Python layer writes .bin files).  Verified against
// the patterns the reference ships: bin/erasure.bin and bin/erasure2.bin are
// generate_Fritchman_varying(360010, ALPHA, BETA, EPSILON=1e-4, NUMBER_OF_STATES, seed 0 / 1)
// (tests/test_erasure.py).
#include <cmath>
#include <cstdint>
#include <random>

#include "fec_amd.h"

namespace {

// SEED_ARTIFICIAL_ERASURE (include/FEC_Macro.h:80)
constexpr int kSeedArtificialErasure = 0;

struct Canonical {
    std::mt19937 gen;
    explicit Canonical(int seed) : gen(static_cast<std::mt19937::result_type>(seed)) {}
    // uniform_real_distribution<double>(0, 1)(gen) as libstdc++ computes it
    double operator()() {
        const double r = 4294967296.0;  // engine range: max - min + 1 = 2^32
        double sum = static_cast<double>(gen());
        sum += static_cast<double>(gen()) * r;
        const double u = sum / (r * r);
        return u >= 1.0 ? std::nextafter(1.0, 0.0) : u;
    }
};

bool bad_out(const uint8_t* out, int count) { return count < 0 || (count > 0 && out == nullptr); }

}  // namespace

extern "C" {

// Erasure_File_Generator::generate_IID (Erasure_File_Generator.cpp:25-63): seed 0 means
// SEED_ARTIFICIAL_ERASURE.
int fec_erasure_iid(uint8_t* out, int count, float erasure_prob, int seed) {
    if (bad_out(out, count)) return FEC_ERR_ARG;
    Canonical dist(seed == 0 ? kSeedArtificialErasure : seed);
    for (int i = 0; i < count; ++i) out[i] = dist() < erasure_prob ? 1 : 0;
    return FEC_OK;
}

// generate_three_sections_IID (Erasure_File_Generator.cpp:65-121): one engine, three sections.
int fec_erasure_three_sections_iid(uint8_t* out, int count1, float prob1, int count2, float prob2,
                                   int count3, float prob3, int seed) {
    if (count1 < 0 || count2 < 0 || count3 < 0 || bad_out(out, count1 + count2 + count3)) return FEC_ERR_ARG;
    Canonical dist(seed);
    int i = 0;
    for (int e = 0; e < count1; ++e, ++i) out[i] = dist() < prob1 ? 1 : 0;
    for (int e = 0; e < count2; ++e, ++i) out[i] = dist() < prob2 ? 1 : 0;
    for (int e = 0; e < count3; ++e, ++i) out[i] = dist() < prob3 ? 1 : 0;
    return FEC_OK;
}

// generate_GE (Erasure_File_Generator.cpp:123-170): Gilbert-Elliott channel.  The reference keeps
// the state in the generator object (good_state, true at construction) across calls: pass it in
// *good_state (NULL = a fresh object) and read it back.
int fec_erasure_ge(uint8_t* out, int count, float alpha, float beta, float erasure_prob, int seed,
                   int* good_state) {
    if (bad_out(out, count)) return FEC_ERR_ARG;
    Canonical dist(seed);
    bool good = good_state ? *good_state != 0 : true;
    for (int i = 0; i < count; ++i) {
        out[i] = good ? (dist() < erasure_prob ? 1 : 0) : 1;
        if (good) {
            if (dist() < alpha) good = false;
        } else {
            if (dist() < beta) good = true;
        }
    }
    if (good_state) *good_state = good ? 1 : 0;
    return FEC_OK;
}

// generate_GE_varying (Erasure_File_Generator.cpp:172-213): in the middle third a bad state
// always returns to good (one draw is still consumed).
int fec_erasure_ge_varying(uint8_t* out, int count, float alpha, float beta, float erasure_prob, int seed,
                           int* good_state) {
    if (bad_out(out, count)) return FEC_ERR_ARG;
    Canonical dist(seed);
    bool good = good_state ? *good_state != 0 : true;
    for (int i = 0; i < count; ++i) {
        out[i] = good ? (dist() < erasure_prob ? 1 : 0) : 1;
        if (good) {
            if (dist() < alpha) good = false;
        } else {
            const bool middle = i >= count / 3 && i <= count * 2 / 3;
            const double u = dist();
            if (!middle) {
                if (u < beta) good = true;
            } else {
                good = true;
            }
        }
    }
    if (good_state) *good_state = good ? 1 : 0;
    return FEC_OK;
}

// generate_Fritchman_varying (Erasure_File_Generator.cpp:215-264): state 0 = good; a bad state
// advances (state+1) % number_of_states with probability beta, and in the middle half it returns
// to 0.  `count * 3 / 4` is int arithmetic, as in the reference.
int fec_erasure_fritchman_varying(uint8_t* out, int count, float alpha, float beta, float erasure_prob,
                                  int number_of_states, int seed) {
    if (bad_out(out, count) || number_of_states < 1) return FEC_ERR_ARG;
    Canonical dist(seed);
    int state = 0;
    for (int i = 0; i < count; ++i) {
        out[i] = state == 0 ? (dist() < erasure_prob ? 1 : 0) : 1;
        if (state == 0) {
            if (dist() < alpha) state = 1;
        } else {
            const bool middle = i >= count / 4 && i <= count * 3 / 4;
            const double u = dist();
            if (!middle) {
                if (u < beta) state = (state + 1) % number_of_states;
            } else {
                state = 0;
            }
        }
    }
    return FEC_OK;
}

// generate_periodic (Erasure_File_Generator.cpp:266-287): the first B packets of every window of
// T-N+1+B are erased.
int fec_erasure_periodic(uint8_t* out, int count, int T, int B, int N) {
    const int period = T - N + 1 + B;
    if (bad_out(out, count) || period <= 0) return FEC_ERR_ARG;
    for (int i = 0; i < count; ++i) out[i] = (i % period) <= B - 1 ? 1 : 0;
    return FEC_OK;
}

}  // extern "C"
