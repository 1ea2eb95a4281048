// Relay drop-in check: siphon::Decoder_Symbol_Wise (include/fec_amd_dropin.h: host control flow,
// GF work on the GPU) driven the way Variable_Rate_FEC_Decoder drives the reference's relay and
// destination (src/Variable_Rate_FEC_Decoder.cpp:950-1879, one relay frame per seq), for
// RELAYING_TYPE 2 (symbol_wise_encode_1 / decode_1) and 3 (the state-dependent pair), against
//   (1) the oracle's whole fixed-rate chains (or_swdf_run / or_sdswdf_run), and
//   (2) the same driver over OracleSW: the reference's Decoder_Symbol_Wise restated over its member
//       arrays with the oracle's methods (or_sw_*), including a double-coding stretch (two live
//       objects per node, the frame [BE16 size][cur][old], copy_elements at its end,
//       Variable_Rate_FEC_Decoder.cpp:1423-1600, :1772-1873).
// Frames, destination outputs and loss flags must be equal per seq.
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "fec_amd_dropin.h"
#include "../../oracle/fec_oracle.h"

namespace {
constexpr int TT = 10;            // T_TOT
constexpr int GMAX = 20000;       // GLOBAL_MAX_SIZE_OF_CODEWORD
constexpr int SLOT = GMAX + 16;
constexpr int L = 300;

// The reference object restated over its members with the oracle's methods (test side only).
struct OracleSW {
    int max_payload;
    unsigned char** codeword_vector;
    unsigned char** codeword_new_vector;
    unsigned char** codeword_vector_to_transmit;
    unsigned char** codeword_vector_state_dependent;
    bool* temp_erasure_vector_state_dependent;
    int** header;
    unsigned char codeword_new_symbol_wise[30000];
    bool* temp_erasure_vector;
    Decoder* decoder_current = nullptr;
    Encoder* encoder_current = nullptr;
    static unsigned char** slots(int c) {
        unsigned char** v = static_cast<unsigned char**>(std::calloc(c, sizeof(void*)));
        for (int i = 0; i < c; ++i) v[i] = static_cast<unsigned char*>(std::calloc(SLOT, 1));
        return v;
    }
    explicit OracleSW(int mp) : max_payload(mp) {
        codeword_vector = slots(TT + 1);
        codeword_new_vector = slots(TT + 1);
        codeword_vector_to_transmit = slots(TT + 1);
        codeword_vector_state_dependent = slots(3 * TT);
        temp_erasure_vector = static_cast<bool*>(std::calloc(TT + 1, 1));
        temp_erasure_vector_state_dependent = static_cast<bool*>(std::calloc(3 * TT, 1));
        header = static_cast<int**>(std::calloc(3 * TT, sizeof(int*)));
        for (int i = 0; i < 3 * TT; ++i) {
            header[i] = static_cast<int*>(std::calloc(TT + 1, sizeof(int)));
            for (int j = 0; j < TT + 1; ++j) header[i][j] = j + 1;
        }
        std::memset(codeword_new_symbol_wise, 0, sizeof(codeword_new_symbol_wise));
    }
    ~OracleSW() {
        for (int i = 0; i < TT + 1; ++i) {
            std::free(codeword_vector[i]);
            std::free(codeword_new_vector[i]);
            std::free(codeword_vector_to_transmit[i]);
        }
        for (int i = 0; i < 3 * TT; ++i) {
            std::free(codeword_vector_state_dependent[i]);
            std::free(header[i]);
        }
        std::free(codeword_vector);
        std::free(codeword_new_vector);
        std::free(codeword_vector_to_transmit);
        std::free(codeword_vector_state_dependent);
        std::free(header);
        std::free(temp_erasure_vector);
        std::free(temp_erasure_vector_state_dependent);
        delete decoder_current;
        delete encoder_current;
    }
    // rows [0, m-1) take the contents of rows [1, m), row m-1 keeps its own: as the reference's
    // memcpy loop, by moving the row pointers and copying only the last row's GMAX bytes once
    static void shift_rows(unsigned char** v, int m) {
        if (m < 2) return;
        unsigned char* p0 = v[0];
        for (int i = 0; i < m - 1; ++i) v[i] = v[i + 1];
        std::memcpy(p0, v[m - 1], GMAX);
        v[m - 1] = p0;
    }
    void shift(int n, int n2) {  // Decoder_Symbol_Wise.cpp:120-135
        shift_rows(codeword_vector, n);
        for (int i = 0; i < n - 1; ++i) temp_erasure_vector[i] = temp_erasure_vector[i + 1];
        shift_rows(codeword_new_vector, n2);
        shift_rows(codeword_vector_to_transmit, n2);
        shift_rows(codeword_vector_state_dependent, 3 * TT);
        for (int i = 0; i < 3 * TT - 1; ++i) {
            std::memcpy(header[i], header[i + 1], sizeof(int) * TT);  // (entry TT stays with its row)
            temp_erasure_vector_state_dependent[i] = temp_erasure_vector_state_dependent[i + 1];
        }
    }
    void push_current_codeword(unsigned char* m, int n, int n2, int, int) {
        shift(n, n2);
        std::memcpy(&codeword_vector[n - 1][2], m, GMAX);
        temp_erasure_vector[n - 1] = false;
    }
    void rotate_pointers_and_insert_zero_word(int n, int n2, int, int, bool) {
        shift(n, n2);
        std::memset(codeword_vector[n - 1], 0, GMAX);
        temp_erasure_vector[n - 1] = true;
    }
    void symbol_wise_encode_1(int k, int n, int k2, int n2, bool* flag) {
        int f = 0;
        or_sw_encode_1(max_payload, k, n, k2, n2, codeword_vector, reinterpret_cast<uint8_t*>(temp_erasure_vector),
                       codeword_new_vector, codeword_new_symbol_wise, &f);
        *flag = f != 0;
    }
    void symbol_wise_decode_1(unsigned char* buffer, bool* flag, int k, int n) {
        int f = 0;
        or_sw_decode_1(max_payload, k, n, codeword_vector, reinterpret_cast<uint8_t*>(temp_erasure_vector), buffer, &f);
        *flag = f != 0;
    }
    void symbol_wise_encode_state_dependent(int k, int n, int k2, int n2, bool* flag) {
        *flag = false;
        or_sw_state_encode(max_payload, k, n, k2, n2, 0, codeword_vector_state_dependent,
                           reinterpret_cast<uint8_t*>(temp_erasure_vector_state_dependent), header,
                           codeword_new_vector[n2 - 1], codeword_new_symbol_wise);
    }
    void symbol_wise_decode_state_dependent(unsigned char* buffer, bool* flag, int k, int n) {
        int f = 0;
        or_sw_state_decode(max_payload, k, n, codeword_vector_state_dependent, header, buffer, &f);
        *flag = f != 0;
    }
    void extract_data(unsigned char* buffer, int k, int n, int, unsigned char* temp_buffer) {
        const int blocks = max_payload / k + 1;
        int ind = 0;
        for (int j = 0; j < blocks; ++j)
            for (int i = 0; i < k; ++i) temp_buffer[ind++] = buffer[j * n + n - k + i];
    }
    void copy_elements(OracleSW* s, bool encode) {  // :88-117
        for (int i = 0; i < TT + 1; ++i) {
            std::memcpy(codeword_vector[i], s->codeword_vector[i], GMAX);
            std::memcpy(codeword_new_vector[i], s->codeword_new_vector[i], GMAX);
            std::memcpy(codeword_vector_to_transmit[i], s->codeword_vector_to_transmit[i], GMAX);
            temp_erasure_vector[i] = s->temp_erasure_vector[i];
        }
        for (int i = 0; i < 3 * TT; ++i) {
            std::memcpy(codeword_vector_state_dependent[i], s->codeword_vector_state_dependent[i], GMAX);
            std::memcpy(header[i], s->header[i], sizeof(int) * (TT + 1));
            temp_erasure_vector_state_dependent[i] = s->temp_erasure_vector_state_dependent[i];
        }
        delete decoder_current;
        decoder_current = new Decoder(s->decoder_current->T, s->decoder_current->B, s->decoder_current->N, s->max_payload);
        if (encode) {
            delete encoder_current;
            encoder_current = new Encoder(s->encoder_current->T, s->encoder_current->B, s->encoder_current->N,
                                          s->max_payload);
        }
    }
};

// --time mode: wall time per seq of each node's object calls, split into the slot shifts of
// push_current_codeword / rotate_pointers_and_insert_zero_word and the GF call of the type
struct CallClock {
    double relay_shift = 0, relay_gf = 0, dest_shift = 0, dest_gf = 0;
};
CallClock g_clock;
double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// A relayed code: the source's (n, k) on hop 1, the relay's (n2, k) on hop 2 (T2 = n2 - 1 <= T).
struct Code {
    int k, n, n2, S, CW;
};
Code code(int T, int N, int T2 = -1) {
    Code c{T - N + 1, T + 1, (T2 < 0 ? T : T2) + 1, 0, 0};
    c.S = (L + 2 + c.k - 1) / c.k;
    c.CW = c.S * c.n;
    return c;
}
int rd_size(const Code& c) { return (c.S + 1) * c.n2; }  // codeword_r_d_size (:997-999), k2 == k

// One node's relay step for one code (an object, a codeword or nullptr = erased): the object calls
// of :1051-1062 / :1459-1467, then the code's part of the frame appended to `frame`.
template <class SW>
void relay_step(SW* w, int R, const Code& c, const unsigned char* cw, std::vector<unsigned char>& frame) {
    static std::vector<unsigned char> buf(SLOT);
    bool flag = false;
    const double t0 = now_us();
    if (cw) {
        std::memset(buf.data(), 0, SLOT);
        std::memcpy(buf.data(), cw, c.CW);
        w->push_current_codeword(buf.data(), c.n, c.n2, c.CW, rd_size(c));
        if (R == 3) {
            std::memcpy(&w->codeword_vector_state_dependent[2 * TT][2], buf.data(), GMAX);
            w->temp_erasure_vector_state_dependent[2 * TT] = false;
        }
    } else {
        w->rotate_pointers_and_insert_zero_word(c.n, c.n2, 0, 0, true);
        if (R == 3) {
            std::memset(w->codeword_vector_state_dependent[2 * TT], 0, GMAX);
            w->temp_erasure_vector_state_dependent[2 * TT] = true;
        }
    }
    const double t1 = now_us();
    if (R == 3) w->symbol_wise_encode_state_dependent(c.k, c.n, c.k, c.n2, &flag);
    else w->symbol_wise_encode_1(c.k, c.n, c.k, c.n2, &flag);
    const double t2 = now_us();
    g_clock.relay_shift += t1 - t0;
    g_clock.relay_gf += t2 - t1;
    if (R == 3)
        for (int a = 0; a < TT + 1; ++a) frame.push_back(static_cast<unsigned char>(w->header[c.n2 - 1][a]));
    const unsigned char* row = w->codeword_new_vector[c.n2 - 1];
    frame.insert(frame.end(), row, row + rd_size(c));
}

// The destination's step for one code (:1703-1721 missing, :1798-1815 received): part = the
// code's frame part ([header 11]? [codeword_new_vector row]) or nullptr; out = blocks*k bytes.
template <class SW>
int dest_step(SW* d, int R, const Code& c, const unsigned char* part, unsigned char* out) {
    static std::vector<unsigned char> buf(SLOT), buffer(30000);
    bool flag = false;
    const double t0 = now_us();
    if (part) {
        const unsigned char* cw = part + (R == 3 ? TT + 1 : 0);
        std::memset(buf.data(), 0, SLOT);
        std::memcpy(buf.data(), cw, rd_size(c));
        d->push_current_codeword(buf.data(), c.n2, 0, rd_size(c), 0);
        if (R == 3) {
            for (int i = 0; i < TT + 1; ++i) d->header[3 * TT - 1][i] = part[i];
            std::memcpy(&d->codeword_vector_state_dependent[3 * TT - 1][2], buf.data(), GMAX);
            d->temp_erasure_vector_state_dependent[3 * TT - 1] = false;
        }
    } else {
        d->rotate_pointers_and_insert_zero_word(c.n2, 0, 0, 0, false);
        if (R == 3) {
            for (int i = 0; i < TT + 1; ++i) d->header[3 * TT - 1][i] = 0;
            std::memset(d->codeword_vector_state_dependent[3 * TT - 1], 0, GMAX);
            d->temp_erasure_vector_state_dependent[3 * TT - 1] = true;
        }
    }
    const double t1 = now_us();
    if (R == 3) d->symbol_wise_decode_state_dependent(buffer.data(), &flag, c.k, c.n2);
    else d->symbol_wise_decode_1(buffer.data(), &flag, c.k, c.n2);
    const double t2 = now_us();
    g_clock.dest_shift += t1 - t0;
    g_clock.dest_gf += t2 - t1;
    d->extract_data(buffer.data(), c.k, c.n2, 0, out);
    return flag ? 1 : 0;
}

struct Trace {
    std::vector<std::vector<unsigned char>> frames;
    std::vector<std::vector<unsigned char>> outs;
    std::vector<int> flags;
};

// A code schedule: entry i's source code (T_i, N_i, N_i) starts at seq s_i (s_0 = 0, and
// s_{i+1} >= s_i + T_TOT + 1: the encoder double codes the T_TOT + 1 packets from a switch,
// Variable_Rate_FEC_Encoder.cpp:74-235, and cannot switch again before that ends).
struct Switch {
    int seq, T, N;
};

// The chain: per seq t the source encoder(s) of the schedule, hop-1 erasures e1 (both codewords of
// a seq are lost together), the relay, hop-2 erasures e2, the destination.  During double coding
// the relay runs two objects -- the old code's and a new one for the new code (:1437-1456) -- and
// sends [BE16 size_cur][new code's part][old code's part] (:1502-1571); the destination's old
// object reports, the new one decodes the new part (:1823-1873); at the end both nodes copy the
// new object into the main one (copy_elements, :1423-1433).  Th2 >= 0: the hop-2 code of a
// one-entry schedule (n2 = Th2 + 1 <= n).
template <class SW>
Trace chain(int R, const std::vector<Switch>& sched, int Th2, int P, const std::vector<unsigned char>& e1,
            const std::vector<unsigned char>& e2) {
    const int ns = static_cast<int>(sched.size());
    std::vector<Code> codes;
    for (int i = 0; i < ns; ++i) codes.push_back(code(sched[i].T, sched[i].N, ns == 1 ? Th2 : -1));
    auto mk = [&](int i, bool with_encoder) {
        SW* w = new SW(L);
        const Code& c = codes[static_cast<size_t>(i)];
        w->decoder_current = new Decoder(c.n - 1, c.n - c.k, c.n - c.k, L);
        if (with_encoder) w->encoder_current = new Encoder(c.n - 1, c.n - c.k, c.n - c.k, L);
        return w;
    };
    std::vector<or_encoder*> enc(static_cast<size_t>(ns), nullptr);
    enc[0] = or_encoder_new(L, sched[0].T, sched[0].N, sched[0].N);
    SW* relay = mk(0, true);
    SW* relay_new = nullptr;
    SW* dest = mk(0, false);
    SW* dest_new = nullptr;
    int ci = 0;  // the schedule entry of the newest code
    std::vector<unsigned char> payload(L), cwo(8192), cwn(8192);
    Trace tr;
    for (int t = 0; t < P; ++t) {
        if (ci + 1 < ns && t == sched[static_cast<size_t>(ci) + 1].seq) {  // a switch: new objects
            ++ci;
            enc[static_cast<size_t>(ci)] = or_encoder_new(L, sched[ci].T, sched[ci].N, sched[ci].N);
            relay_new = mk(ci, true);
            dest_new = mk(ci, false);
        }
        const int s0 = sched[static_cast<size_t>(ci)].seq;
        if (ci > 0 && t == s0 + TT + 1) {  // end of double coding: the new objects take over
            relay->copy_elements(relay_new, true);
            dest->copy_elements(dest_new, false);
            delete relay_new;
            delete dest_new;
            relay_new = dest_new = nullptr;
            or_encoder_free(enc[static_cast<size_t>(ci) - 1]);
            enc[static_cast<size_t>(ci) - 1] = nullptr;
        }
        const bool dc = ci > 0 && t <= s0 + TT;  // seq_end_double_coding = start + T_TOT (:1438)
        const Code& c_new = codes[static_cast<size_t>(ci)];
        const Code& c_old = codes[static_cast<size_t>(dc ? ci - 1 : ci)];
        or_fill_payload(payload.data(), t, 1, L, 0x5EED);
        or_encoder_transmit(enc[static_cast<size_t>(ci)], payload.data(), L, t, cwn.data());
        if (dc) or_encoder_transmit(enc[static_cast<size_t>(ci) - 1], payload.data(), L, t, cwo.data());
        const bool lost1 = e1[t] != 0;
        std::vector<unsigned char> frame(2);
        int size_cur;
        if (dc) {  // the old code's object gets the old codeword, the new one the new
            std::vector<unsigned char> pn, po;
            relay_step(relay_new, R, c_new, lost1 ? nullptr : cwn.data(), pn);
            relay_step(relay, R, c_old, lost1 ? nullptr : cwo.data(), po);
            size_cur = rd_size(c_new);
            frame.insert(frame.end(), pn.begin(), pn.end());
            frame.insert(frame.end(), po.begin(), po.end());
        } else {
            std::vector<unsigned char> pc;
            relay_step(relay, R, c_new, lost1 ? nullptr : cwn.data(), pc);
            size_cur = rd_size(c_new);
            frame.insert(frame.end(), pc.begin(), pc.end());
        }
        frame[0] = static_cast<unsigned char>(size_cur / 256);
        frame[1] = static_cast<unsigned char>(size_cur % 256);
        const bool lost2 = e2[t] != 0;
        const int hdr = R == 3 ? TT + 1 : 0;
        std::vector<unsigned char> out(static_cast<size_t>(L + 32), 0);
        int flag;
        if (dc) {
            const unsigned char* pn = lost2 ? nullptr : frame.data() + 2;
            const unsigned char* po = lost2 ? nullptr : frame.data() + 2 + hdr + size_cur;
            flag = dest_step(dest, R, c_old, po, out.data());
            std::vector<unsigned char> tmp(static_cast<size_t>(L + 32), 0);
            dest_step(dest_new, R, c_new, pn, tmp.data());
        } else {
            flag = dest_step(dest, R, c_new, lost2 ? nullptr : frame.data() + 2, out.data());
        }
        tr.frames.push_back(frame);
        tr.outs.push_back(out);
        tr.flags.push_back(flag);
    }
    for (auto* e : enc)
        if (e) or_encoder_free(e);
    delete relay;
    delete relay_new;
    delete dest;
    delete dest_new;
    return tr;
}

std::vector<unsigned char> pattern(int P, unsigned seed, int per_mille, int burst_every) {
    std::vector<unsigned char> e(P, 0);
    unsigned s = seed;
    for (int t = 0; t < P; ++t) {
        s = s * 1103515245u + 12345u;
        if (static_cast<int>((s >> 16) % 1000) < per_mille) e[t] = 1;
        if (burst_every && t % burst_every >= 40 && t % burst_every < 43) e[t] = 1;
    }
    return e;
}

int compare(const char* what, const Trace& a, const Trace& b, int P) {
    for (int t = 0; t < P; ++t) {
        if (a.frames[t] != b.frames[t]) {
            std::printf("%s: frame %d differs (%zu vs %zu bytes)\n", what, t, a.frames[t].size(), b.frames[t].size());
            return 1;
        }
        if (a.outs[t] != b.outs[t] || a.flags[t] != b.flags[t]) {
            std::printf("%s: destination output %d differs (flag %d vs %d)\n", what, t, a.flags[t], b.flags[t]);
            return 1;
        }
    }
    return 0;
}

// (1) a fixed-rate chain over SW against the oracle's own chain functions
template <class SW>
int fixed_vs_oracle_run(int R, int T1, int N1, int T2, int N2, int P) {
    const auto e1 = pattern(P, 7, 30, 173), e2 = pattern(P, 11, 25, 211);
    const Trace d = chain<SW>(R, {{0, T1, N1}}, T2, P, e1, e2);
    const Code c = code(T1, N1, T2);
    const int F = 2 + (R == 3 ? TT + 1 : 0) + rd_size(c);
    std::vector<unsigned char> frames(static_cast<size_t>(P) * F), out(static_cast<size_t>(P) * c.S * c.k),
        rf(P), df(P);
    const int st = R == 3 ? or_sdswdf_run(L, T1, N1, T2, N2, P, e1.data(), e2.data(), 0x5EED, 0, frames.data(),
                                          out.data(), df.data())
                          : or_swdf_run(L, T1, N1, T2, N2, P, e1.data(), e2.data(), 0x5EED, frames.data(), rf.data(),
                                        out.data(), df.data());
    if (st) {
        std::printf("oracle chain failed\n");
        return 1;
    }
    const int blocks = L / c.k + 1;
    for (int t = 0; t < P; ++t) {
        if (d.frames[t].size() != static_cast<size_t>(F) || std::memcmp(d.frames[t].data(), &frames[size_t(t) * F], F)) {
            std::printf("type %d (%d,%d): frame %d differs from the oracle chain\n", R, T1, N1, t);
            return 1;
        }
        if (std::memcmp(d.outs[t].data(), &out[size_t(t) * c.S * c.k], blocks * c.k) || d.flags[t] != df[t]) {
            std::printf("type %d (%d,%d): destination %d differs from the oracle chain\n", R, T1, N1, t);
            return 1;
        }
    }
    std::printf("type %d (%d,%d)->(%d,%d) fixed rate: %d seqs equal to the oracle chain\n", R, T1, N1, T2, N2, P);
    return 0;
}

#ifndef RELAY_ORACLE_ONLY
// (2) double coding: the same driver over the drop-in and over OracleSW
int double_coding(int R, int T1, int N1, int T2, int N2, int s0, int P) {
    const auto e1 = pattern(P, 5, 20, 149), e2 = pattern(P, 9, 20, 0);
    const Trace d = chain<siphon::Decoder_Symbol_Wise>(R, {{0, T1, N1}, {s0, T2, N2}}, -1, P, e1, e2);
    const Trace o = chain<OracleSW>(R, {{0, T1, N1}, {s0, T2, N2}}, -1, P, e1, e2);
    char what[96];
    std::snprintf(what, sizeof what, "type %d (%d,%d)=>(%d,%d) at %d", R, T1, N1, T2, N2, s0);
    if (compare(what, d, o, P)) return 1;
    int good = 0;
    for (int t = 0; t < P; ++t) good += d.flags[t] == 0;
    std::printf("%s: %d seqs equal (double coding %d..%d), %d unflagged\n", what, P, s0, s0 + TT, good);
    return 0;
}
#endif
}  // namespace

// (3) a schedule from files: argv = --schedule <sched.txt> <e1.bin> <e2.bin>; sched.txt = "P" then
// one "seq T N" line per switch (the first at seq 0); e1 / e2 = P hop erasure bytes.  Types 2 and
// 3 over SW and over OracleSW (or over OracleSW alone, ref == nullptr: CPU build).
std::vector<unsigned char> read_bytes(const char* path, int P) {
    std::vector<unsigned char> v(static_cast<size_t>(P), 0);
    FILE* f = std::fopen(path, "rb");
    if (!f || std::fread(v.data(), 1, v.size(), f) != v.size()) {
        std::printf("cannot read %d bytes from %s\n", P, path);
        std::exit(2);
    }
    std::fclose(f);
    return v;
}
// CRC-32 (IEEE, zlib's) of the seqs' [frame_len LE32][frame][out][flag], per block of kDigestBlock
// seqs: the digest a product run (fec_relay_vr) is compared with (tests/golden/relay_vr_360k.json).
constexpr int kDigestBlock = 100;
uint32_t crc32_update(uint32_t c, const unsigned char* p, size_t n) {
    static uint32_t tab[256];
    static bool init = false;
    if (!init) {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t x = i;
            for (int b = 0; b < 8; ++b) x = (x & 1) ? 0xEDB88320u ^ (x >> 1) : x >> 1;
            tab[i] = x;
        }
        init = true;
    }
    c = ~c;
    for (size_t i = 0; i < n; ++i) c = tab[(c ^ p[i]) & 0xff] ^ (c >> 8);
    return ~c;
}
void write_digest(FILE* f, int R, const Trace& d, int P) {
    int good = 0;
    for (int fl : d.flags) good += fl == 0;
    std::fprintf(f, "type %d P %d unflagged %d\n", R, P, good);
    for (int b0 = 0; b0 < P; b0 += kDigestBlock) {
        uint32_t c = 0;
        for (int t = b0; t < std::min(P, b0 + kDigestBlock); ++t) {
            const uint32_t fl = static_cast<uint32_t>(d.frames[t].size());
            const unsigned char le[4] = {static_cast<unsigned char>(fl), static_cast<unsigned char>(fl >> 8),
                                         static_cast<unsigned char>(fl >> 16), static_cast<unsigned char>(fl >> 24)};
            c = crc32_update(c, le, 4);
            c = crc32_update(c, d.frames[t].data(), d.frames[t].size());
            c = crc32_update(c, d.outs[t].data(), d.outs[t].size());
            const unsigned char f1 = static_cast<unsigned char>(d.flags[t]);
            c = crc32_update(c, &f1, 1);
        }
        std::fprintf(f, "%08x\n", c);
    }
}

template <class SW>
int schedule_run(int argc, char** argv, bool compare_with_oracle) {
    if (argc < 5) return 2;
    FILE* dig = nullptr;  // --schedule s e1 e2 --digest out.txt: per-block digests of each type's trace
    if (argc >= 7 && std::strcmp(argv[5], "--digest") == 0) dig = std::fopen(argv[6], "w");
    FILE* f = std::fopen(argv[2], "r");
    int P = 0;
    if (!f || std::fscanf(f, "%d", &P) != 1) return 2;
    std::vector<Switch> sched;
    Switch w;
    while (std::fscanf(f, "%d %d %d", &w.seq, &w.T, &w.N) == 3) sched.push_back(w);
    std::fclose(f);
    const auto e1 = read_bytes(argv[3], P), e2 = read_bytes(argv[4], P);
    int rc = 0;
    for (int R : {2, 3}) {
        const Trace d = chain<SW>(R, sched, -1, P, e1, e2);
        int good = 0;
        for (int fl : d.flags) good += fl == 0;
        if (dig) write_digest(dig, R, d, P);
        if (compare_with_oracle) {
            const Trace o = chain<OracleSW>(R, sched, -1, P, e1, e2);
            char what[64];
            std::snprintf(what, sizeof what, "type %d schedule", R);
            if (compare(what, d, o, P)) {
                rc = 1;
                continue;
            }
        }
        std::printf("type %d schedule: %zu codes, %d seqs%s, %d unflagged\n", R, sched.size(), P,
                    compare_with_oracle ? " equal to the oracle methods" : "", good);
    }
    if (dig) std::fclose(dig);
    return rc;
}

// --time P: the fixed-rate (10,3) chain over SW for P seqs, per type; prints microseconds per seq
// of the relay's and the destination's object calls (slot shifts, GF call)
template <class SW>
void time_run(const char* what, int P) {
    const auto e1 = pattern(P, 7, 30, 173), e2 = pattern(P, 11, 25, 211);
    for (int R : {2, 3}) {
        chain<SW>(R, {{0, 10, 3}}, -1, 64, e1, e2);  // warm-up: contexts, planners, device buffers
        g_clock = CallClock{};
        const double t0 = now_us();
        chain<SW>(R, {{0, 10, 3}}, -1, P, e1, e2);
        const double total = now_us() - t0;
        std::printf("{\"class\": \"%s\", \"type\": %d, \"seqs\": %d, \"us_per_seq\": {\"relay_shift\": %.2f, "
                    "\"relay_gf\": %.2f, \"dest_shift\": %.2f, \"dest_gf\": %.2f, \"chain\": %.2f}}\n",
                    what, R, P, g_clock.relay_shift / P, g_clock.relay_gf / P, g_clock.dest_shift / P,
                    g_clock.dest_gf / P, total / P);
    }
}

#ifdef RELAY_ORACLE_ONLY
// CPU build (tests/test_sdswdf.py): the driver over OracleSW against the oracle's chains, which
// checks the driver and the or_sw_* methods without a GPU.
int main(int argc, char** argv) {
    if (argc > 2 && std::strcmp(argv[1], "--time") == 0) {
        time_run<OracleSW>("oracle", std::atoi(argv[2]));
        return 0;
    }
    if (argc > 1 && std::strcmp(argv[1], "--schedule") == 0) {
        const int rc = schedule_run<OracleSW>(argc, argv, false);
        if (rc == 0) std::printf("RELAY ORACLE DRIVER OK\n");
        return rc;
    }
    int rc = 0;
    rc |= fixed_vs_oracle_run<OracleSW>(3, 10, 3, 10, 3, 600);
    rc |= fixed_vs_oracle_run<OracleSW>(3, 10, 5, 8, 3, 400);
    rc |= fixed_vs_oracle_run<OracleSW>(2, 10, 3, 10, 3, 600);
    rc |= fixed_vs_oracle_run<OracleSW>(2, 10, 1, 10, 1, 400);
    for (int R : {2, 3}) {  // the double-coding driver runs (memory-clean under -fsanitize) over OracleSW
        const Trace o = chain<OracleSW>(R, {{0, 10, 3}, {200, 10, 5}}, -1, 420, pattern(420, 5, 20, 149), pattern(420, 9, 20, 0));
        int good = 0;
        for (int f : o.flags) good += f == 0;
        std::printf("type %d double coding over OracleSW: %d of 420 unflagged\n", R, good);
        if (good < 300) rc = 1;
    }
    if (rc == 0) std::printf("RELAY ORACLE DRIVER OK\n");
    return rc;
}
#else
int main(int argc, char** argv) {
    using DSW = siphon::Decoder_Symbol_Wise;
    if (argc > 2 && std::strcmp(argv[1], "--time") == 0) {
        time_run<DSW>("dropin", std::atoi(argv[2]));
        time_run<OracleSW>("oracle", std::atoi(argv[2]));
        return 0;
    }
    if (argc > 1 && std::strcmp(argv[1], "--schedule") == 0) {
        const int rc = schedule_run<DSW>(argc, argv, true);
        if (rc == 0) std::printf("RELAY DROPIN OK\n");
        return rc;
    }
    int rc = 0;
    rc |= fixed_vs_oracle_run<DSW>(3, 10, 3, 10, 3, 600);
    rc |= fixed_vs_oracle_run<DSW>(3, 10, 5, 8, 3, 400);
    rc |= fixed_vs_oracle_run<DSW>(2, 10, 3, 10, 3, 600);
    rc |= fixed_vs_oracle_run<DSW>(2, 10, 1, 10, 1, 400);
    rc |= double_coding(3, 10, 3, 10, 5, 200, 420);
    rc |= double_coding(2, 10, 3, 10, 5, 200, 420);
    rc |= double_coding(3, 10, 5, 10, 1, 150, 380);
    if (rc == 0) std::printf("RELAY DROPIN OK\n");
    return rc;
}
#endif
