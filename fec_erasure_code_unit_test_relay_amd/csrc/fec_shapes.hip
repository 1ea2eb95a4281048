// fec_shapes.hip -- the decode planner's first launch: resync points, loss episodes and their
// shapes, erased outputs, in one pass over the erasure flags.
//
// An episode starts at an erased packet tr with no erasure in [tr-T-1, tr-1] (the decoder's
// resynchronisation, Decoder.cpp:109-133) and ends at the first received packet t with no erasure
// in [t-T, t-1] (Decoder.cpp:80-83): packet latest+T+1 ends it only if it is received, an
// erasure there continues the episode.  Every erased packet lies in exactly one episode.
// Everything the planner derives for the episode's erased packets -- which symbols are recovered
// and their coefficient rows -- is a function of the block states at tr and of the erasure flags
// inside the episode.  For tr >= T the block state at tr is the post-resync state of the block's
// phase, and the phase of the block holding symbol i of packet x is (tr - x + i) mod n: the
// results depend on x - tr, not on tr.  Two episodes with the same erasure shape (bit j = packet
// tr+j erased) therefore have identical results at equal offsets.
//
// fec_episode_kernel (16 packets per lane, 1024 per wave):
//   * erased output packets -> `erased` (one atomic per wave), src_d[x] = 0;
//   * each resync point tr found by a thread: the thread walks the episode (flags in 64-packet
//     windows) to its shape and last erasure, and inserts keyable shapes (tr >= T, span < 64, not
//     running into the batch end) into the hash table `keys` (relaxed load first, CAS on a miss);
//     the winner of a shape records its tr in reps_tr and goes to the replay list `work` with every
//     unkeyed episode; the others go to `dups` as (tr, slot).
// The plan kernels (fec_plan_fast.hip / fec_kernels.hip) replay `work` and, for each entry of
// `dups`, point src_d of its erased packets at the representative's (x + reps_tr - tr): the
// recovery reads the representative's rows there, so nothing is copied.
#include "fec_device.h"
#include "fec_kernels.h"

namespace fec {

namespace {

__device__ __forceinline__ uint32_t shape_hash(uint64_t m, int bits) {
    return static_cast<uint32_t>((m * 0x9E3779B97F4A7C15ull) >> (64 - bits));
}

// Erasure flags of packets t0 .. t0+63 as bits (bit j = packet t0+j erased; past P: 0).  Nine
// aligned 8-byte loads instead of 64 byte loads.
__device__ __forceinline__ uint64_t erasure_bits64(const uint8_t* er, int64_t P, int64_t t0) {
    uint64_t fl = 0;
    const uintptr_t ad = reinterpret_cast<uintptr_t>(er + t0);
    const uintptr_t a0 = ad & ~uintptr_t(7);  // the nine words cover [a0, a0 + 72) inside er[0, P)
    if (t0 >= 8 && t0 + 72 <= P) {
        const int sh = static_cast<int>(ad - a0) * 8;
        const uint64_t* p = reinterpret_cast<const uint64_t*>(a0);
        uint64_t w[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) w[i] = p[i];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint64_t x = sh ? ((w[i] >> sh) | (w[i + 1] << (64 - sh))) : w[i];
            // byte != 0 -> 0x01, then bit b of the result = byte b
            const uint64_t nz = ((((x & 0x7F7F7F7F7F7F7F7Full) + 0x7F7F7F7F7F7F7F7Full) | x) >> 7) & 0x0101010101010101ull;
            fl |= ((nz * 0x0102040810204080ull) >> 56) << (8 * i);
        }
    } else {
        for (int j = 0; j < 64; ++j) {
            const int64_t t = t0 + j;
            if (t >= 0 && t < P && er[t]) fl |= uint64_t(1) << j;
        }
    }
    return fl;
}

__device__ __forceinline__ uint32_t nz_bytes_mask(uint32_t w) {  // bit e: byte e of w non-zero
    return (((w & 0xffu) != 0) ? 1u : 0u) | (((w & 0xff00u) != 0) ? 2u : 0u) |
           (((w & 0xff0000u) != 0) ? 4u : 0u) | (((w & 0xff000000u) != 0) ? 8u : 0u);
}

__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(v, o);
        if (lane >= o) v += y;
    }
    return v;
}

// Wave-aggregated append of `n` items for the lanes where n > 0; returns the lane's first index.
__device__ __forceinline__ int wave_reserve(int n, int32_t* counter) {
    const int lane = threadIdx.x & 63;
    const int incl = wave_incl_scan(n, lane);
    const int tot = __shfl(incl, 63);
    if (tot == 0) return 0;
    int base = 0;
    if (lane == 63) base = atomicAdd(counter, tot);
    base = __shfl(base, 63);
    return base + incl - n;
}

}  // namespace

// One wave per workgroup, kLanePk = 16 packets per lane, 1024 per wave and pass: a wave's episode
// rounds (one per resync point of its busiest lane, each a walk, a table probe and an append) are
// at most 16 / (T + 2) + 1 instead of 64 / (T + 2) + 1, and the launch has four times the waves
// (config 3, 360 000 packets: 88 waves of 4096 took 26 us).  Device-scope atomics are
// performed beyond the XCDs' L2s and serialise per address, so a wave issues few of them: one for
// its erased outputs, one 64-bit one per round for its replay and duplicate entries; the shape
// table is probed with plain loads (a key never changes once set, so a stale line can only read
// as empty, and the CAS that follows returns the real key) by one lane per distinct shape of the
// wave.
__global__ __launch_bounds__(64) void fec_episode_kernel(EpisodeArgs a) {
    const int lane = threadIdx.x;
    const int T = a.T;  // < 64 (host check): the look-back of a resync test fits one word
    const int64_t TS = int64_t(1) << a.tbits;
    constexpr int kLanePk = 16;
    constexpr int64_t kPerWave = 64 * kLanePk;
    unsigned long long* wd = reinterpret_cast<unsigned long long*>(a.counters + 6);  // (replayed, dups)
    phase_stamp(a.stamps, blockIdx.x, 0);
    for (int64_t w0 = static_cast<int64_t>(blockIdx.x) * kPerWave; w0 < a.P;
         w0 += static_cast<int64_t>(gridDim.x) * kPerWave) {
        const int64_t t0 = w0 + lane * kLanePk;
        uint64_t m64 = 0;  // bit e: packet t0+e erased (e < kLanePk)
        if (t0 + kLanePk - 1 < a.P && (reinterpret_cast<uintptr_t>(a.er + t0) & 15) == 0) {
            const uint4 v = *reinterpret_cast<const uint4*>(a.er + t0);
            m64 = nz_bytes_mask(v.x) | (nz_bytes_mask(v.y) << 4) | (nz_bytes_mask(v.z) << 8) | (nz_bytes_mask(v.w) << 12);
        } else if (t0 < a.P) {
            m64 = erasure_bits64(a.er, a.P, t0) & ((uint64_t(1) << kLanePk) - 1u);
        }
        // resync points: erased t with no erasure in [t-T-1, t-1] (Decoder.cpp:80-83, 109-133)
        uint64_t resm = 0;
        // packets t0-64 .. t0-1: the four lanes below (shuffled with every lane active) and, for
        // lanes 0..3, the word in front of them
        const uint64_t b1 = __shfl_up(m64, 1), b2 = __shfl_up(m64, 2), b3 = __shfl_up(m64, 3), b4 = __shfl_up(m64, 4);
        if (m64) {
            const uint64_t bw = lane < 4 ? erasure_bits64(a.er, a.P, t0 - 64)
                                         : (b4 | (b3 << 16) | (b2 << 32) | (b1 << 48));
            for (uint64_t rest = m64; rest; rest &= rest - 1) {
                const int e = __builtin_ctzll(rest);
                const int lo = e - T - 1;
                uint64_t inside = m64 & ((uint64_t(1) << e) - 1u);
                if (lo > 0) inside &= ~((uint64_t(1) << lo) - 1u);
                const bool rs = inside == 0 && (lo >= 0 || (bw >> (64 + lo)) == 0);
                if (rs) resm |= uint64_t(1) << e;
            }
        }
        phase_stamp(a.stamps, blockIdx.x, 1);
        // erased outputs (src_d: own plan rows until the plan says otherwise)
        uint64_t outm = m64;
        if (t0 + kLanePk > a.Pout) outm &= (t0 >= a.Pout) ? 0u : ((uint64_t(1) << (a.Pout - t0)) - 1u);
        int so = wave_reserve(__builtin_popcountll(outm), &a.counters[1]);
        for (uint64_t rest = outm; rest; rest &= rest - 1) {
            const int64_t x = t0 + __builtin_ctzll(rest);
            a.erased[so++] = static_cast<int32_t>(x);
            a.src_d[x] = 0;
        }
        phase_stamp(a.stamps, blockIdx.x, 2);

        // episodes of this lane, one per round (wave-uniform loop)
        uint64_t rest = resm;
        while (__builtin_amdgcn_ballot_w64(rest != 0)) {
            const bool have = rest != 0;
            int64_t tr = 0;
            uint64_t m = 1;
            bool keyed = false;
            if (have) {
                tr = t0 + __builtin_ctzll(rest);
                rest &= rest - 1;
                // walk the episode: positions relative to tr, flags in windows of 64
                int latest = 0;
                bool big = false, done = false, truncated = false;
                for (int base = 1; !done; base += 64) {
                    uint64_t fl = erasure_bits64(a.er, a.P, tr + base);
                    while (fl) {
                        const int j = __builtin_ctzll(fl);
                        fl &= fl - 1;
                        const int pos = base + j;
                        if (pos - latest > T + 1) {  // packet latest+T+1 was received: ended
                            done = true;
                            break;
                        }
                        latest = pos;
                        if (pos < 64) m |= uint64_t(1) << pos;
                        else big = true;
                    }
                    if (!done && latest + T + 1 <= base + 63) done = true;  // latest+T+1 seen, received
                    if (!done && tr + base + 64 >= a.P) {
                        done = true;
                        truncated = true;
                    }
                }
                keyed = a.dedup && tr >= T && !big && !truncated && tr + latest + T + 1 < a.P;
            }
            // one lane per distinct shape of the wave probes the table
            int leader = lane;
            {
                uint64_t pend = __builtin_amdgcn_ballot_w64(keyed);
                while (pend) {
                    const int l = __builtin_ctzll(pend);
                    const uint64_t ml = (static_cast<uint64_t>(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(m >> 32), l))) << 32) |
                                        static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(m), l));
                    const uint64_t grp = __builtin_amdgcn_ballot_w64(keyed && m == ml);
                    if ((grp >> lane) & 1u) leader = l;
                    pend &= ~grp;
                }
            }
            int32_t slot = -1;
            bool won = false;
            if (keyed && leader == lane) {
                int64_t h = shape_hash(m, a.tbits);
                for (int64_t probe = 0; probe < TS; ++probe) {  // the table has > 2x slots: ends
                    unsigned long long cur = *reinterpret_cast<volatile unsigned long long*>(a.keys + h);
                    if (cur == 0ull)
                        cur = atomicCAS(reinterpret_cast<unsigned long long*>(a.keys + h), 0ull,
                                        static_cast<unsigned long long>(m));
                    if (cur == 0ull) {
                        a.reps_tr[h] = static_cast<int32_t>(tr);
                        slot = static_cast<int32_t>(h);
                        won = true;
                        break;
                    }
                    if (cur == m) {
                        slot = static_cast<int32_t>(h);
                        break;
                    }
                    h = (h + 1) & (TS - 1);
                }
            }
            const int gslot = __shfl(slot, leader);
            const bool gwon = __shfl(won ? 1 : 0, leader) != 0;
            // the representative replays (and every unkeyed episode); the rest reuse its rows
            const bool rep = have && (!keyed || (leader == lane && gwon));
            const bool dup = have && !rep;
            if (keyed) slot = gslot;
            // one 64-bit atomic reserves the wave's replay (low half) and duplicate (high) entries
            const int ir = wave_incl_scan(rep ? 1 : 0, lane), id = wave_incl_scan(dup ? 1 : 0, lane);
            const int nr = __shfl(ir, 63), nd = __shfl(id, 63);
            unsigned long long base = 0;
            if (lane == 63 && (nr | nd))
                base = atomicAdd(wd, (static_cast<unsigned long long>(nd) << 32) | static_cast<unsigned>(nr));
            base = __shfl(base, 63);
            if (rep) a.work[static_cast<int>(base & 0xffffffffu) + ir - 1] = static_cast<int32_t>(tr);
            if (dup) {
                const int di = static_cast<int>(base >> 32) + id - 1;
                a.dups[2 * di] = static_cast<int32_t>(tr);
                a.dups[2 * di + 1] = slot;
            }
        }
    }
    phase_stamp(a.stamps, blockIdx.x, 3);
}

}  // namespace fec
