// fec_shapes.hip -- loss-episode deduplication for the decode planner.
//
// An episode starts at an erased packet tr with no erasure in [tr-T-1, tr-1] (the decoder's
// resynchronisation, Decoder.cpp:109-133) and ends at the first received packet t with no erasure
// in [t-T, t-1] (Decoder.cpp:80-83): packet latest+T+1 ends it only if it is received, an
// erasure there continues the episode.  Everything the planner derives for the episode's
// erased packets -- which symbols are recovered and their coefficient rows -- is a function of
// the block states at tr and of the erasure flags inside the episode.  For tr >= T the block
// state at tr is the post-resync state of the block's phase, and the phase of the block holding
// symbol i of packet x is (tr - x + i) mod n: the results depend on x - tr, not on tr.  Two
// episodes with the same erasure shape (bit j = packet tr+j erased) therefore have identical
// results at equal offsets.
//
// Per batch (the table is cleared by every plan launch; nothing is carried between batches):
//   fec_shape_kernel      one thread per episode: the shape (64-bit mask), hash-table insert;
//                         the first episode of a shape and every episode that cannot be keyed
//                         (startup tr < T, span >= 64, or running into the batch end) go to the
//                         replay work list, the others to the fill list;
//   (fec_plan_kernel / fec_plan_fast_kernel replay the work list)
//   fec_shape_fill_kernel one wave per filled episode: sym_ok and coef rows of each erased
//                         packet copied from the representative's packet at the same offset.
#include "fec_kernels.h"

namespace fec {

namespace {

constexpr int kLocalSlots = 512;  // per-workgroup table (256 episodes per pass)

__device__ __forceinline__ uint32_t shape_hash(uint64_t m, int bits) {
    return static_cast<uint32_t>((m * 0x9E3779B97F4A7C15ull) >> (64 - bits));
}

// Erasure flags of packets t0 .. t0+63 as bits (bit j = packet t0+j erased; past P: 0).  Nine
// aligned 8-byte loads instead of 64 byte loads: one thread walks one episode, so these loads
// are scattered, and their number is what the planner pays beside the copy kernel.
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
            if (t < P && er[t]) fl |= uint64_t(1) << j;
        }
    }
    return fl;
}

// Wave-aggregated append of `item` for the lanes where `want` holds.
__device__ __forceinline__ void wave_append(bool want, int32_t* counter, int32_t* list, int item) {
    const uint64_t bal = __ballot(want);
    if (!bal) return;
    const int lane = threadIdx.x & 63;
    const int leader = __builtin_ctzll(bal);
    int base = 0;
    if (lane == leader) base = atomicAdd(counter, __popcll(bal));
    base = __shfl(base, leader);
    if (want) list[base + __popcll(bal & ((uint64_t(1) << lane) - 1))] = item;
}

}  // namespace

// One thread per episode.  Shapes are first deduplicated in a workgroup-local LDS table; only
// the local representative of a shape touches the global table (one CAS per shape per
// workgroup), so hot shapes do not serialise on one address.
__global__ __launch_bounds__(256) void fec_shape_kernel(ShapeArgs a) {
    __shared__ unsigned long long lkey[kLocalSlots];
    __shared__ int32_t lslot[kLocalSlots];   // global slot of the local shape
    __shared__ int32_t lrep[kLocalSlots];    // 1: the local representative won the global slot
    const int tid = threadIdx.x;
    const int ne = a.counters[0];
    const int64_t TS = int64_t(1) << a.tbits;
    for (int e0 = blockIdx.x * 256; e0 < ne; e0 += gridDim.x * 256) {
        for (int i = tid; i < kLocalSlots; i += 256) lkey[i] = 0ull;
        const int e = e0 + tid;
        const bool valid = e < ne;
        int64_t tr = 0, last = 0;
        uint64_t m = 1;
        bool keyed = false;
        if (valid) {
            tr = a.episodes[e];
            // walk the episode: positions relative to tr, flags in windows of 64
            int latest = 0;
            bool big = false, done = false, truncated = false;
            for (int base = 1; !done; base += 64) {
                uint64_t fl = erasure_bits64(a.er, a.P, tr + base);
                while (fl) {
                    const int j = __builtin_ctzll(fl);
                    fl &= fl - 1;
                    const int pos = base + j;
                    if (pos - latest > a.T + 1) {  // packet latest+T+1 was received: ended
                        done = true;
                        break;
                    }
                    latest = pos;
                    if (pos < 64) m |= uint64_t(1) << pos;
                    else big = true;
                }
                if (!done && latest + a.T + 1 <= base + 63) done = true;  // latest+T+1 seen, received
                if (!done && tr + base + 64 >= a.P) {
                    done = true;
                    truncated = true;
                }
            }
            last = tr + latest;
            a.ep_last[e] = static_cast<int32_t>(last);
            keyed = a.dedup && tr >= a.T && !big && !truncated && last + a.T + 1 < a.P;
        }
        __syncthreads();
        // local insert: the first thread of a shape in this workgroup is its local representative
        int ls = -1;
        bool lfirst = false;
        if (keyed) {
            uint32_t h = shape_hash(m, 9);
            for (int probe = 0; probe < kLocalSlots; ++probe) {
                const unsigned long long prev = atomicCAS(&lkey[h], 0ull, static_cast<unsigned long long>(m));
                if (prev == 0ull || prev == m) {
                    ls = static_cast<int>(h);
                    lfirst = prev == 0ull;
                    break;
                }
                h = (h + 1) & (kLocalSlots - 1);
            }
        }
        // global insert by the local representatives
        if (lfirst) {
            int64_t h = shape_hash(m, a.tbits);
            int32_t gs = -1, won = 0;
            for (int64_t probe = 0; probe < TS; ++probe) {  // the table has > 2x slots: ends
                unsigned long long cur = __hip_atomic_load(reinterpret_cast<unsigned long long*>(a.keys + h),
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (cur == 0ull)
                    cur = atomicCAS(reinterpret_cast<unsigned long long*>(a.keys + h), 0ull,
                                    static_cast<unsigned long long>(m));
                if (cur == 0ull) {
                    a.reps[h] = e;
                    gs = static_cast<int32_t>(h);
                    won = 1;
                    break;
                }
                if (cur == m) {
                    gs = static_cast<int32_t>(h);
                    break;
                }
                h = (h + 1) & (TS - 1);
            }
            lslot[ls] = gs;
            lrep[ls] = won;
        }
        __syncthreads();
        int32_t gslot = -1;
        bool rep = valid;
        if (keyed && ls >= 0) {
            gslot = lslot[ls];
            rep = lfirst && lrep[ls];
        }
        if (valid) a.ep_slot[e] = gslot;
        wave_append(valid && rep, &a.counters[3], a.work, e);
        wave_append(valid && !rep, &a.counters[4], a.fill, e);
        __syncthreads();  // lkey is cleared for the next pass
    }
}

__global__ __launch_bounds__(64) void fec_shape_fill_kernel(ShapeArgs a) {
    const int lane = threadIdx.x;
    const int nf = a.counters[4];
    const int k = a.k, kn = a.k * a.n;
    for (int f = blockIdx.x; f < nf; f += gridDim.x) {
        const int e = a.fill[f];
        const int rep = a.reps[a.ep_slot[e]];
        const int64_t tr = a.episodes[e];
        const int64_t d = static_cast<int64_t>(a.episodes[rep]) - tr;
        const int64_t last = a.ep_last[e];  // last - tr < 64 for a keyed episode
        const int64_t xl = tr + lane;
        uint64_t bits = __ballot(xl <= last && a.er[xl] != 0);
        while (bits) {
            const int j = __builtin_ctzll(bits);
            bits &= bits - 1;
            const int64_t x = tr + j, xr = x + d;
            for (int o = lane; o < kn; o += 64) a.coef[x * kn + o] = a.coef[xr * kn + o];
            if (lane < k) a.sym_ok[x * k + lane] = a.sym_ok[xr * k + lane];
        }
    }
}

}  // namespace fec
