// fec_shapes.hip -- loss-episode deduplication for the decode planner.
//
// An episode starts at an erased packet tr with no erasure in [tr-T-1, tr-1] (the decoder's
// resynchronisation, Decoder.cpp:109-133) and lasts until T+1 packets after its latest erasure
// have been received (Decoder.cpp:80-83).  Everything the planner derives for the episode's
// erased packets -- which symbols are recovered and their coefficient rows -- is a function of
// the block states at tr and of the erasure flags inside the episode.  For tr >= T the block
// state at tr is the post-resync state of the block's phase, and the phase of the block holding
// symbol i of packet x is (tr - x + i) mod n: the results depend on x - tr, not on tr.  Two
// episodes with the same erasure shape (bit j = packet tr+j erased) therefore have identical
// results at equal offsets.
//
// Per batch (the table is cleared by every plan launch; nothing is carried between batches):
//   fec_shape_kernel      one wave per episode: the shape (64-bit mask), hash-table insert;
//                         the first episode of a shape and every episode that cannot be keyed
//                         (startup tr < T, span >= 64, or running into the batch end) go to the
//                         replay work list, the others to the fill list;
//   (fec_plan_kernel / fec_plan_fast_kernel replay the work list)
//   fec_shape_fill_kernel one wave per filled episode: sym_ok and coef rows of each erased
//                         packet copied from the representative's packet at the same offset.
#include "fec_kernels.h"

namespace fec {

__global__ __launch_bounds__(64) void fec_shape_kernel(ShapeArgs a) {
    const int lane = threadIdx.x;
    const int ne = a.counters[0];
    const int64_t TS = int64_t(1) << a.tbits;
    for (int e = blockIdx.x; e < ne; e += gridDim.x) {
        const int64_t tr = a.episodes[e];
        // walk the episode in windows of 64 packets; positions relative to tr
        int latest = 0;
        uint64_t m = 1;
        bool big = false, done = false, truncated = false;
        for (int base = 1; !done; base += 64) {
            const int64_t t = tr + base + lane;
            const bool f = t < a.P && a.er[t] != 0;
            uint64_t bits = __ballot(f);
            while (bits) {
                const int j = __builtin_ctzll(bits);
                bits &= bits - 1;
                const int pos = base + j;
                if (pos - latest > a.T) {
                    done = true;
                    break;
                }
                latest = pos;
                if (pos < 64) m |= uint64_t(1) << pos;
                else big = true;
            }
            if (!done && latest + a.T <= base + 63) done = true;  // the gap after latest is complete
            if (!done && tr + base + 64 >= a.P) {
                done = true;
                truncated = true;
            }
        }
        if (lane == 0) {
            const int64_t last = tr + latest;
            a.ep_last[e] = static_cast<int32_t>(last);
            const bool keyed = a.dedup && tr >= a.T && !big && !truncated && last + a.T + 1 < a.P;
            int32_t slot = -1;
            bool rep = true;
            if (keyed) {
                int64_t h = static_cast<int64_t>((m * 0x9E3779B97F4A7C15ull) >> (64 - a.tbits));
                // the table holds > 2x as many slots as a batch can have episodes: probing ends
                for (int64_t probe = 0; probe < TS; ++probe) {
                    const unsigned long long prev = atomicCAS(
                        reinterpret_cast<unsigned long long*>(a.keys + h), 0ull, static_cast<unsigned long long>(m));
                    if (prev == 0ull) {
                        a.reps[h] = e;  // this episode represents the shape
                        slot = static_cast<int32_t>(h);
                        break;
                    }
                    if (prev == m) {
                        rep = false;
                        slot = static_cast<int32_t>(h);
                        break;
                    }
                    h = (h + 1) & (TS - 1);
                }
            }
            a.ep_slot[e] = slot;
            if (rep) a.work[atomicAdd(&a.counters[3], 1)] = e;
            else a.fill[atomicAdd(&a.counters[4], 1)] = e;
        }
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
