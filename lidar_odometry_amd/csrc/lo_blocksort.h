// lo_blocksort.h — sorting the iteration-0 residuals for reference-exact mode without a chip-wide rank pass.
//
// The reference sorts the accepted residuals before it sums them (IterativeClosestPointOptimizer.cpp:304-316).  The
// residuals are non-negative doubles, so their IEEE bit patterns order as unsigned integers; a point without a
// correspondence gets +inf's bits (sorted after every finite residual) and a NaN residual sorts after +inf.
//   1. presort_block: the correspondence launch of iteration 0 (k_correspond / k_plane) sorts its own 256 keys in
//      place -- a bitonic network with the in-wave exchanges done by DPP / permlane swaps (no LDS) and the two
//      cross-wave distances through LDS -- and writes the sorted run;
//   2. k_exact_scale_m (lo_exact.hip) merges the runs in LDS (merge path, one workgroup) and sums them.
// Equal keys are equal values, so the order among them does not change any sum: no stability is needed.
#pragma once
#include "lo_device.h"

namespace lo {

constexpr uint64_t kInfKey = 0x7FF0000000000000ull;     // +inf: no correspondence / past the scan

// v of lane (lane ^ J) for J < 64, without LDS: quad_perm (1, 2), half-row mirror + quad reverse (4),
// row_ror:8 (8), v_permlane16_swap (16), v_permlane32_swap (32).
template <int J>
__device__ __forceinline__ uint32_t xor_lane32(uint32_t v) {
    const int lane = threadIdx.x & 63;
    if constexpr (J == 1) {
        return static_cast<uint32_t>(dpp32m<0xB1>(static_cast<int>(v)));
    } else if constexpr (J == 2) {
        return static_cast<uint32_t>(dpp32m<0x4E>(static_cast<int>(v)));
    } else if constexpr (J == 4) {
        // b[l] = a[rev(l)], a[l] = v[mirror8(l)]  =>  b[l] = v[7 - ((l & 4) | (3 - (l & 3)))] = v[l ^ 4]
        const int a = dpp32m<0x141>(static_cast<int>(v));
        return static_cast<uint32_t>(dpp32m<0x1B>(a));
    } else if constexpr (J == 8) {
        return static_cast<uint32_t>(dpp32m<0x128>(static_cast<int>(v)));
    } else if constexpr (J == 16) {
        // swap(v, v): r[0] = rows [v0 v0 v2 v2], r[1] = [v1 v1 v3 v3]
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (lane & 16) ? static_cast<uint32_t>(r[0]) : static_cast<uint32_t>(r[1]);
    } else {
        static_assert(J == 32, "lane distance");
        // swap(v, v): r[0] = [v_lo | v_lo], r[1] = [v_hi | v_hi]
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (lane & 32) ? static_cast<uint32_t>(r[0]) : static_cast<uint32_t>(r[1]);
    }
}
template <int J>
__device__ __forceinline__ uint64_t xor_lane64(uint64_t v) {
    const uint32_t lo = xor_lane32<J>(static_cast<uint32_t>(v));
    const uint32_t hi = xor_lane32<J>(static_cast<uint32_t>(v >> 32));
    return (static_cast<uint64_t>(hi) << 32) | lo;
}

// One compare-exchange step of the bitonic network: element e keeps the min of (its key, the key of e ^ j) when
// the ascending/descending direction of its k-block and its position in the pair agree, else the max.
__device__ __forceinline__ uint64_t cx_keep(uint64_t mine, uint64_t other, int e, int k, int j) {
    const bool keep_min = ((e & k) == 0) == ((e & j) == 0);
    const uint64_t mn = other < mine ? other : mine, mx = other < mine ? mine : other;
    return keep_min ? mn : mx;
}

template <int J>
__device__ __forceinline__ uint64_t bitonic_wave_stage(uint64_t key, int e, int k) {
    return cx_keep(key, xor_lane64<J>(key), e, k, J);
}

// The in-wave tail of merge level k (distances 32 .. 1 that are < k).
__device__ __forceinline__ uint64_t bitonic_wave_tail(uint64_t key, int e, int k) {
    if (k > 32) key = bitonic_wave_stage<32>(key, e, k);
    if (k > 16) key = bitonic_wave_stage<16>(key, e, k);
    if (k > 8) key = bitonic_wave_stage<8>(key, e, k);
    if (k > 4) key = bitonic_wave_stage<4>(key, e, k);
    if (k > 2) key = bitonic_wave_stage<2>(key, e, k);
    return bitonic_wave_stage<1>(key, e, k);
}

// Sort the 256 keys of a 256-thread workgroup (one per thread) ascending; thread t returns the key of rank t.
// s_tmp: 256 uint64 of LDS.  Every thread of the workgroup must call it.
__device__ __forceinline__ uint64_t block_sort256(uint64_t key, uint64_t* s_tmp) {
    const int e = threadIdx.x;
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) key = bitonic_wave_tail(key, e, k);
#pragma unroll
    for (int k = 128; k <= 256; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j >= 64; j >>= 1) {
            __syncthreads();
            s_tmp[e] = key;
            __syncthreads();
            key = cx_keep(key, s_tmp[e ^ j], e, k, j);
        }
        key = bitonic_wave_tail(key, e, k);
    }
    return key;
}

// The iteration-0 correspondence launch's part of the exact scale: this block's 256 residual keys (accepted
// residual bits, +inf otherwise), sorted, written as run `blk` of `runs`.
__device__ __forceinline__ void presort_block(uint64_t* runs, int blk, uint64_t key) {
    __shared__ uint64_t s_sort[kBlock];
    const uint64_t sorted = block_sort256(key, s_sort);
    runs[static_cast<size_t>(blk) * kBlock + threadIdx.x] = sorted;
}

}  // namespace lo
