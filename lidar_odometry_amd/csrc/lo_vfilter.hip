// lo_vfilter.hip — FastVoxelFilter::filter (VoxelMap.h:73-104; called by Estimator::preprocess_frame,
// Estimator.cpp:561-588) on the device, bit-identical to the reference's sequential pass:
//   * points i = 0, stride, 2*stride, ...; non-finite points skipped (:83-84);
//   * voxel = per-axis clamp((int64)floor(x * (1/voxel)) + 2^20, 0, 2^21 - 1) (computeMortonKey :123-135);
//   * fp32 running sums per voxel from 0 in point order, count (:86-90);
//   * output = sum * (1 / count) per voxel, in first-occurrence order (unordered_dense iterates in
//     insertion order, :93-102).
// Device plan (integer / gather work, launch-latency bound at a KITTI scan's 15k samples; five launches):
//   k_vf_insert  one lane per sample: key, open-addressing insert (CAS), per voxel atomicMin / atomicMax of the
//                sample index and a member count;
//   k_vf_heads   a sample is its voxel's head iff it is the voxel's first index; a block scan of (head, members)
//                gives each head its output slot (first-occurrence order) and bucket start inside the block, and
//                each block writes its totals (no inter-block hand-off: r06, the last-block pattern's agent-scope
//                fences cost ~14 us);
//   k_vf_place   every workgroup scans the block totals (one wave), block 0 publishes the prefix; every sample
//                appends its index to its voxel's bucket (arrival order);
//   k_vf_small   one lane per head with <= 16 members: register bitonic sort of the member indices, fp32 sums in
//                index order, output, slot reset; larger voxels are listed for
//   k_vf_wide    one wave per voxel with <= 64 members (wave bitonic sort, in-order sum by readlane), one
//                workgroup per larger voxel (up to 1024 members: its bucket sorted in LDS, wave 0 adds in order;
//                beyond, an ordered compaction of its index range), slot reset.
// The table slots are reset by the kernel that consumes them last, so the next pass starts from an empty table
// without a memset.  The output count stays on the device (n_dev): the ICP kernels read it, no host round trip.
#include "lo_device.h"
#include "lo_vfilter.h"

#include <algorithm>
#include <climits>

namespace lo {

constexpr uint64_t kVfEmpty = ~0ull;     // no 3 x 21-bit key has bit 63 set
constexpr int kVfHeadsBlock = 1024;
constexpr int kVfSmall = 16;
constexpr int kVfMid = 64;
constexpr int kVfWideGrid = 64;
constexpr int kVfBigSort = 1024;         // k_vf_wide: voxels up to this many members sort their bucket in LDS

// computeMortonKey's per-axis cell.  The reference converts floor(x * inv) to int64 with static_cast; on
// x86-64 (cvttss2si) every out-of-range value (|f| >= 2^63, inf) becomes INT64_MIN, which the clamp maps to 0.
__device__ __forceinline__ uint32_t vf_cell(float v, float inv) {
    const float f = floorf(v * inv);
    int64_t k = (f >= -9.2233720e18f && f < 9.2233720e18f) ? static_cast<int64_t>(f) : INT64_MIN;
    if (k != INT64_MIN) k += (1 << 20);
    if (k < 0) k = 0;
    if (k > (1 << 21) - 1) k = (1 << 21) - 1;
    return static_cast<uint32_t>(k);
}

__device__ __forceinline__ void vf_reset(uint64_t* tkey, VfSlot* tslot, int b) {
    tkey[b] = kVfEmpty;
    tslot[b] = VfSlot{0xFFFFFFFFu, 0u, 0u, 0u};
}

__device__ __forceinline__ const float* vf_point(const float* raw, int stride, int j) {
    return raw + 3 * (static_cast<size_t>(j) * stride);
}

__global__ __launch_bounds__(256) void k_vf_init(uint64_t* tkey, VfSlot* tslot, int n, VfCounters* ctr) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) vf_reset(tkey, tslot, i);
    if (i == 0) *ctr = VfCounters{0, 0u, 0, 0};
}

// raw may be device memory or pinned host memory (read over the bus exactly once, here: later kernels read the
// compact per-sample copy)
__global__ __launch_bounds__(256) void k_vf_insert(const float* __restrict__ raw, int stride, float inv, int m,
                                                   uint64_t* tkey, VfSlot* tslot, uint64_t mask, int l2,
                                                   int32_t* __restrict__ sslot, float* __restrict__ samp) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= m) return;
    const float* p = vf_point(raw, stride, j);
    const float x = p[0], y = p[1], z = p[2];
    samp[3 * j] = x;
    samp[3 * j + 1] = y;
    samp[3 * j + 2] = z;
    if (!(isfinite(x) && isfinite(y) && isfinite(z))) { sslot[j] = -1; return; }
    const uint64_t key = static_cast<uint64_t>(vf_cell(x, inv)) | (static_cast<uint64_t>(vf_cell(y, inv)) << 21) |
                         (static_cast<uint64_t>(vf_cell(z, inv)) << 42);
    uint64_t b = (key * 0x9E3779B97F4A7C15ull) >> (64 - l2);
    for (;;) {
        const unsigned long long old = atomicCAS(reinterpret_cast<unsigned long long*>(tkey + b),
                                                 static_cast<unsigned long long>(kVfEmpty),
                                                 static_cast<unsigned long long>(key));
        if (old == kVfEmpty || old == key) break;
        b = (b + 1) & mask;
    }
    atomicMin(&tslot[b].first, static_cast<uint32_t>(j));
    atomicMax(&tslot[b].last, static_cast<uint32_t>(j));
    atomicAdd(&tslot[b].cnt, 1u);
    sslot[j] = static_cast<int32_t>(b);
}

// inclusive scan of an int2 over the 64 lanes of a wave
__device__ __forceinline__ int2 wave_incl_scan2(int2 v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int ax = __shfl_up(v.x, o, 64), ay = __shfl_up(v.y, o, 64);
        if (lane >= o) { v.x += ax; v.y += ay; }
    }
    return v;
}

// exclusive scan of an int2 over a block of NT threads; tot = block total (every thread)
template <int NT>
__device__ __forceinline__ int2 block_excl_scan2(int2 v, int2& tot, int2* s_w /* NT/64 + 1 entries */) {
    constexpr int NW = NT / 64;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int2 inc = wave_incl_scan2(v);
    if (lane == 63) s_w[wid] = inc;
    __syncthreads();
    if (wid == 0) {
        const int2 w = lane < NW ? s_w[lane] : make_int2(0, 0);
        const int2 wi = wave_incl_scan2(w);
        if (lane < NW) s_w[lane] = make_int2(wi.x - w.x, wi.y - w.y);
        if (lane == NW - 1) s_w[NW] = wi;
    }
    __syncthreads();
    tot = s_w[NW];
    const int2 off = s_w[wid];
    const int2 ex = make_int2(off.x + inc.x - v.x, off.y + inc.y - v.y);
    __syncthreads();                                    // s_w may be reused right after
    return ex;
}

// Every block writes its (heads, members) totals; the exclusive prefix over the blocks is formed by each consumer
// workgroup itself (vf_block_prefix) -- r05's last-block-done hand-off needed agent-scope fences (an L2 write-back per
// block) and cost ~14 us at KITTI size.
__global__ __launch_bounds__(kVfHeadsBlock) void k_vf_heads(int m, const int32_t* __restrict__ sslot,
                                                            const VfSlot* __restrict__ tslot, int2* __restrict__ loc,
                                                            int2* blk) {
    __shared__ int2 s_w[kVfHeadsBlock / 64 + 1];
    const int tid = threadIdx.x;
    const int j = blockIdx.x * kVfHeadsBlock + tid;
    int2 v = make_int2(0, 0);
    if (j < m) {
        const int b = sslot[j];
        if (b >= 0) {
            const VfSlot s = tslot[b];
            if (s.first == static_cast<uint32_t>(j)) v = make_int2(1, static_cast<int>(s.cnt));
        }
    }
    int2 tot;
    const int2 ex = block_excl_scan2<kVfHeadsBlock>(v, tot, s_w);
    if (v.x) loc[j] = ex;
    if (tid == 0) blk[blockIdx.x] = tot;
}

// The exclusive prefix of the heads blocks' totals into out[0 .. nb] (out[nb] = the grand total; LDS or global), by
// wave 0 of the calling workgroup; the caller synchronises before reading LDS output.  nb = ceil(m / kVfHeadsBlock).
__device__ __forceinline__ void vf_block_prefix(const int2* __restrict__ blk, int nb, int2* out) {
    if ((threadIdx.x >> 6) != 0) return;
    const int lane = threadIdx.x & 63;
    int2 carry = make_int2(0, 0);
    for (int b0 = 0; b0 < nb; b0 += 64) {
        const int2 t = b0 + lane < nb ? blk[b0 + lane] : make_int2(0, 0);
        const int2 inc = wave_incl_scan2(t);
        if (b0 + lane < nb) out[b0 + lane] = make_int2(carry.x + inc.x - t.x, carry.y + inc.y - t.y);
        carry.x += __shfl(inc.x, 63, 64);
        carry.y += __shfl(inc.y, 63, 64);
    }
    if (lane == 0) out[nb] = carry;
}

__device__ __forceinline__ int2 vf_head_offsets(const int2* loc, const int2* blk, int h) {
    const int2 o = blk[h / kVfHeadsBlock], l = loc[h];
    return make_int2(o.x + l.x, o.y + l.y);            // (output slot, bucket start)
}

// k_vf_place forms the block prefix in every workgroup (up to kVfMaxPre blocks, 2^20 samples, in LDS; beyond, each
// sample sums the totals before its head's block), block 0 also publishes it (blk_pre, nb + 1 entries) and the pass's
// counters for the later launches
constexpr int kVfMaxPre = 1024;
__global__ __launch_bounds__(256) void k_vf_place(int m, const int32_t* __restrict__ sslot, VfSlot* tslot,
                                                  const int2* __restrict__ loc, const int2* __restrict__ blk,
                                                  int2* __restrict__ blk_pre, VfCounters* ctr,
                                                  int32_t* __restrict__ bucket) {
    __shared__ int2 s_pre[kVfMaxPre + 1];
    const int nb = (m + kVfHeadsBlock - 1) / kVfHeadsBlock;
    const int j = blockIdx.x * 256 + threadIdx.x;
    int b = -1, h = 0;
    if (j < m) {                                     // the sample's loads go out before the prefix is formed
        b = sslot[j];
        if (b >= 0) h = static_cast<int>(tslot[b].first);
    }
    if (blockIdx.x == 0) {
        vf_block_prefix(blk, nb, blk_pre);
        if (threadIdx.x == 0) { ctr->n_mid = 0; ctr->n_big = 0; }
    }
    if (nb <= kVfMaxPre) {
        vf_block_prefix(blk, nb, s_pre);
        __syncthreads();
        if (blockIdx.x == 0 && threadIdx.x == 0) ctr->n_out = s_pre[nb].x;
    } else if (blockIdx.x == 0 && threadIdx.x == 0) {
        int tot = 0;
        for (int q = 0; q < nb; ++q) tot += blk[q].x;
        ctr->n_out = tot;
    }
    if (j >= m || b < 0) return;
    int start;
    if (nb <= kVfMaxPre) {
        start = s_pre[h / kVfHeadsBlock].y + loc[h].y;
    } else {
        int o = 0;                                   // (beyond 2^20 samples only: C5 is 1M samples = 977 blocks)
        for (int q = 0; q < h / kVfHeadsBlock; ++q) o += blk[q].y;
        start = o + loc[h].y;
    }
    const unsigned r = atomicAdd(&tslot[b].fill, 1u);
    bucket[start + static_cast<int>(r)] = j;
}

// ascending bitonic sort of N register values (compile-time indices: stays in VGPRs)
template <int N>
__device__ __forceinline__ void bitonic_regs(int (&a)[N]) {
#pragma unroll
    for (int k = 2; k <= N; k <<= 1)
#pragma unroll
        for (int jj = k >> 1; jj > 0; jj >>= 1)
#pragma unroll
            for (int i = 0; i < N; ++i) {
                const int l = i ^ jj;
                if (l > i) {
                    const bool up = (i & k) == 0;
                    const int lo = min(a[i], a[l]), hi = max(a[i], a[l]);
                    a[i] = up ? lo : hi;
                    a[l] = up ? hi : lo;
                }
            }
}

__global__ __launch_bounds__(256) void k_vf_small(const float* __restrict__ samp, int m,
                                                  const int32_t* __restrict__ sslot, uint64_t* tkey, VfSlot* tslot,
                                                  const int2* __restrict__ loc, const int2* __restrict__ blk,
                                                  const int32_t* __restrict__ bucket, int32_t* mid, int32_t* big,
                                                  VfCounters* ctr, float* __restrict__ out) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= m) return;
    const int b = sslot[j];
    if (b < 0) return;
    const VfSlot s = tslot[b];
    if (s.first != static_cast<uint32_t>(j)) return;   // one lane per voxel: its head
    const int c = static_cast<int>(s.cnt);
    if (c > kVfSmall) {
        if (c <= kVfMid) mid[atomicAdd(&ctr->n_mid, 1)] = j;
        else big[atomicAdd(&ctr->n_big, 1)] = j;
        return;
    }
    const int2 o = vf_head_offsets(loc, blk, j);
    int a[kVfSmall];
#pragma unroll
    for (int t = 0; t < kVfSmall; ++t) a[t] = t < c ? bucket[o.y + t] : INT_MAX;
    bitonic_regs<kVfSmall>(a);
    float px[kVfSmall] = {}, py[kVfSmall] = {}, pz[kVfSmall] = {};
#pragma unroll
    for (int t = 0; t < kVfSmall; ++t) {
        if (t < c) {
            const float* p = samp + 3 * a[t];
            px[t] = p[0]; py[t] = p[1]; pz[t] = p[2];
        }
    }
    float sx = 0.0f, sy = 0.0f, sz = 0.0f;             // FilterAcc starts at 0 (VoxelMap.h:86-90)
#pragma unroll
    for (int t = 0; t < kVfSmall; ++t)
        if (t < c) { sx += px[t]; sy += py[t]; sz += pz[t]; }
    const float inv = 1.0f / static_cast<float>(c);
    out[3 * o.x] = sx * inv;
    out[3 * o.x + 1] = sy * inv;
    out[3 * o.x + 2] = sz * inv;
    vf_reset(tkey, tslot, b);
}

__global__ __launch_bounds__(256) void k_vf_wide(const float* __restrict__ samp,
                                                 const int32_t* __restrict__ sslot, uint64_t* tkey, VfSlot* tslot,
                                                 const int2* __restrict__ loc, const int2* __restrict__ blk,
                                                 const int32_t* __restrict__ bucket, const int32_t* __restrict__ mid,
                                                 const int32_t* __restrict__ big, const VfCounters* ctr,
                                                 float* __restrict__ out) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // ---- 17..64 members: one wave per voxel ----
    const int n_mid = ctr->n_mid;
    for (int q = blockIdx.x * 4 + wid; q < n_mid; q += gridDim.x * 4) {
        const int j = mid[q];
        const int b = sslot[j];
        const int c = static_cast<int>(tslot[b].cnt);
        const int2 o = vf_head_offsets(loc, blk, j);
        int v = lane < c ? bucket[o.y + lane] : INT_MAX;
#pragma unroll
        for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
            for (int jj = k >> 1; jj > 0; jj >>= 1) {
                const int w = __shfl_xor(v, jj, 64);
                const bool up = (lane & k) == 0, lower = (lane & jj) == 0;
                v = (lower == up) ? min(v, w) : max(v, w);
            }
        float px = 0.0f, py = 0.0f, pz = 0.0f;
        if (lane < c) { const float* p = samp + 3 * v; px = p[0]; py = p[1]; pz = p[2]; }
        float sx = 0.0f, sy = 0.0f, sz = 0.0f;         // in index order = lane order (c is wave-uniform: readlane)
        for (int t = 0; t < c; ++t) {
            sx += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(px), t));
            sy += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(py), t));
            sz += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pz), t));
        }
        if (lane == 0) {
            const float inv = 1.0f / static_cast<float>(c);
            out[3 * o.x] = sx * inv;
            out[3 * o.x + 1] = sy * inv;
            out[3 * o.x + 2] = sz * inv;
            vf_reset(tkey, tslot, b);
        }
    }
    // ---- 65..kVfBigSort members: one workgroup per voxel sorts the voxel's bucket (its member indices) in LDS and
    // wave 0 adds the members in index order; more: ordered compaction of the index range [first, last] ----
    __shared__ float s_p[256][3];
    __shared__ int s_wc[4];
    __shared__ int s_srt[kVfBigSort];
    const int n_big = ctr->n_big;
    for (int q = blockIdx.x; q < n_big; q += gridDim.x) {
        const int j = big[q];
        const int b = sslot[j];
        const VfSlot s = tslot[b];
        const int2 o = vf_head_offsets(loc, blk, j);
        const int c = static_cast<int>(s.cnt);
        if (c <= kVfBigSort) {
            // a voxel of a nearby surface is hit by several rings: its members span thousands of samples, so the range
            // walk took ~18 dependent passes; the bucket holds exactly the members
            int np2 = 128;
            while (np2 < c) np2 <<= 1;                  // the sort's width: the next power of two (block-uniform)
            for (int t = tid; t < np2; t += 256) s_srt[t] = t < c ? bucket[o.y + t] : INT_MAX;
            __syncthreads();
            for (int k = 2; k <= np2; k <<= 1) {                            // bitonic sort, ascending
                for (int jj = k >> 1; jj > 0; jj >>= 1) {
                    for (int t = tid; t < np2; t += 256) {
                        const int l = t ^ jj;
                        if (l > t) {
                            const int a0 = s_srt[t], a1 = s_srt[l];
                            const bool up = (t & k) == 0;
                            if ((a0 > a1) == up) { s_srt[t] = a1; s_srt[l] = a0; }
                        }
                    }
                    __syncthreads();
                }
            }
            if (wid == 0) {                             // wave 0: 64 members' points at a time, added in order
                float sx = 0.0f, sy = 0.0f, sz = 0.0f;
                for (int t0 = 0; t0 < c; t0 += 64) {
                    float px = 0.0f, py = 0.0f, pz = 0.0f;
                    if (t0 + lane < c) { const float* p = samp + 3 * s_srt[t0 + lane]; px = p[0]; py = p[1]; pz = p[2]; }
                    const int e = min(64, c - t0);
                    for (int t = 0; t < e; ++t) {
                        sx += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(px), t));
                        sy += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(py), t));
                        sz += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pz), t));
                    }
                }
                if (lane == 0) {
                    const float inv = 1.0f / static_cast<float>(c);
                    out[3 * o.x] = sx * inv;
                    out[3 * o.x + 1] = sy * inv;
                    out[3 * o.x + 2] = sz * inv;
                    vf_reset(tkey, tslot, b);
                }
            }
            __syncthreads();                            // s_srt is reused by this workgroup's next voxel
            continue;
        }
        float sx = 0.0f, sy = 0.0f, sz = 0.0f;         // thread 0's running sums
        for (int base = static_cast<int>(s.first); base <= static_cast<int>(s.last); base += 256) {
            const int jj = base + tid;
            const bool f = jj <= static_cast<int>(s.last) && sslot[jj] == b;
            const uint64_t bal = __ballot(f);
            if (lane == 0) s_wc[wid] = __popcll(bal);
            __syncthreads();
            int off = 0, cnt = 0;
#pragma unroll
            for (int w = 0; w < 4; ++w) { off += (w < wid) ? s_wc[w] : 0; cnt += s_wc[w]; }
            if (f) {
                const int r = off + __popcll(bal & ((1ull << lane) - 1ull));
                const float* p = samp + 3 * jj;
                s_p[r][0] = p[0]; s_p[r][1] = p[1]; s_p[r][2] = p[2];
            }
            __syncthreads();
            if (tid == 0)
                for (int t = 0; t < cnt; ++t) { sx += s_p[t][0]; sy += s_p[t][1]; sz += s_p[t][2]; }
            __syncthreads();
        }
        if (tid == 0) {
            const float inv = 1.0f / static_cast<float>(s.cnt);
            out[3 * o.x] = sx * inv;
            out[3 * o.x + 1] = sy * inv;
            out[3 * o.x + 2] = sz * inv;
            vf_reset(tkey, tslot, b);
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------- host side (called from lo_icp.hip)
// Grows the filter's buffers on the context stream s: the old buffers may still be read by filter launches
// queued on s, so s (only) is drained before they are freed, and the table init runs on s, ordered before the
// next k_vf_insert without a device-wide synchronisation that would stall other contexts sharing the GPU.
hipError_t vf_reserve(VfBuffers& b, size_t m, hipStream_t s) {
    if (b.ctr != nullptr && m <= b.cap) return hipSuccess;
    if (b.ctr != nullptr) {
        hipError_t e0 = hipStreamSynchronize(s);
        if (e0 != hipSuccess) return e0;
    }
    void* old[] = {b.tkey, b.tslot, b.sslot, b.samp, b.loc, b.blk, b.blk_pre, b.bucket, b.mid, b.big, b.ctr};
    for (void* p : old) if (p) (void)hipFree(p);
    b = VfBuffers{};
    const size_t cap = std::max<size_t>(m, 4096);
    size_t tcap = 2;
    while (tcap < 2 * cap) tcap <<= 1;                  // load factor <= 0.5
    const size_t nb = (cap + kVfHeadsBlock - 1) / kVfHeadsBlock;
    hipError_t e;
    if ((e = hipMalloc(&b.tkey, tcap * sizeof(uint64_t))) != hipSuccess) return e;
    if ((e = hipMalloc(&b.tslot, tcap * sizeof(VfSlot))) != hipSuccess) return e;
    if ((e = hipMalloc(&b.sslot, cap * sizeof(int32_t))) != hipSuccess) return e;
    if ((e = hipMalloc(&b.samp, cap * 3 * sizeof(float))) != hipSuccess) return e;
    if ((e = hipMalloc(&b.loc, cap * sizeof(int2))) != hipSuccess) return e;
    if ((e = hipMalloc(&b.blk, nb * sizeof(int2))) != hipSuccess) return e;
    if ((e = hipMalloc(&b.blk_pre, (nb + 1) * sizeof(int2))) != hipSuccess) return e;
    if ((e = hipMalloc(&b.bucket, cap * sizeof(int32_t))) != hipSuccess) return e;
    if ((e = hipMalloc(&b.mid, cap * sizeof(int32_t))) != hipSuccess) return e;
    if ((e = hipMalloc(&b.big, cap * sizeof(int32_t))) != hipSuccess) return e;
    if ((e = hipMalloc(&b.ctr, sizeof(VfCounters))) != hipSuccess) return e;
    hipLaunchKernelGGL(k_vf_init, dim3(static_cast<unsigned>((tcap + 255) / 256)), dim3(256), 0, s, b.tkey, b.tslot,
                       static_cast<int>(tcap), b.ctr);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    b.cap = cap;
    b.tcap = tcap;
    b.n_out = &b.ctr->n_out;
    return hipSuccess;
}

void vf_free(VfBuffers& b) {
    void* all[] = {b.tkey, b.tslot, b.sslot, b.samp, b.loc, b.blk, b.blk_pre, b.bucket, b.mid, b.big, b.ctr};
    for (void* p : all) if (p) (void)hipFree(p);
    b = VfBuffers{};
}

// Enqueue the filter of d_raw (n_raw AoS float3, device or pinned host memory) into d_out; the count lands in
// b.n_out (device).
// Returns the number of samples m = ceil(n_raw / stride), an upper bound of the output count.
hipError_t vf_enqueue(VfBuffers& b, const float* d_raw, size_t n_raw, int stride, float voxel_size, float* d_out,
                      hipStream_t s, int& m_out) {
    const size_t m = (n_raw + stride - 1) / stride;
    m_out = static_cast<int>(m);
    hipError_t e = vf_reserve(b, m, s);
    if (e != hipSuccess) return e;
    if (m == 0) return hipMemsetAsync(b.n_out, 0, sizeof(int), s);
    const float inv = 1.0f / voxel_size;                 // m_inv_voxel_size (VoxelMap.h:57)
    int l2 = 0;
    while ((size_t(1) << l2) < b.tcap) ++l2;
    const int mi = static_cast<int>(m);
    const dim3 g256(static_cast<unsigned>((m + 255) / 256)), t256(256);
    const dim3 gh(static_cast<unsigned>((m + kVfHeadsBlock - 1) / kVfHeadsBlock)), th(kVfHeadsBlock);
    hipLaunchKernelGGL(k_vf_insert, g256, t256, 0, s, d_raw, stride, inv, mi, b.tkey, b.tslot,
                       static_cast<uint64_t>(b.tcap - 1), l2, b.sslot, b.samp);
    hipLaunchKernelGGL(k_vf_heads, gh, th, 0, s, mi, b.sslot, b.tslot, b.loc, b.blk);
    hipLaunchKernelGGL(k_vf_place, g256, t256, 0, s, mi, b.sslot, b.tslot, b.loc, b.blk, b.blk_pre, b.ctr, b.bucket);
    hipLaunchKernelGGL(k_vf_small, g256, t256, 0, s, b.samp, mi, b.sslot, b.tkey, b.tslot, b.loc, b.blk_pre,
                       b.bucket, b.mid, b.big, b.ctr, d_out);
    hipLaunchKernelGGL(k_vf_wide, dim3(kVfWideGrid), t256, 0, s, b.samp, b.sslot, b.tkey, b.tslot, b.loc,
                       b.blk_pre, b.bucket, b.mid, b.big, b.ctr, d_out);
    return hipGetLastError();
}

}  // namespace lo
