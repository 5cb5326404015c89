// lo_vfilter.hip — FastVoxelFilter::filter (VoxelMap.h:73-104; called by Estimator::preprocess_frame,
// Estimator.cpp:561-588) on the device, bit-identical to the reference's sequential pass:
//   * points i = 0, stride, 2*stride, ...; non-finite points skipped (:83-84);
//   * voxel = per-axis clamp((int64)floor(x * (1/voxel)) + 2^20, 0, 2^21 - 1) (computeMortonKey :123-135);
//   * fp32 running sums per voxel in point order, count (:86-90);
//   * output = sum * (1 / count) per voxel, in first-occurrence order (unordered_dense iterates in
//     insertion order, :93-102).
// Device plan (HBM-bound integer work, no MFMA): key per sampled point -> stable radix sort of (key, sample
// index) [hipCUB] -> segment heads mark each voxel's first sample -> exclusive scan of those marks over the
// sample index = output slot in first-occurrence order -> one lane per voxel sums its samples in index order.
// The output count stays on the device (n_dev) so the ICP kernels can consume it without a host round trip.
#include "lo_device.h"
#include "lo_vfilter.h"

#include <algorithm>
#include <hipcub/hipcub.hpp>

namespace lo {

constexpr uint64_t kVfInvalid = ~0ull;

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

__global__ __launch_bounds__(256) void k_vf_keys(const float* __restrict__ raw, int stride, float inv, int m,
                                                 uint64_t* __restrict__ keys, int32_t* __restrict__ idx) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= m) return;
    const size_t i = static_cast<size_t>(j) * stride;
    const float x = raw[3 * i], y = raw[3 * i + 1], z = raw[3 * i + 2];
    uint64_t key = kVfInvalid;
    if (isfinite(x) && isfinite(y) && isfinite(z))
        key = static_cast<uint64_t>(vf_cell(x, inv)) | (static_cast<uint64_t>(vf_cell(y, inv)) << 21) |
              (static_cast<uint64_t>(vf_cell(z, inv)) << 42);
    keys[j] = key;
    idx[j] = j;
}

// first[j] = 1 iff sample j is the first (lowest index) sample of its voxel (every j is written once), and the
// samples' coordinates gathered into sorted order (one parallel pass, so the per-voxel sums read contiguously)
__global__ __launch_bounds__(256) void k_vf_heads(const uint64_t* __restrict__ ks, const int32_t* __restrict__ is, int m,
                                                  const float* __restrict__ raw, int stride, int32_t* __restrict__ first,
                                                  float4* __restrict__ ps) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= m) return;
    const uint64_t key = ks[k];
    const int j = is[k];
    const bool head = key != kVfInvalid && (k == 0 || ks[k - 1] != key);
    first[j] = head ? 1 : 0;
    const size_t i = static_cast<size_t>(j) * stride;
    // .w = 1 starts a run: a voxel head, or an invalid sample (they sort last and must end the last voxel's run)
    ps[k] = make_float4(raw[3 * i], raw[3 * i + 1], raw[3 * i + 2], (head || key == kVfInvalid) ? 1.0f : 0.0f);
}

// one lane per voxel: fp32 running sums over its samples in index order (contiguous after the sort; 4 loads
// in flight per step, the .w head mark ends the run)
__global__ __launch_bounds__(256) void k_vf_reduce(const float4* __restrict__ ps, const int32_t* __restrict__ is, int m,
                                                   const int32_t* __restrict__ first, const int32_t* __restrict__ pos,
                                                   float* __restrict__ out, int* __restrict__ n_out, const uint64_t* __restrict__ ks) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k == 0) *n_out = m > 0 ? pos[m - 1] + first[m - 1] : 0;
    if (k >= m) return;
    const float4 p0 = ps[k];
    if (p0.w == 0.0f || ks[k] == kVfInvalid) return;                // not a voxel head (invalid samples sort last)
    float sx = p0.x, sy = p0.y, sz = p0.z;
    uint32_t count = 1;
    bool run = true;
    for (int q = k + 1; run && q < m; q += 4) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = (q + u < m) ? ps[q + u] : make_float4(0.0f, 0.0f, 0.0f, 1.0f);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (!run) break;
            if (v[u].w != 0.0f) { run = false; break; }             // next voxel (or the end) starts here
            sx += v[u].x;
            sy += v[u].y;
            sz += v[u].z;
            ++count;
        }
    }
    const float inv = 1.0f / static_cast<float>(count);
    const int o = pos[is[k]];
    out[3 * o] = sx * inv;
    out[3 * o + 1] = sy * inv;
    out[3 * o + 2] = sz * inv;
}

// ---------------------------------------------------------------- host side (called from lo_icp.hip)
hipError_t vf_reserve(VfBuffers& b, size_t m) {
    if (b.n_out == nullptr) {
        hipError_t e = hipMalloc(&b.n_out, sizeof(int));
        if (e != hipSuccess) return e;
    }
    if (m <= b.cap) return hipSuccess;
    void* old[] = {b.keys, b.keys_s, b.idx, b.idx_s, b.first, b.pos, b.temp, b.pts_s};
    for (void* p : old) if (p) (void)hipFree(p);
    const size_t cap = std::max<size_t>(m, 4096);
    hipError_t e;
    if ((e = hipMalloc(&b.keys, cap * 8)) != hipSuccess) return e;
    if ((e = hipMalloc(&b.keys_s, cap * 8)) != hipSuccess) return e;
    if ((e = hipMalloc(&b.idx, cap * 4)) != hipSuccess) return e;
    if ((e = hipMalloc(&b.idx_s, cap * 4)) != hipSuccess) return e;
    if ((e = hipMalloc(&b.first, cap * 4)) != hipSuccess) return e;
    if ((e = hipMalloc(&b.pos, cap * 4)) != hipSuccess) return e;
    if ((e = hipMalloc(&b.pts_s, cap * sizeof(float4))) != hipSuccess) return e;
    size_t sort_bytes = 0, scan_bytes = 0;
    if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, b.keys, b.keys_s, b.idx, b.idx_s,
                                                static_cast<int>(cap), 0, 64)) != hipSuccess) return e;
    if ((e = hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, b.first, b.pos, static_cast<int>(cap))) != hipSuccess) return e;
    b.temp_bytes = std::max(sort_bytes, scan_bytes);
    if ((e = hipMalloc(&b.temp, b.temp_bytes)) != hipSuccess) return e;
    b.cap = cap;
    return hipSuccess;
}

void vf_free(VfBuffers& b) {
    void* all[] = {b.keys, b.keys_s, b.idx, b.idx_s, b.first, b.pos, b.temp, b.n_out, b.pts_s};
    for (void* p : all) if (p) (void)hipFree(p);
    b = VfBuffers{};
}

// Enqueue the filter of d_raw (n_raw AoS float3) into d_out; the count lands in b.n_out (device).
// Returns the number of samples m = ceil(n_raw / stride), an upper bound of the output count.
hipError_t vf_enqueue(VfBuffers& b, const float* d_raw, size_t n_raw, int stride, float voxel_size, float* d_out,
                      hipStream_t s, int& m_out) {
    const size_t m = (n_raw + stride - 1) / stride;
    m_out = static_cast<int>(m);
    hipError_t e = vf_reserve(b, m);
    if (e != hipSuccess) return e;
    if (m == 0) return hipMemsetAsync(b.n_out, 0, sizeof(int), s);
    const float inv = 1.0f / voxel_size;                         // m_inv_voxel_size (VoxelMap.h:57)
    const dim3 g(static_cast<unsigned>((m + 255) / 256)), t(256);
    hipLaunchKernelGGL(k_vf_keys, g, t, 0, s, d_raw, stride, inv, static_cast<int>(m), b.keys, b.idx);
    size_t bytes = b.temp_bytes;
    if ((e = hipcub::DeviceRadixSort::SortPairs(b.temp, bytes, b.keys, b.keys_s, b.idx, b.idx_s, static_cast<int>(m),
                                                0, 64, s)) != hipSuccess) return e;   // all 64 bits: ~0 marks invalid
    hipLaunchKernelGGL(k_vf_heads, g, t, 0, s, b.keys_s, b.idx_s, static_cast<int>(m), d_raw, stride, b.first, b.pts_s);
    bytes = b.temp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(b.temp, bytes, b.first, b.pos, static_cast<int>(m), s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_vf_reduce, g, t, 0, s, b.pts_s, b.idx_s, static_cast<int>(m), b.first, b.pos, d_out, b.n_out,
                       b.keys_s);
    return hipGetLastError();
}

}  // namespace lo
