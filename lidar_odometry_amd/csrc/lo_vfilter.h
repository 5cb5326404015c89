// lo_vfilter.h — device FastVoxelFilter (lo_vfilter.hip), host-side interface for lo_icp.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace lo {

// Voxel slot of the filter's hash table: first / last sample index, member count, bucket fill cursor.
struct VfSlot {
    uint32_t first, last, cnt, fill;
};

// Device counters of one filter pass (reset by the pass itself).
struct VfCounters {
    int n_out;                   // voxels = output points (read by the ICP kernels as KParams::n_dev)
    unsigned arrive;             // (unused since r06: no last-block hand-off)
    int n_mid, n_big;            // voxels with 17..64 / more than 64 samples (k_vf_wide)
};

struct VfBuffers {
    size_t cap = 0;              // samples
    size_t tcap = 0;             // table slots (power of two >= 2 * cap)
    uint64_t* tkey = nullptr;    // table keys (kVfEmpty = free)
    VfSlot* tslot = nullptr;
    int32_t* sslot = nullptr;    // per sample: table slot, -1 = non-finite point
    float* samp = nullptr;       // per sample: its point (compact AoS float3; the raw scan is read once)
    int2* loc = nullptr;         // per head sample: (output slot, bucket start) inside its k_vf_heads block
    int2* blk = nullptr;         // per k_vf_heads block: (heads, members)
    int2* blk_pre = nullptr;     // their exclusive prefix (+ the total), published by k_vf_place's block 0
    int32_t* bucket = nullptr;   // members of each voxel (bucket order = arrival order; sorted when summed)
    int32_t* mid = nullptr;      // head samples of voxels with 17..64 members
    int32_t* big = nullptr;      // head samples of voxels with more than 64 members
    VfCounters* ctr = nullptr;
    int* n_out = nullptr;        // &ctr->n_out
};

hipError_t vf_reserve(VfBuffers& b, size_t m, hipStream_t s);
void vf_free(VfBuffers& b);
// Filter d_raw (n_raw AoS float3) into d_out on stream s; the output count lands in b.n_out (device).
// m_out = ceil(n_raw / stride), an upper bound of the output count.
hipError_t vf_enqueue(VfBuffers& b, const float* d_raw, size_t n_raw, int stride, float voxel_size, float* d_out,
                      hipStream_t s, int& m_out);

}  // namespace lo
