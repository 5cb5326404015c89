// lo_vfilter.h — device FastVoxelFilter (lo_vfilter.hip), host-side interface for lo_icp.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace lo {

struct VfBuffers {
    size_t cap = 0;
    uint64_t* keys = nullptr;
    uint64_t* keys_s = nullptr;
    int32_t* idx = nullptr;
    int32_t* idx_s = nullptr;
    int32_t* first = nullptr;
    int32_t* pos = nullptr;
    float4* pts_s = nullptr;     // sample coordinates in sorted order, .w = voxel head mark
    void* temp = nullptr;
    size_t temp_bytes = 0;
    int* n_out = nullptr;
};

hipError_t vf_reserve(VfBuffers& b, size_t m);
void vf_free(VfBuffers& b);
// Filter d_raw (n_raw AoS float3) into d_out on stream s; the output count lands in b.n_out (device).
// m_out = ceil(n_raw / stride), an upper bound of the output count.
hipError_t vf_enqueue(VfBuffers& b, const float* d_raw, size_t n_raw, int stride, float voxel_size, float* d_out,
                      hipStream_t s, int& m_out);

}  // namespace lo
