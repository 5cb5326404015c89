// lo_ctx_internal.h — library-internal accessors of an ICP context (C++ linkage, not part of the C ABI).
#pragma once
#include <cstdint>

#include "../../include/lo_icp.h"

namespace lo {
// Which host voxel map the context's device surfel table mirrors, and at which journal position / epoch
// (lo_map_sync_voxelmap); src = 0 after any other table upload.
void ctx_map_source(const lo_ctx* c, uint64_t* src, uint64_t* epoch, uint64_t* pos);
void ctx_set_map_source(lo_ctx* c, uint64_t src, uint64_t epoch, uint64_t pos);
}  // namespace lo
