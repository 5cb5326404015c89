// map_order_golden.cpp — golden iteration orders of the voxel map's containers.  TEST INFRASTRUCTURE ONLY.
//
// Built by oracle/Makefile (target `ref`) against the REFERENCE's vendored ankerl::unordered_dense 4.8.1
// (/root/reference/thirdparty/unordered_dense, in place; output only into oracle/_ref/).  The map side's results
// depend on container iteration order: GetPointCloud (VoxelMap.cpp:388-403) follows m_voxels_L0, the surfel sums
// (:211-236) follow occupied_children, the surfel pass follows the affected set, and unordered_dense's erase moves
// the last value into the hole (unordered_dense.h do_erase).  The restated containers (oracle DenseMap,
// lo_voxelmap.cpp OrderedMap) claim that order; this program replays the container-operation trace the oracle's
// UpdateVoxelMap / ApplyTransformAndRehash issue (or_map_trace: insert / erase / clear on L0, L1 and the children
// sets) on the real containers, typed as the reference declares them (VoxelMap.h:152-183, :300-324:
// map<VoxelKey, VoxelNode_L0, VoxelKeyHash>, map<VoxelKey, VoxelNode_L1{set<VoxelKey, VoxelKeyHash>}, ...>), with
// the reference's Morton VoxelKeyHash, and writes the real iteration orders at every checkpoint (end of an update).
//
// Input (binary): int32 records of 7 (op, key xyz, child xyz), op codes as lo_oracle.cpp VoxelMap::emit.
// Output (binary): per checkpoint: int32 n0, n1, nc; n0 L0 keys; n1 L1 keys; n1 child counts; nc children (xyz).
#include "unordered_dense.h"

#include <cstdint>
#include <cstdio>
#include <vector>

namespace {

// VoxelKey / VoxelKeyHash as src/database/VoxelMap.h:152-183 declares them (restated: that header needs Eigen)
struct VoxelKey {
    int x, y, z;
    VoxelKey() : x(0), y(0), z(0) {}
    VoxelKey(int x_, int y_, int z_) : x(x_), y(y_), z(z_) {}
    bool operator==(const VoxelKey& o) const { return x == o.x && y == o.y && z == o.z; }
};

struct VoxelKeyHash {
    static inline uint64_t ExpandBits(int32_t v) {
        uint64_t x = static_cast<uint64_t>(v + (1 << 20)) & 0x1fffff;
        x = (x | (x << 32)) & 0x1f00000000ffffULL;
        x = (x | (x << 16)) & 0x1f0000ff0000ffULL;
        x = (x | (x << 8)) & 0x100f00f00f00f00fULL;
        x = (x | (x << 4)) & 0x10c30c30c30c30c3ULL;
        x = (x | (x << 2)) & 0x1249249249249249ULL;
        return x;
    }
    std::size_t operator()(const VoxelKey& k) const {
        return static_cast<std::size_t>(ExpandBits(k.x) | (ExpandBits(k.y) << 1) | (ExpandBits(k.z) << 2));
    }
};

struct NodeL0 { float c[3] = {0, 0, 0}; int hit_count = 1; int point_count = 0; };
struct NodeL1 {
    ankerl::unordered_dense::set<VoxelKey, VoxelKeyHash> occupied_children;
    bool has_surfel = false;
};

using MapL0 = ankerl::unordered_dense::map<VoxelKey, NodeL0, VoxelKeyHash>;
using MapL1 = ankerl::unordered_dense::map<VoxelKey, NodeL1, VoxelKeyHash>;

void put(FILE* f, int32_t v) { std::fwrite(&v, 4, 1, f); }
void put_key(FILE* f, const VoxelKey& k) { put(f, k.x); put(f, k.y); put(f, k.z); }

void checkpoint(FILE* f, const MapL0& L0, const MapL1& L1) {
    int32_t nc = 0;
    for (const auto& kv : L1) nc += static_cast<int32_t>(kv.second.occupied_children.size());
    put(f, static_cast<int32_t>(L0.size()));
    put(f, static_cast<int32_t>(L1.size()));
    put(f, nc);
    for (const auto& kv : L0) put_key(f, kv.first);
    for (const auto& kv : L1) put_key(f, kv.first);
    for (const auto& kv : L1) put(f, static_cast<int32_t>(kv.second.occupied_children.size()));
    for (const auto& kv : L1)
        for (const auto& ck : kv.second.occupied_children) put_key(f, ck);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc != 3) { std::fprintf(stderr, "usage: map_order_golden trace.bin out.bin\n"); return 2; }
    FILE* fi = std::fopen(argv[1], "rb");
    if (!fi) return 3;
    std::vector<int32_t> tr;
    int32_t buf[7];
    while (std::fread(buf, 4, 7, fi) == 7) tr.insert(tr.end(), buf, buf + 7);
    std::fclose(fi);
    FILE* fo = std::fopen(argv[2], "wb");
    if (!fo) return 4;
    MapL0 L0;
    MapL1 L1;
    for (size_t r = 0; r + 7 <= tr.size(); r += 7) {
        const int op = tr[r];
        const VoxelKey k(tr[r + 1], tr[r + 2], tr[r + 3]), c(tr[r + 4], tr[r + 5], tr[r + 6]);
        switch (op) {
            case 1: L0[k]; break;                                        // m_voxels_L0[key] (AddPoint :104)
            case 2: L0.erase(k); break;                                  // m_voxels_L0.erase(key)
            case 3: L1[k]; break;                                        // m_voxels_L1[parent] (:77-80)
            case 4: L1.erase(k); break;                                  // m_voxels_L1.erase(..)
            case 5: L1[k].occupied_children.insert(c); break;            // occupied_children.insert(key_L0)
            case 6: {                                                    // occupied_children.erase(key_L0)
                auto it = L1.find(k);
                if (it != L1.end()) it->second.occupied_children.erase(c);
                break;
            }
            case 7: L0.clear(); break;
            case 8: L1.clear(); break;
            case 9: checkpoint(fo, L0, L1); break;
            default: std::fclose(fo); return 5;
        }
    }
    std::fclose(fo);
    return 0;
}
