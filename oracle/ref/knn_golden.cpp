// knn_golden.cpp — golden-vector generator for the KDTree correspondence variant's 5-NN.  TEST INFRASTRUCTURE ONLY.
//
// Built by oracle/Makefile (target `ref`) against the REFERENCE's vendored nanoflann 1.7.1 header, in place under
// /root/reference/thirdparty/nanoflann (output only into oracle/_ref/).  The index is configured exactly as the
// reference's util::KdTree does (src/util/PointCloudUtils.h:346-423): KDTreeSingleIndexAdaptor over
// L2_Simple_Adaptor<float, adapter>, DIM 3, KDTreeSingleIndexAdaptorParams(10) (leaf size 10, single-threaded
// build), an adapter returning Point3D x/y/z with no user bounding box, and knnSearch(query, k, uint32 indices,
// float distances) -- so the neighbour sets, their order and their tie-breaks are nanoflann's own.
//
// Input (binary, little endian): int32 m, float32 cloud[m][3], int32 nq, float32 queries[nq][3], int32 k.
// Output (binary): per query int32 found, uint32 idx[k], float32 dist[k] (unused slots 0xffffffff / +inf).
#include "nanoflann.hpp"

#include <cstdint>
#include <cstdio>
#include <limits>
#include <vector>

namespace {

struct Pt { float x, y, z; };

// the reference's PointCloudAdapter (PointCloudUtils.h:346-365)
struct Adapter {
    const std::vector<Pt>& cloud;
    explicit Adapter(const std::vector<Pt>& c) : cloud(c) {}
    size_t kdtree_get_point_count() const { return cloud.size(); }
    float kdtree_get_pt(const size_t idx, const size_t dim) const {
        const Pt& p = cloud.at(idx);
        switch (dim) {
            case 0: return p.x;
            case 1: return p.y;
            case 2: return p.z;
            default: return 0.0f;
        }
    }
    template <class BBOX>
    bool kdtree_get_bbox(BBOX&) const { return false; }
};

using Tree = nanoflann::KDTreeSingleIndexAdaptor<nanoflann::L2_Simple_Adaptor<float, Adapter>, Adapter, 3>;

bool read_all(FILE* f, void* p, size_t bytes) { return std::fread(p, 1, bytes, f) == bytes; }

}  // namespace

int main(int argc, char** argv) {
    if (argc != 3) { std::fprintf(stderr, "usage: knn_golden in.bin out.bin\n"); return 2; }
    FILE* fi = std::fopen(argv[1], "rb");
    if (!fi) return 3;
    int32_t m = 0, nq = 0, k = 0;
    if (!read_all(fi, &m, 4) || m < 0) return 4;
    std::vector<Pt> cloud(static_cast<size_t>(m));
    if (m && !read_all(fi, cloud.data(), sizeof(Pt) * m)) return 4;
    if (!read_all(fi, &nq, 4) || nq < 0) return 4;
    std::vector<Pt> qs(static_cast<size_t>(nq));
    if (nq && !read_all(fi, qs.data(), sizeof(Pt) * nq)) return 4;
    if (!read_all(fi, &k, 4) || k < 1) return 4;
    std::fclose(fi);

    FILE* fo = std::fopen(argv[2], "wb");
    if (!fo) return 5;
    Adapter ad(cloud);
    std::vector<uint32_t> idx(k);
    std::vector<float> dist(k);
    if (m == 0) {                               // KdTree::setInputCloud leaves no tree: nearestKSearch finds 0
        for (int32_t q = 0; q < nq; ++q) {
            const int32_t found = 0;
            std::fwrite(&found, 4, 1, fo);
            for (int j = 0; j < k; ++j) { idx[j] = 0xffffffffu; dist[j] = std::numeric_limits<float>::infinity(); }
            std::fwrite(idx.data(), 4, k, fo);
            std::fwrite(dist.data(), 4, k, fo);
        }
        std::fclose(fo);
        return 0;
    }
    Tree tree(3, ad, nanoflann::KDTreeSingleIndexAdaptorParams(10));
    tree.buildIndex();                          // as KdTree::setInputCloud (PointCloudUtils.h:391-392)
    for (int32_t q = 0; q < nq; ++q) {
        const float query[3] = {qs[q].x, qs[q].y, qs[q].z};
        for (int j = 0; j < k; ++j) { idx[j] = 0xffffffffu; dist[j] = std::numeric_limits<float>::infinity(); }
        const int32_t found = static_cast<int32_t>(tree.knnSearch(query, static_cast<size_t>(k), idx.data(), dist.data()));
        for (int j = found; j < k; ++j) { idx[j] = 0xffffffffu; dist[j] = std::numeric_limits<float>::infinity(); }
        std::fwrite(&found, 4, 1, fo);
        std::fwrite(idx.data(), 4, k, fo);
        std::fwrite(dist.data(), 4, k, fo);
    }
    std::fclose(fo);
    return 0;
}
