/*
 * GpuIterativeClosestPointOptimizer.h -- the reference-side binding of the MI355X ICP core.
 *
 * A header a maintainer adds to the reference tree (SiarheiHerasiuta/lidar_odometry), compiled with its include root
 * (-I<reference>/src) and this repository's include/ directory, linked against lidar_odometry_amd/liblo_icp.so.  It
 * has the interface of lidar_slam::optimization::IterativeClosestPointOptimizer
 * (src/optimization/IterativeClosestPointOptimizer.h:42-43, :159-227):
 *   - constructed from `const ICPConfig&` + `std::shared_ptr<AdaptiveMEstimator>` (:165-166); the estimator's
 *     AdaptiveMEstimatorConfig (AdaptiveMEstimator.h:27-41, reached via get_config(), :85) gives the PKO parameters,
 *     the ICP's loss_type (read at IterativeClosestPointOptimizer.cpp:354-357) and pko_kernel_type (every kernel of
 *     AdaptiveMEstimator.cpp:128-156; an unknown name is Cauchy there and here);
 *   - bool optimize(map::VoxelMap*, std::shared_ptr<database::LidarFrame>, const SE3f&, SE3f&) (:182-185) with the
 *     reference's contract (IterativeClosestPointOptimizer.cpp:255-463): false <=> a GN iteration found fewer than
 *     min_correspondence_points correspondences, optimized_transform == initial_transform then (:266, :298-302);
 *   - bool optimize_loop(...) (:194-197, IterativeClosestPointOptimizer.cpp:40-251);
 *   - const OptimizationStats& get_last_stats() (:203-215), filled as the reference fills it;
 *   - update_config / get_config (:220-225).
 * The map the kernels read is a device copy of the VoxelMap's L1 surfels (VoxelMap::GetSurfelAtPoint's table,
 * VoxelMap.cpp:368-386).  sync_map() reads it from the map's PUBLIC interface only and sends the device only the
 * surfels that changed since the previous sync (lo_map_sync_surfels); call it after every mutation
 * (Estimator.cpp:457 UpdateVoxelMap, :877 / :1181 ApplyTransformAndRehash).  In the KDTree configuration
 * (use_surfel_correspondence = false) it uploads VoxelMap::GetPointCloud() instead (RebuildKdTree's input, :461).
 *
 * Nothing here is compiled in this repository (the reference needs the system Eigen3 this image lacks);
 * tests/test_integration_adapter.py checks every reference identifier it names against the reference headers.
 */
#pragma once

#include <chrono>
#include <cmath>
#include <memory>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include "database/LidarFrame.h"
#include "database/VoxelMap.h"
#include "optimization/AdaptiveMEstimator.h"
#include "optimization/IterativeClosestPointOptimizer.h"
#include "util/MathUtils.h"
#include "util/PointCloudUtils.h"

#include "lo_icp.h"

namespace lidar_slam {
namespace optimization {

class GpuIterativeClosestPointOptimizer {
public:
    using OptimizationStats = IterativeClosestPointOptimizer::OptimizationStats;

    // Estimator.cpp:62-72 builds the reference optimizer from exactly these two objects.  map_voxel_size /
    // hierarchy_factor: the VoxelMap's geometry (VoxelMap::GetVoxelSize / GetHierarchyFactor, VoxelMap.h:204-205;
    // Estimator.cpp:75-80 sets them from map_voxel_size and 3).  device: the HIP device of this optimizer's context.
    GpuIterativeClosestPointOptimizer(const ICPConfig& config, std::shared_ptr<AdaptiveMEstimator> adaptive_estimator,
                                      float map_voxel_size, int hierarchy_factor = 3, int device = 0,
                                      int max_points = 1 << 17)
        : m_config(config), m_adaptive_estimator(std::move(adaptive_estimator)), m_voxel_size(map_voxel_size),
          m_hierarchy_factor(hierarchy_factor), m_device(device), m_max_points(max_points) {
        create_context();
    }
    ~GpuIterativeClosestPointOptimizer() { lo_destroy(m_ctx); }
    GpuIterativeClosestPointOptimizer(const GpuIterativeClosestPointOptimizer&) = delete;
    GpuIterativeClosestPointOptimizer& operator=(const GpuIterativeClosestPointOptimizer&) = delete;

    bool optimize(map::VoxelMap* voxel_map, std::shared_ptr<database::LidarFrame> curr_frame,
                  const SE3f& initial_transform, SE3f& optimized_transform) {
        (void)voxel_map;                                     // its surfels are on the device since sync_map()
        m_last_stats = OptimizationStats();                  // :262
        optimized_transform = initial_transform;            // :266
        util::PointCloudConstPtr cloud = frame_cloud(curr_frame);          // get_frame_cloud :769-783
        const float* xyz = cloud ? &cloud->points[0].x : nullptr;          // Point3D = AoS float x, y, z
        const size_t n = cloud ? cloud->size() : 0;
        float T0[12], T1[12];
        to_row_major(initial_transform, T0);
        std::vector<lo_iter_log> logs(static_cast<size_t>(m_config.max_iterations));
        lo_stats st{};
        const int rc = lo_icp_optimize(m_ctx, xyz, n, T0, T1, logs.data(), &st);
        if (rc < 0) throw std::runtime_error(std::string("lo_icp_optimize: ") + lo_last_error(m_ctx));
        // curr_frame->set_pose(T) runs at the start of every iteration (:284): the frame ends at the pose the last
        // attempted iteration started from (a failing iteration is attempted too)
        const int attempted = st.iterations + (rc == LO_OK ? 0 : 1);
        curr_frame->set_pose(attempted >= 2 ? from_row_major(logs[attempted - 2].pose) : initial_transform);
        // num_correspondences is set once an iteration passed its check (:340), the rest only on success (:452-460)
        m_last_stats.num_correspondences = st.iterations > 0 ? static_cast<size_t>(logs[st.iterations - 1].n_corr) : 0;
        if (rc != LO_OK) return false;                       // :298-302 (LOG_WARN there)
        optimized_transform = from_row_major(T1);
        m_last_stats.num_iterations = static_cast<size_t>(st.iterations);
        m_last_stats.initial_cost = st.initial_cost;
        m_last_stats.final_cost = st.final_cost;
        m_last_stats.converged = true;                       // always true on success (:456)
        // the reference's is whole milliseconds of host wall time (duration_cast<milliseconds>); this is the device
        // time of the whole GN loop (HIP events), fractional
        m_last_stats.optimization_time_ms = st.gpu_ms;
        return true;
    }

    bool optimize_loop(std::shared_ptr<database::LidarFrame> curr_keyframe,
                       std::shared_ptr<database::LidarFrame> matched_keyframe, SE3f& optimized_relative_transform,
                       float& inlier_ratio) {
        util::PointCloudConstPtr cur = frame_cloud(curr_keyframe), mat = frame_cloud(matched_keyframe);
        float Tc[12], Tm[12], Tr[12];
        to_row_major(curr_keyframe->get_pose(), Tc);
        to_row_major(matched_keyframe->get_pose(), Tm);
        lo_stats st{};
        const int rc = lo_icp_optimize_loop(m_ctx, cur ? &cur->points[0].x : nullptr, cur ? cur->size() : 0, Tc,
                                            mat ? &mat->points[0].x : nullptr, mat ? mat->size() : 0, Tm, Tr,
                                            &inlier_ratio, nullptr, &st);
        if (rc < 0) throw std::runtime_error(std::string("lo_icp_optimize_loop: ") + lo_last_error(m_ctx));
        if (st.converged) optimized_relative_transform = from_row_major(Tr);   // written only on convergence (:240)
        return rc == LO_OK;
    }

    // The device map from the VoxelMap's public interface: every L1 surfel (GetL1Surfels, VoxelMap.cpp:405-418)
    // filed under its L1 key.  The key is PointToVoxelKey(centroid, 1) (VoxelMap.cpp:50-58) confirmed through
    // GetSurfelAtPoint at the key's voxel centre, or the neighbouring voxel whose centre returns this surfel (a
    // centroid on an L1 face may round across it).  KDTree configuration: GetPointCloud() (L0 centroids, L0 order).
    void sync_map(const map::VoxelMap& vm) {
        if (!m_config.use_surfel_correspondence) {
            util::PointCloudPtr cloud = vm.GetPointCloud();
            check(lo_map_set_points(m_ctx, cloud && !cloud->empty() ? &cloud->points[0].x : nullptr,
                                    cloud ? cloud->size() : 0), "lo_map_set_points");
            return;
        }
        const float l1 = vm.GetVoxelSize() * static_cast<float>(vm.GetHierarchyFactor());
        std::vector<int32_t> keys;
        std::vector<float> nrm, ctr;
        for (const auto& s : vm.GetL1Surfels()) {
            const Eigen::Vector3f& c = std::get<0>(s);
            const Eigen::Vector3f& nv = std::get<1>(s);
            int k[3] = {static_cast<int>(std::floor(c.x() / l1)), static_cast<int>(std::floor(c.y() / l1)),
                        static_cast<int>(std::floor(c.z() / l1))};
            if (!find_key(vm, l1, c, nv, k)) continue;       // not reachable by any lookup: never a correspondence
            keys.insert(keys.end(), {k[0], k[1], k[2]});
            nrm.insert(nrm.end(), {nv.x(), nv.y(), nv.z()});
            ctr.insert(ctr.end(), {c.x(), c.y(), c.z()});
        }
        // only the voxels UpdateVoxelMap changed since the last sync reach the device (VoxelMap.cpp:187-261: new and
        // refitted surfels, surfels that lost planarity or were pruned); the first sync uploads the whole table
        int patched = 0;
        check(lo_map_sync_surfels(m_ctx, keys.data(), nrm.data(), ctr.data(), keys.size() / 3, &patched),
              "lo_map_sync_surfels");
        m_last_sync_patched = patched;
        m_synced_once = true;
    }
    // The keyed sync: only the L1 voxels UpdateVoxelMap changed reach the device.  `changed` is what
    // the two-line hook in VoxelMap::UpdateVoxelMap collects (INTEGRATION.md "Incremental map sync"): the parents of
    // the pruned L0 voxels (:146-169) and every key of the touched loop (:187-261).  Each key's surfel is read with
    // GetSurfelAtPoint at the voxel's centre (PointToVoxelKey(centre, 1) is the key itself, :50-58) and patched in
    // place (lo_map_patch_surfels: upsert, or erase when the voxel has none) -- O(changed voxels) on the host, no walk
    // over the whole surfel set and no key search.  The first sync, a table too full for the patch, or the KDTree
    // configuration fall back to the full sync_map(vm).
    void sync_map(const map::VoxelMap& vm, const std::vector<map::VoxelKey>& changed) {
        if (!m_config.use_surfel_correspondence || !m_synced_once) { sync_map(vm); return; }
        const float l1 = vm.GetVoxelSize() * static_cast<float>(vm.GetHierarchyFactor());
        std::vector<int32_t> keys;
        std::vector<float> nrm, ctr;
        std::vector<uint8_t> present;
        keys.reserve(3 * changed.size());
        nrm.reserve(3 * changed.size());
        ctr.reserve(3 * changed.size());
        present.reserve(changed.size());
        for (const map::VoxelKey& k : changed) {
            const Eigen::Vector3f centre((static_cast<float>(k.x) + 0.5f) * l1, (static_cast<float>(k.y) + 0.5f) * l1,
                                         (static_cast<float>(k.z) + 0.5f) * l1);
            Eigen::Vector3f n = Eigen::Vector3f::Zero(), c = Eigen::Vector3f::Zero();
            const bool has = vm.GetSurfelAtPoint(centre, n, c);
            keys.insert(keys.end(), {k.x, k.y, k.z});
            nrm.insert(nrm.end(), {n.x(), n.y(), n.z()});
            ctr.insert(ctr.end(), {c.x(), c.y(), c.z()});
            present.push_back(has ? 1 : 0);
        }
        const int rc = lo_map_patch_surfels(m_ctx, keys.data(), nrm.data(), ctr.data(), present.data(), present.size());
        if (rc == LO_ERR_CAPACITY) { sync_map(vm); return; }   // tombstones: a full upload rebuilds the table
        check(rc, "lo_map_patch_surfels");
        m_last_sync_patched = static_cast<int>(present.size());
    }
    int last_sync_patched() const { return m_last_sync_patched; }   // records sent by the last sync_map (-1: full)

    const OptimizationStats& get_last_stats() const { return m_last_stats; }
    void update_config(const ICPConfig& config) {            // :220: only the parameters change; the device map stays
        lo_config c = make_config(config);
        check(lo_update_config(m_ctx, &c), "lo_update_config");
        m_config = config;
    }
    const ICPConfig& get_config() const { return m_config; }
    lo_ctx* context() const { return m_ctx; }                // reference-exact by default; lo_set_exact(context(), 0) =
                                                             // the opt-in fast mode (not parity-safe)

private:
    lo_config make_config(const ICPConfig& cfg) const {
        lo_config c;
        lo_config_default_kitti(&c);
        c.max_iterations = cfg.max_iterations;
        c.translation_tolerance = cfg.translation_tolerance;
        c.rotation_tolerance = cfg.rotation_tolerance;
        c.max_correspondence_distance = cfg.max_correspondence_distance;
        c.min_correspondence_points = cfg.min_correspondence_points;
        c.use_robust_loss = cfg.use_robust_loss ? 1 : 0;
        c.robust_loss_delta = cfg.robust_loss_delta;
        c.use_surfel_correspondence = cfg.use_surfel_correspondence ? 1 : 0;
        // outlier_rejection_ratio, use_kdtree, max_kdtree_neighbors: not read by optimize
        c.use_adaptive_m_estimator = 0;                      // no estimator: robust_loss_delta, Huber (:70-73, :320)
        c.loss_cauchy = 0;
        if (m_adaptive_estimator) {
            const AdaptiveMEstimatorConfig& p = m_adaptive_estimator->get_config();
            c.use_adaptive_m_estimator = p.use_adaptive_m_estimator ? 1 : 0;
            c.loss_cauchy = p.loss_type == "cauchy" ? 1 : 0; // :354-357, :394: anything else weighs as Huber
            c.min_scale_factor = p.min_scale_factor;
            c.max_scale_factor = p.max_scale_factor;
            c.num_alpha_segments = p.num_alpha_segments;
            c.truncated_threshold = p.truncated_threshold;
            c.gmm_components = p.gmm_components;
            c.gmm_sample_size = p.gmm_sample_size;
            c.pko_kernel = lo_pko_kernel_from_name(p.pko_kernel_type.c_str());
            // scale_method / fixed_scale_factor: calculate_scale_factor always runs PKO (AdaptiveMEstimator.cpp:63-79)
        }
        c.voxel_size = m_voxel_size;
        c.hierarchy_factor = m_hierarchy_factor;
        c.max_points = m_max_points;
        return c;
    }
    void create_context() {
        lo_config c = make_config(m_config);
        int err = 0;
        m_ctx = lo_create(&c, m_device, &err);   // rejects what the device kernels cannot take (gmm_components > 3, ...)
        if (!m_ctx) throw std::runtime_error("lo_create failed with code " + std::to_string(err));
    }

    static util::PointCloudConstPtr frame_cloud(const std::shared_ptr<database::LidarFrame>& frame) {
        util::PointCloudConstPtr feature = frame->get_feature_cloud();
        if (feature && !feature->empty()) return feature;
        util::PointCloudConstPtr processed = frame->get_processed_cloud();
        if (processed && !processed->empty()) return processed;
        return nullptr;
    }

    static bool find_key(const map::VoxelMap& vm, float l1, const Eigen::Vector3f& c, const Eigen::Vector3f& nv,
                         int (&k)[3]) {
        for (int dz = 0; dz < 3; ++dz)                       // offsets 0, -1, +1 per axis, the computed key first
            for (int dy = 0; dy < 3; ++dy)
                for (int dx = 0; dx < 3; ++dx) {
                    const int o[3] = {dx == 2 ? -1 : dx, dy == 2 ? -1 : dy, dz == 2 ? -1 : dz};
                    const Eigen::Vector3f centre((static_cast<float>(k[0] + o[0]) + 0.5f) * l1,
                                                 (static_cast<float>(k[1] + o[1]) + 0.5f) * l1,
                                                 (static_cast<float>(k[2] + o[2]) + 0.5f) * l1);
                    Eigen::Vector3f n2, c2;
                    if (vm.GetSurfelAtPoint(centre, n2, c2) && n2 == nv && c2 == c) {
                        for (int a = 0; a < 3; ++a) k[a] += o[a];
                        return true;
                    }
                }
        return false;
    }

    void check(int rc, const char* what) const {
        if (rc != LO_OK) throw std::runtime_error(std::string(what) + ": " + lo_last_error(m_ctx));
    }

    static void to_row_major(const SE3f& T, float out[12]) {
        const Eigen::Matrix3f R = T.RotationMatrix();       // MathUtils.h:137
        const Eigen::Vector3f& t = T.Translation();          // :140
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) out[r * 4 + c] = R(r, c);
            out[r * 4 + 3] = t[r];
        }
    }
    // The device's pose is the reference's current_transform bit for bit: its rotation already came out of
    // SE3::operator*'s SO3(Matrix3f) projection (MathUtils.h:144-147).  SE3f(R, t) would run that JacobiSVD projection a
    // second time (MathUtils.h:116-117, MathUtils.cpp:86-92), and the fp32 projection is not idempotent: re-projecting
    // the exact mode's poses moves entries by up to ~3e-7 (tests/test_integration_adapter.py
    // test_so3_reprojection_not_idempotent).  So the matrix is written into a default SE3f through the mutable accessors
    // (MathUtils.h:75, :131, :140), which copy without projecting -- what `optimized_transform = current_transform`
    // (:452) hands the caller.
    static SE3f from_row_major(const float T[12]) {
        SE3f out;
        Eigen::Matrix3f& R = out.Rotation().Matrix();
        Eigen::Vector3f& t = out.Translation();
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) R(r, c) = T[r * 4 + c];
            t[r] = T[r * 4 + 3];
        }
        return out;
    }

    ICPConfig m_config;
    std::shared_ptr<AdaptiveMEstimator> m_adaptive_estimator;
    float m_voxel_size;
    int m_hierarchy_factor;
    int m_device;
    int m_max_points;
    OptimizationStats m_last_stats;
    int m_last_sync_patched = 0;
    bool m_synced_once = false;                         // a whole-map sync_map ran (the keyed one patches on top)
    lo_ctx* m_ctx = nullptr;
};

}  // namespace optimization
}  // namespace lidar_slam
