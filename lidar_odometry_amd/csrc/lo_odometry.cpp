// lo_odometry.cpp — Estimator::process_frame without loop closure / PGO (see include/lo_odometry.h), host C++
// driving the device path: each frame is one lo_icp_optimize_raw call (device voxel filter + GN loop); the
// pose bookkeeping uses the reference's SE3f algebra (lo_math.h); keyframes update the voxel map: in surfel mode the
// device-resident map (lo_devmap: the filtered scan never leaves the device, the context's table is patched in
// place, no host sync), in KDTree mode the host VoxelMap (bit-identical UpdateVoxelMap restatement) + re-upload.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/lo_map.h"
#include "../../include/lo_odometry.h"
#include "lo_math.h"

using lo::SE3f;

struct lo_odometry {
    lo_odom_config cfg{};
    lo_ctx* icp = nullptr;
    lo_voxelmap* map = nullptr;
    lo_devmap* dmap = nullptr;            // surfel mode (LO_HOST_MAP=1: the host map + patch sync instead)
    std::string err;
    bool initialized = false;
    SE3f initial, prev, velocity, last_kf;
    size_t keyframes = 0;
    std::vector<float> feat, world;
};

static int create_keyframe(lo_odometry* o, const SE3f& pose, lo_odom_frame* info) {
    // create_keyframe (:370-530): world feature cloud -> UpdateVoxelMap(cloud, position, 1.2 max_range) -> device
    const auto t0 = std::chrono::steady_clock::now();
    if (o->dmap) {
        float T[12];
        lo::se3_to12(pose, T);
        int rc = lo_devmap_update_from_scan(o->dmap, T, o->cfg.max_range * 1.2);
        if (rc == LO_OK && !o->cfg.icp.use_surfel_correspondence)
            rc = lo_devmap_sync_points(o->dmap);         // RebuildKdTree (Estimator.cpp:460-462) on the device
        if (rc != LO_OK) { o->err = lo_devmap_last_error(o->dmap); return rc; }
        o->last_kf = pose;
        ++o->keyframes;
        // the map's error bits (an update that overflowed a capacity aborted; tracking would go on against a stale
        // map): copied back behind the update without a sync, read after the next frame's ICP (lo_odom_process)
        if ((rc = lo_devmap_status_async(o->dmap)) != LO_OK) {
            o->err = lo_devmap_last_error(o->dmap);
            return rc;
        }
        if (info) {
            info->keyframe = 1;
            info->map_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        }
        return LO_OK;
    }
    const long long n = lo_filtered_points(o->icp, nullptr, 0);
    if (n < 0) { o->err = lo_last_error(o->icp); return static_cast<int>(n); }
    o->feat.resize(3 * static_cast<size_t>(std::max<long long>(n, 1)));
    lo_filtered_points(o->icp, o->feat.data(), static_cast<size_t>(n));
    o->world.resize(o->feat.size());
    lo::transform_points(pose, o->feat.data(), static_cast<size_t>(n), o->world.data());   // feature_cloud_global
    const double sensor[3] = {pose.t[0], pose.t[1], pose.t[2]};                          // Vector3f -> Vector3d
    int rc = lo_voxelmap_update(o->map, o->world.data(), static_cast<size_t>(n), sensor, o->cfg.max_range * 1.2, 1);
    if (rc == LO_OK) rc = lo_map_sync_voxelmap(o->icp, o->map, nullptr);                 // patch (+ RebuildKdTree)
    if (rc != LO_OK) { o->err = "keyframe map update failed"; return rc; }
    o->last_kf = pose;
    ++o->keyframes;
    if (info) {
        info->keyframe = 1;
        info->map_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return LO_OK;
}

extern "C" {

void lo_odom_config_default_kitti(lo_odom_config* c) {
    std::memset(c, 0, sizeof(*c));
    lo_config_default_kitti(&c->icp);
    c->point_stride = 8;
    c->filter_voxel_size = 0.5f;
    c->max_range = 100.0;
    c->keyframe_distance = 1.0;
    c->keyframe_rotation = 0.3;
    c->planarity_threshold = 0.1f;
}

lo_odometry* lo_odom_create(const lo_odom_config* cfg, int device, int* err) {
    if (!cfg || cfg->point_stride < 1 || !(cfg->filter_voxel_size > 0.0f)) { if (err) *err = LO_ERR_ARG; return nullptr; }
    lo_odometry* o = new (std::nothrow) lo_odometry();
    if (!o) { if (err) *err = LO_ERR_ARG; return nullptr; }
    o->cfg = *cfg;
    o->icp = lo_create(&cfg->icp, device, err);
    if (!o->icp) { delete o; return nullptr; }
    o->map = lo_voxelmap_create(cfg->icp.voxel_size, cfg->icp.hierarchy_factor, cfg->planarity_threshold,
                                cfg->icp.use_surfel_correspondence ? 1 : 0);   // SetComputeSurfels (Estimator.cpp:79)
    if (!o->map) { lo_destroy(o->icp); delete o; if (err) *err = LO_ERR_ARG; return nullptr; }
    if (cfg->icp.use_surfel_correspondence) lo_voxelmap_set_device_fit(o->map, 1);   // refits run in the sync's patch
    const char* hm = std::getenv("LO_HOST_MAP");
    if (!(hm && std::atoi(hm))) {                        // both correspondence modes (KDTree: lo_devmap_sync_points)
        int e = LO_OK;
        size_t max_l0 = size_t(1) << 21;                                   // LO_DEVMAP_MAX_L0: capacity override
        if (const char* cap = std::getenv("LO_DEVMAP_MAX_L0"); cap && std::atoll(cap) > 0) max_l0 = std::atoll(cap);
        o->dmap = lo_devmap_create(o->icp, cfg->icp.voxel_size, cfg->icp.hierarchy_factor, cfg->planarity_threshold,
                                   max_l0, static_cast<size_t>(std::max(cfg->icp.max_points, 16)), &e);
        if (!o->dmap) { lo_voxelmap_destroy(o->map); lo_destroy(o->icp); delete o; if (err) *err = e; return nullptr; }
    }
    if (err) *err = LO_OK;
    return o;
}

void lo_odom_destroy(lo_odometry* o) {
    if (!o) return;
    lo_devmap_destroy(o->dmap);
    lo_voxelmap_destroy(o->map);
    lo_destroy(o->icp);
    delete o;
}

const char* lo_odom_last_error(const lo_odometry* o) { return o ? o->err.c_str() : "null odometry"; }

int lo_odom_set_initial_pose(lo_odometry* o, const float T[12]) {
    if (!o || !T) return LO_ERR_ARG;
    o->initial = lo::se3_from12(T);
    return LO_OK;
}

int lo_odom_set_exact(lo_odometry* o, int enable) {
    if (!o) return LO_ERR_ARG;
    return lo_set_exact(o->icp, enable);
}

int lo_odom_process(lo_odometry* o, const float* raw, size_t n, float T_out[12], lo_odom_frame* info) {
    if (!o || !T_out || (n > 0 && !raw)) return LO_ERR_ARG;
    lo_odom_frame local{};
    lo_odom_frame* fi = info ? info : &local;
    std::memset(fi, 0, sizeof(*fi));
    const int stride = o->cfg.point_stride;
    const float voxel = o->cfg.filter_voxel_size;
    if (!o->initialized) {                                                    // initialize_first_frame (:235-269)
        float tmp[12];
        lo::se3_to12(o->initial, tmp);
        const long long nf = lo_voxel_filter_gpu(o->icp, raw, n, voxel, stride, nullptr, 0);
        if (nf < 0) { o->err = lo_last_error(o->icp); return static_cast<int>(nf); }
        fi->n_filtered = static_cast<int>(nf);
        o->prev = o->initial;
        o->velocity = SE3f();
        if (nf > 0) {
            const int rc = create_keyframe(o, o->initial, fi);
            if (rc != LO_OK) return rc;
        }
        o->initialized = true;
        std::memcpy(T_out, tmp, sizeof(tmp));
        fi->status = LO_OK;
        return LO_OK;
    }
    if (o->keyframes == 0) {
        // the first frame filtered to nothing: the reference made no keyframe and every later frame returns at
        // "No keyframe available" (Estimator.cpp:140-144) without ICP, pose update or keyframe test
        lo::se3_to12(o->prev, T_out);
        fi->status = LO_OK;
        return LO_OK;
    }
    const SE3f guess = lo::se3_mul(o->prev, o->velocity);                    // :154
    // estimate_motion_dual_frame hands optimize SE3f(guess.R, guess.t), i.e. SO3(R) re-projected (:284), and
    // wraps the result the same way (:308); on failure it returns the guess itself (:304-307)
    SE3f g_in = guess;
    lo::so3_project_svd(guess.R, g_in.R);
    float g12[12], p12[12];
    lo::se3_to12(g_in, g12);
    lo_iter_log logs[LO_MAX_ITERS];
    lo_stats st{};
    int rc = lo_icp_optimize_raw(o->icp, raw, n, stride, voxel, g12, p12, logs, &st);
    if (rc < 0) { o->err = lo_last_error(o->icp); return rc; }
    if (o->dmap) {      // the last keyframe's map update: the ICP's sync has drained it (same stream), so no wait here
        const int mrc = lo_devmap_status_poll(o->dmap);
        if (mrc != LO_OK) { o->err = lo_devmap_last_error(o->dmap); return mrc; }
    }
    fi->status = rc;
    fi->icp_iterations = st.iterations;
    fi->n_corr = st.n_corr;
    fi->device_ms = st.gpu_ms;
    const long long nf = lo_filtered_points(o->icp, nullptr, 0);
    fi->n_filtered = static_cast<int>(nf > 0 ? nf : 0);
    SE3f pose = guess;
    if (rc == LO_OK) {
        const SE3f r = lo::se3_from12(p12);
        pose = r;
        lo::so3_project_svd(r.R, pose.R);
    }
    lo::se3_to12(pose, p12);
    o->velocity = lo::se3_mul(lo::se3_inv(o->prev), pose);                    // :177
    o->prev = pose;
    // should_create_keyframe (:349-368)
    const float dt[3] = {pose.t[0] - o->last_kf.t[0], pose.t[1] - o->last_kf.t[1], pose.t[2] - o->last_kf.t[2]};
    const float dist = std::sqrt(lo::dot3e(dt[0], dt[1], dt[2], dt[0], dt[1], dt[2]));
    float Rki[3][3], Rkt[3][3], Rrel[3][3], Rrel_p[3][3];
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) Rkt[r][c] = o->last_kf.R[c][r];
    lo::so3_project_svd(Rkt, Rki);                                                // SO3::Inverse -> SO3(R^T)
    lo::mul33e(Rki, pose.R, Rrel);
    lo::so3_project_svd(Rrel, Rrel_p);                                            // SO3::operator*
    const double ang = lo::so3_log_norm(Rrel_p);
    if (static_cast<double>(dist) > o->cfg.keyframe_distance || ang > o->cfg.keyframe_rotation) {
        const int krc = create_keyframe(o, pose, fi);
        if (krc != LO_OK) return krc;
    }
    std::memcpy(T_out, p12, sizeof(p12));
    return rc;
}

int lo_odom_flush(lo_odometry* o) {
    if (!o) return LO_ERR_ARG;
    if (!o->dmap) return LO_OK;                          // the host map reports inside lo_voxelmap_update
    const int rc = lo_devmap_status(o->dmap);            // synchronous: the last update's error bits
    if (rc != LO_OK) o->err = lo_devmap_last_error(o->dmap);
    return rc;
}

size_t lo_odom_keyframe_count(const lo_odometry* o) { return o ? o->keyframes : 0; }
size_t lo_odom_map_surfels(const lo_odometry* o) {
    if (!o) return 0;
    if (o->dmap) {
        size_t c[4] = {0, 0, 0, 0};
        lo_devmap_counts(o->dmap, c);
        return c[2];
    }
    return lo_voxelmap_surfel_count(o->map);
}

}  // extern "C"
