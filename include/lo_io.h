/* lo_io.h — on-disk formats either side of the ICP step, host C++ in liblo_icp.so.
 *
 * Counts are returned as long long (negative = error).  Passing out_xyz = NULL returns the number of points
 * the file holds (for sizing); otherwise at most cap points are written as AoS float3 (Point3D).
 */
#ifndef LO_IO_H
#define LO_IO_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LO_IO_ERR_ARG  (-1)
#define LO_IO_ERR_OPEN (-2)

/* util::load_kitti_binary (src/util/PointCloudUtils.cpp:18-65): float32 (x, y, z, intensity) records,
 * intensity dropped, a trailing partial record ignored. */
long long lo_load_kitti_bin(const char* path, float* out_xyz, size_t cap);

/* PLYPlayer::load_ply_point_cloud + parse_ply_header (app/player/ply_player.cpp:267-461): ASCII or binary
 * vertex x/y/z with the reference's quirks (every "property" line counts toward the vertex stride; x/y/z are
 * read as 4-byte floats whatever their declared type; no byte swap for binary_big_endian).  A file without
 * x/y/z or vertices yields 0 points, as the reference's empty cloud. */
long long lo_load_ply(const char* path, float* out_xyz, size_t cap);

/* KittiPlayer::pose_to_kitti_string (app/player/kitti_player.cpp:934-953): the 3x4 LiDAR pose (row-major)
 * moved to the KITTI camera frame (T_lidar_to_cam * pose * T_lidar_to_cam^-1), 12 numbers, std::fixed,
 * 9 decimals (signed zeros printed as 0).  Returns the string length, or LO_IO_ERR_ARG if cap is too small. */
int lo_kitti_pose_line(const float pose_3x4[12], char* out, size_t cap);

/* KittiPlayer::save_trajectory_kitti_format (:530-546): one lo_kitti_pose_line per pose. 0 on success. */
int lo_save_trajectory_kitti(const char* path, const float* poses_3x4, size_t n);

#ifdef __cplusplus
}
#endif

#endif
