// lo_io.cpp — the on-disk formats either side of the ICP step, host C++:
//   * KITTI velodyne .bin (util::load_kitti_binary, src/util/PointCloudUtils.cpp:18-65);
//   * PLY point clouds (PLYPlayer::load_ply_point_cloud / parse_ply_header, app/player/ply_player.cpp:267-461);
//   * KITTI trajectory lines with the LiDAR -> camera frame change (KittiPlayer::pose_to_kitti_string,
//     app/player/kitti_player.cpp:934-953; save_trajectory_kitti_format :530-546).
// Parsing follows the reference's stream semantics, including its quirks (noted inline), so a file loads to
// the same points here as there.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/lo_io.h"

namespace {

struct PlyProp {
    std::string name, type;
    size_t bytes;
};

size_t ply_type_size(const std::string& t) {                    // get_type_size (:392-398)
    if (t == "char" || t == "uchar" || t == "int8" || t == "uint8") return 1;
    if (t == "short" || t == "ushort" || t == "int16" || t == "uint16") return 2;
    if (t == "int" || t == "uint" || t == "float" || t == "int32" || t == "uint32" || t == "float32") return 4;
    if (t == "double" || t == "float64") return 8;
    return 4;                                                    // default to float
}

// parse_ply_header (:371-461).  Quirks kept: every "property" line counts as a vertex property, whatever
// element it belongs to; "binary_big_endian" is read without byte swapping; lines must match exactly
// (a "\r\n" file never reaches end_header).
bool ply_header(const char* path, size_t& vertex_count, std::vector<PlyProp>& props, bool& binary) {
    std::ifstream f(path);
    if (!f.is_open()) return false;
    vertex_count = 0;
    props.clear();
    binary = false;
    std::string line;
    bool in_header = false;
    int xi = -1, yi = -1, zi = -1;
    while (std::getline(f, line)) {
        if (line == "ply") { in_header = true; continue; }
        if (!in_header) continue;
        if (line == "end_header") break;
        std::istringstream iss(line);
        std::string tok;
        iss >> tok;
        if (tok == "format") {
            std::string fmt;
            iss >> fmt;
            binary = (fmt == "binary_little_endian" || fmt == "binary_big_endian");
        } else if (tok == "element") {
            std::string et;
            iss >> et;
            if (et == "vertex") iss >> vertex_count;
        } else if (tok == "property") {
            std::string type, name;
            iss >> type >> name;
            props.push_back({name, type, ply_type_size(type)});
            const int idx = static_cast<int>(props.size()) - 1;
            if (name == "x") xi = idx;
            else if (name == "y") yi = idx;
            else if (name == "z") zi = idx;
        }
    }
    return xi >= 0 && yi >= 0 && zi >= 0 && vertex_count != 0;
}

}  // namespace

extern "C" {

long long lo_load_kitti_bin(const char* path, float* out_xyz, size_t cap) {
    if (!path) return LO_IO_ERR_ARG;
    std::ifstream f(path, std::ios::binary);
    if (!f.is_open()) return LO_IO_ERR_OPEN;
    f.seekg(0, std::ios::end);
    const size_t size = static_cast<size_t>(f.tellg());
    f.seekg(0, std::ios::beg);
    const size_t n = size / (4 * sizeof(float));                 // x, y, z, intensity records (:41-42)
    if (!out_xyz) return static_cast<long long>(n);
    size_t k = 0;
    float rec[4];
    for (size_t i = 0; i < n && k < cap; ++i) {
        f.read(reinterpret_cast<char*>(rec), sizeof(rec));
        if (f.gcount() != static_cast<std::streamsize>(sizeof(rec))) break;   // incomplete read ends the cloud
        out_xyz[3 * k] = rec[0];
        out_xyz[3 * k + 1] = rec[1];
        out_xyz[3 * k + 2] = rec[2];
        ++k;
    }
    return static_cast<long long>(k);
}

long long lo_load_ply(const char* path, float* out_xyz, size_t cap) {
    if (!path) return LO_IO_ERR_ARG;
    size_t vc = 0;
    std::vector<PlyProp> props;
    bool binary = false;
    {
        std::ifstream probe(path);
        if (!probe.is_open()) return LO_IO_ERR_OPEN;
    }
    if (!ply_header(path, vc, props, binary)) return 0;         // the reference returns an empty cloud
    if (!out_xyz) return static_cast<long long>(vc);
    int xi = -1, yi = -1, zi = -1;
    for (size_t i = 0; i < props.size(); ++i) {
        if (props[i].name == "x") xi = static_cast<int>(i);
        else if (props[i].name == "y") yi = static_cast<int>(i);
        else if (props[i].name == "z") zi = static_cast<int>(i);
    }
    std::ifstream f(path, binary ? std::ios::binary : std::ios::in);
    if (!f.is_open()) return LO_IO_ERR_OPEN;
    std::string line;
    while (std::getline(f, line))
        if (line == "end_header") break;
    size_t k = 0;
    if (binary) {
        size_t bpv = 0;
        for (const auto& p : props) bpv += p.bytes;
        std::vector<char> buf(bpv);
        for (size_t i = 0; i < vc && k < cap; ++i) {
            f.read(buf.data(), static_cast<std::streamsize>(bpv));
            if (!f.good()) break;
            float x = 0.0f, y = 0.0f, z = 0.0f;
            size_t off = 0;
            for (size_t pi = 0; pi < props.size(); ++pi) {       // 4 bytes copied whatever the declared type
                if (static_cast<int>(pi) == xi) std::memcpy(&x, buf.data() + off, sizeof(float));
                else if (static_cast<int>(pi) == yi) std::memcpy(&y, buf.data() + off, sizeof(float));
                else if (static_cast<int>(pi) == zi) std::memcpy(&z, buf.data() + off, sizeof(float));
                off += props[pi].bytes;
            }
            out_xyz[3 * k] = x;
            out_xyz[3 * k + 1] = y;
            out_xyz[3 * k + 2] = z;
            ++k;
        }
    } else {
        for (size_t i = 0; i < vc && k < cap; ++i) {
            if (!std::getline(f, line)) break;
            std::istringstream iss(line);
            std::vector<float> vals;
            float v;
            while (iss >> v) vals.push_back(v);
            if (vals.size() >= props.size()) {                   // short lines are skipped (:339-344)
                out_xyz[3 * k] = vals[xi];
                out_xyz[3 * k + 1] = vals[yi];
                out_xyz[3 * k + 2] = vals[zi];
                ++k;
            }
        }
    }
    return static_cast<long long>(k);
}

// converted = T_lidar_to_cam * pose * T_cam_to_lidar with T_lidar_to_cam = [[0,-1,0],[0,0,-1],[1,0,0]]: an exact
// signed permutation of the pose entries (every product term is 0 or +-x), written with std::fixed and 9 decimals.
int lo_kitti_pose_line(const float pose_3x4[12], char* out, size_t cap) {
    if (!pose_3x4 || !out || cap == 0) return LO_IO_ERR_ARG;
    const float* P = pose_3x4;
    auto p = [&](int r, int c) { return P[r * 4 + c]; };
    // camera axes: x_c = -y_l, y_c = -z_l, z_c = x_l  =>  C = A P A^T with rows of A = (-e_y, -e_z, e_x)
    const int src[3] = {1, 2, 0};
    const float sgn[3] = {-1.0f, -1.0f, 1.0f};
    float C[12];
    for (int r = 0; r < 3; ++r) {
        for (int c = 0; c < 3; ++c) C[r * 4 + c] = sgn[r] * sgn[c] * p(src[r], src[c]);
        C[r * 4 + 3] = sgn[r] * p(src[r], 3);
    }
    for (float& v : C) if (v == 0.0f) v = 0.0f;                 // print signed zeros as 0.000000000
    std::ostringstream oss;
    oss.setf(std::ios::fixed);
    oss.precision(9);
    for (int k = 0; k < 12; ++k) {
        if (k) oss << ' ';
        oss << C[k];
    }
    const std::string s = oss.str();
    if (s.size() + 1 > cap) return LO_IO_ERR_ARG;
    std::memcpy(out, s.c_str(), s.size() + 1);
    return static_cast<int>(s.size());
}

int lo_save_trajectory_kitti(const char* path, const float* poses_3x4, size_t n) {
    if (!path || (n > 0 && !poses_3x4)) return LO_IO_ERR_ARG;
    std::ofstream f(path);
    if (!f.is_open()) return LO_IO_ERR_OPEN;
    char line[512];
    for (size_t i = 0; i < n; ++i) {
        if (lo_kitti_pose_line(poses_3x4 + 12 * i, line, sizeof(line)) < 0) return LO_IO_ERR_ARG;
        f << line << '\n';
    }
    return f.good() ? 0 : LO_IO_ERR_OPEN;
}

}  // extern "C"
