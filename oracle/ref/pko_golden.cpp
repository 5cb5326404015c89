// pko_golden.cpp — golden-vector generator for the PKO oracle.  TEST INFRASTRUCTURE ONLY.
//
// Linked against the REFERENCE's own src/optimization/AdaptiveMEstimator.cpp, compiled in place from
// /root/reference by oracle/Makefile (target `ref`, output only into oracle/_ref/).  It configures the
// estimator exactly as Estimator.cpp:49-59 does with config/kitti.yaml (huber kernel, alpha in [0.1, 10],
// 100 segments, truncation 10, 3 GMM components, 100 samples) and, for every residual vector in the input
// file, writes the reference's alpha and fitted GMM parameters (AdaptiveMEstimator.cpp:243-485), plus the
// libstdc++ std::shuffle(mt19937(42)) sample prefix and the k-means seed draws the reference consumes.
//
// An optional third argument selects pko_kernel_type (default "huber", as kitti.yaml); the other kernels
// (AdaptiveMEstimator.cpp:99-156) feed tests/golden/pko_golden_kernels.jsonl.
// Input (binary): int32 ncases; per case: int32 n, then n float64.
// Output: JSON lines, one per case, doubles printed with 17 significant digits (exact round trip).
#define private public   // read the fitted GMM (m_gmm_*) without modifying the reference source
#include "optimization/AdaptiveMEstimator.h"
#undef private

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

static void put_d(FILE* f, double v) {
    if (std::isnan(v)) std::fprintf(f, "NaN");
    else if (std::isinf(v)) std::fprintf(f, v > 0 ? "Infinity" : "-Infinity");
    else std::fprintf(f, "%.17g", v);
}
static void put_vec(FILE* f, const char* name, const std::vector<double>& v) {
    std::fprintf(f, "\"%s\": [", name);
    for (size_t i = 0; i < v.size(); ++i) { if (i) std::fprintf(f, ", "); put_d(f, v[i]); }
    std::fprintf(f, "]");
}

int main(int argc, char** argv) {
    if (argc < 3) { std::fprintf(stderr, "usage: %s input.bin output.jsonl [pko_kernel_type]\n", argv[0]); return 2; }
    const char* kernel = argc > 3 ? argv[3] : "huber";   // AdaptiveMEstimatorConfig::pko_kernel_type
    FILE* in = std::fopen(argv[1], "rb");
    FILE* out = std::fopen(argv[2], "w");
    if (!in || !out) return 3;
    int32_t ncases = 0;
    if (std::fread(&ncases, 4, 1, in) != 1) return 4;
    lidar_slam::optimization::AdaptiveMEstimator est(true, "huber", 0.1, 10.0, 100, 10.0, 3, 100, kernel);
    for (int c = 0; c < ncases; ++c) {
        int32_t n = 0;
        if (std::fread(&n, 4, 1, in) != 1) return 5;
        std::vector<double> r(n);
        if (n > 0 && std::fread(r.data(), 8, n, in) != static_cast<size_t>(n)) return 6;
        est.reset();
        double alpha = est.calculate_scale_factor(r);
        int k = n < 100 ? n : 100;
        std::vector<int> idx(n);
        std::iota(idx.begin(), idx.end(), 0);
        std::mt19937 g(42);
        std::shuffle(idx.begin(), idx.end(), g);
        std::mt19937 gen(42);
        std::vector<double> draws;
        if (k > 0) {
            std::uniform_int_distribution<> dis(0, k - 1);
            draws.push_back(dis(gen));
            draws.push_back(dis(gen));
        }
        std::fprintf(out, "{\"case\": %d, \"n\": %d, \"alpha\": ", c, n);
        put_d(out, alpha);
        std::fprintf(out, ", ");
        put_vec(out, "w", est.m_gmm_weights); std::fprintf(out, ", ");
        put_vec(out, "mu", est.m_gmm_means); std::fprintf(out, ", ");
        put_vec(out, "var", est.m_gmm_variances); std::fprintf(out, ", ");
        put_vec(out, "alphas", est.m_alpha_candidates); std::fprintf(out, ", ");
        put_vec(out, "Z", est.m_partition_functions); std::fprintf(out, ", ");
        std::vector<double> perm(idx.begin(), idx.begin() + k);
        put_vec(out, "perm", perm); std::fprintf(out, ", ");
        put_vec(out, "kmeans_draws", draws);
        std::fprintf(out, "}\n");
    }
    std::fclose(out);
    std::fclose(in);
    return 0;
}
