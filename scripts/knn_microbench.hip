// Back-to-back timing of the all-pairs kNN / inlier kernels (lo_kdtree.hip) on a synthetic loop-closure-sized case
// (diagnostic; not part of the product): ~3.7k queries against ~3.8k points, and the same launches with no queries
// (staging only) and with a 64-point set (compute-light), to split a launch into staging, search and overhead.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -Ilidar_odometry_amd/csrc \
//         -o scripts/knn_microbench scripts/knn_microbench.hip && scripts/knn_microbench
#include "../lidar_odometry_amd/csrc/lo_kdtree.hip"

#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

using namespace lo;

template <typename F>
static float time_launches(F launch, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 5; ++i) launch();
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i) launch();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms * 1e3f / reps;
}

int main() {
    const int n = 3700, m = 3800;
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> U(-40.0f, 40.0f), Z(-2.0f, 3.0f), J(-0.3f, 0.3f);
    std::vector<float> q(3 * n);
    std::vector<float4> mp(m);
    for (int i = 0; i < m; ++i) {
        const float x = U(rng), y = U(rng), z = Z(rng);
        int id = i;
        float w;
        std::memcpy(&w, &id, 4);
        mp[i] = make_float4(x, y, z, w);
    }
    for (int i = 0; i < n; ++i) {                         // queries near map points
        const float4 v = mp[i % m];
        q[3 * i] = v.x + J(rng); q[3 * i + 1] = v.y + J(rng); q[3 * i + 2] = v.z + J(rng);
    }
    float *d_q;
    float4* d_m;
    DevState* d_st;
    int32_t* d_nbr;
    CK(hipMalloc(&d_q, q.size() * 4));
    CK(hipMalloc(&d_m, m * sizeof(float4)));
    CK(hipMalloc(&d_st, sizeof(DevState)));
    CK(hipMalloc(&d_nbr, 5 * sizeof(int32_t) * (n + 256)));
    CK(hipMemcpy(d_q, q.data(), q.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_m, mp.data(), m * sizeof(float4), hipMemcpyHostToDevice));
    CK(hipMemset(d_st, 0, sizeof(DevState)));
    const float I[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    CK(hipMemcpy(d_st, I, sizeof(I), hipMemcpyHostToDevice));
    for (const void* f : {reinterpret_cast<const void*>(&k_knn_all), reinterpret_cast<const void*>(&k_inlier_all)})
        CK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kKnnAllMax * sizeof(float4)));
    KParams P{};
    P.pts = d_q;
    P.n = n;
    P.nb = (n + kBlock - 1) / kBlock;
    P.kd_pts = d_m;
    P.kd_m = m;
    P.kd_all = 1;
    P.kd_nbr = d_nbr;
    P.st = d_st;
    std::memcpy(P.T0, I, sizeof(I));
    auto run = [&](const char* what, KParams Q) {
        const dim3 g((std::max(Q.n, 1) + kAllThreads / 64 - 1) / (kAllThreads / 64)), b(kAllThreads);
        const size_t lds = static_cast<size_t>((std::max(Q.kd_m, 1) + 511) / 512 * 512) * sizeof(float4);
        const float t_knn = time_launches([&] { hipLaunchKernelGGL(k_knn_all, g, b, lds, 0, Q); }, 200);
        const float t_in = time_launches([&] { hipLaunchKernelGGL(k_inlier_all, g, b, lds, 0, Q); }, 200);
        std::printf("%-34s n %5d m %5d blocks %4u  k_knn_all %7.2f us  k_inlier_all %7.2f us\n", what, Q.n, Q.kd_m, g.x,
                    t_knn, t_in);
    };
    run("full", P);
    KParams Pi = P;
    Pi.init = 1;                                          // the scan's first search: no seed
    run("first search (no seed)", Pi);
    KParams P0 = P;
    P0.n = 0;
    run("no queries (staging only)", P0);
    KParams Ps = P;
    Ps.kd_m = 64;
    run("64-point set", Ps);
    KParams Ph = P;
    Ph.n = n / 4;
    run("quarter of the queries", Ph);
    CK(hipDeviceSynchronize());
    std::vector<int32_t> nb(5 * n);
    CK(hipMemcpy(nb.data(), d_nbr, nb.size() * 4, hipMemcpyDeviceToHost));
    int ok = 0;
    for (int i = 0; i < n; ++i) ok += nb[5 * i] >= 0;
    std::printf("queries with five neighbours: %d / %d\n", ok, n);
    return 0;
}
