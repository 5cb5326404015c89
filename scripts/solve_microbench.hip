// Latency of the reference-exact GN solve (lo_exact.h exact_solve_step) on one lane, and of its parts (diagnostic;
// not part of the product).  hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I lidar_odometry_amd/csrc
//   -o scripts/solve_microbench scripts/solve_microbench.hip && scripts/solve_microbench
// One wave, lane 0 active (as in a candidate workgroup): s_memtime cycles per call, inputs chained through the outputs.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "lo_exact.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

using namespace lo;

template <int V>
__global__ void k_bench(const float* in, float* out, unsigned long long* cyc, int reps) {
    if (threadIdx.x != 0) return;
    float tot[kExactTerms], pose[12];
    for (int k = 0; k < kExactTerms; ++k) tot[k] = in[k];
    for (int k = 0; k < 12; ++k) pose[k] = in[64 + k];
    float acc = 0.0f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        float pn[12], delta[6];
        if constexpr (V == 0) {
            const bool c = exact_solve_step(tot, pose, 1e-4, 1e-4, pn, delta);
            acc += pn[0] + pn[5] + pn[11] + (c ? 1.0f : 0.0f);
        } else if constexpr (V == 1) {
            float H[36], g[6];
            for (int k = 0; k < 36; ++k) H[k] = tot[k];
            for (int j = 0; j < 6; ++j) g[j] = -tot[36 + j];
            ldlt6_solve_f32(H, g, delta);
            acc += delta[0] + delta[5];
        } else if constexpr (V == 2) {
            const float w[3] = {tot[36] * 1e-3f, tot[37] * 1e-3f, tot[38] * 1e-3f};
            float Rd[3][3];
            so3_exp_exact(w, Rd);
            acc += Rd[0][0] + Rd[2][1];
        } else if constexpr (V == 3) {
            float M[3][3], R[3][3];
            for (int a = 0; a < 3; ++a) for (int b = 0; b < 3; ++b) M[a][b] = pose[a * 4 + b] * (1.0f + 1e-7f * tot[a * 3 + b]);
            so3_project_svd(M, R);
            acc += R[0][0] + R[1][2];
        } else {
            float x = tot[0] + 3.0f;                     // 64 dependent divisions, then 64 dependent square roots
            for (int k = 0; k < 64; ++k) x = tot[k & 31] / x + 1.0f;
            for (int k = 0; k < 64; ++k) x = sqrtf(x + tot[k & 31]);
            acc += x;
        }
        tot[r % kExactTerms] += acc * 1e-30f;            // chain the next call on this one
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    cyc[0] = t1 - t0;
    out[0] = acc;
}

int main() {
    float h_in[128] = {};
    std::srand(3);
    // a typical candidate: H = sum of J^T J (SPD), g, cost; the pose a 0.3 rad yaw
    float J[6];
    for (int i = 0; i < 400; ++i) {
        for (int k = 0; k < 6; ++k) J[k] = (std::rand() % 2001 - 1000) * 1e-3f * (k < 3 ? 1.0f : 10.0f);
        for (int r = 0; r < 6; ++r) for (int c = 0; c < 6; ++c) h_in[r * 6 + c] += J[c] * J[r];
        const float res = (std::rand() % 2001 - 1000) * 1e-5f;
        for (int k = 0; k < 6; ++k) h_in[36 + k] += res * J[k];
        h_in[42] += res * res;
    }
    const float c = 0.9553365f, s = 0.2955202f;
    const float P[12] = {c, -s, 0, 10.0f, s, c, 0, -3.0f, 0, 0, 1, 0.5f};
    for (int k = 0; k < 12; ++k) h_in[64 + k] = P[k];
    float *d_in, *d_out;
    unsigned long long* d_c;
    CK(hipMalloc(&d_in, sizeof(h_in)));
    CK(hipMalloc(&d_out, 64));
    CK(hipMalloc(&d_c, 64));
    CK(hipMemcpy(d_in, h_in, sizeof(h_in), hipMemcpyHostToDevice));
    const char* names[] = {"exact_solve_step (full)", "ldlt6_solve_f32", "so3_exp_exact (incl. SVD)", "so3_project_svd",
                           "64 div + 64 sqrt chain"};
    const int reps = 64;
    for (int v = 0; v < 5; ++v) {
        for (int w = 0; w < 2; ++w) {                    // the second run from a warm instruction cache
            switch (v) {
                case 0: hipLaunchKernelGGL(k_bench<0>, dim3(1), dim3(64), 0, 0, d_in, d_out, d_c, reps); break;
                case 1: hipLaunchKernelGGL(k_bench<1>, dim3(1), dim3(64), 0, 0, d_in, d_out, d_c, reps); break;
                case 2: hipLaunchKernelGGL(k_bench<2>, dim3(1), dim3(64), 0, 0, d_in, d_out, d_c, reps); break;
                case 3: hipLaunchKernelGGL(k_bench<3>, dim3(1), dim3(64), 0, 0, d_in, d_out, d_c, reps); break;
                default: hipLaunchKernelGGL(k_bench<4>, dim3(1), dim3(64), 0, 0, d_in, d_out, d_c, reps); break;
            }
            CK(hipDeviceSynchronize());
        }
        unsigned long long cyc = 0;
        CK(hipMemcpy(&cyc, d_c, 8, hipMemcpyDeviceToHost));
        if (v < 4) std::printf("%-28s %8.0f cycles per call\n", names[v], static_cast<double>(cyc) / reps);
        else std::printf("%-28s %8.1f cycles per dependent op\n", names[v], static_cast<double>(cyc) / reps / 128.0);
    }
    // one call per launch: the instruction cache as a candidate workgroup meets the solve (once per PKO launch)
    for (int w = 0; w < 4; ++w) {
        hipLaunchKernelGGL(k_bench<0>, dim3(1), dim3(64), 0, 0, d_in, d_out, d_c, 1);
        CK(hipDeviceSynchronize());
        unsigned long long cyc = 0;
        CK(hipMemcpy(&cyc, d_c, 8, hipMemcpyDeviceToHost));
        std::printf("exact_solve_step, one call per launch (launch %d): %llu cycles\n", w, cyc);
    }
    return 0;
}
