// Diagnostic micro-benchmark (not part of the product): the exact candidates' consumer loop (exact_sums_wg, wave 0:
// per 16 staged rows 8 ds_read_b128 of two factor rows, 16 fp32 products and 16 dependent adds) alone in one
// workgroup, in shader cycles (s_memtime) per 16 rows -- the loop's cost without the PKO launch around it.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/consumer_microbench.hip -o scripts/consumer_microbench
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kStride = 212, kRows = 192, kF = 14;

__global__ __launch_bounds__(256) void k_consume(unsigned long long* out, const float* in, float* sink, int chunks) {
    __shared__ float s_f[kF * kStride];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < kF * kStride; i += 256) s_f[i] = in[i % 1024];
    __syncthreads();
    const int k = lane < 43 ? lane : 0;
    const int fa = k < 36 ? k % 6 : 12, fb = k < 36 ? 6 + k / 6 : (k < 42 ? k - 36 : 13);
    float sum = 0.0f;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int ch = 0; ch < chunks; ++ch) {
        if (wid == 0) {
            const float4* A = reinterpret_cast<const float4*>(s_f + fa * kStride);
            const float4* B = reinterpret_cast<const float4*>(s_f + fb * kStride);
            const int ng = kRows / 16;
            float4 a[4], b[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) { a[q] = A[q]; b[q] = B[q]; }
            for (int g = 0; g < ng; ++g) {
                float4 an[4], bn[4];
                const int gn = g + 1 < ng ? g + 1 : g;
#pragma unroll
                for (int q = 0; q < 4; ++q) { an[q] = A[4 * gn + q]; bn[q] = B[4 * gn + q]; }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    sum += a[q].x * b[q].x;
                    sum += a[q].y * b[q].y;
                    sum += a[q].z * b[q].z;
                    sum += a[q].w * b[q].w;
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) { a[q] = an[q]; b[q] = bn[q]; }
            }
        }
        __syncthreads();
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    sink[threadIdx.x] = sum;
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}

int main() {
    unsigned long long* d;
    float *in, *sink;
    (void)hipMalloc(&d, 4096 * 8);
    (void)hipMalloc(&in, 4096);
    (void)hipMalloc(&sink, 4096);
    (void)hipMemset(in, 0, 4096);
    const int chunks = 20;
    for (int grid : {1, 202, 1024}) {
        for (int r = 0; r < 3; ++r) {
            hipLaunchKernelGGL(k_consume, dim3(grid), dim3(256), 0, 0, d, in, sink, chunks);
            (void)hipDeviceSynchronize();
        }
        unsigned long long h[4096];
        (void)hipMemcpy(h, d, grid * 8, hipMemcpyDeviceToHost);
        double m = 0;
        for (int i = 0; i < grid; ++i) m += double(h[i]);
        m /= grid;
        printf("grid %4d: consumer loop %.1f cycles per 16 rows (mean over workgroups)\n", grid, m / (chunks * kRows / 16));
    }
    return 0;
}
