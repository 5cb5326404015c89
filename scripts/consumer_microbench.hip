// Diagnostic micro-benchmark (not part of the product): forms of the exact candidates' consumer loop (exact_sums_wg,
// wave 0: per 16 staged rows 8 ds_read_b128 of two factor rows, 16 fp32 products and 16 dependent adds) alone in
// one workgroup, in shader cycles (s_memtime) per 16 rows.  V0: the next group's reads at the top of the loop body
// (the compiler's schedule); V1 / V2: two / three register stages, the reads pinned by sched_barrier one / two groups
// ahead of their adds.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/consumer_microbench.hip -o scripts/consumer_microbench
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kStride = 212, kRows = 192, kF = 14;

struct G4 { float4 a[4], b[4]; };
__device__ __forceinline__ void ld(G4& r, const float4* A, const float4* B, int g) {
#pragma unroll
    for (int q = 0; q < 4; ++q) { r.a[q] = A[4 * g + q]; r.b[q] = B[4 * g + q]; }
}
__device__ __forceinline__ void add(float& sum, const G4& r) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        sum += r.a[q].x * r.b[q].x;
        sum += r.a[q].y * r.b[q].y;
        sum += r.a[q].z * r.b[q].z;
        sum += r.a[q].w * r.b[q].w;
    }
}

template <int V>
__global__ __launch_bounds__(256) void k_consume(unsigned long long* out, const float* in, float* sink, int chunks) {
    __shared__ __attribute__((aligned(16))) float s_f[kF * kStride];
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
            if constexpr (V == 0) {
                G4 c;
                ld(c, A, B, 0);
                for (int g = 0; g < ng; ++g) {
                    G4 n;
                    ld(n, A, B, g + 1 < ng ? g + 1 : g);
                    add(sum, c);
                    c = n;
                }
            } else if constexpr (V == 1) {
                G4 c0, c1;
                ld(c0, A, B, 0);
                int g = 0;
                for (; g + 2 <= ng; g += 2) {
                    ld(c1, A, B, g + 1);
                    __builtin_amdgcn_sched_barrier(0);
                    add(sum, c0);
                    __builtin_amdgcn_sched_barrier(0);
                    ld(c0, A, B, g + 2 < ng ? g + 2 : g);
                    __builtin_amdgcn_sched_barrier(0);
                    add(sum, c1);
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (g < ng) add(sum, c0);
            } else {
                G4 c0, c1, c2;
                ld(c0, A, B, 0);
                ld(c1, A, B, ng > 1 ? 1 : 0);
                int g = 0;
                for (; g + 3 <= ng; g += 3) {
                    ld(c2, A, B, g + 2);
                    __builtin_amdgcn_sched_barrier(0);
                    add(sum, c0);
                    __builtin_amdgcn_sched_barrier(0);
                    ld(c0, A, B, g + 3 < ng ? g + 3 : g);
                    __builtin_amdgcn_sched_barrier(0);
                    add(sum, c1);
                    __builtin_amdgcn_sched_barrier(0);
                    ld(c1, A, B, g + 4 < ng ? g + 4 : g);
                    __builtin_amdgcn_sched_barrier(0);
                    add(sum, c2);
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (g < ng) add(sum, c0);
                if (g + 1 < ng) add(sum, c1);
            }
        }
        __syncthreads();
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    sink[threadIdx.x] = sum;
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}

template <int V>
static void run(unsigned long long* d, float* in, float* sink) {
    const int chunks = 20;
    for (int r = 0; r < 3; ++r) {
        hipLaunchKernelGGL(k_consume<V>, dim3(1), dim3(256), 0, 0, d, in, sink, chunks);
        (void)hipDeviceSynchronize();
    }
    unsigned long long h;
    (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    printf("V%d: %.1f cycles per 16 rows\n", V, double(h) / (chunks * kRows / 16));
}

int main() {
    unsigned long long* d;
    float *in, *sink;
    (void)hipMalloc(&d, 4096 * 8);
    (void)hipMalloc(&in, 4096);
    (void)hipMalloc(&sink, 4096);
    (void)hipMemset(in, 0, 4096);
    run<0>(d, in, sink);
    run<1>(d, in, sink);
    run<2>(d, in, sink);
    return 0;
}
