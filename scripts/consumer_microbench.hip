// Diagnostic micro-benchmark (not part of the product): forms of the exact candidates' consumer loop (exact_sums_wg,
// wave 0: per 16 staged rows 8 ds_read_b128 of two factor rows, 16 fp32 products and 16 dependent adds) alone in
// one workgroup, in shader cycles (s_memtime) per 16 rows.  V0: the next group's reads at the top of the loop body
// (the compiler's schedule); V1 / V2: two / three register stages, the reads pinned by sched_barrier one / two groups
// ahead of their adds; V3: the next group's 16 products formed (two per v_pk_mul_f32) while the current group's are
// added; V4: V3 with the adder wave at issue priority 3.  busy = 1: waves 1-3 run a dependent VALU loop meanwhile;
// wgs = 1024: four workgroups per CU.  V5 / V6: V3 / V4 with one packed product placed between every two adds
// (sched_barrier), so the products issue in the adds' latency; V7: V5 with the reads of the group after next placed
// one ds_read_b128 between every add pair too.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off scripts/consumer_microbench.hip -o scripts/consumer_microbench
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kStride = 212, kRows = 192, kF = 14;

struct G4 { float4 a[4], b[4]; };
typedef float f2 __attribute__((ext_vector_type(2)));
struct P16 { f2 p[8]; };
__device__ __forceinline__ void mulg(P16& r, const G4& c) {   // 16 separately rounded fp32 products, two per v_pk_mul_f32
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        r.p[2 * q] = f2{c.a[q].x, c.a[q].y} * f2{c.b[q].x, c.b[q].y};
        r.p[2 * q + 1] = f2{c.a[q].z, c.a[q].w} * f2{c.b[q].z, c.b[q].w};
    }
}
__device__ __forceinline__ f2 mul1(const G4& c, int i) {   // products 2i, 2i+1 of a group
    const float4 a = c.a[i >> 1], b = c.b[i >> 1];
    return (i & 1) ? f2{a.z, a.w} * f2{b.z, b.w} : f2{a.x, a.y} * f2{b.x, b.y};
}
// the current group's 16 adds with the next group's 8 packed products placed one between every two adds
__device__ __forceinline__ void add_mul(float& sum, const P16& p, P16& pn, const G4& c) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        sum += p.p[i].x;
        __builtin_amdgcn_sched_barrier(0);
        pn.p[i] = mul1(c, i);
        __builtin_amdgcn_sched_barrier(0);
        sum += p.p[i].y;
        __builtin_amdgcn_sched_barrier(0);
    }
}
// V7: as add_mul, with the group after next read one ds_read_b128 at a time between the add pairs
__device__ __forceinline__ void add_mul_ld(float& sum, const P16& p, P16& pn, const G4& c, G4& n, const float4* A,
                                           const float4* B, int gl) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        sum += p.p[i].x;
        __builtin_amdgcn_sched_barrier(0);
        pn.p[i] = mul1(c, i);
        __builtin_amdgcn_sched_barrier(0);
        sum += p.p[i].y;
        __builtin_amdgcn_sched_barrier(0);
        if (i < 4) n.a[i] = A[4 * gl + i]; else n.b[i - 4] = B[4 * gl + i - 4];
        __builtin_amdgcn_sched_barrier(0);
    }
}
__device__ __forceinline__ void addp(float& sum, const P16& r) {
#pragma unroll
    for (int q = 0; q < 8; ++q) { sum += r.p[q].x; sum += r.p[q].y; }
}
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
__global__ __launch_bounds__(256) void k_consume(unsigned long long* out, const float* in, float* sink, int chunks, int busy) {
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
            } else if constexpr (V == 7) {
                G4 c;
                P16 p;
                ld(c, A, B, 0);
                mulg(p, c);
                ld(c, A, B, ng > 1 ? 1 : 0);
                for (int g = 0; g < ng; ++g) {
                    G4 n;
                    P16 pn;
                    add_mul_ld(sum, p, pn, c, n, A, B, g + 2 < ng ? g + 2 : g);
                    p = pn;
                    c = n;
                }
            } else if constexpr (V == 5 || V == 6) {
                if (V == 6) __builtin_amdgcn_s_setprio(3);
                G4 c;
                P16 p;
                ld(c, A, B, 0);
                mulg(p, c);
                ld(c, A, B, ng > 1 ? 1 : 0);
                for (int g = 0; g < ng; ++g) {
                    G4 n;
                    ld(n, A, B, g + 2 < ng ? g + 2 : g);
                    P16 pn;
                    add_mul(sum, p, pn, c);
                    p = pn;
                    c = n;
                }
                if (V == 6) __builtin_amdgcn_s_setprio(0);
            } else if constexpr (V == 3 || V == 4) {
                if (V == 4) __builtin_amdgcn_s_setprio(3);
                G4 c;
                P16 p;
                ld(c, A, B, 0);
                mulg(p, c);
                ld(c, A, B, ng > 1 ? 1 : 0);
                for (int g = 0; g < ng; ++g) {
                    G4 n;
                    ld(n, A, B, g + 2 < ng ? g + 2 : g);
                    P16 pn;
                    mulg(pn, c);
                    addp(sum, p);
                    p = pn;
                    c = n;
                }
                if (V == 4) __builtin_amdgcn_s_setprio(0);
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
        } else if (busy) {
            float x = sum + lane, y = x * 0.5f;
            for (int i = 0; i < 64 * kRows / 16; ++i) { x = x * 1.0001f + y; y = y * 0.9999f + x; }
            sum += x + y;
        }
        __syncthreads();
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    sink[threadIdx.x] = sum;
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}

template <int V>
static void run(unsigned long long* d, float* in, float* sink, int busy, int wgs) {
    const int chunks = 20;
    for (int r = 0; r < 3; ++r) {
        hipLaunchKernelGGL(k_consume<V>, dim3(wgs), dim3(256), 0, 0, d, in, sink, chunks, busy);
        (void)hipDeviceSynchronize();
    }
    unsigned long long h;
    (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    printf("V%d busy=%d wgs=%d: %.1f cycles per 16 rows\n", V, busy, wgs, double(h) / (chunks * kRows / 16));
}

int main() {
    unsigned long long* d;
    float *in, *sink;
    (void)hipMalloc(&d, 4096 * 8);
    (void)hipMalloc(&in, 4096);
    (void)hipMalloc(&sink, 4096);
    (void)hipMemset(in, 0, 4096);
    for (int busy = 0; busy < 1; ++busy)
        for (int wgs : {1, 256 * 4}) {
            run<0>(d, in, sink, busy, wgs);
            run<1>(d, in, sink, busy, wgs);
            run<2>(d, in, sink, busy, wgs);
            run<3>(d, in, sink, busy, wgs);
            run<4>(d, in, sink, busy, wgs);
            run<5>(d, in, sink, busy, wgs);
            run<6>(d, in, sink, busy, wgs);
            run<7>(d, in, sink, busy, wgs);
        }
    return 0;
}
