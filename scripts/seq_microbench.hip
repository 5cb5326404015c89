// Diagnostic micro-benchmark (not part of the product): the cost in shader cycles (s_memtime) of the building blocks
// of the exact-mode sum kernels inside ONE workgroup of NT threads -- barriers, DPP block scans of doubles / two-state
// segment maps, the per-term map push, LDS round trips.  Each primitive runs REPS times back to back between two
// stamps of thread 0; the printed figure is cycles per repetition.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I lidar_odometry_amd/csrc scripts/seq_microbench.hip -o scripts/seq_microbench
#include <hip/hip_runtime.h>

#include <cstdio>

#include "lo_seqsum.h"

using namespace lo;

constexpr int REPS = 64;

template <int NT>
__global__ __launch_bounds__(NT) void k_bench(unsigned long long* out, const double* in, double* sink) {
    __shared__ MonoScratch<NT> S;
    __shared__ double s_x[NT * 8];
    const int tid = threadIdx.x;
    double acc = in[tid];
    unsigned long long t[16];
    int k = 0;
    __syncthreads();
    t[k++] = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int r = 0; r < REPS; ++r) __syncthreads();                                        // 1: barrier
    t[k++] = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int r = 0; r < REPS; ++r) {                                                      // 2: block scan of a double
        acc = block_excl_scan_dpp<NT>(acc, 0.0, [](double a, double b) { return a + b; }, S.wd) * 0.5 + 1.0;
    }
    t[k++] = __builtin_amdgcn_s_memtime();
    int g = tid & 15;
#pragma unroll 1
    for (int r = 0; r < REPS; ++r) {                                                      // 3: block scan of the XOR state
        int tot;
        g = block_excl_scan_dpp<NT>(g, 0, [](int a, int b) { return xs_op(a & 15, b & 15) | (((a >> 4) + (b >> 4)) << 4); },
                                    S.wi, &tot) + r;
    }
    t[k++] = __builtin_amdgcn_s_memtime();
    long long mf = 0;
#pragma unroll 1
    for (int r = 0; r < REPS; ++r) {                                                      // 4: one term's integer step
        const TermBits b = term_bits(acc + r + mf, 40);
        mf += b.f + b.up + b.tie;
    }
    t[k++] = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int r = 0; r < REPS; ++r) {                                                      // 5: wave scan of a double
        acc = wave_incl_scan(acc, 0.0, [](double a, double b) { return a + b; }) * 0.5;
    }
    t[k++] = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int r = 0; r < REPS; ++r) {                                                      // 6: LDS write + barrier + read
        s_x[tid] = acc;
        __syncthreads();
        acc = s_x[(tid + 1) % NT] * 0.5 + 1.0;
        __syncthreads();
    }
    t[k++] = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int r = 0; r < REPS; ++r) acc = __shfl_up(acc, 1, 64) * 0.5 + 1.0;               // 7: shfl_up of a double
    t[k++] = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int r = 0; r < REPS; ++r) acc = acc + 1.0000001;                                 // 8: dependent fp64 add
    t[k++] = __builtin_amdgcn_s_memtime();
    float f = static_cast<float>(acc);
    const float fi = 1.0000001f + static_cast<float>(tid & 1);
#pragma unroll
    for (int r = 0; r < REPS; ++r) f = f + fi;                                            // 9: unrolled fp32 chain
    t[k++] = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int r = 0; r < REPS; ++r) acc = acc + static_cast<double>(fi);                  // 10: unrolled fp64 chain
    t[k++] = __builtin_amdgcn_s_memtime();
    const double one = 1.0;
#pragma unroll
    for (int r = 0; r < REPS / 16; ++r) {                                                 // 11: fma-dpp broadcast chain
        bcast_add<0>(acc, acc, one); bcast_add<1>(acc, acc, one); bcast_add<2>(acc, acc, one); bcast_add<3>(acc, acc, one);
        bcast_add<4>(acc, acc, one); bcast_add<5>(acc, acc, one); bcast_add<6>(acc, acc, one); bcast_add<7>(acc, acc, one);
        bcast_add<8>(acc, acc, one); bcast_add<9>(acc, acc, one); bcast_add<10>(acc, acc, one); bcast_add<11>(acc, acc, one);
        bcast_add<12>(acc, acc, one); bcast_add<13>(acc, acc, one); bcast_add<14>(acc, acc, one); bcast_add<15>(acc, acc, one);
    }
    t[k++] = __builtin_amdgcn_s_memtime();
    int iv = static_cast<int>(acc) + tid;
#pragma unroll
    for (int r = 0; r < REPS; ++r) iv = iv * 3 + 1;                                       // 12: unrolled int32 chain
    t[k++] = __builtin_amdgcn_s_memtime();
    acc += f + iv;
    sink[tid] = acc + g + static_cast<double>(mf);
    if (tid == 0)
        for (int i = 0; i < k; ++i) out[i] = t[i];
}

template <int NT>
static void run(const char* tag) {
    unsigned long long* d_out;
    double *d_in, *d_sink;
    (void)hipMalloc(&d_out, 16 * sizeof(unsigned long long));
    (void)hipMalloc(&d_in, NT * sizeof(double));
    (void)hipMalloc(&d_sink, NT * sizeof(double));
    (void)hipMemset(d_in, 0, NT * sizeof(double));
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_bench<NT>, dim3(1), dim3(NT), 0, nullptr, d_out, d_in, d_sink);
        (void)hipDeviceSynchronize();
    }
    unsigned long long h[16];
    (void)hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost);
    const char* names[] = {"barrier", "block scan f64", "block scan xor state", "term step", "wave scan f64",
                           "LDS write+barrier+read x2", "shfl_up f64", "dependent f64 add (rolled loop)",
                           "fp32 add chain", "fp64 add chain", "fma-dpp bcast chain", "int32 mad chain"};
    printf("%s:\n", tag);
    for (int i = 0; i < 12; ++i) printf("    %-30s %8.1f\n", names[i], double(h[i + 1] - h[i]) / REPS);
    printf("\n");
    (void)hipFree(d_out);
    (void)hipFree(d_in);
    (void)hipFree(d_sink);
}

int main() {
    run<64>("NT=64");
    run<256>("NT=256");
    run<512>("NT=512");
    run<1024>("NT=1024");
    return 0;
}
