// Dependent fp32 add chains on gfx950 (diagnostic; not part of the product): cycles per dependent v_add_f32 with 0, 1
// and 2 independent v_mul_f32 between the adds, one wave alone on a CU.  Bounds the exact candidates' running sums.
//   hipcc --offload-arch=gfx950 -O3 -o scripts/chain_microbench scripts/chain_microbench.hip && scripts/chain_microbench
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int V>
__global__ void k_chain(const float* in, float* out, unsigned long long* cyc) {
    const int lane = threadIdx.x;
    float s = in[lane], a = in[lane + 64], b = in[lane + 128], c = in[lane + 192];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 64
    for (int i = 0; i < 1024; ++i) {
        if constexpr (V == 0) {
            asm volatile("v_add_f32 %0, %0, %1" : "+v"(s) : "v"(a));
        } else if constexpr (V == 1) {
            float p;
            asm volatile("v_mul_f32 %0, %1, %2\n\tv_add_f32 %3, %3, %0" : "=&v"(p), "+v"(a), "+v"(b), "+v"(s));
        } else {
            float p, q;
            asm volatile("v_mul_f32 %0, %2, %3\n\tv_mul_f32 %1, %3, %4\n\tv_add_f32 %5, %5, %0\n\tv_add_f32 %5, %5, %1"
                         : "=&v"(p), "=&v"(q), "+v"(a), "+v"(b), "+v"(c), "+v"(s));
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[lane] = s;
    if (lane == 0) cyc[0] = t1 - t0;
}

int main() {
    float* d;
    unsigned long long* c;
    CK(hipMalloc(&d, 4096));
    CK(hipMalloc(&c, 64));
    CK(hipMemset(d, 0, 4096));
    const char* names[] = {"add chain", "mul + dependent add", "2 x (mul + dependent add)"};
    const double adds[] = {1024, 1024, 2048};
    for (int v = 0; v < 3; ++v) {
        for (int w = 0; w < 2; ++w) {
            if (v == 0) hipLaunchKernelGGL(k_chain<0>, dim3(1), dim3(64), 0, 0, d, d + 512, c);
            else if (v == 1) hipLaunchKernelGGL(k_chain<1>, dim3(1), dim3(64), 0, 0, d, d + 512, c);
            else hipLaunchKernelGGL(k_chain<2>, dim3(1), dim3(64), 0, 0, d, d + 512, c);
            CK(hipDeviceSynchronize());
        }
        unsigned long long h = 0;
        CK(hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost));
        std::printf("%-28s %6.2f cycles per dependent add\n", names[v], static_cast<double>(h) / adds[v]);
    }
    return 0;
}
