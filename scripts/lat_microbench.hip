#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned long long* out, const float* in, float* sink, int reps) {
    float s = in[threadIdx.x], x = in[threadIdx.x + 64], y = s;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < reps; ++i) {
#pragma unroll
        for (int u = 0; u < 64; ++u) asm volatile("v_add_f32 %0, %0, %1" : "+v"(s) : "v"(x));
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < reps; ++i) {
#pragma unroll
        for (int u = 0; u < 32; ++u) { asm volatile("v_add_f32 %0, %0, %1" : "+v"(s) : "v"(x)); asm volatile("v_add_f32 %0, %0, %1" : "+v"(y) : "v"(x)); }
    }
    unsigned long long t2 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < reps; ++i) {
#pragma unroll
        for (int u = 0; u < 64; ++u) asm volatile("s_nop 0");
    }
    unsigned long long t3 = __builtin_amdgcn_s_memtime();
    sink[threadIdx.x] = s + y;
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = t2 - t1; out[2] = t3 - t2; }
}
int main() {
    unsigned long long* d; float *in, *sink;
    hipMalloc(&d, 64); hipMalloc(&in, 1024); hipMalloc(&sink, 1024); hipMemset(in, 0, 1024);
    for (int r = 0; r < 3; ++r) { hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, in, sink, 100); hipDeviceSynchronize(); }
    unsigned long long h[3]; hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
    printf("dependent v_add_f32: %.2f cyc, 2 chains interleaved: %.2f cyc/instr, s_nop: %.2f\n", h[0] / 6400.0, h[1] / 6400.0, h[2] / 6400.0);
    // clock: s_memtime ticks per wall second
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0); hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, in, sink, 200000); hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1); hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
    printf("memtime ticks per us (long run): %.1f\n", (h[0] + h[1] + h[2]) / (ms * 1000.0));
    return 0;
}
