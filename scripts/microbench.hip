// Floors for the 1M-point correspondence kernel on MI355X (diagnostic; not part of the product).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/microbench scripts/microbench.hip && /tmp/microbench
// Reports HIP-event means over back-to-back launches of:
//   empty     grid of 3907 x 256 threads that only exits (launch + drain floor)
//   stream    read 12 B AoS float3 per point, write 4 B per point (the compulsory HBM traffic, 16 MB)
//   gather    stream + one random 8-B key load from a 1 MB table per point (L2-resident probe)
//   gather32  stream + one random 32-B slot load per point
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

struct __attribute__((aligned(32))) Slot { uint64_t key; float n[3]; float c[3]; };

__global__ void k_empty(int n) { if (n < 0) __builtin_trap(); }

__global__ void k_stream(const float* __restrict__ p, int* __restrict__ out, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float x = p[3 * i], y = p[3 * i + 1], z = p[3 * i + 2];
    out[i] = static_cast<int>(x + y + z);
}

__global__ void k_gather(const float* __restrict__ p, const Slot* __restrict__ tab, uint32_t mask, int* __restrict__ out, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float x = p[3 * i], y = p[3 * i + 1], z = p[3 * i + 2];
    const uint32_t h = (static_cast<uint32_t>(__float_as_uint(x) * 2654435761u) ^ __float_as_uint(y) ^ __float_as_uint(z)) & mask;
    const uint64_t k = tab[h].key;
    out[i] = static_cast<int>(k) + static_cast<int>(x);
}

__global__ void k_gather32(const float* __restrict__ p, const Slot* __restrict__ tab, uint32_t mask, int* __restrict__ out, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float x = p[3 * i], y = p[3 * i + 1], z = p[3 * i + 2];
    const uint32_t h = (static_cast<uint32_t>(__float_as_uint(x) * 2654435761u) ^ __float_as_uint(y) ^ __float_as_uint(z)) & mask;
    const Slot s = tab[h];
    out[i] = static_cast<int>(s.key) + static_cast<int>(s.n[0] + s.c[2] + x);
}

// gather + dependent 32-B slot re-load (k_correspond's probe-then-payload pattern)
__global__ void k_gather_dep(const float* __restrict__ p, const Slot* __restrict__ tab, uint32_t mask, int* __restrict__ out, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float x = p[3 * i], y = p[3 * i + 1], z = p[3 * i + 2];
    const uint32_t h = (static_cast<uint32_t>(__float_as_uint(x) * 2654435761u) ^ __float_as_uint(y) ^ __float_as_uint(z)) & mask;
    const uint64_t k = tab[h].key;
    const Slot s = tab[(h + static_cast<uint32_t>(k & 1)) & mask];
    out[i] = static_cast<int>(s.key) + static_cast<int>(s.n[0] + s.c[2] + x);
}

// + correctly rounded fp32 divisions and floor as PointToVoxelKey
__global__ void k_gather_div(const float* __restrict__ p, const Slot* __restrict__ tab, uint32_t mask, int* __restrict__ out, int n, float sc) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float x = p[3 * i], y = p[3 * i + 1], z = p[3 * i + 2];
    const int kx = static_cast<int>(floorf(x / sc)), ky = static_cast<int>(floorf(y / sc)), kz = static_cast<int>(floorf(z / sc));
    const uint32_t h = (static_cast<uint32_t>(kx * 2654435761u) ^ static_cast<uint32_t>(ky * 40503u) ^ static_cast<uint32_t>(kz)) & mask;
    const uint64_t k = tab[h].key;
    const Slot s = tab[(h + static_cast<uint32_t>(k & 1)) & mask];
    out[i] = static_cast<int>(s.key) + static_cast<int>(s.n[0] + s.c[2] + x);
}

// + ballot / LDS / barrier epilogue (per-wave mask, per-block count)
__global__ __launch_bounds__(256) void k_gather_epi(const float* __restrict__ p, const Slot* __restrict__ tab, uint32_t mask, int* __restrict__ out,
                                                    uint64_t* __restrict__ wm, int* __restrict__ bc, int n, float sc) {
    __shared__ int s_cnt[4];
    const int i = blockIdx.x * 256 + threadIdx.x;
    int v = -1;
    if (i < n) {
        const float x = p[3 * i], y = p[3 * i + 1], z = p[3 * i + 2];
        const int kx = static_cast<int>(floorf(x / sc)), ky = static_cast<int>(floorf(y / sc)), kz = static_cast<int>(floorf(z / sc));
        const uint32_t h = (static_cast<uint32_t>(kx * 2654435761u) ^ static_cast<uint32_t>(ky * 40503u) ^ static_cast<uint32_t>(kz)) & mask;
        const uint64_t k = tab[h].key;
        const Slot s = tab[(h + static_cast<uint32_t>(k & 1)) & mask];
        v = (s.n[0] + s.c[2] + x > 0.5f) ? static_cast<int>(h) : -1;
        out[i] = v;
    }
    const uint64_t m = __ballot(v >= 0);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) { wm[blockIdx.x * 4 + wid] = m; s_cnt[wid] = __popcll(m); }
    __syncthreads();
    if (threadIdx.x == 0) bc[blockIdx.x] = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
}

int main() {
    const int n = 1000000, nb = (n + 255) / 256, reps = 200;
    const uint32_t cap = 1u << 15;
    std::vector<float> hp(3 * static_cast<size_t>(n));
    for (size_t i = 0; i < hp.size(); ++i) hp[i] = static_cast<float>((i * 2654435761ull) % 100000) * 0.001f;
    std::vector<Slot> ht(cap);
    for (uint32_t i = 0; i < cap; ++i) { ht[i].key = i; for (int a = 0; a < 3; ++a) { ht[i].n[a] = 1.0f; ht[i].c[a] = 0.0f; } }
    float* dp; Slot* dt; int* dout; uint64_t* dwm; int* dbc;
    CK(hipMalloc(&dp, hp.size() * 4)); CK(hipMalloc(&dt, cap * sizeof(Slot))); CK(hipMalloc(&dout, n * 4));
    CK(hipMalloc(&dwm, nb * 4 * 8)); CK(hipMalloc(&dbc, nb * 4));
    CK(hipMemcpy(dp, hp.data(), hp.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dt, ht.data(), cap * sizeof(Slot), hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto run = [&](const char* name, auto launch, double bytes) {
        for (int r = 0; r < 20; ++r) launch();
        hipEventRecord(a);
        for (int r = 0; r < reps; ++r) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0; hipEventElapsedTime(&ms, a, b);
        const double us = ms * 1e3 / reps;
        std::printf("%-9s %8.2f us  %8.1f GB/s (%.1f MB/launch)\n", name, us, bytes / (us * 1e-6) / 1e9, bytes / 1e6);
    };
    run("empty", [&] { hipLaunchKernelGGL(k_empty, dim3(nb), dim3(256), 0, 0, n); }, 0.0);
    run("stream", [&] { hipLaunchKernelGGL(k_stream, dim3(nb), dim3(256), 0, 0, dp, dout, n); }, 16.0 * n);
    run("gather", [&] { hipLaunchKernelGGL(k_gather, dim3(nb), dim3(256), 0, 0, dp, dt, cap - 1, dout, n); }, 24.0 * n);
    run("gather32", [&] { hipLaunchKernelGGL(k_gather32, dim3(nb), dim3(256), 0, 0, dp, dt, cap - 1, dout, n); }, 48.0 * n);
    run("gdep", [&] { hipLaunchKernelGGL(k_gather_dep, dim3(nb), dim3(256), 0, 0, dp, dt, cap - 1, dout, n); }, 24.0 * n);
    run("gdiv", [&] { hipLaunchKernelGGL(k_gather_div, dim3(nb), dim3(256), 0, 0, dp, dt, cap - 1, dout, n, 1.5f); }, 24.0 * n);
    run("gepi", [&] { hipLaunchKernelGGL(k_gather_epi, dim3(nb), dim3(256), 0, 0, dp, dt, cap - 1, dout, dwm, dbc, n, 1.5f); }, 24.0 * n);
    return 0;
}
