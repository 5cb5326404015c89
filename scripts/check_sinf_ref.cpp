// lo::sincosf_ref (lo_math.h, the device's SO3::Exp sin / cos) against the host's glibc sinf / cosf, bit for bit:
// every float in (1e-7, 120) and its negative (or every k-th with a stride argument), plus tiny / special values.
// g++ -O2 -ffp-contract=off -std=c++17 scripts/check_sinf_ref.cpp -o /tmp/check_sinf_ref && /tmp/check_sinf_ref [stride]
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "../lidar_odometry_amd/csrc/lo_math.h"

static uint32_t bits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

int main(int argc, char** argv) {
    const uint32_t stride = argc > 1 ? static_cast<uint32_t>(std::atol(argv[1])) : 1u;
    long n = 0, bad_s = 0, bad_c = 0;
    for (int sgn = 0; sgn < 2; ++sgn)
        for (uint32_t u = 0x33d6bf95u; u < 0x42f00000u; u += stride) {      // 1e-7 .. 120
            float y;
            const uint32_t v = u | (sgn ? 0x80000000u : 0u);
            std::memcpy(&y, &v, 4);
            volatile float a = std::sin(y), b = std::cos(y);
            bad_s += bits(a) != bits(lo::sincosf_ref(y, 0));
            bad_c += bits(b) != bits(lo::sincosf_ref(y, 1));
            ++n;
        }
    const float sp[] = {0.0f, -0.0f, 1e-30f, -1e-30f, 1e-10f, 1.4e-45f, 0x1p-12f, 0x1.921FB6p-1f, 119.99f};
    for (float y : sp) {
        volatile float a = std::sin(y), b = std::cos(y);
        bad_s += bits(a) != bits(lo::sincosf_ref(y, 0));
        bad_c += bits(b) != bits(lo::sincosf_ref(y, 1));
        ++n;
    }
    std::printf("args=%ld sinf_mismatch=%ld cosf_mismatch=%ld\n", n, bad_s, bad_c);
    return (bad_s || bad_c) ? 1 : 0;
}
