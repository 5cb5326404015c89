// Accuracy of lo::log_pos (lo_math.h) against glibc log: ulp histogram over log-uniform samples in
// [1e-300, 1e300], uniform samples near 1 and the JS-term range (0, 2], plus the special values.
// g++ -O2 -ffp-contract=off -std=c++17 scripts/check_log_pos.cpp -o /tmp/check_log_pos && /tmp/check_log_pos [n]
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include "../lidar_odometry_amd/csrc/lo_math.h"

static int64_t ord(double x) { int64_t i; std::memcpy(&i, &x, 8); return i < 0 ? INT64_MIN - i : i; }

int main(int argc, char** argv) {
    const long n = argc > 1 ? std::atol(argv[1]) : 20000000;
    std::mt19937_64 g(12345);
    std::uniform_real_distribution<double> le(-690.0, 690.0), u1(0.5, 1.5), u2(0.0, 2.0);
    long hist[4] = {0, 0, 0, 0};
    int64_t worst = 0;
    double wx = 0;
    for (long i = 0; i < n; ++i) {
        const int c = i % 3;
        const double x = c == 0 ? std::exp(le(g)) : (c == 1 ? u1(g) : u2(g));
        if (!(x > 0)) continue;
        const int64_t d = std::llabs(ord(lo::log_pos(x)) - ord(std::log(x)));
        ++hist[d > 3 ? 3 : d];
        if (d > worst) { worst = d; wx = x; }
    }
    const double sp[] = {0.0, INFINITY, -1.0, NAN, 1.0, 4.9e-324, 2.2250738585072014e-308, 1.7976931348623157e308};
    int bad = 0;
    for (double x : sp) {
        const double a = lo::log_pos(x), b = std::log(x);
        const bool same = (std::isnan(a) && std::isnan(b)) || a == b || std::llabs(ord(a) - ord(b)) <= 1;
        if (!same) { ++bad; std::printf("special %g: %.17g vs %.17g\n", x, a, b); }
    }
    std::printf("n=%ld ulp0=%ld ulp1=%ld ulp2=%ld ulp>=3=%ld worst=%lld at %.17g specials_bad=%d\n", n, hist[0], hist[1],
                hist[2], hist[3], static_cast<long long>(worst), wx, bad);
    return (worst <= 1 && bad == 0) ? 0 : 1;
}
