// lo_pko_tables.cpp — see lo_pko_tables.h.
#include "lo_pko_tables.h"

#include <algorithm>
#include <cmath>

namespace lo {

Mt19937::Mt19937(uint32_t seed) {
    mt[0] = seed;
    for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + static_cast<uint32_t>(i);
    idx = 624;
}

uint32_t Mt19937::operator()() {
    if (idx >= 624) {
        for (int k = 0; k < 624; ++k) {
            uint32_t y = (mt[k] & 0x80000000u) | (mt[(k + 1) % 624] & 0x7fffffffu);
            mt[k] = mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        idx = 0;
    }
    uint32_t z = mt[idx++];
    z ^= (z >> 11);
    z ^= (z << 7) & 0x9d2c5680u;
    z ^= (z << 15) & 0xefc60000u;
    z ^= (z >> 18);
    return z;
}

// uniform_int_distribution::operator() downscaling branch with a 32-bit generator (uniform_int_dist.h, GCC 11):
// range r = b - a + 1 (< 2^32); Lemire's nearly-divisionless method with 64-bit products.
uint64_t uniform_u32range(Mt19937& g, uint64_t a, uint64_t b) {
    const uint64_t urange = b - a;
    if (urange == 0xffffffffull) return static_cast<uint64_t>(g()) + a;
    const uint32_t r = static_cast<uint32_t>(urange + 1);
    uint64_t prod = static_cast<uint64_t>(g()) * r;
    uint32_t low = static_cast<uint32_t>(prod);
    if (low < r) {
        const uint32_t thr = static_cast<uint32_t>(-r) % r;
        while (low < thr) {
            prod = static_cast<uint64_t>(g()) * r;
            low = static_cast<uint32_t>(prod);
        }
    }
    return (prod >> 32) + a;
}

// Swap-partner sequence k_i (i = 1..last) of std::shuffle for the given mode.
// mode 0: n odd, n <= 65535 (pairs (1,2),(3,4),...); mode 1: n even, n <= 65535 (lone 1, then (2,3),...);
// mode 2: n > 65535 (one uniform(0,i) per position).
static void partner_sequence(int mode, int last, std::vector<int32_t>& k) {
    k.assign(static_cast<size_t>(std::max(last, 0)) + 1, 0);
    Mt19937 g(42);
    if (last < 1) return;
    if (mode == 2) {
        for (int i = 1; i <= last; ++i) k[i] = static_cast<int32_t>(uniform_u32range(g, 0, static_cast<uint64_t>(i)));
        return;
    }
    int i = 1;
    if (mode == 1) { k[1] = static_cast<int32_t>(uniform_u32range(g, 0, 1)); i = 2; }
    while (i <= last) {
        const uint64_t b0 = static_cast<uint64_t>(i) + 1, b1 = b0 + 1;
        const uint64_t x = uniform_u32range(g, 0, b0 * b1 - 1);
        k[i] = static_cast<int32_t>(x / b1);
        if (i + 1 <= last) k[i + 1] = static_cast<int32_t>(x % b1);
        i += 2;
    }
}

static void full_perm(int n, std::vector<int32_t>& out) {
    out.resize(n);
    for (int i = 0; i < n; ++i) out[i] = i;
    if (n <= 1) return;
    const int mode = (n <= 65535) ? ((n % 2) ? 0 : 1) : 2;
    std::vector<int32_t> k;
    partner_sequence(mode, n - 1, k);
    for (int i = 1; i <= n - 1; ++i) std::swap(out[i], out[k[i]]);
}

void build_pko_tables(PkoTables& t, int S, int K, int max_n, double min_scale, double max_scale, int nseg,
                      double trunc, int kernel_type) {
    t.S = S; t.K = K; t.max_n = max_n;
    // ---- alpha grid + partition functions (AdaptiveMEstimator.cpp:218-241, :692-708) with pko_kernel_weight
    //      (:99-156, glibc exp / pow as the reference) ----
    auto kernel = [&](double r, double d) -> double {
        switch (kernel_type) {
            case 0: { double a = std::fabs(r); return a <= d ? 1.0 : d / a; }                 // huber
            case 2: {                                                                          // tukey
                double a = std::fabs(r);
                if (a < d) { double x = a / d, x2 = x * x; return (1 - x2) * (1 - x2); }
                return 0.0;
            }
            case 3: { double e2 = r * r, d2 = d * d; return std::exp(-e2 / d2 / 2.0); }      // welsch
            case 4: { double e2 = r * r, d2 = d * d; return r * d2 / (d2 + e2) / (d2 + e2); } // gemanMcClure
            case 5: { double d2 = d * d; return d2 / std::pow(d2 + r * r, 1.5); }             // pseudoHuber
            default: { double e2 = r * r, d2 = d * d; return d2 / (d2 + e2); }                // cauchy
        }
    };
    auto partition = [&](double alpha) {
        double integral = 0.0;
        for (double x = 0.0; x <= trunc; x += 0.01) integral += kernel(x, alpha) * 0.01;
        return std::max(integral, 1e-10);
    };
    t.alphas.assign(nseg + 1, 0.0);
    t.Z.assign(nseg + 1, 0.0);
    t.alphas[0] = min_scale;
    t.Z[0] = partition(min_scale);
    for (int i = 1; i <= nseg; ++i) {
        double tt = static_cast<double>(i) / static_cast<double>(nseg);
        double ls = (std::pow(100.0, tt) - 1.0) / 99.0;
        double a = min_scale + (max_scale - min_scale) * ls;
        t.alphas[i] = a;
        t.Z[i] = partition(a);
    }
    // ---- small n: explicit permutations ----
    t.small_off.assign(S + 1, 0);
    t.small_perm.clear();
    std::vector<int32_t> p;
    for (int n = 1; n < S; ++n) {
        t.small_off[n] = static_cast<int32_t>(t.small_perm.size());
        full_perm(n, p);
        t.small_perm.insert(t.small_perm.end(), p.begin(), p.end());
    }
    t.small_off[S] = static_cast<int32_t>(t.small_perm.size());
    // ---- n >= S: base + event lists per mode ----
    t.base.assign(3 * S, 0);
    t.ev_off.assign(3 * (S + 1), 0);
    t.ev_steps.clear();
    for (int mode = 0; mode < 3; ++mode) {
        int last;
        if (mode < 2) last = std::min(65534, max_n - 1);
        else last = max_n - 1;
        if (mode == 2 && max_n <= 65535) last = std::max(S - 1, 0);
        last = std::max(last, S - 1);
        std::vector<int32_t> k;
        partner_sequence(mode, last, k);
        std::vector<int32_t> slots(S);
        for (int s = 0; s < S; ++s) slots[s] = s;
        for (int i = 1; i <= std::min(S - 1, last); ++i) std::swap(slots[i], slots[k[i]]);
        for (int s = 0; s < S; ++s) t.base[mode * S + s] = slots[s];
        std::vector<std::vector<int32_t>> ev(S);
        for (int i = S; i <= last; ++i) if (k[i] < S) ev[k[i]].push_back(i);
        for (int s = 0; s < S; ++s) {
            t.ev_off[mode * (S + 1) + s] = static_cast<int32_t>(t.ev_steps.size());
            t.ev_steps.insert(t.ev_steps.end(), ev[s].begin(), ev[s].end());
        }
        t.ev_off[mode * (S + 1) + S] = static_cast<int32_t>(t.ev_steps.size());
    }
    // ---- k-means seed draws for sample count m = 1..S (fresh mt19937(42) each) ----
    const int D = std::max(K - 1, 1);
    t.km_draws.assign(static_cast<size_t>(S + 1) * D, 0);
    for (int m = 1; m <= S; ++m) {
        Mt19937 g(42);
        for (int j = 0; j < K - 1; ++j) t.km_draws[m * D + j] = static_cast<int32_t>(uniform_u32range(g, 0, m - 1));
    }
}

int32_t pko_sample_host(const PkoTables& t, int n, int s) {
    if (n < t.S) return t.small_perm[t.small_off[n] + s];
    const int mode = (n <= 65535) ? ((n % 2) ? 0 : 1) : 2;
    const int32_t* b = t.ev_steps.data() + t.ev_off[mode * (t.S + 1) + s];
    const int32_t* e = t.ev_steps.data() + t.ev_off[mode * (t.S + 1) + s + 1];
    const int32_t* it = std::upper_bound(b, e, n - 1);
    if (it == b) return t.base[mode * t.S + s];
    return *(it - 1);
}

}  // namespace lo
