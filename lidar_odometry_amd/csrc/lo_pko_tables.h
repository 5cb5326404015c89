// lo_pko_tables.h — host-built tables that let the device reproduce the reference's PKO sampling.
//
// The reference fits its GMM on residuals[perm[0..S-1]] where perm = std::shuffle(iota(n), std::mt19937(42))
// (AdaptiveMEstimator.cpp:319-328) and seeds k-means with uniform_int_distribution<>(0, S-1) draws of a
// fresh mt19937(42) (:336-345).  n (the correspondence count) is only known on the device, so the host
// precomputes, once per context, everything needed to answer "perm_n[s]" for any n in O(log) on device:
//
//  libstdc++ (GCC 11, bits/stl_algo.h) shuffles n <= 65535 two positions per draw (__gen_two_uniform_ints),
//  with a lone first swap when n is even; larger n take one uniform(0, i) draw per position.  So for each
//  of the three "modes" (odd n <= 65535, even n <= 65535, n > 65535) the swap partner k_i of position i is
//  a fixed sequence independent of n; n only decides where the sequence stops.  Positions i >= S write
//  value i into slot k_i < S and never read the first S slots, so
//      perm_n[s] = (last i <= n-1 with k_i == s)  or  base_mode[s]  if there is none,
//  where base_mode is the state of the first S slots after positions 1..S-1.  Per (mode, slot) the event
//  list has ~S*ln(n/S)/S entries.  n < S uses explicit full permutations.
#pragma once
#include <cstdint>
#include <vector>

namespace lo {

// std::mt19937 (32-bit Mersenne Twister, seed 42 in all uses here)
struct Mt19937 {
    uint32_t mt[624];
    int idx;
    explicit Mt19937(uint32_t seed);
    uint32_t operator()();
};

// libstdc++ uniform_int_distribution<>::operator() for a 32-bit URBG and range < 2^32 (Lemire, _S_nd)
uint64_t uniform_u32range(Mt19937& g, uint64_t a, uint64_t b);

struct PkoTables {
    int S = 0;                 // gmm_sample_size
    int K = 0;                 // gmm_components
    int max_n = 0;
    std::vector<double> alphas, Z;            // initialize_pko (:218-241), num_alpha_segments+1
    std::vector<int32_t> small_off;           // [S+1]: offsets of the full permutation of n (n < S)
    std::vector<int32_t> small_perm;
    std::vector<int32_t> base;                // [3*S]
    std::vector<int32_t> ev_off;              // [3*(S+1)] into ev_steps
    std::vector<int32_t> ev_steps;
    std::vector<int32_t> km_draws;            // [(S+1)*(K-1)]: k-means seed draws for sample count m
};

void build_pko_tables(PkoTables& t, int S, int K, int max_n, double min_scale, double max_scale, int nseg,
                      double trunc, int kernel);   // kernel: LO_PKO_*
int32_t pko_sample_host(const PkoTables& t, int n, int s);

}  // namespace lo
