// ksort.hip -- key order for K1.  A batch of one-way Chord lookups arrives in
// the caller's order; K1 runs faster when the lanes of a wave walk neighbouring keys, because their
// last hops then land on the same few ring nodes and share L2 lines (a batch presorted
// by the caller, 85 -> 67 B per hop).  This is a counting sort of the batch by the top 12 or 14
// bits of each key -- one histogram pass, a scan, one scatter pass -- that writes the keys and sources in
// that order into context scratch, with the caller's index of each; K1 reads the sorted copies in
// order and writes every result at its caller index.  Order inside a bin is whatever the scatter's
// LDS atomics give: a lookup's result does not depend on the batch order, only its position does.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "engine.hpp"
#include "launch.hpp"

namespace ovs {

constexpr int KS_MAXBITS = 14;       // 2^14 bins: a 64 KB LDS histogram per block
constexpr int KS_BLOCKS = 256;       // one block per CU; a block's slice of the batch is contiguous
constexpr int KS_THREADS = 1024;

// per-block histogram of the block's slice: hist[block * KS_BINS + bin]
template <int KS_BITS>
__global__ __launch_bounds__(KS_THREADS) void k_ks_hist(const K160* __restrict__ keys, uint64_t n, uint64_t chunk,
                                                        uint32_t* __restrict__ hist)
{
    constexpr uint32_t KS_BINS = 1u << KS_BITS;
    __shared__ uint32_t h[KS_BINS];
    for (uint32_t i = threadIdx.x; i < KS_BINS; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const uint64_t lo = (uint64_t)blockIdx.x * chunk, hi = min(n, lo + chunk);
    for (uint64_t q = lo + threadIdx.x; q < hi; q += blockDim.x) atomicAdd(&h[keys[q].w[4] >> (32 - KS_BITS)], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < KS_BINS; i += blockDim.x) hist[(uint64_t)blockIdx.x * KS_BINS + i] = h[i];
}

// one thread per bin: the exclusive prefix of the bin over the blocks, in place, and the bin's total
template <int KS_BITS>
__global__ __launch_bounds__(256) void k_ks_colscan(uint32_t* __restrict__ hist, uint32_t* __restrict__ tot)
{
    constexpr uint32_t KS_BINS = 1u << KS_BITS;
    const uint32_t bin = blockIdx.x * blockDim.x + threadIdx.x;
    if (bin >= KS_BINS) return;
    uint32_t acc = 0;
    for (int g0 = 0; g0 < KS_BLOCKS; g0 += 16) {
        uint32_t v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = hist[(uint64_t)(g0 + j) * KS_BINS + bin];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            hist[(uint64_t)(g0 + j) * KS_BINS + bin] = acc;
            acc += v[j];
        }
    }
    tot[bin] = acc;
}

// exclusive scan of the bin totals (one block): base[bin]
template <int KS_BITS>
__global__ __launch_bounds__(1024) void k_ks_binscan(const uint32_t* __restrict__ tot, uint32_t* __restrict__ base)
{
    constexpr uint32_t KS_BINS = 1u << KS_BITS;
    constexpr int PER = KS_BINS / 1024;
    __shared__ uint32_t part[1024];
    const int t = threadIdx.x;
    uint32_t v[PER], s = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) { v[j] = tot[t * PER + j]; s += v[j]; }
    part[t] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        const uint32_t x = t >= off ? part[t - off] : 0u;
        __syncthreads();
        part[t] += x;
        __syncthreads();
    }
    uint32_t run = part[t] - s;   // exclusive
#pragma unroll
    for (int j = 0; j < PER; ++j) { base[t * PER + j] = run; run += v[j]; }
}

// every lookup of the block's slice to its place: position = base[bin] + the block's prefix in the
// bin + its rank among the block's lookups of that bin (LDS atomics)
template <int KS_BITS>
__global__ __launch_bounds__(KS_THREADS) void k_ks_scatter(const K160* __restrict__ keys, const uint32_t* __restrict__ src,
                                                           uint64_t n, uint64_t chunk, const uint32_t* __restrict__ hist,
                                                           const uint32_t* __restrict__ base, K160* __restrict__ skeys,
                                                           uint32_t* __restrict__ ssrc, uint32_t* __restrict__ perm)
{
    constexpr uint32_t KS_BINS = 1u << KS_BITS;
    __shared__ uint32_t cur[KS_BINS];
    for (uint32_t i = threadIdx.x; i < KS_BINS; i += blockDim.x)
        cur[i] = base[i] + hist[(uint64_t)blockIdx.x * KS_BINS + i];
    __syncthreads();
    const uint64_t lo = (uint64_t)blockIdx.x * chunk, hi = min(n, lo + chunk);
    for (uint64_t q = lo + threadIdx.x; q < hi; q += blockDim.x) {
        const K160 k = keys[q];
        const uint32_t p = atomicAdd(&cur[k.w[4] >> (32 - KS_BITS)], 1u);
        skeys[p] = k;
        ssrc[p] = src[q];
        perm[p] = (uint32_t)q;
    }
}

// scratch: hist KS_BLOCKS * bins + tot bins + base bins words, for the widest bins
uint64_t ksort_scratch_words() { return ((uint64_t)KS_BLOCKS + 2) << KS_MAXBITS; }

template <int B>
static hipError_t ksort_bits(const K160* keys, const uint32_t* src, uint64_t n, uint32_t* scratch, K160* skeys,
                             uint32_t* ssrc, uint32_t* perm, hipStream_t s)
{
    constexpr uint32_t BINS = 1u << B;
    uint32_t* hist = scratch;
    uint32_t* tot = hist + (uint64_t)KS_BLOCKS * BINS;
    uint32_t* base = tot + BINS;
    const uint64_t chunk = (n + KS_BLOCKS - 1) / KS_BLOCKS;
    hipLaunchKernelGGL(k_ks_hist<B>, dim3(KS_BLOCKS), dim3(KS_THREADS), 0, s, keys, n, chunk, hist);
    hipLaunchKernelGGL(k_ks_colscan<B>, dim3(BINS / 256), dim3(256), 0, s, hist, tot);
    hipLaunchKernelGGL(k_ks_binscan<B>, dim3(1), dim3(1024), 0, s, tot, base);
    hipLaunchKernelGGL(k_ks_scatter<B>, dim3(KS_BLOCKS), dim3(KS_THREADS), 0, s, keys, src, n, chunk, hist, base, skeys,
                       ssrc, perm);
    return hipGetLastError();
}

// bits: 12 or 14 (the top bits of a key that order the batch)
hipError_t ksort_launch(const K160* keys, const uint32_t* src, uint64_t n, uint32_t* scratch, K160* skeys,
                        uint32_t* ssrc, uint32_t* perm, int bits, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    if (n >= 0xFFFFFFFFull) return hipErrorInvalidValue;     // positions and caller indices are u32
    if (bits == 12) return ksort_bits<12>(keys, src, n, scratch, skeys, ssrc, perm, s);
    if (bits == 14) return ksort_bits<14>(keys, src, n, scratch, skeys, ssrc, perm, s);
    return hipErrorInvalidValue;
}

}  // namespace ovs
