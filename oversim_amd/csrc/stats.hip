// stats.hip -- KBRTestApp one-way statistics over a batch of route results.
//
// Reference: KBRTestApp::deliver / evaluateData / finishApp (KBRTestApp.cc:380-520),
// SendToKeyListener::lookupFinished failure branch (BaseOverlay.cc:1258-1270),
// GlobalStatistics::addStdDev / recordOutVector / finalizeStatistics
// (GlobalStatistics.cc:103-200).  OMNeT++'s cStdDev is not in the image; its
// published accumulator (count, sum, sum of squares, min, max) is restated here.
//
// Pass 1 (k_stats_lookups): one thread per lookup, grid-stride.  Integer
// counters only, so the result is independent of scheduling: register
// accumulation -> wave reduction -> one global atomic per wave; per-node
// sent/delivered/dropped counts by global atomics; hop histogram in LDS.
// Pass 2 (k_stats_nodes): per-node rates folded into cStdDev accumulators in
// a FIXED order (fixed grid, fixed stride, fixed tree), so the fp64 sums are
// deterministic run to run.  Pass 3 (k_stats_final): one block folds the
// per-block partials in index order.
// All passes are HBM-streaming (20 B per lookup + 12 B per node) and tiny
// next to the route kernels.
#include <hip/hip_runtime.h>

#include "engine.hpp"
#include "stats.hpp"

namespace ovs {

namespace {

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t w = __shfl_xor(v, o);
        v = w < v ? w : v;
    }
    return v;
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t w = __shfl_xor(v, o);
        v = w > v ? w : v;
    }
    return v;
}

// LK = false: one-way test over ovs_route_out (delivered / dropped / failed lookups).
// LK = true: lookup test over ovs_lookup_out (same 16 B slot: num_siblings, hops, status,
// is_valid, latency) and the first column of the sibling vectors: delivered = numLookupSuccess,
// dropped = numLookupFailed, failed = the !isValid part of it (KBRTestApp.cc:331-371).
template <bool LK>
__global__ __launch_bounds__(256) void k_stats_lookups(const ovs_route_out* __restrict__ out,
                                                       const K160* __restrict__ keys,
                                                       const uint32_t* __restrict__ src,
                                                       const KeyRec* __restrict__ recs, uint64_t n, uint32_t nnodes,
                                                       int lookup_node_ids, StatsDev* __restrict__ S,
                                                       uint32_t* __restrict__ node_sent,
                                                       uint32_t* __restrict__ node_deliv,
                                                       uint32_t* __restrict__ node_drop,
                                                       const uint32_t* __restrict__ first, uint64_t first_stride)
{
    __shared__ uint32_t hist[64];
    __shared__ uint32_t stat[8];
    if (threadIdx.x < 64) hist[threadIdx.x] = 0;
    if (threadIdx.x < 8) stat[threadIdx.x] = 0;
    __syncthreads();

    uint64_t deliv = 0, drop = 0, failed = 0, hops = 0, lat = 0, fhops = 0;
    uint64_t hmin = ~0ull, hmax = 0, lmin = ~0ull, lmax = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const ovs_route_out o = out[i];
        const uint32_t s = src[i];
        const bool valid_src = s < nnodes;
        atomicAdd(&stat[o.status & 7], 1u);
        if (valid_src) atomicAdd(&node_sent[s], 1u);
        if constexpr (LK) {
            // KBRTestApp::handleLookupResponse: isValid && (!lookupNodeIds || (siblings non-empty,
            // siblings[0].key == key, siblings[0] == destAddr)) -- unique IDs: the node owning key
            const bool valid = o.one_way_hops != 0;
            bool ok = valid;
            if (ok && lookup_node_ids) {
                const uint32_t f = o.responsible > 0 ? first[i * first_stride] : NONE;
                if (f < nnodes) {
                    const KeyRec r = load_rec(recs, f);
                    const K160 k = keys[i];
                    ok = r.w[0] == k.w[0] && r.w[1] == k.w[1] && r.w[2] == k.w[2] && r.w[3] == k.w[3] &&
                         r.w[4] == k.w[4];
                } else {
                    ok = false;
                }
            }
            if (!ok) {
                ++drop;
                failed += valid ? 0 : 1;
                fhops += o.hops;                  // "Failed Lookup Hop Count"
                if (valid_src) atomicAdd(&node_drop[s], 1u);
                continue;
            }
            ++deliv;
            if (valid_src) atomicAdd(&node_deliv[s], 1u);
            const uint64_t h = o.hops;          // "Lookup Hop Count"
            const uint64_t l = (uint64_t)o.latency_ns;   // "Lookup Success Latency"
            hops += h;
            lat += l;
            hmin = h < hmin ? h : hmin;
            hmax = h > hmax ? h : hmax;
            lmin = l < lmin ? l : lmin;
            lmax = l > lmax ? l : lmax;
            atomicAdd(&hist[h < 63 ? h : 63], 1u);
            continue;
        }
        if (o.status != OVS_LOOKUP_OK) {
            ++failed;
            continue;
        }
        bool ok = true;
        if (lookup_node_ids) {
            // KBRTestApp::deliver: getThisNode().getKey() == destKey (KBRTestApp.cc:407)
            if (o.responsible < nnodes) {
                const KeyRec r = load_rec(recs, o.responsible);
                const K160 k = keys[i];
                ok = r.w[0] == k.w[0] && r.w[1] == k.w[1] && r.w[2] == k.w[2] && r.w[3] == k.w[3] && r.w[4] == k.w[4];
            } else {
                ok = false;
            }
        }
        if (!ok) {
            ++drop;
            if (valid_src) atomicAdd(&node_drop[s], 1u);
            continue;
        }
        ++deliv;
        if (valid_src) atomicAdd(&node_deliv[s], 1u);
        const uint64_t h = o.one_way_hops;
        const uint64_t l = (uint64_t)o.latency_ns;
        hops += h;
        lat += l;
        hmin = h < hmin ? h : hmin;
        hmax = h > hmax ? h : hmax;
        lmin = l < lmin ? l : lmin;
        lmax = l > lmax ? l : lmax;
        atomicAdd(&hist[h < 63 ? h : 63], 1u);
    }
    deliv = wave_sum_u64(deliv);
    drop = wave_sum_u64(drop);
    failed = wave_sum_u64(failed);
    hops = wave_sum_u64(hops);
    lat = wave_sum_u64(lat);
    fhops = wave_sum_u64(fhops);
    hmin = wave_min_u64(hmin);
    hmax = wave_max_u64(hmax);
    lmin = wave_min_u64(lmin);
    lmax = wave_max_u64(lmax);
    if ((threadIdx.x & 63) == 0) {
        if (deliv) atomicAdd(&S->delivered, deliv);
        if (drop) atomicAdd(&S->dropped, drop);
        if (failed) atomicAdd(&S->failed, failed);
        if (hops) atomicAdd(&S->hop_sum, hops);
        if (lat) atomicAdd(&S->lat_sum, lat);
        if (fhops) atomicAdd(&S->fhop_sum, fhops);
        if (hmin != ~0ull) {
            atomicMin(&S->hop_min, hmin);
            atomicMax(&S->hop_max, hmax);
            atomicMin(&S->lat_min, lmin);
            atomicMax(&S->lat_max, lmax);
        }
    }
    __syncthreads();
    if (threadIdx.x < 64 && hist[threadIdx.x]) atomicAdd(&S->hist[threadIdx.x], (unsigned long long)hist[threadIdx.x]);
    if (threadIdx.x < 8 && stat[threadIdx.x]) atomicAdd(&S->status[threadIdx.x], (unsigned long long)stat[threadIdx.x]);
}

// cStdDev accumulator (OMNeT++ cStdDev::collect: n, sum, sqrsum, min, max)
struct Acc {
    double sum, sq, mn, mx;
    uint64_t n;
};

__device__ __forceinline__ void acc_init(Acc& a)
{
    a.sum = 0; a.sq = 0; a.mn = __longlong_as_double(0x7FF0000000000000ll); a.mx = -a.mn; a.n = 0;
}

__device__ __forceinline__ void acc_add(Acc& a, double v)
{
    a.sum = __dadd_rn(a.sum, v);
    a.sq = __dadd_rn(a.sq, __dmul_rn(v, v));
    a.mn = v < a.mn ? v : a.mn;
    a.mx = v > a.mx ? v : a.mx;
    ++a.n;
}

__device__ __forceinline__ void acc_merge(Acc& a, const Acc& b)
{
    a.sum = __dadd_rn(a.sum, b.sum);
    a.sq = __dadd_rn(a.sq, b.sq);
    a.mn = b.mn < a.mn ? b.mn : a.mn;
    a.mx = b.mx > a.mx ? b.mx : a.mx;
    a.n += b.n;
}

__device__ __forceinline__ void acc_store(double* p, const Acc& a)
{
    p[0] = a.sum; p[1] = a.sq; p[2] = a.mn; p[3] = a.mx; p[4] = __longlong_as_double((long long)a.n);
}

__device__ __forceinline__ void acc_load(const double* p, Acc& a)
{
    a.sum = p[0]; a.sq = p[1]; a.mn = p[2]; a.mx = p[3]; a.n = (uint64_t)__double_as_longlong(p[4]);
}

// fixed-shape tree reduction of NSTAT accumulators over a 256-thread block
__device__ void block_reduce_store(Acc (&a)[NSTAT], double* __restrict__ dst)
{
    __shared__ double sh[NSTAT * 5][256];
#pragma unroll
    for (int k = 0; k < NSTAT; ++k) {
        sh[k * 5 + 0][threadIdx.x] = a[k].sum;
        sh[k * 5 + 1][threadIdx.x] = a[k].sq;
        sh[k * 5 + 2][threadIdx.x] = a[k].mn;
        sh[k * 5 + 3][threadIdx.x] = a[k].mx;
        sh[k * 5 + 4][threadIdx.x] = __longlong_as_double((long long)a[k].n);
    }
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
#pragma unroll
            for (int k = 0; k < NSTAT; ++k) {
                Acc x, y;
                x.sum = sh[k * 5 + 0][threadIdx.x]; y.sum = sh[k * 5 + 0][threadIdx.x + w];
                x.sq = sh[k * 5 + 1][threadIdx.x]; y.sq = sh[k * 5 + 1][threadIdx.x + w];
                x.mn = sh[k * 5 + 2][threadIdx.x]; y.mn = sh[k * 5 + 2][threadIdx.x + w];
                x.mx = sh[k * 5 + 3][threadIdx.x]; y.mx = sh[k * 5 + 3][threadIdx.x + w];
                x.n = (uint64_t)__double_as_longlong(sh[k * 5 + 4][threadIdx.x]);
                y.n = (uint64_t)__double_as_longlong(sh[k * 5 + 4][threadIdx.x + w]);
                acc_merge(x, y);
                sh[k * 5 + 0][threadIdx.x] = x.sum;
                sh[k * 5 + 1][threadIdx.x] = x.sq;
                sh[k * 5 + 2][threadIdx.x] = x.mn;
                sh[k * 5 + 3][threadIdx.x] = x.mx;
                sh[k * 5 + 4][threadIdx.x] = __longlong_as_double((long long)x.n);
            }
        }
        __syncthreads();
    }
    if (threadIdx.x < NSTAT * 5) dst[threadIdx.x] = sh[threadIdx.x][0];
}

__global__ __launch_bounds__(256) void k_stats_nodes(const uint32_t* __restrict__ node_sent,
                                                     const uint32_t* __restrict__ node_deliv,
                                                     const uint32_t* __restrict__ node_drop, uint32_t nnodes,
                                                     double time_s, uint64_t msg_bytes, int rates, int lk,
                                                     double* __restrict__ partial)
{
    Acc a[NSTAT];
#pragma unroll
    for (int k = 0; k < NSTAT; ++k) acc_init(a[k]);
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nnodes; i += stride) {
        const uint32_t s = node_sent[i], d = node_deliv[i], r = node_drop[i];
        if (rates && lk) {
            // KBRTestApp::finishApp, kbrLookupTest (KBRTestApp.cc:546-557): Successful Lookups/s,
            // Failed Lookups/s, Lookup Success Ratio
            acc_add(a[0], __ddiv_rn((double)d, time_s));
            acc_add(a[2], __ddiv_rn((double)r, time_s));
            if (s > 0) acc_add(a[4], (double)__fdiv_rn((float)d, (float)s));
        } else if (rates) {
            // KBRTestApp::finishApp (KBRTestApp.cc:503-512): numDelivered / time etc.
            // (the reference divides long / simtime_t; as doubles here)
            acc_add(a[0], __ddiv_rn((double)d, time_s));
            acc_add(a[1], __ddiv_rn((double)((uint64_t)d * msg_bytes), time_s));
            acc_add(a[2], __ddiv_rn((double)r, time_s));
            acc_add(a[3], __ddiv_rn((double)((uint64_t)r * msg_bytes), time_s));
            if (s > 0) acc_add(a[4], (double)__fdiv_rn((float)d, (float)s));
        }
    }
    block_reduce_store(a, partial + (uint64_t)blockIdx.x * NSTAT * 5);
}

__global__ __launch_bounds__(256) void k_stats_final(const double* __restrict__ partial, int nblocks,
                                                     double* __restrict__ result)
{
    Acc a[NSTAT];
#pragma unroll
    for (int k = 0; k < NSTAT; ++k) acc_init(a[k]);
    for (int b = threadIdx.x; b < nblocks; b += blockDim.x) {
#pragma unroll
        for (int k = 0; k < NSTAT; ++k) {
            Acc x;
            acc_load(partial + ((uint64_t)b * NSTAT + k) * 5, x);
            acc_merge(a[k], x);
        }
    }
    block_reduce_store(a, result);
}

}  // namespace

hipError_t launch_stats(const ovs_route_out* out, const K160* keys, const uint32_t* src, const KeyRec* recs,
                        uint64_t n, uint32_t nnodes, int lookup_node_ids, double time_s, uint64_t msg_bytes,
                        int rates, StatsDev* S, uint32_t* node_counts, double* partial, double* result,
                        int num_cu, hipStream_t st, const uint32_t* first, uint64_t first_stride)
{
    const bool lk = first != nullptr;
    uint32_t* node_sent = node_counts;
    uint32_t* node_deliv = node_counts + nnodes;
    uint32_t* node_drop = node_counts + 2 * (uint64_t)nnodes;
    hipError_t e = hipMemsetAsync(node_counts, 0, sizeof(uint32_t) * 3 * (uint64_t)nnodes, st);
    if (e != hipSuccess) return e;
    StatsDev init{};
    init.hop_min = ~0ull;
    init.lat_min = ~0ull;
    e = hipMemcpyAsync(S, &init, sizeof init, hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return e;
    if (n) {
        uint64_t blocks = (n + 255) / 256;
        const uint64_t cap = (uint64_t)num_cu * 8;
        if (blocks > cap) blocks = cap;
        if (lk)
            hipLaunchKernelGGL(k_stats_lookups<true>, dim3((unsigned)blocks), dim3(256), 0, st, out, keys, src, recs, n,
                               nnodes, lookup_node_ids, S, node_sent, node_deliv, node_drop, first, first_stride);
        else
            hipLaunchKernelGGL(k_stats_lookups<false>, dim3((unsigned)blocks), dim3(256), 0, st, out, keys, src, recs, n,
                               nnodes, lookup_node_ids, S, node_sent, node_deliv, node_drop, first, first_stride);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_stats_nodes, dim3(STATS_NODE_BLOCKS), dim3(256), 0, st, node_sent, node_deliv, node_drop,
                       nnodes, time_s, msg_bytes, rates, lk ? 1 : 0, partial);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_stats_final, dim3(1), dim3(256), 0, st, partial, STATS_NODE_BLOCKS, result);
    return hipGetLastError();
}

}  // namespace ovs
