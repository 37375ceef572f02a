// compact.hip -- stable compaction by class tag (compact.hpp): count, scan, scatter.
#include "compact.hpp"

#include <hipcub/hipcub.hpp>

namespace ovs {

namespace {

// one wave per tile of CT_STEPS elements per lane: 8 measured 0.34 ms against 0.41 for 16 (10M
// elements at W = 8's tag mix, tools/diag/compact_bench.hip, profiles/r05_cbench)
constexpr int CT_STEPS = 8;
constexpr uint64_t CT_TILE = 64 * CT_STEPS;
constexpr int CT_BATCH = 4;                     // steps whose record loads precede their stores

__device__ __forceinline__ uint8_t tag_at(const uint8_t* __restrict__ tags, uint64_t n, uint64_t e)
{
    return e < n ? tags[e] : (uint8_t)0xFF;
}

// cnt[c * nb + b] = elements of class c in tile b
__global__ __launch_bounds__(64) void k_compact_count(const uint8_t* __restrict__ tags, uint64_t n, int nclass,
                                                      uint64_t nb, unsigned long long* __restrict__ cnt)
{
    __shared__ unsigned int h[CMAX];
    const int lane = threadIdx.x;
    const uint64_t b = blockIdx.x;
    for (int c = lane; c < nclass; c += 64) h[c] = 0;
    __syncthreads();
#pragma unroll 4
    for (int k = 0; k < CT_STEPS; ++k) {
        const uint8_t t = tag_at(tags, n, b * CT_TILE + (uint64_t)k * 64 + lane);
        if (t < nclass) atomicAdd(&h[t], 1u);
    }
    __syncthreads();
    for (int c = lane; c < nclass; c += 64) cnt[(uint64_t)c * nb + b] = h[c];
}

// per class: the position of its first record (one thread, <= CMAX classes).  A counter group (a
// class and the classes chained to it) reserves its records with one atomicAdd on its counter:
// compactions on other streams may share the counter (the two cohorts of a Chord shard step
// append to one done buffer), and a plain read-modify-write there let two groups take the same
// positions.
__global__ void k_compact_base(CPlan P, int nclass, uint64_t nb, const unsigned long long* __restrict__ scan,
                               long long* __restrict__ cbase)
{
    int c = 0;
    while (c < nclass) {
        int e = c + 1;
        while (e < nclass && plan_class(P, e).chain) ++e;
        unsigned long long* hc = plan_class(P, c).counter;
        const unsigned long long g0 = scan[(uint64_t)c * nb], g1 = scan[(uint64_t)e * nb];
        long long run = hc ? (long long)atomicAdd(hc, g1 - g0) : 0;
        for (int j = c; j < e; ++j) {
            const unsigned long long s0 = scan[(uint64_t)j * nb], s1 = scan[(uint64_t)(j + 1) * nb];
            cbase[j] = run - (long long)s0;
            run += (long long)(s1 - s0);
        }
        c = e;
    }
}

// The tile's ranks first (ballots and the LDS class offsets only), then its copies in batches of
// CT_BATCH steps whose record loads are all issued before their stores (ranking, loading and
// storing step by step measured 0.41 ms against 0.34; staging the tile's records in LDS by class
// to write each class's run as whole lines, 0.40-0.78 ms: 25-50 KB of LDS a wave left too few
// waves resident).  Records above 48 B (Kademlia migration records) are copied where ranked.
__global__ __launch_bounds__(64) void k_compact_scatter(const uint8_t* __restrict__ tags, uint64_t n, CPlan P,
                                                        int nclass, uint64_t nb,
                                                        const unsigned long long* __restrict__ scan,
                                                        const long long* __restrict__ cbase)
{
    __shared__ long long off[CMAX];
    const int lane = threadIdx.x;
    const uint64_t b = blockIdx.x;
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    for (int c = lane; c < nclass; c += 64) off[c] = cbase[c] + (long long)scan[(uint64_t)c * nb + b];
    // the tile's tags, all requested before the first step needs one
    uint8_t tt[CT_STEPS];
#pragma unroll
    for (int k = 0; k < CT_STEPS; ++k) tt[k] = tag_at(tags, n, b * CT_TILE + (uint64_t)k * 64 + lane);
    __syncthreads();
    long long pos[CT_STEPS];
#pragma unroll
    for (int k = 0; k < CT_STEPS; ++k) {
        const uint8_t t = tt[k];
        const bool mine = t < nclass;
        uint64_t rem = __ballot(mine);
        long long p = -1;
        // one pass per class present in this group of 64: stable ranks by ballot
        while (rem) {
            const int l0 = __ffsll((long long)rem) - 1;
            const int c = __shfl((int)t, l0);
            const uint64_t m = __ballot(mine && (int)t == c);
            const long long o = off[c];
            if (mine && (int)t == c) p = o + (long long)__popcll(m & lt);
            __builtin_amdgcn_wave_barrier();
            if (lane == l0) off[c] = o + (long long)__popcll(m);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            rem &= ~m;
        }
        pos[k] = p;
    }
#pragma unroll
    for (int k0 = 0; k0 < CT_STEPS; k0 += CT_BATCH) {
        uint4 q[CT_BATCH][3];
        uint8_t* dp[CT_BATCH];
        int mode[CT_BATCH];     // 0: nothing, 1: 16 B words, 2: 8 B words, 3: copied already (> 48 B)
        uint32_t nw[CT_BATCH];
#pragma unroll
        for (int kk = 0; kk < CT_BATCH; ++kk) {
            const int k = k0 + kk;
            const uint64_t e = b * CT_TILE + (uint64_t)k * 64 + lane;
            const uint8_t t = tt[k];
            mode[kk] = 0; dp[kk] = nullptr; nw[kk] = 0;
            if (t < nclass) {
                const CClass C = plan_class(P, t);
                if (C.dst && pos[k] >= 0 && (uint64_t)pos[k] < C.cap) {
                    const uint8_t* sp = C.src + e * C.src_stride;
                    dp[kk] = C.dst + (uint64_t)pos[k] * C.rec_bytes;
                    if (C.lab) C.lab[pos[k]] = C.label;
                    if (C.rec_bytes > 48) {
                        mode[kk] = 3;
                        const uint2* s = reinterpret_cast<const uint2*>(sp);
                        uint2* d = reinterpret_cast<uint2*>(dp[kk]);
                        for (uint32_t w = 0; w < C.rec_bytes / 8; ++w) d[w] = s[w];
                    } else if (((C.rec_bytes | (uint32_t)C.src_stride | (uint32_t)(uintptr_t)sp |
                                 (uint32_t)(uintptr_t)dp[kk]) & 15) == 0) {
                        // 16 B moves (the 48 B hand-off records: 3 per record)
                        mode[kk] = 1; nw[kk] = C.rec_bytes / 16;
                        const uint4* s = reinterpret_cast<const uint4*>(sp);
#pragma unroll
                        for (int w = 0; w < 3; ++w)
                            if ((uint32_t)w < nw[kk]) q[kk][w] = s[w];
                    } else {
                        mode[kk] = 2; nw[kk] = C.rec_bytes / 8;
                        const uint2* s = reinterpret_cast<const uint2*>(sp);
#pragma unroll
                        for (int w = 0; w < 6; ++w)
                            if ((uint32_t)w < nw[kk]) {
                                const uint2 x = s[w];
                                if (w & 1) { q[kk][w >> 1].z = x.x; q[kk][w >> 1].w = x.y; }
                                else { q[kk][w >> 1].x = x.x; q[kk][w >> 1].y = x.y; }
                            }
                    }
                }
            }
        }
#pragma unroll
        for (int kk = 0; kk < CT_BATCH; ++kk) {
            if (mode[kk] == 1) {
                uint4* d = reinterpret_cast<uint4*>(dp[kk]);
#pragma unroll
                for (int w = 0; w < 3; ++w)
                    if ((uint32_t)w < nw[kk]) d[w] = q[kk][w];
            } else if (mode[kk] == 2) {
                uint2* d = reinterpret_cast<uint2*>(dp[kk]);
#pragma unroll
                for (int w = 0; w < 6; ++w)
                    if ((uint32_t)w < nw[kk])
                        d[w] = (w & 1) ? make_uint2(q[kk][w >> 1].z, q[kk][w >> 1].w)
                                       : make_uint2(q[kk][w >> 1].x, q[kk][w >> 1].y);
            }
        }
    }
}

}  // namespace

void compact_free(CompactScratch& s)
{
    if (s.buf) hipFree(s.buf);
    s.buf = nullptr;
    s.bytes = 0;
}

void stage_free(StageBuf& b)
{
    if (b.buf) hipFree(b.buf);
    b.buf = nullptr;
    b.bytes = 0;
    compact_free(b.cs);
}

hipError_t stage_ensure(StageBuf& b, size_t bytes, hipStream_t s)
{
    if (bytes <= b.bytes) return hipSuccess;
    hipError_t e;
    if (b.buf) {
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        hipFree(b.buf);
        b.buf = nullptr;
        b.bytes = 0;
    }
    bytes = (bytes + 255) & ~(size_t)255;
    if ((e = hipMalloc(&b.buf, bytes)) != hipSuccess) return e;
    b.bytes = bytes;
    return hipSuccess;
}

hipError_t compact_by_tag(const uint8_t* tags, uint64_t n, const CPlan& P, CompactScratch& scr, hipStream_t s)
{
    const int nclass = P.seg.n + P.nextra;
    if (nclass < 1 || nclass > CMAX || P.nextra < 0 || P.nextra > 2) return hipErrorInvalidValue;
    for (int c = 0; c < nclass; ++c) {
        const CClass k = plan_class(P, c);
        if (k.dst && (k.rec_bytes % 8 != 0 || k.src_stride % 8 != 0)) return hipErrorInvalidValue;
    }
    const uint64_t nb = n ? (n + CT_TILE - 1) / CT_TILE : 1;
    const uint64_t ncnt = (uint64_t)nclass * nb + 1;
    size_t tmpb = 0;
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, tmpb, (unsigned long long*)nullptr,
                                                    (unsigned long long*)nullptr, ncnt, s);
    if (e != hipSuccess) return e;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_base = 0, o_cnt = o_base + al(sizeof(long long) * CMAX), o_scan = o_cnt + al(8 * ncnt),
                 o_tmp = o_scan + al(8 * ncnt), need = o_tmp + al(tmpb);
    if (need > scr.bytes) {
        // the stream may still use the old buffer
        if (scr.buf && (e = hipStreamSynchronize(s)) != hipSuccess) return e;
        compact_free(scr);
        if ((e = hipMalloc(&scr.buf, need)) != hipSuccess) return e;
        scr.bytes = need;
    }
    uint8_t* base = static_cast<uint8_t*>(scr.buf);
    long long* cbase = reinterpret_cast<long long*>(base + o_base);
    unsigned long long* cnt = reinterpret_cast<unsigned long long*>(base + o_cnt);
    unsigned long long* scan = reinterpret_cast<unsigned long long*>(base + o_scan);
    // the trailing entry (0) makes scan[nclass * nb] the grand total
    if ((e = hipMemsetAsync(cnt + ncnt - 1, 0, 8, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_compact_count, dim3((unsigned)nb), dim3(64), 0, s, tags, n, nclass, nb, cnt);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipcub::DeviceScan::ExclusiveSum(base + o_tmp, tmpb, cnt, scan, ncnt, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_compact_base, dim3(1), dim3(1), 0, s, P, nclass, nb, scan, cbase);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_compact_scatter, dim3((unsigned)nb), dim3(64), 0, s, tags, n, P, nclass, nb, scan, cbase);
    return hipGetLastError();
}

// finished records whose qid word is 0xFFFFFFFF: rows of an exchange receive buffer nobody wrote
// (0xFF-filled), which the step kernel finishes as BROKEN instead of routing
__global__ void k_count_sentinel(const ovs_done_rec* __restrict__ done, uint64_t n, unsigned long long* out)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool hit = i < n && done[i].qid == 0xFFFFFFFFu;
    const uint64_t b = __ballot(hit);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(out, (unsigned long long)__popcll(b));
}

hipError_t count_sentinel_records(const ovs_done_rec* done, uint64_t n, unsigned long long* out, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(out, 0, sizeof(unsigned long long), s);
    if (e != hipSuccess || n == 0) return e;
    hipLaunchKernelGGL(k_count_sentinel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, done, n, out);
    return hipGetLastError();
}

}  // namespace ovs
