// kad.hip -- Kademlia snapshot builder, findNode and the iterative-lookup kernel (K2)
// for gfx950 (MI355X).
//
// K2 kad_route: one lane per lookup; the lane runs OverSim's IterativePathLookup
// state machine (IterativeLookup.cc:760-1195, merge = true, parallel RPCs)
// against a per-lookup future-event list of <= alpha pending FindNodeCalls
// ordered by simulated arrival time (int64 ns).  Each processed response
// evaluates the responder's Kademlia::findNode (Kademlia.cc:1101-1246) from
// its 64 B record and one 192 B bucket slot with member keys inline; sorted
// vectors (the findNode result and the LookupVector nextHops) live in
// registers with static indexing, ordered by the top 64 bits of the XOR
// distance with an exact 160-bit fallback on ties.
#include <hipcub/hipcub.hpp>

#include <cstdlib>

#include "kad_dev.hpp"

namespace ovs {

void kad_free(KadTables& t)
{
    if (t.recs) hipFree(t.recs);
    if (t.sib) hipFree(t.sib);
    if (t.sibe) hipFree(t.sibe);
    if (t.slots) hipFree(t.slots);
    t.recs = nullptr; t.sib = nullptr; t.sibe = nullptr; t.slots = nullptr; t.total_slots = 0;
}

// ---------------------------------------------------------------------------
// builder, pass A: sibling table (the 5s XOR-closest nodes, what routingAdd
// converges to: Kademlia.cc:537-616), its radius R and bucket mask

__global__ void k_kad_siblings(const KeyRec* __restrict__ recs, uint32_t n, int S5, uint32_t* __restrict__ sib,
                               KadRec* __restrict__ out, uint64_t* __restrict__ rowlen)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const K160 me = kload(recs, v);
    uint32_t* L = sib + (uint64_t)v * S5;
    int cnt = 0;
    if (n - 1 < (uint32_t)S5) {
        for (uint32_t x = 0; x < n; ++x)
            if (x != v) L[cnt++] = x;
    } else {
        uint32_t lo = 0, hi = n;
        for (int b = KEYBITS - 1; b >= 0; --b) {
            const uint32_t mid = split_bit(recs, lo, hi, b);
            const uint32_t nb = kbit(me, b);
            const uint32_t nlo = nb ? mid : lo, nhi = nb ? hi : mid;
            const uint32_t flo = nb ? lo : mid, fhi = nb ? mid : hi;
            if (nhi - nlo >= (uint32_t)S5 + 1) { lo = nlo; hi = nhi; continue; }
            // the block sharing one more bit holds < 5s+1 nodes: all of it, plus the
            // XOR-closest remainder of the other half T_b
            for (uint32_t x = nlo; x < nhi; ++x)
                if (x != v) L[cnt++] = x;
            int need = S5 - cnt;
            uint32_t rl = flo, rh = fhi;
            for (int bb = b - 1; need > 0; --bb) {
                if (rh - rl <= (uint32_t)need || bb < 0) {
                    for (uint32_t x = rl; x < rh && need > 0; ++x) { L[cnt++] = x; --need; }
                    break;
                }
                const uint32_t m2 = split_bit(recs, rl, rh, bb);
                const uint32_t nbb = kbit(me, bb);
                const uint32_t nl = nbb ? m2 : rl, nh = nbb ? rh : m2;
                const uint32_t fl = nbb ? rl : m2, fh = nbb ? m2 : rh;
                if (nh - nl >= (uint32_t)need) { rl = nl; rh = nh; }
                else {
                    for (uint32_t x = nl; x < nh; ++x) L[cnt++] = x;
                    need -= (int)(nh - nl);
                    rl = fl; rh = fh;
                }
            }
            break;
        }
    }
    for (int i = cnt; i < S5; ++i) L[i] = NONE;
    K160 R{}, M{};
    for (int i = 0; i < 5; ++i) { R.w[i] = 0; M.w[i] = 0; }
    for (int i = 0; i < cnt; ++i) {
        const K160 d = k_xor(kload(recs, L[i]), me);
        if (k_gt(d, R)) R = d;
        const int mb = k_msb(d);
        M.w[mb >> 5] |= 1u << (mb & 31);
    }
    KadRec o;
    for (int i = 0; i < 5; ++i) { o.key[i] = me.w[i]; o.R[i] = R.w[i]; o.mask[i] = M.w[i]; }
    o.boff = 0;
    out[v] = o;
    rowlen[v] = cnt > 0 ? (uint64_t)(KEYBITS - k_msb(R)) : 0;
}

__global__ void k_kad_sibentries(const KeyRec* __restrict__ recs, const uint32_t* __restrict__ sib, uint64_t total,
                                 KadEntry* __restrict__ sibe)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const uint32_t x = sib[i];
    KadEntry e;
    e.idx = x;
    const K160 k = x == NONE ? K160{{0, 0, 0, 0, 0}} : kload(recs, x);
    for (int w = 0; w < 5; ++w) e.key[w] = k.w[w];
    sibe[i] = e;
}

// 1 when two node IDs share their top 63 bits (then top-64 XOR distances of distinct nodes can
// tie and the K2 comparisons need the exact fallback, cand_lt<true>); IDs are sorted, so
// adjacent pairs suffice
__global__ void k_kad_prefix_ties(const KeyRec* __restrict__ recs, uint32_t n, uint32_t* flag)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i + 1 >= n) return;
    if (((top64(kload(recs, i)) ^ top64(kload(recs, i + 1))) >> 1) == 0) atomicOr(flag, 1u);
}

__global__ void k_kad_set_boff(KadRec* recs, const uint64_t* off, uint32_t n)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v < n) recs[v].boff = (uint32_t)off[v];
}

// builder, pass B: buckets m = 159 .. endIndex, up to k members of T_m minus
// siblings chosen by Floyd sampling (snapshot rule)
__global__ void k_kad_buckets(const KeyRec* __restrict__ recs, const KadRec* __restrict__ krec, uint32_t n, int k,
                              int S5, uint64_t seed, const uint32_t* __restrict__ sib, KadEntry* __restrict__ slots,
                              uint32_t own_lo, uint32_t own_hi)
{
    const uint32_t v = own_lo + blockIdx.x * blockDim.x + threadIdx.x;   // rows of the owned arc
    if (v >= own_hi) return;
    const KadRec r = krec[v];
    const K160 me = as_key(r.key);
    const K160 R = as_key(r.R);
    if (k_msb(R) < 0) return;
    const int endIndex = k_msb(R);
    const uint32_t* L = sib + (uint64_t)(v - own_lo) * S5;
    uint32_t lo = 0, hi = n;
    uint32_t chosen[32];
    for (int m = KEYBITS - 1; m >= endIndex; --m) {
        const uint32_t mid = split_bit(recs, lo, hi, m);
        const uint32_t nb = kbit(me, m);
        const uint32_t flo = nb ? lo : mid, fhi = nb ? mid : hi;
        KadEntry* dst = slots + ((uint64_t)r.boff + (uint64_t)(KEYBITS - 1 - m)) * k;
        uint32_t nsin = 0;
        for (int i = 0; i < S5; ++i) nsin += (L[i] != NONE && L[i] >= flo && L[i] < fhi) ? 1u : 0u;
        const uint32_t c = (fhi - flo) - nsin;
        int nch = 0;
        if (c <= (uint32_t)k) {
            for (uint32_t j = 0; j < c; ++j) chosen[nch++] = j;
        } else {
            for (uint32_t j = c - (uint32_t)k; j < c; ++j) {
                const uint32_t t = (uint32_t)(kad_hash(seed, v, (uint32_t)m, j) % (uint64_t)(j + 1));
                bool dup = false;
                for (int q = 0; q < nch; ++q) dup |= (chosen[q] == t);
                chosen[nch++] = dup ? j : t;
            }
            for (int a = 1; a < nch; ++a) {
                const uint32_t x = chosen[a];
                int q = a - 1;
                while (q >= 0 && chosen[q] > x) { chosen[q + 1] = chosen[q]; --q; }
                chosen[q + 1] = x;
            }
        }
        int outn = 0;
        if (nsin == 0) {
            for (int q = 0; q < nch; ++q) {
                const uint32_t x = flo + chosen[q];
                const K160 kx = kload(recs, x);
                for (int w = 0; w < 5; ++w) dst[outn].key[w] = kx.w[w];
                dst[outn].idx = x;
                ++outn;
            }
        } else {
            uint32_t rank = 0;
            int q = 0;
            for (uint32_t x = flo; x < fhi && q < nch; ++x) {
                bool is_sib = false;
                for (int i = 0; i < S5; ++i) is_sib |= (L[i] == x);
                if (is_sib) continue;
                if (rank == chosen[q]) {
                    const K160 kx = kload(recs, x);
                    for (int w = 0; w < 5; ++w) dst[outn].key[w] = kx.w[w];
                    dst[outn].idx = x;
                    ++outn; ++q;
                }
                ++rank;
            }
        }
        for (int q = outn; q < k; ++q) { dst[q].idx = NONE; for (int w = 0; w < 5; ++w) dst[q].key[w] = 0; }
        lo = nb ? mid : lo;
        hi = nb ? hi : mid;
    }
}

__global__ void k_kad_export(const KadRec* __restrict__ krec, const KadEntry* __restrict__ slots, uint32_t n, int k,
                             uint8_t* __restrict__ bcount, uint32_t* __restrict__ bnodes)
{
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)n * KEYBITS) return;
    const uint32_t v = (uint32_t)(t / KEYBITS);
    const int m = (int)(t % KEYBITS);
    const KadRec r = krec[v];
    const int endIndex = k_msb(as_key(r.R));
    int c = 0;
    uint32_t* o = bnodes + t * k;
    if (endIndex >= 0 && m >= endIndex) {
        const KadEntry* s = slots + ((uint64_t)r.boff + (uint64_t)(KEYBITS - 1 - m)) * k;
        for (int q = 0; q < k; ++q) {
            o[q] = s[q].idx;
            c += s[q].idx != NONE;
        }
    } else {
        for (int q = 0; q < k; ++q) o[q] = NONE;
    }
    bcount[t] = (uint8_t)c;
}

struct SendNothing {
    __device__ __forceinline__ void operator()(int, uint32_t, bool) const {}
};

// the responder's findNode evaluated in place (all tables on this GPU)
template <bool EX, bool LK>
struct LocalFindNode {
    const KadView& V;
    const K160& K;
    int redundant;
    int numSiblings;
    __device__ __forceinline__ bool ready(int) const { return true; }
    __device__ __forceinline__ void fill(int, uint32_t r, const RespGeo& g, bool sb, SVec<8>& res) const
    {
        Blk8 b;
        const int n = kad_find_node_blk<EX>(V, r, g, K, redundant, sb, b, LK ? numSiblings : 1);
#pragma unroll
        for (int i = 0; i < 8; ++i) { res.idx[i] = b.x[i]; res.d[i] = b.d[i]; }
        res.n = n;
        res.used = 0;
    }
};

template <bool RECORD>
struct HopRecorder {
    uint32_t* __restrict__ hopseq;
    uint64_t base;
    int hcm;
    __device__ __forceinline__ void operator()(int h, uint32_t r) const
    {
        if (RECORD && h < hcm) hopseq[base + h] = r;
    }
};

template <int A, bool RECORD, bool EX, bool LK>
__global__ __launch_bounds__(256) void k_kad_route(KadView V, DelayConsts DC, KadLC LC, const K160* __restrict__ qkeys,
                                                   const uint32_t* __restrict__ qsrc, uint64_t nq, uint64_t chunk,
                                                   ovs_route_out* __restrict__ out, uint32_t* __restrict__ hopseq,
                                                   uint32_t* __restrict__ rpcs_out, uint32_t* __restrict__ sib_out)
{
    const int lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    uint64_t cursor = wave * chunk;
    const uint64_t end = min(cursor + chunk, nq);
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

    bool active = false;
    uint64_t q = 0;
    KadLookup<A> L;
    SVec<8> res;
    const SendNothing on;

    while (true) {
        const uint64_t need = __ballot(!active);
        if (need != 0 && cursor < end) {
            const uint64_t mine = cursor + (uint64_t)__popcll(need & lt_mask);
            if (!active && mine < end) {
                q = mine;
                active = true;
                kad_lookup_init(L, qkeys[q], qsrc[q], V.xy);
                kad_lookup_start<A, EX, LK>(L, V, DC, LC, res, on);
            }
            cursor += (uint64_t)__popcll(need);
        }
        if (!__any(active)) break;
        if (!active) continue;

        if (!kad_lookup_done(L)) {
            const LocalFindNode<EX, LK> fn{V, L.K, LC.redundant, LC.numSiblings};
            const HopRecorder<RECORD> rec{hopseq, q * (uint64_t)LC.hopCountMax, LC.hopCountMax};
            kad_lookup_event<A, EX, LK>(L, V, DC, LC, res, fn, on, rec);
        }
        if (kad_lookup_done(L)) {
            const ovs_route_out o = kad_lookup_output(L, V, DC, LC);
            out[q] = o;
            if (rpcs_out) rpcs_out[q] = L.nsent;
            if (LK) {
                // LookupCall: the siblings vector = the answering response's nodes (start(): the
                // local findNode result), pushed in order up to numSiblings (IterativeLookup.cc:406-449)
                const bool ok = o.status == OVS_LOOKUP_OK;
                uint32_t* row = sib_out + q * (uint64_t)LC.numSiblings;
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (j < LC.numSiblings) row[j] = (ok && j < res.n) ? res.idx[j] : NONE;
            }
            active = false;
        }
    }
}

// batched findNode (general numRedundantNodes <= 16, 1 <= numSiblings <= 16) for the ABI
__global__ void k_kad_find_node(KadView V, const uint32_t* __restrict__ node, const K160* __restrict__ keys, uint64_t n,
                                int numRedundant, int numSiblings, uint32_t* __restrict__ out_nodes, uint32_t max_out,
                                uint8_t* __restrict__ out_count, uint8_t* __restrict__ out_sib)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = node[i];
    const K160 K = keys[i];
    const KadRec r = kad_rec(V.recs, c);
    const bool sb = kad_is_sibling(V, r, c, K, numSiblings);
    SVec<16> res;
    kad_find_node1(V, c, r, K, numRedundant, sb, res, numSiblings);
    uint32_t* o = out_nodes + i * max_out;
    for (uint32_t j = 0; j < max_out; ++j) o[j] = NONE;
#pragma unroll
    for (int j = 0; j < 16; ++j)
        if (j < res.n && (uint32_t)j < max_out) o[j] = res.idx[j];
    out_count[i] = (uint8_t)(res.n < (int)max_out ? res.n : (int)max_out);
    out_sib[i] = sb ? 1 : 0;
}

// ---------------------------------------------------------------------------
// host side

static inline unsigned nblk(uint64_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

hipError_t kad_build(const KeyRec* recs, uint32_t n, int k, int s, uint64_t seed, KadTables& t, hipStream_t st,
                     uint32_t lo, uint32_t hi)
{
    hipError_t e;
    kad_free(t);
    if (hi > n) hi = n;
    if (lo >= hi) return hipErrorInvalidValue;
    t.k = k; t.s = s; t.seed = seed; t.lo = lo; t.hi = hi;
    const int S5 = 5 * s;
    const uint32_t nown = hi - lo;
    const bool whole = lo == 0 && hi == n;
    uint64_t *rowlen = nullptr, *off = nullptr;
    uint32_t* sib_all = nullptr;
    void* tmp = nullptr;
    size_t tmpb = 0;
    auto cleanup = [&]() {
        if (rowlen) hipFree(rowlen);
        if (off) hipFree(off);
        if (tmp) hipFree(tmp);
        if (sib_all && sib_all != t.sib) hipFree(sib_all);
    };
    // node records (key, sibling radius R, mask) for the whole ring: a lookup needs every
    // responder's isSiblingFor when it sends the call; sibling lists are a build temporary
    if ((e = hipMalloc(&t.recs, sizeof(KadRec) * n)) != hipSuccess) return e;
    if ((e = hipMalloc(&sib_all, sizeof(uint32_t) * (uint64_t)n * S5)) != hipSuccess) return e;
    if ((e = hipMalloc(&rowlen, sizeof(uint64_t) * (n + 1))) != hipSuccess) { cleanup(); return e; }
    if ((e = hipMalloc(&off, sizeof(uint64_t) * (n + 1))) != hipSuccess) { cleanup(); return e; }
    hipLaunchKernelGGL(k_kad_siblings, dim3(nblk(n, 128)), dim3(128), 0, st, recs, n, S5, sib_all, t.recs, rowlen);
    // bucket rows only for the owned arc
    if (lo) hipMemsetAsync(rowlen, 0, sizeof(uint64_t) * lo, st);
    hipMemsetAsync(rowlen + hi, 0, sizeof(uint64_t) * (n + 1 - hi), st);
    hipcub::DeviceScan::ExclusiveSum(nullptr, tmpb, rowlen, off, n + 1, st);
    if ((e = hipMalloc(&tmp, tmpb)) != hipSuccess) { cleanup(); return e; }
    hipcub::DeviceScan::ExclusiveSum(tmp, tmpb, rowlen, off, n + 1, st);
    uint64_t total = 0;
    hipMemcpyAsync(&total, off + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st);
    if ((e = hipStreamSynchronize(st)) != hipSuccess) { cleanup(); return e; }
    if (total >= 0xFFFFFFFFull) { cleanup(); return hipErrorInvalidValue; }
    t.total_slots = total;
    if ((e = hipMalloc(&t.slots, sizeof(KadEntry) * (total + 1) * k)) != hipSuccess) { cleanup(); return e; }
    hipLaunchKernelGGL(k_kad_set_boff, dim3(nblk(n, 256)), dim3(256), 0, st, t.recs, off, n);
    if (whole) {
        t.sib = sib_all;
    } else {
        if ((e = hipMalloc(&t.sib, sizeof(uint32_t) * (uint64_t)nown * S5)) != hipSuccess) { cleanup(); return e; }
        hipMemcpyAsync(t.sib, sib_all + (uint64_t)lo * S5, sizeof(uint32_t) * (uint64_t)nown * S5,
                       hipMemcpyDeviceToDevice, st);
    }
    if ((e = hipMalloc(&t.sibe, sizeof(KadEntry) * (uint64_t)nown * S5)) != hipSuccess) { cleanup(); return e; }
    hipLaunchKernelGGL(k_kad_sibentries, dim3(nblk((uint64_t)nown * S5, 256)), dim3(256), 0, st, recs, t.sib,
                       (uint64_t)nown * S5, t.sibe);
    hipLaunchKernelGGL(k_kad_buckets, dim3(nblk(nown, 64)), dim3(64), 0, st, recs, t.recs, n, k, S5, seed, t.sib,
                       t.slots, lo, hi);
    uint32_t* tie = nullptr;
    uint32_t htie = 1;
    if ((e = hipMalloc(&tie, sizeof(uint32_t))) != hipSuccess) { cleanup(); return e; }
    hipMemsetAsync(tie, 0, sizeof(uint32_t), st);
    if (n > 1) hipLaunchKernelGGL(k_kad_prefix_ties, dim3(nblk(n, 256)), dim3(256), 0, st, recs, n, tie);
    hipMemcpyAsync(&htie, tie, sizeof(uint32_t), hipMemcpyDeviceToHost, st);
    e = hipStreamSynchronize(st);
    hipFree(tie);
    cleanup();
    if (e != hipSuccess) return e;
    t.exact = htie != 0 || getenv("OVS_KAD_EXACT") != nullptr;
    return hipGetLastError();
}

hipError_t kad_export(const KadTables& t, uint32_t n, uint32_t* siblings, uint8_t* bucket_count, uint32_t* bucket_nodes,
                      hipStream_t st)
{
    hipError_t e;
    const int S5 = 5 * t.s;
    uint8_t* dc = nullptr;
    uint32_t* dn = nullptr;
    const uint64_t tot = (uint64_t)n * KEYBITS;
    if ((e = hipMalloc(&dc, tot)) != hipSuccess) return e;
    if ((e = hipMalloc(&dn, sizeof(uint32_t) * tot * t.k)) != hipSuccess) { hipFree(dc); return e; }
    hipLaunchKernelGGL(k_kad_export, dim3(nblk(tot, 256)), dim3(256), 0, st, t.recs, t.slots, n, t.k, dc, dn);
    hipMemcpyAsync(bucket_count, dc, tot, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(bucket_nodes, dn, sizeof(uint32_t) * tot * t.k, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(siblings, t.sib, sizeof(uint32_t) * (uint64_t)n * S5, hipMemcpyDeviceToHost, st);
    e = hipStreamSynchronize(st);
    hipFree(dc); hipFree(dn);
    return e;
}

template <int A, bool RECORD, bool EX, bool LK>
static int kad_blocks_per_cu()
{
    static int bpc = 0;
    if (bpc == 0) {
        int b = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_kad_route<A, RECORD, EX, LK>, 256, 0) != hipSuccess || b < 1)
            b = 1;
        bpc = b;
    }
    return bpc;
}

template <int A, bool RECORD, bool EX, bool LK>
static hipError_t kad_launch(const KadView& V, const DelayConsts& DC, const KadLC& LC, const K160* qkeys,
                             const uint32_t* qsrc, uint64_t nq, ovs_route_out* out, uint32_t* hopseq, uint32_t* rpcs,
                             uint32_t* sibs, int num_cu, hipStream_t st)
{
    const uint64_t waves = (uint64_t)num_cu * kad_blocks_per_cu<A, RECORD, EX, LK>() * 4;
    uint64_t chunk = (nq + waves - 1) / waves;
    if (chunk < 1) chunk = 1;
    const uint64_t need_waves = (nq + chunk - 1) / chunk;
    hipLaunchKernelGGL((k_kad_route<A, RECORD, EX, LK>), dim3((unsigned)((need_waves + 3) / 4)), dim3(256), 0, st, V, DC, LC,
                       qkeys, qsrc, nq, chunk, out, hopseq, rpcs, sibs);
    return hipGetLastError();
}

hipError_t kad_route(const KadTables& t, const KeyRec* recs, const double2* xy, uint32_t n, const ovs_params& P,
                     const DelayConsts& DC, const K160* qkeys, const uint32_t* qsrc, uint64_t nq, ovs_route_out* out,
                     uint32_t* hopseq, uint32_t* rpcs, int num_cu, hipStream_t st, uint32_t* sibs)
{
    (void)recs;
    if (nq == 0) return hipSuccess;
    if (!kad_params_supported(P, t)) return hipErrorNotSupported;
    const KadLC LC = kad_make_lc(P, t);
    const KadView V = kad_make_view(t, xy, n);
    // strictParallelRpcs: never more than alpha FindNodeCalls in flight (IterativeLookup.cc:1078-1079)
    const int A = P.lookupParallelRpcs;
    // LookupCall batches (sibs != nullptr) record no hop sequence
    if (sibs && hopseq) return hipErrorNotSupported;
#define KLX(a, x) (sibs     ? kad_launch<a, false, x, true>(V, DC, LC, qkeys, qsrc, nq, out, hopseq, rpcs, sibs, num_cu, st) \
                   : hopseq ? kad_launch<a, true, x, false>(V, DC, LC, qkeys, qsrc, nq, out, hopseq, rpcs, sibs, num_cu, st) \
                            : kad_launch<a, false, x, false>(V, DC, LC, qkeys, qsrc, nq, out, hopseq, rpcs, sibs, num_cu, st))
#define KL(a) (t.exact ? KLX(a, true) : KLX(a, false))
    switch (A) {
    case 1: return KL(1);
    case 2: return KL(2);
    case 3: return KL(3);
    default: return KL(4);
    }
#undef KL
#undef KLX
}

hipError_t kad_find_node(const KadTables& t, const KeyRec* recs, uint32_t n, const ovs_params& P, const uint32_t* node,
                         const K160* keys, uint64_t nq, int numRedundant, int numSiblings, uint32_t* out_nodes,
                         uint32_t max_out, uint8_t* out_count, uint8_t* out_sib, hipStream_t st)
{
    (void)recs; (void)P;
    if (nq == 0) return hipSuccess;
    if (numSiblings < 1 || numSiblings > 16 || numRedundant > 16) return hipErrorNotSupported;
    const KadView V = kad_make_view(t, nullptr, n);
    hipLaunchKernelGGL(k_kad_find_node, dim3(nblk(nq, 128)), dim3(128), 0, st, V, node, keys, nq, numRedundant, numSiblings, out_nodes,
                       max_out, out_count, out_sib);
    return hipGetLastError();
}

}  // namespace ovs
