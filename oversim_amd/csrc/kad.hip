// kad.hip -- Kademlia table builders (snapshot rule and explicit tables), findNode and the
// iterative-lookup kernel (K2) for gfx950 (MI355X).
//
// K2 k_kad_lanes: one lane per lookup running OverSim's IterativePathLookup (IterativeLookup.cc:
// 760-1195, merge = true, parallel RPCs) against <= alpha pending FindNodeCalls ordered by
// simulated arrival time (int64 ns), as a per-lane state machine in the manner of K1: every loop
// iteration a lane consumes the one 64 B table line it requested in the previous iteration --
// the KadNode of a node it sends a FindNodeCall to, or a line of the bucket / sibling rows the
// responder's Kademlia::findNode scans (Kademlia.cc:1101-1246) -- advances its lookup as far as
// it can without memory (event selection, timeouts, the LookupVector merge, the sends' tx-queue
// timing), and requests its next line.  Lines are gathered cooperatively (4 lanes x 16 B per
// line) through LDS, finished lanes refill from the wave's slice; the grid is persistent.
#include <hipcub/hipcub.hpp>

#include <cstdlib>

#include "kad_dev.hpp"

namespace ovs {

void kad_free(KadTables& t)
{
    if (t.nodes) hipFree(t.nodes);
    if (t.nodex) hipFree(t.nodex);
    if (t.lines) hipFree(t.lines);
    if (t.sib) hipFree(t.sib);
    t.nodes = nullptr; t.nodex = nullptr; t.lines = nullptr; t.sib = nullptr; t.rows_lines = 0;
}

// ---------------------------------------------------------------------------
// builders

// the KadNode summary of a node's sibling set: R = max (s ^ key), level mask = OR 2^msb(s ^ key)
__device__ void kad_node_summary(const KeyRec* __restrict__ recs, const double2* __restrict__ xy, uint32_t v,
                                 const uint32_t* L, int cnt, int rowlo, KadNode* __restrict__ out, KadX* __restrict__ ox)
{
    const K160 me = kload(recs, v);
    K160 R{}, M{};
    for (int i = 0; i < 5; ++i) { R.w[i] = 0; M.w[i] = 0; }
    for (int i = 0; i < cnt; ++i) {
        const K160 d = k_xor(kload(recs, L[i]), me);
        if (k_gt(d, R)) R = d;
        const int mb = k_msb(d);
        M.w[mb >> 5] |= 1u << (mb & 31);
    }
    const int end = cnt > 0 ? k_msb(R) : -1;
    const int mlo = end > 63 ? end - 63 : 0;
    // mask window: bits [mlo, mlo + 63]
    const int wi = mlo >> 5, sh = mlo & 31;
    const uint64_t lo = (uint64_t)M.w[wi] | ((uint64_t)(wi + 1 < 5 ? M.w[wi + 1] : 0u) << 32);
    const uint64_t hi = wi + 2 < 5 ? (uint64_t)M.w[wi + 2] : 0ull;
    const uint64_t win = sh ? ((lo >> sh) | (hi << (64 - sh))) : lo;
    bool out_bits = false;
    for (int b = 0; b < mlo; ++b) out_bits |= kbit(M, b) != 0;
    const double2 p = xy[v];
    KadNode o;
    for (int i = 0; i < 5; ++i) o.key[i] = me.w[i];
    o.boff = 0;
    o.x = p.x; o.y = p.y;
    o.rtop = ktop(R);
    o.mwin = win;
    o.meta = (uint32_t)(end + 1) | ((uint32_t)(rowlo + 1) << 8) | ((uint32_t)cnt << 16) | (out_bits ? KMETA_MASK_OUT : 0u);
    o.spare = 0;
    out[v] = o;
    KadX x;
    for (int i = 0; i < 5; ++i) { x.R[i] = R.w[i]; x.mask[i] = M.w[i]; }
    ox[v] = x;
}

// snapshot pass A: sibling table (the 5s XOR-closest nodes, what routingAdd converges to:
// Kademlia.cc:537-616) and the node summary; the row length for the owned arc
__global__ void k_kad_siblings(const KeyRec* __restrict__ recs, const double2* __restrict__ xy, uint32_t n, int S5,
                               int lps, uint32_t own_lo, uint32_t own_hi, uint32_t* __restrict__ sib,
                               KadNode* __restrict__ out, KadX* __restrict__ ox, uint64_t* __restrict__ rowlen)
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
    // buckets below endIndex hold only siblings: the stored row starts at endIndex
    int end = -1;
    {
        K160 R{};
        for (int i = 0; i < 5; ++i) R.w[i] = 0;
        for (int i = 0; i < cnt; ++i) {
            const K160 d = k_xor(kload(recs, L[i]), me);
            if (k_gt(d, R)) R = d;
        }
        end = cnt > 0 ? k_msb(R) : -1;
    }
    kad_node_summary(recs, xy, v, L, cnt, end, out, ox);
    rowlen[v] = (v >= own_lo && v < own_hi && end >= 0) ? (uint64_t)(KEYBITS - end) * lps : 0;
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

__global__ void k_kad_set_boff(KadNode* nodes, const uint64_t* off, uint32_t lo, uint32_t hi)
{
    const uint32_t v = lo + blockIdx.x * blockDim.x + threadIdx.x;
    if (v < hi) nodes[v].boff = (uint32_t)off[v];
}

__device__ __forceinline__ void put_entry(KadLine* __restrict__ lines, uint64_t line0, int q, uint32_t x,
                                          const KeyRec* __restrict__ recs)
{
    KadLine* l = lines + line0 + q / KLINE;
    l->idx[q % KLINE] = x;
    l->top[q % KLINE] = x == NONE ? ~0ull : ktop(kload(recs, x));
}

// snapshot pass B: buckets m = 159 .. endIndex of the owned nodes, up to k members of T_m minus
// siblings chosen by Floyd sampling (snapshot rule); sibling rows
__global__ void k_kad_buckets(const KeyRec* __restrict__ recs, const KadNode* __restrict__ nodes, uint32_t n, int k,
                              int lps, int S5, int sln, uint64_t seed, const uint32_t* __restrict__ sib,
                              KadLine* __restrict__ lines, uint64_t sib_base, uint32_t own_lo, uint32_t own_hi)
{
    const uint32_t v = own_lo + blockIdx.x * blockDim.x + threadIdx.x;   // rows of the owned arc
    if (v >= own_hi) return;
    const KadNode r = nodes[v];
    const K160 me = as_key(r.key);
    const uint32_t* L = sib + (uint64_t)v * S5;
    // sibling row
    for (int q = 0; q < sln * KLINE; ++q) put_entry(lines, sib_base + (uint64_t)(v - own_lo) * sln, q, q < S5 ? L[q] : NONE, recs);
    const int endIndex = kad_end(r.meta);
    if (endIndex < 0) return;
    uint32_t lo = 0, hi = n;
    uint32_t chosen[32];
    for (int m = KEYBITS - 1; m >= endIndex; --m) {
        const uint32_t mid = split_bit(recs, lo, hi, m);
        const uint32_t nb = kbit(me, m);
        const uint32_t flo = nb ? lo : mid, fhi = nb ? mid : hi;
        const uint64_t line0 = (uint64_t)r.boff + (uint64_t)(KEYBITS - 1 - m) * lps;
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
            for (int q = 0; q < nch; ++q) put_entry(lines, line0, outn++, flo + chosen[q], recs);
        } else {
            uint32_t rank = 0;
            int q = 0;
            for (uint32_t x = flo; x < fhi && q < nch; ++x) {
                bool is_sib = false;
                for (int i = 0; i < S5; ++i) is_sib |= (L[i] == x);
                if (is_sib) continue;
                if (rank == chosen[q]) { put_entry(lines, line0, outn++, x, recs); ++q; }
                ++rank;
            }
        }
        for (int q = outn; q < lps * KLINE; ++q) put_entry(lines, line0, q, NONE, recs);
        lo = nb ? mid : lo;
        hi = nb ? hi : mid;
    }
}

// explicit tables, pass A: validate a node's tables against the invariants OverSim's routingAdd
// keeps (Kademlia.cc:432-756): members are other nodes, a bucket m holds only nodes with
// msb(x ^ self) = m, no node twice, no node both sibling and bucket member; summary + row length
__global__ void k_kad_explicit_nodes(const KeyRec* __restrict__ recs, const double2* __restrict__ xy, uint32_t n,
                                     int k, int S5, int lps, uint32_t* __restrict__ sib, const uint8_t* __restrict__ bcount,
                                     const uint32_t* __restrict__ bnodes, KadNode* __restrict__ out, KadX* __restrict__ ox,
                                     uint64_t* __restrict__ rowlen, uint32_t* err, uint32_t* short_flag)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const K160 me = kload(recs, v);
    uint32_t* L = sib + (uint64_t)v * S5;
    // compact the sibling list (NONE entries may be anywhere)
    int cnt = 0;
    for (int i = 0; i < S5; ++i) {
        const uint32_t x = L[i];
        if (x == NONE) continue;
        L[cnt++] = x;
    }
    for (int i = cnt; i < S5; ++i) L[i] = NONE;
    uint32_t code = 0;
    for (int i = 0; i < cnt && !code; ++i) {
        if (L[i] >= n || L[i] == v) code = 1;
        for (int j = 0; j < i && !code; ++j) if (L[j] == L[i]) code = 2;
    }
    int lowest = -1;
    for (int m = 0; m < KEYBITS && !code; ++m) {
        const int c = bcount[(uint64_t)v * KEYBITS + m];
        if (c > k) { code = 3; break; }
        if (c && lowest < 0) lowest = m;
        const uint32_t* B = bnodes + ((uint64_t)v * KEYBITS + m) * k;
        for (int q = 0; q < c && !code; ++q) {
            const uint32_t x = B[q];
            if (x >= n || x == v) { code = 4; break; }
            if (k_msb(k_xor(kload(recs, x), me)) != m) { code = 5; break; }
            for (int j = 0; j < q; ++j) if (B[j] == x) code = 6;
            for (int i = 0; i < cnt; ++i) if (L[i] == x) code = 7;
        }
    }
    if (code) {
        if (atomicCAS(err, NONE, v) == NONE) err[1] = code;
        return;
    }
    K160 R{};
    for (int i = 0; i < 5; ++i) R.w[i] = 0;
    for (int i = 0; i < cnt; ++i) {
        const K160 d = k_xor(kload(recs, L[i]), me);
        if (k_gt(d, R)) R = d;
    }
    const int end = cnt > 0 ? k_msb(R) : -1;
    const int rowlo = end < 0 ? lowest : (lowest >= 0 && lowest < end ? lowest : end);
    kad_node_summary(recs, xy, v, L, cnt, rowlo, out, ox);
    rowlen[v] = rowlo >= 0 ? (uint64_t)(KEYBITS - rowlo) * lps : 0;
    if (cnt + 1 < 8) atomicOr(short_flag, 1u);
}

// explicit tables, pass B: bucket rows and sibling rows as lines
__global__ void k_kad_explicit_rows(const KeyRec* __restrict__ recs, const KadNode* __restrict__ nodes, uint32_t n,
                                    int k, int lps, int S5, int sln, const uint32_t* __restrict__ sib,
                                    const uint8_t* __restrict__ bcount, const uint32_t* __restrict__ bnodes,
                                    KadLine* __restrict__ lines, uint64_t sib_base)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const KadNode r = nodes[v];
    const uint32_t* L = sib + (uint64_t)v * S5;
    for (int q = 0; q < sln * KLINE; ++q) put_entry(lines, sib_base + (uint64_t)v * sln, q, q < S5 ? L[q] : NONE, recs);
    const int rowlo = kad_rowlo(r.meta);
    if (rowlo < 0) return;
    for (int m = KEYBITS - 1; m >= rowlo; --m) {
        const uint64_t line0 = (uint64_t)r.boff + (uint64_t)(KEYBITS - 1 - m) * lps;
        const int c = bcount[(uint64_t)v * KEYBITS + m];
        const uint32_t* B = bnodes + ((uint64_t)v * KEYBITS + m) * k;
        for (int q = 0; q < lps * KLINE; ++q) put_entry(lines, line0, q, q < c ? B[q] : NONE, recs);
    }
}

__global__ void k_kad_export(const KadNode* __restrict__ nodes, const KadLine* __restrict__ lines, uint32_t n, int k,
                             int lps, uint8_t* __restrict__ bcount, uint32_t* __restrict__ bnodes)
{
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)n * KEYBITS) return;
    const uint32_t v = (uint32_t)(t / KEYBITS);
    const int m = (int)(t % KEYBITS);
    const KadNode r = nodes[v];
    const int rowlo = kad_rowlo(r.meta);
    int c = 0;
    uint32_t* o = bnodes + t * k;
    for (int q = 0; q < k; ++q) o[q] = NONE;
    if (rowlo >= 0 && m >= rowlo) {
        const KadLine* l = lines + (uint64_t)r.boff + (uint64_t)(KEYBITS - 1 - m) * lps;
        for (int q = 0; q < k; ++q) {
            const uint32_t x = l[q / KLINE].idx[q % KLINE];
            if (x == NONE) break;
            o[c++] = x;
        }
    }
    bcount[t] = (uint8_t)c;
}

// ---------------------------------------------------------------------------
// K2: the lookup as a per-lane state machine

// what the pending line is
enum : uint32_t { KP_NONE = 0, KP_SRC = 1, KP_SEND = 2, KP_FN = 3 };
// findNode scan stage (Kademlia.cc:1166-1232)
enum : int { FS_MAIN = 0, FS_LOWER = 1, FS_SIB = 2, FS_ABOVE = 3 };

// orders one wave's LDS stores before its loads of other lanes' slots (and the loads before the
// next iteration's stores) for the compiler; a wave's LDS instructions execute in issue order
__device__ __forceinline__ void kad_wave_fence()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint64_t u64w(uint32_t lo, uint32_t hi) { return (uint64_t)lo | ((uint64_t)hi << 32); }

template <int A, bool RECORD, bool EX, bool LK>
__global__ __launch_bounds__(256) void k_kad_lanes(KadView V, DelayConsts DC, KadLC LC,
                                                   const K160* __restrict__ qkeys, const uint32_t* __restrict__ qsrc,
                                                   uint64_t nq, uint64_t chunk, ovs_route_out* __restrict__ out,
                                                   uint32_t* __restrict__ hopseq, uint32_t* __restrict__ rpcs_out,
                                                   uint32_t* __restrict__ sib_out)
{
    const int lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    uint64_t cursor = wave * chunk;                       // wave-uniform
    const uint64_t end = min(cursor + chunk, nq);
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int ns = LK ? LC.numSiblings : 1;
    const int64_t bwc = bw_ns(DC.callBytes, DC.datarate, DC.round);

    bool active = false;
    uint64_t q = 0;
    // ---- the lookup (IterativeLookup + its IterativePathLookup)
    K160 K;
    uint32_t S = 0;
    double sx = 0, sy = 0;
    int64_t now = 0, txf = 0, rcd = 0;
    uint32_t seq = 0;
    uint32_t nx[8];
    uint64_t nd[8];
    uint32_t nused = 0, nnew = 0;          // LookupVector flags: alreadyUsed; entered from the response
    int nn = 0;
    uint32_t pn[A], ptag[A], pdins[A], pgeo[A], pboff[A], pnsib[A];
    int64_t pt[A];
    uint64_t pdt[A];
    uint32_t pvalid = 0, pfin = 0;         // pending FindNodeCalls; those whose target line is consumed
    int step = 0, hops = 0, pending = 0;
    bool pfinished = false, psuccess = false, any_to = false;
    uint32_t result = NONE, nsent = 0;
    // ---- the findNode being evaluated (at the source: local; at a responder: its response)
    uint32_t fr = 0;
    RespGeo fg{};
    uint64_t fdt = 0;
    int fstage = 0, fb = 0, fj = 0, fseen = 0, frs = 0;
    bool fsb = false, flocal = false, fdone = false;
    SVec<8> res;                           // LK: the responding sibling's answer (the siblings vector)
    uint32_t fbx = NONE;                   // one-way: the responding sibling's answer (resultSize 1)
    uint64_t fbd = ~0ull;
    // ---- the gather
    uint32_t ph = KP_NONE;
    const uint4* lp = nullptr;
    uint4 L0 = make_uint4(0, 0, 0, 0), L1 = L0, L2 = L0, L3 = L0;

    __shared__ uint4 xbuf[4][256];
    uint4* const xb = xbuf[threadIdx.x >> 6];

#pragma unroll
    for (int i = 0; i < 8; ++i) { nx[i] = NONE; nd[i] = ~0ull; }
#pragma unroll
    for (int i = 0; i < A; ++i) { pn[i] = 0; ptag[i] = 0; pdins[i] = 0; pgeo[i] = 0; pboff[i] = 0; pnsib[i] = 0; pt[i] = 0; pdt[i] = 0; }
    if (LK) svec_clear(res);

    // LookupVector::add (BaseKeySortedVector::add, NodeVector.h:432-512) of one candidate with its
    // "from this response" flag; dedupe by node, cap = lookupRedundantNodes
    auto nh_insert = [&](uint32_t x, uint64_t d) {
        bool dup = false;
        int pos = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (i < nn) {
                dup |= nx[i] == x;
                pos += (nx[i] != x && cand_lt<EX>(nd[i], nx[i], d, x, K, V.nodes)) ? 1 : 0;
            }
        }
        if (dup || pos >= LC.redundant) return;
        const uint32_t low = (1u << pos) - 1u, capm = (1u << LC.redundant) - 1u;
        nused = ((nused & low) | ((nused & ~low) << 1)) & capm;
        nnew = ((nnew & low) | ((nnew & ~low) << 1) | (1u << pos)) & capm;
#pragma unroll
        for (int i = 7; i >= 0; --i) {
            if (i > pos) { nx[i] = nx[i - 1]; nd[i] = nd[i - 1]; }
            else if (i == pos) { nx[i] = x; nd[i] = d; }
        }
        nn = nn + 1 > LC.redundant ? LC.redundant : nn + 1;
    };
    // the findNode result of a sibling (LookupCall siblings vector), cap = resultSize
    auto res_insert = [&](uint32_t x, uint64_t d) {
        if (LK) {
            int pos = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i)
                if (i < res.n) pos += cand_lt<EX>(res.d[i], res.idx[i], d, x, K, V.nodes) ? 1 : 0;
            if (pos >= frs || pos >= 8) return;
#pragma unroll
            for (int i = 7; i >= 0; --i) {
                if (i > pos) { res.idx[i] = res.idx[i - 1]; res.d[i] = res.d[i - 1]; }
                else if (i == pos) { res.idx[i] = x; res.d[i] = d; }
            }
            res.n = res.n + 1 > frs ? frs : res.n + 1;
        }
    };
    // one candidate of the findNode scan: into nextHops, or (a sibling's answer, which ends the
    // lookup) into the result
    auto fn_cand = [&](uint32_t x, uint64_t d) {
        ++fseen;
        if (!fsb) nh_insert(x, d);
        else if (LK) res_insert(x, d);
        else if (fbx == NONE || cand_lt<EX>(d, x, fbd, fbx, K, V.nodes)) { fbx = x; fbd = d; }
    };
    auto has_slot = [&](int b) { return fg.rowlo >= 0 && b >= fg.rowlo; };
    auto req_slot = [&](int bucket, int j) {
        lp = reinterpret_cast<const uint4*>(V.lines + (uint64_t)fg.boff + (uint64_t)(KEYBITS - 1 - bucket) * V.lps + j);
        ph = KP_FN;
    };
    // the scan's next line after bucket fb's slot is done (fn stage machine); fdone when complete
    auto fn_next = [&]() {
        for (int guard = 0; guard < 2 * KEYBITS + 4; ++guard) {
            if (fstage == FS_MAIN) {
                // Kademlia.cc:1180 -- lower buckets, siblings and self when m >= endIndex or short
                if (fg.m >= fg.endIndex || fseen < frs) { fstage = FS_LOWER; fb = fg.m - 1; }
                else { fstage = FS_ABOVE; fb = fg.m + 1; }
                continue;
            }
            if (fstage == FS_LOWER) {
                if (fb >= fg.endIndex && has_slot(fb)) { fj = 0; req_slot(fb, 0); return; }
                if (fb >= fg.endIndex) { --fb; continue; }
                fstage = FS_SIB; fj = 0;
                if (fg.nsib > 0) {
                    lp = reinterpret_cast<const uint4*>(V.sibl + (uint64_t)(fr - V.lo) * V.sln);
                    ph = KP_FN;
                    return;
                }
                continue;
            }
            if (fstage == FS_SIB) {
                fn_cand(fr, fdt);                       // the local node (Kademlia.cc:1204)
                fstage = FS_ABOVE; fb = fg.m + 1;
                continue;
            }
            // FS_ABOVE: more distant buckets while the result is short (Kademlia.cc:1218-1232)
            if (fseen < frs && fb < KEYBITS) {
                if (has_slot(fb)) { fj = 0; req_slot(fb, 0); return; }
                ++fb;
                continue;
            }
            fdone = true;
            return;
        }
        fdone = true;
    };
    // findNode at fr begins (its line fields were captured in the pending call, or read for S)
    auto fn_start = [&]() {
        fseen = 0; fdone = false;
        fbx = NONE; fbd = ~0ull;
        if (LK) { svec_clear(res); }
        if (fg.nsib == 0 || (V.snapshot && fsb && ns <= 1)) {
            // empty sibling table: [self]; on snapshot tables a sibling with numSiblings = 1 answers
            // [self]
            fn_cand(fr, fdt);
            fdone = true;
            return;
        }
        if (fg.m >= 0 && has_slot(fg.m)) { fstage = FS_MAIN; fb = fg.m; fj = 0; req_slot(fb, 0); return; }
        fstage = FS_MAIN;
        fn_next();
    };
    // IterativePathLookup::sendRpc (IterativeLookup.cc:1067-1170): the calls are reserved here
    // (tx queue, sequence numbers), completed when their target's line arrives (KP_SEND)
    auto send_rpcs = [&](int num) {
        if (pfinished) return;
        if (LC.hopCountMax && hops >= LC.hopCountMax) { pfinished = true; psuccess = false; return; }
        if (LC.strict) num = min(num, LC.alpha - pending);
        if (num == 0 && pending == 0 && !LC.finishOnFirst) num = LC.alpha;
        for (int i = 0; num > 0 && i < LC.redundant; ++i) {
            const uint32_t unused = ~nused & ((1u << nn) - 1u);
            if (!unused) break;
            const int e = __ffs((int)unused) - 1;
            uint32_t h = NONE;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (j == e) h = nx[j];
            // visitOnlyOnce: an unused entry can only be a visited node if it is the source
            if (!LC.visitOnlyOnce || h != S) {
                ++pending;
                --num;
                int slot = 0;
#pragma unroll
                for (int s = A - 1; s >= 0; --s)
                    if (!((pvalid >> s) & 1u)) slot = s;
                const int64_t newTx = (txf > now ? txf : now) + bwc;
                txf = newTx;
#pragma unroll
                for (int s = 0; s < A; ++s) {
                    if (s == slot) { pn[s] = h; pt[s] = newTx; ptag[s] = (uint32_t)step | (seq << 16); }
                }
                seq += 2;
                ++nsent;
                pvalid |= 1u << slot;
                pfin &= ~(1u << slot);
            }
            nused |= 1u << e;
        }
        if (pending == 0) { psuccess = false; pfinished = true; }
    };
    auto timeoutlike = [&]() {
        // IterativePathLookup::handleTimeout (IterativeLookup.cc:935-1023), failedNodeRpcs = false
        --pending;
        if (now > DC.lookupTimeout) { pfinished = true; psuccess = false; }
        else if (LC.newOnTimeout) send_rpcs(1);
        else if (pending == 0) send_rpcs(LC.alpha);
    };

    while (true) {
        // ---- gathered lines to their lanes (chunk (lane & 3) of the line of lane 16k + (lane >> 2))
        xb[lane] = L0; xb[64 + lane] = L1; xb[128 + lane] = L2; xb[192 + lane] = L3;
        kad_wave_fence();
        L0 = xb[4 * lane]; L1 = xb[4 * lane + 1]; L2 = xb[4 * lane + 2]; L3 = xb[4 * lane + 3];
        kad_wave_fence();

        // ---- refill: lanes without a lookup take the next of the wave's slice
        bool fresh = false;
        const uint64_t need = __ballot(!active);
        if (need != 0 && cursor < end) {
            const uint64_t mine = cursor + (uint64_t)__popcll(need & lt_mask);
            if (!active && mine < end) {
                q = mine;
                active = true;
                fresh = true;
                K = qkeys[q];
                S = qsrc[q];
                now = 0; txf = 0; rcd = 0; seq = 0;
#pragma unroll
                for (int i = 0; i < 8; ++i) { nx[i] = NONE; nd[i] = ~0ull; }
                nused = 0; nnew = 0; nn = 0;
                pvalid = 0; pfin = 0;
                step = 0; hops = 0; pending = 0;
                pfinished = false; psuccess = false; any_to = false;
                result = NONE; nsent = 0;
                lp = reinterpret_cast<const uint4*>(V.nodes + S);
                ph = KP_SRC;
            }
            cursor += (uint64_t)__popcll(need);
        }
        if (!__any(active)) break;

        if (active && !fresh) {
            const uint32_t cph = ph;
            lp = nullptr;
            ph = KP_NONE;
            // ---- consume the pending line
            if (cph == KP_SRC || cph == KP_SEND) {
                const KadNode r = node_from_line(L0, L1, L2, L3);
                if (cph == KP_SRC) {
                    // IterativeLookup::start (IterativeLookup.cc:133-244): findNode at the source
                    sx = r.x; sy = r.y;
                    fr = S;
                    fsb = kad_is_sibling(V, r, S, K, ns);
                    fg = resp_geo(r, K);
                    fdt = dist_hi(as_key(r.key), K);
                    frs = fsb ? ns : LC.maxRedundantLocal;
                    flocal = true;
                    fn_start();
                } else {
                    // complete the lowest reserved call: its target is known, its timing now
                    const uint32_t open = pvalid & ~pfin;
                    const int e = __ffs((int)open) - 1;
                    uint32_t x = 0;
                    int64_t newTx = 0;
                    uint32_t tg = 0;
#pragma unroll
                    for (int s = 0; s < A; ++s)
                        if (s == e) { x = pn[s]; newTx = pt[s]; tg = ptag[s]; }
                    const bool xsb = kad_is_sibling(V, r, x, K, ns);
                    const RespGeo rg = resp_geo(r, K);
                    const int csz = kad_response_size<EX>(V, x, rg, K, xsb ? ns : LC.redundant, xsb, ns);
                    const int64_t cd = coord_ns(sx, sy, r.x, r.y, DC.round);
                    const int64_t d1 = (newTx - now) + DC.access2 + cd + bwc;
                    const int64_t bwr = bw_ns(DC.respBase + DC.respPerNode * csz, DC.datarate, DC.round);
                    const int64_t d2 = 2 * bwr + DC.access2 + cd;
                    const int64_t tTo = now + DC.rpcTimeout;
                    const int64_t tResp = now + d1 + d2;
                    const bool isTo = tTo <= tResp;   // the timeout was scheduled first: it wins ties
                    const uint32_t sTo = tg >> 16;
                    const uint32_t tag = (tg & 0xFFFFu) | ((isTo ? sTo : sTo + 1) << 16) | (isTo ? 0x80000000u : 0u);
#pragma unroll
                    for (int s = 0; s < A; ++s) {
                        if (s == e) {
                            pt[s] = isTo ? tTo : tResp;
                            pdins[s] = (uint32_t)(isTo ? DC.rpcTimeout : d2);
                            ptag[s] = tag;
                            pgeo[s] = pack_geo(rg, xsb) | ((uint32_t)csz << 25);
                            pboff[s] = rg.boff;
                            pnsib[s] = (uint32_t)rg.nsib;
                            pdt[s] = dist_hi(as_key(r.key), K);
                        }
                    }
                    pfin |= 1u << e;
                }
            } else if (cph == KP_FN) {
                // a line of the findNode scan: up to 5 candidates
                const uint64_t kt = ktop(K);
                const uint64_t tops[5] = {u64w(L0.x, L0.y), u64w(L0.z, L0.w), u64w(L1.x, L1.y), u64w(L1.z, L1.w),
                                          u64w(L2.x, L2.y)};
                const uint32_t ids[5] = {L2.z, L2.w, L3.x, L3.y, L3.z};
                int cnt = 0;
#pragma unroll
                for (int i = 0; i < 5; ++i) {
                    if (ids[i] != NONE) { fn_cand(ids[i], dclamp(tops[i] ^ kt)); ++cnt; }
                }
                if (fstage == FS_SIB) {
                    ++fj;
                    if (fj * KLINE < fg.nsib) {
                        lp = reinterpret_cast<const uint4*>(V.sibl + (uint64_t)(fr - V.lo) * V.sln + fj);
                        ph = KP_FN;
                    } else {
                        fn_next();
                    }
                } else {
                    ++fj;
                    if (cnt == KLINE && fj < V.lps) {
                        req_slot(fb, fj);
                    } else {
                        // slot fb done
                        if (fstage == FS_LOWER) --fb;
                        else if (fstage == FS_ABOVE) ++fb;
                        fn_next();
                    }
                }
            }

            // ---- advance without memory until a line is needed or the lookup ends
            for (int guard = 0; guard < 4 * A + 8 && !lp; ++guard) {
                if (fdone) {
                    fdone = false;
                    if (flocal) {
                        flocal = false;
                        if (fseen == 0) { pfinished = true; psuccess = false; }
                        else if (LC.numSiblings != 0 && fsb) {
                            result = LK ? res.idx[0] : fbx;
                            pfinished = true; psuccess = true;
                        } else {
                            nnew = 0;
                            send_rpcs(LC.alpha);
                        }
                    } else {
                        int numNew = __popc(nnew);
                        nnew = 0;
                        if (LC.numSiblings != 0 && fsb) {
                            if (result == NONE) {
                                result = LK ? res.idx[0] : fbx;
                                // explicit tables: the answer's first node need not be the responder
                                if (result != fr) {
                                    const double2 rxy = V.xy[result];
                                    rcd = coord_ns(sx, sy, rxy.x, rxy.y, DC.round);
                                }
                            }
                            pfinished = true; psuccess = true;
                        } else {
                            if (numNew == 0 && LC.newOnResp) numNew = 1;
                            send_rpcs(min(numNew, LC.alpha));
                        }
                    }
                    continue;
                }
                const uint32_t open = pvalid & ~pfin;
                if (open && !pfinished) {
                    const int e = __ffs((int)open) - 1;
                    uint32_t x = 0;
#pragma unroll
                    for (int s = 0; s < A; ++s)
                        if (s == e) x = pn[s];
                    lp = reinterpret_cast<const uint4*>(V.nodes + x);
                    ph = KP_SEND;
                    break;
                }
                if (pfinished || pvalid == 0) {
                    // checkStop -> stop -> SendToKeyListener::lookupFinished (BaseOverlay.cc:1241-1307)
                    ovs_route_out o;
                    o.hops = (uint16_t)hops;
                    if (pfinished && psuccess && result != NONE) {
                        o.status = OVS_LOOKUP_OK;
                        o.responsible = result;
                        o.one_way_hops = (uint8_t)(hops + (result != S ? 1 : 0));
                        int64_t lat = now;
                        if (result != S && !DC.lookupCall) {
                            // sendRouteMessage through the source's tx queue (SimpleNodeEntry.cc:164-194);
                            // the coordinate delay S -> result is the one of its FindNodeCall
                            const int64_t bwr = bw_ns(DC.routeBytes, DC.datarate, DC.round);
                            const int64_t newTx = (txf > now ? txf : now) + bwr;
                            lat = newTx + DC.access2 + rcd + bwr;
                        }
                        o.latency_ns = lat;
                    } else {
                        o.responsible = NONE;
                        o.one_way_hops = 0;
                        o.latency_ns = -1;
                        if (now > DC.lookupTimeout) o.status = OVS_LOOKUP_TIMEOUT;
                        else if (any_to) o.status = OVS_LOOKUP_RPC_TIMEOUT;
                        else if (LC.hopCountMax && hops >= LC.hopCountMax) o.status = OVS_LOOKUP_HOPMAX;
                        else o.status = OVS_LOOKUP_NO_NEXT;
                    }
                    out[q] = o;
                    if (rpcs_out) rpcs_out[q] = nsent;
                    if (LK) {
                        const bool ok = o.status == OVS_LOOKUP_OK;
                        uint32_t* row = sib_out + q * (uint64_t)LC.numSiblings;
#pragma unroll
                        for (int j = 0; j < 8; ++j)
                            if (j < LC.numSiblings) row[j] = (ok && j < res.n) ? res.idx[j] : NONE;
                    }
                    active = false;
                    break;
                }
                // ---- the earliest pending event: (time, insertion time, insertion sequence)
                int e = -1;
                int64_t bt = 0, bi = 0;
                uint32_t bs = 0;
#pragma unroll
                for (int i = 0; i < A; ++i) {
                    if ((pvalid >> i) & 1u) {
                        const int64_t ti = pt[i] - (int64_t)pdins[i];
                        const uint32_t si = (ptag[i] >> 16) & 0x7FFFu;
                        const bool better = e < 0 || pt[i] < bt || (pt[i] == bt && (ti < bi || (ti == bi && si < bs)));
                        if (better) { e = i; bt = pt[i]; bi = ti; bs = si; }
                    }
                }
                uint32_t r = 0, tag = 0, geo = 0, boff = 0, nsib = 0, dins = 0;
                uint64_t dt = 0;
#pragma unroll
                for (int i = 0; i < A; ++i)
                    if (i == e) { r = pn[i]; tag = ptag[i]; geo = pgeo[i]; boff = pboff[i]; nsib = pnsib[i]; dt = pdt[i]; dins = pdins[i]; }
                pvalid &= ~(1u << e);
                now = bt;
                if (tag & 0x80000000u) {
                    // BaseRpc timeout -> IterativeLookup::handleRpcTimeout (IterativeLookup.cc:588-654)
                    any_to = true;
                    timeoutlike();
                    continue;
                }
                const bool sb = (geo >> 24) & 1u;
                const bool acc = (LC.useAll && LC.merge) ? true : ((int)(tag & 0xFFFFu) == step);
                if (!(acc || (sb && LC.acceptLateSiblings))) {
                    // not accepted: handled as a timeout, its nodes are dropped (IterativeLookup.cc:534-548)
                    timeoutlike();
                    continue;
                }
                // IterativePathLookup::handleResponse (IterativeLookup.cc:803-921)
                if (now > DC.lookupTimeout) { pfinished = true; psuccess = false; continue; }
                if (r != S) {
                    if (RECORD && hops < LC.hopCountMax) hopseq[q * (uint64_t)LC.hopCountMax + hops] = r;
                    ++hops;
                }
                ++step;
                --pending;
                fr = r;
                fsb = sb;
                fg = unpack_geo(geo & 0x1FFFFFFu, boff, nsib);
                fdt = dt;
                frs = sb ? ns : LC.redundant;
                flocal = false;
                if (sb) {
                    // the response ends the lookup: the route message's coordinate delay S -> r
                    const int csz = (int)(geo >> 25);
                    rcd = (int64_t)dins - 2 * bw_ns(DC.respBase + DC.respPerNode * csz, DC.datarate, DC.round) - DC.access2;
                }
                nnew = 0;
                fn_start();
            }
        }

        // ---- request the next line: 4 lanes fetch one 64 B line with one 16 B load each
        {
            const uint64_t mine = (active && lp) ? reinterpret_cast<uint64_t>(lp) : 0ull;
            const uint32_t mlo = (uint32_t)mine, mhi = (uint32_t)(mine >> 32);
            const int ch = lane & 3;
            uint4 v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int owner = 16 * k + (lane >> 2);
                const uint64_t a = (uint64_t)__shfl(mlo, owner) | ((uint64_t)__shfl(mhi, owner) << 32);
                if (a != 0) v[k] = reinterpret_cast<const uint4*>(a)[ch];
                else v[k] = make_uint4(0, 0, 0, 0);
            }
            L0 = v[0]; L1 = v[1]; L2 = v[2]; L3 = v[3];
        }
    }
}

// the synchronous form (one event per loop iteration, loads inside): the sharded path's state
// machine on one GPU, kept selectable (OVS_KAD_SYNC=1) as a cross-check of k_kad_lanes
struct SendNothing {
    __device__ __forceinline__ void operator()(int, uint32_t, bool) const {}
};

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
__global__ __launch_bounds__(256) void k_kad_route_sync(KadView V, DelayConsts DC, KadLC LC, const K160* __restrict__ qkeys,
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

// batched findNode (general numRedundantNodes <= 8, 1 <= numSiblings <= 8) for the ABI
template <bool EX>
__global__ void k_kad_find_node(KadView V, const uint32_t* __restrict__ node, const K160* __restrict__ keys, uint64_t n,
                                int numRedundant, int numSiblings, uint32_t* __restrict__ out_nodes, uint32_t max_out,
                                uint8_t* __restrict__ out_count, uint8_t* __restrict__ out_sib)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = node[i];
    const K160 K = keys[i];
    const KadNode r = load_node(V.nodes, c);
    const bool sb = kad_is_sibling(V, r, c, K, numSiblings);
    Blk8 b;
    const int cnt = kad_find_node_blk<EX>(V, c, resp_geo(r, K), K, numRedundant, sb, b, numSiblings);
    uint32_t* o = out_nodes + i * max_out;
    for (uint32_t j = 0; j < max_out; ++j) o[j] = NONE;
#pragma unroll
    for (int j = 0; j < 8; ++j)
        if (j < cnt && (uint32_t)j < max_out) o[j] = b.x[j];
    out_count[i] = (uint8_t)(cnt < (int)max_out ? cnt : (int)max_out);
    out_sib[i] = sb ? 1 : 0;
}

// ---------------------------------------------------------------------------
// host side

static inline unsigned nblk(uint64_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

static hipError_t kad_prefix_flag(const KeyRec* recs, uint32_t n, KadTables& t, hipStream_t st)
{
    uint32_t* tie = nullptr;
    uint32_t htie = 1;
    hipError_t e;
    if ((e = hipMalloc(&tie, sizeof(uint32_t))) != hipSuccess) return e;
    hipMemsetAsync(tie, 0, sizeof(uint32_t), st);
    if (n > 1) hipLaunchKernelGGL(k_kad_prefix_ties, dim3(nblk(n, 256)), dim3(256), 0, st, recs, n, tie);
    hipMemcpyAsync(&htie, tie, sizeof(uint32_t), hipMemcpyDeviceToHost, st);
    e = hipStreamSynchronize(st);
    hipFree(tie);
    if (e != hipSuccess) return e;
    t.exact = htie != 0 || getenv("OVS_KAD_EXACT") != nullptr;
    return hipSuccess;
}

hipError_t kad_build(const KeyRec* recs, const double2* xy, uint32_t n, int k, int s, uint64_t seed, KadTables& t,
                     hipStream_t st, uint32_t lo, uint32_t hi)
{
    hipError_t e;
    kad_free(t);
    if (hi > n) hi = n;
    if (lo >= hi) return hipErrorInvalidValue;
    t.k = k; t.s = s; t.seed = seed; t.lo = lo; t.hi = hi; t.snapshot = 1; t.maybe_short = 0;
    const int S5 = 5 * s, lps = (k + KLINE - 1) / KLINE, sln = (S5 + KLINE - 1) / KLINE;
    const uint32_t nown = hi - lo;
    uint64_t *rowlen = nullptr, *off = nullptr;
    uint32_t* sib_all = nullptr;
    void* tmp = nullptr;
    size_t tmpb = 0;
    auto cleanup = [&]() {
        if (rowlen) hipFree(rowlen);
        if (off) hipFree(off);
        if (tmp) hipFree(tmp);
        if (sib_all) hipFree(sib_all);
    };
    // node lines for the whole network (a lookup needs every target's summary when it sends the
    // call); sibling lists are a build temporary
    if ((e = hipMalloc(&t.nodes, sizeof(KadNode) * n)) != hipSuccess) return e;
    if ((e = hipMalloc(&t.nodex, sizeof(KadX) * n)) != hipSuccess) return e;
    if ((e = hipMalloc(&sib_all, sizeof(uint32_t) * (uint64_t)n * S5)) != hipSuccess) return e;
    if ((e = hipMalloc(&rowlen, sizeof(uint64_t) * (n + 1))) != hipSuccess) { cleanup(); return e; }
    if ((e = hipMalloc(&off, sizeof(uint64_t) * (n + 1))) != hipSuccess) { cleanup(); return e; }
    hipLaunchKernelGGL(k_kad_siblings, dim3(nblk(n, 128)), dim3(128), 0, st, recs, xy, n, S5, lps, lo, hi, sib_all,
                       t.nodes, t.nodex, rowlen);
    hipMemsetAsync(rowlen + n, 0, sizeof(uint64_t), st);
    hipcub::DeviceScan::ExclusiveSum(nullptr, tmpb, rowlen, off, n + 1, st);
    if ((e = hipMalloc(&tmp, tmpb)) != hipSuccess) { cleanup(); return e; }
    hipcub::DeviceScan::ExclusiveSum(tmp, tmpb, rowlen, off, n + 1, st);
    uint64_t total = 0;
    hipMemcpyAsync(&total, off + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st);
    if ((e = hipStreamSynchronize(st)) != hipSuccess) { cleanup(); return e; }
    if (total >= 0xFFFFFFFFull) { cleanup(); return hipErrorInvalidValue; }
    t.rows_lines = total;
    const uint64_t nlines = total + (uint64_t)nown * sln + 1;
    if ((e = hipMalloc(&t.lines, sizeof(KadLine) * nlines)) != hipSuccess) { cleanup(); return e; }
    hipLaunchKernelGGL(k_kad_set_boff, dim3(nblk(nown, 256)), dim3(256), 0, st, t.nodes, off, lo, hi);
    if ((e = hipMalloc(&t.sib, sizeof(uint32_t) * (uint64_t)nown * S5)) != hipSuccess) { cleanup(); return e; }
    hipMemcpyAsync(t.sib, sib_all + (uint64_t)lo * S5, sizeof(uint32_t) * (uint64_t)nown * S5, hipMemcpyDeviceToDevice, st);
    hipLaunchKernelGGL(k_kad_buckets, dim3(nblk(nown, 64)), dim3(64), 0, st, recs, t.nodes, n, k, lps, S5, sln, seed,
                       sib_all, t.lines, t.rows_lines, lo, hi);
    e = hipStreamSynchronize(st);
    cleanup();
    if (e != hipSuccess) return e;
    if ((e = kad_prefix_flag(recs, n, t, st)) != hipSuccess) return e;
    return hipGetLastError();
}

hipError_t kad_build_explicit(const KeyRec* recs, const double2* xy, uint32_t n, int k, int s, const uint32_t* sib,
                              const uint8_t* bcount, const uint32_t* bnodes, KadTables& t, uint32_t* bad_node,
                              uint32_t* bad_code, hipStream_t st)
{
    hipError_t e;
    kad_free(t);
    t.k = k; t.s = s; t.seed = 0; t.lo = 0; t.hi = n; t.snapshot = 0;
    const int S5 = 5 * s, lps = (k + KLINE - 1) / KLINE, sln = (S5 + KLINE - 1) / KLINE;
    uint64_t *rowlen = nullptr, *off = nullptr;
    uint32_t* flags = nullptr;
    void* tmp = nullptr;
    size_t tmpb = 0;
    auto cleanup = [&]() {
        if (rowlen) hipFree(rowlen);
        if (off) hipFree(off);
        if (tmp) hipFree(tmp);
        if (flags) hipFree(flags);
    };
    if ((e = hipMalloc(&t.nodes, sizeof(KadNode) * n)) != hipSuccess) return e;
    if ((e = hipMalloc(&t.nodex, sizeof(KadX) * n)) != hipSuccess) return e;
    if ((e = hipMalloc(&t.sib, sizeof(uint32_t) * (uint64_t)n * S5)) != hipSuccess) return e;
    hipMemcpyAsync(t.sib, sib, sizeof(uint32_t) * (uint64_t)n * S5, hipMemcpyDeviceToDevice, st);
    if ((e = hipMalloc(&rowlen, sizeof(uint64_t) * (n + 1))) != hipSuccess) { cleanup(); return e; }
    if ((e = hipMalloc(&off, sizeof(uint64_t) * (n + 1))) != hipSuccess) { cleanup(); return e; }
    if ((e = hipMalloc(&flags, sizeof(uint32_t) * 3)) != hipSuccess) { cleanup(); return e; }
    const uint32_t init[3] = {NONE, 0u, 0u};
    hipMemcpyAsync(flags, init, sizeof init, hipMemcpyHostToDevice, st);
    hipLaunchKernelGGL(k_kad_explicit_nodes, dim3(nblk(n, 128)), dim3(128), 0, st, recs, xy, n, k, S5, lps, t.sib,
                       bcount, bnodes, t.nodes, t.nodex, rowlen, flags, flags + 2);
    uint32_t hf[3] = {0, 0, 0};
    hipMemcpyAsync(hf, flags, sizeof hf, hipMemcpyDeviceToHost, st);
    if ((e = hipStreamSynchronize(st)) != hipSuccess) { cleanup(); return e; }
    if (hf[0] != NONE) {
        *bad_node = hf[0];
        *bad_code = hf[1];
        cleanup();
        return hipErrorInvalidValue;
    }
    t.maybe_short = hf[2] != 0;
    hipMemsetAsync(rowlen + n, 0, sizeof(uint64_t), st);
    hipcub::DeviceScan::ExclusiveSum(nullptr, tmpb, rowlen, off, n + 1, st);
    if ((e = hipMalloc(&tmp, tmpb)) != hipSuccess) { cleanup(); return e; }
    hipcub::DeviceScan::ExclusiveSum(tmp, tmpb, rowlen, off, n + 1, st);
    uint64_t total = 0;
    hipMemcpyAsync(&total, off + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st);
    if ((e = hipStreamSynchronize(st)) != hipSuccess) { cleanup(); return e; }
    if (total >= 0xFFFFFFFFull) { cleanup(); return hipErrorInvalidValue; }
    t.rows_lines = total;
    if ((e = hipMalloc(&t.lines, sizeof(KadLine) * (total + (uint64_t)n * sln + 1))) != hipSuccess) { cleanup(); return e; }
    hipLaunchKernelGGL(k_kad_set_boff, dim3(nblk(n, 256)), dim3(256), 0, st, t.nodes, off, 0u, n);
    hipLaunchKernelGGL(k_kad_explicit_rows, dim3(nblk(n, 64)), dim3(64), 0, st, recs, t.nodes, n, k, lps, S5, sln,
                       t.sib, bcount, bnodes, t.lines, t.rows_lines);
    e = hipStreamSynchronize(st);
    cleanup();
    if (e != hipSuccess) return e;
    if ((e = kad_prefix_flag(recs, n, t, st)) != hipSuccess) return e;
    return hipGetLastError();
}

hipError_t kad_export(const KadTables& t, uint32_t n, uint32_t* siblings, uint8_t* bucket_count, uint32_t* bucket_nodes,
                      hipStream_t st)
{
    hipError_t e;
    const int S5 = 5 * t.s, lps = (t.k + KLINE - 1) / KLINE;
    uint8_t* dc = nullptr;
    uint32_t* dn = nullptr;
    const uint64_t tot = (uint64_t)n * KEYBITS;
    if ((e = hipMalloc(&dc, tot)) != hipSuccess) return e;
    if ((e = hipMalloc(&dn, sizeof(uint32_t) * tot * t.k)) != hipSuccess) { hipFree(dc); return e; }
    hipLaunchKernelGGL(k_kad_export, dim3(nblk(tot, 256)), dim3(256), 0, st, t.nodes, t.lines, n, t.k, lps, dc, dn);
    hipMemcpyAsync(bucket_count, dc, tot, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(bucket_nodes, dn, sizeof(uint32_t) * tot * t.k, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(siblings, t.sib, sizeof(uint32_t) * (uint64_t)n * S5, hipMemcpyDeviceToHost, st);
    e = hipStreamSynchronize(st);
    hipFree(dc); hipFree(dn);
    return e;
}

template <class Kern>
static uint64_t kad_chunk(Kern kern, int* cache, uint64_t nq, int num_cu, uint64_t* blocks)
{
    if (*cache == 0) {
        int b = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kern, 256, 0) != hipSuccess || b < 1) b = 1;
        *cache = b;
    }
    const uint64_t waves = (uint64_t)num_cu * (uint64_t)(*cache) * 4;
    uint64_t chunk = (nq + waves - 1) / waves;
    if (chunk < 1) chunk = 1;
    const uint64_t need_waves = (nq + chunk - 1) / chunk;
    *blocks = (need_waves + 3) / 4;
    return chunk;
}

template <int A, bool RECORD, bool EX, bool LK>
static hipError_t kad_launch(const KadView& V, const DelayConsts& DC, const KadLC& LC, const K160* qkeys,
                             const uint32_t* qsrc, uint64_t nq, ovs_route_out* out, uint32_t* hopseq, uint32_t* rpcs,
                             uint32_t* sibs, int num_cu, hipStream_t st, bool sync)
{
    uint64_t blocks = 0;
    if (sync) {
        static int bpc = 0;
        const uint64_t chunk = kad_chunk(k_kad_route_sync<A, RECORD, EX, LK>, &bpc, nq, num_cu, &blocks);
        hipLaunchKernelGGL((k_kad_route_sync<A, RECORD, EX, LK>), dim3((unsigned)blocks), dim3(256), 0, st, V, DC, LC,
                           qkeys, qsrc, nq, chunk, out, hopseq, rpcs, sibs);
    } else {
        static int bpc = 0;
        const uint64_t chunk = kad_chunk(k_kad_lanes<A, RECORD, EX, LK>, &bpc, nq, num_cu, &blocks);
        hipLaunchKernelGGL((k_kad_lanes<A, RECORD, EX, LK>), dim3((unsigned)blocks), dim3(256), 0, st, V, DC, LC,
                           qkeys, qsrc, nq, chunk, out, hopseq, rpcs, sibs);
    }
    return hipGetLastError();
}

hipError_t kad_route(const KadTables& t, const double2* xy, uint32_t n, const ovs_params& P, const DelayConsts& DC,
                     const K160* qkeys, const uint32_t* qsrc, uint64_t nq, ovs_route_out* out, uint32_t* hopseq,
                     uint32_t* rpcs, int num_cu, hipStream_t st, uint32_t* sibs)
{
    if (nq == 0) return hipSuccess;
    if (!kad_params_supported(P, t)) return hipErrorNotSupported;
    const KadLC LC = kad_make_lc(P, t);
    const KadView V = kad_make_view(t, xy, n);
    static const bool sync = getenv("OVS_KAD_SYNC") != nullptr;
    // strictParallelRpcs: never more than alpha FindNodeCalls in flight (IterativeLookup.cc:1078-1079)
    const int A = P.lookupParallelRpcs;
    // LookupCall batches (sibs != nullptr) record no hop sequence
    if (sibs && hopseq) return hipErrorNotSupported;
#define KLX(a, x) (sibs     ? kad_launch<a, false, x, true>(V, DC, LC, qkeys, qsrc, nq, out, hopseq, rpcs, sibs, num_cu, st, sync) \
                   : hopseq ? kad_launch<a, true, x, false>(V, DC, LC, qkeys, qsrc, nq, out, hopseq, rpcs, sibs, num_cu, st, sync) \
                            : kad_launch<a, false, x, false>(V, DC, LC, qkeys, qsrc, nq, out, hopseq, rpcs, sibs, num_cu, st, sync))
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

hipError_t kad_find_node(const KadTables& t, uint32_t n, const ovs_params& P, const uint32_t* node, const K160* keys,
                         uint64_t nq, int numRedundant, int numSiblings, uint32_t* out_nodes, uint32_t max_out,
                         uint8_t* out_count, uint8_t* out_sib, hipStream_t st)
{
    (void)P;
    if (nq == 0) return hipSuccess;
    if (numSiblings < 1 || numSiblings > 8 || numRedundant > 8) return hipErrorNotSupported;
    const KadView V = kad_make_view(t, nullptr, n);
    if (t.exact)
        hipLaunchKernelGGL(k_kad_find_node<true>, dim3(nblk(nq, 128)), dim3(128), 0, st, V, node, keys, nq, numRedundant,
                           numSiblings, out_nodes, max_out, out_count, out_sib);
    else
        hipLaunchKernelGGL(k_kad_find_node<false>, dim3(nblk(nq, 128)), dim3(128), 0, st, V, node, keys, nq, numRedundant,
                           numSiblings, out_nodes, max_out, out_count, out_sib);
    return hipGetLastError();
}

}  // namespace ovs
