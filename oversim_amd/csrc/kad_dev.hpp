// kad_dev.hpp -- Kademlia device building blocks shared by the single-GPU kernels (kad.hip)
// and the sharded request/response kernels (kad_shard.hip): node / line loads, sorted vectors,
// isSiblingFor / findNode from the tables (kad.hpp), and the IterativePathLookup state machine
// in its synchronous (one call = one event) form used by the sharded path.
#pragma once
#include "kad.hpp"

namespace ovs {

// ---------------------------------------------------------------------------
// helpers

// word i (0..4, 5+ reads 0) of a key by selects: a dynamic k.w[i] would put the key in scratch
__device__ __forceinline__ uint32_t kword(const K160& k, int i)
{
    uint32_t r = i == 0 ? k.w[0] : 0u;
    r = i == 1 ? k.w[1] : r;
    r = i == 2 ? k.w[2] : r;
    r = i == 3 ? k.w[3] : r;
    r = i == 4 ? k.w[4] : r;
    return r;
}

__device__ __forceinline__ uint32_t kbit(const K160& k, int b) { return (kword(k, b >> 5) >> (b & 31)) & 1u; }

__device__ __forceinline__ K160 kload(const KeyRec* __restrict__ recs, uint32_t i) { return key_of(load_rec(recs, i)); }

// Kademlia::routingBucketIndex (Kademlia.cc:357-382) of the XOR distance D for digit width b: the
// b-bit digits sit at bits i = 160 % b + j * b (the bits below 160 % b belong to none); the highest
// nonzero digit d, at i, gives bucket (i / b) * (2^b - 1) + d - 1 (firstOnLayer: + 2^b - 2, the
// layer's last); -1 when every digit is zero
__device__ __forceinline__ int kad_bucket_index(const K160& D, int b, bool first)
{
    const int m = k_msb(D);
    const int r = KEYBITS % b;
    if (m < r) return -1;
    const int i = r + ((m - r) / b) * b;
    const uint64_t win = (uint64_t)kword(D, i >> 5) | ((uint64_t)kword(D, (i >> 5) + 1) << 32);
    const int d = (int)((win >> (i & 31)) & ((1u << b) - 1u));
    return (i / b) * ((1 << b) - 1) + (first ? (1 << b) - 2 : d - 1);
}

__device__ __forceinline__ K160 node_key(const KadNode* __restrict__ nodes, uint32_t i)
{
    const uint4* p = reinterpret_cast<const uint4*>(nodes + i);
    const uint4 a = p[0], b = p[1];
    K160 k;
    k.w[0] = a.x; k.w[1] = a.y; k.w[2] = a.z; k.w[3] = a.w; k.w[4] = b.x;
    return k;
}

__device__ __forceinline__ KadNode load_node(const KadNode* __restrict__ nodes, uint32_t i)
{
    const uint4* p = reinterpret_cast<const uint4*>(nodes + i);
    const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
    KadNode o;
    o.key[0] = a.x; o.key[1] = a.y; o.key[2] = a.z; o.key[3] = a.w; o.key[4] = b.x;
    o.boff = b.y;
    o.x = __hiloint2double((int)b.w, (int)b.z);
    o.y = __hiloint2double((int)c.y, (int)c.x);
    o.rtop = (uint64_t)c.z | ((uint64_t)c.w << 32);
    o.mwin = (uint64_t)d.x | ((uint64_t)d.y << 32);
    o.meta = d.z;
    o.spare = d.w;
    return o;
}

// a KadNode from the four 16 B chunks of its line (the cooperative gather of kad.hip)
__device__ __forceinline__ KadNode node_from_line(uint4 a, uint4 b, uint4 c, uint4 d)
{
    KadNode o;
    o.key[0] = a.x; o.key[1] = a.y; o.key[2] = a.z; o.key[3] = a.w; o.key[4] = b.x;
    o.boff = b.y;
    o.x = __hiloint2double((int)b.w, (int)b.z);
    o.y = __hiloint2double((int)c.y, (int)c.x);
    o.rtop = (uint64_t)c.z | ((uint64_t)c.w << 32);
    o.mwin = (uint64_t)d.x | ((uint64_t)d.y << 32);
    o.meta = d.z;
    o.spare = d.w;
    return o;
}

__device__ __forceinline__ K160 as_key(const uint32_t* w)
{
    K160 k;
    k.w[0] = w[0]; k.w[1] = w[1]; k.w[2] = w[2]; k.w[3] = w[3]; k.w[4] = w[4];
    return k;
}

// first index in [lo,hi) whose bit b is set; all keys in [lo,hi) share the bits above b
__device__ uint32_t split_bit(const KeyRec* __restrict__ recs, uint32_t lo, uint32_t hi, int b)
{
    while (lo < hi) {
        const uint32_t mid = lo + ((hi - lo) >> 1);
        if (kbit(kload(recs, mid), b)) hi = mid; else lo = mid + 1;
    }
    return lo;
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
// h mod d for d < 2^32, exact (the same result as the 64-bit %): three steps of at most 48-bit
// dividends through an fp64 reciprocal, each quotient off by at most one and corrected -- the
// compiler's 64-bit unsigned remainder is ~130 instructions, this ~35 (the snapshot bucket
// builders draw 8 of them per bucket)
__host__ __device__ __forceinline__ uint32_t mod_step48(uint64_t x, uint32_t d, double rd)
{
    const uint64_t q = (uint64_t)((double)x * rd);
    int64_t r = (int64_t)(x - q * (uint64_t)d);
    if (r < 0) r += d;
    else if (r >= (int64_t)d) r -= d;
    return (uint32_t)r;
}
__host__ __device__ __forceinline__ uint32_t mod_u64_u32(uint64_t h, uint32_t d)
{
    const double rd = 1.0 / (double)d;
#ifndef OVS_MOD3
    // two steps: h >> 21 (< 2^43), then (r << 21) | low 21 bits (< d * 2^21 <= 2^53).  Both dividends
    // convert to double exactly and their quotients stay below 2^52, where x * rd (two roundings,
    // relative error <= 2^-52) is off the true quotient by less than one: the step's +-1 correction
    // suffices (checked against % by tests/test_mod.py's host build)
    const uint32_t r = mod_step48(h >> 21, d, rd);
    return mod_step48(((uint64_t)r << 21) | (h & 0x1FFFFFull), d, rd);
#else
    uint32_t r = mod_step48(h >> 32, d, rd);
    r = mod_step48(((uint64_t)r << 16) | ((h >> 16) & 0xFFFFull), d, rd);
    return mod_step48(((uint64_t)r << 16) | (h & 0xFFFFull), d, rd);
#endif
}

// identical to the oracle's kad_hash (bucket sampling of the snapshot rule)
__device__ __forceinline__ uint64_t kad_hash(uint64_t seed, uint32_t node, uint32_t m, uint32_t j)
{
    return splitmix64(seed ^ splitmix64(((uint64_t)node << 32) ^ ((uint64_t)m << 16) ^ (uint64_t)j));
}

// ---------------------------------------------------------------------------
// XOR distances: ordered by their top 64 bits, exact 160-bit fallback on ties

// top 64 bits of the XOR distance, clamped below the empty-entry sentinel ~0 (a real distance
// of ~0 becomes ~0 - 1: ordered before every empty entry, and with KadTables::exact == 0 still
// unique, as no two node IDs then share their top 63 bits)
__device__ __forceinline__ uint64_t dclamp(uint64_t d) { return d == ~0ull ? ~0ull - 1 : d; }

__device__ __forceinline__ uint64_t ktop(const K160& x) { return ((uint64_t)x.w[4] << 32) | (uint64_t)x.w[3]; }

__device__ __forceinline__ uint64_t dist_hi(const K160& x, const K160& K) { return dclamp(ktop(x) ^ ktop(K)); }

// XOR distances of distinct nodes to one key are distinct (XOR is a bijection); their top 64
// bits can tie only when the two node IDs share their top 64 bits.  EX = false is used when the
// build found no two IDs sharing their top 63 bits (KadTables::exact == 0): the one 64-bit
// compare is then exact and branch-free.  EX = true keeps the 160-bit fallback on ties.
template <bool EX>
__device__ __forceinline__ bool cand_lt(uint64_t da, uint32_t ia, uint64_t db, uint32_t ib, const K160& K,
                                        const KadNode* __restrict__ nodes)
{
    if constexpr (!EX) {
        (void)ia; (void)ib; (void)K; (void)nodes;
        return da < db;
    }
    if (da != db) return da < db;
    if (ia == ib || ia == NONE) return false;
    if (ib == NONE) return true;
    const K160 xa = k_xor(node_key(nodes, ia), K), xb = k_xor(node_key(nodes, ib), K);   // rare
    return k_lt(xa, xb);
}

#ifdef OVS_KAD_STATS
// cost experiment (-DOVS_KAD_STATS builds): lane occupancy of K2's phases (kad_route.hip)
__device__ unsigned long long g_kad_stats[8];
#endif

template <int CAP>
struct SVec {
    uint32_t idx[CAP];
    uint64_t d[CAP];
    uint32_t used;   // bit i: entry i alreadyUsed (LookupVector only)
    int n;
};

template <int CAP>
__device__ __forceinline__ void svec_clear(SVec<CAP>& v)
{
    v.n = 0;
    v.used = 0;
#pragma unroll
    for (int i = 0; i < CAP; ++i) { v.idx[i] = NONE; v.d[i] = ~0ull; }
}

// ---------------------------------------------------------------------------
// Sorting networks over 8 (distance, node) pairs.  The findNode result and the LookupVector
// are "the cap XOR-closest distinct nodes seen" -- BaseKeySortedVector::add (NodeVector.h:
// 381-512) applied to a sequence of candidates yields exactly that set in distance order,
// whatever the order of the adds -- so a block of candidates is sorted with a 19-comparator
// network and merged into the running top 8 with a bitonic merge (8 min + 12 comparators).
// Empty entries are (~0, NONE) and sort last.

template <int C>
struct BlkN {
    uint64_t d[C];
    uint32_t x[C];
    uint32_t f[C];     // payload flags (LookupVector merge: bit 0 alreadyUsed, bit 1 from the response)
};
using Blk8 = BlkN<8>;

template <bool F, bool EX, int C>
__device__ __forceinline__ void blk_ce(BlkN<C>& b, int i, int j, const K160& K, const KadNode* __restrict__ nodes)
{
    const bool s = cand_lt<EX>(b.d[j], b.x[j], b.d[i], b.x[i], K, nodes);
    const uint64_t di = s ? b.d[j] : b.d[i], dj = s ? b.d[i] : b.d[j];
    const uint32_t xi = s ? b.x[j] : b.x[i], xj = s ? b.x[i] : b.x[j];
    b.d[i] = di; b.d[j] = dj; b.x[i] = xi; b.x[j] = xj;
    if (F) {
        const uint32_t fi = s ? b.f[j] : b.f[i], fj = s ? b.f[i] : b.f[j];
        b.f[i] = fi; b.f[j] = fj;
    }
}

// Batcher odd-even merge sort, 19 comparators
template <bool F, bool EX>
__device__ __forceinline__ void blk_sort8(Blk8& b, const K160& K, const KadNode* __restrict__ nodes)
{
    blk_ce<F, EX>(b, 0, 1, K, nodes); blk_ce<F, EX>(b, 2, 3, K, nodes); blk_ce<F, EX>(b, 4, 5, K, nodes); blk_ce<F, EX>(b, 6, 7, K, nodes);
    blk_ce<F, EX>(b, 0, 2, K, nodes); blk_ce<F, EX>(b, 1, 3, K, nodes); blk_ce<F, EX>(b, 4, 6, K, nodes); blk_ce<F, EX>(b, 5, 7, K, nodes);
    blk_ce<F, EX>(b, 1, 2, K, nodes); blk_ce<F, EX>(b, 5, 6, K, nodes);
    blk_ce<F, EX>(b, 0, 4, K, nodes); blk_ce<F, EX>(b, 1, 5, K, nodes); blk_ce<F, EX>(b, 2, 6, K, nodes); blk_ce<F, EX>(b, 3, 7, K, nodes);
    blk_ce<F, EX>(b, 2, 4, K, nodes); blk_ce<F, EX>(b, 3, 5, K, nodes);
    blk_ce<F, EX>(b, 1, 2, K, nodes); blk_ce<F, EX>(b, 3, 4, K, nodes); blk_ce<F, EX>(b, 5, 6, K, nodes);
}

// a <- the C smallest of sorted a (C entries) and sorted b (CB <= C entries, as if padded with empty
// ones), sorted: a against reversed b is bitonic, then half-cleaners at C/2 .. 1
template <bool F, bool EX, int C, int CB>
__device__ __forceinline__ void blk_merge_top(BlkN<C>& a, const BlkN<CB>& b, const K160& K,
                                              const KadNode* __restrict__ nodes)
{
    static_assert(CB <= C, "merge a smaller block into a larger vector");
#pragma unroll
    for (int i = 0; i < C; ++i) {
        const int j = C - 1 - i;
        if (j < CB) {
            const bool s = cand_lt<EX>(b.d[j], b.x[j], a.d[i], a.x[i], K, nodes);
            a.d[i] = s ? b.d[j] : a.d[i];
            a.x[i] = s ? b.x[j] : a.x[i];
            if (F) a.f[i] = s ? b.f[j] : a.f[i];
        }
    }
#pragma unroll
    for (int w = C / 2; w >= 1; w >>= 1) {
#pragma unroll
        for (int i = 0; i < C; ++i)
            if ((i & w) == 0) blk_ce<F, EX>(a, i, i + w, K, nodes);
    }
}

// a <- the 8 smallest of sorted a and sorted b, sorted (8 min + 12 comparators)
template <bool F, bool EX>
__device__ __forceinline__ void blk_merge_top8(Blk8& a, const Blk8& b, const K160& K, const KadNode* __restrict__ nodes)
{
    blk_merge_top<F, EX, 8, 8>(a, b, K, nodes);
}

// a <- the C smallest of sorted a and the single entry (d, x): its position is the count of entries
// closer, the entries from there on move down one (the last drops) -- what blk_merge_top computes
// for a block holding one entry, in C compares and selects instead of C min + (C/2)log2(C) comparators
// (no payload flags: the findNode blocks)
template <bool EX, int C>
__device__ __forceinline__ void blk_insert1(BlkN<C>& a, uint64_t d, uint32_t x, const K160& K,
                                            const KadNode* __restrict__ nodes)
{
    bool lt[C];
#pragma unroll
    for (int i = 0; i < C; ++i) lt[i] = cand_lt<EX>(d, x, a.d[i], a.x[i], K, nodes);   // x goes before entry i
#pragma unroll
    for (int i = C - 1; i >= 0; --i) {
        const bool here = lt[i] && (i == 0 || !lt[i - 1]);
        const bool down = i > 0 && lt[i - 1];
        a.d[i] = down ? a.d[i > 0 ? i - 1 : 0] : here ? d : a.d[i];
        a.x[i] = down ? a.x[i > 0 ? i - 1 : 0] : here ? x : a.x[i];
    }
}

template <int C>
__device__ __forceinline__ void blk_clear(BlkN<C>& b)
{
#pragma unroll
    for (int i = 0; i < C; ++i) { b.d[i] = ~0ull; b.x[i] = NONE; b.f[i] = 0; }
}

// a <- sorted 8-block b (the rest of a empty)
template <int C>
__device__ __forceinline__ void blk_assign(BlkN<C>& a, const Blk8& b)
{
#pragma unroll
    for (int i = 0; i < C; ++i) {
        a.d[i] = i < 8 ? b.d[i < 8 ? i : 0] : ~0ull;
        a.x[i] = i < 8 ? b.x[i < 8 ? i : 0] : NONE;
        a.f[i] = i < 8 ? b.f[i < 8 ? i : 0] : 0u;
    }
}

// the (up to 8) entries of one table block, unsorted; returns how many
__device__ __forceinline__ int blk_load_block(Blk8& b, const KadBlk* __restrict__ blk, const K160& K)
{
    const uint4* p = reinterpret_cast<const uint4*>(blk);
    const uint4 t0 = p[0], t1 = p[1], t2 = p[2], t3 = p[3], i0 = p[4], i1 = p[5];
    const uint64_t tops[8] = {(uint64_t)t0.x | ((uint64_t)t0.y << 32), (uint64_t)t0.z | ((uint64_t)t0.w << 32),
                              (uint64_t)t1.x | ((uint64_t)t1.y << 32), (uint64_t)t1.z | ((uint64_t)t1.w << 32),
                              (uint64_t)t2.x | ((uint64_t)t2.y << 32), (uint64_t)t2.z | ((uint64_t)t2.w << 32),
                              (uint64_t)t3.x | ((uint64_t)t3.y << 32), (uint64_t)t3.z | ((uint64_t)t3.w << 32)};
    const uint32_t ids[8] = {i0.x, i0.y, i0.z, i0.w, i1.x, i1.y, i1.z, i1.w};
    const uint64_t kt = ktop(K);
    int n = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        b.x[q] = ids[q];
        b.d[q] = ids[q] == NONE ? ~0ull : dclamp(tops[q] ^ kt);
        b.f[q] = 0;
        n += ids[q] != NONE ? 1 : 0;
    }
    return n;
}

// keep the first cap entries; returns how many are non-empty
template <int C>
__device__ __forceinline__ int blk_trunc(BlkN<C>& b, int cap)
{
    int n = 0;
#pragma unroll
    for (int i = 0; i < C; ++i) {
        if (i >= cap) { b.x[i] = NONE; b.d[i] = ~0ull; b.f[i] = 0; }
        n += b.x[i] != NONE ? 1 : 0;
    }
    return n;
}

// ---------------------------------------------------------------------------
// Kademlia::isSiblingFor (Kademlia.cc:888-962) from the node's line

// D > R, decided on the top 64 bits, exact on a tie
__device__ __forceinline__ bool beyond_radius(const KadView& V, const KadNode& r, uint32_t c, const K160& D)
{
    const uint64_t dt = ktop(D);
    if (dt != r.rtop) return dt > r.rtop;
    return k_gt(D, as_key(V.nodex[c].R));
}

// (D & levelmask) != 0: some sibling is XOR-closer to the key than the node
__device__ __forceinline__ bool mask_hits(const KadView& V, const KadNode& r, uint32_t c, const K160& D)
{
    if (r.meta & KMETA_MASK_OUT) {
        const KadX& X = V.nodex[c];
        return ((D.w[0] & X.mask[0]) | (D.w[1] & X.mask[1]) | (D.w[2] & X.mask[2]) | (D.w[3] & X.mask[3]) |
                (D.w[4] & X.mask[4])) != 0;
    }
    const int end = kad_end(r.meta);
    const int mlo = end > 63 ? end - 63 : 0;
    // bits [mlo, mlo + 63] of D
    const int wi = mlo >> 5, sh = mlo & 31;
    const uint64_t lo = (uint64_t)kword(D, wi) | ((uint64_t)kword(D, wi + 1) << 32);
    const uint64_t hi = (uint64_t)kword(D, wi + 2);
    const uint64_t win = sh ? ((lo >> sh) | (hi << (64 - sh))) : lo;
    return (win & r.mwin) != 0;
}

// isSiblingFor(thisNode = c, key, 1): table shorter than 1, or (not beyond a full table's radius
// and no sibling closer)
__device__ __forceinline__ bool kad_is_sibling1(const KadView& V, const KadNode& r, uint32_t c, const K160& K)
{
    const int nsib = kad_nsib(r.meta);
    if (nsib < 1) return true;
    const K160 D = k_xor(as_key(r.key), K);
    if (nsib == V.S5 && beyond_radius(V, r, c, D)) return false;
    return !mask_hits(V, r, c, D);
}

// isSiblingFor(thisNode = c, key, numSiblings) for numSiblings >= 1: c is in the numSiblings
// XOR-closest of siblings + c.  A sibling x is closer to K than c exactly when bit msb(x ^ c)
// of D = c ^ K is set (x ^ K = (x ^ c) ^ D differs from D first at that bit), so c qualifies when
// fewer than numSiblings siblings have their level bit set in D.  The mask decides the common
// case; otherwise c's sibling row (owned arc) is counted.
__device__ __forceinline__ bool kad_is_sibling(const KadView& V, const KadNode& r, uint32_t c, const K160& K,
                                               int numSiblings)
{
    if (numSiblings == 0) return k_eq(as_key(r.key), K);   // exact-key lookups (Kademlia.cc:913-916)
    if (numSiblings <= 1) return kad_is_sibling1(V, r, c, K);
    const int nsib = kad_nsib(r.meta);
    if (nsib < numSiblings) return true;
    const K160 me = as_key(r.key);
    const K160 D = k_xor(me, K);
    if (nsib == V.S5 && beyond_radius(V, r, c, D)) return false;
    if (!mask_hits(V, r, c, D)) return true;
    int closer = 0;
    if (kad_off_arc(V, c)) {
        // a responder off this rank's arc (sharded LookupCalls): its replicated sibling levels.
        // Its sibling row lives on its owner only: reading V.sibb at (c - lo) here was the
        // round-2 illegal-address fault (c < lo wraps to ~2^32 rows), DESIGN.md §6
        if (!V.slev) { kad_count_error(V); return false; }
        const uint8_t* lv = V.slev + (uint64_t)c * V.S5;
        for (int i = 0; i < nsib; ++i) closer += (int)kbit(D, lv[i]);
        return closer < numSiblings;
    }
    const KadBlk* L = V.sibb + (uint64_t)(c - V.lo) * V.sbn;
    for (int i = 1; i <= nsib; ++i) {           // row entry 0 is c itself
        const uint32_t x = L[i / KBLK].idx[i % KBLK];
        closer += (int)kbit(D, k_msb(k_xor(node_key(V.nodes, x), me)));
    }
    return closer < numSiblings;
}

// What findNode at a responder needs of its line, captured when the FindNodeCall is sent (the
// line is read then anyway, for the siblings flag and the delay): m = msb(key ^ K) (-1: key == K),
// endIndex, the lowest stored bucket, the bucket-row offset, the sibling count.
struct RespGeo {
    int m, endIndex, rowlo, nsib;
    uint32_t boff;
};

__device__ __forceinline__ RespGeo resp_geo(const KadNode& r, const K160& K)
{
    RespGeo g;
    g.m = k_msb(k_xor(as_key(r.key), K));
    g.endIndex = kad_end(r.meta);
    g.rowlo = kad_rowlo(r.meta);
    g.nsib = kad_nsib(r.meta);
    g.boff = r.boff;
    return g;
}

// entries of a sibling row (c itself + its siblings by level) read for a prefix of pre siblings:
// whole blocks
__device__ __forceinline__ int kad_row_read(int pre) { return KBLK * ((pre + 1 + KBLK - 1) / KBLK); }

// the first of the V.bpb blocks of bucket `bucket` of a node whose row starts at boff
__device__ __forceinline__ const KadBlk* slot_blk(const KadView& V, uint32_t boff, int bucket)
{
    return V.blks + (uint64_t)boff + (uint64_t)(KEYBITS - 1 - bucket) * (uint64_t)V.bpb;
}

// Kademlia::findNode(key, numRedundantNodes, numSiblings) at node c (Kademlia.cc:1101-1246),
// block form: the candidate sets of the reference's scan (bucket m, then buckets m-1..endIndex with
// the sibling table and self when m >= endIndex or the result is short, then buckets above m while
// it is short) merged one table block at a time into the top C.  Returns the result size.
// pre >= 0 (a findNode in the sibling zone, m <= endIndex): only c and the first pre siblings of c's
// level-sorted row can enter the result (kad_sib_prefix); the rest are counted, not read.
// r0 > 0: the entries before row entry r0 cannot enter the result either (kad_sib_range: the
// siblings at level m alone fill it); they are counted, not read.
// KAD_FN_HOOK(kind): a census build's count of the table blocks one findNode reads -- kind 0 bucket
// m, 1 the buckets m-1 .. endIndex, 2 sibling-row blocks, 3 buckets above m (a translation unit
// defines it before including this header; nothing by default)
#ifndef KAD_FN_HOOK
#define KAD_FN_HOOK(kind) ((void)0)
#endif
template <bool EX, int C = 8>
__device__ __forceinline__ int kad_find_node_blk(const KadView& V, uint32_t c, const RespGeo& g, const K160& K,
                                                 int numRedundant, bool sib, BlkN<C>& res, int numSiblings = 1,
                                                 int pre = -1, int r0 = 0)
{
    blk_clear(res);
    if (V.err && ((kad_off_arc(V, c) && g.boff >= V.tend) || g.boff > V.nblk)) {
        // sharded kernels: c's bucket and sibling rows live on its owner only -- counted
        // (ovs_kad_shard_errors), answered empty.  (A row offset below V.tend names c's replicated
        // top buckets, which every rank holds.)  A row offset past this rank's rows (another arc's
        // layout, the round-5 fault) is counted the same way, never dereferenced.
        kad_count_error(V);
        return 0;
    }
    if (g.nsib == 0 || (V.snapshot && sib && numSiblings <= 1)) {
        // an empty sibling table answers [self]; on snapshot tables a sibling for numSiblings = 1
        // is the XOR-closest of everything it knows: nothing below the main bucket beats it
        // 
        res.x[0] = c;
        res.d[0] = dist_hi(node_key(V.nodes, c), K);
        return 1;
    }
    // resultSize = numSiblings (1 for 0) when c is a sibling for K, else numRedundantNodes (Kademlia.cc:1127-1131)
    const int rs = sib ? (numSiblings ? numSiblings : 1) : numRedundant;
    const int cap = rs < C ? rs : C;
    int n = 0, seen = 0;
    auto add_blk = [&](const KadBlk* blk) {
        Blk8 b;
        const int cnt = blk_load_block(b, blk, K);
        if (cnt) {
            // a block holding one entry at its start (a sibling row's last block: 9 entries at s = 8)
            // is sorted and enters the result by one insertion
#ifdef OVS_KAD_NO_INSERT1
            const bool one = false;                  // A/B: the round-3 sort + merge for every block
#else
            const bool one = cnt == 1 && b.x[0] != NONE;
#endif
            if (!one) blk_sort8<false, EX>(b, K, V.nodes);
            if (seen == 0) blk_assign(res, b);       // into an empty result the merge is the sorted block itself
            else if (one) blk_insert1<EX, C>(res, b.d[0], b.x[0], K, V.nodes);
            else blk_merge_top<false, EX, C, 8>(res, b, K, V.nodes);
            n = blk_trunc(res, cap);
            seen += cnt;
        }
    };
    auto add_slot = [&](int bucket) {
        if (g.rowlo < 0 || bucket < g.rowlo) return;      // buckets below the stored row are empty
        const KadBlk* blk = slot_blk(V, g.boff, bucket);
        KAD_FN_HOOK(bucket == g.m ? 0 : bucket < g.m ? 1 : 3);
        // the 8-entry instantiations run only on tables with k <= 8 (one block per bucket; the
        // launchers pick C = 16 otherwise)
        if constexpr (C == 8) add_blk(blk);
        else for (int j = 0; j < V.bpb; ++j) add_blk(blk + j);
    };
    if (g.m >= 0) add_slot(g.m);
    // Members of bucket m are XOR-closer to K than everything below it (buckets < m, siblings --
    // all at msb <= endIndex < m from c -- and c itself all differ from K at bit m): once bucket
    // m fills the result, the rest of the scan cannot change it
    if ((g.m >= g.endIndex || seen < rs) && !(g.m > g.endIndex && n >= cap)) {
        for (int b = g.m - 1; b >= g.endIndex; --b) add_slot(b);
        // the row: c itself, then its siblings by level (put_sibling_row)
        const KadBlk* L = V.sibb + (uint64_t)(c - V.lo) * V.sbn;
        const int tot = g.nsib + 1;
        const int rd = pre < 0 ? tot : min(tot, kad_row_read(pre));
        const int j0 = r0 / KBLK;
        for (int j = j0; j * KBLK < rd; ++j) { KAD_FN_HOOK(2); add_blk(L + j); }
        seen += tot - (rd - j0 * KBLK);
    }
    for (int b = g.m + 1; seen < rs && b < KEYBITS; ++b) add_slot(b);
    return n;
}

// BaseKeySortedVector::add with a KeyDistanceComparator<KeyXorMetric> (NodeVector.h:381-512):
// dedupe by key (== by node index), insert before the first farther entry, truncate to cap.
template <int CAP, bool EX>
__device__ __forceinline__ int svec_add(SVec<CAP>& v, int cap, uint32_t x, uint64_t dx, const K160& K,
                                        const KadNode* __restrict__ nodes)
{
    bool dup = false;
    int pos = 0;
#pragma unroll
    for (int i = 0; i < CAP; ++i) {
        if (i < v.n) {
            dup |= (v.idx[i] == x);
            pos += (v.idx[i] != x && cand_lt<EX>(v.d[i], v.idx[i], dx, x, K, nodes)) ? 1 : 0;
        }
    }
    if (dup || pos >= cap) return -1;
#pragma unroll
    for (int i = CAP - 1; i >= 0; --i) {
        if (i > pos) {
            if (i >= 1) { v.idx[i] = v.idx[i - 1]; v.d[i] = v.d[i - 1]; }
        } else if (i == pos) {
            v.idx[i] = x; v.d[i] = dx;
        }
    }
    v.n = v.n + 1 > cap ? cap : v.n + 1;
    return pos;
}

// findNode for results of up to CAP nodes, one insertion per candidate: the batch ABI
// (ovs_find_node_batch accepts numRedundantNodes / numSiblings up to 16); same scan as
// kad_find_node_blk
template <int CAP, bool EX>
__device__ __forceinline__ int kad_find_node_ins(const KadView& V, uint32_t c, const RespGeo& g, const K160& K,
                                                 int numRedundant, bool sib, SVec<CAP>& res, int numSiblings)
{
    svec_clear(res);
    if (g.nsib == 0 || (V.snapshot && sib && numSiblings <= 1)) {
        svec_add<CAP, EX>(res, 1, c, dist_hi(node_key(V.nodes, c), K), K, V.nodes);
        return 1;
    }
    const int rs = sib ? (numSiblings ? numSiblings : 1) : numRedundant;
    const int cap = rs < CAP ? rs : CAP;
    int seen = 0;
    const uint64_t kt = ktop(K);
    auto add_blk = [&](const KadBlk* blk) {
        for (int q = 0; q < KBLK; ++q) {
            const uint32_t x = blk->idx[q];
            if (x == NONE) break;
            svec_add<CAP, EX>(res, cap, x, dclamp(blk->top[q] ^ kt), K, V.nodes);
            ++seen;
        }
    };
    auto add_slot = [&](int bucket) {
        if (g.rowlo < 0 || bucket < g.rowlo) return;
        const KadBlk* blk = slot_blk(V, g.boff, bucket);
        for (int j = 0; j < V.bpb; ++j) add_blk(blk + j);
    };
    if (g.m >= 0) add_slot(g.m);
    if ((g.m >= g.endIndex || seen < rs) && !(g.m > g.endIndex && res.n >= cap)) {   // as kad_find_node_blk
        for (int b = g.m - 1; b >= g.endIndex; --b) add_slot(b);
        const KadBlk* L = V.sibb + (uint64_t)(c - V.lo) * V.sbn;   // c itself, then its siblings
        for (int j = 0; j * KBLK < g.nsib + 1; ++j) add_blk(L + j);
    }
    for (int b = g.m + 1; seen < rs && b < KEYBITS; ++b) add_slot(b);
    return res.n;
}

// LookupVector merge (IterativePathLookup::handleResponse's add loop, IterativeLookup.cc:853-870):
// nh <- the cap closest distinct nodes of nh and the (sorted) response; alreadyUsed flags stay
// with their nodes.  Returns numNewRpcs: response nodes that entered nh (a response node the
// reference inserts at a position < cap can never be pushed out again by the later, farther
// response nodes, so "inserted" and "in the final vector" coincide).
template <bool EX, int C>
__device__ __forceinline__ int nh_merge(SVec<C>& nh, const SVec<C>& res, int cap, const K160& K,
                                        const KadNode* __restrict__ nodes)
{
    BlkN<C> a, b;
    bool dup = false;
#pragma unroll
    for (int i = 0; i < C; ++i) {
        const bool ina = i < nh.n;
        a.x[i] = ina ? nh.idx[i] : NONE;
        a.d[i] = ina ? nh.d[i] : ~0ull;
        a.f[i] = ina ? ((nh.used >> i) & 1u) : 0u;
        const bool inb = i < res.n;
        b.x[i] = inb ? res.idx[i] : NONE;
        b.d[i] = inb ? res.d[i] : ~0ull;
        b.f[i] = 2u;
    }
#pragma unroll
    for (int j = 0; j < C; ++j) {
        bool dj = false;
#pragma unroll
        for (int i = 0; i < C; ++i) dj |= (b.x[j] != NONE && b.x[j] == a.x[i]);
        if (dj) { b.x[j] = NONE; b.d[j] = ~0ull; }
        dup |= dj;
    }
    if (dup) {
        // holes to the end (every b flag is 2: nothing to carry)
        if constexpr (C == 8) {
            blk_sort8<false, EX>(b, K, nodes);
        } else {
            // a sorted vector with holes stays sorted when the holes move back one place at a time
#pragma unroll
            for (int r = 0; r < C; ++r)
#pragma unroll
                for (int i = r & 1; i + 1 < C; i += 2) blk_ce<false, EX>(b, i, i + 1, K, nodes);
        }
    }
    blk_merge_top<true, EX, C, C>(a, b, K, nodes);
    const int n = blk_trunc(a, cap);
    int numNew = 0;
    uint32_t used = 0;
#pragma unroll
    for (int i = 0; i < C; ++i) {
        nh.idx[i] = a.x[i];
        nh.d[i] = a.d[i];
        numNew += (a.x[i] != NONE && (a.f[i] & 2u)) ? 1 : 0;
        used |= (a.x[i] != NONE && (a.f[i] & 1u)) ? (1u << i) : 0u;
    }
    nh.used = used;
    nh.n = n;
    return numNew;
}

// findNode(key, numRedundantNodes, numSiblings) at node c into a sorted vector
template <int CAP, bool EX>
__device__ __forceinline__ void kad_find_node_vec(const KadView& V, uint32_t c, const KadNode& r, const K160& K,
                                                  int numRedundant, bool sib, SVec<CAP>& res, int numSiblings = 1)
{
    BlkN<CAP> b;
    const int n = kad_find_node_blk<EX, CAP>(V, c, resp_geo(r, K), K, numRedundant, sib, b, numSiblings);
#pragma unroll
    for (int i = 0; i < CAP; ++i) { res.idx[i] = b.x[i]; res.d[i] = b.d[i]; }
    res.n = n;
    res.used = 0;
}

// The scan of kad_find_node_blk counted: only explicit tables with short sibling tables reach it
// (inlined: an out-of-line call costs the lookup kernels more registers than the second copy)
template <bool EX, int C>
__device__ __forceinline__ int kad_scan_size(KadView V, uint32_t c, RespGeo g, K160 K, int rs, int numSiblings)
{
    BlkN<C> b;
    return kad_find_node_blk<EX, C>(V, c, g, K, rs, false, b, numSiblings);
}

// The FindNodeResponse size of node c (its findNode result size): resultSize, unless explicit
// tables leave c fewer candidates on its scan (then counted by running the scan).  SHORT = false:
// tables where that cannot happen (KadTables::maybe_short == 0, every snapshot build) -- the kernel
// then carries no second findNode in its send path (K2: 2000 fewer instructions, no spills)
template <bool EX, int C = 8, bool SHORT = true>
__device__ __forceinline__ int kad_response_size(const KadView& V, uint32_t c, const RespGeo& g, const K160& K,
                                                 int rs, bool sib, int numSiblings)
{
    if (g.nsib == 0 || (sib && numSiblings <= 1)) return 1;
    const int full = rs < (int)V.n ? rs : (int)V.n;
    if constexpr (!SHORT) {
        (void)c; (void)K;
        return full;
    } else {
        if (!V.maybe_short || g.nsib + 1 >= rs) return full;
        return kad_scan_size<EX, C>(V, c, g, K, rs, numSiblings);
    }
}

// ---------------------------------------------------------------------------
// IterativePathLookup, one event per call (K2 in kad_route.hip, the sharded path in kad_shard.hip)

constexpr int MAXA = 8;    // lookupParallelRpcs <= 8 (maidsafe.ini:18-19 sets 8); K2 objects for A = 1..4 and 8
static_assert(MAXA == KAD_MAX_ALPHA, "kad.hpp's kad_pend_slots assumes the A = 8 objects");


struct KadLC {
    int hopCountMax, numSiblings, redundant, alpha;
    int strict, visitOnlyOnce, acceptLateSiblings, useAll, merge, newOnResp, newOnTimeout, finishOnFirst;
    int maxRedundantLocal;   // getMaxNumRedundantNodes() = k
    int full;                // a non-sibling's response size min(numRedundantNodes, n) ...
    int64_t bwFull;          // ... and its serialisation delay
};

// One in-flight FindNodeCall = one future event: its response arrival or its RPC timeout.
// Event order: (time, insertion time, insertion sequence); insertion time is kept as the
// (always < 2^32 ns) gap back from the event time.
struct Pend {
    uint32_t node;
    uint32_t tag;      // step at send (bits 0..15) | insertion sequence (bits 16..30) | timeout (bit 31)
    int64_t t;         // event time (bits 0..55, ns) | the responder's sibling-row blocks (56..63, kad_row_blocks)
    uint32_t dins;     // t - insertion time
    uint32_t geo;      // responder: m + 1 (bits 0..7) | endIndex + 1 (8..15) | rowlo + 1 (16..23) | sib (24)
                       // | sibling count (25..31; 5s <= 120)
    uint32_t boff;     // responder's bucket-row offset
};

constexpr int64_t PEND_TMASK = (1ll << 56) - 1;   // event times stay below 2^56 ns (kad_params_supported)

// How many entries of c's level-sorted sibling row (kad.hip put_sibling_row) a sibling-zone
// findNode(K) with result capacity cap must read.  A sibling at level l = msb(x ^ c) lies at XOR
// distance [2^l, 2^(l+1)) from K when l > m = msb(c ^ K), below 2^(m+1) otherwise, and so does c
// itself: for the smallest l in [m, endIndex) whose siblings at levels <= l plus c reach cap
// candidates, nothing beyond that prefix of the row can enter the result.  lev = KadNode.spare:
// byte k-1 = the siblings at levels <= endIndex - k, k = 1..4.
__device__ __forceinline__ int kad_sib_prefix(const RespGeo& g, uint32_t lev, int cap)
{
    int pre = g.nsib;
    bool found = false;
#pragma unroll
    for (int k = 4; k >= 1; --k) {
        const int c = (int)((lev >> (8 * (k - 1))) & 0xFFu);
        if (!found && g.endIndex - k >= g.m && c + 1 >= cap) { pre = c; found = true; }
    }
    return pre;
}

// The row range a sibling-zone findNode with result capacity cap must read: (first entry, prefix
// as kad_sib_prefix).  The siblings at level m = msb(c ^ K) lie below 2^m from K -- closer than c
// and every other sibling -- so when m is one of the four levels endIndex .. endIndex - 3 whose
// counts KadNode.spare carries and that level alone holds cap siblings, they are the only row
// entries that can enter the result (row entries 1 + count(levels < m) .. count(levels <= m)).
__device__ __forceinline__ int2 kad_sib_range(const RespGeo& g, uint32_t lev, int cap)
{
    const int k = g.endIndex - g.m;
    if (k >= 0 && k <= 3) {
        const int hi = k == 0 ? g.nsib : (int)((lev >> (8 * (k - 1))) & 0xFFu);   // siblings at levels <= m
        const int lo = (int)((lev >> (8 * k)) & 0xFFu);                            // at levels < m
        if (hi - lo >= cap) return make_int2(1 + lo, hi);
    }
    return make_int2(0, kad_sib_prefix(g, lev, cap));
}

// kad_sib_range at block granularity, in one byte (Pend.t bits 56..63): the first row block to
// read (bits 0..3) and the last (4..7); rows hold at most 121 entries = 16 blocks
__device__ __forceinline__ int kad_row_blocks(const RespGeo& g, uint32_t lev, int cap)
{
    const int2 r = kad_sib_range(g, lev, cap);
    return (r.x / KBLK) | ((r.y / KBLK) << 4);
}
__device__ __forceinline__ int rb_pre(int rb) { return (rb >> 4) * KBLK; }   // a prefix through the last block
__device__ __forceinline__ int rb_r0(int rb) { return (rb & 15) * KBLK; }    // the first block's first entry

__device__ __forceinline__ uint32_t pack_geo(const RespGeo& g, bool sb)
{
    return (uint32_t)(g.m + 1) | ((uint32_t)(g.endIndex + 1) << 8) | ((uint32_t)(g.rowlo + 1) << 16) |
           (sb ? 1u << 24 : 0u) | ((uint32_t)g.nsib << 25);
}

__device__ __forceinline__ RespGeo unpack_geo(uint32_t geo, uint32_t boff)
{
    RespGeo g;
    g.m = (int)(geo & 0xFFu) - 1;
    g.endIndex = (int)((geo >> 8) & 0xFFu) - 1;
    g.rowlo = (int)((geo >> 16) & 0xFFu) - 1;
    g.boff = boff;
    g.nsib = (int)(geo >> 25);
    return g;
}

// per-lane lookup state (IterativeLookup + its single IterativePathLookup); C = the LookupVector's and
// findNode's capacity (8; 16 for KademliaLarge's k = lookupRedundantNodes = 16)
template <int A, int C = 8>
struct KadLookup {
    K160 K;
    uint32_t S;
    double sx, sy;
    int64_t now, txf;
    uint32_t seq;
    SVec<C> nh;            // LookupVector nextHops (cap redundantNodes), used bits = alreadyUsed
    Pend p[A];
    uint32_t pvalid;
    int step, hops, pending;
    bool started, pfinished, psuccess, any_to;
    uint32_t result, nsent;
};

// A suspended lookup (the sharded step) in HBM, structure of arrays: word w of lookup q at
// base[w * stride + q], so a wave's lanes touch consecutive words (one 256 B line per word per
// wave).  Written and read field by field: copying the aggregate made the compiler keep the whole
// record addressable, which spilled the step kernel (r04: 0.6 ms at config E, W = 1, for a path
// that never runs there).
template <int A, int C>
struct KadStateWords {
    static constexpr int value = 5 + 1 + 4 + 4 + 1 + 3 * C + 2 + 7 * A + 4 + 3;
};

template <int A, int C>
__device__ __forceinline__ void kad_state_put(uint32_t* __restrict__ base, uint64_t stride, uint64_t q,
                                              const KadLookup<A, C>& L)
{
    int w = 0;
    auto put = [&](uint32_t v) { base[(uint64_t)(w++) * stride + q] = v; };
    auto put64 = [&](uint64_t v) { put((uint32_t)v); put((uint32_t)(v >> 32)); };
#pragma unroll
    for (int k = 0; k < 5; ++k) put(L.K.w[k]);
    put(L.S);
    put64((uint64_t)__double_as_longlong(L.sx));
    put64((uint64_t)__double_as_longlong(L.sy));
    put64((uint64_t)L.now);
    put64((uint64_t)L.txf);
    put(L.seq);
#pragma unroll
    for (int i = 0; i < C; ++i) put(L.nh.idx[i]);
#pragma unroll
    for (int i = 0; i < C; ++i) put64(L.nh.d[i]);
    put(L.nh.used);
    put((uint32_t)L.nh.n);
#pragma unroll
    for (int i = 0; i < A; ++i) {
        put(L.p[i].node); put(L.p[i].tag); put64((uint64_t)L.p[i].t); put(L.p[i].dins); put(L.p[i].geo);
        put(L.p[i].boff);
    }
    put(L.pvalid);
    put((uint32_t)L.step);
    put((uint32_t)L.hops);
    put((uint32_t)L.pending);
    put((L.started ? 1u : 0u) | (L.pfinished ? 2u : 0u) | (L.psuccess ? 4u : 0u) | (L.any_to ? 8u : 0u));
    put(L.result);
    put(L.nsent);
}

template <int A, int C>
__device__ __forceinline__ void kad_state_get(KadLookup<A, C>& L, const uint32_t* __restrict__ base, uint64_t stride,
                                              uint64_t q)
{
    int w = 0;
    auto get = [&]() -> uint32_t { return base[(uint64_t)(w++) * stride + q]; };
    auto get64 = [&]() -> uint64_t { const uint64_t lo = get(); return lo | ((uint64_t)get() << 32); };
#pragma unroll
    for (int k = 0; k < 5; ++k) L.K.w[k] = get();
    L.S = get();
    L.sx = __longlong_as_double((long long)get64());
    L.sy = __longlong_as_double((long long)get64());
    L.now = (int64_t)get64();
    L.txf = (int64_t)get64();
    L.seq = get();
#pragma unroll
    for (int i = 0; i < C; ++i) L.nh.idx[i] = get();
#pragma unroll
    for (int i = 0; i < C; ++i) L.nh.d[i] = get64();
    L.nh.used = get();
    L.nh.n = (int)get();
#pragma unroll
    for (int i = 0; i < A; ++i) {
        L.p[i].node = get(); L.p[i].tag = get(); L.p[i].t = (int64_t)get64(); L.p[i].dins = get(); L.p[i].geo = get();
        L.p[i].boff = get();
    }
    L.pvalid = get();
    L.step = (int)get();
    L.hops = (int)get();
    L.pending = (int)get();
    const uint32_t f = get();
    L.started = f & 1u; L.pfinished = f & 2u; L.psuccess = f & 4u; L.any_to = f & 8u;
    L.result = get();
    L.nsent = get();
}

// A migrating lookup (the sharded step's migration mode, kad_route.hip): its state as one record of
// KadRecWords words -- the lookup id, then the KadStateWords fields -- written and read with 16 B
// accesses (a lane's record is contiguous; the exchange moves records between ranks as rows).
template <int A, int C>
struct KadRecWords {
    static constexpr int value = (1 + KadStateWords<A, C>::value + 3) / 4 * 4;
};

// (fields are streamed through 16 B chunks -- a whole record held in registers spilled the step)
template <int A, int C>
__device__ __forceinline__ void kad_rec_put(uint32_t* __restrict__ rec, uint32_t qid, const KadLookup<A, C>& L)
{
    constexpr int RW = KadRecWords<A, C>::value;
    uint4* o = reinterpret_cast<uint4*>(rec);
    uint32_t b[4] = {0u, 0u, 0u, 0u};
    int i = 0;
    auto put = [&](uint32_t v) {
        b[i & 3] = v;
        if ((i & 3) == 3) o[i >> 2] = make_uint4(b[0], b[1], b[2], b[3]);
        ++i;
    };
    auto put64 = [&](uint64_t v) { put((uint32_t)v); put((uint32_t)(v >> 32)); };
    put(qid);
#pragma unroll
    for (int k = 0; k < 5; ++k) put(L.K.w[k]);
    put(L.S);
    put64((uint64_t)__double_as_longlong(L.sx));
    put64((uint64_t)__double_as_longlong(L.sy));
    put64((uint64_t)L.now);
    put64((uint64_t)L.txf);
    put(L.seq);
#pragma unroll
    for (int k = 0; k < C; ++k) put(L.nh.idx[k]);
#pragma unroll
    for (int k = 0; k < C; ++k) put64(L.nh.d[k]);
    put(L.nh.used);
    put((uint32_t)L.nh.n);
#pragma unroll
    for (int k = 0; k < A; ++k) {
        put(L.p[k].node); put(L.p[k].tag); put64((uint64_t)L.p[k].t); put(L.p[k].dins); put(L.p[k].geo);
        put(L.p[k].boff);
    }
    put(L.pvalid);
    put((uint32_t)L.step);
    put((uint32_t)L.hops);
    put((uint32_t)L.pending);
    put((L.started ? 1u : 0u) | (L.pfinished ? 2u : 0u) | (L.psuccess ? 4u : 0u) | (L.any_to ? 8u : 0u));
    put(L.result);
    put(L.nsent);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (i < RW) put(0u);
}

template <int A, int C>
__device__ __forceinline__ uint32_t kad_rec_get(KadLookup<A, C>& L, const uint32_t* __restrict__ rec)
{
    const uint4* in = reinterpret_cast<const uint4*>(rec);
    uint4 b = make_uint4(0, 0, 0, 0);
    int i = 0;
    auto get = [&]() -> uint32_t {
        if ((i & 3) == 0) b = in[i >> 2];
        const int j = i & 3;
        ++i;
        return j == 0 ? b.x : j == 1 ? b.y : j == 2 ? b.z : b.w;
    };
    auto get64 = [&]() -> uint64_t { const uint64_t lo = get(); return lo | ((uint64_t)get() << 32); };
    const uint32_t qid = get();
#pragma unroll
    for (int k = 0; k < 5; ++k) L.K.w[k] = get();
    L.S = get();
    L.sx = __longlong_as_double((long long)get64());
    L.sy = __longlong_as_double((long long)get64());
    L.now = (int64_t)get64();
    L.txf = (int64_t)get64();
    L.seq = get();
#pragma unroll
    for (int k = 0; k < C; ++k) L.nh.idx[k] = get();
#pragma unroll
    for (int k = 0; k < C; ++k) L.nh.d[k] = get64();
    L.nh.used = get();
    L.nh.n = (int)get();
#pragma unroll
    for (int k = 0; k < A; ++k) {
        L.p[k].node = get(); L.p[k].tag = get(); L.p[k].t = (int64_t)get64(); L.p[k].dins = get(); L.p[k].geo = get();
        L.p[k].boff = get();
    }
    L.pvalid = get();
    L.step = (int)get();
    L.hops = (int)get();
    L.pending = (int)get();
    const uint32_t f = get();
    L.started = f & 1u; L.pfinished = f & 2u; L.psuccess = f & 4u; L.any_to = f & 8u;
    L.result = get();
    L.nsent = get();
    return qid;
}

template <int A, int C>
__device__ __forceinline__ void kad_lookup_init(KadLookup<A, C>& L, const K160& K, uint32_t S,
                                                const double2* __restrict__ xy)
{
    L.K = K;
    L.S = S;
    const double2 sxy = xy[S];
    L.sx = sxy.x; L.sy = sxy.y;
    L.now = 0; L.txf = 0; L.seq = 0;
    svec_clear(L.nh);
    L.pvalid = 0;
    L.step = 0; L.hops = 0; L.pending = 0;
    L.started = false; L.pfinished = false; L.psuccess = false; L.any_to = false;
    L.result = NONE;
    L.nsent = 0;
}

// The FindNodeResponse size of a call's target on the 160-bucket tables (kad_response_size); the
// general tables (K2g, kad_general.hip) bring their own
template <bool EX, int C, bool SHORT>
struct KadBlkSizer {
    __device__ __forceinline__ int operator()(const KadView& V, uint32_t x, const RespGeo& g, const K160& K, int rs,
                                              bool sib, int ns) const
    {
        return kad_response_size<EX, C, SHORT>(V, x, g, K, rs, sib, ns);
    }
};

// FindNodeCall from the source to x at `now` (IterativeLookup::sendRpc 656-689, BaseRpc timeout,
// SimpleNodeEntry::calcDelay with the source's tx queue).  on(slot, x, isTimeout) is told which
// pending-event slot the call occupies (the sharded path requests x's findNode result there).
template <int A, bool EX, bool LK, bool SHORT, class OnSend, int C, class Sizer = KadBlkSizer<EX, C, SHORT>>
__device__ __forceinline__ void kad_send(KadLookup<A, C>& L, const KadView& V, const DelayConsts& DC, const KadLC& LC,
                                         uint32_t x, const OnSend& on, const Sizer& size = Sizer{})
{
    const KadNode rr = load_node(V.nodes, x);
    const int ns = LK ? LC.numSiblings : 1;
    const bool sb = kad_is_sibling(V, rr, x, L.K, ns);
    const RespGeo rg = resp_geo(rr, L.K);
#ifdef OVS_DUP_SEND
    {   // cost experiment: the send's target evaluation (siblings flag, geometry, size, delay) again
        K160 K2 = L.K;
        double sx2 = L.sx;
        asm volatile("" : "+v"(K2.w[0]), "+v"(sx2));
        const bool sb2 = kad_is_sibling(V, rr, x, K2, ns);
        const RespGeo rg2 = resp_geo(rr, K2);
        const int csz2 = kad_response_size<EX>(V, x, rg2, K2, sb2 ? ns : LC.redundant, sb2, ns);
        const int64_t cd2 = coord_ns(sx2, L.sy, rr.x, rr.y, DC.round);
        uint32_t z = (uint32_t)csz2 ^ (uint32_t)cd2 ^ (uint32_t)(cd2 >> 32) ^ (sb2 ? 1u : 0u) ^ (uint32_t)rg2.m;
        asm volatile("" :: "v"(z));
    }
#endif
    // the response carries findNode's result (Kademlia.cc:1127-1131 resultSize)
    const int csz = size(V, x, rg, L.K, sb ? ns : LC.redundant, sb, ns);
    const int64_t cd = coord_ns(L.sx, L.sy, rr.x, rr.y, DC.round);
    const int64_t bwc = DC.bwCall;
    const int64_t newTx = (L.txf > L.now ? L.txf : L.now) + bwc;
    L.txf = newTx;
    const int64_t d1 = (newTx - L.now) + DC.access2 + cd + bwc;
    // the response sizes of a lookup are 1 (a sibling) or resultSize (LC.full) but for short
    // explicit tables: the constant terms, else T(L*8/datarate) itself
    const int64_t bwr = csz == 1 ? DC.bwResp[1] : csz == LC.full ? LC.bwFull
                                                 : bw_ns(DC.respBase + DC.respPerNode * csz, DC.datarate, DC.round);
    const int64_t d2 = 2 * bwr + DC.access2 + cd;
    const int64_t tTo = L.now + DC.rpcTimeout;
    const int64_t tResp = L.now + d1 + d2;
    const bool isTo = tTo <= tResp;   // the timeout was scheduled first: it wins ties
    const uint32_t sTo = L.seq++;
    const uint32_t sR = L.seq++;
    const uint32_t tag = (uint32_t)L.step | ((isTo ? sTo : sR) << 16) | (isTo ? 0x80000000u : 0u);
    const int rcap = min(sb ? (ns ? ns : 1) : LC.redundant, C);
    const int64_t pre = rg.m <= rg.endIndex ? (int64_t)kad_row_blocks(rg, rr.spare, rcap) : 0;
    int slot = 0;
#pragma unroll
    for (int i = A - 1; i >= 0; --i)
        if (!((L.pvalid >> i) & 1u)) slot = i;
#pragma unroll
    for (int i = 0; i < A; ++i) {
        if (i == slot) {
            L.p[i].node = x;
            L.p[i].t = (isTo ? tTo : tResp) | (pre << 56);
            L.p[i].dins = (uint32_t)(isTo ? DC.rpcTimeout : d2);
            L.p[i].tag = tag;
            L.p[i].geo = pack_geo(rg, sb);
            L.p[i].boff = on.boff(x, rr, rg, sb);    // the row findNode will read (OnSend::boff)
        }
    }
    L.pvalid |= 1u << slot;
    ++L.nsent;
    on(slot, x, isTo);
}

// IterativePathLookup::sendRpc (IterativeLookup.cc:1067-1170)
template <int A, bool EX, bool LK, bool SHORT, class OnSend, int C, class Sizer = KadBlkSizer<EX, C, SHORT>>
__device__ __forceinline__ void kad_send_rpcs(KadLookup<A, C>& L, const KadView& V, const DelayConsts& DC, const KadLC& LC,
                                              int num, const OnSend& on, const Sizer& size = Sizer{})
{
    if (L.pfinished) return;
    if (LC.hopCountMax && L.hops >= LC.hopCountMax) { L.pfinished = true; L.psuccess = false; return; }
    if (LC.strict) num = min(num, LC.alpha - L.pending);
    if (num == 0 && L.pending == 0 && !LC.finishOnFirst) num = LC.alpha;
    for (int i = 0; num > 0 && i < LC.redundant; ++i) {
        // getNextEntry: first entry not alreadyUsed (a node that timed out is dead, but it is
        // used already: entries leave nextHops for good once evicted)
        const uint32_t unused = ~L.nh.used & ((1u << L.nh.n) - 1u);
        if (!unused) break;
        const int e = __ffs((int)unused) - 1;
        uint32_t h = NONE;
#pragma unroll
        for (int j = 0; j < C; ++j)
            if (j == e) h = L.nh.idx[j];
        // visitOnlyOnce: an unused entry can only be a visited node if it is the source
        if (!LC.visitOnlyOnce || h != L.S) {
            ++L.pending;
            --num;
            kad_send<A, EX, LK, SHORT>(L, V, DC, LC, h, on, size);
        }
        L.nh.used |= 1u << e;
    }
    if (L.pending == 0) { L.psuccess = false; L.pfinished = true; }
}

// checkStop (IterativeLookup.cc:295-349): the single path finished, or nothing pending
template <int A, int C>
__device__ __forceinline__ bool kad_lookup_done(const KadLookup<A, C>& L)
{
    return L.started && (L.pfinished || L.pvalid == 0);
}

// ---------------------------------------------------------------------------
// The state machine in phases, for kernels that evaluate the sibling-zone findNode
// cooperatively across the wave (K2 k_kad_route, its shard step):
//   kad_event_begin      per lane: pick the earliest event, account for it; tells whether a
//                        findNode result is needed (KEV_FIND), only sends follow (KEV_SENDS),
//                        the event was handled completely (KEV_HANDLED) or, in the shard step,
//                        its remote result has not arrived yet (KEV_WAIT: state untouched)
//   kad_coop_sibzone     whole wave: the findNode scans that need the sibling table
//   kad_event_after_find per lane: LookupVector merge and the finish rules; the RPCs to send
//   kad_send_rpcs        per lane: IterativePathLookup::sendRpc
// A findNode in the sibling zone reads the responder's 5s-entry sibling table (5 blocks at s = 8)
// plus its own main bucket: one lane doing that alone serialises six block loads and sorts, and
// one such lane in a wave made every wave iteration pay for it (42 % of K2's time on config E,
// profiles/r03_dup).  The cooperative form gives each such findNode four lanes (OVS_COOP_G), a block
// each per pass, and merges the sorted blocks in two butterfly steps.

enum : int { KEV_IDLE = 0, KEV_WAIT = 1, KEV_HANDLED = 2, KEV_FIND = 3, KEV_SENDS = 4 };

struct KadEv {
    uint32_t r;        // responder (the source itself at start)
    uint32_t geo;      // its geometry for K and its siblings flag (pack_geo)
    uint32_t boff;
    int e;             // pending slot of the event (-1 at start)
    int numR;          // numRedundantNodes of the findNode
    int num;           // KEV_SENDS: RPCs to send
    int pre;           // the sibling-row blocks a sibling-zone findNode reads (kad_row_blocks)
    bool start;
    __device__ __forceinline__ bool sb() const { return (geo >> 24) & 1u; }
    __device__ __forceinline__ RespGeo rg() const { return unpack_geo(geo, boff); }
};

// IterativeLookup::start / handleRpcResponse / handleRpcTimeout up to the findNode
// (kad_lookup_event's first half).  ready(slot, node, row offset): the result of a response event is
// available (on KEV_WAIT, ev.r names the responder it waits for).
template <int A, bool EX, bool LK, class Ready, class Rec, int C>
__device__ __forceinline__ int kad_event_begin(KadLookup<A, C>& L, const KadView& V, const DelayConsts& DC,
                                               const KadLC& LC, const Ready& ready, const Rec& record, KadEv& ev)
{
    const int ns = LK ? LC.numSiblings : 1;
    ev.r = L.S;
    ev.geo = 0;
    ev.boff = 0;
    ev.e = -1;
    ev.numR = LC.redundant;
    ev.num = 0;
    ev.pre = 0;
    ev.start = !L.started;
    bool resp = true;
    if (ev.start) {
        L.started = true;
        const KadNode rn = load_node(V.nodes, L.S);
        const RespGeo g = resp_geo(rn, L.K);
        const bool sb = kad_is_sibling(V, rn, L.S, L.K, ns);
        ev.geo = pack_geo(g, sb);
        ev.boff = g.boff;
        ev.numR = LC.maxRedundantLocal;
        ev.pre = g.m <= g.endIndex ? kad_row_blocks(g, rn.spare, min(sb ? (ns ? ns : 1) : ev.numR, C)) : 0;
    } else {
        int e = -1;
        int64_t bt = 0, bi = 0;
        uint32_t bs = 0;
#pragma unroll
        for (int i = 0; i < A; ++i) {
            if ((L.pvalid >> i) & 1u) {
                const int64_t t = L.p[i].t & PEND_TMASK;
                const int64_t ti = t - (int64_t)L.p[i].dins;
                const uint32_t si = (L.p[i].tag >> 16) & 0x7FFFu;
                const bool better = e < 0 || t < bt || (t == bt && (ti < bi || (ti == bi && si < bs)));
                if (better) { e = i; bt = t; bi = ti; bs = si; }
            }
        }
        uint32_t r = 0, tag = 0, geo = 0, boff = 0;
        int pre = 0;
#pragma unroll
        for (int i = 0; i < A; ++i)
            if (i == e) {
                r = L.p[i].node; tag = L.p[i].tag; geo = L.p[i].geo; boff = L.p[i].boff;
                pre = (int)((uint64_t)L.p[i].t >> 56);
            }
        ev.pre = pre;
        if (!(tag & 0x80000000u) && !ready(e, r, boff)) { ev.r = r; return KEV_WAIT; }
        ev.r = r;
        ev.e = e;
        L.pvalid &= ~(1u << e);
        L.now = bt;
        if (tag & 0x80000000u) {
            // BaseRpc timeout -> IterativeLookup::handleRpcTimeout (IterativeLookup.cc:588-654)
            L.any_to = true;
            resp = false;
        } else {
            ev.geo = geo;
            ev.boff = boff;
            const bool acc = (LC.useAll && LC.merge) ? true : ((int)(tag & 0xFFFFu) == L.step);
            resp = acc || (ev.sb() && LC.acceptLateSiblings);
        }
    }
    if (resp) {
        if (!ev.start) {
            // IterativePathLookup::handleResponse (IterativeLookup.cc:803-921)
            if (L.now > DC.lookupTimeout) { L.pfinished = true; L.psuccess = false; return KEV_HANDLED; }
            if (ev.r != L.S) {
                record(L.hops, ev.r);
                ++L.hops;
            }
            ++L.step;
            --L.pending;
        }
        if (LK && ns == 0 && ev.start && ev.sb()) {
            // an exact-key lookup of the source's own key (IterativeLookup::start 171-184)
            L.result = L.S;
            L.pfinished = true; L.psuccess = true;
            return KEV_HANDLED;
        }
        return KEV_FIND;
    }
    // IterativePathLookup::handleTimeout (IterativeLookup.cc:935-1023), failedNodeRpcs = false
    --L.pending;
    if (L.now > DC.lookupTimeout) { L.pfinished = true; L.psuccess = false; return KEV_HANDLED; }
    if (LC.newOnTimeout) ev.num = 1;
    else if (L.pending == 0) ev.num = LC.alpha;
    else return KEV_HANDLED;
    return KEV_SENDS;
}

// the findNode answer for the response (kad_lookup_event's second half): numNew, the finish rules;
// returns the RPCs to send, or -1 when the lookup finished
template <int A, bool EX, bool LK, int C>
__device__ __forceinline__ int kad_event_after_find(KadLookup<A, C>& L, const KadView& V, const KadLC& LC, const KadEv& ev,
                                                    const SVec<C>& res)
{
    const int ns = LK ? LC.numSiblings : 1;
    if (LK && ns == 0 && !ev.start && res.n > 0 && k_eq(node_key(V.nodes, res.idx[0]), L.K)) {
        // the key's node is in the response (handleResponse 862-870): XOR distance 0, so first
        L.result = res.idx[0];
        L.pfinished = true; L.psuccess = true;
        return -1;
    }
#ifdef OVS_DUP_MERGE
    {   // cost experiment: the LookupVector merge a second time, on a copy
        SVec<C> nh2 = L.nh;
        asm volatile("" : "+v"(nh2.idx[0]));
        const int k2 = nh_merge<EX>(nh2, res, LC.redundant, L.K, V.nodes);
        uint32_t z = (uint32_t)k2 ^ nh2.used;
        for (int q = 0; q < C; ++q) z ^= nh2.idx[q] ^ (uint32_t)nh2.d[q] ^ (uint32_t)(nh2.d[q] >> 32);
        asm volatile("" :: "v"(z));
    }
#endif
    int numNew = nh_merge<EX>(L.nh, res, LC.redundant, L.K, V.nodes);
    if (LC.numSiblings != 0 && ev.sb() && res.n > 0) {
        if (L.result == NONE) L.result = res.idx[0];
        L.pfinished = true; L.psuccess = true;
        return -1;
    }
    if (numNew == 0 && LC.newOnResp) numNew = 1;
    return ev.start ? LC.alpha : min(numNew, LC.alpha);
}

// Does findNode(K) at c take the cooperative sibling-zone scan?  Kademlia::findNode (Kademlia.cc:
// 1101-1246) scans the main bucket m and, when m >= endIndex or the result is short, the buckets
// m-1 .. endIndex, the sibling table and c itself.  In the sibling zone m <= endIndex the buckets
// below m are empty unless an imported table stores bucket m < endIndex: those (and the [self]
// answers, the buckets above endIndex, off-arc responders) stay on the per-lane path.
// A scan of one block (no main bucket, the row prefix within the first block) stays on the lane.
__device__ __forceinline__ bool kad_find_is_coop(const KadView& V, uint32_t c, const RespGeo& g, bool sib,
                                                 int numSiblings, int pre, int r0 = 0)
{
    if (g.nsib == 0 || (V.snapshot && sib && numSiblings <= 1)) return false;
    if (V.err && kad_off_arc(V, c)) return false;
    if (g.m > g.endIndex) return false;
    const bool stored_below = g.m < g.endIndex && g.rowlo >= 0 && g.m >= g.rowlo;
    if (stored_below) return false;
    const int nmain = g.m >= 0 && g.rowlo >= 0 && g.m >= g.rowlo ? 1 : 0;
    return nmain + kad_row_read(pre) / KBLK - r0 / KBLK >= 2;
}

// position of the t-th (from 0) set bit of m (m has more than t set bits)
__device__ __forceinline__ int nth_set_bit(uint64_t m, int t)
{
    int pos = 0;
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) {
        const uint64_t low = pos + w >= 64 ? ~0ull : ((1ull << (pos + w)) - 1ull);
        if (__popcll(m & low) <= t) pos += w;
    }
    return pos;
}

// LDS of the cooperative findNode, per 256-lane block, entry-major (dword k of lane t at [k][t]:
// a wave's lanes touch consecutive words): the lanes' partial top-8 vectors during the butterfly,
// and each owner's result until its lane picks it up
struct CoopLds {
    uint32_t acc[24][256];
    uint32_t cnt[256];
    uint32_t res[24][256];
    uint32_t rcnt[256];
};

__device__ __forceinline__ void coop_put(uint32_t (*a)[256], int t, const Blk8& b)
{
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        a[3 * q][t] = (uint32_t)b.d[q];
        a[3 * q + 1][t] = (uint32_t)(b.d[q] >> 32);
        a[3 * q + 2][t] = b.x[q];
    }
}

__device__ __forceinline__ void coop_get(const uint32_t (*a)[256], int t, Blk8& b)
{
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        b.d[q] = (uint64_t)a[3 * q][t] | ((uint64_t)a[3 * q + 1][t] << 32);
        b.x[q] = a[3 * q + 2][t];
        b.f[q] = 0;
    }
}

// wave-level ordering of LDS writes and reads between lanes of one wave
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Whole wave (uniform control flow): for every lane with want set, the candidates of its sibling-zone
// findNode -- bucket m if stored, the row blocks rb names (kad_row_blocks) -- merged into the top 8
// by XOR distance to K (left in S.res at the lane's slot) and how many candidates there were
// (S.rcnt).  G lanes per findNode (OVS_COOP_G, 4): lane j of a group loads and sorts item j (and
// j + G, ...), the group merges in log2 G butterfly steps through LDS, the leader stores the result
// for the owner.  64 / G findNodes per pass.
template <bool EX>
__device__ __forceinline__ void kad_coop_sibzone(const KadView& V, bool want, uint32_t c, uint32_t geo, uint32_t boff,
                                                 int rb, const K160& K, CoopLds& S)
{
    const uint64_t tasks = __ballot(want);
    if (tasks == 0) return;
#ifndef OVS_COOP_G
#define OVS_COOP_G 4
#endif
    constexpr int G = OVS_COOP_G;           // lanes per findNode
    constexpr int LG = G == 8 ? 3 : G == 4 ? 2 : 1;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int T = __popcll(tasks);
    const int grp = lane >> LG, j = lane & (G - 1);
    for (int p = 0; p * (64 / G) < T; ++p) {
        const int t = p * (64 / G) + grp;
        const bool live = t < T;
        const int owner = live ? nth_set_bit(tasks, t) : lane;
        const uint32_t oc = __shfl(c, owner);
        const RespGeo og = unpack_geo(__shfl(geo, owner), __shfl(boff, owner));
        const int orb = __shfl(rb, owner);
        K160 oK;
#pragma unroll
        for (int w = 0; w < 5; ++w) oK.w[w] = __shfl(K.w[w], owner);
        const int nmain = og.m >= 0 && og.rowlo >= 0 && og.m >= og.rowlo ? 1 : 0;   // k <= 8: one block
        const int j0 = orb & 15, nsb = (orb >> 4) - j0 + 1;   // the row blocks that matter (kad_row_blocks)
        // sharded kernels: a responder whose rows this rank does not hold (off the arc, or a row
        // offset past its rows) is counted and answered empty, as in kad_find_node_blk
        const bool foreign = V.err && live && (kad_off_arc(V, oc) || og.boff > V.nblk);
        if (foreign && j == 0) kad_count_error(V);
        const int nitems = live && !foreign ? nmain + nsb : 0;
        auto load_item = [&](int i, Blk8& b) -> int {
            if (i < nmain) return blk_load_block(b, slot_blk(V, og.boff, og.m), oK);
            return blk_load_block(b, V.sibb + (uint64_t)(oc - V.lo) * V.sbn + (uint64_t)(j0 + i - nmain), oK);
        };
        Blk8 acc;
        int cnt = 0;
        if (j < nitems) {
            cnt = load_item(j, acc);
            blk_sort8<false, EX>(acc, oK, V.nodes);
        } else {
            blk_clear(acc);
        }
        for (int i = j + G; i < nitems; i += G) {   // more than G items
            Blk8 b;
            const int bc = load_item(i, b);
            blk_sort8<false, EX>(b, oK, V.nodes);
            blk_merge_top8<false, EX>(acc, b, oK, V.nodes);
            cnt += bc;
        }
        // butterfly: after step w every lane holds the top 8 of its aligned 2w lanes
#pragma unroll
        for (int w = 1; w < G; w <<= 1) {
            coop_put(S.acc, tid, acc);
            S.cnt[tid] = (uint32_t)cnt;
            wave_lds_sync();
            const int pt = tid ^ w;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint64_t bd = (uint64_t)S.acc[3 * (7 - i)][pt] | ((uint64_t)S.acc[3 * (7 - i) + 1][pt] << 32);
                const uint32_t bx = S.acc[3 * (7 - i) + 2][pt];
                const bool s = cand_lt<EX>(bd, bx, acc.d[i], acc.x[i], oK, V.nodes);
                acc.d[i] = s ? bd : acc.d[i];
                acc.x[i] = s ? bx : acc.x[i];
            }
            cnt += (int)S.cnt[pt];
            // acc is bitonic: half-cleaners at distance 4, 2, 1
            blk_ce<false, EX>(acc, 0, 4, oK, V.nodes); blk_ce<false, EX>(acc, 1, 5, oK, V.nodes);
            blk_ce<false, EX>(acc, 2, 6, oK, V.nodes); blk_ce<false, EX>(acc, 3, 7, oK, V.nodes);
            blk_ce<false, EX>(acc, 0, 2, oK, V.nodes); blk_ce<false, EX>(acc, 1, 3, oK, V.nodes);
            blk_ce<false, EX>(acc, 4, 6, oK, V.nodes); blk_ce<false, EX>(acc, 5, 7, oK, V.nodes);
            blk_ce<false, EX>(acc, 0, 1, oK, V.nodes); blk_ce<false, EX>(acc, 2, 3, oK, V.nodes);
            blk_ce<false, EX>(acc, 4, 5, oK, V.nodes); blk_ce<false, EX>(acc, 6, 7, oK, V.nodes);
            wave_lds_sync();
        }
        if (live && j == 0) {
            const int ot = tid - lane + owner;
            coop_put(S.res, ot, acc);
            S.rcnt[ot] = (uint32_t)cnt;
        }
    }
    wave_lds_sync();
}

// the per-lane end of a cooperative findNode: truncation to resultSize, then the buckets above m
// while the result is short (Kademlia.cc:1233-1242; only tiny networks / short tables get there)
template <bool EX, int C>
__device__ __forceinline__ int kad_coop_finish(const KadView& V, const RespGeo& g, const K160& K, int numRedundant,
                                               bool sib, int numSiblings, BlkN<C>& res, int seen)
{
    const int rs = sib ? (numSiblings ? numSiblings : 1) : numRedundant;
    const int cap = rs < C ? rs : C;
    int n = blk_trunc(res, cap);
    for (int b = g.m + 1; seen < rs && b < KEYBITS; ++b) {
        if (g.rowlo < 0 || b < g.rowlo) continue;
        for (int j = 0; j < (C == 8 ? 1 : V.bpb); ++j) {
            Blk8 blk;
            const int cnt = blk_load_block(blk, slot_blk(V, g.boff, b) + j, K);
            if (cnt) {
                blk_sort8<false, EX>(blk, K, V.nodes);
                blk_merge_top<false, EX, C, 8>(res, blk, K, V.nodes);
                n = blk_trunc(res, cap);
                seen += cnt;
            }
        }
    }
    return n;
}

// LookupListener::lookupFinished -> KBRTestApp statistics (BaseOverlay.cc:1241-1307)
template <int A, int C>
__device__ __forceinline__ ovs_route_out kad_lookup_output(const KadLookup<A, C>& L, const KadView& V,
                                                           const DelayConsts& DC, const KadLC& LC)
{
    ovs_route_out o;
    o.hops = (uint16_t)L.hops;
    if (L.pfinished && L.psuccess && L.result != NONE) {
        o.status = OVS_LOOKUP_OK;
        o.responsible = L.result;
        o.one_way_hops = (uint8_t)(L.hops + (L.result != L.S ? 1 : 0));
        int64_t lat = L.now;
        if (L.result != L.S && !DC.lookupCall) {
            // sendRouteMessage through the source's tx queue (SimpleNodeEntry.cc:164-194)
            const double2 rxy = V.xy[L.result];
            const int64_t bwr = DC.bwRoute;
            const int64_t newTx = (L.txf > L.now ? L.txf : L.now) + bwr;
            lat = newTx + DC.access2 + coord_ns(L.sx, L.sy, rxy.x, rxy.y, DC.round) + bwr;
        }
        o.latency_ns = lat;
    } else {
        o.responsible = NONE;
        o.one_way_hops = 0;
        o.latency_ns = -1;
        if (L.now > DC.lookupTimeout) o.status = OVS_LOOKUP_TIMEOUT;
        else if (L.any_to) o.status = OVS_LOOKUP_RPC_TIMEOUT;
        else if (LC.hopCountMax && L.hops >= LC.hopCountMax) o.status = OVS_LOOKUP_HOPMAX;
        else o.status = OVS_LOOKUP_NO_NEXT;
    }
    return o;
}

// ---------------------------------------------------------------------------
// host helpers shared by the single-GPU and sharded launchers

inline KadView kad_make_view(const KadTables& t, const double2* xy, uint32_t n)
{
    KadView V{};
    V.nodes = t.nodes; V.nodex = t.nodex; V.blks = t.blks; V.sibb = t.blks ? t.blks + t.rows_blks : nullptr;
    V.slev = t.slev;
    V.xy = xy; V.n = n; V.k = t.k; V.bpb = t.bpb; V.S5 = 5 * t.s;
    V.sbn = (V.S5 + 1 + KBLK - 1) / KBLK;     // c itself + its siblings
    V.lo = t.lo; V.hi = t.hi;
    V.tl = t.tl; V.tend = (uint32_t)t.tend;
    V.nblk = t.rows_blks < 0xFFFFFFFFull ? (uint32_t)t.rows_blks : 0xFFFFFFFFu;
    V.maybe_short = t.maybe_short;
    V.snapshot = t.snapshot;
    return V;
}

// the lookup configurations the K2 state machine implements (others: OVS_ENOTSUP)
inline bool kad_params_supported(const ovs_params& P, const KadTables& t)
{
    // event times of a lookup stay below 2^55 ns (Pend packs a 7-bit field above bit 56)
    const bool times_fit = P.lookupTimeout >= 0 && P.rpcUdpTimeout >= 0 && P.lookupTimeout + 2 * P.rpcUdpTimeout < 3.0e7;
    return times_fit && P.lookupParallelRpcs >= 1 && P.lookupParallelRpcs <= MAXA && P.lookupRedundantNodes >= 1 &&
           P.lookupRedundantNodes <= KMAX && P.lookupMerge && P.lookupStrictParallelRpcs && P.numSiblings >= 0 &&
           P.numSiblings <= t.s && P.numSiblings <= 8 &&
           t.k <= KMAX && P.hopCountMax <= 0x7FFF;
}

inline KadLC kad_make_lc(const ovs_params& P, const KadTables& t)
{
    KadLC LC{};
    LC.hopCountMax = P.hopCountMax;
    LC.numSiblings = P.numSiblings;
    LC.redundant = P.lookupRedundantNodes;
    LC.alpha = P.lookupParallelRpcs;
    LC.strict = P.lookupStrictParallelRpcs;
    LC.visitOnlyOnce = P.lookupVisitOnlyOnce;
    LC.acceptLateSiblings = P.lookupAcceptLateSiblings;
    LC.useAll = P.lookupUseAllParallelResponses;
    LC.merge = P.lookupMerge;
    LC.newOnResp = P.lookupNewRpcOnEveryResponse;
    LC.newOnTimeout = P.lookupNewRpcOnEveryTimeout;
    LC.finishOnFirst = P.lookupFinishOnFirstUnchanged;
    LC.maxRedundantLocal = t.k;
    LC.full = 0;
    LC.bwFull = 0;
    return LC;
}

// the response-size constants of a lookup batch over n nodes (kad_make_lc's caller has DC)
inline void kad_lc_sizes(KadLC& LC, const DelayConsts& DC, uint32_t n)
{
    LC.full = LC.redundant < (int)n ? LC.redundant : (int)n;
    LC.bwFull = DC.bwResp[LC.full <= 16 ? LC.full : 16];
    if (LC.full > 16) LC.full = -1;
}

struct KadShardStepArgs;   // kad_shard.hpp
struct KadMigStepArgs;

// the migration-step instantiation of K2 for one (alpha, exact) pair (kad_route.hip)
template <int A, bool EX>
hipError_t kad_mig_step_launch(const KadView& V, const DelayConsts& DC, const KadLC& LC, const KadMigStepArgs& a,
                               int num_cu, hipStream_t st);

// the shard-step instantiation of K2 for one (alpha, exact) pair (kad_route.hip)
template <int A, bool EX>
hipError_t kad_shard_step_launch(const KadView& V, const DelayConsts& DC, const KadLC& LC, const KadShardStepArgs& a,
                                 int num_cu, hipStream_t st);

// K2 for one (alpha, exact) pair; instantiated in kad_route.hip (one object per pair)
template <int A, bool EX>
hipError_t kad_route_launch(const KadView& V, const DelayConsts& DC, const KadLC& LC, const K160* qkeys,
                            const uint32_t* qsrc, uint64_t nq, ovs_route_out* out, uint32_t* hopseq, uint32_t* rpcs,
                            uint32_t* sibs, int num_cu, hipStream_t st, unsigned long long* dyn = nullptr);

}  // namespace ovs
