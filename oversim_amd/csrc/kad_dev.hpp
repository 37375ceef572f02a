// kad_dev.hpp -- Kademlia device building blocks shared by the single-GPU kernel (kad.hip)
// and the sharded request/response kernels (kad_shard.hip): record loads, sorted vectors,
// isSiblingFor / findNode from the snapshot tables, and the IterativePathLookup state machine.
#pragma once
#include "kad.hpp"

namespace ovs {

// ---------------------------------------------------------------------------
// helpers

__device__ __forceinline__ uint32_t kbit(const K160& k, int b) { return (k.w[b >> 5] >> (b & 31)) & 1u; }

__device__ __forceinline__ K160 kload(const KeyRec* __restrict__ recs, uint32_t i) { return key_of(load_rec(recs, i)); }

__device__ __forceinline__ K160 kad_key(const KadRec* __restrict__ r, uint32_t i)
{
    const uint4* p = reinterpret_cast<const uint4*>(r + i);
    const uint4 a = p[0];
    K160 k;
    k.w[0] = a.x; k.w[1] = a.y; k.w[2] = a.z; k.w[3] = a.w; k.w[4] = r[i].key[4];
    return k;
}

__device__ __forceinline__ KadRec kad_rec(const KadRec* __restrict__ r, uint32_t i)
{
    const uint4* p = reinterpret_cast<const uint4*>(r + i);
    const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
    KadRec o;
    o.key[0] = a.x; o.key[1] = a.y; o.key[2] = a.z; o.key[3] = a.w; o.key[4] = b.x;
    o.R[0] = b.y; o.R[1] = b.z; o.R[2] = b.w; o.R[3] = c.x; o.R[4] = c.y;
    o.mask[0] = c.z; o.mask[1] = c.w; o.mask[2] = d.x; o.mask[3] = d.y; o.mask[4] = d.z;
    o.boff = d.w;
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
// identical to the oracle's kad_hash (bucket sampling of the snapshot rule)
__device__ __forceinline__ uint64_t kad_hash(uint64_t seed, uint32_t node, uint32_t m, uint32_t j)
{
    return splitmix64(seed ^ splitmix64(((uint64_t)node << 32) ^ ((uint64_t)m << 16) ^ (uint64_t)j));
}


// ---------------------------------------------------------------------------
// sorted vectors in registers (static indexing only)

// XOR-distance order of node a vs node b to key K: top 64 bits, exact fallback on ties
__device__ __forceinline__ bool closer(uint64_t da, uint32_t ia, uint64_t db, uint32_t ib, const K160& K,
                                       const KadRec* __restrict__ recs)
{
    if (da != db) return da < db;
    const K160 xa = k_xor(kad_key(recs, ia), K), xb = k_xor(kad_key(recs, ib), K);
    return k_lt(xa, xb);
}

// top 64 bits of the XOR distance, clamped below the empty-entry sentinel ~0 (a real distance
// of ~0 becomes ~0 - 1: ordered before every empty entry, and with KadView::exact == 0 still
// unique, as no two node IDs then share their top 63 bits)
__device__ __forceinline__ uint64_t dclamp(uint64_t d) { return d == ~0ull ? ~0ull - 1 : d; }

__device__ __forceinline__ uint64_t dist_hi(const K160& x, const K160& K)
{
    return dclamp(((uint64_t)(x.w[4] ^ K.w[4]) << 32) | (uint64_t)(x.w[3] ^ K.w[3]));
}

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

// BaseKeySortedVector::add with a KeyDistanceComparator<KeyXorMetric> (NodeVector.h:381-512):
// dedupe by key (== by node index), insert before the first farther entry, truncate to cap.
template <int CAP>
__device__ __forceinline__ int svec_add(SVec<CAP>& v, int cap, uint32_t x, uint64_t dx, const K160& K,
                                        const KadRec* __restrict__ recs)
{
    bool dup = false;
    int pos = 0;
#pragma unroll
    for (int i = 0; i < CAP; ++i) {
        if (i < v.n) {
            dup |= (v.idx[i] == x);
            pos += (v.idx[i] != x && closer(v.d[i], v.idx[i], dx, x, K, recs)) ? 1 : 0;
        }
    }
    if (dup || pos >= cap) return -1;
    const uint32_t lowmask = (1u << pos) - 1u;
    v.used = ((v.used & lowmask) | ((v.used & ~lowmask) << 1)) & ((1u << cap) - 1u);
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

// ---------------------------------------------------------------------------
// Sorting networks over 8 (distance, node) pairs.  The findNode result and the LookupVector
// are "the cap XOR-closest distinct nodes seen" -- BaseKeySortedVector::add applied to a
// sequence of candidates yields exactly that set in distance order, whatever the order of
// the adds -- so instead of one insertion per candidate (an 8-step compare + shift each), a
// block of 8 candidates is sorted with a 19-comparator network and merged into the running
// top 8 with a bitonic merge (8 min + 12 comparators).  Empty entries are (~0, NONE) and
// sort last; equal top-64-bit distances fall back to the exact 160-bit compare.

// XOR distances of distinct nodes to one key are distinct (XOR is a bijection); their top 64
// bits can tie only when the two node IDs share their top 64 bits.  EX = false is used when the
// build found no two IDs sharing their top 63 bits (KadTables::exact == 0): the one 64-bit
// compare is then exact and branch-free.  EX = true keeps the 160-bit fallback on ties.
template <bool EX>
__device__ __forceinline__ bool cand_lt(uint64_t da, uint32_t ia, uint64_t db, uint32_t ib, const K160& K,
                                        const KadRec* __restrict__ recs)
{
    if constexpr (!EX) {
        (void)ia; (void)ib; (void)K; (void)recs;
        return da < db;
    }
    if (da != db) return da < db;
    if (ia == ib || ia == NONE) return false;
    if (ib == NONE) return true;
    const K160 xa = k_xor(kad_key(recs, ia), K), xb = k_xor(kad_key(recs, ib), K);   // rare
    return k_lt(xa, xb);
}

struct Blk8 {
    uint64_t d[8];
    uint32_t x[8];
    uint32_t f[8];     // payload flags (LookupVector merge: bit 0 alreadyUsed, bit 1 from the response)
};

template <bool F, bool EX>
__device__ __forceinline__ void blk_ce(Blk8& b, int i, int j, const K160& K, const KadRec* __restrict__ recs)
{
    const bool s = cand_lt<EX>(b.d[j], b.x[j], b.d[i], b.x[i], K, recs);
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
__device__ __forceinline__ void blk_sort8(Blk8& b, const K160& K, const KadRec* __restrict__ recs)
{
    blk_ce<F, EX>(b, 0, 1, K, recs); blk_ce<F, EX>(b, 2, 3, K, recs); blk_ce<F, EX>(b, 4, 5, K, recs); blk_ce<F, EX>(b, 6, 7, K, recs);
    blk_ce<F, EX>(b, 0, 2, K, recs); blk_ce<F, EX>(b, 1, 3, K, recs); blk_ce<F, EX>(b, 4, 6, K, recs); blk_ce<F, EX>(b, 5, 7, K, recs);
    blk_ce<F, EX>(b, 1, 2, K, recs); blk_ce<F, EX>(b, 5, 6, K, recs);
    blk_ce<F, EX>(b, 0, 4, K, recs); blk_ce<F, EX>(b, 1, 5, K, recs); blk_ce<F, EX>(b, 2, 6, K, recs); blk_ce<F, EX>(b, 3, 7, K, recs);
    blk_ce<F, EX>(b, 2, 4, K, recs); blk_ce<F, EX>(b, 3, 5, K, recs);
    blk_ce<F, EX>(b, 1, 2, K, recs); blk_ce<F, EX>(b, 3, 4, K, recs); blk_ce<F, EX>(b, 5, 6, K, recs);
}

// a <- the 8 smallest of sorted a and sorted b, sorted
template <bool F, bool EX>
__device__ __forceinline__ void blk_merge_top8(Blk8& a, const Blk8& b, const K160& K, const KadRec* __restrict__ recs)
{
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const bool s = cand_lt<EX>(b.d[7 - i], b.x[7 - i], a.d[i], a.x[i], K, recs);
        a.d[i] = s ? b.d[7 - i] : a.d[i];
        a.x[i] = s ? b.x[7 - i] : a.x[i];
        if (F) a.f[i] = s ? b.f[7 - i] : a.f[i];
    }
    // a is bitonic: half-cleaners at distance 4, 2, 1
    blk_ce<F, EX>(a, 0, 4, K, recs); blk_ce<F, EX>(a, 1, 5, K, recs); blk_ce<F, EX>(a, 2, 6, K, recs); blk_ce<F, EX>(a, 3, 7, K, recs);
    blk_ce<F, EX>(a, 0, 2, K, recs); blk_ce<F, EX>(a, 1, 3, K, recs); blk_ce<F, EX>(a, 4, 6, K, recs); blk_ce<F, EX>(a, 5, 7, K, recs);
    blk_ce<F, EX>(a, 0, 1, K, recs); blk_ce<F, EX>(a, 2, 3, K, recs); blk_ce<F, EX>(a, 4, 5, K, recs); blk_ce<F, EX>(a, 6, 7, K, recs);
}

__device__ __forceinline__ void blk_clear(Blk8& b)
{
#pragma unroll
    for (int i = 0; i < 8; ++i) { b.d[i] = ~0ull; b.x[i] = NONE; b.f[i] = 0; }
}

// up to 8 entries of a contiguous KadEntry array (bucket slot / sibling block), unsorted
__device__ __forceinline__ void blk_load(Blk8& b, const KadEntry* __restrict__ s, int cnt, const K160& K)
{
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        if (q < cnt) {
            const uint2* p = reinterpret_cast<const uint2*>(s + q);
            const uint2 bb = p[1], c = p[2];
            b.x[q] = c.y;
            b.d[q] = c.y == NONE ? ~0ull : dclamp(((uint64_t)(c.x ^ K.w[4]) << 32) | (uint64_t)(bb.y ^ K.w[3]));
        } else {
            b.x[q] = NONE;
            b.d[q] = ~0ull;
        }
        b.f[q] = 0;
    }
}

// keep the first cap entries; returns how many are non-empty
__device__ __forceinline__ int blk_trunc(Blk8& b, int cap)
{
    int n = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if (i >= cap) { b.x[i] = NONE; b.d[i] = ~0ull; b.f[i] = 0; }
        n += b.x[i] != NONE ? 1 : 0;
    }
    return n;
}

// ---------------------------------------------------------------------------
// Kademlia::isSiblingFor(thisNode, key, 1) (Kademlia.cc:888-962) from the 64 B record
__device__ __forceinline__ bool kad_is_sibling1(const KadView& V, const KadRec& r, const K160& K)
{
    if (V.nsib < 1) return true;
    const K160 D = k_xor(as_key(r.key), K);
    if (V.nsib == V.S5 && k_gt(D, as_key(r.R))) return false;
    const K160 M = as_key(r.mask);
    return ((D.w[0] & M.w[0]) | (D.w[1] & M.w[1]) | (D.w[2] & M.w[2]) | (D.w[3] & M.w[3]) | (D.w[4] & M.w[4])) == 0;
}

// Kademlia::isSiblingFor(thisNode = c, key, numSiblings) for numSiblings >= 1 (Kademlia.cc:888-962):
// c is in the numSiblings XOR-closest of siblings + c.  A sibling x is closer to K than c exactly
// when bit msb(x ^ c) of D = c ^ K is set (x ^ K = (x ^ c) ^ D differs from D first at that bit),
// so c qualifies when fewer than numSiblings siblings have their level bit set in D.  The mask
// (OR of the level bits) decides the common case; the count reads c's sibling row (owned arc).
__device__ __forceinline__ bool kad_is_sibling(const KadView& V, const KadRec& r, uint32_t c, const K160& K,
                                               int numSiblings)
{
    if (numSiblings <= 1) return kad_is_sibling1(V, r, K);
    if (V.nsib < numSiblings) return true;
    const K160 me = as_key(r.key);
    const K160 D = k_xor(me, K);
    if (V.nsib == V.S5 && k_gt(D, as_key(r.R))) return false;
    const K160 M = as_key(r.mask);
    if (((D.w[0] & M.w[0]) | (D.w[1] & M.w[1]) | (D.w[2] & M.w[2]) | (D.w[3] & M.w[3]) | (D.w[4] & M.w[4])) == 0)
        return true;
    const KadEntry* L = V.sibe + (uint64_t)(c - V.lo) * V.S5;
    int closer = 0;
    for (int i = 0; i < V.nsib; ++i) {
        const K160 x = as_key(L[i].key);
        closer += (int)kbit(D, k_msb(k_xor(x, me)));
    }
    return closer < numSiblings;
}

// insert up to 8 entries of a contiguous entry array (bucket slot or sibling block); the
// loads are issued together before the dependent sorted inserts
template <int CAP>
__device__ __forceinline__ void add_entries8(SVec<CAP>& res, int cap, const KadEntry* __restrict__ s, int cnt,
                                             const K160& K, const KadRec* __restrict__ recs)
{
    uint32_t ix[8];
    uint64_t dd[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        if (q < cnt) {
            const uint2* p = reinterpret_cast<const uint2*>(s + q);
            const uint2 a = p[0], b = p[1], c = p[2];
            ix[q] = c.y;
            dd[q] = dclamp(((uint64_t)(c.x ^ K.w[4]) << 32) | (uint64_t)(b.y ^ K.w[3]));
            (void)a;
        } else {
            ix[q] = NONE;
            dd[q] = 0;
        }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q)
        if (ix[q] != NONE) svec_add(res, cap, ix[q], dd[q], K, recs);
}

template <int CAP>
__device__ __forceinline__ void add_slot(SVec<CAP>& res, int cap, const KadView& V, uint32_t slot, const K160& K)
{
    const KadEntry* e = V.slots + (uint64_t)slot * V.k;
    for (int q0 = 0; q0 < V.k; q0 += 8) add_entries8(res, cap, e + q0, min(8, V.k - q0), K, V.recs);
}

// What findNode at a responder needs of its 64 B record, captured when the FindNodeCall is sent
// (the record is read then anyway, for the siblings flag): m = msb(key ^ K) (-1: key == K),
// endIndex = msb(R), the bucket-row offset.  Its key is re-read only on the rare paths.
struct RespGeo {
    int m, endIndex;
    uint32_t boff;
};

__device__ __forceinline__ RespGeo resp_geo(const KadRec& r, const K160& K)
{
    RespGeo g;
    g.m = k_msb(k_xor(as_key(r.key), K));
    g.endIndex = k_msb(as_key(r.R));
    g.boff = r.boff;
    return g;
}

// Kademlia::findNode(key, numRedundantNodes, numSiblings=1) at node c (Kademlia.cc:1101-1246),
// block form: the candidate sets of the reference's scan (bucket m, then buckets below it with
// the sibling table and self, then buckets above while the result is short) merged 8 at a time
template <bool EX>
__device__ __forceinline__ int kad_find_node_blk(const KadView& V, uint32_t c, const RespGeo& g, const K160& K,
                                                 int numRedundant, bool sib, Blk8& res, int numSiblings = 1)
{
    blk_clear(res);
    if (V.nsib == 0 || (sib && numSiblings <= 1)) {
        // resultSize = 1 and self is the XOR-closest of siblings + self (see kad_find_node1)
        res.x[0] = c;
        res.d[0] = dist_hi(kad_key(V.recs, c), K);
        return 1;
    }
    // resultSize = numSiblings when c is a sibling for K, else numRedundantNodes (Kademlia.cc:1127-1129)
    const int rs = sib ? numSiblings : numRedundant;
    const int cap = rs < 8 ? rs : 8;
    const int m = g.m;
    const int endIndex = g.endIndex;
    int n = 0;
    auto add_block = [&](const KadEntry* e, int cnt) {
        Blk8 b;
        blk_load(b, e, cnt, K);
        blk_sort8<false, EX>(b, K, V.recs);
        blk_merge_top8<false, EX>(res, b, K, V.recs);
        n = blk_trunc(res, cap);
    };
    auto add_slot8 = [&](int bucket) {
        const KadEntry* e = V.slots + (uint64_t)(g.boff + (uint32_t)(KEYBITS - 1 - bucket)) * V.k;
        for (int q0 = 0; q0 < V.k; q0 += 8) add_block(e + q0, min(8, V.k - q0));
    };
    if (m >= 0 && m >= endIndex) add_slot8(m);
    if (m >= endIndex || n < cap) {
        if (!(m > endIndex && n >= cap)) {
            for (int b = m - 1; b >= endIndex; --b) add_slot8(b);
            const KadEntry* L = V.sibe + (uint64_t)(c - V.lo) * V.S5;
            for (int i = 0; i < V.nsib; i += 8) add_block(L + i, min(8, V.nsib - i));
            Blk8 self;
            blk_clear(self);
            self.x[0] = c;
            self.d[0] = dist_hi(kad_key(V.recs, c), K);
            blk_merge_top8<false, EX>(res, self, K, V.recs);
            n = blk_trunc(res, cap);
        }
    }
    for (int b = m + 1; n < cap && b < KEYBITS; ++b)
        if (b >= endIndex) add_slot8(b);
    return n;
}

// LookupVector merge (IterativePathLookup::handleResponse's add loop, IterativeLookup.cc:853-870):
// nh <- the cap closest distinct nodes of nh and the (sorted) response; alreadyUsed flags stay
// with their nodes.  Returns numNewRpcs: response nodes that entered nh (a response node the
// reference inserts at a position < cap can never be pushed out again by the later, farther
// response nodes, so "inserted" and "in the final vector" coincide).
template <bool EX>
__device__ __forceinline__ int nh_merge(SVec<8>& nh, const SVec<8>& res, int cap, const K160& K,
                                        const KadRec* __restrict__ recs)
{
    Blk8 a, b;
    bool dup = false;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
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
    for (int j = 0; j < 8; ++j) {
        bool dj = false;
#pragma unroll
        for (int i = 0; i < 8; ++i) dj |= (b.x[j] != NONE && b.x[j] == a.x[i]);
        if (dj) { b.x[j] = NONE; b.d[j] = ~0ull; }
        dup |= dj;
    }
    if (dup) blk_sort8<true, EX>(b, K, recs);     // holes to the end
    blk_merge_top8<true, EX>(a, b, K, recs);
    const int n = blk_trunc(a, cap);
    int numNew = 0;
    uint32_t used = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        nh.idx[i] = a.x[i];
        nh.d[i] = a.d[i];
        numNew += (a.x[i] != NONE && (a.f[i] & 2u)) ? 1 : 0;
        used |= (a.x[i] != NONE && (a.f[i] & 1u)) ? (1u << i) : 0u;
    }
    nh.used = used;
    nh.n = n;
    return numNew;
}

// Kademlia::findNode(key, numRedundantNodes, numSiblings=1) at node c (Kademlia.cc:1101-1246)
template <int CAP, bool EX = true>
__device__ __forceinline__ void kad_find_node1(const KadView& V, uint32_t c, const KadRec& r, const K160& K, int numRedundant,
                               bool sib, SVec<CAP>& res, int numSiblings = 1)
{
    if constexpr (CAP == 8) {
        Blk8 b;
        const int n = kad_find_node_blk<EX>(V, c, resp_geo(r, K), K, numRedundant, sib, b, numSiblings);
#pragma unroll
        for (int i = 0; i < 8; ++i) { res.idx[i] = b.x[i]; res.d[i] = b.d[i]; }
        res.n = n;
        res.used = 0;
        return;
    }
    svec_clear(res);
    const K160 me = as_key(r.key);
    if (V.nsib == 0 || (sib && numSiblings <= 1)) {
        // resultSize = 1 and self is the XOR-closest of siblings + self; with a full table the
        // key lies below endIndex so bucket msb(D) is all siblings
        svec_add(res, 1, c, dist_hi(me, K), K, V.recs);
        return;
    }
    const int rs = sib ? numSiblings : numRedundant;
    const int cap = rs < CAP ? rs : CAP;
    const K160 D = k_xor(me, K);
    const int m = k_msb(D);
    const int endIndex = k_msb(as_key(r.R));
    auto slot_of = [&](int b) { return r.boff + (uint32_t)(KEYBITS - 1 - b); };
    if (m >= 0 && m >= endIndex) add_slot(res, cap, V, slot_of(m), K);
    if (m >= endIndex || res.n < cap) {
        // nothing below bucket m can beat a full result unless siblings share bucket m
        if (!(m > endIndex && res.n >= cap)) {
            for (int b = m - 1; b >= endIndex; --b) add_slot(res, cap, V, slot_of(b), K);
            const KadEntry* L = V.sibe + (uint64_t)(c - V.lo) * V.S5;   // rows of the owned arc
            for (int i = 0; i < V.nsib; i += 8) add_entries8(res, cap, L + i, min(8, V.nsib - i), K, V.recs);
            svec_add(res, cap, c, dist_hi(me, K), K, V.recs);
        }
    }
    for (int b = m + 1; res.n < cap && b < KEYBITS; ++b)
        if (b >= endIndex) add_slot(res, cap, V, slot_of(b), K);
}

// ---------------------------------------------------------------------------
// K2: batched iterative lookups

constexpr int MAXA = 4;    // lookupParallelRpcs <= 4

struct KadLC {
    int hopCountMax, numSiblings, redundant, alpha;
    int strict, visitOnlyOnce, acceptLateSiblings, useAll, merge, newOnResp, newOnTimeout, finishOnFirst;
    int maxRedundantLocal;   // getMaxNumRedundantNodes() = k
};

// One in-flight FindNodeCall = one future event: its response arrival or its RPC timeout.
// Event order: (time, insertion time, insertion sequence); insertion time is kept as the
// (always < 2^32 ns) gap back from the event time.
struct Pend {
    uint32_t node;
    uint32_t tag;      // step at send (bits 0..15) | insertion sequence (bits 16..30) | timeout (bit 31)
    int64_t t;         // event time
    uint32_t dins;     // t - insertion time
    uint32_t geo;      // responder: m + 1 (bits 0..7) | endIndex + 1 (bits 8..15) | siblings flag (bit 16)
    uint32_t boff;     // responder's bucket-row offset
};

// per-lane lookup state (IterativeLookup + its single IterativePathLookup)
template <int A>
struct KadLookup {
    K160 K;
    uint32_t S;
    double sx, sy;
    int64_t now, txf;
    uint32_t seq;
    SVec<8> nh;            // LookupVector nextHops (cap redundantNodes), used bits = alreadyUsed
    Pend p[A];
    uint32_t pvalid;
    int step, hops, pending;
    bool pfinished, psuccess, any_to;
    uint32_t result, nsent;
};

template <int A>
__device__ __forceinline__ void kad_lookup_init(KadLookup<A>& L, const K160& K, uint32_t S,
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
    L.pfinished = false; L.psuccess = false; L.any_to = false;
    L.result = NONE;
    L.nsent = 0;
}

// FindNodeCall from the source to x at `now` (IterativeLookup::sendRpc 656-689, BaseRpc timeout,
// SimpleNodeEntry::calcDelay with the source's tx queue).  on(slot, x, isTimeout) is told which
// pending-event slot the call occupies (the sharded path requests x's findNode result there).
// LK: a LookupCall batch (numSiblings = LC.numSiblings); otherwise numSiblings = 1 at compile time
template <int A, bool LK, class OnSend>
__device__ __forceinline__ void kad_send(KadLookup<A>& L, const KadView& V, const DelayConsts& DC, const KadLC& LC,
                                         uint32_t x, const OnSend& on)
{
    const double2 cxy = V.xy[x];
    const KadRec rr = kad_rec(V.recs, x);
    const int ns = LK ? LC.numSiblings : 1;
    const bool sb = kad_is_sibling(V, rr, x, L.K, ns);
    const RespGeo rg = resp_geo(rr, L.K);
    const uint32_t geo = (uint32_t)(rg.m + 1) | ((uint32_t)(rg.endIndex + 1) << 8) | (sb ? 0x10000u : 0u);
    // the response carries findNode's result: min(numSiblings, n) nodes when x is sibling,
    // else min(redundant, n)
    const int rsz = sb ? ns : LC.redundant;
    const int csz = rsz < (int)V.n ? rsz : (int)V.n;
    const int64_t cd = coord_ns(L.sx, L.sy, cxy.x, cxy.y, DC.round);
    const int64_t bwc = bw_ns(DC.callBytes, DC.datarate, DC.round);
    const int64_t newTx = (L.txf > L.now ? L.txf : L.now) + bwc;
    L.txf = newTx;
    const int64_t d1 = (newTx - L.now) + DC.access2 + cd + bwc;
    const int64_t bwr = bw_ns(DC.respBase + DC.respPerNode * csz, DC.datarate, DC.round);
    const int64_t d2 = 2 * bwr + DC.access2 + cd;
    const int64_t tTo = L.now + DC.rpcTimeout;
    const int64_t tResp = L.now + d1 + d2;
    const bool isTo = tTo <= tResp;   // the timeout was scheduled first: it wins ties
    const uint32_t sTo = L.seq++;
    const uint32_t sR = L.seq++;
    const uint32_t tag = (uint32_t)L.step | ((isTo ? sTo : sR) << 16) | (isTo ? 0x80000000u : 0u);
    int slot = 0;
#pragma unroll
    for (int i = A - 1; i >= 0; --i)
        if (!((L.pvalid >> i) & 1u)) slot = i;
#pragma unroll
    for (int i = 0; i < A; ++i) {
        if (i == slot) {
            L.p[i].node = x;
            L.p[i].t = isTo ? tTo : tResp;
            L.p[i].dins = (uint32_t)(isTo ? DC.rpcTimeout : d2);
            L.p[i].tag = tag;
            L.p[i].geo = geo;
            L.p[i].boff = rg.boff;
        }
    }
    L.pvalid |= 1u << slot;
    ++L.nsent;
    on(slot, x, isTo);
}

// IterativePathLookup::sendRpc (IterativeLookup.cc:1067-1170)
template <int A, bool LK, class OnSend>
__device__ __forceinline__ void kad_send_rpcs(KadLookup<A>& L, const KadView& V, const DelayConsts& DC, const KadLC& LC,
                                              int num, const OnSend& on)
{
    if (L.pfinished) return;
    if (LC.hopCountMax && L.hops >= LC.hopCountMax) { L.pfinished = true; L.psuccess = false; return; }
    if (LC.strict) num = min(num, LC.alpha - L.pending);
    if (num == 0 && L.pending == 0 && !LC.finishOnFirst) num = LC.alpha;
    for (int i = 0; num > 0 && i < LC.redundant; ++i) {
        // getNextEntry: first entry not alreadyUsed (no node is ever dead in a stable network)
        const uint32_t unused = ~L.nh.used & ((1u << L.nh.n) - 1u);
        if (!unused) break;
        const int e = __ffs((int)unused) - 1;
        uint32_t h = NONE;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (j == e) h = L.nh.idx[j];
        // visitOnlyOnce: an unused entry can only be a visited node if it is the source
        // (responders stay in nextHops as used entries or are evicted for good)
        if (!LC.visitOnlyOnce || h != L.S) {
            ++L.pending;
            --num;
            kad_send<A, LK>(L, V, DC, LC, h, on);
        }
        L.nh.used |= 1u << e;
    }
    if (L.pending == 0) { L.psuccess = false; L.pfinished = true; }
}

template <int A, bool LK, class OnSend>
__device__ __forceinline__ void kad_timeoutlike(KadLookup<A>& L, const KadView& V, const DelayConsts& DC,
                                                const KadLC& LC, const OnSend& on)
{
    // IterativePathLookup::handleTimeout (IterativeLookup.cc:935-1023), failedNodeRpcs = false
    --L.pending;
    if (L.now > DC.lookupTimeout) { L.pfinished = true; L.psuccess = false; }
    else if (LC.newOnTimeout) kad_send_rpcs<A, LK>(L, V, DC, LC, 1, on);
    else if (L.pending == 0) kad_send_rpcs<A, LK>(L, V, DC, LC, LC.alpha, on);
}

// IterativeLookup::start (IterativeLookup.cc:133-244): local findNode at the source
template <int A, bool EX, bool LK, class OnSend>
__device__ __forceinline__ void kad_lookup_start(KadLookup<A>& L, const KadView& V, const DelayConsts& DC,
                                                 const KadLC& LC, SVec<8>& res, const OnSend& on)
{
    const KadRec rs = kad_rec(V.recs, L.S);
    const int ns = LK ? LC.numSiblings : 1;
    const bool sb = kad_is_sibling(V, rs, L.S, L.K, ns);
    kad_find_node1<8, EX>(V, L.S, rs, L.K, LC.maxRedundantLocal, sb, res, ns);
    if (res.n == 0) { L.pfinished = true; L.psuccess = false; }
    else if (LC.numSiblings != 0 && sb) {
        L.result = res.idx[0];
        L.pfinished = true; L.psuccess = true;
    } else {
        nh_merge<EX>(L.nh, res, LC.redundant, L.K, V.recs);
        kad_send_rpcs<A, LK>(L, V, DC, LC, LC.alpha, on);
    }
}

// checkStop (IterativeLookup.cc:295-349): the single path finished, or nothing pending
template <int A>
__device__ __forceinline__ bool kad_lookup_done(const KadLookup<A>& L)
{
    return L.pfinished || L.pvalid == 0;
}

// Process the earliest pending event (response or RPC timeout) of a running lookup.
// getres.ready(slot) says whether the responder's findNode result is available (always on a
// single GPU); getres.fill(slot, node, geometry, sibling, res) produces it.  Returns false, with the
// state untouched, when the earliest event is a response whose result has not arrived yet.
template <int A, bool EX, bool LK, class GetRes, class OnSend, class Rec>
__device__ __forceinline__ bool kad_lookup_event(KadLookup<A>& L, const KadView& V, const DelayConsts& DC,
                                                 const KadLC& LC, SVec<8>& res, const GetRes& getres,
                                                 const OnSend& on, const Rec& record)
{
    int e = -1;
    int64_t bt = 0, bi = 0;
    uint32_t bs = 0;
#pragma unroll
    for (int i = 0; i < A; ++i) {
        if ((L.pvalid >> i) & 1u) {
            const int64_t ti = L.p[i].t - (int64_t)L.p[i].dins;
            const uint32_t si = (L.p[i].tag >> 16) & 0x7FFFu;
            const bool better = e < 0 || L.p[i].t < bt || (L.p[i].t == bt && (ti < bi || (ti == bi && si < bs)));
            if (better) { e = i; bt = L.p[i].t; bi = ti; bs = si; }
        }
    }
    uint32_t r = 0, tag = 0, geo = 0, boff = 0;
#pragma unroll
    for (int i = 0; i < A; ++i)
        if (i == e) { r = L.p[i].node; tag = L.p[i].tag; geo = L.p[i].geo; boff = L.p[i].boff; }
    if (!(tag & 0x80000000u) && !getres.ready(e)) return false;
    L.pvalid &= ~(1u << e);
    L.now = bt;
    const int vr = (int)(tag & 0xFFFFu);
    if (tag & 0x80000000u) {
        // BaseRpc timeout -> IterativeLookup::handleRpcTimeout (IterativeLookup.cc:588-654)
        L.any_to = true;
        kad_timeoutlike<A, LK>(L, V, DC, LC, on);
        return true;
    }
    // the responder's siblings flag and bucket geometry were captured at send (kad_send)
    const bool sb = (geo & 0x10000u) != 0;
    RespGeo rg;
    rg.m = (int)(geo & 0xFFu) - 1;
    rg.endIndex = (int)((geo >> 8) & 0xFFu) - 1;
    rg.boff = boff;
    const bool acc = (LC.useAll && LC.merge) ? true : (vr == L.step);
    if (!(acc || (sb && LC.acceptLateSiblings))) {
        // not accepted: handled as a timeout, its nodes are dropped
        kad_timeoutlike<A, LK>(L, V, DC, LC, on);
        return true;
    }
    // IterativePathLookup::handleResponse (IterativeLookup.cc:803-921)
    if (L.now > DC.lookupTimeout) { L.pfinished = true; L.psuccess = false; return true; }
    if (r != L.S) {
        record(L.hops, r);
        ++L.hops;
    }
    ++L.step;
    --L.pending;
    getres.fill(e, r, rg, sb, res);
    int numNew = nh_merge<EX>(L.nh, res, LC.redundant, L.K, V.recs);
    if (LC.numSiblings != 0 && sb && res.n > 0 && L.result == NONE) L.result = res.idx[0];
    if (sb && res.n != 0 && LC.numSiblings != 0) { L.pfinished = true; L.psuccess = true; }
    else {
        if (numNew == 0 && LC.newOnResp) numNew = 1;
        kad_send_rpcs<A, LK>(L, V, DC, LC, min(numNew, LC.alpha), on);
    }
    return true;
}

// LookupListener::lookupFinished -> KBRTestApp statistics (BaseOverlay.cc:1241-1307)
template <int A>
__device__ __forceinline__ ovs_route_out kad_lookup_output(const KadLookup<A>& L, const KadView& V,
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
            const int64_t bwr = bw_ns(DC.routeBytes, DC.datarate, DC.round);
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
    V.recs = t.recs; V.xy = xy; V.sib = t.sib; V.sibe = t.sibe; V.slots = t.slots; V.n = n; V.k = t.k; V.S5 = 5 * t.s;
    V.lo = t.lo; V.hi = t.hi;
    V.nsib = (int)((uint64_t)(n - 1) < (uint64_t)V.S5 ? n - 1 : (uint32_t)V.S5);
    return V;
}

// the lookup configurations the K2 state machine implements (others: OVS_ENOTSUP)
inline bool kad_params_supported(const ovs_params& P, const KadTables& t)
{
    return P.lookupParallelRpcs >= 1 && P.lookupParallelRpcs <= MAXA && P.lookupRedundantNodes >= 1 &&
           P.lookupRedundantNodes <= 8 && P.lookupMerge && P.lookupStrictParallelRpcs && P.numSiblings >= 1 &&
           P.numSiblings <= t.s && P.numSiblings <= 8 &&
           t.k <= 8 && P.hopCountMax <= 0x7FFF;
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
    return LC;
}

}  // namespace ovs
