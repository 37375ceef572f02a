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

#include "kad.hpp"

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

__global__ void k_kad_set_boff(KadRec* recs, const uint64_t* off, uint32_t n)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v < n) recs[v].boff = (uint32_t)off[v];
}

// builder, pass B: buckets m = 159 .. endIndex, up to k members of T_m minus
// siblings chosen by Floyd sampling (snapshot rule)
__global__ void k_kad_buckets(const KeyRec* __restrict__ recs, const KadRec* __restrict__ krec, uint32_t n, int k,
                              int S5, uint64_t seed, const uint32_t* __restrict__ sib, KadEntry* __restrict__ slots)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const KadRec r = krec[v];
    const K160 me = as_key(r.key);
    const K160 R = as_key(r.R);
    if (k_msb(R) < 0) return;
    const int endIndex = k_msb(R);
    const uint32_t* L = sib + (uint64_t)v * S5;
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

__device__ __forceinline__ uint64_t dist_hi(const K160& x, const K160& K)
{
    return ((uint64_t)(x.w[4] ^ K.w[4]) << 32) | (uint64_t)(x.w[3] ^ K.w[3]);
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
// Kademlia::isSiblingFor(thisNode, key, 1) (Kademlia.cc:888-962) from the 64 B record
__device__ __forceinline__ bool kad_is_sibling1(const KadView& V, const KadRec& r, const K160& K)
{
    if (V.nsib < 1) return true;
    const K160 D = k_xor(as_key(r.key), K);
    if (V.nsib == V.S5 && k_gt(D, as_key(r.R))) return false;
    const K160 M = as_key(r.mask);
    return ((D.w[0] & M.w[0]) | (D.w[1] & M.w[1]) | (D.w[2] & M.w[2]) | (D.w[3] & M.w[3]) | (D.w[4] & M.w[4])) == 0;
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
            dd[q] = ((uint64_t)(c.x ^ K.w[4]) << 32) | (uint64_t)(b.y ^ K.w[3]);
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

// Kademlia::findNode(key, numRedundantNodes, numSiblings=1) at node c (Kademlia.cc:1101-1246)
template <int CAP>
__device__ __forceinline__ void kad_find_node1(const KadView& V, uint32_t c, const KadRec& r, const K160& K, int numRedundant,
                               bool sib, SVec<CAP>& res)
{
    svec_clear(res);
    const K160 me = as_key(r.key);
    if (V.nsib == 0 || sib) {
        // resultSize = 1 and self is the XOR-closest of siblings + self; with a full table the
        // key lies below endIndex so bucket msb(D) is all siblings
        svec_add(res, 1, c, dist_hi(me, K), K, V.recs);
        return;
    }
    const int cap = numRedundant < CAP ? numRedundant : CAP;
    const K160 D = k_xor(me, K);
    const int m = k_msb(D);
    const int endIndex = k_msb(as_key(r.R));
    auto slot_of = [&](int b) { return r.boff + (uint32_t)(KEYBITS - 1 - b); };
    if (m >= 0 && m >= endIndex) add_slot(res, cap, V, slot_of(m), K);
    if (m >= endIndex || res.n < cap) {
        // nothing below bucket m can beat a full result unless siblings share bucket m
        if (!(m > endIndex && res.n >= cap)) {
            for (int b = m - 1; b >= endIndex; --b) add_slot(res, cap, V, slot_of(b), K);
            const KadEntry* L = V.sibe + (uint64_t)c * V.S5;
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

// FindNodeCall from the source to x at `now` (IterativeLookup::sendRpc 656-689, BaseRpc timeout,
// SimpleNodeEntry::calcDelay with the source's tx queue)
template <int A>
__device__ __forceinline__ void kad_send(KadLookup<A>& L, const KadView& V, const DelayConsts& DC, const KadLC& LC,
                                         uint32_t x)
{
    const double2 cxy = V.xy[x];
    const KadRec rr = kad_rec(V.recs, x);
    const bool sb = kad_is_sibling1(V, rr, L.K);
    // the response carries findNode's result: 1 node when x is sibling, else min(redundant, n)
    const int csz = sb ? 1 : (LC.redundant < (int)V.n ? LC.redundant : (int)V.n);
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
        }
    }
    L.pvalid |= 1u << slot;
    ++L.nsent;
}

// IterativePathLookup::sendRpc (IterativeLookup.cc:1067-1170)
template <int A>
__device__ __forceinline__ void kad_send_rpcs(KadLookup<A>& L, const KadView& V, const DelayConsts& DC, const KadLC& LC,
                                              int num)
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
            kad_send(L, V, DC, LC, h);
        }
        L.nh.used |= 1u << e;
    }
    if (L.pending == 0) { L.psuccess = false; L.pfinished = true; }
}

template <int A>
__device__ __forceinline__ void kad_timeoutlike(KadLookup<A>& L, const KadView& V, const DelayConsts& DC,
                                                const KadLC& LC)
{
    // IterativePathLookup::handleTimeout (IterativeLookup.cc:935-1023), failedNodeRpcs = false
    --L.pending;
    if (L.now > DC.lookupTimeout) { L.pfinished = true; L.psuccess = false; }
    else if (LC.newOnTimeout) kad_send_rpcs(L, V, DC, LC, 1);
    else if (L.pending == 0) kad_send_rpcs(L, V, DC, LC, LC.alpha);
}

template <int A, bool RECORD>
__global__ __launch_bounds__(256) void k_kad_route(KadView V, DelayConsts DC, KadLC LC, const K160* __restrict__ qkeys,
                                                   const uint32_t* __restrict__ qsrc, uint64_t nq, uint64_t chunk,
                                                   ovs_route_out* __restrict__ out, uint32_t* __restrict__ hopseq,
                                                   uint32_t* __restrict__ rpcs_out)
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

    while (true) {
        const uint64_t need = __ballot(!active);
        if (need != 0 && cursor < end) {
            const uint64_t mine = cursor + (uint64_t)__popcll(need & lt_mask);
            if (!active && mine < end) {
                q = mine;
                active = true;
                L.K = qkeys[q];
                L.S = qsrc[q];
                const double2 sxy = V.xy[L.S];
                L.sx = sxy.x; L.sy = sxy.y;
                L.now = 0; L.txf = 0; L.seq = 0;
                svec_clear(L.nh);
                L.pvalid = 0;
                L.step = 0; L.hops = 0; L.pending = 0;
                L.pfinished = false; L.psuccess = false; L.any_to = false;
                L.result = NONE;
                L.nsent = 0;
                // IterativeLookup::start (IterativeLookup.cc:133-244): local findNode at S
                const KadRec rs = kad_rec(V.recs, L.S);
                const bool sb = kad_is_sibling1(V, rs, L.K);
                kad_find_node1(V, L.S, rs, L.K, LC.maxRedundantLocal, sb, res);
                if (res.n == 0) { L.pfinished = true; L.psuccess = false; }
                else if (LC.numSiblings != 0 && sb) {
                    L.result = res.idx[0];
                    L.pfinished = true; L.psuccess = true;
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if (j < res.n) svec_add(L.nh, LC.redundant, res.idx[j], res.d[j], L.K, V.recs);
                    kad_send_rpcs(L, V, DC, LC, LC.alpha);
                }
            }
            cursor += (uint64_t)__popcll(need);
        }
        if (!__any(active)) break;
        if (!active) continue;

        if (!L.pfinished && L.pvalid) {
            // earliest event
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
            uint32_t r = 0, tag = 0;
#pragma unroll
            for (int i = 0; i < A; ++i)
                if (i == e) { r = L.p[i].node; tag = L.p[i].tag; }
            L.pvalid &= ~(1u << e);
            L.now = bt;
            const int vr = (int)(tag & 0xFFFFu);
            if (tag & 0x80000000u) {
                // BaseRpc timeout -> IterativeLookup::handleRpcTimeout (IterativeLookup.cc:588-654)
                L.any_to = true;
                kad_timeoutlike(L, V, DC, LC);
            } else {
                const KadRec rr = kad_rec(V.recs, r);
                const bool sb = kad_is_sibling1(V, rr, L.K);
                const bool acc = (LC.useAll && LC.merge) ? true : (vr == L.step);
                if (acc || (sb && LC.acceptLateSiblings)) {
                    // IterativePathLookup::handleResponse (IterativeLookup.cc:803-921)
                    if (L.now > DC.lookupTimeout) { L.pfinished = true; L.psuccess = false; }
                    else {
                        if (r != L.S) {
                            if (RECORD && L.hops < LC.hopCountMax)
                                hopseq[q * (uint64_t)LC.hopCountMax + L.hops] = r;
                            ++L.hops;
                        }
                        ++L.step;
                        --L.pending;
                        kad_find_node1(V, r, rr, L.K, LC.redundant, sb, res);
                        int numNew = 0;
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            if (j < res.n) {
                                const int pos = svec_add(L.nh, LC.redundant, res.idx[j], res.d[j], L.K, V.recs);
                                if (pos >= 0 && pos < LC.redundant) ++numNew;
                            }
                        }
                        if (LC.numSiblings != 0 && sb && res.n > 0 && L.result == NONE) L.result = res.idx[0];
                        if (sb && res.n != 0 && LC.numSiblings != 0) { L.pfinished = true; L.psuccess = true; }
                        else {
                            if (numNew == 0 && LC.newOnResp) numNew = 1;
                            kad_send_rpcs(L, V, DC, LC, min(numNew, LC.alpha));
                        }
                    }
                } else {
                    // not accepted: handled as a timeout, its nodes are dropped
                    kad_timeoutlike(L, V, DC, LC);
                }
            }
        }
        // checkStop (IterativeLookup.cc:295-349): the single path finished, or nothing pending
        if (L.pfinished || L.pvalid == 0) {
            ovs_route_out o;
            o.hops = (uint16_t)L.hops;
            if (L.pfinished && L.psuccess && L.result != NONE) {
                o.status = OVS_LOOKUP_OK;
                o.responsible = L.result;
                o.one_way_hops = (uint8_t)(L.hops + (L.result != L.S ? 1 : 0));
                int64_t lat = L.now;
                if (L.result != L.S) {
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
            out[q] = o;
            if (rpcs_out) rpcs_out[q] = L.nsent;
            active = false;
        }
    }
}

// batched findNode (general numRedundantNodes <= 16, numSiblings == 1) for the ABI
__global__ void k_kad_find_node(KadView V, const uint32_t* __restrict__ node, const K160* __restrict__ keys, uint64_t n,
                                int numRedundant, uint32_t* __restrict__ out_nodes, uint32_t max_out,
                                uint8_t* __restrict__ out_count, uint8_t* __restrict__ out_sib)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = node[i];
    const K160 K = keys[i];
    const KadRec r = kad_rec(V.recs, c);
    const bool sb = kad_is_sibling1(V, r, K);
    SVec<16> res;
    kad_find_node1(V, c, r, K, numRedundant, sb, res);
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

hipError_t kad_build(const KeyRec* recs, uint32_t n, int k, int s, uint64_t seed, KadTables& t, hipStream_t st)
{
    hipError_t e;
    kad_free(t);
    t.k = k; t.s = s; t.seed = seed;
    const int S5 = 5 * s;
    uint64_t *rowlen = nullptr, *off = nullptr;
    void* tmp = nullptr;
    size_t tmpb = 0;
    if ((e = hipMalloc(&t.recs, sizeof(KadRec) * n)) != hipSuccess) return e;
    if ((e = hipMalloc(&t.sib, sizeof(uint32_t) * (uint64_t)n * S5)) != hipSuccess) return e;
    if ((e = hipMalloc(&rowlen, sizeof(uint64_t) * (n + 1))) != hipSuccess) return e;
    if ((e = hipMalloc(&off, sizeof(uint64_t) * (n + 1))) != hipSuccess) { hipFree(rowlen); return e; }
    hipLaunchKernelGGL(k_kad_siblings, dim3(nblk(n, 128)), dim3(128), 0, st, recs, n, S5, t.sib, t.recs, rowlen);
    hipMemsetAsync(rowlen + n, 0, sizeof(uint64_t), st);
    hipcub::DeviceScan::ExclusiveSum(nullptr, tmpb, rowlen, off, n + 1, st);
    if ((e = hipMalloc(&tmp, tmpb)) != hipSuccess) { hipFree(rowlen); hipFree(off); return e; }
    hipcub::DeviceScan::ExclusiveSum(tmp, tmpb, rowlen, off, n + 1, st);
    uint64_t total = 0;
    hipMemcpyAsync(&total, off + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st);
    if ((e = hipStreamSynchronize(st)) != hipSuccess) { hipFree(rowlen); hipFree(off); hipFree(tmp); return e; }
    if (total >= 0xFFFFFFFFull) { hipFree(rowlen); hipFree(off); hipFree(tmp); return hipErrorInvalidValue; }
    t.total_slots = total;
    if ((e = hipMalloc(&t.slots, sizeof(KadEntry) * (total + 1) * k)) != hipSuccess) {
        hipFree(rowlen); hipFree(off); hipFree(tmp); return e;
    }
    hipLaunchKernelGGL(k_kad_set_boff, dim3(nblk(n, 256)), dim3(256), 0, st, t.recs, off, n);
    if ((e = hipMalloc(&t.sibe, sizeof(KadEntry) * (uint64_t)n * S5)) != hipSuccess) {
        hipFree(rowlen); hipFree(off); hipFree(tmp); return e;
    }
    hipLaunchKernelGGL(k_kad_sibentries, dim3(nblk((uint64_t)n * S5, 256)), dim3(256), 0, st, recs, t.sib,
                       (uint64_t)n * S5, t.sibe);
    hipLaunchKernelGGL(k_kad_buckets, dim3(nblk(n, 64)), dim3(64), 0, st, recs, t.recs, n, k, S5, seed, t.sib, t.slots);
    e = hipStreamSynchronize(st);
    hipFree(rowlen); hipFree(off); hipFree(tmp);
    if (e != hipSuccess) return e;
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

static KadView make_view(const KadTables& t, const double2* xy, uint32_t n)
{
    KadView V{};
    V.recs = t.recs; V.xy = xy; V.sib = t.sib; V.sibe = t.sibe; V.slots = t.slots; V.n = n; V.k = t.k; V.S5 = 5 * t.s;
    V.nsib = (int)((uint64_t)(n - 1) < (uint64_t)V.S5 ? n - 1 : (uint32_t)V.S5);
    return V;
}

template <int A, bool RECORD>
static int kad_blocks_per_cu()
{
    static int bpc = 0;
    if (bpc == 0) {
        int b = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_kad_route<A, RECORD>, 256, 0) != hipSuccess || b < 1) b = 1;
        bpc = b;
    }
    return bpc;
}

template <int A, bool RECORD>
static hipError_t kad_launch(const KadView& V, const DelayConsts& DC, const KadLC& LC, const K160* qkeys,
                             const uint32_t* qsrc, uint64_t nq, ovs_route_out* out, uint32_t* hopseq, uint32_t* rpcs,
                             int num_cu, hipStream_t st)
{
    const uint64_t waves = (uint64_t)num_cu * kad_blocks_per_cu<A, RECORD>() * 4;
    uint64_t chunk = (nq + waves - 1) / waves;
    if (chunk < 1) chunk = 1;
    const uint64_t need_waves = (nq + chunk - 1) / chunk;
    hipLaunchKernelGGL((k_kad_route<A, RECORD>), dim3((unsigned)((need_waves + 3) / 4)), dim3(256), 0, st, V, DC, LC,
                       qkeys, qsrc, nq, chunk, out, hopseq, rpcs);
    return hipGetLastError();
}

hipError_t kad_route(const KadTables& t, const KeyRec* recs, const double2* xy, uint32_t n, const ovs_params& P,
                     const DelayConsts& DC, const K160* qkeys, const uint32_t* qsrc, uint64_t nq, ovs_route_out* out,
                     uint32_t* hopseq, uint32_t* rpcs, int num_cu, hipStream_t st)
{
    (void)recs;
    if (nq == 0) return hipSuccess;
    if (P.lookupParallelRpcs < 1 || P.lookupParallelRpcs > MAXA || P.lookupRedundantNodes < 1 ||
        P.lookupRedundantNodes > 8 || !P.lookupMerge || !P.lookupStrictParallelRpcs || P.numSiblings != 1 || t.k > 8 ||
        P.hopCountMax > 0x7FFF)
        return hipErrorNotSupported;
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
    const KadView V = make_view(t, xy, n);
    // strictParallelRpcs: never more than alpha FindNodeCalls in flight (IterativeLookup.cc:1078-1079)
    const int A = P.lookupParallelRpcs;
#define KL(a) (hopseq ? kad_launch<a, true>(V, DC, LC, qkeys, qsrc, nq, out, hopseq, rpcs, num_cu, st) \
                      : kad_launch<a, false>(V, DC, LC, qkeys, qsrc, nq, out, hopseq, rpcs, num_cu, st))
    switch (A) {
    case 1: return KL(1);
    case 2: return KL(2);
    case 3: return KL(3);
    default: return KL(4);
    }
#undef KL
}

hipError_t kad_find_node(const KadTables& t, const KeyRec* recs, uint32_t n, const ovs_params& P, const uint32_t* node,
                         const K160* keys, uint64_t nq, int numRedundant, int numSiblings, uint32_t* out_nodes,
                         uint32_t max_out, uint8_t* out_count, uint8_t* out_sib, hipStream_t st)
{
    (void)recs; (void)P;
    if (nq == 0) return hipSuccess;
    if (numSiblings != 1 || numRedundant > 16) return hipErrorNotSupported;
    const KadView V = make_view(t, nullptr, n);
    hipLaunchKernelGGL(k_kad_find_node, dim3(nblk(nq, 128)), dim3(128), 0, st, V, node, keys, nq, numRedundant, out_nodes,
                       max_out, out_count, out_sib);
    return hipGetLastError();
}

}  // namespace ovs
