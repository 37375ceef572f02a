// koorde.hip -- Koorde routing (src/overlay/koorde/Koorde.cc) for gfx950 (MI355X).
//
// K3 k_koorde_route: one lane per lookup running IterativeLookup with Koorde::findNode (one next
// hop per response; lookupRedundantNodes = lookupParallelRpcs = 1, merge off: a chain of
// FindNodeCalls).  Every FindNodeCall carries the KoordeFindNodeExtMessage (de Bruijn route key
// + step) of the response that produced it, and the responder's findNode advances it
// (IterativeLookup.cc:200-230, 903-920; BaseOverlay.cc:1841-1907).  Per hop the lane reads the
// responder's key, predecessor and first successor (24 B records of the sorted ring), its
// KoordeNode (16 B), and walks its successor / de Bruijn lists -- consecutive ring nodes -- by
// binary search over clockwise distance, which picks the same node as the reference's interval
// loops (walkSuccessorList 572-582, walkDeBruijnList 558-570).  Finished lanes refill from the
// wave's slice of the batch (ballot + popcount); the grid is persistent.
#include "koorde.hpp"

#include <cstdlib>

namespace ovs {

void koorde_free(KoordeTables& t)
{
    if (t.nd) hipFree(t.nd);
    if (t.rec) hipFree(t.rec);
    t.nd = nullptr;
    t.rec = nullptr;
    t.n = 0;
}

namespace {

__device__ __forceinline__ K160 rkey(const KeyRec* __restrict__ recs, uint32_t i) { return key_of(load_rec(recs, i)); }

__device__ __forceinline__ uint32_t ring_add(uint32_t i, uint32_t d, uint32_t n)
{
    const uint64_t j = (uint64_t)i + d;
    return (uint32_t)(j >= n ? j - n : j);
}

// OverlayKey::operator<< / operator>> (OverlayKey.cc:386-425) with trim() to 160 bits, exact for
// every count (the reference's mpn shifts are undefined for counts that are multiples of 64:
// DESIGN.md §Koorde)
__device__ __forceinline__ K160 k_shl(const K160& a, int n)
{
    K160 r;
    const int q = n >> 5, b = n & 31;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const uint32_t hi = k_word(a, i - q), lo = (i - q - 1 >= 0) ? k_word(a, i - q - 1) : 0u;
        r.w[i] = (i - q < 0 || n >= 160) ? 0u : (b ? (hi << b) | (lo >> (32 - b)) : hi);
    }
    return r;
}
__device__ __forceinline__ K160 k_shr(const K160& a, int n)
{
    K160 r;
    const int q = n >> 5, b = n & 31;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const uint32_t lo = k_word(a, i + q), hi = k_word(a, i + q + 1);
        r.w[i] = (n >= 160) ? 0u : (b ? (lo >> b) | (hi << (32 - b)) : lo);
    }
    return r;
}

__device__ __forceinline__ K160 k_small(uint32_t v)
{
    K160 r;
    r.w[0] = v; r.w[1] = 0; r.w[2] = 0; r.w[3] = 0; r.w[4] = 0;
    return r;
}

// The node of the `num` consecutive ring nodes a_0 .. a_{num-1} from sorted index `first` that
// the reference's interval loop returns for key: the last one strictly (clockwise) before key if
// key lies in (a_0, a_{num-1}], else a_{num-1}.  Both are a_i with i = #{j >= 1 : d(a_0, a_j) <
// d(a_0, key)} (the distances grow with j): the largest j with d(a_0, a_j) < d(a_0, key), found
// by bisection over the ring records.  (A precomputed 128 B window of successor distances per
// node, one read instead of the dependent probes, measured 1.4x slower on config K: DESIGN.md.)
__device__ __forceinline__ uint32_t walk_list(const KeyRec* __restrict__ recs, uint32_t n, uint32_t first, int num,
                                              const K160& key)
{
    if (num <= 1) return first;
    const K160 a0 = rkey(recs, first);
    const K160 dk = k_sub(key, a0);
    const uint32_t last = ring_add(first, (uint32_t)(num - 1), n);
    if ((dk.w[0] | dk.w[1] | dk.w[2] | dk.w[3] | dk.w[4]) == 0) return last;
    if (k_lt(k_sub(rkey(recs, last), a0), dk)) return last;
    int lo = 0, hi = num - 1;   // d(a_lo) < dk <= d(a_hi)
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (k_lt(k_sub(rkey(recs, ring_add(first, (uint32_t)mid, n)), a0), dk)) lo = mid; else hi = mid;
    }
    return ring_add(first, (uint32_t)lo, n);
}

struct KView {
    const KeyRec* __restrict__ recs;
    const KoordeNode* __restrict__ nd;
    const KoordeRec* __restrict__ rec;
    uint32_t n;
    int ns, sb, useOther, useSuc;
};

// Koorde::findStartKey (664-762); false = cRuntimeError (invalid start key)
__device__ bool find_start_key(const KView& V, const K160& self, const K160& s0, const K160& dest, K160& out, int& step)
{
    if (k_eq(self, s0)) { out = self; return true; }
    int nBits = k_msb(k_sub(s0, self));
    if (nBits < 0) nBits = 0;
    while ((160 - nBits) % V.sb != 0) nBits--;
    step = nBits + 1;
    const K160 newStart = k_shl(k_shr(self, nBits), nBits);
    K160 newKey = k_add(k_shr(dest, 160 - nBits), newStart);
    if (between_R(newKey, self, s0)) { out = newKey; return true; }
    newKey = k_add(newKey, k_pow2(nBits));
    if (between_R(newKey, self, s0)) { out = newKey; return true; }
    return false;
}

// Koorde::findNode (405-471) at node c, state READY, with findDeBruijnHop (473-556) inlined;
// returns the next hop, NONE where the reference throws
__device__ uint32_t koorde_find_node_dev(const KView& V, uint32_t c, const K160& key, KExt& e)
{
    const uint32_t n = V.n;
    const uint32_t pred = c == 0 ? n - 1 : c - 1;
    const uint32_t s0 = ring_add(c, 1, n);
    const uint32_t slast = ring_add(c, (uint32_t)V.ns, n);
    const K160 me = rkey(V.recs, c);
    const K160 kp = rkey(V.recs, pred);
    const K160 ks0 = rkey(V.recs, s0);
    if (between_R(key, kp, me)) return c;
    if (between_R(key, me, ks0)) return s0;
    if (V.useOther) {
        const uint32_t tmp = walk_list(V.recs, n, s0, V.ns, key);
        if (tmp != slast) return tmp;
    }
    const KoordeNode kn = V.nd[c];
    const K160 kdb = rkey(V.recs, kn.db);
    for (int guard = 0; guard < 200; ++guard) {   // the self-recursion: every round adds shiftingBits to step
        bool brk = false;
        uint32_t h;
        if (!e.has) {
            K160 rk;
            int step = e.step;
            if (!find_start_key(V, me, ks0, key, rk, step)) return NONE;
            e.rk = rk; e.step = step; e.has = 1;
        }
        if (between_R(e.rk, me, ks0)) {
            if (e.step > 160) return NONE;                          // "Bounding error"
            if (160 - e.step - (V.sb - 1) < 0) return NONE;         // getBit below bit 0: getBitRange throws
            // the shiftingBits key bits below position 160 - step, most significant first
            const uint32_t add = (uint32_t)((k_shr(key, 160 - e.step - V.sb + 1).w[0]) & ((1u << V.sb) - 1u));
            e.rk = k_add(k_shl(e.rk, V.sb), k_small(add));
            e.step += V.sb;
            if (kn.dbNum > 0) {
                if (between_R(e.rk, kdb, rkey(V.recs, kn.dbStart))) h = kn.db;
                else h = walk_list(V.recs, n, kn.dbStart, (int)kn.dbNum, e.rk);
            } else {
                h = kn.db;
            }
        } else {
            brk = true;
            if (V.useSuc) {
                const uint32_t tmp = walk_list(V.recs, n, s0, V.ns, e.rk);
                h = between_open(kdb, rkey(V.recs, tmp), e.rk) ? kn.db : tmp;
            } else {
                h = s0;
            }
        }
        if (h != c || brk) return h;
        // findNode calls itself again with the advanced extension; the key checks above
        // (predecessor, successor, successor-list walk) give the same answers again
    }
    return NONE;
}

// ---------------------------------------------------------------------------
// Record form (KoordeRec): the same findNode with every ring distance the reference compares
// decided from the 32-bit codes of the responder's record, the exact keys read only on a code tie.
// A hop then reads the responder's 128 B record and, on the de Bruijn step, the record of the de
// Bruijn list's first node: two dependent loads instead of the list bisections' chain of probes.

__device__ __forceinline__ uint32_t code32(const K160& v) { return (uint32_t)(k_code64(v) >> 32); }

// the first line of a record (and its first successor-distance code)
struct KRec {
    K160 k;
    uint32_t cP, db, dbStart, dbNum;
    double x, y;
    uint32_t s0;         // sum[0] = code(succ0 - v)
};

// the record's second line (the 16 successor-distance codes), where the walks read it: in LDS for
// the responder's own record (its codes are needed again after the de Bruijn record arrives), in
// registers for the de Bruijn list's first node (used at once)
struct CodesLds {
    uint4 (*a)[256];
    int t;
    __device__ __forceinline__ uint4 get(int c) const { return a[c][t]; }
};
struct CodesReg {
    uint4 q[4];
    __device__ __forceinline__ uint4 get(int c) const { return q[c]; }
};

// one record: the 8 chunks are requested together (one memory round trip)
template <class Codes>
__device__ __forceinline__ KRec load_krec(const KoordeRec* __restrict__ rec, uint32_t i, Codes& codes);

__device__ __forceinline__ KRec krec_head(uint4 q0, uint4 q1, uint4 q2, uint4 q3, uint4 q4)
{
    KRec r;
    r.k.w[0] = q0.x; r.k.w[1] = q0.y; r.k.w[2] = q0.z; r.k.w[3] = q0.w; r.k.w[4] = q1.x;
    r.cP = q1.y; r.db = q1.z; r.dbStart = q1.w; r.dbNum = q2.x;
    r.x = __hiloint2double((int)q2.w, (int)q2.z);
    r.y = __hiloint2double((int)q3.y, (int)q3.x);
    r.s0 = q4.x;
    return r;
}

template <>
__device__ __forceinline__ KRec load_krec<CodesLds>(const KoordeRec* __restrict__ rec, uint32_t i, CodesLds& codes)
{
    const uint4* p = reinterpret_cast<const uint4*>(rec + i);
    uint4 q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) q[j] = p[j];
#pragma unroll
    for (int c = 0; c < 4; ++c) codes.a[c][codes.t] = q[4 + c];
    return krec_head(q[0], q[1], q[2], q[3], q[4]);
}

template <>
__device__ __forceinline__ KRec load_krec<CodesReg>(const KoordeRec* __restrict__ rec, uint32_t i, CodesReg& codes)
{
    const uint4* p = reinterpret_cast<const uint4*>(rec + i);
    uint4 q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) q[j] = p[j];
#pragma unroll
    for (int c = 0; c < 4; ++c) codes.q[c] = q[4 + c];
    return krec_head(q[0], q[1], q[2], q[3], q[4]);
}

// #{i in [lo, hi) : sum[i] < ck}; tie: some sum[i] == ck
template <class Codes>
__device__ __forceinline__ int count_codes(const Codes& codes, int lo, int hi, uint32_t ck, bool& tie)
{
    int cnt = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const uint4 q = codes.get(c);
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = 4 * c + j;
            if (i >= lo && i < hi) {
                cnt += w[j] < ck ? 1 : 0;
                tie |= w[j] == ck;
            }
        }
    }
    return cnt;
}

// sign of (exact value e) against the value whose code is c: -1 / +1 decided, 0 = code tie
__device__ __forceinline__ int code_cmp(const K160& e, uint32_t c)
{
    const uint32_t ce = code32(e);
    return ce < c ? -1 : (ce > c ? 1 : 0);
}

// x in (pred(v), v] of the node v of record R: (v - x) < (v - pred) (isBetweenR, pred != v)
__device__ __forceinline__ bool in_pred_r(const KView& V, const KRec& R, uint32_t v, const K160& x)
{
    const int s = code_cmp(k_sub(R.k, x), R.cP);
    if (s) return s < 0;
    return between_R(x, rkey(V.recs, v == 0 ? V.n - 1 : v - 1), R.k);
}

// x in (v, succ0(v)]: 0 < (x - v) <= (succ0 - v)
__device__ __forceinline__ bool in_succ_r(const KView& V, const KRec& R, uint32_t v, const K160& x)
{
    const K160 d = k_sub(x, R.k);
    if ((d.w[0] | d.w[1] | d.w[2] | d.w[3] | d.w[4]) == 0) return false;
    const int s = code_cmp(d, R.s0);
    if (s) return s < 0;
    return between_R(x, R.k, rkey(V.recs, ring_add(v, 1, V.n)));
}

// Koorde::findNode (405-471) at node c with record R: the structure of koorde_find_node_dev with
// record decisions.  The extension e is advanced in place (the caller drops it when the hop ends
// the lookup).
__device__ uint32_t koorde_find_node_rec(const KView& V, uint32_t c, const KRec& R, const CodesLds& RC, const K160& key,
                                         KExt& e)
{
    const uint32_t n = V.n;
    const uint32_t s0 = ring_add(c, 1, n);
    const uint32_t slast = ring_add(c, (uint32_t)V.ns, n);
    if (in_pred_r(V, R, c, key)) return c;
    if (in_succ_r(V, R, c, key)) return s0;
    // the successor-list walk (walkSuccessorList 572-582) from s0: with x beyond s0,
    // d(s0, s_j) < d(s0, x) <=> d(c, s_j) < d(c, x), i.e. the record's codes sum[1 .. ns-1]
    auto succ_walk = [&](const K160& x) -> uint32_t {
        const K160 d = k_sub(x, R.k);
        if ((d.w[0] | d.w[1] | d.w[2] | d.w[3] | d.w[4]) == 0) return slast;   // x == c: d(s0, c) is the largest
        bool tie = false;
        const int cnt = count_codes(RC, 1, V.ns, code32(d), tie);
        if (tie) return walk_list(V.recs, n, s0, V.ns, x);
        return ring_add(s0, (uint32_t)cnt, n);
    };
    if (V.useOther) {
        const uint32_t tmp = succ_walk(key);
        if (tmp != slast) return tmp;
    }
    const uint32_t db = R.db, dbStart = R.dbStart;
    const int dbNum = (int)R.dbNum;
    for (int guard = 0; guard < 200; ++guard) {   // the self-recursion, as koorde_find_node_dev
        bool brk = false;
        uint32_t h;
        if (!e.has) {
            // findStartKey (664-762): nBits = msb(succ0 - c) from the record's code
            int nBits = (int)(R.s0 >> 24) - 1;
            if (nBits < 0) nBits = 0;
            while ((160 - nBits) % V.sb != 0) nBits--;
            const int step = nBits + 1;
            const K160 newStart = k_shl(k_shr(R.k, nBits), nBits);
            K160 newKey = k_add(k_shr(key, 160 - nBits), newStart);
            if (!in_succ_r(V, R, c, newKey)) {
                newKey = k_add(newKey, k_pow2(nBits));
                if (!in_succ_r(V, R, c, newKey)) return NONE;    // invalid start key
            }
            e.rk = newKey; e.step = step; e.has = 1;
        }
        if (in_succ_r(V, R, c, e.rk)) {
            if (e.step > 160) return NONE;
            if (160 - e.step - (V.sb - 1) < 0) return NONE;
            const uint32_t add = (uint32_t)((k_shr(key, 160 - e.step - V.sb + 1).w[0]) & ((1u << V.sb) - 1u));
            e.rk = k_add(k_shl(e.rk, V.sb), k_small(add));
            e.step += V.sb;
            if (dbNum > 0) {
                CodesReg BC;
                const KRec B = load_krec(V.rec, dbStart, BC);
                // rk in (db, dbStart]: db is dbStart's ring predecessor (k_koorde_build)
                if (in_pred_r(V, B, dbStart, e.rk)) {
                    h = db;
                } else {
                    // walkDeBruijnList (558-570) over dbStart's codes sum[0 .. dbNum-2]
                    const K160 dk = k_sub(e.rk, B.k);
                    if ((dk.w[0] | dk.w[1] | dk.w[2] | dk.w[3] | dk.w[4]) == 0 || dbNum <= 1) {
                        h = dbNum <= 1 ? dbStart : ring_add(dbStart, (uint32_t)(dbNum - 1), n);
                    } else {
                        bool tie = false;
                        const int cnt = count_codes(BC, 0, dbNum - 1, code32(dk), tie);
                        h = tie ? walk_list(V.recs, n, dbStart, dbNum, e.rk) : ring_add(dbStart, (uint32_t)cnt, n);
                    }
                }
            } else {
                h = db;
            }
        } else {
            brk = true;
            if (V.useSuc) {
                const uint32_t tmp = succ_walk(e.rk);
                h = between_open(rkey(V.recs, db), rkey(V.recs, tmp), e.rk) ? db : tmp;
            } else {
                h = s0;
            }
        }
        if (h != c || brk) return h;
    }
    return NONE;
}

// the records (after k_koorde_build)
__global__ void k_koorde_rec(const KeyRec* __restrict__ recs, const double2* __restrict__ xy,
                             const KoordeNode* __restrict__ nd, uint32_t n, KoordeRec* __restrict__ out)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const K160 me = rkey(recs, v);
    KoordeRec r;
    for (int i = 0; i < 5; ++i) r.w[i] = me.w[i];
    r.cP = code32(k_sub(me, rkey(recs, v == 0 ? n - 1 : v - 1)));
    const KoordeNode k = nd[v];
    r.db = k.db; r.dbStart = k.dbStart; r.dbNum = k.dbNum;
    r.pad0 = 0; r.pad1[0] = r.pad1[1] = 0;
    r.x = xy[v].x; r.y = xy[v].y;
    for (int j = 1; j <= KREC_LIST; ++j) r.sum[j - 1] = code32(k_sub(rkey(recs, (uint32_t)(((uint64_t)v + j) % n)), me));
    out[v] = r;
}

// handleDeBruijnTimerExpired (164-230) on the converged ring; the DeBruijnCall of the third
// case is answered by the node responsible for its key (328-367)
__global__ void k_koorde_build(const KeyRec* __restrict__ recs, uint32_t n, int ns, int sb, int dbls,
                               KoordeNode* __restrict__ nd)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const K160 me = rkey(recs, v);
    K160 lookup = k_shl(me, sb);
    if (ns > 0) lookup = k_sub(lookup, k_sub(rkey(recs, ring_add(v, 1 + (uint32_t)(ns / 2), n)), me));
    const uint32_t s0 = ring_add(v, 1, n), pred = v == 0 ? n - 1 : v - 1;
    KoordeNode o;
    o.pad = 0;
    if (ns == 0 || between_R(lookup, me, rkey(recs, s0))) {
        o.db = v; o.dbStart = s0; o.dbNum = (uint32_t)min(ns, dbls);
    } else if (between_R(lookup, rkey(recs, pred), me)) {
        const int sucNum = ns + 1 > dbls ? dbls - 1 : ns;
        o.db = pred; o.dbStart = v; o.dbNum = (uint32_t)(sucNum + 1);
    } else {
        // responsible(lookup): the first key >= lookup, wrapping to node 0
        uint32_t lo = 0, hi = n;
        while (lo < hi) {
            const uint32_t mid = lo + ((hi - lo) >> 1);
            if (k_lt(rkey(recs, mid), lookup)) lo = mid + 1; else hi = mid;
        }
        const uint32_t R = lo == n ? 0 : lo;
        o.db = R == 0 ? n - 1 : R - 1; o.dbStart = R; o.dbNum = (uint32_t)min(ns + 1, dbls);
    }
    nd[v] = o;
}

// visitOnlyOnce filter: one bit per node hash; a clear bit proves the node unvisited
__device__ __forceinline__ uint64_t vis_bit(uint32_t x) { return 1ull << ((x * 0x9E3779B1u) >> 26); }

#ifndef OVS_KOORDE_WAVES
#define OVS_KOORDE_WAVES 1
#endif
// the first KVL responders of a lookup whose hop sequence nobody asked for stay in LDS (the
// visitOnlyOnce list, read only when the filter bit is set): one dword per hop written to HBM had
// been 1.6 GB of scattered 32 B sectors per launch on config K, 17 % of its traffic
constexpr int KVL = 16;

// KR: the record form (KoordeRec), else the list walks on recs[].  RECORD: hopseq is the caller's
// hop sequence (every responder written); otherwise it is scratch for responders past the first
// KVL.  OVS_KOORDE_WAVES: minimum waves per SIMD the record form's register allocation must allow
// DEF: the default configuration (default.ini: successorListSize 16, shiftingBits 4, useOtherLookup
// and useSucList on, hopCountMax 50) as compile-time constants -- the start-key arithmetic's
// modulo by shiftingBits folds to a mask: 5963 -> 4931 static instructions
// the dynamic tail (as K1's, chord.hip): static slices cover [0, from), the rest goes out
// K3_DYN_CH lookups at a time from the zeroed per-launch counter *ctr (nullptr: static slices only)
struct KDyn {
    unsigned long long* ctr;
    uint64_t from;
};
#ifndef K3_DYN_CH
#define K3_DYN_CH 64
#endif
#ifndef K3_DYN_STATIC
#define K3_DYN_STATIC 0.70
#endif

template <bool KR, bool RECORD, bool DEF = false>
__global__ __launch_bounds__(256, KR ? OVS_KOORDE_WAVES : 1) void k_koorde_route(KView V0, const double2* __restrict__ xy, DelayConsts DC, int hcm0,
                                                      const K160* __restrict__ qkeys, const uint32_t* __restrict__ qsrc,
                                                      uint64_t nq, uint64_t chunk, KDyn dy, ovs_route_out* __restrict__ out,
                                                      uint32_t* __restrict__ hopseq, uint32_t* __restrict__ rpcs)
{
    const int lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    uint64_t cursor = wave * chunk;
    uint64_t end = min(cursor + chunk, dy.ctr ? dy.from : nq);
    bool more = dy.ctr != nullptr;                // dynamic chunks may be left
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    KView V = V0;
    if (DEF) { V.ns = 16; V.sb = 4; V.useOther = 1; V.useSuc = 1; }
    const int hcm = DEF ? 50 : hcm0;
    const uint64_t H = hcm > 0 ? (uint64_t)hcm : 1ull;

    bool active = false, local = true;
    uint64_t q = 0;
    K160 K;
    __shared__ uint4 rcodes[4][256];            // the responder record's codes, per lane (record form)
    CodesLds RC{rcodes, (int)threadIdx.x};
    __shared__ uint32_t vlist[RECORD ? 1 : KVL][256];   // the lane's first KVL responders (!RECORD)
    const int tid = (int)threadIdx.x;
    uint32_t S = 0, cur = 0;
    double sx = 0, sy = 0;
    int64_t t = 0;
    int hops = 0;
    uint64_t vis = 0;
    KExt e;
    e.has = 0; e.step = 1;
    while (true) {
        const uint64_t need = __ballot(!active);
        if (more && need != 0 && cursor >= end) {
            unsigned long long b = 0;
            if (lane == 0) b = atomicAdd(dy.ctr, (unsigned long long)K3_DYN_CH);
            const uint64_t nb = dy.from + (((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                                           (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)b));
            if (nb < nq) {
                cursor = nb;
                end = min(nb + (uint64_t)K3_DYN_CH, nq);
            } else {
                more = false;
            }
        }
        if (need != 0 && cursor < end) {
            const uint64_t mine = cursor + (uint64_t)__popcll(need & lt_mask);
            if (!active && mine < end) {
                q = mine;
                active = true;
                local = true;
                K = qkeys[q];
                S = qsrc[q];
                const double2 p = xy[S];
                sx = p.x; sy = p.y;
                t = 0; hops = 0;
                vis = vis_bit(S);
                // the local FindNodeCall gets a fresh extension (Koorde.cc:421-429)
                e.has = 0; e.step = 1;
            }
            cursor += (uint64_t)__popcll(need);
        }
        if (!__any(active)) break;
        if (!active) continue;

        uint32_t* seq = hopseq + q * H;
        uint8_t status = OVS_LOOKUP_OK;
        bool fin = false;
        uint32_t R = NONE;
        const uint32_t c = local ? S : cur;
        const uint32_t pred = c == 0 ? V.n - 1 : c - 1;
        // isSiblingFor(c, K, 1) (Chord.cc:452-457): K in (pred, c]
        KExt e2;
        bool sib;
        uint32_t nx;
        double cx, cy;
        if constexpr (KR) {
            // the extension advances in place: every outcome that does not take nx as the next
            // hop ends the lookup
            const KRec Rc = load_krec(V.rec, c, RC);
            sib = in_pred_r(V, Rc, c, K);
            nx = sib ? c : koorde_find_node_rec(V, c, Rc, RC, K, e);
            cx = Rc.x; cy = Rc.y;
            e2 = e;
        } else {
            e2 = e;
            sib = between_R(K, rkey(V.recs, pred), rkey(V.recs, c));
            nx = sib ? c : koorde_find_node_dev(V, c, K, e2);
            const double2 p = xy[c];
            cx = p.x; cy = p.y;
        }
        if (local) {
            // IterativeLookup::start (133-244)
            local = false;
            if (sib) { fin = true; R = S; }
            else if (nx == NONE) { fin = true; status = OVS_LOOKUP_BROKEN; }
            else if (nx == S) { fin = true; status = OVS_LOOKUP_NO_NEXT; }   // visited: nothing to send
            else { cur = nx; e = e2; }
        } else if (nx == NONE) {
            fin = true; status = OVS_LOOKUP_BROKEN;    // the responder's findNode throws
        } else {
            // FindNodeCall S -> c and its FindNodeResponse (one NodeHandle), both with the extension
            const int64_t cd = coord_ns(sx, sy, cx, cy, DC.round);
            const int64_t rtt = DC.msgCall + DC.msgResp1 + 2 * cd;
            if (rtt >= DC.rpcTimeout) {
                fin = true;
                status = (t + DC.rpcTimeout > DC.lookupTimeout) ? OVS_LOOKUP_TIMEOUT : OVS_LOOKUP_RPC_TIMEOUT;
            } else {
                t += rtt;
                if (t > DC.lookupTimeout) { fin = true; status = OVS_LOOKUP_TIMEOUT; }
                else {
                    if (hops < (int)H) {
                        if (RECORD || hops >= KVL) seq[hops] = c;
                        else vlist[RECORD ? 0 : hops][tid] = c;
                    }
                    ++hops;
                    vis |= vis_bit(c);
                    if (sib) { fin = true; R = c; }
                    else if (hcm && hops >= hcm) { fin = true; status = OVS_LOOKUP_HOPMAX; }
                    else {
                        // visitOnlyOnce: the next hop must not be the source or an earlier responder
                        // (the responder list is read only when the filter bit is set)
                        bool seen = nx == S;
                        if (!seen && (vis & vis_bit(nx)))
                            for (int i = 0; i < hops && !seen; ++i)
                                seen = (RECORD || i >= KVL ? seq[i] : vlist[RECORD ? 0 : i][tid]) == nx;
                        if (seen) { fin = true; status = OVS_LOOKUP_NO_NEXT; }
                        else { cur = nx; e = e2; }
                    }
                }
            }
        }
        if (fin) {
            ovs_route_out o;
            o.hops = (uint16_t)hops;
            o.status = status;
            if (status == OVS_LOOKUP_OK) {
                o.responsible = R;
                o.one_way_hops = (uint8_t)(hops + (R != S ? 1 : 0));
                int64_t lat = t;
                if (R != S) {
                    // sendRouteMessage to the result (BaseOverlay.cc:1107-1146): R is this iteration's c
                    lat += DC.msgRoute + coord_ns(sx, sy, cx, cy, DC.round);
                }
                o.latency_ns = lat;
            } else {
                o.responsible = NONE;
                o.one_way_hops = 0;
                o.latency_ns = -1;
            }
            out[q] = o;
            // FindNodeCalls sent: one per accepted responder, plus a call to c whose response did
            // not count (its findNode threw, it timed out, or it came after the lookup timeout)
            const bool lost = c != S && (status == OVS_LOOKUP_BROKEN || status == OVS_LOOKUP_RPC_TIMEOUT ||
                                         status == OVS_LOOKUP_TIMEOUT);
            if (rpcs) rpcs[q] = (uint32_t)hops + (lost ? 1u : 0u);
            active = false;
        }
    }
}

template <bool KR>
__global__ void k_koorde_find_node(KView V, const uint32_t* __restrict__ node, const K160* __restrict__ keys,
                                   KExt* __restrict__ ext, uint32_t* __restrict__ next, uint64_t nq)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nq) return;
    KExt e = ext[i];
    const uint32_t c = node[i];
    uint32_t h;
    if constexpr (KR) {
        __shared__ uint4 rcodes[4][256];      // 128-thread blocks use the first half of each row
        CodesLds RC{rcodes, (int)threadIdx.x};
        const KRec R = load_krec(V.rec, c, RC);
        h = koorde_find_node_rec(V, c, R, RC, keys[i], e);
    }
    else h = koorde_find_node_dev(V, c, keys[i], e);
    next[i] = h;
    if (h != NONE) ext[i] = e;
}

inline unsigned nblk(uint64_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

KView make_view(const KoordeTables& t, const KeyRec* recs)
{
    KView V;
    V.recs = recs; V.nd = t.nd; V.rec = t.rec; V.n = t.n; V.ns = t.ns; V.sb = t.sb; V.useOther = t.useOther; V.useSuc = t.useSuc;
    return V;
}

}  // namespace

hipError_t koorde_build(const KeyRec* recs, const double2* xy, uint32_t n, int successorListSize, int shiftingBits,
                        int deBruijnListSize, int useOtherLookup, int useSucList, KoordeTables& t, hipStream_t st)
{
    koorde_free(t);
    if (n < 2 || shiftingBits < 1 || shiftingBits > 32 || deBruijnListSize < 1) return hipErrorInvalidValue;
    t.n = n;
    t.ns = (int)std::min<uint64_t>((uint64_t)successorListSize, (uint64_t)n - 1);
    t.sb = shiftingBits; t.dbls = deBruijnListSize; t.useOther = useOtherLookup; t.useSuc = useSucList;
    hipError_t e = hipMalloc(&t.nd, sizeof(KoordeNode) * n);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_koorde_build, dim3(nblk(n, 256)), dim3(256), 0, st, recs, n, t.ns, shiftingBits,
                       deBruijnListSize, t.nd);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    // the record form covers successor / de Bruijn lists of up to 16 nodes (the Koorde defaults)
#ifdef OVS_KOORDE_NOREC
    const bool rec_form = false;      // diagnostic build: the list form only
#else
    const bool rec_form = true;
#endif
    if (rec_form && t.ns <= KREC_LIST && deBruijnListSize <= KREC_LIST) {
        e = hipMalloc(&t.rec, sizeof(KoordeRec) * n);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_koorde_rec, dim3(nblk(n, 256)), dim3(256), 0, st, recs, xy, t.nd, n, t.rec);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipStreamSynchronize(st);
}

hipError_t koorde_route(const KoordeTables& t, const KeyRec* recs, const double2* xy, const DelayConsts& DC,
                        int hopCountMax, const K160* keys, const uint32_t* src, uint64_t nq, ovs_route_out* out,
                        uint32_t* hopseq, bool record, uint32_t* rpcs, int num_cu, hipStream_t st,
                        unsigned long long* dyn)
{
    // a grid of `waves` persistent waves: static slices, with the dynamic tail when dyn is given
    auto slices = [&](uint64_t waves, uint64_t* chunk, uint64_t* blocks, KDyn* dy) {
        uint64_t c = (nq + waves - 1) / waves;
        if (c < 1) c = 1;
        *blocks = ((nq + c - 1) / c + 3) / 4;
        dy->ctr = nullptr;
        dy->from = nq;
        const uint64_t cs = dyn ? (uint64_t)((double)nq * K3_DYN_STATIC) / (*blocks * 4) : 0;
        if (cs >= (uint64_t)K3_DYN_CH) {
            c = cs;
            dy->ctr = dyn;
            dy->from = cs * *blocks * 4;
        }
        *chunk = c;
    };
    if (nq == 0) return hipSuccess;
    if (!hopseq) return hipErrorInvalidValue;
    static int bpc[4] = {0, 0, 0, 0};
    const int kr = t.rec ? 1 : 0;
    const int ki = kr + (record ? 2 : 0);
#define KRT(a, b) k_koorde_route<a, b>
    if (bpc[ki] == 0) {
        int b = 0;
        const hipError_t oe =
            kr ? (record ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, KRT(true, true), 256, 0)
                         : hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, KRT(true, false), 256, 0))
               : (record ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, KRT(false, true), 256, 0)
                         : hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, KRT(false, false), 256, 0));
        bpc[ki] = (oe == hipSuccess && b > 0) ? b : 1;
    }
    const uint64_t waves = (uint64_t)num_cu * (uint64_t)bpc[ki] * 4;
    uint64_t chunk = 0, blocks = 0;
    KDyn dy;
    slices(waves, &chunk, &blocks, &dy);
#define KRL(a, b) hipLaunchKernelGGL((KRT(a, b)), dim3((unsigned)blocks), dim3(256), 0, st, make_view(t, recs), xy, DC, \
                                     hopCountMax, keys, src, nq, chunk, dy, out, hopseq, rpcs)
    const KView kv = make_view(t, recs);
#ifdef OVS_KOORDE_NO_DEF
    const bool def = false;             // A/B build: the generic instantiation
#else
    const bool def = kr && !record && kv.ns == 16 && kv.sb == 4 && kv.useOther == 1 && kv.useSuc == 1 && hopCountMax == 50;
#endif
    if (def) {
        static int bpd = 0;
        if (bpd == 0) {
            int b = 0;
            bpd = (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_koorde_route<true, false, true>, 256, 0) == hipSuccess && b > 0) ? b : 1;
        }
        const uint64_t wd = (uint64_t)num_cu * (uint64_t)bpd * 4;
        uint64_t cd = 0, bd = 0;
        KDyn dd;
        slices(wd, &cd, &bd, &dd);
        hipLaunchKernelGGL((k_koorde_route<true, false, true>), dim3((unsigned)bd), dim3(256), 0, st, kv, xy, DC, hopCountMax, keys,
                           src, nq, cd, dd, out, hopseq, rpcs);
    } else if (kr) { if (record) KRL(true, true); else KRL(true, false); }
    else { if (record) KRL(false, true); else KRL(false, false); }
#undef KRL
#undef KRT
    return hipGetLastError();
}

hipError_t koorde_find_node(const KoordeTables& t, const KeyRec* recs, const uint32_t* node, const K160* keys,
                            KExt* ext, uint32_t* next, uint64_t nq, hipStream_t st)
{
    if (nq == 0) return hipSuccess;
    if (t.rec)
        hipLaunchKernelGGL(k_koorde_find_node<true>, dim3(nblk(nq, 128)), dim3(128), 0, st, make_view(t, recs), node, keys,
                           ext, next, nq);
    else
        hipLaunchKernelGGL(k_koorde_find_node<false>, dim3(nblk(nq, 128)), dim3(128), 0, st, make_view(t, recs), node,
                           keys, ext, next, nq);
    return hipGetLastError();
}

}  // namespace ovs
