// chord.hip -- Chord iterative-lookup kernels for gfx950 (MI355X).
//
// K1 chord_route: one lane per in-flight lookup, the whole lookup runs in
// registers (no per-round state round trip through HBM); a wave refills its
// finished lanes from its own contiguous slice of the batch (ballot + popcount
// prefix, no atomics), so all 64 lanes stay busy until the slice drains.
// Per hop the lane evaluates the responder's Chord::findNode + isSiblingFor
// (Chord.cc:422-500, 548-674) and charges the SimpleUnderlay delay
// (SimpleNodeEntry.cc:145-195) in exact int64 ns.
//
// Memory per hop (ideal tables): the responder's ring window (pred, succ0,
// succ[ns-1], 24 B records), its coordinates, one finger-row word and the
// finger's record -- two dependent gather rounds.  Nothing here is a dense
// contraction, so there is no MFMA; the kernel is HBM/Infinity-Cache gather
// bound.
#include <hipcub/hipcub.hpp>

#include "engine.hpp"
#include "launch.hpp"

namespace ovs {

// ---------------------------------------------------------------------------
// table builder (ideal NoChurn state, Chord.cc:845-875 fixed point)

__global__ void k_check_sorted(const KeyRec* __restrict__ recs, uint32_t n, uint32_t* bad)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i + 1 < n) {
        const K160 a = key_of(load_rec(recs, i)), b = key_of(load_rec(recs, i + 1));
        if (!k_lt(a, b)) atomicOr(bad, 1u);
    }
}

// row length = number of non-trivial fingers: i with 2^i > succ0 - self
__global__ void k_chord_rowlen(const KeyRec* __restrict__ recs, uint32_t n, uint32_t lo, uint32_t cnt, uint64_t* rowlen)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= cnt) return;
    const uint32_t v = lo + t;
    const K160 self = key_of(load_rec(recs, v));
    const K160 s0 = key_of(load_rec(recs, v + 1 == n ? 0 : v + 1));
    const int ilo = k_msb(k_sub(s0, self)) + 1;
    rowlen[t] = (uint64_t)(KEYBITS - ilo);
}

__global__ void k_set_aux(KeyRec* recs, const uint64_t* off, uint32_t lo, uint32_t cnt)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < cnt) recs[lo + t].aux = (uint32_t)off[t];
}

// first index with key >= target, wrapping to 0 (the responsible node)
__device__ __forceinline__ uint32_t ring_lower_bound(const KeyRec* __restrict__ recs, uint32_t n,
                                                     const K160& t)
{
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = lo + ((hi - lo) >> 1);
        if (k_lt(key_of(load_rec(recs, mid)), t)) lo = mid + 1; else hi = mid;
    }
    return lo == n ? 0 : lo;
}

// finger i of node v = responsible(v + 2^i) (rpcFixfingers answers thisNode, Chord.cc:1228-1270)
__global__ void k_chord_fill(const KeyRec* __restrict__ recs, uint32_t n, uint32_t lo, uint32_t cnt,
                             uint2* __restrict__ fingers)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= cnt) return;
    const uint32_t v = lo + t;
    const KeyRec r = load_rec(recs, v);
    const K160 self = key_of(r);
    const K160 s0 = key_of(load_rec(recs, v + 1 == n ? 0 : v + 1));
    const int ilo = k_msb(k_sub(s0, self)) + 1;
    uint2* row = fingers + r.aux;
    for (int i = KEYBITS - 1; i >= ilo; --i) {
        const uint32_t f = ring_lower_bound(recs, n, k_add(self, k_pow2(i)));
        // entry = {finger, code32 of its distance from v} (decide_compact's finger test)
        row[KEYBITS - 1 - i] = make_uint2(f, (uint32_t)(k_code64(k_sub(key_of(load_rec(recs, f)), self)) >> 32));
    }
}

// NodeRec of every node (ideal ring): key, finger-row offset, coordinates, window codes
__global__ void k_chord_nodes(const KeyRec* __restrict__ recs, const double2* __restrict__ xy, uint32_t n, int ns,
                              NodeRec* __restrict__ nodes)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const KeyRec r = load_rec(recs, v);
    const K160 C = key_of(r);
    const K160 P = key_of(load_rec(recs, v == 0 ? n - 1 : v - 1));
    const K160 S0 = key_of(load_rec(recs, v + 1 == n ? 0 : v + 1));
    const uint32_t sl = v + (uint32_t)ns >= n ? v + (uint32_t)ns - n : v + (uint32_t)ns;
    const K160 SL = key_of(load_rec(recs, sl));
    const double2 p = xy[v];
    const uint64_t cP = k_code64(k_sub(P, C)), cS0 = k_code64(k_sub(S0, C)), cSL = k_code64(k_sub(SL, C));
    uint4* o = reinterpret_cast<uint4*>(nodes + v);
    o[0] = make_uint4(r.w[0], r.w[1], r.w[2], r.w[3]);
    o[1] = make_uint4(r.w[4], r.aux, (uint32_t)__double2loint(p.x), (uint32_t)__double2hiint(p.x));
    o[2] = make_uint4((uint32_t)__double2loint(p.y), (uint32_t)__double2hiint(p.y), (uint32_t)cP, (uint32_t)(cP >> 32));
    o[3] = make_uint4((uint32_t)cS0, (uint32_t)(cS0 >> 32), (uint32_t)cSL, (uint32_t)(cSL >> 32));
}

// resolved getFinger(pos) for every position (test export)
__global__ void k_chord_export(const KeyRec* __restrict__ recs, const uint2* __restrict__ fingers,
                               uint32_t n, uint32_t* __restrict__ out)
{
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)n * KEYBITS) return;
    const uint32_t v = (uint32_t)(t / KEYBITS);
    const int pos = (int)(t % KEYBITS);
    const KeyRec r = load_rec(recs, v);
    const uint32_t s0i = v + 1 == n ? 0 : v + 1;
    const int ilo = k_msb(k_sub(key_of(load_rec(recs, s0i)), key_of(r))) + 1;
    out[t] = pos >= ilo ? fingers[r.aux + (KEYBITS - 1 - pos)].x : s0i;
}

// ---------------------------------------------------------------------------
// findNode + isSiblingFor at responder c for key K (numRedundantNodes = 1,
// numSiblings = 1): the per-hop routing decision.

struct Decision {
    uint32_t next;   // next hop (== c when c is responsible)
    KeyRec rec;      // its record
    uint8_t sib;     // siblings flag of the FindNodeResponse
    uint8_t broken;  // Chord::closestPreceedingNode threw
};

__device__ __forceinline__ uint32_t ring_next(uint32_t i, uint32_t d, uint32_t n)
{
    uint32_t j = i + d;
    return j >= n ? j - n : j;
}

// Ideal tables, compact layout (NodeRec + coded finger rows).  Successor j of c
// is c+1+j, the predecessor c-1.  Every ring test is taken relative to c with
// D = K - c: each interval of Chord.cc:452-457, 583-590, 602-674 becomes a
// compare of D against a distance from c, decided on the order-preserving codes
// stored in the node record and the finger rows; an equal code (a tie at the
// code's precision, e.g. a node-ID key) falls back to the exact keys in recs[].
struct Hop {
    uint32_t next;   // next hop (== c when c is responsible), NONE when broken
    uint8_t sib;     // siblings flag of the FindNodeResponse
    uint8_t broken;  // Chord::closestPreceedingNode threw
};

__device__ __forceinline__ Hop decide_compact(const ChordView& V, uint32_t c, const NodeRec& R, const K160& K)
{
    Hop h;
    h.sib = 0; h.broken = 0; h.next = NONE;
    const K160 C = key_of_node(R);
    const K160 D = k_sub(K, C);
    const int i0 = k_msb(D);                     // -1 only when K == C
    // finger entry i0, issued before anything that depends on it (rows are padded by 160 entries)
    const uint2 f0 = V.frow[R.row + (uint32_t)(KEYBITS - 1 - (i0 < 0 ? KEYBITS - 1 : i0))];
    if (i0 < 0) { h.sib = 1; h.next = c; return h; }
    const uint64_t cD = k_code64(D);
    // isSiblingFor(thisNode, key, 1): K in (pred, C]  <=>  D > pred - C  (Chord.cc:452-457)
    bool t;
    if (cD != R.cP) t = cD > R.cP;
    else t = between_R(K, key_of(load_rec(V.recs, c == 0 ? V.n - 1 : c - 1)), C);
    if (t) { h.sib = 1; h.next = c; return h; }
    // K in (C, succ0]  <=>  D <= succ0 - C  (Chord.cc:583-590)
    const uint32_t s0 = ring_next(c, 1, V.n);
    if (cD != R.cS0) t = cD < R.cS0;
    else t = between_R(K, C, key_of(load_rec(V.recs, s0)));
    if (t) { h.next = s0; return h; }
    // closestPreceedingNode (Chord.cc:602-674): temp = farthest successor in (C, K]
    int tj;
    uint32_t cT;                 // code32 of temp - C
    bool tIsK = false, gTexact = false;
    K160 gT;
    if (cD > R.cSL) {
        tj = V.ns - 1;
        cT = (uint32_t)(R.cSL >> 32);
    } else {
        tj = -1;
        for (int j = V.ns - 1; j >= 0; --j) {
            const K160 SJ = key_of(load_rec(V.recs, ring_next(c, (uint32_t)j + 1, V.n)));
            if (between_R(SJ, C, K)) { tj = j; gT = k_sub(SJ, C); tIsK = k_eq(SJ, K); break; }
        }
        if (tj < 0) { h.broken = 1; return h; }
        gTexact = true;
        cT = (uint32_t)(k_code64(gT) >> 32);
    }
    // finger scan from i0 down (fingers above i0 lie beyond the key):
    // finger F in [temp, K]  <=>  temp - C <= F - C <= D
    const uint32_t cD32 = (uint32_t)(cD >> 32);
    const int ilo = (int)(R.cS0 >> 56);
    for (int i = i0; i >= ilo; --i) {
        const uint2 e = (i == i0) ? f0 : V.frow[R.row + (uint32_t)(KEYBITS - 1 - i)];
        bool hit;
        if (e.y != cD32 && e.y != cT) {
            hit = (e.y < cD32) & (e.y > cT);
        } else {
            const K160 dF = k_sub(key_of(load_rec(V.recs, e.x)), C);
            if (!gTexact) {
                gT = k_sub(key_of(load_rec(V.recs, ring_next(c, (uint32_t)V.ns, V.n))), C);
                gTexact = true;
            }
            hit = k_le(gT, dF) & k_le(dF, D);
        }
        if (hit) { h.next = e.x; return h; }
    }
    // trivial positions resolve to succ0 (ChordFingerTable.cc:183-184); succ0 lies in
    // [temp, K] only when temp is succ0
    if (tj == 0) { h.next = s0; return h; }
    // no finger: farthest successor in the OPEN interval (C, K) (Chord.cc:653-658) --
    // temp itself unless temp == K
    const int j = tIsK ? tj - 1 : tj;
    h.next = ring_next(c, (uint32_t)j + 1, V.n);
    return h;
}

// general (explicit snapshot) tables: literal restatement incl. unspecified predecessor
__device__ __forceinline__ bool sibling_general(const ChordView& V, uint32_t self, const K160& K,
                                                int numSiblings)
{
    const uint32_t pred = V.pred[self];
    const int ssize = V.nsucc[self];
    const K160 C = key_of(load_rec(V.recs, self));
    if (pred == NONE) {
        const bool isEmpty = ssize == 0 || (ssize == 1 && V.succ[(uint64_t)self * V.sls] == self);
        return isEmpty || k_eq(C, K);
    }
    const K160 PK = key_of(load_rec(V.recs, pred));
    if (between_R(K, PK, C)) return true;
    // loop of Chord.cc:462-495 with node == thisNode matches at i = -1 only
    (void)numSiblings;
    return false;
}

__device__ __forceinline__ Decision decide_general(const ChordView& V, uint32_t c, const KeyRec& crec,
                                                   const K160& K)
{
    Decision d;
    d.broken = 0; d.sib = 0;
    const K160 C = key_of(crec);
    const uint64_t sb = (uint64_t)c * V.sls;
    const int ssize = V.nsucc[c];
    if (sibling_general(V, c, K, 1)) { d.sib = 1; d.next = c; d.rec = crec; return d; }
    const uint32_t s0 = V.succ[sb];
    const KeyRec S0 = load_rec(V.recs, s0);
    if (between_R(K, C, key_of(S0))) { d.next = s0; d.rec = S0; return d; }
    int tj = -1;
    K160 T;
    for (int j = ssize - 1; j >= 0; --j) {
        const K160 SJ = key_of(load_rec(V.recs, V.succ[sb + j]));
        if (between_R(SJ, C, K)) { tj = j; T = SJ; break; }
    }
    if (tj < 0) { d.broken = 1; d.next = NONE; return d; }
    for (int i = KEYBITS - 1; i >= 0; --i) {
        const uint32_t f = V.fres[(uint64_t)c * KEYBITS + i];
        const KeyRec F = load_rec(V.recs, f);
        if (between_LR(key_of(F), T, K)) { d.next = f; d.rec = F; return d; }
    }
    for (int j = ssize - 1; j >= 0; --j) {
        const uint32_t sj = V.succ[sb + j];
        const KeyRec SJ = load_rec(V.recs, sj);
        if (between_open(key_of(SJ), C, K)) { d.next = sj; d.rec = SJ; return d; }
    }
    if (V.pred[c] == NONE && s0 == c) { d.next = c; d.rec = crec; return d; }
    d.broken = 1; d.next = NONE;
    return d;
}

// ---------------------------------------------------------------------------
// K1: batched one-way lookups

// Responder state carried in registers between hops.  Ideal rings: the 64 B
// NodeRec of the current responder (key, finger-row offset, coordinates, window
// codes); explicit tables: its 24 B KeyRec (coordinates gathered per hop).
template <bool IDEAL> struct Responder;
template <> struct Responder<true> {
    NodeRec n;
    __device__ __forceinline__ void load(const ChordView& V, uint32_t c) { n = load_node(V.nodes, c); }
    __device__ __forceinline__ double2 xy(const ChordView&, uint32_t) const { return make_double2(n.x, n.y); }
    __device__ __forceinline__ Hop decide(const ChordView& V, uint32_t c, const K160& K) const
    {
        return decide_compact(V, c, n, K);
    }
    __device__ __forceinline__ void advance(const ChordView& V, const Hop& h) { load(V, h.next); }
};
template <> struct Responder<false> {
    KeyRec r;
    KeyRec nxt;
    __device__ __forceinline__ void load(const ChordView& V, uint32_t c) { r = load_rec(V.recs, c); }
    __device__ __forceinline__ double2 xy(const ChordView& V, uint32_t c) const { return V.xy[c]; }
    __device__ __forceinline__ Hop decide(const ChordView& V, uint32_t c, const K160& K)
    {
        const Decision d = decide_general(V, c, r, K);
        nxt = d.rec;
        Hop h;
        h.next = d.next; h.sib = d.sib; h.broken = d.broken;
        return h;
    }
    __device__ __forceinline__ void advance(const ChordView&, const Hop&) { r = nxt; }
};

template <bool IDEAL, bool RECORD, bool REC>
__global__ __launch_bounds__(256) void k_chord_route(ChordView V, DelayConsts DC, LookupConsts LC,
                                                     const K160* __restrict__ qkeys,
                                                     const uint32_t* __restrict__ qsrc, uint64_t nq,
                                                     uint64_t chunk, ovs_route_out* __restrict__ out,
                                                     uint32_t* __restrict__ hopseq)
{
    const int lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    uint64_t cursor = wave * chunk;                       // wave-uniform
    const uint64_t end = min(cursor + chunk, nq);
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

    bool active = false;
    uint64_t q = 0;
    uint32_t S = 0, cur = 0;
    K160 K;
    Responder<IDEAL> rs;
    double sx = 0, sy = 0;
    int64_t t = 0;
    int hops = 0;
    bool local = true;

    while (true) {
        const uint64_t need = __ballot(!active);
        if (need != 0 && cursor < end) {
            const uint64_t mine = cursor + (uint64_t)__popcll(need & lt_mask);
            if (!active && mine < end) {
                q = mine;
                active = true;
                K = qkeys[q];
                S = qsrc[q];
                rs.load(V, S);
                const double2 sxy = rs.xy(V, S);
                sx = sxy.x; sy = sxy.y;
                cur = S; t = 0; hops = 0; local = true;
            }
            cursor += (uint64_t)__popcll(need);
        }
        if (!__any(active)) break;
        if (!active) continue;

        const double2 cxy = rs.xy(V, cur);
        const Hop d = rs.decide(V, cur, K);

        uint8_t status = 0xFF;   // 0xFF = still running
        uint32_t R = NONE;
        if (REC) {
            // Recursive one-way route message (BaseOverlay::sendToKey recursive branch,
            // BaseOverlay.cc:1445-1582; receipt 907-914).  (sx, sy) = the last sender.
            const bool at_src = local;
            if (!local) t += DC.msgRoute + coord_ns(sx, sy, cxy.x, cxy.y, DC.round);   // sendRouteMessage
            local = false;
            sx = cxy.x; sy = cxy.y;
            // a forwarded message is delivered on receipt (907-914); at the source sendToKey's
            // hop-count check precedes the delivery to itself (1464 before 1555)
            if (d.sib && (!at_src || hops < LC.hopCountMax)) { status = OVS_LOOKUP_OK; R = cur; }
            else if (d.sib) status = OVS_LOOKUP_HOPMAX;
            else if (d.broken) status = OVS_LOOKUP_BROKEN;
            else if (hops >= LC.hopCountMax) status = OVS_LOOKUP_HOPMAX;               // 1464-1488
            else if (d.next == S || d.next == cur) {
                // loop detection (1502-1516) rejects findNode's first candidate: on a converged
                // ring this cannot happen (every hop moves strictly towards the key), and the
                // recursive path is only enabled for converged rings
                status = OVS_LOOKUP_NO_NEXT;
            } else {
                if (RECORD && hops < LC.hopCountMax) hopseq[q * (uint64_t)LC.hopCountMax + hops] = d.next;
                ++hops;
                cur = d.next;
                rs.advance(V, d);
            }
            if (status != 0xFF) {
                ovs_route_out o;
                o.hops = (uint16_t)(status == OVS_LOOKUP_OK ? hops : 0);
                o.status = status;
                o.responsible = R;
                o.one_way_hops = (uint8_t)(status == OVS_LOOKUP_OK ? hops : 0);
                o.latency_ns = status == OVS_LOOKUP_OK ? t : -1;
                out[q] = o;
                active = false;
            }
            continue;
        }
        if (local) {
            // IterativeLookup::start (IterativeLookup.cc:157-204): local step, no hop, no delay
            local = false;
            if (d.broken) status = OVS_LOOKUP_BROKEN;
            else if (d.sib) { status = OVS_LOOKUP_OK; R = S; }
        } else {
            // FindNodeCall S->cur, FindNodeResponse cur->S (one NodeHandle)
            const int64_t cd = coord_ns(sx, sy, cxy.x, cxy.y, DC.round);
            const int64_t rtt = DC.msgCall + DC.msgResp1 + 2 * cd;
            if (rtt >= DC.rpcTimeout) {
                status = (t + DC.rpcTimeout > DC.lookupTimeout) ? OVS_LOOKUP_TIMEOUT : OVS_LOOKUP_RPC_TIMEOUT;
            } else {
                t += rtt;
                if (t > DC.lookupTimeout) status = OVS_LOOKUP_TIMEOUT;   // IterativeLookup.cc:808-815
                else {
                    if (RECORD && hops < LC.hopCountMax) hopseq[q * (uint64_t)LC.hopCountMax + hops] = cur;
                    ++hops;
                    if (d.broken) status = OVS_LOOKUP_BROKEN;
                    else if (d.sib) { status = OVS_LOOKUP_OK; R = cur; }  // IterativeLookup.cc:896-905
                }
            }
        }
        if (status == 0xFF) {
            // IterativePathLookup::sendRpc (IterativeLookup.cc:1067-1170)
            if (LC.hopCountMax && hops >= LC.hopCountMax) status = OVS_LOOKUP_HOPMAX;
            else {
                bool visited = (d.next == S);
                if (!IDEAL && !visited) {
                    // explicit tables can loop: check every responder so far
                    for (int h = 0; h < hops && h < LC.hopCountMax; ++h)
                        visited |= hopseq[q * (uint64_t)LC.hopCountMax + h] == d.next;
                }
                if (visited) status = OVS_LOOKUP_NO_NEXT;
                else { cur = d.next; rs.advance(V, d); }
            }
        }
        if (status != 0xFF) {
            ovs_route_out o;
            o.hops = (uint16_t)hops;
            o.status = status;
            if (status == OVS_LOOKUP_OK) {
                o.responsible = R;
                o.one_way_hops = (uint8_t)(hops + (R != S ? 1 : 0));
                // sendRouteMessage to result[0] (BaseOverlay.cc:1107-1146); 0 delay to self
                o.latency_ns = t + (R != S ? DC.msgRoute + coord_ns(sx, sy, cxy.x, cxy.y, DC.round) : 0);
            } else {
                o.responsible = NONE;
                o.one_way_hops = 0;
                o.latency_ns = -1;
            }
            out[q] = o;
            active = false;
        }
    }
}

// ---------------------------------------------------------------------------
// multi-GPU: one hop round over in-flight records (ovs_shard_step)

// owner rank of node c: r with lo[r] <= c < lo[r+1] (uniform trip count, no divergent loop)
__device__ __forceinline__ int shard_owner(const uint64_t* __restrict__ lo, int nsh, uint32_t c)
{
    int r = 0;
    for (int i = 1; i < nsh; ++i) r += ((uint64_t)c >= lo[i]) ? 1 : 0;
    return r;
}

__device__ __forceinline__ ovs_lookup_rec load_lrec(const ovs_lookup_rec* __restrict__ p, uint64_t i)
{
    const uint4* q = reinterpret_cast<const uint4*>(p + i);
    const uint4 a = q[0], b = q[1], c = q[2];
    ovs_lookup_rec r;
    r.key[0] = a.x; r.key[1] = a.y; r.key[2] = a.z; r.key[3] = a.w; r.key[4] = b.x;
    r.src = b.y; r.cur = b.z; r.qid = b.w;
    r.t_ns = (int64_t)((uint64_t)c.x | ((uint64_t)c.y << 32));
    r.hops = (uint16_t)(c.z & 0xFFFF);
    r.local = (uint8_t)((c.z >> 16) & 0xFF);
    return r;
}

__device__ __forceinline__ void store_lrec(ovs_lookup_rec* __restrict__ p, uint64_t i, const K160& K, uint32_t S,
                                           uint32_t cur, uint32_t qid, int64_t t, int hops, int local)
{
    uint4* q = reinterpret_cast<uint4*>(p + i);
    q[0] = make_uint4(K.w[0], K.w[1], K.w[2], K.w[3]);
    q[1] = make_uint4(K.w[4], S, cur, qid);
    q[2] = make_uint4((uint32_t)(uint64_t)t, (uint32_t)((uint64_t)t >> 32), (uint32_t)hops | ((uint32_t)local << 16), 0u);
}

template <bool REC>
__global__ __launch_bounds__(256) void k_chord_shard_step(ChordView V, DelayConsts DC, LookupConsts LC,
                                                          const uint64_t* __restrict__ shard_lo, int nsh, int me, const ovs_lookup_rec* __restrict__ in, uint64_t nin,
                                                          uint64_t chunk, ovs_lookup_rec* __restrict__ out,
                                                          uint32_t* __restrict__ out_dest, uint64_t out_cap,
                                                          unsigned long long* out_count, ovs_done_rec* __restrict__ done,
                                                          uint64_t done_cap, unsigned long long* done_count)
{
    const int lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    uint64_t cursor = wave * chunk;
    const uint64_t end = min(cursor + chunk, nin);
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

    bool active = false;
    uint32_t S = 0, cur = 0, qid = 0;
    K160 K;
    NodeRec cn;
    double sx = 0, sy = 0;
    int64_t t = 0;
    int hops = 0;
    bool local = false;

    while (true) {
        const uint64_t need = __ballot(!active);
        if (need != 0 && cursor < end) {
            const uint64_t mine = cursor + (uint64_t)__popcll(need & lt_mask);
            if (!active && mine < end) {
                const ovs_lookup_rec r = load_lrec(in, mine);
                active = true;
                for (int w = 0; w < 5; ++w) K.w[w] = r.key[w];
                S = r.src; cur = r.cur; qid = r.qid; t = r.t_ns; hops = r.hops; local = r.local != 0;
                cn = load_node(V.nodes, cur);
                const double2 sxy = V.xy[S];     // source coordinates (replicated on every rank)
                sx = sxy.x; sy = sxy.y;
            }
            cursor += (uint64_t)__popcll(need);
        }
        if (!__any(active)) break;

        bool emit_done = false, emit_out = false;
        int dest = 0;
        ovs_route_out o;
        if (active) {
            const double2 cxy = make_double2(cn.x, cn.y);
            const Hop d = decide_compact(V, cur, cn, K);
            uint8_t status = 0xFF;
            uint32_t R = NONE;
            if (REC) {
                // recursive route message (same rules as k_chord_route<.., REC>); the hop's
                // delay was charged when the message was sent
                const bool at_src = local;
                local = false;
                if (d.sib && (!at_src || hops < LC.hopCountMax)) { status = OVS_LOOKUP_OK; R = cur; }
                else if (d.sib) status = OVS_LOOKUP_HOPMAX;
                else if (d.broken) status = OVS_LOOKUP_BROKEN;
                else if (hops >= LC.hopCountMax) status = OVS_LOOKUP_HOPMAX;
                else if (d.next == S || d.next == cur) status = OVS_LOOKUP_NO_NEXT;
                else {
                    const double2 nxy = V.xy[d.next];   // coordinates are replicated on every rank
                    t += DC.msgRoute + coord_ns(cxy.x, cxy.y, nxy.x, nxy.y, DC.round);
                    ++hops;
                    cur = d.next;
                    dest = shard_owner(shard_lo, nsh, cur);
                    if (dest != me) { emit_out = true; active = false; }
                    else cn = load_node(V.nodes, cur);
                }
                if (status != 0xFF) {
                    o.hops = (uint16_t)(status == OVS_LOOKUP_OK ? hops : 0);
                    o.status = status;
                    o.responsible = R;
                    o.one_way_hops = (uint8_t)(status == OVS_LOOKUP_OK ? hops : 0);
                    o.latency_ns = status == OVS_LOOKUP_OK ? t : -1;
                    emit_done = true;
                    active = false;
                }
            } else if (local) {
                local = false;
                if (d.broken) status = OVS_LOOKUP_BROKEN;
                else if (d.sib) { status = OVS_LOOKUP_OK; R = S; }
            } else {
                const int64_t cd = coord_ns(sx, sy, cxy.x, cxy.y, DC.round);
                const int64_t rtt = DC.msgCall + DC.msgResp1 + 2 * cd;
                if (rtt >= DC.rpcTimeout) {
                    status = (t + DC.rpcTimeout > DC.lookupTimeout) ? OVS_LOOKUP_TIMEOUT : OVS_LOOKUP_RPC_TIMEOUT;
                } else {
                    t += rtt;
                    if (t > DC.lookupTimeout) status = OVS_LOOKUP_TIMEOUT;
                    else {
                        ++hops;
                        if (d.broken) status = OVS_LOOKUP_BROKEN;
                        else if (d.sib) { status = OVS_LOOKUP_OK; R = cur; }
                    }
                }
            }
            if (!REC && status == 0xFF) {
                if (LC.hopCountMax && hops >= LC.hopCountMax) status = OVS_LOOKUP_HOPMAX;
                else if (d.next == S) status = OVS_LOOKUP_NO_NEXT;
                else {
                    cur = d.next;
                    dest = shard_owner(shard_lo, nsh, cur);
                    if (dest != me) { emit_out = true; active = false; }
                    else cn = load_node(V.nodes, cur);
                }
            }
            if (!REC && status != 0xFF) {
                o.hops = (uint16_t)hops;
                o.status = status;
                if (status == OVS_LOOKUP_OK) {
                    o.responsible = R;
                    o.one_way_hops = (uint8_t)(hops + (R != S ? 1 : 0));
                    o.latency_ns = t + (R != S ? DC.msgRoute + coord_ns(sx, sy, cxy.x, cxy.y, DC.round) : 0);
                } else {
                    o.responsible = NONE;
                    o.one_way_hops = 0;
                    o.latency_ns = -1;
                }
                emit_done = true;
                active = false;
            }
        }
        // append (hipcc turns these per-lane adds into one wave-level atomic per counter)
        if (emit_done) {
            const unsigned long long di = atomicAdd(done_count, 1ull);
            if (di < done_cap) {
                ovs_done_rec dr;
                dr.qid = qid; dr.pad = 0; dr.out = o;
                done[di] = dr;
            }
        }
        if (emit_out) {
            const unsigned long long oi = atomicAdd(out_count, 1ull);
            if (oi < out_cap) {
                store_lrec(out, oi, K, S, cur, qid, t, hops, 0);
                out_dest[oi] = (uint32_t)dest;
            }
        }
    }
}

__global__ void k_make_records(const KeyRec* __restrict__ recs, const K160* __restrict__ keys,
                               const uint32_t* __restrict__ src, uint64_t n, uint32_t qid_base,
                               ovs_lookup_rec* __restrict__ out)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    (void)recs;
    store_lrec(out, i, keys[i], src[i], src[i], qid_base + (uint32_t)i, 0, 0, 1);
}

// ---------------------------------------------------------------------------
// findNode batch (general numRedundantNodes / numSiblings), Chord.cc:548-599

__global__ void k_chord_find_node(ChordView V, int ideal, const uint32_t* __restrict__ node,
                                  const K160* __restrict__ keys, uint64_t n, int numRedundant,
                                  int numSiblings, uint32_t* __restrict__ out_nodes, uint32_t max_out,
                                  uint8_t* __restrict__ out_count, uint8_t* __restrict__ out_sib)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = node[i];
    const K160 K = keys[i];
    const KeyRec crec = load_rec(V.recs, c);
    const K160 C = key_of(crec);
    uint32_t* o = out_nodes + i * max_out;
    for (uint32_t j = 0; j < max_out; ++j) o[j] = NONE;
    const int ssize = ideal ? V.ns : V.nsucc[c];
    auto succ_at = [&](int j) -> uint32_t {
        return ideal ? ring_next(c, (uint32_t)j + 1, V.n) : V.succ[(uint64_t)c * V.sls + j];
    };
    // getFinger(pos) (ChordFingerTable.cc:174-193), resolved
    const uint32_t s0 = ssize > 0 ? succ_at(0) : c;
    const int ilo = ideal ? k_msb(k_sub(key_of(load_rec(V.recs, s0)), C)) + 1 : 0;
    auto finger_at = [&](int pos) -> uint32_t {
        if (ideal) return pos >= ilo ? V.frow[crec.aux + (uint32_t)(KEYBITS - 1 - pos)].x : s0;
        return V.fres[(uint64_t)c * KEYBITS + pos];
    };
    const bool sib = ideal ? between_R(K, key_of(load_rec(V.recs, c == 0 ? V.n - 1 : c - 1)), C)
                           : sibling_general(V, c, K, 1);
    int cnt = 0;
    auto push = [&](uint32_t v) { if ((uint32_t)cnt < max_out) o[cnt] = v; ++cnt; };
    if (sib) {
        // [self, succ...] downsized to numSiblings (Chord.cc:573-580)
        push(c);
        for (int j = 0; j < ssize; ++j) push(succ_at(j));
        if (cnt > numSiblings) cnt = numSiblings;
    } else if (ssize > 0 && between_R(K, C, key_of(load_rec(V.recs, s0)))) {
        // [succ...] downsized to numRedundantNodes (Chord.cc:583-590)
        for (int j = 0; j < ssize; ++j) push(succ_at(j));
        if (cnt > numRedundant) cnt = numRedundant;
    } else {
        // closestPreceedingNode (Chord.cc:602-674)
        K160 T;
        int tj = -1;
        for (int j = ssize - 1; j >= 0; --j) {
            const K160 SJ = key_of(load_rec(V.recs, succ_at(j)));
            if (between_R(SJ, C, K)) { tj = j; T = SJ; break; }
        }
        bool hit = false;
        for (int pos = KEYBITS - 1; pos >= 0 && tj >= 0; --pos) {
            const uint32_t f = finger_at(pos);
            if (between_LR(key_of(load_rec(V.recs, f)), T, K)) { push(f); hit = true; break; }
        }
        if (!hit && tj >= 0) {
            for (int j = ssize - 1; j >= 0 && cnt <= V.numFingerCandidates; --j) {
                const uint32_t sj = succ_at(j);
                if (between_open(key_of(load_rec(V.recs, sj)), C, K)) push(sj);
            }
        }
        if (cnt > numRedundant) cnt = numRedundant;
    }
    out_count[i] = (uint8_t)(cnt < (int)max_out ? cnt : (int)max_out);
    // findNodeRpc siblings flag: isSiblingFor(thisNode, key, numSiblings) (BaseOverlay.cc:1866-1871)
    out_sib[i] = (uint8_t)sib;
}

__global__ void k_delay(const double2* __restrict__ xy, DelayConsts DC, const uint32_t* __restrict__ a,
                        const uint32_t* __restrict__ b, const int32_t* __restrict__ bytes, uint64_t n,
                        int64_t* __restrict__ out)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (a[i] == b[i]) { out[i] = 0; return; }   // SimpleUDP.cc:322
    const double2 p = xy[a[i]], r = xy[b[i]];
    const int64_t bw = bw_ns(bytes[i], DC.datarate, DC.round);
    out[i] = 2 * bw + DC.access2 + coord_ns(p.x, p.y, r.x, r.y, DC.round);
}

// ---------------------------------------------------------------------------
// host launchers

static inline unsigned nblk(uint64_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

hipError_t launch_check_sorted(const KeyRec* recs, uint32_t n, uint32_t* bad, hipStream_t s)
{
    if (n < 2) return hipSuccess;
    hipLaunchKernelGGL(k_check_sorted, dim3(nblk(n, 256)), dim3(256), 0, s, recs, n, bad);
    return hipGetLastError();
}

hipError_t launch_chord_build(KeyRec* recs, uint32_t n, uint32_t lo, uint32_t hi, uint2** fingers_out,
                              uint64_t* nfing_out, hipStream_t s)
{
    hipError_t e;
    uint64_t* rowlen = nullptr;
    uint64_t* off = nullptr;
    void* tmp = nullptr;
    size_t tmpb = 0;
    const uint32_t cnt = hi - lo;
    *fingers_out = nullptr;
    if ((e = hipMalloc(&rowlen, sizeof(uint64_t) * (cnt + 1))) != hipSuccess) return e;
    if ((e = hipMalloc(&off, sizeof(uint64_t) * (cnt + 1))) != hipSuccess) { hipFree(rowlen); return e; }
    hipLaunchKernelGGL(k_chord_rowlen, dim3(nblk(cnt, 256)), dim3(256), 0, s, recs, n, lo, cnt, rowlen);
    hipMemsetAsync(rowlen + cnt, 0, sizeof(uint64_t), s);
    hipcub::DeviceScan::ExclusiveSum(nullptr, tmpb, rowlen, off, cnt + 1, s);
    if ((e = hipMalloc(&tmp, tmpb)) != hipSuccess) { hipFree(rowlen); hipFree(off); return e; }
    hipcub::DeviceScan::ExclusiveSum(tmp, tmpb, rowlen, off, cnt + 1, s);
    uint64_t total = 0;
    hipMemcpyAsync(&total, off + cnt, sizeof(uint64_t), hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    if (total + KEYBITS >= 0xFFFFFFFFull) { hipFree(rowlen); hipFree(off); hipFree(tmp); return hipErrorInvalidValue; }
    uint2* fing = nullptr;
    // +160 entries of padding: the kernel's speculative first-finger read may run past a row
    if ((e = hipMalloc(&fing, sizeof(uint2) * (total + KEYBITS))) != hipSuccess) {
        hipFree(rowlen); hipFree(off); hipFree(tmp); return e;
    }
    hipMemsetAsync(fing, 0, sizeof(uint2) * (total + KEYBITS), s);
    hipLaunchKernelGGL(k_set_aux, dim3(nblk(cnt, 256)), dim3(256), 0, s, recs, off, lo, cnt);
    hipLaunchKernelGGL(k_chord_fill, dim3(nblk(cnt, 128)), dim3(128), 0, s, recs, n, lo, cnt, fing);
    e = hipStreamSynchronize(s);
    hipFree(rowlen); hipFree(off); hipFree(tmp);
    if (e != hipSuccess) { hipFree(fing); return e; }
    *fingers_out = fing;
    *nfing_out = total;
    return hipGetLastError();
}

hipError_t launch_chord_nodes(const KeyRec* recs, const double2* xy, uint32_t n, int ns, NodeRec* nodes, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_chord_nodes, dim3(nblk(n, 256)), dim3(256), 0, s, recs, xy, n, ns, nodes);
    return hipGetLastError();
}

hipError_t launch_chord_export(const KeyRec* recs, const uint2* fingers, uint32_t n, uint32_t* out,
                               hipStream_t s)
{
    const uint64_t tot = (uint64_t)n * KEYBITS;
    hipLaunchKernelGGL(k_chord_export, dim3(nblk(tot, 256)), dim3(256), 0, s, recs, fingers, n, out);
    return hipGetLastError();
}

template <bool IDEAL, bool RECORD, bool REC>
static int route_blocks_per_cu()
{
    static int bpc = 0;
    if (bpc == 0) {
        int b = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_chord_route<IDEAL, RECORD, REC>, 256, 0) != hipSuccess ||
            b < 1)
            b = 1;
        bpc = b;
    }
    return bpc;
}

template <bool IDEAL, bool RECORD, bool REC>
static hipError_t chord_route_launch(const ChordView& V, const DelayConsts& DC, const LookupConsts& LC,
                                     const K160* qkeys, const uint32_t* qsrc, uint64_t nq, ovs_route_out* out,
                                     uint32_t* hopseq, int num_cu, hipStream_t s)
{
    // persistent grid: every resident wave owns one contiguous slice of the batch
    const uint64_t waves = (uint64_t)num_cu * route_blocks_per_cu<IDEAL, RECORD, REC>() * 4;   // 4 waves per block
    uint64_t chunk = (nq + waves - 1) / waves;
    if (chunk < 1) chunk = 1;
    const uint64_t need_waves = (nq + chunk - 1) / chunk;
    const uint64_t blocks = (need_waves + 3) / 4;
    hipLaunchKernelGGL((k_chord_route<IDEAL, RECORD, REC>), dim3((unsigned)blocks), dim3(256), 0, s, V, DC, LC, qkeys,
                       qsrc, nq, chunk, out, hopseq);
    return hipGetLastError();
}

hipError_t launch_chord_route(const ChordView& V, bool ideal, const DelayConsts& DC, const LookupConsts& LC,
                              const K160* qkeys, const uint32_t* qsrc, uint64_t nq, ovs_route_out* out,
                              uint32_t* hopseq, int num_cu, hipStream_t s)
{
    if (nq == 0) return hipSuccess;
    if (LC.recursive) {
        if (!ideal) return hipErrorNotSupported;
        return hopseq ? chord_route_launch<true, true, true>(V, DC, LC, qkeys, qsrc, nq, out, hopseq, num_cu, s)
                      : chord_route_launch<true, false, true>(V, DC, LC, qkeys, qsrc, nq, out, hopseq, num_cu, s);
    }
    if (!ideal) return chord_route_launch<false, true, false>(V, DC, LC, qkeys, qsrc, nq, out, hopseq, num_cu, s);
    return hopseq ? chord_route_launch<true, true, false>(V, DC, LC, qkeys, qsrc, nq, out, hopseq, num_cu, s)
                  : chord_route_launch<true, false, false>(V, DC, LC, qkeys, qsrc, nq, out, hopseq, num_cu, s);
}

hipError_t launch_chord_find_node(const ChordView& V, bool ideal, const uint32_t* node, const K160* keys,
                                  uint64_t n, int numRedundant, int numSiblings, uint32_t* out_nodes,
                                  uint32_t max_out, uint8_t* out_count, uint8_t* out_sib, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_chord_find_node, dim3(nblk(n, 128)), dim3(128), 0, s, V, ideal ? 1 : 0, node, keys, n,
                       numRedundant, numSiblings, out_nodes, max_out, out_count, out_sib);
    return hipGetLastError();
}

__global__ void k_fill_rpcs(const ovs_route_out* __restrict__ out, uint64_t n, uint32_t* __restrict__ rpcs)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    // alpha = 1: one FindNodeCall per counted hop, plus the call whose response came too late
    const ovs_route_out o = out[i];
    rpcs[i] = o.hops + ((o.status == OVS_LOOKUP_TIMEOUT || o.status == OVS_LOOKUP_RPC_TIMEOUT) ? 1u : 0u);
}

hipError_t launch_fill_rpcs_from_hops(const ovs_route_out* out, uint64_t n, uint32_t* rpcs, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_fill_rpcs, dim3(nblk(n, 256)), dim3(256), 0, s, out, n, rpcs);
    return hipGetLastError();
}

hipError_t launch_delay(const double2* xy, const DelayConsts& DC, const uint32_t* a, const uint32_t* b,
                        const int32_t* bytes, uint64_t n, int64_t* out, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_delay, dim3(nblk(n, 256)), dim3(256), 0, s, xy, DC, a, b, bytes, n, out);
    return hipGetLastError();
}

template <bool REC>
static int shard_blocks_per_cu()
{
    static int bpc = 0;
    if (bpc == 0) {
        int b = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_chord_shard_step<REC>, 256, 0) != hipSuccess || b < 1)
            b = 1;
        bpc = b;
    }
    return bpc;
}

hipError_t launch_chord_shard_step(const ChordView& V, const DelayConsts& DC, const LookupConsts& LC,
                                   const uint64_t* shard_lo, int nsh, int me, const ovs_lookup_rec* in, uint64_t nin,
                                   ovs_lookup_rec* out, uint32_t* out_dest, uint64_t out_cap,
                                   unsigned long long* out_count, ovs_done_rec* done, uint64_t done_cap,
                                   unsigned long long* done_count, int num_cu, hipStream_t s)
{
    if (nin == 0) return hipSuccess;
    const int bpc = LC.recursive ? shard_blocks_per_cu<true>() : shard_blocks_per_cu<false>();
    const uint64_t waves = (uint64_t)num_cu * bpc * 4;
    uint64_t chunk = (nin + waves - 1) / waves;
    if (chunk < 1) chunk = 1;
    const uint64_t need_waves = (nin + chunk - 1) / chunk;
    const dim3 g((unsigned)((need_waves + 3) / 4)), b(256);
    if (LC.recursive)
        hipLaunchKernelGGL(k_chord_shard_step<true>, g, b, 0, s, V, DC, LC, shard_lo, nsh, me, in, nin, chunk, out,
                           out_dest, out_cap, out_count, done, done_cap, done_count);
    else
        hipLaunchKernelGGL(k_chord_shard_step<false>, g, b, 0, s, V, DC, LC, shard_lo, nsh, me, in, nin, chunk, out,
                           out_dest, out_cap, out_count, done, done_cap, done_count);
    return hipGetLastError();
}

hipError_t launch_make_records(const KeyRec* recs, const K160* keys, const uint32_t* src, uint64_t n, uint32_t qid_base,
                               ovs_lookup_rec* out, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_make_records, dim3(nblk(n, 256)), dim3(256), 0, s, recs, keys, src, n, qid_base, out);
    return hipGetLastError();
}

}  // namespace ovs
