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

#include <algorithm>
#include <cstdio>
#include <vector>

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

// finger i of node v = responsible(v + 2^i) (rpcFixfingers answers thisNode, Chord.cc:1228-1270);
// only the index is written here, k_chord_entries completes the entry from the finger's NodeRec
__global__ void k_chord_fill(const KeyRec* __restrict__ recs, uint32_t n, uint32_t lo, uint32_t cnt,
                             FingerEnt* __restrict__ fingers)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= cnt) return;
    const uint32_t v = lo + t;
    const KeyRec r = load_rec(recs, v);
    const K160 self = key_of(r);
    const K160 s0 = key_of(load_rec(recs, v + 1 == n ? 0 : v + 1));
    const int ilo = k_msb(k_sub(s0, self)) + 1;
    FingerEnt* row = fingers + r.aux;
    for (int i = KEYBITS - 1; i >= ilo; --i)
        row[KEYBITS - 1 - i].idx = ring_lower_bound(recs, n, k_add(self, k_pow2(i)));
}

// replicated top levels of a sharded ring: finger i = responsible(v + 2^i) of EVERY node v for the
// top L levels (i = 159 .. 160 - L), ftop[v * L + (159 - i)]; k_chord_entries completes the entries
// from the fingers' NodeRecs.  A trivial position (2^i <= succ0 - v, tiny rings) resolves to succ0,
// which is what the lower bound gives there, and is never probed (pi >= ilo is checked first)
__global__ void k_chord_top(const KeyRec* __restrict__ recs, uint32_t n, int L, FingerEnt* __restrict__ ftop)
{
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)n * (uint32_t)L) return;
    const uint32_t v = (uint32_t)(t / (uint32_t)L);
    const int i = KEYBITS - 1 - (int)(t % (uint32_t)L);
    const K160 self = key_of(load_rec(recs, v));
    ftop[t].idx = ring_lower_bound(recs, n, k_add(self, k_pow2(i)));
}

// NodeRec of every node (ideal ring): key, finger-row offset, coordinates, window distances
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
    const uint64_t gP = top64(k_sub(P, C)), gS0 = top64(k_sub(S0, C)), gSL = top64(k_sub(SL, C));
    uint4* o = reinterpret_cast<uint4*>(nodes + v);
    o[0] = make_uint4(r.w[0], r.w[1], r.w[2], r.w[3]);
    o[1] = make_uint4(r.w[4], r.aux, (uint32_t)__double2loint(p.x), (uint32_t)__double2hiint(p.x));
    o[2] = make_uint4((uint32_t)__double2loint(p.y), (uint32_t)__double2hiint(p.y), (uint32_t)gS0, (uint32_t)(gS0 >> 32));
    o[3] = make_uint4((uint32_t)gSL, (uint32_t)(gSL >> 32), (uint32_t)gP, (uint32_t)(gP >> 32));
}

// WinRec of every node of the arc [lo, lo + cnt): top64 of the distances to successors 0..ns-1
__global__ void k_chord_win(const KeyRec* __restrict__ recs, uint32_t n, uint32_t lo, uint32_t cnt, int ns,
                            WinRec* __restrict__ win)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= cnt) return;
    const uint32_t v = lo + t;
    const K160 C = key_of(load_rec(recs, v));
    uint64_t g[8];
    for (int j = 0; j < 8; ++j) {
        uint32_t sj = v + (uint32_t)j + 1;
        while (sj >= n) sj -= n;
        g[j] = j < ns ? top64(k_sub(key_of(load_rec(recs, sj)), C)) : ~0ull;
    }
    uint4* o = reinterpret_cast<uint4*>(win + t);
    for (int j = 0; j < 4; ++j)
        o[j] = make_uint4((uint32_t)g[2 * j], (uint32_t)(g[2 * j] >> 32), (uint32_t)g[2 * j + 1], (uint32_t)(g[2 * j + 1] >> 32));
}

// complete every finger entry from its finger's NodeRec (rerun when the NodeRecs change)
__global__ void k_chord_entries(const NodeRec* __restrict__ nodes, FingerEnt* __restrict__ ents, uint64_t total)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= total) return;
    const uint32_t f = ents[e].idx;
    const uint4* q = reinterpret_cast<const uint4*>(nodes + f);
    const uint4 a = q[0], b = q[1], c = q[2], d = q[3];
    uint4* o = reinterpret_cast<uint4*>(ents + e);
    o[0] = a;                                     // key
    o[1] = make_uint4(b.x, f, b.z, b.w);          // key[4], idx, x
    o[2] = c;                                     // y, gS0
    o[3] = make_uint4(d.x, d.y, b.y, 0u);         // gSL, the finger's row offset
}

// resolved getFinger(pos) for every position (test export)
__global__ void k_chord_export(const KeyRec* __restrict__ recs, const FingerEnt* __restrict__ fingers,
                               uint32_t n, uint32_t* __restrict__ out)
{
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)n * KEYBITS) return;
    const uint32_t v = (uint32_t)(t / KEYBITS);
    const int pos = (int)(t % KEYBITS);
    const KeyRec r = load_rec(recs, v);
    const uint32_t s0i = v + 1 == n ? 0 : v + 1;
    const int ilo = k_msb(k_sub(key_of(load_rec(recs, s0i)), key_of(r))) + 1;
    out[t] = pos >= ilo ? fingers[r.aux + (KEYBITS - 1 - pos)].idx : s0i;
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

// Responder state carried in registers between hops for explicit (non-converged)
// tables: its 24 B KeyRec (coordinates gathered per hop).
template <bool IDEAL> struct Responder;
template <> struct Responder<false> {
    KeyRec r;
    __device__ __forceinline__ void load(const ChordView& V, uint32_t c) { r = load_rec(V.recs, c); }
    __device__ __forceinline__ double2 xy(const ChordView& V, uint32_t c) const { return V.xy[c]; }
    __device__ __forceinline__ Decision decide(const ChordView& V, uint32_t c, const K160& K) const
    {
        return decide_general(V, c, r, K);
    }
    __device__ __forceinline__ void advance(const ChordView&, const Decision& d) { r = d.rec; }
};

// K1 on explicit (non-converged) tables: literal restatement, full finger scan.
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
        const Decision d = rs.decide(V, cur, K);

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
            // the responsible node answers [cur, succ...] downsized to numSiblings (Chord.cc:573-580)
            const int64_t mresp = (d.sib && DC.lookupCall)
                ? resp_ns(DC, min(LC.numSiblings, 1 + (int)V.nsucc[cur])) : DC.msgResp1;
            const int64_t rtt = DC.msgCall + mresp + 2 * cd;
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
                o.latency_ns = t + ((R != S && !DC.lookupCall) ? DC.msgRoute + coord_ns(sx, sy, cxy.x, cxy.y, DC.round) : 0);
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

// ---------------------------------------------------------------------------
// K1 on a converged ring: the lookup as a per-lane state machine.
//
// Every loop iteration a lane consumes the one 64 B line it requested in the
// previous iteration, advances its lookup, and requests the next line; no lane
// waits inside an iteration for a second dependent load of its own.  A wave's
// iteration therefore costs one memory latency however its 64 lanes diverge (a
// finger probe that misses, a successor hand-off and a lookup start are each one
// more iteration of that lane only), and the waves of a SIMD overlap their
// latencies.  Phases (what the pending line is):
//   FETCH  the lookup's key and source (route) or its 48 B hand-off record (shard)
//   START  NodeRec of the responder where the lookup starts / arrives from a shard
//   NODE   NodeRec of a successor chosen as next hop
//   PROBE  FingerEnt pi of the current responder (whose key/row stay in registers)
//   WIN    WinRec of the current responder (K inside its successor window)
// Exact-key fallbacks on top64 ties read recs[] synchronously (rare).
enum : uint32_t { PH_FETCH = 0, PH_START = 1, PH_NODE = 2, PH_PROBE = 3, PH_WIN = 4 };

// a responder as unpacked from its NodeRec or from the finger entry pointing at it
struct Hdr {
    K160 k;
    uint32_t row;
    double x, y;
    uint64_t gS0, gSL;
};

__device__ __forceinline__ bool k_zero(const K160& a) { return (a.w[0] | a.w[1] | a.w[2] | a.w[3] | a.w[4]) == 0; }

// orders one wave's LDS stores before its loads of other lanes' slots (and the loads before the
// next iteration's stores) for the compiler; a wave's LDS instructions execute in issue order
__device__ __forceinline__ void lds_wave_fence()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int msb64(uint64_t x) { return 63 - __clzll((long long)x); }

__device__ __forceinline__ uint64_t u64(uint32_t lo, uint32_t hi) { return (uint64_t)lo | ((uint64_t)hi << 32); }

// sign of (D - gap) where gap = key(recs[g]) - C and gt = top64(gap): decided on the top
// 64 bits, exact on a tie
__device__ __forceinline__ int cmp_gap(const ChordView& V, const K160& D, uint64_t gt, const K160& C, uint32_t g)
{
    const uint64_t Dt = top64(D);
    if (Dt != gt) return Dt < gt ? -1 : 1;
    const K160 G = k_sub(key_of(load_rec(V.recs, g)), C);
    return k_lt(D, G) ? -1 : (k_eq(D, G) ? 0 : 1);
}

struct LaneIO {
    // single-GPU route (ovs_route_batch)
    const K160* __restrict__ qkeys;
    const uint32_t* __restrict__ qsrc;
    ovs_route_out* __restrict__ out;
    uint32_t* __restrict__ hopseq;
    // key order (ksort.hip): qkeys / qsrc are the batch sorted by key bits, perm[q] the caller's index
    // of sorted lookup q, where its result (and hop sequence) goes; nullptr = caller order
    const uint32_t* __restrict__ perm;
    // one hop round of an arc (ovs_shard_step)
    const ovs_lookup_rec* __restrict__ in;
    const K160* __restrict__ fkeys;        // a batch's first round straight from its keys and sources
    const uint32_t* __restrict__ fsrc;     // (ovs_shard_step_keys; in == nullptr): lookup q has qid fqid + q
    uint32_t fqid;
    ovs_lookup_rec* __restrict__ sout;     // nsh segments of scap records, one per destination arc
    uint64_t scap;
    unsigned long long* scount;            // nsh counters
    ovs_done_rec* __restrict__ done;
    uint64_t dcap;
    unsigned long long* dcount;
    const uint64_t* __restrict__ shard_lo;
    int nsh, me;
    uint64_t n, chunk;
    // the step's outcome per input record (compact_by_tag sorts them into sout / done)
    ovs_lookup_rec* __restrict__ stage_hand;
    ovs_done_rec* __restrict__ stage_done;
    uint8_t* __restrict__ stag;            // arc of the hand-off, or nsh: finished
    // dynamic tail (dyn != nullptr; routes and shard steps): each wave's static slice covers [0, dyn_from);
    // the rest is handed out K1_DYN_CH lookups at a time from the zeroed counter *dyn
    unsigned long long* dyn;
    uint64_t dyn_from;
};

// Persistent waves finish their static slices up to a quarter of the kernel apart (a census of
// their exit times, -DOVS_K1_TAIL): the last ~30 % of a batch is handed out dynamically instead, in
// chunks of one refill, so that the waves that run ahead take more
#ifndef K1_DYN_CH
#define K1_DYN_CH 64
#endif
#ifndef K1_DYN_STATIC
#define K1_DYN_STATIC 0.70
#endif

#ifdef OVS_K1_TAIL
// tail census (-DOVS_K1_TAIL builds): each wave's start and exit on the 100 MHz real-time clock, so
// the spread of the persistent waves' finishing times (the kernel's tail) can be read off one launch
constexpr int K1_TAIL_MAX = 1 << 16;
__device__ unsigned long long g_k1_tail[2 * K1_TAIL_MAX];
// lane 0 of the wave records the real-time counter in slot 2 * wave + which; the slot comes from
// wave-uniform values, so nothing stays live across the kernel's loop (a first version that kept the
// wave index and the start time live spilled the kernel)
__device__ __forceinline__ void ovs_tail_mark(unsigned long long* arr, int max, int which)
{
    const uint32_t wib = __builtin_amdgcn_readfirstlane(threadIdx.x) >> 6;
    const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wib;
    const unsigned long long t = wall_clock64();
    if (__lane_id() == 0 && w < (uint64_t)max) arr[2 * w + which] = t;
}
#endif
#ifdef OVS_CHORD_STATS
// lines consumed by kind: [0] FETCH, [1] START, [2] NODE, [3] first probe of a hop, [4] a further probe
// (the finger at msb(D) overshot K), [5] WIN
__device__ unsigned long long g_k1_stats[8];
#endif

// LKC: a LookupCall batch (ovs_lookup_batch): the responsible node's larger answer, no route message
// minimum waves per SIMD: every instantiation at the single-GPU route's 5 (its 89 VGPRs); the shard
// step's outcome staging had taken it to 98 VGPRs = 4 waves/SIMD
#ifndef OVS_K1_WAVES
#define OVS_K1_WAVES 5
#endif
// the shard step: 5 waves as well, with its outcomes staged where they are decided (held to the end
// of the iteration they had taken it to 107 VGPRs: at 5 waves 28-40 B per lane spilled to scratch
// inside the hop loop, every iteration waiting for a scratch reload; at 4 waves no spill)
#ifndef OVS_K1_SHARD_WAVES
#define OVS_K1_SHARD_WAVES 5
#endif
// DEF: the default configuration (successorListSize 8 on a ring of more than 8 nodes, hopCountMax
// 50) with those two as compile-time constants -- 1694 -> 1599 static instructions for the one-way
// route (the successor-window scans and hop checks fold); lanes_launch picks it
template <bool REC, bool RECORD, bool SHARD, bool LKC = false, bool DEF = false>
__global__ __launch_bounds__(256, SHARD ? OVS_K1_SHARD_WAVES : OVS_K1_WAVES) void k_chord_lanes(ChordView V, DelayConsts DC, LookupConsts LC, LaneIO io)
{
    const int lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    uint64_t cursor = wave * io.chunk;                    // wave-uniform
    const bool dyn = io.dyn != nullptr;
    uint64_t end = min(cursor + io.chunk, dyn ? io.dyn_from : io.n);
    bool more = dyn;                                      // dynamic chunks may be left
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int ns = DEF ? 8 : V.ns;
    const int hcm = DEF ? 50 : LC.hopCountMax;

    bool active = false;
    uint32_t ph = PH_FETCH;
    uint64_t q = 0;
    uint32_t dst = 0;                 // the caller index of lookup q (io.perm)
    uint32_t qid = 0;
    K160 K;
    uint32_t S = 0, cur = 0;
    int64_t t = 0;
    int hops = 0;
    bool local = true, nsib = false, pend = false;
    double sx = 0, sy = 0;            // iterative: the source's coordinates; recursive: the last sender's
    // the responder whose next hop is being determined (PROBE / WIN)
    K160 C;
    uint32_t row = 0;
    uint64_t gSL = 0;
    int pi = 0, ilo = 0, esl = 0;
    uint32_t fb = 0;                  // closestPreceedingNode's successor fallback (Chord.cc:653-658)
    bool gTx = false;                 // temp == K (node-ID key): a finger hits only when it is K
    const uint4* lp = nullptr;        // the line requested for the next iteration
    uint4 L0 = make_uint4(0, 0, 0, 0), L1 = L0, L2 = L0, L3 = L0;
    // shard with replicated top finger levels (V.ftl > 0): `remote` -- the current responder lies off
    // this arc and is being decided from the replicated levels; `redo` -- the record arrived as a
    // responder already reached whose decision needs its owner's rows (record local byte 2).
    // A lookup's outcome of a shard step (hand-off record or done record) is staged where it is
    // decided: holding it to the end of the iteration kept ~10 more VGPRs live across the loop
    bool remote = false, redo = false;

    __shared__ uint4 xbuf[4][256];    // per wave: the 64 gathered lines, 4 chunks each
    uint4* const xb = xbuf[threadIdx.x >> 6];
    // shard: the arcs' bounds in LDS and this rank's in registers -- a next hop's owner was a loop
    // of global reads of shard_lo per hop (most hops stay on the arc: one compare)
    __shared__ uint32_t sbnd[SHARD ? MAXSHARDS + 1 : 1];
    uint32_t arc_lo = 0, arc_hi = 0;
    if (SHARD) {
        for (int i = threadIdx.x; i <= io.nsh && i <= MAXSHARDS; i += blockDim.x) sbnd[i] = (uint32_t)io.shard_lo[i];
        __syncthreads();
        arc_lo = sbnd[io.me];
        arc_hi = sbnd[io.me + 1];
    }
    auto owner = [&](uint32_t c) -> int {
        if (c >= arc_lo && c < arc_hi) return io.me;
        int r = 0;
        for (int i = 1; i < io.nsh; ++i) r += c >= sbnd[i] ? 1 : 0;
        return r;
    };

    // Lookups started from their key and source (the single-GPU route): the sources of the wave's
    // next 64 candidates are preloaded one per lane, so a refilled lane has its source at once and
    // requests its source's NodeRec in the refill iteration itself (its key is loaded there too,
    // used from the next iteration on) -- one iteration per lookup fewer than requesting the line
    // in a PH_FETCH iteration after the refill.
#ifdef OVS_K1_NO_PRELOAD
    constexpr bool pre_ok = false;    // A/B build: the PH_FETCH iteration for every lookup
#else
    // (the shard step keeps the PH_FETCH iteration: a preloaded source spills 20 B per lane at 5
    // waves/SIMD even with its outcomes staged where decided)
    constexpr bool pre_ok = !SHARD;
#endif
    const K160* const pkeys = SHARD ? io.fkeys : io.qkeys;
    const uint32_t* const psrc = SHARD ? io.fsrc : io.qsrc;
    uint32_t pS = 0;
    auto preload = [&](uint64_t from) {
        if (pre_ok && from + (uint64_t)lane < end) pS = psrc[from + lane];
    };
    preload(cursor);

    while (true) {
        // ---- gathered lines to their lanes: chunk (lane & 3) of the line of lane 16k + (lane >> 2)
        // was fetched into Lk; LDS slot 4 * owner + chunk = 64 k + lane.  The reads below take
        // slots other lanes wrote: the wavefront fences keep the compiler from moving a ds_read
        // above the ds_write it depends on (the LDS itself executes one wave's ops in order)
        xb[lane] = L0; xb[64 + lane] = L1; xb[128 + lane] = L2; xb[192 + lane] = L3;
        lds_wave_fence();
        L0 = xb[4 * lane]; L1 = xb[4 * lane + 1]; L2 = xb[4 * lane + 2]; L3 = xb[4 * lane + 3];
        lds_wave_fence();

        // ---- refill: lanes without a lookup take the next of the wave's slice
        bool fresh = false;
        const uint64_t need = __ballot(!active);
        if (more && need != 0 && cursor >= end) {
            // the static slice is spent: the next dynamic chunk (one atomic a chunk, lane 0)
            unsigned long long b = 0;
            if (lane == 0) b = atomicAdd(io.dyn, (unsigned long long)K1_DYN_CH);
            const uint64_t nb = io.dyn_from + (((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                                               (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)b));
            if (nb < io.n) {
                cursor = nb;
                end = min(nb + (uint64_t)K1_DYN_CH, io.n);
                preload(cursor);
            } else {
                more = false;
            }
        }
        if (need != 0 && cursor < end && pre_ok) {
            const int rank = __popcll(need & lt_mask);
            const uint64_t mine = cursor + (uint64_t)rank;
            const uint32_t s0 = __shfl(pS, rank);
            if (!active && mine < end) {
                q = mine;
                if (!SHARD) dst = io.perm ? io.perm[q] : (uint32_t)q;
                active = true;
                fresh = true;
                K = pkeys[q];
                S = s0;
                if (SHARD) qid = io.fqid + (uint32_t)q;
                if (S < V.n) {
                    // what PH_FETCH does for a lookup at its source, and the source's line requested now
                    cur = S; t = 0; hops = 0; local = true;
                    lp = reinterpret_cast<const uint4*>(V.nodes + cur);
                    ph = PH_START;
                } else {
                    ph = PH_FETCH;        // a source outside the ring: PH_FETCH reports it
                    lp = nullptr;
                }
            }
            cursor += (uint64_t)__popcll(need);
            preload(cursor);
        } else if (need != 0 && cursor < end) {
            const uint64_t mine = cursor + (uint64_t)__popcll(need & lt_mask);
            if (!active && mine < end) {
                q = mine;
                active = true;
                fresh = true;
                ph = PH_FETCH;
                remote = false; redo = false;
                if (SHARD && io.fkeys) {
                    // a batch's first round: no record, the lookup starts from its key and source,
                    // whose line is requested in this refill iteration (what PH_FETCH would do one
                    // iteration later; the shard step has no register for the preloaded source)
                    K = io.fkeys[q];
                    S = io.fsrc[q];
                    qid = io.fqid + (uint32_t)q;
                    if (S < V.n) {
                        cur = S; t = 0; hops = 0; local = true;
                        lp = reinterpret_cast<const uint4*>(V.nodes + cur);
                        ph = PH_START;
                    } else {
                        lp = nullptr;          // PH_FETCH reports the source outside the ring
                    }
                } else if (SHARD) {
                    // the 48 B hand-off record, read here (a wave's records are consecutive: coalesced
                    // 16 B loads) so that its responder's line is requested in this refill iteration --
                    // through the cooperative gather it took an iteration of its own
                    const uint4* rp = reinterpret_cast<const uint4*>(io.in + q);
                    const uint4 r0 = rp[0], r1 = rp[1], r2 = rp[2];
                    K.w[0] = r0.x; K.w[1] = r0.y; K.w[2] = r0.z; K.w[3] = r0.w; K.w[4] = r1.x;
                    S = r1.y; cur = r1.z; qid = r1.w;
                    t = (int64_t)u64(r2.x, r2.y);
                    hops = (int)(r2.z & 0xFFFF);
                    const uint32_t lb = (r2.z >> 16) & 0xFF;
                    local = lb == 1;
                    redo = lb == 2;
                    if (S < V.n && cur < V.n) {
                        if (!REC) {
                            const double2 sxy = V.xy[S];      // coordinates are replicated on every rank
                            sx = sxy.x; sy = sxy.y;
                        }
                        lp = reinterpret_cast<const uint4*>(V.nodes + cur);
                        ph = PH_START;
                    } else {
                        lp = nullptr;          // PH_FETCH finishes it as BROKEN
                    }
                } else {
                    K = io.qkeys[q];
                    S = io.qsrc[q];
                    dst = io.perm ? io.perm[q] : (uint32_t)q;
                    lp = nullptr;
                }
            }
            cursor += (uint64_t)__popcll(need);
        }
        if (!__any(active)) break;
#ifdef OVS_CHORD_STATS
        {   // [6] wave iterations, [7] lanes that consume a line in them (diagnostic build)
            const uint64_t w = __ballot(active && !fresh);
            if (lane == 0) { atomicAdd(&g_k1_stats[6], 1ull); atomicAdd(&g_k1_stats[7], (unsigned long long)__popcll(w)); }
        }
#endif

        // finger pi of the current responder: its own row on this arc, or the replicated top levels
        // of an off-arc responder (pi >= 160 - V.ftl there, checked by the callers)
        auto fptr = [&](int p) -> const uint4* {
            if (SHARD && remote)
                return reinterpret_cast<const uint4*>(V.ftop + (uint64_t)cur * (uint32_t)V.ftl + (uint32_t)(KEYBITS - 1 - p));
            return reinterpret_cast<const uint4*>(V.frow + (uint64_t)row + (uint32_t)(KEYBITS - 1 - p));
        };
        if (active && !fresh) {
            bool arrived = false, asib = false, fin = false;
            uint8_t status = OVS_LOOKUP_OK;
            uint32_t R = NONE;
            Hdr A;
            uint32_t nxt = NONE;      // next hop chosen this iteration ...
            bool nxt_node = false;    // ... whose header must be read from its NodeRec
            bool nxt_sib = false;
            lp = nullptr;
            // an off-arc responder whose decision needs its owner's rows (a finger below the
            // replicated levels, or its successor window): the lookup goes to the owner as a
            // responder already reached (its response accounted here), which decides there
            auto redo_hand = [&]() {
                store_lrec(io.stage_hand, q, K, S, cur, qid, t, hops, 2);
                io.stag[q] = (uint8_t)owner(cur);
                active = false;
                lp = nullptr;
            };

#ifdef OVS_CHORD_STATS
            {   // line accounting (diagnostic build, tools/diag): which kind of line each lane consumes
                const K160 Dd = k_sub(K, C);
                const bool reprobe = ph == PH_PROBE && !gTx && pi < k_msb(Dd);
                const uint64_t b[6] = {__ballot(ph == PH_FETCH), __ballot(ph == PH_START), __ballot(ph == PH_NODE),
                                       __ballot(ph == PH_PROBE && !reprobe), __ballot(reprobe), __ballot(ph == PH_WIN)};
                if (lane == __ffsll((long long)__ballot(1)) - 1)
                    for (int k = 0; k < 6; ++k) atomicAdd(&g_k1_stats[k], (unsigned long long)__popcll(b[k]));
            }
#endif
            // ---- consume the pending line
            if (ph == PH_FETCH) {
                if (SHARD) {
                    // (a received record was decoded at the refill: only an invalid one gets here)
                    if (io.fkeys) { cur = S; t = 0; hops = 0; local = true; }
                    if (S >= V.n || cur >= V.n) {
                        // a row the exchange never wrote (receive buffers are 0xFF-filled) or a corrupted
                        // record: finished as BROKEN with its qid (0xFFFFFFFF for the sentinel), which
                        // the host's completeness check reports -- never a table read
                        fin = true; status = OVS_LOOKUP_BROKEN;
                    } else if (!REC) {
                        const double2 sxy = V.xy[S];      // coordinates are replicated on every rank
                        sx = sxy.x; sy = sxy.y;
                    }
                } else {
                    cur = S; t = 0; hops = 0; local = true;
                }
                if (!fin) {
                    lp = reinterpret_cast<const uint4*>(V.nodes + cur);
                    ph = PH_START;
                }
            } else {
                // the 64 B line: NodeRec and FingerEnt share key, coordinates and window distances
                A.k.w[0] = L0.x; A.k.w[1] = L0.y; A.k.w[2] = L0.z; A.k.w[3] = L0.w; A.k.w[4] = L1.x;
                A.x = dbl(L1.z, L1.w);
                A.y = dbl(L2.x, L2.y);
                A.gS0 = u64(L2.z, L2.w);
                A.gSL = u64(L3.x, L3.y);
                if (ph == PH_START) {
                    A.row = L1.y;
                    // isSiblingFor(cur, K, 1): K in (pred, cur]  <=>  D == 0 or D > pred - cur (Chord.cc:452-457)
                    const K160 D = k_sub(K, A.k);
                    asib = k_zero(D) || cmp_gap(V, D, u64(L3.z, L3.w), A.k, cur == 0 ? V.n - 1 : cur - 1) > 0;
                    // the source's own line (a lookup that left its source never comes back to START
                    // in one launch; a shard record's START is its responder's: coordinates from FETCH)
                    if (!REC && (!SHARD || local)) { sx = A.x; sy = A.y; }
                    arrived = true;
                } else if (ph == PH_NODE) {
                    A.row = L1.y;
                    asib = nsib;
                    if (REC && pend) t += DC.msgRoute + coord_ns(sx, sy, A.x, A.y, DC.round);   // to a successor
                    arrived = true;
                } else if (ph == PH_PROBE) {
                    // finger pi of C lies in [temp, K]  <=>  temp - C <= F - C <= D
                    A.row = L3.z;
                    const K160 D = k_sub(K, C);
                    const K160 dF = k_sub(A.k, C);
                    bool hit = k_le(dF, D);
                    if (hit) {
                        if (gTx) hit = k_eq(dF, D);                        // temp == K
                        else if (pi >= esl) hit = !k_zero(dF);             // 2^pi > temp - C
                        else hit = cmp_gap(V, dF, gSL, C, ring_next(cur, (uint32_t)ns, V.n)) >= 0;
                    }
                    if (hit) {
                        // a finger short of K is not responsible: (pred F, F] lies inside (C, F]
                        nxt = L1.y; nxt_sib = k_eq(A.k, K);
                    } else if (--pi >= ilo) {
                        if (SHARD && remote && pi < KEYBITS - V.ftl) redo_hand();
                        else lp = fptr(pi);
                    } else {
                        nxt = fb; nxt_node = true;       // Chord.cc:653-658 (succ0 via 183-184 when temp == succ0)
                    }
                } else {
                    // PH_WIN: K inside the successor window; temp = farthest s_j <= K (Chord.cc:612-623)
                    const K160 D = k_sub(K, C);
                    const uint64_t Dt = top64(D);
                    const uint64_t g[8] = {u64(L0.x, L0.y), u64(L0.z, L0.w), u64(L1.x, L1.y), u64(L1.z, L1.w),
                                           u64(L2.x, L2.y), u64(L2.z, L2.w), u64(L3.x, L3.y), u64(L3.z, L3.w)};
                    int tj = -1;
                    // the WinRec holds 8 successor distances: a longer successor list takes the
                    // exact scan over all ns successors below (Chord.cc:612-623)
                    bool tie = ns > 8;
                    #pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        if (j < ns) {
                            tie |= g[j] == Dt;
                            if (g[j] < Dt) tj = j;
                        }
                    }
                    bool tIsK = false;
                    if (tie) {
                        tj = -1;
                        for (int j = ns - 1; j >= 0; --j) {
                            const K160 SJ = key_of(load_rec(V.recs, ring_next(cur, (uint32_t)j + 1, V.n)));
                            if (between_R(SJ, C, K)) { tj = j; tIsK = k_eq(SJ, K); break; }
                        }
                    }
                    if (tj < 0) {
                        fin = true; status = OVS_LOOKUP_BROKEN;
                    } else if (!tIsK) {
                        // the only node in [temp, K] is temp: every finger that hits is temp and the
                        // successor fallback is temp too -- the next hop is temp either way
                        nxt = ring_next(cur, (uint32_t)tj + 1, V.n); nxt_node = true;
                    } else {
                        // temp == K: temp if a finger points at it, else s_{tj-1}
                        gTx = true;
                        fb = ring_next(cur, (uint32_t)tj, V.n);
                        pi = k_msb(D);
                        if (pi >= ilo) {
                            lp = reinterpret_cast<const uint4*>(V.frow + (uint64_t)row + (uint32_t)(KEYBITS - 1 - pi));
                            ph = PH_PROBE;
                        } else {
                            nxt = fb; nxt_node = true;
                        }
                    }
                }
            }

            // ---- IterativePathLookup::sendRpc / BaseOverlay::sendToKey for a chosen next hop;
            // returns true when the next responder's header is already in A (finger entry)
            auto send = [&](uint32_t nx, bool via_node, bool nx_sib) -> bool {
                if (REC) {
                    if (nx == S || nx == cur) { fin = true; status = OVS_LOOKUP_NO_NEXT; return false; }  // BaseOverlay.cc:1502-1516
                    if (RECORD && !SHARD && hops < hcm) io.hopseq[dst * (uint64_t)hcm + hops] = nx;
                    ++hops;
                } else if (nx == S) {
                    fin = true; status = OVS_LOOKUP_NO_NEXT; return false;                             // visitOnlyOnce
                }
                if (SHARD) {
                    const int dest = owner(nx);
                    remote = false;
                    // an off-arc responder reached through a finger entry (its header in A) whose first
                    // probe lies in the replicated top levels -- or which is the key's node, decided
                    // without a probe -- is decided here instead of on its owner
                    if (dest != io.me && V.ftl > 0 && !via_node &&
                        (nx_sib || k_msb(k_sub(K, A.k)) >= KEYBITS - V.ftl))
                        remote = true;
                    else if (dest != io.me) {
                        // hand the lookup to the owner of its next responder
                        if (REC) {
                            const double2 nxy = via_node ? V.xy[nx] : make_double2(A.x, A.y);
                            t += DC.msgRoute + coord_ns(sx, sy, nxy.x, nxy.y, DC.round);
                        }
                        cur = nx;
                        store_lrec(io.stage_hand, q, K, S, cur, qid, t, hops, 0);
                        io.stag[q] = (uint8_t)dest;
                        active = false;
                        lp = nullptr;
                        return false;
                    }
                }
                cur = nx;
                if (via_node) {
                    nsib = nx_sib; pend = REC;
                    lp = reinterpret_cast<const uint4*>(V.nodes + nx);
                    ph = PH_NODE;
                    return false;
                }
                if (REC) t += DC.msgRoute + coord_ns(sx, sy, A.x, A.y, DC.round);
                asib = nx_sib;
                return true;
            };
            if (!fin && nxt != NONE) arrived = send(nxt, nxt_node, nxt_sib);

            // ---- a responder is reached: its FindNodeResponse (iterative) / the route message (recursive)
            if (arrived) {
                uint32_t nx2 = NONE;
                bool nx2_sib = false;
                if (SHARD && redo) {
                    // a responder reached on another rank, which accounted for its response (or route
                    // message) and handed its decision here (record local byte 2)
                    redo = false;
                    local = false;
                    if (REC) { sx = A.x; sy = A.y; }
                } else if (REC) {
                    const bool at_src = local;
                    local = false;
                    sx = A.x; sy = A.y;
                    if (asib && (!at_src || hops < hcm)) { fin = true; R = cur; }       // BaseOverlay.cc:907-914
                    else if (asib || hops >= hcm) { fin = true; status = OVS_LOOKUP_HOPMAX; }   // 1464-1488
                } else if (local) {
                    // IterativeLookup::start (IterativeLookup.cc:157-204): local step, no hop, no delay
                    local = false;
                    if (asib) { fin = true; R = S; }
                } else {
                    // FindNodeCall S->cur, FindNodeResponse cur->S (one NodeHandle)
                    const int64_t cd = coord_ns(sx, sy, A.x, A.y, DC.round);
                    const int64_t rtt = DC.msgCall + ((LKC && asib) ? DC.msgRespSib : DC.msgResp1) + 2 * cd;
                    if (rtt >= DC.rpcTimeout) {
                        fin = true;
                        status = (t + DC.rpcTimeout > DC.lookupTimeout) ? OVS_LOOKUP_TIMEOUT : OVS_LOOKUP_RPC_TIMEOUT;
                    } else {
                        t += rtt;
                        if (t > DC.lookupTimeout) { fin = true; status = OVS_LOOKUP_TIMEOUT; }  // IterativeLookup.cc:808-815
                        else {
                            if (RECORD && !SHARD && hops < hcm) io.hopseq[dst * (uint64_t)hcm + hops] = cur;
                            ++hops;
                            if (asib) { fin = true; R = cur; }                                   // 896-905
                        }
                    }
                }
                // sendRpc's hop limit (IterativeLookup.cc:1067-1170) is checked before the next hop
                // is known: equivalent, as findNode cannot throw on a converged ring
                if (!REC && !fin && hcm && hops >= hcm) { fin = true; status = OVS_LOOKUP_HOPMAX; }
                if (!fin) {
                    // findNode at cur for a key it is not responsible for (Chord.cc:583-674)
                    C = A.k; row = A.row; gSL = A.gSL; gTx = false;
                    const K160 D = k_sub(K, C);
                    const uint32_t s0 = ring_next(cur, 1, V.n);
                    if (cmp_gap(V, D, A.gS0, C, s0) <= 0) {
                        nx2 = s0; nx2_sib = true;                      // K in (C, succ0] (Chord.cc:583-590)
                    } else {
                        ilo = A.gS0 ? 97 + msb64(A.gS0) : k_msb(k_sub(key_of(load_rec(V.recs, s0)), C)) + 1;
                        esl = gSL ? 97 + msb64(gSL) : 96;
                        const uint32_t sl = ring_next(cur, (uint32_t)ns, V.n);
                        const int c = cmp_gap(V, D, gSL, C, sl);
                        if (c < 0) {
                            if (SHARD && remote) {
                                redo_hand();                       // the window exists on the owner only
                            } else {
                                lp = reinterpret_cast<const uint4*>(V.win + (cur - V.lo));   // K inside the window
                                ph = PH_WIN;
                            }
                        } else {
                            // temp = succ[ns-1]; fingers from msb(D) down
                            gTx = c == 0;
                            fb = gTx ? ring_next(cur, (uint32_t)ns - 1, V.n) : sl;
                            pi = k_msb(D);
                            if (pi >= ilo) {
                                if (SHARD && remote && pi < KEYBITS - V.ftl) {
                                    redo_hand();
                                } else {
                                    lp = fptr(pi);
                                    ph = PH_PROBE;
                                }
                            } else {
                                nx2 = fb;
                            }
                        }
                    }
                }
                if (!fin && nx2 != NONE) send(nx2, true, nx2_sib);
            }

            if (fin) {
                ovs_route_out o;
                if (REC) {
                    const bool ok = status == OVS_LOOKUP_OK;
                    o.hops = (uint16_t)(ok ? hops : 0);
                    o.one_way_hops = (uint8_t)(ok ? hops : 0);
                    o.latency_ns = ok ? t : -1;
                    o.responsible = ok ? R : NONE;
                } else if (status == OVS_LOOKUP_OK) {
                    o.hops = (uint16_t)hops;
                    o.responsible = R;
                    o.one_way_hops = (uint8_t)(hops + (R != S ? 1 : 0));
                    // sendRouteMessage to result[0] (BaseOverlay.cc:1107-1146); 0 delay to self
                    o.latency_ns = t + ((R != S && !LKC) ? DC.msgRoute + coord_ns(sx, sy, A.x, A.y, DC.round) : 0);
                } else {
                    o.hops = (uint16_t)hops;
                    o.responsible = NONE;
                    o.one_way_hops = 0;
                    o.latency_ns = -1;
                }
                o.status = status;
                if (SHARD) {
                    ovs_done_rec dr;
                    dr.qid = qid; dr.pad = 0; dr.out = o;
                    io.stage_done[q] = dr;
                    io.stag[q] = (uint8_t)io.nsh;
                } else {
                    io.out[dst] = o;
                }
                active = false;
                lp = nullptr;
            }
        }
        // (shard: every input record has exactly one outcome this launch, staged at its own index
        // where it was decided -- no atomics: compact_by_tag moves them to the per-arc segments and
        // the done buffer)
        // ---- request the next line: a cooperative gather, 4 lanes fetch one 64 B line with one
        // 16 B load each, so one wave instruction touches 16 lines instead of 64 (on HBM-resident
        // tables this moves 2.3x the lines/s of per-lane 4 x 16 B loads: tools/ubench/gather.hip)
        {
            const uint64_t mine = (active && lp) ? reinterpret_cast<uint64_t>(lp) : 0ull;
            const uint32_t mlo = (uint32_t)mine, mhi = (uint32_t)(mine >> 32);
            const int ch = lane & 3;
            uint4 v[4];
            #pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int owner = 16 * k + (lane >> 2);
                const uint64_t a = (uint64_t)__shfl(mlo, owner) | ((uint64_t)__shfl(mhi, owner) << 32);
                // tag 1 = a 48 B record: no fourth chunk
                if (a != 0 && (ch < 3 || !(a & 1))) v[k] = reinterpret_cast<const uint4*>(a & ~(uint64_t)15)[ch];
                else v[k] = make_uint4(0, 0, 0, 0);
            }
            L0 = v[0]; L1 = v[1]; L2 = v[2]; L3 = v[3];
        }
    }
#ifdef OVS_K1_TAIL
    ovs_tail_mark(g_k1_tail, K1_TAIL_MAX, 1);
#endif
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
        if (ideal) return pos >= ilo ? V.frow[crec.aux + (uint32_t)(KEYBITS - 1 - pos)].idx : s0;
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

hipError_t launch_chord_build(KeyRec* recs, uint32_t n, uint32_t lo, uint32_t hi, FingerEnt** fingers_out,
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
    FingerEnt* fing = nullptr;
    // +160 entries of padding: the kernel's speculative first-finger read may run past a row
    if ((e = hipMalloc(&fing, sizeof(FingerEnt) * (total + KEYBITS))) != hipSuccess) {
        hipFree(rowlen); hipFree(off); hipFree(tmp); return e;
    }
    hipMemsetAsync(fing, 0, sizeof(FingerEnt) * (total + KEYBITS), s);
    hipLaunchKernelGGL(k_set_aux, dim3(nblk(cnt, 256)), dim3(256), 0, s, recs, off, lo, cnt);
    hipLaunchKernelGGL(k_chord_fill, dim3(nblk(cnt, 128)), dim3(128), 0, s, recs, n, lo, cnt, fing);
    e = hipStreamSynchronize(s);
    hipFree(rowlen); hipFree(off); hipFree(tmp);
    if (e != hipSuccess) { hipFree(fing); return e; }
    *fingers_out = fing;
    *nfing_out = total;
    return hipGetLastError();
}

hipError_t launch_chord_nodes(const KeyRec* recs, const double2* xy, uint32_t n, int ns, NodeRec* nodes,
                              FingerEnt* fingers, uint64_t nfing, WinRec* win, uint32_t lo, uint32_t hi, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_chord_nodes, dim3(nblk(n, 256)), dim3(256), 0, s, recs, xy, n, ns, nodes);
    if (hi > lo) hipLaunchKernelGGL(k_chord_win, dim3(nblk(hi - lo, 256)), dim3(256), 0, s, recs, n, lo, hi - lo, ns, win);
    if (nfing) hipLaunchKernelGGL(k_chord_entries, dim3(nblk(nfing, 256)), dim3(256), 0, s, nodes, fingers, nfing);
    return hipGetLastError();
}

hipError_t launch_chord_top(const KeyRec* recs, uint32_t n, int L, FingerEnt* ftop, hipStream_t s)
{
    const uint64_t tot = (uint64_t)n * (uint32_t)L;
    if (tot == 0) return hipSuccess;
    hipLaunchKernelGGL(k_chord_top, dim3(nblk(tot, 256)), dim3(256), 0, s, recs, n, L, ftop);
    return hipGetLastError();
}

hipError_t launch_chord_entries(const NodeRec* nodes, FingerEnt* ents, uint64_t total, hipStream_t s)
{
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(k_chord_entries, dim3(nblk(total, 256)), dim3(256), 0, s, nodes, ents, total);
    return hipGetLastError();
}

hipError_t launch_chord_export(const KeyRec* recs, const FingerEnt* fingers, uint32_t n, uint32_t* out,
                               hipStream_t s)
{
    const uint64_t tot = (uint64_t)n * KEYBITS;
    hipLaunchKernelGGL(k_chord_export, dim3(nblk(tot, 256)), dim3(256), 0, s, recs, fingers, n, out);
    return hipGetLastError();
}

// occupancy-sized persistent grid: every resident wave owns one contiguous slice of the work
template <class Kern>
static uint64_t persistent_chunk(Kern k, int* cache, uint64_t n, int num_cu, uint64_t* blocks)
{
    if (*cache == 0) {
        int b = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k, 256, 0) != hipSuccess || b < 1) b = 1;
        *cache = b;
    }
    const uint64_t waves = (uint64_t)num_cu * (uint64_t)(*cache) * 4;   // 4 waves per block
    uint64_t chunk = (n + waves - 1) / waves;
    if (chunk < 1) chunk = 1;
    const uint64_t need_waves = (n + chunk - 1) / chunk;
    *blocks = (need_waves + 3) / 4;
    return chunk;
}

template <bool REC, bool RECORD, bool SHARD, bool LKC = false, bool DEF = false>
static hipError_t lanes_launch(const ChordView& V, const DelayConsts& DC, const LookupConsts& LC, LaneIO io,
                               int num_cu, hipStream_t s)
{
    static int bpc = 0;
    uint64_t blocks = 0;
    io.chunk = persistent_chunk(k_chord_lanes<REC, RECORD, SHARD, LKC, DEF>, &bpc, io.n, num_cu, &blocks);
    if (io.dyn) {
        // static slices cover K1_DYN_STATIC of the batch, the rest goes out in chunks (tiny batches: static)
        const uint64_t waves = blocks * 4;
        const uint64_t cs = (uint64_t)((double)io.n * K1_DYN_STATIC) / waves;
        if (cs < (uint64_t)K1_DYN_CH) {
            io.dyn = nullptr;
        } else {
            io.chunk = cs;
            io.dyn_from = cs * waves;
        }
    }
#ifdef OVS_CHORD_STATS
    unsigned long long z[8] = {};
    hipMemcpyToSymbolAsync(HIP_SYMBOL(g_k1_stats), z, sizeof z, 0, hipMemcpyHostToDevice, s);
#endif
    hipLaunchKernelGGL((k_chord_lanes<REC, RECORD, SHARD, LKC, DEF>), dim3((unsigned)blocks), dim3(256), 0, s, V, DC,
                       LC, io);
#ifdef OVS_K1_TAIL
    if (!SHARD) {
        const uint64_t nw = blocks * 4 < (uint64_t)K1_TAIL_MAX ? blocks * 4 : (uint64_t)K1_TAIL_MAX;
        std::vector<unsigned long long> tt(2 * nw);
        hipMemcpyFromSymbolAsync(tt.data(), HIP_SYMBOL(g_k1_tail), sizeof(unsigned long long) * 2 * nw, 0,
                                 hipMemcpyDeviceToHost, s);
        hipStreamSynchronize(s);
        unsigned long long t0 = ~0ull;
        std::vector<double> fin;
        for (uint64_t w = 0; w < nw; ++w) t0 = tt[2 * w + 1] < t0 ? tt[2 * w + 1] : t0;
        for (uint64_t w = 0; w < nw; ++w) fin.push_back((double)(tt[2 * w + 1] - t0) * 0.01);   // 100 MHz -> us
        std::sort(fin.begin(), fin.end());
        auto pct = [&](double f) { return fin[(size_t)(f * (fin.size() - 1))]; };
        fprintf(stderr, "k1tail waves=%llu chunk=%llu finish_us_after_first_exit p0=%.1f p10=%.1f p50=%.1f p90=%.1f p99=%.1f max=%.1f\n",
                (unsigned long long)nw, (unsigned long long)io.chunk, pct(0), pct(0.1), pct(0.5), pct(0.9), pct(0.99),
                fin.back());
    }
#endif
#ifdef OVS_CHORD_STATS
    hipMemcpyFromSymbolAsync(z, HIP_SYMBOL(g_k1_stats), sizeof z, 0, hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    fprintf(stderr, "k1stats n=%llu fetch=%llu start=%llu node=%llu probe1=%llu reprobe=%llu win=%llu "
            "wave_iters=%llu busy_lanes=%llu\n",
            (unsigned long long)io.n, z[0], z[1], z[2], z[3], z[4], z[5], z[6], z[7]);
#endif
    return hipGetLastError();
}

template <bool IDEAL, bool RECORD, bool REC>
static hipError_t chord_route_launch(const ChordView& V, const DelayConsts& DC, const LookupConsts& LC,
                                     const K160* qkeys, const uint32_t* qsrc, uint64_t nq, ovs_route_out* out,
                                     uint32_t* hopseq, int num_cu, hipStream_t s, const uint32_t* perm = nullptr,
                                     unsigned long long* dyn = nullptr)
{
    if constexpr (IDEAL) {
        LaneIO io{};
        io.qkeys = qkeys; io.qsrc = qsrc; io.out = out; io.hopseq = hopseq; io.n = nq; io.perm = perm;
        io.dyn = dyn;
        if constexpr (!REC && !RECORD) {
            if (DC.lookupCall) return lanes_launch<false, false, false, true>(V, DC, LC, io, num_cu, s);
        }
        if (DC.lookupCall) return hipErrorNotSupported;
#ifndef OVS_K1_NO_DEF
        if constexpr (!REC && !RECORD) {
            if (V.ns == 8 && LC.hopCountMax == 50) return lanes_launch<false, false, false, false, true>(V, DC, LC, io, num_cu, s);
        }
#endif
        return lanes_launch<REC, RECORD, false>(V, DC, LC, io, num_cu, s);
    } else {
        static int bpc = 0;
        uint64_t blocks = 0;
        const uint64_t chunk = persistent_chunk(k_chord_route<false, RECORD, REC>, &bpc, nq, num_cu, &blocks);
        hipLaunchKernelGGL((k_chord_route<false, RECORD, REC>), dim3((unsigned)blocks), dim3(256), 0, s, V, DC, LC,
                           qkeys, qsrc, nq, chunk, out, hopseq);
        return hipGetLastError();
    }
}

hipError_t launch_chord_route(const ChordView& V, bool ideal, const DelayConsts& DC, const LookupConsts& LC,
                              const K160* qkeys, const uint32_t* qsrc, uint64_t nq, ovs_route_out* out,
                              uint32_t* hopseq, int num_cu, hipStream_t s, const uint32_t* perm,
                              unsigned long long* dyn)
{
    if (nq == 0) return hipSuccess;
    if (perm) {
        // key order: one-way iterative routes on a converged ring only (the LookupCall finish and the
        // recursive and explicit-table kernels index their outputs by batch position)
        if (!ideal || LC.recursive || DC.lookupCall) return hipErrorNotSupported;
        return hopseq ? chord_route_launch<true, true, false>(V, DC, LC, qkeys, qsrc, nq, out, hopseq, num_cu, s, perm, dyn)
                      : chord_route_launch<true, false, false>(V, DC, LC, qkeys, qsrc, nq, out, hopseq, num_cu, s, perm, dyn);
    }
    if (LC.recursive) {
        if (!ideal) return hipErrorNotSupported;
        return hopseq ? chord_route_launch<true, true, true>(V, DC, LC, qkeys, qsrc, nq, out, hopseq, num_cu, s, nullptr, dyn)
                      : chord_route_launch<true, false, true>(V, DC, LC, qkeys, qsrc, nq, out, hopseq, num_cu, s, nullptr, dyn);
    }
    if (!ideal) return chord_route_launch<false, true, false>(V, DC, LC, qkeys, qsrc, nq, out, hopseq, num_cu, s, nullptr, dyn);
    return hopseq ? chord_route_launch<true, true, false>(V, DC, LC, qkeys, qsrc, nq, out, hopseq, num_cu, s, nullptr, dyn)
                  : chord_route_launch<true, false, false>(V, DC, LC, qkeys, qsrc, nq, out, hopseq, num_cu, s, nullptr, dyn);
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

// LookupCall results from the lookups' route records, in place (ovs_route_out and ovs_lookup_out
// share their 16 B slot).  Chord: the sibling vector is the responsible node's findNode answer
// [R, succ...] downsized to numSiblings (Chord.cc:573-580; IterativeLookup::addSibling pushes it
// in order, 406-449).  Kademlia: the route kernel has written the answering response's nodes.
// SendToKeyListener::lookupFinished's LookupResponse (BaseOverlay.cc:1272-1300) of one finished
// LookupCall from its route record: on Chord the sibling vector is [R, succ(R)...] (Chord.cc:573-580)
__device__ __forceinline__ ovs_lookup_out lookup_finish_one(const ChordView& V, int chord, int ideal, int ns,
                                                            const ovs_route_out r, uint32_t* __restrict__ row)
{
    const bool ok = r.status == OVS_LOOKUP_OK;
    uint32_t cnt = 0;
    if (chord) {
        if (ok) {
            const uint32_t R = r.responsible;
            const int ssize = ideal ? V.ns : (int)V.nsucc[R];
            const int m = min(ns, 1 + ssize);
            row[0] = R;
            for (int j = 1; j < m; ++j)
                row[j] = ideal ? ring_next(R, (uint32_t)j, V.n) : V.succ[(uint64_t)R * V.sls + (j - 1)];
            cnt = (uint32_t)m;
        }
        for (int j = (int)cnt; j < ns; ++j) row[j] = NONE;
    } else if (ok) {
        while (cnt < (uint32_t)ns && row[cnt] != NONE) ++cnt;
    } else {
        for (int j = 0; j < ns; ++j) row[j] = NONE;
    }
    ovs_lookup_out o;
    o.num_siblings = ok ? cnt : 0;
    o.hops = r.hops;
    o.status = r.status;
    o.is_valid = ok ? 1 : 0;
    o.latency_ns = ok ? r.latency_ns : -1;
    return o;
}

__global__ void k_lookup_finish(ChordView V, int chord, int ideal, int ns, ovs_route_out* __restrict__ io,
                                uint32_t* __restrict__ sibs, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const ovs_lookup_out o = lookup_finish_one(V, chord, ideal, ns, io[i], sibs + i * (uint64_t)ns);
    reinterpret_cast<ovs_lookup_out*>(io)[i] = o;
}

// the LookupCalls finished across arcs: done records (any order) -> LookupResponses in that order
__global__ void k_shard_lookup_finish(ChordView V, int ns, const ovs_done_rec* __restrict__ done,
                                      ovs_lookup_out* __restrict__ out, uint32_t* __restrict__ sibs, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = lookup_finish_one(V, 1, 1, ns, done[i].out, sibs + i * (uint64_t)ns);
}

hipError_t launch_shard_lookup_finish(const ChordView& V, int ns, const ovs_done_rec* done, ovs_lookup_out* out,
                                      uint32_t* sibs, uint64_t n, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_shard_lookup_finish, dim3(nblk(n, 256)), dim3(256), 0, s, V, ns, done, out, sibs, n);
    return hipGetLastError();
}

// Chord LookupCalls with numSiblings = 0 (exact-key lookups).  findNode's choice at a node that is
// not responsible for K does not depend on numSiblings (Chord.cc:548-599), so the lookup follows the
// chain R1, R2, ... of the same key routed as a one-way lookup; io holds that route, run without
// RPC / lookup timeouts and with hopCountMax + 1 hops recorded in hopseq (stride H).  Replayed here
// with the exact-key rules (IterativeLookup.cc:157-184, 803-921, 1067-1170):
//  * the source responsible: its findNode answers [S, succ...] downsized to 0 -> no next hop, fail;
//  * response i from a node not responsible for K carries the next hop R(i+1): the lookup succeeds
//    there when R(i+1)'s key is K (862-870), the LookupResponse holding R(i+1);
//  * the responsible node answers an empty vector (and no sibling flag counts for numSiblings = 0):
//    nothing left to ask, fail (HOPMAX when the hop budget is spent, as sendRpc checks that first);
//  * every call's RTT with the response's real size (0 nodes from the responsible node), with the
//    RPC / lookup timeouts of k_chord_route and K1.
__global__ void k_chord_exact_finish(ChordView V, DelayConsts DC, int hcm, const K160* __restrict__ keys,
                                     const uint32_t* __restrict__ src, const uint32_t* __restrict__ hopseq, int H,
                                     ovs_route_out* __restrict__ io, uint64_t n)
{
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    const ovs_route_out r = io[q];
    const uint32_t S = src[q];
    const K160 K = keys[q];
    const int nrec = min((int)r.hops, H);
    const int k = r.status == OVS_LOOKUP_OK ? (int)r.hops : -1;   // the responsible node answered response k
    const double2 sxy = V.xy[S];
    ovs_route_out o;
    o.responsible = NONE;
    o.one_way_hops = 0;
    o.latency_ns = -1;
    o.hops = 0;
    o.status = k == 0 ? (uint8_t)OVS_LOOKUP_NO_NEXT : r.status;   // nothing sent: the start's outcome
    int64_t t = 0;
    for (int i = 1; i <= nrec; ++i) {
        const uint32_t Ri = hopseq[q * (uint64_t)H + (i - 1)];
        const bool resp = i == k;
        const double2 rxy = V.xy[Ri];
        const int64_t cd = coord_ns(sxy.x, sxy.y, rxy.x, rxy.y, DC.round);
        const int64_t rtt = DC.msgCall + (resp ? resp_ns(DC, 0) : DC.msgResp1) + 2 * cd;
        if (rtt >= DC.rpcTimeout) {
            o.status = (t + DC.rpcTimeout > DC.lookupTimeout) ? OVS_LOOKUP_TIMEOUT : OVS_LOOKUP_RPC_TIMEOUT;
            break;
        }
        t += rtt;
        if (t > DC.lookupTimeout) { o.status = OVS_LOOKUP_TIMEOUT; break; }
        o.hops = (uint16_t)i;
        if (i == nrec && r.status == OVS_LOOKUP_BROKEN) { o.status = OVS_LOOKUP_BROKEN; break; }
        if (resp) { o.status = (hcm && i >= hcm) ? OVS_LOOKUP_HOPMAX : OVS_LOOKUP_NO_NEXT; break; }
        if (i < nrec) {
            const uint32_t nx = hopseq[q * (uint64_t)H + i];
            if (k_eq(key_of(load_rec(V.recs, nx)), K)) {
                o.status = OVS_LOOKUP_OK;
                o.responsible = nx;
                o.one_way_hops = (uint8_t)(i + 1);
                o.latency_ns = t;
                break;
            }
        }
        if (hcm && i >= hcm) { o.status = OVS_LOOKUP_HOPMAX; break; }
        // the route ended after response i without a recorded next hop: its next was visited
        if (i == nrec) { o.status = r.status; break; }
    }
    io[q] = o;
}

hipError_t launch_chord_exact_finish(const ChordView& V, const DelayConsts& DC, int hcm, const K160* keys,
                                     const uint32_t* src, const uint32_t* hopseq, int H, ovs_route_out* io,
                                     uint64_t n, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_chord_exact_finish, dim3(nblk(n, 256)), dim3(256), 0, s, V, DC, hcm, keys, src, hopseq, H,
                       io, n);
    return hipGetLastError();
}

hipError_t launch_lookup_finish(const ChordView& V, bool chord, bool ideal, int ns, ovs_route_out* io,
                                uint32_t* sibs, uint64_t n, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_lookup_finish, dim3(nblk(n, 256)), dim3(256), 0, s, V, chord ? 1 : 0, ideal ? 1 : 0, ns, io,
                       sibs, n);
    return hipGetLastError();
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

hipError_t launch_chord_shard_step(const ChordView& V, const DelayConsts& DC, const LookupConsts& LC,
                                   const uint64_t* shard_lo, int nsh, int me, const ovs_lookup_rec* in, uint64_t nin,
                                   ovs_lookup_rec* out, uint64_t out_cap,
                                   unsigned long long* out_count, ovs_done_rec* done, uint64_t done_cap,
                                   unsigned long long* done_count, StageBuf& stage, int num_cu, hipStream_t s,
                                   const K160* fkeys, const uint32_t* fsrc, uint32_t fqid, unsigned long long* dyn)
{
    if (nin == 0) return hipSuccess;
    if (nsh < 1 || nsh + 1 > CMAX) return hipErrorInvalidValue;
    // stage: a hand-off record and a done record per input, and its outcome tag
    const size_t oh = 0, od = oh + sizeof(ovs_lookup_rec) * nin, ot = od + sizeof(ovs_done_rec) * nin;
    hipError_t e = stage_ensure(stage, ot + nin, s);
    if (e != hipSuccess) return e;
    uint8_t* sb = static_cast<uint8_t*>(stage.buf);
    LaneIO io{};
    io.in = in; io.sout = out; io.scap = out_cap; io.scount = out_count;
    io.fkeys = fkeys; io.fsrc = fsrc; io.fqid = fqid;
    io.done = done; io.dcap = done_cap; io.dcount = done_count;
    io.shard_lo = shard_lo; io.nsh = nsh; io.me = me; io.n = nin;
    io.dyn = dyn;
    io.stage_hand = reinterpret_cast<ovs_lookup_rec*>(sb + oh);
    io.stage_done = reinterpret_cast<ovs_done_rec*>(sb + od);
    io.stag = sb + ot;
    if ((e = hipMemsetAsync(io.stag, 0xFF, nin, s)) != hipSuccess) return e;
    // DC.lookupCall: a LookupCall batch (the responsible node's larger answer, no route message)
    e = LC.recursive ? lanes_launch<true, false, true>(V, DC, LC, io, num_cu, s)
        : DC.lookupCall ? lanes_launch<false, false, true, true>(V, DC, LC, io, num_cu, s)
#ifndef OVS_K1_NO_DEF
                        : (V.ns == 8 && LC.hopCountMax == 50) ? lanes_launch<false, false, true, false, true>(V, DC, LC, io, num_cu, s)
#endif
                        : lanes_launch<false, false, true>(V, DC, LC, io, num_cu, s);
    if (e != hipSuccess) return e;
    // outcomes to their outputs: class d < nsh = hand-offs to arc d (segment d of out), nsh = done
    CPlan P{};
    P.seg.src = sb + oh; P.seg.src_stride = P.seg.rec_bytes = sizeof(ovs_lookup_rec);
    P.seg.dst = reinterpret_cast<uint8_t*>(out); P.seg.dst_stride = sizeof(ovs_lookup_rec) * out_cap;
    P.seg.cap = out_cap; P.seg.counter = out_count; P.seg.n = nsh; P.seg.chain = 0;
    P.nextra = 1;
    CClass& d = P.extra[0];
    d.src = sb + od; d.src_stride = d.rec_bytes = sizeof(ovs_done_rec);
    d.dst = reinterpret_cast<uint8_t*>(done); d.cap = done_cap; d.counter = done_count;
    return compact_by_tag(io.stag, nin, P, stage.cs, s);
}

__global__ __launch_bounds__(256) void k_xy_bbox(const double2* __restrict__ xy, uint64_t n, double* __restrict__ out)
{
    __shared__ double sh[4][256];
    double x0 = INFINITY, x1 = -INFINITY, y0 = INFINITY, y1 = -INFINITY;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const double2 p = xy[i];
        x0 = fmin(x0, p.x); x1 = fmax(x1, p.x); y0 = fmin(y0, p.y); y1 = fmax(y1, p.y);
    }
    sh[0][threadIdx.x] = x0; sh[1][threadIdx.x] = x1; sh[2][threadIdx.x] = y0; sh[3][threadIdx.x] = y1;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            sh[0][threadIdx.x] = fmin(sh[0][threadIdx.x], sh[0][threadIdx.x + w]);
            sh[1][threadIdx.x] = fmax(sh[1][threadIdx.x], sh[1][threadIdx.x + w]);
            sh[2][threadIdx.x] = fmin(sh[2][threadIdx.x], sh[2][threadIdx.x + w]);
            sh[3][threadIdx.x] = fmax(sh[3][threadIdx.x], sh[3][threadIdx.x + w]);
        }
        __syncthreads();
    }
    if (threadIdx.x < 4) out[4 * blockIdx.x + threadIdx.x] = sh[threadIdx.x][0];
}

hipError_t launch_xy_bbox(const double2* xy, uint64_t n, double* out, int* blocks, hipStream_t s)
{
    const uint64_t b = nblk(n, 256);
    *blocks = (int)(b < 256 ? (b ? b : 1) : 256);
    hipLaunchKernelGGL(k_xy_bbox, dim3((unsigned)*blocks), dim3(256), 0, s, xy, n, out);
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
