// engine.hpp -- device-side data layout and shared device functions of the
// MI355X lookup-routing engine (internal; the public boundary is include/ovs_kbr.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "key160.hpp"
#include "../../include/ovs_kbr.h"

namespace ovs {

constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr int KEYBITS = 160;

// ---------------------------------------------------------------------------
// Per-launch constants derived from ovs_params on the host.  All times are
// int64 ns (simtime-scale = -9, default.ini:27).
struct DelayConsts {
    int64_t msgCall;     // 2*T(L*8/datarate) + 2*T(accessDelay) for FindNodeCall (83 B)
    int64_t msgResp1;    // same for a FindNodeResponse with one NodeHandle (87 B)
    int64_t msgRoute;    // same for the one-way route message (186 B)
    int64_t rpcTimeout;  // T(rpcUdpTimeout)
    int64_t lookupTimeout;  // T(LOOKUP_TIMEOUT)
    int32_t round;       // SimTime(double) rounding rule
    int32_t respBase;    // FindNodeResponse bytes with zero nodes (61 B)
    int32_t respPerNode; // 26 B per NodeHandle
    int32_t callBytes;   // 83 B
    int32_t routeBytes;  // one-way route message, 186 B for testMsgSize = 100 B
    double datarate;
    int64_t access2;     // 2*T(accessDelay)
    int64_t msgRespSib;  // same for the responsible node's FindNodeResponse on a converged Chord ring:
                         // min(numSiblings, 1 + successors) NodeHandles (== msgResp1 for numSiblings = 1)
    int32_t lookupCall;  // LookupCall (ovs_lookup_batch): the lookup ends at the last response, no route message
    int64_t bwCall;      // T(L*8/datarate) of a FindNodeCall, of the route message, and of a FindNodeResponse
    int64_t bwRoute;     // with 0..16 NodeHandles: the constant serialisation terms, precomputed on the host
    int64_t bwResp[17];
};


// SimTime(double) at scale 1e-9: truncation or round-half-up (recorded in every fixture)
__device__ __forceinline__ int64_t simtime_ns(double seconds, int round)
{
    const double x = __dmul_rn(seconds, 1e9);
    return round ? (int64_t)floor(__dadd_rn(x, 0.5)) : (int64_t)x;
}

// coordDelay = SimTime(0.001 * (float)||a-b||), SimpleNodeEntry.cc:145-153,186.
// Explicit _rn operations: no FMA contraction, identical rounding to the
// reference's x86-64 double arithmetic; sqrt correctly rounded, then to float.
__device__ __forceinline__ int64_t coord_ns(double ax, double ay, double bx, double by, int round)
{
    const double dx = __dsub_rn(ax, bx);
    const double dy = __dsub_rn(ay, by);
    const double s = __dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy));
    const float f = __double2float_rn(__dsqrt_rn(s));
    return simtime_ns(__dmul_rn(0.001, (double)f), round);
}

// T(L*8 / datarate): the serialisation delay of an L-byte packet
__device__ __forceinline__ int64_t bw_ns(int32_t bytes, double datarate, int round)
{
    return simtime_ns(__ddiv_rn((double)((int64_t)bytes * 8), datarate), round);
}

// 2*T(L*8/datarate) + 2*T(accessDelay) of a FindNodeResponse carrying `nodes` NodeHandles
__device__ __forceinline__ int64_t resp_ns(const DelayConsts& DC, int nodes)
{
    return 2 * bw_ns(DC.respBase + DC.respPerNode * nodes, DC.datarate, DC.round) + DC.access2;
}

__device__ __forceinline__ KeyRec load_rec(const KeyRec* __restrict__ recs, uint32_t i)
{
    const uint2* p = reinterpret_cast<const uint2*>(recs + i);
    const uint2 a = p[0], b = p[1], c = p[2];
    KeyRec r;
    r.w[0] = a.x; r.w[1] = a.y; r.w[2] = b.x; r.w[3] = b.y; r.w[4] = c.x; r.aux = c.y;
    return r;
}

// ---------------------------------------------------------------------------
// Converged-ring (ideal) Chord layout.  A hop at responder c normally reads ONE
// 64 B line: the finger entry closestPreceedingNode selects carries, besides the
// finger's index, everything the NEXT hop needs about that finger (key,
// coordinates, finger-row offset, the distances of its successor window), so
// the lookup never gathers the next node's record separately.  Ring distances
// d from a node enter as their top 64 bits (bits 96..159, top64()); a compare of
// D = K - c against such a distance is decided unless the top bits are equal,
// and then falls back to the exact keys in recs[] (a tie means K lies within
// 2^96 of a node: node-ID keys, or adjacent IDs closer than 2^96).
//
// NodeRec: per node -- lookup sources, successor hand-offs, shard arrivals.
struct alignas(64) NodeRec {
    uint32_t w[5];   // node key
    uint32_t row;    // offset of the node's finger row (valid on the arc that owns the row)
    double x, y;     // SimpleUnderlay coordinates
    uint64_t gS0;    // top64(succ0 - v)
    uint64_t gSL;    // top64(succ[ns-1] - v), ns = min(successorListSize, n - 1)
    uint64_t gP;     // top64((pred - v) mod 2^160)
};
static_assert(sizeof(NodeRec) == 64, "NodeRec is one 64 B line");

// FingerEnt: row(v)[159 - i] = finger i of v (non-trivial i >= i_lo(v)).
struct alignas(64) FingerEnt {
    uint32_t w[5];   // finger key
    uint32_t idx;    // finger node index
    double x, y;     // finger coordinates
    uint64_t gS0;    // the finger's own window distances (its NodeRec fields)
    uint64_t gSL;
    uint32_t row;    // the finger's own row offset
    uint32_t pad;
};
static_assert(sizeof(FingerEnt) == 64, "FingerEnt is one 64 B line");

// WinRec: per node of the arc, top64(succ_j - v) for j = 0..7 (unused slots all-ones);
// read only when K falls inside the successor window.
struct alignas(64) WinRec {
    uint64_t g[8];
};

__device__ __host__ __forceinline__ uint64_t top64(const K160& a) { return (uint64_t)a.w[3] | ((uint64_t)a.w[4] << 32); }

__device__ __forceinline__ double dbl(uint32_t lo, uint32_t hi) { return __hiloint2double((int)hi, (int)lo); }

// Chord device view.
//  recs[n]      : sorted node keys (24 B), aux = offset of the node's finger row
//  xy[n]        : SimpleUnderlay coordinates (fp64)
//  nodes[n]     : ideal mode -- NodeRec per node (64 B)
//  win[hi-lo]   : ideal mode -- WinRec per node of the arc [lo, hi)
//  frow[...]    : ideal mode -- CSR rows of FingerEnt (64 B),
//                 row(v)[159 - i] = finger i for the non-trivial positions
//                 i >= i_lo(v) = msb(succ0 - v) + 1 (trivial positions resolve to
//                 succ0, ChordFingerTable.cc:183-184)
//  general mode : pred[n], succ[n*sls], nsucc[n], fres[n*160] = getFinger(i) resolved
struct ChordView {
    const KeyRec* __restrict__ recs;
    const double2* __restrict__ xy;
    const NodeRec* __restrict__ nodes;
    const FingerEnt* __restrict__ frow;
    const WinRec* __restrict__ win;
    uint32_t lo;       // ideal: first node of this context's arc (win index base)
    const uint32_t* __restrict__ pred;
    const uint32_t* __restrict__ succ;
    const uint8_t* __restrict__ nsucc;
    const uint32_t* __restrict__ fres;
    uint32_t n;
    int32_t ns;        // ideal: min(successorListSize, n-1)
    int32_t sls;       // successor list stride (general)
    int32_t numFingerCandidates;
    // sharded rings (ovs_chord_shard_replicate): the top `ftl` finger levels of EVERY node,
    // ftop[v * ftl + (159 - i)] = finger i of v for i >= 160 - ftl, so a lookup's first hops --
    // the long jumps that cross arcs -- are decided on the rank that holds the lookup
    const FingerEnt* __restrict__ ftop;
    int32_t ftl;
};

constexpr int MAXSHARDS = 64;
struct ShardMap {
    uint64_t lo[MAXSHARDS + 1];   // arc r = [lo[r], lo[r+1]) of the sorted ring
    int n;
};

struct LookupConsts {
    int32_t hopCountMax;
    int32_t numSiblings;
    int32_t numRedundantNodes;
    int32_t recursive;          // routingType semi-/full-recursive: hop-by-hop route message
};

}  // namespace ovs
