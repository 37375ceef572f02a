// kad_route.hip -- K2, the Kademlia iterative-lookup kernel, for gfx950 (MI355X): the single-GPU
// batch and the shard step of the multi-GPU path (kad_shard.hip) are two instantiations of it.
//
// Compiled once per (alpha, exact) pair (build.py: -DOVS_KAD_A, -DOVS_KAD_EX) so the heavy
// instantiation sets build in parallel; kad.hip's kad_route and kad_shard.hip dispatch to them.
//
// K2 k_kad_route: one lane per lookup running OverSim's IterativePathLookup (IterativeLookup.cc:
// 760-1195, merge = true, parallel RPCs) against <= alpha pending FindNodeCalls ordered by
// simulated arrival time (int64 ns).  Each loop iteration processes the lookup's earliest event:
// a response is the responder's Kademlia::findNode (Kademlia.cc:1101-1246) merged into the
// LookupVector, then the sends it triggers (one 64 B KadNode line per target: its key,
// coordinates and isSiblingFor summary).  A findNode outside the sibling zone reads its main
// bucket's 96 B block on its own lane; the sibling-zone findNodes of the wave's lanes are
// evaluated together, four lanes each (kad_coop_sibzone, OVS_COOP_G).  Finished lanes refill from the wave's
// slice of the batch (ballot + popcount); the grid is persistent.
//
// Shard step (SHARD = true): the lookups of this rank (their sources lie on its arc) advance
// while their responders are local; a FindNodeCall to a node on another arc is staged as a
// request, and a lookup whose earliest event waits for such a result is suspended (state to HBM)
// until the next round.  At world size 1 every responder is local and the step is the
// single-GPU batch.
#include "kad_dev.hpp"
#include "kad_shard.hpp"

#include <algorithm>
#include <cstdio>
#include <vector>

#ifndef OVS_KAD_A
#error "kad_route.hip is compiled with -DOVS_KAD_A=<alpha> -DOVS_KAD_EX=<0|1> (oversim_amd/build.py)"
#endif
#ifndef OVS_KAD_WAVES
// minimum waves per SIMD the register allocator must allow (profiles/r02_b_kad: 3 beat 2 and 4)
#define OVS_KAD_WAVES 3
#endif
#ifndef OVS_KAD_MIG2
// the migration step (SM = 2) runs at OVS_KAD_WAVES = 3 waves/SIMD although its record load / store
// then spill 34 VGPRs (186 VGPRs at 2, no spill): with the dynamic tail the W = 8 model's E step is
// 9.72 ms per arc at 2 waves and 8.96 ms at 3 (same box, profiles/r06_shard/w8_E_mig_w2_vs_w3.txt);
// -DOVS_KAD_MIG2=2 builds it at 2 (A/B).  The A = 8 objects (alpha 5..8) keep 2: at 3 their spills
// come out as misaligned 64-bit scratch loads gfx950 rejects
#define OVS_KAD_MIG2 -1
#endif

namespace ovs {

namespace {

#ifdef OVS_KAD_TAIL
// tail census (-DOVS_KAD_TAIL builds): each persistent wave's start and exit on the real-time
// counter, read back and summarised by kad_launch (the spread of the waves' finishing times)
constexpr int KAD_TAIL_MAX = 1 << 16;
__device__ unsigned long long g_kad_tail[2 * KAD_TAIL_MAX];
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

struct SendNothing {
    __device__ __forceinline__ void operator()(int, uint32_t, bool) const {}
    __device__ __forceinline__ uint32_t boff(uint32_t, const KadNode&, const RespGeo& g, bool) const { return g.boff; }
};

struct AlwaysReady {
    __device__ __forceinline__ bool operator()(int, uint32_t, uint32_t) const { return true; }
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

// shard step: a response from a node off this arc is ready once its result was delivered
template <int C>
struct RemoteReady {
    const KadResN<C>* __restrict__ res;
    uint64_t base;
    uint32_t lo, hi;
    __device__ __forceinline__ bool operator()(int slot, uint32_t r, uint32_t) const
    {
        return (r >= lo && r < hi) || res[base + slot].ready != 0;
    }
};

// migration step: a response is processed here when its responder is on this arc or its findNode
// reads the responder's replicated top bucket (a row offset below tend, MigSend)
struct MigReady {
    uint32_t lo, hi, tend;
    __device__ __forceinline__ bool operator()(int, uint32_t r, uint32_t boff) const
    {
        return (r >= lo && r < hi) || boff < tend;
    }
};

// migration step: at send time the target's line says whether its findNode can be answered on any
// rank -- the [self] answer of a sibling (snapshot tables, numSiblings 1) or of an empty sibling
// table, or the full main bucket m above its sibling zone among the replicated top buckets
// (KMETA_TOPFULL): then the call's row offset names the replicated row (x * tl * bpb; the [self]
// answers read none), else the owner's row (valid on the owner, where the lookup then moves)
struct MigSend {
    int tl, bpb;
    bool full_ok;      // lookupRedundantNodes <= k: a full main bucket alone is the answer
    uint32_t lo, hi;   // this rank's arc
    __device__ __forceinline__ void operator()(int, uint32_t, bool) const {}
    __device__ __forceinline__ uint32_t boff(uint32_t x, const KadNode& rr, const RespGeo& g, bool sb) const
    {
        if (tl > 0) {
            if (sb || g.nsib == 0) return 0u;
            const int j = KEYBITS - 1 - g.m;
            if (full_ok && g.m > g.endIndex && j < tl && ((rr.meta >> (KMETA_TOPFULL_SHIFT + j)) & 1u))
                return x * (uint32_t)(tl * bpb);
        }
        // the owner's row: valid on the owner only.  Off this arc the call names no row here (NONE
        // >= tend: MigReady holds the lookup until it has moved to the owner, which re-reads the
        // responder's own line, and kad_find_node_blk never reads a row through it)
        return (x >= lo && x < hi) ? g.boff : NONE;
    }
};

// shard step: a FindNodeCall to a node off this arc becomes a request to its owner, staged in the
// call's slot (a slot carries at most one request per round: a response cannot be ready in the
// round it is requested)
template <int C>
struct ShardSend {
    KadResN<C>* __restrict__ res;
    uint64_t base;
    const K160* K;
    const uint64_t* __restrict__ shard_lo;
    int nsh;
    uint32_t lo, hi;
    ovs_kad_req* __restrict__ stage;
    uint8_t* __restrict__ rtag;
    uint32_t pad;   // LookupCall: bit 31 | numSiblings (the responder's findNode argument); 0 for KBR routes
    __device__ __forceinline__ uint32_t boff(uint32_t, const KadNode&, const RespGeo& g, bool) const { return g.boff; }
    __device__ __forceinline__ void operator()(int slot, uint32_t x, bool isTo) const
    {
        if (isTo || (x >= lo && x < hi)) return;   // a timeout carries no result; a local findNode runs here
        res[base + slot].ready = 0u;
        ovs_kad_req q;
        for (int w = 0; w < 5; ++w) q.key[w] = K->w[w];
        q.node = x;
        q.tag = (uint32_t)(base + slot);
        q.pad = pad;
        stage[base + slot] = q;
        int r = 0;
        for (int i = 1; i < nsh; ++i) r += ((uint64_t)x >= shard_lo[i]) ? 1 : 0;
        rtag[base + slot] = (uint8_t)r;
    }
};

struct KadRouteIO {
    const K160* __restrict__ qkeys;
    const uint32_t* __restrict__ qsrc;
    uint64_t nq;             // lookups (single GPU) / entries of the round's list (shard step)
    uint64_t chunk;
    ovs_route_out* __restrict__ out;
    uint32_t* __restrict__ hopseq;
    uint32_t* __restrict__ rpcs_out;
    uint32_t* __restrict__ sib_out;
    // shard step
    void* st;                               // suspended lookups, KadStateWords<A, C> words each (SoA)
    uint64_t sstride;                       // their word stride (the batch's lookups)
    uint8_t* __restrict__ act;               // 2 not started, 1 suspended in st, 0 never runs
    void* res;                               // KadResN<C>[nlook * A]
    const uint64_t* __restrict__ list;      // this round's lookups (indices), *nlist_dev of them
    const unsigned long long* __restrict__ nlist_dev;
    const uint32_t* __restrict__ qids;
    const uint64_t* __restrict__ shard_lo;
    int nsh;
    ovs_kad_req* __restrict__ rstage;
    uint8_t* __restrict__ rtag;
    ovs_done_rec* __restrict__ dstage;
    uint8_t* __restrict__ ltag;
    // migration step (SM = 2): this round's input -- migrated lookup records (min, nq of them) or,
    // in a batch's first round, keys and sources (qkeys / qsrc, lookup q has id fqid + q); per input
    // one outcome at its own index: a record moving to rank mtag[q] (mstage) or a done record
    // (dstage, mtag[q] = nsh)
    const uint32_t* __restrict__ min;
    uint32_t fqid;
    uint32_t* __restrict__ mstage;
    uint8_t* __restrict__ mtag;
    int me;
    int tl, bpb, full_ok;
    // dynamic tail (single-GPU batches, dyn != nullptr): static slices cover [0, dyn_from), the rest
    // goes out KAD_DYN_CH lookups at a time from the zeroed counter *dyn (as K1's, chord.hip; K2's
    // lookups run longer, so half K1's chunk: E 4.01 -> 3.97 ms against 64, profiles/r06_dyn/tune.txt)
    unsigned long long* dyn;
    uint64_t dyn_from;
};

#ifndef KAD_DYN_CH
#define KAD_DYN_CH 32
#endif
#ifndef KAD_DYN_STATIC
#define KAD_DYN_STATIC 0.70
#endif

// SH: explicit tables with short sibling tables (KadTables::maybe_short): a send may have to count
// the responder's scan (kad_response_size); snapshot tables never do
// SM: 0 single GPU; 1 shard step, request/response (lookups stay home, remote findNodes answered by
// their owners); 2 shard step, migration (a lookup moves to the rank whose rows its next findNode
// needs; the replicated top buckets answer the long first hops anywhere)
// DEF (single GPU, one-way, snapshot tables): the default configuration's lookup rules (default.ini:
// hopCountMax 50, lookupRedundantNodes = k = 8, numSiblings 1, strictParallelRpcs, visitOnlyOnce,
// acceptLateSiblings and merge on, the useAll / newRpcOn* / finishOnFirstUnchanged rules off) as
// compile-time constants (alpha is A already); kad_is_def_lc picks it
__host__ __device__ inline bool kad_is_def_lc(const KadLC& L)
{
    return L.hopCountMax == 50 && L.numSiblings == 1 && L.redundant == 8 && L.strict == 1 && L.visitOnlyOnce == 1 &&
           L.acceptLateSiblings == 1 && L.useAll == 0 && L.merge == 1 && L.newOnResp == 0 && L.newOnTimeout == 0 &&
           L.finishOnFirst == 0 && L.maxRedundantLocal == 8;
}
__device__ __forceinline__ KadLC kad_def_lc(KadLC L)
{
    L.hopCountMax = 50; L.numSiblings = 1; L.redundant = 8; L.strict = 1; L.visitOnlyOnce = 1; L.acceptLateSiblings = 1;
    L.useAll = 0; L.merge = 1; L.newOnResp = 0; L.newOnTimeout = 0; L.finishOnFirst = 0; L.maxRedundantLocal = 8;
    return L;
}

template <int A, bool RECORD, bool EX, bool LK, int SM, int C, bool SH, bool DEF = false>
// the shard step's exact-compare and LookupCall instantiations run at 2 waves/SIMD: their HBM state
// traffic and request staging need the registers (at 3 the exact-compare ones spilled in misaligned
// 96-bit pieces gfx950 rejects, the LookupCall one 109 VGPRs); the one-way route step keeps K2's 3
__global__ __launch_bounds__(256, ((SM && (EX || LK)) || C > 8 || (SM == 2 && (OVS_KAD_MIG2 == 2 || A > 4))) ? 2 : OVS_KAD_WAVES) void k_kad_route(KadView V, DelayConsts DC, KadLC LC0,
                                                                            KadRouteIO io)
{
    const KadLC LC = DEF ? kad_def_lc(LC0) : LC0;
    constexpr bool SHARD = SM == 1;
    constexpr bool MIG = SM == 2;
    const int lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    uint64_t nq = io.nq, chunk = io.chunk;
    if (SHARD) {
        // the round's list length is the previous round's device count (no host round trip)
        nq = *io.nlist_dev;
        const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
        chunk = (nq + waves - 1) / waves;
    }
    uint64_t cursor = wave * chunk;
    const bool dyn = SM != 1 && io.dyn != nullptr;      // single GPU and the migration step
    uint64_t end = min(cursor + chunk, dyn ? io.dyn_from : nq);
    bool more = dyn;                                      // dynamic chunks may be left
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int ns = LK ? LC.numSiblings : 1;
    uint32_t* st = static_cast<uint32_t*>(io.st);

#ifndef OVS_NOCOOP
    __shared__ CoopLds lds;
#else
    CoopLds& lds = *(CoopLds*)nullptr;    // experiment build: never touched
#endif
    bool active = false;
    bool dead = false;     // shard step: a listed lookup that does not run (source off the arc)
    bool go = false;       // migration step: a fresh lookup whose source lies off this arc moves at once
    uint64_t q = 0;
    uint32_t qid = 0;
    KadLookup<A, C> L;

    while (true) {
        const uint64_t need = __ballot(!active);
        if (SM != 1 && more && need != 0 && cursor >= end) {
            // the static slice is spent: the next dynamic chunk (one atomic a chunk, lane 0)
            unsigned long long b = 0;
            if (lane == 0) b = atomicAdd(io.dyn, (unsigned long long)KAD_DYN_CH);
            const uint64_t nb = io.dyn_from + (((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                                               (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)b));
            if (nb < nq) {
                cursor = nb;
                end = min(nb + (uint64_t)KAD_DYN_CH, nq);
            } else {
                more = false;
            }
        }
        if (need != 0 && cursor < end) {
            const uint64_t mine = cursor + (uint64_t)__popcll(need & lt_mask);
            if (!active && mine < end) {
                active = true;
                if (MIG) {
                    q = mine;
                    if (io.min) {
                        qid = kad_rec_get(L, io.min + q * (uint64_t)KadRecWords<A, C>::value);
                    } else {
                        qid = io.fqid + (uint32_t)q;
                        kad_lookup_init(L, io.qkeys[q], io.qsrc[q], V.xy);
                        // the start is the source's own findNode: its rows are on its owner
                        go = L.S < V.lo || L.S >= V.hi;
                    }
                } else if (SHARD) {
                    q = io.list[mine];
                    const uint8_t a = io.act[q];
                    dead = a == 0;
#if !defined(OVS_SHARD_NOSUSPEND) && !defined(OVS_SHARD_NOLOAD)
                    if (a == 2) kad_lookup_init(L, io.qkeys[q], io.qsrc[q], V.xy);   // first visit
                    else if (a == 1) kad_state_get(L, st, io.sstride, q);
#else
                    if (a) kad_lookup_init(L, io.qkeys[q], io.qsrc[q], V.xy);   // cost experiment (W = 1 only)
#endif
                } else {
                    q = mine;
                    kad_lookup_init(L, io.qkeys[q], io.qsrc[q], V.xy);
                }
            }
            cursor += (uint64_t)__popcll(need);
        }
        // (a `continue` for a wave without work here, instead of the dead flag, made the compiler
        // spill 240 B of the lookup state per lane)
        if (!__any(active)) break;

        // phase 1 (per lane): the earliest event up to its findNode
        int ph = KEV_IDLE;
        KadEv ev;
        ev.r = 0; ev.geo = 0; ev.boff = 0; ev.e = 0; ev.num = 0; ev.numR = 0; ev.pre = 0; ev.start = false;
        bool coop = false;
        if (active && !dead && !go && !kad_lookup_done(L)) {
            const HopRecorder<RECORD> rec{io.hopseq, q * (uint64_t)LC.hopCountMax, LC.hopCountMax};
            // An event that only accounts (a response of an older step, a timeout with calls still
            // pending) leaves the lane idle through the findNode, merge and send phases: the lane
            // takes its next event in the same iteration instead (at most A pending events).  With
            // α = 3 these are ~40 % of the events (most parallel responses arrive a step late).
#ifndef OVS_KAD_ONE_EVENT
            for (int r = 0; r < A; ++r) {
#endif
                if (SHARD) {
                    const RemoteReady<C> rd{static_cast<const KadResN<C>*>(io.res), q * A, V.lo, V.hi};
                    ph = kad_event_begin<A, EX, LK>(L, V, DC, LC, rd, rec, ev);
                } else if (MIG) {
                    ph = kad_event_begin<A, EX, LK>(L, V, DC, LC, MigReady{V.lo, V.hi, V.tend}, rec, ev);
                } else {
                    ph = kad_event_begin<A, EX, LK>(L, V, DC, LC, AlwaysReady{}, rec, ev);
                }
#ifndef OVS_KAD_ONE_EVENT
                if (ph != KEV_HANDLED || kad_lookup_done(L)) break;
            }
#endif
            const bool local = !SM || (ev.r >= V.lo && ev.r < V.hi);
            // migration step: a call sent from another rank names no row of this one (MigSend:
            // NONE); its responder's row here is the responder's own line's
            if (MIG && ph == KEV_FIND && local && ev.boff >= V.tend) ev.boff = V.nodes[ev.r].boff;
            coop = ph == KEV_FIND && local && kad_find_is_coop(V, ev.r, ev.rg(), ev.sb(), ns, rb_pre(ev.pre), rb_r0(ev.pre));
        }

#ifdef OVS_KAD_STATS
        {   // lane occupancy of the phases (cost experiment): [0] wave iterations, [1] active lanes,
            // [2] per-lane findNodes, [3] cooperative findNodes, [4] send-only events
            const uint64_t act = __ballot(active), lf = __ballot(active && ph == KEV_FIND && !coop);
            const uint64_t cp = __ballot(coop), se = __ballot(active && ph == KEV_SENDS);
            if ((threadIdx.x & 63) == 0) {
                atomicAdd(&g_kad_stats[0], 1ull);
                atomicAdd(&g_kad_stats[1], (unsigned long long)__popcll(act));
                atomicAdd(&g_kad_stats[2], (unsigned long long)__popcll(lf));
                atomicAdd(&g_kad_stats[3], (unsigned long long)__popcll(cp));
                atomicAdd(&g_kad_stats[4], (unsigned long long)__popcll(se));
            }
        }
#endif
        // phase 2 (whole wave): the sibling-zone findNodes (results in LDS).  The exact-compare
        // instantiation (networks with IDs sharing their top 63 bits) keeps the per-lane scan: its
        // tie fallbacks in the cooperative merge made the register allocator emit misaligned
        // 96-bit spills that gfx950 rejects.
#ifndef OVS_NOCOOP
        if constexpr (!EX && C == 8) {
            kad_coop_sibzone<EX>(V, coop, ev.r, ev.geo, ev.boff, ev.pre, L.K, lds);
#ifdef OVS_DUP_COOP
            kad_coop_sibzone<EX>(V, coop, ev.r, ev.geo, ev.boff, ev.pre, L.K, lds);   // cost experiment
#endif
        } else {
            coop = false;
        }
#else
        coop = false;
#endif

        // phase 3 (per lane): the rest of the findNode, the LookupVector, the sends
        if (SHARD && dead) {
            active = false;
            dead = false;
        } else if (MIG && active && go) {
            // a fresh lookup whose source lies off this arc: to the source's owner before it starts
            kad_rec_put(io.mstage + q * (uint64_t)KadRecWords<A, C>::value, qid, L);
            int r = 0;
            for (int i = 1; i < io.nsh; ++i) r += ((uint64_t)L.S >= io.shard_lo[i]) ? 1 : 0;
            io.mtag[q] = (uint8_t)r;
            active = false;
            go = false;
        } else if (active) {
            SVec<C> res;
            res.n = 0;
            res.used = 0;
            int num = -1;
            if (ph == KEV_FIND) {
                int n;
                BlkN<C> fb;
                if (coop) {
                    if constexpr (C == 8) coop_get(lds.res, threadIdx.x, fb);
                    // the candidates findNode saw: the row entries past the prefix's blocks count too
                    const RespGeo g = ev.rg();
                    const int tot = g.nsib + 1, rd = min(tot, kad_row_read(rb_pre(ev.pre))) - rb_r0(ev.pre);
                    n = kad_coop_finish<EX>(V, g, L.K, ev.numR, ev.sb(), ns, fb, (int)lds.rcnt[threadIdx.x] + tot - rd);
#ifndef OVS_SHARD_NOREMOTE
                } else if (SHARD && !(ev.r >= V.lo && ev.r < V.hi)) {
                    // the owner's answer, delivered by k_kad_shard_deliver
                    const KadResN<C>& rr = static_cast<const KadResN<C>*>(io.res)[q * A + ev.e];
                    n = (int)rr.count;
#pragma unroll
                    for (int k = 0; k < C; ++k) {
                        fb.x[k] = k < n ? rr.nodes[k] : NONE;
                        fb.d[k] = k < n ? rr.dist[k] : ~0ull;
                    }
#endif
                } else {
                    // in the sibling zone only c and the row prefix can enter the answer (ev.pre)
                    const RespGeo g = ev.rg();
                    n = kad_find_node_blk<EX, C>(V, ev.r, g, L.K, ev.numR, ev.sb(), fb, ns,
                                                 g.m <= g.endIndex ? rb_pre(ev.pre) : -1, rb_r0(ev.pre));
#ifdef OVS_DUP_LANEFIND
                    {   // cost experiment: the per-lane findNode again
                        K160 K2 = L.K;
                        asm volatile("" : "+v"(K2.w[0]));
                        BlkN<C> b2;
                        const int n2 = kad_find_node_blk<EX, C>(V, ev.r, g, K2, ev.numR, ev.sb(), b2, ns,
                                                                g.m <= g.endIndex ? rb_pre(ev.pre) : -1, rb_r0(ev.pre));
                        uint32_t z = (uint32_t)n2;
                        for (int k = 0; k < C; ++k) z ^= b2.x[k] ^ (uint32_t)b2.d[k] ^ (uint32_t)(b2.d[k] >> 32);
                        asm volatile("" :: "v"(z));
                    }
#endif
                }
#pragma unroll
                for (int k = 0; k < C; ++k) { res.idx[k] = fb.x[k]; res.d[k] = fb.d[k]; }
                res.n = n;
                num = kad_event_after_find<A, EX, LK>(L, V, LC, ev, res);
            } else if (ph == KEV_SENDS) {
                num = ev.num;
            }
#ifdef OVS_KAD_STATS
            {   // [5] lanes sending, [6] the wave's send-loop trips (max num), [7] sends wanted
                const uint64_t t1 = __ballot(num >= 1), t2 = __ballot(num >= 2), t3 = __ballot(num >= 3);
                const uint64_t all = __ballot(true);
                if ((int)(threadIdx.x & 63) == __ffsll((long long)all) - 1) {
                    atomicAdd(&g_kad_stats[5], (unsigned long long)__popcll(t1));
                    atomicAdd(&g_kad_stats[6], (unsigned long long)((t1 != 0) + (t2 != 0) + (t3 != 0)));
                    atomicAdd(&g_kad_stats[7], (unsigned long long)(__popcll(t1) + __popcll(t2) + __popcll(t3)));
                }
            }
#endif
            if (num >= 0) {
                if (SHARD) {
                    const ShardSend<C> on{static_cast<KadResN<C>*>(io.res), q * A, &L.K, io.shard_lo, io.nsh, V.lo,
                                          V.hi, io.rstage, io.rtag, LK ? (0x80000000u | (uint32_t)ns) : 0u};
                    kad_send_rpcs<A, EX, LK, SH>(L, V, DC, LC, num, on);
                } else if (MIG) {
                    kad_send_rpcs<A, EX, LK, SH>(L, V, DC, LC, num, MigSend{io.tl, io.bpb, io.full_ok != 0, V.lo, V.hi});
                } else {
                    kad_send_rpcs<A, EX, LK, SH>(L, V, DC, LC, num, SendNothing{});
                }
            }
            if (kad_lookup_done(L)) {
                const ovs_route_out o = kad_lookup_output(L, V, DC, LC);
                const bool ok = o.status == OVS_LOOKUP_OK;
                if (LK) {
                    // the LookupResponse's sibling vector: the answering sibling's findNode result
                    // (an exact-key lookup: the key's node); res is this iteration's answer
                    if (ns == 0) {
                        io.sib_out[q] = ok ? L.result : NONE;
                    } else {
                        uint32_t* row = io.sib_out + q * (uint64_t)ns;
#pragma unroll
                        for (int j = 0; j < 8; ++j)
                            if (j < ns) row[j] = (ok && j < res.n) ? res.idx[j] : NONE;
                    }
                }
                if (MIG) {
                    ovs_done_rec dr;
                    dr.qid = qid;
                    dr.pad = L.nsent;
                    dr.out = o;
                    io.dstage[q] = dr;
                    io.mtag[q] = (uint8_t)io.nsh;
                } else if (SHARD) {
                    ovs_done_rec dr;
                    dr.qid = io.qids[q];
                    dr.pad = L.nsent;     // the lookup's FindNodeCalls (local and remote)
                    dr.out = o;
                    if (LK) {
                        uint32_t cnt = 0;
                        if (ns == 0) cnt = ok ? 1u : 0u;
                        else cnt = ok ? (uint32_t)min(res.n, ns) : 0u;
                        ovs_lookup_out lo;
                        lo.num_siblings = cnt;
                        lo.hops = o.hops;
                        lo.status = o.status;
                        lo.is_valid = ok ? 1 : 0;
                        lo.latency_ns = ok ? o.latency_ns : -1;
                        __builtin_memcpy(&dr.out, &lo, sizeof lo);
                    }
                    io.dstage[q] = dr;
                    io.ltag[q] = 0;
                } else {
                    io.out[q] = o;
                    if (io.rpcs_out) io.rpcs_out[q] = L.nsent;
                }
                active = false;
            } else if (MIG && ph == KEV_WAIT) {
                // the earliest event needs the rows of a responder off this arc: the lookup moves to
                // that responder's owner (its record staged at its input index, compacted by rank)
                kad_rec_put(io.mstage + q * (uint64_t)KadRecWords<A, C>::value, qid, L);
                int r = 0;
                for (int i = 1; i < io.nsh; ++i) r += ((uint64_t)ev.r >= io.shard_lo[i]) ? 1 : 0;
                io.mtag[q] = (uint8_t)r;
                active = false;
            } else if (SHARD && ph == KEV_WAIT) {
                // the earliest event waits for an owner's answer: suspended until the next round
#if !defined(OVS_SHARD_NOSUSPEND) && !defined(OVS_SHARD_NOSTORE)
                kad_state_put(st, io.sstride, q, L);
#endif
                io.act[q] = 1;
                io.ltag[q] = 1;
                active = false;
            }
        }
    }
#ifdef OVS_KAD_TAIL
    ovs_tail_mark(g_kad_tail, KAD_TAIL_MAX, 1);
#endif
}

}  // namespace

// persistent grid: as many waves as are resident, each with a contiguous slice of the batch
template <int A, bool RECORD, bool EX, bool LK, int SM, int C = 8, bool SH = true, bool DEF = false>
static hipError_t kad_launch(const KadView& V, const DelayConsts& DC, const KadLC& LC, KadRouteIO io, int num_cu,
                             hipStream_t st)
{
    // occupancy of this instantiation (the same on every gfx950 device; a function-local static is
    // initialised once, thread-safely)
    static const int bpc = [] {
        int b = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_kad_route<A, RECORD, EX, LK, SM, C, SH, DEF>, 256, 0) !=
                hipSuccess ||
            b < 1)
            b = 1;
        return b;
    }();
#ifndef OVS_KAD_OVERSUB
#define OVS_KAD_OVERSUB 1
#endif
    // OVS_KAD_OVERSUB > 1 (A/B builds): that many waves per resident slot, each with a shorter slice
    const uint64_t waves = (uint64_t)num_cu * (uint64_t)bpc * 4 * (SM ? 1 : OVS_KAD_OVERSUB);
    io.chunk = (io.nq + waves - 1) / waves;
    if (io.chunk < 1) io.chunk = 1;
    const uint64_t need_waves = (io.nq + io.chunk - 1) / io.chunk;
    const uint64_t blocks = (need_waves + 3) / 4;
    if (SM != 1 && io.dyn) {
        // static slices cover KAD_DYN_STATIC of the batch, the rest goes out in chunks (small batches: static)
        const uint64_t cs = (uint64_t)((double)io.nq * KAD_DYN_STATIC) / (blocks * 4);
        if (cs < (uint64_t)KAD_DYN_CH) {
            io.dyn = nullptr;
        } else {
            io.chunk = cs;
            io.dyn_from = cs * blocks * 4;
        }
    }
#ifdef OVS_KAD_STATS
    unsigned long long z[8] = {};
    hipMemcpyToSymbolAsync(HIP_SYMBOL(g_kad_stats), z, sizeof z, 0, hipMemcpyHostToDevice, st);
#endif
    hipLaunchKernelGGL((k_kad_route<A, RECORD, EX, LK, SM, C, SH, DEF>), dim3((unsigned)blocks), dim3(256), 0, st, V, DC, LC,
                       io);
#ifdef OVS_KAD_TAIL
    if (!SM) {
        const uint64_t nw = blocks * 4 < (uint64_t)KAD_TAIL_MAX ? blocks * 4 : (uint64_t)KAD_TAIL_MAX;
        std::vector<unsigned long long> tt(2 * nw);
        hipMemcpyFromSymbolAsync(tt.data(), HIP_SYMBOL(g_kad_tail), sizeof(unsigned long long) * 2 * nw, 0,
                                 hipMemcpyDeviceToHost, st);
        hipStreamSynchronize(st);
        unsigned long long t0 = ~0ull;
        std::vector<double> fin;
        for (uint64_t w = 0; w < nw; ++w) t0 = tt[2 * w + 1] < t0 ? tt[2 * w + 1] : t0;
        for (uint64_t w = 0; w < nw; ++w) fin.push_back((double)(tt[2 * w + 1] - t0) * 0.01);   // 100 MHz -> us
        std::sort(fin.begin(), fin.end());
        auto pct = [&](double f) { return fin[(size_t)(f * (fin.size() - 1))]; };
        fprintf(stderr, "kadtail waves=%llu chunk=%llu finish_us_after_first_exit p0=%.1f p10=%.1f p50=%.1f p90=%.1f p99=%.1f max=%.1f\n",
                (unsigned long long)nw, (unsigned long long)io.chunk, pct(0), pct(0.1), pct(0.5), pct(0.9), pct(0.99),
                fin.back());
    }
#endif
#ifdef OVS_KAD_STATS
    hipMemcpyFromSymbolAsync(z, HIP_SYMBOL(g_kad_stats), sizeof z, 0, hipMemcpyDeviceToHost, st);
    hipStreamSynchronize(st);
    fprintf(stderr, "kadstats nq=%llu iters=%llu active=%llu lanefind=%llu coop=%llu sendonly=%llu sending=%llu sendtrips=%llu sends=%llu\n",
            (unsigned long long)io.nq, z[0], z[1], z[2], z[3], z[4], z[5], z[6], z[7]);
#endif
    return hipGetLastError();
}

template <int A, bool EX>
hipError_t kad_route_launch(const KadView& V, const DelayConsts& DC, const KadLC& LC, const K160* qkeys,
                            const uint32_t* qsrc, uint64_t nq, ovs_route_out* out, uint32_t* hopseq, uint32_t* rpcs,
                            uint32_t* sibs, int num_cu, hipStream_t st, unsigned long long* dyn)
{
    KadRouteIO io{};
    io.qkeys = qkeys; io.qsrc = qsrc; io.nq = nq; io.out = out; io.hopseq = hopseq; io.rpcs_out = rpcs; io.sib_out = sibs;
    io.dyn = dyn;
    // LookupCall batches (sibs != nullptr) record no hop sequence.  KademliaLarge (k or
    // lookupRedundantNodes above 8) takes the 16-entry LookupVector / findNode instantiation.
    if (LC.redundant > 8 || LC.maxRedundantLocal > 8) {
        if (sibs) return kad_launch<A, false, EX, true, 0, 16>(V, DC, LC, io, num_cu, st);
        if (hopseq) return kad_launch<A, true, EX, false, 0, 16>(V, DC, LC, io, num_cu, st);
        return kad_launch<A, false, EX, false, 0, 16>(V, DC, LC, io, num_cu, st);
    }
    if (V.maybe_short) {
        if (sibs) return kad_launch<A, false, EX, true, 0, 8, true>(V, DC, LC, io, num_cu, st);
        if (hopseq) return kad_launch<A, true, EX, false, 0, 8, true>(V, DC, LC, io, num_cu, st);
        return kad_launch<A, false, EX, false, 0, 8, true>(V, DC, LC, io, num_cu, st);
    }
    if (sibs) return kad_launch<A, false, EX, true, 0, 8, false>(V, DC, LC, io, num_cu, st);
    if (hopseq) return kad_launch<A, true, EX, false, 0, 8, false>(V, DC, LC, io, num_cu, st);
#ifndef OVS_KAD_NO_DEF
    if (kad_is_def_lc(LC)) return kad_launch<A, false, EX, false, 0, 8, false, true>(V, DC, LC, io, num_cu, st);
#endif
    return kad_launch<A, false, EX, false, 0, 8, false>(V, DC, LC, io, num_cu, st);
}

template <int A, bool EX>
hipError_t kad_shard_step_launch(const KadView& V, const DelayConsts& DC, const KadLC& LC, const KadShardStepArgs& a,
                                 int num_cu, hipStream_t st)
{
    if (a.nlist_max == 0) return hipSuccess;
    KadRouteIO io{};
    io.nq = a.nlist_max;     // sizes the grid; the kernel reads the list length from nlist_dev
    io.sib_out = a.sib_out;
    io.st = a.st; io.sstride = a.nlist_max; io.act = a.act; io.qkeys = a.qkeys; io.qsrc = a.qsrc; io.res = a.res; io.list = a.list; io.nlist_dev = a.nlist_dev; io.qids = a.qids;
    io.shard_lo = a.shard_lo; io.nsh = a.nsh;
    io.rstage = a.rstage; io.rtag = a.rtag; io.dstage = a.dstage; io.ltag = a.ltag;
    // sharded networks are snapshot builds: never short.  KademliaLarge (k or lookupRedundantNodes
    // above 8) takes the 16-entry instantiation, its results travel as ovs_kad_resp16
    if (V.maybe_short) return hipErrorNotSupported;
    if (LC.redundant > 8 || LC.maxRedundantLocal > 8) {
        if (a.sib_out) return kad_launch<A, false, EX, true, 1, 16, false>(V, DC, LC, io, num_cu, st);
        return kad_launch<A, false, EX, false, 1, 16, false>(V, DC, LC, io, num_cu, st);
    }
    if (a.sib_out) return kad_launch<A, false, EX, true, 1, 8, false>(V, DC, LC, io, num_cu, st);
    return kad_launch<A, false, EX, false, 1, 8, false>(V, DC, LC, io, num_cu, st);
}

template <int A, bool EX>
hipError_t kad_mig_step_launch(const KadView& V, const DelayConsts& DC, const KadLC& LC, const KadMigStepArgs& a,
                               int num_cu, hipStream_t st)
{
    if (a.nin == 0) return hipSuccess;
    KadRouteIO io{};
    io.nq = a.nin;
    io.qkeys = a.fkeys; io.qsrc = a.fsrc; io.fqid = a.fqid; io.min = a.in;
    io.shard_lo = a.shard_lo; io.nsh = a.nsh; io.me = a.me;
    io.mstage = a.mstage; io.mtag = a.mtag; io.dstage = a.dstage;
    io.tl = V.tl; io.bpb = V.bpb; io.full_ok = LC.redundant <= V.k ? 1 : 0;
    io.dyn = a.dyn;
    // one-way routes on snapshot tables, findNode results of up to 8 nodes (kad_mig_supported)
    if (V.maybe_short || LC.redundant > 8 || LC.maxRedundantLocal > 8) return hipErrorNotSupported;
    return kad_launch<A, false, EX, false, 2, 8, false>(V, DC, LC, io, num_cu, st);
}

template hipError_t kad_mig_step_launch<OVS_KAD_A, OVS_KAD_EX != 0>(const KadView&, const DelayConsts&, const KadLC&,
                                                                    const KadMigStepArgs&, int, hipStream_t);
template hipError_t kad_route_launch<OVS_KAD_A, OVS_KAD_EX != 0>(const KadView&, const DelayConsts&, const KadLC&,
                                                                 const K160*, const uint32_t*, uint64_t, ovs_route_out*,
                                                                 uint32_t*, uint32_t*, uint32_t*, int, hipStream_t,
                                                                 unsigned long long*);
template hipError_t kad_shard_step_launch<OVS_KAD_A, OVS_KAD_EX != 0>(const KadView&, const DelayConsts&, const KadLC&,
                                                                      const KadShardStepArgs&, int, hipStream_t);

}  // namespace ovs
