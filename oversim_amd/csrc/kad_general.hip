// kad_general.hip -- K2g: Kademlia lookups over the general tables (ovs_kad_load_tables_csr) for
// gfx950 (MI355X): b > 1 (routingBucketIndex's b-bit digits, numBuckets = (2^b - 1) * (160 / b),
// Kademlia.cc:176, 357-382) and the fork's bucketType variants nr128 / nkademlia
// (routingBucketSize 384-411, routingAdd 620-664), whose buckets may hold far more than the 16
// entries K2's two 96 B blocks carry.
//
// The lookup state machine is K2's (kad_dev.hpp: kad_event_begin / kad_event_after_find /
// kad_send_rpcs -- IterativeLookup.cc:133-1195 with merge, parallel RPCs, int64-ns event order);
// only Kademlia::findNode (Kademlia.cc:1101-1246) differs: it walks the CSR buckets in the
// reference's order -- the main bucket, then (main bucket at or above the sibling zone, or a short
// result) the buckets startIndex .. endIndex other than the main one, the sibling table and the
// node itself, then the buckets above the main one while the result is short -- inserting each
// member into the XOR-sorted result by its top-64 distance (exact compare on ties, cand_lt<EX>).
// One lane per lookup, to completion: a variant path, not the tuned K2 (no cooperative
// sibling-zone pass, no persistent refill); parity first (tests/test_gpu_kad_general.py).
#include "kad_dev.hpp"

namespace ovs {

namespace {

struct GSendNothing {
    __device__ __forceinline__ void operator()(int, uint32_t, bool) const {}
    __device__ __forceinline__ uint32_t boff(uint32_t, const KadNode&, const RespGeo& g, bool) const { return g.boff; }
};

struct GAlwaysReady {
    __device__ __forceinline__ bool operator()(int, uint32_t, uint32_t) const { return true; }
};

template <bool RECORD>
struct GHopRecorder {
    uint32_t* __restrict__ hopseq;
    uint64_t base;
    int hcm;
    __device__ __forceinline__ void operator()(int h, uint32_t r) const
    {
        if (RECORD && h < hcm) hopseq[base + h] = r;
    }
};

// Kademlia::findNode(K, numRedundantNodes, numSiblings) at node c (nsib siblings) over the general
// tables; numSiblings = -1: an exhaustive-iterative call (resultSize = numRedundantNodes, no
// siblings flag).  Returns the result size.
template <bool EX, int C>
__device__ int kadg_find_node(const KadView& V, const KadGenView& G, uint32_t c, int nsib, const K160& K,
                              int numRedundant, bool sib, int numSiblings, SVec<C>& res)
{
    svec_clear(res);
    const K160 me = node_key(V.nodes, c);
    if (nsib == 0) {                       // an empty sibling table answers [self] (Kademlia.cc:1133-1137)
        svec_add<C, EX>(res, 1, c, dist_hi(me, K), K, V.nodes);
        return 1;
    }
    // resultSize (Kademlia.cc:1125-1131)
    const int rs = numSiblings < 0 ? numRedundant : sib ? (numSiblings ? numSiblings : 1) : numRedundant;
    const int cap = rs < C ? rs : C;
    const K160 D = k_xor(me, K);
    const int mainI = kad_bucket_index(D, G.b, false);
    const int startI = kad_bucket_index(D, G.b, true);
    const int endI = G.gend[c];
    const uint64_t kt = ktop(K);
    const uint64_t row = (uint64_t)c * (uint64_t)G.nb;
    auto add_bucket = [&](int m) {
        const uint32_t a = G.goff[row + m], z = G.goff[row + m + 1];
        for (uint32_t e = a; e < z; ++e) svec_add<C, EX>(res, cap, G.gidx[e], dclamp(G.gtop[e] ^ kt), K, V.nodes);
    };
    if (mainI >= 0) add_bucket(mainI);
    if (startI >= endI || res.n < cap) {
        for (int m = startI; m >= endI && m >= 0; --m)
            if (m != mainI) add_bucket(m);
        const KadBlk* Lr = V.sibb + (uint64_t)c * V.sbn;     // c itself, then its siblings
        for (int i = 0; i <= nsib; ++i) {
            const KadBlk& bk = Lr[i / KBLK];
            svec_add<C, EX>(res, cap, bk.idx[i % KBLK], dclamp(bk.top[i % KBLK] ^ kt), K, V.nodes);
        }
    }
    for (int m = mainI + 1; res.n < cap && m < G.nb; ++m) add_bucket(m);
    return res.n;
}

// the FindNodeResponse size of a call's target: resultSize unless the target's scan sees fewer
// candidates, which needs a sibling table shorter than resultSize - 1 (then the scan is counted)
template <bool EX, int C>
struct KadGenSizer {
    KadGenView G;
    __device__ __forceinline__ int operator()(const KadView& V, uint32_t x, const RespGeo& g, const K160& K, int rs,
                                              bool sib, int ns) const
    {
        if (g.nsib == 0 || (sib && ns <= 1)) return 1;
        const int full = rs < (int)V.n ? rs : (int)V.n;
        if (g.nsib + 1 >= rs) return full;
        SVec<C> r;
        return kadg_find_node<EX, C>(V, G, x, g.nsib, K, rs, sib, ns, r);
    }
};

template <bool RECORD, bool EX, bool LK, int C>
__global__ __launch_bounds__(128) void k_kadg_route(KadView V, KadGenView G, DelayConsts DC, KadLC LC,
                                                    const K160* __restrict__ qkeys, const uint32_t* __restrict__ qsrc,
                                                    uint64_t nq, ovs_route_out* __restrict__ out,
                                                    uint32_t* __restrict__ hopseq, uint32_t* __restrict__ rpcs_out,
                                                    uint32_t* __restrict__ sib_out)
{
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    constexpr int A = KAD_MAX_ALPHA;     // slots; strictParallelRpcs keeps alpha of them in use
    const int ns = LK ? LC.numSiblings : 1;
    KadLookup<A, C> L;
    kad_lookup_init(L, qkeys[q], qsrc[q], V.xy);
    const GHopRecorder<RECORD> rec{hopseq, q * (uint64_t)LC.hopCountMax, LC.hopCountMax};
    const KadGenSizer<EX, C> size{G};
    SVec<C> res;
    res.n = 0;
    res.used = 0;
    while (!kad_lookup_done(L)) {
        KadEv ev;
        ev.r = 0; ev.geo = 0; ev.boff = 0; ev.e = 0; ev.num = 0; ev.numR = 0; ev.pre = 0; ev.start = false;
        const int ph = kad_event_begin<A, EX, LK>(L, V, DC, LC, GAlwaysReady{}, rec, ev);
        res.n = 0;
        res.used = 0;
        int num = -1;
        if (ph == KEV_FIND) {
            kadg_find_node<EX, C>(V, G, ev.r, ev.rg().nsib, L.K, ev.numR, ev.sb(), ns, res);
            num = kad_event_after_find<A, EX, LK>(L, V, LC, ev, res);
        } else if (ph == KEV_SENDS) {
            num = ev.num;
        }
        if (num >= 0) kad_send_rpcs<A, EX, LK, true>(L, V, DC, LC, num, GSendNothing{}, size);
    }
    const ovs_route_out o = kad_lookup_output(L, V, DC, LC);
    const bool ok = o.status == OVS_LOOKUP_OK;
    if (LK) {
        // the LookupResponse's sibling vector: the answering sibling's findNode result (K2's rule)
        if (ns == 0) {
            sib_out[q] = ok ? L.result : NONE;
        } else {
            uint32_t* row = sib_out + q * (uint64_t)ns;
            for (int j = 0; j < ns && j < 8; ++j) row[j] = (ok && j < res.n) ? res.idx[j] : NONE;
        }
    }
    out[q] = o;
    if (rpcs_out) rpcs_out[q] = L.nsent;
}

template <bool EX, int CAP>
__global__ void k_kadg_find_node(KadView V, KadGenView G, const uint32_t* __restrict__ node,
                                 const K160* __restrict__ keys, uint64_t n, int numRedundant, int numSiblings,
                                 uint32_t* __restrict__ out_nodes, uint32_t max_out, uint8_t* __restrict__ out_count,
                                 uint8_t* __restrict__ out_sib)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = node[i];
    const K160 K = keys[i];
    const KadNode r = load_node(V.nodes, c);
    const bool sb = numSiblings >= 0 && kad_is_sibling(V, r, c, K, numSiblings);
    SVec<CAP> res;
    const int cnt = kadg_find_node<EX, CAP>(V, G, c, kad_nsib(r.meta), K, numRedundant, sb, numSiblings, res);
    uint32_t* o = out_nodes + i * max_out;
    for (uint32_t j = 0; j < max_out; ++j) o[j] = NONE;
#pragma unroll
    for (int j = 0; j < CAP; ++j)
        if (j < cnt && (uint32_t)j < max_out) o[j] = res.idx[j];
    out_count[i] = (uint8_t)(cnt < (int)max_out ? cnt : (int)max_out);
    out_sib[i] = sb ? 1 : 0;
}

// ---------------------------------------------------------------------------
// Recursive routing (R/Kademlia): semi- / full-recursive one-way routes and LookupCalls over either
// table form.  One lane per message, hop by hop: BaseOverlay::sendToKey / handleBaseOverlayMessage
// (BaseOverlay.cc:880-1004, 1380-1582) with Kademlia::recursiveRoutingHook (Kademlia.cc:1022-1057,
// altRecMode off): every node the message reaches other than its source first sends the source a
// KademliaRoutingInfoMessage (findNode(key, k, s) nodes, 47 + 27 n + 28 B), which leaves the
// node's tx queue ahead of the route message.  LookupCalls: RecursiveLookup (RecursiveLookup.cc:
// 52-139) -- a routed FindNodeCall (136 B), findNodeRpc at the delivering node, the response back
// by UDP (semi) or routed to the source's key (full).  oracle: rec_route / run_recursive_call.

constexpr int KREC_C = 16;     // result capacity: recNumRedundantNodes, lookupRedundantNodes, k, s <= 16

struct KadRecCfg {
    int hcm, recR, R, k, s;
    int64_t keyTimeout2;       // 2 * rpcKeyTimeout (the call is resent once)
};

template <bool GEN, bool EX>
__device__ __forceinline__ int krec_find(const KadView& V, const KadGenView& G, uint32_t c, const KadNode& r,
                                         const K160& K, int numRedundant, bool sib, int ns, SVec<KREC_C>& res)
{
    if constexpr (GEN) return kadg_find_node<EX, KREC_C>(V, G, c, kad_nsib(r.meta), K, numRedundant, sib, ns, res);
    else return kad_find_node_ins<KREC_C, EX>(V, c, resp_geo(r, K), K, numRedundant, sib, res, ns);
}

struct KRecEnd {
    uint32_t node;
    int hops, status;
    int64_t t, tx;
};

// one BaseRouteMessage from `from` towards K, leaving at t0 with from's queue busy until tx0;
// bwMsg = its serialisation time; nsFrom = numSiblings of the first sendToKey.
// SRC (routingType source-routing-recursive): the message records its senders (visitedHops,
// BaseOverlay.cc:888-897) -- `from`, then the hop list hopseq[0 .. hops-2], which SRC always records --
// and the loop detection skips every one of them (1502-1516); the message's length stays the one set
// when it was created (1398), so the delays are semi-recursive's.
template <bool GEN, bool EX, bool RECORD, bool SRC = false>
__device__ KRecEnd krec_walk(const KadView& V, const KadGenView& G, const DelayConsts& DC, const KadRecCfg& RC,
                             const K160& K, uint32_t from, int nsFrom, int64_t bwMsg, int64_t t0, int64_t tx0,
                             uint32_t* __restrict__ hopseq)
{
    KRecEnd e;
    e.node = NONE; e.hops = 0; e.status = 0; e.t = t0; e.tx = tx0;
    uint32_t cur = from, last = from;
    int hops = 0;
    int64_t t = t0, tx = tx0;
    SVec<KREC_C> res;
    // the hook's KademliaRoutingInfoMessage at node c: tx queue busy for its serialisation first
    auto info = [&](uint32_t c, const KadNode& r) {
        const bool sbs = kad_is_sibling(V, r, c, K, RC.s);
        const int n = krec_find<GEN, EX>(V, G, c, r, K, RC.k, sbs, RC.s, res);
        tx = (tx > t ? tx : t) + bw_ns(47 + 27 * n + 28, DC.datarate, DC.round);
    };
    for (;;) {
        const KadNode r = load_node(V.nodes, cur);
        const int ns = cur == from ? nsFrom : 1;
        if (cur != from) {
            tx = 0;                                   // a node's queue is idle when the message arrives
            if (kad_is_sibling(V, r, cur, K, 1)) {    // delivery (BaseOverlay.cc:907-914), hook first
                info(cur, r);
                break;
            }
        }
        const bool sb = kad_is_sibling(V, r, cur, K, ns);
        const int n = krec_find<GEN, EX>(V, G, cur, r, K, RC.recR, sb, ns, res);
        if (n == 0) { e.status = OVS_LOOKUP_NO_NEXT; return e; }           // 1449-1461
        if (hops >= RC.hcm) { e.status = OVS_LOOKUP_HOPMAX; return e; }     // 1464-1488
        uint32_t next = NONE;
        for (int i = 0; i < KREC_C && next == NONE; ++i) {                   // loop detection 1502-1516
            if (i >= n) break;
            const uint32_t h = res.idx[i];
            if ((h == last && h != cur) || (h == from && cur != from) || (h == cur && !sb)) continue;
            if (SRC) {
                bool seen = false;
                for (int j = 0; j + 1 < hops && !seen; ++j) seen = hopseq[j] == h;
                if (seen) continue;
            }
            next = h;
        }
        if (next == NONE) { e.status = OVS_LOOKUP_NO_NEXT; return e; }
        if (next == cur) break;                                              // 1555-1570: responsible
        if (cur != from) info(cur, r);
        // sendRouteMessage (1107-1146) through the node's queue
        const double2 b = V.xy[next];
        const int64_t newTx = (tx > t ? tx : t) + bwMsg;
        tx = newTx;
        t = newTx + DC.access2 + coord_ns(r.x, r.y, b.x, b.y, DC.round) + bwMsg;
        if ((RECORD || SRC) && hops < RC.hcm) hopseq[hops] = next;
        ++hops;
        last = cur;
        cur = next;
    }
    e.node = cur; e.hops = hops; e.t = t; e.tx = tx;
    return e;
}

// MODE 0: one-way route, 1: one-way route with the hop sequence, 2 / 3: LookupCall with a
// semi- / full-recursive response; source-routing-recursive: 4 one-way route (the hop list in hopseq:
// the caller's or the context's scratch), 5 LookupCall whose response goes back along the call's
// visited hops reversed (BaseRpc.cc:575-588), the R/Kademlia hook at every node on the way
template <bool GEN, bool EX, int MODE>
__global__ __launch_bounds__(128) void k_kad_recursive(KadView V, KadGenView G, DelayConsts DC, KadRecCfg RC, int ns,
                                                       const K160* __restrict__ qkeys, const uint32_t* __restrict__ qsrc,
                                                       uint64_t nq, ovs_route_out* __restrict__ out,
                                                       uint32_t* __restrict__ hopseq, uint32_t* __restrict__ sib_out)
{
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    const K160 K = qkeys[q];
    const uint32_t S = qsrc[q];
    ovs_route_out o;
    o.responsible = NONE; o.hops = 0; o.one_way_hops = 0; o.latency_ns = -1; o.status = 0;
    if constexpr (MODE <= 1 || MODE == 4) {
        const KRecEnd e = krec_walk<GEN, EX, MODE == 1, MODE == 4>(V, G, DC, RC, K, S, 1, DC.bwRoute, 0, 0,
                                                                   hopseq + q * (uint64_t)RC.hcm);
        o.status = (uint8_t)e.status;
        if (!e.status) {
            o.responsible = e.node;
            o.hops = (uint16_t)e.hops;
            o.one_way_hops = (uint8_t)e.hops;
            o.latency_ns = e.t;
        }
    } else {
        const int nslots = ns ? ns : 1;
        uint32_t* row = sib_out + q * (uint64_t)nslots;
        for (int j = 0; j < nslots; ++j) row[j] = NONE;
        // the routed FindNodeCall: BASEROUTE_L 424 + FINDNODECALL_L 440 bits + UDP/IP 28 B
        uint32_t* vl = MODE == 5 ? hopseq + q * (uint64_t)RC.hcm : nullptr;   // its hops (source routing)
        const KRecEnd d = krec_walk<GEN, EX, false, MODE == 5>(V, G, DC, RC, K, S, ns,
                                                               bw_ns(53 + 55 + 28, DC.datarate, DC.round), 0, 0, vl);
        o.status = (uint8_t)d.status;
        if (!d.status) {
            // findNodeRpc at D (BaseOverlay.cc:1841-1915)
            const KadNode rd = load_node(V.nodes, d.node);
            const bool flag = kad_is_sibling(V, rd, d.node, K, ns);
            SVec<KREC_C> res;
            const int n = krec_find<GEN, EX>(V, G, d.node, rd, K, RC.R, flag, ns, res);
            int64_t T = d.t;
            bool lost = false;
            if (d.node != S) {
                const int32_t rb = DC.respBase + DC.respPerNode * n;
                const double2 sxy = V.xy[S];
                if (MODE == 2) {          // semi-recursive: UDP straight back (1807-1813)
                    const int64_t bwr = bw_ns(rb, DC.datarate, DC.round);
                    const int64_t newTx = (d.tx > d.t ? d.tx : d.t) + bwr;
                    T = newTx + DC.access2 + coord_ns(rd.x, rd.y, sxy.x, sxy.y, DC.round) + bwr;
                } else if (MODE == 5) {   // source routing: the senders reversed, h_{k-1} .. h_1, S
                    const K160 KS = node_key(V.nodes, S);
                    const int64_t bwm = bw_ns(53 + rb, DC.datarate, DC.round);
                    uint32_t cur = d.node;
                    int64_t t = d.t, tx = d.tx;
                    SVec<KREC_C> ires;
                    for (int i = d.hops - 2; i >= -1; --i) {
                        const uint32_t nx = i >= 0 ? vl[i] : S;
                        const KadNode rc = load_node(V.nodes, cur);
                        if (cur != d.node) {
                            // the node's queue is idle on arrival; R/Kademlia's hook toward the
                            // response's source (D) leaves it first (Kademlia.cc:1022-1057)
                            const bool sbs = kad_is_sibling(V, rc, cur, KS, RC.s);
                            const int ni = krec_find<GEN, EX>(V, G, cur, rc, KS, RC.k, sbs, RC.s, ires);
                            tx = t + bw_ns(47 + 27 * ni + 28, DC.datarate, DC.round);
                        }
                        const double2 b = V.xy[nx];
                        const int64_t newTx = (tx > t ? tx : t) + bwm;
                        tx = newTx;
                        t = newTx + DC.access2 + coord_ns(rc.x, rc.y, b.x, b.y, DC.round) + bwm;
                        cur = nx;
                    }
                    T = t;
                } else {                  // full-recursive: routed to the source's key (1814-1818)
                    const K160 KS = node_key(V.nodes, S);
                    const KRecEnd b = krec_walk<GEN, EX, false>(V, G, DC, RC, KS, d.node, 1,
                                                                bw_ns(53 + rb, DC.datarate, DC.round), d.t, d.tx, nullptr);
                    lost = b.status != 0 || b.node != S;
                    T = b.t;
                }
            }
            if (lost || T >= RC.keyTimeout2) {
                o.status = OVS_LOOKUP_RPC_TIMEOUT;
            } else if (!flag || n == 0) {
                o.status = OVS_LOOKUP_INVALID;
            } else {
                for (int j = 0; j < KREC_C; ++j)
                    if (j < n && j < nslots) row[j] = res.idx[j];
                o.responsible = d.node;
                o.latency_ns = T;     // hops: RecursiveLookup::getMinHops() = 0
            }
        }
    }
    out[q] = o;
}

inline unsigned gblocks(uint64_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

inline KadGenView gen_view(const KadTables& t) { return KadGenView{t.goff, t.gtop, t.gidx, t.gend, t.b, t.nb}; }

}  // namespace

hipError_t kad_route_general(const KadTables& t, const double2* xy, uint32_t n, const ovs_params& P,
                             const DelayConsts& DC, const K160* qkeys, const uint32_t* qsrc, uint64_t nq,
                             ovs_route_out* out, uint32_t* hopseq, uint32_t* rpcs, hipStream_t st, uint32_t* sibs)
{
    if (nq == 0) return hipSuccess;
    if (!t.general || !kad_params_supported(P, t)) return hipErrorNotSupported;
    if (sibs && hopseq) return hipErrorNotSupported;
    KadLC LC = kad_make_lc(P, t);
    kad_lc_sizes(LC, DC, n);
    const KadView V = kad_make_view(t, xy, n);
    const KadGenView G = gen_view(t);
    const bool wide = LC.redundant > 8 || LC.maxRedundantLocal > 8;
    const dim3 grid(gblocks(nq, 128)), blk(128);
#define KG(rec, ex, lk, c) hipLaunchKernelGGL((k_kadg_route<rec, ex, lk, c>), grid, blk, 0, st, V, G, DC, LC, qkeys, qsrc, nq, \
                                              out, hopseq, rpcs, sibs)
#define KGC(rec, lk, c) do { if (t.exact) KG(rec, true, lk, c); else KG(rec, false, lk, c); } while (0)
    if (wide) {
        if (sibs) KGC(false, true, 16);
        else if (hopseq) KGC(true, false, 16);
        else KGC(false, false, 16);
    } else {
        if (sibs) KGC(false, true, 8);
        else if (hopseq) KGC(true, false, 8);
        else KGC(false, false, 8);
    }
#undef KGC
#undef KG
    return hipGetLastError();
}

hipError_t kad_find_node_general(const KadTables& t, uint32_t n, const uint32_t* node, const K160* keys, uint64_t nq,
                                 int numRedundant, int numSiblings, uint32_t* out_nodes, uint32_t max_out,
                                 uint8_t* out_count, uint8_t* out_sib, hipStream_t st)
{
    if (nq == 0) return hipSuccess;
    if (!t.general) return hipErrorNotSupported;
    if ((numSiblings < 1 && numSiblings != -1) || numSiblings > 64 || numRedundant > 64) return hipErrorNotSupported;
    const KadView V = kad_make_view(t, nullptr, n);
    const KadGenView G = gen_view(t);
    const bool wide = numSiblings > 16 || numRedundant > 16;
#define KFN(ex, cap) hipLaunchKernelGGL((k_kadg_find_node<ex, cap>), dim3(gblocks(nq, 128)), dim3(128), 0, st, V, G, node, keys, \
                                        nq, numRedundant, numSiblings, out_nodes, max_out, out_count, out_sib)
    if (t.exact) { if (wide) KFN(true, 64); else KFN(true, 16); }
    else { if (wide) KFN(false, 64); else KFN(false, 16); }
#undef KFN
    return hipGetLastError();
}

hipError_t kad_route_recursive(const KadTables& t, const double2* xy, uint32_t n, const ovs_params& P,
                               const DelayConsts& DC, int64_t key_timeout, int lookup_ns, const K160* qkeys,
                               const uint32_t* qsrc, uint64_t nq, ovs_route_out* out, uint32_t* hopseq, uint32_t* sibs,
                               hipStream_t st)
{
    if (nq == 0) return hipSuccess;
    if (P.routingType != 1 && P.routingType != 2 && P.routingType != 4) return hipErrorNotSupported;
    if (P.routingType == 4 && !hopseq) return hipErrorInvalidValue;   // source routing keeps the hop lists
    if (P.recNumRedundantNodes < 1 || P.recNumRedundantNodes > KREC_C || P.lookupRedundantNodes < 1 ||
        P.lookupRedundantNodes > KREC_C || t.k > KREC_C || t.s > KREC_C || P.hopCountMax < 0)
        return hipErrorNotSupported;
    const KadView V = kad_make_view(t, xy, n);
    const KadGenView G = gen_view(t);
    KadRecCfg RC;
    RC.hcm = P.hopCountMax; RC.recR = P.recNumRedundantNodes; RC.R = P.lookupRedundantNodes; RC.k = t.k; RC.s = t.s;
    RC.keyTimeout2 = 2 * key_timeout;
    const dim3 grid(gblocks(nq, 128)), blk(128);
    const int mode = P.routingType == 4 ? (sibs ? 5 : 4) : sibs ? (P.routingType == 1 ? 2 : 3) : (hopseq ? 1 : 0);
#define KR(gen, ex, m) hipLaunchKernelGGL((k_kad_recursive<gen, ex, m>), grid, blk, 0, st, V, G, DC, RC, lookup_ns, qkeys, qsrc, \
                                          nq, out, hopseq, sibs)
#define KRM(gen, ex) do { switch (mode) { case 0: KR(gen, ex, 0); break; case 1: KR(gen, ex, 1); break; \
                                          case 2: KR(gen, ex, 2); break; case 3: KR(gen, ex, 3); break; \
                                          case 4: KR(gen, ex, 4); break; default: KR(gen, ex, 5); } } while (0)
    if (t.general) { if (t.exact) KRM(true, true); else KRM(true, false); }
    else { if (t.exact) KRM(false, true); else KRM(false, false); }
#undef KRM
#undef KR
    return hipGetLastError();
}

}  // namespace ovs
