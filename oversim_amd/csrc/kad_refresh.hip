// kad_refresh.hip -- K2x: Kademlia refresh lookups (exhaustive-iterative routing) for gfx950.
//
// Kademlia::handleBucketRefreshTimerExpired (Kademlia.cc:1591-1686) with exhaustiveRefresh = true
// (default.ini:200) refreshes the sibling table with a lookup of the node's own key and every
// stale bucket i with a lookup of self ^ 2^i, each an EXHAUSTIVE_ITERATIVE_ROUTING IterativeLookup
// with config.redundantNodes = numSiblings = R (bucketRefreshNodes = k, siblingRefreshNodes = 5s).
// Its rules differ from the one-way lookup of K2 (IterativeLookup.cc):
//   * nextHops holds 2R entries (770-778); findNode calls carry numSiblings -1: resultSize = R,
//     no siblings flag (BaseOverlay.cc:1857-1871, Kademlia.cc:1125-1127);
//   * every response is accepted (534-540) and nothing ends the path but running out of
//     unqueried next hops: the lookup then succeeds with nextHops[0..R) as its siblings
//     (1144-1168); hopCountMax and LOOKUP_TIMEOUT still end it unsuccessfully;
//   * a node whose RPC timed out leaves nextHops (948-957).
// R reaches 40 (siblingRefreshNodes = 5s), so the vectors do not fit registers: each lane keeps
// its LookupVector (2R entries) and the findNode results of its <= alpha pending calls in a
// per-lane scratch slice laid out entry-major (entry j of lane l at j * lanes + l), so lanes that
// walk their vectors in step touch consecutive addresses.  The responder's findNode is evaluated
// when the call is sent (the tables do not change during a batch): its size fixes the response's
// delay, and the result waits in the pending slot's scratch until the response event.  One lane
// runs one lookup to completion, then takes the next one of the grid-stride loop.
#include <hipcub/hipcub.hpp>

#include "kad_dev.hpp"

namespace ovs {

namespace {

constexpr int XMAXA = 4;        // lookupParallelRpcs <= 4 (strictParallelRpcs: <= alpha calls in flight)
constexpr int XMAXDEAD = 64;    // nodes whose RPC timed out, per lookup

struct XCfg {
    int R, ns, alpha, hcm, k;      // ns: the siblings vector's size (numSiblings <= R)
    int oneway;                    // 1: a KBRTestApp one-way lookup (route message to the result)
    int strict, visitOnlyOnce, newOnResp, newOnTimeout, finishOnFirst;
};

struct XScratch {
    uint32_t* nh_idx;    // [2R][lanes]
    uint64_t* nh_d;      // [2R][lanes]
    uint8_t* nh_used;    // [2R][lanes]
    uint32_t* res_idx;   // [A * R + max(R, k)][lanes]: findNode results of the pending calls (slot A: the start)
    uint64_t* res_d;
    uint32_t* dead;      // [XMAXDEAD][lanes]
    uint64_t lanes;
};

struct XPend {
    uint32_t node, ninfo, seq;
    int rn;              // findNode result size (scratch slot)
    int64_t t, tins, tsend;
    bool to;
};

struct XLookup {
    K160 K;
    uint32_t S;
    double sx, sy;
    int64_t now, txf;
    uint32_t seq, nsent;
    int nnh, nd, nhop;
    int step, hops, pending;
    bool pfinished, psuccess, counted, any_to, success, err;
    int finishedPaths, successfulPaths, minHops;
    XPend p[XMAXA];
    uint32_t pvalid;
};

template <bool EX>
struct XCtx {
    const KadView& V;
    const DelayConsts& DC;
    const XCfg& C;
    const XScratch& X;
    uint64_t lane;
    uint32_t* __restrict__ resp;      // responders of this lookup (hop order), hcm entries
    int64_t* __restrict__ rtt;        // their RTTs (may be null)
    uint32_t* __restrict__ sib;       // ns siblings of this lookup

    __device__ __forceinline__ uint64_t at(int j) const { return (uint64_t)j * X.lanes + lane; }

    // --- sorted vectors in scratch (BaseKeySortedVector::add, NodeVector.h:381-512) -----------------
    // insert x (distance top dx) into the vector at scratch rows [base, base + cap) holding *n
    // entries; returns the position or -1 (full and farther than the last, or already present)
    __device__ int vadd(uint32_t* idx, uint64_t* d, uint8_t* used, int base, int cap, int* n, uint32_t x,
                        uint64_t dx, const K160& K) const
    {
        const int m = *n;
        if (m == cap) {
            const uint32_t li = idx[at(base + m - 1)];
            if (li != x && cand_lt<EX>(d[at(base + m - 1)], li, dx, x, K, V.nodes)) return -1;
        }
        int pos = m;
        for (int i = 0; i < m; ++i) {
            const uint32_t ei = idx[at(base + i)];
            if (ei == x) return -1;
            if (cand_lt<EX>(dx, x, d[at(base + i)], ei, K, V.nodes)) { pos = i; break; }
        }
        const int last = m < cap ? m : cap - 1;
        for (int i = last; i > pos; --i) {
            idx[at(base + i)] = idx[at(base + i - 1)];
            d[at(base + i)] = d[at(base + i - 1)];
            if (used) used[at(base + i)] = used[at(base + i - 1)];
        }
        idx[at(base + pos)] = x;
        d[at(base + pos)] = dx;
        if (used) used[at(base + pos)] = 0;
        *n = m < cap ? m + 1 : cap;
        return pos;
    }

    // Kademlia::findNode(key, numRedundantNodes = rs, numSiblings = -1) at node c into result slot
    // `slot` (Kademlia.cc:1101-1246; b = 1: startIndex = mainIndex).  Returns the result size.
    __device__ int find_node(uint32_t c, const K160& K, int rs, int slot) const
    {
        const KadNode r = load_node(V.nodes, c);
        const RespGeo g = resp_geo(r, K);
        const int base = slot * C.R;
        rs = min(rs, slot < C.alpha ? C.R : max(C.R, C.k));   // the slot's capacity (XScratch::res_idx)
        int n = 0;
        const uint64_t kt = ktop(K);
        if (g.nsib == 0) {      // an empty sibling table answers [self]
            vadd(X.res_idx, X.res_d, nullptr, base, rs, &n, c, dist_hi(as_key(r.key), K), K);
            return n;
        }
        auto add_blk = [&](const KadBlk* blk) {
            for (int q = 0; q < KBLK; ++q) {
                const uint32_t x = blk->idx[q];
                if (x == NONE) break;
                vadd(X.res_idx, X.res_d, nullptr, base, rs, &n, x, dclamp(blk->top[q] ^ kt), K);
            }
        };
        auto add_slot = [&](int bucket) {
            if (g.rowlo < 0 || bucket < g.rowlo) return;   // buckets below the stored row are empty
            add_blk(slot_blk(V, g.boff, bucket));
        };
        if (g.m >= 0) add_slot(g.m);
        if (g.m >= g.endIndex || n < rs) {
            for (int b = g.m - 1; b >= g.endIndex; --b) add_slot(b);
            const KadBlk* L = V.sibb + (uint64_t)(c - V.lo) * V.sbn;
            for (int j = 0; j * KBLK < g.nsib; ++j) add_blk(L + j);
            vadd(X.res_idx, X.res_d, nullptr, base, rs, &n, c, dist_hi(as_key(r.key), K), K);
        }
        for (int b = g.m + 1; n < rs && b < KEYBITS; ++b) add_slot(b);
        return n;
    }

    __device__ bool is_dead(const XLookup& L, uint32_t x) const
    {
        for (int i = 0; i < L.nd; ++i)
            if (X.dead[at(i)] == x) return true;
        return false;
    }

    // visited = the source and every responder.  Without a timeout no responder can be an unused
    // next hop (an evicted entry is farther than the vector's last and never re-enters while the
    // vector only shrinks by eviction), so the list is scanned only after one.
    __device__ bool visited(const XLookup& L, uint32_t x) const
    {
        if (x == L.S) return true;
        if (!L.any_to) return false;
        for (int i = 0; i < L.nhop; ++i)
            if (resp[i] == x) return true;
        return false;
    }

    // IterativeLookup::sendRpc (656-689) + BaseRpc timeout + SimpleNodeEntry::calcDelay
    __device__ void lookup_send(XLookup& L, uint32_t x) const
    {
        for (int i = 0; i < C.alpha; ++i)
            if (((L.pvalid >> i) & 1u) && L.p[i].node == x) { ++L.p[i].ninfo; return; }   // "RPC already sent"
        int slot = -1;
        for (int i = C.alpha - 1; i >= 0; --i)
            if (!((L.pvalid >> i) & 1u)) slot = i;
        if (slot < 0) { L.err = true; return; }
        const int rn = find_node(x, L.K, C.R, slot);
        int64_t d1 = 0, d2 = 0;
        if (x != L.S) {                         // SimpleUDP delivers to itself without delay
            const double2 xy = V.xy[x];
            const int64_t cd = coord_ns(L.sx, L.sy, xy.x, xy.y, DC.round);
            const int64_t bwc = DC.bwCall;
            const int64_t newTx = (L.txf > L.now ? L.txf : L.now) + bwc;
            L.txf = newTx;
            d1 = (newTx - L.now) + DC.access2 + cd + bwc;
            const int64_t bwr = rn <= 16 ? DC.bwResp[rn] : bw_ns(DC.respBase + DC.respPerNode * rn, DC.datarate, DC.round);
            d2 = 2 * bwr + DC.access2 + cd;
        }
        const int64_t tTo = L.now + DC.rpcTimeout;
        const int64_t tResp = L.now + d1 + d2;
        XPend& P = L.p[slot];
        P.node = x;
        P.ninfo = 1;
        P.rn = rn;
        P.tsend = L.now;
        P.to = tTo <= tResp;                    // the timeout was scheduled first: it wins a tie
        const uint32_t sTo = L.seq++, sR = L.seq++;
        P.seq = P.to ? sTo : sR;
        P.t = P.to ? tTo : tResp;
        P.tins = P.to ? L.now : L.now + d1;
        L.pvalid |= 1u << slot;
        ++L.nsent;
    }

    // IterativePathLookup::sendRpc (1067-1170), exhaustive
    __device__ void send_rpcs(XLookup& L, int num) const
    {
        if (L.pfinished) return;
        if (C.hcm && L.hops >= C.hcm) { L.pfinished = true; L.psuccess = false; return; }
        if (C.strict) num = min(num, C.alpha - L.pending);
        if (num == 0 && L.pending == 0 && !C.finishOnFirst) num = C.alpha;
        for (int i = 0; num > 0 && i < C.R; ++i) {
            int e = -1;                          // getNextEntry: not alreadyUsed, not dead (1172-1182)
            for (int q = 0; q < L.nnh && e < 0; ++q)
                if (!X.nh_used[at(q)] && !(L.nd && is_dead(L, X.nh_idx[at(q)]))) e = q;
            if (e < 0) break;
            const uint32_t h = X.nh_idx[at(e)];
            if (!C.visitOnlyOnce || !visited(L, h)) {
                ++L.pending;
                --num;
                lookup_send(L, h);
            }
            X.nh_used[at(e)] = 1;
        }
        if (L.pending == 0) {
            // exhaustive lookups are always successful: addSibling(nextHops[0..R)) -- push_back while
            // the numSiblings-sized vector has room (1147-1156, 436-440)
            int m = L.nnh < C.R ? L.nnh : C.R;
            m = m < C.ns ? m : C.ns;
            for (int q = 0; q < m; ++q) sib[q] = X.nh_idx[at(q)];
            L.psuccess = true;
            L.pfinished = true;
        }
    }

    // IterativePathLookup::handleTimeout (935-1023), failedNodeRpcs = false
    __device__ void path_timeout(XLookup& L, uint32_t dest) const
    {
        if (L.pfinished) return;
        if (L.nd && is_dead(L, dest)) {          // exhaustive: a dead node leaves nextHops (948-957)
            for (int q = 0; q < L.nnh; ++q)
                if (X.nh_idx[at(q)] == dest) {
                    for (int j = q; j + 1 < L.nnh; ++j) {
                        X.nh_idx[at(j)] = X.nh_idx[at(j + 1)];
                        X.nh_d[at(j)] = X.nh_d[at(j + 1)];
                        X.nh_used[at(j)] = X.nh_used[at(j + 1)];
                    }
                    --L.nnh;
                    break;
                }
        }
        --L.pending;
        if (L.now > DC.lookupTimeout) { L.pfinished = true; L.psuccess = false; return; }
        if (C.newOnTimeout) send_rpcs(L, 1);
        else if (L.pending == 0) send_rpcs(L, C.alpha);
    }

    // IterativePathLookup::handleResponse (803-921), exhaustive: no siblings flag
    __device__ void path_response(XLookup& L, uint32_t src, int slot, int rn, int64_t rt) const
    {
        if (L.pfinished) return;
        if (L.now > DC.lookupTimeout) { L.pfinished = true; L.psuccess = false; return; }
        if (src != L.S) {
            if (L.nhop < C.hcm) {
                resp[L.nhop] = src;
                if (rtt) rtt[L.nhop] = rt;
            }
            ++L.nhop;
            ++L.hops;
        }
        ++L.step;
        --L.pending;
        int numNew = 0;
        const int base = slot * C.R;
        for (int i = 0; i < rn; ++i) {
            const int pos = vadd(X.nh_idx, X.nh_d, X.nh_used, 0, 2 * C.R, &L.nnh, X.res_idx[at(base + i)],
                                 X.res_d[at(base + i)], L.K);
            if (pos >= 0 && pos < C.R) ++numNew;
        }
        if (numNew == 0 && C.newOnResp) numNew = 1;
        send_rpcs(L, min(numNew, C.alpha));
    }

    __device__ void count_finished(XLookup& L) const
    {
        if (L.pfinished && !L.counted) {
            L.counted = true;
            ++L.finishedPaths;
            if (L.hops < L.minHops) L.minHops = L.hops;
            if (L.psuccess) ++L.successfulPaths;
        }
    }

    // checkStop (295-349), parallelPaths = 1, numSiblings = R > 0
    __device__ bool check_stop(XLookup& L) const
    {
        if (L.finishedPaths == 1 || L.pvalid == 0) {
            L.success = L.successfulPaths >= 1 || L.psuccess;
            return true;
        }
        return false;
    }

    __device__ void run(XLookup& L) const
    {
        // IterativeLookup::start (133-244): the source's own findNode(key, k, -1)
        const int rn0 = find_node(L.S, L.K, C.k, C.alpha);
        bool done = false;
        if (rn0 == 0) {
            L.success = false;
            done = true;
        } else {
            const int base = C.alpha * C.R;
            for (int i = 0; i < rn0; ++i)
                vadd(X.nh_idx, X.nh_d, X.nh_used, 0, 2 * C.R, &L.nnh, X.res_idx[at(base + i)], X.res_d[at(base + i)],
                     L.K);
            send_rpcs(L, C.alpha);
            done = check_stop(L);
        }
        while (!done && !L.err) {
            int e = -1;
            int64_t bt = 0, bi = 0;
            uint32_t bs = 0;
            for (int i = 0; i < C.alpha; ++i) {
                if (!((L.pvalid >> i) & 1u)) continue;
                const XPend& P = L.p[i];
                if (e < 0 || P.t < bt || (P.t == bt && (P.tins < bi || (P.tins == bi && P.seq < bs)))) {
                    e = i; bt = P.t; bi = P.tins; bs = P.seq;
                }
            }
            if (e < 0) break;
            const XPend P = L.p[e];
            L.pvalid &= ~(1u << e);
            L.now = bt;
            if (P.to) {
                // BaseRpc timeout -> IterativeLookup::handleRpcTimeout (588-654)
                L.any_to = true;
                if (L.nd < XMAXDEAD) X.dead[at(L.nd++)] = P.node;
                else L.err = true;
                for (uint32_t q = 0; q < P.ninfo; ++q) {
                    if (L.pfinished) continue;
                    path_timeout(L, P.node);
                    count_finished(L);
                }
            } else {
                // handleRpcResponse (488-585): exhaustive lookups accept every response
                bool handled = false;
                for (uint32_t q = 0; q < P.ninfo; ++q) {
                    if (L.pfinished) continue;
                    if (!handled) {
                        path_response(L, P.node, e, P.rn, L.now - P.tsend);
                        handled = true;
                    } else {
                        path_timeout(L, P.node);
                    }
                    count_finished(L);
                }
            }
            done = check_stop(L);
        }
    }
};

template <bool EX>
__global__ __launch_bounds__(256) void k_kad_refresh(KadView V, DelayConsts DC, XCfg C, XScratch X,
                                                     const K160* __restrict__ qkeys, const uint32_t* __restrict__ qsrc,
                                                     uint64_t nq, ovs_route_out* __restrict__ out,
                                                     uint32_t* __restrict__ sib_out, uint32_t* __restrict__ resp_out,
                                                     int64_t* __restrict__ rtt_out, uint32_t* __restrict__ rpcs_out,
                                                     uint32_t* __restrict__ err)
{
    const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= X.lanes) return;
    for (uint64_t q = lane; q < nq; q += X.lanes) {
        XLookup L;
        L.K = qkeys[q];
        L.S = qsrc[q];
        const double2 sxy = V.xy[L.S];
        L.sx = sxy.x; L.sy = sxy.y;
        L.now = 0; L.txf = 0; L.seq = 0; L.nsent = 0;
        L.nnh = 0; L.nd = 0; L.nhop = 0;
        L.step = 0; L.hops = 0; L.pending = 0;
        L.pfinished = false; L.psuccess = false; L.counted = false; L.any_to = false; L.success = false; L.err = false;
        L.finishedPaths = 0; L.successfulPaths = 0; L.minHops = 0x7FFFFFFF;
        L.pvalid = 0;
        uint32_t* sib = sib_out + q * (uint64_t)C.ns;
        for (int j = 0; j < C.ns; ++j) sib[j] = NONE;
        uint32_t* resp = resp_out + q * (uint64_t)C.hcm;
        int64_t* rtt = rtt_out ? rtt_out + q * (uint64_t)C.hcm : nullptr;
        const XCtx<EX> ctx{V, DC, C, X, lane, resp, rtt, sib};
        ctx.run(L);
        if (L.err) atomicOr(err, 1u);
        for (int j = L.nhop; j < C.hcm; ++j) {
            resp[j] = NONE;
            if (rtt) rtt[j] = -1;
        }
        // SendToKeyListener / LookupResponse fields (as ovs_lookup_batch): the ovs_lookup_out is
        // written through its ovs_route_out twin (same size; k_lookup_finish's convention)
        const bool valid = L.success && !L.err;
        const uint8_t fail_status = L.now > DC.lookupTimeout ? OVS_LOOKUP_TIMEOUT
                                    : L.nd > 0                 ? OVS_LOOKUP_RPC_TIMEOUT
                                    : (C.hcm && L.hops >= C.hcm) ? OVS_LOOKUP_HOPMAX
                                                                 : OVS_LOOKUP_NO_NEXT;
        if (rpcs_out) rpcs_out[q] = L.nsent;
        if (C.oneway) {
            // SendToKeyListener::lookupFinished -> sendRouteMessage to getResult()[0] through the
            // source's tx queue (BaseOverlay.cc:1107-1146, 1241-1259; SimpleNodeEntry.cc:164-194)
            ovs_route_out o;
            o.hops = (uint16_t)(L.minHops == 0x7FFFFFFF ? 0 : L.minHops);
            const uint32_t R0 = sib[0];
            if (valid && R0 != NONE) {
                o.status = OVS_LOOKUP_OK;
                o.responsible = R0;
                o.one_way_hops = (uint8_t)(o.hops + (R0 != L.S ? 1 : 0));
                int64_t lat = L.now;
                if (R0 != L.S) {
                    const double2 rxy = V.xy[R0];
                    const int64_t newTx = (L.txf > L.now ? L.txf : L.now) + DC.bwRoute;
                    lat = newTx + DC.access2 + coord_ns(L.sx, L.sy, rxy.x, rxy.y, DC.round) + DC.bwRoute;
                }
                o.latency_ns = lat;
            } else {
                o.status = fail_status;
                o.responsible = NONE;
                o.one_way_hops = 0;
                o.latency_ns = -1;
            }
            out[q] = o;
            continue;
        }
        ovs_lookup_out o;
        o.hops = (uint16_t)(L.minHops == 0x7FFFFFFF ? 0 : L.minHops);
        o.is_valid = valid ? 1 : 0;
        if (valid) {
            int ns = 0;
            for (int j = 0; j < C.ns; ++j) ns += sib[j] != NONE ? 1 : 0;
            o.num_siblings = (uint32_t)ns;
            o.latency_ns = L.now;
            o.status = OVS_LOOKUP_OK;
        } else {
            for (int j = 0; j < C.ns; ++j) sib[j] = NONE;
            o.num_siblings = 0;
            o.latency_ns = -1;
            o.status = fail_status;
        }
        reinterpret_cast<ovs_lookup_out*>(out)[q] = o;
    }
}

// refresh keys (Kademlia.cc:1631-1676, b = 1): node v refreshes buckets i = 159 .. diff with
// diff = L - (sharedPrefixLength(self, siblingTable->front()) + 1) = msb(self ^ front) -- the
// lowest level of the sibling set, the lowest set bit of the level mask in KadX
__device__ __forceinline__ int refresh_diff(const KadView& V, uint32_t v)
{
    const KadX& x = V.nodex[v];
    for (int w = 0; w < 5; ++w)
        if (x.mask[w]) return 32 * w + __ffs((int)x.mask[w]) - 1;
    return -1;
}

__device__ __forceinline__ bool refresh_stale(const uint32_t* stale, uint64_t j, int i)
{
    return !stale || ((stale[j * 5 + (uint64_t)(i >> 5)] >> (i & 31)) & 1u);
}

__global__ void k_kad_refresh_count(KadView V, const uint32_t* __restrict__ nodes, uint64_t m,
                                    const uint32_t* __restrict__ stale, uint64_t* __restrict__ cnt)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const uint32_t v = nodes[j];
    uint64_t c = 0;
    if (kad_nsib(V.nodes[v].meta) > 0) {
        const int diff = refresh_diff(V, v);
        for (int i = KEYBITS - 1; i >= diff; --i) c += refresh_stale(stale, j, i) ? 1 : 0;
    }
    cnt[j] = c;
}

__global__ void k_kad_refresh_fill(KadView V, const uint32_t* __restrict__ nodes, uint64_t m,
                                   const uint32_t* __restrict__ stale, const uint64_t* __restrict__ off, uint64_t cap,
                                   K160* __restrict__ keys, uint32_t* __restrict__ src)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const uint32_t v = nodes[j];
    if (kad_nsib(V.nodes[v].meta) == 0) return;
    const int diff = refresh_diff(V, v);
    const K160 me = as_key(V.nodes[v].key);
    uint64_t o = off[j];
    for (int i = KEYBITS - 1; i >= diff; --i) {
        if (!refresh_stale(stale, j, i)) continue;
        if (o < cap) {
            K160 k = me;
            k.w[i >> 5] ^= 1u << (i & 31);       // thisNode.key ^ (OverlayKey(1) << i)
            keys[o] = k;
            src[o] = v;
        }
        ++o;
    }
}

}  // namespace

hipError_t kad_exhaustive(const KadTables& t, const double2* xy, uint32_t n, const ovs_params& P, const DelayConsts& DC,
                          int R, int ns, bool oneway, const K160* qkeys, const uint32_t* qsrc, uint64_t nq, void* out,
                          uint32_t* sibs, uint32_t* responders, int64_t* rtts, uint32_t* rpcs, int num_cu,
                          hipStream_t st, bool* capacity_error)
{
    *capacity_error = false;
    if (nq == 0) return hipSuccess;
    const int A = P.lookupParallelRpcs;
    if (A < 1 || A > XMAXA || R < 1 || R > 64 || ns < 1 || ns > R || !P.lookupMerge || !P.lookupStrictParallelRpcs ||
        P.hopCountMax < 1 || t.k > 8)
        return hipErrorNotSupported;
    const KadView V = kad_make_view(t, xy, n);
    XCfg C;
    C.R = R; C.ns = ns; C.alpha = A; C.hcm = P.hopCountMax; C.k = t.k;
    C.oneway = oneway ? 1 : 0;
    C.strict = P.lookupStrictParallelRpcs; C.visitOnlyOnce = P.lookupVisitOnlyOnce;
    C.newOnResp = P.lookupNewRpcOnEveryResponse; C.newOnTimeout = P.lookupNewRpcOnEveryTimeout;
    C.finishOnFirst = P.lookupFinishOnFirstUnchanged;
    // one lane per lookup, up to 1024 lanes per CU; the scratch is sized for the lanes
    uint64_t lanes = (uint64_t)num_cu * 1024;
    if (lanes > nq) lanes = nq;
    lanes = (lanes + 255) / 256 * 256;
    const uint64_t nhE = 2ull * R, resE = (uint64_t)A * R + (uint64_t)(R > t.k ? R : t.k);
    const uint64_t bytes = lanes * (nhE * (4 + 8 + 1) + resE * (4 + 8) + XMAXDEAD * 4) + 4;
    char* buf = nullptr;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&buf), bytes);
    if (e != hipSuccess) return e;
    XScratch X;
    char* p = buf;
    X.nh_d = reinterpret_cast<uint64_t*>(p); p += lanes * nhE * 8;
    X.res_d = reinterpret_cast<uint64_t*>(p); p += lanes * resE * 8;
    X.nh_idx = reinterpret_cast<uint32_t*>(p); p += lanes * nhE * 4;
    X.res_idx = reinterpret_cast<uint32_t*>(p); p += lanes * resE * 4;
    X.dead = reinterpret_cast<uint32_t*>(p); p += lanes * XMAXDEAD * 4;
    uint32_t* err = reinterpret_cast<uint32_t*>(p); p += 4;
    X.nh_used = reinterpret_cast<uint8_t*>(p);
    X.lanes = lanes;
    hipMemsetAsync(err, 0, 4, st);
    const unsigned blocks = (unsigned)(lanes / 256);
    ovs_route_out* o = reinterpret_cast<ovs_route_out*>(out);   // or ovs_lookup_out (same size)
    if (t.exact)
        hipLaunchKernelGGL(k_kad_refresh<true>, dim3(blocks), dim3(256), 0, st, V, DC, C, X, qkeys, qsrc, nq, o, sibs,
                           responders, rtts, rpcs, err);
    else
        hipLaunchKernelGGL(k_kad_refresh<false>, dim3(blocks), dim3(256), 0, st, V, DC, C, X, qkeys, qsrc, nq, o, sibs,
                           responders, rtts, rpcs, err);
    e = hipGetLastError();
    uint32_t herr = 0;
    hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, st);
    const hipError_t e2 = hipStreamSynchronize(st);
    hipFree(buf);
    if (e == hipSuccess) e = e2;
    *capacity_error = herr != 0;
    return e;
}

hipError_t kad_refresh_keys(const KadTables& t, uint32_t n, const uint32_t* nodes, uint64_t m, const uint32_t* stale,
                            K160* keys, uint32_t* src, uint64_t cap, uint64_t* total, hipStream_t st)
{
    *total = 0;
    if (m == 0) return hipSuccess;
    const KadView V = kad_make_view(t, nullptr, n);
    uint64_t *cnt = nullptr, *off = nullptr;
    void* tmp = nullptr;
    size_t tmpb = 0;
    hipError_t e;
    if ((e = hipMalloc(&cnt, sizeof(uint64_t) * (m + 1))) != hipSuccess) return e;
    if ((e = hipMalloc(&off, sizeof(uint64_t) * (m + 1))) != hipSuccess) { hipFree(cnt); return e; }
    const unsigned b = (unsigned)((m + 255) / 256);
    hipLaunchKernelGGL(k_kad_refresh_count, dim3(b), dim3(256), 0, st, V, nodes, m, stale, cnt);
    hipMemsetAsync(cnt + m, 0, sizeof(uint64_t), st);
    hipcub::DeviceScan::ExclusiveSum(nullptr, tmpb, cnt, off, m + 1, st);
    if ((e = hipMalloc(&tmp, tmpb)) == hipSuccess) {
        hipcub::DeviceScan::ExclusiveSum(tmp, tmpb, cnt, off, m + 1, st);
        if (keys && src && cap)
            hipLaunchKernelGGL(k_kad_refresh_fill, dim3(b), dim3(256), 0, st, V, nodes, m, stale, off, cap, keys, src);
        hipMemcpyAsync(total, off + m, sizeof(uint64_t), hipMemcpyDeviceToHost, st);
        e = hipStreamSynchronize(st);
    }
    hipFree(cnt); hipFree(off);
    if (tmp) hipFree(tmp);
    return e;
}

}  // namespace ovs
