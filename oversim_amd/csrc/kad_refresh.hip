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
// R reaches 40 (siblingRefreshNodes = 5s), so the LookupVector (2R entries) does not fit
// registers: each lane keeps it in a per-lane scratch slice laid out entry-major (entry j of lane l
// at j * lanes + l), so lanes that walk their vectors in step touch consecutive addresses.  A
// responder's findNode is evaluated when its response is processed (the tables do not change
// during a batch) -- with K2's sorting networks for R <= 8, by insertion into scratch beyond; at
// send time only its size is needed (the response's delay).  The start, responses and timeouts
// share one findNode / merge / sendRpc site.  One lane runs one lookup to completion, then takes
// the next one of the grid-stride loop.
#include <hipcub/hipcub.hpp>

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <mutex>

#include <hip/hip_runtime.h>

#ifdef OVS_KX_STATS
// census build (-DOVS_KX_STATS): what one K2x launch reads and writes, by kind (kad_exhaustive
// prints the counts to stderr as "kxstats ...")
namespace ovs {
__device__ unsigned long long g_kx_stats[16];
}
#define KAD_FN_HOOK(kind) atomicAdd(&::ovs::g_kx_stats[4 + (kind)], 1ull)
#define KX_STAT(i, v) atomicAdd(&::ovs::g_kx_stats[i], (unsigned long long)(v))
#else
#define KX_STAT(i, v) ((void)0)
#endif

#include "kad_dev.hpp"

namespace ovs {

namespace {

// pending-call slots (strictParallelRpcs: <= alpha calls in flight): 4, or 8 for lookupParallelRpcs
// 5..8 (maidsafe.ini:18-19) -- a template parameter XA of the lookup state and the kernel
constexpr int XMAXDEAD = 64;    // nodes whose RPC timed out, per lookup
// responders of a lookup kept in the lane's LDS column when the caller asked for none (the visited
// set, read only after a timeout): scattered 4 B stores to HBM had been ~0.8 GB of partial-sector
// writes per launch on workload R; responders past KXVL go to the HBM row
constexpr int KXVL = 32;

struct XCfg {
    int R, ns, alpha, hcm, k;      // ns: the siblings vector's size (numSiblings <= R)
    int oneway;                    // 1: a KBRTestApp one-way lookup (route message to the result)
    int pad;                       // 1: responder / RTT rows padded to hopCountMax (NONE / -1)
    int lvis;                      // 1: nobody reads the responder rows -- the first KXVL stay in LDS
    int64_t bwFull, bwOne;         // T(L*8/datarate) of a FindNodeResponse with R nodes / one node
    int strict, visitOnlyOnce, newOnResp, newOnTimeout, finishOnFirst;
};

struct XScratch {
    uint32_t* nh_idx;    // [2R][lanes]
    uint64_t* nh_d;      // [2R][lanes]
    uint8_t* nh_used;    // [2R][lanes]
    uint32_t* res_idx;   // [max(R, k)][lanes]: a findNode result of more than 8 nodes
    uint64_t* res_d;
    uint32_t* dead;      // [XMAXDEAD][lanes]
    uint64_t lanes;
};

struct XPend {
    uint32_t node, ninfo, seq;
    int64_t t, tins, tsend;
    bool to;
};

template <int XA>
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
    XPend p[XA];
    uint32_t pvalid;
};

// LookupVector nextHops of 2R <= 16 entries in registers (R <= 8: the bucket refreshes and the
// exhaustive-iterative lookups of the default configuration)
struct XRegNh {
    uint32_t idx[16];
    uint64_t d[16];
    uint32_t used;      // bit i: entry i alreadyUsed
};

// Maintenance-round trace (TR instantiations, kad_maintenance_round): per accepted response its
// arrival at the source; per FindNodeCall sent its destination and its arrival there -- the events
// at which Kademlia::handleRpcCall / handleRpcResponse run routingAdd (Kademlia.cc:1328-1420).
struct XTrace {
    int64_t* tarr;       // [nq][hcm]
    uint32_t* cnode;     // [nq][ccap]
    int64_t* ctime;      // [nq][ccap]
    int ccap;
};

template <bool EX, bool REG, int XA, bool TR = false>
struct XCtx {
    using XL = XLookup<XA>;
    const KadView& V;
    const DelayConsts& DC;
    const XCfg& C;
    const XScratch& X;
    uint64_t lane;
    uint32_t* __restrict__ resp;      // responders of this lookup (hop order), hcm entries
    int64_t* __restrict__ rtt;        // their RTTs (may be null)
    uint32_t* __restrict__ sib;       // ns siblings of this lookup
    uint32_t (*vis)[256] = nullptr;   // C.lvis: the lane's LDS column of its first KXVL responders
    int64_t* __restrict__ tarr = nullptr;    // TR: response arrivals (hop order)
    uint32_t* __restrict__ cn = nullptr;     // TR: calls sent: destination ...
    int64_t* __restrict__ ct = nullptr;      // ... and its arrival there
    int ccap = 0;

    __device__ __forceinline__ uint64_t at(int j) const { return (uint64_t)j * X.lanes + lane; }

    // --- sorted vectors in scratch (BaseKeySortedVector::add, NodeVector.h:381-512) -----------------
    // insert x (distance top dx) into the vector at scratch rows [0, cap) holding *n entries;
    // returns the position or -1 (full and farther than the last, or already present)
    __device__ __forceinline__ int vadd(uint32_t* idx, uint64_t* d, uint8_t* used, int cap, int* n, uint32_t x,
                                        uint64_t dx, const K160& K) const
    {
        const int m = *n;
        if (m == cap) {
            const uint32_t li = idx[at(m - 1)];
            if (li != x && cand_lt<EX>(d[at(m - 1)], li, dx, x, K, V.nodes)) return -1;
        }
        int pos = m;
        for (int i = 0; i < m; ++i) {
            const uint32_t ei = idx[at(i)];
            if (ei == x) return -1;
            if (cand_lt<EX>(dx, x, d[at(i)], ei, K, V.nodes)) { pos = i; break; }
        }
        const int last = m < cap ? m : cap - 1;
        for (int i = last; i > pos; --i) {
            idx[at(i)] = idx[at(i - 1)];
            d[at(i)] = d[at(i - 1)];
            if (used) used[at(i)] = used[at(i - 1)];
        }
        idx[at(pos)] = x;
        d[at(pos)] = dx;
        if (used) used[at(pos)] = 0;
        *n = m < cap ? m + 1 : cap;
        return pos;
    }

    // Kademlia::findNode(key, numRedundantNodes = rs > 8, numSiblings = -1) at node c into the
    // scratch result (Kademlia.cc:1101-1246; b = 1: startIndex = mainIndex).  Returns its size.
    __device__ __forceinline__ int find_node_scratch(uint32_t c, const RespGeo& g, const K160& K, int rs) const
    {
        int n = 0;
        const uint64_t kt = ktop(K);
        const uint64_t dself = dist_hi(node_key(V.nodes, c), K);
        if (g.nsib == 0) {      // an empty sibling table answers [self]
            vadd(X.res_idx, X.res_d, nullptr, rs, &n, c, dself, K);
            return n;
        }
        auto add_blk = [&](const KadBlk* blk) {
            for (int q = 0; q < KBLK; ++q) {
                const uint32_t x = blk->idx[q];
                if (x == NONE) break;
                vadd(X.res_idx, X.res_d, nullptr, rs, &n, x, dclamp(blk->top[q] ^ kt), K);
            }
        };
        auto add_slot = [&](int bucket) {
            if (g.rowlo < 0 || bucket < g.rowlo) return;   // buckets below the stored row are empty
            const KadBlk* blk = slot_blk(V, g.boff, bucket);
            for (int j = 0; j < V.bpb; ++j) add_blk(blk + j);
        };
        if (g.m >= 0) add_slot(g.m);
        if (g.m >= g.endIndex || n < rs) {
            for (int b = g.m - 1; b >= g.endIndex; --b) add_slot(b);
            const KadBlk* L = V.sibb + (uint64_t)(c - V.lo) * V.sbn;     // c itself, then its siblings
            for (int j = 0; j * KBLK < g.nsib + 1; ++j) add_blk(L + j);
        }
        for (int b = g.m + 1; n < rs && b < KEYBITS; ++b) add_slot(b);
        return n;
    }

    // The size of that result without evaluating it: the scan's candidate sets (buckets, sibling
    // table, self) are disjoint (routingAdd's invariants), so the result holds min(rs, candidates
    // visited) nodes.  Needed at send time for the response's delay.
    __device__ __forceinline__ int find_node_size(uint32_t c, const RespGeo& g, int rs) const
    {
        if (g.nsib == 0) return 1;
        const int full = rs < (int)V.n ? rs : (int)V.n;
        if (!V.maybe_short || g.nsib + 1 >= rs) return full;   // the scan always reaches siblings + self
        int n = 0;
        auto cnt_slot = [&](int bucket) {
            if (g.rowlo < 0 || bucket < g.rowlo) return;
            const KadBlk* blk = slot_blk(V, g.boff, bucket);
            for (int q = 0; q < V.bpb * KBLK && blk[q / KBLK].idx[q % KBLK] != NONE; ++q) ++n;
        };
        if (g.m >= 0) cnt_slot(g.m);
        if (g.m >= g.endIndex || n < rs) {
            for (int b = g.m - 1; b >= g.endIndex; --b) cnt_slot(b);
            n += g.nsib + 1;
        }
        for (int b = g.m + 1; n < rs && b < KEYBITS; ++b) cnt_slot(b);
        return n < rs ? n : rs;
    }

    // --- the LookupVector: registers (REG, 2R <= 16) or the lane's scratch ---------------------------
    __device__ __forceinline__ int nh_add(XL& L, XRegNh& H, uint32_t x, uint64_t dx) const
    {
        const int cap = 2 * C.R;
        if constexpr (!REG) return vadd(X.nh_idx, X.nh_d, X.nh_used, cap, &L.nnh, x, dx, L.K);
        // BaseKeySortedVector::add: position = entries closer than x; rejected if present or if the
        // vector is full and x is farther than its last entry
        bool dup = false;
        int pos = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if (i < L.nnh) {
                dup |= H.idx[i] == x;
                pos += (H.idx[i] != x && cand_lt<EX>(H.d[i], H.idx[i], dx, x, L.K, V.nodes)) ? 1 : 0;
            }
        }
        if (dup || pos >= cap) return -1;
#pragma unroll
        for (int i = 15; i >= 1; --i)
            if (i > pos) { H.idx[i] = H.idx[i - 1]; H.d[i] = H.d[i - 1]; }
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (i == pos) { H.idx[i] = x; H.d[i] = dx; }
        const uint32_t lo = H.used & ((1u << pos) - 1u);
        H.used = (lo | ((H.used >> pos) << (pos + 1))) & ((1u << cap) - 1u);
        L.nnh = L.nnh + 1 > cap ? cap : L.nnh + 1;
        return pos;
    }

    // The register LookupVector's add loop over one sorted findNode block (handleResponse 853-870),
    // as a merge: nextHops <- the 2R closest distinct nodes of nextHops and the block, alreadyUsed
    // flags travelling with their nodes.  The adds run in the block's (distance) order, so a block
    // node's insertion position is its position in the merged vector; returns how many entered at a
    // position < R (numNewRpcs).
    __device__ __forceinline__ int nh_merge_blk(XL& L, XRegNh& H, const Blk8& r, int cnt) const
    {
        const int cap = 2 * C.R;
        BlkN<16> a;
        Blk8 b;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const bool in = i < L.nnh;
            a.x[i] = in ? H.idx[i] : NONE;
            a.d[i] = in ? H.d[i] : ~0ull;
            a.f[i] = in ? ((H.used >> i) & 1u) : 0u;
        }
        bool dup = false;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            bool dj = j >= cnt;
#pragma unroll
            for (int i = 0; i < 16; ++i) dj |= r.x[j] == a.x[i];
            dup |= j < cnt && dj;
            b.x[j] = dj ? NONE : r.x[j];
            b.d[j] = dj ? ~0ull : r.d[j];
            b.f[j] = 2u;
        }
        if (dup) blk_sort8<false, EX>(b, L.K, V.nodes);     // the nodes already present leave holes: to the end
        blk_merge_top<true, EX, 16, 8>(a, b, L.K, V.nodes);
        L.nnh = blk_trunc(a, cap);
        int numNew = 0;
        uint32_t used = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            H.idx[i] = a.x[i];
            H.d[i] = a.d[i];
            numNew += (i < C.R && a.x[i] != NONE && (a.f[i] & 2u)) ? 1 : 0;
            used |= (a.x[i] != NONE && (a.f[i] & 1u)) ? (1u << i) : 0u;
        }
        H.used = used;
        return numNew;
    }

    __device__ __forceinline__ uint32_t nh_idx(const XRegNh& H, int q) const
    {
        if constexpr (!REG) return X.nh_idx[at(q)];
        uint32_t r = NONE;
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (i == q) r = H.idx[i];
        return r;
    }

    // getNextEntry (IterativeLookup.cc:1172-1182): the first entry neither alreadyUsed nor dead; -1
    __device__ __forceinline__ int nh_next(const XL& L, const XRegNh& H) const
    {
        if constexpr (!REG) {
            for (int q = 0; q < L.nnh; ++q)
                if (!X.nh_used[at(q)] && !(L.nd && is_dead(L, X.nh_idx[at(q)]))) return q;
            return -1;
        }
        uint32_t cand = ~H.used & ((1u << L.nnh) - 1u);
        while (cand) {
            const int e = __ffs((int)cand) - 1;
            if (!L.nd || !is_dead(L, nh_idx(H, e))) return e;
            cand &= cand - 1u;
        }
        return -1;
    }

    __device__ __forceinline__ void nh_set_used(XRegNh& H, int e) const
    {
        if constexpr (!REG) X.nh_used[at(e)] = 1;
        else H.used |= 1u << e;
    }

    __device__ __forceinline__ void nh_remove(XL& L, XRegNh& H, uint32_t x) const
    {
        int q = -1;
        for (int i = 0; i < L.nnh && q < 0; ++i)
            if (nh_idx(H, i) == x) q = i;
        if (q < 0) return;
        if constexpr (!REG) {
            for (int j = q; j + 1 < L.nnh; ++j) {
                X.nh_idx[at(j)] = X.nh_idx[at(j + 1)];
                X.nh_d[at(j)] = X.nh_d[at(j + 1)];
                X.nh_used[at(j)] = X.nh_used[at(j + 1)];
            }
        } else {
#pragma unroll
            for (int j = 0; j < 15; ++j)
                if (j >= q) { H.idx[j] = H.idx[j + 1]; H.d[j] = H.d[j + 1]; }
            H.used = (H.used & ((1u << q) - 1u)) | ((H.used >> (q + 1)) << q);
        }
        --L.nnh;
    }

    __device__ __forceinline__ bool is_dead(const XL& L, uint32_t x) const
    {
        for (int i = 0; i < L.nd; ++i)
            if (X.dead[at(i)] == x) return true;
        return false;
    }

    // visited = the source and every responder.  Without a timeout no responder can be an unused
    // next hop (an evicted entry is farther than the vector's last and never re-enters while the
    // vector only shrinks by eviction), so the list is scanned only after one.
    __device__ __forceinline__ bool visited(const XL& L, uint32_t x) const
    {
        if (x == L.S) return true;
        if (!L.any_to) return false;
        const int t = (int)(threadIdx.x);
        for (int i = 0; i < L.nhop; ++i) {
            KX_STAT(11, (C.lvis && i < KXVL) ? 0 : 1);
            if ((C.lvis && i < KXVL ? vis[i][t] : resp[i]) == x) return true;
        }
        return false;
    }

    // IterativeLookup::sendRpc (656-689) + BaseRpc timeout + SimpleNodeEntry::calcDelay
    __device__ __forceinline__ void lookup_send(XL& L, uint32_t x) const
    {
        // pending slots are indexed by compile-time constants only (a dynamic index would put the
        // array in private memory)
        bool dup = false;
#pragma unroll
        for (int i = 0; i < XA; ++i) {
            const bool me = ((L.pvalid >> i) & 1u) && L.p[i].node == x;   // "RPC already sent"
            L.p[i].ninfo += me ? 1u : 0u;
            dup |= me;
        }
        if (dup) return;
        int slot = -1;
#pragma unroll
        for (int i = XA - 1; i >= 0; --i)
            if (i < C.alpha && !((L.pvalid >> i) & 1u)) slot = i;
        if (slot < 0) { L.err = true; return; }
        int64_t d1 = 0, d2 = 0;
        if (x != L.S) {                         // SimpleUDP delivers to itself without delay
            KX_STAT(3, 1);
            const KadNode rr = load_node(V.nodes, x);
            const int rn = find_node_size(x, resp_geo(rr, L.K), C.R);
            const int64_t cd = coord_ns(L.sx, L.sy, rr.x, rr.y, DC.round);
            const int64_t bwc = DC.bwCall;
            const int64_t newTx = (L.txf > L.now ? L.txf : L.now) + bwc;
            L.txf = newTx;
            d1 = (newTx - L.now) + DC.access2 + cd + bwc;
            const int64_t bwr = rn == C.R ? C.bwFull : rn == 1 ? C.bwOne
                                                              : bw_ns(DC.respBase + DC.respPerNode * rn, DC.datarate, DC.round);
            d2 = 2 * bwr + DC.access2 + cd;
        }
        if constexpr (TR) {
            // the call reaches x at now + d1 whatever happens to its response
            if ((int)L.nsent < ccap) { cn[L.nsent] = x; ct[L.nsent] = L.now + d1; }
            else L.err = true;
        }
        const int64_t tTo = L.now + DC.rpcTimeout;
        const int64_t tResp = L.now + d1 + d2;
        const bool to = tTo <= tResp;           // the timeout was scheduled first: it wins a tie
        const uint32_t sTo = L.seq++, sR = L.seq++;
        // unconditional selects per slot: a guarded store would be folded into one store through a
        // dynamic index, which moves the pending array to private memory
#pragma unroll
        for (int i = 0; i < XA; ++i) {
            const bool me = i == slot;
            XPend& P = L.p[i];
            P.node = me ? x : P.node;
            P.ninfo = me ? 1u : P.ninfo;
            P.tsend = me ? L.now : P.tsend;
            P.to = me ? to : P.to;
            P.seq = me ? (to ? sTo : sR) : P.seq;
            P.t = me ? (to ? tTo : tResp) : P.t;
            P.tins = me ? (to ? L.now : L.now + d1) : P.tins;
        }
        L.pvalid |= 1u << slot;
        ++L.nsent;
        KX_STAT(12, 1);
    }

    // IterativePathLookup::sendRpc (1067-1170), exhaustive
    __device__ __forceinline__ void send_rpcs(XL& L, XRegNh& H, int num) const
    {
        if (L.pfinished) return;
        if (C.hcm && L.hops >= C.hcm) { L.pfinished = true; L.psuccess = false; return; }
        if (C.strict) num = min(num, C.alpha - L.pending);
        if (num == 0 && L.pending == 0 && !C.finishOnFirst) num = C.alpha;
        for (int i = 0; num > 0 && i < C.R; ++i) {
            const int e = nh_next(L, H);
            if (e < 0) break;
            const uint32_t h = nh_idx(H, e);
            if (!C.visitOnlyOnce || !visited(L, h)) {
                ++L.pending;
                --num;
                lookup_send(L, h);
            }
            nh_set_used(H, e);
        }
        if (L.pending == 0) {
            // exhaustive lookups are always successful: addSibling(nextHops[0..R)) -- push_back while
            // the numSiblings-sized vector has room (1147-1156, 436-440)
            int m = L.nnh < C.R ? L.nnh : C.R;
            m = m < C.ns ? m : C.ns;
            KX_STAT(10, m);
            if constexpr (REG) {
#pragma unroll
                for (int q = 0; q < 16; ++q)
                    if (q < m) sib[q] = H.idx[q];
            } else {
                for (int q = 0; q < m; ++q) sib[q] = X.nh_idx[at(q)];
            }
            L.psuccess = true;
            L.pfinished = true;
        }
    }

    __device__ __forceinline__ void count_finished(XL& L) const
    {
        if (L.pfinished && !L.counted) {
            L.counted = true;
            ++L.finishedPaths;
            if (L.hops < L.minHops) L.minHops = L.hops;
            if (L.psuccess) ++L.successfulPaths;
        }
    }

    // checkStop (295-349), parallelPaths = 1, numSiblings > 0
    __device__ __forceinline__ bool check_stop(XL& L) const
    {
        if (L.finishedPaths == 1 || L.pvalid == 0) {
            L.success = L.successfulPaths >= 1 || L.psuccess;
            return true;
        }
        return false;
    }

    // The lookup as one loop with a single findNode, LookupVector merge and sendRpc site (the start,
    // a response and a timeout each reach them through the same code, so each is inlined once):
    //   start (IterativeLookup::start 133-244): findNode(key, k, -1) at the source, all into nextHops,
    //     sendRpc(alpha), checkStop;
    //   per event (handleRpcResponse 488-585 / handleRpcTimeout 588-654): every RpcInfo of the node in
    //     turn -- the first of a response is handleResponse (803-921), the others and those of a
    //     timeout handleTimeout (935-1023) -- each possibly followed by a sendRpc, then checkStop.
    // the loop state of a lookup between iterations (start, the event in hand, its RpcInfos left)
    struct Run {
        XRegNh H;
        XPend cur;
        bool start, handled;
        uint32_t infos;
    };

    __device__ __forceinline__ void init(const XL& L, Run& R) const
    {
        R.H.used = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) { R.H.idx[i] = NONE; R.H.d[i] = ~0ull; }
        R.cur.node = L.S; R.cur.ninfo = 1; R.cur.to = false; R.cur.tsend = 0;
        R.cur.seq = 0; R.cur.t = 0; R.cur.tins = 0;
        R.start = true; R.handled = false;
        R.infos = 1;
    }

    // the next event of the lookup (after checkStop): the earliest pending one by (time, insertion
    // time, sequence); true when the lookup has ended
    __device__ __forceinline__ bool pick(XL& L, Run& R) const
    {
        XPend& cur = R.cur;
        if (check_stop(L)) return true;
        int e = -1;
        int64_t bt = 0, bi = 0;
        uint32_t bs = 0;
#pragma unroll
        for (int i = 0; i < XA; ++i) {
            if (!((L.pvalid >> i) & 1u)) continue;
            const XPend& P = L.p[i];
            if (e < 0 || P.t < bt || (P.t == bt && (P.tins < bi || (P.tins == bi && P.seq < bs)))) {
                e = i; bt = P.t; bi = P.tins; bs = P.seq;
            }
        }
        if (e < 0) return true;
#pragma unroll
        for (int i = 0; i < XA; ++i) {
            const bool me = i == e;
            cur.node = me ? L.p[i].node : cur.node;
            cur.ninfo = me ? L.p[i].ninfo : cur.ninfo;
            cur.tsend = me ? L.p[i].tsend : cur.tsend;
            cur.to = me ? L.p[i].to : cur.to;
        }
        L.pvalid &= ~(1u << e);
        L.now = bt;
        if (cur.to) {
            KX_STAT(13, 1);
            L.any_to = true;                 // setDead(dest)
            if (L.nd < XMAXDEAD) X.dead[at(L.nd++)] = cur.node;
            else { L.err = true; return true; }
        }
        R.infos = cur.ninfo;
        R.handled = false;
        return false;
    }

    // One iteration of the lookup's loop: one RpcInfo of the event in hand, then -- when that was
    // its last -- checkStop and the pick of the next event, in the same iteration (a wave's lanes
    // do not split its iterations between picking and handling); true when the lookup has ended.
    __device__ __forceinline__ bool step(XL& L, Run& R) const
    {
        if (L.err) return true;
        if (handle(L, R)) return true;
        return R.infos == 0 ? pick(L, R) : false;
    }

    // one RpcInfo of the event in hand; true when the lookup has ended
    __device__ __forceinline__ bool handle(XL& L, Run& R) const
    {
        XRegNh& H = R.H;
        XPend& cur = R.cur;
        int num = -1;
        --R.infos;
        if (!R.start && L.pfinished) return false;     // "do not handle finished paths"
        if (R.start || (!cur.to && !R.handled)) {
            R.handled = true;
            bool merge = true;
            if (!R.start) {
                // handleResponse (exhaustive: accepted whatever its step)
                if (L.now > DC.lookupTimeout) { L.pfinished = true; L.psuccess = false; merge = false; }
                else {
                    if (cur.node != L.S) {
                        if (L.nhop < C.hcm) {
                            if (C.lvis && L.nhop < KXVL) vis[L.nhop][threadIdx.x] = cur.node;
                            else { resp[L.nhop] = cur.node; KX_STAT(8, 1); }
                            if (rtt) { rtt[L.nhop] = L.now - cur.tsend; KX_STAT(9, 1); }
                            if constexpr (TR) tarr[L.nhop] = L.now;
                        }
                        ++L.nhop;
                        ++L.hops;
                    }
                    ++L.step;
                    --L.pending;
                }
            }
            if (merge) {
                // the responder's findNode (the source's own at the start) into nextHops (2R)
                const KadNode rn = load_node(V.nodes, cur.node);
                KX_STAT(2, 1);
                KX_STAT(1, R.start ? 0 : 1);
                const RespGeo g = resp_geo(rn, L.K);
                const int rs = R.start ? C.k : C.R;
                int numNew = 0, cnt = 0;
                if (REG || (rs <= 8 && V.bpb == 1)) {
                    // the block form of K2 (sorting networks, kad_dev.hpp): its 8-entry instantiation
                    // reads one block per bucket, so only on tables with k <= 8 (a k = 16 table's
                    // bucket refresh, R = 8, scans both blocks of each bucket below)
                    Blk8 b;
                    // in the sibling zone only the level-sorted row's prefix can enter the answer
                    const int2 rr = g.m <= g.endIndex ? kad_sib_range(g, rn.spare, rs < 8 ? rs : 8) : make_int2(0, -1);
                    cnt = kad_find_node_blk<EX>(V, cur.node, g, L.K, rs, false, b, 1, rr.y, rr.x);
                    if constexpr (REG) numNew = nh_merge_blk(L, H, b, cnt);
                    else {
                        for (int i = 0; i < cnt; ++i) {
                            const int pos = nh_add(L, H, b.x[i], b.d[i]);
                            numNew += (pos >= 0 && pos < C.R) ? 1 : 0;
                        }
                    }
                } else {
                    cnt = find_node_scratch(cur.node, g, L.K, rs);
                    for (int i = 0; i < cnt; ++i) {
                        const int pos = nh_add(L, H, X.res_idx[at(i)], X.res_d[at(i)]);
                        numNew += (pos >= 0 && pos < C.R) ? 1 : 0;
                    }
                }
                if (R.start) {
                    if (cnt == 0) { L.success = false; return true; }   // no next hops known
                    num = C.alpha;
                } else {
                    if (numNew == 0 && C.newOnResp) numNew = 1;
                    num = min(numNew, C.alpha);
                }
            }
        } else {
            // handleTimeout (for a timeout, or a response's further RpcInfos)
            if (L.nd && is_dead(L, cur.node)) nh_remove(L, H, cur.node);   // exhaustive: dead nodes leave nextHops (948-957)
            --L.pending;
            if (L.now > DC.lookupTimeout) { L.pfinished = true; L.psuccess = false; }
            else if (C.newOnTimeout) num = 1;
            else if (L.pending == 0) num = C.alpha;
        }
        if (num >= 0) send_rpcs(L, H, num);
        if (!R.start) count_finished(L);
        R.start = false;
        return false;
    }
};


template <bool EX, bool REG, int XA>
__device__ __forceinline__ void kx_init_lookup(XLookup<XA>& L, const KadView& V, const XCfg& C, const K160* __restrict__ qkeys,
                                               uint32_t S, uint32_t* __restrict__ sib_out, uint64_t q)
{
    L.K = qkeys[q];
    L.S = S;
    const double2 sxy = V.xy[L.S];
    L.sx = sxy.x; L.sy = sxy.y;
    L.now = 0; L.txf = 0; L.seq = 0; L.nsent = 0;
    L.nnh = 0; L.nd = 0; L.nhop = 0;
    L.step = 0; L.hops = 0; L.pending = 0;
    L.pfinished = false; L.psuccess = false; L.counted = false; L.any_to = false; L.success = false; L.err = false;
    L.finishedPaths = 0; L.successfulPaths = 0; L.minHops = 0x7FFFFFFF;
    L.pvalid = 0;
#pragma unroll
    for (int i = 0; i < XA; ++i) {
        L.p[i].node = NONE; L.p[i].ninfo = 0; L.p[i].seq = 0;
        L.p[i].t = 0; L.p[i].tins = 0; L.p[i].tsend = 0; L.p[i].to = false;
    }
    uint32_t* sib = sib_out + q * (uint64_t)C.ns;
    for (int j = 0; j < C.ns; ++j) sib[j] = NONE;
    KX_STAT(0, 1);
    KX_STAT(10, C.ns);
}

// SendToKeyListener / LookupResponse fields of a finished lookup (as ovs_lookup_batch; the
// ovs_lookup_out is written through its ovs_route_out twin, k_lookup_finish's convention), or the
// one-way route message
template <int XA>
__device__ __forceinline__ void kx_emit(const XLookup<XA>& L, const KadView& V, const DelayConsts& DC, const XCfg& C,
                                        uint64_t q, ovs_route_out* __restrict__ out, uint32_t* __restrict__ sib,
                                        uint32_t* __restrict__ resp, int64_t* __restrict__ rtt,
                                        uint32_t* __restrict__ rpcs_out, uint32_t* __restrict__ err)
{
    if (L.err) atomicOr(err, 1u);
    if (C.pad)
        for (int j = L.nhop; j < C.hcm; ++j) {
            resp[j] = NONE;
            if (rtt) rtt[j] = -1;
        }
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
        return;
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

#ifndef OVS_KX_WAVES
// minimum waves per SIMD the register allocator must allow for the register-vector (R <= 8) form
#define OVS_KX_WAVES 2
#endif

// One lane per lookup, one loop iteration per kernel-loop iteration; a lane whose lookup ended
// takes the next one of its wave's contiguous slice of the batch (ballot + popcount, no atomics),
// so a wave does not wait for its longest lookup before its lanes move on (as K2).
// DEF: the default configuration's bucket refresh (default.ini: k = 8, redundantNodes = numSiblings =
// 8, lookupParallelRpcs = 3, hopCountMax 50, strictParallelRpcs and visitOnlyOnce on, the newRpcOn*
// and finishOnFirstUnchanged rules off, no one-way message, no responder record) with those fields
// compile-time constants and three pending slots (XA = 3): 6.9k -> 6.2k instructions, 240 -> 221
// VGPRs, SGPR spills 211 -> 181; workload R 6.06 -> 5.69 ms (profiles/r05_kxdef)
__host__ __device__ inline bool kad_is_def_cfg(const XCfg& C)
{
    return C.R == 8 && C.ns == 8 && C.alpha == 3 && C.k == 8 && C.oneway == 0 && C.strict == 1 && C.visitOnlyOnce == 1 &&
           C.newOnResp == 0 && C.newOnTimeout == 0 && C.finishOnFirst == 0 && C.hcm == 50 && C.pad == 0 && C.lvis == 1;
}
__device__ __forceinline__ XCfg kad_def_cfg(XCfg C)
{
    C.R = 8; C.ns = 8; C.alpha = 3; C.k = 8; C.oneway = 0; C.strict = 1; C.visitOnlyOnce = 1;
    C.newOnResp = 0; C.newOnTimeout = 0; C.finishOnFirst = 0; C.hcm = 50; C.pad = 0; C.lvis = 1;
    return C;
}

// the dynamic tail (as K1's and K2's): static slices cover KX_DYN_STATIC of the batch, the rest goes
// out KX_DYN_CH lookups at a time from a zeroed counter at the front of the lanes' scratch.  The
// exhaustive lookups run long (17 RPCs each on R), so smaller chunks and a larger dynamic share than
// K1's: R 5.34 (0.7, 32) -> 5.24 ms (0.4, 16), profiles/r06_dyn/tune_kx.txt
#ifndef KX_DYN_CH
#define KX_DYN_CH 16
#endif
#ifndef KX_DYN_STATIC
#define KX_DYN_STATIC 0.40
#endif
template <bool EX, bool REG, int XA, bool TR, bool DEF = false>
__global__ __launch_bounds__(256, REG ? OVS_KX_WAVES : 1) void k_kad_refresh(KadView V, DelayConsts DC, XCfg C0, XScratch X,
                                                     const K160* __restrict__ qkeys, const uint32_t* __restrict__ qsrc,
                                                     uint64_t nq, uint64_t chunk, unsigned long long* dyn, uint64_t dyn_from,
                                                     ovs_route_out* __restrict__ out,
                                                     uint32_t* __restrict__ sib_out, uint32_t* __restrict__ resp_out,
                                                     int64_t* __restrict__ rtt_out, uint32_t* __restrict__ rpcs_out,
                                                     uint32_t* __restrict__ err, XTrace T)
{
    const XCfg C = DEF ? kad_def_cfg(C0) : C0;
    const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int wl = threadIdx.x & 63;
    const uint64_t wave = lane >> 6;
    uint64_t cursor = wave * chunk;
    uint64_t end = min(cursor + chunk, dyn ? dyn_from : nq);
    bool more = dyn != nullptr;       // the dynamic tail (as K2's): chunks of KX_DYN_CH may be left
    const uint64_t lt_mask = (wl == 0) ? 0ull : (~0ull >> (64 - wl));
    bool active = false;
    uint64_t q = 0;
    XLookup<XA> L;
    typename XCtx<EX, REG, XA, TR>::Run R;
    // the LDS visited set (C.lvis) is never used by the trace instantiations (kad_exhaustive sets
    // lvis only without a trace): they reserve one row instead of 32 KB
    __shared__ uint32_t kxvis[TR ? 1 : KXVL][256];
    // the sources of the wave's next 64 lookups, preloaded one per lane: a refilled lane's first
    // loads (its coordinates, its own KadNode and rows for the start's findNode) wait for nothing
    // loaded in the same iteration
#ifdef OVS_KX_NO_PRELOAD
    constexpr bool pre_ok = false;    // A/B build
#else
    constexpr bool pre_ok = true;
#endif
    uint32_t pS = 0;
    if (pre_ok && cursor + (uint64_t)wl < end) pS = qsrc[cursor + wl];
    while (true) {
        const uint64_t need = __ballot(!active);
        if (more && need != 0 && cursor >= end) {
            unsigned long long b = 0;
            if (wl == 0) b = atomicAdd(dyn, (unsigned long long)KX_DYN_CH);
            const uint64_t nb = dyn_from + (((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                                            (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)b));
            if (nb < nq) {
                cursor = nb;
                end = min(nb + (uint64_t)KX_DYN_CH, nq);
                if (pre_ok && cursor + (uint64_t)wl < end) pS = qsrc[cursor + wl];
            } else {
                more = false;
            }
        }
        if (need != 0 && cursor < end) {
            const int rank = __popcll(need & lt_mask);
            const uint64_t mine = cursor + (uint64_t)rank;
            const uint32_t ps = pre_ok ? (uint32_t)__shfl((int)pS, rank) : 0u;
            if (!active && mine < end) {
                q = mine;
                active = true;
                kx_init_lookup<EX, REG>(L, V, C, qkeys, pre_ok ? ps : qsrc[q], sib_out, q);
                const XCtx<EX, REG, XA, TR> c0{V, DC, C, X, lane, nullptr, nullptr, nullptr};
                c0.init(L, R);
            }
            cursor += (uint64_t)__popcll(need);
            if (pre_ok && cursor + (uint64_t)wl < end) pS = qsrc[cursor + wl];
        }
        if (!__any(active)) break;
        if (!active) continue;
        uint32_t* sib = sib_out + q * (uint64_t)C.ns;
        uint32_t* resp = resp_out + q * (uint64_t)C.hcm;
        int64_t* rtt = rtt_out ? rtt_out + q * (uint64_t)C.hcm : nullptr;
        XCtx<EX, REG, XA, TR> ctx{V, DC, C, X, lane, resp, rtt, sib};
        ctx.vis = kxvis;
        if constexpr (TR) {
            ctx.tarr = T.tarr + q * (uint64_t)C.hcm;
            ctx.cn = T.cnode + q * (uint64_t)T.ccap;
            ctx.ct = T.ctime + q * (uint64_t)T.ccap;
            ctx.ccap = T.ccap;
        }
        if (ctx.step(L, R)) {
            kx_emit(L, V, DC, C, q, out, sib, resp, rtt, rpcs_out, err);
            if constexpr (TR) {
                for (int j = L.nhop; j < C.hcm; ++j) ctx.tarr[j] = -1;
                for (int j = (int)L.nsent; j < T.ccap; ++j) { ctx.cn[j] = NONE; ctx.ct[j] = -1; }
            }
            active = false;
        }
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

// SimTime(double) on the host (the device's simtime_ns; same IEEE double arithmetic)
int64_t simtime_ns_host(double seconds, int round)
{
    const double x = seconds * 1e9;
    return round ? (int64_t)std::floor(x + 0.5) : (int64_t)x;
}

// The lanes' scratch, kept per device between calls (a batch synchronises before it returns; the
// mutex serialises contexts sharing a device)
std::mutex g_scratch_mu;
char* g_scratch[64] = {};
size_t g_scratch_cap[64] = {};

}  // namespace

hipError_t kad_exhaustive(const KadTables& t, const double2* xy, uint32_t n, const ovs_params& P, const DelayConsts& DC,
                          int R, int ns, bool oneway, const K160* qkeys, const uint32_t* qsrc, uint64_t nq, void* out,
                          uint32_t* sibs, uint32_t* responders, int64_t* rtts, uint32_t* rpcs, int num_cu,
                          hipStream_t st, bool* capacity_error, const KadExhTrace* trace, bool pad, bool internal_resp)
{
    *capacity_error = false;
    if (nq == 0) return hipSuccess;
    const int A = P.lookupParallelRpcs;
    if (A < 1 || A > KAD_MAX_ALPHA || R < 1 || R > 64 || ns < 1 || ns > R || !P.lookupMerge || !P.lookupStrictParallelRpcs ||
        P.hopCountMax < 1 || t.k > KMAX)
        return hipErrorNotSupported;
    const KadView V = kad_make_view(t, xy, n);
    XCfg C;
    C.R = R; C.ns = ns; C.alpha = A; C.hcm = P.hopCountMax; C.k = t.k;
    C.oneway = oneway ? 1 : 0;
    C.pad = pad ? 1 : 0;
#ifdef OVS_KX_NO_LVIS
    C.lvis = 0;                       // A/B build: every responder to the HBM row
#else
    C.lvis = internal_resp && !trace ? 1 : 0;
#endif
    C.strict = P.lookupStrictParallelRpcs; C.visitOnlyOnce = P.lookupVisitOnlyOnce;
    C.newOnResp = P.lookupNewRpcOnEveryResponse; C.newOnTimeout = P.lookupNewRpcOnEveryTimeout;
    C.finishOnFirst = P.lookupFinishOnFirstUnchanged;
    C.bwFull = simtime_ns_host((double)((int64_t)(DC.respBase + DC.respPerNode * R) * 8) / P.datarate, P.simtimeRound);
    C.bwOne = DC.bwResp[1];
    // 2R <= 16: the LookupVector lives in registers and findNode results in sorting-network blocks
    // (the start's own findNode answers k nodes: k = 16, KademliaLarge, takes the scratch form)
    const bool reg = R <= 8 && t.k <= 8;
    // one lane per lookup, as many lanes as are resident at once (occupancy-sized grid); the
    // scratch is sized for the lanes
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess || dev < 0 || dev >= 64) return e != hipSuccess ? e : hipErrorInvalidDevice;
    // the occupancy of each instantiation, per device, filled under the scratch mutex
    static int bpc[64][32] = {};
    const bool a8 = A > 4;     // the 8-slot instantiations serve lookupParallelRpcs 5..8
    const bool tr = trace != nullptr;
    // the default configuration's instantiation (register LookupVector, no trace, <= 4 slots)
#ifdef OVS_KX_NO_DEF
    const bool def = false;          // A/B build: the generic instantiation
#else
    const bool def = reg && !tr && !a8 && !t.exact && kad_is_def_cfg(C);
#endif
    const int ki = (t.exact ? 2 : 0) + (reg ? 1 : 0) + (a8 ? 4 : 0) + (tr ? 8 : 0) + (def ? 16 : 0);
    std::unique_lock<std::mutex> lock(g_scratch_mu);
    if (bpc[dev][ki] == 0) {
        int b = 0;
        hipError_t oe;
#define KOCC(ex, rg, xa) (tr ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_kad_refresh<ex, rg, xa, true>, 256, 0) \
                            : hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_kad_refresh<ex, rg, xa, false>, 256, 0))
        if (a8) {
            if (t.exact) oe = reg ? KOCC(true, true, 8) : KOCC(true, false, 8);
            else oe = reg ? KOCC(false, true, 8) : KOCC(false, false, 8);
        } else {
            if (t.exact) oe = reg ? KOCC(true, true, 4) : KOCC(true, false, 4);
            else if (def) oe = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_kad_refresh<false, true, 3, false, true>, 256, 0);
            else oe = reg ? KOCC(false, true, 4) : KOCC(false, false, 4);
        }
#undef KOCC
        bpc[dev][ki] = (oe == hipSuccess && b > 0) ? b : 1;
    }
#ifndef OVS_KX_OVERSUB
#define OVS_KX_OVERSUB 1
#endif
    // OVS_KX_OVERSUB > 1 (A/B builds): that many lanes per resident slot, each wave a shorter slice
    uint64_t lanes = (uint64_t)num_cu * (uint64_t)bpc[dev][ki] * 256 * OVS_KX_OVERSUB;
    if (lanes > nq) lanes = nq;
    lanes = (lanes + 255) / 256 * 256;
    const uint64_t nhE = reg ? 0 : 2ull * R, resE = reg ? 0 : (uint64_t)(R > t.k ? R : t.k);
    const uint64_t bytes = 8 + lanes * (nhE * (4 + 8 + 1) + resE * (4 + 8) + XMAXDEAD * 4) + 4;
    if (g_scratch_cap[dev] < bytes) {
        if (g_scratch[dev]) { hipDeviceSynchronize(); hipFree(g_scratch[dev]); }
        g_scratch[dev] = nullptr; g_scratch_cap[dev] = 0;
        if ((e = hipMalloc(reinterpret_cast<void**>(&g_scratch[dev]), bytes)) != hipSuccess) return e;
        g_scratch_cap[dev] = bytes;
    }
    char* buf = g_scratch[dev];
    XScratch X;
    unsigned long long* dyn = reinterpret_cast<unsigned long long*>(buf);   // the dynamic tail's counter
    char* p = buf + 8;
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
    const uint64_t waves = lanes / 64;
    uint64_t chunk = (nq + waves - 1) / waves;
    uint64_t dyn_from = nq;
    {
        const uint64_t cs = (uint64_t)((double)nq * KX_DYN_STATIC) / waves;
        if (cs >= (uint64_t)KX_DYN_CH && !std::getenv("OVS_NO_DYN")) {
            chunk = cs;
            dyn_from = cs * waves;
            hipMemsetAsync(dyn, 0, sizeof *dyn, st);
        } else {
            dyn = nullptr;
        }
    }
    ovs_route_out* o = reinterpret_cast<ovs_route_out*>(out);   // or ovs_lookup_out (same size)
    XTrace T{};
    if (tr) { T.tarr = trace->tarr; T.cnode = trace->cnode; T.ctime = trace->ctime; T.ccap = trace->ccap; }
#define KRL(ex, rg, xa)                                                                                                 \
    do {                                                                                                                \
        if (tr) hipLaunchKernelGGL((k_kad_refresh<ex, rg, xa, true>), dim3(blocks), dim3(256), 0, st, V, DC, C, X,    \
                                   qkeys, qsrc, nq, chunk, dyn, dyn_from, o, sibs, responders, rtts, rpcs, err, T);                  \
        else hipLaunchKernelGGL((k_kad_refresh<ex, rg, xa, false>), dim3(blocks), dim3(256), 0, st, V, DC, C, X,      \
                                qkeys, qsrc, nq, chunk, dyn, dyn_from, o, sibs, responders, rtts, rpcs, err, T);                     \
    } while (0)
    if (a8) {
        if (t.exact) { if (reg) KRL(true, true, 8); else KRL(true, false, 8); }
        else { if (reg) KRL(false, true, 8); else KRL(false, false, 8); }
    } else {
        if (t.exact) { if (reg) KRL(true, true, 4); else KRL(true, false, 4); }
        else if (def)
            hipLaunchKernelGGL((k_kad_refresh<false, true, 3, false, true>), dim3(blocks), dim3(256), 0, st, V, DC, C, X,
                               qkeys, qsrc, nq, chunk, dyn, dyn_from, o, sibs, responders, rtts, rpcs, err, T);
        else { if (reg) KRL(false, true, 4); else KRL(false, false, 4); }
    }
#undef KRL
    e = hipGetLastError();
    uint32_t herr = 0;
    hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, st);
    const hipError_t e2 = hipStreamSynchronize(st);
    if (e == hipSuccess) e = e2;
    *capacity_error = herr != 0;
#ifdef OVS_KX_STATS
    {
        unsigned long long s[16] = {};
        hipMemcpyFromSymbol(s, HIP_SYMBOL(g_kx_stats), sizeof(s));
        fprintf(stderr,
                "kxstats lookups=%llu responses=%llu node_handle=%llu node_send=%llu blk_main=%llu blk_lower=%llu "
                "blk_row=%llu blk_higher=%llu resp_w=%llu rtt_w=%llu sib_w=%llu vis_r=%llu rpcs=%llu timeouts=%llu\n",
                s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7], s[8], s[9], s[10], s[11], s[12], s[13]);
        const unsigned long long z[16] = {};
        hipMemcpyToSymbol(HIP_SYMBOL(g_kx_stats), z, sizeof(z));
    }
#endif
    return e;
}

void kad_exhaustive_release(int device)
{
    if (device < 0 || device >= 64) return;
    std::lock_guard<std::mutex> lock(g_scratch_mu);
    if (g_scratch[device]) {
        hipDeviceSynchronize();
        hipFree(g_scratch[device]);
    }
    g_scratch[device] = nullptr;
    g_scratch_cap[device] = 0;
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
