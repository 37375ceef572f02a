// epichord.hip -- EpiChord::findNode (EpiChord.cc:517-629) for a batch of FindNodeCalls against one
// routing snapshot, for gfx950.
//
// One lane per call.  The responder's successor / predecessor lists are copied into the lane and
// the source's receiveNewNode (EpiChord.cc:1178-1209) is applied to them: EpiChordNodeList::addNode
// (EpiChordNodeList.cc:108-161) with its resize, the cache updates updateFinger / setFingerTTL make
// on the way (EpiChordFingerCache.cc:79-142) kept as at most three per-lane deltas over the
// read-only cache row.  findBestHops (EpiChordFingerCache.cc:309-356) then walks the row in its map
// order: removeOldFingers' expiry is a liveness test on the walk, and the source's virtual entry is
// excluded from every answer, so it only counts towards the "cache not empty" test.  Not a hot
// path: it exists so that an EpiChord adapter can delegate findNode exactly.
#include "epichord.hpp"

namespace ovs {

namespace {

struct EpiDelta {
    uint32_t node;
    int64_t last, ttl;
};

struct EpiLane {
    const KeyRec* __restrict__ recs;
    const uint32_t* __restrict__ cnode;
    const int64_t* __restrict__ clast;
    const int64_t* __restrict__ cttl;
    uint64_t c0;
    uint32_t m;            // cache entries of the responder
    uint32_t self;
    K160 me, base;         // the responder's key and key + 1
    int64_t now, cacheTTL;
    EpiDelta d[3];
    int nd;

    __device__ K160 key(uint32_t x) const { return key_of(load_rec(recs, x)); }
    // liveCache map key of x: x - (thisNode + 1)
    __device__ K160 sum(uint32_t x) const { return k_sub(key(x), base); }

    // liveCache.lower_bound(k) over the responder's row
    __device__ uint32_t lower_bound(const K160& k) const
    {
        uint32_t lo = 0, hi = m;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (k_lt(sum(cnode[c0 + mid]), k)) lo = mid + 1; else hi = mid;
        }
        return lo;
    }
    __device__ bool in_row(uint32_t x, uint32_t& j) const
    {
        j = lower_bound(sum(x));
        return j < m && cnode[c0 + j] == x;
    }
    // liveCache entry of x as the call has changed it so far
    __device__ bool get(uint32_t x, int64_t& last, int64_t& ttl) const
    {
        for (int i = 0; i < nd; ++i)
            if (d[i].node == x) { last = d[i].last; ttl = d[i].ttl; return true; }
        uint32_t j;
        if (x == NONE || !in_row(x, j)) return false;
        last = clast[c0 + j];
        ttl = cttl[c0 + j];
        return true;
    }
    __device__ void put(uint32_t x, int64_t last, int64_t ttl)
    {
        for (int i = 0; i < nd; ++i)
            if (d[i].node == x) { d[i].last = last; d[i].ttl = ttl; return; }
        d[nd].node = x; d[nd].last = last; d[nd].ttl = ttl;
        ++nd;
    }
    // EpiChordFingerCache::updateFinger (79-127); a FindNodeCall's source is heard from directly, so
    // the dead cache never decides anything here (oracle/ovs_oracle_epichord.c)
    __device__ void update_finger(uint32_t x, int64_t lu, int64_t ttl)
    {
        if (x == NONE || x == self) return;
        int64_t last, t;
        if (get(x, last, t)) {
            if (lu > last) last = lu;
            if (t > 0 && (ttl > t || ttl == 0)) t = ttl;
            put(x, last, t);
        } else {
            put(x, lu, ttl);
        }
    }
    // EpiChordFingerCache::setFingerTTL (129-142)
    __device__ void set_ttl(uint32_t x, int64_t ttl)
    {
        int64_t last, t;
        if (get(x, last, t)) put(x, last, ttl);
    }
    // lastUpdate of row entry j (an entry the call changed carries its new one)
    __device__ int64_t last_of(uint32_t j) const
    {
        const uint32_t x = cnode[c0 + j];
        int64_t last = clast[c0 + j];
        for (int i = 0; i < nd; ++i)
            if (d[i].node == x) last = d[i].last;
        return last;
    }
    __device__ bool alive(uint32_t j) const
    {
        const uint32_t x = cnode[c0 + j];
        int64_t last = clast[c0 + j], ttl = cttl[c0 + j];
        for (int i = 0; i < nd; ++i)
            if (d[i].node == x) { last = d[i].last; ttl = d[i].ttl; }
        return !(ttl > 0 && last + ttl < now);      // removeOldFingers (162-187)
    }
};

// one of the responder's node lists: its real entries closest first, thisNode last while !isFull()
struct EpiList {
    uint32_t e[EPI_MAXL + 1];
    int n;
    bool has_self;
    bool forwards;
};

// map key of x in a list: ring offset from the responder (backwards for the predecessor list) - 1
__device__ __forceinline__ K160 list_sum(const EpiLane& S, const EpiList& Lst, uint32_t x)
{
    const K160 one = k_pow2(0);
    K160 off = k_sub(S.key(x), S.me);
    if (!Lst.forwards) off = k_sub(K160{{0, 0, 0, 0, 0}}, off);
    return k_sub(off, one);
}

__device__ __forceinline__ bool list_contains(const EpiLane& S, const EpiList& Lst, uint32_t x)
{
    if (Lst.has_self && x == S.self) return true;
    for (int i = 0; i < Lst.n; ++i)
        if (Lst.e[i] == x) return true;
    return false;
}

__device__ __forceinline__ uint32_t list_last(const EpiLane& S, const EpiList& Lst)
{
    return Lst.has_self ? S.self : Lst.e[Lst.n - 1];
}

// EpiChordNodeList::addNode(x, resize = true) (108-161), x a node other than the responder
__device__ void list_add(EpiLane& S, EpiList& Lst, int L, uint32_t x)
{
    if (!list_contains(S, Lst, x)) {
        const K160 k = list_sum(S, Lst, x);
        int pos = Lst.n;
        while (pos > 0 && k_lt(k, list_sum(S, Lst, Lst.e[pos - 1]))) {
            Lst.e[pos] = Lst.e[pos - 1];
            --pos;
        }
        Lst.e[pos] = x;
        ++Lst.n;
    }
    S.update_finger(x, S.now, 0);
    if (Lst.n + (Lst.has_self ? 1 : 0) > L) {
        if (Lst.has_self) {
            Lst.has_self = false;                 // thisNode has the largest map key: it goes first
        } else {
            S.set_ttl(Lst.e[Lst.n - 1], S.cacheTTL);
            --Lst.n;
        }
    }
}

__device__ __forceinline__ K160 ring_distance(const K160& x, const K160& y)
{
    const K160 d1 = k_sub(x, y), d2 = k_sub(y, x);
    return k_gt(d1, d2) ? d2 : d1;      // KeyRingMetric::distance (Comparator.h:121-131)
}

__global__ __launch_bounds__(128) void k_epichord_find_node(EpiTables T, const KeyRec* __restrict__ recs,
                                                            const uint32_t* __restrict__ qnode,
                                                            const K160* __restrict__ qkey,
                                                            const uint32_t* __restrict__ qsrc,
                                                            const int64_t* __restrict__ qnow, uint64_t nq, int R,
                                                            int64_t cacheTTL, uint32_t* __restrict__ out_nodes,
                                                            int64_t* __restrict__ out_last, uint32_t max_out,
                                                            uint8_t* __restrict__ out_count,
                                                            uint8_t* __restrict__ out_status)
{
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    const uint32_t v = qnode[q];
    const K160 K = qkey[q];
    const uint32_t src = qsrc[q];
    if (v >= T.n || (src != NONE && src >= T.n)) {
        // a device-pointer call with an index outside the network: answered as invalid, never read
        out_count[q] = 0;
        out_status[q] = 3;
        for (uint32_t i = 0; i < max_out; ++i) { out_nodes[q * max_out + i] = NONE; out_last[q * max_out + i] = -1; }
        return;
    }
    EpiLane S;
    S.recs = recs; S.cnode = T.cnode; S.clast = T.clast; S.cttl = T.cttl;
    S.c0 = T.coff[v];
    S.m = (uint32_t)(T.coff[v + 1] - S.c0);
    S.self = v;
    S.me = S.key(v);
    S.base = k_add(S.me, k_pow2(0));
    S.now = qnow[q];
    S.cacheTTL = cacheTTL;
    S.nd = 0;
    const uint32_t meta = T.meta[v];
    EpiList Sl, Pl;
    Sl.n = (int)(meta & 0xFFu);
    Pl.n = (int)((meta >> 8) & 0xFFu);
    Sl.has_self = !((meta >> 16) & 1u);
    Pl.has_self = !((meta >> 17) & 1u);
    Sl.forwards = true;
    Pl.forwards = false;
    for (int i = 0; i < Sl.n; ++i) Sl.e[i] = T.succ[(uint64_t)v * T.L + i];
    for (int i = 0; i < Pl.n; ++i) Pl.e[i] = T.pred[(uint64_t)v * T.L + i];

    uint32_t* on = out_nodes + q * max_out;
    int64_t* ol = out_last + q * max_out;
    uint32_t cnt = 0;
    auto push = [&](uint32_t x, int64_t t) {
        on[cnt] = x;
        ol[cnt] = t;
        ++cnt;
    };
    uint32_t ex[3] = {v, NONE, NONE};

    if (src != NONE) {
        // receiveNewNode(source, true, OBSERVED, now) (546-553, 1178-1209)
        ex[1] = src;
        S.update_finger(src, S.now, cacheTTL);
        if (!list_contains(S, Sl, src) &&
            (Sl.has_self || between_open(S.key(src), S.me, S.key(list_last(S, Sl)))))
            list_add(S, Sl, T.L, src);
        if (!list_contains(S, Pl, src) &&
            (Pl.has_self || between_open(S.key(src), S.key(list_last(S, Pl)), S.me)))
            list_add(S, Pl, T.L, src);
    }
    const bool pempty = Pl.n == 0, sempty = Sl.n == 0;
    const uint32_t pred0 = pempty ? v : Pl.e[0], succ0 = sempty ? v : Sl.e[0];
    // isSiblingFor(thisNode, key, 1) (650-721)
    const bool sib = pempty ? (sempty || k_eq(K, S.me)) : between_R(K, S.key(pred0), S.me);
    uint8_t status = 0;
    if (sib) {
        push(v, S.now);
        int64_t last, ttl;
        if (!pempty) push(pred0, S.get(pred0, last, ttl) ? last : S.now);
        if (!sempty) push(succ0, S.get(succ0, last, ttl) ? last : S.now);
    } else {
        uint32_t choice;
        if (src == NONE) {
            const K160 sd = ring_distance(S.key(succ0), K), pd = ring_distance(S.key(pred0), K);
            choice = k_lt(pd, sd) ? pred0 : succ0;
        } else if (between_open(S.me, S.key(src), K)) {
            choice = succ0;
        } else {
            choice = pred0;
        }
        int64_t last, ttl;
        if (choice != v && S.get(choice, last, ttl)) {
            push(choice, last);
            ex[2] = choice;
        }
        // findBestHops (309-356): the row's live entries from lower_bound(key - (self + 1))
        bool nonempty = false;
        uint32_t j;
        if (src != NONE && src != v && !S.in_row(src, j)) nonempty = true;    // the source's new entry
        for (uint32_t i = 0; i < S.m && !nonempty; ++i) nonempty = S.alive(i);
        if (!nonempty) {
            status = 2;
        } else if (S.m > 0) {
            uint32_t lb = S.lower_bound(k_sub(K, S.base));
            if (lb == S.m) lb = 0;
            bool found = false;
            uint32_t first = 0;
            for (uint32_t s = 0; s < S.m && !found; ++s) {
                const uint32_t i = lb + s < S.m ? lb + s : lb + s - S.m;
                const uint32_t x = S.cnode[S.c0 + i];
                if (S.alive(i) && x != ex[0] && x != ex[1] && x != ex[2]) { found = true; first = i; }
            }
            int taken = 0;
            for (uint32_t s = 0; found && s < S.m && taken < R; ++s) {
                const uint32_t i = first >= s ? first - s : first + S.m - s;
                const uint32_t x = S.cnode[S.c0 + i];
                if (S.alive(i) && x != ex[0] && x != ex[1] && x != ex[2]) {
                    push(x, S.last_of(i));
                    ++taken;
                }
            }
        }
        if (status == 0 && cnt == 0) status = 1;    // "EpiChord::findNode() Failed to find node"
    }
    out_count[q] = (uint8_t)cnt;
    out_status[q] = status;
    for (uint32_t i = cnt; i < max_out; ++i) { on[i] = NONE; ol[i] = -1; }
}

}  // namespace

void epichord_free(EpiTables& t)
{
    void* ptrs[] = {t.succ, t.pred, t.meta, t.coff, t.cnode, t.clast, t.cttl};
    for (void* p : ptrs)
        if (p) hipFree(p);
    t = EpiTables{};
}

hipError_t epichord_find_node(const EpiTables& t, const KeyRec* recs, const uint32_t* node, const K160* keys,
                              const uint32_t* src, const int64_t* now, uint64_t nq, int numRedundant, int64_t cacheTTL,
                              uint32_t* out_nodes, int64_t* out_last, uint32_t max_out, uint8_t* out_count,
                              uint8_t* out_status, hipStream_t st)
{
    if (nq == 0) return hipSuccess;
    const uint64_t blocks = (nq + 127) / 128;
    hipLaunchKernelGGL(k_epichord_find_node, dim3((unsigned)blocks), dim3(128), 0, st, t, recs, node, keys, src, now,
                       nq, numRedundant, cacheTTL, out_nodes, out_last, max_out, out_count, out_status);
    return hipGetLastError();
}

}  // namespace ovs
