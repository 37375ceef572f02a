// kad_shard.hip -- multi-GPU Kademlia: lookups stay on their home rank, FindNodeCalls
// are requests to the rank that owns the responder.
//
// The sorted ID array is cut into contiguous arcs (= ID prefixes); rank r owns the
// sibling entries and bucket rows of its arc.  The 64 B node records (key, sibling
// radius, mask) and the coordinates are replicated, so everything a lookup needs at
// *send* time -- the responder's isSiblingFor flag, hence the response size and the
// RTT (IterativeLookup::sendRpc -> SimpleNodeEntry::calcDelay) -- is local.  Only the
// responder's findNode result (Kademlia.cc:1101-1246) needs the owner's tables: it is
// requested when the RPC is sent and delivered before the lookup's next round, i.e.
// before the simulated response event can be processed.
//
// Per round (oversim_amd/shard.py drives it):
//   k_kad_shard_step  : every active lookup processes its events in simulated-time
//                       order until the earliest one still waits for a findNode result;
//                       a new RPC stages its request (32 B) in the call's slot, tagged
//                       by owner; compact_by_tag groups them by owner rank (no atomics)
//   all-to-allv       : requests to their owners
//   k_kad_shard_serve : findNode at the responder -> response (104 B)
//   all-to-allv       : responses back to the home rank (reverse splits)
//   k_kad_shard_deliver: results into the lookups' pending-event slots
// The event processing is the single-GPU state machine (kad_dev.hpp), so the result of
// every lookup is identical to k_kad_route's.
#include "kad_dev.hpp"
#include "kad_shard.hpp"

namespace ovs {

namespace {

__device__ __forceinline__ int kshard_owner(const uint64_t* __restrict__ lo, int nsh, uint32_t c)
{
    int r = 0;
    for (int i = 1; i < nsh; ++i) r += ((uint64_t)c >= lo[i]) ? 1 : 0;
    return r;
}

// result slot of pending event `slot` of lookup i
template <bool EX>
struct ShardRes {
    KadRes* __restrict__ res;
    uint64_t base;
    const KadView& V;
    const K160& K;
    int ns;        // numSiblings of the lookup's findNode calls (1 for KBR routes)
    __device__ __forceinline__ bool ready(int slot) const { return res[base + slot].ready != 0; }
    __device__ __forceinline__ void fill(int slot, uint32_t c, const RespGeo& g, bool sb, int numR, bool local,
                                         SVec<8>& v) const
    {
        if (local) {
            // IterativeLookup::start: findNode at the source, on its home rank
            Blk8 b;
            const int n = kad_find_node_blk<EX>(V, c, g, K, numR, sb, b, ns);
#pragma unroll
            for (int i = 0; i < 8; ++i) { v.idx[i] = b.x[i]; v.d[i] = b.d[i]; }
            v.n = n;
            v.used = 0;
            return;
        }
        const KadRes& r = res[base + slot];
        svec_clear(v);
        const int n = (int)r.count;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (j < n) { v.idx[j] = r.nodes[j]; v.d[j] = r.dist[j]; }
        }
        v.n = n;
    }
};

// new FindNodeCall: mark its slot pending and stage the request, tagged with the responder's
// owner, in the call's own slot (a slot carries at most one request per round: a response
// cannot be ready in the round it is requested)
struct ShardSend {
    KadRes* __restrict__ res;
    uint64_t base;
    const K160* K;
    const uint64_t* __restrict__ shard_lo;
    int nsh;
    ovs_kad_req* __restrict__ stage;
    uint8_t* __restrict__ rtag;
    uint32_t pad;   // LookupCall: bit 31 | numSiblings (the responder's findNode argument); 0 for KBR routes
    __device__ __forceinline__ void operator()(int slot, uint32_t x, bool isTo) const
    {
        // a timeout event carries no result
        res[base + slot].ready = isTo ? 1u : 0u;
        if (isTo) return;
        ovs_kad_req q;
        for (int w = 0; w < 5; ++w) q.key[w] = K->w[w];
        q.node = x;
        q.tag = (uint32_t)(base + slot);
        q.pad = pad;
        stage[base + slot] = q;
        rtag[base + slot] = (uint8_t)kshard_owner(shard_lo, nsh, x);
    }
};

struct NoRecord {
    __device__ __forceinline__ void operator()(int, uint32_t) const {}
};

template <int A, bool EX, bool LK>
__global__ __launch_bounds__(256) void k_kad_shard_step(KadView V, DelayConsts DC, KadLC LC,
                                                        KadLookup<A>* __restrict__ st, uint8_t* __restrict__ act,
                                                        const uint32_t* __restrict__ qids, KadRes* __restrict__ res,
                                                        uint64_t nlook, const uint64_t* __restrict__ shard_lo, int nsh,
                                                        ovs_kad_req* __restrict__ rstage, uint8_t* __restrict__ rtag,
                                                        ovs_done_rec* __restrict__ dstage, uint8_t* __restrict__ ltag,
                                                        uint32_t* __restrict__ sib_out)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nlook) return;
    const uint8_t a = act[i];
    if (a == 0) return;            // finished in an earlier round: tags stay 0xFF
    KadLookup<A> L = st[i];
    SVec<8> r;
    const int ns = LK ? LC.numSiblings : 1;
    ShardSend on{res, i * A, &L.K, shard_lo, nsh, rstage, rtag, LK ? (0x80000000u | (uint32_t)ns) : 0u};
    const ShardRes<EX> gr{res, i * A, V, L.K, ns};   // the first event is IterativeLookup::start
    const NoRecord rec;
    while (!kad_lookup_done(L)) {
        if (!kad_lookup_event<A, EX, LK>(L, V, DC, LC, r, gr, on, rec)) break;   // earliest event still waits
    }
    // the lookup's outcome this round, staged at its own index: finished (class 0, its done
    // record) or still active (class 1, counted)
    if (kad_lookup_done(L)) {
        ovs_done_rec dr;
        dr.qid = qids[i];
        dr.pad = 0;
        dr.out = kad_lookup_output(L, V, DC, LC);
        if (LK) {
            // the LookupResponse (BaseOverlay.cc:1272-1300): the answering sibling's findNode
            // result (an exact-key lookup: the key's node), in the lookup's own sibling row
            const bool ok = dr.out.status == OVS_LOOKUP_OK;
            uint32_t cnt = 0;
            if (ns == 0) {
                sib_out[i] = ok ? L.result : NONE;
                cnt = ok ? 1u : 0u;
            } else {
                uint32_t* row = sib_out + i * (uint64_t)ns;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    if (j < ns) {
                        const bool has = ok && j < r.n;
                        row[j] = has ? r.idx[j] : NONE;
                        cnt += has ? 1u : 0u;
                    }
                }
            }
            ovs_lookup_out lo;
            lo.num_siblings = cnt;
            lo.hops = dr.out.hops;
            lo.status = dr.out.status;
            lo.is_valid = ok ? 1 : 0;
            lo.latency_ns = ok ? dr.out.latency_ns : -1;
            __builtin_memcpy(&dr.out, &lo, sizeof lo);
        }
        dstage[i] = dr;
        ltag[i] = 0;
        act[i] = 0;
    } else {
        st[i] = L;
        ltag[i] = 1;
    }
}

template <int A>
__global__ void k_kad_shard_init(const K160* __restrict__ keys, const uint32_t* __restrict__ src, uint64_t n,
                                 uint32_t qid_base, const double2* __restrict__ xy, KadLookup<A>* __restrict__ st,
                                 uint8_t* __restrict__ act, uint32_t* __restrict__ qids, KadRes* __restrict__ res,
                                 uint32_t lo, uint32_t hi, unsigned long long* bad)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t S = src[i];
    qids[i] = qid_base + (uint32_t)i;
    if (S < lo || S >= hi) {
        // the source's own findNode needs its rows: a source off this arc is an error
        // (ovs_kad_shard_errors), and its lookup never runs
        act[i] = 0;
        atomicAdd(bad, 1ull);
        return;
    }
    KadLookup<A> L;
    kad_lookup_init(L, keys[i], S, xy);
    st[i] = L;
    act[i] = 1;
    for (int s = 0; s < A; ++s) res[i * A + s].ready = 1;
}

// findNode at the responder (owned by this rank) for each received request
template <bool EX>
__global__ void k_kad_shard_serve(KadView V, KadLC LC, const ovs_kad_req* __restrict__ in, uint64_t n,
                                  ovs_kad_resp* __restrict__ out)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const ovs_kad_req q = in[j];
    // a LookupCall's request names its numSiblings (ShardSend); a KBR route's uses 1
    const int ns = (q.pad & 0x80000000u) ? (int)(q.pad & 0xFFu) : 1;
    K160 K;
    for (int w = 0; w < 5; ++w) K.w[w] = q.key[w];
    ovs_kad_resp o;
    o.tag = q.tag;
    if (kad_off_arc(V, q.node) || ns > 8 || ns > V.S5) {
        // not this rank's node (the caller mis-routed the request) or a numSiblings the home rank
        // would have refused: answered as undeliverable, counted by the requester's deliver
        o.count = 0xFFFFFFFFu;
        out[j] = o;
        return;
    }
    const KadNode rr = load_node(V.nodes, q.node);
    const bool sb = kad_is_sibling(V, rr, q.node, K, ns);
    SVec<8> r;
    kad_find_node_vec<8, EX>(V, q.node, rr, K, LC.redundant, sb, r, ns);
    o.count = (uint32_t)r.n;
#pragma unroll
    for (int k = 0; k < 8; ++k) { o.nodes[k] = r.idx[k]; o.dist_hi[k] = r.d[k]; }
    out[j] = o;
}

__global__ void k_kad_shard_deliver(const ovs_kad_resp* __restrict__ in, uint64_t n, KadRes* __restrict__ res,
                                    uint64_t nslots, unsigned long long* bad)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const ovs_kad_resp o = in[j];
    if (o.tag >= nslots) { atomicAdd(bad, 1ull); return; }
    KadRes r;
    if (o.count > 8) {
        // a request the serving rank could not answer (not its node): counted for
        // ovs_kad_shard_errors, and the slot completes with an empty result so the lookup ends
        atomicAdd(bad, 1ull);
        r.count = 0;
        r.ready = 1;
#pragma unroll
        for (int k = 0; k < 8; ++k) { r.nodes[k] = NONE; r.dist[k] = ~0ull; }
        res[o.tag] = r;
        return;
    }
    r.count = o.count;
    r.ready = 1;
#pragma unroll
    for (int k = 0; k < 8; ++k) { r.nodes[k] = o.nodes[k]; r.dist[k] = o.dist_hi[k]; }
    res[o.tag] = r;
}

inline unsigned nblk(uint64_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

}  // namespace

bool kad_params_supported_host(const ovs_params& P, const KadTables& t) { return kad_params_supported(P, t); }

size_t kad_lookup_state_bytes(int alpha)
{
    switch (alpha) {
    case 1: return sizeof(KadLookup<1>);
    case 2: return sizeof(KadLookup<2>);
    case 3: return sizeof(KadLookup<3>);
    default: return sizeof(KadLookup<4>);
    }
}

hipError_t kad_shard_init(int alpha, const K160* keys, const uint32_t* src, uint64_t n, uint32_t qid_base,
                          const double2* xy, void* st, uint8_t* act, uint32_t* qids, KadRes* res, uint32_t lo,
                          uint32_t hi, unsigned long long* bad, hipStream_t s)
{
    if (n == 0) return hipSuccess;
#define KI(a) hipLaunchKernelGGL(k_kad_shard_init<a>, dim3(nblk(n, 256)), dim3(256), 0, s, keys, src, n, qid_base, xy, \
                                 (KadLookup<a>*)st, act, qids, res, lo, hi, bad)
    switch (alpha) {
    case 1: KI(1); break;
    case 2: KI(2); break;
    case 3: KI(3); break;
    default: KI(4); break;
    }
#undef KI
    return hipGetLastError();
}

hipError_t kad_shard_step(const KadTables& t, const double2* xy, uint32_t n, const ovs_params& P,
                          const DelayConsts& DC, void* st, uint8_t* act, const uint32_t* qids, KadRes* res,
                          uint64_t nlook, const uint64_t* shard_lo, int nsh, ovs_kad_req* out, uint32_t* out_dest,
                          uint64_t out_cap, unsigned long long* out_count, ovs_done_rec* done, uint64_t done_cap,
                          unsigned long long* done_count, unsigned long long* active_count, int lk_ns,
                          uint32_t* sib_out, unsigned long long* bad, StageBuf& stage, hipStream_t s)
{
    const bool lk = lk_ns >= 0;
    ovs_params Q = P;
    if (lk) Q.numSiblings = lk_ns;
    if (!kad_params_supported(Q, t) || Q.numSiblings != (lk ? lk_ns : 1) || (lk && !sib_out))
        return hipErrorNotSupported;
    if (nlook == 0) return hipSuccess;
    if (nsh < 1 || nsh > MAXSHARDS) return hipErrorInvalidValue;
    KadView V = kad_make_view(t, xy, n);
    V.err = bad;
    KadLC LC = kad_make_lc(Q, t);
    DelayConsts DL = DC;
    DL.lookupCall = lk ? 1 : 0;     // a LookupCall ends at its last response (no route message)
    kad_lc_sizes(LC, DL, n);
    const int A = LC.alpha;
    // stage: a request per pending-call slot, a done record per lookup, and their tags
    const uint64_t ns = nlook * (uint64_t)A;
    const size_t orq = 0, odn = orq + sizeof(ovs_kad_req) * ns, ort = odn + sizeof(ovs_done_rec) * nlook,
                 olt = ort + ns;
    hipError_t e = stage_ensure(stage, olt + nlook, s);
    if (e != hipSuccess) return e;
    uint8_t* sb = static_cast<uint8_t*>(stage.buf);
    ovs_kad_req* rstage = reinterpret_cast<ovs_kad_req*>(sb + orq);
    ovs_done_rec* dstage = reinterpret_cast<ovs_done_rec*>(sb + odn);
    uint8_t* rtag = sb + ort;
    uint8_t* ltag = sb + olt;
    if ((e = hipMemsetAsync(rtag, 0xFF, ns + nlook, s)) != hipSuccess) return e;   // rtag and ltag are adjacent
#define KSX(a, x, l) hipLaunchKernelGGL((k_kad_shard_step<a, x, l>), dim3(nblk(nlook, 256)), dim3(256), 0, s, V, DL, \
                                    LC, (KadLookup<a>*)st, act, qids, res, nlook, shard_lo, nsh, rstage, rtag, dstage, \
                                    ltag, sib_out)
#define KS(a) do { if (t.exact) { if (lk) KSX(a, true, true); else KSX(a, true, false); } \
                   else { if (lk) KSX(a, false, true); else KSX(a, false, false); } } while (0)
    switch (A) {
    case 1: KS(1); break;
    case 2: KS(2); break;
    case 3: KS(3); break;
    default: KS(4); break;
    }
#undef KS
#undef KSX
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // requests grouped by owner rank into out (labels in out_dest), after out_count's records
    CPlan R{};
    R.seg.src = reinterpret_cast<const uint8_t*>(rstage);
    R.seg.src_stride = R.seg.rec_bytes = sizeof(ovs_kad_req);
    R.seg.dst = reinterpret_cast<uint8_t*>(out); R.seg.lab = out_dest; R.seg.counter = out_count;
    R.seg.cap = out_cap; R.seg.n = nsh; R.seg.chain = 1;
    if ((e = compact_by_tag(rtag, ns, R, stage.cs, s)) != hipSuccess) return e;
    // finished lookups appended to done; the still active ones counted
    CPlan D{};
    D.seg.n = 0;
    D.nextra = 2;
    D.extra[0].src = reinterpret_cast<const uint8_t*>(dstage);
    D.extra[0].src_stride = D.extra[0].rec_bytes = sizeof(ovs_done_rec);
    D.extra[0].dst = reinterpret_cast<uint8_t*>(done); D.extra[0].cap = done_cap; D.extra[0].counter = done_count;
    D.extra[1].counter = active_count;
    return compact_by_tag(ltag, nlook, D, stage.cs, s);
}

hipError_t kad_shard_serve(const KadTables& t, uint32_t n, const ovs_params& P, const ovs_kad_req* in, uint64_t nreq,
                           ovs_kad_resp* out, unsigned long long* bad, hipStream_t s)
{
    // numSiblings travels with each request; the rest of the configuration is the rank's
    ovs_params Q = P;
    Q.numSiblings = 1;
    if (!kad_params_supported(Q, t)) return hipErrorNotSupported;
    if (nreq == 0) return hipSuccess;
    KadView V = kad_make_view(t, nullptr, n);
    V.err = bad;
    const KadLC LC = kad_make_lc(P, t);
    if (t.exact) hipLaunchKernelGGL(k_kad_shard_serve<true>, dim3(nblk(nreq, 128)), dim3(128), 0, s, V, LC, in, nreq, out);
    else hipLaunchKernelGGL(k_kad_shard_serve<false>, dim3(nblk(nreq, 128)), dim3(128), 0, s, V, LC, in, nreq, out);
    return hipGetLastError();
}

hipError_t kad_shard_deliver(const ovs_kad_resp* in, uint64_t n, KadRes* res, uint64_t nslots,
                             unsigned long long* bad, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_kad_shard_deliver, dim3(nblk(n, 256)), dim3(256), 0, s, in, n, res, nslots, bad);
    return hipGetLastError();
}

}  // namespace ovs
