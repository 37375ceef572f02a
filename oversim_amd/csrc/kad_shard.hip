// kad_shard.hip -- multi-GPU Kademlia: lookups stay on their home rank, FindNodeCalls to nodes
// of other arcs are requests to the rank that owns the responder.
//
// The sorted ID array is cut into contiguous arcs (= ID prefixes); rank r owns the
// sibling entries and bucket rows of its arc.  The 64 B node records (key, sibling
// radius, mask) and the coordinates are replicated, so everything a lookup needs at
// *send* time -- the responder's isSiblingFor flag, hence the response size and the
// RTT (IterativeLookup::sendRpc -> SimpleNodeEntry::calcDelay) -- is local.  Only the
// responder's findNode result (Kademlia.cc:1101-1246) needs the owner's tables: computed on the
// spot for a responder on this arc, otherwise requested when the RPC is sent and delivered before
// the lookup's next round, i.e. before the simulated response event can be processed.
//
// Per round (oversim_amd/shard.py drives it):
//   shard step (K2,    : the round's lookups process their events in simulated-time order
//   kad_route.hip)       until the earliest one waits for a remote findNode result (then the
//                        lookup is suspended to HBM); a new RPC to another arc stages its request
//                        (32 B) in the call's slot, tagged by owner; compact_by_tag groups them
//                        into per-owner segments and builds the next round's list (no atomics)
//   count all-gather   : per-owner request counts + active lookups of every rank: the round's only
//                        host synchronisation (sizes of both exchanges and the termination test)
//   all-to-allv        : requests to their owners
//   k_kad_shard_serve  : findNode at the responder -> response (104 B)
//   all-to-allv        : responses back to the home rank (reverse splits)
//   k_kad_shard_deliver: results into the lookups' pending-event slots
// The event processing is the single-GPU state machine (kad_dev.hpp), so the result of
// every lookup is identical to the single-GPU K2's; at world size 1 the first round is K2.
#include "kad_dev.hpp"
#include "kad_shard.hpp"

namespace ovs {

namespace {

// a lookup's state record is written only when it first suspends: round 1 starts every lookup
// from its key and source (act = 2), so at world size 1 no state crosses HBM at all.  A result
// slot's ready flag is read only after the send that requested it cleared it: nothing to initialise.
__global__ void k_kad_shard_init(const K160* __restrict__ keys, const uint32_t* __restrict__ src, uint64_t n,
                                 uint32_t qid_base, K160* __restrict__ qkeys, uint32_t* __restrict__ qsrc,
                                 uint8_t* __restrict__ act, uint32_t* __restrict__ qids, uint64_t* __restrict__ iota,
                                 unsigned long long* nlist, uint32_t lo, uint32_t hi, unsigned long long* bad)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) *nlist = n;        // round 1 visits every lookup of the batch
    if (i >= n) return;
    const uint32_t S = src[i];
    qids[i] = qid_base + (uint32_t)i;
    iota[i] = i;
    qkeys[i] = keys[i];
    qsrc[i] = S;
    // the source's own findNode needs its rows: a source off this arc is an error
    // (ovs_kad_shard_errors), and its lookup never runs
    const bool off = S < lo || S >= hi;
    act[i] = off ? 0 : 2;
    if (off) atomicAdd(bad, 1ull);
}

// findNode at the responder (owned by this rank) for each received request
template <bool EX, int C>
__global__ void k_kad_shard_serve(KadView V, KadLC LC, const ovs_kad_req* __restrict__ in, uint64_t n,
                                  typename KadWire<C>::type* __restrict__ out)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const ovs_kad_req q = in[j];
    // a LookupCall's request names its numSiblings (ShardSend); a KBR route's uses 1
    const int ns = (q.pad & 0x80000000u) ? (int)(q.pad & 0xFFu) : 1;
    K160 K;
    for (int w = 0; w < 5; ++w) K.w[w] = q.key[w];
    typename KadWire<C>::type o;
    o.tag = q.tag;
    if (kad_off_arc(V, q.node) || ns > 8 || ns > V.S5) {
        // not this rank's node (the caller mis-routed the request, or the record was never written:
        // TorchExchange fills receive buffers with 0xFF) or a numSiblings the home rank would have
        // refused: answered as undeliverable, counted by the requester's deliver
        o.count = 0xFFFFFFFFu;
        out[j] = o;
        return;
    }
    const KadNode rr = load_node(V.nodes, q.node);
    const bool sb = kad_is_sibling(V, rr, q.node, K, ns);
    SVec<C> r;
    kad_find_node_vec<C, EX>(V, q.node, rr, K, LC.redundant, sb, r, ns);
    o.count = (uint32_t)r.n;
#pragma unroll
    for (int k = 0; k < C; ++k) { o.nodes[k] = r.idx[k]; o.dist_hi[k] = r.d[k]; }
    out[j] = o;
}

template <int C>
__global__ void k_kad_shard_deliver(const typename KadWire<C>::type* __restrict__ in, uint64_t n,
                                    KadResN<C>* __restrict__ res, uint64_t nslots, unsigned long long* bad)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const typename KadWire<C>::type o = in[j];
    if (o.tag >= nslots) { atomicAdd(bad, 1ull); return; }
    KadResN<C> r;
    if (o.count > (uint32_t)C) {
        // a request the serving rank could not answer (not its node): counted for
        // ovs_kad_shard_errors, and the slot completes with an empty result so the lookup ends
        atomicAdd(bad, 1ull);
        r.count = 0;
        r.ready = 1;
#pragma unroll
        for (int k = 0; k < C; ++k) { r.nodes[k] = NONE; r.dist[k] = ~0ull; }
        res[o.tag] = r;
        return;
    }
    r.count = o.count;
    r.ready = 1;
#pragma unroll
    for (int k = 0; k < C; ++k) { r.nodes[k] = o.nodes[k]; r.dist[k] = o.dist_hi[k]; }
    res[o.tag] = r;
}

inline unsigned nblk(uint64_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

template <bool EX>
hipError_t kad_mig_step_dispatch(int A, const KadView& V, const DelayConsts& DC, const KadLC& LC, const KadMigStepArgs& a,
                                 int num_cu, hipStream_t s)
{
    switch (A) {
    case 1: return kad_mig_step_launch<1, EX>(V, DC, LC, a, num_cu, s);
    case 2: return kad_mig_step_launch<2, EX>(V, DC, LC, a, num_cu, s);
    case 3: return kad_mig_step_launch<3, EX>(V, DC, LC, a, num_cu, s);
    case 4: return kad_mig_step_launch<4, EX>(V, DC, LC, a, num_cu, s);
    default: return kad_mig_step_launch<8, EX>(V, DC, LC, a, num_cu, s);
    }
}

template <bool EX>
hipError_t kad_shard_step_dispatch(int A, const KadView& V, const DelayConsts& DC, const KadLC& LC,
                                   const KadShardStepArgs& a, int num_cu, hipStream_t s)
{
    switch (A) {
    case 1: return kad_shard_step_launch<1, EX>(V, DC, LC, a, num_cu, s);
    case 2: return kad_shard_step_launch<2, EX>(V, DC, LC, a, num_cu, s);
    case 3: return kad_shard_step_launch<3, EX>(V, DC, LC, a, num_cu, s);
    case 4: return kad_shard_step_launch<4, EX>(V, DC, LC, a, num_cu, s);
    default: return kad_shard_step_launch<8, EX>(V, DC, LC, a, num_cu, s);
    }
}

}  // namespace

// the sharded path exchanges findNode results of up to 8 nodes (ovs_kad_resp), or 16 for
// KademliaLarge (ovs_kad_resp16): k and lookupRedundantNodes <= 16 (kad_params_supported)
static bool kad_shard_params_supported(const ovs_params& P, const KadTables& t)
{
    return kad_params_supported(P, t) && P.lookupRedundantNodes <= 16 && t.k <= 16;
}

bool kad_params_supported_host(const ovs_params& P, const KadTables& t) { return kad_shard_params_supported(P, t); }

size_t kad_lookup_state_bytes(int alpha, int cap)
{
    const int A = kad_pend_slots(alpha);
    return cap > 8 ? 4 * (size_t)(KadStateWords<1, 16>::value + 7 * (A - 1))
                   : 4 * (size_t)(KadStateWords<1, 8>::value + 7 * (A - 1));
}

uint32_t kad_rec_bytes(int alpha)
{
    switch (kad_pend_slots(alpha)) {
    case 1: return 4u * KadRecWords<1, 8>::value;
    case 2: return 4u * KadRecWords<2, 8>::value;
    case 3: return 4u * KadRecWords<3, 8>::value;
    case 4: return 4u * KadRecWords<4, 8>::value;
    default: return 4u * KadRecWords<8, 8>::value;
    }
}

bool kad_mig_supported(const ovs_params& P, const KadTables& t)
{
    return kad_params_supported(P, t) && P.lookupRedundantNodes <= 8 && t.k <= 8 && t.snapshot && !t.maybe_short &&
           P.numSiblings == 1 && P.routingType == 0;
}

hipError_t kad_mig_step(const KadTables& t, const double2* xy, uint32_t n, const ovs_params& P, const DelayConsts& DC,
                        const void* in, uint64_t nin, const K160* fkeys, const uint32_t* fsrc, uint32_t fqid,
                        const uint64_t* shard_lo, int nsh, int me, void* out, uint64_t out_cap,
                        unsigned long long* out_count, ovs_done_rec* done, uint64_t done_cap,
                        unsigned long long* done_count, unsigned long long* bad, int num_cu, StageBuf& stage,
                        hipStream_t s, unsigned long long* dyn)
{
    if (!kad_mig_supported(P, t)) return hipErrorNotSupported;
    if (nsh < 1 || nsh + 1 > CMAX) return hipErrorInvalidValue;
    if (nin == 0) return hipSuccess;
    const uint32_t RB = kad_rec_bytes(P.lookupParallelRpcs);
    // stage: a record and a done record per input, and its outcome tag
    const size_t om = 0, od = om + (size_t)RB * nin, ot = od + sizeof(ovs_done_rec) * nin;
    hipError_t e = stage_ensure(stage, ot + nin, s);
    if (e != hipSuccess) return e;
    uint8_t* sb = static_cast<uint8_t*>(stage.buf);
    KadView V = kad_make_view(t, xy, n);
    V.err = bad;
    KadLC LC = kad_make_lc(P, t);
    DelayConsts DL = DC;
    DL.lookupCall = 0;
    kad_lc_sizes(LC, DL, n);
    KadMigStepArgs a{};
    a.in = static_cast<const uint32_t*>(in);
    a.fkeys = fkeys; a.fsrc = fsrc; a.fqid = fqid; a.nin = nin;
    a.shard_lo = shard_lo; a.nsh = nsh; a.me = me;
    a.mstage = reinterpret_cast<uint32_t*>(sb + om);
    a.dstage = reinterpret_cast<ovs_done_rec*>(sb + od);
    a.mtag = sb + ot;
    a.dyn = dyn;
    if ((e = hipMemsetAsync(a.mtag, 0xFF, nin, s)) != hipSuccess) return e;
    const int A = kad_pend_slots(LC.alpha);
    e = t.exact ? kad_mig_step_dispatch<true>(A, V, DL, LC, a, num_cu, s)
                : kad_mig_step_dispatch<false>(A, V, DL, LC, a, num_cu, s);
    if (e != hipSuccess) return e;
    CPlan Pl{};
    Pl.seg.src = sb + om; Pl.seg.src_stride = Pl.seg.rec_bytes = RB;
    Pl.seg.dst = static_cast<uint8_t*>(out); Pl.seg.dst_stride = (uint64_t)RB * out_cap;
    Pl.seg.cap = out_cap; Pl.seg.counter = out_count; Pl.seg.n = nsh; Pl.seg.chain = 0;
    Pl.nextra = 1;
    CClass& d = Pl.extra[0];
    d.src = sb + od; d.src_stride = d.rec_bytes = sizeof(ovs_done_rec);
    d.dst = reinterpret_cast<uint8_t*>(done); d.cap = done_cap; d.counter = done_count;
    return compact_by_tag(a.mtag, nin, Pl, stage.cs, s);
}

hipError_t kad_shard_init(const K160* keys, const uint32_t* src, uint64_t n, uint32_t qid_base, K160* qkeys,
                          uint32_t* qsrc, uint8_t* act, uint32_t* qids, uint64_t* iota, unsigned long long* nlist,
                          uint32_t lo, uint32_t hi, unsigned long long* bad, hipStream_t s)
{
    const uint64_t g = n ? n : 1;
    hipLaunchKernelGGL(k_kad_shard_init, dim3(nblk(g, 256)), dim3(256), 0, s, keys, src, n, qid_base, qkeys, qsrc, act,
                       qids, iota, nlist, lo, hi, bad);
    return hipGetLastError();
}

hipError_t kad_shard_step(const KadTables& t, const double2* xy, uint32_t n, const ovs_params& P,
                          const DelayConsts& DC, void* st, uint8_t* act, const K160* qkeys, const uint32_t* qsrc,
                          const uint32_t* qids, void* res,
                          uint64_t nlook, const uint64_t* list, const unsigned long long* nlist, const uint64_t* iota,
                          uint64_t* list_next, unsigned long long* nlist_next, const uint64_t* shard_lo, int nsh,
                          ovs_kad_req* out, uint64_t out_cap, unsigned long long* out_count, ovs_done_rec* done,
                          uint64_t done_cap, unsigned long long* done_count, unsigned long long* active_count, int lk_ns,
                          uint32_t* sib_out, unsigned long long* bad, int num_cu, StageBuf& stage, hipStream_t s)
{
    const bool lk = lk_ns >= 0;
    ovs_params Q = P;
    if (lk) Q.numSiblings = lk_ns;
    if (!kad_shard_params_supported(Q, t) || Q.numSiblings != (lk ? lk_ns : 1) || (lk && !sib_out))
        return hipErrorNotSupported;
    if (nsh < 1 || nsh > MAXSHARDS) return hipErrorInvalidValue;
    hipError_t e;
    if ((e = hipMemsetAsync(nlist_next, 0, sizeof(unsigned long long), s)) != hipSuccess) return e;
    if (nlook == 0) return hipMemsetAsync(active_count, 0, sizeof(unsigned long long), s);
    KadView V = kad_make_view(t, xy, n);
    V.err = bad;
    KadLC LC = kad_make_lc(Q, t);
    DelayConsts DL = DC;
    DL.lookupCall = lk ? 1 : 0;     // a LookupCall ends at its last response (no route message)
    kad_lc_sizes(LC, DL, n);
    const int A = kad_pend_slots(LC.alpha);
    // stage: a request per pending-call slot, a done record per lookup, and their tags
    const uint64_t nslot = nlook * (uint64_t)A;
    const size_t orq = 0, odn = orq + sizeof(ovs_kad_req) * nslot, ort = odn + sizeof(ovs_done_rec) * nlook,
                 olt = ort + nslot;
    if ((e = stage_ensure(stage, olt + nlook, s)) != hipSuccess) return e;
    uint8_t* sb = static_cast<uint8_t*>(stage.buf);
    KadShardStepArgs a{};
    a.st = st; a.act = act; a.qkeys = qkeys; a.qsrc = qsrc; a.res = res; a.list = list; a.nlist_dev = nlist; a.nlist_max = nlook; a.qids = qids;
    a.shard_lo = shard_lo; a.nsh = nsh;
    a.rstage = reinterpret_cast<ovs_kad_req*>(sb + orq);
    a.dstage = reinterpret_cast<ovs_done_rec*>(sb + odn);
    a.rtag = sb + ort;
    a.ltag = sb + olt;
    a.sib_out = lk ? sib_out : nullptr;
    if ((e = hipMemsetAsync(a.rtag, 0xFF, nslot + nlook, s)) != hipSuccess) return e;   // rtag and ltag are adjacent
    e = t.exact ? kad_shard_step_dispatch<true>(A, V, DL, LC, a, num_cu, s)
                : kad_shard_step_dispatch<false>(A, V, DL, LC, a, num_cu, s);
    if (e != hipSuccess) return e;
    // requests grouped by owner rank: segment d at out + d * out_cap, counted in out_count[d]
    CPlan R{};
    R.seg.src = reinterpret_cast<const uint8_t*>(a.rstage);
    R.seg.src_stride = R.seg.rec_bytes = sizeof(ovs_kad_req);
    R.seg.dst = reinterpret_cast<uint8_t*>(out);
    R.seg.dst_stride = out_cap * sizeof(ovs_kad_req);
    R.seg.counter = out_count;
    R.seg.cap = out_cap; R.seg.n = nsh; R.seg.chain = 0;
    if ((e = compact_by_tag(a.rtag, nslot, R, stage.cs, s)) != hipSuccess) return e;
    // finished lookups appended to done; the still active ones are the next round's list
    CPlan D{};
    D.seg.n = 0;
    D.nextra = 2;
    D.extra[0].src = reinterpret_cast<const uint8_t*>(a.dstage);
    D.extra[0].src_stride = D.extra[0].rec_bytes = sizeof(ovs_done_rec);
    D.extra[0].dst = reinterpret_cast<uint8_t*>(done); D.extra[0].cap = done_cap; D.extra[0].counter = done_count;
    D.extra[1].src = reinterpret_cast<const uint8_t*>(iota);
    D.extra[1].src_stride = D.extra[1].rec_bytes = sizeof(uint64_t);
    D.extra[1].dst = reinterpret_cast<uint8_t*>(list_next); D.extra[1].cap = nlook; D.extra[1].counter = nlist_next;
    if ((e = compact_by_tag(a.ltag, nlook, D, stage.cs, s)) != hipSuccess) return e;
    return hipMemcpyAsync(active_count, nlist_next, sizeof(unsigned long long), hipMemcpyDeviceToDevice, s);
}

hipError_t kad_shard_serve(const KadTables& t, uint32_t n, const ovs_params& P, const ovs_kad_req* in, uint64_t nreq,
                           void* out, unsigned long long* bad, hipStream_t s)
{
    // numSiblings travels with each request; the rest of the configuration is the rank's
    ovs_params Q = P;
    Q.numSiblings = 1;
    if (!kad_shard_params_supported(Q, t)) return hipErrorNotSupported;
    if (nreq == 0) return hipSuccess;
    KadView V = kad_make_view(t, nullptr, n);
    V.err = bad;
    const KadLC LC = kad_make_lc(P, t);
#define KS(ex, c) hipLaunchKernelGGL((k_kad_shard_serve<ex, c>), dim3(nblk(nreq, 128)), dim3(128), 0, s, V, LC, in, nreq, \
                                     static_cast<KadWire<c>::type*>(out))
    if (kad_shard_cap(P, t) > 8) { if (t.exact) KS(true, 16); else KS(false, 16); }
    else { if (t.exact) KS(true, 8); else KS(false, 8); }
#undef KS
    return hipGetLastError();
}

hipError_t kad_shard_deliver(int cap, const void* in, uint64_t n, void* res, uint64_t nslots, unsigned long long* bad,
                             hipStream_t s)
{
    if (n == 0) return hipSuccess;
    if (cap > 8)
        hipLaunchKernelGGL(k_kad_shard_deliver<16>, dim3(nblk(n, 256)), dim3(256), 0, s,
                           static_cast<const ovs_kad_resp16*>(in), n, static_cast<KadResN<16>*>(res), nslots, bad);
    else
        hipLaunchKernelGGL(k_kad_shard_deliver<8>, dim3(nblk(n, 256)), dim3(256), 0, s,
                           static_cast<const ovs_kad_resp*>(in), n, static_cast<KadResN<8>*>(res), nslots, bad);
    return hipGetLastError();
}

}  // namespace ovs
