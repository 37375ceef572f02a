// ovs_kbr.cpp -- host implementation of the C ABI declared in include/ovs_kbr.h.
//
// The context owns the device routing tables (sorted 24 B node records,
// fp64 coordinates, CSR finger rows / Kademlia buckets) and one HIP stream.
// Host-pointer calls stage through context-owned scratch buffers and are
// synchronous; OVS_DEVICE_PTRS calls launch asynchronously on the caller's
// stream.  No C++ exception crosses the boundary.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <type_traits>
#include <vector>

#include "ctx_internal.hpp"
#include "epichord.hpp"
#include "host_tables.hpp"
#include "kad.hpp"
#include "kad_shard.hpp"
#include "koorde.hpp"
#include "launch.hpp"
#include "stats.hpp"

using namespace ovs;

struct ovs_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    ovs_params P{};
    int overlay = 0;          // loaded overlay
    uint64_t n = 0;
    bool ideal = true;
    int num_cu = 0;
    // chord
    KeyRec* recs = nullptr;
    double2* xy = nullptr;
    FingerEnt* fingers = nullptr;  // ideal finger rows (64 B entries)
    uint64_t nfing = 0;
    NodeRec* nodes = nullptr;      // ideal node records + finger entries built for successorListSize = nodes_ns
    WinRec* win = nullptr;         // ideal successor windows of the arc [shard_lo, shard_hi)
    int nodes_ns = -1;
    uint32_t* pred = nullptr;
    uint32_t* succ = nullptr;
    uint8_t* nsucc = nullptr;
    uint32_t* fres = nullptr;
    int sls = 0;
    // explicit tables: host copies for batched maintenance (ovs_chord_fix_fingers / _stabilize)
    ChordHost ch;
    // explicit Kademlia tables: host copy for maintenance rounds (ovs_kad_maintenance_round)
    KadHost kh;
    uint64_t shard_lo = 0, shard_hi = 0;   // finger rows exist for [shard_lo, shard_hi)
    FingerEnt* ftop = nullptr;              // replicated top finger levels of every node (ovs_chord_shard_replicate)
    int ftl = 0;
    uint64_t* d_bounds = nullptr;           // device copy of the arc boundaries (MAXSHARDS + 1)
    std::vector<uint64_t> h_bounds;         // ... as last uploaded (uploaded again only on a change)
    std::map<hipStream_t, StageBuf> stage;  // shard-step stage records per stream (cohorts)
    bool bbox_ok = false;                   // the coordinates' bounding box (x0, x1, y0, y1), computed
    double bbox[4] = {0, 0, 0, 0};          // on first use (extendedFingerTable's acceptance rule)
    // kademlia
    KadTables kad{};
    // koorde (on the sorted ring in recs / xy)
    KoordeTables koorde{};
    // epichord routing snapshot (ovs_epichord_load)
    EpiTables epi{};
    uint32_t* kvis = nullptr;            // internal visited lists (K3 without hop_seq, K2x without responders)
    uint64_t kvis_cap = 0;
    hipEvent_t kvis_ev = nullptr;        // recorded after the last launch that used kvis (kvis_acquire)
    bool kvis_used = false;
    // K1's key-order buffers (ksort.hip): sorted keys, sources, caller indices and the sort's
    // histograms, one allocation shared by the calls on this context like kvis (ks_ev orders them)
    uint8_t* ks = nullptr;
    uint64_t ks_cap = 0;
    hipEvent_t ks_ev = nullptr;
    bool ks_used = false;
    // the persistent route kernels' dynamic-tail counters (dyn_acquire): one 64 B slot per launch, a
    // slot's previous launch ordered before its reuse by an event, so concurrent calls on different
    // streams never share a counter
    static constexpr int DYN_SLOTS = 32;
    unsigned long long* dyn = nullptr;
    hipEvent_t dyn_ev[DYN_SLOTS] = {};
    bool dyn_used[DYN_SLOTS] = {};
    uint32_t dyn_seq = 0;
    // multi-GPU Kademlia: this rank's in-flight lookups (ovs_kad_shard_begin)
    void* kst = nullptr;                 // KadLookup<alpha> state records
    uint8_t* kact = nullptr;             // 0 never runs, 1 suspended in kst, 2 not started
    K160* kkeys = nullptr;               // the batch's keys and sources (a lookup starts from them)
    uint32_t* ksrc = nullptr;
    uint32_t* kqids = nullptr;
    void* kres = nullptr;                // alpha findNode result slots per lookup (KadResN<kfcap>)
    unsigned long long* kbad = nullptr;  // undeliverable responses
    uint64_t* kiota = nullptr;           // lookup indices 0..n-1: round 1's list, the source of the next lists
    uint64_t* klist[2] = {nullptr, nullptr};   // ping-pong lists of the still active lookups
    unsigned long long* knl = nullptr;   // [3]: length of iota (round 1), klist[0], klist[1]
    int kcur = 0;                        // list of the next round: 0 = iota, 1/2 = klist[0/1]
    uint64_t knlook = 0, kcap = 0;
    int kalpha = 0;
    int kfcap = 8;                       // findNode capacity of the shard records (8; 16 KademliaLarge)
    int32_t kns = -1;                    // LookupCall batch: numSiblings (-1: KBR routes)
    uint32_t* ksib = nullptr;            // ... and the caller's sibling rows
    // scratch for host-pointer calls
    std::vector<void*> scratch;
    // the sharded round loop (shard_route.cpp): cohort streams and cached buffers
    hipStream_t cohort[4] = {nullptr, nullptr, nullptr, nullptr};
    void* route_scratch = nullptr;
    void (*route_scratch_release)(void*) = nullptr;
};

namespace ovs {

int ctx_device(const ovs_ctx* c) { return c->device; }

ovs_status ctx_fail(ovs_ctx* c, ovs_status s, const std::string& msg)
{
    if (c) c->err = msg;
    return s;
}

hipStream_t ctx_cohort_stream(ovs_ctx* c, int i)
{
    if (i < 0 || i >= 4) return nullptr;
    if (!c->cohort[i] && hipStreamCreateWithFlags(&c->cohort[i], hipStreamNonBlocking) != hipSuccess)
        c->cohort[i] = nullptr;
    return c->cohort[i];
}

void* ctx_route_scratch(ovs_ctx* c) { return c->route_scratch; }

void ctx_set_route_scratch(ovs_ctx* c, void* p, void (*release)(void*))
{
    c->route_scratch = p;
    c->route_scratch_release = release;
}

}  // namespace ovs

namespace {

ovs_status fail(ovs_ctx* c, ovs_status s, const std::string& m)
{
    if (c) c->err = m;
    return s;
}

bool fault_injected(const char* what)
{
    const char* f = std::getenv("OVS_FAULT_INJECT");
    return f && std::strcmp(f, what) == 0;
}

ovs_status hip_fail(ovs_ctx* c, hipError_t e, const char* where)
{
    return fail(c, OVS_EDEVICE, std::string(where) + ": " + hipGetErrorString(e));
}

#define HIPCHK(c, expr)                                        \
    do {                                                       \
        hipError_t e_ = (expr);                                \
        if (e_ != hipSuccess) return hip_fail((c), e_, #expr); \
    } while (0)

void free_tables(ovs_ctx* c)
{
    void* ptrs[] = {c->recs, c->xy, c->fingers, c->pred, c->succ, c->nsucc, c->fres, c->nodes, c->win, c->ftop};
    for (void* p : ptrs)
        if (p) hipFree(p);
    c->nodes = nullptr; c->win = nullptr; c->nodes_ns = -1; c->ftop = nullptr; c->ftl = 0;
    c->recs = nullptr; c->xy = nullptr; c->fingers = nullptr; c->pred = nullptr;
    c->succ = nullptr; c->nsucc = nullptr; c->fres = nullptr;
    kad_free(c->kad);
    koorde_free(c->koorde);
    epichord_free(c->epi);
    if (c->kvis) hipFree(c->kvis);      // hipFree waits for the launches that use it
    c->kvis = nullptr; c->kvis_cap = 0; c->kvis_used = false;
    if (c->ks) hipFree(c->ks);
    c->ks = nullptr; c->ks_cap = 0; c->ks_used = false;
    c->overlay = 0; c->n = 0; c->nfing = 0;
    c->bbox_ok = false;
    c->ch.clear();
    c->kh.clear();
}

void free_kad_shard(ovs_ctx* c)
{
    void* ptrs[] = {c->kst, c->kact, c->kqids, c->kres, c->kbad, c->kiota, c->klist[0], c->klist[1], c->knl,
                    c->kkeys, c->ksrc};
    for (void* p : ptrs)
        if (p) hipFree(p);
    c->kst = nullptr; c->kact = nullptr; c->kqids = nullptr; c->kres = nullptr; c->kbad = nullptr;
    c->kkeys = nullptr; c->ksrc = nullptr;
    c->kiota = nullptr; c->klist[0] = c->klist[1] = nullptr; c->knl = nullptr; c->kcur = 0;
    c->knlook = 0; c->kcap = 0; c->kalpha = 0;
}

// The context's cached scratch for internal visited / hop lists (kvis) is one buffer shared by every
// call on the context.  A call on stream s first waits for the last launch that used it (kvis_ev, on
// whichever stream that was) and records its own use after its launch (kvis_release), so calls on
// different streams -- device-pointer calls return while their kernels run -- never rewrite each
// other's rows.  Growing the buffer waits for that last use only, not for the whole device.
// A zeroed work counter for one launch of a persistent route kernel (the dynamic tail of K1,
// launch_chord_route, and K2, kad_route): nullptr when none can be had -- the kernel then runs static slices only.
static unsigned long long* dyn_acquire(ovs_ctx* c, uint64_t n, hipStream_t s, int* slot)
{
    *slot = -1;
    if (std::getenv("OVS_NO_DYN")) return nullptr;       // A/B: static slices only
    if (n < (1ull << 18)) return nullptr;                 // small batches: static slices (no memset, no event)
    if (!c->dyn && hipMalloc(&c->dyn, 64 * ovs_ctx::DYN_SLOTS) != hipSuccess) { c->dyn = nullptr; return nullptr; }
    const int k = (int)(c->dyn_seq++ % ovs_ctx::DYN_SLOTS);
    if (!c->dyn_ev[k] && hipEventCreateWithFlags(&c->dyn_ev[k], hipEventDisableTiming) != hipSuccess) {
        c->dyn_ev[k] = nullptr;
        return nullptr;
    }
    if (c->dyn_used[k] && hipStreamWaitEvent(s, c->dyn_ev[k], 0) != hipSuccess) return nullptr;
    unsigned long long* p = c->dyn + 8 * k;
    if (hipMemsetAsync(p, 0, sizeof *p, s) != hipSuccess) return nullptr;
    *slot = k;
    return p;
}

static void dyn_release(ovs_ctx* c, hipStream_t s, int slot)
{
    if (slot < 0) return;
    if (hipEventRecord(c->dyn_ev[slot], s) == hipSuccess) c->dyn_used[slot] = true;
    else hipStreamSynchronize(s);                          // no event: the slot is free once the stream is
}

ovs_status kvis_acquire(ovs_ctx* c, uint64_t need, hipStream_t s, uint32_t** out)
{
    if (!c->kvis_ev) {
        const hipError_t e = hipEventCreateWithFlags(&c->kvis_ev, hipEventDisableTiming);
        if (e != hipSuccess) { c->kvis_ev = nullptr; return fail(c, OVS_EDEVICE, std::string("kvis event: ") + hipGetErrorString(e)); }
    }
    if (c->kvis_cap < need) {
        if (c->kvis) {
            if (c->kvis_used) {
                const hipError_t e = hipEventSynchronize(c->kvis_ev);
                if (e != hipSuccess) return fail(c, OVS_EDEVICE, std::string("kvis wait: ") + hipGetErrorString(e));
            }
            hipFree(c->kvis);
            c->kvis = nullptr; c->kvis_cap = 0; c->kvis_used = false;
        }
        const hipError_t e = hipMalloc(&c->kvis, sizeof(uint32_t) * need);
        if (e != hipSuccess) { c->kvis = nullptr; return fail(c, OVS_ENOMEM, "kvis allocation"); }
        c->kvis_cap = need;
    } else if (c->kvis_used) {
        const hipError_t e = hipStreamWaitEvent(s, c->kvis_ev, 0);
        if (e != hipSuccess) return fail(c, OVS_EDEVICE, std::string("kvis stream wait: ") + hipGetErrorString(e));
    }
    *out = c->kvis;
    return OVS_OK;
}

void kvis_release(ovs_ctx* c, hipStream_t s)
{
    if (c->kvis_ev && hipEventRecord(c->kvis_ev, s) == hipSuccess) c->kvis_used = true;
}

// K1 key order, opt-in (OVS_K1_SORT=1): one-way iterative Chord batches of at least
// OVS_K1_SORT_MIN lookups (default 2^20) routed in the order of their keys' top bits.  Off by default:
// measured, the sort costs more than the locality it buys at any bin width one pass can sort
bool ksort_wanted(uint64_t n)
{
    const char* o = std::getenv("OVS_K1_SORT");      // read per call (one getenv per batch)
    const int on = o ? std::atoi(o) : 0;
    const char* m = std::getenv("OVS_K1_SORT_MIN");
    const uint64_t lim = m ? (uint64_t)std::strtoull(m, nullptr, 10) : (1ull << 20);
    return on != 0 && n >= lim && n < 0xFFFFFFFFull;
}

// the key-order buffers for n lookups: sorted keys, sources, caller indices, the sort's scratch
ovs_status ks_acquire(ovs_ctx* c, uint64_t n, hipStream_t s, K160** skeys, uint32_t** ssrc, uint32_t** perm,
                      uint32_t** scr)
{
    const uint64_t need = n * (sizeof(K160) + 8) + 4 * ksort_scratch_words() + 256;
    if (!c->ks_ev) {
        const hipError_t e = hipEventCreateWithFlags(&c->ks_ev, hipEventDisableTiming);
        if (e != hipSuccess) { c->ks_ev = nullptr; return fail(c, OVS_EDEVICE, std::string("ks event: ") + hipGetErrorString(e)); }
    }
    if (c->ks_cap < need) {
        if (c->ks) {
            if (c->ks_used) {
                const hipError_t e = hipEventSynchronize(c->ks_ev);
                if (e != hipSuccess) return fail(c, OVS_EDEVICE, std::string("ks wait: ") + hipGetErrorString(e));
            }
            hipFree(c->ks);
            c->ks = nullptr; c->ks_cap = 0; c->ks_used = false;
        }
        const hipError_t e = hipMalloc(reinterpret_cast<void**>(&c->ks), need);
        if (e != hipSuccess) { c->ks = nullptr; return fail(c, OVS_ENOMEM, "key-order buffers"); }
        c->ks_cap = need;
    } else if (c->ks_used) {
        const hipError_t e = hipStreamWaitEvent(s, c->ks_ev, 0);
        if (e != hipSuccess) return fail(c, OVS_EDEVICE, std::string("ks stream wait: ") + hipGetErrorString(e));
    }
    uint8_t* p = c->ks;
    *scr = reinterpret_cast<uint32_t*>(p);
    p += 4 * ksort_scratch_words();
    *perm = reinterpret_cast<uint32_t*>(p);
    p += 4 * n;
    *ssrc = reinterpret_cast<uint32_t*>(p);
    p += 4 * n;
    *skeys = reinterpret_cast<K160*>(p);
    return OVS_OK;
}

void ks_release(ovs_ctx* c, hipStream_t s)
{
    if (c->ks_ev && hipEventRecord(c->ks_ev, s) == hipSuccess) c->ks_used = true;
}

void free_scratch(ovs_ctx* c)
{
    for (void* p : c->scratch)
        if (p) hipFree(p);
    c->scratch.clear();
}

// SimTime(double) on the host (identical IEEE double arithmetic to the device path)
int64_t simtime_host(double seconds, int round)
{
    const double x = seconds * 1e9;
    return round ? (int64_t)std::floor(x + 0.5) : (int64_t)x;
}

int32_t route_bytes(const ovs_params& P)
{
    // BASEROUTE_L 424 bits + BASEAPPDATA_L 40 bits + KBRTestMessage payload + UDP/IP 28 B
    // (CommonMessages.msg:50-59, SimpleUDP.cc:291)
    return 58 + P.testMsgSize + 28;
}

DelayConsts delay_consts(const ovs_params& P)
{
    DelayConsts d{};
    d.round = P.simtimeRound;
    auto bw = [&](int32_t bytes) { return simtime_host((double)((int64_t)bytes * 8) / P.datarate, P.simtimeRound); };
    const int64_t acc = simtime_host(P.accessDelay, P.simtimeRound);
    d.access2 = 2 * acc;
    d.callBytes = 83;        // FINDNODECALL_L 440 bits + 28 B
    d.respBase = 61;         // FINDNODERESPONSE_L 264 bits + 28 B
    // measureAuthBlock: BASERESPONSE_L adds AUTHBLOCK_L = SIGNATURE_L + CERT_L + PUBKEY_L = 800 bits to
    // every response (CommonMessages.msg:45-47, 57, 73); calls and route messages are unchanged
    if (P.measureAuthBlock) d.respBase += 100;
    if (P.overlay == OVS_OVERLAY_KOORDE) {
        // every Koorde FindNodeCall / FindNodeResponse carries a KoordeFindNodeExtMessage,
        // KEY_L + STEP_L = 168 bits (ChordMessage.msg:33,55; IterativeLookup.cc:385-388,
        // BaseOverlay.cc:1903-1907)
        d.callBytes += 21;
        d.respBase += 21;
    }
    d.respPerNode = 26;      // NODEHANDLE_L 208 bits
    d.routeBytes = route_bytes(P);
    d.msgCall = 2 * bw(d.callBytes) + 2 * acc;
    d.msgResp1 = 2 * bw(d.respBase + d.respPerNode) + 2 * acc;
    d.msgRoute = 2 * bw(route_bytes(P)) + 2 * acc;
    d.rpcTimeout = simtime_host(P.rpcUdpTimeout, P.simtimeRound);
    d.lookupTimeout = simtime_host(P.lookupTimeout, P.simtimeRound);
    d.datarate = P.datarate;
    d.msgRespSib = d.msgResp1;
    d.lookupCall = 0;
    d.bwCall = bw(d.callBytes);
    d.bwRoute = bw(d.routeBytes);
    for (int i = 0; i <= 16; ++i) d.bwResp[i] = bw(d.respBase + d.respPerNode * i);
    return d;
}

ovs_status check_common(ovs_ctx* c, const ovs_params& P)
{
    if (P.keyLength != 160) return fail(c, OVS_ENOTSUP, "keyLength != 160 not supported");
    if (P.routingType < 0 || P.routingType > 4)
        return fail(c, OVS_ENOTSUP, "routingType must be iterative, semi-recursive, full-recursive, exhaustive-iterative "
                                    "or source-routing-recursive");
    const bool rec = P.routingType == 1 || P.routingType == 2 || P.routingType == 4;
    if (P.routingType == 3 && P.overlay != OVS_OVERLAY_KADEMLIA)
        return fail(c, OVS_ENOTSUP, "exhaustive-iterative routing is implemented for Kademlia");
    if (P.routingType == 3 && P.numSiblings > P.lookupRedundantNodes)
        return fail(c, OVS_EINVAL, "With EXHAUSTIVE_ITERATIVE_ROUTING numRedundantNodes must be >= numSiblings!");
    if (rec && P.recNumRedundantNodes < 1)
        return fail(c, OVS_EINVAL, "recNumRedundantNodes must be >= 1");
    if (rec && P.overlay == OVS_OVERLAY_KADEMLIA &&
        (P.recNumRedundantNodes > 16 || P.lookupRedundantNodes > 16 || !(P.rpcKeyTimeout >= 0)))
        return fail(c, OVS_ENOTSUP, "recursive Kademlia implements recNumRedundantNodes, lookupRedundantNodes <= 16 "
                                    "and rpcKeyTimeout >= 0");
    if (P.extendedFingerTable && P.overlay != OVS_OVERLAY_CHORD)
        return fail(c, OVS_ENOTSUP, "extendedFingerTable is implemented for Chord");
    if (P.extendedFingerTable && (P.numFingerCandidates < 1 || P.numFingerCandidates > 64))
        return fail(c, OVS_EINVAL, "numFingerCandidates must be 1..64");
    if (P.lookupParallelPaths != 1) return fail(c, OVS_ENOTSUP, "lookupParallelPaths != 1 not supported");
    if (P.lookupVerifySiblings || P.lookupMajoritySiblings)
        return fail(c, OVS_ENOTSUP, "lookupVerifySiblings/lookupMajoritySiblings not supported");
    if (P.jitter != 0.0)
        return fail(c, OVS_ENOTSUP, "udp.jitter must be 0 (truncnormal jitter is not reproducible)");
    if (!P.useCoordinateBasedDelay) return fail(c, OVS_ENOTSUP, "useCoordinateBasedDelay = false not supported");
    if (P.numSiblings < 0 || P.numSiblings > 8) return fail(c, OVS_EINVAL, "numSiblings out of range");
    if (P.hopCountMax < 0 || P.hopCountMax > 255) return fail(c, OVS_EINVAL, "hopCountMax out of range");
    if (!(P.datarate > 0)) return fail(c, OVS_EINVAL, "datarate must be > 0");
    return OVS_OK;
}

// coordDelay of the farthest pair the bounding box admits (host copy of engine.hpp coord_ns: the
// same IEEE operations; every step is monotone in |dx|, |dy|, so no pair of nodes exceeds it)
int64_t coord_ns_host(double dx, double dy, int round)
{
    const double s2 = dx * dx + dy * dy;
    const float f = (float)std::sqrt(s2);
    return simtime_host(0.001 * (double)f, round);
}

// extendedFingerTable (Chord.cc:416-419, 627-641; ChordFingerTable.cc:195-228) changes a lookup only
// through its start: IterativeLookup::start takes numFingerCandidates nodes from the source's
// findNode, the first of them the non-extended choice, and with lookupMerge = false the first
// response replaces them (IterativeLookup.cc:840-846) while every later FindNodeCall asks for one
// node -- so routes differ only when a first FindNodeCall times out (the reference then tries the
// next candidate).  Accepted when no call can: the largest RTT the coordinates' bounding box admits
// (call + the largest response + twice the farthest coordinate delay) is below rpcUdpTimeout
// (the oracle restates the candidates, tests/test_oracle_extended.py).
ovs_status check_extended_fingers(ovs_ctx* c, const ovs_params& P)
{
    if (!c->ideal)
        return fail(c, OVS_ENOTSUP, "extendedFingerTable: explicit tables carry no finger candidate lists");
    if (P.routingType != 0) return OVS_OK;     // recursive routes: route messages, no RPC timeouts
    if (!c->bbox_ok) {
        if (!c->xy || c->n == 0) return fail(c, OVS_ESTATE, "no network loaded");
        double* d = nullptr;
        HIPCHK(c, hipMalloc(&d, sizeof(double) * 4 * 256));
        int blocks = 0;
        double h[4 * 256];
        hipError_t e = launch_xy_bbox(c->xy, c->n, d, &blocks, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(h, d, sizeof(double) * 4 * blocks, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        hipFree(d);
        if (e != hipSuccess) return hip_fail(c, e, "coordinate bounding box");
        c->bbox[0] = h[0]; c->bbox[1] = h[1]; c->bbox[2] = h[2]; c->bbox[3] = h[3];
        for (int b = 1; b < blocks; ++b) {
            c->bbox[0] = std::min(c->bbox[0], h[4 * b]); c->bbox[1] = std::max(c->bbox[1], h[4 * b + 1]);
            c->bbox[2] = std::min(c->bbox[2], h[4 * b + 2]); c->bbox[3] = std::max(c->bbox[3], h[4 * b + 3]);
        }
        c->bbox_ok = true;
    }
    const DelayConsts DC = delay_consts(P);
    const int64_t cd = coord_ns_host(c->bbox[1] - c->bbox[0], c->bbox[3] - c->bbox[2], P.simtimeRound);
    const int64_t resp = 2 * simtime_host((double)((int64_t)(DC.respBase + DC.respPerNode * (1 + P.successorListSize)) * 8) /
                                              P.datarate, P.simtimeRound) + DC.access2;
    const int64_t rtt = DC.msgCall + std::max(resp, DC.msgResp1) + 2 * cd;
    if (rtt >= DC.rpcTimeout)
        return fail(c, OVS_ENOTSUP,
                    "extendedFingerTable: a FindNodeCall could time out (largest RTT " + std::to_string(rtt) +
                        " ns >= rpcUdpTimeout), where the extended table's next start candidate would be tried");
    return OVS_OK;
}

ovs_status check_chord_route(ovs_ctx* c, const ovs_params& P)
{
    if (P.lookupMerge) return fail(c, OVS_EINVAL, "Chord doesn't work with iterativeLookupConfig.merge = true!");
    if (P.extendedFingerTable) {
        const ovs_status st = check_extended_fingers(c, P);
        if (st != OVS_OK) return st;
    }
    if (P.routingType != 0) {
        // recursive: the route message follows findNode's first acceptable candidate hop by hop
        if (P.numSiblings != 1) return fail(c, OVS_ENOTSUP, "recursive Chord routing implements numSiblings=1");
        if (!c->ideal)
            return fail(c, OVS_ENOTSUP, "recursive routing is implemented for converged (ovs_chord_load) rings");
        return OVS_OK;
    }
    if (P.lookupRedundantNodes != 1 || P.lookupParallelRpcs != 1 || P.numSiblings != 1)
        return fail(c, OVS_ENOTSUP,
                    "Chord route kernel implements lookupRedundantNodes=1, lookupParallelRpcs=1, numSiblings=1");
    return OVS_OK;
}

template <class T>
ovs_status to_device(ovs_ctx* c, const T* src, uint64_t count, bool dev, T** out, bool* owned)
{
    if (dev) { *out = const_cast<T*>(src); *owned = false; return OVS_OK; }
    T* d = nullptr;
    HIPCHK(c, hipMalloc(&d, sizeof(T) * (count ? count : 1)));
    if (count) HIPCHK(c, hipMemcpyAsync(d, src, sizeof(T) * count, hipMemcpyHostToDevice, c->stream));
    *out = d; *owned = true;
    return OVS_OK;
}

// device buffers of one call, freed on every path (early returns included)
struct DevBufs {
    std::vector<void*> p;
    template <class T>
    hipError_t get(T** out, uint64_t count)
    {
        *out = nullptr;
        const hipError_t e = hipMalloc(out, sizeof(T) * (count ? count : 1));
        if (e == hipSuccess) p.push_back(*out);
        return e;
    }
    void own(void* q, bool owned) { if (owned && q) p.push_back(q); }
    ~DevBufs() { for (void* q : p) hipFree(q); }
};

ChordView chord_view(const ovs_ctx* c)
{
    ChordView V{};
    V.recs = c->recs; V.xy = c->xy; V.nodes = c->nodes; V.frow = c->fingers; V.win = c->win;
    V.lo = (uint32_t)c->shard_lo;
    V.pred = c->pred; V.succ = c->succ;
    V.nsucc = c->nsucc; V.fres = c->fres; V.n = (uint32_t)c->n;
    V.ns = (int)std::min<uint64_t>((uint64_t)c->P.successorListSize, c->n - 1);
    V.sls = c->sls;
    V.numFingerCandidates = c->P.numFingerCandidates;
    V.ftop = c->ftop; V.ftl = c->ftop ? c->ftl : 0;
    return V;
}

// NodeRec array of an ideal ring for the current successorListSize (rebuilt when it changes)
ovs_status ensure_nodes(ovs_ctx* c, hipStream_t s)
{
    if (!c->ideal || c->overlay != OVS_OVERLAY_CHORD) return OVS_OK;
    const int ns = (int)std::min<uint64_t>((uint64_t)c->P.successorListSize, c->n - 1);
    if (c->nodes && c->nodes_ns == ns) return OVS_OK;
    if (ns < 1) return fail(c, OVS_EINVAL, "successorListSize must be >= 1");
    if (!c->nodes) HIPCHK(c, hipMalloc(&c->nodes, sizeof(NodeRec) * c->n));
    if (!c->win) HIPCHK(c, hipMalloc(&c->win, sizeof(WinRec) * (c->shard_hi - c->shard_lo)));
    HIPCHK(c, launch_chord_nodes(c->recs, c->xy, (uint32_t)c->n, ns, c->nodes, c->fingers, c->nfing, c->win,
                                 (uint32_t)c->shard_lo, (uint32_t)c->shard_hi, s));
    // the replicated top levels carry their fingers' window distances too
    if (c->ftop) HIPCHK(c, launch_chord_entries(c->nodes, c->ftop, c->n * (uint64_t)c->ftl, s));
    // the records are built once and then read by kernels on any stream (e.g. one stream per
    // cohort of ovs_shard_step): complete them before any other call can see nodes_ns set
    HIPCHK(c, hipStreamSynchronize(s));
    c->nodes_ns = ns;
    return OVS_OK;
}

// upload sorted ids (+ coordinates) into KeyRec / double2 arrays
ovs_status upload_nodes(ovs_ctx* c, const ovs_key160* ids, uint64_t n, const double* xy, bool dev)
{
    if (n < 2) return fail(c, OVS_EINVAL, "need at least 2 nodes");
    if (n >= 0xFFFFFFFFull) return fail(c, OVS_EINVAL, "too many nodes for 32-bit node indices");
    // device inputs may still be being written by work on any of the caller's streams (the load
    // call takes none to order against): the copies below run on the context's own
    // non-blocking stream, so wait for the whole device first (loads are not on the hot path)
    if (dev) HIPCHK(c, hipDeviceSynchronize());
    HIPCHK(c, hipMalloc(&c->recs, sizeof(KeyRec) * n));
    HIPCHK(c, hipMalloc(&c->xy, sizeof(double2) * n));
    // interleave 20 B keys into 24 B records with a strided 2-D copy
    HIPCHK(c, hipMemset2DAsync(c->recs, sizeof(KeyRec), 0, sizeof(KeyRec), n, c->stream));
    HIPCHK(c, hipMemcpy2DAsync(c->recs, sizeof(KeyRec), ids, sizeof(ovs_key160), sizeof(ovs_key160), n,
                               dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->xy, xy, sizeof(double2) * n, dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                             c->stream));
    uint32_t* bad = nullptr;
    HIPCHK(c, hipMalloc(&bad, sizeof(uint32_t)));
    HIPCHK(c, hipMemsetAsync(bad, 0, sizeof(uint32_t), c->stream));
    HIPCHK(c, launch_check_sorted(c->recs, (uint32_t)n, bad, c->stream));
    uint32_t hbad = 0;
    HIPCHK(c, hipMemcpyAsync(&hbad, bad, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    hipFree(bad);
    if (hbad) return fail(c, OVS_EINVAL, "node ids must be sorted ascending and unique");
    c->n = n;
    return OVS_OK;
}

}  // namespace

// ===========================================================================
extern "C" {

int ovs_abi_version(void) { return OVS_ABI_VERSION; }

ovs_status ovs_ctx_create(int hip_device, ovs_ctx** out)
{
    if (!out) return OVS_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return OVS_EDEVICE;
    if (hip_device < 0 || hip_device >= ndev) return OVS_EINVAL;
    ovs_ctx* c = new (std::nothrow) ovs_ctx();
    if (!c) return OVS_ENOMEM;
    c->device = hip_device;
    if (hipSetDevice(hip_device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return OVS_EDEVICE;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, hip_device) == hipSuccess) c->num_cu = prop.multiProcessorCount;
    if (c->num_cu <= 0) c->num_cu = 256;
    ovs_params_default(OVS_OVERLAY_CHORD, &c->P);
    *out = c;
    return OVS_OK;
}

void ovs_ctx_destroy(ovs_ctx* c)
{
    if (!c) return;
    hipSetDevice(c->device);
    // this context's own stream; work the caller queued on its streams (c->stage keys, which the
    // caller may already have destroyed) is ordered before the frees below by hipFree itself, so
    // destroy waits for no other context's or communicator's work
    if (c->stream) hipStreamSynchronize(c->stream);
    free_tables(c);
    free_kad_shard(c);
    free_scratch(c);
    kad_exhaustive_release(c->device);
    if (c->d_bounds) hipFree(c->d_bounds);
    if (c->kvis_ev) hipEventDestroy(c->kvis_ev);
    if (c->ks_ev) hipEventDestroy(c->ks_ev);
    for (int i = 0; i < ovs_ctx::DYN_SLOTS; ++i)
        if (c->dyn_ev[i]) hipEventDestroy(c->dyn_ev[i]);
    if (c->dyn) hipFree(c->dyn);
    if (c->route_scratch && c->route_scratch_release) c->route_scratch_release(c->route_scratch);
    for (auto& kv : c->stage) stage_free(kv.second);
    for (hipStream_t cs : c->cohort)
        if (cs) hipStreamDestroy(cs);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
}

const char* ovs_last_error(const ovs_ctx* c) { return c ? c->err.c_str() : "null context"; }

ovs_status ovs_set_params(ovs_ctx* c, const ovs_params* p)
{
    if (!c || !p) return OVS_EINVAL;
    ovs_status s = check_common(c, *p);
    if (s != OVS_OK) return s;
    if (c->overlay && p->overlay != c->overlay) return fail(c, OVS_ESTATE, "overlay type differs from loaded network");
    if (c->overlay == OVS_OVERLAY_KADEMLIA &&
        (p->k != c->P.k || p->s != c->P.s || p->b != c->P.b || p->kadSeed != c->P.kadSeed ||
         p->bucketType != c->P.bucketType || p->extraNodesFinalBucket != c->P.extraNodesFinalBucket ||
         p->globalNodeLimit != c->P.globalNodeLimit))
        return fail(c, OVS_ESTATE, "k/s/b/kadSeed/bucketType are fixed once a Kademlia network is loaded");
    if (c->overlay == OVS_OVERLAY_KOORDE &&
        (p->successorListSize != c->P.successorListSize || p->shiftingBits != c->P.shiftingBits ||
         p->deBruijnListSize != c->P.deBruijnListSize || p->useOtherLookup != c->P.useOtherLookup ||
         p->useSucList != c->P.useSucList))
        return fail(c, OVS_ESTATE, "the Koorde ring parameters are fixed once a Koorde network is loaded");
    if (c->overlay == OVS_OVERLAY_EPICHORD && p->successorListSize != c->P.successorListSize)
        return fail(c, OVS_ESTATE, "successorListSize is fixed once an EpiChord snapshot is loaded");
    c->P = *p;
    return OVS_OK;
}

ovs_status ovs_get_params(const ovs_ctx* c, ovs_params* p)
{
    if (!c || !p) return OVS_EINVAL;
    *p = c->P;
    return OVS_OK;
}

ovs_status ovs_chord_load(ovs_ctx* c, const ovs_key160* ids, uint64_t n, const double* xy, uint32_t flags)
{
    if (!c || !ids || !xy) return OVS_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    free_tables(c);
    if (c->P.overlay != OVS_OVERLAY_CHORD) return fail(c, OVS_ESTATE, "params.overlay is not Chord");
    ovs_status s = upload_nodes(c, ids, n, xy, flags & OVS_DEVICE_PTRS);
    if (s != OVS_OK) { free_tables(c); return s; }
    hipError_t e = launch_chord_build(c->recs, (uint32_t)n, 0, (uint32_t)n, &c->fingers, &c->nfing, c->stream);
    if (e != hipSuccess) { free_tables(c); return hip_fail(c, e, "chord finger build"); }
    c->overlay = OVS_OVERLAY_CHORD;
    c->ideal = true;
    c->sls = c->P.successorListSize;
    c->shard_lo = 0; c->shard_hi = n;
    return OVS_OK;
}

ovs_status ovs_chord_load_shard(ovs_ctx* c, const ovs_key160* ids, uint64_t n, const double* xy, uint64_t lo,
                                uint64_t hi, uint32_t flags)
{
    if (!c || !ids || !xy || lo >= hi || hi > n) return OVS_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    free_tables(c);
    if (c->P.overlay != OVS_OVERLAY_CHORD) return fail(c, OVS_ESTATE, "params.overlay is not Chord");
    ovs_status s = upload_nodes(c, ids, n, xy, flags & OVS_DEVICE_PTRS);
    if (s != OVS_OK) { free_tables(c); return s; }
    hipError_t e = launch_chord_build(c->recs, (uint32_t)n, (uint32_t)lo, (uint32_t)hi, &c->fingers, &c->nfing, c->stream);
    if (e != hipSuccess) { free_tables(c); return hip_fail(c, e, "chord finger build"); }
    c->overlay = OVS_OVERLAY_CHORD;
    c->ideal = true;
    c->sls = c->P.successorListSize;
    c->shard_lo = lo; c->shard_hi = hi;
    return OVS_OK;
}

ovs_status ovs_chord_shard_replicate(ovs_ctx* c, int32_t top_levels)
{
    if (!c) return OVS_EINVAL;
    if (c->overlay != OVS_OVERLAY_CHORD || !c->ideal) return fail(c, OVS_ESTATE, "no Chord ring (shard) loaded");
    if (top_levels < 0 || top_levels > 32) return fail(c, OVS_EINVAL, "top_levels must be 0..32");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipDeviceSynchronize());        // kernels of earlier steps may still read the old levels
    if (c->ftop) hipFree(c->ftop);
    c->ftop = nullptr; c->ftl = 0;
    if (top_levels == 0) return OVS_OK;
    const uint64_t tot = c->n * (uint64_t)top_levels;
    HIPCHK(c, hipMalloc(&c->ftop, sizeof(FingerEnt) * tot));
    c->ftl = top_levels;
    HIPCHK(c, launch_chord_top(c->recs, (uint32_t)c->n, top_levels, c->ftop, c->stream));
    if (c->nodes) HIPCHK(c, launch_chord_entries(c->nodes, c->ftop, tot, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return OVS_OK;
}

int32_t ovs_chord_shard_levels(const ovs_ctx* c) { return c && c->ftop ? c->ftl : 0; }

ovs_status ovs_shard_make_records(ovs_ctx* c, const ovs_key160* keys, const uint32_t* src, uint64_t n,
                                  uint32_t qid_base, ovs_lookup_rec* recs, void* stream)
{
    if (!c || (n && (!keys || !src || !recs))) return OVS_EINVAL;
    if (c->overlay != OVS_OVERLAY_CHORD || !c->ideal) return fail(c, OVS_ESTATE, "no Chord ring (shard) loaded");
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;   // device-pointer call: NULL = the default stream
    HIPCHK(c, launch_make_records(c->recs, reinterpret_cast<const K160*>(keys), src, n, qid_base, recs, s));
    return OVS_OK;
}

// the arc boundaries on the device: uploaded (synchronously) only when they change, so a step
// never waits for the host copy of a pageable buffer behind the work queued on its stream
ovs_status upload_bounds(ovs_ctx* c, const uint64_t* lo, uint32_t nshards)
{
    if (!c->d_bounds) HIPCHK(c, hipMalloc(&c->d_bounds, sizeof(uint64_t) * (MAXSHARDS + 1)));
    if (c->h_bounds.size() == nshards + 1 && std::equal(lo, lo + nshards + 1, c->h_bounds.begin())) return OVS_OK;
    HIPCHK(c, hipDeviceSynchronize());
    HIPCHK(c, hipMemcpy(c->d_bounds, lo, sizeof(uint64_t) * (nshards + 1), hipMemcpyHostToDevice));
    c->h_bounds.assign(lo, lo + nshards + 1);
    return OVS_OK;
}

// ns = 0: one-way routes (ovs_shard_step); ns >= 1: LookupCalls with that many siblings
static ovs_status shard_step(ovs_ctx* c, int ns, const ovs_lookup_rec* in, uint64_t n_in, ovs_lookup_rec* out,
                             uint64_t out_cap, unsigned long long* out_count, ovs_done_rec* done, uint64_t done_cap,
                             unsigned long long* done_count, const uint64_t* shard_lo, uint32_t nshards, void* stream,
                             const ovs_key160* fkeys = nullptr, const uint32_t* fsrc = nullptr, uint32_t fqid = 0)
{
    if (!c || !shard_lo || nshards == 0 || nshards > (uint32_t)MAXSHARDS) return OVS_EINVAL;
    if (n_in && ((!in && !(fkeys && fsrc)) || !out || !out_count || !done || !done_count)) return OVS_EINVAL;
    if (c->overlay != OVS_OVERLAY_CHORD || !c->ideal) return fail(c, OVS_ESTATE, "no Chord ring (shard) loaded");
    ovs_status st = check_common(c, c->P);
    if (st == OVS_OK) st = check_chord_route(c, c->P);
    if (st != OVS_OK) return st;
    ShardMap M{};
    M.n = (int)nshards;
    int me = -1;
    for (uint32_t r = 0; r <= nshards; ++r) {
        M.lo[r] = shard_lo[r];
        if (r > 0 && shard_lo[r] < shard_lo[r - 1]) return fail(c, OVS_EINVAL, "shard_lo must be non-decreasing");
    }
    if (shard_lo[0] != 0 || shard_lo[nshards] != c->n) return fail(c, OVS_EINVAL, "shard_lo must cover [0, n)");
    for (uint32_t r = 0; r < nshards; ++r)
        if (shard_lo[r] == c->shard_lo && shard_lo[r + 1] == c->shard_hi) me = (int)r;
    if (me < 0) return fail(c, OVS_EINVAL, "this context's arc is not one of shard_lo's arcs");
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;   // device-pointer call: NULL = the default stream
    st = upload_bounds(c, M.lo, nshards);
    if (st != OVS_OK) return st;
    LookupConsts LC{c->P.hopCountMax, ns ? ns : c->P.numSiblings, c->P.lookupRedundantNodes, c->P.routingType != 0};
    DelayConsts DC = delay_consts(c->P);
    if (ns) {
        if (c->P.routingType != 0) return fail(c, OVS_ENOTSUP, "LookupCall is implemented for routingType = iterative");
        // as ovs_lookup_batch: the responsible node answers min(numSiblings, 1 + successors) nodes
        DC.lookupCall = 1;
        const int64_t nsucc = std::min<int64_t>(c->P.successorListSize, (int64_t)c->n - 1);
        const int nodes = (int)std::min<int64_t>(ns, 1 + nsucc);
        DC.msgRespSib = 2 * simtime_host((double)((int64_t)(DC.respBase + DC.respPerNode * nodes) * 8) / c->P.datarate,
                                         c->P.simtimeRound) + DC.access2;
    }
    st = ensure_nodes(c, s);
    if (st != OVS_OK) return st;
    int slot = -1;
    unsigned long long* dyn = dyn_acquire(c, n_in, s, &slot);
    const hipError_t e = launch_chord_shard_step(chord_view(c), DC, LC, c->d_bounds, (int)nshards, me, in, n_in, out,
                                                 out_cap, out_count, done, done_cap, done_count, c->stage[s], c->num_cu,
                                                 s, reinterpret_cast<const K160*>(fkeys), fsrc, fqid, dyn);
    dyn_release(c, s, slot);
    HIPCHK(c, e);
    return OVS_OK;
}

ovs_status ovs_shard_step_keys(ovs_ctx* c, int32_t num_siblings, const ovs_key160* keys, const uint32_t* src, uint64_t n,
                               uint32_t qid_base, ovs_lookup_rec* out, uint64_t out_cap, unsigned long long* out_count,
                               ovs_done_rec* done, uint64_t done_cap, unsigned long long* done_count,
                               const uint64_t* shard_lo, uint32_t nshards, void* stream)
{
    if (!c || (n && (!keys || !src))) return OVS_EINVAL;
    int32_t ns = 0;
    if (num_siblings != 0) {
        ns = num_siblings < 0 ? c->P.successorListSize : num_siblings;
        if (ns > c->P.successorListSize) return fail(c, OVS_EINVAL, "numSiblings too big!");
        if (ns < 1 || ns > 8) return fail(c, OVS_ENOTSUP, "LookupCall across arcs implements numSiblings 1..8");
    }
    return shard_step(c, ns, nullptr, n, out, out_cap, out_count, done, done_cap, done_count, shard_lo, nshards, stream,
                      keys, src, qid_base);
}

ovs_status ovs_shard_step(ovs_ctx* c, const ovs_lookup_rec* in, uint64_t n_in, ovs_lookup_rec* out, uint64_t out_cap,
                          unsigned long long* out_count, ovs_done_rec* done, uint64_t done_cap,
                          unsigned long long* done_count, const uint64_t* shard_lo, uint32_t nshards, void* stream)
{
    return shard_step(c, 0, in, n_in, out, out_cap, out_count, done, done_cap, done_count, shard_lo, nshards, stream);
}

static int32_t shard_lookup_ns(ovs_ctx* c, int32_t num_siblings)
{
    return num_siblings < 0 ? c->P.successorListSize : num_siblings;
}

ovs_status ovs_shard_step_lookup(ovs_ctx* c, int32_t num_siblings, const ovs_lookup_rec* in, uint64_t n_in,
                                 ovs_lookup_rec* out, uint64_t out_cap, unsigned long long* out_count,
                                 ovs_done_rec* done, uint64_t done_cap, unsigned long long* done_count,
                                 const uint64_t* shard_lo, uint32_t nshards, void* stream)
{
    if (!c) return OVS_EINVAL;
    const int32_t ns = shard_lookup_ns(c, num_siblings);
    if (ns > c->P.successorListSize) return fail(c, OVS_EINVAL, "numSiblings too big!");
    if (ns < 1 || ns > 8) return fail(c, OVS_ENOTSUP, "LookupCall across arcs implements numSiblings 1..8");
    return shard_step(c, ns, in, n_in, out, out_cap, out_count, done, done_cap, done_count, shard_lo, nshards, stream);
}

ovs_status ovs_shard_lookup_finish(ovs_ctx* c, const ovs_done_rec* done, uint64_t n, int32_t num_siblings,
                                   ovs_lookup_out* out, uint32_t* siblings, void* stream)
{
    if (!c || (n && (!done || !out || !siblings))) return OVS_EINVAL;
    if (c->overlay != OVS_OVERLAY_CHORD || !c->ideal) return fail(c, OVS_ESTATE, "no Chord ring (shard) loaded");
    const int32_t ns = shard_lookup_ns(c, num_siblings);
    if (ns < 1 || ns > 8) return fail(c, OVS_ENOTSUP, "LookupCall across arcs implements numSiblings 1..8");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, launch_shard_lookup_finish(chord_view(c), ns, done, out, siblings, n, (hipStream_t)stream));
    return OVS_OK;
}

ovs_status ovs_chord_load_tables(ovs_ctx* c, const ovs_key160* ids, uint64_t n, const double* xy,
                                 const uint32_t* pred, const uint32_t* succ, const uint8_t* nsucc,
                                 const uint32_t* fingers, const uint8_t* deque_size, uint32_t flags)
{
    if (!c || !ids || !xy || !pred || !succ || !nsucc || !fingers || !deque_size) return OVS_EINVAL;
    if (flags & OVS_DEVICE_PTRS) return fail(c, OVS_ENOTSUP, "explicit tables are taken from host memory");
    HIPCHK(c, hipSetDevice(c->device));
    free_tables(c);
    if (c->P.overlay != OVS_OVERLAY_CHORD) return fail(c, OVS_ESTATE, "params.overlay is not Chord");
    ovs_status s = upload_nodes(c, ids, n, xy, false);
    if (s != OVS_OK) { free_tables(c); return s; }
    const int sls = c->P.successorListSize;
    // keep the tables on the host too (batched maintenance rewrites them) and resolve
    // ChordFingerTable::getFinger(pos) there (ChordFingerTable.cc:174-193)
    std::string err;
    if (!c->ch.import(reinterpret_cast<const K160*>(ids), n, pred, succ, nsucc, fingers, deque_size, sls, &err)) {
        free_tables(c);
        return fail(c, OVS_EINVAL, err);
    }
    const std::vector<uint32_t>& fres = c->ch.fres;
    HIPCHK(c, hipMalloc(&c->pred, sizeof(uint32_t) * n));
    HIPCHK(c, hipMalloc(&c->succ, sizeof(uint32_t) * n * sls));
    HIPCHK(c, hipMalloc(&c->nsucc, n));
    HIPCHK(c, hipMalloc(&c->fres, sizeof(uint32_t) * n * 160));
    HIPCHK(c, hipMemcpy(c->pred, pred, sizeof(uint32_t) * n, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->succ, succ, sizeof(uint32_t) * n * sls, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->nsucc, nsucc, n, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->fres, fres.data(), sizeof(uint32_t) * n * 160, hipMemcpyHostToDevice));
    c->overlay = OVS_OVERLAY_CHORD;
    c->ideal = false;
    c->sls = sls;
    return OVS_OK;
}

ovs_status ovs_chord_export_fingers(ovs_ctx* c, uint32_t* out)
{
    if (!c || !out) return OVS_EINVAL;
    if (c->overlay != OVS_OVERLAY_CHORD) return fail(c, OVS_ESTATE, "no Chord network loaded");
    if (c->ideal && (c->shard_lo != 0 || c->shard_hi != c->n)) return fail(c, OVS_ESTATE, "sharded ring");
    HIPCHK(c, hipSetDevice(c->device));
    const uint64_t tot = c->n * 160;
    if (!c->ideal) {
        HIPCHK(c, hipMemcpy(out, c->fres, sizeof(uint32_t) * tot, hipMemcpyDeviceToHost));
        return OVS_OK;
    }
    uint32_t* d = nullptr;
    HIPCHK(c, hipMalloc(&d, sizeof(uint32_t) * tot));
    HIPCHK(c, launch_chord_export(c->recs, c->fingers, (uint32_t)c->n, d, c->stream));
    HIPCHK(c, hipMemcpyAsync(out, d, sizeof(uint32_t) * tot, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    hipFree(d);
    return OVS_OK;
}

ovs_status ovs_chord_fix_fingers(ovs_ctx* c, const uint32_t* nodes, uint64_t m, ovs_fixfingers_stats* stats)
{
    if (!c || (m && !nodes)) return OVS_EINVAL;
    if (c->overlay != OVS_OVERLAY_CHORD) return fail(c, OVS_ESTATE, "no Chord network loaded");
    if (c->ideal)
        return fail(c, OVS_ESTATE, "fixfingers rounds run on explicit tables (ovs_chord_load_tables); "
                                   "a converged ring is already their fixed point");
    if (c->P.extendedFingerTable)
        return fail(c, OVS_ENOTSUP, "extendedFingerTable: maintenance rounds keep one node per finger");
    const uint64_t n = c->n;
    for (uint64_t j = 0; j < m; ++j)
        if (nodes[j] >= n) return fail(c, OVS_EINVAL, "node index out of range");
    // 1. handleFixFingersTimerExpired (Chord.cc:851-870): trivial fingers removed, lookups for the rest
    std::vector<K160> kk;
    std::vector<uint32_t> src;
    std::vector<uint8_t> pos;
    kk.reserve(m * 32); src.reserve(m * 32); pos.reserve(m * 32);
    c->ch.fix_fingers_plan(nodes, m, &kk, &src, &pos);
    std::vector<ovs_key160> keys(kk.size());
    for (size_t q = 0; q < kk.size(); ++q)
        for (int w = 0; w < 5; ++w) keys[q].w[w] = kk[q].w[w];
    auto upload_rows = [&]() -> ovs_status {
        if (m * 8 >= n) {
            HIPCHK(c, hipMemcpy(c->fres, c->ch.fres.data(), sizeof(uint32_t) * n * 160, hipMemcpyHostToDevice));
        } else {
            for (uint64_t j = 0; j < m; ++j)
                HIPCHK(c, hipMemcpy(c->fres + (uint64_t)nodes[j] * 160, c->ch.fres.data() + (uint64_t)nodes[j] * 160,
                                    sizeof(uint32_t) * 160, hipMemcpyHostToDevice));
        }
        return OVS_OK;
    };
    ovs_status st = upload_rows();
    if (st != OVS_OK) return st;
    // 2. the FixfingersCalls, routed as KBR lookups on the device (sendRouteRpcCall -> sendToKey)
    std::vector<ovs_route_out> out(keys.size());
    st = ovs_route_batch(c, keys.data(), src.data(), keys.size(), out.data(), nullptr, nullptr, 0, nullptr);
    if (st != OVS_OK) return st;
    // 3. handleRpcFixfingersResponse: finger i := the answering (responsible) node
    uint64_t ok = 0, hops = 0;
    std::vector<uint32_t> resp(out.size());
    std::vector<uint8_t> okv(out.size());
    for (size_t q = 0; q < out.size(); ++q) {
        hops += out[q].hops;
        okv[q] = out[q].status == OVS_LOOKUP_OK;
        resp[q] = out[q].responsible;
        ok += okv[q];
    }
    const uint64_t changed = c->ch.fix_fingers_apply(src, pos, resp, okv);
    for (uint64_t j = 0; j < m; ++j) c->ch.resolve_row(nodes[j]);
    st = upload_rows();
    if (st != OVS_OK) return st;
    if (stats) { stats->lookups = keys.size(); stats->ok = ok; stats->changed = changed; stats->hops = hops; }
    return OVS_OK;
}

ovs_status ovs_chord_stabilize(ovs_ctx* c, const uint32_t* nodes, uint64_t m, ovs_stabilize_stats* stats)
{
    if (!c || (m && !nodes)) return OVS_EINVAL;
    if (c->overlay != OVS_OVERLAY_CHORD) return fail(c, OVS_ESTATE, "no Chord network loaded");
    if (c->ideal) return fail(c, OVS_ESTATE, "stabilize rounds run on explicit tables (ovs_chord_load_tables)");
    if (c->P.extendedFingerTable)
        return fail(c, OVS_ENOTSUP, "extendedFingerTable: maintenance rounds keep one node per finger");
    const uint64_t n = c->n;
    const int sls = c->sls;
    for (uint64_t j = 0; j < m; ++j)
        if (nodes[j] >= n) return fail(c, OVS_EINVAL, "node index out of range");
    uint64_t pred_changed = 0, succ_changed = 0, lists_changed = 0;
    std::vector<uint32_t> changed_succ0;
    c->ch.stabilize(nodes, m, &succ_changed, &lists_changed, &pred_changed, &changed_succ0);
    // upload: the lists, the predecessors, and the resolved finger rows whose successor changed
    // (getFinger falls back to the successor, ChordFingerTable.cc:174-193)
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpy(c->pred, c->ch.pred.data(), sizeof(uint32_t) * n, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->succ, c->ch.succ.data(), sizeof(uint32_t) * n * sls, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->nsucc, c->ch.nsucc.data(), n, hipMemcpyHostToDevice));
    if (changed_succ0.size() * 8 >= n) {
        HIPCHK(c, hipMemcpy(c->fres, c->ch.fres.data(), sizeof(uint32_t) * n * 160, hipMemcpyHostToDevice));
    } else {
        for (uint32_t v : changed_succ0)
            HIPCHK(c, hipMemcpy(c->fres + (uint64_t)v * 160, c->ch.fres.data() + (uint64_t)v * 160,
                                sizeof(uint32_t) * 160, hipMemcpyHostToDevice));
    }
    if (stats) {
        stats->nodes = m; stats->succ_changed = succ_changed; stats->lists_changed = lists_changed;
        stats->pred_changed = pred_changed;
    }
    return OVS_OK;
}

ovs_status ovs_chord_export_tables(ovs_ctx* c, uint32_t* pred, uint32_t* succ, uint8_t* nsucc)
{
    if (!c || !pred || !succ || !nsucc) return OVS_EINVAL;
    if (c->overlay != OVS_OVERLAY_CHORD || c->ideal)
        return fail(c, OVS_ESTATE, "explicit Chord tables (ovs_chord_load_tables) needed");
    std::copy(c->ch.pred.begin(), c->ch.pred.end(), pred);
    std::copy(c->ch.succ.begin(), c->ch.succ.end(), succ);
    std::copy(c->ch.nsucc.begin(), c->ch.nsucc.end(), nsucc);
    return OVS_OK;
}

static ovs_status kad_load_arc(ovs_ctx* c, const ovs_key160* ids, uint64_t n, const double* xy, uint64_t lo,
                               uint64_t hi, uint32_t flags)
{
    if (!c || !ids || !xy) return OVS_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    free_tables(c);
    free_kad_shard(c);
    if (c->P.overlay != OVS_OVERLAY_KADEMLIA) return fail(c, OVS_ESTATE, "params.overlay is not Kademlia");
    if (c->P.b != 1 || c->P.bucketType != 0)
        return fail(c, OVS_ENOTSUP, "the snapshot rule builds b = 1 kademlia tables: other b / bucketType through "
                                    "ovs_kad_load_tables_csr");
    if (c->P.k < 1 || c->P.k > KMAX || c->P.s < 1 || 5 * c->P.s > 64)
        return fail(c, OVS_ENOTSUP, "Kademlia k must be 1..16 (two 96 B bucket blocks) and 5*s <= 64");
    if (lo >= hi || hi > n) return fail(c, OVS_EINVAL, "arc [lo, hi) must be a non-empty part of [0, n)");
    ovs_status s = upload_nodes(c, ids, n, xy, flags & OVS_DEVICE_PTRS);
    if (s != OVS_OK) { free_tables(c); return s; }
    hipError_t e = kad_build(c->recs, c->xy, (uint32_t)n, c->P.k, c->P.s, c->P.kadSeed, c->kad, c->stream, (uint32_t)lo,
                             (uint32_t)hi);
    if (e != hipSuccess) { free_tables(c); return hip_fail(c, e, "kademlia table build"); }
    c->overlay = OVS_OVERLAY_KADEMLIA;
    return OVS_OK;
}

ovs_status ovs_kad_load(ovs_ctx* c, const ovs_key160* ids, uint64_t n, const double* xy, uint32_t flags)
{
    return kad_load_arc(c, ids, n, xy, 0, n, flags);
}

ovs_status ovs_kad_load_tables(ovs_ctx* c, const ovs_key160* ids, uint64_t n, const double* xy, const uint32_t* siblings,
                               const uint8_t* bucket_count, const uint32_t* bucket_nodes, uint32_t flags)
{
    if (!c || !ids || !xy || !siblings || !bucket_count || !bucket_nodes) return OVS_EINVAL;
    if (flags & OVS_DEVICE_PTRS) return fail(c, OVS_ENOTSUP, "explicit tables are taken from host memory");
    HIPCHK(c, hipSetDevice(c->device));
    free_tables(c);
    free_kad_shard(c);
    if (c->P.overlay != OVS_OVERLAY_KADEMLIA) return fail(c, OVS_ESTATE, "params.overlay is not Kademlia");
    if (c->P.b != 1 || c->P.bucketType != 0)
        return fail(c, OVS_ENOTSUP, "k-stride tables hold b = 1 kademlia buckets: other b / bucketType through "
                                    "ovs_kad_load_tables_csr");
    if (c->P.k < 1 || c->P.k > KMAX || c->P.s < 1 || 5 * c->P.s > 64)
        return fail(c, OVS_ENOTSUP, "Kademlia k must be 1..16 (two 96 B bucket blocks) and 5*s <= 64");
    ovs_status s = upload_nodes(c, ids, n, xy, false);
    if (s != OVS_OK) { free_tables(c); return s; }
    const uint64_t S5 = 5ull * (uint64_t)c->P.s, k = (uint64_t)c->P.k;
    uint32_t *dsib = nullptr, *dbn = nullptr;
    uint8_t* dbc = nullptr;
    auto release = [&]() { if (dsib) hipFree(dsib); if (dbn) hipFree(dbn); if (dbc) hipFree(dbc); };
    if (hipMalloc(&dsib, sizeof(uint32_t) * n * S5) != hipSuccess || hipMalloc(&dbc, n * 160) != hipSuccess ||
        hipMalloc(&dbn, sizeof(uint32_t) * n * 160 * k) != hipSuccess) {
        release(); free_tables(c);
        return fail(c, OVS_ENOMEM, "explicit Kademlia tables: device allocation failed");
    }
    hipError_t e = hipMemcpy(dsib, siblings, sizeof(uint32_t) * n * S5, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dbc, bucket_count, n * 160, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dbn, bucket_nodes, sizeof(uint32_t) * n * 160 * k, hipMemcpyHostToDevice);
    uint32_t bad_node = 0, bad_code = 0;
    if (e == hipSuccess)
        e = kad_build_explicit(c->recs, c->xy, (uint32_t)n, c->P.k, c->P.s, dsib, dbc, dbn, c->kad, &bad_node, &bad_code,
                               c->stream);
    release();
    if (e == hipErrorInvalidValue && bad_code) {
        static const char* why[] = {"", "sibling index out of range or the node itself", "sibling listed twice",
                                    "bucket holds more than k entries", "bucket member out of range or the node itself",
                                    "bucket member in the wrong bucket (msb(member ^ node) != bucket index)",
                                    "bucket member listed twice", "node is both sibling and bucket member"};
        free_tables(c);
        char m[192];
        std::snprintf(m, sizeof m, "explicit Kademlia tables of node %u: %s", bad_node, bad_code < 8 ? why[bad_code] : "?");
        return fail(c, OVS_EINVAL, m);
    }
    if (e != hipSuccess) { free_tables(c); return hip_fail(c, e, "explicit Kademlia table build"); }
    c->overlay = OVS_OVERLAY_KADEMLIA;
    c->kh.import(reinterpret_cast<const K160*>(ids), n, c->P.k, c->P.s, siblings, bucket_count, bucket_nodes);
    return OVS_OK;
}

// Kademlia::routingBucketSize (Kademlia.cc:384-411); 0 = no maximum (nkademlia)
static int kad_bucket_size_host(const ovs_params& P, int index)
{
    if (P.bucketType == 1) return 0;
    if (P.bucketType == 2) {
        const int extra = P.extraNodesFinalBucket == 0 ? KEYBITS : P.extraNodesFinalBucket;   // 146-148
        const int limit = (int)(std::log((double)extra) / std::log(2.0));
        int offset = limit - (KEYBITS - (index + 1));
        if (offset > 0) {
            offset = 1 << offset;
            if (offset > P.k) return offset;
        }
    }
    return P.k;
}

int32_t ovs_kad_num_buckets(const ovs_params* p)
{
    if (!p || p->b < 1 || p->b > 5) return -1;
    return ((1 << p->b) - 1) * (KEYBITS / p->b);      // Kademlia.cc:176
}

ovs_status ovs_kad_load_tables_csr(ovs_ctx* c, const ovs_key160* ids, uint64_t n, const double* xy,
                                   const uint32_t* siblings, const uint64_t* bucket_off, const uint32_t* bucket_nodes,
                                   uint32_t flags)
{
    if (!c || !ids || !xy || !siblings || !bucket_off) return OVS_EINVAL;
    if (flags & OVS_DEVICE_PTRS) return fail(c, OVS_ENOTSUP, "explicit tables are taken from host memory");
    HIPCHK(c, hipSetDevice(c->device));
    free_tables(c);
    free_kad_shard(c);
    const ovs_params& P = c->P;
    if (P.overlay != OVS_OVERLAY_KADEMLIA) return fail(c, OVS_ESTATE, "params.overlay is not Kademlia");
    if (P.b < 1 || P.b > 5) return fail(c, OVS_ENOTSUP, "Kademlia b must be 1..5 (numBuckets <= 992)");
    if (P.bucketType < 0 || P.bucketType > 2) return fail(c, OVS_EINVAL, "bucketType must be 0..2 (kademlia, nkademlia, nr128)");
    // routingBucketSize counts indices as if b = 1 (Kademlia.cc:400-406): for b > 1 the indices past
    // 159 get sizes 2^8 .. 2^30 and then (int)pow(2, >= 31) -- undefined, not followed
    if (P.bucketType == 2 && P.b != 1) return fail(c, OVS_ENOTSUP, "nr128 buckets need b = 1");
    if (P.bucketType == 2 && (P.extraNodesFinalBucket < 0 || P.extraNodesFinalBucket > 511))
        return fail(c, OVS_ENOTSUP, "nr128: extraNodesFinalBucket must be 0..511");
    if (P.k < 1 || P.k > KMAX || P.s < 1 || 5 * P.s > 64)
        return fail(c, OVS_ENOTSUP, "Kademlia k must be 1..16 and 5*s <= 64");
    if (n == 0 || n >= 0xFFFFFFFFull) return fail(c, OVS_EINVAL, "network size out of range");
    const int nb = ovs_kad_num_buckets(&P);
    const uint64_t dir = n * (uint64_t)nb;
    if (bucket_off[0] != 0) return fail(c, OVS_EINVAL, "bucket_off[0] must be 0");
    for (uint64_t j = 0; j < dir; ++j)
        if (bucket_off[j + 1] < bucket_off[j]) return fail(c, OVS_EINVAL, "bucket_off must not decrease");
    const uint64_t total = bucket_off[dir];
    if (total >= 0xFFFFFFFFull) return fail(c, OVS_ENOTSUP, "more than 2^32 - 1 bucket members");
    if (total && !bucket_nodes) return fail(c, OVS_EINVAL, "bucket_nodes is NULL");
    ovs_status s = upload_nodes(c, ids, n, xy, false);
    if (s != OVS_OK) { free_tables(c); return s; }
    const uint64_t S5 = 5ull * (uint64_t)P.s;
    std::vector<uint32_t> off32(dir + 1);
    for (uint64_t j = 0; j <= dir; ++j) off32[j] = (uint32_t)bucket_off[j];
    std::vector<int> caps(nb);
    for (int m = 0; m < nb; ++m) caps[m] = kad_bucket_size_host(P, m);
    DevBufs d;
    uint32_t *dsib = nullptr, *doff = nullptr, *dmem = nullptr;
    if (d.get(&dsib, n * S5) != hipSuccess || d.get(&doff, dir + 1) != hipSuccess || d.get(&dmem, total) != hipSuccess) {
        free_tables(c);
        return fail(c, OVS_ENOMEM, "CSR Kademlia tables: device allocation failed");
    }
    hipError_t e = hipMemcpy(dsib, siblings, sizeof(uint32_t) * n * S5, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(doff, off32.data(), sizeof(uint32_t) * (dir + 1), hipMemcpyHostToDevice);
    if (e == hipSuccess && total) e = hipMemcpy(dmem, bucket_nodes, sizeof(uint32_t) * total, hipMemcpyHostToDevice);
    uint32_t bad_node = 0, bad_code = 0;
    if (e == hipSuccess)
        e = kad_build_general(c->recs, c->xy, (uint32_t)n, P.k, P.s, P.b, caps.data(), dsib, doff, dmem, total, c->kad,
                              &bad_node, &bad_code, c->stream);
    if (e == hipErrorInvalidValue && bad_code) {
        static const char* why[] = {"", "sibling index out of range or the node itself", "sibling listed twice",
                                    "bucket holds more than routingBucketSize(i) entries",
                                    "bucket member out of range or the node itself",
                                    "bucket member in the wrong bucket (routingBucketIndex(member) != bucket index)",
                                    "bucket member listed twice", "node is both sibling and bucket member"};
        free_tables(c);
        char m[192];
        std::snprintf(m, sizeof m, "CSR Kademlia tables of node %u: %s", bad_node, bad_code < 8 ? why[bad_code] : "?");
        return fail(c, OVS_EINVAL, m);
    }
    if (e != hipSuccess) { free_tables(c); return hip_fail(c, e, "CSR Kademlia table build"); }
    c->overlay = OVS_OVERLAY_KADEMLIA;
    return OVS_OK;
}

ovs_status ovs_kad_export_csr(ovs_ctx* c, uint32_t* siblings, uint64_t* bucket_off, uint32_t* bucket_nodes, uint64_t cap,
                              uint64_t* total)
{
    if (!c || !siblings || !bucket_off || !total || (cap && !bucket_nodes)) return OVS_EINVAL;
    if (c->overlay != OVS_OVERLAY_KADEMLIA) return fail(c, OVS_ESTATE, "no Kademlia network loaded");
    if (c->kad.lo != 0 || c->kad.hi != c->n) return fail(c, OVS_ESTATE, "export needs the whole network");
    HIPCHK(c, hipSetDevice(c->device));
    const uint64_t n = c->n, S5 = 5ull * (uint64_t)c->P.s;
    const KadTables& t = c->kad;
    if (t.general) {
        const uint64_t dir = n * (uint64_t)t.nb;
        std::vector<uint32_t> off32(dir + 1);
        HIPCHK(c, hipMemcpyAsync(siblings, t.sib, sizeof(uint32_t) * n * S5, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipMemcpyAsync(off32.data(), t.goff, sizeof(uint32_t) * (dir + 1), hipMemcpyDeviceToHost, c->stream));
        const uint64_t ncopy = std::min<uint64_t>(cap, t.gtotal);
        if (ncopy)
            HIPCHK(c, hipMemcpyAsync(bucket_nodes, t.gidx, sizeof(uint32_t) * ncopy, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        for (uint64_t j = 0; j <= dir; ++j) bucket_off[j] = off32[j];
        *total = t.gtotal;
        return OVS_OK;
    }
    // the 160-bucket tables, converted
    const uint64_t k = (uint64_t)t.k;
    std::vector<uint8_t> bc(n * KEYBITS);
    std::vector<uint32_t> bn(n * KEYBITS * k);
    hipError_t e = kad_export(t, (uint32_t)n, siblings, bc.data(), bn.data(), c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "kademlia export");
    uint64_t w = 0;
    bucket_off[0] = 0;
    for (uint64_t j = 0; j < n * KEYBITS; ++j) {
        for (uint64_t q = 0; q < bc[j]; ++q, ++w)
            if (w < cap) bucket_nodes[w] = bn[j * k + q];
        bucket_off[j + 1] = w;
    }
    *total = w;
    return OVS_OK;
}

ovs_status ovs_kad_load_shard(ovs_ctx* c, const ovs_key160* ids, uint64_t n, const double* xy, uint64_t lo,
                              uint64_t hi, uint32_t flags)
{
    return kad_load_arc(c, ids, n, xy, lo, hi, flags);
}

namespace {

ovs_status kad_shard_begin_impl(ovs_ctx* c, int32_t lk_ns, uint32_t* sib, const ovs_key160* keys, const uint32_t* src,
                                uint64_t n, uint32_t qid_base, void* stream)
{
    if (!c || (n && (!keys || !src))) return OVS_EINVAL;
    if (c->overlay != OVS_OVERLAY_KADEMLIA) return fail(c, OVS_ESTATE, "no Kademlia network loaded");
    ovs_params P = c->P;
    if (lk_ns >= 0) P.numSiblings = 1;     // the route checks; numSiblings is the LookupCall's
    ovs_status st = check_common(c, P);
    if (st != OVS_OK) return st;
    if (P.routingType != 0) return fail(c, OVS_ENOTSUP, "Kademlia routing is implemented for routingType = iterative");
    if (lk_ns >= 0) P.numSiblings = lk_ns;
    if (!kad_params_supported_host(P, c->kad) || (lk_ns < 0 && P.numSiblings != 1))
        return fail(c, OVS_ENOTSUP, "lookup configuration not implemented");
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    const int alpha = c->P.lookupParallelRpcs;
    const int fcap = kad_shard_cap(P, c->kad);
    if (n > c->kcap || alpha != c->kalpha || fcap != c->kfcap) {
        free_kad_shard(c);
        const uint64_t cap = n ? n : 1;
        HIPCHK(c, hipMalloc(&c->kst, kad_lookup_state_bytes(alpha, fcap) * cap));
        HIPCHK(c, hipMalloc(&c->kact, cap));
        HIPCHK(c, hipMalloc(&c->kkeys, sizeof(K160) * cap));
        HIPCHK(c, hipMalloc(&c->ksrc, sizeof(uint32_t) * cap));
        HIPCHK(c, hipMalloc(&c->kqids, sizeof(uint32_t) * cap));
        HIPCHK(c, hipMalloc(&c->kres, (fcap > 8 ? sizeof(KadResN<16>) : sizeof(KadResN<8>)) * cap * kad_pend_slots(alpha)));
        HIPCHK(c, hipMalloc(&c->kbad, sizeof(unsigned long long)));
        HIPCHK(c, hipMalloc(&c->kiota, sizeof(uint64_t) * cap));
        HIPCHK(c, hipMalloc(&c->klist[0], sizeof(uint64_t) * cap));
        HIPCHK(c, hipMalloc(&c->klist[1], sizeof(uint64_t) * cap));
        HIPCHK(c, hipMalloc(&c->knl, sizeof(unsigned long long) * 3));
        c->kcap = cap;
        c->kalpha = alpha;
        c->kfcap = fcap;
    }
    c->knlook = n;
    c->kns = lk_ns;
    c->ksib = sib;
    HIPCHK(c, hipMemsetAsync(c->kbad, 0, sizeof(unsigned long long), s));
    c->kcur = 0;
    HIPCHK(c, kad_shard_init(reinterpret_cast<const K160*>(keys), src, n, qid_base, c->kkeys, c->ksrc, c->kact,
                             c->kqids, c->kiota, c->knl, c->kad.lo, c->kad.hi, c->kbad, s));
    return OVS_OK;
}

}  // namespace

ovs_status ovs_kad_shard_begin(ovs_ctx* c, const ovs_key160* keys, const uint32_t* src, uint64_t n, uint32_t qid_base,
                               void* stream)
{
    return kad_shard_begin_impl(c, -1, nullptr, keys, src, n, qid_base, stream);
}

ovs_status ovs_kad_shard_begin_lookup(ovs_ctx* c, int32_t num_siblings, const ovs_key160* keys, const uint32_t* src,
                                      uint64_t n, uint32_t qid_base, uint32_t* siblings, void* stream)
{
    if (!c || (n && !siblings)) return OVS_EINVAL;
    if (c->overlay != OVS_OVERLAY_KADEMLIA) return fail(c, OVS_ESTATE, "no Kademlia network loaded");
    // BaseOverlay::lookupRpc: numSiblings < 0 -> getMaxNumSiblings() = s (Kademlia.cc:347-350)
    const int32_t ns = num_siblings < 0 ? c->P.s : num_siblings;
    if (ns > c->P.s) return fail(c, OVS_EINVAL, "numSiblings too big!");
    if (ns > 8) return fail(c, OVS_ENOTSUP, "LookupCall implements numSiblings <= 8");
    return kad_shard_begin_impl(c, ns, siblings, keys, src, n, qid_base, stream);
}

ovs_status ovs_kad_shard_step(ovs_ctx* c, ovs_kad_req* out, uint64_t out_cap, unsigned long long* out_count,
                              ovs_done_rec* done, uint64_t done_cap, unsigned long long* done_count,
                              unsigned long long* active_count, const uint64_t* shard_lo, uint32_t nshards, void* stream)
{
    if (!c || !shard_lo || nshards == 0 || nshards > (uint32_t)MAXSHARDS) return OVS_EINVAL;
    if (!out || !out_count || !done || !done_count || !active_count) return OVS_EINVAL;
    if (c->overlay != OVS_OVERLAY_KADEMLIA) return fail(c, OVS_ESTATE, "no Kademlia network loaded");
    if (!c->kst) return fail(c, OVS_ESTATE, "no lookups started (ovs_kad_shard_begin)");
    if (c->P.lookupParallelRpcs != c->kalpha && c->knlook)
        return fail(c, OVS_ESTATE, "lookupParallelRpcs changed since ovs_kad_shard_begin");
    if (kad_shard_cap(c->P, c->kad) != c->kfcap && c->knlook)
        return fail(c, OVS_ESTATE, "lookupRedundantNodes / k changed the findNode capacity since ovs_kad_shard_begin");
    if (out_cap < c->knlook * (uint64_t)kad_pend_slots(c->kalpha))
        return fail(c, OVS_EINVAL, "out_cap must hold a request per pending-call slot "
                                   "(n * lookupParallelRpcs; n * 8 for lookupParallelRpcs 5..8)");
    uint64_t lo_h[MAXSHARDS + 1];
    for (uint32_t r = 0; r <= nshards; ++r) {
        lo_h[r] = shard_lo[r];
        if (r > 0 && shard_lo[r] < shard_lo[r - 1]) return fail(c, OVS_EINVAL, "shard_lo must be non-decreasing");
    }
    if (shard_lo[0] != 0 || shard_lo[nshards] != c->n) return fail(c, OVS_EINVAL, "shard_lo must cover [0, n)");
    bool mine = false;
    for (uint32_t r = 0; r < nshards; ++r) mine |= shard_lo[r] == c->kad.lo && shard_lo[r + 1] == c->kad.hi;
    if (!mine) return fail(c, OVS_EINVAL, "this context's arc is not one of shard_lo's arcs");
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    ovs_status bst = upload_bounds(c, lo_h, nshards);
    if (bst != OVS_OK) return bst;
    // this round's list: iota in round 1, then the ping-pong lists the previous round compacted
    const int cur = c->kcur, nxt = cur == 1 ? 2 : 1;
    const uint64_t* list = cur == 0 ? c->kiota : c->klist[cur - 1];
    hipError_t e = kad_shard_step(c->kad, c->xy, (uint32_t)c->n, c->P, delay_consts(c->P), c->kst, c->kact, c->kkeys,
                                  c->ksrc, c->kqids,
                                  c->kres, c->knlook, list, c->knl + cur, c->kiota, c->klist[nxt - 1], c->knl + nxt,
                                  c->d_bounds, (int)nshards, out, out_cap, out_count, done, done_cap, done_count,
                                  active_count, c->kns, c->ksib, c->kbad, c->num_cu, c->stage[s], s);
    if (e != hipSuccess) return hip_fail(c, e, "kademlia shard step");
    c->kcur = nxt;
    return OVS_OK;
}

int32_t ovs_kad_shard_resp_bytes(const ovs_ctx* c)
{
    if (!c || c->overlay != OVS_OVERLAY_KADEMLIA) return -1;
    return kad_shard_cap(c->P, c->kad) > 8 ? (int32_t)sizeof(ovs_kad_resp16) : (int32_t)sizeof(ovs_kad_resp);
}

ovs_status ovs_kad_shard_serve(ovs_ctx* c, const ovs_kad_req* in, uint64_t n, void* out, void* stream)
{
    if (!c || (n && (!in || !out))) return OVS_EINVAL;
    if (c->overlay != OVS_OVERLAY_KADEMLIA) return fail(c, OVS_ESTATE, "no Kademlia network loaded");
    if (c->kst && c->knlook && kad_shard_cap(c->P, c->kad) != c->kfcap)
        return fail(c, OVS_ESTATE, "lookupRedundantNodes / k changed the findNode capacity since ovs_kad_shard_begin");
    HIPCHK(c, hipSetDevice(c->device));
    hipError_t e = kad_shard_serve(c->kad, (uint32_t)c->n, c->P, in, n, out, c->kbad, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(c, e, "kademlia shard serve");
    return OVS_OK;
}

ovs_status ovs_kad_shard_deliver(ovs_ctx* c, const void* in, uint64_t n, void* stream)
{
    if (!c || (n && !in)) return OVS_EINVAL;
    if (!c->kres) return fail(c, OVS_ESTATE, "no lookups started (ovs_kad_shard_begin)");
    if (c->overlay != OVS_OVERLAY_KADEMLIA) return fail(c, OVS_ESTATE, "no Kademlia network loaded");
    if (c->knlook && kad_shard_cap(c->P, c->kad) != c->kfcap)
        return fail(c, OVS_ESTATE, "lookupRedundantNodes / k changed the findNode capacity since ovs_kad_shard_begin");
    HIPCHK(c, hipSetDevice(c->device));
    hipError_t e = kad_shard_deliver(c->kfcap, in, n, c->kres, c->knlook * (uint64_t)kad_pend_slots(c->kalpha), c->kbad,
                                     (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(c, e, "kademlia shard deliver");
    return OVS_OK;
}

ovs_status ovs_kad_shard_replicate(ovs_ctx* c, int32_t top_levels)
{
    if (!c) return OVS_EINVAL;
    if (c->overlay != OVS_OVERLAY_KADEMLIA || !c->kad.snapshot || c->kad.general)
        return fail(c, OVS_ESTATE, "no Kademlia snapshot network (ovs_kad_load_shard) loaded");
    if (top_levels < 0 || top_levels > KTOP_MAX) return fail(c, OVS_EINVAL, "top_levels must be 0..7");
    if (c->kad.tl == top_levels) return OVS_OK;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipDeviceSynchronize());      // kernels of earlier rounds may still read the tables
    const uint32_t lo = c->kad.lo, hi = c->kad.hi;
    hipError_t e = kad_build(c->recs, c->xy, (uint32_t)c->n, c->P.k, c->P.s, c->P.kadSeed, c->kad, c->stream, lo, hi,
                             top_levels);
    if (e != hipSuccess) { free_tables(c); return hip_fail(c, e, "kademlia table rebuild (replicated top buckets)"); }
    return OVS_OK;
}

int32_t ovs_kad_shard_levels(const ovs_ctx* c)
{
    return c && c->overlay == OVS_OVERLAY_KADEMLIA ? c->kad.tl : 0;
}

int32_t ovs_kad_shard_rec_bytes(const ovs_ctx* c)
{
    if (!c || c->overlay != OVS_OVERLAY_KADEMLIA) return -1;
    return (int32_t)kad_rec_bytes(c->P.lookupParallelRpcs);
}


ovs_status ovs_kad_shard_mig_step(ovs_ctx* c, const void* in, uint64_t n_in, const ovs_key160* fkeys, const uint32_t* fsrc,
                                  uint32_t fqid, void* out, uint64_t out_cap, unsigned long long* out_count,
                                  ovs_done_rec* done, uint64_t done_cap, unsigned long long* done_count,
                                  const uint64_t* shard_lo, uint32_t nshards, void* stream)
{
    // a batch's first round (in == NULL) starts the error count afresh
    return ovs::kad_mig_step_impl(c, in, n_in, fkeys, fsrc, fqid, out, out_cap, out_count, done, done_cap, done_count,
                                  shard_lo, nshards, stream, in == nullptr);
}

extern "C++" {
ovs_status ovs::kad_shard_reset_errors(ovs_ctx* c, void* stream)
{
    HIPCHK(c, hipSetDevice(c->device));
    if (!c->kbad) HIPCHK(c, hipMalloc(&c->kbad, sizeof(unsigned long long)));
    HIPCHK(c, hipMemsetAsync(c->kbad, 0, sizeof(unsigned long long), (hipStream_t)stream));
    return OVS_OK;
}

ovs_status ovs::kad_mig_step_impl(ovs_ctx* c, const void* in, uint64_t n_in, const ovs_key160* fkeys,
                                  const uint32_t* fsrc, uint32_t fqid, void* out, uint64_t out_cap,
                                  unsigned long long* out_count, ovs_done_rec* done, uint64_t done_cap,
                                  unsigned long long* done_count, const uint64_t* shard_lo, uint32_t nshards,
                                  void* stream, bool reset_errors)
{
    if (!c || !shard_lo || nshards == 0 || nshards > (uint32_t)MAXSHARDS) return OVS_EINVAL;
    if (n_in && ((!in && !(fkeys && fsrc)) || !out || !out_count || !done || !done_count)) return OVS_EINVAL;
    if (c->overlay != OVS_OVERLAY_KADEMLIA) return fail(c, OVS_ESTATE, "no Kademlia network loaded");
    ovs_status st = check_common(c, c->P);
    if (st != OVS_OK) return st;
    if (!kad_mig_supported(c->P, c->kad))
        return fail(c, OVS_ENOTSUP, "the migration step implements one-way iterative KBR routes on snapshot tables with "
                                    "k and lookupRedundantNodes <= 8");
    uint64_t lo_h[MAXSHARDS + 1];
    int me = -1;
    for (uint32_t r = 0; r <= nshards; ++r) {
        lo_h[r] = shard_lo[r];
        if (r > 0 && shard_lo[r] < shard_lo[r - 1]) return fail(c, OVS_EINVAL, "shard_lo must be non-decreasing");
    }
    if (shard_lo[0] != 0 || shard_lo[nshards] != c->n) return fail(c, OVS_EINVAL, "shard_lo must cover [0, n)");
    for (uint32_t r = 0; r < nshards; ++r)
        if (shard_lo[r] == c->kad.lo && shard_lo[r + 1] == c->kad.hi) me = (int)r;
    if (me < 0) return fail(c, OVS_EINVAL, "this context's arc is not one of shard_lo's arcs");
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    ovs_status bst = upload_bounds(c, lo_h, nshards);
    if (bst != OVS_OK) return bst;
    if (!c->kbad) {
        HIPCHK(c, hipMalloc(&c->kbad, sizeof(unsigned long long)));
        HIPCHK(c, hipMemsetAsync(c->kbad, 0, sizeof(unsigned long long), s));
    }
    if (reset_errors) HIPCHK(c, hipMemsetAsync(c->kbad, 0, sizeof(unsigned long long), s));
    int slot = -1;
    unsigned long long* dyn = dyn_acquire(c, n_in, s, &slot);
    hipError_t e = kad_mig_step(c->kad, c->xy, (uint32_t)c->n, c->P, delay_consts(c->P), in, n_in,
                                reinterpret_cast<const K160*>(fkeys), fsrc, fqid, c->d_bounds, (int)nshards, me, out,
                                out_cap, out_count, done, done_cap, done_count, c->kbad, c->num_cu, c->stage[s], s, dyn);
    dyn_release(c, s, slot);
    if (e != hipSuccess) return hip_fail(c, e, "kademlia migration step");
    return OVS_OK;
}
}  // extern "C++"

ovs_status ovs_kad_shard_errors(ovs_ctx* c, uint64_t* bad)
{
    if (!c || !bad) return OVS_EINVAL;
    *bad = 0;
    if (!c->kbad) return OVS_OK;
    HIPCHK(c, hipSetDevice(c->device));
    unsigned long long h = 0;
    HIPCHK(c, hipDeviceSynchronize());
    HIPCHK(c, hipMemcpy(&h, c->kbad, sizeof h, hipMemcpyDeviceToHost));
    *bad = h;
    return OVS_OK;
}

ovs_status ovs_kad_export(ovs_ctx* c, uint32_t* siblings, uint8_t* bucket_count, uint32_t* bucket_nodes)
{
    if (!c || !siblings || !bucket_count || !bucket_nodes) return OVS_EINVAL;
    if (c->overlay != OVS_OVERLAY_KADEMLIA) return fail(c, OVS_ESTATE, "no Kademlia network loaded");
    if (c->kad.lo != 0 || c->kad.hi != c->n) return fail(c, OVS_ESTATE, "export needs the whole network");
    if (c->kad.general) return fail(c, OVS_ENOTSUP, "CSR tables: ovs_kad_export_csr");
    HIPCHK(c, hipSetDevice(c->device));
    hipError_t e = kad_export(c->kad, (uint32_t)c->n, siblings, bucket_count, bucket_nodes, c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "kademlia export");
    return OVS_OK;
}

ovs_status ovs_koorde_load(ovs_ctx* c, const ovs_key160* ids, uint64_t n, const double* xy, uint32_t flags)
{
    if (!c || !ids || !xy) return OVS_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    free_tables(c);
    free_kad_shard(c);
    if (c->P.overlay != OVS_OVERLAY_KOORDE) return fail(c, OVS_ESTATE, "params.overlay is not Koorde");
    if (n < 2) return fail(c, OVS_EINVAL, "Koorde needs at least 2 nodes");
    if (c->P.successorListSize < 1) return fail(c, OVS_EINVAL, "successorListSize must be >= 1");
    if (c->P.shiftingBits < 1 || c->P.shiftingBits > 16 || c->P.deBruijnListSize < 1 || c->P.deBruijnListSize > 255)
        return fail(c, OVS_ENOTSUP, "Koorde shiftingBits must be 1..16 and deBruijnListSize 1..255");
    ovs_status s = upload_nodes(c, ids, n, xy, flags & OVS_DEVICE_PTRS);
    if (s != OVS_OK) { free_tables(c); return s; }
    hipError_t e = koorde_build(c->recs, c->xy, (uint32_t)n, c->P.successorListSize, c->P.shiftingBits, c->P.deBruijnListSize,
                                c->P.useOtherLookup, c->P.useSucList, c->koorde, c->stream);
    if (e != hipSuccess) { free_tables(c); return hip_fail(c, e, "koorde build"); }
    c->overlay = OVS_OVERLAY_KOORDE;
    return OVS_OK;
}

ovs_status ovs_koorde_export(ovs_ctx* c, uint32_t* db_node, uint32_t* db_start, uint8_t* db_num)
{
    if (!c || !db_node || !db_start || !db_num) return OVS_EINVAL;
    if (c->overlay != OVS_OVERLAY_KOORDE) return fail(c, OVS_ESTATE, "no Koorde network loaded");
    HIPCHK(c, hipSetDevice(c->device));
    std::vector<KoordeNode> h(c->n);
    HIPCHK(c, hipMemcpyAsync(h.data(), c->koorde.nd, sizeof(KoordeNode) * c->n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (uint64_t i = 0; i < c->n; ++i) {
        db_node[i] = h[i].db; db_start[i] = h[i].dbStart; db_num[i] = (uint8_t)h[i].dbNum;
    }
    return OVS_OK;
}

ovs_status ovs_koorde_find_node_batch(ovs_ctx* c, const uint32_t* node, const ovs_key160* keys, ovs_koorde_ext* ext,
                                      uint32_t* next, uint64_t n)
{
    static_assert(sizeof(ovs_koorde_ext) == sizeof(KExt), "ovs_koorde_ext mirrors KExt");
    if (!c || (n && (!node || !keys || !ext || !next))) return OVS_EINVAL;
    if (c->overlay != OVS_OVERLAY_KOORDE) return fail(c, OVS_ESTATE, "no Koorde network loaded");
    if (n == 0) return OVS_OK;
    HIPCHK(c, hipSetDevice(c->device));
    for (uint64_t i = 0; i < n; ++i)
        if (node[i] >= c->n) return fail(c, OVS_EINVAL, "node index out of range");
    uint32_t *dn = nullptr, *dnext = nullptr;
    K160* dk = nullptr;
    KExt* de = nullptr;
    bool o1, o2;
    ovs_status st = to_device(c, node, n, false, &dn, &o1);
    if (st != OVS_OK) return st;
    st = to_device(c, reinterpret_cast<const K160*>(keys), n, false, &dk, &o2);
    if (st != OVS_OK) { hipFree(dn); return st; }
    HIPCHK(c, hipMalloc(&de, sizeof(KExt) * n));
    HIPCHK(c, hipMalloc(&dnext, sizeof(uint32_t) * n));
    HIPCHK(c, hipMemcpyAsync(de, ext, sizeof(KExt) * n, hipMemcpyHostToDevice, c->stream));
    hipError_t e = koorde_find_node(c->koorde, c->recs, dn, dk, de, dnext, n, c->stream);
    if (e != hipSuccess) return hip_fail(c, e, "koorde findNode kernel");
    HIPCHK(c, hipMemcpyAsync(ext, de, sizeof(KExt) * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(next, dnext, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    hipFree(dn); hipFree(dk); hipFree(de); hipFree(dnext);
    return OVS_OK;
}

ovs_status ovs_epichord_load(ovs_ctx* c, const ovs_key160* ids, uint64_t n, const double* xy, const uint32_t* succ,
                             const uint8_t* nsucc, const uint32_t* pred, const uint8_t* npred, const uint8_t* lists_full,
                             const uint64_t* cache_off, const uint32_t* cache_node, const int64_t* cache_last_ns,
                             const int64_t* cache_ttl_ns, uint32_t flags)
{
    if (!c || !ids || !xy || !succ || !nsucc || !pred || !npred || !lists_full || !cache_off) return OVS_EINVAL;
    if (flags & OVS_DEVICE_PTRS) return fail(c, OVS_ENOTSUP, "ovs_epichord_load takes host buffers");
    HIPCHK(c, hipSetDevice(c->device));
    free_tables(c);
    free_kad_shard(c);
    if (c->P.overlay != OVS_OVERLAY_EPICHORD) return fail(c, OVS_ESTATE, "params.overlay is not EpiChord");
    const int L = c->P.successorListSize;
    if (L < 1 || L > EPI_MAXL) return fail(c, OVS_ENOTSUP, "EpiChord successorListSize must be 1..16");
    if (!(c->P.cacheTTL >= 0)) return fail(c, OVS_EINVAL, "cacheTTL must be >= 0");
    if (n < 2 || n >= 0xFFFFFFFFull) return fail(c, OVS_EINVAL, "node count out of range");
    std::vector<uint32_t> meta, cn;
    std::vector<int64_t> cl, ct;
    std::string err;
    if (!epichord_prepare(reinterpret_cast<const K160*>(ids), n, L, succ, nsucc, pred, npred, lists_full, cache_off,
                          cache_node, cache_last_ns, cache_ttl_ns, &meta, &cn, &cl, &ct, &err))
        return fail(c, OVS_EINVAL, err);
    const uint64_t E = cache_off[n];
    ovs_status st = upload_nodes(c, ids, n, xy, false);
    if (st != OVS_OK) { free_tables(c); return st; }
    EpiTables& T = c->epi;
    T.n = (uint32_t)n;
    T.L = L;
    T.nent = E;
    auto up = [&](auto** d, const auto* h, uint64_t cnt) -> hipError_t {
        using TT = std::remove_pointer_t<std::remove_reference_t<decltype(*d)>>;
        hipError_t e = hipMalloc((void**)d, sizeof(TT) * (cnt ? cnt : 1));
        if (e == hipSuccess && cnt) e = hipMemcpyAsync(*d, h, sizeof(TT) * cnt, hipMemcpyHostToDevice, c->stream);
        return e;
    };
    hipError_t e = up(&T.succ, succ, n * L);
    if (e == hipSuccess) e = up(&T.pred, pred, n * L);
    if (e == hipSuccess) e = up(&T.meta, meta.data(), n);
    if (e == hipSuccess) e = up(&T.coff, cache_off, n + 1);
    if (e == hipSuccess) e = up(&T.cnode, cn.data(), E);
    if (e == hipSuccess) e = up(&T.clast, cl.data(), E);
    if (e == hipSuccess) e = up(&T.cttl, ct.data(), E);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) { free_tables(c); return hip_fail(c, e, "EpiChord snapshot upload"); }
    c->overlay = OVS_OVERLAY_EPICHORD;
    return OVS_OK;
}

ovs_status ovs_epichord_find_node_batch(ovs_ctx* c, const uint32_t* node, const ovs_key160* keys, const uint32_t* src,
                                        const int64_t* now_ns, uint64_t n, int32_t numRedundantNodes,
                                        uint32_t* out_nodes, int64_t* out_last_ns, uint32_t max_out, uint8_t* out_count,
                                        uint8_t* out_status, uint32_t flags, void* stream)
{
    if (!c || (n && (!node || !keys || !src || !now_ns || !out_nodes || !out_last_ns || !out_count || !out_status)))
        return OVS_EINVAL;
    if (c->overlay != OVS_OVERLAY_EPICHORD) return fail(c, OVS_ESTATE, "no EpiChord snapshot loaded");
    if (numRedundantNodes < 0 || numRedundantNodes > EPI_MAXR)
        return fail(c, OVS_EINVAL, "numRedundantNodes must be 0..32");
    if (max_out < 3 || max_out < (uint32_t)(1 + numRedundantNodes))
        return fail(c, OVS_EINVAL, "max_out must be >= max(3, 1 + numRedundantNodes)");
    HIPCHK(c, hipSetDevice(c->device));
    const bool dev = flags & OVS_DEVICE_PTRS;
    hipStream_t s = dev ? (hipStream_t)stream : c->stream;
    if (n == 0) return OVS_OK;
    if (!dev) {
        for (uint64_t i = 0; i < n; ++i)
            if (node[i] >= c->n || (src[i] != NONE && src[i] >= c->n))
                return fail(c, OVS_EINVAL, "node / source index out of range");
    }
    uint32_t *dn = nullptr, *dsrc = nullptr, *dout = nullptr;
    K160* dk = nullptr;
    int64_t *dnow = nullptr, *dlast = nullptr;
    uint8_t *dc = nullptr, *dst = nullptr;
    bool o1 = false, o2 = false, o3 = false, o4 = false;
    DevBufs own;          // the temporaries of a host-buffer call, freed on every path
    ovs_status st = to_device(c, node, n, dev, &dn, &o1);
    own.own(dn, o1);
    if (st == OVS_OK) { st = to_device(c, reinterpret_cast<const K160*>(keys), n, dev, &dk, &o2); own.own(dk, o2); }
    if (st == OVS_OK) { st = to_device(c, src, n, dev, &dsrc, &o3); own.own(dsrc, o3); }
    if (st == OVS_OK) { st = to_device(c, now_ns, n, dev, &dnow, &o4); own.own(dnow, o4); }
    if (st != OVS_OK) return st;
    if (!dev) {
        HIPCHK(c, own.get(&dout, n * max_out));
        HIPCHK(c, own.get(&dlast, n * max_out));
        HIPCHK(c, own.get(&dc, n));
        HIPCHK(c, own.get(&dst, n));
    } else {
        dout = out_nodes; dlast = out_last_ns; dc = out_count; dst = out_status;
    }
    const int64_t ttl = simtime_host(c->P.cacheTTL, c->P.simtimeRound);
    hipError_t e = epichord_find_node(c->epi, c->recs, dn, dk, dsrc, dnow, n, numRedundantNodes, ttl, dout, dlast,
                                      max_out, dc, dst, s);
    if (e != hipSuccess) return hip_fail(c, e, "EpiChord findNode kernel");
    if (!dev) {
        HIPCHK(c, hipMemcpyAsync(out_nodes, dout, sizeof(uint32_t) * n * max_out, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(out_last_ns, dlast, sizeof(int64_t) * n * max_out, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(out_count, dc, n, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(out_status, dst, n, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
    }
    return OVS_OK;
}

// host-pointer calls: every lookup's source must be a node of the network (a source past it would
// be read out of bounds by the lookup kernels); device-pointer calls leave that to the caller (ovs_kbr.h)
static ovs_status check_sources(ovs_ctx* c, const uint32_t* src, uint64_t n, bool dev)
{
    if (dev) return OVS_OK;
    for (uint64_t i = 0; i < n; ++i)
        if (src[i] >= c->n) return fail(c, OVS_EINVAL, "source index out of range (lookup " + std::to_string(i) + ")");
    return OVS_OK;
}

ovs_status ovs_route_batch(ovs_ctx* c, const ovs_key160* keys, const uint32_t* src, uint64_t n,
                           ovs_route_out* out, uint32_t* hop_seq, uint32_t* rpcs, uint32_t flags, void* stream)
{
    if (!c || (!keys && n) || (!src && n) || (!out && n)) return OVS_EINVAL;
    if (!c->overlay) return fail(c, OVS_ESTATE, "no network loaded");
    if (c->overlay == OVS_OVERLAY_EPICHORD)
        return fail(c, OVS_ENOTSUP, "EpiChord lookups rewrite the caches they route over (DESIGN.md §9): "
                                    "ovs_epichord_find_node_batch only");
    ovs_status st = check_common(c, c->P);
    if (st != OVS_OK) return st;
    HIPCHK(c, hipSetDevice(c->device));
    const bool dev = flags & OVS_DEVICE_PTRS;
    hipStream_t s = dev ? (hipStream_t)stream : c->stream;   // NULL = the default stream
    const int H = c->P.hopCountMax > 0 ? c->P.hopCountMax : 1;
    if (c->overlay == OVS_OVERLAY_CHORD) {
        st = check_chord_route(c, c->P);
        if (st != OVS_OK) return st;
        if (c->ideal && (c->shard_lo != 0 || c->shard_hi != c->n))
            return fail(c, OVS_ESTATE, "context holds one arc of a sharded ring: use ovs_shard_step");
        st = ensure_nodes(c, s);
        if (st != OVS_OK) return st;
    } else if (c->overlay == OVS_OVERLAY_KOORDE) {
        if (c->P.routingType != 0) return fail(c, OVS_ENOTSUP, "Koorde routing is implemented for routingType = iterative");
        if (c->P.lookupRedundantNodes != 1 || c->P.lookupParallelRpcs != 1 || c->P.lookupMerge ||
            c->P.numSiblings != 1 || !c->P.lookupVisitOnlyOnce)
            return fail(c, OVS_ENOTSUP,
                        "Koorde route kernel implements lookupRedundantNodes=1, lookupParallelRpcs=1, merge off, "
                        "visitOnlyOnce, numSiblings=1 (the Koorde defaults)");
    } else if (c->P.routingType < 0 || c->P.routingType > 4) {
        return fail(c, OVS_ENOTSUP, "Kademlia routing is implemented for routingType = iterative / semi-recursive / "
                                    "full-recursive / exhaustive-iterative / source-routing-recursive");
    } else if (c->kad.general && c->P.routingType == 3) {
        return fail(c, OVS_ENOTSUP, "CSR (b > 1 / nr128 / nkademlia) tables: routingType iterative or recursive");
    } else if (c->P.numSiblings != 1) {
        return fail(c, OVS_ENOTSUP, "the one-way route implements numSiblings = 1 (LookupCall: ovs_lookup_batch)");
    } else if (c->kad.lo != 0 || c->kad.hi != c->n) {
        return fail(c, OVS_ESTATE, "context holds one arc of a sharded network: use ovs_kad_shard_step");
    }
    if (n == 0) return OVS_OK;
    st = check_sources(c, src, n, dev);
    if (st != OVS_OK) return st;
    // stage inputs
    K160* dk = nullptr; uint32_t* ds = nullptr; ovs_route_out* dout = nullptr;
    uint32_t* dhop = nullptr; uint32_t* drpc = nullptr;
    bool ok_k = false, ok_s = false;
    if (!dev) {
        st = to_device(c, reinterpret_cast<const K160*>(keys), n, false, &dk, &ok_k);
        if (st != OVS_OK) return st;
        st = to_device(c, src, n, false, &ds, &ok_s);
        if (st != OVS_OK) { hipFree(dk); return st; }
        HIPCHK(c, hipMalloc(&dout, sizeof(ovs_route_out) * n));
    } else {
        dk = const_cast<K160*>(reinterpret_cast<const K160*>(keys));
        ds = const_cast<uint32_t*>(src);
        dout = out;
    }
    // hop sequence buffer: always needed for explicit Chord tables and Koorde (the visited check).
    // Koorde without a hop_seq request uses a context scratch buffer, unpadded: K3 reads back only
    // the entries a lookup wrote
    const bool koorde_scratch = c->overlay == OVS_OVERLAY_KOORDE && !hop_seq;
    // exhaustive-iterative Kademlia: the responder list is the lookup's visited set
    const bool kad_exh = c->overlay == OVS_OVERLAY_KADEMLIA && c->P.routingType == 3;
    // source-routing-recursive Kademlia: the hop list is the message's visitedHops
    const bool kad_src = c->overlay == OVS_OVERLAY_KADEMLIA && c->P.routingType == 4;
    const bool need_hop = hop_seq || (c->overlay == OVS_OVERLAY_CHORD && !c->ideal) || kad_exh || kad_src;
    bool own_hop = false;
    if (koorde_scratch) {
        {
            const ovs_status ks = kvis_acquire(c, n * (uint64_t)H, s, &dhop);
            if (ks != OVS_OK) return ks;
        }
    } else if (need_hop) {
        if (dev && hop_seq) {
            dhop = hop_seq;
        } else if (!hop_seq) {
            // an internal hop list (explicit Chord tables, exhaustive Kademlia: the visited sets) in the
            // context's cached buffer, not a per-call allocation
            {
                const ovs_status ks = kvis_acquire(c, n * (uint64_t)H, s, &dhop);
                if (ks != OVS_OK) return ks;
            }
        } else {
            HIPCHK(c, hipMalloc(&dhop, sizeof(uint32_t) * n * H));
            own_hop = true;
        }
        HIPCHK(c, hipMemsetAsync(dhop, 0xFF, sizeof(uint32_t) * n * H, s));
    }
    bool own_rpc = false;
    if (rpcs) {
        if (dev) drpc = rpcs;
        else { HIPCHK(c, hipMalloc(&drpc, sizeof(uint32_t) * n)); own_rpc = true; }
    }
    hipError_t e;
    if (c->overlay == OVS_OVERLAY_CHORD) {
        LookupConsts LC{c->P.hopCountMax, c->P.numSiblings, c->P.lookupRedundantNodes, c->P.routingType != 0};
        if (drpc) {
            // Chord with alpha = 1: one FindNodeCall per hop; filled after the route below
        }
        if (c->ideal && !LC.recursive && ksort_wanted(n)) {
            // key order: the batch sorted by its keys' top bits, results written at the caller's indices
            K160* sk = nullptr;
            uint32_t *ss = nullptr, *pm = nullptr, *scr = nullptr;
            const ovs_status ks = ks_acquire(c, n, s, &sk, &ss, &pm, &scr);
            if (ks != OVS_OK) return ks;
            const char* kb = std::getenv("OVS_K1_SORT_BITS");
            e = ksort_launch(dk, ds, n, scr, sk, ss, pm, kb ? std::atoi(kb) : 14, s);
            if (e == hipSuccess)
                e = launch_chord_route(chord_view(c), c->ideal, delay_consts(c->P), LC, sk, ss, n, dout, dhop, c->num_cu,
                                       s, pm);
            ks_release(c, s);
        } else {
            int slot = -1;
            unsigned long long* dyn = dyn_acquire(c, n, s, &slot);
            e = launch_chord_route(chord_view(c), c->ideal, delay_consts(c->P), LC, dk, ds, n, dout, dhop, c->num_cu, s,
                                   nullptr, dyn);
            dyn_release(c, s, slot);
        }
        if (e == hipSuccess && drpc) {
            if (LC.recursive) e = hipMemsetAsync(drpc, 0, sizeof(uint32_t) * n, s);   // no FindNodeCalls
            else e = launch_fill_rpcs_from_hops(dout, n, drpc, s);
        }
    } else if (c->overlay == OVS_OVERLAY_KOORDE) {
        int slot = -1;
        unsigned long long* dyn = dyn_acquire(c, n, s, &slot);
        e = koorde_route(c->koorde, c->recs, c->xy, delay_consts(c->P), c->P.hopCountMax, dk, ds, n, dout, dhop,
                         !koorde_scratch, drpc, c->num_cu, s, dyn);
        dyn_release(c, s, slot);
    } else if (kad_exh) {
        // sendToKey with EXHAUSTIVE_ITERATIVE_ROUTING (BaseOverlay.cc:1434-1442): lookup(key, numSiblings = 1)
        // with redundantNodes = lookupRedundantNodes, the route message to getResult()[0]
        uint32_t* dres = nullptr;
        HIPCHK(c, hipMalloc(&dres, sizeof(uint32_t) * n));
        bool cap_err = false;
        // dhop was filled with NONE above: the kernel leaves the rows unpadded
        e = kad_exhaustive(c->kad, c->xy, (uint32_t)c->n, c->P, delay_consts(c->P), c->P.lookupRedundantNodes, 1, true,
                           dk, ds, n, dout, dres, dhop, nullptr, drpc, c->num_cu, s, &cap_err, nullptr, false,
                           hop_seq == nullptr /* nobody reads the visited sets: their first entries in LDS */);
        hipFree(dres);
        if (e == hipSuccess && cap_err) return fail(c, OVS_ENOTSUP, "a lookup exceeded the kernel's capacity (64 timed-out nodes)");
    } else if (c->P.routingType == 1 || c->P.routingType == 2 || kad_src) {
        // R/Kademlia: recursive routing with Kademlia's recursiveRoutingHook (kad_general.hip)
        e = kad_route_recursive(c->kad, c->xy, (uint32_t)c->n, c->P, delay_consts(c->P),
                                simtime_host(c->P.rpcKeyTimeout, c->P.simtimeRound), 1, dk, ds, n, dout, dhop, nullptr, s);
        if (e == hipSuccess && drpc) e = hipMemsetAsync(drpc, 0, sizeof(uint32_t) * n, s);   // no FindNodeCalls
    } else if (c->kad.general) {
        e = kad_route_general(c->kad, c->xy, (uint32_t)c->n, c->P, delay_consts(c->P), dk, ds, n, dout, dhop, drpc, s,
                              nullptr);
    } else {
        int slot = -1;
        unsigned long long* dyn = dyn_acquire(c, n, s, &slot);
        e = kad_route(c->kad, c->xy, (uint32_t)c->n, c->P, delay_consts(c->P), dk, ds, n, dout, dhop, drpc,
                      c->num_cu, s, nullptr, dyn);
        dyn_release(c, s, slot);
    }
    if (dhop && dhop == c->kvis) kvis_release(c, s);
    if (e != hipSuccess) return hip_fail(c, e, "route kernel");
    if (!dev) {
        HIPCHK(c, hipMemcpyAsync(out, dout, sizeof(ovs_route_out) * n, hipMemcpyDeviceToHost, s));
        if (hop_seq) HIPCHK(c, hipMemcpyAsync(hop_seq, dhop, sizeof(uint32_t) * n * H, hipMemcpyDeviceToHost, s));
        if (rpcs) HIPCHK(c, hipMemcpyAsync(rpcs, drpc, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        hipFree(dk); hipFree(ds); hipFree(dout);
    } else if (own_hop || own_rpc) {
        HIPCHK(c, hipStreamSynchronize(s));
    }
    if (own_hop) hipFree(dhop);
    if (own_rpc) hipFree(drpc);
    return OVS_OK;
}

ovs_status ovs_lookup_batch(ovs_ctx* c, const ovs_key160* keys, const uint32_t* src, uint64_t n, int32_t num_siblings,
                            ovs_lookup_out* out, uint32_t* siblings, uint32_t flags, void* stream)
{
    static_assert(sizeof(ovs_lookup_out) == sizeof(ovs_route_out), "lookup results are finished in place");
    if (!c || (n && (!keys || !src || !out || !siblings))) return OVS_EINVAL;
    if (!c->overlay) return fail(c, OVS_ESTATE, "no network loaded");
    if (c->overlay == OVS_OVERLAY_KOORDE)
        return fail(c, OVS_ENOTSUP, "Koorde: ovs_route_batch and ovs_koorde_find_node_batch only");
    if (c->overlay == OVS_OVERLAY_EPICHORD)
        return fail(c, OVS_ENOTSUP, "EpiChord: ovs_epichord_find_node_batch only");
    const bool chord = c->overlay == OVS_OVERLAY_CHORD;
    // BaseOverlay::lookupRpc: numSiblings < 0 -> getMaxNumSiblings() (Chord.cc getMaxNumSiblings =
    // successorListSize, Kademlia.cc:347-350 = s); isSiblingFor rejects larger values
    const int32_t maxs = chord ? c->P.successorListSize : c->P.s;
    const int32_t ns = num_siblings < 0 ? maxs : num_siblings;
    if (ns > maxs) return fail(c, OVS_EINVAL, "numSiblings too big!");
    if (ns == 0 && c->P.routingType == 3)
        return fail(c, OVS_ENOTSUP, "LookupCall with numSiblings = 0 (exact-key lookup): iterative or recursive routing");
    if (ns == 0 && chord && c->P.routingType != 0)
        return fail(c, OVS_ENOTSUP, "Chord LookupCall with numSiblings = 0 (exact-key lookup): iterative routing");
    if (ns == 0 && chord && c->P.hopCountMax < 1)
        return fail(c, OVS_ENOTSUP, "Chord exact-key LookupCalls need hopCountMax >= 1");
    if (ns > 8) return fail(c, OVS_ENOTSUP, "LookupCall implements numSiblings <= 8");
    ovs_params P = c->P;
    P.numSiblings = 1;          // the route checks: one-way configuration, numSiblings applied below
    ovs_status st = check_common(c, P);
    if (st != OVS_OK) return st;
    const bool kad_exh = !chord && P.routingType == 3;
    const bool kad_rec = !chord && (P.routingType == 1 || P.routingType == 2 || P.routingType == 4);
    if (P.routingType != 0 && !kad_exh && !kad_rec)
        return fail(c, OVS_ENOTSUP, "LookupCall is implemented for routingType = iterative (Kademlia: also recursive and "
                                    "exhaustive-iterative)");
    if (kad_exh && c->kad.general)
        return fail(c, OVS_ENOTSUP, "CSR (b > 1 / nr128 / nkademlia) tables: LookupCalls with routingType = iterative");
    if (kad_exh && ns > P.lookupRedundantNodes)
        return fail(c, OVS_EINVAL, "With EXHAUSTIVE_ITERATIVE_ROUTING numRedundantNodes must be >= numSiblings!");
    HIPCHK(c, hipSetDevice(c->device));
    const bool dev = flags & OVS_DEVICE_PTRS;
    hipStream_t s = dev ? (hipStream_t)stream : c->stream;
    if (chord) {
        st = check_chord_route(c, P);
        if (st != OVS_OK) return st;
        if (c->ideal && (c->shard_lo != 0 || c->shard_hi != c->n))
            return fail(c, OVS_ESTATE, "context holds one arc of a sharded ring: LookupCall needs the whole ring");
        st = ensure_nodes(c, s);
        if (st != OVS_OK) return st;
    } else if (c->kad.lo != 0 || c->kad.hi != c->n) {
        return fail(c, OVS_ESTATE, "context holds one arc of a sharded network: LookupCall needs the whole network");
    }
    if (n == 0) return OVS_OK;
    st = check_sources(c, src, n, dev);
    if (st != OVS_OK) return st;
    P.numSiblings = ns;
    const int nslots = ns ? ns : 1;      // an exact-key lookup keeps a one-slot sibling vector (IterativeLookup.cc:149)
    DelayConsts DC = delay_consts(P);
    DC.lookupCall = 1;
    if (chord && c->ideal) {
        // converged ring: every responsible node answers min(numSiblings, 1 + successors) nodes
        const int64_t nsucc = std::min<int64_t>(P.successorListSize, (int64_t)c->n - 1);
        const int nodes = (int)std::min<int64_t>(ns, 1 + nsucc);
        DC.msgRespSib = 2 * simtime_host((double)((int64_t)(DC.respBase + DC.respPerNode * nodes) * 8) / P.datarate,
                                         P.simtimeRound) + DC.access2;
    }
    K160* dk = nullptr; uint32_t* ds = nullptr; ovs_route_out* dout = nullptr; uint32_t* dsib = nullptr;
    uint32_t* dhop = nullptr;
    bool ok_k = false, ok_s = false;
    if (!dev) {
        st = to_device(c, reinterpret_cast<const K160*>(keys), n, false, &dk, &ok_k);
        if (st != OVS_OK) return st;
        st = to_device(c, src, n, false, &ds, &ok_s);
        if (st != OVS_OK) { hipFree(dk); return st; }
        HIPCHK(c, hipMalloc(&dout, sizeof(ovs_route_out) * n));
        HIPCHK(c, hipMalloc(&dsib, sizeof(uint32_t) * n * nslots));
    } else {
        dk = const_cast<K160*>(reinterpret_cast<const K160*>(keys));
        ds = const_cast<uint32_t*>(src);
        dout = reinterpret_cast<ovs_route_out*>(out);
        dsib = siblings;
    }
    // Chord exact-key lookups replay the one-way chain recorded one hop beyond hopCountMax
    const bool chord_exact = chord && ns == 0;
    const int H = chord_exact ? P.hopCountMax + 1 : P.hopCountMax > 0 ? P.hopCountMax : 1;
    // visited check (explicit tables; exhaustive lookups; source routing: the call's route, reversed by the response)
    const bool need_hop = (chord && !c->ideal) || kad_exh || chord_exact || (kad_rec && P.routingType == 4);
    if (need_hop) {
        // internal (a LookupCall records no hop sequence): the context's cached buffer
        {
            const ovs_status ks = kvis_acquire(c, n * (uint64_t)H, s, &dhop);
            if (ks != OVS_OK) return ks;
        }
        HIPCHK(c, hipMemsetAsync(dhop, 0xFF, sizeof(uint32_t) * n * H, s));
    }
    hipError_t e;
    if (chord_exact) {
        // the chain: a one-way route (numSiblings 1, no LookupCall sizes) without timeouts
        DelayConsts DR = delay_consts(P);
        DR.rpcTimeout = DR.lookupTimeout = INT64_MAX / 4;
        LookupConsts LR{H, 1, P.lookupRedundantNodes, 0};
        e = launch_chord_route(chord_view(c), c->ideal, DR, LR, dk, ds, n, dout, dhop, c->num_cu, s);
        if (e == hipSuccess)
            e = launch_chord_exact_finish(chord_view(c), delay_consts(P), P.hopCountMax, dk, ds, dhop, H, dout, n, s);
    } else if (chord) {
        LookupConsts LC{P.hopCountMax, ns, P.lookupRedundantNodes, 0};
        int slot = -1;
        unsigned long long* dyn = dyn_acquire(c, n, s, &slot);
        e = launch_chord_route(chord_view(c), c->ideal, DC, LC, dk, ds, n, dout, dhop, c->num_cu, s, nullptr, dyn);
        dyn_release(c, s, slot);
    } else if (kad_exh) {
        // lookupRpc with EXHAUSTIVE_ITERATIVE_ROUTING: redundantNodes = lookupRedundantNodes, numSiblings = ns
        bool cap_err = false;
        e = kad_exhaustive(c->kad, c->xy, (uint32_t)c->n, P, delay_consts(P), P.lookupRedundantNodes, ns, false, dk, ds,
                           n, dout, dsib, dhop, nullptr, nullptr, c->num_cu, s, &cap_err, nullptr, false,
                           true /* a LookupCall records no hop sequence: the visited sets' first entries in LDS */);
        if (e == hipSuccess && cap_err) e = hipErrorNotSupported;
    } else if (kad_rec) {
        // RecursiveLookup (RecursiveLookup.cc:52-139): a routed FindNodeCall, the response back by UDP
        // (semi-recursive), routed to the source's key (full-recursive) or along the call's route
        // reversed (source-routing-recursive)
        e = kad_route_recursive(c->kad, c->xy, (uint32_t)c->n, P, delay_consts(P),
                                simtime_host(P.rpcKeyTimeout, P.simtimeRound), ns, dk, ds, n, dout,
                                P.routingType == 4 ? dhop : nullptr, dsib, s);
    } else if (c->kad.general) {
        e = kad_route_general(c->kad, c->xy, (uint32_t)c->n, P, DC, dk, ds, n, dout, nullptr, nullptr, s, dsib);
    } else {
        int slot = -1;
        unsigned long long* dyn = dyn_acquire(c, n, s, &slot);
        e = kad_route(c->kad, c->xy, (uint32_t)c->n, P, DC, dk, ds, n, dout, nullptr, nullptr, c->num_cu, s,
                      dsib, dyn);
        dyn_release(c, s, slot);
    }
    if (e == hipSuccess && !kad_exh) e = launch_lookup_finish(chord_view(c), chord, c->ideal, nslots, dout, dsib, n, s);
    if (dhop && dhop == c->kvis) kvis_release(c, s);
    if (e != hipSuccess) {
        if (!dev) { hipFree(dk); hipFree(ds); hipFree(dout); hipFree(dsib); }
        /* dhop: the context's cached buffer */
        return hip_fail(c, e, "lookup kernel");
    }
    if (!dev) {
        HIPCHK(c, hipMemcpyAsync(out, dout, sizeof(ovs_lookup_out) * n, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(siblings, dsib, sizeof(uint32_t) * n * nslots, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        hipFree(dk); hipFree(ds); hipFree(dout); hipFree(dsib);
    }
    /* dhop: the context's cached buffer, ordered by kvis_ev: a device-pointer call stays asynchronous */
    return OVS_OK;
}

ovs_status ovs_kad_refresh_batch(ovs_ctx* c, const ovs_key160* keys, const uint32_t* src, uint64_t n,
                                 int32_t R, ovs_lookup_out* out, uint32_t* siblings, uint32_t* responders,
                                 int64_t* rtt_ns, uint32_t* rpcs, uint32_t flags, void* stream)
{
    if (!c || (n && (!keys || !src || !out || !siblings))) return OVS_EINVAL;
    if (!c->overlay) return fail(c, OVS_ESTATE, "no network loaded");
    if (c->overlay != OVS_OVERLAY_KADEMLIA) return fail(c, OVS_ESTATE, "refresh lookups: Kademlia only");
    if (c->kad.lo != 0 || c->kad.hi != c->n)
        return fail(c, OVS_ESTATE, "context holds one arc of a sharded network: refresh lookups need the whole network");
    if (c->kad.general) return fail(c, OVS_ENOTSUP, "refresh lookups run on the 160-bucket kademlia tables");
    if (R < 1 || R > 64) return fail(c, OVS_ENOTSUP, "refresh lookups implement redundantNodes 1..64");
    const ovs_params& P = c->P;
    if (P.hopCountMax < 1) return fail(c, OVS_ENOTSUP, "refresh lookups need hopCountMax >= 1");
    if (!P.lookupMerge || !P.lookupStrictParallelRpcs || P.lookupParallelRpcs < 1 || P.lookupParallelRpcs > KAD_MAX_ALPHA)
        return fail(c, OVS_ENOTSUP, "refresh lookups implement lookupMerge, strictParallelRpcs, parallelRpcs 1..8");
    if (P.lookupParallelPaths != 1 || P.lookupVerifySiblings || P.lookupMajoritySiblings || P.jitter != 0.0)
        return fail(c, OVS_ENOTSUP, "parallelPaths 1, no verify/majority siblings, jitter 0");
    HIPCHK(c, hipSetDevice(c->device));
    const bool dev = flags & OVS_DEVICE_PTRS;
    hipStream_t s = dev ? (hipStream_t)stream : c->stream;
    if (n == 0) return OVS_OK;
    if (!dev)
        for (uint64_t i = 0; i < n; ++i)
            if (src[i] >= c->n) return fail(c, OVS_EINVAL, "source index out of range");
    const uint64_t H = (uint64_t)P.hopCountMax;
    K160* dk = nullptr; uint32_t* ds = nullptr; ovs_lookup_out* dout = nullptr; uint32_t* dsib = nullptr;
    uint32_t* dresp = nullptr; int64_t* drtt = nullptr; uint32_t* drpc = nullptr;
    bool ok_k = false, ok_s = false;
    ovs_status st = to_device(c, reinterpret_cast<const K160*>(keys), n, dev, &dk, &ok_k);
    if (st != OVS_OK) return st;
    st = to_device(c, src, n, dev, &ds, &ok_s);
    if (st != OVS_OK) { if (ok_k) hipFree(dk); return st; }
    // the responder list is the lookup's visited set: always present on the device -- when the
    // caller asked for none, in the context's cached buffer (as K3's; a per-call hipMalloc / hipFree
    // of n * hopCountMax entries had put an allocation and a device synchronisation into every call)
    const bool internal_resp = !responders;
    const bool own_resp = !dev && responders, own_rtt = !dev && rtt_ns, own_rpc = !dev && rpcs;
    auto cleanup = [&]() {
        if (ok_k) hipFree(dk);
        if (ok_s) hipFree(ds);
        if (!dev) { hipFree(dout); hipFree(dsib); }
        if (own_resp) hipFree(dresp);
        if (own_rtt) hipFree(drtt);
        if (own_rpc) hipFree(drpc);
    };
    if (!dev) {
        HIPCHK(c, hipMalloc(&dout, sizeof(ovs_lookup_out) * n));
        HIPCHK(c, hipMalloc(&dsib, sizeof(uint32_t) * n * R));
    } else { dout = out; dsib = siblings; }
    if (internal_resp) {
        {
            const ovs_status ks = kvis_acquire(c, n * H, s, &dresp);
            if (ks != OVS_OK) return ks;
        }
    } else if (own_resp) {
        HIPCHK(c, hipMalloc(&dresp, sizeof(uint32_t) * n * H));
    } else {
        dresp = responders;
    }
    if (own_rtt) HIPCHK(c, hipMalloc(&drtt, sizeof(int64_t) * n * H));
    else drtt = rtt_ns;
    if (own_rpc) HIPCHK(c, hipMalloc(&drpc, sizeof(uint32_t) * n));
    else drpc = rpcs;
    bool cap_err = false;
    const hipError_t e = kad_exhaustive(c->kad, c->xy, (uint32_t)c->n, P, delay_consts(P), R, R, false, dk, ds, n, dout,
                                        dsib, dresp, drtt, drpc, c->num_cu, s, &cap_err, nullptr,
                                        responders != nullptr /* else the internal visited lists: no padding */,
                                        responders == nullptr /* ... and their first entries in LDS */);
    if (internal_resp) kvis_release(c, s);
    if (e != hipSuccess) { cleanup(); return hip_fail(c, e, "refresh lookup kernel"); }
    if (cap_err) { cleanup(); return fail(c, OVS_ENOTSUP, "a refresh lookup exceeded the kernel's capacity (64 timed-out nodes)"); }
    if (!dev) {
        HIPCHK(c, hipMemcpyAsync(out, dout, sizeof(ovs_lookup_out) * n, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(siblings, dsib, sizeof(uint32_t) * n * R, hipMemcpyDeviceToHost, s));
        if (responders) HIPCHK(c, hipMemcpyAsync(responders, dresp, sizeof(uint32_t) * n * H, hipMemcpyDeviceToHost, s));
        if (rtt_ns) HIPCHK(c, hipMemcpyAsync(rtt_ns, drtt, sizeof(int64_t) * n * H, hipMemcpyDeviceToHost, s));
        if (rpcs) HIPCHK(c, hipMemcpyAsync(rpcs, drpc, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
    }
    cleanup();
    return OVS_OK;
}

extern "C++" {
namespace {

// rebuild the device tables of a whole-network Kademlia context from its host copy
ovs_status kad_upload_host_tables(ovs_ctx* c)
{
    const uint64_t n = c->n, S5 = 5ull * (uint64_t)c->P.s, k = (uint64_t)c->P.k;
    std::vector<uint32_t> hs(n * S5), hn(n * 160 * k);
    std::vector<uint8_t> hc(n * 160);
    if (!c->kh.export_k(hs.data(), hc.data(), hn.data())) {
        free_tables(c);    // the host copy was changed by the round: the device tables no longer match it
        return fail(c, OVS_ENOTSUP, "a bucket outgrew k (bucketType kademlia keeps k per bucket)");
    }
    uint32_t *dsib = nullptr, *dbn = nullptr;
    uint8_t* dbc = nullptr;
    auto release = [&]() { if (dsib) hipFree(dsib); if (dbn) hipFree(dbn); if (dbc) hipFree(dbc); };
    if (hipMalloc(&dsib, sizeof(uint32_t) * n * S5) != hipSuccess || hipMalloc(&dbc, n * 160) != hipSuccess ||
        hipMalloc(&dbn, sizeof(uint32_t) * n * 160 * k) != hipSuccess) {
        release();
        return fail(c, OVS_ENOMEM, "maintenance round: device allocation failed");
    }
    hipError_t e = hipMemcpy(dsib, hs.data(), sizeof(uint32_t) * n * S5, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dbc, hc.data(), n * 160, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dbn, hn.data(), sizeof(uint32_t) * n * 160 * k, hipMemcpyHostToDevice);
    uint32_t bad_node = 0, bad_code = 0;
    // build into a temporary and swap it in only on success: a failed rebuild must leave the context
    // either with its previous tables or with none (free_tables below), never with null or half-built
    // tables that a later route would launch on
    KadTables nt{};
    if (e == hipSuccess)
        e = kad_build_explicit(c->recs, c->xy, (uint32_t)n, c->P.k, c->P.s, dsib, dbc, dbn, nt, &bad_node, &bad_code,
                               c->stream);
    // test hook: OVS_FAULT_INJECT=kad_rebuild makes the rebuild report a broken invariant
    // (tests/test_gpu_kad_maint.py::test_failed_rebuild_leaves_no_tables)
    if (e == hipSuccess && fault_injected("kad_rebuild")) { e = hipErrorInvalidValue; bad_code = 99; }
    release();
    if (e == hipSuccess) {
        kad_free(c->kad);
        c->kad = nt;
    } else {
        kad_free(nt);
        // the host copy has already been changed by the round: the old device tables no longer
        // describe it, so the context drops its network (later calls fail with OVS_ESTATE)
        free_tables(c);
    }
    if (e == hipErrorInvalidValue && bad_code) {
        char m[160];
        std::snprintf(m, sizeof m, "maintenance round broke a table invariant at node %u (code %u)", bad_node, bad_code);
        return fail(c, OVS_EDEVICE, m);
    }
    if (e != hipSuccess) return hip_fail(c, e, "maintenance round: table rebuild");
    return OVS_OK;
}

}  // namespace
}  // extern "C++"

ovs_status ovs_kad_maintenance_round(ovs_ctx* c, const uint32_t* nodes, uint64_t m, const uint8_t* flags,
                                     const uint32_t* stale, ovs_kad_round_stats* stats)
{
    if (!c || (m && !nodes)) return OVS_EINVAL;
    if (c->overlay != OVS_OVERLAY_KADEMLIA) return fail(c, OVS_ESTATE, "no Kademlia network loaded");
    if (c->kad.lo != 0 || c->kad.hi != c->n) return fail(c, OVS_ESTATE, "maintenance rounds need the whole network");
    if (c->kad.general) return fail(c, OVS_ENOTSUP, "maintenance rounds run on the 160-bucket kademlia tables");
    const ovs_params& P = c->P;
    if (P.routingType != 0) return fail(c, OVS_ENOTSUP, "maintenance rounds run iterative refresh lookups");
    if (P.hopCountMax < 1) return fail(c, OVS_ENOTSUP, "refresh lookups need hopCountMax >= 1");
    if (!P.lookupMerge || !P.lookupStrictParallelRpcs || P.lookupParallelRpcs < 1 || P.lookupParallelRpcs > KAD_MAX_ALPHA)
        return fail(c, OVS_ENOTSUP, "refresh lookups implement lookupMerge, strictParallelRpcs, parallelRpcs 1..8");
    if (P.lookupParallelPaths != 1 || P.lookupVerifySiblings || P.lookupMajoritySiblings || P.jitter != 0.0)
        return fail(c, OVS_ENOTSUP, "parallelPaths 1, no verify/majority siblings, jitter 0");
    const int Rs = 5 * P.s, Rb = P.lookupRedundantNodes;
    if (Rs > 64 || Rb > 64) return fail(c, OVS_ENOTSUP, "refresh lookups implement redundantNodes 1..64");
    for (uint64_t j = 0; j < m; ++j)
        if (nodes[j] >= c->n) return fail(c, OVS_EINVAL, "node index out of range");
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t s = c->stream;
    if (c->kh.n() != c->n) {
        // a snapshot network (ovs_kad_load): its tables become the host copy
        const uint64_t n = c->n, S5 = 5ull * (uint64_t)P.s, k = (uint64_t)P.k;
        std::vector<uint32_t> hs(n * S5), hn(n * 160 * k);
        std::vector<uint8_t> hc(n * 160);
        const hipError_t e = kad_export(c->kad, (uint32_t)n, hs.data(), hc.data(), hn.data(), s);
        if (e != hipSuccess) return hip_fail(c, e, "maintenance round: table export");
        std::vector<K160> ids(n);
        std::vector<KeyRec> recs(n);
        HIPCHK(c, hipMemcpy(recs.data(), c->recs, sizeof(KeyRec) * n, hipMemcpyDeviceToHost));
        for (uint64_t v = 0; v < n; ++v) ids[v] = key_of(recs[v]);
        c->kh.import(ids.data(), n, P.k, P.s, hs.data(), hc.data(), hn.data());
    }
    KadRoundCount cnt;
    std::vector<K160> keys;
    std::vector<uint32_t> src;
    std::vector<int> R;
    c->kh.refresh_plan(nodes, m, flags, stale, Rs, Rb, &keys, &src, &R);
    const uint64_t nt = keys.size(), H = (uint64_t)P.hopCountMax;
    const int ccap = 2 * P.hopCountMax + 2 * P.lookupParallelRpcs + 16;
    cnt.lookups = nt;
    // host results of every lookup
    std::vector<uint32_t> resp(nt * H), cnode(nt * (uint64_t)ccap);
    std::vector<int64_t> tarr(nt * H), ctime(nt * (uint64_t)ccap);
    std::vector<ovs_lookup_out> outv(nt);
    const DelayConsts DC = delay_consts(P);
    for (int g = 0; g < 2 && nt; ++g) {
        const int Rg = g == 0 ? Rs : Rb;
        if (g == 1 && Rb == Rs) break;
        std::vector<uint64_t> ix;
        for (uint64_t t = 0; t < nt; ++t)
            if (R[t] == Rg) ix.push_back(t);
        if (ix.empty()) continue;
        const uint64_t ng = ix.size();
        std::vector<K160> gk(ng);
        std::vector<uint32_t> gs(ng);
        for (uint64_t q = 0; q < ng; ++q) { gk[q] = keys[ix[q]]; gs[q] = src[ix[q]]; }
        DevBufs d;
        K160* dk; uint32_t *ds, *dsib, *dresp, *drpc, *dcn; ovs_lookup_out* dout; int64_t *dta, *dct;
        HIPCHK(c, d.get(&dk, ng)); HIPCHK(c, d.get(&ds, ng)); HIPCHK(c, d.get(&dsib, ng * (uint64_t)Rg));
        HIPCHK(c, d.get(&dresp, ng * H)); HIPCHK(c, d.get(&drpc, ng)); HIPCHK(c, d.get(&dout, ng));
        HIPCHK(c, d.get(&dta, ng * H)); HIPCHK(c, d.get(&dcn, ng * (uint64_t)ccap)); HIPCHK(c, d.get(&dct, ng * (uint64_t)ccap));
        HIPCHK(c, hipMemcpyAsync(dk, gk.data(), sizeof(K160) * ng, hipMemcpyHostToDevice, s));
        HIPCHK(c, hipMemcpyAsync(ds, gs.data(), sizeof(uint32_t) * ng, hipMemcpyHostToDevice, s));
        const KadExhTrace tr{dta, dcn, dct, ccap};
        bool cap_err = false;
        const hipError_t e = kad_exhaustive(c->kad, c->xy, (uint32_t)c->n, P, DC, Rg, Rg, false, dk, ds, ng, dout, dsib,
                                            dresp, nullptr, drpc, c->num_cu, s, &cap_err, &tr);
        if (e != hipSuccess) return hip_fail(c, e, "maintenance round: refresh lookups");
        if (cap_err) return fail(c, OVS_ENOTSUP, "a refresh lookup exceeded the kernel's capacity");
        std::vector<uint32_t> hr(ng * H), hc(ng * (uint64_t)ccap);
        std::vector<int64_t> hta(ng * H), hct(ng * (uint64_t)ccap);
        std::vector<ovs_lookup_out> ho(ng);
        HIPCHK(c, hipMemcpyAsync(hr.data(), dresp, sizeof(uint32_t) * ng * H, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(hta.data(), dta, sizeof(int64_t) * ng * H, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(hc.data(), dcn, sizeof(uint32_t) * ng * ccap, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(hct.data(), dct, sizeof(int64_t) * ng * ccap, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(ho.data(), dout, sizeof(ovs_lookup_out) * ng, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        for (uint64_t q = 0; q < ng; ++q) {
            const uint64_t t = ix[q];
            std::copy(hr.begin() + q * H, hr.begin() + (q + 1) * H, resp.begin() + t * H);
            std::copy(hta.begin() + q * H, hta.begin() + (q + 1) * H, tarr.begin() + t * H);
            std::copy(hc.begin() + q * ccap, hc.begin() + (q + 1) * ccap, cnode.begin() + t * ccap);
            std::copy(hct.begin() + q * ccap, hct.begin() + (q + 1) * ccap, ctime.begin() + t * ccap);
            outv[t] = ho[q];
        }
    }
    // the carried nodes of every handled response: findNode(key, R, -1) at the responder on the
    // round-start tables (BaseOverlay::findNodeRpc, BaseOverlay.cc:1841-1915), on the device
    std::vector<uint64_t> pair_off(nt * H + 1, 0);
    std::vector<uint32_t> carried;
    std::vector<uint8_t> ncarried(nt * H, 0);
    std::vector<int> nresp(nt, 0), ncall(nt, 0);
    for (uint64_t t = 0; t < nt; ++t) {
        while (nresp[t] < (int)H && resp[t * H + nresp[t]] != 0xFFFFFFFFu) ++nresp[t];
        while (ncall[t] < ccap && cnode[t * ccap + ncall[t]] != 0xFFFFFFFFu) ++ncall[t];
        if (outv[t].status != OVS_LOOKUP_OK) cnt.failed++;
    }
    std::vector<uint64_t> roff(nt * H, 0);
    {
        uint64_t tot = 0;
        for (uint64_t t = 0; t < nt; ++t)
            for (int i = 0; i < nresp[t]; ++i) { roff[t * H + i] = tot; tot += (uint64_t)R[t]; }
        carried.assign(tot ? tot : 1, 0xFFFFFFFFu);
        for (int g = 0; g < 2; ++g) {
            const int Rg = g == 0 ? Rs : Rb;
            if (g == 1 && Rb == Rs) break;
            std::vector<uint32_t> pn;
            std::vector<K160> pk;
            std::vector<uint64_t> pri;
            for (uint64_t t = 0; t < nt; ++t)
                if (R[t] == Rg)
                    for (int i = 0; i < nresp[t]; ++i) { pn.push_back(resp[t * H + i]); pk.push_back(keys[t]); pri.push_back(t * H + i); }
            const uint64_t np = pn.size();
            if (np == 0) continue;
            DevBufs d;
            uint32_t *dn, *dout; K160* dk; uint8_t *dcount, *dsb;
            HIPCHK(c, d.get(&dn, np)); HIPCHK(c, d.get(&dk, np)); HIPCHK(c, d.get(&dout, np * (uint64_t)Rg));
            HIPCHK(c, d.get(&dcount, np)); HIPCHK(c, d.get(&dsb, np));
            HIPCHK(c, hipMemcpyAsync(dn, pn.data(), sizeof(uint32_t) * np, hipMemcpyHostToDevice, s));
            HIPCHK(c, hipMemcpyAsync(dk, pk.data(), sizeof(K160) * np, hipMemcpyHostToDevice, s));
            const hipError_t e = kad_find_node(c->kad, (uint32_t)c->n, P, dn, dk, np, Rg, -1, dout, (uint32_t)Rg, dcount,
                                               dsb, s);
            if (e != hipSuccess) return hip_fail(c, e, "maintenance round: findNode of the responses");
            std::vector<uint32_t> ho(np * (uint64_t)Rg);
            std::vector<uint8_t> hcount(np);
            HIPCHK(c, hipMemcpyAsync(ho.data(), dout, sizeof(uint32_t) * np * Rg, hipMemcpyDeviceToHost, s));
            HIPCHK(c, hipMemcpyAsync(hcount.data(), dcount, np, hipMemcpyDeviceToHost, s));
            HIPCHK(c, hipStreamSynchronize(s));
            for (uint64_t q = 0; q < np; ++q) {
                ncarried[pri[q]] = hcount[q];
                std::copy(ho.begin() + q * Rg, ho.begin() + q * Rg + hcount[q], carried.begin() + roff[pri[q]]);
            }
        }
    }
    std::vector<const uint32_t*> cptr(nt * H, nullptr);
    for (uint64_t t = 0; t < nt; ++t)
        for (int i = 0; i < nresp[t]; ++i) cptr[t * H + i] = carried.data() + roff[t * H + i];
    std::vector<KadRoundLookup> lk(nt);
    for (uint64_t t = 0; t < nt; ++t) {
        KadRoundLookup& L = lk[t];
        L.src = src[t];
        L.cnode = cnode.data() + t * ccap; L.ctime = ctime.data() + t * ccap; L.ncall = ncall[t];
        L.resp = resp.data() + t * H; L.tarr = tarr.data() + t * H; L.nresp = nresp[t];
        L.carried = cptr.data() + t * H; L.ncarried = ncarried.data() + t * H;
    }
    c->kh.apply_round(lk, &cnt);
    const ovs_status us = kad_upload_host_tables(c);
    if (us != OVS_OK) return us;
    if (stats) {
        stats->lookups = cnt.lookups; stats->failed = cnt.failed; stats->responses = cnt.responses;
        stats->sib_changes = cnt.sib_changes; stats->bucket_changes = cnt.bucket_changes; stats->lost = cnt.lost;
        stats->replacement = cnt.replacement; stats->refreshed = cnt.refreshed;
    }
    return OVS_OK;
}

ovs_status ovs_kad_refresh_keys(ovs_ctx* c, const uint32_t* nodes, uint64_t m, const uint32_t* stale,
                                ovs_key160* keys, uint32_t* src, uint64_t cap, uint64_t* count, uint32_t flags,
                                void* stream)
{
    if (!c || !count || (m && !nodes) || (cap && (!keys || !src))) return OVS_EINVAL;
    if (c->overlay != OVS_OVERLAY_KADEMLIA) return fail(c, OVS_ESTATE, "bucket refresh: Kademlia network needed");
    if (c->kad.lo != 0 || c->kad.hi != c->n) return fail(c, OVS_ESTATE, "bucket refresh needs the whole network");
    if (c->kad.general) return fail(c, OVS_ENOTSUP, "refresh keys are generated for the 160-bucket kademlia tables");
    HIPCHK(c, hipSetDevice(c->device));
    const bool dev = flags & OVS_DEVICE_PTRS;
    hipStream_t s = dev ? (hipStream_t)stream : c->stream;
    *count = 0;
    if (m == 0) return OVS_OK;
    if (!dev)
        for (uint64_t i = 0; i < m; ++i)
            if (nodes[i] >= c->n) return fail(c, OVS_EINVAL, "node index out of range");
    uint32_t* dn = nullptr; uint32_t* dst = nullptr; K160* dk = nullptr; uint32_t* dsrc = nullptr;
    bool o1 = false, o2 = false;
    ovs_status st = to_device(c, nodes, m, dev, &dn, &o1);
    if (st != OVS_OK) return st;
    if (stale) {
        st = to_device(c, stale, m * 5, dev, &dst, &o2);
        if (st != OVS_OK) { if (o1) hipFree(dn); return st; }
    }
    if (cap && !dev) {
        HIPCHK(c, hipMalloc(&dk, sizeof(K160) * cap));
        HIPCHK(c, hipMalloc(&dsrc, sizeof(uint32_t) * cap));
    } else if (cap) {
        dk = reinterpret_cast<K160*>(keys);
        dsrc = src;
    }
    uint64_t total = 0;
    const hipError_t e = kad_refresh_keys(c->kad, (uint32_t)c->n, dn, m, dst, dk, dsrc, cap, &total, s);
    if (e == hipSuccess && cap && !dev) {
        const uint64_t w = total < cap ? total : cap;
        HIPCHK(c, hipMemcpyAsync(keys, dk, sizeof(K160) * w, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(src, dsrc, sizeof(uint32_t) * w, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
    }
    if (o1) hipFree(dn);
    if (o2) hipFree(dst);
    if (cap && !dev) { hipFree(dk); hipFree(dsrc); }
    if (e != hipSuccess) return hip_fail(c, e, "bucket refresh keys");
    *count = total;
    return OVS_OK;
}

ovs_status ovs_find_node_batch(ovs_ctx* c, const uint32_t* node, const ovs_key160* keys, uint64_t n,
                               int32_t numRedundantNodes, int32_t numSiblings, uint32_t* out_nodes,
                               uint32_t max_out, uint8_t* out_count, uint8_t* out_sibling, uint32_t flags,
                               void* stream)
{
    if (!c || (n && (!node || !keys || !out_nodes || !out_count || !out_sibling)) || max_out == 0) return OVS_EINVAL;
    if (!c->overlay) return fail(c, OVS_ESTATE, "no network loaded");
    if (c->overlay == OVS_OVERLAY_KOORDE)
        return fail(c, OVS_ENOTSUP, "Koorde: ovs_route_batch and ovs_koorde_find_node_batch only");
    if (c->overlay == OVS_OVERLAY_EPICHORD)
        return fail(c, OVS_ENOTSUP, "EpiChord: ovs_epichord_find_node_batch only");
    if (numSiblings > (c->overlay == OVS_OVERLAY_CHORD ? c->P.successorListSize : c->P.s))
        return fail(c, OVS_EINVAL, "numSiblings too big!");
    if (numRedundantNodes < 1 || numRedundantNodes > 64) return fail(c, OVS_EINVAL, "numRedundantNodes out of range");
    if (c->overlay == OVS_OVERLAY_CHORD && c->P.extendedFingerTable && numRedundantNodes > 1)
        return fail(c, OVS_ENOTSUP, "extendedFingerTable: findNode answers of more than one node (finger candidate "
                                    "lists) are not implemented");
    if (numSiblings < 0 && (numSiblings != -1 || c->overlay != OVS_OVERLAY_KADEMLIA))
        return fail(c, OVS_ENOTSUP, "numSiblings -1 (an exhaustive-iterative call) is implemented for Kademlia");
    HIPCHK(c, hipSetDevice(c->device));
    const bool dev = flags & OVS_DEVICE_PTRS;
    hipStream_t s = dev ? (hipStream_t)stream : c->stream;   // NULL = the default stream
    if (n == 0) return OVS_OK;
    uint32_t* dn = nullptr; K160* dk = nullptr; uint32_t* dout = nullptr; uint8_t* dc = nullptr; uint8_t* dsb = nullptr;
    bool o1, o2;
    ovs_status st = to_device(c, node, n, dev, &dn, &o1);
    if (st != OVS_OK) return st;
    st = to_device(c, reinterpret_cast<const K160*>(keys), n, dev, &dk, &o2);
    if (st != OVS_OK) return st;
    if (!dev) {
        HIPCHK(c, hipMalloc(&dout, sizeof(uint32_t) * n * max_out));
        HIPCHK(c, hipMalloc(&dc, n));
        HIPCHK(c, hipMalloc(&dsb, n));
    } else { dout = out_nodes; dc = out_count; dsb = out_sibling; }
    // validate node indices on the host for host calls
    if (!dev) {
        for (uint64_t i = 0; i < n; ++i)
            if (node[i] >= c->n) return fail(c, OVS_EINVAL, "node index out of range");
    }
    hipError_t e;
    if (c->overlay == OVS_OVERLAY_CHORD)
        e = launch_chord_find_node(chord_view(c), c->ideal, dn, dk, n, numRedundantNodes, numSiblings, dout, max_out,
                                   dc, dsb, s);
    else if (c->kad.general)
        e = kad_find_node_general(c->kad, (uint32_t)c->n, dn, dk, n, numRedundantNodes, numSiblings, dout, max_out, dc,
                                  dsb, s);
    else
        e = kad_find_node(c->kad, (uint32_t)c->n, c->P, dn, dk, n, numRedundantNodes, numSiblings, dout,
                          max_out, dc, dsb, s);
    if (e != hipSuccess) return hip_fail(c, e, "findNode kernel");
    if (!dev) {
        HIPCHK(c, hipMemcpyAsync(out_nodes, dout, sizeof(uint32_t) * n * max_out, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(out_count, dc, n, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(out_sibling, dsb, n, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        hipFree(dn); hipFree(dk); hipFree(dout); hipFree(dc); hipFree(dsb);
    }
    return OVS_OK;
}

ovs_status ovs_delay_batch(ovs_ctx* c, const uint32_t* a, const uint32_t* b, const int32_t* bytes, uint64_t n,
                           int64_t* out_ns, uint32_t flags, void* stream)
{
    if (!c || (n && (!a || !b || !bytes || !out_ns))) return OVS_EINVAL;
    if (!c->overlay) return fail(c, OVS_ESTATE, "no network loaded");
    HIPCHK(c, hipSetDevice(c->device));
    const bool dev = flags & OVS_DEVICE_PTRS;
    hipStream_t s = dev ? (hipStream_t)stream : c->stream;   // NULL = the default stream
    if (n == 0) return OVS_OK;
    if (!dev) {
        for (uint64_t i = 0; i < n; ++i)
            if (a[i] >= c->n || b[i] >= c->n) return fail(c, OVS_EINVAL, "node index out of range");
    }
    uint32_t *da, *db; int32_t* dbytes; int64_t* dout;
    bool o1, o2, o3;
    ovs_status st = to_device(c, a, n, dev, &da, &o1);
    if (st == OVS_OK) st = to_device(c, b, n, dev, &db, &o2);
    if (st == OVS_OK) st = to_device(c, bytes, n, dev, &dbytes, &o3);
    if (st != OVS_OK) return st;
    if (!dev) HIPCHK(c, hipMalloc(&dout, sizeof(int64_t) * n)); else dout = out_ns;
    hipError_t e = launch_delay(c->xy, delay_consts(c->P), da, db, dbytes, n, dout, s);
    if (e != hipSuccess) return hip_fail(c, e, "delay kernel");
    if (!dev) {
        HIPCHK(c, hipMemcpyAsync(out_ns, dout, sizeof(int64_t) * n, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        hipFree(da); hipFree(db); hipFree(dbytes); hipFree(dout);
    }
    return OVS_OK;
}

ovs_status ovs_kbrtest_stats_batch(ovs_ctx* c, const ovs_route_out* out, const ovs_key160* keys, const uint32_t* src,
                                   uint64_t n, double measured_time_s, int32_t lookup_node_ids,
                                   ovs_kbrtest_stats* stats, uint32_t flags, void* stream)
{
    if (!c || !stats || (n && (!out || !src || (lookup_node_ids && !keys)))) return OVS_EINVAL;
    if (!c->overlay) return fail(c, OVS_ESTATE, "no network loaded");
    if (!(measured_time_s >= 0)) return fail(c, OVS_EINVAL, "measured_time_s must be >= 0");
    HIPCHK(c, hipSetDevice(c->device));
    const bool dev = flags & OVS_DEVICE_PTRS;
    hipStream_t s = dev ? (hipStream_t)stream : c->stream;   // NULL = the default stream
    const ovs_route_out* dout = out;
    const K160* dk = reinterpret_cast<const K160*>(keys);
    const uint32_t* ds = src;
    std::vector<void*> owned;
    auto cleanup = [&]() { for (void* p : owned) hipFree(p); };
    if (!dev && n) {
        ovs_route_out* o; K160* k = nullptr; uint32_t* r; bool ow;
        ovs_status st = to_device(c, out, n, false, &o, &ow);
        if (st != OVS_OK) return st;
        owned.push_back(o);
        st = to_device(c, src, n, false, &r, &ow);
        if (st != OVS_OK) { cleanup(); return st; }
        owned.push_back(r);
        if (lookup_node_ids) {
            st = to_device(c, reinterpret_cast<const K160*>(keys), n, false, &k, &ow);
            if (st != OVS_OK) { cleanup(); return st; }
            owned.push_back(k);
        }
        dout = o; dk = k; ds = r;
    }
    StatsDev* S = nullptr; uint32_t* counts = nullptr; double* partial = nullptr; double* result = nullptr;
    if (hipMalloc(&S, sizeof(StatsDev)) != hipSuccess ||
        hipMalloc(&counts, sizeof(uint32_t) * 3 * c->n) != hipSuccess ||
        hipMalloc(&partial, sizeof(double) * STATS_NODE_BLOCKS * NSTAT * 5) != hipSuccess ||
        hipMalloc(&result, sizeof(double) * NSTAT * 5) != hipSuccess) {
        owned.push_back(S); owned.push_back(counts); owned.push_back(partial); owned.push_back(result);
        cleanup();
        return fail(c, OVS_ENOMEM, "statistics scratch allocation failed");
    }
    owned.push_back(S); owned.push_back(counts); owned.push_back(partial); owned.push_back(result);
    // GlobalStatistics::MIN_MEASURED = 0.1 s (GlobalStatistics.cc:32, KBRTestApp.cc:502)
    const int rates = measured_time_s >= 0.1;
    hipError_t e = launch_stats(dout, dk, ds, c->recs, n, (uint32_t)c->n, lookup_node_ids,
                                measured_time_s, (uint64_t)c->P.testMsgSize, rates, S, counts,
                                partial, result, c->num_cu, s);
    StatsDev h{};
    double r[NSTAT * 5];
    if (e == hipSuccess) e = hipMemcpyAsync(&h, S, sizeof h, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipMemcpyAsync(r, result, sizeof r, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    cleanup();
    if (e != hipSuccess) return hip_fail(c, e, "statistics kernels");

    ovs_kbrtest_stats& o = *stats;
    std::memset(&o, 0, sizeof o);
    const uint64_t B = (uint64_t)c->P.testMsgSize;
    o.num_sent = n;
    o.num_delivered = h.delivered;
    o.num_dropped = h.dropped;
    o.num_lookup_failed = h.failed;
    o.bytes_sent = n * B;
    o.bytes_delivered = h.delivered * B;
    o.bytes_dropped = h.dropped * B;
    o.hop_count_sum = h.hop_sum;
    o.latency_sum_ns = (int64_t)h.lat_sum;
    if (h.delivered) {
        o.hop_count_min = (uint32_t)h.hop_min;
        o.hop_count_max = (uint32_t)h.hop_max;
        o.latency_min_ns = (int64_t)h.lat_min;
        o.latency_max_ns = (int64_t)h.lat_max;
        // GlobalStatistics::finalizeStatistics: OutVector value / count (GlobalStatistics.cc:134-139);
        // latency values are SIMTIME_DBL(latency), summed here exactly in ns
        o.hop_count_mean = (double)h.hop_sum / (double)h.delivered;
        o.latency_mean_s = ((double)h.lat_sum / (double)h.delivered) * 1e-9;
    }
    for (int i = 0; i < 8; ++i) o.status_count[i] = h.status[i];
    for (int i = 0; i < 64; ++i) o.hop_hist[i] = h.hist[i];
    ovs_stddev* sd[NSTAT] = {&o.delivered_msgs_per_s, &o.delivered_bytes_per_s, &o.dropped_msgs_per_s,
                             &o.dropped_bytes_per_s, &o.delivery_ratio};
    for (int k = 0; k < NSTAT; ++k) {
        const double sum = r[k * 5 + 0], sq = r[k * 5 + 1];
        uint64_t cnt;
        std::memcpy(&cnt, &r[k * 5 + 4], sizeof cnt);
        ovs_stddev& d = *sd[k];
        d.count = cnt;
        if (!cnt) continue;
        // cStdDev::getMean / getVariance (OMNeT++ 4.x): sample variance, 0 below two values or if negative
        d.mean = sum / (double)cnt;
        double var = 0.0;
        if (cnt > 1) {
            var = (sq - sum * sum / (double)cnt) / (double)(cnt - 1);
            if (var < 0) var = 0;
        }
        d.stddev = std::sqrt(var);
        d.min = r[k * 5 + 2];
        d.max = r[k * 5 + 3];
    }
    return OVS_OK;
}

ovs_status ovs_kbrtest_lookup_stats_batch(ovs_ctx* c, const ovs_lookup_out* out, const uint32_t* siblings,
                                          int32_t siblings_stride, const ovs_key160* keys, const uint32_t* src,
                                          uint64_t n, double measured_time_s, int32_t lookup_node_ids,
                                          double failure_latency_s, ovs_kbrtest_lookup_stats* stats, uint32_t flags,
                                          void* stream)
{
    if (!c || !stats || siblings_stride < 1 || (n && (!out || !src || !siblings || (lookup_node_ids && !keys))))
        return OVS_EINVAL;
    if (!c->overlay) return fail(c, OVS_ESTATE, "no network loaded");
    if (!(measured_time_s >= 0)) return fail(c, OVS_EINVAL, "measured_time_s must be >= 0");
    HIPCHK(c, hipSetDevice(c->device));
    const bool dev = flags & OVS_DEVICE_PTRS;
    hipStream_t s = dev ? (hipStream_t)stream : c->stream;
    const ovs_route_out* dout = reinterpret_cast<const ovs_route_out*>(out);
    const K160* dk = reinterpret_cast<const K160*>(keys);
    const uint32_t* ds = src;
    const uint32_t* dsib = siblings;
    std::vector<void*> owned;
    auto cleanup = [&]() { for (void* p : owned) hipFree(p); };
    if (!dev && n) {
        ovs_route_out* o; K160* k = nullptr; uint32_t* r; uint32_t* f; bool ow;
        ovs_status st = to_device(c, reinterpret_cast<const ovs_route_out*>(out), n, false, &o, &ow);
        if (st != OVS_OK) return st;
        owned.push_back(o);
        st = to_device(c, src, n, false, &r, &ow);
        if (st != OVS_OK) { cleanup(); return st; }
        owned.push_back(r);
        st = to_device(c, siblings, n * (uint64_t)siblings_stride, false, &f, &ow);
        if (st != OVS_OK) { cleanup(); return st; }
        owned.push_back(f);
        if (lookup_node_ids) {
            st = to_device(c, reinterpret_cast<const K160*>(keys), n, false, &k, &ow);
            if (st != OVS_OK) { cleanup(); return st; }
            owned.push_back(k);
        }
        dout = o; dk = k; ds = r; dsib = f;
    }
    StatsDev* S = nullptr; uint32_t* counts = nullptr; double* partial = nullptr; double* result = nullptr;
    const bool okm = hipMalloc(&S, sizeof(StatsDev)) == hipSuccess &&
                     hipMalloc(&counts, sizeof(uint32_t) * 3 * c->n) == hipSuccess &&
                     hipMalloc(&partial, sizeof(double) * STATS_NODE_BLOCKS * NSTAT * 5) == hipSuccess &&
                     hipMalloc(&result, sizeof(double) * NSTAT * 5) == hipSuccess;
    owned.push_back(S); owned.push_back(counts); owned.push_back(partial); owned.push_back(result);
    if (!okm) { cleanup(); return fail(c, OVS_ENOMEM, "statistics scratch allocation failed"); }
    const int rates = measured_time_s >= 0.1;      // GlobalStatistics::MIN_MEASURED (KBRTestApp.cc:502)
    hipError_t e = launch_stats(dout, dk, ds, c->recs, n, (uint32_t)c->n, lookup_node_ids, measured_time_s, 0, rates,
                                S, counts, partial, result, c->num_cu, s, dsib ? dsib : src,
                                (uint64_t)siblings_stride);
    StatsDev h{};
    double r[NSTAT * 5];
    if (e == hipSuccess) e = hipMemcpyAsync(&h, S, sizeof h, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipMemcpyAsync(r, result, sizeof r, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    cleanup();
    if (e != hipSuccess) return hip_fail(c, e, "statistics kernels");

    ovs_kbrtest_lookup_stats& o = *stats;
    std::memset(&o, 0, sizeof o);
    o.num_sent = n;
    o.num_success = h.delivered;
    o.num_failed = h.dropped;
    o.num_invalid = h.failed;
    o.hop_count_sum = h.hop_sum;
    o.failed_hop_count_sum = h.fhop_sum;
    o.success_latency_sum_ns = (int64_t)h.lat_sum;
    if (h.delivered) {
        o.hop_count_min = (uint32_t)h.hop_min;
        o.hop_count_max = (uint32_t)h.hop_max;
        o.success_latency_min_ns = (int64_t)h.lat_min;
        o.success_latency_max_ns = (int64_t)h.lat_max;
        o.hop_count_mean = (double)h.hop_sum / (double)h.delivered;
        o.success_latency_mean_s = ((double)h.lat_sum / (double)h.delivered) * 1e-9;
    }
    if (h.dropped) o.failed_hop_count_mean = (double)h.fhop_sum / (double)h.dropped;
    if (n) o.total_latency_mean_s = ((double)h.lat_sum * 1e-9 + (double)h.dropped * failure_latency_s) / (double)n;
    for (int i = 0; i < 8; ++i) o.status_count[i] = h.status[i];
    for (int i = 0; i < 64; ++i) o.hop_hist[i] = h.hist[i];
    const int slot[3] = {0, 2, 4};
    ovs_stddev* sd[3] = {&o.successful_lookups_per_s, &o.failed_lookups_per_s, &o.success_ratio};
    for (int q = 0; q < 3; ++q) {
        const int k = slot[q];
        const double sum = r[k * 5 + 0], sq = r[k * 5 + 1];
        uint64_t cnt;
        std::memcpy(&cnt, &r[k * 5 + 4], sizeof cnt);
        ovs_stddev& d = *sd[q];
        d.count = cnt;
        if (!cnt) continue;
        d.mean = sum / (double)cnt;
        double var = 0.0;
        if (cnt > 1) {
            var = (sq - sum * sum / (double)cnt) / (double)(cnt - 1);
            if (var < 0) var = 0;
        }
        d.stddev = std::sqrt(var);
        d.min = r[k * 5 + 2];
        d.max = r[k * 5 + 3];
    }
    return OVS_OK;
}

ovs_status ovs_sync(ovs_ctx* c)
{
    if (!c) return OVS_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipDeviceSynchronize());
    return OVS_OK;
}

}  // extern "C"
