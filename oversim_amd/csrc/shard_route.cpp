// shard_route.cpp -- the multi-GPU round loop behind the C ABI (ovs_shard_route_batch,
// ovs_kad_shard_route_batch) and the exchanges it runs over (RCCL over xGMI; W in-process ranks).
//
// It replaces BaseOverlay::sendToKey's iterative branch (BaseOverlay.cc:1367-1442) for a network
// whose routing tables are split over the ranks.  One call routes one batch on one rank; every rank
// calls it collectively.  Per round (Chord):
//   1. the step kernel of each cohort (ovs_shard_step*: K1's shard instantiation + the atomic-free
//      compaction into per-destination segments) on the cohort's own stream;
//   2. the per-destination counts of every rank, all-gathered -- the round's one host
//      synchronisation, which also decides, identically on every rank, whether the cohort is done;
//   3. the all-to-allv of the 48 B records straight out of the segments into one receive buffer
//      (0xFF-filled first: a row nobody wrote finishes as a sentinel record the end check counts),
//      then the cohort's next step is queued behind it on the cohort stream, so one cohort's
//      exchange overlaps the other cohort's kernel.
// Kademlia one-way routes over replicated top buckets take the same loop with migrating lookup
// records (ovs_kad_shard_mig_step); otherwise (LookupCalls, no replicated buckets) the lookups stay
// home: step -> count all-gather -> requests all-to-allv -> serve -> responses all-to-allv (reverse
// splits) -> deliver.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "compact.hpp"
#include "ctx_internal.hpp"

using namespace ovs;

namespace {

thread_local std::string g_ex_err;

int ex_fail(const std::string& m)
{
    g_ex_err = m;
    return 1;
}

double now_ms()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ---------------------------------------------------------------------------
// cached device buffers of the loop (one set per context)

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
};

// grow to at least `bytes` (x1.25); the stream may still use the old buffer, so it drains first
hipError_t ensure(DevBuf& b, size_t bytes, hipStream_t s)
{
    if (bytes <= b.cap) return hipSuccess;
    hipError_t e;
    if (b.p) {
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        hipFree(b.p);
        b.p = nullptr;
        b.cap = 0;
    }
    const size_t want = bytes + bytes / 4 + 256;
    if ((e = hipMalloc(&b.p, want)) != hipSuccess) return e;
    b.cap = want;
    return hipSuccess;
}

struct CohortBufs {
    DevBuf out, recv, cnt;
    hipEvent_t e0 = nullptr, e1 = nullptr;
};

struct RouteScratch {
    CohortBufs coh[4];
    DevBuf done_cnt, sentinel;
    DevBuf kout, kcnt, kreq, kresp, kback;
    hipEvent_t ev = nullptr;
    std::vector<hipEvent_t> cev;
};

void release_scratch(void* p)
{
    RouteScratch* R = static_cast<RouteScratch*>(p);
    auto fr = [](DevBuf& b) { if (b.p) hipFree(b.p); b.p = nullptr; b.cap = 0; };
    for (CohortBufs& c : R->coh) {
        fr(c.out); fr(c.recv); fr(c.cnt);
        if (c.e0) hipEventDestroy(c.e0);
        if (c.e1) hipEventDestroy(c.e1);
    }
    fr(R->done_cnt); fr(R->sentinel); fr(R->kout); fr(R->kcnt); fr(R->kreq); fr(R->kresp); fr(R->kback);
    if (R->ev) hipEventDestroy(R->ev);
    for (hipEvent_t e : R->cev) hipEventDestroy(e);
    delete R;
}

RouteScratch* scratch(ovs_ctx* c)
{
    RouteScratch* R = static_cast<RouteScratch*>(ctx_route_scratch(c));
    if (!R) {
        R = new RouteScratch();
        ctx_set_route_scratch(c, R, release_scratch);
    }
    return R;
}

hipEvent_t mk_event(hipEvent_t* e, bool timing)
{
    if (!*e) hipEventCreateWithFlags(e, timing ? hipEventDefault : hipEventDisableTiming);
    return *e;
}

#define RCHK(expr)                                                                          \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess) return ctx_fail(c, OVS_EDEVICE, std::string(#expr) + ": " +   \
                                              hipGetErrorString(e_));                        \
    } while (0)

#define XCHK(call, what)                                                                    \
    do {                                                                                    \
        const double t_ = now_ms();                                                         \
        const int r_ = (call);                                                              \
        xms += now_ms() - t_;                                                               \
        if (r_ != 0) return ctx_fail(c, OVS_EDEVICE, std::string("exchange ") + (what) +    \
                                     " failed (" + std::to_string(r_) + ")" +               \
                                     (g_ex_err.empty() ? "" : ": " + g_ex_err));             \
    } while (0)

ovs_status check_exchange(ovs_ctx* c, const ovs_exchange* ex, const uint64_t* shard_lo)
{
    if (!ex || !ex->allgather_i64 || !ex->alltoallv || !ex->allreduce_sum_i64 || !shard_lo)
        return ctx_fail(c, OVS_EINVAL, "exchange callbacks and shard_lo are required");
    if (ex->world < 1 || ex->world > 64 || ex->rank >= ex->world)
        return ctx_fail(c, OVS_EINVAL, "exchange rank / world out of range (world 1..64)");
    return OVS_OK;
}

// A failure only one rank sees (an allocation, a step that did not launch, a segment or done-buffer
// overflow) must not leave the other ranks blocked in the next collective.  It is recorded here and
// carried by that collective -- a status slot of the count all-gather, or a term of check_totals' sum
// -- so every rank returns a failure from the same round.  (no early return between
// collectives.)
struct LocalErr {
    ovs_status st = OVS_OK;
    std::string msg;
    void set(ovs_status s, const std::string& m)
    {
        if (st == OVS_OK) { st = s; msg = m; }
    }
    void hip(hipError_t e, const char* what)
    {
        if (e != hipSuccess) set(OVS_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
    }
    bool ok() const { return st == OVS_OK; }
};

// the collective every rank is in (read by a caller's watchdog through ovs_exchange_stage)
std::atomic<const char*> g_stage{"idle"};
std::atomic<uint32_t> g_stage_round{0};

void stage(const char* s, uint32_t round)
{
    g_stage_round.store(round, std::memory_order_relaxed);
    g_stage.store(s, std::memory_order_release);
}

// after a gathered status slot: every rank fails when any did (its own message, or the failing rank)
ovs_status gathered_failure(ovs_ctx* c, const LocalErr& le, const int64_t* M, uint32_t W, uint32_t stride,
                            uint32_t slot, const char* what)
{
    int first = -1, nfail = 0;
    for (uint32_t r = 0; r < W; ++r)
        if (M[(size_t)r * stride + slot] != 0) { if (first < 0) first = (int)r; ++nfail; }
    if (nfail == 0) return OVS_OK;
    if (!le.ok()) return ctx_fail(c, le.st, std::string(what) + ": " + le.msg);
    return ctx_fail(c, (ovs_status)M[(size_t)first * stride + slot],
                    std::string(what) + ": rank " + std::to_string(first) + " failed (" + std::to_string(nfail) +
                        " rank(s)); its error names the cause");
}

// the batch is complete on every rank: finished records (all ranks) == lookups started (all ranks);
// a local failure on any rank fails all of them here
ovs_status check_totals(ovs_ctx* c, const ovs_exchange* ex, int64_t have, int64_t want, int64_t sentinel,
                        const LocalErr& le, double& xms, const char* what)
{
    int64_t v[4] = {have, want, sentinel, le.ok() ? 0 : 1};
    stage("completeness allreduce", 0);
    XCHK(ex->allreduce_sum_i64(ex->user, v, 4), "allreduce");
    if (v[3] != 0) {
        if (!le.ok()) return ctx_fail(c, le.st, std::string(what) + ": " + le.msg);
        return ctx_fail(c, OVS_EDEVICE, std::string(what) + ": " + std::to_string(v[3]) +
                                            " other rank(s) failed; their errors name the cause");
    }
    if (v[2] != 0)
        return ctx_fail(c, OVS_EDEVICE, std::string(what) + ": " + std::to_string(v[2]) +
                                            " finished records came from exchange rows nobody wrote");
    if (v[0] != v[1])
        return ctx_fail(c, OVS_EDEVICE, std::string(what) + ": " + std::to_string(v[0]) + " finished records for " +
                                            std::to_string(v[1]) + " lookups");
    return OVS_OK;
}

}  // namespace

// ===========================================================================

namespace {

// the record loop of a batch whose lookups move between ranks (Chord hand-offs, Kademlia migration):
// step(k, first, in, nin, b0, out, cap, cnt, stream) runs one round of cohort k -- a batch's first
// round from keys[b0, b0 + nin) (first = true), else over nin received records -- appending
// hand-offs to segment d of out and finished lookups to done (the shared counter dcnt)
template <class Step>
ovs_status route_records(ovs_ctx* c, const ovs_exchange* ex, uint64_t n, uint32_t RB, const Step& step,
                         ovs_done_rec* done, uint64_t done_cap, uint64_t* n_done, uint32_t cohorts,
                         ovs_shard_route_stats* stats, void* stream, const char* what)
{
    const double t_start = now_ms();
    double xms = 0, kms = 0;
    const uint32_t W = ex->world, me = ex->rank;
    // the cohort count must be the same on every rank (every cohort takes part in every round's
    // collectives until the gathered counts say it is done everywhere): not derived from n
    const int nc = cohorts == 0 ? 2 : (int)std::min<uint32_t>(cohorts, 4);
    // a cohort's all-gather row: [0, W) records for each destination, W = this rank's status
    // (LocalErr), W + 1 = its receive buffer's capacity in rows
    const uint32_t SW = W + 2, SLOT_ST = W, SLOT_CAP = W + 1;
    LocalErr le;
    RCHK(hipSetDevice(ctx_device(c)));
    RouteScratch* R = scratch(c);
    hipStream_t s0 = (hipStream_t)stream;
    hipStream_t cs[4];
    for (int k = 0; k < nc; ++k) {
        cs[k] = ctx_cohort_stream(c, k);
        if (!cs[k]) le.set(OVS_EDEVICE, "cohort stream");
    }
    unsigned long long* dcnt = nullptr;
    if (le.ok()) {
        le.hip(ensure(R->done_cnt, sizeof(unsigned long long), s0), "done counter");
        if (le.ok()) {
            dcnt = static_cast<unsigned long long*>(R->done_cnt.p);
            le.hip(hipMemsetAsync(dcnt, 0, sizeof(unsigned long long), s0), "done counter reset");
        }
        // every cohort stream starts after the caller's stream (inputs, the counter reset)
        if (le.ok()) le.hip(hipEventRecord(mk_event(&R->ev, false), s0), "start event");
    }
    uint64_t nin[4] = {0, 0, 0, 0}, cap[4] = {0, 0, 0, 0};
    bool live[4] = {false, false, false, false};
    std::vector<int64_t> M((size_t)W * SW);
    std::vector<uint64_t> scl(W), rcl(W), roff(W);
    std::vector<const void*> sendp(W);
    uint64_t sent = 0, sent_bytes = 0;
    // queue one round of cohort k; a failure is recorded, not returned (the cohort's next all-gather
    // carries it)
    auto issue = [&](int k, bool first, uint64_t b0) {
        if (!le.ok()) return;
        CohortBufs& B = R->coh[k];
        // a segment receives at most the step's input records
        cap[k] = std::max<uint64_t>(nin[k], 1);
        if (ensure(B.out, (size_t)W * cap[k] * RB, cs[k]) != hipSuccess ||
            ensure(B.cnt, sizeof(unsigned long long) * W, cs[k]) != hipSuccess) {
            le.set(OVS_ENOMEM, "shard route: segment allocation");
            return;
        }
        cap[k] = B.out.cap / ((size_t)W * RB);
        le.hip(hipMemsetAsync(B.cnt.p, 0, sizeof(unsigned long long) * W, cs[k]), "count reset");
        if (le.ok()) le.hip(hipEventRecord(mk_event(&B.e0, true), cs[k]), "step event");
        if (!le.ok()) return;
        const ovs_status st = step(k, first, first ? nullptr : B.recv.p, nin[k], b0, B.out.p, cap[k],
                                   static_cast<unsigned long long*>(B.cnt.p), dcnt, cs[k]);
        if (st != OVS_OK) { le.set(st, ovs_last_error(c)); return; }
        le.hip(hipEventRecord(mk_event(&B.e1, true), cs[k]), "step event");
    };
    for (int k = 0; k < nc; ++k) {
        if (le.ok()) le.hip(hipStreamWaitEvent(cs[k], R->ev, 0), "cohort start");
        const uint64_t b0 = (uint64_t)k * n / nc, b1 = (uint64_t)(k + 1) * n / nc;
        nin[k] = b1 - b0;
        live[k] = true;
        issue(k, true, b0);
    }
    uint32_t rounds = 1;
    std::vector<int64_t> hc(SW);
    while (true) {
        bool any = false;
        for (int k = 0; k < nc; ++k) {
            if (!live[k]) continue;
            CohortBufs& B = R->coh[k];
            // this cohort's counts on the host (waits for its step), then every rank's
            std::fill(hc.begin(), hc.end(), 0);
            if (le.ok()) {
                le.hip(hipMemcpyAsync(hc.data(), B.cnt.p, sizeof(int64_t) * W, hipMemcpyDeviceToHost, cs[k]), "counts");
                if (le.ok()) le.hip(hipStreamSynchronize(cs[k]), "cohort step");
                float ms = 0;
                if (le.ok() && hipEventElapsedTime(&ms, B.e0, B.e1) == hipSuccess) kms += ms;
                for (uint32_t r = 0; r < W && le.ok(); ++r)
                    if ((uint64_t)hc[r] > cap[k]) le.set(OVS_EDEVICE, "shard route: a segment overflowed");
                if (!le.ok()) std::fill(hc.begin(), hc.end(), 0);
            }
            hc[SLOT_ST] = le.st;
            hc[SLOT_CAP] = (int64_t)(B.recv.cap / RB);
            stage("count allgather", rounds);
            XCHK(ex->allgather_i64(ex->user, hc.data(), SW, M.data()), "allgather");
            const ovs_status gf = gathered_failure(c, le, M.data(), W, SW, SLOT_ST, what);
            if (gf != OVS_OK) return gf;
            int64_t tot = 0;
            for (uint32_t r = 0; r < W; ++r)
                for (uint32_t d = 0; d < W; ++d) tot += M[(size_t)r * SW + d];
            if (tot == 0) { live[k] = false; continue; }
            any = true;
            // receive buffers: every rank sees which ones must grow; if any, one allreduce tells all
            // ranks whether every allocation succeeded before anyone enters the all-to-allv
            bool grow = false;
            uint64_t tin = 0;
            for (uint32_t r = 0; r < W; ++r) {
                uint64_t in_r = 0;
                for (uint32_t s = 0; s < W; ++s) in_r += (uint64_t)M[(size_t)s * SW + r];
                if (in_r > (uint64_t)M[(size_t)r * SW + SLOT_CAP]) grow = true;
                if (r == me) tin = in_r;
            }
            if (grow) {
                int64_t bad[1] = {ensure(B.recv, std::max<size_t>((size_t)tin * RB, RB), cs[k]) != hipSuccess ? 1 : 0};
                stage("buffer allreduce", rounds);
                XCHK(ex->allreduce_sum_i64(ex->user, bad, 1), "allreduce");
                if (bad[0] != 0) return ctx_fail(c, OVS_ENOMEM, std::string(what) + ": receive buffer allocation failed on " +
                                                                   std::to_string(bad[0]) + " rank(s)");
            }
            uint64_t off = 0;
            for (uint32_t r = 0; r < W; ++r) {
                scl[r] = (uint64_t)M[(size_t)me * SW + r];
                rcl[r] = (uint64_t)M[(size_t)r * SW + me];
                roff[r] = off;
                off += rcl[r];
                if (r != me) { sent += scl[r]; sent_bytes += scl[r] * RB; }
                sendp[r] = static_cast<const uint8_t*>(B.out.p) + (size_t)r * cap[k] * RB;
            }
            // sentinel: a row the exchange never writes reads as an impossible record
            le.hip(hipMemsetAsync(B.recv.p, 0xFF, (size_t)tin * RB, cs[k]), "receive sentinel");
            stage("records alltoallv", rounds);
            XCHK(ex->alltoallv(ex->user, sendp.data(), scl.data(), B.recv.p, roff.data(), rcl.data(), RB, cs[k]),
                 "alltoallv");
            nin[k] = tin;
            issue(k, false, 0);
        }
        if (!any) break;
        if (++rounds > 10000) {
            // every rank counts the same rounds: all stop here
            return ctx_fail(c, OVS_EDEVICE, std::string(what) + " did not terminate");
        }
    }
    // the caller's stream continues after every cohort
    R->cev.resize(std::max<size_t>(R->cev.size(), (size_t)nc), nullptr);
    for (int k = 0; k < nc && le.ok(); ++k) {
        le.hip(hipEventRecord(mk_event(&R->cev[k], false), cs[k]), "cohort end event");
        if (le.ok()) le.hip(hipStreamWaitEvent(s0, R->cev[k], 0), "cohort join");
    }
    unsigned long long hd = 0, hs = 0;
    if (le.ok()) {
        le.hip(hipMemcpyAsync(&hd, dcnt, sizeof hd, hipMemcpyDeviceToHost, s0), "done count");
        if (le.ok()) le.hip(hipStreamSynchronize(s0), "done count");
    }
    if (le.ok() && hd > done_cap)
        le.set(OVS_EINVAL, "done buffer overflow (done_cap " + std::to_string(done_cap) + " < " + std::to_string(hd) +
                               " finished records)");
    if (le.ok()) {
        le.hip(ensure(R->sentinel, sizeof(unsigned long long), s0), "sentinel counter");
        if (le.ok())
            le.hip(count_sentinel_records(done, hd, static_cast<unsigned long long*>(R->sentinel.p), s0), "sentinel count");
        if (le.ok()) le.hip(hipMemcpyAsync(&hs, R->sentinel.p, sizeof hs, hipMemcpyDeviceToHost, s0), "sentinel count");
        if (le.ok()) le.hip(hipStreamSynchronize(s0), "sentinel count");
    }
    const ovs_status st = check_totals(c, ex, (int64_t)hd, (int64_t)n, (int64_t)hs, le, xms, what);
    stage("idle", 0);
    if (st != OVS_OK) return st;
    *n_done = hd;
    if (stats) {
        stats->rounds = rounds;
        stats->cohorts = (uint32_t)nc;
        stats->sent = sent;
        stats->sent_bytes = sent_bytes;
        stats->done = hd;
        stats->step_ms = kms;
        stats->exchange_ms = xms;
        stats->total_ms = now_ms() - t_start;
    }
    return OVS_OK;
}

}  // namespace

extern "C" {

ovs_status ovs_shard_route_batch(ovs_ctx* c, const ovs_exchange* ex, const uint64_t* shard_lo, int32_t num_siblings,
                                 const ovs_key160* keys, const uint32_t* src, uint64_t n, uint32_t qid_base,
                                 ovs_done_rec* done, uint64_t done_cap, uint64_t* n_done, uint32_t cohorts,
                                 ovs_shard_route_stats* stats, void* stream)
{
    if (!c || !n_done || (n && (!keys || !src)) || !done) return OVS_EINVAL;
    ovs_status st = check_exchange(c, ex, shard_lo);
    if (st != OVS_OK) return st;
    const uint32_t W = ex->world;
    const int32_t ns = num_siblings;
    auto step = [&](int, bool first, const void* in, uint64_t nin, uint64_t b0, void* out, uint64_t cap,
                    unsigned long long* cnt, unsigned long long* dcnt, hipStream_t s) -> ovs_status {
        auto* o = static_cast<ovs_lookup_rec*>(out);
        if (first)
            return ovs_shard_step_keys(c, ns, keys + b0, src + b0, nin, qid_base + (uint32_t)b0, o, cap, cnt, done,
                                       done_cap, dcnt, shard_lo, W, s);
        const auto* r = static_cast<const ovs_lookup_rec*>(in);
        if (ns == 0) return ovs_shard_step(c, r, nin, o, cap, cnt, done, done_cap, dcnt, shard_lo, W, s);
        return ovs_shard_step_lookup(c, ns, r, nin, o, cap, cnt, done, done_cap, dcnt, shard_lo, W, s);
    };
    return route_records(c, ex, n, (uint32_t)sizeof(ovs_lookup_rec), step, done, done_cap, n_done, cohorts,
                         stats, stream, "sharded Chord");
}

ovs_status ovs_kad_shard_route_batch(ovs_ctx* c, const ovs_exchange* ex, const uint64_t* shard_lo,
                                     int32_t num_siblings, const ovs_key160* keys, const uint32_t* src, uint64_t n,
                                     uint32_t qid_base, ovs_done_rec* done, uint64_t done_cap, uint64_t* n_done,
                                     uint32_t* siblings, ovs_shard_route_stats* stats, void* stream)
{
    if (!c || !n_done || (n && (!keys || !src)) || !done) return OVS_EINVAL;
    ovs_status st = check_exchange(c, ex, shard_lo);
    if (st != OVS_OK) return st;
    if (num_siblings < -1 && ovs_kad_shard_levels(c) > 0) {
        // one-way routes over replicated top buckets: the lookups migrate (ovs_kad_shard_mig_step)
        const int32_t rb = ovs_kad_shard_rec_bytes(c);
        if (rb <= 0) return ctx_fail(c, OVS_ESTATE, "no Kademlia network loaded");
        const uint32_t W = ex->world;
        auto step = [&](int, bool first, const void* in, uint64_t nin, uint64_t b0, void* out, uint64_t cap,
                        unsigned long long* cnt, unsigned long long* dcnt, hipStream_t s) -> ovs_status {
            return kad_mig_step_impl(c, first ? nullptr : in, nin, first ? keys + b0 : nullptr,
                                     first ? src + b0 : nullptr, qid_base + (uint32_t)b0, out, cap, cnt, done, done_cap,
                                     dcnt, shard_lo, W, s, false);
        };
        // the error count starts once per batch, before any cohort's first step (the cohort streams
        // wait for the caller's stream)
        if ((st = kad_shard_reset_errors(c, stream)) != OVS_OK) return st;
        // two cohorts (OVS_KAD_MIG_COHORTS): one cohort's records are exchanged while the other's
        // step runs, as for Chord
        static const uint32_t mig_cohorts = [] {
            const char* e = std::getenv("OVS_KAD_MIG_COHORTS");
            const int v = e ? std::atoi(e) : 2;
            return (uint32_t)std::max(1, std::min(v, 4));
        }();
        st = route_records(c, ex, n, (uint32_t)rb, step, done, done_cap, n_done, mig_cohorts, stats, stream,
                           "sharded Kademlia (migration)");
        if (st != OVS_OK) return st;
        uint64_t bad = 0;
        LocalErr le;
        const ovs_status es = ovs_kad_shard_errors(c, &bad);
        if (es != OVS_OK) le.set(es, ovs_last_error(c));
        int64_t v[2] = {(int64_t)bad, le.ok() ? 0 : 1};
        double xms = 0;
        stage("error allreduce", 0);
        XCHK(ex->allreduce_sum_i64(ex->user, v, 2), "allreduce");
        stage("idle", 0);
        if (stats) stats->exchange_ms += xms;
        if (!le.ok()) return ctx_fail(c, le.st, le.msg);
        if (v[1] != 0) return ctx_fail(c, OVS_EDEVICE, "sharded Kademlia (migration): another rank failed");
        if (v[0] != 0)
            return ctx_fail(c, OVS_EDEVICE, std::to_string(v[0]) + " Kademlia shard errors (table reads off an arc)");
        return OVS_OK;
    }
    const double t_start = now_ms();
    double xms = 0, kms = 0;
    const uint32_t W = ex->world, me = ex->rank;
    // local failures ride the next collective (LocalErr): preconditions that depend on this rank's
    // own batch, allocations, launches
    LocalErr le;
    if (done_cap < n) le.set(OVS_EINVAL, "done_cap must hold the batch (Kademlia lookups finish at home)");
    RCHK(hipSetDevice(ctx_device(c)));
    RouteScratch* R = scratch(c);
    hipStream_t s = (hipStream_t)stream;
    ovs_params P;
    if ((st = ovs_get_params(c, &P)) != OVS_OK) return st;
    if (le.ok()) {
        if (num_siblings >= -1) st = ovs_kad_shard_begin_lookup(c, num_siblings, keys, src, n, qid_base, siblings, stream);
        else st = ovs_kad_shard_begin(c, keys, src, n, qid_base, stream);
        if (st != OVS_OK) le.set(st, ovs_last_error(c));
    }
    const int rb = ovs_kad_shard_resp_bytes(c);
    if (rb <= 0) return ctx_fail(c, OVS_ESTATE, "no Kademlia network loaded");
    const uint32_t RB = (uint32_t)rb, QB = sizeof(ovs_kad_req);
    // one round sends at most one request per pending-call slot of every lookup
    const uint64_t slots = P.lookupParallelRpcs <= 4 ? (uint64_t)P.lookupParallelRpcs : 8;
    const uint64_t seg = std::max<uint64_t>(n * slots, 1);
    if (le.ok() && (ensure(R->kout, (size_t)W * seg * QB, s) != hipSuccess ||
                    ensure(R->kcnt, sizeof(unsigned long long) * (W + 2), s) != hipSuccess))
        le.set(OVS_ENOMEM, "kademlia shard route: buffers");
    auto* cnt = static_cast<unsigned long long*>(R->kcnt.p);
    if (le.ok()) le.hip(hipMemsetAsync(cnt, 0, sizeof(unsigned long long) * (W + 2), s), "counter reset");
    hipEvent_t e0 = nullptr, e1 = nullptr;
    RCHK(hipEventCreate(&e0));
    RCHK(hipEventCreate(&e1));
    struct EvFree { hipEvent_t a, b; ~EvFree() { hipEventDestroy(a); hipEventDestroy(b); } } evf{e0, e1};
    // all-gather row: [0, W) requests to each rank, W = lookups still active here, W + 1 = status,
    // W + 2 = request/response rows the receive buffers hold, W + 3 = rows the response buffer holds
    const uint32_t SW = W + 4, SLOT_ACT = W, SLOT_ST = W + 1, SLOT_CIN = W + 2, SLOT_CBK = W + 3;
    std::vector<int64_t> M((size_t)W * SW), hc(SW);
    std::vector<uint64_t> scl(W), rcl(W), roff(W), boff(W);
    std::vector<const void*> sendp(W), backp(W);
    uint64_t sent = 0, sent_bytes = 0;
    uint32_t rounds = 0;
    auto rows = [](const DevBuf& b, uint32_t row) { return (int64_t)(b.cap / row); };
    while (true) {
        if (++rounds > 5000) return ctx_fail(c, OVS_EDEVICE, "sharded Kademlia routing did not terminate");
        std::fill(hc.begin(), hc.end(), 0);
        if (le.ok()) {
            le.hip(hipMemsetAsync(cnt, 0, sizeof(unsigned long long) * W, s), "counter reset");
            if (le.ok()) le.hip(hipEventRecord(e0, s), "step event");
            if (le.ok()) {
                st = ovs_kad_shard_step(c, static_cast<ovs_kad_req*>(R->kout.p), seg, cnt, done, done_cap, cnt + W + 1,
                                        cnt + W, shard_lo, W, stream);
                if (st != OVS_OK) le.set(st, ovs_last_error(c));
            }
            if (le.ok()) le.hip(hipEventRecord(e1, s), "step event");
            if (le.ok()) le.hip(hipMemcpyAsync(hc.data(), cnt, sizeof(int64_t) * (W + 1), hipMemcpyDeviceToHost, s), "counts");
            if (le.ok()) le.hip(hipStreamSynchronize(s), "step");
            float ms = 0;
            if (le.ok() && hipEventElapsedTime(&ms, e0, e1) == hipSuccess) kms += ms;
            if (!le.ok()) std::fill(hc.begin(), hc.end(), 0);
        }
        hc[SLOT_ST] = le.st;
        hc[SLOT_CIN] = std::min(rows(R->kreq, QB), rows(R->kresp, RB));
        hc[SLOT_CBK] = rows(R->kback, RB);
        // M[r, d] requests r -> d, M[r, W] lookups still active on r
        stage("request-count allgather", rounds);
        XCHK(ex->allgather_i64(ex->user, hc.data(), SW, M.data()), "allgather");
        const ovs_status gf = gathered_failure(c, le, M.data(), W, SW, SLOT_ST, "sharded Kademlia");
        if (gf != OVS_OK) return gf;
        int64_t tot = 0;
        for (uint32_t r = 0; r < W; ++r)
            for (uint32_t d = 0; d <= W; ++d) tot += M[(size_t)r * SW + d];
        if (tot == 0) break;
        // buffer growth decided identically on every rank (see route_records)
        bool grow = false;
        uint64_t tin = 0, tback = 0;
        for (uint32_t r = 0; r < W; ++r) {
            uint64_t in_r = 0, back_r = 0;
            for (uint32_t q = 0; q < W; ++q) {
                in_r += (uint64_t)M[(size_t)q * SW + r];
                back_r += (uint64_t)M[(size_t)r * SW + q];
            }
            if (in_r > (uint64_t)M[(size_t)r * SW + SLOT_CIN] || back_r > (uint64_t)M[(size_t)r * SW + SLOT_CBK]) grow = true;
            if (r == me) { tin = in_r; tback = back_r; }
        }
        if (grow) {
            int64_t bad[1] = {(ensure(R->kreq, std::max<size_t>((size_t)tin * QB, QB), s) != hipSuccess ||
                               ensure(R->kresp, std::max<size_t>((size_t)tin * RB, RB), s) != hipSuccess ||
                               ensure(R->kback, std::max<size_t>((size_t)tback * RB, RB), s) != hipSuccess) ? 1 : 0};
            stage("buffer allreduce", rounds);
            XCHK(ex->allreduce_sum_i64(ex->user, bad, 1), "allreduce");
            if (bad[0] != 0)
                return ctx_fail(c, OVS_ENOMEM, "kademlia shard route: exchange buffers failed on " + std::to_string(bad[0]) +
                                                   " rank(s)");
        }
        uint64_t oin = 0, oback = 0;
        for (uint32_t r = 0; r < W; ++r) {
            scl[r] = (uint64_t)M[(size_t)me * SW + r];
            rcl[r] = (uint64_t)M[(size_t)r * SW + me];
            roff[r] = oin; oin += rcl[r];
            boff[r] = oback; oback += scl[r];
            if (r != me) { sent += scl[r]; sent_bytes += scl[r] * (QB + RB); }
            sendp[r] = static_cast<const uint8_t*>(R->kout.p) + (size_t)r * seg * QB;
        }
        // requests to the responders' owners (0xFF-filled: a request nobody wrote is refused by serve)
        le.hip(hipMemsetAsync(R->kreq.p, 0xFF, (size_t)tin * QB, s), "request sentinel");
        stage("request alltoallv", rounds);
        XCHK(ex->alltoallv(ex->user, sendp.data(), scl.data(), R->kreq.p, roff.data(), rcl.data(), QB, stream),
             "alltoallv (requests)");
        if (le.ok()) {
            st = ovs_kad_shard_serve(c, static_cast<const ovs_kad_req*>(R->kreq.p), tin, R->kresp.p, stream);
            if (st != OVS_OK) le.set(st, ovs_last_error(c));
        }
        // a rank whose serve failed still answers (0xFF rows: unknown tags, deliver counts them as
        // errors), so nobody waits; the failure is gathered next round
        if (!le.ok()) le.hip(hipMemsetAsync(R->kresp.p, 0xFF, (size_t)tin * RB, s), "response sentinel");
        // the responses back with the reverse splits (a response nobody wrote has an unknown tag:
        // deliver counts it as an error)
        for (uint32_t r = 0; r < W; ++r) backp[r] = static_cast<const uint8_t*>(R->kresp.p) + (size_t)roff[r] * RB;
        le.hip(hipMemsetAsync(R->kback.p, 0xFF, (size_t)tback * RB, s), "response buffer sentinel");
        stage("response alltoallv", rounds);
        XCHK(ex->alltoallv(ex->user, backp.data(), rcl.data(), R->kback.p, boff.data(), scl.data(), RB, stream),
             "alltoallv (responses)");
        if (le.ok()) {
            st = ovs_kad_shard_deliver(c, R->kback.p, tback, stream);
            if (st != OVS_OK) le.set(st, ovs_last_error(c));
        }
    }
    unsigned long long hd = 0;
    le.hip(hipMemcpyAsync(&hd, cnt + W + 1, sizeof hd, hipMemcpyDeviceToHost, s), "done count");
    if (le.ok()) le.hip(hipStreamSynchronize(s), "done count");
    uint64_t bad = 0;
    if (le.ok()) {
        const ovs_status es = ovs_kad_shard_errors(c, &bad);
        if (es != OVS_OK) le.set(es, ovs_last_error(c));
    }
    if (le.ok() && hd > done_cap) le.set(OVS_EINVAL, "done buffer overflow");
    // every rank finishes exactly its own lookups; errors (undeliverable responses, reads off the arc,
    // sources off the arc, local failures) fail the batch on every rank
    int64_t v[3] = {(int64_t)hd == (int64_t)n ? 0 : 1, (int64_t)bad, le.ok() ? 0 : 1};
    stage("completeness allreduce", 0);
    XCHK(ex->allreduce_sum_i64(ex->user, v, 3), "allreduce");
    stage("idle", 0);
    if (!le.ok()) return ctx_fail(c, le.st, "sharded Kademlia: " + le.msg);
    if (v[2] != 0) return ctx_fail(c, OVS_EDEVICE, "sharded Kademlia: " + std::to_string(v[2]) + " other rank(s) failed");
    if (v[1] != 0)
        return ctx_fail(c, OVS_EDEVICE, std::to_string(v[1]) + " Kademlia shard errors: responses that could not be "
                                        "delivered, table reads off an arc, or sources off their rank's arc");
    if (v[0] != 0)
        return ctx_fail(c, OVS_EDEVICE, "sharded Kademlia: " + std::to_string(hd) + " finished records for " +
                                            std::to_string(n) + " lookups on this rank (or another rank incomplete)");
    *n_done = hd;
    if (stats) {
        stats->rounds = rounds;
        stats->cohorts = 1;
        stats->sent = sent;
        stats->sent_bytes = sent_bytes;
        stats->done = hd;
        stats->step_ms = kms;
        stats->exchange_ms = xms;
        stats->total_ms = now_ms() - t_start;
    }
    return OVS_OK;
}

}  // extern "C"

// ===========================================================================
// RCCL exchange (loaded at run time: the process's librccl.so.1 when one is mapped -- PyTorch's --
// else /opt/rocm's; either resolves libamdhip64 to the runtime already loaded)

namespace {

struct RcclFns {
    ncclResult_t (*GetUniqueId)(ncclUniqueId*);
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int);
    ncclResult_t (*CommDestroy)(ncclComm_t);
    ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
    ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
    ncclResult_t (*GroupStart)();
    ncclResult_t (*GroupEnd)();
    const char* (*GetErrorString)(ncclResult_t);
};

std::mutex g_rccl_mu;
RcclFns g_rccl{};
bool g_rccl_ok = false;

bool load_rccl()
{
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    if (g_rccl_ok) return true;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) { ex_fail(std::string("cannot load librccl.so.1: ") + dlerror()); return false; }
    bool ok = true;
    auto sym = [&](const char* name) {
        void* p = dlsym(h, name);
        if (!p) { ok = false; ex_fail(std::string("librccl: missing ") + name); }
        return p;
    };
    g_rccl.GetUniqueId = reinterpret_cast<decltype(g_rccl.GetUniqueId)>(sym("ncclGetUniqueId"));
    g_rccl.CommInitRank = reinterpret_cast<decltype(g_rccl.CommInitRank)>(sym("ncclCommInitRank"));
    g_rccl.CommDestroy = reinterpret_cast<decltype(g_rccl.CommDestroy)>(sym("ncclCommDestroy"));
    g_rccl.AllGather = reinterpret_cast<decltype(g_rccl.AllGather)>(sym("ncclAllGather"));
    g_rccl.AllReduce = reinterpret_cast<decltype(g_rccl.AllReduce)>(sym("ncclAllReduce"));
    g_rccl.Send = reinterpret_cast<decltype(g_rccl.Send)>(sym("ncclSend"));
    g_rccl.Recv = reinterpret_cast<decltype(g_rccl.Recv)>(sym("ncclRecv"));
    g_rccl.GroupStart = reinterpret_cast<decltype(g_rccl.GroupStart)>(sym("ncclGroupStart"));
    g_rccl.GroupEnd = reinterpret_cast<decltype(g_rccl.GroupEnd)>(sym("ncclGroupEnd"));
    g_rccl.GetErrorString = reinterpret_cast<decltype(g_rccl.GetErrorString)>(sym("ncclGetErrorString"));
    g_rccl_ok = ok;
    return ok;
}

int nccl_fail(ncclResult_t r, const char* what)
{
    return ex_fail(std::string(what) + ": " + (g_rccl.GetErrorString ? g_rccl.GetErrorString(r) : "rccl error"));
}

#define NCHK(expr, what)                                    \
    do {                                                    \
        ncclResult_t r_ = (expr);                           \
        if (r_ != ncclSuccess) return nccl_fail(r_, what);  \
    } while (0)
#define HCHK(expr)                                                                          \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess) return ex_fail(std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

// rows of an all-to-allv go out in pieces of at most 256 MB; both sides cut a transfer the same
// way and RCCL matches the point-to-point messages between two ranks in order
constexpr size_t RCCL_CHUNK = 256ull << 20;

struct RcclEx {
    ncclComm_t comm = nullptr;
    int device = 0;
    uint32_t rank = 0, world = 1;
    hipStream_t cs = nullptr;          // the communicator stream: every collective, in issue order
    hipEvent_t ev_in = nullptr, ev_out = nullptr;
    int64_t* dbuf = nullptr;           // all-gather / all-reduce staging (device)
    size_t dcap = 0;
    int64_t* hpin = nullptr;           // ... and its pinned host side
    size_t hcap = 0;
};

int rccl_stage(RcclEx* X, size_t elems)
{
    if (elems <= X->dcap) return 0;
    if (X->dbuf) hipFree(X->dbuf);
    if (X->hpin) hipHostFree(X->hpin);
    X->dbuf = nullptr; X->hpin = nullptr; X->dcap = X->hcap = 0;
    HCHK(hipMalloc(&X->dbuf, sizeof(int64_t) * elems));
    HCHK(hipHostMalloc(reinterpret_cast<void**>(&X->hpin), sizeof(int64_t) * elems, hipHostMallocDefault));
    X->dcap = X->hcap = elems;
    return 0;
}

int rccl_allgather(void* user, const int64_t* host_send, uint32_t n, int64_t* host_recv)
{
    RcclEx* X = static_cast<RcclEx*>(user);
    HCHK(hipSetDevice(X->device));
    const size_t tot = (size_t)n * X->world;
    if (rccl_stage(X, tot + n)) return 1;
    int64_t* dsend = X->dbuf + tot;
    std::memcpy(X->hpin + tot, host_send, sizeof(int64_t) * n);
    HCHK(hipMemcpyAsync(dsend, X->hpin + tot, sizeof(int64_t) * n, hipMemcpyHostToDevice, X->cs));
    NCHK(g_rccl.AllGather(dsend, X->dbuf, n, ncclInt64, X->comm, X->cs), "ncclAllGather");
    HCHK(hipMemcpyAsync(X->hpin, X->dbuf, sizeof(int64_t) * tot, hipMemcpyDeviceToHost, X->cs));
    HCHK(hipStreamSynchronize(X->cs));
    std::memcpy(host_recv, X->hpin, sizeof(int64_t) * tot);
    return 0;
}

int rccl_allreduce(void* user, int64_t* values, uint32_t n)
{
    RcclEx* X = static_cast<RcclEx*>(user);
    HCHK(hipSetDevice(X->device));
    if (rccl_stage(X, n)) return 1;
    std::memcpy(X->hpin, values, sizeof(int64_t) * n);
    HCHK(hipMemcpyAsync(X->dbuf, X->hpin, sizeof(int64_t) * n, hipMemcpyHostToDevice, X->cs));
    NCHK(g_rccl.AllReduce(X->dbuf, X->dbuf, n, ncclInt64, ncclSum, X->comm, X->cs), "ncclAllReduce");
    HCHK(hipMemcpyAsync(X->hpin, X->dbuf, sizeof(int64_t) * n, hipMemcpyDeviceToHost, X->cs));
    HCHK(hipStreamSynchronize(X->cs));
    std::memcpy(values, X->hpin, sizeof(int64_t) * n);
    return 0;
}

int rccl_alltoallv(void* user, const void* const* send, const uint64_t* send_rows, void* recv, const uint64_t* recv_off,
                   const uint64_t* recv_rows, uint32_t row_bytes, void* stream)
{
    RcclEx* X = static_cast<RcclEx*>(user);
    HCHK(hipSetDevice(X->device));
    hipStream_t s = (hipStream_t)stream;
    // the communicator stream waits for the segments (written on `stream`), and `stream` for the transfer
    HCHK(hipEventRecord(X->ev_in, s));
    HCHK(hipStreamWaitEvent(X->cs, X->ev_in, 0));
    uint8_t* rb = static_cast<uint8_t*>(recv);
    const uint32_t me = X->rank;
    if (send_rows[me] != recv_rows[me]) return ex_fail("alltoallv: own share differs");
    if (send_rows[me])
        HCHK(hipMemcpyAsync(rb + recv_off[me] * row_bytes, send[me], send_rows[me] * row_bytes, hipMemcpyDeviceToDevice,
                            X->cs));
    NCHK(g_rccl.GroupStart(), "ncclGroupStart");
    for (uint32_t p = 0; p < X->world; ++p) {
        if (p == me) continue;
        const size_t sb = send_rows[p] * row_bytes, rbytes = recv_rows[p] * row_bytes;
        for (size_t o = 0; o < sb; o += RCCL_CHUNK)
            NCHK(g_rccl.Send(static_cast<const uint8_t*>(send[p]) + o, std::min(RCCL_CHUNK, sb - o), ncclUint8, (int)p,
                             X->comm, X->cs), "ncclSend");
        for (size_t o = 0; o < rbytes; o += RCCL_CHUNK)
            NCHK(g_rccl.Recv(rb + recv_off[p] * row_bytes + o, std::min(RCCL_CHUNK, rbytes - o), ncclUint8, (int)p,
                             X->comm, X->cs), "ncclRecv");
    }
    NCHK(g_rccl.GroupEnd(), "ncclGroupEnd");
    HCHK(hipEventRecord(X->ev_out, X->cs));
    HCHK(hipStreamWaitEvent(s, X->ev_out, 0));
    return 0;
}

void rccl_destroy(void* user)
{
    RcclEx* X = static_cast<RcclEx*>(user);
    hipSetDevice(X->device);
    if (X->cs) hipStreamSynchronize(X->cs);
    if (X->comm && g_rccl.CommDestroy) g_rccl.CommDestroy(X->comm);
    if (X->dbuf) hipFree(X->dbuf);
    if (X->hpin) hipHostFree(X->hpin);
    if (X->ev_in) hipEventDestroy(X->ev_in);
    if (X->ev_out) hipEventDestroy(X->ev_out);
    if (X->cs) hipStreamDestroy(X->cs);
    delete X;
}

// ---------------------------------------------------------------------------
// W ranks as threads of one process

struct LocalShared {
    uint32_t world = 0;
    std::mutex mu;
    std::condition_variable cv;
    uint32_t arrived = 0;
    uint64_t gen = 0;
    uint32_t refs = 0;
    std::vector<std::vector<int64_t>> vals;
    std::vector<const void* const*> sendp;
    std::vector<const uint64_t*> srows;
    std::vector<uint32_t> row_bytes;

    void barrier()
    {
        std::unique_lock<std::mutex> lk(mu);
        const uint64_t g = gen;
        if (++arrived == world) {
            arrived = 0;
            ++gen;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != g; });
        }
    }
};

struct LocalEx {
    LocalShared* sh;
    uint32_t rank;
};

int local_allgather(void* user, const int64_t* host_send, uint32_t n, int64_t* host_recv)
{
    LocalEx* X = static_cast<LocalEx*>(user);
    LocalShared* S = X->sh;
    S->vals[X->rank].assign(host_send, host_send + n);
    S->barrier();
    int rc = 0;
    for (uint32_t r = 0; r < S->world; ++r) {
        if (S->vals[r].size() != n) { rc = ex_fail("local allgather: ranks disagree on the count"); break; }
        std::memcpy(host_recv + (size_t)r * n, S->vals[r].data(), sizeof(int64_t) * n);
    }
    // every rank reaches the second barrier, failed or not, so the arrival count stays in step
    S->barrier();
    return rc;
}

int local_allreduce(void* user, int64_t* values, uint32_t n)
{
    LocalEx* X = static_cast<LocalEx*>(user);
    LocalShared* S = X->sh;
    S->vals[X->rank].assign(values, values + n);
    S->barrier();
    int rc = 0;
    for (uint32_t r = 0; r < S->world; ++r)
        if (S->vals[r].size() != n) rc = ex_fail("local allreduce: ranks disagree on the count");
    for (uint32_t i = 0; i < n && rc == 0; ++i) {
        int64_t t = 0;
        for (uint32_t r = 0; r < S->world; ++r) t += S->vals[r][i];
        values[i] = t;
    }
    S->barrier();
    return rc;
}

int local_alltoallv(void* user, const void* const* send, const uint64_t* send_rows, void* recv, const uint64_t* recv_off,
                    const uint64_t* recv_rows, uint32_t row_bytes, void* stream)
{
    LocalEx* X = static_cast<LocalEx*>(user);
    LocalShared* S = X->sh;
    const uint32_t me = X->rank;
    hipStream_t s = (hipStream_t)stream;
    // this rank's segments are complete before another rank copies them
    HCHK(hipStreamSynchronize(s));
    S->sendp[me] = send;
    S->srows[me] = send_rows;
    S->row_bytes[me] = row_bytes;
    S->barrier();
    int rc = 0;
    for (uint32_t r = 0; r < S->world && rc == 0; ++r) {
        const uint64_t rows = S->srows[r][me];
        if (rows != recv_rows[r] || S->row_bytes[r] != row_bytes) { rc = ex_fail("local alltoallv: splits disagree"); break; }
        if (rows) {
            const hipError_t e = hipMemcpyAsync(static_cast<uint8_t*>(recv) + recv_off[r] * row_bytes, S->sendp[r][me],
                                                rows * row_bytes, hipMemcpyDeviceToDevice, s);
            if (e != hipSuccess) rc = ex_fail(std::string("local alltoallv copy: ") + hipGetErrorString(e));
        }
    }
    // the copies out of other ranks' segments finish before those ranks move on
    const hipError_t e = hipStreamSynchronize(s);
    if (rc == 0 && e != hipSuccess) rc = ex_fail(std::string("local alltoallv: ") + hipGetErrorString(e));
    S->barrier();
    return rc;
}

void local_destroy(void* user)
{
    LocalEx* X = static_cast<LocalEx*>(user);
    LocalShared* S = X->sh;
    bool last = false;
    {
        std::lock_guard<std::mutex> lk(S->mu);
        last = --S->refs == 0;
    }
    if (last) delete S;
    delete X;
}

}  // namespace

extern "C" {

const char* ovs_exchange_last_error(void) { return g_ex_err.c_str(); }

const char* ovs_exchange_stage(uint32_t* round)
{
    if (round) *round = g_stage_round.load(std::memory_order_relaxed);
    return g_stage.load(std::memory_order_acquire);
}

ovs_status ovs_rccl_unique_id(void* unique_id_128)
{
    if (!unique_id_128) return OVS_EINVAL;
    if (!load_rccl()) return OVS_EDEVICE;
    ncclUniqueId id;
    const ncclResult_t r = g_rccl.GetUniqueId(&id);
    if (r != ncclSuccess) { nccl_fail(r, "ncclGetUniqueId"); return OVS_EDEVICE; }
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
    std::memcpy(unique_id_128, &id, sizeof id);
    return OVS_OK;
}

ovs_status ovs_exchange_rccl_create(int device, uint32_t rank, uint32_t world, const void* unique_id_128,
                                    ovs_exchange* out)
{
    if (!out || !unique_id_128 || world < 1 || rank >= world) return OVS_EINVAL;
    std::memset(out, 0, sizeof *out);
    if (!load_rccl()) return OVS_EDEVICE;
    if (hipSetDevice(device) != hipSuccess) { ex_fail("hipSetDevice"); return OVS_EDEVICE; }
    RcclEx* X = new RcclEx();
    X->device = device;
    X->rank = rank;
    X->world = world;
    if (hipStreamCreateWithFlags(&X->cs, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&X->ev_in, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&X->ev_out, hipEventDisableTiming) != hipSuccess) {
        ex_fail("rccl exchange: stream / events");
        rccl_destroy(X);
        return OVS_EDEVICE;
    }
    ncclUniqueId id;
    std::memcpy(&id, unique_id_128, sizeof id);
    const ncclResult_t r = g_rccl.CommInitRank(&X->comm, (int)world, id, (int)rank);
    if (r != ncclSuccess) {
        nccl_fail(r, "ncclCommInitRank");
        X->comm = nullptr;
        rccl_destroy(X);
        return OVS_EDEVICE;
    }
    out->user = X;
    out->rank = rank;
    out->world = world;
    out->allgather_i64 = rccl_allgather;
    out->alltoallv = rccl_alltoallv;
    out->allreduce_sum_i64 = rccl_allreduce;
    out->destroy = rccl_destroy;
    return OVS_OK;
}

ovs_status ovs_exchange_local_create(uint32_t world, ovs_exchange* out)
{
    if (!out || world < 1 || world > 64) return OVS_EINVAL;
    LocalShared* S = new LocalShared();
    S->world = world;
    S->refs = world;
    S->vals.resize(world);
    S->sendp.resize(world, nullptr);
    S->srows.resize(world, nullptr);
    S->row_bytes.resize(world, 0);
    for (uint32_t r = 0; r < world; ++r) {
        LocalEx* X = new LocalEx{S, r};
        out[r].user = X;
        out[r].rank = r;
        out[r].world = world;
        out[r].allgather_i64 = local_allgather;
        out[r].alltoallv = local_alltoallv;
        out[r].allreduce_sum_i64 = local_allreduce;
        out[r].destroy = local_destroy;
    }
    return OVS_OK;
}

void ovs_exchange_destroy(ovs_exchange* ex)
{
    if (!ex) return;
    if (ex->destroy && ex->user) ex->destroy(ex->user);
    std::memset(ex, 0, sizeof *ex);
}

}  // extern "C"
