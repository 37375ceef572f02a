// kad_shard.hpp -- multi-GPU Kademlia request/response kernels (internal).
#pragma once
#include "kad.hpp"
#include "compact.hpp"

namespace ovs {

// findNode result slot of one pending FindNodeCall of a lookup (home rank); C = the findNode
// capacity of the network (8; 16 for KademliaLarge)
template <int C>
struct KadResN {
    uint32_t count;      // result size (<= C)
    uint32_t ready;      // 0 = requested, not delivered yet
    uint32_t nodes[C];
    uint64_t dist[C];    // top 64 bits of node XOR key
};
using KadRes = KadResN<8>;
static_assert(sizeof(KadResN<8>) == 104 && sizeof(KadResN<16>) == 200, "KadRes layout");
// the response record on the wire: ovs_kad_resp (C = 8) / ovs_kad_resp16
template <int C> struct KadWire;
template <> struct KadWire<8> { using type = ovs_kad_resp; };
template <> struct KadWire<16> { using type = ovs_kad_resp16; };
// the network's findNode capacity on the shard path: 16 when k or lookupRedundantNodes exceed 8
inline int kad_shard_cap(const ovs_params& P, const KadTables& t)
{
    return (P.lookupRedundantNodes > 8 || t.k > 8) ? 16 : 8;
}

// what the shard-step instantiation of K2 (kad_route.hip) reads and writes in one round
struct KadShardStepArgs {
    void* st;                          // the suspended lookups: KadStateWords words each, stride nlist_max (SoA)
    uint8_t* act;                      // 2: not started, 1: suspended in st, 0: never runs (source off the arc)
    const K160* qkeys;                 // the batch's keys and sources (a lookup starts from them in the
    const uint32_t* qsrc;              // round that first visits it: no state record before its first suspend)
    void* res;                         // nlook * A result slots (KadResN<C>)
    const uint64_t* list;              // this round's lookups (indices), *nlist_dev of them
    const unsigned long long* nlist_dev;
    uint64_t nlist_max;                // sizes the grid (the lookups of the batch)
    const uint32_t* qids;
    const uint64_t* shard_lo;          // device copy of the arc bounds
    int nsh;
    ovs_kad_req* rstage;               // a request per pending-call slot, tagged by owner in rtag
    uint8_t* rtag;
    ovs_done_rec* dstage;              // a done record per lookup; ltag: 0 finished, 1 still active
    uint8_t* ltag;
    uint32_t* sib_out;                 // LookupCalls: the sibling rows (nullptr: KBR routes)
};

// the migration step (k_kad_route<.., SM = 2>): one round over migrated lookup records or a batch's
// keys; every input gets one outcome at its own index -- a record moving to rank mtag[q] (mstage,
// KadRecWords words each) or a done record (dstage, mtag[q] = nsh)
struct KadMigStepArgs {
    const uint32_t* in;                // nin migrated records, or nullptr: the batch's first round ...
    const K160* fkeys;                 // ... from its keys and sources (lookup q has id fqid + q)
    const uint32_t* fsrc;
    uint32_t fqid;
    uint64_t nin;
    const uint64_t* shard_lo;          // device copy of the arc bounds
    int nsh, me;
    uint32_t* mstage;
    uint8_t* mtag;
    ovs_done_rec* dstage;
    unsigned long long* dyn;           // the dynamic tail's zeroed counter (nullptr: static slices)
};

size_t kad_lookup_state_bytes(int alpha, int cap);
// bytes of a migrating lookup record (KadRecWords) for lookupParallelRpcs alpha
uint32_t kad_rec_bytes(int alpha);
// does the migration step implement these parameters (one-way KBR routes on snapshot tables, findNode
// results of up to 8 nodes)
bool kad_mig_supported(const ovs_params& P, const KadTables& t);
// one migration round: the outcomes compacted by tag into per-rank segments of out (out + d * out_cap
// records, counter out_count[d]) and the done buffer (done_count)
hipError_t kad_mig_step(const KadTables& t, const double2* xy, uint32_t n, const ovs_params& P, const DelayConsts& DC,
                        const void* in, uint64_t nin, const K160* fkeys, const uint32_t* fsrc, uint32_t fqid,
                        const uint64_t* shard_lo, int nsh, int me, void* out, uint64_t out_cap,
                        unsigned long long* out_count, ovs_done_rec* done, uint64_t done_cap,
                        unsigned long long* done_count, unsigned long long* bad, int num_cu, StageBuf& stage,
                        hipStream_t s, unsigned long long* dyn = nullptr);
bool kad_params_supported_host(const ovs_params& P, const KadTables& t);
// lookups of this rank: their keys and sources (copied to qkeys / qsrc), act = 2 (not started), qids,
// the round-1 list (indices 0..n-1) and its count; sources off [lo, hi) are counted in *bad and never run
hipError_t kad_shard_init(const K160* keys, const uint32_t* src, uint64_t n, uint32_t qid_base, K160* qkeys,
                          uint32_t* qsrc, uint8_t* act, uint32_t* qids, uint64_t* iota, unsigned long long* nlist,
                          uint32_t lo, uint32_t hi, unsigned long long* bad, hipStream_t s);
// one round: the list's lookups advance while their responders are local (k_kad_route<.., SHARD>);
// requests to the owners of the others go to segment d of out (out + d * out_cap, counter
// out_count[d]); finished lookups are appended to done (done_count); the still active ones form the
// next list (*nlist_next) and are counted in *active_count.  bad: table reads off the arc.
hipError_t kad_shard_step(const KadTables& t, const double2* xy, uint32_t n, const ovs_params& P,
                          const DelayConsts& DC, void* st, uint8_t* act, const K160* qkeys, const uint32_t* qsrc,
                          const uint32_t* qids, void* res,
                          uint64_t nlook, const uint64_t* list, const unsigned long long* nlist, const uint64_t* iota,
                          uint64_t* list_next, unsigned long long* nlist_next, const uint64_t* shard_lo, int nsh,
                          ovs_kad_req* out, uint64_t out_cap, unsigned long long* out_count, ovs_done_rec* done,
                          uint64_t done_cap, unsigned long long* done_count, unsigned long long* active_count, int lk_ns,
                          uint32_t* sib_out, unsigned long long* bad, int num_cu, StageBuf& stage, hipStream_t s);
hipError_t kad_shard_serve(const KadTables& t, uint32_t n, const ovs_params& P, const ovs_kad_req* in, uint64_t nreq,
                           void* out, unsigned long long* bad, hipStream_t s);
// cap: the network's findNode capacity (kad_shard_cap): the record types of in / res
hipError_t kad_shard_deliver(int cap, const void* in, uint64_t n, void* res, uint64_t nslots, unsigned long long* bad,
                             hipStream_t s);

}  // namespace ovs
