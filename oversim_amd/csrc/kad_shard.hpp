// kad_shard.hpp -- multi-GPU Kademlia request/response kernels (internal).
#pragma once
#include "kad.hpp"
#include "compact.hpp"

namespace ovs {

// findNode result slot of one pending FindNodeCall of a lookup (home rank)
struct KadRes {
    uint32_t count;      // result size (<= 8)
    uint32_t ready;      // 0 = requested, not delivered yet
    uint32_t nodes[8];
    uint64_t dist[8];    // top 64 bits of node XOR key
};
static_assert(sizeof(KadRes) == 104, "KadRes layout");

size_t kad_lookup_state_bytes(int alpha);
bool kad_params_supported_host(const ovs_params& P, const KadTables& t);
hipError_t kad_shard_init(int alpha, const K160* keys, const uint32_t* src, uint64_t n, uint32_t qid_base,
                          const double2* xy, void* st, uint8_t* act, uint32_t* qids, KadRes* res, uint32_t lo,
                          uint32_t hi, unsigned long long* bad, hipStream_t s);   // bad: sources off [lo, hi)
hipError_t kad_shard_step(const KadTables& t, const double2* xy, uint32_t n, const ovs_params& P,
                          const DelayConsts& DC, void* st, uint8_t* act, const uint32_t* qids, KadRes* res,
                          uint64_t nlook, const uint64_t* shard_lo, int nsh, ovs_kad_req* out, uint32_t* out_dest,
                          uint64_t out_cap, unsigned long long* out_count, ovs_done_rec* done, uint64_t done_cap,
                          unsigned long long* done_count, unsigned long long* active_count, int lk_ns,
                          uint32_t* sib_out, unsigned long long* bad, StageBuf& stage,
                          hipStream_t s);   // lk_ns < 0: KBR routes; bad: table reads off the arc
hipError_t kad_shard_serve(const KadTables& t, uint32_t n, const ovs_params& P, const ovs_kad_req* in, uint64_t nreq,
                           ovs_kad_resp* out, unsigned long long* bad, hipStream_t s);
hipError_t kad_shard_deliver(const ovs_kad_resp* in, uint64_t n, KadRes* res, uint64_t nslots,
                             unsigned long long* bad, hipStream_t s);

}  // namespace ovs
