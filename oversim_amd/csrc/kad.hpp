// kad.hpp -- Kademlia device tables and launchers (internal).
#pragma once
#include "engine.hpp"

namespace ovs {

// Kademlia snapshot on the device (DESIGN.md "Kademlia snapshot rule").
//  sib[n*S5]      : sibling table, XOR-sorted to the owner, NONE padded (S5 = 5s)
//  nsib[n]
//  boff[n*161]    : CSR offsets of the owner's non-empty buckets by index m
//  bnodes[...]    : bucket members (up to k per bucket)
struct KadTables {
    uint32_t* sib = nullptr;
    uint8_t* nsib = nullptr;
    uint32_t* bcount = nullptr;   // n*160 packed counts (u8 in u32 words: 4 per word) -- see kad.hip
    uint32_t* bnodes = nullptr;   // n*160*k, NONE padded
    int k = 8, s = 8;
    uint64_t seed = 0;
};

void kad_free(KadTables& t);
hipError_t kad_build(const KeyRec* recs, uint32_t n, int k, int s, uint64_t seed, KadTables& t, hipStream_t st);
hipError_t kad_export(const KadTables& t, uint32_t n, uint32_t* siblings, uint8_t* bucket_count,
                      uint32_t* bucket_nodes, hipStream_t st);
hipError_t kad_route(const KadTables& t, const KeyRec* recs, const double2* xy, uint32_t n, const ovs_params& P,
                     const DelayConsts& DC, const K160* qkeys, const uint32_t* qsrc, uint64_t nq,
                     ovs_route_out* out, uint32_t* hopseq, uint32_t* rpcs, int num_cu, hipStream_t st);
hipError_t kad_find_node(const KadTables& t, const KeyRec* recs, uint32_t n, const ovs_params& P,
                         const uint32_t* node, const K160* keys, uint64_t nq, int numRedundant, int numSiblings,
                         uint32_t* out_nodes, uint32_t max_out, uint8_t* out_count, uint8_t* out_sib,
                         hipStream_t st);

}  // namespace ovs
