// kad.hpp -- Kademlia device tables and launchers (internal).
#pragma once
#include "engine.hpp"

namespace ovs {

// 64 B node record of the Kademlia snapshot (one HBM line per responder visit):
//  key   : node id
//  R     : key ^ back(siblingTable)  -- the sibling radius; isSiblingFor's
//          "(self ^ key) > (self ^ back)" test (Kademlia.cc:923-935)
//  mask  : OR over siblings s of 2^msb(s ^ key) -- with it, "self is the
//          XOR-closest of siblings + self" is (D & mask) == 0 for D = self ^ lookup key
//  boff  : first bucket slot of the node's row; slot s <-> bucket m = 159 - s,
//          for m = 159 .. endIndex = msb(R) (buckets below endIndex are all siblings)
struct alignas(16) KadRec {
    uint32_t key[5];
    uint32_t R[5];
    uint32_t mask[5];
    uint32_t boff;
};
static_assert(sizeof(KadRec) == 64, "KadRec must be one 64 B line");

// bucket entry with the member's key inline (24 B); a slot holds k entries,
// NONE idx marks an empty entry (entries are packed at the front)
struct KadEntry {
    uint32_t key[5];
    uint32_t idx;
};

struct KadTables {
    KadRec* recs = nullptr;
    uint32_t* sib = nullptr;      // n * S5 member indices (unordered set), NONE padded
    KadEntry* sibe = nullptr;     // n * S5 sibling entries with the member key inline
    KadEntry* slots = nullptr;    // total_slots * k
    uint64_t total_slots = 0;
    uint32_t lo = 0, hi = 0;      // sib / sibe / bucket rows exist for nodes [lo, hi) (the whole ring unsharded)
    int k = 8, s = 8;
    uint64_t seed = 0;
    int exact = 1;                // two IDs share their top 63 bits: K2 uses the 160-bit tie fallback
};

struct KadView {
    const KadRec* __restrict__ recs;
    const double2* __restrict__ xy;
    const uint32_t* __restrict__ sib;
    const KadEntry* __restrict__ sibe;
    const KadEntry* __restrict__ slots;
    uint32_t n;
    int k;
    int S5;       // sibling table capacity 5s
    int nsib;     // entries in every sibling table = min(5s, n-1)
    uint32_t lo, hi;   // owned arc: sibling / bucket rows of nodes [lo, hi)
};

void kad_free(KadTables& t);
// tables for nodes [lo, hi) of the sorted ring (node records for all n)
hipError_t kad_build(const KeyRec* recs, uint32_t n, int k, int s, uint64_t seed, KadTables& t, hipStream_t st,
                     uint32_t lo = 0, uint32_t hi = 0xFFFFFFFFu);
hipError_t kad_export(const KadTables& t, uint32_t n, uint32_t* siblings, uint8_t* bucket_count,
                      uint32_t* bucket_nodes, hipStream_t st);
hipError_t kad_route(const KadTables& t, const KeyRec* recs, const double2* xy, uint32_t n, const ovs_params& P,
                     const DelayConsts& DC, const K160* qkeys, const uint32_t* qsrc, uint64_t nq,
                     ovs_route_out* out, uint32_t* hopseq, uint32_t* rpcs, int num_cu, hipStream_t st,
                     uint32_t* sibs = nullptr);
hipError_t kad_find_node(const KadTables& t, const KeyRec* recs, uint32_t n, const ovs_params& P,
                         const uint32_t* node, const K160* keys, uint64_t nq, int numRedundant, int numSiblings,
                         uint32_t* out_nodes, uint32_t max_out, uint8_t* out_count, uint8_t* out_sib,
                         hipStream_t st);

}  // namespace ovs
