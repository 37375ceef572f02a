// host_tables.hpp -- the host-side table bookkeeping of the C ABI (no HIP): explicit Chord tables
// and the batched maintenance rounds' updates of them, and the validation / ordering of an
// EpiChord snapshot.  ovs_kbr.cpp uploads what these produce; tests/test_sanitizers.py builds this
// translation unit with plain g++ under ASan/UBSan and drives it (tests/host_tables_driver.cpp).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "key160.hpp"

namespace ovs {

// An explicit (possibly non-converged) Chord ring as the host keeps it between rounds
// (ovs_chord_load_tables): ChordFingerTable deques (index p = 159 - position), their sizes, the
// successor lists and predecessors, and the resolved getFinger(pos) rows the device reads.
struct ChordHost {
    std::vector<K160> ids;
    std::vector<uint32_t> deque;      // n * 160
    std::vector<uint8_t> fsize;       // deque sizes
    std::vector<uint32_t> succ0;      // successorList->getSuccessor()
    std::vector<uint32_t> fres;       // n * 160 resolved getFinger(pos)
    std::vector<uint32_t> pred;       // predecessorNode (0xFFFFFFFF unspecified)
    std::vector<uint32_t> succ;       // n * sls successor lists
    std::vector<uint8_t> nsucc;
    int sls = 0;

    uint64_t n() const { return ids.size(); }
    void clear();
    // import and validate; false with *err set on an inconsistent table
    bool import(const K160* keys, uint64_t n, const uint32_t* pred, const uint32_t* succ, const uint8_t* nsucc,
                const uint32_t* fingers, const uint8_t* deque_size, int sls, std::string* err);
    // ChordFingerTable::getFinger(pos) of node v from its deque (ChordFingerTable.cc:174-193)
    void resolve_row(uint64_t v);
    // handleFixFingersTimerExpired (Chord.cc:851-870) for the listed nodes: trivial fingers removed,
    // the FixfingersCall keys (v + 2^i) with their source and position appended
    void fix_fingers_plan(const uint32_t* nodes, uint64_t m, std::vector<K160>* keys, std::vector<uint32_t>* src,
                          std::vector<uint8_t>* pos);
    // handleRpcFixfingersResponse (1228-1270): finger pos[q] of src[q] := responsible[q] where ok[q];
    // returns the deque entries that changed
    uint64_t fix_fingers_apply(const std::vector<uint32_t>& src, const std::vector<uint8_t>& pos,
                               const std::vector<uint32_t>& responsible, const std::vector<uint8_t>& ok);
    // one synchronous stabilize round (Chord.cc:793-842, 1055-1225; ChordSuccessorList.cc:101-194)
    // for the listed nodes; changed_succ0 = nodes whose successor changed (their rows re-resolved)
    void stabilize(const uint32_t* nodes, uint64_t m, uint64_t* succ_changed, uint64_t* lists_changed,
                   uint64_t* pred_changed, std::vector<uint32_t>* changed_succ0);
};

// Counters of a Kademlia maintenance round (ovs_kad_round_stats' twin)
struct KadRoundCount {
    uint64_t lookups = 0, failed = 0, responses = 0, sib_changes = 0, bucket_changes = 0, lost = 0, replacement = 0,
             refreshed = 0;
};

// What one refresh lookup of a maintenance round produced (device results copied to the host):
// the FindNodeCalls it sent (destination, arrival there), the responses it handled (responder,
// arrival at the source) and each response's carried nodes (findNode(key, R, -1) at the responder).
struct KadRoundLookup {
    uint32_t src;
    const uint32_t* cnode; const int64_t* ctime; int ncall;
    const uint32_t* resp; const int64_t* tarr; int nresp;
    const uint32_t* const* carried; const uint8_t* ncarried;   // per response
};

// Explicit Kademlia tables as the host keeps them between maintenance rounds: per node the sibling
// table sorted by XOR distance to the node (Kademlia::siblingTable, a KademliaBucket with
// KeyDistanceComparator<KeyXorMetric>, Kademlia.cc:179, 315-317) and the routing buckets in LRU
// order (KademliaBucket push_back / erase in routingAdd, 432-756).
struct KadHost {
    std::vector<K160> ids;
    int k = 0, s = 0;
    std::vector<std::vector<uint32_t>> sib;    // n
    std::vector<std::vector<uint32_t>> bk;     // n * 160

    uint64_t n() const { return ids.size(); }
    void clear();
    // import siblings[n*5s] (any order) and bucket_count[n*160] / bucket_nodes[n*160*k] (LRU
    // order); the device builder validates the invariants, this keeps a copy
    void import(const K160* keys, uint64_t n, int k, int s, const uint32_t* siblings, const uint8_t* bucket_count,
                const uint32_t* bucket_nodes);
    // the k-stride arrays ovs_kad_load_tables takes (siblings XOR-sorted); false when a bucket holds
    // more than k entries
    bool export_k(uint32_t* siblings, uint8_t* bucket_count, uint32_t* bucket_nodes) const;
    // Kademlia::routingAdd (Kademlia.cc:432-756) at node v: secureMaintenance, pingNewSiblings,
    // activePing and proximityNeighborSelection off, bucketType "kademlia"; returns its result
    bool routing_add(uint32_t v, uint32_t h, bool alive, KadRoundCount* st);
    // a round's refresh lookups (handleBucketRefreshTimerExpired, 1591-1686) for nodes[0..m): per
    // node, flags bit 0 the sibling refresh (own key, Rs), bit 1 the bucket refreshes of the buckets
    // stale[j*5..] marks (NULL = all; key self ^ 2^i, i = 159 .. msb(self ^ front), Rb)
    void refresh_plan(const uint32_t* nodes, uint64_t m, const uint8_t* flags, const uint32_t* stale, int Rs, int Rb,
                      std::vector<K160>* keys, std::vector<uint32_t>* src, std::vector<int>* R) const;
    // apply a round's routingAdd events: at every node, in simulated-time order (ties: calls first,
    // then lookup and index order), a call reaching it adds its source alive (handleRpcCall,
    // 1328-1349), a handled response adds the carried nodes not alive, then the responder alive
    // (handleRpcResponse, 1352-1420)
    void apply_round(const std::vector<KadRoundLookup>& lk, KadRoundCount* st);
};

// An EpiChord snapshot (ovs_epichord_load): validates the lists and the finger caches and returns the
// per-node meta words and the cache rows sorted in liveCache map order (x - (v + 1)); false with
// *err naming the node on an inconsistent snapshot.
bool epichord_prepare(const K160* keys, uint64_t n, int L, const uint32_t* succ, const uint8_t* nsucc,
                      const uint32_t* pred, const uint8_t* npred, const uint8_t* lists_full, const uint64_t* cache_off,
                      const uint32_t* cache_node, const int64_t* cache_last, const int64_t* cache_ttl,
                      std::vector<uint32_t>* meta, std::vector<uint32_t>* cnode, std::vector<int64_t>* clast,
                      std::vector<int64_t>* cttl, std::string* err);

}  // namespace ovs
