// epichord.hpp -- EpiChord (src/overlay/epichord/) routing snapshots on the device and the batched
// per-call findNode (internal).
//
// EpiChord's routing state is a finger cache that every message rewrites, so the
// engine does not route batches of EpiChord lookups; it evaluates EpiChord::findNode (EpiChord.cc:
// 517-629) for a batch of FindNodeCalls against one snapshot of the responders' state, each call
// with the side effects the reference applies on its way to the answer (the source's cache and
// node-list insertion).  Layout per node v:
//   succ / pred   [n * L] u32: successorList / predecessorList entries closest first (L =
//                 successorListSize); meta[v] = nsucc | npred << 8 | isFull bits << 16
//   cache CSR     coff[v] .. coff[v + 1]: v's live finger cache sorted by (x - (v + 1)) mod 2^160
//                 (the liveCache map order, EpiChordFingerCache.h), node / lastUpdate ns / ttl ns
#pragma once
#include "engine.hpp"

namespace ovs {

constexpr int EPI_MAXL = 16;     // successorListSize the device form holds
constexpr int EPI_MAXR = 32;     // numRedundantNodes

struct EpiTables {
    uint32_t n = 0;
    int L = 0;
    uint32_t* succ = nullptr;
    uint32_t* pred = nullptr;
    uint32_t* meta = nullptr;
    uint64_t* coff = nullptr;
    uint32_t* cnode = nullptr;
    int64_t* clast = nullptr;
    int64_t* cttl = nullptr;
    uint64_t nent = 0;
};

void epichord_free(EpiTables& t);
// status per call: 0 answered, 1 the reference throws "Failed to find node" (EpiChord.cc:613-614),
// 2 the reference dereferences an empty finger cache (EpiChordFingerCache.cc:317-322: undefined),
// 3 node / source index outside the network
hipError_t epichord_find_node(const EpiTables& t, const KeyRec* recs, const uint32_t* node, const K160* keys,
                              const uint32_t* src, const int64_t* now, uint64_t nq, int numRedundant, int64_t cacheTTL,
                              uint32_t* out_nodes, int64_t* out_last, uint32_t max_out, uint8_t* out_count,
                              uint8_t* out_status, hipStream_t st);

}  // namespace ovs
