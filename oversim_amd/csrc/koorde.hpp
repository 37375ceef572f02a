// koorde.hpp -- Koorde (src/overlay/koorde/Koorde.cc) on a converged ring: device tables and
// launchers (internal).
//
// Koorde is a Chord ring (sorted node keys; predecessor, successor list) plus, per node, the
// de Bruijn pointer handleDeBruijnTimerExpired converges to (Koorde.cc:164-230, answered by
// handleRpcDeBruijnRequest 328-367): deBruijnNode and the deBruijnNodes list, which on a
// converged ring are dbNum consecutive ring nodes starting at sorted index dbStart.
#pragma once
#include "engine.hpp"

namespace ovs {

struct alignas(16) KoordeNode {
    uint32_t db;         // deBruijnNode
    uint32_t dbStart;    // deBruijnNodes[0] (the list is dbNum consecutive ring nodes)
    uint32_t dbNum;      // deBruijnNumber
    uint32_t pad;
};
static_assert(sizeof(KoordeNode) == 16, "KoordeNode is 16 B");

// K3's per-node record (two 64 B lines, one 128 B L2 line): everything a hop at v reads.  Ring
// distances enter as 32-bit codes (k_code64 >> 32: msb + 1 in the top byte, the 24 bits below it),
// order-preserving and decided unless two codes are equal -- then the exact keys in recs[] decide.
//   line 0: key, code(key - pred key), the de Bruijn pointer (KoordeNode), coordinates
//   line 1: sum[j-1] = code(key(v + j) - key(v)), j = 1..16: the successor-list distances, which
//           also answer a de Bruijn-list walk that starts at v (the lists are consecutive ring nodes)
struct alignas(128) KoordeRec {
    uint32_t w[5];
    uint32_t cP;
    uint32_t db, dbStart, dbNum;
    uint32_t pad0;
    double x, y;
    uint32_t pad1[2];
    uint32_t sum[16];
};
static_assert(sizeof(KoordeRec) == 128, "KoordeRec is one 128 B line");
constexpr int KREC_LIST = 16;    // successorListSize / deBruijnListSize the record form covers

// KoordeFindNodeExtMessage (ChordMessage.msg:168-172): the de Bruijn route key and step a
// FindNodeCall / FindNodeResponse carries
struct KExt {
    K160 rk;
    int32_t step;
    int32_t has;         // 0: routeKey unspecified
};

struct KoordeTables {
    KoordeNode* nd = nullptr;
    KoordeRec* rec = nullptr;   // record form (ns, deBruijnListSize <= 16); nullptr: list walks on recs[]
    uint32_t n = 0;
    int ns = 0;          // successor list size min(successorListSize, n - 1)
    int sb = 4;          // shiftingBits
    int dbls = 16;       // deBruijnListSize
    int useOther = 1;    // useOtherLookup
    int useSuc = 1;      // useSucList
};

void koorde_free(KoordeTables& t);
hipError_t koorde_build(const KeyRec* recs, const double2* xy, uint32_t n, int successorListSize, int shiftingBits, int deBruijnListSize,
                        int useOtherLookup, int useSucList, KoordeTables& t, hipStream_t st);
// K3: batched one-way lookups (KBRTestApp -> IterativeLookup with Koorde::findNode); hopseq
// (n * hopCountMax) is required: it is also the lookup's visited set
hipError_t koorde_route(const KoordeTables& t, const KeyRec* recs, const double2* xy, const DelayConsts& DC,
                        int hopCountMax, const K160* keys, const uint32_t* src, uint64_t nq, ovs_route_out* out,
                        uint32_t* hopseq, bool record, uint32_t* rpcs, int num_cu, hipStream_t st,
                        unsigned long long* dyn = nullptr);
// Koorde::findNode at node[i] for keys[i] with extension ext[i] (updated in place); next[i] =
// the hop, 0xFFFFFFFF where the reference throws
hipError_t koorde_find_node(const KoordeTables& t, const KeyRec* recs, const uint32_t* node, const K160* keys,
                            KExt* ext, uint32_t* next, uint64_t nq, hipStream_t st);

}  // namespace ovs
