// kad.hpp -- Kademlia device tables and launchers (internal).
//
// Layout:
//  KadNode nodes[n]   one 64 B line per node: everything the *sender* of a FindNodeCall needs of
//                     its target (key, coordinates, isSiblingFor summary, bucket-row offset), read
//                     once per RPC when the call is sent
//  KadX    nodex[n]   the exact sibling radius R and level mask (fallback on summary ties, rare)
//  KadBlk  blks[]     bucket rows and sibling rows as 96 B blocks of 8 entries (top 64 bits of the
//                     member key, member index): bucket m of node v = the bpb = ceil(k/8) blocks at
//                     blks[nodes[v].boff + (159 - m) * bpb] for m = rowlo(v) .. 159 (k <= 8: one block,
//                     two lines; KademliaLarge's k = 16: two); sibling row of an owned node v =
//                     ceil(5s/8) blocks at sib_base + (v - lo) * sbn, in ascending level msb(x ^ v)
//  uint8_t slev[n*5s] one arc of a sharded network: the level msb(x ^ v) of each sibling x of every
//                     node v (5s bytes a node), so a LookupCall decides isSiblingFor(numSiblings > 1)
//                     of any responder on its home rank
// The reference's structures these hold: Kademlia::siblingTable (a KademliaBucket of 5s entries
// sorted by XOR distance to this node, Kademlia.cc:179, 315-317) and routingTable[160] (buckets
// of up to k entries in LRU order, KademliaBucket.h:30-69, filled by routingAdd 432-756).
#pragma once
#include "engine.hpp"

namespace ovs {

// lookupParallelRpcs <= 8 (maidsafe.ini:18-19 sets 8).  Pending-call slots of a lookup with
// lookupParallelRpcs = alpha: the K2 instantiation's capacity A (alpha 5..8 run on the A = 8
// objects); the slots a sharded lookup owns follow A, not alpha.
constexpr int KAD_MAX_ALPHA = 8;
inline int kad_pend_slots(int alpha) { return alpha <= 4 ? alpha : KAD_MAX_ALPHA; }

// meta bits of KadNode
constexpr uint32_t KMETA_MASK_OUT = 1u << 24;   // level-mask bits below the 64-bit window: exact check
// sharded networks with replicated top buckets (KadTables::tl): bit 25 + j set when the node's
// bucket 159 - j (j < tl <= KTOP_MAX) holds k members and lies above its sibling zone -- then
// findNode there is that bucket's XOR-closest, answerable from the replicated block on any rank
constexpr int KTOP_MAX = 7;
constexpr int KMETA_TOPFULL_SHIFT = 25;
constexpr uint32_t KMETA_TOPFULL_ALL = 0x7Fu << KMETA_TOPFULL_SHIFT;
struct alignas(64) KadNode {
    uint32_t key[5];
    uint32_t boff;     // first line of the bucket row
    double x, y;       // SimpleUnderlay coordinates
    uint64_t rtop;     // top64(R), R = key ^ back(siblingTable) = max over siblings of (s ^ key)
    uint64_t mwin;     // level mask bits [mlo, mlo + 63], mlo = max(endIndex - 63, 0); level mask =
                       // OR over siblings s of 2^msb(s ^ key): this node is the XOR-closest of
                       // siblings + itself to D = key ^ K  <=>  (D & mask) == 0
    uint32_t meta;     // endIndex + 1 (bits 0-7, 0 = no siblings), rowlo + 1 (8-15, 0 = no row),
                       // nsib (16-23), KMETA_* flags (24-31)
    uint32_t spare;
};
static_assert(sizeof(KadNode) == 64, "KadNode is one 64 B line");

struct KadX {
    uint32_t R[5];
    uint32_t mask[5];
};

constexpr int KBLK = 8;   // entries per block; a bucket of k entries takes bpb = ceil(k / 8) blocks (k <= 16)
constexpr int KMAX = 16;  // largest bucket size k (and findNode result) the engine implements
struct alignas(32) KadBlk {
    uint64_t top[KBLK];    // top 64 bits (bits 96..159) of the member key; ~0 for an empty entry
    uint32_t idx[KBLK];    // member node index; NONE for an empty entry (entries packed at the front)
};
static_assert(sizeof(KadBlk) == 96, "KadBlk is 96 B");

__host__ __device__ __forceinline__ int kad_end(uint32_t meta) { return (int)(meta & 0xFFu) - 1; }
__host__ __device__ __forceinline__ int kad_rowlo(uint32_t meta) { return (int)((meta >> 8) & 0xFFu) - 1; }
__host__ __device__ __forceinline__ int kad_nsib(uint32_t meta) { return (int)((meta >> 16) & 0xFFu); }

struct KadTables {
    KadNode* nodes = nullptr;
    KadX* nodex = nullptr;
    KadBlk* blks = nullptr;        // bucket rows (rows_blks blocks), then the sibling rows of the owned arc
    uint64_t rows_blks = 0;        // bucket-row blocks; sibling rows start here
    uint32_t* sib = nullptr;       // (hi - lo) * S5 sibling member indices of the owned arc, NONE padded (export)
    uint8_t* slev = nullptr;       // sharded networks: n * S5 sibling levels msb(x ^ v), 0xFF padded, for
                                   // isSiblingFor(numSiblings > 1) of a responder off the owned arc
    uint32_t lo = 0, hi = 0;       // sibling / bucket rows exist for nodes [lo, hi) (the whole network unsharded)
    int k = 8, s = 8;
    int bpb = 1;                   // blocks per bucket, ceil(k / 8)
    uint64_t seed = 0;
    int exact = 1;                 // two IDs share their top 63 bits: comparisons use the 160-bit tie fallback
    int snapshot = 1;              // 0: explicit tables (ovs_kad_load_tables)
    int maybe_short = 0;           // explicit tables: some node may answer fewer than resultSize nodes
    // general tables (ovs_kad_load_tables_csr: b > 1, bucketType nr128 / nkademlia): the buckets in
    // CSR form instead of the 160 bucket rows (blks then holds the sibling rows only)
    int general = 0;
    int b = 1, nb = KEYBITS;       // digit width, numBuckets
    uint32_t* goff = nullptr;      // n * nb + 1 member offsets (bucket i of node v: [goff[v*nb+i], goff[v*nb+i+1]))
    uint64_t* gtop = nullptr;      // per member: top 64 bits of its key
    uint32_t* gidx = nullptr;      // per member: node index (LRU order within a bucket)
    int16_t* gend = nullptr;       // per node: routingBucketIndex of its farthest sibling (-1: none)
    uint64_t gtotal = 0;           // members
    // sharded networks: the top tl buckets of EVERY node replicated at the front of blks (tend
    // blocks: bucket 159 - j of v at (v * tl + j) * bpb), so a responder off the owned arc whose
    // findNode is its full main bucket there is answered on this rank (Kademlia migration, §6)
    int tl = 0;
    uint64_t tend = 0;
};

// the general-table view of K2g and the batched findNode (kad_general.hip)
struct KadGenView {
    const uint32_t* __restrict__ goff;
    const uint64_t* __restrict__ gtop;
    const uint32_t* __restrict__ gidx;
    const int16_t* __restrict__ gend;
    int b, nb;
};

struct KadView {
    const KadNode* __restrict__ nodes;
    const KadX* __restrict__ nodex;
    const KadBlk* __restrict__ blks;
    const KadBlk* __restrict__ sibb;    // sibling rows of the owned arc
    const uint8_t* __restrict__ slev;   // sibling levels of every node (sharded networks only)
    const double2* __restrict__ xy;
    uint32_t n;
    int k;
    int bpb;      // blocks per bucket
    int S5;       // sibling table capacity 5s
    int sbn;      // blocks per sibling row = ceil(5s / 8)
    uint32_t lo, hi;   // owned arc: sibling / bucket rows of nodes [lo, hi)
    int tl;            // replicated top buckets (KadTables::tl) ...
    uint32_t tend;     // ... in blocks [0, tend): a row offset below tend is a replicated (virtual) row
    uint32_t nblk;     // blocks of blks[] before the sibling rows (rows_blks): every valid row offset is
                       // <= nblk, so a larger one names no row of this rank (checked in sharded kernels)
    int maybe_short;
    int snapshot;      // tables built by the snapshot rule (ovs_kad_load), not imported
    unsigned long long* err;   // sharded kernels: a table read this arc cannot serve is counted here
                               // (ovs_kad_shard_errors) instead of made; nullptr on one GPU
};

// a table access outside the owned arc [lo, hi): counted (sharded kernels), never performed
__device__ __forceinline__ bool kad_off_arc(const KadView& V, uint32_t c) { return c < V.lo || c >= V.hi; }
__device__ __forceinline__ void kad_count_error(const KadView& V)
{
    if (V.err) atomicAdd(V.err, 1ull);
}

void kad_free(KadTables& t);
// snapshot tables for nodes [lo, hi) of the sorted ring (node records for all n)
hipError_t kad_build(const KeyRec* recs, const double2* xy, uint32_t n, int k, int s, uint64_t seed, KadTables& t,
                     hipStream_t st, uint32_t lo = 0, uint32_t hi = 0xFFFFFFFFu, int tl = 0);
// explicit tables (device copies of the caller's siblings / bucket members); returns
// hipErrorInvalidValue with *bad_node set when a table breaks the reference's invariants
hipError_t kad_build_explicit(const KeyRec* recs, const double2* xy, uint32_t n, int k, int s, const uint32_t* sib,
                              const uint8_t* bcount, const uint32_t* bnodes, KadTables& t, uint32_t* bad_node,
                              uint32_t* bad_code, hipStream_t st);
hipError_t kad_export(const KadTables& t, uint32_t n, uint32_t* siblings, uint8_t* bucket_count,
                      uint32_t* bucket_nodes, hipStream_t st);
// general tables from CSR (device copies of the caller's arrays: sib n*5s, off n*nb+1 (< 2^32
// members), nodes); caps[nb] = routingBucketSize per bucket index (0: unbounded, nkademlia).
// hipErrorInvalidValue with *bad_node / *bad_code when a table breaks routingAdd's invariants.
hipError_t kad_build_general(const KeyRec* recs, const double2* xy, uint32_t n, int k, int s, int b, const int* caps,
                             const uint32_t* sib, const uint32_t* off, const uint32_t* nodes, uint64_t total,
                             KadTables& t, uint32_t* bad_node, uint32_t* bad_code, hipStream_t st);
// K2g (kad_general.hip): one-way routes (sibs == nullptr) or LookupCalls over general tables
hipError_t kad_route_general(const KadTables& t, const double2* xy, uint32_t n, const ovs_params& P,
                             const DelayConsts& DC, const K160* qkeys, const uint32_t* qsrc, uint64_t nq,
                             ovs_route_out* out, uint32_t* hopseq, uint32_t* rpcs, hipStream_t st, uint32_t* sibs);
// recursive routing (R/Kademlia, kad_general.hip) over either table form: one-way routes (sibs ==
// nullptr; hopseq optional) or LookupCalls with numSiblings lookup_ns (semi- / full-recursive
// response as P.routingType says); key_timeout = rpcKeyTimeout in ns
hipError_t kad_route_recursive(const KadTables& t, const double2* xy, uint32_t n, const ovs_params& P,
                               const DelayConsts& DC, int64_t key_timeout, int lookup_ns, const K160* qkeys,
                               const uint32_t* qsrc, uint64_t nq, ovs_route_out* out, uint32_t* hopseq, uint32_t* sibs,
                               hipStream_t st);
hipError_t kad_find_node_general(const KadTables& t, uint32_t n, const uint32_t* node, const K160* keys, uint64_t nq,
                                 int numRedundant, int numSiblings, uint32_t* out_nodes, uint32_t max_out,
                                 uint8_t* out_count, uint8_t* out_sib, hipStream_t st);
hipError_t kad_route(const KadTables& t, const double2* xy, uint32_t n, const ovs_params& P,
                     const DelayConsts& DC, const K160* qkeys, const uint32_t* qsrc, uint64_t nq,
                     ovs_route_out* out, uint32_t* hopseq, uint32_t* rpcs, int num_cu, hipStream_t st,
                     uint32_t* sibs = nullptr, unsigned long long* dyn = nullptr);
// exhaustive-iterative lookups (K2x, kad_refresh.hip): config.redundantNodes = R, a siblings vector
// of ns <= R; out = ovs_route_out (oneway: KBRTestApp one-way test) or ovs_lookup_out; responders =
// the accepted responders in order (= hop_seq); *capacity_error: a lookup ran past the kernel's
// fixed capacities (more than 64 timed-out nodes)
// trace: (maintenance rounds) per accepted response its arrival at the source (tarr, hopCountMax
// per lookup), per FindNodeCall sent its destination and arrival there (cnode / ctime, ccap per
// lookup; a lookup sending more is a capacity error)
struct KadExhTrace {
    int64_t* tarr;
    uint32_t* cnode;
    int64_t* ctime;
    int ccap;
};
hipError_t kad_exhaustive(const KadTables& t, const double2* xy, uint32_t n, const ovs_params& P, const DelayConsts& DC,
                          int R, int ns, bool oneway, const K160* qkeys, const uint32_t* qsrc, uint64_t nq, void* out,
                          uint32_t* sibs, uint32_t* responders, int64_t* rtts, uint32_t* rpcs, int num_cu,
                          hipStream_t st, bool* capacity_error, const KadExhTrace* trace = nullptr, bool pad = true,
                          bool internal_resp = false);
// pad = false: the responder / RTT rows are left unwritten past a lookup's responders (the caller
// filled them, or reads only the lookup's hops entries -- the internal visited lists)
// internal_resp: nobody reads the responder rows (they are the lookups' visited sets): the first
// KXVL responders of a lookup stay in LDS (kad_refresh.hip)
// free the exhaustive-lookup scratch K2x keeps for `device` between calls (ovs_ctx_destroy)
void kad_exhaustive_release(int device);
// bucket-refresh keys of nodes[0..m) (device buffers); *total = how many (up to cap written)
hipError_t kad_refresh_keys(const KadTables& t, uint32_t n, const uint32_t* nodes, uint64_t m, const uint32_t* stale,
                            K160* keys, uint32_t* src, uint64_t cap, uint64_t* total, hipStream_t st);
hipError_t kad_find_node(const KadTables& t, uint32_t n, const ovs_params& P, const uint32_t* node, const K160* keys,
                         uint64_t nq, int numRedundant, int numSiblings, uint32_t* out_nodes, uint32_t max_out,
                         uint8_t* out_count, uint8_t* out_sib, hipStream_t st);

}  // namespace ovs
