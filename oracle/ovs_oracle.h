/*
 * ovs_oracle.h -- CPU restatement of OverSim's iterative KBR lookup path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the *checker* for the MI355X
 * engine in oversim_amd/: only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it.  The product path never links,
 * calls or falls back to it.
 *
 * Parity status: the reference (trucndt/oversim) cannot be built here -- it
 * needs OMNeT++ 4.x, INET and opp_msgc output.  The
 * reference ships no golden vectors for routing results, so the routing parts
 * of this restatement are "parity unpinned" against reference outputs; they
 * are pinned only by hand-derived known answers taken from the input cases of
 * OverlayKey::test() (OverlayKey.cc:720-828) and by a second, independent
 * pure-Python restatement in tests/refmodel.py for small rings.
 *
 * Every function cites the reference file:line it restates.
 */
#ifndef OVS_ORACLE_H
#define OVS_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- keys: 5 x u32, w[0] least significant (same wire layout as ovs_key160) */
typedef struct { uint32_t w[5]; } orc_key;

/* OverlayKey operations (OverlayKey.cc).  Results are written to *out. */
int      orc_key_cmp(const orc_key* a, const orc_key* b);                  /* compareTo 842-847 */
void     orc_key_add(const orc_key* a, const orc_key* b, orc_key* out);    /* operator+ 247-253,283-288 */
void     orc_key_sub(const orc_key* a, const orc_key* b, orc_key* out);    /* operator- 256-262,291-296 */
void     orc_key_xor(const orc_key* a, const orc_key* b, orc_key* out);    /* operator^ 341-349 */
/* which: 0=isBetween (a,b), 1=isBetweenR (a,b], 2=isBetweenL [a,b), 3=isBetweenLR [a,b]
 * unspec_mask bit0: x unspecified, bit1: a unspecified, bit2: b unspecified */
int      orc_key_between(int which, const orc_key* x, const orc_key* a, const orc_key* b,
                         int unspec_mask);                                 /* 587-644 */
uint32_t orc_key_bit_range(const orc_key* k, uint32_t p, uint32_t n);      /* getBitRange 458-474 */
uint32_t orc_key_shared_prefix(const orc_key* a, const orc_key* b, uint32_t bitsPerDigit); /* 530-555 */
int      orc_key_log2(const orc_key* k);                                   /* log_2 558-578 */
void     orc_key_pow2(uint32_t e, orc_key* out);                           /* pow2 704-717 */

/* ---- parameters (names follow the .ini / NED parameter names) */
typedef struct {
    int32_t hopCountMax;              /* BaseOverlay.ned, default.ini:385 = 50 */
    int32_t successorListSize;        /* Chord.ned, default.ini:174 = 8 */
    int32_t numFingerCandidates;      /* default.ini:176 = 3 */
    int32_t k, s, b;                  /* Kademlia.ned, default.ini:197-199 */
    int32_t lookupRedundantNodes;
    int32_t lookupParallelRpcs;
    int32_t lookupMerge;
    int32_t lookupStrictParallelRpcs;
    int32_t lookupVisitOnlyOnce;
    int32_t lookupAcceptLateSiblings;
    int32_t lookupUseAllParallelResponses;
    int32_t lookupNewRpcOnEveryTimeout;
    int32_t lookupNewRpcOnEveryResponse;
    int32_t lookupFinishOnFirstUnchanged;
    int32_t numSiblings;              /* sendToKey(..., numSiblings=1) for KBRTestApp one-way */
    int32_t simtimeRound;             /* 1: SimTime(double) rounds half-up, 0: truncates */
    double  rpcUdpTimeout;            /* default.ini:483 = 1.5 s */
    double  lookupTimeout;            /* IterativeLookup.h:44 LOOKUP_TIMEOUT = 10 s */
    double  datarate;                 /* channels.ned simple_ethernetline = 10 Mbps */
    double  accessDelay;              /* channels.ned = 0 ms */
    int32_t callBytes;                /* FindNodeCall incl. 28 B UDP/IP = 83 */
    int32_t respBaseBytes;            /* FindNodeResponse with 0 nodes incl. UDP/IP = 61 */
    int32_t respPerNodeBytes;         /* + 26 B per NodeHandle */
    int32_t routeBytes;               /* one-way KBRTestMessage route msg = 186 */
    uint64_t kadSeed;                 /* Kademlia snapshot bucket-sampling seed */
    int32_t routingType;              /* 0 iterative, 1 semi-recursive, 2 full-recursive, 3 exhaustive-iterative, 4 source-routing-recursive (default.ini:392) */
    int32_t recNumRedundantNodes;     /* default.ini:386 = 3 */
    /* Koorde (Koorde.ned, default.ini:268-291) */
    int32_t shiftingBits;             /* = 4 */
    int32_t deBruijnListSize;         /* = 16 */
    int32_t useOtherLookup;           /* = true */
    int32_t useSucList;               /* = true */
    /* the fork's Kademlia bucket variants (Kademlia.cc:135-151, 384-411; default.ini:209-211):
     * bucketType 0 "kademlia" (k per bucket), 1 "nkademlia" (buckets unbounded while the table
     * holds fewer than globalNodeLimit entries), 2 "nr128" (the top buckets hold up to 2^offset,
     * offset from extraNodesFinalBucket, 0 = keyLength) */
    int32_t bucketType;
    int32_t globalNodeLimit;          /* = 1000 */
    int32_t extraNodesFinalBucket;    /* = 0 */
    double  rpcKeyTimeout;            /* default.ini:484 = 10 s: a routed RPC (recursive LookupCalls) */
    /* Chord.ned extendedFingerTable (default.ini:176 = false): finger entries hold the finger's
     * FixfingersResponse candidates, getMaxNumRedundantNodes() = numFingerCandidates.  Stable
     * (orc_chord_build / _lazy) rings only: explicit tables do not carry the candidate lists */
    int32_t extendedFingerTable;
    /* BaseOverlay.ned measureAuthBlock (default.ini:399 = false): every RPC response carries
     * AUTHBLOCK_L = SIGNATURE_L + CERT_L + PUBKEY_L = 800 bits (CommonMessages.msg:45-47, 57, 73) */
    int32_t measureAuthBlock;
} orc_params;

void orc_params_chord_default(orc_params* p);
void orc_params_kad_default(orc_params* p);
/* Koorde defaults: successorListSize = deBruijnListSize = 16, shiftingBits = 4, useOtherLookup,
 * useSucList; FindNodeCall / FindNodeResponse carry the 168-bit KoordeFindNodeExtMessage */
void orc_params_koorde_default(orc_params* p);

/* ---- networks */
typedef struct orc_net orc_net;
/* Chord stable state: ids sorted ascending, unique.  xy = 2n doubles.      */
orc_net* orc_chord_build(const orc_key* ids, uint32_t n, const double* xy, const orc_params* p);
/* Explicit Chord snapshot: pred[n], succ[n*succ_stride] (count in nsucc[n]),
 * fingers[n*160] indexed by finger position i (0..159), 0xFFFFFFFF = unspecified.
 * deque_size[n] = fingerTable.size() (ChordFingerTable.cc:61-87). */
orc_net* orc_chord_build_tables(const orc_key* ids, uint32_t n, const double* xy,
                                const uint32_t* pred, const uint32_t* succ, const uint8_t* nsucc,
                                uint32_t succ_stride, const uint32_t* fingers,
                                const uint8_t* deque_size, const orc_params* p);
/* Kademlia snapshot (DESIGN.md "Kademlia snapshot rule"). */
orc_net* orc_kad_build(const orc_key* ids, uint32_t n, const double* xy, const orc_params* p);
/* The same networks with lazy tables: nothing but ids / coordinates is stored; every table
 * entry is evaluated on access by the rule the eager builders store (Chord: pred, successor
 * list, finger i = responsible(n + 2^i); Kademlia: a node's sibling table and buckets, built
 * on first use into a per-thread cache).  Results are identical; memory is O(n), so samples of
 * configs D (2^26-node Chord) and E (2^24-node Kademlia) can be checked. */
orc_net* orc_chord_build_lazy(const orc_key* ids, uint32_t n, const double* xy, const orc_params* p);
orc_net* orc_kad_build_lazy(const orc_key* ids, uint32_t n, const double* xy, const orc_params* p);
/* Explicit Kademlia tables: siblings[n*5s] (UINT32_MAX padded, any order: kept XOR-sorted like
 * Kademlia::siblingTable), bucket_count[n*160], bucket_nodes[n*160*k] (routingTable buckets). */
orc_net* orc_kad_build_tables(const orc_key* ids, uint32_t n, const double* xy, const uint32_t* siblings,
                              const uint8_t* bucket_count, const uint32_t* bucket_nodes, const orc_params* p);
/* Koorde (Koorde.cc) on the converged Chord ring of the same ids: successor lists of
 * successorListSize, the de Bruijn pointer and list each node's handleDeBruijnTimerExpired /
 * DeBruijnCall exchange converges to (Koorde.cc:164-230, 328-390). */
orc_net* orc_koorde_build(const orc_key* ids, uint32_t n, const double* xy, const orc_params* p);
/* de Bruijn state: node db[i], list = the db_num[i] ring nodes from sorted index db_start[i] */
void     orc_koorde_export(const orc_net* net, uint32_t* db, uint32_t* db_start, uint8_t* db_num);
/* Koorde::findNode at `node` for key with a KoordeFindNodeExtMessage (route_key, step);
 * *has_route_key = 0: routeKey unspecified.  Updates route_key / step / has_route_key to the
 * extension the response carries; returns the next hop, or UINT32_MAX when the reference
 * throws (findDeBruijnHop bounding error, findStartKey invalid start key). */
uint32_t orc_koorde_find_node(const orc_net* net, uint32_t node, const orc_key* key, orc_key* route_key,
                              int* has_route_key, int* step);
void     orc_net_free(orc_net* net);

/* export the Kademlia snapshot so the GPU builder can be checked:
 * siblings[n*5s] (UINT32_MAX padded), bucket_count[n*160], bucket_nodes[n*160*k] */
void orc_kad_export(const orc_net* net, uint32_t* siblings, uint8_t* bucket_count, uint32_t* bucket_nodes);
/* export the Chord finger table resolved through getFinger(): out[n*160] */
void orc_chord_export_fingers(const orc_net* net, uint32_t* out);

/* findNode at `node` (Chord.cc:548-599 / Kademlia.cc:1101-1246).
 * returns count, nodes in out[] (cap 64); *sibling_flag = isSiblingFor(node,key,numSiblings) */
int orc_find_node(const orc_net* net, uint32_t node, const orc_key* key, int numRedundantNodes,
                  int numSiblings, uint32_t* out, int* sibling_flag);

/* ---- batched one-way lookups (KBRTestApp one-way test, iterative routing) */
typedef struct {
    uint32_t responsible;   /* node index or 0xFFFFFFFF */
    uint16_t hops;          /* IterativeLookup::getMinHops() */
    uint8_t  status;        /* 0 ok, see ovs_kbr.h */
    uint8_t  one_way_hops;  /* KBRTestApp "One-way Hop Count" = hops + (R != S) */
    int64_t  latency_ns;    /* "One-way Latency" in ns */
} orc_route_out;

/* hop_seq may be NULL; else n*hopCountMax entries (accepted responders, UINT32_MAX padded).
 * rpcs_out may be NULL; else per-lookup count of FindNodeCalls sent.
 * nthreads<=0 -> all OpenMP threads. Returns total accepted hops, or ORC_FAIL when a fixed
 * capacity of the restatement was exceeded (orc_last_error; never a silent truncation). */
#define ORC_FAIL 0xFFFFFFFFFFFFFFFFull
uint64_t orc_route_batch(const orc_net* net, const orc_key* keys, const uint32_t* src, uint64_t n,
                         orc_route_out* out, uint32_t* hop_seq, uint32_t* rpcs_out, int nthreads);

/* ---- batched LookupCalls (KBRTestApp lookup test) */
typedef struct {
    uint32_t num_siblings;  /* LookupResponse siblings array size (0 when !isValid) */
    uint16_t hops;          /* getMinHops() */
    uint8_t  status;        /* 0 ok, see ovs_kbr.h */
    uint8_t  is_valid;
    int64_t  latency_ns;    /* lookup duration; -1 when !isValid */
} orc_lookup_out;

/* numSiblings < 0 -> getMaxNumSiblings().  siblings = n * numSiblings (NONE padded).
 * Returns the numSiblings used, -1 on error (orc_last_error). */
int orc_lookup_batch(const orc_net* net, const orc_key* keys, const uint32_t* src, uint64_t n, int numSiblings,
                     orc_lookup_out* out, uint32_t* siblings, int nthreads);

/* Exhaustive-iterative Kademlia lookups (the bucket / sibling refresh of Kademlia.cc:1591-1686 with
 * exhaustiveRefresh): lookup i of keys[i] from src[i] with numSiblings = config.redundantNodes = R.
 * out/siblings as orc_lookup_batch (siblings = n*R); responders / rtts (may be NULL) = n*hopCountMax
 * accepted responders in order and their RTTs in ns (NONE / -1 padded); rpcs (may be NULL) = n
 * FindNodeCall counts.  Returns R, -1 on error. */
int orc_kad_exhaustive_batch(const orc_net* net, const orc_key* keys, const uint32_t* src, uint64_t n, int R,
                             orc_lookup_out* out, uint32_t* siblings, uint32_t* responders, int64_t* rtts,
                             uint32_t* rpcs, int nthreads);
/* The bucket-refresh keys of Kademlia::handleBucketRefreshTimerExpired (Kademlia.cc:1631-1676, b = 1)
 * for nodes[0..m): self ^ 2^i for i = 159 .. msb(self ^ closest sibling) where bit i of the node's
 * 160-bit stale mask is set (stale = m*5 words, NULL = every bucket stale).  Writes up to cap
 * (key, src) pairs, returns how many there are (ORC_FAIL on error). */
uint64_t orc_kad_refresh_keys(const orc_net* net, const uint32_t* nodes, uint64_t m, const uint32_t* stale,
                              orc_key* keys, uint32_t* src, uint64_t cap);

/* orc_kad_exhaustive_batch plus, per accepted response, the time it reached the source (tarrs,
 * hopCountMax slots, -1 padded), and every FindNodeCall the lookup sent: its destination (cnode,
 * ccap slots, NONE padded) and the time it reached it (ctime), ns from the lookup's start. */
int orc_kad_exhaustive_batch_t(const orc_net* net, const orc_key* keys, const uint32_t* src, uint64_t n, int R,
                               orc_lookup_out* out, uint32_t* siblings, uint32_t* responders, int64_t* rtts,
                               int64_t* tarrs, uint32_t* cnode, int64_t* ctime, int ccap, uint32_t* rpcs,
                               int nthreads);

/* One synchronous Kademlia maintenance round on explicit tables (orc_kad_build_tables): for the
 * listed nodes, handleBucketRefreshTimerExpired's exhaustive-iterative refresh lookups
 * (Kademlia.cc:1591-1686; flags[j] bit 0 = the sibling-table refresh of the node's own key with
 * 5s redundant nodes, bit 1 = the bucket refreshes of the buckets stale[j*5..] marks (NULL = all)
 * with lookupRedundantNodes; flags NULL = both) all routed on the round-start tables; then every
 * node applies Kademlia::routingAdd (432-756) for the FindNodeCalls that reached it (handleRpcCall,
 * 1328-1349; every call sent, answered or not) and the FindNodeResponses its lookups handled
 * (handleRpcResponse, 1352-1420: the carried nodes not alive, then the responder alive) in
 * simulated-time order, every lookup of the round starting at instant 0 (ties: calls first, then
 * task and index order).  Returns the membership changes
 * (sibling insertions + bucket insertions + preempted siblings lost), ORC_FAIL on error. */
typedef struct {
    uint64_t lookups;        /* refresh lookups routed */
    uint64_t failed;         /* lookups that did not end successfully (hopCountMax, timeouts) */
    uint64_t responses;      /* FindNodeResponses applied */
    uint64_t sib_changes;    /* handles inserted into a sibling table */
    uint64_t bucket_changes; /* handles inserted into a bucket */
    uint64_t lost;           /* preempted siblings whose bucket was full */
    uint64_t replacement;    /* alive handles a full bucket turned away (replacement cache) */
    uint64_t refreshed;      /* alive handles already known (LRU move / sibling refresh) */
} orc_kad_round_stats;
uint64_t orc_kad_maintenance_round(orc_net* net, const uint32_t* nodes, uint64_t m, const uint8_t* flags,
                                   const uint32_t* stale, orc_kad_round_stats* st, int nthreads);
/* Kademlia::routingAdd(x, isAlive) at node v on explicit tables (the rules the round applies);
 * returns its result, -1 on error */
int orc_kad_routing_add(orc_net* net, uint32_t v, uint32_t x, int isAlive);
/* explicit / snapshot tables in CSR form: siblings[n*5s] (NONE padded), bucket_off[n*NB+1],
 * bucket_nodes[bucket_off[n*NB]] (each bucket in LRU order); NB = numBuckets = (2^b - 1) * (160 / b)
 * (Kademlia.cc:176); bucket_nodes NULL = size query */
void orc_kad_export_csr(const orc_net* net, uint32_t* siblings, uint64_t* bucket_off, uint32_t* bucket_nodes);
/* explicit tables of any b and bucket sizes in that CSR form (buckets in LRU order) */
orc_net* orc_kad_build_tables_csr(const orc_key* ids, uint32_t n, const double* xy, const uint32_t* siblings,
                                  const uint64_t* bucket_off, const uint32_t* bucket_nodes, const orc_params* p);
/* Kademlia::routingBucketSize(index) (Kademlia.cc:384-411): 0 = unbounded */
int orc_kad_bucket_size(const orc_params* p, int index);
int orc_kad_num_buckets(const orc_params* p);

/* One synchronous stabilize round for nodes[0..m) on explicit tables (Chord.cc:793-842, 1055-1225,
 * ChordSuccessorList.cc:101-194): returns the number of successor lists that changed (ORC_FAIL on
 * error), *succ_changed the successors that changed, *pred_changed the predecessors set. */
uint64_t orc_chord_stabilize(orc_net* net, const uint32_t* nodes, uint64_t m, uint64_t* succ_changed,
                             uint64_t* pred_changed);
void orc_chord_export_lists(const orc_net* net, uint32_t* pred, uint32_t* succ, uint8_t* nsucc);

/* One synchronous fixfingers round for nodes[0..m) (Chord.cc:845-875, 1228-1270): trivial
 * fingers removed, then lookups of n + 2^i routed over the tables, then finger i := result.
 * Explicit or converged networks.  Returns total hops; *out_ok successful lookups,
 * *out_changed fingers whose deque entry changed. */
uint64_t orc_chord_fix_fingers(orc_net* net, const uint32_t* nodes, uint64_t m, uint64_t* out_ok,
                               uint64_t* out_changed, int nthreads);

/* SimpleNodeEntry::calcDelay for an idle tx queue, in ns (SimpleNodeEntry.cc:155-195) */
int64_t orc_delay_ns(const orc_net* net, uint32_t a, uint32_t b, int32_t bytes);
/* float distance (SimpleNodeEntry.cc:145-153) */
float orc_coord_dist(const orc_net* net, uint32_t a, uint32_t b);

/* ---- KBRTestApp one-way statistics (KBRTestApp.cc:380-520, BaseOverlay.cc:1258-1270,
 * GlobalStatistics.cc:103-200).  Per-node KBRTestApp counters, then finishApp in node
 * order feeding cStdDev accumulators (OMNeT++ cStdDev: n, sum, sqrsum, min, max;
 * sample variance, 0 below two values).  Rates only when T >= MIN_MEASURED = 0.1 s. */
typedef struct { uint64_t count; double mean, stddev, min, max; } orc_stddev;
typedef struct {
    uint64_t num_sent, num_delivered, num_dropped, num_lookup_failed;
    uint64_t hop_count_sum;
    int64_t  latency_sum_ns;
    double   hop_count_mean, latency_mean_s;   /* "Vector: ... .mean" scalars */
    orc_stddev sd[5];   /* delivered msg/s, delivered B/s, dropped msg/s, dropped B/s, delivery ratio */
} orc_kbrtest_result;
void orc_kbrtest_stats(const orc_net* net, const orc_route_out* out, const orc_key* keys, const uint32_t* src,
                       uint64_t n, double measured_time_s, int lookupNodeIds, int32_t testMsgSize,
                       orc_kbrtest_result* st);
typedef struct {
    uint64_t num_sent, num_success, num_failed, num_invalid;
    uint64_t hop_count_sum, failed_hop_count_sum;
    int64_t  success_latency_sum_ns;
    double   hop_count_mean, failed_hop_count_mean, success_latency_mean_s, total_latency_mean_s;
    orc_stddev sd[3];   /* successful lookups/s, failed lookups/s, success ratio */
} orc_kbrtest_lookup_result;
/* KBRTestApp lookup-test statistics (KBRTestApp.cc:331-371, 546-557) of orc_lookup_batch output */
void orc_kbrtest_lookup_stats(const orc_net* net, const orc_lookup_out* out, const uint32_t* siblings, int stride,
                              const orc_key* keys, const uint32_t* src, uint64_t n, double measured_time_s,
                              int lookupNodeIds, double failureLatency, orc_kbrtest_lookup_result* st);
/* EpiChord::findNode (EpiChord.cc:517-629) at node `self` on one routing snapshot
 * (ovs_oracle_epichord.c): succ/pred = the successor / predecessor list entries closest first
 * (nsucc/npred of them), lists_full bit 0 / bit 1 = successorList / predecessorList->isFull()
 * (else thisNode ends the list), listSize = successorListSize; the live finger cache as ncache
 * (node, lastUpdate ns, ttl ns) entries in any order.  src = the FindNodeCall's source
 * (UINT32_MAX: a local call, msg == NULL), now = simTime() in ns, cacheTTL in ns.  Writes the
 * next hops and their lastUpdates (the EpiChordFindNodeExtMessage) to out/out_last (cap slots).
 * Returns the count; -1 where the reference throws "Failed to find node", -2 where it
 * dereferences an empty finger cache (undefined), -3 bad input, -4 cap too small. */
int orc_epichord_find_node(const orc_key* ids, uint32_t n, uint32_t self, const uint32_t* succ, int nsucc,
                           const uint32_t* pred, int npred, int lists_full, int listSize, const uint32_t* cnode,
                           const int64_t* clast, const int64_t* cttl, int ncache, const orc_key* key, uint32_t src,
                           int64_t now, int64_t cacheTTL, int numRedundantNodes, uint32_t* out, int64_t* out_last,
                           int cap);
const char* orc_last_error(void);
int orc_cap_failed(void);      /* 1 once a capacity was exceeded (sticky until orc_clear_error) */
void orc_clear_error(void);

#ifdef __cplusplus
}
#endif
#endif
