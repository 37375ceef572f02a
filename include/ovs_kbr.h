/*
 * ovs_kbr.h -- C ABI of the MI355X batched KBR lookup-routing engine.
 *
 * This is the drop-in boundary for OverSim's iterative key lookup.  In the
 * reference the boundary is C++ virtual dispatch inside one process; each
 * entry point below names the reference interface it replaces:
 *
 *   BaseOverlay::findNode          src/common/BaseOverlay.h:693-696
 *     Chord::findNode              src/overlay/chord/Chord.cc:548-599
 *     Kademlia::findNode           src/overlay/kademlia/Kademlia.cc:1101-1246
 *   BaseOverlay::isSiblingFor      src/common/BaseOverlay.h:417-418
 *     Chord::isSiblingFor          src/overlay/chord/Chord.cc:422-500
 *     Kademlia::isSiblingFor       src/overlay/kademlia/Kademlia.cc:888-962
 *   BaseOverlay::findNodeRpc       src/common/BaseOverlay.cc:1841-1915 (siblings flag)
 *   AbstractLookup::lookup +       src/common/AbstractLookup.h, IterativeLookup.cc:695-723
 *   LookupListener::lookupFinished src/common/LookupListener.h, BaseOverlay.cc:1241-1307
 *   SimpleNodeEntry::calcDelay     src/underlay/simpleunderlay/SimpleNodeEntry.cc:155-195
 *   Kademlia bucket refresh        src/overlay/kademlia/Kademlia.cc:1591-1686 (exhaustive lookups)
 *   EpiChord::findNode             src/overlay/epichord/EpiChord.cc:517-629 (per call, on a snapshot)
 *   .ini parameter binding         simulations/default.ini (same key names)
 *
 * Plain C: no C++ exceptions cross this boundary, no torch types.  Every call
 * returns an ovs_status; ovs_last_error() gives the message (the C++ adapter
 * in INTEGRATION.md turns it into a cRuntimeError, like the reference's
 * throws at Chord.cc:560,619,672).
 *
 * Threading: one context per HIP device; calls on one context are
 * stream-ordered and must not race; different contexts are independent.
 * Ownership: the caller owns every input/output buffer; the context owns the
 * device routing tables.  Buffers are host memory unless the call's `flags`
 * include OVS_DEVICE_PTRS, in which case they are device pointers on the
 * context's device and the call is asynchronous on `stream` (NULL = the HIP
 * default stream, as everywhere in HIP).  Host-pointer calls are synchronous
 * and run on the context's own stream.
 * Context scratch: internal visited / hop lists (explicit-table Chord,
 * exhaustive Kademlia, Koorde without hop_seq, refresh batches without
 * responders) live in one buffer the context caches.  Every call that uses it
 * makes its stream wait for the previous user's launch (an event), so
 * device-pointer calls on different streams stay correct and asynchronous;
 * they serialise on the device through that buffer.
 */
#ifndef OVS_KBR_H
#define OVS_KBR_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OVS_ABI_VERSION 12

/* 160-bit OverlayKey: w[0] = least significant 32 bits.  Equal to the
 * reference's GMP limbs 0..2 with the top limb trimmed to 32 bits
 * (OverlayKey.cc:41-47, 835-838; keyLength = 160, default.ini:393). */
typedef struct ovs_key160 { uint32_t w[5]; } ovs_key160;

typedef enum ovs_status {
    OVS_OK = 0,
    OVS_EINVAL = 1,    /* bad argument (reference: cRuntimeError / opp_error) */
    OVS_ENOMEM = 2,
    OVS_EDEVICE = 3,   /* HIP error or no device */
    OVS_ESTATE = 4,    /* no network loaded / wrong overlay for this call */
    OVS_ENOTSUP = 5    /* parameter combination the engine does not implement */
} ovs_status;

/* per-lookup status (why IterativeLookup::isValid() is false) */
enum {
    OVS_LOOKUP_OK = 0,
    OVS_LOOKUP_TIMEOUT = 1,      /* response after startTime + LOOKUP_TIMEOUT (IterativeLookup.cc:808-815) */
    OVS_LOOKUP_RPC_TIMEOUT = 2,  /* RTT >= rpcUdpTimeout (BaseRpc.cc:191-211) */
    OVS_LOOKUP_HOPMAX = 3,       /* hops >= hopCountMax (IterativeLookup.cc:1074-1086) */
    OVS_LOOKUP_NO_NEXT = 4,      /* no unvisited next hop (IterativeLookup.cc:1147-1168) */
    OVS_LOOKUP_BROKEN = 5,       /* Chord successor list broken (Chord.cc:615-620, 671-672); Koorde::findNode
                                    throws (Koorde.cc:490-493 bounding error, 756-760 invalid start key) */
    OVS_LOOKUP_INVALID = 6       /* recursive LookupCall answered without the siblings flag (RecursiveLookup.cc:120-139) */
};

enum { OVS_OVERLAY_CHORD = 1, OVS_OVERLAY_KADEMLIA = 2, OVS_OVERLAY_KOORDE = 3, OVS_OVERLAY_EPICHORD = 4 };

/* flags */
#define OVS_DEVICE_PTRS  0x1u   /* buffers are device pointers; call is async on `stream` */

/* Parameters.  Field names are the NED/.ini parameter names. */
typedef struct ovs_params {
    int32_t overlay;                    /* OVS_OVERLAY_* */
    int32_t keyLength;                  /* **.keyLength = 160 (only 160 supported) */
    int32_t hopCountMax;                /* **.hopCountMax = 50 */
    int32_t successorListSize;          /* **.chord.successorListSize = 8 */
    int32_t extendedFingerTable;        /* **.chord.extendedFingerTable = false.  true: Chord on a converged
                                           ring (ovs_chord_load / _load_shard) when no FindNodeCall can time
                                           out -- largest RTT from the coordinates' bounding box below
                                           rpcUdpTimeout -- where its routes equal the non-extended ones;
                                           refused otherwise, and for findNode answers of > 1 node and
                                           maintenance rounds (OVS_ENOTSUP) */
    int32_t numFingerCandidates;        /* **.chord.numFingerCandidates = 3 */
    int32_t k, s, b;                    /* **.kademlia.k/s/b = 8/8/1 (b 2..5, bucketType != kademlia:
                                           tables through ovs_kad_load_tables_csr) */
    int32_t lookupRedundantNodes;
    int32_t lookupParallelPaths;        /* 1 only */
    int32_t lookupParallelRpcs;
    int32_t lookupMerge;
    int32_t lookupStrictParallelRpcs;
    int32_t lookupVisitOnlyOnce;
    int32_t lookupAcceptLateSiblings;
    int32_t lookupUseAllParallelResponses;
    int32_t lookupNewRpcOnEveryTimeout;
    int32_t lookupNewRpcOnEveryResponse;
    int32_t lookupFinishOnFirstUnchanged;
    int32_t lookupVerifySiblings;       /* false only */
    int32_t lookupMajoritySiblings;     /* false only */
    int32_t routingType;                /* **.routingType: 0 = "iterative", 1 = "semi-recursive",
                                           2 = "full-recursive" (recursive: Chord stable rings),
                                           3 = "exhaustive-iterative" (Kademlia, BaseOverlay.cc:123-124) */
    int32_t numSiblings;                /* sendToKey numSiblings (1 for KBRTestApp one-way) */
    int32_t useCoordinateBasedDelay;    /* **.udp.useCoordinateBasedDelay = true */
    int32_t simtimeRound;               /* SimTime(double): 1 = round half up, 0 = truncate */
    int32_t testMsgSize;                /* **.kbrTestApp.testMsgSize = 100 B */
    int32_t recNumRedundantNodes;       /* **.recNumRedundantNodes = 3 (default.ini:386) */
    double  rpcUdpTimeout;              /* **.rpcUdpTimeout = 1.5 s */
    double  lookupTimeout;              /* LOOKUP_TIMEOUT = 10 s (IterativeLookup.h:44) */
    double  jitter;                     /* **.udp.jitter (must be 0 for bit-exact latency) */
    double  constantDelay;              /* **.udp.constantDelay = 50 ms */
    double  datarate;                   /* channel datarate, simple_ethernetline = 10 Mbps */
    double  accessDelay;                /* channel delay = 0 ms */
    uint64_t kadSeed;                   /* Kademlia snapshot bucket-sampling seed */
    int32_t shiftingBits;               /* **.koorde.shiftingBits = 4 */
    int32_t deBruijnListSize;           /* **.koorde.deBruijnListSize = 16 */
    int32_t useOtherLookup;             /* **.koorde.useOtherLookup = true */
    int32_t useSucList;                 /* **.koorde.useSucList = true */
    int32_t bucketType;                 /* **.kademlia.bucketType: 0 = "kademlia", 1 = "nkademlia",
                                           2 = "nr128" (Kademlia.cc:135-151; ABI 10, formerly padding) */
    double  cacheTTL;                   /* **.epichord.cacheTTL = 120 s (ABI 8) */
    int32_t globalNodeLimit;            /* **.kademlia.globalNodeLimit = 1000 (nkademlia; ABI 10) */
    int32_t extraNodesFinalBucket;      /* **.kademlia.extraNodesFinalBucket = 0 (nr128; 0 = keyLength) */
    double  rpcKeyTimeout;              /* **.rpcKeyTimeout = 10 s: routed RPCs (recursive LookupCalls; ABI 10) */
    int32_t measureAuthBlock;           /* **.overlay*.*.measureAuthBlock = false (default.ini:399).  true: every
                                           RPC response carries AUTHBLOCK_L = SIGNATURE_L + CERT_L + PUBKEY_L
                                           = 800 bits (CommonMessages.msg:45-47, 57, 73), i.e. +100 B on each
                                           FindNodeResponse / LookupResponse length in the delay (ABI 12) */
} ovs_params;

/* Result of one one-way KBR test lookup (KBRTestApp with kbrOneWayTest). */
typedef struct ovs_route_out {
    uint32_t responsible;   /* node index (sorted-ID order) of getResult()[0]; 0xFFFFFFFF on failure */
    uint16_t hops;          /* IterativeLookup::getMinHops() */
    uint8_t  status;        /* OVS_LOOKUP_* */
    uint8_t  one_way_hops;  /* "KBRTestApp: One-way Hop Count" = hops + (responsible != source) */
    int64_t  latency_ns;    /* "KBRTestApp: One-way Latency" in ns (simtime-scale -9); -1 on failure */
} ovs_route_out;

typedef struct ovs_ctx ovs_ctx;

int         ovs_abi_version(void);
void        ovs_params_default(int32_t overlay, ovs_params* out);
/* Parse OMNeT++ .ini text (sections [General] / [Config X] with `extends`,
 * wildcard keys such as `**.overlay*.chord.successorListSize = 8`, units s/ms/B/Mbps)
 * and overwrite the matching fields of *p.  config_name may be NULL ([General]).
 * Keys the engine does not model but that would change a route, a response size or a
 * delay are refused with OVS_ENOTSUP and a message naming the key (ABI 12): e.g.
 * optimizeTimeouts = true, udp.delayFaultType != "no_fault", neighborCache.ncsType !=
 * "none", kademlia.proximityRouting with a recursive routingType, the Kademlia
 * routingAdd options (proximityNeighborSelection, enableManagedConnections, activePing,
 * secureMaintenance, pingNewSiblings), chord.proximityRouting with extendedFingerTable,
 * malicious nodes; the full list is in DESIGN.md §9. */
ovs_status  ovs_params_from_ini(ovs_params* p, const char* ini_text, const char* config_name,
                                char* err, int err_len);
/* The same from a file, resolving OMNeT++ `include <file>` lines relative to the including
 * file (omnetpp.ini:520 `include ./default.ini`), as Cmdenv reads it (ABI 12). */
ovs_status  ovs_params_from_ini_file(ovs_params* p, const char* path, const char* config_name,
                                     char* err, int err_len);

ovs_status  ovs_ctx_create(int hip_device, ovs_ctx** out);
void        ovs_ctx_destroy(ovs_ctx* ctx);
const char* ovs_last_error(const ovs_ctx* ctx);
ovs_status  ovs_set_params(ovs_ctx* ctx, const ovs_params* p);
ovs_status  ovs_get_params(const ovs_ctx* ctx, ovs_params* p);

/* Chord stable (NoChurn, converged) network: ids sorted ascending and unique,
 * xy = 2n doubles (SimpleUnderlay coordinates).  The context builds the
 * stabilised successor lists and finger tables on the device
 * (Chord.cc:845-875 fixfingers fixed point). */
ovs_status  ovs_chord_load(ovs_ctx* ctx, const ovs_key160* ids_sorted, uint64_t n,
                           const double* xy, uint32_t flags);
/* Explicit (possibly non-converged) Chord snapshot.  pred[n] (0xFFFFFFFF =
 * unspecified), succ[n*successorListSize] with nsucc[n] valid entries,
 * fingers[n*160] by finger position (0xFFFFFFFF = unspecified entry),
 * deque_size[n] = ChordFingerTable deque size (ChordFingerTable.cc:61-87). */
ovs_status  ovs_chord_load_tables(ovs_ctx* ctx, const ovs_key160* ids_sorted, uint64_t n,
                                  const double* xy, const uint32_t* pred, const uint32_t* succ,
                                  const uint8_t* nsucc, const uint32_t* fingers,
                                  const uint8_t* deque_size, uint32_t flags);
/* Kademlia snapshot (DESIGN.md "Kademlia snapshot rule": the converged tables a stable network
 * ends up with), built on the device.  Replaces Kademlia's join / routingAdd / bucket refresh
 * history for a NoChurn network; ovs_kad_load_tables imports the tables of a running one. */
ovs_status  ovs_kad_load(ovs_ctx* ctx, const ovs_key160* ids_sorted, uint64_t n,
                         const double* xy, uint32_t flags);
/* Explicit Kademlia tables -- the k-buckets and sibling tables an OverSim node actually holds
 * (Kademlia::siblingTable / routingTable, Kademlia.cc:179, 432-756; KademliaBucket.h:30-69).
 * siblings[n*5s]: node v's sibling table (0xFFFFFFFF padded; any order -- the reference keeps it
 * XOR-sorted, its back() is the farthest); bucket_count[n*160], bucket_nodes[n*160*k]: routing
 * bucket i of node v (0xFFFFFFFF padded; LRU order, findNode re-sorts by XOR distance).  The
 * tables must keep routingAdd's invariants: members are other nodes of [0, n), a bucket i holds
 * only nodes x with msb(x ^ v) = i and at most k of them, no node twice, no node both sibling and
 * bucket member -- else OVS_EINVAL naming the node.  Host buffers. */
ovs_status  ovs_kad_load_tables(ovs_ctx* ctx, const ovs_key160* ids_sorted, uint64_t n, const double* xy,
                                const uint32_t* siblings, const uint8_t* bucket_count,
                                const uint32_t* bucket_nodes, uint32_t flags);
/* Kademlia variants (ABI 10) through explicit tables in CSR form: b = 1..5 (numBuckets =
 * (2^b - 1) * (160 / b); routingBucketIndex's b-bit digits, Kademlia.cc:176, 357-382) and
 * bucketType "nr128" (b = 1: bigger final buckets, routingBucketSize 384-411) or "nkademlia" (no
 * per-bucket maximum, 620-664), as params.b / params.bucketType say.  siblings[n*5s] as for
 * ovs_kad_load_tables; bucket i of node v = bucket_nodes[bucket_off[v*nb + i] ..
 * bucket_off[v*nb + i + 1]) in LRU order, nb = ovs_kad_num_buckets(params), bucket_off[0] = 0.
 * The tables must keep routingAdd's invariants: members are other nodes of [0, n) whose
 * routingBucketIndex is the bucket's, at most routingBucketSize(i) of them (kademlia / nr128), no
 * node twice, none both sibling and member -- else OVS_EINVAL naming the node.  One-way routes and
 * LookupCalls (iterative routing) and ovs_find_node_batch run on these tables (kernel K2g);
 * exhaustive-iterative routing, refresh batches and maintenance rounds take the 160-bucket
 * kademlia tables only (OVS_ENOTSUP).  Host buffers. */
int32_t     ovs_kad_num_buckets(const ovs_params* p);   /* -1 when b is outside 1..5 */
ovs_status  ovs_kad_load_tables_csr(ovs_ctx* ctx, const ovs_key160* ids_sorted, uint64_t n, const double* xy,
                                    const uint32_t* siblings, const uint64_t* bucket_off,
                                    const uint32_t* bucket_nodes, uint32_t flags);
/* The loaded Kademlia tables in CSR form (host buffers): siblings[n*5s] (0xFFFFFFFF padded),
 * bucket_off[n*nb + 1], up to cap bucket members; *total = how many there are (cap 0 sizes the
 * call; bucket_nodes may then be NULL).  Any loaded whole network (ovs_kad_load, _tables, _csr). */
ovs_status  ovs_kad_export_csr(ovs_ctx* ctx, uint32_t* siblings, uint64_t* bucket_off, uint32_t* bucket_nodes,
                               uint64_t cap, uint64_t* total);
/* Koorde (src/overlay/koorde/Koorde.cc, class Koorde : public Chord) on a converged ring: the
 * Chord ring of ids (predecessor, successorListSize successors) plus every node's de Bruijn
 * pointer and list as handleDeBruijnTimerExpired / the DeBruijnCall exchange leave them
 * (Koorde.cc:164-230, 328-390).  Routing goes through ovs_route_batch (Koorde::findNode,
 * 405-556, for every FindNodeCall of IterativeLookup, iterative routing with
 * lookupRedundantNodes = lookupParallelRpcs = 1 and merge off -- the Koorde defaults). */
ovs_status  ovs_koorde_load(ovs_ctx* ctx, const ovs_key160* ids_sorted, uint64_t n, const double* xy,
                            uint32_t flags);
/* de Bruijn state per node (host buffers): deBruijnNode, and the deBruijnNodes list as
 * db_num[i] consecutive ring nodes from sorted index db_start[i] */
ovs_status  ovs_koorde_export(ovs_ctx* ctx, uint32_t* db_node, uint32_t* db_start, uint8_t* db_num);
/* KoordeFindNodeExtMessage (ChordMessage.msg:168-172): the route key and step a Koorde
 * FindNodeCall carries; has_route_key = 0 is an unspecified route key */
typedef struct ovs_koorde_ext {
    uint32_t route_key[5];
    int32_t  step;
    int32_t  has_route_key;
} ovs_koorde_ext;
/* Koorde::findNode at node[i] for keys[i] with the call's extension ext[i], which is replaced by
 * the one the response carries; next[i] = the single next hop, 0xFFFFFFFF where the reference
 * throws.  Host buffers. */
ovs_status  ovs_koorde_find_node_batch(ovs_ctx* ctx, const uint32_t* node, const ovs_key160* keys,
                                       ovs_koorde_ext* ext, uint32_t* next, uint64_t n);
/* EpiChord (src/overlay/epichord/): one snapshot of every node's routing state, for
 * ovs_epichord_find_node_batch.  EpiChord's finger cache is rewritten by every message a node
 * sends or receives (EpiChord.cc:546-553, 754-780), so the engine does not route EpiChord lookups
 * in batches; it answers findNode calls exactly against a given state.  Per node v:
 * succ[v*L ..] / pred[v*L ..] (L = successorListSize <= 16): the EpiChordNodeList entries closest
 * first, nsucc[v] / npred[v] of them; lists_full[v] bit 0 / bit 1 = successorList /
 * predecessorList->isFull() (when clear, thisNode ends the list, so it has fewer than L entries);
 * the live finger cache (EpiChordFingerCache::liveCache) as cache_node / cache_last_ns (lastUpdate)
 * / cache_ttl_ns (ttl, 0 = never expires) entries cache_off[v] .. cache_off[v+1], any order, each
 * node at most once and never v itself.  The dead cache is not needed: a FindNodeCall's source is
 * heard from directly, which removes it from the dead cache before anything reads it.  Host
 * buffers; params.overlay must be OVS_OVERLAY_EPICHORD. */
ovs_status  ovs_epichord_load(ovs_ctx* ctx, const ovs_key160* ids_sorted, uint64_t n, const double* xy,
                              const uint32_t* succ, const uint8_t* nsucc, const uint32_t* pred,
                              const uint8_t* npred, const uint8_t* lists_full, const uint64_t* cache_off,
                              const uint32_t* cache_node, const int64_t* cache_last_ns,
                              const int64_t* cache_ttl_ns, uint32_t flags);
/* EpiChord::findNode(keys[i], numRedundantNodes, 1, FindNodeCall from src[i]) at node[i] at
 * simulated time now_ns[i], each call on the loaded snapshot with the side effects the reference
 * applies before it answers (the source enters the finger cache and, where it fits, the node lists,
 * whose resize may put an evicted member under cacheTTL; EpiChord.cc:1178-1209).  src[i] =
 * 0xFFFFFFFF is a local call (msg == NULL).  out_nodes / out_last_ns: max_out slots per call
 * (max_out >= max(3, 1 + numRedundantNodes), 0xFFFFFFFF / -1 padded): the next hops and the
 * lastUpdates the EpiChordFindNodeExtMessage carries; out_count the count; out_status 0 =
 * answered, 1 = the reference throws "Failed to find node" (613-614), 2 = the reference
 * dereferences an empty finger cache (EpiChordFingerCache.cc:317-322, undefined), 3 = node or
 * source index outside the network (device-pointer calls; host calls return OVS_EINVAL).  Buffers
 * follow `flags`. */
ovs_status  ovs_epichord_find_node_batch(ovs_ctx* ctx, const uint32_t* node, const ovs_key160* keys,
                                         const uint32_t* src, const int64_t* now_ns, uint64_t n,
                                         int32_t numRedundantNodes, uint32_t* out_nodes, int64_t* out_last_ns,
                                         uint32_t max_out, uint8_t* out_count, uint8_t* out_status,
                                         uint32_t flags, void* stream);
/* copy the device Kademlia tables out (host buffers): siblings[n*5s],
 * bucket_count[n*160], bucket_nodes[n*160*k] (0xFFFFFFFF padded) */
ovs_status  ovs_kad_export(ovs_ctx* ctx, uint32_t* siblings, uint8_t* bucket_count,
                           uint32_t* bucket_nodes);
/* copy the resolved Chord finger table out: out[n*160] = getFinger(pos) */
ovs_status  ovs_chord_export_fingers(ovs_ctx* ctx, uint32_t* out);

/* Batched maintenance lookups: one synchronous fixfingers round for the listed
 * nodes of an explicit-table ring (Chord::handleFixFingersTimerExpired,
 * Chord.cc:845-875; rpcFixfingers + handleRpcFixfingersResponse, 1228-1270,
 * extendedFingerTable = false).  At every listed node the trivial fingers
 * (2^i <= succ0 - n) are removed, the lookups of n + 2^i from n are routed on
 * the device over the tables as they then are, and finger i is set to each
 * successful lookup's result.  The reference fires the nodes' timers at
 * different times; the round fixes all listed nodes at one instant.  Host
 * buffers; stats may be NULL. */
typedef struct ovs_fixfingers_stats {
    uint64_t lookups;        /* FixfingersCalls routed */
    uint64_t ok;             /* answered (lookup valid) */
    uint64_t changed;        /* finger entries that changed */
    uint64_t hops;           /* accepted hops of all lookups */
} ovs_fixfingers_stats;
ovs_status  ovs_chord_fix_fingers(ovs_ctx* ctx, const uint32_t* nodes, uint64_t m,
                                  ovs_fixfingers_stats* stats);

/* One synchronous stabilize round for the listed nodes of an explicit-table
 * ring (Chord::handleStabilizeTimerExpired -> StabilizeCall, Chord.cc:793-842,
 * 1055-1104; NotifyCall / rpcNotify / handleRpcNotifyResponse, 1106-1225;
 * ChordSuccessorList::addSuccessor / updateList / removeOldSuccessors,
 * ChordSuccessorList.cc:101-194; mergeOptimizationL1-L4 = false, no failed
 * nodes).  Every listed node v asks its successor s for its predecessor p,
 * takes p as successor when p lies in (v, s), notifies the successor t, which
 * makes v its predecessor when v lies in (pred(t), t), and replaces its list
 * by t and t's successors.  All messages of the round see the tables as they
 * stand at its start (the reference fires the nodes' timers at different
 * times); successor-list entries count as settled at the start (newEntry =
 * false).  Fingers whose resolution falls back to a changed successor follow;
 * ovs_chord_fix_fingers then repairs the fingers -- alternating the two is the
 * convergence of a ring after joins.  Host buffers; stats may be NULL. */
typedef struct ovs_stabilize_stats {
    uint64_t nodes;          /* nodes that stabilised */
    uint64_t succ_changed;   /* successors (list position 0) that changed */
    uint64_t lists_changed;  /* successor lists that changed */
    uint64_t pred_changed;   /* predecessors set by a NotifyCall */
} ovs_stabilize_stats;
ovs_status  ovs_chord_stabilize(ovs_ctx* ctx, const uint32_t* nodes, uint64_t m, ovs_stabilize_stats* stats);
/* the explicit tables as they now stand (host buffers): pred[n], succ[n*successorListSize]
 * (0xFFFFFFFF padded), nsucc[n] */
ovs_status  ovs_chord_export_tables(ovs_ctx* ctx, uint32_t* pred, uint32_t* succ, uint8_t* nsucc);

/* Batched iterative lookups: lookup i routes keys[i] from node src[i]
 * (KBRTestApp one-way test: createDestKey -> callRoute -> sendToKey ->
 * IterativeLookup -> sendRouteMessage).  hop_seq may be NULL, else
 * n*hopCountMax node indices (accepted responders in order, 0xFFFFFFFF padded).
 * rpcs may be NULL, else n FindNodeCall counts.  src[i] < n: a host-pointer call
 * returns OVS_EINVAL for a source outside the network; device-pointer calls do not
 * check (the caller's sources must be node indices). */
ovs_status  ovs_route_batch(ovs_ctx* ctx, const ovs_key160* keys, const uint32_t* src,
                            uint64_t n, ovs_route_out* out, uint32_t* hop_seq, uint32_t* rpcs,
                            uint32_t flags, void* stream);

/* Result of one LookupCall (KBRTestApp lookup test, kbrLookupTest = true:
 * KBRTestApp.cc:190-206 sends LookupCall{key, numSiblings = getMaxNumSiblings()};
 * BaseOverlay::lookupRpc, BaseOverlay.cc:1938-1968; the answer is built by
 * SendToKeyListener::lookupFinished, BaseOverlay.cc:1272-1300). */
typedef struct ovs_lookup_out {
    uint32_t num_siblings;  /* LookupResponse siblings array size (getResult().size()); 0 when !isValid */
    uint16_t hops;          /* LookupResponse hopCount = IterativeLookup::getMinHops() */
    uint8_t  status;        /* OVS_LOOKUP_* */
    uint8_t  is_valid;      /* LookupResponse isValid = lookup->isValid() */
    int64_t  latency_ns;    /* the LookupCall's RTT (an internal RPC: the lookup's duration), ns; -1 when !isValid */
} ovs_lookup_out;

/* Batched LookupCalls: lookup i resolves keys[i] at node src[i] with
 * num_siblings siblings (-1 = getMaxNumSiblings(): Chord successorListSize,
 * Kademlia s; larger than that is OVS_EINVAL like the reference's
 * "numSiblings too big!"; 0 = an exact-key lookup: the lookup ends at the first
 * response that carries the key's node, IterativeLookup.cc:171-184, 862-870;
 * Chord's responsible node answers nothing then, Chord.cc:573-580).  siblings = n*max(num_siblings, 1) node indices, the
 * response's sibling vector in order, 0xFFFFFFFF padded.  Iterative routing,
 * single-context (unsharded) networks.  Sources as ovs_route_batch (host calls check them). */
ovs_status  ovs_lookup_batch(ovs_ctx* ctx, const ovs_key160* keys, const uint32_t* src,
                             uint64_t n, int32_t num_siblings, ovs_lookup_out* out,
                             uint32_t* siblings, uint32_t flags, void* stream);

/* Batched Kademlia refresh lookups (Kademlia::handleBucketRefreshTimerExpired,
 * Kademlia.cc:1591-1686, exhaustiveRefresh = true, iterative routing):
 * lookup i is createLookup(EXHAUSTIVE_ITERATIVE_ROUTING)->lookup(keys[i],
 * R, hopCountMax) from node src[i] with config.redundantNodes = R
 * (bucketRefreshNodes = k for a bucket refresh, siblingRefreshNodes = 5s for
 * the sibling-table refresh of the node's own key; IterativeLookup.cc:
 * 133-244, 488-585, 714-781, 803-921, 935-1170 with the exhaustive rules).
 * out / siblings as ovs_lookup_batch (siblings = n*R, the lookup's result:
 * nextHops[0..R) when it ran out of unqueried nodes).  responders (may be NULL)
 * = n*hopCountMax node indices, every FindNodeResponse the lookup received in
 * order -- the nodes Kademlia::handleRpcResponse routingAdd()s with their RTT
 * (Kademlia.cc:1352-1420) -- 0xFFFFFFFF padded; rtt_ns (may be NULL) their
 * RTTs, -1 padded; rpcs (may be NULL) = n FindNodeCall counts.  Requires
 * lookupMerge, lookupStrictParallelRpcs, lookupParallelRpcs <= 8,
 * 1 <= R <= 64, 1 <= hopCountMax.  Single-context networks. */
ovs_status  ovs_kad_refresh_batch(ovs_ctx* ctx, const ovs_key160* keys, const uint32_t* src, uint64_t n,
                                  int32_t redundant_nodes, ovs_lookup_out* out, uint32_t* siblings,
                                  uint32_t* responders, int64_t* rtt_ns, uint32_t* rpcs, uint32_t flags,
                                  void* stream);
/* One synchronous Kademlia maintenance round (ABI 9; replaces the bucket / sibling refresh
 * timers and Kademlia::routingAdd, Kademlia.cc:432-756, 1328-1420, 1591-1686, for a NoChurn
 * network).  For nodes[0..m): flags[j] bit 0 = the sibling-table refresh (an exhaustive-iterative
 * lookup of the node's own key with siblingRefreshNodes = 5s), bit 1 = the bucket refreshes of the
 * buckets stale[j*5..] marks (NULL = all; key self ^ 2^i, bucketRefreshNodes =
 * lookupRedundantNodes); flags NULL = both.  All lookups run on the device over the tables of the
 * round's start; then every node applies routingAdd, on the host, for each FindNodeCall that
 * reached it (handleRpcCall: the caller, alive) and each FindNodeResponse its lookups handled
 * (handleRpcResponse: the carried nodes, not alive, then the responder, alive) in simulated-time
 * order -- every lookup of the round starts at its instant 0; ties: calls first, then lookup and
 * message order -- with secureMaintenance, pingNewSiblings, activePing and PNS off (the
 * defaults) and bucketType "kademlia".  The device tables are rebuilt from the result.  Needs the
 * whole network in this context (ovs_kad_load or ovs_kad_load_tables); nodes / flags / stale are
 * host buffers; stats may be NULL. */
typedef struct ovs_kad_round_stats {
    uint64_t lookups;        /* refresh lookups routed */
    uint64_t failed;         /* lookups that did not end successfully (hopCountMax, timeouts) */
    uint64_t responses;      /* FindNodeResponses applied */
    uint64_t sib_changes;    /* handles inserted into a sibling table */
    uint64_t bucket_changes; /* handles inserted into a bucket */
    uint64_t lost;           /* preempted siblings whose bucket was full */
    uint64_t replacement;    /* alive handles a full bucket turned away (replacement cache) */
    uint64_t refreshed;      /* alive handles already known (LRU move / sibling refresh) */
} ovs_kad_round_stats;
ovs_status  ovs_kad_maintenance_round(ovs_ctx* ctx, const uint32_t* nodes, uint64_t m, const uint8_t* flags,
                                      const uint32_t* stale, ovs_kad_round_stats* stats);
/* The bucket-refresh lookups of nodes[0..m) (Kademlia.cc:1631-1676, b = 1):
 * key self ^ 2^i from the node for i = 159 down to msb(self ^ closest sibling)
 * where bit i of the node's stale mask is set -- stale = m*5 words (bit i of
 * word i/32: bucket i is NULL or unused for minBucketRefreshInterval), NULL =
 * every bucket.  Writes up to cap (keys, src) pairs in the reference's order
 * and sets *count to how many there are (keys/src may be NULL with cap 0 to
 * size the call).  nodes / stale / keys / src follow `flags`; *count is host. */
ovs_status  ovs_kad_refresh_keys(ovs_ctx* ctx, const uint32_t* nodes, uint64_t m, const uint32_t* stale,
                                 ovs_key160* keys, uint32_t* src, uint64_t cap, uint64_t* count,
                                 uint32_t flags, void* stream);

/* Batched responder step: for each i, findNode(keys[i], numRedundantNodes,
 * numSiblings) evaluated at node[i] and the findNodeRpc siblings flag
 * isSiblingFor(node[i], keys[i], numSiblings).  Kademlia also takes
 * numSiblings = -1: the FindNodeCall of an exhaustive-iterative lookup
 * (resultSize = numRedundantNodes, no siblings flag; BaseOverlay.cc:1857-1871).  out_nodes has max_out slots per
 * query (0xFFFFFFFF padded), out_count the result size. */
ovs_status  ovs_find_node_batch(ovs_ctx* ctx, const uint32_t* node, const ovs_key160* keys,
                                uint64_t n, int32_t numRedundantNodes, int32_t numSiblings,
                                uint32_t* out_nodes, uint32_t max_out, uint8_t* out_count,
                                uint8_t* out_sibling, uint32_t flags, void* stream);

/* SimpleNodeEntry::calcDelay (idle queues) for n (a,b,bytes) triples, in ns */
ovs_status  ovs_delay_batch(ovs_ctx* ctx, const uint32_t* a, const uint32_t* b,
                            const int32_t* bytes, uint64_t n, int64_t* out_ns,
                            uint32_t flags, void* stream);

ovs_status  ovs_sync(ovs_ctx* ctx);

/* ---- KBRTestApp statistics (one-way test) ----
 * Replaces the statistics a KBRTestApp run hands to GlobalStatistics:
 *   KBRTestApp::evaluateData -> recordOutVector("KBRTestApp: One-way Hop Count" /
 *     "One-way Latency")                    KBRTestApp.cc:479-496
 *   KBRTestApp::deliver lookupNodeIds check  KBRTestApp.cc:380-440 (numDropped)
 *   KBRTestApp::finishApp -> addStdDev(...)  KBRTestApp.cc:498-520
 *   SendToKeyListener failed lookup          BaseOverlay.cc:1258-1270 (overlay numDropped)
 *   GlobalStatistics::finalizeStatistics     GlobalStatistics.cc:103-140 (".mean" scalars)
 * One cStdDev summary over the nodes of the network (every node runs
 * finishApp; the delivery ratio only for nodes with numSent > 0). */
typedef struct ovs_stddev {
    uint64_t count;
    double   mean, stddev, min, max;    /* cStdDev: stddev = sample (n-1) deviation, 0 if n < 2 */
} ovs_stddev;

typedef struct ovs_kbrtest_stats {
    uint64_t num_sent;               /* one-way test messages (= lookups in the batch) */
    uint64_t num_delivered;          /* evaluateData calls */
    uint64_t num_dropped;            /* lookupNodeIds: delivered to a node whose key != destKey */
    uint64_t num_lookup_failed;      /* !isValid(): dropped by SendToKeyListener (overlay numDropped) */
    uint64_t bytes_sent, bytes_delivered, bytes_dropped;
    uint64_t hop_count_sum;          /* sum of One-way Hop Count over delivered messages */
    int64_t  latency_sum_ns;         /* sum of One-way Latency over delivered messages */
    uint32_t hop_count_min, hop_count_max;
    int64_t  latency_min_ns, latency_max_ns;
    double   hop_count_mean;         /* "Vector: KBRTestApp: One-way Hop Count.mean" */
    double   latency_mean_s;         /* "Vector: KBRTestApp: One-way Latency.mean" */
    uint64_t status_count[8];        /* lookups by OVS_LOOKUP_* status */
    uint64_t hop_hist[64];           /* delivered messages by one-way hop count (63 = 63 or more) */
    ovs_stddev delivered_msgs_per_s; /* "KBRTestApp: One-way Delivered Messages/s" */
    ovs_stddev delivered_bytes_per_s;
    ovs_stddev dropped_msgs_per_s;
    ovs_stddev dropped_bytes_per_s;
    ovs_stddev delivery_ratio;       /* "KBRTestApp: One-way Delivery Ratio" ((float)d / (float)s) */
} ovs_kbrtest_stats;

/* Reduce a batch of route results (out/keys/src as passed to ovs_route_batch)
 * to KBRTestApp statistics.  measured_time_s = each node's measured lifetime
 * (GlobalStatistics::calcMeasuredLifetime); per-node rates are only produced
 * when it is >= GlobalStatistics::MIN_MEASURED = 0.1 s.  lookup_node_ids =
 * the kbrTestApp.lookupNodeIds parameter; message sizes come from
 * testMsgSize.  *stats is host memory; out/keys/src follow `flags`. */
ovs_status  ovs_kbrtest_stats_batch(ovs_ctx* ctx, const ovs_route_out* out, const ovs_key160* keys,
                                    const uint32_t* src, uint64_t n, double measured_time_s,
                                    int32_t lookup_node_ids, ovs_kbrtest_stats* stats,
                                    uint32_t flags, void* stream);

/* ---- KBRTestApp statistics (lookup test, kbrLookupTest = true) ----
 *   KBRTestApp::handleLookupResponse / RPC timeout  KBRTestApp.cc:315-371
 *     success = isValid && (!lookupNodeIds || siblings[0] is the node owning the key);
 *     recordOutVector("KBRTestApp: Lookup Success Latency" / "Lookup Total Latency" /
 *     "Lookup Hop Count"), failures: "Lookup Total Latency" = failureLatency,
 *     "Failed Lookup Hop Count"
 *   KBRTestApp::finishApp                          KBRTestApp.cc:546-557 */
typedef struct ovs_kbrtest_lookup_stats {
    uint64_t num_sent;               /* numLookupSent (= lookups in the batch) */
    uint64_t num_success;            /* numLookupSuccess */
    uint64_t num_failed;             /* numLookupFailed */
    uint64_t num_invalid;            /* the failed lookups with isValid == false */
    uint64_t hop_count_sum;          /* "Lookup Hop Count" over successful lookups */
    uint64_t failed_hop_count_sum;   /* "Failed Lookup Hop Count" */
    int64_t  success_latency_sum_ns; /* "Lookup Success Latency" */
    uint32_t hop_count_min, hop_count_max;
    int64_t  success_latency_min_ns, success_latency_max_ns;
    double   hop_count_mean;         /* "Vector: KBRTestApp: Lookup Hop Count.mean" */
    double   failed_hop_count_mean;  /* "Vector: KBRTestApp: Failed Lookup Hop Count.mean" */
    double   success_latency_mean_s; /* "Vector: KBRTestApp: Lookup Success Latency.mean" */
    double   total_latency_mean_s;   /* "Vector: KBRTestApp: Lookup Total Latency.mean" */
    uint64_t status_count[8];        /* lookups by OVS_LOOKUP_* status */
    uint64_t hop_hist[64];           /* successful lookups by hop count (63 = 63 or more) */
    ovs_stddev successful_lookups_per_s;  /* "KBRTestApp: Successful Lookups/s" */
    ovs_stddev failed_lookups_per_s;      /* "KBRTestApp: Failed Lookups/s" */
    ovs_stddev success_ratio;             /* "KBRTestApp: Lookup Success Ratio" ((float)s / (float)sent) */
} ovs_kbrtest_lookup_stats;

/* Reduce a batch of LookupCall results (out/siblings/keys/src as passed to
 * ovs_lookup_batch; siblings_stride = its num_siblings) to the KBRTestApp lookup
 * statistics.  failure_latency_s = kbrTestApp.failureLatency (default.ini:41, 10 s). */
ovs_status  ovs_kbrtest_lookup_stats_batch(ovs_ctx* ctx, const ovs_lookup_out* out, const uint32_t* siblings,
                                           int32_t siblings_stride, const ovs_key160* keys, const uint32_t* src,
                                           uint64_t n, double measured_time_s, int32_t lookup_node_ids,
                                           double failure_latency_s, ovs_kbrtest_lookup_stats* stats,
                                           uint32_t flags, void* stream);

/* ---- multi-GPU sharding (one process per GPU; the host exchanges records) ----
 * The sorted ring is cut into contiguous arcs, one per rank.  Node keys,
 * coordinates and 64 B node records are replicated; the finger rows -- the bulk
 * of the routing state -- exist only for the rank's own arc, so a lookup is
 * handed to the rank that owns its next responder.  The exchange of in-flight
 * records between hop rounds is done by the caller (RCCL all-to-allv over xGMI,
 * see oversim_amd/shard.py).  All shard calls take device pointers. */
typedef struct ovs_lookup_rec {     /* 48 B in-flight lookup */
    uint32_t key[5];                /* lookup key */
    uint32_t src;                   /* global index of the source node */
    uint32_t cur;                   /* global index of the node whose findNode runs next */
    uint32_t qid;                   /* caller's lookup id */
    int64_t  t_ns;                  /* simulated time since lookup start */
    uint16_t hops;
    uint8_t  local;                 /* 1: the source's local step (no hop, no delay) is pending;
                                       2: `cur` was reached (its response accounted) on another rank,
                                          only its findNode decision is pending (replicated levels) */
    uint8_t  pad[5];
} ovs_lookup_rec;

typedef struct ovs_done_rec {       /* 24 B finished lookup */
    uint32_t qid;
    uint32_t pad;                   /* Kademlia shard step: the lookup's FindNodeCalls; 0 otherwise */
    ovs_route_out out;
} ovs_done_rec;

/* Load arc [lo, hi) of a Chord ring of n_total nodes (ids/xy of the whole ring). */
ovs_status  ovs_chord_load_shard(ovs_ctx* ctx, const ovs_key160* ids_all_sorted, uint64_t n_total,
                                 const double* xy_all, uint64_t lo, uint64_t hi, uint32_t flags);
/* Replicate the top `top_levels` finger levels (fingers 159 .. 160 - top_levels) of EVERY node of
 * the ring on this arc's context (ABI 11; 64 B per node and level: 2^26 nodes x 4 levels = 17 GB).
 * A lookup's first hops are its long jumps, and they are the ones whose responders lie on other
 * arcs: a responder off this arc whose next finger probe falls in the replicated levels is decided
 * here, from the same finger the owner's row holds (Chord.cc:602-674, ChordFingerTable.cc:174-193),
 * so the lookup crosses to another arc about once instead of once per long hop.  A decision that
 * needs the owner's rows after all (a finger below the replicated levels, the successor window) is
 * handed to the owner as a record with local = 2.  0 = none (the default). */
ovs_status  ovs_chord_shard_replicate(ovs_ctx* ctx, int32_t top_levels);
int32_t     ovs_chord_shard_levels(const ovs_ctx* ctx);
/* Initial records for lookups whose sources lie on this arc: qid = qid_base + i. */
ovs_status  ovs_shard_make_records(ovs_ctx* ctx, const ovs_key160* keys, const uint32_t* src,
                                   uint64_t n, uint32_t qid_base, ovs_lookup_rec* recs, void* stream);
/* One hop round: advance every record of `in` while its responder is on this
 * arc.  A record whose next responder lies on arc d != this one is appended to
 * segment d of `out` (out + d * out_cap records, the send buffer of the
 * all-to-allv, grouped by destination in the kernel itself) and counted in
 * out_count[d]; finished lookups are appended to `done` (done_count).
 * out_count (nshards counters) and done_count are device counters the kernel
 * increments; the caller zeroes them.  A segment never receives more than
 * n_in records, so out_cap = n_in is always enough.
 * shard_lo is a HOST array of nshards+1 arc boundaries (sorted-index space). */
ovs_status  ovs_shard_step(ovs_ctx* ctx, const ovs_lookup_rec* in, uint64_t n_in,
                           ovs_lookup_rec* out, uint64_t out_cap, unsigned long long* out_count,
                           ovs_done_rec* done, uint64_t done_cap, unsigned long long* done_count,
                           const uint64_t* shard_lo, uint32_t nshards, void* stream);

/* LookupCalls across arcs (KBRTestApp lookup test on a sharded ring): rounds as
 * ovs_shard_step, with num_siblings (-1 = successorListSize, at most 8): the
 * responsible node's FindNodeResponse carries the sibling vector and the lookup
 * ends there (no route message).  ovs_shard_lookup_finish turns n finished
 * records (from `done`, any order) into the LookupResponses, in that order:
 * out[i] and siblings[i * num_siblings] (0xFFFFFFFF padded) for done[i].qid.
 * The successor lists of a converged ring are replicated, so any rank finishes
 * any record.  Device buffers. */
ovs_status  ovs_shard_step_lookup(ovs_ctx* ctx, int32_t num_siblings, const ovs_lookup_rec* in, uint64_t n_in,
                                  ovs_lookup_rec* out, uint64_t out_cap, unsigned long long* out_count,
                                  ovs_done_rec* done, uint64_t done_cap, unsigned long long* done_count,
                                  const uint64_t* shard_lo, uint32_t nshards, void* stream);
/* The first round of a batch straight from its keys and sources (device memory, ABI 10): the same
 * as ovs_shard_make_records followed by ovs_shard_step / ovs_shard_step_lookup on those records,
 * without writing and reading them (lookup i has qid qid_base + i).  num_siblings 0: one-way KBR
 * routes (ovs_shard_step); otherwise LookupCalls with that many siblings (-1 = successorListSize). */
ovs_status  ovs_shard_step_keys(ovs_ctx* ctx, int32_t num_siblings, const ovs_key160* keys, const uint32_t* src,
                                uint64_t n, uint32_t qid_base, ovs_lookup_rec* out, uint64_t out_cap,
                                unsigned long long* out_count, ovs_done_rec* done, uint64_t done_cap,
                                unsigned long long* done_count, const uint64_t* shard_lo, uint32_t nshards,
                                void* stream);
ovs_status  ovs_shard_lookup_finish(ovs_ctx* ctx, const ovs_done_rec* done, uint64_t n, int32_t num_siblings,
                                    ovs_lookup_out* out, uint32_t* siblings, void* stream);

/* ---- multi-GPU Kademlia ----
 * The sorted ring is cut into contiguous arcs (ID prefixes); a rank holds the
 * sibling entries and bucket rows of its arc, while the 64 B node records and
 * coordinates are replicated.  A lookup stays on the rank of its source; every
 * FindNodeCall it sends becomes a request to the rank owning the responder, whose
 * findNode result (Kademlia.cc:1101-1246) comes back before the lookup's next
 * round -- before the simulated response is processed.  A FindNodeCall to a node of
 * the rank's own arc is answered on the spot (at world size 1 the first round
 * finishes every lookup).  Per round the caller runs ovs_kad_shard_step, gathers
 * every rank's out_count[0..nshards) and *active_count (the round's one host
 * synchronisation), exchanges the requests (all-to-allv of the per-owner
 * segments), runs ovs_kad_shard_serve on what it received, sends the responses
 * back with the reverse splits and hands them to ovs_kad_shard_deliver; it stops
 * when every rank's requests and active lookups are 0.  All buffers are device
 * memory. */
typedef struct ovs_kad_req {        /* 32 B FindNodeCall */
    uint32_t key[5];
    uint32_t node;                  /* responder (global index, on the receiving rank's arc) */
    uint32_t tag;                   /* opaque to the receiver; returned in the response */
    uint32_t pad;                   /* LookupCall: 0x80000000 | numSiblings of findNode; 0 = KBR route */
} ovs_kad_req;

typedef struct ovs_kad_resp {       /* 104 B FindNodeResponse */
    uint32_t tag;
    uint32_t count;                 /* result size, <= 8 */
    uint32_t nodes[8];
    uint64_t dist_hi[8];            /* top 64 bits of (node key XOR lookup key) */
} ovs_kad_resp;

/* The FindNodeResponse record of KademliaLarge networks (k or lookupRedundantNodes 9..16,
 * omnetpp.ini:113-126): ovs_kad_shard_serve writes and ovs_kad_shard_deliver reads these when
 * ovs_kad_shard_resp_bytes(ctx) says 200 (ABI 10). */
typedef struct ovs_kad_resp16 {     /* 200 B */
    uint32_t tag;
    uint32_t count;                 /* result size, <= 16 */
    uint32_t nodes[16];
    uint64_t dist_hi[16];
} ovs_kad_resp16;

/* Load arc [lo, hi) of a Kademlia network of n_total nodes (ids/xy of all nodes). */
ovs_status  ovs_kad_load_shard(ovs_ctx* ctx, const ovs_key160* ids_all_sorted, uint64_t n_total,
                               const double* xy_all, uint64_t lo, uint64_t hi, uint32_t flags);
/* Start a batch of lookups whose sources lie on this arc (lookup id = qid_base + i). */
ovs_status  ovs_kad_shard_begin(ovs_ctx* ctx, const ovs_key160* keys, const uint32_t* src, uint64_t n,
                                uint32_t qid_base, void* stream);
/* LookupCalls (KBRTestApp lookup test, BaseOverlay::lookupRpc) on a sharded network:
 * as ovs_kad_shard_begin, with num_siblings (-1 = s, 0 = exact-key lookup, at most 8;
 * replaces ovs_lookup_batch's single-GPU LookupCall).  The rounds are the same calls;
 * each request then carries numSiblings (ovs_kad_req.pad), so the serving rank answers
 * findNode(key, numRedundantNodes, numSiblings).  A finished lookup's done record holds
 * its LookupResponse (an ovs_lookup_out in the ovs_route_out slot) and its sibling
 * vector goes to siblings[(qid - qid_base) * max(num_siblings, 1)], 0xFFFFFFFF padded:
 * device memory of n rows that stays valid until the batch ends. */
ovs_status  ovs_kad_shard_begin_lookup(ovs_ctx* ctx, int32_t num_siblings, const ovs_key160* keys,
                                       const uint32_t* src, uint64_t n, uint32_t qid_base,
                                       uint32_t* siblings, void* stream);
/* One round for this rank's lookups (ABI 7).  Requests for rank d go to segment d of
 * `out` (out + d * out_cap requests; out_cap >= n * lookupParallelRpcs, n * 8 when
 * lookupParallelRpcs is 5..8: a lookup owns 1, 2, 3, 4 or 8 pending-call slots) and are
 * counted in out_count[d]; finished lookups are appended to `done` (done_count).
 * out_count[0..nshards) and done_count are device counters the step adds to (the
 * caller zeroes out_count before each round, done_count once per batch);
 * *active_count is set to the lookups still running after the round.
 * shard_lo: HOST array of nshards+1 arc bounds. */
ovs_status  ovs_kad_shard_step(ovs_ctx* ctx, ovs_kad_req* out, uint64_t out_cap, unsigned long long* out_count,
                               ovs_done_rec* done, uint64_t done_cap, unsigned long long* done_count,
                               unsigned long long* active_count, const uint64_t* shard_lo, uint32_t nshards,
                               void* stream);
/* Bytes of this context's response records: 104 (ovs_kad_resp) when k and lookupRedundantNodes
 * are <= 8, else 200 (ovs_kad_resp16); -1 without a Kademlia network. */
int32_t     ovs_kad_shard_resp_bytes(const ovs_ctx* ctx);
/* findNode at the (local) responders of n received requests; out = n response records of
 * ovs_kad_shard_resp_bytes(ctx) bytes. */
ovs_status  ovs_kad_shard_serve(ovs_ctx* ctx, const ovs_kad_req* in, uint64_t n, void* out,
                                void* stream);
/* Hand n responses (to this rank's requests) back to the waiting lookups.  A response
 * with an unknown tag, or one the serving rank could not answer (the request named a
 * node outside its arc: count 0xFFFFFFFF), is counted as an error; the latter still
 * completes its slot with an empty result, so the lookup terminates. */
ovs_status  ovs_kad_shard_deliver(ovs_ctx* ctx, const void* in, uint64_t n, void* stream);
/* Errors since ovs_kad_shard_begin: responses ovs_kad_shard_deliver could not hand over,
 * and lookups whose source lies off this arc (they never run).  Synchronises the
 * device.  The caller fails the batch when it is non-zero. */
ovs_status  ovs_kad_shard_errors(ovs_ctx* ctx, uint64_t* bad);

/* Kademlia lookups that MIGRATE (ABI 11).  Under the XOR-prefix partition a lookup's late
 * FindNodeCalls all go to nodes within 2^(160 - log2 W) of its key, i.e. to the key's own arc, and
 * its early ones to nodes anywhere.  ovs_kad_shard_replicate keeps the top `top_levels` buckets of
 * EVERY node on every rank (96 B per node and level): a findNode whose answer is a full main bucket
 * among them (the long first hops) is answered on any rank, and a lookup whose next findNode needs
 * another arc's rows moves there as one record (ovs_kad_shard_rec_bytes bytes: its whole
 * IterativeLookup state) instead of exchanging a request and a response per call -- on prefix arcs
 * it moves at most once, to its key's arc.  Rebuilds the arc's tables; 0 = none.  The results are
 * the single-context K2's (the same event order, findNode answers and delays). */
ovs_status  ovs_kad_shard_replicate(ovs_ctx* ctx, int32_t top_levels);
int32_t     ovs_kad_shard_levels(const ovs_ctx* ctx);
int32_t     ovs_kad_shard_rec_bytes(const ovs_ctx* ctx);
/* One migration round (one-way KBR routes): advance the lookups of `in` (n_in records of
 * ovs_kad_shard_rec_bytes bytes) -- or, in a batch's first round (in == NULL), n_in lookups from
 * fkeys / fsrc with ids fqid + i -- until each finishes (appended to done, done_count) or needs
 * another rank's rows (appended to segment d of out: out + d * out_cap records, out_count[d]).
 * A segment never receives more than n_in records.  Lookups finish on whichever rank holds them
 * last.  shard_lo: HOST array of nshards + 1 arc bounds; errors via ovs_kad_shard_errors. */
ovs_status  ovs_kad_shard_mig_step(ovs_ctx* ctx, const void* in, uint64_t n_in, const ovs_key160* fkeys,
                                   const uint32_t* fsrc, uint32_t fqid, void* out, uint64_t out_cap,
                                   unsigned long long* out_count, ovs_done_rec* done, uint64_t done_cap,
                                   unsigned long long* done_count, const uint64_t* shard_lo, uint32_t nshards,
                                   void* stream);

/* ---------------------------------------------------------------------------
 * Sharded routing behind the ABI (ABI 11): the whole multi-GPU batch in one call.
 *
 * Replaces BaseOverlay::sendToKey's iterative branch (src/common/BaseOverlay.cc:1367-1442) for a
 * network whose tables are split over the ranks (one context per GPU, one process or thread per
 * rank).  The round loop -- step kernels, the per-round count all-gather, the all-to-allv of the
 * records, the completeness check -- runs in C++ inside the library; every rank calls the entry
 * point collectively with the same exchange.  The exchange is a table of callbacks:
 * ovs_exchange_rccl_create fills it with RCCL over xGMI (ncclSend / ncclRecv groups, one
 * communicator, collectives serialised on one communicator stream); ovs_exchange_local_create with
 * W ranks that are threads of one process (contexts on one or more devices, device-to-device
 * copies); a caller may plug its own (tests: gloo through Python callbacks).  All callbacks are
 * collective and are called in the same order on every rank; they return 0 on success. */
typedef struct ovs_exchange {
    void* user;
    uint32_t rank, world;
    /* every rank contributes n host int64 (host_send); on return host_recv[world * n] (rank-major)
     * holds all contributions -- the round's count matrix, the loop's one host synchronisation */
    int (*allgather_i64)(void* user, const int64_t* host_send, uint32_t n, int64_t* host_recv);
    /* all-to-allv of row_bytes-sized rows in DEVICE memory: the rows for rank d are send[d]
     * (send_rows[d] of them); the rows from rank s land at recv + recv_off[s] * row_bytes
     * (recv_rows[s] of them).  Ordered after the work queued on `stream`; work queued on `stream`
     * afterwards sees the received rows (the callback may return before the transfer ends) */
    int (*alltoallv)(void* user, const void* const* send, const uint64_t* send_rows, void* recv,
                     const uint64_t* recv_off, const uint64_t* recv_rows, uint32_t row_bytes, void* stream);
    /* element-wise sum over the ranks of n host int64, in place */
    int (*allreduce_sum_i64)(void* user, int64_t* values, uint32_t n);
    /* releases `user` (ovs_exchange_destroy); may be NULL */
    void (*destroy)(void* user);
} ovs_exchange;

/* RCCL exchange for rank `rank` of `world` on HIP device `device`.  unique_id: the 128 bytes
 * ovs_rccl_unique_id produced on rank 0 and the caller distributed (as ncclGetUniqueId's).  RCCL is
 * loaded at run time (the process's librccl.so.1 when one is loaded, else /opt/rocm's). */
ovs_status  ovs_rccl_unique_id(void* unique_id_128);
ovs_status  ovs_exchange_rccl_create(int device, uint32_t rank, uint32_t world, const void* unique_id_128,
                                     ovs_exchange* out);
/* W in-process ranks (threads): fills out[0..world), one exchange per rank */
ovs_status  ovs_exchange_local_create(uint32_t world, ovs_exchange* out);
void        ovs_exchange_destroy(ovs_exchange* ex);
/* The last RCCL / exchange error text of this thread (ovs_exchange_* calls have no context) */
const char* ovs_exchange_last_error(void);
/* The collective the process's round loop last entered ("count allgather", "records alltoallv",
 * "completeness allreduce", ..., "idle") and its round: for a caller's watchdog to name a stuck
 * stage.  Safe to call from any thread (ABI 12).  A failure only one rank sees (allocation, launch,
 * segment or done-buffer overflow, a rank-local precondition) is carried by the next collective,
 * so every rank of a sharded route returns a failure from the same round instead of blocking. */
const char* ovs_exchange_stage(uint32_t* round);

typedef struct ovs_shard_route_stats {
    uint32_t rounds;         /* hop rounds (Chord) / request rounds (Kademlia) of the batch */
    uint32_t cohorts;
    uint64_t sent;           /* records this rank sent to other ranks (hand-offs / FindNodeCalls) */
    uint64_t sent_bytes;     /* ... and their bytes, responses included (Kademlia) */
    uint64_t done;           /* lookups that finished on this rank */
    double   step_ms;        /* step kernels incl. compaction (HIP events), summed over rounds */
    double   exchange_ms;    /* host wall time inside the exchange callbacks */
    double   total_ms;       /* host wall time of the call */
} ovs_shard_route_stats;

/* Route one batch of Chord lookups whose sources lie on this context's arc (ovs_chord_load_shard;
 * lookup i has qid qid_base + i).  shard_lo: HOST array of world + 1 arc bounds (every rank's).
 * num_siblings 0: one-way KBR routes; otherwise LookupCalls with that many siblings (-1 =
 * successorListSize; finish them with ovs_shard_lookup_finish).  keys / src / done are DEVICE
 * buffers; a lookup finishes on whichever rank holds it last, so done_cap must hold every record
 * that can finish here (the total over all ranks is always enough); *n_done = records in done.
 * cohorts (1..4, 0 = 2): the batch is split so one cohort's exchange overlaps another's kernel.
 * The call returns when the batch is complete on every rank: it fails (OVS_EDEVICE) when the
 * records finished on all ranks do not add up to the lookups started, or when a finished record came
 * from an exchange row nobody wrote (receive buffers are 0xFF-filled).  stats may be NULL. */
ovs_status  ovs_shard_route_batch(ovs_ctx* ctx, const ovs_exchange* ex, const uint64_t* shard_lo,
                                  int32_t num_siblings, const ovs_key160* keys, const uint32_t* src, uint64_t n,
                                  uint32_t qid_base, ovs_done_rec* done, uint64_t done_cap, uint64_t* n_done,
                                  uint32_t cohorts, ovs_shard_route_stats* stats, void* stream);
/* The same for Kademlia (ovs_kad_load_shard): num_siblings OVS_KAD_ONEWAY: one-way KBR routes;
 * -1 / 0..8: LookupCalls (as ovs_kad_shard_begin_lookup; siblings = n rows of max(num_siblings, 1),
 * device memory).  One-way routes on a context with replicated top buckets (ovs_kad_shard_replicate)
 * MIGRATE (ovs_kad_shard_mig_step rounds; a lookup finishes on any rank, so done_cap must hold every
 * record that can finish here, as for Chord); otherwise the lookups stay home and FindNodeCalls and
 * their responses are exchanged (done receives exactly this rank's n lookups, done_cap >= n).
 * done[i].pad = the lookup's FindNodeCalls. */
ovs_status  ovs_kad_shard_route_batch(ovs_ctx* ctx, const ovs_exchange* ex, const uint64_t* shard_lo,
                                      int32_t num_siblings, const ovs_key160* keys, const uint32_t* src, uint64_t n,
                                      uint32_t qid_base, ovs_done_rec* done, uint64_t done_cap, uint64_t* n_done,
                                      uint32_t* siblings, ovs_shard_route_stats* stats, void* stream);
#define OVS_KAD_ONEWAY (-2)

#ifdef __cplusplus
}
#endif
#endif /* OVS_KBR_H */
