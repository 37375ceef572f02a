/*
 * ovs_oracle.c -- CPU restatement of OverSim's iterative KBR lookup path.
 *
 * TEST INFRASTRUCTURE ONLY (see ovs_oracle.h).  This is the checker for the
 * MI355X engine; it is never linked into, called by, or used as a fallback of
 * the product library.
 *
 * Layout of this file follows the reference:
 *   1. OverlayKey on GMP-style 64-bit limbs   (src/common/OverlayKey.cc)
 *   2. BaseKeySortedVector::add                (src/common/NodeVector.h:381-512)
 *   3. SimpleUnderlay delay                    (src/underlay/simpleunderlay/SimpleNodeEntry.cc:145-195,
 *                                               SimpleUDP.cc:320-373)
 *   4. Chord stable state + routing            (src/overlay/chord/Chord.cc, ChordFingerTable.cc,
 *                                               ChordSuccessorList.cc)
 *   5. Kademlia snapshot + routing             (src/overlay/kademlia/Kademlia.cc)
 *   6. IterativeLookup / IterativePathLookup   (src/common/IterativeLookup.cc) driven by a
 *      per-lookup future-event list in simulated int64 ns.
 *
 * Compile with -ffp-contract=off: the delay arithmetic must round exactly like
 * the reference's x86-64 build (no FMA contraction).
 */
#include "ovs_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static __thread char g_err[256];
static void set_err(const char* m) { snprintf(g_err, sizeof g_err, "%s", m); }

/* A fixed capacity of this restatement was exceeded (e.g. more than MAXRPC RPCs in one lookup).
 * Never truncated silently: the first breach is recorded here, from any OpenMP thread, and the
 * batch entry points fail (orc_route_batch returns ORC_FAIL, orc_lookup_batch -1). */
static volatile int g_cap_fail = 0;
static char g_cap_msg[256];
static void cap_error(const char* m)
{
    if (__sync_bool_compare_and_swap(&g_cap_fail, 0, 1)) snprintf(g_cap_msg, sizeof g_cap_msg, "capacity exceeded: %s", m);
}
const char* orc_last_error(void) { return g_cap_fail ? g_cap_msg : g_err; }
int orc_cap_failed(void) { return g_cap_fail; }
void orc_clear_error(void) { g_cap_fail = 0; g_cap_msg[0] = 0; g_err[0] = 0; }

/* ===================================================================== */
/* 1. OverlayKey (OverlayKey.cc) with keyLength=160 => aSize=3 limbs of   */
/*    64 bits, GMP_MSB_MASK = 2^32-1 (OverlayKey.cc:41-47,143-148).        */
/* ===================================================================== */
#define A_SIZE 3
#define MSB_MASK 0xFFFFFFFFull
typedef struct { uint64_t key[A_SIZE]; int isUnspec; } OKey;

static OKey ok_from(const orc_key* k)
{
    OKey r;
    r.key[0] = (uint64_t)k->w[0] | ((uint64_t)k->w[1] << 32);
    r.key[1] = (uint64_t)k->w[2] | ((uint64_t)k->w[3] << 32);
    r.key[2] = (uint64_t)k->w[4];
    r.isUnspec = 0;
    return r;
}
static void ok_to(const OKey* k, orc_key* o)
{
    o->w[0] = (uint32_t)k->key[0]; o->w[1] = (uint32_t)(k->key[0] >> 32);
    o->w[2] = (uint32_t)k->key[1]; o->w[3] = (uint32_t)(k->key[1] >> 32);
    o->w[4] = (uint32_t)k->key[2];
}
static void ok_trim(OKey* k) { k->key[A_SIZE - 1] &= MSB_MASK; }           /* 835-838 */

static int g_unspec_cmp = 0;  /* compareTo on unspecified keys -> opp_error (844-845) */
static int ok_cmp(const OKey* a, const OKey* b)                           /* 842-847: mpn_cmp */
{
    if (a->isUnspec || b->isUnspec) { g_unspec_cmp = 1; return 0; }
    for (int i = A_SIZE - 1; i >= 0; --i) {
        if (a->key[i] != b->key[i]) return a->key[i] > b->key[i] ? 1 : -1;
    }
    return 0;
}
static OKey ok_add(OKey a, const OKey* b)                                 /* 247-253 */
{
    uint64_t c = 0;
    for (int i = 0; i < A_SIZE; ++i) {                                     /* mpn_add_n */
        uint64_t s = a.key[i] + b->key[i];
        uint64_t c1 = s < a.key[i];
        uint64_t s2 = s + c;
        uint64_t c2 = s2 < s;
        a.key[i] = s2; c = c1 | c2;
    }
    ok_trim(&a); a.isUnspec = 0; return a;
}
static OKey ok_sub(OKey a, const OKey* b)                                 /* 256-262 */
{
    uint64_t br = 0;
    for (int i = 0; i < A_SIZE; ++i) {                                     /* mpn_sub_n */
        uint64_t d = a.key[i] - b->key[i];
        uint64_t b1 = a.key[i] < b->key[i];
        uint64_t d2 = d - br;
        uint64_t b2 = d < br;
        a.key[i] = d2; br = b1 | b2;
    }
    ok_trim(&a); a.isUnspec = 0; return a;
}
static OKey ok_xor(OKey a, const OKey* b)                                 /* 341-349 */
{
    for (int i = 0; i < A_SIZE; ++i) a.key[i] ^= b->key[i];
    return a;
}
#define LT(x, y) (ok_cmp((x), (y)) < 0)
#define GT(x, y) (ok_cmp((x), (y)) > 0)
#define LE(x, y) (ok_cmp((x), (y)) <= 0)
#define GE(x, y) (ok_cmp((x), (y)) >= 0)
#define EQ(x, y) (ok_cmp((x), (y)) == 0)

static int ok_isBetween(const OKey* x, const OKey* a, const OKey* b)      /* 587-599 */
{
    if (x->isUnspec || a->isUnspec || b->isUnspec) return 0;
    if (EQ(x, a)) return 0;
    else if (LT(a, b)) return GT(x, a) && LT(x, b);
    else return GT(x, a) || LT(x, b);
}
static int ok_isBetweenR(const OKey* x, const OKey* a, const OKey* b)     /* 602-614 */
{
    if (x->isUnspec || a->isUnspec || b->isUnspec) return 0;
    if (EQ(a, b) && EQ(x, a)) return 1;
    else if (LE(a, b)) return GT(x, a) && LE(x, b);
    else return GT(x, a) || LE(x, b);
}
static int ok_isBetweenL(const OKey* x, const OKey* a, const OKey* b)     /* 617-629 */
{
    if (x->isUnspec || a->isUnspec || b->isUnspec) return 0;
    if (EQ(a, b) && EQ(x, a)) return 1;
    else if (LE(a, b)) return GE(x, a) && LT(x, b);
    else return GE(x, a) || LT(x, b);
}
static int ok_isBetweenLR(const OKey* x, const OKey* a, const OKey* b)    /* 632-644 */
{
    if (x->isUnspec || a->isUnspec || b->isUnspec) return 0;
    if (EQ(a, b) && EQ(x, a)) return 1;
    else if (LE(a, b)) return GE(x, a) && LE(x, b);
    else return GE(x, a) || LE(x, b);
}
static uint32_t ok_getBitRange(const OKey* k, uint32_t p, uint32_t n)     /* 458-474 */
{
    int i = p / 64, f = p % 64, f2 = f + (int)n - 64;
    if ((p + n > 160) || (n > 32)) { set_err("getBitRange: invalid range"); return 0; }
    uint64_t lo = k->key[i] >> f;
    uint64_t hi = (f2 > 0) ? (k->key[i + 1] << (64 - f)) : 0;
    return (uint32_t)((lo | hi) & (((uint32_t)(~0u)) >> (32 - n)));
}
static OKey ok_pow2(uint32_t e)                                           /* 704-717 */
{
    OKey r; memset(&r, 0, sizeof r);
    if (e >= 160) { set_err("pow2: exponent >= keyLength"); return r; }
    r.key[e / 64] = (uint64_t)1 << (e % 64);
    return r;
}
static int ok_log2(const OKey* k)                                         /* 558-578 */
{
    int i = A_SIZE - 1;
    while (i >= 0 && k->key[i] == 0) i--;
    if (i < 0) return -1;
    uint64_t j = k->key[i];
    i *= 64;
    while (j != 0) { j >>= 1; i++; }
    return i - 1;
}

/* public wrappers */
int orc_key_cmp(const orc_key* a, const orc_key* b) { OKey x = ok_from(a), y = ok_from(b); return ok_cmp(&x, &y); }
void orc_key_add(const orc_key* a, const orc_key* b, orc_key* out) { OKey x = ok_from(a), y = ok_from(b); x = ok_add(x, &y); ok_to(&x, out); }
void orc_key_sub(const orc_key* a, const orc_key* b, orc_key* out) { OKey x = ok_from(a), y = ok_from(b); x = ok_sub(x, &y); ok_to(&x, out); }
void orc_key_xor(const orc_key* a, const orc_key* b, orc_key* out) { OKey x = ok_from(a), y = ok_from(b); x = ok_xor(x, &y); ok_to(&x, out); }
int orc_key_between(int which, const orc_key* x, const orc_key* a, const orc_key* b, int m)
{
    OKey X = ok_from(x), A = ok_from(a), B = ok_from(b);
    X.isUnspec = (m & 1) != 0; A.isUnspec = (m & 2) != 0; B.isUnspec = (m & 4) != 0;
    switch (which) {
    case 0: return ok_isBetween(&X, &A, &B);
    case 1: return ok_isBetweenR(&X, &A, &B);
    case 2: return ok_isBetweenL(&X, &A, &B);
    default: return ok_isBetweenLR(&X, &A, &B);
    }
}
uint32_t orc_key_bit_range(const orc_key* k, uint32_t p, uint32_t n) { OKey x = ok_from(k); return ok_getBitRange(&x, p, n); }
uint32_t orc_key_shared_prefix(const orc_key* a, const orc_key* b, uint32_t bitsPerDigit) /* 530-555 */
{
    OKey x = ok_from(a), y = ok_from(b);
    if (ok_cmp(&x, &y) == 0) return 160;
    uint32_t length = 0; int msb = 1;
    for (int i = A_SIZE - 1; i >= 0; --i) {
        if (x.key[i] != y.key[i]) {
            uint64_t d = x.key[i] ^ y.key[i];
            uint32_t j;
            if (msb) d <<= (64 - (160 % 64));
            for (j = 63; d >>= 1; --j);
            length += j;
            break;
        }
        length += 64;
        msb = 0;
    }
    return length / bitsPerDigit;
}
int orc_key_log2(const orc_key* k) { OKey x = ok_from(k); return ok_log2(&x); }
void orc_key_pow2(uint32_t e, orc_key* out) { OKey x = ok_pow2(e); ok_to(&x, out); }

/* ===================================================================== */
/* parameters                                                            */
/* ===================================================================== */
/* response length: BASERESPONSE_L (+ AUTHBLOCK_L when measureAuthBlock, CommonMessages.msg:57, 73)
 * + NEIGHBORSFLAG_L + the carried NodeHandles (FINDNODERESPONSE_L, CommonMessages.msg:71-72) */
#define AUTHBLOCK_BYTES ((40 * 8 + 40 * 8 + 20 * 8) / 8)   /* SIGNATURE_L + CERT_L + PUBKEY_L, msg:45-47 */
static int32_t resp_bytes(const orc_params* p, int nodes)
{
    return p->respBaseBytes + (p->measureAuthBlock ? AUTHBLOCK_BYTES : 0) + p->respPerNodeBytes * nodes;
}

static void params_common(orc_params* p)
{
    memset(p, 0, sizeof *p);
    p->hopCountMax = 50;
    p->successorListSize = 8;
    p->numFingerCandidates = 3;
    p->k = 8; p->s = 8; p->b = 1;
    p->lookupRedundantNodes = 1;
    p->lookupParallelRpcs = 1;
    p->lookupMerge = 0;
    p->lookupStrictParallelRpcs = 1;
    p->lookupVisitOnlyOnce = 1;
    p->lookupAcceptLateSiblings = 1;
    p->numSiblings = 1;
    p->simtimeRound = 1;
    p->rpcUdpTimeout = 1.5;
    p->lookupTimeout = 10.0;
    p->datarate = 10e6;
    p->accessDelay = 0.0;
    p->callBytes = 55 + 28;      /* FINDNODECALL_L = 440 bits, CommonMessages.msg:68-69; UDP+IP 28 B SimpleUDP.cc:291 */
    p->respBaseBytes = 33 + 28;  /* FINDNODERESPONSE_L = 264 + 208c bits, CommonMessages.msg:71-72 */
    p->respPerNodeBytes = 26;    /* NODEHANDLE_L = 208 bits */
    p->routeBytes = 158 + 28;    /* BASEROUTE_L 424 + BASEAPPDATA_L 40 + testMsgSize 100 B */
    p->kadSeed = 0x4b41444dull;
    p->routingType = 0;          /* default.ini:392 "iterative" */
    p->recNumRedundantNodes = 3; /* default.ini:386 */
    p->shiftingBits = 4;         /* default.ini:277 */
    p->deBruijnListSize = 16;    /* default.ini:276 */
    p->useOtherLookup = 1;       /* default.ini:279 */
    p->useSucList = 1;           /* default.ini:280 */
    p->bucketType = 0;           /* default.ini:209 "kademlia" */
    p->globalNodeLimit = 1000;   /* default.ini:210 */
    p->extraNodesFinalBucket = 0;/* default.ini:211 (0 = key length) */
    p->rpcKeyTimeout = 10.0;     /* default.ini:484 */
}
void orc_params_chord_default(orc_params* p) { params_common(p); }
void orc_params_koorde_default(orc_params* p)
{
    params_common(p);
    p->successorListSize = 16;   /* default.ini:275 */
    /* KOORDEFINDNODEEXTMESSAGE_L = KEY_L + STEP_L = 168 bits (ChordMessage.msg:33,55) rides on
     * every FindNodeCall and FindNodeResponse of a Koorde lookup (IterativeLookup.cc:359-390,
     * BaseOverlay.cc:1903-1907) */
    p->callBytes += 21;
    p->respBaseBytes += 21;
}
void orc_params_kad_default(orc_params* p)
{
    params_common(p);
    p->lookupRedundantNodes = 8;   /* default.ini:186 */
    p->lookupParallelRpcs = 3;     /* default.ini:188 */
    p->lookupMerge = 1;            /* default.ini:189 */
}

/* ===================================================================== */
/* networks                                                              */
/* ===================================================================== */
enum { NET_CHORD = 1, NET_KAD = 2, NET_KOORDE = 3 };   /* NET_KOORDE: Chord tables + de Bruijn state */
#define NONE 0xFFFFFFFFu

struct orc_net {
    int type;
    uint32_t n;
    OKey* ids;
    double* xy;
    orc_params p;
    /* lazy = 1: the tables of the stable state are not stored but evaluated per access by the
     * same rule that builds them (Chord: pred / successor list / finger i = responsible(n + 2^i);
     * Kademlia: a node's sibling table and buckets built on first use, kept in a small per-thread
     * cache).  Used for networks whose stored tables would not fit in memory (configs D, E). */
    int lazy;
    uint32_t ns;            /* lazy Chord: successor list length min(successorListSize, n-1) */
    /* Chord */
    uint32_t* pred;         /* n */
    uint32_t* succ;         /* n * sls */
    uint8_t* nsucc;         /* n */
    uint32_t sls;
    uint32_t* fdeque;       /* n * 160: deque entry p (p = 159 - pos), NONE = unspecified */
    uint8_t* fsize;         /* deque size */
    /* Kademlia */
    uint32_t* sib;          /* n * 5s, sorted by XOR to self */
    uint8_t* nsib;
    int nb;                 /* numBuckets = (2^b - 1) * (160 / b) (Kademlia.cc:176) */
    int bks;                /* snapshot builds: slots per bucket (the largest routingBucketSize) */
    uint32_t* bucket;       /* n * nb * bks (snapshot builds) */
    uint8_t* bcount;        /* n * nb */
    uint32_t* rts;          /* explicit tables: currentRoutingTableSize per node (bucket entries) */
    /* explicit (mutable) tables: bucket (v, m) is a growable array in LRU order (KademliaBucket,
     * push_back / erase in routingAdd), bdyn[v * nb + m] with bdcnt entries of bdcap */
    uint32_t** bdyn;
    uint16_t* bdcnt;
    uint16_t* bdcap;
    /* Koorde: deBruijnNode, deBruijnNodes = kdbNum ring nodes from sorted index kdbStart */
    uint32_t* kdb;
    uint32_t* kdbStart;
    uint8_t* kdbNum;
};

void orc_net_free(orc_net* net)
{
    if (!net) return;
    free(net->ids); free(net->xy); free(net->pred); free(net->succ); free(net->nsucc);
    free(net->fdeque); free(net->fsize); free(net->sib); free(net->nsib); free(net->bucket);
    free(net->bcount); free(net->kdb); free(net->kdbStart); free(net->kdbNum);
    if (net->bdyn) for (size_t i = 0; i < (size_t)net->n * (size_t)net->nb; ++i) free(net->bdyn[i]);
    free(net->bdyn); free(net->bdcnt); free(net->bdcap); free(net->rts);
    free(net);
}

static orc_net* net_alloc(int type, const orc_key* ids, uint32_t n, const double* xy, const orc_params* p)
{
    orc_net* net = (orc_net*)calloc(1, sizeof *net);
    net->type = type; net->n = n; net->p = *p;
    net->ids = (OKey*)malloc(sizeof(OKey) * (size_t)n);
    for (uint32_t i = 0; i < n; ++i) net->ids[i] = ok_from(&ids[i]);
    net->xy = (double*)malloc(sizeof(double) * 2 * (size_t)n);
    memcpy(net->xy, xy, sizeof(double) * 2 * (size_t)n);
    for (uint32_t i = 1; i < n; ++i) {
        if (ok_cmp(&net->ids[i - 1], &net->ids[i]) >= 0) {
            set_err("ids must be sorted ascending and unique");
            orc_net_free(net);
            return NULL;
        }
    }
    return net;
}

/* responsible(key): the node m with key in (pred(m), m] (Chord.cc:422-457) ==
 * first id >= key, wrapping to ids[0]. */
static uint32_t ring_responsible(const orc_net* net, const OKey* key)
{
    uint32_t lo = 0, hi = net->n;
    while (lo < hi) {
        uint32_t mid = lo + (hi - lo) / 2;
        if (ok_cmp(&net->ids[mid], key) < 0) lo = mid + 1; else hi = mid;
    }
    return lo == net->n ? 0 : lo;
}

/* ---- ChordFingerTable (ChordFingerTable.cc) -------------------------------- */
static void ft_setFinger(orc_net* net, uint32_t node, uint32_t pos, uint32_t v)   /* 66-87 */
{
    uint32_t p = 160 - pos - 1;
    uint32_t* dq = net->fdeque + (size_t)node * 160;
    while (net->fsize[node] <= p) dq[net->fsize[node]++] = NONE;
    dq[p] = v;
}
static void ft_removeFinger(orc_net* net, uint32_t node, uint32_t pos)            /* 154-172 */
{
    uint32_t p = 160 - pos - 1;
    if (p >= net->fsize[node]) return;
    else if (p == (uint32_t)net->fsize[node] - 1) net->fsize[node]--;
    else net->fdeque[(size_t)node * 160 + p] = NONE;
}
/* the successor list, predecessor and finger deque of a node: stored, or (lazy stable ring)
 * the values orc_chord_build would have stored */
static uint32_t succ_get(const orc_net* net, uint32_t node, uint32_t pos)
{
    if (net->lazy) return (uint32_t)(((uint64_t)node + 1 + pos) % net->n);
    return net->succ[(size_t)node * net->sls + pos];
}
static int nsucc_get(const orc_net* net, uint32_t node)
{
    return net->lazy ? (int)net->ns : (int)net->nsucc[node];
}
static uint32_t pred_get(const orc_net* net, uint32_t node)
{
    return net->lazy ? (node + net->n - 1) % net->n : net->pred[node];
}
static uint32_t ft_getFinger(const orc_net* net, uint32_t node, uint32_t pos)     /* 174-193 */
{
    if (net->lazy) {
        /* stable state (Chord.cc:845-875): finger pos is set to responsible(n + 2^pos) iff
         * 2^pos > succ0 - n, else removed; the removed (trivial) ones are exactly the deque
         * positions p >= size, which getFinger answers with the successor (183-184) */
        const OKey* self = &net->ids[node];
        uint32_t s0 = succ_get(net, node, 0);
        OKey d = ok_sub(net->ids[s0], self);
        OKey off = ok_pow2(pos);
        if (ok_cmp(&off, &d) <= 0) return s0;
        OKey lk = ok_add(*self, &off);
        return ring_responsible(net, &lk);
    }
    uint32_t p = 160 - pos - 1;
    const uint32_t* dq = net->fdeque + (size_t)node * 160;
    uint32_t size = net->fsize[node];
    if (p >= size) return succ_get(net, node, 0);
    while (dq[p] == NONE && (p < size - 1)) ++p;
    if (dq[p] == NONE) return succ_get(net, node, 0);
    return dq[p];
}

/* Stable (NoChurn, converged) Chord state:
 *  - predecessor = previous id on the ring,
 *  - successor list = next min(successorListSize, n-1) ids (ChordSuccessorList.cc:122-151,
 *    keyed by succ-(self+1); self evicted once others are known, 170-194),
 *  - fingers as left by handleFixFingersTimerExpired (Chord.cc:845-875): for
 *    nextFinger = 0..159, trivial fingers (2^i <= succ - self) are removed, the
 *    others set to the node answering rpcFixfingers for self+2^i, i.e. the
 *    responsible node (Chord.cc:1228-1270, non-extended finger table). */
static int check_params(const orc_params* p)
{
    /* the fixed capacities below (NVec 128 entries, 16 siblings) bound these parameters */
    if (p->successorListSize < 1 || p->successorListSize > 120) { set_err("successorListSize must be 1..120"); return 0; }
    if (p->s < 1 || 5 * p->s > 120 || p->k < 1 || p->k > 64) { set_err("kademlia k must be 1..64, 5s <= 120"); return 0; }
    if (p->numSiblings < 0 || p->numSiblings > 16) { set_err("numSiblings must be 0..16"); return 0; }
    if (p->lookupRedundantNodes < 1 || p->lookupRedundantNodes > 64) { set_err("lookupRedundantNodes must be 1..64"); return 0; }
    if (p->extendedFingerTable && (p->numFingerCandidates < 1 || p->numFingerCandidates > 64)) {
        set_err("numFingerCandidates must be 1..64"); return 0;
    }
    return 1;
}

static orc_net* chord_build(const orc_key* ids, uint32_t n, const double* xy, const orc_params* p, int lazy)
{
    if (n < 2) { set_err("chord: need at least 2 nodes"); return NULL; }
    if (!check_params(p)) return NULL;
    orc_net* net = net_alloc(NET_CHORD, ids, n, xy, p);
    if (!net) return NULL;
    uint32_t sls = (uint32_t)p->successorListSize;
    net->sls = sls;
    net->ns = (n - 1 < sls) ? n - 1 : sls;
    if (lazy) { net->lazy = 1; return net; }
    net->pred = (uint32_t*)malloc(sizeof(uint32_t) * n);
    net->succ = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n * sls);
    net->nsucc = (uint8_t*)malloc(n);
    net->fdeque = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n * 160);
    net->fsize = (uint8_t*)calloc(n, 1);
    uint32_t ns = (n - 1 < sls) ? n - 1 : sls;
    for (uint32_t i = 0; i < n; ++i) {
        net->pred[i] = (i + n - 1) % n;
        net->nsucc[i] = (uint8_t)ns;
        for (uint32_t j = 0; j < ns; ++j) net->succ[(size_t)i * sls + j] = (i + 1 + j) % n;
    }
    for (uint32_t i = 0; i < n; ++i) {
        const OKey* self = &net->ids[i];
        OKey d = ok_sub(net->ids[succ_get(net, i, 0)], self);
        for (uint32_t nf = 0; nf < 160; ++nf) {
            OKey off = ok_pow2(nf);
            OKey lk = ok_add(*self, &off);
            if (ok_cmp(&off, &d) > 0) ft_setFinger(net, i, nf, ring_responsible(net, &lk));
            else ft_removeFinger(net, i, nf);
        }
    }
    return net;
}

orc_net* orc_chord_build(const orc_key* ids, uint32_t n, const double* xy, const orc_params* p)
{
    return chord_build(ids, n, xy, p, 0);
}

orc_net* orc_chord_build_lazy(const orc_key* ids, uint32_t n, const double* xy, const orc_params* p)
{
    return chord_build(ids, n, xy, p, 1);
}

/* store the tables of a lazy stable ring (a fixfingers round rewrites them) */
static void chord_materialize(orc_net* net)
{
    if (!net->lazy) return;
    uint32_t n = net->n, sls = net->sls;
    net->pred = (uint32_t*)malloc(sizeof(uint32_t) * n);
    net->succ = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n * sls);
    net->nsucc = (uint8_t*)malloc(n);
    net->fdeque = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n * 160);
    net->fsize = (uint8_t*)calloc(n, 1);
    for (uint32_t i = 0; i < n; ++i) {
        net->pred[i] = pred_get(net, i);
        net->nsucc[i] = (uint8_t)net->ns;
        for (uint32_t j = 0; j < net->ns; ++j) net->succ[(size_t)i * sls + j] = succ_get(net, i, j);
    }
    /* deque entries from the lazy rule, then switch over */
    for (uint32_t i = 0; i < n; ++i) {
        OKey d = ok_sub(net->ids[succ_get(net, i, 0)], &net->ids[i]);
        for (uint32_t nf = 0; nf < 160; ++nf) {
            OKey off = ok_pow2(nf);
            uint32_t f = ft_getFinger(net, i, nf);
            uint32_t p = 160 - nf - 1;
            if (ok_cmp(&off, &d) > 0) {
                if (net->fsize[i] <= p) net->fsize[i] = (uint8_t)(p + 1);
                net->fdeque[(size_t)i * 160 + p] = f;
            }
        }
    }
    net->lazy = 0;
}

orc_net* orc_chord_build_tables(const orc_key* ids, uint32_t n, const double* xy,
                                const uint32_t* pred, const uint32_t* succ, const uint8_t* nsucc,
                                uint32_t succ_stride, const uint32_t* fingers,
                                const uint8_t* deque_size, const orc_params* p)
{
    if (!check_params(p)) return NULL;
    if (p->extendedFingerTable) {
        set_err("extendedFingerTable: explicit tables carry no finger candidate lists"); return NULL;
    }
    orc_net* net = net_alloc(NET_CHORD, ids, n, xy, p);
    if (!net) return NULL;
    net->sls = succ_stride;
    net->pred = (uint32_t*)malloc(sizeof(uint32_t) * n);
    net->succ = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n * succ_stride);
    net->nsucc = (uint8_t*)malloc(n);
    net->fdeque = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n * 160);
    net->fsize = (uint8_t*)malloc(n);
    memcpy(net->pred, pred, sizeof(uint32_t) * n);
    memcpy(net->succ, succ, sizeof(uint32_t) * (size_t)n * succ_stride);
    memcpy(net->nsucc, nsucc, n);
    memcpy(net->fsize, deque_size, n);
    for (uint32_t i = 0; i < n; ++i)
        for (uint32_t pos = 0; pos < 160; ++pos)
            net->fdeque[(size_t)i * 160 + (160 - pos - 1)] = fingers[(size_t)i * 160 + pos];
    return net;
}

void orc_chord_export_fingers(const orc_net* net, uint32_t* out)
{
    for (uint32_t i = 0; i < net->n; ++i)
        for (uint32_t pos = 0; pos < 160; ++pos) out[(size_t)i * 160 + pos] = ft_getFinger(net, i, pos);
}

/* ---- NodeVector / BaseKeySortedVector::add (NodeVector.h:381-512) ----------- */
typedef struct {
    uint32_t v[128];
    int size;
    int maxSize;            /* 0 = unbounded */
    int metric;             /* 0 none (push only), 1 XOR, 2 uni-ring (Chord::distance) */
    OKey rel;               /* relative key of the comparator */
} NVec;

static OKey metric_dist(int metric, const OKey* x, const OKey* key)
{
    if (metric == 1) return ok_xor(*x, key);              /* KeyXorMetric, Comparator.h:90-106 */
    return ok_sub(*key, x);                               /* KeyUniRingMetric: y - x, Comparator.h:137-153 */
}
static int nv_compare(const orc_net* net, const NVec* nv, uint32_t a, uint32_t b) /* Comparator.h:193-222 */
{
    OKey da = metric_dist(nv->metric, &net->ids[a], &nv->rel);
    OKey db = metric_dist(nv->metric, &net->ids[b], &nv->rel);
    return ok_cmp(&da, &db);
}
static void nv_init(NVec* nv, int maxSize, int metric, const OKey* rel)
{
    nv->size = 0; nv->maxSize = maxSize; nv->metric = metric;
    if (rel) nv->rel = *rel; else memset(&nv->rel, 0, sizeof nv->rel);
}
static int nv_isFull(const NVec* nv) { return nv->maxSize != 0 && nv->size == nv->maxSize; }
static int nv_isAddable(const orc_net* net, const NVec* nv, uint32_t e)          /* 381-399 */
{
    if (nv->maxSize == 0) return 1;
    return nv->size != nv->maxSize || (nv->metric && nv_compare(net, nv, e, nv->v[nv->size - 1]) <= 0);
}
static void nv_push_back(NVec* nv, uint32_t e)
{
    if (nv->size < 128) nv->v[nv->size++] = e;
    else cap_error("NodeVector of 128 entries");
}
static int nv_add(const orc_net* net, NVec* nv, uint32_t e)                      /* 432-512 */
{
    int pos = -1;
    if (!nv_isAddable(net, nv, e)) return -1;
    if (nv->size != 0 && nv->metric) {
        int i;
        for (i = 0, pos = 0; i < nv->size; i++, pos++) {
            if (EQ(&net->ids[e], &net->ids[nv->v[i]])) return -1;
            if (nv_compare(net, nv, e, nv->v[i]) < 0) {
                memmove(&nv->v[i + 1], &nv->v[i], sizeof(uint32_t) * (size_t)(nv->size - i));
                nv->v[i] = e; nv->size++;
                break;
            }
        }
        if (i == nv->size && pos == nv->size) { /* reached end without insert */
            pos = nv->size;
            nv_push_back(nv, e);
        }
    } else {
        for (int i = 0; i < nv->size; i++)
            if (EQ(&net->ids[e], &net->ids[nv->v[i]])) return -1;
        pos = nv->size;
        nv_push_back(nv, e);
    }
    if (nv->maxSize != 0 && nv->size > nv->maxSize) nv->size = nv->maxSize;
    return pos;
}
static void nv_downsizeTo(NVec* nv, int m) { if (nv->size > m) nv->size = m; }  /* 566-571 */
static int nv_contains(const orc_net* net, const NVec* nv, const OKey* key)
{
    for (int i = 0; i < nv->size; ++i) if (EQ(&net->ids[nv->v[i]], key)) return 1;
    return 0;
}

/* ---- Chord routing (Chord.cc) ------------------------------------------------ */
static int chord_isSiblingFor(const orc_net* net, uint32_t node, uint32_t self,
                              const OKey* key, int numSiblings, int* err)          /* 422-500 */
{
    /* state == READY; numSiblings <= successorListSize asserted by caller */
    if (numSiblings == -1) numSiblings = net->p.successorListSize;
    uint32_t pred = pred_get(net, self);
    int predUnspec = (pred == NONE);
    int ssize = nsucc_get(net, self);
    if (predUnspec && node == self) {
        int isEmpty = (ssize == 1 && succ_get(net, self, 0) == self) || ssize == 0;
        if (isEmpty || EQ(&net->ids[node], key)) { *err = 0; return 1; }
        *err = 1; return 0;
    }
    if (node == self && ok_isBetweenR(key, &net->ids[pred], &net->ids[self])) { *err = 0; return 1; }
    uint32_t prevNode = pred, curNode;
    for (int i = -1; i < ssize; i++, prevNode = curNode) {
        curNode = (i < 0) ? self : succ_get(net, self, (uint32_t)i);
        if (node == curNode) {
            OKey prevKey = (prevNode == NONE) ? (OKey){{0, 0, 0}, 1} : net->ids[prevNode];
            if (ok_isBetweenR(key, &prevKey, &net->ids[curNode])) {
                if (numSiblings <= (ssize - i)) { *err = 0; return 1; }
                *err = 1; return 0;
            } else {
                if (numSiblings <= 1) { *err = 0; return 0; }
                *err = 1; return 0;
            }
        }
    }
    *err = 1;
    return 0;
}

/* finger pos of a stable ring is trivial (2^pos <= succ0 - node): removed from the deque, which
 * getFinger answers with the successor (Chord.cc:845-875, ChordFingerTable.cc:174-193) */
static int ft_trivial(const orc_net* net, uint32_t node, uint32_t pos)
{
    if (net->lazy) {
        OKey d = ok_sub(net->ids[succ_get(net, node, 0)], &net->ids[node]);
        OKey off = ok_pow2(pos);
        return ok_cmp(&off, &d) <= 0;
    }
    return 160 - pos - 1 >= net->fsize[node];
}

/* ChordFingerTable::getFinger(pos, key) with extendedFingerTable (ChordFingerTable.cc:195-228) on
 * a stable ring: entry pos holds the FixfingersResponse of its finger f -- f, then f's first
 * min(successorListSize, numFingerCandidates) successors (Chord::rpcFixfingers 1228-1251) --
 * inserted in that order under the one key MAXTIME up to this node (handleRpcFixfingersResponse
 * 1268-1287; no proximity routing); the answer keeps the candidates that do not reach past the
 * key (!key.isBetweenLR(f, c)), else f.  A trivial position answers the successor. */
static int chord_getFinger_ext(const orc_net* net, uint32_t self, uint32_t pos, const OKey* key, NVec* out)
{
    if (ft_trivial(net, self, pos)) { nv_push_back(out, succ_get(net, self, 0)); return 0; }
    const uint32_t f = ft_getFinger(net, self, pos);
    const int nf = nsucc_get(net, f);
    const int m = nf < net->p.numFingerCandidates ? nf : net->p.numFingerCandidates;
    for (int j = -1; j < m; ++j) {
        const uint32_t c = j < 0 ? f : succ_get(net, f, (uint32_t)j);
        if (c == self) break;
        if (!ok_isBetweenLR(key, &net->ids[f], &net->ids[c])) nv_push_back(out, c);
    }
    if (out->size == 0) nv_push_back(out, f);
    return 0;
}

static int chord_closestPreceedingNode(const orc_net* net, uint32_t self, const OKey* key, NVec* out) /* 602-674 */
{
    uint32_t temp = NONE;
    int ssize = nsucc_get(net, self);
    for (int j = ssize - 1; j >= 0; j--) {
        uint32_t s = succ_get(net, self, (uint32_t)j);
        if (ok_isBetweenR(&net->ids[s], &net->ids[self], key)) { temp = s; break; }
    }
    if (temp == NONE) { set_err("Chord::closestPreceedingNode(): Successor list broken"); return -1; }
    for (int i = 160 - 1; i >= 0; i--) {
        uint32_t f = ft_getFinger(net, self, (uint32_t)i);
        if (ok_isBetweenLR(&net->ids[f], &net->ids[temp], key)) {
            if (net->p.extendedFingerTable) return chord_getFinger_ext(net, self, (uint32_t)i, key, out);
            nv_push_back(out, f);
            return 0;
        }
    }
    for (int i = ssize - 1; i >= 0 && out->size <= net->p.numFingerCandidates; i--) {
        uint32_t s = succ_get(net, self, (uint32_t)i);
        if (ok_isBetween(&net->ids[s], &net->ids[self], key)) nv_push_back(out, s);
    }
    if (out->size != 0) return 0;
    if (pred_get(net, self) == NONE && succ_get(net, self, 0) == self) { nv_push_back(out, self); return 0; }
    set_err("Error in Chord::closestPreceedingNode()!");
    return -1;
}

static int chord_findNode(const orc_net* net, uint32_t self, const OKey* key,
                          int numRedundantNodes, int numSiblings, NVec* out)       /* 548-599 */
{
    int err;
    nv_init(out, 0, 0, NULL);
    if (key->isUnspec) { nv_push_back(out, self); return 0; }
    if (chord_isSiblingFor(net, self, self, key, 1, &err)) {
        nv_push_back(out, self);
        for (int i = 0; i < nsucc_get(net, self); i++) nv_push_back(out, succ_get(net, self, (uint32_t)i));
        nv_downsizeTo(out, numSiblings);
    } else if (ok_isBetweenR(key, &net->ids[self], &net->ids[succ_get(net, self, 0)])) {
        for (int i = 0; i < nsucc_get(net, self); i++) nv_push_back(out, succ_get(net, self, (uint32_t)i));
        nv_downsizeTo(out, numRedundantNodes);
    } else {
        if (chord_closestPreceedingNode(net, self, key, out) < 0) return -1;
        nv_downsizeTo(out, numRedundantNodes);
    }
    return 0;
}

/* ---- Kademlia (Kademlia.cc) -------------------------------------------------- */
int orc_kad_num_buckets(const orc_params* p)                                  /* Kademlia.cc:176 */
{
    return (int)(((1L << p->b) - 1L) * (160 / p->b));
}

int orc_kad_bucket_size(const orc_params* p, int index)                       /* 384-411 */
{
    if (p->bucketType == 1) return 0;                     /* NKADEMLIA: no maximum per bucket */
    if (p->bucketType == 2) {                             /* NR128: the final buckets hold more */
        const int extra = p->extraNodesFinalBucket == 0 ? 160 : p->extraNodesFinalBucket;   /* 146-148 */
        const int limit = (int)(log((double)extra) / log(2.0));
        int offset = limit - (160 - (index + 1));
        if (offset > 0) {
            offset = (int)pow(2, offset);
            if (offset > p->k) return offset;
        }
        return p->k;
    }
    return p->k;
}

static int kad_routingBucketIndex(const orc_net* net, uint32_t self, const OKey* key, int firstOnLayer) /* 357-382 */
{
    int b = net->p.b;
    OKey delta = ok_xor(*key, &net->ids[self]);
    int i;
    for (i = 160 - b; i >= 0 && ok_getBitRange(&delta, (uint32_t)i, (uint32_t)b) == 0; i -= b);
    if (i < 0) return -1;
    if (!firstOnLayer) return (i / b) * ((1 << b) - 1) + (int)(ok_getBitRange(&delta, (uint32_t)i, (uint32_t)b) - 1);
    return (i / b) * ((1 << b) - 1) + (int)(pow(2, b) - 2);
}

/* Kademlia snapshot rule: sibling table = the min(5s, n-1) XOR-closest
 * nodes (what routingAdd, Kademlia.cc:537-616, converges to), buckets hold up to k
 * of the remaining nodes of each subtree, chosen by Floyd sampling driven by
 * splitmix64(seed, node, bucket, j); bucket order is irrelevant to findNode since
 * the result NodeVector is XOR-sorted and XOR distances are unique. */
static uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
static uint64_t kad_hash(uint64_t seed, uint32_t node, uint32_t m, uint32_t j)
{
    return splitmix64(seed ^ splitmix64(((uint64_t)node << 32) ^ ((uint64_t)m << 16) ^ (uint64_t)j));
}
/* The tables of one node under the snapshot rule: sib[] (its sibling table, XOR-sorted to
 * self), *nsib, and per bucket index m (0 .. nb-1) the members bk[m*bks ..] (bc[m] of them): up to
 * routingBucketSize(m) of the bucket's subtree minus the siblings.  For b > 1 bucket
 * (layer L, digit d) holds the ids that share self's bits above the digit at bit i = L*b + 160 % b
 * and whose digit there is self's ^ d (routingBucketIndex, Kademlia.cc:357-382). */
static void kad_node_build(const orc_net* net, uint32_t self, uint32_t* sibOut, int* nsibOut, uint8_t* bc,
                           uint32_t* bk)
{
    const orc_params* p = &net->p;
    int sibCap = 5 * p->s;
    const int B = p->b, per = (1 << B) - 1, bks = net->bks;
    /* sibling table: walk subtrees m = 0.. upward, gather members, keep 5s closest */
    /* T_m = [tlo[m], thi[m]): the ids sharing the bits above m with self and differing at bit m
     * (subtree_range(self, m)), found by one descent over the sorted ids: the ids sharing the
     * bits above m form one block, split at its first id with bit m set */
    uint32_t tlo[160], thi[160];
    uint32_t slo[161], shi[161];     /* S[b'] = the ids sharing bits b' .. 159 with self */
    {
        const OKey* me = &net->ids[self];
        uint32_t lo = 0, hi = net->n;
        slo[160] = lo; shi[160] = hi;
        for (int b = 159; b >= 0; --b) {
            uint32_t a = lo, z = hi;
            while (a < z) {
                uint32_t mid = a + (z - a) / 2;
                if ((net->ids[mid].key[b / 64] >> (b % 64)) & 1) z = mid; else a = mid + 1;
            }
            if ((me->key[b / 64] >> (b % 64)) & 1) { tlo[b] = lo; thi[b] = a; lo = a; }
            else { tlo[b] = a; thi[b] = hi; hi = a; }
            slo[b] = lo; shi[b] = hi;
        }
    }
    NVec sib; nv_init(&sib, sibCap, 1, &net->ids[self]);
    int m;
    for (m = 0; m < 160; ++m) {
        for (uint32_t x = tlo[m]; x < thi[m]; ++x) nv_add(net, &sib, x);
        if (nv_isFull(&sib)) break;   /* all later subtrees are farther (XOR >= 2^(m+1)) */
    }
    *nsibOut = sib.size;
    for (int i = 0; i < sibCap; ++i) sibOut[i] = i < sib.size ? sib.v[i] : NONE;
    /* buckets */
    for (m = 0; m < net->nb; ++m) {
        bc[m] = 0;
        uint32_t lo, hi;
        if (B == 1) { lo = tlo[m]; hi = thi[m]; }
        else {
            /* index m = layer L * (2^b - 1) + digit d - 1; the digit sits at bits i .. i+b-1 */
            const int L = m / per, d = m % per + 1, i = L * B + 160 % B;
            const uint32_t want = ok_getBitRange(&net->ids[self], (uint32_t)i, (uint32_t)B) ^ (uint32_t)d;
            uint32_t a = slo[i + B], z = shi[i + B];
            while (a < z) {               /* first id of the block whose digit >= want */
                uint32_t mid = a + (z - a) / 2;
                if (ok_getBitRange(&net->ids[mid], (uint32_t)i, (uint32_t)B) < want) a = mid + 1; else z = mid;
            }
            lo = a; z = shi[i + B];
            while (a < z) {               /* ... and > want */
                uint32_t mid = a + (z - a) / 2;
                if (ok_getBitRange(&net->ids[mid], (uint32_t)i, (uint32_t)B) <= want) a = mid + 1; else z = mid;
            }
            hi = a;
        }
        if (hi <= lo) continue;
        const int k = orc_kad_bucket_size(p, m);
        if (k <= 0 || k > bks) { cap_error("snapshot tables need a bounded bucketType (kademlia / nr128)"); return; }
        /* members not in the sibling table, in ascending id order */
        uint32_t cnt = hi - lo;
        uint32_t nsib_in = 0;
        for (int s2 = 0; s2 < sib.size; ++s2) if (sib.v[s2] >= lo && sib.v[s2] < hi) nsib_in++;
        uint32_t c = cnt - nsib_in;
        uint32_t* dst = bk + (size_t)m * bks;
        uint32_t chosen[256]; int nch = 0;
        if (c <= (uint32_t)k) {
            for (uint32_t j = 0; j < c; ++j) chosen[nch++] = j;
        } else {
            for (uint32_t j = c - (uint32_t)k; j < c; ++j) {       /* Floyd sampling */
                uint32_t t = (uint32_t)(kad_hash(p->kadSeed, self, (uint32_t)m, j) % (uint64_t)(j + 1));
                int dup = 0;
                for (int q = 0; q < nch; ++q) if (chosen[q] == t) { dup = 1; break; }
                chosen[nch++] = dup ? j : t;
            }
            /* ascending member order */
            for (int a = 1; a < nch; ++a) { uint32_t v = chosen[a]; int q = a - 1; while (q >= 0 && chosen[q] > v) { chosen[q + 1] = chosen[q]; q--; } chosen[q + 1] = v; }
        }
        /* map member rank -> node index (skipping siblings) */
        int out = 0;
        if (nsib_in == 0) {
            for (int q = 0; q < nch; ++q) dst[out++] = lo + chosen[q];
        } else {
            uint32_t rank = 0; int q = 0;
            for (uint32_t x = lo; x < hi && q < nch; ++x) {
                int is_sib = 0;
                for (int s2 = 0; s2 < sib.size; ++s2) if (sib.v[s2] == x) { is_sib = 1; break; }
                if (is_sib) continue;
                if (rank == chosen[q]) { dst[out++] = x; q++; }
                rank++;
            }
        }
        bc[m] = (uint8_t)out;
    }
}

/* explicit tables: growable bucket arrays */
static void kad_dyn_alloc(orc_net* net)
{
    net->bdyn = (uint32_t**)calloc((size_t)net->n * (size_t)net->nb, sizeof(uint32_t*));
    net->bdcnt = (uint16_t*)calloc((size_t)net->n * (size_t)net->nb, sizeof(uint16_t));
    net->bdcap = (uint16_t*)calloc((size_t)net->n * (size_t)net->nb, sizeof(uint16_t));
    net->rts = (uint32_t*)calloc((size_t)net->n, sizeof(uint32_t));
}
static void kad_dyn_push(orc_net* net, uint32_t v, int m, uint32_t x)       /* KademliaBucket::push_back */
{
    const size_t i = (size_t)v * (size_t)net->nb + (size_t)m;
    if (net->bdcnt[i] == net->bdcap[i]) {
        if (net->bdcap[i] >= 32768) { cap_error("bucket over 32768 entries"); return; }
        net->bdcap[i] = (uint16_t)(net->bdcap[i] ? 2 * net->bdcap[i] : 8);
        net->bdyn[i] = (uint32_t*)realloc(net->bdyn[i], sizeof(uint32_t) * net->bdcap[i]);
    }
    net->bdyn[i][net->bdcnt[i]++] = x;
}
static void kad_dyn_erase(orc_net* net, uint32_t v, int m, int pos)        /* bucket->erase(i) */
{
    const size_t i = (size_t)v * (size_t)net->nb + (size_t)m;
    memmove(&net->bdyn[i][pos], &net->bdyn[i][pos + 1], sizeof(uint32_t) * (size_t)(net->bdcnt[i] - pos - 1));
    net->bdcnt[i]--;
}

/* A node's Kademlia tables: pointers into the stored arrays, or (lazy network) into a
 * per-thread cache entry built on first use.  Consecutive findNode / isSiblingFor calls of a
 * lookup are at the same node, so a small direct-mapped cache suffices. */
typedef struct {
    const uint32_t* sib; int nsib;
    const uint8_t* bc; const uint32_t* bk; int k;      /* snapshot layout: bucket m = bk[m*k ..], bc[m] (k = bks) */
    uint32_t* const* bd; const uint16_t* bdc;           /* explicit tables: bucket m = bd[m][0 .. bdc[m]) */
} KadTab;
static inline int kt_count(const KadTab* T, int m) { return T->bd ? (int)T->bdc[m] : (int)T->bc[m]; }
static inline const uint32_t* kt_members(const KadTab* T, int m)
{
    return T->bd ? T->bd[m] : T->bk + (size_t)m * (size_t)T->k;
}

#define KCACHE 16
typedef struct {
    const orc_net* net;
    uint32_t node;
    int nsib;
    uint32_t sib[128];
    uint8_t bc[160];
    uint32_t bk[160 * 64];
} KadCacheEnt;
static __thread KadCacheEnt* tl_kcache = NULL;

static KadTab kad_tab(const orc_net* net, uint32_t self)
{
    KadTab t;
    memset(&t, 0, sizeof t);
    t.k = net->bks;
    if (!net->lazy) {
        size_t sibCap = (size_t)5 * net->p.s;
        t.sib = net->sib + (size_t)self * sibCap;
        t.nsib = net->nsib[self];
        if (net->bdyn) {
            t.bd = net->bdyn + (size_t)self * (size_t)net->nb;
            t.bdc = net->bdcnt + (size_t)self * (size_t)net->nb;
        } else {
            t.bc = net->bcount + (size_t)self * (size_t)net->nb;
            t.bk = net->bucket + (size_t)self * (size_t)net->nb * (size_t)net->bks;
        }
        return t;
    }
    if (!tl_kcache) {
        tl_kcache = (KadCacheEnt*)calloc(KCACHE, sizeof(KadCacheEnt));
        for (int i = 0; i < KCACHE; ++i) tl_kcache[i].net = NULL;
    }
    KadCacheEnt* e = &tl_kcache[(self * 2654435761u) >> 28];
    if (e->net != net || e->node != self) {
        kad_node_build(net, self, e->sib, &e->nsib, e->bc, e->bk);
        e->net = net;
        e->node = self;
    }
    t.sib = e->sib; t.nsib = e->nsib; t.bc = e->bc; t.bk = e->bk;
    return t;
}

static int kad_isSiblingFor(const orc_net* net, uint32_t node, uint32_t self, const OKey* key,
                            int numSiblings, int* err)                              /* 888-962 */
{
    int sibCap = 5 * net->p.s;
    if (numSiblings == -1) numSiblings = net->p.s;
    if (numSiblings == 0) { *err = 0; return EQ(&net->ids[node], key); }
    KadTab T = kad_tab(net, self);
    int nsib = T.nsib;
    const uint32_t* sib = T.sib;
    if (nsib < numSiblings) { *err = 0; return 1; }
    if (nsib == sibCap) {
        OKey a = ok_xor(net->ids[self], key);
        OKey b = ok_xor(net->ids[self], &net->ids[sib[nsib - 1]]);
        if (ok_cmp(&a, &b) > 0) { *err = 1; return 0; }
    }
    NVec result; nv_init(&result, numSiblings, 1, key);
    for (int i = 0; i < nsib; i++) nv_add(net, &result, sib[i]);
    nv_add(net, &result, self);
    *err = 0;
    return nv_contains(net, &result, &net->ids[node]);
}

static int kad_findNode(const orc_net* net, uint32_t self, const OKey* key,
                        int numRedundantNodes, int numSiblings, NVec* result)       /* 1101-1246 */
{
    int err, resultSize;
    int k = net->p.k;
    if (numSiblings < 0) resultSize = numRedundantNodes;
    else resultSize = kad_isSiblingFor(net, self, self, key, numSiblings, &err) ?
                      (numSiblings ? numSiblings : 1) : numRedundantNodes;
    nv_init(result, resultSize, 1, key);
    KadTab T = kad_tab(net, self);
    int nsib = T.nsib;
    const uint32_t* sib = T.sib;
    if (nsib == 0) { nv_add(net, result, self); return 0; }
    int mainIndex = kad_routingBucketIndex(net, self, key, 0);
    int startIndex = kad_routingBucketIndex(net, self, key, 1);
    int endIndex = kad_routingBucketIndex(net, self, &net->ids[sib[nsib - 1]], 0);
    (void)k;
    if (mainIndex != -1) {
        const uint32_t* bk = kt_members(&T, mainIndex);
        for (int i = 0; i < kt_count(&T, mainIndex); ++i) nv_add(net, result, bk[i]);
    }
    if (startIndex >= endIndex || !nv_isFull(result)) {
        for (int index = startIndex; index >= endIndex; --index) {
            if (index == mainIndex) continue;
            const uint32_t* bk = kt_members(&T, index);
            for (int i = 0; i < kt_count(&T, index); ++i) nv_add(net, result, bk[i]);
        }
        for (int i = 0; i < nsib; ++i) nv_add(net, result, sib[i]);
        nv_add(net, result, self);
    }
    for (int index = mainIndex + 1; !nv_isFull(result) && index < net->nb; ++index) {
        const uint32_t* bk = kt_members(&T, index);
        for (int i = 0; i < kt_count(&T, index); ++i) nv_add(net, result, bk[i]);
    }
    return 0;
}

/* Kademlia parameters the restatement covers: b = 1..5 (numBuckets <= 992), the three bucketTypes */
static int kad_check(const orc_params* p)
{
    if (p->b < 1 || p->b > 5) { set_err("kademlia: b must be 1..5"); return 0; }
    if (p->bucketType < 0 || p->bucketType > 2) { set_err("kademlia: bucketType must be 0..2"); return 0; }
    if (p->bucketType == 1 && p->globalNodeLimit < 0) { set_err("kademlia: globalNodeLimit < 0"); return 0; }
    /* routingBucketSize (384-411) counts indices as if b = 1 (offset = limit - (160 - (index + 1))):
     * for b > 1 the indices 160 .. numBuckets-1 get sizes 2^8 .. 2^30 and then (int)pow(2, >= 31),
     * undefined behaviour -- not a configuration the restatement follows */
    if (p->bucketType == 2 && p->b != 1) { set_err("kademlia: nr128 buckets need b = 1"); return 0; }
    if (p->bucketType == 2 && (p->extraNodesFinalBucket < 0 || p->extraNodesFinalBucket > 511)) {
        set_err("kademlia: extraNodesFinalBucket must be 0..511"); return 0;
    }
    return check_params(p);
}
static void kad_net_init(orc_net* net)
{
    net->nb = orc_kad_num_buckets(&net->p);
    int mx = 0;
    for (int m = 0; m < net->nb; ++m) {
        const int c = orc_kad_bucket_size(&net->p, m);
        mx = c > mx ? c : mx;
    }
    net->bks = mx;        /* 0: unbounded buckets (nkademlia) -- explicit tables only */
}

static orc_net* kad_build(const orc_key* ids, uint32_t n, const double* xy, const orc_params* p, int lazy)
{
    if (!kad_check(p)) return NULL;
    if (p->bucketType == 1) { set_err("kademlia: nkademlia tables are order-dependent: explicit tables only"); return NULL; }
    orc_net* net = net_alloc(NET_KAD, ids, n, xy, p);
    if (!net) return NULL;
    kad_net_init(net);
    if (lazy) {
        if (net->nb != 160 || net->bks > 64) { set_err("lazy kademlia tables: b = 1, buckets of <= 64"); orc_net_free(net); return NULL; }
        net->lazy = 1;
        return net;
    }
    const int sibCap = 5 * p->s;
    const size_t nb = (size_t)net->nb, bks = (size_t)net->bks;
    net->sib = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n * sibCap);
    net->nsib = (uint8_t*)calloc(n, 1);
    net->bucket = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n * nb * bks);
    net->bcount = (uint8_t*)calloc((size_t)n * nb, 1);
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 64)
#endif
    for (int64_t self = 0; self < (int64_t)n; ++self) {
        int ns = 0;
        kad_node_build(net, (uint32_t)self, net->sib + (size_t)self * sibCap, &ns, net->bcount + (size_t)self * nb,
                       net->bucket + (size_t)self * nb * bks);
        net->nsib[self] = (uint8_t)ns;
    }
    if (g_cap_fail) { orc_net_free(net); return NULL; }
    return net;
}

orc_net* orc_kad_build(const orc_key* ids, uint32_t n, const double* xy, const orc_params* p)
{
    return kad_build(ids, n, xy, p, 0);
}

orc_net* orc_kad_build_lazy(const orc_key* ids, uint32_t n, const double* xy, const orc_params* p)
{
    return kad_build(ids, n, xy, p, 1);
}

/* Explicit tables (a running network's k-buckets): the sibling table is kept XOR-sorted to the
 * node as Kademlia::siblingTable is (KademliaBucket with KeyDistanceComparator<KeyXorMetric>,
 * Kademlia.cc:315-317), so back() is its farthest entry; buckets keep the caller's (LRU) order. */
orc_net* orc_kad_build_tables(const orc_key* ids, uint32_t n, const double* xy, const uint32_t* siblings,
                              const uint8_t* bucket_count, const uint32_t* bucket_nodes, const orc_params* p)
{
    if (p->b != 1) { set_err("kademlia: k-stride tables are b = 1 (orc_kad_build_tables_csr for b > 1)"); return NULL; }
    if (!kad_check(p)) return NULL;
    orc_net* net = net_alloc(NET_KAD, ids, n, xy, p);
    if (!net) return NULL;
    kad_net_init(net);
    int k = p->k, sibCap = 5 * p->s;
    net->sib = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n * sibCap);
    net->nsib = (uint8_t*)calloc(n, 1);
    kad_dyn_alloc(net);
    for (uint32_t v = 0; v < n; ++v) {
        NVec sib; nv_init(&sib, sibCap, 1, &net->ids[v]);
        for (int i = 0; i < sibCap; ++i) {
            uint32_t x = siblings[(size_t)v * sibCap + i];
            if (x == NONE) continue;
            if (x >= n) { set_err("sibling index out of range"); orc_net_free(net); return NULL; }
            nv_add(net, &sib, x);
        }
        net->nsib[v] = (uint8_t)sib.size;
        for (int i = 0; i < sibCap; ++i) net->sib[(size_t)v * sibCap + i] = i < sib.size ? sib.v[i] : NONE;
        for (int m = 0; m < 160; ++m) {
            int c = bucket_count[(size_t)v * 160 + m];
            if (c > k) { set_err("bucket holds more than k entries"); orc_net_free(net); return NULL; }
            for (int q = 0; q < c; ++q) {
                uint32_t x = bucket_nodes[((size_t)v * 160 + m) * k + q];
                if (x >= n) { set_err("bucket member index out of range"); orc_net_free(net); return NULL; }
                kad_dyn_push(net, v, m, x);
                net->rts[v]++;
            }
        }
    }
    return net;
}

orc_net* orc_kad_build_tables_csr(const orc_key* ids, uint32_t n, const double* xy, const uint32_t* siblings,
                                  const uint64_t* bucket_off, const uint32_t* bucket_nodes, const orc_params* p)
{
    if (!kad_check(p)) return NULL;
    orc_net* net = net_alloc(NET_KAD, ids, n, xy, p);
    if (!net) return NULL;
    kad_net_init(net);
    const int sibCap = 5 * p->s, nb = net->nb;
    net->sib = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n * sibCap);
    net->nsib = (uint8_t*)calloc(n, 1);
    kad_dyn_alloc(net);
    for (uint32_t v = 0; v < n; ++v) {
        NVec sib; nv_init(&sib, sibCap, 1, &net->ids[v]);
        for (int i = 0; i < sibCap; ++i) {
            uint32_t x = siblings[(size_t)v * sibCap + i];
            if (x == NONE) continue;
            if (x >= n) { set_err("sibling index out of range"); orc_net_free(net); return NULL; }
            nv_add(net, &sib, x);
        }
        net->nsib[v] = (uint8_t)sib.size;
        for (int i = 0; i < sibCap; ++i) net->sib[(size_t)v * sibCap + i] = i < sib.size ? sib.v[i] : NONE;
        for (int m = 0; m < nb; ++m) {
            const size_t bi = (size_t)v * nb + (size_t)m;
            const int cap = orc_kad_bucket_size(p, m);
            if (cap && bucket_off[bi + 1] - bucket_off[bi] > (uint64_t)cap) {
                set_err("a bucket holds more than routingBucketSize entries"); orc_net_free(net); return NULL;
            }
            for (uint64_t q = bucket_off[bi]; q < bucket_off[bi + 1]; ++q) {
                if (bucket_nodes[q] >= n) { set_err("bucket member index out of range"); orc_net_free(net); return NULL; }
                kad_dyn_push(net, v, m, bucket_nodes[q]);
                net->rts[v]++;
            }
        }
    }
    return net;
}

void orc_kad_export(const orc_net* net, uint32_t* siblings, uint8_t* bucket_count, uint32_t* bucket_nodes)
{
    size_t sc = (size_t)5 * net->p.s, k = (size_t)net->p.k;
    if (net->nb != 160) { cap_error("orc_kad_export: b > 1 (use orc_kad_export_csr)"); return; }
    for (uint32_t v = 0; v < net->n; ++v) {
        KadTab T = kad_tab(net, v);
        for (size_t i = 0; i < sc; ++i) siblings[(size_t)v * sc + i] = (int)i < T.nsib ? T.sib[i] : NONE;
        for (size_t m = 0; m < 160; ++m) {
            const int c = kt_count(&T, (int)m);
            const uint32_t* bk = kt_members(&T, (int)m);
            if (c > (int)k) cap_error("orc_kad_export: a bucket holds more than k entries (use orc_kad_export_csr)");
            bucket_count[(size_t)v * 160 + m] = (uint8_t)(c < (int)k ? c : (int)k);
            for (size_t j = 0; j < k; ++j)
                bucket_nodes[((size_t)v * 160 + m) * k + j] = (int)j < c ? bk[j] : NONE;
        }
    }
}

/* ---- Koorde (src/overlay/koorde/Koorde.cc) ------------------------------------ */
/* OverlayKey::operator<< / operator>> (OverlayKey.cc:386-425): limb shift, then trim() to
 * keyLength.  The reference shifts with mpn_lshift / mpn_rshift, which GMP defines only for
 * counts 1..63: a shift whose count is a multiple of 64 (by 0, 64 or 128 bits) is undefined
 * there and its result depends on the GMP build; this restatement takes the exact shift
 * (DESIGN.md §Koorde). */
static OKey ok_shl(OKey a, int n)
{
    OKey r; memset(&r, 0, sizeof r);
    if (n >= 160) return r;
    for (int i = A_SIZE - 1; i >= 0; --i) {
        int src = i - n / 64, b = n % 64;
        uint64_t v = 0;
        if (src >= 0) v = a.key[src] << b;
        if (b && src - 1 >= 0) v |= a.key[src - 1] >> (64 - b);
        r.key[i] = v;
    }
    ok_trim(&r);
    return r;
}
static OKey ok_shr(OKey a, int n)
{
    OKey r; memset(&r, 0, sizeof r);
    if (n >= 160) return r;
    for (int i = 0; i < A_SIZE; ++i) {
        int src = i + n / 64, b = n % 64;
        uint64_t v = 0;
        if (src < A_SIZE) v = a.key[src] >> b;
        if (b && src + 1 < A_SIZE) v |= a.key[src + 1] << (64 - b);
        r.key[i] = v;
    }
    ok_trim(&r);
    return r;
}
static OKey ok_small(uint32_t v)                                          /* OverlayKey(uint32_t) 73-78 */
{
    OKey r; memset(&r, 0, sizeof r);
    r.key[0] = v;
    return r;
}

typedef struct { OKey routeKey; int step; } KExt;   /* KoordeFindNodeExtMessage (ChordMessage.msg:168-172) */

static uint32_t koorde_walkSuccessorList(const orc_net* net, uint32_t self, const OKey* key)   /* 572-582 */
{
    int size = nsucc_get(net, self);
    for (int i = 0; i < size - 1; i++) {
        uint32_t a = succ_get(net, self, (uint32_t)i), b = succ_get(net, self, (uint32_t)i + 1);
        if (ok_isBetweenR(key, &net->ids[a], &net->ids[b])) return a;
    }
    return succ_get(net, self, (uint32_t)size - 1);
}
static uint32_t koorde_db(const orc_net* net, uint32_t self, int i)
{
    return (uint32_t)(((uint64_t)net->kdbStart[self] + (uint64_t)i) % net->n);
}
static uint32_t koorde_walkDeBruijnList(const orc_net* net, uint32_t self, const OKey* key)   /* 558-570 */
{
    int num = net->kdbNum[self];
    if (num == 0) return NONE;
    for (int i = 0; i < num - 1; i++) {
        uint32_t a = koorde_db(net, self, i), b = koorde_db(net, self, i + 1);
        if (ok_isBetweenR(key, &net->ids[a], &net->ids[b])) return a;
    }
    return koorde_db(net, self, num - 1);
}
/* Koorde::findStartKey (664-762) without its disabled #if 0 block; -1 = cRuntimeError */
static int koorde_findStartKey(const orc_net* net, const OKey* startKey, const OKey* endKey, const OKey* destKey,
                               OKey* out, int* step)
{
    if (EQ(startKey, endKey)) { *out = *startKey; return 0; }   /* step is left as it was */
    OKey diffKey = ok_sub(*endKey, startKey);
    int nBits = ok_log2(&diffKey);
    if (nBits < 0) nBits = 0;
    while ((160 - nBits) % net->p.shiftingBits != 0) nBits--;
    *step = nBits + 1;
    OKey newStart = ok_shl(ok_shr(*startKey, nBits), nBits);
    OKey tmpDest = ok_shr(*destKey, 160 - nBits);
    OKey newKey = ok_add(tmpDest, &newStart);
    if (ok_isBetweenR(&newKey, startKey, endKey)) { *out = newKey; return 0; }
    OKey pw = ok_pow2((uint32_t)nBits);
    newKey = ok_add(newKey, &pw);
    if (ok_isBetweenR(&newKey, startKey, endKey)) { *out = newKey; return 0; }
    set_err("Koorde::findStartKey(): Invalid start key");
    return -1;
}
/* Koorde::findDeBruijnHop (473-556) on a converged ring (deBruijnNode specified) */
static uint32_t koorde_findDeBruijnHop(const orc_net* net, uint32_t self, const OKey* destKey, KExt* ext,
                                       int* breakLookup, int* err)
{
    const orc_params* p = &net->p;
    uint32_t s0 = succ_get(net, self, 0);
    uint32_t dbNode = net->kdb[self];
    if (ext->routeKey.isUnspec) {
        int step = ext->step;
        OKey rk;
        if (koorde_findStartKey(net, &net->ids[self], &net->ids[s0], destKey, &rk, &step) < 0) { *err = 1; return NONE; }
        ext->routeKey = rk;
        ext->step = step;
    }
    if (ok_isBetweenR(&ext->routeKey, &net->ids[self], &net->ids[s0])) {
        if (ext->step > 160) { set_err("Koorde::findDeBruijnHop - Bounding error"); *err = 1; return NONE; }
        OKey add; memset(&add, 0, sizeof add);
        for (int i = 0; i < p->shiftingBits; i++) {
            int pos = 160 - ext->step - i;
            /* getBit(p) = getBitRange(p, 1): a position below 0 wraps to a huge uint32 -> throws */
            if (pos < 0) { set_err("OverlayKey::getBitRange(): invalid range"); *err = 1; return NONE; }
            OKey bit = ok_small(ok_getBitRange(destKey, (uint32_t)pos, 1));
            add = (i == 0) ? bit : ok_add(ok_shl(add, 1), &bit);
        }
        OKey rk = ok_add(ok_shl(ext->routeKey, p->shiftingBits), &add);
        ext->routeKey = rk;
        ext->step += p->shiftingBits;
        if (net->kdbNum[self] > 0) {
            uint32_t db0 = koorde_db(net, self, 0);
            if (ok_isBetweenR(&ext->routeKey, &net->ids[dbNode], &net->ids[db0])) return dbNode;
            return koorde_walkDeBruijnList(net, self, &ext->routeKey);
        }
        return dbNode;
    }
    *breakLookup = 1;
    if (p->useSucList) {
        uint32_t tmp = koorde_walkSuccessorList(net, self, &ext->routeKey);
        if (ok_isBetween(&net->ids[dbNode], &net->ids[tmp], &ext->routeKey)) return dbNode;
        return tmp;
    }
    return s0;
}
/* Koorde::findNode (405-471), state READY; the self-recursion (tmpHandle == thisNode and not
 * breakLookup) is the loop.  breakLookup is a member flag, but every return of findNode leaves
 * it false, so each call starts with it false. */
static int koorde_findNode(const orc_net* net, uint32_t self, const OKey* key, KExt* ext, NVec* out)
{
    nv_init(out, 0, 0, NULL);
    int breakLookup = 0;
    uint32_t pred = pred_get(net, self), s0 = succ_get(net, self, 0);
    int size = nsucc_get(net, self);
    for (;;) {
        if (ok_isBetweenR(key, &net->ids[pred], &net->ids[self])) { nv_push_back(out, self); return 0; }
        if (ok_isBetweenR(key, &net->ids[self], &net->ids[s0])) { nv_push_back(out, s0); return 0; }
        if (net->p.useOtherLookup) {
            uint32_t tmp = koorde_walkSuccessorList(net, self, key);
            if (tmp != succ_get(net, self, (uint32_t)size - 1)) { nv_push_back(out, tmp); return 0; }
        }
        int err = 0;
        uint32_t h = koorde_findDeBruijnHop(net, self, key, ext, &breakLookup, &err);
        if (err) return -1;
        if (h != self || breakLookup) { nv_push_back(out, h); return 0; }
    }
}

/* handleDeBruijnTimerExpired (164-230) once the ring has converged; the DeBruijnCall of its
 * third case is answered by the node responsible for the call's key (328-367) */
static void koorde_state(orc_net* net, uint32_t v)
{
    const orc_params* p = &net->p;
    int size = nsucc_get(net, v);
    OKey lookup = ok_shl(net->ids[v], p->shiftingBits);
    if (size > 0) {
        OKey d = ok_sub(net->ids[succ_get(net, v, (uint32_t)size / 2)], &net->ids[v]);
        lookup = ok_sub(lookup, &d);
    }
    uint32_t s0 = succ_get(net, v, 0), pred = pred_get(net, v);
    if (size == 0 || ok_isBetweenR(&lookup, &net->ids[v], &net->ids[s0])) {
        int sucNum = size < p->deBruijnListSize ? size : p->deBruijnListSize;
        net->kdb[v] = v; net->kdbStart[v] = s0; net->kdbNum[v] = (uint8_t)sucNum;
    } else if (ok_isBetweenR(&lookup, &net->ids[pred], &net->ids[v])) {
        int sucNum = size;
        if (sucNum + 1 > p->deBruijnListSize) sucNum = p->deBruijnListSize - 1;
        net->kdb[v] = pred; net->kdbStart[v] = v; net->kdbNum[v] = (uint8_t)(sucNum + 1);
    } else {
        uint32_t R = ring_responsible(net, &lookup);
        int sucNum = nsucc_get(net, R) + 1;
        if (sucNum > p->deBruijnListSize) sucNum = p->deBruijnListSize;
        net->kdb[v] = pred_get(net, R); net->kdbStart[v] = R; net->kdbNum[v] = (uint8_t)sucNum;
    }
}

orc_net* orc_koorde_build(const orc_key* ids, uint32_t n, const double* xy, const orc_params* p)
{
    if (p->shiftingBits < 1 || p->shiftingBits > 32 || p->deBruijnListSize < 1 || p->deBruijnListSize > 255) {
        set_err("koorde: shiftingBits must be 1..32, deBruijnListSize 1..255");
        return NULL;
    }
    /* the Chord part as lazy stable tables: Koorde's findNode reads only pred and successors */
    orc_net* net = chord_build(ids, n, xy, p, 1);
    if (!net) return NULL;
    net->type = NET_KOORDE;
    net->kdb = (uint32_t*)malloc(sizeof(uint32_t) * n);
    net->kdbStart = (uint32_t*)malloc(sizeof(uint32_t) * n);
    net->kdbNum = (uint8_t*)malloc(n);
    for (uint32_t v = 0; v < n; ++v) koorde_state(net, v);
    return net;
}

void orc_koorde_export(const orc_net* net, uint32_t* db, uint32_t* db_start, uint8_t* db_num)
{
    if (net->type != NET_KOORDE) return;
    memcpy(db, net->kdb, sizeof(uint32_t) * net->n);
    memcpy(db_start, net->kdbStart, sizeof(uint32_t) * net->n);
    memcpy(db_num, net->kdbNum, net->n);
}

uint32_t orc_koorde_find_node(const orc_net* net, uint32_t node, const orc_key* key, orc_key* route_key,
                              int* has_route_key, int* step)
{
    if (net->type != NET_KOORDE) { set_err("not a Koorde network"); return NONE; }
    OKey k = ok_from(key);
    KExt e;
    if (*has_route_key) e.routeKey = ok_from(route_key);
    else { memset(&e.routeKey, 0, sizeof e.routeKey); e.routeKey.isUnspec = 1; }
    e.step = *step;
    NVec v;
    if (koorde_findNode(net, node, &k, &e, &v) < 0) return NONE;
    *has_route_key = !e.routeKey.isUnspec;
    if (!e.routeKey.isUnspec) ok_to(&e.routeKey, route_key);
    *step = e.step;
    return v.v[0];
}

/* ---- overlay dispatch ---------------------------------------------------------- */
static int ov_findNode(const orc_net* net, uint32_t self, const OKey* key, int nr, int ns, NVec* out)
{
    if (net->type == NET_CHORD) return chord_findNode(net, self, key, nr, ns, out);
    if (net->type == NET_KOORDE) {
        KExt e;   /* a call without an extension: Koorde::findNode attaches a fresh one */
        memset(&e.routeKey, 0, sizeof e.routeKey); e.routeKey.isUnspec = 1; e.step = 1;
        return koorde_findNode(net, self, key, &e, out);
    }
    return kad_findNode(net, self, key, nr, ns, out);
}
static int ov_isSiblingFor(const orc_net* net, uint32_t node, uint32_t self, const OKey* key, int ns, int* err)
{
    if (net->type != NET_KAD) return chord_isSiblingFor(net, node, self, key, ns, err);   /* Koorde: Chord's */
    return kad_isSiblingFor(net, node, self, key, ns, err);
}
static int ov_maxRedundant(const orc_net* net)
{
    if (net->type == NET_CHORD && net->p.extendedFingerTable) return net->p.numFingerCandidates;   /* Chord.cc:416-419 */
    return net->type != NET_KAD ? 1 : net->p.k;   /* Chord.cc:416-419, Kademlia.cc:352-355 */
}

int orc_find_node(const orc_net* net, uint32_t node, const orc_key* key, int numRedundantNodes,
                  int numSiblings, uint32_t* out, int* sibling_flag)
{
    OKey k = ok_from(key);
    NVec v;
    int err = 0;
    if (ov_findNode(net, node, &k, numRedundantNodes, numSiblings, &v) < 0) return -1;
    for (int i = 0; i < v.size && i < 64; ++i) out[i] = v.v[i];
    *sibling_flag = ov_isSiblingFor(net, node, node, &k, numSiblings, &err);
    return v.size;
}

/* ===================================================================== */
/* 3. SimpleUnderlay delay                                               */
/* ===================================================================== */
static int64_t simtime(double d, int rnd)       /* SimTime(double) at simtime-scale -9 (default.ini:27) */
{
    double x = d * 1e9;
    return rnd ? (int64_t)floor(x + 0.5) : (int64_t)x;
}
float orc_coord_dist(const orc_net* net, uint32_t a, uint32_t b)                 /* SimpleNodeEntry.cc:145-153 */
{
    double sum_of_squares = 0;
    for (int i = 0; i < 2; i++) {
        double d = net->xy[2 * (size_t)a + i] - net->xy[2 * (size_t)b + i];
        sum_of_squares += d * d;                  /* pow(d, 2) == d*d */
    }
    return (float)sqrt(sum_of_squares);
}
/* calcDelay with the sender's tx.finished state (SimpleNodeEntry.cc:155-195) */
static int64_t calc_delay(const orc_net* net, uint32_t a, uint32_t b, int32_t bytes,
                          int64_t now, int64_t* txFinished)
{
    if (a == b) return 0;                                                          /* SimpleUDP.cc:322 */
    const orc_params* p = &net->p;
    int64_t bw = simtime((double)((int64_t)bytes * 8) / p->datarate, p->simtimeRound);
    int64_t newTx = (*txFinished > now ? *txFinished : now) + bw;
    *txFinished = newTx;
    int64_t access = simtime(p->accessDelay, p->simtimeRound);
    int64_t destBw = simtime((double)((int64_t)bytes * 8) / p->datarate, p->simtimeRound);
    int64_t coord = simtime(0.001 * (double)orc_coord_dist(net, a, b), p->simtimeRound);
    return (newTx - now) + access + coord + destBw + access;
}
int64_t orc_delay_ns(const orc_net* net, uint32_t a, uint32_t b, int32_t bytes)
{
    int64_t tx = 0;
    return calc_delay(net, a, b, bytes, 0, &tx);
}

/* ===================================================================== */
/* 6. IterativeLookup restatement (parallelPaths = 1, ITERATIVE_ROUTING, */
/*    no verify/majority siblings, failedNodeRpcs = false).              */
/* ===================================================================== */
#define MAXRPC 256
#define MAXNH 128

typedef struct { uint32_t handle; int alreadyUsed; } LEntry;

typedef struct {
    uint32_t node;          /* destination */
    int active;             /* in rpcs map / pending events */
    int64_t tResp, tTimeout, tIns;
    uint64_t seqResp, seqTimeout;
    int nInfo;
    int vrpcId[8];          /* RpcInfoVector (one path) */
    KExt extIn, extOut;     /* Koorde: the call's findNodeExt, and the one its response carries */
    int extInPresent;
} Rpc;

typedef struct {
    const orc_net* net;
    OKey key;
    uint32_t S;
    int numSiblings, hopCountMax;
    /* lookup */
    int finished, success, running;
    int64_t startTime, now, txFinished;
    uint32_t siblings[64]; int nsiblings;
    uint32_t* visited; int nvisited, capVisited;
    uint32_t dead[MAXRPC]; int ndead;
    int finishedPaths, successfulPaths, minHops;
    Rpc rpcs[MAXRPC]; int nrpcs;
    uint64_t seq;
    /* path */
    LEntry nh[MAXNH]; int nnh;
    int hops, step, pendingRpcs, pfinished, psuccess;
    /* outputs */
    uint32_t* hopseq; int nhop;
    uint32_t rpcsSent;
    /* Koorde: the findNodeExt the next FindNodeCalls carry (sendRpc's argument) */
    KExt ext; int extPresent;
    int broken;             /* a findNode threw (cRuntimeError in the reference): status BROKEN */
    /* EXHAUSTIVE_ITERATIVE_ROUTING (Kademlia bucket / sibling refresh): R = config.redundantNodes
     * of this lookup (the refresh sets it to bucketRefreshNodes / siblingRefreshNodes,
     * Kademlia.cc:1606-1611, 1660-1665), nextHops holds 2R (IterativeLookup.cc:770-778) */
    int exh, R, nhCap;
    int64_t* rtts;          /* exhaustive: RTT of every accepted response (hop order) */
    int64_t* tarrs;         /* ... the time the response reached the source (maintenance rounds) */
    uint32_t* cnode;        /* every FindNodeCall sent (maintenance rounds): its destination ... */
    int64_t* ctime;         /* ... and the time it reached it; ccap slots */
    int ncall, ccap;
} Lookup;

static int lk_getVisited(Lookup* L, uint32_t n)
{
    for (int i = 0; i < L->nvisited; ++i) if (L->visited[i] == n) return 1;
    return 0;
}
static void lk_setVisited(Lookup* L, uint32_t n)
{
    if (lk_getVisited(L, n)) return;
    if (L->nvisited == L->capVisited) {
        L->capVisited = L->capVisited ? 2 * L->capVisited : 64;
        L->visited = (uint32_t*)realloc(L->visited, sizeof(uint32_t) * (size_t)L->capVisited);
    }
    L->visited[L->nvisited++] = n;
}
static int lk_getDead(Lookup* L, uint32_t n)
{
    for (int i = 0; i < L->ndead; ++i) if (L->dead[i] == n) return 1;
    return 0;
}
static Rpc* lk_findRpc(Lookup* L, uint32_t n)
{
    for (int i = 0; i < L->nrpcs; ++i) if (L->rpcs[i].active && L->rpcs[i].node == n) return &L->rpcs[i];
    return NULL;
}
static int lk_activeRpcs(Lookup* L)
{
    int c = 0;
    for (int i = 0; i < L->nrpcs; ++i) c += L->rpcs[i].active;
    return c;
}

/* LookupVector comparator: IterativeLookup::compare -> overlay->distance(., key) (IterativeLookup.cc:397-400) */
static int lv_compare(Lookup* L, uint32_t a, uint32_t b)
{
    int metric = L->net->type != NET_KAD ? 2 : 1;
    OKey da = metric_dist(metric, &L->net->ids[a], &L->key);
    OKey db = metric_dist(metric, &L->net->ids[b], &L->key);
    return ok_cmp(&da, &db);
}
/* LookupVector::add (BaseKeySortedVector::add with LookupEntry, cap = redundantNodes) */
static int lv_add(Lookup* L, uint32_t h)
{
    int maxSize = L->nhCap;
    if (!(L->nnh != maxSize || lv_compare(L, h, L->nh[L->nnh - 1].handle) <= 0)) return -1;
    int pos = -1, i;
    if (L->nnh != 0) {
        for (i = 0, pos = 0; i < L->nnh; i++, pos++) {
            if (EQ(&L->net->ids[h], &L->net->ids[L->nh[i].handle])) return -1;
            if (lv_compare(L, h, L->nh[i].handle) < 0) {
                memmove(&L->nh[i + 1], &L->nh[i], sizeof(LEntry) * (size_t)(L->nnh - i));
                L->nh[i].handle = h; L->nh[i].alreadyUsed = 0; L->nnh++;
                break;
            }
        }
        if (i == L->nnh && pos == L->nnh) { pos = L->nnh; L->nh[L->nnh].handle = h; L->nh[L->nnh].alreadyUsed = 0; L->nnh++; }
    } else {
        pos = 0; L->nh[0].handle = h; L->nh[0].alreadyUsed = 0; L->nnh = 1;
    }
    if (L->nnh > maxSize) L->nnh = maxSize;
    return pos;
}
static int path_add(Lookup* L, uint32_t h)                                       /* 1184-1195 */
{
    if (L->net->p.lookupMerge) return lv_add(L, h);
    if (L->nnh < MAXNH) { L->nh[L->nnh].handle = h; L->nh[L->nnh].alreadyUsed = 0; L->nnh++; }
    else cap_error("more than MAXNH next hops");
    return L->nnh - 1;
}

static void lk_addSibling(Lookup* L, uint32_t h)                                /* 406-449 */
{
    /* numSiblings != 0, parallelPaths == 1, !verifySiblings -> push_back if not full */
    int cap = L->numSiblings == 0 ? 1 : L->numSiblings;
    if (L->numSiblings == 0) {
        if (EQ(&L->net->ids[h], &L->key)) { L->siblings[0] = h; L->nsiblings = 1; }
        return;
    }
    if (L->nsiblings < cap) L->siblings[L->nsiblings++] = h;   /* cap <= 64 (check_params, orc_lookup_batch, orc_kad_exhaustive_batch) */
}

/* IterativeLookup::sendRpc (656-689) + BaseRpc::sendRpcCall timeout (BaseRpc.cc:173-253) */
static void lk_sendRpc(Lookup* L, uint32_t handle, int rpcId)
{
    if (L->finished || !L->running) return;
    Rpc* r = lk_findRpc(L, handle);
    if (!r) {
        if (L->nrpcs == MAXRPC) { cap_error("more than MAXRPC FindNodeCalls in one lookup"); return; }
        r = &L->rpcs[L->nrpcs++];
        memset(r, 0, sizeof *r);
        r->node = handle; r->active = 1;
        const orc_params* p = &L->net->p;
        r->tTimeout = L->now + simtime(p->rpcUdpTimeout, p->simtimeRound);
        r->seqTimeout = L->seq++;
        /* the call travels S -> handle, the responder answers at once */
        const int koorde = L->net->type == NET_KOORDE;
        /* a Koorde call sent without an extension (after a late response) lacks its 21 B */
        int64_t d1 = calc_delay(L->net, L->S, handle, p->callBytes - ((koorde && !L->extPresent) ? 21 : 0), L->now,
                                &L->txFinished);
        int64_t tArr = L->now + d1;
        NVec res; int sflag, err;
        if (koorde) {
            r->extIn = L->ext; r->extInPresent = L->extPresent;
            r->extOut = L->ext;
            if (!L->extPresent) {   /* Koorde::findNode attaches a fresh extension (421-429) */
                memset(&r->extOut.routeKey, 0, sizeof r->extOut.routeKey);
                r->extOut.routeKey.isUnspec = 1; r->extOut.step = 1;
            }
            if (koorde_findNode(L->net, handle, &L->key, &r->extOut, &res) < 0) { L->broken = 1; res.size = 0; }
        } else   /* findNodeRpc: an exhaustive call asks findNode with numSiblings -1 (BaseOverlay.cc:1857-1859) */
            ov_findNode(L->net, handle, &L->key, L->R, L->exh ? -1 : L->numSiblings, &res);
        sflag = L->exh ? 0 : ov_isSiblingFor(L->net, handle, handle, &L->key, L->numSiblings, &err);
        (void)sflag;
        int64_t respTx = 0;   /* responder's tx queue idle */
        int64_t d2 = calc_delay(L->net, handle, L->S, resp_bytes(p, res.size), tArr, &respTx);
        r->tResp = tArr + d2;
        r->tIns = tArr;
        if (L->cnode) {
            if (L->ncall < L->ccap) { L->cnode[L->ncall] = handle; L->ctime[L->ncall] = tArr; ++L->ncall; }
            else cap_error("more FindNodeCalls than the call-record capacity");
        }
        r->seqResp = L->seq++;
        L->rpcsSent++;
    }
    if (r->nInfo < 8) r->vrpcId[r->nInfo++] = rpcId;
}

static void path_sendRpc(Lookup* L, int num)                                     /* 1067-1170 */
{
    const orc_params* p = &L->net->p;
    if (L->pfinished) return;
    if (L->hopCountMax && (L->hops >= L->hopCountMax)) { L->pfinished = 1; L->psuccess = 0; return; }
    if (p->lookupStrictParallelRpcs) num = num < (p->lookupParallelRpcs - L->pendingRpcs) ? num : (p->lookupParallelRpcs - L->pendingRpcs);
    if ((num == 0) && (L->pendingRpcs == 0) && !p->lookupFinishOnFirstUnchanged) num = p->lookupParallelRpcs;
    for (int i = 0; num > 0 && i < L->R; i++) {
        LEntry* it = NULL;
        for (int q = 0; q < L->nnh; ++q) {                                       /* getNextEntry 1172-1182 */
            if (L->nh[q].alreadyUsed || lk_getDead(L, L->nh[q].handle)) continue;
            it = &L->nh[q]; break;
        }
        if (it == NULL) break;
        if (!p->lookupVisitOnlyOnce || !lk_getVisited(L, it->handle)) {
            L->pendingRpcs++;
            num--;
            lk_sendRpc(L, it->handle, L->step);
        }
        it->alreadyUsed = 1;
    }
    if (L->pendingRpcs == 0) {
        if (L->exh) {   /* exhaustive lookups are always successful: siblings = nextHops[0..R) (1147-1156) */
            for (int q = 0; q < L->R && q < L->nnh; ++q) lk_addSibling(L, L->nh[q].handle);
            L->psuccess = 1;
        } else
            L->psuccess = 0;
        L->pfinished = 1;
    }
}

static void path_sendNewRpcAfterTimeout(Lookup* L)                               /* 923-933 */
{
    if (L->net->p.lookupNewRpcOnEveryTimeout) path_sendRpc(L, 1);
    else if (L->pendingRpcs == 0) path_sendRpc(L, L->net->p.lookupParallelRpcs);
}

static void path_handleTimeout(Lookup* L, uint32_t dest)                         /* 935-1023 */
{
    if (L->pfinished) return;
    if (L->exh && lk_getDead(L, dest)) {   /* exhaustive: dead nodes leave nextHops (948-957) */
        for (int q = 0; q < L->nnh; ++q)
            if (L->nh[q].handle == dest) {
                memmove(&L->nh[q], &L->nh[q + 1], sizeof(LEntry) * (size_t)(L->nnh - q - 1));
                L->nnh--;
                break;
            }
    }
    L->pendingRpcs--;
    if (L->now > L->startTime + simtime(L->net->p.lookupTimeout, L->net->p.simtimeRound)) {
        L->pfinished = 1; L->psuccess = 0; return;
    }
    path_sendNewRpcAfterTimeout(L);   /* failedNodeRpcs = false */
}

static int path_accepts(Lookup* L, int rpcId)                                    /* 786-801 */
{
    if (L->pfinished) return 0;
    if (L->net->p.lookupUseAllParallelResponses && L->net->p.lookupMerge) return 1;
    return rpcId == L->step;
}

static void path_handleResponse(Lookup* L, uint32_t source, const NVec* closest, int siblingsFlag,
                                int64_t rtt)                                     /* 803-921 */
{
    const orc_params* p = &L->net->p;
    if (L->pfinished) return;
    if (L->now > L->startTime + simtime(p->lookupTimeout, p->simtimeRound)) { L->pfinished = 1; L->psuccess = 0; return; }
    if (source != L->S) {
        L->hops++;
        if (L->hopseq && L->nhop < L->hopCountMax) L->hopseq[L->nhop] = source;
        if (L->rtts && L->nhop < L->hopCountMax) L->rtts[L->nhop] = rtt;
        if (L->tarrs && L->nhop < L->hopCountMax) L->tarrs[L->nhop] = L->now;
        L->nhop++;
    }
    lk_setVisited(L, source);
    L->step++;
    L->pendingRpcs--;
    if (closest->size != 0 && !p->lookupMerge) L->nnh = 0;
    int numNewRpcs = 0;
    for (int i = 0; i < closest->size; i++) {
        uint32_t h = closest->v[i];
        int pos = path_add(L, h);
        if ((pos >= 0) && (pos < L->R)) numNewRpcs++;
        if ((L->numSiblings == 0) && EQ(&L->net->ids[h], &L->key)) {
            lk_addSibling(L, h);
            L->pfinished = 1; L->psuccess = 1; return;
        } else if (L->numSiblings != 0 && !L->exh && siblingsFlag) {
            lk_addSibling(L, h);
        }
    }
    if (!L->exh && siblingsFlag && closest->size != 0 && L->numSiblings != 0) { L->pfinished = 1; L->psuccess = 1; return; }
    if ((numNewRpcs == 0) && p->lookupNewRpcOnEveryResponse) numNewRpcs = 1;
    path_sendRpc(L, numNewRpcs < p->lookupParallelRpcs ? numNewRpcs : p->lookupParallelRpcs);
}

static void lk_countFinished(Lookup* L)
{
    if (L->pfinished) {
        L->finishedPaths++;
        if (L->hops < L->minHops) L->minHops = L->hops;
        if (L->psuccess) L->successfulPaths++;
    }
}

/* checkStop (295-349) with parallelPaths = 1, numSiblings > 0 */
static int lk_checkStop(Lookup* L)
{
    int finishLookup = 0;
    if ((L->successfulPaths >= 1 && L->numSiblings == 0 && L->nsiblings >= 1) ||
        (L->finishedPaths == 1 && L->numSiblings > 0)) {
        L->success |= L->psuccess;
        finishLookup = 1;
    } else if (lk_activeRpcs(L) == 0) {
        finishLookup = 1;
    }
    if (finishLookup) {
        if (L->successfulPaths >= 1) L->success = 1;
        L->success |= L->psuccess;   /* stop(): success |= paths[i]->success */
        L->running = 0; L->finished = 1;
        return 1;
    }
    return 0;
}

/* lout != NULL: the lookup answers a LookupCall with numSiblings (KBRTestApp.cc:190-206,
 * BaseOverlay::lookupRpc 1938-1968) instead of routing the one-way message; the response is
 * built by SendToKeyListener::lookupFinished (BaseOverlay.cc:1272-1300) and sibs receives the
 * sibling vector (numSiblings slots, NONE padded). */
static void run_lookup(const orc_net* net, const OKey* key, uint32_t S, orc_route_out* out,
                       uint32_t* hopseq, uint32_t* rpcsOut, int numSiblings, orc_lookup_out* lout, uint32_t* sibs,
                       int exhR, int64_t* rtts, int64_t* tarrs, uint32_t* cnode, int64_t* ctime, int ccap)
{
    const orc_params* p = &net->p;
    Lookup* L = (Lookup*)calloc(1, sizeof(Lookup));
    L->net = net; L->key = *key; L->S = S;
    L->numSiblings = lout ? numSiblings : p->numSiblings; L->hopCountMax = p->hopCountMax;
    L->exh = exhR > 0;
    L->R = L->exh ? exhR : p->lookupRedundantNodes;
    L->nhCap = L->exh ? 2 * exhR : p->lookupRedundantNodes;
    L->rtts = rtts;
    L->tarrs = tarrs;
    L->cnode = cnode; L->ctime = ctime; L->ccap = ccap;
    L->hopseq = hopseq;
    L->minHops = 0x7fffffff;
    L->running = 1; L->startTime = 0; L->now = 0; L->txFinished = 0;
    /* start() 133-244 */
    NVec nextHops; int err;
    if (net->type == NET_KOORDE) {
        /* the local FindNodeCall gets a fresh extension from Koorde::findNode; start() hands it
         * to the first sendRpc (200-230) */
        memset(&L->ext.routeKey, 0, sizeof L->ext.routeKey);
        L->ext.routeKey.isUnspec = 1; L->ext.step = 1; L->extPresent = 1;
        if (koorde_findNode(net, S, key, &L->ext, &nextHops) < 0) { L->broken = 1; nextHops.size = 0; }
    } else
        ov_findNode(net, S, key, ov_maxRedundant(net), L->exh ? -1 : L->numSiblings, &nextHops);
    lk_setVisited(L, S);
    if (nextHops.size == 0) {
        L->finished = 1; L->success = 0;
    } else if (L->numSiblings == 0 && ov_isSiblingFor(net, S, S, key, 0, &err)) {
        /* an exact-key lookup the source is a sibling for (start() 171-184): found if it is the
         * source's own key */
        lk_addSibling(L, S);
        L->success = EQ(&net->ids[S], key);
        L->finished = 1;
    } else if (L->numSiblings != 0 && !L->exh && ov_isSiblingFor(net, S, S, key, L->numSiblings, &err)) {
        for (int i = 0; i < nextHops.size; i++) lk_addSibling(L, nextHops.v[i]);
        L->success = L->finished = 1;
    }
    int done = L->finished || L->broken;
    if (!done) {
        for (int i = 0; i < nextHops.size; ++i) path_add(L, nextHops.v[i]);
        path_sendRpc(L, p->lookupParallelRpcs);
        done = L->broken || lk_checkStop(L);
    }
    /* event loop */
    while (!done) {
        /* earliest pending event: (time, insertion time, seq); timeouts inserted at send */
        int best = -1, bestIsTimeout = 0;
        int64_t bt = 0, bi = 0; uint64_t bs = 0;
        for (int i = 0; i < L->nrpcs; ++i) {
            Rpc* r = &L->rpcs[i];
            if (!r->active) continue;
            int64_t t, ti; uint64_t s; int isTo;
            if (r->tTimeout <= r->tResp) { t = r->tTimeout; ti = r->tTimeout - simtime(p->rpcUdpTimeout, p->simtimeRound); s = r->seqTimeout; isTo = 1; }
            else { t = r->tResp; ti = r->tIns; s = r->seqResp; isTo = 0; }
            if (best < 0 || t < bt || (t == bt && (ti < bi || (ti == bi && s < bs)))) {
                best = i; bt = t; bi = ti; bs = s; bestIsTimeout = isTo;
            }
        }
        if (best < 0) { done = 1; break; }
        Rpc r = L->rpcs[best];
        L->rpcs[best].active = 0;            /* rpcs.erase(src) */
        L->now = bt;
        if (bestIsTimeout) {                 /* handleRpcTimeout 588-654 */
            if (L->ndead < MAXRPC) L->dead[L->ndead++] = r.node;
            else cap_error("more than MAXRPC dead nodes in one lookup");
            for (int q = 0; q < r.nInfo; ++q) {
                if (L->pfinished) continue;
                L->ext = r.extIn; L->extPresent = r.extInPresent;   /* the timed-out call's extension (965-969) */
                path_handleTimeout(L, r.node);
                lk_countFinished(L);
            }
        } else {                             /* handleRpcResponse 488-585 */
            NVec res; int sflag, err2;
            if (net->type == NET_KOORDE) {
                KExt e = r.extIn;
                if (!r.extInPresent) { memset(&e.routeKey, 0, sizeof e.routeKey); e.routeKey.isUnspec = 1; e.step = 1; }
                if (koorde_findNode(net, r.node, key, &e, &res) < 0) res.size = 0;   /* BROKEN was set at send */
            } else
                ov_findNode(net, r.node, key, L->R, L->exh ? -1 : L->numSiblings, &res);  /* BaseOverlay.cc:1857-1871 */
            sflag = L->exh ? 0 : ov_isSiblingFor(net, r.node, r.node, key, L->numSiblings, &err2);
            int rpcHandled = 0;
            for (int q = 0; q < r.nInfo; ++q) {
                if (L->pfinished) continue;
                if (!rpcHandled && (path_accepts(L, r.vrpcId[q]) || L->exh || (sflag && p->lookupAcceptLateSiblings))) {
                    L->ext = r.extOut; L->extPresent = 1;            /* the response's extension (908-911) */
                    path_handleResponse(L, r.node, &res, sflag,
                                        bt - (r.tTimeout - simtime(p->rpcUdpTimeout, p->simtimeRound)));
                    rpcHandled = 1;
                } else {
                    L->extPresent = 0;                               /* handleTimeout(NULL, ...): no extension */
                    path_handleTimeout(L, r.node);
                }
                lk_countFinished(L);
            }
        }
        done = L->broken || lk_checkStop(L);
    }
    if (L->broken) {
        /* the reference aborts (cRuntimeError) inside a Koorde findNode; the lookup is reported
         * BROKEN with the hops accepted so far */
        if (lout) {
            lout->hops = (uint16_t)L->hops; lout->is_valid = 0; lout->num_siblings = 0; lout->latency_ns = -1;
            lout->status = 5;
            for (int i = 0; i < (numSiblings ? numSiblings : 1); ++i) sibs[i] = NONE;
        } else {
            out->hops = (uint16_t)L->hops; out->responsible = NONE; out->status = 5;
            out->one_way_hops = 0; out->latency_ns = -1;
            if (rpcsOut) *rpcsOut = L->rpcsSent;
        }
        free(L->visited);
        free(L);
        return;
    }
    /* stop() -> SendToKeyListener::lookupFinished (BaseOverlay.cc:1241-1307) */
    int valid = L->success && L->finished;
    int minHops = (L->minHops == 0x7fffffff) ? 0 : L->minHops;
    if (lout) {
        /* LookupResponse: hopCount = getMinHops(), isValid, siblings = getResult() (1274-1286);
         * the internal LookupCall's RTT is the lookup's duration */
        lout->hops = (uint16_t)minHops;
        lout->is_valid = (uint8_t)(valid ? 1 : 0);
        lout->num_siblings = valid ? (uint32_t)L->nsiblings : 0;
        lout->latency_ns = valid ? L->now - L->startTime : -1;
        if (valid) lout->status = 0;
        else if (L->now > L->startTime + simtime(p->lookupTimeout, p->simtimeRound)) lout->status = 1;
        else if (L->ndead > 0) lout->status = 2;
        else if (L->hopCountMax && L->hops >= L->hopCountMax) lout->status = 3;
        else lout->status = 4;
        for (int i = 0; i < (numSiblings ? numSiblings : 1); ++i) sibs[i] = (valid && i < L->nsiblings) ? L->siblings[i] : NONE;
        if (rpcsOut) *rpcsOut = L->rpcsSent;
        free(L->visited);
        free(L);
        return;
    }
    out->hops = (uint16_t)minHops;
    if (valid && L->nsiblings > 0) {
        uint32_t R = L->siblings[0];
        out->responsible = R;
        out->status = 0;
        out->one_way_hops = (uint8_t)(minHops + (R != S ? 1 : 0));    /* sendRouteMessage 1130-1132 */
        int64_t tx = L->txFinished;
        int64_t dfin = calc_delay(net, S, R, p->routeBytes, L->now, &tx);
        out->latency_ns = L->now - L->startTime + dfin;
    } else {
        out->responsible = NONE;
        /* classify the failure */
        if (L->now > L->startTime + simtime(p->lookupTimeout, p->simtimeRound)) out->status = 1;
        else if (L->ndead > 0) out->status = 2;
        else if (L->hopCountMax && L->hops >= L->hopCountMax) out->status = 3;
        else out->status = 4;
        out->one_way_hops = 0;
        out->latency_ns = -1;
    }
    if (rpcsOut) *rpcsOut = L->rpcsSent;
    free(L->visited);
    free(L);
}

/* ===================================================================== */
/* 7. Recursive routing (SEMI_RECURSIVE / FULL_RECURSIVE).  recordRoute =  */
/*    false, routeMsgAcks = false (default.ini:398, 434).  A one-way      */
/*    KBRTestMessage travels the same way under both: they differ only in */
/*    how an RPC response travels back (BaseOverlay.cc:1802-1818).        */
/* ===================================================================== */
typedef struct {
    uint32_t node;     /* the node the message was delivered to */
    int hops;          /* route hops */
    int status;        /* 0 delivered, else OVS_LOOKUP_* of the drop */
    int64_t t;         /* delivery time */
    int64_t tx;        /* the delivering node's tx queue (busy until) after its R/Kademlia hook */
} RecEnd;

/* the KademliaRoutingInfoMessage of R/Kademlia's hook at node x (Kademlia.cc:1031-1045):
 * findNode(key, k, s) nodes, KADEMLIAROUTINGINFO_L = TYPE_L + NODEHANDLE_L + KEY_L + n *
 * MARKEDNODEHANDLE_L = 376 + 216 n bits (KademliaMessage.msg:27-37), + UDP/IP 28 B */
static int32_t kad_info_bytes(const orc_net* net, uint32_t x, const OKey* key)
{
    NVec v;
    kad_findNode(net, x, key, net->p.k, net->p.s, &v);
    return 47 + 27 * v.size + 28;
}

/* One BaseRouteMessage from `from` (its srcNode) towards key, leaving `from` at t0 with from's
 * tx queue busy until tx0.  nsFrom: numSiblings of the first sendToKey (the route RPC of a
 * LookupCall passes the call's own, BaseOverlay.cc:1764-1775); forwarding hops use 1 (1003).
 * At every node: delivery when sibling (907-914, not at the source), findNode(key,
 * recNumRedundantNodes, numSiblings), drop on an empty result or hopCountMax (1449-1488),
 * loop detection (1497-1521), local delivery when the first usable candidate is the node itself
 * (1555-1570), else sendRouteMessage (1107-1146) with the node's queue idle on arrival.
 * R/Kademlia (recursiveRoutingHook, Kademlia.cc:1022-1057, altRecMode = false): every node the
 * message reaches other than its srcNode first sends a KademliaRoutingInfoMessage to the srcNode
 * -- at a forwarding hop before sendRouteMessage (BaseOverlay.cc:1577-1579), at the delivering
 * node before the message is handled (978-984) -- so that message leaves the node's queue first.
 * Its routingAdd calls change tables the batch holds fixed. */
/* routingType "source-routing-recursive" (RECURSIVE_SOURCE_ROUTING, BaseOverlay.cc:129-130): every
 * node a route message reaches appends its sender to the message's visitedHops (888-897), and the
 * loop detection of the forwarding node also skips every visited hop (1502-1516).  The message's
 * length is set once, when sendToKey creates it (1398: BASEROUTE_L with empty visited / next-hop
 * arrays) and is not updated as visitedHops grows, so the per-hop delays equal semi-recursive
 * routing's.  visited: the senders in arrival order (visited[0] = the source), nvis of them. */
#define REC_MAXVIS 256
static RecEnd rec_route_v(const orc_net* net, const OKey* key, uint32_t from, int nsFrom, int32_t bytes, int64_t t0,
                          int64_t tx0, uint32_t* hopseq, uint32_t* visited, int* nvis)
{
    const orc_params* p = &net->p;
    const int hook = net->type == NET_KAD;
    const int srcroute = p->routingType == 4;
    RecEnd e;
    e.node = NONE; e.hops = 0; e.status = 0; e.t = t0; e.tx = tx0;
    uint32_t cur = from, lastHop = from;   /* routeCtrlInfo->setLastHop(thisNode) (BaseOverlay.cc:1400) */
    int hopCount = 0, nv = 0;
    int64_t t = t0, tx = tx0;
    if (nvis) *nvis = 0;
    for (;;) {
        int err = 0;
        const int ns = cur == from ? nsFrom : 1;
        if (cur != from && srcroute) {
            /* receipt: the sender joins visitedHops (BaseOverlay.cc:888-897) */
            if (nv >= REC_MAXVIS) { cap_error("source route longer than 256 hops"); e.status = 3; return e; }
            if (visited) visited[nv] = lastHop;
            ++nv;
            if (nvis) *nvis = nv;
        }
        if (cur != from) {
            tx = 0;
            if (ov_isSiblingFor(net, cur, cur, key, 1, &err)) {
                if (hook) calc_delay(net, cur, from, kad_info_bytes(net, cur, key), t, &tx);
                break;
            }
        }
        NVec nextHops;
        if (ov_findNode(net, cur, key, p->recNumRedundantNodes, ns, &nextHops) < 0) {
            e.status = 5;               /* Chord throws: successor list broken (Chord.cc:615-620) */
            return e;
        }
        if (nextHops.size == 0) { e.status = 4; return e; }            /* 1449-1461: dropped */
        if (hopCount >= p->hopCountMax) { e.status = 3; return e; }    /* 1464-1488: dropped */
        const int isSibling = ov_isSiblingFor(net, cur, cur, key, ns, &err);
        uint32_t next = NONE;
        for (int i = 0; next == NONE && i < nextHops.size; ++i) {      /* 1502-1516 loop detection */
            const uint32_t h = nextHops.v[i];
            if ((h == lastHop && h != cur) ||                          /* back to the last hop */
                (h == from && cur != from) ||                          /* never to the source */
                (h == cur && !isSibling))                              /* self without being sibling */
                continue;
            if (srcroute && visited) {                                 /* a visited hop (source routing) */
                int seen = 0;
                for (int j = 0; j < nv && !seen; ++j) seen = visited[j] == h;
                if (seen) continue;
            }
            next = h;
        }
        if (next == NONE) { e.status = 4; return e; }                  /* 1518-1538: no useful next hop */
        if (next == cur) {                                             /* 1555-1570: this node is responsible */
            if (isSibling && !err) break;
            e.status = 5;
            return e;
        }
        if (hook && cur != from) calc_delay(net, cur, from, kad_info_bytes(net, cur, key), t, &tx);
        t += calc_delay(net, cur, next, bytes, t, &tx);
        if (hopseq && hopCount < p->hopCountMax) hopseq[hopCount] = next;
        ++hopCount;
        lastHop = cur;
        cur = next;
    }
    e.node = cur; e.hops = hopCount; e.t = t; e.tx = tx;
    return e;
}

static RecEnd rec_route(const orc_net* net, const OKey* key, uint32_t from, int nsFrom, int32_t bytes, int64_t t0,
                        int64_t tx0, uint32_t* hopseq)
{
    uint32_t vis[REC_MAXVIS];
    int nv = 0;
    return rec_route_v(net, key, from, nsFrom, bytes, t0, tx0, hopseq, vis, &nv);
}

/* A source-routed message from `from` along route[0 .. nroute) (sendToKey with a sourceRoute,
 * BaseOverlay.cc:1419-1431; each hop pops itself off nextHops and forwards to the next, 888-905,
 * 1003), delivered at the last node.  No findNode, no hop limit.  R/Kademlia: every node it reaches
 * other than its srcNode (`from`) first sends the srcNode a KademliaRoutingInfoMessage about the
 * message's destKey (Kademlia.cc:1022-1057) -- forwarding nodes before sendRouteMessage, so the
 * message waits for that one's serialisation.  Returns the delivery time. */
static int64_t src_route(const orc_net* net, const OKey* destKey, uint32_t from, const uint32_t* route, int nroute,
                         int32_t bytes, int64_t t0, int64_t tx0)
{
    const int hook = net->type == NET_KAD;
    uint32_t cur = from;
    int64_t t = t0, tx = tx0;
    for (int i = 0; i < nroute; ++i) {
        const uint32_t next = route[i];
        if (cur != from) {
            tx = 0;
            if (hook) calc_delay(net, cur, from, kad_info_bytes(net, cur, destKey), t, &tx);
        }
        t += calc_delay(net, cur, next, bytes, t, &tx);
        cur = next;
    }
    return t;
}

/* a one-way KBRTestMessage: sendToKey(key, msg, numSiblings = 1) (BaseOverlay.cc:1357) ->
 * KBRTestApp::deliver -> evaluateData(simTime() - creationTime, hopCount) (KBRTestApp.cc:404-410) */
static void run_recursive(const orc_net* net, const OKey* key, uint32_t S, orc_route_out* out, uint32_t* hopseq)
{
    const RecEnd e = rec_route(net, key, S, net->p.numSiblings, net->p.routeBytes, 0, 0, hopseq);
    out->responsible = NONE; out->hops = 0; out->one_way_hops = 0; out->latency_ns = -1;
    out->status = (uint8_t)e.status;
    if (e.status) return;
    out->responsible = e.node;
    out->hops = (uint16_t)e.hops;
    out->one_way_hops = (uint8_t)e.hops;
    out->latency_ns = e.t;
}

/* A LookupCall with recursive routing: BaseOverlay::lookupRpc -> RecursiveLookup::lookup
 * (BaseOverlay.cc:1938-1969, RecursiveLookup.cc:52-70): FindNodeCall{key, numRedundantNodes =
 * lookupRedundantNodes (BaseOverlay.cc:162), numSiblings} routed as a route RPC (136 B: BASEROUTE_L
 * 424 + FINDNODECALL_L 440 bits + UDP/IP); the delivering node D answers findNodeRpc (1841-1915):
 * findNode(key, numRedundantNodes, numSiblings) and the flag isSiblingFor(D, key, numSiblings).
 * The response (internalSendRpcResponse, 1779-1822): semi-recursive -> UDP from D to the source;
 * full-recursive -> routed from D to the source's key (numSiblings 1), lost when it ends at another
 * node; D = the source -> zero delay (SimpleUDP.cc:322).  RecursiveLookup::handleRpcResponse
 * (RecursiveLookup.cc:120-139): valid = flag && nodes; siblings = the response's nodes; hops =
 * getMinHops() = 0.  A lost or dropped call times out after rpcKeyTimeout (BaseRpc.cc:201-205) and
 * is resent once (lookupRpc passes retries = 1; the nonce stays, so a late first response still
 * counts): it fails from 2 * rpcKeyTimeout on.  Statuses: the drop's (3 / 4 / 5), 2 for a lost
 * response or a response after 2 * rpcKeyTimeout, 6 for an answer without the siblings flag. */
static void run_recursive_call(const orc_net* net, const OKey* key, uint32_t S, int numSiblings, orc_lookup_out* out,
                               uint32_t* sib)
{
    const orc_params* p = &net->p;
    const int nslots = numSiblings ? numSiblings : 1;
    for (int i = 0; i < nslots; ++i) sib[i] = NONE;
    out->num_siblings = 0; out->hops = 0; out->is_valid = 0; out->latency_ns = -1;
    uint32_t dvis[REC_MAXVIS];
    int dv = 0;
    const RecEnd d = rec_route_v(net, key, S, numSiblings, 53 + 55 + 28, 0, 0, NULL, dvis, &dv);
    if (d.status) { out->status = (uint8_t)d.status; return; }
    NVec res;
    int err = 0;
    if (ov_findNode(net, d.node, key, p->lookupRedundantNodes, numSiblings, &res) < 0) res.size = 0;
    const int flag = ov_isSiblingFor(net, d.node, d.node, key, numSiblings, &err);
    int64_t T = d.t;
    if (d.node != S) {
        const int32_t resp = resp_bytes(p, res.size);
        if (p->routingType == 1) {
            int64_t tx = d.tx;
            T += calc_delay(net, d.node, S, resp, d.t, &tx);
        } else if (p->routingType == 4) {
            /* source routing: the response goes back along the call's recorded route, reversed
             * (BaseRpc.cc:575-588: sourceRoute = visitedHops from the last to the first, sent with
             * ROUTE_TRANSPORT and RECURSIVE_SOURCE_ROUTING), a 53 B route header + the response */
            uint32_t rev[REC_MAXVIS];
            for (int i = 0; i < dv; ++i) rev[i] = dvis[dv - 1 - i];
            T = src_route(net, &net->ids[S], d.node, rev, dv, 53 + resp, d.t, d.tx);
        } else {
            const RecEnd r = rec_route(net, &net->ids[S], d.node, 1, 53 + resp, d.t, d.tx, NULL);
            if (r.status || r.node != S) { out->status = 2; return; }
            T = r.t;
        }
    }
    if (T >= 2 * simtime(p->rpcKeyTimeout, p->simtimeRound)) { out->status = 2; return; }
    if (!flag || res.size == 0) { out->status = 6; return; }
    const int cnt = res.size < nslots ? res.size : nslots;
    for (int i = 0; i < cnt; ++i) sib[i] = res.v[i];
    out->num_siblings = (uint32_t)res.size;
    out->status = 0;
    out->is_valid = 1;
    out->latency_ns = T;
}

uint64_t orc_route_batch(const orc_net* net, const orc_key* keys, const uint32_t* src, uint64_t n,
                         orc_route_out* out, uint32_t* hop_seq, uint32_t* rpcs_out, int nthreads)
{
    uint64_t total = 0;
    int hcm = net->p.hopCountMax > 0 ? net->p.hopCountMax : 1;
    if (net->type == NET_KOORDE && net->p.routingType != 0) { set_err("Koorde: iterative routing only"); return ORC_FAIL; }
    if (hop_seq) for (uint64_t i = 0; i < n * (uint64_t)hcm; ++i) hop_seq[i] = NONE;
    /* routingType "exhaustive-iterative" (BaseOverlay.cc:123-124, 1434-1442): an exhaustive
     * IterativeLookup with config.redundantNodes = lookupRedundantNodes (Kademlia only here) */
    const int exh = net->p.routingType == 3 ? net->p.lookupRedundantNodes : 0;
    if (exh && (net->type != NET_KAD || net->p.numSiblings > exh)) {
        set_err("exhaustive-iterative: Kademlia, numSiblings <= lookupRedundantNodes (IterativeLookup.cc:714-719)");
        return ORC_FAIL;
    }
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 256) reduction(+ : total) num_threads(nthreads)
#endif
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        OKey k = ok_from(&keys[i]);
        if (net->p.routingType == 0 || net->p.routingType == 3)    /* 1, 2, 4: recursive */
            run_lookup(net, &k, src[i], &out[i], hop_seq ? hop_seq + (size_t)i * hcm : NULL,
                       rpcs_out ? &rpcs_out[i] : NULL, 0, NULL, NULL, exh, NULL, NULL, NULL, NULL, 0);
        else {
            run_recursive(net, &k, src[i], &out[i], hop_seq ? hop_seq + (size_t)i * hcm : NULL);
            if (rpcs_out) rpcs_out[i] = 0;     /* no FindNodeCalls in recursive routing */
        }
        total += out[i].hops;
    }
    (void)nthreads;
    return g_cap_fail ? ORC_FAIL : total;
}

int orc_lookup_batch(const orc_net* net, const orc_key* keys, const uint32_t* src, uint64_t n, int numSiblings,
                     orc_lookup_out* out, uint32_t* siblings, int nthreads)
{
    const int maxs = net->type != NET_KAD ? net->p.successorListSize : net->p.s;
    if (numSiblings < 0) numSiblings = maxs;                              /* BaseOverlay.cc:1942-1944 */
    if (numSiblings > maxs) { set_err("numSiblings too big!"); return -1; }
    if (numSiblings < 0 || numSiblings > 16) { set_err("numSiblings must be 0..16"); return -1; }
    if (numSiblings == 0 && net->type == NET_KOORDE) { set_err("numSiblings = 0: Chord and Kademlia only"); return -1; }
    if (net->p.routingType < 0 || net->p.routingType > 4) { set_err("LookupCall: routingType 0..4"); return -1; }
    if (net->type == NET_KOORDE && net->p.routingType != 0) { set_err("Koorde: iterative routing only"); return -1; }
    const int exh = net->p.routingType == 3 ? net->p.lookupRedundantNodes : 0;
    if (exh && (net->type != NET_KAD || numSiblings > exh)) {
        set_err("exhaustive-iterative: Kademlia, numSiblings <= lookupRedundantNodes (IterativeLookup.cc:714-719)");
        return -1;
    }
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 256) num_threads(nthreads)
#endif
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        OKey k = ok_from(&keys[i]);
        orc_route_out dummy;
        /* numSiblings = 0 (an exact-key lookup) keeps a one-slot sibling vector (start() 149) */
        if (net->p.routingType == 1 || net->p.routingType == 2 || net->p.routingType == 4)
            run_recursive_call(net, &k, src[i], numSiblings, &out[i], siblings + (size_t)i * (numSiblings ? numSiblings : 1));
        else
            run_lookup(net, &k, src[i], &dummy, NULL, NULL, numSiblings, &out[i],
                       siblings + (size_t)i * (numSiblings ? numSiblings : 1), exh, NULL, NULL, NULL, NULL, 0);
    }
    (void)nthreads;
    return g_cap_fail ? -1 : numSiblings;
}

/* ======================================================================== */
/* Kademlia refresh lookups (Kademlia::handleBucketRefreshTimerExpired,      */
/* Kademlia.cc:1591-1686, exhaustiveRefresh = true, iterative routing).      */
/* ======================================================================== */
int orc_kad_exhaustive_batch_t(const orc_net* net, const orc_key* keys, const uint32_t* src, uint64_t n, int R,
                               orc_lookup_out* out, uint32_t* siblings, uint32_t* responders, int64_t* rtts,
                               int64_t* tarrs, uint32_t* cnode, int64_t* ctime, int ccap, uint32_t* rpcs,
                               int nthreads)
{
    if (net->type != NET_KAD) { set_err("exhaustive refresh lookups: Kademlia only"); return -1; }
    if (R < 1 || R > 64) { set_err("redundantNodes of a refresh lookup must be 1..64"); return -1; }
    if (net->p.routingType != 0) { set_err("exhaustive-iterative: iterative routing only"); return -1; }
    const int hcm = net->p.hopCountMax > 0 ? net->p.hopCountMax : 1;
    if (responders) for (uint64_t i = 0; i < n * (uint64_t)hcm; ++i) responders[i] = NONE;
    if (rtts) for (uint64_t i = 0; i < n * (uint64_t)hcm; ++i) rtts[i] = -1;
    if (tarrs) for (uint64_t i = 0; i < n * (uint64_t)hcm; ++i) tarrs[i] = -1;
    if (cnode) for (uint64_t i = 0; i < n * (uint64_t)ccap; ++i) { cnode[i] = NONE; ctime[i] = -1; }
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 64) num_threads(nthreads)
#endif
    for (int64_t i = 0; i < (int64_t)n; ++i) {
        OKey k = ok_from(&keys[i]);
        orc_route_out dummy;
        /* lookup(key, numSiblings = R, ...) with config.redundantNodes = R (1606-1610, 1660-1664) */
        run_lookup(net, &k, src[i], &dummy, responders ? responders + (size_t)i * hcm : NULL,
                   rpcs ? &rpcs[i] : NULL, R, &out[i], siblings + (size_t)i * R, R,
                   rtts ? rtts + (size_t)i * hcm : NULL, tarrs ? tarrs + (size_t)i * hcm : NULL,
                   cnode ? cnode + (size_t)i * ccap : NULL, ctime ? ctime + (size_t)i * ccap : NULL, ccap);
    }
    (void)nthreads;
    return g_cap_fail ? -1 : R;
}

int orc_kad_exhaustive_batch(const orc_net* net, const orc_key* keys, const uint32_t* src, uint64_t n, int R,
                             orc_lookup_out* out, uint32_t* siblings, uint32_t* responders, int64_t* rtts,
                             uint32_t* rpcs, int nthreads)
{
    return orc_kad_exhaustive_batch_t(net, keys, src, n, R, out, siblings, responders, rtts, NULL, NULL, NULL, 0,
                                      rpcs, nthreads);
}

uint64_t orc_kad_refresh_keys(const orc_net* net, const uint32_t* nodes, uint64_t m, const uint32_t* stale,
                              orc_key* keys, uint32_t* src, uint64_t cap)
{
    uint64_t cnt = 0;
    if (net->type != NET_KAD) { set_err("bucket refresh: Kademlia only"); return ORC_FAIL; }
    for (uint64_t j = 0; j < m; ++j) {
        const uint32_t v = nodes[j];
        KadTab T = kad_tab(net, v);
        if (T.nsib == 0) continue;                       /* if (siblingTable->size()) (1632) */
        /* diff = L - b*(sharedPrefixLength(front, b) + 1) (1636-1637) */
        const int B = net->p.b, per = (1 << B) - 1;
        orc_key me, fr;
        ok_to(&net->ids[v], &me);
        {
            /* the front: the XOR-closest sibling */
            uint32_t f = T.sib[0];
            for (int q = 1; q < T.nsib; ++q) {
                OKey d1 = ok_xor(net->ids[v], &net->ids[T.sib[q]]), d0 = ok_xor(net->ids[v], &net->ids[f]);
                if (ok_cmp(&d1, &d0) < 0) f = T.sib[q];
            }
            ok_to(&net->ids[f], &fr);
        }
        const int spl = (int)orc_key_shared_prefix(&me, &fr, (uint32_t)B);
        const int diff = 160 - B * (spl + 1);
        const uint64_t sw = ((uint64_t)net->nb + 31) / 32;      /* stale mask words per node */
        for (int i = 160 - B; i >= diff; i -= B) {               /* 1639-1676 */
            for (int d = 0; d < per; ++d) {
                const int index = (i / B) * per + d;
                if (index < 0) continue;
                if (stale && !((stale[j * sw + (uint64_t)(index >> 5)] >> (index & 31)) & 1u)) continue;
                if (cnt < cap) {
                    /* thisNode.key ^ (OverlayKey(d + 1) << i) (1647-1648) */
                    OKey key = net->ids[v];
                    for (int bit = 0; bit < B; ++bit)
                        if (((d + 1) >> bit) & 1) { OKey pw = ok_pow2((uint32_t)(i + bit)); key = ok_xor(key, &pw); }
                    ok_to(&key, &keys[cnt]);
                    src[cnt] = v;
                }
                ++cnt;
            }
        }
    }
    return cnt;
}

/* ======================================================================== */
/* Kademlia maintenance: routingAdd and one synchronous refresh round.       */
/* ======================================================================== */
/* Kademlia::routingAdd (Kademlia.cc:432-756) on explicit tables, with the default
 * secureMaintenance = false, pingNewSiblings = false, activePing = false and
 * proximityNeighborSelection = false (default.ini:191, 201, 219-221), any bucketType
 * (routingBucketSize, 384-411; the nkademlia branch 620-664 with currentRoutingTableSize).  The replacement cache (729-745) and its pings never change
 * a table's membership without RPC timeouts, so a rejected add is only counted.  rtt / lastSeen
 * are not modelled (nothing in routing reads them).  Returns routingAdd's result. */
static int kad_routingAdd(orc_net* net, uint32_t self, uint32_t h, int isAlive, orc_kad_round_stats* st)
{
    if (h == self) return 0;                                          /* 437-439 */
    const int sibCap = 5 * net->p.s;
    uint32_t* sib = net->sib + (size_t)self * sibCap;
    const int nsib = net->nsib[self];
    for (int i = 0; i < nsib; ++i)                                    /* already a sibling: 454-481 */
        if (sib[i] == h) { if (isAlive) st->refreshed++; return 1; }
    const int bi = kad_routingBucketIndex(net, self, &net->ids[h], 0);
    if (bi >= 0) {                                                    /* routingBucket(key, false) */
        const size_t bx = (size_t)self * (size_t)net->nb + (size_t)bi;
        for (int i = 0; i < net->bdcnt[bx]; ++i)                      /* already in a bucket: 483-535 */
            if (net->bdyn[bx][i] == h) {
                if (isAlive) {                                        /* erase + push_back (514-517) */
                    kad_dyn_erase(net, self, bi, i);
                    kad_dyn_push(net, self, bi, h);
                    st->refreshed++;
                }
                return 1;
            }
    }
    int result = 0;
    uint32_t cur = h;
    NVec sv; nv_init(&sv, sibCap, 1, &net->ids[self]);               /* siblingTable, XOR to self */
    for (int i = 0; i < nsib; ++i) sv.v[i] = sib[i];
    sv.size = nsib;
    if (nv_isAddable(net, &sv, h)) {                                  /* 537-616 */
        if (nv_isFull(&sv)) {
            const uint32_t old = sv.v[sv.size - 1];                   /* preempted handle (579) */
            nv_add(net, &sv, h);
            cur = old;
            result = 1;
            st->sib_changes++;
        } else {
            nv_add(net, &sv, h);
            for (int i = 0; i < sv.size; ++i) sib[i] = sv.v[i];
            net->nsib[self] = (uint8_t)sv.size;
            st->sib_changes++;
            return 1;
        }
        for (int i = 0; i < sv.size; ++i) sib[i] = sv.v[i];
        net->nsib[self] = (uint8_t)sv.size;
    }
    const int b2 = kad_routingBucketIndex(net, self, &net->ids[cur], 0);   /* routingBucket(.., true) 619 */
    if (b2 < 0) { cap_error("routingAdd: bucket index -1 (the reference dereferences a NULL bucket)"); return result; }
    const size_t bx2 = (size_t)self * (size_t)net->nb + (size_t)b2;
    if (net->p.bucketType == 1) {                                     /* NKADEMLIA (620-664) */
        if (net->bdcnt[bx2] >= net->p.k && (int64_t)net->rts[self] >= (int64_t)net->p.globalNodeLimit) {
            if (cur != h) st->lost++;
            else if (isAlive) st->replacement++;
            return 0;
        }
        kad_dyn_push(net, self, b2, cur);
        net->rts[self]++;
        st->bucket_changes++;
        return 1;
    }
    const int cap = orc_kad_bucket_size(&net->p, b2);
    if (net->bdcnt[bx2] < cap) {                                      /* !bucket->isFull() 665-701 */
        kad_dyn_push(net, self, b2, cur);
        net->rts[self]++;
        st->bucket_changes++;
        return 1;
    }
    if (cur != h) st->lost++;            /* a preempted sibling whose bucket is full leaves the tables */
    else if (isAlive) st->replacement++; /* replacement cache (729-745) */
    return result;
}

/* FindNodeCalls a lookup can send: at most alpha pending, a new one per response or timeout,
 * responses bounded by hopCountMax (sendRpc stops there); timeouts add one each, bounded by the
 * MAXRPC calls of the restatement */
static int kad_call_cap(const orc_net* net)
{
    const int hcm = net->p.hopCountMax > 0 ? net->p.hopCountMax : 1;
    return 2 * hcm + 2 * net->p.lookupParallelRpcs + 16;
}

int orc_kad_routing_add(orc_net* net, uint32_t v, uint32_t x, int isAlive)
{
    orc_kad_round_stats st; memset(&st, 0, sizeof st);
    if (net->type != NET_KAD || net->lazy || !net->bdyn || v >= net->n || x >= net->n) { set_err("routing_add: explicit Kademlia tables"); return -1; }
    return kad_routingAdd(net, v, x, isAlive, &st);
}

/* one routingAdd event of a round at one node */
typedef struct { int64_t t; int kind; uint32_t task, idx; } KEvt;

static int kevt_cmp(const void* a, const void* b)
{
    const KEvt* x = (const KEvt*)a; const KEvt* y = (const KEvt*)b;
    if (x->t != y->t) return x->t < y->t ? -1 : 1;
    if (x->kind != y->kind) return x->kind < y->kind ? -1 : 1;
    if (x->task != y->task) return x->task < y->task ? -1 : 1;
    if (x->idx != y->idx) return x->idx < y->idx ? -1 : 1;
    return 0;
}

uint64_t orc_kad_maintenance_round(orc_net* net, const uint32_t* nodes, uint64_t m, const uint8_t* flags,
                                   const uint32_t* stale, orc_kad_round_stats* st, int nthreads)
{
    orc_kad_round_stats z; memset(&z, 0, sizeof z);
    if (st) *st = z; else st = &z;
    if (net->type != NET_KAD || net->lazy || !net->bdyn) { set_err("maintenance round: explicit Kademlia tables"); return ORC_FAIL; }
    if (net->p.routingType != 0) { set_err("maintenance round: iterative routing"); return ORC_FAIL; }
    const int hcm = net->p.hopCountMax > 0 ? net->p.hopCountMax : 1;
    /* the round's tasks, per listed node in list order (handleBucketRefreshTimerExpired,
     * Kademlia.cc:1591-1686, exhaustiveRefresh): flags bit 0 = the sibling-table refresh, a lookup
     * of the node's own key with siblingRefreshNodes = 5s (1604-1611); bit 1 = the bucket
     * refreshes of the stale buckets with bucketRefreshNodes = lookupRedundantNodes (1631-1676) */
    const int Rs = 5 * net->p.s, Rb = net->p.lookupRedundantNodes;
    uint64_t cap = 0;
    for (uint64_t j = 0; j < m; ++j) cap += 1 + (uint64_t)net->nb;
    orc_key* keys = (orc_key*)malloc(sizeof(orc_key) * cap);
    uint32_t* src = (uint32_t*)malloc(sizeof(uint32_t) * cap);
    int* tR = (int*)malloc(sizeof(int) * cap);
    uint64_t nt = 0;
    for (uint64_t j = 0; j < m; ++j) {
        const uint32_t v = nodes[j];
        if (v >= net->n) { set_err("maintenance round: node index out of range"); free(keys); free(src); free(tR); return ORC_FAIL; }
        const uint8_t f = flags ? flags[j] : 3;
        if (f & 1) { ok_to(&net->ids[v], &keys[nt]); src[nt] = v; tR[nt] = Rs; ++nt; }
        if (f & 2) {
            const uint64_t sw = ((uint64_t)net->nb + 31) / 32;
            const uint64_t c = orc_kad_refresh_keys(net, &v, 1, stale ? stale + j * sw : NULL, keys + nt, src + nt,
                                                    (uint64_t)net->nb);
            for (uint64_t q = 0; q < c; ++q) tR[nt + q] = Rb;
            nt += c;
        }
    }
    st->lookups = nt;
    /* the lookups, all on the round-start tables (grouped by R, task order kept); every lookup's
     * FindNodeCalls (destination, arrival) and accepted responses (responder, arrival) */
    const int ccap = kad_call_cap(net);
    uint32_t* resp = (uint32_t*)malloc(sizeof(uint32_t) * nt * (size_t)hcm);
    int64_t* tarr = (int64_t*)malloc(sizeof(int64_t) * nt * (size_t)hcm);
    uint32_t* cnode = (uint32_t*)malloc(sizeof(uint32_t) * nt * (size_t)ccap);
    int64_t* ctime = (int64_t*)malloc(sizeof(int64_t) * nt * (size_t)ccap);
    uint32_t* rpcs = (uint32_t*)malloc(sizeof(uint32_t) * (nt ? nt : 1));
    orc_lookup_out* out = (orc_lookup_out*)malloc(sizeof(orc_lookup_out) * (nt ? nt : 1));
    for (int g = 0; g < 2; ++g) {
        const int R = g == 0 ? Rs : Rb;
        uint64_t cnt = 0;
        for (uint64_t t = 0; t < nt; ++t) cnt += tR[t] == R && (g == 0 || Rs != Rb);
        if (cnt == 0) continue;
        uint64_t* ix = (uint64_t*)malloc(sizeof(uint64_t) * cnt);
        orc_key* gk = (orc_key*)malloc(sizeof(orc_key) * cnt);
        uint32_t* gs = (uint32_t*)malloc(sizeof(uint32_t) * cnt);
        uint64_t c = 0;
        for (uint64_t t = 0; t < nt; ++t)
            if (tR[t] == R && (g == 0 || Rs != Rb)) { ix[c] = t; gk[c] = keys[t]; gs[c] = src[t]; ++c; }
        uint32_t* gsib = (uint32_t*)malloc(sizeof(uint32_t) * cnt * (size_t)R);
        uint32_t* gresp = (uint32_t*)malloc(sizeof(uint32_t) * cnt * (size_t)hcm);
        int64_t* gta = (int64_t*)malloc(sizeof(int64_t) * cnt * (size_t)hcm);
        uint32_t* gcn = (uint32_t*)malloc(sizeof(uint32_t) * cnt * (size_t)ccap);
        int64_t* gct = (int64_t*)malloc(sizeof(int64_t) * cnt * (size_t)ccap);
        uint32_t* grp = (uint32_t*)malloc(sizeof(uint32_t) * cnt);
        orc_lookup_out* go = (orc_lookup_out*)malloc(sizeof(orc_lookup_out) * cnt);
        const int rr = orc_kad_exhaustive_batch_t(net, gk, gs, cnt, R, go, gsib, gresp, NULL, gta, gcn, gct, ccap, grp,
                                                  nthreads);
        for (uint64_t q = 0; q < cnt; ++q) {
            const uint64_t t = ix[q];
            memcpy(resp + t * hcm, gresp + q * hcm, sizeof(uint32_t) * (size_t)hcm);
            memcpy(tarr + t * hcm, gta + q * hcm, sizeof(int64_t) * (size_t)hcm);
            memcpy(cnode + t * ccap, gcn + q * ccap, sizeof(uint32_t) * (size_t)ccap);
            memcpy(ctime + t * ccap, gct + q * ccap, sizeof(int64_t) * (size_t)ccap);
            rpcs[t] = grp[q]; out[t] = go[q];
        }
        free(ix); free(gk); free(gs); free(gsib); free(gresp); free(gta); free(gcn); free(gct); free(grp); free(go);
        if (rr < 0) { free(keys); free(src); free(tR); free(resp); free(tarr); free(cnode); free(ctime); free(rpcs); free(out); return ORC_FAIL; }
    }
    /* the responses' contents: findNode(key, R, -1) at each responder on the round-start tables
     * (BaseOverlay::findNodeRpc, BaseOverlay.cc:1841-1915); CSR over (task, responder) */
    uint64_t* roff = (uint64_t*)malloc(sizeof(uint64_t) * (nt * (size_t)hcm + 1));
    uint64_t tot = 0;
    for (uint64_t t = 0; t < nt; ++t) {
        int nr = 0;
        for (int i = 0; i < hcm && resp[t * hcm + i] != NONE; ++i) ++nr;
        if (out[t].status != 0) st->failed++;
        st->responses += (uint64_t)nr;
        for (int i = 0; i < hcm; ++i) { roff[t * hcm + i] = tot; tot += resp[t * hcm + i] != NONE ? (uint64_t)tR[t] : 0; }
    }
    roff[nt * hcm] = tot;
    uint32_t* rnodes = (uint32_t*)malloc(sizeof(uint32_t) * (tot ? tot : 1));
    uint8_t* rcnt = (uint8_t*)calloc(nt * (size_t)hcm + 1, 1);
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 64) num_threads(nthreads > 0 ? nthreads : omp_get_max_threads())
#endif
    for (int64_t t = 0; t < (int64_t)nt; ++t) {
        OKey k = ok_from(&keys[t]);
        for (int i = 0; i < hcm && resp[t * hcm + i] != NONE; ++i) {
            NVec res;
            kad_findNode(net, resp[t * hcm + i], &k, tR[t], -1, &res);
            rcnt[t * hcm + i] = (uint8_t)res.size;
            for (int q = 0; q < res.size; ++q) rnodes[roff[t * hcm + i] + q] = res.v[q];
        }
    }
    /* the routingAdd events per node: every FindNodeCall reaching its destination x adds its
     * source there (Kademlia::handleRpcCall, 1328-1349: routingAdd(src, true)) -- also the calls
     * whose response the lookup never handled (IterativeLookup::stop cancels only the RPC state,
     * 256-261); every FindNodeResponse the lookup handled adds, at the source, the nodes it carries,
     * not alive, then the responder, alive (handleRpcResponse, 1352-1420).  Each node applies its
     * events in simulated-time order -- every refresh lookup of the round starts at its instant 0
     * -- ties by (kind: calls first, task, index). */
    uint64_t* ecnt = (uint64_t*)calloc((size_t)net->n + 1, sizeof(uint64_t));
    for (uint64_t t = 0; t < nt; ++t) {
        for (int i = 0; i < ccap && cnode[t * ccap + i] != NONE; ++i) ecnt[cnode[t * ccap + i]]++;
        for (int i = 0; i < hcm && resp[t * hcm + i] != NONE; ++i) ecnt[src[t]]++;
    }
    uint64_t* eoff = (uint64_t*)malloc(sizeof(uint64_t) * ((size_t)net->n + 1));
    uint64_t acc = 0;
    for (uint32_t v = 0; v < net->n; ++v) { eoff[v] = acc; acc += ecnt[v]; ecnt[v] = 0; }
    eoff[net->n] = acc;
    KEvt* ev = (KEvt*)malloc(sizeof(KEvt) * (acc ? acc : 1));
    for (uint64_t t = 0; t < nt; ++t) {
        for (int i = 0; i < ccap && cnode[t * ccap + i] != NONE; ++i) {
            const uint32_t x = cnode[t * ccap + i];
            KEvt a = {ctime[t * ccap + i], 0, (uint32_t)t, (uint32_t)i};
            ev[eoff[x] + ecnt[x]++] = a;
        }
        for (int i = 0; i < hcm && resp[t * hcm + i] != NONE; ++i) {
            const uint32_t v = src[t];
            KEvt b = {tarr[t * hcm + i], 1, (uint32_t)t, (uint32_t)i};
            ev[eoff[v] + ecnt[v]++] = b;
        }
    }
    for (uint32_t v = 0; v < net->n; ++v) {
        KEvt* e = ev + eoff[v];
        const uint64_t ne = eoff[v + 1] - eoff[v];
        qsort(e, ne, sizeof(KEvt), kevt_cmp);
        for (uint64_t q = 0; q < ne; ++q) {
            const uint64_t t = e[q].task, i = e[q].idx;
            if (e[q].kind == 0) {
                kad_routingAdd(net, v, src[t], 1, st);
            } else {
                const uint64_t ri = t * hcm + i;
                for (int c = 0; c < rcnt[ri]; ++c) kad_routingAdd(net, v, rnodes[roff[ri] + c], 0, st);
                kad_routingAdd(net, v, resp[ri], 1, st);
            }
        }
    }
    free(keys); free(src); free(tR); free(resp); free(tarr); free(cnode); free(ctime); free(rpcs); free(out);
    free(roff); free(rnodes); free(rcnt); free(ecnt); free(eoff); free(ev);
    if (g_cap_fail) return ORC_FAIL;
    return st->sib_changes + st->bucket_changes + st->lost;
}

/* explicit tables in CSR form (buckets of any size): siblings[n*5s]; bucket_off[n*160+1];
 * bucket_nodes[bucket_off[n*160]] in LRU order.  orc_kad_export_csr with bucket_nodes = NULL
 * only fills bucket_off (the size query). */
void orc_kad_export_csr(const orc_net* net, uint32_t* siblings, uint64_t* bucket_off, uint32_t* bucket_nodes)
{
    const size_t sc = (size_t)5 * net->p.s;
    uint64_t o = 0;
    for (uint32_t v = 0; v < net->n; ++v) {
        KadTab T = kad_tab(net, v);
        if (siblings) for (size_t i = 0; i < sc; ++i) siblings[(size_t)v * sc + i] = (int)i < T.nsib ? T.sib[i] : NONE;
        for (int mm = 0; mm < net->nb; ++mm) {
            bucket_off[(size_t)v * (size_t)net->nb + mm] = o;
            const int c = kt_count(&T, mm);
            const uint32_t* bk = kt_members(&T, mm);
            if (bucket_nodes) for (int j = 0; j < c; ++j) bucket_nodes[o + j] = bk[j];
            o += (uint64_t)c;
        }
    }
    bucket_off[(size_t)net->n * (size_t)net->nb] = o;
}

/* ======================================================================== */
/* One synchronous stabilize round (Chord::handleStabilizeTimerExpired,      */
/* Chord.cc:793-842; rpcStabilize / handleRpcStabilizeResponse 1055-1104;   */
/* rpcNotify / handleRpcNotifyResponse 1106-1225; mergeOptimizationL1-L4 off, */
/* no failed nodes).  Every message sees the tables of the round's start.    */
/* ======================================================================== */
/* ChordSuccessorList (ChordSuccessorList.cc): a map keyed by succ - (self + 1), newEntry flags */
typedef struct { OKey key[64]; uint32_t node[64]; int fresh[64]; int size; } SuccMap;

static void sm_add(const orc_net* net, SuccMap* m, uint32_t self, uint32_t x, int resize, int sls)  /* 122-151 */
{
    OKey one = ok_small(1);
    OKey base = ok_add(net->ids[self], &one);
    OKey k = ok_sub(net->ids[x], &base);
    int i;
    for (i = 0; i < m->size; ++i)
        if (EQ(&m->key[i], &k)) {                       /* successorMap.erase(it) */
            memmove(&m->key[i], &m->key[i + 1], sizeof(OKey) * (size_t)(m->size - i - 1));
            memmove(&m->node[i], &m->node[i + 1], sizeof(uint32_t) * (size_t)(m->size - i - 1));
            memmove(&m->fresh[i], &m->fresh[i + 1], sizeof(int) * (size_t)(m->size - i - 1));
            m->size--;
            break;
        }
    for (i = 0; i < m->size && ok_cmp(&m->key[i], &k) < 0; ++i) {}
    if (m->size == 64) { cap_error("successor map over 64 entries"); return; }
    memmove(&m->key[i + 1], &m->key[i], sizeof(OKey) * (size_t)(m->size - i));
    memmove(&m->node[i + 1], &m->node[i], sizeof(uint32_t) * (size_t)(m->size - i));
    memmove(&m->fresh[i + 1], &m->fresh[i], sizeof(int) * (size_t)(m->size - i));
    m->key[i] = k; m->node[i] = x; m->fresh[i] = 1; m->size++;
    if (resize && m->size > sls) m->size--;             /* erase the last (farthest) entry */
}

static void sm_removeOld(const orc_net* net, SuccMap* m, uint32_t self, int sls)                 /* 170-194 */
{
    int w = 0;
    for (int i = 0; i < m->size; ++i) {
        if (!m->fresh[i]) continue;
        m->key[w] = m->key[i]; m->node[w] = m->node[i]; m->fresh[w] = 0; ++w;
    }
    m->size = w;
    if (m->size > sls) m->size = sls;
    if (m->size == 0) sm_add(net, m, self, self, 1, sls);
}

uint64_t orc_chord_stabilize(orc_net* net, const uint32_t* nodes, uint64_t m, uint64_t* out_succ_changed,
                             uint64_t* out_pred_changed)
{
    if (net->type != NET_CHORD || net->lazy || !net->pred) { set_err("stabilize: explicit Chord tables"); return ORC_FAIL; }
    if (net->p.extendedFingerTable) { set_err("stabilize: extendedFingerTable rounds not restated"); return ORC_FAIL; }
    const uint32_t n = net->n, sls = net->sls;
    uint32_t* pred0 = (uint32_t*)malloc(sizeof(uint32_t) * n);
    uint32_t* succ0 = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n * sls);
    uint8_t* nsucc0 = (uint8_t*)malloc(n);
    memcpy(pred0, net->pred, sizeof(uint32_t) * n);
    memcpy(succ0, net->succ, sizeof(uint32_t) * (size_t)n * sls);
    memcpy(nsucc0, net->nsucc, n);
    uint32_t* tgt = (uint32_t*)malloc(sizeof(uint32_t) * (m ? m : 1));
    uint64_t lists = 0, sch = 0, pch = 0;
    for (uint64_t j = 0; j < m; ++j) {
        const uint32_t v = nodes[j];
        SuccMap L; L.size = 0;
        for (int q = 0; q < nsucc0[v]; ++q) {           /* the list as it stands: entries settled */
            sm_add(net, &L, v, succ0[(size_t)v * sls + q], 0, (int)sls);
            L.fresh[L.size - 1] = 0;
        }
        for (int q = 0; q < L.size; ++q) L.fresh[q] = 0;
        /* handleRpcStabilizeResponse: the successor's predecessor */
        const uint32_t s = L.node[0];
        const uint32_t p = pred0[s];
        if (p != NONE && ok_isBetween(&net->ids[p], &net->ids[v], &net->ids[s]))
            sm_add(net, &L, v, p, 1, (int)sls);
        /* NotifyCall to successorList->getSuccessor(); its response carries t's list (sucNum) */
        const uint32_t t = L.node[0];
        tgt[j] = t;
        /* handleRpcNotifyResponse -> updateList (101-119) */
        sm_add(net, &L, v, t, 0, (int)sls);
        for (uint32_t k = 0; k < nsucc0[t] && k < sls - 1; ++k) {
            const uint32_t x = succ0[(size_t)t * sls + k];
            if (ok_isBetweenLR(&net->ids[x], &net->ids[v], &net->ids[t])) continue;
            sm_add(net, &L, v, x, 0, (int)sls);
        }
        sm_removeOld(net, &L, v, (int)sls);
        int same = L.size == nsucc0[v];
        for (int q = 0; same && q < L.size; ++q) same = L.node[q] == succ0[(size_t)v * sls + q];
        lists += !same;
        sch += L.node[0] != succ0[(size_t)v * sls];
        for (uint32_t q = 0; q < sls; ++q) net->succ[(size_t)v * sls + q] = (int)q < L.size ? L.node[q] : NONE;
        net->nsucc[v] = (uint8_t)L.size;
    }
    /* rpcNotify (1106-1161), one call after the other in the listed order */
    for (uint64_t j = 0; j < m; ++j) {
        const uint32_t t = tgt[j], v = nodes[j];
        const uint32_t cur = net->pred[t];
        if (cur == NONE || ok_isBetween(&net->ids[v], &net->ids[cur], &net->ids[t])) {
            if (cur == NONE || v != cur) net->pred[t] = v;
        }
    }
    for (uint32_t t = 0; t < n; ++t) pch += net->pred[t] != pred0[t];
    free(pred0); free(succ0); free(nsucc0); free(tgt);
    if (out_succ_changed) *out_succ_changed = sch;
    if (out_pred_changed) *out_pred_changed = pch;
    return g_cap_fail ? ORC_FAIL : lists;
}

void orc_chord_export_lists(const orc_net* net, uint32_t* pred, uint32_t* succ, uint8_t* nsucc)
{
    memcpy(pred, net->pred, sizeof(uint32_t) * net->n);
    memcpy(succ, net->succ, sizeof(uint32_t) * (size_t)net->n * net->sls);
    memcpy(nsucc, net->nsucc, net->n);
}

/* ======================================================================== */
/* One synchronous fixfingers round (Chord::handleFixFingersTimerExpired,   */
/* Chord.cc:845-875; rpcFixfingers / handleRpcFixfingersResponse,           */
/* Chord.cc:1228-1270, extendedFingerTable = false) for a list of nodes:     */
/*  1. at every listed node, trivial fingers (2^i <= succ0 - n) are removed   */
/*     in the order i = 0..159 (they all precede the non-trivial ones);      */
/*  2. the lookups of n + 2^i from n (iterative, numSiblings = 1) route over */
/*     the tables as they are then;                                          */
/*  3. every successful lookup sets finger i to its result (the node that    */
/*     answers the FixfingersCall).                                          */
/* The reference runs the timers of different nodes at different times; the */
/* round fixes all listed nodes at one instant of a frozen snapshot.         */
/* ======================================================================== */
uint64_t orc_chord_fix_fingers(orc_net* net, const uint32_t* nodes, uint64_t m, uint64_t* out_ok,
                               uint64_t* out_changed, int nthreads)
{
    if (net->type != NET_CHORD) { set_err("fix_fingers: not a Chord network"); return 0; }
    if (net->p.extendedFingerTable) { set_err("fix_fingers: extendedFingerTable rounds not restated"); return 0; }
    chord_materialize(net);
    uint64_t cap = m * 160, nl = 0;
    orc_key* keys = (orc_key*)malloc(sizeof(orc_key) * (cap ? cap : 1));
    uint32_t* src = (uint32_t*)malloc(sizeof(uint32_t) * (cap ? cap : 1));
    uint16_t* pos = (uint16_t*)malloc(sizeof(uint16_t) * (cap ? cap : 1));
    for (uint64_t j = 0; j < m; ++j) {
        const uint32_t v = nodes[j];
        const OKey* self = &net->ids[v];
        OKey gap = ok_sub(net->ids[succ_get(net, v, 0)], self);
        for (uint32_t i = 0; i < 160; ++i) {
            OKey off = ok_pow2(i);
            if (ok_cmp(&off, &gap) > 0) {
                OKey lk = ok_add(*self, &off);
                ok_to(&lk, &keys[nl]);
                src[nl] = v;
                pos[nl] = (uint16_t)i;
                ++nl;
            } else {
                ft_removeFinger(net, v, i);
            }
        }
    }
    orc_route_out* out = (orc_route_out*)malloc(sizeof(orc_route_out) * (nl ? nl : 1));
    uint64_t hops = orc_route_batch(net, keys, src, nl, out, NULL, NULL, nthreads);
    uint64_t ok = 0, changed = 0;
    for (uint64_t q = 0; q < nl; ++q) {
        if (out[q].status != 0) continue;
        ++ok;
        const uint32_t v = src[q], i = pos[q];
        const uint32_t p = 160 - i - 1;
        const uint32_t before = p < net->fsize[v] ? net->fdeque[(size_t)v * 160 + p] : NONE;
        if (before != out[q].responsible) ++changed;
        ft_setFinger(net, v, i, out[q].responsible);
    }
    free(keys); free(src); free(pos); free(out);
    if (out_ok) *out_ok = ok;
    if (out_changed) *out_changed = changed;
    return hops;
}

/* ======================================================================== */
/* KBRTestApp one-way statistics                                             */
/* ======================================================================== */

typedef struct { uint64_t n; double sum, sqrsum, min, max; } StdDev;   /* OMNeT++ cStdDev */

static void sd_collect(StdDev* s, double v)                 /* cStdDev::collect */
{
    if (s->n == 0 || v < s->min) s->min = v;
    if (s->n == 0 || v > s->max) s->max = v;
    s->n++;
    s->sum += v;
    s->sqrsum += v * v;
}

static void sd_finish(const StdDev* s, orc_stddev* o)       /* getMean / getStddev */
{
    o->count = s->n;
    o->mean = o->stddev = o->min = o->max = 0;
    if (!s->n) return;
    o->mean = s->sum / (double)s->n;
    double var = 0;
    if (s->n > 1) {
        var = (s->sqrsum - s->sum * s->sum / (double)s->n) / (double)(s->n - 1);
        if (var < 0) var = 0;
    }
    o->stddev = sqrt(var);
    o->min = s->min;
    o->max = s->max;
}

void orc_kbrtest_stats(const orc_net* net, const orc_route_out* out, const orc_key* keys, const uint32_t* src,
                       uint64_t n, double T, int lookupNodeIds, int32_t testMsgSize, orc_kbrtest_result* st)
{
    /* per-node KBRTestApp members numSent / numDelivered / numDropped (KBRTestApp.cc:70-80) */
    uint64_t* sent = calloc(net->n, sizeof(uint64_t));
    uint64_t* deliv = calloc(net->n, sizeof(uint64_t));
    uint64_t* drop = calloc(net->n, sizeof(uint64_t));
    memset(st, 0, sizeof *st);
    double hopVec = 0, latVec = 0;     /* GlobalStatistics OutVector value sums */
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t s = src[i];
        if (s < net->n) sent[s]++;                        /* handleTimerEvent: numSent++ (180-181) */
        st->num_sent++;
        if (out[i].status != 0) {                         /* SendToKeyListener: lookup failed (1258-1270) */
            st->num_lookup_failed++;
            continue;
        }
        int match = 1;
        if (lookupNodeIds) {                              /* deliver: thisNode.key == destKey (407) */
            OKey k = ok_from(&keys[i]);
            match = out[i].responsible < net->n && ok_cmp(&net->ids[out[i].responsible], &k) == 0;
        }
        if (!match) {                                     /* deliver: numDropped++ (411-413) */
            st->num_dropped++;
            if (s < net->n) drop[s]++;
            continue;
        }
        st->num_delivered++;                              /* evaluateData (481-482) */
        if (s < net->n) deliv[s]++;
        st->hop_count_sum += out[i].one_way_hops;
        st->latency_sum_ns += out[i].latency_ns;
        hopVec += (double)out[i].one_way_hops;            /* recordOutVector (492-495) */
        latVec += (double)out[i].latency_ns * 1e-9;       /* SIMTIME_DBL(latency) */
    }
    if (st->num_delivered) {                              /* finalizeStatistics (134-139) */
        st->hop_count_mean = hopVec / (double)st->num_delivered;
        st->latency_mean_s = latVec / (double)st->num_delivered;
    }
    StdDev sd[5];
    memset(sd, 0, sizeof sd);
    if (T >= 0.1) {                                       /* finishApp: time >= MIN_MEASURED (502) */
        for (uint32_t c = 0; c < net->n; ++c) {
            sd_collect(&sd[0], (double)deliv[c] / T);
            sd_collect(&sd[1], (double)(deliv[c] * (uint64_t)testMsgSize) / T);
            sd_collect(&sd[2], (double)drop[c] / T);
            sd_collect(&sd[3], (double)(drop[c] * (uint64_t)testMsgSize) / T);
            if (sent[c] > 0) sd_collect(&sd[4], (double)((float)deliv[c] / (float)sent[c]));
        }
    }
    for (int k = 0; k < 5; ++k) sd_finish(&sd[k], &st->sd[k]);
    free(sent); free(deliv); free(drop);
}

/* ======================================================================== */
/* KBRTestApp lookup-test statistics (kbrLookupTest): handleLookupResponse  */
/* (KBRTestApp.cc:331-371) per LookupResponse in batch order, finishApp      */
/* (546-557) per node in node order.                                         */
/* ======================================================================== */
void orc_kbrtest_lookup_stats(const orc_net* net, const orc_lookup_out* out, const uint32_t* siblings, int stride,
                              const orc_key* keys, const uint32_t* src, uint64_t n, double T, int lookupNodeIds,
                              double failureLatency, orc_kbrtest_lookup_result* st)
{
    uint64_t* sent = calloc(net->n, sizeof(uint64_t));
    uint64_t* succ = calloc(net->n, sizeof(uint64_t));
    uint64_t* fail = calloc(net->n, sizeof(uint64_t));
    memset(st, 0, sizeof *st);
    double hopVec = 0, fhopVec = 0, succLatVec = 0, totLatVec = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t s = src[i];
        if (s < net->n) sent[s]++;                                   /* numLookupSent++ (205) */
        st->num_sent++;
        int ok = out[i].is_valid != 0;                               /* msg->getIsValid() (341) */
        if (ok && lookupNodeIds) {                                   /* 341-344 */
            OKey k = ok_from(&keys[i]);
            const uint32_t f = siblings[(size_t)i * stride];
            ok = out[i].num_siblings > 0 && f < net->n && ok_cmp(&net->ids[f], &k) == 0;
        }
        if (ok) {
            st->num_success++;
            if (s < net->n) succ[s]++;
            st->hop_count_sum += out[i].hops;
            st->success_latency_sum_ns += out[i].latency_ns;
            succLatVec += (double)out[i].latency_ns * 1e-9;          /* "Lookup Success Latency" */
            totLatVec += (double)out[i].latency_ns * 1e-9;           /* "Lookup Total Latency" */
            hopVec += (double)out[i].hops;                           /* "Lookup Hop Count" */
        } else {
            st->num_failed++;
            if (!out[i].is_valid) st->num_invalid++;
            if (s < net->n) fail[s]++;
            st->failed_hop_count_sum += out[i].hops;
            totLatVec += failureLatency;                             /* failureLatency (363-366) */
            fhopVec += (double)out[i].hops;                          /* "Failed Lookup Hop Count" */
        }
    }
    if (st->num_success) {
        st->hop_count_mean = hopVec / (double)st->num_success;
        st->success_latency_mean_s = succLatVec / (double)st->num_success;
    }
    if (st->num_failed) st->failed_hop_count_mean = fhopVec / (double)st->num_failed;
    if (n) st->total_latency_mean_s = totLatVec / (double)n;
    StdDev sd[3];
    memset(sd, 0, sizeof sd);
    if (T >= 0.1) {
        for (uint32_t c = 0; c < net->n; ++c) {
            sd_collect(&sd[0], (double)succ[c] / T);                 /* Successful Lookups/s */
            sd_collect(&sd[1], (double)fail[c] / T);                 /* Failed Lookups/s */
            if (sent[c] > 0) sd_collect(&sd[2], (double)((float)succ[c] / (float)sent[c]));
        }
    }
    for (int k = 0; k < 3; ++k) sd_finish(&sd[k], &st->sd[k]);
    free(sent); free(succ); free(fail);
}
