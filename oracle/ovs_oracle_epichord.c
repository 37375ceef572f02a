/*
 * ovs_oracle_epichord.c -- CPU restatement of EpiChord::findNode over one routing snapshot.
 *
 * TEST INFRASTRUCTURE ONLY (see ovs_oracle.h): the checker of the engine's
 * ovs_epichord_find_node_batch.  Parity unpinned against reference outputs (the reference
 * is unbuildable here and ships no EpiChord fixtures); tests/refmodel.py holds a second,
 * independent reading.
 *
 * One call = one FindNodeCall served by node `self` (EpiChord.cc:517-629) on a copy of its
 * routing state, with every side effect the reference has on the way to its answer:
 *   receiveNewNode(source, direct, OBSERVED, now)       EpiChord.cc:546-553, 1178-1209
 *     EpiChordFingerCache::updateFinger                 EpiChordFingerCache.cc:79-127
 *     EpiChordNodeList::addNode (successor / predecessor lists, resize) EpiChordNodeList.cc:108-161
 *     EpiChordFingerCache::setFingerTTL                 EpiChordFingerCache.cc:129-142
 *   isSiblingFor(thisNode, key, 1)                      EpiChord.cc:650-721
 *   the successor / predecessor entry                   EpiChord.cc:581-606
 *   EpiChordFingerCache::findBestHops                   EpiChordFingerCache.cc:309-356
 *     removeOldFingers                                  EpiChordFingerCache.cc:162-187
 * The std::maps (liveCache keyed by node - (self + 1), the node lists keyed by their ring
 * offset - 1) are sorted arrays here, walked with the reference's iterator moves.  The dead
 * cache is not an input: a FindNodeCall's source is heard from directly, which takes it out of
 * the dead cache before anything reads it (EpiChordFingerCache.cc:87-96), and nothing else on
 * this path looks at it.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "ovs_oracle.h"

#define EC_NONE 0xFFFFFFFFu
#define EC_MAXL 64

typedef struct {
    orc_key sum;           /* map key: node - (self + 1) */
    uint32_t node;
    int64_t added, last, ttl;
} ec_entry;

typedef struct {
    ec_entry* e;
    int n, cap;
} ec_cache;

typedef struct {
    orc_key sum;           /* map key: ring offset from self (backwards for the predecessor list) - 1 */
    uint32_t node;
} ec_lent;

typedef struct {
    ec_lent e[EC_MAXL + 2];
    int n;                 /* nodeMap.size(), thisNode included when present */
    int size;              /* nodeListSize */
    int forwards;
} ec_list;

typedef struct {
    const orc_key* ids;
    uint32_t self;
    int64_t now, cacheTTL;
    ec_cache cache;
    ec_list succ, pred;
} ec_state;

static const orc_key ONE = {{1, 0, 0, 0, 0}};
static const orc_key ZERO = {{0, 0, 0, 0, 0}};

static orc_key sub(const orc_key* a, const orc_key* b)
{
    orc_key r;
    orc_key_sub(a, b, &r);
    return r;
}

static orc_key add(const orc_key* a, const orc_key* b)
{
    orc_key r;
    orc_key_add(a, b, &r);
    return r;
}

/* node.getKey() - (thisNode.getKey() + OverlayKey::ONE) */
static orc_key cache_sum(const ec_state* s, uint32_t node)
{
    const orc_key base = add(&s->ids[s->self], &ONE);
    return sub(&s->ids[node], &base);
}

/* liveCache.lower_bound(k) as an index (n = end()) */
static int cache_lower_bound(const ec_cache* c, const orc_key* k)
{
    int lo = 0, hi = c->n;
    while (lo < hi) {
        const int mid = (lo + hi) / 2;
        if (orc_key_cmp(&c->e[mid].sum, k) < 0) lo = mid + 1; else hi = mid;
    }
    return lo;
}

static ec_entry* cache_find(ec_state* s, uint32_t node)
{
    const orc_key k = cache_sum(s, node);
    const int i = cache_lower_bound(&s->cache, &k);
    if (i < s->cache.n && orc_key_cmp(&s->cache.e[i].sum, &k) == 0) return &s->cache.e[i];
    return NULL;
}

/* EpiChordFingerCache::updateFinger (EpiChordFingerCache.cc:79-127); dead cache: see header */
static void update_finger(ec_state* s, uint32_t node, int64_t lastUpdate, int64_t ttl)
{
    if (node == EC_NONE || node == s->self) return;
    const orc_key k = cache_sum(s, node);
    ec_cache* c = &s->cache;
    const int i = cache_lower_bound(c, &k);
    if (i < c->n && orc_key_cmp(&c->e[i].sum, &k) == 0) {
        ec_entry* e = &c->e[i];
        if (lastUpdate < e->added) e->added = lastUpdate;
        if (lastUpdate > e->last) e->last = lastUpdate;
        if (e->ttl > 0 && (ttl > e->ttl || ttl == 0)) e->ttl = ttl;
        return;
    }
    if (c->n == c->cap) {
        c->cap = c->cap ? 2 * c->cap : 8;
        c->e = (ec_entry*)realloc(c->e, (size_t)c->cap * sizeof(ec_entry));
    }
    memmove(&c->e[i + 1], &c->e[i], (size_t)(c->n - i) * sizeof(ec_entry));
    c->e[i].sum = k;
    c->e[i].node = node;
    c->e[i].added = lastUpdate;
    c->e[i].last = lastUpdate;
    c->e[i].ttl = ttl;
    c->n++;
}

/* EpiChordFingerCache::setFingerTTL (129-142) */
static void set_finger_ttl(ec_state* s, uint32_t node, int64_t ttl)
{
    if (node == EC_NONE) return;
    ec_entry* e = cache_find(s, node);
    if (e) e->ttl = ttl;
}

static orc_key list_sum(const ec_state* s, const ec_list* L, uint32_t node)
{
    orc_key sum = sub(&s->ids[node], &s->ids[s->self]);
    if (!L->forwards) sum = sub(&ZERO, &sum);
    return sub(&sum, &ONE);
}

static int list_contains(const ec_list* L, uint32_t node)
{
    for (int i = 0; i < L->n; ++i)
        if (L->e[i].node == node) return 1;
    return 0;
}

/* isFull: the last entry is not thisNode (EpiChordNodeList.cc:78-87) */
static int list_full(const ec_state* s, const ec_list* L)
{
    return L->n > 0 && L->e[L->n - 1].node != s->self;
}

/* EpiChordNodeList::addNode(node, resize = true) (108-161); callUpdate / additions are bookkeeping */
static void list_add(ec_state* s, ec_list* L, uint32_t node)
{
    if (node == EC_NONE) return;
    const orc_key k = list_sum(s, L, node);
    int i = 0;
    while (i < L->n && orc_key_cmp(&L->e[i].sum, &k) < 0) ++i;
    if (!(i < L->n && orc_key_cmp(&L->e[i].sum, &k) == 0)) {
        memmove(&L->e[i + 1], &L->e[i], (size_t)(L->n - i) * sizeof(ec_lent));
        L->e[i].sum = k;
        L->e[i].node = node;
        L->n++;
    }
    if (node != s->self) update_finger(s, node, s->now, 0);
    if (L->n > L->size) {
        set_finger_ttl(s, L->e[L->n - 1].node, s->cacheTTL);
        L->n--;
    }
}

/* EpiChord::receiveNewNode(node, direct = true, ..., now) (1178-1209) */
static void receive_new_node(ec_state* s, uint32_t node)
{
    if (node == EC_NONE) return;
    update_finger(s, node, s->now, s->cacheTTL);
    ec_list* S = &s->succ;
    if (!list_contains(S, node) &&
        (!list_full(s, S) ||
         orc_key_between(0, &s->ids[node], &s->ids[s->self], &s->ids[S->e[S->n - 1].node], 0)))
        list_add(s, S, node);
    ec_list* P = &s->pred;
    if (!list_contains(P, node) &&
        (!list_full(s, P) ||
         orc_key_between(0, &s->ids[node], &s->ids[P->e[P->n - 1].node], &s->ids[s->self], 0)))
        list_add(s, P, node);
}

static uint32_t list_first(const ec_state* s, const ec_list* L) { return L->n ? L->e[0].node : s->self; }
static int list_empty(const ec_state* s, const ec_list* L) { return L->n == 1 && L->e[0].node == s->self; }

static int excluded(const uint32_t* ex, int nex, uint32_t node)
{
    for (int i = 0; i < nex; ++i)
        if (ex[i] == node) return 1;
    return 0;
}

/* KeyRingMetric::distance (Comparator.h:121-131) */
static orc_key ring_distance(const orc_key* x, const orc_key* y)
{
    const orc_key d1 = sub(x, y), d2 = sub(y, x);
    return orc_key_cmp(&d1, &d2) > 0 ? d2 : d1;
}

int orc_epichord_find_node(const orc_key* ids, uint32_t n, uint32_t self, const uint32_t* succ, int nsucc,
                           const uint32_t* pred, int npred, int lists_full, int listSize, const uint32_t* cnode,
                           const int64_t* clast, const int64_t* cttl, int ncache, const orc_key* key, uint32_t src,
                           int64_t now, int64_t cacheTTL, int numRedundantNodes, uint32_t* out, int64_t* out_last,
                           int cap)
{
    if (self >= n || listSize < 1 || listSize > EC_MAXL || nsucc < 0 || npred < 0 || nsucc > listSize ||
        npred > listSize || (src != EC_NONE && src >= n))
        return -3;
    ec_state s;
    memset(&s, 0, sizeof s);
    s.ids = ids;
    s.self = self;
    s.now = now;
    s.cacheTTL = cacheTTL;
    /* the lists as nodeMaps: the given entries (closest first), thisNode last unless isFull() */
    ec_list* Ls[2] = {&s.succ, &s.pred};
    const uint32_t* in[2] = {succ, pred};
    const int cnt[2] = {nsucc, npred};
    for (int l = 0; l < 2; ++l) {
        ec_list* L = Ls[l];
        L->size = listSize;
        L->forwards = l == 0;
        for (int i = 0; i < cnt[l]; ++i) {
            if (in[l][i] >= n || in[l][i] == self) return -3;
            L->e[L->n].node = in[l][i];
            L->e[L->n].sum = list_sum(&s, L, in[l][i]);
            if (L->n && orc_key_cmp(&L->e[L->n - 1].sum, &L->e[L->n].sum) >= 0) return -3;   /* not closest first */
            L->n++;
        }
        if (!((lists_full >> l) & 1)) {
            if (cnt[l] >= listSize) return -3;
            L->e[L->n].node = self;
            L->e[L->n].sum = list_sum(&s, L, self);
            L->n++;
        } else if (cnt[l] == 0) {
            return -3;
        }
    }
    for (int i = 0; i < ncache; ++i) {
        if (cnode[i] >= n || cnode[i] == self || cache_find(&s, cnode[i])) { free(s.cache.e); return -3; }
        update_finger(&s, cnode[i], clast[i], cttl[i]);
        ec_entry* e = cache_find(&s, cnode[i]);
        e->added = clast[i];
    }

    uint32_t ex[4];
    int nex = 0;
    ex[nex++] = self;
    if (src != EC_NONE) {
        ex[nex++] = src;
        receive_new_node(&s, src);
    }
    int cnt_out = 0;
#define PUSH(x, t) do { if (cnt_out >= cap) { free(s.cache.e); return -4; } out[cnt_out] = (x); out_last[cnt_out] = (t); ++cnt_out; } while (0)
    /* isSiblingFor(thisNode, key, 1, &err) (650-721): err is ignored by findNode */
    int sib;
    if (list_empty(&s, &s.pred))
        sib = list_empty(&s, &s.succ) || orc_key_cmp(key, &ids[self]) == 0;
    else
        sib = orc_key_between(1, key, &ids[list_first(&s, &s.pred)], &ids[self], 0);
    if (sib) {
        PUSH(self, now);
        if (!list_empty(&s, &s.pred)) {
            const uint32_t p = list_first(&s, &s.pred);
            const ec_entry* e = cache_find(&s, p);
            PUSH(p, e ? e->last : now);
        }
        if (!list_empty(&s, &s.succ)) {
            const uint32_t q = list_first(&s, &s.succ);
            const ec_entry* e = cache_find(&s, q);
            PUSH(q, e ? e->last : now);
        }
    } else {
        uint32_t choice;
        if (src == EC_NONE) {
            const orc_key sd = ring_distance(&ids[list_first(&s, &s.succ)], key);
            const orc_key pd = ring_distance(&ids[list_first(&s, &s.pred)], key);
            choice = orc_key_cmp(&pd, &sd) < 0 ? list_first(&s, &s.pred) : list_first(&s, &s.succ);
        } else if (orc_key_between(0, &ids[self], &ids[src], key, 0)) {
            choice = list_first(&s, &s.succ);
        } else {
            choice = list_first(&s, &s.pred);
        }
        const ec_entry* e = cache_find(&s, choice);
        if (e) {
            PUSH(e->node, e->last);
            ex[nex++] = e->node;
        }
        /* findBestHops (309-356) */
        const orc_key base = add(&ids[self], &ONE);
        const orc_key k = sub(key, &base);
        ec_cache* c = &s.cache;
        int w = 0;      /* removeOldFingers (162-187) */
        for (int i = 0; i < c->n; ++i)
            if (!(c->e[i].ttl > 0 && c->e[i].last + c->e[i].ttl < now)) c->e[w++] = c->e[i];
        c->n = w;
        if (c->n == 0) {
            /* liveCache.begin() == end() is dereferenced: undefined in the reference */
            free(s.cache.e);
            return -2;
        }
        int it = cache_lower_bound(c, &k);
        if (it == c->n) it = 0;
        int first = it;
        int done = 0;
        while (excluded(ex, nex, c->e[it].node)) {
            ++it;
            if (it == c->n) it = 0;
            if (it == first) { done = 1; break; }
        }
        if (!done) {
            first = it;
            for (int i = 0; i < numRedundantNodes;) {
                if (!excluded(ex, nex, c->e[it].node)) {
                    PUSH(c->e[it].node, c->e[it].last);
                    ++i;
                }
                if (it == 0) it = c->n;
                --it;
                if (it == first) break;
            }
        }
    }
#undef PUSH
    free(s.cache.e);
    return cnt_out ? cnt_out : -1;   /* -1: "EpiChord::findNode() Failed to find node" (613-614) */
}
