// host_tables_driver.cpp -- drives the host-side table bookkeeping of the C ABI
// (oversim_amd/csrc/host_tables.cpp) under ASan/UBSan (tests/test_sanitizers.py): explicit Chord
// tables through import, fixfingers rounds and stabilize rounds until a ring with late joiners
// converges, the import's error paths, and EpiChord snapshot validation / ordering on valid and
// broken snapshots.  Prints "clean" when every check holds.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "host_tables.hpp"

using namespace ovs;

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint64_t rnd()
{
    uint64_t x = (rng_state += 0x9E3779B97F4A7C15ull);
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

#define CHECK(c)                                                                  \
    do {                                                                          \
        if (!(c)) { std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); std::exit(1); } \
    } while (0)

static std::vector<K160> sorted_keys(uint64_t n)
{
    std::vector<K160> k(n);
    for (uint64_t i = 0; i < n; ++i) {
        // ascending: top word carries i, the rest random
        k[i].w[4] = (uint32_t)(i * (0xFFFFFFFFull / n));
        for (int w = 0; w < 4; ++w) k[i].w[w] = (uint32_t)rnd();
    }
    return k;
}

// responsible node of key x: the first id >= x, wrapping to 0
static uint32_t responsible(const std::vector<K160>& id, const K160& x)
{
    uint64_t lo = 0, hi = id.size();
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (k_lt(id[mid], x)) lo = mid + 1; else hi = mid;
    }
    return (uint32_t)(lo == id.size() ? 0 : lo);
}

static void chord_rounds()
{
    const uint64_t n = 300;
    const int sls = 4;
    const std::vector<K160> id = sorted_keys(n);
    // late joiners: every 7th node is known to nobody (its predecessor skips it)
    std::vector<bool> late(n);
    for (uint64_t v = 0; v < n; ++v) late[v] = v % 7 == 3;
    std::vector<uint32_t> pred(n), succ(n * sls, 0xFFFFFFFFu), fingers(n * 160, 0xFFFFFFFFu);
    std::vector<uint8_t> nsucc(n), dq(n);
    for (uint64_t v = 0; v < n; ++v) {
        int k = 0;
        for (uint64_t j = 1; k < sls && j < n; ++j) {
            const uint64_t x = (v + j) % n;
            if (late[x] && !late[v]) continue;
            succ[v * sls + k++] = (uint32_t)x;
        }
        nsucc[v] = (uint8_t)k;
        uint64_t p = (v + n - 1) % n;
        while (late[p]) p = (p + n - 1) % n;
        pred[v] = (uint32_t)p;
        dq[v] = (uint8_t)(rnd() % 161);
        for (int i = 0; i < 160; ++i)
            if (rnd() % 3) fingers[v * 160 + i] = (uint32_t)(rnd() % n);
    }
    ChordHost h;
    std::string err;
    CHECK(h.import(id.data(), n, pred.data(), succ.data(), nsucc.data(), fingers.data(), dq.data(), sls, &err));
    std::vector<uint32_t> all(n);
    for (uint64_t v = 0; v < n; ++v) all[v] = (uint32_t)v;
    for (int round = 0; round < 40; ++round) {
        uint64_t sc = 0, lc = 0, pc = 0;
        std::vector<uint32_t> changed;
        h.stabilize(all.data(), n, &sc, &lc, &pc, &changed);
        std::vector<K160> keys;
        std::vector<uint32_t> src, resp;
        std::vector<uint8_t> pos, ok;
        h.fix_fingers_plan(all.data(), n, &keys, &src, &pos);
        for (const K160& k : keys) { resp.push_back(responsible(id, k)); ok.push_back(rnd() % 10 != 0); }
        h.fix_fingers_apply(src, pos, resp, ok);
        for (uint64_t v = 0; v < n; ++v) h.resolve_row(v);
        if (sc == 0 && lc == 0 && pc == 0 && round > 2) break;
    }
    // converged: every node's successor list is the next sls nodes, its predecessor the previous one
    for (uint64_t v = 0; v < n; ++v) {
        CHECK(h.pred[v] == (uint32_t)((v + n - 1) % n));
        CHECK(h.nsucc[v] == sls);
        for (int j = 0; j < sls; ++j) CHECK(h.succ[v * sls + j] == (uint32_t)((v + 1 + j) % n));
        for (int pos = 0; pos < 160; ++pos) CHECK(h.fres[v * 160 + pos] < n);
    }
    // import error paths
    std::vector<uint8_t> bad_ns = nsucc;
    bad_ns[5] = 0;
    CHECK(!h.import(id.data(), n, pred.data(), succ.data(), bad_ns.data(), fingers.data(), dq.data(), sls, &err));
    std::vector<uint32_t> bad_f = fingers;
    bad_f[17] = (uint32_t)n;
    CHECK(!h.import(id.data(), n, pred.data(), succ.data(), nsucc.data(), bad_f.data(), dq.data(), sls, &err));
    std::vector<uint8_t> bad_dq = dq;
    bad_dq[9] = 200;
    CHECK(!h.import(id.data(), n, pred.data(), succ.data(), nsucc.data(), fingers.data(), bad_dq.data(), sls, &err));
}

static void epichord_snapshots()
{
    const uint64_t n = 200;
    const int L = 4;
    const std::vector<K160> id = sorted_keys(n);
    for (int trial = 0; trial < 20; ++trial) {
        std::vector<uint32_t> succ(n * L, 0xFFFFFFFFu), pred(n * L, 0xFFFFFFFFu), cnode;
        std::vector<uint8_t> ns(n), np(n), full(n);
        std::vector<uint64_t> off(n + 1, 0);
        std::vector<int64_t> last, ttl;
        for (uint64_t v = 0; v < n; ++v) {
            const int a = (int)(rnd() % (L + 1)), b = (int)(rnd() % (L + 1));
            for (int j = 0; j < a; ++j) succ[v * L + j] = (uint32_t)((v + 1 + j) % n);
            for (int j = 0; j < b; ++j) pred[v * L + j] = (uint32_t)((v + n - 1 - j) % n);
            ns[v] = (uint8_t)a; np[v] = (uint8_t)b;
            full[v] = (uint8_t)((a == L ? 1 : 0) | (b == L ? 2 : 0));
            const int c = (int)(rnd() % 12);
            std::vector<bool> used(n);
            used[v] = true;
            for (int j = 0; j < c; ++j) {
                const uint32_t x = (uint32_t)(rnd() % n);
                if (used[x]) continue;
                used[x] = true;
                cnode.push_back(x); last.push_back((int64_t)(rnd() % 1000000)); ttl.push_back((int64_t)(rnd() % 3) * 1000);
            }
            off[v + 1] = cnode.size();
        }
        std::vector<uint32_t> meta, cn;
        std::vector<int64_t> cl, ct;
        std::string err;
        CHECK(epichord_prepare(id.data(), n, L, succ.data(), ns.data(), pred.data(), np.data(), full.data(), off.data(),
                               cnode.data(), last.data(), ttl.data(), &meta, &cn, &cl, &ct, &err));
        for (uint64_t v = 0; v < n; ++v) {
            const K160 base = k_add(id[v], K160{{1, 0, 0, 0, 0}});
            for (uint64_t i = off[v] + 1; i < off[v + 1]; ++i)
                CHECK(k_lt(k_sub(id[cn[i - 1]], base), k_sub(id[cn[i]], base)));
        }
        // broken snapshots are refused
        if (!cnode.empty()) {
            std::vector<uint32_t> bad = cnode;
            uint64_t v = 0;
            while (off[v + 1] == off[v]) ++v;
            bad[off[v]] = (uint32_t)v;                       // a node in its own cache
            CHECK(!epichord_prepare(id.data(), n, L, succ.data(), ns.data(), pred.data(), np.data(), full.data(),
                                    off.data(), bad.data(), last.data(), ttl.data(), &meta, &cn, &cl, &ct, &err));
        }
        std::vector<uint8_t> badfull = full;
        for (uint64_t v = 0; v < n; ++v)
            if (ns[v] == 0) { badfull[v] |= 1; break; }      // isFull() with an empty list
        CHECK(!epichord_prepare(id.data(), n, L, succ.data(), ns.data(), pred.data(), np.data(), badfull.data(),
                                off.data(), cnode.data(), last.data(), ttl.data(), &meta, &cn, &cl, &ct, &err) ||
              badfull == full);
        std::vector<uint32_t> badsucc = succ;
        for (uint64_t v = 0; v < n; ++v)
            if (ns[v] >= 2) { std::swap(badsucc[v * L], badsucc[v * L + 1]); break; }   // not closest first
        CHECK(!epichord_prepare(id.data(), n, L, badsucc.data(), ns.data(), pred.data(), np.data(), full.data(),
                                off.data(), cnode.data(), last.data(), ttl.data(), &meta, &cn, &cl, &ct, &err) ||
              badsucc == succ);
    }
}

// routingAdd's invariants on every node: siblings XOR-sorted, at most 5s of them; every bucket member
// in its own bucket msb(x ^ v), at most k; no node twice, never v itself
static void kad_check(const KadHost& h)
{
    const uint64_t n = h.n();
    std::vector<uint32_t> seen(n, 0xFFFFFFFFu);
    for (uint64_t v = 0; v < n; ++v) {
        const std::vector<uint32_t>& S = h.sib[v];
        CHECK(S.size() <= 5u * (size_t)h.s);
        for (size_t i = 0; i < S.size(); ++i) {
            CHECK(S[i] < n && S[i] != v && seen[S[i]] != v);
            seen[S[i]] = (uint32_t)v;
            if (i) CHECK(k_lt(k_xor(h.ids[S[i - 1]], h.ids[v]), k_xor(h.ids[S[i]], h.ids[v])));
        }
        for (int m = 0; m < 160; ++m) {
            const std::vector<uint32_t>& B = h.bk[v * 160 + (uint64_t)m];
            CHECK(B.size() <= (size_t)h.k);
            for (uint32_t x : B) {
                CHECK(x < n && x != v && seen[x] != v);
                seen[x] = (uint32_t)v;
                CHECK(k_msb(k_xor(h.ids[x], h.ids[v])) == m);
            }
        }
    }
}

// Kademlia maintenance bookkeeping: routingAdd from empty tables (sibling insertions, preemption
// into buckets, full buckets, LRU moves), the refresh plan, and a round of synthetic events
static void kad_maintenance()
{
    const uint64_t n = 400;
    const int k = 4, s = 2;
    std::vector<K160> id = sorted_keys(n);
    std::vector<uint32_t> sib(n * 5 * s, 0xFFFFFFFFu), bn(n * 160 * k, 0xFFFFFFFFu);
    std::vector<uint8_t> bc(n * 160, 0);
    KadHost h;
    h.import(id.data(), n, k, s, sib.data(), bc.data(), bn.data());
    KadRoundCount st;
    for (int i = 0; i < 40000; ++i) {
        const uint32_t v = (uint32_t)(rnd() % n), x = (uint32_t)(rnd() % n);
        const bool alive = (rnd() & 1) != 0;
        const bool r = h.routing_add(v, x, alive, &st);
        CHECK(r || x == v || h.bk[v * 160 + (uint64_t)k_msb(k_xor(id[x], id[v]))].size() == (size_t)k);
    }
    CHECK(st.sib_changes > 0 && st.bucket_changes > 0 && st.lost + st.replacement > 0 && st.refreshed > 0);
    kad_check(h);
    std::vector<uint32_t> hs(n * 5 * s), hn(n * 160 * k);
    std::vector<uint8_t> hc(n * 160);
    CHECK(h.export_k(hs.data(), hc.data(), hn.data()));
    KadHost h2;
    h2.import(id.data(), n, k, s, hs.data(), hc.data(), hn.data());
    CHECK(h2.sib == h.sib && h2.bk == h.bk);
    // refresh plan: the sibling refresh first, then keys self ^ 2^i down to msb(self ^ front)
    std::vector<uint32_t> nodes = {0, 7, 399};
    std::vector<uint8_t> fl = {3, 1, 2};
    std::vector<uint32_t> stale(3 * 5, 0xFFFFFFFFu);
    stale[2 * 5 + 4] = 0;    // node 399: buckets 128..159 fresh
    std::vector<K160> keys;
    std::vector<uint32_t> src;
    std::vector<int> R;
    h.refresh_plan(nodes.data(), nodes.size(), fl.data(), stale.data(), 10, 4, &keys, &src, &R);
    CHECK(!keys.empty() && src[0] == 0 && R[0] == 10 && k_eq(keys[0], id[0]));
    for (size_t t = 0; t < keys.size(); ++t) {
        const int i = k_msb(k_xor(keys[t], id[src[t]]));
        CHECK(R[t] == 10 ? i < 0 : (i >= k_msb(k_xor(id[h.sib[src[t]][0]], id[src[t]])) && !(src[t] == 399 && i >= 128)));
    }
    // a round of synthetic lookups: calls and responses at random times
    std::vector<KadRoundLookup> lk(300);
    std::vector<std::vector<uint32_t>> cn(lk.size()), rs(lk.size()), car(lk.size() * 8);
    std::vector<std::vector<int64_t>> ct(lk.size()), ta(lk.size());
    std::vector<std::vector<const uint32_t*>> cp(lk.size());
    std::vector<std::vector<uint8_t>> nc(lk.size());
    for (size_t t = 0; t < lk.size(); ++t) {
        const int nr = (int)(rnd() % 8);
        for (int i = 0; i < nr + 2; ++i) { cn[t].push_back((uint32_t)(rnd() % n)); ct[t].push_back((int64_t)(rnd() % 1000)); }
        for (int i = 0; i < nr; ++i) {
            rs[t].push_back(cn[t][i]); ta[t].push_back(ct[t][i] + (int64_t)(rnd() % 1000));
            std::vector<uint32_t>& C = car[t * 8 + i];
            for (int q = 0; q < (int)(rnd() % 6); ++q) C.push_back((uint32_t)(rnd() % n));
        }
        for (int i = 0; i < nr; ++i) { cp[t].push_back(car[t * 8 + i].data()); nc[t].push_back((uint8_t)car[t * 8 + i].size()); }
        KadRoundLookup& L = lk[t];
        L.src = (uint32_t)(rnd() % n);
        L.cnode = cn[t].data(); L.ctime = ct[t].data(); L.ncall = (int)cn[t].size();
        L.resp = rs[t].data(); L.tarr = ta[t].data(); L.nresp = nr;
        L.carried = cp[t].data(); L.ncarried = nc[t].data();
    }
    KadRoundCount st2;
    h.apply_round(lk, &st2);
    CHECK(st2.responses > 0);
    kad_check(h);
}

int main()
{
    chord_rounds();
    epichord_snapshots();
    kad_maintenance();
    std::printf("clean\n");
    return 0;
}
