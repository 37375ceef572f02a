// host_tables.cpp -- host-side table bookkeeping of the C ABI (see host_tables.hpp).  Plain C++:
// compiled into libovs_kbr.so by hipcc and, for the sanitizer test, by g++ alone.
#include "host_tables.hpp"

#include <algorithm>

namespace ovs {

void ChordHost::clear()
{
    ids.clear(); deque.clear(); fsize.clear(); succ0.clear(); fres.clear();
    pred.clear(); succ.clear(); nsucc.clear();
    sls = 0;
}

bool ChordHost::import(const K160* keys, uint64_t n, const uint32_t* pred_in, const uint32_t* succ_in,
                       const uint8_t* nsucc_in, const uint32_t* fingers, const uint8_t* deque_size, int sls_in,
                       std::string* err)
{
    clear();
    sls = sls_in;
    ids.assign(keys, keys + n);
    deque.resize((size_t)n * 160);
    fsize.assign(deque_size, deque_size + n);
    succ0.resize(n);
    fres.resize((size_t)n * 160);
    for (uint64_t v = 0; v < n; ++v) {
        if (nsucc_in[v] == 0) { *err = "empty successor list"; return false; }
        if (deque_size[v] > 160) { *err = "deque_size > 160"; return false; }
        if (nsucc_in[v] > sls) { *err = "nsucc > successorListSize"; return false; }
        for (uint32_t p = 0; p < 160; ++p) {
            const uint32_t f = fingers[v * 160 + (159 - p)];
            if (f != 0xFFFFFFFFu && f >= n) { *err = "finger index out of range"; return false; }
            deque[v * 160 + p] = f;
        }
        if (pred_in[v] != 0xFFFFFFFFu && pred_in[v] >= n) { *err = "pred index out of range"; return false; }
        for (int j = 0; j < nsucc_in[v]; ++j)
            if (succ_in[v * sls + j] >= n) { *err = "successor index out of range"; return false; }
        succ0[v] = succ_in[v * sls];
        resolve_row(v);
    }
    pred.assign(pred_in, pred_in + n);
    succ.assign(succ_in, succ_in + n * sls);
    nsucc.assign(nsucc_in, nsucc_in + n);
    return true;
}

void ChordHost::resolve_row(uint64_t v)
{
    const uint32_t* dq = deque.data() + v * 160;
    const uint32_t size = fsize[v];
    for (int pos = 0; pos < 160; ++pos) {
        uint32_t p = 160 - pos - 1;
        uint32_t r;
        if (p >= size) r = succ0[v];
        else {
            while (dq[p] == 0xFFFFFFFFu && p < size - 1) ++p;
            r = dq[p] == 0xFFFFFFFFu ? succ0[v] : dq[p];
        }
        fres[v * 160 + pos] = r;
    }
}

void ChordHost::fix_fingers_plan(const uint32_t* nodes, uint64_t m, std::vector<K160>* keys,
                                 std::vector<uint32_t>* src, std::vector<uint8_t>* pos)
{
    for (uint64_t j = 0; j < m; ++j) {
        const uint32_t v = nodes[j];
        const K160 self = ids[v];
        const K160 gap = k_sub(ids[succ0[v]], self);
        for (int i = 0; i < 160; ++i) {
            const K160 off = k_pow2(i);
            if (k_lt(gap, off)) {                              // offset > successor - thisNode
                keys->push_back(k_add(self, off));
                src->push_back(v);
                pos->push_back((uint8_t)i);
            } else {                                           // ChordFingerTable::removeFinger (154-172)
                const uint32_t p = 160 - i - 1;
                uint8_t& size = fsize[v];
                if (p >= size) continue;
                if (p == (uint32_t)size - 1) --size;
                else deque[(uint64_t)v * 160 + p] = 0xFFFFFFFFu;
            }
        }
    }
    for (uint64_t j = 0; j < m; ++j) resolve_row(nodes[j]);
}

uint64_t ChordHost::fix_fingers_apply(const std::vector<uint32_t>& src, const std::vector<uint8_t>& pos,
                                      const std::vector<uint32_t>& responsible, const std::vector<uint8_t>& ok)
{
    uint64_t changed = 0;
    for (size_t q = 0; q < src.size(); ++q) {
        if (!ok[q]) continue;
        const uint32_t v = src[q], p = 160 - pos[q] - 1;
        uint32_t* dq = deque.data() + (uint64_t)v * 160;
        uint8_t& size = fsize[v];
        const uint32_t before = p < size ? dq[p] : 0xFFFFFFFFu;
        while (size <= p) dq[size++] = 0xFFFFFFFFu;          // ChordFingerTable::setFinger (66-87)
        dq[p] = responsible[q];
        changed += before != responsible[q];
    }
    return changed;
}

void ChordHost::stabilize(const uint32_t* nodes, uint64_t m, uint64_t* succ_changed, uint64_t* lists_changed,
                          uint64_t* pred_changed, std::vector<uint32_t>* changed_succ0)
{
    const uint64_t n = ids.size();
    const std::vector<K160>& id = ids;
    // every message of the round sees the tables as they stand at its start (as the fixfingers round)
    std::vector<uint32_t> nl((size_t)m * sls, 0xFFFFFFFFu), tgt(m);
    std::vector<uint8_t> nn(m);
    for (uint64_t j = 0; j < m; ++j) {
        const uint32_t v = nodes[j];
        const uint32_t s = succ[(size_t)v * sls];
        // handleRpcStabilizeResponse (Chord.cc:1072-1104): the successor's predecessor p becomes
        // the successor when p lies in (v, s); NotifyCall to the (new) successor t
        const uint32_t p = pred[s];
        const uint32_t t = (p != 0xFFFFFFFFu && between_open(id[p], id[v], id[s])) ? p : s;
        tgt[j] = t;
        // handleRpcNotifyResponse -> ChordSuccessorList::updateList (ChordSuccessorList.cc:101-119):
        // t, then t's successors outside [v, t], at most successorListSize - 1 of them looked at;
        // every entry not re-added is dropped (removeOldSuccessors, 170-194)
        uint32_t* row = nl.data() + (size_t)j * sls;
        int k = 0;
        row[k++] = t;
        const int ts = std::min<int>(nsucc[t], sls - 1);
        for (int q = 0; q < ts; ++q) {
            const uint32_t x = succ[(size_t)t * sls + q];
            if (!between_LR(id[x], id[v], id[t])) row[k++] = x;
        }
        nn[j] = (uint8_t)k;
    }
    // rpcNotify at t (1106-1189): the caller becomes t's predecessor when it lies in (pred, t); over
    // the round's callers that leaves the one nearest t (every acceptance moves pred closer), if
    // it is in (pred0, t)
    std::vector<uint32_t> best(n, 0xFFFFFFFFu);
    for (uint64_t j = 0; j < m; ++j) {
        const uint32_t t = tgt[j], v = nodes[j];
        if (best[t] == 0xFFFFFFFFu || k_lt(k_sub(id[t], id[v]), k_sub(id[t], id[best[t]]))) best[t] = v;
    }
    *pred_changed = *succ_changed = *lists_changed = 0;
    for (uint64_t t = 0; t < n; ++t) {
        const uint32_t b = best[t];
        if (b == 0xFFFFFFFFu) continue;
        const uint32_t p0 = pred[t];
        if ((p0 == 0xFFFFFFFFu || between_open(id[b], id[p0], id[t])) && b != p0) {
            pred[t] = b;
            ++*pred_changed;
        }
    }
    for (uint64_t j = 0; j < m; ++j) {
        const uint32_t v = nodes[j];
        uint32_t* row = succ.data() + (size_t)v * sls;
        const bool same = nn[j] == nsucc[v] && std::equal(row, row + nn[j], nl.data() + (size_t)j * sls);
        if (!same) ++*lists_changed;
        if (row[0] != nl[(size_t)j * sls]) { ++*succ_changed; changed_succ0->push_back(v); }
        std::copy(nl.data() + (size_t)j * sls, nl.data() + (size_t)(j + 1) * sls, row);
        nsucc[v] = nn[j];
        succ0[v] = row[0];
    }
    // getFinger falls back to the successor (ChordFingerTable.cc:174-193)
    for (uint32_t v : *changed_succ0) resolve_row(v);
}

// ---------------------------------------------------------------------------------------------
// Kademlia maintenance

void KadHost::clear()
{
    ids.clear(); sib.clear(); bk.clear();
    k = s = 0;
}

void KadHost::import(const K160* keys, uint64_t n, int k_in, int s_in, const uint32_t* siblings,
                     const uint8_t* bucket_count, const uint32_t* bucket_nodes)
{
    clear();
    k = k_in; s = s_in;
    ids.assign(keys, keys + n);
    sib.assign(n, {});
    bk.assign(n * 160, {});
    const uint64_t S5 = 5ull * (uint64_t)s;
    for (uint64_t v = 0; v < n; ++v) {
        std::vector<uint32_t>& L = sib[v];
        for (uint64_t i = 0; i < S5; ++i)
            if (siblings[v * S5 + i] != 0xFFFFFFFFu) L.push_back(siblings[v * S5 + i]);
        const K160 me = ids[v];
        std::sort(L.begin(), L.end(), [&](uint32_t a, uint32_t b) { return k_lt(k_xor(ids[a], me), k_xor(ids[b], me)); });
        for (int m = 0; m < 160; ++m) {
            const uint64_t bi = v * 160 + (uint64_t)m;
            bk[bi].assign(bucket_nodes + bi * (uint64_t)k, bucket_nodes + bi * (uint64_t)k + bucket_count[bi]);
        }
    }
}

bool KadHost::export_k(uint32_t* siblings, uint8_t* bucket_count, uint32_t* bucket_nodes) const
{
    const uint64_t S5 = 5ull * (uint64_t)s, nn = n();
    bool ok = true;
    for (uint64_t v = 0; v < nn; ++v) {
        for (uint64_t i = 0; i < S5; ++i) siblings[v * S5 + i] = i < sib[v].size() ? sib[v][i] : 0xFFFFFFFFu;
        for (int m = 0; m < 160; ++m) {
            const uint64_t bi = v * 160 + (uint64_t)m;
            const std::vector<uint32_t>& B = bk[bi];
            ok &= B.size() <= (size_t)k;
            bucket_count[bi] = (uint8_t)std::min(B.size(), (size_t)k);
            for (int q = 0; q < k; ++q) bucket_nodes[bi * (uint64_t)k + q] = (size_t)q < B.size() ? B[q] : 0xFFFFFFFFu;
        }
    }
    return ok;
}

bool KadHost::routing_add(uint32_t v, uint32_t h, bool alive, KadRoundCount* st)
{
    if (h == v) return false;                                     // 437-439
    const K160 me = ids[v];
    std::vector<uint32_t>& S = sib[v];
    for (uint32_t x : S)                                          // already a sibling (454-481)
        if (x == h) { if (alive) st->refreshed++; return true; }
    const K160 dh = k_xor(ids[h], me);
    std::vector<uint32_t>& B = bk[(uint64_t)v * 160 + (uint64_t)k_msb(dh)];
    for (size_t i = 0; i < B.size(); ++i)                         // already in its bucket (483-535)
        if (B[i] == h) {
            if (alive) {                                          // erase, re-add to the tail (514-517)
                B.erase(B.begin() + (long)i);
                B.push_back(h);
                st->refreshed++;
            }
            return true;
        }
    bool result = false;
    uint32_t cur = h;
    const size_t cap = 5u * (size_t)s;
    // siblingTable->isAddable: room, or closer than back() (NodeVector.h:381-399)
    if (S.size() < cap || !k_lt(k_xor(ids[S.back()], me), dh)) {    // 537-616
        size_t pos = 0;
        while (pos < S.size() && !k_lt(dh, k_xor(ids[S[pos]], me))) ++pos;
        S.insert(S.begin() + (long)pos, h);
        st->sib_changes++;
        if (S.size() <= cap) return true;                         // simply added
        cur = S.back();                                           // the preempted handle goes on
        S.pop_back();
        result = true;
    }
    std::vector<uint32_t>& B2 = bk[(uint64_t)v * 160 + (uint64_t)k_msb(k_xor(ids[cur], me))];
    if (B2.size() < (size_t)k) {                                  // !bucket->isFull() (665-701)
        B2.push_back(cur);
        st->bucket_changes++;
        return true;
    }
    if (cur != h) st->lost++;             // a preempted sibling whose bucket is full leaves the tables
    else if (alive) st->replacement++;    // replacement cache (729-745): membership unchanged
    return result;
}

void KadHost::refresh_plan(const uint32_t* nodes, uint64_t m, const uint8_t* flags, const uint32_t* stale, int Rs,
                           int Rb, std::vector<K160>* keys, std::vector<uint32_t>* src, std::vector<int>* R) const
{
    for (uint64_t j = 0; j < m; ++j) {
        const uint32_t v = nodes[j];
        const uint8_t f = flags ? flags[j] : 3;
        const K160 me = ids[v];
        if (f & 1) { keys->push_back(me); src->push_back(v); R->push_back(Rs); }
        if (!(f & 2) || sib[v].empty()) continue;                 // if (siblingTable->size()) (1632)
        // diff = L - (sharedPrefixLength(front) + 1) = msb(self ^ front) for b = 1 (1636-1637)
        const int diff = k_msb(k_xor(ids[sib[v][0]], me));
        for (int i = 159; i >= diff; --i) {
            if (stale && !((stale[j * 5 + (uint64_t)(i >> 5)] >> (i & 31)) & 1u)) continue;
            K160 key = me;
            key.w[i >> 5] ^= 1u << (i & 31);                      // self ^ (OverlayKey(1) << i) (1647-1648)
            keys->push_back(key); src->push_back(v); R->push_back(Rb);
        }
    }
}

void KadHost::apply_round(const std::vector<KadRoundLookup>& lk, KadRoundCount* st)
{
    struct Ev { int64_t t; uint32_t kind, task, idx; };
    const uint64_t nn = n();
    std::vector<uint64_t> off(nn + 1, 0);
    for (const KadRoundLookup& L : lk) {
        for (int i = 0; i < L.ncall; ++i) off[L.cnode[i] + 1]++;
        off[L.src + 1] += (uint64_t)L.nresp;
        st->responses += (uint64_t)L.nresp;
    }
    for (uint64_t v = 0; v < nn; ++v) off[v + 1] += off[v];
    std::vector<Ev> ev(off[nn]);
    std::vector<uint64_t> fill(off.begin(), off.end() - 1);
    for (size_t t = 0; t < lk.size(); ++t) {
        const KadRoundLookup& L = lk[t];
        for (int i = 0; i < L.ncall; ++i) ev[fill[L.cnode[i]]++] = Ev{L.ctime[i], 0u, (uint32_t)t, (uint32_t)i};
        for (int i = 0; i < L.nresp; ++i) ev[fill[L.src]++] = Ev{L.tarr[i], 1u, (uint32_t)t, (uint32_t)i};
    }
    for (uint64_t v = 0; v < nn; ++v) {
        Ev* b = ev.data() + off[v];
        Ev* e = ev.data() + off[v + 1];
        std::sort(b, e, [](const Ev& x, const Ev& y) {
            if (x.t != y.t) return x.t < y.t;
            if (x.kind != y.kind) return x.kind < y.kind;
            if (x.task != y.task) return x.task < y.task;
            return x.idx < y.idx;
        });
        for (Ev* q = b; q < e; ++q) {
            const KadRoundLookup& L = lk[q->task];
            if (q->kind == 0) {
                routing_add((uint32_t)v, L.src, true, st);
            } else {
                for (int c = 0; c < L.ncarried[q->idx]; ++c) routing_add((uint32_t)v, L.carried[q->idx][c], false, st);
                routing_add((uint32_t)v, L.resp[q->idx], true, st);
            }
        }
    }
}

bool epichord_prepare(const K160* keys, uint64_t n, int L, const uint32_t* succ, const uint8_t* nsucc,
                      const uint32_t* pred, const uint8_t* npred, const uint8_t* lists_full, const uint64_t* cache_off,
                      const uint32_t* cache_node, const int64_t* cache_last, const int64_t* cache_ttl,
                      std::vector<uint32_t>* meta, std::vector<uint32_t>* cn, std::vector<int64_t>* cl,
                      std::vector<int64_t>* ct, std::string* err)
{
    for (uint64_t v = 1; v < n; ++v)
        if (!k_lt(keys[v - 1], keys[v])) { *err = "node ids must be sorted ascending and unique"; return false; }
    const K160 one{{1, 0, 0, 0, 0}}, zero{{0, 0, 0, 0, 0}};
    auto node_err = [&](uint64_t v, const char* what) {
        *err = "EpiChord snapshot, node " + std::to_string(v) + ": " + what;
        return false;
    };
    meta->assign(n, 0);
    for (uint64_t v = 0; v < n; ++v) {
        const int ns = nsucc[v], np = npred[v], full = lists_full[v] & 3;
        const int cnt[2] = {ns, np};
        const uint32_t* lst[2] = {succ + v * L, pred + v * L};
        for (int l = 0; l < 2; ++l) {
            // EpiChordNodeList (EpiChordNodeList.cc:56-161): thisNode stays in the map (last) until
            // the list holds nodeListSize other nodes; isFull() is its absence
            const bool isfull = (full >> l) & 1;
            if (cnt[l] > L) return node_err(v, "more list entries than successorListSize");
            if (isfull ? cnt[l] == 0 : cnt[l] == L) return node_err(v, "isFull() inconsistent with the list length");
            K160 prev{};
            for (int i = 0; i < cnt[l]; ++i) {
                const uint32_t x = lst[l][i];
                if (x >= n || x == v) return node_err(v, "list entry is not another node");
                K160 off = k_sub(keys[x], keys[v]);
                if (l == 1) off = k_sub(zero, off);
                if (i && !k_lt(prev, off)) return node_err(v, "list entries not closest first / repeated");
                prev = off;
            }
        }
        (*meta)[v] = (uint32_t)ns | ((uint32_t)np << 8) | ((uint32_t)full << 16);
    }
    if (cache_off[0] != 0) { *err = "cache_off[0] must be 0"; return false; }
    const uint64_t E = cache_off[n];
    if (E && (!cache_node || !cache_last || !cache_ttl)) { *err = "cache arrays missing"; return false; }
    cn->assign(E, 0);
    cl->assign(E, 0);
    ct->assign(E, 0);
    std::vector<uint64_t> perm;
    std::vector<K160> sums;
    for (uint64_t v = 0; v < n; ++v) {
        const uint64_t a = cache_off[v], b = cache_off[v + 1];
        if (b < a || b > E) return node_err(v, "cache_off not monotone");
        // liveCache order: x - (thisNode + 1) (EpiChordFingerCache.cc:85, 117-126)
        const K160 base = k_add(keys[v], one);
        perm.resize(b - a);
        sums.resize(b - a);
        for (uint64_t i = a; i < b; ++i) {
            const uint32_t x = cache_node[i];
            if (x >= n || x == v) return node_err(v, "cache entry is not another node");
            if (cache_ttl[i] < 0) return node_err(v, "negative cache ttl");
            perm[i - a] = i;
            sums[i - a] = k_sub(keys[x], base);
        }
        std::sort(perm.begin(), perm.end(), [&](uint64_t p, uint64_t q) { return k_lt(sums[p - a], sums[q - a]); });
        for (uint64_t i = 0; i < b - a; ++i) {
            const uint64_t j = perm[i];
            if (i && cache_node[j] == (*cn)[a + i - 1]) return node_err(v, "a node twice in the finger cache");
            (*cn)[a + i] = cache_node[j];
            (*cl)[a + i] = cache_last[j];
            (*ct)[a + i] = cache_ttl[j];
        }
    }
    return true;
}

}  // namespace ovs
