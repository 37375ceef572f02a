// kad.hip -- Kademlia table builders (snapshot rule and explicit tables), findNode and the
// dispatch of the iterative-lookup kernel K2 (kad_route.hip, one object per alpha x exact) for
// gfx950 (MI355X).
#include <hipcub/hipcub.hpp>

#include <cstdlib>

#include "kad_dev.hpp"

namespace ovs {

void kad_free(KadTables& t)
{
    if (t.nodes) hipFree(t.nodes);
    if (t.nodex) hipFree(t.nodex);
    if (t.blks) hipFree(t.blks);
    if (t.sib) hipFree(t.sib);
    if (t.slev) hipFree(t.slev);
    if (t.goff) hipFree(t.goff);
    if (t.gtop) hipFree(t.gtop);
    if (t.gidx) hipFree(t.gidx);
    if (t.gend) hipFree(t.gend);
    t.nodes = nullptr; t.nodex = nullptr; t.blks = nullptr; t.sib = nullptr; t.slev = nullptr; t.rows_blks = 0;
    t.goff = nullptr; t.gtop = nullptr; t.gidx = nullptr; t.gend = nullptr; t.gtotal = 0;
    t.general = 0; t.b = 1; t.nb = KEYBITS;
    t.tl = 0; t.tend = 0;
}

// ---------------------------------------------------------------------------
// builders

// the KadNode summary of a node's sibling set: R = max (s ^ key), level mask = OR 2^msb(s ^ key).
// One pass over the siblings' keys: endIndex = msb(R) is the largest level, and the siblings at the
// four levels endIndex .. endIndex - 3 are counted while it rises (kad_sib_prefix's counts follow).
// rowlo = -2: the row starts at endIndex.  Returns endIndex.
__device__ int kad_node_summary(const KeyRec* __restrict__ recs, const double2* __restrict__ xy, uint32_t v,
                                const uint32_t* L, int cnt, int rowlo, KadNode* __restrict__ out, KadX* __restrict__ ox)
{
    const K160 me = kload(recs, v);
    K160 R{}, M{};
    for (int i = 0; i < 5; ++i) { R.w[i] = 0; M.w[i] = 0; }
    int end = -1;
    uint32_t n0 = 0, n1 = 0, n2 = 0, n3 = 0;     // siblings at levels end, end - 1, end - 2, end - 3
    for (int i = 0; i < cnt; ++i) {
        const K160 d = k_xor(kload(recs, L[i]), me);
        if (k_gt(d, R)) R = d;
        const int mb = k_msb(d);
#pragma unroll
        for (int w = 0; w < 5; ++w) M.w[w] |= (mb >> 5) == w ? 1u << (mb & 31) : 0u;   // selects: no scratch
        if (mb > end) {
            const int s = mb - end;               // the counts move s levels down
            const uint32_t a0 = n0, a1 = n1, a2 = n2;
            n3 = s == 1 ? a2 : s == 2 ? a1 : s == 3 ? a0 : 0u;
            n2 = s == 1 ? a1 : s == 2 ? a0 : 0u;
            n1 = s == 1 ? a0 : 0u;
            n0 = 1;
            end = mb;
        } else {
            const int j = end - mb;
            n0 += j == 0 ? 1u : 0u;
            n1 += j == 1 ? 1u : 0u;
            n2 += j == 2 ? 1u : 0u;
            n3 += j == 3 ? 1u : 0u;
        }
    }
    if (rowlo == -2) rowlo = end;
    const int mlo = end > 63 ? end - 63 : 0;
    // mask window: bits [mlo, mlo + 63]
    const int wi = mlo >> 5, sh = mlo & 31;
    const uint64_t lo = (uint64_t)kword(M, wi) | ((uint64_t)kword(M, wi + 1) << 32);   // kword: 5+ reads 0
    const uint64_t hi = (uint64_t)kword(M, wi + 2);
    const uint64_t win = sh ? ((lo >> sh) | (hi << (64 - sh))) : lo;
    bool out_bits = false;                        // any mask bit below mlo
#pragma unroll
    for (int w = 0; w < 5; ++w) {
        const int b0 = 32 * w;
        const uint32_t below = b0 + 32 <= mlo ? ~0u : b0 >= mlo ? 0u : (1u << (mlo - b0)) - 1u;
        out_bits |= (M.w[w] & below) != 0;
    }
    // siblings at levels <= endIndex - k, k = 1..4 (kad_sib_prefix)
    const uint32_t c1 = (uint32_t)cnt - n0, c2 = c1 - n1, c3 = c2 - n2, c4 = c3 - n3;
    const uint32_t lev = c1 | (c2 << 8) | (c3 << 16) | (c4 << 24);
    const double2 p = xy[v];
    KadNode o;
    for (int i = 0; i < 5; ++i) o.key[i] = me.w[i];
    o.boff = 0;
    o.x = p.x; o.y = p.y;
    o.rtop = ktop(R);
    o.mwin = win;
    o.meta = (uint32_t)(end + 1) | ((uint32_t)(rowlo + 1) << 8) | ((uint32_t)cnt << 16) | (out_bits ? KMETA_MASK_OUT : 0u);
    o.spare = lev;
    out[v] = o;
    KadX x;
    for (int i = 0; i < 5; ++i) { x.R[i] = R.w[i]; x.mask[i] = M.w[i]; }
    ox[v] = x;
    return end;
}

// top 64 key bits (96..159) of every node: the bucket builder's searches and member tops read this
// 8 B array (128 MB at 2^24 nodes, resident in the MALL) instead of the 24 B key records
__global__ void k_kad_tops(const KeyRec* __restrict__ recs, uint32_t n, uint64_t* __restrict__ tops)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) tops[i] = ktop(kload(recs, i));
}

constexpr int KB_DMAX = 26;    // prefix tables for depths 1 .. D <= 26 (2^(D+1) entries, 4 B each)

// first entry of depth d's prefix table: tables of 2^j + 1 entries for j = 1 .. d-1 precede it
__host__ __device__ __forceinline__ uint64_t kb_tab_off(int d) { return ((1ull << d) - 2) + (uint64_t)(d - 1); }

// prefix tables: B_d[P] = the first node whose top d key bits are >= P (d = 1 .. D, P = 0 .. 2^d;
// B_d[2^d] = n).  One pass over the sorted top keys: node i fills the prefixes between its
// predecessor's and its own.  T_m of any node is then [B_d[Q], B_d[Q + 1]) with d = 160 - m.
__global__ void k_kad_prefix_tables(const uint64_t* __restrict__ tops, uint32_t n, int D, uint32_t* __restrict__ tab)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t t = tops[i], tp = i ? tops[i - 1] : 0ull;
    for (int d = 1; d <= D; ++d) {
        uint32_t* B = tab + kb_tab_off(d);
        const uint64_t p = t >> (64 - d);
        const uint64_t from = i ? (tp >> (64 - d)) + 1 : 0ull;
        for (uint64_t P = from; P <= p; ++P) B[P] = i;
        if (i == n - 1)
            for (uint64_t P = p + 1; P <= (1ull << d); ++P) B[P] = n;
    }
}

// snapshot pass A: sibling table (the 5s XOR-closest nodes, what routingAdd converges to:
// Kademlia.cc:537-616) and the node summary; the row length for the owned arc
// a block's sibling lists live in LDS (row stride KS_STRIDE words, 5s <= 64): built, read and written
// out as whole rows with coalesced copies -- per-lane lists at a 4 * 5s byte stride touch a line per
// lane for every entry
constexpr int KS_BLOCK = 128;
constexpr int KS_STRIDE = 65;

__device__ __forceinline__ void ks_load_rows(uint32_t* lsb, const uint32_t* __restrict__ sib, uint32_t v0, uint32_t nv,
                                             int S5)
{
    const uint32_t tot = nv * (uint32_t)S5;
    for (uint32_t i = threadIdx.x; i < tot; i += blockDim.x) {
        const uint32_t r = i / (uint32_t)S5, c = i - r * (uint32_t)S5;
        lsb[r * KS_STRIDE + c] = sib[(uint64_t)v0 * S5 + i];
    }
    __syncthreads();
}

__global__ __launch_bounds__(KS_BLOCK) void k_kad_siblings(const KeyRec* __restrict__ recs,
                                                            const double2* __restrict__ xy, uint32_t n, int S5, int bpb,
                                                            uint32_t own_lo, uint32_t own_hi,
                                                            const uint64_t* __restrict__ tops,
                                                            const uint32_t* __restrict__ tab, int D, int dg,
                                                            uint32_t* __restrict__ sib, KadNode* __restrict__ out,
                                                            KadX* __restrict__ ox, uint64_t* __restrict__ rowlen)
{
    __shared__ uint32_t lsb[KS_BLOCK * KS_STRIDE];
    const uint32_t v0 = blockIdx.x * KS_BLOCK;
    const uint32_t v = v0 + threadIdx.x;
    uint32_t* L = lsb + threadIdx.x * KS_STRIDE;
    if (v < n) {
    const K160 me = kload(recs, v);
    int cnt = 0;
    if (n - 1 < (uint32_t)S5) {
        for (uint32_t x = 0; x < n; ++x)
            if (x != v) L[cnt++] = x;
    } else {
        // the descent below starts at the first bit whose split leaves the node's block with fewer
        // than 5s+1 nodes: found in the prefix tables (v's block at depth d = [B_d[P], B_d[P+1]),
        // sizes shrink with d), not by one binary search per level
        const uint64_t mtop = tops[v];
        auto range = [&](int d, uint32_t& a, uint32_t& z) {
            if (d == 0) { a = 0; z = n; return; }
            const uint32_t* B = tab + kb_tab_off(d);
            const uint64_t P = mtop >> (64 - d);
            a = B[P]; z = B[P + 1];
        };
        // deepest depth whose block still holds >= 5s+1 nodes: a linear walk from the depth where
        // an average block holds that many (dg, the same for every lane, so a wave's table reads
        // stay in a few lines; a per-lane binary search over the depths scattered them over
        // every table and ran 2.5x slower)
        int d0 = dg;
#ifdef OVS_KS_NOTAB
        d0 = 0;                                    // A/B build: the whole descent by binary searches
        if (false)
#endif
        {
            uint32_t ra, rz;
            range(d0, ra, rz);
            if (rz - ra >= (uint32_t)S5 + 1) {
                while (d0 < D) {
                    range(d0 + 1, ra, rz);
                    if (rz - ra < (uint32_t)S5 + 1) break;
                    ++d0;
                }
            } else {
                while (d0 > 0) {
                    --d0;
                    range(d0, ra, rz);
                    if (rz - ra >= (uint32_t)S5 + 1) break;
                }
            }
        }
        uint32_t lo, hi;
        range(d0, lo, hi);
        for (int b = KEYBITS - 1 - d0; b >= 0; --b) {
            const uint32_t mid = split_bit(recs, lo, hi, b);
            const uint32_t nb = kbit(me, b);
            const uint32_t nlo = nb ? mid : lo, nhi = nb ? hi : mid;
            const uint32_t flo = nb ? lo : mid, fhi = nb ? mid : hi;
            if (nhi - nlo >= (uint32_t)S5 + 1) { lo = nlo; hi = nhi; continue; }
            // the block sharing one more bit holds < 5s+1 nodes: all of it, plus the
            // XOR-closest remainder of the other half T_b
            for (uint32_t x = nlo; x < nhi; ++x)
                if (x != v) L[cnt++] = x;
            int need = S5 - cnt;
            uint32_t rl = flo, rh = fhi;
            for (int bb = b - 1; need > 0; --bb) {
                if (rh - rl <= (uint32_t)need || bb < 0) {
                    for (uint32_t x = rl; x < rh && need > 0; ++x) { L[cnt++] = x; --need; }
                    break;
                }
                const uint32_t m2 = split_bit(recs, rl, rh, bb);
                const uint32_t nbb = kbit(me, bb);
                const uint32_t nl = nbb ? m2 : rl, nh = nbb ? rh : m2;
                const uint32_t fl = nbb ? rl : m2, fh = nbb ? m2 : rh;
                if (nh - nl >= (uint32_t)need) { rl = nl; rh = nh; }
                else {
                    for (uint32_t x = nl; x < nh; ++x) L[cnt++] = x;
                    need -= (int)(nh - nl);
                    rl = fl; rh = fh;
                }
            }
            break;
        }
    }
    for (int i = cnt; i < S5; ++i) L[i] = NONE;
    // buckets below endIndex hold only siblings: the stored row starts at endIndex
    const int end = kad_node_summary(recs, xy, v, L, cnt, -2, out, ox);
    rowlen[v] = (v >= own_lo && v < own_hi && end >= 0) ? (uint64_t)(KEYBITS - end) * (uint64_t)bpb : 0;
    }
    __syncthreads();
    const uint32_t nv = min((uint32_t)KS_BLOCK, n > v0 ? n - v0 : 0u), tot = nv * (uint32_t)S5;
    for (uint32_t i = threadIdx.x; i < tot; i += blockDim.x) {
        const uint32_t r = i / (uint32_t)S5, c = i - r * (uint32_t)S5;
        sib[(uint64_t)v0 * S5 + i] = lsb[r * KS_STRIDE + c];
    }
}

// 1 when two node IDs share their top 63 bits (then top-64 XOR distances of distinct nodes can
// tie and the K2 comparisons need the exact fallback, cand_lt<true>); IDs are sorted, so
// adjacent pairs suffice
__global__ void k_kad_prefix_ties(const KeyRec* __restrict__ recs, uint32_t n, uint32_t* flag)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i + 1 >= n) return;
    if (((top64(kload(recs, i)) ^ top64(kload(recs, i + 1))) >> 1) == 0) atomicOr(flag, 1u);
}

// row offsets of the owned nodes; an off-arc node's row exists on its owner only: NONE (>= every
// replicated-region end, so a sharded kernel can never read a row through it)
__global__ void k_kad_set_boff(KadNode* nodes, const uint64_t* off, uint32_t lo, uint32_t hi, uint64_t base,
                               uint32_t n)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v < n) nodes[v].boff = (v >= lo && v < hi) ? (uint32_t)(base + off[v]) : NONE;
}

__device__ __forceinline__ void put_entry(KadBlk* __restrict__ blks, uint64_t blk0, int q, uint32_t x,
                                          const KeyRec* __restrict__ recs)
{
    KadBlk* b = blks + blk0 + q / KBLK;
    b->idx[q % KBLK] = x;
    b->top[q % KBLK] = x == NONE ? ~0ull : ktop(kload(recs, x));
}

// a node's sibling row: the node itself, then its S5 siblings (NONE padded) in ascending level
// msb(x ^ v), stable -- the node and its siblings at levels <= l are a prefix, so a findNode whose
// answer lies below 2^(l+1) reads only that prefix's blocks (kad_sib_prefix), and the node itself --
// a candidate of every sibling-zone findNode (Kademlia.cc:1207-1211) -- comes with the first block
__device__ void put_sibling_row(KadBlk* __restrict__ blks, uint64_t blk0, int sbn, const uint32_t* L, int S5,
                                uint32_t self, const K160& me, const KeyRec* __restrict__ recs)
{
    uint32_t x[65];
    uint8_t lv[65];
    x[0] = self;
    lv[0] = 0;
    int cnt = 1;
    for (int i = 0; i < S5 && i < 64; ++i) {
        if (L[i] == NONE) continue;
        // insertion by level, stable
        const uint8_t l = (uint8_t)k_msb(k_xor(kload(recs, L[i]), me));
        int j = cnt++;
        while (j > 1 && lv[j - 1] > l) { x[j] = x[j - 1]; lv[j] = lv[j - 1]; --j; }
        x[j] = L[i];
        lv[j] = l;
    }
    for (int q = 0; q < sbn * KBLK; ++q) put_entry(blks, blk0, q, q < cnt ? x[q] : NONE, recs);
}

// bucket m of node v under the snapshot rule: up to k members of T_m = [flo, fhi) (the nodes at
// msb(x ^ v) = m) minus v's siblings L, chosen by Floyd sampling with kad_hash(seed, v, m, j)
// (DESIGN.md §4), written in ascending index order to the bpb blocks at blk0.  Returns the members.
// Siblings lie at levels <= endIndex (the farthest one's level), so only the bucket m = endIndex can
// hold any: may_sib = false skips the sibling scans for the buckets above it.  L (S5 entries) is read
// with stride ls (the builders stage it in LDS).
__device__ int kad_bucket_fill(const KeyRec* __restrict__ recs, uint32_t v, int m, uint32_t flo, uint32_t fhi,
                               const uint32_t* L, int ls, int S5, int k, uint64_t seed, KadBlk* __restrict__ blks,
                               uint64_t blk0, bool may_sib)
{
    uint32_t chosen[KMAX];
    const int bpb = (k + KBLK - 1) / KBLK;
    uint32_t nsin = 0;
    if (may_sib)
        for (int i = 0; i < S5; ++i) {
            const uint32_t x = L[i * ls];
            nsin += (x != NONE && x >= flo && x < fhi) ? 1u : 0u;
        }
    const uint32_t c = (fhi - flo) - nsin;
    int nch = 0;
    if (c <= (uint32_t)k) {
        for (uint32_t j = 0; j < c; ++j) chosen[nch++] = j;
    } else {
        for (uint32_t j = c - (uint32_t)k; j < c; ++j) {
            const uint32_t t = mod_u64_u32(kad_hash(seed, v, (uint32_t)m, j), j + 1);
            bool dup = false;
            for (int q = 0; q < nch; ++q) dup |= (chosen[q] == t);
            chosen[nch++] = dup ? j : t;
        }
        for (int a = 1; a < nch; ++a) {
            const uint32_t x = chosen[a];
            int q = a - 1;
            while (q >= 0 && chosen[q] > x) { chosen[q + 1] = chosen[q]; --q; }
            chosen[q + 1] = x;
        }
    }
    int outn = 0;
    if (nsin == 0) {
        for (int q = 0; q < nch; ++q) put_entry(blks, blk0, outn++, flo + chosen[q], recs);
    } else {
        uint32_t rank = 0;
        int q = 0;
        for (uint32_t x = flo; x < fhi && q < nch; ++x) {
            bool is_sib = false;
            for (int i = 0; i < S5; ++i) is_sib |= (L[i * ls] == x);
            if (is_sib) continue;
            if (rank == chosen[q]) { put_entry(blks, blk0, outn++, x, recs); ++q; }
            ++rank;
        }
    }
    for (int q = outn; q < bpb * KBLK; ++q) put_entry(blks, blk0, q, NONE, recs);
    return outn;
}

// first x in [lo, hi) whose key bits m..159 are >= Q's (upper: > Q's); keys sorted ascending, so the
// prefix is monotone.  m >= 96: the prefix lies in the top 64 bits (tops); below, the full keys.
__device__ uint32_t kad_prefix_bound(const KeyRec* __restrict__ recs, const uint64_t* __restrict__ tops, uint32_t lo,
                                     uint32_t hi, int m, const K160& Q, bool upper)
{
    if (m >= 96) {
        const int sh = m - 96;
        const uint64_t q = ktop(Q) >> sh;
        while (lo < hi) {
            const uint32_t mid = lo + ((hi - lo) >> 1);
            const uint64_t p = tops[mid] >> sh;
            if (upper ? p <= q : p < q) lo = mid + 1; else hi = mid;
        }
        return lo;
    }
    K160 qm = Q;
#pragma unroll
    for (int w = 0; w < 5; ++w) {
        const int b0 = 32 * w;
        qm.w[w] = b0 + 32 <= m ? 0u : b0 >= m ? qm.w[w] : qm.w[w] & (~0u << (m - b0));
    }
    while (lo < hi) {
        const uint32_t mid = lo + ((hi - lo) >> 1);
        K160 x = kload(recs, mid);
#pragma unroll
        for (int w = 0; w < 5; ++w) {
            const int b0 = 32 * w;
            x.w[w] = b0 + 32 <= m ? 0u : b0 >= m ? x.w[w] : x.w[w] & (~0u << (m - b0));
        }
        if (upper ? k_le(x, qm) : k_lt(x, qm)) lo = mid + 1; else hi = mid;
    }
    return lo;
}

constexpr int KB_LANES = 24;   // k_kad_bucket_rows: lanes per node, lane j builds buckets m = 159 - j - 24 i (rows ~ log2 n - 4 long)
// T_m of node v = [flo, fhi): the nodes at msb(x ^ v) = m, one contiguous index range of the sorted
// keys, from two prefix-table reads (depth 160 - m <= D; deeper levels search the few nodes of v's own
// depth-D prefix)
__device__ __forceinline__ void kb_tm_range(const KeyRec* __restrict__ recs, const uint64_t* __restrict__ tops,
                                            const uint32_t* __restrict__ tab, int D, uint32_t v, uint64_t mtop, int m,
                                            uint32_t& flo, uint32_t& fhi)
{
    const int d = KEYBITS - m;
    if (d <= D) {
        const uint64_t Q = (mtop >> (64 - d)) ^ 1ull;              // v's top d bits, bit m flipped
        const uint32_t* B = tab + kb_tab_off(d);
        flo = B[Q];
        fhi = B[Q + 1];
    } else {
        // T_m lies inside v's own depth-D prefix range: search there (small or irregular networks:
        // the full key is read only here)
        const K160 me = kload(recs, v);
        const uint64_t PD = mtop >> (64 - D);
        const uint32_t* B = tab + kb_tab_off(D);
        const bool below = kbit(me, m) != 0;
        const uint32_t slo = below ? B[PD] : v + 1, shi = below ? v : B[PD + 1];
        K160 Q = me;
#pragma unroll
        for (int w = 0; w < 5; ++w) Q.w[w] ^= (m >> 5) == w ? 1u << (m & 31) : 0u;   // selects: no scratch
        flo = kad_prefix_bound(recs, tops, slo, shi, m, Q, false);
        fhi = kad_prefix_bound(recs, tops, flo, shi, m, Q, true);
    }
}

// Floyd's draw i (i < k) of the snapshot rule: min(k, c) ranks out of the c candidates of bucket m
// of node v; the draws are resolved in order (a repeat of an earlier draw takes j), kb_floyd_resolve
__device__ __forceinline__ uint32_t kb_floyd_draw(uint64_t seed, uint32_t v, int m, uint32_t c, int k, int i)
{
    if (i >= k || (uint32_t)i >= c) return NONE;
    if (c <= (uint32_t)k) return (uint32_t)i;
    const uint32_t j = c - (uint32_t)k + (uint32_t)i;
    return mod_u64_u32(kad_hash(seed, v, (uint32_t)m, j), j + 1);
}

// ch[0..KC) <- the resolved draws in ascending order (NONE = unused, the largest)
template <int KC>
__device__ __forceinline__ void kb_floyd_resolve(uint32_t (&ch)[KC], uint32_t c, int k)
{
#pragma unroll
    for (int i = 0; i < KC; ++i) {
        if (c > (uint32_t)k && i < k) {
            const uint32_t j = c - (uint32_t)k + (uint32_t)i;
            bool dup = false;
#pragma unroll
            for (int q = 0; q < i; ++q) dup |= ch[q] == ch[i];
            ch[i] = dup ? j : ch[i];
        }
    }
#pragma unroll
    for (int a = 0; a < KC; ++a)          // odd-even transposition sort (NONE = the largest)
#pragma unroll
        for (int b = a & 1; b + 1 < KC; b += 2) {
            const uint32_t x = ch[b], y = ch[b + 1];
            ch[b] = x < y ? x : y;
            ch[b + 1] = x < y ? y : x;
        }
}

// the rank-th set bit of the 256-bit mask z0..z3
__device__ __forceinline__ uint32_t kb_nth_bit256(uint64_t z0, uint64_t z1, uint64_t z2, uint64_t z3, uint32_t rnk)
{
    const uint32_t c0 = __popcll(z0), c1 = __popcll(z1), c2 = __popcll(z2);
    uint64_t z = z0;
    uint32_t base = 0;
    if (rnk >= c0) { rnk -= c0; z = z1; base = 64;
        if (rnk >= c1) { rnk -= c1; z = z2; base = 128;
            if (rnk >= c2) { rnk -= c2; z = z3; base = 192; } } }
    uint32_t pos = 0;
#pragma unroll
    for (int sh = 32; sh > 0; sh >>= 1) {
        const uint32_t c = __popcll(z & ((1ull << sh) - 1));
        if (rnk >= c) { rnk -= c; z >>= sh; pos += sh; }
    }
    return base + pos;
}

// the row blocks' 16 B stores (OVS_KB_NT: non-temporal, so the 29 GB of rows a 2^24 build writes
// do not displace the 128 MB top-key array the member gathers read from the MALL -- an A/B build)
typedef unsigned int kb_u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void kb_store(kb_u4* p, kb_u4 v)
{
#ifdef OVS_KB_NT
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}

// bucket m > endIndex of node v under the snapshot rule: up to k members of T_m chosen
// by Floyd sampling with kad_hash(seed, v, m, j), in ascending index order, written as bpb KadBlks.
// (The bucket m = endIndex, the only one that can hold siblings, is built in k_kad_sib_rows.)  Same
// blocks as kad_bucket_fill.
template <int KC>
__device__ __forceinline__ void kad_bucket_row(const KeyRec* __restrict__ recs, const uint64_t* __restrict__ tops,
                                               const uint32_t* __restrict__ tab, int D, int k, uint64_t seed,
                                               KadBlk* __restrict__ blks, uint32_t v, uint64_t mtop, uint32_t boff, int m)
{
    const int bpb = (k + KBLK - 1) / KBLK;
    uint32_t flo, fhi;
    kb_tm_range(recs, tops, tab, D, v, mtop, m, flo, fhi);
    const uint32_t c = fhi - flo;
    uint32_t ch[KC];
#pragma unroll
    for (int i = 0; i < KC; ++i) ch[i] = kb_floyd_draw(seed, v, m, c, k, i);
    kb_floyd_resolve(ch, c, k);
#pragma unroll
    for (int q = 0; q < KC; ++q) ch[q] = ch[q] == NONE ? NONE : flo + ch[q];
    uint64_t tp[KC];
#pragma unroll
    for (int q = 0; q < KC; ++q) tp[q] = ch[q] == NONE ? ~0ull : tops[ch[q]];
    KadBlk* B = blks + (uint64_t)boff + (uint64_t)(KEYBITS - 1 - m) * (uint64_t)bpb;
#pragma unroll
    for (int b = 0; b < KC / KBLK; ++b) {
        if (b >= bpb) break;
        kb_u4* dd = reinterpret_cast<kb_u4*>(B + b);
#pragma unroll
        for (int q = 0; q < KBLK; q += 2) {
            const uint64_t t0 = tp[b * KBLK + q], t1 = tp[b * KBLK + q + 1];
            kb_store(dd + q / 2, kb_u4{(uint32_t)t0, (uint32_t)(t0 >> 32), (uint32_t)t1, (uint32_t)(t1 >> 32)});
        }
        kb_store(dd + 4, kb_u4{ch[b * KBLK], ch[b * KBLK + 1], ch[b * KBLK + 2], ch[b * KBLK + 3]});
        kb_store(dd + 5, kb_u4{ch[b * KBLK + 4], ch[b * KBLK + 5], ch[b * KBLK + 6], ch[b * KBLK + 7]});
    }
}

// snapshot pass B: the buckets m = 159 .. endIndex + 1 of every owned node, one lane per (node,
// bucket): consecutive lanes write consecutive KadBlks of a row (coalesced runs), and a lane's
// dependent chain is the node line, the prefix table, the members' tops.  The bucket endIndex
// (sibling exclusion) is built with the sibling rows (k_kad_sib_rows), eight lanes a node -- inside
// this kernel its sibling scans would hold every wave.
// (A packed layout -- one lane per bucket actually built, a wave's tasks assigned through a scan of
// its 64 nodes' bucket counts, no idle lanes -- measured 26.5 vs 25.5 ms at 2^24: the kernel is bound
// by the top buckets' random member-top reads, not by its lanes)
template <int KC>
__global__ __launch_bounds__(256) void k_kad_bucket_rows(const KeyRec* __restrict__ recs,
                                                          const uint64_t* __restrict__ tops,
                                                          const uint32_t* __restrict__ tab, int D,
                                                          const KadNode* __restrict__ nodes, int k, uint64_t seed,
                                                          KadBlk* __restrict__ blks, uint32_t own_lo, uint32_t own_hi)
{
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t v = own_lo + (uint32_t)(g / KB_LANES);
    const int lane = (int)(g % KB_LANES);
    if (v >= own_hi) return;
    const KadNode r = nodes[v];
    const int endIndex = kad_end(r.meta);
    if (endIndex < 0) return;
    for (int m = KEYBITS - 1 - lane; m > endIndex; m -= KB_LANES)
        kad_bucket_row<KC>(recs, tops, tab, D, k, seed, blks, v, ktop(as_key(r.key)), r.boff, m);
}
static inline dim3 kb_rows_grid(uint32_t nown) { return dim3((unsigned)(((uint64_t)nown * KB_LANES + 255) / 256)); }

// the owned nodes' sibling rows (put_sibling_row's layout): the node, then its siblings stable by
// level msb(x ^ v).  Eight lanes a node: lane r takes list entries r, r+8, ... (coalesced reads of
// the list), computes their levels (top 64 bits, the full keys on a tie) and ranks every entry by
// the key level * 64 + position against the node's 64 keys in LDS (stable by construction); the
// row is assembled in LDS and written as consecutive 16 B pieces, 128 B per node and instruction.
// (One lane a node, emitting level by level, had each lane's 16 B stores 576 B apart: 15.9 GB
// written for 9.7 GB of rows at 2^24 nodes, and the lists read at a 160 B lane stride.)
// Then the node's bucket m = endIndex, the only one that can hold siblings (they lie at levels <=
// endIndex), with the same eight lanes: T_m from the prefix tables, the siblings inside it counted
// and masked over the lanes' list entries, Floyd's k draws computed one a lane (the hash and
// remainder dominate) and resolved in order on every lane, the c-th non-sibling of T_m = the c-th zero
// bit of the sibling mask (a fixed-point count over the row beyond 256 nodes), and the 96 B block
// written as six 16 B pieces.  (Round 5 ran this bucket as its own kernel, one lane a node, re-reading
// the lists: 4.0 ms at 2^24.)
// a wave's LDS stores before its lanes' loads of them (a node's lanes lie in one wave)
__device__ __forceinline__ void sr_wave_fence()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr int SR_G = 8;                 // lanes per node
constexpr int SR_NPB = 256 / SR_G;      // nodes per block
constexpr int SR_ROW = 72;              // row entries: 8 * ceil((1 + 5s) / 8) for 5s <= 64

template <int KC>
__global__ __launch_bounds__(256) void k_kad_sib_rows(const KeyRec* __restrict__ recs,
                                                      const uint64_t* __restrict__ tops, const uint32_t* __restrict__ tab,
                                                      int D, const KadNode* __restrict__ nodes, int k, uint64_t seed,
                                                      int S5, int sbn, const uint32_t* __restrict__ sib,
                                                      KadBlk* __restrict__ blks, uint64_t sib_base, uint32_t own_lo,
                                                      uint32_t own_hi)
{
    __shared__ uint32_t rowx[SR_NPB][SR_ROW];
    __shared__ uint4 keys[SR_NPB][8];        // the node's 64 keys, 16 bits each
    const int g = threadIdx.x / SR_G, r = threadIdx.x % SR_G;
    const uint32_t v = own_lo + blockIdx.x * SR_NPB + (uint32_t)g;
    const bool ok = v < own_hi;
    const uint64_t mt = ok ? tops[v] : 0ull;
    uint32_t x[8], key[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int i = r + SR_G * j;
        uint32_t xx = NONE;
        if (ok && i < S5) xx = sib[(uint64_t)v * S5 + i];
        uint32_t kq = 0x7FFFu;               // past every valid key (level * 64 + i <= 10239)
        if (xx != NONE) {
            const uint64_t d = tops[xx] ^ mt;
            const int l = d ? 96 + (63 - __clzll((long long)d)) : k_msb(k_xor(kload(recs, xx), kload(recs, v)));
            kq = (uint32_t)l * 64u + (uint32_t)i;
        }
        x[j] = xx;
        key[j] = kq;
    }
    uint16_t* kh = reinterpret_cast<uint16_t*>(keys[g]);
#pragma unroll
    for (int j = 0; j < 8; ++j) kh[r + SR_G * j] = (uint16_t)key[j];
    uint32_t* row = rowx[g];
    for (int q = r; q < SR_ROW; q += SR_G) row[q] = q == 0 ? v : NONE;
    sr_wave_fence();
    // rank = keys below mine among the node's 64 (the invalid ones are 0x7FFF), two keys per packed
    // 16-bit subtract: a - key < 0 (all keys < 2^15) sets the half's sign bit, a shift turns it into
    // 1 and a packed add counts it -- 1.5 instructions a comparison (a compare, a select and an add
    // per comparison took 80 % of the kernel's VALU)
    typedef short sr_s2 __attribute__((ext_vector_type(2)));
    sr_s2 acc[8];
    sr_s2 kk[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        acc[j] = sr_s2{0, 0};
        kk[j] = sr_s2{(short)key[j], (short)key[j]};
    }
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        const uint4 q = keys[g][w];
        const uint32_t ws[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const sr_s2 a = __builtin_bit_cast(sr_s2, ws[h]);
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] -= (a - kk[j]) >> 15;
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t rank = (uint32_t)(uint16_t)acc[j].x + (uint32_t)(uint16_t)acc[j].y;
        if (key[j] != 0x7FFFu) row[1 + rank] = x[j];
    }
    sr_wave_fence();
    if (ok) {
        // block b of the row: tops of its 8 entries (four 16 B pieces), then their indices (two)
        uint4* out = reinterpret_cast<uint4*>(blks + sib_base + (uint64_t)(v - own_lo) * sbn);
        for (int p = r; p < sbn * 6; p += SR_G) {
            const int b = p / 6, w = p - 6 * (p / 6);
            uint4 val;
            if (w < 4) {
                const uint32_t e0 = row[b * KBLK + 2 * w], e1 = row[b * KBLK + 2 * w + 1];
                const uint64_t t0 = e0 == NONE ? ~0ull : tops[e0], t1 = e1 == NONE ? ~0ull : tops[e1];
                val = make_uint4((uint32_t)t0, (uint32_t)(t0 >> 32), (uint32_t)t1, (uint32_t)(t1 >> 32));
            } else {
                const int o = b * KBLK + 4 * (w - 4);
                val = make_uint4(row[o], row[o + 1], row[o + 2], row[o + 3]);
            }
            out[p] = val;
        }
    }

    // ---- the bucket m = endIndex (every lane of the group takes part in the shuffles) ----
    int m = -1;
    uint32_t boff = 0;
    if (ok) {
        const uint4* pn = reinterpret_cast<const uint4*>(nodes + v);
        boff = pn[1].y;
        m = kad_end(pn[3].z);
    }
    const bool act = m >= 0;                 // the same on the group's eight lanes
    uint32_t flo = 0, fhi = 0;
    if (act) kb_tm_range(recs, tops, tab, D, v, mt, m, flo, fhi);
    const uint32_t span = fhi - flo;
    // the siblings inside T_m: counted, and as a mask over T_m's first 256 nodes
    uint32_t nsin = 0;
    uint64_t mk[4] = {0ull, 0ull, 0ull, 0ull};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t xx = x[j];
        const bool in = xx != NONE && xx >= flo && xx < fhi;
        nsin += in ? 1u : 0u;
        const uint32_t o = xx - flo;
        const uint64_t bit = (in && o < 256) ? 1ull << (o & 63) : 0ull;
#pragma unroll
        for (int w = 0; w < 4; ++w) mk[w] |= (o >> 6) == (uint32_t)w ? bit : 0ull;
    }
#pragma unroll
    for (int s2 = 1; s2 < SR_G; s2 <<= 1) {
        nsin += __shfl_xor(nsin, s2, SR_G);
#pragma unroll
        for (int w = 0; w < 4; ++w) mk[w] |= __shfl_xor(mk[w], s2, SR_G);
    }
    const uint32_t c = span - nsin;
    // Floyd: lane r computes draws r, r + 8, ...; every lane gathers and resolves all of them
    constexpr int DPL = KC / SR_G;           // draws a lane
    uint32_t mine[DPL];
#pragma unroll
    for (int h = 0; h < DPL; ++h) mine[h] = act ? kb_floyd_draw(seed, v, m, c, k, r + SR_G * h) : NONE;
    uint32_t ch[KC];
#pragma unroll
    for (int i = 0; i < KC; ++i) ch[i] = __shfl(mine[i / SR_G], i % SR_G, SR_G);
    kb_floyd_resolve(ch, c, k);
    // this lane's members (ranks r, r + 8, ...) as node indices, and their tops
    uint32_t mem[DPL];
    uint64_t mtp[DPL];
    const auto valid = [&](int w) -> uint64_t {    // the bits of word w inside T_m
        const int b = (int)span - 64 * w;
        return b >= 64 ? ~0ull : b <= 0 ? 0ull : ((1ull << b) - 1);
    };
#pragma unroll
    for (int h = 0; h < DPL; ++h) {
        uint32_t rk = NONE;
#pragma unroll
        for (int i = 0; i < KC; ++i)
            if (i == r + SR_G * h) rk = ch[i];
        uint32_t xm = NONE;
        if (rk != NONE) {
            if (nsin == 0) {
                xm = flo + rk;
            } else if (span <= 256) {
                xm = flo + kb_nth_bit256(~mk[0] & valid(0), ~mk[1] & valid(1), ~mk[2] & valid(2), ~mk[3] & valid(3), rk);
            } else {
                // the least fixed point of x = flo + rank + #{siblings in [flo, x]} (row entries 1..S5)
                const uint32_t base = flo + rk;
                uint32_t xx = base;
                for (;;) {
                    uint32_t cs = 0;
                    for (int i = 1; i <= S5; ++i) {
                        const uint32_t y = row[i];
                        cs += (y != NONE && y >= flo && y <= xx) ? 1u : 0u;
                    }
                    if (base + cs == xx) break;
                    xx = base + cs;
                }
                xm = xx;
            }
        }
        mem[h] = xm;
        mtp[h] = xm == NONE ? ~0ull : tops[xm];
    }
    // the block(s): piece p of block b -- tops of entries 2p, 2p + 1 (p < 4), indices 4(p - 4) .. + 3
    const int bpb = (k + KBLK - 1) / KBLK;
#pragma unroll
    for (int b = 0; b < KC / KBLK; ++b) {
        uint32_t e[8];
        uint64_t t[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {        // entry b * 8 + q is lane q's member h = b
            e[q] = __shfl(mem[b], q, SR_G);
            t[q] = __shfl(mtp[b], q, SR_G);
        }
        if (act && b < bpb && r < 6) {
            uint4* dd = reinterpret_cast<uint4*>(blks + (uint64_t)boff + (uint64_t)(KEYBITS - 1 - m) * (uint64_t)bpb + b);
            uint4 val;
            if (r < 4) {
                uint64_t t0 = t[0], t1 = t[1];
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (q == r) { t0 = t[2 * q]; t1 = t[2 * q + 1]; }
                val = make_uint4((uint32_t)t0, (uint32_t)(t0 >> 32), (uint32_t)t1, (uint32_t)(t1 >> 32));
            } else {
                val = r == 4 ? make_uint4(e[0], e[1], e[2], e[3]) : make_uint4(e[4], e[5], e[6], e[7]);
            }
            dd[r] = val;
        }
    }
}

// sharded networks (KadTables::tl > 0): the top tl buckets m = 159 .. 160 - tl of EVERY node, at
// blks[(v * tl + (159 - m)) * bpb] -- the same members its owner's row holds (the same snapshot rule),
// so findNode(K) at any node whose main bucket m is one of them, lies above its sibling zone and is
// full can be answered on any rank (the kernels' virtual row offset v * tl * bpb).  The node line
// records which of them are full (KMETA_TOPFULL bits), which decides that at send time.
__global__ void k_kad_top_buckets(const KeyRec* __restrict__ recs, KadNode* __restrict__ nodes, uint32_t n, int k,
                                  int S5, uint64_t seed, const uint32_t* __restrict__ sib, KadBlk* __restrict__ blks,
                                  int tl)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const K160 me = kload(recs, v);
    const uint32_t* L = sib + (uint64_t)v * S5;
    const int endIndex = kad_end(nodes[v].meta);
    const int bpb = (k + KBLK - 1) / KBLK;
    uint32_t lo = 0, hi = n, full = 0;
    for (int m = KEYBITS - 1; m >= KEYBITS - tl; --m) {
        const uint32_t mid = split_bit(recs, lo, hi, m);
        const uint32_t nb = kbit(me, m);
        const uint32_t flo = nb ? lo : mid, fhi = nb ? mid : hi;
        const int j = KEYBITS - 1 - m;
        const uint64_t blk0 = ((uint64_t)v * (uint32_t)tl + (uint32_t)j) * (uint64_t)bpb;
        if (m >= endIndex) {
            const int cnt = kad_bucket_fill(recs, v, m, flo, fhi, L, 1, S5, k, seed, blks, blk0, m == endIndex);
            if (cnt >= k && m > endIndex) full |= 1u << j;
        } else {
            for (int q = 0; q < bpb * KBLK; ++q) put_entry(blks, blk0, q, NONE, recs);
        }
        lo = nb ? mid : lo;
        hi = nb ? hi : mid;
    }
    nodes[v].meta = (nodes[v].meta & ~KMETA_TOPFULL_ALL) | (full << KMETA_TOPFULL_SHIFT);
}

// explicit tables, pass A: validate a node's tables against the invariants OverSim's routingAdd
// keeps (Kademlia.cc:432-756): members are other nodes, a bucket m holds only nodes with
// msb(x ^ self) = m, no node twice, no node both sibling and bucket member; summary + row length
__global__ void k_kad_explicit_nodes(const KeyRec* __restrict__ recs, const double2* __restrict__ xy, uint32_t n,
                                     int k, int S5, uint32_t* __restrict__ sib, const uint8_t* __restrict__ bcount,
                                     const uint32_t* __restrict__ bnodes, KadNode* __restrict__ out, KadX* __restrict__ ox,
                                     uint64_t* __restrict__ rowlen, uint32_t* err, uint32_t* short_flag)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const K160 me = kload(recs, v);
    uint32_t* L = sib + (uint64_t)v * S5;
    // compact the sibling list (NONE entries may be anywhere)
    int cnt = 0;
    for (int i = 0; i < S5; ++i) {
        const uint32_t x = L[i];
        if (x == NONE) continue;
        L[cnt++] = x;
    }
    for (int i = cnt; i < S5; ++i) L[i] = NONE;
    uint32_t code = 0;
    for (int i = 0; i < cnt && !code; ++i) {
        if (L[i] >= n || L[i] == v) code = 1;
        for (int j = 0; j < i && !code; ++j) if (L[j] == L[i]) code = 2;
    }
    int lowest = -1;
    for (int m = 0; m < KEYBITS && !code; ++m) {
        const int c = bcount[(uint64_t)v * KEYBITS + m];
        if (c > k) { code = 3; break; }
        if (c && lowest < 0) lowest = m;
        const uint32_t* B = bnodes + ((uint64_t)v * KEYBITS + m) * k;
        for (int q = 0; q < c && !code; ++q) {
            const uint32_t x = B[q];
            if (x >= n || x == v) { code = 4; break; }
            if (k_msb(k_xor(kload(recs, x), me)) != m) { code = 5; break; }
            for (int j = 0; j < q; ++j) if (B[j] == x) code = 6;
            for (int i = 0; i < cnt; ++i) if (L[i] == x) code = 7;
        }
    }
    if (code) {
        if (atomicCAS(err, NONE, v) == NONE) err[1] = code;
        return;
    }
    K160 R{};
    for (int i = 0; i < 5; ++i) R.w[i] = 0;
    for (int i = 0; i < cnt; ++i) {
        const K160 d = k_xor(kload(recs, L[i]), me);
        if (k_gt(d, R)) R = d;
    }
    const int end = cnt > 0 ? k_msb(R) : -1;
    const int rowlo = end < 0 ? lowest : (lowest >= 0 && lowest < end ? lowest : end);
    kad_node_summary(recs, xy, v, L, cnt, rowlo, out, ox);
    rowlen[v] = rowlo >= 0 ? (uint64_t)(KEYBITS - rowlo) * (uint64_t)((k + KBLK - 1) / KBLK) : 0;
    if (cnt + 1 < 8) atomicOr(short_flag, 1u);
}

// explicit tables, pass B: bucket rows and sibling rows as blocks
__global__ void k_kad_explicit_rows(const KeyRec* __restrict__ recs, const KadNode* __restrict__ nodes, uint32_t n,
                                    int k, int S5, int sbn, const uint32_t* __restrict__ sib,
                                    const uint8_t* __restrict__ bcount, const uint32_t* __restrict__ bnodes,
                                    KadBlk* __restrict__ blks, uint64_t sib_base)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const KadNode r = nodes[v];
    const uint32_t* L = sib + (uint64_t)v * S5;
    put_sibling_row(blks, sib_base + (uint64_t)v * sbn, sbn, L, S5, v, kload(recs, v), recs);
    const int rowlo = kad_rowlo(r.meta);
    if (rowlo < 0) return;
    const int bpb = (k + KBLK - 1) / KBLK;
    for (int m = KEYBITS - 1; m >= rowlo; --m) {
        const uint64_t blk0 = (uint64_t)r.boff + (uint64_t)(KEYBITS - 1 - m) * (uint64_t)bpb;
        const int c = bcount[(uint64_t)v * KEYBITS + m];
        const uint32_t* B = bnodes + ((uint64_t)v * KEYBITS + m) * k;
        for (int q = 0; q < bpb * KBLK; ++q) put_entry(blks, blk0, q, q < c ? B[q] : NONE, recs);
    }
}

// general tables (CSR buckets), pass A: routingAdd's invariants under b and the bucket sizes
// (codes as k_kad_explicit_nodes; 3 = more than routingBucketSize(i), 5 = routingBucketIndex of the
// member is not the bucket's), the node summary, the bucket index of the farthest sibling
__global__ void k_kad_general_nodes(const KeyRec* __restrict__ recs, const double2* __restrict__ xy, uint32_t n, int S5,
                                    int b, int nb, const int* __restrict__ caps, uint32_t* __restrict__ sib,
                                    const uint32_t* __restrict__ off, const uint32_t* __restrict__ members,
                                    KadNode* __restrict__ out, KadX* __restrict__ ox, int16_t* __restrict__ gend,
                                    uint32_t* err, uint32_t* short_flag)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= n) return;
    const K160 me = kload(recs, v);
    uint32_t* L = sib + (uint64_t)v * S5;
    int cnt = 0;
    for (int i = 0; i < S5; ++i) {
        const uint32_t x = L[i];
        if (x == NONE) continue;
        L[cnt++] = x;
    }
    for (int i = cnt; i < S5; ++i) L[i] = NONE;
    uint32_t code = 0;
    for (int i = 0; i < cnt && !code; ++i) {
        if (L[i] >= n || L[i] == v) code = 1;
        for (int j = 0; j < i && !code; ++j) if (L[j] == L[i]) code = 2;
    }
    for (int m = 0; m < nb && !code; ++m) {
        const uint32_t a = off[(uint64_t)v * nb + m], z = off[(uint64_t)v * nb + m + 1];
        if (z < a) { code = 3; break; }
        if (caps[m] > 0 && z - a > (uint32_t)caps[m]) { code = 3; break; }
        for (uint32_t q = a; q < z && !code; ++q) {
            const uint32_t x = members[q];
            if (x >= n || x == v) { code = 4; break; }
            if (kad_bucket_index(k_xor(kload(recs, x), me), b, false) != m) { code = 5; break; }
            for (uint32_t j = a; j < q; ++j) if (members[j] == x) code = 6;
            for (int i = 0; i < cnt; ++i) if (L[i] == x) code = 7;
        }
    }
    if (code) {
        if (atomicCAS(err, NONE, v) == NONE) err[1] = code;
        return;
    }
    K160 R{};
    for (int i = 0; i < 5; ++i) R.w[i] = 0;
    for (int i = 0; i < cnt; ++i) {
        const K160 d = k_xor(kload(recs, L[i]), me);
        if (k_gt(d, R)) R = d;
    }
    // no 160-bucket rows: rowlo = -1
    kad_node_summary(recs, xy, v, L, cnt, -1, out, ox);
    gend[v] = (int16_t)(cnt > 0 ? kad_bucket_index(R, b, false) : -1);
    if (cnt + 1 < 8) atomicOr(short_flag, 1u);
}

__global__ void k_kad_general_tops(const KeyRec* __restrict__ recs, const uint32_t* __restrict__ members, uint64_t total,
                                   uint64_t* __restrict__ tops)
{
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < total) tops[e] = ktop(kload(recs, members[e]));
}

__global__ void k_kad_export(const KadNode* __restrict__ nodes, const KadBlk* __restrict__ blks, uint32_t n, int k,
                             uint8_t* __restrict__ bcount, uint32_t* __restrict__ bnodes)
{
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)n * KEYBITS) return;
    const uint32_t v = (uint32_t)(t / KEYBITS);
    const int m = (int)(t % KEYBITS);
    const KadNode r = nodes[v];
    const int rowlo = kad_rowlo(r.meta);
    int c = 0;
    uint32_t* o = bnodes + t * k;
    for (int q = 0; q < k; ++q) o[q] = NONE;
    if (rowlo >= 0 && m >= rowlo) {
        const int bpb = (k + KBLK - 1) / KBLK;
        const KadBlk* b = blks + (uint64_t)r.boff + (uint64_t)(KEYBITS - 1 - m) * (uint64_t)bpb;
        for (int q = 0; q < k; ++q) {
            const uint32_t x = b[q / KBLK].idx[q % KBLK];
            if (x == NONE) break;
            o[c++] = x;
        }
    }
    bcount[t] = (uint8_t)c;
}

// batched findNode (numRedundantNodes <= CAP, 1 <= numSiblings <= CAP, or numSiblings = -1: the call
// of an exhaustive-iterative lookup, resultSize = numRedundantNodes and no siblings flag,
// Kademlia.cc:1125-1127, BaseOverlay.cc:1857-1871) for the ABI.  CAP = 64: the responses of the
// sibling-table refresh (siblingRefreshNodes = 5s = 40) in maintenance rounds.
template <bool EX, int CAP>
__global__ void k_kad_find_node(KadView V, const uint32_t* __restrict__ node, const K160* __restrict__ keys, uint64_t n,
                                int numRedundant, int numSiblings, uint32_t* __restrict__ out_nodes, uint32_t max_out,
                                uint8_t* __restrict__ out_count, uint8_t* __restrict__ out_sib)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = node[i];
    const K160 K = keys[i];
    const KadNode r = load_node(V.nodes, c);
    const bool sb = numSiblings >= 0 && kad_is_sibling(V, r, c, K, numSiblings);
    SVec<CAP> res;
    const int cnt = kad_find_node_ins<CAP, EX>(V, c, resp_geo(r, K), K, numRedundant, sb, res, numSiblings);
    uint32_t* o = out_nodes + i * max_out;
    for (uint32_t j = 0; j < max_out; ++j) o[j] = NONE;
#pragma unroll
    for (int j = 0; j < CAP; ++j)
        if (j < cnt && (uint32_t)j < max_out) o[j] = res.idx[j];
    out_count[i] = (uint8_t)(cnt < (int)max_out ? cnt : (int)max_out);
    out_sib[i] = sb ? 1 : 0;
}

// ---------------------------------------------------------------------------
// host side

static inline unsigned nblk(uint64_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

// the level msb(x ^ v) of every sibling x of every node v (sharded networks, KadTables::slev)
__global__ void k_kad_sib_levels(const KadNode* __restrict__ nodes, const uint32_t* __restrict__ sib, uint32_t n,
                                 int S5, uint8_t* __restrict__ slev)
{
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= (uint64_t)n * S5) return;
    const uint32_t v = (uint32_t)(j / S5);
    const uint32_t x = sib[j];
    slev[j] = x == NONE ? 0xFFu : (uint8_t)k_msb(k_xor(as_key(nodes[x].key), as_key(nodes[v].key)));
}

static hipError_t kad_prefix_flag(const KeyRec* recs, uint32_t n, KadTables& t, hipStream_t st)
{
    uint32_t* tie = nullptr;
    uint32_t htie = 1;
    hipError_t e;
    if ((e = hipMalloc(&tie, sizeof(uint32_t))) != hipSuccess) return e;
    hipMemsetAsync(tie, 0, sizeof(uint32_t), st);
    if (n > 1) hipLaunchKernelGGL(k_kad_prefix_ties, dim3(nblk(n, 256)), dim3(256), 0, st, recs, n, tie);
    hipMemcpyAsync(&htie, tie, sizeof(uint32_t), hipMemcpyDeviceToHost, st);
    e = hipStreamSynchronize(st);
    hipFree(tie);
    if (e != hipSuccess) return e;
    t.exact = htie != 0 || getenv("OVS_KAD_EXACT") != nullptr;
    return hipSuccess;
}

hipError_t kad_build(const KeyRec* recs, const double2* xy, uint32_t n, int k, int s, uint64_t seed, KadTables& t,
                     hipStream_t st, uint32_t lo, uint32_t hi, int tl)
{
    hipError_t e;
    kad_free(t);
    if (hi > n) hi = n;
    if (lo >= hi) return hipErrorInvalidValue;
    t.k = k; t.s = s; t.seed = seed; t.lo = lo; t.hi = hi; t.snapshot = 1; t.maybe_short = 0;
    if (k < 1 || k > KMAX) return hipErrorNotSupported;
    if (tl < 0 || tl > KTOP_MAX) return hipErrorInvalidValue;
    const int bpb = (k + KBLK - 1) / KBLK;
    t.bpb = bpb;
    const int S5 = 5 * s, sbn = (S5 + 1 + KBLK - 1) / KBLK;   // the node + its siblings
    const uint32_t nown = hi - lo;
    uint64_t *rowlen = nullptr, *off = nullptr;
    uint32_t* sib_all = nullptr;
    uint64_t* tops = nullptr;
    void* tmp = nullptr;
    size_t tmpb = 0;
    auto cleanup = [&]() {
        if (rowlen) hipFree(rowlen);
        if (off) hipFree(off);
        if (tmp) hipFree(tmp);
        if (sib_all) hipFree(sib_all);
        if (tops) hipFree(tops);
    };
    // node lines for the whole network (a lookup needs every target's summary when it sends the
    // call); sibling lists are a build temporary
    if ((e = hipMalloc(&t.nodes, sizeof(KadNode) * n)) != hipSuccess) return e;
    if ((e = hipMalloc(&t.nodex, sizeof(KadX) * n)) != hipSuccess) return e;
    if ((e = hipMalloc(&sib_all, sizeof(uint32_t) * (uint64_t)n * S5)) != hipSuccess) return e;
    if ((e = hipMalloc(&rowlen, sizeof(uint64_t) * (n + 1))) != hipSuccess) { cleanup(); return e; }
    if ((e = hipMalloc(&off, sizeof(uint64_t) * (n + 1))) != hipSuccess) { cleanup(); return e; }
    // top-key array (8 B a node) and the prefix tables: read by the sibling, bucket and sibling-row builders
    int D = 1;
    while (D < KB_DMAX && (1ull << D) < 2ull * n) ++D;
    if ((e = hipMalloc(&tops, sizeof(uint64_t) * n + sizeof(uint32_t) * kb_tab_off(D + 1))) != hipSuccess) {
        cleanup();
        return e;
    }
    uint32_t* tab = reinterpret_cast<uint32_t*>(tops + n);
    hipLaunchKernelGGL(k_kad_tops, dim3(nblk(n, 256)), dim3(256), 0, st, recs, n, tops);
    hipLaunchKernelGGL(k_kad_prefix_tables, dim3(nblk(n, 256)), dim3(256), 0, st, tops, n, D, tab);
    int dg = 0;                                    // log2(n / (5s + 1)): the typical sibling-block depth
    while (dg < D && ((uint64_t)n >> (dg + 1)) >= (uint64_t)S5 + 1) ++dg;
    hipLaunchKernelGGL(k_kad_siblings, dim3(nblk(n, KS_BLOCK)), dim3(KS_BLOCK), 0, st, recs, xy, n, S5, bpb, lo, hi, tops, tab, D,
                       dg, sib_all, t.nodes, t.nodex, rowlen);
    hipMemsetAsync(rowlen + n, 0, sizeof(uint64_t), st);
    hipcub::DeviceScan::ExclusiveSum(nullptr, tmpb, rowlen, off, n + 1, st);
    if ((e = hipMalloc(&tmp, tmpb)) != hipSuccess) { cleanup(); return e; }
    hipcub::DeviceScan::ExclusiveSum(tmp, tmpb, rowlen, off, n + 1, st);
    uint64_t total = 0;
    hipMemcpyAsync(&total, off + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st);
    if ((e = hipStreamSynchronize(st)) != hipSuccess) { cleanup(); return e; }
    // the replicated top buckets of every node come first (the same offsets on every rank), then
    // the owned rows, then the owned sibling rows
    const uint64_t tend = (uint64_t)n * (uint32_t)tl * (uint32_t)bpb;
    if (total + tend >= 0xFFFFFFFFull) { cleanup(); return hipErrorInvalidValue; }
    t.tl = tl;
    t.tend = tend;
    t.rows_blks = tend + total;
    const uint64_t nblks = t.rows_blks + (uint64_t)nown * sbn + 1;
    if ((e = hipMalloc(&t.blks, sizeof(KadBlk) * nblks)) != hipSuccess) { cleanup(); return e; }
    hipLaunchKernelGGL(k_kad_set_boff, dim3(nblk(n, 256)), dim3(256), 0, st, t.nodes, off, lo, hi, tend, n);
    if ((e = hipMalloc(&t.sib, sizeof(uint32_t) * (uint64_t)nown * S5)) != hipSuccess) { cleanup(); return e; }
    hipMemcpyAsync(t.sib, sib_all + (uint64_t)lo * S5, sizeof(uint32_t) * (uint64_t)nown * S5, hipMemcpyDeviceToDevice, st);
    {
        if (S5 > 64 || sbn * KBLK > SR_ROW) { cleanup(); return hipErrorInvalidValue; }
        // (the sibling rows and sibling buckets on a second stream beside the bucket rows measured no
        // faster: all three are bound by gathers and stretched each other)
        const dim3 grid = kb_rows_grid(nown), blk(256), grid1(nblk(nown, SR_NPB));
        if (k <= KBLK) {
            hipLaunchKernelGGL(k_kad_sib_rows<KBLK>, grid1, blk, 0, st, recs, tops, tab, D, t.nodes, k, seed, S5, sbn,
                               sib_all, t.blks, t.rows_blks, lo, hi);
            hipLaunchKernelGGL(k_kad_bucket_rows<KBLK>, grid, blk, 0, st, recs, tops, tab, D, t.nodes, k, seed, t.blks,
                               lo, hi);
        } else {
            hipLaunchKernelGGL(k_kad_sib_rows<2 * KBLK>, grid1, blk, 0, st, recs, tops, tab, D, t.nodes, k, seed, S5,
                               sbn, sib_all, t.blks, t.rows_blks, lo, hi);
            hipLaunchKernelGGL(k_kad_bucket_rows<2 * KBLK>, grid, blk, 0, st, recs, tops, tab, D, t.nodes, k, seed,
                               t.blks, lo, hi);
        }
    }
    if (tl > 0)
        hipLaunchKernelGGL(k_kad_top_buckets, dim3(nblk(n, 64)), dim3(64), 0, st, recs, t.nodes, n, k, S5, seed, sib_all,
                           t.blks, tl);
    if (lo != 0 || hi != n) {
        if ((e = hipMalloc(&t.slev, (uint64_t)n * S5)) != hipSuccess) { cleanup(); return e; }
        hipLaunchKernelGGL(k_kad_sib_levels, dim3(nblk((uint64_t)n * S5, 256)), dim3(256), 0, st, t.nodes, sib_all, n,
                           S5, t.slev);
    }
    e = hipStreamSynchronize(st);
    cleanup();
    if (e != hipSuccess) return e;
    if ((e = kad_prefix_flag(recs, n, t, st)) != hipSuccess) return e;
    return hipGetLastError();
}

hipError_t kad_build_explicit(const KeyRec* recs, const double2* xy, uint32_t n, int k, int s, const uint32_t* sib,
                              const uint8_t* bcount, const uint32_t* bnodes, KadTables& t, uint32_t* bad_node,
                              uint32_t* bad_code, hipStream_t st)
{
    hipError_t e;
    kad_free(t);
    t.k = k; t.s = s; t.seed = 0; t.lo = 0; t.hi = n; t.snapshot = 0;
    if (k < 1 || k > KMAX) return hipErrorNotSupported;
    t.bpb = (k + KBLK - 1) / KBLK;
    const int S5 = 5 * s, sbn = (S5 + 1 + KBLK - 1) / KBLK;   // the node + its siblings
    uint64_t *rowlen = nullptr, *off = nullptr;
    uint32_t* flags = nullptr;
    void* tmp = nullptr;
    size_t tmpb = 0;
    auto cleanup = [&]() {
        if (rowlen) hipFree(rowlen);
        if (off) hipFree(off);
        if (tmp) hipFree(tmp);
        if (flags) hipFree(flags);
    };
    if ((e = hipMalloc(&t.nodes, sizeof(KadNode) * n)) != hipSuccess) return e;
    if ((e = hipMalloc(&t.nodex, sizeof(KadX) * n)) != hipSuccess) return e;
    if ((e = hipMalloc(&t.sib, sizeof(uint32_t) * (uint64_t)n * S5)) != hipSuccess) return e;
    hipMemcpyAsync(t.sib, sib, sizeof(uint32_t) * (uint64_t)n * S5, hipMemcpyDeviceToDevice, st);
    if ((e = hipMalloc(&rowlen, sizeof(uint64_t) * (n + 1))) != hipSuccess) { cleanup(); return e; }
    if ((e = hipMalloc(&off, sizeof(uint64_t) * (n + 1))) != hipSuccess) { cleanup(); return e; }
    if ((e = hipMalloc(&flags, sizeof(uint32_t) * 3)) != hipSuccess) { cleanup(); return e; }
    const uint32_t init[3] = {NONE, 0u, 0u};
    hipMemcpyAsync(flags, init, sizeof init, hipMemcpyHostToDevice, st);
    hipLaunchKernelGGL(k_kad_explicit_nodes, dim3(nblk(n, 128)), dim3(128), 0, st, recs, xy, n, k, S5, t.sib,
                       bcount, bnodes, t.nodes, t.nodex, rowlen, flags, flags + 2);
    uint32_t hf[3] = {0, 0, 0};
    hipMemcpyAsync(hf, flags, sizeof hf, hipMemcpyDeviceToHost, st);
    if ((e = hipStreamSynchronize(st)) != hipSuccess) { cleanup(); return e; }
    if (hf[0] != NONE) {
        *bad_node = hf[0];
        *bad_code = hf[1];
        cleanup();
        return hipErrorInvalidValue;
    }
    t.maybe_short = hf[2] != 0;
    hipMemsetAsync(rowlen + n, 0, sizeof(uint64_t), st);
    hipcub::DeviceScan::ExclusiveSum(nullptr, tmpb, rowlen, off, n + 1, st);
    if ((e = hipMalloc(&tmp, tmpb)) != hipSuccess) { cleanup(); return e; }
    hipcub::DeviceScan::ExclusiveSum(tmp, tmpb, rowlen, off, n + 1, st);
    uint64_t total = 0;
    hipMemcpyAsync(&total, off + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st);
    if ((e = hipStreamSynchronize(st)) != hipSuccess) { cleanup(); return e; }
    if (total >= 0xFFFFFFFFull) { cleanup(); return hipErrorInvalidValue; }
    t.rows_blks = total;
    if ((e = hipMalloc(&t.blks, sizeof(KadBlk) * (total + (uint64_t)n * sbn + 1))) != hipSuccess) { cleanup(); return e; }
    hipLaunchKernelGGL(k_kad_set_boff, dim3(nblk(n, 256)), dim3(256), 0, st, t.nodes, off, 0u, n, 0ull, n);
    hipLaunchKernelGGL(k_kad_explicit_rows, dim3(nblk(n, 64)), dim3(64), 0, st, recs, t.nodes, n, k, S5, sbn,
                       t.sib, bcount, bnodes, t.blks, t.rows_blks);
    e = hipStreamSynchronize(st);
    cleanup();
    if (e != hipSuccess) return e;
    if ((e = kad_prefix_flag(recs, n, t, st)) != hipSuccess) return e;
    return hipGetLastError();
}

hipError_t kad_build_general(const KeyRec* recs, const double2* xy, uint32_t n, int k, int s, int b, const int* caps,
                             const uint32_t* sib, const uint32_t* off, const uint32_t* members, uint64_t total,
                             KadTables& t, uint32_t* bad_node, uint32_t* bad_code, hipStream_t st)
{
    hipError_t e;
    kad_free(t);
    t.k = k; t.s = s; t.seed = 0; t.lo = 0; t.hi = n; t.snapshot = 0; t.general = 1;
    t.b = b; t.nb = (int)(((1 << b) - 1) * (KEYBITS / b));
    if (k < 1 || k > KMAX || b < 1 || b > 5) return hipErrorNotSupported;
    t.bpb = (k + KBLK - 1) / KBLK;
    const int S5 = 5 * s, sbn = (S5 + 1 + KBLK - 1) / KBLK;
    const uint64_t dir = (uint64_t)n * t.nb + 1;
    uint32_t* flags = nullptr;
    int* dcaps = nullptr;
    auto cleanup = [&]() {
        if (flags) hipFree(flags);
        if (dcaps) hipFree(dcaps);
    };
    if ((e = hipMalloc(&t.nodes, sizeof(KadNode) * n)) != hipSuccess) return e;
    if ((e = hipMalloc(&t.nodex, sizeof(KadX) * n)) != hipSuccess) return e;
    if ((e = hipMalloc(&t.sib, sizeof(uint32_t) * (uint64_t)n * S5)) != hipSuccess) return e;
    if ((e = hipMalloc(&t.goff, sizeof(uint32_t) * dir)) != hipSuccess) return e;
    if ((e = hipMalloc(&t.gidx, sizeof(uint32_t) * (total ? total : 1))) != hipSuccess) return e;
    if ((e = hipMalloc(&t.gtop, sizeof(uint64_t) * (total ? total : 1))) != hipSuccess) return e;
    if ((e = hipMalloc(&t.gend, sizeof(int16_t) * n)) != hipSuccess) return e;
    if ((e = hipMalloc(&flags, sizeof(uint32_t) * 3)) != hipSuccess) { cleanup(); return e; }
    if ((e = hipMalloc(&dcaps, sizeof(int) * t.nb)) != hipSuccess) { cleanup(); return e; }
    t.gtotal = total;
    hipMemcpyAsync(t.sib, sib, sizeof(uint32_t) * (uint64_t)n * S5, hipMemcpyDeviceToDevice, st);
    hipMemcpyAsync(t.goff, off, sizeof(uint32_t) * dir, hipMemcpyDeviceToDevice, st);
    if (total) hipMemcpyAsync(t.gidx, members, sizeof(uint32_t) * total, hipMemcpyDeviceToDevice, st);
    hipMemcpyAsync(dcaps, caps, sizeof(int) * t.nb, hipMemcpyHostToDevice, st);
    const uint32_t init[3] = {NONE, 0u, 0u};
    hipMemcpyAsync(flags, init, sizeof init, hipMemcpyHostToDevice, st);
    hipLaunchKernelGGL(k_kad_general_nodes, dim3(nblk(n, 128)), dim3(128), 0, st, recs, xy, n, S5, b, t.nb, dcaps, t.sib,
                       t.goff, t.gidx, t.nodes, t.nodex, t.gend, flags, flags + 2);
    uint32_t hf[3] = {0, 0, 0};
    hipMemcpyAsync(hf, flags, sizeof hf, hipMemcpyDeviceToHost, st);
    if ((e = hipStreamSynchronize(st)) != hipSuccess) { cleanup(); return e; }
    if (hf[0] != NONE) {
        *bad_node = hf[0];
        *bad_code = hf[1];
        cleanup();
        return hipErrorInvalidValue;
    }
    t.maybe_short = hf[2] != 0;
    if (total)
        hipLaunchKernelGGL(k_kad_general_tops, dim3(nblk(total, 256)), dim3(256), 0, st, recs, t.gidx, total, t.gtop);
    // the sibling rows (level-sorted, the node first) as blocks: isSiblingFor(numSiblings > 1) and
    // findNode's sibling part read them as on the 160-bucket tables; no bucket rows (rowlo = -1)
    t.rows_blks = 0;
    if ((e = hipMalloc(&t.blks, sizeof(KadBlk) * ((uint64_t)n * sbn + 1))) != hipSuccess) { cleanup(); return e; }
    hipLaunchKernelGGL(k_kad_explicit_rows, dim3(nblk(n, 64)), dim3(64), 0, st, recs, t.nodes, n, k, S5, sbn, t.sib,
                       (const uint8_t*)nullptr, (const uint32_t*)nullptr, t.blks, (uint64_t)0);
    e = hipStreamSynchronize(st);
    cleanup();
    if (e != hipSuccess) return e;
    if ((e = kad_prefix_flag(recs, n, t, st)) != hipSuccess) return e;
    return hipGetLastError();
}

hipError_t kad_export(const KadTables& t, uint32_t n, uint32_t* siblings, uint8_t* bucket_count, uint32_t* bucket_nodes,
                      hipStream_t st)
{
    hipError_t e;
    const int S5 = 5 * t.s;
    uint8_t* dc = nullptr;
    uint32_t* dn = nullptr;
    const uint64_t tot = (uint64_t)n * KEYBITS;
    if ((e = hipMalloc(&dc, tot)) != hipSuccess) return e;
    if ((e = hipMalloc(&dn, sizeof(uint32_t) * tot * t.k)) != hipSuccess) { hipFree(dc); return e; }
    hipLaunchKernelGGL(k_kad_export, dim3(nblk(tot, 256)), dim3(256), 0, st, t.nodes, t.blks, n, t.k, dc, dn);
    hipMemcpyAsync(bucket_count, dc, tot, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(bucket_nodes, dn, sizeof(uint32_t) * tot * t.k, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(siblings, t.sib, sizeof(uint32_t) * (uint64_t)n * S5, hipMemcpyDeviceToHost, st);
    e = hipStreamSynchronize(st);
    hipFree(dc); hipFree(dn);
    return e;
}

hipError_t kad_route(const KadTables& t, const double2* xy, uint32_t n, const ovs_params& P, const DelayConsts& DC,
                     const K160* qkeys, const uint32_t* qsrc, uint64_t nq, ovs_route_out* out, uint32_t* hopseq,
                     uint32_t* rpcs, int num_cu, hipStream_t st, uint32_t* sibs, unsigned long long* dyn)
{
    if (nq == 0) return hipSuccess;
    if (!kad_params_supported(P, t)) return hipErrorNotSupported;
    KadLC LC = kad_make_lc(P, t);
    kad_lc_sizes(LC, DC, n);
    const KadView V = kad_make_view(t, xy, n);
    // strictParallelRpcs: never more than alpha FindNodeCalls in flight (IterativeLookup.cc:1078-1079)
    const int A = P.lookupParallelRpcs;
    // LookupCall batches (sibs != nullptr) record no hop sequence
    if (sibs && hopseq) return hipErrorNotSupported;
#define KLX(a, x) kad_route_launch<a, x>(V, DC, LC, qkeys, qsrc, nq, out, hopseq, rpcs, sibs, num_cu, st, dyn)
#define KL(a) (t.exact ? KLX(a, true) : KLX(a, false))
    switch (A) {
    case 1: return KL(1);
    case 2: return KL(2);
    case 3: return KL(3);
    case 4: return KL(4);
    default: return KL(8);     // 5..8: A is the pending-call capacity (kad_params_supported)
    }
#undef KL
#undef KLX
}

hipError_t kad_find_node(const KadTables& t, uint32_t n, const ovs_params& P, const uint32_t* node, const K160* keys,
                         uint64_t nq, int numRedundant, int numSiblings, uint32_t* out_nodes, uint32_t max_out,
                         uint8_t* out_count, uint8_t* out_sib, hipStream_t st)
{
    (void)P;
    if (nq == 0) return hipSuccess;
    if ((numSiblings < 1 && numSiblings != -1) || numSiblings > 64 || numRedundant > 64) return hipErrorNotSupported;
    const KadView V = kad_make_view(t, nullptr, n);
    const bool wide = numSiblings > 16 || numRedundant > 16;
#define KFN(ex, cap) hipLaunchKernelGGL((k_kad_find_node<ex, cap>), dim3(nblk(nq, 128)), dim3(128), 0, st, V, node, keys, nq, \
                                        numRedundant, numSiblings, out_nodes, max_out, out_count, out_sib)
    if (t.exact) { if (wide) KFN(true, 64); else KFN(true, 16); }
    else { if (wide) KFN(false, 64); else KFN(false, 16); }
#undef KFN
    return hipGetLastError();
}

}  // namespace ovs
