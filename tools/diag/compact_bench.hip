// Micro-benchmark of the stable compaction by tag (oversim_amd/csrc/compact.hip) on the shape of
// a Chord shard step's first round at W = 8: 10M stage records of 48 B (hand-offs, 88 % of the
// lookups, spread over the 7 other arcs) and 24 B done records (12 %).  Prints the compaction's
// average time, a D2D copy of the same bytes for scale, and a hash of the outputs (equal across
// variants of the kernels).  Built by tools/diag/compact_bench.sh; one GPU.
#include "../../oversim_amd/csrc/compact.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace ovs;

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

static uint64_t splitmix(uint64_t& s)
{
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main(int argc, char** argv)
{
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 10000000ull;
    const int W = 8, me = 3, reps = 20;
    std::vector<uint8_t> tags(n);
    uint64_t s = 12345;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t r = splitmix(s);
        if (r % 100 < 12) tags[i] = (uint8_t)W;     // done
        else {
            int d = (int)((r >> 8) % (W - 1));
            tags[i] = (uint8_t)(d >= me ? d + 1 : d);
        }
    }
    uint8_t *dtags, *hand, *done, *seg, *dout;
    unsigned long long* cnt;
    CK(hipMalloc(&dtags, n));
    CK(hipMalloc(&hand, n * 48));
    CK(hipMalloc(&done, n * 24));
    CK(hipMalloc(&seg, (uint64_t)W * n * 48));
    CK(hipMalloc(&dout, n * 24));
    CK(hipMalloc(&cnt, 16 * sizeof(unsigned long long)));
    CK(hipMemcpy(dtags, tags.data(), n, hipMemcpyHostToDevice));
    {
        std::vector<uint32_t> w(n * 12);
        for (auto& x : w) x = (uint32_t)splitmix(s);
        CK(hipMemcpy(hand, w.data(), n * 48, hipMemcpyHostToDevice));
        CK(hipMemcpy(done, w.data(), n * 24, hipMemcpyHostToDevice));
    }
    CPlan P{};
    P.seg.src = hand; P.seg.dst = seg; P.seg.lab = nullptr; P.seg.counter = cnt; P.seg.cap = n;
    P.seg.dst_stride = n * 48; P.seg.src_stride = 48; P.seg.rec_bytes = 48; P.seg.n = W; P.seg.chain = 0;
    P.nextra = 1;
    P.extra[0].src = done; P.extra[0].dst = dout; P.extra[0].lab = nullptr; P.extra[0].counter = cnt + W;
    P.extra[0].cap = n; P.extra[0].src_stride = 24; P.extra[0].rec_bytes = 24; P.extra[0].label = 0; P.extra[0].chain = 0;
    CompactScratch scr;
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e9, tot = 0;
    for (int r = 0; r < reps + 2; ++r) {
        CK(hipMemsetAsync(cnt, 0, 16 * sizeof(unsigned long long), st));
        CK(hipEventRecord(a, st));
        CK(compact_by_tag(dtags, n, P, scr, st));
        CK(hipEventRecord(b, st));
        CK(hipStreamSynchronize(st));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r >= 2) { tot += ms; best = ms < best ? ms : best; }
    }
    // outputs: counts and an FNV hash of every class's records
    unsigned long long hc[16];
    CK(hipMemcpy(hc, cnt, sizeof(hc), hipMemcpyDeviceToHost));
    uint64_t h = 1469598103934665603ull, moved = 0;
    for (int c = 0; c <= W; ++c) {
        const uint64_t bytes = c < W ? hc[c] * 48 : hc[W] * 24;
        moved += bytes;
        std::vector<uint8_t> v(bytes);
        CK(hipMemcpy(v.data(), c < W ? seg + (uint64_t)c * n * 48 : dout, bytes, hipMemcpyDeviceToHost));
        for (uint8_t x : v) h = (h ^ x) * 1099511628211ull;
    }
    // a D2D copy of the bytes moved, for scale
    float cms = 0;
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(a, st));
        CK(hipMemcpyAsync(seg, hand, moved, hipMemcpyDeviceToDevice, st));
        CK(hipEventRecord(b, st));
        CK(hipStreamSynchronize(st));
        CK(hipEventElapsedTime(&cms, a, b));
    }
    printf("{\"batch\": %d, \"steps\": %d, \"n\": %llu, \"ms_avg\": %.4f, \"ms_best\": %.4f, "
           "\"moved_bytes\": %llu, \"GBps\": %.1f, \"d2d_copy_ms\": %.4f, \"hash\": \"%016llx\"}\n",
           CT_BATCH, CT_STEPS, (unsigned long long)n, tot / reps, best, (unsigned long long)moved,
           2.0 * moved / (tot / reps) / 1e6, cms, (unsigned long long)h);
    return 0;
}
