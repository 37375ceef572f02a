// compact.hpp -- stable compaction of per-element stage records by class tag (internal).
//
// The multi-GPU step kernels give every input element exactly one outcome (a finished lookup, a
// hand-off to arc d, a FindNodeCall to rank d, ...) and write it to a stage slot indexed by the
// element plus a one-byte class tag, with no atomics: a result-returning atomic on one counter
// from every wave of all 8 XCDs made the Chord shard step 9x slower than the single-GPU route
// (tools/diag/chord_ab.sh).  compact_by_tag then moves each class's records, in element order,
// to that class's output: a per-tile class count, one exclusive scan over (class, tile), and a
// scatter that ranks the elements of a tile within their class with ballots.
#pragma once
#include "engine.hpp"

namespace ovs {

// one output class
struct CClass {
    const uint8_t* src;            // stage records, element i at src + i * src_stride
    uint8_t* dst;                  // nullptr: the class is only counted
    uint32_t* lab;                 // optional: lab[pos] = label for every record written
    unsigned long long* counter;   // position of the class's first record (read), then + its total
                                   // (written); nullptr = 0 (a chained class has none)
    uint64_t cap;                  // records dst holds (later ones are counted, not written)
    uint32_t src_stride, rec_bytes, label;
    int chain;                     // 1: continues the previous class in the same dst and counter
};

// The classes of one compaction, small enough to travel as a kernel argument: n per-destination
// classes 0..n-1 sharing a stage array (chained into one dst with labels d, or segment d at
// dst + d * dst_stride with counter + d), then up to two explicit classes.
struct CSeg {
    const uint8_t* src;
    uint8_t* dst;
    uint32_t* lab;
    unsigned long long* counter;
    uint64_t cap, dst_stride;
    uint32_t src_stride, rec_bytes;
    int n, chain;
};
struct CPlan {
    CSeg seg;
    int nextra;
    CClass extra[2];
};

__host__ __device__ inline CClass plan_class(const CPlan& P, int c)
{
    if (c >= P.seg.n) return P.extra[c - P.seg.n];
    CClass k{};
    k.src = P.seg.src; k.src_stride = P.seg.src_stride; k.rec_bytes = P.seg.rec_bytes; k.cap = P.seg.cap;
    if (P.seg.chain) {
        k.dst = P.seg.dst; k.lab = P.seg.lab; k.label = (uint32_t)c;
        k.counter = c == 0 ? P.seg.counter : nullptr; k.chain = c > 0;
    } else {
        k.dst = P.seg.dst ? P.seg.dst + (uint64_t)c * P.seg.dst_stride : nullptr;
        k.counter = P.seg.counter ? P.seg.counter + c : nullptr;
    }
    return k;
}
constexpr int CMAX = MAXSHARDS + 2;   // classes of one compaction

struct CompactScratch {
    void* buf = nullptr;
    size_t bytes = 0;
};
void compact_free(CompactScratch& s);

// per-stream stage records + compaction scratch of the shard step launchers (one per stream:
// the cohorts of a rank step concurrently on their own streams)
struct StageBuf {
    void* buf = nullptr;
    size_t bytes = 0;
    CompactScratch cs;
};
void stage_free(StageBuf& b);
// b.buf holds at least `bytes` (grown after the stream drained)
hipError_t stage_ensure(StageBuf& b, size_t bytes, hipStream_t s);

// tags[i] < the plan's class count selects the class of element i (other values: no output);
// stream-ordered, no host synchronisation
// out = the finished records of done[0, n) with qid 0xFFFFFFFF (exchange rows nobody wrote)
hipError_t count_sentinel_records(const ovs_done_rec* done, uint64_t n, unsigned long long* out, hipStream_t s);

hipError_t compact_by_tag(const uint8_t* tags, uint64_t n, const CPlan& plan, CompactScratch& scr, hipStream_t s);

}  // namespace ovs
