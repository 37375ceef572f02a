// stats.hpp -- KBRTestApp statistics reduction (internal).
#pragma once
#include "engine.hpp"

namespace ovs {

constexpr int NSTAT = 5;                // delivered msg/s, delivered B/s, dropped msg/s, dropped B/s, ratio
constexpr int STATS_NODE_BLOCKS = 512;  // fixed grid of the per-node pass (deterministic fp64 sums)

// device-side integer counters of pass 1
struct StatsDev {
    unsigned long long delivered, dropped, failed, hop_sum, lat_sum, fhop_sum;
    unsigned long long hop_min, hop_max, lat_min, lat_max;
    unsigned long long status[8];
    unsigned long long hist[64];
};

// node_counts: 3 * nnodes u32 scratch; partial: STATS_NODE_BLOCKS * NSTAT * 5 doubles;
// result: NSTAT * 5 doubles {sum, sqrsum, min, max, count(bit pattern)} per statistic.
// first != nullptr: lookup test (out holds ovs_lookup_out, first[i * first_stride] = siblings[0]).
hipError_t launch_stats(const ovs_route_out* out, const K160* keys, const uint32_t* src, const KeyRec* recs,
                        uint64_t n, uint32_t nnodes, int lookup_node_ids, double time_s, uint64_t msg_bytes,
                        int rates, StatsDev* S, uint32_t* node_counts, double* partial, double* result,
                        int num_cu, hipStream_t st, const uint32_t* first = nullptr, uint64_t first_stride = 0);

}  // namespace ovs
