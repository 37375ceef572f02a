/* Prints the layout of every struct in include/ovs_kbr.h as JSON, compiled by a plain C
 * compiler against the header alone (tests/test_abi_layout.py compares it with the Python
 * mirrors in oversim_amd/kbr.py and oversim_amd/shard.py). */
#include <stddef.h>
#include <stdio.h>

#include "ovs_kbr.h"

static int first_struct = 1, first_field;

static void begin(const char* name, size_t size)
{
    printf("%s\"%s\": {\"size\": %zu, \"fields\": {", first_struct ? "" : ", ", name, size);
    first_struct = 0;
    first_field = 1;
}

static void field(const char* name, size_t off)
{
    printf("%s\"%s\": %zu", first_field ? "" : ", ", name, off);
    first_field = 0;
}

static void end(void) { printf("}}"); }

#define S(T) begin(#T, sizeof(T))
#define F(T, f) field(#f, offsetof(T, f))

int main(void)
{
    printf("{");
    S(ovs_key160); F(ovs_key160, w); end();
    S(ovs_params);
    F(ovs_params, overlay); F(ovs_params, keyLength); F(ovs_params, hopCountMax); F(ovs_params, successorListSize);
    F(ovs_params, extendedFingerTable); F(ovs_params, numFingerCandidates); F(ovs_params, k); F(ovs_params, s);
    F(ovs_params, b); F(ovs_params, lookupRedundantNodes); F(ovs_params, lookupParallelPaths);
    F(ovs_params, lookupParallelRpcs); F(ovs_params, lookupMerge); F(ovs_params, lookupStrictParallelRpcs);
    F(ovs_params, lookupVisitOnlyOnce); F(ovs_params, lookupAcceptLateSiblings);
    F(ovs_params, lookupUseAllParallelResponses); F(ovs_params, lookupNewRpcOnEveryTimeout);
    F(ovs_params, lookupNewRpcOnEveryResponse); F(ovs_params, lookupFinishOnFirstUnchanged);
    F(ovs_params, lookupVerifySiblings); F(ovs_params, lookupMajoritySiblings); F(ovs_params, routingType);
    F(ovs_params, numSiblings); F(ovs_params, useCoordinateBasedDelay); F(ovs_params, simtimeRound);
    F(ovs_params, testMsgSize); F(ovs_params, recNumRedundantNodes); F(ovs_params, rpcUdpTimeout);
    F(ovs_params, lookupTimeout); F(ovs_params, jitter); F(ovs_params, constantDelay); F(ovs_params, datarate);
    F(ovs_params, accessDelay); F(ovs_params, kadSeed); F(ovs_params, shiftingBits);
    F(ovs_params, deBruijnListSize); F(ovs_params, useOtherLookup); F(ovs_params, useSucList);
    F(ovs_params, bucketType); F(ovs_params, cacheTTL);
    F(ovs_params, globalNodeLimit); F(ovs_params, extraNodesFinalBucket); F(ovs_params, rpcKeyTimeout);
    F(ovs_params, measureAuthBlock);
    end();
    S(ovs_koorde_ext);
    F(ovs_koorde_ext, route_key); F(ovs_koorde_ext, step); F(ovs_koorde_ext, has_route_key);
    end();
    S(ovs_route_out);
    F(ovs_route_out, responsible); F(ovs_route_out, hops); F(ovs_route_out, status); F(ovs_route_out, one_way_hops);
    F(ovs_route_out, latency_ns);
    end();
    S(ovs_lookup_out);
    F(ovs_lookup_out, num_siblings); F(ovs_lookup_out, hops); F(ovs_lookup_out, status); F(ovs_lookup_out, is_valid);
    F(ovs_lookup_out, latency_ns);
    end();
    S(ovs_fixfingers_stats);
    F(ovs_fixfingers_stats, lookups); F(ovs_fixfingers_stats, ok); F(ovs_fixfingers_stats, changed);
    F(ovs_fixfingers_stats, hops);
    end();
    S(ovs_stabilize_stats);
    F(ovs_stabilize_stats, nodes); F(ovs_stabilize_stats, succ_changed); F(ovs_stabilize_stats, lists_changed);
    F(ovs_stabilize_stats, pred_changed);
    end();
    S(ovs_stddev);
    F(ovs_stddev, count); F(ovs_stddev, mean); F(ovs_stddev, stddev); F(ovs_stddev, min); F(ovs_stddev, max);
    end();
    S(ovs_kbrtest_stats);
    F(ovs_kbrtest_stats, num_sent); F(ovs_kbrtest_stats, num_delivered); F(ovs_kbrtest_stats, num_dropped);
    F(ovs_kbrtest_stats, num_lookup_failed); F(ovs_kbrtest_stats, bytes_sent); F(ovs_kbrtest_stats, bytes_delivered);
    F(ovs_kbrtest_stats, bytes_dropped); F(ovs_kbrtest_stats, hop_count_sum); F(ovs_kbrtest_stats, latency_sum_ns);
    F(ovs_kbrtest_stats, hop_count_min); F(ovs_kbrtest_stats, hop_count_max); F(ovs_kbrtest_stats, latency_min_ns);
    F(ovs_kbrtest_stats, latency_max_ns); F(ovs_kbrtest_stats, hop_count_mean); F(ovs_kbrtest_stats, latency_mean_s);
    F(ovs_kbrtest_stats, status_count); F(ovs_kbrtest_stats, hop_hist); F(ovs_kbrtest_stats, delivered_msgs_per_s);
    F(ovs_kbrtest_stats, delivered_bytes_per_s); F(ovs_kbrtest_stats, dropped_msgs_per_s);
    F(ovs_kbrtest_stats, dropped_bytes_per_s); F(ovs_kbrtest_stats, delivery_ratio);
    end();
    S(ovs_kbrtest_lookup_stats);
    F(ovs_kbrtest_lookup_stats, num_sent); F(ovs_kbrtest_lookup_stats, num_success);
    F(ovs_kbrtest_lookup_stats, num_failed); F(ovs_kbrtest_lookup_stats, num_invalid);
    F(ovs_kbrtest_lookup_stats, hop_count_sum); F(ovs_kbrtest_lookup_stats, failed_hop_count_sum);
    F(ovs_kbrtest_lookup_stats, success_latency_sum_ns); F(ovs_kbrtest_lookup_stats, hop_count_min);
    F(ovs_kbrtest_lookup_stats, hop_count_max); F(ovs_kbrtest_lookup_stats, success_latency_min_ns);
    F(ovs_kbrtest_lookup_stats, success_latency_max_ns); F(ovs_kbrtest_lookup_stats, hop_count_mean);
    F(ovs_kbrtest_lookup_stats, failed_hop_count_mean); F(ovs_kbrtest_lookup_stats, success_latency_mean_s);
    F(ovs_kbrtest_lookup_stats, total_latency_mean_s); F(ovs_kbrtest_lookup_stats, status_count);
    F(ovs_kbrtest_lookup_stats, hop_hist); F(ovs_kbrtest_lookup_stats, successful_lookups_per_s);
    F(ovs_kbrtest_lookup_stats, failed_lookups_per_s); F(ovs_kbrtest_lookup_stats, success_ratio);
    end();
    S(ovs_lookup_rec);
    F(ovs_lookup_rec, key); F(ovs_lookup_rec, src); F(ovs_lookup_rec, cur); F(ovs_lookup_rec, qid);
    F(ovs_lookup_rec, t_ns); F(ovs_lookup_rec, hops); F(ovs_lookup_rec, local); F(ovs_lookup_rec, pad);
    end();
    S(ovs_done_rec);
    F(ovs_done_rec, qid); F(ovs_done_rec, pad); F(ovs_done_rec, out);
    end();
    S(ovs_kad_req);
    F(ovs_kad_req, key); F(ovs_kad_req, node); F(ovs_kad_req, tag); F(ovs_kad_req, pad);
    end();
    S(ovs_kad_resp);
    F(ovs_kad_resp, tag); F(ovs_kad_resp, count); F(ovs_kad_resp, nodes); F(ovs_kad_resp, dist_hi);
    end();
    S(ovs_kad_resp16);
    F(ovs_kad_resp16, tag); F(ovs_kad_resp16, count); F(ovs_kad_resp16, nodes); F(ovs_kad_resp16, dist_hi);
    end();
    printf("}\n");
    return 0;
}
