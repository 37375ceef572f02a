// ctx_internal.hpp -- what the host layers outside ovs_kbr.cpp may use of a context (internal).
//
// The sharded round loop (shard_route.cpp) drives a context through the public ABI; these give it
// the context's device, its error slot, cohort streams the context owns (the shard step keeps its
// stage records per stream, so the streams must live as long as the context) and one cached
// scratch object the context frees with itself.
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/ovs_kbr.h"

namespace ovs {

int ctx_device(const ovs_ctx* c);
ovs_status ctx_fail(ovs_ctx* c, ovs_status s, const std::string& msg);
// cohort stream i (0..3) of the context, created non-blocking on first use
hipStream_t ctx_cohort_stream(ovs_ctx* c, int i);
// the context's slot for the round loop's cached buffers, released with `release` at destroy
void* ctx_route_scratch(ovs_ctx* c);
void ctx_set_route_scratch(ovs_ctx* c, void* p, void (*release)(void*));
// the Kademlia migration step without the first-round error reset (several cohorts of one batch
// start concurrently: the round loop resets the count once, on the caller's stream, before them)
ovs_status kad_mig_step_impl(ovs_ctx* c, const void* in, uint64_t n_in, const ovs_key160* fkeys, const uint32_t* fsrc,
                             uint32_t fqid, void* out, uint64_t out_cap, unsigned long long* out_count, ovs_done_rec* done,
                             uint64_t done_cap, unsigned long long* done_count, const uint64_t* shard_lo,
                             uint32_t nshards, void* stream, bool reset_errors);
ovs_status kad_shard_reset_errors(ovs_ctx* c, void* stream);

}  // namespace ovs
