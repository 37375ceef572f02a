// kad.hip -- Kademlia kernels (placeholder until the K2 kernel lands).
#include "kad.hpp"

namespace ovs {
void kad_free(KadTables& t) { (void)t; }
hipError_t kad_build(const KeyRec*, uint32_t, int, int, uint64_t, KadTables&, hipStream_t) { return hipErrorNotSupported; }
hipError_t kad_export(const KadTables&, uint32_t, uint32_t*, uint8_t*, uint32_t*, hipStream_t) { return hipErrorNotSupported; }
hipError_t kad_route(const KadTables&, const KeyRec*, const double2*, uint32_t, const ovs_params&, const DelayConsts&,
                     const K160*, const uint32_t*, uint64_t, ovs_route_out*, uint32_t*, uint32_t*, int, hipStream_t)
{ return hipErrorNotSupported; }
hipError_t kad_find_node(const KadTables&, const KeyRec*, uint32_t, const ovs_params&, const uint32_t*, const K160*,
                         uint64_t, int, int, uint32_t*, uint32_t, uint8_t*, uint8_t*, hipStream_t)
{ return hipErrorNotSupported; }
}  // namespace ovs
