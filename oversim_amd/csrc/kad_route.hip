// kad_route.hip -- K2, the Kademlia iterative-lookup kernel, for gfx950 (MI355X).
//
// Compiled once per (alpha, exact) pair (build.py: -DOVS_KAD_A, -DOVS_KAD_EX) so the eight
// heavy instantiation sets build in parallel; kad.hip's kad_route dispatches to them.
//
// K2 k_kad_route: one lane per lookup running OverSim's IterativePathLookup (IterativeLookup.cc:
// 760-1195, merge = true, parallel RPCs) against <= alpha pending FindNodeCalls ordered by
// simulated arrival time (int64 ns).  Each loop iteration processes the lookup's earliest event:
// a response is the responder's Kademlia::findNode (Kademlia.cc:1101-1246) over its 96 B bucket
// blocks (one per k <= 8 bucket) merged into the LookupVector, then the sends it triggers (one
// 64 B KadNode line per target: its key, coordinates and isSiblingFor summary).  Finished lanes
// refill from the wave's slice of the batch (ballot + popcount); the grid is persistent.
// (A per-line state machine in the manner of K1 was tried in this round and reverted: the union
// of the divergent findNode stages every iteration cost 7x the VALU work)
#include "kad_dev.hpp"

#ifndef OVS_KAD_A
#error "kad_route.hip is compiled with -DOVS_KAD_A=<alpha> -DOVS_KAD_EX=<0|1> (oversim_amd/build.py)"
#endif
#ifndef OVS_KAD_WAVES
// minimum waves per SIMD the register allocator must allow: 3 (<= 168 VGPRs) costs a few spills
// and runs E 1.2x faster than the unconstrained 176-188 VGPRs (2 waves); profiles/r02_b_kad
#define OVS_KAD_WAVES 3
#endif

namespace ovs {

namespace {

struct SendNothing {
    __device__ __forceinline__ void operator()(int, uint32_t, bool) const {}
};

template <bool EX, bool LK>
struct LocalFindNode {
    const KadView& V;
    const K160& K;
    int numSiblings;
    __device__ __forceinline__ bool ready(int) const { return true; }
    __device__ __forceinline__ void fill(int, uint32_t r, const RespGeo& g, bool sb, int numR, bool, SVec<8>& res) const
    {
        Blk8 b;
        const int n = kad_find_node_blk<EX>(V, r, g, K, numR, sb, b, LK ? numSiblings : 1);
#pragma unroll
        for (int i = 0; i < 8; ++i) { res.idx[i] = b.x[i]; res.d[i] = b.d[i]; }
        res.n = n;
        res.used = 0;
    }
};

template <bool RECORD>
struct HopRecorder {
    uint32_t* __restrict__ hopseq;
    uint64_t base;
    int hcm;
    __device__ __forceinline__ void operator()(int h, uint32_t r) const
    {
        if (RECORD && h < hcm) hopseq[base + h] = r;
    }
};

template <int A, bool RECORD, bool EX, bool LK>
__global__ __launch_bounds__(256, OVS_KAD_WAVES) void k_kad_route(KadView V, DelayConsts DC, KadLC LC, const K160* __restrict__ qkeys,
                                                        const uint32_t* __restrict__ qsrc, uint64_t nq, uint64_t chunk,
                                                        ovs_route_out* __restrict__ out, uint32_t* __restrict__ hopseq,
                                                        uint32_t* __restrict__ rpcs_out, uint32_t* __restrict__ sib_out)
{
    const int lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    uint64_t cursor = wave * chunk;
    const uint64_t end = min(cursor + chunk, nq);
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

    bool active = false;
    uint64_t q = 0;
    KadLookup<A> L;
    SVec<8> res;
    const SendNothing on;

    while (true) {
        const uint64_t need = __ballot(!active);
        if (need != 0 && cursor < end) {
            const uint64_t mine = cursor + (uint64_t)__popcll(need & lt_mask);
            if (!active && mine < end) {
                q = mine;
                active = true;
                kad_lookup_init(L, qkeys[q], qsrc[q], V.xy);
            }
            cursor += (uint64_t)__popcll(need);
        }
        if (!__any(active)) break;
        if (!active) continue;

        if (!kad_lookup_done(L)) {
            const LocalFindNode<EX, LK> fn{V, L.K, LC.numSiblings};
            const HopRecorder<RECORD> rec{hopseq, q * (uint64_t)LC.hopCountMax, LC.hopCountMax};
            kad_lookup_event<A, EX, LK>(L, V, DC, LC, res, fn, on, rec);
        }
        if (kad_lookup_done(L)) {
            const ovs_route_out o = kad_lookup_output(L, V, DC, LC);
            out[q] = o;
            if (rpcs_out) rpcs_out[q] = L.nsent;
            if (LK) {
                const bool ok = o.status == OVS_LOOKUP_OK;
                if (LC.numSiblings == 0) {
                    sib_out[q] = ok ? L.result : NONE;    // the one-slot vector of an exact-key lookup
                } else {
                    uint32_t* row = sib_out + q * (uint64_t)LC.numSiblings;
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if (j < LC.numSiblings) row[j] = (ok && j < res.n) ? res.idx[j] : NONE;
                }
            }
            active = false;
        }
    }
}

}  // namespace

template <class Kern>
static uint64_t kad_chunk(Kern kern, int* cache, uint64_t nq, int num_cu, uint64_t* blocks)
{
    if (*cache == 0) {
        int b = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kern, 256, 0) != hipSuccess || b < 1) b = 1;
        *cache = b;
    }
    const uint64_t waves = (uint64_t)num_cu * (uint64_t)(*cache) * 4;
    uint64_t chunk = (nq + waves - 1) / waves;
    if (chunk < 1) chunk = 1;
    const uint64_t need_waves = (nq + chunk - 1) / chunk;
    *blocks = (need_waves + 3) / 4;
    return chunk;
}

template <int A, bool RECORD, bool EX, bool LK>
static hipError_t kad_launch(const KadView& V, const DelayConsts& DC, const KadLC& LC, const K160* qkeys,
                             const uint32_t* qsrc, uint64_t nq, ovs_route_out* out, uint32_t* hopseq, uint32_t* rpcs,
                             uint32_t* sibs, int num_cu, hipStream_t st)
{
    static int bpc = 0;    // one per instantiation
    uint64_t blocks = 0;
    const uint64_t chunk = kad_chunk(k_kad_route<A, RECORD, EX, LK>, &bpc, nq, num_cu, &blocks);
    hipLaunchKernelGGL((k_kad_route<A, RECORD, EX, LK>), dim3((unsigned)blocks), dim3(256), 0, st, V, DC, LC, qkeys,
                       qsrc, nq, chunk, out, hopseq, rpcs, sibs);
    return hipGetLastError();
}

template <int A, bool EX>
hipError_t kad_route_launch(const KadView& V, const DelayConsts& DC, const KadLC& LC, const K160* qkeys,
                            const uint32_t* qsrc, uint64_t nq, ovs_route_out* out, uint32_t* hopseq, uint32_t* rpcs,
                            uint32_t* sibs, int num_cu, hipStream_t st)
{
    // LookupCall batches (sibs != nullptr) record no hop sequence
    if (sibs) return kad_launch<A, false, EX, true>(V, DC, LC, qkeys, qsrc, nq, out, hopseq, rpcs, sibs, num_cu, st);
    if (hopseq) return kad_launch<A, true, EX, false>(V, DC, LC, qkeys, qsrc, nq, out, hopseq, rpcs, sibs, num_cu, st);
    return kad_launch<A, false, EX, false>(V, DC, LC, qkeys, qsrc, nq, out, hopseq, rpcs, sibs, num_cu, st);
}

template hipError_t kad_route_launch<OVS_KAD_A, OVS_KAD_EX != 0>(const KadView&, const DelayConsts&, const KadLC&,
                                                                 const K160*, const uint32_t*, uint64_t, ovs_route_out*,
                                                                 uint32_t*, uint32_t*, uint32_t*, int, hipStream_t);

}  // namespace ovs
