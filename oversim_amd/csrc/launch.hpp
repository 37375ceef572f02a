// launch.hpp -- host launchers of the device kernels (internal).
#pragma once
#include "engine.hpp"
#include "compact.hpp"

namespace ovs {

hipError_t launch_check_sorted(const KeyRec* recs, uint32_t n, uint32_t* bad, hipStream_t s);
hipError_t launch_chord_build(KeyRec* recs, uint32_t n, uint32_t lo, uint32_t hi, FingerEnt** fingers_out,
                              uint64_t* nfing_out, hipStream_t s);
hipError_t launch_chord_shard_step(const ChordView& V, const DelayConsts& DC, const LookupConsts& LC,
                                   const uint64_t* shard_lo, int nsh, int me, const ovs_lookup_rec* in, uint64_t nin,
                                   ovs_lookup_rec* out, uint64_t out_cap,
                                   unsigned long long* out_count, ovs_done_rec* done, uint64_t done_cap,
                                   unsigned long long* done_count, StageBuf& stage, int num_cu, hipStream_t s,
                                   const K160* fkeys = nullptr, const uint32_t* fsrc = nullptr, uint32_t fqid = 0,
                                   unsigned long long* dyn = nullptr);
hipError_t launch_make_records(const KeyRec* recs, const K160* keys, const uint32_t* src, uint64_t n, uint32_t qid_base,
                               ovs_lookup_rec* out, hipStream_t s);
hipError_t launch_chord_nodes(const KeyRec* recs, const double2* xy, uint32_t n, int ns, NodeRec* nodes,
                              FingerEnt* fingers, uint64_t nfing, WinRec* win, uint32_t lo, uint32_t hi, hipStream_t s);
// replicated top finger levels of a sharded ring (finger indices; launch_chord_entries completes them)
hipError_t launch_chord_top(const KeyRec* recs, uint32_t n, int L, FingerEnt* ftop, hipStream_t s);
hipError_t launch_chord_entries(const NodeRec* nodes, FingerEnt* ents, uint64_t total, hipStream_t s);
hipError_t launch_chord_export(const KeyRec* recs, const FingerEnt* fingers, uint32_t n, uint32_t* out,
                               hipStream_t s);
// perm != nullptr: qkeys / qsrc are the batch in key order (ksort_launch), perm[q] the caller index of
// sorted lookup q, where its result goes (one-way iterative routes on a converged ring).  dyn: a zeroed
// device counter for this launch alone -- K1 then hands out the batch's last ~30 % dynamically
// (ctx_dyn_acquire); nullptr: static slices only
hipError_t launch_chord_route(const ChordView& V, bool ideal, const DelayConsts& DC, const LookupConsts& LC,
                              const K160* qkeys, const uint32_t* qsrc, uint64_t nq, ovs_route_out* out,
                              uint32_t* hopseq, int num_cu, hipStream_t s, const uint32_t* perm = nullptr,
                              unsigned long long* dyn = nullptr);
// ksort.hip: the batch's keys and sources in the order of their top key bits (a counting sort), with
// the caller index of each; scratch = ksort_scratch_words() u32
uint64_t ksort_scratch_words();
hipError_t ksort_launch(const K160* keys, const uint32_t* src, uint64_t n, uint32_t* scratch, K160* skeys,
                        uint32_t* ssrc, uint32_t* perm, int bits, hipStream_t s);
hipError_t launch_chord_find_node(const ChordView& V, bool ideal, const uint32_t* node, const K160* keys,
                                  uint64_t n, int numRedundant, int numSiblings, uint32_t* out_nodes,
                                  uint32_t max_out, uint8_t* out_count, uint8_t* out_sib, hipStream_t s);
hipError_t launch_shard_lookup_finish(const ChordView& V, int ns, const ovs_done_rec* done, ovs_lookup_out* out,
                                      uint32_t* sibs, uint64_t n, hipStream_t s);
// Chord exact-key LookupCalls (numSiblings = 0) replayed from the recorded one-way chain (chord.hip)
hipError_t launch_chord_exact_finish(const ChordView& V, const DelayConsts& DC, int hcm, const K160* keys,
                                     const uint32_t* src, const uint32_t* hopseq, int H, ovs_route_out* io,
                                     uint64_t n, hipStream_t s);
hipError_t launch_lookup_finish(const ChordView& V, bool chord, bool ideal, int ns, ovs_route_out* io,
                                uint32_t* sibs, uint64_t n, hipStream_t s);
hipError_t launch_fill_rpcs_from_hops(const ovs_route_out* out, uint64_t n, uint32_t* rpcs, hipStream_t s);
// per-block min / max of the coordinates (x0, x1, y0, y1 per block into out[4 * blocks], blocks <= 256):
// the bounding box that bounds every coordinate delay (extendedFingerTable's acceptance, ovs_kbr.cpp)
hipError_t launch_xy_bbox(const double2* xy, uint64_t n, double* out, int* blocks, hipStream_t s);
hipError_t launch_delay(const double2* xy, const DelayConsts& DC, const uint32_t* a, const uint32_t* b,
                        const int32_t* bytes, uint64_t n, int64_t* out, hipStream_t s);

}  // namespace ovs
