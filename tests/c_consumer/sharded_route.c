/*
 * sharded_route.c -- a plain C consumer of the sharded route behind the C ABI (ovs_shard_route_batch /
 * ovs_kad_shard_route_batch, include/ovs_kbr.h): W ranks as threads of one process, one engine
 * context per arc, the library's in-process exchange (ovs_exchange_local_create).  This is the call
 * an OverSim-side GpuChord / GpuKademlia adapter makes for configs D and E, with
 * RCCL (ovs_exchange_rccl_create) in place of the local exchange on a real multi-GPU node.  The same
 * batch is also routed by ovs_route_batch on a context holding the whole network; both results go to
 * the output file, which tests/test_gpu_c_consumer.py compares with each other and with the oracle.
 *
 * input  (little endian): u32 overlay, u64 n, u64 m, n x 5 u32 ids, n x 2 f64 xy, m x 5 u32 keys,
 *                         m x u32 src, u32 world, i32 top_levels (replicated levels / buckets)
 * output: m x ovs_route_out of the sharded route (batch order), m x u32 FindNodeCall counts
 *         (Kademlia; 0 for Chord), m x ovs_route_out of ovs_route_batch, u32 rounds
 * usage: sharded_route <in> <out>
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "ovs_kbr.h"

#define MAXW 16

static void* xread(FILE* f, size_t bytes)
{
    void* p = malloc(bytes ? bytes : 1);
    if (!p || fread(p, 1, bytes, f) != bytes) {
        fprintf(stderr, "sharded_route: short input\n");
        exit(2);
    }
    return p;
}

static int check(ovs_ctx* ctx, ovs_status st, const char* what)
{
    if (st == OVS_OK) return 0;
    fprintf(stderr, "sharded_route: %s failed (%d): %s\n", what, (int)st, ctx ? ovs_last_error(ctx) : "");
    return 1;
}

#define HIPOK(x)                                                                        \
    do {                                                                                \
        if ((x) != hipSuccess) { fprintf(stderr, "sharded_route: %s failed\n", #x); exit(1); } \
    } while (0)

typedef struct Rank {
    int r;
    uint32_t overlay;
    ovs_ctx* ctx;
    ovs_exchange ex;
    const uint64_t* bounds;
    uint64_t m;                 /* lookups whose source lies on this arc */
    uint32_t qid_base;
    ovs_key160* dkeys;
    uint32_t* dsrc;
    ovs_done_rec* ddone;
    uint64_t done_cap, n_done;
    ovs_shard_route_stats stats;
    int rc;
} Rank;

static void* rank_main(void* arg)
{
    Rank* R = (Rank*)arg;
    if (R->overlay == OVS_OVERLAY_CHORD)
        R->rc = check(R->ctx, ovs_shard_route_batch(R->ctx, &R->ex, R->bounds, 0, R->dkeys, R->dsrc, R->m, R->qid_base,
                                                    R->ddone, R->done_cap, &R->n_done, 2, &R->stats, NULL),
                      "ovs_shard_route_batch");
    else
        R->rc = check(R->ctx, ovs_kad_shard_route_batch(R->ctx, &R->ex, R->bounds, OVS_KAD_ONEWAY, R->dkeys, R->dsrc,
                                                        R->m, R->qid_base, R->ddone, R->done_cap, &R->n_done, NULL,
                                                        &R->stats, NULL),
                      "ovs_kad_shard_route_batch");
    return NULL;
}

int main(int argc, char** argv)
{
    if (argc != 3) {
        fprintf(stderr, "usage: %s <in> <out>\n", argv[0]);
        return 2;
    }
    if (ovs_abi_version() != OVS_ABI_VERSION) {
        fprintf(stderr, "sharded_route: library ABI %d, header %d\n", ovs_abi_version(), OVS_ABI_VERSION);
        return 2;
    }
    FILE* f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 2; }
    uint32_t overlay, world;
    int32_t top;
    uint64_t n, m;
    if (fread(&overlay, 4, 1, f) != 1 || fread(&n, 8, 1, f) != 1 || fread(&m, 8, 1, f) != 1) return 2;
    ovs_key160* ids = (ovs_key160*)xread(f, sizeof(ovs_key160) * n);
    double* xy = (double*)xread(f, sizeof(double) * 2 * n);
    ovs_key160* keys = (ovs_key160*)xread(f, sizeof(ovs_key160) * m);
    uint32_t* src = (uint32_t*)xread(f, sizeof(uint32_t) * m);
    if (fread(&world, 4, 1, f) != 1 || fread(&top, 4, 1, f) != 1) return 2;
    fclose(f);
    if (world < 1 || world > MAXW) return 2;

    ovs_params p;
    ovs_params_default((int32_t)overlay, &p);
    if (overlay == OVS_OVERLAY_KADEMLIA) p.lookupParallelRpcs = 3;
    uint64_t bounds[MAXW + 1];
    for (uint32_t r = 0; r <= world; ++r) bounds[r] = (uint64_t)r * n / world;

    /* lookups by the arc of their source, in batch order within an arc: qid = batch index via a map */
    uint64_t* order = (uint64_t*)malloc(sizeof(uint64_t) * (m ? m : 1));
    uint64_t cnt[MAXW] = {0}, off[MAXW + 1] = {0};
    for (uint64_t i = 0; i < m; ++i) {
        uint32_t r = 0;
        while (r + 1 < world && src[i] >= bounds[r + 1]) ++r;
        ++cnt[r];
    }
    for (uint32_t r = 0; r < world; ++r) off[r + 1] = off[r] + cnt[r];
    uint64_t fill[MAXW];
    memcpy(fill, off, sizeof(uint64_t) * MAXW);
    for (uint64_t i = 0; i < m; ++i) {
        uint32_t r = 0;
        while (r + 1 < world && src[i] >= bounds[r + 1]) ++r;
        order[fill[r]++] = i;
    }

    ovs_exchange ex[MAXW];
    if (ovs_exchange_local_create(world, ex) != OVS_OK) {
        fprintf(stderr, "sharded_route: ovs_exchange_local_create: %s\n", ovs_exchange_last_error());
        return 1;
    }
    Rank ranks[MAXW];
    memset(ranks, 0, sizeof ranks);
    int rc = 0;
    for (uint32_t r = 0; r < world && !rc; ++r) {
        Rank* R = &ranks[r];
        R->r = (int)r;
        R->overlay = overlay;
        R->ex = ex[r];
        R->bounds = bounds;
        R->m = cnt[r];
        R->qid_base = (uint32_t)off[r];
        rc |= check(NULL, ovs_ctx_create(0, &R->ctx), "ovs_ctx_create");
        if (rc) break;
        rc |= check(R->ctx, ovs_set_params(R->ctx, &p), "ovs_set_params");
        if (overlay == OVS_OVERLAY_CHORD) {
            rc |= check(R->ctx, ovs_chord_load_shard(R->ctx, ids, n, xy, bounds[r], bounds[r + 1], 0),
                        "ovs_chord_load_shard");
            if (!rc && top > 0) rc |= check(R->ctx, ovs_chord_shard_replicate(R->ctx, top), "ovs_chord_shard_replicate");
        } else {
            rc |= check(R->ctx, ovs_kad_load_shard(R->ctx, ids, n, xy, bounds[r], bounds[r + 1], 0), "ovs_kad_load_shard");
            /* replicated top buckets: the one-way lookups migrate between the arcs */
            if (!rc && top > 0) rc |= check(R->ctx, ovs_kad_shard_replicate(R->ctx, top), "ovs_kad_shard_replicate");
        }
        /* a Chord lookup (or a migrating Kademlia one) may finish on any rank: every done buffer
         * holds the whole batch */
        R->done_cap = (overlay == OVS_OVERLAY_CHORD || top > 0) ? (m ? m : 1) : (R->m ? R->m : 1);
        ovs_key160* hk = (ovs_key160*)malloc(sizeof(ovs_key160) * (R->m ? R->m : 1));
        uint32_t* hs = (uint32_t*)malloc(sizeof(uint32_t) * (R->m ? R->m : 1));
        for (uint64_t j = 0; j < R->m; ++j) { hk[j] = keys[order[off[r] + j]]; hs[j] = src[order[off[r] + j]]; }
        HIPOK(hipMalloc((void**)&R->dkeys, sizeof(ovs_key160) * (R->m ? R->m : 1)));
        HIPOK(hipMalloc((void**)&R->dsrc, sizeof(uint32_t) * (R->m ? R->m : 1)));
        HIPOK(hipMalloc((void**)&R->ddone, sizeof(ovs_done_rec) * R->done_cap));
        HIPOK(hipMemcpy(R->dkeys, hk, sizeof(ovs_key160) * R->m, hipMemcpyHostToDevice));
        HIPOK(hipMemcpy(R->dsrc, hs, sizeof(uint32_t) * R->m, hipMemcpyHostToDevice));
        free(hk);
        free(hs);
    }
    if (rc) return 1;
    pthread_t th[MAXW];
    for (uint32_t r = 0; r < world; ++r) pthread_create(&th[r], NULL, rank_main, &ranks[r]);
    for (uint32_t r = 0; r < world; ++r) pthread_join(th[r], NULL);
    for (uint32_t r = 0; r < world; ++r) rc |= ranks[r].rc;
    if (rc) return 1;

    /* finished records back to batch order: qid = position in `order` */
    ovs_route_out* sh = (ovs_route_out*)calloc(m ? m : 1, sizeof(ovs_route_out));
    uint32_t* rpcs = (uint32_t*)calloc(m ? m : 1, sizeof(uint32_t));
    uint8_t* seen = (uint8_t*)calloc(m ? m : 1, 1);
    uint64_t total = 0;
    for (uint32_t r = 0; r < world; ++r) {
        Rank* R = &ranks[r];
        ovs_done_rec* hd = (ovs_done_rec*)malloc(sizeof(ovs_done_rec) * (R->n_done ? R->n_done : 1));
        HIPOK(hipMemcpy(hd, R->ddone, sizeof(ovs_done_rec) * R->n_done, hipMemcpyDeviceToHost));
        for (uint64_t j = 0; j < R->n_done; ++j) {
            const uint64_t q = hd[j].qid;
            if (q >= m || seen[q]) { fprintf(stderr, "sharded_route: bad or repeated qid %llu\n", (unsigned long long)q); return 1; }
            seen[q] = 1;
            sh[order[q]] = hd[j].out;
            rpcs[order[q]] = overlay == OVS_OVERLAY_KADEMLIA ? hd[j].pad : 0;
        }
        total += R->n_done;
        free(hd);
    }
    if (total != m) { fprintf(stderr, "sharded_route: %llu records for %llu lookups\n", (unsigned long long)total, (unsigned long long)m); return 1; }

    /* the same batch on one context holding the whole network */
    ovs_ctx* whole = NULL;
    rc |= check(NULL, ovs_ctx_create(0, &whole), "ovs_ctx_create");
    rc |= check(whole, ovs_set_params(whole, &p), "ovs_set_params");
    if (overlay == OVS_OVERLAY_CHORD) rc |= check(whole, ovs_chord_load(whole, ids, n, xy, 0), "ovs_chord_load");
    else rc |= check(whole, ovs_kad_load(whole, ids, n, xy, 0), "ovs_kad_load");
    ovs_route_out* ref = (ovs_route_out*)calloc(m ? m : 1, sizeof(ovs_route_out));
    if (!rc) rc |= check(whole, ovs_route_batch(whole, keys, src, m, ref, NULL, NULL, 0, NULL), "ovs_route_batch");
    if (rc) return 1;

    FILE* o = fopen(argv[2], "wb");
    if (!o) { perror(argv[2]); return 2; }
    uint32_t rounds = ranks[0].stats.rounds;
    fwrite(sh, sizeof(ovs_route_out), m, o);
    fwrite(rpcs, sizeof(uint32_t), m, o);
    fwrite(ref, sizeof(ovs_route_out), m, o);
    fwrite(&rounds, 4, 1, o);
    fclose(o);
    for (uint32_t r = 0; r < world; ++r) {
        ovs_exchange_destroy(&ranks[r].ex);
        hipFree(ranks[r].dkeys); hipFree(ranks[r].dsrc); hipFree(ranks[r].ddone);
        ovs_ctx_destroy(ranks[r].ctx);
    }
    ovs_ctx_destroy(whole);
    return 0;
}
