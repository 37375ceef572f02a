/*
 * route_batch.c -- a plain C consumer of the engine's C ABI (include/ovs_kbr.h), built with gcc
 * and linked against oversim_amd/libovs_kbr.so, the way an OverSim-side adapter
 * would call it.  No Python, no torch: ovs_params_from_ini binds the reference's .ini names, the
 * network and lookups come from a binary input file, results go to a binary output file that
 * tests/test_gpu_c_consumer.py compares with the oracle.
 *
 * input  (little endian): u32 overlay, u64 n, u64 m, n x 5 u32 ids, n x 2 f64 xy, m x 5 u32 keys,
 *                         m x u32 src, u32 ini_len, ini_len bytes of .ini text
 * output: m x ovs_route_out, m x u32 FindNodeCall counts, then m x ovs_lookup_out and
 *         m x s u32 siblings of the LookupCalls (numSiblings = getMaxNumSiblings())
 * usage: route_batch <in> <out>
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ovs_kbr.h"

static void* xread(FILE* f, size_t bytes)
{
    void* p = malloc(bytes ? bytes : 1);
    if (!p || fread(p, 1, bytes, f) != bytes) {
        fprintf(stderr, "route_batch: short input\n");
        exit(2);
    }
    return p;
}

static int check(ovs_ctx* ctx, ovs_status st, const char* what)
{
    if (st == OVS_OK) return 0;
    fprintf(stderr, "route_batch: %s failed (%d): %s\n", what, (int)st, ctx ? ovs_last_error(ctx) : "");
    return 1;
}

int main(int argc, char** argv)
{
    if (argc != 3) {
        fprintf(stderr, "usage: %s <in> <out>\n", argv[0]);
        return 2;
    }
    if (ovs_abi_version() != OVS_ABI_VERSION) {
        fprintf(stderr, "route_batch: library ABI %d, header %d\n", ovs_abi_version(), OVS_ABI_VERSION);
        return 2;
    }
    FILE* f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 2; }
    uint32_t overlay;
    uint64_t n, m;
    if (fread(&overlay, 4, 1, f) != 1 || fread(&n, 8, 1, f) != 1 || fread(&m, 8, 1, f) != 1) return 2;
    ovs_key160* ids = (ovs_key160*)xread(f, sizeof(ovs_key160) * n);
    double* xy = (double*)xread(f, sizeof(double) * 2 * n);
    ovs_key160* keys = (ovs_key160*)xread(f, sizeof(ovs_key160) * m);
    uint32_t* src = (uint32_t*)xread(f, sizeof(uint32_t) * m);
    uint32_t ini_len;
    if (fread(&ini_len, 4, 1, f) != 1) return 2;
    char* ini = (char*)malloc((size_t)ini_len + 1);
    if (!ini || fread(ini, 1, ini_len, f) != ini_len) {
        fprintf(stderr, "route_batch: short input\n");
        return 2;
    }
    ini[ini_len] = 0;
    fclose(f);

    ovs_params p;
    ovs_params_default((int32_t)overlay, &p);
    char err[256];
    if (ovs_params_from_ini(&p, ini, NULL, err, (int)sizeof err) != OVS_OK) {
        fprintf(stderr, "route_batch: .ini: %s\n", err);
        return 1;
    }
    ovs_ctx* ctx = NULL;
    if (check(NULL, ovs_ctx_create(0, &ctx), "ovs_ctx_create")) return 1;
    int rc = 0;
    rc |= check(ctx, ovs_set_params(ctx, &p), "ovs_set_params");
    if (!rc) {
        if (overlay == OVS_OVERLAY_CHORD) rc |= check(ctx, ovs_chord_load(ctx, ids, n, xy, 0), "ovs_chord_load");
        else if (overlay == OVS_OVERLAY_KADEMLIA) rc |= check(ctx, ovs_kad_load(ctx, ids, n, xy, 0), "ovs_kad_load");
        else rc |= check(ctx, ovs_koorde_load(ctx, ids, n, xy, 0), "ovs_koorde_load");
    }
    ovs_route_out* out = (ovs_route_out*)calloc(m ? m : 1, sizeof *out);
    uint32_t* rpcs = (uint32_t*)calloc(m ? m : 1, sizeof *rpcs);
    if (!rc) rc |= check(ctx, ovs_route_batch(ctx, keys, src, m, out, NULL, rpcs, 0, NULL), "ovs_route_batch");
    const int32_t s = overlay == OVS_OVERLAY_KADEMLIA ? p.s : p.successorListSize;
    ovs_lookup_out* lo = (ovs_lookup_out*)calloc(m ? m : 1, sizeof *lo);
    uint32_t* sib = (uint32_t*)calloc((m ? m : 1) * (size_t)s, sizeof *sib);
    if (!rc && overlay != OVS_OVERLAY_KOORDE)
        rc |= check(ctx, ovs_lookup_batch(ctx, keys, src, m, -1, lo, sib, 0, NULL), "ovs_lookup_batch");
    ovs_ctx_destroy(ctx);
    if (rc) return 1;
    FILE* o = fopen(argv[2], "wb");
    if (!o) { perror(argv[2]); return 2; }
    fwrite(out, sizeof *out, m, o);
    fwrite(rpcs, sizeof *rpcs, m, o);
    fwrite(lo, sizeof *lo, m, o);
    fwrite(sib, sizeof *sib, m * (size_t)s, o);
    fclose(o);
    free(ids); free(xy); free(keys); free(src); free(ini); free(out); free(rpcs); free(lo); free(sib);
    return 0;
}
