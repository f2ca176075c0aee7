/* abi_client.c -- TEST: a plain-C host program on the C-ABI of include/bithashgpu.h, the way a
 * cgo binding would call it: no Python, no torch, only the header and
 * libbithashgpu.so.  The CPU restatement (oracle/, liboracle.so) is the checker.
 *
 *   1. Reader.readData over 20,000 blocks (NoCompressor and snappy records in one table image),
 *      device-resident (bhg_decode_batch with expected CRCs) and from host memory
 *      (bhg_decode_batch_host): descriptors and decoded values equal bho_decode_batch.
 *   2. BithashWriter.Add over 3,000 pairs with snappy and table splits (bhg_encode_batch): the
 *      packed bytes and every per-record output equal bho_encode_batch.
 *   3. The long-range checksum (bhg_crc32c_masked_long) over ranges of 0 B .. 9 MB equals
 *      bho_crc_masked.
 * Exit 0 and "abi_client ok" on success; 2 without a GPU; 1 on any mismatch. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bithash_oracle.h"
#include "bithashgpu.h"

static uint64_t rng = 0x243F6A8885A308D3ull;
static uint32_t rnd(void) {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return (uint32_t)rng;
}

#define CHECK(cond, ...)                                   \
    do {                                                   \
        if (!(cond)) {                                     \
            fprintf(stderr, "abi_client: " __VA_ARGS__);   \
            fprintf(stderr, "\n");                         \
            exit(1);                                       \
        }                                                  \
    } while (0)
#define OK(ctx, call) CHECK((call) == BHG_OK, "%s failed: %s", #call, bhg_last_error(ctx))

static void *dev(bhg_ctx *c, const void *host, uint64_t bytes) {
    void *d = bhg_malloc_device(c, bytes ? bytes : 8);
    CHECK(d != NULL, "bhg_malloc_device(%llu): %s", (unsigned long long)bytes, bhg_last_error(c));
    if (host && bytes) OK(c, bhg_memcpy_h2d(c, d, host, bytes, NULL));
    return d;
}

static void fill_value(uint8_t *v, size_t n, int compressible) {
    for (size_t i = 0; i < n; i++) v[i] = compressible ? (uint8_t)("abcdefgh"[(i / 16 + rnd() % 2) % 8]) : (uint8_t)rnd();
}

static void test_decode(bhg_ctx *c) {
    enum { N = 20000 };
    const size_t cap = (size_t)N * 1400;
    uint8_t *src = malloc(cap), key[32], val[1024], enc[1400];
    bho_handle *h = malloc(N * sizeof *h);
    uint32_t *crc = malloc(N * 4);
    size_t len = 0;
    for (int i = 0; i < N; i++) {
        for (int k = 0; k < 32; k++) key[k] = (uint8_t)('a' + rnd() % 26);
        const size_t vl = (i % 7 == 0) ? rnd() % 1024 + 1 : 1024;
        fill_value(val, vl, i % 3 != 0);
        const uint8_t *v = val;
        size_t el = vl;
        if (i % 2) {  /* snappy records in the odd slots: the snappy batch decodes those */
            el = bho_snappy_encode(enc, val, vl);
            v = enc;
        }
        h[i].offset = len;
        h[i].length = (uint32_t)bho_record_set(src + len, key, 32, ((uint64_t)(i + 1) << 8) | 1, v, el, 1 + i / 5000);
        h[i].pad = 0;
        crc[i] = bho_crc_masked(src + len, h[i].length);
        len += h[i].length + (rnd() % 4);  /* unaligned records */
    }
    /* two batches: even handles NoCompressor, odd handles snappy */
    bho_handle *hb = malloc(N / 2 * sizeof *hb);
    uint32_t *cb = malloc(N / 2 * 4);
    bho_desc *want = malloc(N / 2 * sizeof *want);
    bhg_desc *got = malloc(N / 2 * sizeof *got), *got_h = malloc(N / 2 * sizeof *got_h);
    uint8_t *dsrc = dev(c, src, len);
    for (int codec = 0; codec < 2; codec++) {
        uint64_t vtotal = 0, *voff = calloc(N / 2 + 1, 8), *voff_h = calloc(N / 2 + 1, 8);
        for (int j = 0; j < N / 2; j++) {
            hb[j] = h[2 * j + codec];
            cb[j] = crc[2 * j + codec];
        }
        uint8_t *wvals = NULL, *gvals = NULL, *gvals_h = NULL;
        if (codec == 1) {
            uint64_t *sz = malloc(N / 2 * 8);
            bho_decode_sizes(src, len, hb, N / 2, sz);
            for (int j = 0; j < N / 2; j++) voff[j + 1] = voff[j] + sz[j];
            vtotal = voff[N / 2];
            free(sz);
            wvals = malloc(vtotal + 1);
            gvals = malloc(vtotal + 1);
            gvals_h = malloc(vtotal + 1);
        }
        bho_decode_batch(src, len, hb, N / 2, codec, cb, want, wvals, voff, 0);
        /* device-resident */
        void *dh = dev(c, hb, N / 2 * sizeof *hb), *dc = dev(c, cb, N / 2 * 4);
        bhg_desc *dd = dev(c, NULL, N / 2 * sizeof(bhg_desc));
        uint8_t *dv = codec ? dev(c, NULL, vtotal) : NULL;
        uint64_t *doff = codec ? dev(c, NULL, (N / 2 + 1) * 8) : NULL;
        OK(c, bhg_decode_batch(c, dsrc, len, dh, N / 2, codec, dc, dd, dv, vtotal, doff, NULL));
        OK(c, bhg_stream_sync(c, NULL));
        OK(c, bhg_memcpy_d2h(c, got, dd, N / 2 * sizeof(bhg_desc), NULL));
        uint64_t *goff = calloc(N / 2 + 1, 8);
        if (codec) {
            OK(c, bhg_memcpy_d2h(c, goff, doff, (N / 2 + 1) * 8, NULL));
            OK(c, bhg_memcpy_d2h(c, gvals, dv, vtotal, NULL));
        }
        OK(c, bhg_stream_sync(c, NULL));
        CHECK(memcmp(got, want, N / 2 * sizeof(bhg_desc)) == 0, "codec %d: device descriptors differ", codec);
        if (codec) {
            CHECK(memcmp(goff, voff, (N / 2 + 1) * 8) == 0, "snappy value offsets differ");
            CHECK(memcmp(gvals, wvals, vtotal) == 0, "snappy values differ");
        }
        /* host buffers: the end-to-end entry point */
        OK(c, bhg_decode_batch_host(c, src, len, (const bhg_handle *)hb, N / 2, codec, cb, got_h, gvals_h, vtotal,
                                    codec ? voff_h : NULL));
        CHECK(memcmp(got_h, want, N / 2 * sizeof(bhg_desc)) == 0, "codec %d: host-path descriptors differ", codec);
        if (codec) CHECK(memcmp(gvals_h, wvals, vtotal) == 0, "host-path snappy values differ");
        int ok_blocks = 0;
        for (int j = 0; j < N / 2; j++) ok_blocks += want[j].status == BHG_ST_OK;
        printf("decode codec %d: %d blocks (%d OK), device + host paths equal the restatement\n", codec, N / 2,
               ok_blocks);
        bhg_free_device(c, dh);
        bhg_free_device(c, dc);
        bhg_free_device(c, dd);
        if (dv) bhg_free_device(c, dv);
        if (doff) bhg_free_device(c, doff);
        free(voff); free(voff_h); free(goff); free(wvals); free(gvals); free(gvals_h);
    }
    bhg_free_device(c, dsrc);
    free(src); free(h); free(crc); free(hb); free(cb); free(want); free(got); free(got_h);
}

static void test_encode(bhg_ctx *c) {
    enum { N = 3000, T = 64 };
    uint8_t *keys = malloc(N * 32);
    uint64_t *koff = malloc((N + 1) * 8), *voff = malloc((N + 1) * 8), *tr = malloc(N * 8);
    koff[0] = voff[0] = 0;
    for (int i = 0; i < N; i++) {
        for (int k = 0; k < 32; k++) keys[i * 32 + k] = (uint8_t)('a' + rnd() % 26);
        koff[i + 1] = koff[i] + 32;
        voff[i + 1] = voff[i] + 64 + rnd() % 4033;  /* 64 B .. 4 KiB, the C4 mix */
        tr[i] = ((uint64_t)(i + 1) << 8) | 1;
    }
    const uint64_t vlen = voff[N];
    uint8_t *vals = malloc(vlen);
    for (int i = 0; i < N; i++) fill_value(vals + voff[i], voff[i + 1] - voff[i], i % 4 != 0);
    uint32_t fns[T];
    for (int t = 0; t < T; t++) fns[t] = 100 + t;
    const uint64_t table_max = 1 << 20, ocap = vlen + (uint64_t)N * 80 + 4096;
    /* the restatement */
    uint8_t *wout = malloc(ocap);
    uint64_t wlen = 0, *wpos = malloc(N * 8);
    uint32_t *wbo = malloc(N * 4), *wbl = malloc(N * 4), *wt = malloc(N * 4), *wf = malloc(N * 4), *wc = malloc(N * 4),
             *ws = malloc(N * 4), wts[T];
    const int wnt = bho_encode_batch(keys, koff, tr, vals, voff, N, 1, fns, T, 0, table_max, wout, &wlen, wpos, wbo, wbl,
                                     wt, wf, wc, ws, wts);
    CHECK(wnt >= 2, "restatement used %d tables", wnt);
    /* the device */
    uint8_t *dk = dev(c, keys, N * 32), *dv = dev(c, vals, vlen), *dout = dev(c, NULL, ocap);
    uint64_t *dko = dev(c, koff, (N + 1) * 8), *dvo = dev(c, voff, (N + 1) * 8), *dtr = dev(c, tr, N * 8);
    uint32_t *dfn = dev(c, fns, sizeof fns);
    bhg_encode_out o;
    memset(&o, 0, sizeof o);
    o.pos = dev(c, NULL, N * 8);
    o.bh_off = dev(c, NULL, N * 4);
    o.bh_len = dev(c, NULL, N * 4);
    o.table = dev(c, NULL, N * 4);
    o.fnv1 = dev(c, NULL, N * 4);
    o.crc = dev(c, NULL, N * 4);
    o.status = dev(c, NULL, N * 4);
    o.table_start = dev(c, NULL, T * 4);
    o.summary = dev(c, NULL, 4 * 8);
    OK(c, bhg_encode_batch(c, dk, dko, dtr, dv, dvo, vlen, N, BHG_CODEC_SNAPPY, dfn, T, 0, table_max, dout, ocap, &o,
                           NULL));
    OK(c, bhg_stream_sync(c, NULL));
    uint64_t summary[4], *gpos = malloc(N * 8);
    uint32_t *g = malloc(N * 4), gts[T];
    OK(c, bhg_memcpy_d2h(c, summary, o.summary, sizeof summary, NULL));
    OK(c, bhg_stream_sync(c, NULL));
    CHECK(summary[1] == (uint64_t)wnt && summary[0] == wlen && summary[2] == 0, "summary %llu tables %llu bytes",
          (unsigned long long)summary[1], (unsigned long long)summary[0]);
    uint8_t *gout = malloc(wlen + 1);
    OK(c, bhg_memcpy_d2h(c, gout, dout, wlen, NULL));
    OK(c, bhg_memcpy_d2h(c, gpos, o.pos, N * 8, NULL));
    OK(c, bhg_memcpy_d2h(c, gts, o.table_start, wnt * 4, NULL));
    OK(c, bhg_stream_sync(c, NULL));
    CHECK(memcmp(gout, wout, wlen) == 0, "packed records differ");
    CHECK(memcmp(gpos, wpos, N * 8) == 0, "record positions differ");
    CHECK(memcmp(gts, wts, wnt * 4) == 0, "table starts differ");
    const struct { uint32_t *d, *w; const char *name; } cols[] = {
        {o.bh_off, wbo, "bh_off"}, {o.bh_len, wbl, "bh_len"}, {o.table, wt, "table"},
        {o.fnv1, wf, "fnv1"},      {o.crc, wc, "crc"},        {o.status, ws, "status"}};
    for (size_t k = 0; k < sizeof cols / sizeof cols[0]; k++) {
        OK(c, bhg_memcpy_d2h(c, g, cols[k].d, N * 4, NULL));
        OK(c, bhg_stream_sync(c, NULL));
        CHECK(memcmp(g, cols[k].w, N * 4) == 0, "%s differs", cols[k].name);
    }
    printf("encode: %d pairs, %d tables, %llu bytes equal the restatement\n", N, wnt, (unsigned long long)wlen);
    void *ptrs[] = {dk, dv, dout, dko, dvo, dtr, dfn, o.pos, o.bh_off, o.bh_len, o.table, o.fnv1, o.crc, o.status,
                    o.table_start, o.summary};
    for (size_t k = 0; k < sizeof ptrs / sizeof ptrs[0]; k++) bhg_free_device(c, ptrs[k]);
    free(keys); free(koff); free(voff); free(tr); free(vals); free(wout); free(wpos); free(wbo); free(wbl);
    free(wt); free(wf); free(wc); free(ws); free(gpos); free(g); free(gout);
}

static void test_crc_long(bhg_ctx *c) {
    const uint64_t size = 9u << 20;
    uint8_t *buf = malloc(size);
    for (uint64_t i = 0; i < size; i++) buf[i] = (uint8_t)rnd();
    const uint64_t lens[] = {0, 1, 1023, 1024, 1025, 65536 + 7, 1510000, size - 3, size};
    enum { M = sizeof lens / sizeof lens[0] };
    bhg_handle hs[M];
    uint32_t got[M];
    for (int i = 0; i < M; i++) {
        hs[i].offset = (lens[i] <= size - 3) ? 3 : 0;
        hs[i].length = (uint32_t)lens[i];
        hs[i].pad = 0;
    }
    uint8_t *d = dev(c, buf, size);
    bhg_handle *dh = dev(c, hs, sizeof hs);
    uint32_t *dout = dev(c, NULL, sizeof got);
    OK(c, bhg_crc32c_masked_long(c, d, size, dh, M, dout, NULL));
    OK(c, bhg_stream_sync(c, NULL));
    OK(c, bhg_memcpy_d2h(c, got, dout, sizeof got, NULL));
    OK(c, bhg_stream_sync(c, NULL));
    for (int i = 0; i < M; i++)
        CHECK(got[i] == bho_crc_masked(buf + hs[i].offset, hs[i].length), "crc_long range %d (%llu B)", i,
              (unsigned long long)lens[i]);
    printf("crc_long: %d ranges (0 B .. 9 MiB) equal the restatement\n", M);
    bhg_free_device(c, d);
    bhg_free_device(c, dh);
    bhg_free_device(c, dout);
    free(buf);
}

int main(void) {
    printf("bithashgpu ABI %d, %d device(s)\n", bhg_abi_version(), bhg_device_count());
    bhg_ctx *c = bhg_create(0, 0);
    if (!c) {
        fprintf(stderr, "abi_client: no device context (no GPU)\n");
        return 2;
    }
    test_decode(c);
    test_encode(c);
    test_crc_long(c);
    bhg_destroy(c);
    printf("abi_client ok\n");
    return 0;
}
