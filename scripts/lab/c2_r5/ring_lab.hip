// ring_lab.hip -- development harness (not product code): the LDS-DMA ring decode
// (decode_ring.hip) checked descriptor for descriptor against the product
// library's bhg_decode_batch and timed beside it, on
//   c2      BASELINE configs[1]: 1M x 1,076-B records in 128 MiB tables, expected CRCs, a few bad
//           handles / records / CRCs;
//   shuf    the same handles in random order;
//   mixed   contiguous records with values of 0..12,000 B (some larger than a ring slot) at odd
//           offsets, so every record end alignment and the big-record path occur.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <numeric>
#include <random>
#include <vector>

#include "decode_ring.hip"

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

using namespace bhg;

static std::mt19937_64 rng(12345);

struct Set {
    std::vector<uint8_t> src;
    std::vector<bhg_handle> h;
};

static void put_record(std::vector<uint8_t> &b, uint64_t off, uint32_t klen, uint32_t vlen, uint32_t fn, uint64_t seq) {
    const uint32_t hdr[3] = {klen + 8, vlen, fn};
    memcpy(&b[off], hdr, 12);
    for (uint32_t i = 0; i < klen; i++) b[off + 12 + i] = (uint8_t)('a' + rng() % 26);
    const uint64_t tr = (seq << 8) | 1;
    memcpy(&b[off + 12 + klen], &tr, 8);
    for (uint32_t i = 0; i < vlen; i++) b[off + 20 + klen + i] = (uint8_t)rng();
}

static Set make_c2(uint32_t n) {
    Set s;
    const uint32_t L = 1076, R = (128u << 20) / L + 1, TB = R * L + 12;
    const uint32_t ntab = (n + R - 1) / R;
    s.src.assign((uint64_t)ntab * TB, 0);
    s.h.resize(n);
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t off = (uint64_t)(i / R) * TB + (uint64_t)(i % R) * L;
        put_record(s.src, off, 32, 1024, 1 + i / R, i + 1);
        s.h[i] = bhg_handle{off, L, 0};
    }
    if (n > 10) s.h[7].length = 0;          // ILLEGAL_LENGTH
    if (n > 20) s.h[13].length = L - 1;     // RECORD_NIL
    if (n > 40) s.h[35].offset = s.src.size();  // INCOMPLETE
    return s;
}

static Set make_mixed(uint32_t n) {
    Set s;
    std::vector<uint32_t> kl(n), vl(n);
    uint64_t tot = 3;
    for (uint32_t i = 0; i < n; i++) {
        kl[i] = (uint32_t)(rng() % 8 == 0 ? 40 + rng() % 60 : rng() % 37);  // some keys longer than 36 B
        const uint32_t r = (uint32_t)(rng() % 100);
        vl[i] = r < 2 ? (uint32_t)(9000 + rng() % 3000) : r < 30 ? (uint32_t)(rng() % 300) : (uint32_t)(rng() % 4200);
        if (vl[i] == 0) vl[i] = 1;
        tot += 20 + kl[i] + vl[i];
    }
    s.src.assign(tot + 64, 0);
    s.h.resize(n);
    uint64_t off = 3;  // odd start: every record end alignment occurs
    for (uint32_t i = 0; i < n; i++) {
        put_record(s.src, off, kl[i], vl[i], 7, i + 1);
        s.h[i] = bhg_handle{off, 20 + kl[i] + vl[i], 0};
        off += 20 + kl[i] + vl[i];
    }
    if (n > 100) s.h[50].length = 5;       // short record: RECORD_NIL
    if (n > 100) s.h[77].length = 0;
    return s;
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 30;
    const uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : 1000000u;
    bhg_ctx *ctx = bhg_create(0, 0);
    if (!ctx) { fprintf(stderr, "no ctx\n"); return 1; }
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    hipStream_t s = (hipStream_t)bhg_stream(ctx);
    std::vector<uint32_t> z(kRingZN * 1024);
    build_ring_ztab(z.data());
    uint32_t *rz, *err;
    CK(hipMalloc(&rz, z.size() * 4));
    CK(hipMemcpy(rz, z.data(), z.size() * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&err, 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    int fails = 0;
    const int nsets = argc > 3 ? atoi(argv[3]) : 3;  // 1: the C2 set only (profiling runs)
    const bool quick = argc > 4;                     // no knock-out / clock-profile variants
    for (int which = 0; which < nsets; which++) {
        Set st = which == 2 ? make_mixed(n / 4) : make_c2(n);
        const char *name = which == 0 ? "c2" : which == 1 ? "shuf" : "mixed";
        if (which == 1) std::shuffle(st.h.begin(), st.h.end(), rng);
        const uint32_t nn = (uint32_t)st.h.size();
        const uint64_t len = st.src.size();
        uint8_t *src; bhg_handle *dh; uint32_t *ec; bhg_desc *o1, *o2;
        CK(hipMalloc(&src, len + 64)); CK(hipMalloc(&dh, nn * 16ull)); CK(hipMalloc(&ec, nn * 4ull));
        CK(hipMalloc(&o1, nn * 40ull)); CK(hipMalloc(&o2, nn * 40ull));
        CK(hipMemcpy(src, st.src.data(), len, hipMemcpyHostToDevice));
        CK(hipMemcpy(dh, st.h.data(), nn * 16ull, hipMemcpyHostToDevice));
        if (bhg_crc32c_masked_batch(ctx, src, len, dh, nn, ec, s) != 0) { fprintf(stderr, "crc batch\n"); return 1; }
        CK(hipStreamSynchronize(s));
        if (nn > 30) {  // one wrong expected CRC -> CRC_MISMATCH
            uint32_t x; CK(hipMemcpy(&x, ec + 29, 4, hipMemcpyDeviceToHost)); x ^= 1; CK(hipMemcpy(ec + 29, &x, 4, hipMemcpyHostToDevice));
        }
        auto prod = [&]() { if (bhg_decode_batch(ctx, src, len, dh, nn, 0, ec, o1, nullptr, 0, nullptr, s)) { fprintf(stderr, "prod\n"); exit(1); } };
        auto ringk = [&]() {
            hipLaunchKernelGGL((ring::k_decode_ring<0>), dim3(cus), dim3(64 * (ring::kNC + 1)), 0, s, src, len, dh, nn, ec, o2, rz, err, (unsigned long long *)nullptr);
        };
        for (int it = 0; it < 50; it++) prod();  // clocks
        CK(hipStreamSynchronize(s));
        CK(hipMemset(o2, 0xee, nn * 40ull));
        ringk();
        CK(hipStreamSynchronize(s));
        CK(hipGetLastError());
        uint32_t herr = 0;
        CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
        std::vector<bhg_desc> d1(nn), d2(nn);
        CK(hipMemcpy(d1.data(), o1, nn * 40ull, hipMemcpyDeviceToHost));
        CK(hipMemcpy(d2.data(), o2, nn * 40ull, hipMemcpyDeviceToHost));
        uint32_t bad = 0, first = 0xffffffffu, nok = 0;
        for (uint32_t i = 0; i < nn; i++) {
            if (memcmp(&d1[i], &d2[i], 40) != 0) { if (!bad) first = i; bad++; }
            nok += d1[i].status == 0;
        }
        auto timeit = [&](auto fn) {
            std::vector<float> ts;
            for (int it = 0; it < iters; it++) {
                CK(hipEventRecord(a, s)); fn(); CK(hipEventRecord(b, s)); CK(hipEventSynchronize(b));
                float ms; CK(hipEventElapsedTime(&ms, a, b)); ts.push_back(ms);
            }
            std::sort(ts.begin(), ts.end());
            return std::make_pair(ts[ts.size() / 2], ts[0]);
        };
        uint64_t tot = 0;
        for (const bhg_handle &h : st.h) tot += h.length;
        const double alg = (double)tot + 60.0 * nn;  // record bytes + handle + expected CRC + descriptor
        auto tp = timeit(prod);
        auto tr = timeit(ringk);
        if (which == 0 && !quick) {
            auto ko = [&](auto kern, const char *nm) {
                auto t = timeit([&]() { hipLaunchKernelGGL(kern, dim3(cus), dim3(64 * (ring::kNC + 1)), 0, s, src, len, dh, nn, ec, o2, rz, err, (unsigned long long *)nullptr); });
                printf("   ko %-22s %.4f ms (frac-equiv %.4f)\n", nm, t.first, alg / (t.first * 1e-3) / 8e12);
            };
            ko(ring::k_decode_ring<1>, "no window CRC");
            ko(ring::k_decode_ring<2>, "no head copy");
            ko(ring::k_decode_ring<4>, "no parse");
            ko(ring::k_decode_ring<7>, "none of the three");
            ko(ring::k_decode_ring<8 | 4>, "protocol only");
            unsigned long long *prof;
            CK(hipMalloc(&prof, 16 * 8));
            auto prun = [&](auto kern, const char *nm) {
                CK(hipMemset(prof, 0, 16 * 8));
                hipLaunchKernelGGL(kern, dim3(cus), dim3(64 * (ring::kNC + 1)), 0, s, src, len, dh, nn, ec, o2, rz, err, prof);
                CK(hipStreamSynchronize(s));
                unsigned long long h[16];
                CK(hipMemcpy(h, prof, 16 * 8, hipMemcpyDeviceToHost));
                const double Lw = (double)h[8] / cus, Cw = (double)h[9] / (cus * ring::kNC);
                printf("   prof %-12s loader total %.0f clk: FREE-wait %.1f%% vm-wait %.1f%% drain %.1f%% idle-iters %.0f | "
                       "consumer total %.0f: mail-wait %.1f%% tile %.1f%% parse %.1f%%\n", nm, Lw, 100.0 * h[0] / cus / Lw,
                       100.0 * h[1] / cus / Lw, 100.0 * h[2] / cus / Lw, (double)h[3] / cus, Cw,
                       100.0 * h[4] / (cus * ring::kNC) / Cw, 100.0 * h[5] / (cus * ring::kNC) / Cw,
                       100.0 * h[6] / (cus * ring::kNC) / Cw);
            };
            prun(ring::k_decode_ring<16>, "full");
            prun(ring::k_decode_ring<16 | 1>, "no-winCRC");
            prun(ring::k_decode_ring<16 | 8 | 4>, "protocol");
            CK(hipFree(prof));
        }
        CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
        printf("%-6s n=%u ok=%u  product %.4f ms (frac %.4f)  ring %.4f ms best %.4f (frac %.4f)  mismatches %u (first %u) err %u\n",
               name, nn, nok, tp.first, alg / (tp.first * 1e-3) / 8e12, tr.first, tr.second, alg / (tr.first * 1e-3) / 8e12,
               bad, first, herr);
        if (bad) {
            const uint32_t i = first;
            printf("  h off %llu len %u | prod: kl %u vo %u vl %u crc %08x st %u fnv %08x tr %llx | ring: kl %u vo %u vl %u crc %08x st %u fnv %08x tr %llx\n",
                   (unsigned long long)st.h[i].offset, st.h[i].length, d1[i].key_len, d1[i].val_off, d1[i].val_len,
                   d1[i].crc, d1[i].status, d1[i].fnv1, (unsigned long long)d1[i].trailer, d2[i].key_len,
                   d2[i].val_off, d2[i].val_len, d2[i].crc, d2[i].status, d2[i].fnv1, (unsigned long long)d2[i].trailer);
            fails++;
        }
        fflush(stdout);
        CK(hipFree(src)); CK(hipFree(dh)); CK(hipFree(ec)); CK(hipFree(o1)); CK(hipFree(o2));
        if (herr) { printf("protocol error %u: stop\n", herr); return 2; }
    }
    bhg_destroy(ctx);
    return fails ? 1 : 0;
}
