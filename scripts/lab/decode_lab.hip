// decode_lab.hip -- development harness (not product code): times candidate
// C2 decode kernels against the production bhg_decode_batch on the same
// device-resident batch and checks every descriptor byte-for-byte.
//
// build: make -C scripts/lab      run: scripts/lab/decode_lab [iters]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../bitalosdb_amd/csrc/bhg_device.h"
#include "../../bitalosdb_amd/csrc/bhg_crc_tables.h"
#include "../../include/bithashgpu.h"

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

using namespace bhg;

// ---------------------------------------------------------------- data
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
__constant__ uint8_t kAlpha[62] = {'1','q','a','z','2','w','s','x','3','e','d','c','4','r','f','v','5','t','g','b','6','y',
                                   'h','n','7','u','j','m','8','i','k','9','o','l','0','p','A','B','C','D','E','F','G','H',
                                   'I','J','K','L','M','N','O','P','Q','R','S','T','U','V','W','X','Y','Z'};

// record i: header {40, 1024, fn}, key 32 alnum, trailer (i+1)<<8|1, value 1024 alnum
__global__ void k_gen(uint8_t *src, const bhg_handle *h, uint32_t n, uint32_t per_table) {
    uint32_t i = blockIdx.x;
    if (i >= n) return;
    uint8_t *r = src + h[i].offset;
    const uint32_t L = h[i].length;
    for (uint32_t b = threadIdx.x; b < L; b += blockDim.x) {
        uint8_t x;
        if (b < 12) {
            uint32_t w = b < 4 ? 40u : b < 8 ? 1024u : 1u + i / per_table;
            x = (uint8_t)(w >> (8 * (b & 3)));
        } else if (b >= 44 && b < 52) {
            uint64_t t = ((uint64_t)(i + 1) << 8) | 1;
            x = (uint8_t)(t >> (8 * (b - 44)));
        } else {
            x = kAlpha[mix64(((uint64_t)i << 12) ^ b ^ 0xB17A105DBull) % 62];
        }
        r[b] = x;
    }
}

typedef void (*launch_fn)(const uint8_t *, uint64_t, const bhg_handle *, uint32_t, bhg_desc *, const uint32_t *,
                          hipStream_t);
// ---------------------------------------------------------------- kernels under test
#include "lab_kernels.h"

// ---------------------------------------------------------------- driver

static float time_it(launch_fn f, const uint8_t *src, uint64_t len, const bhg_handle *h, uint32_t n, bhg_desc *out,
                      const uint32_t *tabs, hipStream_t s, int iters, float *best) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f(src, len, h, n, out, tabs, s);
    f(src, len, h, n, out, tabs, s);
    CK(hipStreamSynchronize(s));
    std::vector<float> ts;
    for (int it = 0; it < iters; it++) {
        CK(hipEventRecord(a, s));
        f(src, len, h, n, out, tabs, s);
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    *best = ts[0];
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ts[ts.size() / 2];
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20;
    const char *only = argc > 2 ? argv[2] : nullptr;
    const uint32_t n = 1000000, L = 1076;
    const uint32_t R = (uint32_t)((128ull << 20) / L + 1);  // records per 128 MiB table
    const uint64_t tbytes = (uint64_t)R * L + 12;
    std::vector<bhg_handle> hh(n);
    for (uint32_t i = 0; i < n; i++) hh[i] = bhg_handle{(uint64_t)(i / R) * tbytes + (uint64_t)(i % R) * L, L, 0};
    const uint64_t len = hh[n - 1].offset + L + 12;
    uint8_t *src;
    bhg_handle *dh;
    bhg_desc *ref, *out;
    CK(hipMalloc(&src, len));
    CK(hipMalloc(&dh, n * sizeof(bhg_handle)));
    CK(hipMalloc(&ref, n * sizeof(bhg_desc)));
    CK(hipMalloc(&out, n * sizeof(bhg_desc)));
    CK(hipMemset(src, 0, len));
    CK(hipMemcpy(dh, hh.data(), n * sizeof(bhg_handle), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_gen, dim3(n), dim3(256), 0, 0, src, dh, n, R);
    CK(hipDeviceSynchronize());

    uint32_t *tabs = nullptr;  // precomputed global tables (lab kernels copy what they need into LDS)
    CK(hipMalloc(&tabs, kLabTabBytes));
    lab_init_tables(tabs);

    bhg_ctx *ctx = bhg_create(0, 0);
    if (!ctx) { fprintf(stderr, "bhg_create failed\n"); return 1; }
    hipStream_t s = (hipStream_t)bhg_stream(ctx);
    // clocks ramp over the first ~100 launches (profiles/r1_s6_clock_ramp_probe.txt): warm up first
    {
        const int warm = getenv("LAB_WARM") ? atoi(getenv("LAB_WARM")) : 300;
        for (int it = 0; it < warm; it++)
            if (bhg_decode_batch(ctx, src, len, dh, n, 0, nullptr, ref, nullptr, 0, nullptr, s) != 0) return 1;
        CK(hipStreamSynchronize(s));
    }
    // production reference
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> ts;
    for (int it = 0; it < iters + 2; it++) {
        CK(hipEventRecord(a, s));
        if (bhg_decode_batch(ctx, src, len, dh, n, 0, nullptr, ref, nullptr, 0, nullptr, s) != 0) {
            fprintf(stderr, "decode failed: %s\n", bhg_last_error(ctx));
            return 1;
        }
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (it >= 2) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const double gb = (double)n * 1132 / 1e9;
    printf("%-34s median %.4f ms  best %.4f  %.0f GB/s alg (%.3f of 8 TB/s)\n", "production(default)", ts[ts.size() / 2],
           ts[0], gb / ts[ts.size() / 2] * 1e3, gb / ts[ts.size() / 2] / 8.0 * 1e3);
    std::vector<bhg_desc> hr(n), ho(n);
    CK(hipMemcpy(hr.data(), ref, n * sizeof(bhg_desc), hipMemcpyDeviceToHost));
    for (int k = 0; k < kNumLab; k++) {
        if (only) {
            bool hit = false;
            char buf[256];
            snprintf(buf, sizeof buf, "%s", only);
            for (char *tok = strtok(buf, ","); tok; tok = strtok(nullptr, ","))
                if (tok[0] == '=' ? strcmp(kLab[k].name, tok + 1) == 0 : strstr(kLab[k].name, tok) != nullptr) hit = true;
            if (!hit) continue;
        }
        CK(hipMemset(out, 0xAB, n * sizeof(bhg_desc)));
        float best;
        float med = time_it(kLab[k].fn, src, len, dh, n, out, tabs, s, iters, &best);
        CK(hipMemcpy(ho.data(), out, n * sizeof(bhg_desc), hipMemcpyDeviceToHost));
        uint32_t bad = 0, first = ~0u;
        for (uint32_t i = 0; i < n; i++)
            if (memcmp(&hr[i], &ho[i], sizeof(bhg_desc)) != 0) {
                if (first == ~0u) first = i;
                bad++;
            }
        printf("%-34s median %.4f ms  best %.4f  %.0f GB/s alg (%.3f)  %s", kLab[k].name, med, best, gb / med * 1e3,
               gb / med / 8.0 * 1e3, kLab[k].diag ? "[diag]" : (bad ? "MISMATCH" : "bit-exact"));
        if (bad && !kLab[k].diag)
            printf(" %u bad, first %u crc %08x vs %08x st %u", bad, first, ho[first].crc, hr[first].crc, ho[first].status);
        printf("\n");
        fflush(stdout);
    }
    bhg_destroy(ctx);
    return 0;
}
