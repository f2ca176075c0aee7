// stream_lab.hip -- development harness (not product code): times
// configurations of k_decode_stream (bhg_decode_stream.h) on the C2 batch
// (1M x 1076 B records in 128 MiB tables, device-resident) against the
// library's bhg_decode_batch and checks every descriptor byte for byte.
// Optionally shuffles the handle order (scattered reads, e.g. MultiGet).
//
// build: make -C scripts/lab stream_lab      run: scripts/lab/stream_lab [iters] [filter] [shuffle]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <random>
#include <vector>

#include "../../bitalosdb_amd/csrc/bhg_decode_stream.h"
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

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// record i: header {40, 1024, fn}, key 32 B, trailer (i+1)<<8|1, value 1024 B
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
            x = (uint8_t)(48 + mix64(((uint64_t)i << 12) ^ b ^ 0xB17A105DBull) % 75);
        }
        r[b] = x;
    }
}

// linear read of the same bytes (the access-pattern floor)
__global__ __launch_bounds__(256) void k_linear(const uint8_t *__restrict__ src, uint64_t len, uint32_t *sink) {
    const uint64_t base = (uint64_t)src;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t W = (uint64_t)gridDim.x * 4, w0 = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint64_t nt = len / 8192;
    uint32_t acc = 0;
    for (uint64_t t = w0; t < nt; t += W) {
#pragma unroll
        for (uint32_t o = 0; o < 8192; o += 1024) {
            const u32x4 x = gld<u32x4>(base + t * 8192 + o + 16 * lane);
            acc ^= x.x ^ x.y ^ x.z ^ x.w;
        }
    }
    if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

// access-pattern probes at the stream kernel's occupancy: one workgroup of
// 64*WPB threads per CU holding ~156 KiB of LDS; each wave streams passes of
// 64 lanes x 128 B (lane-contiguous windows, LANE=1) or coalesced 1 KiB rows
// (LANE=0), PF passes in flight
template <int WPB, int LANE, int PF>
__global__ __launch_bounds__(64 * WPB) void k_probe(const uint8_t *__restrict__ src, uint64_t len, uint32_t *sink) {
    __shared__ uint32_t pad[39000];
    pad[threadIdx.x] = threadIdx.x;
    __syncthreads();
    const uint64_t base = (uint64_t)src;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t W = (uint64_t)gridDim.x * WPB, w0 = (threadIdx.x >> 6) * gridDim.x + blockIdx.x;
    const uint64_t np = len / 8192;
    uint32_t acc = pad[(threadIdx.x * 7) & 1023];
    for (uint64_t t = w0; t < np; t += W * PF) {
        u32x4 x[PF][8];
#pragma unroll
        for (int f = 0; f < PF; f++) {
            const uint64_t tt = t + f * W < np ? t + f * W : t;
#pragma unroll
            for (int q = 0; q < 8; q++)
                x[f][q] = LANE ? gld<u32x4>(base + tt * 8192 + 128 * lane + 16 * q) : gld<u32x4>(base + tt * 8192 + 1024 * q + 16 * lane);
        }
#pragma unroll
        for (int f = 0; f < PF; f++)
#pragma unroll
            for (int q = 0; q < 8; q++) acc ^= x[f][q].x ^ x[f][q].y ^ x[f][q].z ^ x[f][q].w;
    }
    if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

struct Ctx {
    const uint8_t *src;
    uint64_t len;
    const bhg_handle *h;
    uint32_t n;
    bhg_desc *out;
    const uint32_t *exp;
    const uint32_t *tab;
    uint32_t *sink;
    hipStream_t s;
    int cus;
};
typedef void (*launch_fn)(const Ctx &);
// table sets: (128,4) (128,2) (256,4) (256,8)
static int tab_index(int win, int nch) { return win == 128 ? (nch == 4 ? 0 : 1) : (nch == 4 ? 2 : 3); }

template <int NCH, int WPB, int WIN, int KO, int PIPE = 0>
static void L_stream(const Ctx &c) {
    constexpr int WGS = 1;
    const uint64_t tiles = (c.n + 63) / 64;
    uint64_t need = (tiles + WPB - 1) / WPB, cap = (uint64_t)c.cus * WGS;
    uint32_t grid = (uint32_t)(need < cap ? need : cap);
    hipLaunchKernelGGL((k_decode_stream<0, NCH, WPB, WIN, PIPE, KO>), dim3(grid), dim3(64 * WPB), 0, c.s, c.src, c.len, c.h, c.n,
                       c.exp, c.out, nullptr, c.tab + tab_index(WIN, NCH) * kStreamTabWords);
}
template <int WPB, int LANE, int PF>
static void L_probe(const Ctx &c) {
    hipLaunchKernelGGL((k_probe<WPB, LANE, PF>), dim3(c.cus), dim3(64 * WPB), 0, c.s, c.src, c.len, c.sink);
}
static void L_linear(const Ctx &c) {
    hipLaunchKernelGGL(k_linear, dim3(c.cus * 8), dim3(256), 0, c.s, c.src, c.len, c.sink);
}

struct Lab {
    const char *name;
    launch_fn fn;
    bool diag;
};
static const Lab kLab[] = {
    {"stream_c4", L_stream<4, 8, 128, 0>, false},
    {"stream_pipe", L_stream<4, 8, 128, 0, 1>, false},
    {"stream_pipe2", L_stream<4, 8, 128, 0, 2>, false},
    {"stream_w256_c4", L_stream<4, 8, 256, 0>, false},
    {"stream_w256_c8", L_stream<8, 8, 256, 0>, false},
    {"stream_w16", L_stream<4, 16, 128, 0>, false},
    {"stream_w12", L_stream<4, 12, 128, 0>, false},
    {"bis_probe", L_stream<4, 8, 128, 59 | 256 | 512 | 1024>, true},
    {"bis_probe_desc", L_stream<4, 8, 128, 59 | 256 | 512>, true},
    {"bis_probe_absorb", L_stream<4, 8, 128, 59 | 256 | 1024>, true},
    {"bis_probe_locate", L_stream<4, 8, 128, 43 | 512 | 1024>, true},
    {"bis_probe_locate_u", L_stream<4, 8, 128, 59 | 512 | 1024>, true},
    {"bis_probe_nohdr", L_stream<4, 8, 128, 63 | 4 | 256 | 512 | 1024>, true},
    {"ko_nodesc", L_stream<4, 8, 128, 64>, true},
    {"ko_noztab", L_stream<4, 8, 128, 128>, true},
    {"ko_all_nodesc", L_stream<4, 8, 128, 63 | 64 | 128>, true},
    {"ko_uniform_locate", L_stream<4, 8, 128, 16>, false},
    {"ko_noscan", L_stream<4, 8, 128, 2>, true},
    {"ko_nohdr", L_stream<4, 8, 128, 4>, true},
    {"ko_nofold", L_stream<4, 8, 128, 8>, true},
    {"ko_nohead", L_stream<4, 8, 128, 32>, true},
    {"ko_nocrc", L_stream<4, 8, 128, 1>, true},
    {"ko_nocrc_noscan_nohdr", L_stream<4, 8, 128, 7>, true},
    {"ko_nocrc_noscan_nohdr_uloc", L_stream<4, 8, 128, 23>, true},
    {"ko_all", L_stream<4, 8, 128, 63>, true},
    {"probe_w8_lane_pf1", L_probe<8, 1, 1>, true},
};

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20;
    const char *only = argc > 2 && strcmp(argv[2], "all") ? argv[2] : nullptr;
    const bool shuffle = argc > 3 && atoi(argv[3]) != 0;
    const bool use_exp = getenv("LAB_EXPECTED") != nullptr;
    const uint32_t n = 1000000, L = 1076;
    const uint32_t R = (uint32_t)((128ull << 20) / L + 1);  // records per 128 MiB table
    const uint64_t tbytes = (uint64_t)R * L + 12;
    std::vector<bhg_handle> hh(n);
    for (uint32_t i = 0; i < n; i++) hh[i] = bhg_handle{(uint64_t)(i / R) * tbytes + (uint64_t)(i % R) * L, L, 0};
    const uint64_t len = hh[n - 1].offset + L + 12;
    uint8_t *src;
    bhg_handle *dh;
    bhg_desc *ref, *out;
    uint32_t *tab, *sink, *dexp;
    CK(hipMalloc(&src, len));
    CK(hipMalloc(&dh, n * sizeof(bhg_handle)));
    CK(hipMalloc(&ref, n * sizeof(bhg_desc)));
    CK(hipMalloc(&out, n * sizeof(bhg_desc)));
    CK(hipMalloc(&sink, 4096));
    CK(hipMalloc(&dexp, n * 4));
    CK(hipMemset(src, 0, len));
    CK(hipMemcpy(dh, hh.data(), n * sizeof(bhg_handle), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_gen, dim3(n), dim3(256), 0, 0, src, dh, n, R);
    CK(hipDeviceSynchronize());
    if (shuffle) {
        std::mt19937_64 rng(7);
        std::shuffle(hh.begin(), hh.end(), rng);
        CK(hipMemcpy(dh, hh.data(), n * sizeof(bhg_handle), hipMemcpyHostToDevice));
    }
    std::vector<uint32_t> ht(4 * kStreamTabWords);
    build_stream_tab(ht.data(), 128, 4);
    build_stream_tab(ht.data() + kStreamTabWords, 128, 2);
    build_stream_tab(ht.data() + 2 * kStreamTabWords, 256, 4);
    build_stream_tab(ht.data() + 3 * kStreamTabWords, 256, 8);
    CK(hipMalloc(&tab, ht.size() * 4));
    CK(hipMemcpy(tab, ht.data(), ht.size() * 4, hipMemcpyHostToDevice));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));

    bhg_ctx *ctx = bhg_create(0, 0);
    if (!ctx) { fprintf(stderr, "bhg_create failed\n"); return 1; }
    hipStream_t s = (hipStream_t)bhg_stream(ctx);
    // reference descriptors (library), then its CRCs as expected_crc
    if (bhg_decode_batch(ctx, src, len, dh, n, 0, nullptr, ref, nullptr, 0, nullptr, s) != 0) return 1;
    CK(hipStreamSynchronize(s));
    std::vector<bhg_desc> hr(n), ho(n);
    CK(hipMemcpy(hr.data(), ref, n * sizeof(bhg_desc), hipMemcpyDeviceToHost));
    {
        std::vector<uint32_t> e(n);
        for (uint32_t i = 0; i < n; i++) e[i] = hr[i].crc;
        CK(hipMemcpy(dexp, e.data(), n * 4, hipMemcpyHostToDevice));
    }
    const uint32_t nrun = getenv("LAB_N") ? (uint32_t)atoi(getenv("LAB_N")) : n;
    Ctx c{src, len, dh, nrun, out, use_exp ? dexp : nullptr, tab, sink, s, prop.multiProcessorCount};
    // clocks ramp over the first ~100 launches: warm up
    const int warm = getenv("LAB_WARM") ? atoi(getenv("LAB_WARM")) : 300;
    for (int it = 0; it < warm; it++)
        if (bhg_decode_batch(ctx, src, len, dh, n, 0, c.exp, ref, nullptr, 0, nullptr, s) != 0) return 1;
    CK(hipStreamSynchronize(s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const double gb = (double)n * 1132 / 1e9;
    auto report = [&](const char *name, std::vector<float> &ts, const char *tag) {
        std::sort(ts.begin(), ts.end());
        printf("%-26s median %.4f ms  best %.4f  %.0f GB/s alg (%.3f of 8 TB/s)  %s\n", name, ts[ts.size() / 2], ts[0],
               gb / ts[ts.size() / 2] * 1e3, gb / ts[ts.size() / 2] / 8.0 * 1e3, tag);
        fflush(stdout);
    };
    {
        std::vector<float> ts;
        for (int it = 0; it < iters; it++) {
            CK(hipEventRecord(a, s));
            if (bhg_decode_batch(ctx, src, len, dh, nrun, 0, c.exp, ref, nullptr, 0, nullptr, s) != 0) return 1;
            CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            ts.push_back(ms);
        }
        report("library(default)", ts, "");
    }
    for (const Lab &l : kLab) {
        if (only) {
            bool hit = false;
            char buf[256];
            snprintf(buf, sizeof buf, "%s", only);
            for (char *tok = strtok(buf, ","); tok; tok = strtok(nullptr, ","))
                if (tok[0] == '=' ? strcmp(l.name, tok + 1) == 0 : strstr(l.name, tok) != nullptr) hit = true;
            if (!hit) continue;
        }
        CK(hipMemset(out, 0xAB, n * sizeof(bhg_desc)));
        l.fn(c);
        l.fn(c);
        CK(hipStreamSynchronize(s));
        std::vector<float> ts;
        for (int it = 0; it < iters; it++) {
            CK(hipEventRecord(a, s));
            l.fn(c);
            CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            ts.push_back(ms);
        }
        CK(hipGetLastError());
        char tag[160] = "[diag]";
        if (!l.diag) {
            CK(hipMemcpy(ho.data(), out, n * sizeof(bhg_desc), hipMemcpyDeviceToHost));
            uint32_t bad = 0, first = ~0u;
            for (uint32_t i = 0; i < nrun; i++)
                if (memcmp(&hr[i], &ho[i], sizeof(bhg_desc)) != 0) {
                    if (first == ~0u) first = i;
                    bad++;
                }
            if (bad)
                snprintf(tag, sizeof tag, "MISMATCH %u bad, first %u crc %08x vs %08x st %u/%u", bad, first,
                         ho[first].crc, hr[first].crc, ho[first].status, hr[first].status);
            else
                snprintf(tag, sizeof tag, "bit-exact");
        }
        report(l.name, ts, tag);
    }
    bhg_destroy(ctx);
    return 0;
}
