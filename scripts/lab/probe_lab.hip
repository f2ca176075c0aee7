// probe_lab.hip -- development harness (not product code): memory-pattern
// probes for the C2 decode on the 1M x 1076 B batch layout (1.08 GB).
// Each probe streams the whole buffer in passes of 64 lanes x 128-B windows
// (8 KB contiguous per wave pass, one workgroup of 8 waves per CU, LDS padded
// like the decode kernels) and varies one thing at a time:
//   OFF   byte offset of the windows from 128-B alignment
//   HDR   4 extra 16-B loads per pass (8 of 64 lanes real, the rest one shared address)
//   X8    one extra 8-B load per lane at the window end (straddle word)
//   CRC   slice-by-4 CRC of the window (4 chains, Crc4Perm tables in LDS)
//   PF    passes kept in flight per wave (1 or 2)
// build: make -C scripts/lab probe_lab     run: scripts/lab/probe_lab [iters]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "../../bitalosdb_amd/csrc/bhg_crc_tables.h"
#include "../../bitalosdb_amd/csrc/bhg_device.h"

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

using namespace bhg;
static uint8_t *g_dout;

template <int OFF, int HDR, int X8, int CRC, int PF, int ORD = 0, int ST = 0, int BP = 0, int NTL = 0>
__global__ __launch_bounds__(512) void k_probe(const uint8_t *__restrict__ src, uint64_t len, uint32_t *sink, uint8_t *dout) {
    __shared__ __attribute__((aligned(16))) uint32_t T[Crc4Perm::kWords + 6000];
    if (CRC) Crc4Perm::fill(T);
    else T[threadIdx.x] = threadIdx.x;
    __syncthreads();
    const Crc4Perm crc(T);
    const uint64_t base = (uint64_t)src + OFF;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t W = (uint64_t)gridDim.x * 8, w0 = (threadIdx.x >> 6) * gridDim.x + blockIdx.x;
    const uint64_t np = (len - 256) / 8192;
    uint32_t acc = T[(threadIdx.x * 7) & 1023];
    const uint64_t ntile = ORD == 1 ? np / 9 : np / 72;
    uint64_t it_tile = (ORD == 1 || ORD == 3) ? w0 : blockIdx.x, it_k = 0;
    const uint32_t wv = threadIdx.x >> 6;
    const uint64_t ntile3 = (len - 80000) / 68864;
    uint32_t ntiles_done = 0;
    for (uint64_t t = ORD == 0 ? w0 : (ORD == 1 || ORD == 3 ? w0 * 9 : blockIdx.x * 72 + wv);;) {
        if (ORD == 0 && t >= np) break;
        if ((ORD == 1 || ORD == 2) && it_tile >= ntile) break;
        if (ORD == 3 && it_tile >= ntile3) break;
        uint32_t w[PF][34];
        uint32_t hw[PF][16];
#pragma unroll
        for (int f = 0; f < PF; f++) {
            const uint64_t tt = ORD == 0 ? (t + f * W < np ? t + f * W : t) : t;
            uint64_t a = ORD == 3 ? base + it_tile * 68864 + it_k * 8192 + 128 * lane : base + tt * 8192 + 128 * lane;
            const uint64_t arow = (ORD == 3 ? base + it_tile * 68864 + it_k * 8192 : base + tt * 8192) + 16 * lane;
            if (BP) a = (uint64_t)__shfl((int64_t)a, (int)((lane + 1) & 63), 64) - 128 * ((lane + 1) & 63) + 128 * lane;  // LDS round trip before issue
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const uint64_t la = (NTL & 2) ? arow + 1024 * q : a + 16 * q;
                const u32x4 x = (NTL & 1) ? __builtin_nontemporal_load(reinterpret_cast<const BHG_GLOBAL u32x4 *>(la)) : gld<u32x4_a4>(la);
                w[f][4 * q] = x.x; w[f][4 * q + 1] = x.y; w[f][4 * q + 2] = x.z; w[f][4 * q + 3] = x.w;
            }
            if (X8) {
                typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
                typedef u32x2 u32x2_a4 __attribute__((aligned(4)));
                const u32x2 y = gld<u32x2_a4>(a + 128);
                w[f][32] = y.x; w[f][33] = y.y;
            } else {
                w[f][32] = w[f][33] = 0;
            }
            if (HDR) {
                const uint64_t ha = (lane & 7) == 0 ? a + 4 : (uint64_t)src;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const u32x4 x = gld<u32x4_a4>(ha + 16 * q);
                    hw[f][4 * q] = x.x; hw[f][4 * q + 1] = x.y; hw[f][4 * q + 2] = x.z; hw[f][4 * q + 3] = x.w;
                }
            }
        }
#pragma unroll
        for (int f = 0; f < PF; f++) {
            if (CRC) {
                uint32_t cc[4] = {0, 0, 0, 0};
#pragma unroll
                for (int u = 0; u < 8; u++)
#pragma unroll
                    for (int c = 0; c < 4; c++) cc[c] = crc.word(cc[c], w[f][8 * c + u]);
                acc ^= cc[0] ^ cc[1] ^ cc[2] ^ cc[3] ^ w[f][32] ^ w[f][33];
            } else {
#pragma unroll
                for (int q = 0; q < 34; q++) acc ^= w[f][q];
            }
            if (HDR) {
#pragma unroll
                for (int q = 0; q < 16; q++) acc += hw[f][q];
            }
        }
        if (ST == 2 && ORD == 1 && it_k == 0 && it_tile != w0) {  // previous tile's descriptors, after this pass's loads
            uint2 *o = reinterpret_cast<uint2 *>(dout + ((it_tile - W) * 64 + lane) * 40);
            o[0] = make_uint2(acc, 1); o[1] = make_uint2(acc, 2); o[2] = make_uint2(acc, 3); o[3] = make_uint2(acc, 4); o[4] = make_uint2(acc, 5);
        }
        if (ST >= 1 && ST != 2 && (ORD == 1 || ORD == 3) && it_k == 8) {  // this tile's descriptors at the tile end
            __builtin_amdgcn_s_waitcnt(0x0F70);
            if (ST == 1) {  // AoS 40 B per lane, 8-B pieces
                uint2 *o = reinterpret_cast<uint2 *>(dout + (it_tile * 64 + lane) * 40);
                o[0] = make_uint2(acc, 1); o[1] = make_uint2(acc, 2); o[2] = make_uint2(acc, 3); o[3] = make_uint2(acc, 4); o[4] = make_uint2(acc, 5);
            } else if (ST == 3) {  // same bytes, coalesced 16 B per lane
                uint8_t *o = dout + it_tile * 64 * 40;
                u32x4 v = {acc, 1, 2, 3};
                gst<u32x4>((uint64_t)o + 16 * lane, v);
                gst<u32x4>((uint64_t)o + 1024 + 16 * lane, v);
                if (lane < 32) gst<u32x4>((uint64_t)o + 2048 + 16 * lane, v);
            } else if (ST == 4) {  // AoS, 4-B pieces
                uint32_t *o = reinterpret_cast<uint32_t *>(dout + (it_tile * 64 + lane) * 40);
#pragma unroll
                for (int q = 0; q < 10; q++) o[q] = acc + q;
            } else if (ST == 5) {  // SoA: 10 arrays of u32
                uint32_t *o = reinterpret_cast<uint32_t *>(dout);
#pragma unroll
                for (int q = 0; q < 10; q++) o[(uint64_t)q * (1u << 20) + it_tile * 64 + lane] = acc + q;
            } else if (ST == 7) {  // AoS into a per-wave 2.5 KB slot reused every tile (stays in L2)
                uint2 *o = reinterpret_cast<uint2 *>(dout + (w0 * 64 + lane) * 40);
                o[0] = make_uint2(acc, 1); o[1] = make_uint2(acc, 2); o[2] = make_uint2(acc, 3); o[3] = make_uint2(acc, 4); o[4] = make_uint2(acc, 5);
            } else if (ST == 8) {  // coalesced 16 B per lane, non-temporal
                u32x4 *o = reinterpret_cast<u32x4 *>(dout + it_tile * 64 * 40);
                u32x4 v = {acc, 1, 2, 3};
                __builtin_nontemporal_store(v, o + lane);
                __builtin_nontemporal_store(v, o + 64 + lane);
                if (lane < 32) __builtin_nontemporal_store(v, o + 128 + lane);
            } else if (ST == 6) {  // AoS 8-B pieces, non-temporal
                uint64_t *o = reinterpret_cast<uint64_t *>(dout + (it_tile * 64 + lane) * 40);
#pragma unroll
                for (int q = 0; q < 5; q++) __builtin_nontemporal_store((uint64_t)acc << 32 | q, o + q);
            }
        }
        if (ST == 9 && ORD == 0) {  // chip-linear: 8 lanes store one 40-B descriptor each per pass (~7.6 records / 8 KB)
            __builtin_amdgcn_s_waitcnt(0x0F70);
            if ((lane & 7) == 0) {
                uint64_t *o = reinterpret_cast<uint64_t *>(dout + ((t * 8 + (lane >> 3)) % (1u << 20)) * 40);
#pragma unroll
                for (int q = 0; q < 5; q++) __builtin_nontemporal_store((uint64_t)acc << 32 | q, o + q);
            }
        }
        if (ST == 10 && ORD == 3 && it_k == 8) ntiles_done++;
        if (ORD == 0) t += W * PF;
        else if (ORD == 1 || ORD == 3) {
            if (++it_k == 9) { it_k = 0; it_tile += W; t = it_tile * 9; } else t++;
        } else {
            if (++it_k == 9) { it_k = 0; it_tile += gridDim.x; t = it_tile * 72 + wv; } else t += 8;
        }
    }
    if (ST == 10) {  // all of this wave's descriptors in one burst at the end
        for (uint32_t k = 0; k < ntiles_done; k++) {
            uint64_t *o = reinterpret_cast<uint64_t *>(dout + (((uint64_t)(w0 + (uint64_t)k * W)) * 64 + lane) * 40);
#pragma unroll
            for (int q = 0; q < 5; q++) __builtin_nontemporal_store((uint64_t)acc << 32 | q, o + q);
        }
    }
    if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

template <int OFF, int HDR, int X8, int CRC, int PF, int ORD = 0, int ST = 0, int BP = 0, int NTL = 0>
static void L(const uint8_t *src, uint64_t len, uint32_t *sink, int cus, hipStream_t s) {
    hipLaunchKernelGGL((k_probe<OFF, HDR, X8, CRC, PF, ORD, ST, BP, NTL>), dim3(cus), dim3(512), 0, s, src, len, sink, g_dout);
}

// 8 reader waves stream tiles (tile9 order); a 9th wave per block writes 40 B per record for the
// block's share of the records (plain 16-B stores), like a dedicated descriptor writer
__global__ __launch_bounds__(576) void k_probe_writer(const uint8_t *__restrict__ src, uint64_t len, uint32_t *sink, uint8_t *dout) {
    __shared__ uint32_t T[32768 + 6000];
    T[threadIdx.x] = threadIdx.x;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t base = (uint64_t)src;
    uint32_t acc = T[(threadIdx.x * 7) & 1023];
    if (wv == 8) {
        const uint64_t total = 40ull * 1000000, per = (total / gridDim.x) & ~1023ull;
        const uint64_t o = (uint64_t)dout + per * blockIdx.x;
        for (uint64_t b = 0; b < per; b += 1024) gst<u32x4>(o + b + 16 * lane, u32x4{acc, 1, 2, (uint32_t)b});
        return;
    }
    const uint64_t W = (uint64_t)gridDim.x * 8, w0 = wv * gridDim.x + blockIdx.x;
    const uint64_t ntile = (len - 80000) / 68864;
    for (uint64_t tile = w0; tile < ntile; tile += W)
        for (uint32_t k = 0; k < 9; k++) {
            const uint64_t a = base + tile * 68864 + k * 8192 + 128 * lane;
            uint32_t w[32];
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const u32x4 x = gld<u32x4>(a + 16 * q);
                w[4 * q] = x.x; w[4 * q + 1] = x.y; w[4 * q + 2] = x.z; w[4 * q + 3] = x.w;
            }
#pragma unroll
            for (int q = 0; q < 32; q++) acc ^= w[q];
        }
    if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}
static void L_writer(const uint8_t *src, uint64_t len, uint32_t *sink, int cus, hipStream_t s) {
    hipLaunchKernelGGL(k_probe_writer, dim3(cus), dim3(576), 0, s, src, len, sink, g_dout);
}

// tile-kernel phase-2 load shapes (8 records x 8 lanes per round, 8 rounds per 64-record tile, 1076-B
// records, window region = record + 52 .. + 1076): GRP 0 = today's lane-own-window (lane (g, j) reads
// its window 8 - j as 8 x 16 B), GRP 1 = column chunks (instruction k: lane (g, j) reads chunk j of window k,
// 128 contiguous bytes per group per instruction); NT: non-temporal loads; ST: 40-B descriptor per lane-record
template <int GRP, int NT, int ST>
__global__ __launch_bounds__(512) void k_probe_round(const uint8_t *__restrict__ src, uint64_t len, uint32_t *sink,
                                                     uint8_t *dout) {
    __shared__ uint32_t T[32768 + 6000];
    T[threadIdx.x] = threadIdx.x;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, g = lane >> 3, j = lane & 7;
    const uint64_t base = (uint64_t)src;
    const uint64_t W = (uint64_t)gridDim.x * 8, w0 = (threadIdx.x >> 6) * gridDim.x + blockIdx.x;
    const uint64_t ntile = (len - 80000) / 68864;
    uint32_t acc = T[(threadIdx.x * 7) & 1023];
    for (uint64_t tile = w0; tile < ntile; tile += W) {
        for (uint32_t s = 0; s < 8; s++) {
            const uint64_t region = base + tile * 68864 + (uint64_t)(8 * s + g) * 1076 + 52;
            u32x4 x[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint64_t a = GRP ? region + 128 * k + 16 * j : region + 128 * (7 - j) + 16 * k;
                x[k] = NT ? __builtin_nontemporal_load(reinterpret_cast<const BHG_GLOBAL u32x4 *>(a)) : gld<u32x4_a4>(a);
            }
#pragma unroll
            for (int k = 0; k < 8; k++) acc ^= x[k].x ^ x[k].y ^ x[k].z ^ x[k].w;
        }
        if (ST) {
            __builtin_amdgcn_s_waitcnt(0x0F70);
            uint64_t *o = reinterpret_cast<uint64_t *>(dout + ((tile * 64 + lane) % (1u << 20)) * 40);
#pragma unroll
            for (int q = 0; q < 5; q++) __builtin_nontemporal_store((uint64_t)acc << 32 | q, o + q);
        }
    }
    if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}
template <int GRP, int NT, int ST>
static void LR(const uint8_t *src, uint64_t len, uint32_t *sink, int cus, hipStream_t s) {
    hipLaunchKernelGGL((k_probe_round<GRP, NT, ST>), dim3(cus), dim3(512), 0, s, src, len, sink, g_dout);
}
typedef void (*fn_t)(const uint8_t *, uint64_t, uint32_t *, int, hipStream_t);
struct P {
    const char *name;
    fn_t fn;
};
static const P kP[] = {
    {"aligned", L<0, 0, 0, 0, 1>},
    {"tile9", L<0, 0, 0, 0, 1, 1>},
    {"tile9_off52", L<52, 0, 0, 0, 1, 1>},
    {"tile9r", L<0, 0, 0, 0, 1, 3>},
    {"tile9r_off4", L<4, 0, 0, 0, 1, 3>},
    {"tile9r_crc_x8_hdr_st", L<4, 1, 1, 1, 1, 3, 1>},
    {"tile9r_st", L<4, 0, 0, 0, 1, 3, 1>},
    {"tile9r_writer_wave", L_writer},
    {"tile9r_ntld", L<0, 0, 0, 0, 1, 3, 0, 0, 1>},
    {"tile9r_st_nt", L<0, 0, 0, 0, 1, 3, 6>},
    {"linear_st_nt", L<0, 0, 0, 0, 1, 0, 9>},
    {"tile9r_st_burst", L<0, 0, 0, 0, 1, 3, 10>},
    {"round_own", LR<0, 0, 0>},
    {"round_col", LR<1, 0, 0>},
    {"round_col_nt", LR<1, 1, 0>},
    {"round_own_st", LR<0, 0, 1>},
    {"round_col_st", LR<1, 0, 1>},
    {"round_col_nt_st", LR<1, 1, 1>},
    {"tile9r_coal", L<0, 0, 0, 0, 1, 3, 0, 0, 2>},
    {"tile9r_coal_nt", L<0, 0, 0, 0, 1, 3, 0, 0, 3>},
    {"tile9r_coal_st_nt", L<0, 0, 0, 0, 1, 3, 6, 0, 2>},
    {"tile9r_coalnt_st_nt", L<0, 0, 0, 0, 1, 3, 6, 0, 3>},
    {"tile9r_coalnt_st", L<0, 0, 0, 0, 1, 3, 1, 0, 3>},
    {"tile9r_coalnt_crc_hdr_st_nt", L<0, 1, 0, 1, 1, 3, 6, 0, 3>},
    {"tile9r_coal_crc_hdr_st_nt", L<0, 1, 0, 1, 1, 3, 6, 0, 2>},
    {"tile9r_crc_x8_hdr_st_burst", L<4, 1, 1, 1, 1, 3, 10>},
    {"linear_crc_x8_hdr_st_nt", L<52, 1, 1, 1, 1, 0, 9>},
    {"tile9r_st_coal_nt", L<0, 0, 0, 0, 1, 3, 8>},
    {"tile9r_ntld_st_nt", L<0, 0, 0, 0, 1, 3, 6, 0, 1>},
    {"tile9r_ntld_st_coal_nt", L<0, 0, 0, 0, 1, 3, 8, 0, 1>},
    {"tile9r_crc_x8_hdr_st_nt", L<4, 1, 1, 1, 1, 3, 6>},
    {"tile9r_crc_x8_hdr_ntld_st_nt", L<4, 1, 1, 1, 1, 3, 6, 0, 1>},
    {"tile9_st_end", L<0, 0, 0, 0, 1, 1, 1>},
    {"tile9_st_coal", L<0, 0, 0, 0, 1, 1, 3>},
    {"tile9_st_aos4", L<0, 0, 0, 0, 1, 1, 4>},
    {"tile9_st_soa", L<0, 0, 0, 0, 1, 1, 5>},
    {"tile9_st_nt", L<0, 0, 0, 0, 1, 1, 6>},
    {"tile9_st_slot", L<0, 0, 0, 0, 1, 1, 7>},
    {"tile9_st_coal_nt", L<0, 0, 0, 0, 1, 1, 8>},
    {"tile9_crc_x8_hdr_st_nt", L<52, 1, 1, 1, 1, 1, 6>},
    {"tile9_crc_x8_hdr_st_coal_nt", L<52, 1, 1, 1, 1, 1, 8>},
    {"tile9_crc_x8_hdr_st_end", L<52, 1, 1, 1, 1, 1, 1>},
    {"tile9_crc_x8_hdr_st_coal", L<52, 1, 1, 1, 1, 1, 3>},
    {"wgtile72", L<0, 0, 0, 0, 1, 2>},
    {"tile9_crc_x8_hdr", L<52, 1, 1, 1, 1, 1>},
    {"wgtile72_crc_x8_hdr", L<52, 1, 1, 1, 1, 2>},
    {"off4", L<4, 0, 0, 0, 1>},
    {"off52", L<52, 0, 0, 0, 1>},
    {"off64", L<64, 0, 0, 0, 1>},
    {"aligned_x8", L<0, 0, 1, 0, 1>},
    {"aligned_hdr", L<0, 1, 0, 0, 1>},
    {"off52_x8_hdr", L<52, 1, 1, 0, 1>},
    {"aligned_pf2", L<0, 0, 0, 0, 2>},
    {"aligned_crc", L<0, 0, 0, 1, 1>},
    {"aligned_crc_pf2", L<0, 0, 0, 1, 2>},
    {"off52_crc", L<52, 0, 0, 1, 1>},
    {"off52_x8_hdr_crc", L<52, 1, 1, 1, 1>},
    {"off52_x8_hdr_crc_pf2", L<52, 1, 1, 1, 2>},
};

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 30;
    const uint64_t len = 1076000000ull + 4096;
    uint8_t *src;
    uint32_t *sink;
    CK(hipMalloc(&src, len));
    CK(hipMalloc(&sink, 4096));
    CK(hipMalloc(&g_dout, 48ull << 20));  // SoA: 10 x 4 MiB
    CK(hipMemset(src, 0x5a, len));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    for (int it = 0; it < 300; it++) kP[0].fn(src, len, sink, cus, s);  // clocks ramp: warm up
    CK(hipStreamSynchronize(s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const double gb = 1.076;
    for (const P &p : kP) {
        p.fn(src, len, sink, cus, s);
        std::vector<float> ts;
        for (int it = 0; it < iters; it++) {
            CK(hipEventRecord(a, s));
            p.fn(src, len, sink, cus, s);
            CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            ts.push_back(ms);
        }
        CK(hipGetLastError());
        std::sort(ts.begin(), ts.end());
        printf("%-24s median %.4f ms  best %.4f  %.0f GB/s\n", p.name, ts[ts.size() / 2], ts[0], gb / ts[ts.size() / 2] * 1e3);
        fflush(stdout);
    }
    return 0;
}
