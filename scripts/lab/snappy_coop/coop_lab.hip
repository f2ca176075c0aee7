// coop_lab.hip -- LAB (not product code): the first two stages of a wave-cooperative snappy block
// decode (VERDICT r3 #2 / SURVEY 7 step 4), timed on the C3 batch to bound what such a decoder can
// reach before any byte is moved.  One wave per block:
//   1. stage the block's stream in LDS (16 B per lane, the next block's chunk prefetched into VGPRs);
//   2. tag discovery in parallel: lane l computes, for every byte position p = l + 64 j of the stream,
//      where an element starting at p would end (decode_other.go's tag rules) -> next[p] (u16, LDS);
//   3. the true element starts: the chain hdr -> next[hdr] -> ... (one dependent LDS read per
//      element, wave-uniform), counted per block.
// MODE 1 stops after stage 1 (staging floor).  Output: the element count per block (checked on the
// host against a CPU parse of the same streams).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../../include/bithashgpu.h"

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4u __attribute__((aligned(1)));
typedef uint64_t u64u __attribute__((aligned(1), may_alias));
typedef u32x4 u32x4_lds_u __attribute__((aligned(1), may_alias));

constexpr uint32_t CW = 4;           // waves per workgroup
constexpr uint32_t SB = 1152;        // stream bytes per wave (streams <= 1,088 B here)
constexpr uint32_t PER_WAVE = SB + 64 + 2 * SB;

template <int MODE>
__global__ __launch_bounds__(64 * CW) void k_coop(const uint8_t *__restrict__ src, uint64_t src_len,
                                                  const bhg_handle *__restrict__ hs, uint32_t n,
                                                  uint32_t *__restrict__ count) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[CW * PER_WAVE];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint8_t *st = lds + w * PER_WAVE;
    uint16_t *nx = reinterpret_cast<uint16_t *>(st + SB + 64);
    const uint64_t base = (uint64_t)src, end = base + src_len;
    const uint32_t W = gridDim.x * CW;
    uint32_t i = __builtin_amdgcn_readfirstlane(blockIdx.x * CW + w);
    auto geo = [&](uint32_t b, uint64_t &cp, uint32_t &clen) {
        const bhg_handle h = hs[b];
        const uint64_t rec = base + h.offset;
        const uint32_t k = *reinterpret_cast<const uint32_t *>(rec);
        cp = rec + 12 + k;
        clen = h.length - 12 - k;
    };
    auto ld = [&](uint64_t cp, uint32_t clen) -> u32x4 {
        const uint64_t a = cp + 16 * lane;
        if (16 * lane < clen && a + 16 <= end) return *reinterpret_cast<const u32x4u *>(a);
        return u32x4{0, 0, 0, 0};
    };
    uint64_t cp = 0;
    uint32_t clen = 0;
    u32x4 v = {0, 0, 0, 0};
    if (i < n) {
        geo(i, cp, clen);
        v = ld(cp, clen);
    }
    for (; i < n; i += W) {
        const uint64_t ccp = cp;
        const uint32_t cl = clen;
        *reinterpret_cast<u32x4_lds_u *>(st + 16 * lane) = v;
        if (cl > 1024) {  // rare: the rest synchronously
            const uint64_t a = ccp + 1024 + 16 * lane;
            u32x4 x = {0, 0, 0, 0};
            if (1024 + 16 * lane < cl && a + 16 <= end) x = *reinterpret_cast<const u32x4u *>(a);
            if (1024 + 16 * lane < SB) *reinterpret_cast<u32x4_lds_u *>(st + 1024 + 16 * lane) = x;
        }
        const uint32_t in = i + W;
        if (in < n) {  // next block's chunk in flight during this block
            geo(in, cp, clen);
            v = ld(cp, clen);
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        uint32_t cnt = 0;
        if (MODE == 0) {
            uint32_t hdr = 0;
            while (hdr < 5 && st[hdr] >= 0x80) hdr++;
            hdr++;
            for (uint32_t p = lane; p < cl; p += 64) {
                const uint64_t t8 = *reinterpret_cast<const u64u *>(st + p);
                const uint32_t tag = (uint32_t)t8 & 0xffu, ty = tag & 3u, x = tag >> 2;
                uint32_t nxt;
                if (ty == 0) {
                    if (x < 60) nxt = p + 2 + x;
                    else {
                        const uint32_t nb = x - 59;
                        const uint32_t b14 = (uint32_t)(t8 >> 8);
                        const uint32_t ln = (nb >= 4 ? b14 : (b14 & ((1u << (8 * nb)) - 1u))) + 1u;
                        nxt = p + 1 + nb + ln;
                    }
                } else {
                    nxt = p + (ty == 1 ? 2u : ty == 2 ? 3u : 5u);
                }
                nx[p] = (uint16_t)(nxt < 0xffffu ? nxt : 0xffffu);
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            for (uint32_t s = hdr; s < cl; s = nx[s]) cnt++;
        } else {
            cnt = st[lane] + st[cl - 1];
        }
        if (lane == 0) count[i] = cnt;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

}  // namespace

extern "C" int coop_run(const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n, uint32_t *count,
                        int mode, int wg_per_cu, void *stream) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
    const uint32_t grid = (uint32_t)cus * (uint32_t)wg_per_cu;
    if (mode == 0)
        hipLaunchKernelGGL(k_coop<0>, dim3(grid), dim3(64 * CW), 0, (hipStream_t)stream, src, src_len, h, n, count);
    else
        hipLaunchKernelGGL(k_coop<1>, dim3(grid), dim3(64 * CW), 0, (hipStream_t)stream, src, src_len, h, n, count);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
