// LDS access cost by alignment and width on gfx950 (lab probe).
// Each active lane runs ITERS dependent read -> write steps (the walk's shape: an op reads 16 B
// and writes them elsewhere in its own slot; the next read waits for nothing but the previous
// read's data).  Reported: ns per step per wave at a given resident-wave count.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_u __attribute__((aligned(1), may_alias));
typedef uint64_t u64_u __attribute__((aligned(1), may_alias));
typedef uint32_t u32_u __attribute__((aligned(1), may_alias));

constexpr int SLOT = 1088;
constexpr int ITERS = 4096;

// W: bytes per access (16, 8, 4); RA / WA: read / write address alignment offset (bytes) within a
// 16-B line; NL: active lanes per wave; SPREAD: consecutive ops move 16 B (like a copy) or jump
template <int W, int RA, int WA, int NL>
__global__ __launch_bounds__(64) void k_probe(uint32_t *out, uint32_t seed) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[18 * SLOT + 64];
    const uint32_t lane = threadIdx.x;
    for (uint32_t i = lane; i < (18 * SLOT + 64) / 4; i += 64) reinterpret_cast<uint32_t *>(lds)[i] = i * 2654435761u ^ seed;
    __syncthreads();
    uint32_t acc = 0;
    if (lane < NL) {
        const uint32_t sb = (lane % 18) * SLOT;
        uint32_t r = 512 + RA, w = 16 + WA;
        for (int it = 0; it < ITERS; it++) {
            if (W == 16) {
                u32x4 v = *reinterpret_cast<const u32x4_u *>(lds + sb + r);
                v.x ^= acc;
                *reinterpret_cast<u32x4_u *>(lds + sb + w) = v;
                acc += v.y;
            } else if (W == 8) {
                uint64_t v = *reinterpret_cast<const u64_u *>(lds + sb + r);
                v ^= acc;
                *reinterpret_cast<u64_u *>(lds + sb + w) = v;
                acc += (uint32_t)(v >> 32);
            } else {
                uint32_t v = *reinterpret_cast<const u32_u *>(lds + sb + r);
                v ^= acc;
                *reinterpret_cast<u32_u *>(lds + sb + w) = v;
                acc += v;
            }
            r = 512 + RA + ((it * 48) & 0x1f0);   // stays 16-B phase RA
            w = 16 + WA + ((it * 80) & 0x1f0);
        }
    }
    out[blockIdx.x * 64 + lane] = acc;
}

template <int W, int RA, int WA, int NL>
static void run(const char *name, int waves_per_cu, int ncu) {
    uint32_t *d;
    const int grid = waves_per_cu * ncu;
    hipMalloc(&d, (size_t)grid * 64 * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int k = 0; k < 3; k++) hipLaunchKernelGGL((k_probe<W, RA, WA, NL>), dim3(grid), dim3(64), 0, 0, d, k);
    hipEventRecord(a);
    const int reps = 10;
    for (int k = 0; k < reps; k++) hipLaunchKernelGGL((k_probe<W, RA, WA, NL>), dim3(grid), dim3(64), 0, 0, d, k);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    // per CU: waves_per_cu waves x ITERS steps; ns per step per wave, and per CU-step
    printf("%-28s W=%2d RA=%2d WA=%2d lanes=%2d waves/CU=%2d  %8.4f ms  %7.2f ns/step/wave  %6.2f ns/CU-step\n", name, W,
           RA, WA, NL, waves_per_cu, ms, ms * 1e6 / ITERS, ms * 1e6 / ITERS / waves_per_cu);
    hipFree(d);
}

int main(int argc, char **argv) {
    int ncu = 256;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) == hipSuccess) ncu = p.multiProcessorCount;
    const int wv = argc > 1 ? atoi(argv[1]) : 8;
    printf("CUs %d\n", ncu);
    for (int w : {2, wv}) {
        run<16, 0, 0, 18>("b128 aligned", w, ncu);
        run<16, 4, 4, 18>("b128 dword-aligned", w, ncu);
        run<16, 8, 8, 18>("b128 8-aligned", w, ncu);
        run<16, 1, 0, 18>("b128 read+1 write aligned", w, ncu);
        run<16, 0, 1, 18>("b128 read aligned write+1", w, ncu);
        run<16, 1, 3, 18>("b128 read+1 write+3", w, ncu);
        run<16, 5, 11, 18>("b128 read+5 write+11", w, ncu);
        run<8, 0, 0, 18>("b64 aligned", w, ncu);
        run<8, 1, 3, 18>("b64 +1/+3", w, ncu);
        run<4, 0, 0, 18>("b32 aligned", w, ncu);
        run<4, 1, 3, 18>("b32 +1/+3", w, ncu);
        run<16, 0, 0, 6>("b128 aligned 6 lanes", w, ncu);
        run<16, 1, 3, 6>("b128 +1/+3 6 lanes", w, ncu);
        run<16, 0, 0, 64>("b128 aligned 64 lanes", w, ncu);
        run<16, 1, 3, 64>("b128 +1/+3 64 lanes", w, ncu);
        run<16, 4, 12, 64>("b128 +4/+12 64 lanes", w, ncu);
    }
    return 0;
}
