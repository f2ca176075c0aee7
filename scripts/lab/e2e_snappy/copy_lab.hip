// Lab: do hipMemcpyAsync calls on page-locked host memory return before the copy ends, and do an
// H2D and a D2H stream overlap?  Host buffers from hipHostMalloc and from malloc +
// hipHostRegister(Mapped | Portable) (what bhg_host_register does); pieces of 16..256 MiB, issued
// alternately H2D / D2H on two streams (the snappy host pipeline's pattern).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
static double now() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char **argv) {
    // argv[1]: streams created (and used once) before the two copy streams, as a process that
    // already holds torch's and the library's streams would have
    const int extra = argc > 1 ? atoi(argv[1]) : 0;
    hipStream_t xs[64];
    for (int i = 0; i < extra && i < 64; i++) {
        CK(hipStreamCreateWithFlags(&xs[i], hipStreamNonBlocking));
        CK(hipMemsetAsync(nullptr, 0, 0, xs[i]));
    }
    printf("extra streams: %d\n", extra);
    const size_t H = 640ull << 20, D = 1088ull << 20;
    for (int reg = 0; reg < 2; reg++) {
        void *hs, *hd;
        if (reg) {
            hs = aligned_alloc(4096, H); hd = aligned_alloc(4096, D);
            CK(hipHostRegister(hs, H, hipHostRegisterMapped | hipHostRegisterPortable));
            CK(hipHostRegister(hd, D, hipHostRegisterMapped | hipHostRegisterPortable));
        } else {
            CK(hipHostMalloc(&hs, H, hipHostMallocDefault)); CK(hipHostMalloc(&hd, D, hipHostMallocDefault));
        }
        void *ds, *dd;
        CK(hipMalloc(&ds, H)); CK(hipMalloc(&dd, D));
        hipStream_t s1, s2;
        CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking)); CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
        for (size_t piece : {64ull << 20, 256ull << 20}) {
            for (int mode = 0; mode < 3; mode++) {  // 0 H2D only, 1 D2H only, 2 both alternating
                double best = 1e30, issue = 0;
                for (int rep = 0; rep < 4; rep++) {
                    CK(hipDeviceSynchronize());
                    const double t0 = now();
                    size_t oh = 0, od = 0;
                    while ((mode != 1 && oh < H) || (mode != 0 && od < D)) {
                        if (mode != 1 && oh < H) {
                            const size_t b = H - oh < piece ? H - oh : piece;
                            CK(hipMemcpyAsync((char *)ds + oh, (char *)hs + oh, b, hipMemcpyHostToDevice, s1));
                            oh += b;
                        }
                        if (mode != 0 && od < D) {
                            const size_t b = D - od < piece ? D - od : piece;
                            CK(hipMemcpyAsync((char *)hd + od, (char *)dd + od, b, hipMemcpyDeviceToHost, s2));
                            od += b;
                        }
                    }
                    const double t1 = now();
                    CK(hipStreamSynchronize(s1)); CK(hipStreamSynchronize(s2));
                    const double t2 = now();
                    if (rep && t2 - t0 < best) { best = t2 - t0; issue = t1 - t0; }
                }
                printf("%s piece %4zu MiB %-9s total %7.2f ms  issue %7.2f ms\n", reg ? "registered" : "hostmalloc",
                       piece >> 20, mode == 0 ? "H2D" : mode == 1 ? "D2H" : "both", best, issue);
                fflush(stdout);
            }
        }
        CK(hipStreamDestroy(s1)); CK(hipStreamDestroy(s2));
        CK(hipFree(ds)); CK(hipFree(dd));
        if (reg) { CK(hipHostUnregister(hs)); CK(hipHostUnregister(hd)); free(hs); free(hd); }
        else { CK(hipHostFree(hs)); CK(hipHostFree(hd)); }
    }
    return 0;
}
