// Lab: does a D2H hipMemcpyAsync into page-locked host memory block the calling thread when
// the host or device address is not aligned?  (The pipelined snappy host path copies each
// chunk's values to out_vals + base, base = any byte count.)  112 MiB copies, host buffer
// registered (bhg_host_register flags) or hipHostMalloc'd; host / device offsets 0, 5, 256 + 5,
// 4096 + 5.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
static double now() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main() {
    const size_t B = 112ull << 20, CAP = B + (1 << 20);
    hipStream_t xs[4];
    for (int i = 0; i < 4; i++) { CK(hipStreamCreateWithFlags(&xs[i], hipStreamNonBlocking)); CK(hipMemsetAsync(nullptr, 0, 0, xs[i])); }
    for (int reg = 0; reg < 2; reg++) {
        char *h;
        if (reg) { h = (char *)malloc(CAP + 16) + 16; CK(hipHostRegister(h, CAP, hipHostRegisterMapped | hipHostRegisterPortable)); }
        else CK(hipHostMalloc((void **)&h, CAP, hipHostMallocDefault));
        char *d;
        CK(hipMalloc((void **)&d, CAP));
        CK(hipMemset(d, 1, CAP));
        hipStream_t s;
        CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        const size_t offs[] = {0, 5, 261, 4101};
        for (size_t ho : offs)
            for (size_t dof : offs) {
                double best = 1e30, issue = 0;
                for (int rep = 0; rep < 4; rep++) {
                    CK(hipDeviceSynchronize());
                    const double t0 = now();
                    CK(hipMemcpyAsync(h + ho, d + dof, B, hipMemcpyDeviceToHost, s));
                    const double t1 = now();
                    CK(hipStreamSynchronize(s));
                    const double t2 = now();
                    if (rep && t2 - t0 < best) { best = t2 - t0; issue = t1 - t0; }
                }
                printf("%s host+%4zu dev+%4zu  total %6.2f ms  issue %6.2f ms\n", reg ? "registered(+16)" : "hostmalloc     ",
                       ho, dof, best, issue);
                fflush(stdout);
            }
        CK(hipStreamDestroy(s));
        CK(hipFree(d));
        if (reg) { CK(hipHostUnregister(h)); free(h - 16); } else CK(hipHostFree(h));
    }
    return 0;
}
