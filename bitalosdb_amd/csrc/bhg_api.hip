// bhg_api.hip -- implementation of the C-ABI in include/bithashgpu.h.
//
// Host orchestration only: argument checks, per-call scratch from the
// context's stream-ordered pool, launch sequencing on the caller's stream.  All byte work runs in the kernels
// (bhg_decode.hip, bhg_encode.hip, bhg_scan.hip); there is no CPU fallback:
// without a usable HIP device bhg_create() fails and every entry point
// returns an error.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <condition_variable>
#include <mutex>
#include <thread>

#include <vector>

#include "bhg_crc_tables.h"
#include "bhg_internal.h"

// Host threads that copy page-locked staging buffers into pageable caller buffers (the pipelined
// snappy host path with a pageable out_vals): one job at a time, every thread taking an equal
// share of each segment.  submit() returns at once; wait() blocks until the job is done.
struct HostCopyPool {
    struct Seg {
        uint8_t *dst;
        const uint8_t *src;
        size_t n;
    };
    explicit HostCopyPool(int nthreads) : nt(nthreads) {
        segs.reserve(4);  // submit() then never allocates
        try {
            for (int t = 0; t < nthreads; t++) th.emplace_back([this, t] { worker(t); });
        } catch (...) {  // the threads already started are stopped before the exception leaves
            shutdown();
            throw;
        }
    }
    ~HostCopyPool() { shutdown(); }
    void submit(std::initializer_list<Seg> s) {
        wait();
        {
            std::lock_guard<std::mutex> lk(m);
            segs.assign(s);
            pending = nt;
            gen++;
        }
        cv.notify_all();
    }
    void wait() {
        std::unique_lock<std::mutex> lk(m);
        done.wait(lk, [&] { return pending == 0; });
    }

  private:
    void shutdown() {
        {
            std::lock_guard<std::mutex> lk(m);
            stop = true;
        }
        cv.notify_all();
        for (auto &t : th) t.join();
        th.clear();
    }
    void worker(int id) {
        uint64_t seen = 0;
        for (;;) {
            std::vector<Seg> job;
            {
                std::unique_lock<std::mutex> lk(m);
                cv.wait(lk, [&] { return stop || gen != seen; });
                if (stop) return;
                seen = gen;
                job = segs;
            }
            for (const Seg &g : job) {
                const size_t per = ((g.n + nt - 1) / nt + 63) & ~(size_t)63;
                const size_t a = (size_t)id * per, b = a + per < g.n ? a + per : g.n;
                if (a < b) memcpy(g.dst + a, g.src + a, b - a);
            }
            {
                std::lock_guard<std::mutex> lk(m);
                if (--pending == 0) done.notify_all();
            }
        }
    }
    const int nt;
    std::vector<std::thread> th;
    std::mutex m;
    std::condition_variable cv, done;
    std::vector<Seg> segs;
    uint64_t gen = 0;
    int pending = 0;
    bool stop = false;
};

struct bhg_ctx {
    int device;
    hipStream_t stream;
    int num_cus;
    char err[512];
    hipMemPool_t pool = nullptr;  // per-call scratch (stream ordered, never shared between calls)
    std::mutex mu;                // guards the host-path staging buffers and pipeline streams
    // host (end-to-end) path device buffers
    void *h_src = nullptr; size_t h_src_cap = 0;
    void *h_aux = nullptr; size_t h_aux_cap = 0;
    void *h_vals = nullptr; size_t h_vals_cap = 0;
    void *h_big = nullptr; size_t h_big_cap = 0;  // the snappy big-block path's scratch (host paths)
    uint32_t *ztab = nullptr;  // tile-kernel shift tables (bhg_crc_tables.h build_tile_ztab)
    uint32_t *stab = nullptr;  // stream-kernel shift tables (bhg_decode_stream.h build_stream_tab)
    uint32_t *xtab = nullptr;  // CrcR8-kernel shift tables (bhg_crc_tables.h build_xtab)
    // pipelined host path: kPipe slots, each with its own stream and device ring buffers
    static constexpr int kPipe = 3;
    hipStream_t pstream[kPipe] = {nullptr, nullptr, nullptr};
    void *pbuf[kPipe] = {nullptr, nullptr, nullptr};
    size_t pbuf_cap[kPipe] = {0, 0, 0};
    // ... the snappy pipeline's per-slot decoded values, chunk totals (page-locked) and their events
    void *pvals[kPipe] = {nullptr, nullptr, nullptr};
    size_t pvals_cap[kPipe] = {0, 0, 0};
    void *pbig[kPipe] = {nullptr, nullptr, nullptr};  // ... per slot: the snappy big-block path's scratch
    size_t pbig_cap[kPipe] = {0, 0, 0};
    uint64_t *ptot = nullptr;
    hipEvent_t pev[kPipe] = {nullptr, nullptr, nullptr};   // chunk total in ptot
    hipEvent_t pevb[kPipe] = {nullptr, nullptr, nullptr};  // chunk values decoded
    hipEvent_t pevd[kPipe] = {nullptr, nullptr, nullptr};  // chunk copied back (slot free)
    // ... with a pageable out_vals: page-locked staging per slot (values, offsets, descriptors,
    // written by copy kernels) and the host threads that copy it on into the caller's buffers
    uint8_t *pstage[kPipe] = {nullptr, nullptr, nullptr};
    uint8_t *pstage_dev[kPipe] = {nullptr, nullptr, nullptr};  // its device address
    size_t pstage_cap[kPipe] = {0, 0, 0};
    HostCopyPool *hpool = nullptr;
};

namespace {

void set_err(bhg_ctx *c, const char *fmt, ...) {
    if (!c) return;
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(c->err, sizeof c->err, fmt, ap);
    va_end(ap);
}

int hip_fail(bhg_ctx *c, hipError_t e, const char *what) {
    set_err(c, "%s: %s", what, hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? BHG_ENOMEM : BHG_EHIP;
}

#define HIP_TRY(ctx, expr)                                     \
    do {                                                       \
        hipError_t _e = (expr);                                \
        if (_e != hipSuccess) return hip_fail(ctx, _e, #expr); \
    } while (0)

bhg::Launch launch_of(bhg_ctx *c, void *stream) {
    bhg::Launch L;
    L.stream = stream ? reinterpret_cast<hipStream_t>(stream) : c->stream;
    L.num_cus = c->num_cus;
    L.ztab = c->ztab;
    L.stab = c->stab;
    L.xtab = c->xtab;
    return L;
}

// Per-call device scratch: carved from one stream-ordered allocation of the
// context's pool, released on the call's stream when the object goes out of
// scope -- after every kernel the call enqueued, whatever path returns.
struct Scratch {
    hipStream_t s = nullptr;
    uint8_t *base = nullptr;
    size_t used = 0, cap = 0;
    ~Scratch() {
        if (base) (void)hipFreeAsync(base, s);
    }
    static size_t al(size_t x) { return (x + 255) & ~(size_t)255; }
    uint8_t *take(size_t bytes) {
        uint8_t *p = base + used;
        used += al(bytes);
        return p;
    }
};

int scratch_alloc(bhg_ctx *c, hipStream_t s, size_t bytes, Scratch &sc) {
    sc.s = s;
    sc.cap = bytes + 256;
    void *p = nullptr;
    hipError_t e = hipMallocFromPoolAsync(&p, sc.cap, c->pool, s);
    if (e != hipSuccess) return hip_fail(c, e, "hipMallocFromPoolAsync(scratch)");
    sc.base = reinterpret_cast<uint8_t *>(p);
    return BHG_OK;
}

// grow a host-path staging buffer (synchronous; the host paths are synchronous)
int ensure_buf(bhg_ctx *c, void **buf, size_t *cap, size_t need) {
    if (need <= *cap) return BHG_OK;
    if (*buf) {
        (void)hipStreamSynchronize(c->stream);
        for (int k = 0; k < bhg_ctx::kPipe; k++)
            if (c->pstream[k]) (void)hipStreamSynchronize(c->pstream[k]);
        (void)hipFree(*buf);
        *buf = nullptr;
        *cap = 0;
    }
    size_t sz = need + need / 4 + 4096;
    hipError_t e = hipMalloc(buf, sz);
    if (e != hipSuccess) return hip_fail(c, e, "hipMalloc(scratch)");
    *cap = sz;
    return BHG_OK;
}

int set_device(bhg_ctx *c) {
    hipError_t e = hipSetDevice(c->device);
    if (e != hipSuccess) return hip_fail(c, e, "hipSetDevice");
    return BHG_OK;
}

}  // namespace

extern "C" {

int bhg_abi_version(void) { return BHG_ABI_VERSION; }

int bhg_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

bhg_ctx *bhg_create(int device, int flags) {
    (void)flags;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return nullptr;
    if (hipSetDevice(device) != hipSuccess) return nullptr;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return nullptr;
    bhg_ctx *c = new bhg_ctx();
    c->device = device;
    c->num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    c->err[0] = 0;
    // blocking stream: orders against the legacy NULL stream, so callers that
    // stage buffers on the default stream need no extra event
    if (hipStreamCreateWithFlags(&c->stream, hipStreamDefault) != hipSuccess) {
        delete c;
        return nullptr;
    }
    bool ok = true;
    {
        hipMemPoolProps pp;
        memset(&pp, 0, sizeof pp);
        pp.allocType = hipMemAllocationTypePinned;
        pp.location.type = hipMemLocationTypeDevice;
        pp.location.id = device;
        ok = hipMemPoolCreate(&c->pool, &pp) == hipSuccess;
        // keep freed scratch in the pool: steady-state calls allocate nothing from the driver
        uint64_t keep = UINT64_MAX;
        ok = ok && hipMemPoolSetAttribute(c->pool, hipMemPoolAttrReleaseThreshold, &keep) == hipSuccess;
    }
    if (ok) {
        std::vector<uint32_t> z(bhg::kZTabWords);
        bhg::build_tile_ztab(z.data());
        ok = hipMalloc(reinterpret_cast<void **>(&c->ztab), z.size() * 4) == hipSuccess &&
             hipMemcpy(c->ztab, z.data(), z.size() * 4, hipMemcpyHostToDevice) == hipSuccess;
    }
    if (ok) {
        std::vector<uint32_t> z(bhg::stream_tab_words());
        bhg::build_stream_tab_default(z.data());
        ok = hipMalloc(reinterpret_cast<void **>(&c->stab), z.size() * 4) == hipSuccess &&
             hipMemcpy(c->stab, z.data(), z.size() * 4, hipMemcpyHostToDevice) == hipSuccess;
    }
    if (ok) {
        std::vector<uint32_t> z(bhg::kXTabWords);
        bhg::build_xtab(z.data());
        ok = hipMalloc(reinterpret_cast<void **>(&c->xtab), z.size() * 4) == hipSuccess &&
             hipMemcpy(c->xtab, z.data(), z.size() * 4, hipMemcpyHostToDevice) == hipSuccess;
    }
    if (ok) {  // the LDS store ordering the snappy encoder relies on (bhg_snappy_enc.hip k_lds_order_probe)
        uint32_t *bad = nullptr, h = 1;
        ok = hipMalloc(reinterpret_cast<void **>(&bad), 4) == hipSuccess &&
             bhg::launch_lds_order_probe(c->stream, bad) == hipSuccess &&
             hipMemcpyAsync(&h, bad, 4, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
             hipStreamSynchronize(c->stream) == hipSuccess && h == 0;
        if (bad) (void)hipFree(bad);
        if (!ok) fprintf(stderr, "bithashgpu: device %d failed the LDS store-ordering probe\n", device);
    }
    if (!ok) {
        bhg_destroy(c);
        return nullptr;
    }
    return c;
}

void bhg_destroy(bhg_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (int k = 0; k < bhg_ctx::kPipe; k++) {
        if (c->pstream[k]) { (void)hipStreamSynchronize(c->pstream[k]); (void)hipStreamDestroy(c->pstream[k]); }
        if (c->pbuf[k]) (void)hipFree(c->pbuf[k]);
        if (c->pvals[k]) (void)hipFree(c->pvals[k]);
        if (c->pbig[k]) (void)hipFree(c->pbig[k]);
        if (c->pev[k]) (void)hipEventDestroy(c->pev[k]);
        if (c->pevb[k]) (void)hipEventDestroy(c->pevb[k]);
        if (c->pevd[k]) (void)hipEventDestroy(c->pevd[k]);
    }
    if (c->ptot) (void)hipHostFree(c->ptot);
    delete c->hpool;  // joins its threads (idle: every host call waits for its copies)
    for (int k = 0; k < bhg_ctx::kPipe; k++)
        if (c->pstage[k]) (void)hipHostFree(c->pstage[k]);
    if (c->h_src) (void)hipFree(c->h_src);
    if (c->h_aux) (void)hipFree(c->h_aux);
    if (c->h_vals) (void)hipFree(c->h_vals);
    if (c->h_big) (void)hipFree(c->h_big);
    if (c->ztab) (void)hipFree(c->ztab);
    if (c->stab) (void)hipFree(c->stab);
    if (c->xtab) (void)hipFree(c->xtab);
    if (c->pool) {
        (void)hipDeviceSynchronize();  // frees enqueued on caller streams have completed
        (void)hipMemPoolDestroy(c->pool);
    }
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char *bhg_last_error(const bhg_ctx *c) { return c ? c->err : "null context"; }

void *bhg_stream(bhg_ctx *c) { return c ? reinterpret_cast<void *>(c->stream) : nullptr; }

int bhg_stream_sync(bhg_ctx *c, void *stream) {
    if (!c) return BHG_EINVAL;
    if (int r = set_device(c)) return r;
    HIP_TRY(c, hipStreamSynchronize(stream ? reinterpret_cast<hipStream_t>(stream) : c->stream));
    return BHG_OK;
}

void *bhg_malloc_device(bhg_ctx *c, uint64_t bytes) {
    if (!c || set_device(c)) return nullptr;
    void *p = nullptr;
    hipError_t e = hipMalloc(&p, bytes ? bytes : 1);
    if (e != hipSuccess) { hip_fail(c, e, "hipMalloc"); return nullptr; }
    return p;
}

int bhg_free_device(bhg_ctx *c, void *p) {
    if (!c) return BHG_EINVAL;
    if (int r = set_device(c)) return r;
    HIP_TRY(c, hipFree(p));
    return BHG_OK;
}

void *bhg_malloc_host(bhg_ctx *c, uint64_t bytes) {
    if (!c || set_device(c)) return nullptr;
    void *p = nullptr;
    hipError_t e = hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault);
    if (e != hipSuccess) { hip_fail(c, e, "hipHostMalloc"); return nullptr; }
    return p;
}

int bhg_free_host(bhg_ctx *c, void *p) {
    if (!c) return BHG_EINVAL;
    HIP_TRY(c, hipHostFree(p));
    return BHG_OK;
}

int bhg_memcpy_h2d(bhg_ctx *c, void *dst, const void *src, uint64_t bytes, void *stream) {
    if (!c || (!dst && bytes) || (!src && bytes)) return BHG_EINVAL;
    if (int r = set_device(c)) return r;
    bhg::Launch L = launch_of(c, stream);
    HIP_TRY(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, L.stream));
    return BHG_OK;
}

int bhg_memcpy_d2h(bhg_ctx *c, void *dst, const void *src, uint64_t bytes, void *stream) {
    if (!c || (!dst && bytes) || (!src && bytes)) return BHG_EINVAL;
    if (int r = set_device(c)) return r;
    bhg::Launch L = launch_of(c, stream);
    HIP_TRY(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, L.stream));
    return BHG_OK;
}

int bhg_memset_device(bhg_ctx *c, void *dst, int value, uint64_t bytes, void *stream) {
    if (!c || (!dst && bytes)) return BHG_EINVAL;
    if (int r = set_device(c)) return r;
    bhg::Launch L = launch_of(c, stream);
    HIP_TRY(c, hipMemsetAsync(dst, value, bytes, L.stream));
    return BHG_OK;
}

int bhg_decode_batch(bhg_ctx *c, const uint8_t *src, uint64_t src_len, const bhg_handle *handles, uint32_t n,
                     int codec, const uint32_t *expected_crc, bhg_desc *out_desc, uint8_t *out_vals,
                     uint64_t out_vals_cap, uint64_t *out_val_off, void *stream) {
    if (!c) return BHG_EINVAL;
    if (codec != BHG_CODEC_NONE && codec != BHG_CODEC_SNAPPY) { set_err(c, "bad codec %d", codec); return BHG_EINVAL; }
    if (n == 0) {
        if (codec == BHG_CODEC_SNAPPY && out_val_off) return bhg_memset_device(c, out_val_off, 0, 8, stream);
        return BHG_OK;
    }
    if (!handles || !out_desc || (!src && src_len)) { set_err(c, "null buffer"); return BHG_EINVAL; }
    if (codec == BHG_CODEC_SNAPPY && !out_val_off) { set_err(c, "snappy decode needs out_val_off[n+1]"); return BHG_EINVAL; }
    if (int r = set_device(c)) return r;
    bhg::Launch L = launch_of(c, stream);
    if (codec != BHG_CODEC_SNAPPY) {
        if (bhg::long_batch(src_len, n)) {  // long records: their CRCs by the long-record pass (bhg_longcrc.hip)
            Scratch sc;
            if (int r = scratch_alloc(c, L.stream, bhg::long_crc_scratch_bytes(n, src_len), sc)) return r;
            HIP_TRY(c, bhg::launch_decode_tile(L, src, src_len, handles, n, expected_crc, out_desc, sc.base));
            return BHG_OK;
        }
        HIP_TRY(c, bhg::launch_decode(L, src, src_len, handles, n, codec, expected_crc, out_desc, out_val_off));
        return BHG_OK;
    }
    // snappy: the header pass also sorts the blocks into the decode lists (when values are wanted)
    Scratch sc;
    const size_t scan_b = (bhg::scan_scratch_bytes(n) + 255) & ~(size_t)255;
    const size_t list_b = out_vals ? (bhg::snappy_list_bytes(n) + 255) & ~(size_t)255 : 0;
    const size_t big_b = out_vals ? (bhg::snappy_big_bytes(n, out_vals_cap) + 255) & ~(size_t)255 : 0;
    // long records: their CRCs by the long-record pass after the header pass (bhg_longcrc.hip)
    const size_t long_b = bhg::long_batch(src_len, n) ? bhg::long_crc_scratch_bytes(n, src_len) : 0;
    if (int r = scratch_alloc(c, L.stream, scan_b + list_b + big_b + long_b, sc)) return r;
    uint32_t *lists = out_vals ? reinterpret_cast<uint32_t *>(sc.base + scan_b) : nullptr;
    HIP_TRY(c, bhg::launch_decode(L, src, src_len, handles, n, codec, expected_crc, out_desc, out_val_off, lists,
                                  long_b ? sc.base + scan_b + list_b + big_b : nullptr));
    HIP_TRY(c, bhg::launch_exclusive_scan_u64(L, out_val_off, out_val_off, n, sc.base));
    if (out_vals)
        HIP_TRY(c, bhg::launch_snappy(L, src, src_len, handles, n, out_desc, out_vals, out_vals_cap, out_val_off, lists,
                                      sc.base + scan_b + list_b));
    return BHG_OK;
}

namespace {

// Pipelined end-to-end NoCompressor decode for handles sorted by offset (a
// table scan, a compaction pass): the batch is cut into chunks of at most
// kChunkBytes of src; chunk k goes to slot k % kPipe (own stream + device
// buffer): H2D of its src byte range and handles, the decode kernel on the
// rebased range, D2H of its descriptors.  Copies of one slot overlap the
// kernels and copies of the others; slot reuse is ordered by its stream.
constexpr uint64_t kChunkBytesDefault = 64ull << 20;

// The next chunk [a, return) of the pipelined host paths: grown while the in-bounds records' byte
// span [*lo, *hi) of src stays within chunk_bytes (a record larger than that makes a chunk of its
// own) and at most max_cn handles.  A handle whose offset is below its predecessor's (*prev_off,
// carried across calls) ends the chunk before it and sets *unsorted.
uint32_t next_chunk(const bhg_handle *handles, uint32_t a, uint32_t n, uint64_t src_len, uint64_t chunk_bytes,
                    uint32_t max_cn, uint64_t *prev_off, uint64_t *lo_out, uint64_t *hi_out, bool *unsorted) {
    uint64_t lo = UINT64_MAX, hi = 0;
    uint32_t b = a;
    while (b < n && b - a < max_cn) {
        const bhg_handle &h = handles[b];
        if (h.offset < *prev_off) {
            *unsorted = true;
            break;
        }
        *prev_off = h.offset;
        const bool inb = h.length != 0 && h.offset <= src_len && (uint64_t)h.length <= src_len - h.offset;
        if (inb) {
            const uint64_t nlo = h.offset < lo ? h.offset : lo;
            const uint64_t nhi = h.offset + h.length > hi ? h.offset + h.length : hi;
            if (b > a && nhi - nlo > chunk_bytes) break;
            if (nhi - nlo > chunk_bytes) { lo = nlo; hi = nhi; b++; break; }  // one oversized record
            lo = nlo;
            hi = nhi;
        }
        b++;
    }
    if (lo == UINT64_MAX) lo = hi = 0;
    *lo_out = lo;
    *hi_out = hi;
    return b;
}

uint64_t host_chunk_bytes() {
    uint64_t v = kChunkBytesDefault;
    if (const char *e = getenv("BHG_HOST_CHUNK_BYTES")) v = strtoull(e, nullptr, 10);  // tests
    return v < 4096 ? 4096 : v;
}

// Handles out of offset order end the pipeline where they start: the chunk walk below checks the order
// as it goes (no separate host pass over the batch), the chunks already issued complete, and the
// function returns -100 with *done = the handles decoded; the caller decodes the rest another way.
int decode_host_pipelined(bhg_ctx *c, const uint8_t *src, uint64_t src_len, const bhg_handle *handles, uint32_t n,
                          const uint32_t *expected_crc, bhg_desc *out_desc, uint32_t *done) {
    *done = 0;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const uint64_t kChunkBytes = host_chunk_bytes();
    const uint32_t max_chunk_n = 1u << 17;
    // kHead bytes of headroom before each chunk's src bytes: the decode kernels may load (and mask) a
    // window that starts up to 131 B before a record, which must be mapped memory
    constexpr size_t kHead = 256;
    const size_t need = kHead + al(kChunkBytes + 64) + al((size_t)max_chunk_n * sizeof(bhg_handle)) +
                        al((size_t)max_chunk_n * sizeof(bhg_desc)) + al((size_t)max_chunk_n * 4);
    for (int k = 0; k < bhg_ctx::kPipe; k++) {
        if (!c->pstream[k]) HIP_TRY(c, hipStreamCreateWithFlags(&c->pstream[k], hipStreamNonBlocking));
        if (int r = ensure_buf(c, &c->pbuf[k], &c->pbuf_cap[k], need)) return r;
    }
    bhg::Launch L = launch_of(c, nullptr);
    uint32_t a = 0;
    int slot = 0;
    uint64_t prev_off = 0;
    bool unsorted = false;
    while (a < n) {
        uint64_t lo, hi;
        const uint32_t b = next_chunk(handles, a, n, src_len, kChunkBytes, max_chunk_n, &prev_off, &lo, &hi, &unsorted);
        const uint32_t cn = b - a;
        const uint64_t span = hi - lo;
        if (span > kChunkBytes || cn == 0) {
            // a single record larger than the ring slot, or handles out of order from a on: the caller
            // decodes [a, n) unpipelined
            for (int k = 0; k < bhg_ctx::kPipe; k++) HIP_TRY(c, hipStreamSynchronize(c->pstream[k]));
            *done = a;
            return -100;
        }
        uint8_t *base = reinterpret_cast<uint8_t *>(c->pbuf[slot]) + kHead;
        bhg_handle *dh = reinterpret_cast<bhg_handle *>(base + al(kChunkBytes + 64));
        bhg_desc *dd = reinterpret_cast<bhg_desc *>(reinterpret_cast<uint8_t *>(dh) + al((size_t)max_chunk_n * sizeof(bhg_handle)));
        uint32_t *de = expected_crc ? reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(dd) +
                                                                   al((size_t)max_chunk_n * sizeof(bhg_desc)))
                                    : nullptr;
        hipStream_t s = c->pstream[slot];
        // the chunk's handles keep their src-relative offsets: the kernel sees src' = base - lo, src_len' = hi,
        // and never addresses more than kHead bytes below base (every in-bounds handle of the chunk has
        // offset >= lo; head windows reach back at most W + 3 bytes)
        if (span) HIP_TRY(c, hipMemcpyAsync(base, src + lo, span, hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(dh, handles + a, (size_t)cn * sizeof(bhg_handle), hipMemcpyHostToDevice, s));
        if (de) HIP_TRY(c, hipMemcpyAsync(de, expected_crc + a, (size_t)cn * 4, hipMemcpyHostToDevice, s));
        bhg::Launch Ls = L;
        Ls.stream = s;
        HIP_TRY(c, bhg::launch_decode(Ls, base - lo, hi, dh, cn, BHG_CODEC_NONE, de, dd, nullptr));
        HIP_TRY(c, hipMemcpyAsync(out_desc + a, dd, (size_t)cn * sizeof(bhg_desc), hipMemcpyDeviceToHost, s));
        a = b;
        slot = (slot + 1) % bhg_ctx::kPipe;
        if (unsorted) {
            for (int k = 0; k < bhg_ctx::kPipe; k++) HIP_TRY(c, hipStreamSynchronize(c->pstream[k]));
            *done = a;
            return -100;
        }
    }
    for (int k = 0; k < bhg_ctx::kPipe; k++) HIP_TRY(c, hipStreamSynchronize(c->pstream[k]));
    *done = n;
    return BHG_OK;
}

const void *mapped_device_ptr(const void *p);

// Pipelined end-to-end SnappyCompressor decode for handles sorted by offset, every in-bounds
// record within one chunk (else -100 before anything is issued: the caller decodes the whole
// batch at once).  Two streams: the context stream carries the H2D copies and the kernels, a
// second one the D2H copies, so chunk k + 1's H2D runs under chunk k's D2H (PCIe carries both
// directions at once).  Per chunk k, in slot k % kPipe:
//   A (context stream): H2D of its src byte range [lo, hi), handles and expected CRCs; the
//     handles rebased onto the staged range (the kernels see a source of hi - lo bytes: they
//     may load from its first bytes on behalf of any lane, so the source they are given must
//     be mapped from its start); the header/CRC pass; the chunk-local size scan; D2H of the
//     chunk total into page-locked ptot[slot] (event pev).
//   B (context stream, once the host has that total): the offsets rebased onto the batch and
//     the value decode into the slot's value buffer (event pevb).  The decode gets out_vals =
//     slot buffer - batch base and a cap of min(out_vals_cap, base + chunk total): the same
//     SNAPPY_TOO_LARGE verdicts as one batch-wide launch.
//   D (copy stream, after pevb): values, offsets and descriptors back to the host (event pevd,
//     which A of the chunk that next takes the slot waits for).  Values into a page-locked,
//     mapped out_vals go by a copy kernel (k_copy_out: the link rate; a D2H copy may get a DMA
//     engine that runs at half of it), the slot buffer then holding them at the host address's
//     offset mod 16; offsets and descriptors by D2H copies.  With a pageable out_vals, copy
//     kernels write values, offsets and descriptors into the slot's page-locked staging
//     buffer, and host threads (HostCopyPool) copy chunk k - 1's staging into the caller's
//     buffers while the host thread issues chunk k + 1 (a pageable D2H copy would hold the
//     host thread for its whole length).
// The host issues B(k), A(k + 1), D(k) in that order, so an H2D is always queued before the
// D2H it should overlap (a D2H call may return only when its copy is done).  Rebasing keeps
// every status: in-bounds records lie in [lo, hi); the others stay past the end (the offsets
// of those below lo wrap).
int decode_host_snappy_pipelined(bhg_ctx *c, const uint8_t *src, uint64_t src_len, const bhg_handle *handles,
                                 uint32_t n, const uint32_t *expected_crc, bhg_desc *out_desc, uint8_t *out_vals,
                                 uint64_t out_vals_cap, uint64_t *out_val_off) {
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const uint64_t kChunkBytes = host_chunk_bytes();
    {
        uint64_t prev = 0;
        for (uint32_t i = 0; i < n; i++) {
            const bhg_handle &h = handles[i];
            if (h.offset < prev) return -100;
            prev = h.offset;
            const bool inb = h.length != 0 && h.offset <= src_len && (uint64_t)h.length <= src_len - h.offset;
            if (inb && h.length > kChunkBytes) return -100;
        }
    }
    const uint32_t max_chunk_n = 1u << 17;
    const size_t b_src = al(kChunkBytes + 64), b_h = al((size_t)max_chunk_n * sizeof(bhg_handle));
    const size_t b_d = al((size_t)max_chunk_n * sizeof(bhg_desc)), b_e = al((size_t)max_chunk_n * 4);
    const size_t b_o = al(((size_t)max_chunk_n + 1) * 8), b_s = al(bhg::scan_scratch_bytes(max_chunk_n));
    const size_t b_l = al(bhg::snappy_list_bytes(max_chunk_n));
    const size_t need = b_src + b_h + b_d + b_e + b_o + b_s + b_l;
    if (!c->pstream[0]) HIP_TRY(c, hipStreamCreateWithFlags(&c->pstream[0], hipStreamNonBlocking));
    for (int k = 0; k < bhg_ctx::kPipe; k++) {
        if (!c->pev[k]) HIP_TRY(c, hipEventCreateWithFlags(&c->pev[k], hipEventDisableTiming));
        if (!c->pevb[k]) HIP_TRY(c, hipEventCreateWithFlags(&c->pevb[k], hipEventDisableTiming));
        if (!c->pevd[k]) HIP_TRY(c, hipEventCreateWithFlags(&c->pevd[k], hipEventDisableTiming));
        if (int r = ensure_buf(c, &c->pbuf[k], &c->pbuf_cap[k], need)) return r;
    }
    if (!c->ptot) HIP_TRY(c, hipHostMalloc(reinterpret_cast<void **>(&c->ptot), bhg_ctx::kPipe * sizeof(uint64_t),
                                           hipHostMallocDefault));
    struct Slot {
        uint8_t *src;
        bhg_handle *h;
        bhg_desc *d;
        uint32_t *e;
        uint64_t *off;
        void *scan;
        uint32_t *list;
    };
    auto slot_of = [&](int k) {
        uint8_t *p = reinterpret_cast<uint8_t *>(c->pbuf[k]);
        Slot S;
        S.src = p; p += b_src;
        S.h = reinterpret_cast<bhg_handle *>(p); p += b_h;
        S.d = reinterpret_cast<bhg_desc *>(p); p += b_d;
        S.e = expected_crc ? reinterpret_cast<uint32_t *>(p) : nullptr; p += b_e;
        S.off = reinterpret_cast<uint64_t *>(p); p += b_o;
        S.scan = p; p += b_s;
        S.list = reinterpret_cast<uint32_t *>(p);
        return S;
    };
    struct Chunk {
        uint32_t a, cn;
        int slot;
        uint64_t lo, hi, vb, fit;  // vb, fit, mis: set by stage B (batch value base, bytes copied back,
        uint32_t mis;              // the values' offset in the slot buffer)
    };
    bhg::Launch L = launch_of(c, nullptr);  // the context stream
    hipStream_t sc = c->stream, sd = c->pstream[0];
    bhg::Launch Ld = L;
    Ld.stream = sd;
    uint8_t *mvals = const_cast<uint8_t *>(static_cast<const uint8_t *>(mapped_device_ptr(out_vals)));
    const bool staged = mvals == nullptr;
    if (staged && !c->hpool) {
        const unsigned hc = std::thread::hardware_concurrency();
        try {
            // 4 / 8 / 12 / 16 threads measured equal (17.5-17.8 GiB/s on disk, C3 batch pageable:
            // profiles/r4/e2e_snappy/hpool_threads.txt)
            c->hpool = new HostCopyPool(hc < 2 ? 2 : hc > 8 ? 8 : (int)hc);
        } catch (...) {  // no exception crosses the C ABI
            set_err(c, "host copy threads could not be started");
            return BHG_ENOMEM;
        }
    }
    // No return, error paths included, leaves a copy kernel, a D2H copy or a host copy running into
    // the caller's buffers: both streams are drained (best effort), then the host copy threads.
    struct PoolWait {
        HostCopyPool *p;
        hipStream_t s1, s2;
        ~PoolWait() {
            (void)hipStreamSynchronize(s1);
            (void)hipStreamSynchronize(s2);
            if (p) p->wait();
        }
    } pool_wait{staged ? c->hpool : nullptr, sc, sd};
    bool dpend[bhg_ctx::kPipe] = {false, false, false};  // the slot's last D2H has an event to wait for
    uint64_t vbase = 0;                                   // the batch offset of the next chunk's first value
    uint64_t prev_off = 0;
    bool unsorted = false;  // cannot happen: checked above
    auto stage_a = [&](Chunk &ch) -> int {
        const Slot S = slot_of(ch.slot);
        if (dpend[ch.slot]) HIP_TRY(c, hipStreamWaitEvent(sc, c->pevd[ch.slot], 0));
        if (ch.hi > ch.lo) HIP_TRY(c, hipMemcpyAsync(S.src, src + ch.lo, ch.hi - ch.lo, hipMemcpyHostToDevice, sc));
        HIP_TRY(c, hipMemcpyAsync(S.h, handles + ch.a, (size_t)ch.cn * sizeof(bhg_handle), hipMemcpyHostToDevice, sc));
        if (S.e) HIP_TRY(c, hipMemcpyAsync(S.e, expected_crc + ch.a, (size_t)ch.cn * 4, hipMemcpyHostToDevice, sc));
        HIP_TRY(c, bhg::launch_add_u64(L, reinterpret_cast<uint64_t *>(S.h), ch.cn, 0 - ch.lo, 2));
        HIP_TRY(c, bhg::launch_decode(L, S.src, ch.hi - ch.lo, S.h, ch.cn, BHG_CODEC_SNAPPY, S.e, S.d, S.off, S.list));
        HIP_TRY(c, bhg::launch_exclusive_scan_u64(L, S.off, S.off, ch.cn, S.scan));
        HIP_TRY(c, hipMemcpyAsync(c->ptot + ch.slot, S.off + ch.cn, 8, hipMemcpyDeviceToHost, sc));
        HIP_TRY(c, hipEventRecord(c->pev[ch.slot], sc));
        return BHG_OK;
    };
    auto stage_b = [&](Chunk &ch) -> int {
        const Slot S = slot_of(ch.slot);
        HIP_TRY(c, hipEventSynchronize(c->pev[ch.slot]));
        const uint64_t tot = c->ptot[ch.slot];
        ch.vb = vbase;
        ch.fit = vbase >= out_vals_cap ? 0 : (tot < out_vals_cap - vbase ? tot : out_vals_cap - vbase);
        if (int r = ensure_buf(c, &c->pvals[ch.slot], &c->pvals_cap[ch.slot], ch.fit + 80)) return r;
        ch.mis = mvals ? (((uintptr_t)mvals + vbase) & 15u) : 0u;
        uint8_t *dv = reinterpret_cast<uint8_t *>(c->pvals[ch.slot]) + ch.mis;
        const uint64_t ecap = out_vals_cap < vbase + tot ? out_vals_cap : vbase + tot;
        HIP_TRY(c, bhg::launch_add_u64(L, S.off, (uint64_t)ch.cn + 1, vbase, 1));
        if (int r = ensure_buf(c, &c->pbig[ch.slot], &c->pbig_cap[ch.slot], bhg::snappy_big_bytes(ch.cn, ecap))) return r;
        HIP_TRY(c, bhg::launch_snappy(L, S.src, ch.hi - ch.lo, S.h, ch.cn, S.d, dv - vbase, ecap, S.off, S.list,
                                      c->pbig[ch.slot]));
        HIP_TRY(c, hipEventRecord(c->pevb[ch.slot], sc));
        vbase += tot;
        return BHG_OK;
    };
    // staging layout of a slot: values (fit bytes), offsets, descriptors
    auto stage_offs = [&](const Chunk &ch, size_t &o_off, size_t &o_desc) {
        o_off = al(ch.fit + 16);
        o_desc = o_off + al(((size_t)ch.cn + 1) * 8);
        return o_desc + al((size_t)ch.cn * sizeof(bhg_desc));
    };
    auto stage_d = [&](const Chunk &ch) -> int {
        const Slot S = slot_of(ch.slot);
        HIP_TRY(c, hipStreamWaitEvent(sd, c->pevb[ch.slot], 0));
        if (staged) {
            size_t o_off, o_desc;
            const size_t need_s = stage_offs(ch, o_off, o_desc);
            if (need_s > c->pstage_cap[ch.slot]) {  // free: its last chunk was copied on (see drain)
                if (c->pstage[ch.slot]) HIP_TRY(c, hipHostFree(c->pstage[ch.slot]));
                c->pstage[ch.slot] = nullptr;
                c->pstage_cap[ch.slot] = 0;
                const size_t sz = need_s + need_s / 4 + 4096;
                HIP_TRY(c, hipHostMalloc(reinterpret_cast<void **>(&c->pstage[ch.slot]), sz, hipHostMallocMapped));
                c->pstage_cap[ch.slot] = sz;
                void *dp = nullptr;
                HIP_TRY(c, hipHostGetDevicePointer(&dp, c->pstage[ch.slot], 0));
                c->pstage_dev[ch.slot] = static_cast<uint8_t *>(dp);
            }
            uint8_t *sdv = c->pstage_dev[ch.slot];
            const uint8_t *dv = reinterpret_cast<const uint8_t *>(c->pvals[ch.slot]) + ch.mis;
            HIP_TRY(c, bhg::launch_copy_out(Ld, dv, sdv, ch.fit));
            HIP_TRY(c, bhg::launch_copy_out(Ld, reinterpret_cast<const uint8_t *>(S.off), sdv + o_off,
                                            ((size_t)ch.cn + 1) * 8));
            HIP_TRY(c, bhg::launch_copy_out(Ld, reinterpret_cast<const uint8_t *>(S.d), sdv + o_desc,
                                            (size_t)ch.cn * sizeof(bhg_desc)));
            HIP_TRY(c, hipEventRecord(c->pevd[ch.slot], sd));
            dpend[ch.slot] = true;
            return BHG_OK;
        }
        const uint8_t *dv = reinterpret_cast<const uint8_t *>(c->pvals[ch.slot]) + ch.mis;
        if (ch.fit && mvals) HIP_TRY(c, bhg::launch_copy_out(Ld, dv, mvals + ch.vb, ch.fit));
        else if (ch.fit) HIP_TRY(c, hipMemcpyAsync(out_vals + ch.vb, dv, ch.fit, hipMemcpyDeviceToHost, sd));
        HIP_TRY(c, hipMemcpyAsync(out_val_off + ch.a, S.off, ((size_t)ch.cn + 1) * 8, hipMemcpyDeviceToHost, sd));
        HIP_TRY(c, hipMemcpyAsync(out_desc + ch.a, S.d, (size_t)ch.cn * sizeof(bhg_desc), hipMemcpyDeviceToHost, sd));
        HIP_TRY(c, hipEventRecord(c->pevd[ch.slot], sd));
        dpend[ch.slot] = true;
        return BHG_OK;
    };
    auto next = [&](uint32_t a, int slot) {
        Chunk ch{};
        ch.a = a;
        ch.slot = slot;
        const uint32_t b = next_chunk(handles, a, n, src_len, kChunkBytes, max_chunk_n, &prev_off, &ch.lo, &ch.hi,
                                      &unsorted);
        ch.cn = b - a;
        return ch;
    };
    // staged: chunk ch's staging -> the caller's buffers on the host threads (the offsets' last
    // entry only from the batch's last chunk: the next chunk writes the same word)
    auto drain = [&](const Chunk &ch) -> int {
        HIP_TRY(c, hipEventSynchronize(c->pevd[ch.slot]));
        size_t o_off, o_desc;
        stage_offs(ch, o_off, o_desc);
        const uint8_t *st = c->pstage[ch.slot];
        const bool last = ch.a + ch.cn >= n;
        c->hpool->submit({{out_vals + ch.vb, st, ch.fit},
                          {reinterpret_cast<uint8_t *>(out_val_off + ch.a), st + o_off, ((size_t)ch.cn + last) * 8},
                          {reinterpret_cast<uint8_t *>(out_desc + ch.a), st + o_desc, (size_t)ch.cn * sizeof(bhg_desc)}});
        return BHG_OK;
    };
    Chunk cur = next(0, 0), prev{};
    bool have_prev = false;
    if (int r = stage_a(cur)) return r;
    for (;;) {
        if (int r = stage_b(cur)) return r;
        const uint32_t b = cur.a + cur.cn;
        Chunk nx{};
        if (b < n) {
            nx = next(b, (cur.slot + 1) % bhg_ctx::kPipe);
            if (int r = stage_a(nx)) return r;
        }
        if (int r = stage_d(cur)) return r;
        if (staged) {
            // a slot's staging is rewritten by stage D three chunks on: submit() first waits for the
            // previous host copy, so chunk k - 3's copy is done before chunk k's kernels are queued
            if (have_prev)
                if (int r = drain(prev)) return r;
            prev = cur;
            have_prev = true;
        }
        if (b >= n) break;
        cur = nx;
    }
    if (staged && have_prev)
        if (int r = drain(prev)) return r;
    HIP_TRY(c, hipStreamSynchronize(sd));
    HIP_TRY(c, hipStreamSynchronize(sc));
    return BHG_OK;
}

// Device address of a host pointer that is page-locked AND mapped into this
// device's address space (bhg_host_register / bhg_malloc_host), else nullptr.
const void *mapped_device_ptr(const void *p) {
    if (!p) return nullptr;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory: clear the sticky "invalid value"
        return nullptr;
    }
    if (at.type != hipMemoryTypeHost || !at.devicePointer) return nullptr;
    return at.devicePointer;
}

// Zero-copy end-to-end NoCompressor decode: src is page-locked and mapped, so
// the decode kernel reads the table bytes straight over PCIe (one pass, no
// staging copy, any handle order); handles / expected CRCs go H2D and the
// descriptors come back D2H (or are written straight into out_desc when it is
// mapped as well).  Used for UNSORTED handles (sorted ones take the chunked
// pipeline, which is faster: 49.7 vs 40 GiB/s, scripts/lab/e2e_lab.py); the bare
// kernel on mapped bytes runs at 45 GiB/s vs 53 GiB/s for an SDMA copy
// (scripts/lab/h2d_lab.hip).
int decode_host_mapped(bhg_ctx *c, const uint8_t *dsrc, uint64_t src_len, const bhg_handle *handles, uint32_t n,
                       const uint32_t *expected_crc, bhg_desc *out_desc) {
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t hb = (size_t)n * sizeof(bhg_handle), db = (size_t)n * sizeof(bhg_desc);
    const size_t eb = expected_crc ? (size_t)n * 4 : 0;
    bhg_desc *ddesc = const_cast<bhg_desc *>(static_cast<const bhg_desc *>(mapped_device_ptr(out_desc)));
    const bhg_handle *mh = static_cast<const bhg_handle *>(mapped_device_ptr(handles));
    const uint32_t *me = static_cast<const uint32_t *>(mapped_device_ptr(expected_crc));
    if (int r = ensure_buf(c, &c->h_aux, &c->h_aux_cap, al(hb) + al(db) + al(eb) + 256)) return r;
    uint8_t *a = reinterpret_cast<uint8_t *>(c->h_aux);
    bhg_handle *dh = reinterpret_cast<bhg_handle *>(a); a += al(hb);
    bhg_desc *dd = reinterpret_cast<bhg_desc *>(a); a += al(db);
    uint32_t *de = expected_crc ? reinterpret_cast<uint32_t *>(a) : nullptr;
    hipStream_t s = c->stream;
    if (mh) dh = const_cast<bhg_handle *>(mh);
    else HIP_TRY(c, hipMemcpyAsync(dh, handles, hb, hipMemcpyHostToDevice, s));
    if (de) {
        if (me) de = const_cast<uint32_t *>(me);
        else HIP_TRY(c, hipMemcpyAsync(de, expected_crc, eb, hipMemcpyHostToDevice, s));
    }
    bhg::Launch L = launch_of(c, nullptr);
    HIP_TRY(c, bhg::launch_decode(L, dsrc, src_len, dh, n, BHG_CODEC_NONE, de, ddesc ? ddesc : dd, nullptr));
    if (!ddesc) HIP_TRY(c, hipMemcpyAsync(out_desc, dd, db, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    return BHG_OK;
}

}  // namespace

int bhg_decode_batch_host(bhg_ctx *c, const uint8_t *src, uint64_t src_len, const bhg_handle *handles, uint32_t n,
                          int codec, const uint32_t *expected_crc, bhg_desc *out_desc, uint8_t *out_vals,
                          uint64_t out_vals_cap, uint64_t *out_val_off) {
    if (!c) return BHG_EINVAL;
    if (codec != BHG_CODEC_NONE && codec != BHG_CODEC_SNAPPY) { set_err(c, "bad codec %d", codec); return BHG_EINVAL; }
    if (n == 0) {
        if (codec == BHG_CODEC_SNAPPY && out_val_off) out_val_off[0] = 0;
        return BHG_OK;
    }
    if (!handles || !out_desc || (!src && src_len)) { set_err(c, "null buffer"); return BHG_EINVAL; }
    if (codec == BHG_CODEC_SNAPPY && !out_val_off) { set_err(c, "snappy decode needs out_val_off[n+1]"); return BHG_EINVAL; }
    if (int r = set_device(c)) return r;
    std::lock_guard<std::mutex> g(c->mu);
    if (codec == BHG_CODEC_SNAPPY && out_vals) {
        // sorted handles: the chunked two-stage pipeline (H2D of chunk k + 1 under chunk k's D2H);
        // otherwise the whole batch below
        const int r = decode_host_snappy_pipelined(c, src, src_len, handles, n, expected_crc, out_desc, out_vals,
                                                   out_vals_cap, out_val_off);
        if (r != -100) return r;
    }
    if (codec == BHG_CODEC_NONE) {
        // handles in offset order: the chunked pipeline (49.7 GiB/s with src, handles and descriptors
        // pinned, 44 pageable; scripts/lab/e2e_lab.py); from the first handle out of order on (or an
        // oversized record), a mapped src is decoded in place (40 GiB/s), which beats copying all of
        // src before the kernel, else the whole-batch path below
        uint32_t done = 0;
        const int r = decode_host_pipelined(c, src, src_len, handles, n, expected_crc, out_desc, &done);
        if (r != -100) return r;
        handles += done;
        out_desc += done;
        if (expected_crc) expected_crc += done;
        n -= done;
        if (const void *dsrc = mapped_device_ptr(src))
            return decode_host_mapped(c, static_cast<const uint8_t *>(dsrc), src_len, handles, n, expected_crc,
                                      out_desc);
    }
    const size_t hb = (size_t)n * sizeof(bhg_handle), db = (size_t)n * sizeof(bhg_desc);
    const size_t eb = expected_crc ? (size_t)n * 4 : 0, ob = codec == BHG_CODEC_SNAPPY ? ((size_t)n + 1) * 8 : 0;
    const size_t sb = codec == BHG_CODEC_SNAPPY ? bhg::scan_scratch_bytes(n) : 0;
    const size_t lb = codec == BHG_CODEC_SNAPPY && out_vals ? bhg::snappy_list_bytes(n) : 0;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    if (int r = ensure_buf(c, &c->h_src, &c->h_src_cap, src_len + 64)) return r;
    if (int r = ensure_buf(c, &c->h_aux, &c->h_aux_cap, al(hb) + al(db) + al(eb) + al(ob) + al(sb) + al(lb) + 256)) return r;
    uint8_t *a = reinterpret_cast<uint8_t *>(c->h_aux);
    bhg_handle *dh = reinterpret_cast<bhg_handle *>(a); a += al(hb);
    bhg_desc *dd = reinterpret_cast<bhg_desc *>(a); a += al(db);
    uint32_t *de = expected_crc ? reinterpret_cast<uint32_t *>(a) : nullptr; a += al(eb);
    uint64_t *doff = ob ? reinterpret_cast<uint64_t *>(a) : nullptr; a += al(ob);
    void *dscan = sb ? a : nullptr; a += al(sb);
    uint32_t *dlist = lb ? reinterpret_cast<uint32_t *>(a) : nullptr;
    hipStream_t s = c->stream;
    HIP_TRY(c, hipMemcpyAsync(c->h_src, src, src_len, hipMemcpyHostToDevice, s));
    HIP_TRY(c, hipMemcpyAsync(dh, handles, hb, hipMemcpyHostToDevice, s));
    if (de) HIP_TRY(c, hipMemcpyAsync(de, expected_crc, eb, hipMemcpyHostToDevice, s));
    bhg::Launch L = launch_of(c, nullptr);
    const uint8_t *dsrc = reinterpret_cast<const uint8_t *>(c->h_src);
    HIP_TRY(c, bhg::launch_decode(L, dsrc, src_len, dh, n, codec, de, dd, doff,
                                  codec == BHG_CODEC_SNAPPY && out_vals ? dlist : nullptr));
    if (codec == BHG_CODEC_SNAPPY) {
        HIP_TRY(c, bhg::launch_exclusive_scan_u64(L, doff, doff, n, dscan));
        HIP_TRY(c, hipMemcpyAsync(out_val_off, doff, ob, hipMemcpyDeviceToHost, s));
        HIP_TRY(c, hipStreamSynchronize(s));
        if (out_vals) {
            // the device value buffer is sized from the scanned total, capped by what the caller can take;
            // a page-locked + mapped out_vals is written by the copy kernel (the link rate, see
            // decode_host_snappy_pipelined), the values then placed at its address's offset mod 16
            uint64_t total = out_val_off[n];
            if (total > out_vals_cap) total = out_vals_cap;
            if (int r = ensure_buf(c, &c->h_vals, &c->h_vals_cap, total + 80)) return r;
            uint8_t *mv = const_cast<uint8_t *>(static_cast<const uint8_t *>(mapped_device_ptr(out_vals)));
            uint8_t *dv = reinterpret_cast<uint8_t *>(c->h_vals) + (mv ? ((uintptr_t)mv & 15u) : 0u);
            if (int r = ensure_buf(c, &c->h_big, &c->h_big_cap, bhg::snappy_big_bytes(n, total))) return r;
            HIP_TRY(c, bhg::launch_snappy(L, dsrc, src_len, dh, n, dd, dv, total, doff, dlist, c->h_big));
            if (total && mv) HIP_TRY(c, bhg::launch_copy_out(L, dv, mv, total));
            else if (total) HIP_TRY(c, hipMemcpyAsync(out_vals, dv, total, hipMemcpyDeviceToHost, s));
        }
    }
    HIP_TRY(c, hipMemcpyAsync(out_desc, dd, db, hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    return BHG_OK;
}

int bhg_get_batch(bhg_ctx *c, const uint8_t *src, uint64_t src_len, const bhg_table *tables, uint32_t ntables,
                  const uint8_t *keys, const uint64_t *key_off, const uint32_t *table_idx, const uint32_t *khash,
                  uint32_t n, bhg_handle *out_handles, uint32_t *out_status, void *stream) {
    if (!c) return BHG_EINVAL;
    if (n == 0) return BHG_OK;
    if (!tables || !key_off || !table_idx || !out_handles || !out_status || (!src && src_len) || !keys) {
        set_err(c, "null buffer");
        return BHG_EINVAL;
    }
    if (int r = set_device(c)) return r;
    HIP_TRY(c, bhg::launch_get(launch_of(c, stream), src, src_len, tables, ntables, keys, key_off, table_idx, khash, n,
                               out_handles, out_status));
    return BHG_OK;
}

int bhg_writer_index_build(bhg_ctx *c, const uint32_t *khash, uint32_t n, uint32_t *sorted, uint32_t *sorted_kh,
                           void *stream) {
    if (!c) return BHG_EINVAL;
    if (n == 0) return BHG_OK;
    if (!khash || !sorted || !sorted_kh) {
        set_err(c, "null buffer");
        return BHG_EINVAL;
    }
    if (int r = set_device(c)) return r;
    bhg::Launch L = launch_of(c, stream);
    Scratch sc;
    if (int r = scratch_alloc(c, L.stream, bhg::writer_index_scratch_bytes(n), sc)) return r;
    HIP_TRY(c, bhg::launch_writer_index(L, khash, n, sorted, sorted_kh, sc.base));
    return BHG_OK;
}

int bhg_bithash_get_batch(bhg_ctx *c, const uint8_t *src, uint64_t src_len, const bhg_writer_index *writers,
                          uint32_t nwriters, const bhg_table *tables, uint32_t ntables, const uint32_t *fn_map,
                          const uint32_t *fn_table, uint32_t fn_count, const uint8_t *keys, const uint64_t *key_off,
                          const uint32_t *file_nums, const uint32_t *khash, int codec, uint32_t n,
                          bhg_handle *out_handles, uint32_t *out_status, void *stream) {
    if (!c) return BHG_EINVAL;
    if (codec != BHG_CODEC_NONE && codec != BHG_CODEC_SNAPPY) {
        set_err(c, "unknown codec");
        return BHG_EINVAL;
    }
    if (n == 0) return BHG_OK;
    if (!key_off || !file_nums || !out_handles || !out_status || (!src && src_len) || !keys ||
        (nwriters && !writers) || (ntables && !tables) || (fn_count && (!fn_map || !fn_table))) {
        set_err(c, "null buffer");
        return BHG_EINVAL;
    }
    if (int r = set_device(c)) return r;
    HIP_TRY(c, bhg::launch_bithash_get(launch_of(c, stream), src, src_len, writers, nwriters, tables, ntables, fn_map,
                                       fn_table, fn_count, keys, key_off, file_nums, khash, codec, n,
                                       out_handles, out_status));
    return BHG_OK;
}

int bhg_host_register(bhg_ctx *c, void *p, uint64_t bytes) {
    if (!c || !p || !bytes) return BHG_EINVAL;
    if (int r = set_device(c)) return r;
    // mapped: the NoCompressor host path then decodes the bytes in place over PCIe (zero copy)
    HIP_TRY(c, hipHostRegister(p, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
    return BHG_OK;
}

int bhg_host_unregister(bhg_ctx *c, void *p) {
    if (!c || !p) return BHG_EINVAL;
    if (int r = set_device(c)) return r;
    HIP_TRY(c, hipHostUnregister(p));
    return BHG_OK;
}

int bhg_crc32c_masked_batch(bhg_ctx *c, const uint8_t *src, uint64_t src_len, const bhg_handle *handles, uint32_t n,
                            uint32_t *out_crc, void *stream) {
    if (!c) return BHG_EINVAL;
    if (n == 0) return BHG_OK;
    if (!handles || !out_crc || (!src && src_len)) { set_err(c, "null buffer"); return BHG_EINVAL; }
    if (int r = set_device(c)) return r;
    HIP_TRY(c, bhg::launch_crc_ranges(launch_of(c, stream), src, src_len, handles, n, out_crc));
    return BHG_OK;
}

int bhg_crc32c_masked_long(bhg_ctx *c, const uint8_t *src, uint64_t src_len, const bhg_handle *handles, uint32_t n,
                           uint32_t *out_crc, void *stream) {
    if (!c) return BHG_EINVAL;
    if (n == 0) return BHG_OK;
    if (!handles || !out_crc || (!src && src_len)) { set_err(c, "null buffer"); return BHG_EINVAL; }
    if (int r = set_device(c)) return r;
    bhg::Launch L = launch_of(c, stream);
    Scratch sc;
    if (int r = scratch_alloc(c, L.stream, bhg::crc_long_scratch_bytes(n), sc)) return r;
    HIP_TRY(c, bhg::launch_crc_long(L, src, src_len, handles, n, out_crc, sc.base));
    return BHG_OK;
}

int bhg_fnv32_batch(bhg_ctx *c, const uint8_t *src, uint64_t src_len, const bhg_handle *handles, uint32_t n,
                    uint32_t *out_fnv, void *stream) {
    if (!c) return BHG_EINVAL;
    if (n == 0) return BHG_OK;
    if (!handles || !out_fnv || (!src && src_len)) { set_err(c, "null buffer"); return BHG_EINVAL; }
    if (int r = set_device(c)) return r;
    HIP_TRY(c, bhg::launch_fnv_ranges(launch_of(c, stream), src, src_len, handles, n, out_fnv));
    return BHG_OK;
}

namespace {

bool encode_outputs_ok(bhg_ctx *c, const bhg_encode_out *o, uint32_t n, uint32_t max_tables) {
    if (!o || !o->table_start || !o->summary || max_tables < 1) { set_err(c, "bad encode outputs"); return false; }
    if (n && (!o->pos || !o->bh_off || !o->bh_len || !o->table || !o->fnv1 || !o->crc || !o->status)) {
        set_err(c, "null buffer");
        return false;
    }
    return true;
}

// empty batch: summary {0, 1, 0, 0}, table_start[0] = 0
int encode_empty(bhg_ctx *c, const bhg_encode_out *o, hipStream_t s) {
    static const uint64_t summ[4] = {0, 1, 0, 0};
    HIP_TRY(c, hipMemcpyAsync(o->summary, summ, 32, hipMemcpyHostToDevice, s));
    HIP_TRY(c, hipMemsetAsync(o->table_start, 0, 4, s));
    return BHG_OK;
}

}  // namespace

int bhg_encode_batch(bhg_ctx *c, const uint8_t *keys, const uint64_t *key_off, const uint64_t *trailers,
                     const uint8_t *vals, const uint64_t *val_off, uint64_t vals_len, uint32_t n, int codec,
                     const uint32_t *file_nums, uint32_t max_tables, uint32_t init_size, uint64_t table_max,
                     uint8_t *out, uint64_t out_cap, const bhg_encode_out *o, void *stream) {
    if (!c) return BHG_EINVAL;
    if (!encode_outputs_ok(c, o, n, max_tables)) return BHG_EINVAL;
    if (!file_nums) { set_err(c, "null file_nums"); return BHG_EINVAL; }
    if (codec != BHG_CODEC_NONE && codec != BHG_CODEC_SNAPPY) { set_err(c, "bad codec %d", codec); return BHG_EINVAL; }
    // DATA_MAX_EXCEEDED (writer.go:266-269) cannot trigger when size < table_max and
    // table_max + max record <= dataMaxSize; larger tables are rejected up front.
    const uint64_t data_max = 0xFFFFFFFFull - (256ull << 20);
    if (table_max == 0 || table_max + (33ull << 10) + (256ull << 20) + 12 > data_max || init_size >= table_max) {
        set_err(c, "table_max/init_size out of range");
        return BHG_EINVAL;
    }
    if (int r = set_device(c)) return r;
    bhg::Launch L = launch_of(c, stream);
    if (n == 0) return encode_empty(c, o, L.stream);
    if (!keys || !key_off || !trailers || !vals || !val_off || !out) { set_err(c, "null buffer"); return BHG_EINVAL; }
    const size_t lens_b = ((size_t)n + 1) * 8, vlen_b = ((size_t)n + 1) * 8, scan_b = bhg::scan_scratch_bytes(n);
    size_t snap_b = 0, soff_b = 0, blk_b = 0, cls_b = 0;
    if (codec == BHG_CODEC_SNAPPY) {
        // sum MaxEncodedLen = 32 n + V + sum(v_i / 6) <= 32 n + V + V / 6 (encode.go MaxEncodedLen)
        snap_b = (size_t)(32ull * n + vals_len + vals_len / 6 + 64);
        soff_b = ((size_t)n + 1) * 8;
        blk_b = bhg::snappy_block_scratch_bytes(n, vals_len);
        cls_b = bhg::snappy_enc_list_bytes(n);
    }
    // a batch of long values (mean past kLongMean, the decode's rule): records longer than kLongRec are
    // copied and CRC'd by whole-chip passes (bhg_encode.hip k_enc_lcopy + bhg_longcrc.hip)
    const uint64_t vbound = codec == BHG_CODEC_SNAPPY ? snap_b : vals_len;  // the buffer value' bytes lie in
    const size_t long_b = bhg::long_batch(vals_len, n) ? bhg::enc_long_scratch_bytes(n, vbound) : 0;
    Scratch sc;
    const size_t al6 = 7 * 256;
    if (int r = scratch_alloc(c, L.stream, lens_b + vlen_b + scan_b + snap_b + soff_b + blk_b + cls_b + long_b + al6, sc))
        return r;
    bhg::EncodeLaunch E;
    memset(&E, 0, sizeof E);
    E.lens = reinterpret_cast<uint64_t *>(sc.take(lens_b));
    uint64_t *vlen = reinterpret_cast<uint64_t *>(sc.take(vlen_b));
    E.scan_scratch = sc.take(scan_b);
    E.long_scratch = long_b ? sc.take(long_b) : nullptr;
    if (codec == BHG_CODEC_SNAPPY) {
        uint8_t *snap = sc.take(snap_b);
        uint64_t *soff = reinterpret_cast<uint64_t *>(sc.take(soff_b));
        void *blk = sc.take(blk_b);
        uint32_t *cls = reinterpret_cast<uint32_t *>(sc.take(cls_b));
        HIP_TRY(c, bhg::launch_snappy_maxlen(L, val_off, n, soff));
        HIP_TRY(c, bhg::launch_exclusive_scan_u64(L, soff, soff, n, E.scan_scratch));
        HIP_TRY(c, bhg::launch_snappy_enc(L, vals, val_off, n, vals_len, snap, snap_b, soff, vlen, cls, blk));
        E.vbase = snap; E.vpos = soff; E.vlen = vlen; E.vend = snap + snap_b;
    } else {
        HIP_TRY(c, bhg::launch_enc_rawvals(L, val_off, n, vlen));
        E.vbase = vals; E.vpos = val_off; E.vlen = vlen; E.vend = vals + vals_len;
    }
    E.keys = keys; E.key_off = key_off; E.trailers = trailers;
    E.n = n; E.file_nums = file_nums; E.max_tables = max_tables; E.init_size = init_size; E.table_max = table_max;
    E.out = out; E.out_cap = out_cap; E.o = *o;
    HIP_TRY(c, bhg::launch_encode(L, E));
    return BHG_OK;
}

int bhg_encode_ikey_batch(bhg_ctx *c, const uint8_t *keys, const uint64_t *key_off, const uint64_t *trailers,
                          const uint8_t *vals, const uint64_t *val_off, uint32_t n, const uint32_t *khash,
                          const uint32_t *rec_file_nums, const uint8_t *live, uint32_t init_size, uint8_t *out,
                          uint64_t out_cap, const bhg_encode_out *o, void *stream) {
    if (!c) return BHG_EINVAL;
    if (!encode_outputs_ok(c, o, n, 1)) return BHG_EINVAL;
    if (int r = set_device(c)) return r;
    bhg::Launch L = launch_of(c, stream);
    if (n == 0) return encode_empty(c, o, L.stream);
    if (!keys || !key_off || !trailers || !vals || !val_off || !out || !rec_file_nums) {
        set_err(c, "null buffer");
        return BHG_EINVAL;
    }
    const size_t lens_b = ((size_t)n + 1) * 8, vlen_b = ((size_t)n + 1) * 8, scan_b = bhg::scan_scratch_bytes(n);
    Scratch sc;
    if (int r = scratch_alloc(c, L.stream, lens_b + vlen_b + scan_b + 3 * 256, sc)) return r;
    bhg::EncodeLaunch E;
    memset(&E, 0, sizeof E);
    E.lens = reinterpret_cast<uint64_t *>(sc.take(lens_b));
    uint64_t *vlen = reinterpret_cast<uint64_t *>(sc.take(vlen_b));
    E.scan_scratch = sc.take(scan_b);
    HIP_TRY(c, bhg::launch_enc_rawvals(L, val_off, n, vlen));
    E.vbase = vals; E.vpos = val_off; E.vlen = vlen;
    E.keys = keys; E.key_off = key_off; E.trailers = trailers; E.n = n;
    E.file_nums = rec_file_nums;  // unused for the header (rec_file_nums wins); table 0's entry is record 0's
    E.rec_file_nums = rec_file_nums; E.live = live; E.khash = khash; E.single_table = 1;
    E.max_tables = 1; E.init_size = init_size; E.table_max = UINT64_MAX;
    E.out = out; E.out_cap = out_cap; E.o = *o;
    HIP_TRY(c, bhg::launch_encode(L, E));
    return BHG_OK;
}

int bhg_repack_batch(bhg_ctx *c, const uint8_t *src, uint64_t src_len, const bhg_handle *handles, uint32_t n,
                     const uint8_t *live, const uint32_t *khash, uint32_t init_size, uint8_t *out, uint64_t out_cap,
                     const bhg_encode_out *o, void *stream) {
    if (!c) return BHG_EINVAL;
    if (!encode_outputs_ok(c, o, n, 1)) return BHG_EINVAL;
    if (int r = set_device(c)) return r;
    bhg::Launch L = launch_of(c, stream);
    if (n == 0) return encode_empty(c, o, L.stream);
    if (!src || !handles || !out) { set_err(c, "null buffer"); return BHG_EINVAL; }
    const size_t N = (size_t)n + 1;
    // a compaction of long records: their copies and CRCs by whole-chip passes, as bhg_encode_batch's
    const size_t long_b = bhg::long_batch(src_len, n) ? bhg::enc_long_scratch_bytes(n, src_len) : 0;
    Scratch sc;
    if (int r = scratch_alloc(c, L.stream, 7 * N * 8 + 3 * N * 4 + bhg::scan_scratch_bytes(n) + long_b + 13 * 256, sc))
        return r;
    bhg::EncodeLaunch E;
    memset(&E, 0, sizeof E);
    E.lens = reinterpret_cast<uint64_t *>(sc.take(N * 8));
    E.scan_scratch = sc.take(bhg::scan_scratch_bytes(n));
    E.long_scratch = long_b ? sc.take(long_b) : nullptr;
    uint64_t *key_off = reinterpret_cast<uint64_t *>(sc.take(N * 8));
    uint32_t *key_len = reinterpret_cast<uint32_t *>(sc.take(N * 4));
    uint64_t *trailers = reinterpret_cast<uint64_t *>(sc.take(N * 8));
    uint64_t *vpos = reinterpret_cast<uint64_t *>(sc.take(N * 8));
    uint64_t *vlen = reinterpret_cast<uint64_t *>(sc.take(N * 8));
    uint32_t *fns = reinterpret_cast<uint32_t *>(sc.take(N * 4));
    uint32_t *pre = reinterpret_cast<uint32_t *>(sc.take(N * 4));
    HIP_TRY(c, bhg::launch_repack_prep(L, src, src_len, handles, n, key_off, key_len, trailers, vpos, vlen, fns, pre));
    E.keys = src; E.key_off = key_off; E.key_len = key_len; E.trailers = trailers;
    E.vbase = src; E.vpos = vpos; E.vlen = vlen; E.vend = src + src_len; E.n = n;
    E.file_nums = fns; E.rec_file_nums = fns; E.live = live; E.khash = khash; E.pre_status = pre;
    E.single_table = 1; E.max_tables = 1; E.init_size = init_size; E.table_max = UINT64_MAX;
    E.out = out; E.out_cap = out_cap; E.o = *o;
    HIP_TRY(c, bhg::launch_encode(L, E));
    return BHG_OK;
}

namespace {
int scan_tables(bhg_ctx *c, const uint8_t *src, const uint64_t *table_off, uint32_t ntables, int mode,
                bhg_handle *out_handles, uint64_t max_out, uint64_t *out_first, uint64_t *out_end, uint32_t *out_path,
                void *stream) {
    if (!c) return BHG_EINVAL;
    if (mode != 0 && mode != 1) { set_err(c, "bad scan mode %d", mode); return BHG_EINVAL; }
    if (!out_first) { set_err(c, "scan needs out_first[ntables+1]"); return BHG_EINVAL; }
    if (ntables == 0) return bhg_memset_device(c, out_first, 0, 8, stream);
    if (!src || !table_off || (!out_handles && max_out)) { set_err(c, "null buffer"); return BHG_EINVAL; }
    if (int r = set_device(c)) return r;
    bhg::Launch L = launch_of(c, stream);
    Scratch sc;
    const size_t sb = (bhg::scan_scratch_bytes(ntables) + 255) & ~(size_t)255;
    if (int r = scratch_alloc(c, L.stream, sb + bhg::tscan_uni_bytes(ntables), sc)) return r;
    HIP_TRY(c, bhg::launch_tscan(L, src, table_off, ntables, mode, out_handles, max_out, out_first, out_end, sc.base,
                                 static_cast<uint8_t *>(sc.base) + sb, out_path));
    return BHG_OK;
}
}  // namespace

int bhg_scan_tables(bhg_ctx *c, const uint8_t *src, const uint64_t *table_off, uint32_t ntables, int mode,
                    bhg_handle *out_handles, uint64_t max_out, uint64_t *out_first, uint64_t *out_end, void *stream) {
    return scan_tables(c, src, table_off, ntables, mode, out_handles, max_out, out_first, out_end, nullptr, stream);
}

int bhg_scan_tables_paths(bhg_ctx *c, const uint8_t *src, const uint64_t *table_off, uint32_t ntables, int mode,
                          bhg_handle *out_handles, uint64_t max_out, uint64_t *out_first, uint64_t *out_end,
                          uint32_t *out_path, void *stream) {
    if (!out_path && ntables) { set_err(c, "null out_path"); return BHG_EINVAL; }
    return scan_tables(c, src, table_off, ntables, mode, out_handles, max_out, out_first, out_end, out_path, stream);
}

uint64_t bhg_scan_scratch_bytes(uint32_t ntables) {
    return ((bhg::scan_scratch_bytes(ntables) + 255) & ~(size_t)255) + bhg::tscan_uni_bytes(ntables);
}

int bhg_table_tail(bhg_ctx *c, const uint8_t *recs, const bhg_handle *rec, const uint32_t *bh_off,
                   const uint32_t *khash, const uint32_t *table, const uint32_t *status, uint32_t n,
                   uint32_t ntables, const uint64_t *data_end, uint8_t *tail, uint64_t tail_cap,
                   uint64_t *tail_off, uint64_t *tail_len, uint32_t *stats, void *stream) {
    if (!c) return BHG_EINVAL;
    if (!tail_off) { set_err(c, "table tail needs tail_off[ntables+1]"); return BHG_EINVAL; }
    if (ntables == 0) return bhg_memset_device(c, tail_off, 0, 8, stream);
    if (!data_end || !tail_len || (!tail && tail_cap)) { set_err(c, "null buffer"); return BHG_EINVAL; }
    if (n && (!recs || !rec || !bh_off || !khash || !table)) { set_err(c, "null buffer"); return BHG_EINVAL; }
    if (int r = set_device(c)) return r;
    bhg::Launch L = launch_of(c, stream);
    Scratch sc;
    if (int r = scratch_alloc(c, L.stream, bhg::tail_scratch_bytes(n, ntables), sc)) return r;
    bhg::TailLaunch T;
    T.recs = recs; T.rec = rec; T.bh_off = bh_off; T.khash = khash; T.table = table; T.status = status;
    T.n = n; T.ntables = ntables; T.data_end = data_end; T.tail = tail; T.tail_cap = tail ? tail_cap : 0;
    T.tail_off = tail_off; T.tail_len = tail_len; T.stats = stats;
    HIP_TRY(c, bhg::launch_table_tail(L, T, sc.base));
    return BHG_OK;
}

int bhg_rebuild_tables(bhg_ctx *c, const uint8_t *src, const uint64_t *table_off, uint32_t ntables,
                       bhg_handle *out_handles, uint64_t max_out, uint64_t *out_first, uint64_t *out_end,
                       uint32_t *out_khash, uint32_t *out_bh_off, uint32_t *out_table, void *stream) {
    if (!c) return BHG_EINVAL;
    if (max_out && (!out_khash || !out_bh_off || !out_table)) { set_err(c, "null buffer"); return BHG_EINVAL; }
    if (int r = bhg_scan_tables(c, src, table_off, ntables, 1, out_handles, max_out, out_first, out_end, stream))
        return r;
    if (ntables == 0 || max_out == 0) return BHG_OK;
    HIP_TRY(c, bhg::launch_rebuild_recs(launch_of(c, stream), src, table_off, ntables, out_handles, max_out,
                                        out_first, out_khash, out_bh_off, out_table));
    return BHG_OK;
}

}  // extern "C"
