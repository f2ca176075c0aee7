// bhg_decode_stream.hip -- launcher of k_decode_stream (bhg_decode_stream.h):
// the snappy header / CRC pass (MODE 1) of bhg_decode_batch.
#include "bhg_decode_stream.h"
#include "bhg_internal.h"

namespace bhg {

// CRC chains per window: 4 / 2 chains of 128-B windows, 4 / 8 of 256-B ones measured C3 595.5 / 599.1 /
// 566.8 / 565.0 GiB/s, mixdec 287.5 / 288.6 / 282.7 / 282.5 (2 alternating runs each, profiles/r6/stream/)
constexpr int kStreamNch = 2;
constexpr int kStreamWin = 128;   // window bytes
constexpr int kStreamPipe = 0;    // software-pipelined window loads (measured no faster)

size_t stream_tab_words() { return kStreamTabWords; }
void build_stream_tab_default(uint32_t *out) { build_stream_tab(out, kStreamWin, kStreamNch); }

// MODE 1 only: the NoCompressor decode is k_decode_tile (MODE 0 of this kernel measured
// slower, DESIGN.md 4.1, and stays a lab build)
hipError_t launch_decode_stream(const Launch &L, const uint8_t *src, uint64_t src_len, const bhg_handle *h, uint32_t n,
                                int mode, const uint32_t *expected_crc, bhg_desc *out, uint64_t *sizes,
                                uint32_t *lists, void *long_scratch) {
    if (mode != 1) return hipErrorInvalidValue;
    constexpr int WPB = 8;  // 156.5 KiB of LDS: one workgroup per CU
    const uint64_t tiles = (n + 63) / 64;
    const uint64_t need = (tiles + WPB - 1) / WPB, cap = (uint64_t)L.num_cus;
    uint32_t grid = (uint32_t)(need < cap ? need : cap);
    if (grid == 0) grid = 1;
    if (!long_scratch) {
        hipLaunchKernelGGL((k_decode_stream<1, kStreamNch, WPB, kStreamWin, kStreamPipe>), dim3(grid),
                           dim3(64 * WPB), 0, L.stream, src, src_len, h, n, expected_crc, out, sizes, L.stab, lists,
                           (uint32_t)snappy_sub_cap(n));
        return hipGetLastError();
    }
    // a batch of long records (long_batch): one wave streaming a multi-MiB record's windows was the
    // step's tail (bench.py --config bigval: 2.2 ms); their CRCs go to the whole-chip pass instead
    hipLaunchKernelGGL((k_decode_stream<1, kStreamNch, WPB, kStreamWin, kStreamPipe, 0, 1>), dim3(grid),
                       dim3(64 * WPB), 0, L.stream, src, src_len, h, n, expected_crc, out, sizes, L.stab, lists,
                       (uint32_t)snappy_sub_cap(n));
    if (hipError_t e = hipGetLastError()) return e;
    return launch_long_crc(L, src, src_len, h, n, expected_crc, out, long_scratch);
}

}  // namespace bhg
