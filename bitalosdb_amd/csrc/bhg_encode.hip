// bhg_encode.hip -- placeholder (encode kernels land in the next milestone)
#include "bhg_internal.h"
extern "C" {
int bhg_encode_batch(bhg_ctx *, const uint8_t *, const uint64_t *, const uint64_t *, const uint8_t *, const uint64_t *,
                     uint32_t, int, const uint32_t *, uint32_t, uint32_t, uint64_t, uint8_t *, uint64_t,
                     const bhg_encode_out *, void *) { return BHG_EINVAL; }
int bhg_scan_tables(bhg_ctx *, const uint8_t *, const uint64_t *, uint32_t, int, bhg_handle *, uint64_t, uint64_t *,
                    uint64_t *, void *) { return BHG_EINVAL; }
}
