// lab instantiations of k_decode_tile variants (not product code): the current source and the
// committed HEAD~ copy (old_tile.hip, namespace bhg_old) for A/B timing
#include "../../../bitalosdb_amd/csrc/bhg_decode_tile.hip"
#include "old_tile.hip"
namespace bhg {
template __global__ void k_decode_tile<8, 2, 2, 2, 0>(const uint8_t *, uint64_t, const bhg_handle *, uint32_t, const uint32_t *, bhg_desc *, const uint32_t *);
}
namespace bhg_old {
template __global__ void k_decode_tile<8, 2, 2, 2, 0>(const uint8_t *, uint64_t, const bhg_handle *, uint32_t, const uint32_t *, bhg_desc *, const uint32_t *);
}
