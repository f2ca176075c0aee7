// lab instantiations of k_decode_tile variants (not product code)
#include "../../../bitalosdb_amd/csrc/bhg_decode_tile.hip"
namespace bhg {
template __global__ void k_decode_tile<16, 2, 2, 1>(const uint8_t *, uint64_t, const bhg_handle *, uint32_t, const uint32_t *, bhg_desc *, const uint32_t *);
template __global__ void k_decode_tile<12, 2, 2, 1>(const uint8_t *, uint64_t, const bhg_handle *, uint32_t, const uint32_t *, bhg_desc *, const uint32_t *);
template __global__ void k_decode_tile<8, 2, 2, 1>(const uint8_t *, uint64_t, const bhg_handle *, uint32_t, const uint32_t *, bhg_desc *, const uint32_t *);
}
