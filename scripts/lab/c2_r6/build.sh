#!/bin/bash
# builds the round-6 C2 labs (not product code)
set -e -o pipefail
cd "$(dirname "$0")"
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 --offload-arch=gfx950"
L="-L../../../bitalosdb_amd/lib -lbithashgpu -Wl,-rpath,\$ORIGIN/../../../bitalosdb_amd/lib"
$H $F -o tile_lab tile_lab.hip tile_var.hip $L
