#!/bin/bash
# builds the round-5 ring labs (not product code); non-zero exit on any compile error
set -e -o pipefail
cd "$(dirname "$0")"
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 --offload-arch=gfx950"
L="-L../../../bitalosdb_amd/lib -lbithashgpu -Wl,-rpath,\$ORIGIN/../../../bitalosdb_amd/lib"
$H $F -o ring_lab ring_lab.hip $L
$H $F -o ring_floor ring_floor.hip
