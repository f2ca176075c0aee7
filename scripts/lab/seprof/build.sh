#!/bin/bash
# lab build of the library with the encoder's phase clocks (-DBHG_SE_PROF) into scripts/lab/seprof/lib/
set -e
cd "$(dirname "$0")/../../../bitalosdb_amd/csrc"
O=../../scripts/lab/seprof/lib
mkdir -p $O/obj
for f in *.hip; do /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-function -munsafe-fp-atomics -DBHG_SE_PROF -c $f -o $O/obj/${f%.hip}.o & done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o $O/libbithashgpu.so $O/obj/*.o -lpthread
