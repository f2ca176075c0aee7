#!/bin/bash
# lab: the library of the committed tree (HEAD) into scripts/lab/abprev/lib/, for an A/B against the
# working tree's bitalosdb_amd/lib (bench.py with BHG_LIB_PATH=scripts/lab/abprev/lib/libbithashgpu.so)
set -e
R="$(cd "$(dirname "$0")/../../.." && pwd)"
T=$(mktemp -d)
git -C "$R" archive HEAD bitalosdb_amd/csrc include | tar -x -C "$T"
O="$R/scripts/lab/abprev/lib"
mkdir -p "$O/obj"
cd "$T/bitalosdb_amd/csrc"
for f in *.hip; do /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-function -munsafe-fp-atomics -c $f -o "$O/obj/${f%.hip}.o" & done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o "$O/libbithashgpu.so" "$O"/obj/*.o -lpthread
rm -rf "$T"
