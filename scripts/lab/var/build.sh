#!/bin/bash
# lab: a variant of the committed library -- HEAD's csrc with sed expressions applied -- into
# scripts/lab/var/<name>/lib/libbithashgpu.so (bench.py with BHG_LIB_PATH=<that>)
#   bash scripts/lab/var/build.sh <name> <file> '<sed expr>' [<file> '<sed expr>' ...]
set -e
R="$(cd "$(dirname "$0")/../../.." && pwd)"
name=$1; shift
T=$(mktemp -d)
git -C "$R" archive HEAD bitalosdb_amd/csrc include | tar -x -C "$T"
while [ $# -ge 2 ]; do sed -i "$2" "$T/bitalosdb_amd/csrc/$1"; grep -q . "$T/bitalosdb_amd/csrc/$1"; shift 2; done
O="$R/scripts/lab/var/$name/lib"
mkdir -p "$O/obj"
cd "$T/bitalosdb_amd/csrc"
for f in *.hip; do /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-unused-function -munsafe-fp-atomics -c $f -o "$O/obj/${f%.hip}.o" & done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o "$O/libbithashgpu.so" "$O"/obj/*.o -lpthread
rm -rf "$T" "$O/obj"
