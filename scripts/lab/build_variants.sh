#!/bin/bash
# builds libbithashgpu.so variants with one source file recompiled under extra -D flags, into
# scripts/lab/libvar/<name>/ (lab use: BHG_LIB_PATH=.../libbithashgpu.so python bench.py ...)
# usage: scripts/lab/build_variants.sh <file.hip> name1:"-DX=1" name2:"-DY=2" ...
set -e
F=$1; shift
cd "$(dirname "$0")/../../bitalosdb_amd/csrc"
OBJ=../lib/obj
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}
  d=../../scripts/lab/libvar/$name
  mkdir -p $d
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function -munsafe-fp-atomics $defs -c $F -o $d/var.o
  objs=$(ls $OBJ/*.o | grep -v "/${F%.hip}.o")
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o $d/libbithashgpu.so $objs $d/var.o -lpthread
  rm -f $d/var.o
done
