#!/bin/bash
# A/B builds of the allocation: a source file (default alloc.hip; $SRC) compiled with extra flags ($2, e.g. "-DSWARM_ALLOC_WU=8"),
# linked with the other objects of the regular build into swarm_amd/libswarm_$1.so
# (tools/alloc_ab.py takes the library name).  CPU only; run `make` first.
set -eu
cd "$(dirname "$0")/../distributed-swarm-algorithm_amd/csrc"
name=$1; flags=${2:-}
mkdir -p build_dbg/var_$name
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
    -munsafe-fp-atomics $flags -c -o build_dbg/var_$name/${SRC:-alloc}.o ${SRC:-alloc}.hip
objs=$(ls build/*.o | grep -v "/${SRC:-alloc}.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../swarm_amd/libswarm_$name.so $objs build_dbg/var_$name/${SRC:-alloc}.o -ldl
echo "built swarm_amd/libswarm_$name.so"
