#!/bin/bash
# A/B builds: one source ($3, default elect.hip) compiled with extra flags ($2, e.g. "-DSWARM_PROBE_MARK2"),
# linked with the other objects of the regular build into swarm_amd/libswarm_$1.so
# (tools/elect_ab.py, tools/trace_ab.sh, tools/codec_probe.py take the library name).  CPU only; run
# `make` first.
set -eu
cd "$(dirname "$0")/../distributed-swarm-algorithm_amd/csrc"
name=$1; flags=${2:-}; src=${3:-elect.hip}; obj=${src%.hip}.o
mkdir -p build_dbg/var_$name
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
    -munsafe-fp-atomics $flags -c -o build_dbg/var_$name/$obj $src
objs=$(ls build/*.o | grep -v "/$obj\$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../swarm_amd/libswarm_$name.so $objs build_dbg/var_$name/$obj -ldl
echo "built swarm_amd/libswarm_$name.so"
