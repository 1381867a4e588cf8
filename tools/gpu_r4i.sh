#!/bin/bash
# Single-XCD persistent-round microbenchmark.
mkdir -p gpurun_out
timeout -k 10 120 tools/build/xcd_barrier_bench 2000 > gpurun_out/xcd_barrier_bench.json 2> gpurun_out/xcd_barrier_bench.err
echo "xcd rc=$?"
cat gpurun_out/xcd_barrier_bench.json gpurun_out/xcd_barrier_bench.err
