#!/bin/bash
# Rehearse the N>1 bench path on a 1-GPU box: 2 ranks on cuda:0, gloo halo staged via host.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-dist}
SWARM_DIST_BACKEND=gloo timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --agents ${AGENTS:-2000000} --tasks 2000 \
    --steps 2 --warmup 1 > gpurun_out/bench_dist_$TAG.json 2> gpurun_out/bench_dist_$TAG.err
rc=$?; echo "dist bench rc=$rc"; cat gpurun_out/bench_dist_$TAG.json; tail -5 gpurun_out/bench_dist_$TAG.err
