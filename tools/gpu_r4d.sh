#!/bin/bash
# Round 4: the N > 1 bench path rehearsed on one GPU: 2 ranks over gloo, so the sharded C loops run
# over the shared-memory transport (election + allocation headline, C4 sharded auction row).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r4d}
SWARM_DIST_BACKEND=gloo timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --agents 2000000 \
    --cpu-baseline 0 > gpurun_out/bench_dist2_$TAG.json 2> gpurun_out/bench_dist2_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_dist2_$TAG.json; tail -5 gpurun_out/bench_dist2_$TAG.err
exit $rc
