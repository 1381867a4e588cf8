#!/bin/bash
# C5's exact shape on ONE GPU: NPROC ranks (default 8) x 100M / NPROC agents over the
# host-staged gloo group (libswarm's native loop over the shared-memory transport), checked against the C
# oracle on the 100M union (result_check.union_oracle), the union also elected on one GPU (the model's
# N = 1 time), and the election cost model.  PARTITION=blocks (Morton IDs; bench.py defaults to 16
# pieces per rank and a 4-round halo there) or strips.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${PARTITION:-blocks}; N=${NPROC:-8}; TAG=${TAG:-c5}
SWARM_DIST_BACKEND=gloo timeout -k 10 ${LIMIT:-900} python -u -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus $N --config ${CONFIG:-C5} \
    --partition $P --steps ${STEPS:-2} --warmup 1 --cpu-baseline 0 ${EXTRA:-} \
    > gpurun_out/${TAG}_$P.json 2> gpurun_out/${TAG}_$P.err
rc=$?; echo "c5 $P rc=$rc"; tail -c 3000 gpurun_out/${TAG}_$P.json; grep -v "^\[Gloo\]" gpurun_out/${TAG}_$P.err | tail -5
exit $rc
