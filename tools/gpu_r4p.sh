#!/bin/bash
# Two RCCL ranks on one GPU (tools/rccl_same_gpu_probe.py), bounded.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4p
rm -rf $O; mkdir -p $O
timeout -k 10 120 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 tools/rccl_same_gpu_probe.py > $O/probe.log 2>&1
rc=$?; echo "rc=$rc"; grep -E "rank|rror|uplicate" $O/probe.log | head -20
