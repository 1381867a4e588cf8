"""C5's shape through the bench's N > 1 path, scaled down to fit the GPU suite.

bench.py --config C5 with EIGHT ranks sharing one GPU (SWARM_DIST_BACKEND=gloo: libswarm's native
sharded loop over the shared-memory transport, 7 peers' worth of ranks), Morton blocks with Morton IDs
(SURVEY §8e's C5 partition: contiguous ID ranges, up to 8 neighbouring ranks) and strips; the line's
result_check.union_oracle compares every rank's leaders, rounds_exec and per-round global changes with
the C oracle over the union swarm.  --pieces 8: the same Morton swarm, its IDs cut into 64 ranges dealt
round-robin (rank q owns the q-th Morton piece of every block: 7 peers each).  The full-size run (8 x 12.5M) is the same command without --agents
(profiles/).  Transport "rccl-double": the same runs through the native loop's RCCL branch
(SWARM_NATIVE_COMM=rccl) over the RCCL test double (tests/rccl_double, SWARM_RCCL_PATH): the
ncclSend/ncclRecv pairing, per-peer counts and datatypes and the ncclSum counter all-reduce that C5 on 8
GPUs runs, executed with 8 real peers (real RCCL refuses several ranks on one GPU)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("partition,agents,pieces,transport",
                         [("blocks", 150_000, 1, "shm"), ("strips", 100_000, 1, "shm"), ("blocks", 150_000, 8, "shm"),
                          ("blocks", 150_000, 8, "rccl-double"), ("strips", 100_000, 1, "rccl-double")])
def test_c5_bench_eight_ranks_one_gpu_matches_union_oracle(partition, agents, pieces, transport, rccl_double):
    env = dict(os.environ, SWARM_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    if transport == "rccl-double":
        env.update(SWARM_NATIVE_COMM="rccl", SWARM_RCCL_PATH=rccl_double, RCCL_DOUBLE_TIMEOUT_S="60")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "8", "--config", "C5", "--agents", str(agents), "--tasks", "200", "--steps", "1",
           "--warmup", "0", "--cpu-baseline", "0", "--partition", partition, "--pieces", str(pieces)]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    if p.returncode:
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        with open(os.path.join(ROOT, "gpurun_out", f"c5_rehearsal_{partition}_{transport}.err"), "w") as f:
            f.write(p.stderr)
        keep = [q for q in p.stderr.splitlines() if "Error" in q or "error" in q or q.strip().startswith("File ")]
        raise AssertionError("\n".join(keep[:80]))
    line = [q for q in p.stdout.splitlines() if q.startswith("{")][-1]
    out = json.loads(line)
    u = out["result_check"]["union_oracle"]
    assert u["all_equal"] and u["agents_checked"] == 8 * agents == u["agents_union"], u
    assert out["n_gpus"] == 8 and out["scaling"] == "strong" and "REHEARSAL" in out["rehearsal"]
    if transport == "shm":
        assert "shared-memory" in out["config"]["parallelism"]
    else:  # the RCCL branch ran: ncclSend/ncclRecv groups and the counter all-reduces, through the double
        assert "native RCCL loop" in out["config"]["parallelism"] and "rccl_double" in out["config"]["parallelism"]
        st = out["rccl_double"]
        assert st["groups"] > 0 and st["sends"] > 0 and st["recvs"] > 0 and st["allreduce"] > 0, st
    if partition == "blocks":
        assert len(out["config"]["peers_rank0"]) >= (4 if pieces > 1 else 2)
    assert out["config"]["pieces"] == pieces
