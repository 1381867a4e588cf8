"""swarm_amd -- MI355X-native batched swarm step (leader election + task allocation).

Public surface:
  Swarm, ElectResult, AllocResult   batched HBM-resident swarm (swarm.py), HIP kernels via
                                    libswarm.so (include/swarm.h)
  gen                               seeded synthetic inputs
  dist                              multi-GPU sharded election / allocation (torch.distributed)
The scalar drop-in for the reference's `agent` module lives next to this package (agent.py).
"""
from . import gen  # noqa: F401  (numpy-only; importable without a GPU)

__all__ = ["gen", "Swarm", "ElectResult", "AllocResult"]


def __getattr__(name):  # lazy: importing swarm_amd does not initialise HIP
    if name in ("Swarm", "ElectResult", "AllocResult"):
        from . import swarm
        return getattr(swarm, name)
    raise AttributeError(name)
