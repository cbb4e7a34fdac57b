"""minpaxos_amd — MI355X-native batched-consensus engine for the MinPaxos hot path.

The product is libmpx.so (HIP kernels for gfx950 behind the C ABI of include/mpx.h); this
package is its Python host binding (ctypes), the synthetic workload generators and the group
sharding helpers used by bench.py and the tests.
"""
from . import records  # noqa: F401
from .records import *  # noqa: F401,F403

__all__ = ["records", "engine", "synth", "shard"]


def __getattr__(name):
    if name == "Engine":
        from .engine import Engine
        return Engine
    raise AttributeError(name)
