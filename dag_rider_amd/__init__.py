"""dag_rider_amd -- MI355X-native causal-history reachability for DAG-Rider.

Drop-in for the hot path of xenowits/dag-rider (process/process.go: path,
waveReady, orderVertices) behind a C ABI (include/dagrider_gpu.h) implemented
by hand-written HIP kernels for gfx950 (csrc/).  Python here is orchestration:
ctypes handles (engine.py, shard.py), the DRW1 capture format (wire.py) and
workload generation (gen.py).  The reference-shaped Process mirror is C++
(host/process.hpp); the Go binding is go/dagridergpu.
"""
from .dag import PackedDag, Vertex, VertexID, flatten_lists, pack_lists  # noqa: F401

__all__ = ["PackedDag", "Vertex", "VertexID", "flatten_lists", "pack_lists"]
