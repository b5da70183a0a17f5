"""dag_rider_amd -- MI355X-native causal-history reachability for DAG-Rider.

Drop-in for the hot path of xenowits/dag-rider (process/process.go: path,
waveReady, orderVertices) behind a C ABI (include/dagrider_gpu.h) implemented
by hand-written HIP kernels for gfx950 (csrc/).  Python here is orchestration:
ctypes handles (engine.py), the reference-shaped Process mirror (process.py),
workload generation (gen.py).
"""
from .dag import PackedDag, Vertex, VertexID, flatten_lists, pack_lists  # noqa: F401

__all__ = ["PackedDag", "Vertex", "VertexID", "flatten_lists", "pack_lists"]
