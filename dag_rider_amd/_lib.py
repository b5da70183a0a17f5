"""ctypes binding of libdagrider_gpu.so (C ABI: include/dagrider_gpu.h, include/dagrider_gen.h).

The library is built in-tree by ``make`` / ``__graft_entry__.build()``.  There is no
fallback: if it is missing, importing anything that needs it raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# DR_LIB_VARIANT=timing loads the profiling build (tools/sweep_timing.py only)
LIB_PATH = os.path.join(_HERE, "libdagrider_gpu_timing.so" if os.environ.get("DR_LIB_VARIANT") == "timing"
                        else "libdagrider_gpu.so")
# kernel experiments only (never set by tests, smoke or the bench): an alternative build
LIB_PATH = os.environ.get("DR_LIB_PATH_EXPT", LIB_PATH)

DR_OK, DR_E_INVAL, DR_E_CAPACITY, DR_E_HIP, DR_E_RCCL, DR_E_CONTRACT, DR_E_STATE = 0, -1, -2, -3, -4, -5, -6
DR_CHAIN_LITERAL, DR_CHAIN_PERSISTENT = 0, 1
DR_DELIVER_REF, DR_DELIVER_PAPER = 0, 1
DR_WEAK_LITERAL, DR_WEAK_PAPER = 0, 1
DR_OPT_MEMO = 1
DR_OPT_DEVICE_PLAN = 2
DR_OPT_PHASE_TIMING = 3
DR_OPT_BATCH_FORM = 4
DR_OPT_COMMIT_SPLIT = 5
DR_OPT_REPLAY_GRAPH = 6
DR_OPT_FUSE = 7
DR_OPT_CALL_OVERLAP = 8
DR_CREATE_SHARED_STREAM = 1
DR_BATCH_AUTO, DR_BATCH_WORKGROUP, DR_BATCH_WAVE = 0, 1, 2
DR_LEADER_CONST1, DR_LEADER_SEEDED, DR_LEADER_TABLE = 0, 1, 2
DR_SHARD_ID_BYTES = 128
DR_SHARD_OPT_PERSISTENT = 1
DR_SHARD_OPT_MEMO = 2
DR_SHARD_OPT_STEPPED = 3
DR_SHARD_OPT_PHASE_TIMING = 4
DR_SHARD_OPT_STEP_HINTS = 5

P = C.c_void_p
i32, u32, i64, u64, f32 = C.c_int32, C.c_uint32, C.c_int64, C.c_uint64, C.c_float


class GenParams(C.Structure):
    _fields_ = [("n", i32), ("last_round", i32), ("seed", u64), ("p_present", C.c_double),
                ("p_late", C.c_double), ("p_w", C.c_double), ("p_la", C.c_double),
                ("weak_depth", i32), ("nthreads", i32)]


class ReplayOut(C.Structure):
    _fields_ = [("commit", P), ("vcount", P), ("push_off", P), ("push_wave", P), ("push_cap", i64),
                ("pop_count", P), ("pop_digest", P), ("pop_edges", P), ("ids", P), ("ids_cap", i64),
                ("n_push", i64), ("n_ids", i64), ("commit_edges", u64), ("chain_edges", u64),
                ("deliver_edges", u64), ("ms_commit", f32), ("ms_chain", f32), ("ms_deliver", f32),
                ("ms_emit", f32), ("ms_summary", f32), ("canon_segments", i32), ("sweep_count", u64),
                ("sweep_partial", u64), ("sweep_row_bytes", u64), ("sweep_weak_scanned", u64), ("sweep_shortcut", u64)]


class ReplayView(C.Structure):
    _fields_ = [("commit", P), ("vcount", P), ("push_off", P), ("push_wave", P), ("pop_count", P),
                ("pop_digest", P), ("pop_edges", P), ("n_push", i64), ("commit_edges", u64), ("chain_edges", u64),
                ("deliver_edges", u64), ("ms_deliver", f32)]


class SliceCfg(C.Structure):
    _fields_ = [("round_offset", i32), ("seeded_top", i32), ("pos_base", u64), ("own_w0", i32), ("nprobe", i32),
                ("probe", i32 * 8)]


class SliceOut(C.Structure):
    _fields_ = [("C", u64 * 8), ("G", u64 * 8), ("E", u64 * 8), ("min_stop", i32), ("pad_", i32),
                ("own_chain_edges", u64)]


# symbol -> (restype, argtypes); every symbol declared in include/*.h
SIGNATURES = {
    "dr_abi_version": (C.c_int, []),
    "dr_build_id": (C.c_char_p, []),
    "dr_create": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(P)]),
    "dr_mirror_stats": (C.c_int, [P, C.c_void_p, C.c_int]),
    "dr_create_ex": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(P)]),
    "dr_destroy": (None, [P]),
    "dr_last_error": (C.c_char_p, [P]),
    "dr_num_rounds": (C.c_int, [P]),
    "dr_set_option": (C.c_int, [P, C.c_int, C.c_int]),
    "dr_set_leader_coin": (C.c_int, [P, C.c_int, C.c_uint64, C.c_int, P]),
    "dr_coin_leader": (C.c_int, [C.c_uint64, C.c_int, C.c_int]),
    "dr_wave_leader": (C.c_int, [P, C.c_int]),
    "dr_replay_graph_state": (C.c_int, [P]),
    "dr_append_rounds_lists": (C.c_int, [P, C.c_int, C.c_int, P, P, P, P, P, P]),
    "dr_append_rounds_packed": (C.c_int, [P, C.c_int, C.c_int, P, P, P, P, P]),
    "dr_append_vertices": (C.c_int, [P, C.c_int, P, P, P, P, P, P]),
    "dr_path_batch": (C.c_int, [P, C.c_int, P, P, C.c_int, P]),
    "dr_reach_sets": (C.c_int, [P, C.c_int, P, P, C.c_int, P, C.c_size_t, C.POINTER(C.c_size_t)]),
    "dr_wave_commit": (C.c_int, [P, C.c_int, C.c_int, P, P]),
    "dr_set_weak_edges": (C.c_int, [P, C.c_int, C.c_int, P, C.c_int, P, C.c_size_t, C.POINTER(C.c_size_t)]),
    "dr_buffer_admit": (C.c_int, [P, C.c_int, C.c_int, P, P, P, P]),
    "dr_wave_ready": (C.c_int, [P, C.c_int, C.c_int, P, P, P, C.c_int, C.POINTER(C.c_int)]),
    "dr_order_vertices": (C.c_int, [P, P, C.c_int, C.c_int, C.c_int, P, C.c_size_t,
                                    C.POINTER(C.c_size_t), P, P]),
    "dr_replay": (C.c_int, [P, C.c_int, C.c_int, C.c_int, C.POINTER(ReplayOut)]),
    "dr_replay_batch": (C.c_int, [C.POINTER(P), C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(ReplayOut)]),
    "dr_replay_batch_view": (C.c_int, [C.POINTER(P), C.c_int, C.c_int, C.c_int, C.c_int, i64,
                                       C.POINTER(ReplayView)]),
    "dr_last_kernel_ms": (C.c_int, [P, C.POINTER(f32)]),
    "dr_exception_stats": (C.c_int, [P, P]),
    "dr_last_batch_phases": (C.c_int, [P, C.POINTER(f32)]),
    "dr_last_batch_form": (C.c_int, [P]),
    "dr_last_append_phases": (C.c_int, [P, C.POINTER(f32)]),
    "dr_set_slice": (C.c_int, [P, C.POINTER(SliceCfg)]),
    "dr_last_replay_path": (C.c_int, [P]),
    "dr_slice_result": (C.c_int, [P, C.POINTER(SliceOut)]),
    # include/dagrider_shard.h
    "dr_shard_unique_id": (C.c_int, [P]),
    "dr_shard_create": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P, C.POINTER(P)]),
    "dr_shard_destroy": (None, [P]),
    "dr_shard_last_error": (C.c_char_p, [P]),
    "dr_shard_num_rounds": (C.c_int, [P]),
    "dr_shard_info": (C.c_int, [P, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int),
                                C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "dr_shard_append_rounds_packed": (C.c_int, [P, C.c_int, C.c_int, P, P, P, P, P]),
    "dr_shard_reach_sets": (C.c_int, [P, C.c_int, P, P, C.c_int, P, C.c_size_t, C.POINTER(C.c_size_t)]),
    "dr_shard_path_batch": (C.c_int, [P, C.c_int, P, P, C.c_int, P]),
    "dr_shard_stats": (C.c_int, [P, C.POINTER(f32), C.POINTER(u64), C.POINTER(u64)]),
    "dr_shard_host_syncs": (C.c_int, [P, C.POINTER(u64)]),
    "dr_shard_set_option": (C.c_int, [P, C.c_int, C.c_int]),
    "dr_shard_set_leader_coin": (C.c_int, [P, C.c_int, C.c_uint64, C.c_int, P]),
    "dr_shard_wave_commit": (C.c_int, [P, C.c_int, C.c_int, P, P]),
    "dr_shard_wave_ready": (C.c_int, [P, C.c_int, C.c_int, P, P, P, C.c_int, C.POINTER(C.c_int)]),
    "dr_shard_order_vertices": (C.c_int, [P, P, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_size_t), P, P]),
    "dr_shard_replay": (C.c_int, [P, C.c_int, C.c_int, C.c_int, C.POINTER(ReplayOut)]),
    # include/dagrider_wire.h
    "dr_wire_check": (C.c_int, [P, C.c_size_t, C.POINTER(i32), C.POINTER(i32)]),
    "dr_wire_append": (C.c_int, [P, P, C.c_size_t]),
    "dr_wire_block": (C.c_int, [P, C.c_size_t, i64, C.POINTER(P), C.POINTER(C.c_size_t)]),
    "dr_gen_create": (C.c_int, [C.POINTER(GenParams), C.POINTER(P)]),
    "dr_gen_free": (None, [P]),
    "dr_gen_info": (C.c_int, [P, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32), C.POINTER(u64),
                              C.POINTER(u64)]),
    "dr_gen_slot_off": (P, [P]),
    "dr_gen_slot_src": (P, [P]),
    "dr_gen_strong": (P, [P]),
    "dr_gen_weak_off": (P, [P]),
    "dr_gen_weak_tgt": (P, [P]),
}

# include/dagrider_tuning.h: exported by the profiling build only (DR_LIB_VARIANT=timing)
TUNING_SIGNATURES = {
    "dr_profile_kernel": (C.c_int, [P, C.c_int, C.c_int, C.c_int, C.POINTER(f32)]),
}

_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `make` (or __graft_entry__.build()); "
                               "there is no CPU fallback")
        L = C.CDLL(LIB_PATH)
        sigs = dict(SIGNATURES)
        if LIB_PATH.endswith("_timing.so"):
            sigs.update(TUNING_SIGNATURES)
        for name, (res, args) in sigs.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def source_hash(root: str | None = None) -> str:
    """The hash the Makefile stamps into dr_build_id(): sha256 (first 16 hex digits) of
    dag_rider_amd/csrc/*.{hip,hpp,cpp} and include/*.h, concatenated in byte order of
    their paths.  Equal to build_id() when the library was built from this tree."""
    import glob
    import hashlib

    root = root or os.path.dirname(_HERE)
    paths = []
    for pat in ("dag_rider_amd/csrc/*.hip", "dag_rider_amd/csrc/*.hpp", "dag_rider_amd/csrc/*.cpp", "include/*.h"):
        paths += glob.glob(pat, root_dir=root)
    h = hashlib.sha256()
    for p in sorted(paths):
        with open(os.path.join(root, p), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def build_id() -> str:
    """dr_build_id(): the source hash the library was built from."""
    return lib().dr_build_id().decode()


def provenance() -> dict:
    """The loaded library's build id next to this tree's source hash (a prebuilt library
    pushed to the GPU box must match the sources it runs beside)."""
    b, s = build_id(), source_hash()
    return {"build_id": b, "source_hash": s, "match": b == s, "lib": LIB_PATH}


class DrError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def ptr(a):
    """numpy array -> void* (None passes NULL)."""
    return None if a is None else a.ctypes.data_as(P)
