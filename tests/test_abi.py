"""CPU checks of the drop-in boundary: the C-ABI library loads, exports every symbol
declared in include/*.h, and refuses to run without a GPU (no CPU fallback)."""
import ctypes
import os
import re
import subprocess

import pytest

from dag_rider_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    syms = set()
    for h in ("dagrider_gpu.h", "dagrider_gen.h", "dagrider_shard.h", "dagrider_wire.h"):
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        syms |= set(re.findall(r"\b(dr_[a-z_]+)\s*\(", txt))
    return syms


def test_every_declared_symbol_exported():
    syms = declared_symbols()
    assert len(syms) >= 20
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (dr_\w+)", out))
    assert syms <= exported, syms - exported
    assert set(_lib.SIGNATURES) == syms  # the Python binding binds exactly the header
    assert "dr_profile_kernel" not in exported  # tuning hook: profiling build only


def test_tuning_hook_only_in_profiling_build():
    timing = os.path.join(ROOT, "dag_rider_amd", "libdagrider_gpu_timing.so")
    if not os.path.exists(timing):
        pytest.skip("profiling build not made")
    txt = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "dagrider_tuning.h")).read(), flags=re.S)
    tsyms = set(re.findall(r"\b(dr_[a-z_]+)\s*\(", txt))
    assert tsyms == set(_lib.TUNING_SIGNATURES)
    out = subprocess.run(["nm", "-D", "--defined-only", timing], capture_output=True, text=True, check=True).stdout
    assert tsyms <= set(re.findall(r" T (dr_\w+)", out))


def test_library_loads_and_binds():
    L = _lib.lib()
    assert L.dr_abi_version() == 2


def test_no_cpu_fallback():
    L = _lib.lib()
    h = ctypes.c_void_p()
    if os.environ.get("HIP_VISIBLE_DEVICES") is None:
        try:
            import torch

            if torch.cuda.is_available():
                pytest.skip("a GPU is visible")
        except Exception:
            pass
    rc = L.dr_create(4, 1, 8, 0, ctypes.byref(h))
    assert rc == _lib.DR_E_HIP
    assert b"no CPU fallback" in L.dr_last_error(None)
    assert L.dr_create(4, 1, 8, -1, ctypes.byref(h)) == _lib.DR_E_INVAL


def test_oracle_not_linked_by_product():
    out = subprocess.run(["ldd", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in out
    for root, _, files in os.walk(os.path.join(ROOT, "dag_rider_amd")):
        for f in files:
            if f.endswith((".py", ".hip", ".hpp", ".cpp", ".h")):
                txt = open(os.path.join(root, f)).read()
                assert "import oracle" not in txt and "from oracle" not in txt and "oracle.h" not in txt, f


def test_build_id_matches_tree():
    """dr_build_id() (the source hash the Makefile stamps) equals the hash of this tree's
    sources: the library under test was built from them, not left over from other ones."""
    p = _lib.provenance()
    assert len(p["build_id"]) == 16 and int(p["build_id"], 16) >= 0
    assert p["match"], p
