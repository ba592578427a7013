"""The C-ABI library loads and exports every entry point include/emqx_gpumatch.h declares.
CPU only: no compute call is made (there is no GPU here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "emqx_gpumatch.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(emqxgm_[a-z_]+)\s*\(", src)))


def test_header_declares_expected_api():
    names = _declared()
    for must in ("emqxgm_create", "emqxgm_destroy", "emqxgm_trie_insert", "emqxgm_trie_delete",
                 "emqxgm_commit", "emqxgm_match_batch", "emqxgm_match_device",
                 "emqxgm_filter_bytes", "emqxgm_trie_empty", "emqxgm_route_ref"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from emqx_amd import build
    so = build.build_engine()
    lib = ctypes.CDLL(so)
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing
    lib.emqxgm_abi_version.restype = ctypes.c_int
    from emqx_amd.engine import ABI_VERSION
    assert lib.emqxgm_abi_version() == ABI_VERSION


def test_python_binding_covers_header():
    from emqx_amd import engine
    assert sorted(engine.SYMBOLS) == _declared()


def test_kernels_are_gfx950_code_objects():
    """The shipped .so carries gfx950 device code (hand-written HIP, no other targets)."""
    from emqx_amd import build
    so = build.build_engine()
    data = open(so, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    for other in (b"amdgcn-amd-amdhsa--gfx90a", b"amdgcn-amd-amdhsa--gfx942"):
        assert other not in data  # no other AMD targets bundled


def test_no_cpu_fallback_when_library_missing(tmp_path):
    from emqx_amd import engine
    with pytest.raises(ImportError):
        engine.load_library(str(tmp_path / "absent.so"))


def test_engine_refuses_without_device():
    """No GPU in this container: creating an engine must fail loudly, not fall back."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from emqx_amd import Engine, EngineError
    with pytest.raises(EngineError):
        Engine(device=0)
