"""The C-ABI library builds, loads and exports every symbol include/mmsbm.h and
include/mmsbm_pairs.h declare.
No compute calls: this runs on the CPU-only build container."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(REPO, "include", h) for h in ("mmsbm.h", "mmsbm_pairs.h")]


def declared_symbols():
    text = "".join(open(h).read() for h in HEADERS)
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(mmsbm_\w+)\s*\(", text, re.M)))


@pytest.fixture(scope="module")
def lib():
    from trigenicinteractionpredictor_amd import build, _lib
    build.build(verbose=False)
    return _lib.load()


def test_header_declares_the_abi():
    syms = declared_symbols()
    for need in ("mmsbm_create", "mmsbm_set_links", "mmsbm_iterate", "mmsbm_loglik", "mmsbm_predict",
                 "mmsbm_pairs_accumulate", "mmsbm_pairs_qstep", "mmsbm_pairs_loglik"):
        assert need in syms


def test_library_exports_every_declared_symbol(lib):
    for name in declared_symbols():
        assert hasattr(lib, name), name


def test_python_binding_covers_the_header():
    from trigenicinteractionpredictor_amd import _lib
    assert sorted(_lib.SIGNATURES) == declared_symbols()


def test_constants_and_error_string(lib):
    from trigenicinteractionpredictor_amd import _lib
    assert lib.mmsbm_chunk() == 4
    assert lib.mmsbm_version() >= 2
    # argument validation happens before any device call
    assert lib.mmsbm_create(0, None) == _lib.MMSBM_ERR_INVALID
    assert b"null" in lib.mmsbm_last_error()
    assert lib.mmsbm_set_shape(None, 10, 2, 1, 10, 1e-10) == _lib.MMSBM_ERR_INVALID
    # the pair ABI reports through the same error channel
    assert lib.mmsbm_pairs_create(0, None) == _lib.MMSBM_ERR_INVALID
    assert b"null" in lib.mmsbm_last_error()
    assert lib.mmsbm_pairs_set_shape(None, 10, 2, 1, 10, 1e-10) == _lib.MMSBM_ERR_INVALID


def test_library_is_gfx950_code_object():
    from trigenicinteractionpredictor_amd.build import LIB
    data = open(LIB, "rb").read()
    assert b"gfx950" in data


def test_no_cpu_fallback_in_product_path():
    """The product package never imports the oracle."""
    pkg = os.path.join(REPO, "trigenicinteractionpredictor_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(root, f)).read()
                assert "oracle" not in re.sub(r"#.*", "", src).replace('"""', ""), f


def test_ingest_library_exports_its_header():
    """include/mmsbm_io.h (host fold reader) is exported by libmmsbm_io.so."""
    from trigenicinteractionpredictor_amd import build
    text = open(os.path.join(REPO, "include", "mmsbm_io.h")).read()
    syms = sorted(set(re.findall(r"^\s*(?:int|void)\s*(mmsbm_\w+)\s*\(", text, re.M)))
    assert syms == ["mmsbm_fold_export", "mmsbm_fold_free", "mmsbm_fold_parse", "mmsbm_fold_sizes"]
    lib = ctypes.CDLL(build.build_io(verbose=False))
    for name in syms:
        assert hasattr(lib, name), name
