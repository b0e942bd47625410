"""The C-ABI library loads (no GPU needed) and exports exactly what
include/maxk_spgemm.h declares; host-only entry points work; the product
path fails loudly without the library."""
import ctypes
import os
import re
import subprocess

import pytest

from spgemm_new_amd import _lib

HEADER = _lib.HEADER


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(maxk_\w+)\s*\(", text)))


def test_header_declares_bound_functions():
    decl = declared_functions()
    assert decl == sorted(_lib.SIGNATURES), (decl, sorted(_lib.SIGNATURES))


def test_library_exports_every_declared_symbol():
    L = _lib.load()
    for name in declared_functions():
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (maxk_\w+)", out))
    assert set(declared_functions()) <= exported


def test_library_is_gfx950_code_object():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"sm_" not in blob.split(b"amdgcn-amd-amdhsa")[0][-64:]  # no CUDA target bundled


def test_host_entry_points():
    L = _lib.load()
    assert b"gfx950" in L.maxk_version()
    n = ctypes.c_int64(0)
    assert L.maxk_schedule_num_panels(232965, 114615892, 2048, 16, ctypes.byref(n)) == 0
    assert n.value == -(-(114615892 + 232965 * 16) // 2048)
    assert L.maxk_schedule_num_panels(10, 5, 0, 16, ctypes.byref(n)) == _lib.MAXK_E_ARG
    assert L.maxk_forward_workspace_bytes(10, 256) >= 10 * 256 * 4 + 40
    assert L.maxk_backward_workspace_bytes(_lib.MAXK_BWD_ATOMIC, 100, 32, 5) == 0
    assert L.maxk_backward_workspace_bytes(_lib.MAXK_BWD_STAGED, 100, 32, 5) >= 100 * 32 * 4


def test_argument_validation_without_gpu():
    """Invalid arguments are rejected before any launch (no device touched)."""
    L = _lib.load()
    # dim_origin > 256
    rc = L.maxk_spgemm_forward(1, 1, 1, 1, 1, 1, 1, 10, 300, 32, 1, 1, 1 << 20, None)
    assert rc == _lib.MAXK_E_DIM
    # k > dim
    rc = L.maxk_spmm_forward_warp4(1, 1, 1, 1, 1, 1, 10, 10, 64, 65, 1, None)
    assert rc == _lib.MAXK_E_DIM
    # workspace too small
    rc = L.maxk_spgemm_forward(1, 4, 1, 1, 1, 1, 1, 10, 256, 32, 1, 1, 16, None)
    assert rc == _lib.MAXK_E_WORKSPACE
    with pytest.raises(_lib.MaxKError):
        _lib.check(rc, "x")


def test_missing_library_fails_loudly(tmp_path, monkeypatch):
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(_lib.MaxKError):
        _lib.load()


def test_library_of_other_abi_is_refused(monkeypatch):
    """A library built from sources with another ABI revision (an entry point
    whose arguments changed) is refused at load, not bound with wrong argtypes
    (ADVICE r4)."""
    L = _lib.load()
    assert L.maxk_abi_version() == _lib.ABI_VERSION
    hdr = open(HEADER).read()
    assert re.search(r"#define MAXK_ABI_VERSION %d\b" % _lib.ABI_VERSION, hdr)
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "ABI_VERSION", _lib.ABI_VERSION + 1)
    with pytest.raises(_lib.MaxKError, match="other sources"):
        _lib.load()


def test_oracle_not_imported_by_product_package():
    import spgemm_new_amd
    pkg = os.path.dirname(spgemm_new_amd.__file__)
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in re.findall(r"^\s*(?:from|import)\s+(\w+)", src, re.M), f


_NULL_SWEEP = r"""
import ctypes, sys
sys.path.insert(0, sys.argv[1])
from spgemm_new_amd import _lib
L = ctypes.CDLL(_lib.LIB_PATH)
for name, (res, args) in _lib.SIGNATURES.items():
    if res is not ctypes.c_int or name in ("maxk_abi_version", "maxk_tile_record_words",
                                            "maxk_tile_part_planes"):
        continue
    f = getattr(L, name)
    f.restype, f.argtypes = res, args
    for n in (1, 1 << 20):
        vals = [n if a in (ctypes.c_int, ctypes.c_int64, ctypes.c_size_t) else
                0.0 if a is ctypes.c_float else None for a in args]
        print(name, n, f(*vals), flush=True)
"""


def test_null_buffers_rejected_before_any_launch():
    """Every buffer-taking entry point, called with null pointers and non-zero
    sizes (1 and 2^20 for every integer argument), returns a MAXK_E_* code from
    its argument checks -- no crash, and no HIP call (which would launch on null
    buffers on a GPU; here it would return a positive HIP error).  One child
    process for the sweep, so a crash is reported with the entry point it hit."""
    import ctypes

    from spgemm_new_amd import _lib
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    # no device visible to the child: an entry point that missed a check
    # then fails with a HIP error code instead of launching on null buffers
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="")
    p = subprocess.run([__import__("sys").executable, "-c", _NULL_SWEEP, root],
                       capture_output=True, text=True, timeout=300, env=env)
    lines = p.stdout.strip().splitlines()
    assert p.returncode == 0, (lines[-1:] if lines else "", p.stderr[-2000:])
    swept = [n for n, (res, _) in _lib.SIGNATURES.items() if res is ctypes.c_int and n not in
             ("maxk_abi_version", "maxk_tile_record_words", "maxk_tile_part_planes")]
    assert len(lines) == 2 * len(swept), (len(lines), len(swept))
    for ln in lines:
        name, n, rc = ln.split()
        assert int(rc) < 0, f"{name} with null buffers and sizes {n} returned {rc}"
