"""CPU: the drop-in boundary. libpfilter_hip.so loads and exports every entry point declared in
include/pfilter_hip.h (no compute calls — this container has no GPU)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pfilter_hip.h")
LIB = os.path.join(ROOT, "pfilter-noetic_amd", "libpfilter_hip.so")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pf_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = declared()
    assert len(names) >= 20
    for must in ("pf_fe_extract", "pf_odom_update", "pf_odom_init_map", "pf_odom_get_map", "pf_knn_query"):
        assert must in names


def test_library_exports_every_declared_symbol():
    if not os.path.exists(LIB):
        pytest.fail("libpfilter_hip.so is not built (run __graft_entry__.build())")
    L = ctypes.CDLL(LIB)
    missing = [n for n in declared() if not hasattr(L, n)]
    assert not missing, missing


def test_python_binding_lists_the_header():
    import pfilter_amd
    assert sorted(pfilter_amd.EXPORTS) == declared()


def test_header_compiles_as_c():
    """The boundary is plain C: no torch or C++ types in the signatures."""
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        with open(c, "w") as f:
            f.write('#include "pfilter_hip.h"\nint main(void){return 0;}\n')
        subprocess.check_call(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                               "-c", c, "-o", os.path.join(d, "t.o")])


def test_cpp_shim_compiles():
    """The header-only C++ drop-in (pfilter-noetic_amd/shim) compiles against PCL-shaped types."""
    import subprocess
    for drv in ("shim_driver.cpp", "shim_bpf_driver.cpp", "shim_cls_driver.cpp", "shim_map_driver.cpp",
                "shim_dcvc_driver.cpp"):   # ES + LaserProcessing, BPF, front end, global map, curvedVoxel
        subprocess.check_call(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Werror", "-I",
                               os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "shim", drv)])
