"""CPU tests of the drop-in boundary: the C-ABI library loads, exports every symbol that
include/nmpc.h declares, and fails loudly (no CPU fallback) when no GPU is present."""
import ctypes
import os
import re

import numpy as np
import pytest

from drone_attitude_control_amd import _lib, build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "nmpc.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(nmpc_[a-z_0-9]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    build.build(verbose=False)
    return _lib.load()


def test_header_parsed():
    fns = header_functions()
    assert "nmpc_create" in fns and "nmpc_solve" in fns and len(fns) >= 20


def test_library_exports_every_header_symbol(lib):
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_binding_covers_header():
    assert sorted(_lib.SIGNATURES) == header_functions()


def test_desc_struct_matches_header_field_order():
    src = open(HEADER).read()
    body = src[src.index("typedef struct nmpc_ocp_desc {"):src.index("} nmpc_ocp_desc;")]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    names = []
    for decl in body.split(";")[:-1]:
        decl = decl.replace("typedef struct nmpc_ocp_desc {", "")
        decl = re.sub(r"\bconst\b|\bint\b|\bdouble\b|\bchar\b|\*", " ", decl)
        names += [n.strip() for n in decl.split(",") if n.strip()]
    assert names == [f[0] for f in _lib.OcpDesc._fields_]


def test_abi_version(lib):
    assert lib.nmpc_abi_version() == _lib.NMPC_ABI_VERSION


def test_no_gpu_fails_loudly(lib):
    if lib.nmpc_device_count() > 0:
        pytest.skip("a GPU is visible; covered by the gpu tests")
    from drone_attitude_control_amd.models import force_ocp
    from drone_attitude_control_amd import AcadosOcpSolver, NmpcError
    with pytest.raises(NmpcError, match="no HIP device"):
        AcadosOcpSolver(force_ocp(20))


def test_create_rejects_bad_descriptor(lib):
    h = ctypes.c_void_p()
    assert lib.nmpc_create(None, 1, 0, 0, ctypes.byref(h)) == -1
    d = _lib.OcpDesc()
    d.abi_version = 999
    assert lib.nmpc_create(ctypes.byref(d), 1, 0, 0, ctypes.byref(h)) == -1
    assert b"ABI" in lib.nmpc_last_error_global()


def test_sim_plant_arg_checks(lib):
    x = np.zeros(4)
    assert lib.nmpc_sim_plant(0, 1, 3, 0.02, 0.03, 9.81, _lib.dptr(x), _lib.dptr(x), _lib.dptr(x)) == -1


def test_affine_extraction_rejects_nonlinear():
    from drone_attitude_control_amd.acados import AcadosModel, affine_form
    m = AcadosModel()
    m.x, m.u = np.zeros(2), np.zeros(1)
    m.f_expl_expr = lambda x, u: np.array([x[1], np.sin(x[0]) + u[0]])
    with pytest.raises(NotImplementedError):
        affine_form(m)
    m.f_expl_expr = lambda x, u: np.array([x[1], -2.0 * x[0] + u[0] + 1.0])
    A, B, c = affine_form(m)
    assert np.allclose(A, [[0, 1], [-2, 0]]) and np.allclose(B, [[0], [1]]) and np.allclose(c, [0, 1])
