"""CPU checks of the C-ABI boundary (no GPU, no compute launches).

* libmrec.so loads and exports every function include/mrec.h declares, and the
  ctypes signature table (pytorchrec_amd/_mrec.py) covers exactly that set;
* host-only entry points (ABI version, workspace-size queries) answer;
* argument validation fails with MREC_EINVAL and a readable mrec_last_error()
  before anything touches a device — the error contract of SURVEY.md §8(b) B2.
"""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADERS = [os.path.join(ROOT, "include", h) for h in sorted(os.listdir(os.path.join(ROOT, "include")))
           if h.endswith(".h")]


def _declared():
    names = set()
    for h in HEADERS:
        txt = open(h).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[\w\s\*]+?\b(mrec_\w+)\s*\(", txt, flags=re.M):
            names.add(m.group(1))
    return names


@pytest.fixture(scope="module")
def lib():
    from pytorchrec_amd import _mrec
    return _mrec.lib()


def test_header_declares_functions():
    names = _declared()
    assert "mrec_abi_version" in names and "mrec_gemm" in names and len(names) >= 15


def test_every_declared_symbol_is_exported(lib):
    missing = [n for n in sorted(_declared()) if not hasattr(lib, n)]
    assert not missing, missing


def test_signature_table_matches_header():
    from pytorchrec_amd import _mrec
    assert set(_mrec.SIGNATURES) == _declared()


def test_abi_version(lib):
    from pytorchrec_amd import _mrec
    assert lib.mrec_abi_version() == _mrec.ABI_VERSION


def test_workspace_queries(lib):
    assert lib.mrec_emb_bwd_workspace_size(26, 4096) >= 26 * 4096 * 12
    assert lib.mrec_emb_bwd_workspace_size(0, 10) == 0
    assert lib.mrec_gemm_workspace_size(400, 429, 400, 1) == 0       # one K slab: no split
    assert lib.mrec_gemm_workspace_size(400, 429, 4096, 10) >= 10 * 400 * 430 * 4


def test_invalid_arguments_return_einval(lib):
    from pytorchrec_amd import _mrec
    # NULL operands
    st = lib.mrec_gemm(4, 4, 4, None, None, -1, 4, None, None, _mrec.BF16, 4, 1, None, 0, None)
    assert st == _mrec.EINVAL
    assert b"NULL" in lib.mrec_last_error()
    # misaligned bf16 operand rows (ld not a multiple of 8 elements)
    a = _mrec.Operand(64, _mrec.BF16, _mrec.LAYOUT_ROW, 7)
    b = _mrec.Operand(64, _mrec.BF16, _mrec.LAYOUT_ROW, 8)
    st = lib.mrec_gemm(4, 4, 4, ctypes.byref(a), ctypes.byref(b), -1, 4, None, 64, _mrec.BF16, 8,
                       1, None, 0, None)
    assert st == _mrec.EINVAL
    assert b"16-byte" in lib.mrec_last_error()
    # a bank whose row pitch is not a power of two in [16, 256] bytes
    rows = (ctypes.c_int64 * 1)(10)
    offs = (ctypes.c_int64 * 1)(0)
    bank = _mrec.TableBank(64, offs, rows, 1, 16, 24, 0, _mrec.BF16)
    ids = _mrec.Ids((ctypes.c_void_p * 1)(64), _mrec.I32, 1)
    st = lib.mrec_emb_gather_fwd(ctypes.byref(bank), ctypes.byref(ids), 4, 64, _mrec.BF16, 16,
                                 None, None, None)
    assert st == _mrec.EINVAL
    assert lib.mrec_last_error()
    # data-parallel SGD: too many jobs, NULL gradient
    jobs = (_mrec.SgdJob * 17)()
    assert lib.mrec_sgd_multi(17, jobs, None) == _mrec.EINVAL
    jobs[0] = _mrec.SgdJob(64, None, 4, 4, 4, 8, 0.1, None, 0, None, 0)
    assert lib.mrec_sgd_multi(1, jobs, None) == _mrec.EINVAL
    assert b"NULL" in lib.mrec_last_error()


def test_apply_refuses_a_workspace_no_plan_was_issued_into(lib):
    """ABI 28 layout rule (mrec.h, above mrec_emb_bwd_plan): every embedding-backward
    apply checks the layout its workspace's last plan recorded, on the host, before
    any launch -- here no plan was ever issued into that address, so each apply entry
    refuses with MREC_EINVAL (the GPU suite covers the padded-plan / plain-apply
    mismatch, test_plan_body_instantiations_match_standalone)."""
    from pytorchrec_amd import _mrec
    rows = (ctypes.c_int64 * 1)(100)
    offs = (ctypes.c_int64 * 1)(0)
    bank = _mrec.TableBank(64, offs, rows, 1, 16, 32, 1, _mrec.BF16)
    ws_addr, B = 1 << 20, 100
    wsb = lib.mrec_emb_bwd_workspace_size(1, B)
    st = lib.mrec_emb_bwd_apply(ctypes.byref(bank), B, ws_addr, wsb, None, _mrec.F32, 0, None,
                                None, None, _mrec.F32, 0, None, _mrec.BWD_SGD, 0.1, 0, None, None,
                                None)
    assert st == _mrec.EINVAL
    assert b"no embedding-backward plan" in lib.mrec_last_error()
    st = lib.mrec_emb_bwd_apply_wire(ctypes.byref(bank), B, ws_addr, wsb, 256, 36, _mrec.BF16, 512,
                                     8, 1, 1, _mrec.BWD_SGD, 0.1, 0, None, None, 0, None, None)
    assert st == _mrec.EINVAL
    assert b"mrec_emb_bwd_apply_wire" in lib.mrec_last_error()


def test_sgd_table_build_is_host_only_and_validates(lib):
    """mrec_sgd_table_build (ABI 28) fills a host table and its workgroup count, no
    device call: 32 x 32 tiles per job; bad jobs fail with MREC_EINVAL."""
    from pytorchrec_amd import _mrec
    nb = int(lib.mrec_sgd_table_bytes())
    assert nb > 16 * 64
    host = (ctypes.c_uint8 * nb)()
    blocks = ctypes.c_int32(-1)
    jobs = (_mrec.SgdJob * 2)(
        _mrec.SgdJob(64, 128, 400, 429, 429, 432, 0.1, None, 0, None, 0, _mrec.IMG_TOWER),
        _mrec.SgdJob(256, 512, 1, 400, 400, 400, 0.1, None, 0, None, 0, _mrec.IMG_ROW_TR))
    assert lib.mrec_sgd_table_build(2, jobs, ctypes.addressof(host), nb, ctypes.byref(blocks)) == _mrec.OK
    assert blocks.value == 13 * 14 + 1 * 13
    assert lib.mrec_sgd_table_build(2, jobs, ctypes.addressof(host), nb - 1,
                                    ctypes.byref(blocks)) == _mrec.EINVAL
    jobs[0].g = None
    assert lib.mrec_sgd_table_build(2, jobs, ctypes.addressof(host), nb, ctypes.byref(blocks)) == _mrec.EINVAL
    assert b"NULL" in lib.mrec_last_error()


def test_product_path_has_no_cpu_fallback_for_gpu_tensors():
    """The HIP ops raise MrecUnavailable (never fall back) when the library is gone."""
    from pytorchrec_amd import _mrec
    saved_lib, saved_path = _mrec._lib, _mrec.LIB_PATH
    try:
        _mrec._lib = None
        _mrec.LIB_PATH = os.path.join(ROOT, "does-not-exist", "libmrec.so")
        with pytest.raises(_mrec.MrecUnavailable):
            _mrec.lib()
    finally:
        _mrec._lib, _mrec.LIB_PATH = saved_lib, saved_path
