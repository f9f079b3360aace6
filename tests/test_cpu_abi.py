"""The C-ABI library loads on a host without a GPU, exports every entry point that
include/ivit.h declares, and validates arguments before touching the device (CPU only:
no compute call is made)."""
import ctypes
import os
import re

import pytest

import _lib
from conftest import REPO

LIB = os.path.join(REPO, "visiontransformer-intention-prediction_amd", "libivit_hip.so")
HEADER = os.path.join(REPO, "include", "ivit.h")

pytestmark = pytest.mark.skipif(not os.path.exists(LIB), reason="libivit_hip.so not built (run __graft_entry__.build())")


def _declared():
    txt = re.sub(r"/\*.*?\*/", " ", open(HEADER).read(), flags=re.S)
    txt = re.sub(r"//[^\n]*", " ", txt)
    return sorted(set(re.findall(r"\b(ivit_\w+)\s*\(", txt)))


def test_header_parse_covers_every_prototype():
    names = _declared()
    assert len(names) >= 40
    assert sorted(_lib.parse_header()) == names


def test_every_declared_symbol_is_exported():
    dll = ctypes.CDLL(LIB)
    missing = [n for n in _declared() if not hasattr(dll, n)]
    assert not missing, missing


def test_exports_are_c_linkage_only():
    # nm -D: every exported ivit_* symbol is a declared, unmangled C name
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = sorted({ln.split()[-1] for ln in out.splitlines() if " T ivit_" in ln})
    assert exported == _declared()


def test_version_and_error_strings():
    dll = _lib.lib.load()
    v = dll.ivit_version().decode()
    assert "gfx950" in v
    assert isinstance(dll.ivit_last_error(), bytes)


def test_argument_validation_without_device():
    dll = _lib.lib.load()
    # head dim != 64 is rejected before any HIP call (IVIT_ERR_ARG < 0), with a message
    rc = dll.ivit_attn_fwd(_lib.BF16, None, 1, 16, 1, 32, None, None, None, 0, None)
    assert rc < 0
    assert b"head dim" in dll.ivit_last_error()
    with pytest.raises(RuntimeError, match="ivit_attn_fwd failed"):
        _lib.lib.ivit_attn_fwd(_lib.BF16, None, 1, 16, 1, 32, None, None, None, 0, None)


def test_workspace_queries_are_pure_host():
    dll = _lib.lib.load()
    B, N, H = 8, 4501, 6
    npad = (N + 63) // 64 * 64  # lse2 + delta rows, padded to the 64-row tile, + the prescaled Q copy
    assert dll.ivit_attn_workspace(_lib.BF16, B, N, H, 64, 1) == 2 * B * H * npad * 4 + B * N * H * 64 * 2
    assert dll.ivit_attn_workspace(_lib.BF16, B, N, H, 64, 0) == 0
    assert dll.ivit_nms_workspace(22500) > 0
    assert dll.ivit_eval_post_workspace(32, 22500) >= 32 * 22500 * 352 * 8  # the padded suppression masks
    assert dll.ivit_eval_post_workspace(0, 22500) == 64
    # BatchNorm partials: 32-row blocks, doubled past 65 535 blocks (the grid's y dimension)
    assert dll.ivit_bn_workspace(36000, 512) == (1125 * 2 + 2) * 512 * 4
    m = 8 * 400 * 720
    assert dll.ivit_bn_workspace(m, 64) == (-(-m // 64) * 2 + 2) * 64 * 4


def test_ptr_refuses_host_tensors():
    import torch
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _lib.ptr(torch.zeros(4))
