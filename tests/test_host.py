"""CPU tests: the C-ABI library loads and exports every symbol of include/fa2_amd.h, the ctypes
structs match the header layout, and the host-side helpers keep the reference's contract
(/root/reference/src/utils.py:57-109, src/forward/caller.py:27-42).  No kernel is launched.
"""
import ctypes
import os
import re

import pytest
import torch

from fa2_triton_amd import _lib
from fa2_triton_amd.utils import encode_dtype, handle_dropout, infer_bias_strides

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = open(os.path.join(ROOT, "include", "fa2_amd.h")).read()


def test_library_exports_every_header_symbol():
    declared = set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(fa2_\w+)\s*\(", HEADER, flags=re.M))
    assert declared == set(_lib.EXPORTED_SYMBOLS)
    lib = _lib.load()
    for sym in declared:
        assert hasattr(lib, sym), sym
    assert lib.fa2_version() == _lib.ABI_VERSION == int(re.search(r"FA2_ABI_VERSION (\d+)", HEADER).group(1))


def _header_struct_fields(name):
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), HEADER, flags=re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    fields = []
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        names = decl.split(None, 1)[1] if not decl.startswith("const") else decl.split(None, 2)[2]
        for n in names.split(","):
            n = n.strip().lstrip("*").strip()
            fields.append(re.sub(r"\[.*\]", "", n))
    return fields


@pytest.mark.parametrize("cname,pystruct", [("fa2_fwd_args", _lib.FwdArgs), ("fa2_bwd_args", _lib.BwdArgs),
                                           ("fa2_policy", _lib.Policy)])
def test_ctypes_struct_matches_header(cname, pystruct):
    assert _header_struct_fields(cname) == [f[0] for f in pystruct._fields_]


def test_policy_is_per_call_and_validated():
    """ABI 9: the kernel-path policy travels with each call (fa2_fwd_ex / fa2_bwd_stages_ex); the
    library keeps no mutable state between calls (no fa2_set_path_policy).  Bad policies are
    rejected before any launch."""
    lib = _lib.load()
    assert not hasattr(lib, "fa2_set_path_policy")
    a, b = _lib.FwdArgs(), _lib.BwdArgs()
    assert lib.fa2_fwd_ex(ctypes.byref(a), ctypes.byref(_lib.Policy(8, 0)), None) == _lib.FA2_E_INVALID
    assert b"path bits" in lib.fa2_last_error()
    assert lib.fa2_bwd_stages_ex(ctypes.byref(b), 6, ctypes.byref(_lib.Policy(0, -1)), None) == _lib.FA2_E_INVALID
    assert b"grid_cap" in lib.fa2_last_error()
    with pytest.raises(ValueError):
        _lib.set_path_policy(8, 0)
    _lib.set_path_policy(_lib.PATH_FWD_HP, 2)
    try:
        assert (_lib._policy.disable, _lib._policy.grid_cap) == (_lib.PATH_FWD_HP, 2)
    finally:
        _lib.set_path_policy(0, 0)


def test_invalid_arguments_are_rejected_without_a_gpu():
    lib = _lib.load()
    a = _lib.FwdArgs()
    a.batch, a.heads_q, a.heads_kv, a.seqlen_q, a.seqlen_k, a.head_dim = 1, 3, 2, 16, 16, 64
    a.dtype, a.lse_row_stride = _lib.FA2_BF16, 128
    rc = lib.fa2_fwd(ctypes.byref(a), None)
    assert rc == _lib.FA2_E_INVALID and b"divisible" in lib.fa2_last_error()
    a.heads_kv, a.head_dim = 1, 300
    assert lib.fa2_fwd(ctypes.byref(a), None) == _lib.FA2_E_UNSUPPORTED
    a.head_dim, a.dtype = 64, _lib.FA2_F32
    assert lib.fa2_fwd(ctypes.byref(a), None) == _lib.FA2_E_INVALID
    b = _lib.BwdArgs()
    b.batch, b.heads_q, b.heads_kv, b.seqlen_q, b.seqlen_k, b.head_dim = 1, 2, 2, 16, 16, 64
    b.dtype, b.dq_dtype, b.lse_row_stride, b.dropout_p = _lib.FA2_F16, _lib.FA2_F16, 128, 1.5
    assert lib.fa2_bwd(ctypes.byref(b), None) == _lib.FA2_E_INVALID
    b.dropout_p, b.head_dim = 0.1, 300
    assert lib.fa2_bwd(ctypes.byref(b), None) == _lib.FA2_E_UNSUPPORTED
    with pytest.raises(NotImplementedError):
        _lib.check(_lib.FA2_E_UNSUPPORTED)


def test_bias_gradient_stage_is_validated_without_a_gpu():
    """Stage bit 3 (the bias gradient) needs a dbias buffer, and a dbias buffer needs a bias."""
    lib = _lib.load()
    a = _lib.BwdArgs()
    a.batch, a.heads_q, a.heads_kv, a.seqlen_q, a.seqlen_k, a.head_dim = 1, 2, 2, 64, 64, 128
    a.dtype, a.dq_dtype, a.lse_row_stride = _lib.FA2_BF16, _lib.FA2_BF16, 128
    for name in ("q", "k", "v", "o", "dout", "lse", "delta", "dq", "dk", "dv"):
        setattr(a, name, 4096)  # never dereferenced: validation fails first
    assert lib.fa2_bwd_stages(ctypes.byref(a), 8, None) == _lib.FA2_E_INVALID and b"dbias" in lib.fa2_last_error()
    a.dbias = 4096
    assert lib.fa2_bwd(ctypes.byref(a), None) == _lib.FA2_E_INVALID and b"without a bias" in lib.fa2_last_error()
    assert lib.fa2_bwd_stages(ctypes.byref(a), 16, None) == _lib.FA2_E_INVALID


def test_infer_bias_strides():
    bias = torch.zeros(1, 1, 5, 7)
    assert infer_bias_strides(bias, 4, 9, 5, 7) == (0, 0, 7)
    bias = torch.zeros(4, 9, 5, 7)
    assert infer_bias_strides(bias, 4, 9, 5, 7) == (9 * 35, 35, 7)  # per-head bias accepted
    with pytest.raises(ValueError):
        infer_bias_strides(torch.zeros(3, 1, 5, 7), 4, 9, 5, 7)
    with pytest.raises(ValueError):
        infer_bias_strides(torch.zeros(1, 2, 5, 7), 4, 9, 5, 7)
    assert infer_bias_strides(None, 4, 9, 5, 7) == (0, 0, 0)


def test_handle_dropout_and_dtype_codes():
    assert handle_dropout(0.0, None, True) == 0
    assert handle_dropout(0.1, 1234, True) == 1234
    assert 0 <= handle_dropout(0.1, None, True) < 2**32
    assert handle_dropout(0.1, 77, False) == 77  # backward regenerates the forward's mask
    with pytest.raises(ValueError):
        handle_dropout(0.1, None, False)
    with pytest.raises(AssertionError):
        handle_dropout(1.0, None, True)
    assert encode_dtype(torch.zeros(1, dtype=torch.float16)) == 16
    assert encode_dtype(torch.zeros(1, dtype=torch.bfloat16)) == 17
    assert encode_dtype(torch.zeros(1, dtype=torch.float32)) == 32
