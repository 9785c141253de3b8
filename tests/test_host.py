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


@pytest.mark.parametrize("cname,pystruct", [("fa2_fwd_args", _lib.FwdArgs), ("fa2_bwd_args", _lib.BwdArgs)])
def test_ctypes_struct_matches_header(cname, pystruct):
    assert _header_struct_fields(cname) == [f[0] for f in pystruct._fields_]


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


def _visible_tiles(sq, sk, causal):
    """Brute-force count of the 32 x 32 (query, key) tiles dK/dV writes for one (batch, head):
    key tile kt of query tile t holds a visible pair iff 32 kt <= 32 t + 31 + (sk - sq)."""
    nqt, nkt = -(-sq // 32), -(-sk // 32)
    return sum(1 for t in range(nqt) for kt in range(nkt) if not causal or 32 * kt <= 32 * t + 31 + sk - sq)


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("b,hq,sq,sk,d", [(8, 32, 4096, 4096, 128), (2, 32, 8192, 8192, 128), (3, 4, 517, 203, 64),
                                           (1, 2, 33, 1, 256), (2, 2, 100, 100, 32), (2, 2, 100, 100, 72),
                                           (2, 2, 100, 100, 111), (1, 3, 517, 203, 128), (1, 3, 203, 517, 96),
                                           (1, 1, 1000, 37, 128), (1, 1, 37, 1000, 128), (1, 1, 1, 1, 128),
                                           (1, 1, 64, 95, 80), (1, 1, 95, 64, 80), (2, 2, 4000, 33, 128)])
def test_ds_workspace_bytes_matches_library(b, hq, sq, sk, d, causal):
    from fa2_triton_amd.backward import ds_workspace_bytes

    lib = _lib.load()
    a = _lib.BwdArgs()
    a.batch, a.heads_q, a.heads_kv, a.seqlen_q, a.seqlen_k, a.head_dim = b, hq, 1, sq, sk, d
    a.causal = int(causal)
    q, k = torch.empty(b, sq, hq, d, device="meta"), torch.empty(b, sk, 1, d, device="meta")
    got = ds_workspace_bytes(q, k, k, q, q, causal)
    assert lib.fa2_bwd_ds_workspace_bytes(ctypes.byref(a)) == got
    if d % 8 == 0 and 64 < d <= 128:
        assert got == b * hq * _visible_tiles(sq, sk, causal) * 2048
    else:
        assert got == 0


def test_ds_workspace_causal_is_half_the_grid():
    from fa2_triton_amd.backward import ds_workspace_bytes

    q = torch.empty(8, 4096, 32, 128, device="meta")
    assert ds_workspace_bytes(q, q, q, q, q, True) == 8 * 32 * (128 * 129 // 2) * 2048  # 4.33 GB
    assert ds_workspace_bytes(q, q, q, q, q, False) == 8 * 32 * 128 * 128 * 2048


def test_ds_workspace_needs_aligned_tensors():
    """The dS path runs only on the 16-byte vector layout; otherwise the size query says 0."""
    from fa2_triton_amd.backward import ds_workspace_bytes

    base = torch.empty(1, 64, 2, 128 + 1, dtype=torch.bfloat16)
    odd = base[..., 1:]  # data pointer 2 bytes past a 16-byte boundary, row stride 129
    ok = torch.empty(1, 64, 2, 128, dtype=torch.bfloat16)
    assert ds_workspace_bytes(ok, ok, ok, ok, ok, True) > 0
    assert ds_workspace_bytes(odd, ok, ok, ok, ok, True) == 0
    assert ds_workspace_bytes(ok, ok, ok, ok, odd, True) == 0
    kv = torch.empty(1, 64, 4, 128, dtype=torch.bfloat16)[:, :, :2]  # K and V row strides differ
    assert ds_workspace_bytes(ok, kv, ok, ok, ok, True) == 0


def test_ds_workspace_is_validated_without_a_gpu():
    lib = _lib.load()
    a = _lib.BwdArgs()
    a.batch, a.heads_q, a.heads_kv, a.seqlen_q, a.seqlen_k, a.head_dim = 1, 2, 2, 64, 64, 128
    a.dtype, a.dq_dtype, a.lse_row_stride = _lib.FA2_BF16, _lib.FA2_BF16, 128
    for name in ("q", "k", "v", "o", "dout", "lse", "delta", "dq", "dk", "dv"):
        setattr(a, name, 4096)  # never dereferenced: validation fails first
    a.ds_workspace, a.ds_workspace_bytes = 4096, 1024
    assert lib.fa2_bwd(ctypes.byref(a), None) == _lib.FA2_E_INVALID and b"ds_workspace_bytes" in lib.fa2_last_error()
    a.head_dim, a.ds_workspace_bytes = 111, 1 << 30
    assert lib.fa2_bwd(ctypes.byref(a), None) == _lib.FA2_E_INVALID and b"does not apply" in lib.fa2_last_error()


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
