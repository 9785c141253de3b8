"""ctypes binding of libfa2_amd.so (the C ABI declared in include/fa2_amd.h).

This is the reference-side binding a host needs for the HIP kernels: plain pointers, int64
strides and scalars, no torch types cross the boundary.  torch is imported first so that the
HIP runtime torch already loaded (SONAME libamdhip64.so.7) is the one the library binds to;
streams are passed as raw hipStream_t handles from torch.cuda.current_stream().cuda_stream.

There is deliberately no fallback: if the library is missing or fails to load, every op
raises.  The Python layer never computes attention itself.
"""
import ctypes
import os
import threading

import torch  # noqa: F401  (must be loaded before the library: shared HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FA2_AMD_LIB", os.path.join(_HERE, "libfa2_amd.so"))

FA2_F16, FA2_BF16, FA2_F32 = 16, 17, 32
FA2_OK, FA2_E_INVALID, FA2_E_UNSUPPORTED, FA2_E_HIP = 0, -1, -2, -3

_i64x3 = ctypes.c_int64 * 3


class FwdArgs(ctypes.Structure):
    """Mirror of fa2_fwd_args (include/fa2_amd.h)."""

    _fields_ = [
        ("q", ctypes.c_void_p),
        ("k", ctypes.c_void_p),
        ("v", ctypes.c_void_p),
        ("o", ctypes.c_void_p),
        ("lse", ctypes.c_void_p),
        ("bias", ctypes.c_void_p),
        ("cu_seqlens", ctypes.c_void_p),
        ("q_stride", _i64x3),
        ("k_stride", _i64x3),
        ("v_stride", _i64x3),
        ("o_stride", _i64x3),
        ("bias_stride", _i64x3),
        ("batch", ctypes.c_int32),
        ("heads_q", ctypes.c_int32),
        ("heads_kv", ctypes.c_int32),
        ("seqlen_q", ctypes.c_int32),
        ("seqlen_k", ctypes.c_int32),
        ("head_dim", ctypes.c_int32),
        ("lse_row_stride", ctypes.c_int32),
        ("causal", ctypes.c_int32),
        ("dtype", ctypes.c_int32),
        ("bias_dtype", ctypes.c_int32),
        ("softmax_scale", ctypes.c_float),
        ("dropout_p", ctypes.c_float),
        ("dropout_seed", ctypes.c_uint64),
        ("dropout_mask", ctypes.c_void_p),
    ]


class BwdArgs(ctypes.Structure):
    """Mirror of fa2_bwd_args (include/fa2_amd.h)."""

    _fields_ = [
        ("q", ctypes.c_void_p),
        ("k", ctypes.c_void_p),
        ("v", ctypes.c_void_p),
        ("o", ctypes.c_void_p),
        ("dout", ctypes.c_void_p),
        ("lse", ctypes.c_void_p),
        ("delta", ctypes.c_void_p),
        ("dq", ctypes.c_void_p),
        ("dk", ctypes.c_void_p),
        ("dv", ctypes.c_void_p),
        ("bias", ctypes.c_void_p),
        ("cu_seqlens", ctypes.c_void_p),
        ("q_stride", _i64x3),
        ("k_stride", _i64x3),
        ("v_stride", _i64x3),
        ("o_stride", _i64x3),
        ("do_stride", _i64x3),
        ("dq_stride", _i64x3),
        ("dk_stride", _i64x3),
        ("dv_stride", _i64x3),
        ("bias_stride", _i64x3),
        ("batch", ctypes.c_int32),
        ("heads_q", ctypes.c_int32),
        ("heads_kv", ctypes.c_int32),
        ("seqlen_q", ctypes.c_int32),
        ("seqlen_k", ctypes.c_int32),
        ("head_dim", ctypes.c_int32),
        ("lse_row_stride", ctypes.c_int32),
        ("causal", ctypes.c_int32),
        ("dtype", ctypes.c_int32),
        ("bias_dtype", ctypes.c_int32),
        ("dq_dtype", ctypes.c_int32),
        ("softmax_scale", ctypes.c_float),
        ("dropout_p", ctypes.c_float),
        ("dropout_seed", ctypes.c_uint64),
        ("dbias", ctypes.c_void_p),
        ("dbias_stride", _i64x3),
        ("dkv_workspace", ctypes.c_void_p),
        ("dkv_workspace_bytes", ctypes.c_int64),
        ("dropout_mask", ctypes.c_void_p),
    ]


class Policy(ctypes.Structure):
    """Mirror of fa2_policy (include/fa2_amd.h, ABI 9): the kernel-path policy of one call."""

    _fields_ = [("disable", ctypes.c_uint32), ("grid_cap", ctypes.c_int32)]


ABI_VERSION = 9  # FA2_ABI_VERSION in include/fa2_amd.h

EXPORTED_SYMBOLS = ("fa2_fwd", "fa2_fwd_ex", "fa2_bwd", "fa2_bwd_stages", "fa2_bwd_stages_ex",
                    "fa2_bwd_dkv_workspace_bytes", "fa2_dropout_mask_bytes", "fa2_cu_seqlens_from_mask",
                    "fa2_last_error", "fa2_version")
# fa2_path bits (fa2_policy.disable)
PATH_FWD_HP, PATH_DQ_HP, PATH_DKDV_HP = 1, 2, 4

_lock = threading.Lock()
_lib = None


def bind(lib: ctypes.CDLL) -> ctypes.CDLL:
    """Declare the argument and result types of every exported function on `lib`."""
    lib.fa2_fwd.argtypes = [ctypes.POINTER(FwdArgs), ctypes.c_void_p]
    lib.fa2_fwd.restype = ctypes.c_int
    lib.fa2_bwd.argtypes = [ctypes.POINTER(BwdArgs), ctypes.c_void_p]
    lib.fa2_bwd.restype = ctypes.c_int
    lib.fa2_bwd_stages.argtypes = [ctypes.POINTER(BwdArgs), ctypes.c_int, ctypes.c_void_p]
    lib.fa2_bwd_stages.restype = ctypes.c_int
    lib.fa2_bwd_dkv_workspace_bytes.argtypes = [ctypes.POINTER(BwdArgs)]
    lib.fa2_bwd_dkv_workspace_bytes.restype = ctypes.c_int64
    lib.fa2_cu_seqlens_from_mask.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                             ctypes.c_void_p, ctypes.c_void_p]
    lib.fa2_cu_seqlens_from_mask.restype = ctypes.c_int
    lib.fa2_last_error.argtypes = []
    lib.fa2_last_error.restype = ctypes.c_char_p
    lib.fa2_dropout_mask_bytes.argtypes = [ctypes.c_int32] * 4
    lib.fa2_dropout_mask_bytes.restype = ctypes.c_int64
    lib.fa2_fwd_ex.argtypes = [ctypes.POINTER(FwdArgs), ctypes.POINTER(Policy), ctypes.c_void_p]
    lib.fa2_fwd_ex.restype = ctypes.c_int
    lib.fa2_bwd_stages_ex.argtypes = [ctypes.POINTER(BwdArgs), ctypes.c_int, ctypes.POINTER(Policy), ctypes.c_void_p]
    lib.fa2_bwd_stages_ex.restype = ctypes.c_int
    lib.fa2_version.argtypes = []
    lib.fa2_version.restype = ctypes.c_int
    return lib


def load() -> ctypes.CDLL:
    """Load (once) and return the library; raises if it is missing or of another ABI."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"fa2_triton_amd: HIP library not found at {LIB_PATH}; build it with "
                "`python -m fa2_triton_amd.build` (hipcc --offload-arch=gfx950)"
            )
        lib = bind(ctypes.CDLL(LIB_PATH))
        version = lib.fa2_version()
        if version != ABI_VERSION:
            raise RuntimeError(f"fa2_triton_amd: library ABI version {version}, expected {ABI_VERSION}")
        _lib = lib
    return _lib


def check(rc: int) -> None:
    """Raise for a non-zero fa2_* status, with the library's message."""
    if rc == FA2_OK:
        return
    msg = load().fa2_last_error().decode(errors="replace")
    if rc == FA2_E_UNSUPPORTED:
        raise NotImplementedError(msg)
    if rc == FA2_E_INVALID:
        raise ValueError(msg)
    raise RuntimeError(f"fa2_triton_amd: {msg} (status {rc})")


# The kernel-path policy the host layer passes with each call (fa2_fwd_ex / fa2_bwd_stages_ex):
# a test / A/B hook of this Python layer, (0, 0) = the defaults.  The library itself keeps no
# state between calls (ABI 9); a module variable rather than a thread-local one so that it also
# reaches the backward, which autograd runs on its own device thread.
_policy = Policy(0, 0)


def set_path_policy(disable: int = 0, grid_cap: int = 0) -> None:
    """Turn the hand-placed paths named by `disable` (PATH_* bits) off and cap the persistent
    kernels' grid (0: one workgroup per CU) for the following calls of this process.  (0, 0)
    restores the defaults."""
    if disable & ~(PATH_FWD_HP | PATH_DQ_HP | PATH_DKDV_HP):
        raise ValueError(f"unknown path bits {disable:#x}")
    if grid_cap < 0:
        raise ValueError(f"grid_cap {grid_cap} < 0")
    _policy.disable, _policy.grid_cap = disable, grid_cap


def fwd(args: FwdArgs, stream) -> int:
    """fa2_fwd_ex with the host layer's policy (NULL when it is the default)."""
    pol = ctypes.byref(_policy) if (_policy.disable or _policy.grid_cap) else None
    return load().fa2_fwd_ex(ctypes.byref(args), pol, stream)


def bwd_stages(args: BwdArgs, stages: int, stream) -> int:
    """fa2_bwd_stages_ex with the host layer's policy (NULL when it is the default)."""
    pol = ctypes.byref(_policy) if (_policy.disable or _policy.grid_cap) else None
    return load().fa2_bwd_stages_ex(ctypes.byref(args), stages, pol, stream)
