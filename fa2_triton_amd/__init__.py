"""fa2_triton_amd -- FlashAttention-2 forward/backward for AMD MI355X (gfx950).

Drop-in for the operator of remi-or/fa2_triton (/root/reference/src/__init__.py:1-4):
`flash_attn_func` / `FlashAttnFunc` keep the reference's signature and BSHD layout; the
Triton kernels are replaced by hand-written HIP kernels in libfa2_amd.so (C ABI:
include/fa2_amd.h).  The reference's pure-PyTorch oracle `flash_attn_reference` is test
infrastructure here and lives in `oracle/` (it is not part of the shipped operator).
"""
from .wrapper import FlashAttnFunc, flash_attn_func

__all__ = ["flash_attn_func", "FlashAttnFunc"]
