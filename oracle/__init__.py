"""CPU/torch oracle for the FlashAttention-2 path -- TEST INFRASTRUCTURE ONLY.

Nothing in the shipped package (`fa2_triton_amd/`) may import this package.  Only
`tests/`, `__graft_entry__.smoke()` and the `cpu_baseline` leg of `bench.py` use it,
and only as the checker / the timed CPU baseline, never as the product path.

Contents
--------
* `reference.attention_reference` -- restatement of the reference's O(S^2) oracle
  `flash_attn_reference` (/root/reference/src/reference_implementation.py:38-123) and of
  `construct_local_mask` (:8-35).  Pinned against golden vectors produced by the imported
  original (tests/golden/make_golden.py).
* `reference.lse2_reference` -- base-2 logsumexp per query row, the quantity the forward
  kernel stores (/root/reference/src/forward/kernel.py:119, compute_row_blocks.py:100-101).
* `philox` -- numpy Philox4x32-10 + uint->float conversion equal to Triton's `tl.rand`
  (triton/language/random.py of the installed Triton 3.6.0: philox_impl :13-43,
  randint4x :89-111, uint_to_uniform_float :127-144), as used by the reference dropout
  (/root/reference/src/forward/compute_row_blocks.py:76-79) and its test mask generator
  (/root/reference/tests/utils.py:169-207).  Pinned by a known-answer vector captured from
  the Triton interpreter (tests/golden/philox_kat.npz).
* `tolerance.check_fa_tolerance` -- the reference tests' acceptance rule
  (/root/reference/tests/utils.py:68-142).
"""
