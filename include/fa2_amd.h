/*
 * fa2_amd.h -- C ABI of the MI355X (gfx950) FlashAttention-2 forward/backward kernels.
 *
 * This library replaces the three Triton launches of the reference
 * (remi-or/fa2_triton @ 2024-10-08):
 *   fa2_fwd  <- _fwd_kernel[grid](...)      /root/reference/src/forward/caller.py:83-116
 *   fa2_bwd  <- _compute_delta[grid](...)   /root/reference/src/backward/caller.py:95-114
 *             + _bwd_kernel[grid](...)      /root/reference/src/backward/caller.py:122-160
 *             + the host GQA dK/dV sum      /root/reference/src/backward/caller.py:162-165
 * and the host varlen pack/unpack loops (/root/reference/src/utils.py:8-31) through
 *   fa2_cu_seqlens_from_mask  (device-side cumulative lengths of a right-padded mask).
 *
 * Conventions
 *  - All tensors live in device memory and are addressed by element strides; the last
 *    (head_dim) stride must be 1 (/root/reference/src/wrapper.py:41-43).  Q/K/V/O/dO/dQ/dK/dV
 *    use the reference's [batch, seqlen, heads, head_dim] (BSHD) indexing, but any stride
 *    order works (e.g. BHSD views), so no copies are needed.
 *  - lse / delta are [batch, heads_q, lse_row_stride] fp32, lse_row_stride >= seqlen_q
 *    (the reference rounds it up to a multiple of 128, src/forward/caller.py:73-74).
 *    lse holds the base-2 log-sum-exp: LSE2 = ln(sum_j exp(s_ij)) * log2(e); rows with no
 *    visible key (causal seqlen_q > seqlen_k, padded rows) hold -inf.
 *  - Nothing is allocated inside the library; every buffer is caller-owned.
 *  - Launches are asynchronous on `stream` (a hipStream_t; NULL = default stream).
 *  - Return 0 on success or a negative FA2_E* code; fa2_last_error() then describes it
 *    (thread-local string).  The Python host layer raises RuntimeError with that text.
 */
#ifndef FA2_AMD_H
#define FA2_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FA2_ABI_VERSION 9

/* dtype codes: same numbers as the reference's encode_dtype (src/utils.py:102-109). */
enum fa2_dtype { FA2_F16 = 16, FA2_BF16 = 17, FA2_F32 = 32 };

enum fa2_status {
  FA2_OK = 0,
  FA2_E_INVALID = -1,     /* bad shape / stride / pointer */
  FA2_E_UNSUPPORTED = -2, /* valid but not implemented (e.g. head_dim > 256) */
  FA2_E_HIP = -3          /* a HIP runtime call failed */
};

/* Forward: O = softmax(scale * Q K^T + bias, masks) V  (dropout optional), plus LSE2.
 * Mirrors the argument list of _fwd_kernel (/root/reference/src/forward/kernel.py:61-96). */
typedef struct fa2_fwd_args {
  const void* q;      /* [B, Sq, Hq, D] */
  const void* k;      /* [B, Sk, Hkv, D] */
  const void* v;      /* [B, Sk, Hkv, D] */
  void* o;            /* [B, Sq, Hq, D], same dtype as q; every element is written */
  float* lse;         /* [B, Hq, lse_row_stride]; rows [0, Sq) written */
  const void* bias;   /* optional additive bias [1|B, 1|Hq, Sq, Sk] (strides below), or NULL */
  const int32_t* cu_seqlens; /* optional [B+1] cumulative valid lengths (varlen, Sq == Sk), or NULL */
  int64_t q_stride[3];    /* batch, seq, head strides (elements) */
  int64_t k_stride[3];
  int64_t v_stride[3];
  int64_t o_stride[3];
  int64_t bias_stride[3]; /* batch, head, row strides; 0 = broadcast */
  int32_t batch, heads_q, heads_kv, seqlen_q, seqlen_k, head_dim;
  int32_t lse_row_stride;
  int32_t causal;         /* bottom-right aligned causal mask */
  int32_t dtype;          /* FA2_F16 or FA2_BF16 (q, k, v, o) */
  int32_t bias_dtype;     /* FA2_F16, FA2_BF16 or FA2_F32 when bias != NULL */
  float softmax_scale;
  float dropout_p;        /* 0 <= p < 1 */
  uint64_t dropout_seed;  /* Philox4x32-10 key, identical to Triton's tl.rand */
  /* optional dropout keep mask out (ABI 6): when non-NULL and dropout_p > 0, the forward also
   * writes the keep bits it drew (keep = tl.rand > p) into this buffer of
   * fa2_dropout_mask_bytes(batch, heads_q, seqlen_q, seqlen_k) bytes (ABI 8: the tiles below plus
   * one 128-byte tile of slack the backward may read past the last one), so that the backward reads
   * them instead of regenerating Philox (fa2_bwd_args.dropout_mask).  Layout: 32 x 32 bit tiles,
   * word[((b * Hq + h) * ceil(Sq / 32) + i / 32) * ceil(Sk / 32) + j / 32][i % 32], bit j % 32 =
   * keep(b, h, i, j).  Only the tiles the (causal) mask leaves visible are written.  The buffer is
   * also the forward's input: with it the forward first draws every visible word (an all-VALU
   * Philox launch) and then reads them (the D = 128 hand-placed forward runs with dropout only
   * then); O equals the no-buffer forward's within rounding, not bitwise. */
  uint32_t* dropout_mask;
} fa2_fwd_args;

/* Backward: dQ, dK, dV of the forward above.  dK/dV are written with heads_kv heads: the GQA
 * group sum is done in fp32 inside the kernel.  dropout_p > 0 is supported (the reference
 * raises NotImplementedError, /root/reference/src/utils.py:80-88): the kernels read the keep
 * mask the forward saved (dropout_mask) or regenerate it with Philox, so dropout_p and
 * dropout_seed must equal the forward's. */
typedef struct fa2_bwd_args {
  const void* q;
  const void* k;
  const void* v;
  const void* o;
  const void* dout;       /* dO, [B, Sq, Hq, D] */
  const float* lse;       /* as written by fa2_fwd */
  float* delta;           /* workspace [B, Hq, lse_row_stride] fp32: -rowsum(O * dO) (scratch) */
  void* dq;               /* [B, Sq, Hq, D] in dq_dtype */
  void* dk;               /* [B, Sk, Hkv, D] in dtype */
  void* dv;               /* [B, Sk, Hkv, D] in dtype */
  const void* bias;
  const int32_t* cu_seqlens;
  int64_t q_stride[3];
  int64_t k_stride[3];
  int64_t v_stride[3];
  int64_t o_stride[3];
  int64_t do_stride[3];
  int64_t dq_stride[3];
  int64_t dk_stride[3];
  int64_t dv_stride[3];
  int64_t bias_stride[3];
  int32_t batch, heads_q, heads_kv, seqlen_q, seqlen_k, head_dim;
  int32_t lse_row_stride;
  int32_t causal;
  int32_t dtype;
  int32_t bias_dtype;
  int32_t dq_dtype;       /* dtype, or FA2_F32 */
  float softmax_scale;
  float dropout_p;
  uint64_t dropout_seed;
  /* optional bias gradient (ABI 5): when non-NULL (bias must be non-NULL too), the backward
   * also writes dL/d(bias) in fp32 into this buffer, which has the BIAS's shape
   * [1|B, 1|Hq, Sq, Sk] (element strides below: batch, head, row; unit key stride): element
   * (b', h', i, j) = sum over the batches and q-heads the bias broadcasts over (a zero batch /
   * head stride in bias_stride) of dS[b, hq, i, j] = P (dP - delta), summed in a fixed order
   * (bitwise reproducible), 0 where no pair is visible.  Every element is written; no
   * initialisation needed; no workspace beyond this buffer.  (The reference returns no bias
   * gradient, /root/reference/src/wrapper.py:86.) */
  float* dbias;
  int64_t dbias_stride[3];
  /* optional dK/dV split workspace (ABI 4): when non-NULL and at least
   * fa2_bwd_dkv_workspace_bytes(args) bytes (> 0 only for GQA / MQA problems whose
   * B * Hkv * ceil(Sk / 128) key blocks are too few to fill the GPU), the q-heads of each GQA
   * group are split over several dK/dV workgroups that write fp32 partial sums here, and a
   * reduction kernel adds them in a fixed order (bitwise reproducible).  NULL: one workgroup
   * per key block sums the whole group (the reference launches per q-head and sums on the
   * host, /root/reference/src/backward/caller.py:118-121,162-165).  Contents are scratch. */
  float* dkv_workspace;
  int64_t dkv_workspace_bytes;
  /* optional (ABI 6): the keep mask a forward with the same dropout_p / dropout_seed wrote
   * (fa2_fwd_args.dropout_mask); NULL = regenerate it with Philox (dQ, dK/dV and the bias
   * gradient each draw it again).  The backward kernels may READ words the forward never wrote
   * (tiles the causal mask hides, prefetches one tile past the last live one): such a word only
   * ever gates a (row, key) pair whose probability is 0, so its contents never reach a result and
   * the buffer needs no initialisation. */
  const uint32_t* dropout_mask;
} fa2_bwd_args;

int fa2_fwd(const fa2_fwd_args* args, void* stream);
int fa2_bwd(const fa2_bwd_args* args, void* stream);

/* The backward's launches selected by a bit mask, for per-kernel timing and profiling.
 * Launch order: bit 0 delta = rowsum(O * dO) (standalone kernel), bit 2 dQ (which also computes
 * delta for its rows and writes it to args->delta), bit 1 dK/dV (reads delta), bit 3 the bias
 * gradient (reads delta; needs args->dbias).  A mask must produce delta before dK/dV or the
 * bias gradient read it (bit 0 or bit 2, now or in an earlier call);
 * fa2_bwd == fa2_bwd_stages(args, 6, stream), 14 when args->dbias is set. */
int fa2_bwd_stages(const fa2_bwd_args* args, int stages, void* stream);
/* Bytes of dK/dV split workspace for these sizes (batch, heads_q, heads_kv, seqlen_k, head_dim):
 * 2 * nsplit * B * Hkv * Sk * D * 4, with nsplit the smallest divisor of the group size Hq / Hkv
 * that gives at least 512 dK/dV workgroups (two per CU), or 0 when no split applies (Hq == Hkv,
 * or the grid is already that large). */
int64_t fa2_bwd_dkv_workspace_bytes(const fa2_bwd_args* args);
/* Bytes of a dropout keep mask (ABI 6): batch * heads_q * ceil(seqlen_q / 32) * ceil(seqlen_k / 32) * 128. */
int64_t fa2_dropout_mask_bytes(int32_t batch, int32_t heads_q, int32_t seqlen_q, int32_t seqlen_k);

/* cu_seqlens[0] = 0, cu_seqlens[b+1] = cu_seqlens[b] + sum_s mask[b, s]  (mask: uint8/bool,
 * row stride mask_row_stride bytes).  Replaces attention_mask.sum(1).cumsum(0) and the
 * .item() syncs of the reference callers (src/forward/caller.py:48-50, src/utils.py:8-17). */
int fa2_cu_seqlens_from_mask(const uint8_t* mask, int64_t mask_row_stride, int32_t batch,
                             int32_t seqlen, int32_t* cu_seqlens, void* stream);

/* Kernel-path policy of ONE call (ABI 9; replaces ABI 7's process-wide fa2_set_path_policy: the
 * library keeps no mutable state between calls), for tests and A/B timing.  Bits of `disable`
 * turn a specialised path off so that the general kernels of the same launch run instead (same
 * math; the tests compare the two): FA2_PATH_FWD_HP the hand-placed D = 128 forward,
 * FA2_PATH_DQ_HP / FA2_PATH_DKDV_HP the hand-placed D = 128 dQ / dK-dV.  grid_cap > 0 caps the
 * grid of the persistent (one workgroup per CU) kernels, so that small problems run several work
 * units per workgroup.  A NULL policy, or {0, 0}, is the default: every path on, one workgroup
 * per CU (fa2_fwd / fa2_bwd_stages).  The environment is never read. */
enum fa2_path { FA2_PATH_FWD_HP = 1, FA2_PATH_DQ_HP = 2, FA2_PATH_DKDV_HP = 4 };
typedef struct fa2_policy {
  uint32_t disable;  /* fa2_path bits */
  int32_t grid_cap;  /* 0: no cap */
} fa2_policy;
int fa2_fwd_ex(const fa2_fwd_args* args, const fa2_policy* policy, void* stream);
int fa2_bwd_stages_ex(const fa2_bwd_args* args, int stages, const fa2_policy* policy, void* stream);

const char* fa2_last_error(void);
int fa2_version(void);

#ifdef __cplusplus
}
#endif
#endif /* FA2_AMD_H */
