// api.hip -- the C ABI (include/fa2_amd.h): argument validation, kernel selection, errors.
//
// Validation mirrors the reference callers' asserts (/root/reference/src/forward/caller.py:27-41,
// /root/reference/src/backward/caller.py:30-53) and error types (src/utils.py:57-109); the
// Python layer re-raises our codes as the reference's exception types.
#include <stdarg.h>
#include <stdio.h>

#include "fa2_internal.h"
#if FA2_HP_STAMPS
#include "common.h"
#endif

namespace {

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int hip_status(hipError_t e, const char* what) {
  if (e == hipSuccess) return FA2_OK;
  return fail(FA2_E_HIP, "%s: %s", what, hipGetErrorString(e));
}

int pick_dt(int d) {
  if (d <= 32) return 32;
  if (d <= 64) return 64;
  if (d <= 128) return 128;
  if (d <= 256) return 256;
  return 0;
}

bool aligned16(const void* ptr) { return ((uintptr_t)ptr & 15) == 0; }
bool strides8(const int64_t* s) { return s[0] % 8 == 0 && s[1] % 8 == 0 && s[2] % 8 == 0; }

// 16-byte vector path: every row of every 16-bit tensor starts on a 16-byte boundary.
bool vec_ok(int d, const void* ptr, const int64_t* s) { return d % 8 == 0 && aligned16(ptr) && strides8(s); }

int check_common(int B, int Hq, int Hkv, int Sq, int Sk, int D, int dtype, int lse_rs,
                 const int32_t* cu, float p) {
  if (B < 1 || Hq < 1 || Hkv < 1 || Sq < 0 || Sk < 0 || D < 1)
    return fail(FA2_E_INVALID, "bad sizes B=%d Hq=%d Hkv=%d Sq=%d Sk=%d D=%d", B, Hq, Hkv, Sq, Sk, D);
  if (Hq % Hkv != 0) return fail(FA2_E_INVALID, "heads_q=%d is not divisible by heads_kv=%d", Hq, Hkv);
  if (dtype != FA2_F16 && dtype != FA2_BF16) return fail(FA2_E_INVALID, "dtype %d: only fp16 and bf16", dtype);
  if (!pick_dt(D)) return fail(FA2_E_UNSUPPORTED, "head_dim %d > 256", D);
  if (lse_rs < ((Sq + 31) / 32) * 32 || lse_rs % 32 != 0)
    return fail(FA2_E_INVALID, "lse_row_stride %d must be a multiple of 32 and >= seqlen_q rounded up (%d)", lse_rs, Sq);
  if (cu && Sq != Sk) return fail(FA2_E_INVALID, "varlen (cu_seqlens) requires seqlen_q == seqlen_k");
  if (!(p >= 0.f && p < 1.f)) return fail(FA2_E_INVALID, "dropout_p=%f must be in [0, 1)", p);
  return FA2_OK;
}

template <typename F4, typename F8, typename F12, typename F16>
hipError_t dispatch_dt(int dt, F4 f32, F8 f64, F12 f128, F16 f256) {
  switch (dt) {
    case 32: return f32();
    case 64: return f64();
    case 128: return f128();
    default: return f256();
  }
}

}  // namespace

namespace fa2 {
// the policy of the fa2_*_ex call running on this thread (nullptr: defaults); set only for the
// duration of that call (PolicyScope), so the library keeps no state between calls
thread_local const fa2_policy* g_call_policy = nullptr;
}  // namespace fa2

namespace {
struct PolicyScope {
  const fa2_policy* prev;
  explicit PolicyScope(const fa2_policy* p) : prev(fa2::g_call_policy) { fa2::g_call_policy = p; }
  ~PolicyScope() { fa2::g_call_policy = prev; }
};
int check_policy(const fa2_policy* p) {
  if (!p) return FA2_OK;
  if (p->disable & ~(uint32_t)(FA2_PATH_FWD_HP | FA2_PATH_DQ_HP | FA2_PATH_DKDV_HP))
    return fail(FA2_E_INVALID, "unknown path bits 0x%x", p->disable);
  if (p->grid_cap < 0) return fail(FA2_E_INVALID, "grid_cap %d < 0", p->grid_cap);
  return FA2_OK;
}
}  // namespace

extern "C" {

int fa2_version(void) { return FA2_ABI_VERSION; }

const char* fa2_last_error(void) { return g_err; }

int fa2_fwd(const fa2_fwd_args* a, void* stream) { return fa2_fwd_ex(a, nullptr, stream); }

int fa2_fwd_ex(const fa2_fwd_args* a, const fa2_policy* policy, void* stream) {
  if (!a) return fail(FA2_E_INVALID, "null args");
  if (int prc = check_policy(policy)) return prc;
  PolicyScope scope(policy);
  int rc = check_common(a->batch, a->heads_q, a->heads_kv, a->seqlen_q, a->seqlen_k, a->head_dim, a->dtype,
                        a->lse_row_stride, a->cu_seqlens, a->dropout_p);
  if (rc) return rc;
  // an empty side may come with null pointers (torch gives size-0 tensors data_ptr 0)
  const bool qs = a->seqlen_q > 0, ks = a->seqlen_k > 0;
  if ((qs && (!a->q || !a->o || !a->lse)) || (ks && (!a->k || !a->v))) return fail(FA2_E_INVALID, "null tensor pointer");
  if (a->bias && a->bias_dtype != FA2_F16 && a->bias_dtype != FA2_BF16 && a->bias_dtype != FA2_F32)
    return fail(FA2_E_INVALID, "bias dtype %d", a->bias_dtype);
  if (a->seqlen_q == 0) return FA2_OK;
  const int D = a->head_dim;
  const bool aligned = vec_ok(D, a->q, a->q_stride) && vec_ok(D, a->k, a->k_stride) &&
                       vec_ok(D, a->v, a->v_stride) && vec_ok(D, a->o, a->o_stride);
  hipStream_t st = (hipStream_t)stream;
  const bool bf = a->dtype == FA2_BF16;
  const int dt = pick_dt(D);
  hipError_t e;
  if (bf)
    e = dispatch_dt(dt, [&] { return fa2::launch_fwd_dt<true, 32>(*a, aligned, st); },
                    [&] { return fa2::launch_fwd_dt<true, 64>(*a, aligned, st); },
                    [&] { return fa2::launch_fwd_dt<true, 128>(*a, aligned, st); },
                    [&] { return fa2::launch_fwd_dt<true, 256>(*a, aligned, st); });
  else
    e = dispatch_dt(dt, [&] { return fa2::launch_fwd_dt<false, 32>(*a, aligned, st); },
                    [&] { return fa2::launch_fwd_dt<false, 64>(*a, aligned, st); },
                    [&] { return fa2::launch_fwd_dt<false, 128>(*a, aligned, st); },
                    [&] { return fa2::launch_fwd_dt<false, 256>(*a, aligned, st); });
  return hip_status(e, "fa2_fwd launch");
}

int fa2_bwd_stages(const fa2_bwd_args* a, int stages, void* stream) { return fa2_bwd_stages_ex(a, stages, nullptr, stream); }

int fa2_bwd_stages_ex(const fa2_bwd_args* a, int stages, const fa2_policy* policy, void* stream) {
  if (!a) return fail(FA2_E_INVALID, "null args");
  if (int prc = check_policy(policy)) return prc;
  PolicyScope scope(policy);
  int rc = check_common(a->batch, a->heads_q, a->heads_kv, a->seqlen_q, a->seqlen_k, a->head_dim, a->dtype,
                        a->lse_row_stride, a->cu_seqlens, a->dropout_p);
  if (rc) return rc;
  const bool qs = a->seqlen_q > 0, ks = a->seqlen_k > 0;
  if ((qs && (!a->q || !a->o || !a->dout || !a->lse || !a->delta || !a->dq)) || (ks && (!a->k || !a->v || !a->dk || !a->dv)))
    return fail(FA2_E_INVALID, "null tensor pointer");
  if (a->dq_dtype != a->dtype && a->dq_dtype != FA2_F32) return fail(FA2_E_INVALID, "dq dtype %d", a->dq_dtype);
  if (a->bias && a->bias_dtype != FA2_F16 && a->bias_dtype != FA2_BF16 && a->bias_dtype != FA2_F32)
    return fail(FA2_E_INVALID, "bias dtype %d", a->bias_dtype);
  if (stages & ~15) return fail(FA2_E_INVALID, "stage mask %d", stages);
  if (a->dbias && !a->bias) return fail(FA2_E_INVALID, "dbias requested without a bias");
  if ((stages & 8) && !a->dbias) return fail(FA2_E_INVALID, "stage 8 (bias gradient) without a dbias buffer");
  if (a->seqlen_q == 0 && a->seqlen_k == 0) return FA2_OK;  // empty dQ, dK, dV
  const int D = a->head_dim;
  bool aligned = vec_ok(D, a->q, a->q_stride) && vec_ok(D, a->k, a->k_stride) && vec_ok(D, a->v, a->v_stride) &&
                 vec_ok(D, a->o, a->o_stride) && vec_ok(D, a->dout, a->do_stride) &&
                 vec_ok(D, a->dk, a->dk_stride) && vec_ok(D, a->dv, a->dv_stride) &&
                 a->k_stride[1] == a->v_stride[1];  // dq_kernel stages K and V with one offset set
  if (a->dq_dtype == FA2_F32)
    aligned = aligned && aligned16(a->dq) && a->dq_stride[0] % 4 == 0 && a->dq_stride[1] % 4 == 0 && a->dq_stride[2] % 4 == 0;
  else
    aligned = aligned && vec_ok(D, a->dq, a->dq_stride);
  if (a->dkv_workspace) {
    const int64_t need = fa2_bwd_dkv_workspace_bytes(a);
    if (need == 0) return fail(FA2_E_INVALID, "dkv_workspace given but no dK/dV split applies to these sizes");
    if (a->dkv_workspace_bytes < need)
      return fail(FA2_E_INVALID, "dkv_workspace_bytes %lld < %lld required", (long long)a->dkv_workspace_bytes, (long long)need);
    if (!aligned16(a->dkv_workspace)) return fail(FA2_E_INVALID, "dkv_workspace must be 16-byte aligned");
  }
  hipStream_t st = (hipStream_t)stream;
  const bool bf = a->dtype == FA2_BF16;
  const int dt = pick_dt(D);
  hipError_t e;
  if (bf)
    e = dispatch_dt(dt, [&] { return fa2::launch_bwd_dt<true, 32>(*a, aligned, stages, st); },
                    [&] { return fa2::launch_bwd_dt<true, 64>(*a, aligned, stages, st); },
                    [&] { return fa2::launch_bwd_dt<true, 128>(*a, aligned, stages, st); },
                    [&] { return fa2::launch_bwd_dt<true, 256>(*a, aligned, stages, st); });
  else
    e = dispatch_dt(dt, [&] { return fa2::launch_bwd_dt<false, 32>(*a, aligned, stages, st); },
                    [&] { return fa2::launch_bwd_dt<false, 64>(*a, aligned, stages, st); },
                    [&] { return fa2::launch_bwd_dt<false, 128>(*a, aligned, stages, st); },
                    [&] { return fa2::launch_bwd_dt<false, 256>(*a, aligned, stages, st); });
  return hip_status(e, "fa2_bwd launch");
}

int fa2_bwd(const fa2_bwd_args* a, void* stream) { return fa2_bwd_stages(a, a && a->dbias ? 14 : 6, stream); }

int64_t fa2_bwd_dkv_workspace_bytes(const fa2_bwd_args* a) {
  if (!a || a->seqlen_q <= 0 || a->seqlen_k <= 0 || a->head_dim < 1) return 0;
  return fa2::dkv_workspace_bytes(a->batch, a->heads_q, a->heads_kv, a->seqlen_k, a->head_dim);
}

int64_t fa2_dropout_mask_bytes(int32_t batch, int32_t heads_q, int32_t seqlen_q, int32_t seqlen_k) {
  if (batch < 1 || heads_q < 1 || seqlen_q < 1 || seqlen_k < 1) return 0;
  // + one tile of slack: the hand-placed dK/dV reads a wave's two key tiles as one 256-byte run,
  // whose second tile lies past the end when the first is the last of the buffer (ABI 8)
  return (int64_t)batch * heads_q * ((seqlen_q + 31) / 32) * ((seqlen_k + 31) / 32) * 128 + 128;
}

int fa2_cu_seqlens_from_mask(const uint8_t* mask, int64_t mask_row_stride, int32_t batch, int32_t seqlen,
                             int32_t* cu_seqlens, void* stream) {
  if (!mask || !cu_seqlens || batch < 1 || seqlen < 0) return fail(FA2_E_INVALID, "bad cu_seqlens arguments");
  return hip_status(fa2::launch_cu_seqlens(mask, mask_row_stride, batch, seqlen, cu_seqlens, (hipStream_t)stream),
                    "fa2_cu_seqlens_from_mask launch");
}

#if FA2_HP_STAMPS
// development builds only (not part of the C ABI in include/fa2_amd.h): read and clear the
// hand-placed kernels' s_memtime sums
int fa2_debug_hp_stamps(unsigned long long* out16) {
  unsigned long long* b = fa2::hp_stamp_buf();
  if (!b || !out16) return -1;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpy(out16, b, 16 * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return hipMemset(b, 0, 16 * sizeof(unsigned long long)) == hipSuccess ? 0 : -1;
}
#endif

}  // extern "C"
