// fa2_internal.h -- launcher entry points shared between the kernel TUs and the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include "fa2_amd.h"  // include/ (build.py passes -I)

namespace fa2 {

// the fa2_policy of the fa2_fwd_ex / fa2_bwd_stages_ex call running on this thread, nullptr for
// the defaults (api.hip; set for the duration of that call only)
extern thread_local const fa2_policy* g_call_policy;
inline bool path_on(uint32_t bit) { return !(g_call_policy && (g_call_policy->disable & bit)); }
inline int capped_grid(int ncu) {
  const int c = g_call_policy ? g_call_policy->grid_cap : 0;
  return c > 0 && c < ncu ? c : ncu;
}

// Forward, one translation unit per (dtype, head-dim tile); see fwd_inst.hip.
template <bool BF16, int DT>
hipError_t launch_fwd_dt(const fa2_fwd_args& a, bool aligned, hipStream_t st);

// Backward: delta = rowsum(O * dO), then dK/dV (key-stationary) and dQ (query-stationary).
// stages: bit 0 delta, bit 1 dK/dV, bit 2 dQ (7 = the whole backward).
template <bool BF16, int DT>
hipError_t launch_bwd_dt(const fa2_bwd_args& a, bool aligned, int stages, hipStream_t st);

hipError_t launch_cu_seqlens(const uint8_t* mask, int64_t stride, int batch, int seqlen,
                             int32_t* out, hipStream_t st);

// Dropout keep words of a forward (misc.hip, into a.dropout_mask) drawn ahead of a kernel that
// reads them; keep <=> the Philox integer x' > dropout_keep_threshold(p).
uint32_t dropout_keep_threshold(float p);
hipError_t launch_dropout_mask(const fa2_fwd_args& a, hipStream_t st);

// q-head split of dK/dV (ABI 4): the smallest divisor s of the GQA group size G = Hq / Hkv with
// s * B * Hkv * ceil(Sk / 128) >= kDkvTargetGrid workgroups (two per CU), G if none is; 1 when
// G == 1 or the grid is already that large.
constexpr int kDkvTargetGrid = 512;
inline int dkv_split_count(int B, int Hq, int Hkv, int Sk) {
  if (B < 1 || Hkv < 1 || Hq % Hkv != 0 || Sk < 1) return 1;
  const int G = Hq / Hkv;
  const int64_t grid = (int64_t)((Sk + 127) / 128) * B * Hkv;
  if (G <= 1 || grid >= kDkvTargetGrid) return 1;
  for (int s = 2; s < G; ++s)
    if (G % s == 0 && grid * s >= kDkvTargetGrid) return s;
  return G;
}
inline int64_t dkv_workspace_bytes(int B, int Hq, int Hkv, int Sk, int D) {
  const int s = dkv_split_count(B, Hq, Hkv, Sk);
  return s > 1 ? 2 * (int64_t)s * B * Hkv * Sk * D * 4 : 0;
}
// the split a launch uses: only with a large enough workspace (checked by fa2_bwd_stages)
inline int dkv_split(const fa2_bwd_args& a) {
  return a.dkv_workspace ? dkv_split_count(a.batch, a.heads_q, a.heads_kv, a.seqlen_k) : 1;
}

}  // namespace fa2
