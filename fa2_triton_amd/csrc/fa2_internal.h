// fa2_internal.h -- launcher entry points shared between the kernel TUs and the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/fa2_amd.h"

namespace fa2 {

// Forward, one translation unit per (dtype, head-dim tile); see fwd_inst.hip.
template <bool BF16, int DT>
hipError_t launch_fwd_dt(const fa2_fwd_args& a, bool aligned, hipStream_t st);

// Backward: delta = rowsum(O * dO), then dK/dV (key-stationary) and dQ (query-stationary).
// stages: bit 0 delta, bit 1 dK/dV, bit 2 dQ (7 = the whole backward).
template <bool BF16, int DT>
hipError_t launch_bwd_dt(const fa2_bwd_args& a, bool aligned, int stages, hipStream_t st);

hipError_t launch_cu_seqlens(const uint8_t* mask, int64_t stride, int batch, int seqlen,
                             int32_t* out, hipStream_t st);

}  // namespace fa2
