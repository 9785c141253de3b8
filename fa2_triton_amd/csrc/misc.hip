// misc.hip -- device-side varlen bookkeeping.
//
// The reference computes cum_seqlens with attention_mask.sum(1).cumsum(0) and then packs and
// unpacks the batch with per-row host loops that each call .item()
// (/root/reference/src/forward/caller.py:44-63,118-120, src/utils.py:8-31).  Our kernels read
// the padded [B, S, H, D] tensors in place, so all they need is cu_seqlens, built here on
// the device with no host synchronisation.
#include "common.h"
#include "fa2_internal.h"

namespace fa2 {

__global__ void __launch_bounds__(256) cu_seqlens_kernel(const uint8_t* mask, int64_t stride, int batch,
                                                         int seqlen, int32_t* cu) {
  __shared__ int part[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int running = 0;
  if (tid == 0) cu[0] = 0;
  for (int b = 0; b < batch; ++b) {
    int c = 0;
    for (int s = tid; s < seqlen; s += 256) c += mask[(int64_t)b * stride + s] != 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if (lane == 0) part[w] = c;
    __syncthreads();
    if (tid == 0) {
      running += part[0] + part[1] + part[2] + part[3];
      cu[b + 1] = running;
    }
    __syncthreads();
  }
}

hipError_t launch_cu_seqlens(const uint8_t* mask, int64_t stride, int batch, int seqlen, int32_t* out,
                             hipStream_t st) {
  hipLaunchKernelGGL(cu_seqlens_kernel, dim3(1), dim3(256), 0, st, mask, stride, batch, seqlen, out);
  return hipGetLastError();
}

}  // namespace fa2
