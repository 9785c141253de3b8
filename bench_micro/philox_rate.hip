// Philox-4x32-10 throughput on this box (dev microbenchmark; not part of the library): the VALU
// bound of the dropout forward, which draws one philox_uniform per (row, key) element exactly as
// the reference's tl.rand does (/root/reference/src/forward/compute_row_blocks.py:76-79).
// Every lane of a full-occupancy grid draws N uniforms with the library's philox_uniform
// (csrc/common.h) and keeps a count of kept elements (so nothing is dead code); reported as
// elements per second over the whole chip, median of 10 launches after 2 warm-ups.
// build: hipcc --offload-arch=gfx950 -O3 -I fa2_triton_amd/csrc -I include bench_micro/philox_rate.hip -o bench_micro/philox_rate
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#include "common.h"

// the same rounds with separate 32-bit high / low multiplies (A/B of the multiply form)
__device__ __forceinline__ float philox_uniform_hilo(uint64_t seed, uint64_t offset) {
  uint32_t c0 = (uint32_t)offset, c1 = (uint32_t)(offset >> 32), c2 = 0, c3 = 0;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t hi0 = __umulhi(0xCD9E8D57u, c2), lo0 = 0xCD9E8D57u * c2;
    const uint32_t hi1 = __umulhi(0xD2511F53u, c0), lo1 = 0xD2511F53u * c0;
    c0 = hi0 ^ c1 ^ k0;
    c2 = hi1 ^ c3 ^ k1;
    c1 = lo0;
    c3 = lo1;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  int32_t x = (int32_t)c0;
  x = x < 0 ? -x - 1 : x;
  return (float)x * 4.6566127342e-10f;
}

template <int FORM>
__global__ void __launch_bounds__(256) philox_draw(uint64_t seed, int per_lane, float p, unsigned* out) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned kept = 0;
  for (int i = 0; i < per_lane; ++i) {
    const uint64_t off = tid * (uint64_t)per_lane + i;
    kept += (FORM == 0 ? fa2::philox_uniform(seed, off) : philox_uniform_hilo(seed, off)) > p ? 1u : 0u;
  }
  if (kept == 0xFFFFFFFFu) out[0] = kept;  // never true: keeps the draws live
}

int main() {
  const int blocks = 256 * 8, per_lane = 4096;
  unsigned* out;
  hipMalloc(&out, 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int form = 0; form < 2; ++form) {
    std::vector<float> ms;
    for (int r = 0; r < 12; ++r) {
      hipEventRecord(e0);
      if (form == 0)
        hipLaunchKernelGGL(philox_draw<0>, dim3(blocks), dim3(256), 0, 0, 0x1234567890ABCDEFull, per_lane, 0.1f, out);
      else
        hipLaunchKernelGGL(philox_draw<1>, dim3(blocks), dim3(256), 0, 0, 0x1234567890ABCDEFull, per_lane, 0.1f, out);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float t;
      hipEventElapsedTime(&t, e0, e1);
      if (r >= 2) ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    const double med = ms[ms.size() / 2];
    const double n = (double)blocks * 256 * per_lane;
    printf("{\"kernel\": \"philox_draw\", \"multiply\": \"%s\", \"elements\": %.0f, \"median_ms\": %.4f, "
           "\"elements_per_s\": %.4e}\n", form == 0 ? "v_mad_u64_u32" : "mul_hi + mul_lo", n, med, n / (med * 1e-3));
  }
  return 0;
}
