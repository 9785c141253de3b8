// HBM copy bandwidth on this box (dev microbenchmark; not part of the library): BASELINE.md section 2
// asks for the 8 TB/s spec to be re-measured beside the MFMA microbenchmark.
// A float4 grid-stride copy of a 2 GiB buffer (far past the 256 MiB Infinity Cache), 256-thread
// workgroups, 4 independent 16-byte loads in flight per thread; reported as (read + write) bytes / time,
// median of 10 launches after 2 warm-ups.
// build: hipcc --offload-arch=gfx950 -O3 bench_micro/hbm_copy.hip -o bench_micro/hbm_copy
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) copy4(const f32x4* __restrict__ src, f32x4* __restrict__ dst, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    const f32x4 a = __builtin_nontemporal_load(src + i), b = __builtin_nontemporal_load(src + i + stride);
    const f32x4 c = __builtin_nontemporal_load(src + i + 2 * stride), d = __builtin_nontemporal_load(src + i + 3 * stride);
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n; i += stride) dst[i] = src[i];
}

__global__ void __launch_bounds__(256) fill(f32x4* p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = f32x4{(float)(i & 1023), 1.f, 2.f, 3.f};
}

int main() {
  const size_t bytes = (size_t)2 << 30, n = bytes / 16;
  f32x4 *a, *b;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, a, n);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int blocks : {2048, 4096, 8192}) {
    std::vector<float> ms;
    for (int rep = 0; rep < 12; ++rep) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(copy4, dim3(blocks), dim3(256), 0, 0, a, b, n);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float t;
      hipEventElapsedTime(&t, e0, e1);
      if (rep >= 2) ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    const double med = ms[ms.size() / 2];
    printf("{\"kernel\": \"copy4\", \"blocks\": %d, \"bytes_moved\": %zu, \"median_ms\": %.4f, \"GBps\": %.1f, \"frac_of_8TBps\": %.3f}\n",
           blocks, 2 * bytes, med, 2.0 * bytes / (med * 1e-3) / 1e9, 2.0 * bytes / (med * 1e-3) / 8e12);
  }
  hipFree(a);
  hipFree(b);
  return 0;
}
