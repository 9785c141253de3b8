// MFMA throughput on random operands: v_mfma_f32_32x32x16_bf16 vs v_mfma_f32_16x16x32_bf16,
// every CU, 2 waves per SIMD, operands in registers (dev microbenchmark; not part of the library).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int SHAPE>
__global__ void __launch_bounds__(512, 2) k(const bf16x8* in, float* out, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  bf16x8 a = in[t & 4095], b = in[(t * 7 + 3) & 4095];
  bf16x8 a2 = in[(t + 17) & 4095], b2 = in[(t * 5 + 11) & 4095];
  if constexpr (SHAPE == 32) {
    f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int i = 0; i < iters; ++i) {
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b2, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b2, c3, 0, 0, 0);
    }
    float s = 0;
    for (int i = 0; i < 16; ++i) s += c0[i] + c1[i] + c2[i] + c3[i];
    out[t] = s;
  } else {
    f32x4 c[8] = {};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) c[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16((j & 1) ? a2 : a, (j & 2) ? b2 : b, c[j], 0, 0, 0);
    }
    float s = 0;
    for (int j = 0; j < 8; ++j) s += c[j][0] + c[j][1] + c[j][2] + c[j][3];
    out[t] = s;
  }
}

int main(int argc, char** argv) {
  int zero = argc > 1 && argv[1][0] == 'z';
  bf16x8* in; float* out;
  (void)hipMalloc(&in, 4096 * 16); (void)hipMalloc(&out, 256 * 2 * 512 * 4 * 8);
  unsigned short h[4096 * 8];
  srand(1);
  for (int i = 0; i < 4096 * 8; ++i) {
    float f = zero ? 0.f : ((rand() % 2000) - 1000) / 500.f;
    unsigned u; memcpy(&u, &f, 4); h[i] = u >> 16;
  }
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  const int blocks = 256 * 2, iters = 20000;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int shape : {32, 16, 32, 16}) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      if (shape == 32) hipLaunchKernelGGL(k<32>, dim3(blocks), dim3(512), 0, 0, in, out, iters);
      else hipLaunchKernelGGL(k<16>, dim3(blocks), dim3(512), 0, 0, in, out, iters / 2);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      // flops: 32x32x16: 4 mfma x 32768 flop; 16x16x32: 8 mfma x 16384 flop (half the iters)
      double fl = (double)blocks * 8 * iters * 4 * 32768.0;
      if (rep) printf("%s shape %d: %.3f ms  %.1f TFLOP/s\n", zero ? "zeros" : "random", shape, ms, fl / ms / 1e9);
    }
  }
  return 0;
}
