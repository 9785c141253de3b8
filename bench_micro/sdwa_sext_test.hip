// SDWA byte sign-extension on gfx950 (dev check behind hp_gen.py FwdGen.mask_and / mask_prep_items):
// sext(byte) keeps the byte's low 7 bits (0x80 -> 0xFFFFFF80), so the AND masks must be whole
// 0x00 / 0xFF bytes; the v_perm_b32 sign selectors (0x0B090A08 on S0 = W << (7 - c),
// S1 = W << (15 - c)) build byte n = bit c + 8 n of W ? 0xFF : 0x00.
// build: hipcc --offload-arch=gfx950 -O2 bench_micro/sdwa_sext_test.hip -o bench_micro/sdwa_sext_test
#include <hip/hip_runtime.h>
#include <stdio.h>
#define T(N, H)                                                                                   \
  {                                                                                              \
    unsigned a = 0x12345678u;                                                                    \
    asm volatile("v_and_b32_sdwa %0, sext(%1), %0 dst_sel:WORD_" #H                              \
                 " dst_unused:UNUSED_PRESERVE src0_sel:BYTE_" #N " src1_sel:WORD_" #H            \
                 : "+v"(a) : "v"(m));                                                            \
    r[2 * N + H] = a;                                                                            \
  }
__global__ void k(unsigned* out, unsigned m) {
  unsigned r[8];
  T(0, 0) T(0, 1) T(1, 0) T(1, 1) T(2, 0) T(2, 1) T(3, 0) T(3, 1)
  if (threadIdx.x == 0)
    for (int i = 0; i < 8; ++i) out[i] = r[i];
}
__global__ void kp(unsigned* out, unsigned w) {
  unsigned r[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    unsigned s0 = w << (7 - c), s1 = w << (15 - c), m;
    asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(m) : "v"(s0), "v"(s1), "s"(0x0b090a08u));
    r[c] = m;
  }
  if (threadIdx.x == 0)
    for (int c = 0; c < 4; ++c) out[c] = r[c];
}
int main() {
  unsigned* d;
  hipMalloc(&d, 32);
  const unsigned ms[4] = {0x00000080u, 0x00008000u, 0x80800000u, 0x7f7f7f7fu};
  for (unsigned m : ms) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, m);
    unsigned h[8];
    hipMemcpy(h, d, 32, hipMemcpyDeviceToHost);
    printf("m=%08x:", m);
    for (int i = 0; i < 8; ++i) printf(" n%d/w%d=%08x", i / 2, i % 2, h[i]);
    printf("\n");
  }
  int bad = 0;
  for (unsigned w : {0x01020408u, 0x80402010u, 0xdeadbeefu, 0x12345678u}) {
    hipLaunchKernelGGL(kp, dim3(1), dim3(64), 0, 0, d, w);
    unsigned h[4];
    hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    for (int c = 0; c < 4; ++c) {
      unsigned want = 0;
      for (int n = 0; n < 4; ++n) want |= ((w >> (c + 8 * n)) & 1u ? 0xFFu : 0u) << (8 * n);
      if (h[c] != want) { printf("perm w=%08x c=%d: %08x want %08x\n", w, c, h[c], want); bad = 1; }
    }
  }
  printf("perm byte masks: %s\n", bad ? "MISMATCH" : "ok");
  return bad;
}
