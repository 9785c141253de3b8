// SDWA semantics on gfx950 (dev check behind hp_gen.py DkdvGen.pack_keep): an op with
// dst_sel:WORD_1 writes the LOW 16 bits of its result into the destination's high word, so the
// sources must select WORD_1 too.  build: hipcc --offload-arch=gfx950 -O2 bench_micro/sdwa_test.hip -o bench_micro/sdwa_test
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned* out) {
  unsigned a0 = 0x12345678u, a1 = 0x12345678u, a2 = 0x12345678u, a3 = 0x12345678u;
  unsigned ones = 0xFFFFFFFFu, zero = 0u;
  asm volatile("v_and_b32_sdwa %0, %1, %0 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD" : "+v"(a0) : "v"(ones));
  asm volatile("v_and_b32_sdwa %0, %1, %0 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD" : "+v"(a1) : "v"(zero));
  asm volatile("v_and_b32_sdwa %0, %1, %0 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1" : "+v"(a2) : "v"(ones));
  asm volatile("v_and_b32_sdwa %0, %1, %0 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1" : "+v"(a3) : "v"(zero));
  if (threadIdx.x == 0) { out[0] = a0; out[1] = a1; out[2] = a2; out[3] = a3; }
}
int main() {
  unsigned* d; hipMalloc(&d, 16);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  unsigned h[4]; hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
  printf("%08x %08x %08x %08x (expect 12345678 12340000 12345678 00005678)\n", h[0], h[1], h[2], h[3]);
  return 0;
}
