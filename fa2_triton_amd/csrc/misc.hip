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

// ---------------------------------------------------------------------------------------------
// Dropout keep mask ahead of the forward.  keep(off) = tl.rand(seed, off) > p
// (/root/reference/src/forward/compute_row_blocks.py:76-79; common.h philox_uniform): the
// uniform is (float)x' * 2^-31-ish with x' = x < 0 ? -x - 1 : x, monotone in x', so keep <=> x' > T
// for the integer T = dropout_keep_threshold(p), and with u = x + T + 1 (mod 2^32) that is
// u > 2T + 1 -- two integer ops instead of the convert / multiply / compare of the float.
uint32_t dropout_keep_threshold(float p) {
  // largest x' in [0, 2^31 - 1] whose uniform is <= p (the uniform of 0 is 0 <= p)
  auto uni = [](uint32_t x) { return (float)(int32_t)x * 4.6566127342e-10f; };
  uint32_t lo = 0, hi = 0x7fffffffu;
  while (lo < hi) {
    const uint32_t mid = lo + (hi - lo + 1) / 2;
    if (uni(mid) <= p) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// One lane = one 32-key word of one row: bit j = keep(off0 + j).  Within a word the counter's
// high half is constant unless its low half wraps (checked per lane), so Philox round 0's
// c0 = hi ^ k0 and round 1's B * c0 product are per-word constants, the round-0 product
// B * (lo + j) a running 64-bit sum; rounds 2-9 are the full ones (common.h philox_uniform).
FA2_DEV uint32_t keep_word(uint32_t k0, uint32_t k1, uint64_t off0, uint32_t t1, uint32_t span) {
  constexpr uint32_t kA = 0xD2511F53u, kB = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
  const uint32_t lo = (uint32_t)off0, hi = (uint32_t)(off0 >> 32);
  uint32_t word = 0;
  if (lo <= 0xffffffe0u) {
    const uint32_t c0r = hi ^ k0;                    // c0 after round 0 (c2 = c3 = 0)
    const uint64_t pb1 = (uint64_t)kA * c0r;         // round 1: the c0 product, per word
    const uint32_t x1 = (uint32_t)(pb1 >> 32) ^ (k1 + W1), c3r = (uint32_t)pb1;
    uint64_t pb0 = (uint64_t)kA * (lo + 31);         // round 0: kA * (lo + j), j = 31 .. 0
#pragma unroll 2
    for (int j = 31; j >= 0; --j) {
      uint32_t c2 = (uint32_t)(pb0 >> 32) ^ k1, c3 = (uint32_t)pb0;  // round 0 (c1 = 0)
      pb0 -= kA;
      const uint64_t pa1 = (uint64_t)kB * c2;        // round 1
      uint32_t c0 = (uint32_t)(pa1 >> 32) ^ (k0 + W0), c1 = (uint32_t)pa1;
      c2 = x1 ^ c3;
      c3 = c3r;
      uint32_t r0 = k0 + 2 * W0, r1 = k1 + 2 * W1;
#pragma unroll
      for (int i = 2; i < 10; ++i) {
        const uint64_t pa = (uint64_t)kB * c2, pb = (uint64_t)kA * c0;
        c0 = xor3((uint32_t)(pa >> 32), c1, r0);
        c2 = xor3((uint32_t)(pb >> 32), c3, r1);
        c1 = (uint32_t)pa;
        c3 = (uint32_t)pb;
        r0 += W0;
        r1 += W1;
      }
      word = word + word + (c0 + t1 > span ? 1u : 0u);  // shifted in from bit 31 down
    }
  } else {
    for (int j = 0; j < 32; ++j) {
      uint32_t c0 = (uint32_t)(off0 + j), c1 = (uint32_t)((off0 + j) >> 32), c2 = 0, c3 = 0, r0 = k0, r1 = k1;
      for (int i = 0; i < 10; ++i) {
        const uint64_t pa = (uint64_t)kB * c2, pb = (uint64_t)kA * c0;
        c0 = xor3((uint32_t)(pa >> 32), c1, r0);
        c2 = xor3((uint32_t)(pb >> 32), c3, r1);
        c1 = (uint32_t)pa;
        c3 = (uint32_t)pb;
        r0 += W0;
        r1 += W1;
      }
      word |= (c0 + t1 > span ? 1u : 0u) << j;
    }
  }
  return word;
}

// Writes the keep words of the tiled layout (include/fa2_amd.h, fa2_fwd_args.dropout_mask) that a
// forward can read: rows < seqlen_q (< Lq with cu_seqlens), key words starting below Lk and, under
// the causal mask, not wholly past the last row of their 32-row tile.  The bits equal fwd_kernel's
// (same offsets: /root/reference/src/forward/kernel.py:146-148, int64).  A workgroup = 8 key words
// x 32 rows of one (batch, q-head, row tile): 1 KiB of contiguous words; persistent over the
// (head, row tile) lines, taken in pairs (rt, nrb - 1 - rt) so that under the causal mask every
// pair holds about the same number of words.
__global__ void __launch_bounds__(256) dropout_mask_kernel(const fa2_fwd_args p, uint32_t t1, uint32_t span) {
  const int nrb = (p.seqlen_q + 31) >> 5, ncw = (p.seqlen_k + 31) >> 5;
  const int half = (nrb + 1) >> 1;
  const int pairs = p.batch * p.heads_q * half;
  const int r32 = threadIdx.x & 31, kwl = threadIdx.x >> 5;
  const uint32_t k0 = (uint32_t)p.dropout_seed, k1 = (uint32_t)(p.dropout_seed >> 32);
  for (int ln = blockIdx.x * 2; ln < 2 * pairs; ln += (ln & 1) ? 2 * gridDim.x - 1 : 1) {
    const int pr = ln >> 1, bh = pr / half, j = pr - bh * half;
    const int rt = (ln & 1) ? nrb - 1 - j : j;
    if ((ln & 1) && rt == j) continue;  // odd nrb: the middle tile once
    const int b = bh / p.heads_q, hq = bh - b * p.heads_q;
    int Lq = p.seqlen_q, Lk = p.seqlen_k, cu = 0;
    if (p.cu_seqlens) {
      cu = p.cu_seqlens[b];
      Lq = Lk = p.cu_seqlens[b + 1] - cu;
    }
    const int r0 = rt * 32;
    if (r0 >= Lq) continue;
    int kend = Lk;  // keys the line's rows can see
    if (p.causal) kend = max(0, min(Lk, r0 + 31 + (Lk - Lq) + 1));
    const int nkw = (kend + 31) >> 5;
    const int qi = r0 + r32;
    const uint64_t base = (uint64_t)Lk * ((uint64_t)cu + (uint64_t)Lq * ((uint64_t)hq + (uint64_t)p.heads_q * (p.cu_seqlens ? 0 : b)));
    const uint64_t rowoff = base + (uint64_t)qi * Lk;
    uint32_t* out = p.dropout_mask + ((int64_t)bh * nrb + rt) * ncw * 32 + r32;
    for (int kw = kwl; kw < nkw; kw += 8) {
      if (qi < Lq) out[(int64_t)kw * 32] = keep_word(k0, k1, rowoff + (uint64_t)kw * 32, t1, span);
    }
  }
}

hipError_t launch_dropout_mask(const fa2_fwd_args& a, hipStream_t st) {
  const uint32_t T = dropout_keep_threshold(a.dropout_p);
  const int pairs = a.batch * a.heads_q * ((((a.seqlen_q + 31) >> 5) + 1) >> 1);
  const int grid = min(pairs, 8 * device_cu_count());
  if (grid <= 0) return hipSuccess;
  hipLaunchKernelGGL(dropout_mask_kernel, dim3(grid), dim3(256), 0, st, a, T + 1u, 2u * T + 1u);
  return hipGetLastError();
}

}  // namespace fa2
