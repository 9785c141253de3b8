// fwd_w64_kernel.h -- FlashAttention-2 forward, one wave per SIMD, 64 query rows per wave.
//
// Same semantics as fwd_kernel.h (/root/reference/src/forward/kernel.py:61-291,
// compute_row_blocks.py:7-103) for the hot configuration: 16-byte aligned rows, no bias, no
// dropout, head_dim tile 64 or 128.  Everything else keeps using fwd_kernel.h.
//
// Why a second kernel: at two waves per SIMD (fwd_kernel.h) each wave runs QK^T -> softmax ->
// PV as one dependent chain, and the SIMD only overlaps one wave's softmax VALU with the other
// wave's MFMAs when the hardware happens to interleave them.  Here a workgroup is 4 waves (one
// per SIMD, up to 512 registers each) and each wave owns two independent 32-row halves A and B
// whose chains are offset by half a tile, so every phase pairs one half's MFMAs with the other
// half's softmax VALU inside ONE instruction stream:
//
//   phase 1:  S_A(i)  = K_i Q_A^T        (16 MFMA)  ||  softmax_B(i-1), slots 16-31
//   phase 2:  O_B    += V_{i-1}^T P_B^T   (16 MFMA)  ||  softmax_A(i),   slots 0-15
//   phase 3:  S_B(i)  = K_i Q_B^T        (16 MFMA)  ||  softmax_A(i),   slots 16-31
//   phase 4:  O_A    += V_i^T P_A^T       (16 MFMA)  ||  softmax_B(i),   slots 0-15
//
// A phase is a sequence of steps fenced by sched_barrier(0), so the schedule is the source
// order: each step issues one MFMA, the fragment read kLead MFMAs ahead, one slot of the
// softmax software pipeline and (phases 1-2) one LDS-DMA piece of the next K/V tile.
//
// Softmax without waiting for the row max ("speculative defer-max"): the exponentials of a
// tile are computed against the running reference m_use (the stale max), element by element
// in a pipeline whose stages (mask select, scale-and-subtract, exp2 + max, sum + bf16 pack)
// are one slot apart, so no VALU op waits on its producer.  The tile's max is only checked at
// the end: if some row grew past m_use + kDeferMax (first tile of a row, rare afterwards) a
// slow path recomputes that tile's P from the kept scaled scores and rescales O and l.
//
// K tiles are double buffered and V tiles triple buffered in LDS (V_{i-1} is still read in
// tile i), with one barrier per tile.  Causal / key-tail masks are applied only in the tiles
// that cross a row's limit (a separate loop body).
#pragma once
#include <type_traits>

#include "common.h"

namespace fa2 {

#ifndef FA2_ABL
#define FA2_ABL 0  // timing ablations: 1 = no softmax fillers, 2 = no K/V prefetch
#endif
#ifndef FA2_LEAD
#define FA2_LEAD 4  // fragment reads in flight ahead of their MFMA
#endif

template <bool BF16, int DT, bool CAUSAL>
__global__ void __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) fwd_w64_kernel(const fa2_fwd_args p) {
  using E = Elem<BF16>;
  constexpr int NT = 256;
  constexpr int BM = 256;            // query rows per workgroup (64 per wave)
  constexpr int BN = 64;             // keys per tile
  constexpr int KS = DT / 16;        // k-steps of Q K^T
  constexpr int NDT = DT / 32;       // 32-wide d tiles of O
  constexpr int TILE = BN * DT * 2;  // bytes per K (or V) tile
  __shared__ __attribute__((aligned(16))) char smem[5 * TILE];  // K0 K1 V0 V1 V2

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r32 = lane & 31, hh = lane >> 5;

  // ---- work item (as fwd_kernel.h) ----------------------------------------------------------
  const int nmb = (p.seqlen_q + BM - 1) / BM;
  const int item = xcd_item(blockIdx.x, gridDim.x);
  const int bh = item / nmb;
  const int mbi = item - bh * nmb;
  const int mb = CAUSAL ? (nmb - 1 - mbi) : mbi;
  const int b = bh / p.heads_q, hq = bh - b * p.heads_q;
  const int hkv = hq / (p.heads_q / p.heads_kv);
  int Lq = p.seqlen_q, Lk = p.seqlen_k;  // varlen: padded [B, S, H, D] rows, valid prefix
  if (p.cu_seqlens) Lq = Lk = p.cu_seqlens[b + 1] - p.cu_seqlens[b];
  const int m0 = mb * BM;
  const int qw0 = m0 + w * 64;  // first row of this wave; half h owns rows qw0 + 32 h + r32
  const int D = p.head_dim;
  const int diag = Lk - Lq;     // key j visible to query i iff j <= i + diag

  const uint16_t* qg = (const uint16_t*)p.q + b * p.q_stride[0] + hq * p.q_stride[2];
  const uint16_t* kg = (const uint16_t*)p.k + b * p.k_stride[0] + hkv * p.k_stride[2];
  const uint16_t* vg = (const uint16_t*)p.v + b * p.v_stride[0] + hkv * p.v_stride[2];

  int n_end = 0;  // key range of the workgroup
  if (m0 < Lq) {
    n_end = Lk;
    if (CAUSAL) n_end = min(Lk, m0 + BM + diag);
    n_end = max(n_end, 0);
  }
  const int ntiles = (n_end + BN - 1) / BN;
  // tiles [0, n_int) are fully visible to every row of the workgroup: no masks
  int n_int = CAUSAL ? min(Lk, m0 + diag + 1) : Lk;
  n_int = min(max(n_int, 0) / BN, ntiles);

  auto kt = [&](int i) { return smem + (i & 1) * TILE; };
  auto vt = [&](int i) { return smem + (2 + i % 3) * TILE; };
  Stager<DT, BN, NT> kst, vst;
  kst.init(tid, p.k_stride[1], D);
  vst.init(tid, p.v_stride[1], D);
  auto stage = [&](int i) {
    kst.issue(kt(i), kg, p.k_stride[1], i * BN, Lk, tid);
    vst.issue(vt(i), vg, p.v_stride[1], i * BN, Lk, tid);
  };
  if (ntiles > 0) stage(0);

  // ---- Q fragments (B operand of S^T = K Q^T) -------------------------------------------------
  u32x4 qf[2][KS];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int qi = qw0 + 32 * h + r32;
    const bool qvalid = qi < Lq;
    const uint16_t* qrow = qg + (int64_t)(qvalid ? qi : 0) * p.q_stride[1];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[h][ks] = load_row_frag<true>(qrow, 16 * ks + 8 * hh, D, qvalid);
  }

  const float sc = p.softmax_scale * kLog2e;  // x = s * sc - m_use; p = exp2(x)
  f32x16 acc[2][NDT];
  f32x16 s[2][2];     // raw scores S^T of the half's current tile (MFMA accumulators)
  u32x4 pf[2][2][2];  // bf16/fp16 P: B operand of O^T += V^T P^T
  float m_run[2], m_use[2], l_run[2], rs[2], mxc[2][2], pt[2][32], x[2][32];
  int lim[2];         // per-lane key limit of half h: key kj visible iff kj < lim
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) acc[h][dt] = zero16();
    m_run[h] = kNegInf;
    m_use[h] = 0.f;
    l_run[h] = 0.f;
    const int qi = qw0 + 32 * h + r32;
    lim[h] = CAUSAL ? min(Lk, qi + diag + 1) : Lk;
  }

  // ---- steps -------------------------------------------------------------------------------
  constexpr int kLead = FA2_LEAD;
  constexpr int NQK = 2 * KS;   // QK^T steps: (t = m & 1, ks = m >> 1), two independent chains
  constexpr int NPV = 4 * NDT;  // PV steps: (dt = m % NDT, kk = m / NDT), NDT chains
  static_assert(NQK == NPV, "a softmax half spans one QK and one PV phase of equal length");
  constexpr int NSTEP = NQK;
  constexpr int SPS = 32 / (2 * NSTEP);  // softmax slots per step
  constexpr int kSlots = 32 + 4;        // 32 elements, pipeline depth 5

  // element e of a half: t = e >> 4, i = e & 15 -> key n0 + 32 t + (i & 3) + 8 (i >> 2) + 4 hh
  // softmax slot j of half h, one stage per slot so no op waits on its producer:
  //   x = s*sc - m_use (e = j - 1) | mask select (MASK, e = j - 2) | max + exp2 (e = j - 3) |
  //   row sum + pack (e = j - 4).  x (scaled scores) is kept for the slow path.
  auto slot = [&](auto mask_c, int h, int rel, int j) {
    constexpr bool MASK = decltype(mask_c)::value;
    if (j == 0) {
      mxc[h][0] = mxc[h][1] = kNegInf;
      rs[h] = 0.f;
    }
    const int e1 = j - 1, e2 = j - 2, e3 = j - 3, e4 = j - 4;
    if (e1 >= 0 && e1 < 32) x[h][e1] = fmaf(x[h][e1], sc, -m_use[h]);
    if (MASK && e2 >= 0 && e2 < 32) {
      const int o = 32 * (e2 >> 4) + (e2 & 3) + 8 * ((e2 & 15) >> 2);
      x[h][e2] = o < rel ? x[h][e2] : kNegInf;
    }
    if (e3 >= 0 && e3 < 32) {
      if (e3 & 1) mxc[h][(e3 >> 1) & 1] = fmaxf(mxc[h][(e3 >> 1) & 1], fmaxf(x[h][e3 - 1], x[h][e3]));
      pt[h][e3] = __builtin_amdgcn_exp2f(x[h][e3]);
    }
    if (e4 >= 0 && e4 < 32) {
      rs[h] += pt[h][e4];
      if (e4 & 1) pf[h][e4 >> 4][(e4 >> 3) & 1][(e4 & 7) >> 1] = E::pack2(pt[h][e4 - 1], pt[h][e4]);
    }
  };
  // slots of step m of a half's first (FIRST_PHASE) or second phase
  auto slots = [&](auto mask_c, int h, int rel, bool second, int m) {
#pragma unroll
    for (int u = 0; u < SPS; ++u) {
      const int j = (second ? NSTEP * SPS : 0) + m * SPS + u;
      slot(mask_c, h, rel, j);
      if (second && m == NSTEP - 1 && u == SPS - 1)
#pragma unroll
        for (int jj = 32; jj < kSlots; ++jj) slot(mask_c, h, rel, jj);
    }
  };
  // end of a half's tile: keep the pipeline's outputs in this block, then check the max
  auto finish = [&](int h) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) asm volatile("" : "+v"(pf[h][t][sp]));
    asm volatile("" : "+v"(rs[h]), "+v"(mxc[h][0]), "+v"(mxc[h][1]));
    const float mx = half_max(fmaxf(mxc[h][0], mxc[h][1]));  // max of x over the row
    const bool ok = m_run[h] > kNegInf ? mx <= kDeferMax : mx == kNegInf;
#ifdef FA2_NOSLOW
    if (true) {
#else
    if (__all(ok)) {
#endif
      l_run[h] += rs[h];
    } else {
      // slow path: move the reference to the new max, recompute this tile's P from x
      // (the empty asm keeps this block a real branch: if-converted, its 32 exp2 would run
      // on every tile)
      asm volatile("" ::: "memory");
      const float m_new = fmaxf(m_run[h], mx + m_use[h]);
      const float mu = m_new == kNegInf ? 0.f : m_new;
      const float alpha = __builtin_amdgcn_exp2f(m_run[h] - mu);
      const float dm = m_use[h] - mu;
      float r = 0.f;
#pragma unroll
      for (int e = 0; e < 32; e += 2) {
        const float p0 = __builtin_amdgcn_exp2f(x[h][e] + dm), p1 = __builtin_amdgcn_exp2f(x[h][e + 1] + dm);
        r += p0 + p1;
        pf[h][e >> 4][(e >> 3) & 1][(e & 7) >> 1] = E::pack2(p0, p1);
      }
      l_run[h] = l_run[h] * alpha + r;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[h][dt][i] *= alpha;
      m_run[h] = m_new;
      m_use[h] = mu;
    }
  };

  // next tile's K/V pieces, spread over phases 1 (K) and 2 (V)
  constexpr int kPcs = Stager<DT, BN, NT>::kIters;
  const char* kbuf;
  const char* vbuf;
  const uint16_t *kgt, *vgt;
  int64_t kadj, vadj;
  auto dma = [&](bool vphase, int m) {
    constexpr int every = NSTEP / kPcs;
    if (m % every == 1) {
      const int it = m / every;
      if (vphase) vst.piece((char*)vbuf, vgt, vadj, it);
      else kst.piece((char*)kbuf, kgt, kadj, it);
    }
  };

  // S^T of half h for the tile in K, with fill(m) after step m's MFMA
  auto qk_phase = [&](int h, const char* K, auto fill) {
    u32x4 kf[NQK];
#pragma unroll
    for (int j = 0; j < kLead && j < NQK; ++j) kf[j] = lds_row_frag<DT, BN>(K, 32 * (j & 1), r32, j >> 1, hh);
    s[h][0] = zero16();
    s[h][1] = zero16();
#pragma unroll
    for (int m = 0; m < NQK; ++m) {
      if (m + kLead < NQK) kf[m + kLead] = lds_row_frag<DT, BN>(K, 32 * ((m + kLead) & 1), r32, (m + kLead) >> 1, hh);
      s[h][m & 1] = E::mfma(kf[m], qf[h][m >> 1], s[h][m & 1]);
#if !(FA2_ABL & 1)
      fill(m);
#endif
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int e = 0; e < 32; ++e) x[h][e] = s[h][e >> 4][e & 15];  // scalars: updated in place
  };
  // O^T of half h += V^T P^T for the tile in V
  auto pv_phase = [&](int h, const char* V, auto fill) {
    u32x4 vf[NPV];
    auto rd = [&](int m) { return lds_tr_frag<DT, BN>(V, 16 * (m / NDT), 32 * (m % NDT), lane); };
#pragma unroll
    for (int j = 0; j < kLead && j < NPV; ++j) vf[j] = rd(j);
#pragma unroll
    for (int m = 0; m < NPV; ++m) {
      if (m + kLead < NPV) vf[m + kLead] = rd(m + kLead);
      const int dt = m % NDT, kk = m / NDT;
      acc[h][dt] = E::mfma(vf[m], pf[h][kk >> 1][kk & 1], acc[h][dt]);
#if !(FA2_ABL & 1)
      fill(m);
#endif
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  __builtin_amdgcn_s_waitcnt(0);  // prologue: Q fragments (compiler-tracked) + first tile
  __syncthreads();

  int relB = 0;  // mask limit of half B relative to its current tile
  // one tile: FIRST = no pending half-B work of a previous tile; MASK = tile i crosses a limit;
  // PMASK = the previous tile did (its half B still has slots 16-31 to run)
  auto tile = [&](auto first_c, auto mask_c, auto pmask_c, int i) {
    constexpr bool FIRST = decltype(first_c)::value;
    const int n0 = i * BN;
    const int relA = lim[0] - n0 - 4 * hh;
    const int relBp = relB;  // half B of tile i-1 still runs slots 16+ in phase 1
    relB = lim[1] - n0 - 4 * hh;
    // the next tile's DMA targets buffers last read in tile i-1 (rows clamped past the end)
    kbuf = kt(i + 1);
    vbuf = vt(i + 1);
    kgt = kg + (int64_t)(n0 + BN) * p.k_stride[1];
    vgt = vg + (int64_t)(n0 + BN) * p.v_stride[1];
    kadj = kst.row_adjust(p.k_stride[1], n0 + BN, Lk, tid);
    vadj = vst.row_adjust(p.v_stride[1], n0 + BN, Lk, tid);
    __builtin_amdgcn_sched_barrier(0);
    // phase 1: S_A(i) || softmax_B(i-1) slots 16-31
    qk_phase(0, kt(i), [&](int m) {
#if !(FA2_ABL & 2)
      dma(false, m);
#endif
      if constexpr (!FIRST) slots(pmask_c, 1, relBp, true, m);
    });
    if constexpr (!FIRST) finish(1);
    __builtin_amdgcn_sched_barrier(0);
    // phase 2: O_B += V_{i-1}^T P_B^T || softmax_A(i) slots 0-15
    auto f2 = [&](int m) {
#if !(FA2_ABL & 2)
      dma(true, m);
#endif
      slots(mask_c, 0, relA, false, m);
    };
    if constexpr (FIRST) {
#pragma unroll
      for (int m = 0; m < NPV; ++m) {
        f2(m);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
      pv_phase(1, vt(i - 1), f2);
    }
    // phase 3: S_B(i) || softmax_A(i) slots 16-31
    qk_phase(1, kt(i), [&](int m) { slots(mask_c, 0, relA, true, m); });
    finish(0);
    __builtin_amdgcn_sched_barrier(0);
    // phase 4: O_A += V_i^T P_A^T || softmax_B(i) slots 0-15
    pv_phase(0, vt(i), [&](int m) { slots(mask_c, 1, relB, false, m); });
    vm_wait_all();
    __syncthreads();
  };

  if (ntiles > 0) {
    using T = std::true_type;
    using F = std::false_type;
    if (n_int > 0) tile(T{}, F{}, F{}, 0);
    else tile(T{}, T{}, F{}, 0);
    int i = 1;
    for (; i < n_int; ++i) tile(F{}, F{}, F{}, i);
    if (i < ntiles && i > 0) {  // first masked tile after interior ones
      if (n_int > 0) tile(F{}, T{}, F{}, i);
      else tile(F{}, T{}, T{}, i);
      ++i;
    }
    for (; i < ntiles; ++i) tile(F{}, T{}, T{}, i);
    // drain: half B of the last tile
    const bool lastmask = ntiles > n_int;
#pragma unroll
    for (int m = 0; m < NSTEP; ++m) {
      if (lastmask) slots(T{}, 1, relB, true, m);
      else slots(F{}, 1, relB, true, m);
    }
    finish(1);
    pv_phase(1, vt(ntiles - 1), [](int) {});
  }

  // ---- epilogue --------------------------------------------------------------------------------
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int qi = qw0 + 32 * h + r32;
    const float l_tot = half_sum(l_run[h]);
    const bool row_ok = qi < Lq && l_tot > 0.f;
    const float inv = row_ok ? 1.f / l_tot : 0.f;
    if (hh == 0 && qi < p.lse_row_stride) {
      float* lrow = p.lse + (int64_t)bh * p.lse_row_stride;
      lrow[qi] = row_ok ? m_run[h] + __log2f(l_tot) : kNegInf;
    }
    if (qi < p.seqlen_q) {
      uint16_t* orow = (uint16_t*)p.o + b * p.o_stride[0] + hq * p.o_stride[2] + (int64_t)qi * p.o_stride[1];
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int d0 = 32 * dt + 8 * g4 + 4 * hh;
          const float o0 = acc[h][dt][4 * g4 + 0] * inv, o1 = acc[h][dt][4 * g4 + 1] * inv;
          const float o2 = acc[h][dt][4 * g4 + 2] * inv, o3 = acc[h][dt][4 * g4 + 3] * inv;
          if (d0 < D) *(u32x2*)(orow + d0) = u32x2{E::pack2(o0, o1), E::pack2(o2, o3)};
        }
    }
  }
}

template <bool BF16, int DT, bool CAUSAL>
static hipError_t launch_fwd_w64(const fa2_fwd_args& a, hipStream_t st) {
  dim3 grid(((a.seqlen_q + 255) / 256) * a.batch * a.heads_q);
  hipLaunchKernelGGL((fwd_w64_kernel<BF16, DT, CAUSAL>), grid, dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace fa2
