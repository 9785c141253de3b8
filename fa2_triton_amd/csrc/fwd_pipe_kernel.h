// fwd_pipe_kernel.h -- software-pipelined FlashAttention-2 forward for gfx950 (the hot path:
// aligned head dim, no bias, no dropout).  Same semantics as fwd_kernel (fwd_kernel.h) and the
// reference's _fwd_kernel / compute_row_block (/root/reference/src/forward/kernel.py:61-291,
// /root/reference/src/forward/compute_row_blocks.py:7-103).
//
// Work decomposition as fwd_kernel's causal path: 4 waves x 32 query rows per workgroup, two
// workgroups per CU, 64-key K/V tiles double buffered in LDS by LDS-DMA, one barrier per tile.
//
// What is different is the order of work inside a wave.  fwd_kernel runs
//   QK^T(i) -> softmax(i) -> PV(i)
// so a wave's softmax (~110 VALU ops, 32 of them v_exp) has no MFMA of its own to hide behind.
// Here the wave keeps the raw scores of the NEXT tile in registers and every iteration runs two
// fenced phases:
//   phase X: QK^T(i+1) MFMAs, each step carrying two exponentials, the row-sum adds and one
//            bf16 pack of softmax(i), plus one LDS-DMA piece every other step;
//   phase Y: PV(i) MFMAs, each step carrying one v_max3 of the row max of S(i+1).
// The defer-max decision for tile i+1 (one wave vote) and the rare O rescale sit between
// iterations.  The LDS schedule shifts K by one tile: iteration i reads K(i+1) and V(i) while
// K(i+2) and V(i+1) land in the buffers K(i) and V(i-1) vacated in iteration i-1.
#pragma once
#include <type_traits>

#include "common.h"

namespace fa2 {

// NW = 4: two independent workgroups per CU; NW = 8 (one workgroup of 256 rows per CU, the two
// waves of a SIMD sharing every K/V tile) measured neutral to -1 % and is kept for A/Bs.
// BIASK = 16 / 17: an additive fp16 / bf16 bias with 16-byte aligned rows.  Each wave stages its
// own [32 rows x 64 keys] bias tile by LDS-DMA (4 KiB, single buffered, wave-private: no barrier
// involved): the pieces of tile i+1 go out first in phase X(i), and phase Y(i) waits for them
// with a counted vmcnt that leaves the period's K/V pieces in flight.  The bias enters the scores
// in phase Y, x = s scale + b (natural units), z = x log2(e) - m_ref, as the reference adds it
// before the softmax (/root/reference/src/forward/compute_row_blocks.py:58-66).
// Occupancy: two workgroups per CU (<= 256 VGPRs); three for the non-causal D <= 64 forward
// without bias (<= 168 VGPRs, 96 KiB of LDS), where the softmax VALU per MFMA doubles and the
// third wave per SIMD pays: a 176-VGPR build (two waves) ran cfg2 10 % slower (profiles/
// r03_ab_fwd_handoff.txt).  The causal D = 64 kernel spills at 168 and keeps two.
template <bool BF16, int DT, bool CAUSAL, int NW, int BIASK>
__global__ void __launch_bounds__(NW * 64, DT <= 64 && !CAUSAL && NW == 4 && BIASK == 0 ? 3 : 2)
    fwd_pipe_kernel(const fa2_fwd_args p) {
  using E = Elem<BF16>;
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  constexpr bool BIAS = BIASK != 0;
  constexpr int NKB = 2, NVB = 2;  // K, V tile buffers
  constexpr int NT = NW * 64;
  constexpr int BM = NW * 32;        // query rows per workgroup
  constexpr int BN = 64;             // keys per tile
  constexpr int KS = DT / 16;        // k-steps of Q K^T
  constexpr int NDT = DT / 32;       // 32-wide d tiles of O
  constexpr int NQK = 2 * KS;        // QK^T MFMA steps per tile (two 32-key halves)
  constexpr int NPV = 4 * NDT;       // PV MFMA steps per tile
  constexpr int EPS = 32 / NQK;      // exponentials per QK^T step
  constexpr int TILE = BN * DT * 2;  // bytes per K (or V) tile
  constexpr int LEAD = 3;            // fragment reads in flight ahead of their MFMA
  constexpr int BTILE = BIAS ? kBiasTile : 0;  // bytes per wave's bias tile ([32 rows][BN keys], 16-bit)
  __shared__ __attribute__((aligned(16))) char smem[(NKB + NVB) * TILE + NW * BTILE];  // K, V, bias tiles
  static_assert(NQK % 8 == 0 && 32 % NQK == 0, "QK^T steps must carry whole pack pairs");

  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: scalar branches

  // ---- work items -------------------------------------------------------------------------
  // Head-major per XCD (xcd_item), heaviest first.  Under a causal mask each workgroup runs a
  // mirrored pair of row blocks of one head, nmb-1-j then j (equal causal work per workgroup,
  // half the workgroup launches; the second item starts after a barrier).
  const int nmb = (p.seqlen_q + BM - 1) / BM;
  constexpr bool PAIR = CAUSAL;
  const int per_bh = PAIR ? (nmb + 1) / 2 : nmb;
  const int item = xcd_item(blockIdx.x, gridDim.x);
  const int bh = item / per_bh;
  const int mbi = item - bh * per_bh;
  const int nrep = PAIR && nmb - 1 - mbi != mbi ? 2 : 1;
  for (int rep = 0; rep < nrep; ++rep) {
  if (rep > 0) __syncthreads();  // every wave is past the first item's LDS epilogue
  // lane-dependent values from an opaque copy of the thread id per item: nothing per-lane (the
  // DMA offsets above all) is hoisted out of the item loop and kept live across both items
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int lane = tid & 63, r32 = lane & 31, hh = lane >> 5;
  const int mb = PAIR ? (rep == 0 ? nmb - 1 - mbi : mbi) : (CAUSAL ? (nmb - 1 - mbi) : mbi);
  const int b = bh / p.heads_q, hq = bh - b * p.heads_q;
  const int hkv = hq / (p.heads_q / p.heads_kv);
  int Lq = p.seqlen_q, Lk = p.seqlen_k;
  if (p.cu_seqlens) {
    const int cu = p.cu_seqlens[b];
    Lq = Lk = p.cu_seqlens[b + 1] - cu;
  }
  const int m0 = mb * BM;
  // 8 waves: the waves sharing a SIMD (w, w + 4) take alternate 32-row blocks, so both see the
  // same causal extent
  const int qw0 = m0 + 32 * (NW == 8 ? 2 * (w & 3) + (w >> 2) : w);  // first row of this wave
  const int qi = qw0 + r32;     // this lane's query row
  const int D = p.head_dim;

  const uint16_t* qg = (const uint16_t*)p.q + b * p.q_stride[0] + hq * p.q_stride[2];
  const uint16_t* kg = (const uint16_t*)p.k + b * p.k_stride[0] + hkv * p.k_stride[2];
  const uint16_t* vg = (const uint16_t*)p.v + b * p.v_stride[0] + hkv * p.v_stride[2];

  int n_end = 0;
  if (m0 < Lq) {
    n_end = Lk;
    if (CAUSAL) n_end = min(Lk, m0 + BM + Lk - Lq);
    n_end = max(n_end, 0);
  }
  const int ntiles = (n_end + BN - 1) / BN;
  const int diag = Lk - Lq;  // key j visible to query i iff j <= i + diag

  auto kt = [&](int t) { return smem + (t & 1) * TILE; };                       // buffer of K tile t
  auto vt = [&](int t) { return smem + (NKB + (t & 1)) * TILE; };                // buffer of V tile t
  char* const bw = smem + (NKB + NVB) * TILE + w * BTILE;  // this wave's bias tile
  BufStager<DT, BN, NT> kst;  // K and V share row strides (checked by the launcher): one offset set
  kst.init(tid, p.k_stride[1], D);
  const int mrows = BufStager<DT, BN, NT>::max_rows(p.k_stride[1]);
  // this wave's bias tiles: [32 rows from qw0][BN keys], row stride bias_stride[2] (16-byte
  // aligned rows, checked by the launcher); rows past seqlen_q read as zeros, keys past seqlen_k
  // are masked
  using BiasStager = BufStager<BN, 32, 64>;
  BiasStager bst;
  const uint16_t* bg = nullptr;
  int brows = 0;
  if constexpr (BIAS) {
    bst.init(lane, p.bias_stride[2], BN);
    brows = BiasStager::max_rows(p.bias_stride[2]);
    bg = (const uint16_t*)p.bias + b * p.bias_stride[0] + hq * p.bias_stride[1];
  }
  auto bias_issue = [&](int t) {
    if constexpr (BIAS) {
      const i32x4 r = bias_tile_rsrc(bg + t * BN, p.bias_stride[2], qw0, p.seqlen_q, brows, p.seqlen_k - t * BN, BN);
#pragma unroll
      for (int it = 0; it < BiasStager::kIters; ++it) bst.piece(bw, r, it);
    }
  };
  if (ntiles > 0) {
    kst.issue(kt(0), kg, p.k_stride[1], 0, Lk, mrows);
    kst.issue(vt(0), vg, p.v_stride[1], 0, Lk, mrows);
    if (ntiles > 1) kst.issue(kt(1), kg, p.k_stride[1], BN, Lk, mrows);
    bias_issue(0);
  }

  // ---- Q fragments (B operand of S^T = K Q^T) ------------------------------------------------
  u32x4 qf[KS];
  {
    const bool qvalid = qi < Lq;
    const uint16_t* qrow = qg + (int64_t)(qvalid ? qi : 0) * p.q_stride[1];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = load_row_frag<true>(qrow, 16 * ks + 8 * hh, D, qvalid);
  }

  const float sc = p.softmax_scale * kLog2e;
  // Scores enter the softmax as x = score(s) in units of uz: the raw s in units of scale log2(e)
  // without a bias; x = s scale + b in natural units (uz = log2(e)) with one.  The exponent
  // argument is z = x uz - m_ref, the running max is kept in log2 units.
  const float uz = BIAS ? kLog2e : sc;
  float m_run = kNegInf, l_run = 0.f;
  float m_ref = 0.f;  // the max the stored exponent arguments are relative to (0 while m_run = -inf)
  f32x16 acc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) acc[dt] = zero16();

  // per-lane key limit: key kj is visible to this lane's row iff kj < lim_lane
  const int lim_lane = CAUSAL ? min(Lk, qi + diag + 1) : Lk;
  // wave-uniform tile classes
  auto tile_live = [&](int t) { return t < ntiles && !(CAUSAL && t * BN > qw0 + 31 + diag); };
  auto tile_mask = [&](int t) { return (t * BN + BN > Lk) || (CAUSAL && t * BN + BN - 1 > qw0 + diag); };

  f32x16 s[2];   // raw scores S^T of the tile whose softmax is next
  float mx = kNegInf;  // their (masked) row max, both lane halves combined, times sc
  u32x4 pf[2][2];      // P of the current tile, packed: B operand of O^T += V^T P^T

  // bias of tile t for this lane (register i of half h: key 32 h + (i & 3) + 8 (i >> 2) + 4 hh of
  // row qi): group g = i >> 2 of half h is one 8-byte read of the staged tile
  auto bias_frag = [&](int h, int g) -> u32x2 {  // (of the tile in this wave's buffer)
    if constexpr (BIAS) return bias_tile_frag(bw, r32, hh, h, g);
    else return u32x2{0u, 0u};
  };
  auto bias_val = [&](u32x2 bv, int j) -> float { return bias_elem<BIASK>(bv, j); };
  // score(s) with the bias of tile t added (BIAS), in place, then masked (MASK: keys >= rel)
  auto add_bias = [&](f32x16* v) {
    if constexpr (BIAS) {
      const float scale = p.softmax_scale;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const u32x2 bv = bias_frag(h, g);
#pragma unroll
          for (int j = 0; j < 4; ++j) v[h][4 * g + j] = fmaf(v[h][4 * g + j], scale, bias_val(bv, j));
        }
    }
  };
  // masked scores + row max (register i of half t holds key n0 + 32 t + (i & 3) + 8 (i >> 2) + 4 hh)
  auto mask_max = [&](int n0) {
    add_bias(s);
    const int rel = lim_lane - n0 - 4 * hh;
    float m = kNegInf;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int o = 32 * t + (i & 3) + 8 * (i >> 2);
        s[t][i] = o < rel ? s[t][i] : kNegInf;
        m = fmaxf(m, s[t][i]);
      }
    mx = half_max(m) * uz;
  };
  auto plain_max = [&]() {
    add_bias(s);
    float m0_ = kNegInf, m1_ = kNegInf;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      m0_ = fmaxf(m0_, s[0][i]);
      m1_ = fmaxf(m1_, s[1][i]);
    }
    mx = half_max(fmaxf(m0_, m1_)) * uz;
  };
  auto kfrag = [&](const char* K, int m) { return lds_row_frag<DT, BN>(K, 32 * (m & 1), r32, m >> 1, hh); };
  auto vfrag = [&](const char* V, int m) { return lds_tr_frag<DT, BN>(V, 16 * (m / NDT), 32 * (m % NDT), lane); };

  // QK^T of one tile into s (no interleaved work)
  auto qk_plain = [&](const char* K) {
    u32x4 kf[NQK];
#pragma unroll
    for (int j = 0; j < LEAD; ++j) kf[j] = kfrag(K, j);
    s[0] = zero16();
    s[1] = zero16();
#pragma unroll
    for (int m = 0; m < NQK; ++m) {
      if (m + LEAD < NQK) kf[m + LEAD] = kfrag(K, m + LEAD);
      s[m & 1] = E::mfma(kf[m], qf[m >> 1], s[m & 1]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // Defer-max decision for the tile whose exponent arguments z = x uz - m_ref sit in z[].
  // Usually the running max stays (m_use == m_ref) and z is final; when some row of the wave
  // outgrew it by more than kDeferMax, O and l are rescaled and z shifted (rare: first tiles).
  auto softmax_begin = [&](f32x16* z) {
    const bool rescale = !__all(mx - m_run <= kDeferMax);
    if (rescale) {
      const float m_new = fmaxf(m_run, mx);
      const float m_use = m_new == kNegInf ? 0.f : m_new;
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_use);
      const float shift = m_use - m_ref;
      l_run *= alpha;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[dt][i] *= alpha;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) z[t][i] -= shift;
      m_run = m_new;
      m_ref = m_use;
    }
  };
  // exponent arguments of the scores in v (in place), relative to the current reference max
  auto to_z = [&](f32x16* v) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) v[t][i] = fmaf(v[t][i], uz, -m_ref);
  };

  // exponentials e..e+1 of the flat 32-score list -> P, row-sum partials
  auto exp_pair = [&](const f32x16* src, int e, float& rs0, float& rs1) {
    const int t = e >> 4, i = e & 15;
    const float p0 = __builtin_amdgcn_exp2f(src[t][i]);
    const float p1 = __builtin_amdgcn_exp2f(src[t][i + 1]);
    rs0 += p0;
    rs1 += p1;
    pf[t][i >> 3][(i & 7) >> 1] = E::pack2(p0, p1);
  };

  __builtin_amdgcn_s_waitcnt(0);  // Q fragments + K0, V0, K1 (+ bias 0, 1)
  __syncthreads();

  constexpr int kPieces = BufStager<DT, BN, NT>::kIters;  // LDS-DMA ops per thread per K/V tile
  // DMA pieces of a period (K and V; one barrier per tile) ride in phase X
  constexpr int kPerX = 2 * kPieces;
  constexpr int kEveryX = NQK / kPerX > 0 ? NQK / kPerX : 1;

  // Rows past the end read as zeros (buffer range check); tiles wholly past it land in buffers
  // nobody reads again.
  auto dma_k = [&](int t, int pc) {
    kst.piece(kt(t), BufStager<DT, BN, NT>::tile_rsrc(kg, p.k_stride[1], t * BN, Lk, mrows), pc);
  };
  auto dma_v = [&](int t, int pc) {
    kst.piece(vt(t), BufStager<DT, BN, NT>::tile_rsrc(vg, p.v_stride[1], t * BN, Lk, mrows), pc);
  };
  // One-barrier schedule, period i: K(i+2) -> the buffer of K(i), V(i+1) -> that of V(i-1).
  auto dma = [&](int i, int pc) {
    if (pc < kPieces) dma_k(i + 2, pc);
    else dma_v(i + 1, pc - kPieces);
  };
  // prologue: S(0)
  if (tile_live(0)) {
    qk_plain(kt(0));
    if (tile_mask(0)) mask_max(0);
    else plain_max();
    to_z(s);
  }
  __syncthreads();  // every wave is done with K(0) before K(2) lands in its buffer

  // Phase X(i): softmax(i) of the exponent arguments in cur, QK^T(i+1) into nxt when QK (tile
  // i+1 live for this wave), with the period's DMA pieces when DMA.  One key half after the
  // other (nxt[0]: steps 0..KS-1, nxt[1]: KS..2KS-1) while the exponentials consume cur[0] then
  // cur[1]: 48 score registers live at any step, not 64.
  auto phase_x = [&](int i, f32x16* cur, f32x16* nxt, auto qk_c) {
    constexpr bool QK = decltype(qk_c)::value;
    const char* K1 = kt(i + 1);
    if constexpr (QK) bias_issue(i + 1);  // (this wave read bias tile i in phase Y(i-1))
    softmax_begin(cur);
    float rs0 = 0.f, rs1 = 0.f;
    u32x4 kf[NQK];
    auto kfs = [&](int m) { return kfrag(K1, 2 * (m % KS) + m / KS); };
    if constexpr (QK) {
#pragma unroll
      for (int j = 0; j < LEAD; ++j) kf[j] = kfs(j);
    }
#pragma unroll
    for (int m = 0; m < NQK; ++m) {
      if constexpr (QK) {
        if (m + LEAD < NQK) kf[m + LEAD] = kfs(m + LEAD);
        const int t = m / KS, ks = m % KS;
        nxt[t] = E::mfma(kf[m], qf[ks], ks == 0 ? zero16() : nxt[t]);
      }
#pragma unroll
      for (int e = 0; e < EPS; e += 2) exp_pair(cur, m * EPS + e, rs0, rs1);
      // the row-sum adds stay in this step: left alone, the compiler moves all 32 to the end of the
      // phase as two serial chains beside the last MFMA (sched_barrier does not bind that motion)
      asm volatile("" : "+v"(rs0), "+v"(rs1));
      if (m % kEveryX == 0 && m / kEveryX < kPerX) dma(i, m / kEveryX);
      __builtin_amdgcn_sched_barrier(0);
    }
    l_run += rs0 + rs1;
  };
  // Phase Y(i): PV(i) with the row max and exponent arguments of S(i+1) in nxt when QK (masked
  // when MASK; bias of tile i+1 added first), one v_max3 per step.
  auto phase_y = [&](int i, f32x16* nxt, auto qk_c, auto mask_c) {
    constexpr bool QK = decltype(qk_c)::value, MASK = decltype(mask_c)::value;
    const char* V0 = vt(i);
    constexpr int L = 2 * LEAD > NPV ? NPV : 2 * LEAD;
    constexpr int PER = 32 / NPV;
    u32x4 vf[NPV];
    float ma = kNegInf, mb_ = kNegInf;
    const int rel = lim_lane - (i + 1) * BN - 4 * hh;
    // bias of tile i+1, one 4-key group per read: key half 0 read up front, half 1 two steps
    // before its first element (fewer registers live than all eight reads at once)
    u32x2 bz[2][4];
    auto read_bias = [&](int h) {
#pragma unroll
      for (int g = 0; g < 4; ++g) bz[h][g] = bias_frag(h, g);
    };
    if constexpr (BIAS && QK) {
      // bias tile i+1 (issued first in phase X(i)) has landed; the period's K/V pieces after it
      // may stay in flight
      if constexpr (kPerX == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else if constexpr (kPerX == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if constexpr (kPerX == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else vm_wait_all();
      read_bias(0);
    }
    const float scale = p.softmax_scale;
#pragma unroll
    for (int j = 0; j < L; ++j) vf[j] = vfrag(V0, j);
#pragma unroll
    for (int m = 0; m < NPV; ++m) {
      if (m + L < NPV) vf[m + L] = vfrag(V0, m + L);
      if constexpr (BIAS && QK) {
        if (m == (NPV / 2 >= 2 ? NPV / 2 - 2 : 0)) read_bias(1);
      }
      const int kk = m / NDT;
      acc[m % NDT] = E::mfma(vf[m], pf[kk >> 1][kk & 1], acc[m % NDT]);
      if constexpr (QK) {
#pragma unroll
        for (int e = m * PER; e < (m + 1) * PER; ++e) {
          const int t = e >> 4, r = e & 15;
          if constexpr (BIAS) nxt[t][r] = fmaf(nxt[t][r], scale, bias_val(bz[t][r >> 2], r & 3));
          if constexpr (MASK) {
            const int o = 32 * t + (r & 3) + 8 * (r >> 2);
            nxt[t][r] = o < rel ? nxt[t][r] : kNegInf;
          }
          float& mm = t ? mb_ : ma;
          mm = fmaxf(mm, nxt[t][r]);
          nxt[t][r] = fmaf(nxt[t][r], uz, -m_ref);
        }
        asm volatile("" : "+v"(ma), "+v"(mb_));  // the row-max chain stays in its steps
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (QK) mx = half_max(fmaxf(ma, mb_)) * uz;
  };
  auto sync = [&]() {
    vm_wait_all();
    __syncthreads();
  };
  auto dma_only = [&](int period) {
#pragma unroll
    for (int pc = 0; pc < kPerX; ++pc) dma(period, pc);
  };
  using T = std::true_type;
  using F = std::false_type;

  // Leading tiles that need no mask for any row of this wave, and its last live tile.  The
  // counts differ between the waves of a workgroup (causal diagonal), so each wave runs its own
  // loops; every period of every loop ends in the same one barrier, and the waves stay in step by
  // period index.
  int n_full = Lk / BN;
  if (CAUSAL) n_full = min(n_full, qw0 + diag + 1 >= 0 ? (qw0 + diag + 1) / BN : 0);
  int last = -1;  // last live tile of this wave
  if (ntiles > 0 && tile_live(0)) {
    last = ntiles - 1;
    if (CAUSAL) last = min(last, (qw0 + 31 + diag) / BN);
  }
  // one period: X(i), Y(i), barrier
  auto step = [&](int i, f32x16* cur, f32x16* nxt, auto qk_c, auto mask_c) {
    phase_x(i, cur, nxt, qk_c);
    phase_y(i, nxt, qk_c, mask_c);
    sync();
  };
  // steady periods (tile i+1 live and unmasked) unrolled by two with the roles of the two score
  // arrays swapped, so no register copies between periods
  f32x16 s2[2];
  const int n_steady = max(0, min(n_full, ntiles) - 1);
  int i = 0;
  for (; i + 1 < n_steady; i += 2) {
    step(i, s, s2, T{}, F{});
    step(i + 1, s2, s, T{}, F{});
  }
  if (i < n_steady) {
    step(i, s, s2, T{}, F{});
    s[0] = s2[0];
    s[1] = s2[1];
    ++i;
  }
  // tail: next tile on the diagonal / key tail (masked), the last live tile (softmax + PV only),
  // then tiles past the diagonal (DMA + barrier only)
  for (; i < last; ++i) {
    step(i, s, s2, T{}, T{});
    s[0] = s2[0];
    s[1] = s2[1];
  }
  if (i == last) {
    step(i, s, s2, F{}, F{});
    ++i;
  }
  for (; i < ntiles; ++i) {
    dma_only(i);
    sync();
  }
  vm_wait_all();

  // ---- epilogue ----------------------------------------------------------------------------
  const float l_tot = half_sum(l_run);
  const bool row_ok = qi < Lq && l_tot > 0.f;
  const float inv = row_ok ? 1.f / l_tot : 0.f;
  if (hh == 0 && qi < p.lse_row_stride) {
    float* lrow = p.lse + (int64_t)bh * p.lse_row_stride;
    lrow[qi] = row_ok ? m_run + __log2f(l_tot) : kNegInf;
  }
  {
    // every wave passed the last tile's barrier: the K/V buffers are free for the staging image
    uint16_t* o0 = (uint16_t*)p.o + b * p.o_stride[0] + hq * p.o_stride[2] + (int64_t)qw0 * p.o_stride[1];
    store_rows_lds<BF16, DT>(smem + w * 32 * DT * 2, acc, inv, row_ok, o0, p.o_stride[1],
                             min(32, p.seqlen_q - qw0), D, lane);
  }
  }
}

template <bool BF16, int DT, bool CAUSAL, int BIASK>
static hipError_t launch_fwd_pipe(const fa2_fwd_args& a, hipStream_t st) {
  constexpr int NW = 4;
  constexpr int BM = NW * 32;
  const int nmb = (a.seqlen_q + BM - 1) / BM;
  dim3 grid((CAUSAL ? (nmb + 1) / 2 : nmb) * a.batch * a.heads_q);
  hipLaunchKernelGGL((fwd_pipe_kernel<BF16, DT, CAUSAL, NW, BIASK>), grid, dim3(NW * 64), 0, st, a);
  return hipGetLastError();
}

}  // namespace fa2
