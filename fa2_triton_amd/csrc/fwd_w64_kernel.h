// fwd_w64_kernel.h -- forward with 64 query rows per wave at one wave per SIMD (gfx950).
// Same semantics as fwd_pipe_kernel (fwd_pipe_kernel.h) and the reference's _fwd_kernel /
// compute_row_block (/root/reference/src/forward/kernel.py:61-291,
// /root/reference/src/forward/compute_row_blocks.py:7-103); no bias, no dropout, aligned D.
//
// Why: fwd_pipe_kernel (32 rows per wave, two waves per SIMD) reads one 1-KiB LDS fragment per
// MFMA and its MFMA -> softmax -> MFMA chains are paced by the partner wave's arbitration.  Here
// each wave owns two 32-row blocks (rb 0, 1) of one 256-row workgroup: every K fragment (Q K^T)
// and every V^T fragment (P V) feeds two MFMAs, one per row block, so a phase is 32 MFMAs of
// independent chains with half the LDS reads, and the softmax VALU of one block sits beside the
// other block's MFMAs.  The register file is the whole 512 of the SIMD lane: O^T (128) and the
// Q fragments (64) live in accumulation registers, owned by inline-asm MFMAs; scores, P and the
// fragments in flight use the architectural registers.
//
// Inline-asm MFMAs are invisible to the compiler's hazard recognizer, so the kernel keeps every
// VALU read of an asm MFMA result structurally far (>= 8 MFMA steps) from the MFMA, and pads
// the few places where that does not hold by construction (prologue scores, rescale, epilogue)
// with explicit s_nop runs between scheduling fences.
//
// Period i (one barrier): phase X = QK^T(i+1) for both row blocks (16 K-fragment steps, 2 MFMAs
// each) beside the exponentials, row sums and packs of tile i and the period's LDS-DMA; phase Y
// = PV(i) (16 V-fragment steps, 2 MFMAs each) beside mask, row max and exponent arguments of
// tile i+1 -- the schedule of fwd_pipe_kernel, doubled in rows.
#pragma once
#include <type_traits>

#include "common.h"

namespace fa2 {

template <bool BF16>
struct AsmMfma;
template <>
struct AsmMfma<true> {
  // c (accumulation registers) += a b
  FA2_DEV static void acc(f32x16& c, u32x4 a, u32x4 b) {
    asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  }
  // d = a b (b in accumulation registers)
  FA2_DEV static f32x16 first(u32x4 a, u32x4 b) {
    f32x16 d;
    asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(d) : "v"(a), "a"(b));
    return d;
  }
  // d += a b (b in accumulation registers)
  FA2_DEV static void next(f32x16& d, u32x4 a, u32x4 b) {
    asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(d) : "v"(a), "a"(b));
  }
};
template <>
struct AsmMfma<false> {
  FA2_DEV static void acc(f32x16& c, u32x4 a, u32x4 b) {
    asm("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  }
  FA2_DEV static f32x16 first(u32x4 a, u32x4 b) {
    f32x16 d;
    asm("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(d) : "v"(a), "a"(b));
    return d;
  }
  FA2_DEV static void next(f32x16& d, u32x4 a, u32x4 b) {
    asm("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(d) : "v"(a), "a"(b));
  }
};

// >= 24 wait states between an asm MFMA's last write and a VALU / accvgpr access of its result
FA2_DEV void mfma_drain() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <bool BF16, int DT, bool CAUSAL>
__global__ void __launch_bounds__(256, 1) fwd_w64_kernel(const fa2_fwd_args p) {
  using M = AsmMfma<BF16>;
  using E = Elem<BF16>;
  constexpr int NW = 4, NT = 256;
  constexpr int BM = NW * 64;        // query rows per workgroup
  constexpr int BN = 64;             // keys per tile
  constexpr int KS = DT / 16;        // k-steps of Q K^T
  constexpr int NDT = DT / 32;       // 32-wide d tiles of O
  constexpr int NQK = 2 * KS;        // K-fragment steps per tile (two 32-key halves)
  constexpr int NPV = 4 * NDT;       // V-fragment steps per tile
  constexpr int TILE = BN * DT * 2;  // bytes per K (or V) tile
  constexpr int LEAD = 3;            // fragment reads in flight ahead of their MFMA
  // LDS: K(2) and V(2) tiles, the unit's Q tile (requested during the previous unit), and each
  // wave's 32-row O staging image: 64 + 64 + 32 KiB at D = 128
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE + BM * DT * 2 + NW * 32 * DT * 2];
  static_assert(NQK == 16 || NQK == 8, "D = 64 or 128");

  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  // ---- persistent work list ----------------------------------------------------------------
  // Items are numbered head-major (causal: mirrored pairs of row blocks nmb-1-j, j of one head);
  // XCD x (workgroups x, x + 8, ...) owns one contiguous slice of the list and its workgroups take
  // every (G/8)-th item of it, so the blocks of a head run together on one XCD's L2.  A *unit* is
  // one 256-row block; the next unit's Q, K(0), K(1), V(0) are requested during the current
  // unit's final period, so no unit after the first waits for its prologue loads.
  const int nmb = (p.seqlen_q + BM - 1) / BM;
  constexpr bool PAIR = CAUSAL;
  const int per_bh = PAIR ? (nmb + 1) / 2 : nmb;
  const int n_items = per_bh * p.batch * p.heads_q;
  const int xcd = blockIdx.x & 7, per = gridDim.x >> 3;
  const int iq = n_items >> 3, ir = n_items & 7;
  const int i_begin = xcd < ir ? xcd * (iq + 1) : ir * (iq + 1) + (xcd - ir) * iq;
  const int i_count = iq + (xcd < ir ? 1 : 0);
  int k_item = blockIdx.x >> 3;  // index in this XCD's slice
  if (k_item >= i_count) return;

  struct Unit {
    int bh, mb, b, hq, Lq, Lk, m0, ntiles;
    const uint16_t *qg, *kg, *vg;
  };
  auto make_unit = [&](int k, int rep) {
    Unit u;
    const int item = i_begin + k;
    u.bh = item / per_bh;
    const int mbi = item - u.bh * per_bh;
    u.mb = PAIR ? (rep == 0 ? nmb - 1 - mbi : mbi) : mbi;
    u.b = u.bh / p.heads_q;
    u.hq = u.bh - u.b * p.heads_q;
    const int hkv = u.hq / (p.heads_q / p.heads_kv);
    u.Lq = p.seqlen_q;
    u.Lk = p.seqlen_k;
    if (p.cu_seqlens) u.Lq = u.Lk = p.cu_seqlens[u.b + 1] - p.cu_seqlens[u.b];
    u.m0 = u.mb * BM;
    int n_end = 0;
    if (u.m0 < u.Lq) {
      n_end = u.Lk;
      if (CAUSAL) n_end = min(u.Lk, u.m0 + BM + u.Lk - u.Lq);
      n_end = max(n_end, 0);
    }
    u.ntiles = (n_end + BN - 1) / BN;
    u.qg = (const uint16_t*)p.q + u.b * p.q_stride[0] + u.hq * p.q_stride[2];
    u.kg = (const uint16_t*)p.k + u.b * p.k_stride[0] + hkv * p.k_stride[2];
    u.vg = (const uint16_t*)p.v + u.b * p.v_stride[0] + hkv * p.v_stride[2];
    return u;
  };
  auto nrep_of = [&](int k) {
    const int mbi = (i_begin + k) % per_bh;
    return PAIR && nmb - 1 - mbi != mbi ? 2 : 1;
  };

  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int D = p.head_dim;
  char* const qs = smem + 4 * TILE;                          // Q tile of the unit (next unit's, late)
  char* const ostage = smem + 4 * TILE + BM * DT * 2 + w * (32 * DT * 2);  // this wave's O staging
  BufStager<DT, BN, NT> kst;  // K and V share row strides (checked by the launcher)
  kst.init(tid, p.k_stride[1], D);
  const int mrows = BufStager<DT, BN, NT>::max_rows(p.k_stride[1]);
  const int qrows = BufStager<DT, BN, NT>::max_rows(p.q_stride[1]);
  // Q tile [BM rows][DT] by LDS-DMA: piece it (0..kQIters-1) of thread tid is row
  // 64 (it % 4) + tid / 4, chunk 4 (it / 4) + ((tid & 3) ^ ((tid >> 4) & 3)) -- one lane offset
  // plus a wave-uniform step (the instruction's immediate offset would move the LDS side too)
  constexpr int kQIters = BM * DT / 8 / NT;
  static_assert(kQIters % 4 == 0, "whole 256-row groups");
  const uint32_t q_voff = ((uint32_t)(tid >> 2) * (uint32_t)p.q_stride[1] +
                           (uint32_t)(((tid & 3) ^ ((tid >> 4) & 3)) * 8)) * 2u;
  const uint32_t q_rowgrp = __builtin_amdgcn_readfirstlane((uint32_t)(64 * p.q_stride[1] * 2));
  auto q_piece = [&](const Unit& u, int it) {
    const i32x4 r = BufStager<DT, BN, NT>::tile_rsrc(u.qg, p.q_stride[1], u.m0, u.Lq, qrows);
    const uint32_t lds = __builtin_amdgcn_readfirstlane(lds_addr(qs)) + (uint32_t)(it * NT * 16 + w * 1024);
    const uint32_t voff = q_voff + (uint32_t)(it & 3) * q_rowgrp + (uint32_t)((it >> 2) * 64);
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(r), "s"(lds)
        : "memory");
  };
  int boff = 0;  // ring offset: tile t of the unit is in K / V buffer (t + boff) & 1
  auto kt = [&](int t) { return smem + ((t + boff) & 1) * TILE; };
  auto vt = [&](int t) { return smem + (2 + ((t + boff) & 1)) * TILE; };
  constexpr int kPieces = BufStager<DT, BN, NT>::kIters;
  constexpr int kPerX = 2 * kPieces;                 // pieces of a regular period
  constexpr int kNext = kQIters + 3 * kPieces;       // pieces requesting the next unit
  // the next unit's loads: Q, then K(0), K(1), V(0) into the buffers tiles ntiles, ntiles + 1 of
  // the current unit would use (free in its final period: no QK^T, V(ntiles - 1) in the other)
  auto next_piece = [&](const Unit& cu, const Unit& nu, int pc) {
    if (pc < kQIters) {
      q_piece(nu, pc);
      return;
    }
    pc -= kQIters;
    const int t = pc / kPieces, it = pc % kPieces;
    char* dst = t == 2 ? vt(cu.ntiles) : kt(cu.ntiles + t);
    const uint16_t* g = t == 2 ? nu.vg : nu.kg;
    kst.piece(dst, BufStager<DT, BN, NT>::tile_rsrc(g, p.k_stride[1], t == 1 ? BN : 0, nu.Lk, mrows), it);
  };

  Unit u = make_unit(k_item, 0);
  int rep = 0;
  // first unit: its own loads
#pragma unroll
  for (int it = 0; it < kQIters; ++it) q_piece(u, it);
  kst.issue(kt(0), u.kg, p.k_stride[1], 0, u.Lk, mrows);
  kst.issue(vt(0), u.vg, p.v_stride[1], 0, u.Lk, mrows);
  kst.issue(kt(1), u.kg, p.k_stride[1], BN, u.Lk, mrows);  // past the end: empty range, zeros

  while (true) {
  // the unit after this one (same pair, or this workgroup's next item)
  const int nrep = nrep_of(k_item);
  int k_next = k_item, rep_next = rep + 1;
  if (rep_next == nrep) {
    k_next = k_item + per;
    rep_next = 0;
  }
  const bool has_next = k_next < i_count;
  const Unit nu = make_unit(has_next ? k_next : k_item, rep_next);

  const int lane = tid & 63, r32 = lane & 31, hh = lane >> 5;
  const int bh = u.bh, b = u.b, hq = u.hq, Lq = u.Lq, Lk = u.Lk, m0 = u.m0, ntiles = u.ntiles;
  const int qw0 = m0 + 64 * w;  // first row of this wave; row block r: qw0 + 32 r
  const uint16_t *kg = u.kg, *vg = u.vg;
  const int diag = Lk - Lq;

  vm_wait_all();  // this unit's Q / K / V requests (the previous unit's O stores may be in flight too)
  __syncthreads();

  // ---- Q fragments of both row blocks (B operand of S^T = K Q^T), into accumulation registers
  u32x4 qf[2][KS];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      qf[r][ks] = lds_row_frag<DT, BM>(qs, 64 * w + 32 * r, r32, ks, hh);
      asm volatile("" : "+a"(qf[r][ks]));  // into accumulation registers here, once per unit
    }

  const float uz = p.softmax_scale * kLog2e;
  float m_run[2] = {kNegInf, kNegInf}, l_run[2] = {0.f, 0.f}, m_ref[2] = {0.f, 0.f};
  f32x16 acc[2][NDT];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      acc[r][dt] = zero16();
      asm volatile("" : "+a"(acc[r][dt]));  // initialised here, not rematerialised at the first MFMA
    }

  int lim_lane[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) lim_lane[r] = CAUSAL ? min(Lk, qw0 + 32 * r + r32 + diag + 1) : Lk;
  // wave-uniform tile classes: live for the wave's last row, unmasked for its first
  auto tile_live = [&](int t) { return t < ntiles && !(CAUSAL && t * BN > qw0 + 63 + diag); };
  auto tile_mask = [&](int t) { return (t * BN + BN > Lk) || (CAUSAL && t * BN + BN - 1 > qw0 + diag); };

  typedef f32x16 Sc[2][2];  // [row block][key half]
  // Re-define O in place at this point (volatile, so after a preceding mfma_drain): the compiler's
  // accumulation-register copies for VALU work on O cannot be hoisted above the drain, nor sunk
  // below a drain that follows.
  auto pin_acc = [&]() {
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) asm volatile("" : "+a"(acc[r][dt]));
  };
  Sc s;                     // scores / exponent arguments of the tile whose softmax is next
  float mx[2] = {kNegInf, kNegInf};
  u32x4 pf[2][2][2];  // [row block][key half][k-step pair]: P packed, B operand of O^T += V^T P^T

  auto kfrag = [&](const char* K, int m) { return lds_row_frag<DT, BN>(K, 32 * (m & 1), r32, m >> 1, hh); };
  auto vfrag = [&](const char* V, int m) { return lds_tr_frag<DT, BN>(V, 16 * (m / NDT), 32 * (m % NDT), lane); };

  // exponent arguments z = s uz - m_ref of row block r
  auto to_z = [&](Sc& v) {
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) v[r][t][i] = fmaf(v[r][t][i], uz, -m_ref[r]);
  };

  // prologue QK^T of tile 0 (no interleaved work), masked when needed, row max, z
  auto qk_plain = [&](const char* K, bool mask) {
    u32x4 kf[NQK];
    auto kfs = [&](int m) { return kfrag(K, 2 * (m % KS) + m / KS); };  // half m / KS, k-step m % KS
#pragma unroll
    for (int j = 0; j < LEAD; ++j) kf[j] = kfs(j);
#pragma unroll
    for (int m = 0; m < NQK; ++m) {
      if (m + LEAD < NQK) kf[m + LEAD] = kfs(m + LEAD);
      const int t = m / KS, ks = m % KS;
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        if (ks == 0) s[r][t] = M::first(kf[m], qf[r][ks]);
        else M::next(s[r][t], kf[m], qf[r][ks]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    mfma_drain();
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int t = 0; t < 2; ++t) asm volatile("" : "+v"(s[r][t]));  // read only after the drain
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int rel = lim_lane[r] - 4 * hh;
      float mm = kNegInf;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int o = 32 * t + (i & 3) + 8 * (i >> 2);
          if (mask) s[r][t][i] = o < rel ? s[r][t][i] : kNegInf;
          mm = fmaxf(mm, s[r][t][i]);
        }
      mx[r] = half_max(mm) * uz;
    }
    to_z(s);
  };

  // Defer-max decision for the tile whose exponent arguments sit in z (one wave vote for both
  // row blocks); rare rescale of O (accumulation registers: drained first), l and z
  auto softmax_begin = [&](Sc& z) {
    const bool rescale = !__all(mx[0] - m_run[0] <= kDeferMax && mx[1] - m_run[1] <= kDeferMax);
    if (rescale) {
      mfma_drain();
      pin_acc();
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const float m_new = fmaxf(m_run[r], mx[r]);
        const float m_use = m_new == kNegInf ? 0.f : m_new;
        const float alpha = __builtin_amdgcn_exp2f(m_run[r] - m_use);
        const float shift = m_use - m_ref[r];
        l_run[r] *= alpha;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
          for (int i = 0; i < 16; ++i) acc[r][dt][i] *= alpha;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int i = 0; i < 16; ++i) z[r][t][i] -= shift;
        m_run[r] = m_new;
        m_ref[r] = m_use;
      }
      pin_acc();
      mfma_drain();
    }
  };

  mfma_drain();  // accumulation-register writes of Q and O before the first asm MFMA reads them

  auto dma_k = [&](int t, int pc) {
    kst.piece(kt(t), BufStager<DT, BN, NT>::tile_rsrc(kg, p.k_stride[1], t * BN, Lk, mrows), pc);
  };
  auto dma_v = [&](int t, int pc) {
    kst.piece(vt(t), BufStager<DT, BN, NT>::tile_rsrc(vg, p.v_stride[1], t * BN, Lk, mrows), pc);
  };
  // piece pc of period i's requests: K(i + 2) into the buffer of K(i) (read in period i - 1),
  // V(i + 1) into that of V(i - 1); the final period requests the next unit instead
  // (only a period without QK^T -- a wave's last live tile, or a DMA-only period -- can be final)
  auto dma = [&](int i, int pc, auto may_be_final) {
    if (decltype(may_be_final)::value && i == ntiles - 1) {
      if (has_next && pc < kNext) next_piece(u, nu, pc);
    } else if (pc < kPerX) {
      if (pc < kPieces) dma_k(i + 2, pc);
      else dma_v(i + 1, pc - kPieces);
    }
  };
  if (tile_live(0)) qk_plain(kt(0), tile_mask(0));
  __syncthreads();  // every wave is done with K(0) before K(2) lands in its buffer

  // Phase X(i): softmax(i) of cur, QK^T(i+1) into nxt (QK).  Key half t of nxt is produced in
  // steps t KS .. t KS + KS - 1 while the exponentials consume half t of cur.
  auto phase_x = [&](int i, Sc& cur, Sc& nxt, auto qk_c) {
    constexpr bool QK = decltype(qk_c)::value;
    const char* K1 = kt(i + 1);
    softmax_begin(cur);
    float rs[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
    u32x4 kf[NQK];
    auto kfs = [&](int m) { return kfrag(K1, 2 * (m % KS) + m / KS); };
    if constexpr (QK) {
#pragma unroll
      for (int j = 0; j < LEAD; ++j) kf[j] = kfs(j);
    }
    // One MFMA per scheduling region: at one wave per SIMD an MFMA issued right behind another
    // waits for the pipe in order, so the fillers must sit between the two.  Region g = 2 m + r
    // issues the exponentials of its pairs and finishes (row sums, bf16 pack) the pairs region
    // g - 1 issued, so no filler waits on a transcendental it just issued.
    constexpr int EPS = 16 / KS;   // exponentials per row block per step (2 at D = 128, 4 at D = 64)
    constexpr int PPR = EPS / 2;   // exponential pairs per region
    float pe[2][PPR][2];           // exponentials in flight: [region parity][pair][0 / 1]
    auto finish = [&](int g) {     // row sums + packs of region g's pairs
      const int m = g >> 1, r = g & 1, t = m / KS, ks = m % KS;
#pragma unroll
      for (int j = 0; j < PPR; ++j) {
        const int e = ks * EPS + 2 * j;
        const float p0 = pe[g & 1][j][0], p1 = pe[g & 1][j][1];
        rs[r][0] += p0;
        rs[r][1] += p1;
        pf[r][t][e >> 3][(e & 7) >> 1] = E::pack2(p0, p1);
      }
      // row-sum adds pinned to this region (IR sinking would chain all of them after the last MFMA)
      asm volatile("" : "+v"(rs[r][0]), "+v"(rs[r][1]));
    };
#pragma unroll
    for (int m = 0; m < NQK; ++m) {
      const int t = m / KS, ks = m % KS;
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int g = 2 * m + r;
        if constexpr (QK) {
          if (r == 0 && m + LEAD < NQK) kf[m + LEAD] = kfs(m + LEAD);
          if (ks == 0) nxt[r][t] = M::first(kf[m], qf[r][ks]);
          else M::next(nxt[r][t], kf[m], qf[r][ks]);
        }
#pragma unroll
        for (int j = 0; j < PPR; ++j) {
          const int e = ks * EPS + 2 * j;
          pe[g & 1][j][0] = __builtin_amdgcn_exp2f(cur[r][t][e]);
          pe[g & 1][j][1] = __builtin_amdgcn_exp2f(cur[r][t][e + 1]);
          asm volatile("" : "+v"(pe[g & 1][j][0]), "+v"(pe[g & 1][j][1]));
        }
        if (g > 0) finish(g - 1);
        if constexpr (QK) {
          if (g < kPerX) dma(i, g, std::false_type{});
        } else {
          if (g < kNext) dma(i, g, std::true_type{});
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    finish(2 * NQK - 1);
#pragma unroll
    for (int r = 0; r < 2; ++r) l_run[r] += rs[r][0] + rs[r][1];
  };
  // Phase Y(i): PV(i) of both row blocks, with mask, row max and exponent arguments of S(i+1)
  // in nxt (QK): key half 0 of both blocks in the first half of the steps, half 1 (whose last
  // MFMAs closed phase X) in the second.
  auto phase_y = [&](int i, Sc& nxt, auto qk_c, auto mask_c) {
    constexpr bool QK = decltype(qk_c)::value, MASK = decltype(mask_c)::value;
    const char* V0 = vt(i);
    constexpr int L = 2 * LEAD > NPV ? NPV : 2 * LEAD;
    constexpr int PER = 32 / NPV;  // elements per row block per step
    u32x4 vf[NPV];
    float ma[2][2] = {{kNegInf, kNegInf}, {kNegInf, kNegInf}};
    int rel[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) rel[r] = lim_lane[r] - (i + 1) * BN - 4 * hh;
#pragma unroll
    for (int j = 0; j < L; ++j) vf[j] = vfrag(V0, j);
    // one MFMA per scheduling region (see phase_x)
#pragma unroll
    for (int m = 0; m < NPV; ++m) {
      const int kk = m / NDT;
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        if (r == 0 && m + L < NPV) vf[m + L] = vfrag(V0, m + L);
        M::acc(acc[r][m % NDT], vf[m], pf[r][kk >> 1][kk & 1]);
        if constexpr (QK) {
#pragma unroll
          for (int e = m * PER; e < (m + 1) * PER; ++e) {
            const int t = e >> 4, ii = e & 15;
            if constexpr (MASK) {
              const int o = 32 * t + (ii & 3) + 8 * (ii >> 2);
              nxt[r][t][ii] = o < rel[r] ? nxt[r][t][ii] : kNegInf;
            }
            ma[r][t] = fmaxf(ma[r][t], nxt[r][t][ii]);
            nxt[r][t][ii] = fmaf(nxt[r][t][ii], uz, -m_ref[r]);
          }
          asm volatile("" : "+v"(ma[r][0]), "+v"(ma[r][1]));  // the max chains stay in their regions
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if constexpr (QK) {
#pragma unroll
      for (int r = 0; r < 2; ++r) mx[r] = half_max(fmaxf(ma[r][0], ma[r][1])) * uz;
    }
  };
  auto sync = [&]() {
    vm_wait_all();
    __syncthreads();
  };
  auto dma_only = [&](int period) {
#pragma unroll
    for (int pc = 0; pc < kNext; ++pc) dma(period, pc, std::true_type{});
  };
  using T = std::true_type;
  using F = std::false_type;

  int n_full = Lk / BN;
  if (CAUSAL) n_full = min(n_full, qw0 + diag + 1 >= 0 ? (qw0 + diag + 1) / BN : 0);
  int last = -1;
  if (ntiles > 0 && tile_live(0)) {
    last = ntiles - 1;
    if (CAUSAL) last = min(last, (qw0 + 63 + diag) / BN);
  }
  auto step = [&](int i, Sc& cur, Sc& nxt, auto qk_c, auto mask_c) {
    phase_x(i, cur, nxt, qk_c);
    phase_y(i, nxt, qk_c, mask_c);
    sync();
  };
  Sc s2;
  const int n_steady = max(0, min(n_full, ntiles) - 1);
  int i = 0;
  for (; i + 1 < n_steady; i += 2) {
    step(i, s, s2, T{}, F{});
    step(i + 1, s2, s, T{}, F{});
  }
  auto copy_back = [&]() {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      s[r][0] = s2[r][0];
      s[r][1] = s2[r][1];
    }
  };
  if (i < n_steady) {
    step(i, s, s2, T{}, F{});
    copy_back();
    ++i;
  }
  for (; i < last; ++i) {
    step(i, s, s2, T{}, T{});
    copy_back();
  }
  if (i == last) {
    step(i, s, s2, F{}, F{});
    ++i;
  }
  for (; i < ntiles; ++i) {
    dma_only(i);
    sync();
  }
  if (ntiles == 0 && has_next) {  // no period to carry the next unit's requests
#pragma unroll
    for (int pc = 0; pc < kNext; ++pc) next_piece(u, nu, pc);
  }

  // ---- epilogue ----------------------------------------------------------------------------
  mfma_drain();
  pin_acc();
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int qi = qw0 + 32 * r + r32;
    const float l_tot = half_sum(l_run[r]);
    const bool row_ok = qi < Lq && l_tot > 0.f;
    const float inv = row_ok ? 1.f / l_tot : 0.f;
    if (hh == 0 && qi < p.lse_row_stride) {
      float* lrow = p.lse + (int64_t)bh * p.lse_row_stride;
      lrow[qi] = row_ok ? m_run[r] + __log2f(l_tot) : kNegInf;
    }
    const int r0 = qw0 + 32 * r;
    if (r0 < p.seqlen_q) {
      uint16_t* o0 = (uint16_t*)p.o + b * p.o_stride[0] + hq * p.o_stride[2] + (int64_t)r0 * p.o_stride[1];
      // the wave's own 32-row staging image, reused for the second row block (in-order LDS)
      store_rows_lds<BF16, DT>(ostage, acc[r], inv, row_ok, o0, p.o_stride[1], min(32, p.seqlen_q - r0), D, lane);
    }
  }
  if (!has_next) break;
  boff = (boff + ntiles) & 1;
  u = nu;
  k_item = k_next;
  rep = rep_next;
  }
}

template <bool BF16, int DT, bool CAUSAL>
static hipError_t launch_fwd_w64(const fa2_fwd_args& a, hipStream_t st) {
  constexpr int BM = 256;
  const int nmb = (a.seqlen_q + BM - 1) / BM;
  const int items = (CAUSAL ? (nmb + 1) / 2 : nmb) * a.batch * a.heads_q;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
  }
  const int grid = min((items + 7) / 8 * 8, (cus + 7) / 8 * 8);  // one workgroup per CU, 8 | grid
  hipLaunchKernelGGL((fwd_w64_kernel<BF16, DT, CAUSAL>), dim3(grid), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace fa2
