// bwd_kernel.h -- FlashAttention-2 backward for gfx950 (CDNA4).
//
// Replaces the reference's backward launches (/root/reference/src/backward/caller.py:95-165):
//   delta_kernel  <- _compute_delta        (/root/reference/src/backward/compute_delta.py:17-73);
//                    the default backward folds it into dq_kernel, which runs first
//   dkdv_kernel   <- _bwd_kernel, pid < NUM_BLOCKS_KV branch + the host GQA sum
//                    (/root/reference/src/backward/kernel.py:154-166, compute_dkdv.py:7-296,
//                     caller.py:162-165)
//   dq_kernel     <- _bwd_kernel, dQ branch (kernel.py:168-182, compute_dq.py:7-261)
// Same math (src/backward/compute_dkdv.py:89-110, compute_dq.py:70-76):
//   P = exp2(s * scale * log2e - LSE2), dV = P^T dO, dP = dO V^T, dS = P (dP - delta) scale,
//   dK = dS^T Q, dQ = dS K; P and dS rounded to the input dtype before their MFMAs; fp32
//   accumulation; no atomics (bitwise reproducible, as tests/test_repeatability.py demands).
// Differences by design: the GQA group sum of dK/dV is done in fp32 registers inside
// dkdv_kernel (the reference sums bf16/fp16 tensors on the host), dQ is written directly in
// the requested dtype, and padded varlen rows are handled in place (no pack/unpack).
#include <type_traits>

#include <stdlib.h>

#include "common.h"
#include "fa2_internal.h"
#include "dkdv_hp_kernel.h"
#include "dq_hp_kernel.h"

// Schedule constants (measured; the variants they replaced are recorded in DESIGN.md):
//  dK/dV: S chain with its Q fragments kDkdvLS MFMAs ahead, then the dP chain with its
//         (dO, V) fragment pairs kDkdvLD ahead, then the dV/dK steps kDkdvLT transposed
//         fragments ahead -- at the 256-register limit a deeper prefetch spills;
//  dQ (recompute): fragments kDqLead k-steps ahead; interior tiles software-pipelined by
//         32-key halves with kDqPipeLead step of fragments in flight.

namespace fa2 {

constexpr int kDkdvLS = 2;
constexpr int kDkdvLD = 1;
constexpr int kDkdvLT = 2;
constexpr int kDqLead = 2;
constexpr int kDqPipeLead = 1;

// ---------------------------------------------------------------------------------------------
// delta[b, h, i] = -sum_d O[b, i, h, d] * dO[b, i, h, d]   (fp32; 0 for padded rows).  The
// workspace holds the NEGATED row sum: it is the initial dP accumulator of dkdv_kernel.
template <bool BF16, bool ALIGNED>
__global__ void __launch_bounds__(256) delta_kernel(const fa2_bwd_args p) {
  using E = Elem<BF16>;
  constexpr int LPR = 16;             // lanes per row
  constexpr int ROWS = 256 / LPR;     // rows per block
  const int tid = threadIdx.x;
  const int row = blockIdx.x * ROWS + tid / LPR;
  const int sub = tid % LPR;
  const int bh = blockIdx.y;
  const int b = bh / p.heads_q, h = bh - b * p.heads_q;
  int Lq = p.seqlen_q;
  if (p.cu_seqlens) Lq = p.cu_seqlens[b + 1] - p.cu_seqlens[b];
  float acc = 0.f;
  if (row < Lq) {
    const uint16_t* orow = (const uint16_t*)p.o + b * p.o_stride[0] + h * p.o_stride[2] + (int64_t)row * p.o_stride[1];
    const uint16_t* drow = (const uint16_t*)p.dout + b * p.do_stride[0] + h * p.do_stride[2] + (int64_t)row * p.do_stride[1];
    for (int d0 = sub * 8; d0 < p.head_dim; d0 += LPR * 8) {
      const u32x4 ov = load_row_frag<ALIGNED>(orow, d0, p.head_dim, true);
      const u32x4 dv = load_row_frag<ALIGNED>(drow, d0, p.head_dim, true);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc += E::to_f32((uint16_t)(ov[j] & 0xFFFF)) * E::to_f32((uint16_t)(dv[j] & 0xFFFF));
        acc += E::to_f32((uint16_t)(ov[j] >> 16)) * E::to_f32((uint16_t)(dv[j] >> 16));
      }
    }
  }
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, LPR);
  // rows [Lq, lse_row_stride) get 0 so that masked rows can never inject NaN/Inf garbage
  // stored negated: the dK/dV kernel starts its dP accumulator at -delta
  if (sub == 0 && row < p.lse_row_stride) p.delta[(int64_t)bh * p.lse_row_stride + row] = -acc;
}

// ---------------------------------------------------------------------------------------------
// dK, dV: one workgroup = 4 waves = 128 keys of one (batch, kv-head); wave w owns keys
// n0 + 32 w + (lane & 31).  K stays in VGPRs (B operand of S = Q K^T), the workgroup's V rows
// sit in LDS (B operand of dP = dO V^T, read as row fragments), and the workgroup sweeps the
// q-heads of its GQA group and 32-row query tiles (Q, dO, LSE2 and delta staged in LDS by
// LDS-DMA, double buffered).  Per tile and wave:
//   S[q][key], dP[q][key]   8 + 8 MFMA (A = Q / dO row fragments)
//   dV^T[d][key] += dO^T P  NDT*2 MFMA (A = dO^T via ds_read_b64_tr_b16, B = P registers)
//   dK^T[d][key] += Q^T dS  NDT*2 MFMA
// dK/dV accumulate the whole GQA group in fp32 and are rounded once.  <= 256 VGPRs, so two
// workgroups share a CU (DT <= 128).
// q-head split (nsplit > 1, small grids: GQA / MQA with few (batch, kv-head, key block) items):
// the group's q-heads are dealt to nsplit workgroups per key block, each writes its fp32 partial
// dK/dV sums to p.dkv_workspace ([nsplit][B][Hkv][Sk][D], unscaled) and dkv_reduce_kernel adds
// them in split order (deterministic).
// BIASK as dq_kernel: 0 none, 1 element loads from global memory, 16 / 17 a 16-bit bias with
// 16-byte aligned rows staged per wave by LDS-DMA: [32 query rows x 32 keys] of the step (2 KiB,
// single buffered), read with the transposing ds_read_b64_tr_b16 straight into the register
// order of the S accumulator (key on the lane).  The tile of step j+1 goes out as soon as step j
// has formed P, so it lands under the dV / dK chains (the step's closing wait covers it).
template <bool BF16, int DT, bool CAUSAL, int BIASK, bool DROPOUT, bool ALIGNED>
__global__ void __launch_bounds__(256, DT >= 256 ? 1 : 2) dkdv_kernel(const fa2_bwd_args p, int nsplit) {
  using E = Elem<BF16>;
  constexpr bool BIAS = BIASK != 0, BIASL = BIASK >= 16;
  constexpr int kBiasKTile = 32 * 32 * 2;  // one wave's [32 rows][32 keys] bias tile
  constexpr int NT = 256;
  constexpr int BNK = 128;          // keys per workgroup
  constexpr int BMQ = 32;           // query rows per tile
  constexpr int KS = DT / 16;
  constexpr int NDT = DT / 32;
  constexpr int VT = BNK * DT * 2;  // V tile bytes
  constexpr int QT = BMQ * DT * 2;  // Q (or dO) tile bytes
  constexpr int ST = 2 * BMQ * 4;   // LSE2 + delta rows of a tile
  __shared__ __attribute__((aligned(16))) char smem[VT + 4 * QT + 2 * ST + (BIASL ? 4 * kBiasKTile : 0)];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(w);  // the same, in an SGPR: scalar branches
  const int r32 = lane & 31, hh = lane >> 5;
  const int nkb = (p.seqlen_k + BNK - 1) / BNK;
  const int item = xcd_item(blockIdx.x, gridDim.x);  // head-major, see xcd_item
  const int grp = item / nkb;                        // (batch, kv-head, q-head split)
  const int n0 = (item - grp * nkb) * BNK;           // causal: low keys see the most rows
  const int bkv = grp / nsplit, split = grp - bkv * nsplit;
  const int b = bkv / p.heads_kv, hkv = bkv - b * p.heads_kv;
  const int G = p.heads_q / p.heads_kv / nsplit;     // q-heads of this workgroup
  const int h0 = (hkv * nsplit + split) * G;         // its first q-head
  int Lq = p.seqlen_q, Lk = p.seqlen_k;
  if (p.cu_seqlens) Lq = Lk = p.cu_seqlens[b + 1] - p.cu_seqlens[b];
  const int D = p.head_dim;
  const int diag = Lk - Lq;
  const int kw0 = n0 + 32 * w;   // first key of this wave
  const int kj = kw0 + r32;      // this lane's key
  const bool kval = kj < Lk;
  const float scale = p.softmax_scale, scale2 = scale * kLog2e;
  const float sc = BIAS ? 1.f : scale2;
  // dropout: flat Philox offset of (b, hq, row, key) exactly as the forward (fwd_kernel.h)
  const int cu0 = p.cu_seqlens ? p.cu_seqlens[b] : 0;
  auto drop_base = [&](int hq_) -> uint64_t {
    return (uint64_t)Lk * ((uint64_t)cu0 + (uint64_t)Lq * ((uint64_t)hq_ + (uint64_t)p.heads_q * (p.cu_seqlens ? 0 : b)));
  };
  const float inv_keep = DROPOUT ? 1.f / (1.f - p.dropout_p) : 1.f;

  char* Vs = smem;
  auto qt = [&](int buf) { return smem + VT + buf * 2 * QT; };
  auto ot = [&](int buf) { return smem + VT + QT + buf * 2 * QT; };
  auto st = [&](int buf) { return smem + VT + 4 * QT + buf * ST; };

  // query tiles: causal -> the first row that sees key n0 is n0 - diag
  int m_begin = 0;
  if (CAUSAL) m_begin = max(0, n0 - diag) & ~(BMQ - 1);
  const int n_mt = (n0 < Lk && m_begin < Lq) ? (Lq - m_begin + BMQ - 1) / BMQ : 0;
  // Query tiles are swept from the last one down: every workgroup of a (batch, kv-head) then
  // reads the same Q / dO tile at the same step -- one HBM read, the other key blocks hit L2 --
  // where an ascending sweep from each block's own first visible tile spreads the reads of one
  // tile over the whole pass (dkdv HBM reads halved).
  const int m_last = m_begin + (n_mt - 1) * BMQ;
  auto tile_row = [&](int t) { return m_last - t * BMQ; };
  const int total = n_mt * G;  // (q-head, tile) steps

  // buffer-resource LDS-DMA (rows past Lq read as zeros; masked out of every product)
  BufStager<DT, BMQ, NT> qst, ost;
  int qrows = 0, orows = 0;
  if (ALIGNED) {
    qst.init(tid, p.q_stride[1], D);
    ost.init(tid, p.do_stride[1], D);
    qrows = BufStager<DT, BMQ, NT>::max_rows(p.q_stride[1]);
    orows = BufStager<DT, BMQ, NT>::max_rows(p.do_stride[1]);
  }
  int st_g = 0, st_mt = 0;  // (q-head in group, query tile) of the next step to stage
  auto stage = [&](int buf) {
    const int hq = h0 + st_g;
    const int m = tile_row(st_mt);
    if (++st_mt == n_mt) {
      st_mt = 0;
      ++st_g;
    }
    const uint16_t* qg = (const uint16_t*)p.q + b * p.q_stride[0] + hq * p.q_stride[2];
    const uint16_t* og = (const uint16_t*)p.dout + b * p.do_stride[0] + hq * p.do_stride[2];
    if constexpr (ALIGNED) {
      qst.issue(qt(buf), qg, p.q_stride[1], m, Lq, qrows);
      ost.issue(ot(buf), og, p.do_stride[1], m, Lq, orows);
    } else {
      stage_tile<DT, BMQ, NT, false>(qt(buf), qg, p.q_stride[1], m, Lq, D, tid);
      stage_tile<DT, BMQ, NT, false>(ot(buf), og, p.do_stride[1], m, Lq, D, tid);
    }
    if (wu < 2) {  // LSE2 rows (wave 0) then delta rows (wave 1): 32 dwords each, lanes 0..31
      // wave-uniform row bases in SGPR descriptors (no per-lane 64-bit address at the register
      // limit)
      const int64_t row0 = (int64_t)(b * p.heads_q + hq) * p.lse_row_stride + m;
      const uint32_t lds = __builtin_amdgcn_readfirstlane(lds_addr(st(buf))) + wu * BMQ * 4;
      int t = threadIdx.x;
      asm volatile("" : "+v"(t));
      blds4_lo32((uint32_t)(t & 31) * 4u, make_rsrc((wu == 0 ? p.lse : p.delta) + row0, BMQ * 4), lds);
    }
  };
  // The same staging for the descending sweep with every address carried from step to step in
  // SGPRs: the byte address of the next tile's first Q / dO row and the index of its first
  // LSE2 / delta row move by one tile per step and jump to the next q-head's last tile when the
  // head changes, so a step's staging is a few scalar adds and the descriptor words.  (Recomputed
  // per step from the head and row indices, the 64-bit address arithmetic of `stage` put ~130
  // scalar instructions in front of every step; a timing ablation without it ran 4-7 % faster.)
  const int64_t q_rb = p.q_stride[1] * 2, o_rb = p.do_stride[1] * 2;  // row bytes
  uint64_t nq = 0, no = 0;  // next tile's first-row byte addresses
  int64_t nl = 0;           // next tile's first LSE2 / delta element
  int nm = m_last;          // next tile's first row
  if constexpr (ALIGNED) {
    nq = uniform64((int64_t)(uintptr_t)p.q + 2 * (b * p.q_stride[0] + h0 * p.q_stride[2]) + (int64_t)m_last * q_rb);
    no = uniform64((int64_t)(uintptr_t)p.dout + 2 * (b * p.do_stride[0] + h0 * p.do_stride[2]) + (int64_t)m_last * o_rb);
    nl = uniform64((int64_t)(b * p.heads_q + h0) * p.lse_row_stride + m_last);
  }
  const int64_t q_wrap = (int64_t)(n_mt - 1) * BMQ * q_rb + 2 * p.q_stride[2];
  const int64_t o_wrap = (int64_t)(n_mt - 1) * BMQ * o_rb + 2 * p.do_stride[2];
  const int64_t l_wrap = (int64_t)(n_mt - 1) * BMQ + p.lse_row_stride;
  auto stage_desc = [&](int buf) {
    const int rows = Lq - nm;  // >= 1: rows past Lq read as zeros (descriptor range)
    const i32x4 rq = make_rsrc((const void*)(uintptr_t)nq, (uint32_t)min(rows, qrows) * (uint32_t)q_rb);
    const i32x4 ro = make_rsrc((const void*)(uintptr_t)no, (uint32_t)min(rows, orows) * (uint32_t)o_rb);
#pragma unroll
    for (int it = 0; it < BufStager<DT, BMQ, NT>::kIters; ++it) {
      qst.piece(qt(buf), rq, it);
      ost.piece(ot(buf), ro, it);
    }
    if (wu < 2) {
      const uint32_t lds = __builtin_amdgcn_readfirstlane(lds_addr(st(buf))) + wu * BMQ * 4;
      int t = threadIdx.x;
      asm volatile("" : "+v"(t));
      blds4_lo32((uint32_t)(t & 31) * 4u, make_rsrc((wu == 0 ? p.lse : p.delta) + nl, BMQ * 4), lds);
    }
    if (++st_mt == n_mt) {
      st_mt = 0;
      nm = m_last;
      nq = uniform64(nq + q_wrap);
      no = uniform64(no + o_wrap);
      nl = uniform64(nl + l_wrap);
    } else {
      nm -= BMQ;
      nq = uniform64(nq - BMQ * q_rb);
      no = uniform64(no - BMQ * o_rb);
      nl = uniform64(nl - BMQ);
    }
  };

  // this wave's bias tiles (BIASL): [32 query rows from m][32 keys from kw0] of step (hq, m)
  using BiasStager = BufStager<32, 32, 64>;
  BiasStager bst;
  int brows = 0;
  char* const bwk = smem + VT + 4 * QT + 2 * ST + w * kBiasKTile;
  if constexpr (BIASL) {
    bst.init(lane, p.bias_stride[2], 32);
    brows = BiasStager::max_rows(p.bias_stride[2]);
  }
  auto bias_issue = [&](int hq_, int m_) {
    if constexpr (BIASL) {
      const uint16_t* bg = (const uint16_t*)p.bias + b * p.bias_stride[0] + hq_ * p.bias_stride[1] + kw0;
      const i32x4 r = bias_tile_rsrc(bg, p.bias_stride[2], m_, p.seqlen_q, brows, p.seqlen_k - kw0, 32);
#pragma unroll
      for (int it = 0; it < BiasStager::kIters; ++it) bst.piece(bwk, r, it);
    }
  };
  // the bias of register i (query row m + (i & 3) + 8 (i >> 2) + 4 hh, this lane's key): element
  // i & 7 of transposed read i >> 3
  auto bias_rd = [&](int half) -> u32x4 { return lds_tr_frag<32, 32>(bwk, 16 * half, 0, lane); };
  auto bias_of = [&](const u32x4* bt2, int i) -> float {
    const int j = i & 7;
    const u32x2 pair = {bt2[i >> 3][(j >> 2) * 2], bt2[i >> 3][(j >> 2) * 2 + 1]};
    return bias_elem<BIASK>(pair, j & 3);
  };

  u32x4 kf[KS];
  {
    const uint16_t* krow = (const uint16_t*)p.k + b * p.k_stride[0] + hkv * p.k_stride[2] + (int64_t)(kval ? kj : 0) * p.k_stride[1];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) kf[ks] = load_row_frag<ALIGNED>(krow, 16 * ks + 8 * hh, D, kval);
  }
  if (total > 0) {
    const uint16_t* vg = (const uint16_t*)p.v + b * p.v_stride[0] + hkv * p.v_stride[2];
    stage_tile<DT, BNK, NT, ALIGNED>(Vs, vg, p.v_stride[1], n0, Lk, D, tid);
    if constexpr (ALIGNED) stage_desc(0);
    else stage(0);
    bias_issue(h0, tile_row(0));
  }
  f32x16 dk[NDT], dv[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) { dk[dt] = zero16(); dv[dt] = zero16(); }


  // dropout keep words (the forward's saved mask, tiled layout of fa2_amd.h) of a step: lane
  // (r32, hh) loads row r32 of the step's 32 x 32 tile; loaded one step ahead so the loop's
  // vm_wait_all retires them (a load consumed in its own step would wait for the Q / dO DMA)
  uint32_t mw_cur = 0u, mw_nxt = 0u;
  auto load_mw = [&](int hq_, int m_) -> uint32_t {
    if constexpr (DROPOUT && DT <= 128) {
      if (p.dropout_mask && kw0 < p.seqlen_k) {
        const int nrb = (p.seqlen_q + 31) >> 5, ncw = (p.seqlen_k + 31) >> 5;
        return p.dropout_mask[(((int64_t)(b * p.heads_q + hq_) * nrb + (m_ >> 5)) * ncw + (kw0 >> 5)) * 32 + r32];
      }
    }
    return 0u;
  };
  // Phases (sched_barrier-separated so each phase's LDS fragments stay inside it and the
  // register peak stays under 256): S, dP -> P, dS -> dV, dK.
  auto body = [&](auto mask_c, const char* Q, const char* O, const char* S, int hq, int m, auto next_bias) {
    constexpr bool MASK = decltype(mask_c)::value;
    // the forward's keep mask M of this lane's key and the 16 rows m + o + 4 hh, first: no score
    // or fragment registers are live yet
    uint32_t keep16 = 0u;
    if constexpr (DROPOUT) {
      // (D = 256: redrawn -- the mask read there crashes ROCm 7.2's AGPR-copy rewrite pass)
      if (DT <= 128 && p.dropout_mask) {
        // the forward's saved 32 x 32 bit tile of this step (rows m.., keys kw0..), loaded one
        // step ahead: lane (r32, hh) holds row r32's word (bit k = key kw0 + k).  Transposed
        // across each 32-lane half (5 ds_swizzle xor stages), lane r32 then holds key kw0 + r32's
        // column (bit r = row m + r); register i of the lane is row (i & 3) + 8 (i >> 2) + 4 hh.
        const uint32_t xs = transpose32_lanes(mw_cur, r32) >> (4 * hh);
        keep16 = (xs & 0xFu) | ((xs >> 4) & 0xF0u) | ((xs >> 8) & 0xF00u) | ((xs >> 12) & 0xF000u);
      } else {
        keep16 = dropout_keep16(p.dropout_seed, drop_base(hq) + (uint64_t)(m + 4 * hh) * (uint64_t)Lk + (uint64_t)kj,
                                (uint64_t)Lk, p.dropout_p);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    f32x16 s = zero16(), dp = zero16();
    u32x4 bt2[2];
    if constexpr (BIASL) {
      bt2[0] = bias_rd(0);
      bt2[1] = bias_rd(1);
    }
    {
      // fenced steps: the S chain (one fragment per MFMA, read kDkdvLS MFMAs ahead), then the dP
      // chain (two fragments per MFMA, kDkdvLD ahead): deeper prefetch than alternating chains
      // for the same registers in flight
      constexpr int LS = kDkdvLS < KS ? kDkdvLS : KS, LD = kDkdvLD < KS ? kDkdvLD : KS;
      u32x4 fq[KS], fo[KS], fv[KS];
#pragma unroll
      for (int j = 0; j < LS; ++j) fq[j] = lds_row_frag<DT, BMQ>(Q, 0, r32, j, hh);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if (ks + LS < KS) fq[ks + LS] = lds_row_frag<DT, BMQ>(Q, 0, r32, ks + LS, hh);
        // the dP chain's first fragments ride in the S chain's last steps
        if (ks + LD >= KS) {
          const int j = ks + LD - KS;
          fo[j] = lds_row_frag<DT, BMQ>(O, 0, r32, j, hh);
          fv[j] = lds_row_frag<DT, BNK>(Vs, 32 * w, r32, j, hh);
        }
        s = E::mfma(fq[ks], kf[ks], s);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if (ks + LD < KS) {
          fo[ks + LD] = lds_row_frag<DT, BMQ>(O, 0, r32, ks + LD, hh);
          fv[ks + LD] = lds_row_frag<DT, BNK>(Vs, 32 * w, r32, ks + LD, hh);
        }
        dp = E::mfma(fo[ks], fv[ks], dp);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    // rows of register i: m + (i & 3) + 8 (i >> 2) + 4 hh.  The row window [q_lo, q_hi) of this
    // lane's key is recomputed from an opaque lane id: hoisted out of the loop it gets spilled
    // and its scratch reload would drain the LDS-DMA prefetch (vmcnt(0)).
    int lo = 0, hi = 0;
    if (MASK) {
      int ln = threadIdx.x;
      asm volatile("" : "+v"(ln));
      const int kl = n0 + 32 * (ln >> 6) + (ln & 31);
      const int qlo = CAUSAL ? max(kl - diag, 0) : 0;
      const int qhi = kl < Lk ? Lq : -1;
      lo = qlo - m - 4 * ((ln >> 5) & 1);  // (hh, likewise from the opaque id)
      hi = qhi - m - 4 * ((ln >> 5) & 1);
    }
    u32x4 pp[2], dsp[2];
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const f32x4 l4 = *(const f32x4*)(S + 4 * (8 * g4 + 4 * hh));
      const f32x4 d4 = *(const f32x4*)(S + 4 * BMQ + 4 * (8 * g4 + 4 * hh));
      float pv[4], dsv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = 4 * g4 + j;
        const int o = j + 8 * g4;
        float x = s[i];
        if constexpr (BIASL) {
          x = fmaf(x, scale2, kLog2e * bias_of(bt2, i));
        } else if constexpr (BIAS) {
          const int qr = m + o + 4 * hh;
          const int qc = qr < Lq ? qr : Lq - 1;
          const int kc = kval ? kj : Lk - 1;
          x = fmaf(x, scale2, kLog2e * load_bias(p.bias, b * p.bias_stride[0] + hq * p.bias_stride[1] +
                                                           (int64_t)qc * p.bias_stride[2] + kc, p.bias_dtype));
        }
        float pr = __builtin_amdgcn_exp2f(fmaf(x, sc, -l4[j]));
        if (MASK) pr = (o >= lo && o < hi) ? pr : 0.f;
        if (DROPOUT) {
          // the forward's keep mask (same Philox offsets), P~ = P M / (1 - p):
          // dV += P~^T dO, dS = P (dP~ M / (1 - p) - delta)
          const float kp = (keep16 >> i) & 1u ? inv_keep : 0.f;
          pv[j] = pr * kp;
          dsv[j] = pr * (dp[i] * kp + d4[j]);  // d4 = -delta (workspace convention)
        } else {
          pv[j] = pr;
          dsv[j] = pr * (dp[i] + d4[j]);  // softmax_scale is applied to dK once, at the end
        }
      }
      pp[g4 >> 1][2 * (g4 & 1) + 0] = E::pack2(pv[0], pv[1]);
      pp[g4 >> 1][2 * (g4 & 1) + 1] = E::pack2(pv[2], pv[3]);
      dsp[g4 >> 1][2 * (g4 & 1) + 0] = E::pack2(dsv[0], dsv[1]);
      dsp[g4 >> 1][2 * (g4 & 1) + 1] = E::pack2(dsv[2], dsv[3]);
    }
    next_bias();  // this step's bias tile is consumed: the next one may land in its buffer
    __builtin_amdgcn_sched_barrier(0);
    {
      // steps m: dt = m % NDT (independent chains back to back), r = m / NDT: (sp, dV | dK);
      // transposed fragments two steps ahead
      constexpr int N = 4 * NDT, L = 2 < N ? 2 : N;
      u32x4 fr[N];
      auto rd = [&](int m) {
        const int dt = m % NDT, r = m / NDT;
        return lds_tr_frag<DT, BMQ>((r & 1) ? Q : O, 16 * (r >> 1), 32 * dt, lane);
      };
#pragma unroll
      for (int j = 0; j < L; ++j) fr[j] = rd(j);
#pragma unroll
      for (int m = 0; m < N; ++m) {
        if (m + L < N) fr[m + L] = rd(m + L);
        const int dt = m % NDT, r = m / NDT;
        if (r & 1) dk[dt] = E::mfma(fr[m], dsp[r >> 1], dk[dt]);
        else dv[dt] = E::mfma(fr[m], pp[r >> 1], dv[dt]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };

  // The plain step (no bias, no dropout), software-pipelined inside the wave so that the
  // softmax-gradient VALU work sits beside MFMAs of the same wave instead of in a VALU-only phase:
  //   [S chain] [dP chain | P = exp2(S sc - LSE2)] [dV, dK chains | dS = P dP', packs]
  // The dP accumulator starts at -delta (the delta workspace holds -rowsum(O dO)), so the chain
  // yields dP - delta and dS is one multiply; the LSE2 and -delta rows are read from LDS at the
  // start of the step, long before their use.
  auto body_pipe = [&](auto mask_c, const char* Q, const char* O, const char* S, int m, auto next_bias) {
    constexpr bool MASK = decltype(mask_c)::value;
    // A bias (BIASL) enters as the S chain's initial accumulator together with the LSE2 rows,
    // b / scale - LSE2 / (scale log2 e): the chain yields x with P = exp2(x scale log2 e), so the
    // P phase needs neither the bias nor the LSE2 registers (at the 256-register limit both spilled
    // there, and the spilled DMA offsets' reloads drained the Q / dO prefetch).
    f32x16 binit;
    if constexpr (BIASL) {
      const u32x4 bt2[2] = {bias_rd(0), bias_rd(1)};
      const float rs = 1.f / scale, rl = -1.f / scale2;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const f32x4 lg = *(const f32x4*)(S + 4 * (8 * g4 + 4 * hh));
#pragma unroll
        for (int j = 0; j < 4; ++j) binit[4 * g4 + j] = fmaf(bias_of(bt2, 4 * g4 + j), rs, lg[j] * rl);
      }
    }
    constexpr int LS = kDkdvLS < KS ? kDkdvLS : KS, LD = kDkdvLD < KS ? kDkdvLD : KS;
    constexpr int EP = 16 / KS;          // P elements per dP step
    constexpr int N = 4 * NDT;           // dV / dK steps
    constexpr int ED = 8 / NDT;          // dS elements per dV / dK step (first 2 NDT steps)
    constexpr int LT = kDkdvLT < N ? kDkdvLT : N;  // transposed fragments in flight
    f32x16 s, dp;
    f32x4 l4[4];  // LSE2 rows of register group g4 (rows 8 g4 + 4 hh + 0..3), read just ahead
    auto rd_lse = [&](int g4) { l4[g4] = *(const f32x4*)(S + 4 * (8 * g4 + 4 * hh)); };
    auto rd_nd = [&](int g4) {  // -delta rows of group g4 into the dP accumulator
      const f32x4 d4 = *(const f32x4*)(S + 4 * BMQ + 4 * (8 * g4 + 4 * hh));
#pragma unroll
      for (int j = 0; j < 4; ++j) dp[4 * g4 + j] = d4[j];
    };
    u32x4 fq[KS], fo[KS], fv[KS];
#pragma unroll
    for (int j = 0; j < LS; ++j) fq[j] = lds_row_frag<DT, BMQ>(Q, 0, r32, j, hh);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + LS < KS) fq[ks + LS] = lds_row_frag<DT, BMQ>(Q, 0, r32, ks + LS, hh);
      if (ks + LD >= KS) {
        const int j = ks + LD - KS;
        fo[j] = lds_row_frag<DT, BMQ>(O, 0, r32, j, hh);
        fv[j] = lds_row_frag<DT, BNK>(Vs, 32 * w, r32, j, hh);
      }
      // the -delta rows land in the dP accumulator over the last S steps, LSE group 0 last
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4)
        if ((KS >= 4 ? ks == KS - 4 + g4 : ks == KS - 2 + g4 / 2)) rd_nd(g4);
      // LSE group g4 is first used at dP step 4 g4 / EP and read one step ahead; the groups
      // needed in dP step 0 are read here
      if (!BIASL && ks == KS - 1) {
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4)
          if ((4 * g4) / EP == 0) rd_lse(g4);
      }
      if constexpr (BIASL) s = E::mfma(fq[ks], kf[ks], ks == 0 ? binit : s);
      else s = E::mfma(fq[ks], kf[ks], ks == 0 ? zero16() : s);
      __builtin_amdgcn_sched_barrier(0);
    }
    int lo = 0, hi = 0;  // as in body(): the visible row window of this lane's key
    if (MASK) {
      int ln = threadIdx.x;
      asm volatile("" : "+v"(ln));
      const int kl = n0 + 32 * (ln >> 6) + (ln & 31);
      const int qlo = CAUSAL ? max(kl - diag, 0) : 0;
      const int qhi = kl < Lk ? Lq : -1;
      lo = qlo - m - 4 * ((ln >> 5) & 1);  // (hh, likewise from the opaque id)
      hi = qhi - m - 4 * ((ln >> 5) & 1);
    }
    u32x4 pp[2], dsp[2];
    auto p_elem = [&](int i) {  // P in place of S, packed pairwise
      const int o = (i & 3) + 8 * (i >> 2);
      float pr;
      if constexpr (BIASL) pr = __builtin_amdgcn_exp2f(s[i] * scale2);
      else pr = __builtin_amdgcn_exp2f(fmaf(s[i], sc, -l4[i >> 2][i & 3]));
      if (MASK) pr = (o >= lo && o < hi) ? pr : 0.f;
      s[i] = pr;
    };
    auto p_pack = [&](int sp) {  // P packed for the dV product, right before its first use
#pragma unroll
      for (int t = 0; t < 4; ++t) pp[sp][t] = E::pack2(s[8 * sp + 2 * t], s[8 * sp + 2 * t + 1]);
    };
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + LD < KS) {
        fo[ks + LD] = lds_row_frag<DT, BMQ>(O, 0, r32, ks + LD, hh);
        fv[ks + LD] = lds_row_frag<DT, BNK>(Vs, 32 * w, r32, ks + LD, hh);
      }
      dp = E::mfma(fo[ks], fv[ks], dp);
#pragma unroll
      for (int e = ks * EP; e < (ks + 1) * EP; ++e) p_elem(e);
#pragma unroll
      for (int g4 = 1; g4 < 4; ++g4)
        if (!BIASL && (4 * g4) / EP > 0 && ks == (4 * g4) / EP - 1) rd_lse(g4);
      __builtin_amdgcn_sched_barrier(0);
    }
    auto ds_elem = [&](int i) {  // dS = P (dP - delta) in place of dP, packed pairwise
      dp[i] = s[i] * dp[i];
      if (i & 1) dsp[i >> 3][(i & 7) >> 1] = E::pack2(dp[i - 1], dp[i]);
    };
    // steps m: dt = m % NDT, r = m / NDT: dV (sp 0), dK (sp 0), dV (sp 1), dK (sp 1); dS elements
    // 0..7 ride on the first NDT steps, 8..15 on the next NDT (dsp[1] is first read at r = 3)
    u32x4 fr[N];
    auto rd = [&](int mm) {
      const int dt = mm % NDT, r = mm / NDT;
      return lds_tr_frag<DT, BMQ>((r & 1) ? Q : O, 16 * (r >> 1), 32 * dt, lane);
    };
    next_bias();  // P is formed: the next step's bias tile may land in this wave's buffer
#pragma unroll
    for (int j = 0; j < LT; ++j) fr[j] = rd(j);
    p_pack(0);
#pragma unroll
    for (int mm = 0; mm < N; ++mm) {
      if (mm + LT < N) fr[mm + LT] = rd(mm + LT);
      const int dt = mm % NDT, r = mm / NDT;
      if (mm == 2 * NDT - 1) p_pack(1);  // pp[1] is first read at r = 2
      if (r & 1) dk[dt] = E::mfma(fr[mm], dsp[r >> 1], dk[dt]);
      else dv[dt] = E::mfma(fr[mm], pp[r >> 1], dv[dt]);
      if (mm < 2 * NDT) {
#pragma unroll
        for (int e = mm * ED; e < (mm + 1) * ED; ++e) ds_elem(e);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  __builtin_amdgcn_s_waitcnt(0);  // prologue: Q fragments (compiler-tracked) + first tiles
  __syncthreads();
  if (ALIGNED && D < DT && total > 0) {
    // dP = dO V^T reads both operands from LDS, whose clamped staging repeats the last real
    // chunk in the padding columns: zero V's padding once so those columns contribute nothing.
    constexpr int kChunks = DT / 8;
    const int c0 = D >> 3;
    for (int idx = tid; idx < BNK * kChunks; idx += NT) {
      const int r = idx / kChunks, c = idx % kChunks;
      if (c >= c0) *(u32x4*)(Vs + Tile<DT, BNK>::off(r, c)) = u32x4{0u, 0u, 0u, 0u};
    }
    __syncthreads();
  }

  if (total > 0) mw_cur = load_mw(h0, tile_row(0));
  int g = 0, mt = 0;  // (q-head in group, query tile) of the current step
  for (int step = 0; step < total; ++step) {
    const int cur = step & 1;
    if (DROPOUT && step + 1 < total) {
      const bool wrap = mt + 1 == n_mt;
      mw_nxt = load_mw(h0 + g + (wrap ? 1 : 0), tile_row(wrap ? 0 : mt + 1));
    }
    if (step + 1 < total) {
      if constexpr (ALIGNED) stage_desc(cur ^ 1);
      else stage(cur ^ 1);
    }
    const int hq = h0 + g;
    const int m = tile_row(mt);
    // wave-uniform tile class
    const bool dead = kw0 >= Lk || (CAUSAL && kw0 > m + BMQ - 1 + diag);
    const bool need_mask = (m + BMQ > Lq) || (kw0 + 31 >= Lk) || (CAUSAL && kw0 + 31 > m + diag);
    // the bias tile of the next step (BIASL), issued once this step's P no longer needs the buffer
    auto next_bias = [&]() {
      if (step + 1 < total) {
        const bool wrap = mt + 1 == n_mt;
        bias_issue(hq + (wrap ? 1 : 0), tile_row(wrap ? 0 : mt + 1));
      }
    };
    if (!dead) {
      if constexpr ((!BIAS || BIASL) && !DROPOUT) {
        if (need_mask)
          body_pipe(std::true_type{}, qt(cur), ot(cur), st(cur), m, next_bias);
        else
          body_pipe(std::false_type{}, qt(cur), ot(cur), st(cur), m, next_bias);
      } else {
        if (need_mask)
          body(std::true_type{}, qt(cur), ot(cur), st(cur), hq, m, next_bias);
        else
          body(std::false_type{}, qt(cur), ot(cur), st(cur), hq, m, next_bias);
      }
    } else {
      next_bias();
    }
    vm_wait_all();
    __syncthreads();
    if constexpr (DROPOUT) mw_cur = mw_nxt;
    if (++mt == n_mt) {
      mt = 0;
      ++g;
    }
  }

  // ---- store dK, dV (kv heads; fp32 group sum rounded once) ----------------------------
  if (nsplit > 1) {
    // partial sums of this split: [split][b][hkv][key][D] fp32, unscaled (dkv_reduce_kernel)
    if (kj < p.seqlen_k) {
      const int64_t row = (((int64_t)split * p.batch + b) * p.heads_kv + hkv) * p.seqlen_k + kj;
      float* pk = p.dkv_workspace + row * D;
      float* pv = p.dkv_workspace + ((int64_t)nsplit * p.batch * p.heads_kv * p.seqlen_k + row) * D;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int d0 = 32 * dt + 8 * g4 + 4 * hh;
          float a[4], c[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            a[j] = kval ? dk[dt][4 * g4 + j] : 0.f;
            c[j] = kval ? dv[dt][4 * g4 + j] : 0.f;
          }
          if (ALIGNED) {  // D % 8 == 0: whole 4-column groups
            if (d0 < D) {
              *(f32x4*)(pk + d0) = f32x4{a[0], a[1], a[2], a[3]};
              *(f32x4*)(pv + d0) = f32x4{c[0], c[1], c[2], c[3]};
            }
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (d0 + j < D) {
                pk[d0 + j] = a[j];
                pv[d0 + j] = c[j];
              }
          }
        }
      }
    }
    return;
  }
  if constexpr (ALIGNED) {
    // every wave passed the last step's barrier: V and Q/dO buffers hold the staging images
    uint16_t* k0 = (uint16_t*)p.dk + b * p.dk_stride[0] + hkv * p.dk_stride[2] + (int64_t)kw0 * p.dk_stride[1];
    uint16_t* v0 = (uint16_t*)p.dv + b * p.dv_stride[0] + hkv * p.dv_stride[2] + (int64_t)kw0 * p.dv_stride[1];
    const int nrows = min(32, p.seqlen_k - kw0);
    store_rows_lds<BF16, DT>(smem + w * 32 * DT * 2, dk, scale, kval, k0, p.dk_stride[1], nrows, D, lane);
    store_rows_lds<BF16, DT>(smem + (4 + w) * 32 * DT * 2, dv, 1.f, kval, v0, p.dv_stride[1], nrows, D, lane);
    return;
  }
  if (kj < p.seqlen_k) {
    uint16_t* dkrow = (uint16_t*)p.dk + b * p.dk_stride[0] + hkv * p.dk_stride[2] + (int64_t)kj * p.dk_stride[1];
    uint16_t* dvrow = (uint16_t*)p.dv + b * p.dv_stride[0] + hkv * p.dv_stride[2] + (int64_t)kj * p.dv_stride[1];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d0 = 32 * dt + 8 * g4 + 4 * hh;
        float a[4], c[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          a[j] = kval ? dk[dt][4 * g4 + j] * scale : 0.f;
          c[j] = kval ? dv[dt][4 * g4 + j] : 0.f;
        }
        if (ALIGNED) {
          if (d0 < D) {
            *(u32x2*)(dkrow + d0) = u32x2{E::pack2(a[0], a[1]), E::pack2(a[2], a[3])};
            *(u32x2*)(dvrow + d0) = u32x2{E::pack2(c[0], c[1]), E::pack2(c[2], c[3])};
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (d0 + j < D) {
              dkrow[d0 + j] = E::from_f32(a[j]);
              dvrow[d0 + j] = E::from_f32(c[j]);
            }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// dK/dV of a q-head split (dkdv_kernel, nsplit > 1): dK = scale * sum_s dK_s, dV = sum_s dV_s
// over the fp32 partials in split order (deterministic), rounded once.  One thread per four
// columns of one (batch, kv-head, key) row; HBM-bound (2 nsplit fp32 reads per output element).
template <bool BF16>
__global__ void __launch_bounds__(256) dkv_reduce_kernel(const fa2_bwd_args p, int nsplit) {
  using E = Elem<BF16>;
  const int D = p.head_dim;
  const int cpr = (D + 3) >> 2;
  const int64_t rows = (int64_t)p.batch * p.heads_kv * p.seqlen_k;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= rows * cpr) return;
  const int64_t row = idx / cpr;
  const int d0 = (int)(idx - row * cpr) * 4;
  const int kj = (int)(row % p.seqlen_k);
  const int64_t bh = row / p.seqlen_k;
  const int hkv = (int)(bh % p.heads_kv), b = (int)(bh / p.heads_kv);
  const int64_t half = (int64_t)nsplit * rows * D;
  float a[4] = {0.f, 0.f, 0.f, 0.f}, c[4] = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < nsplit; ++s) {
    const float* pk = p.dkv_workspace + ((int64_t)s * rows + row) * D + d0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (d0 + j < D) {
        a[j] += pk[j];
        c[j] += pk[half + j];
      }
  }
  uint16_t* dkrow = (uint16_t*)p.dk + b * p.dk_stride[0] + hkv * p.dk_stride[2] + (int64_t)kj * p.dk_stride[1];
  uint16_t* dvrow = (uint16_t*)p.dv + b * p.dv_stride[0] + hkv * p.dv_stride[2] + (int64_t)kj * p.dv_stride[1];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (d0 + j < D) {
      dkrow[d0 + j] = E::from_f32(a[j] * p.softmax_scale);
      dvrow[d0 + j] = E::from_f32(c[j]);
    }
}

// ---------------------------------------------------------------------------------------------
template <int DT>
struct DqCfg {
  static constexpr int NW = 4;  // two independent workgroups per CU (measured faster than 8 waves)
  static constexpr int kWavesPerSimd = DT >= 256 ? 1 : 2;
};

// dQ: one workgroup = 4 waves = 128 query rows of one (batch, q-head); K/V tiles of 64 keys in
// LDS (double buffered).  Per tile and wave:
//   S^T, dP^T [key][q]   2 x (8 + 8) MFMA (A = K / V row fragments, B = Q / dO in VGPRs)
//   dQ^T[d][q] += K^T dS^T   NDT*4 MFMA (A = K^T via ds_read_b64_tr_b16)
// BIASK: 0 no bias; 1 any bias, read element by element from global memory; 16 / 17 an fp16 /
// bf16 bias with 16-byte aligned rows, staged per wave by LDS-DMA like the forward's
// (fwd_pipe_kernel.h): each wave's [32 rows x 64 keys] bias tile of tile i goes out first at the
// top of tile i and is waited for (counted vmcnt, the next K/V tile left in flight) right before
// the softmax gradient of its first key half.
#ifndef FA2_DQ_BIAS_WPS
#define FA2_DQ_BIAS_WPS 2
#endif
template <bool BF16, int DT, bool CAUSAL, int BIASK, bool DROPOUT, bool ALIGNED, bool DQF32>
__global__ void __launch_bounds__(DqCfg<DT>::NW * 64, BIASK != 0 && DT == 128 ? FA2_DQ_BIAS_WPS : DqCfg<DT>::kWavesPerSimd)
    dq_kernel(const fa2_bwd_args p) {
  using E = Elem<BF16>;
  constexpr bool BIAS = BIASK != 0, BIASL = BIASK >= 16;
  constexpr int NW = DqCfg<DT>::NW;
  constexpr int NT = NW * 64;
  constexpr int BM = NW * 32, BN = 64;
  constexpr int KS = DT / 16;
  constexpr int NDT = DT / 32;
  constexpr int TILE = BN * DT * 2;
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE + (BIASL ? NW * kBiasTile : 0)];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r32 = lane & 31, hh = lane >> 5;
  char* const bw = smem + 4 * TILE + w * kBiasTile;  // this wave's bias tile (BIASL)
  // work items head-major per XCD (xcd_item), heaviest first; under a causal mask a workgroup runs
  // a mirrored pair of row blocks of one head (nmb-1-j, then j: equal causal work per workgroup)
  const int nmb = (p.seqlen_q + BM - 1) / BM;
  constexpr bool PAIR = CAUSAL;
  const int per_bh = PAIR ? (nmb + 1) / 2 : nmb;
  const int item = xcd_item(blockIdx.x, gridDim.x);
  const int bh = item / per_bh;
  const int mbi = item - bh * per_bh;
  const int nrep = PAIR && nmb - 1 - mbi != mbi ? 2 : 1;
  for (int rep = 0; rep < nrep; ++rep) {
  if (rep > 0) __syncthreads();  // every wave is past the first item's LDS epilogue
  const int mb = PAIR ? (rep == 0 ? nmb - 1 - mbi : mbi) : (CAUSAL ? (nmb - 1 - mbi) : mbi);
  const int b = bh / p.heads_q, hq = bh - b * p.heads_q;
  const int hkv = hq / (p.heads_q / p.heads_kv);
  int Lq = p.seqlen_q, Lk = p.seqlen_k;
  if (p.cu_seqlens) Lq = Lk = p.cu_seqlens[b + 1] - p.cu_seqlens[b];
  const int D = p.head_dim;
  const int diag = Lk - Lq;
  const int m0 = mb * BM;
  const int mw0 = m0 + 32 * w;
  const int qi = mw0 + r32;
  const float scale = p.softmax_scale, scale2 = scale * kLog2e;

  const uint16_t* kg = (const uint16_t*)p.k + b * p.k_stride[0] + hkv * p.k_stride[2];
  const uint16_t* vg = (const uint16_t*)p.v + b * p.v_stride[0] + hkv * p.v_stride[2];
  int n_end = 0;
  if (m0 < Lq) {
    n_end = Lk;
    if (CAUSAL) n_end = min(Lk, m0 + BM + diag);
    n_end = max(n_end, 0);
  }
  const int ntiles = (n_end + BN - 1) / BN;
  auto kt = [&](int buf) { return smem + buf * 2 * TILE; };
  auto vt = [&](int buf) { return smem + TILE + buf * 2 * TILE; };
  // buffer-resource LDS-DMA, rows past Lk zero-filled; K and V row strides are equal on the
  // aligned path (api.hip), so one set of lane offsets serves both
  BufStager<DT, BN, NT> kst;
  int mrows = 0;
  if (ALIGNED) {
    kst.init(tid, p.k_stride[1], D);
    mrows = BufStager<DT, BN, NT>::max_rows(p.k_stride[1]);
  }
  auto stage_kv = [&](int buf, int n) {
    if constexpr (ALIGNED) {
      kst.issue(kt(buf), kg, p.k_stride[1], n, Lk, mrows);
      kst.issue(vt(buf), vg, p.v_stride[1], n, Lk, mrows);
    } else {
      stage_tile<DT, BN, NT, false>(kt(buf), kg, p.k_stride[1], n, Lk, D, tid);
      stage_tile<DT, BN, NT, false>(vt(buf), vg, p.v_stride[1], n, Lk, D, tid);
    }
  };
  // this wave's bias tiles (BIASL): [32 rows from mw0][64 keys], rows past seqlen_q read as zeros
  using BiasStager = BufStager<64, 32, 64>;
  BiasStager bst;
  const uint16_t* bg = nullptr;
  int brows = 0;
  if constexpr (BIASL) {
    int ln = lane;  // opaque: the offsets are not hoisted out of the item loop (spilled across it)
    asm volatile("" : "+v"(ln));
    bst.init(ln, p.bias_stride[2], 64);
    brows = BiasStager::max_rows(p.bias_stride[2]);
    bg = (const uint16_t*)p.bias + b * p.bias_stride[0] + hq * p.bias_stride[1];
  }
  auto bias_issue = [&](int n) {
    if constexpr (BIASL) {
      const i32x4 r = bias_tile_rsrc(bg + n, p.bias_stride[2], mw0, p.seqlen_q, brows, p.seqlen_k - n, 64);
#pragma unroll
      for (int it = 0; it < BiasStager::kIters; ++it) bst.piece(bw, r, it);
    }
  };
  // bias of the current tile landed; `later` (the next K/V tile's pieces) may stay in flight
  constexpr int kKV = 2 * BufStager<DT, BN, NT>::kIters;
  auto bias_wait = [&](bool later) {
    if constexpr (BIASL) {
      if (later) {
        if constexpr (kKV == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else if constexpr (kKV == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else vm_wait_all();
      } else {
        vm_wait_all();
      }
    }
  };
  auto bias_frag = [&](int h, int g) -> u32x2 {
    if constexpr (BIASL) return bias_tile_frag(bw, r32, hh, h, g);
    else return u32x2{0u, 0u};
  };
  if (ntiles > 0) stage_kv(0, 0);

  const bool qvalid = qi < Lq;
  u32x4 qf[KS], of[KS];
  {
    const uint16_t* qrow = (const uint16_t*)p.q + b * p.q_stride[0] + hq * p.q_stride[2] + (int64_t)(qvalid ? qi : 0) * p.q_stride[1];
    const uint16_t* orow = (const uint16_t*)p.dout + b * p.do_stride[0] + hq * p.do_stride[2] + (int64_t)(qvalid ? qi : 0) * p.do_stride[1];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      qf[ks] = load_row_frag<ALIGNED>(qrow, 16 * ks + 8 * hh, D, qvalid);
      of[ks] = load_row_frag<ALIGNED>(orow, 16 * ks + 8 * hh, D, qvalid);
    }
  }
  const int64_t srow = (int64_t)bh * p.lse_row_stride;
  const float lse_i = qvalid ? p.lse[srow + qi] : 0.f;
  // delta_i = rowsum(O * dO) of this lane's row (/root/reference/src/backward/compute_delta.py:
  // 17-73), computed here from the dO fragments already in registers and published to the
  // workspace for dkdv_kernel, which runs after this kernel (rows [Lq, grid rows) get 0)
  float del_i;
  {
    const uint16_t* orow = (const uint16_t*)p.o + b * p.o_stride[0] + hq * p.o_stride[2] + (int64_t)(qvalid ? qi : 0) * p.o_stride[1];
    float part = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const u32x4 ov = load_row_frag<ALIGNED>(orow, 16 * ks + 8 * hh, D, qvalid);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        part = fmaf(E::to_f32((uint16_t)(ov[j] & 0xFFFF)), E::to_f32((uint16_t)(of[ks][j] & 0xFFFF)), part);
        part = fmaf(E::to_f32((uint16_t)(ov[j] >> 16)), E::to_f32((uint16_t)(of[ks][j] >> 16)), part);
      }
    }
    del_i = qvalid ? half_sum(part) : 0.f;
    if (hh == 0 && qi < p.lse_row_stride) p.delta[srow + qi] = -del_i;  // negated (delta_kernel)
  }

  f32x16 acc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) acc[dt] = zero16();

  __builtin_amdgcn_s_waitcnt(0);  // prologue: Q fragments (compiler-tracked) + first tiles
  __syncthreads();

  // key kj visible to this lane's row iff kj < lim_lane (0 for padded rows)
  const int lim_lane = !qvalid ? 0 : (CAUSAL ? min(Lk, qi + diag + 1) : Lk);
  const float sc = BIAS ? 1.f : scale2;
  const float nlse = -lse_i;
  // dropout: Philox offset of (b, hq, qi, key 0), as the forward (fwd_kernel.h)
  uint64_t drop_row = 0;
  float inv_keep = 1.f;
  if (DROPOUT) {
    const uint64_t cu0 = p.cu_seqlens ? (uint64_t)p.cu_seqlens[b] : 0;
    drop_row = (uint64_t)Lk * (cu0 + (uint64_t)Lq * ((uint64_t)hq + (uint64_t)p.heads_q * (p.cu_seqlens ? 0 : b))) +
               (uint64_t)qi * (uint64_t)Lk;
    inv_keep = 1.f / (1.f - p.dropout_p);
  }

  // dropout keep words of this lane's row for the two 32-key halves of a tile (the forward's saved
  // mask, tiled layout of fa2_amd.h), loaded one tile ahead: the loop's vm_wait_all retires them
  uint32_t mwc[2] = {0u, 0u}, mwn[2] = {0u, 0u};
  auto load_mw = [&](int n0, uint32_t* out) {
    if constexpr (DROPOUT) {
      if (p.dropout_mask) {
        const int nrb = (p.seqlen_q + 31) >> 5, ncw = (p.seqlen_k + 31) >> 5;
        const int64_t rowbase = ((int64_t)(b * p.heads_q + hq) * nrb + (qi >> 5)) * ncw;
#pragma unroll
        for (int t = 0; t < 2; ++t)
          out[t] = (qvalid && n0 + 32 * t < p.seqlen_k) ? p.dropout_mask[(rowbase + ((n0 >> 5) + t)) * 32 + (qi & 31)] : 0u;
      }
    }
  };
  // one 64-key tile: S^T and dP^T for both 32-key halves first, then the softmax-gradient
  // VALU of each half beside the other half's MFMAs, then dQ^T += K^T dS^T.
  auto tile = [&](auto mask_c, const char* K, const char* V, int n0, bool later) {
    constexpr bool MASK = decltype(mask_c)::value;
    const int rel = lim_lane - n0 - 4 * hh;
    bias_wait(later);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if (MASK && !(n0 + 32 * t < Lk && (!CAUSAL || n0 + 32 * t <= mw0 + 31 + diag))) continue;
      f32x16 s = zero16(), dp = zero16();
      {
        constexpr int L = kDqLead < KS ? kDqLead : KS;
        u32x4 fk[KS], fv[KS];
        auto rd = [&](int ks) {
          fk[ks] = lds_row_frag<DT, BN>(K, 32 * t, r32, ks, hh);
          fv[ks] = lds_row_frag<DT, BN>(V, 32 * t, r32, ks, hh);
        };
#pragma unroll
        for (int j = 0; j < L; ++j) rd(j);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          if (ks + L < KS) rd(ks + L);
          s = E::mfma(fk[ks], qf[ks], s);
          dp = E::mfma(fv[ks], of[ks], dp);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      u32x4 dsp[2];
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        float dsv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int i = 8 * sp + j;
          const int o = 32 * t + (i & 3) + 8 * (i >> 2);
          float x = s[i];
          if constexpr (BIASL) {
            x = fmaf(x, scale2, kLog2e * bias_elem<BIASK>(bias_frag(t, i >> 2), i & 3));
          } else if constexpr (BIAS) {
            const int kj = n0 + o + 4 * hh;
            const int kc = kj < Lk ? kj : Lk - 1;
            const int qc = qvalid ? qi : 0;
            x = fmaf(x, scale2, kLog2e * load_bias(p.bias, b * p.bias_stride[0] + hq * p.bias_stride[1] +
                                                             (int64_t)qc * p.bias_stride[2] + kc, p.bias_dtype));
          }
          float pr = __builtin_amdgcn_exp2f(fmaf(x, sc, nlse));
          if (MASK) pr = o < rel ? pr : 0.f;
          if (DROPOUT) {  // dS = P (dP~ M / (1 - p) - delta), the forward's keep mask M
            // the forward's keep mask M (fully unrolled here: the rolled dropout_keep16 measured
            // 8 % slower in this kernel, which does not spill either way)
            bool keep;
            if (p.dropout_mask) {  // the forward's saved bits (loaded a tile ahead)
              keep = (mwc[t] >> ((i & 3) + 8 * (i >> 2) + 4 * hh)) & 1u;
            } else {
              const uint64_t kjj = (uint64_t)(n0 + o + 4 * hh);
              keep = philox_uniform(p.dropout_seed, drop_row + kjj) > p.dropout_p;
            }
            dsv[j] = pr * (dp[i] * (keep ? inv_keep : 0.f) - del_i);
          } else {
            dsv[j] = pr * (dp[i] - del_i);  // softmax_scale is applied to dQ once, at the end
          }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) dsp[sp][j] = E::pack2(dsv[2 * j], dsv[2 * j + 1]);
      }
      __builtin_amdgcn_sched_barrier(0);
      {
        constexpr int N = 2 * NDT, L = 2 * kDqLead < N ? 2 * kDqLead : N;
        u32x4 fr[N];
        auto rd = [&](int m) { return lds_tr_frag<DT, BN>(K, 32 * t + 16 * (m / NDT), 32 * (m % NDT), lane); };
#pragma unroll
        for (int j = 0; j < L; ++j) fr[j] = rd(j);
#pragma unroll
        for (int m = 0; m < N; ++m) {
          if (m + L < N) fr[m + L] = rd(m + L);
          acc[m % NDT] = E::mfma(fr[m], dsp[m / NDT], acc[m % NDT]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
  };

  // Interior tiles (no mask, no bias, no dropout): the two 32-key halves are software
  // pipelined inside the tile so that every softmax-gradient VALU op sits beside an MFMA of
  // the same wave:
  //   [S, dP of half 0] [S, dP of half 1 | dS of half 0] [dQ of half 0 | dS 0-7 of half 1]
  //   [dQ of half 1 | dS 8-15 of half 1 beside its first steps]
  auto tile_pipe = [&](const char* K, const char* V, bool later) {
    constexpr int L = kDqPipeLead;  // two score pairs live: one step of fragments in flight
    f32x16 s[2], dp[2];
    u32x4 dsp[2][2];
    u32x2 bz[2];  // bias of the current 4-key group (BIASL), read one element group ahead
    // dS of element e (0..15) of half t -> packed pair in dsp[t]
    float dsv_lo = 0.f;
    auto ds_elem = [&](int t, int e) {
      float x = s[t][e], u = sc;
      if constexpr (BIASL) {
        if ((e & 3) == 0) bz[t] = bias_frag(t, e >> 2);
        x = fmaf(x, p.softmax_scale, bias_elem<BIASK>(bz[t], e & 3));
        u = kLog2e;
      }
      const float pr = __builtin_amdgcn_exp2f(fmaf(x, u, nlse));
      const float d = pr * (dp[t][e] - del_i);
      if (e & 1) dsp[t][e >> 3][(e & 7) >> 1] = E::pack2(dsv_lo, d);
      else dsv_lo = d;
    };
    // S and dP of half t: 2 KS fenced steps; step k of the S/dP chains, VALU hook per step
    auto sdp = [&](int t, auto hook) {
      u32x4 fk[KS], fv[KS];
      auto rd = [&](int ks) {
        fk[ks] = lds_row_frag<DT, BN>(K, 32 * t, r32, ks, hh);
        fv[ks] = lds_row_frag<DT, BN>(V, 32 * t, r32, ks, hh);
      };
#pragma unroll
      for (int j = 0; j < L; ++j) rd(j);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if (ks + L < KS) rd(ks + L);
        s[t] = E::mfma(fk[ks], qf[ks], ks == 0 ? zero16() : s[t]);
        hook(2 * ks);
        __builtin_amdgcn_sched_barrier(0);
        dp[t] = E::mfma(fv[ks], of[ks], ks == 0 ? zero16() : dp[t]);
        hook(2 * ks + 1);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    // dQ^T += K^T dS^T of half t: 2 NDT fenced steps with a VALU hook per step
    auto dq_half = [&](int t, auto hook) {
      constexpr int N = 2 * NDT, LL = 2 * L < N ? 2 * L : N;
      u32x4 fr[N];
      auto rd = [&](int m) { return lds_tr_frag<DT, BN>(K, 32 * t + 16 * (m / NDT), 32 * (m % NDT), lane); };
#pragma unroll
      for (int j = 0; j < LL; ++j) fr[j] = rd(j);
#pragma unroll
      for (int m = 0; m < N; ++m) {
        if (m + LL < N) fr[m + LL] = rd(m + LL);
        acc[m % NDT] = E::mfma(fr[m], dsp[t][m / NDT], acc[m % NDT]);
        hook(m);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    constexpr int SDP_STEPS = 2 * KS, DQ_STEPS = 2 * NDT;
    sdp(0, [](int) {});
    bias_wait(later);
    sdp(1, [&](int st) {  // 16 dS elements of half 0 over the S/dP steps of half 1
#pragma unroll
      for (int e = st * 16 / SDP_STEPS; e < (st + 1) * 16 / SDP_STEPS; ++e) ds_elem(0, e);
    });
    // dS of half 1: elements 0-7 (packed fragment dsp[1][0]) beside the dQ steps of half 0,
    // elements 8-15 (dsp[1][1], first read at step DQ_STEPS / 2 of dq_half(1)) beside the dQ
    // steps of half 1 that read dsp[1][0].  (All 16 over half 0's dQ steps: 1.8 % slower causal,
    // profiles/r02_ab_dq_spread.txt.)
    dq_half(0, [&](int st) {
#pragma unroll
      for (int e = st * 8 / DQ_STEPS; e < (st + 1) * 8 / DQ_STEPS; ++e) ds_elem(1, e);
    });
    dq_half(1, [&](int st) {
      constexpr int H = DQ_STEPS / 2;
      if (st < H) {
#pragma unroll
        for (int e = 8 + st * 8 / H; e < 8 + (st + 1) * 8 / H; ++e) ds_elem(1, e);
      }
    });
  };

  load_mw(0, mwc);
  for (int it = 0; it < ntiles; ++it) {
    const int cur = it & 1;
    const int n0 = it * BN;
    const bool dead = CAUSAL && (n0 > mw0 + 31 + diag);
    // (the bias tile first: its counted wait leaves the next K/V tile in flight)
    if (!dead) bias_issue(n0);
    const bool later = it + 1 < ntiles;
    if (DROPOUT && later) load_mw(n0 + BN, mwn);
    if (later) stage_kv(cur ^ 1, n0 + BN);
    const bool need_mask = (n0 + BN > Lk) || (mw0 + 31 >= Lq) || (CAUSAL && n0 + BN - 1 > mw0 + diag);
    if (!dead) {
      if (need_mask)
        tile(std::true_type{}, kt(cur), vt(cur), n0, later);
      else if constexpr ((!BIAS || BIASL) && !DROPOUT)
        tile_pipe(kt(cur), vt(cur), later);
      else
        tile(std::false_type{}, kt(cur), vt(cur), n0, later);
    }
    vm_wait_all();
    __syncthreads();
    if constexpr (DROPOUT) {
      mwc[0] = mwn[0];
      mwc[1] = mwn[1];
    }
  }

  if constexpr (ALIGNED && !DQF32) {
    // the last tile's barrier is behind every wave: the K/V buffers hold the staging images
    uint16_t* q0 = (uint16_t*)p.dq + b * p.dq_stride[0] + hq * p.dq_stride[2] + (int64_t)mw0 * p.dq_stride[1];
    store_rows_lds<BF16, DT>(smem + w * 32 * DT * 2, acc, scale, qvalid, q0, p.dq_stride[1],
                             min(32, p.seqlen_q - mw0), D, lane);
  } else if (qi < p.seqlen_q) {
    const bool ok = qvalid;
    char* base = (char*)p.dq;
    const int esz = DQF32 ? 4 : 2;
    char* row = base + (int64_t)esz * (b * p.dq_stride[0] + hq * p.dq_stride[2] + (int64_t)qi * p.dq_stride[1]);
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d0 = 32 * dt + 8 * g4 + 4 * hh;
        float a[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] = ok ? acc[dt][4 * g4 + j] * scale : 0.f;
        if (DQF32) {
          float* r = (float*)row;
          if (ALIGNED) {
            if (d0 < D) *(f32x4*)(r + d0) = f32x4{a[0], a[1], a[2], a[3]};
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) if (d0 + j < D) r[d0 + j] = a[j];
          }
        } else {
          uint16_t* r = (uint16_t*)row;
          if (ALIGNED) {
            if (d0 < D) *(u32x2*)(r + d0) = u32x2{E::pack2(a[0], a[1]), E::pack2(a[2], a[3])};
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) if (d0 + j < D) r[d0 + j] = E::from_f32(a[j]);
          }
        }
      }
    }
  }
  }
}

// ---------------------------------------------------------------------------------------------
// Bias gradient (ABI 5; the reference has none, /root/reference/src/wrapper.py:86):
//   dbias[b', h', i, j] = sum over the (batch, q-head) pairs the bias broadcasts to of
//                         dS[b, hq, i, j] = P (dP~ - delta),   P = exp2(s scale log2e + bias log2e - LSE2)
// (dP~ = dP M / (1 - p) under dropout, M the forward's keep mask), in fp32, deterministic.
// One workgroup owns a 128-row x (64 kDbiasChunk)-key block of one bias slice (b', h') and sums
// the pairs of its broadcast group into registers, pair after pair in index order, then stores
// the block once: no read-modify-write of the output, and the memory is the bias-shaped output
// alone -- no [B, Hq, Sq, Sk] buffer.  The bias values are the same for every pair of the group
// (the summed dimensions have stride 0), so the block's bias is read once, into registers.
// Per pair the structure is dq_kernel's (query on the lane, Q / dO in registers, 64-key K/V tiles
// in LDS): S^T = K Q^T and dP^T = V dO^T (the same products as compute_dq.py:38-69), without the
// dQ GEMM; the next K/V tile and the next pair's Q/dO rows stream into LDS while the current
// pair computes.
// delta comes from the dQ (or delta) kernel that ran before (-rowsum(O dO), negated).
// 64-key tiles per dbias workgroup.  One: the block's sums and bias (32 + 32 fp32 per lane) leave
// the arch VGPRs room to read the K/V fragments ahead of the MFMAs; with two (64 + 64) the
// compiler read each fragment just before its MFMA and waited out the LDS latency every time.
#ifndef FA2_DBIAS_CHUNK
#define FA2_DBIAS_CHUNK 1
#endif
constexpr int kDbiasChunk = FA2_DBIAS_CHUNK;

// XCD-aware block order: workgroup g runs on XCD g % 8 as that XCD's (g / 8)-th; the blocks go
// out in 8 x 8 squares of (row block, key chunk), so the workgroups an XCD runs together share
// 8 row blocks' Q / dO and 8 key chunks' K / V in its L2 (each read by 8 workgroups instead of
// 1).  Square (r, c) goes to XCD (r + c) % 8: anti-diagonals, so that the causal triangle's
// squares spread evenly over the XCDs (square columns would give XCD 0 fifteen times XCD 7's
// work).  The square columns are padded to a multiple of 8 (dbias_blocks); padding
// workgroups get mb = -1.
// (grids under 32 x 32 blocks use 1 x 1 "squares": whole squares would crowd them onto few XCDs)
__host__ __device__ inline int dbias_side(int nmb, int nkc) { return nmb >= 32 && nkc >= 32 ? 8 : 1; }
__host__ __device__ inline int dbias_blocks(int nmb, int nkc) {  // the padded grid
  const int e = dbias_side(nmb, nkc);
  const int sqr = (nmb + e - 1) / e, sqk = (nkc + e - 1) / e;
  return sqr * ((sqk + 7) / 8 * 8) * e * e;
}
FA2_DEV void dbias_block(int g, int nmb, int nkc, int& mb, int& kc) {
  const int e = dbias_side(nmb, nkc);
  const int x = g & 7, j = g >> 3;
  const int q = j / (e * e), within = j % (e * e);
  const int sqk = (nkc + e - 1) / e, per_row = (sqk + 7) / 8;
  const int r = q / per_row, m = q - r * per_row;
  const int c = ((x - r) & 7) + 8 * m;  // (r + c) % 8 == x
  mb = r * e + within / e;
  kc = c * e + within % e;
  if (c >= sqk || mb >= nmb || kc >= nkc) mb = -1;
}

template <bool BF16, int DT, bool CAUSAL, bool DROPOUT, bool ALIGNED>
__global__ void __launch_bounds__(256, DT <= 64 && !DROPOUT ? 2 : 1) dbias_kernel(const fa2_bwd_args p) {
  using E = Elem<BF16>;
  constexpr int NT = 256, BM = 128, BN = 64, C = kDbiasChunk;
  constexpr int KS = DT / 16;
  constexpr int TILE = BN * DT * 2;
  // D <= 128: the pair's Q / dO rows go through LDS (coalesced 16-byte DMA pieces, then one
  // fragment read per lane): loaded straight into the row-per-lane registers, every load
  // instruction would touch 32 rows x 32 bytes and the address unit, not the MFMAs, would set
  // the pace.  D = 256 loads them into registers directly (the LDS would not hold both tiles).
  constexpr bool QLDS = DT <= 128;
  constexpr int QTILE = QLDS ? BM * DT * 2 : 0;
  // K/V tiles: a ring of 3 (D <= 128; staged two steps ahead) or 2 (D = 256, one step ahead)
  constexpr int RING = QLDS ? 3 : 2;
  // the deep pipeline counts its loads: fixed VMEM instructions per step (LDS-DMA pieces per
  // K/V tile and per Q/dO block; the two -LSE / -delta loads land before those go out)
  constexpr int KV_VM = 2 * BufStager<DT, BN, NT>::kIters, QO_VM = 2 * BufStager<DT, BM, NT>::kIters;
  constexpr bool DEEP = QLDS && ALIGNED && !DROPOUT;
  __shared__ __attribute__((aligned(16))) char smem[2 * RING * TILE + 2 * QTILE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const int nkt = (p.seqlen_k + BN - 1) / BN;        // key tiles of the output rows
  const int nkc = (nkt + C - 1) / C;
  int mb, kc;
  dbias_block(blockIdx.x, (p.seqlen_q + BM - 1) / BM, nkc, mb, kc);
  if (mb < 0) return;                                // grid padding
  const int t0 = kc * C, t1 = min(nkt, t0 + C);     // this workgroup's key tiles
  const int Hb = p.bias_stride[1] != 0 ? p.heads_q : 1;
  const int slice = blockIdx.y;                       // (b', h') of the bias
  const int bb = slice / Hb, hb = slice - bb * Hb;
  const bool sum_b = p.bias_stride[0] == 0, sum_h = p.bias_stride[1] == 0;
  const int nb = sum_b ? p.batch : 1, nh = sum_h ? p.heads_q : 1;
  const int np = nb * nh;
  const int D = p.head_dim;
  const int m0 = mb * BM;
  const int qi = m0 + 32 * w + r32;                  // this lane's row
  const float scale2 = p.softmax_scale * kLog2e;
  const bool row_in = qi < p.seqlen_q;

  auto kt = [&](int buf) { return smem + buf * 2 * TILE; };
  auto vt = [&](int buf) { return smem + TILE + buf * 2 * TILE; };
  char* const qt = smem + 2 * RING * TILE;
  char* const ot = smem + 2 * RING * TILE + QTILE;
  BufStager<DT, BN, NT> kst;
  BufStager<DT, BM, NT> qst, ost;
  int mrows = 0, qrows = 0, orows = 0;
  if (ALIGNED) {
    kst.init(tid, p.k_stride[1], D);
    mrows = BufStager<DT, BN, NT>::max_rows(p.k_stride[1]);
    if (QLDS) {
      qst.init(tid, p.q_stride[1], D);
      ost.init(tid, p.do_stride[1], D);
      qrows = BufStager<DT, BM, NT>::max_rows(p.q_stride[1]);
      orows = BufStager<DT, BM, NT>::max_rows(p.do_stride[1]);
    }
  }

  // element i of half t of tile c: key (t0 + c) 64 + 32 t + 8 (i / 4) + 4 hh + i % 4
  float acc[C][2][16], bl[C][2][16];
  {
    const int64_t brow = bb * p.bias_stride[0] + hb * p.bias_stride[1] + (int64_t)(row_in ? qi : 0) * p.bias_stride[2];
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int kj = (t0 + c) * BN + 32 * t + (i & 3) + 8 * (i >> 2) + 4 * hh;
          acc[c][t][i] = 0.f;
          bl[c][t][i] = kLog2e * load_bias(p.bias, brow + (kj < p.seqlen_k ? kj : p.seqlen_k - 1), p.bias_dtype);
        }
  }

  // The pair cursor: the pair's index with its (batch, q-head, kv-head) carried along, so a step
  // moves it by increments (index -> (b, hq) -> kv-head by division costs ~25 instructions per
  // division, seven per step, on a one-wave-per-SIMD kernel whose step is short).  Pair order:
  // index = b nh + hq over the summed dims (as the dims of the bias's broadcast group).
  const int group = p.heads_q / p.heads_kv;
  struct Cur {
    int i, b, hq, hkv, gi;  // gi = hq - hkv group
  };
  Cur first;
  first.i = 0;
  first.b = sum_b ? 0 : bb;
  first.hq = sum_h ? 0 : hb;
  first.hkv = first.hq / group;
  first.gi = first.hq - first.hkv * group;
  auto step_cur = [&](Cur c) {
    ++c.i;
    if (sum_h) {
      if (++c.gi == group) {
        c.gi = 0;
        ++c.hkv;
      }
      if (++c.hq == nh) {
        c.hq = c.hkv = c.gi = 0;
        ++c.b;
      }
    } else {
      ++c.b;  // (a single pair when neither dim is summed: past the end)
    }
    return c;
  };
  // the pair's visible key tiles are [t0, tend); a pair with none adds nothing
  struct Pair {
    int b, hq, hkv, Lq, Lk, tend;
  };
  auto pair_of = [&](const Cur& c) {
    Pair r;
    r.b = c.b;
    r.hq = c.hq;
    r.hkv = c.hkv;
    r.Lq = p.seqlen_q;
    r.Lk = p.seqlen_k;
    if (p.cu_seqlens) r.Lq = r.Lk = p.cu_seqlens[r.b + 1] - p.cu_seqlens[r.b];
    int n_end = 0;
    if (m0 < r.Lq) n_end = max(CAUSAL ? min(r.Lk, m0 + BM + r.Lk - r.Lq) : r.Lk, 0);
    r.tend = min(t1, (n_end + BN - 1) / BN);
    return r;
  };
  auto next_visible = [&](Cur c) {
    while (c.i < np && pair_of(c).tend <= t0) c = step_cur(c);
    return c;
  };
  auto stage_kv = [&](int buf, const Pair& r, int n) {
    const uint16_t* kg = (const uint16_t*)p.k + r.b * p.k_stride[0] + r.hkv * p.k_stride[2];
    const uint16_t* vg = (const uint16_t*)p.v + r.b * p.v_stride[0] + r.hkv * p.v_stride[2];
    if constexpr (ALIGNED) {
      kst.issue(kt(buf), kg, p.k_stride[1], n, r.Lk, mrows);
      kst.issue(vt(buf), vg, p.v_stride[1], n, r.Lk, mrows);
    } else {
      stage_tile<DT, BN, NT, false>(kt(buf), kg, p.k_stride[1], n, r.Lk, D, tid);
      stage_tile<DT, BN, NT, false>(vt(buf), vg, p.v_stride[1], n, r.Lk, D, tid);
    }
  };
  auto q_base = [&](const Pair& r) { return (const uint16_t*)p.q + r.b * p.q_stride[0] + r.hq * p.q_stride[2]; };
  auto o_base = [&](const Pair& r) { return (const uint16_t*)p.dout + r.b * p.do_stride[0] + r.hq * p.do_stride[2]; };
  auto stage_qo = [&](const Pair& r) {  // the pair's 128 Q / dO rows of this block into LDS
    if constexpr (QLDS) {
      if constexpr (ALIGNED) {
        qst.issue(qt, q_base(r), p.q_stride[1], m0, r.Lq, qrows);
        ost.issue(ot, o_base(r), p.do_stride[1], m0, r.Lq, orows);
      } else {
        stage_tile<DT, BM, NT, false>(qt, q_base(r), p.q_stride[1], m0, r.Lq, D, tid);
        stage_tile<DT, BM, NT, false>(ot, o_base(r), p.do_stride[1], m0, r.Lq, D, tid);
      }
    }
  };
  // the lane's row of the pair's LSE2 and -delta (row 0 exists: Lq > 0)
  auto rowstats = [&](const Pair& r, float& l, float& d) {
    const int64_t srow = (int64_t)(r.b * p.heads_q + r.hq) * p.lse_row_stride + (qi < r.Lq ? qi : 0);
    l = p.lse[srow];
    d = p.delta[srow];
  };

  Cur cur = next_visible(first);
  int buf = 0;
  // staging cursor (pair, tile) of the K/V ring, RING - 1 steps ahead of the compute; past the
  // last pair it re-stages a tile of the current pair (unused) so every step issues the same loads
  Cur scur = cur;
  int sc = 0;
  auto advance = [&]() {
    if (++sc == C) {
      sc = 0;
      scur = next_visible(step_cur(scur));
    }
  };
  float lse_v = 0.f, del_v = 0.f;
  if (cur.i < np) {
    const Pair r = pair_of(cur);
    rowstats(r, lse_v, del_v);
    stage_qo(r);
    for (int k = 0; k < RING - 1; ++k) {
      stage_kv(k, scur.i < np ? pair_of(scur) : r, t0 * BN + (scur.i < np ? sc : 0) * BN);
      advance();
    }
  }
  vm_wait_all();
  __syncthreads();
  while (cur.i < np) {
    const Pair r = pair_of(cur);
    const Cur nxc = next_visible(step_cur(cur));
    const bool has_next = nxc.i < np;
    const int b = r.b, hq = r.hq, Lq = r.Lq, Lk = r.Lk;
    const bool qvalid = qi < Lq;
    // this pair's LSE2 / -delta were loaded a step ago: landed before this step's LDS-DMA goes out
    // (the compiler's own wait for them counts no LDS-DMA: waited at their use it would be a
    // vmcnt(0) that drains this step's prefetches)
    asm volatile("" : "+v"(lse_v), "+v"(del_v));
    const float nlse = qvalid ? -lse_v : 0.f;
    const float ndel = qvalid ? del_v : 0.f;  // the workspace holds -delta
    // the next pair's go out ahead of this step's LDS-DMA, so the step-end wait retires them
    // (loaded at the step start and waited at once, each step had exposed one load latency)
    float lse_n = 0.f, del_n = 0.f;
    if (has_next) rowstats(pair_of(nxc), lse_n, del_n);
    u32x4 qf[KS], of[KS];
    if constexpr (QLDS) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        qf[ks] = lds_row_frag<DT, BM>(qt, 32 * w, r32, ks, hh);
        of[ks] = lds_row_frag<DT, BM>(ot, 32 * w, r32, ks, hh);
      }
    } else {
      const uint16_t* qrow = q_base(r) + (int64_t)(qvalid ? qi : 0) * p.q_stride[1];
      const uint16_t* orow = o_base(r) + (int64_t)(qvalid ? qi : 0) * p.do_stride[1];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        qf[ks] = load_row_frag<ALIGNED>(qrow, 16 * ks + 8 * hh, D, qvalid);
        of[ks] = load_row_frag<ALIGNED>(orow, 16 * ks + 8 * hh, D, qvalid);
      }
    }
    if constexpr (QLDS) {
      // every wave holds its fragments: the next pair's rows may overwrite the tiles
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
      __syncthreads();
      if (has_next) stage_qo(pair_of(nxc));
      else if (DEEP) stage_qo(r);  // (unused: keeps the step's load count)
    }
    const int lim_lane = !qvalid ? 0 : (CAUSAL ? min(Lk, qi + Lk - Lq + 1) : Lk);
    uint64_t drop_row = 0;
    float inv_keep = 1.f;
    if (DROPOUT) {
      const uint64_t cu0 = p.cu_seqlens ? (uint64_t)p.cu_seqlens[b] : 0;
      drop_row = (uint64_t)Lk * (cu0 + (uint64_t)Lq * ((uint64_t)hq + (uint64_t)p.heads_q * (p.cu_seqlens ? 0 : b))) +
                 (uint64_t)qi * (uint64_t)Lk;
      inv_keep = 1.f / (1.f - p.dropout_p);
    }

#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int it = t0 + c;
      if (RING == 3 || it < r.tend) {
        const int n0 = it * BN;
        if constexpr (RING == 3) {  // the tile RING - 1 steps ahead (every step of a pair runs)
          stage_kv(buf == 0 ? 2 : buf - 1, scur.i < np ? pair_of(scur) : r, (t0 + (scur.i < np ? sc : 0)) * BN);
          advance();
        } else {  // the next tile: this pair's, else the next visible pair's first
          if (it + 1 < r.tend) stage_kv(buf ^ 1, r, n0 + BN);
          else if (has_next) stage_kv(buf ^ 1, pair_of(nxc), t0 * BN);
        }
        const char* K = kt(buf);
        const char* V = vt(buf);
        const int rel = lim_lane - n0 - 4 * hh;
        // the tile's K / V fragments of both key halves, read ahead of the MFMAs (read next to
        // each MFMA, every one of them waited out the LDS latency)
        // (D = 256: read next to the MFMAs, the register file would not hold them)
        u32x4 kf[2][QLDS ? KS : 1], vf[2][QLDS ? KS : 1];
        if (QLDS && it < r.tend) {
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
              kf[t][QLDS ? ks : 0] = lds_row_frag<DT, BN>(K, 32 * t, r32, ks, hh);
              vf[t][QLDS ? ks : 0] = lds_row_frag<DT, BN>(V, 32 * t, r32, ks, hh);
            }
          __builtin_amdgcn_sched_barrier(0);  // (the scheduler would sink each read to its MFMA)
        }
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          if (it >= r.tend) break;  // a ring step over a tile this pair does not see
          uint32_t mwd = 0u;  // the forward's saved keep word of this row and key half
          if (DROPOUT && p.dropout_mask && qvalid && n0 + 32 * t < p.seqlen_k) {
            const int nrb = (p.seqlen_q + 31) >> 5, ncw = (p.seqlen_k + 31) >> 5;
            mwd = p.dropout_mask[((((int64_t)(b * p.heads_q + hq) * nrb + (qi >> 5)) * ncw + ((n0 >> 5) + t)) * 32) + (qi & 31)];
          }
          f32x16 s = zero16(), dp = zero16();
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            if constexpr (QLDS) {
              s = E::mfma(kf[t][ks], qf[ks], s);
              dp = E::mfma(vf[t][ks], of[ks], dp);
            } else {
              s = E::mfma(lds_row_frag<DT, BN>(K, 32 * t, r32, ks, hh), qf[ks], s);
              dp = E::mfma(lds_row_frag<DT, BN>(V, 32 * t, r32, ks, hh), of[ks], dp);
            }
          }
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int o = 32 * t + (i & 3) + 8 * (i >> 2);
            float pr = __builtin_amdgcn_exp2f(fmaf(s[i], scale2, bl[c][t][i]) + nlse);
            pr = o < rel ? pr : 0.f;
            float dpv = dp[i];
            if (DROPOUT) {
              const bool keep = p.dropout_mask ? ((mwd >> ((i & 3) + 8 * (i >> 2) + 4 * hh)) & 1u) != 0
                                               : philox_uniform(p.dropout_seed, drop_row + (uint64_t)(n0 + o + 4 * hh)) > p.dropout_p;
              dpv *= keep ? inv_keep : 0.f;
            }
            acc[c][t][i] += pr * (dpv + ndel);
          }
        }
        if constexpr (DEEP) {
          // all but the loads this step issued after what the next step needs: the next step's
          // tile, and at a pair's last step the next pair's Q / dO (issued at its first step,
          // before that step's K/V); s_waitcnt vmcnt(n): bits 3:0 and 15:14 of the count
          static_assert(KV_VM + QO_VM < 64, "vmcnt range");
          constexpr int n0c = KV_VM + QO_VM, n1c = KV_VM;
          if (c < C - 1)
            __builtin_amdgcn_s_waitcnt((n0c & 15) | ((n0c >> 4) << 14) | 0x0f70);
          else
            __builtin_amdgcn_s_waitcnt((n1c & 15) | ((n1c >> 4) << 14) | 0x0f70);
        } else {
          vm_wait_all();
        }
        __syncthreads();
        buf = RING == 3 ? (buf == 2 ? 0 : buf + 1) : buf ^ 1;
      }
    }
    cur = nxc;
    lse_v = lse_n;
    del_v = del_n;
  }

  // one store of the block (16-byte stores when the rows allow them: a group's 4 keys are contiguous)
  if (!row_in) return;
  float* drow = p.dbias + bb * p.dbias_stride[0] + hb * p.dbias_stride[1] + (int64_t)qi * p.dbias_stride[2];
  const bool vec4 = ((uintptr_t)p.dbias & 15) == 0 && p.dbias_stride[0] % 4 == 0 && p.dbias_stride[1] % 4 == 0 &&
                    p.dbias_stride[2] % 4 == 0;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    if (t0 + c >= t1) break;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int k0 = (t0 + c) * BN + 32 * t + 8 * g + 4 * hh;
        if (vec4 && k0 + 4 <= p.seqlen_k) {
          *(f32x4*)(drow + k0) = f32x4{acc[c][t][4 * g], acc[c][t][4 * g + 1], acc[c][t][4 * g + 2], acc[c][t][4 * g + 3]};
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (k0 + j < p.seqlen_k) drow[k0 + j] = acc[c][t][4 * g + j];
        }
      }
  }
}

// ---------------------------------------------------------------------------------------------
template <bool BF16>
static void launch_dkv_reduce(const fa2_bwd_args& a, int nsplit, hipStream_t st) {
  if (nsplit <= 1) return;
  const int64_t n = (int64_t)a.batch * a.heads_kv * a.seqlen_k * ((a.head_dim + 3) / 4);
  hipLaunchKernelGGL((dkv_reduce_kernel<BF16>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a, nsplit);
}

template <bool BF16, int DT, bool CAUSAL, bool BIAS, bool DROPOUT, bool ALIGNED>
static hipError_t launch_bwd_t(const fa2_bwd_args& a, int stages, hipStream_t st) {
  // order: standalone delta (bit 0), dQ (bit 2; also writes delta), then dK/dV (bit 1, reads it)
  // zero-sized problems launch nothing for that side: Sk == 0 -> dQ = 0 (dq_kernel sees no key
  // tile and writes zeros), no dK/dV rows; Sq == 0 -> dK/dV = 0 (dkdv_kernel sees no query
  // tile and writes zeros), no dQ rows
  if ((stages & 1) && a.lse_row_stride > 0) {
    dim3 grid((a.lse_row_stride + 15) / 16, a.batch * a.heads_q);
    hipLaunchKernelGGL((delta_kernel<BF16, ALIGNED>), grid, dim3(256), 0, st, a);
  }
  if ((stages & 4) && a.seqlen_q > 0) {
    if constexpr (DT == 128 && !BIAS && ALIGNED) {
      // hand-placed one-wave-per-SIMD dQ (dq_hp_kernel.h) for D = 128 exactly (dropout: with
      // the forward's saved keep words)
      if (dq_hp_ok(a, true)) {
        launch_dq_hp<BF16, CAUSAL, DROPOUT>(a, st);
        goto dq_done;
      }
    }
    {
    constexpr int NW = DqCfg<DT>::NW, BM = NW * 32;
    constexpr bool PAIR = CAUSAL;
    const int nmb = (a.seqlen_q + BM - 1) / BM;
    dim3 grid((PAIR ? (nmb + 1) / 2 : nmb) * a.batch * a.heads_q);
    auto dq = [&](auto biask_c) {
      constexpr int BK = decltype(biask_c)::value;
      if (a.dq_dtype == FA2_F32)
        hipLaunchKernelGGL((dq_kernel<BF16, DT, CAUSAL, BK, DROPOUT, ALIGNED, true>), grid, dim3(NW * 64), 0, st, a);
      else
        hipLaunchKernelGGL((dq_kernel<BF16, DT, CAUSAL, BK, DROPOUT, ALIGNED, false>), grid, dim3(NW * 64), 0, st, a);
    };
    if constexpr (!BIAS) {
      dq(std::integral_constant<int, 0>{});
    } else if constexpr (ALIGNED) {
      // a 16-bit bias with 16-byte aligned rows: LDS-staged bias tiles
      if (bias16_rows(a.bias, a.bias_dtype, a.bias_stride))
        a.bias_dtype == FA2_BF16 ? dq(std::integral_constant<int, 17>{}) : dq(std::integral_constant<int, 16>{});
      else
        dq(std::integral_constant<int, 1>{});
    } else {
      dq(std::integral_constant<int, 1>{});
    }
    }
  }
dq_done:
  if ((stages & 8) && BIAS && a.dbias && a.seqlen_q > 0 && a.seqlen_k > 0) {
    const int bb = a.bias_stride[0] != 0 ? a.batch : 1, hb = a.bias_stride[1] != 0 ? a.heads_q : 1;
    const int nkc = ((a.seqlen_k + 63) / 64 + kDbiasChunk - 1) / kDbiasChunk;
    dim3 grid(dbias_blocks((a.seqlen_q + 127) / 128, nkc), bb * hb);
    hipLaunchKernelGGL((dbias_kernel<BF16, DT, CAUSAL, DROPOUT, ALIGNED>), grid, dim3(256), 0, st, a);
  }
  if ((stages & 2) && a.seqlen_k > 0) {
    const int ns = dkv_split(a);
    if constexpr (DT == 128 && !BIAS && ALIGNED) {
      // hand-placed one-wave-per-SIMD dK/dV (dkdv_hp_kernel.h) for D = 128 exactly (dropout: with
      // the forward's saved keep words)
      if (dkdv_hp_ok(a, true)) {
        launch_dkdv_hp<BF16, CAUSAL, DROPOUT>(a, ns, st);
        launch_dkv_reduce<BF16>(a, ns, st);
        return hipGetLastError();
      }
    }
    dim3 grid(((a.seqlen_k + 127) / 128) * a.batch * a.heads_kv * ns);
    auto dkdv = [&](auto biask_c) {
      constexpr int BK = decltype(biask_c)::value;
      hipLaunchKernelGGL((dkdv_kernel<BF16, DT, CAUSAL, BK, DROPOUT, ALIGNED>), grid, dim3(256), 0, st, a, ns);
    };
    if constexpr (!BIAS) {
      dkdv(std::integral_constant<int, 0>{});
    } else if constexpr (ALIGNED) {
      if (bias16_rows(a.bias, a.bias_dtype, a.bias_stride))
        a.bias_dtype == FA2_BF16 ? dkdv(std::integral_constant<int, 17>{}) : dkdv(std::integral_constant<int, 16>{});
      else
        dkdv(std::integral_constant<int, 1>{});
    } else {
      dkdv(std::integral_constant<int, 1>{});
    }
    launch_dkv_reduce<BF16>(a, ns, st);
  }
  return hipGetLastError();
}

template <bool BF16, int DT>
hipError_t launch_bwd_dt(const fa2_bwd_args& a, bool aligned, int stages, hipStream_t st) {
  const bool c = a.causal != 0, bi = a.bias != nullptr, dr = a.dropout_p > 0.f;
#define FA2_BWD_CASE(C, B, R, A) \
  if (c == C && bi == B && dr == R && aligned == A) return launch_bwd_t<BF16, DT, C, B, R, A>(a, stages, st);
#define FA2_BWD_A(C, B, R) FA2_BWD_CASE(C, B, R, true) FA2_BWD_CASE(C, B, R, false)
#define FA2_BWD_R(C, B) FA2_BWD_A(C, B, true) FA2_BWD_A(C, B, false)
  FA2_BWD_R(true, true)
  FA2_BWD_R(true, false)
  FA2_BWD_R(false, true)
  FA2_BWD_R(false, false)
#undef FA2_BWD_R
#undef FA2_BWD_A
#undef FA2_BWD_CASE
  return hipErrorInvalidValue;
}

}  // namespace fa2
