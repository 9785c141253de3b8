// fwd.hip -- FlashAttention-2 forward for gfx950 (CDNA4).
//
// Replaces _fwd_kernel + compute_row_block (/root/reference/src/forward/kernel.py:61-291,
// /root/reference/src/forward/compute_row_blocks.py:7-103) with the same semantics:
//   s_ij = scale * <q_i, k_j> + bias_ij, bottom-right causal (j <= i + Lk - Lq), key padding,
//   online softmax in base 2, optional Philox dropout on P after the row sum, O = P V / l,
//   LSE2_i = m_i + log2(l_i) (kernel.py:119, compute_row_blocks.py:58-101).
//
// Work decomposition: one workgroup = NW waves = NW*32 query rows of one (batch, q-head);
// each wave owns 32 rows.  K/V tiles of 64 keys are staged in LDS (double buffered, LDS-DMA)
// and shared by the waves.  Per 64-key tile and wave:
//   S^T[key][q] = K Q^T        16 MFMA 32x32x16 (A = K row frags from LDS, B = Q frags in VGPRs)
//   softmax on the lane pair (l, l^32) holding one query row (16+16 keys per 32-key tile)
//   O^T[d][q]  += V^T P^T      16 MFMA (A = V^T via ds_read_b64_tr_b16, B = P in registers)
//
// Ping-pong schedule (NW = 8): waves w and w+4 share a SIMD.  Each tile takes two barrier-
// separated phases; in phase A waves 0-3 run QK^T + softmax of tile i while waves 4-7 run the
// PV of tile i-1, in phase B the roles swap.  So on every SIMD one wave's softmax VALU and
// fragment reads overlap its partner's MFMAs, instead of both waves hitting LDS, MFMA and VALU
// in lockstep.  K_{i+1} is issued at the start of A_i and V_{i+1} at the start of B_i (each
// two phases ahead of its first reader), retired by counted vmcnt waits before the barriers.
#include <stdlib.h>

#include <type_traits>

#include "common.h"
#include "fa2_internal.h"
#include "fwd_hp_kernel.h"
#include "fwd_pipe_kernel.h"

namespace fa2 {

// Waves per workgroup: 8 (256 query rows share each K/V tile, one workgroup per CU, two waves
// per SIMD) up to DT = 128; 4 for DT = 256, whose ~300 live registers allow one wave per SIMD.
// Causal: 4 waves (two independent workgroups per CU desynchronise each SIMD's pair of waves
// by themselves, and 128-row blocks waste less on the diagonal); non-causal: 8 waves with the
// ping-pong schedule below.
template <int DT, bool CAUSAL>
struct FwdCfg {
  static constexpr int NW = (DT >= 256 || CAUSAL) ? 4 : 8;
  static constexpr int kWavesPerSimd = DT >= 256 ? 1 : 2;
};


constexpr int kFwdLead = 3;  // fragment reads in flight ahead of their MFMA

// DROP: 0 no dropout, 1 Philox draws in the softmax (writing the keep words when asked), 2 the keep
// words a dropout_mask_kernel launch wrote just before (misc.hip) are read instead
template <bool BF16, int DT, bool CAUSAL, bool BIAS, int DROP, bool ALIGNED>
__global__ void __launch_bounds__((FwdCfg<DT, CAUSAL>::NW * 64), (FwdCfg<DT, CAUSAL>::kWavesPerSimd)) fwd_kernel(const fa2_fwd_args p) {
  using E = Elem<BF16>;
  constexpr bool DROPOUT = DROP != 0;
  constexpr int NW = FwdCfg<DT, CAUSAL>::NW;
  constexpr bool PINGPONG = NW == 8;
  constexpr int NT = NW * 64;
  constexpr int BM = NW * 32;        // query rows per workgroup
  constexpr int BN = 64;             // keys per tile
  constexpr int KS = DT / 16;        // k-steps of Q K^T
  constexpr int NDT = DT / 32;       // 32-wide d tiles of O
  constexpr int TILE = BN * DT * 2;  // bytes per K (or V) tile
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE];  // K0 K1 V0 V1

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r32 = lane & 31, hh = lane >> 5;
  const int grp = PINGPONG ? (w >> 2) : 0;  // phase offset of this wave

  // ---- work item -----------------------------------------------------------------------
  const int nmb = (p.seqlen_q + BM - 1) / BM;
  const int item = xcd_item(blockIdx.x, gridDim.x);  // head-major, see xcd_item
  const int bh = item / nmb;
  const int mbi = item - bh * nmb;
  const int mb = CAUSAL ? (nmb - 1 - mbi) : mbi;  // heaviest (longest key range) blocks first
  const int b = bh / p.heads_q, hq = bh - b * p.heads_q;
  const int hkv = hq / (p.heads_q / p.heads_kv);
  int Lq = p.seqlen_q, Lk = p.seqlen_k, cu = 0;
  if (p.cu_seqlens) {
    cu = p.cu_seqlens[b];
    Lq = Lk = p.cu_seqlens[b + 1] - cu;
  }
  const int m0 = mb * BM;
  const int qi = m0 + w * 32 + r32;  // this lane's query row
  const int D = p.head_dim;

  const uint16_t* qg = (const uint16_t*)p.q + b * p.q_stride[0] + hq * p.q_stride[2];
  const uint16_t* kg = (const uint16_t*)p.k + b * p.k_stride[0] + hkv * p.k_stride[2];
  const uint16_t* vg = (const uint16_t*)p.v + b * p.v_stride[0] + hkv * p.v_stride[2];

  // key range of the workgroup
  int n_end = 0;
  if (m0 < Lq) {
    n_end = Lk;
    if (CAUSAL) n_end = min(Lk, m0 + BM + Lk - Lq);
    n_end = max(n_end, 0);
  }
  const int ntiles = (n_end + BN - 1) / BN;

  auto kt = [&](int buf) { return smem + buf * TILE; };
  auto vt = [&](int buf) { return smem + (2 + buf) * TILE; };
  Stager<DT, BN, NT> kst, vst;
  if (ALIGNED) {
    kst.init(tid, p.k_stride[1], D);
    vst.init(tid, p.v_stride[1], D);
  }
  auto stage_k = [&](int buf, int n0) {
    if constexpr (ALIGNED) kst.issue(kt(buf), kg, p.k_stride[1], n0, Lk, tid);
    else stage_tile<DT, BN, NT, false>(kt(buf), kg, p.k_stride[1], n0, Lk, D, tid);
  };
  auto stage_v = [&](int buf, int n0) {
    if constexpr (ALIGNED) vst.issue(vt(buf), vg, p.v_stride[1], n0, Lk, tid);
    else stage_tile<DT, BN, NT, false>(vt(buf), vg, p.v_stride[1], n0, Lk, D, tid);
  };
  if (ntiles > 0) {
    stage_k(0, 0);
    stage_v(0, 0);
  }

  // ---- Q fragments (B operand of S^T = K Q^T): Q[qi][16 ks + 8 hh + j] -------------------
  u32x4 qf[KS];
  {
    const bool qvalid = qi < Lq;
    const uint16_t* qrow = qg + (int64_t)(qvalid ? qi : 0) * p.q_stride[1];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = load_row_frag<ALIGNED>(qrow, 16 * ks + 8 * hh, D, qvalid);
  }

  const float scale2 = p.softmax_scale * kLog2e;
  const int diag = Lk - Lq;  // key j visible to query i iff j <= i + diag
  float m_run = kNegInf, l_run = 0.f;
  f32x16 acc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) acc[dt] = zero16();

  const char* biasb = nullptr;
  if (BIAS) biasb = (const char*)p.bias;
  uint64_t drop_base = 0;
  if (DROPOUT) {
    // flat Philox offset, /root/reference/src/forward/kernel.py:146-148 (int64 here)
    drop_base = (uint64_t)Lk * ((uint64_t)cu + (uint64_t)Lq * ((uint64_t)hq + (uint64_t)p.heads_q * (p.cu_seqlens ? 0 : b)));
  }

  // Per-lane key limit: key kj is visible to this lane's row iff kj < lim_lane.
  const int qw0 = m0 + w * 32;  // first row of this wave
  const int lim_lane = CAUSAL ? min(Lk, qi + diag + 1) : Lk;
  // Scores are kept raw (no bias) or already in base-2 units (bias): exp2 argument = x*sc - m.
  const float sc = BIAS ? 1.f : scale2;

  // DROP == 2: keep words of this lane's row for the two 32-key halves of a tile, loaded a tile
  // ahead (mwn) and retired by the loop's waits before use (mwc)
  uint32_t mwc[2] = {0u, 0u}, mwn[2] = {0u, 0u};
  auto load_mw = [&](int n0) {
    if constexpr (DROP == 2) {
      const int nrb = (p.seqlen_q + 31) >> 5, ncw = (p.seqlen_k + 31) >> 5;
      const int64_t rowbase = ((int64_t)bh * nrb + (qi >> 5)) * ncw;
#pragma unroll
      for (int t = 0; t < 2; ++t)
        mwn[t] = (qi < p.seqlen_q && n0 + 32 * t < p.seqlen_k) ? p.dropout_mask[(rowbase + ((n0 >> 5) + t)) * 32 + (qi & 31)] : 0u;
    }
  };
  auto next_mw = [&](int n0) {
    if constexpr (DROP == 2) {
      mwc[0] = mwn[0];
      mwc[1] = mwn[1];
      load_mw(n0 + BN);
    }
  };

  // state handed from a wave's QK phase to its PV phase
  u32x4 pf[2][2];
  float alpha = 1.f;
  bool rescale = false;

  // QK^T + online softmax of one 64-key tile for this wave (MASK: diagonal / tail variant).
  auto qk_softmax = [&](auto mask_c, const char* K, int n0, auto fill) {
    constexpr bool MASK = decltype(mask_c)::value;
    f32x16 s[2];
    {
      // fenced steps: each fragment read runs kFwdLead MFMAs ahead, the two key halves'
      // chains alternate
      constexpr int N = 2 * KS, L = kFwdLead;
      u32x4 kf[N];
#pragma unroll
      for (int j = 0; j < L; ++j) kf[j] = lds_row_frag<DT, BN>(K, 32 * (j & 1), r32, j >> 1, hh);
      s[0] = zero16();
      s[1] = zero16();
#pragma unroll
      for (int m = 0; m < N; ++m) {
        if (m + L < N) kf[m + L] = lds_row_frag<DT, BN>(K, 32 * ((m + L) & 1), r32, (m + L) >> 1, hh);
        s[m & 1] = E::mfma(kf[m], qf[m >> 1], s[m & 1]);
        fill(m);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // register i of half t holds key n0 + 32 t + (i & 3) + 8 (i >> 2) + 4 hh
    const int rel = lim_lane - n0 - 4 * hh;
    float mx = kNegInf;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int o = 32 * t + (i & 3) + 8 * (i >> 2);
        float x = s[t][i];
        if (BIAS) {
          const int kj = n0 + o + 4 * hh;
          const int kc = kj < Lk ? kj : Lk - 1;
          const int qc = qi < Lq ? qi : 0;
          x = fmaf(x, scale2, kLog2e * load_bias(biasb, b * p.bias_stride[0] + hq * p.bias_stride[1] +
                                                          (int64_t)qc * p.bias_stride[2] + kc, p.bias_dtype));
        }
        if (MASK) x = o < rel ? x : kNegInf;
        s[t][i] = x;
        mx = fmaxf(mx, x);
      }
    }
    mx = half_max(mx) * sc;
    // defer-max: keep the stale max unless some row of the wave outgrew it by > kDeferMax
    // (the first finite max always moves it: -inf - m is never <= threshold)
    rescale = !__all(mx - m_run <= kDeferMax);
    const float m_new = rescale ? fmaxf(m_run, mx) : m_run;
    const float m_use = m_new == kNegInf ? 0.f : m_new;
    alpha = __builtin_amdgcn_exp2f(m_run - m_use);
    m_run = m_new;

    float rs = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float pv[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        pv[i] = __builtin_amdgcn_exp2f(fmaf(s[t][i], sc, -m_use));
        rs += pv[i];
      }
      if (DROP == 2) {
        // the word of the row's 32 keys (loaded a tile ahead); this lane's bits sit at 4 hh + ..
        const uint32_t wd = mwc[t] >> (4 * hh);
#pragma unroll
        for (int i = 0; i < 16; ++i) pv[i] = ((wd >> ((i & 3) + 8 * (i >> 2))) & 1u) ? pv[i] : 0.f;
      } else if (DROPOUT) {
        const uint64_t rowoff = drop_base + (uint64_t)qi * Lk;
        uint32_t kb = 0;  // keep bits of this lane's 16 keys at their positions in the 32-key word
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int kj = n0 + 32 * t + (i & 3) + 8 * (i >> 2) + 4 * hh;
          const bool keep = philox_uniform(p.dropout_seed, rowoff + kj) > p.dropout_p;
          pv[i] = keep ? pv[i] : 0.f;
          kb |= (uint32_t)keep << ((i & 3) + 8 * (i >> 2) + 4 * hh);
        }
        if (p.dropout_mask) {
          // the row's 32-key word = this lane's bits | the partner lane's (l ^ 32, same row);
          // lanes of half t store it: word (qi, key word (n0 + 32 t) / 32) of the tiled layout
          const auto r = __builtin_amdgcn_permlane32_swap(kb, kb, false, false);
          if (hh == t && qi < p.seqlen_q && n0 + 32 * t < p.seqlen_k) {
            const int nrb = (p.seqlen_q + 31) >> 5, ncw = (p.seqlen_k + 31) >> 5;
            const int64_t wi = (((int64_t)bh * nrb + (qi >> 5)) * ncw + ((n0 + 32 * t) >> 5)) * 32 + (qi & 31);
            p.dropout_mask[wi] = r[0] | r[1];
          }
        }
      }
#pragma unroll
      for (int sp = 0; sp < 2; ++sp)
#pragma unroll
        for (int j = 0; j < 4; ++j) pf[t][sp][j] = E::pack2(pv[8 * sp + 2 * j], pv[8 * sp + 2 * j + 1]);
    }
    l_run = l_run * alpha + rs;  // lane-partial row sum (the partner lane holds the rest)
  };

  // O^T = alpha O^T + V^T P^T
  auto pv_update = [&](const char* V) {
    if (rescale) {
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[dt][i] *= alpha;
    }
    {
      constexpr int N = 4 * NDT, L = 2 * kFwdLead > N ? N : 2 * kFwdLead;
      u32x4 vf[N];
      auto rd = [&](int m) { return lds_tr_frag<DT, BN>(V, 16 * (m / NDT), 32 * (m % NDT), lane); };
#pragma unroll
      for (int j = 0; j < L; ++j) vf[j] = rd(j);
#pragma unroll
      for (int m = 0; m < N; ++m) {
        if (m + L < N) vf[m + L] = rd(m + L);
        const int kk = m / NDT;
        acc[m % NDT] = E::mfma(vf[m], pf[kk >> 1][kk & 1], acc[m % NDT]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };

  load_mw(0);
  __builtin_amdgcn_s_waitcnt(0);  // prologue: Q fragments (compiler-tracked) + first tiles
  __syncthreads();

  constexpr int kPieces = Stager<DT, BN, NT>::kIters;  // LDS-DMA ops per thread per tile
  auto nofill = [](int) {};

  // Phase ph = 2 i + x: x = 0 (A_i) issues K_{i+1}, x = 1 (B_i) issues V_{i+1}.  A wave of
  // group g runs QK of tile (ph - g) / 2 when ph - g is even, PV of tile (ph - g - 1) / 2 when odd.
  bool live = false;  // the pending PV of this wave has unmasked rows
  if constexpr (!PINGPONG) {
    // one barrier per tile: prefetch K/V_{i+1}, QK + softmax + PV of tile i
    // With SPREAD the next tile's LDS-DMA pieces ride in the QK^T steps (one every other MFMA)
    // instead of a burst at the top of the tile; rows past the end are clamped, so the issue
    // is branch free (the last tile re-reads valid rows into a buffer nobody reads).
    constexpr bool SPREAD = ALIGNED && NT == BN * 4;
    for (int i = 0; i < ntiles; ++i) {
      const int n0 = i * BN;
      next_mw(n0);
      const uint16_t* kgt = kg + (int64_t)(n0 + BN) * p.k_stride[1];
      const uint16_t* vgt = vg + (int64_t)(n0 + BN) * p.v_stride[1];
      int64_t kadj = 0, vadj = 0;
      if constexpr (SPREAD) {
        kadj = kst.row_adjust(p.k_stride[1], n0 + BN, Lk, tid);
        vadj = vst.row_adjust(p.v_stride[1], n0 + BN, Lk, tid);
      } else if (i + 1 < ntiles) {
        stage_k((i + 1) & 1, (i + 1) * BN);
        stage_v((i + 1) & 1, (i + 1) * BN);
      }
      auto dma = [&](int pc) {
        if (pc < kPieces) kst.piece(kt((i + 1) & 1), kgt, kadj, pc);
        else vst.piece(vt((i + 1) & 1), vgt, vadj, pc - kPieces);
      };
      auto fill = [&](int m) {
        if constexpr (SPREAD) {
          constexpr int every = KS / kPieces;  // 2 QK steps per piece: K then V pieces
          if (m % every == 0 && m / every < 2 * kPieces) dma(m / every);
        }
      };
      const bool dead = CAUSAL && (n0 > qw0 + 31 + diag);
      const bool need_mask = (n0 + BN > Lk) || (CAUSAL && (n0 + BN - 1 > qw0 + diag));
      if (!dead) {
        if (need_mask) qk_softmax(std::true_type{}, kt(i & 1), n0, fill);
        else qk_softmax(std::false_type{}, kt(i & 1), n0, fill);
        pv_update(vt(i & 1));
      } else if constexpr (SPREAD) {
#pragma unroll
        for (int pc = 0; pc < 2 * kPieces; ++pc) dma(pc);
      }
      vm_wait_all();
      __syncthreads();
    }
  }
  const int nphase = PINGPONG && ntiles > 0 ? 2 * ntiles + 1 : 0;
  for (int ph = 0; ph < nphase; ++ph) {
    const int i = ph >> 1;
    const bool issued = ((ph & 1) == 0) ? (i + 1 < ntiles) : (i + 1 < ntiles);
    if (i + 1 < ntiles) {
      if ((ph & 1) == 0) stage_k((i + 1) & 1, (i + 1) * BN);
      else stage_v((i + 1) & 1, (i + 1) * BN);
    }
    const int rel_ph = ph - grp;
    if (rel_ph >= 0) {
      const int tile = rel_ph >> 1;
      if ((rel_ph & 1) == 0) {
        if (tile < ntiles) {
          const int n0 = tile * BN;
          // wave-uniform tile class: fully masked for this wave / needs masks / interior
          const bool dead = CAUSAL && (n0 > qw0 + 31 + diag);
          const bool need_mask = (n0 + BN > Lk) || (CAUSAL && (n0 + BN - 1 > qw0 + diag));
          live = !dead;
          next_mw(n0);
          if (!dead) {
            if (need_mask) qk_softmax(std::true_type{}, kt(tile & 1), n0, nofill);
            else qk_softmax(std::false_type{}, kt(tile & 1), n0, nofill);
          }
        }
      } else if (live) {
        pv_update(vt(tile & 1));
        live = false;
      }
    }
    // retire the tile the next phase reads; the DMA issued in this phase may stay in flight
    if (PINGPONG && issued) {
      if constexpr (kPieces == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
      else if constexpr (kPieces == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else if constexpr (kPieces == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else vm_wait_all();
    } else {
      vm_wait_all();
    }
    __syncthreads();
  }

  // ---- epilogue ----------------------------------------------------------------------------
  const float l_tot = half_sum(l_run);
  const bool row_ok = qi < Lq && l_tot > 0.f;
  float inv = row_ok ? 1.f / l_tot : 0.f;
  if (DROPOUT) inv *= 1.f / (1.f - p.dropout_p);
  if (hh == 0 && qi < p.lse_row_stride) {
    float* lrow = p.lse + (int64_t)bh * p.lse_row_stride;
    lrow[qi] = row_ok ? m_run + __log2f(l_tot) : kNegInf;
  }
  if constexpr (ALIGNED) {
    // every loop iteration ends in a barrier: the K/V buffers (NW x 32 rows x DT fit exactly) are free
    uint16_t* o0 = (uint16_t*)p.o + b * p.o_stride[0] + hq * p.o_stride[2] + (int64_t)qw0 * p.o_stride[1];
    store_rows_lds<BF16, DT>(smem + w * 32 * DT * 2, acc, inv, row_ok, o0, p.o_stride[1],
                             min(32, p.seqlen_q - qw0), D, lane);
  } else if (qi < p.seqlen_q) {
    uint16_t* orow = (uint16_t*)p.o + b * p.o_stride[0] + hq * p.o_stride[2] + (int64_t)qi * p.o_stride[1];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d0 = 32 * dt + 8 * g4 + 4 * hh;
        const float o0 = acc[dt][4 * g4 + 0] * inv, o1 = acc[dt][4 * g4 + 1] * inv;
        const float o2 = acc[dt][4 * g4 + 2] * inv, o3 = acc[dt][4 * g4 + 3] * inv;
        if (ALIGNED) {
          if (d0 < D) *(u32x2*)(orow + d0) = u32x2{E::pack2(o0, o1), E::pack2(o2, o3)};
        } else {
          if (d0 + 0 < D) orow[d0 + 0] = E::from_f32(o0);
          if (d0 + 1 < D) orow[d0 + 1] = E::from_f32(o1);
          if (d0 + 2 < D) orow[d0 + 2] = E::from_f32(o2);
          if (d0 + 3 < D) orow[d0 + 3] = E::from_f32(o3);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
template <bool BF16, int DT, bool CAUSAL, bool BIAS, bool DROPOUT, bool ALIGNED>
static hipError_t launch_fwd_t(const fa2_fwd_args& a, hipStream_t st) {
  constexpr int NW = FwdCfg<DT, CAUSAL>::NW, BM = NW * 32;
  dim3 grid(((a.seqlen_q + BM - 1) / BM) * a.batch * a.heads_q);
  if constexpr (DROPOUT) {
    // with a keep-mask buffer the bits are drawn by dropout_mask_kernel (all VALU, full
    // occupancy) and read here; without one the softmax draws them
    if (a.dropout_mask) {
      if (hipError_t e = launch_dropout_mask(a, st); e != hipSuccess) return e;
      hipLaunchKernelGGL((fwd_kernel<BF16, DT, CAUSAL, BIAS, 2, ALIGNED>), grid, dim3(NW * 64), 0, st, a);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((fwd_kernel<BF16, DT, CAUSAL, BIAS, DROPOUT ? 1 : 0, ALIGNED>), grid, dim3(NW * 64), 0, st, a);
  return hipGetLastError();
}

template <bool BF16, int DT>
hipError_t launch_fwd_dt(const fa2_fwd_args& a, bool aligned, hipStream_t st) {
  const bool c = a.causal != 0, bi = a.bias != nullptr, dr = a.dropout_p > 0.f;
  // hot path: software-pipelined kernel (fwd_pipe_kernel.h), also with a 16-bit bias whose rows
  // are 16-byte aligned (its tiles are staged by LDS-DMA)
  if constexpr (DT == 128) {
    // hand-placed one-wave-per-SIMD kernel (fwd_hp_kernel.h) for D = 128 exactly
    if (a.head_dim == DT && fwd_hp_ok(a, aligned))
      return c ? launch_fwd_hp<BF16, true, DT>(a, st) : launch_fwd_hp<BF16, false, DT>(a, st);
  }
  if constexpr (DT == 64 || DT == 128) {
    const bool bias16 = bias16_rows(a.bias, a.bias_dtype, a.bias_stride);
    if (aligned && !dr && a.k_stride[1] == a.v_stride[1] && (!bi || bias16)) {
      if (!bi) return c ? launch_fwd_pipe<BF16, DT, true, 0>(a, st) : launch_fwd_pipe<BF16, DT, false, 0>(a, st);
      if (a.bias_dtype == FA2_BF16)
        return c ? launch_fwd_pipe<BF16, DT, true, 17>(a, st) : launch_fwd_pipe<BF16, DT, false, 17>(a, st);
      return c ? launch_fwd_pipe<BF16, DT, true, 16>(a, st) : launch_fwd_pipe<BF16, DT, false, 16>(a, st);
    }
  }
#define FA2_FWD_CASE(C, B, R, A)                                  \
  if (c == C && bi == B && dr == R && aligned == A)               \
    return launch_fwd_t<BF16, DT, C, B, R, A>(a, st);
#define FA2_FWD_A(C, B, R) FA2_FWD_CASE(C, B, R, true) FA2_FWD_CASE(C, B, R, false)
#define FA2_FWD_R(C, B) FA2_FWD_A(C, B, true) FA2_FWD_A(C, B, false)
#define FA2_FWD_B(C) FA2_FWD_R(C, true) FA2_FWD_R(C, false)
  FA2_FWD_B(true)
  FA2_FWD_B(false)
#undef FA2_FWD_B
#undef FA2_FWD_R
#undef FA2_FWD_A
#undef FA2_FWD_CASE
  return hipErrorInvalidValue;
}

}  // namespace fa2
