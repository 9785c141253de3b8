// dkdv_pipe_kernel.h -- software-pipelined dK/dV for gfx950 at one wave per SIMD (the hot path
// of the backward: head_dim 128, 16-byte aligned tensors, no bias, no dropout).  Same
// semantics as dkdv_kernel (bwd_kernel.h) and the reference's dK/dV program
// (/root/reference/src/backward/compute_dkdv.py:7-296, math at :89-110):
//   P = exp2(s * scale * log2e - LSE2), dV^T += dO^T P, dP = dO V^T, dS = P (dP - delta),
//   dK^T += Q^T dS;  P and dS rounded to the input dtype before their MFMAs, fp32 accumulation.
//
// Work decomposition as dkdv_kernel: one workgroup = 4 waves = 128 keys of one (batch, kv-head),
// wave w owns keys n0 + 32 w + (lane & 31); the workgroup sweeps the q-heads of its GQA group x
// 32-row query tiles ("steps").  What differs is the schedule:
//  * One wave per SIMD with the whole 512-register file: K and V of the wave's 32 keys stay in
//    registers for the kernel's life (no V re-reads from LDS), dK/dV accumulate in 128 more.
//  * Each step i runs two fenced phases, the wave overlapping its own work across steps:
//      phase A: S(i+1) = Q(i+1) K^T and dP(i+1) MFMA chains, carrying the softmax-gradient VALU
//               of step i (P(i) beside the S chain, dS(i) beside the dP chain);
//      phase B: dV += dO(i)^T P(i), dK += Q(i)^T dS(i) (transposed LDS reads), dS(i) stores.
//  * The dP accumulator starts at delta (loaded straight from LDS) and V is negated once at load,
//    so the chain yields delta - dP and dS = -P (delta - dP) costs one multiply (the sign goes
//    into the bf16/fp16 pack's source modifier).
//  * Q/dO/LSE/delta tiles arrive by LDS-DMA into a ring of 4 buffers, 3 steps ahead; the dS
//    stores of the dS-workspace path (DSOUT) then have two steps to retire before any wait
//    covers them (vmcnt retires in issue order).
#pragma once
#include <type_traits>

#include "common.h"
#include "fa2_internal.h"

namespace fa2 {

// dV^T and dK^T live in asm-owned accumulator registers: dV tile dt in a[128 + 16 dt ..], dK
// tile dt in a[192 + 16 dt ..].  The unit is built with MFMA accumulators in arch VGPRs
// (-amdgpu-mfma-vgpr-form, where S and dP must be for their VALU consumers); what hipcc still
// puts in the accumulator file (MFMA operands beyond the 256 arch VGPRs) it allocates from a0
// upwards, below the asm-owned range.  Every statement that writes a[128:255] declares it
// clobbered (that also makes the kernel descriptor allocate it), and tests/test_host.py audits
// the compiled kernel: no compiler-generated instruction may name a[128:255].
// hipcc does not pad hazards inside asm: the A operands come straight from LDS reads (counted by
// hipcc's lgkmcnt waits) and the B operands (packed P / dS) are written by VALU one phase
// earlier, behind the `s_nop 1` that opens each phase B (VALU write -> MFMA read); the accumulate
// chain itself needs none; readers after the last MFMA wait 12 states (agpr_drain).
#define FA2_A8(n) "a" #n "0", "a" #n "1", "a" #n "2", "a" #n "3", "a" #n "4", "a" #n "5", "a" #n "6", "a" #n "7", "a" #n "8", "a" #n "9"
#define FA2_ACC_CLOBBERS                                                                                          \
  "a128", "a129", FA2_A8(13), FA2_A8(14), FA2_A8(15), FA2_A8(16), FA2_A8(17), FA2_A8(18), FA2_A8(19), FA2_A8(20), \
      FA2_A8(21), FA2_A8(22), FA2_A8(23), FA2_A8(24), "a250", "a251", "a252", "a253", "a254", "a255"
constexpr int kAccV = 128, kAccK = 192;  // first accumulator register of dV^T / dK^T

template <bool BF16, int BASE>
FA2_DEV void mfma_acc(u32x4 a, u32x4 b) {
  if constexpr (BF16)
    asm volatile("v_mfma_f32_32x32x16_bf16 a[%c2:%c3], %0, %1, a[%c2:%c3]"
                 :: "v"(a), "v"(b), "i"(BASE), "i"(BASE + 15) : FA2_ACC_CLOBBERS);
  else
    asm volatile("v_mfma_f32_32x32x16_f16 a[%c2:%c3], %0, %1, a[%c2:%c3]"
                 :: "v"(a), "v"(b), "i"(BASE), "i"(BASE + 15) : FA2_ACC_CLOBBERS);
}
FA2_DEV void acc_zero() {
  asm volatile(
#define FA2_Z4(i) "v_accvgpr_write_b32 a" #i ", 0\n\t"
#define FA2_Z40(n) FA2_Z4(n##0) FA2_Z4(n##1) FA2_Z4(n##2) FA2_Z4(n##3) FA2_Z4(n##4) FA2_Z4(n##5) FA2_Z4(n##6) FA2_Z4(n##7) FA2_Z4(n##8) FA2_Z4(n##9)
      FA2_Z4(128) FA2_Z4(129) FA2_Z40(13) FA2_Z40(14) FA2_Z40(15) FA2_Z40(16) FA2_Z40(17) FA2_Z40(18) FA2_Z40(19)
      FA2_Z40(20) FA2_Z40(21) FA2_Z40(22) FA2_Z40(23) FA2_Z40(24) FA2_Z4(250) FA2_Z4(251) FA2_Z4(252) FA2_Z4(253)
      FA2_Z4(254) FA2_Z4(255) "s_nop 1" ::: FA2_ACC_CLOBBERS);
#undef FA2_Z40
#undef FA2_Z4
}
// 8-pass MFMA result -> any other reader: 12 wait states (hipcc does not count asm MFMAs)
FA2_DEV void agpr_drain() { asm volatile("s_nop 7\n\ts_nop 7" ::: "memory"); }
// four consecutive accumulators a[i .. i+3]
template <int I>
FA2_DEV f32x4 acc_read4() {
  f32x4 r;
  asm volatile("v_accvgpr_read_b32 %0, a%c4\n\tv_accvgpr_read_b32 %1, a%c5\n\tv_accvgpr_read_b32 %2, a%c6\n\tv_accvgpr_read_b32 %3, a%c7"
               : "=v"(r[0]), "=v"(r[1]), "=v"(r[2]), "=v"(r[3])
               : "i"(I), "i"(I + 1), "i"(I + 2), "i"(I + 3));
  return r;
}

#ifndef FA2_PIPE_ABL
#define FA2_PIPE_ABL 0  // timing ablations: 1 no DMA, 2 no mid barrier, 4 no phase-B VALU, 8 no LDS reads
#endif

template <bool BF16, bool CAUSAL, bool DSOUT>
__global__ void __launch_bounds__(256, 1) dkdv_pipe_kernel(const fa2_bwd_args p) {
  using E = Elem<BF16>;
  constexpr int DT = 128, NT = 256, BNK = 128, BMQ = 32;
  constexpr int KS = DT / 16;        // k-steps of S and dP
  constexpr int NDT = DT / 32;       // 32-wide d tiles of dK / dV
  constexpr int QB = BMQ * DT * 2;   // Q (or dO) tile bytes
  constexpr int SB = 2 * BMQ * 4;    // LSE2 + delta rows of a tile
  constexpr int BUF = 2 * QB + SB;
  constexpr int NB = 4;              // ring depth (DMA issued NB - 1 steps ahead)
  __shared__ __attribute__((aligned(16))) char smem[NB * BUF];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const int nkb = (p.seqlen_k + BNK - 1) / BNK;
  const int item = xcd_item(blockIdx.x, gridDim.x);  // head-major, heaviest key blocks first
  const int bkv = item / nkb;
  const int n0 = (item - bkv * nkb) * BNK;
  const int b = bkv / p.heads_kv, hkv = bkv - b * p.heads_kv;
  const int G = p.heads_q / p.heads_kv;
  int Lq = p.seqlen_q, Lk = p.seqlen_k;
  if (p.cu_seqlens) Lq = Lk = p.cu_seqlens[b + 1] - p.cu_seqlens[b];
  const int D = p.head_dim;
  const int diag = Lk - Lq;
  const int kw0 = n0 + 32 * w;  // first key of this wave
  const int kj = kw0 + r32;     // this lane's key
  const bool kval = kj < Lk;
  const float scale = p.softmax_scale, sc = scale * kLog2e;

  int m_begin = 0;  // causal: the first row that sees key n0 is n0 - diag
  if (CAUSAL) m_begin = max(0, n0 - diag) & ~(BMQ - 1);
  const int n_mt = (n0 < Lk && m_begin < Lq) ? (Lq - m_begin + BMQ - 1) / BMQ : 0;
  const int total = n_mt * G;  // (q-head, query tile) steps

  // K (B operand of S = Q K^T) and -V (B operand of delta - dP = delta + dO (-V)^T) in registers
  u32x4 kf[KS], vf[KS];
  {
    const uint16_t* krow = (const uint16_t*)p.k + b * p.k_stride[0] + hkv * p.k_stride[2] + (int64_t)(kval ? kj : 0) * p.k_stride[1];
    const uint16_t* vrow = (const uint16_t*)p.v + b * p.v_stride[0] + hkv * p.v_stride[2] + (int64_t)(kval ? kj : 0) * p.v_stride[1];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      kf[ks] = load_row_frag<true>(krow, 16 * ks + 8 * hh, D, kval);
      const u32x4 v4 = load_row_frag<true>(vrow, 16 * ks + 8 * hh, D, kval);
      vf[ks] = v4 ^ u32x4{0x80008000u, 0x80008000u, 0x80008000u, 0x80008000u};  // exact sign flip
    }
  }
  acc_zero();  // dV^T, dK^T accumulators (a[128:191], a[192:255])

  if (total > 0) {
    auto qbuf = [&](int j) { return smem + (j & (NB - 1)) * BUF; };
    auto obuf = [&](int j) { return smem + (j & (NB - 1)) * BUF + QB; };
    // LSE2 / delta rows, in groups of 8 rows: [LSE r..r+7][delta r..r+7] (64 bytes per group)
    auto sbuf = [&](int j) { return smem + (j & (NB - 1)) * BUF + 2 * QB; };

    BufStager<DT, BMQ, NT> qst, ost;  // per-lane byte offsets of the 2 + 2 pieces of a tile
    qst.init(tid, p.q_stride[1], D);
    ost.init(tid, p.do_stride[1], D);
    static_assert(BufStager<DT, BMQ, NT>::kIters == 2, "two 16-byte pieces per lane and tile");

    // ---- LDS-DMA of step dj: 5 VMEM ops per lane (Q, dO: 2 each; LSE2/delta rows: 1), issued
    // from an incrementally advanced cursor (no per-step address arithmetic beyond adds).  Past
    // the last step the last tile is loaded again into a buffer nobody reads, so every step
    // issues the same count.
    const int64_t qrb = p.q_stride[1] * 2, orb = p.do_stride[1] * 2;  // row bytes (< 2^27: launcher)
    const char* q_head = (const char*)p.q + 2 * (b * p.q_stride[0] + (int64_t)(hkv * G) * p.q_stride[2]) + m_begin * qrb;
    const char* o_head = (const char*)p.dout + 2 * (b * p.do_stride[0] + (int64_t)(hkv * G) * p.do_stride[2]) + m_begin * orb;
    const char* q_t = q_head;
    const char* o_t = o_head;
    int rows_left = Lq - m_begin;
    // this lane's LSE2 (lanes 0-7) / delta (lanes 8-15) row: wave w loads rows m + 8 w + (lane & 7)
    const float* l_head = ((lane & 8) ? p.delta : p.lse) + (int64_t)(b * p.heads_q + hkv * G) * p.lse_row_stride +
                          m_begin + 8 * w + (lane & 7);
    const float* l_t = l_head;
    int dj = 0, dmt = 0;
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(smem));
    // one tile's DMA = 5 pieces (Q 0-1, dO 2-3, LSE2/delta 4), issued one by one so that a step can
    // spread them over MFMA gaps (an LDS-DMA piece holds the wave's issue for 60-185 cycles,
    // MI355X_MICROARCH.md): stage_prep() once, stage_piece(k) for k = 0..4, stage_advance() after
    struct Stage {
      i32x4 rq, ro;
      uint32_t base;  // LDS byte address of this wave's first piece of the tile
    } sg{};
    auto stage_prep = [&]() {
      const int rows = min(rows_left, BMQ);
      sg.rq = make_rsrc(q_t, (uint32_t)(rows * qrb));
      sg.ro = make_rsrc(o_t, (uint32_t)(rows * orb));
      sg.base = lds0 + (uint32_t)((dj & (NB - 1)) * BUF);
    };
    auto stage_piece = [&](int k) {
      if (FA2_PIPE_ABL & 1) return;
      uint32_t keep;
      const uint32_t dst = sg.base + qst.wave_lds + (k & 1) * NT * 16 + (k >> 1) * QB;
      switch (k) {
        case 0:
        case 1:
          asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                       : "=&s"(keep) : "v"(qst.voff[k & 1]), "s"(sg.rq), "s"(dst) : "memory");
          break;
        case 2:
        case 3:
          asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                       : "=&s"(keep) : "v"(ost.voff[k & 1]), "s"(sg.ro), "s"(dst) : "memory");
          break;
        default:
          if (lane < 16) glds4(l_t, sg.base + 2 * QB + 64 * w);
      }
    };
    auto stage_advance = [&]() {
      if (dj + 1 < total) {
        if (++dmt == n_mt) {  // next q-head of the group
          dmt = 0;
          q_head += 2 * p.q_stride[2];
          o_head += 2 * p.do_stride[2];
          l_head += p.lse_row_stride;
          q_t = q_head;
          o_t = o_head;
          l_t = l_head;
          rows_left = Lq - m_begin;
        } else {
          q_t += BMQ * qrb;
          o_t += BMQ * orb;
          l_t += BMQ;
          rows_left -= BMQ;
        }
      }
      ++dj;
    };
    auto stage_next = [&]() {
      stage_prep();
#pragma unroll
      for (int k = 0; k < 5; ++k) stage_piece(k);
      stage_advance();
    };

    // ---- compute-side step state (wave-uniform) ---------------------------------------------
    int cg = 0, cmt = 0;   // (q-head in group, query tile) of the current step
    bool st_prev = false;  // the previous step issued dS stores
    const DsLayout L(p.seqlen_q, p.seqlen_k, CAUSAL);
    // dS tile of the current step in the workspace: chunk (b, hq, q-tile m / 32, key block kw0 / 32)
    // of the compact layout; advanced per step by the visible tiles of the q-tile it leaves
    int64_t ch_head = (int64_t)(b * p.heads_q + hkv * G) * L.per_head() + L.prefix(m_begin >> 5) + (kw0 >> 5);
    int64_t ch = ch_head;
    char* const ds_lane = (char*)p.ds_workspace + r32 * 64 + 32 * hh;
    auto m_of = [&](int mt) { return m_begin + mt * BMQ; };
    auto is_dead = [&](int m) { return kw0 >= Lk || (CAUSAL && kw0 > m + BMQ - 1 + diag); };
    auto needs_mask = [&](int m) {
      return (m + BMQ > Lq) || (kw0 + 31 >= Lk) || (CAUSAL && kw0 + 31 > m + diag);
    };

    f32x16 s, dp;            // S and delta - dP of the step whose softmax gradient is next
    u32x4 pp[2], dsp[2];     // P, dS of the current step (B operands of dV^T, dK^T)
    u32x4 ppn[2], dspn[2];   // ... of the next step, produced during the current one

    // softmax-gradient VALU of one step, 16 elements of s / dp -> packed P and dS in pn / dn:
    //   P = exp2(s sc - LSE2) (masked: rows outside this key's window, padded rows -> 0),
    //   dS = P (dP - delta) = -(P (delta - dP)), the sign riding in the pack's source modifier.
    // Element e: row m + (e & 3) + 8 (e >> 2) + 4 hh of this lane's key.
    struct Win {
      int lo, hi;
    };
    auto window = [&](int m) {
      const int qlo = CAUSAL ? max(kj - diag, 0) : 0;
      const int qhi = kj < Lk ? Lq : -1;
      return Win{qlo - m - 4 * hh, qhi - m - 4 * hh};
    };
    auto p_elem = [&](auto mask_c, int e, const f32x4* l4, Win wn) {
      constexpr bool MASK = decltype(mask_c)::value;
      const int g4 = e >> 2, jj = e & 3;
      float pr = __builtin_amdgcn_exp2f(fmaf(s[e], sc, -l4[g4][jj]));
      if (MASK) {
        const int o = jj + 8 * g4;
        pr = (o >= wn.lo && o < wn.hi) ? pr : 0.f;
      }
      s[e] = pr;
    };
    auto ds_elem = [&](int e) { dp[e] = s[e] * dp[e]; };
    auto pack = [&](int g4, u32x4* pn, u32x4* dn) {
      pn[g4 >> 1][2 * (g4 & 1) + 0] = E::pack2(s[4 * g4 + 0], s[4 * g4 + 1]);
      pn[g4 >> 1][2 * (g4 & 1) + 1] = E::pack2(s[4 * g4 + 2], s[4 * g4 + 3]);
      dn[g4 >> 1][2 * (g4 & 1) + 0] = E::pack2(-dp[4 * g4 + 0], -dp[4 * g4 + 1]);
      dn[g4 >> 1][2 * (g4 & 1) + 1] = E::pack2(-dp[4 * g4 + 2], -dp[4 * g4 + 3]);
    };
    auto load_l4 = [&](int j, f32x4* l4) {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) l4[g4] = *(const f32x4*)(sbuf(j) + 64 * g4 + 16 * hh);
    };
    // Fragment sets, each read one phase before the phase that consumes it:
    //   fa[16] = rows of Q (0-7) and dO (8-15) of the tile S / dP are computed from (phase A),
    //   fb[16] = transposed dO (dV) / Q (dK) fragments of the current tile (phase B).
    u32x4 fa[2 * KS], fb[4 * NDT];
    auto rd_a = [&](int j, int mm) { return lds_row_frag<DT, BMQ>(mm < KS ? qbuf(j) : obuf(j), 0, r32, mm % KS, hh); };
    auto rd_b = [&](int j, int mm) {
      const int dt = mm % NDT, r = mm / NDT;  // r: (sp, dV | dK)
      return lds_tr_frag<DT, BMQ>((r & 1) ? qbuf(j) : obuf(j), 16 * (r >> 1), 32 * dt, lane);
    };
    auto load_d4 = [&](int j) {  // delta rows of tile j: the initial dP accumulator
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const f32x4 d4 = *(const f32x4*)(sbuf(j) + 64 * g4 + 32 + 16 * hh);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) dp[4 * g4 + jj] = d4[jj];
      }
    };
    // S(j), delta - dP(j) into s, dp from fa (the chains; hook(mm) runs in MFMA gap mm)
    auto sdp = [&](auto hook) {
#pragma unroll
      for (int mm = 0; mm < 2 * KS; ++mm) {
        if (mm < KS) s = E::mfma(fa[mm], kf[mm], mm == 0 ? zero16() : s);
        else dp = E::mfma(fa[mm], vf[mm - KS], dp);
        hook(mm);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    // mid-step wait: the tile of step i + 2 has landed (issued in phase A of step i - 1; younger
    // VMEM ops: the dS stores of step i - 1 (phase B) and the DMA of step i + 3 (phase A of this
    // step)); every wave done with its LDS reads of phase A
    auto mid_wait = [&](bool a) {
      if (FA2_PIPE_ABL & 2) asm volatile("s_waitcnt vmcnt(7) lgkmcnt(0)" ::: "memory");
      else if (a) asm volatile("s_waitcnt vmcnt(7) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(5) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };

    // ---- one step i ---------------------------------------------------------------------------
    //   top:     DMA of step i + 3 (into the buffer of step i - 1), dS(i) stores
    //   phase A: S(i+1), dP(i+1) chains from fa; reads fb (tile i) and LSE2 of tile i + 1
    //   barrier: tile i + 2 landed in every wave's view
    //   phase B: dV(i), dK(i) from fb; P(i+1), dS(i+1) VALU in its gaps; reads fa (tile i + 2)
    // Buffer j is read from phase B of step j - 2 to phase A of step j and rewritten at the top of
    // step j + 1, after the barrier of step j: one barrier per step.
    auto step = [&](int i, auto mask_c) {
      const int m = m_of(cmt);
      const bool st_cur = DSOUT && !is_dead(m);
      // next step's tile coordinates (past the last step: anything; its results are unused)
      int cmt1 = cmt + 1, cg1 = cg;
      if (cmt1 == n_mt) {
        cmt1 = 0;
        ++cg1;
      }
      const int m1 = m_of(cmt1);
      stage_prep();  // DMA of step i + NB - 1 into the buffer step i - 1 used (pieces in phase A)
      char* const ds_dst = ds_lane + ch * (32 * 32 * 2);
      if constexpr (DSOUT) {
        if (cmt + 1 == n_mt) {
          ch_head += L.per_head();
          ch = ch_head;
        } else {
          const int t = m >> 5;  // q-tile left behind: nvis(t) = clamp(t + c, 0, nkt) chunks
          ch += min(max(t + L.c, 0), L.nkt);
        }
      }
      // phase A
      f32x4 l4[4];
      load_d4(i + 1);
      sdp([&](int mm) {
        if (!(FA2_PIPE_ABL & 8)) fb[mm] = rd_b(i, mm);
        if (mm == 12) load_l4(i + 1, l4);
        if (mm % 3 == 1) stage_piece(mm / 3);  // gaps 1, 4, 7, 10, 13
      });
      stage_advance();
      mid_wait(st_prev);
      if (st_cur) {
        // publish the rounded dS tile of this step for dq_ds_kernel (layout: dkdv_kernel's store_ds)
        __builtin_nontemporal_store(dsp[0], (u32x4*)ds_dst);
        __builtin_nontemporal_store(dsp[1], (u32x4*)(ds_dst + 16));
      }
      // phase B
      asm volatile("s_nop 1" ::: "memory");  // VALU-written B operands -> asm MFMA (see mfma_acc)
      {
        const Win wn = window(m1);
#pragma unroll
        for (int mm = 0; mm < 4 * NDT; ++mm) {
          // (mm, dt, r) are compile-time after unrolling: dV tile dt at a[kAccV + 16 dt], dK at a[kAccK + 16 dt]
          switch (mm) {
#define FA2_ACC_CASE(M)                                                                                  \
  case M:                                                                                                \
    if constexpr (((M) / NDT) & 1) mfma_acc<BF16, kAccK + 16 * ((M) % NDT)>(fb[M], dsp[(M) / NDT >> 1]); \
    else mfma_acc<BF16, kAccV + 16 * ((M) % NDT)>(fb[M], pp[(M) / NDT >> 1]);                            \
    break;
            FA2_ACC_CASE(0) FA2_ACC_CASE(1) FA2_ACC_CASE(2) FA2_ACC_CASE(3) FA2_ACC_CASE(4) FA2_ACC_CASE(5)
            FA2_ACC_CASE(6) FA2_ACC_CASE(7) FA2_ACC_CASE(8) FA2_ACC_CASE(9) FA2_ACC_CASE(10) FA2_ACC_CASE(11)
            FA2_ACC_CASE(12) FA2_ACC_CASE(13) FA2_ACC_CASE(14) FA2_ACC_CASE(15)
#undef FA2_ACC_CASE
          }
          // hipcc sees an asm MFMA read its operands at issue; the MFMA reads them for several
          // cycles more, so an operand register rewritten right after it (the next LDS read into
          // it, an address add) stalls or races the read: keep each A fragment alive two gaps on
          if (mm >= 2) asm volatile("" ::"v"(fb[mm - 2]));
          if (!(FA2_PIPE_ABL & 8)) fa[mm] = rd_a(i + 2, mm);
          // gaps 0-7: P of step i+1 (2 elements each); gaps 8-15: its dS (2 each) + packs
          if (FA2_PIPE_ABL & 4) {
          } else if (mm < 8) {
            p_elem(mask_c, 2 * mm, l4, wn);
            p_elem(mask_c, 2 * mm + 1, l4, wn);
          } else {
            ds_elem(2 * (mm - 8));
            ds_elem(2 * (mm - 8) + 1);
            if (mm & 1) pack((mm - 8) >> 1, ppn, dspn);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        asm volatile("" ::"v"(fb[14]), "v"(fb[15]), "v"(pp[0]), "v"(pp[1]), "v"(dsp[0]), "v"(dsp[1]));
      }
      pp[0] = ppn[0];
      pp[1] = ppn[1];
      dsp[0] = dspn[0];
      dsp[1] = dspn[1];
      st_prev = st_cur;
      cmt = cmt1;
      cg = cg1;
    };

    // ---- prologue: tiles 0 .. NB - 2 in flight; S(0), dP(0), their softmax gradient, and the
    // rows of tile 1 for phase A of step 0 ----------------------------------------------------
#pragma unroll
    for (int j = 0; j < NB - 1; ++j) stage_next();
    asm volatile("s_waitcnt vmcnt(5)\n\ts_barrier" ::: "memory");  // tiles 0 and 1 landed
#pragma unroll
    for (int mm = 0; mm < 2 * KS; ++mm) fa[mm] = rd_a(0, mm);
    load_d4(0);
    sdp([](int) {});
#pragma unroll
    for (int mm = 0; mm < 2 * KS; ++mm) fa[mm] = rd_a(1, mm);
    {
      f32x4 l4[4];
      load_l4(0, l4);
      const Win wn = window(m_of(0));
      // the first step is masked or not; one masked pass covers both (prologue only)
#pragma unroll
      for (int e = 0; e < 16; ++e) p_elem(std::true_type{}, e, l4, wn);
#pragma unroll
      for (int e = 0; e < 16; ++e) ds_elem(e);
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) pack(g4, pp, dsp);
    }
    for (int i = 0; i < total; ++i) {
      // mask class of step i + 1, whose softmax gradient this step computes
      int cmt1 = cmt + 1;
      if (cmt1 == n_mt) cmt1 = 0;
      if (needs_mask(m_of(cmt1))) step(i, std::true_type{});
      else step(i, std::false_type{});
    }
    vm_wait_all();  // no LDS-DMA may land after the workgroup's LDS is handed on
    agpr_drain();
  }

  // ---- store dK, dV (kv heads; fp32 group sum rounded once) ------------------------------
  if (total <= 0) agpr_drain();
  {
    uint16_t* dkrow = (uint16_t*)p.dk + b * p.dk_stride[0] + hkv * p.dk_stride[2] + (int64_t)kj * p.dk_stride[1];
    uint16_t* dvrow = (uint16_t*)p.dv + b * p.dv_stride[0] + hkv * p.dv_stride[2] + (int64_t)kj * p.dv_stride[1];
    const bool row_in = kj < p.seqlen_k;
    auto put = [&](uint16_t* row, int d0, f32x4 x, float mul) {
      float a[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = kval ? x[j] * mul : 0.f;
      if (row_in && d0 < D) *(u32x2*)(row + d0) = u32x2{E::pack2(a[0], a[1]), E::pack2(a[2], a[3])};
    };
    // accumulator register 4 g4 + j of d tile dt holds d = 32 dt + 8 g4 + 4 hh + j of this key
#define FA2_PUT(DT_, G4)                                                            \
    put(dvrow, 32 * (DT_) + 8 * (G4) + 4 * hh, acc_read4<kAccV + 16 * (DT_) + 4 * (G4)>(), 1.f); \
    put(dkrow, 32 * (DT_) + 8 * (G4) + 4 * hh, acc_read4<kAccK + 16 * (DT_) + 4 * (G4)>(), scale);
#define FA2_PUT_DT(DT_) FA2_PUT(DT_, 0) FA2_PUT(DT_, 1) FA2_PUT(DT_, 2) FA2_PUT(DT_, 3)
    FA2_PUT_DT(0) FA2_PUT_DT(1) FA2_PUT_DT(2) FA2_PUT_DT(3)
#undef FA2_PUT_DT
#undef FA2_PUT
    static_assert(NDT == 4, "accumulator map of the store above");
  }
}

template <bool BF16>
hipError_t launch_dkdv_pipe(const fa2_bwd_args& a, bool dsout, hipStream_t st) {
  dim3 grid(((a.seqlen_k + 127) / 128) * a.batch * a.heads_kv);
  const bool c = a.causal != 0;
  if (c && dsout) hipLaunchKernelGGL((dkdv_pipe_kernel<BF16, true, true>), grid, dim3(256), 0, st, a);
  else if (c) hipLaunchKernelGGL((dkdv_pipe_kernel<BF16, true, false>), grid, dim3(256), 0, st, a);
  else if (dsout) hipLaunchKernelGGL((dkdv_pipe_kernel<BF16, false, true>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((dkdv_pipe_kernel<BF16, false, false>), grid, dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace fa2
