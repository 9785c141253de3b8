// common.h -- CDNA4 (gfx950) building blocks shared by the forward and backward kernels.
//
// * MFMA: v_mfma_f32_32x32x16_{bf16,f16}.  Lane l (r = l & 31, h = l >> 5) holds
//     A[row r][k = 8h + j], B[k = 8h + j][col r]  (j = 0..7, one 16-byte fragment each),
//     C[row (i & 3) + 8 (i >> 2) + 4h][col r]    (i = 0..15, f32).
//   Every product in these kernels is arranged "swapped" (S^T = K Q^T, O^T = V^T P^T, ...)
//   so that the softmax row (one query) sits on one lane pair (l, l ^ 32): row statistics
//   are per-lane scalars and the probability accumulator is already the B operand of the next
//   product (the k order inside a 16-wide k-step is then 8(j>>2) + 4h + (j&3); the other
//   operand is read in that same order through ds_read_b64_tr_b16).
// * LDS tiles are stored d-tile major (32-column sub-tiles, 64-byte rows, 16-byte chunks
//   XOR-swizzled) so that 16-byte row reads (ds_read_b128, A/B fragments) and 4-row transposed
//   reads (ds_read_b64_tr_b16) are both bank-conflict free (layout below).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace fa2 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

typedef __attribute__((address_space(3))) char lds_char;

#define FA2_DEV __device__ __forceinline__

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kNegInf = -__builtin_inff();

// Defer-max threshold (log2 units): the running row max is only moved -- and O rescaled --
// when some row of the wave grows by more than this; P then stays <= 2^kDeferMax, which fp32
// accumulation and bf16/fp16 P (same relative precision at any magnitude) absorb exactly.
constexpr float kDeferMax = 8.f;

// ---------------------------------------------------------------------------------------------
// Element traits: raw 16-bit storage, conversions and the matching MFMA.
template <bool BF16>
struct Elem;

template <>
struct Elem<true> {
  FA2_DEV static float to_f32(uint16_t x) { return __uint_as_float(uint32_t(x) << 16); }
  FA2_DEV static uint16_t from_f32(float x) {
    __bf16 b = (__bf16)x;  // RNE, v_cvt_pk_bf16_f32 on gfx950
    return __builtin_bit_cast(uint16_t, b);
  }
  FA2_DEV static uint32_t pack2(float lo, float hi) {
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
    bf16x2 v = {(__bf16)lo, (__bf16)hi};
    return __builtin_bit_cast(uint32_t, v);
  }
  FA2_DEV static f32x16 mfma(u32x4 a, u32x4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  }
};

template <>
struct Elem<false> {
  FA2_DEV static float to_f32(uint16_t x) { return (float)__builtin_bit_cast(_Float16, x); }
  FA2_DEV static uint16_t from_f32(float x) {
    _Float16 h = (_Float16)x;
    return __builtin_bit_cast(uint16_t, h);
  }
  FA2_DEV static uint32_t pack2(float lo, float hi) {
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
    f16x2 v = {(_Float16)lo, (_Float16)hi};
    return __builtin_bit_cast(uint32_t, v);
  }
  FA2_DEV static f32x16 mfma(u32x4 a, u32x4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  }
};

// Bias element loads (bias may be f16, bf16 or f32; code 16 / 17 / 32 as encode_dtype).
FA2_DEV float load_bias(const void* base, int64_t idx, int code) {
  if (code == 32) return ((const float*)base)[idx];
  uint16_t x = ((const uint16_t*)base)[idx];
  return code == 17 ? Elem<true>::to_f32(x) : Elem<false>::to_f32(x);
}

// 16-bit bias tiles (BIASK 16: fp16, 17: bf16) of one wave: [32 rows][64 keys] staged by LDS-DMA
// in the Tile<64, 32> image (BufStager<64, 32, 64>).  Lane (r32, hh) of a swapped S^T accumulator
// holds keys 32 h + 8 g + 4 hh + (0..3) of row r32 in registers 4 g .. 4 g + 3 of half h: one
// 8-byte read per (h, g), unpacked by bias_elem.
FA2_DEV u32x2 bias_tile_frag(const char* tile, int r32, int hh, int h, int g) {
  const int off = h * (32 * 64) + r32 * 64 + (((g ^ (r32 >> 2)) & 3) << 4) + 8 * hh;
  return *(const u32x2*)(tile + off);
}
template <int BIASK>
FA2_DEV float bias_elem(u32x2 bv, int j) {  // element j (0..3) of a 4-key group
  const uint32_t wd = bv[j >> 1];
  if constexpr (BIASK == 17) return __uint_as_float((j & 1) ? (wd & 0xFFFF0000u) : (wd << 16));
  else return (float)__builtin_bit_cast(_Float16, (uint16_t)((j & 1) ? (wd >> 16) : (wd & 0xFFFFu)));
}
constexpr int kBiasTile = 32 * 64 * 2;  // bytes of one wave's bias tile
// host side: a bias the LDS-staged paths take (16-bit, every row 16-byte aligned)
inline bool bias16_rows(const void* bias, int dtype, const int64_t* stride) {
  return bias && (dtype == 16 || dtype == 17) && ((uintptr_t)bias & 15) == 0 && stride[0] % 8 == 0 &&
         stride[1] % 8 == 0 && stride[2] % 8 == 0;
}
#if FA2_HP_STAMPS
// development builds (-DFA2_HP_STAMPS=1): per-wave s_memtime sums of the hand-placed kernels,
// accumulated into one device buffer of 16 counters (fa2_debug_hp_stamps reads and clears it)
inline unsigned long long* hp_stamp_buf() {
  static unsigned long long* buf = nullptr;
  if (!buf && hipMalloc((void**)&buf, 16 * sizeof(unsigned long long)) == hipSuccess)
    (void)hipMemset(buf, 0, 16 * sizeof(unsigned long long));
  return buf;
}
#endif
// host side: compute units of the current device (persistent grids), cached per device id
inline int device_cu_count() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (!cached[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

// ---------------------------------------------------------------------------------------------
// Cross-half exchange: returns {x of lanes 0-31, x of lanes 32-63} in every lane.
FA2_DEV float half_max(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
FA2_DEV float half_sum(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

FA2_DEV f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// ---------------------------------------------------------------------------------------------
// XCD-aware work order.  Workgroups are dealt round-robin to the 8 XCDs (block L -> XCD L % 8),
// each with its own L2.  With a 2-D grid whose x extent is a multiple of 8, every XCD would get
// the same few x indices for all heads -- under a causal mask that is 2.4x more work on one
// XCD than on another.  Instead the work items are numbered head-major (all blocks of a head
// consecutive, heaviest first) and XCD x gets one contiguous slice of that list (bijective
// remap for any count): balanced work per XCD, and the blocks of a head -- which share its K/V
// -- run together on one XCD's L2.
FA2_DEV int xcd_item(int L, int total) {
  const int x = L & 7, idx = L >> 3;
  const int q = total >> 3, r = total & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + idx;
}

// The unit sequence of one workgroup of a persistent kernel (fwd_hp, dq_hp, dkdv_hp).  Work items
// -- a causal pair of mirrored blocks (rep 0 = heavy, 1 = light) or one block -- are numbered
// head-major, `per` items per head of n blocks; XCD x (workgroups L = x + 8 j) owns a contiguous
// slice [start, end) in proportion to its W workgroups.
//  * whole items (no pairs, or W odd): workgroup j runs items start + j + k W, an item's blocks
//    back to back;
//  * split pairs (pairs, W even): the W workgroups form W/2 slots of two, and in round k the two
//    workgroups of slot s run the two blocks of item start + k W/2 + s side by side (rep =
//    side ^ (k & 1)).  The XCD's workgroups then touch W/2 items at once -- half the heads of one
//    pair per workgroup (cfg3: two heads' K / V, 4 MiB = one L2, instead of four) -- and a
//    workgroup alternates heavy and light blocks (balanced over two rounds).  A self-mirrored
//    middle item (one block) leaves its side-1 workgroup to the next round.
// State is (item, rep, k); everything else is recomputed from the grid, so little stays live.
struct PersistSched {
  int item, rep, k;

  struct Slice {
    int start, end, W, j;
  };
  static FA2_DEV Slice slice(int T) {
    // opaque copies: nothing of the schedule is hoisted out of a kernel's unit loop and kept live
    // (in VGPRs, for the divisions) across its asm statement
    int G = gridDim.x, L = blockIdx.x;
    asm volatile("" : "+s"(G), "+s"(L), "+s"(T));
    const int x = L & 7;
    const int g8 = G >> 3, gr = G & 7;
    const int cw0 = x * g8 + min(x, gr);
    Slice s;
    s.W = g8 + (x < gr ? 1 : 0);
    s.j = L >> 3;
    s.start = (int)((int64_t)T * cw0 / G);
    s.end = (int)((int64_t)T * (cw0 + s.W) / G);
    return s;
  }
  static FA2_DEV bool split(const Slice& s, bool pair) { return pair && s.W >= 2 && !(s.W & 1); }
  static FA2_DEV int reps(int it, int n, int per, bool pair) {
    const int m = it % per;
    return pair && n - 1 - m != m ? 2 : 1;
  }
  FA2_DEV void place(const Slice& s) {
    const int h = s.W >> 1, slot = s.j % h, side = s.j / h;
    item = s.start + k * h + slot;
    rep = side ^ (k & 1);
  }
  // the first unit; false: this workgroup has none
  FA2_DEV bool first(int T, int n, int per, bool pair) {
    const Slice s = slice(T);
    k = 0;
    if (split(s, pair)) {
      place(s);
      while (item < s.end && rep >= reps(item, n, per, pair)) {
        ++k;
        place(s);
      }
    } else {
      item = s.start + s.j;
      rep = 0;
    }
    uniform();
    return item < s.end;
  }
  // advance to the next unit; false: none left
  FA2_DEV bool next(int T, int n, int per, bool pair) {
    const Slice s = slice(T);
    if (split(s, pair)) {
      do {
        ++k;
        place(s);
      } while (item < s.end && rep >= reps(item, n, per, pair));
    } else if (++rep >= reps(item, n, per, pair)) {
      item += s.W;
      rep = 0;
    }
    uniform();
    return item < s.end;
  }
  // the state in SGPRs (the integer divisions run on the VALU)
  FA2_DEV void uniform() {
    item = __builtin_amdgcn_readfirstlane(item);
    rep = __builtin_amdgcn_readfirstlane(rep);
    k = __builtin_amdgcn_readfirstlane(k);
  }
};

// ---------------------------------------------------------------------------------------------
// LDS tile layout ("d-tile major").  A tile of ROWS x DT 16-bit elements is stored as DT/32
// sub-tiles of ROWS x 32 columns; each sub-tile row is 64 bytes (four 16-byte chunks) and
// chunk cc of row r sits at cc ^ ((r >> 2) & 3).  With this image
//  (a) a ds_read_b128 lane group (16 lanes, 16 distinct rows, one chunk each) hits 16 distinct
//      16-byte bank slots, and
//  (b) a ds_read_b64_tr_b16 half wave (4 consecutive rows x 64 bytes of one sub-tile) covers
//      one whole 256-byte bank row,
// so both are conflict free, and -- unlike an XOR over 256-byte rows -- every read of a
// (sub-tile, row block) differs from the lane's base address by a compile-time constant, so the
// loops keep only a couple of address registers per tile (ds_read offset immediates).
template <int DT, int ROWS>
struct Tile {
  static constexpr int kChunks = DT / 8;
  static constexpr int kSub = ROWS * 64;  // bytes per 32-column sub-tile
  // byte offset of global chunk c (8 columns) of row r
  FA2_DEV static int off(int r, int c) { return (c >> 2) * kSub + r * 64 + (((c & 3) ^ ((r >> 2) & 3)) << 4); }
};

// 16-byte row fragment for k-step ks of a 32x32x16 MFMA: row row0 + r32 (row0 % 16 == 0),
// columns 16 ks + 8 hh + (0..7).  Written so that every (row0, ks) differs from the lane's
// base address by an immediate (only the parity of ks changes the swizzled chunk).
template <int DT, int ROWS>
FA2_DEV u32x4 lds_row_frag(const char* tile, int row0, int r32, int ks, int hh) {
  const int cc = ((ks & 1) << 1) | hh;
  const int off = (ks >> 1) * Tile<DT, ROWS>::kSub + (row0 + r32) * 64 + ((cc ^ ((r32 >> 2) & 3)) << 4);
  return *(const u32x4*)(tile + off);
}

// Transposed fragment for the operand whose k index runs over tile ROWS (row0 % 16 == 0,
// col0 % 32 == 0): element j of lane (r32 = l & 31, h = l >> 5) is
//   tile[row0 + 8 (j >> 2) + 4 h + (j & 3)][col0 + r32]
// i.e. the permuted k order of a C-layout accumulator reused as the other MFMA operand.
// ds_read_b64_tr_b16: lane 4q+p of each 16-lane group addresses row q, columns 4p..4p+3 of its
// block and receives column (lane & 15) of the 4 rows.
template <int DT, int ROWS>
FA2_DEV u32x4 lds_tr_frag(const char* tile, int row0, int col0, int lane) {
  const int i = lane & 15, g = lane >> 4, h = lane >> 5;
  const int q = i >> 2, pq = i & 3;
  const int cc = 2 * (g & 1) + (pq >> 1);
  // rows row0 + 4h + q (first read) and row0 + 8 + 4h + q: (row >> 2) & 3 = h and h ^ 2
  const int base = (col0 >> 5) * Tile<DT, ROWS>::kSub + (row0 + 4 * h + q) * 64 + 8 * (pq & 1);
  const lds_char* pa = (const lds_char*)(tile + base + ((cc ^ h) << 4));
  const lds_char* pb = (const lds_char*)(tile + base + 8 * 64 + ((cc ^ h ^ 2) << 4));
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)pa);
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)pb);
  u32x2 a = __builtin_bit_cast(u32x2, lo), b = __builtin_bit_cast(u32x2, hi);
  return u32x4{a[0], a[1], b[0], b[1]};
}

// ---------------------------------------------------------------------------------------------
// LDS-DMA issued from inline asm.  hipcc tracks its own global_load_lds builtins and, unable to
// tell the DMA's LDS destination from the buffer being read, inserts s_waitcnt vmcnt(0) before
// the next ds_read -- which drains the next tile's prefetch in the middle of the current tile.
// Issued from asm the DMA is invisible to that pass; the kernels retire it themselves with
// vm_wait_all() right before the barrier that publishes the tile (the compiler's own waits
// for its own loads only over-wait, never under-wait, since VMEM ops retire in issue order).
FA2_DEV uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
FA2_DEV void glds16(const void* gsrc, uint32_t lds_base_uniform) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_base_uniform)
      : "memory");
}
FA2_DEV void glds4(const void* gsrc, uint32_t lds_base_uniform) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_base_uniform)
      : "memory");
}
// a wave-uniform 64-bit integer pinned to SGPRs (keeps loop-carried counters out of VGPRs)
FA2_DEV int64_t uniform64(int64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
FA2_DEV void vm_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ---------------------------------------------------------------------------------------------
// Global -> LDS tile staging.  ROWS rows starting at global row `row0` (row stride
// `row_stride` elements) of a [*, D] slice; rows >= row_end and columns >= D must not leak
// NaN/Inf garbage into the MFMAs, so:
//  ALIGNED (D % 8 == 0, 16-byte aligned rows): LDS-DMA 16-byte pieces
//    (global_load_lds_dwordx4: LDS destination = wave base + lane*16, so the swizzle is applied
//    to the per-lane SOURCE address); out-of-range rows / chunks are clamped to valid memory
//    (finite data that is masked out of every result).
//  otherwise: element loads with zero fill + ds_write.
template <int DT, int ROWS, int NTHREADS, bool ALIGNED>
FA2_DEV void stage_tile(char* tile, const uint16_t* g, int64_t row_stride, int row0, int row_end,
                        int D, int tid) {
  constexpr int kChunks = DT / 8;
  constexpr int kPieces = ROWS * kChunks;  // 16-byte pieces in the tile
  if constexpr (ALIGNED) {
    static_assert(kPieces % 64 == 0, "tile must be a whole number of wave pieces");
    const int wave = tid >> 6, lane = tid & 63;
    const int dchunks = D >> 3;
#pragma unroll
    for (int it = 0; it < (kPieces + NTHREADS - 1) / NTHREADS; ++it) {
      const int wbase = (it * (NTHREADS / 64) + wave) * 64;  // first piece of this wave
      if (kPieces % NTHREADS != 0 && wbase >= kPieces) break;  // wave-uniform
      const int piece = wbase + lane;
      const int sub = piece / (ROWS * 4);                      // 32-column sub-tile
      const int within = piece % (ROWS * 4);
      const int pr = within >> 2;                              // row
      const int cc = (within & 3) ^ ((pr >> 2) & 3);           // logical chunk stored here
      const int c = sub * 4 + cc;
      int grow = row0 + pr;
      grow = grow < row_end ? grow : row_end - 1;
      const int gc = c < dchunks ? c : dchunks - 1;
      const uint16_t* src = g + (int64_t)grow * row_stride + gc * 8;
      glds16(src, __builtin_amdgcn_readfirstlane(lds_addr(tile + wbase * 16)));
    }
  } else {
    // one thread per (row, chunk); 8 scalar loads each
    for (int piece = tid; piece < kPieces; piece += NTHREADS) {
      const int r = piece / kChunks, c = piece % kChunks;
      const int grow = row0 + r;
      uint16_t vals[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int d = c * 8 + j;
        vals[j] = (grow < row_end && d < D) ? g[(int64_t)grow * row_stride + d] : (uint16_t)0;
      }
      u32x4 pk;
#pragma unroll
      for (int j = 0; j < 4; ++j) pk[j] = uint32_t(vals[2 * j]) | (uint32_t(vals[2 * j + 1]) << 16);
      *(u32x4*)(tile + Tile<DT, ROWS>::off(r, c)) = pk;
    }
  }
}

// LDS-DMA stager for a ROWS x DT tile with the per-lane source offsets precomputed once
// (row * row_stride + chunk * 8, elements), so that issuing a full tile costs one 64-bit add
// per 16-byte piece.  Only a tile that crosses row_end takes the clamping path.
template <int DT, int ROWS, int NTHREADS>
struct Stager {
  static constexpr int kPieces = ROWS * DT / 8;
  static constexpr int kIters = (kPieces + NTHREADS - 1) / NTHREADS;
  static_assert(kPieces % 64 == 0, "tile must be a whole number of wave pieces");
  int32_t off[kIters];  // element offset of this lane's piece relative to the tile's first row
  int wave;
  uint32_t wave_lds;    // byte offset of this wave's first piece (wave-uniform, SGPR)

  FA2_DEV void init(int tid, int64_t row_stride, int D) {
    wave = tid >> 6;
    wave_lds = __builtin_amdgcn_readfirstlane(wave * 64 * 16);
    const int lane = tid & 63, dchunks = D >> 3;
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
      const int piece = (it * (NTHREADS / 64) + wave) * 64 + lane;
      const int sub = piece / (ROWS * 4), within = piece % (ROWS * 4);
      const int pr = within >> 2;
      const int c = sub * 4 + ((within & 3) ^ ((pr >> 2) & 3));
      const int gc = c < dchunks ? c : dchunks - 1;
      off[it] = (int32_t)(pr * row_stride) + gc * 8;
    }
  }
  // Branch-free single-piece issue for kernels that spread a tile's DMA over their steps
  // (requires NTHREADS % (ROWS * 4) == 0: piece it of a lane is it * NTHREADS + tid, so all
  // its pieces lie in tile row (tid % (ROWS * 4)) / 4 and one per-tile row clamp `adj`
  // (elements, from row_adjust) serves them all).
  FA2_DEV int64_t row_adjust(int64_t row_stride, int row0, int row_end, int tid) const {
    static_assert(NTHREADS % (ROWS * 4) == 0, "one tile row per lane");
    const int pr = (tid % (ROWS * 4)) >> 2;
    const int over = row0 + pr - (row_end - 1);
    return over > 0 ? -(int64_t)over * row_stride : 0;
  }
  FA2_DEV void piece(char* tile, const uint16_t* gt, int64_t adj, int it) const {
    const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(tile)) + wave_lds;
    glds16(gt + off[it] + adj, base + it * NTHREADS * 16);
  }
  // rows [row0, row0 + ROWS) of g (row stride row_stride); rows >= row_end re-read row_end - 1
  FA2_DEV void issue(char* tile, const uint16_t* g, int64_t row_stride, int row0, int row_end, int tid) {
    const uint16_t* gt = g + (int64_t)row0 * row_stride;
    const uint32_t base = __builtin_amdgcn_readfirstlane(lds_addr(tile)) + wave_lds;
    if (row0 + ROWS <= row_end) {  // whole tile in range: one add per piece
#pragma unroll
      for (int it = 0; it < kIters; ++it) {
        if (kPieces % NTHREADS != 0 && (it * (NTHREADS / 64) + wave) * 64 >= kPieces) break;
        glds16(gt + off[it], base + it * NTHREADS * 16);
      }
    } else {
#pragma unroll
      for (int it = 0; it < kIters; ++it) {
        const int wbase = (it * (NTHREADS / 64) + wave) * 64;
        if (kPieces % NTHREADS != 0 && wbase >= kPieces) break;  // wave-uniform
        const int piece = wbase + (tid & 63);
        const int pr = (piece % (ROWS * 4)) >> 2;
        const int clamp = row0 + pr < row_end ? 0 : (row0 + pr - (row_end - 1));
        glds16(gt + off[it] - (int64_t)clamp * row_stride, base + it * NTHREADS * 16);
      }
    }
  }
};

// Buffer-resource LDS-DMA stager (buffer_load_dwordx4 ... lds) for a ROWS x DT tile.  The
// descriptor of each tile starts at the tile's first row and its range ends at the last valid
// row, so rows past the end read as zeros by the hardware range check: no clamping and no
// per-piece address arithmetic -- every lane's byte offset of its piece is a constant.
// Requires NTHREADS % (ROWS * 4) == 0 (all pieces of a lane in one tile row).
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));

FA2_DEV i32x4 make_rsrc(const void* base, uint32_t n) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  i32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((int32_t)(uint32_t)a);
  r[1] = __builtin_amdgcn_readfirstlane((int32_t)((uint32_t)(a >> 32) & 0xFFFFu));  // stride 0
  r[2] = __builtin_amdgcn_readfirstlane((int32_t)n);
  r[3] = 0x00020000;  // gfx9 raw buffer: 32-bit data, no swizzle
  return r;
}

// Descriptor of a 16-bit bias tile [rows from row0][tile_keys keys] whose key 0 is element g of
// row 0 (row stride `stride` elements, a multiple of 8 -- bias16_rows).  The range ends at the
// last valid key of the last valid row, rounded up to a whole 16-byte chunk (which a 16-byte
// aligned row always holds): pieces for keys past seqlen_k of the final row read as zeros
// instead of past the end of the tensor.  keys_left = seqlen_k - (first key of the tile).
// Rows past row_end read as zeros as in BufStager::tile_rsrc.
FA2_DEV i32x4 bias_tile_rsrc(const uint16_t* g, int64_t stride, int row0, int row_end, int max_rows, int keys_left,
                             int tile_keys) {
  const int rows = min(max(row_end - row0, 0), max_rows);
  const int kv = min(max((keys_left + 7) & ~7, 0), tile_keys);
  const uint32_t n = (rows > 0 && kv > 0) ? (uint32_t)(rows - 1) * (uint32_t)(stride * 2) + (uint32_t)kv * 2u : 0u;
  return make_rsrc(g + (int64_t)row0 * stride, n);
}

// One dword per lane by buffer LDS-DMA (buffer_load_dword ... lds): LDS destination =
// lds_base_uniform + 4 * lane (active lanes), source = descriptor base + voff bytes.
FA2_DEV void blds4(uint32_t voff, i32x4 rsrc, uint32_t lds_base_uniform) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dword %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rsrc), "s"(lds_base_uniform)
      : "memory");
}

// The same for lanes 0..31 only (EXEC's high half cleared around the one instruction and
// restored): a 32-dword row piece from a whole-wave branch, without a divergent branch per half.
FA2_DEV void blds4_lo32(uint32_t voff, i32x4 rsrc, uint32_t lds_base_uniform) {
  uint32_t keep;
  uint64_t save;
  asm volatile(
      "s_mov_b64 %1, exec\n\ts_mov_b32 exec_hi, 0\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 1\n\t"
      "buffer_load_dword %2, %3, 0 offen lds\n\ts_mov_b32 m0, %0\n\ts_mov_b64 exec, %1"
      : "=&s"(keep), "=&s"(save)
      : "v"(voff), "s"(rsrc), "s"(lds_base_uniform)
      : "memory");
}

template <int DT, int ROWS, int NTHREADS>
struct BufStager {
  static constexpr int kPieces = ROWS * DT / 8;
  static constexpr int kIters = (kPieces + NTHREADS - 1) / NTHREADS;
  static_assert(kPieces % 64 == 0 && (kPieces % NTHREADS == 0 || kIters == 1), "whole wave pieces");
  uint32_t voff[kIters];  // byte offset of this lane's pieces from the tile's first row
  uint32_t wave_lds;      // byte offset of this wave's first piece in the tile (SGPR)
  int wave;               // wave-uniform (SGPR)

  FA2_DEV void init(int tid, int64_t row_stride, int D) {
    wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63, dchunks = D >> 3;
    wave_lds = __builtin_amdgcn_readfirstlane(wave * 64 * 16);
#pragma unroll
    for (int it = 0; it < kIters; ++it) {
      const int piece = (it * (NTHREADS / 64) + wave) * 64 + lane;
      const int sub = piece / (ROWS * 4), within = piece % (ROWS * 4);
      const int pr = within >> 2;
      const int c = sub * 4 + ((within & 3) ^ ((pr >> 2) & 3));
      const int gc = c < dchunks ? c : dchunks - 1;
      // 32-bit lane offsets (a tile's byte range fits the descriptor's 32-bit range anyway):
      // 64-bit products here get kept as register pairs, which kernels at the register limit spill
      voff[it] = ((uint32_t)pr * (uint32_t)row_stride + (uint32_t)(gc * 8)) * 2u;
    }
  }
  // descriptor of the tile starting at row row0 of g (rows >= row_end read as zero)
  // (max_rows = rows whose bytes fit the 32-bit range field, see max_rows())
  FA2_DEV static i32x4 tile_rsrc(const uint16_t* g, int64_t row_stride, int row0, int row_end, int max_rows) {
    const int rows = min(max(row_end - row0, 0), max_rows);
    return make_rsrc(g + (int64_t)row0 * row_stride, (uint32_t)rows * (uint32_t)(row_stride * 2));
  }
  FA2_DEV static int max_rows(int64_t row_stride) {  // wave-uniform: kept in an SGPR
    return __builtin_amdgcn_readfirstlane((int)min((int64_t)0x7FFFFFFF, 0xFFFFFFFFll / (row_stride * 2)));
  }
  // returns the saved m0: a token a caller can feed to a later statement to keep it behind the DMA
  FA2_DEV uint32_t piece(char* tile, i32x4 rsrc, int it) const {
    if (kPieces % NTHREADS != 0 && wave * 64 >= kPieces) return 0;  // small tile: idle waves
    const uint32_t lds = __builtin_amdgcn_readfirstlane(lds_addr(tile)) + wave_lds + it * NTHREADS * 16;
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff[it]), "s"(rsrc), "s"(lds)
        : "memory");
    return keep;
  }
  FA2_DEV uint32_t issue(char* tile, const uint16_t* g, int64_t row_stride, int row0, int row_end, int max_rows) const {
    const i32x4 r = tile_rsrc(g, row_stride, row0, row_end, max_rows);
    uint32_t tok = 0;
#pragma unroll
    for (int it = 0; it < kIters; ++it) tok = piece(tile, r, it);
    return tok;
  }
};

// 16-byte register fragment straight from global memory: elements [d0, d0 + 8) of one row;
// zero outside [0, D) or when !valid.
template <bool ALIGNED>
FA2_DEV u32x4 load_row_frag(const uint16_t* row, int d0, int D, bool valid) {
  if constexpr (ALIGNED) {
    if (valid && d0 < D) return *(const u32x4*)(row + d0);
    return u32x4{0u, 0u, 0u, 0u};
  } else {
    uint16_t v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (valid && d0 + j < D) ? row[d0 + j] : (uint16_t)0;
    u32x4 pk;
#pragma unroll
    for (int j = 0; j < 4; ++j) pk[j] = uint32_t(v[2 * j]) | (uint32_t(v[2 * j + 1]) << 16);
    return pk;
  }
}

// ---------------------------------------------------------------------------------------------
// Epilogue store of one wave's 32 x DT accumulator image through a wave-private LDS staging area.
// acc[dt] is C^T of a swapped product: lane (r = lane & 31, h = lane >> 5) holds output row r,
// columns 32 dt + 8 (i >> 2) + 4 h + (i & 3).  Stored straight from registers, every store
// instruction touches 32 rows x 16 bytes (row-per-lane); the epilogue tail is bound by the number
// of such row segments, not by bytes (MI355X_MICROARCH.md, "attention epilogue store tail").  Here
// each lane pair first writes its row into LDS (one ds_write_b128 per 8 columns after a
// v_permlane32_swap pairing), then the wave reads the image back row-contiguous: instruction j
// stores rows j * RPI .. j * RPI + RPI - 1 as whole D * 2-byte segments.
// Staging image: row r at r * DT * 2 bytes, 16-byte chunk c at c ^ (r % CPR) -- conflict free for
// the 8-lane write groups (8 rows, one chunk) and for the ds_read_b128 lane groups (whole rows).
// Element value: valid ? acc * mul : 0, rounded once.  Rows [nrows, 32) and columns [D, DT) are
// not stored (D % 8 == 0).  The caller guarantees no other wave still reads `stage`.
template <bool BF16, int DT>
FA2_DEV void store_rows_lds(char* stage, const f32x16* acc, float mul, bool valid, uint16_t* g0, int64_t rstride,
                            int nrows, int D, int lane, uint64_t* tacc = nullptr) {
#if FA2_HP_STAMPS
  uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
  using E = Elem<BF16>;
  constexpr int NDT = DT / 32;
  constexpr int CPR = DT / 8;   // 16-byte chunks per row
  constexpr int RPI = 64 / CPR;  // rows per store instruction
  // the row offsets below depend on the lane only: computed from an opaque copy of it, so that
  // they cannot be hoisted out of a kernel's work-item loop and kept live (spilled) across it
  asm volatile("" : "+v"(lane));
  const int r = lane & 31, h = lane >> 5;
  const float m = valid ? mul : 0.f;
  char* row = stage + r * (DT * 2);
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
    for (int g4 = 0; g4 < 4; g4 += 2) {
      const uint32_t a0 = E::pack2(acc[dt][4 * g4 + 0] * m, acc[dt][4 * g4 + 1] * m);
      const uint32_t a1 = E::pack2(acc[dt][4 * g4 + 2] * m, acc[dt][4 * g4 + 3] * m);
      const uint32_t b0 = E::pack2(acc[dt][4 * g4 + 4] * m, acc[dt][4 * g4 + 5] * m);
      const uint32_t b1 = E::pack2(acc[dt][4 * g4 + 6] * m, acc[dt][4 * g4 + 7] * m);
      const auto s0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
      const auto s1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
      const int c = 4 * dt + g4 + h;  // chunk: columns 8c .. 8c + 7
      *(u32x4*)(row + 16 * (c ^ (r % CPR))) = u32x4{s0[0], s1[0], s0[1], s1[1]};
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#if FA2_HP_STAMPS
  if (tacc) {  // (development stamp builds: pack + LDS write, read back, global stores)
    const uint64_t t = __builtin_amdgcn_s_memtime();
    tacc[0] += t - t0;
    t0 = t;
  }
#endif
  const int c = lane % CPR;
  // every row read issued before the first store (one LDS wait, not one per store)
  u32x4 v[32 / RPI];
#pragma unroll
  for (int j = 0; j < 32 / RPI; ++j) {
    const int R = j * RPI + lane / CPR;
    v[j] = *(const u32x4*)(stage + R * (DT * 2) + 16 * (c ^ (R % CPR)));
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#if FA2_HP_STAMPS
  if (tacc) {
    const uint64_t t = __builtin_amdgcn_s_memtime();
    tacc[1] += t - t0;
    t0 = t;
  }
#endif
#pragma unroll
  for (int j = 0; j < 32 / RPI; ++j) {
    const int R = j * RPI + lane / CPR;
    if (R < nrows && 8 * c < D) *(u32x4*)(g0 + (int64_t)R * rstride + 8 * c) = v[j];
  }
#if FA2_HP_STAMPS
  if (tacc) tacc[2] += __builtin_amdgcn_s_memtime() - t0;
#endif
}

// a ^ b ^ c in one gfx950 v_bitop3_b32 (truth table 0x96); the backend emits two v_xor_b32 here.
// c must be wave-uniform (it is bound to an SGPR).
FA2_DEV uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(c));
  return r;
}

// ---------------------------------------------------------------------------------------------
// 32 x 32 bit-matrix transpose across each 32-lane half: lane r holds row r (bit k = element
// (r, k)); afterwards lane k holds column k (bit r = element (r, k)).  Five xor stages of
// ds_swizzle (bitmask mode, no LDS access); every lane of the wave must be active.
template <int J>
FA2_DEV uint32_t transpose32_stage(uint32_t x, int r32) {
  constexpr uint32_t m = J == 16 ? 0x0000FFFFu : J == 8 ? 0x00FF00FFu : J == 4 ? 0x0F0F0F0Fu : J == 2 ? 0x33333333u : 0x55555555u;
  const uint32_t y = (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, (J << 10) | 0x1F);
  // branch-free select on the lane bit (a ternary here compiles to five divergent branches)
  const uint32_t hi = 0u - (uint32_t)((r32 >> __builtin_ctz(J)) & 1);
  return ((((y >> J) & m) | (x & ~m)) & hi) | (((x & m) | ((y & m) << J)) & ~hi);
}
FA2_DEV uint32_t transpose32_lanes(uint32_t x, int r32) {
  x = transpose32_stage<16>(x, r32);
  x = transpose32_stage<8>(x, r32);
  x = transpose32_stage<4>(x, r32);
  x = transpose32_stage<2>(x, r32);
  return transpose32_stage<1>(x, r32);
}

// ---------------------------------------------------------------------------------------------
// Philox4x32-10, first output word, counter (lo, hi, 0, 0), key (seed_lo, seed_hi), converted
// to [0,1) exactly like Triton's tl.rand (triton/language/random.py:13-156; see
// oracle/philox.py).  Used for the forward dropout mask keep = rand > p
// (/root/reference/src/forward/compute_row_blocks.py:76-79).  seed is a kernel argument (wave-uniform:
// the round keys live in SGPRs).
FA2_DEV float philox_uniform(uint64_t seed, uint64_t offset) {
  uint32_t c0 = (uint32_t)offset, c1 = (uint32_t)(offset >> 32), c2 = 0, c3 = 0;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    // one 32 x 32 -> 64-bit product per multiplier (v_mad_u64_u32) gives both the high word
    // and the low word: half the integer multiplies of separate mul_hi / mul_lo
    const uint64_t pa = (uint64_t)0xCD9E8D57u * c2, pb = (uint64_t)0xD2511F53u * c0;
    c0 = xor3((uint32_t)(pa >> 32), c1, k0);
    c2 = xor3((uint32_t)(pb >> 32), c3, k1);
    c1 = (uint32_t)pa;
    c3 = (uint32_t)pb;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  int32_t x = (int32_t)c0;
  x = x < 0 ? -x - 1 : x;
  return (float)x * 4.6566127342e-10f;
}

// Dropout keep bits of one lane's 16 accumulator registers: bit i = (philox_uniform(seed,
// base + o(i) * step) > p), o(i) = (i & 3) + 8 (i >> 2) (the register's row or key offset in a
// 32 x 32 accumulator).  A rolled loop (two chains in flight) for dkdv_kernel's step start: fully
// unrolled next to its MFMA operands, the 16 Philox states spilled 180-230 bytes per lane
// (cfg3 dropout dK/dV 6.51 -> 5.42 ms with this, r03k).
FA2_DEV uint32_t dropout_keep16(uint64_t seed, uint64_t base, uint64_t step, float p) {
  uint32_t bits = 0;
#pragma unroll 2
  for (int i = 0; i < 16; ++i) {
    const uint64_t o = (uint64_t)((i & 3) + 8 * (i >> 2));
    bits |= (philox_uniform(seed, base + o * step) > p ? 1u : 0u) << i;
  }
  return bits;
}

}  // namespace fa2
