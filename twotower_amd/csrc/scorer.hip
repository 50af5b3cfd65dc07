// Fused in-batch sampled-softmax cross entropy on gfx950 MFMA
// (in_batch_sampled_softmax_loss, twotower/losses.py:88-118):
//   S = Q D^T (B x M), logits = S / tau, labels = arange(B) (+label_off under data parallel),
//   loss = mean_i (logsumexp_j logits_ij - logits_i,label_i).
// B x M is never materialised.  One engine serves both passes:
//   * a workgroup keeps 4 x 32 "column" rows resident in VGPRs as the MFMA B operand and
//     streams the other matrix through a double-buffered, XOR-swizzled LDS tile;
//   * X = R_tile C^T (32x32 per wave; 32x32x16 bf16 or 32x32x2 f32 MFMA), an elementwise map
//     G = f(X) in registers, then Acc^T += R_tile^T G with the X accumulator reused as the next
//     MFMA's B operand (no LDS round trip) and R_tile^T read with ds_read_b64_tr_b16.
//   forward  (R = D, C = Q): G = 2^(X c2 - shift_i), shift_i >= max_j X_ij c2 a per-query bound
//            (no running max, no accumulator rescale); Acc = O^T, so dQ needs no extra pass.
//   backward (R = Q, C = D): G = 2^(X c2 - lse2_i); Acc = dD^T.
// The inner loop has no masks and no label logic: rows past the end are zero rows staged from
// a pad buffer (backward: their lse = +inf, so G = 0); in the forward each pad row adds exactly
// 2^-shift_i to l_i and nothing to O, removed by the combine.  The label terms (the diagonal
// logit, the -q_i contribution to dD) are applied by the combine kernels.
// The streamed dimension is split over workgroups (blockIdx % S == split: one split per XCD
// when S == 8); split partials are merged by the combine kernels.
#include <atomic>
#include <type_traits>
#include <cstdlib>
#include <cstring>

#include "common.hpp"

namespace tt {
int launch_mean(const float* x, int64_t n, float* out, hipStream_t s);

namespace {

constexpr int NW = 4;
constexpr int NT = NW * kWave;
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
constexpr int kPadBytes = 2048;  // zero row source (>= one 1 KiB row) + one +inf float after it
enum Mode { FWD = 0, DD = 1 };
constexpr int kMaxPrepBlocks = 512;  // per-block norm maxima of the prep (readers fold <= this many)
constexpr int kTailRows = 64;         // zero rows after each bf16 operand copy (>= the bf16 engine's BJ)
static_assert(kTailRows == TT_INBATCH_TAIL_ROWS && kMaxPrepBlocks == TT_INBATCH_MAX_PARTS, "ABI constants");

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(3))) char lds_char_t;
typedef __attribute__((address_space(3))) bf16x8 lds_bf16x8_t;
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;
typedef __attribute__((address_space(3))) f32x4 lds_f32x4_t;
typedef __attribute__((address_space(3))) float lds_float_t;

__host__ __device__ constexpr int acc_row(int v, int hh) { return (v & 3) + 8 * (v >> 2) + 4 * hh; }

// ------------------------------------------------------------------------------------------
// LDS tile image shared by both engines: BJ rows of H elements, row-major, 16-byte chunk c of
// row r stored at chunk c ^ (r & SWM).  The swizzle makes the 32-rows-same-column ds_read_b128
// operand reads hit distinct slots; the column reads (ds_read_b32 / ds_read_b64_tr_b16) stay
// inside one row.  Tiles are filled by global_load_lds (16 B per lane, 1 KiB per wave-
// instruction, no staging VGPRs): the LDS side is written linearly, so the swizzle is applied
// to the per-lane SOURCE address (cdna_hip_programming.md rule 21).
template <typename ET, int H>
struct Tile {
  static constexpr int BJ = sizeof(ET) == 2 ? 64 : 32;
  static constexpr int ROWB = H * (int)sizeof(ET);
  static constexpr int NCH = ROWB / 16;
  // bf16: 4-bit XOR (row reads conflict-free).  f32: 3-bit XOR keeps every h-tile of a column
  // read at a constant byte offset from the first, at the price of 2-way row-read conflicts.
  static constexpr int SWM = ((sizeof(ET) == 2 && NCH >= 16) ? 16 : (NCH >= 8 ? 8 : NCH)) - 1;
  static constexpr int STAGE_B = BJ * ROWB;
  static constexpr int NI = STAGE_B / 1024 / NW;  // glds wave-instructions per wave per stage
  static_assert(NI * 1024 * NW == STAGE_B, "stage must be a whole number of 1 KiB pieces per wave");
  static constexpr int NSTAGE = sizeof(ET) == 2 ? 4 : 2;  // bf16: four-stage ring (see the engine)
  static constexpr int LSE_OFF = NSTAGE * STAGE_B;
  static constexpr int LDS_BYTES = NSTAGE * STAGE_B + NSTAGE * 64 * 4;  // stages + one 64-float lse row each
  // Chunk XOR of a row.  bf16 rows of >= 256 B use the dual-use swizzle (cdna_hip_programming.md
  // T10 (b)): bits 0-1 of the row go to chunk bits 2-3 and bits 2-3 to chunk bits 0-1, so both
  // the 16-row ds_read_b128 operand reads and the 4-row x 64-B transposed reads of a 32-lane half
  // cover all 64 banks once (a plain (row & 15) XOR leaves the transposed reads 4-way conflicted).
  __device__ static __forceinline__ int swz(int row) {
    if constexpr (sizeof(ET) == 2 && NCH >= 16) return ((row & 3) << 2) | ((row >> 2) & 3);
    else return row & SWM;
  }
};

// LDS-DMA issued through inline asm: hipcc treats a builtin global_load_lds as a pending write
// to ALL of LDS and waits vmcnt(0) before the next transposed LDS read, which would drain the
// next stage's prefetch right after issuing it.  The asm form is invisible to that pass; the
// kernels drain it themselves with one explicit vmcnt(0) in front of the stage barrier (the
// compiler's own counted waits stay correct: extra older VMEM ops only make them wait longer).
__device__ __forceinline__ void glds_dwordx4(const void* gsrc, unsigned lds_base) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc), "s"(lds_base)
               : "memory");  // m0 is reserved (no live compiler value: no other LDS-DMA here)
}
__device__ __forceinline__ void glds_dword(const void* gsrc, unsigned lds_base) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(gsrc), "s"(lds_base)
               : "memory");  // m0 is reserved (no live compiler value: no other LDS-DMA here)
}
// saddr forms: wave-uniform 64-bit base in SGPRs + a 32-bit per-lane byte offset (no per-lane
// 64-bit address arithmetic per load).
__device__ __forceinline__ void glds_dwordx4_s(unsigned voff, const void* sbase, unsigned lds_base) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(lds_base)
               : "memory");
}
__device__ __forceinline__ void glds_dword_s(unsigned voff, const void* sbase, unsigned lds_base) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %0, %1" ::"v"(voff), "s"(sbase), "s"(lds_base)
               : "memory");
}
__device__ __forceinline__ void drain_dma() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// max_j |d_j| from the per-block maxima (every lane of the calling wave gets it).
// n <= kMaxPrepBlocks: the loads are unrolled and predicated, so all of them are in flight at once
// (a runtime-bounded loop waited one L2 round trip per 64 values: 8 in a row at 512 parts).  A
// kernel that needs dmax late issues the loads early (load_dmax) and folds them where it is used.
struct DmaxParts {
  float v[kMaxPrepBlocks / kWave];
};
__device__ __forceinline__ DmaxParts load_dmax(const float* __restrict__ part, int n) {
  DmaxParts d;
#pragma unroll
  for (int k = 0; k < kMaxPrepBlocks / kWave; ++k) {
    const int i = lane_id() + k * kWave;
    const float x = part[i < n ? i : 0];  // unconditional (clamped) load: no branch, no wait per load
    d.v[k] = i < n ? x : 0.f;
  }
  return d;
}
__device__ __forceinline__ float fold_loaded(const DmaxParts& d) {
  float m = 0.f;
#pragma unroll
  for (int k = 0; k < kMaxPrepBlocks / kWave; ++k) m = fmaxf(m, d.v[k]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  return m;
}
__device__ __forceinline__ float fold_dmax(const float* __restrict__ part, int n) {
  return fold_loaded(load_dmax(part, n));
}

// Column shift for the forward: an upper bound of row i's logits in log2 units,
// |q~_i . d~_j| * c2 <= c2 * |q_i| * max_j |d_j| * (1 + 2^-6) (bf16 rounding slack included),
// rounded up to an integer: two launches whose bounds differ (the data-parallel forward's local
// and remote candidates) then form the same bf16 G up to an exact power of two, so rescaling the
// local partials changes no product.  Computed where it is used (engine and combine) from the
// same floats, so both agree exactly.
__device__ __forceinline__ float col_shift(float c2, float qn, float dmax) {
  return ceilf(fabsf(c2) * qn * dmax * 1.015625f);
}

__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const lds_char_t*)p;  // 32-bit LDS byte address
}

// Fill stage `buf` with rows [r0, r0 + BJ) of R; rows at or past row_end come from the zero pad
// (and, backward, an lse of +inf).
template <typename ET, int H, int MODE>
__device__ __forceinline__ void stage_tile(char* smem, int buf, const ET* __restrict__ R, int64_t r0, int64_t row_end,
                                           const float* __restrict__ lse2_rows, const char* __restrict__ pad) {
  using T = Tile<ET, H>;
  const int lane = lane_id(), wid = threadIdx.x >> 6;
  const unsigned base = lds_addr(smem) + buf * T::STAGE_B;
#pragma unroll
  for (int c = 0; c < T::NI; ++c) {
    const int wbase = (c * NW + wid) * 1024;
    const int p = wbase + lane * 16;
    const int row = p / T::ROWB, slot = (p % T::ROWB) >> 4;
    const int ch = slot ^ T::swz(row);
    const int64_t g = r0 + row;
    const char* src = (g < row_end) ? reinterpret_cast<const char*>(R + g * H) + ch * 16 : pad + ch * 16;
    glds_dwordx4(src, __builtin_amdgcn_readfirstlane(base + wbase));
  }
  if constexpr (MODE == DD) {
    if (wid == 0) {
      const int64_t g = r0 + lane;
      const float* src = (g < row_end) ? lse2_rows + g : reinterpret_cast<const float*>(pad + kPadBytes - 16);
      glds_dword(src, __builtin_amdgcn_readfirstlane(lds_addr(smem) + T::LSE_OFF + buf * 256));
    }
  }
}

// Per-lane source byte offsets of the NI pieces of a stage, relative to the stage's first row:
// the same for every stage, so they are computed once per kernel.
template <typename ET, int H>
struct FillOffs {
  unsigned v[Tile<ET, H>::NI];
};

template <typename ET, int H>
__device__ __forceinline__ FillOffs<ET, H> make_fill_offs() {
  using T = Tile<ET, H>;
  const int lane = lane_id(), wid = threadIdx.x >> 6;
  FillOffs<ET, H> o;
#pragma unroll
  for (int c = 0; c < T::NI; ++c) {
    const int p = (c * NW + wid) * 1024 + lane * 16;
    const int row = p / T::ROWB, slot = (p % T::ROWB) >> 4;
    o.v[c] = (unsigned)(row * T::ROWB + ((slot ^ T::swz(row)) << 4));
  }
  return o;
}

// Stage fill for a stage whose BJ rows all exist: scalar stage base + precomputed lane offsets.
// A stage that reaches past row_end takes stage_tile (per-lane pad redirection).
template <typename ET, int H, int MODE>
__device__ __forceinline__ void stage_fill(char* smem, int buf, const ET* __restrict__ R, int64_t r0, int64_t row_end,
                                           const float* __restrict__ lse2_rows, const char* __restrict__ pad,
                                           const FillOffs<ET, H>& fo) {
  using T = Tile<ET, H>;
  if (r0 + T::BJ > row_end) {
    stage_tile<ET, H, MODE>(smem, buf, R, r0, row_end, lse2_rows, pad);
    return;
  }
  const int lane = lane_id(), wid = threadIdx.x >> 6;
  const unsigned base = lds_addr(smem) + buf * T::STAGE_B;
  const char* src = reinterpret_cast<const char*>(R + r0 * H);
#pragma unroll
  for (int c = 0; c < T::NI; ++c) glds_dwordx4_s(fo.v[c], src, __builtin_amdgcn_readfirstlane(base + (c * NW + wid) * 1024));
  if constexpr (MODE == DD) {
    if (wid == 0)
      glds_dword_s((unsigned)lane * 4, lse2_rows + r0,
                   __builtin_amdgcn_readfirstlane(lds_addr(smem) + T::LSE_OFF + buf * 256));
  }
}

// The scorer's hand-offs (split partials, stored probabilities) written through (common.hpp
// store16_wt): round 6, scorer -4 us in the C3 step (profiles/r06n_wt_stores_ab.txt);
// -DTT_WT_STORES=0: plain stores.
#ifndef TT_WT_STORES
#define TT_WT_STORES 1
#endif
template <typename V16>
__device__ __forceinline__ void store16(void* base, uint32_t byte_off, const V16& v) {
#if TT_WT_STORES
  store16_wt(base, byte_off, v);
#else
  *reinterpret_cast<V16*>(static_cast<char*>(base) + byte_off) = v;
#endif
}
__device__ __forceinline__ void store4(void* base, uint32_t byte_off, float v) {
#if TT_WT_STORES
  store4_wt(base, byte_off, v);
#else
  *reinterpret_cast<float*>(static_cast<char*>(base) + byte_off) = v;
#endif
}

template <int MODE, int H>
__device__ __forceinline__ void write_partials(const f32x16 (&acc)[H / 32], float l_run, int split, int64_t nC,
                                               int64_t my_col, int hh, float* acc_part, float* l_part) {
  if (my_col < nC) {
    float* dst = acc_part + ((int64_t)split * nC + my_col) * H;
#pragma unroll
    for (int ht = 0; ht < H / 32; ++ht)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4)
        *reinterpret_cast<f32x4*>(dst + ht * 32 + 8 * g4 + 4 * hh) =
            f32x4{acc[ht][4 * g4], acc[ht][4 * g4 + 1], acc[ht][4 * g4 + 2], acc[ht][4 * g4 + 3]};
  }
  if constexpr (MODE == FWD) {
    l_run += __shfl_xor(l_run, 32);
    if (my_col < nC && hh == 0) l_part[(int64_t)split * nC + my_col] = l_run;
  }
}

// write_partials through the wave's LDS image (32 columns x H fp32 = 128 H bytes at img; the
// caller has passed a barrier after its last read of the ring): every lane writes its 16-B pieces
// to [column][16-B chunk ^ (column & 15)], then each 1 KiB store instruction takes whole rows of
// acc_part (1024 / 4H rows) instead of 32 rows x 32 B (a store-issue-bound epilogue,
// MI355X_MICROARCH.md 'epilogue store tail').  Same values, same places as write_partials.
template <int MODE, int H>
__device__ __forceinline__ void write_partials_t(const f32x16 (&acc)[H / 32], float l_run, int split, int64_t nC,
                                                 int64_t col0, int r32, int hh, float* acc_part, float* l_part,
                                                 lds_char_t* img) {
  if constexpr (H < 64) {  // (a 128-B row: the direct stores are already whole 128-B pieces)
    write_partials<MODE, H>(acc, l_run, split, nC, col0 + r32, hh, acc_part, l_part);
    return;
  }
  constexpr int NCH = H / 4, RPI = kWave / NCH;  // 16-B chunks per row, rows per store instruction
  static_assert(H < 64 || (NCH >= 16 && NCH <= kWave), "H = 32 .. 256");
#pragma unroll
  for (int ht = 0; ht < H / 32; ++ht)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int ch = 8 * ht + 2 * g4 + hh;
      *(lds_f32x4_t*)(img + r32 * (H * 4) + ((ch ^ (r32 & 15)) << 4)) =
          f32x4{acc[ht][4 * g4], acc[ht][4 * g4 + 1], acc[ht][4 * g4 + 2], acc[ht][4 * g4 + 3]};
    }
  const int lane = lane_id(), rl = lane / NCH, ch = lane % NCH;
  float* const blk = acc_part + ((int64_t)split * nC + col0) * H;  // this wave's 32 rows (wave-uniform)
#pragma unroll
  for (int k = 0; k < 32 / RPI; ++k) {
    const int row = k * RPI + rl;
    const f32x4 v = *(const lds_f32x4_t*)(img + row * (H * 4) + ((ch ^ (row & 15)) << 4));
    if (col0 + row < nC) store16(blk, (uint32_t)((row * H + 4 * ch) * 4), v);
  }
  if constexpr (MODE == FWD) {
    l_run += __shfl_xor(l_run, 32);
    if (col0 + r32 < nC && hh == 0) store4(l_part + (int64_t)split * nC + col0, (uint32_t)(r32 * 4), l_run);
  }
}

// G for one 32x32 X tile: forward 2^(x c2 - shift) (accumulating l), backward 2^(x c2 - lse2_row).
template <int MODE>
__device__ __forceinline__ void map_tile(const f32x16& x, float (&e)[16], float c2, float shift,
                                         const lds_f32x4_t* lse4, int hh, float& l_run) {
  if constexpr (MODE == FWD) {
    float ls = 0.f;
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      e[v] = __builtin_amdgcn_exp2f(x[v] * c2 - shift);
      ls += e[v];
    }
    l_run += ls;
  } else {
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const f32x4 l4 = lse4[2 * g4 + hh];  // lse2 of rows 8*g4 + 4*hh + u
#pragma unroll
      for (int u = 0; u < 4; ++u) e[4 * g4 + u] = __builtin_amdgcn_exp2f(x[4 * g4 + u] * c2 - l4[u]);
    }
  }
}

// ------------------------------------------------------------------------------------------
// bf16 engine (32x32x16 bf16 MFMA).  PRECISE splits G into hi + lo bf16 so the second product
// carries ~16 mantissa bits; otherwise G is rounded once (flash-attention style).
// The schedule: 'Forward unit U(j)' below.

// The softmax map of one 32x32 X tile (16 elements per lane), processed in "slots" of one
// element: an even slot forms the pair's scaled exponent with one v_pk_fma_f32 and takes the
// first exp; the odd slot takes the second exp, adds the pair to the row sum (v_pk_add_f32) and
// packs both to bf16.  Slots 0-7 (G rows 0-15, the B operand of the Acc chain's first half) run
// beside the next tile's S chain, slots 8-15 beside the first half of this tile's Acc chain,
// which needs them only from its second half: the vector work is split between both MFMA runs.
#ifndef TT_FWD_DEFER_PAIR
#define TT_FWD_DEFER_PAIR 1
#endif
constexpr bool kDeferPair = TT_FWD_DEFER_PAIR != 0;
template <int MODE, bool PRECISE>
struct MapState {
  // scalar f32 only: packed f32 VALU beside MFMAs costs +22-26 cycles per instruction
  // (MI355X_MICROARCH.md, 'price of one filler'), so no f32x2 here
  float c2, ls;
  float sub[16];
  float e[16];

  __device__ __forceinline__ void init(float c2_, float shift, const lds_f32x4_t* lse4, int hh) {
    c2 = c2_;
    ls = 0.f;
    if constexpr (MODE == FWD) {
#pragma unroll
      for (int v = 0; v < 16; ++v) sub[v] = shift;
    } else {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const f32x4 l4 = lse4[2 * g4 + hh];  // lse2 of rows 8*g4 + 4*hh + u
#pragma unroll
        for (int u = 0; u < 4; ++u) sub[4 * g4 + u] = l4[u];
      }
    }
  }

  // slot v: element v's exponent and exp; a pair's row-sum add and bf16 pack follow its second
  // exp (TT_FWD_DEFER_PAIR: one slot later, so no dependent VALU sits right behind a transcendental
  // -- that needs a wait state, an s_nop per pair; pairs 6-7 and 14-15 stay immediate: they
  // complete an MFMA operand (G rows 0-15, 16-31) that the next step may read).  The adds keep
  // their order: bit-identical either way.
  __device__ __forceinline__ void pair(int p, bf16x8 (&bh)[2], bf16x8 (&bl)[2]) {
    if constexpr (MODE == FWD) {
      ls += e[p] + e[p + 1];
      asm volatile("" : "+v"(ls));  // keeps the sum in this step (not sunk to the unit's end)
    }
#pragma unroll
    for (int w = p; w <= p + 1; ++w) {
      const __bf16 h = (__bf16)e[w];
      bh[w >> 3][w & 7] = h;
      if constexpr (PRECISE) bl[w >> 3][w & 7] = (__bf16)(e[w] - (float)h);
    }
  }
  __device__ __forceinline__ void slot(int v, const f32x16& xa, bf16x8 (&bh)[2], bf16x8 (&bl)[2]) {
    if (kDeferPair && (v & 1) == 0 && (v & 7) != 0) pair(v - 2, bh, bl);  // before this slot's exp
    const float y = __builtin_fmaf(xa[v], c2, -sub[v]);
    e[v] = __builtin_amdgcn_exp2f(y);
    asm volatile("" : "+v"(e[v]));  // side-effecting use: keeps the exp inside this step
    if ((v & 1) && (!kDeferPair || (v & 7) == 7)) pair(v & ~1, bh, bl);
  }
};

// Per-lane LDS byte offsets of the operand reads, relative to a stage base (computed once per
// kernel).  S chain: chunk (2k + hh) ^ swz(row) of row r32 for k = 0..min(NK,8)-1; k >= 8 adds
// 16 chunks (+256 B) and tile jt adds 32 rows: immediates.  Acc chain: the transposed 4-row
// blocks of rows r0 and r0 + 8 at chunk (4 ht + cbase) ^ swz = 4 (ht ^ (swz >> 2)) + (cbase ^
// (swz & 3)) for ht = 0..3; ht >= 4 (+256 B), the second 16-row half and jt: immediates.
template <int H>
struct LdsOffs {
  using T = Tile<__bf16, H>;
  static constexpr int NS8 = (H / 16) < 8 ? (H / 16) : 8;
  static constexpr int NA4 = (H / 32) < 4 ? (H / 32) : 4;
  unsigned s[NS8];
  unsigned a0[NA4], a1[NA4];
  // the same offsets + 64 KiB: a ds_read's offset field holds 16 bits, so reads of the ring slots
  // at 64 KiB and above take these (lds_at) instead of a v_add_u32 per read address
  unsigned sh[NS8], a0h[NA4], a1h[NA4];
  __device__ __forceinline__ void init(int lane) {
    const int r32 = lane & 31, hh = lane >> 5, x = T::swz(r32);
#pragma unroll
    for (int k = 0; k < NS8; ++k) s[k] = r32 * T::ROWB + (((2 * k + hh) ^ x) << 4);
    const int tg = lane >> 4, ti = lane & 15, tq = ti >> 2, tp = ti & 3;
    const int r0 = 4 * (tg >> 1) + tq;
    const int x0 = T::swz(r0), x1 = T::swz(r0 + 8);
    const int cbase = 2 * (tg & 1) + (tp >> 1), bo = (tp & 1) * 8;
#pragma unroll
    for (int ht = 0; ht < NA4; ++ht) {
      a0[ht] = r0 * T::ROWB + bo + (((4 * ht + cbase) ^ x0) << 4);
      a1[ht] = (r0 + 8) * T::ROWB + bo + (((4 * ht + cbase) ^ x1) << 4);
    }
#pragma unroll
    for (int k = 0; k < NS8; ++k) {
      sh[k] = s[k] + 65536u;
      asm volatile("" : "+v"(sh[k]));  // a register of its own, not rematerialised as an add per read
    }
#pragma unroll
    for (int ht = 0; ht < NA4; ++ht) {
      a0h[ht] = a0[ht] + 65536u;
      a1h[ht] = a1[ht] + 65536u;
      asm volatile("" : "+v"(a0h[ht]), "+v"(a1h[ht]));
    }
  }
};

// LDS address of a read at lane offset vo (vo_hi = vo + 64 KiB) from `tile`, a compile-time
// constant offset from `base` once the stage loop is unrolled over its ring slots: tiles at 64 KiB
// and above go through the +64 KiB offsets, so offset + immediate stays inside the 16-bit field.
__device__ __forceinline__ const lds_char_t* lds_at(const lds_char_t* base, const lds_char_t* tile, unsigned vo,
                                                    unsigned vo_hi) {
  const int off = (int)(tile - base);
  if (off >= 65536) return base + (off - 65536) + vo_hi;
  return tile + vo;
}

// ------------------------------------------------------------------------------------------
// Forward unit U(j) as ONE stream of MFMA steps with a uniform operand prefetch distance kSd:
//   steps [0, NK):        S chain of X tile j+1 (xb = R_{j+1} C^T), one ds_read_b128 operand each,
//                         beside map slots 0-7 of X tile j (xa);
//   steps [NK, NK + NSA): Acc chain of tile j (Acc^T += R_j^T G_j), two ds_read_b64_tr_b16 each,
//                         beside map slots 8-15 and the P stores.
// The operand of step i is read kSd steps ahead, ACROSS the chain boundaries: the Acc chain's first
// operands are read during the last S steps, and the next unit's first S operands (X tile j+2)
// during the last Acc steps, so no chain starts by waiting out a full LDS latency (round 2: 100-
// 180 cycles at each of the four chain starts per stage).  The S chain accumulates into VGPRs by
// inline asm (hipcc puts every MFMA accumulator in AGPRs here, which cost 16 v_accvgpr_read per
// tile before the map could read X); its result is first read kSd + NSA steps later by the map of
// the next unit, far beyond the 8-pass MFMA's wait states.
#ifndef TT_SD
#define TT_SD 4
#endif
template <int H>
constexpr int kSdFor = TT_SD < H / 8 ? TT_SD : H / 8;  // <= NSTEP: never past the next unit
// Where the softmax map of X tile j runs: TT_FWD_MAP_S=1 puts all 16 slots beside the S chain of
// tile j+1 (the Acc chain then carries only its operand reads, the P stores and the fills);
// 0 splits them 8 + 8 between the S chain and the first half of the Acc chain.  Same arithmetic
// in the same order either way.
#ifndef TT_FWD_MAP_S
#define TT_FWD_MAP_S 1
#endif
constexpr bool kMapInS = TT_FWD_MAP_S != 0;

__device__ __forceinline__ void mfma_v_first(f32x16& d, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(d) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_v(f32x16& d, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(d) : "v"(a), "v"(b));
}

template <int H>
struct UnitSrc {
  const lds_char_t* s;  // S chain source: stage tile + 32-row X tile base (bytes)
  const lds_char_t* a;  // Acc chain source: stage tile + 32-row tile base (bytes)
  const lds_char_t* n;  // next unit's S chain source
  const lds_char_t* base;  // LDS byte 0 (lds_at)
};

// Operand i of the step stream that starts at this unit: i in [0, NSTEP) is this unit's, i >= NSTEP
// the next unit's (whose S source is u.n and whose Acc tile is this unit's S tile, u.s).
template <int H>
__device__ __forceinline__ bf16x8 unit_operand(int i, const UnitSrc<H>& u, const LdsOffs<H>& lo) {
  using T = Tile<__bf16, H>;
  constexpr int NK = H / 16, NHT = H / 32, NSA = 2 * NHT, NSTEP = NK + NSA;
  const bool nxt = i >= NSTEP;
  const int w = nxt ? i - NSTEP : i;
#define TT_LO_HI(f, i) lo.f##h[i]
  if (w < NK) {
    const lds_char_t* tb = nxt ? u.n : u.s;
    return *reinterpret_cast<const lds_bf16x8_t*>(lds_at(u.base, tb, lo.s[w & 7], TT_LO_HI(s, w & 7)) +
                                                   (w >= 8 ? 256 : 0));
  }
  const lds_char_t* ta = nxt ? u.s : u.a;
  const int st = w - NK, s2 = st / NHT, ht = st % NHT;
  const int imm = s2 * 16 * T::ROWB + (ht >= 4 ? 256 : 0);
  const bf16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
      (lds_bf16x4_t*)(lds_at(u.base, ta, lo.a0[ht & 3], TT_LO_HI(a0, ht & 3)) + imm));
  const bf16x4 t2 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
      (lds_bf16x4_t*)(lds_at(u.base, ta, lo.a1[ht & 3], TT_LO_HI(a1, ht & 3)) + imm));
#undef TT_LO_HI
  return bf16x8{t1[0], t1[1], t1[2], t1[3], t2[0], t2[1], t2[2], t2[3]};
}

// One unit.  ring[] holds the operands of steps 0..kSd-1 on entry and of the next unit's steps
// 0..kSd-1 on exit.  hook(step) places fills and P stores.
template <int MODE, bool PRECISE, int H, class Hook>
__device__ __forceinline__ void fwd_unit(const UnitSrc<H>& u, const LdsOffs<H>& lo, const bf16x8 (&cf)[H / 16],
                                         const f32x16& xa, f32x16& xb, MapState<MODE, PRECISE>& ms,
                                         bf16x8 (&ring)[kSdFor<H>], f32x16 (&acc)[H / 32], float& l_run, Hook hook) {
  constexpr int NK = H / 16, NHT = H / 32, NSA = 2 * NHT, NSTEP = NK + NSA;
  constexpr int kSd = kSdFor<H>;
  static_assert(kSd <= NSTEP, "the prefetch may not reach past the next unit (stage barrier)");
  bf16x8 bh[2], bl[2];
  // The map's first read of xa follows the previous unit's last S MFMA by that unit's NSA Acc
  // steps.  A VALU read of an 8-pass XDL result needs 12 wait states, and hipcc does not count the
  // asm MFMAs: at H <= 64 (NSA <= 4, fewer than 12 instructions in between) pad them here.
  if constexpr (NSA <= 4) asm volatile("s_nop 7\n\ts_nop 4" ::: "memory");
#pragma unroll
  for (int i = 0; i < NSTEP; ++i) {
    const bf16x8 op = ring[i % kSd];
    if (i < NK) {
      if (i == 0) mfma_v_first(xb, op, cf[0]);
      else mfma_v(xb, op, cf[i]);
    } else {
      const int st = i - NK, s2 = st / NHT, ht = st % NHT;
      acc[ht] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(op, bh[s2], acc[ht], 0, 0, 0);
      if constexpr (PRECISE) acc[ht] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(op, bl[s2], acc[ht], 0, 0, 0);
    }
    ring[i % kSd] = unit_operand<H>(i + kSd, u, lo);
    if (kMapInS && i < NK) {  // all 16 map slots beside the S chain (one exp per MFMA gap at H = 256)
#pragma unroll
      for (int v = 16 * i / NK; v < 16 * (i + 1) / NK; ++v) ms.slot(v, xa, bh, bl);
    } else if (i < NK) {
#pragma unroll
      for (int v = 8 * i / NK; v < 8 * (i + 1) / NK; ++v) ms.slot(v, xa, bh, bl);
    } else if (!kMapInS && i - NK < NHT) {  // map slots 8-15 (G rows 16-31, first used at Acc step NHT)
      const int st = i - NK;
#pragma unroll
      for (int v = 8 + 8 * st / NHT; v < 8 + 8 * (st + 1) / NHT; ++v) ms.slot(v, xa, bh, bl);
    }
    hook(i, bh);
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (MODE == FWD) l_run += ms.ls;
}

#ifdef TT_SCORER_TRACE  // debug builds only (tools/trace_scorer.py): s_memtime at region boundaries
__device__ long long g_tt_trace[8 * 64];
#define TT_TRACE(slot)                                                                               \
  do {                                                                                               \
    if (blockIdx.x == 0 && threadIdx.x == 0 && t < 64) g_tt_trace[t * 8 + (slot)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
__device__ long long g_tt_trace_b[8 * 64];
__device__ long long g_tt_ktrace[2 * 1024 * 4];  // [bwd, fwd] per workgroup (wave 0): s_memrealtime at entry, loop start, loop end, exit
#define TT_KTRACE(slot) TT_KTRACE_K(0, slot)
#define TT_KTRACE_K(k, slot)                                                                        \
  do {                                                                                              \
    if (threadIdx.x == 0 && blockIdx.x < 1024) g_tt_ktrace[(k) * 4096 + blockIdx.x * 4 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define TT_TRACE_B(slot)                                                                             \
  do {                                                                                               \
    if (blockIdx.x == 0 && threadIdx.x == 0 && t < 64) g_tt_trace_b[t * 8 + (slot)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define TT_TRACE(slot) \
  do {                 \
  } while (0)
#define TT_TRACE_B(slot) \
  do {                   \
  } while (0)
#define TT_KTRACE(slot) \
  do {                  \
  } while (0)
#define TT_KTRACE_K(k, slot) \
  do {                       \
  } while (0)
#endif

// Stored probabilities (forward, bf16 engine): the backward can take G from the forward instead of
// recomputing S = R C^T.  P is a grid of 2 KiB blocks, block (ct, qt) = candidates [32 ct, +32) x
// queries [32 qt, +32), at byte ((ct * nqt) + qt) * 2048.  Inside a block, byte
//   1024 s2 + 32 c + 16 hh + 2 j   holds   G[candidate c][query 16 s2 + 8 (j >> 2) + 4 hh + (j & 3)]
// for j = 0..7: the 16-byte fragment the backward's lane (c, hh) takes as its B operand of k-step
// s2 (the queries in the A operand's k order), so one backward load and one forward store are each
// a contiguous 1 KiB per wave-instruction.  The values are this wave's bf16 G = 2^(x c2 - shift_q);
// the backward folds 2^(shift_q - lse2_q) into its query rows.
// In the forward a lane holds one query and 16 candidates (registers 4g .. 4g+3 of the tile are
// candidates 8g + 4hh + 0..3), so the tile is transposed through a 2 KiB per-wave LDS image
// [query][candidate] with 64-B rows (cdna_hip_programming.md §3, 'An accumulator tile as the next
// MFMA's operand'): four ds_write_b64 per lane, read back with four ds_read_b64_tr_b16 (lane i of
// a 16-lane group receives candidate i of four query rows), then two 16-B stores per lane.  The
// image's 8-byte slots are XOR-swizzled by (row >> 1) & 7 so both the writes (16 contiguous lanes,
// 32 banks) and the transposed reads (32-lane halves, 64 banks) are conflict-free.  Round 3 did the
// transpose in registers (a DPP move and a v_perm per register, eight 4-byte stores per tile).
struct PStore {
  unsigned w[4];  // LDS byte offsets of this lane's four 8-byte writes (register groups g = 0..3)
  unsigned r[2];  // LDS byte offsets of its transposed reads (query rows +0 / +8); s2 adds 1024 B
  unsigned g;     // byte offset of its 16-B fragment in a P block (s2 adds 1024 B)
  __device__ __forceinline__ void init(unsigned img, int lane) {
    const int r32 = lane & 31, hh = lane >> 5;
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = img + r32 * 64 + 8 * ((2 * k + hh) ^ ((r32 >> 1) & 7));
    const int i = lane & 15, g16 = lane >> 4, slot = 4 * (g16 & 1) + (i & 3);
#pragma unroll
    for (int j2 = 0; j2 < 2; ++j2) {
      const int q = 8 * j2 + 4 * (g16 >> 1) + (i >> 2);  // (+16 s2 leaves (q >> 1) & 7 unchanged)
      r[j2] = img + q * 64 + 8 * (slot ^ ((q >> 1) & 7));
    }
    this->g = (unsigned)(r32 * 32 + hh * 16);
  }
};

// Acc-chain step `st` of a unit's P transpose (NSA steps per unit; bh[1] is complete from step
// `w1`): the writes, the transposed reads two steps later, the stores once the reads have had a
// few MFMAs to return.  Two stores per tile (kPStores): the stage's vmcnt waits count them.
constexpr int kPStores = 2;
template <int NSA>
__device__ __forceinline__ void p_transpose_step(int st, int w1, const PStore& ps, const lds_char_t* lds, char* blk,
                                                 const bf16x8 (&bh)[2], bf16x4 (&pt)[2][2]) {
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  typedef __attribute__((address_space(3))) u32x2 lds_u32x2_t;
  auto at = [&](int step) { return step < NSA ? step : NSA - 1; };
  lds_char_t* img = (lds_char_t*)lds;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (st == at(k < 2 ? 0 : w1)) {
      const bf16x4 v = bf16x4{bh[k >> 1][4 * (k & 1)], bh[k >> 1][4 * (k & 1) + 1], bh[k >> 1][4 * (k & 1) + 2],
                              bh[k >> 1][4 * (k & 1) + 3]};
      *reinterpret_cast<lds_u32x2_t*>(img + ps.w[k]) = __builtin_bit_cast(u32x2, v);
    }
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
    if (st == at(w1 + 1 + s2))
#pragma unroll
      for (int j2 = 0; j2 < 2; ++j2)
        pt[s2][j2] = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(lds + ps.r[j2] + 1024 * s2));
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
    if (st == at(w1 + 5 + 2 * s2)) {
      const bf16x8 v = bf16x8{pt[s2][0][0], pt[s2][0][1], pt[s2][0][2], pt[s2][0][3],
                              pt[s2][1][0], pt[s2][1][1], pt[s2][1][2], pt[s2][1][3]};
      // not non-temporal: the backward, right after, finds part of P still in the Infinity Cache
      // (measured: nt stores and loads cost the backward 10 us at C3); write-through (sc1) keeps that
      store16(blk, (uint32_t)(ps.g + 1024 * s2), v);
    }
}

__device__ __forceinline__ f32x4 load4(const float* p, int lane) { return reinterpret_cast<const f32x4*>(p)[lane]; }
__device__ __forceinline__ f32x4 load4(const __bf16* p, int lane) {
  const bf16x4 v = reinterpret_cast<const bf16x4*>(p)[lane];
  return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}
// V consecutive elements per lane (rows of H = 64 V): the combines' row bodies
template <int V>
struct RowVec {
  typedef float f __attribute__((ext_vector_type(V)));
  typedef __bf16 b __attribute__((ext_vector_type(V)));
};
template <int V>
__device__ __forceinline__ typename RowVec<V>::f loadv(const float* p, int lane) {
  return reinterpret_cast<const typename RowVec<V>::f*>(p)[lane];
}
template <int V>
__device__ __forceinline__ typename RowVec<V>::f loadv(const __bf16* p, int lane) {
  const typename RowVec<V>::b v = reinterpret_cast<const typename RowVec<V>::b*>(p)[lane];
  typename RowVec<V>::f o;
#pragma unroll
  for (int u = 0; u < V; ++u) o[u] = (float)v[u];
  return o;
}
// sum over s < S of p[s * stride4], in split order (the same order as the generic path), with up
// to eight splits' loads in flight (round 3: four; C2's forward has S = 8)
// sum over s < S of w_s p[s * stride] (w_s = f_loc for s < S_loc, else 1: the product is skipped,
// x * 1 == x), added in the order s = 0, 1, ... as the plain loop does (the same bits), with up to
// eight loads in flight instead of one dependent round trip per split.
// (one load per step, the loop before round 3's end: C2 0.4299 vs 0.4273 ms/step batched, same
// box, profiles/r03zp_c2_combine_ab.txt)
__device__ __forceinline__ float sum_parts1(const float* __restrict__ p, int64_t stride, int S, int S_loc = 0,
                                            float f_loc = 1.f) {
  float o = 0.f;
  for (int s0 = 0; s0 < S; s0 += 8) {  // up to 8 splits' loads in one round (S <= 8 by plan_for)
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = s0 + u < S ? p[(int64_t)(s0 + u) * stride] : 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (s0 + u < S) o += s0 + u < S_loc ? f_loc * v[u] : v[u];
  }
  return o;
}

template <typename VT>
__device__ __forceinline__ VT sum_parts4(const VT* __restrict__ p, int64_t stride4, int S) {
  VT o = VT{};
  for (int s0 = 0; s0 < S; s0 += 8) {  // up to 8 splits' loads in one round
    VT v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = s0 + u < S ? p[(int64_t)(s0 + u) * stride4] : VT{};
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (s0 + u < S) o += v[u];
  }
  return o;
}

// Exact row of the loss for a query whose shift bound overshot (l < 2^-100 would lose the row):
// two passes over all M candidates with the true row max, as F.cross_entropy does
// (twotower/losses.py:116).  One wave, fp32 dot products of the same operands the engine scores;
// lane owns elements h = lane + 64 u.  Returns the row max m2 (log2 units), l = sum 2^(x c2 - m2)
// and o = sum 2^(x c2 - m2) d~_j (the lane's elements).  A correctness net for pathological inputs
// (small tau with large or weakly aligned rows): M dot products per row, far slower than the
// engine, and never taken when the bound is within 100 log2 units of the row max.
template <typename DT>
__device__ float exact_row_dot(const DT* __restrict__ qr, const DT* __restrict__ dj, int H, int lane) {
  float acc = 0.f;
  for (int h = lane; h < H; h += kWave) acc += (float)qr[h] * (float)dj[h];
  return wave_sum(acc);
}

template <typename DT>
__device__ void exact_row(const DT* __restrict__ qr, const DT* __restrict__ Dm, int64_t M, int H, float c2, int lane,
                          float& m2, float& l, float (&o)[4]) {
  m2 = -INFINITY;
  for (int64_t j = 0; j < M; ++j) m2 = fmaxf(m2, exact_row_dot(qr, Dm + j * H, H, lane) * c2);
  l = 0.f;
#pragma unroll
  for (int u = 0; u < 4; ++u) o[u] = 0.f;
  for (int64_t j = 0; j < M; ++j) {
    const DT* dj = Dm + j * H;
    const float p = __builtin_amdgcn_exp2f(exact_row_dot(qr, dj, H, lane) * c2 - m2);
    l += p;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (lane + kWave * u < H) o[u] += p * (float)dj[lane + kWave * u];
  }
}

// fwd_combine's row body at H = 64 V (V consecutive floats per lane: every load of the row in
// one round): l = the split-summed row sum of query row i (before the pad correction), get_o() =
// this lane's V floats of O_i = sum_s Acc_s,i.  Writes lse, lse2, dqu and qs / qsp (and xrows for
// a row redone exactly); returns loss_i on every lane.  The fma chains are spelled out so no
// contraction choice changes a bit.
template <int V>
__device__ __forceinline__ float dotv(const typename RowVec<V>::f& a, const typename RowVec<V>::f& b) {
  float d = a[0] * b[0];
#pragma unroll
  for (int u = 1; u < V; ++u) d = __builtin_fmaf(a[u], b[u], d);
  return d;
}

template <typename DT, int V, class GetO>
__device__ __forceinline__ float combine_rowv(int64_t i, float l, GetO get_o, float sh, int n_pad, int64_t M,
                                                float c2, float inv_tau, int64_t label_off,
                                                const DT* __restrict__ Qmat, const DT* __restrict__ Dmat,
                                                float* __restrict__ lse, float* __restrict__ lse2,
                                                float* __restrict__ dqu, DT* __restrict__ qs,
                                                int* __restrict__ xrows, int lane, __bf16* __restrict__ qsp = nullptr,
                                                int64_t qsp_plane = 0) {
  constexpr int H = V * kWave;
  using FV = typename RowVec<V>::f;
  using BV = typename RowVec<V>::b;
  const DT* qr = Qmat + i * H;
  const DT* dl = Dmat + (i + label_off) * H;
  // every load of the row issued here, before l is needed (round 6): one memory round trip per row
  // instead of three (l, then q / d, then the split partials); the exact path below ignores them
  const FV qv = loadv<V>(qr, lane), dv = loadv<V>(dl, lane);
  const FV o = dqu ? get_o() : FV{};
  l = __builtin_fmaf(-(float)n_pad, __builtin_amdgcn_exp2f(-sh), l);  // pad rows: X = 0 exactly
  if (!(l >= 7.888609052210118e-31f)) {  // l < 2^-100 (or NaN): the bound overshot, redo the row exactly
    float m2, lx, o[4];
    exact_row(qr, Dmat, M, H, c2, lane, m2, lx, o);
    const float lse2_i = m2 + log2f(lx);
    const float dot = exact_row_dot(qr, dl, H, lane);
    if (lane == 0) {
      lse[i] = lse2_i * kLn2;
      lse2[i] = lse2_i;
    }
    const float inv_l = 1.f / lx;
#pragma unroll
    for (int u = 0; u < V; ++u) {  // (exact_row's layout: element lane + 64 u)
      const int h = lane + kWave * u;
      if (dqu) dqu[i * H + h] = o[u] * inv_l - (float)dl[h];
      if (qs) qs[i * H + h] = (DT)0.f;  // its stored P underflowed: the backward combine adds the row
      if (qsp)
        for (int pl = 0; pl < 3; ++pl) qsp[pl * qsp_plane + i * H + h] = (__bf16)0.f;
    }
    if ((qs || qsp) && xrows && lane == 0) {  // flagged for the backward combine (adds flagged rows in row order)
      xrows[1 + i] = 1;
      atomicAdd(xrows, 1);
    }
    return __builtin_fmaf(-dot, inv_tau, lse2_i * kLn2);
  }
  const float lse2_i = sh + log2f(l);  // log2 units, for the backward engine
  const float lse_i = lse2_i * kLn2;
  const float dot = wave_sum(dotv<V>(qv, dv));
  if (qs) {  // q~ 2^(shift - lse2): the backward's G = P_stored * that factor, folded into q~
    const float f = __builtin_amdgcn_exp2f(sh - lse2_i);
    if constexpr (std::is_same_v<DT, float>) {
      reinterpret_cast<FV*>(qs + i * H)[lane] = qv * f;
    } else {
      BV o;
#pragma unroll
      for (int u = 0; u < V; ++u) o[u] = (__bf16)(qv[u] * f);
      reinterpret_cast<BV*>(qs + i * H)[lane] = o;
    }
  }
  if (qsp) {  // the split-bf16 backward's planes of the same fp32 products
    const float f = __builtin_amdgcn_exp2f(sh - lse2_i);
    BV pl[3];
#pragma unroll
    for (int u = 0; u < V; ++u) { __bf16 a0, a1, a2; split3(qv[u] * f, a0, a1, a2); pl[0][u] = a0; pl[1][u] = a1; pl[2][u] = a2; }
#pragma unroll
    for (int k = 0; k < 3; ++k) reinterpret_cast<BV*>(qsp + k * qsp_plane + i * H)[lane] = pl[k];
  }
  if (lane == 0) {
    lse[i] = lse_i;
    lse2[i] = lse2_i;
  }
  if (dqu) {
    const float inv_l = 1.f / l;
    FV r;
#pragma unroll
    for (int u = 0; u < V; ++u) r[u] = __builtin_fmaf(o[u], inv_l, -dv[u]);
    reinterpret_cast<FV*>(dqu + i * H)[lane] = r;
  }
  return __builtin_fmaf(-dot, inv_tau, lse_i);
}

template <int MODE, bool PRECISE, int H, bool STOREP = false>
__global__ __launch_bounds__(NT, (H <= 128 ? 2 : 1)) void score_bf16_kernel(
    const __bf16* __restrict__ R, int64_t nR, const __bf16* __restrict__ C, int64_t nC, int S,
    int64_t rows_per_split, float c2, const float* __restrict__ lse2_rows, const float* __restrict__ qnorm,
    const float* __restrict__ dmax_part, int n_dmax,
    const char* __restrict__ pad, float* __restrict__ acc_part, float* __restrict__ l_part,
    char* __restrict__ pstore = nullptr, int64_t p_nqt = 0, int64_t skip_begin = 0, int64_t skip_len = 0,
    int split_base = 0, float* __restrict__ dmax_out = nullptr) {
  // skip_begin / skip_len: the streamed rows are R's rows with [skip_begin, skip_begin + skip_len)
  // left out (a data-parallel rank's remote candidates around its own block; stages never straddle
  // the gap: skip_begin % BJ == 0); split_base: the slot of split 0 in the partial buffers.
  static_assert(!STOREP || (MODE == FWD && !PRECISE), "stored probabilities: forward, single-rounded G");
  using T = Tile<__bf16, H>;
  constexpr int NK = H / 16;
  constexpr int NHT = H / 32;
  constexpr int NJ = T::BJ / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const lds_char_t* lds = (const lds_char_t*)smem;  // addrspacecast: 32-bit LDS offsets from here on

  const int lane = lane_id(), wid = threadIdx.x >> 6;
  const int r32 = lane & 31, hh = lane >> 5;
  const int split = blockIdx.x % S;
  const int64_t cb = blockIdx.x / S;
  const int64_t my_col = cb * (32 * NW) + wid * 32 + r32;
  const int64_t row_begin = (int64_t)split * rows_per_split;
  const int64_t row_end = min(nR, row_begin + rows_per_split);
  const int64_t ntiles = row_end > row_begin ? (row_end - row_begin + T::BJ - 1) / T::BJ : 0;
  if (MODE == FWD) TT_KTRACE_K(1, 0);
  const float dmax = MODE == FWD ? fold_dmax(dmax_part, n_dmax) : 0.f;  // wave-uniform call
  const float shift = (MODE == FWD && my_col < nC) ? col_shift(c2, qnorm[my_col], dmax) : 0.f;
  // the folded bound for the combine (one float instead of every row's wave folding the block maxima)
  if (dmax_out && blockIdx.x == 0 && threadIdx.x == 0) *dmax_out = dmax;

  // Four-stage LDS ring.  After the barrier of stage t (which proves every wave is done with
  // stage t-1's buffer) the fill of stage t+3 goes into that buffer, one 1 KiB piece at a time
  // spread over the remaining MFMA steps of stage t (a burst of 8 pieces per wave stalled the
  // issuing wave ~600 cycles per stage on the address/TA queue).  Each fill then has more than
  // a stage to land.  The R operand (ws bf16 copy) carries a BJ-row zero tail (lse2: +inf), so
  // every fill is a full stage from one scalar base: no per-lane pad redirection, no branches;
  // fills past the last stage reload stage 0's rows into a buffer nobody reads again.
  static_assert(T::NSTAGE == 4, "ring indexing assumes four stages");
  constexpr int NPC = T::NI + (MODE == DD ? 1 : 0);  // pieces per stage per wave (DD: + lse row)
  const FillOffs<__bf16, H> fo = make_fill_offs<__bf16, H>();
  LdsOffs<H> lo;
  lo.init(lane);
  // stored probabilities: this wave's query tile qt, candidate tile of (stage t, tile jt)
  const int64_t p_qt = cb * NW + wid;
  PStore ps;  // its per-wave transpose image follows the ring and the lse rows
  if constexpr (STOREP) ps.init(T::LDS_BYTES + wid * 2048, lane);
  auto pblk = [&](int64_t t, int jt) {
    const int64_t ct = (row_begin + t * T::BJ) / 32 + jt;
    return pstore + (ct * p_nqt + p_qt) * 2048;
  };
  (void)pblk;
  (void)ps;
  const unsigned lds0 = __builtin_amdgcn_readfirstlane(lds_addr(smem));
  const unsigned wbase = __builtin_amdgcn_readfirstlane(lds_addr(smem) + wid * 1024);  // scalar per wave
  auto piece = [&](int c, int b, int64_t r0) {  // piece c of the stage at row r0 into buffer b
    if (c < T::NI) {
      glds_dwordx4_s(fo.v[c], R + r0 * H, wbase + b * T::STAGE_B + c * NW * 1024);
    } else if constexpr (MODE == DD) {  // every wave loads the lse row (same bytes): uniform vmcnt
      glds_dword_s((unsigned)lane * 4, lse2_rows + r0, lds0 + T::LSE_OFF + b * 256);
    }
  };
  auto stage_row = [&](int64_t t) {
    const int64_t r = t < ntiles ? row_begin + t * T::BJ : row_begin;
    return r >= skip_begin ? r + skip_len : r;
  };
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int c = 0; c < NPC; ++c) piece(c, k, stage_row(k));

  bf16x8 cf[NK];
  {
    const bool ok = my_col < nC;
    const bf16x8* src = reinterpret_cast<const bf16x8*>(C + (ok ? my_col : 0) * H);
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) {
      bf16x8 v = src[2 * kk + hh];
      if (!ok) v = bf16x8{};
      cf[kk] = v;
    }
  }
  f32x16 acc[NHT];
#pragma unroll
  for (int t = 0; t < NHT; ++t) acc[t] = f32x16{};
  float l_run = 0.f;
  // stage 0 landed (stages 1 and 2 may still be in flight)
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NPC) : "memory");
  __syncthreads();

  // Stage t = units U(2t) (jt 0) and U(2t+1) (jt 1); each unit's S chain scores the NEXT 32-row
  // X tile, so jt 1's reads tile 0 of stage t+1.  One barrier per stage, at the start of U(2t):
  // after it stage t+1 is visible (the fills of this wave landed: vmcnt; in every wave: barrier),
  // and every wave is past stage t-1, whose buffer then takes the fills of stage t+3, spread over
  // both units.  The next unit's first operands are read ahead across that barrier only from
  // buffers it already covers (tile 1 of stage t, read at the end of U(2t-1)).
  static_assert(NJ % 2 == 0, "X tiles alternate between two register sets");
  f32x16 xa, xb;
  {  // X tile 0 (its operand reads exposed once), into VGPRs like every later X tile
    const UnitSrc<H> u0{lds, lds, lds, lds};
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const bf16x8 a = unit_operand<H>(k, u0, lo);
      // cf was just formed by VALU (v_cndmask): a VALU write -> MFMA operand read needs 2 wait
      // states, which hipcc does not insert ahead of an asm statement
      asm volatile("s_nop 1" ::"v"(cf[k]), "v"(a));
      if (k == 0) mfma_v_first(xa, a, cf[0]);
      else mfma_v(xa, a, cf[k]);
    }
    // the first unit's map reads xa within a few instructions: 12+ wait states after the last
    // asm MFMA (8-pass XDL write -> VALU read; hipcc pads nothing for an asm statement)
    asm volatile("s_nop 7\n\ts_nop 7" : "+v"(xa));
  }
  bf16x8 ring[kSdFor<H>];
  {
    UnitSrc<H> u0{lds + 32 * T::ROWB, lds, lds, lds};  // the first unit's S source: tile 1 of stage 0
#pragma unroll
    for (int k = 0; k < kSdFor<H>; ++k) ring[k] = unit_operand<H>(k, u0, lo);
  }
  constexpr int NSTEP = NK + 2 * NHT;
  if (MODE == FWD) TT_KTRACE_K(1, 1);
  // One stage.  bufc: the ring slot (t & 3) as a compile-time constant when the loop is unrolled
  // over the ring, so every LDS operand address is a per-lane offset plus an
  // immediate (no per-read address add); -1: the slot computed at run time.
  auto stage = [&](int64_t t, auto bufc) {
    constexpr int bc = decltype(bufc)::value;
    const int buf = bc >= 0 ? bc : (int)(t & 3), nbuf = (buf + 1) & 3, fbuf = (buf + 3) & 3;
    const int64_t frow = stage_row(t + 3);
    const lds_char_t* tile = lds + buf * T::STAGE_B;
    const lds_char_t* ntl = lds + nbuf * T::STAGE_B;
    const lds_f32x4_t* lse4 = reinterpret_cast<const lds_f32x4_t*>(lds + T::LSE_OFF + buf * 256);
    TT_TRACE(0);
    // every VMEM op of stage t-1 (NPC fills, kPStores P stores per tile) may still be in flight; all older
    // ones, among them the fills of stage t+1 (issued during stage t-2), have landed
    if (t == 0)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPC) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPC + (STOREP ? kPStores * NJ : 0)) : "memory");
    TT_TRACE(1);
    asm volatile("s_barrier" ::: "memory");
    TT_TRACE(2);
    auto unit = [&](auto jtc, const f32x16& xin, f32x16& xout) {
      constexpr int jt = decltype(jtc)::value;
      auto src = [&](int k) {  // 32-row tile k of stage t (k >= NJ: of stage t+1)
        return k < NJ ? tile + k * 32 * T::ROWB : ntl + (k - NJ) * 32 * T::ROWB;
      };
      const UnitSrc<H> u{src(jt + 1), src(jt), src(jt + 2), lds};
      MapState<MODE, PRECISE> ms;
      ms.init(c2, shift, lse4 + jt * 8, hh);
      char* blk = STOREP ? pblk(t, jt) : nullptr;
      bf16x4 pt[2][2];  // the transposed P fragments between their reads and stores
      auto hook = [&](int i, const bf16x8 (&bh)[2]) {
#pragma unroll
        for (int c = 0; c < NPC; ++c)
          if (c * (NJ * NSTEP) / NPC == jt * NSTEP + i) piece(c, fbuf, frow);
        // bh[1] is complete after the S chain (kMapInS) or after Acc step NHT - 1
        if constexpr (STOREP)
          if (i >= NK) p_transpose_step<2 * NHT>(i - NK, kMapInS ? 1 : NHT, ps, lds, blk, bh, pt);
      };
      fwd_unit<MODE, PRECISE, H>(u, lo, cf, xin, xout, ms, ring, acc, l_run, hook);
      TT_TRACE(3 + jt);
    };
    // the X tiles alternate between xa and xb: no copy between units
    static_assert(NJ == 2, "two units per stage");
    unit(std::integral_constant<int, 0>{}, xa, xb);
    unit(std::integral_constant<int, 1>{}, xb, xa);
  };
  for (int64_t t = 0; t < ntiles; t += 4) {  // wave-uniform conditions: the ring slot of each call is constant
    stage(t, std::integral_constant<int, 0>{});
    if (t + 1 < ntiles) stage(t + 1, std::integral_constant<int, 1>{});
    if (t + 2 < ntiles) stage(t + 2, std::integral_constant<int, 2>{});
    if (t + 3 < ntiles) stage(t + 3, std::integral_constant<int, 3>{});
  }
  if (MODE == FWD) TT_KTRACE_K(1, 2);
  drain_dma();  // no LDS-DMA may outlive the workgroup
  __syncthreads();  // every wave is past its last ring read: the ring takes the partial images
  write_partials_t<MODE, H>(acc, l_run, split + split_base, nC, my_col - r32, r32, hh, acc_part, l_part,
                            (lds_char_t*)smem + wid * 32 * H * 4);
#ifdef TT_SCORER_TRACE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  if (MODE == FWD) TT_KTRACE_K(1, 3);
}

// ------------------------------------------------------------------------------------------
// bf16 backward from stored probabilities (single-rounded G): Acc^T = Qs^T P_tile for every
// 32-row query tile, with Qs = q~ scaled per row by 2^(shift_q - lse2_q) (fwd_combine), so that
// Qs^T P = q~^T G exactly as the recompute engine forms it, minus its S chain and softmax map.
// The Qs tiles stream through the same four-stage LDS ring (stage fills by LDS-DMA, transposed
// A-operand reads); the P fragments (two 16-B loads per lane per tile, one contiguous 1 KiB per
// wave-instruction) go straight to registers three stages ahead.  Both are issued by inline asm
// so the compiler inserts no vmcnt waits of its own: per stage t the order is [P(t+3),
// fills(t+3)], and the barrier that opens stage t+1 waits until at most the P loads and fills of
// stages t+2 and t+3 are in flight, i.e. vmcnt(2 NPC + 8).  Rows past the last query are the
// zero tail of Qs.
template <int s2, int imm_extra = 0>
__device__ __forceinline__ bf16x8 p_load(const char* sbase, unsigned voff) {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  i32x4 r;
  asm volatile("global_load_dwordx4 %0, %1, %2 offset:%3" : "=v"(r) : "v"(voff), "s"(sbase), "n"(1024 * s2 + imm_extra)
               : "memory");
  return __builtin_bit_cast(bf16x8, r);
}

// CW = candidate tiles (of 32) per wave.  CW = 2 (H = 256): every transposed Qs operand read feeds
// two MFMAs and every staged Qs byte twice the MFMAs, which halves the LDS-DMA fill pieces per
// MFMA; the stage's vector-memory instructions (fills + P loads), issued while every wave of the
// CU issues them too, were what bounded this kernel (round 2 trace: a 16-MFMA tile carrying 12
// of them took 1488 cycles, the same tile without them 592).
template <int H, int CW>
__global__ __launch_bounds__(NT, (H <= 128 ? 2 : 1)) void score_ddp_kernel(
    const __bf16* __restrict__ R, int64_t nR, int64_t nC, int S, int64_t rows_per_split, const char* __restrict__ P,
    int64_t p_nqt, float* __restrict__ acc_part) {
  using T = Tile<__bf16, H>;
  constexpr int NHT = H / 32;
  constexpr int NJ = T::BJ / 32;
  static_assert(NJ == 2 && T::NSTAGE == 4, "two 32-row tiles per stage, four-stage ring");
  constexpr int NPC = T::NI;                // fill pieces per stage per wave
  constexpr int NS = 2 * NHT;               // operand steps per 32-row tile (CW MFMAs each)
  constexpr int NSTEP = NJ * NS;            // operand steps per stage
  constexpr int NPL = 2 * NJ * CW;          // P loads per stage per wave
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const lds_char_t* lds = (const lds_char_t*)smem;

  const int lane = lane_id(), wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const int split = blockIdx.x % S;
  const int64_t cb = blockIdx.x / S;
  const int64_t ct0 = (cb * NW + wid) * CW;  // this wave's first 32-candidate tile
  const int64_t row_begin = (int64_t)split * rows_per_split;
  const int64_t row_end = min(nR, row_begin + rows_per_split);
  const int64_t ntiles = row_end > row_begin ? (row_end - row_begin + T::BJ - 1) / T::BJ : 0;

  TT_KTRACE(0);
  const FillOffs<__bf16, H> fo = make_fill_offs<__bf16, H>();
  LdsOffs<H> lo;
  lo.init(lane);
  const unsigned wbase = __builtin_amdgcn_readfirstlane(lds_addr(smem) + wid * 1024);
  auto stage_row = [&](int64_t t) { return t < ntiles ? row_begin + t * T::BJ : row_begin; };
  auto fill = [&](int c, int b, int64_t r0) {
    glds_dwordx4_s(fo.v[c], R + r0 * H, wbase + b * T::STAGE_B + c * NW * 1024);
  };
  // a lane's fragment of a P block: candidate r32, queries 16 s2 + 8 (j >> 2) + 4 hh + (j & 3) (PStore)
  const char* pcol = P + ct0 * p_nqt * 2048;
  const unsigned pvo = (unsigned)(r32 * 32 + hh * 16);
  // P fragments of stages t .. t+3 in five register sets (index t % 5): the loads of stage t+3
  // go into the set stage t-2 read, so no load is in flight into registers an MFMA of the
  // previous stage may still be reading (the asm loads are outside the compiler's hazard checks)
  struct PSet {
    bf16x8 v[NJ][CW][2];
  };
  PSet pf[5];
  auto pload = [&](PSet& dst, int64_t t, int k) {  // P load k (of NPL) of stage t
    const int c = k / (2 * NJ), jt = (k / 2) % NJ;
    const char* b = pcol + (c * p_nqt + stage_row(t) / 32 + jt) * 2048;
    if (k % 2 == 0) dst.v[jt][c][0] = p_load<0>(b, pvo);
    else dst.v[jt][c][1] = p_load<1>(b, pvo);
  };
  auto pissue = [&](PSet& dst, int64_t t) {
#pragma unroll
    for (int k = 0; k < NPL; ++k) pload(dst, t, k);
  };
  auto tie = [&](PSet& x) {
#pragma unroll
    for (int jt = 0; jt < NJ; ++jt)
#pragma unroll
      for (int c = 0; c < CW; ++c)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) asm volatile("" : "+v"(x.v[jt][c][s2]));
  };
  constexpr int kPl = NPL;
  // prologue in steady-state order: [P(k), fills(k)] for k = 0, 1, 2, but only the first half
  // of fills(2): the second half of every stage's fills comes from the first tile of the stage
  // two before it (below)
  constexpr int NPC2 = NPC / 2, NPC1 = NPC - NPC2;  // pieces in the first / second half
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    pissue(pf[k], k);
#pragma unroll
    for (int c = 0; c < (k < 2 ? NPC : NPC1); ++c) fill(c, k, stage_row(k));
  }

  f32x16 acc[CW][NHT];
#pragma unroll
  for (int c = 0; c < CW; ++c)
#pragma unroll
    for (int t = 0; t < NHT; ++t) acc[c][t] = f32x16{};
  // stage 0 and P(0) landed: only P(1), fills(1), P(2) and fills(2)'s first half may be in flight
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPC + NPC1 + 2 * kPl) : "memory");
  __syncthreads();
  tie(pf[0]);

  // One stream of NSTEP operand steps per stage whose A operands (two transposed reads each) are
  // read kDd steps ahead, across the tile boundary and into the next stage: the stage barrier sits
  // in the MIDDLE of stage t (before tile 1) and waits for stage t+1 (its fills and P(t+1)), so
  // the last steps of stage t may read stage t+1's first operands.  After that barrier every wave
  // is past stage t-1, so the first half of fills(t+3) (into stage t-1's buffer) is issued over
  // tile 1 and its second half over tile 0 of stage t+1; P(t+3) is loaded over tile 0 of stage t,
  // after that tile's fill pieces.  The vector-memory instructions are spread over the whole
  // stage: in bursts they cost each wave ~75 cycles apiece (round 2 trace).  At the barrier of stage t the VMEM ops younger than fills(t+1)'s last
  // piece (tile 0 of stage t-1) are P(t+2), fills(t+2) and P(t+3): vmcnt(NPC + 2 NPL).
  constexpr int kDd = kSdFor<H> < NS ? kSdFor<H> : NS;
  auto opnd = [&](const lds_char_t* stile, int i) {  // A operand of step i of the stage at stile
    const int jt = i / NS, st = i % NS, s2 = st / NHT, ht = st % NHT;
    const lds_char_t* tb = stile + jt * 32 * T::ROWB;
    const int imm = s2 * 16 * T::ROWB + (ht >= 4 ? 256 : 0);
    const bf16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(tb + lo.a0[ht & 3] + imm));
    const bf16x4 t2 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(tb + lo.a1[ht & 3] + imm));
    return bf16x8{t1[0], t1[1], t1[2], t1[3], t2[0], t2[1], t2[2], t2[3]};
  };
  bf16x8 ring[kDd];
#pragma unroll
  for (int k = 0; k < kDd; ++k) ring[k] = opnd(lds, k);
  auto stage = [&](int64_t t, PSet& cur, PSet& ahead, PSet& next) {
    const int buf = (int)(t & 3), fbuf = (buf + 3) & 3, hbuf = (buf + 2) & 3;
    const int64_t frow = stage_row(t + 3), hrow = stage_row(t + 2);
    const lds_char_t* tile = lds + buf * T::STAGE_B;
    const lds_char_t* ntile = lds + ((buf + 1) & 3) * T::STAGE_B;
    TT_TRACE_B(0);
#pragma unroll
    for (int i = 0; i < NSTEP; ++i) {
      if (i == NS) {
        TT_TRACE_B(1);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPC + 2 * kPl) : "memory");
        TT_TRACE_B(2);
        asm volatile("s_barrier" ::: "memory");
        TT_TRACE_B(3);
        tie(next);
      }
      const int jt = i / NS, st = i % NS, s2 = st / NHT, ht = st % NHT;
#pragma unroll
      for (int c = 0; c < CW; ++c)
        acc[c][ht] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ring[i % kDd], cur.v[jt][c][s2], acc[c][ht], 0, 0, 0);
      const int j = i + kDd;
      ring[i % kDd] = j < NSTEP ? opnd(tile, j) : opnd(ntile, j - NSTEP);
      // tile 0: the second half of fills(t+2) in its first half, then P(t+3) one load at a time
      constexpr int F0 = NS / 2;
#pragma unroll
      for (int c = 0; c < NPC2; ++c)
        if (c * F0 / (NPC2 > 0 ? NPC2 : 1) == i) fill(NPC1 + c, hbuf, hrow);
#pragma unroll
      for (int k = 0; k < NPL; ++k)
        if (F0 + k * (NS - F0) / NPL == i) pload(ahead, t + 3, k);
#pragma unroll
      for (int c = 0; c < NPC1; ++c)
        if (NS + c * NS / NPC1 == i) fill(c, fbuf, frow);    // tile 1: first half of fills(t+3)
      __builtin_amdgcn_sched_barrier(0);
    }
    TT_TRACE_B(4);
  };
  static_assert(NJ == 2, "the stage barrier sits before tile 1");
  TT_KTRACE(1);
  // Full rounds of five stages, then the remaining 0-4 stages as nested conditionals: no path
  // through the code reaches a stage whose predecessor was skipped, and every register set is
  // named again after the final drain.  The P loads of the last three stages are still in flight
  // when the stages end; a set that were dead on some path (round 1: the sets of stages t+3/t+4
  // when the loop ended after stage t or t+1, leaving through the latch) is free for the compiler
  // to reuse while its load lands.  Round 1 found exactly that: the latch's loop-bound compare was
  // allocated into the in-flight set of stage t+3, so a cold (slow) P load overwrote the bound and
  // the wave ran on past its last tile (wrong dD for that wave's 32 candidates).
  // tools/isa_audit.py checks the emitted ISA for any such use (tests/test_isa_audit.py).
  int64_t t = 0;
  for (; t + 5 <= ntiles; t += 5) {
    stage(t, pf[0], pf[3], pf[1]);
    stage(t + 1, pf[1], pf[4], pf[2]);
    stage(t + 2, pf[2], pf[0], pf[3]);
    stage(t + 3, pf[3], pf[1], pf[4]);
    stage(t + 4, pf[4], pf[2], pf[0]);
  }
  if (t < ntiles) {
    stage(t, pf[0], pf[3], pf[1]);
    if (t + 1 < ntiles) {
      stage(t + 1, pf[1], pf[4], pf[2]);
      if (t + 2 < ntiles) {
        stage(t + 2, pf[2], pf[0], pf[3]);
        if (t + 3 < ntiles) stage(t + 3, pf[3], pf[1], pf[4]);
      }
    }
  }
  TT_KTRACE(2);
  drain_dma();  // no load may outlive the workgroup
#pragma unroll
  for (int k = 0; k < 5; ++k) tie(pf[k]);
  __syncthreads();  // every wave is past its last ring read: the ring takes the partial images
#pragma unroll
  for (int c = 0; c < CW; ++c)
    write_partials_t<DD, H>(acc[c], 0.f, split, nC, (ct0 + c) * 32, r32, hh, acc_part, nullptr,
                            (lds_char_t*)smem + wid * 32 * H * 4);
#ifdef TT_SCORER_TRACE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  TT_KTRACE(3);
}

// ------------------------------------------------------------------------------------------
// fp32 engine (exact f32 MFMA, 32x32x2).  The k order inside the X product is permuted
// (k = 8*blk + 4*hh + u) so each lane reads one 16-byte chunk per four MFMAs; the Acc product
// consumes X register t directly as its B operand (k = row of X held by register t).
// Waves per SIMD the H = 128 fp32 engine is compiled for.  Round 2: two waves spilled 80 B/lane of
// scratch (256 VGPRs), so the forward ran at one (217 VGPRs + 64 AGPRs).  Round 3: the Acc chain's
// LDS addresses come from four per-lane offsets plus immediates (hipcc had held
// 16 x NHT loop-invariant addresses in VGPRs across the loop), so both passes fit two waves with no
// scratch (225 / 221 VGPRs): C2 forward 205 -> 175 us, backward 180 -> 160 us, bit-identical,
// step 0.520 -> 0.469 ms (profiles/r03t_f32_variants.txt, r03t_c2_ab.txt).
#ifndef TT_F32_MINW128_FWD
#define TT_F32_MINW128_FWD 2
#endif
#ifndef TT_F32_MINW128_DD
#define TT_F32_MINW128_DD 2
#endif
// Waves per SIMD of the fp32 backward from stored probabilities (no X chain: fewer registers), by H
#ifndef TT_F32_MINW_LOADP128
#define TT_F32_MINW_LOADP128 2
#endif
#ifndef TT_F32_MINW_LOADP256
#define TT_F32_MINW_LOADP256 1
#endif
#ifndef TT_F32_MINW_LOADP64
#define TT_F32_MINW_LOADP64 2
#endif
__host__ __device__ constexpr int f32_waves(int mode, int H, bool loadp) {
  return loadp ? (H < 128 ? TT_F32_MINW_LOADP64 : H > 128 ? TT_F32_MINW_LOADP256 : TT_F32_MINW_LOADP128)
               : (H < 128 ? 2 : H > 128 ? 1 : mode == FWD ? TT_F32_MINW128_FWD : TT_F32_MINW128_DD);
}
// STOREP (round 3, the fp32 form of the stored-probability backward): the forward also writes each
// 32 x 32 G tile to P, block (candidate tile ct, query tile qt) = 1,024 floats [candidate][query] at
// (ct * p_nqt + qt) * 1024; the backward (MODE DD, R = the scaled query copy Qs) reads its G^T
// tile from there (four 16-B loads per lane: lane (candidate r32, hh) takes queries 8k + 4hh + u)
// instead of forming X = R C^T and its exp: half the backward's MFMAs, no transcendental.
template <int MODE, int H, bool STOREP = false>
__global__ __launch_bounds__(NT, f32_waves(MODE, H, STOREP && MODE == DD))
void score_f32_kernel(
    const float* __restrict__ R, int64_t nR, const float* __restrict__ C, int64_t nC, int S,
    int64_t rows_per_split, float c2, const float* __restrict__ lse2_rows, const float* __restrict__ qnorm,
    const float* __restrict__ dmax_part, int n_dmax,
    const char* __restrict__ pad, float* __restrict__ acc_part, float* __restrict__ l_part,
    float* __restrict__ P = nullptr, int64_t p_nqt = 0) {
  using T = Tile<float, H>;
  constexpr bool LOADP = STOREP && MODE == DD;  // G from P (no X chain, no map)
  constexpr int FILLMODE = LOADP ? FWD : MODE;   // no lse2 row staging when G comes from P
  constexpr int NB = H / 8;
  constexpr int NHT = H / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const lds_char_t* lds = (const lds_char_t*)smem;

  const int lane = lane_id(), wid = threadIdx.x >> 6;
  const int r32 = lane & 31, hh = lane >> 5;
  const int split = blockIdx.x % S;
  const int64_t cb = blockIdx.x / S;
  const int64_t my_col = cb * (32 * NW) + wid * 32 + r32;
  const int64_t row_begin = (int64_t)split * rows_per_split;
  const int64_t row_end = min(nR, row_begin + rows_per_split);
  const int64_t ntiles = row_end > row_begin ? (row_end - row_begin + T::BJ - 1) / T::BJ : 0;
  const float dmax = MODE == FWD ? fold_dmax(dmax_part, n_dmax) : 0.f;  // wave-uniform call
  const float shift = (MODE == FWD && my_col < nC) ? col_shift(c2, qnorm[my_col], dmax) : 0.f;

  const FillOffs<float, H> fo = make_fill_offs<float, H>();
  if (ntiles > 0) stage_fill<float, H, FILLMODE>(smem, 0, R, row_begin, row_end, lse2_rows, pad, fo);
  // LOADP: this lane's G^T row of stored block (ct = my_col / 32, qt), as four float4
  const f32x4* pcol = nullptr;
  f32x4 pn[4];
  if constexpr (LOADP) {
    pcol = reinterpret_cast<const f32x4*>(P + ((my_col >> 5) * p_nqt + (row_begin >> 5)) * 1024 + r32 * 32 + 4 * hh);
    if (ntiles > 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) pn[k] = pcol[2 * k];
    }
  }

  f32x4 cf[NB];
  if constexpr (!LOADP) {
    const bool ok = my_col < nC;
    const f32x4* src = reinterpret_cast<const f32x4*>(C + (ok ? my_col : 0) * H);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      f32x4 v = src[2 * b + hh];
      if (!ok) v = f32x4{};
      cf[b] = v;
    }
  }
  f32x16 acc[NHT];
#pragma unroll
  for (int t = 0; t < NHT; ++t) acc[t] = f32x16{};
  float l_run = 0.f;
  const int rx = T::swz(r32);
  static_assert(T::SWM == 7, "the Acc chain's offsets assume the f32 tile's 3-bit row XOR");
  unsigned aoff[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) aoff[u] = (u + 4 * hh) * T::ROWB + (((r32 >> 2) ^ (u + 4 * hh)) << 4) + (r32 & 3) * 4;
  drain_dma();
  __syncthreads();

  for (int64_t t = 0; t < ntiles; ++t) {
    const int buf = (int)(t & 1);
    if (t + 1 < ntiles)
      stage_fill<float, H, FILLMODE>(smem, buf ^ 1, R, row_begin + (t + 1) * T::BJ, row_end, lse2_rows, pad, fo);
    const lds_char_t* tile = lds + buf * T::STAGE_B;
    float e[16];
    if constexpr (LOADP) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int u = 0; u < 4; ++u) e[4 * k + u] = pn[k][u];
      if (t + 1 < ntiles) {  // the next tile's G, in flight beside this tile's Acc chain
#pragma unroll
        for (int k = 0; k < 4; ++k) pn[k] = pcol[(t + 1) * 256 + 2 * k];
      }
    } else {
      const lds_f32x4_t* lse4 = reinterpret_cast<const lds_f32x4_t*>(lds + T::LSE_OFF + buf * 256);
      f32x16 x = f32x16{};
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const f32x4 a = *reinterpret_cast<const lds_f32x4_t*>(tile + r32 * T::ROWB + (((2 * b + hh) ^ rx) << 4));
#pragma unroll
        for (int u = 0; u < 4; ++u) x = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u], cf[b][u], x, 0, 0, 0);
      }
      map_tile<MODE>(x, e, c2, shift, lse4, hh, l_run);
      if constexpr (STOREP) {  // forward: G of (candidate tile, this wave's query tile) to P
        float* blk = P + (((row_begin >> 5) + t) * p_nqt + (my_col >> 5)) * 1024 + r32;
#pragma unroll
        for (int v = 0; v < 16; ++v) blk[acc_row(v, hh) * 32] = e[v];
      }
    }
#pragma unroll
    for (int ht = 0; ht < NHT; ++ht) {
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        // row = (v & 3) + 8 (v >> 2) + 4 hh and swz(row) = row & 7 = (v & 3) + 4 hh, so the XOR only
        // touches the chunk's low three bits: four per-lane offsets (one per v & 3, kernel-constant)
        // plus immediates, instead of 16 x NHT loop-invariant addresses held across the loop
        const float a = *reinterpret_cast<const lds_float_t*>(tile + aoff[v & 3] + 8 * (v >> 2) * T::ROWB + 128 * ht);
        acc[ht] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, e[v], acc[ht], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    drain_dma();
    __syncthreads();
  }
  write_partials<MODE, H>(acc, l_run, split, nC, my_col, hh, acc_part, l_part);
}

// ------------------------------------------------------------------------------------------
// Split-bf16 engine for fp32 operands (round 4; the fp32 stored-P forward and backward at
// H = 64, 128, 256).  Each fp32 operand is cut into three bf16 terms, x = x0 + x1 + x2 exactly
// (split3, the tower head's scheme), and a product x y is formed from the six cross terms of
// order >= 2^-16 (x0y2, x1y1, x2y0, x0y1, x1y0, x0y0, smallest first) on the 32x32x16 bf16 MFMA
// with fp32 accumulation: six 32-cycle MFMAs do the work of eight 64-cycle 32x32x2 f32 MFMAs,
// 2.7x the fp32 MFMA rate at fp32-product accuracy (the dropped terms are below 2^-24 relative).
//   forward:  X = R C^T from the candidate planes (an LDS ring of 32-row stages, three planes per
//             stage in the bf16 engine's row layout) and the query planes (VGPRs, split at entry
//             from the fp32 rows); G = 2^(X c2 - shift) in fp32 (score_f32_kernel's map), stored
//             to P as fp32 in score_f32_kernel's block layout; then Acc^T += R^T G with G split
//             into three planes (the B operand) and R^T read with ds_read_b64_tr_b16.
//   backward: Acc^T = Qs^T G (= dD^T) from the scaled-query planes (fwd_combine writes them) and G
//             loaded from P (asm loads two units ahead) and split in registers.
// One wave per SIMD (the one-round grids of these shapes hold one workgroup per CU).  Both kernels
// run software-pipelined unit streams (score_split_fwd_kernel, score_split_ddp_kernel): every
// MFMA gap carries one operand piece read kSd steps ahead, and the map / split of the next tile
// sits beside the current tile's MFMAs, pinned there by sched_barrier per MFMA.
template <int H>
struct SplitTile {
  using T = Tile<__bf16, H>;  // a plane's rows: the bf16 engine's layout (ROWB, swizzle, LdsOffs)
  static constexpr int BJ = 32;
  static constexpr int PLANE_B = BJ * T::ROWB;
  static constexpr int STAGE_B = 3 * PLANE_B;
  static constexpr int NPP = PLANE_B / 1024 / NW;  // fill pieces per wave per plane
  static constexpr int NF = 3 * NPP;                // ... per stage
  static constexpr int NSTAGE = 3;  // the backward's ring (the forward's: SplitFwdRing)
  static constexpr int LDS_BYTES = NSTAGE * STAGE_B;
  static_assert(NPP >= 1 && NPP * 1024 * NW == PLANE_B, "a plane tile is a whole number of 1 KiB pieces per wave");
  static_assert(BJ == Tile<float, H>::BJ, "the plan's row tiles (bj_for(TT_F32)) are this engine's stages");
};

__device__ __forceinline__ f32x16 mfma_bf16(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// G planes of a 32x32 tile from its 16 fp32 values per lane: plane p, k-step s2, element j = G row
// 16 s2 + 8 (j >> 2) + 4 hh + (j & 3) (the accumulator order: the B operand of the Acc chain).
__device__ __forceinline__ void split_tile(const float (&e)[16], bf16x8 (&g)[3][2]) {
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    __bf16 a0, a1, a2;
    split3(e[v], a0, a1, a2);
    g[0][v >> 3][v & 7] = a0;
    g[1][v >> 3][v & 7] = a1;
    g[2][v >> 3][v & 7] = a2;
  }
}

// Per-lane source offsets of a plane tile's NPP fill pieces (the swizzle on the source side, as
// make_fill_offs).
template <int H>
__device__ __forceinline__ void split_fill_offs(unsigned (&fo)[SplitTile<H>::NPP]) {
  using T = typename SplitTile<H>::T;
  const int lane = lane_id(), wid = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < SplitTile<H>::NPP; ++c) {
    const int p = (c * NW + wid) * 1024 + lane * 16;
    const int row = p / T::ROWB, slot = (p % T::ROWB) >> 4;
    fo[c] = (unsigned)(row * T::ROWB + ((slot ^ T::swz(row)) << 4));
  }
}

// The forward's LDS ring: four stages where they fit beside nothing else (H <= 128), else three.
template <int H>
struct SplitFwdRing {
  static constexpr int NSLOT = 4 * SplitTile<H>::STAGE_B <= 128 * 1024 ? 4 : 3;
  static constexpr int LDS_BYTES = NSLOT * SplitTile<H>::STAGE_B;
};

// Operand registers of one MFMA step: three planes of a 32x16 fragment, held as 8-byte halves
// (an Acc operand arrives as two ds_read_b64_tr_b16 per plane).
struct SplitOp {
  bf16x4 h[3][2];
  __device__ __forceinline__ bf16x8 a(int p) const {
    return bf16x8{h[p][0][0], h[p][0][1], h[p][0][2], h[p][0][3], h[p][1][0], h[p][1][1], h[p][1][2], h[p][1][3]};
  }
};

// Piece j (0..5) of the Acc chain's operand of step st (G rows 16 s2, h-tile ht): half j & 1 of
// plane j >> 1, one ds_read_b64_tr_b16.
template <int H>
__device__ __forceinline__ void split_acc_piece(SplitOp& o, int st, int j, const lds_char_t* tile, const LdsOffs<H>& lo) {
  using ST = SplitTile<H>;
  using T = typename ST::T;
  constexpr int NHT = H / 32;
  const int s2 = st / NHT, ht = st % NHT, p = j >> 1;
  const lds_char_t* tb = tile + p * ST::PLANE_B + s2 * 16 * T::ROWB + (ht >= 4 ? 256 : 0);
  o.h[p][j & 1] = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(tb + ((j & 1) ? lo.a1[ht & 3] : lo.a0[ht & 3])));
}

// Piece j (0..5) of the operand of step i of a forward unit: steps [0, NK) are the S chain's (plane
// j, one ds_read_b128, j < 3) from s_tile, steps [NK, NSTEP) the Acc chain's (half j & 1 of plane
// j >> 1, one ds_read_b64_tr_b16) from a_tile, steps >= NSTEP the next unit's S steps from n_tile.
template <int H>
__device__ __forceinline__ void split_fwd_piece(SplitOp& o, int i, int j, const lds_char_t* s_tile,
                                                const lds_char_t* a_tile, const lds_char_t* n_tile,
                                                const LdsOffs<H>& lo) {
  using ST = SplitTile<H>;
  constexpr int NK = H / 16, NHT = H / 32, NSTEP = NK + 2 * NHT;
  if (i >= NSTEP) {
    i -= NSTEP;
    s_tile = n_tile;
  }
  if (i < NK) {
    if (j < 3) {
      const bf16x8 v =
          *reinterpret_cast<const lds_bf16x8_t*>(s_tile + j * ST::PLANE_B + lo.s[i & 7] + (i >= 8 ? 256 : 0));
      o.h[j][0] = bf16x4{v[0], v[1], v[2], v[3]};
      o.h[j][1] = bf16x4{v[4], v[5], v[6], v[7]};
    }
  } else {
    split_acc_piece<H>(o, i - NK, j, a_tile, lo);
  }
}

// The six cross terms of a split product, smallest first (x0y2, x1y1, x2y0, x0y1, x1y0, x0y0):
// MFMA j takes plane kPa[j] of the A operand and plane kPb[j] of the B operand.
constexpr int kPa[6] = {0, 1, 2, 0, 1, 0};
constexpr int kPb[6] = {2, 1, 0, 1, 0, 0};

// R: three bf16 planes of nR rows + a kTailRows zero tail each (plane stride `plane` elements), so
// every stage is a full tile from one scalar base.  C: the fp32 query rows.  P: fp32 blocks of
// score_f32_kernel's layout.
//
// Software-pipelined like the bf16 engine's fwd_unit: unit t is one stream of NSTEP MFMA steps
// (six MFMAs each), steps [0, NK) the S chain of tile t+1 (into xb) beside the map
// of tile t (xa: exp, row sum, P store, split of G into three planes, SPS = 16 / NK slots a step,
// spread over the step's six MFMA gaps), steps [NK, NSTEP) the Acc chain of tile t.  Each step's
// operand is read kSd steps ahead in six pieces, one per MFMA, across the chain and unit
// boundaries.  Round 4's first form ran the S chain, the map and the Acc chain back to back
// (0.48 MFMA busy at C2: the map and each chain's first operand reads exposed).
//   Ring (NSLOT stages of 32 rows): unit t reads tiles t, t+1 and, in its last kSd steps, t+2.  At
//   step NSTEP - kSd (the barrier point) fill(t+2) must have landed in every wave: wait, barrier.
//   Four slots: the barrier point also frees tile t-1's slot, which takes fill(t+3) right there,
//   one 1 KiB piece per MFMA gap (six LDS-DMA issues in a row cost ~480 cycles of MFMA idle).
//   Three slots (H = 256): a second barrier at the unit's start frees it for fill(t+2).
//   P stores: unit t's 16 stores come from register set e[t & 1]; the barrier point of unit t+1
//   (its vmcnt wait sees them complete) releases that set to unit t+2.
template <int H>
__global__ __launch_bounds__(NT, 1) void score_split_fwd_kernel(
    const __bf16* __restrict__ R, int64_t plane, int64_t nR, const float* __restrict__ C, int64_t nC, int S,
    int64_t rows_per_split, float c2, const float* __restrict__ qnorm, const float* __restrict__ dmax_part, int n_dmax,
    float* __restrict__ acc_part, float* __restrict__ l_part, float* __restrict__ P, int64_t p_nqt,
    float* __restrict__ dmax_out = nullptr) {
  using ST = SplitTile<H>;
  constexpr int NK = H / 16, NHT = H / 32, NSTEP = NK + 2 * NHT, NF = ST::NF;
  constexpr int NSLOT = SplitFwdRing<H>::NSLOT;
  constexpr int kSd = 2, SPS = 16 / NK;
  static_assert(NSTEP % kSd == 0 && kSd <= 2 * NHT, "the barrier point follows the map's stores");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const lds_char_t* lds = (const lds_char_t*)smem;
  const int lane = lane_id(), wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const int split = blockIdx.x % S;
  const int64_t cb = blockIdx.x / S;
  const int64_t my_col = cb * (32 * NW) + wid * 32 + r32;
  const int64_t row_begin = (int64_t)split * rows_per_split;
  const int64_t row_end = min(nR, row_begin + rows_per_split);
  const int64_t ntiles = row_end > row_begin ? (row_end - row_begin + ST::BJ - 1) / ST::BJ : 0;
  TT_KTRACE_K(1, 0);
  f32x16 acc[NHT];
#pragma unroll
  for (int t = 0; t < NHT; ++t) acc[t] = f32x16{};
  float l_run = 0.f;
  if (ntiles == 0) {  // (workgroup-uniform) no rows: zero partials
    const float dmax = fold_dmax(dmax_part, n_dmax);
    if (dmax_out && blockIdx.x == 0 && threadIdx.x == 0) *dmax_out = dmax;
    write_partials<FWD, H>(acc, l_run, split, nC, my_col, hh, acc_part, l_part);
    return;
  }

  unsigned fo[ST::NPP];
  split_fill_offs<H>(fo);
  const unsigned wbase = __builtin_amdgcn_readfirstlane(lds_addr(smem) + wid * 1024);
  auto fill = [&](int b, int64_t t) {  // stage t into ring slot b (past the last stage: stage 0 again)
    const int64_t r0 = t < ntiles ? row_begin + t * ST::BJ : row_begin;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int c = 0; c < ST::NPP; ++c)
        glds_dwordx4_s(fo[c], R + p * plane + r0 * H, wbase + b * ST::STAGE_B + p * ST::PLANE_B + c * NW * 1024);
  };
  auto fill_piece = [&](int b, int64_t t, int f) {  // piece f (plane f / NPP) of fill(b, t)
    const int64_t r0 = t < ntiles ? row_begin + t * ST::BJ : row_begin;
    const int p = f / ST::NPP, c = f % ST::NPP;
    glds_dwordx4_s(fo[c], R + p * plane + r0 * H, wbase + b * ST::STAGE_B + p * ST::PLANE_B + c * NW * 1024);
  };
  auto slot_tile = [&](int b) { return lds + b * ST::STAGE_B; };
  const DmaxParts dparts = load_dmax(dmax_part, n_dmax);  // (folded after tile 0's S chain)
  const float qn = my_col < nC ? qnorm[my_col] : 0.f;
  fill(0, 0);

  bf16x8 cf[3][NK];  // query planes: lane (r32, hh) holds elements 16 kk + 8 hh + 0..7 of its query
  {
    const bool ok = my_col < nC;
    const f32x4* src = reinterpret_cast<const f32x4*>(C + (ok ? my_col : 0) * H);
    f32x4 u[2 * NK];
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) {
      u[2 * kk] = src[4 * kk + 2 * hh];
      u[2 * kk + 1] = src[4 * kk + 2 * hh + 1];
    }
    __builtin_amdgcn_sched_barrier(0);  // every query load issued before the first wait
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) {
      const f32x4 u0 = u[2 * kk], u1 = u[2 * kk + 1];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = ok ? (j < 4 ? u0[j] : u1[j - 4]) : 0.f;
        __bf16 a0, a1, a2;
        split3(x, a0, a1, a2);
        cf[0][kk][j] = a0;
        cf[1][kk][j] = a1;
        cf[2][kk][j] = a2;
      }
    }
  }
  LdsOffs<H> lo;
  lo.init(lane);
  // P: tile t's block of this wave's 32 queries at a wave-uniform base, the lane's column and
  // half (4 hh rows) as a 32-bit offset, the register's row as the store's immediate
  const float* pcol = P + (cb * NW + wid) * 1024;  // (= my_col >> 5: wave-uniform)
  const int64_t pstride = p_nqt * 1024;          // floats from one candidate tile's blocks to the next
  const unsigned pvo = (unsigned)((4 * hh * 32 + r32) * 4);

  // Prologue: stage 0 and the query rows in flight together (an all-CU burst runs ~11 B/cycle/CU:
  // every KiB waited for here costs ~50 ns); stage 1 is issued once the queries are split and
  // lands beside tile 0's S chain, stage 2 after it.
  fill(1, 1);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NF) : "memory");  // stage 0 landed (younger: stage 1)
  asm volatile("s_barrier" ::: "memory");

  f32x16 X[2];  // S chain results: X[t & 1] = tile t's
  {             // tile 0's S chain (the prologue)
    const lds_char_t* t0 = slot_tile(0);
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) {
      SplitOp o;
#pragma unroll
      for (int j = 0; j < 3; ++j) split_fwd_piece<H>(o, kk, j, t0, t0, t0, lo);
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        X[0] = mfma_bf16(o.a(kPa[j]), cf[kPb[j]][kk], kk == 0 && j == 0 ? f32x16{} : X[0]);
      }
    }
  }
  const float dmax = fold_loaded(dparts);  // wave-uniform
  const float shift = my_col < nC ? col_shift(c2, qn, dmax) : 0.f;
  if (dmax_out && blockIdx.x == 0 && threadIdx.x == 0) *dmax_out = dmax;  // (as score_bf16_kernel)
  if constexpr (NSLOT == 4) {
    fill(2, 2);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NF) : "memory");  // stage 1 landed (younger: stage 2)
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stage 1 landed
  }
  asm volatile("s_barrier" ::: "memory");
  SplitOp ring[kSd];  // operands of the next kSd steps
#pragma unroll
  for (int i = 0; i < kSd; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) split_fwd_piece<H>(ring[i], i, j, slot_tile(1), slot_tile(0), slot_tile(1), lo);

  float ev[2][16];
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int v = 0; v < 16; ++v) ev[k][v] = 0.f;

  int sl = 0;  // ring slot of tile t
  auto unit = [&](int64_t t, const f32x16& xa, f32x16& xb, float (&e)[16], float (&e_prev)[16]) {
    const int s1 = sl + 1 == NSLOT ? 0 : sl + 1, s2n = s1 + 1 == NSLOT ? 0 : s1 + 1;
    const lds_char_t* a_tile = slot_tile(sl);   // tile t (Acc chain)
    const lds_char_t* s_tile = slot_tile(s1);   // tile t+1 (S chain)
    const lds_char_t* n_tile = slot_tile(s2n);  // tile t+2 (next unit's first operands)
    if constexpr (NSLOT == 3) {
      asm volatile("s_barrier" ::: "memory");  // every wave is past tile t-1's Acc chain
      fill(s2n, t + 2);
    }
    const float* pblk = pcol + ((row_begin >> 5) + t) * pstride;
    TT_TRACE(0);
#ifdef TT_SCORER_TRACE
    if (blockIdx.x == 0 && threadIdx.x == 0 && t < 64) g_tt_trace[t * 8 + 2] = __builtin_amdgcn_s_memrealtime();
#endif
    float ls = 0.f;
    bf16x8 g[3][2];
    float r1[SPS], r2[SPS];
    auto pstore = [&](int v) {
      asm volatile("global_store_dword %0, %1, %2 offset:%3" ::"v"(pvo), "v"(e[v]), "s"(pblk), "n"(acc_row(v, 0) * 128)
                   : "memory");  // (+ 4 hh rows in pvo: hh is per lane)
    };
#pragma unroll
    for (int i = 0; i < NSTEP; ++i) {
      if (i == NSTEP - kSd) {  // the barrier point: fill(t+2) landed (younger: this unit's 16 P stores)
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
#pragma unroll
        for (int v = 0; v < 16; ++v) asm volatile("" : "+v"(e_prev[v]));  // unit t-1's stores have read them
        TT_TRACE(1);
        asm volatile("s_barrier" ::: "memory");
        TT_TRACE(3);
      }
      SplitOp nx;
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const SplitOp& cur = ring[i % kSd];
        if (i < NK) {
          xb = mfma_bf16(cur.a(kPa[j]), cf[kPb[j]][i], i == 0 && j == 0 ? f32x16{} : xb);
        } else {
          const int st = i - NK, s2 = st / NHT, ht = st % NHT;
          acc[ht] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur.a(kPa[j]), g[kPb[j]][s2], acc[ht], 0, 0, 0);
        }
        if constexpr (NSLOT == 4) {  // fill(t+3) into tile t-1's slot, one piece per MFMA gap after the barrier
          const int f = (i - (NSTEP - kSd)) * 6 + j;
          if (f >= 0 && f < NF) fill_piece(sl == 0 ? 3 : sl - 1, t + 3, f);
        }
        split_fwd_piece<H>(nx, i + kSd, j, s_tile, a_tile, n_tile, lo);
        if (i < NK) {  // the map of tile t, slots [SPS i, SPS (i + 1))
#pragma unroll
          for (int q = 0; q < SPS; ++q) {
            const int v = SPS * i + q;
            if (j == 0) {
              e[v] = __builtin_amdgcn_exp2f(xa[v] * c2 - shift);
              asm volatile("" : "+v"(e[v]));
            } else if (j == 1) {
              ls += e[v];
              pstore(v);
            } else if (j == 2) {
              const __bf16 h0 = (__bf16)e[v];
              g[0][v >> 3][v & 7] = h0;
              r1[q] = e[v] - (float)h0;
              asm volatile("" : "+v"(r1[q]));
            } else if (j == 3) {
              const __bf16 h1 = (__bf16)r1[q];
              g[1][v >> 3][v & 7] = h1;
              r2[q] = r1[q] - (float)h1;
              asm volatile("" : "+v"(r2[q]));
            } else if (j == 4) {
              g[2][v >> 3][v & 7] = (__bf16)r2[q];
            }
          }
          if (j == 1) asm volatile("" : "+v"(ls));
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      ring[i % kSd] = nx;
    }
    l_run += ls;
    sl = s1;
  };
  TT_KTRACE_K(1, 1);
  int64_t t = 0;
  for (; t + 2 <= ntiles; t += 2) {
    unit(t, X[0], X[1], ev[0], ev[1]);
    unit(t + 1, X[1], X[0], ev[1], ev[0]);
  }
  if (t < ntiles) unit(t, X[0], X[1], ev[0], ev[1]);
  TT_KTRACE_K(1, 2);
  drain_dma();  // no LDS-DMA or P store may outlive the workgroup
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int v = 0; v < 16; ++v) asm volatile("" : "+v"(ev[k][v]));
  __syncthreads();  // every wave is past its last ring read: the ring takes the partial images
  write_partials_t<FWD, H>(acc, l_run, split, nC, my_col - r32, r32, hh, acc_part, l_part,
                           (lds_char_t*)smem + wid * 32 * H * 4);
  TT_KTRACE_K(1, 3);
}

// P fragment of one 32-query tile for lane (candidate r32, hh): queries 8k + 4 hh + u (k, u < 4)
// of its candidate row, four 16-B asm loads (no compiler vmcnt waits: the unit's own waits count
// them).
struct SplitPSet {
  f32x4 v[4];
};
__device__ __forceinline__ void split_p_load(SplitPSet& d, const float* sbase, unsigned voff) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    i32x4 r;
    asm volatile("global_load_dwordx4 %0, %1, %2 offset:%3" : "=v"(r) : "v"(voff), "s"(sbase), "n"(32 * k) : "memory");
    d.v[k] = __builtin_bit_cast(f32x4, r);
  }
}
__device__ __forceinline__ void split_p_tie(SplitPSet& d) {
#pragma unroll
  for (int k = 0; k < 4; ++k) asm volatile("" : "+v"(d.v[k]));
}

// Backward from stored fp32 P: R = the scaled-query planes (nR = B rows + zero tail), columns =
// candidates (nC = M), dD^T partials per query split.
// Software-pipelined like the forward: unit t is the Acc chain of tile t (NSA steps of six MFMAs,
// operands read kSd steps ahead in one piece per MFMA gap, across the unit boundary), with the
// split of the next tile's G (P(t+1): two of its 16 values a step) beside it.  Round 4's first
// form split a tile's G and then ran its chain (0.44 MFMA busy at C2).
//   Ring (three 32-row stages): unit t reads tile t and, in its last kSd steps, tile t+1.  At step
//   NSA - kSd (the barrier point) fill(t+1) must have landed in every wave: wait, barrier; that
//   also frees tile t-1's slot, which takes fill(t+2), one 1 KiB piece per MFMA gap.
//   P: four register sets; P(t+3) is issued at unit t's start (into the set P(t-1) left), two
//   units ahead of its split.  VMEM order per unit: P(t+3), fill(t+2), so at unit t's start
//   P(t+1) has landed once at most fill(t), P(t+2), fill(t+1) are in flight (2 NF + 4), and at
//   its barrier point fill(t+1) has once at most P(t+3) is (4).
template <int H>
__global__ __launch_bounds__(NT, 1) void score_split_ddp_kernel(const __bf16* __restrict__ R, int64_t plane, int64_t nR,
                                                                int64_t nC, int S, int64_t rows_per_split,
                                                                const float* __restrict__ P, int64_t p_nqt,
                                                                float* __restrict__ acc_part) {
  using ST = SplitTile<H>;
  constexpr int NHT = H / 32, NSA = 2 * NHT, NF = ST::NF;
  constexpr int kSd = 2, EPS = 16 / NSA;  // operand distance (steps), G values split per step
  static_assert(NSA % kSd == 0 && NF <= 6 * kSd, "a fill's pieces fit the steps after the barrier point");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const lds_char_t* lds = (const lds_char_t*)smem;
  const int lane = lane_id(), wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r32 = lane & 31, hh = lane >> 5;
  const int split = blockIdx.x % S;
  const int64_t cb = blockIdx.x / S;
  const int64_t ct = cb * NW + wid;  // this wave's 32-candidate tile
  const int64_t row_begin = (int64_t)split * rows_per_split;
  const int64_t row_end = min(nR, row_begin + rows_per_split);
  const int64_t ntiles = row_end > row_begin ? (row_end - row_begin + ST::BJ - 1) / ST::BJ : 0;
  TT_KTRACE_K(0, 0);
  f32x16 acc[NHT];
#pragma unroll
  for (int t = 0; t < NHT; ++t) acc[t] = f32x16{};
  if (ntiles == 0) {  // (workgroup-uniform) no rows: zero partials
    write_partials<DD, H>(acc, 0.f, split, nC, ct * 32 + r32, hh, acc_part, nullptr);
    return;
  }

  unsigned fo[ST::NPP];
  split_fill_offs<H>(fo);
  const unsigned wbase = __builtin_amdgcn_readfirstlane(lds_addr(smem) + wid * 1024);
  auto stage_row = [&](int64_t t) { return t < ntiles ? row_begin + t * ST::BJ : row_begin; };
  auto fill_piece = [&](int b, int64_t t, int f) {  // piece f (plane f / NPP) of stage t into slot b
    const int p = f / ST::NPP, c = f % ST::NPP;
    glds_dwordx4_s(fo[c], R + p * plane + stage_row(t) * H, wbase + b * ST::STAGE_B + p * ST::PLANE_B + c * NW * 1024);
  };
  auto fill = [&](int b, int64_t t) {
#pragma unroll
    for (int f = 0; f < NF; ++f) fill_piece(b, t, f);
  };
  auto slot_tile = [&](int b) { return lds + b * ST::STAGE_B; };
  const float* pcol = P + ct * p_nqt * 1024;
  const unsigned pvo = (unsigned)(r32 * 128 + hh * 16);
  auto pload = [&](SplitPSet& d, int64_t t) { split_p_load(d, pcol + (stage_row(t) >> 5) * 1024, pvo); };
  LdsOffs<H> lo;
  lo.init(lane);

  SplitPSet pf[4];
  pload(pf[0], 0);
  pload(pf[1], 1);
  fill(0, 0);
  pload(pf[2], 2);
  fill(1, 1);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NF + 4) : "memory");  // P(0), P(1), stage 0 landed
  asm volatile("s_barrier" ::: "memory");
  bf16x8 g[2][3][2];  // G planes: g[t & 1] = tile t's
  {
    split_p_tie(pf[0]);
    float e[16];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int u = 0; u < 4; ++u) e[4 * k + u] = pf[0].v[k][u];
    split_tile(e, g[0]);
  }
  SplitOp ring[kSd];
#pragma unroll
  for (int i = 0; i < kSd; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) split_acc_piece<H>(ring[i], i, j, slot_tile(0), lo);

  int sl = 0;  // ring slot of tile t
  // unit t: Acc chain of tile t from gc; P(t+1) (pn) split into gn; P(t+3) issued into pi
  auto unit = [&](int64_t t, const bf16x8 (&gc)[3][2], bf16x8 (&gn)[3][2], SplitPSet& pn, SplitPSet& pi) {
    const int s1 = sl == 2 ? 0 : sl + 1, sf = s1 == 2 ? 0 : s1 + 1;
    const lds_char_t* tile = slot_tile(sl);
    const lds_char_t* ntile = slot_tile(s1);
    TT_TRACE_B(0);
#ifdef TT_SCORER_TRACE
    if (blockIdx.x == 0 && threadIdx.x == 0 && t < 64) g_tt_trace_b[t * 8 + 4] = __builtin_amdgcn_s_memrealtime();
#endif
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NF + 4) : "memory");  // P(t+1) landed
    TT_TRACE_B(1);
    split_p_tie(pn);
    pload(pi, t + 3);
    float r1[EPS], r2[EPS];
#pragma unroll
    for (int i = 0; i < NSA; ++i) {
      if (i == NSA - kSd) {  // the barrier point: fill(t+1) landed (younger: P(t+3))
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        TT_TRACE_B(2);
        asm volatile("s_barrier" ::: "memory");
        TT_TRACE_B(3);
      }
      SplitOp nx;
      const int s2 = i / NHT, ht = i % NHT;
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        acc[ht] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ring[i % kSd].a(kPa[j]), gc[kPb[j]][s2], acc[ht], 0, 0, 0);
        const int f = (i - (NSA - kSd)) * 6 + j;  // fill(t+2) into tile t-1's slot, after the barrier
        if (f >= 0 && f < NF) fill_piece(sf, t + 2, f);
        if (i + kSd < NSA) split_acc_piece<H>(nx, i + kSd, j, tile, lo);
        else split_acc_piece<H>(nx, i + kSd - NSA, j, ntile, lo);
#pragma unroll
        for (int q = 0; q < EPS; ++q) {  // G values v = EPS i + q of tile t+1 (e index 4k + u)
          const int v = EPS * i + q;
          const float x = pn.v[v >> 2][v & 3];
          if (j == 2) {
            const __bf16 h0 = (__bf16)x;
            gn[0][v >> 3][v & 7] = h0;
            r1[q] = x - (float)h0;
            asm volatile("" : "+v"(r1[q]));
          } else if (j == 3) {
            const __bf16 h1 = (__bf16)r1[q];
            gn[1][v >> 3][v & 7] = h1;
            r2[q] = r1[q] - (float)h1;
            asm volatile("" : "+v"(r2[q]));
          } else if (j == 4) {
            gn[2][v >> 3][v & 7] = (__bf16)r2[q];
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      ring[i % kSd] = nx;
    }
    sl = s1;
  };
  TT_KTRACE_K(0, 1);
  int64_t t = 0;
  for (; t + 4 <= ntiles; t += 4) {
    unit(t, g[0], g[1], pf[1], pf[3]);
    unit(t + 1, g[1], g[0], pf[2], pf[0]);
    unit(t + 2, g[0], g[1], pf[3], pf[1]);
    unit(t + 3, g[1], g[0], pf[0], pf[2]);
  }
  if (t < ntiles) {  // (nested: no path runs a later unit without the earlier, whose loads it counts on)
    unit(t, g[0], g[1], pf[1], pf[3]);
    if (t + 1 < ntiles) {
      unit(t + 1, g[1], g[0], pf[2], pf[0]);
      if (t + 2 < ntiles) unit(t + 2, g[0], g[1], pf[3], pf[1]);
    }
  }
  TT_KTRACE_K(0, 2);
  drain_dma();  // no load may outlive the workgroup
#pragma unroll
  for (int k = 0; k < 4; ++k) split_p_tie(pf[k]);
  __syncthreads();  // every wave is past its last ring read: the ring takes the partial images
  write_partials_t<DD, H>(acc, 0.f, split, nC, ct * 32, r32, hh, acc_part, nullptr, (lds_char_t*)smem + wid * 32 * H * 4);
  TT_KTRACE_K(0, 3);
}

// ------------------------------------------------------------------------------------------
// Operand prep, one launch for both matrices: blocks [0, gq) take the q rows, blocks [gq, grid)
// the d rows (grid-stride, one wave per row).  Optional fp32 -> bf16 (RNE) copy, the row L2
// norms of q, and for d one max norm per block (dmax_part[b]; readers fold the <= kMaxPrepBlocks
// values themselves: no zero-initialised accumulator, no atomics).  Block 0 also writes the pad
// rows (kPadBytes - 16 zero bytes, then +inf for the backward lse2).

// xp: the rows as three bf16 planes (split3; plane stride xp_plane elements) for the split-bf16
// fp32 engine.
__device__ __forceinline__ void prep_rows(const float* __restrict__ x, int64_t rows, int H, __bf16* __restrict__ xb,
                                          float* __restrict__ norms, int64_t b0, int64_t nb, float& mx,
                                          __bf16* __restrict__ xp = nullptr, int64_t xp_plane = 0) {
  const int lane = lane_id(), wid = threadIdx.x >> 6;
  if (H == 4 * kWave) {  // one float4 per lane per row: four rows' loads in flight per wave
    constexpr int U = 4;
    const int64_t step = nb * 4;
    for (int64_t r0 = b0 * 4 + wid; r0 < rows; r0 += U * step) {
      f32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t r = r0 + u * step;
        v[u] = r < rows ? reinterpret_cast<const f32x4*>(x + r * H)[lane] : f32x4{0.f, 0.f, 0.f, 0.f};
      }
      float ss[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t r = r0 + u * step;
        ss[u] = sumsq4(v[u]);
        if (xb && r < rows)
          reinterpret_cast<bf16x4*>(xb + r * H)[lane] =
              bf16x4{(__bf16)v[u][0], (__bf16)v[u][1], (__bf16)v[u][2], (__bf16)v[u][3]};
        if (xp && r < rows) {
          bf16x4 pl[3];
#pragma unroll
          for (int e = 0; e < 4; ++e) { __bf16 a0, a1, a2; split3(v[u][e], a0, a1, a2); pl[0][e] = a0; pl[1][e] = a1; pl[2][e] = a2; }
#pragma unroll
          for (int k = 0; k < 3; ++k) reinterpret_cast<bf16x4*>(xp + k * xp_plane + r * H)[lane] = pl[k];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t r = r0 + u * step;
        const float n = sqrtf(wave_sum(ss[u]));
        if (r < rows) {
          if (lane == 0 && norms) norms[r] = n;
          mx = fmaxf(mx, n);
        }
      }
    }
    return;
  }
  for (int64_t r = b0 * 4 + wid; r < rows; r += nb * 4) {
    const f32x4* src = reinterpret_cast<const f32x4*>(x + r * H);
    float ss = 0.f;
    for (int c = lane; c < H / 4; c += kWave) {
      const f32x4 v = src[c];
      ss += sumsq4(v);
      if (xb)
        reinterpret_cast<bf16x4*>(xb + r * H)[c] = bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
      if (xp) {
        bf16x4 pl[3];
#pragma unroll
        for (int e = 0; e < 4; ++e) { __bf16 a0, a1, a2; split3(v[e], a0, a1, a2); pl[0][e] = a0; pl[1][e] = a1; pl[2][e] = a2; }
#pragma unroll
        for (int k = 0; k < 3; ++k) reinterpret_cast<bf16x4*>(xp + k * xp_plane + r * H)[c] = pl[k];
      }
    }
    const float n = sqrtf(wave_sum(ss));
    if (lane == 0 && norms) norms[r] = n;
    mx = fmaxf(mx, n);
  }
}

__global__ __launch_bounds__(256) void prep_qd_kernel(const float* __restrict__ q, int64_t B,
                                                      const float* __restrict__ d, int64_t M, int H, int gq,
                                                      __bf16* __restrict__ qb, __bf16* __restrict__ db,
                                                      float* __restrict__ qnorm, float* __restrict__ dmax_part,
                                                      char* __restrict__ pad, float* __restrict__ lse2,
                                                      int* __restrict__ xrows, __bf16* __restrict__ dp = nullptr) {
  __shared__ float wmax[4];
  const int64_t dp_plane = (M + kTailRows) * H;  // dp: the candidate planes (split-bf16 fp32 forward)
  if (blockIdx.x == 0) {
    if (xrows && threadIdx.x == 0) xrows[0] = 0;
    for (int i = threadIdx.x; i < kPadBytes / 4; i += blockDim.x)
      reinterpret_cast<float*>(pad)[i] = (i >= (kPadBytes - 16) / 4) ? INFINITY : 0.f;
    for (int i = threadIdx.x; i < kTailRows; i += blockDim.x) lse2[B + i] = INFINITY;
    if (qb) {  // H % 8 == 0: 16-B stores (B * H and M * H are multiples of 8 elements)
      for (int64_t i = threadIdx.x; i < (int64_t)kTailRows * H / 8; i += blockDim.x) {
        reinterpret_cast<bf16x8*>(qb + B * H)[i] = bf16x8{};
        reinterpret_cast<bf16x8*>(db + M * H)[i] = bf16x8{};
      }
    }
    if (dp)
      for (int64_t i = threadIdx.x; i < (int64_t)kTailRows * H; i += blockDim.x)
        for (int k = 0; k < 3; ++k) dp[k * dp_plane + M * H + i] = (__bf16)0.f;
  }
  float mx = 0.f;
  if ((int)blockIdx.x < gq) {
    if (xrows)  // no query row redone exactly yet (see combine_rowv)
      for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < B; i += (int64_t)gq * blockDim.x)
        xrows[1 + i] = 0;
    prep_rows(q, B, H, qb, qnorm, blockIdx.x, gq, mx);
    return;
  }
  const int b = blockIdx.x - gq, gd = gridDim.x - gq;
  prep_rows(d, M, H, db, nullptr, b, gd, mx, dp, dp_plane);
  const int lane = lane_id(), wid = threadIdx.x >> 6;
  if (lane == 0) wmax[wid] = mx;
  __syncthreads();
  if (threadIdx.x == 0) dmax_part[b] = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
}


// The tower head's F.normalize (encoders.py:77) fused with the prep above, for the fused
// TwoTower output y = [q; d] (B + M rows, H = 256, one float4 per lane): each row is normalised
// in place exactly as head_normalize_kernel does it (norms[r] = |row| for the L2 backward), and
// the normalised row then takes prep_rows' path (bf16 copy, its norm, the per-block max) from the
// registers, so the scorer's prep pass and its 25 MB re-read disappear.  Same block partition
// and arithmetic as prep_qd_kernel + head_normalize_kernel: the workspace is bit-identical.
// One block of kL2PrepWaves waves: the grid keeps prep_qd_kernel's block counts (the candidate
// blocks' maxima are what the engines fold), but 16-wave blocks put 4x the rows in flight: with
// 4-wave blocks the pass ran 20 us for 63 MB (each wave walked 4-8 rows in dependent rounds).
// Round 3: 8-wave blocks with four rows' loads in flight per wave (the candidate blocks' waves
// each take their four rows in one round; the grid fits the chip in one round of blocks):
// 16.9 vs 20.1 us in the step (profiles/r03r_prep_ab.txt); TT_L2PREP_WAVES / _U for A/B.
#ifndef TT_L2PREP_WAVES
#define TT_L2PREP_WAVES 8
#endif
#ifndef TT_L2PREP_U
#define TT_L2PREP_U 4
#endif
constexpr int kL2PrepWaves = TT_L2PREP_WAVES;
__device__ __forceinline__ void l2_prep_rows(float* __restrict__ x, int64_t rows, __bf16* __restrict__ xb,
                                             float* __restrict__ norms, float* __restrict__ pnorms, int64_t b0,
                                             int64_t nb, float& mx) {
  constexpr int H = 4 * kWave, U = TT_L2PREP_U;
  const int lane = lane_id(), wid = threadIdx.x >> 6;
  const int64_t step = nb * kL2PrepWaves;
  for (int64_t r0 = b0 * kL2PrepWaves + wid; r0 < rows; r0 += U * step) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t r = r0 + u * step;
      v[u] = r < rows ? reinterpret_cast<const f32x4*>(x + r * H)[lane] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {  // head_normalize_kernel's arithmetic
      const int64_t r = r0 + u * step;
      const float ss = wave_sum(sumsq4(v[u]));
      const float nrm = sqrtf(ss), inv = 1.f / fmaxf(nrm, 1e-12f);
      v[u][0] *= inv;
      v[u][1] *= inv;
      v[u][2] *= inv;
      v[u][3] *= inv;
      if (r < rows) {
        reinterpret_cast<f32x4*>(x + r * H)[lane] = v[u];
        if (lane == 0) norms[r] = nrm;
      }
    }
    float ss[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // prep_rows' arithmetic on the normalised row
      const int64_t r = r0 + u * step;
      ss[u] = sumsq4(v[u]);
      if (r < rows)
        reinterpret_cast<bf16x4*>(xb + r * H)[lane] =
            bf16x4{(__bf16)v[u][0], (__bf16)v[u][1], (__bf16)v[u][2], (__bf16)v[u][3]};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t r = r0 + u * step;
      const float n = sqrtf(wave_sum(ss[u]));
      if (r < rows) {
        if (lane == 0 && pnorms) pnorms[r] = n;
        mx = fmaxf(mx, n);
      }
    }
  }
}

__global__ __launch_bounds__(64 * kL2PrepWaves) void l2_prep_kernel(float* __restrict__ y, int64_t B, int64_t M, int gq,
                                                      float* __restrict__ norms, __bf16* __restrict__ qb,
                                                      __bf16* __restrict__ db, float* __restrict__ qnorm,
                                                      float* __restrict__ dmax_part, char* __restrict__ pad,
                                                      float* __restrict__ lse2, int* __restrict__ xrows) {
  constexpr int H = 4 * kWave;
  __shared__ float wmax[kL2PrepWaves];
  if (blockIdx.x == 0) {  // prep_qd_kernel's block-0 set-up
    if (xrows && threadIdx.x == 0) xrows[0] = 0;
    for (int i = threadIdx.x; i < kPadBytes / 4; i += blockDim.x)
      reinterpret_cast<float*>(pad)[i] = (i >= (kPadBytes - 16) / 4) ? INFINITY : 0.f;
    for (int i = threadIdx.x; i < kTailRows; i += blockDim.x) lse2[B + i] = INFINITY;
    for (int64_t i = threadIdx.x; i < (int64_t)kTailRows * H / 8; i += blockDim.x) {  // 16-B stores
      reinterpret_cast<bf16x8*>(qb + B * H)[i] = bf16x8{};
      reinterpret_cast<bf16x8*>(db + M * H)[i] = bf16x8{};
    }
  }
  float mx = 0.f;
  if ((int)blockIdx.x < gq) {
    if (xrows)  // no query row redone exactly yet (see combine_rowv)
      for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < B; i += (int64_t)gq * blockDim.x)
        xrows[1 + i] = 0;
    l2_prep_rows(y, B, qb, norms, qnorm, blockIdx.x, gq, mx);
    return;
  }
  const int b = blockIdx.x - gq, gd = gridDim.x - gq;
  l2_prep_rows(y + B * H, M, db, norms + B, nullptr, b, gd, mx);
  const int lane = lane_id(), wid = threadIdx.x >> 6;
  if (lane == 0) wmax[wid] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    float m = wmax[0];
#pragma unroll
    for (int k = 1; k < kL2PrepWaves; ++k) m = fmaxf(m, wmax[k]);
    dmax_part[b] = m;
  }
}

// The same fusion for the fp32 scorer at H = 128 (C2): each row is normalised in place exactly as
// head_normalize_kernel<128> does it (two floats per lane), and prep_rows' arithmetic for an fp32
// scorer (no copies: the row norm from the normalised row as its 32 lanes of float4 would form it,
// the per-block maximum) runs on the registers: lane L < 32 takes the float4 of lanes 2L and 2L + 1,
// so the sum and its wave reduction are prep_qd_kernel's, bit for bit.  Blocks [0, gq) take the
// query rows, [gq, gq + gd) the candidate rows (4 waves per block, grid-stride as prep_qd_kernel).
__global__ __launch_bounds__(256) void l2_prep128_kernel(float* __restrict__ y, int64_t B, int64_t M, int gq,
                                                         float* __restrict__ norms, float* __restrict__ qnorm,
                                                         float* __restrict__ dmax_part, char* __restrict__ pad,
                                                         float* __restrict__ lse2, int* __restrict__ xrows,
                                                         __bf16* __restrict__ dp) {
  constexpr int H = 128;
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  __shared__ float wmax[4];
  const int64_t dp_plane = (M + kTailRows) * H;  // dp: the candidate planes (split-bf16 fp32 forward)
  if (blockIdx.x == 0) {  // prep_qd_kernel's block-0 set-up (fp32: no operand copies)
    if (xrows && threadIdx.x == 0) xrows[0] = 0;
    for (int i = threadIdx.x; i < kPadBytes / 4; i += blockDim.x)
      reinterpret_cast<float*>(pad)[i] = (i >= (kPadBytes - 16) / 4) ? INFINITY : 0.f;
    for (int i = threadIdx.x; i < kTailRows; i += blockDim.x) lse2[B + i] = INFINITY;
    if (dp)
      for (int64_t i = threadIdx.x; i < (int64_t)kTailRows * H; i += blockDim.x)
        for (int k = 0; k < 3; ++k) dp[k * dp_plane + M * H + i] = (__bf16)0.f;
  }
  const bool isq = (int)blockIdx.x < gq;
  const int64_t b0 = isq ? blockIdx.x : blockIdx.x - gq, nb = isq ? gq : gridDim.x - gq;
  const int64_t rows = isq ? B : M, base = isq ? 0 : B;
  if (isq && xrows)  // no query row redone exactly yet (see combine_rowv)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < B; i += (int64_t)gq * blockDim.x)
      xrows[1 + i] = 0;
  const int lane = lane_id(), wid = threadIdx.x >> 6;
  float mx = 0.f;
  // a wave's rows r0 + k stride (k < NR) at once: their loads in flight together and their shuffle
  // reductions interleaved (one row at a time waited a load and 12 shuffles per row); NR = 2 keeps
  // the kernel near 50 VGPRs (every wave of the grid resident)
  constexpr int NR = 2;
  const int64_t stride = nb * 4;
  for (int64_t r0 = b0 * 4 + wid; r0 < rows; r0 += NR * stride) {
    f32x2 v[NR];
    float nrm[NR], n[NR];
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const int64_t r = r0 + k * stride;
      v[k] = reinterpret_cast<const f32x2*>(y + (base + (r < rows ? r : r0)) * H)[lane];
    }
#pragma unroll
    for (int k = 0; k < NR; ++k) {  // (rows past the end repeat row r0: computed, never stored)
      const float ss = wave_sum(__builtin_fmaf(v[k][1], v[k][1], v[k][0] * v[k][0]));  // head_normalize_kernel<128>
      nrm[k] = sqrtf(ss);
      const float inv = 1.f / fmaxf(nrm[k], 1e-12f);
      v[k][0] *= inv;
      v[k][1] *= inv;
      // prep_rows (H = 128): lane L < 32 holds elements 4L .. 4L + 3, i.e. lanes 2L and 2L + 1 here
      const int src = (2 * lane) & (kWave - 1);
      const f32x4 v4 = {__shfl(v[k][0], src), __shfl(v[k][1], src), __shfl(v[k][0], src + 1), __shfl(v[k][1], src + 1)};
      n[k] = sqrtf(wave_sum(lane < 32 ? sumsq4(v4) : 0.f));
    }
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const int64_t r = r0 + k * stride;
      if (r >= rows) break;  // (wave-uniform)
      reinterpret_cast<f32x2*>(y + (base + r) * H)[lane] = v[k];
      if (lane == 0) norms[base + r] = nrm[k];
      if (dp && !isq) {
        bf16x2 pl[3];
#pragma unroll
        for (int e = 0; e < 2; ++e) { __bf16 a0, a1, a2; split3(v[k][e], a0, a1, a2); pl[0][e] = a0; pl[1][e] = a1; pl[2][e] = a2; }
#pragma unroll
        for (int q = 0; q < 3; ++q) reinterpret_cast<bf16x2*>(dp + q * dp_plane + r * H)[lane] = pl[q];
      }
      if (isq && lane == 0) qnorm[r] = n[k];
      mx = fmaxf(mx, n[k]);
    }
  }
  if (isq) return;
  if (lane == 0) wmax[wid] = mx;
  __syncthreads();
  if (threadIdx.x == 0) dmax_part[b0] = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
}

// One matrix: optional bf16 copy (with a kTailRows zero tail written by block 0), optional row
// norms, optional per-block max norm (max_parts[b], gridDim.x <= kMaxPrepBlocks values).
__global__ __launch_bounds__(256) void prep_rows_kernel(const float* __restrict__ x, int64_t rows, int H,
                                                        __bf16* __restrict__ xb, float* __restrict__ norms,
                                                        float* __restrict__ max_parts) {
  __shared__ float wmax[4];
  if (blockIdx.x == 0 && xb)
    for (int64_t i = threadIdx.x; i < (int64_t)kTailRows * H; i += blockDim.x) xb[rows * H + i] = (__bf16)0.f;
  float mx = 0.f;
  prep_rows(x, rows, H, xb, norms, blockIdx.x, gridDim.x, mx);
  if (!max_parts) return;
  const int lane = lane_id(), wid = threadIdx.x >> 6;
  if (lane == 0) wmax[wid] = mx;
  __syncthreads();
  if (threadIdx.x == 0) max_parts[blockIdx.x] = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
}

// lse2 tail of the backward engine's R rows: +inf (G = 0 on the zero rows).
__global__ void fill_inf_kernel(float* __restrict__ p, int n) {
  if ((int)threadIdx.x < n) p[threadIdx.x] = INFINITY;
}

// Merge forward split partials, one wave per query row:
//   l_i    = sum_s l_s,i - n_pad 2^-shift_i             (pad rows: X = 0 exactly)
//   lse_i  = (shift_i + log2 l_i) ln 2
//   loss_i = lse_i - (q~_i . d~_label) inv_tau           (diagonal logit, fp32 dot of the operands)
//   dqu_i  = O_i / l_i - d~_label,   O_i = sum_s Acc_s,i
// Rows whose bound sits so far above the true max that l underflows (l < 2^-100) are redone
// exactly (exact_row); with a stored-P backward they are listed in xrows for the backward combine.
template <typename DT>
__global__ __launch_bounds__(256) void fwd_combine_kernel(
    int64_t B, int64_t M, int H, int S, int n_pad, float c2, const float* __restrict__ qnorm,
    const float* __restrict__ dmax_part, int n_dmax, const float* __restrict__ l_part,
    const float* __restrict__ acc_part, float inv_tau, int64_t label_off, const DT* __restrict__ Qmat,
    const DT* __restrict__ Dmat, float* __restrict__ lse, float* __restrict__ lse2, float* __restrict__ loss_rows,
    float* __restrict__ dqu, DT* __restrict__ qs = nullptr, int* __restrict__ xrows = nullptr,
    int S_loc = 0, const float* __restrict__ dmax_loc = nullptr, int n_dmax_loc = 0,
    __bf16* __restrict__ qsp = nullptr, const float* __restrict__ dmax_folded = nullptr) {
  // S_loc > 0 (data-parallel forward in two launches): slots [0, S_loc) hold the local launch's
  // partials, formed with the local norm bound; they are rescaled to this launch's shift.
  // qsp: the scaled query rows as three bf16 planes (split-bf16 fp32 backward) instead of qs.
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = lane_id();
  const int64_t qsp_plane = (B + kTailRows) * H;
  if (i >= B) {  // the zero tail of the scaled query copy (the stored-P backward's R rows)
    if (qs && i < B + kTailRows)
      for (int h = lane; h < H; h += kWave) qs[i * H + h] = (DT)0.f;
    if (qsp && i < B + kTailRows)
      for (int h = lane; h < H; h += kWave)
        for (int pl = 0; pl < 3; ++pl) qsp[pl * qsp_plane + i * H + h] = (__bf16)0.f;
    return;
  }
  // dmax_folded: the engine's fold of the same block maxima (the same float)
  const float sh = col_shift(c2, qnorm[i], dmax_folded ? *dmax_folded : fold_dmax(dmax_part, n_dmax));
  const float f_loc = S_loc > 0 ? __builtin_amdgcn_exp2f(col_shift(c2, qnorm[i], fold_dmax(dmax_loc, n_dmax_loc)) - sh)
                                : 1.f;
  float l = sum_parts1(l_part + i, B, S, S_loc, f_loc);
  auto row_v = [&](auto vtag) {  // V = H / 64 floats per lane: every split's loads in flight together
    constexpr int V = decltype(vtag)::value;
    using FV = typename RowVec<V>::f;
    const float loss_i = combine_rowv<DT, V>(
        i, l,
        [&] {
          const FV* p = reinterpret_cast<const FV*>(acc_part) + i * (H / V) + lane;
          if (S_loc == 0) return sum_parts4(p, B * (H / V), S);
          return sum_parts4(p + (int64_t)S_loc * B * (H / V), B * (H / V), S - S_loc) +
                 f_loc * sum_parts4(p, B * (H / V), S_loc);
        },
        sh, n_pad, M, c2, inv_tau, label_off, Qmat, Dmat, lse, lse2, dqu, qs, xrows, lane, qsp, qsp_plane);
    if (lane == 0) loss_rows[i] = loss_i;
  };
  if (H == 4 * kWave) return row_v(std::integral_constant<int, 4>{});
  if (H == 2 * kWave) return row_v(std::integral_constant<int, 2>{});
  l -= (float)n_pad * __builtin_amdgcn_exp2f(-sh);
  const DT* qr = Qmat + i * H;
  const DT* dl = Dmat + (i + label_off) * H;
  if (!(l >= 7.888609052210118e-31f)) {  // l < 2^-100 (or NaN): the bound overshot, redo the row exactly
    float m2, lx, o[4];
    exact_row(qr, Dmat, M, H, c2, lane, m2, lx, o);
    const float lse2_i = m2 + log2f(lx);
    const float dot = exact_row_dot(qr, dl, H, lane);
    if (lane == 0) {
      lse[i] = lse2_i * kLn2;
      lse2[i] = lse2_i;
      loss_rows[i] = lse2_i * kLn2 - dot * inv_tau;
    }
    const float inv_l = 1.f / lx;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int h = lane + kWave * u;
      if (h >= H) break;
      if (dqu) dqu[i * H + h] = o[u] * inv_l - (float)dl[h];
      if (qs) qs[i * H + h] = (DT)0.f;  // its stored P underflowed: the backward combine adds the row
      if (qsp)
        for (int pl = 0; pl < 3; ++pl) qsp[pl * qsp_plane + i * H + h] = (__bf16)0.f;
    }
    if ((qs || qsp) && xrows && lane == 0) {  // flagged for the backward combine (adds flagged rows in row order)
      xrows[1 + i] = 1;
      atomicAdd(xrows, 1);
    }
    return;
  }
  const float lse2_i = sh + log2f(l);  // log2 units, for the backward engine
  const float lse_i = lse2_i * kLn2;
  float dot = 0.f;
  for (int h = lane; h < H; h += kWave) dot += (float)qr[h] * (float)dl[h];
  dot = wave_sum(dot);
  if (qs) {
    const float f = __builtin_amdgcn_exp2f(sh - lse2_i);
    for (int h = lane; h < H; h += kWave) qs[i * H + h] = (DT)((float)qr[h] * f);
  }
  if (qsp) {
    const float f = __builtin_amdgcn_exp2f(sh - lse2_i);
    for (int h = lane; h < H; h += kWave) {
      __bf16 a0, a1, a2;
      split3((float)qr[h] * f, a0, a1, a2);
      qsp[i * H + h] = a0;
      qsp[qsp_plane + i * H + h] = a1;
      qsp[2 * qsp_plane + i * H + h] = a2;
    }
  }
  if (lane == 0) {
    lse[i] = lse_i;
    lse2[i] = lse2_i;
    loss_rows[i] = lse_i - dot * inv_tau;
  }
  if (dqu) {
    const float inv_l = 1.f / l;
    for (int h = lane; h < H; h += kWave) {
      const float o = sum_parts1(acc_part + i * H + h, B * H, S, S_loc, f_loc);
      dqu[i * H + h] = o * inv_l - (float)dl[h];
    }
  }
}

// dd_j = scale (sum_s Acc_s,j - [0 <= j - off < B] q~_{j-off});  dq = scale * dqu;
// scale = grad_loss * grad_scale * inv_tau.
// Stored-P backward only (xrows non-null): query rows the forward redid exactly (their stored P
// underflowed, their scaled-query rows are zero) add sum_i 2^(x_ij c2 - lse2_i) q~_i here.
// xrows = [count, flag of row 0, flag of row 1, ...]: the flagged rows are added in ascending row
// order (a list filled by atomics would fix the order of these fp32 sums per run, not per input).
template <class F>
__device__ __forceinline__ void for_exact_rows(const int* __restrict__ xrows, int64_t B, int lane, F f) {
  if (xrows[0] == 0) return;  // the usual case: one load per wave
  for (int64_t base = 0; base < B; base += kWave) {
    unsigned long long m = __ballot(base + lane < B && xrows[1 + base + lane] != 0);
    while (m) {
      const int k = __builtin_ctzll(m);
      m &= m - 1;
      f(base + k);
    }
  }
}

template <typename DT>
__device__ __forceinline__ void add_exact_rows(f32x4& a, const int* __restrict__ xrows, int64_t B,
                                               const DT* __restrict__ Qmat, const DT* __restrict__ dr,
                                               const float* __restrict__ lse2, float c2, int H, int lane) {
  for_exact_rows(xrows, B, lane, [&](int64_t i) {
    const DT* qr = Qmat + i * H;
    const float g = __builtin_amdgcn_exp2f(exact_row_dot(qr, dr, H, lane) * c2 - lse2[i]);
    a += g * load4(qr, lane);
  });
}

template <typename DT>
__global__ __launch_bounds__(256) void bwd_combine_kernel(int64_t B, int64_t M, int H, int S, int64_t label_off,
                                                          const float* __restrict__ acc_part,
                                                          const DT* __restrict__ Qmat, const float* __restrict__ dqu,
                                                          const float* __restrict__ grad_loss, float grad_scale,
                                                          float inv_tau, float* __restrict__ dq,
                                                          float* __restrict__ dd, const int* __restrict__ xrows = nullptr,
                                                          const DT* __restrict__ Dmat = nullptr,
                                                          const float* __restrict__ lse2 = nullptr, float c2 = 0.f,
                                                          const float* __restrict__ mean_x = nullptr,
                                                          float* __restrict__ mean_out = nullptr) {
  // one extra block, dispatched first (as in bwd_combine_l2_kernel): the forward's deferred loss mean
  if (mean_out && blockIdx.x == 0) {
    __shared__ float part[1024];
    const float m = block256_mean_as_1024(mean_x, B, part);
    if (threadIdx.x == 0) mean_out[0] = m;
    return;
  }
  const int64_t r = (int64_t)(blockIdx.x - (mean_out ? 1 : 0)) * 4 + (threadIdx.x >> 6);
  const int lane = lane_id();
  const float scale = grad_loss[0] * grad_scale * inv_tau;
  if (H == 4 * kWave) {
    if (r < M) {
      const int64_t qi = r - label_off;
      f32x4 a = sum_parts4(reinterpret_cast<const f32x4*>(acc_part) + r * (H / 4) + lane, M * (H / 4), S);
      if (xrows) add_exact_rows(a, xrows, B, Qmat, Dmat + r * H, lse2, c2, H, lane);
      if (qi >= 0 && qi < B) a -= load4(Qmat + qi * H, lane);
      reinterpret_cast<f32x4*>(dd + r * H)[lane] = a * scale;
    }
    if (r < B) reinterpret_cast<f32x4*>(dq + r * H)[lane] = reinterpret_cast<const f32x4*>(dqu + r * H)[lane] * scale;
    return;
  }
  if (r < M) {
    const int64_t qi = r - label_off;
    const bool lab = qi >= 0 && qi < B;
    for (int h0 = 0; h0 < H; h0 += kWave) {
      const int h = h0 + lane;
      float a = 0.f;
      if (h < H) a = sum_parts1(acc_part + r * H + h, M * H, S);
      if (xrows)  // exact rows (stored-P backward; see add_exact_rows)
        for_exact_rows(xrows, B, lane, [&](int64_t i) {
          const float g = __builtin_amdgcn_exp2f(exact_row_dot(Qmat + i * H, Dmat + r * H, H, lane) * c2 - lse2[i]);
          if (h < H) a += g * (float)Qmat[i * H + h];
        });
      if (h < H) {
        if (lab) a -= (float)Qmat[qi * H + h];
        dd[r * H + h] = a * scale;
      }
    }
  }
  if (r < B) {
    for (int h = lane; h < H; h += kWave) dq[r * H + h] = dqu[r * H + h] * scale;
  }
}

// bwd_combine_kernel fused with the tower head's F.normalize backward, for the fused TwoTower
// output y = [q; d] (H = 256): row r < B takes dq_r, row B + j takes dd_j, each formed exactly as
// bwd_combine_kernel forms it, and the row goes straight into l2_bwd_row4 (the arithmetic of
// l2norm_bwd_kernel) with y_r and norms[r]: dx = d loss / d(pre-normalise row).  dq and dd are
// never written; the result equals bwd_combine_kernel + l2norm_bwd_kernel bit for bit.
template <typename DT>
__global__ __launch_bounds__(256) void bwd_combine_l2_kernel(int64_t B, int64_t M, int S, int64_t label_off,
                                                             const float* __restrict__ acc_part,
                                                             const DT* __restrict__ Qmat, const float* __restrict__ dqu,
                                                             const float* __restrict__ grad_loss, float grad_scale,
                                                             float inv_tau, const float* __restrict__ y,
                                                             const float* __restrict__ norms, float* __restrict__ dx,
                                                             const int* __restrict__ xrows, const DT* __restrict__ Dmat,
                                                             const float* __restrict__ lse2, float c2,
                                                             const float* __restrict__ mean_x = nullptr,
                                                             float* __restrict__ mean_out = nullptr) {
  constexpr int H = 4 * kWave;
  // one extra block, dispatched first so its serial ~7 us hide under the other blocks (placed
  // last it ran after them and lengthened the launch by as much): the forward's deferred loss mean
  if (mean_out && blockIdx.x == 0) {
    __shared__ float part[1024];
    const float m = block256_mean_as_1024(mean_x, B, part);
    if (threadIdx.x == 0) mean_out[0] = m;
    return;
  }
  const int64_t r = (int64_t)(blockIdx.x - (mean_out ? 1 : 0)) * 4 + (threadIdx.x >> 6);
  if (r >= B + M) return;
  const int lane = lane_id();
  const float scale = grad_loss[0] * grad_scale * inv_tau;
  const f32x4 o = reinterpret_cast<const f32x4*>(y + r * H)[lane];  // issued first: independent of g
  const float nrm = norms[r];
  f32x4 g;
  if (r < B) {
    g = reinterpret_cast<const f32x4*>(dqu + r * H)[lane] * scale;
  } else {
    const int64_t j = r - B, qi = j - label_off;
    f32x4 a = sum_parts4(reinterpret_cast<const f32x4*>(acc_part) + j * (H / 4) + lane, M * (H / 4), S);
    if (xrows) add_exact_rows(a, xrows, B, Qmat, Dmat + j * H, lse2, c2, H, lane);
    if (qi >= 0 && qi < B) a -= load4(Qmat + qi * H, lane);
    g = a * scale;
  }
  reinterpret_cast<f32x4*>(dx + r * H)[lane] = l2_bwd_row4(g, o, nrm);
}

// The same fusion for the fp32 scorer at H = 128 (C2): row r < B takes dq_r, row B + j takes dd_j,
// each element formed exactly as bwd_combine_kernel's generic path forms it (split partials in
// split order, the exact rows of the stored-P form, the label row), then l2_bwd_row2 (the
// arithmetic of l2norm_bwd_kernel at H = 128) with y_r and norms[r].  Elements lane and lane + 64
// of each row per lane.
__global__ __launch_bounds__(256) void bwd_combine_l2_128_kernel(
    int64_t B, int64_t M, int S, int64_t label_off, const float* __restrict__ acc_part, const float* __restrict__ Qmat,
    const float* __restrict__ dqu, const float* __restrict__ grad_loss, float grad_scale, float inv_tau,
    const float* __restrict__ y, const float* __restrict__ norms, float* __restrict__ dx, const int* __restrict__ xrows,
    const float* __restrict__ Dmat, const float* __restrict__ lse2, float c2, const float* __restrict__ mean_x = nullptr,
    float* __restrict__ mean_out = nullptr) {
  constexpr int H = 2 * kWave;
  if (mean_out && blockIdx.x == 0) {  // the forward's deferred loss mean, as bwd_combine_kernel
    __shared__ float part[1024];
    const float m = block256_mean_as_1024(mean_x, B, part);
    if (threadIdx.x == 0) mean_out[0] = m;
    return;
  }
  const int64_t r = (int64_t)(blockIdx.x - (mean_out ? 1 : 0)) * 4 + (threadIdx.x >> 6);
  if (r >= B + M) return;
  const int lane = lane_id();
  const float scale = grad_loss[0] * grad_scale * inv_tau;
  const float o0 = y[r * H + lane], o1 = y[r * H + lane + kWave];  // issued first: independent of g
  const float nrm = norms[r];
  float g[2];
  if (r < B) {
    g[0] = dqu[r * H + lane] * scale;
    g[1] = dqu[r * H + lane + kWave] * scale;
  } else {
    const int64_t j = r - B, qi = j - label_off;
    float a[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) a[u] = sum_parts1(acc_part + j * H + lane + u * kWave, M * H, S);
    if (xrows)  // exact rows (stored-P backward; see add_exact_rows)
      for_exact_rows(xrows, B, lane, [&](int64_t i) {
        const float gi = __builtin_amdgcn_exp2f(exact_row_dot(Qmat + i * H, Dmat + j * H, H, lane) * c2 - lse2[i]);
#pragma unroll
        for (int u = 0; u < 2; ++u) a[u] += gi * Qmat[i * H + lane + u * kWave];
      });
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (qi >= 0 && qi < B) a[u] -= Qmat[qi * H + lane + u * kWave];
      g[u] = a[u] * scale;
    }
  }
  float y0, y1;
  l2_bwd_row2(g[0], g[1], o0, o1, nrm, y0, y1);
  dx[r * H + lane] = y0;
  dx[r * H + lane + kWave] = y1;
}

// Where the backward's combine goes: dq / dd (the loss gradients), or, with `dx` set, the fused
// F.normalize backward above (y = [q; d] rows, norms of the tower head; H = 256 with bf16
// operands, H = 128 with fp32).
struct BwdOut {
  float* dq;
  float* dd;
  const float* y = nullptr;
  const float* norms = nullptr;
  float* dx = nullptr;
  const float* loss_rows = nullptr;  // with dx: the forward's per-row losses, whose mean this launch
  float* loss = nullptr;             // forms in one extra block (the forward deferred it)
};

template <typename DT>
void launch_bwd_combine(int64_t B, int64_t M, int H, int S, int64_t label_off, const float* acc_part, const DT* Qlab,
                        const float* dqu, const float* grad_loss, float grad_scale, float inv_tau, const BwdOut& out,
                        const int* xrows, const DT* Db, const float* lse2, hipStream_t s) {
  const float c2 = inv_tau * kLog2e;
  if constexpr (std::is_same<DT, float>::value) {
    if (out.dx) {  // fp32, H = 128 (tt_inbatch_bwd_l2 checks the shape)
      bwd_combine_l2_128_kernel<<<dim3((unsigned)((B + M + 3) / 4 + (out.loss ? 1 : 0))), dim3(256), 0, s>>>(
          B, M, S, label_off, acc_part, Qlab, dqu, grad_loss, grad_scale, inv_tau, out.y, out.norms, out.dx, xrows, Db,
          lse2, c2, out.loss_rows, out.loss);
      return;
    }
  }
  if (out.dx) {
    bwd_combine_l2_kernel<DT><<<dim3((unsigned)((B + M + 3) / 4 + (out.loss ? 1 : 0))), dim3(256), 0, s>>>(
        B, M, S, label_off, acc_part, Qlab, dqu, grad_loss, grad_scale, inv_tau, out.y, out.norms, out.dx, xrows, Db,
        lse2, c2, out.loss_rows, out.loss);
    return;
  }
  const int64_t rows = std::max(B, M);
  bwd_combine_kernel<DT><<<dim3((unsigned)((rows + 3) / 4 + (out.loss ? 1 : 0))), dim3(256), 0, s>>>(
      B, M, H, S, label_off, acc_part, Qlab, dqu, grad_loss, grad_scale, inv_tau, out.dq, out.dd, xrows, Db, lse2, c2,
      out.loss_rows, out.loss);
}

// ------------------------------------------------------------------------------------------
// Host side.
struct Plan {
  int S;
  int64_t rows_per_split;
  int grid;
  int n_pad;  // zero rows processed past the end of the last split
};

// Split the streamed rows so the grid is one round of resident workgroups (256 CUs x wg_per_cu):
// a second round would only add prologues/epilogues and twice the split partials.
Plan plan_for(int64_t nR, int64_t nC, int BJ, int wg_per_cu, int cols_per_block = 32 * NW, int cus = 256) {
  const int64_t ncb = (nC + cols_per_block - 1) / cols_per_block;
  const int64_t row_tiles = (nR + BJ - 1) / BJ;
  const int64_t target = (int64_t)cus * wg_per_cu;
  int64_t S = (target + ncb - 1) / ncb;
  if (S > 8) S = 8;
  if (S > row_tiles) S = row_tiles;
  if (S < 1) S = 1;
  const int64_t rps = (row_tiles + S - 1) / S * BJ;
  S = (nR + rps - 1) / rps;
  if (S < 1) S = 1;
  const int64_t last = nR - (S - 1) * rps;
  const int64_t n_pad = (last + BJ - 1) / BJ * BJ - last;
  return Plan{(int)S, rps, (int)(ncb * S), (int)n_pad};
}

int bj_for(int dtype) { return dtype == TT_F32 ? Tile<float, 64>::BJ : Tile<__bf16, 64>::BJ; }

// resident workgroups per CU (register-limited: launch_bounds min-blocks of the engines)
int wg_per_cu(int H, int dtype, int mode) {
  if (H == 128 && dtype == TT_F32) return mode == FWD ? TT_F32_MINW128_FWD : TT_F32_MINW128_DD;
  return H <= 128 ? 2 : 1;
}

struct Ws {
  __bf16* Qb;
  __bf16* Db;
  __bf16* Qs;   // stored-P backward: q~ scaled by 2^(shift - lse2) (+ zero tail)
  float* Qs32;  // ... the fp32 form (fp32 scorer: q scaled in fp32, P fp32)
  __bf16* Qsp;  // ... as three bf16 planes (the split-bf16 fp32 backward), plane stride (B + tail) H
  __bf16* Dp;   // split-bf16 fp32 forward: the candidate planes, plane stride (M + tail) H
  char* P;      // stored-P backward: bf16 probabilities, p_nct x p_nqt blocks of 2 KiB
  int* xrows;   // stored-P backward: [count, flag per query row] of queries the forward redid exactly
  int64_t p_nqt;
  float* qnorm;
  float* lse2;
  float* dmax_part;
  float* dmax_fold;  // the stored-P forward engine's fold of dmax_part (one float), read by the combine
  char* pad;
  float* l_part;
  float* acc_part;
  size_t total;
};

// Backward form of the single-process bf16 loss.  Default: stored probabilities (the backward
// takes G from the forward's bf16 P instead of recomputing S = Q D^T; executed flops 6BMH instead
// of 8BMH).  TT_INBATCH_BWD=recompute (read at load) or tt_inbatch_set_backward(0) selects the
// recompute engine.  P is kept only up to 2^31 entries (4 GiB of bf16); larger batches recompute.
std::atomic<int>& bwd_mode() {
  static std::atomic<int> m{[] {
    const char* e = std::getenv("TT_INBATCH_BWD");
    return (e && std::strcmp(e, "recompute") == 0) ? 0 : 1;
  }()};
  return m;
}
bool stored_p(int dtype, int64_t B, int64_t M) {
  if (bwd_mode().load(std::memory_order_relaxed) != 1) return false;
  if (dtype == TT_BF16) return B * M <= (int64_t(1) << 31);
  return dtype == TT_F32 && B * M <= (int64_t(1) << 30);  // fp32 P: up to 4 GiB
}

// The fp32 stored-P passes run the split-bf16 engines (score_split_*_kernel) at H = 64, 128, 256;
// H = 32 keeps score_f32_kernel's stored-P form (a 32-row plane tile is under one 1 KiB piece per
// wave).  One workgroup per CU.
bool split_f32(int H, int dtype, int64_t B, int64_t M) {
  return dtype == TT_F32 && (H == 64 || H == 128 || H == 256) && stored_p(dtype, B, M);
}

// P grid: query tiles up to the forward's 128-column blocks, candidate tiles up to the
// backward's 128-column blocks (every tile either engine touches exists)
int64_t p_nqt_for(int64_t B) { return (B + 127) / 128 * 4; }
int64_t p_nct_for(int64_t M) { return (M + 255) / 256 * 8; }  // also the 256-candidate backward blocks
// fp32 P (score_f32_kernel<., ., true>): 32 x 32 blocks of 4 KiB, candidate tiles up to the
// backward's 128-candidate blocks, query tiles as above
int64_t p32_nct_for(int64_t M) { return (M + 127) / 128 * 4; }

// candidate tiles per wave of the stored-P backward (score_ddp_kernel<H, CW>)
#ifndef TT_DDP_CW256
#define TT_DDP_CW256 1  // CW = 2 runs the loop ~15 % faster but doubles the split partials (S = 4): net slower (round 2)
#endif
int ddp_cw(int H) { return H == 256 ? TT_DDP_CW256 : 1; }
Plan ddp_plan(int64_t B, int64_t M, int H) {
  return plan_for(B, M, Tile<__bf16, 64>::BJ, wg_per_cu(H, TT_BF16, DD), 32 * NW * ddp_cw(H));
}

// Layout: [Qb | Db | Qs | P] persist from forward to backward (the backward's MFMA operands);
// everything else is scratch reused by both passes.
Ws carve(void* base, int64_t B, int64_t M, int H, int dtype) {
  const int BJ = bj_for(dtype);
  const bool spl = split_f32(H, dtype, B, M);
  // (sized for the engines' largest split counts: the split-bf16 passes plan for one workgroup per
  // CU, never more splits than the fp32 engine's two)
  const Plan pf = plan_for(M, B, BJ, wg_per_cu(H, dtype, FWD)), pd = plan_for(B, M, BJ, wg_per_cu(H, dtype, DD));
  const bool bf = dtype != TT_F32;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off = align_up(off + bytes, 256);
    return o;
  };
  // bf16 operand copies and lse2 carry a kTailRows tail (zeros / +inf): the engine's stage fills
  // never need per-lane redirection past the last row
  const size_t oq = take(bf ? (size_t)(B + kTailRows) * H * 2 : 0), od = take(bf ? (size_t)(M + kTailRows) * H * 2 : 0);
  const bool sp = stored_p(dtype, B, M);
  const size_t oqs = take(sp ? (size_t)(B + kTailRows) * H * (bf ? 2 : spl ? 6 : 4) : 0);
  const size_t odp = take(spl ? (size_t)3 * (M + kTailRows) * H * 2 : 0);
  const size_t op = take(sp ? (bf ? (size_t)p_nqt_for(B) * p_nct_for(M) * 2048 : (size_t)p_nqt_for(B) * p32_nct_for(M) * 4096)
                            : 0);
  const size_t ox = take(sp ? (size_t)(B + 1) * 4 : 0);
  const size_t oqn = take((size_t)B * 4), ol2 = take((size_t)(B + kTailRows) * 4), omx = take(kMaxPrepBlocks * 4 + 4);
  const size_t opad = take(kPadBytes), ol = take((size_t)pf.S * B * 4);
  size_t parts = std::max((size_t)pf.S * B, (size_t)pd.S * M) * H * 4;
  if (sp && bf) parts = std::max(parts, (size_t)ddp_plan(B, M, H).S * M * H * 4);
  if (sp && !bf) parts = std::max(parts, (size_t)plan_for(B, M, BJ, spl ? 1 : f32_waves(DD, H, true)).S * M * H * 4);
  const size_t oa = take(parts);
  Ws w{};
  char* b = static_cast<char*>(base);
  if (b) {
    w.Qb = reinterpret_cast<__bf16*>(b + oq);
    w.Db = reinterpret_cast<__bf16*>(b + od);
    w.Qs = sp && bf ? reinterpret_cast<__bf16*>(b + oqs) : nullptr;
    w.Qs32 = sp && !bf && !spl ? reinterpret_cast<float*>(b + oqs) : nullptr;
    w.Qsp = spl ? reinterpret_cast<__bf16*>(b + oqs) : nullptr;
    w.Dp = spl ? reinterpret_cast<__bf16*>(b + odp) : nullptr;
    w.P = sp ? b + op : nullptr;
    w.xrows = sp ? reinterpret_cast<int*>(b + ox) : nullptr;
    w.p_nqt = p_nqt_for(B);
    w.qnorm = reinterpret_cast<float*>(b + oqn);
    w.lse2 = reinterpret_cast<float*>(b + ol2);
    w.dmax_part = reinterpret_cast<float*>(b + omx);
    w.dmax_fold = sp ? w.dmax_part + kMaxPrepBlocks : nullptr;
    w.pad = b + opad;
    w.l_part = reinterpret_cast<float*>(b + ol);
    w.acc_part = reinterpret_cast<float*>(b + oa);
  }
  w.total = off;
  return w;
}

// Engine sub-range (data-parallel forward in two launches; see fwd_ex_local / fwd_ex_remote)
struct Skip {
  int64_t begin = 0, len = 0;  // streamed rows leave out R's rows [begin, begin + len)
  int split_base = 0;          // partial slot of split 0
};

template <int MODE, int H>
int launch_engine(int dtype, const void* R, int64_t nR, const void* C, int64_t nC, const Plan& p, float c2,
                  const float* lse2, const Ws& w, int n_dmax, hipStream_t s, const Skip& sk = Skip{}) {
  if constexpr (H >= 64) {
    if (dtype == TT_F32 && MODE == FWD && w.P && w.Dp) {  // split-bf16 forward storing fp32 G
      score_split_fwd_kernel<H><<<dim3(p.grid), dim3(NT), SplitFwdRing<H>::LDS_BYTES, s>>>(
          w.Dp, (nR + kTailRows) * H, nR, static_cast<const float*>(C), nC, p.S, p.rows_per_split, c2, w.qnorm,
          w.dmax_part, n_dmax, w.acc_part, w.l_part, reinterpret_cast<float*>(w.P), w.p_nqt, w.dmax_fold);
      TT_LAUNCH_CHECK("score_split_fwd");
      return TT_OK;
    }
  }
  if (H < 64 && dtype == TT_F32 && MODE == FWD && w.P) {  // H = 32: score_f32_kernel's stored-P forward
    score_f32_kernel<FWD, (H < 64 ? H : 32), true><<<dim3(p.grid), dim3(NT), Tile<float, H>::LDS_BYTES, s>>>(
        static_cast<const float*>(R), nR, static_cast<const float*>(C), nC, p.S, p.rows_per_split, c2, lse2,
        w.qnorm, w.dmax_part, n_dmax, w.pad, w.acc_part, w.l_part, reinterpret_cast<float*>(w.P), w.p_nqt);
  } else if (dtype == TT_F32) {
    score_f32_kernel<MODE, H><<<dim3(p.grid), dim3(NT), Tile<float, H>::LDS_BYTES, s>>>(
        static_cast<const float*>(R), nR, static_cast<const float*>(C), nC, p.S, p.rows_per_split, c2, lse2,
        w.qnorm, w.dmax_part, n_dmax, w.pad, w.acc_part, w.l_part);
  } else if (dtype == TT_BF16_SPLIT) {
    score_bf16_kernel<MODE, true, H><<<dim3(p.grid), dim3(NT), Tile<__bf16, H>::LDS_BYTES, s>>>(
        static_cast<const __bf16*>(R), nR, static_cast<const __bf16*>(C), nC, p.S, p.rows_per_split, c2, lse2,
        w.qnorm, w.dmax_part, n_dmax, w.pad, w.acc_part, w.l_part, nullptr, 0, sk.begin, sk.len, sk.split_base);
  } else if (MODE == FWD && w.P) {
    score_bf16_kernel<FWD, false, H, true><<<dim3(p.grid), dim3(NT), Tile<__bf16, H>::LDS_BYTES + NW * 2048, s>>>(
        static_cast<const __bf16*>(R), nR, static_cast<const __bf16*>(C), nC, p.S, p.rows_per_split, c2, lse2,
        w.qnorm, w.dmax_part, n_dmax, w.pad, w.acc_part, w.l_part, w.P, w.p_nqt, 0, 0, 0, w.dmax_fold);
  } else {
    score_bf16_kernel<MODE, false, H><<<dim3(p.grid), dim3(NT), Tile<__bf16, H>::LDS_BYTES, s>>>(
        static_cast<const __bf16*>(R), nR, static_cast<const __bf16*>(C), nC, p.S, p.rows_per_split, c2, lse2,
        w.qnorm, w.dmax_part, n_dmax, w.pad, w.acc_part, w.l_part, nullptr, 0, sk.begin, sk.len, sk.split_base);
  }
  TT_LAUNCH_CHECK(MODE == FWD ? "score_fwd" : "score_dd");
  return TT_OK;
}

template <int MODE>
int dispatch_engine(int H, int dtype, const void* R, int64_t nR, const void* C, int64_t nC, const Plan& p,
                    float c2, const float* lse2, const Ws& w, int n_dmax, hipStream_t s, const Skip& sk = Skip{}) {
  switch (H) {
    case 32: return launch_engine<MODE, 32>(dtype, R, nR, C, nC, p, c2, lse2, w, n_dmax, s, sk);
    case 64: return launch_engine<MODE, 64>(dtype, R, nR, C, nC, p, c2, lse2, w, n_dmax, s, sk);
    case 128: return launch_engine<MODE, 128>(dtype, R, nR, C, nC, p, c2, lse2, w, n_dmax, s, sk);
    case 256: return launch_engine<MODE, 256>(dtype, R, nR, C, nC, p, c2, lse2, w, n_dmax, s, sk);
    default: set_error("in-batch scorer: H=%d unsupported (32, 64, 128, 256)", H); return TT_ERR_UNSUPPORTED;
  }
}

int check_args(int64_t B, int64_t M, int H, int dtype, int64_t label_off) {
  TT_REQUIRE(B > 0 && M > 0, "B=%lld M=%lld must be positive", (long long)B, (long long)M);
  TT_REQUIRE(H == 32 || H == 64 || H == 128 || H == 256, "H=%d unsupported (32, 64, 128, 256)", H);
  TT_REQUIRE(dtype == TT_F32 || dtype == TT_BF16 || dtype == TT_BF16_SPLIT, "dtype=%d", dtype);
  TT_REQUIRE(label_off >= 0 && label_off + B <= M, "labels [%lld, %lld) fall outside the %lld candidate columns",
             (long long)label_off, (long long)(label_off + B), (long long)M);
  return TT_OK;
}

Ws carve_user(void* ws, int64_t B, int64_t M, int H, int dtype) {
  void* base = reinterpret_cast<void*>(align_up(reinterpret_cast<size_t>(ws), 256));
  return carve(base, B, M, H, dtype);
}

}  // namespace
}  // namespace tt

using namespace tt;

extern "C" int tt_inbatch_set_backward(int mode) {
  if (mode != TT_INBATCH_BWD_RECOMPUTE && mode != TT_INBATCH_BWD_STORED) return bwd_mode().load();
  return bwd_mode().exchange(mode);
}

extern "C" size_t tt_inbatch_ws_size(int64_t B, int64_t M, int H, int dtype) {
  return carve(nullptr, B, M, H, dtype).total + 256;
}

namespace tt {
namespace {

// Forward from prepared operands: Rm = candidates (M rows; bf16 copies carry the zero tail),
// Cm = queries (B rows), qnorm (B), dmax_part (n_dmax per-block maxima of the candidate norms).
// Writes lse, lse2 (log2 units, B), loss_rows, the mean loss and (want_grad) dq_unscaled.
int fwd_core(int dtype, const void* Rm, int64_t M, const void* Cm, int64_t B, int H, const float* qnorm,
             const float* dmax_part, int n_dmax, float inv_tau, int64_t label_off, float* lse, float* lse2,
             float* loss_rows, float* loss, float* dqu, const char* pad, float* l_part, float* acc_part,
             hipStream_t s, char* P = nullptr, int64_t p_nqt = 0, __bf16* Qs = nullptr, int* xrows = nullptr,
             float* Qs32 = nullptr, const __bf16* Dp = nullptr, __bf16* Qsp = nullptr) {
  const Plan p = plan_for(M, B, bj_for(dtype), Dp ? 1 : wg_per_cu(H, dtype, FWD));
  const float c2 = inv_tau * kLog2e;
  Ws w{};
  w.qnorm = const_cast<float*>(qnorm);
  w.dmax_part = const_cast<float*>(dmax_part);
  w.pad = const_cast<char*>(pad);
  w.l_part = l_part;
  w.acc_part = acc_part;
  w.P = P;
  w.p_nqt = p_nqt;
  w.Dp = const_cast<__bf16*>(Dp);
  // the stored-P engines (bf16, split-bf16) fold dmax once into the slot after the block maxima
  // (carve reserves it); the combine then reads that one float
  w.dmax_fold = P && (dtype == TT_BF16 || Dp) ? const_cast<float*>(dmax_part) + kMaxPrepBlocks : nullptr;
  int rc;
  if ((rc = dispatch_engine<FWD>(H, dtype, Rm, M, Cm, B, p, c2, nullptr, w, n_dmax, s))) return rc;
  const dim3 grid((unsigned)((B + (Qs || Qs32 || Qsp ? kTailRows : 0) + 3) / 4)), block(256);
  if (dtype == TT_F32)
    fwd_combine_kernel<float><<<grid, block, 0, s>>>(B, M, H, p.S, p.n_pad, c2, qnorm, dmax_part, n_dmax, l_part,
                                                    acc_part, inv_tau, label_off, static_cast<const float*>(Cm),
                                                    static_cast<const float*>(Rm), lse, lse2, loss_rows, dqu, Qs32,
                                                    Qs32 || Qsp ? xrows : nullptr, 0, nullptr, 0, Qsp, w.dmax_fold);
  else
    fwd_combine_kernel<__bf16><<<grid, block, 0, s>>>(B, M, H, p.S, p.n_pad, c2, qnorm, dmax_part, n_dmax, l_part,
                                                     acc_part, inv_tau, label_off, static_cast<const __bf16*>(Cm),
                                                     static_cast<const __bf16*>(Rm), lse, lse2, loss_rows, dqu, Qs,
                                                     xrows, 0, nullptr, 0, nullptr, w.dmax_fold);
  TT_LAUNCH_CHECK("score_fwd_combine");
  return loss ? launch_mean(loss_rows, B, loss, s) : TT_OK;
}

// Backward from prepared operands: Rm = queries (nQ rows + zero tail for bf16), lse2_R (nQ rows
// + a +inf tail), Cm = candidates (M rows).  The label of candidate j is query row q_label of
// Qlab (j - label_off in [0, B)); dq = scale * dq_unscaled (B rows).
int bwd_core(int dtype, const void* Rm, int64_t nQ, const float* lse2_R, const void* Cm, int64_t M, const void* Qlab,
             int64_t B, int64_t label_off, int H, float inv_tau, const float* dqu, const float* grad_loss,
             float grad_scale, const BwdOut& out, const char* pad, float* acc_part, hipStream_t s) {
  const Plan p = plan_for(nQ, M, bj_for(dtype), wg_per_cu(H, dtype, DD));
  const float c2 = inv_tau * kLog2e;
  Ws w{};
  w.pad = const_cast<char*>(pad);
  w.acc_part = acc_part;
  int rc;
  if ((rc = dispatch_engine<DD>(H, dtype, Rm, nQ, Cm, M, p, c2, lse2_R, w, 0, s))) return rc;
  if (dtype == TT_F32)
    launch_bwd_combine<float>(B, M, H, p.S, label_off, acc_part, static_cast<const float*>(Qlab), dqu, grad_loss,
                              grad_scale, inv_tau, out, nullptr, nullptr, nullptr, s);
  else
    launch_bwd_combine<__bf16>(B, M, H, p.S, label_off, acc_part, static_cast<const __bf16*>(Qlab), dqu, grad_loss,
                               grad_scale, inv_tau, out, nullptr, nullptr, nullptr, s);
  TT_LAUNCH_CHECK("score_bwd_combine");
  return TT_OK;
}

// Backward from the forward's stored probabilities (bf16): score_ddp_kernel over Qs (B rows +
// zero tail) and P, then the same combine (label terms from the unscaled q~).
int bwd_core_p(int64_t B, int64_t M, int H, int64_t label_off, float inv_tau, const __bf16* Qs, const char* P,
               int64_t p_nqt, const __bf16* Qlab, const float* dqu, const float* grad_loss, float grad_scale,
               const BwdOut& out, float* acc_part, const int* xrows, const __bf16* Db, const float* lse2,
               hipStream_t s) {
  const Plan p = ddp_plan(B, M, H);
  switch (H) {
#define TT_DDP(HH, CW)                                                                                               \
  case HH:                                                                                                           \
    score_ddp_kernel<HH, CW><<<dim3(p.grid), dim3(NT), Tile<__bf16, HH>::LDS_BYTES, s>>>(                           \
        Qs, B, M, p.S, p.rows_per_split, P, p_nqt, acc_part);                                                        \
    break;
    TT_DDP(32, 1)
    TT_DDP(64, 1)
    TT_DDP(128, 1)
    TT_DDP(256, TT_DDP_CW256)
#undef TT_DDP
    default: set_error("in-batch scorer: H=%d unsupported (32, 64, 128, 256)", H); return TT_ERR_UNSUPPORTED;
  }
  TT_LAUNCH_CHECK("score_ddp");
  launch_bwd_combine<__bf16>(B, M, H, p.S, label_off, acc_part, Qlab, dqu, grad_loss, grad_scale, inv_tau, out, xrows,
                             Db, lse2, s);
  TT_LAUNCH_CHECK("score_bwd_combine");
  return TT_OK;
}

// Backward from the forward's stored fp32 probabilities: score_f32_kernel<DD, H, true> over Qs32
// (q scaled by 2^(shift - lse2) in fp32) and P, then the fp32 combine (label terms from q, the
// exact rows from q, d and lse2).
int bwd_core_p32(int64_t B, int64_t M, int H, int64_t label_off, float inv_tau, const float* Qs32, const __bf16* Qsp,
                 const char* P, int64_t p_nqt, const float* q, const float* d, const float* dqu, const float* grad_loss,
                 float grad_scale, const BwdOut& out, const char* pad, float* acc_part, const int* xrows,
                 const float* lse2, hipStream_t s) {
  const Plan p = plan_for(B, M, bj_for(TT_F32), Qsp ? 1 : f32_waves(DD, H, true));
  float* Pf = reinterpret_cast<float*>(const_cast<char*>(P));
  const int64_t plane = (B + kTailRows) * H;
  switch (Qsp ? H : -H) {
#define TT_SPLIT_DDP(HH)                                                                                           \
  case HH:                                                                                                         \
    score_split_ddp_kernel<HH><<<dim3(p.grid), dim3(NT), SplitTile<HH>::LDS_BYTES, s>>>(                            \
        Qsp, plane, B, M, p.S, p.rows_per_split, Pf, p_nqt, acc_part);                                              \
    break;
    TT_SPLIT_DDP(64)
    TT_SPLIT_DDP(128)
    TT_SPLIT_DDP(256)
#undef TT_SPLIT_DDP
    case -32:  // H = 32: score_f32_kernel's stored-P backward (split_f32)
      score_f32_kernel<DD, 32, true><<<dim3(p.grid), dim3(NT), Tile<float, 32>::LDS_BYTES, s>>>(
          Qs32, B, d, M, p.S, p.rows_per_split, 0.f, lse2, nullptr, nullptr, 0, pad, acc_part, nullptr, Pf, p_nqt);
      break;
    default: set_error("in-batch scorer: fp32 stored-P backward at H=%d", H); return TT_ERR_UNSUPPORTED;
  }
  TT_LAUNCH_CHECK("score_dd_p32");
  launch_bwd_combine<float>(B, M, H, p.S, label_off, acc_part, q, dqu, grad_loss, grad_scale, inv_tau, out, xrows, d,
                            lse2, s);
  TT_LAUNCH_CHECK("score_bwd_combine");
  return TT_OK;
}

int launch_prep_rows(const float* x, int64_t rows, int H, __bf16* xb, float* norms, float* max_parts,
                     hipStream_t s) {
  const int g = (int)std::max<int64_t>(1, std::min<int64_t>((rows + 3) / 4, kMaxPrepBlocks));
  if (max_parts && g < kMaxPrepBlocks) TT_HIP(hipMemsetAsync(max_parts + g, 0, (kMaxPrepBlocks - g) * 4, s), "memset max_parts");
  prep_rows_kernel<<<dim3((unsigned)g), dim3(256), 0, s>>>(x, rows, H, xb, norms, max_parts);
  TT_LAUNCH_CHECK("score_prep_rows");
  return TT_OK;
}

// partial buffers of the explicit-operand passes
struct ExWs {
  float* l_part;
  float* acc_part;
  size_t total;
};
// The local launch of the two-launch data-parallel forward runs beside the candidate all-gather,
// whose kernels hold CUs of their own: its one-round grid is sized for 3/4 of the chip, so no
// workgroup waits for the collective to finish.
constexpr int kLocalCus = 192;
Plan plan_local(int64_t B, int64_t M, int H, int dtype) {
  return plan_for(M, B, bj_for(dtype), wg_per_cu(H, dtype, FWD), 32 * NW, kLocalCus);
}
// split slots of the two-launch data-parallel forward (fwd_ex_local + fwd_ex_remote)
int split_fwd_slots(int64_t B, int64_t M, int64_t M_all, int H, int dtype) {
  if (M_all <= M || M % bj_for(dtype) != 0) return 0;  // no two-launch forward for this shape
  return plan_local(B, M, H, dtype).S + plan_for(M_all - M, B, bj_for(dtype), wg_per_cu(H, dtype, FWD)).S;
}

ExWs carve_ex(void* base, int64_t B, int64_t M_all, int64_t nQ_all, int64_t M, int H, int dtype) {
  const int BJ = bj_for(dtype);
  const Plan pf = plan_for(M_all, B, BJ, wg_per_cu(H, dtype, FWD)), pd = plan_for(nQ_all, M, BJ, wg_per_cu(H, dtype, DD));
  const int64_t sf = std::max<int64_t>(pf.S, split_fwd_slots(B, M, M_all, H, dtype));
  const size_t ol = 0;
  const size_t oa = align_up((size_t)sf * B * 4, 256);
  const size_t parts = std::max((size_t)sf * B, (size_t)pd.S * M) * H * 4;
  ExWs w{};
  if (base) {
    char* b = reinterpret_cast<char*>(align_up(reinterpret_cast<size_t>(base), 256));
    w.l_part = reinterpret_cast<float*>(b + ol);
    w.acc_part = reinterpret_cast<float*>(b + oa);
  }
  w.total = oa + parts + 256;
  return w;
}

}  // namespace
}  // namespace tt

namespace tt {
namespace {
int prep_blocks_q(int64_t B) { return (int)std::min<int64_t>((B + 3) / 4, 512); }
int prep_blocks_d(int64_t M) { return (int)std::min<int64_t>((M + 3) / 4, kMaxPrepBlocks); }

int inbatch_fwd(const float* q, const float* d, int64_t B, int64_t M, int H, int dtype, float inv_tau,
                int64_t label_off, int want_grad, float* lse, float* loss_rows, float* loss, float* dq_unscaled,
                void* ws, size_t ws_bytes, hipStream_t s, bool prepped) {
  int rc = check_args(B, M, H, dtype, label_off);
  if (rc) return rc;
  TT_REQUIRE(q && d && lse && loss_rows && ws, "null pointer");  // loss NULL: the caller forms the mean (tt_mean)
  TT_REQUIRE(!want_grad || dq_unscaled, "want_grad needs dq_unscaled");
  TT_REQUIRE(((reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(d)) & 15) == 0, "q/d must be 16-byte aligned");
  TT_REQUIRE(!prepped || dtype != TT_F32 || H == 2 * kWave, "prepared fp32 operands: H = 128 (tt_inbatch_l2_prep)");
  const Ws w = carve_user(ws, B, M, H, dtype);
  TT_REQUIRE(w.total + 256 <= ws_bytes, "workspace too small: need %zu have %zu", w.total + 256, ws_bytes);
  const bool bf = dtype != TT_F32;
  const int gd = prep_blocks_d(M);
  if (!prepped) {
    const int gq = prep_blocks_q(B);
    prep_qd_kernel<<<dim3((unsigned)(gq + gd)), dim3(256), 0, s>>>(q, B, d, M, H, gq, bf ? w.Qb : nullptr,
                                                                   bf ? w.Db : nullptr, w.qnorm, w.dmax_part, w.pad,
                                                                   w.lse2, w.xrows, w.Dp);
    TT_LAUNCH_CHECK("score_prep");
  }
  const void* Rm = bf ? (const void*)w.Db : (const void*)d;
  const void* Cm = bf ? (const void*)w.Qb : (const void*)q;
  const bool sp = want_grad && w.P;
  return fwd_core(dtype, Rm, M, Cm, B, H, w.qnorm, w.dmax_part, gd, inv_tau, label_off, lse, w.lse2, loss_rows, loss,
                  want_grad ? dq_unscaled : nullptr, w.pad, w.l_part, w.acc_part, s, sp ? w.P : nullptr, w.p_nqt,
                  sp ? w.Qs : nullptr, sp ? w.xrows : nullptr, sp ? w.Qs32 : nullptr, sp ? w.Dp : nullptr,
                  sp ? w.Qsp : nullptr);
}
}  // namespace
}  // namespace tt

extern "C" int tt_inbatch_fwd(const float* q, const float* d, int64_t B, int64_t M, int H, int dtype, float inv_tau,
                              int64_t label_off, int want_grad, float* lse, float* loss_rows, float* loss,
                              float* dq_unscaled, void* ws, size_t ws_bytes, tt_stream_t stream) {
  return inbatch_fwd(q, d, B, M, H, dtype, inv_tau, label_off, want_grad, lse, loss_rows, loss, dq_unscaled, ws,
                     ws_bytes, reinterpret_cast<hipStream_t>(stream), false);
}

extern "C" int tt_inbatch_l2_prep(float* y, int64_t B, int64_t M, int H, int dtype, float* norms, void* ws,
                                  size_t ws_bytes, tt_stream_t stream) {
  TT_REQUIRE(B > 0 && M > 0, "B=%lld M=%lld must be positive", (long long)B, (long long)M);
  TT_REQUIRE((H == 4 * kWave && (dtype == TT_BF16 || dtype == TT_BF16_SPLIT)) || (H == 2 * kWave && dtype == TT_F32),
             "tt_inbatch_l2_prep: H = 256 with bf16 / bf16_split or H = 128 with fp32 (got H=%d dtype=%d)", H, dtype);
  TT_REQUIRE(y && norms && ws, "null pointer");
  TT_REQUIRE((reinterpret_cast<uintptr_t>(y) & 15) == 0, "y must be 16-byte aligned");
  const Ws w = carve_user(ws, B, M, H, dtype);
  TT_REQUIRE(w.total + 256 <= ws_bytes, "workspace too small: need %zu have %zu", w.total + 256, ws_bytes);
  const int gq = prep_blocks_q(B), gd = prep_blocks_d(M);
  if (dtype == TT_F32) {
    l2_prep128_kernel<<<dim3((unsigned)(gq + gd)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream)>>>(
        y, B, M, gq, norms, w.qnorm, w.dmax_part, w.pad, w.lse2, w.xrows, w.Dp);
    TT_LAUNCH_CHECK("score_l2_prep128");
    return TT_OK;
  }
  l2_prep_kernel<<<dim3((unsigned)(gq + gd)), dim3(64 * kL2PrepWaves), 0, reinterpret_cast<hipStream_t>(stream)>>>(
      y, B, M, gq, norms, w.Qb, w.Db, w.qnorm, w.dmax_part, w.pad, w.lse2, w.xrows);
  TT_LAUNCH_CHECK("score_l2_prep");
  return TT_OK;
}

extern "C" int tt_inbatch_fwd_prepped(const float* q, const float* d, int64_t B, int64_t M, int H, int dtype,
                                      float inv_tau, int64_t label_off, int want_grad, float* lse, float* loss_rows,
                                      float* loss, float* dq_unscaled, void* ws, size_t ws_bytes,
                                      tt_stream_t stream) {
  return inbatch_fwd(q, d, B, M, H, dtype, inv_tau, label_off, want_grad, lse, loss_rows, loss, dq_unscaled, ws,
                     ws_bytes, reinterpret_cast<hipStream_t>(stream), true);
}

namespace tt {
namespace {
int inbatch_bwd(const float* q, const float* d, int64_t B, int64_t M, int H, int dtype, float inv_tau,
                int64_t label_off, const float* dq_unscaled, const float* grad_loss, float grad_scale,
                const BwdOut& out, void* ws, size_t ws_bytes, hipStream_t s) {
  const Ws w = carve_user(ws, B, M, H, dtype);
  TT_REQUIRE(w.total + 256 <= ws_bytes, "workspace too small: need %zu have %zu", w.total + 256, ws_bytes);
  const bool bf = dtype != TT_F32;
  // lse in log2 units (ws.lse2) and the pad rows were left in the workspace by the forward
  const void* Rm = bf ? (const void*)w.Qb : (const void*)q;  // operands left by the forward
  const void* Cm = bf ? (const void*)w.Db : (const void*)d;
  if (w.P && !bf)
    return bwd_core_p32(B, M, H, label_off, inv_tau, w.Qs32, w.Qsp, w.P, w.p_nqt, q, d, dq_unscaled, grad_loss, grad_scale,
                        out, w.pad, w.acc_part, w.xrows, w.lse2, s);
  if (w.P) return bwd_core_p(B, M, H, label_off, inv_tau, w.Qs, w.P, w.p_nqt, w.Qb, dq_unscaled, grad_loss, grad_scale,
                             out, w.acc_part, w.xrows, w.Db, w.lse2, s);
  return bwd_core(dtype, Rm, B, w.lse2, Cm, M, Rm, B, label_off, H, inv_tau, dq_unscaled, grad_loss, grad_scale, out,
                  w.pad, w.acc_part, s);
}
}  // namespace
}  // namespace tt

extern "C" int tt_inbatch_bwd_l2(const float* qd, int64_t B, int64_t M, int H, int dtype, float inv_tau,
                                      int64_t label_off, const float* lse, const float* dq_unscaled,
                                      const float* grad_loss, float grad_scale, const float* norms, float* dx,
                                      const float* loss_rows, float* loss, void* ws, size_t ws_bytes,
                                      tt_stream_t stream) {
  int rc = check_args(B, M, H, dtype, label_off);
  if (rc) return rc;
  TT_REQUIRE((H == 4 * kWave && dtype != TT_F32) || (H == 2 * kWave && dtype == TT_F32),
             "tt_inbatch_bwd_l2: H = 256 with bf16 operands or H = 128 fp32 (H=%d dtype=%d)", H, dtype);
  TT_REQUIRE(qd && lse && dq_unscaled && grad_loss && norms && dx && ws, "null pointer");
  TT_REQUIRE(!loss == !loss_rows, "tt_inbatch_bwd_l2: loss and loss_rows together");
  BwdOut out{nullptr, nullptr, qd, norms, dx, loss_rows, loss};
  return inbatch_bwd(qd, qd + B * H, B, M, H, dtype, inv_tau, label_off, dq_unscaled, grad_loss, grad_scale, out, ws,
                     ws_bytes, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int tt_inbatch_bwd(const float* q, const float* d, int64_t B, int64_t M, int H, int dtype,
                                   float inv_tau, int64_t label_off, const float* lse, const float* dq_unscaled,
                                   const float* grad_loss, float grad_scale, float* dq, float* dd,
                                   const float* loss_rows, float* loss, void* ws, size_t ws_bytes, tt_stream_t stream) {
  int rc = check_args(B, M, H, dtype, label_off);
  if (rc) return rc;
  TT_REQUIRE(q && d && lse && dq_unscaled && grad_loss && dq && dd && ws, "null pointer");
  TT_REQUIRE(!loss == !loss_rows, "tt_inbatch_bwd: loss and loss_rows together");
  BwdOut out{dq, dd};
  out.loss_rows = loss_rows;
  out.loss = loss;
  return inbatch_bwd(q, d, B, M, H, dtype, inv_tau, label_off, dq_unscaled, grad_loss, grad_scale, out, ws, ws_bytes,
                     reinterpret_cast<hipStream_t>(stream));
}

// ---- explicit operands (data parallel with candidate-owner gradients; see twotower_amd.h)
extern "C" int tt_inbatch_prep_rows(const float* x, int64_t rows, int H, void* xb, float* norms, float* max_parts,
                                    tt_stream_t stream) {
  TT_REQUIRE(x && rows >= 0, "bad rows/pointer");
  TT_REQUIRE(H % 4 == 0 && H >= 4, "H=%d must be a positive multiple of 4", H);
  TT_REQUIRE((reinterpret_cast<uintptr_t>(x) & 15) == 0, "x must be 16-byte aligned");
  if (rows == 0 && !max_parts && !xb) return TT_OK;
  return launch_prep_rows(x, rows, H, static_cast<__bf16*>(xb), norms, max_parts,
                          reinterpret_cast<hipStream_t>(stream));
}

extern "C" size_t tt_inbatch_ex_ws_size(int64_t B, int64_t M_all, int64_t nQ_all, int64_t M, int H, int dtype) {
  return carve_ex(nullptr, B, M_all, nQ_all, M, H, dtype).total;
}

extern "C" int tt_inbatch_fwd_ex(const void* Qb, const float* qnorm, int64_t B, const void* Db_all,
                                 const float* dmax_parts, int n_parts, int64_t M_all, int H, int dtype, float inv_tau,
                                 int64_t label_off, int want_grad, float* lse, float* lse2, float* loss_rows,
                                 float* loss, float* dq_unscaled, void* ws, size_t ws_bytes, tt_stream_t stream) {
  int rc = check_args(B, M_all, H, dtype, label_off);
  if (rc) return rc;
  TT_REQUIRE(dtype != TT_F32, "explicit-operand passes take bf16 operand copies (dtype bf16 / bf16_split)");
  TT_REQUIRE(Qb && qnorm && Db_all && dmax_parts && lse && lse2 && loss_rows && loss && ws, "null pointer");
  TT_REQUIRE(n_parts > 0, "n_parts=%d", n_parts);
  TT_REQUIRE(!want_grad || dq_unscaled, "want_grad needs dq_unscaled");
  const size_t need = tt_inbatch_ex_ws_size(B, M_all, B, 1, H, dtype);
  TT_REQUIRE(need <= ws_bytes, "workspace too small: need %zu have %zu", need, ws_bytes);
  const ExWs w = carve_ex(ws, B, M_all, B, 1, H, dtype);
  return fwd_core(dtype, Db_all, M_all, Qb, B, H, qnorm, dmax_parts, n_parts, inv_tau, label_off, lse, lse2,
                  loss_rows, loss, want_grad ? dq_unscaled : nullptr, nullptr, w.l_part, w.acc_part,
                  reinterpret_cast<hipStream_t>(stream));
}

// Data-parallel forward in two launches, so the candidate all-gather overlaps the scoring of the
// rank's own candidates.  local: the engine over Db_loc (M rows + zero tail; this rank's own
// candidates, global rows [own_begin, own_begin + M) of Db_all) with the local norm bound, into
// partial slots [0, S_loc).  remote: the engine over Db_all's other M_all - M rows (the own block
// skipped) with the global bound, into the next S_rem slots; then the combine over all slots, the
// local ones rescaled by 2^(shift_loc - shift), and the mean.  Same result as tt_inbatch_fwd_ex on
// Db_all within fp32 rounding.
namespace tt {
namespace {
int check_split_fwd(int64_t B, int64_t M, int64_t M_all, int64_t own_begin, int H, int dtype) {
  int rc = check_args(B, M_all, H, dtype, own_begin);
  if (rc) return rc;
  TT_REQUIRE(dtype != TT_F32, "explicit-operand passes take bf16 operand copies (dtype bf16 / bf16_split)");
  const int BJ = bj_for(dtype);
  TT_REQUIRE(M > 0 && M_all > M && M % BJ == 0 && own_begin % BJ == 0 && own_begin + M <= M_all,
             "split forward: M=%lld own_begin=%lld must be multiples of %d inside M_all=%lld", (long long)M,
             (long long)own_begin, BJ, (long long)M_all);
  return TT_OK;
}
}  // namespace
}  // namespace tt

extern "C" int tt_inbatch_fwd_ex_local(const void* Qb, const float* qnorm, int64_t B, const void* Db_loc,
                                       const float* dmax_loc, int n_loc, int64_t M, int64_t M_all, int64_t own_begin,
                                       int H, int dtype, float inv_tau, void* ws, size_t ws_bytes,
                                       tt_stream_t stream) {
  int rc = check_split_fwd(B, M, M_all, own_begin, H, dtype);
  if (rc) return rc;
  TT_REQUIRE(Qb && qnorm && Db_loc && dmax_loc && ws && n_loc > 0, "null pointer / n_loc");
  const size_t need = tt_inbatch_ex_ws_size(B, M_all, B, M, H, dtype);
  TT_REQUIRE(need <= ws_bytes, "workspace too small: need %zu have %zu", need, ws_bytes);
  const ExWs w = carve_ex(ws, B, M_all, B, M, H, dtype);
  Ws e{};
  e.qnorm = const_cast<float*>(qnorm);
  e.dmax_part = const_cast<float*>(dmax_loc);
  e.l_part = w.l_part;
  e.acc_part = w.acc_part;
  const Plan p = plan_local(B, M, H, dtype);
  return dispatch_engine<FWD>(H, dtype, Db_loc, M, Qb, B, p, inv_tau * kLog2e, nullptr, e, n_loc,
                              reinterpret_cast<hipStream_t>(stream));
}

extern "C" int tt_inbatch_fwd_ex_remote(const void* Qb, const float* qnorm, int64_t B, const void* Db_all,
                                        const float* dmax_parts, int n_parts, const float* dmax_loc, int n_loc,
                                        int64_t M, int64_t M_all, int64_t own_begin, int H, int dtype, float inv_tau,
                                        int want_grad, float* lse, float* lse2, float* loss_rows, float* loss,
                                        float* dq_unscaled, void* ws, size_t ws_bytes, tt_stream_t stream) {
  int rc = check_split_fwd(B, M, M_all, own_begin, H, dtype);
  if (rc) return rc;
  TT_REQUIRE(Qb && qnorm && Db_all && dmax_parts && dmax_loc && lse && lse2 && loss_rows && loss && ws, "null pointer");
  TT_REQUIRE(n_parts > 0 && n_loc > 0, "n_parts=%d n_loc=%d", n_parts, n_loc);
  TT_REQUIRE(!want_grad || dq_unscaled, "want_grad needs dq_unscaled");
  const size_t need = tt_inbatch_ex_ws_size(B, M_all, B, M, H, dtype);
  TT_REQUIRE(need <= ws_bytes, "workspace too small: need %zu have %zu", need, ws_bytes);
  const ExWs w = carve_ex(ws, B, M_all, B, M, H, dtype);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int BJ = bj_for(dtype);
  const Plan pl = plan_local(B, M, H, dtype), pr = plan_for(M_all - M, B, BJ, wg_per_cu(H, dtype, FWD));
  const float c2 = inv_tau * kLog2e;
  Ws e{};
  e.qnorm = const_cast<float*>(qnorm);
  e.dmax_part = const_cast<float*>(dmax_parts);
  e.l_part = w.l_part;
  e.acc_part = w.acc_part;
  Skip sk;
  sk.begin = own_begin;
  sk.len = M;
  sk.split_base = pl.S;
  if ((rc = dispatch_engine<FWD>(H, dtype, Db_all, M_all - M, Qb, B, pr, c2, nullptr, e, n_parts, s, sk))) return rc;
  const int S = pl.S + pr.S;
  const dim3 grid((unsigned)((B + 3) / 4)), block(256);
  fwd_combine_kernel<__bf16><<<grid, block, 0, s>>>(
      B, M_all, H, S, pl.n_pad + pr.n_pad, c2, qnorm, dmax_parts, n_parts, w.l_part, w.acc_part, inv_tau, own_begin,
      static_cast<const __bf16*>(Qb), static_cast<const __bf16*>(Db_all), lse, lse2, loss_rows,
      want_grad ? dq_unscaled : nullptr, nullptr, nullptr, pl.S, dmax_loc, n_loc);
  TT_LAUNCH_CHECK("score_fwd_combine (split)");
  return launch_mean(loss_rows, B, loss, s);
}

extern "C" int tt_inbatch_bwd_ex(const void* Qb_all, const float* lse2_all, int64_t nQ_all, int64_t q_row0,
                                 const void* Db, int64_t M, int64_t B, int64_t label_off, int H, int dtype,
                                 float inv_tau, const float* dq_unscaled, const float* grad_loss, float grad_scale,
                                 float* dq, float* dd, void* ws, size_t ws_bytes, tt_stream_t stream) {
  int rc = check_args(B, M, H, dtype, label_off);
  if (rc) return rc;
  TT_REQUIRE(dtype != TT_F32, "explicit-operand passes take bf16 operand copies (dtype bf16 / bf16_split)");
  TT_REQUIRE(Qb_all && lse2_all && Db && dq_unscaled && grad_loss && dq && dd && ws, "null pointer");
  TT_REQUIRE(q_row0 >= 0 && q_row0 + B <= nQ_all, "query rows [%lld, %lld) outside the %lld gathered rows",
             (long long)q_row0, (long long)(q_row0 + B), (long long)nQ_all);
  const size_t need = tt_inbatch_ex_ws_size(1, 1, nQ_all, M, H, dtype);
  TT_REQUIRE(need <= ws_bytes, "workspace too small: need %zu have %zu", need, ws_bytes);
  const ExWs w = carve_ex(ws, 1, 1, nQ_all, M, H, dtype);
  const void* Qlab = static_cast<const __bf16*>(Qb_all) + q_row0 * H;
  return bwd_core(dtype, Qb_all, nQ_all, lse2_all, Db, M, Qlab, B, label_off, H, inv_tau, dq_unscaled, grad_loss,
                  grad_scale, BwdOut{dq, dd}, nullptr, w.acc_part, reinterpret_cast<hipStream_t>(stream));
}

#ifdef TT_SCORER_TRACE
extern "C" int tt_debug_scorer_trace(long long* host_out) {
  return (int)hipMemcpyFromSymbol(host_out, HIP_SYMBOL(tt::g_tt_trace), sizeof(long long) * 8 * 64);
}
extern "C" int tt_debug_scorer_ktrace(long long* host_out) {
  return (int)hipMemcpyFromSymbol(host_out, HIP_SYMBOL(tt::g_tt_ktrace), sizeof(long long) * 2 * 1024 * 4);
}
extern "C" int tt_debug_scorer_trace_bwd(long long* host_out) {
  return (int)hipMemcpyFromSymbol(host_out, HIP_SYMBOL(tt::g_tt_trace_b), sizeof(long long) * 8 * 64);
}
#endif
