// Tower head as two fused GEMM chains on gfx950 (MeanPoolingTower, twotower/encoders.py:38-42,77):
//   forward   h = relu(x W1^T + b1) (stored, with its ReLU bits), y = h W2^T + b2, out = y / max(|y|, 1e-12)
//   backward  dh = (dy W2) * relu'(h) (stored, for dW1), dx = dh W1 (optionally / the bag denominators)
// in ONE launch each: a wave owns 32 whole rows, the first product's 32 x R1 result stays in its
// registers and is the second product's operand, so h (dh) never makes an HBM round trip, the two
// launches of each pass become one, and the F.normalize epilogue has whole rows in the wave.
//
// fp32 accuracy on the bf16 MFMA as in head.hip: each fp32 operand is split into three bf16 terms and
// the six cross products of order >= 2^-16 are accumulated in fp32, smallest first.
//
// Layout of the work.  The first product is computed TRANSPOSED, h^T = W1 x^T: the W1 planes are the
// A operand (rows = hidden units) and the x rows the B operand (lane = row, 8 consecutive k), so in
// the 32 x 32 accumulator a lane holds one ROW and 16 hidden units (4 consecutive per group g = 0..3,
// 8 apart).  One half-wave exchange per register pair (groups 2s, 2s + 1; a ds_bpermute) turns that
// into the A operand layout of the second product (lane = row, 8 consecutive hidden units per k-half): the
// second product y = h W2^T is then an ordinary A x B^T with the W2 planes as B, whose accumulator
// (lane = output column, 16 rows) stores whole 128-B row segments.  The products are the ones
// head.hip's kernels form, operand for operand, so h, dh and the unnormalised y equal theirs.
//
// Weights: the planes stream through a 3-slot LDS ring in 16-k chunks ([plane][row][32 B], lane
// (row r, half hh) reads 16 B at 32 r + 16 (hh ^ bit 3 of r): one 1 KiB per wave-instruction), filled by
// LDS-DMA two chunks ahead, one barrier per chunk; the four waves (128 rows) share each chunk.  A
// workgroup walks row blocks b, b + grid, ... and the ring continues across them; the next block's
// B-operand rows (x or dy) ride in the same chunks (their 16 k of the block's 128 rows), so the next
// block's first chunks arrive while the current block's second product runs.
#include "common.hpp"

// Measured slower than head.hip's four launches (54.6 / 56.2 against 46.7 / 46.8 us per
// pass at 24,576 rows; one wave per SIMD serialises the split, the plane reads and the fills with the
// products), so ops.TowerHead runs it only under TT_HEAD_CHAIN=1.
//
// Timing ablations (tools/build_variants.sh; never in the shipped build): TT_CHAB_NOMFMA keeps the
// operand reads and drops the products, TT_CHAB_NOFILL drops the LDS-DMA pieces, TT_CHAB_NOBAR the
// chunk barriers, TT_CHAB_NOSTORE the h and y stores.  Their results are wrong by construction.
#ifdef TT_CHAB_NOMFMA
__device__ __forceinline__ tt::f32x16 tt_ch_nomfma(tt::bf16x8 a, tt::bf16x8 b, tt::f32x16 c) {
  asm volatile("" ::"v"(a), "v"(b));
  return c;
}
#define TT_CH_MFMA(a, b, c) tt_ch_nomfma((a), (b), (c))
#else
#define TT_CH_MFMA(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_bf16((a), (b), (c), 0, 0, 0)
#endif

namespace tt {
namespace {

constexpr int kCW = 4;       // waves per workgroup
constexpr int kCRows = 32;   // rows per wave
constexpr int kCSlots = 3;   // LDS ring slots

// MODE1: 0 forward first Linear (bias + ReLU, ReLU bits written, h stored)
//        1 backward dh GEMM (ReLU bits read, dh stored)
// MODE2: 0 bias (y unnormalised: the in-batch scorer's l2_prep normalises it)
//        1 bias + F.normalize (out, norms)
//        2 row divide (dx / the bag denominators, the division autograd applies at encoders.py:72)
//        3 plain (dx)
template <int K1, int R1, int R2, int MODE1, int MODE2>
__global__ __launch_bounds__(256, 1) void head_chain_kernel(
    const float* __restrict__ X, int64_t rows, int64_t ldx, const __bf16* __restrict__ P1,
    const __bf16* __restrict__ P2, const float* __restrict__ bias1, const float* __restrict__ bias2,
    unsigned* __restrict__ bits, float* __restrict__ Hout, float* __restrict__ Y, float* __restrict__ norms,
    int64_t nblk) {
  static_assert(K1 % 16 == 0 && R1 % 32 == 0 && R2 % 32 == 0, "chain shapes");
  constexpr int C1 = K1 / 16, C2 = R1 / 16, CT = C1 + C2;
  constexpr int NT1 = R1 / 32, NT2 = R2 / 32;
  constexpr int RMAX = R1 > R2 ? R1 : R2;
  constexpr int WB = 3 * RMAX * 32;                        // weight bytes of a ring slot
  constexpr int XB = kCW * kCRows * 64;                    // B-operand rows of a first-product chunk (8 KiB)
  constexpr int SLOT = WB + XB;
  constexpr int XP = XB / 1024;                            // its LDS-DMA pieces
  constexpr int WP1 = 3 * R1 / 32, WP2 = 3 * R2 / 32;       // plane pieces of a first / second chunk
  constexpr int WU1 = WP1 / kCW, XU = XP / kCW;             // ... per wave (first: plane, then row pieces)
  constexpr int F1 = WU1 + XU, F2 = (WP2 + kCW - 1) / kCW;  // LDS-DMA pieces per wave: first / second chunk
  static_assert(WP1 % kCW == 0 && XP % kCW == 0, "first-chunk pieces split evenly over the waves");
  constexpr int NW1 = (NT1 + 1) / 2;                       // ReLU words per lane and row tile
  constexpr int STG_ROW = R2 * 4 + 16;                     // MODE2 1 staging row (padded: no bank conflicts)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef __attribute__((address_space(3))) bf16x8 lds_bf16x8_t;
  typedef __attribute__((address_space(3))) f32x4 lds_f32x4_t;
  typedef __attribute__((address_space(3))) char lds_char_t;
  lds_char_t* lds = (lds_char_t*)smem;
  const int lane = lane_id(), r32 = lane & 31, hh = lane >> 5;
  const int wid0 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (scalar fill addressing)
  const int wid = wid0;
  const int nmine = (int)((nblk - (int64_t)blockIdx.x + gridDim.x - 1) / gridDim.x);
  if (nmine <= 0) return;  // workgroup-uniform
  const unsigned lds_base = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds);

  // Chunk cl of row block rb goes to ring slot `slot` (chunks are numbered continuously over this
  // workgroup's blocks, slot = number % 3).  Chunks [0, C1): the P1 planes' 16-k slice j = cl (32 B
  // per plane row) and the block's 128 B-operand rows at k 16 j .. 16 j + 15 (64 B per row); [C1, CT):
  // the P2 planes' slice cl - C1.  Swizzles (so the lanes of every ds_read_b128 quarter hit distinct
  // bank groups): the 16-B half s of plane row r sits at half s ^ ((r >> 3) & 1); the 16-B slot s of
  // B-operand row r at slot s ^ ((r >> 2) & 3).  LDS-DMA writes linearly (lane l: byte 16 l of the
  // piece), so the swizzle goes on the source.  Source offsets: a per-lane part (below) plus a
  // wave-uniform part per piece; the chunk's k offset goes on the scalar base.
  const int lw = lane >> 1;                                        // plane piece: row within 32
  const unsigned wsw = (unsigned)(((lane & 1) ^ ((lw >> 3) & 1)) * 16);
  const unsigned lw1 = (unsigned)(lw * K1 * 2) + wsw, lw2 = (unsigned)(lw * R1 * 2) + wsw;
  const int lx = lane >> 2;                                        // row piece: row within 16
  const unsigned lxs = (unsigned)(((lane & 3) ^ ((lx >> 2) & 3)) * 16);
  const unsigned ldx4 = (unsigned)(ldx * 4);
  auto issue = [&](unsigned off, const void* base, unsigned m0) {
#ifndef TT_CHAB_NOFILL
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(off), "s"(base), "s"(m0)
                 : "memory");
#endif
  };
  auto fill = [&](const int cl, const int64_t rb, const int slot) {
    const unsigned sbase = lds_base + (unsigned)(slot * SLOT);
    int wid = wid0;  // laundered: the pieces' wave-uniform offsets are recomputed per fill (a few
    asm volatile("" : "+s"(wid));  // SALU) rather than hoisted out of the block loop and spilled
    if (cl < C1) {
      const char* wb = reinterpret_cast<const char*>(P1) + cl * 32;
#pragma unroll
      for (int u = 0; u < WU1; ++u) {
        const int q = u * kCW + wid, pl = q / (R1 / 32), g = q % (R1 / 32);
        issue(lw1 + (unsigned)((pl * R1 + g * 32) * K1 * 2), wb, sbase + q * 1024);
      }
      const float* xb = X + rb * (kCW * kCRows) * ldx + cl * 16;
      const int64_t left = rows - 1 - rb * (kCW * kCRows);  // rows past the end read the last row
      const int lim = (int)(left < kCW * kCRows - 1 ? left : kCW * kCRows - 1);
#pragma unroll
      for (int u = 0; u < XU; ++u) {
        const int xq = u * kCW + wid, rl = min(xq * 16 + lx, lim);
        issue((unsigned)rl * ldx4 + lxs, xb, sbase + WB + xq * 1024);
      }
    } else {
      const char* wb = reinterpret_cast<const char*>(P2) + (cl - C1) * 32;
#pragma unroll
      for (int u = 0; u < F2; ++u) {
        const int q = min(u * kCW + wid, WP2 - 1), pl = q / (R2 / 32), g = q % (R2 / 32);
        issue(lw2 + (unsigned)((pl * R2 + g * 32) * R1 * 2), wb, sbase + q * 1024);
      }
    }
  };
  // the chunk two ahead of chunk cl of block rb (the next block's when it wraps; none past the last)
  // (the chunk number is laundered through an SGPR in the unrolled second product: with it a
  // compile-time constant the compiler hoists every chunk's addresses out of the block loop)
  auto fill_ahead = [&](int cl, const int bi, const int64_t rb, const int slot) {
    int nc = cl + 2;
    asm volatile("" : "+s"(nc));
    const int ns = slot + 2 >= kCSlots ? slot + 2 - kCSlots : slot + 2;
    if (nc < CT) {
      fill(nc, rb, ns);
    } else if (bi + 1 < nmine) {
      fill(nc - CT, rb + gridDim.x, ns);
    }
  };
  // chunk cl's pieces landed for every wave (this wave's: all but the pieces of chunk cl + 1 may be
  // outstanding, F1 or F2 of them, none after the last chunk), and every wave is done with the
  // previous chunk.  lgkmcnt(0): this wave's ring reads of that chunk have returned (the compiler
  // may sink the MFMAs that consume them, and their waits, below an asm barrier), so the fill two
  // ahead that some wave issues after the barrier cannot overwrite a slot still being read.
  auto arrive = [&](const int cl, const int bi) {
    const int nc = cl + 1;
    if (nc < C1 || (nc == CT && bi + 1 < nmine)) {
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(F1) : "memory");
    } else if (nc < CT) {
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(F2) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
#ifndef TT_CHAB_NOBAR
    asm volatile("s_barrier" ::: "memory");  // (not __syncthreads: its fence would drain the fills ahead)
#endif
  };

  fill(0, blockIdx.x, 0);
  if (CT > 1) fill(1, blockIdx.x, 1);

  int slot = 0;  // ring slot of the current chunk
  for (int bi = 0; bi < nmine; ++bi) {
    const int64_t rb = blockIdx.x + (int64_t)bi * gridDim.x;
    const int64_t r0 = rb * (kCW * kCRows) + wid * kCRows;  // this wave's first row
    f32x16 acc1[NT1];
#pragma unroll
    for (int t = 0; t < NT1; ++t) acc1[t] = f32x16{};
    // ---- first product, transposed: acc1[t] = (P1 rows 32 t .. 32 t + 31) x (this wave's rows)^T
    const int xr = wid * kCRows + r32;  // this lane's row in the block
#pragma unroll 1
    for (int j = 0; j < C1; ++j) {
      arrive(j, bi);
      fill_ahead(j, bi, rb, slot);
      const lds_char_t* sl = lds + slot * SLOT;
      const lds_char_t* ch = sl + r32 * 32 + (hh ^ ((r32 >> 3) & 1)) * 16;
      const lds_char_t* xrow = sl + WB + xr * 64;
      // the tile-0 weight operands and the rows first, then the split while they arrive; each tile's
      // operands are read one tile ahead into the other register set (no LDS round trip between tiles)
      bf16x8 w[2][3];
#pragma unroll
      for (int p = 0; p < 3; ++p) w[0][p] = *reinterpret_cast<const lds_bf16x8_t*>(ch + p * R1 * 32);
      const f32x4 xa = *reinterpret_cast<const lds_f32x4_t*>(xrow + (((2 * hh) ^ ((xr >> 2) & 3)) << 4));
      const f32x4 xb = *reinterpret_cast<const lds_f32x4_t*>(xrow + (((2 * hh + 1) ^ ((xr >> 2) & 3)) << 4));
      __bf16 x0[8], x1[8], x2[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) split3(i < 4 ? xa[i] : xb[i - 4], x0[i], x1[i], x2[i]);
      bf16x8 b0, b1, b2;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        b0[i] = x0[i];
        b1[i] = x1[i];
        b2[i] = x2[i];
      }
#pragma unroll
      for (int t = 0; t < NT1; ++t) {
        if (t + 1 < NT1) {
#pragma unroll
          for (int p = 0; p < 3; ++p)
            w[(t + 1) & 1][p] = *reinterpret_cast<const lds_bf16x8_t*>(ch + p * R1 * 32 + (t + 1) * 1024);
        }
        __builtin_amdgcn_sched_barrier(0);
        const bf16x8(&wt)[3] = w[t & 1];
        // head.hip's products with the operands in the other roles (x terms b, W terms w):
        // x2 W0, x1 W1, x0 W2, x1 W0, x0 W1, x0 W0
        acc1[t] = TT_CH_MFMA(wt[0], b2, acc1[t]);
        acc1[t] = TT_CH_MFMA(wt[1], b1, acc1[t]);
        acc1[t] = TT_CH_MFMA(wt[2], b0, acc1[t]);
        acc1[t] = TT_CH_MFMA(wt[0], b1, acc1[t]);
        acc1[t] = TT_CH_MFMA(wt[1], b0, acc1[t]);
        acc1[t] = TT_CH_MFMA(wt[0], b0, acc1[t]);
        __builtin_amdgcn_sched_barrier(0);
      }
      slot = slot + 1 == kCSlots ? 0 : slot + 1;
    }
    // ---- first epilogue: lane = row r0 + r32, acc1[t][v] = unit 32 t + (v & 3) + 8 (v >> 2) + 4 hh
    const int64_t row = r0 + r32;
    const bool row_ok = row < rows;
    unsigned* bw = bits + ((r0 / kCRows) * NW1) * 64 + lane;
    if constexpr (MODE1 == 0) {
      unsigned word[NW1];
#pragma unroll
      for (int w = 0; w < NW1; ++w) word[w] = 0;
#pragma unroll
      for (int t = 0; t < NT1; ++t) {
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const f32x4 bv = *reinterpret_cast<const f32x4*>(bias1 + 32 * t + 8 * gq + 4 * hh);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int v = 4 * gq + i;
            const float y = fmaxf(acc1[t][v] + bv[i], 0.f);  // head.hip EPI_BIAS_RELU
            word[t >> 1] |= (y > 0.f ? 1u : 0u) << (16 * (t & 1) + v);
            acc1[t][v] = y;
          }
        }
      }
#pragma unroll
      for (int w = 0; w < NW1; ++w) bw[w * 64] = word[w];  // rows past the end: never read back
    } else {
      unsigned word[NW1];
#pragma unroll
      for (int w = 0; w < NW1; ++w) word[w] = bw[w * 64];
#pragma unroll
      for (int t = 0; t < NT1; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc1[t][v] = (word[t >> 1] >> (16 * (t & 1) + v)) & 1u ? acc1[t][v] : 0.f;
    }
#ifdef TT_CHAB_NOSTORE
    if (row_ok && rows < 0) {
#else
    if (row_ok) {
#endif
      float* hrow = Hout + row * R1 + 4 * hh;
#pragma unroll
      for (int t = 0; t < NT1; ++t)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq)
          *reinterpret_cast<f32x4*>(hrow + 32 * t + 8 * gq) =
              f32x4{acc1[t][4 * gq], acc1[t][4 * gq + 1], acc1[t][4 * gq + 2], acc1[t][4 * gq + 3]};
    }
    // to the A operand layout: registers (8 s + i, 8 s + 4 + i) hold units 16 s + 8 hh + [0, 8): the
    // upper half's group 2 s goes to the lower half's group 2 s + 1 register and the lower half's
    // group 2 s + 1 to the upper half's group 2 s register (T21's half exchange)
#pragma unroll
    for (int t = 0; t < NT1; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          // (the pair made opaque first: a select between two elements of one vector otherwise becomes
          // a lane-varying element index, extracted and inserted by 16-way v_cndmask chains)
          float a = acc1[t][8 * s + i], b = acc1[t][8 * s + 4 + i];
          asm volatile("" : "+v"(a), "+v"(b));
          const float got = __shfl_xor(hh ? a : b, 32);
          acc1[t][8 * s + i] = hh ? got : a;
          acc1[t][8 * s + 4 + i] = hh ? b : got;
        }
    // ---- second product: acc2[t2] = (this wave's rows, as A) x (P2 rows 32 t2 .. +31)^T
    f32x16 acc2[NT2];
#pragma unroll
    for (int t = 0; t < NT2; ++t) acc2[t] = f32x16{};
#pragma unroll
    for (int j = 0; j < C2; ++j) {
      arrive(C1 + j, bi);
      fill_ahead(C1 + j, bi, rb, slot);
      const lds_char_t* ch = lds + slot * SLOT + r32 * 32 + (hh ^ ((r32 >> 3) & 1)) * 16;
      bf16x8 w[2][3];
#pragma unroll
      for (int p = 0; p < 3; ++p) w[0][p] = *reinterpret_cast<const lds_bf16x8_t*>(ch + p * R2 * 32);
      const f32x16& hv = acc1[j >> 1];
      const int o = 8 * (j & 1);
      __bf16 h0[8], h1[8], h2[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) split3(hv[o + i], h0[i], h1[i], h2[i]);
      bf16x8 a0, a1, a2;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        a0[i] = h0[i];
        a1[i] = h1[i];
        a2[i] = h2[i];
      }
#pragma unroll
      for (int t = 0; t < NT2; ++t) {
        if (t + 1 < NT2) {
#pragma unroll
          for (int p = 0; p < 3; ++p)
            w[(t + 1) & 1][p] = *reinterpret_cast<const lds_bf16x8_t*>(ch + p * R2 * 32 + (t + 1) * 1024);
        }
        __builtin_amdgcn_sched_barrier(0);
        const bf16x8(&wt)[3] = w[t & 1];
        acc2[t] = TT_CH_MFMA(a2, wt[0], acc2[t]);
        acc2[t] = TT_CH_MFMA(a1, wt[1], acc2[t]);
        acc2[t] = TT_CH_MFMA(a0, wt[2], acc2[t]);
        acc2[t] = TT_CH_MFMA(a1, wt[0], acc2[t]);
        acc2[t] = TT_CH_MFMA(a0, wt[1], acc2[t]);
        acc2[t] = TT_CH_MFMA(a0, wt[0], acc2[t]);
        __builtin_amdgcn_sched_barrier(0);
      }
      slot = slot + 1 == kCSlots ? 0 : slot + 1;
    }
    // ---- second epilogue: acc2[t][v] = row r0 + (v & 3) + 8 (v >> 2) + 4 hh, column 32 t + r32
    if constexpr (MODE2 == 0 || MODE2 == 1) {
#pragma unroll
      for (int t = 0; t < NT2; ++t) {
        const float bv = bias2[32 * t + r32];
#pragma unroll
        for (int v = 0; v < 16; ++v) acc2[t][v] += bv;  // head.hip EPI_BIAS_L2's y += bias
      }
    }
    if constexpr (MODE2 == 1) {
      // F.normalize (x / max(|x|, 1e-12)) with head_normalize_kernel's arithmetic bit for bit (so the
      // head's output is the same whether or not tt_inbatch_l2_prep normalises it): 8 rows at a time
      // through this wave's LDS staging area into that kernel's layout (lane L: columns G L .. G L + G - 1,
      // G = R2 / 64), its sum-of-squares chain and butterfly, and whole 1-KiB rows stored.
      static_assert(R2 == 128 || R2 == 256, "F.normalize epilogue widths");
      constexpr int G = R2 / 64;
      lds_char_t* stg = lds + kCSlots * SLOT + wid * (8 * STG_ROW);
#pragma unroll
      for (int k = 0; k < 4; ++k) {  // rows 8 k .. 8 k + 7 of the tile: v = 4 k .. 4 k + 3, both halves
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int t = 0; t < NT2; ++t)
            *reinterpret_cast<__attribute__((address_space(3))) float*>(stg + (4 * hh + i) * STG_ROW +
                                                                        (32 * t + r32) * 4) = acc2[t][4 * k + i];
#pragma unroll
        for (int rr = 0; rr < 8; ++rr) {
          const int64_t row = r0 + 8 * k + rr;
          if constexpr (G == 4) {
            f32x4 v = *reinterpret_cast<const lds_f32x4_t*>(stg + rr * STG_ROW + 16 * lane);
            const float ss = wave_sum(sumsq4(v));
            const float nrm = sqrtf(ss), inv = 1.f / fmaxf(nrm, 1e-12f);
            v[0] *= inv;
            v[1] *= inv;
            v[2] *= inv;
            v[3] *= inv;
            if (row < rows) {
              reinterpret_cast<f32x4*>(Y + row * R2)[lane] = v;
              if (lane == 0) norms[row] = nrm;
            }
          } else {
            typedef float f32x2 __attribute__((ext_vector_type(2)));
            typedef __attribute__((address_space(3))) f32x2 lds_f32x2_t;
            f32x2 v = *reinterpret_cast<const lds_f32x2_t*>(stg + rr * STG_ROW + 8 * lane);
            const float ss = wave_sum(__builtin_fmaf(v[1], v[1], v[0] * v[0]));
            const float nrm = sqrtf(ss), inv = 1.f / fmaxf(nrm, 1e-12f);
            v[0] *= inv;
            v[1] *= inv;
            if (row < rows) {
              reinterpret_cast<f32x2*>(Y + row * R2)[lane] = v;
              if (lane == 0) norms[row] = nrm;
            }
          }
        }
      }
      continue;  // the rows are stored
    }
    if constexpr (MODE2 == 2) {
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int64_t rr = r0 + (v & 3) + 8 * (v >> 2) + 4 * hh;
        const float dv = bias2[rr < rows ? rr : rows - 1];
#pragma unroll
        for (int t = 0; t < NT2; ++t) acc2[t][v] = acc2[t][v] / dv;  // IEEE division, as bag_scale_rows
      }
    }
    float* orow = Y + r0 * R2 + r32;
#ifdef TT_CHAB_NOSTORE
    if (rows < 0) {
#else
    if (__builtin_amdgcn_readfirstlane((int)(r0 + kCRows <= rows))) {
#endif
#pragma unroll
      for (int t = 0; t < NT2; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v) orow[((v & 3) + 8 * (v >> 2) + 4 * hh) * R2 + 32 * t] = acc2[t][v];
    } else {
#pragma unroll
      for (int t = 0; t < NT2; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int rl = (v & 3) + 8 * (v >> 2) + 4 * hh;
          if (r0 + rl < rows) orow[rl * R2 + 32 * t] = acc2[t][v];
        }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int K1, int R1, int R2, int MODE1, int MODE2>
int launch_chain(const float* X, int64_t rows, int64_t ldx, const __bf16* P1, const __bf16* P2, const float* b1,
                 const float* b2, unsigned* bits, float* Hout, float* Y, float* norms, hipStream_t s) {
  constexpr int RMAX = R1 > R2 ? R1 : R2;
  const int64_t nblk = (rows + kCW * kCRows - 1) / (kCW * kCRows);
  const dim3 grid((unsigned)std::min<int64_t>(nblk, 256)), block(kCW * 64);
  const int lds_bytes = kCSlots * (3 * RMAX * 32 + kCW * kCRows * 64) + (MODE2 == 1 ? kCW * 8 * (R2 * 4 + 16) : 0);
  head_chain_kernel<K1, R1, R2, MODE1, MODE2><<<grid, block, lds_bytes, s>>>(
      X, rows, ldx, P1, P2, b1, b2, bits, Hout, Y, norms, nblk);
  TT_LAUNCH_CHECK("tt_head_chain");
  return TT_OK;
}

bool chain_width_ok(int w) { return w == 64 || w == 128 || w == 256; }

}  // namespace
}  // namespace tt

using namespace tt;

extern "C" size_t tt_head_chain_bits_bytes(int64_t rows, int H) {
  return (size_t)((rows + kCRows - 1) / kCRows + kCW) * ((H / 32 + 1) / 2) * 64 * sizeof(uint32_t);
}

extern "C" int tt_head_fwd_chain(const float* x, int64_t rows, int64_t ldx, int E, int H, const void* planes_w1,
                                 const void* planes_w2, const float* b1, const float* b2, uint32_t* relu_bits,
                                 float* h, float* out, float* norms, int normalize, tt_stream_t stream) {
  TT_REQUIRE(chain_width_ok(E) && (H == 128 || H == 256), "tt_head_fwd_chain: E in {64, 128, 256}, H in {128, 256} "
             "(got E=%d H=%d)", E, H);
  TT_REQUIRE(rows >= 0 && rows < (int64_t(1) << 31) && ldx >= E && ldx % 4 == 0, "bad shape rows=%lld ldx=%lld",
             (long long)rows, (long long)ldx);
  if (rows == 0) return TT_OK;
  TT_REQUIRE(x && planes_w1 && planes_w2 && b1 && b2 && relu_bits && h && out && (norms || !normalize),
             "null pointer");
  TT_REQUIRE(((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(h) | reinterpret_cast<uintptr_t>(out) |
               reinterpret_cast<uintptr_t>(b1)) & 15) == 0, "x / h / out / b1 must be 16-byte aligned");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const __bf16* p1 = static_cast<const __bf16*>(planes_w1);
  const __bf16* p2 = static_cast<const __bf16*>(planes_w2);
  unsigned* bits = reinterpret_cast<unsigned*>(relu_bits);
#define TT_FC(EE, HH)                                                                                             \
  if (E == EE && H == HH)                                                                                         \
    return normalize ? launch_chain<EE, HH, HH, 0, 1>(x, rows, ldx, p1, p2, b1, b2, bits, h, out, norms, s)       \
                     : launch_chain<EE, HH, HH, 0, 0>(x, rows, ldx, p1, p2, b1, b2, bits, h, out, norms, s);
  TT_FC(256, 256)
  TT_FC(128, 128)
  TT_FC(64, 128)
  TT_FC(128, 256)
  TT_FC(64, 256)
  TT_FC(256, 128)
#undef TT_FC
  return TT_ERR_UNSUPPORTED;
}

extern "C" int tt_head_bwd_chain(const float* dy, int64_t rows, int64_t lddy, int E, int H, const void* planes_w2t,
                                 const void* planes_w1t, const uint32_t* relu_bits, const float* row_div, float* dh,
                                 float* dx, tt_stream_t stream) {
  TT_REQUIRE(chain_width_ok(E) && (H == 128 || H == 256), "tt_head_bwd_chain: E in {64, 128, 256}, H in {128, 256} "
             "(got E=%d H=%d)", E, H);
  TT_REQUIRE(rows >= 0 && rows < (int64_t(1) << 31) && lddy >= H && lddy % 4 == 0, "bad shape rows=%lld lddy=%lld",
             (long long)rows, (long long)lddy);
  if (rows == 0) return TT_OK;
  TT_REQUIRE(dy && planes_w2t && planes_w1t && relu_bits && dh && dx, "null pointer");
  TT_REQUIRE(((reinterpret_cast<uintptr_t>(dy) | reinterpret_cast<uintptr_t>(dh) | reinterpret_cast<uintptr_t>(dx)) &
              15) == 0, "dy / dh / dx must be 16-byte aligned");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const __bf16* p1 = static_cast<const __bf16*>(planes_w2t);
  const __bf16* p2 = static_cast<const __bf16*>(planes_w1t);
  unsigned* bits = const_cast<unsigned*>(reinterpret_cast<const unsigned*>(relu_bits));
#define TT_BC(EE, HH)                                                                                              \
  if (E == EE && H == HH)                                                                                          \
    return row_div ? launch_chain<HH, HH, EE, 1, 2>(dy, rows, lddy, p1, p2, nullptr, row_div, bits, dh, dx, nullptr, s) \
                   : launch_chain<HH, HH, EE, 1, 3>(dy, rows, lddy, p1, p2, nullptr, nullptr, bits, dh, dx, nullptr, s);
  TT_BC(256, 256)
  TT_BC(128, 128)
  TT_BC(64, 128)
  TT_BC(128, 256)
  TT_BC(64, 256)
  TT_BC(256, 128)
#undef TT_BC
  return TT_ERR_UNSUPPORTED;
}
