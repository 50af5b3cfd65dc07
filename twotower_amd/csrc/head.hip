// Tower head GEMMs on gfx950: Linear(E,H)-ReLU-Linear(H,H) + F.normalize of MeanPoolingTower
// (twotower/encoders.py:38-42,77) and their activation gradients, for E = H = 256.
//
// fp32 GEMM on the bf16 MFMA: each fp32 operand is split into three bf16 terms (a = a0 + a1 + a2,
// exact to 2^-24 relative) and the six cross products whose order is >= 2^-16 are accumulated in
// fp32 (a0b0, a0b1, a1b0, a0b2, a1b1, a2b0); the dropped terms are <= 2^-24 of the product, so
// results agree with an fp32 GEMM to rounding of the accumulation order.  Six 32x32x16 bf16 MFMAs
// (32 cycles each) do the work of eight 32x32x2 f32 MFMAs (64 cycles each): 2.7x the rate.
//
// out[r, n] = epi(sum_k A[r, k] W[n, k]), A fp32 row-major (rows x 256), W given as three
// pre-split bf16 planes [3][256 n][256 k] (tt_head_split: the weight, or its transpose).
// A workgroup owns a 64-column slice of the output for a group of rows: its slice of the three
// B planes (96 KiB) is loaded into LDS once (16-B chunks XOR-swizzled by row, so the MFMA operand
// reads are conflict-free) and stays resident; the four waves stream 32-row tiles of A straight
// from HBM into registers in the MFMA operand layout (8 consecutive k per lane, a whole tile = 128
// VGPRs), split them into bf16 terms in registers, and fetch each k chunk of their next tile as
// soon as the current one is consumed -- a full tile (~3 us) of latency cover with no barrier in
// the main loop.  The four column slices of a row group run on the same XCD (blockIdx % 8), so
// A is fetched from HBM once and served to the other three from that XCD's L2.
// The L2-normalise epilogue needs whole rows: the slices write the biased rows and
// head_normalize_kernel (one wave per row) forms each row's norm and scales it in place.
#include "common.hpp"

namespace tt {
namespace {

constexpr int kColsWG = 64;                         // output column slice per workgroup
constexpr int kKS = 16;                             // k per MFMA step
constexpr int kWaves = 4;
constexpr int kTileRows = 32;
constexpr int kMaxSlices = 4;                       // N <= 256: the ReLU mask is sized for 4 slices

// A head GEMM shape: out (rows x N) = A (rows x K) W^T, K, N in {64, 128, 256} (MeanPoolingTower:
// E = H = d at C2 (128) and C3 / C5 (256); C1's char tower E = 64 -> H = 128, whose first Linear
// is K = 64 and whose dx GEMM is N = 64).
template <int K, int N>
struct HeadShape {
  static_assert((K == 64 || K == 128 || K == 256) && (N == 64 || N == 128 || N == 256),
                "head GEMM shapes: K, N in {64, 128, 256}");
  static constexpr int kSlices = N / kColsWG;       // column slices (workgroups per row group)
  static constexpr int kRowB = K * 2;               // one bf16 row of W (bytes)
  static constexpr int kCH = K / 8;                 // 16-B chunks per row
  static constexpr int kPlaneB = kColsWG * kRowB;   // one bf16 plane of the slice
  static constexpr int kSliceB = 3 * kPlaneB;       // resident in LDS (96 KiB at K = 256)
  static constexpr int kSteps = K / kKS;
};

enum Epi { EPI_BIAS_RELU = 0, EPI_BIAS_L2 = 1, EPI_RELU_MASK = 2, EPI_PLAIN = 3, EPI_ROWDIV = 5 };

// blockIdx.y selects one of up to 4 (weight, transpose) jobs (SplitJobs, common.hpp).
__global__ __launch_bounds__(256) void split_planes_kernel(SplitJobs jobs, __bf16* __restrict__ planes_base) {
  split_planes_elem(jobs, blockIdx.y, blockIdx.x * 256 + threadIdx.x, planes_base);
}

// Workgroup b -> (row group g, column slice c).  Blocks b, b+8, ... share an XCD (round-robin
// dispatch over the 8 XCDs) and take the S slices of one row group.
template <int S>
__device__ __forceinline__ void head_block(int b, int& g, int& c) {
  c = (b >> 3) % S;
  g = (b >> 3) / S * 8 + (b & 7);
}

template <int EPI, int K, int N>
__global__ __launch_bounds__(256, 1) void head_gemm_kernel(const float* __restrict__ A, int64_t rows, int64_t lda,
                                                           const __bf16* __restrict__ planes,
                                                           const float* __restrict__ bias,
                                                           unsigned* __restrict__ relu_mask, float* __restrict__ out,
                                                           float* __restrict__ part, int groups, int tiles) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef __attribute__((address_space(3))) bf16x8 lds_bf16x8_t;
  typedef __attribute__((address_space(3))) char lds_char_t;
  lds_char_t* lds = (lds_char_t*)smem;
  using HS = HeadShape<K, N>;
  constexpr int kSlices = HS::kSlices, kPlaneB = HS::kPlaneB, kSliceB = HS::kSliceB, kSteps = HS::kSteps;
  constexpr int kCH = HS::kCH, kRowB = HS::kRowB;
  int g, c;
  head_block<kSlices>(blockIdx.x, g, c);
  if (g >= groups) return;
  const int tid = threadIdx.x, lane = lane_id(), wid = tid >> 6;
  const int r32 = lane & 31, hh = lane >> 5;

  // resident B slice: lds[p][n][chunk ^ (n % kCH)], chunk = 8 k (16 B), n = local column.
  // LDS-DMA writes each 1 KiB piece linearly (lane l -> byte 16 l = row n0 + l / kCH, slot
  // l % kCH), so the swizzle goes on the source: slot s of row n holds chunk s ^ (n % kCH).
  // kSliceB / 4 KiB pieces per wave (24 at K = 256), all in flight together, no staging registers.
  {
    constexpr int kPiecesW = kSliceB / 1024 / kWaves;
    constexpr int kRowsPiece = 1024 / kRowB;
    const unsigned wl = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds);
    const char* src = reinterpret_cast<const char*>(planes);
#pragma unroll
    for (int u = 0; u < kPiecesW; ++u) {
      const int piece = u * kWaves + wid;  // 1 KiB = kRowsPiece rows of the slice image
      const int row = kRowsPiece * piece + lane / kCH, p = row / kColsWG, n = row % kColsWG;
      const int q = (lane % kCH) ^ (n % kCH);
      const unsigned off = (unsigned)(((size_t)p * N * K + (size_t)(c * kColsWG + n) * K + q * 8) * 2);
      asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(off), "s"(src),
                   "s"(__builtin_amdgcn_readfirstlane(wl + piece * 1024))
                   : "memory");
    }
  }
  // this wave's tiles: rows g*tiles*128 + t*128 + wid*32 + [0, 32)
  const int64_t wrow0 = (int64_t)g * tiles * (kWaves * kTileRows) + wid * kTileRows;
  auto a_src = [&](int t) {
    int64_t r = wrow0 + (int64_t)t * (kWaves * kTileRows) + r32;
    r = r < rows ? r : rows - 1;  // rows past the end are computed from a clamped row, never stored
    return reinterpret_cast<const f32x4*>(A + r * lda + hh * 8);
  };
  constexpr int kAStep = 4, kAHalf = 1;
  // A chunks in flight: the whole next tile (kAR = kSteps: 128 VGPRs at K = 256, one wave per SIMD
  // with the rest), or TT_HEAD_AHALF: half a tile ahead (kAR = kSteps / 2, ~64 VGPRs less, so the
  // kernel fits 256 registers and other kernels' waves can share its SIMDs)
#ifndef TT_HEAD_AHALF
#define TT_HEAD_AHALF 1
#endif
#ifndef TT_HEAD_ADIV
#define TT_HEAD_ADIV 4  // with TT_HEAD_AHALF: 1 / TT_HEAD_ADIV of a tile ahead
#endif
  constexpr int kAR = TT_HEAD_AHALF && kSteps >= 2 * TT_HEAD_ADIV ? kSteps / TT_HEAD_ADIV : kSteps;
  f32x4 areg[kAR][2];
  {
    const f32x4* src = a_src(0);
#pragma unroll
    for (int j = 0; j < kAR; ++j) {
      areg[j][0] = *(src + j * kAStep);
      areg[j][1] = *(src + j * kAStep + kAHalf);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces (and A tile 0) landed
  __syncthreads();                                   // B slice resident

  // B operand of column tile ct, plane p, step j: local column n = 32 ct + r32, chunk 2 j + hh
  const lds_char_t* bbase = lds + r32 * kRowB;
  auto rdb = [&](int ct, int p, int j) {  // (32 ct + r32) % kCH == r32 % kCH picks the swizzle
    return *reinterpret_cast<const lds_bf16x8_t*>(bbase + ct * 32 * kRowB + p * kPlaneB +
                                                  (((2 * j + hh) ^ (r32 % kCH)) << 4));
  };

  // Software pipeline: while step j's twelve MFMAs run, the wave reads step j+1's B operands from
  // LDS and splits step j+1's A chunk in twelve packed pieces of 2-4 VALU, one per MFMA gap
  // (pinned by volatile register ties and sched_barrier fences).  Step 15 prepares step 0 of the
  // next tile.  Split words: w[plane][pair] = bf16 pair (x_2i, x_2i+1) of that plane.
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  struct SplitState {
    f32x2 r;         // running remainder of the pair
    bf16x2 h;        // last rounded term
  };
  // piece k of the split of chunk ar: pair k/3, stage k%3
  auto split_piece = [&](const f32x4 (&ar)[2], int k, SplitState (&st)[4], u32x4 (&w)[3]) {
    const int i = k / 3, stage = k % 3;
    if (stage == 0) {
      const f32x2 x = i < 2 ? f32x2{ar[0][2 * i], ar[0][2 * i + 1]} : f32x2{ar[1][2 * i - 4], ar[1][2 * i - 3]};
      st[i].h = __builtin_convertvector(x, bf16x2);
      w[0][i] = __builtin_bit_cast(unsigned, st[i].h);
      st[i].r = x - __builtin_convertvector(st[i].h, f32x2);
      asm volatile("" : "+v"(st[i].r), "+v"(w[0][i]));
    } else if (stage == 1) {
      st[i].h = __builtin_convertvector(st[i].r, bf16x2);
      w[1][i] = __builtin_bit_cast(unsigned, st[i].h);
      st[i].r = st[i].r - __builtin_convertvector(st[i].h, f32x2);
      asm volatile("" : "+v"(st[i].r), "+v"(w[1][i]));
    } else {
      w[2][i] = __builtin_bit_cast(unsigned, __builtin_convertvector(st[i].r, bf16x2));
      asm volatile("" : "+v"(w[2][i]));
    }
  };
  u32x4 ca[3];
  bf16x8 cb[2][3];
  {
    SplitState st[4];
#pragma unroll
    for (int k = 0; k < 12; ++k) split_piece(areg[0], k, st, ca);
  }
#pragma unroll
  for (int ct = 0; ct < 2; ++ct)
#pragma unroll
    for (int p = 0; p < 3; ++p) cb[ct][p] = rdb(ct, p, 0);

  float bv[2] = {0.f, 0.f};  // this lane's two bias columns, loaded once
  if constexpr (EPI == EPI_BIAS_RELU || EPI == EPI_BIAS_L2) {
    bv[0] = bias[c * kColsWG + r32];
    bv[1] = bias[c * kColsWG + 32 + r32];
  }
  // ReLU mask: tile-private words.  The forward and the backward launch the same tiling for the
  // same rows, so lane l of the tile (row tile trow0 / 32, slice c) keeps its own 32 bits
  // (bit 16 ct + v = element acc[ct][v] > 0) in word ((trow0 / 32) * 4 + c) * 64 + l.

  for (int t = 0; t < tiles; ++t) {
    const int64_t trow0 = wrow0 + (int64_t)t * (kWaves * kTileRows);
    if (__builtin_amdgcn_readfirstlane((int)(trow0 >= rows))) break;
    const bool more = t + 1 < tiles && trow0 + kWaves * kTileRows < rows;
    // unconditional refills keep each step one basic block; the last tile re-reads itself (L2)
    const f32x4* csrc = a_src(t);
    const f32x4* nsrc = more ? a_src(t + 1) : csrc;
    f32x16 acc[2] = {f32x16{}, f32x16{}};
    const int64_t mask_idx = ((trow0 / kTileRows) * kSlices + c) * 64 + lane;
    unsigned mword = 0;
    if constexpr (EPI == EPI_RELU_MASK)  // issued before the tile's A refills: no flush to wait on it
      mword = relu_mask[mask_idx];
    float rdiv[16];  // EPI_ROWDIV: the divisor of each of this lane's 16 rows (bias = per-row divisors)
    if constexpr (EPI == EPI_ROWDIV) {
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int64_t r = trow0 + (v & 3) + 8 * (v >> 2) + 4 * hh;
        rdiv[v] = bias[r < rows ? r : rows - 1];
      }
    }
#pragma unroll
    for (int j = 0; j < kSteps; ++j) {
      const int jn = (j + 1) % kSteps;
      u32x4 na[3];
      bf16x8 nb[2][3];
      SplitState st[4];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int p = 0; p < 3; ++p) nb[ct][p] = rdb(ct, p, jn);
      // chunk j (slot j % kAR) was split during the previous step: refill the slot with chunk j + kAR
      // of the stream (this tile's, or the next tile's once past the end)
      {
        const int c = j + kAR;  // (j is a compile-time constant after unrolling: so is the branch)
        const f32x4* rs = c < kSteps ? csrc + c * kAStep : nsrc + (c - kSteps) * kAStep;
        areg[j % kAR][0] = *rs;
        areg[j % kAR][1] = *(rs + kAHalf);
      }
      __builtin_amdgcn_sched_barrier(0);
      const bf16x8 a0 = __builtin_bit_cast(bf16x8, ca[0]), a1 = __builtin_bit_cast(bf16x8, ca[1]),
                   a2 = __builtin_bit_cast(bf16x8, ca[2]);
#pragma unroll
      for (int m = 0; m < 12; ++m) {
        const int ct = m / 6;
        f32x16& C = acc[ct];
        const bf16x8(&b)[3] = cb[ct];
        switch (m % 6) {
          case 0: C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b[0], C, 0, 0, 0); break;
          case 1: C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b[1], C, 0, 0, 0); break;
          case 2: C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[2], C, 0, 0, 0); break;
          case 3: C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b[0], C, 0, 0, 0); break;
          case 4: C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[1], C, 0, 0, 0); break;
          default: C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[0], C, 0, 0, 0); break;
        }
        split_piece(areg[jn % kAR], m, st, na);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        ca[p] = na[p];
        cb[0][p] = nb[0][p];
        cb[1][p] = nb[1][p];
      }
    }

    // Epilogue.  acc[ct][v] is row trow0 + (v & 3) + 8 (v >> 2) + 4 hh, column
    // 64 c + 32 ct + r32.  Rows past the end are never stored; full tiles store unguarded.
    unsigned my_mask = 0;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        float y = acc[ct][v];
        if constexpr (EPI == EPI_BIAS_RELU) {
          y = fmaxf(y + bv[ct], 0.f);
          my_mask |= (y > 0.f ? 1u : 0u) << (16 * ct + v);
        }
        if constexpr (EPI == EPI_BIAS_L2) y += bv[ct];
        if constexpr (EPI == EPI_RELU_MASK) y = (mword >> (16 * ct + v)) & 1u ? y : 0.f;
        if constexpr (EPI == EPI_ROWDIV) y = y / rdiv[v];  // IEEE division, as bag_scale_rows_kernel
        acc[ct][v] = y;
      }
    }
    float* orow = out + trow0 * N + c * kColsWG + r32;
    if (__builtin_amdgcn_readfirstlane((int)(trow0 + kTileRows <= rows))) {
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int v = 0; v < 16; ++v) orow[((v & 3) + 8 * (v >> 2) + 4 * hh) * N + ct * 32] = acc[ct][v];
    } else {
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int rl = (v & 3) + 8 * (v >> 2) + 4 * hh;
          if (trow0 + rl < rows) orow[rl * N + ct * 32] = acc[ct][v];
        }
    }
    if constexpr (EPI == EPI_BIAS_RELU) {
      if (relu_mask) relu_mask[mask_idx] = my_mask;
    }
  }
}

// Finishes F.normalize (ATen: x / max(|x|, 1e-12)): one 64-lane wave per row, N / 64 floats per
// lane (N = 256: one float4, the arithmetic tt_inbatch_l2_prep repeats bit for bit).
template <int N>
__global__ __launch_bounds__(256) void head_normalize_kernel(float* __restrict__ y, int64_t rows,
                                                             const float* __restrict__ part,
                                                             float* __restrict__ norms) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int lane = lane_id();
  if constexpr (N == 128) {
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    f32x2* p = reinterpret_cast<f32x2*>(y + row * N) + lane;
    f32x2 v = *p;
    const float ss = wave_sum(__builtin_fmaf(v[1], v[1], v[0] * v[0]));
    const float nrm = sqrtf(ss), inv = 1.f / fmaxf(nrm, 1e-12f);
    v[0] *= inv;
    v[1] *= inv;
    *p = v;
    if (lane == 0) norms[row] = nrm;
    return;
  }
  f32x4* p = reinterpret_cast<f32x4*>(y + row * N) + lane;
  f32x4 v = *p;
  const float ss = wave_sum(sumsq4(v));
  const float nrm = sqrtf(ss), inv = 1.f / fmaxf(nrm, 1e-12f);
  v[0] *= inv;
  v[1] *= inv;
  v[2] *= inv;
  v[3] *= inv;
  *p = v;
  if (lane == 0) norms[row] = nrm;
}

// ------------------------------------------------------------------------------------------
// Weight and bias gradients of a head Linear: dW = G^T X (256 x 256), db = colsum(G), for tall
// G, X (rows x 256 fp32; G = dh / dy, X = x / h).  K (= rows) is split over 64 slabs: a
// workgroup owns one 128 x 128 output block of one slab (grid = 4 blocks x slabs), its four waves
// 2 x 2 tiles of 32 x 32 each.  Rows stream in chunks of 16: every thread loads 4 floats of G and
// 4 of X for two rows (raw loads run three chunks ahead in registers), splits them into bf16
// terms and writes the three planes row-major into LDS (XOR-swizzled by row & 3 in 64-B units);
// the MFMA operands, which need 8 consecutive ROWS of one column per lane, come back with
// ds_read_b64_tr_b16.  One barrier per chunk (double-buffered planes).  The loader threads of the
// j-block-0 workgroups also sum their G columns (db).  Slab partials are reduced in fixed order
// by head_wgrad_reduce_kernel: deterministic.
constexpr int kWgChunk = 16;                              // rows per chunk
constexpr int kWgBlk = 128;                               // output block edge
constexpr int kWgPlane = kWgChunk * kWgBlk * 2;           // 4 KiB: one bf16 plane of a chunk
constexpr int kWgBuf = 2 * 3 * kWgPlane;                  // G and X planes: 24 KiB

__device__ __forceinline__ int wg_off(int row, int col) {  // byte offset in a plane
  return row * (kWgBlk * 2) + ((col * 2) ^ ((row & 3) << 6));
}

// Two problems in one launch (tt_head_wgrad2): blocks [0, 4 slabs) take (G, X), the rest (G2, X2)
// with partials at part_w2 / part_b2; each problem keeps the one-problem block mapping.
struct WgradProblem2 {
  const float* G;
  const float* X;
  float* part_w;
  float* part_b;
  int nblk;  // blocks of the first problem (4 * slabs); 0: one problem
};

template <int NG, int NX>
__global__ __launch_bounds__(256, 1) void head_wgrad_kernel(const float* __restrict__ G, const float* __restrict__ X,
                                                            int64_t rows, int64_t slab_rows,
                                                            float* __restrict__ part_w, float* __restrict__ part_b,
                                                            WgradProblem2 second = WgradProblem2{}) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;
  typedef __attribute__((address_space(3))) char lds_char_t;
  typedef __attribute__((address_space(3))) uint64_t lds_u64_t;
  lds_char_t* lds = (lds_char_t*)smem;
  unsigned bid = blockIdx.x;
  if (second.nblk && bid >= (unsigned)second.nblk) {  // block-uniform: the second problem
    bid -= second.nblk;
    G = second.G;
    X = second.X;
    part_w = second.part_w;
    part_b = second.part_b;
  }
  // blocks b, b+8, ... share an XCD (round-robin dispatch): they take the NB output blocks of
  // one slab, so its G / X rows come from HBM once and from that XCD's L2 after
  // output blocks per slab: (NG / 128) x (NX / 128) (4 at 256 x 256, 1 at 128 x 128); an X narrower
  // than a block (C1's E = 64) takes one block whose columns past NX are zero and never stored
  constexpr int NBI = NG / kWgBlk, NBJ = NX < kWgBlk ? 1 : NX / kWgBlk, NB = NBI * NBJ;
  constexpr int XW = NX < kWgBlk ? NX : kWgBlk;  // valid columns of an X block
  const int blk = (bid >> 3) % NB, slab = (bid >> 3) / NB * 8 + (bid & 7);
  const int bi = blk % NBI, bj = blk / NBI;  // output block rows i in [128 bi, +128), cols j in [128 bj, +XW)
  const int tid = threadIdx.x, lane = lane_id(), wid = tid >> 6;
  const int64_t r_begin = (int64_t)slab * slab_rows;
  const int64_t r_end = r_begin + slab_rows < rows ? r_begin + slab_rows : rows;
  // every slab runs slab_rows / 16 chunks (a multiple of the ring depth): no tail branches;
  // rows past r_end load a clamped row and are zeroed when staged
  const int nchunks = (int)(slab_rows / kWgChunk);

  // loader: float4 column group lc (4 columns) of rows lr and lr + 8 of each chunk
  const int lc = tid & 31, lr = tid >> 5;
  const float* gsrc = G + 128 * bi + 4 * lc;
  const bool xok = 4 * lc < XW;
  const float* xsrc = X + 128 * bj + (xok ? 4 * lc : 0);
  constexpr int kRing = 3;  // chunks in flight (registers); the loop is unrolled by it
  f32x4 raw[kRing][4];     // per chunk: G row lr, G row lr+8, X row lr, X row lr+8
  auto load_chunk = [&](int ch, f32x4 (&r)[4]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      int64_t row = r_begin + (int64_t)ch * kWgChunk + lr + 8 * h;
      row = row < rows ? row : 0;
      r[h] = *reinterpret_cast<const f32x4*>(gsrc + row * NG);  // rows past the end: zeroed when staged
      r[2 + h] = *reinterpret_cast<const f32x4*>(xsrc + row * NX);
    }
  };
  f32x4 colsum = {0.f, 0.f, 0.f, 0.f};
  auto stage_chunk = [&](const f32x4 (&r)[4], int ch, int buf) {
    const int64_t row0 = r_begin + (int64_t)ch * kWgChunk + lr;
    const bool ok[2] = {row0 < r_end, row0 + 8 < r_end};
    f32x4 rv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      rv[q] = r[q];
      asm volatile("" : "+v"(rv[q]));  // keeps the use (and its vmcnt wait) here, not hoisted
      rv[q] = ok[q & 1] && (q < 2 || xok) ? rv[q] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // q: 0,1 = G rows lr, lr+8; 2,3 = X rows lr, lr+8
      const int row = lr + 8 * (q & 1);
      lds_char_t* base = lds + buf * kWgBuf + (q >> 1) * 3 * kWgPlane + wg_off(row, 4 * lc);
      bf16x4 t0, t1, t2;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        __bf16 u0, u1, u2;
        split3(rv[q][e], u0, u1, u2);
        t0[e] = u0;
        t1[e] = u1;
        t2[e] = u2;
      }
      *reinterpret_cast<lds_u64_t*>(base) = __builtin_bit_cast(uint64_t, t0);
      *reinterpret_cast<lds_u64_t*>(base + kWgPlane) = __builtin_bit_cast(uint64_t, t1);
      *reinterpret_cast<lds_u64_t*>(base + 2 * kWgPlane) = __builtin_bit_cast(uint64_t, t2);
    }
    if (bj == 0) colsum += rv[0] + rv[1];
  };

  // transposed operand reads: lane (kh, gh, q, p) reads rows 8 kh + q (+4), columns 16 gh + 4 p of
  // the 32-column tile; it receives column (lane & 31) of rows 8 kh + 0..7
  const int kh = lane >> 5, gh = (lane >> 4) & 1, q = (lane >> 2) & 3, pp = lane & 3;
  auto rd = [&](int buf, int mat, int plane, int tile) {
    const lds_char_t* b = lds + buf * kWgBuf + mat * 3 * kWgPlane + plane * kWgPlane;
    const int col = 32 * tile + 16 * gh + 4 * pp;
    const bf16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(b + wg_off(8 * kh + q, col)));
    const bf16x4 t2 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(b + wg_off(8 * kh + 4 + q, col)));
    return bf16x8{t1[0], t1[1], t1[2], t1[3], t2[0], t2[1], t2[2], t2[3]};
  };
  const int wi = wid & 1, wj = wid >> 1;  // wave tiles: i tiles 2 wi, 2 wi + 1; j tiles 2 wj, 2 wj + 1
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a) acc[a][0] = acc[a][1] = f32x16{};

#pragma unroll
  for (int k = 0; k < kRing; ++k) load_chunk(k, raw[k]);
  stage_chunk(raw[0], 0, 0);
  // one chunk: its planes are in buffer ch & 1; raw[S] held chunk ch (staged last step) and is
  // refilled with chunk ch + kRing; raw[(S + 1) % kRing] holds chunk ch + 1, staged now
  auto step = [&](int ch, f32x4 (&refill)[4], const f32x4 (&next)[4]) {
    __syncthreads();  // planes of chunk ch visible; everyone is done with chunk ch-1's buffer
    const int buf = ch & 1;
    load_chunk(ch + kRing < nchunks ? ch + kRing : ch, refill);  // past the end: a harmless reload
    bf16x8 ga[2][3], xb[2][3];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        ga[t][p] = rd(buf, 0, p, 2 * wi + t);
        xb[t][p] = rd(buf, 1, p, 2 * wj + t);
      }
    stage_chunk(next, ch + 1, buf ^ 1);  // past the end: zeros into the unused buffer
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < 2; ++tj) {
        f32x16& C = acc[ti][tj];
        C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga[ti][2], xb[tj][0], C, 0, 0, 0);
        C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga[ti][1], xb[tj][1], C, 0, 0, 0);
        C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga[ti][0], xb[tj][2], C, 0, 0, 0);
        C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga[ti][1], xb[tj][0], C, 0, 0, 0);
        C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga[ti][0], xb[tj][1], C, 0, 0, 0);
        C = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ga[ti][0], xb[tj][0], C, 0, 0, 0);
      }
  };
  for (int ch = 0; ch < nchunks; ch += kRing) {  // unrolled by the ring depth: static ring slots
#pragma unroll
    for (int k = 0; k < kRing; ++k) step(ch + k, raw[k], raw[(k + 1) % kRing]);
  }

  // partial dW of this slab: acc[ti][tj][v] = (i, j) with i = 128 bi + 32 (2 wi + ti) + (v & 3) +
  // 8 (v >> 2) + 4 kh, j = 128 bj + 32 (2 wj + tj) + (lane & 31)
  float* pw = part_w + (size_t)slab * NG * NX;
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < 2; ++tj)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int i = 128 * bi + 32 * (2 * wi + ti) + (v & 3) + 8 * (v >> 2) + 4 * kh;
        const int j = 128 * bj + 32 * (2 * wj + tj) + (lane & 31);
        if (NX < kWgBlk && 32 * (2 * wj + tj) >= XW) continue;  // zero columns past a narrow X
        pw[i * NX + j] = acc[ti][tj][v];
      }
  if (bj == 0 && part_b) {  // fold the 8 row groups (lr) of each column group in LDS, fixed order
    __syncthreads();
    f32x4* red = reinterpret_cast<f32x4*>(smem);
    red[tid] = colsum;
    __syncthreads();
    if (tid < 32) {
      f32x4 t = red[tid];
#pragma unroll
      for (int g = 1; g < 8; ++g) t += red[g * 32 + tid];
      *reinterpret_cast<f32x4*>(part_b + (size_t)slab * NG + 128 * bi + 4 * tid) = t;
    }
  }
}

// dW[i, j] = sum over slabs of the partials, db likewise.  Four threads per output float4 take
// a quarter of the slabs each (8 loads in flight, slab s to partial s % 8, folded in a fixed
// tree); the quarters are added in a fixed order through LDS -- deterministic.
struct WgradReduce2 {
  const float* part_w;
  const float* part_b;
  float* dW;
  float* db;
  int nblk;  // blocks of the first problem; 0: one problem
};

template <int NG, int NX>
__global__ __launch_bounds__(256) void head_wgrad_reduce_kernel(const float* __restrict__ part_w,
                                                                const float* __restrict__ part_b, int slabs,
                                                                float* __restrict__ dW, float* __restrict__ db,
                                                                WgradReduce2 second = WgradReduce2{}) {
  __shared__ f32x4 red[kRedQ][64];
  unsigned bid = blockIdx.x, nb = gridDim.x;
  if (second.nblk) {  // block-uniform: the first or the second problem
    nb = second.nblk;
    if (bid >= nb) {
      bid -= nb;
      part_w = second.part_w;
      part_b = second.part_b;
      dW = second.dW;
      db = second.db;
    }
  }
  const int o = threadIdx.x & 63, qq = threadIdx.x >> 6;  // output float4 of the block, slab quarter
  const int i = bid * 64 + o;
  const int per = (slabs + kRedQ - 1) / kRedQ;
  const int s0 = qq * per, s1 = min(slabs, s0 + per);
  const bool is_b = bid == nb - 1;  // the last block folds db (N / 4 float4 columns)
  const bool ob = is_b && o < NG / 4;
  const f32x4 t = is_b ? (db && ob ? sum_slabs(reinterpret_cast<const f32x4*>(part_b) + o, NG / 4, s0, s1)
                                   : f32x4{0.f, 0.f, 0.f, 0.f})
                       : sum_slabs(reinterpret_cast<const f32x4*>(part_w) + i, NG * NX / 4, s0, s1);
  red[qq][o] = t;
  __syncthreads();
  if (qq == 0) {
    const f32x4 r = (red[0][o] + red[1][o]) + (red[2][o] + red[3][o]);
    if (!is_b)
      reinterpret_cast<f32x4*>(dW)[i] = r;
    else if (db && ob)
      reinterpret_cast<f32x4*>(db)[o] = r;
  }
}

}  // namespace
}  // namespace tt

using namespace tt;

namespace tt {
namespace {
bool head_width_ok(int n) { return n == 128 || n == 256; }        // H (and E = H)
bool emb_width_ok(int n) { return n == 64 || head_width_ok(n); }   // E of the first Linear
// weight-gradient slabs: one round of 256 workgroups over the two problems of tt_head_wgrad2
// (4 output blocks per slab at N = 256, 1 at N = 128); 64 / 256 for the one-problem form
int wg_slabs2(int N) { return N == 256 ? 32 : 128; }
int wg_blocks2(int NG, int NX) { return (NG / kWgBlk) * (NX < kWgBlk ? 1 : NX / kWgBlk); }
int wg_blocks(int N) { return wg_blocks2(N, N); }
int wg_slabs_ex(int NG, int NX) { return 256 / wg_blocks2(NG, NX); }
}  // namespace
}  // namespace tt

extern "C" size_t tt_head_planes_bytes(int N, int K) { return (size_t)3 * N * K * 2; }

extern "C" int tt_head_split(const float* W, int N, int K, int transpose, void* planes, tt_stream_t stream) {
  TT_REQUIRE(emb_width_ok(N) && emb_width_ok(K), "tt_head_split: N, K in {64, 128, 256} (got %dx%d)", N, K);
  TT_REQUIRE(W && planes, "null pointer");
  SplitJobs jobs{};
  jobs.W[0] = W;
  jobs.transpose[0] = transpose;
  jobs.n[0] = N;
  jobs.k[0] = K;
  split_planes_kernel<<<dim3(N * K / 256, 1), dim3(256), 0, reinterpret_cast<hipStream_t>(stream)>>>(
      jobs, static_cast<__bf16*>(planes));
  TT_LAUNCH_CHECK("tt_head_split");
  return TT_OK;
}

extern "C" int tt_head_split_ff2(const float* W1, const float* W2, int E, int H, void* planes, tt_stream_t stream) {
  TT_REQUIRE(emb_width_ok(E) && head_width_ok(H), "tt_head_split_ff2: E in {64, 128, 256}, H in {128, 256} (got E=%d H=%d)",
             E, H);
  TT_REQUIRE(W1 && W2 && planes, "null pointer");
  // W1 (H x E), W2 (H x H), W1^T (E x H), W2^T (H x H), each as three bf16 planes, in that order
  const SplitJobs jobs = head_ff2_jobs(W1, W2, E, H);
  const int big = std::max(H * E, H * H);
  split_planes_kernel<<<dim3(big / 256, 4), dim3(256), 0, reinterpret_cast<hipStream_t>(stream)>>>(
      jobs, static_cast<__bf16*>(planes));
  TT_LAUNCH_CHECK("tt_head_split_ff2");
  return TT_OK;
}

extern "C" int tt_head_split_ff(const float* W1, const float* W2, void* planes, tt_stream_t stream) {
  return tt_head_split_ff2(W1, W2, 256, 256, planes, stream);
}

extern "C" size_t tt_head_relu_mask_bytes(int64_t rows) {
  return (size_t)((rows + kTileRows - 1) / kTileRows) * kMaxSlices * 64 * sizeof(uint32_t);
}

extern "C" size_t tt_head_gemm_ws_size(int64_t rows, int epi) {
  (void)rows;
  (void)epi;
  return 0;  // the L2 epilogue's row norms are formed by head_normalize_kernel from the rows
}

namespace tt {
namespace {
template <int K, int N>
int launch_head_gemm(const float* A, int64_t rows, int64_t lda, const __bf16* P, int epi, const float* bias,
                     uint32_t* relu_mask, float* out, float* part, hipStream_t s) {
  using HS = HeadShape<K, N>;
  // tiles per wave: enough row groups to give every CU one workgroup of the column slices
  const int64_t tile_rows = kWaves * kTileRows;
  const int64_t wgs_per_group = HS::kSlices;
  const int64_t target_groups = 256 / wgs_per_group;
  const int64_t tiles = std::max<int64_t>(1, (rows + tile_rows * target_groups - 1) / (tile_rows * target_groups));
  const int64_t groups = (rows + tiles * tile_rows - 1) / (tiles * tile_rows);
  const int64_t padded = (groups + 7) / 8 * 8;  // head_block: 8 groups per 8 * kSlices blocks
  const dim3 grid((unsigned)(padded * HS::kSlices)), block(256);
  const int G = (int)groups, T = (int)tiles;
  constexpr int L = HS::kSliceB;
  switch (epi) {
    case EPI_BIAS_RELU: head_gemm_kernel<EPI_BIAS_RELU, K, N><<<grid, block, L, s>>>(A, rows, lda, P, bias, relu_mask, out, part, G, T); break;
    case EPI_BIAS_L2: head_gemm_kernel<EPI_BIAS_L2, K, N><<<grid, block, L, s>>>(A, rows, lda, P, bias, relu_mask, out, part, G, T); break;
    case EPI_RELU_MASK: head_gemm_kernel<EPI_RELU_MASK, K, N><<<grid, block, L, s>>>(A, rows, lda, P, bias, relu_mask, out, part, G, T); break;
    case EPI_ROWDIV: head_gemm_kernel<EPI_ROWDIV, K, N><<<grid, block, L, s>>>(A, rows, lda, P, bias, relu_mask, out, part, G, T); break;
    default: head_gemm_kernel<EPI_PLAIN, K, N><<<grid, block, L, s>>>(A, rows, lda, P, bias, relu_mask, out, part, G, T); break;
  }
  TT_LAUNCH_CHECK("tt_head_gemm");
  return TT_OK;
}
}  // namespace
}  // namespace tt

extern "C" int tt_head_gemm(const float* A, int64_t rows, int64_t lda, int K, const void* planes, int N, int epi,
                            const float* bias, uint32_t* relu_mask, float* out, float* norms, void* ws,
                            size_t ws_bytes, tt_stream_t stream) {
  TT_REQUIRE(emb_width_ok(K) && emb_width_ok(N) && (K > 64 || N > 64), "tt_head_gemm: K, N in {64, 128, 256}, not both 64 (got K=%d N=%d)", K, N);
  TT_REQUIRE(rows >= 0 && lda >= K, "bad shape rows=%lld lda=%lld", (long long)rows, (long long)lda);
  if (rows == 0) return TT_OK;
  TT_REQUIRE(rows < (int64_t(1) << 31), "rows=%lld too large", (long long)rows);
  TT_REQUIRE(A && planes && out, "null pointer");
  TT_REQUIRE(((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(planes) |
               reinterpret_cast<uintptr_t>(out)) & 15) == 0 && lda % 4 == 0,
             "A / planes / out must be 16-byte aligned");
  // epi 4: the Linear of epi 1 without its normalise pass (tt_inbatch_l2_prep normalises)
  const bool defer_l2 = epi == 4;
  if (defer_l2) epi = EPI_BIAS_L2;
  TT_REQUIRE((epi >= EPI_BIAS_RELU && epi <= EPI_PLAIN) || epi == EPI_ROWDIV, "epi=%d", epi);
  TT_REQUIRE(epi != EPI_ROWDIV || bias, "epilogue 5 needs the row divisors (bias)");
  TT_REQUIRE((epi != EPI_BIAS_RELU && epi != EPI_BIAS_L2) || bias, "epilogue needs bias");
  TT_REQUIRE(epi != EPI_RELU_MASK || relu_mask, "epilogue needs the ReLU mask of the forward");
  TT_REQUIRE(epi != EPI_BIAS_L2 || norms || defer_l2, "epilogue needs norms");
  TT_REQUIRE(ws_bytes >= tt_head_gemm_ws_size(rows, epi) && (ws || !tt_head_gemm_ws_size(rows, epi)),
             "workspace too small (%zu < %zu)", ws_bytes, tt_head_gemm_ws_size(rows, epi));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const __bf16* P = static_cast<const __bf16*>(planes);
  float* part = static_cast<float*>(ws);
  int rc;
  TT_REQUIRE(N > 64 || (epi != EPI_BIAS_L2 && epi != EPI_BIAS_RELU), "tt_head_gemm: N = 64 only for the dx GEMMs (epi 3, 5)");
  TT_REQUIRE(K > 64 || epi == EPI_BIAS_RELU || (epi == EPI_BIAS_L2 && defer_l2),
             "tt_head_gemm: K = 64 only for a first Linear (epi 0, or epi 4: AveragePoolingTower's projection)");
#define TT_HG(KK, NN) \
  if (K == KK && N == NN) rc = launch_head_gemm<KK, NN>(A, rows, lda, P, epi, bias, relu_mask, out, part, s)
  TT_HG(256, 256);
  else TT_HG(128, 128);
  else TT_HG(256, 128);
  else TT_HG(128, 256);
  else TT_HG(64, 128);
  else TT_HG(64, 256);
  else TT_HG(128, 64);
  else TT_HG(256, 64);
  else rc = TT_ERR_UNSUPPORTED;
#undef TT_HG
  if (rc) return rc;
  if (epi == EPI_BIAS_L2 && !defer_l2) {
    if (N == 256) head_normalize_kernel<256><<<dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s>>>(out, rows, part, norms);
    else head_normalize_kernel<128><<<dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s>>>(out, rows, part, norms);
    TT_LAUNCH_CHECK("tt_head_gemm normalize");
  }
  return TT_OK;
}

// Both weight gradients of a head in one launch (one round of 256 workgroups over the two
// problems): (dW1, db1) from (G1, X1) and (dW2, db2) from (G2, X2), slab partials into ws; the
// fixed-order slab sums in a second call (tt_head_wgrad2_reduce), which a caller may queue later
// on another stream.  Deterministic.  N = K (the head width, 128 or 256).
extern "C" size_t tt_head_wgrad2_ws_size(int64_t rows, int N) {
  (void)rows;
  if (!head_width_ok(N)) return 0;
  return (size_t)2 * wg_slabs2(N) * N * (N + 1) * sizeof(float);
}

extern "C" int tt_head_wgrad2(const float* G1, const float* X1, const float* G2, const float* X2, int64_t rows, int N,
                              void* ws, size_t ws_bytes, tt_stream_t stream) {
  TT_REQUIRE(head_width_ok(N), "tt_head_wgrad2: N in {128, 256} (got %d)", N);
  TT_REQUIRE(rows >= 0, "bad rows %lld", (long long)rows);
  TT_REQUIRE(rows == 0 || (G1 && X1 && G2 && X2), "null pointer");
  TT_REQUIRE(ws && ws_bytes >= tt_head_wgrad2_ws_size(rows, N), "workspace too small (%zu < %zu)", ws_bytes,
             tt_head_wgrad2_ws_size(rows, N));
  TT_REQUIRE(((reinterpret_cast<uintptr_t>(G1) | reinterpret_cast<uintptr_t>(X1) | reinterpret_cast<uintptr_t>(G2) |
               reinterpret_cast<uintptr_t>(X2) | reinterpret_cast<uintptr_t>(ws)) & 15) == 0,
             "buffers must be 16-byte aligned");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (rows == 0) {  // zero partials: the reduce then writes zero gradients
    TT_HIP(hipMemsetAsync(ws, 0, tt_head_wgrad2_ws_size(rows, N), s), "memset wgrad2 partials");
    return TT_OK;
  }
  const int slabs = wg_slabs2(N), nb = wg_blocks(N) * slabs;
  float* pw1 = static_cast<float*>(ws);
  float* pb1 = pw1 + (size_t)slabs * N * N;
  float* pw2 = pb1 + (size_t)slabs * N;
  float* pb2 = pw2 + (size_t)slabs * N * N;
  constexpr int64_t kQuant = 3 * kWgChunk;
  const int64_t slab_rows = std::max<int64_t>(kQuant, (rows + slabs * kQuant - 1) / (slabs * kQuant) * kQuant);
  if (N == 256)
    head_wgrad_kernel<256, 256><<<dim3(2 * nb), dim3(256), 2 * kWgBuf, s>>>(G1, X1, rows, slab_rows, pw1, pb1,
                                                                           WgradProblem2{G2, X2, pw2, pb2, nb});
  else
    head_wgrad_kernel<128, 128><<<dim3(2 * nb), dim3(256), 2 * kWgBuf, s>>>(G1, X1, rows, slab_rows, pw1, pb1,
                                                                           WgradProblem2{G2, X2, pw2, pb2, nb});
  TT_LAUNCH_CHECK("tt_head_wgrad2");
  return TT_OK;
}

extern "C" int tt_head_wgrad2_reduce(const void* ws, int N, float* dW1, float* db1, float* dW2, float* db2,
                                     tt_stream_t stream) {
  TT_REQUIRE(head_width_ok(N), "tt_head_wgrad2_reduce: N in {128, 256} (got %d)", N);
  TT_REQUIRE(ws && dW1 && db1 && dW2 && db2, "null pointer");
  TT_REQUIRE(((reinterpret_cast<uintptr_t>(ws) | reinterpret_cast<uintptr_t>(dW1) | reinterpret_cast<uintptr_t>(db1) |
               reinterpret_cast<uintptr_t>(dW2) | reinterpret_cast<uintptr_t>(db2)) & 15) == 0,
             "buffers must be 16-byte aligned");
  const int slabs = wg_slabs2(N);
  const float* pw1 = static_cast<const float*>(ws);
  const float* pb1 = pw1 + (size_t)slabs * N * N;
  const float* pw2 = pb1 + (size_t)slabs * N;
  const float* pb2 = pw2 + (size_t)slabs * N * N;
  const int nb = N * N / 4 / 64 + 1;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (N == 256)
    head_wgrad_reduce_kernel<256, 256><<<dim3(2 * nb), dim3(256), 0, s>>>(pw1, pb1, slabs, dW1, db1,
                                                                         WgradReduce2{pw2, pb2, dW2, db2, nb});
  else
    head_wgrad_reduce_kernel<128, 128><<<dim3(2 * nb), dim3(256), 0, s>>>(pw1, pb1, slabs, dW1, db1,
                                                                         WgradReduce2{pw2, pb2, dW2, db2, nb});
  TT_LAUNCH_CHECK("tt_head_wgrad2_reduce");
  return TT_OK;
}

extern "C" int tt_head_wgrad2_parts(int N, int k, int64_t* offset, int64_t* stride) {
  if (!head_width_ok(N) || k < 0 || k > 3 || !offset || !stride) {
    set_error("tt_head_wgrad2_parts: N=%d k=%d", N, k);
    return -1;
  }
  // ws layout (tt_head_wgrad2): dW1 slabs, db1 slabs, dW2 slabs, db2 slabs
  const int slabs = wg_slabs2(N);
  const int64_t w = (int64_t)slabs * N * N, b = (int64_t)slabs * N;
  const int64_t off[4] = {0, w, w + b, 2 * w + b};
  *offset = off[k];
  *stride = (k & 1) ? N : (int64_t)N * N;
  return slabs;
}

namespace tt {
namespace {
template <int NG, int NX>
void launch_wgrad(const float* G, const float* X, int64_t rows, int64_t slab_rows, int slabs, float* part_w,
                  float* part_b, float* dW, float* db, hipStream_t s) {
  head_wgrad_kernel<NG, NX><<<dim3(wg_blocks2(NG, NX) * slabs), dim3(256), 2 * kWgBuf, s>>>(G, X, rows, slab_rows,
                                                                                          part_w, db ? part_b : nullptr);
  const int nred = NG * NX / 4 / 64 + 1;
  head_wgrad_reduce_kernel<NG, NX><<<dim3(nred), dim3(256), 0, s>>>(part_w, part_b, slabs, dW, db);
}
}  // namespace
}  // namespace tt

// dW = G^T X (NG x NX) and db = colsum G (NG): NG = H in {128, 256}, NX in {64, 128, 256} (the
// first Linear's input width E, or H).
extern "C" size_t tt_head_wgrad_ex_ws_size(int64_t rows, int NG, int NX) {
  (void)rows;
  if (!head_width_ok(NG) || !emb_width_ok(NX)) return 0;
  return (size_t)wg_slabs_ex(NG, NX) * NG * (NX + 1) * sizeof(float);
}

extern "C" int tt_head_wgrad_ex(const float* G, const float* X, int64_t rows, int NG, int NX, float* dW, float* db,
                                void* ws, size_t ws_bytes, tt_stream_t stream) {
  TT_REQUIRE(head_width_ok(NG) && emb_width_ok(NX), "tt_head_wgrad_ex: NG in {128, 256}, NX in {64, 128, 256} (got %dx%d)",
             NG, NX);
  TT_REQUIRE(rows >= 0, "bad rows %lld", (long long)rows);
  TT_REQUIRE(dW && (rows == 0 || (G && X)), "null pointer");
  TT_REQUIRE(ws && ws_bytes >= tt_head_wgrad_ex_ws_size(rows, NG, NX), "workspace too small (%zu < %zu)", ws_bytes,
             tt_head_wgrad_ex_ws_size(rows, NG, NX));
  TT_REQUIRE(((reinterpret_cast<uintptr_t>(G) | reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(dW) |
               reinterpret_cast<uintptr_t>(db) | reinterpret_cast<uintptr_t>(ws)) & 15) == 0,
             "buffers must be 16-byte aligned");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (rows == 0) {  // the kernel's clamped loads need row 0 to exist
    TT_HIP(hipMemsetAsync(dW, 0, (size_t)NG * NX * sizeof(float), s), "memset dW");
    if (db) TT_HIP(hipMemsetAsync(db, 0, (size_t)NG * sizeof(float), s), "memset db");
    return TT_OK;
  }
  const int slabs = wg_slabs_ex(NG, NX);
  float* part_w = static_cast<float*>(ws);
  float* part_b = part_w + (size_t)slabs * NG * NX;
  // slab rows: a multiple of the chunk, every slab launched (empty slabs write zero partials)
  constexpr int64_t kQuant = 3 * kWgChunk;  // whole ring turns (kRing chunks) per slab
  const int64_t slab_rows = std::max<int64_t>(kQuant, (rows + slabs * kQuant - 1) / (slabs * kQuant) * kQuant);
#define TT_WG(A, B) \
  if (NG == A && NX == B) launch_wgrad<A, B>(G, X, rows, slab_rows, slabs, part_w, part_b, dW, db, s)
  TT_WG(256, 256);
  else TT_WG(128, 128);
  else TT_WG(128, 64);
  else TT_WG(256, 64);
  else TT_WG(256, 128);
  else TT_WG(128, 256);
#undef TT_WG
  TT_LAUNCH_CHECK("tt_head_wgrad_ex");
  return TT_OK;
}

extern "C" size_t tt_head_wgrad_ws_size(int64_t rows, int N) { return tt_head_wgrad_ex_ws_size(rows, N, N); }

extern "C" int tt_head_wgrad(const float* G, const float* X, int64_t rows, int N, float* dW, float* db, void* ws,
                             size_t ws_bytes, tt_stream_t stream) {
  TT_REQUIRE(head_width_ok(N), "tt_head_wgrad: N in {128, 256} (got %d)", N);
  return tt_head_wgrad_ex(G, X, rows, N, N, dW, db, ws, ws_bytes, stream);
}
