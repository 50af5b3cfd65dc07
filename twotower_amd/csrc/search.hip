// Search over an indexed document set (inference/search/two_tower.py:72-115, evaluate.py:159-199):
//   scores[i, j] = cosine_similarity(q_i, d_j)     (torch.nn.functional.cosine_similarity, eps 1e-8:
//                  each side divided by max(|x|, eps), then the dot product)
//   top-k of each score row, descending, ties broken by the lower document index.
//
// cosine kernel: HBM-bound on the document matrix (nd x H fp32, read once per pass of up to
// kQMax queries) for a few queries, FMA-bound for many; a lane owns documents (below).
// top-k: exact radix select by one 256-thread workgroup (topk_block): four 8-bit digit passes
// over the order-preserving uint32 image of the scores find the k-th largest value (the digit
// chosen by a one-wave scan of the histogram), a collect pass gathers everything above it plus
// the lowest-index ties, and a bitonic sort in LDS orders the k survivors.  Long rows run it in
// two stages (chunks of the row in parallel, then a merge of the chunks' candidates), so a row
// is not left to one CU.
#include <cstring>

#include "common.hpp"

namespace tt {
namespace {

constexpr int kBlock = 256;
constexpr int kTopkMax = 1024;   // k limit (LDS sort of kTopkMax keys + indices)
constexpr float kCosEps = 1e-8f;

// ---- cosine scores.  A lane owns documents, not features: a wave takes a tile of kDocsW = 128
// documents (lane l: documents l and l + 64) and streams them in kFC-feature chunks through a
// wave-private LDS image (rows padded to kFC + 4 floats, so each lane's 16-B reads of its own row
// hit distinct banks), while the pass's normalised queries sit in LDS and are read as broadcasts.
// Each product is an in-lane FMA: no cross-lane reduction per document (the previous one-wave-
// per-document form spent its time in 9 wave reductions per row).  The next chunk's global loads
// are issued before the current chunk's FMAs.  A pass covers up to kQMax queries; more take more
// passes over the documents.
constexpr int kFC = 32;                    // features per staged chunk
constexpr int kRowF = kFC + 4;             // padded LDS row (floats)
constexpr int kDocsW = 128;                // documents per wave tile (2 per lane)
constexpr int kQMax = 32;                  // queries per pass
constexpr int kLoadsW = kDocsW * kFC / 4 / kWave;  // f32x4 loads per lane per chunk (16)

template <int QP>
__global__ __launch_bounds__(kBlock) void cosine_scores_kernel(const float* __restrict__ q, int nq,
                                                               const float* __restrict__ docs, int64_t nd, int H,
                                                               float* __restrict__ scores, int64_t ld_scores) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int Hp = (H + kFC - 1) / kFC * kFC;
  float* qs = smem;                                              // QP x Hp normalised queries (zero padded)
  const int lane = lane_id(), wid = threadIdx.x >> 6;
  float* dl = smem + QP * Hp + wid * (kDocsW * kRowF);           // this wave's document image
  // normalise the queries (ATen: x / max(|x|, eps)); rows past nq and features past H are zero
  for (int i = wid; i < QP; i += kBlock / kWave) {
    float ss = 0.f;
    if (i < nq)
      for (int h = lane; h < H; h += kWave) ss += q[(int64_t)i * H + h] * q[(int64_t)i * H + h];
    const float inv = 1.f / fmaxf(sqrtf(wave_sum(ss)), kCosEps);
    for (int h = lane; h < Hp; h += kWave) qs[i * Hp + h] = (i < nq && h < H) ? q[(int64_t)i * H + h] * inv : 0.f;
  }
  __syncthreads();
  const int nchunks = Hp / kFC;
  const int64_t ntiles = (nd + kDocsW - 1) / kDocsW;
  const int64_t wstride = (int64_t)gridDim.x * (kBlock / kWave);
  // staging: load u of a chunk = row 8 u + lane / 8 of the tile, features 4 (lane % 8) .. + 3
  const int srow = lane >> 3, scol = (lane & 7) * 4;
  for (int64_t t = (int64_t)blockIdx.x * (kBlock / kWave) + wid; t < ntiles; t += wstride) {
    const int64_t j0 = t * kDocsW;
    auto load_chunk = [&](int c, f32x4 (&r)[kLoadsW]) {
#pragma unroll
      for (int u = 0; u < kLoadsW; ++u) {
        int64_t j = j0 + 8 * u + srow;
        j = j < nd ? j : nd - 1;  // rows past the end: a clamped row, never stored
        const int f = c * kFC + scol;
        r[u] = f < H ? *reinterpret_cast<const f32x4*>(docs + j * H + f) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    };
    f32x4 cur[kLoadsW];
    load_chunk(0, cur);
    float acc[QP][2], ss[2] = {0.f, 0.f};
#pragma unroll
    for (int i = 0; i < QP; ++i) acc[i][0] = acc[i][1] = 0.f;
    for (int c = 0; c < nchunks; ++c) {
#pragma unroll
      for (int u = 0; u < kLoadsW; ++u) *reinterpret_cast<f32x4*>(dl + (8 * u + srow) * kRowF + scol) = cur[u];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (c + 1 < nchunks) load_chunk(c + 1, cur);
      float part[QP][2];  // this chunk's sums (two-level: chunk sums of kFC products, then the row)
#pragma unroll
      for (int i = 0; i < QP; ++i) part[i][0] = part[i][1] = 0.f;
      const float* qc = qs + c * kFC;
#pragma unroll
      for (int f = 0; f < kFC; f += 4) {
        const f32x4 d0 = *reinterpret_cast<const f32x4*>(dl + lane * kRowF + f);
        const f32x4 d1 = *reinterpret_cast<const f32x4*>(dl + (lane + kWave) * kRowF + f);
        ss[0] += d0[0] * d0[0] + d0[1] * d0[1] + d0[2] * d0[2] + d0[3] * d0[3];
        ss[1] += d1[0] * d1[0] + d1[1] * d1[1] + d1[2] * d1[2] + d1[3] * d1[3];
#pragma unroll
        for (int i = 0; i < QP; ++i) {
          const f32x4 w = *reinterpret_cast<const f32x4*>(qc + i * Hp + f);  // same address: broadcast
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            part[i][0] = __builtin_fmaf(d0[e], w[e], part[i][0]);
            part[i][1] = __builtin_fmaf(d1[e], w[e], part[i][1]);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < QP; ++i) {
        acc[i][0] += part[i][0];
        acc[i][1] += part[i][1];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // reads of this image before the next writes
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t j = j0 + lane + h * kWave;
      const float inv = 1.f / fmaxf(sqrtf(ss[h]), kCosEps);
      if (j < nd) {
#pragma unroll
        for (int i = 0; i < QP; ++i)
          if (i < nq) scores[(int64_t)i * ld_scores + j] = acc[i][h] * inv;
      }
    }
  }
}

// ---- cosine scores on the matrix cores, for passes of more than kVALUMaxQ queries: the same sums
// as Q^ D^T with v_mfma_f32_32x32x2_f32 (fp32 products and accumulation).  A wave owns a tile of
// 32 documents (the B operand, staged through its LDS image in kMFC-feature chunks) against the
// pass's 32 or 64 normalised queries (the A operand, resident in LDS).  Step s of an 8-feature
// block pairs features (8b + s, 8b + 4 + s): lane (row r32, half hh) supplies feature 8b + 4hh + s
// of its query / document, so one 16-byte LDS read feeds four steps.  The document norms come
// from the same staged chunks (each half sums its features, one exchange joins the halves), and
// the accumulator layout gives each lane one document column: the division needs no shuffle.
constexpr int kMDocs = 32;
constexpr int kMFC = 64;
constexpr int kMRowF = kMFC + 4;
constexpr int kMLoads = kMDocs * kMFC / 4 / kWave;  // f32x4 staging loads per lane per chunk (8)
constexpr int kVALUMaxQ = 8;

template <int QT>
__global__ __launch_bounds__(kBlock) void cosine_mfma_kernel(const float* __restrict__ q, int nq,
                                                             const float* __restrict__ docs, int64_t nd, int H,
                                                             float* __restrict__ scores, int64_t ld_scores) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int Hp = (H + kMFC - 1) / kMFC * kMFC, Hq = Hp + 4;
  float* qs = smem;                                                // QT*32 x Hq normalised queries
  const int lane = lane_id(), wid = threadIdx.x >> 6, r32 = lane & 31, hh = lane >> 5;
  float* dl = smem + QT * 32 * Hq + wid * (kMDocs * kMRowF);
  for (int i = wid; i < QT * 32; i += kBlock / kWave) {
    float ss = 0.f;
    if (i < nq)
      for (int h = lane; h < H; h += kWave) ss += q[(int64_t)i * H + h] * q[(int64_t)i * H + h];
    const float inv = 1.f / fmaxf(sqrtf(wave_sum(ss)), kCosEps);
    for (int h = lane; h < Hp; h += kWave) qs[i * Hq + h] = (i < nq && h < H) ? q[(int64_t)i * H + h] * inv : 0.f;
  }
  __syncthreads();
  const int nchunks = Hp / kMFC;
  const int64_t ntiles = (nd + kMDocs - 1) / kMDocs;
  const int64_t wstride = (int64_t)gridDim.x * (kBlock / kWave);
  const int srow = lane >> 4, scol = (lane & 15) * 4;  // staging: load u = row 4u + srow, features scol..+3
  for (int64_t t = (int64_t)blockIdx.x * (kBlock / kWave) + wid; t < ntiles; t += wstride) {
    const int64_t j0 = t * kMDocs;
    auto load_chunk = [&](int c, f32x4 (&r)[kMLoads]) {
#pragma unroll
      for (int u = 0; u < kMLoads; ++u) {
        int64_t j = j0 + 4 * u + srow;
        j = j < nd ? j : nd - 1;  // rows past the end: a clamped row, never stored
        const int f = c * kMFC + scol;
        r[u] = f < H ? *reinterpret_cast<const f32x4*>(docs + j * H + f) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    };
    f32x4 cur[kMLoads];
    load_chunk(0, cur);
    f32x16 acc[QT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) acc[qt] = f32x16{};
    float ssp = 0.f;
    for (int c = 0; c < nchunks; ++c) {
#pragma unroll
      for (int u = 0; u < kMLoads; ++u) *reinterpret_cast<f32x4*>(dl + (4 * u + srow) * kMRowF + scol) = cur[u];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (c + 1 < nchunks) load_chunk(c + 1, cur);
#pragma unroll
      for (int b = 0; b < kMFC / 8; ++b) {
        const f32x4 bv = *reinterpret_cast<const f32x4*>(dl + r32 * kMRowF + 8 * b + 4 * hh);
        ssp += bv[0] * bv[0] + bv[1] * bv[1] + bv[2] * bv[2] + bv[3] * bv[3];
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
          const f32x4 av = *reinterpret_cast<const f32x4*>(qs + (qt * 32 + r32) * Hq + c * kMFC + 8 * b + 4 * hh);
#pragma unroll
          for (int st = 0; st < 4; ++st)
            acc[qt] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[st], bv[st], acc[qt], 0, 0, 0);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // reads of this image before the next writes
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    const float ss = ssp + __shfl_xor(ssp, 32);
    const float inv = 1.f / fmaxf(sqrtf(ss), kCosEps);
    const int64_t j = j0 + r32;
    if (j < nd) {
#pragma unroll
      for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int i = qt * 32 + (v & 3) + 8 * (v >> 2) + 4 * hh;
          if (i < nq) scores[(int64_t)i * ld_scores + j] = acc[qt][v] * inv;
        }
    }
  }
}

// order-preserving image: larger float -> larger unsigned
__device__ __forceinline__ uint32_t f2key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// Exact top-k of one row by one 256-thread workgroup; emit(i, value, position) receives the k
// survivors in order (value descending, position ascending among equal values).
template <class Emit>
__device__ __forceinline__ void topk_block(const float* __restrict__ row, int64_t ncols, int k, Emit emit) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t sel_prefix, sel_mask, sel_need;  // digits fixed so far, how many still to take
  __shared__ uint32_t sel_all;  // every key under the fixed digits is taken: no further digit needed
  __shared__ uint32_t n_above, n_tie;
  __shared__ uint32_t skey[kTopkMax];
  __shared__ int32_t sidx[kTopkMax];
  const int tid = threadIdx.x;
  if (tid == 0) {
    sel_prefix = 0;
    sel_mask = 0;
    sel_need = (uint32_t)k;
    sel_all = 0;
  }
  // 1. radix select of the k-th largest key, most significant digit first
  for (int shift = 24; shift >= 0; shift -= 8) {
    hist[tid] = 0;
    __syncthreads();
    const uint32_t pre = sel_prefix, msk = sel_mask;
    for (int64_t j = tid; j < ncols; j += kBlock) {
      const uint32_t key = f2key(row[j]);
      if ((key & msk) == pre) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid < kWave) {  // the digit: from the largest down, the first whose running count reaches need
      // lane l holds digits 255 - 4l .. 252 - 4l (descending); an inclusive scan over the lanes
      const int lane = tid;
      uint32_t c[4], tot = 0;
#pragma unroll
      for (int t = 0; t < 4; ++t) tot += (c[t] = hist[255 - 4 * lane - t]);
      uint32_t inc = tot;
#pragma unroll
      for (int o = 1; o < kWave; o <<= 1) {
        const uint32_t v = __shfl_up(inc, o);
        if (lane >= o) inc += v;
      }
      const uint32_t need0 = sel_need;
      const uint64_t hit = __ballot(inc >= need0);
      const int L = hit ? __builtin_ctzll(hit) : kWave - 1;  // none: the last digit (0) takes the rest
      if (lane == L) {
        uint32_t need = need0 - (inc - tot), d = 255 - 4 * lane;
        for (int t = 0; t < 4; ++t, --d) {
          if (c[t] >= need || t == 3) break;
          need -= c[t];
        }
        sel_prefix = pre | (d << shift);
        sel_mask = msk | (255u << shift);
        sel_need = need;  // how many keys equal to the final threshold are taken
        sel_all = hist[d] == need;
      }
    }
    __syncthreads();
    if (sel_all) break;  // the digit's whole bucket is taken: the lower digits decide nothing
  }
  const uint32_t thr = sel_prefix, take_eq = sel_need;
  // 2. collect: every key above the threshold, then the take_eq lowest-index keys equal to it
  if (tid == 0) {
    n_above = 0;
    n_tie = 0;
  }
  for (int i = tid; i < kTopkMax; i += kBlock) {
    skey[i] = 0;
    sidx[i] = 0x7fffffff;
  }
  __syncthreads();
  if (sel_all) {
    // every key whose fixed digits reach the threshold's is taken (exactly k): slots in any order,
    // the sort below orders them
    const uint32_t msk = sel_mask;
    for (int64_t j = tid; j < ncols; j += kBlock) {
      const uint32_t key = f2key(row[j]);
      if ((key & msk) >= thr) {
        const uint32_t slot = atomicAdd(&n_above, 1u);
        skey[slot] = key;
        sidx[slot] = (int32_t)j;
      }
    }
    __syncthreads();
  }
  const uint32_t above_total = (uint32_t)k - take_eq;
  for (int64_t j0 = 0; j0 < (sel_all ? 0 : ncols); j0 += kBlock) {
    const int64_t j = j0 + tid;
    uint32_t key = 0;
    bool eq = false;
    if (j < ncols) {
      key = f2key(row[j]);
      if (key > thr) {
        const uint32_t slot = atomicAdd(&n_above, 1u);
        skey[slot] = key;
        sidx[slot] = (int32_t)j;
      }
      eq = key == thr;
    }
    // ties in index order: a block-wide ordered count per chunk (ballots per wave)
    const uint64_t m = __ballot(eq);
    __shared__ uint32_t wave_eq[kBlock / kWave];
    const int lane = lane_id(), wid = tid >> 6;
    if (lane == 0) wave_eq[wid] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t before = n_tie;
    for (int w = 0; w < wid; ++w) before += wave_eq[w];
    before += (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    if (eq && before < take_eq) {
      skey[above_total + before] = key;
      sidx[above_total + before] = (int32_t)j;
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t t = 0;
      for (int w = 0; w < kBlock / kWave; ++w) t += wave_eq[w];
      n_tie += t;
    }
    __syncthreads();
  }
  // 3. bitonic sort of the k (padded to a power of two) survivors: key desc, index asc
  int n2 = 1;
  while (n2 < k) n2 <<= 1;
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < n2; i += kBlock) {
        const int partner = i ^ stride;
        if (partner > i) {
          const bool desc = (i & size) == 0;
          const uint32_t ka = skey[i], kb = skey[partner];
          const int32_t ia = sidx[i], ib = sidx[partner];
          // "a before b" when a's key is larger, or equal with the lower index
          const bool a_first = ka > kb || (ka == kb && ia < ib);
          if (a_first != desc) {
            skey[i] = kb;
            skey[partner] = ka;
            sidx[i] = ib;
            sidx[partner] = ia;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < k; i += kBlock) emit(i, key2f(skey[i]), sidx[i]);
}

// one workgroup per row (rows short enough that a second stage would not pay)
__global__ __launch_bounds__(kBlock) void topk_rows_kernel(const float* __restrict__ scores, int64_t ncols, int k,
                                                           float* __restrict__ out_vals, int64_t* __restrict__ out_idx) {
  const int64_t r = blockIdx.x;
  topk_block(scores + r * ncols, ncols, k, [&](int i, float v, int32_t pos) {
    out_vals[r * k + i] = v;
    out_idx[r * k + i] = (int64_t)pos;
  });
}

// Two stages for long rows.  Stage 1: the row is cut into nch chunks of C columns (the last one
// takes the remainder, so every chunk holds >= k); workgroup (c, r) writes its chunk's exact top k
// as (value, column) candidates.  Stage 2: one workgroup per row takes the top k of the nch * k
// candidates.  Every member of the row's top k is in its chunk's top k, and among candidates of
// equal value the position order is the column order (chunks in column order, each chunk's list
// sorted by column among equal values), so breaking ties by position breaks them by column.
__global__ __launch_bounds__(kBlock) void topk_chunks_kernel(const float* __restrict__ scores, int64_t ncols, int k,
                                                             int64_t C, int nch, float* __restrict__ cand_val,
                                                             int32_t* __restrict__ cand_idx) {
  const int c = blockIdx.x;
  const int64_t r = blockIdx.y;
  const int64_t c0 = (int64_t)c * C, n = c + 1 < nch ? C : ncols - c0;
  const int64_t o = (r * nch + c) * k;
  topk_block(scores + r * ncols + c0, n, k, [&](int i, float v, int32_t pos) {
    cand_val[o + i] = v;
    cand_idx[o + i] = (int32_t)(c0 + pos);
  });
}

__global__ __launch_bounds__(kBlock) void topk_merge_kernel(const float* __restrict__ cand_val,
                                                            const int32_t* __restrict__ cand_idx, int nch, int k,
                                                            float* __restrict__ out_vals, int64_t* __restrict__ out_idx) {
  const int64_t r = blockIdx.x;
  const int64_t m = (int64_t)nch * k;
  const int32_t* ci = cand_idx + r * m;
  topk_block(cand_val + r * m, m, k, [&](int i, float v, int32_t pos) {
    out_vals[r * k + i] = v;
    out_idx[r * k + i] = (int64_t)ci[pos];
  });
}

// chunk length of the two-stage form: about sqrt(ncols k) (balances the stages), >= 2048 and
// >= 2k; 0 when the row is too short for two stages
inline int64_t topk_chunk(int64_t ncols, int k) {
  int64_t C = 2048;
  while (C * C < ncols * (int64_t)k) C <<= 1;
  while (C < 2 * (int64_t)k) C <<= 1;
  return ncols >= 4 * C ? C : 0;
}

}  // namespace
}  // namespace tt

using namespace tt;

extern "C" int tt_cosine_scores(const float* q, int64_t nq, const float* docs, int64_t nd, int H, float* scores,
                                tt_stream_t stream) {
  TT_REQUIRE(nq >= 0 && nd >= 0 && H > 0 && H % 4 == 0, "bad shape nq=%lld nd=%lld H=%d (H %% 4 == 0)",
             (long long)nq, (long long)nd, H);
  if (nq == 0 || nd == 0) return TT_OK;
  TT_REQUIRE(q && docs && scores, "null pointer");
  TT_REQUIRE((reinterpret_cast<uintptr_t>(docs) & 15) == 0, "docs must be 16-byte aligned");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int Hp = (H + kFC - 1) / kFC * kFC;
  const int64_t ntiles = (nd + kDocsW - 1) / kDocsW;
  // queries per pass: up to kQMax, as many (a power of two) as fit the LDS beside the document images
  const size_t doc_lds = (size_t)(kBlock / kWave) * kDocsW * kRowF * 4, q_row = (size_t)Hp * 4;
  int qcap = kQMax;
  while (qcap > 1 && doc_lds + qcap * q_row > 160 * 1024) qcap >>= 1;
  TT_REQUIRE(doc_lds + q_row <= 160 * 1024, "H=%d too large for the cosine kernel's LDS", H);
  // the matrix-core form: 64 (or 32) queries per pass when its LDS fits
  const int Hm = (H + kMFC - 1) / kMFC * kMFC;
  const size_t mdoc_lds = (size_t)(kBlock / kWave) * kMDocs * kMRowF * 4, mq_rows = (size_t)(Hm + 4) * 4 * 32;
  const int mqt = mdoc_lds + 2 * mq_rows <= 160 * 1024 ? 2 : mdoc_lds + mq_rows <= 160 * 1024 ? 1 : 0;
  const int64_t mtiles = (nd + kMDocs - 1) / kMDocs;
  for (int64_t i0 = 0; i0 < nq;) {
    const int64_t rest = nq - i0;
    const float* qi = q + i0 * H;
    float* si = scores + i0 * nd;
    if (mqt > 0 && rest > kVALUMaxQ) {
      const int n = (int)std::min<int64_t>(32 * mqt, rest);
      const int QT = n > 32 ? 2 : 1;
      const size_t lds = mdoc_lds + QT * mq_rows;
      const unsigned grid = (unsigned)std::min<int64_t>((mtiles + 3) / 4, 256 * 4);
      if (QT == 2)
        cosine_mfma_kernel<2><<<dim3(grid), dim3(kBlock), lds, s>>>(qi, n, docs, nd, H, si, nd);
      else
        cosine_mfma_kernel<1><<<dim3(grid), dim3(kBlock), lds, s>>>(qi, n, docs, nd, H, si, nd);
      TT_LAUNCH_CHECK("tt_cosine_scores (mfma)");
      i0 += n;
      continue;
    }
    const int n = (int)std::min<int64_t>(qcap, rest);
    const int QP = n <= 1 ? 1 : n <= 2 ? 2 : n <= 4 ? 4 : n <= 8 ? 8 : n <= 16 ? 16 : 32;
    const size_t lds = doc_lds + (size_t)QP * q_row;
    // one tile per wave until every CU holds a workgroup, then the waves walk tiles
    const unsigned grid = (unsigned)std::min<int64_t>((ntiles + 3) / 4, 256 * 4);
    switch (QP) {
#define TT_COS_CASE(P)                                                                                         \
  case P:                                                                                                      \
    cosine_scores_kernel<P><<<dim3(grid), dim3(kBlock), lds, s>>>(qi, n, docs, nd, H, si, nd);                 \
    break;
      TT_COS_CASE(1) TT_COS_CASE(2) TT_COS_CASE(4) TT_COS_CASE(8) TT_COS_CASE(16) TT_COS_CASE(32)
#undef TT_COS_CASE
    }
    TT_LAUNCH_CHECK("tt_cosine_scores");
    i0 += n;
  }
  return TT_OK;
}

extern "C" size_t tt_topk_rows_ws_size(int64_t nrows, int64_t ncols, int k) {
  if (nrows <= 0 || k < 1) return 0;
  const int64_t C = topk_chunk(ncols, k);
  if (C == 0) return 0;
  const int64_t nch = ncols / C;
  return (size_t)nrows * nch * k * (sizeof(float) + sizeof(int32_t));
}

extern "C" int tt_topk_rows_ex(const float* scores, int64_t nrows, int64_t ncols, int k, void* ws, size_t ws_bytes,
                               float* out_vals, int64_t* out_idx, tt_stream_t stream) {
  TT_REQUIRE(nrows >= 0 && ncols >= 0, "bad shape");
  TT_REQUIRE(k >= 1 && k <= kTopkMax && k <= ncols, "k=%d must be in [1, min(%d, ncols=%lld)]", k, kTopkMax,
             (long long)ncols);
  TT_REQUIRE(ncols < (int64_t(1) << 31), "ncols too large");
  if (nrows == 0) return TT_OK;
  TT_REQUIRE(scores && out_vals && out_idx, "null pointer");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const size_t need = tt_topk_rows_ws_size(nrows, ncols, k);
  if (need == 0 || ws == nullptr) {  // short rows, or no workspace: one workgroup per row
    topk_rows_kernel<<<dim3((unsigned)nrows), dim3(kBlock), 0, s>>>(scores, ncols, k, out_vals, out_idx);
    TT_LAUNCH_CHECK("tt_topk_rows");
    return TT_OK;
  }
  TT_REQUIRE(ws_bytes >= need, "topk workspace %zu bytes < %zu", ws_bytes, need);
  const int64_t C = topk_chunk(ncols, k);
  const int nch = (int)(ncols / C);
  float* cv = reinterpret_cast<float*>(ws);
  int32_t* ci = reinterpret_cast<int32_t*>(cv + (size_t)nrows * nch * k);
  // rows ride grid.y (at most 65,535): longer query batches go in row blocks of that many
  constexpr int64_t kRowBlock = 65535;
  for (int64_t r0 = 0; r0 < nrows; r0 += kRowBlock) {
    const int64_t nr = std::min<int64_t>(kRowBlock, nrows - r0);
    const size_t co = (size_t)r0 * nch * k;
    topk_chunks_kernel<<<dim3((unsigned)nch, (unsigned)nr), dim3(kBlock), 0, s>>>(scores + r0 * ncols, ncols, k, C,
                                                                                   nch, cv + co, ci + co);
    TT_LAUNCH_CHECK("tt_topk_rows (chunks)");
    topk_merge_kernel<<<dim3((unsigned)nr), dim3(kBlock), 0, s>>>(cv + co, ci + co, nch, k, out_vals + r0 * k,
                                                                  out_idx + r0 * k);
    TT_LAUNCH_CHECK("tt_topk_rows (merge)");
  }
  return TT_OK;
}

extern "C" int tt_topk_rows(const float* scores, int64_t nrows, int64_t ncols, int k, float* out_vals,
                            int64_t* out_idx, tt_stream_t stream) {
  return tt_topk_rows_ex(scores, nrows, ncols, k, nullptr, 0, out_vals, out_idx, stream);
}
