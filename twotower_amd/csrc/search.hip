// Search over an indexed document set (inference/search/two_tower.py:72-115, evaluate.py:159-199):
//   scores[i, j] = cosine_similarity(q_i, d_j)     (torch.nn.functional.cosine_similarity, eps 1e-8:
//                  each side divided by max(|x|, eps), then the dot product)
//   top-k of each score row, descending, ties broken by the lower document index.
//
// cosine kernel: HBM-bound on the document matrix (nd x H fp32, read once per pass of up to
// kQ queries).  One wave per document row; the queries' normalised rows sit in LDS; each lane
// holds 4 consecutive features (16 B loads, a 1 KiB row per wave-instruction at H = 256).
// top-k kernel: exact radix select per row (one 256-thread workgroup per row): four 8-bit digit
// passes over the order-preserving uint32 image of the scores find the k-th largest value, a
// collect pass gathers everything above it plus the lowest-index ties, and a bitonic sort in
// LDS orders the k survivors.
#include <cstring>

#include "common.hpp"

namespace tt {
namespace {

constexpr int kQ = 8;            // queries per cosine pass
constexpr int kBlock = 256;
constexpr int kTopkMax = 1024;   // k limit (LDS sort of kTopkMax keys + indices)
constexpr float kCosEps = 1e-8f;

__global__ __launch_bounds__(kBlock) void cosine_scores_kernel(const float* __restrict__ q, int nq,
                                                               const float* __restrict__ docs, int64_t nd, int H,
                                                               float* __restrict__ scores, int64_t ld_scores) {
  extern __shared__ float qs[];  // nq x H normalised query rows
  const int lane = lane_id(), wid = threadIdx.x >> 6;
  // normalise the queries (each wave takes some rows), ATen: x / max(|x|, eps)
  for (int i = wid; i < nq; i += kBlock / kWave) {
    float ss = 0.f;
    for (int h = lane; h < H; h += kWave) ss += q[(int64_t)i * H + h] * q[(int64_t)i * H + h];
    const float inv = 1.f / fmaxf(sqrtf(wave_sum(ss)), kCosEps);
    for (int h = lane; h < H; h += kWave) qs[i * H + h] = q[(int64_t)i * H + h] * inv;
  }
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * (kBlock / kWave);
  for (int64_t j = (int64_t)blockIdx.x * (kBlock / kWave) + wid; j < nd; j += stride) {
    const float* row = docs + j * H;
    float dot[kQ];
#pragma unroll
    for (int i = 0; i < kQ; ++i) dot[i] = 0.f;
    float ss = 0.f;
    for (int c = lane; c < H / 4; c += kWave) {
      const f32x4 v = reinterpret_cast<const f32x4*>(row)[c];
      ss += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
#pragma unroll
      for (int i = 0; i < kQ; ++i) {
        if (i < nq) {
          const f32x4 w = *reinterpret_cast<const f32x4*>(qs + i * H + 4 * c);
          dot[i] += v[0] * w[0] + v[1] * w[1] + v[2] * w[2] + v[3] * w[3];
        }
      }
    }
    const float inv = 1.f / fmaxf(sqrtf(wave_sum(ss)), kCosEps);
#pragma unroll
    for (int i = 0; i < kQ; ++i) {
      if (i < nq) {
        const float s = wave_sum(dot[i]) * inv;
        if (lane == 0) scores[(int64_t)i * ld_scores + j] = s;
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

__global__ __launch_bounds__(kBlock) void topk_rows_kernel(const float* __restrict__ scores, int64_t ncols, int k,
                                                           float* __restrict__ out_vals, int64_t* __restrict__ out_idx) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t sel_prefix, sel_mask, sel_need;  // digits fixed so far, how many still to take
  __shared__ uint32_t n_above, n_tie;
  __shared__ uint32_t skey[kTopkMax];
  __shared__ int32_t sidx[kTopkMax];
  const int64_t r = blockIdx.x;
  const float* row = scores + r * ncols;
  const int tid = threadIdx.x;
  if (tid == 0) {
    sel_prefix = 0;
    sel_mask = 0;
    sel_need = (uint32_t)k;
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
    if (tid == 0) {
      uint32_t need = sel_need, d = 255;
      for (;; --d) {  // from the largest digit down
        if (hist[d] >= need || d == 0) break;
        need -= hist[d];
      }
      sel_prefix = pre | (d << shift);
      sel_mask = msk | (255u << shift);
      sel_need = need;  // how many keys equal to the final threshold are taken
    }
    __syncthreads();
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
  const uint32_t above_total = (uint32_t)k - take_eq;
  for (int64_t j0 = 0; j0 < ncols; j0 += kBlock) {
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
  for (int i = tid; i < k; i += kBlock) {
    out_vals[r * k + i] = key2f(skey[i]);
    out_idx[r * k + i] = (int64_t)sidx[i];
  }
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
  TT_REQUIRE((size_t)kQ * H * 4 <= 64 * 1024, "H=%d too large", H);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t waves = nd;
  const unsigned grid = (unsigned)std::min<int64_t>((waves + 3) / 4, 256 * 8);
  for (int64_t i0 = 0; i0 < nq; i0 += kQ) {
    const int n = (int)std::min<int64_t>(kQ, nq - i0);
    cosine_scores_kernel<<<dim3(grid), dim3(kBlock), (size_t)n * H * 4, s>>>(q + i0 * H, n, docs, nd, H,
                                                                            scores + i0 * nd, nd);
    TT_LAUNCH_CHECK("tt_cosine_scores");
  }
  return TT_OK;
}

extern "C" int tt_topk_rows(const float* scores, int64_t nrows, int64_t ncols, int k, float* out_vals,
                            int64_t* out_idx, tt_stream_t stream) {
  TT_REQUIRE(nrows >= 0 && ncols >= 0, "bad shape");
  TT_REQUIRE(k >= 1 && k <= kTopkMax && k <= ncols, "k=%d must be in [1, min(%d, ncols=%lld)]", k, kTopkMax,
             (long long)ncols);
  TT_REQUIRE(ncols < (int64_t(1) << 31), "ncols too large");
  if (nrows == 0) return TT_OK;
  TT_REQUIRE(scores && out_vals && out_idx, "null pointer");
  topk_rows_kernel<<<dim3((unsigned)nrows), dim3(kBlock), 0, reinterpret_cast<hipStream_t>(stream)>>>(
      scores, ncols, k, out_vals, out_idx);
  TT_LAUNCH_CHECK("tt_topk_rows");
  return TT_OK;
}
