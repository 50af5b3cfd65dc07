// Embedding bag on gfx950: lookup + masked mean-pool forward, sorted / atomic scatter-add
// backward, and the sorted backward fused with a dense AdamW step on the table.
//
// Reference semantics (k0r1g/two-towers):
//   twotower/embeddings.py:30,40  nn.Embedding(V, E, padding_idx=0)(ids)
//   twotower/encoders.py:62       mask = (ids > 0).float()
//   twotower/encoders.py:67       emb = embedding(ids) * mask
//   twotower/encoders.py:72       pooled = emb.sum(1) / (mask.sum(1) + 1e-9)
//   backward (twotower/train.py:138): G[id] += dpooled[s] / denom[s] for non-pad tokens,
//   dense V x E gradient, padding row excluded (embedding_dense_backward).
//
// Layout: the table is V x E fp32 row-major (1 KiB rows at E = 256).  A wavefront owns a
// sequence (forward) or a table row (backward).  Each lane moves 16 B per row-load so a
// wave-instruction reads 64 x 16 B = 1 KiB: one E=256 row, two E=128 rows or four E=64 rows.
#include <algorithm>
#include <cstdlib>
#include <cstring>


#include "common.hpp"

namespace tt {
namespace {

constexpr int kBlock = 256;                 // 4 waves per workgroup
constexpr int kWavesPerBlock = kBlock / kWave;

// ---------------------------------------------------------------------------------------
// Forward: one wave per sequence.  LPR lanes cover one row with NV float4 each
// (E = 4 * LPR * NV); RPI = 64 / LPR rows are in flight per wave-instruction and U such
// instructions are issued before the adds, so each wave keeps U * 1 KiB of gathers in flight.
// Token order is preserved per sub-row (sequential adds), sub-rows are folded at the end.
// The first split_blocks workgroups (tt_bag_mean_fwd_split) form the tower head's weight planes
// instead (SplitJobs, common.hpp: the bits of tt_head_split_ff2), one element of each job per
// thread: the split rides in the gather's launch, off the path between it and the first head GEMM.
template <typename IdT, int LPR, int NV, int U>
__global__ __launch_bounds__(kBlock) void bag_fwd_kernel(
    const float* __restrict__ table, int64_t V, int E, const IdT* __restrict__ ids, int64_t nseq,
    int L, int64_t ld, float* __restrict__ pooled, float* __restrict__ denom, SplitJobs sj,
    __bf16* __restrict__ planes, int split_blocks) {
  if ((int)blockIdx.x < split_blocks) {  // workgroup-uniform
    const int i = blockIdx.x * kBlock + threadIdx.x;
#pragma unroll
    for (int job = 0; job < 4; ++job) split_planes_elem(sj, job, i, planes);
    return;
  }
  constexpr int RPI = kWave / LPR;
  const int lane = lane_id();
  const int sub = lane / LPR, c = lane % LPR;
  // one wave per sequence (the loop also covers a grid smaller than the sequences)
  const int64_t nwaves = (int64_t)(gridDim.x - split_blocks) * kWavesPerBlock;
  for (int64_t seq = (int64_t)(blockIdx.x - split_blocks) * kWavesPerBlock + (threadIdx.x >> 6); seq < nseq;
       seq += nwaves) {
  const IdT* rid = ids + seq * ld;

  f32x4 acc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  int cnt = 0;

  for (int base = 0; base < L; base += kWave) {
    const int t = base + lane;
    const int64_t id = (t < L) ? (int64_t)rid[t] : 0;
    const bool valid = id > 0 && id < V;
    const int id32 = valid ? (int)id : 0;
    uint64_t m = __ballot(valid);
    cnt += __popcll(m);
    while (m) {
      int pos[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        int mine = -1;
#pragma unroll
        for (int s = 0; s < RPI; ++s) {
          if (m) {
            const int q = __builtin_ctzll(m);
            m &= m - 1;
            if (s == sub) mine = q;
          }
        }
        pos[u] = mine;
      }
      f32x4 v[U][NV];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        int r;
        if constexpr (RPI == 1) {
          r = __builtin_amdgcn_readlane(id32, pos[u] < 0 ? 0 : pos[u]);
        } else {
          r = __shfl(id32, pos[u] < 0 ? 0 : pos[u]);
        }
        const f32x4* rowp = reinterpret_cast<const f32x4*>(table + (int64_t)r * E);
#pragma unroll
        for (int k = 0; k < NV; ++k)
          v[u][k] = (pos[u] >= 0) ? rowp[k * LPR + c] : f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int k = 0; k < NV; ++k) acc[k] += v[u][k];
    }
  }
  if constexpr (RPI > 1) {
#pragma unroll
    for (int o = LPR; o < kWave; o <<= 1)
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        acc[k][0] += __shfl_xor(acc[k][0], o);
        acc[k][1] += __shfl_xor(acc[k][1], o);
        acc[k][2] += __shfl_xor(acc[k][2], o);
        acc[k][3] += __shfl_xor(acc[k][3], o);
      }
  }
  const float den = (float)cnt + 1e-9f;  // mask.sum(1) + 1e-9, encoders.py:72
  if (sub == 0) {
    f32x4* out = reinterpret_cast<f32x4*>(pooled + seq * E);
#pragma unroll
    for (int k = 0; k < NV; ++k) out[k * LPR + c] = acc[k] / den;
  }
  if (lane == 0) denom[seq] = den;
  }
}

// Column slab forward (table_sync "column"): pooled columns of a (V, El) slab summed in the
// order bag_fwd_kernel sums them at the full width E, so the pooled rows every rank assembles
// equal the one-GPU forward's bit for bit.  That order: valid token j of each 64-token chunk goes
// to sub-row j % RPIF (RPIF = 64 / LPR of the full-width launch: 4 at E = 64, 2 at E = 128, 1 from
// E = 256 on, where the sum is plain token order), each sub-row summed in token order, the
// sub-rows folded pairwise ((s0 + s1) + (s2 + s3): the butterfly's result in sub-row 0).  Here a
// wave holds 64 / LPRC sequences (LPRC = El / 4 lanes each), a lane keeps the RPIF sub-row sums of
// its float4 column, and U tokens' rows are in flight per step.
template <typename IdT, int LPRC, int RPIF, int U>
__global__ __launch_bounds__(kBlock) void bag_fwd_cols_kernel(
    const float* __restrict__ slab, int64_t V, int El, const IdT* __restrict__ ids, int64_t nseq, int L,
    int64_t ld, float* __restrict__ pooled, float* __restrict__ denom) {
  constexpr int SPW = kWave / LPRC;
  const int lane = lane_id(), g = lane / LPRC, c = lane % LPRC;
  const int64_t seq = ((int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * SPW + g;
  const bool live = seq < nseq;
  const IdT* rid = ids + (live ? seq : 0) * ld;
  f32x4 acc[RPIF];
#pragma unroll
  for (int r = 0; r < RPIF; ++r) acc[r] = f32x4{0.f, 0.f, 0.f, 0.f};
  int cnt = 0;
  for (int base = 0; base < L; base += kWave) {
    const int lim = L - base < kWave ? L - base : kWave;
    int j = 0;  // valid tokens of this chunk so far
    for (int t0 = 0; t0 < lim; t0 += U) {
      int id[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int t = t0 + u;
        const int64_t v = (live && t < lim) ? (int64_t)rid[base + t] : 0;
        id[u] = (v > 0 && v < V) ? (int)v : -1;
      }
      f32x4 x[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        x[u] = id[u] >= 0 ? reinterpret_cast<const f32x4*>(slab + (int64_t)id[u] * El)[c] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (id[u] >= 0) {
          if constexpr (RPIF == 1) {
            acc[0] += x[u];
          } else {
            const int r = j % RPIF;
#pragma unroll
            for (int k = 0; k < RPIF; ++k)
              if (k == r) acc[k] += x[u];
          }
          ++j;
        }
      }
    }
    cnt += j;
  }
  f32x4 sum = acc[0];
  if constexpr (RPIF == 2) sum = acc[0] + acc[1];
  if constexpr (RPIF == 4) sum = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  if (!live) return;
  const float den = (float)cnt + 1e-9f;  // mask.sum(1) + 1e-9, encoders.py:72
  reinterpret_cast<f32x4*>(pooled + seq * El)[c] = sum / den;
  if (c == 0) denom[seq] = den;
}

template <typename IdT>
int launch_fwd_cols(const float* slab, int64_t V, int El, int E, const IdT* ids, int64_t nseq, int L, int64_t ld,
                    float* pooled, float* denom, hipStream_t s) {
  const int rpif = E == 64 ? 4 : E == 128 ? 2 : 1;
  const int spw = kWave / (El / 4);
  const int64_t waves = (nseq + spw - 1) / spw;
  const dim3 grid((unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock)), block(kBlock);
#define TT_FC(LPRC, R) \
  bag_fwd_cols_kernel<IdT, LPRC, R, 8><<<grid, block, 0, s>>>(slab, V, El, ids, nseq, L, ld, pooled, denom)
#define TT_FCR(LPRC) \
  if (rpif == 4) TT_FC(LPRC, 4); else if (rpif == 2) TT_FC(LPRC, 2); else TT_FC(LPRC, 1)
  switch (El) {
    case 32: TT_FCR(8); break;
    case 64: TT_FCR(16); break;
    case 128: TT_FCR(32); break;
    default: TT_FCR(64); break;  // 256
  }
#undef TT_FCR
#undef TT_FC
  TT_LAUNCH_CHECK("tt_bag_mean_fwd_cols");
  return TT_OK;
}

// Any E: lanes stride the columns, tokens are walked one at a time (wave-uniform row).
template <typename IdT>
__global__ __launch_bounds__(kBlock) void bag_fwd_generic_kernel(
    const float* __restrict__ table, int64_t V, int E, const IdT* __restrict__ ids, int64_t nseq,
    int L, int64_t ld, float* __restrict__ pooled, float* __restrict__ denom) {
  const int lane = lane_id();
  const int64_t seq = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (seq >= nseq) return;
  const IdT* rid = ids + seq * ld;
  int cnt = 0;
  for (int base = 0; base < L; base += kWave) {
    const int t = base + lane;
    const int64_t id = (t < L) ? (int64_t)rid[t] : 0;
    cnt += __popcll(__ballot(id > 0 && id < V));
  }
  const float den = (float)cnt + 1e-9f;
  for (int c0 = 0; c0 < E; c0 += kWave) {
    const int c = c0 + lane;
    float acc = 0.f;
    for (int base = 0; base < L; base += kWave) {
      const int t = base + lane;
      const int64_t id = (t < L) ? (int64_t)rid[t] : 0;
      const bool valid = id > 0 && id < V;
      const int id32 = valid ? (int)id : 0;
      uint64_t m = __ballot(valid);
      while (m) {
        const int q = __builtin_ctzll(m);
        m &= m - 1;
        const int r = __builtin_amdgcn_readlane(id32, q);
        if (c < E) acc += table[(int64_t)r * E + c];
      }
    }
    if (c < E) pooled[seq * E + c] = acc / den;
  }
  if (lane == 0) denom[seq] = den;
}

// ---------------------------------------------------------------------------------------
// Backward, sorted (deterministic) path, in two halves:
//   plan  (ids only, may run as soon as the ids exist, e.g. beside the forward):
//         keys = row id (V for masked tokens), vals = seq -> stable LSD counting sort -> segment
//         bounds;
//   apply (needs d_pooled): gs[s] = dpooled[s] / denom[s] (the division autograd applies,
//         encoders.py:72), then the per-row reduce (optionally fused with AdamW).
__global__ __launch_bounds__(kBlock) void bag_scale_rows_kernel(const float* __restrict__ dpooled,
                                                                const float* __restrict__ denom, int64_t nseq,
                                                                int E, float* __restrict__ gs) {
  const int64_t seq = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (seq >= nseq) return;
  const int lane = lane_id();
  const float den = denom[seq];
  const float* src = dpooled + seq * E;
  float* dst = gs + seq * E;
  if ((E & 3) == 0) {
    for (int c = lane; c < E / 4; c += kWave)
      reinterpret_cast<f32x4*>(dst)[c] = reinterpret_cast<const f32x4*>(src)[c] / den;
  } else {
    for (int c = lane; c < E; c += kWave) dst[c] = src[c] / den;
  }
}

// Long rows (Zipf-hot ids) are split so no wave walks tens of thousands of tokens: a row with
// more than kPieceT tokens is cut into pieces of max(kPieceT, ceil(len / kMaxPieces)) tokens;
// one wave per piece sums its gs rows (token order) into a partial, and the row's reduce wave
// sums the <= kMaxPieces partials in piece order instead of the tokens.  Deterministic.
constexpr int kPieceT = 128;
constexpr int kMaxPieces = 256;

__device__ __forceinline__ int piece_len(int len) {
  const int t = (len + kMaxPieces - 1) / kMaxPieces;
  return t > kPieceT ? t : kPieceT;
}

// ---------------------------------------------------------------------------------------
// The plan's sort, hand-written: a least-significant-digit counting sort of the row keys in P
// passes of D <= 11 bits (C3: keys in [0, 200000], 18 bits = 2 passes of 9; C2: 2 of 8), each
// pass three launches with no inter-workgroup waiting:
//   count   one workgroup per tile of kSortTile consecutive entries: the tile's digit histogram
//           (LDS), written digit-major, cnt[d * ntiles + tile];
//   scan    one workgroup per digit: exclusive scan of its row over the tiles, in place, and the
//           row total;
//   scatter one workgroup per tile: digit base (exclusive scan of the totals + the tile's row
//           offset) + the entry's rank among the tile's entries of its digit, in entry order, so
//           every pass is stable and the result is THE stable sort of (key, seq) by key.
// Pass 0 reads the ids directly (the key and the sequence index are formed on the fly), so no
// keys/values arrays are staged, and drops the masked slots (pads, ids >= V: 46 % of C3's slots),
// so the later passes and the segment starts handle the tokens only; the tokens' order is the
// same as when the masked slots sorted last under key V.  The in-tile rank: entry j of a tile sits at wave j / 256,
// step (j / 64) % 4, lane j % 64; a wave forms each step's same-digit lane set with D ballots,
// and keeps its running per-digit counts in its own LDS row; the wave offsets per digit are an
// exclusive scan over the waves' rows.  Bytes per pass: keys (+ values) read twice, written once.
constexpr int kSortThreads = 512;  // (256: the C3 step 0.870-0.874 vs 0.861-0.863 ms, round 4)
constexpr int kSortWaves = kSortThreads / kWave;
constexpr int kSortIPT = 4;  // entries per thread per tile
constexpr int kSortTile = kSortThreads * kSortIPT;
constexpr int kSortMaxD = 11;
constexpr int kSortDefaultD = 9;

template <typename IdT>
struct SortSrc {  // pass 0: ids (keys == nullptr); later passes: the previous pass's output
  const IdT* ids;
  int64_t L, ld, V, padding_idx;
  const uint32_t* keys;
  const int32_t* vals;
  double inv_L;  // 1 / L: the entry -> (sequence, position) split without a 64-bit division
  const int32_t* nvalid;  // passes after the first: the first pass's output length (device)
  // entries this pass reads: every id slot in the first pass (masked ones are dropped there),
  // the first pass's valid entries after it
  __device__ __forceinline__ int64_t count(int64_t n) const { return keys ? (int64_t)*nvalid : n; }
  // an entry the pass keeps: the first pass drops the masked slots (key V: pads, ids >= V), so
  // the later passes and the segment starts see only the tokens (stable: their order is kept)
  __device__ __forceinline__ bool keep(uint32_t key) const { return keys || key != (uint32_t)V; }
  __device__ __forceinline__ void load(int64_t i, uint32_t& key, int32_t& val) const {
    if (keys) {
      key = keys[i];
      val = vals[i];
      return;
    }
    // i < 2^31: i * (1 / L) in double is within one of the quotient; fixed up exactly (no
    // 64-bit integer division, which gfx950 emulates in ~40 instructions)
    int64_t seq = (int64_t)((double)i * inv_L);
    seq -= seq * L > i ? 1 : 0;
    seq += (seq + 1) * L <= i ? 1 : 0;
    const int64_t t = i - seq * L;
    const int64_t id = (int64_t)ids[seq * ld + t];
    const bool valid = id > 0 && id < V && id != padding_idx;
    key = valid ? (uint32_t)id : (uint32_t)V;
    val = (int32_t)seq;
  }
};

// Exclusive scan of one int per thread over a kSortThreads workgroup; *total = the sum.
__device__ __forceinline__ int32_t sort_block_excl_scan(int32_t x, int32_t* wsum, int32_t* total) {
  const int lane = lane_id(), w = threadIdx.x >> 6;
  int32_t inc = x;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const int32_t y = __shfl_up(inc, o, kWave);
    if (lane >= o) inc += y;
  }
  if (lane == kWave - 1) wsum[w] = inc;
  __syncthreads();
  int32_t before = 0, all = 0;
#pragma unroll
  for (int k = 0; k < kSortWaves; ++k) {
    const int32_t s = wsum[k];
    before += k < w ? s : 0;
    all += s;
  }
  __syncthreads();  // wsum may be reused by the caller
  if (total) *total = all;
  return before + inc - x;
}

template <typename IdT>
__global__ __launch_bounds__(kSortThreads) void plan_sort_count_kernel(SortSrc<IdT> src, int64_t n, int shift,
                                                                       int D, int64_t ntiles,
                                                                       int32_t* __restrict__ cnt) {
  __shared__ int32_t h[1 << kSortMaxD];
  const int nd = 1 << D;
  const int64_t ne = src.count(n);
  // tiles past the entries (a later pass reads fewer entries than the grid was sized for): no
  // counts -- the scan and the scatter stop at the last tile that holds entries
  const int64_t nt = (ne + kSortTile - 1) / kSortTile;
  for (int64_t tile = blockIdx.x; tile < nt; tile += gridDim.x) {  // (a capped grid walks tiles)
    for (int d = threadIdx.x; d < nd; d += kSortThreads) h[d] = 0;
    __syncthreads();
    const int64_t base = tile * kSortTile;
#pragma unroll
    for (int k = 0; k < kSortIPT; ++k) {
      const int64_t i = base + k * kSortThreads + threadIdx.x;
      if (i < ne) {
        uint32_t key;
        int32_t val;
        src.load(i, key, val);
        if (src.keep(key)) atomicAdd(&h[(key >> shift) & (nd - 1)], 1);
      }
    }
    __syncthreads();
    for (int d = threadIdx.x; d < nd; d += kSortThreads) cnt[(int64_t)d * ntiles + tile] = h[d];
    __syncthreads();
  }
}

// One WAVE per digit: cnt[d][0..ntiles) -> its exclusive scan, total[d] = the row sum.  Every
// chunk of 64 tiles is loaded before the first scan step (up to kScanChunks loads in flight per
// lane), then scanned with a carry.  Round 3 ran one 512-thread workgroup per digit (512 of them
// at D = 9): 4.8 us alone but 42 us beside the gather, whose CUs those workgroups had to share.
// Round 4: 2-wave workgroups of 2 digits, which find room beside the gather's workgroups more
// readily than 8-wave ones (C3 step 0.8566 / 0.8566 vs 0.8611 / 0.8631 ms with 8 waves, 0.8592 /
// 0.8543 with 1; profiles/r04z_plan_shapes_ab.txt).
constexpr int kScanWaves = 2;
constexpr int kScanChunks = 16;  // chunks of 64 tiles held per lane: 1,024 tiles per round
__global__ __launch_bounds__(kScanWaves * kWave) void plan_sort_scan_kernel(int32_t* __restrict__ cnt, int64_t ntiles,
                                                                            int nd, int32_t* __restrict__ total,
                                                                            const int32_t* __restrict__ nvalid) {
  const int d = blockIdx.x * kScanWaves + (threadIdx.x >> 6);
  if (d >= nd) return;
  const int lane = lane_id();
  int32_t* row = cnt + (int64_t)d * ntiles;  // (rows keep the grid's stride)
  // a later pass: only the tiles holding the first pass's output (the rest were not counted)
  if (nvalid) ntiles = ((int64_t)*nvalid + kSortTile - 1) / kSortTile;
  int32_t carry = 0;
  for (int64_t t0 = 0; t0 < ntiles; t0 += kScanChunks * kWave) {
    int32_t x[kScanChunks];
#pragma unroll
    for (int c = 0; c < kScanChunks; ++c) {
      const int64_t t = t0 + c * kWave + lane;
      x[c] = t < ntiles ? row[t] : 0;
    }
#pragma unroll
    for (int c = 0; c < kScanChunks; ++c) {
      int32_t inc = x[c];
#pragma unroll
      for (int o = 1; o < kWave; o <<= 1) {
        const int32_t y = __shfl_up(inc, o, kWave);
        if (lane >= o) inc += y;
      }
      const int64_t t = t0 + c * kWave + lane;
      if (t < ntiles) row[t] = carry + inc - x[c];
      carry += __shfl(inc, kWave - 1, kWave);
    }
  }
  if (lane == 0) total[d] = carry;
}

template <typename IdT, int D>
__global__ __launch_bounds__(kSortThreads) void plan_sort_scatter_kernel(SortSrc<IdT> src, int64_t n, int shift,
                                                                         int64_t ntiles,
                                                                         const int32_t* __restrict__ cnt,
                                                                         const int32_t* __restrict__ total,
                                                                         uint32_t* __restrict__ keys_out,
                                                                         int32_t* __restrict__ vals_out,
                                                                         int32_t* __restrict__ nvalid_out) {
  constexpr int ND = 1 << D;
  constexpr int DPT = (ND + kSortThreads - 1) / kSortThreads;  // digits per thread in the digit scans
  __shared__ int32_t hw[kSortWaves][ND];  // per-wave running counts, then per-wave tile offsets
  __shared__ int32_t gdst[ND];            // where digit d's run of this tile starts in the output
  __shared__ int32_t tst[ND];             // ... and in the tile's sorted order
  __shared__ uint32_t sk[kSortTile];      // the tile in sorted order (staged so the global
  __shared__ int32_t sv[kSortTile];       // writes of a digit's run are consecutive lanes)
  __shared__ int32_t wsum[kSortWaves];
  const int w = threadIdx.x >> 6, lane = lane_id();
  const int64_t ne = src.count(n);
  const int64_t row_stride = ntiles;  // the count matrix's digit rows keep the grid's stride
  ntiles = (ne + kSortTile - 1) / kSortTile;  // tiles past the entries: nothing to place
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {  // (a capped grid walks tiles)
    for (int d = threadIdx.x; d < kSortWaves * ND; d += kSortThreads) (&hw[0][0])[d] = 0;
    __syncthreads();

    const int64_t base = (int64_t)tile * kSortTile;
    const int64_t wbase = base + (int64_t)w * (kWave * kSortIPT);
    const uint64_t lt = (uint64_t(1) << lane) - 1;
    uint32_t key[kSortIPT];
    int32_t val[kSortIPT], rk[kSortIPT];
    bool kept[kSortIPT];
  #pragma unroll
    for (int k = 0; k < kSortIPT; ++k) {
      const int64_t i = wbase + k * kWave + lane;
      key[k] = 0;
      val[k] = 0;
      if (i < ne) src.load(i, key[k], val[k]);
      kept[k] = i < ne && src.keep(key[k]);
    }
  #pragma unroll
    for (int k = 0; k < kSortIPT; ++k) {
      const bool ok = kept[k];
      const int d = (int)((key[k] >> shift) & (ND - 1));
      uint64_t peers = __ballot(ok);
  #pragma unroll
      for (int b = 0; b < D; ++b) {
        const bool bit = (d >> b) & 1;
        const uint64_t bal = __ballot(bit);
        peers &= bit ? bal : ~bal;
      }
      const int below = __popcll(peers & lt);
      const int32_t prior = ok ? hw[w][d] : 0;
      rk[k] = prior + below;
      if (ok && below == 0) hw[w][d] = prior + __popcll(peers);  // the lowest peer lane writes
    }
    __syncthreads();
    // per digit: the waves' offsets inside the tile's run, the run's length, its global start
    // (exclusive scan of the digit totals + this tile's row offset) and its tile-sorted start
    int32_t tv[DPT], tl[DPT], part = 0, tpart = 0;
  #pragma unroll
    for (int j = 0; j < DPT; ++j) {
      const int d = threadIdx.x * DPT + j;
      tv[j] = d < ND ? total[d] : 0;
      tl[j] = 0;
      if (d < ND) {
  #pragma unroll
        for (int v = 0; v < kSortWaves; ++v) {
          const int32_t c = hw[v][d];
          hw[v][d] = tl[j];
          tl[j] += c;
        }
      }
      part += tv[j];
      tpart += tl[j];
    }
    int32_t all = 0, tile_n = 0;  // every digit's total (the pass's output length), this tile's share
    int32_t run = sort_block_excl_scan(part, wsum, &all);
    int32_t trun = sort_block_excl_scan(tpart, wsum, &tile_n);
    if (nvalid_out && tile == 0 && threadIdx.x == 0) *nvalid_out = all;
  #pragma unroll
    for (int j = 0; j < DPT; ++j) {
      const int d = threadIdx.x * DPT + j;
      if (d < ND) {
        gdst[d] = run + cnt[(int64_t)d * row_stride + tile];
        tst[d] = trun;
      }
      run += tv[j];
      trun += tl[j];
    }
    __syncthreads();
  #pragma unroll
    for (int k = 0; k < kSortIPT; ++k) {
      if (kept[k]) {
        const int d = (int)((key[k] >> shift) & (ND - 1));
        const int lp = tst[d] + hw[w][d] + rk[k];
        sk[lp] = key[k];
        sv[lp] = val[k];
      }
    }
    __syncthreads();
    // the tile in sorted order: consecutive lanes write consecutive positions of each digit's run
  #pragma unroll
    for (int k = 0; k < kSortIPT; ++k) {
      const int s = k * kSortThreads + threadIdx.x;
      if (s < tile_n) {
        const uint32_t kk = sk[s];
        const int d = (int)((kk >> shift) & (ND - 1));
        const int64_t pos = (int64_t)gdst[d] + (s - tst[d]);
        keys_out[pos] = kk;
        vals_out[pos] = sv[s];
      }
    }
    __syncthreads();  // the tile's LDS reads done before the next tile's writes
  }
}

// seg_start from the sorted keys, kStartsPT consecutive boundaries i in [0, n] per thread: every
// row r with key[i - 1] < r <= key[i] starts at i (the first sorted position with key >= r).  The
// rows are written once each; thread 0 also resets the piece counter bag_plan_pieces_kernel
// allocates from.  (Round 3: one thread per boundary, 6,144 workgroups at C3, 4.8 us alone but
// 25 us beside the gather; four per thread dispatch a quarter of the workgroups.)
constexpr int kStartsPT = 4;
__global__ __launch_bounds__(kBlock) void bag_plan_starts_kernel(const uint32_t* __restrict__ keys,
                                                                 const int32_t* __restrict__ nvalid, int64_t V,
                                                                 int32_t* __restrict__ seg_start,
                                                                 int32_t* __restrict__ n_pieces) {
  const int64_t n = *nvalid;  // the sorted tokens (masked slots were dropped by the first pass)
  const int64_t i0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * kStartsPT;
  if (i0 == 0) *n_pieces = 0;
  if (i0 > n) return;
  int64_t prev = i0 > 0 ? (int64_t)keys[i0 - 1] : -1;
#pragma unroll
  for (int j = 0; j < kStartsPT; ++j) {
    const int64_t i = i0 + j;
    if (i > n) break;
    const int64_t hi = i < n ? (int64_t)keys[i] : V;
    for (int64_t r = prev + 1; r <= hi; ++r) seg_start[r] = (int32_t)i;
    prev = hi;
  }
}

// Row r's pieces ([st, en) its sorted range): nch[r] = their number (0 = short row); a long row
// takes its slots from one counter (piece_off[V]), in token order.
__device__ __forceinline__ void plan_row_pieces(int64_t r, int32_t st, int32_t en, int64_t V, int32_t* nch,
                                                int32_t* piece_off, int32_t* piece_beg, int32_t* piece_end) {
  const int len = en - st;
  const int np = len > kPieceT ? (len + piece_len(len) - 1) / piece_len(len) : 0;
  nch[r] = np;
  if (np == 0) return;
  const int k0 = atomicAdd(piece_off + V, np), t = piece_len(len);
  piece_off[r] = k0;
  for (int k = 0; k < np; ++k) {
    piece_beg[k0 + k] = st + k * t;
    piece_end[k0 + k] = min(st + (k + 1) * t, en);
  }
}


// The pieces of every row r < V from seg_start (bag_plan_starts_kernel); nch[V] = 0.
__global__ __launch_bounds__(kBlock) void bag_plan_pieces_kernel(const int32_t* __restrict__ seg_start, int64_t V,
                                                                 int32_t* __restrict__ nch,
                                                                 int32_t* __restrict__ piece_off,
                                                                 int32_t* __restrict__ piece_beg,
                                                                 int32_t* __restrict__ piece_end) {
  const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (r > V) return;
  if (r == V) {
    nch[V] = 0;
    return;
  }
  plan_row_pieces(r, seg_start[r], seg_start[r + 1], V, nch, piece_off, piece_beg, piece_end);
}

// One wave per piece (LPR lanes x NV float4 per row, RPI pieces per wave): partial = sum of its
// tokens' gs rows in token order (U interleaved partial sums folded in a fixed order).  LD >= U
// rows are loaded per iteration (LD / U per partial sum, added in token order), so a piece of
// 128-256 tokens takes LD-fold fewer dependent load round trips; the sums are the LD = U sums.
template <int LPR, int NV, int U, int LD>
__global__ __launch_bounds__(kBlock) void bag_piece_sum_kernel(const int32_t* __restrict__ piece_off, int64_t V,
                                                               const int32_t* __restrict__ piece_beg,
                                                               const int32_t* __restrict__ piece_end,
                                                               const int32_t* __restrict__ vals,
                                                               const float* __restrict__ gs, int E,
                                                               float* __restrict__ partial) {
  static_assert(LD % U == 0, "LD must be a multiple of U");
  constexpr int RPI = kWave / LPR;
  const int lane = lane_id();
  const int sub = lane / LPR, c = lane % LPR;
  const int64_t np = piece_off[V];
  const int64_t pstride = (int64_t)gridDim.x * kWavesPerBlock * RPI;
  for (int64_t pc = ((int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * RPI + sub; pc < np; pc += pstride) {
  const int st = piece_beg[pc], en = piece_end[pc];
  f32x4 part[U][NV];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int k = 0; k < NV; ++k) part[u][k] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int e = st; e < en; e += LD) {
    int sq[LD];
#pragma unroll
    for (int u = 0; u < LD; ++u) sq[u] = (e + u < en) ? vals[e + u] : -1;
    f32x4 v[LD][NV];
#pragma unroll
    for (int u = 0; u < LD; ++u) {
      const f32x4* rp = reinterpret_cast<const f32x4*>(gs + (int64_t)(sq[u] < 0 ? 0 : sq[u]) * E);
#pragma unroll
      for (int k = 0; k < NV; ++k) v[u][k] = (sq[u] >= 0) ? rp[k * LPR + c] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < LD; ++u)  // entry e + u goes to partial (e + u - st) % U: e - st is a multiple of U
#pragma unroll
      for (int k = 0; k < NV; ++k) part[u % U][k] += v[u][k];
  }
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    f32x4 a = part[0][k];
#pragma unroll
    for (int u = 1; u < U; ++u) a += part[u][k];
    reinterpret_cast<f32x4*>(partial + pc * E)[k * LPR + c] = a;
  }
  }
}

__global__ __launch_bounds__(kBlock) void bag_piece_sum_generic_kernel(const int32_t* __restrict__ piece_off,
                                                                       int64_t V, const int32_t* __restrict__ piece_beg,
                                                                       const int32_t* __restrict__ piece_end,
                                                                       const int32_t* __restrict__ vals,
                                                                       const float* __restrict__ gs, int E,
                                                                       float* __restrict__ partial) {
  const int64_t np = piece_off[V];
  for (int64_t pc = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); pc < np;
       pc += (int64_t)gridDim.x * kWavesPerBlock) {
    const int st = piece_beg[pc], en = piece_end[pc];
    for (int c = lane_id(); c < E; c += kWave) {
      float acc = 0.f;
      for (int e = st; e < en; ++e) acc += gs[(int64_t)vals[e] * E + c];
      partial[pc * E + c] = acc;
    }
  }
}

// Row reduce: wave owns RPI rows (LPR lanes x NV float4 each); sums gs[seq] over the
// row's sorted entries (ascending seq => fixed order) and either writes the gradient row or
// applies AdamW to (table, exp_avg, exp_avg_sq) in place.
template <int LPR, int NV, int U, bool FUSED>
__global__ __launch_bounds__(kBlock) void bag_bwd_reduce_kernel(
    const int32_t* __restrict__ seg_start, const int32_t* __restrict__ seg_end,
    const int32_t* __restrict__ vals, const float* __restrict__ gs, int64_t V, int E,
    float* __restrict__ grad, float* __restrict__ param, float* __restrict__ exp_avg,
    float* __restrict__ exp_avg_sq, AdamArgs aa, const AdamArgs* __restrict__ aa_dev,
    const int32_t* __restrict__ nch, const int32_t* __restrict__ piece_off, const float* __restrict__ partial,
    int64_t row_lo) {
  constexpr int RPI = kWave / LPR;
  const int lane = lane_id();
  const int sub = lane / LPR, c = lane % LPR;
  const int64_t row = row_lo + ((int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * RPI + sub;
  if (row >= V) return;
  // a long row sums its piece partials (in piece order) instead of its tokens
  const int np = nch[row];
  const bool pieces = np > 0;
  const int st = pieces ? piece_off[row] : seg_start[row], en = pieces ? st + np : seg_end[row];
  const float* src = pieces ? partial : gs;
  // AdamW operands first: independent of the segment, so their HBM reads overlap the gather chain.
  f32x4 pv[NV], mv[NV], vv[NV];
  if constexpr (FUSED) {
    if (aa_dev) aa = *aa_dev;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int idx = k * LPR + c;
      pv[k] = reinterpret_cast<const f32x4*>(param + row * E)[idx];
      mv[k] = reinterpret_cast<const f32x4*>(exp_avg + row * E)[idx];
      vv[k] = reinterpret_cast<const f32x4*>(exp_avg_sq + row * E)[idx];
    }
  }
  // U interleaved partial sums (entry e goes to partial (e - st) % U), folded in a fixed order:
  // deterministic, ~U x shorter dependent add chains and error growth on hot (Zipf) rows.
  f32x4 part[U][NV];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int k = 0; k < NV; ++k) part[u][k] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int e = st; e < en; e += U) {
    int s[U];
#pragma unroll
    for (int u = 0; u < U; ++u) s[u] = (e + u < en) ? (pieces ? e + u : vals[e + u]) : -1;
    f32x4 v[U][NV];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const f32x4* rp = reinterpret_cast<const f32x4*>(src + (int64_t)(s[u] < 0 ? 0 : s[u]) * E);
#pragma unroll
      for (int k = 0; k < NV; ++k) v[u][k] = (s[u] >= 0) ? rp[k * LPR + c] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < NV; ++k) part[u][k] += v[u][k];
  }
  f32x4 acc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    acc[k] = part[0][k];
#pragma unroll
    for (int u = 1; u < U; ++u) acc[k] += part[u][k];
  }
  if constexpr (!FUSED) {
    f32x4* out = reinterpret_cast<f32x4*>(grad + row * E);
#pragma unroll
    for (int k = 0; k < NV; ++k) out[k * LPR + c] = acc[k];
  } else {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int idx = k * LPR + c;
      f32x4 p = pv[k], m = mv[k], v = vv[k];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float pj = p[j], mj = m[j], vj = v[j];
        adam_update(pj, acc[k][j], mj, vj, aa);
        p[j] = pj;
        m[j] = mj;
        v[j] = vj;
      }
      reinterpret_cast<f32x4*>(param + row * E)[idx] = p;
      reinterpret_cast<f32x4*>(exp_avg + row * E)[idx] = m;
      reinterpret_cast<f32x4*>(exp_avg_sq + row * E)[idx] = v;
    }
  }
}

template <bool NT>
__device__ __forceinline__ f32x4 ld4(const float* p, int64_t i) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p) + i);
  else return reinterpret_cast<const f32x4*>(p)[i];
}
template <bool NT>
__device__ __forceinline__ void st4(float* p, int64_t i, f32x4 x) {
  if constexpr (NT) __builtin_nontemporal_store(x, reinterpret_cast<f32x4*>(p) + i);
  else reinterpret_cast<f32x4*>(p)[i] = x;
}

// Column-sliced row reduce, XCD-aware: the row is cut into NS column slices of 4 * LPR floats
// and the blocks that share an XCD under round-robin placement (equal blockIdx % 8) work on one
// slice (8 / NS XCDs per slice), so an XCD gathers only its slice of the gs rows (at C3, NS = 4:
// 6.3 MB per XCD instead of 25 MB).  Placement is a speed choice only: any block -> XCD map
// computes the same (slice, rows) work.  With NT the streamed table / moment (or gradient) bytes
// carry the non-temporal hint so they do not push the gathered gs slice out of L2: at C3 the
// pair cut the update from 300 to 261 us (NS = 2: 277, NS = 8: 296 -- 128-B pieces of each row
// stream worse; without NT no gain).  RPI = 64 / LPR rows per wave, one slice each; the
// per-element sums are bag_bwd_reduce_kernel's, in the same order.
// The row's bounds (nch, piece_off, seg_start, seg_end) loaded together instead of nch first: one
// dependent memory round trip less before the gathers (round 3: apply 272 -> 267 us standalone,
// step 0.8640 -> 0.8564 ms same box, bit-identical; profiles/r03v_reduce_bounds_ab.txt).
#ifndef TT_REDUCE_SEG_EARLY
#define TT_REDUCE_SEG_EARLY 1
#endif
template <int LPR, int U, bool FUSED, bool NT>
__global__ __launch_bounds__(kBlock) void bag_bwd_reduce_sliced_kernel(
    const int32_t* __restrict__ seg_start, const int32_t* __restrict__ seg_end,
    const int32_t* __restrict__ vals, const float* __restrict__ gs, int64_t V, int E, int NS,
    float* __restrict__ grad, float* __restrict__ param, float* __restrict__ exp_avg,
    float* __restrict__ exp_avg_sq, AdamArgs aa, const AdamArgs* __restrict__ aa_dev,
    const int32_t* __restrict__ nch, const int32_t* __restrict__ piece_off, const float* __restrict__ partial,
    int64_t row_lo) {
  constexpr int RPI = kWave / LPR;
  const int lane = lane_id();
  const int sub = lane / LPR, c = lane % LPR;
  const int xg = blockIdx.x & 7, gps = 8 / NS;
  const int slice = xg % NS;
  const int64_t rb = (int64_t)(blockIdx.x >> 3) * gps + xg / NS;
  const int64_t row = row_lo + (rb * kWavesPerBlock + (threadIdx.x >> 6)) * RPI + sub;
  if (row >= V) return;
  const int col = slice * LPR + c;  // float4 index inside the row
#if TT_REDUCE_SEG_EARLY
  // the row's four bounds loaded together (piece_off holds V + 1 in-bounds entries, stale for rows
  // without pieces and then unused): one memory round trip before the gathers' index loads
  const int np = nch[row], po = piece_off[row], s0 = seg_start[row], e0 = seg_end[row];
  const bool pieces = np > 0;
  const int st = pieces ? po : s0, en = pieces ? po + np : e0;
#else
  const int np = nch[row];
  const bool pieces = np > 0;
  const int st = pieces ? piece_off[row] : seg_start[row], en = pieces ? st + np : seg_end[row];
#endif
  const float* src = pieces ? partial : gs;
  f32x4 pv, mv, vv;
  if constexpr (FUSED) {
    if (aa_dev) aa = *aa_dev;
    pv = ld4<NT>(param + row * E, col);
    mv = ld4<NT>(exp_avg + row * E, col);
    vv = ld4<NT>(exp_avg_sq + row * E, col);
  }
  f32x4 part[U];
#pragma unroll
  for (int u = 0; u < U; ++u) part[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int e = st; e < en; e += U) {
    int sq[U];
#pragma unroll
    for (int u = 0; u < U; ++u) sq[u] = (e + u < en) ? (pieces ? e + u : vals[e + u]) : -1;
    f32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      x[u] = (sq[u] >= 0) ? reinterpret_cast<const f32x4*>(src + (int64_t)sq[u] * E)[col] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < U; ++u) part[u] += x[u];
  }
  f32x4 acc = part[0];
#pragma unroll
  for (int u = 1; u < U; ++u) acc += part[u];
  if constexpr (!FUSED) {
    st4<NT>(grad + row * E, col, acc);
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float pj = pv[j], mj = mv[j], vj = vv[j];
      adam_update(pj, acc[j], mj, vj, aa);
      pv[j] = pj;
      mv[j] = mj;
      vv[j] = vj;
    }
    // (non-temporal, not write-through: sc1 stores of the p / m / v stream measured slower, C5
    // 1,194 -> 1,278 us and the C3 step 0.833 -> 0.843 ms, profiles/r06o_bag_wt_ab.txt)
    st4<NT>(param + row * E, col, pv);
    st4<NT>(exp_avg + row * E, col, mv);
    st4<NT>(exp_avg_sq + row * E, col, vv);
  }
}

// Generic-E row reduce (scalar columns).
template <bool FUSED>
__global__ __launch_bounds__(kBlock) void bag_bwd_reduce_generic_kernel(
    const int32_t* __restrict__ seg_start, const int32_t* __restrict__ seg_end,
    const int32_t* __restrict__ vals, const float* __restrict__ gs, int64_t V, int E,
    float* __restrict__ grad, float* __restrict__ param, float* __restrict__ exp_avg,
    float* __restrict__ exp_avg_sq, AdamArgs aa, const AdamArgs* __restrict__ aa_dev,
    const int32_t* __restrict__ nch, const int32_t* __restrict__ piece_off, const float* __restrict__ partial,
    int64_t row_lo) {
  const int lane = lane_id();
  const int64_t row = row_lo + (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (row >= V) return;
  if (FUSED && aa_dev) aa = *aa_dev;
  const int np = nch[row];
  const bool pieces = np > 0;
  const int st = pieces ? piece_off[row] : seg_start[row], en = pieces ? st + np : seg_end[row];
  for (int c = lane; c < E; c += kWave) {
    float acc = 0.f;
    for (int e = st; e < en; ++e) acc += pieces ? partial[(int64_t)e * E + c] : gs[(int64_t)vals[e] * E + c];
    if constexpr (!FUSED) {
      grad[row * E + c] = acc;
    } else {
      float p = param[row * E + c], m = exp_avg[row * E + c], v = exp_avg_sq[row * E + c];
      adam_update(p, acc, m, v, aa);
      param[row * E + c] = p;
      exp_avg[row * E + c] = m;
      exp_avg_sq[row * E + c] = v;
    }
  }
}

// Column-sharded table (data parallel, table_sync "column"): this rank owns columns [c0, c0 + El)
// of every row as its slab (V x El, with its moments), and their gradient sums every rank's tokens.
// Each rank sorted only its own tokens (tt_bag_plan); the plans are all-gathered -- vals (nsrc, nL)
// sorted sequence indices, seg (nsrc, V + 1) row starts -- and gs (nsrc * nseq, El) holds every
// rank's d_pooled / denom at these columns (all-to-all).  Row r's tokens in the global stable order
// (ascending global sequence src * nseq + s, the order of the reference's dense backward over the
// global batch) are source 0's segment of row r, then source 1's, ...: the per-source plans merged
// inside the reduce, no global sort.  Merged entry k goes to partial k % U, as entry (e - st) does in
// bag_bwd_reduce(_sliced)_kernel, and the partials fold in the same order, so a row's sum equals the
// single-plan reduce of the concatenated batch bit for bit (rows without pieces).  The invariant
// "the next entry goes to part[0]" is kept by rotating the partials at each source boundary.
// One wave holds RPI = 64 / LPR rows (El = 4 * LPR floats each: 128 B at El = 32), then AdamW on
// (slab, m, v) row r (FUSED) or the gradient row is written.
template <int U>
__device__ __forceinline__ void rotate_parts(f32x4 (&part)[U], int r) {
  // part[j] <- part[(j + r) % U]
  static_assert(U == 4, "rotation written for U = 4");
  if (r & 1) {
    const f32x4 t = part[0];
    part[0] = part[1]; part[1] = part[2]; part[2] = part[3]; part[3] = t;
  }
  if (r & 2) {
    f32x4 t = part[0]; part[0] = part[2]; part[2] = t;
    t = part[1]; part[1] = part[3]; part[3] = t;
  }
}

// Hot rows of the column-sharded reduce (Zipf ids, a character vocabulary).  A row whose merged
// length (every rank's tokens of it) exceeds kPieceT is cut into pieces of piece_len_col(len) merged
// entries; one sub-wave per piece sums its gs rows in merged order (entry j of the piece -> partial
// j % 4, folded 0 + 1 + 2 + 3), and the row's reduce folds the piece partials the same way.  Up to
// kMaxPieces pieces (rows of <= kPieceT * kMaxPieces merged tokens) the partition and both folds
// are the single-plan path's (bag_plan_pieces_kernel, bag_piece_sum_kernel, the sliced reduce), so
// such rows equal the one-GPU reduce of the concatenated batch bit for bit.  Longer rows (only a
// global batch of N ranks reaches them) take up to kColMaxPieces pieces and a middle level: groups
// of kMaxPieces piece partials summed by one sub-wave each, the row folding its <= 16 group sums.
// Every sum has a fixed order; only the slot numbering (atomic allocation) varies between runs.
constexpr int kColMaxPieces = 4096;
constexpr int kColLD = 16;  // partial rows loaded per sub-wave iteration of a group sum (a multiple of 4)
#ifndef TT_COL_PIECE_LD
#define TT_COL_PIECE_LD 16  // (8 / 32: C5 N = 8 at Zipf 1.05 606 / 607-615 us against 572-580, profiles/r06j_col_piece_ld_ab.txt)
#endif
constexpr int kColPieceLD = TT_COL_PIECE_LD;  // entries per iteration of a piece sum (its next indices prefetched)

__device__ __forceinline__ int piece_len_col(int len) {
  if (len <= kPieceT * kMaxPieces) return kPieceT;  // piece_len(len) there
  const int t = (len + kColMaxPieces - 1) / kColMaxPieces;
  return t > kPieceT ? t : kPieceT;
}

// One thread per row: merged length and piece count.  A long row takes its piece slots and its entry
// in the hot-row list with ONE 64-bit atomic add on {rows, pieces}: list index idx and first slot k0
// come back together, so hot_k0 increases with idx and a piece slot finds its row by a binary search
// over the list (no per-slot descriptors: a 4,096-piece row written by one thread took ~40 us).
// Rows of more than kMaxPieces pieces likewise take group slots from a second {rows, groups} counter.
__global__ __launch_bounds__(kBlock) void bag_col_pieces_kernel(const int32_t* __restrict__ seg, int nsrc, int64_t V,
                                                                int32_t* __restrict__ nch, int32_t* __restrict__ off,
                                                                int32_t* __restrict__ plen, int32_t* __restrict__ goff,
                                                                unsigned long long* __restrict__ cnt,
                                                                int32_t* __restrict__ hot_row,
                                                                int32_t* __restrict__ hot_k0,
                                                                int32_t* __restrict__ grp_row,
                                                                int32_t* __restrict__ grp_g0) {
  const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (r >= V) return;
  int len = 0;
  for (int src = 0; src < nsrc; ++src) {
    const int32_t* sg = seg + (int64_t)src * (V + 1);
    len += sg[r + 1] - sg[r];
  }
  const int t = piece_len_col(len);
  const int np = len > kPieceT ? (len + t - 1) / t : 0;
  nch[r] = np;
  if (np == 0) return;
  plen[r] = len;
  const unsigned long long o = atomicAdd(cnt, (1ull << 32) | (unsigned)np);
  const int idx = (int)(o >> 32), k0 = (int)(o & 0xffffffffu);
  off[r] = k0;
  hot_row[idx] = (int32_t)r;
  hot_k0[idx] = k0;
  if (np > kMaxPieces) {
    const int ng = (np + kMaxPieces - 1) / kMaxPieces;
    const unsigned long long og = atomicAdd(cnt + 1, (1ull << 32) | (unsigned)ng);
    const int gi = (int)(og >> 32), g0 = (int)(og & 0xffffffffu);
    goff[r] = g0;
    grp_row[gi] = (int32_t)r;
    grp_g0[gi] = g0;
  }
}

// The list entry whose slot range holds slot k: the last idx < n with first[idx] <= k (first[] ascending).
__device__ __forceinline__ int hot_entry(const int32_t* __restrict__ first, int n, int64_t k) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (first[mid] <= k) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// Sum rows [b, e) of src (El floats each) into part[] with entry j -> part[j % 4] (j from 0), LD
// loads in flight per iteration.  Zero rows pad the last iteration (x + 0 = x).
template <int LPR, int LD = kColLD>
__device__ __forceinline__ void fold_rows(const float* __restrict__ src, int b, int e, int c, f32x4 (&part)[4]) {
  static_assert(LD % 4 == 0, "entry j goes to part[j % 4]: LD a multiple of 4");
  constexpr int El = 4 * LPR;
  for (int i = b; i < e; i += LD) {
    f32x4 x[LD];
#pragma unroll
    for (int u = 0; u < LD; ++u)
      x[u] = (i + u < e) ? reinterpret_cast<const f32x4*>(src + (int64_t)(i + u) * El)[c] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < LD; ++u) part[u % 4] += x[u];
  }
}

// One sub-wave (LPR lanes, El = 4 LPR columns) per piece: its merged entries [k t, min((k+1) t, len))
// walked over the sources in rank order (source src's segment of the row is entries [acc, acc +
// cnt) of the merged order), entry j of the piece into partial j % 4.
template <int LPR>
__global__ __launch_bounds__(kBlock) void bag_col_piece_sum_kernel(const int32_t* __restrict__ seg,
                                                                   const int32_t* __restrict__ vals, int64_t nL,
                                                                   int nsrc, int64_t nseq, const float* __restrict__ gs,
                                                                   int64_t V, const int32_t* __restrict__ plen,
                                                                   const unsigned long long* __restrict__ cnt,
                                                                   const int32_t* __restrict__ hot_row,
                                                                   const int32_t* __restrict__ hot_k0,
                                                                   float* __restrict__ partial) {
  constexpr int RPI = kWave / LPR;
  constexpr int El = 4 * LPR;
  constexpr int LD = kColPieceLD;
  const int lane = lane_id();
  const int sub = lane / LPR, c = lane % LPR;
  const unsigned long long n = *cnt;
  const int64_t npc = (int64_t)(n & 0xffffffffu), pstride = (int64_t)gridDim.x * kWavesPerBlock * RPI;
  for (int64_t pc = ((int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * RPI + sub; pc < npc;
       pc += pstride) {  // (a grid of at most one round: its sub-waves walk the pieces)
  const int h = hot_entry(hot_k0, (int)(n >> 32), pc);
  const int64_t r = hot_row[h];
  const int len = plen[r], t = piece_len_col(len);
  const int b = (int)(pc - hot_k0[h]) * t, e = min(b + t, len);
  f32x4 part[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) part[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  int acc = 0, done = 0;
  for (int src = 0; src < nsrc && acc < e; ++src) {
    const int32_t* sg = seg + (int64_t)src * (V + 1);
    const int st = sg[r], n = sg[r + 1] - st;
    const int lo = max(b, acc), hi = min(e, acc + n);
    if (lo < hi) {
      const int32_t* vl = vals + (int64_t)src * nL + st - acc;  // merged entry m at vl[m]
      const float* g = gs + (int64_t)src * nseq * El;
      // the next chunk's sequence indices are loaded before this chunk's gathers: one dependent
      // memory round trip per chunk instead of two
      int nq[LD];
#pragma unroll
      for (int u = 0; u < LD; ++u) nq[u] = (lo + u < hi) ? vl[lo + u] : -1;
      for (int i = lo; i < hi; i += LD) {
        int sq[LD];
#pragma unroll
        for (int u = 0; u < LD; ++u) {
          sq[u] = nq[u];
          nq[u] = (i + LD + u < hi) ? vl[i + LD + u] : -1;
        }
        f32x4 x[LD];
#pragma unroll
        for (int u = 0; u < LD; ++u)
          x[u] = (sq[u] >= 0) ? reinterpret_cast<const f32x4*>(g + (int64_t)sq[u] * El)[c] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < LD; ++u) part[u % 4] += x[u];
      }
      done += hi - lo;
      rotate_parts(part, (hi - lo) % 4);  // the next source's first entry goes to part[0]
    }
    acc += n;
  }
  rotate_parts(part, (4 - done % 4) % 4);  // back to part[j] = entries j (mod 4)
  reinterpret_cast<f32x4*>(partial + pc * El)[c] = part[0] + part[1] + part[2] + part[3];
  }
}

// One sub-wave per group of <= kMaxPieces piece partials (rows of more than kMaxPieces pieces).
template <int LPR>
__global__ __launch_bounds__(kBlock) void bag_col_group_sum_kernel(const unsigned long long* __restrict__ cnt,
                                                                   const int32_t* __restrict__ grp_row,
                                                                   const int32_t* __restrict__ grp_g0,
                                                                   const int32_t* __restrict__ nch,
                                                                   const int32_t* __restrict__ off,
                                                                   const float* __restrict__ partial,
                                                                   float* __restrict__ gpart) {
  constexpr int RPI = kWave / LPR;
  constexpr int El = 4 * LPR;
  const int lane = lane_id();
  const int sub = lane / LPR, c = lane % LPR;
  const unsigned long long n = cnt[1];
  const int64_t ngc = (int64_t)(n & 0xffffffffu), gstride = (int64_t)gridDim.x * kWavesPerBlock * RPI;
  for (int64_t gc = ((int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * RPI + sub; gc < ngc;
       gc += gstride) {
  const int h = hot_entry(grp_g0, (int)(n >> 32), gc);
  const int64_t r = grp_row[h];
  const int k0 = off[r], np = nch[r];
  const int b = k0 + (int)(gc - grp_g0[h]) * kMaxPieces, e = min(b + kMaxPieces, k0 + np);
  f32x4 part[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) part[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  fold_rows<LPR>(partial, b, e, c, part);
  reinterpret_cast<f32x4*>(gpart + gc * El)[c] = part[0] + part[1] + part[2] + part[3];
  }
}

struct ColPieces {  // the hot-row path's outputs (nch == nullptr: no pieces, every row merged)
  const int32_t* nch;
  const int32_t* off;
  const int32_t* goff;
  const float* partial;
  const float* gpart;
};

template <int LPR, int U, bool FUSED, bool NT>
__global__ __launch_bounds__(kBlock) void bag_col_reduce_kernel(
    const int32_t* __restrict__ seg, const int32_t* __restrict__ vals, int64_t nL, int nsrc, int64_t nseq,
    const float* __restrict__ gs, int64_t V, float* __restrict__ grad, float* __restrict__ param,
    float* __restrict__ exp_avg, float* __restrict__ exp_avg_sq, const AdamArgs* __restrict__ aa_dev,
    ColPieces pcs) {
  constexpr int RPI = kWave / LPR;
  constexpr int El = 4 * LPR;
  const int lane = lane_id();
  const int sub = lane / LPR, c = lane % LPR;
  const int64_t row = ((int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * RPI + sub;
  if (row >= V) return;
  f32x4 pv, mv, vv;
  AdamArgs aa{};
  if constexpr (FUSED) {
    aa = *aa_dev;
    pv = ld4<NT>(param + row * El, c);
    mv = ld4<NT>(exp_avg + row * El, c);
    vv = ld4<NT>(exp_avg_sq + row * El, c);
  }
  f32x4 part[U];
#pragma unroll
  for (int u = 0; u < U; ++u) part[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  int64_t total = 0;
  const int np = pcs.nch ? pcs.nch[row] : 0;
  if (np > 0) {  // a hot row: its piece partials (or, past kMaxPieces pieces, its group sums)
    static_assert(U == 4, "piece folds are written for U = 4");
    // 4 partial rows in flight: the row reduce keeps its register count (and so its occupancy, which
    // the merged per-source path of every other row needs) at the round-5 kernel's; only hot rows
    // come here, and their waves overlap the rest of the launch
    if (np <= kMaxPieces) fold_rows<LPR, 4>(pcs.partial, pcs.off[row], pcs.off[row] + np, c, part);
    else fold_rows<LPR, 4>(pcs.gpart, pcs.goff[row], pcs.goff[row] + (np + kMaxPieces - 1) / kMaxPieces, c, part);
  }
  for (int src = 0; src < nsrc && np == 0; ++src) {
    const int32_t* sg = seg + (int64_t)src * (V + 1);
    const int st = sg[row], en = sg[row + 1];
    const int32_t* vl = vals + (int64_t)src * nL;
    const float* g = gs + (int64_t)src * nseq * El;
    for (int e = st; e < en; e += U) {
      int sq[U];
#pragma unroll
      for (int u = 0; u < U; ++u) sq[u] = (e + u < en) ? vl[e + u] : -1;
      f32x4 x[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        x[u] = (sq[u] >= 0) ? reinterpret_cast<const f32x4*>(g + (int64_t)sq[u] * El)[c] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < U; ++u) part[u] += x[u];
    }
    const int cnt = en - st;
    total += cnt;
    rotate_parts(part, cnt % U);  // the next source's first entry goes to part[0]
  }
  // part[j] holds the entries k == total + j (mod U): back to part[j] = entries k == j (mod U)
  rotate_parts(part, (int)((U - total % U) % U));
  f32x4 acc = part[0];
#pragma unroll
  for (int u = 1; u < U; ++u) acc += part[u];
  if constexpr (!FUSED) {
    st4<NT>(grad + row * El, c, acc);
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float pj = pv[j], mj = mv[j], vj = vv[j];
      adam_update(pj, acc[j], mj, vj, aa);
      pv[j] = pj;
      mv[j] = mj;
      vv[j] = vj;
    }
    st4<NT>(param + row * El, c, pv);
    st4<NT>(exp_avg + row * El, c, mv);
    st4<NT>(exp_avg_sq + row * El, c, vv);
  }
}

// Atomic path: one wave per sequence; lane owns columns lane, lane+64, ... so each
// global_atomic_add_f32 wave-instruction covers 256 contiguous bytes of the row.
template <typename IdT>
__global__ __launch_bounds__(kBlock) void bag_bwd_atomic_kernel(
    const float* __restrict__ dpooled, const float* __restrict__ denom, const IdT* __restrict__ ids,
    int64_t nseq, int L, int64_t ld, int64_t V, int64_t padding_idx, int E, float* __restrict__ grad) {
  const int lane = lane_id();
  const int64_t seq = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (seq >= nseq) return;
  const IdT* rid = ids + seq * ld;
  const float den = denom[seq];
  for (int c0 = 0; c0 < E; c0 += kWave) {
    const int c = c0 + lane;
    const float g = (c < E) ? dpooled[seq * E + c] / den : 0.f;
    for (int base = 0; base < L; base += kWave) {
      const int t = base + lane;
      const int64_t id = (t < L) ? (int64_t)rid[t] : 0;
      const bool valid = id > 0 && id < V && id != padding_idx;
      const int id32 = valid ? (int)id : 0;
      uint64_t m = __ballot(valid);
      while (m) {
        const int q = __builtin_ctzll(m);
        m &= m - 1;
        const int r = __builtin_amdgcn_readlane(id32, q);
        if (c < E) atomicAdd(grad + (int64_t)r * E + c, g);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// Host side
int end_bit_for(int64_t V) {
  int b = 1;
  while ((int64_t(1) << b) <= V) ++b;  // keys in [0, V] (V = masked sentinel)
  return b;
}

struct BwdWs {
  uint32_t* keys_in;
  uint32_t* keys_out;
  int32_t* vals_in;
  int32_t* vals_out;
  float* gs;
  int32_t* seg_start;  // V + 1 (bag_plan_starts_kernel)
  int32_t* seg_end;    // = seg_start + 1
  void* sort_tmp;
  size_t sort_bytes;
  int32_t* nch;        // V + 1 piece counts (0 = short row)
  int32_t* piece_off;  // V + 1: a long row's first piece slot; piece_off[V] = number of pieces
  int32_t* piece_beg;  // max_pieces token ranges
  int32_t* piece_end;
  float* partial;      // max_pieces x E
  int64_t max_pieces;
  size_t total;
};

// sum over long rows of ceil(len / piece_len) <= sum (len / kPieceT + 1) < 2 n / kPieceT
int64_t max_pieces_for(int64_t n) { return 2 * ((n + kPieceT - 1) / kPieceT) + 1; }

BwdWs carve(void* base, int64_t nseq, int L, int64_t V, int E, size_t sort_bytes) {
  BwdWs w{};
  const size_t n = (size_t)nseq * L;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off = align_up(off + bytes, 256);
    return o;
  };
  char* b = static_cast<char*>(base);
  const size_t o_ki = take(n * 4), o_ko = take(n * 4), o_vi = take(n * 4), o_vo = take(n * 4);
  const size_t o_gs = take((size_t)nseq * E * 4);
  const size_t o_ss = take((size_t)(V + 1) * 4);
  const size_t o_tmp = take(sort_bytes);
  const int64_t mp = max_pieces_for((int64_t)n);
  const size_t o_nch = take((size_t)(V + 1) * 4), o_po = take((size_t)(V + 1) * 4);
  const size_t o_pb = take((size_t)mp * 4), o_pe = take((size_t)mp * 4), o_pp = take((size_t)mp * E * 4);
  w.max_pieces = mp;
  if (b) {
    w.nch = reinterpret_cast<int32_t*>(b + o_nch);
    w.piece_off = reinterpret_cast<int32_t*>(b + o_po);
    w.piece_beg = reinterpret_cast<int32_t*>(b + o_pb);
    w.piece_end = reinterpret_cast<int32_t*>(b + o_pe);
    w.partial = reinterpret_cast<float*>(b + o_pp);
    w.keys_in = reinterpret_cast<uint32_t*>(b + o_ki);
    w.keys_out = reinterpret_cast<uint32_t*>(b + o_ko);
    w.vals_in = reinterpret_cast<int32_t*>(b + o_vi);
    w.vals_out = reinterpret_cast<int32_t*>(b + o_vo);
    w.gs = reinterpret_cast<float*>(b + o_gs);
    w.seg_start = reinterpret_cast<int32_t*>(b + o_ss);
    w.seg_end = w.seg_start + 1;
    w.sort_tmp = b + o_tmp;
  }
  w.sort_bytes = sort_bytes;
  w.total = off;
  return w;
}


// The sort's shape: P passes of D bits over ntiles tiles; its workspace holds the digit-major
// tile counts and the digit totals.  The widest digit is kSortDefaultD: wider digits mean fewer
// passes but a digits x tiles count matrix that grows as 2^D (its transposed 4-byte accesses, not
// the entries' bytes, bound a pass; sweep in profiles/r03o_plan_digit_sweep.txt).
struct SortShape {
  int P, D;
  int64_t ntiles;
};
SortShape sort_shape(int64_t n, int64_t V) {
  const int bits = end_bit_for(V), maxd = kSortDefaultD;
  const int P = (bits + maxd - 1) / maxd;
  return SortShape{P, (bits + P - 1) / P, (n + kSortTile - 1) / kSortTile};
}
size_t sort_tmp_bytes(int64_t n, int64_t V) {
  const SortShape sh = sort_shape(n, V);
  // digit-major tile counts, the digit totals, then the first pass's output length
  return align_up((((size_t)sh.ntiles + 1) * ((size_t)1 << sh.D) + 1) * 4, 256);
}

// planes != nullptr: the split workgroups of tt_bag_mean_fwd_split first (E in the templated set)
template <typename IdT>
int launch_fwd(const float* table, int64_t V, int E, const IdT* ids, int64_t nseq, int L, int64_t ld,
               float* pooled, float* denom, hipStream_t s, const SplitJobs& sj = SplitJobs{},
               __bf16* planes = nullptr) {
  int nsplit = 0;
  if (planes) {
    int64_t big = 0;
    for (int j = 0; j < 4; ++j) big = std::max<int64_t>(big, (int64_t)sj.n[j] * sj.k[j]);
    nsplit = (int)((big + kBlock - 1) / kBlock);
  }
  const int64_t gblocks = (nseq + kWavesPerBlock - 1) / kWavesPerBlock;
  const dim3 grid((unsigned)(nsplit + gblocks)), block(kBlock);
#define TT_FWD(LPR, NV, U) \
  bag_fwd_kernel<IdT, LPR, NV, U><<<grid, block, 0, s>>>(table, V, E, ids, nseq, L, ld, pooled, denom, sj, planes, nsplit)
  switch (E) {
    case 32: TT_FWD(8, 1, 4); break;  // a column slab of E = 256 over 8 ranks (table_sync "column")
    case 64: TT_FWD(16, 1, 4); break;
    case 128: TT_FWD(32, 1, 4); break;
    case 256: TT_FWD(64, 1, 8); break;
    case 512: TT_FWD(64, 2, 4); break;
    case 1024: TT_FWD(64, 4, 2); break;
    default:
      TT_REQUIRE(!planes, "tt_bag_mean_fwd_split: E %d", E);
      bag_fwd_generic_kernel<IdT><<<grid, block, 0, s>>>(table, V, E, ids, nseq, L, ld, pooled, denom);
      break;
  }
#undef TT_FWD
  TT_LAUNCH_CHECK("tt_bag_mean_fwd");
  return TT_OK;
}

// E in {256, 512, 1024}: the XCD-sliced reduce with non-temporal table/moment traffic (C3:
// 261 us against 300 us for the whole-row kernel, tools/mb_bag_bwd.py; same sums in the same
// order); the whole-row kernels for other widths.
bool use_sliced_reduce(int E) { return E == 256 || E == 512 || E == 1024; }

// Rows [row_lo, V) of the table (row_lo > 0: a row range of the dense gradient; `grad` then
// points at row 0's position, so row r lands at grad + r * E).
template <bool FUSED>
int launch_reduce(const BwdWs& w, int64_t V, int E, float* grad, float* param, float* m, float* v,
                  const AdamArgs& aa, const AdamArgs* aa_dev, hipStream_t s, int64_t row_lo = 0) {
  const int64_t nrows = V - row_lo;
  if (nrows <= 0) return TT_OK;
  auto grid_for = [&](int rpi) {
    const int64_t waves = (nrows + rpi - 1) / rpi;
    return dim3((unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock));
  };
  const dim3 block(kBlock);
  if (use_sliced_reduce(E)) {
    // NS = 4 column slices of LPR = E / 16 float4 (256 B at E = 256); the row blocks of a slice
    // are dealt to 8 / NS = 2 block groups, the grid padded to whole groups of 8 blocks
    constexpr int NS = 4;
    const int LPR = E / (4 * NS);
    const int64_t rpb = kWavesPerBlock * (kWave / LPR), rbs = (nrows + rpb - 1) / rpb, gps = 8 / NS;
    const dim3 grid((unsigned)(((rbs + gps - 1) / gps) * 8));
#define TT_SL(L) bag_bwd_reduce_sliced_kernel<L, 4, FUSED, true><<<grid, block, 0, s>>>(w.seg_start, w.seg_end, w.vals_out, w.gs, V, E, NS, grad, param, m, v, aa, aa_dev, w.nch, w.piece_off, w.partial, row_lo)
    if (LPR == 16) TT_SL(16);
    else if (LPR == 32) TT_SL(32);
    else TT_SL(64);
#undef TT_SL
    TT_LAUNCH_CHECK("bag_bwd_reduce_sliced");
    return TT_OK;
  }
  switch (E) {
    case 64: bag_bwd_reduce_kernel<16, 1, 4, FUSED><<<grid_for(4), block, 0, s>>>(w.seg_start, w.seg_end, w.vals_out, w.gs, V, E, grad, param, m, v, aa, aa_dev, w.nch, w.piece_off, w.partial, row_lo); break;
    case 128: bag_bwd_reduce_kernel<32, 1, 4, FUSED><<<grid_for(2), block, 0, s>>>(w.seg_start, w.seg_end, w.vals_out, w.gs, V, E, grad, param, m, v, aa, aa_dev, w.nch, w.piece_off, w.partial, row_lo); break;
    case 256: bag_bwd_reduce_kernel<64, 1, 4, FUSED><<<grid_for(1), block, 0, s>>>(w.seg_start, w.seg_end, w.vals_out, w.gs, V, E, grad, param, m, v, aa, aa_dev, w.nch, w.piece_off, w.partial, row_lo); break;
    case 512: bag_bwd_reduce_kernel<64, 2, 4, FUSED><<<grid_for(1), block, 0, s>>>(w.seg_start, w.seg_end, w.vals_out, w.gs, V, E, grad, param, m, v, aa, aa_dev, w.nch, w.piece_off, w.partial, row_lo); break;
    case 1024: bag_bwd_reduce_kernel<64, 4, 2, FUSED><<<grid_for(1), block, 0, s>>>(w.seg_start, w.seg_end, w.vals_out, w.gs, V, E, grad, param, m, v, aa, aa_dev, w.nch, w.piece_off, w.partial, row_lo); break;
    default: bag_bwd_reduce_generic_kernel<FUSED><<<grid_for(1), block, 0, s>>>(w.seg_start, w.seg_end, w.vals_out, w.gs, V, E, grad, param, m, v, aa, aa_dev, w.nch, w.piece_off, w.partial, row_lo); break;
  }
  TT_LAUNCH_CHECK("bag_bwd_reduce");
  return TT_OK;
}

constexpr int64_t kPieceSumMaxBlocks = 2048;  // 8 per CU: one round

int launch_piece_sum(const BwdWs& w, int64_t V, int E, hipStream_t s) {
  // the pieces are counted on the device (piece_off[V]); the grid covers the most a batch can have
  // up to one round of waves on the chip (kPieceSumMaxBlocks), whose waves walk any further pieces:
  // a batch without long rows (C3's uniform ids) then costs one short launch, not 6,000 workgroups
  auto grid_for = [&](int rpi) {
    const int64_t waves = (w.max_pieces + rpi - 1) / rpi;
    return dim3((unsigned)std::min<int64_t>((waves + kWavesPerBlock - 1) / kWavesPerBlock, kPieceSumMaxBlocks));
  };
  const dim3 block(kBlock);
  switch (E) {
    case 64: bag_piece_sum_kernel<16, 1, 4, 16><<<grid_for(4), block, 0, s>>>(w.piece_off, V, w.piece_beg, w.piece_end, w.vals_out, w.gs, E, w.partial); break;
    case 128: bag_piece_sum_kernel<32, 1, 4, 16><<<grid_for(2), block, 0, s>>>(w.piece_off, V, w.piece_beg, w.piece_end, w.vals_out, w.gs, E, w.partial); break;
    case 256: bag_piece_sum_kernel<64, 1, 4, 16><<<grid_for(1), block, 0, s>>>(w.piece_off, V, w.piece_beg, w.piece_end, w.vals_out, w.gs, E, w.partial); break;
    case 512: bag_piece_sum_kernel<64, 2, 4, 8><<<grid_for(1), block, 0, s>>>(w.piece_off, V, w.piece_beg, w.piece_end, w.vals_out, w.gs, E, w.partial); break;
    case 1024: bag_piece_sum_kernel<64, 4, 2, 8><<<grid_for(1), block, 0, s>>>(w.piece_off, V, w.piece_beg, w.piece_end, w.vals_out, w.gs, E, w.partial); break;
    default: bag_piece_sum_generic_kernel<<<grid_for(1), block, 0, s>>>(w.piece_off, V, w.piece_beg, w.piece_end, w.vals_out, w.gs, E, w.partial); break;
  }
  TT_LAUNCH_CHECK("bag_piece_sum");
  return TT_OK;
}

// plan: keys/vals -> stable counting sort (key = row id, value = seq) -> segment starts and the
// pieces of long rows (bag_plan_starts_kernel, bag_plan_pieces_kernel).
template <typename IdT>
int plan_front(const IdT* ids, int64_t nseq, int L, int64_t ld, int64_t V, int64_t padding_idx, const BwdWs& w,
               hipStream_t s, int part = -1) {
  // part -1: the whole plan; 0: every sort pass but the last; 1: the last pass, the segment starts
  // and the pieces (tt_bag_plan_part: the two halves on one stream compute what one call does)
  const int64_t n = nseq * L;
  const dim3 block(kBlock);
  if (part == 0 && n == 0) return TT_OK;
  if (n == 0) {  // no tokens: every segment empty, no pieces
    TT_HIP(hipMemsetAsync(w.seg_start, 0, (size_t)(V + 1) * 4, s), "memset seg_start");
    TT_HIP(hipMemsetAsync(w.nch, 0, (size_t)(V + 1) * 4, s), "memset nch");
    TT_HIP(hipMemsetAsync(w.piece_off, 0, (size_t)(V + 1) * 4, s), "memset piece_off");
    return TT_OK;
  }
  // hand-written LSD counting sort: pass p writes (keys_out, vals_out) when P - 1 - p is even,
  // (keys_in, vals_in) otherwise, so the last pass lands in the _out arrays
  const SortShape sh = sort_shape(n, V);
  const int nd = 1 << sh.D;
  // one workgroup per tile (capped grids whose workgroups walk several tiles measured slower in
  // the step: profiles/r05n_plan_grid_ab.txt)
  const unsigned sgrid = (unsigned)sh.ntiles;
  int32_t* cnt = static_cast<int32_t*>(w.sort_tmp);
  int32_t* total = cnt + (size_t)nd * sh.ntiles;
  int32_t* nvalid = total + nd;  // written by the first pass's scatter
  SortSrc<IdT> src{ids, L, ld, V, padding_idx, nullptr, nullptr, L > 0 ? 1.0 / (double)L : 0.0, nvalid};
  const int p_begin = part == 1 ? sh.P - 1 : 0, p_end = part == 0 ? sh.P - 1 : sh.P;
  if (p_begin > 0) {  // the previous pass's output (pass p writes _out when P - 1 - p is even)
    const bool prev_out = ((sh.P - 1 - (p_begin - 1)) & 1) == 0;
    src.keys = prev_out ? w.keys_out : w.keys_in;
    src.vals = prev_out ? w.vals_out : w.vals_in;
  }
  for (int p = p_begin; p < p_end; ++p) {
    const bool to_out = ((sh.P - 1 - p) & 1) == 0;
    uint32_t* ko = to_out ? w.keys_out : w.keys_in;
    int32_t* vo = to_out ? w.vals_out : w.vals_in;
    const int shift = p * sh.D;
    plan_sort_count_kernel<IdT><<<dim3(sgrid), dim3(kSortThreads), 0, s>>>(src, n, shift, sh.D,
                                                                                       sh.ntiles, cnt);
    TT_LAUNCH_CHECK("plan_sort_count");
    plan_sort_scan_kernel<<<dim3((unsigned)((nd + kScanWaves - 1) / kScanWaves)), dim3(kScanWaves * kWave), 0, s>>>(
        cnt, sh.ntiles, nd, total, p == 0 ? nullptr : nvalid);
    TT_LAUNCH_CHECK("plan_sort_scan");
    switch (sh.D) {
#define TT_SC(DD)                                                                                         \
  case DD:                                                                                                \
    plan_sort_scatter_kernel<IdT, DD><<<dim3(sgrid), dim3(kSortThreads), 0, s>>>(src, n, shift,            \
                                                                                             sh.ntiles, cnt, \
                                                                                             total, ko, vo,   \
                                                                                             p == 0 ? nvalid : nullptr); \
    break;
      TT_SC(1) TT_SC(2) TT_SC(3) TT_SC(4) TT_SC(5) TT_SC(6) TT_SC(7) TT_SC(8) TT_SC(9) TT_SC(10) TT_SC(11)
#undef TT_SC
      default: TT_REQUIRE(false, "plan sort: digit width %d", sh.D);
    }
    TT_LAUNCH_CHECK("plan_sort_scatter");
    src.keys = ko;
    src.vals = vo;
  }
  if (part == 0) return TT_OK;
  const int64_t nst = (n + 1 + kStartsPT - 1) / kStartsPT;
  bag_plan_starts_kernel<<<dim3((unsigned)((nst + kBlock - 1) / kBlock)), block, 0, s>>>(w.keys_out, nvalid, V,
                                                                                       w.seg_start, w.piece_off + V);
  TT_LAUNCH_CHECK("bag_plan_starts");
  bag_plan_pieces_kernel<<<dim3((unsigned)((V + 1 + kBlock - 1) / kBlock)), block, 0, s>>>(
      w.seg_start, V, w.nch, w.piece_off, w.piece_beg, w.piece_end);
  TT_LAUNCH_CHECK("bag_plan_pieces");
  return TT_OK;
}

// apply, first half: gs = dpooled / denom (denom NULL: the caller passed gs itself) and the long
// rows' piece sums.  Returns the workspace view whose gs the reduce reads.
int apply_prepare(const float* dpooled, const float* denom, int64_t nseq, int64_t V, int E, const BwdWs& w,
                  BwdWs& wa, hipStream_t s, bool launch = true) {
  wa = w;
  if (nseq > 0) {
    if (denom) {
      if (launch) {
        bag_scale_rows_kernel<<<dim3((unsigned)((nseq + kWavesPerBlock - 1) / kWavesPerBlock)), dim3(kBlock), 0, s>>>(
            dpooled, denom, nseq, E, w.gs);
        TT_LAUNCH_CHECK("bag_scale_rows");
      }
    } else {
      wa.gs = const_cast<float*>(dpooled);
    }
    if (launch) return launch_piece_sum(wa, V, E, s);
  }
  return TT_OK;
}

// apply: gs = dpooled / denom, then the row reduce (dense gradient or fused AdamW).
template <bool FUSED>
int apply_plan(const float* dpooled, const float* denom, int64_t nseq, int64_t V, int E, const BwdWs& w,
               float* grad, float* param, float* m, float* v, const AdamArgs& aa, const AdamArgs* aa_dev,
               hipStream_t s) {
  BwdWs wa;
  int rc = apply_prepare(dpooled, denom, nseq, V, E, w, wa, s);
  if (rc) return rc;
  return launch_reduce<FUSED>(wa, V, E, grad, param, m, v, aa, aa_dev, s);
}

int check_common(int64_t V, int E, const void* ids, int ids_dtype, int64_t nseq, int L, int64_t ld) {
  TT_REQUIRE(V > 0 && V < (int64_t(1) << 31) - 1, "V=%lld out of range", (long long)V);
  TT_REQUIRE(E > 0, "E=%d must be positive", E);
  TT_REQUIRE(nseq >= 0 && L >= 0 && ld >= L, "bad ids shape nseq=%lld L=%d ld=%lld", (long long)nseq, L, (long long)ld);
  TT_REQUIRE(nseq * (int64_t)L < (int64_t(1) << 31), "too many tokens (%lld)", (long long)(nseq * L));
  TT_REQUIRE(ids_dtype == TT_IDS_I32 || ids_dtype == TT_IDS_I64, "ids_dtype=%d", ids_dtype);
  TT_REQUIRE(ids != nullptr || nseq * L == 0, "ids is NULL");
  return TT_OK;
}

}  // namespace
}  // namespace tt

using namespace tt;

extern "C" int tt_bag_mean_fwd(const float* table, int64_t V, int E, const void* ids, int ids_dtype,
                               int64_t nseq, int L, int64_t ld_ids, float* pooled, float* denom,
                               tt_stream_t stream) {
  int rc = check_common(V, E, ids, ids_dtype, nseq, L, ld_ids);
  if (rc) return rc;
  TT_REQUIRE(table && pooled && denom, "null pointer");
  if (nseq == 0) return TT_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (ids_dtype == TT_IDS_I32)
    return launch_fwd(table, V, E, static_cast<const int32_t*>(ids), nseq, L, ld_ids, pooled, denom, s);
  return launch_fwd(table, V, E, static_cast<const int64_t*>(ids), nseq, L, ld_ids, pooled, denom, s);
}

extern "C" int tt_bag_mean_fwd_cols(const float* slab, int64_t V, int El, int E, const void* ids, int ids_dtype,
                                    int64_t nseq, int L, int64_t ld_ids, float* pooled, float* denom,
                                    tt_stream_t stream) {
  int rc = check_common(V, El, ids, ids_dtype, nseq, L, ld_ids);
  if (rc) return rc;
  TT_REQUIRE(slab && pooled && denom, "null pointer");
  TT_REQUIRE((El == 32 || El == 64 || El == 128 || El == 256) && E >= El && E % El == 0,
             "tt_bag_mean_fwd_cols: El in {32, 64, 128, 256} dividing E (got El=%d E=%d)", El, E);
  if (nseq == 0) return TT_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (ids_dtype == TT_IDS_I32)
    return launch_fwd_cols(slab, V, El, E, static_cast<const int32_t*>(ids), nseq, L, ld_ids, pooled, denom, s);
  return launch_fwd_cols(slab, V, El, E, static_cast<const int64_t*>(ids), nseq, L, ld_ids, pooled, denom, s);
}

extern "C" int tt_bag_mean_fwd_split(const float* table, int64_t V, int E, const void* ids, int ids_dtype,
                                     int64_t nseq, int L, int64_t ld_ids, float* pooled, float* denom,
                                     const float* W1, const float* W2, int H, void* planes, tt_stream_t stream) {
  int rc = check_common(V, E, ids, ids_dtype, nseq, L, ld_ids);
  if (rc) return rc;
  TT_REQUIRE(table && pooled && denom && W1 && W2 && planes, "null pointer");
  TT_REQUIRE((E == 64 || E == 128 || E == 256) && (H == 128 || H == 256),
             "tt_bag_mean_fwd_split: E in {64, 128, 256}, H in {128, 256} (got E=%d H=%d)", E, H);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const SplitJobs sj = head_ff2_jobs(W1, W2, E, H);
  __bf16* pl = static_cast<__bf16*>(planes);
  if (ids_dtype == TT_IDS_I32)
    return launch_fwd(table, V, E, static_cast<const int32_t*>(ids), nseq, L, ld_ids, pooled, denom, s, sj, pl);
  return launch_fwd(table, V, E, static_cast<const int64_t*>(ids), nseq, L, ld_ids, pooled, denom, s, sj, pl);
}

extern "C" size_t tt_bag_mean_bwd_ws_size(int64_t nseq, int L, int64_t V, int E) {
  const size_t sb = sort_tmp_bytes(nseq * (int64_t)L, V);
  return carve(nullptr, nseq, L, V, E, sb).total + 256;
}

static BwdWs plan_layout(void* ws, int64_t nseq, int L, int64_t V, int E) {
  if (nseq == 0 || L == 0) nseq = 0, L = 0;
  const size_t sb = nseq > 0 ? sort_tmp_bytes(nseq * (int64_t)L, V) : 0;
  void* base = ws ? reinterpret_cast<void*>(align_up(reinterpret_cast<size_t>(ws), 256)) : nullptr;
  return carve(base, nseq, L, V, E, sb);
}

static int plan_impl(const void* ids, int ids_dtype, int64_t nseq, int L, int64_t ld, int64_t V, int E,
                     int64_t padding_idx, void* ws, size_t ws_bytes, hipStream_t s, int part = -1) {
  const BwdWs w = plan_layout(ws, nseq, L, V, E);
  TT_REQUIRE(ws != nullptr && w.total + 256 <= ws_bytes, "workspace too small: need %zu have %zu",
             w.total + 256, ws_bytes);
  if (nseq == 0 || L == 0) return plan_front<int32_t>(nullptr, 0, 0, 0, V, padding_idx, w, s, part);
  return ids_dtype == TT_IDS_I32
             ? plan_front(static_cast<const int32_t*>(ids), nseq, L, ld, V, padding_idx, w, s, part)
             : plan_front(static_cast<const int64_t*>(ids), nseq, L, ld, V, padding_idx, w, s, part);
}

template <bool FUSED>
static int apply_impl(const float* dpooled, const float* denom, int64_t nseq, int L, int64_t V, int E, void* ws,
                      size_t ws_bytes, float* grad, float* param, float* m, float* v, const AdamArgs& aa,
                      const AdamArgs* aa_dev, hipStream_t s) {
  const BwdWs w = plan_layout(ws, nseq, L, V, E);
  TT_REQUIRE(ws != nullptr && w.total + 256 <= ws_bytes, "workspace too small: need %zu have %zu",
             w.total + 256, ws_bytes);
  return apply_plan<FUSED>(dpooled, denom, (nseq == 0 || L == 0) ? 0 : nseq, V, E, w, grad, param, m, v, aa, aa_dev,
                           s);
}

extern "C" size_t tt_bag_plan_ws_size(int64_t nseq, int L, int64_t V, int E) {
  return tt_bag_mean_bwd_ws_size(nseq, L, V, E);
}

extern "C" int tt_bag_plan(const void* ids, int ids_dtype, int64_t nseq, int L, int64_t ld_ids, int64_t V, int E,
                           int64_t padding_idx, void* plan, size_t plan_bytes, tt_stream_t stream) {
  int rc = check_common(V, E, ids, ids_dtype, nseq, L, ld_ids);
  if (rc) return rc;
  return plan_impl(ids, ids_dtype, nseq, L, ld_ids, V, E, padding_idx, plan, plan_bytes,
                   reinterpret_cast<hipStream_t>(stream));
}

extern "C" int tt_bag_plan_part(const void* ids, int ids_dtype, int64_t nseq, int L, int64_t ld_ids, int64_t V,
                                int E, int64_t padding_idx, void* plan, size_t plan_bytes, int part,
                                tt_stream_t stream) {
  int rc = check_common(V, E, ids, ids_dtype, nseq, L, ld_ids);
  if (rc) return rc;
  TT_REQUIRE(part == 0 || part == 1, "tt_bag_plan_part: part 0 or 1 (got %d)", part);
  return plan_impl(ids, ids_dtype, nseq, L, ld_ids, V, E, padding_idx, plan, plan_bytes,
                   reinterpret_cast<hipStream_t>(stream), part);
}

extern "C" int tt_bag_plan_layout(int64_t nseq, int L, int64_t V, int E, int64_t* offs) {
  TT_REQUIRE(offs != nullptr && V > 0 && E > 0 && nseq >= 0 && L >= 0, "tt_bag_plan_layout: bad arguments");
  const BwdWs z = plan_layout(reinterpret_cast<void*>(256), nseq, L, V, E);  // offsets from a 256-B base
  offs[0] = reinterpret_cast<char*>(z.keys_out) - reinterpret_cast<char*>(256);
  offs[1] = reinterpret_cast<char*>(z.vals_out) - reinterpret_cast<char*>(256);
  offs[2] = reinterpret_cast<char*>(z.seg_start) - reinterpret_cast<char*>(256);
  return TT_OK;
}

extern "C" int tt_bag_mean_bwd_planned(const float* d_pooled, const float* denom, int64_t nseq, int L, int64_t V,
                                       int E, const void* plan, size_t plan_bytes, float* grad_table,
                                       tt_stream_t stream) {
  TT_REQUIRE(V > 0 && E > 0 && nseq >= 0 && L >= 0, "bad shape");
  TT_REQUIRE(grad_table && (nseq == 0 || d_pooled), "null pointer");  // denom NULL: d_pooled is gs
  AdamArgs aa{};
  return apply_impl<false>(d_pooled, denom, nseq, L, V, E, const_cast<void*>(plan), plan_bytes, grad_table, nullptr,
                           nullptr, nullptr, aa, nullptr, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int tt_bag_mean_bwd_planned_prepare(const float* d_pooled, const float* denom, int64_t nseq, int L,
                                               int64_t V, int E, void* plan, size_t plan_bytes, tt_stream_t stream) {
  TT_REQUIRE(V > 0 && E > 0 && nseq >= 0 && L >= 0, "bad shape");
  TT_REQUIRE(nseq == 0 || d_pooled, "null pointer");
  const BwdWs w = plan_layout(plan, nseq, L, V, E);
  TT_REQUIRE(plan != nullptr && w.total + 256 <= plan_bytes, "plan workspace too small: need %zu have %zu",
             w.total + 256, plan_bytes);
  BwdWs wa;
  return apply_prepare(d_pooled, denom, (nseq == 0 || L == 0) ? 0 : nseq, V, E, w, wa,
                       reinterpret_cast<hipStream_t>(stream));
}

extern "C" int tt_bag_mean_bwd_planned_rows(const float* d_pooled, const float* denom, int64_t nseq, int L,
                                            int64_t V, int E, const void* plan, size_t plan_bytes, int64_t row_begin,
                                            int64_t row_end, float* grad_rows, tt_stream_t stream) {
  TT_REQUIRE(V > 0 && E > 0 && nseq >= 0 && L >= 0, "bad shape");
  TT_REQUIRE(0 <= row_begin && row_begin <= row_end && row_end <= V, "rows [%lld, %lld) outside [0, %lld)",
             (long long)row_begin, (long long)row_end, (long long)V);
  TT_REQUIRE(grad_rows && (nseq == 0 || d_pooled), "null pointer");
  const BwdWs w = plan_layout(const_cast<void*>(plan), nseq, L, V, E);
  TT_REQUIRE(plan != nullptr && w.total + 256 <= plan_bytes, "plan workspace too small: need %zu have %zu",
             w.total + 256, plan_bytes);
  BwdWs wa;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int rc = apply_prepare(d_pooled, denom, (nseq == 0 || L == 0) ? 0 : nseq, V, E, w, wa, s, false);
  if (rc) return rc;
  AdamArgs aa{};
  // row r of the range lands at grad_rows + (r - row_begin) * E
  return launch_reduce<false>(wa, row_end, E, grad_rows - row_begin * (int64_t)E, nullptr, nullptr, nullptr, aa,
                              nullptr, s, row_begin);
}

extern "C" int tt_bag_mean_bwd_adamw_planned(const float* d_pooled, const float* denom, int64_t nseq, int L,
                                             int64_t V, int E, const void* plan, size_t plan_bytes, float* table,
                                             float* exp_avg, float* exp_avg_sq, const void* adam_args,
                                             tt_stream_t stream) {
  TT_REQUIRE(V > 0 && E > 0 && nseq >= 0 && L >= 0, "bad shape");
  TT_REQUIRE(table && exp_avg && exp_avg_sq && adam_args, "null pointer");
  TT_REQUIRE(nseq == 0 || d_pooled, "null pointer");  // denom NULL: d_pooled is gs already
  AdamArgs aa{};
  return apply_impl<true>(d_pooled, denom, nseq, L, V, E, const_cast<void*>(plan), plan_bytes, nullptr, table,
                          exp_avg, exp_avg_sq, aa, static_cast<const AdamArgs*>(adam_args),
                          reinterpret_cast<hipStream_t>(stream));
}

extern "C" int tt_bag_mean_bwd_adamw_planned_rows(const float* d_pooled, const float* denom, int64_t nseq, int L,
                                                  int64_t V, int E, const void* plan, size_t plan_bytes,
                                                  int64_t row_begin, int64_t row_end, float* table_rows,
                                                  float* exp_avg_rows, float* exp_avg_sq_rows, const void* adam_args,
                                                  tt_stream_t stream) {
  TT_REQUIRE(V > 0 && E > 0 && nseq >= 0 && L >= 0, "bad shape");
  TT_REQUIRE(0 <= row_begin && row_begin <= row_end && row_end <= V, "rows [%lld, %lld) outside [0, %lld)",
             (long long)row_begin, (long long)row_end, (long long)V);
  TT_REQUIRE(table_rows && exp_avg_rows && exp_avg_sq_rows && adam_args && (nseq == 0 || d_pooled), "null pointer");
  const BwdWs w = plan_layout(const_cast<void*>(plan), nseq, L, V, E);
  TT_REQUIRE(plan != nullptr && w.total + 256 <= plan_bytes, "plan workspace too small: need %zu have %zu",
             w.total + 256, plan_bytes);
  BwdWs wa;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int rc = apply_prepare(d_pooled, denom, (nseq == 0 || L == 0) ? 0 : nseq, V, E, w, wa, s, false);
  if (rc) return rc;
  AdamArgs aa{};
  // row r of the range updates table_rows / the moment rows at (r - row_begin) * E
  const int64_t sh = row_begin * (int64_t)E;
  return launch_reduce<true>(wa, row_end, E, nullptr, table_rows - sh, exp_avg_rows - sh, exp_avg_sq_rows - sh, aa,
                             static_cast<const AdamArgs*>(adam_args), s, row_begin);
}

extern "C" int tt_bag_mean_bwd(const float* d_pooled, const float* denom, const void* ids, int ids_dtype,
                               int64_t nseq, int L, int64_t ld_ids, int64_t V, int E, int64_t padding_idx,
                               float* grad_table, int mode, void* ws, size_t ws_bytes, tt_stream_t stream) {
  int rc = check_common(V, E, ids, ids_dtype, nseq, L, ld_ids);
  if (rc) return rc;
  TT_REQUIRE(grad_table && (nseq == 0 || (d_pooled && denom)), "null pointer");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (mode == TT_SCATTER_ATOMIC) {
    if (nseq == 0) return TT_OK;
    const dim3 grid((unsigned)((nseq + kWavesPerBlock - 1) / kWavesPerBlock)), block(kBlock);
    if (ids_dtype == TT_IDS_I32)
      bag_bwd_atomic_kernel<int32_t><<<grid, block, 0, s>>>(d_pooled, denom, static_cast<const int32_t*>(ids), nseq, L, ld_ids, V, padding_idx, E, grad_table);
    else
      bag_bwd_atomic_kernel<int64_t><<<grid, block, 0, s>>>(d_pooled, denom, static_cast<const int64_t*>(ids), nseq, L, ld_ids, V, padding_idx, E, grad_table);
    TT_LAUNCH_CHECK("tt_bag_mean_bwd(atomic)");
    return TT_OK;
  }
  TT_REQUIRE(mode == TT_SCATTER_SORTED, "unknown scatter mode %d", mode);
  AdamArgs aa{};
  rc = plan_impl(ids, ids_dtype, nseq, L, ld_ids, V, E, padding_idx, ws, ws_bytes, s);
  if (rc) return rc;
  return apply_impl<false>(d_pooled, denom, nseq, L, V, E, ws, ws_bytes, grad_table, nullptr, nullptr, nullptr, aa,
                           nullptr, s);
}

extern "C" int tt_bag_mean_bwd_adamw(const float* d_pooled, const float* denom, const void* ids, int ids_dtype,
                                     int64_t nseq, int L, int64_t ld_ids, int64_t V, int E, int64_t padding_idx,
                                     float* table, float* exp_avg, float* exp_avg_sq, double lr, double beta1,
                                     double beta2, double eps, double weight_decay, int64_t step, void* ws,
                                     size_t ws_bytes, tt_stream_t stream) {
  int rc = check_common(V, E, ids, ids_dtype, nseq, L, ld_ids);
  if (rc) return rc;
  TT_REQUIRE(table && exp_avg && exp_avg_sq, "null pointer");
  TT_REQUIRE(step >= 1, "step must be >= 1 (got %lld)", (long long)step);
  TT_REQUIRE(nseq * (int64_t)L == 0 || (d_pooled && denom), "null pointer");
  const AdamArgs aa = make_adam(lr, beta1, beta2, eps, weight_decay, step);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  rc = plan_impl(ids, ids_dtype, nseq, L, ld_ids, V, E, padding_idx, ws, ws_bytes, s);
  if (rc) return rc;
  return apply_impl<true>(d_pooled, denom, nseq, L, V, E, ws, ws_bytes, nullptr, table, exp_avg, exp_avg_sq, aa,
                          nullptr, s);
}

// ---- column-sharded table (table_sync "column") ------------------------------------------------
extern "C" int tt_bag_scale_rows(const float* d_pooled, const float* denom, int64_t nseq, int E, float* gs,
                                 tt_stream_t stream) {
  TT_REQUIRE(nseq >= 0 && E > 0 && E % 4 == 0, "tt_bag_scale_rows: nseq=%lld E=%d (E a multiple of 4)",
             (long long)nseq, E);
  TT_REQUIRE(nseq == 0 || (d_pooled && denom && gs), "null pointer");
  if (nseq == 0) return TT_OK;
  bag_scale_rows_kernel<<<dim3((unsigned)((nseq + kWavesPerBlock - 1) / kWavesPerBlock)), dim3(kBlock), 0,
                          reinterpret_cast<hipStream_t>(stream)>>>(d_pooled, denom, nseq, E, gs);
  TT_LAUNCH_CHECK("tt_bag_scale_rows");
  return TT_OK;
}

namespace tt {
namespace {
struct ColWs {
  int32_t *nch, *off, *plen, *goff, *hot_row, *hot_k0, *grp_row, *grp_g0;
  unsigned long long* cnt;  // {hot rows, pieces}, {group rows, groups}
  float *partial, *gpart;
  int64_t maxp, maxg;
  size_t total;
};
ColWs col_carve(void* base, int64_t V, int nsrc, int64_t nL, int El) {
  ColWs w{};
  const int64_t n = (int64_t)nsrc * nL;
  w.maxp = max_pieces_for(n);
  // groups: sum over rows of more than kMaxPieces pieces of ceil(np / kMaxPieces) <= maxp / 256 + (rows of
  // more than 32,768 tokens, at most n / 32,768 <= maxp / 512)
  w.maxg = 2 * ((w.maxp + kMaxPieces - 1) / kMaxPieces) + 1;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o = align_up(o + bytes, 256);
    return at;
  };
  const size_t onch = take((size_t)V * 4), ooff = take((size_t)V * 4), olen = take((size_t)V * 4),
               ogoff = take((size_t)V * 4), ocnt = take(16), ohr = take((size_t)w.maxp * 4),
               ohk = take((size_t)w.maxp * 4), ogr = take((size_t)w.maxg * 4), ogg = take((size_t)w.maxg * 4),
               opart = take((size_t)w.maxp * El * 4), ogp = take((size_t)w.maxg * El * 4);
  w.total = o + 256;
  if (base) {
    char* b = reinterpret_cast<char*>(align_up(reinterpret_cast<size_t>(base), 256));
    w.nch = reinterpret_cast<int32_t*>(b + onch);
    w.off = reinterpret_cast<int32_t*>(b + ooff);
    w.plen = reinterpret_cast<int32_t*>(b + olen);
    w.goff = reinterpret_cast<int32_t*>(b + ogoff);
    w.cnt = reinterpret_cast<unsigned long long*>(b + ocnt);
    w.hot_row = reinterpret_cast<int32_t*>(b + ohr);
    w.hot_k0 = reinterpret_cast<int32_t*>(b + ohk);
    w.grp_row = reinterpret_cast<int32_t*>(b + ogr);
    w.grp_g0 = reinterpret_cast<int32_t*>(b + ogg);
    w.partial = reinterpret_cast<float*>(b + opart);
    w.gpart = reinterpret_cast<float*>(b + ogp);
  }
  return w;
}
}  // namespace
}  // namespace tt

extern "C" size_t tt_bag_col_reduce_ws_size(int64_t V, int nsrc, int64_t nL, int El) {
  if (V <= 0 || nsrc <= 0 || nL < 0 || El <= 0) return 0;
  return col_carve(nullptr, V, nsrc, nL, El).total;
}

extern "C" int tt_bag_col_reduce(const int32_t* seg_all, const int32_t* vals_all, int64_t nL, int nsrc,
                                 int64_t nseq, const float* gs_all, int64_t V, int El, float* grad, float* slab,
                                 float* exp_avg, float* exp_avg_sq, const void* adam_args, tt_stream_t stream) {
  return tt_bag_col_reduce_ex(seg_all, vals_all, nL, nsrc, nseq, gs_all, V, El, grad, slab, exp_avg, exp_avg_sq,
                              adam_args, nullptr, 0, stream);
}

extern "C" int tt_bag_col_reduce_ex(const int32_t* seg_all, const int32_t* vals_all, int64_t nL, int nsrc,
                                    int64_t nseq, const float* gs_all, int64_t V, int El, float* grad, float* slab,
                                    float* exp_avg, float* exp_avg_sq, const void* adam_args, void* ws,
                                    size_t ws_bytes, tt_stream_t stream) {
  TT_REQUIRE(V > 0 && V < (int64_t(1) << 31) - 1 && nsrc > 0 && nseq >= 0 && nL >= 0 && nL < (int64_t(1) << 31),
             "tt_bag_col_reduce: bad shape (V=%lld nsrc=%d nseq=%lld nL=%lld)", (long long)V, nsrc, (long long)nseq,
             (long long)nL);
  TT_REQUIRE(El == 32 || El == 64 || El == 128 || El == 256, "tt_bag_col_reduce: El %d not in {32, 64, 128, 256}", El);
  TT_REQUIRE(seg_all && (nL == 0 || (vals_all && gs_all)), "null pointer");
  const bool fused = grad == nullptr;
  TT_REQUIRE(fused ? (slab && exp_avg && exp_avg_sq && adam_args) : true, "null pointer (fused update)");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const AdamArgs* aa = static_cast<const AdamArgs*>(adam_args);
  const int LPR = El / 4, rpi = kWave / LPR;
  const int64_t waves = (V + rpi - 1) / rpi;
  const dim3 grid((unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock)), block(kBlock);
  // hot rows (ws != NULL): piece plan, piece sums, group sums, then the reduce folds them
  ColPieces pcs{};
  ColWs w{};
  if (ws) {
    w = col_carve(ws, V, nsrc, nL, El);
    TT_REQUIRE(ws_bytes >= w.total, "tt_bag_col_reduce_ex: workspace %zu bytes < %zu", ws_bytes, w.total);
    TT_HIP(hipMemsetAsync(w.cnt, 0, 16, s), "memset piece counters");
    bag_col_pieces_kernel<<<dim3((unsigned)((V + kBlock - 1) / kBlock)), block, 0, s>>>(
        seg_all, nsrc, V, w.nch, w.off, w.plen, w.goff, w.cnt, w.hot_row, w.hot_k0, w.grp_row, w.grp_g0);
    TT_LAUNCH_CHECK("tt_bag_col_reduce (pieces)");
    pcs = ColPieces{w.nch, w.off, w.goff, w.partial, w.gpart};
  }
  auto sub_grid = [&](int64_t n) {  // n sub-wave jobs of El columns each, at most one round of waves
    return dim3((unsigned)std::min<int64_t>(
        kPieceSumMaxBlocks, std::max<int64_t>(1, ((n + rpi - 1) / rpi + kWavesPerBlock - 1) / kWavesPerBlock)));
  };
#define TT_COL(L)                                                                                             \
  do {                                                                                                        \
    if (ws) {                                                                                                 \
      bag_col_piece_sum_kernel<L><<<sub_grid(w.maxp), block, 0, s>>>(seg_all, vals_all, nL, nsrc, nseq, gs_all, V, \
                                                                     w.plen, w.cnt, w.hot_row, w.hot_k0, w.partial); \
      bag_col_group_sum_kernel<L><<<sub_grid(w.maxg), block, 0, s>>>(w.cnt, w.grp_row, w.grp_g0, w.nch, w.off,  \
                                                                     w.partial, w.gpart);                      \
    }                                                                                                         \
    if (fused)                                                                                                \
      bag_col_reduce_kernel<L, 4, true, false><<<grid, block, 0, s>>>(seg_all, vals_all, nL, nsrc, nseq, gs_all, V, \
                                                                     nullptr, slab, exp_avg, exp_avg_sq, aa, pcs); \
    else                                                                                                      \
      bag_col_reduce_kernel<L, 4, false, false><<<grid, block, 0, s>>>(seg_all, vals_all, nL, nsrc, nseq, gs_all, V, \
                                                                      grad, nullptr, nullptr, nullptr, nullptr, pcs); \
  } while (0)
  switch (El) {
    case 32: TT_COL(8); break;
    case 64: TT_COL(16); break;
    case 128: TT_COL(32); break;
    default: TT_COL(64); break;
  }
#undef TT_COL
  TT_LAUNCH_CHECK("tt_bag_col_reduce");
  return TT_OK;
}
