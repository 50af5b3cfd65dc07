// Device-resident batch feeder: the encoded (query, doc+, doc-) rows of a dataset live in HBM;
// each batch is gathered by a (shuffled) index list straight into the packed [q; p; n] int32
// buffer the fused TwoTower forward reads (replaces TripletDataset.__getitem__ + DataLoader
// collate + .to(device), twotower/dataset.py:262-285, twotower/train.py:411-417).
//
// A group of lanes per destination row (16 at L = 64: one 16-byte unit each), the three fields
// in one launch, HBM-bound (a batch of 3 x 8192 x 64 ids is 6.3 MB).
#include "common.hpp"

namespace tt {
namespace {

constexpr int kBlock = 256;

// G lanes per destination row (G = 64 / rows per wave), 16-byte units when the rows are 16-byte
// aligned; blockIdx.y = the field (q, d+, d-: src / dst advanced by their field strides).  An
// index out of range writes a zero (all padding) row and raises the flag: atomicMax(bad, gen), so
// a caller that passes a new gen per call reads "bad == gen" without clearing the flag first.
template <typename U, int G>
__global__ __launch_bounds__(kBlock) void gather_rows_kernel(const int32_t* __restrict__ src, int64_t ld_src,
                                                             int64_t n_src, int64_t src_field,
                                                             const int64_t* __restrict__ idx, int64_t n, int L,
                                                             int32_t* __restrict__ dst, int64_t ld_dst,
                                                             int64_t dst_field, int* __restrict__ bad, int gen) {
  constexpr int kRows = kBlock / G;
  const int64_t r = (int64_t)blockIdx.x * kRows + threadIdx.x / G;
  if (r >= n) return;
  const int g = threadIdx.x % G;
  const int64_t s = idx[r];
  constexpr int kPer = sizeof(U) / 4;  // int32 per unit
  U* out = reinterpret_cast<U*>(dst + blockIdx.y * dst_field + r * ld_dst);
  const int units = L / kPer;
  if (s < 0 || s >= n_src) {
    for (int c = g; c < units; c += G) out[c] = U{};
    if (g == 0) atomicMax(bad, gen);
    return;
  }
  const U* in = reinterpret_cast<const U*>(src + blockIdx.y * src_field + s * ld_src);
  for (int c = g; c < units; c += G) out[c] = in[c];
}

// tt_pack_blocks: up to kPackMax contiguous byte blocks copied into consecutive ranges of one
// buffer (the graph-replayed step's packed [q; p; n] input) in one launch, 16 bytes per lane
// when every block is 16-byte sized and aligned, bytes otherwise.
constexpr int kPackMax = 8;
struct PackArgs {
  const char* src[kPackMax];
  int64_t start[kPackMax + 1];  // units (16 B or 1 B) before each block; start[count] = total
  int count;
};

// blockIdx.y = the block of the source (a uniform index into the kernel arguments), one unit
// per lane over a grid that covers the largest source.  (Four units per lane over a quarter of
// the grid measured 20-24 us for the C3 batch instead of 6-7.)
template <typename U>
__global__ __launch_bounds__(kBlock) void pack_blocks_kernel(PackArgs pa, char* __restrict__ dst) {
  const int k = blockIdx.y;
  const int64_t n = pa.start[k + 1] - pa.start[k];
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i < n) (reinterpret_cast<U*>(dst) + pa.start[k])[i] = reinterpret_cast<const U*>(pa.src[k])[i];
}

}  // namespace
}  // namespace tt

using namespace tt;

extern "C" int tt_pack_blocks(const void* const* srcs, const int64_t* bytes, int count, void* dst,
                              tt_stream_t stream) {
  TT_REQUIRE(count >= 0 && count <= kPackMax, "count=%d (max %d)", count, kPackMax);
  TT_REQUIRE(count == 0 || (srcs && bytes), "null srcs/bytes");
  PackArgs pa{};
  pa.count = count;
  int64_t total = 0;
  bool vec = (reinterpret_cast<uintptr_t>(dst) & 15) == 0;
  for (int k = 0; k < count; ++k) {
    TT_REQUIRE(bytes[k] >= 0, "block %d: bytes=%lld", k, (long long)bytes[k]);
    TT_REQUIRE(bytes[k] == 0 || srcs[k], "block %d: null source", k);
    pa.src[k] = static_cast<const char*>(srcs[k]);
    vec = vec && bytes[k] % 16 == 0 && (reinterpret_cast<uintptr_t>(srcs[k]) & 15) == 0;
    total += bytes[k];
  }
  if (total == 0) return TT_OK;
  TT_REQUIRE(dst, "null dst");
  const int64_t unit = vec ? 16 : 1;
  int64_t acc = 0;
  for (int k = 0; k < count; ++k) {
    pa.start[k] = acc;
    acc += bytes[k] / unit;
  }
  pa.start[count] = acc;
  int64_t most = 0;
  for (int k = 0; k < count; ++k) most = std::max(most, pa.start[k + 1] - pa.start[k]);
  TT_REQUIRE((most + kBlock - 1) / kBlock < (int64_t(1) << 31), "pack_blocks: a block of %lld units is too large",
             (long long)most);
  const int64_t blocks = std::max<int64_t>(1, (most + kBlock - 1) / kBlock);
  const dim3 grid((unsigned)blocks, (unsigned)count);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (vec)
    pack_blocks_kernel<int4><<<grid, dim3(kBlock), 0, s>>>(pa, static_cast<char*>(dst));
  else
    pack_blocks_kernel<char><<<grid, dim3(kBlock), 0, s>>>(pa, static_cast<char*>(dst));
  TT_LAUNCH_CHECK("tt_pack_blocks");
  return TT_OK;
}

extern "C" int tt_gather_rows_i32_ex(const int32_t* src, int64_t ld_src, int64_t n_src, int64_t src_field,
                                     int nfield, const int64_t* idx, int64_t n, int L, int32_t* dst, int64_t ld_dst,
                                     int64_t dst_field, int* bad, int gen, tt_stream_t stream) {
  TT_REQUIRE(n >= 0 && L >= 0 && n_src >= 0 && ld_src >= L && ld_dst >= L && nfield >= 1 && nfield <= 65535,
             "bad shape");
  TT_REQUIRE(gen >= 1, "gen=%d must be >= 1", gen);
  if (n == 0 || L == 0) return TT_OK;
  TT_REQUIRE(src && idx && dst && bad, "null pointer");
  const bool vec = (L % 4 == 0) && (ld_src % 4 == 0) && (ld_dst % 4 == 0) && (src_field % 4 == 0) &&
                   (dst_field % 4 == 0) &&
                   ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int units = vec ? L / 4 : L;
  // lanes per row: the units of a row rounded up to a power of two, 4..64
  int G = 4;
  while (G < 64 && G < units) G <<= 1;
  const dim3 grid((unsigned)((n + kBlock / G - 1) / (kBlock / G)), (unsigned)nfield), block(kBlock);
#define TT_GATHER(U, GG)                                                                                     \
  gather_rows_kernel<U, GG><<<grid, block, 0, s>>>(src, ld_src, n_src, src_field, idx, n, L, dst, ld_dst,   \
                                                   dst_field, bad, gen)
  if (vec) {
    switch (G) {
      case 4: TT_GATHER(int4, 4); break;
      case 8: TT_GATHER(int4, 8); break;
      case 16: TT_GATHER(int4, 16); break;
      case 32: TT_GATHER(int4, 32); break;
      default: TT_GATHER(int4, 64); break;
    }
  } else {
    switch (G) {
      case 4: TT_GATHER(int, 4); break;
      case 8: TT_GATHER(int, 8); break;
      case 16: TT_GATHER(int, 16); break;
      case 32: TT_GATHER(int, 32); break;
      default: TT_GATHER(int, 64); break;
    }
  }
#undef TT_GATHER
  TT_LAUNCH_CHECK("tt_gather_rows_i32");
  return TT_OK;
}

extern "C" int tt_gather_rows_i32(const int32_t* src, int64_t ld_src, int64_t n_src, const int64_t* idx, int64_t n,
                                  int L, int32_t* dst, int64_t ld_dst, int* bad, tt_stream_t stream) {
  return tt_gather_rows_i32_ex(src, ld_src, n_src, 0, 1, idx, n, L, dst, ld_dst, 0, bad, 1, stream);
}

// ------------------------------------------------------------------------------------------
// Measurement: one device timestamp (the constant-rate wall clock, tt_wall_clock_khz ticks per
// ms) written by a one-wave kernel, so that a captured graph can time the ops it replays: stamps
// launched around an op on its stream run after the previous kernel of that stream and before the
// next (bench.py's stamped replay).  Lane 0 stores through a vector store; nothing reads the slot
// on the device.
namespace {
__global__ __launch_bounds__(64) void stamp_kernel(unsigned long long* __restrict__ slot) {
  const unsigned long long t = wall_clock64();
  if (threadIdx.x == 0) *slot = t;
}
}  // namespace

extern "C" int tt_stamp(uint64_t* slot, tt_stream_t stream) {
  TT_REQUIRE(slot && (reinterpret_cast<uintptr_t>(slot) & 7) == 0, "tt_stamp: 8-byte aligned slot");
  stamp_kernel<<<dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream)>>>(
      reinterpret_cast<unsigned long long*>(slot));
  TT_LAUNCH_CHECK("tt_stamp");
  return TT_OK;
}

extern "C" int tt_wall_clock_khz(int device) {
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess) return -1;
  return khz;
}
