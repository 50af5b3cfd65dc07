// Device-resident batch feeder: the encoded (query, doc+, doc-) rows of a dataset live in HBM;
// each batch is gathered by a (shuffled) index list straight into the packed [q; p; n] int32
// buffer the fused TwoTower forward reads (replaces TripletDataset.__getitem__ + DataLoader
// collate + .to(device), twotower/dataset.py:262-285, twotower/train.py:411-417).
//
// One wave per destination row: L int32 ids (L*4 bytes) copied with 16-byte loads when the
// rows are 16-byte aligned, HBM-bound (a batch of 3 x 8192 x 64 ids is 6.3 MB).
#include "common.hpp"

namespace tt {
namespace {

constexpr int kBlock = 256;

template <bool VEC>
__global__ __launch_bounds__(kBlock) void gather_rows_kernel(const int32_t* __restrict__ src, int64_t ld_src,
                                                             int64_t n_src, const int64_t* __restrict__ idx,
                                                             int64_t n, int L, int32_t* __restrict__ dst,
                                                             int64_t ld_dst, int* __restrict__ bad) {
  const int64_t r = (int64_t)blockIdx.x * (kBlock / kWave) + (threadIdx.x >> 6);
  if (r >= n) return;
  const int lane = lane_id();
  const int64_t s = idx[r];
  int32_t* out = dst + r * ld_dst;
  if (s < 0 || s >= n_src) {  // out of range: a zero (all padding) row, and the flag is raised
    for (int c = lane; c < L; c += kWave) out[c] = 0;
    if (lane == 0) atomicOr(bad, 1);
    return;
  }
  const int32_t* in = src + s * ld_src;
  if constexpr (VEC) {
    for (int c = lane; c < L / 4; c += kWave)
      reinterpret_cast<int4*>(out)[c] = reinterpret_cast<const int4*>(in)[c];
  } else {
    for (int c = lane; c < L; c += kWave) out[c] = in[c];
  }
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

extern "C" int tt_gather_rows_i32(const int32_t* src, int64_t ld_src, int64_t n_src, const int64_t* idx, int64_t n,
                                  int L, int32_t* dst, int64_t ld_dst, int* bad, tt_stream_t stream) {
  TT_REQUIRE(n >= 0 && L >= 0 && n_src >= 0 && ld_src >= L && ld_dst >= L, "bad shape");
  if (n == 0 || L == 0) return TT_OK;
  TT_REQUIRE(src && idx && dst && bad, "null pointer");
  const bool vec = (L % 4 == 0) && (ld_src % 4 == 0) && (ld_dst % 4 == 0) &&
                   ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0;
  const dim3 grid((unsigned)((n + kBlock / kWave - 1) / (kBlock / kWave))), block(kBlock);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (vec)
    gather_rows_kernel<true><<<grid, block, 0, s>>>(src, ld_src, n_src, idx, n, L, dst, ld_dst, bad);
  else
    gather_rows_kernel<false><<<grid, block, 0, s>>>(src, ld_src, n_src, idx, n, L, dst, ld_dst, bad);
  TT_LAUNCH_CHECK("tt_gather_rows_i32");
  return TT_OK;
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
