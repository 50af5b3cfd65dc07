// Shared device/host helpers for libtwotower_amd (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstddef>

#include "../../include/twotower_amd.h"

namespace tt {

void set_error(const char* fmt, ...);

constexpr int kWave = 64;  // CDNA wavefront; never 32

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// Write-through (sc1) 16-B / 4-B stores: the line leaves the XCD's L2 as it is written, so a launch
// that hands large outputs to the next one ends without dirty L2 lines to write back at the
// boundary (MI355X_MICROARCH.md price list, 'boundary': + dirty bytes / 6 TB/s; 'publish-large':
// 16-B sc1 stores cost what plain ones do; 4-B sc1 stores cost ~6x per byte, so only 16-B sites
// use them).  A buffer store: the cache-policy bits are the builtin's operand (sc1 = 16 on gfx950)
// and the compiler keeps the data registers live as for any store.  `base` must be wave-uniform
// (an array base); the byte offset is per lane and below 4 GiB.
typedef unsigned tt_u32x4 __attribute__((ext_vector_type(4)));
// a wave-uniform address as the compiler's SGPR pair (readfirstlane returns int: each half goes
// through uint32_t, or the low half would sign-extend over the high one)
__device__ __forceinline__ uint64_t uniform_addr(const void* p) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)p);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uintptr_t)p >> 32));
  return (uint64_t)lo | ((uint64_t)hi << 32);
}
template <typename V16>
__device__ __forceinline__ void store16_wt(void* base, uint32_t byte_off, const V16& v) {
  static_assert(sizeof(V16) == 16, "16-B stores");
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc((void*)uniform_addr(base), 0, (int)0xffffffffu, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(tt_u32x4, v), r, byte_off, 0, 16 /* sc1 */);
}
__device__ __forceinline__ void store4_wt(void* base, uint32_t byte_off, float v) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc((void*)uniform_addr(base), 0, (int)0xffffffffu, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, byte_off, 0, 16 /* sc1 */);
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

// v0^2 + v1^2 + v2^2 + v3^2 with its fma chain spelled out, so every kernel that forms a row
// norm from the same float4 gets the same bits (contraction of the plain expression may pick
// either product as the fma addend, differently per kernel).
__device__ __forceinline__ float sumsq4(const f32x4& v) {
  return __builtin_fmaf(v[3], v[3], __builtin_fmaf(v[2], v[2], __builtin_fmaf(v[1], v[1], v[0] * v[0])));
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// F.normalize backward (encoders.py:77, autograd of x / max(|x|, 1e-12)) of one H = 256 row held
// as one float4 per lane: g = d(out), o = out, nrm = |x|.  Every fma spelled out, so the tower
// head's own backward (l2norm_bwd_kernel) and the in-batch combine that fuses it
// (bwd_combine_l2_kernel) produce the same bits.
__device__ __forceinline__ f32x4 l2_bwd_row4(const f32x4& g, const f32x4& o, float nrm) {
  const float den = fmaxf(nrm, 1e-12f);
  const float dot = __builtin_fmaf(g[3], o[3], __builtin_fmaf(g[2], o[2], __builtin_fmaf(g[1], o[1], g[0] * o[0])));
  const float sx4 = wave_sum(dot) * den;
  const float coef4 = (nrm >= 1e-12f && nrm > 0.f) ? sx4 / ((den * den) * nrm) : 0.f;
  f32x4 y;
#pragma unroll
  for (int k = 0; k < 4; ++k) y[k] = __builtin_fmaf(-coef4, o[k] * den, g[k] / den);
  return y;
}

// The same for an H = 128 row held as elements (lane, lane + 64) of each lane (g0, g1 / o0, o1):
// l2norm_bwd_kernel at H = 128 and the fp32 in-batch combine that fuses it (bwd_combine_l2_128_kernel)
// both take it, so they agree bit for bit.
__device__ __forceinline__ void l2_bwd_row2(float g0, float g1, float o0, float o1, float nrm, float& y0, float& y1) {
  const float den = fmaxf(nrm, 1e-12f);
  const float sx = wave_sum(__builtin_fmaf(g1, o1, g0 * o0)) * den;
  const float coef = (nrm >= 1e-12f && nrm > 0.f) ? sx / ((den * den) * nrm) : 0.f;
  y0 = __builtin_fmaf(-coef, o0 * den, g0 / den);
  y1 = __builtin_fmaf(-coef, o1 * den, g1 / den);
}

template <typename IdT>
__device__ __forceinline__ int64_t load_id(const IdT* p) { return (int64_t)(*p); }

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// torch.optim.AdamW (foreach form, amsgrad=False, maximize=False) with the per-step scalars
// precomputed on the host in double exactly as torch does in Python floats.
struct AdamArgs {
  float wd_factor;  // 1 - lr * weight_decay
  float one_m_b1;   // lerp weight 1 - beta1
  float beta2;
  float one_m_b2;   // 1 - beta2
  float step_size;  // lr / (1 - beta1^step)
  float bc2_sqrt;   // sqrt(1 - beta2^step)
  float eps;
};

inline AdamArgs make_adam(double lr, double beta1, double beta2, double eps, double wd, int64_t step) {
  AdamArgs a;
  const double bc1 = 1.0 - __builtin_pow(beta1, (double)step);
  const double bc2 = 1.0 - __builtin_pow(beta2, (double)step);
  a.wd_factor = (float)(1.0 - lr * wd);
  a.one_m_b1 = (float)(1.0 - beta1);
  a.beta2 = (float)beta2;
  a.one_m_b2 = (float)(1.0 - beta2);
  a.step_size = (float)(lr / bc1);
  a.bc2_sqrt = (float)__builtin_sqrt(bc2);
  a.eps = (float)eps;
  return a;
}

// Every fused multiply-add is spelled out, so the rounding does not depend on how the
// compiler contracts the expression in each kernel that inlines it (it had picked different
// contractions of v's update in two kernels: 1-ulp differences).
__device__ __forceinline__ void adam_update(float& p, float g, float& m, float& v, const AdamArgs& a) {
  m = __builtin_fmaf(a.one_m_b1, g - m, m);               // exp_avg.lerp_(grad, 1 - beta1)
  v = __builtin_fmaf(v, a.beta2, (a.one_m_b2 * g) * g);   // exp_avg_sq.mul_(b2).addcmul_(g, g, 1 - b2)
  const float den = sqrtf(v) / a.bc2_sqrt + a.eps;
  // param.mul_(1 - lr * wd), then param.addcdiv_(exp_avg, denom, -step_size)
  p = __builtin_fmaf(p, a.wd_factor, -(a.step_size * (m / den)));
}


// The tower head's weight planes (tt_head_split*, head.hip): each fp32 weight is cut into three
// bf16 terms, x = a0 + a1 + a2 exactly.  Job j of SplitJobs writes the three planes of an n x k
// matrix (W is n x k, or k x n when transposed) at planes_base + off[j]; element i = n * k + k'.
// Shared by split_planes_kernel and the bag forward's split workgroups (tt_bag_mean_fwd_split),
// so both produce the same bits.
__device__ __forceinline__ void split3(float x, __bf16& a0, __bf16& a1, __bf16& a2) {
  a0 = (__bf16)x;
  const float r1 = x - (float)a0;
  a1 = (__bf16)r1;
  a2 = (__bf16)(r1 - (float)a1);
}

struct SplitJobs {
  const float* W[4];
  int transpose[4];
  int n[4], k[4];
  int64_t off[4];
};

__device__ __forceinline__ void split_planes_elem(const SplitJobs& jobs, int job, int i, __bf16* __restrict__ planes_base) {
  const int nn = jobs.n[job], kk = jobs.k[job];
  if (i >= nn * kk) return;
  const float* W = jobs.W[job];
  __bf16* planes = planes_base + jobs.off[job];
  const int n = i / kk, k = i % kk;
  const float x = jobs.transpose[job] ? W[k * nn + n] : W[n * kk + k];
  __bf16 a0, a1, a2;
  split3(x, a0, a1, a2);
  planes[i] = a0;
  planes[nn * kk + i] = a1;
  planes[2 * nn * kk + i] = a2;
}

// The four plane sets of an E -> H Linear-ReLU-Linear head: W1 (H x E), W2 (H x H), W1^T (E x H),
// W2^T (H x H), each three bf16 planes, consecutive in that order (tt_head_split_ff2).
inline SplitJobs head_ff2_jobs(const float* W1, const float* W2, int E, int H) {
  const int64_t a = 3LL * H * E, b = 3LL * H * H;
  return SplitJobs{{W1, W2, W1, W2}, {0, 0, 1, 1}, {H, H, E, H}, {E, H, H, H}, {0, a, a + b, 2 * a + b}};
}

// Fixed-order sum of slab partials (tt_head_wgrad2_reduce, tt_adamw_multi_ex): slabs are cut
// into kRedQ quarters; a quarter's slab s goes to partial s % 8 (8 loads in flight), the eight
// partials fold in a fixed tree, and the callers add the quarters as (q0 + q1) + (q2 + q3).
constexpr int kRedQ = 4;
__device__ __forceinline__ f32x4 sum_slabs(const f32x4* __restrict__ p, size_t stride4, int s_begin, int s_end) {
  f32x4 a[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) a[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int s0 = s_begin; s0 < s_end; s0 += 8) {
    f32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = s0 + u < s_end ? p[(size_t)(s0 + u) * stride4] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] += v[u];
  }
  return ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}

// mean_kernel's arithmetic (rows.hip: 1024 threads, thread t adds x[t + 1024 k] in order with
// eight loads in flight, then a halving tree over the 1024 partials) run by one 256-thread
// block, each thread standing in for threads t, t + 256, t + 512, t + 768: the same adds in the
// same order, so the same bits.  `part` is 1024 floats of LDS.  Every thread returns the mean.
__device__ inline float block256_mean_as_1024(const float* __restrict__ x, int64_t n, float* part) {
  const int t = threadIdx.x;
  // thread t's four partials (t + 256 k, k < 4) in element order, eight elements per round with
  // the eight loads in flight (unconditional clamped loads; the adds skip what lies past n).  Kept
  // to eight registers of loads: the block shares its kernel's register budget with latency-bound
  // rows (32 in flight doubled bwd_combine's VGPRs and halved its occupancy).
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float s = 0.f;
    for (int64_t i0 = t + 256 * k; i0 < n; i0 += 8 * 1024) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int64_t i = i0 + 1024 * u;
        v[u] = x[i < n ? i : n - 1];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (i0 + 1024 * u < n) s += v[u];
    }
    part[t + 256 * k] = s;
  }
  __syncthreads();
  part[t] += part[t + 512];  // w = 512: threads t and t + 256 of the 1024
  part[t + 256] += part[t + 768];
  __syncthreads();
  for (int w = 256; w > 0; w >>= 1) {
    if (t < w) part[t] += part[t + w];
    __syncthreads();
  }
  return n > 0 ? part[0] / (float)n : __builtin_nanf("");
}

}  // namespace tt

#define TT_REQUIRE(cond, ...)                 \
  do {                                        \
    if (!(cond)) {                            \
      tt::set_error(__VA_ARGS__);             \
      return TT_ERR_INVALID;                  \
    }                                         \
  } while (0)

#define TT_LAUNCH_CHECK(what)                                                   \
  do {                                                                          \
    hipError_t _e = hipGetLastError();                                          \
    if (_e != hipSuccess) {                                                     \
      tt::set_error("%s: launch failed: %s", what, hipGetErrorString(_e));     \
      return (int)_e;                                                           \
    }                                                                           \
  } while (0)

#define TT_HIP(call, what)                                                      \
  do {                                                                          \
    hipError_t _e = (call);                                                     \
    if (_e != hipSuccess) {                                                     \
      tt::set_error("%s: %s", what, hipGetErrorString(_e));                    \
      return (int)_e;                                                           \
    }                                                                           \
  } while (0)
