// Dense AdamW over a flat fp32 parameter (torch.optim.AdamW at twotower/train.py:359, stepped at
// :139).  HBM-bound: 28 B per parameter (read p, g, m, v; write p, m, v), 16 B per lane per
// stream, grid-stride at <= 8 blocks per CU.
#include "common.hpp"

namespace tt {
namespace {

constexpr int kBlock = 256;

__global__ __launch_bounds__(kBlock) void adamw_vec4_kernel(f32x4* __restrict__ p, const f32x4* __restrict__ g,
                                                            f32x4* __restrict__ m, f32x4* __restrict__ v,
                                                            int64_t n4, AdamArgs a) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kBlock) {
    f32x4 pp = p[i], gg = g[i], mm = m[i], vv = v[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float pj = pp[j], mj = mm[j], vj = vv[j];
      adam_update(pj, gg[j], mj, vj, a);
      pp[j] = pj;
      mm[j] = mj;
      vv[j] = vj;
    }
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
  }
}

__global__ __launch_bounds__(kBlock) void adamw_scalar_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                              float* __restrict__ m, float* __restrict__ v,
                                                              int64_t n, AdamArgs a) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    float pp = p[i], mm = m[i], vv = v[i];
    adam_update(pp, g[i], mm, vv, a);
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
  }
}

}  // namespace
}  // namespace tt

using namespace tt;

extern "C" int tt_adamw(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, double lr,
                        double beta1, double beta2, double eps, double weight_decay, int64_t step, tt_stream_t stream) {
  TT_REQUIRE(n >= 0, "n=%lld", (long long)n);
  TT_REQUIRE(step >= 1, "step must be >= 1 (got %lld)", (long long)step);
  if (n == 0) return TT_OK;
  TT_REQUIRE(param && grad && exp_avg && exp_avg_sq, "null pointer");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const AdamArgs a = make_adam(lr, beta1, beta2, eps, weight_decay, step);
  const bool aligned = ((reinterpret_cast<uintptr_t>(param) | reinterpret_cast<uintptr_t>(grad) |
                         reinterpret_cast<uintptr_t>(exp_avg) | reinterpret_cast<uintptr_t>(exp_avg_sq)) & 15) == 0;
  const int64_t n4 = aligned ? n / 4 : 0;
  if (n4 > 0) {
    const int64_t blocks = std::min<int64_t>((n4 + kBlock - 1) / kBlock, 256 * 8);
    adamw_vec4_kernel<<<dim3((unsigned)blocks), dim3(kBlock), 0, s>>>(
        reinterpret_cast<f32x4*>(param), reinterpret_cast<const f32x4*>(grad), reinterpret_cast<f32x4*>(exp_avg),
        reinterpret_cast<f32x4*>(exp_avg_sq), n4, a);
    TT_LAUNCH_CHECK("tt_adamw(vec4)");
  }
  const int64_t done = n4 * 4, rest = n - done;
  if (rest > 0) {
    const int64_t blocks = std::min<int64_t>((rest + kBlock - 1) / kBlock, 256 * 8);
    adamw_scalar_kernel<<<dim3((unsigned)blocks), dim3(kBlock), 0, s>>>(param + done, grad + done, exp_avg + done,
                                                                     exp_avg_sq + done, rest, a);
    TT_LAUNCH_CHECK("tt_adamw(scalar)");
  }
  return TT_OK;
}
