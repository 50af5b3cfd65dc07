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

// One launch over up to TT_ADAM_MAX_TENSORS tensors (blockIdx.y = tensor), each with its own
// device-resident scalars (tt_adam_prepare): the small tower parameters in one launch.
struct MultiArgs {
  tt_adamw_tensor t[TT_ADAM_MAX_TENSORS];
};

__global__ __launch_bounds__(kBlock) void adamw_multi_kernel(MultiArgs ma) {
  const tt_adamw_tensor& t = ma.t[blockIdx.y];
  if (t.n == 0) return;
  const AdamArgs a = *static_cast<const AdamArgs*>(t.args);
  const bool vec = ((reinterpret_cast<uintptr_t>(t.param) | reinterpret_cast<uintptr_t>(t.grad) |
                     reinterpret_cast<uintptr_t>(t.exp_avg) | reinterpret_cast<uintptr_t>(t.exp_avg_sq)) & 15) == 0;
  const int64_t n4 = vec ? t.n / 4 : 0;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n4; i += stride) {
    f32x4 pp = reinterpret_cast<f32x4*>(t.param)[i], gg = reinterpret_cast<const f32x4*>(t.grad)[i];
    f32x4 mm = reinterpret_cast<f32x4*>(t.exp_avg)[i], vv = reinterpret_cast<f32x4*>(t.exp_avg_sq)[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float pj = pp[j], mj = mm[j], vj = vv[j];
      adam_update(pj, gg[j], mj, vj, a);
      pp[j] = pj;
      mm[j] = mj;
      vv[j] = vj;
    }
    reinterpret_cast<f32x4*>(t.param)[i] = pp;
    reinterpret_cast<f32x4*>(t.exp_avg)[i] = mm;
    reinterpret_cast<f32x4*>(t.exp_avg_sq)[i] = vv;
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < t.n; i += stride) {
    float pp = t.param[i], mm = t.exp_avg[i], vv = t.exp_avg_sq[i];
    adam_update(pp, t.grad[i], mm, vv, a);
    t.param[i] = pp;
    t.exp_avg[i] = mm;
    t.exp_avg_sq[i] = vv;
  }
}

// step += 1 on the device, then the per-step AdamW scalars in double exactly as make_adam does on
// the host (torch computes them in Python floats), rounded to fp32 once.
struct PrepArgs {
  tt_adam_slot s[TT_ADAM_MAX_TENSORS];
};

__global__ void adam_prepare_kernel(PrepArgs pa, int count, double lr, double beta1, double beta2, double eps,
                                    double wd, float inc, float ahead) {
  const int i = threadIdx.x;
  if (i >= count) return;
  const float step = *pa.s[i].step + inc;
  if (inc != 0.f) *pa.s[i].step = step;
  const float at = step + ahead;  // the step whose scalars are formed
  const double bc1 = 1.0 - pow(beta1, (double)at);
  const double bc2 = 1.0 - pow(beta2, (double)at);
  AdamArgs a;
  a.wd_factor = (float)(1.0 - lr * wd);
  a.one_m_b1 = (float)(1.0 - beta1);
  a.beta2 = (float)beta2;
  a.one_m_b2 = (float)(1.0 - beta2);
  a.step_size = (float)(lr / bc1);
  a.bc2_sqrt = (float)sqrt(bc2);
  a.eps = (float)eps;
  *static_cast<AdamArgs*>(pa.s[i].args) = a;
}

static_assert(sizeof(AdamArgs) <= TT_ADAM_ARGS_BYTES, "AdamArgs does not fit TT_ADAM_ARGS_BYTES");

}  // namespace
}  // namespace tt

using namespace tt;

extern "C" int tt_adam_prepare(const tt_adam_slot* slots, int count, double lr, double beta1, double beta2,
                               double eps, double weight_decay, tt_stream_t stream) {
  return tt_adam_prepare_ex(slots, count, lr, beta1, beta2, eps, weight_decay, 1, 0, stream);
}

extern "C" int tt_adam_prepare_ex(const tt_adam_slot* slots, int count, double lr, double beta1, double beta2,
                                  double eps, double weight_decay, int increment, int ahead, tt_stream_t stream) {
  TT_REQUIRE(increment == 0 || increment == 1, "increment=%d", increment);
  TT_REQUIRE(ahead == 0 || ahead == 1, "ahead=%d", ahead);
  TT_REQUIRE(count >= 0 && count <= TT_ADAM_MAX_TENSORS, "count=%d (max %d)", count, TT_ADAM_MAX_TENSORS);
  if (count == 0) return TT_OK;
  TT_REQUIRE(slots != nullptr, "null slots");
  PrepArgs pa{};
  for (int i = 0; i < count; ++i) {
    TT_REQUIRE(slots[i].step && slots[i].args, "null step/args in slot %d", i);
    TT_REQUIRE((reinterpret_cast<uintptr_t>(slots[i].args) & 3) == 0, "args of slot %d misaligned", i);
    pa.s[i] = slots[i];
  }
  adam_prepare_kernel<<<dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream)>>>(
      pa, count, lr, beta1, beta2, eps, weight_decay, (float)increment, (float)ahead);
  TT_LAUNCH_CHECK("tt_adam_prepare");
  return TT_OK;
}

extern "C" int tt_adamw_multi(const tt_adamw_tensor* tensors, int count, tt_stream_t stream) {
  TT_REQUIRE(count >= 0 && count <= TT_ADAM_MAX_TENSORS, "count=%d (max %d)", count, TT_ADAM_MAX_TENSORS);
  if (count == 0) return TT_OK;
  TT_REQUIRE(tensors != nullptr, "null tensors");
  MultiArgs ma{};
  int64_t nmax = 0;
  for (int i = 0; i < count; ++i) {
    const tt_adamw_tensor& t = tensors[i];
    TT_REQUIRE(t.n >= 0, "tensor %d: n=%lld", i, (long long)t.n);
    TT_REQUIRE(t.n == 0 || (t.param && t.grad && t.exp_avg && t.exp_avg_sq && t.args), "tensor %d: null pointer", i);
    ma.t[i] = t;
    nmax = std::max(nmax, t.n);
  }
  if (nmax == 0) return TT_OK;
  const int64_t bx = std::min<int64_t>((nmax / 4 + kBlock - 1) / kBlock + 1, 512);
  adamw_multi_kernel<<<dim3((unsigned)bx, (unsigned)count), dim3(kBlock), 0, reinterpret_cast<hipStream_t>(stream)>>>(ma);
  TT_LAUNCH_CHECK("tt_adamw_multi");
  return TT_OK;
}

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
