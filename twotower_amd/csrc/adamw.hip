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

__device__ void prepare_slot(const tt_adam_slot& sl, double lr, double beta1, double beta2, double eps, double wd,
                             float inc, float ahead) {
  const float step = *sl.step + inc;
  if (inc != 0.f) *sl.step = step;
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
  *static_cast<AdamArgs*>(sl.args) = a;
}

__global__ void adam_prepare_kernel(PrepArgs pa, int count, double lr, double beta1, double beta2, double eps,
                                    double wd, float inc, float ahead) {
  const int i = threadIdx.x;
  if (i >= count) return;
  prepare_slot(pa.s[i], lr, beta1, beta2, eps, wd, inc, ahead);
}

// tt_adamw_multi_ex: tensors with slab partials form their gradient first (the sums of
// tt_head_wgrad2_reduce, bit for bit), write it to .grad and update; the last workgroup to
// finish (ticket) advances the counters and forms the next step's scalars (prepare_slot with
// increment 1, ahead 1), after every workgroup has read this step's.  One flat grid: tensor i
// owns blocks [start[i], start[i + 1]), sized to its own work (a bias takes two, not as many as
// the largest tensor).
struct MultiExArgs {
  tt_adamw_tensor t[TT_ADAM_MAX_TENSORS];
  tt_adamw_grad_parts g[TT_ADAM_MAX_TENSORS];
  tt_adam_slot next[TT_ADAM_MAX_TENSORS];
  int start[TT_ADAM_MAX_TENSORS + 1];
  int count, nnext;
  double lr, beta1, beta2, eps, wd;
  unsigned* ticket;
};

__device__ __forceinline__ void adam_update4(f32x4* p, f32x4* m, f32x4* v, int64_t i, f32x4 gg, const AdamArgs& a) {
  f32x4 pp = p[i], mm = m[i], vv = v[i];
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

// Was this workgroup the last of the launch to finish?  Two levels of relaxed device-scope
// counters: ticket[b % 8] counts the workgroups of one of eight groups, the last of a group
// counts into ticket[8].  One counter taking every workgroup's increment serialises them at the
// memory side (round 2: ≈ 10 us over ~1,000 workgroups, MI355X_MICROARCH.md 'dequeue': one word
// saturates at ≈ 88 increments per us); eight words take an eighth each.  Every wave has waited
// for its own loads before the increment, so the last workgroup's writes follow every read.
__device__ bool last_workgroup(unsigned* ticket, unsigned b, unsigned total) {
  __shared__ unsigned last;
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g = b & 7u, groups = total < 8u ? total : 8u;
    const unsigned in_group = (total - g + 7u) / 8u;
    bool l = false;
    if (__hip_atomic_fetch_add(ticket + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == in_group - 1u)
      l = __hip_atomic_fetch_add(ticket + 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == groups - 1u;
    last = l;
  }
  __syncthreads();
  return last;
}

__global__ __launch_bounds__(kBlock) void adamw_multi_ex_kernel(MultiExArgs ma) {
  __shared__ f32x4 red[kRedQ][64];
  const int b = blockIdx.x;
  int ti = 0;
  while (ti < ma.count && b >= ma.start[ti + 1]) ++ti;  // wave-uniform: <= 16 compares
  if (ti < ma.count && ma.t[ti].n > 0) {
    const tt_adamw_tensor& t = ma.t[ti];
    const tt_adamw_grad_parts& gp = ma.g[ti];
    const int64_t lb = b - ma.start[ti], nb = ma.start[ti + 1] - ma.start[ti];
    const AdamArgs a = *static_cast<const AdamArgs*>(t.args);
    f32x4* p4 = reinterpret_cast<f32x4*>(t.param);
    f32x4* m4 = reinterpret_cast<f32x4*>(t.exp_avg);
    f32x4* v4 = reinterpret_cast<f32x4*>(t.exp_avg_sq);
    if (gp.part) {
      // host-checked: 16-byte aligned, n % 4 == 0, stride % 4 == 0.  64 outputs per block pass,
      // four threads per output each summing a quarter of the slabs (sum_slabs), folded through
      // LDS as (q0 + q1) + (q2 + q3): tt_head_wgrad2_reduce's sums, bit for bit
      const int o = threadIdx.x & 63, qq = threadIdx.x >> 6;
      const int per = (gp.slabs + kRedQ - 1) / kRedQ;
      const int s0 = qq * per, s1 = min(gp.slabs, s0 + per);
      const int64_t n4 = t.n / 4;
      const f32x4* part4 = reinterpret_cast<const f32x4*>(gp.part);
      for (int64_t base = lb * 64; base < n4; base += nb * 64) {
        const int64_t i = base + o;
        red[qq][o] = i < n4 ? sum_slabs(part4 + i, (size_t)gp.stride / 4, s0, s1) : f32x4{0.f, 0.f, 0.f, 0.f};
        __syncthreads();
        if (qq == 0 && i < n4) {
          const f32x4 gg = (red[0][o] + red[1][o]) + (red[2][o] + red[3][o]);
          reinterpret_cast<f32x4*>(const_cast<float*>(t.grad))[i] = gg;
          adam_update4(p4, m4, v4, i, gg, a);
        }
        __syncthreads();
      }
    } else {
      const bool vec = ((reinterpret_cast<uintptr_t>(t.param) | reinterpret_cast<uintptr_t>(t.grad) |
                         reinterpret_cast<uintptr_t>(t.exp_avg) | reinterpret_cast<uintptr_t>(t.exp_avg_sq)) & 15) == 0;
      const int64_t n4 = vec ? t.n / 4 : 0;
      const int64_t stride = nb * kBlock;
      for (int64_t i = lb * kBlock + threadIdx.x; i < n4; i += stride)
        adam_update4(p4, m4, v4, i, reinterpret_cast<const f32x4*>(t.grad)[i], a);
      for (int64_t i = n4 * 4 + lb * kBlock + threadIdx.x; i < t.n; i += stride) {
        float pp = t.param[i], mm = t.exp_avg[i], vv = t.exp_avg_sq[i];
        adam_update(pp, t.grad[i], mm, vv, a);
        t.param[i] = pp;
        t.exp_avg[i] = mm;
        t.exp_avg_sq[i] = vv;
      }
    }
  }
  if (ma.nnext == 0) return;
  if (!last_workgroup(ma.ticket, (unsigned)b, gridDim.x)) return;
  if ((int)threadIdx.x < ma.nnext)
    prepare_slot(ma.next[threadIdx.x], ma.lr, ma.beta1, ma.beta2, ma.eps, ma.wd, 1.f, 1.f);
  if (threadIdx.x < 9)  // every count is in: reset the nine words for the next launch
    __hip_atomic_store(ma.ticket + threadIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

extern "C" int tt_adamw_multi_ex(const tt_adamw_tensor* tensors, const tt_adamw_grad_parts* parts, int count,
                                 const tt_adam_slot* next, int nnext, double lr, double beta1, double beta2,
                                 double eps, double weight_decay, unsigned* ticket, tt_stream_t stream) {
  TT_REQUIRE(count >= 0 && count <= TT_ADAM_MAX_TENSORS, "count=%d (max %d)", count, TT_ADAM_MAX_TENSORS);
  TT_REQUIRE(nnext >= 0 && nnext <= TT_ADAM_MAX_TENSORS, "nnext=%d (max %d)", nnext, TT_ADAM_MAX_TENSORS);
  TT_REQUIRE(count == 0 || tensors != nullptr, "null tensors");
  TT_REQUIRE(nnext == 0 || (next != nullptr && ticket != nullptr), "nnext=%d needs slots and a ticket", nnext);
  MultiExArgs ma{};
  for (int i = 0; i < count; ++i) {
    const tt_adamw_tensor& t = tensors[i];
    TT_REQUIRE(t.n >= 0, "tensor %d: n=%lld", i, (long long)t.n);
    TT_REQUIRE(t.n == 0 || (t.param && t.grad && t.exp_avg && t.exp_avg_sq && t.args), "tensor %d: null pointer", i);
    ma.t[i] = t;
    if (parts && parts[i].part && t.n > 0) {
      const tt_adamw_grad_parts& g = parts[i];
      TT_REQUIRE(g.slabs >= 1 && g.stride >= t.n && g.stride % 4 == 0 && t.n % 4 == 0,
                 "tensor %d: slab partials need slabs >= 1, stride >= n, stride and n multiples of 4", i);
      TT_REQUIRE(((reinterpret_cast<uintptr_t>(t.param) | reinterpret_cast<uintptr_t>(t.grad) |
                   reinterpret_cast<uintptr_t>(t.exp_avg) | reinterpret_cast<uintptr_t>(t.exp_avg_sq) |
                   reinterpret_cast<uintptr_t>(g.part)) & 15) == 0,
                 "tensor %d: slab partials need 16-byte aligned buffers", i);
      ma.g[i] = g;
    }
  }
  for (int i = 0; i < nnext; ++i) {
    TT_REQUIRE(next[i].step && next[i].args, "null step/args in slot %d", i);
    TT_REQUIRE((reinterpret_cast<uintptr_t>(next[i].args) & 3) == 0, "args of slot %d misaligned", i);
    ma.next[i] = next[i];
  }
  ma.count = count;
  ma.nnext = nnext;
  ma.lr = lr;
  ma.beta1 = beta1;
  ma.beta2 = beta2;
  ma.eps = eps;
  ma.wd = weight_decay;
  ma.ticket = ticket;
  if (count == 0 && nnext == 0) return TT_OK;
  // blocks per tensor: its own vec4 grid-stride cover (+1 for a scalar tail), or one block per 64
  // outputs when it sums slab partials; at most 512 each
  int total = 0;
  for (int i = 0; i < count; ++i) {
    ma.start[i] = total;
    const int64_t n = tensors[i].n;
    int64_t nb = n > 0 ? (n / 4 + kBlock - 1) / kBlock + 1 : 0;
    if (ma.g[i].part) nb = std::max<int64_t>(nb, (n / 4 + 63) / 64);
    total += (int)std::min<int64_t>(nb, 512);
  }
  ma.start[count] = total;
  if (total == 0) total = 1;  // scalars only: one workgroup
  adamw_multi_ex_kernel<<<dim3((unsigned)total), dim3(kBlock), 0, reinterpret_cast<hipStream_t>(stream)>>>(ma);
  TT_LAUNCH_CHECK("tt_adamw_multi_ex");
  return TT_OK;
}
