// Row-wise kernels of the tower output and the per-sample losses:
//   F.normalize(x, dim=-1)                       twotower/encoders.py:77  (eps 1e-12)
//   contrastive_triplet_loss                     twotower/losses.py:9-44  (cosine eps 1e-8)
//   multiple_negatives_loss                      twotower/losses.py:47-85
//   deterministic mean of per-row losses          (.mean() / F.cross_entropy reduction)
// One wavefront owns one row; rows are <= a few KiB so re-reads within a wave hit L1/L2.
// Cosine follows ATen's cosine_similarity: sum((x1 / clamp(|x1|, eps)) * (x2 / clamp(|x2|, eps))),
// whose backward differentiates the norm but not the clamp.
#include "common.hpp"

namespace tt {
namespace {

constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;

__device__ __forceinline__ int64_t wave_row() { return (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6); }

__global__ __launch_bounds__(kBlock) void l2norm_fwd_kernel(const float* __restrict__ x, int64_t rows, int H,
                                                            float* __restrict__ out, float* __restrict__ norm) {
  const int64_t r = wave_row();
  if (r >= rows) return;
  const int lane = lane_id();
  const float* xr = x + r * H;
  float ss = 0.f;
  for (int c = lane; c < H; c += kWave) ss += xr[c] * xr[c];
  ss = wave_sum(ss);
  const float nrm = sqrtf(ss);
  const float den = fmaxf(nrm, 1e-12f);
  for (int c = lane; c < H; c += kWave) out[r * H + c] = xr[c] / den;
  if (lane == 0) norm[r] = nrm;
}

__global__ __launch_bounds__(kBlock) void l2norm_bwd_kernel(const float* __restrict__ dout, const float* __restrict__ out,
                                                            const float* __restrict__ norm, int64_t rows, int H,
                                                            float* __restrict__ dx) {
  const int64_t r = wave_row();
  if (r >= rows) return;
  const int lane = lane_id();
  const float nrm = norm[r];
  const float den = fmaxf(nrm, 1e-12f);
  if (H == 4 * kWave) {  // one float4 per lane, both rows kept in registers
    const f32x4 g = reinterpret_cast<const f32x4*>(dout + r * H)[lane];
    const f32x4 o = reinterpret_cast<const f32x4*>(out + r * H)[lane];
    reinterpret_cast<f32x4*>(dx + r * H)[lane] = l2_bwd_row4(g, o, nrm);
    return;
  }
  if (H == 2 * kWave) {  // elements lane and lane + 64 (the fp32 in-batch combine's fused form)
    const float* gr = dout + r * H;
    const float* orow = out + r * H;
    float y0, y1;
    l2_bwd_row2(gr[lane], gr[lane + kWave], orow[lane], orow[lane + kWave], nrm, y0, y1);
    dx[r * H + lane] = y0;
    dx[r * H + lane + kWave] = y1;
    return;
  }
  // x = out * den; s_x = sum(dout * x)
  float sx = 0.f;
  for (int c = lane; c < H; c += kWave) sx += dout[r * H + c] * out[r * H + c];
  sx = wave_sum(sx) * den;
  const float coef = (nrm >= 1e-12f && nrm > 0.f) ? sx / (den * den * nrm) : 0.f;
  for (int c = lane; c < H; c += kWave) {
    const float xv = out[r * H + c] * den;
    dx[r * H + c] = dout[r * H + c] / den - coef * xv;
  }
}

// ---- LayerNorm -> L2 normalise (AveragePoolingTower's projection tail, encoders.py:95-97,150):
// y = (x - mean) * rstd * gamma + beta (biased variance, rstd = 1/sqrt(var + eps) as ATen),
// out = y / max(|y|, 1e-12).  stats per row: mean, rstd, |y|.
__global__ __launch_bounds__(kBlock) void ln_l2_fwd_kernel(const float* __restrict__ x, int64_t rows, int H,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, float eps,
                                                           float* __restrict__ out, float* __restrict__ stats) {
  const int64_t r = wave_row();
  if (r >= rows) return;
  const int lane = lane_id();
  const float* xr = x + r * H;
  float s = 0.f;
  for (int c = lane; c < H; c += kWave) s += xr[c];
  const float mean = wave_sum(s) / (float)H;
  float v = 0.f;
  for (int c = lane; c < H; c += kWave) v += (xr[c] - mean) * (xr[c] - mean);
  const float rstd = 1.f / sqrtf(fmaxf(wave_sum(v) / (float)H, 0.f) + eps);
  float ss = 0.f;
  for (int c = lane; c < H; c += kWave) {
    const float y = (xr[c] - mean) * rstd * gamma[c] + beta[c];
    ss += y * y;
  }
  const float nrm = sqrtf(wave_sum(ss)), den = fmaxf(nrm, 1e-12f);
  for (int c = lane; c < H; c += kWave) out[r * H + c] = ((xr[c] - mean) * rstd * gamma[c] + beta[c]) / den;
  if (lane == 0) {
    stats[3 * r] = mean;
    stats[3 * r + 1] = rstd;
    stats[3 * r + 2] = nrm;
  }
}

// The same forward with the row held in registers (U = ceil(H / 64) floats per lane, H <= 1024):
// one global read per element instead of three, the same sums in the same order (bit-identical).
template <int U>
__global__ __launch_bounds__(kBlock) void ln_l2_fwd_reg_kernel(const float* __restrict__ x, int64_t rows, int H,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ beta, float eps,
                                                               float* __restrict__ out, float* __restrict__ stats) {
  const int64_t r = wave_row();
  if (r >= rows) return;
  const int lane = lane_id();
  const float* xr = x + r * H;
  float xv[U];
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int c = lane + kWave * u;
    xv[u] = c < H ? xr[c] : 0.f;
    if (c < H) s += xv[u];
  }
  const float mean = wave_sum(s) / (float)H;
  float v = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (lane + kWave * u < H) v += (xv[u] - mean) * (xv[u] - mean);
  const float rstd = 1.f / sqrtf(fmaxf(wave_sum(v) / (float)H, 0.f) + eps);
  float y[U], ss = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int c = lane + kWave * u;
    y[u] = 0.f;
    if (c < H) {
      y[u] = (xv[u] - mean) * rstd * gamma[c] + beta[c];
      ss += y[u] * y[u];
    }
  }
  const float nrm = sqrtf(wave_sum(ss)), den = fmaxf(nrm, 1e-12f);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int c = lane + kWave * u;
    if (c < H) out[r * H + c] = y[u] / den;
  }
  if (lane == 0) {
    stats[3 * r] = mean;
    stats[3 * r + 1] = rstd;
    stats[3 * r + 2] = nrm;
  }
}

// Backward: dy = F.normalize backward (norm differentiated, clamp not); LayerNorm backward
// dx = rstd (dxhat - mean(dxhat) - xhat mean(dxhat xhat)), dxhat = dy gamma; the per-row
// gamma/beta contributions (dy xhat, dy) go to gx / gb for fixed-order column sums.
__global__ __launch_bounds__(kBlock) void ln_l2_bwd_kernel(const float* __restrict__ dout, const float* __restrict__ x,
                                                           int64_t rows, int H, const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           const float* __restrict__ stats, float* __restrict__ dx,
                                                           float* __restrict__ gx, float* __restrict__ gb) {
  const int64_t r = wave_row();
  if (r >= rows) return;
  const int lane = lane_id();
  const float mean = stats[3 * r], rstd = stats[3 * r + 1], nrm = stats[3 * r + 2];
  const float den = fmaxf(nrm, 1e-12f);
  const float* xr = x + r * H;
  const float* dr = dout + r * H;
  float sy = 0.f;
  for (int c = lane; c < H; c += kWave) sy += dr[c] * ((xr[c] - mean) * rstd * gamma[c] + beta[c]);
  const float coef = (nrm >= 1e-12f && nrm > 0.f) ? wave_sum(sy) / (den * den * nrm) : 0.f;
  float a = 0.f, b = 0.f;
  for (int c = lane; c < H; c += kWave) {
    const float xh = (xr[c] - mean) * rstd;
    const float dy = dr[c] / den - coef * (xh * gamma[c] + beta[c]);
    gx[r * H + c] = dy * xh;
    gb[r * H + c] = dy;
    const float dxh = dy * gamma[c];
    a += dxh;
    b += dxh * xh;
  }
  a = wave_sum(a) / (float)H;
  b = wave_sum(b) / (float)H;
  for (int c = lane; c < H; c += kWave) {
    const float xh = (xr[c] - mean) * rstd;
    dx[r * H + c] = rstd * (gb[r * H + c] * gamma[c] - a - xh * b);
  }
}

// The same backward with the gamma / beta terms folded over each workgroup's 4 rows before they
// are written (ln_l2_bwd_kernel writes them per row for two column-sum launches: 2 x 2 full
// passes of extra traffic).  One wave per row as there (lane l: columns l + 64 u); the
// workgroup folds its 4 waves in a fixed order into row blockIdx.x of part (nwg x 2H: gamma
// terms, then beta terms), whose columns the colsum kernels then sum in a fixed order.  dx is
// the same arithmetic as ln_l2_bwd_kernel's, element for element.
template <int U>
__global__ __launch_bounds__(kBlock) void ln_l2_bwd_fold_kernel(const float* __restrict__ dout,
                                                                const float* __restrict__ x, int64_t rows, int H,
                                                                const float* __restrict__ gamma,
                                                                const float* __restrict__ beta,
                                                                const float* __restrict__ stats,
                                                                float* __restrict__ dx, float* __restrict__ part) {
  __shared__ float red[kWavesPerBlock][2][U * kWave];
  const int lane = lane_id(), wid = threadIdx.x >> 6;
  float gam[U], bet[U], ga[U], ba[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int c = lane + kWave * u;
    gam[u] = c < H ? gamma[c] : 0.f;
    bet[u] = c < H ? beta[c] : 0.f;
    ga[u] = ba[u] = 0.f;
  }
  const int64_t r = wave_row();
  if (r < rows) {
    const float mean = stats[3 * r], rstd = stats[3 * r + 1], nrm = stats[3 * r + 2];
    const float den = fmaxf(nrm, 1e-12f);
    float xh[U], d[U], sy = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = lane + kWave * u;
      xh[u] = d[u] = 0.f;
      if (c < H) {
        xh[u] = (x[r * H + c] - mean) * rstd;
        d[u] = dout[r * H + c];
        sy += d[u] * (xh[u] * gam[u] + bet[u]);
      }
    }
    const float coef = (nrm >= 1e-12f && nrm > 0.f) ? wave_sum(sy) / (den * den * nrm) : 0.f;
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (lane + kWave * u < H) {
        const float dy = d[u] / den - coef * (xh[u] * gam[u] + bet[u]);
        ga[u] += dy * xh[u];
        ba[u] += dy;
        const float dxh = dy * gam[u];
        a += dxh;
        b += dxh * xh[u];
        d[u] = dy;
      }
    }
    a = wave_sum(a) / (float)H;
    b = wave_sum(b) / (float)H;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = lane + kWave * u;
      if (c < H) dx[r * H + c] = rstd * (d[u] * gam[u] - a - xh[u] * b);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    red[wid][0][lane + kWave * u] = ga[u];
    red[wid][1][lane + kWave * u] = ba[u];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < H; c += kBlock) {
    float g = red[0][0][c], bb = red[0][1][c];
    for (int w = 1; w < kWavesPerBlock; ++w) {
      g += red[w][0][c];
      bb += red[w][1][c];
    }
    part[(int64_t)blockIdx.x * 2 * H + c] = g;
    part[(int64_t)blockIdx.x * 2 * H + H + c] = bb;
  }
}

struct CosStats {
  float dot, n1, n2;  // raw dot and unclamped norms
};

__device__ __forceinline__ CosStats cos_stats(const float* a, const float* b, int H) {
  float d = 0.f, s1 = 0.f, s2 = 0.f;
  for (int c = lane_id(); c < H; c += kWave) {
    const float x = a[c], y = b[c];
    d += x * y;
    s1 += x * x;
    s2 += y * y;
  }
  return CosStats{wave_sum(d), sqrtf(wave_sum(s1)), sqrtf(wave_sum(s2))};
}

__device__ __forceinline__ float cos_value(const CosStats& s) {
  return s.dot / (fmaxf(s.n1, 1e-8f) * fmaxf(s.n2, 1e-8f));
}

// d cos / d x1 = x2 / (n1c n2c) - cos * x1 / (n1c * n1)   (0 at n1 == 0)
__device__ __forceinline__ void cos_grad_coefs(const CosStats& s, float cosv, float& a_other, float& a_self1,
                                               float& a_self2) {
  const float n1c = fmaxf(s.n1, 1e-8f), n2c = fmaxf(s.n2, 1e-8f);
  a_other = 1.f / (n1c * n2c);
  a_self1 = s.n1 > 0.f ? cosv / (n1c * s.n1) : 0.f;
  a_self2 = s.n2 > 0.f ? cosv / (n2c * s.n2) : 0.f;
}

__global__ __launch_bounds__(kBlock) void triplet_fwd_kernel(const float* __restrict__ q, const float* __restrict__ p,
                                                             const float* __restrict__ n, int64_t B, int H, float margin,
                                                             float* __restrict__ loss_rows) {
  const int64_t r = wave_row();
  if (r >= B) return;
  const CosStats sp = cos_stats(q + r * H, p + r * H, H);
  const CosStats sn = cos_stats(q + r * H, n + r * H, H);
  const float h = margin - cos_value(sp) + cos_value(sn);
  if (lane_id() == 0) loss_rows[r] = fmaxf(h, 0.f);
}

__global__ __launch_bounds__(kBlock) void triplet_bwd_kernel(const float* __restrict__ q, const float* __restrict__ p,
                                                             const float* __restrict__ n, int64_t B, int H, float margin,
                                                             const float* __restrict__ grad_loss,
                                                             float* __restrict__ dq, float* __restrict__ dp,
                                                             float* __restrict__ dn) {
  const int64_t r = wave_row();
  if (r >= B) return;
  const float* qr = q + r * H;
  const float* pr = p + r * H;
  const float* nr = n + r * H;
  const CosStats sp = cos_stats(qr, pr, H);
  const CosStats sn = cos_stats(qr, nr, H);
  const float cp = cos_value(sp), cn = cos_value(sn);
  const float h = margin - cp + cn;
  const float gate = (h > 0.f) ? grad_loss[0] / (float)B : 0.f;  // relu' and mean
  const float gcp = -gate, gcn = gate;
  float ap, aqp, app, an, aqn, ann;
  cos_grad_coefs(sp, cp, ap, aqp, app);
  cos_grad_coefs(sn, cn, an, aqn, ann);
  for (int c = lane_id(); c < H; c += kWave) {
    const float qv = qr[c], pv = pr[c], nv = nr[c];
    dq[r * H + c] = gcp * (pv * ap - aqp * qv) + gcn * (nv * an - aqn * qv);
    dp[r * H + c] = gcp * (qv * ap - app * pv);
    dn[r * H + c] = gcn * (qv * an - ann * nv);
  }
}

constexpr int kMaxNeg = 63;

__device__ __forceinline__ const float* mn_doc(const float* p, const float* negs, int64_t r, int k, int N, int H) {
  return k == 0 ? p + r * H : negs + (r * N + (k - 1)) * (int64_t)H;
}

__global__ __launch_bounds__(kBlock) void multi_neg_fwd_kernel(const float* __restrict__ q, const float* __restrict__ p,
                                                               const float* __restrict__ negs, int64_t B, int N, int H,
                                                               float inv_tau, float* __restrict__ loss_rows) {
  const int64_t r = wave_row();
  if (r >= B) return;
  const float* qr = q + r * H;
  float mx = -INFINITY, z0 = 0.f;
  float z[kMaxNeg + 1];
  for (int k = 0; k <= N; ++k) {
    z[k] = cos_value(cos_stats(qr, mn_doc(p, negs, r, k, N, H), H)) * inv_tau;
    mx = fmaxf(mx, z[k]);
  }
  z0 = z[0];
  float se = 0.f;
  for (int k = 0; k <= N; ++k) se += expf(z[k] - mx);
  if (lane_id() == 0) loss_rows[r] = mx + logf(se) - z0;
}

__global__ __launch_bounds__(kBlock) void multi_neg_bwd_kernel(const float* __restrict__ q, const float* __restrict__ p,
                                                               const float* __restrict__ negs, int64_t B, int N, int H,
                                                               float inv_tau, const float* __restrict__ grad_loss,
                                                               float* __restrict__ dq, float* __restrict__ dp,
                                                               float* __restrict__ dnegs) {
  const int64_t r = wave_row();
  if (r >= B) return;
  const float* qr = q + r * H;
  CosStats st[kMaxNeg + 1];
  float cs[kMaxNeg + 1];
  float mx = -INFINITY;
  for (int k = 0; k <= N; ++k) {
    st[k] = cos_stats(qr, mn_doc(p, negs, r, k, N, H), H);
    cs[k] = cos_value(st[k]);
    mx = fmaxf(mx, cs[k] * inv_tau);
  }
  float se = 0.f;
  for (int k = 0; k <= N; ++k) se += expf(cs[k] * inv_tau - mx);
  const float g = grad_loss[0] / (float)B;
  for (int c = lane_id(); c < H; c += kWave) dq[r * H + c] = 0.f;
  for (int k = 0; k <= N; ++k) {
    const float pk = expf(cs[k] * inv_tau - mx) / se;
    const float gcos = g * (pk - (k == 0 ? 1.f : 0.f)) * inv_tau;
    float a_other, a_q, a_d;
    cos_grad_coefs(st[k], cs[k], a_other, a_q, a_d);
    const float* dr = mn_doc(p, negs, r, k, N, H);
    float* ddr = (k == 0) ? dp + r * H : dnegs + (r * N + (k - 1)) * (int64_t)H;
    for (int c = lane_id(); c < H; c += kWave) {
      const float qv = qr[c], dv = dr[c];
      dq[r * H + c] += gcos * (dv * a_other - a_q * qv);
      ddr[c] = gcos * (qv * a_other - a_d * dv);
    }
  }
}

// H = 256 fast path (C5: B x (1 + N) documents of 1 KiB): one float4 per lane, the query and all
// 1 + N document rows loaded up front (register arrays indexed by unrolled constants, NMAX
// documents at most), every partial dot / squared norm reduced in one batch of wave sums, and
// each gradient row written once (no read-modify-write of dq).  Same formulas as the generic
// kernels above; the column sum order differs (4 consecutive columns per lane).
__device__ __forceinline__ float dot4(const f32x4& a, const f32x4& b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3];
}

template <int NMAX>
struct MnRows {
  f32x4 q, d[NMAX + 1];
  CosStats st[NMAX + 1];
};

template <int NMAX>
__device__ __forceinline__ void mn_load_stats(const float* __restrict__ q, const float* __restrict__ p,
                                              const float* __restrict__ negs, int64_t r, int N, MnRows<NMAX>& m) {
  const int lane = lane_id();
  m.q = reinterpret_cast<const f32x4*>(q + r * 256)[lane];
#pragma unroll
  for (int k = 0; k <= NMAX; ++k)
    if (k <= N) m.d[k] = reinterpret_cast<const f32x4*>(mn_doc(p, negs, r, k, N, 256))[lane];
  const float qq = wave_sum(dot4(m.q, m.q));
  const float n1 = sqrtf(qq);
#pragma unroll
  for (int k = 0; k <= NMAX; ++k)
    if (k <= N) {
      m.st[k].dot = wave_sum(dot4(m.q, m.d[k]));
      m.st[k].n1 = n1;
      m.st[k].n2 = sqrtf(wave_sum(dot4(m.d[k], m.d[k])));
    }
}

template <int NMAX>
__global__ __launch_bounds__(kBlock) void multi_neg_fwd_h256_kernel(const float* __restrict__ q,
                                                                    const float* __restrict__ p,
                                                                    const float* __restrict__ negs, int64_t B, int N,
                                                                    float inv_tau, float* __restrict__ loss_rows) {
  const int64_t r = wave_row();
  if (r >= B) return;
  MnRows<NMAX> m;
  mn_load_stats<NMAX>(q, p, negs, r, N, m);
  float z[NMAX + 1], mx = -INFINITY;
#pragma unroll
  for (int k = 0; k <= NMAX; ++k)
    if (k <= N) {
      z[k] = cos_value(m.st[k]) * inv_tau;
      mx = fmaxf(mx, z[k]);
    }
  float se = 0.f;
#pragma unroll
  for (int k = 0; k <= NMAX; ++k)
    if (k <= N) se += expf(z[k] - mx);
  if (lane_id() == 0) loss_rows[r] = mx + logf(se) - z[0];
}

// l2n non-null (tt_multi_neg_bwd_l2: q, p, negs are the consecutive row blocks of the tower head's
// output [q; p; negs] and l2n its row norms in that order): each gradient row goes through the head's
// F.normalize backward (l2_bwd_row4, l2norm_bwd_kernel's arithmetic) before it is stored, so the
// head needs no L2 backward pass of its own (bit for bit the two launches).
template <int NMAX>
__global__ __launch_bounds__(kBlock) void multi_neg_bwd_h256_kernel(const float* __restrict__ q,
                                                                    const float* __restrict__ p,
                                                                    const float* __restrict__ negs, int64_t B, int N,
                                                                    float inv_tau, const float* __restrict__ grad_loss,
                                                                    float* __restrict__ dq, float* __restrict__ dp,
                                                                    float* __restrict__ dnegs,
                                                                    const float* __restrict__ l2n = nullptr) {
  const int64_t r = wave_row();
  if (r >= B) return;
  const int lane = lane_id();
  MnRows<NMAX> m;
  mn_load_stats<NMAX>(q, p, negs, r, N, m);
  float cs[NMAX + 1], mx = -INFINITY;
#pragma unroll
  for (int k = 0; k <= NMAX; ++k)
    if (k <= N) {
      cs[k] = cos_value(m.st[k]);
      mx = fmaxf(mx, cs[k] * inv_tau);
    }
  float se = 0.f;
#pragma unroll
  for (int k = 0; k <= NMAX; ++k)
    if (k <= N) se += expf(cs[k] * inv_tau - mx);
  const float g = grad_loss[0] / (float)B;
  f32x4 gq = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k <= NMAX; ++k)
    if (k <= N) {
      const float pk = expf(cs[k] * inv_tau - mx) / se;
      const float gcos = g * (pk - (k == 0 ? 1.f : 0.f)) * inv_tau;
      float a_other, a_q, a_d;
      cos_grad_coefs(m.st[k], cs[k], a_other, a_q, a_d);
      f32x4 gd;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        gq[j] += gcos * (m.d[k][j] * a_other - a_q * m.q[j]);
        gd[j] = gcos * (m.q[j] * a_other - a_d * m.d[k][j]);
      }
      float* ddr = (k == 0) ? dp + r * 256 : dnegs + (r * N + (k - 1)) * (int64_t)256;
      if (l2n) gd = l2_bwd_row4(gd, m.d[k], l2n[k == 0 ? B + r : 2 * B + r * N + (k - 1)]);
      reinterpret_cast<f32x4*>(ddr)[lane] = gd;
    }
  if (l2n) gq = l2_bwd_row4(gq, m.q, l2n[r]);
  reinterpret_cast<f32x4*>(dq + r * 256)[lane] = gq;
}

// One workgroup: fixed-order strided partial sums then a fixed tree => bitwise reproducible.
__global__ __launch_bounds__(1024) void mean_kernel(const float* __restrict__ x, int64_t n, float* __restrict__ out) {
  __shared__ float part[1024];
  float s = 0.f;
  int64_t i = threadIdx.x;
  for (; i + 7 * 1024 < n; i += 8 * 1024) {  // eight loads in flight, then the same sequential adds
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = x[i + u * 1024];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; i < n; i += 1024) s += x[i];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int w = 512; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = n > 0 ? part[0] / (float)n : NAN;
}

// Column sums, deterministic, two levels.  Level 1: block b owns rows [b*kColRows, ...): 256
// threads = 4 row groups x 64 float4 columns (cols % 4 == 0, cols <= 256 per block column),
// each thread keeps 4 independent partial sums (16 loads in flight), the 4 row groups are added
// in a fixed order through LDS.  Level 2: 4 threads per column add the block partials (strided,
// 4 accumulators each) and fold them in a fixed order.
constexpr int kColRows = 256;

__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* __restrict__ x, int64_t rows, int cols,
                                                             float* __restrict__ part) {
  __shared__ f32x4 red[4][64];
  const int cq = threadIdx.x & 63, rg = threadIdx.x >> 6;  // float4 column, row group
  const int c4 = blockIdx.y * 64 + cq;
  const bool ok = c4 * 4 < cols;
  const int64_t r0 = (int64_t)blockIdx.x * kColRows;
  const int64_t r1 = min<int64_t>(rows, r0 + kColRows);
  f32x4 a[4] = {f32x4{}, f32x4{}, f32x4{}, f32x4{}};
  if (ok) {
    const f32x4* src = reinterpret_cast<const f32x4*>(x) + c4;
    const int stride4 = cols / 4;
    int64_t r = r0 + rg;
    for (; r + 12 < r1; r += 16) {
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] += src[(r + 4 * u) * stride4];
    }
    for (int u = 0; r < r1; r += 4, ++u) a[u & 3] += src[r * stride4];
  }
  red[rg][cq] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (rg == 0 && ok)
    reinterpret_cast<f32x4*>(part + (int64_t)blockIdx.x * cols)[c4] =
        (red[0][cq] + red[1][cq]) + (red[2][cq] + red[3][cq]);
}

__global__ __launch_bounds__(256) void colsum_final_kernel(const float* __restrict__ part, int nblk, int cols,
                                                           float* __restrict__ out) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < cols) {
    int b = g;
    for (; b + 12 < nblk; b += 16) {
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] += part[(int64_t)(b + 4 * u) * cols + c];
    }
    for (int u = 0; b < nblk; b += 4, ++u) a[u & 3] += part[(int64_t)b * cols + c];
  }
  red[g][cl] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (g == 0 && c < cols) out[c] = (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]);
}

dim3 rows_grid(int64_t rows) { return dim3((unsigned)((rows + kWavesPerBlock - 1) / kWavesPerBlock)); }

}  // namespace

int launch_mean(const float* x, int64_t n, float* out, hipStream_t s) {
  mean_kernel<<<dim3(1), dim3(1024), 0, s>>>(x, n, out);
  TT_LAUNCH_CHECK("mean");
  return TT_OK;
}

extern "C" int tt_mean(const float* x, int64_t n, float* out, tt_stream_t stream) {
  TT_REQUIRE(out && (x || n == 0) && n >= 0, "bad mean arguments");
  return launch_mean(x, n, out, reinterpret_cast<hipStream_t>(stream));
}

}  // namespace tt

using namespace tt;

namespace tt {
namespace {
// 16-byte alignment of every non-null pointer (the float4 fast paths)
inline bool aligned16(const void* a, const void* b, const void* c) {
  return ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) | reinterpret_cast<uintptr_t>(c)) & 15) == 0;
}
}  // namespace
}  // namespace tt

extern "C" int tt_l2norm_fwd(const float* x, int64_t rows, int H, float* out, float* norm, tt_stream_t stream) {
  TT_REQUIRE(rows >= 0 && H > 0, "bad shape rows=%lld H=%d", (long long)rows, H);
  if (rows == 0) return TT_OK;
  TT_REQUIRE(x && out && norm, "null pointer");
  l2norm_fwd_kernel<<<rows_grid(rows), dim3(kBlock), 0, reinterpret_cast<hipStream_t>(stream)>>>(x, rows, H, out, norm);
  TT_LAUNCH_CHECK("tt_l2norm_fwd");
  return TT_OK;
}

extern "C" int tt_ln_l2_fwd(const float* x, int64_t rows, int H, const float* gamma, const float* beta, float eps,
                            float* out, float* stats, tt_stream_t stream) {
  TT_REQUIRE(rows >= 0 && H > 0, "bad shape rows=%lld H=%d", (long long)rows, H);
  if (rows == 0) return TT_OK;
  TT_REQUIRE(x && gamma && beta && out && stats, "null pointer");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int U = (H + kWave - 1) / kWave;
#define TT_LNR(UU) ln_l2_fwd_reg_kernel<UU><<<rows_grid(rows), dim3(kBlock), 0, s>>>(x, rows, H, gamma, beta, eps, out, stats)
  if (U <= 1)
    TT_LNR(1);
  else if (U <= 2)
    TT_LNR(2);
  else if (U <= 4)
    TT_LNR(4);
  else if (U <= 8)
    TT_LNR(8);
  else if (U <= 16)
    TT_LNR(16);
  else
    ln_l2_fwd_kernel<<<rows_grid(rows), dim3(kBlock), 0, s>>>(x, rows, H, gamma, beta, eps, out, stats);
#undef TT_LNR
  TT_LAUNCH_CHECK("tt_ln_l2_fwd");
  return TT_OK;
}

extern "C" int tt_ln_l2_bwd(const float* dout, const float* x, int64_t rows, int H, const float* gamma,
                            const float* beta, const float* stats, float* dx, float* gx, float* gb,
                            tt_stream_t stream) {
  TT_REQUIRE(rows >= 0 && H > 0, "bad shape rows=%lld H=%d", (long long)rows, H);
  if (rows == 0) return TT_OK;
  TT_REQUIRE(dout && x && gamma && beta && stats && dx && gx && gb, "null pointer");
  ln_l2_bwd_kernel<<<rows_grid(rows), dim3(kBlock), 0, reinterpret_cast<hipStream_t>(stream)>>>(
      dout, x, rows, H, gamma, beta, stats, dx, gx, gb);
  TT_LAUNCH_CHECK("tt_ln_l2_bwd");
  return TT_OK;
}

extern "C" int tt_l2norm_bwd(const float* dout, const float* out, const float* norm, int64_t rows, int H, float* dx,
                             tt_stream_t stream) {
  TT_REQUIRE(rows >= 0 && H > 0, "bad shape rows=%lld H=%d", (long long)rows, H);
  if (rows == 0) return TT_OK;
  TT_REQUIRE(dout && out && norm && dx, "null pointer");
  l2norm_bwd_kernel<<<rows_grid(rows), dim3(kBlock), 0, reinterpret_cast<hipStream_t>(stream)>>>(dout, out, norm, rows,
                                                                                                 H, dx);
  TT_LAUNCH_CHECK("tt_l2norm_bwd");
  return TT_OK;
}

__global__ __launch_bounds__(256) void relu_bwd_kernel(float* __restrict__ dh, const float* __restrict__ h, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    f32x4 d = reinterpret_cast<f32x4*>(dh)[i];
    const f32x4 v = reinterpret_cast<const f32x4*>(h)[i];
#pragma unroll
    for (int j = 0; j < 4; ++j) d[j] = v[j] > 0.f ? d[j] : 0.f;
    reinterpret_cast<f32x4*>(dh)[i] = d;
  }
}

__global__ __launch_bounds__(256) void relu_bwd_scalar_kernel(float* __restrict__ dh, const float* __restrict__ h,
                                                               int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    dh[i] = h[i] > 0.f ? dh[i] : 0.f;
}

extern "C" int tt_relu_bwd(float* dh, const float* h, int64_t n, tt_stream_t stream) {
  TT_REQUIRE(n >= 0, "tt_relu_bwd: n=%lld", (long long)n);
  if (n == 0) return TT_OK;
  TT_REQUIRE(dh && h, "tt_relu_bwd: null pointer");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const bool vec = n % 4 == 0 && ((reinterpret_cast<uintptr_t>(dh) | reinterpret_cast<uintptr_t>(h)) & 15) == 0;
  if (vec)
    relu_bwd_kernel<<<dim3((unsigned)std::min<int64_t>((n / 4 + 255) / 256, 2048)), dim3(256), 0, s>>>(dh, h, n / 4);
  else
    relu_bwd_scalar_kernel<<<dim3((unsigned)std::min<int64_t>((n + 255) / 256, 2048)), dim3(256), 0, s>>>(dh, h, n);
  TT_LAUNCH_CHECK("tt_relu_bwd");
  return TT_OK;
}

extern "C" size_t tt_colsum_ws_size(int64_t rows, int cols) {
  const int64_t nblk = (rows + kColRows - 1) / kColRows;
  return (size_t)std::max<int64_t>(nblk, 1) * (size_t)cols * sizeof(float);
}

extern "C" int tt_colsum(const float* x, int64_t rows, int cols, float* out, void* ws, size_t ws_bytes,
                         tt_stream_t stream) {
  TT_REQUIRE(rows >= 0 && cols > 0, "bad shape rows=%lld cols=%d", (long long)rows, cols);
  TT_REQUIRE(out && (rows == 0 || (x && ws)), "null pointer");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (rows == 0) {
    TT_HIP(hipMemsetAsync(out, 0, (size_t)cols * 4, s), "memset colsum");
    return TT_OK;
  }
  TT_REQUIRE(ws_bytes >= tt_colsum_ws_size(rows, cols), "workspace too small");
  TT_REQUIRE(cols % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0,
             "tt_colsum needs cols %% 4 == 0 and a 16-byte aligned x");
  const int nblk = (int)((rows + kColRows - 1) / kColRows);
  colsum_partial_kernel<<<dim3(nblk, (cols + 255) / 256), dim3(256), 0, s>>>(x, rows, cols, static_cast<float*>(ws));
  colsum_final_kernel<<<dim3((cols + 63) / 64), dim3(256), 0, s>>>(static_cast<const float*>(ws), nblk, cols, out);
  TT_LAUNCH_CHECK("tt_colsum");
  return TT_OK;
}

extern "C" size_t tt_ln_l2_bwd_ws_size(int64_t rows, int H) {
  const int64_t nwg = (std::max<int64_t>(rows, 1) + kWavesPerBlock - 1) / kWavesPerBlock;
  const int64_t nblk = (nwg + kColRows - 1) / kColRows;
  return (size_t)(nwg + nblk) * 2 * (size_t)H * sizeof(float) + 2 * (size_t)H * sizeof(float);
}

// dgamma / dbeta land in the workspace's tail (2H floats) and are copied out: the column sums of
// the (nwg x 2H) fold are one colsum over 2H columns (2H % 4 == 0: H even).
__global__ void split_pair_kernel(const float* __restrict__ v, int H, float* __restrict__ a, float* __restrict__ b) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < H) {
    a[c] = v[c];
    b[c] = v[H + c];
  }
}

extern "C" int tt_ln_l2_bwd_ex(const float* dout, const float* x, int64_t rows, int H, const float* gamma,
                               const float* beta, const float* stats, float* dx, float* dgamma, float* dbeta, void* ws,
                               size_t ws_bytes, tt_stream_t stream) {
  TT_REQUIRE(rows >= 0 && H > 0 && H <= 16 * kWave && H % 2 == 0, "bad shape rows=%lld H=%d (H even, <= 1024)",
             (long long)rows, H);
  TT_REQUIRE(gamma && beta && dgamma && dbeta, "null pointer");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (rows == 0) {
    TT_HIP(hipMemsetAsync(dgamma, 0, (size_t)H * 4, s), "memset dgamma");
    TT_HIP(hipMemsetAsync(dbeta, 0, (size_t)H * 4, s), "memset dbeta");
    return TT_OK;
  }
  TT_REQUIRE(dout && x && stats && dx && ws, "null pointer");
  TT_REQUIRE(ws_bytes >= tt_ln_l2_bwd_ws_size(rows, H), "workspace too small");
  const int64_t nwg = (rows + kWavesPerBlock - 1) / kWavesPerBlock;
  const int cols = 2 * H;
  float* part = static_cast<float*>(ws);
  float* cpart = part + nwg * cols;
  float* both = cpart + ((nwg + kColRows - 1) / kColRows) * cols;
  const int U = (H + kWave - 1) / kWave;
#define TT_LNF(UU)                                                                                           \
  ln_l2_bwd_fold_kernel<UU><<<dim3((unsigned)nwg), dim3(kBlock), 0, s>>>(dout, x, rows, H, gamma, beta, stats, dx, part)
  if (U <= 1)
    TT_LNF(1);
  else if (U <= 2)
    TT_LNF(2);
  else if (U <= 4)
    TT_LNF(4);
  else if (U <= 8)
    TT_LNF(8);
  else
    TT_LNF(16);
#undef TT_LNF
  const int nblk = (int)((nwg + kColRows - 1) / kColRows);
  colsum_partial_kernel<<<dim3(nblk, (cols + 255) / 256), dim3(256), 0, s>>>(part, nwg, cols, cpart);
  colsum_final_kernel<<<dim3((cols + 63) / 64), dim3(256), 0, s>>>(cpart, nblk, cols, both);
  split_pair_kernel<<<dim3((H + 255) / 256), dim3(256), 0, s>>>(both, H, dgamma, dbeta);
  TT_LAUNCH_CHECK("tt_ln_l2_bwd_ex");
  return TT_OK;
}

extern "C" int tt_triplet_fwd(const float* q, const float* p, const float* n, int64_t B, int H, float margin,
                              float* loss_rows, float* loss, tt_stream_t stream) {
  TT_REQUIRE(B >= 0 && H > 0, "bad shape B=%lld H=%d", (long long)B, H);
  TT_REQUIRE(loss, "null loss");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (B > 0) {
    TT_REQUIRE(q && p && n && loss_rows, "null pointer");
    triplet_fwd_kernel<<<rows_grid(B), dim3(kBlock), 0, s>>>(q, p, n, B, H, margin, loss_rows);
    TT_LAUNCH_CHECK("tt_triplet_fwd");
  }
  return launch_mean(loss_rows, B, loss, s);
}

extern "C" int tt_triplet_bwd(const float* q, const float* p, const float* n, int64_t B, int H, float margin,
                              const float* grad_loss, float* dq, float* dp, float* dn, tt_stream_t stream) {
  TT_REQUIRE(B >= 0 && H > 0, "bad shape B=%lld H=%d", (long long)B, H);
  if (B == 0) return TT_OK;
  TT_REQUIRE(q && p && n && grad_loss && dq && dp && dn, "null pointer");
  triplet_bwd_kernel<<<rows_grid(B), dim3(kBlock), 0, reinterpret_cast<hipStream_t>(stream)>>>(q, p, n, B, H, margin,
                                                                                               grad_loss, dq, dp, dn);
  TT_LAUNCH_CHECK("tt_triplet_bwd");
  return TT_OK;
}

extern "C" int tt_multi_neg_fwd(const float* q, const float* p, const float* negs, int64_t B, int N, int H,
                                float inv_tau, float* loss_rows, float* loss, tt_stream_t stream) {
  TT_REQUIRE(B >= 0 && H > 0 && N >= 0 && N <= kMaxNeg, "bad shape B=%lld N=%d H=%d", (long long)B, N, H);
  TT_REQUIRE(loss, "null loss");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (B > 0) {
    TT_REQUIRE(q && p && loss_rows && (N == 0 || negs), "null pointer");
    if (H == 256 && N <= 4 && aligned16(q, p, negs))
      multi_neg_fwd_h256_kernel<4><<<rows_grid(B), dim3(kBlock), 0, s>>>(q, p, negs, B, N, inv_tau, loss_rows);
    else if (H == 256 && N <= 15 && aligned16(q, p, negs))
      multi_neg_fwd_h256_kernel<15><<<rows_grid(B), dim3(kBlock), 0, s>>>(q, p, negs, B, N, inv_tau, loss_rows);
    else
      multi_neg_fwd_kernel<<<rows_grid(B), dim3(kBlock), 0, s>>>(q, p, negs, B, N, H, inv_tau, loss_rows);
    TT_LAUNCH_CHECK("tt_multi_neg_fwd");
  }
  return launch_mean(loss_rows, B, loss, s);
}

extern "C" int tt_multi_neg_bwd_l2(const float* qpn, int64_t B, int N, const float* norms, float inv_tau,
                                   const float* grad_loss, float* dx, tt_stream_t stream) {
  TT_REQUIRE(B >= 0 && N >= 0 && N <= 15, "tt_multi_neg_bwd_l2: bad shape B=%lld N=%d (N <= 15)", (long long)B, N);
  if (B == 0) return TT_OK;
  TT_REQUIRE(qpn && norms && grad_loss && dx, "null pointer");
  constexpr int H = 256;
  const float *q = qpn, *p = qpn + B * H, *negs = qpn + 2 * B * H;
  float *dq = dx, *dp = dx + B * H, *dn = dx + 2 * B * H;
  TT_REQUIRE(aligned16(q, p, negs) && aligned16(dq, dp, dn), "qpn / dx must be 16-byte aligned");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (N <= 4)
    multi_neg_bwd_h256_kernel<4><<<rows_grid(B), dim3(kBlock), 0, s>>>(q, p, negs, B, N, inv_tau, grad_loss, dq, dp, dn,
                                                                       norms);
  else
    multi_neg_bwd_h256_kernel<15><<<rows_grid(B), dim3(kBlock), 0, s>>>(q, p, negs, B, N, inv_tau, grad_loss, dq, dp,
                                                                        dn, norms);
  TT_LAUNCH_CHECK("tt_multi_neg_bwd_l2");
  return TT_OK;
}

extern "C" int tt_multi_neg_bwd(const float* q, const float* p, const float* negs, int64_t B, int N, int H,
                                float inv_tau, const float* grad_loss, float* dq, float* dp, float* dnegs,
                                tt_stream_t stream) {
  TT_REQUIRE(B >= 0 && H > 0 && N >= 0 && N <= kMaxNeg, "bad shape B=%lld N=%d H=%d", (long long)B, N, H);
  if (B == 0) return TT_OK;
  TT_REQUIRE(q && p && grad_loss && dq && dp && (N == 0 || (negs && dnegs)), "null pointer");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (H == 256 && N <= 4 && aligned16(q, p, negs) && aligned16(dq, dp, dnegs))
    multi_neg_bwd_h256_kernel<4><<<rows_grid(B), dim3(kBlock), 0, s>>>(q, p, negs, B, N, inv_tau, grad_loss, dq, dp,
                                                                       dnegs);
  else if (H == 256 && N <= 15 && aligned16(q, p, negs) && aligned16(dq, dp, dnegs))
    multi_neg_bwd_h256_kernel<15><<<rows_grid(B), dim3(kBlock), 0, s>>>(q, p, negs, B, N, inv_tau, grad_loss, dq, dp,
                                                                        dnegs);
  else
    multi_neg_bwd_kernel<<<rows_grid(B), dim3(kBlock), 0, s>>>(q, p, negs, B, N, H, inv_tau, grad_loss, dq, dp,
                                                               dnegs);
  TT_LAUNCH_CHECK("tt_multi_neg_bwd");
  return TT_OK;
}
