// Microbenchmark: HBM rate of the table update's access pattern, in-place read-modify-write of
// three V x E fp32 arrays (p, m, v as in the fused bag backward + AdamW), against a plain copy.
// Variants (all 256-thread blocks, float4 per lane):
//   copy      : dst = src (one read + one write stream)
//   rmw1      : one wave per 1 KiB row, p/m/v loaded, combined, stored in place (the fused kernel's shape)
//   rmwK<K>   : one wave per K consecutive rows, all 3K loads issued before the stores
//   rmwnt     : rmw1 with non-temporal stores
//   rmwpers   : persistent grid (2048 blocks), each wave strides over rows with the next row's
//               loads issued before the current row's stores
//   il<K>     : the three arrays interleaved by row ([p_r | m_r | v_r], 3 KiB per row, one
//               buffer): one wave per K rows, one contiguous read and write stream
//   ilsl4     : il with the XCD-sliced placement of the fused kernel (4 column slices)
// Prints us and GB/s (bytes = 24 per element for the RMW variants, 8 for copy).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int E4 = 64;  // float4 per 1 KiB row (E = 256)

__device__ __forceinline__ void upd(f32x4& p, f32x4& m, f32x4& v) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    m[j] = 0.9f * m[j] + 0.1f * p[j];
    v[j] = 0.999f * v[j] + 0.001f * p[j] * p[j];
    p[j] = p[j] * 0.99999f - 1e-3f * m[j] / (sqrtf(v[j]) + 1e-8f);
  }
}

__global__ __launch_bounds__(256) void copy_k(const f32x4* __restrict__ s, f32x4* __restrict__ d, long n4) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n4) d[i] = s[i];
}

template <int K, bool NT>
__global__ __launch_bounds__(256) void rmw_k(f32x4* __restrict__ p, f32x4* __restrict__ m, f32x4* __restrict__ v,
                                             long rows) {
  const long w = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const long r0 = w * K;
  if (r0 >= rows) return;
  f32x4 a[K], b[K], c[K];
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (r0 + k < rows) {
      const long i = (r0 + k) * E4 + lane;
      a[k] = p[i];
      b[k] = m[i];
      c[k] = v[i];
    }
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (r0 + k < rows) {
      const long i = (r0 + k) * E4 + lane;
      upd(a[k], b[k], c[k]);
      if constexpr (NT) {
        __builtin_nontemporal_store(a[k], p + i);
        __builtin_nontemporal_store(b[k], m + i);
        __builtin_nontemporal_store(c[k], v + i);
      } else {
        p[i] = a[k];
        m[i] = b[k];
        v[i] = c[k];
      }
    }
}

__global__ __launch_bounds__(256) void rmw_pers_k(f32x4* __restrict__ p, f32x4* __restrict__ m,
                                                  f32x4* __restrict__ v, long rows) {
  const long nw = (long)gridDim.x * 4;
  long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  f32x4 a = p[r * E4 + lane], b = m[r * E4 + lane], c = v[r * E4 + lane];
  for (; r < rows; r += nw) {
    const long rn = r + nw;
    f32x4 an, bn, cn;
    if (rn < rows) {
      an = p[rn * E4 + lane];
      bn = m[rn * E4 + lane];
      cn = v[rn * E4 + lane];
    }
    upd(a, b, c);
    p[r * E4 + lane] = a;
    m[r * E4 + lane] = b;
    v[r * E4 + lane] = c;
    a = an;
    b = bn;
    c = cn;
  }
}


// XCD-sliced: blocks with equal blockIdx % 8 own column slice (blockIdx % 8) % S of every row
// (1 KiB / S contiguous bytes per row), rows dealt in blocks of 4 waves x RPW rows.
template <int S>
__global__ __launch_bounds__(256) void rmw_sliced_k(f32x4* __restrict__ p, f32x4* __restrict__ m,
                                                    f32x4* __restrict__ v, long rows) {
  constexpr int LPR = E4 / S, RPW = 64 / LPR;
  const int xg = blockIdx.x & 7, gps = 8 / S, slice = xg % S;
  const long rb = (long)(blockIdx.x >> 3) * gps + xg / S;
  const int lane = threadIdx.x & 63;
  const long r = (rb * 4 + (threadIdx.x >> 6)) * RPW + lane / LPR;
  if (r >= rows) return;
  const long i = r * E4 + slice * LPR + lane % LPR;
  f32x4 a = p[i], b = m[i], c = v[i];
  upd(a, b, c);
  p[i] = a;
  m[i] = b;
  v[i] = c;
}

template <int K>
__global__ __launch_bounds__(256) void rmw_il_k(f32x4* __restrict__ t, long rows) {
  const long w = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const long r0 = w * K;
  if (r0 >= rows) return;
  f32x4 a[K], b[K], c[K];
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (r0 + k < rows) {
      const long i = (r0 + k) * 3 * E4 + lane;
      a[k] = t[i];
      b[k] = t[i + E4];
      c[k] = t[i + 2 * E4];
    }
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (r0 + k < rows) {
      const long i = (r0 + k) * 3 * E4 + lane;
      upd(a[k], b[k], c[k]);
      t[i] = a[k];
      t[i + E4] = b[k];
      t[i + 2 * E4] = c[k];
    }
}

template <int S>
__global__ __launch_bounds__(256) void rmw_il_sliced_k(f32x4* __restrict__ t, long rows) {
  constexpr int LPR = E4 / S, RPW = 64 / LPR;
  const int xg = blockIdx.x & 7, gps = 8 / S, slice = xg % S;
  const long rb = (long)(blockIdx.x >> 3) * gps + xg / S;
  const int lane = threadIdx.x & 63;
  const long r = (rb * 4 + (threadIdx.x >> 6)) * RPW + lane / LPR;
  if (r >= rows) return;
  const long i = r * 3 * E4 + slice * LPR + lane % LPR;
  f32x4 a = t[i], b = t[i + E4], c = t[i + 2 * E4];
  upd(a, b, c);
  t[i] = a;
  t[i + E4] = b;
  t[i + 2 * E4] = c;
}

int main() {
  const long rows = 200000, n4 = rows * E4;
  f32x4 *p, *m, *v, *d;
  hipMalloc(&p, n4 * 16);
  hipMalloc(&m, n4 * 16);
  hipMalloc(&v, n4 * 16);
  hipMalloc(&d, n4 * 16);
  hipMemset(p, 0, n4 * 16);
  hipMemset(m, 0, n4 * 16);
  hipMemset(v, 0, n4 * 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char* name, double bytes, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    const int it = 20;
    for (int i = 0; i < it; ++i) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / it;
    printf("%-10s %8.1f us  %7.0f GB/s\n", name, us, bytes / us / 1e3);
  };
  const double rmw_bytes = 24.0 * rows * 256, copy_bytes = 8.0 * rows * 256;
  run("copy", copy_bytes, [&] { copy_k<<<(unsigned)((n4 + 255) / 256), 256>>>(p, d, n4); });
  run("rmw1", rmw_bytes, [&] { rmw_k<1, false><<<(unsigned)((rows + 3) / 4), 256>>>(p, m, v, rows); });
  run("rmwK2", rmw_bytes, [&] { rmw_k<2, false><<<(unsigned)((rows / 2 + 3) / 4), 256>>>(p, m, v, rows); });
  run("rmwK4", rmw_bytes, [&] { rmw_k<4, false><<<(unsigned)((rows / 4 + 3) / 4), 256>>>(p, m, v, rows); });
  run("rmwnt", rmw_bytes, [&] { rmw_k<1, true><<<(unsigned)((rows + 3) / 4), 256>>>(p, m, v, rows); });
  run("rmwK4nt", rmw_bytes, [&] { rmw_k<4, true><<<(unsigned)((rows / 4 + 3) / 4), 256>>>(p, m, v, rows); });
  run("rmwpers", rmw_bytes, [&] { rmw_pers_k<<<2048, 256>>>(p, m, v, rows); });
  run("rmwpers4k", rmw_bytes, [&] { rmw_pers_k<<<4096, 256>>>(p, m, v, rows); });
  auto sl = [&](auto kern, int S) {
    const long rpb = 4L * (64 / (E4 / S)), rbs = (rows + rpb - 1) / rpb, gps = 8 / S;
    return dim3((unsigned)(((rbs + gps - 1) / gps) * 8));
  };
  run("sliced2", rmw_bytes, [&] { rmw_sliced_k<2><<<sl(0, 2), 256>>>(p, m, v, rows); });
  run("sliced4", rmw_bytes, [&] { rmw_sliced_k<4><<<sl(0, 4), 256>>>(p, m, v, rows); });
  run("sliced8", rmw_bytes, [&] { rmw_sliced_k<8><<<sl(0, 8), 256>>>(p, m, v, rows); });
  f32x4* t;
  hipMalloc(&t, 3 * n4 * 16);
  hipMemset(t, 0, 3 * n4 * 16);
  run("il1", rmw_bytes, [&] { rmw_il_k<1><<<(unsigned)((rows + 3) / 4), 256>>>(t, rows); });
  run("il2", rmw_bytes, [&] { rmw_il_k<2><<<(unsigned)((rows / 2 + 3) / 4), 256>>>(t, rows); });
  run("ilsl4", rmw_bytes, [&] { rmw_il_sliced_k<4><<<sl(0, 4), 256>>>(t, rows); });
  run("ilsl2", rmw_bytes, [&] { rmw_il_sliced_k<2><<<sl(0, 2), 256>>>(t, rows); });
  run("rmwK4", rmw_bytes, [&] { rmw_k<4, false><<<(unsigned)((rows / 4 + 3) / 4), 256>>>(p, m, v, rows); });
  run("copy", copy_bytes, [&] { copy_k<<<(unsigned)((n4 + 255) / 256), 256>>>(p, d, n4); });
  return 0;
}
