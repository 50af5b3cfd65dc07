// Microbenchmark: cycles per v_mfma_f32_32x32x16_bf16 at one wave per SIMD (256 CUs x 4 waves),
// (a) one dependent accumulator chain, (b) eight independent accumulators, (c) chain where the
// B operand is re-packed by VALU (cvt) every step.  Prints us and cycles/MFMA (s_memtime ticks).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int MODE>
__global__ __launch_bounds__(256, 1) void k(float* out, int iters, long long* ticks) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(threadIdx.x * 0.001f + i); b[i] = (__bf16)(i * 0.5f); }
  f32x16 acc[8];
  for (int t = 0; t < 8; ++t) acc[t] = f32x16{};
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (MODE == 0) acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[0], 0, 0, 0);
      if (MODE == 1) acc[s & 7] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[s & 7], 0, 0, 0);
      if (MODE == 2) {
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[0], 0, 0, 0);
        b[s & 7] = (__bf16)((float)b[s & 7] * 1.0001f);
      }
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float sum = 0;
  for (int t = 0; t < 8; ++t) for (int i = 0; i < 16; ++i) sum += acc[t][i];
  out[blockIdx.x * 256 + threadIdx.x] = sum;
  if (threadIdx.x == 0 && blockIdx.x == 0) *ticks = t1 - t0;
}

int main() {
  float* out; long long* ticks; hipMalloc(&out, 256 * 256 * 4); hipMalloc(&ticks, 8);
  const int iters = 2000;
  for (int mode = 0; mode < 3; ++mode) {
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      if (mode == 0) k<0><<<256, 256>>>(out, iters, ticks);
      if (mode == 1) k<1><<<256, 256>>>(out, iters, ticks);
      if (mode == 2) k<2><<<256, 256>>>(out, iters, ticks);
      hipEventRecord(e1); hipEventSynchronize(e1);
    }
    float ms; hipEventElapsedTime(&ms, e0, e1);
    long long t; hipMemcpy(&t, ticks, 8, hipMemcpyDeviceToHost);
    const double n = 16.0 * iters;
    printf("mode %d: %.1f us, %.1f us per 1000 MFMA/SIMD, memtime ticks/MFMA %.2f\n", mode, ms * 1e3, ms * 1e3 / n * 1000, t / n);
  }
  return 0;
}
