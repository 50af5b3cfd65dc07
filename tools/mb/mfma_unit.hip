// Microbenchmark: cycles per v_mfma_f32_32x32x16_bf16 (one wave per SIMD, 256 CUs x 4 waves) for the
// forward scorer unit's MFMA pattern alone: a 16-MFMA dependent chain into one accumulator (S chain)
// followed by 16 MFMAs over 8 accumulators (Acc chain), repeated.  Modes: 0 both through the
// builtin; 1 S chain by inline asm into VGPRs, Acc chain builtin (the engine's form); 2 = 1 plus a
// VALU read of the S result each unit (dynamic index); 3 pure 8-accumulator builtin stream; 4 one
// static read of the S result per unit; 5 one add reading an S-result element per Acc step (the
// map's pattern); 6 = 5 reading a register no MFMA wrote; 7 = 5 as a dependent fma chain.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void mv0(f32x16& d, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(d) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mv(f32x16& d, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(d) : "v"(a), "v"(b));
}

template <int MODE>
__global__ __launch_bounds__(256, 1) void k(float* out, int iters, long long* ticks) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(threadIdx.x * 0.001f + i); b[i] = (__bf16)(i * 0.5f - 1.f); }
  asm volatile("s_nop 4" : "+v"(a), "+v"(b));
  f32x16 acc[8];
  for (int t = 0; t < 8; ++t) acc[t] = f32x16{};
  f32x16 x = f32x16{}, y;
  for (int i = 0; i < 16; ++i) y[i] = threadIdx.x * 0.01f + i;
  asm volatile("" : "+v"(y));
  float s = 0.f;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if (MODE == 3) {
#pragma unroll
      for (int st = 0; st < 32; ++st) acc[st & 7] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[st & 7], 0, 0, 0);
      continue;
    }
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      if (MODE == 0) x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, kk ? x : f32x16{}, 0, 0, 0);
      else if (kk == 0) mv0(x, a, b);
      else mv(x, a, b);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      acc[st & 7] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[st & 7], 0, 0, 0);
      if (MODE == 2 && st == 15) s += x[threadIdx.x & 15];
      if (MODE == 4 && st == 15) s += x[0];
      if (MODE == 5) s += x[st];
      if (MODE == 6) s += y[st];
      if (MODE == 7) s = __builtin_fmaf(x[st], 1.0001f, s);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float sum = s;
  for (int t = 0; t < 8; ++t) for (int i = 0; i < 16; ++i) sum += acc[t][i] + x[i];
  out[blockIdx.x * 256 + threadIdx.x] = sum;
  if (threadIdx.x == 0 && blockIdx.x == 0) *ticks = t1 - t0;
}

int main() {
  float* out; long long* ticks; hipMalloc(&out, 256 * 256 * 4); hipMalloc(&ticks, 8);
  const int iters = 2000;
  for (int mode = 0; mode < 8; ++mode) {
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      if (mode == 0) k<0><<<256, 256>>>(out, iters, ticks);
      if (mode == 1) k<1><<<256, 256>>>(out, iters, ticks);
      if (mode == 2) k<2><<<256, 256>>>(out, iters, ticks);
      if (mode == 3) k<3><<<256, 256>>>(out, iters, ticks);
      if (mode == 4) k<4><<<256, 256>>>(out, iters, ticks);
      if (mode == 5) k<5><<<256, 256>>>(out, iters, ticks);
      if (mode == 6) k<6><<<256, 256>>>(out, iters, ticks);
      if (mode == 7) k<7><<<256, 256>>>(out, iters, ticks);
      hipEventRecord(e1); hipEventSynchronize(e1);
    }
    float ms; hipEventElapsedTime(&ms, e0, e1);
    long long t; hipMemcpy(&t, ticks, 8, hipMemcpyDeviceToHost);
    const double n = 32.0 * iters;
    printf("mode %d: %.1f us, memtime ticks/MFMA %.2f\n", mode, ms * 1e3, t / n);
  }
  return 0;
}
