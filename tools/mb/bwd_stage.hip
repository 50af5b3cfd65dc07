// Microbenchmark: the stored-P backward engine's stage (score_ddp_kernel<256, 1>) reduced to its
// issue pattern, to price its vector-memory instructions beside the MFMAs.  256 workgroups x 4
// waves (one per SIMD, 128 KiB LDS ring as the engine), per stage and wave: 32
// v_mfma_f32_32x32x16_bf16 whose A operands come from two ds_read_b64_tr_b16 each, one barrier in
// the middle, and by mode
//   0: no vector-memory instruction (the MFMA + LDS floor)
//   1: 8 LDS-DMA fill pieces (global_load_lds_dwordx4, 1 KiB) + 4 global_load_dwordx4 P loads (the engine)
//   2: the fills staged through VGPRs: 8 global_load_dwordx4 + 8 ds_write_b128 one stage later, + 4 P loads
//   3: the 4 P loads only
//   4: the 8 LDS-DMA fill pieces only
// Fill source: a 2 MiB L2-resident buffer (one query split per XCD, as the engine); P: 4 KiB per
// wave per stage streamed from a 256 MiB buffer (the engine's 268 MB P read).  Random bf16 data
// (zero operands raise the clock).  Prints us per launch and s_memtime ticks per stage.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;
typedef __attribute__((address_space(3))) i32x4 lds_i32x4_t;
typedef __attribute__((address_space(3))) char lds_char_t;

constexpr int kStageB = 32768, kQBytes = 2 << 20;

__device__ __forceinline__ void glds(unsigned voff, const void* sbase, unsigned lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(lds)
               : "memory");
}

template <int MODE>
__global__ __launch_bounds__(256, 1) void k(const char* __restrict__ Q, const char* __restrict__ P, int nst,
                                            float* out, long long* ticks) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  lds_char_t* lds = (lds_char_t*)smem;
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const unsigned lbase = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)lds);
  const char* pw = P + (size_t)(blockIdx.x * 4 + wid) * nst * 4096;
  auto qoff = [&](int t) { return (unsigned)(((unsigned)t * 64u * 512u) % kQBytes); };
  f32x16 acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = f32x16{};
  // prologue: stages 0..2 by LDS-DMA in every mode
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int c = 0; c < 8; ++c)
      glds((unsigned)((c * 4 + wid) * 1024 + lane * 16), Q + qoff(t),
           __builtin_amdgcn_readfirstlane(lbase + t * kStageB + (c * 4 + wid) * 1024));
  i32x4 pv[2][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) pv[0][j] = *reinterpret_cast<const i32x4*>(pw + j * 1024 + lane * 16);
  i32x4 sg[2][8];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int c = 0; c < 8; ++c) sg[s][c] = i32x4{};
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // the engine's transposed operand reads (LdsOffs<256>: dual-use swizzle, conflict-free), read
  // four steps ahead across tiles and stages
  auto swz = [](int row) { return ((row & 3) << 2) | ((row >> 2) & 3); };
  const int tg = lane >> 4, ti = lane & 15, tq = ti >> 2, tp = ti & 3;
  const int r0 = 4 * (tg >> 1) + tq, cbase = 2 * (tg & 1) + (tp >> 1), bo = (tp & 1) * 8;
  unsigned a0o[4], a1o[4];
#pragma unroll
  for (int ht = 0; ht < 4; ++ht) {
    a0o[ht] = r0 * 512 + bo + (((4 * ht + cbase) ^ swz(r0)) << 4);
    a1o[ht] = (r0 + 8) * 512 + bo + (((4 * ht + cbase) ^ swz(r0 + 8)) << 4);
  }
  auto opnd = [&](const lds_char_t* tb, int i) {
    const int jt = i / 16, st = i % 16, s2 = st / 8, ht = st % 8;
    const lds_char_t* b = tb + jt * 32 * 512 + s2 * 16 * 512 + (ht >= 4 ? 256 : 0);
    const bf16x4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(b + a0o[ht & 3]));
    const bf16x4 x2 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(b + a1o[ht & 3]));
    return bf16x8{x1[0], x1[1], x1[2], x1[3], x2[0], x2[1], x2[2], x2[3]};
  };
  bf16x8 ring[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) ring[j] = opnd(lds, j);
  long long t0 = __builtin_amdgcn_s_memtime();
  auto stage = [&](int t, auto par) {
    constexpr int p = decltype(par)::value;
    const int buf = t & 3;
    const lds_char_t* tb = lds + buf * kStageB;
    const lds_char_t* ntb = lds + ((buf + 1) & 3) * kStageB;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      if (i == 16) {
        asm volatile("s_waitcnt vmcnt(14)\n\ts_barrier" ::: "memory");
      }
      acc[i & 7] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ring[i & 3], __builtin_bit_cast(bf16x8, pv[p][i >> 3]),
                                                           acc[i & 7], 0, 0, 0);
      ring[i & 3] = i + 4 < 32 ? opnd(tb, i + 4) : opnd(ntb, i + 4 - 32);
      if constexpr (MODE == 1 || MODE == 4) {
        if ((i & 3) == 0) {
          const int c = i >> 2;
          glds((unsigned)((c * 4 + wid) * 1024 + lane * 16), Q + qoff(t + 3),
               __builtin_amdgcn_readfirstlane(lbase + ((t + 3) & 3) * kStageB + (c * 4 + wid) * 1024));
        }
      }
      if constexpr (MODE == 2) {
        if ((i & 3) == 0) {
          const int c = i >> 2;
          sg[p][c] = *reinterpret_cast<const i32x4*>(Q + qoff(t + 3) + (c * 4 + wid) * 1024 + lane * 16);
        }
        if ((i & 3) == 1) {  // the pieces loaded one stage ago (stage t+2's data) into their buffer
          const int c = i >> 2;
          *reinterpret_cast<lds_i32x4_t*>(lds + ((t + 2) & 3) * kStageB + (c * 4 + wid) * 1024 + lane * 16) =
              sg[1 - p][c];
        }
      }
      if constexpr (MODE == 1 || MODE == 2 || MODE == 3) {
        if ((i & 7) == 2) {
          const int j = i >> 3;
          pv[1 - p][j] = *reinterpret_cast<const i32x4*>(pw + (size_t)(t + 1) * 4096 + j * 1024 + lane * 16);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  for (int t = 0; t + 1 < nst; t += 2) {
    stage(t, std::integral_constant<int, 0>{});
    stage(t + 1, std::integral_constant<int, 1>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) s += acc[j][e];
  for (int c = 0; c < 8; ++c) s += (float)sg[0][c][0] + (float)sg[1][c][1];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (blockIdx.x == 0 && threadIdx.x == 0) ticks[0] = t1 - t0;
}

int main(int argc, char** argv) {
  const int nst = argc > 1 ? atoi(argv[1]) : 64;
  char *Q, *P;
  float* out;
  long long* ticks;
  const size_t pbytes = (size_t)256 * 4 * (nst + 2) * 4096;
  hipMalloc(&Q, kQBytes + 65536);
  hipMalloc(&P, pbytes);
  hipMalloc(&out, 256 * 256 * 4);
  hipMalloc(&ticks, 8);
  {  // random bf16 in (-1, 1) for the fills, (0, 1) for P
    std::vector<unsigned short> h(kQBytes / 2 + 32768);
    unsigned x = 12345;
    for (auto& v : h) {
      x = x * 1664525u + 1013904223u;
      v = (unsigned short)(0x3c00 + (x >> 20) % 0x300) | (unsigned short)((x & 0x80000000u) ? 0x8000 : 0);
    }
    hipMemcpy(Q, h.data(), kQBytes + 65536, hipMemcpyHostToDevice);
    std::vector<unsigned short> hp(pbytes / 2);
    for (auto& v : hp) {
      x = x * 1664525u + 1013904223u;
      v = (unsigned short)(0x3a00 + (x >> 20) % 0x500);
    }
    hipMemcpy(P, hp.data(), pbytes, hipMemcpyHostToDevice);
  }
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int L = 4 * kStageB;
  for (int rep = 0; rep < 2; ++rep)
    for (int mode = 0; mode < 5; ++mode) {
      auto launch = [&]() {
        if (mode == 0) k<0><<<256, 256, L>>>(Q, P, nst, out, ticks);
        if (mode == 1) k<1><<<256, 256, L>>>(Q, P, nst, out, ticks);
        if (mode == 2) k<2><<<256, 256, L>>>(Q, P, nst, out, ticks);
        if (mode == 3) k<3><<<256, 256, L>>>(Q, P, nst, out, ticks);
        if (mode == 4) k<4><<<256, 256, L>>>(Q, P, nst, out, ticks);
      };
      for (int w = 0; w < 3; ++w) launch();
      hipDeviceSynchronize();
      const int iters = 20;
      hipEventRecord(a);
      for (int it = 0; it < iters; ++it) launch();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      long long t;
      hipMemcpy(&t, ticks, 8, hipMemcpyDeviceToHost);
      printf("rep %d mode %d: %.1f us per launch, %.0f ticks per stage (block 0)\n", rep, mode, ms * 1e3 / iters,
             (double)t / nst);
    }
  return 0;
}
