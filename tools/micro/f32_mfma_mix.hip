// Micro-benchmark: v_mfma_f32_16x16x4_f32 issue cost per MFMA (cycles per wave, s_memtime) in the operand
// patterns of the f32 slice attention (attention_slice.hip), one workgroup of W waves per CU:
//   regs     4 independent accumulators, operands in registers
//   chain2   2 interleaved accumulators
//   chain1   1 accumulator (dependent chain)
//   ldsb32   4 accumulators, A operand from ds_read_b32 issued 16 MFMAs ahead
//   valu2    4 accumulators + 2 independent v_fma_f32 per MFMA
//   valu6    4 accumulators + 6 independent v_fma_f32 per MFMA
//   exp1     4 accumulators + 1 v_exp_f32 per MFMA
//   ldsb128  4 accumulators, A operand from ds_read_b128 (4 values for 4 MFMAs)
// and the same for v_mfma_f32_16x16x32_bf16 (bf16*): regs, valu2, valu4, ldsb128 (one read per MFMA)
// Build: hipcc -O3 --offload-arch=gfx950 tools/micro/f32_mfma_mix.hip -o tools/micro/f32_mfma_mix
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mf(float a, float b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

template <int MODE>
__global__ __launch_bounds__(512) void kern(float* out, int iters, long long* cyc) {
  __shared__ float lds[4096];
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) lds[i] = 1e-3f * i;
  __syncthreads();
  f32x4 acc[4];
  for (int a = 0; a < 4; ++a) acc[a] = f32x4{0.f, 0.f, 0.f, 0.f};
  float x[16], y = 1.0f + threadIdx.x * 1e-4f;
  for (int k = 0; k < 16; ++k) x[k] = (threadIdx.x + k) * 1e-3f;
  float v[6] = {1.f, 2.f, 3.f, 4.f, 5.f, 6.f};
  const int lb = (threadIdx.x & 63) * 4;
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    if constexpr (MODE == 7) {
      f32x4 a[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) a[k] = *reinterpret_cast<volatile f32x4*>(&lds[(lb + 68 * k + 4 * i) & 4092]);
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[k & 3] = mf(a[k >> 2][k & 3], y, acc[k & 3]);
    } else if constexpr (MODE >= 10) {
      u32x4 bx = {threadIdx.x, threadIdx.x * 3u, threadIdx.x * 5u, threadIdx.x * 7u};
      u32x4 a[16];
      if constexpr (MODE == 13) {
#pragma unroll
        for (int k = 0; k < 16; ++k) a[k] = *reinterpret_cast<volatile u32x4*>(&lds[(lb + 68 * k + 4 * i) & 4092]);
      } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) a[k] = u32x4{(unsigned)k, (unsigned)i, 1u, 2u} + bx;
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        acc[k & 3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a[k]), __builtin_bit_cast(bf16x8, bx),
                                                             acc[k & 3], 0, 0, 0);
        if constexpr (MODE == 11 || MODE == 12) {
          v[0] = fmaf(v[0], 1.0001f, 0.5f);
          v[1] = fmaf(v[1], 1.0001f, 0.5f);
        }
        if constexpr (MODE == 12) {
          v[2] = fmaf(v[2], 1.0001f, 0.5f);
          v[3] = fmaf(v[3], 1.0001f, 0.5f);
        }
      }
    } else if constexpr (MODE == 3) {
      float a[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) a[k] = *reinterpret_cast<volatile float*>(&lds[(lb + 17 * k + i) & 4095]);
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[k & 3] = mf(a[k], y, acc[k & 3]);
    } else {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if constexpr (MODE == 0 || MODE == 4 || MODE == 5 || MODE == 6) acc[k & 3] = mf(x[k], y, acc[k & 3]);
        if constexpr (MODE == 1) acc[k & 1] = mf(x[k], y, acc[k & 1]);
        if constexpr (MODE == 2) acc[0] = mf(x[k], y, acc[0]);
        if constexpr (MODE == 4) {
          v[0] = fmaf(v[0], 1.0001f, 0.5f);
          v[1] = fmaf(v[1], 1.0001f, 0.5f);
        }
        if constexpr (MODE == 5) {
#pragma unroll
          for (int q = 0; q < 6; ++q) v[q] = fmaf(v[q], 1.0001f, 0.5f);
        }
        if constexpr (MODE == 6) v[k % 6] = __builtin_amdgcn_exp2f(v[k % 6]);
      }
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = v[0] + v[1] + v[2] + v[3] + v[4] + v[5];
  for (int a = 0; a < 4; ++a)
    for (int r = 0; r < 4; ++r) s += acc[a][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int MODE>
void run(const char* name, int waves) {
  const int blocks = 256, iters = 2000;
  float* out; long long* cyc;
  hipMalloc(&out, blocks * 512 * sizeof(float));
  hipMalloc(&cyc, blocks * 8 * sizeof(long long));
  hipMemset(cyc, 0, blocks * 8 * sizeof(long long));
  hipLaunchKernelGGL(kern<MODE>, dim3(blocks), dim3(64 * waves), 0, 0, out, iters, cyc);
  hipLaunchKernelGGL(kern<MODE>, dim3(blocks), dim3(64 * waves), 0, 0, out, iters, cyc);
  hipDeviceSynchronize();
  std::vector<long long> h(blocks * 8);
  hipMemcpy(h.data(), cyc, h.size() * sizeof(long long), hipMemcpyDeviceToHost);
  std::vector<double> c;
  for (int b = 0; b < blocks; ++b)
    for (int w = 0; w < waves; ++w) c.push_back((double)h[b * 8 + w]);
  std::sort(c.begin(), c.end());
  // s_memtime ticks at the shader clock; per wave: 16 MFMAs per iteration
  printf("%-8s waves/CU %d: %.1f cycles per MFMA per wave (median), %.1f per SIMD\n", name, waves,
         c[c.size() / 2] / (16.0 * iters), c[c.size() / 2] / (16.0 * iters) / (waves / 4.0 < 1 ? 1 : waves / 4.0));
  hipFree(out); hipFree(cyc);
}

int main() {
  for (int w : {4, 8}) {
    run<0>("regs", w);
    run<1>("chain2", w);
    run<2>("chain1", w);
    run<3>("ldsb32", w);
    run<4>("valu2", w);
    run<5>("valu6", w);
    run<6>("exp1", w);
    run<7>("ldsb128", w);
    run<10>("bf16regs", w);
    run<11>("bf16valu2", w);
    run<12>("bf16valu4", w);
    run<13>("bf16lds", w);
  }
  return 0;
}
