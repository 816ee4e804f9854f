// Micro-benchmark: v_mfma_f32_32x32x2_f32 throughput for one dependent accumulator chain vs 2 / 4
// independent chains, one wave per SIMD and 4 waves per SIMD (cycles from s_memtime).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ void chain(float* out, int iters, long long* cyc) {
  f32x16 acc[NACC];
  for (int a = 0; a < NACC; ++a)
    for (int r = 0; r < 16; ++r) acc[a][r] = 0.f;
  float x = threadIdx.x * 1e-3f, y = 1.0f + threadIdx.x * 1e-4f;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 16 / NACC; ++k)
#pragma unroll
      for (int a = 0; a < NACC; ++a) acc[a] = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, acc[a], 0, 0, 0);
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int a = 0; a < NACC; ++a)
    for (int r = 0; r < 16; ++r) s += acc[a][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NACC>
void run(int waves_per_block, const char* name) {
  const int iters = 2000, nblk = 1024;   // 1024 blocks: one or more waves per SIMD
  float* out; long long* cyc;
  hipMalloc(&out, nblk * 64 * waves_per_block * 4);
  hipMalloc(&cyc, nblk * 8);
  hipLaunchKernelGGL(chain<NACC>, dim3(nblk), dim3(64 * waves_per_block), 0, 0, out, iters, cyc);
  hipDeviceSynchronize();
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(chain<NACC>, dim3(nblk), dim3(64 * waves_per_block), 0, 0, out, iters, cyc);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 32 * 32 * 2 * 16.0 * iters * nblk * waves_per_block;
  printf("%-28s waves/block %d: %8.3f ms  %7.1f TF/s\n", name, waves_per_block, ms, flops / ms / 1e9);
  hipFree(out); hipFree(cyc);
}

int main() {
  for (int w : {1, 4, 8, 16}) {
    run<1>(w, "1 accumulator (dependent)");
    run<2>(w, "2 accumulators");
    run<4>(w, "4 accumulators");
  }
  return 0;
}
