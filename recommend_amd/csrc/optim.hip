// Dense optimizer step: per-variable tf.clip_by_norm (train.py:134-135) followed by Keras-2.12
// RMSprop with momentum (train.py:64-70, 138; config.py:39-48, momentum 0.99999):
//   v = rho v + (1-rho) g^2 ; inc = lr g rsqrt(v + eps) ; m = mom m + inc ; w -= m
// Variables are 2-D strided segments {offset, rows, cols, row_stride} of ONE flat parameter /
// gradient / state buffer (a Keras variable such as Wq_dedicated[3] is a column slice of the fused
// [G, d, 3d] QKV bank).  Three launches, no host sync, deterministic (fixed-order partial sums).
#include "common.h"

namespace ot {

constexpr int OPT_CHUNK = 4096;   // elements per block

__device__ __forceinline__ int64_t seg_addr(const int64_t* sg, int64_t e) {
  const int64_t cols = sg[2];
  return sg[0] + (e / cols) * sg[3] + (e % cols);
}

__global__ __launch_bounds__(256) void seg_sumsq_kernel(const float* __restrict__ g, const int64_t* __restrict__ segs,
                                                        int nchunk, float* part) {
  __shared__ float red[4];
  const int seg = blockIdx.y, ch = blockIdx.x;
  const int64_t* sg = segs + 4 * seg;
  const int64_t n = sg[1] * sg[2];
  const int64_t e0 = (int64_t)ch * OPT_CHUNK;
  float s = 0.f;
  for (int64_t e = e0 + threadIdx.x; e < n && e < e0 + OPT_CHUNK; e += 256) {
    const float v = g[seg_addr(sg, e)];
    s += v * v;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[(int64_t)seg * nchunk + ch] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void seg_scale_kernel(const float* __restrict__ part, const int64_t* __restrict__ segs, int nseg, int nchunk,
                                 float clip, float* scale) {
  const int seg = blockIdx.x * blockDim.x + threadIdx.x;
  if (seg >= nseg) return;
  const int64_t n = segs[4 * seg + 1] * segs[4 * seg + 2];
  const int used = (int)((n + OPT_CHUNK - 1) / OPT_CHUNK);
  float s = 0.f;
  for (int c = 0; c < used; ++c) s += part[(int64_t)seg * nchunk + c];
  const float l2 = sqrtf(s);
  scale[seg] = clip > 0.f ? clip / fmaxf(l2, clip) : 1.f;
}

__global__ __launch_bounds__(256) void rmsprop_kernel(float* w, const float* __restrict__ g, float* v, float* m,
                                                      const int64_t* __restrict__ segs, const float* __restrict__ scale,
                                                      float lr, float rho, float eps, float mom) {
  const int seg = blockIdx.y, ch = blockIdx.x;
  const int64_t* sg = segs + 4 * seg;
  const int64_t n = sg[1] * sg[2];
  const int64_t e0 = (int64_t)ch * OPT_CHUNK;
  const float sc = scale[seg];
  for (int64_t e = e0 + threadIdx.x; e < n && e < e0 + OPT_CHUNK; e += 256) {
    const int64_t a = seg_addr(sg, e);
    const float gg = g[a] * sc;
    const float vv = rho * v[a] + (1.f - rho) * gg * gg;
    const float inc = lr * gg * rsqrtf(vv + eps);
    v[a] = vv;
    if (mom > 0.f) {
      const float mm = mom * m[a] + inc;
      m[a] = mm;
      w[a] -= mm;
    } else {
      w[a] -= inc;
    }
  }
}

inline int nchunks_for(int64_t max_seg_elems) { return (int)((max_seg_elems + OPT_CHUNK - 1) / OPT_CHUNK); }

}  // namespace ot

using namespace ot;

extern "C" size_t ot_clip_rmsprop_workspace_size(int nseg, int64_t max_seg_elems) {
  return ((size_t)nseg * nchunks_for(max_seg_elems) + nseg) * sizeof(float);
}

extern "C" int ot_clip_rmsprop(float* w, float* g, float* v, float* m, const int64_t* segs_dev, int nseg,
                               int64_t max_seg_elems, float lr, float rho, float eps, float momentum, float clip,
                               void* workspace, size_t ws_bytes, void* stream) {
  OT_REQUIRE(w && g && v && m && segs_dev && workspace, "ot_clip_rmsprop: null operand");
  OT_REQUIRE(ws_bytes >= ot_clip_rmsprop_workspace_size(nseg, max_seg_elems), "ot_clip_rmsprop: workspace too small");
  if (nseg == 0) return OT_OK;
  const int nch = nchunks_for(max_seg_elems);
  float* part = (float*)workspace;
  float* scale = part + (size_t)nseg * nch;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(seg_sumsq_kernel, dim3(nch, nseg), dim3(256), 0, s, g, segs_dev, nch, part);
  OT_LAUNCH_CHECK("ot_clip_rmsprop(sumsq)");
  hipLaunchKernelGGL(seg_scale_kernel, dim3(ceil_div(nseg, 256)), dim3(256), 0, s, part, segs_dev, nseg, nch, clip,
                     scale);
  OT_LAUNCH_CHECK("ot_clip_rmsprop(scale)");
  hipLaunchKernelGGL(rmsprop_kernel, dim3(nch, nseg), dim3(256), 0, s, w, g, v, m, segs_dev, scale, lr, rho, eps,
                     momentum);
  OT_LAUNCH_CHECK("ot_clip_rmsprop(apply)");
  return OT_OK;
}
