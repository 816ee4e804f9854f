// Tokenizer glue, task heads and the Keras BCE loss.
//   ot_ns_assemble   model.py:239-254 (NS concat in user+item+context order) + id -> row gather
//   ot_ns_grad_pack  gradient rows of the gathered NS embeddings (for ot_sparse_adagrad)
//   ot_fill_rows     [SEP] rows model.py:270-272
//   ot_seq_rows      item-id row maps of the sequence projection GEMM (embedding gather fused
//                    into the GEMM's A-row load)
//   ot_head_fwd/bwd  task heads model.py:325-330, 388-391 (second Dense(1, sigmoid) + sigmoid)
//   ot_bce_fwd/bwd   tf.keras.losses.BinaryCrossentropy(from_logits=False) train.py:84-87,124-128
//   ot_task_loss_*   per-task BCE ('ctr'/'cvr') or MeanSquaredError (other tasks) train.py:78-93
#include "common.h"

namespace ot {

__global__ void ns_assemble_kernel(const ot_ns_field* __restrict__ f, const float* __restrict__ table, int B,
                                   float* out, int64_t ld) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const ot_ns_field fd = f[blockIdx.y];
  float* dst = out + (int64_t)b * ld + fd.col;
  if (fd.ids) {
    const int64_t row = fd.row_offset + fd.ids[(int64_t)b * fd.stride];
    const float* src = table + row * fd.width;
    for (int c = 0; c < fd.width; ++c) dst[c] = src[c];
  } else {
    dst[0] = fd.dense[(int64_t)b * fd.stride];
  }
}

__global__ void ns_grad_pack_kernel(const ot_ns_field* __restrict__ f, int width, const float* __restrict__ dmat,
                                    int64_t ld, int B, int64_t* keys, float* grads) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const ot_ns_field fd = f[blockIdx.y];
  const int64_t e = (int64_t)blockIdx.y * B + b;
  keys[e] = fd.row_offset + fd.ids[(int64_t)b * fd.stride];
  const float* src = dmat + (int64_t)b * ld + fd.col;
  for (int c = 0; c < width; ++c) grads[e * width + c] = src[c];
}

__global__ void fill_rows_kernel(float* dst, int64_t ld, const int32_t* __restrict__ rows, int64_t nrows,
                                 const float* __restrict__ vec, int d) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nrows * d) return;
  const int64_t r = i / d;
  const int c = (int)(i % d);
  dst[(int64_t)rows[r] * ld + c] = vec[c];
}

__global__ void seq_rows_kernel(const int64_t* __restrict__ ids, int64_t stride_b, int B, int L, int64_t vocab,
                                int32_t* in_rows) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= (int64_t)B * L) return;
  const int64_t b = m / L, p = m % L;
  const int64_t id = ids[b * stride_b + p];
  in_rows[m] = (id >= 0 && id < vocab) ? (int32_t)id : -1;   // out-of-range id -> zero row
}

__global__ __launch_bounds__(256) void head_fwd_kernel(const float* __restrict__ pre1, const float* __restrict__ w2,
                                                       const float* __restrict__ b2, int T, int B, int dh,
                                                       float* logits, float* probs) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= T * B) return;
  const int t = row / B;
  float s = 0.f;
  for (int j = lane; j < dh; j += 64) s += gelu_erf(pre1[(int64_t)row * dh + j]) * w2[t * dh + j];
  s = wave_sum(s);
  if (lane == 0) {
    const float z = s + b2[t];
    logits[row] = z;
    probs[row] = 1.f / (1.f + expf(-z));
  }
}

// grid (NB, T): block (x, t) handles samples b = 4x + wave + k*4NB of task t; partial sums of
// dw2 (dh values) and db2 (1 value) per block -> part[t][x][dh + 1]
__global__ __launch_bounds__(256) void head_bwd_kernel(const float* __restrict__ pre1, const float* __restrict__ w2,
                                                       const float* __restrict__ probs,
                                                       const float* __restrict__ dprobs,
                                                       const float* __restrict__ dlogits, int B, int dh,
                                                       float* dpre1, float* part) {
  extern __shared__ __attribute__((aligned(16))) float red[];   // [4][dh + 1]
  const int t = blockIdx.y, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int NB = gridDim.x;
  float pw[4] = {0.f, 0.f, 0.f, 0.f};
  float pb = 0.f;
  for (int b = blockIdx.x * 4 + wave; b < B; b += NB * 4) {
    const int64_t row = (int64_t)t * B + b;
    const float pr = probs[row];
    const float dz = (dprobs ? dprobs[row] * pr * (1.f - pr) : 0.f) + (dlogits ? dlogits[row] : 0.f);
    pb += dz;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = lane + 64 * q;
      if (j < dh) {
        const float u = pre1[row * dh + j];
        pw[q] += gelu_erf(u) * dz;
        dpre1[row * dh + j] = dz * w2[t * dh + j] * gelu_erf_grad(u);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int j = lane + 64 * q;
    if (j < dh) red[wave * (dh + 1) + j] = pw[q];
  }
  if (lane == 0) red[wave * (dh + 1) + dh] = pb;
  __syncthreads();
  for (int j = threadIdx.x; j <= dh; j += 256) {
    float s = 0.f;
    for (int w = 0; w < 4; ++w) s += red[w * (dh + 1) + j];
    part[((int64_t)t * NB + blockIdx.x) * (dh + 1) + j] = s;
  }
}

__global__ void head_bwd_reduce_kernel(const float* __restrict__ part, int NB, int dh, float* dw2, float* db2,
                                       int64_t sw2, int64_t sb2, int accumulate) {
  const int t = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j > dh) return;
  float s = 0.f;
  for (int x = 0; x < NB; ++x) s += part[((int64_t)t * NB + x) * (dh + 1) + j];
  float* dst = j < dh ? dw2 + t * sw2 + j : db2 + t * sb2;
  *dst = accumulate ? *dst + s : s;
}

// Keras 2.12 on a sigmoid head (model.py:327-329): activations.sigmoid caches its input as the output's
// _keras_logits and backend.binary_crossentropy then returns tf.nn.sigmoid_cross_entropy_with_logits —
// max(z, 0) - z y + log(1 + exp(-|z|)), no clipping; d/dz = sigmoid(z) - y
__device__ __forceinline__ float bce_logits(float y, float z) { return fmaxf(z, 0.f) - z * y + log1pf(expf(-fabsf(z))); }

__device__ __forceinline__ float keras_bce(float y, float p) {
  const float eps = 1e-7f;
  const float pc = fminf(fmaxf(p, eps), 1.f - eps);
  return -(y * logf(pc + eps) + (1.f - y) * logf(1.f - pc + eps));
}

// Keras MeanSquaredError on one [B,1] prediction (train.py:88-91): (y - p)^2
__device__ __forceinline__ float task_loss(float y, float p, bool mse) {
  if (mse) { const float e = p - y; return e * e; }
  return keras_bce(y, p);
}

// part[blk] = sum over this block's elements of loss / B (elements = T*B, task-major; task t uses MSE
// when bit t of mse_mask is set, BCE otherwise)
__global__ __launch_bounds__(256) void bce_fwd_kernel(const float* __restrict__ probs, const float* __restrict__ labels,
                                                      int64_t n, int B, float invB, unsigned mse_mask, float* part) {
  __shared__ float red[4];
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    s += task_loss(labels[i], probs[i], (mse_mask >> (int)(i / B)) & 1u) * invB;
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void bce_reduce_kernel(const float* __restrict__ part, int nb, float* loss) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    float s = 0.f;
    for (int i = 0; i < nb; ++i) s += part[i];
    loss[0] = s;
  }
}

__global__ void bce_bwd_kernel(const float* __restrict__ probs, const float* __restrict__ labels,
                               const float* __restrict__ gscale, int64_t n, int B, float invB, unsigned mse_mask,
                               float* dprobs) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float eps = 1e-7f;
  const float p = probs[i], y = labels[i];
  float g = 0.f;
  if ((mse_mask >> (int)(i / B)) & 1u) g = 2.f * (p - y) * invB;
  else if (p >= eps && p <= 1.f - eps) g = (-y / (p + eps) + (1.f - y) / (1.f - p + eps)) * invB;
  dprobs[i] = g * gscale[0];
}

// the logits form: BCE tasks from z, MSE tasks (bit t of mse_mask) from p
__global__ __launch_bounds__(256) void loss_z_fwd_kernel(const float* __restrict__ logits, const float* __restrict__ probs,
                                                         const float* __restrict__ labels, int64_t n, int B, float invB,
                                                         unsigned mse_mask, float* part) {
  __shared__ float red[4];
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float y = labels[i];
    if ((mse_mask >> (int)(i / B)) & 1u) {
      const float e = probs[i] - y;
      s += e * e * invB;
    } else {
      s += bce_logits(y, logits[i]) * invB;
    }
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void loss_z_bwd_kernel(const float* __restrict__ probs, const float* __restrict__ labels,
                                  const float* __restrict__ gscale, int64_t n, int B, float invB, unsigned mse_mask,
                                  float* dlogits) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float p = probs[i], y = labels[i];
  const float g = ((mse_mask >> (int)(i / B)) & 1u) ? 2.f * (p - y) * p * (1.f - p) : p - y;
  dlogits[i] = g * invB * gscale[0];
}

inline int bce_blocks(int64_t n) {
  int64_t b = (n + 255) / 256;
  return (int)(b < 256 ? (b < 1 ? 1 : b) : 256);
}
inline int head_nb(int B) {
  int nb = (B + 3) / 4;
  return nb < 64 ? (nb < 1 ? 1 : nb) : 64;
}

}  // namespace ot

using namespace ot;

extern "C" int ot_ns_assemble(const ot_ns_field* fields_dev, int nfields, const float* table, int B, float* out,
                              int64_t ld_out, void* stream) {
  OT_REQUIRE(out && (nfields == 0 || fields_dev), "ot_ns_assemble: null operand");
  if (B == 0 || nfields == 0) return OT_OK;
  hipLaunchKernelGGL(ns_assemble_kernel, dim3(ceil_div(B, 256), nfields), dim3(256), 0, (hipStream_t)stream,
                     fields_dev, table, B, out, ld_out);
  OT_LAUNCH_CHECK("ot_ns_assemble");
  return OT_OK;
}

extern "C" int ot_ns_grad_pack(const ot_ns_field* fields_dev, int nsparse, int width, const float* dmat, int64_t ld,
                               int B, int64_t* keys, float* grads, void* stream) {
  OT_REQUIRE(fields_dev && dmat && keys && grads, "ot_ns_grad_pack: null operand");
  if (B == 0 || nsparse == 0) return OT_OK;
  hipLaunchKernelGGL(ns_grad_pack_kernel, dim3(ceil_div(B, 256), nsparse), dim3(256), 0, (hipStream_t)stream,
                     fields_dev, width, dmat, ld, B, keys, grads);
  OT_LAUNCH_CHECK("ot_ns_grad_pack");
  return OT_OK;
}

extern "C" int ot_fill_rows(float* dst, int64_t ld, const int32_t* rows, int64_t nrows, const float* vec, int d,
                            void* stream) {
  OT_REQUIRE(dst && rows && vec, "ot_fill_rows: null operand");
  if (nrows == 0) return OT_OK;
  hipLaunchKernelGGL(fill_rows_kernel, dim3(ceil_div(nrows * d, 256)), dim3(256), 0, (hipStream_t)stream,
                     dst, ld, rows, nrows, vec, d);
  OT_LAUNCH_CHECK("ot_fill_rows");
  return OT_OK;
}

extern "C" int ot_seq_rows(const int64_t* ids, int64_t ids_stride_b, int B, int L, int64_t vocab, int32_t* in_rows,
                           void* stream) {
  OT_REQUIRE(ids && in_rows && vocab > 0 && vocab <= 2147483647LL, "ot_seq_rows: bad args");
  if ((int64_t)B * L == 0) return OT_OK;
  hipLaunchKernelGGL(seq_rows_kernel, dim3(ceil_div((int64_t)B * L, 256)), dim3(256), 0, (hipStream_t)stream,
                     ids, ids_stride_b, B, L, vocab, in_rows);
  OT_LAUNCH_CHECK("ot_seq_rows");
  return OT_OK;
}

extern "C" int ot_head_fwd(const float* pre1, const float* w2, const float* b2, int T, int B, int dh, float* logits,
                           float* probs, void* stream) {
  OT_REQUIRE(pre1 && w2 && b2 && logits && probs, "ot_head_fwd: null operand");
  if ((int64_t)T * B == 0) return OT_OK;
  hipLaunchKernelGGL(head_fwd_kernel, dim3(ceil_div((int64_t)T * B, 4)), dim3(256), 0, (hipStream_t)stream,
                     pre1, w2, b2, T, B, dh, logits, probs);
  OT_LAUNCH_CHECK("ot_head_fwd");
  return OT_OK;
}

extern "C" size_t ot_head_bwd_workspace_size(int T, int B, int dh) {
  return (size_t)T * head_nb(B) * (dh + 1) * sizeof(float);
}

extern "C" int ot_head_bwd(const float* pre1, const float* w2, const float* probs, const float* dprobs, int T, int B,
                           int dh, float* dpre1, float* dw2, float* db2, int64_t task_stride_w2,
                           int64_t task_stride_b2, int accumulate, void* workspace, size_t ws_bytes, void* stream) {
  OT_REQUIRE(dprobs, "ot_head_bwd: null operand");
  return ot_head_bwd_ex(pre1, w2, probs, dprobs, nullptr, T, B, dh, dpre1, dw2, db2, task_stride_w2, task_stride_b2,
                        accumulate, workspace, ws_bytes, stream);
}

extern "C" int ot_head_bwd_ex(const float* pre1, const float* w2, const float* probs, const float* dprobs,
                              const float* dlogits, int T, int B, int dh, float* dpre1, float* dw2, float* db2,
                              int64_t task_stride_w2, int64_t task_stride_b2, int accumulate, void* workspace,
                              size_t ws_bytes, void* stream) {
  OT_REQUIRE(pre1 && w2 && probs && dpre1 && dw2 && db2, "ot_head_bwd: null operand");
  OT_REQUIRE(dprobs || dlogits, "ot_head_bwd_ex: neither dprobs nor dlogits");
  OT_REQUIRE(dh <= 256, "ot_head_bwd: dh=%d > 256 unsupported", dh);
  OT_REQUIRE(workspace && ws_bytes >= ot_head_bwd_workspace_size(T, B, dh), "ot_head_bwd: workspace too small");
  if ((int64_t)T * B == 0) return OT_OK;
  const int nb = head_nb(B);
  hipLaunchKernelGGL(head_bwd_kernel, dim3(nb, T), dim3(256), 4 * (dh + 1) * sizeof(float), (hipStream_t)stream,
                     pre1, w2, probs, dprobs, dlogits, B, dh, dpre1, (float*)workspace);
  OT_LAUNCH_CHECK("ot_head_bwd");
  hipLaunchKernelGGL(head_bwd_reduce_kernel, dim3(ceil_div(dh + 1, 256), T), dim3(256), 0, (hipStream_t)stream,
                     (const float*)workspace, nb, dh, dw2, db2, task_stride_w2, task_stride_b2, accumulate);
  OT_LAUNCH_CHECK("ot_head_bwd(reduce)");
  return OT_OK;
}

extern "C" size_t ot_bce_workspace_size(int T, int B) { return (size_t)bce_blocks((int64_t)T * B) * sizeof(float); }

extern "C" int ot_task_loss_fwd(const float* probs, const float* labels, int T, int B, unsigned mse_mask, float* loss,
                                void* workspace, size_t ws_bytes, void* stream) {
  OT_REQUIRE(probs && labels && loss && workspace, "ot_task_loss_fwd: null operand");
  OT_REQUIRE(ws_bytes >= ot_bce_workspace_size(T, B), "ot_task_loss_fwd: workspace too small");
  OT_REQUIRE(B > 0, "ot_task_loss_fwd: empty batch");
  OT_REQUIRE(T > 0 && T <= 32, "ot_task_loss_fwd: 1..32 tasks");
  const int64_t n = (int64_t)T * B;
  const int nb = bce_blocks(n);
  hipLaunchKernelGGL(bce_fwd_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, probs, labels, n, B, 1.f / B,
                     mse_mask, (float*)workspace);
  OT_LAUNCH_CHECK("ot_task_loss_fwd");
  hipLaunchKernelGGL(bce_reduce_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (const float*)workspace, nb, loss);
  OT_LAUNCH_CHECK("ot_task_loss_fwd(reduce)");
  return OT_OK;
}

extern "C" int ot_task_loss_bwd(const float* probs, const float* labels, const float* gscale, int T, int B,
                                unsigned mse_mask, float* dprobs, void* stream) {
  OT_REQUIRE(probs && labels && gscale && dprobs && B > 0, "ot_task_loss_bwd: bad args");
  OT_REQUIRE(T > 0 && T <= 32, "ot_task_loss_bwd: 1..32 tasks");
  const int64_t n = (int64_t)T * B;
  hipLaunchKernelGGL(bce_bwd_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, (hipStream_t)stream, probs, labels, gscale,
                     n, B, 1.f / B, mse_mask, dprobs);
  OT_LAUNCH_CHECK("ot_task_loss_bwd");
  return OT_OK;
}

extern "C" int ot_task_loss_logits_fwd(const float* logits, const float* probs, const float* labels, int T, int B,
                                       unsigned mse_mask, float* loss, void* workspace, size_t ws_bytes, void* stream) {
  OT_REQUIRE(logits && probs && labels && loss && workspace, "ot_task_loss_logits_fwd: null operand");
  OT_REQUIRE(ws_bytes >= ot_bce_workspace_size(T, B), "ot_task_loss_logits_fwd: workspace too small");
  OT_REQUIRE(B > 0, "ot_task_loss_logits_fwd: empty batch");
  OT_REQUIRE(T > 0 && T <= 32, "ot_task_loss_logits_fwd: 1..32 tasks");
  const int64_t n = (int64_t)T * B;
  const int nb = bce_blocks(n);
  hipLaunchKernelGGL(loss_z_fwd_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, logits, probs, labels, n, B,
                     1.f / B, mse_mask, (float*)workspace);
  OT_LAUNCH_CHECK("ot_task_loss_logits_fwd");
  hipLaunchKernelGGL(bce_reduce_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (const float*)workspace, nb, loss);
  OT_LAUNCH_CHECK("ot_task_loss_logits_fwd(reduce)");
  return OT_OK;
}

extern "C" int ot_task_loss_logits_bwd(const float* probs, const float* labels, const float* gscale, int T, int B,
                                       unsigned mse_mask, float* dlogits, void* stream) {
  OT_REQUIRE(probs && labels && gscale && dlogits && B > 0, "ot_task_loss_logits_bwd: bad args");
  OT_REQUIRE(T > 0 && T <= 32, "ot_task_loss_logits_bwd: 1..32 tasks");
  const int64_t n = (int64_t)T * B;
  hipLaunchKernelGGL(loss_z_bwd_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, (hipStream_t)stream, probs, labels,
                     gscale, n, B, 1.f / B, mse_mask, dlogits);
  OT_LAUNCH_CHECK("ot_task_loss_logits_bwd");
  return OT_OK;
}

extern "C" int ot_bce_fwd(const float* probs, const float* labels, int T, int B, float* loss, void* workspace,
                          size_t ws_bytes, void* stream) {
  return ot_task_loss_fwd(probs, labels, T, B, 0u, loss, workspace, ws_bytes, stream);
}

extern "C" int ot_bce_bwd(const float* probs, const float* labels, const float* gscale, int T, int B, float* dprobs,
                          void* stream) {
  return ot_task_loss_bwd(probs, labels, gscale, T, B, 0u, dprobs, stream);
}
