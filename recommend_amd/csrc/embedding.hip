// Sparse embedding update (build extension; paper: sparse Adagrad + clip 120,
// rank/scaling_up/oneTrans/translation/complete_translation.md:190).
//
// Keras-2.12 Adagrad on a de-duplicated IndexedSlices gradient:
//   1. (key, position) pairs radix-sorted with rocPRIM (stable => rows of one key stay in
//      position order)
//   2. segment heads + inclusive scan -> unique keys and segment starts
//   3. per unique key: sum of its gradient rows in position order (deterministic)
//   4. clip_by_norm(clip) over the unique-row gradient (one device scalar, no host sync)
//   5. acc[r] += g^2 ; w[r] -= lr * g / sqrt(acc[r] + eps)
// HBM-bound: the row reads in step 3 and the table/accumulator row RMW in step 5.
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "common.h"

namespace ot {

__global__ void keys_prep_kernel(const int64_t* __restrict__ keys, int64_t n, int64_t num_rows, uint32_t* k32,
                                 int32_t* vals) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t k = keys[i];
  k32[i] = (k >= 0 && k < num_rows) ? (uint32_t)k : 0xFFFFFFFFu;   // invalid keys sort last, skipped
  vals[i] = (int32_t)i;
}

__global__ void head_flags_kernel(const uint32_t* __restrict__ k, int64_t n, int32_t* flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  flags[i] = (i == 0 || k[i] != k[i - 1]) ? 1 : 0;
}

__global__ void seg_start_kernel(const int32_t* __restrict__ flags, const int32_t* __restrict__ pos, int64_t n,
                                 int32_t* seg_start, int32_t* nuniq) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (flags[i]) seg_start[pos[i] - 1] = (int32_t)i;
  if (i == n - 1) {
    seg_start[pos[i]] = (int32_t)n;
    nuniq[0] = pos[i];
  }
}

// Hot keys (Zipf) can own tens of thousands of rows: every segment is cut into pieces of at most
// PIECE rows; pass 1 sums each piece, pass 2 sums each key's pieces in order (both deterministic).
constexpr int PIECE = 64;

__global__ void piece_count_kernel(const int32_t* __restrict__ seg_start, const int32_t* __restrict__ nuniq,
                                   int64_t n, int32_t* pcount) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s > n) return;
  const int U = nuniq[0];
  pcount[s] = s < U ? (seg_start[s + 1] - seg_start[s] + PIECE - 1) / PIECE : 0;
}

// TPS threads per piece / segment, float4 each (E = 4*TPS*k)
__global__ __launch_bounds__(256) void piece_sum_kernel(const float* __restrict__ grads, int E,
                                                        const int32_t* __restrict__ perm,
                                                        const int32_t* __restrict__ seg_start,
                                                        const int32_t* __restrict__ pstart,
                                                        const int32_t* __restrict__ nuniq, int tps, float* psum) {
  const int ppb = 256 / tps;
  const int64_t pc = (int64_t)blockIdx.x * ppb + threadIdx.x / tps;
  const int lt = threadIdx.x % tps;
  const int U = nuniq[0];
  if (pc >= pstart[U]) return;
  int lo = 0, hi = U - 1;                         // largest s with pstart[s] <= pc
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (pstart[mid] <= pc) lo = mid; else hi = mid - 1;
  }
  const int i0 = seg_start[lo] + (int)(pc - pstart[lo]) * PIECE;
  const int i1 = min(i0 + PIECE, seg_start[lo + 1]);
  for (int c = lt * 4; c < E; c += tps * 4) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int i = i0; i < i1; ++i) acc += *reinterpret_cast<const f32x4*>(grads + (int64_t)perm[i] * E + c);
    *reinterpret_cast<f32x4*>(psum + pc * E + c) = acc;
  }
}

__global__ __launch_bounds__(256) void seg_sum_kernel(const float* __restrict__ psum, int E,
                                                      const uint32_t* __restrict__ ksorted,
                                                      const int32_t* __restrict__ seg_start,
                                                      const int32_t* __restrict__ pstart,
                                                      const int32_t* __restrict__ nuniq, int tps, float* gsum,
                                                      float* sq_part) {
  __shared__ float red[4];
  const int spb = 256 / tps;
  const int64_t s = (int64_t)blockIdx.x * spb + threadIdx.x / tps;
  const int lt = threadIdx.x % tps;
  float sq = 0.f;
  if (s < nuniq[0] && ksorted[seg_start[s]] != 0xFFFFFFFFu) {
    const int b = pstart[s], e = pstart[s + 1];
    for (int c = lt * 4; c < E; c += tps * 4) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int q = b; q < e; ++q) acc += *reinterpret_cast<const f32x4*>(psum + (int64_t)q * E + c);
      *reinterpret_cast<f32x4*>(gsum + s * E + c) = acc;
      sq += acc.x * acc.x + acc.y * acc.y + acc.z * acc.z + acc.w * acc.w;
    }
  }
  sq = wave_sum(sq);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sq;
  __syncthreads();
  if (threadIdx.x == 0) sq_part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void clip_scale_kernel(const float* __restrict__ part, int n, float clip,
                                                         float* scale) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += part[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float l2 = sqrtf((red[0] + red[1]) + (red[2] + red[3]));
    scale[0] = clip > 0.f ? clip / fmaxf(l2, clip) : 1.f;
  }
}

__global__ __launch_bounds__(256) void adagrad_apply_kernel(float* table, float* accum, int E,
                                                            const uint32_t* __restrict__ ksorted,
                                                            const int32_t* __restrict__ seg_start,
                                                            const int32_t* __restrict__ nuniq,
                                                            const float* __restrict__ gsum,
                                                            const float* __restrict__ scale, int tps, float lr,
                                                            float eps) {
  const int spb = 256 / tps;
  const int64_t s = (int64_t)blockIdx.x * spb + threadIdx.x / tps;
  const int lt = threadIdx.x % tps;
  if (s >= nuniq[0]) return;
  const uint32_t key = ksorted[seg_start[s]];
  if (key == 0xFFFFFFFFu) return;
  const float sc = scale[0];
  float* w = table + (int64_t)key * E;
  float* a = accum + (int64_t)key * E;
  for (int c = lt * 4; c < E; c += tps * 4) {
    f32x4 g = *reinterpret_cast<const f32x4*>(gsum + s * E + c) * sc;
    f32x4 av = *reinterpret_cast<const f32x4*>(a + c) + g * g;
    f32x4 wv = *reinterpret_cast<const f32x4*>(w + c);
    wv.x -= lr * g.x / sqrtf(av.x + eps);
    wv.y -= lr * g.y / sqrtf(av.y + eps);
    wv.z -= lr * g.z / sqrtf(av.z + eps);
    wv.w -= lr * g.w / sqrtf(av.w + eps);
    *reinterpret_cast<f32x4*>(a + c) = av;
    *reinterpret_cast<f32x4*>(w + c) = wv;
  }
}

// Dense form of a replicated table's gradient (data-parallel exchange by all-reduce): the unique
// rows' sums scattered into a zeroed [num_rows, E] buffer (unique keys: no conflicts).
__global__ __launch_bounds__(256) void scatter_rows_kernel(float* dense, int E, const uint32_t* __restrict__ ksorted,
                                                           const int32_t* __restrict__ seg_start,
                                                           const int32_t* __restrict__ nuniq,
                                                           const float* __restrict__ gsum, int tps) {
  const int spb = 256 / tps;
  const int64_t s = (int64_t)blockIdx.x * spb + threadIdx.x / tps;
  const int lt = threadIdx.x % tps;
  if (s >= nuniq[0]) return;
  const uint32_t key = ksorted[seg_start[s]];
  if (key == 0xFFFFFFFFu) return;
  for (int c = lt * 4; c < E; c += tps * 4)
    *reinterpret_cast<f32x4*>(dense + (int64_t)key * E + c) = *reinterpret_cast<const f32x4*>(gsum + s * E + c);
}

// sum of squares of a dense gradient: per-block partials (fixed grid-stride order: deterministic)
__global__ __launch_bounds__(256) void dense_sumsq_kernel(const float* __restrict__ g, int64_t n4, float* part) {
  __shared__ float red[4];
  float sq = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(g + 4 * i);
    sq += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  sq = wave_sum(sq);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sq;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// Keras Adagrad over every row; rows with a zero gradient are left bitwise unchanged (acc + 0,
// w - 0), i.e. exactly the sparse update of the touched rows.
__global__ __launch_bounds__(256) void dense_adagrad_kernel(float* table, float* accum, const float* __restrict__ g,
                                                            int64_t n4, const float* __restrict__ scale, float lr,
                                                            float eps) {
  const float sc = scale[0];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const f32x4 gv = *reinterpret_cast<const f32x4*>(g + 4 * i) * sc;
    if (gv.x == 0.f && gv.y == 0.f && gv.z == 0.f && gv.w == 0.f) continue;
    f32x4 av = *reinterpret_cast<const f32x4*>(accum + 4 * i) + gv * gv;
    f32x4 wv = *reinterpret_cast<const f32x4*>(table + 4 * i);
    wv.x -= lr * gv.x / sqrtf(av.x + eps);
    wv.y -= lr * gv.y / sqrtf(av.y + eps);
    wv.z -= lr * gv.z / sqrtf(av.z + eps);
    wv.w -= lr * gv.w / sqrtf(av.w + eps);
    *reinterpret_cast<f32x4*>(accum + 4 * i) = av;
    *reinterpret_cast<f32x4*>(table + 4 * i) = wv;
  }
}
constexpr int DENSE_GRID = 2048;

// fixed-order sum of the per-block squared-norm partials (one block)
__global__ __launch_bounds__(256) void sum_parts_kernel(const float* __restrict__ part, int n, float* out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += part[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = (red[0] + red[1]) + (red[2] + red[3]);
}

// clip scale from an externally reduced squared norm (row-sharded tables: sum over owners)
__global__ void clip_from_sumsq_kernel(const float* __restrict__ sumsq, float clip, float* scale) {
  if (threadIdx.x == 0) {
    const float l2 = sqrtf(sumsq[0]);
    scale[0] = clip > 0.f ? clip / fmaxf(l2, clip) : 1.f;
  }
}

struct SparseWs {
  uint32_t *k_in, *k_out;
  int32_t *v_in, *v_out, *flags, *pos, *seg_start, *nuniq, *pcount, *pstart;
  float *gsum, *psum, *sq_part, *scale;
  void* tmp;
  size_t tmp_bytes;
  size_t total;
};

inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

inline int tps_for(int E) {
  int t = E / 4;
  return t > 64 ? 64 : t;
}

SparseWs carve(void* base, int64_t n, int E) {
  SparseWs w{};
  size_t sort_bytes = 0, scan_bytes = 0;
  (void)rocprim::radix_sort_pairs(nullptr, sort_bytes, (uint32_t*)nullptr, (uint32_t*)nullptr, (int32_t*)nullptr,
                                  (int32_t*)nullptr, (size_t)n, 0, 32);
  (void)rocprim::inclusive_scan(nullptr, scan_bytes, (int32_t*)nullptr, (int32_t*)nullptr, (size_t)n,
                                rocprim::plus<int32_t>());
  size_t escan_bytes = 0;
  (void)rocprim::exclusive_scan(nullptr, escan_bytes, (int32_t*)nullptr, (int32_t*)nullptr, 0, (size_t)n + 1,
                                rocprim::plus<int32_t>());
  w.tmp_bytes = sort_bytes > scan_bytes ? sort_bytes : scan_bytes;
  w.tmp_bytes = w.tmp_bytes > escan_bytes ? w.tmp_bytes : escan_bytes;
  const int spb = 256 / tps_for(E);
  const int64_t nblk = (n + spb - 1) / spb;
  char* p = (char*)base;
  size_t off = 0;
  auto take = [&](size_t bytes) { char* r = p ? p + off : nullptr; off += al(bytes); return (void*)r; };
  w.k_in = (uint32_t*)take(n * 4); w.k_out = (uint32_t*)take(n * 4);
  w.v_in = (int32_t*)take(n * 4); w.v_out = (int32_t*)take(n * 4);
  w.flags = (int32_t*)take(n * 4); w.pos = (int32_t*)take(n * 4);
  w.seg_start = (int32_t*)take((n + 1) * 4); w.nuniq = (int32_t*)take(4);
  w.pcount = (int32_t*)take((n + 1) * 4); w.pstart = (int32_t*)take((n + 1) * 4);
  w.gsum = (float*)take((size_t)n * E * 4); w.psum = (float*)take((size_t)(n + n / PIECE + 1) * E * 4);
  w.sq_part = (float*)take(nblk * 4); w.scale = (float*)take(4);
  w.tmp = take(w.tmp_bytes);
  w.total = off;
  return w;
}

}  // namespace ot

using namespace ot;

extern "C" size_t ot_sparse_adagrad_workspace_size(int64_t n, int E) {
  if (n <= 0) return 256;
  return carve(nullptr, n, E).total;
}

// steps 1-3 (+ the per-block squared-norm partials of the unique-row sums): fills w.k_out,
// w.seg_start, w.nuniq, w.gsum, w.sq_part
static int segment_rows(const SparseWs& w, int E, int64_t num_rows, const int64_t* keys, const float* grads,
                        int64_t n, hipStream_t s) {
  const unsigned g1 = ceil_div(n, 256);
  hipLaunchKernelGGL(keys_prep_kernel, dim3(g1), dim3(256), 0, s, keys, n, num_rows, w.k_in, w.v_in);
  OT_LAUNCH_CHECK("ot_sparse_adagrad(prep)");
  int end_bit = 1;
  while (end_bit < 32 && ((uint64_t)1 << end_bit) < (uint64_t)num_rows + 1) ++end_bit;
  // 2^end_bit > num_rows: the invalid sentinel's low bits (2^end_bit - 1) still sort after every valid key
  size_t tb = w.tmp_bytes;
  hipError_t e = rocprim::radix_sort_pairs(w.tmp, tb, w.k_in, w.k_out, w.v_in, w.v_out, (size_t)n, 0, end_bit, s);
  if (e != hipSuccess) return fail(OT_ERR_HIP, "ot_sparse_adagrad(sort): %s", hipGetErrorString(e));
  hipLaunchKernelGGL(head_flags_kernel, dim3(g1), dim3(256), 0, s, w.k_out, n, w.flags);
  OT_LAUNCH_CHECK("ot_sparse_adagrad(flags)");
  tb = w.tmp_bytes;
  e = rocprim::inclusive_scan(w.tmp, tb, w.flags, w.pos, (size_t)n, rocprim::plus<int32_t>(), s);
  if (e != hipSuccess) return fail(OT_ERR_HIP, "ot_sparse_adagrad(scan): %s", hipGetErrorString(e));
  hipLaunchKernelGGL(seg_start_kernel, dim3(g1), dim3(256), 0, s, w.flags, w.pos, n, w.seg_start, w.nuniq);
  OT_LAUNCH_CHECK("ot_sparse_adagrad(segments)");
  const int tps = tps_for(E);
  hipLaunchKernelGGL(piece_count_kernel, dim3(ceil_div(n + 1, 256)), dim3(256), 0, s, w.seg_start, w.nuniq, n,
                     w.pcount);
  OT_LAUNCH_CHECK("ot_sparse_adagrad(pieces)");
  tb = w.tmp_bytes;
  e = rocprim::exclusive_scan(w.tmp, tb, w.pcount, w.pstart, 0, (size_t)n + 1, rocprim::plus<int32_t>(), s);
  if (e != hipSuccess) return fail(OT_ERR_HIP, "ot_sparse_adagrad(piece scan): %s", hipGetErrorString(e));
  const unsigned gp = ceil_div(n + n / PIECE + 1, 256 / tps);
  hipLaunchKernelGGL(piece_sum_kernel, dim3(gp), dim3(256), 0, s, grads, E, w.v_out, w.seg_start, w.pstart, w.nuniq,
                     tps, w.psum);
  OT_LAUNCH_CHECK("ot_sparse_adagrad(piecesum)");
  const unsigned g2 = ceil_div(n, 256 / tps);
  hipLaunchKernelGGL(seg_sum_kernel, dim3(g2), dim3(256), 0, s, w.psum, E, w.k_out, w.seg_start, w.pstart, w.nuniq,
                     tps, w.gsum, w.sq_part);
  OT_LAUNCH_CHECK("ot_sparse_adagrad(segsum)");
  return OT_OK;
}

extern "C" int ot_sparse_adagrad(float* table, float* accum, int E, int64_t num_rows, const int64_t* keys,
                                 const float* grads, int64_t n, float lr, float eps, float clip, void* workspace,
                                 size_t ws_bytes, void* stream) {
  OT_REQUIRE(table && accum && keys && grads, "ot_sparse_adagrad: null operand");
  OT_REQUIRE(E > 0 && E % 4 == 0 && E <= 1024, "ot_sparse_adagrad: E=%d must be a multiple of 4 <= 1024", E);
  OT_REQUIRE(num_rows > 0 && num_rows < 0xFFFFFFFFLL, "ot_sparse_adagrad: num_rows out of range");
  OT_REQUIRE(n >= 0 && n < 2147483647LL, "ot_sparse_adagrad: n out of range");
  if (n == 0) return OT_OK;
  SparseWs w = carve(workspace, n, E);
  OT_REQUIRE(ws_bytes >= w.total, "ot_sparse_adagrad: workspace too small (%zu < %zu)", ws_bytes, w.total);
  hipStream_t s = (hipStream_t)stream;
  const int rc = segment_rows(w, E, num_rows, keys, grads, n, s);
  if (rc != OT_OK) return rc;
  const int tps = tps_for(E);
  const unsigned g2 = ceil_div(n, 256 / tps);
  hipLaunchKernelGGL(clip_scale_kernel, dim3(1), dim3(256), 0, s, w.sq_part, (int)g2, clip, w.scale);
  OT_LAUNCH_CHECK("ot_sparse_adagrad(clip)");
  hipLaunchKernelGGL(adagrad_apply_kernel, dim3(g2), dim3(256), 0, s, table, accum, E, w.k_out, w.seg_start, w.nuniq,
                     w.gsum, w.scale, tps, lr, eps);
  OT_LAUNCH_CHECK("ot_sparse_adagrad(apply)");
  return OT_OK;
}

extern "C" int ot_sparse_grad_dense(int E, int64_t num_rows, const int64_t* keys, const float* grads, int64_t n,
                                    float* dense, void* workspace, size_t ws_bytes, void* stream) {
  OT_REQUIRE(keys && grads && dense, "ot_sparse_grad_dense: null operand");
  OT_REQUIRE(E > 0 && E % 4 == 0 && E <= 1024, "ot_sparse_grad_dense: E=%d must be a multiple of 4 <= 1024", E);
  OT_REQUIRE(num_rows > 0 && num_rows < 0xFFFFFFFFLL, "ot_sparse_grad_dense: num_rows out of range");
  OT_REQUIRE(n >= 0 && n < 2147483647LL, "ot_sparse_grad_dense: n out of range");
  if (n == 0) return OT_OK;
  SparseWs w = carve(workspace, n, E);
  OT_REQUIRE(ws_bytes >= w.total, "ot_sparse_grad_dense: workspace too small (%zu < %zu)", ws_bytes, w.total);
  hipStream_t s = (hipStream_t)stream;
  const int rc = segment_rows(w, E, num_rows, keys, grads, n, s);
  if (rc != OT_OK) return rc;
  const int tps = tps_for(E);
  hipLaunchKernelGGL(scatter_rows_kernel, dim3(ceil_div(n, 256 / tps)), dim3(256), 0, s, dense, E, w.k_out,
                     w.seg_start, w.nuniq, w.gsum, tps);
  OT_LAUNCH_CHECK("ot_sparse_grad_dense(scatter)");
  return OT_OK;
}

extern "C" size_t ot_dense_adagrad_workspace_size(void) { return (DENSE_GRID + 64) * sizeof(float); }

extern "C" int ot_dense_adagrad(float* table, float* accum, const float* grad, int64_t num_rows, int E, float lr,
                                float eps, float clip, void* workspace, size_t ws_bytes, void* stream) {
  OT_REQUIRE(table && accum && grad && workspace, "ot_dense_adagrad: null operand");
  OT_REQUIRE(E > 0 && E % 4 == 0, "ot_dense_adagrad: E must be a multiple of 4");
  OT_REQUIRE(ws_bytes >= ot_dense_adagrad_workspace_size(), "ot_dense_adagrad: workspace too small");
  if (num_rows <= 0) return OT_OK;
  hipStream_t s = (hipStream_t)stream;
  const int64_t n4 = num_rows * E / 4;
  float* part = (float*)workspace;
  float* scale = part + DENSE_GRID;
  hipLaunchKernelGGL(dense_sumsq_kernel, dim3(DENSE_GRID), dim3(256), 0, s, grad, n4, part);
  OT_LAUNCH_CHECK("ot_dense_adagrad(norm)");
  hipLaunchKernelGGL(clip_scale_kernel, dim3(1), dim3(256), 0, s, part, DENSE_GRID, clip, scale);
  OT_LAUNCH_CHECK("ot_dense_adagrad(clip)");
  hipLaunchKernelGGL(dense_adagrad_kernel, dim3(DENSE_GRID), dim3(256), 0, s, table, accum, grad, n4, scale, lr, eps);
  OT_LAUNCH_CHECK("ot_dense_adagrad(apply)");
  return OT_OK;
}

// Two-phase form for row-sharded tables, whose clip_by_norm spans every owner's rows: prepare
// de-duplicates this rank's received (key, row) pairs and writes the local squared norm; the caller
// all-reduces it; finish applies clip + Adagrad with the global norm.  The workspace (size
// ot_sparse_adagrad_workspace_size(n, E)) carries the segmentation from prepare to finish.
extern "C" int ot_sparse_prepare(int E, int64_t num_rows, const int64_t* keys, const float* grads, int64_t n,
                                 float* sumsq_out, void* workspace, size_t ws_bytes, void* stream) {
  OT_REQUIRE(keys && grads && sumsq_out && workspace, "ot_sparse_prepare: null operand");
  OT_REQUIRE(E > 0 && E % 4 == 0 && E <= 1024, "ot_sparse_prepare: E=%d must be a multiple of 4 <= 1024", E);
  OT_REQUIRE(num_rows > 0 && num_rows < 0xFFFFFFFFLL, "ot_sparse_prepare: num_rows out of range");
  OT_REQUIRE(n >= 0 && n < 2147483647LL, "ot_sparse_prepare: n out of range");
  hipStream_t s = (hipStream_t)stream;
  if (n == 0) {
    (void)hipMemsetAsync(sumsq_out, 0, sizeof(float), s);
    return OT_OK;
  }
  SparseWs w = carve(workspace, n, E);
  OT_REQUIRE(ws_bytes >= w.total, "ot_sparse_prepare: workspace too small (%zu < %zu)", ws_bytes, w.total);
  const int rc = segment_rows(w, E, num_rows, keys, grads, n, s);
  if (rc != OT_OK) return rc;
  const unsigned g2 = ceil_div(n, 256 / tps_for(E));
  hipLaunchKernelGGL(sum_parts_kernel, dim3(1), dim3(256), 0, s, w.sq_part, (int)g2, sumsq_out);
  OT_LAUNCH_CHECK("ot_sparse_prepare(sumsq)");
  return OT_OK;
}

extern "C" int ot_sparse_finish(float* table, float* accum, int E, int64_t n, float lr, float eps, float clip,
                                const float* sumsq_total, void* workspace, size_t ws_bytes, void* stream) {
  OT_REQUIRE(table && accum && sumsq_total && workspace, "ot_sparse_finish: null operand");
  if (n <= 0) return OT_OK;
  SparseWs w = carve(workspace, n, E);
  OT_REQUIRE(ws_bytes >= w.total, "ot_sparse_finish: workspace too small (%zu < %zu)", ws_bytes, w.total);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(clip_from_sumsq_kernel, dim3(1), dim3(64), 0, s, sumsq_total, clip, w.scale);
  OT_LAUNCH_CHECK("ot_sparse_finish(clip)");
  const int tps = tps_for(E);
  const unsigned g2 = ceil_div(n, 256 / tps);
  hipLaunchKernelGGL(adagrad_apply_kernel, dim3(g2), dim3(256), 0, s, table, accum, E, w.k_out, w.seg_start, w.nuniq,
                     w.gsum, w.scale, tps, lr, eps);
  OT_LAUNCH_CHECK("ot_sparse_finish(apply)");
  return OT_OK;
}
