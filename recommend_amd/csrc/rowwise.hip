// Row-wise HBM-bound kernels: RMSNorm (model.py:19-23) forward/backward, the dropout mask
// (model.py:184,193,198) applied to a gradient, and deterministic column sums.
//
// RMSNorm is never materialised in the forward pass of a block: ot_rmsnorm_fwd writes only
// rstd[row] and the consuming GEMM applies x * rstd * gamma in its A-load prologue
// (OT_AX_RMSNORM).  The backward fuses the residual pass-through and the dropout mask of the
// residual branch that produced x:
//   dx   = dres + rstd * (gamma * dy) - x * rstd^3 / d * sum(gamma * dy * x)
//   dx_m = mask(dx)                                  (optional: gradient of the pre-dropout branch)
//   dgamma_partial[block] = sum_rows dy * x * rstd   (reduced by ot_colsum_reduce)
#include "common.h"

namespace ot {

// threads per row: TPR lanes cover d/4 float4 chunks (TPR = min(64, d/4) rounded down to pow2)
__device__ __forceinline__ float group_sum(float v, int tpr) {
  for (int o = tpr >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(256) void rmsnorm_fwd_kernel(const float* __restrict__ x, int64_t ldx,
                                                          const float* __restrict__ gamma, float* y, int64_t ldy,
                                                          float* rstd, int64_t rows, int d, float eps, int tpr) {
  const int rpb = 256 / tpr;
  const int64_t row = (int64_t)blockIdx.x * rpb + threadIdx.x / tpr;
  const int lt = threadIdx.x % tpr;
  const bool live = row < rows;
  const float* xr = x + (live ? row : 0) * ldx;
  float ss = 0.f;
  for (int c = lt * 4; c < d; c += tpr * 4) {
    f32x4 v = *reinterpret_cast<const f32x4*>(xr + c);
    ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  ss = group_sum(ss, tpr);
  const float r = rsqrtf(ss / (float)d + eps);
  if (!live) return;
  if (lt == 0 && rstd) rstd[row] = r;
  if (y) {
    float* yr = y + row * ldy;
    for (int c = lt * 4; c < d; c += tpr * 4) {
      f32x4 v = *reinterpret_cast<const f32x4*>(xr + c);
      f32x4 g = *reinterpret_cast<const f32x4*>(gamma + c);
      *reinterpret_cast<f32x4*>(yr + c) = v * r * g;
    }
  }
}

struct RmsBwdArgs {
  const float* dy; int64_t lddy;
  const float* x; int64_t ldx;
  const float* gamma; const float* rstd;
  const float* dres; int64_t lddres; int dres_K, dres_I;   // dres_K > 0: dres holds only the tail rows
  float* dx; int64_t lddx;
  float* dxm; int64_t lddxm;            // optional masked copy
  uint32_t seed, site, thr; float dscale; int tail_K, tail_I;
  float* dgamma_part;                   // [gridDim.x][d] or null
  int64_t rows; int d; int tpr;
  const int32_t* tail_pos; const int32_t* dres_inv;   // ot_pyramid_select maps or null (tail rule)
};

__global__ __launch_bounds__(256) void rmsnorm_bwd_kernel(RmsBwdArgs p) {
  extern __shared__ __attribute__((aligned(16))) float red[];   // [256/tpr][d] for dgamma
  const int tpr = p.tpr, rpb = 256 / tpr, d = p.d;
  const int lr = threadIdx.x / tpr, lt = threadIdx.x % tpr;
  f32x4 dg[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) dg[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int64_t row0 = (int64_t)blockIdx.x * rpb; row0 < p.rows; row0 += (int64_t)gridDim.x * rpb) {
    const int64_t row = row0 + lr;
    const bool live = row < p.rows;
    const int64_t rr = live ? row : 0;
    const float* dyr = p.dy + rr * p.lddy;
    const float* xr = p.x + rr * p.ldx;
    const float r = live ? p.rstd[rr] : 0.f;
    float s = 0.f;
    for (int c = lt * 4; c < d; c += tpr * 4) {
      f32x4 a = *reinterpret_cast<const f32x4*>(dyr + c);
      f32x4 g = *reinterpret_cast<const f32x4*>(p.gamma + c);
      f32x4 v = *reinterpret_cast<const f32x4*>(xr + c);
      s += a.x * g.x * v.x + a.y * g.y * v.y + a.z * g.z * v.z + a.w * g.w * v.w;
    }
    s = group_sum(s, tpr);
    const float coef = r * r * r * s / (float)d;
    const int64_t tok = p.dxm ? tail_token(rr, p.tail_K, p.tail_I, p.tail_pos) : 0;
    int q = 0;
    for (int c = lt * 4; c < d; c += tpr * 4, ++q) {
      f32x4 a = *reinterpret_cast<const f32x4*>(dyr + c);
      f32x4 g = *reinterpret_cast<const f32x4*>(p.gamma + c);
      f32x4 v = *reinterpret_cast<const f32x4*>(xr + c);
      if (!live) continue;
      f32x4 o = a * g * r - v * coef;
      if (p.dres) {
        const int64_t dr = p.dres_K > 0 ? kept_row(rr, p.dres_K, p.dres_I, p.dres_inv) : rr;
        if (dr >= 0) o += *reinterpret_cast<const f32x4*>(p.dres + dr * p.lddres + c);
      }
      if (q < 4) dg[q] += a * v * r;
      *reinterpret_cast<f32x4*>(p.dx + rr * p.lddx + c) = o;
      if (p.dxm) {
        f32x4 m;
        uint32_t base = (uint32_t)(tok * d + c);
        m.x = drop_keep(p.seed, p.site, base + 0, p.thr) ? o.x * p.dscale : 0.f;
        m.y = drop_keep(p.seed, p.site, base + 1, p.thr) ? o.y * p.dscale : 0.f;
        m.z = drop_keep(p.seed, p.site, base + 2, p.thr) ? o.z * p.dscale : 0.f;
        m.w = drop_keep(p.seed, p.site, base + 3, p.thr) ? o.w * p.dscale : 0.f;
        *reinterpret_cast<f32x4*>(p.dxm + rr * p.lddxm + c) = m;
      }
    }
  }
  if (p.dgamma_part) {
    int q = 0;
    for (int c = lt * 4; c < d; c += tpr * 4, ++q) *reinterpret_cast<f32x4*>(red + lr * d + c) = dg[q];
    __syncthreads();
    for (int c = threadIdx.x; c < d; c += 256) {
      float acc = 0.f;
      for (int k = 0; k < rpb; ++k) acc += red[k * d + c];
      p.dgamma_part[(int64_t)blockIdx.x * d + c] = acc;
    }
  }
}

// out[c] (+)= sum_{b < nparts} part[b][c]   (fixed order: deterministic).  Block = 16 columns x 16
// part-groups (group q sums parts q, q+16, ...), combined in a fixed order through LDS.
__global__ __launch_bounds__(256) void colsum_reduce_kernel(const float* __restrict__ part, int64_t nparts, int ncols,
                                                            float* out, int accumulate) {
  __shared__ float red[16][17];
  const int cc = threadIdx.x & 15, q = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cc;
  float s = 0.f;
  if (c < ncols)
    for (int64_t b = q; b < nparts; b += 16) s += part[b * ncols + c];
  red[q][cc] = s;
  __syncthreads();
  if (q == 0 && c < ncols) {
    float t = red[0][cc];
#pragma unroll
    for (int k = 1; k < 16; ++k) t += red[k][cc];
    out[c] = accumulate ? out[c] + t : t;
  }
}

// First level for tall partial stacks: chunk[k][c] = sum of parts [64k, 64k + 64) of column c.
// Block = 64 columns x 4 groups of 16 consecutive parts (coalesced 256-B rows), fixed-order combine.
__global__ __launch_bounds__(256) void colsum_chunk_kernel(const float* __restrict__ part, int64_t nparts, int ncols,
                                                           float* chunk) {
  __shared__ float red[4][64];
  const int cc = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cc;
  const int64_t b0 = (int64_t)blockIdx.y * 64 + 16 * g;
  float s = 0.f;
  if (c < ncols) {
#pragma unroll 4
    for (int i = 0; i < 16; ++i)
      if (b0 + i < nparts) s += part[(b0 + i) * ncols + c];
  }
  red[g][cc] = s;
  __syncthreads();
  if (g == 0 && c < ncols) chunk[(int64_t)blockIdx.y * ncols + c] = ((red[0][cc] + red[1][cc]) + red[2][cc]) + red[3][cc];
}

// part[blk][c] = sum of rows [blk*RPB, (blk+1)*RPB) of the listed rows, column c
__global__ void rows_colsum_kernel(const float* __restrict__ src, int64_t ld, const int32_t* __restrict__ rows,
                                   int64_t nrows, int ncols, int rows_per_block, float* part) {
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_block;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncols) return;
  float s = 0.f;
  for (int64_t i = r0; i < r0 + rows_per_block && i < nrows; ++i) {
    int64_t r = rows ? rows[i] : i;
    s += src[r * ld + c];
  }
  part[(int64_t)blockIdx.y * ncols + c] = s;
}

// OUT: float (f32 rows) or uint16_t (bf16 rows, rounded to nearest even: the bf16 mode's FFN2 dgrad A operand
// and W2 weight-gradient D operand, which round it so anyway)
constexpr int DROPOUT_PASSES = 4;
template <typename OUT>
__global__ void dropout_apply_kernel(const float* __restrict__ src, int64_t lds, OUT* __restrict__ dst, int64_t ldd,
                                     int64_t rows, int d, uint32_t seed, uint32_t site, uint32_t thr, float scale,
                                     int tail_K, int tail_I, const int32_t* tail_pos, float* amax, float* rowmax,
                                     int rowmax_n) {
  // DROPOUT_PASSES float4s per thread, grid-strided (each pass coalesced; every load issued before the first
  // store): the magnitude outputs cost one wave reduction per DROPOUT_PASSES float4s instead of per one
  const int64_t nthreads = (int64_t)gridDim.x * blockDim.x, n4 = rows * d;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  f32x4 v[DROPOUT_PASSES];
  int64_t rr[DROPOUT_PASSES];
  int cc[DROPOUT_PASSES];
#pragma unroll
  for (int ps = 0; ps < DROPOUT_PASSES; ++ps) {
    const int64_t i4 = (t0 + ps * nthreads) * 4;
    const bool in = i4 < n4;
    rr[ps] = in ? (n4 < (1ll << 31) ? (int64_t)((uint32_t)i4 / (uint32_t)d) : i4 / d) : -1;   // (32-bit divide)
    cc[ps] = (int)(i4 - (in ? rr[ps] : 0) * d);
    v[ps] = in ? *reinterpret_cast<const f32x4*>(src + rr[ps] * lds + cc[ps]) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  float am = 0.f;
#pragma unroll
  for (int ps = 0; ps < DROPOUT_PASSES; ++ps) {
    const int64_t r = rr[ps];
    const int c = cc[ps];
    float pm = 0.f;
    if (r >= 0) {
      const int64_t tok = tail_token(r, tail_K, tail_I, tail_pos);
      const uint32_t base = (uint32_t)(tok * d + c);
      f32x4 w = v[ps];
      w.x = drop_keep(seed, site, base + 0, thr) ? w.x * scale : 0.f;
      w.y = drop_keep(seed, site, base + 1, thr) ? w.y * scale : 0.f;
      w.z = drop_keep(seed, site, base + 2, thr) ? w.z * scale : 0.f;
      w.w = drop_keep(seed, site, base + 3, thr) ? w.w * scale : 0.f;
      if constexpr (sizeof(OUT) == 2) *reinterpret_cast<u32x2*>(dst + r * ldd + c) = bf16_rne4(w);
      else *reinterpret_cast<f32x4*>(dst + r * ldd + c) = w;
      pm = amax4(0.f, w);
    }
    am = fmaxf(am, pm);
    // each row's max |v| per 256-column part (a row is d / 4 consecutive lanes: groups of min(d / 4, 64) lanes; the
    // host checks the shape)
    if (rowmax) {
      const int gl = d / 4 < 64 ? d / 4 : 64;
      for (int o = gl / 2; o > 0; o >>= 1) pm = fmaxf(pm, __shfl_xor(pm, o, 64));
      if (r >= 0 && (c % 256) == 0) rowmax[r * rowmax_n + c / 256] = pm;
    }
  }
  if (amax) amax_flush(amax, am);
}

// out[r][j] = max |x[r][256 j .. 256 j + 255]|: one wave per (row, part), a float4 per lane
__global__ __launch_bounds__(256) void rows_absmax_kernel(const float* __restrict__ x, int64_t ldx, int64_t rows, int d,
                                                          float* out, int parts) {
  const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const int64_t r = w / parts;
  const int j = (int)(w % parts);
  const int c = 256 * j + 4 * lane;
  float m = 0.f;
  if (r < rows && c < d) m = amax4(0.f, *reinterpret_cast<const f32x4*>(x + r * ldx + c));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if (r < rows && lane == 0) out[r * parts + j] = m;
}

inline int tpr_for(int d) {
  int t = d / 4;
  int p = 1;
  while (p * 2 <= t && p * 2 <= 64) p *= 2;
  return p;
}

}  // namespace ot

using namespace ot;

extern "C" int ot_rmsnorm_fwd(const float* x, int64_t ldx, const float* gamma, float* y, int64_t ldy, float* rstd,
                              int64_t rows, int d, float eps, void* stream) {
  OT_REQUIRE(x && (rstd || y), "ot_rmsnorm_fwd: null operand");
  OT_REQUIRE(!y || gamma, "ot_rmsnorm_fwd: y needs gamma");
  OT_REQUIRE(d > 0 && d % 4 == 0 && ldx % 4 == 0 && (!y || ldy % 4 == 0), "ot_rmsnorm_fwd: d/ld must be multiples of 4");
  if (rows == 0) return OT_OK;
  const int tpr = tpr_for(d);
  hipLaunchKernelGGL(rmsnorm_fwd_kernel, dim3(ceil_div(rows, 256 / tpr)), dim3(256), 0, (hipStream_t)stream,
                     x, ldx, gamma, y, ldy, rstd, rows, d, eps, tpr);
  OT_LAUNCH_CHECK("ot_rmsnorm_fwd");
  return OT_OK;
}

inline unsigned rms_bwd_grid(int64_t rows, int d) {
  const int tpr = ot::tpr_for(d);
  unsigned g = ceil_div(rows, 256 / tpr);
  return g < 1024 ? g : 1024;
}

extern "C" size_t ot_rmsnorm_bwd_workspace_size(int64_t rows, int d) {
  const int64_t parts = rms_bwd_grid(rows, d);
  return (size_t)(parts * d + colsum_scratch_floats(parts, d)) * sizeof(float);
}

extern "C" int ot_rmsnorm_bwd(const float* dy, int64_t lddy, const float* x, int64_t ldx, const float* gamma,
                              const float* rstd, const float* dres, int64_t lddres, int dres_tail_K,
                              int dres_tail_I, const int32_t* dres_tail_inv, float* dx, int64_t lddx,
                              float* dx_masked, int64_t lddxm, uint32_t seed, uint32_t site, float drop_rate,
                              int tail_K, int tail_I, const int32_t* tail_pos, float* dgamma, int accumulate_dgamma, int64_t rows, int d,
                              void* workspace, size_t ws_bytes, void* stream) {
  OT_REQUIRE(dy && x && gamma && rstd && dx, "ot_rmsnorm_bwd: null operand");
  OT_REQUIRE(d % 4 == 0 && lddy % 4 == 0 && ldx % 4 == 0 && lddx % 4 == 0, "ot_rmsnorm_bwd: alignment");
  OT_REQUIRE(!dgamma || (workspace && ws_bytes >= ot_rmsnorm_bwd_workspace_size(rows, d)),
             "ot_rmsnorm_bwd: workspace too small");
  OT_REQUIRE(!dx_masked || (tail_K > 0 && tail_I >= tail_K), "ot_rmsnorm_bwd: bad tail map");
  if (rows == 0) return OT_OK;
  OT_REQUIRE(d <= 16 * tpr_for(d), "ot_rmsnorm_bwd: d=%d too large", d);
  const int tpr = tpr_for(d);
  const unsigned grid = rms_bwd_grid(rows, d);
  OT_REQUIRE(dres_tail_K == 0 || (dres_tail_K > 0 && dres_tail_I >= dres_tail_K), "ot_rmsnorm_bwd: bad dres tail");
  RmsBwdArgs p{dy, lddy, x, ldx, gamma, rstd, dres, lddres, dres_tail_K, dres_tail_I, dx, lddx, dx_masked, lddxm, seed, site,
               drop_threshold(drop_rate), drop_rate < 1.f ? 1.f / (1.f - drop_rate) : 0.f, tail_K, tail_I,
               dgamma ? (float*)workspace : nullptr, rows, d, tpr, tail_pos, dres_tail_inv};
  const size_t shmem = dgamma ? (size_t)(256 / tpr) * d * sizeof(float) : 0;
  OT_REQUIRE(shmem <= 65536, "ot_rmsnorm_bwd: d too large for the dgamma staging");
  hipLaunchKernelGGL(rmsnorm_bwd_kernel, dim3(grid), dim3(256), shmem, (hipStream_t)stream, p);
  OT_LAUNCH_CHECK("ot_rmsnorm_bwd");
  if (dgamma) {
    launch_colsum_reduce((const float*)workspace, (int64_t)grid, d, dgamma, accumulate_dgamma, (hipStream_t)stream,
                         (float*)workspace + (int64_t)grid * d);
    OT_LAUNCH_CHECK("ot_rmsnorm_bwd(reduce)");
  }
  return OT_OK;
}

namespace ot {
int64_t colsum_scratch_floats(int64_t nparts, int ncols) { return (int64_t)ceil_div(nparts, 64) * ncols; }

void launch_colsum_reduce(const float* part, int64_t nparts, int ncols, float* out, int accumulate, hipStream_t s,
                          float* scratch) {
  if (nparts > 256 && scratch) {          // two levels: 64-part chunks, then the chunk sums
    const unsigned nch = ceil_div(nparts, 64);
    hipLaunchKernelGGL(colsum_chunk_kernel, dim3(ceil_div(ncols, 64), nch), dim3(256), 0, s, part, nparts, ncols,
                       scratch);
    part = scratch;
    nparts = nch;
  }
  hipLaunchKernelGGL(colsum_reduce_kernel, dim3(ceil_div(ncols, 16)), dim3(256), 0, s, part, nparts, ncols, out,
                     accumulate);
}
}  // namespace ot

extern "C" int ot_dropout_apply(const float* src, int64_t lds, float* dst, int64_t ldd, int64_t rows, int d,
                                uint32_t seed, uint32_t site, float drop_rate, int tail_K, int tail_I,
                                const int32_t* tail_pos, void* stream) {
  OT_REQUIRE(src && dst && d % 4 == 0 && lds % 4 == 0 && ldd % 4 == 0, "ot_dropout_apply: bad args");
  OT_REQUIRE(tail_K > 0 && tail_I >= tail_K, "ot_dropout_apply: bad tail map");
  if (rows == 0) return OT_OK;
  hipLaunchKernelGGL(dropout_apply_kernel<float>, dim3(ceil_div(ceil_div(rows * d / 4, DROPOUT_PASSES), 256)), dim3(256), 0, (hipStream_t)stream,
                     src, lds, dst, ldd, rows, d, seed, site, drop_threshold(drop_rate),
                     drop_rate < 1.f ? 1.f / (1.f - drop_rate) : 0.f, tail_K, tail_I, tail_pos, nullptr, nullptr, 0);
  OT_LAUNCH_CHECK("ot_dropout_apply");
  return OT_OK;
}

extern "C" int ot_dropout_apply_ex(const float* src, int64_t lds, float* dst, int64_t ldd, int64_t rows, int d,
                                   uint32_t seed, uint32_t site, float drop_rate, int tail_K, int tail_I,
                                   const int32_t* tail_pos, float* amax, float* rowmax, int rowmax_n, void* stream) {
  OT_REQUIRE(src && dst && d % 4 == 0 && lds % 4 == 0 && ldd % 4 == 0, "ot_dropout_apply_ex: bad args");
  OT_REQUIRE(tail_K > 0 && tail_I >= tail_K, "ot_dropout_apply_ex: bad tail map");
  const int q = d / 4;
  OT_REQUIRE(!rowmax || (rowmax_n == (d + 255) / 256 && (q % 64 == 0 || (q & (q - 1)) == 0)),
             "ot_dropout_apply_ex: rowmax needs rowmax_n == ceil(d / 256) and d / 4 a power of two or a multiple of 64");
  if (rows == 0) return OT_OK;
  hipLaunchKernelGGL(dropout_apply_kernel<float>, dim3(ceil_div(ceil_div(rows * d / 4, DROPOUT_PASSES), 256)), dim3(256), 0, (hipStream_t)stream,
                     src, lds, dst, ldd, rows, d, seed, site, drop_threshold(drop_rate),
                     drop_rate < 1.f ? 1.f / (1.f - drop_rate) : 0.f, tail_K, tail_I, tail_pos, amax, rowmax, rowmax_n);
  OT_LAUNCH_CHECK("ot_dropout_apply_ex");
  return OT_OK;
}

extern "C" int ot_rows_absmax(const float* x, int64_t ldx, int64_t rows, int d, float* out, int parts,
                              void* stream) {
  OT_REQUIRE(x && out && d % 4 == 0 && ldx % 4 == 0 && parts == (d + 255) / 256,
             "ot_rows_absmax: bad args (d %% 4 == 0, parts == ceil(d / 256))");
  if (rows == 0) return OT_OK;
  hipLaunchKernelGGL(rows_absmax_kernel, dim3(ceil_div(rows * parts, 4)), dim3(256), 0, (hipStream_t)stream, x, ldx,
                     rows, d, out, parts);
  OT_LAUNCH_CHECK("ot_rows_absmax");
  return OT_OK;
}

extern "C" int ot_dropout_apply_bf16(const float* src, int64_t lds, uint16_t* dst, int64_t ldd, int64_t rows, int d,
                                     uint32_t seed, uint32_t site, float drop_rate, int tail_K, int tail_I,
                                     const int32_t* tail_pos, void* stream) {
  OT_REQUIRE(src && dst && d % 4 == 0 && lds % 4 == 0 && ldd % 4 == 0 && ((uintptr_t)dst % 8) == 0,
             "ot_dropout_apply_bf16: bad args");
  OT_REQUIRE(tail_K > 0 && tail_I >= tail_K, "ot_dropout_apply_bf16: bad tail map");
  if (rows == 0) return OT_OK;
  hipLaunchKernelGGL(dropout_apply_kernel<uint16_t>, dim3(ceil_div(ceil_div(rows * d / 4, DROPOUT_PASSES), 256)), dim3(256), 0,
                     (hipStream_t)stream, src, lds, dst, ldd, rows, d, seed, site, drop_threshold(drop_rate),
                     drop_rate < 1.f ? 1.f / (1.f - drop_rate) : 0.f, tail_K, tail_I, tail_pos, nullptr, nullptr, 0);
  OT_LAUNCH_CHECK("ot_dropout_apply_bf16");
  return OT_OK;
}

// rows per partial sum of ot_rows_colsum: short serial chains (each step an index load, then a row
// load) and hundreds of blocks; 256 rows per block left the [SEP] gradient (8192 rows at C2) at 32
// latency-bound blocks, 116 us
constexpr int COLSUM_ROWS = 32;

extern "C" size_t ot_rows_colsum_workspace_size(int64_t nrows, int ncols) {
  const int64_t parts = ceil_div(nrows, COLSUM_ROWS);
  return (size_t)(parts * ncols + colsum_scratch_floats(parts, ncols)) * sizeof(float);
}

extern "C" int ot_rows_colsum(const float* src, int64_t ld, const int32_t* rows, int64_t nrows, int ncols,
                              float* out, int accumulate, void* workspace, size_t ws_bytes, void* stream) {
  OT_REQUIRE(src && out && ncols > 0, "ot_rows_colsum: bad args");
  OT_REQUIRE(workspace && ws_bytes >= ot_rows_colsum_workspace_size(nrows, ncols), "ot_rows_colsum: workspace");
  const unsigned nb = ceil_div(nrows, COLSUM_ROWS);
  if (nb > 0) {
    const int tpb = ncols >= 256 ? 256 : (int)ceil_div((int64_t)ncols, 64) * 64;
    hipLaunchKernelGGL(rows_colsum_kernel, dim3(ceil_div(ncols, tpb), nb), dim3(tpb), 0, (hipStream_t)stream,
                       src, ld, rows, nrows, ncols, COLSUM_ROWS, (float*)workspace);
    OT_LAUNCH_CHECK("ot_rows_colsum");
  }
  launch_colsum_reduce((const float*)workspace, (int64_t)nb, ncols, out, accumulate, (hipStream_t)stream,
                       (float*)workspace + (int64_t)nb * ncols);
  OT_LAUNCH_CHECK("ot_rows_colsum(reduce)");
  return OT_OK;
}
