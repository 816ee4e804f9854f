// Mixed-parameterisation grouped GEMM on gfx950 fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces the reference's per-token Dense loops (model.py:84-92 Q/K/V, model.py:154-161 FFN),
// the Wo Dense (model.py:117), the tokenizer Dense layers (model.py:211-219) and their
// gradients.  One launch covers every weight group: rows are listed per tile (row maps), every
// tile belongs to one group g and multiplies by W[g].
//
//   fwd  (NN): C[out_row] = epi( pro(A[in_row]) @ W[g] )          W[g] stored [K][N] (Keras)
//   dgrad(NT): C[out_row] = epi( A[in_row] @ W[g]^T )             W[g] stored [N][K]
//   wgrad    : dW[g] (+)= sum_rows pro(A[a_row])^T D[d_row], db[g] (+)= sum_rows D[d_row]
//
// Tile 128x128, BK 32, 256 threads = 4 waves (2x2), each wave 64x64 = 2x2 MFMA 32x32 blocks.
// LDS images are [row][BK+4] (k contiguous, 144-B row stride => conflict-free ds_read_b128 for
// 16 consecutive rows).  The k index inside an MFMA step is permuted (lane half h supplies
// k = 16h + s at step s) so each lane reads 4 consecutive k with one ds_read_b128.
#include <mutex>

#include "common.h"

namespace ot {

constexpr int GT = 128;        // tile rows / cols
constexpr int GBK = 32;        // k per LDS stage
constexpr int GLD = GBK + 4;   // LDS row stride (floats)

struct GemmArgs {
  const float* A; int64_t lda; int K;
  const int32_t* in_rows;                       // [ntm*GT] or null (identity)
  int a_xform; const float* a_rstd; const float* a_gamma;
  const float* W; int64_t w_gstride; int64_t ldw; int N;
  const int32_t* tile_group;                    // [ntm] or null (group 0)
  const float* bias; int64_t bias_gstride;
  float* C; int64_t ldc; const int32_t* out_rows;
  int epi;
  const float* res; int64_t ldres; int res_tok;
  const float* aux; int64_t ldaux;
  uint32_t seed, site, drop_thr; float drop_scale; int tail_K, tail_I; int drop_width;
  int ntm, ntn;
};

__device__ __forceinline__ f32x4 apply_pro(f32x4 v, int xf, float rs, const float* gamma, int k) {
  if (xf == OT_AX_RMSNORM) {
    v.x *= rs * gamma[k]; v.y *= rs * gamma[k + 1]; v.z *= rs * gamma[k + 2]; v.w *= rs * gamma[k + 3];
  } else if (xf == OT_AX_GELU) {
    v.x = gelu_erf(v.x); v.y = gelu_erf(v.y); v.z = gelu_erf(v.z); v.w = gelu_erf(v.w);
  }
  return v;
}

// XCD-aware bijective remap (cdna_hip_programming.md T1): blocks b and b+8 share an XCD, so give
// each XCD a contiguous range of tiles (the N tiles of one M tile then share that XCD's L2).
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
  int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (b >> 3);
}

template <bool NT>
__global__ __launch_bounds__(256, 2) void mixed_gemm_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* As = smem;                      // [2][GT][GLD]
  float* Bs = smem + 2 * GT * GLD;       // [2][GT][GLD]

  const int nwg = p.ntm * p.ntn;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int tm = wg / p.ntn, tn = wg % p.ntn;
  const int g = p.tile_group ? p.tile_group[tm] : 0;
  const float* W = p.W + (int64_t)g * p.w_gstride;
  const int n0 = tn * GT;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;

  // ---- per-thread staging coordinates
  // A / NT-B: row = (t>>3) + 32*i (i<4), float4 column c = t&7
  const int sc = t & 7, sr = t >> 3;
  int64_t a_off[4]; float a_rs[4]; bool a_ok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int r = sr + 32 * i;
    int64_t gr = (int64_t)tm * GT + r;
    int ir = p.in_rows ? p.in_rows[gr] : (int)gr;
    a_ok[i] = ir >= 0;
    a_off[i] = (int64_t)(ir < 0 ? 0 : ir) * p.lda;
    a_rs[i] = (p.a_xform == OT_AX_RMSNORM && ir >= 0) ? p.a_rstd[ir] : 1.f;
  }
  // NN-B: kk = lane&31, n4 = 2*wave + (lane>>5) + 8*i (i<4)
  f32x4 ra[4], rb[4];

  auto load_stage = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int k = k0 + 4 * sc;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (a_ok[i] && k < p.K) {
        v = *reinterpret_cast<const f32x4*>(p.A + a_off[i] + k);
        v = apply_pro(v, p.a_xform, a_rs[i], p.a_gamma, k);
      }
      ra[i] = v;
    }
    if (NT) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int n = n0 + sr + 32 * i, k = k0 + 4 * sc;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (n < p.N && k < p.K) v = *reinterpret_cast<const f32x4*>(W + (int64_t)n * p.ldw + k);
        rb[i] = v;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int k = k0 + li, n = n0 + 4 * (2 * wave + h + 8 * i);
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (k < p.K && n < p.N) v = *reinterpret_cast<const f32x4*>(W + (int64_t)k * p.ldw + n);
        rb[i] = v;
      }
    }
  };
  auto store_stage = [&](int buf) {
    float* as = As + buf * GT * GLD;
    float* bs = Bs + buf * GT * GLD;
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<f32x4*>(as + (sr + 32 * i) * GLD + 4 * sc) = ra[i];
    if (NT) {
#pragma unroll
      for (int i = 0; i < 4; ++i) *reinterpret_cast<f32x4*>(bs + (sr + 32 * i) * GLD + 4 * sc) = rb[i];
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int n = 4 * (2 * wave + h + 8 * i);
        bs[(n + 0) * GLD + li] = rb[i].x;
        bs[(n + 1) * GLD + li] = rb[i].y;
        bs[(n + 2) * GLD + li] = rb[i].z;
        bs[(n + 3) * GLD + li] = rb[i].w;
      }
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int nk = (p.K + GBK - 1) / GBK;
  load_stage(0);
  store_stage(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_stage((kt + 1) * GBK);
    const float* as = As + cur * GT * GLD;
    const float* bs = Bs + cur * GT * GLD;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      f32x4 fa[2][2], fb[2][2];
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          fa[m][q] = *reinterpret_cast<const f32x4*>(as + (wm + 32 * m + li) * GLD + 16 * h + 8 * half + 4 * q);
          fb[m][q] = *reinterpret_cast<const f32x4*>(bs + (wn + 32 * m + li) * GLD + 16 * h + 8 * half + 4 * q);
        }
#pragma unroll
      for (int s = 0; s < 8; ++s) {
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int n = 0; n < 2; ++n)
            acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[m][s >> 2][s & 3], fb[n][s >> 2][s & 3],
                                                             acc[m][n], 0, 0, 0);
      }
    }
    if (kt + 1 < nk) {
      __syncthreads();               // everyone finished reading buf cur^1 (previous iteration)
      store_stage(cur ^ 1);
      __syncthreads();
    }
  }

  // ---- epilogue
#pragma unroll
  for (int m = 0; m < 2; ++m) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = wm + 32 * m + (r & 3) + 8 * (r >> 2) + 4 * h;
      const int64_t gr = (int64_t)tm * GT + row;
      const int orow = p.out_rows ? p.out_rows[gr] : (int)gr;
      if (orow < 0) continue;
      const int64_t tok = (p.epi & (OT_EPI_DROPOUT)) || p.res_tok ? tail_token(orow, p.tail_K, p.tail_I) : orow;
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int col = n0 + wn + 32 * n + li;
        if (col >= p.N) continue;
        float v = acc[m][n][r];
        if (p.epi & OT_EPI_BIAS) v += p.bias[(int64_t)g * p.bias_gstride + col];
        if (p.epi & OT_EPI_GELU_BWD) v *= gelu_erf_grad(p.aux[(int64_t)orow * p.ldaux + col]);
        if (p.epi & OT_EPI_GELU) v = gelu_erf(v);
        if (p.epi & OT_EPI_DROPOUT) {
          uint32_t idx = (uint32_t)(tok * p.drop_width + col);
          v = drop_keep(p.seed, p.site, idx, p.drop_thr) ? v * p.drop_scale : 0.f;
        }
        if (p.epi & OT_EPI_RESIDUAL) v += p.res[(p.res_tok ? tok : (int64_t)orow) * p.ldres + col];
        float* dst = p.C + (int64_t)orow * p.ldc + col;
        if (p.epi & OT_EPI_ACCUMULATE) v += *dst;
        *dst = v;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// wgrad: partial slab per (chunk, k-tile, n-tile):  slab[c][k][n] = sum_{rows of chunk} A^T D
// LDS images: As[k][r] and Ds[n][r] (r contiguous, BR = 32 rows per stage).
constexpr int WBR = 32;
constexpr int WLD = WBR + 4;

struct WgradArgs {
  const float* A; int64_t lda; const int32_t* a_rows; int a_xform; const float* a_rstd; const float* a_gamma;
  const float* D; int64_t ldd; const int32_t* d_rows;
  int K, N;
  const int32_t* chunks;     // [nchunks*3] {group, row_begin, row_count} (rows index the row maps)
  int nchunks;
  float* slab;               // [nchunks][K][N]
  float* bslab;              // [nchunks][N] or null
  int ntk, ntn;
};

__global__ __launch_bounds__(256, 2) void wgrad_kernel(WgradArgs p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* As = smem;                 // [GT][WLD]  (k, r)
  float* Ds = smem + GT * WLD;      // [GT][WLD]  (n, r)
  const int per_chunk = p.ntk * p.ntn;
  const int c = blockIdx.x / per_chunk;
  const int rem = blockIdx.x % per_chunk;
  const int tk = rem / p.ntn, tn = rem % p.ntn;
  const int k0 = tk * GT, n0 = tn * GT;
  const int row_begin = p.chunks[3 * c + 1], row_count = p.chunks[3 * c + 2];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  // staging: row r = t>>3 (0..31), float4 column sc = t&7 (+ 8*i, i<4) covering 128 columns
  const int sr = t >> 3, sc = t & 7;

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  float bsum = 0.f;
  const bool do_bias = p.bslab && tk == 0 && t < GT;

  for (int rs = 0; rs < row_count; rs += WBR) {
    // load A rows and D rows of this stage into registers
    const int lr = rs + sr;
    int ar = -1, dr = -1;
    if (lr < row_count) {
      int64_t mi = (int64_t)row_begin + lr;
      ar = p.a_rows ? p.a_rows[mi] : (int)mi;
      dr = p.d_rows ? p.d_rows[mi] : (int)mi;
    }
    if (ar < 0 || dr < 0) { ar = -1; dr = -1; }
    float rsd = (p.a_xform == OT_AX_RMSNORM && ar >= 0) ? p.a_rstd[ar] : 1.f;
    f32x4 va[4], vd[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int k = k0 + 4 * (sc + 8 * i), n = n0 + 4 * (sc + 8 * i);
      f32x4 z = {0.f, 0.f, 0.f, 0.f};
      va[i] = z; vd[i] = z;
      if (ar >= 0 && k < p.K) {
        va[i] = *reinterpret_cast<const f32x4*>(p.A + (int64_t)ar * p.lda + k);
        va[i] = apply_pro(va[i], p.a_xform, rsd, p.a_gamma, k);
      }
      if (dr >= 0 && n < p.N) vd[i] = *reinterpret_cast<const f32x4*>(p.D + (int64_t)dr * p.ldd + n);
    }
    __syncthreads();   // previous stage fully consumed
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int kk = 4 * (sc + 8 * i);
      As[(kk + 0) * WLD + sr] = va[i].x; As[(kk + 1) * WLD + sr] = va[i].y;
      As[(kk + 2) * WLD + sr] = va[i].z; As[(kk + 3) * WLD + sr] = va[i].w;
      Ds[(kk + 0) * WLD + sr] = vd[i].x; Ds[(kk + 1) * WLD + sr] = vd[i].y;
      Ds[(kk + 2) * WLD + sr] = vd[i].z; Ds[(kk + 3) * WLD + sr] = vd[i].w;
    }
    __syncthreads();
    if (do_bias) {
#pragma unroll
      for (int q = 0; q < WBR; q += 4) {
        f32x4 v = *reinterpret_cast<const f32x4*>(Ds + t * WLD + q);
        bsum += (v.x + v.y) + (v.z + v.w);
      }
    }
    // 16 MFMA k-steps over the 32 rows: lane half h supplies row 16h + s
    f32x4 fa[2][4], fb[2][4];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        fa[m][q] = *reinterpret_cast<const f32x4*>(As + (wm + 32 * m + li) * WLD + 16 * h + 4 * q);
        fb[m][q] = *reinterpret_cast<const f32x4*>(Ds + (wn + 32 * m + li) * WLD + 16 * h + 4 * q);
      }
#pragma unroll
    for (int s = 0; s < 16; ++s)
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[m][s >> 2][s & 3], fb[n][s >> 2][s & 3],
                                                           acc[m][n], 0, 0, 0);
  }
  float* slab = p.slab + (int64_t)c * p.K * p.N;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int k = k0 + wm + 32 * m + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (k >= p.K) continue;
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int col = n0 + wn + 32 * n + li;
        if (col < p.N) slab[(int64_t)k * p.N + col] = acc[m][n][r];
      }
    }
  if (do_bias && n0 + t < p.N) p.bslab[(int64_t)c * p.N + n0 + t] = bsum;
}

// Sum the slabs of each group's chunks (chunks of one group are contiguous) into dW[g] (and db).
__global__ void wgrad_reduce_kernel(const float* __restrict__ slab, const float* __restrict__ bslab,
                                    const int32_t* __restrict__ chunks, const int32_t* __restrict__ gchunk,
                                    int ngroups, int K, int N, float* dW, int64_t dw_gstride,
                                    float* db, int64_t db_gstride, int accumulate) {
  const int g = blockIdx.y;
  const int cb = gchunk[2 * g], cn = gchunk[2 * g + 1];
  const int64_t KN = (int64_t)K * N;
  const int64_t i4 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i4 < KN) {
    // a group with no rows (e.g. dedicated groups outside a 1-token tail) has a zero gradient
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    for (int c = cb; c < cb + cn; ++c) s += *reinterpret_cast<const f32x4*>(slab + (int64_t)c * KN + i4);
    float* dst = dW + (int64_t)g * dw_gstride + i4;
    if (accumulate) s += *reinterpret_cast<const f32x4*>(dst);
    *reinterpret_cast<f32x4*>(dst) = s;
  }
  if (db && blockIdx.x == 0) {
    for (int n = threadIdx.x; n < N; n += blockDim.x) {
      float s = 0.f;
      if (bslab)
        for (int c = cb; c < cb + cn; ++c) s += bslab[(int64_t)c * N + n];
      float* dst = db + (int64_t)g * db_gstride + n;
      *dst = accumulate ? *dst + s : s;
    }
  }
}

}  // namespace ot

using namespace ot;

extern "C" int ot_mixed_gemm(int mode, const float* A, int64_t lda, int K, const int32_t* in_rows,
                             int a_xform, const float* a_rstd, const float* a_gamma,
                             const float* W, int64_t w_gstride, int64_t ldw, int N,
                             const int32_t* tile_group, int ntiles,
                             const float* bias, int64_t bias_gstride,
                             float* C, int64_t ldc, const int32_t* out_rows, int epi,
                             const float* res, int64_t ldres, int res_tok,
                             const float* aux, int64_t ldaux,
                             uint32_t seed, uint32_t site, float drop_rate, int tail_K, int tail_I,
                             void* stream) {
  OT_REQUIRE(A && W && C, "ot_mixed_gemm: null operand");
  OT_REQUIRE(K > 0 && N > 0 && ntiles >= 0, "ot_mixed_gemm: bad sizes K=%d N=%d ntiles=%d", K, N, ntiles);
  OT_REQUIRE(K % 4 == 0 && lda % 4 == 0, "ot_mixed_gemm: K and lda must be multiples of 4");
  OT_REQUIRE(ldw % 4 == 0 && w_gstride % 4 == 0, "ot_mixed_gemm: ldw/w_gstride must be multiples of 4");
  OT_REQUIRE(mode == OT_GEMM_NN ? N % 4 == 0 : true, "ot_mixed_gemm: NN mode needs N %% 4 == 0");
  OT_REQUIRE(mode == OT_GEMM_NN || mode == OT_GEMM_NT, "ot_mixed_gemm: bad mode");
  OT_REQUIRE(!(epi & OT_EPI_BIAS) || bias, "ot_mixed_gemm: bias missing");
  OT_REQUIRE(!(epi & OT_EPI_RESIDUAL) || res, "ot_mixed_gemm: residual missing");
  OT_REQUIRE(!(epi & OT_EPI_GELU_BWD) || aux, "ot_mixed_gemm: aux missing");
  OT_REQUIRE(a_xform != OT_AX_RMSNORM || (a_rstd && a_gamma), "ot_mixed_gemm: rmsnorm prologue needs rstd/gamma");
  OT_REQUIRE(!((epi & OT_EPI_DROPOUT) || res_tok) || (tail_K > 0 && tail_I >= tail_K), "ot_mixed_gemm: bad tail map");
  if (ntiles == 0) return OT_OK;
  GemmArgs p{A, lda, K, in_rows, a_xform, a_rstd, a_gamma, W, w_gstride, ldw, N, tile_group,
             bias, bias_gstride, C, ldc, out_rows, epi, res, ldres, res_tok, aux, ldaux,
             seed, site, 0u, 1.f, tail_K, tail_I, N, ntiles, (int)ceil_div(N, GT)};
  if (epi & OT_EPI_DROPOUT) {
    OT_REQUIRE(drop_rate >= 0.f && drop_rate < 1.f, "ot_mixed_gemm: drop_rate out of range");
    p.drop_thr = drop_threshold(drop_rate);
    p.drop_scale = 1.f / (1.f - drop_rate);
  }
  const size_t shmem = 4 * GT * GLD * sizeof(float);
  static std::once_flag once;   // LDS > 64 KiB per workgroup (gfx950 has 160 KiB per CU)
  std::call_once(once, [] {
    constexpr int shmem = 4 * GT * GLD * sizeof(float);
    (void)hipFuncSetAttribute((const void*)mixed_gemm_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, shmem);
    (void)hipFuncSetAttribute((const void*)mixed_gemm_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, shmem);
    (void)hipGetLastError();
  });
  const unsigned nwg = (unsigned)ntiles * p.ntn;
  hipStream_t s = (hipStream_t)stream;
  if (mode == OT_GEMM_NN)
    hipLaunchKernelGGL(mixed_gemm_kernel<false>, dim3(nwg), dim3(256), shmem, s, p);
  else
    hipLaunchKernelGGL(mixed_gemm_kernel<true>, dim3(nwg), dim3(256), shmem, s, p);
  OT_LAUNCH_CHECK("ot_mixed_gemm");
  return OT_OK;
}

extern "C" size_t ot_wgrad_workspace_size(int nchunks, int K, int N) {
  return ((size_t)nchunks * K * N + (size_t)nchunks * N) * sizeof(float);
}

extern "C" int ot_mixed_gemm_wgrad(const float* A, int64_t lda, const int32_t* a_rows, int a_xform,
                                   const float* a_rstd, const float* a_gamma,
                                   const float* D, int64_t ldd, const int32_t* d_rows, int K, int N,
                                   const int32_t* chunks, int nchunks, const int32_t* gchunk, int ngroups,
                                   float* dW, int64_t dw_gstride, float* db, int64_t db_gstride,
                                   int accumulate, void* workspace, size_t ws_bytes, void* stream) {
  OT_REQUIRE(A && D && dW && chunks && gchunk && workspace, "ot_mixed_gemm_wgrad: null operand");
  OT_REQUIRE(K % 4 == 0 && N % 4 == 0 && lda % 4 == 0 && ldd % 4 == 0 && dw_gstride % 4 == 0,
             "ot_mixed_gemm_wgrad: K, N, lda, ldd, dw_gstride must be multiples of 4");
  OT_REQUIRE(ws_bytes >= ot_wgrad_workspace_size(nchunks, K, N), "ot_mixed_gemm_wgrad: workspace too small");
  OT_REQUIRE(a_xform != OT_AX_RMSNORM || (a_rstd && a_gamma), "ot_mixed_gemm_wgrad: rmsnorm prologue needs rstd/gamma");
  hipStream_t s = (hipStream_t)stream;
  float* slab = (float*)workspace;
  float* bslab = db ? slab + (size_t)nchunks * K * N : nullptr;
  if (nchunks > 0) {
    WgradArgs p{A, lda, a_rows, a_xform, a_rstd, a_gamma, D, ldd, d_rows, K, N, chunks, nchunks, slab, bslab,
                (int)ceil_div(K, GT), (int)ceil_div(N, GT)};
    const size_t shmem = 2 * GT * WLD * sizeof(float);
    hipLaunchKernelGGL(wgrad_kernel, dim3((unsigned)nchunks * p.ntk * p.ntn), dim3(256), shmem, s, p);
    OT_LAUNCH_CHECK("ot_mixed_gemm_wgrad");
  }
  dim3 rg(ceil_div((int64_t)K * N / 4, 256), ngroups);
  hipLaunchKernelGGL(wgrad_reduce_kernel, rg, dim3(256), 0, s, slab, bslab, chunks, gchunk, ngroups, K, N,
                     dW, dw_gstride, db, db_gstride, accumulate);
  OT_LAUNCH_CHECK("ot_mixed_gemm_wgrad(reduce)");
  return OT_OK;
}
