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
#include <algorithm>
#include <cstdlib>
#include <atomic>
#include <mutex>

#include "common.h"

namespace ot {

#ifndef OT_GEMM_BK
#define OT_GEMM_BK 16
#endif
#ifndef OT_GEMM_MINWG
#define OT_GEMM_MINWG 3
#endif
#ifndef OT_GEMM_PRIO
#define OT_GEMM_PRIO 0
#endif
#ifndef OT_GEMM_RMS_EARLY
#define OT_GEMM_RMS_EARLY 1
#endif
#ifndef OT_PLANE_BF16_NSTG         // stage buffers of the bf16-mode plane GEMM (3: 4 workgroups / CU)
#define OT_PLANE_BF16_NSTG 3
#endif
constexpr int PLANE_BF16_NSTG = OT_PLANE_BF16_NSTG;
#ifndef OT_PLANE_EPI_RBN          // epilogue rows per operand-load batch of the 4-workgroup plane GEMMs
#define OT_PLANE_EPI_RBN 4
#endif
#ifndef OT_WGRAD_BF16_RS          // 32-row groups per stage of the bf16-mode weight-gradient kernel
#define OT_WGRAD_BF16_RS 2
#endif
constexpr int WGRAD_BF16_RS = OT_WGRAD_BF16_RS;
#ifndef OT_WGRAD_DBUF
#define OT_WGRAD_DBUF 0
#endif
constexpr int GT = 128;           // tile rows / cols
constexpr int GBK = OT_GEMM_BK;   // k per LDS stage (16 or 32)
constexpr int GLD = GBK + 4;      // LDS row stride (floats)

// Split-bf16 MFMA (OT_GEMM_SPLIT = number of product terms, 0 = native f32 MFMA).  Every f32
// operand is split exactly into three bf16 pieces x = x0 + x1 + x2 (x0 = top 8 significant bits,
// x1 the next 8, x2 the last 8; truncation keeps every step exact), and a.b = sum_ij ai.bj with
// each bf16 x bf16 product exact in the f32 accumulator of v_mfma_f32_32x32x16_bf16 (32 cycles per
// 32x32x16 against 64 cycles per 32x32x2 for the f32 form: 16x the rate).  9 terms = every
// product (the f32 result up to accumulation order); 6 terms drop a1.b2, a2.b1, a2.b2, whose sum
// is below 2^-22 |a||b| — the size of one f32 rounding of the product.
#ifndef OT_GEMM_SPLIT
#define OT_GEMM_SPLIT 6           // product terms of the split kernels (6 or 9; 3 is not f32-accurate)
#endif
#ifndef OT_GEMM_SPLIT_SCHED
#define OT_GEMM_SPLIT_SCHED 0     // >0: interleave this many VALU ops after each MFMA (sched_group_barrier)
#endif
#ifndef OT_GEMM_NT_STORE
#define OT_GEMM_NT_STORE 1        // epilogue output rows written with non-temporal (streaming) stores
                                  // (C2 +0.5%, T +0.5%: profiles/r02/gemm_nt_store.txt); 0: plain stores
#endif
constexpr int SPLIT_TERMS = OT_GEMM_SPLIT;
constexpr int SRS = 3 * 16 + 8;   // split LDS row stride (ushorts): 3 planes x 16 k + pad = 112 B
static_assert(SPLIT_TERMS == 3 || SPLIT_TERMS == 6 || SPLIT_TERMS == 9, "OT_GEMM_SPLIT");
// SPLT template argument of the split kernels: 0 = native f32 MFMA, SPLIT_TERMS = split-bf16,
// 1 = OT_MATMUL_BF16 (one bf16 plane rounded to nearest: bf16 MFMA on f32 data, f32 accumulation)
static_assert(GBK == 16, "split-bf16 staging assumes 16-k stages");

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
  // row-norm epilogues (N == GT: the tile holds whole rows; OT_EPI_ROW_RSTD also N > GT on the plane
  // GEMM: per-tile row sums of squares in rowpart, finished by row_rstd_finish_kernel)
  float* rstd_out; float eps;                                   // OT_EPI_ROW_RSTD
  const float* nx; int64_t ldnx; const float* ngamma; const float* nrstd;   // OT_EPI_RMSNORM_BWD
  const float* dres; int64_t lddres; int dres_K, dres_I; const int32_t* dres_inv;
  float* dxm; int64_t lddxm; float* dgpart;
  float* rowpart;                               // OT_EPI_ROW_RSTD with N > GT: [ntm*GT][ntn] row sums of squares
  float* rowdot; int rowdot_n;                  // OT_EPI_ROWDOT output / OT_EPI_RMSNORM_BWD (N > GT) input
  uint16_t* gelu_out; int64_t ldgelu;           // bf16 gelu_erf(aux) with OT_EPI_GELU_BWD, bf16 gelu_erf(C) with
                                                // epi == OT_EPI_BIAS (optional)
  const int32_t* tail_pos;                      // kept positions (ot_pyramid_select) or null (tail)
  // plane GEMM: pre-split B image (ot_split_images), its tiles per group and the first tile used
  const uint16_t* bimg; int bimg_ntn, bimg_tn0;
  // plane GEMM with the RMSNorm prologue: the first column tile's workgroups also store bf16(a * gamma * rstd)
  // of their A rows (the bf16 weight gradient's normalised A operand)
  uint16_t* xn_out; int64_t ldxn;
  uint16_t* c16_out; int64_t ldc16;             // bf16-mode plane GEMM: also C rounded to bf16 (optional)
  float* rowmax_out; int rowmax_n;              // split plane GEMM: per (out row, column tile) max of C after bias
  const float* a_rowmax; int a_rowmax_n;        // split plane GEMM, GELU prologue: A's row maxima (pair arithmetic)
  float* amax_out;                              // vector epilogue: atomic max of |stored output| (pair wgrad bound)
  float* rowabs_out; int rowabs_n;              // vector epilogue: per (out row, column tile) max |stored output|
};

// sum over the 32 lanes that hold one output row in the vector epilogue (same order as the
// row-wise kernels' group_sum with 32 threads per row)
// max over the 32 lanes that hold one output row (the vector epilogue's row maxima): within each 16-lane row by
// DPP (quad swaps, half-row and row mirrors), then across the two rows by v_permlane16_swap — VALU only, where
// five __shfl_xor steps were five ds_bpermute LDS round trips per row (max is order-free: the same result)
__device__ __forceinline__ float row32_max(float v) {
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false)));   // quad [1,0,3,2]
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false)));   // quad [2,3,0,1]
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false)));  // row_half_mirror
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false)));  // row_mirror
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
}
__device__ __forceinline__ float row32_sum(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ f32x4 apply_pro(f32x4 v, int xf, float rs, const float* gamma, int k) {
  if (xf == OT_AX_RMSNORM) {
    v.x *= rs * gamma[k]; v.y *= rs * gamma[k + 1]; v.z *= rs * gamma[k + 2]; v.w *= rs * gamma[k + 3];
  } else if (xf == OT_AX_GELU) {
    v = gelu_erf4(v);
  }
  return v;
}


// Weight-gradient tiles: whole row chunks per XCD.  Block b runs on XCD b % 8 (round-robin dispatch), so XCD x
// takes chunks x, x + 8, x + 16, ... and each chunk's (k, n) tiles occupy consecutive dispatch slots of that XCD:
// every tile of a chunk streams the same rows, and they are then read through one L2.  (The contiguous-range
// remap split chunks across two XCDs whenever a range was not a whole number of chunks: C5's W1 weight gradient
// fetched 2.3x its algorithmic bytes.)  The grid is padded to whole rounds of 8 chunks; padding blocks return.
// Fewer than 8 chunks (small batches): whole chunks per XCD would leave XCDs idle, so the tiles are dealt in
// order (block b = chunk b / per_chunk), spread over every XCD; the grid is then nchunks x per_chunk.
__host__ __device__ inline unsigned wgrad_grid(int nchunks, int per_chunk) {
  return (unsigned)(nchunks < 8 ? nchunks : (nchunks + 7) / 8 * 8) * per_chunk;
}
__device__ __forceinline__ bool wgrad_tile(int b, int per_chunk, int nchunks, int& c, int& rem) {
  if (nchunks < 8) {
    c = b / per_chunk;
    rem = b % per_chunk;
    return true;
  }
  const int x = b & 7, j = b >> 3;
  c = x + 8 * (j / per_chunk);
  rem = j % per_chunk;
  return c < nchunks;
}

// ---- vector epilogue shared by the GEMM kernels (compile-time flags EPIT >= 0, no edge tiles): the
// accumulator tile goes through LDS (the staging buffers are free: the caller's last barrier ended
// every main-loop read) in two 64-row halves; each thread then finishes 8 rows x one float4 column
// chunk, so every global access is a 16-B piece of a 512-B row run and each row index is loaded once
// per row instead of once per element.  Operand loads of a batch of rows are issued together.
// LAYOUT 0: 2x2 waves, acc[2m + n] = rows 64 (wave >> 1) + 32 m, cols 64 (wave & 1) + 32 n;
// LAYOUT 1: 4x1 waves, acc[nb] = rows 32 wave, cols 32 nb; LAYOUT 2 (a 128-column half `sub` of a 256-column
// tile held by 2x2 waves): wave 2 r + sub holds rows 64 r + 32 m, cols 32 nb in acc[4 m + nb]; LAYOUT 3 (128-column
// quarter `sub` of a 512-column tile): wave `sub` holds all 128 rows, rows 32 m / cols 32 nb in acc[4 m + nb];
// LAYOUT 4 (128-column half `sub` of a 256 x 256 tile's row half, the epilogue run by that row half's four waves
// with thread ids `tid` 0..255): wave 2 sub + j holds all 128 rows x columns 64 j + 32 nb in acc[2 m + nb].
// ROWSCALE: multiply row r by
// a_rstd[in_rows[r]] first (the plane GEMM's RMSNorm prologue, folded into the weights).
__device__ __forceinline__ void store_out4(float* dst, f32x4 v) {
  if (OT_GEMM_NT_STORE) __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(dst));
  else *reinterpret_cast<f32x4*>(dst) = v;
}
// four values rounded to bf16 (8 B), streamed like store_out4: the bf16-mode outputs (C, gelu(U), the bf16
// residual copies) are the bulk of those GEMMs' traffic, and written through the L2 they evict the A rows the
// tile's neighbours in N still read
#ifndef OT_GEMM_NT_STORE16
#define OT_GEMM_NT_STORE16 1
#endif
__device__ __forceinline__ void store_out4_bf16(uint16_t* dst, f32x4 v) {
  if (OT_GEMM_NT_STORE16) __builtin_nontemporal_store(bf16_rne4(v), reinterpret_cast<u32x2*>(dst));
  else *reinterpret_cast<u32x2*>(dst) = bf16_rne4(v);
}

// GS: compile the forward stored-GELU path (bf16-mode plane GEMM only: registers elsewhere)
template <int EPIT, int LAYOUT, bool ROWSCALE, int RBN = 8, bool GS = false>
__device__ __forceinline__ void gemm_vec_epilogue(const GemmArgs& p, const f32x16* acc, float* smem, int tm,
                                                  int n0, int g, int sub = 0, int tid = -1) {
  const int epi = EPIT;
  const int t = tid >= 0 ? tid : (int)threadIdx.x, lane = t & 63, wave = t >> 6;
  const int h = lane >> 5, li = lane & 31;
    // ---- vector epilogue: the accumulator tile goes through LDS (the staging buffers are free: the
    // last main-loop barrier ended every read) in two 64-row halves; each thread then finishes 8
    // rows x one float4 column chunk, so every global access is a 16-B piece of a 512-B row run and
    // each row index is loaded once per row instead of once per element.  Operand loads of a batch
    // of rows are issued together.
    constexpr int CLD = GT + 4;
    static_assert(64 * CLD + 8 * GT <= 4 * GT * GLD, "epilogue LDS exceeds the staging buffers");
    float* ct = smem;                                   // [64][CLD]
    const int c4 = t & 31, rb = t >> 5;                 // float4 column chunk, first local row
    const int col = n0 + 4 * c4;
    f32x4 bias4 = {0.f, 0.f, 0.f, 0.f};
    if (epi & OT_EPI_BIAS) bias4 = *reinterpret_cast<const f32x4*>(p.bias + (int64_t)g * p.bias_gstride + col);
    const bool need_tok = (epi & OT_EPI_DROPOUT) || ((epi & OT_EPI_RESIDUAL) && p.res_tok);
    constexpr bool RMSBWD = EPIT >= 0 && (EPIT & OT_EPI_RMSNORM_BWD);
    constexpr bool ROWRSTD = EPIT >= 0 && (EPIT & OT_EPI_ROW_RSTD);
    constexpr bool ROWDOT = EPIT >= 0 && (EPIT & OT_EPI_ROWDOT);
    // gelu_out of a bias-only epilogue: gelu(C) (C in f32 or bf16)
    constexpr bool GSTORE = GS && (EPIT == OT_EPI_BIAS || EPIT == (OT_EPI_BIAS | OT_EPI_C_BF16));
    constexpr bool CBF = EPIT >= 0 && (EPIT & OT_EPI_C_BF16);
    constexpr bool AUXBF = EPIT >= 0 && (EPIT & OT_EPI_AUX_BF16);
    f32x4 rdb4 = {0.f, 0.f, 0.f, 0.f};                 // OT_EPI_ROWDOT: the bias subtracted from aux
    if (ROWDOT) rdb4 = *reinterpret_cast<const f32x4*>(p.bias + (int64_t)g * p.bias_gstride + col);
    // dgamma partials live in a thread-private LDS slot behind ct (a register accumulator here
    // costs the whole kernel ~70 VGPRs of occupancy): dgs[rb][4 c4 .. 4 c4 + 3]
    float* dgs = ct + 64 * CLD;
    f32x4 ngam = {0.f, 0.f, 0.f, 0.f};
    if (RMSBWD) {
      ngam = *reinterpret_cast<const f32x4*>(p.ngamma + col);
      *reinterpret_cast<f32x4*>(dgs + rb * GT + 4 * c4) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    constexpr int RB = RMSBWD ? RBN / 2 : RBN;          // rows per operand-load batch (register budget)
    float am = 0.f;                                     // amax_out: |the output the next consumer reads|
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      // this half's output rows (the loads stay in flight across the accumulator write below)
      int orow[8];
      float rsc[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int lr = rb + 8 * i;                      // local row of the half: tile row below
        const int64_t gr = (int64_t)tm * GT + (LAYOUT == 0 ? (lr >> 5) * 64 + 32 * hf + (lr & 31) : 64 * hf + lr);
        orow[i] = p.out_rows ? p.out_rows[gr] : (int)gr;
        if (ROWSCALE) {                                 // RMSNorm folded into B: scale by the A row's rstd
          const int ir = p.in_rows ? p.in_rows[gr] : (int)gr;
          rsc[i] = ir >= 0 ? p.a_rstd[ir] : 0.f;
        }
      }
      if (LAYOUT == 0) {
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            ct[((wave >> 1) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * CLD + (wave & 1) * 64 + 32 * n + li] = acc[2 * hf + n][r];
      } else if (LAYOUT == 1) {
        if ((wave >> 1) == hf) {
#pragma unroll
          for (int nb = 0; nb < 4; ++nb)
#pragma unroll
            for (int r = 0; r < 16; ++r)
              ct[((wave & 1) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * CLD + 32 * nb + li] = acc[nb][r];
        }
      } else if (LAYOUT == 4) {                         // LAYOUT 4: waves 2 sub, 2 sub + 1 (64 columns each)
        if ((wave >> 1) == sub) {
#pragma unroll
          for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int nb = 0; nb < 2; ++nb)
#pragma unroll
              for (int r = 0; r < 16; ++r)
                ct[(32 * m + (r & 3) + 8 * (r >> 2) + 4 * h) * CLD + 64 * (wave & 1) + 32 * nb + li] =
                    acc[2 * (2 * hf + m) + nb][r];
        }
      } else if (LAYOUT == 3) {                         // LAYOUT 3: sub-tile `sub` is wave `sub`'s 16 blocks
        if (wave == sub) {
#pragma unroll
          for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int nb = 0; nb < 4; ++nb)
#pragma unroll
              for (int r = 0; r < 16; ++r)
                ct[(32 * m + (r & 3) + 8 * (r >> 2) + 4 * h) * CLD + 32 * nb + li] = acc[4 * (2 * hf + m) + nb][r];
        }
      } else if ((wave >> 1) == hf && (wave & 1) == sub) {   // LAYOUT 2: this half's rows are one wave's 64
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int nb = 0; nb < 4; ++nb)
#pragma unroll
            for (int r = 0; r < 16; ++r)
              ct[(32 * m + (r & 3) + 8 * (r >> 2) + 4 * h) * CLD + 32 * nb + li] = acc[4 * m + nb][r];
      }
      __syncthreads();
#pragma unroll
      for (int i0 = 0; i0 < 8; i0 += RB) {
        int64_t tok[RB];
        f32x4 aux4[RB], res4[RB], cp4[RB], x4[RB], dr4[RB];
        float nr[RB];
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          const int orr = orow[i0 + i];
          const int64_t o = orr < 0 ? 0 : orr;
          tok[i] = (need_tok && orr >= 0) ? tail_token(orr, p.tail_K, p.tail_I, p.tail_pos) : o;
          if (RMSBWD) {
            x4[i] = *reinterpret_cast<const f32x4*>(p.nx + o * p.ldnx + col);
            nr[i] = p.nrstd[o];
            dr4[i] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (p.dres) {
              const int64_t dr = p.dres_K > 0 ? kept_row(o, p.dres_K, p.dres_I, p.dres_inv) : o;
              if (dr >= 0) dr4[i] = *reinterpret_cast<const f32x4*>(p.dres + (int64_t)dr * p.lddres + col);
            }
          }
          if (AUXBF) {
            const u32x2 w = *reinterpret_cast<const u32x2*>(reinterpret_cast<const uint16_t*>(p.aux) + o * p.ldaux + col);
            aux4[i] = f32x4{__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
                            __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u)};
          } else if (epi & OT_EPI_GELU_BWD) {
            aux4[i] = *reinterpret_cast<const f32x4*>(p.aux + o * p.ldaux + col);
          }
          if (epi & OT_EPI_RESIDUAL)
            res4[i] = *reinterpret_cast<const f32x4*>(p.res + (p.res_tok ? tok[i] : o) * p.ldres + col);
          if (epi & OT_EPI_ACCUMULATE) cp4[i] = *reinterpret_cast<const f32x4*>(p.C + o * p.ldc + col);
        }
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          const int orr = orow[i0 + i];
          f32x4 v = *reinterpret_cast<const f32x4*>(ct + (rb + 8 * (i0 + i)) * CLD + 4 * c4);
          if (ROWSCALE) v = v * rsc[i0 + i];
          if (epi & OT_EPI_BIAS) v += bias4;
          if (p.rowmax_out) {                                  // this tile's largest C of the row (signed)
            float mx = fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w));
            mx = row32_max(mx);
            if (orr >= 0 && c4 == 0) p.rowmax_out[(int64_t)orr * p.rowmax_n + n0 / GT] = mx;
          }
          if (epi & OT_EPI_GELU_BWD) {
            v *= gelu_erf_grad4(aux4[i]);
            if (p.gelu_out && orr >= 0) {                      // the stored GELU (W2 weight gradient's A)
              const f32x4 hv = gelu_erf4(aux4[i]);
              store_out4_bf16(p.gelu_out + (int64_t)orr * p.ldgelu + col, hv);
            }
            if (ROWDOT) {                                      // this tile's part of sum_f dU_f (U_f - b_f)
              const f32x4 ub = aux4[i] - rdb4;
              const float sd = row32_sum(v.x * ub.x + v.y * ub.y + v.z * ub.z + v.w * ub.w);
              if (orr >= 0 && c4 == 0) p.rowdot[(int64_t)orr * p.rowdot_n + n0 / GT] = sd;
            }
          }
          if (epi & OT_EPI_GELU) {
            v = gelu_erf4(v);
          }
          if (RMSBWD) {
            // v = dL/dy of y = x * rstd * gamma:  dx = rstd * (g - x * rstd^2 * <g, x> / N) + dres
            const f32x4 gv = v * ngam;
            const float r = nr[i];
            float sdot;
            if (p.rowdot) {                                    // N > GT: <g dy, x> = sum of the partials / rstd
              float t = 0.f;
              const float* rp = p.rowdot + (int64_t)(orr < 0 ? 0 : orr) * p.rowdot_n;
              for (int j = 0; j < p.rowdot_n; ++j) t += rp[j];
              sdot = t / r;
            } else {
              sdot = row32_sum(gv.x * x4[i].x + gv.y * x4[i].y + gv.z * x4[i].z + gv.w * x4[i].w);
            }
            const float coef = r * r * r * sdot / (float)p.N;
            if (orr >= 0) {
              f32x4* q = reinterpret_cast<f32x4*>(dgs + rb * GT + 4 * c4);
              *q = *q + v * x4[i] * r;
            }
            v = gv * r - x4[i] * coef + dr4[i];
            if (orr >= 0) store_out4(p.C + (int64_t)orr * p.ldc + col, v);
            if (!(epi & OT_EPI_DROPOUT) && orr >= 0) am = amax4(am, v);
            f32x4 cv = v;                                      // what the next consumer reads (mask(dx) or dx)
            if ((epi & OT_EPI_DROPOUT) && orr >= 0) {          // mask(dx) for the dropout site upstream
              const uint32_t idx = (uint32_t)(tok[i] * p.drop_width + col);
              f32x4 mv;
              mv.x = drop_keep(p.seed, p.site, idx + 0, p.drop_thr) ? v.x * p.drop_scale : 0.f;
              mv.y = drop_keep(p.seed, p.site, idx + 1, p.drop_thr) ? v.y * p.drop_scale : 0.f;
              mv.z = drop_keep(p.seed, p.site, idx + 2, p.drop_thr) ? v.z * p.drop_scale : 0.f;
              mv.w = drop_keep(p.seed, p.site, idx + 3, p.drop_thr) ? v.w * p.drop_scale : 0.f;
              store_out4(p.dxm + (int64_t)orr * p.lddxm + col, mv);
              am = amax4(am, mv);
              cv = mv;
            }
            if (p.rowabs_out) {                                // the consumer's row bound (dx_masked, else dx)
              float mx = amax4(0.f, cv);
              mx = row32_max(mx);
              if (orr >= 0 && c4 == 0) p.rowabs_out[(int64_t)orr * p.rowabs_n + n0 / GT] = mx;
            }
            continue;
          }
          if (epi & OT_EPI_DROPOUT) {
            const uint32_t idx = (uint32_t)(tok[i] * p.drop_width + col);
            v.x = drop_keep(p.seed, p.site, idx + 0, p.drop_thr) ? v.x * p.drop_scale : 0.f;
            v.y = drop_keep(p.seed, p.site, idx + 1, p.drop_thr) ? v.y * p.drop_scale : 0.f;
            v.z = drop_keep(p.seed, p.site, idx + 2, p.drop_thr) ? v.z * p.drop_scale : 0.f;
            v.w = drop_keep(p.seed, p.site, idx + 3, p.drop_thr) ? v.w * p.drop_scale : 0.f;
          }
          if (epi & OT_EPI_RESIDUAL) v += res4[i];
          if (epi & OT_EPI_ACCUMULATE) v += cp4[i];
          if (ROWRSTD) {                                       // rstd of the finished row (next RMSNorm)
            const float ss = row32_sum(v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w);
            if (p.rowpart) {                                   // N > GT: this tile's part of the row sum
              if (c4 == 0) {
                const int lr = rb + 8 * (i0 + i);
                const int64_t gr = (int64_t)tm * GT + (LAYOUT == 0 ? (lr >> 5) * 64 + 32 * hf + (lr & 31) : 64 * hf + lr);
                p.rowpart[gr * p.ntn + n0 / GT] = ss;
              }
            } else if (orr >= 0 && c4 == 0) {
              p.rstd_out[orr] = rsqrtf(ss / (float)p.N + p.eps);
            }
          }
          if (GSTORE && p.gelu_out && orr >= 0) {              // FFN1 forward: also gelu(U) in bf16
            const f32x4 hv = gelu_erf4(v);
            store_out4_bf16(p.gelu_out + (int64_t)orr * p.ldgelu + col, hv);
          }
          if (GS && p.c16_out && orr >= 0)                     // + a bf16 copy of C (the next GEMM's A)
            store_out4_bf16(p.c16_out + (int64_t)orr * p.ldc16 + col, v);
          if (CBF) {                                           // C in bf16 (the FFN2 dgrad's dU)
            if (orr >= 0) store_out4_bf16(reinterpret_cast<uint16_t*>(p.C) + (int64_t)orr * p.ldc + col, v);
          } else if (orr >= 0) {
            store_out4(p.C + (int64_t)orr * p.ldc + col, v);
          }
          if (orr >= 0) am = amax4(am, v);
          if (p.rowabs_out) {                                  // this tile's max |C| of the row (fp16-pair consumer)
            float mx = amax4(0.f, v);
            mx = row32_max(mx);
            if (orr >= 0 && c4 == 0) p.rowabs_out[(int64_t)orr * p.rowabs_n + n0 / GT] = mx;
          }
        }
      }
      __syncthreads();                                  // ct is rewritten by the next half
    }
    if (RMSBWD && t < GT) {                             // dgamma partial of this tile (fixed order)
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) a += dgs[k * GT + t];
      p.dgpart[(int64_t)tm * p.N + n0 + t] = a;
    }
    if (p.amax_out) amax_flush(p.amax_out, am);          // (uniform: every wave reaches it)
}

// AXT / EPIT: compile-time prologue / epilogue (-1 = read p.a_xform / p.epi at run time).
// EDGE: K % 32 != 0 or N % 128 != 0 (bounds checks in staging and epilogue).
// SPLT: split-bf16 MFMA (NT only; the main loop's LDS images and register sets limit it to 2
// workgroups per CU), else native f32 MFMA.
template <bool NT, int AXT, int EPIT, bool EDGE, int SPLT>
__global__ __launch_bounds__(256, (NT && SPLT) ? 2 : OT_GEMM_MINWG) void mixed_gemm_kernel(GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* As = smem;                      // [2][GT][GLD]
  float* Bs = smem + 2 * GT * GLD;       // [2][GT][GLD]
  const int ax = AXT >= 0 ? AXT : p.a_xform;
  const int epi = EPIT >= 0 ? EPIT : p.epi;
  constexpr bool SPL = NT && SPLT != 0;
  constexpr int TERMS = SPLT;

  const int nwg = p.ntm * p.ntn;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int tm = wg / p.ntn, tn = wg % p.ntn;
  const int g = p.tile_group ? p.tile_group[tm] : 0;
  const float* W = p.W + (int64_t)g * p.w_gstride;
  const int n0 = tn * GT;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;

  // ---- staging coordinates: a row holds CPR float4 chunks; thread t stages chunk sc of rows
  // sr + RPP*i (i < NPASS), for A and (NT) B
  // (Consecutive lanes read consecutive 16-B chunks of a row.  Remapping the 8 lanes of each
  // ds_write_b128 group onto 8 rows makes the stores conflict-free but costs ~8 % on the loads.)
  constexpr int CPR = GBK / 4, RPP = 256 / CPR, NPASS = GT / RPP;
  const int sc = t % CPR, sr = t / CPR;
  const float* arow[NPASS];
  const float* brow[NPASS];
  float ars[NPASS];
  bool aok[NPASS], bok[NPASS];
#pragma unroll
  for (int i = 0; i < NPASS; ++i) {
    const int r = sr + RPP * i;
    const int64_t gr = (int64_t)tm * GT + r;
    const int ir = p.in_rows ? p.in_rows[gr] : (int)gr;
    aok[i] = ir >= 0;
    arow[i] = p.A + (int64_t)(ir < 0 ? 0 : ir) * p.lda + 4 * sc;
    ars[i] = (ax == OT_AX_RMSNORM && ir >= 0) ? p.a_rstd[ir] : 1.f;
    const int n = n0 + r;
    bok[i] = !EDGE || n < p.N;
    brow[i] = W + (int64_t)(bok[i] ? n : 0) * p.ldw + 4 * sc;
  }
  // load_stage issues raw, branch-free loads (invalid rows / k read a clamped in-bounds address and
  // are zeroed at store time); the prologue transform runs in store_stage, after the MFMA block, so
  // the global loads of stage k+1 stay in flight across the MFMAs of stage k.
  // (measured: the cheap RMSNorm scale is best applied right at load time, GELU at store time)
  constexpr bool RMS_EARLY = OT_GEMM_RMS_EARLY;
  f32x4 ra[NPASS], rb[NPASS], gm;
  bool kin = true;
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  // NN B staging: lane reads W[k0 + kk][n0 + 4*n4 ...], kk = lane % GBK
  const int nn_kk = lane % GBK, nn_n4 = wave * (64 / GBK) + lane / GBK;
  bool nnok[NPASS];

  auto load_stage = [&](int k0) {
    kin = !EDGE || (k0 + 4 * sc < p.K);
    const int ko = kin ? k0 : -4 * sc;                       // clamped: column 0 of the row
    if (ax == OT_AX_RMSNORM) gm = *reinterpret_cast<const f32x4*>(p.a_gamma + ko + 4 * sc);
#pragma unroll
    for (int i = 0; i < NPASS; ++i) ra[i] = *reinterpret_cast<const f32x4*>(arow[i] + ko);
    if (RMS_EARLY && ax == OT_AX_RMSNORM) {
#pragma unroll
      for (int i = 0; i < NPASS; ++i) ra[i] = ra[i] * gm * ars[i];
    }
    if (NT) {
#pragma unroll
      for (int i = 0; i < NPASS; ++i) rb[i] = *reinterpret_cast<const f32x4*>(brow[i] + ko);
    } else {
#pragma unroll
      for (int i = 0; i < NPASS; ++i) {
        const int k = k0 + nn_kk, n = n0 + 4 * (nn_n4 + (256 / GBK) * i);
        nnok[i] = !EDGE || (k < p.K && n < p.N);
        rb[i] = *reinterpret_cast<const f32x4*>(W + (nnok[i] ? (int64_t)k * p.ldw + n : 0));
      }
    }
  };
  auto store_stage = [&](int buf) {
    float* as = As + buf * GT * GLD;
    float* bs = Bs + buf * GT * GLD;
#pragma unroll
    for (int i = 0; i < NPASS; ++i) {
      f32x4 v = ra[i];
      if (!RMS_EARLY && ax == OT_AX_RMSNORM) {
        v = v * gm * ars[i];
      } else if (ax == OT_AX_GELU) {
        v = gelu_erf4(v);
      }
      if (!(aok[i] && kin)) v = zero4;
      *reinterpret_cast<f32x4*>(as + (sr + RPP * i) * GLD + 4 * sc) = v;
    }
    if (NT) {
#pragma unroll
      for (int i = 0; i < NPASS; ++i)
        *reinterpret_cast<f32x4*>(bs + (sr + RPP * i) * GLD + 4 * sc) = (bok[i] && kin) ? rb[i] : zero4;
    } else {
#pragma unroll
      for (int i = 0; i < NPASS; ++i) {
        const int n = 4 * (nn_n4 + (256 / GBK) * i);
        const f32x4 v = nnok[i] ? rb[i] : zero4;
        bs[(n + 0) * GLD + nn_kk] = v.x;
        bs[(n + 1) * GLD + nn_kk] = v.y;
        bs[(n + 2) * GLD + nn_kk] = v.z;
        bs[(n + 3) * GLD + nn_kk] = v.w;
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
  if constexpr (SPL) {
    // ---- split-bf16 main loop.  A 16-k stage is 4x fewer MFMA cycles than in f32, so the global
    // loads run two stages ahead (two register sets, loop unrolled by 2): stage k+2 is issued before
    // the MFMAs of stage k, stage k+1 (issued one iteration earlier) is split into LDS after them.
    struct SStage { f32x4 a[NPASS], b[NPASS], g; bool kin; };
    auto sload = [&](SStage& st, int k0) {
      st.kin = !EDGE || (k0 + 4 * sc < p.K);
      const int ko = st.kin ? k0 : -4 * sc;
      if (ax == OT_AX_RMSNORM) st.g = *reinterpret_cast<const f32x4*>(p.a_gamma + ko + 4 * sc);
#pragma unroll
      for (int i = 0; i < NPASS; ++i) st.a[i] = *reinterpret_cast<const f32x4*>(arow[i] + ko);
      if (RMS_EARLY && ax == OT_AX_RMSNORM) {
#pragma unroll
        for (int i = 0; i < NPASS; ++i) st.a[i] = st.a[i] * st.g * ars[i];
      }
#pragma unroll
      for (int i = 0; i < NPASS; ++i) st.b[i] = *reinterpret_cast<const f32x4*>(brow[i] + ko);
    };
    // split images [row][plane][16 k] (ushorts, row stride SRS = 112 B): a lane's 8-k read of one
    // plane is a 16-B piece, and 16 consecutive rows land in 16 distinct bank groups
    struct SPlanes { u32x2 a[NPASS][3], b[NPASS][3]; };
    auto ssplit = [&](const SStage& st, SPlanes& q) {
#pragma unroll
      for (int i = 0; i < NPASS; ++i) {
        f32x4 v = st.a[i];
        if (!RMS_EARLY && ax == OT_AX_RMSNORM) {
          v = v * st.g * ars[i];
        } else if (ax == OT_AX_GELU) {
          v = gelu_erf4(v);
        }
        if (!(aok[i] && st.kin)) v = zero4;
        const f32x4 w = (bok[i] && st.kin) ? st.b[i] : zero4;
        if constexpr (TERMS == 1) {
          q.a[i][0] = bf16_rne4(v);
          q.b[i][0] = bf16_rne4(w);
        } else {
          split3(v, q.a[i][0], q.a[i][1], q.a[i][2]);
          split3(w, q.b[i][0], q.b[i][1], q.b[i][2]);
        }
      }
    };
    auto swrite = [&](const SPlanes& q, int buf) {
      uint16_t* as16 = reinterpret_cast<uint16_t*>(smem) + buf * GT * SRS;
      uint16_t* bs16 = reinterpret_cast<uint16_t*>(smem) + (2 + buf) * GT * SRS;
#pragma unroll
      for (int i = 0; i < NPASS; ++i)
#pragma unroll
        for (int pl = 0; pl < (TERMS == 1 ? 1 : 3); ++pl) {
          *reinterpret_cast<u32x2*>(as16 + (sr + RPP * i) * SRS + 16 * pl + 4 * sc) = q.a[i][pl];
          *reinterpret_cast<u32x2*>(bs16 + (sr + RPP * i) * SRS + 16 * pl + 4 * sc) = q.b[i][pl];
        }
    };
    auto smma = [&](int buf) {
      const uint16_t* as16 = reinterpret_cast<const uint16_t*>(smem) + buf * GT * SRS + (wm + li) * SRS + 8 * h;
      const uint16_t* bs16 = reinterpret_cast<const uint16_t*>(smem) + (2 + buf) * GT * SRS + (wn + li) * SRS + 8 * h;
      u32x4 fa[2][3], fb[2][3];
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int q = 0; q < (TERMS == 1 ? 1 : 3); ++q) {
          fa[m][q] = *reinterpret_cast<const u32x4*>(as16 + 32 * m * SRS + 16 * q);
          fb[m][q] = *reinterpret_cast<const u32x4*>(bs16 + 32 * m * SRS + 16 * q);
        }
      // smallest terms first; (plane of A, plane of B)
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          if constexpr (TERMS == 1) {
            acc[m][n] = mfma_bf16(fa[m][0], fb[n][0], acc[m][n]);
            continue;
          }
          if (SPLIT_TERMS >= 9) {
            acc[m][n] = mfma_bf16(fa[m][2], fb[n][2], acc[m][n]);
            acc[m][n] = mfma_bf16(fa[m][1], fb[n][2], acc[m][n]);
            acc[m][n] = mfma_bf16(fa[m][2], fb[n][1], acc[m][n]);
          }
          if (SPLIT_TERMS >= 6) {
            acc[m][n] = mfma_bf16(fa[m][0], fb[n][2], acc[m][n]);
            acc[m][n] = mfma_bf16(fa[m][2], fb[n][0], acc[m][n]);
            acc[m][n] = mfma_bf16(fa[m][1], fb[n][1], acc[m][n]);
          }
          acc[m][n] = mfma_bf16(fa[m][0], fb[n][1], acc[m][n]);
          acc[m][n] = mfma_bf16(fa[m][1], fb[n][0], acc[m][n]);
          acc[m][n] = mfma_bf16(fa[m][0], fb[n][0], acc[m][n]);
        }
    };
    // one stage: issue the loads two stages ahead, MFMAs of the LDS stage interleaved with the split
    // of the next stage (already in registers), which is then written to the other buffer.
    // Branch-free (the loads past the end re-read the last stage; the extra image is never read)
    // so the whole stage is one scheduling region.
    auto stage = [&](SStage& ld, const SStage& nx, int kload, int buf) {
      sload(ld, kload);
      SPlanes q;
      ssplit(nx, q);
      smma(buf);
      swrite(q, buf ^ 1);
#if OT_GEMM_SPLIT_SCHED
#pragma unroll
      for (int i = 0; i < 4 * SPLIT_TERMS; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, OT_GEMM_SPLIT_SCHED, 0);
      }
#endif
      __syncthreads();
    };
    SStage s0, s1;
    sload(s0, 0);
    sload(s1, nk > 1 ? GBK : 0);
    {
      SPlanes q;
      ssplit(s0, q);
      swrite(q, 0);
    }
    __syncthreads();
    const int klast = (nk - 1) * GBK;
    for (int kt = 0; kt < nk; kt += 2) {
      stage(s0, s1, min((kt + 2) * GBK, klast), 0);     // stage kt in buf 0, kt+1 in s1
      if (kt + 1 >= nk) break;
      stage(s1, s0, min((kt + 3) * GBK, klast), 1);     // stage kt+1 in buf 1, kt+2 in s0
    }
  } else {
  load_stage(0);
  store_stage(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) load_stage((kt + 1) * GBK);
    const float* as = As + cur * GT * GLD + (wm + li) * GLD + (GBK / 2) * h;
    const float* bs = Bs + cur * GT * GLD + (wn + li) * GLD + (GBK / 2) * h;
#pragma unroll
    for (int half = 0; half < GBK / 16; ++half) {
      f32x4 fa[2][2], fb[2][2];
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          fa[m][q] = *reinterpret_cast<const f32x4*>(as + 32 * m * GLD + 8 * half + 4 * q);
          fb[m][q] = *reinterpret_cast<const f32x4*>(bs + 32 * m * GLD + 8 * half + 4 * q);
        }
      if (OT_GEMM_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int n = 0; n < 2; ++n)
            acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[m][s >> 2][s & 3], fb[n][s >> 2][s & 3],
                                                             acc[m][n], 0, 0, 0);
      if (OT_GEMM_PRIO) __builtin_amdgcn_s_setprio(0);
    }
    // the other buffer was last read in iteration kt-1, which every wave finished before the
    // barrier that ended it: one barrier per k-tile
    if (more) store_stage(cur ^ 1);
    __syncthreads();
  }
  }

  // ---- epilogue (flags compile-time unless EPIT < 0).  Per 32-row block m: resolve the 16 output
  // rows of this lane, issue every operand load (aux / residual / accumulate source) for the block,
  // then compute and store — no load-use chains per element.
  if constexpr (!EDGE && EPIT >= 0) {
    const f32x16 acc4[4] = {acc[0][0], acc[0][1], acc[1][0], acc[1][1]};
    gemm_vec_epilogue<EPIT, 0, false>(p, acc4, smem, tm, n0, g);
    return;
  }
  // ---- scalar epilogue (EDGE: N % 128 != 0 or unaligned operands; generic run-time flags)
  float bias_v[2] = {0.f, 0.f};
  int cols[2];
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    cols[n] = n0 + wn + 32 * n + li;
    if ((epi & OT_EPI_BIAS) && (!EDGE || cols[n] < p.N)) bias_v[n] = p.bias[(int64_t)g * p.bias_gstride + cols[n]];
  }
  const bool need_tok = (epi & OT_EPI_DROPOUT) || ((epi & OT_EPI_RESIDUAL) && p.res_tok);
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    int orow[16];
    int64_t tok[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = wm + 32 * m + (r & 3) + 8 * (r >> 2) + 4 * h;
      const int64_t gr = (int64_t)tm * GT + row;
      orow[r] = p.out_rows ? p.out_rows[gr] : (int)gr;
      tok[r] = (need_tok && orow[r] >= 0) ? tail_token(orow[r], p.tail_K, p.tail_I, p.tail_pos) : orow[r];
    }
    float ld0[16][2];
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        float v = 0.f;
        const bool ok = orow[r] >= 0 && (!EDGE || cols[n] < p.N);
        if (ok) {
          if (epi & OT_EPI_GELU_BWD) v = p.aux[(int64_t)orow[r] * p.ldaux + cols[n]];
          else if (epi & OT_EPI_RESIDUAL) v = p.res[(p.res_tok ? tok[r] : (int64_t)orow[r]) * p.ldres + cols[n]];
          else if (epi & OT_EPI_ACCUMULATE) v = p.C[(int64_t)orow[r] * p.ldc + cols[n]];
        }
        ld0[r][n] = v;
      }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (orow[r] < 0) continue;
      float* crow = p.C + (int64_t)orow[r] * p.ldc;
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int col = cols[n];
        if (EDGE && col >= p.N) continue;
        float v = acc[m][n][r];
        if (epi & OT_EPI_BIAS) v += bias_v[n];
        if (epi & OT_EPI_GELU_BWD) v *= gelu_erf_grad(ld0[r][n]);
        if (epi & OT_EPI_GELU) v = gelu_erf(v);
        if (epi & OT_EPI_DROPOUT) {
          const uint32_t idx = (uint32_t)(tok[r] * p.drop_width + col);
          v = drop_keep(p.seed, p.site, idx, p.drop_thr) ? v * p.drop_scale : 0.f;
        }
        if (epi & OT_EPI_RESIDUAL) {
          if (!(epi & OT_EPI_GELU_BWD)) v += ld0[r][n];
          else v += p.res[(p.res_tok ? tok[r] : (int64_t)orow[r]) * p.ldres + col];
        }
        if (epi & OT_EPI_ACCUMULATE) {
          if (!(epi & (OT_EPI_GELU_BWD | OT_EPI_RESIDUAL))) v += ld0[r][n];
          else v += crow[col];
        }
        crow[col] = v;
      }
    }
  }
}

// OT_EPI_ROW_RSTD with N > GT (plane GEMM): rstd_out[out_row] = rsqrt(sum of the row's ntn tile sums
// of squares / N + eps), tile sums added in column order (deterministic); one thread per tile row.
__global__ __launch_bounds__(256) void row_rstd_finish_kernel(const float* __restrict__ part, int ntn,
                                                              const int32_t* __restrict__ out_rows, int64_t nrows,
                                                              int N, float eps, float* rstd_out) {
  const int64_t gr = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gr >= nrows) return;
  const int orr = out_rows ? out_rows[gr] : (int)gr;
  if (orr < 0) return;
  float s = 0.f;
  for (int j = 0; j < ntn; ++j) s += part[gr * ntn + j];
  rstd_out[orr] = rsqrtf(s / (float)N + eps);
}

// ------------------------------------------------------------------------------------------
// Plane GEMM (split-bf16, NT): the B operand (a weight bank) arrives pre-split — ot_split_images
// writes, once per optimizer step, every 128-column x 16-k block of B as its three bf16 planes in
// the exact LDS image the MFMA fragments read ([plane][128 n][2 halves of 8 k], the halves of rows
// with bit 3 of n set swapped: conflict-free ds_read_b128) — and the A operand (activations, f32)
// is copied global -> LDS unchanged.  Both move by global_load_lds_dwordx4 (no VGPR staging, no
// LDS store instructions), three stages deep, one raw barrier per 16-k stage with a counted
// vmcnt.  Waves are 4x1: wave w owns rows 32w..32w+31 x all 128 columns, so each A element is
// read and split into its planes exactly once per tile, right before its MFMAs (the A image rows
// are 64 B with the 16-B chunk swizzle c ^ ((r >> 2) & 3): conflict-free ds_read_b128).  An
// RMSNorm prologue is folded into B (gamma scales B's k rows when the image is built) and its row
// factor rstd is applied in the epilogue; a GELU prologue runs on the fragment before the split.
constexpr int PG_A_BYTES = GT * 16 * 4;            // A stage image: 128 rows x 16 f32
constexpr int PG_B_BYTES = 3 * GT * 16 * 2;        // B stage image: 3 planes x 128 n x 16 bf16
constexpr int PG_STG_BYTES = PG_A_BYTES + PG_B_BYTES;
static_assert(64 * (GT + 4) * 4 + 8 * GT * 4 <= 2 * PG_STG_BYTES, "plane GEMM epilogue LDS");

typedef __attribute__((address_space(3))) void lds_void_t;

// TERMS = 6: split mode (three planes, six products); TERMS = 1: OT_MATMUL_BF16 (plane 0 of the image
// holds the weight rounded to nearest, A is rounded at fragment time, one product; only plane 0 is
// copied, so a stage is 12 KiB instead of 20 KiB)
template <int TERMS>
constexpr int pg_stage_bytes() { return PG_A_BYTES + (TERMS == 1 ? GT * 16 * 2 : PG_B_BYTES); }

// Pair-form images carry a tag behind their 128 column scales (plane 2 of the tile's first unit, float 128): the
// TERMS-2 plane GEMM refuses (all-NaN output) an image without it, and the tag's bytes are two bf16 quiet NaNs, so a
// six-product kernel handed a pair image multiplies NaN into its outputs (plane 2 at n = 16, k = 0, 1) instead of
// silently reading the scales as a third bf16 plane.  (The C ABI cannot see an image's form: the host layer pairs
// the images with a_rowmax, recommend_amd/model.py; this makes a mismatch loud.)
constexpr uint32_t PAIR_IMAGE_TAG = 0x7FC17FC1u;

// TERMS = 2 (split mode with the RMSNorm prologue): the scaled fp16 pair, three f16 products.  B's image is the pair
// of B[k][n] s_n (ot_split_images: every gamma-folded image, s_n from the column max); A = x gets one power-of-two
// scale per row from the bound |x_k| <= sqrt(K) / rstd (sum_k x_k^2 = K (1 / rstd^2 - eps)) — no pass over the row;
// the accumulator is unscaled per row and column before the epilogue.  Precision: 22 bits relative to the bound
// (a row whose largest |x| is 2^-b of it keeps 22 - b bits there).
template <int AXT, int EPIT, int NSTG, int MINW, int TERMS = 6>
__global__ __launch_bounds__(256, MINW) void plane_gemm_kernel(GemmArgs p) {
  static_assert(NSTG >= 2 && NSTG <= 4, "plane GEMM stages");
  static_assert(TERMS == 6 || TERMS == 1 || (TERMS == 2 && (AXT == OT_AX_RMSNORM || AXT == OT_AX_GELU || AXT == OT_AX_NONE)),
                "plane GEMM terms");
  // OT_AX_BF16: A holds bf16 values (the FFN1 epilogue's stored gelu(U)): 32 B per row and stage, the
  // lane's fragment is one 16-B LDS read, no conversion (bf16 mode only)
  // OT_AX_BF16_RMSNORM: bf16 x with the RMSNorm applied as the RMSNorm prologue does on this kernel (gamma
  // folded into the B image, rstd as the epilogue's row scale)
  constexpr bool ABF = AXT == OT_AX_BF16 || AXT == OT_AX_BF16_RMSNORM;
  constexpr bool RSC = AXT == OT_AX_RMSNORM || AXT == OT_AX_BF16_RMSNORM;
  static_assert(!ABF || TERMS == 1, "bf16 A operands go with OT_MATMUL_BF16");
  constexpr int STG = pg_stage_bytes<TERMS>();
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char* lds = reinterpret_cast<char*>(smem);
  const int nwg = p.ntm * p.ntn;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int tm = wg / p.ntn, tn = wg % p.ntn;
  const int g = p.tile_group ? p.tile_group[tm] : 0;
  const int n0 = tn * GT;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int nk = p.K >> 4;

  // glds sources.  A: wave w's instruction i fills LDS bytes [(2w+i) KiB, +1 KiB) of the A image =
  // rows 16(2w+i) .. +15, lane j -> row + j/4, physical chunk j%4 = logical chunk (j%4) ^ swizzle.
  // Rows of the tile past the row map (in_rows < 0) read row 0: their outputs are never stored.
  const float* asrc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (2 * wave + i) * 16 + (lane >> 2);
    const int64_t gr = (int64_t)tm * GT + r;
    int ir = p.in_rows ? p.in_rows[gr] : (int)gr;
    ir = ir < 0 ? 0 : ir;
    const int lc = (lane & 3) ^ ((r >> 2) & 3);
    asrc[i] = p.A + (int64_t)ir * p.lda + 4 * lc;
  }
  // bf16 A: one instruction per wave = rows 32w .. +31, lane j -> row + j/2, physical 16-B half j%2 =
  // logical half (j%2) ^ ((row >> 3) & 1) (rows li and li + 8 of a fragment read then hit other banks)
  const char* asrcb;
  {
    const int r = 32 * wave + (lane >> 1);
    const int64_t gr = (int64_t)tm * GT + r;
    int ir = p.in_rows ? p.in_rows[gr] : (int)gr;
    ir = ir < 0 ? 0 : ir;
    asrcb = reinterpret_cast<const char*>(p.A) + ((int64_t)ir * p.lda + 8 * ((lane & 1) ^ ((r >> 3) & 1))) * 2;
  }
  // B: the (g, tile) image is nk consecutive 12-KiB stage blocks; wave w copies KiB 3w .. 3w+2 (a
  // weight shared by every group, w_gstride 0 like Wo, has one group's image)
  const int gb = p.w_gstride ? g : 0;
  const char* bimg0 = reinterpret_cast<const char*>(p.bimg) + ((int64_t)gb * p.bimg_ntn + p.bimg_tn0 + tn) * nk * PG_B_BYTES;
  constexpr int BPL = TERMS == 2 ? 2 : 3;              // B planes copied per stage (split modes)
  const char* bsrc = bimg0 + (BPL * wave) * 1024 + 16 * lane;
  const char* bsrc1 = bimg0 + wave * 1024 + 16 * lane;

  auto issue = [&](int ks, int buf) {
    char* sb = lds + buf * STG;
    if (ABF) {
      __builtin_amdgcn_global_load_lds((const void*)(asrcb + 32 * ks), (lds_void_t*)(sb + wave * 1024), 16, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < 2; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + 16 * ks), (lds_void_t*)(sb + (2 * wave + i) * 1024),
                                         16, 0, 0);
    }
    if (TERMS == 1) {                                 // plane 0 only: wave w copies its KiB w
      __builtin_amdgcn_global_load_lds((const void*)(bsrc1 + (int64_t)ks * PG_B_BYTES),
                                       (lds_void_t*)(sb + PG_A_BYTES + wave * 1024), 16, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < BPL; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(bsrc + (int64_t)ks * PG_B_BYTES + i * 1024),
                                         (lds_void_t*)(sb + PG_A_BYTES + (BPL * wave + i) * 1024), 16, 0, 0);
    }
  };

  f32x16 acc[4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[a][r] = 0.f;

  const int ra = 32 * wave + li;                      // this lane's A row (fragment row li)
  const int aoff0 = ra * 64 + 16 * ((2 * h) ^ ((li >> 2) & 3));
  const int aoff1 = ra * 64 + 16 * ((2 * h + 1) ^ ((li >> 2) & 3));
  const int boff = PG_A_BYTES + li * 32 + 16 * (h ^ ((li >> 3) & 1));
  const int aoffb = ra * 32 + 16 * (h ^ ((li >> 3) & 1));  // bf16 A

  // normalised-A side output (AXT == OT_AX_RMSNORM, first column tile): this lane's fragment row ra; gamma
  // is copied to LDS behind the stage buffers first (a global load in the loop would make the compiler
  // wait for every outstanding stage copy)
  bool xnw = false;
  float xrs = 0.f;
  uint16_t* xnp = nullptr;
  float* gsm = reinterpret_cast<float*>(lds + NSTG * STG);
  constexpr bool XN = RSC && TERMS == 1;             // (bf16 mode only: split-mode registers are full)
  if (XN && p.xn_out && tn == 0) {
    for (int k = 4 * t; k < p.K; k += 4 * 256)
      *reinterpret_cast<f32x4*>(gsm + k) = *reinterpret_cast<const f32x4*>(p.a_gamma + k);
    const int64_t xgr = (int64_t)tm * GT + ra;
    const int xir = p.in_rows ? p.in_rows[xgr] : (int)xgr;
    xnw = xir >= 0;
    if (xnw) {
      xrs = p.a_rstd[xir];
      xnp = p.xn_out + (int64_t)xir * p.ldxn + 8 * h;
    }
  }

  // TERMS 2: this lane's A row scale from the RMSNorm bound sqrt(K) / rstd (the row's rstd, as the epilogue reads
  // it; loaded ahead of the stage copies, so waiting for it does not drain them)
  // (GELU prologue: the row's bound max(max_j a_rowmax, 0.17) >= max |gelu(a)|, from the producer's partial maxima)
  float abound = 1.f;
  if constexpr (TERMS == 2) {
    const int64_t gr = (int64_t)tm * GT + ra;
    int ir = p.in_rows ? p.in_rows[gr] : (int)gr;
    ir = ir < 0 ? 0 : ir;
    if constexpr (AXT == OT_AX_RMSNORM) {
      abound = p.a_rstd[ir];
    } else {
      // GELU prologue: signed maxima of u, floored at 0.17 >= |gelu| of negative u; plain A: the rows' max |a| parts
      abound = AXT == OT_AX_GELU ? 0.17f : 0.f;
      for (int j = 0; j < p.a_rowmax_n; ++j) abound = fmaxf(abound, p.a_rowmax[(int64_t)ir * p.a_rowmax_n + j]);
    }
  }
  issue(0, 0);
  if (NSTG >= 3 && nk > 1) issue(1, 1);
  if (NSTG >= 4 && nk > 2) issue(2, 2);
  float asc = 1.f, ainv = 1.f;
  if constexpr (TERMS == 2) {
    asc = pow2_scale14(AXT == OT_AX_RMSNORM ? sqrtf((float)p.K) / abound : abound);
    ainv = 1.f / asc;
  }
  for (int kt = 0; kt < nk; ++kt) {
    // this wave's copies of stage kt are done (with 3 stages the 5 (TERMS 1: 3) of stage kt+1 may
    // still fly), every wave's after the barrier; the barrier also retires every read of the buffer
    // that the copies of stage kt+NSTG-1 then overwrite (last read in iteration kt-1)
    constexpr int OPS = ABF ? 2 : (TERMS == 1 ? 3 : 2 + BPL);    // copies per wave and stage
    const int ahead = (NSTG - 2 < nk - 1 - kt) ? NSTG - 2 : nk - 1 - kt;   // later stages that may still fly
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * OPS) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(OPS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + NSTG - 1 < nk) issue(kt + NSTG - 1, (kt + NSTG - 1) % NSTG);
    const char* sb = lds + (kt % NSTG) * STG;
    u32x4 fb[4][3];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int q = 0; q < (TERMS == 1 ? 1 : BPL); ++q)
        fb[nb][q] = *reinterpret_cast<const u32x4*>(sb + boff + q * 4096 + nb * 1024);
    if constexpr (ABF) {
      u32x4 fa[3];
      fa[0] = *reinterpret_cast<const u32x4*>(sb + aoffb);
      if (XN && xnw) {                                  // from the bf16 x: (x * gamma) * rstd, rounded
        const float* gp = gsm + 16 * kt + 8 * h;
        const u32x4 w = fa[0];
        const f32x4 a0 = {__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
                          __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u)};
        const f32x4 a1 = {__uint_as_float(w.z << 16), __uint_as_float(w.z & 0xffff0000u),
                          __uint_as_float(w.w << 16), __uint_as_float(w.w & 0xffff0000u)};
        const f32x4 v0 = a0 * *reinterpret_cast<const f32x4*>(gp) * xrs;
        const f32x4 v1 = a1 * *reinterpret_cast<const f32x4*>(gp + 4) * xrs;
        const u32x2 b0 = bf16_rne4(v0), b1 = bf16_rne4(v1);
        *reinterpret_cast<u32x4*>(xnp + 16 * kt) = u32x4{b0.x, b0.y, b1.x, b1.y};
      }
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[nb] = mfma_bf16(fa[0], fb[nb][0], acc[nb]);
      continue;
    }
    f32x4 a0 = *reinterpret_cast<const f32x4*>(sb + aoff0);
    f32x4 a1 = *reinterpret_cast<const f32x4*>(sb + aoff1);
    if (XN && xnw) {                                    // k = 16 kt + 8 h .. + 7: (a * gamma) * rstd, rounded
      const float* gp = gsm + 16 * kt + 8 * h;
      const f32x4 v0 = a0 * *reinterpret_cast<const f32x4*>(gp) * xrs;
      const f32x4 v1 = a1 * *reinterpret_cast<const f32x4*>(gp + 4) * xrs;
      const u32x2 b0 = bf16_rne4(v0), b1 = bf16_rne4(v1);
      *reinterpret_cast<u32x4*>(xnp + 16 * kt) = u32x4{b0.x, b0.y, b1.x, b1.y};
    }
    if (AXT == OT_AX_GELU) {
      // scalar form here (bit-identical per element to gelu_erf4): the packed pairs measured 2-3% slower in this
      // main loop (register pressure next to the stage copies), while the epilogues and the weight gradient gain
      a0.x = gelu_erf(a0.x); a0.y = gelu_erf(a0.y); a0.z = gelu_erf(a0.z); a0.w = gelu_erf(a0.w);
      a1.x = gelu_erf(a1.x); a1.y = gelu_erf(a1.y); a1.z = gelu_erf(a1.z); a1.w = gelu_erf(a1.w);
    }
    const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    u32x4 fa[3];
    if constexpr (TERMS == 2) {
      pair8(av, asc, fa);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[nb] = mfma_pair(fa, fb[nb], acc[nb]);
    } else {
      split8t<TERMS == 1 ? 1 : 6>(av, fa);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[nb] = mfma_terms<TERMS == 1 ? 1 : 6>(fa, fb[nb], acc[nb]);
    }
  }
  if constexpr (TERMS == 2) {
    // unscale: row factor 1 / s_a (held by the lane whose A row it is: lane = row within the wave), column
    // factor 1 / s_b (ot_split_images' column scales, plane 2 of the tile's first unit); exact powers of two
    const float* csc = reinterpret_cast<const float*>(bimg0 + 2 * GT * 16 * 2);
    const float bad = reinterpret_cast<const uint32_t*>(csc)[GT] == PAIR_IMAGE_TAG ? 1.f : __builtin_nanf("");
    float cinv[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) cinv[nb] = bad / csc[32 * nb + li];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float ri = __shfl(ainv, (r & 3) + 8 * (r >> 2) + 4 * h, 64);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[nb][r] *= ri * cinv[nb];
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();                                    // the epilogue reuses the stage buffers
  gemm_vec_epilogue<EPIT, 1, RSC, MINW >= 4 ? OT_PLANE_EPI_RBN : 8, TERMS == 1>(p, acc, smem, tm, n0, g);
}

// Wide plane GEMM (OT_MATMUL_BF16, N % 256 == 0, K % 32 == 0): the plane GEMM's bf16 form on tiles of 128 rows x
// 256 columns with 32 k per stage.  A 128 x 128 tile moves 512 B through L2 -> LDS per 32x32x16 MFMA and 4 MFMAs per
// wave sit between two barriers; at C5's sizes (M = 530k rows, K 512-2048) that tile ran at 12-26% of the bf16 MFMA
// rate with its L2 -> CU stream far below what L2 serves.  Here one A fragment feeds 8 MFMAs (each wave: rows 32 w,
// all 256 columns), a stage is 384 B per MFMA and 16 MFMAs per wave sit between barriers.  A stage is two 16-k
// sub-stages in the plane GEMM's own LDS images (A as there; B = plane 0 of the two 128-column image blocks), copied
// by global_load_lds; three stages for bf16 A (72 KiB, two workgroups per CU), two for f32 A.  The epilogue is the
// plane GEMM's, once per 128-column half (same outputs, bit for bit: one MFMA chain per output in the same k order).
#ifndef OT_PLANE_WIDE
#define OT_PLANE_WIDE 1
#endif
#ifndef OT_PLANE_WIDE_WL
#define OT_PLANE_WIDE_WL 2
#endif
constexpr int PW_COLS = 2 * GT;
template <int AXT>
constexpr bool pw_abf() { return AXT == OT_AX_BF16 || AXT == OT_AX_BF16_RMSNORM; }
template <int AXT>
constexpr int pw_abytes() { return pw_abf<AXT>() ? GT * 32 : GT * 64; }      // one 16-k A image
template <int AXT>
constexpr int pw_sub() { return pw_abytes<AXT>() + 2 * GT * 32; }            // + B plane 0 of two column blocks
template <int AXT>
constexpr int pw_nstg() { return pw_abf<AXT>() ? 3 : 2; }
template <int AXT>
constexpr int pw_stage_lds() { return pw_nstg<AXT>() * 2 * pw_sub<AXT>(); }

template <int AXT, int EPIT, int WL = OT_PLANE_WIDE_WL>
__global__ __launch_bounds__(256, 2) void plane_wide_kernel(GemmArgs p) {
  static_assert(AXT == OT_AX_NONE || pw_abf<AXT>(), "wide plane GEMM: A in f32 (rounded) or bf16");
  constexpr bool ABF = pw_abf<AXT>();
  constexpr bool RSC = AXT == OT_AX_BF16_RMSNORM;
  constexpr int NSTG = pw_nstg<AXT>();
  constexpr int ABYTES = pw_abytes<AXT>();
  constexpr int SUB = pw_sub<AXT>();
  constexpr int STG = 2 * SUB;
  constexpr int OPS = 2 * ((ABF ? 1 : 2) + 2);        // copies per wave and stage
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char* lds = reinterpret_cast<char*>(smem);
  const int ntw = p.N / PW_COLS;
  const int nwg = p.ntm * ntw;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int tm = wg / ntw, tw = wg % ntw;
  const int g = p.tile_group ? p.tile_group[tm] : 0;
  const int n0 = tw * PW_COLS;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int nk = p.K >> 4, ns = nk >> 1;

  // A copy sources as in plane_gemm_kernel (rows of the tile past the row map read row 0: never stored)
  const float* asrc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (2 * wave + i) * 16 + (lane >> 2);
    const int64_t gr = (int64_t)tm * GT + r;
    int ir = p.in_rows ? p.in_rows[gr] : (int)gr;
    ir = ir < 0 ? 0 : ir;
    asrc[i] = p.A + (int64_t)ir * p.lda + 4 * ((lane & 3) ^ ((r >> 2) & 3));
  }
  const char* asrcb;
  {
    const int r = 32 * wave + (lane >> 1);
    const int64_t gr = (int64_t)tm * GT + r;
    int ir = p.in_rows ? p.in_rows[gr] : (int)gr;
    ir = ir < 0 ? 0 : ir;
    asrcb = reinterpret_cast<const char*>(p.A) + ((int64_t)ir * p.lda + 8 * ((lane & 1) ^ ((r >> 3) & 1))) * 2;
  }
  const int gb = p.w_gstride ? g : 0;
  const char* bsrc[2];
#pragma unroll
  for (int c = 0; c < 2; ++c)
    bsrc[c] = reinterpret_cast<const char*>(p.bimg) +
              ((int64_t)gb * p.bimg_ntn + p.bimg_tn0 + 2 * tw + c) * nk * PG_B_BYTES + wave * 1024 + 16 * lane;

  auto issue = [&](int s, int buf) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ks = 2 * s + j;
      char* sb = lds + buf * STG + j * SUB;
      if (ABF) {
        __builtin_amdgcn_global_load_lds((const void*)(asrcb + 32 * ks), (lds_void_t*)(sb + wave * 1024), 16, 0, 0);
      } else {
#pragma unroll
        for (int i = 0; i < 2; ++i)
          __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + 16 * ks), (lds_void_t*)(sb + (2 * wave + i) * 1024),
                                           16, 0, 0);
      }
#pragma unroll
      for (int c = 0; c < 2; ++c)
        __builtin_amdgcn_global_load_lds((const void*)(bsrc[c] + (int64_t)ks * PG_B_BYTES),
                                         (lds_void_t*)(sb + ABYTES + c * 4096 + wave * 1024), 16, 0, 0);
    }
  };

  f32x16 acc[8];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[a][r] = 0.f;

  // WL 1: wave w = rows 32 w, all 256 columns (acc[c * 4 + nb]); WL 2: wave 2 r + c = rows 64 r + 32 m, columns
  // 128 c + 32 nb (acc[4 m + nb]): 6 fragment reads per 8 MFMAs instead of 9
  constexpr int NA = WL == 2 ? 2 : 1;                 // A fragments per 16-k step
  const int wr = WL == 2 ? wave >> 1 : wave, wc = WL == 2 ? wave & 1 : 0;
  int aoff0[NA], aoff1[NA], aoffb[NA];
#pragma unroll
  for (int m = 0; m < NA; ++m) {
    const int ra = (WL == 2 ? 64 : 32) * wr + 32 * m + li;
    aoff0[m] = ra * 64 + 16 * ((2 * h) ^ ((li >> 2) & 3));
    aoff1[m] = ra * 64 + 16 * ((2 * h + 1) ^ ((li >> 2) & 3));
    aoffb[m] = ra * 32 + 16 * (h ^ ((li >> 3) & 1));
  }
  const int boff = ABYTES + li * 32 + 16 * (h ^ ((li >> 3) & 1)) + wc * 4096;

  // normalised-A side output (OT_AX_BF16_RMSNORM, first column tile), as in plane_gemm_kernel (WL 2: the c = 0 waves)
  bool xnw[NA] = {};
  float xrs[NA] = {};
  uint16_t* xnp[NA] = {};
  float* gsm = reinterpret_cast<float*>(lds + NSTG * STG);
  if (RSC && p.xn_out && tw == 0) {
    for (int k = 4 * t; k < p.K; k += 4 * 256)
      *reinterpret_cast<f32x4*>(gsm + k) = *reinterpret_cast<const f32x4*>(p.a_gamma + k);
#pragma unroll
    for (int m = 0; m < NA; ++m) {
      const int64_t xgr = (int64_t)tm * GT + (WL == 2 ? 64 : 32) * wr + 32 * m + li;
      const int xir = p.in_rows ? p.in_rows[xgr] : (int)xgr;
      xnw[m] = xir >= 0 && wc == 0;
      if (xnw[m]) {
        xrs[m] = p.a_rstd[xir];
        xnp[m] = p.xn_out + (int64_t)xir * p.ldxn + 8 * h;
      }
    }
  }

  issue(0, 0);
  if (NSTG >= 3 && ns > 1) issue(1, 1);
  for (int s = 0; s < ns; ++s) {
    // this wave's copies of stage s are done (with three stages those of stage s + 1 may still fly), every
    // wave's after the barrier, which also retires the reads of the buffer the next issue overwrites
    if (NSTG >= 3 && s + 1 < ns) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(OPS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s + NSTG - 1 < ns) issue(s + NSTG - 1, (s + NSTG - 1) % NSTG);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ks = 2 * s + j;
      const char* sb = lds + (s % NSTG) * STG + j * SUB;
      constexpr int NB = WL == 2 ? 4 : 8;
      u32x4 fb[NB];
#pragma unroll
      for (int n = 0; n < NB; ++n) fb[n] = *reinterpret_cast<const u32x4*>(sb + boff + (n >> 2) * 4096 + (n & 3) * 1024);
      u32x4 fa[NA];
#pragma unroll
      for (int m = 0; m < NA; ++m) {
        if constexpr (ABF) {
          fa[m] = *reinterpret_cast<const u32x4*>(sb + aoffb[m]);
          if (RSC && xnw[m]) {                          // (x * gamma) * rstd from the bf16 x, rounded
            const float* gp = gsm + 16 * ks + 8 * h;
            const u32x4 w = fa[m];
            const f32x4 a0 = {__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
                              __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u)};
            const f32x4 a1 = {__uint_as_float(w.z << 16), __uint_as_float(w.z & 0xffff0000u),
                              __uint_as_float(w.w << 16), __uint_as_float(w.w & 0xffff0000u)};
            const u32x2 b0 = bf16_rne4(a0 * *reinterpret_cast<const f32x4*>(gp) * xrs[m]);
            const u32x2 b1 = bf16_rne4(a1 * *reinterpret_cast<const f32x4*>(gp + 4) * xrs[m]);
            *reinterpret_cast<u32x4*>(xnp[m] + 16 * ks) = u32x4{b0.x, b0.y, b1.x, b1.y};
          }
        } else {
          const f32x4 a0 = *reinterpret_cast<const f32x4*>(sb + aoff0[m]);
          const f32x4 a1 = *reinterpret_cast<const f32x4*>(sb + aoff1[m]);
          const u32x2 b0 = bf16_rne4(a0), b1 = bf16_rne4(a1);
          fa[m] = u32x4{b0.x, b0.y, b1.x, b1.y};
        }
      }
#pragma unroll
      for (int m = 0; m < NA; ++m)
#pragma unroll
        for (int n = 0; n < NB; ++n) acc[m * NB + n] = mfma_bf16(fa[m], fb[n], acc[m * NB + n]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();                                    // the epilogue reuses the stage buffers
  if constexpr (WL == 2) {
    gemm_vec_epilogue<EPIT, 2, RSC, OT_PLANE_EPI_RBN, true>(p, acc, smem, tm, n0, g, 0);
    __syncthreads();                                  // (the first half's dgamma / row reads of its LDS are done)
    gemm_vec_epilogue<EPIT, 2, RSC, OT_PLANE_EPI_RBN, true>(p, acc, smem, tm, n0 + GT, g, 1);
  } else {
    gemm_vec_epilogue<EPIT, 1, RSC, OT_PLANE_EPI_RBN, true>(p, acc, smem, tm, n0, g);
    __syncthreads();
    gemm_vec_epilogue<EPIT, 1, RSC, OT_PLANE_EPI_RBN, true>(p, acc + 4, smem, tm, n0 + GT, g);
  }
}
// Big plane GEMM (OT_MATMUL_BF16, N % 512 == 0, K % 32 == 0): tiles of 128 rows x 512 columns, one workgroup of
// four waves per CU, each wave one 128 x 128 quarter (16 accumulator blocks: one A fragment feeds 4 MFMAs and one B
// fragment 4, 0.5 LDS reads per MFMA), 32 k per stage, three stages in flight (bf16 A: 120 KiB of LDS).  The
// epilogue is the plane GEMM's, once per quarter (the quarter's wave stages it through LDS).
constexpr int PB_COLS = 4 * GT;
constexpr int PB_NSTG = 3;
template <int AXT>
constexpr int pb_sub() { return pw_abytes<AXT>() + 4 * GT * 32; }            // A + B plane 0 of four column blocks
template <int AXT>
constexpr int pb_stage_lds() { return PB_NSTG * 2 * pb_sub<AXT>(); }

template <int AXT, int EPIT>
__global__ __launch_bounds__(256, 1) void plane_big_kernel(GemmArgs p) {
  static_assert(AXT == OT_AX_NONE || pw_abf<AXT>(), "big plane GEMM: A in f32 (rounded) or bf16");
  constexpr bool ABF = pw_abf<AXT>();
  constexpr bool RSC = AXT == OT_AX_BF16_RMSNORM;
  constexpr int NSTG = PB_NSTG;
  constexpr int ABYTES = pw_abytes<AXT>();
  constexpr int SUB = pb_sub<AXT>();
  constexpr int STG = 2 * SUB;
  constexpr int OPS = 2 * ((ABF ? 1 : 2) + 4);        // copies per wave and stage
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char* lds = reinterpret_cast<char*>(smem);
  const int ntw = p.N / PB_COLS;
  const int nwg = p.ntm * ntw;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int tm = wg / ntw, tw = wg % ntw;
  const int g = p.tile_group ? p.tile_group[tm] : 0;
  const int n0 = tw * PB_COLS;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int nk = p.K >> 4, ns = nk >> 1;

  const float* asrc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (2 * wave + i) * 16 + (lane >> 2);
    const int64_t gr = (int64_t)tm * GT + r;
    int ir = p.in_rows ? p.in_rows[gr] : (int)gr;
    ir = ir < 0 ? 0 : ir;
    asrc[i] = p.A + (int64_t)ir * p.lda + 4 * ((lane & 3) ^ ((r >> 2) & 3));
  }
  const char* asrcb;
  {
    const int r = 32 * wave + (lane >> 1);
    const int64_t gr = (int64_t)tm * GT + r;
    int ir = p.in_rows ? p.in_rows[gr] : (int)gr;
    ir = ir < 0 ? 0 : ir;
    asrcb = reinterpret_cast<const char*>(p.A) + ((int64_t)ir * p.lda + 8 * ((lane & 1) ^ ((r >> 3) & 1))) * 2;
  }
  const int gb = p.w_gstride ? g : 0;
  const char* bsrc = reinterpret_cast<const char*>(p.bimg) +
                     ((int64_t)gb * p.bimg_ntn + p.bimg_tn0 + 4 * tw) * nk * PG_B_BYTES + wave * 1024 + 16 * lane;
  const int64_t bstride = (int64_t)nk * PG_B_BYTES;   // next 128-column image block

  auto issue = [&](int s, int buf) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ks = 2 * s + j;
      char* sb = lds + buf * STG + j * SUB;
      if (ABF) {
        __builtin_amdgcn_global_load_lds((const void*)(asrcb + 32 * ks), (lds_void_t*)(sb + wave * 1024), 16, 0, 0);
      } else {
#pragma unroll
        for (int i = 0; i < 2; ++i)
          __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + 16 * ks), (lds_void_t*)(sb + (2 * wave + i) * 1024),
                                           16, 0, 0);
      }
#pragma unroll
      for (int c = 0; c < 4; ++c)
        __builtin_amdgcn_global_load_lds((const void*)(bsrc + c * bstride + (int64_t)ks * PG_B_BYTES),
                                         (lds_void_t*)(sb + ABYTES + c * 4096 + wave * 1024), 16, 0, 0);
    }
  };

  f32x16 acc[16];
#pragma unroll
  for (int a = 0; a < 16; ++a)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[a][r] = 0.f;

  int aoff0[4], aoff1[4], aoffb[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int ra = 32 * m + li;
    aoff0[m] = ra * 64 + 16 * ((2 * h) ^ ((li >> 2) & 3));
    aoff1[m] = ra * 64 + 16 * ((2 * h + 1) ^ ((li >> 2) & 3));
    aoffb[m] = ra * 32 + 16 * (h ^ ((li >> 3) & 1));
  }
  const int boff = ABYTES + wave * 4096 + li * 32 + 16 * (h ^ ((li >> 3) & 1));

  // normalised-A side output (OT_AX_BF16_RMSNORM, first column tile): wave 0 writes every row
  bool xnw[4] = {};
  float xrs[4] = {};
  uint16_t* xnp[4] = {};
  float* gsm = reinterpret_cast<float*>(lds + NSTG * STG);
  if (RSC && p.xn_out && tw == 0) {
    for (int k = 4 * t; k < p.K; k += 4 * 256)
      *reinterpret_cast<f32x4*>(gsm + k) = *reinterpret_cast<const f32x4*>(p.a_gamma + k);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int64_t xgr = (int64_t)tm * GT + 32 * m + li;
      const int xir = p.in_rows ? p.in_rows[xgr] : (int)xgr;
      xnw[m] = xir >= 0 && wave == 0;
      if (xnw[m]) {
        xrs[m] = p.a_rstd[xir];
        xnp[m] = p.xn_out + (int64_t)xir * p.ldxn + 8 * h;
      }
    }
  }

  issue(0, 0);
  if (ns > 1) issue(1, 1);
  for (int s = 0; s < ns; ++s) {
    if (s + 1 < ns) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(OPS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s + NSTG - 1 < ns) issue(s + NSTG - 1, (s + NSTG - 1) % NSTG);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ks = 2 * s + j;
      const char* sb = lds + (s % NSTG) * STG + j * SUB;
      u32x4 fb[4], fa[4];
#pragma unroll
      for (int n = 0; n < 4; ++n) fb[n] = *reinterpret_cast<const u32x4*>(sb + boff + n * 1024);
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        if constexpr (ABF) {
          fa[m] = *reinterpret_cast<const u32x4*>(sb + aoffb[m]);
          if (RSC && xnw[m]) {
            const float* gp = gsm + 16 * ks + 8 * h;
            const u32x4 w = fa[m];
            const f32x4 a0 = {__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
                              __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u)};
            const f32x4 a1 = {__uint_as_float(w.z << 16), __uint_as_float(w.z & 0xffff0000u),
                              __uint_as_float(w.w << 16), __uint_as_float(w.w & 0xffff0000u)};
            const u32x2 b0 = bf16_rne4(a0 * *reinterpret_cast<const f32x4*>(gp) * xrs[m]);
            const u32x2 b1 = bf16_rne4(a1 * *reinterpret_cast<const f32x4*>(gp + 4) * xrs[m]);
            *reinterpret_cast<u32x4*>(xnp[m] + 16 * ks) = u32x4{b0.x, b0.y, b1.x, b1.y};
          }
        } else {
          const f32x4 a0 = *reinterpret_cast<const f32x4*>(sb + aoff0[m]);
          const f32x4 a1 = *reinterpret_cast<const f32x4*>(sb + aoff1[m]);
          const u32x2 b0 = bf16_rne4(a0), b1 = bf16_rne4(a1);
          fa[m] = u32x4{b0.x, b0.y, b1.x, b1.y};
        }
      }
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[4 * m + n] = mfma_bf16(fa[m], fb[n], acc[4 * m + n]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();                                    // the epilogue reuses the stage buffers
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (q) __syncthreads();
    gemm_vec_epilogue<EPIT, 3, RSC, OT_PLANE_EPI_RBN, true>(p, acc, smem, tm, n0 + GT * q, g, q);
  }
}
// Square plane GEMM (OT_MATMUL_BF16, N % 256 == 0, K % 32 == 0, an even number of row tiles): 256 x 256 tiles, one
// workgroup of 8 waves per CU (2 per SIMD), wave (rh, cq) = rows 128 rh .. + 127 x columns 64 cq .. + 63 (8 blocks:
// 6 fragment reads per 8 MFMAs), 256 B of L2 -> LDS per MFMA (the 128 x 256 tile: 384; at C5's sizes that stream,
// not the MFMA, set the pace).  The tile's two 128-row halves may belong to different weight groups (tile_group):
// then each half's B image is copied into its own LDS region (uniform tiles copy one).  Epilogue: the plane GEMM's,
// each row half's four waves finishing its two 128-column quarters, both halves at once in separate LDS.
template <int AXT>
constexpr int ps_abytes() { return pw_abf<AXT>() ? 2 * GT * 32 : 2 * GT * 64; }   // one 16-k A image, 256 rows
template <int AXT>
constexpr int ps_sub() { return ps_abytes<AXT>() + 2 * (2 * GT * 32); }           // + two 256-column B planes
template <int AXT>
constexpr int ps_nstg() { return pw_abf<AXT>() ? 3 : 2; }
template <int AXT>
constexpr int ps_stage_lds() { return ps_nstg<AXT>() * 2 * ps_sub<AXT>(); }

template <int AXT, int EPIT>
__global__ __launch_bounds__(512, 1) void plane_sq_kernel(GemmArgs p) {
  static_assert(AXT == OT_AX_NONE || pw_abf<AXT>(), "square plane GEMM: A in f32 (rounded) or bf16");
  constexpr bool ABF = pw_abf<AXT>();
  constexpr bool RSC = AXT == OT_AX_BF16_RMSNORM;
  constexpr int NSTG = ps_nstg<AXT>();
  constexpr int ABYTES = ps_abytes<AXT>();
  constexpr int SUB = ps_sub<AXT>();
  constexpr int STG = 2 * SUB;
  constexpr int AOPS = ABF ? 1 : 2;                   // A copies per wave and sub-stage
  extern __shared__ __attribute__((aligned(16))) float smem[];
  char* lds = reinterpret_cast<char*>(smem);
  const int ntw = p.N / PW_COLS;
  const int ntp = p.ntm >> 1;                          // row-tile pairs
  const int wg = xcd_remap(blockIdx.x, ntp * ntw);
  const int tp = wg / ntw, tw = wg % ntw;
  const int gA = p.tile_group ? p.tile_group[2 * tp] : 0, gB = p.tile_group ? p.tile_group[2 * tp + 1] : 0;
  const bool uni = gA == gB || p.w_gstride == 0;
  const int n0 = tw * PW_COLS;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int rh = wave >> 2, cq = wave & 3;
  const int nk = p.K >> 4, ns = nk >> 1;

  // A copies: bf16 A, wave w = rows 32 w .. + 31 of the 256; f32 A, instruction i of wave w = rows 16 (2 w + i) ..
  const float* asrc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (2 * wave + i) * 16 + (lane >> 2);
    const int64_t gr = (int64_t)tp * 2 * GT + r;
    int ir = p.in_rows ? p.in_rows[gr] : (int)gr;
    ir = ir < 0 ? 0 : ir;
    asrc[i] = p.A + (int64_t)ir * p.lda + 4 * ((lane & 3) ^ ((r >> 2) & 3));
  }
  const char* asrcb;
  {
    const int r = 32 * wave + (lane >> 1);
    const int64_t gr = (int64_t)tp * 2 * GT + r;
    int ir = p.in_rows ? p.in_rows[gr] : (int)gr;
    ir = ir < 0 ? 0 : ir;
    asrcb = reinterpret_cast<const char*>(p.A) + ((int64_t)ir * p.lda + 8 * ((lane & 1) ^ ((r >> 3) & 1))) * 2;
  }
  // B copies: wave w = KiB (w & 3) of column block (w >> 2) of the half's group image (region 1: group gB)
  const char* bsrc[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int gq = p.w_gstride ? (q ? gB : gA) : 0;
    bsrc[q] = reinterpret_cast<const char*>(p.bimg) +
              ((int64_t)gq * p.bimg_ntn + p.bimg_tn0 + 2 * tw + (wave >> 2)) * nk * PG_B_BYTES + (wave & 3) * 1024 +
              16 * lane;
  }
  auto issue = [&](int s, int buf) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ks = 2 * s + j;
      char* sb = lds + buf * STG + j * SUB;
      if (ABF) {
        __builtin_amdgcn_global_load_lds((const void*)(asrcb + 32 * ks), (lds_void_t*)(sb + wave * 1024), 16, 0, 0);
      } else {
#pragma unroll
        for (int i = 0; i < 2; ++i)
          __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + 16 * ks), (lds_void_t*)(sb + (2 * wave + i) * 1024),
                                           16, 0, 0);
      }
      __builtin_amdgcn_global_load_lds((const void*)(bsrc[0] + (int64_t)ks * PG_B_BYTES),
                                       (lds_void_t*)(sb + ABYTES + wave * 1024), 16, 0, 0);
      if (!uni)
        __builtin_amdgcn_global_load_lds((const void*)(bsrc[1] + (int64_t)ks * PG_B_BYTES),
                                         (lds_void_t*)(sb + ABYTES + 8192 + wave * 1024), 16, 0, 0);
    }
  };

  f32x16 acc[8];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[a][r] = 0.f;

  int aoff0[4], aoff1[4], aoffb[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int ra = 128 * rh + 32 * m + li;
    aoff0[m] = ra * 64 + 16 * ((2 * h) ^ ((li >> 2) & 3));
    aoff1[m] = ra * 64 + 16 * ((2 * h + 1) ^ ((li >> 2) & 3));
    aoffb[m] = ra * 32 + 16 * (h ^ ((li >> 3) & 1));
  }
  const int boff = ABYTES + (uni ? 0 : rh * 8192) + (cq >> 1) * 4096 + 2048 * (cq & 1) + li * 32 + 16 * (h ^ ((li >> 3) & 1));

  bool xnw[4] = {};
  float xrs[4] = {};
  uint16_t* xnp[4] = {};
  float* gsm = reinterpret_cast<float*>(lds + NSTG * STG);
  if (RSC && p.xn_out && tw == 0) {
    for (int k = 4 * t; k < p.K; k += 4 * 512)
      *reinterpret_cast<f32x4*>(gsm + k) = *reinterpret_cast<const f32x4*>(p.a_gamma + k);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int64_t xgr = (int64_t)tp * 2 * GT + 128 * rh + 32 * m + li;
      const int xir = p.in_rows ? p.in_rows[xgr] : (int)xgr;
      xnw[m] = xir >= 0 && cq == 0;
      if (xnw[m]) {
        xrs[m] = p.a_rstd[xir];
        xnp[m] = p.xn_out + (int64_t)xir * p.ldxn + 8 * h;
      }
    }
  }

  issue(0, 0);
  if (NSTG >= 3 && ns > 1) issue(1, 1);
  for (int s = 0; s < ns; ++s) {
    if (NSTG >= 3 && s + 1 < ns) {
      if (uni) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * (AOPS + 1)) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * (AOPS + 2)) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (s + NSTG - 1 < ns) issue(s + NSTG - 1, (s + NSTG - 1) % NSTG);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ks = 2 * s + j;
      const char* sb = lds + (s % NSTG) * STG + j * SUB;
      u32x4 fb[2], fa[4];
#pragma unroll
      for (int n = 0; n < 2; ++n) fb[n] = *reinterpret_cast<const u32x4*>(sb + boff + n * 1024);
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        if constexpr (ABF) {
          fa[m] = *reinterpret_cast<const u32x4*>(sb + aoffb[m]);
          if (RSC && xnw[m]) {
            const float* gp = gsm + 16 * ks + 8 * h;
            const u32x4 w = fa[m];
            const f32x4 a0 = {__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
                              __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u)};
            const f32x4 a1 = {__uint_as_float(w.z << 16), __uint_as_float(w.z & 0xffff0000u),
                              __uint_as_float(w.w << 16), __uint_as_float(w.w & 0xffff0000u)};
            const u32x2 b0 = bf16_rne4(a0 * *reinterpret_cast<const f32x4*>(gp) * xrs[m]);
            const u32x2 b1 = bf16_rne4(a1 * *reinterpret_cast<const f32x4*>(gp + 4) * xrs[m]);
            *reinterpret_cast<u32x4*>(xnp[m] + 16 * ks) = u32x4{b0.x, b0.y, b1.x, b1.y};
          }
        } else {
          const f32x4 a0 = *reinterpret_cast<const f32x4*>(sb + aoff0[m]);
          const f32x4 a1 = *reinterpret_cast<const f32x4*>(sb + aoff1[m]);
          const u32x2 b0 = bf16_rne4(a0), b1 = bf16_rne4(a1);
          fa[m] = u32x4{b0.x, b0.y, b1.x, b1.y};
        }
      }
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) acc[2 * m + n] = mfma_bf16(fa[m], fb[n], acc[2 * m + n]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();                                    // the epilogue reuses the stage buffers
  // each row half's four waves finish its two quarters in its own LDS (both halves in step: same barriers)
  float* esm = smem + rh * (64 * (GT + 4) + 8 * GT);
  const int tm = 2 * tp + rh;
  const int g = rh ? gB : gA;
  gemm_vec_epilogue<EPIT, 4, RSC, OT_PLANE_EPI_RBN, true>(p, acc, esm, tm, n0, g, 0, t & 255);
  __syncthreads();
  gemm_vec_epilogue<EPIT, 4, RSC, OT_PLANE_EPI_RBN, true>(p, acc, esm, tm, n0 + GT, g, 1, t & 255);
}
#define OT_WIDE_LIST(X)                                                                        \
  X(OT_AX_NONE, 0)                                                                             \
  X(OT_AX_NONE, OT_EPI_RESIDUAL | OT_EPI_DROPOUT | OT_EPI_ROW_RSTD)                           \
  X(OT_AX_NONE, OT_EPI_RESIDUAL | OT_EPI_ROW_RSTD)                                            \
  X(OT_AX_BF16_RMSNORM, 0)                                                                     \
  X(OT_AX_BF16_RMSNORM, OT_EPI_BIAS)                                                           \
  X(OT_AX_BF16_RMSNORM, OT_EPI_BIAS | OT_EPI_C_BF16)                                           \
  X(OT_AX_BF16, 0)                                                                             \
  X(OT_AX_BF16, OT_EPI_BIAS | OT_EPI_RESIDUAL)                                                 \
  X(OT_AX_BF16, OT_EPI_BIAS | OT_EPI_RESIDUAL | OT_EPI_DROPOUT)                                \
  X(OT_AX_BF16, OT_EPI_BIAS | OT_EPI_RESIDUAL | OT_EPI_DROPOUT | OT_EPI_ROW_RSTD)              \
  X(OT_AX_BF16, OT_EPI_BIAS | OT_EPI_RESIDUAL | OT_EPI_ROW_RSTD)                               \
  X(OT_AX_BF16, OT_EPI_GELU_BWD | OT_EPI_ROWDOT | OT_EPI_C_BF16 | OT_EPI_AUX_BF16)             \
  X(OT_AX_BF16, OT_EPI_GELU_BWD | OT_EPI_ROWDOT | OT_EPI_C_BF16)                               \
  X(OT_AX_BF16, OT_EPI_RMSNORM_BWD | OT_EPI_DROPOUT)                                           \
  X(OT_AX_BF16, OT_EPI_RMSNORM_BWD)

// the tile for a bf16-mode plane GEMM of N % 256 == 0 columns (K % 32 == 0): measured at C5's shapes
// (tools/c5_gemm_bench.py, profiles/r06/c5_gemm_tiles.txt)
// (K >= N: 128 x 256 ~20% faster than 128 x 128 — C5's FFN2 / Wo forwards and input-gradient GEMMs; output-heavy
// shapes (N > K: FFN1 / QKV forwards, FFN2 dgrad) stay on 128 x 128, the 256-column tiles' epilogues serialise there;
// 256 x 256 and 128 x 512 measured slower at every C5 shape)
static int plane_tile_auto(int K, int N, int ntiles) {
  (void)ntiles;
  return N <= K ? 1 : 0;
}

// process-wide switch of the wide tile (ot_plane_wide: A/B timing and the bit-identity tests)
static std::atomic<int> g_plane_wide{OT_PLANE_WIDE};
extern "C" int ot_plane_wide(int on) {
  const int prev = g_plane_wide.load();
  if (on >= 0) g_plane_wide.store(on > 4 ? 4 : on);
  return prev;
}

// the wide kernel for (a_xform, epi), or null; its stage LDS bytes in *stage_lds (opted in above 64 KiB once)
// kind 1: 128 x 256 (plane_wide_kernel), 2: 128 x 512 (plane_big_kernel), 3: 256 x 256 (plane_sq_kernel)
static void (*plane_wide_for(int x, int e, int kind, int* stage_lds))(GemmArgs) {
  void (*k)(GemmArgs) = nullptr;
#define OT_WIDE_PICK(AX_, EP_)                                                                        \
  if (x == (AX_) && e == (EP_)) {                                                                     \
    k = kind == 3 ? plane_sq_kernel<AX_, EP_> : kind == 2 ? plane_big_kernel<AX_, EP_> : plane_wide_kernel<AX_, EP_>; \
    *stage_lds = kind == 3 ? ps_stage_lds<AX_>() : kind == 2 ? pb_stage_lds<AX_>() : pw_stage_lds<AX_>();  \
  }
  OT_WIDE_LIST(OT_WIDE_PICK)
#undef OT_WIDE_PICK
  static std::once_flag once;
  std::call_once(once, [] {
#define OT_WIDE_ATTR(AX_, EP_)                                                                               \
  (void)hipFuncSetAttribute((const void*)plane_wide_kernel<AX_, EP_>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                            pw_stage_lds<AX_>() + 4096);                                                         \
  (void)hipFuncSetAttribute((const void*)plane_big_kernel<AX_, EP_>, hipFuncAttributeMaxDynamicSharedMemorySize,  \
                            pb_stage_lds<AX_>() + 4096);                                                        \
  (void)hipFuncSetAttribute((const void*)plane_sq_kernel<AX_, EP_>, hipFuncAttributeMaxDynamicSharedMemorySize,   \
                            ps_stage_lds<AX_>() + 4096);
    OT_WIDE_LIST(OT_WIDE_ATTR)
#undef OT_WIDE_ATTR
    (void)hipGetLastError();
  });
  return k;
}

// Pre-split B images (ot_split_images).  desc [nd][10] int64: {src_off, sn, sk, gstride, kscale_off
// (-1: none), dst_off (ushorts), first_unit, G, N, K}; B[g][n][k] = src[g*gstride + n*sn + k*sk]
// (* kscale[k]); one unit = one (g, n tile, 16-k stage) block of 3 x 128 x 16 16-bit planes, one thread per
// (row n, 8-k half), each plane's 16 B at its swizzled half.  Split mode: the exact three-plane bf16 split (split8),
// except for gamma-folded images (kscale_off >= 0: the RMSNorm-prologue GEMMs, plane_gemm_kernel TERMS 2): the
// scaled fp16 pair (planes 0, 1) of B[g][n][k] s_n, s_n a power of two per column n (image_colscale_kernel, stored
// as 128 floats in plane 2 of the tile's first unit); bf16 mode: plane 0 = the value rounded to nearest.
__device__ __forceinline__ const int64_t* image_unit(const int64_t* desc, int nd, int64_t unit, int64_t& g, int64_t& tn,
                                                     int64_t& ks) {
  int b = 0;
  while (b + 1 < nd && desc[10 * (b + 1) + 6] <= unit) ++b;
  const int64_t* d = desc + 10 * b;
  const int64_t G = d[7], N = d[8], K = d[9];
  const int64_t ntn = (N + GT - 1) / GT, nks = K / 16;
  int64_t u = unit - d[6];
  if (u >= G * ntn * nks) return nullptr;
  g = u / (ntn * nks);
  u %= ntn * nks;
  tn = u / nks;
  ks = u % nks;
  return d;
}

// per column n of each (group, n tile): the power-of-two scale putting max_k |B[g][n][k]| in [2^13, 2^14) (one
// block per image unit; the tile's first-unit blocks work, two threads per column)
__global__ __launch_bounds__(256) void image_colscale_kernel(const float* __restrict__ base, const int64_t* __restrict__ desc,
                                                             int nd, uint16_t* img) {
  int64_t g, tn, ks;
  const int64_t* d = image_unit(desc, nd, blockIdx.x, g, tn, ks);
  if (!d || ks != 0 || d[4] == -1) return;
  const int64_t N = d[8], K = d[9];
  const int n = threadIdx.x >> 1, hh = threadIdx.x & 1;
  const int64_t gn = tn * GT + n;
  float m = 0.f;
  if (gn < N) {
    const float* src = base + d[0] + g * d[3] + gn * d[1];
#pragma unroll 8
    for (int64_t k = hh; k < K; k += 2) {
      float x = src[k * d[2]];
      if (d[4] >= 0) x *= base[d[4] + k];
      m = fmaxf(m, fabsf(x));
    }
  }
  m = fmaxf(m, __shfl_xor(m, 1, 64));
  float* csc = reinterpret_cast<float*>(img + d[5] + ((int64_t)blockIdx.x - d[6]) * (PG_B_BYTES / 2) + 2 * GT * 16);
  if (hh == 0) csc[n] = pow2_scale14(m);
  if (threadIdx.x == 0) reinterpret_cast<uint32_t*>(csc)[GT] = PAIR_IMAGE_TAG;   // the form tag (see PAIR_IMAGE_TAG)
}

__global__ __launch_bounds__(256) void split_images_kernel(const float* __restrict__ base, const int64_t* __restrict__ desc,
                                                           int nd, uint16_t* img, int one) {
  const int64_t unit = blockIdx.x;
  int64_t g, tn, ks;
  const int64_t* d = image_unit(desc, nd, unit, g, tn, ks);
  if (!d) return;
  const int64_t N = d[8];
  const int n = threadIdx.x >> 1, hh = threadIdx.x & 1;
  const int64_t gn = tn * GT + n;
  const float* src = base + d[0] + g * d[3] + gn * d[1];
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int64_t k = ks * 16 + 8 * hh + j;
    float x = gn < N ? src[k * d[2]] : 0.f;
    if (d[4] >= 0) x *= base[d[4] + k];
    v[j] = x;
  }
  uint16_t* dst = img + d[5] + (unit - d[6]) * (PG_B_BYTES / 2);
  u32x4 pl[3];
  const bool pair = !one && d[4] != -1;                 // gamma-folded (>= 0) or the -2 pair form
  if (one) {
    split8t<1>(v, pl);                                // OT_MATMUL_BF16: plane 0 = round to nearest
  } else if (pair) {
    const float sn = reinterpret_cast<const float*>(dst - ks * (PG_B_BYTES / 2) + 2 * GT * 16)[n];
    pair8(v, sn, pl);
  } else {
    split8(v, pl);
  }
  const int npl = one ? 1 : pair ? 2 : 3;            // (pair: plane 2 of the first unit holds the column scales)
#pragma unroll
  for (int q = 0; q < 3; ++q)
    if (q < npl) *reinterpret_cast<u32x4*>(dst + q * GT * 16 + n * 16 + 8 * (hh ^ ((n >> 3) & 1))) = pl[q];
}

// ------------------------------------------------------------------------------------------
// wgrad: partial slab per (chunk, k-tile, n-tile):  slab[c][k][n] = sum_{rows of chunk} A^T D
// LDS images are row-major, as loaded: As[r][k], Ds[r][n] (BR = 32 rows per stage, row stride 128,
// no padding): the staging stores are whole 16-B pieces of 512-B rows (conflict-free), and the
// MFMA operands need no transpose — the reduction row is the MFMA k index, so lane (li, h) of step
// s reads As[2s + h][k0 + li] (32 consecutive floats per half-wave: conflict-free ds_read_b32, two
// steps per ds_read2st64_b32).
constexpr int WBR = 32;
constexpr int WLD = GT;

struct WgradArgs {
  const float* A; int64_t lda; const int32_t* a_rows; int a_xform; const float* a_rstd; const float* a_gamma;
  const float* D; int64_t ldd; const int32_t* d_rows;
  int K, N;
  const int32_t* chunks;     // [nchunks*3] {group, row_begin, row_count} (rows index the row maps)
  int nchunks;
  float* slab;               // [nchunks][K][N]
  float* bslab;              // [nchunks][N] or null
  int ntk, ntn;
  // TERMS 2 (the scaled fp16 pair): bounds of |A| (null with the RMSNorm prologue: sqrt(K) |gamma_k| per column)
  // and |D|, one float each (ot_mixed_gemm_wgrad_ex)
  const float* a_bound; const float* d_bound;
};

template <int AXT>
__global__ __launch_bounds__(256, 2) void wgrad_kernel(WgradArgs p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  // [NBUF][WBR][WLD] for A (r, k) then [NBUF][WBR][WLD] for D (r, n)
  const int ax = AXT >= 0 ? AXT : p.a_xform;
  const int per_chunk = p.ntk * p.ntn;
  // XCD-aware: the output tiles of one chunk (which share its A or D rows) get consecutive logical
  // ids, and xcd_remap places consecutive ids on one XCD, so the shared rows come from that L2
  int c, rem;
  if (!wgrad_tile(blockIdx.x, per_chunk, p.nchunks, c, rem)) return;
  const int tk = rem / p.ntn, tn = rem % p.ntn;
  const int k0 = tk * GT, n0 = tn * GT;
  const int row_begin = p.chunks[3 * c + 1], row_count = p.chunks[3 * c + 2];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const int sr = t >> 3, sc = t & 7;       // staging: row sr of the stage, float4 columns sc + 8i
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  float bsum = 0.f;
  const bool do_bias = p.bslab && tk == 0 && t < GT;

  // row indices of a stage, raw (the in-range test is applied in load_stage, one stage later, so
  // nothing waits on these loads before the MFMA block)
  auto rows_of = [&](int rs, int& ar, int& dr) {
    const int lr = rs + sr;
    const int64_t mi = (int64_t)row_begin + (lr < row_count ? lr : 0);
    ar = p.a_rows ? p.a_rows[mi] : (int)mi;
    dr = p.d_rows ? p.d_rows[mi] : (int)mi;
  };
  // raw branch-free loads (clamped addresses, masked at store time); the prologue transform runs in
  // store_stage so stage st+1's loads stay in flight across stage st's MFMAs
  f32x4 va[4], vd[4], gv[4];
  float rsd = 1.f;
  bool aok = false, dok = false;
  auto load_stage = [&](int st, int ar, int dr) {
    const bool in = st * WBR + sr < row_count && ar >= 0 && dr >= 0;
    aok = in; dok = in;
    const float* pa = p.A + (int64_t)(aok ? ar : 0) * p.lda;
    const float* pd = p.D + (int64_t)(dok ? dr : 0) * p.ldd;
    if (ax == OT_AX_RMSNORM) rsd = p.a_rstd[aok ? ar : 0];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = k0 + 4 * (sc + 8 * i), n = n0 + 4 * (sc + 8 * i);
      const int kc = k < p.K ? k : 0, nc = n < p.N ? n : 0;
      va[i] = *reinterpret_cast<const f32x4*>(pa + kc);
      vd[i] = *reinterpret_cast<const f32x4*>(pd + nc);
      if (ax == OT_AX_RMSNORM) gv[i] = *reinterpret_cast<const f32x4*>(p.a_gamma + kc);
    }
  };
  constexpr int NBUF = OT_WGRAD_DBUF ? 2 : 1;
  auto store_stage = [&](int buf) {
    float* As = smem + buf * WBR * WLD;
    float* Ds = smem + (NBUF + buf) * WBR * WLD;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int kk = 4 * (sc + 8 * i);
      f32x4 a = va[i], dv = vd[i];
      if (ax == OT_AX_RMSNORM) {
        a = a * gv[i] * rsd;
      } else if (ax == OT_AX_GELU) {
        a = gelu_erf4(a);
      }
      if (!(aok && k0 + kk < p.K)) a = zero4;
      if (!(dok && n0 + kk < p.N)) dv = zero4;
      *reinterpret_cast<f32x4*>(As + sr * WLD + kk) = a;
      *reinterpret_cast<f32x4*>(Ds + sr * WLD + kk) = dv;
    }
  };

  const int nst = (row_count + WBR - 1) / WBR;
  int ar, dr, ar2 = -1, dr2 = -1;
  rows_of(0, ar, dr);
  if (nst > 1) rows_of(WBR, ar2, dr2);
  load_stage(0, ar, dr);
  store_stage(0);
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    const int cur = NBUF == 2 ? (st & 1) : 0;
    const bool more = st + 1 < nst;
    int ar3 = -1, dr3 = -1;
    if (more) {
      load_stage(st + 1, ar2, dr2);                       // stage st+1 data
      if (st + 2 < nst) rows_of((st + 2) * WBR, ar3, dr3);   // stage st+2 row indices
    }
    const float* As = smem + cur * WBR * WLD;
    const float* Ds = smem + (NBUF + cur) * WBR * WLD;
    if (do_bias) {
#pragma unroll
      for (int r = 0; r < WBR; r += 4)
        bsum += (Ds[r * WLD + t] + Ds[(r + 1) * WLD + t]) + (Ds[(r + 2) * WLD + t] + Ds[(r + 3) * WLD + t]);
    }
    // 16 MFMA k-steps over the 32 rows: step s takes rows 2s (lane half 0) and 2s + 1 (half 1)
    float fa[16][2], fb[16][2];
#pragma unroll
    for (int s2 = 0; s2 < 16; ++s2)
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        fa[s2][m] = As[(2 * s2 + h) * WLD + wm + 32 * m + li];
        fb[s2][m] = Ds[(2 * s2 + h) * WLD + wn + 32 * m + li];
      }
#pragma unroll
    for (int s2 = 0; s2 < 16; ++s2)
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[s2][m], fb[s2][n], acc[m][n], 0, 0, 0);
    if (NBUF == 2) {
      if (more) store_stage(cur ^ 1);
      __syncthreads();
    } else {
      __syncthreads();
      if (more) store_stage(0);
      __syncthreads();
    }
    ar2 = ar3; dr2 = dr3;
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

// ------------------------------------------------------------------------------------------
// Split-bf16 wgrad (OT_MATMUL_SPLIT_BF16): same chunk/slab contract as wgrad_kernel.  The 32-row
// stage of A and D is split into three bf16 planes stored ROW-major in LDS (the staging writes stay
// 8-B pieces of the loaded rows), and the MFMA operands, which need 8 consecutive data rows of one
// column per lane, come out of ds_read_b64_tr_b16 transposed reads (4 rows x 16 columns per 16-lane
// group).  Row images are 256 B with the 16-B chunk XOR swizzle ch ^ ((r&3)<<2 | (r>>2)&3), which
// makes both the staging writes and the transposed reads conflict-free (cdna_hip_programming T10).
typedef short v4i16 __attribute__((ext_vector_type(4)));
constexpr int WSPLANE = WBR * 256;          // bytes of one plane image (32 rows x 128 bf16)
constexpr int WSOP = 3 * WSPLANE;           // bytes of one operand (3 planes)

__device__ __forceinline__ int wsw_off(int r, int ch) { return 256 * r + 16 * (ch ^ (((r & 3) << 2) | ((r >> 2) & 3))); }

__device__ __forceinline__ v4i16 ds_tr16(const char* base, int off) {
  typedef __attribute__((address_space(3))) v4i16 lds_v4i16;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base + off));
}

// RS: 32-row groups per stage.  The bf16 mode (TERMS = 1: one plane, 8 MFMAs per 32 rows per wave) takes
// 64-row stages (RS = 2): twice the MFMAs between the stage's two barriers, the two row groups' planes in
// the space the split mode's three planes use (the swizzle depends on r & 15, so row r + 32 keeps it).
template <int TERMS>
constexpr int wgrad_rs() { return WGRAD_BF16_RS > 0 && TERMS == 1 ? WGRAD_BF16_RS : 1; }

// DBF: D holds bf16 values (OT_WG_D_BF16: the FFN2 dgrad's bf16 dU)
// TERMS 2: the scaled fp16 pair (two planes, three f16 products instead of six bf16): A column k scaled by s_k and D
// by t, powers of two from per-tensor bounds (p.a_bound / p.d_bound, written by the operands' producers; the
// RMSNorm prologue's A needs none: |x_k rstd gamma_k| <= sqrt(K) |gamma_k|), the accumulator unscaled by
// 1 / (s_k t) at the store.  Every element keeps 22 significant bits of itself down to 2^-16 of its bound (below,
// an absolute error under 2^-38 of the bound).
template <int AXT, int TERMS, bool DBF = false>
__global__ __launch_bounds__(256, 2) void wgrad_split_kernel(WgradArgs p) {
  constexpr int RS = wgrad_rs<TERMS>();
  static_assert(RS * WSPLANE <= WSOP && (TERMS == 1 || RS == 1), "wgrad stage LDS");
  static_assert(TERMS != 2 || (!DBF && (AXT == OT_AX_NONE || AXT == OT_AX_RMSNORM || AXT == OT_AX_GELU)),
                "pair wgrad forms");
  constexpr bool PAIR = TERMS == 2;
  constexpr int BR = WBR * RS;                   // rows per stage
  constexpr int NPL = TERMS == 1 ? 1 : PAIR ? 2 : 3;
  extern __shared__ __attribute__((aligned(16))) char smem_c[];
  const int ax = AXT >= 0 ? AXT : p.a_xform;
  const int per_chunk = p.ntk * p.ntn;
  int c, rem;
  if (!wgrad_tile(blockIdx.x, per_chunk, p.nchunks, c, rem)) return;
  const int tk = rem / p.ntn, tn = rem % p.ntn;
  const int k0 = tk * GT, n0 = tn * GT;
  const int row_begin = p.chunks[3 * c + 1], row_count = p.chunks[3 * c + 2];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const int sr = t >> 3, sc = t & 7;       // staging: rows sr + 32 j of the stage, float4 columns sc + 8i
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  char* As = smem_c;
  char* Ds = smem_c + WSOP;

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const bool do_bias = p.bslab && tk == 0;
  f32x4 bsum[4] = {zero4, zero4, zero4, zero4};
  f32x4 gv[4];                                   // RMSNorm gamma of this thread's k columns (stage-invariant)
  if (ax == OT_AX_RMSNORM) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = k0 + 4 * (sc + 8 * i);
      gv[i] = *reinterpret_cast<const f32x4*>(p.a_gamma + (k < p.K ? k : 0));
    }
  }
  // TERMS 2: this thread's column scales of A (k columns 4 (sc + 8 i) ..) and D's scale
  f32x4 sa[4];
  float sdv = 1.f;
  if constexpr (PAIR) {
    sdv = pow2_scale14(p.d_bound[0]);
    const float sqk = sqrtf((float)p.K);
    const float s1 = AXT == OT_AX_RMSNORM ? 1.f : pow2_scale14(p.a_bound[0]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      sa[i] = AXT == OT_AX_RMSNORM
                  ? f32x4{pow2_scale14(sqk * fabsf(gv[i].x)), pow2_scale14(sqk * fabsf(gv[i].y)),
                          pow2_scale14(sqk * fabsf(gv[i].z)), pow2_scale14(sqk * fabsf(gv[i].w))}
                  : f32x4{s1, s1, s1, s1};
  }

  auto rows_of = [&](int rs, int (&ar)[RS], int (&dr)[RS]) {
#pragma unroll
    for (int j = 0; j < RS; ++j) {
      const int lr = rs + sr + WBR * j;
      const int64_t mi = (int64_t)row_begin + (lr < row_count ? lr : 0);
      ar[j] = p.a_rows ? p.a_rows[mi] : (int)mi;
      dr[j] = p.d_rows ? p.d_rows[mi] : (int)mi;
    }
  };
  f32x4 va[RS][4], vd[RS][4];
  float rsd[RS];
  bool inr[RS];
  auto load_stage = [&](int st, const int (&ar)[RS], const int (&dr)[RS]) {
#pragma unroll
    for (int j = 0; j < RS; ++j) {
      inr[j] = st * BR + sr + WBR * j < row_count && ar[j] >= 0 && dr[j] >= 0;
      const float* pa = p.A + (int64_t)(inr[j] ? ar[j] : 0) * p.lda;
      const uint16_t* pa16 = reinterpret_cast<const uint16_t*>(p.A) + (int64_t)(inr[j] ? ar[j] : 0) * p.lda;
      const float* pd = p.D + (int64_t)(inr[j] ? dr[j] : 0) * p.ldd;
      rsd[j] = ax == OT_AX_RMSNORM ? p.a_rstd[inr[j] ? ar[j] : 0] : 1.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = k0 + 4 * (sc + 8 * i), n = n0 + 4 * (sc + 8 * i);
        const int kc = k < p.K ? k : 0, nc = n < p.N ? n : 0;
        if (AXT == OT_AX_BF16) {                       // bf16 values: exact in f32 (and in the planes)
          const u32x2 w = *reinterpret_cast<const u32x2*>(pa16 + kc);
          va[j][i] = f32x4{__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
                           __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u)};
        } else {
          va[j][i] = *reinterpret_cast<const f32x4*>(pa + kc);
        }
        if (DBF) {
          const u32x2 w = *reinterpret_cast<const u32x2*>(reinterpret_cast<const uint16_t*>(p.D) +
                                                          (int64_t)(inr[j] ? dr[j] : 0) * p.ldd + nc);
          vd[j][i] = f32x4{__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
                           __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u)};
        } else {
          vd[j][i] = *reinterpret_cast<const f32x4*>(pd + nc);
        }
      }
    }
  };
  auto store_stage = [&]() {
#pragma unroll
    for (int j = 0; j < RS; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int cc = sc + 8 * i;                      // float4 column index 0..31
        f32x4 a = va[j][i], dv = vd[j][i];
        if (ax == OT_AX_RMSNORM) {
          a = a * gv[i] * rsd[j];
        } else if (ax == OT_AX_GELU) {
          a = gelu_erf4(a);
        }
        // only D is zeroed, for rows past the chunk or with a negative id: their A (row 0 of the map, clamped
        // columns) is finite, so its products are 0; columns past K / N feed outputs that are never stored
        // (a 0 / 1 row factor: two packed multiplies instead of four selects).  Finiteness assumption: row 0 of A
        // and D must be finite — a non-finite value there (a diverged step) turns the padding rows' 0 * inf into
        // NaN in every dW tile and bias sum of a chunk with padding, where selects would have kept it to the rows
        // that hold it.  A diverged step's gradients are NaN anyway; bench.py refuses to time non-finite steps.
        dv = dv * (inr[j] ? 1.f : 0.f);
        bsum[i] += dv;                                  // (unconditional: cheaper than the if-converted select;
                                                        // stored only when do_bias)
        const int off = wsw_off(sr + WBR * j, cc >> 1) + 8 * (cc & 1);
        if constexpr (TERMS == 1) {
          *reinterpret_cast<u32x2*>(As + off) = bf16_rne4(a);
          *reinterpret_cast<u32x2*>(Ds + off) = bf16_rne4(dv);
          continue;
        }
        if constexpr (PAIR) {
          u32x2 h0, l0;
          pair4(a * sa[i], h0, l0);
          *reinterpret_cast<u32x2*>(As + off) = h0;
          *reinterpret_cast<u32x2*>(As + WSPLANE + off) = l0;
          pair4(dv * sdv, h0, l0);
          *reinterpret_cast<u32x2*>(Ds + off) = h0;
          *reinterpret_cast<u32x2*>(Ds + WSPLANE + off) = l0;
          continue;
        }
        u32x2 q0, q1, q2;
        split3(a, q0, q1, q2);
        *reinterpret_cast<u32x2*>(As + off) = q0;
        *reinterpret_cast<u32x2*>(As + WSPLANE + off) = q1;
        *reinterpret_cast<u32x2*>(As + 2 * WSPLANE + off) = q2;
        split3(dv, q0, q1, q2);
        *reinterpret_cast<u32x2*>(Ds + off) = q0;
        *reinterpret_cast<u32x2*>(Ds + WSPLANE + off) = q1;
        *reinterpret_cast<u32x2*>(Ds + 2 * WSPLANE + off) = q2;
      }
  };
  // transposed-read addresses (stage-invariant): lane 4q+pp of its 16-lane group reads row
  // r0 + q, chunk c0 + (pp >> 1), half pp & 1; r0 = 16 t2 + 8 h + 4 rd, c0 = (col0 + 16 (g & 1)) / 8
  const int gi = lane & 15, q = gi >> 2, pp = gi & 3, g1 = (lane >> 4) & 1;
  int aoff[2][2], doff[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int rd = 0; rd < 2; ++rd) {
      const int r = 8 * h + 4 * rd + q;
      aoff[m][rd] = wsw_off(r, (wm + 32 * m + 16 * g1) / 8 + (pp >> 1)) + 8 * (pp & 1);
      doff[m][rd] = wsw_off(r, (wn + 32 * m + 16 * g1) / 8 + (pp >> 1)) + 8 * (pp & 1);
    }

  const int nst = (row_count + BR - 1) / BR;
  int ar[RS], dr[RS], ar2[RS], dr2[RS];
  rows_of(0, ar, dr);
  if (nst > 1) rows_of(BR, ar2, dr2);
  load_stage(0, ar, dr);
  store_stage();
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    const bool more = st + 1 < nst;
    int ar3[RS], dr3[RS];
    if (more) {
      load_stage(st + 1, ar2, dr2);
      if (st + 2 < nst) rows_of((st + 2) * BR, ar3, dr3);
    }
#pragma unroll
    for (int t2 = 0; t2 < 2 * RS; ++t2) {               // 16-row MFMA k-steps of the stage
      u32x4 fa[2][3], fb[2][3];
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) {
          const int po = pl * WSPLANE + t2 * 16 * 256;   // row r -> r + 16 keeps the swizzle (r & 15)
          const v4i16 a0 = ds_tr16(As + po, aoff[m][0]), a1 = ds_tr16(As + po, aoff[m][1]);
          const v4i16 d0 = ds_tr16(Ds + po, doff[m][0]), d1 = ds_tr16(Ds + po, doff[m][1]);
          const u32x2 a0u = __builtin_bit_cast(u32x2, a0), a1u = __builtin_bit_cast(u32x2, a1);
          const u32x2 d0u = __builtin_bit_cast(u32x2, d0), d1u = __builtin_bit_cast(u32x2, d1);
          fa[m][pl] = u32x4{a0u.x, a0u.y, a1u.x, a1u.y};
          fb[m][pl] = u32x4{d0u.x, d0u.y, d1u.x, d1u.y};
        }
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          if constexpr (TERMS == 1) {
            acc[m][n] = mfma_bf16(fa[m][0], fb[n][0], acc[m][n]);
            continue;
          }
          if constexpr (PAIR) {
            acc[m][n] = mfma_f16(fa[m][0], fb[n][1], acc[m][n]);
            acc[m][n] = mfma_f16(fa[m][1], fb[n][0], acc[m][n]);
            acc[m][n] = mfma_f16(fa[m][0], fb[n][0], acc[m][n]);
            continue;
          }
          if (SPLIT_TERMS >= 9) {
            acc[m][n] = mfma_bf16(fa[m][2], fb[n][2], acc[m][n]);
            acc[m][n] = mfma_bf16(fa[m][1], fb[n][2], acc[m][n]);
            acc[m][n] = mfma_bf16(fa[m][2], fb[n][1], acc[m][n]);
          }
          if (SPLIT_TERMS >= 6) {
            acc[m][n] = mfma_bf16(fa[m][0], fb[n][2], acc[m][n]);
            acc[m][n] = mfma_bf16(fa[m][2], fb[n][0], acc[m][n]);
            acc[m][n] = mfma_bf16(fa[m][1], fb[n][1], acc[m][n]);
          }
          acc[m][n] = mfma_bf16(fa[m][0], fb[n][1], acc[m][n]);
          acc[m][n] = mfma_bf16(fa[m][1], fb[n][0], acc[m][n]);
          acc[m][n] = mfma_bf16(fa[m][0], fb[n][0], acc[m][n]);
        }
    }
    __syncthreads();
    if (more) store_stage();
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RS; ++j) { ar2[j] = ar3[j]; dr2[j] = dr3[j]; }
  }
  float* slab = p.slab + (int64_t)c * p.K * p.N;
  float ainv1 = 1.f;                                  // TERMS 2: 1 / (s_k t), exact powers of two
  if constexpr (PAIR) ainv1 = 1.f / ((AXT == OT_AX_RMSNORM ? 1.f : pow2_scale14(p.a_bound[0])) * sdv);
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int k = k0 + wm + 32 * m + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (k >= p.K) continue;
      float un = ainv1;
      if (PAIR && AXT == OT_AX_RMSNORM) un = 1.f / (pow2_scale14(sqrtf((float)p.K) * fabsf(p.a_gamma[k])) * sdv);
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int col = n0 + wn + 32 * n + li;
        if (col < p.N) slab[(int64_t)k * p.N + col] = PAIR ? acc[m][n][r] * un : acc[m][n][r];
      }
    }
  if (do_bias) {
    // per-thread column partials (columns 4(sc + 8i)) -> LDS [sr][32 float4] -> fixed-order sum over
    // the 32 staging rows per column
    f32x4* bl = reinterpret_cast<f32x4*>(smem_c);
#pragma unroll
    for (int i = 0; i < 4; ++i) bl[sr * 32 + sc + 8 * i] = bsum[i];
    __syncthreads();
    if (t < GT && n0 + t < p.N) {
      const float* bf = reinterpret_cast<const float*>(smem_c);
      float a = 0.f;
      for (int r = 0; r < WBR; ++r) a += bf[r * GT + t];
      p.bslab[(int64_t)c * p.N + n0 + t] = a;
    }
  }
}


// Weight gradient with both operands in bf16 (a_xform OT_AX_BF16 | OT_WG_D_BF16, OT_MATMUL_BF16: the stored
// normalised inputs / GELU and the bf16 dU / dQKV).  The stage images are plain copies of the rows, so they
// go global -> LDS by global_load_lds straight into the swizzled layout the transposed fragment reads use
// (no VGPR staging, no conversion) through a ring of WG_NST 32-row stages, WG_NST - 1 of them in flight
// (the register-staged kernel keeps one; it waits on load latency, not MFMA: 10% MFMA busy at C5).  The
// row indices of a stage are loaded one iteration before its copies are issued.  Rows past the chunk or
// with a negative row index read a zero D row (A x 0 = 0; their A source is row 0, finite).  Columns past
// K / N read column 0 (their outputs are not stored).  IDL: row maps given (a_rows == d_rows).
#ifndef OT_WGRAD_NST
#define OT_WGRAD_NST 4
#endif
#ifndef OT_WGRAD_SR
#define OT_WGRAD_SR 32                            // rows per stage (16 or 32)
#endif
#ifndef OT_WGRAD_COPY_MINW
#define OT_WGRAD_COPY_MINW 2
#endif
constexpr int WG_NST = OT_WGRAD_NST;
constexpr int WG_SR = OT_WGRAD_SR;
constexpr int WG_NI = WG_SR / 16;                 // copies per wave per operand and stage (4 rows each)
constexpr int WG_IMG = WG_SR * 256;               // one stage's rows x 128-column bf16 image
constexpr int WG_STB = 2 * WG_IMG;                // A + D per stage
static_assert(WG_SR == 16 || WG_SR == 32, "copy-staged wgrad stage rows");
constexpr int WG_IDB = 16;                        // loop iterations per row-id block
constexpr int WG_IDR = WG_IDB * WG_SR;            // ids per block (a multiple of 256: two / thread at SR 32)
constexpr int WG_LDS = WG_NST * WG_STB + 2 * WG_IDR * 4;
__device__ __attribute__((aligned(16))) uint16_t g_zero_row[GT];   // zero-initialised with the module

// ds_read_b64_tr_b16 as inline asm: the intrinsic makes the compiler wait for every outstanding
// global_load_lds (vmcnt(0)) before it, which would drain the copy ring each stage.  The caller waits for
// the results itself (tr16_wait) before using them.
__device__ __forceinline__ v4i16 ds_tr16_nowait(const char* base, int off) {
  typedef __attribute__((address_space(3))) const char lds_cchar;
  const uint32_t a = (uint32_t)(uintptr_t)(lds_cchar*)(base + off);
  v4i16 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a) : "memory");
  return r;
}
__device__ __forceinline__ void tr16_wait(v4i16& a, v4i16& b, v4i16& c, v4i16& d) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) :: "memory");
}

template <bool IDL>
__global__ __launch_bounds__(256, OT_WGRAD_COPY_MINW) void wgrad_bf16_kernel(WgradArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem_c[];
  const int per_chunk = p.ntk * p.ntn;
  int c, rem;
  if (!wgrad_tile(blockIdx.x, per_chunk, p.nchunks, c, rem)) return;
  const int tk = rem / p.ntn, tn = rem % p.ntn;
  const int k0 = tk * GT, n0 = tn * GT;
  const int row_begin = p.chunks[3 * c + 1], row_count = p.chunks[3 * c + 2];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  const uint16_t* A16 = reinterpret_cast<const uint16_t*>(p.A);
  const uint16_t* D16 = reinterpret_cast<const uint16_t*>(p.D);
  // copy lanes: instruction i of wave w fills image bytes [(2w + i) KiB, +1 KiB) = row 4 (2w + i) + lane / 16,
  // physical 16-B chunk lane % 16 = logical chunk (lane % 16) ^ swizzle(row) (wsw_off)
  int lrow[WG_NI], acol[WG_NI], dcol[WG_NI];
#pragma unroll
  for (int i = 0; i < WG_NI; ++i) {
    const int r = 4 * (WG_NI * wave + i) + (lane >> 4);
    const int lc = (lane & 15) ^ (((r & 3) << 2) | ((r >> 2) & 3));
    lrow[i] = r;
    acol[i] = k0 + 8 * lc < p.K ? k0 + 8 * lc : 0;
    dcol[i] = n0 + 8 * lc < p.N ? n0 + 8 * lc : 0;
  }
  const int nst = (row_count + WG_SR - 1) / WG_SR;
  auto row_id = [&](int st, int i) -> int {           // direct lookup (prologue; identity maps)
    const int r = st * WG_SR + lrow[i];
    const int64_t mi = (int64_t)row_begin + (r < row_count ? r : 0);
    return IDL ? p.a_rows[mi] : (int)mi;
  };
  // Row-id blocks (row maps): the ids of the copies issued in iterations [16 b, 16 b + 16) — stages
  // 16 b + NST - 1 .. + 15 — go through an LDS double buffer behind the ring, loaded into registers one block
  // ahead and written at the block's first iteration.  (An id load per stage in the loop made the compiler
  // wait for every outstanding copy before the copies that use it.)
  int* idbuf = reinterpret_cast<int*>(smem_c + WG_NST * WG_STB);   // [2][WG_IDR]
  int pre[WG_IDR / 256];
  auto prefetch_block = [&](int b) {
#pragma unroll
    for (int j = 0; j < WG_IDR / 256; ++j) {
      const int r = (WG_IDB * b + WG_NST - 1) * WG_SR + t + 256 * j;
      const int64_t mi = (int64_t)row_begin + (r < row_count ? r : 0);
      pre[j] = p.a_rows[mi];
    }
  };
  auto issue = [&](int st, const int (&ids)[WG_NI]) {
    char* sb = smem_c + (st % WG_NST) * WG_STB;
#pragma unroll
    for (int i = 0; i < WG_NI; ++i) {
      const bool ok = st * WG_SR + lrow[i] < row_count && ids[i] >= 0;
      const uint16_t* sa = A16 + (int64_t)(ok ? ids[i] : 0) * p.lda + acol[i];
      const uint16_t* sd = ok ? D16 + (int64_t)ids[i] * p.ldd + dcol[i] : g_zero_row + 8 * (lane & 15);
      __builtin_amdgcn_global_load_lds((const void*)sa, (lds_void_t*)(sb + (WG_NI * wave + i) * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)sd, (lds_void_t*)(sb + WG_IMG + (WG_NI * wave + i) * 1024), 16,
                                       0, 0);
    }
  };
  // transposed-read addresses, as in wgrad_split_kernel
  const int gi = lane & 15, q = gi >> 2, pp = gi & 3, g1 = (lane >> 4) & 1;
  int aoff[2][2], doff[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int rd = 0; rd < 2; ++rd) {
      const int r = 8 * h + 4 * rd + q;
      aoff[m][rd] = wsw_off(r, (wm + 32 * m + 16 * g1) / 8 + (pp >> 1)) + 8 * (pp & 1);
      doff[m][rd] = wsw_off(r, (wn + 32 * m + 16 * g1) / 8 + (pp >> 1)) + 8 * (pp & 1);
    }
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  // bias (tk == 0): thread t sums columns 2 (t & 63) + {0, 1} over rows (SR / 4) (t >> 6) .. of every stage
  const bool do_bias = p.bslab && tk == 0;
  const int bcp = t & 63, brs = t >> 6;
  float bs0 = 0.f, bs1 = 0.f;

  for (int s0 = 0; s0 < WG_NST - 1; ++s0)
    if (s0 < nst) {
      int ids[WG_NI];
#pragma unroll
      for (int i = 0; i < WG_NI; ++i) ids[i] = row_id(s0, i);
      issue(s0, ids);
    }
  if (IDL) prefetch_block(0);
  // in flight after stage st's copies when its wait comes: the copies of the NST - 2 stages issued after it
  // (vector memory loads retire in issue order; the id-block loads only add to the count, so the wait
  // is conservative around them)
  for (int st = 0; st < nst; ++st) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (st + WG_NST - 1 <= nst) {
      asm volatile("s_waitcnt vmcnt(%0)" :: "n"((WG_NST - 2) * 2 * WG_NI) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const bool blk = IDL && (st % WG_IDB) == 0;
    if (blk) {                                        // this block's ids into LDS
      int* ib = idbuf + ((st / WG_IDB) & 1) * WG_IDR;
#pragma unroll
      for (int j = 0; j < WG_IDR / 256; ++j) ib[t + 256 * j] = pre[j];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();                     // every wave's copies of stage st are in; slot
    asm volatile("" ::: "memory");                    // (st - 1) % NST is no longer read
    if (blk) prefetch_block(st / WG_IDB + 1);
    if (st + WG_NST - 1 < nst) {
      int ids[WG_NI];
      const int* ib = idbuf + ((st / WG_IDB) & 1) * WG_IDR + (st % WG_IDB) * WG_SR;
#pragma unroll
      for (int i = 0; i < WG_NI; ++i) ids[i] = IDL ? ib[lrow[i]] : row_id(st + WG_NST - 1, i);
      issue(st + WG_NST - 1, ids);
    }
    const char* As = smem_c + (st % WG_NST) * WG_STB;
    const char* Ds = As + WG_IMG;
    if (do_bias) {
#pragma unroll
      for (int r8 = 0; r8 < WG_SR / 4; ++r8) {
        const int r = (WG_SR / 4) * brs + r8;
        const uint32_t w = *reinterpret_cast<const uint32_t*>(Ds + wsw_off(r, bcp >> 2) + 4 * (bcp & 3));
        bs0 += __uint_as_float(w << 16);
        bs1 += __uint_as_float(w & 0xffff0000u);
      }
    }
#pragma unroll
    for (int t2 = 0; t2 < WG_SR / 16; ++t2) {
      u32x4 fa[2], fb[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int po = t2 * 16 * 256;
        v4i16 a0 = ds_tr16_nowait(As + po, aoff[m][0]), a1 = ds_tr16_nowait(As + po, aoff[m][1]);
        v4i16 d0 = ds_tr16_nowait(Ds + po, doff[m][0]), d1 = ds_tr16_nowait(Ds + po, doff[m][1]);
        tr16_wait(a0, a1, d0, d1);
        const u32x2 a0u = __builtin_bit_cast(u32x2, a0), a1u = __builtin_bit_cast(u32x2, a1);
        const u32x2 d0u = __builtin_bit_cast(u32x2, d0), d1u = __builtin_bit_cast(u32x2, d1);
        fa[m] = u32x4{a0u.x, a0u.y, a1u.x, a1u.y};
        fb[m] = u32x4{d0u.x, d0u.y, d1u.x, d1u.y};
      }
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) acc[m][n] = mfma_bf16(fa[m], fb[n], acc[m][n]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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
  if (do_bias) {                                      // fixed-order sum of the 4 row sets per column
    __syncthreads();                                  // every wave is done with the ring
    float* bl = reinterpret_cast<float*>(smem_c);     // [4][128]
    bl[brs * GT + 2 * bcp] = bs0;
    bl[brs * GT + 2 * bcp + 1] = bs1;
    __syncthreads();
    if (t < GT && n0 + t < p.N)
      p.bslab[(int64_t)c * p.N + n0 + t] = ((bl[t] + bl[GT + t]) + bl[2 * GT + t]) + bl[3 * GT + t];
  }
}

// The copy-staged bf16 weight gradient on 128 (k) x 256 (n) output tiles (N % 256 == 0): a stage is the A image
// and two 128-column D images (24 KiB at 32 rows, three stages: two workgroups per CU), each wave 64 k x 128 n
// (one D image, 8 MFMAs per 16 rows against 4), 384 B of L2 -> LDS traffic per MFMA against 512.  Same
// products in the same row order as wgrad_bf16_kernel: the slabs are bit-identical.
#ifndef OT_WGRAD_WIDE
#define OT_WGRAD_WIDE 1                                 // auto: 256 x 256 where K and N allow, else 128 x 256
#endif
constexpr int WW_NST = 3;
constexpr int WW_STB = 3 * WG_IMG;
constexpr int WW_LDS = WW_NST * WW_STB + 2 * WG_IDR * 4;
template <bool IDL>
__global__ __launch_bounds__(256, 2) void wgrad_bf16_wide_kernel(WgradArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem_c[];
  const int ntw = p.N / (2 * GT);
  const int per_chunk = p.ntk * ntw;
  int c, rem;
  if (!wgrad_tile(blockIdx.x, per_chunk, p.nchunks, c, rem)) return;
  const int tk = rem / ntw, tw = rem % ntw;
  const int k0 = tk * GT, n0 = tw * 2 * GT;
  const int row_begin = p.chunks[3 * c + 1], row_count = p.chunks[3 * c + 2];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int wm = (wave >> 1) * 64, wh = wave & 1;
  const uint16_t* A16 = reinterpret_cast<const uint16_t*>(p.A);
  const uint16_t* D16 = reinterpret_cast<const uint16_t*>(p.D);
  int lrow[WG_NI], acol[WG_NI], dcol[WG_NI];
#pragma unroll
  for (int i = 0; i < WG_NI; ++i) {
    const int r = 4 * (WG_NI * wave + i) + (lane >> 4);
    const int lc = (lane & 15) ^ (((r & 3) << 2) | ((r >> 2) & 3));
    lrow[i] = r;
    acol[i] = k0 + 8 * lc < p.K ? k0 + 8 * lc : 0;
    dcol[i] = n0 + 8 * lc;                              // (+ 128 for the second image; N % 256 == 0)
  }
  const int nst = (row_count + WG_SR - 1) / WG_SR;
  auto row_id = [&](int st, int i) -> int {
    const int r = st * WG_SR + lrow[i];
    const int64_t mi = (int64_t)row_begin + (r < row_count ? r : 0);
    return IDL ? p.a_rows[mi] : (int)mi;
  };
  int* idbuf = reinterpret_cast<int*>(smem_c + WW_NST * WW_STB);   // [2][WG_IDR]
  int pre[WG_IDR / 256];
  auto prefetch_block = [&](int b) {
#pragma unroll
    for (int j = 0; j < WG_IDR / 256; ++j) {
      const int r = (WG_IDB * b + WW_NST - 1) * WG_SR + t + 256 * j;
      const int64_t mi = (int64_t)row_begin + (r < row_count ? r : 0);
      pre[j] = p.a_rows[mi];
    }
  };
  auto issue = [&](int st, const int (&ids)[WG_NI]) {
    char* sb = smem_c + (st % WW_NST) * WW_STB;
#pragma unroll
    for (int i = 0; i < WG_NI; ++i) {
      const bool ok = st * WG_SR + lrow[i] < row_count && ids[i] >= 0;
      const uint16_t* sa = A16 + (int64_t)(ok ? ids[i] : 0) * p.lda + acol[i];
      const uint16_t* sd = ok ? D16 + (int64_t)ids[i] * p.ldd + dcol[i] : g_zero_row + 8 * (lane & 15);
      const int o = (WG_NI * wave + i) * 1024;
      __builtin_amdgcn_global_load_lds((const void*)sa, (lds_void_t*)(sb + o), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)sd, (lds_void_t*)(sb + WG_IMG + o), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(ok ? sd + GT : sd), (lds_void_t*)(sb + 2 * WG_IMG + o), 16, 0, 0);
    }
  };
  const int gi = lane & 15, q = gi >> 2, pp = gi & 3, g1 = (lane >> 4) & 1;
  int aoff[2][2], doff[4][2];
#pragma unroll
  for (int rd = 0; rd < 2; ++rd) {
    const int r = 8 * h + 4 * rd + q;
#pragma unroll
    for (int m = 0; m < 2; ++m) aoff[m][rd] = wsw_off(r, (wm + 32 * m + 16 * g1) / 8 + (pp >> 1)) + 8 * (pp & 1);
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) doff[nb][rd] = wsw_off(r, (32 * nb + 16 * g1) / 8 + (pp >> 1)) + 8 * (pp & 1);
  }
  f32x16 acc[2][4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  // bias (tk == 0): thread t sums columns 4 (t & 63) .. + 3 (image (t & 63) >> 5) over rows (SR / 4) (t >> 6) ..
  const bool do_bias = p.bslab && tk == 0;
  const int bcp = t & 63, brs = t >> 6;
  float bs[4] = {0.f, 0.f, 0.f, 0.f};

  for (int s0 = 0; s0 < WW_NST - 1; ++s0)
    if (s0 < nst) {
      int ids[WG_NI];
#pragma unroll
      for (int i = 0; i < WG_NI; ++i) ids[i] = row_id(s0, i);
      issue(s0, ids);
    }
  if (IDL) prefetch_block(0);
  for (int st = 0; st < nst; ++st) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (st + WW_NST - 1 <= nst) {
      asm volatile("s_waitcnt vmcnt(%0)" :: "n"((WW_NST - 2) * 3 * WG_NI) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const bool blk = IDL && (st % WG_IDB) == 0;
    if (blk) {
      int* ib = idbuf + ((st / WG_IDB) & 1) * WG_IDR;
#pragma unroll
      for (int j = 0; j < WG_IDR / 256; ++j) ib[t + 256 * j] = pre[j];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (blk) prefetch_block(st / WG_IDB + 1);
    if (st + WW_NST - 1 < nst) {
      int ids[WG_NI];
      const int* ib = idbuf + ((st / WG_IDB) & 1) * WG_IDR + (st % WG_IDB) * WG_SR;
#pragma unroll
      for (int i = 0; i < WG_NI; ++i) ids[i] = IDL ? ib[lrow[i]] : row_id(st + WW_NST - 1, i);
      issue(st + WW_NST - 1, ids);
    }
    const char* As = smem_c + (st % WW_NST) * WW_STB;
    const char* Ds = As + WG_IMG * (1 + wh);
    if (do_bias) {
      const char* Db = As + WG_IMG * (1 + (bcp >> 5));
      const int bc = 4 * (bcp & 31);
#pragma unroll
      for (int r8 = 0; r8 < WG_SR / 4; ++r8) {
        const int r = (WG_SR / 4) * brs + r8;
        const u32x2 w = *reinterpret_cast<const u32x2*>(Db + wsw_off(r, bc >> 3) + 2 * (bc & 7));
        bs[0] += __uint_as_float(w.x << 16);
        bs[1] += __uint_as_float(w.x & 0xffff0000u);
        bs[2] += __uint_as_float(w.y << 16);
        bs[3] += __uint_as_float(w.y & 0xffff0000u);
      }
    }
#pragma unroll
    for (int t2 = 0; t2 < WG_SR / 16; ++t2) {
      const int po = t2 * 16 * 256;
      u32x4 fa[2], fb[4];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        v4i16 a0 = ds_tr16_nowait(As + po, aoff[m][0]), a1 = ds_tr16_nowait(As + po, aoff[m][1]);
        v4i16 d0 = ds_tr16_nowait(Ds + po, doff[2 * m][0]), d1 = ds_tr16_nowait(Ds + po, doff[2 * m][1]);
        v4i16 e0 = ds_tr16_nowait(Ds + po, doff[2 * m + 1][0]), e1 = ds_tr16_nowait(Ds + po, doff[2 * m + 1][1]);
        tr16_wait(a0, a1, d0, d1);
        asm volatile("" : "+v"(e0), "+v"(e1) :: "memory");   // (complete: the wait above is lgkmcnt(0))
        const u32x2 a0u = __builtin_bit_cast(u32x2, a0), a1u = __builtin_bit_cast(u32x2, a1);
        const u32x2 d0u = __builtin_bit_cast(u32x2, d0), d1u = __builtin_bit_cast(u32x2, d1);
        const u32x2 e0u = __builtin_bit_cast(u32x2, e0), e1u = __builtin_bit_cast(u32x2, e1);
        fa[m] = u32x4{a0u.x, a0u.y, a1u.x, a1u.y};
        fb[2 * m] = u32x4{d0u.x, d0u.y, d1u.x, d1u.y};
        fb[2 * m + 1] = u32x4{e0u.x, e0u.y, e1u.x, e1u.y};
      }
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = mfma_bf16(fa[m], fb[n], acc[m][n]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float* slab = p.slab + (int64_t)c * p.K * p.N;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int k = k0 + wm + 32 * m + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (k >= p.K) continue;
#pragma unroll
      for (int n = 0; n < 4; ++n) slab[(int64_t)k * p.N + n0 + GT * wh + 32 * n + li] = acc[m][n][r];
    }
  if (do_bias) {                                      // fixed-order sum of the 4 row sets per column
    __syncthreads();
    float* bl = reinterpret_cast<float*>(smem_c);     // [4][256]
#pragma unroll
    for (int j = 0; j < 4; ++j) bl[brs * 2 * GT + 4 * bcp + j] = bs[j];
    __syncthreads();
    p.bslab[(int64_t)c * p.N + n0 + t] = ((bl[t] + bl[2 * GT + t]) + bl[4 * GT + t]) + bl[6 * GT + t];
  }
}

// The copy-staged bf16 weight gradient on 256 x 256 output tiles (K % 256 == 0, N % 256 == 0): 8 waves, wave
// (wk, wn) = k rows 64 wk .. + 63 x n columns 128 wn .. + 127; a 32-row stage is four 128-column images (A 0 / 1,
// D 0 / 1; 32 KiB), four stages (three in flight); 256 B of L2 -> LDS per MFMA.  Same products in the same row order
// as wgrad_bf16_kernel (bias: the first 256 threads, as wgrad_bf16_wide_kernel): the slabs are bit-identical.
constexpr int WS_NST = 4;
constexpr int WS_STB = 4 * WG_IMG;
constexpr int WS_IDR = WG_IDB * WG_SR;                 // ids per block: one per thread (512)
constexpr int WS_LDS = WS_NST * WS_STB + 2 * WS_IDR * 4;
static_assert(WG_SR == 32 && WS_IDR == 512, "square wgrad: 32-row stages");
template <bool IDL>
__global__ __launch_bounds__(512, 1) void wgrad_bf16_sq_kernel(WgradArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem_c[];
  const int ntw = p.N / (2 * GT), ntk = p.K / (2 * GT);
  const int per_chunk = ntk * ntw;
  int c, rem;
  if (!wgrad_tile(blockIdx.x, per_chunk, p.nchunks, c, rem)) return;
  const int tk = rem / ntw, tw = rem % ntw;
  const int k0 = tk * 2 * GT, n0 = tw * 2 * GT;
  const int row_begin = p.chunks[3 * c + 1], row_count = p.chunks[3 * c + 2];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int h = lane >> 5, li = lane & 31;
  const int wk = wave >> 1, wn = wave & 1;
  const uint16_t* A16 = reinterpret_cast<const uint16_t*>(p.A);
  const uint16_t* D16 = reinterpret_cast<const uint16_t*>(p.D);
  // copy lanes: wave w fills KiB w of each image = rows 4 w + lane / 16, physical chunk lane % 16
  const int lrow = 4 * wave + (lane >> 4);
  const int lc = (lane & 15) ^ (((lrow & 3) << 2) | ((lrow >> 2) & 3));
  const int acol = k0 + 8 * lc, dcol = n0 + 8 * lc;
  const int nst = (row_count + WG_SR - 1) / WG_SR;
  auto row_id = [&](int st) -> int {
    const int r = st * WG_SR + lrow;
    const int64_t mi = (int64_t)row_begin + (r < row_count ? r : 0);
    return IDL ? p.a_rows[mi] : (int)mi;
  };
  int* idbuf = reinterpret_cast<int*>(smem_c + WS_NST * WS_STB);   // [2][WS_IDR]
  int pre = 0;
  auto prefetch_block = [&](int b) {
    const int r = (WG_IDB * b + WS_NST - 1) * WG_SR + t;
    const int64_t mi = (int64_t)row_begin + (r < row_count ? r : 0);
    pre = p.a_rows[mi];
  };
  auto issue = [&](int st, int id) {
    char* sb = smem_c + (st % WS_NST) * WS_STB;
    const bool ok = st * WG_SR + lrow < row_count && id >= 0;
    const uint16_t* sa = A16 + (int64_t)(ok ? id : 0) * p.lda + acol;
    const uint16_t* sd = ok ? D16 + (int64_t)id * p.ldd + dcol : g_zero_row + 8 * (lane & 15);
    const int o = wave * 1024;
    __builtin_amdgcn_global_load_lds((const void*)sa, (lds_void_t*)(sb + o), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(sa + GT), (lds_void_t*)(sb + WG_IMG + o), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)sd, (lds_void_t*)(sb + 2 * WG_IMG + o), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)(ok ? sd + GT : sd), (lds_void_t*)(sb + 3 * WG_IMG + o), 16, 0, 0);
  };
  const int gi = lane & 15, q = gi >> 2, pp = gi & 3, g1 = (lane >> 4) & 1;
  int aoff[2][2], doff[4][2];
#pragma unroll
  for (int rd = 0; rd < 2; ++rd) {
    const int r = 8 * h + 4 * rd + q;
#pragma unroll
    for (int m = 0; m < 2; ++m)
      aoff[m][rd] = wsw_off(r, (64 * (wk & 1) + 32 * m + 16 * g1) / 8 + (pp >> 1)) + 8 * (pp & 1);
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) doff[nb][rd] = wsw_off(r, (32 * nb + 16 * g1) / 8 + (pp >> 1)) + 8 * (pp & 1);
  }
  f32x16 acc[2][4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const bool do_bias = p.bslab && tk == 0 && t < 256;
  const int bcp = t & 63, brs = (t >> 6) & 3;
  float bs[4] = {0.f, 0.f, 0.f, 0.f};

  for (int s0 = 0; s0 < WS_NST - 1; ++s0)
    if (s0 < nst) issue(s0, row_id(s0));
  if (IDL) prefetch_block(0);
  for (int st = 0; st < nst; ++st) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (st + WS_NST - 1 <= nst) {
      asm volatile("s_waitcnt vmcnt(%0)" :: "n"((WS_NST - 2) * 4) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const bool blk = IDL && (st % WG_IDB) == 0;
    if (blk) {
      idbuf[((st / WG_IDB) & 1) * WS_IDR + t] = pre;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (blk) prefetch_block(st / WG_IDB + 1);
    if (st + WS_NST - 1 < nst) {
      const int id = IDL ? idbuf[((st / WG_IDB) & 1) * WS_IDR + (st % WG_IDB) * WG_SR + lrow] : row_id(st + WS_NST - 1);
      issue(st + WS_NST - 1, id);
    }
    const char* Sb = smem_c + (st % WS_NST) * WS_STB;
    const char* As = Sb + WG_IMG * (wk >> 1);
    const char* Ds = Sb + WG_IMG * (2 + wn);
    if (do_bias) {
      const char* Db = Sb + WG_IMG * (2 + (bcp >> 5));
      const int bc = 4 * (bcp & 31);
#pragma unroll
      for (int r8 = 0; r8 < WG_SR / 4; ++r8) {
        const int r = (WG_SR / 4) * brs + r8;
        const u32x2 w = *reinterpret_cast<const u32x2*>(Db + wsw_off(r, bc >> 3) + 2 * (bc & 7));
        bs[0] += __uint_as_float(w.x << 16);
        bs[1] += __uint_as_float(w.x & 0xffff0000u);
        bs[2] += __uint_as_float(w.y << 16);
        bs[3] += __uint_as_float(w.y & 0xffff0000u);
      }
    }
#pragma unroll
    for (int t2 = 0; t2 < WG_SR / 16; ++t2) {
      const int po = t2 * 16 * 256;
      u32x4 fa[2], fb[4];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        v4i16 a0 = ds_tr16_nowait(As + po, aoff[m][0]), a1 = ds_tr16_nowait(As + po, aoff[m][1]);
        v4i16 d0 = ds_tr16_nowait(Ds + po, doff[2 * m][0]), d1 = ds_tr16_nowait(Ds + po, doff[2 * m][1]);
        v4i16 e0 = ds_tr16_nowait(Ds + po, doff[2 * m + 1][0]), e1 = ds_tr16_nowait(Ds + po, doff[2 * m + 1][1]);
        tr16_wait(a0, a1, d0, d1);
        asm volatile("" : "+v"(e0), "+v"(e1) :: "memory");
        const u32x2 a0u = __builtin_bit_cast(u32x2, a0), a1u = __builtin_bit_cast(u32x2, a1);
        const u32x2 d0u = __builtin_bit_cast(u32x2, d0), d1u = __builtin_bit_cast(u32x2, d1);
        const u32x2 e0u = __builtin_bit_cast(u32x2, e0), e1u = __builtin_bit_cast(u32x2, e1);
        fa[m] = u32x4{a0u.x, a0u.y, a1u.x, a1u.y};
        fb[2 * m] = u32x4{d0u.x, d0u.y, d1u.x, d1u.y};
        fb[2 * m + 1] = u32x4{e0u.x, e0u.y, e1u.x, e1u.y};
      }
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = mfma_bf16(fa[m], fb[n], acc[m][n]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float* slab = p.slab + (int64_t)c * p.K * p.N;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int k = k0 + 64 * wk + 32 * m + (r & 3) + 8 * (r >> 2) + 4 * h;
#pragma unroll
      for (int n = 0; n < 4; ++n) slab[(int64_t)k * p.N + n0 + GT * wn + 32 * n + li] = acc[m][n][r];
    }
  if (p.bslab && tk == 0) {                           // fixed-order sum of the 4 row sets per column
    __syncthreads();
    float* bl = reinterpret_cast<float*>(smem_c);     // [4][256]
    if (t < 256) {
#pragma unroll
      for (int j = 0; j < 4; ++j) bl[brs * 2 * GT + 4 * bcp + j] = bs[j];
    }
    __syncthreads();
    if (t < 256) p.bslab[(int64_t)c * p.N + n0 + t] = ((bl[t] + bl[2 * GT + t]) + bl[4 * GT + t]) + bl[6 * GT + t];
  }
}

// Sum the slabs of each group's chunks (chunks of one group are contiguous) into dW[g] (and db).
// Block = 16 float4 columns x 16 chunk lanes; chunk lane c sums chunks c, c+16, ... and the 16
// partials are combined in a fixed order through LDS (deterministic).
// Blocks past the weight columns (wblocks) reduce the bias slab the same way when N % 4 == 0 (the bias
// sums used to be one block per group looping over every chunk: the reduce's long pole).
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ slab,
                                                           const float* __restrict__ bslab,
                                                           const int32_t* __restrict__ gchunk, int K, int N,
                                                           float* dW, int64_t dw_gstride, float* db,
                                                           int64_t db_gstride, int accumulate, int wblocks) {
  __shared__ f32x4 red[16][16];
  const int g = blockIdx.y;
  const int cb = gchunk[2 * g], cn = gchunk[2 * g + 1];
  const bool bias_blk = (int)blockIdx.x >= wblocks;
  const int64_t KN = bias_blk ? (int64_t)N : (int64_t)K * N;     // slab stride per chunk
  const float* src = bias_blk ? bslab : slab;
  float* out = bias_blk ? db + (int64_t)g * db_gstride : dW + (int64_t)g * dw_gstride;
  const int col = threadIdx.x & 15, cl = threadIdx.x >> 4;
  const int64_t i4 = ((int64_t)(bias_blk ? blockIdx.x - wblocks : blockIdx.x) * 16 + col) * 4;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (i4 < KN && (!bias_blk || bslab)) {
    int c = cb + cl;
    for (; c + 48 < cb + cn; c += 64) {        // four independent loads in flight per lane
      const f32x4 a0 = *reinterpret_cast<const f32x4*>(src + (int64_t)c * KN + i4);
      const f32x4 a1 = *reinterpret_cast<const f32x4*>(src + (int64_t)(c + 16) * KN + i4);
      const f32x4 a2 = *reinterpret_cast<const f32x4*>(src + (int64_t)(c + 32) * KN + i4);
      const f32x4 a3 = *reinterpret_cast<const f32x4*>(src + (int64_t)(c + 48) * KN + i4);
      s += a0; s += a1; s += a2; s += a3;      // fixed order: deterministic
    }
    for (; c < cb + cn; c += 16) s += *reinterpret_cast<const f32x4*>(src + (int64_t)c * KN + i4);
  }
  red[cl][col] = s;
  __syncthreads();
  if (cl == 0 && i4 < KN) {   // a group with no rows (e.g. dedicated groups outside a 1-token tail) -> 0
    f32x4 t = red[0][col];
#pragma unroll
    for (int q = 1; q < 16; ++q) t += red[q][col];
    float* dst = out + i4;
    if (accumulate) t += *reinterpret_cast<const f32x4*>(dst);
    *reinterpret_cast<f32x4*>(dst) = t;
  }
  if (db && N % 4 != 0 && blockIdx.x == 0) {
    for (int n = threadIdx.x; n < N; n += blockDim.x) {
      float t = 0.f;
      if (bslab)
        for (int c = cb; c < cb + cn; ++c) t += bslab[(int64_t)c * N + n];
      float* dst = db + (int64_t)g * db_gstride + n;
      *dst = accumulate ? *dst + t : t;
    }
  }
}

// ------------------------------------------------------------------------------------------
// Transposed weight shadow: dst[g][n][k] = src[g][k][n] for each bank (32x32 LDS tiles).
// banks: [nbanks][6] int64 {src_off, dst_off, G, K, N, first_tile}; tiles of a bank: G*ceil(K/32)*ceil(N/32)
__global__ __launch_bounds__(256) void transpose_banks_kernel(const float* __restrict__ src, float* dst,
                                                              const int64_t* __restrict__ banks, int nbanks) {
  __shared__ float tile[32][33];
  const int64_t tid = blockIdx.x;
  int b = 0;
  while (b + 1 < nbanks && banks[6 * (b + 1) + 5] <= tid) ++b;
  const int64_t* bk = banks + 6 * b;
  const int64_t G = bk[2], K = bk[3], N = bk[4];
  const int64_t tk = (K + 31) / 32, tnn = (N + 31) / 32;
  int64_t rem = tid - bk[5];
  if (rem >= G * tk * tnn) return;
  const int64_t g = rem / (tk * tnn);
  rem %= tk * tnn;
  const int64_t k0 = (rem / tnn) * 32, n0 = (rem % tnn) * 32;
  const float* s = src + bk[0] + g * K * N;
  float* d = dst + bk[1] + g * K * N;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 32 x 8
  for (int i = ty; i < 32; i += 8) {
    const int64_t k = k0 + i, n = n0 + tx;
    tile[i][tx] = (k < K && n < N) ? s[k * N + n] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int64_t n = n0 + i, k = k0 + tx;
    if (k < K && n < N) d[n * K + k] = tile[tx][i];
  }
}


}  // namespace ot

using namespace ot;


extern "C" int ot_transpose_banks(const float* src, float* dst, const int64_t* banks_dev, int nbanks,
                                  int64_t total_tiles, void* stream) {
  OT_REQUIRE(src && dst && banks_dev && nbanks > 0, "ot_transpose_banks: bad args");
  if (total_tiles == 0) return OT_OK;
  hipLaunchKernelGGL(transpose_banks_kernel, dim3((unsigned)total_tiles), dim3(256), 0, (hipStream_t)stream, src, dst,
                     banks_dev, nbanks);
  OT_LAUNCH_CHECK("ot_transpose_banks");
  return OT_OK;
}

static int mixed_gemm_impl(int mode, const float* A, int64_t lda, int K, const int32_t* in_rows,
                           int a_xform, const float* a_rstd, const float* a_gamma,
                           const float* W, int64_t w_gstride, int64_t ldw, int N,
                           const int32_t* tile_group, int ntiles,
                           const float* bias, int64_t bias_gstride,
                           float* C, int64_t ldc, const int32_t* out_rows, int epi,
                           const float* res, int64_t ldres, int res_tok,
                           const float* aux, int64_t ldaux,
                           uint32_t seed, uint32_t site, float drop_rate, int tail_K, int tail_I,
                           const int32_t* tail_pos,
                           const ot_rms_epilogue* rms, const uint16_t* bimg, int bimg_ntn, int bimg_tn0,
                           int prec, void* stream) {
  OT_REQUIRE(prec == OT_MATMUL_F32 || prec == OT_MATMUL_SPLIT_BF16 || prec == OT_MATMUL_BF16,
             "ot_mixed_gemm: unknown precision %d", prec);
  OT_REQUIRE(A && W && C, "ot_mixed_gemm: null operand");
  const int rms_flags = epi & (OT_EPI_ROW_RSTD | OT_EPI_RMSNORM_BWD | OT_EPI_ROWDOT);
  OT_REQUIRE(!rms_flags || rms, "ot_mixed_gemm: row-norm epilogue flags need ot_mixed_gemm_rms");
  OT_REQUIRE(K > 0 && N > 0 && ntiles >= 0, "ot_mixed_gemm: bad sizes K=%d N=%d ntiles=%d", K, N, ntiles);
  OT_REQUIRE(K % 4 == 0 && lda % 4 == 0, "ot_mixed_gemm: K and lda must be multiples of 4");
  OT_REQUIRE(ldw % 4 == 0 && w_gstride % 4 == 0, "ot_mixed_gemm: ldw/w_gstride must be multiples of 4");
  OT_REQUIRE(mode == OT_GEMM_NN ? N % 4 == 0 : true, "ot_mixed_gemm: NN mode needs N %% 4 == 0");
  OT_REQUIRE(mode == OT_GEMM_NN || mode == OT_GEMM_NT, "ot_mixed_gemm: bad mode");
  OT_REQUIRE(!(epi & OT_EPI_BIAS) || bias, "ot_mixed_gemm: bias missing");
  OT_REQUIRE(!(epi & OT_EPI_RESIDUAL) || res, "ot_mixed_gemm: residual missing");
  OT_REQUIRE(!(epi & OT_EPI_GELU_BWD) || aux, "ot_mixed_gemm: aux missing");
  OT_REQUIRE(a_xform != OT_AX_RMSNORM || (a_rstd && a_gamma), "ot_mixed_gemm: rmsnorm prologue needs rstd/gamma");
  OT_REQUIRE(a_xform == OT_AX_NONE || a_xform == OT_AX_RMSNORM || a_xform == OT_AX_GELU || a_xform == OT_AX_BF16 ||
                 a_xform == OT_AX_BF16_RMSNORM,
             "ot_mixed_gemm: bad a_xform %d", a_xform);
  OT_REQUIRE(a_xform != OT_AX_BF16_RMSNORM || (a_rstd && a_gamma),
             "ot_mixed_gemm: OT_AX_BF16_RMSNORM needs rstd / gamma (gamma folded into the B image)");
  OT_REQUIRE((a_xform != OT_AX_BF16 && a_xform != OT_AX_BF16_RMSNORM) ||
                 (prec == OT_MATMUL_BF16 && bimg && mode == OT_GEMM_NT &&
                                       lda % 8 == 0 && ((uintptr_t)A % 16) == 0),
             "ot_mixed_gemm: OT_AX_BF16 (bf16 A) needs the bf16 mode, a B image (plane GEMM), NT mode and 16-B "
             "aligned rows");
  OT_REQUIRE(!rms || !rms->gelu_out || (((epi & OT_EPI_GELU_BWD) || (epi & ~OT_EPI_C_BF16) == OT_EPI_BIAS) &&
                                        rms->ldgelu % 4 == 0 &&
                                        ((uintptr_t)rms->gelu_out % 8) == 0),
             "ot_mixed_gemm_rms: gelu_out needs OT_EPI_GELU_BWD or epi == OT_EPI_BIAS, ldgelu %% 4 == 0 and 8-B "
             "alignment");
  OT_REQUIRE(!((epi & OT_EPI_DROPOUT) || res_tok) || (tail_K > 0 && tail_I >= tail_K), "ot_mixed_gemm: bad tail map");
  if (rms_flags) {
    OT_REQUIRE(mode == OT_GEMM_NT && N % GT == 0 &&
                   (N == GT || !(epi & OT_EPI_RMSNORM_BWD) || (rms->rowdot && rms->rowdot_n > 0)),
               "ot_mixed_gemm_rms: row-norm epilogues need NT mode and N %% %d == 0 (OT_EPI_RMSNORM_BWD with N > %d: "
               "the row-dot partials)", GT, GT);
    OT_REQUIRE(N == GT || !(epi & OT_EPI_ROW_RSTD) ||
                   (rms->workspace && rms->ws_bytes >= ot_mixed_gemm_rms_workspace_size(ntiles, N)),
               "ot_mixed_gemm_rms: OT_EPI_ROW_RSTD with N > %d needs the workspace", GT);
    OT_REQUIRE(!(epi & OT_EPI_ROWDOT) || ((epi & OT_EPI_GELU_BWD) &&
                                          !(epi & ~(OT_EPI_GELU_BWD | OT_EPI_ROWDOT | OT_EPI_C_BF16 | OT_EPI_AUX_BF16)) &&
                                          rms->rowdot && rms->rowdot_n == N / GT && bias),
               "ot_mixed_gemm_rms: OT_EPI_ROWDOT goes with OT_EPI_GELU_BWD only and needs rowdot[rows][N / %d] and "
               "the bias", GT);
    OT_REQUIRE(!(epi & OT_EPI_ROW_RSTD) || rms->rstd_out, "ot_mixed_gemm_rms: rstd_out missing");
    OT_REQUIRE(!(epi & OT_EPI_RMSNORM_BWD) || (rms->x && rms->gamma && rms->rstd && rms->ldx % 4 == 0),
               "ot_mixed_gemm_rms: RMSNorm backward needs x / gamma / rstd");
    OT_REQUIRE(!(epi & OT_EPI_RMSNORM_BWD) || !(epi & ~(OT_EPI_RMSNORM_BWD | OT_EPI_DROPOUT)),
               "ot_mixed_gemm_rms: RMSNorm backward combines with OT_EPI_DROPOUT only");
    OT_REQUIRE(!((epi & OT_EPI_RMSNORM_BWD) && (epi & OT_EPI_DROPOUT)) || rms->dx_masked,
               "ot_mixed_gemm_rms: dx_masked missing");
    OT_REQUIRE(!rms->dgamma || (rms->workspace && rms->ws_bytes >= ot_mixed_gemm_rms_workspace_size(ntiles, N)),
               "ot_mixed_gemm_rms: workspace too small");
    OT_REQUIRE(!rms->dres || rms->lddres % 4 == 0, "ot_mixed_gemm_rms: lddres must be a multiple of 4");
  }
  if (ntiles == 0) return OT_OK;
  GemmArgs p{A, lda, K, in_rows, a_xform, a_rstd, a_gamma, W, w_gstride, ldw, N, tile_group,
             bias, bias_gstride, C, ldc, out_rows, epi, res, ldres, res_tok, aux, ldaux,
             seed, site, 0u, 1.f, tail_K, tail_I, N, ntiles, (int)ceil_div(N, GT)};
  p.tail_pos = tail_pos;
  p.bimg = bimg; p.bimg_ntn = bimg_ntn; p.bimg_tn0 = bimg_tn0;
  float* dgpart = nullptr;
  if (rms && rms->xn_out) {
    p.xn_out = rms->xn_out;
    p.ldxn = rms->ldxn;
  }
  if (rms && rms->c16_out) {
    p.c16_out = rms->c16_out;
    p.ldc16 = rms->ldc16;
  }
  if (rms && rms->rowmax_out) {
    p.rowmax_out = rms->rowmax_out;
    p.rowmax_n = rms->rowmax_n;
  }
  if (rms) {
    p.amax_out = rms->amax_out;
    p.rowabs_out = rms->rowabs_out;
    p.rowabs_n = rms->rowabs_n;
  }
  if (rms && rms->a_rowmax && (a_xform == OT_AX_GELU || a_xform == OT_AX_NONE)) {
    p.a_rowmax = rms->a_rowmax;
    p.a_rowmax_n = rms->a_rowmax_n;
  }
  if (rms && ((epi & OT_EPI_GELU_BWD) || (epi & ~OT_EPI_C_BF16) == OT_EPI_BIAS)) {   // the stored GELU (optional)
    p.gelu_out = rms->gelu_out;
    p.ldgelu = rms->ldgelu;
  }
  if (rms_flags) {
    p.rstd_out = rms->rstd_out; p.eps = rms->eps;
    p.nx = rms->x; p.ldnx = rms->ldx; p.ngamma = rms->gamma; p.nrstd = rms->rstd;
    p.dres = rms->dres; p.lddres = rms->lddres; p.dres_K = rms->dres_tail_K; p.dres_I = rms->dres_tail_I;
    p.dres_inv = rms->dres_tail_inv;
    p.dxm = rms->dx_masked; p.lddxm = rms->lddxm;
    if ((epi & OT_EPI_ROW_RSTD) && N > GT) p.rowpart = (float*)rms->workspace;
    if ((epi & OT_EPI_ROWDOT) || ((epi & OT_EPI_RMSNORM_BWD) && N > GT)) {
      p.rowdot = rms->rowdot;
      p.rowdot_n = rms->rowdot_n;
    }
    if (epi & OT_EPI_RMSNORM_BWD) {
      // without dgamma the partials still need a home: the caller's workspace or nothing
      dgpart = rms->dgamma ? (float*)rms->workspace : nullptr;
      OT_REQUIRE(dgpart, "ot_mixed_gemm_rms: RMSNorm backward needs dgamma and its workspace");
      p.dgpart = dgpart;
    }
  }
  if (epi & OT_EPI_DROPOUT) {
    OT_REQUIRE(drop_rate >= 0.f && drop_rate < 1.f, "ot_mixed_gemm: drop_rate out of range");
    p.drop_thr = drop_threshold(drop_rate);
    p.drop_scale = 1.f / (1.f - drop_rate);
  }
  const bool split = prec != OT_MATMUL_F32 && mode == OT_GEMM_NT;
  const bool one = prec == OT_MATMUL_BF16;
  const size_t shmem = split ? 4 * GT * SRS * sizeof(uint16_t) : 4 * GT * GLD * sizeof(float);
  auto a16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  const bool vec_ok = ldc % 4 == 0 && a16(C) && (!(epi & OT_EPI_RESIDUAL) || (ldres % 4 == 0 && a16(res))) &&
                      (!(epi & OT_EPI_GELU_BWD) || (ldaux % 4 == 0 && a16(aux))) &&
                      (!(epi & (OT_EPI_BIAS | OT_EPI_ROWDOT)) || (bias_gstride % 4 == 0 && a16(bias)));
  const bool edge = (K % GBK) != 0 || (N % GT) != 0 || !vec_ok;
  OT_REQUIRE(!rms_flags || !edge, "ot_mixed_gemm_rms: needs K %% %d == 0 and 16-B aligned operands", GBK);
  const unsigned nwg = (unsigned)ntiles * p.ntn;
  hipStream_t s = (hipStream_t)stream;
  void (*kern)(GemmArgs) = nullptr;
  bool plane = false;
  int wide_lds = 0;                     // > 0: the wide / big / square plane GEMM (its stage LDS bytes, its kind)
  int wide_kind = 0;
  const int e = epi, x = a_xform;
#define OT_SPEC(NT_, AX_, EP_)                                                                  \
  if (mode == (NT_ ? OT_GEMM_NT : OT_GEMM_NN) && x == AX_ && e == (EP_))                         \
    kern = split ? (one ? (edge ? mixed_gemm_kernel<NT_, AX_, EP_, true, 1> : mixed_gemm_kernel<NT_, AX_, EP_, false, 1>) \
                        : (edge ? mixed_gemm_kernel<NT_, AX_, EP_, true, SPLIT_TERMS>                         \
                                : mixed_gemm_kernel<NT_, AX_, EP_, false, SPLIT_TERMS>))                      \
                 : (edge ? mixed_gemm_kernel<NT_, AX_, EP_, true, 0> : mixed_gemm_kernel<NT_, AX_, EP_, false, 0>);
  OT_SPEC(true, OT_AX_RMSNORM, 0)
  OT_SPEC(true, OT_AX_RMSNORM, OT_EPI_BIAS)
  OT_SPEC(true, OT_AX_GELU, OT_EPI_BIAS | OT_EPI_RESIDUAL | OT_EPI_DROPOUT)
  OT_SPEC(true, OT_AX_GELU, OT_EPI_BIAS | OT_EPI_RESIDUAL)
  OT_SPEC(true, OT_AX_NONE, OT_EPI_RESIDUAL | OT_EPI_DROPOUT)
  OT_SPEC(true, OT_AX_NONE, OT_EPI_RESIDUAL)
  OT_SPEC(true, OT_AX_NONE, OT_EPI_BIAS)
  OT_SPEC(true, OT_AX_NONE, OT_EPI_GELU_BWD)
  OT_SPEC(true, OT_AX_NONE, OT_EPI_GELU_BWD | OT_EPI_ROWDOT)
  OT_SPEC(true, OT_AX_NONE, 0)
  OT_SPEC(true, OT_AX_NONE, OT_EPI_ACCUMULATE)
  OT_SPEC(true, OT_AX_NONE, OT_EPI_RESIDUAL | OT_EPI_DROPOUT | OT_EPI_ROW_RSTD)
  OT_SPEC(true, OT_AX_NONE, OT_EPI_RESIDUAL | OT_EPI_ROW_RSTD)
  OT_SPEC(true, OT_AX_GELU, OT_EPI_BIAS | OT_EPI_RESIDUAL | OT_EPI_DROPOUT | OT_EPI_ROW_RSTD)
  OT_SPEC(true, OT_AX_GELU, OT_EPI_BIAS | OT_EPI_RESIDUAL | OT_EPI_ROW_RSTD)
  OT_SPEC(true, OT_AX_NONE, OT_EPI_RMSNORM_BWD)
  OT_SPEC(true, OT_AX_NONE, OT_EPI_RMSNORM_BWD | OT_EPI_DROPOUT)
#undef OT_SPEC
  // plane GEMM: split mode, pre-split B image given, whole tiles, 16-B aligned A rows
  // (the plane GEMM's k-steps are 16 deep: K % 16 suffices, e.g. the NS tokenizer's K = 432)
  const bool plane_edge = (K % 16) != 0 || (N % GT) != 0 || !vec_ok;
  if (bimg && split && !plane_edge && mode == OT_GEMM_NT && lda % 4 == 0 && a16(A)) {
    OT_REQUIRE(bimg_ntn >= bimg_tn0 + (int)p.ntn && bimg_tn0 >= 0, "ot_mixed_gemm: B image has %d tiles per group, "
               "the GEMM needs %d from tile %d", bimg_ntn, (int)p.ntn, bimg_tn0);
    void (*pk)(GemmArgs) = nullptr;
#define OT_PSPEC(AX_, EP_) \
    if (x == AX_ && e == (EP_)) \
      pk = one ? plane_gemm_kernel<AX_, EP_, PLANE_BF16_NSTG, 4, 1> \
         : (p.a_rowmax ? plane_gemm_kernel<AX_, EP_, 2, 4, ((AX_) == OT_AX_RMSNORM || (AX_) == OT_AX_GELU || (AX_) == OT_AX_NONE) ? 2 : 6> \
                       : plane_gemm_kernel<AX_, EP_, 2, 4, (AX_) == OT_AX_RMSNORM ? 2 : 6>);
    OT_PSPEC(OT_AX_RMSNORM, 0)
    OT_PSPEC(OT_AX_RMSNORM, OT_EPI_BIAS)
    OT_PSPEC(OT_AX_GELU, OT_EPI_BIAS | OT_EPI_RESIDUAL | OT_EPI_DROPOUT)
    OT_PSPEC(OT_AX_GELU, OT_EPI_BIAS | OT_EPI_RESIDUAL)
    OT_PSPEC(OT_AX_GELU, OT_EPI_BIAS | OT_EPI_RESIDUAL | OT_EPI_DROPOUT | OT_EPI_ROW_RSTD)
    OT_PSPEC(OT_AX_GELU, OT_EPI_BIAS | OT_EPI_RESIDUAL | OT_EPI_ROW_RSTD)
    OT_PSPEC(OT_AX_NONE, OT_EPI_RESIDUAL | OT_EPI_DROPOUT)
    OT_PSPEC(OT_AX_NONE, OT_EPI_RESIDUAL)
    OT_PSPEC(OT_AX_NONE, OT_EPI_BIAS)
    OT_PSPEC(OT_AX_NONE, OT_EPI_GELU_BWD)
    OT_PSPEC(OT_AX_NONE, OT_EPI_GELU_BWD | OT_EPI_ROWDOT)
    OT_PSPEC(OT_AX_NONE, 0)
    OT_PSPEC(OT_AX_NONE, OT_EPI_ACCUMULATE)
    OT_PSPEC(OT_AX_NONE, OT_EPI_RESIDUAL | OT_EPI_DROPOUT | OT_EPI_ROW_RSTD)
    OT_PSPEC(OT_AX_NONE, OT_EPI_RESIDUAL | OT_EPI_ROW_RSTD)
    OT_PSPEC(OT_AX_NONE, OT_EPI_RMSNORM_BWD)
    OT_PSPEC(OT_AX_NONE, OT_EPI_RMSNORM_BWD | OT_EPI_DROPOUT)
#undef OT_PSPEC
    if (one && x == OT_AX_NONE && e == (OT_EPI_GELU_BWD | OT_EPI_ROWDOT | OT_EPI_C_BF16))
      pk = plane_gemm_kernel<OT_AX_NONE, OT_EPI_GELU_BWD | OT_EPI_ROWDOT | OT_EPI_C_BF16, PLANE_BF16_NSTG, 4, 1>;
    if (one && x == OT_AX_NONE && e == (OT_EPI_GELU_BWD | OT_EPI_C_BF16))
      pk = plane_gemm_kernel<OT_AX_NONE, OT_EPI_GELU_BWD | OT_EPI_C_BF16, PLANE_BF16_NSTG, 4, 1>;
    if (one && x == OT_AX_NONE && e == (OT_EPI_GELU_BWD | OT_EPI_ROWDOT | OT_EPI_C_BF16 | OT_EPI_AUX_BF16))
      pk = plane_gemm_kernel<OT_AX_NONE, OT_EPI_GELU_BWD | OT_EPI_ROWDOT | OT_EPI_C_BF16 | OT_EPI_AUX_BF16, PLANE_BF16_NSTG, 4, 1>;
    if (one && x == OT_AX_NONE && e == (OT_EPI_GELU_BWD | OT_EPI_C_BF16 | OT_EPI_AUX_BF16))
      pk = plane_gemm_kernel<OT_AX_NONE, OT_EPI_GELU_BWD | OT_EPI_C_BF16 | OT_EPI_AUX_BF16, PLANE_BF16_NSTG, 4, 1>;
    if (one && x == OT_AX_NONE && e == (OT_EPI_GELU_BWD | OT_EPI_ROWDOT | OT_EPI_AUX_BF16))
      pk = plane_gemm_kernel<OT_AX_NONE, OT_EPI_GELU_BWD | OT_EPI_ROWDOT | OT_EPI_AUX_BF16, PLANE_BF16_NSTG, 4, 1>;
    if (one && x == OT_AX_RMSNORM && e == (OT_EPI_BIAS | OT_EPI_C_BF16))
      pk = plane_gemm_kernel<OT_AX_RMSNORM, OT_EPI_BIAS | OT_EPI_C_BF16, PLANE_BF16_NSTG, 4, 1>;
#define OT_PSPEC_BF(EP_) if (one && x == OT_AX_BF16 && e == (EP_)) pk = plane_gemm_kernel<OT_AX_BF16, EP_, PLANE_BF16_NSTG, 4, 1>;
    OT_PSPEC_BF(OT_EPI_BIAS | OT_EPI_RESIDUAL | OT_EPI_DROPOUT)
    OT_PSPEC_BF(OT_EPI_BIAS | OT_EPI_RESIDUAL)
    OT_PSPEC_BF(OT_EPI_BIAS | OT_EPI_RESIDUAL | OT_EPI_DROPOUT | OT_EPI_ROW_RSTD)
    OT_PSPEC_BF(OT_EPI_BIAS | OT_EPI_RESIDUAL | OT_EPI_ROW_RSTD)
    OT_PSPEC_BF(OT_EPI_RMSNORM_BWD)
    OT_PSPEC_BF(OT_EPI_RMSNORM_BWD | OT_EPI_DROPOUT)
    OT_PSPEC_BF(0)
    OT_PSPEC_BF(OT_EPI_GELU_BWD | OT_EPI_ROWDOT | OT_EPI_C_BF16 | OT_EPI_AUX_BF16)
    OT_PSPEC_BF(OT_EPI_GELU_BWD | OT_EPI_ROWDOT | OT_EPI_C_BF16)
#undef OT_PSPEC_BF
#define OT_PSPEC_BR(EP_) if (one && x == OT_AX_BF16_RMSNORM && e == (EP_)) pk = plane_gemm_kernel<OT_AX_BF16_RMSNORM, EP_, PLANE_BF16_NSTG, 4, 1>;
    OT_PSPEC_BR(0)
    OT_PSPEC_BR(OT_EPI_BIAS)
    OT_PSPEC_BR(OT_EPI_BIAS | OT_EPI_C_BF16)
#undef OT_PSPEC_BR
    if (pk) { kern = pk; plane = true; }
    // bf16 mode, whole 256-column tiles and 32-k stages: the wide tile (same outputs)
    // tile: 1 auto, 2 / 3 / 4 force 128 x 256 / 128 x 512 / 256 x 256 (where the shape allows it)
    const int wmode = g_plane_wide.load(std::memory_order_relaxed);
    if (pk && one && wmode && N % PW_COLS == 0 && K % 32 == 0 && !(p.xn_out && K > 1024)) {
      int kind = wmode == 1 ? plane_tile_auto(K, N, ntiles) : wmode - 1;
      if (kind == 2 && N % PB_COLS != 0) kind = 1;
      if (kind == 3 && ntiles % 2 != 0) kind = 1;
      int stage_lds = 0;
      void (*wk)(GemmArgs) = kind ? plane_wide_for(x, e, kind, &stage_lds) : nullptr;
      if (wk) {
        kern = wk;
        wide_lds = stage_lds;
        wide_kind = kind;
      }
    }
  }
  OT_REQUIRE((x != OT_AX_BF16 && x != OT_AX_BF16_RMSNORM) || plane,
             "ot_mixed_gemm: no plane GEMM for a_xform %d with epilogue %d (or edge tiles)", x, epi);
  OT_REQUIRE(!p.c16_out || (plane && one && p.ldc16 % 4 == 0 && ((uintptr_t)p.c16_out % 8) == 0 &&
                            !(epi & (OT_EPI_RMSNORM_BWD | OT_EPI_C_BF16))),
             "ot_mixed_gemm_rms: c16_out needs the bf16-mode plane GEMM (not with OT_EPI_RMSNORM_BWD / C_BF16), "
             "ldc16 %% 4 == 0 and 8-B alignment");
  OT_REQUIRE(!(epi & (OT_EPI_C_BF16 | OT_EPI_AUX_BF16)) || plane,
             "ot_mixed_gemm: OT_EPI_C_BF16 / OT_EPI_AUX_BF16 need the bf16-mode plane GEMM with OT_EPI_GELU_BWD "
             "[| OT_EPI_ROWDOT] or OT_EPI_BIAS alone (epilogue %d)", epi);
  OT_REQUIRE(!p.gelu_out || (!edge && (kern != nullptr) && ((epi & OT_EPI_GELU_BWD) || (plane && one))),
             "ot_mixed_gemm_rms: gelu_out needs whole tiles (with epi OT_EPI_BIAS: the bf16-mode plane GEMM)");
  OT_REQUIRE(!p.xn_out || (plane && one && (x == OT_AX_RMSNORM || x == OT_AX_BF16_RMSNORM) && a_rstd && a_gamma &&
                           p.ldxn % 8 == 0 && K <= 1024 &&
                           ((uintptr_t)p.xn_out % 16) == 0),
             "ot_mixed_gemm_rms: xn_out needs the bf16-mode plane GEMM with the RMSNorm prologue, K <= 1024, ldxn %% 8 == 0 and 16-B "
             "alignment");
  OT_REQUIRE(!p.rowpart || plane, "ot_mixed_gemm_rms: OT_EPI_ROW_RSTD with N = %d > %d needs the plane GEMM "
             "(split mode, a pre-split B image, 16-B aligned A)", N, GT);
  // the row maxima are written by the split-mode plane GEMM's vector epilogue only (the edge kernels' scalar
  // epilogue has no row reduction): refuse a call that would leave them unwritten
  OT_REQUIRE(!p.rowmax_out || (plane && !one && p.rowmax_n == (int)ceil_div(N, GT)),
             "ot_mixed_gemm_rms: rowmax_out needs the split-mode plane GEMM (pre-split B image, whole tiles, 16-B "
             "aligned A) and rowmax_n == ceil(N / %d) = %d (got %d)", GT, (int)ceil_div(N, GT), p.rowmax_n);
  OT_REQUIRE(!p.a_rowmax || p.a_rowmax_n >= 1, "ot_mixed_gemm_rms: a_rowmax needs a_rowmax_n >= 1");
  // the output bound is taken in the vector epilogue (whole tiles; the edge kernels' scalar epilogue has none)
  OT_REQUIRE(!p.rowabs_out || (!edge && kern != nullptr && p.rowabs_n == (int)ceil_div(N, GT)),
             "ot_mixed_gemm_rms: rowabs_out needs a specialised whole-tile kernel and rowabs_n == ceil(N / %d)", GT);
  OT_REQUIRE(!p.amax_out || (!edge && kern != nullptr),
             "ot_mixed_gemm_rms: amax_out needs a specialised whole-tile kernel (K %% 16 == 0, N %% 128 == 0, 16-B "
             "aligned operands)");
  // (+ K floats of gamma behind the stage buffers for the xn_out side output)
  const size_t xn_lds = p.xn_out ? (size_t)K * 4 : 0;
  const size_t launch_shmem = !plane ? shmem
                              : one ? std::max((size_t)PLANE_BF16_NSTG * pg_stage_bytes<1>() + xn_lds,
                                               (size_t)(64 * (GT + 4) + 8 * GT) * 4)
                                    : (size_t)2 * PG_STG_BYTES + xn_lds;
  OT_REQUIRE(kern || !rms_flags, "ot_mixed_gemm_rms: no specialised kernel for epilogue flags %d", epi);
  if (!kern) {   // any other combination: generic instantiation (run-time prologue/epilogue)
    if (mode == OT_GEMM_NT && split && one)
      kern = edge ? mixed_gemm_kernel<true, -1, -1, true, 1> : mixed_gemm_kernel<true, -1, -1, false, 1>;
    else if (mode == OT_GEMM_NT && split)
      kern = edge ? mixed_gemm_kernel<true, -1, -1, true, SPLIT_TERMS> : mixed_gemm_kernel<true, -1, -1, false, SPLIT_TERMS>;
    else if (mode == OT_GEMM_NT)
      kern = edge ? mixed_gemm_kernel<true, -1, -1, true, 0> : mixed_gemm_kernel<true, -1, -1, false, 0>;
    else
      kern = edge ? mixed_gemm_kernel<false, -1, -1, true, 0> : mixed_gemm_kernel<false, -1, -1, false, 0>;
  }
  static std::once_flag lds_once;   // opt every instantiation in to > 64 KiB LDS (gfx950: 160 KiB per CU)
  std::call_once(lds_once, [] {
    const int bytes = (int)std::max(4 * GT * GLD * sizeof(float), 4 * GT * SRS * sizeof(uint16_t));
    for (void (*k)(GemmArgs) : {mixed_gemm_kernel<true, -1, -1, true, 0>, mixed_gemm_kernel<true, -1, -1, false, 0>,
                                mixed_gemm_kernel<false, -1, -1, true, 0>, mixed_gemm_kernel<false, -1, -1, false, 0>,
                                mixed_gemm_kernel<true, -1, -1, true, SPLIT_TERMS>,
                                mixed_gemm_kernel<true, -1, -1, false, SPLIT_TERMS>,
                                mixed_gemm_kernel<true, -1, -1, true, 1>, mixed_gemm_kernel<true, -1, -1, false, 1>})
      (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    (void)hipGetLastError();
  });
  if (wide_lds > 0) {
    const size_t wshm = std::max((size_t)wide_lds + xn_lds, (size_t)(64 * (GT + 4) + 8 * GT) * 4);
    const unsigned wg = wide_kind == 3 ? (unsigned)(ntiles / 2) * (unsigned)(N / PW_COLS)
                                       : (unsigned)ntiles * (unsigned)(N / (wide_kind == 2 ? PB_COLS : PW_COLS));
    hipLaunchKernelGGL(kern, dim3(wg), dim3(wide_kind == 3 ? 512 : 256), wshm, s, p);
  } else {
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(256), launch_shmem, s, p);
  }
  OT_LAUNCH_CHECK("ot_mixed_gemm");
  if (dgpart) {
    launch_colsum_reduce(dgpart, ntiles, N, rms->dgamma, rms->accumulate_dgamma, s, dgpart + (int64_t)ntiles * N);
    OT_LAUNCH_CHECK("ot_mixed_gemm_rms(dgamma)");
  }
  if (p.rowpart) {
    const int64_t nr = (int64_t)ntiles * GT;
    hipLaunchKernelGGL(row_rstd_finish_kernel, dim3(ceil_div(nr, 256)), dim3(256), 0, s, p.rowpart, p.ntn, out_rows,
                       nr, N, rms->eps, rms->rstd_out);
    OT_LAUNCH_CHECK("ot_mixed_gemm_rms(rstd)");
  }
  return OT_OK;
}

extern "C" int ot_mixed_gemm(int mode, const float* A, int64_t lda, int K, const int32_t* in_rows,
                             int a_xform, const float* a_rstd, const float* a_gamma,
                             const float* W, int64_t w_gstride, int64_t ldw, int N,
                             const int32_t* tile_group, int ntiles,
                             const float* bias, int64_t bias_gstride,
                             float* C, int64_t ldc, const int32_t* out_rows, int epi,
                             const float* res, int64_t ldres, int res_tok,
                             const float* aux, int64_t ldaux,
                             uint32_t seed, uint32_t site, float drop_rate, int tail_K, int tail_I,
                             const int32_t* tail_pos, int precision, void* stream) {
  return mixed_gemm_impl(mode, A, lda, K, in_rows, a_xform, a_rstd, a_gamma, W, w_gstride, ldw, N, tile_group,
                         ntiles, bias, bias_gstride, C, ldc, out_rows, epi, res, ldres, res_tok, aux, ldaux, seed,
                         site, drop_rate, tail_K, tail_I, tail_pos, nullptr, nullptr, 0, 0, precision, stream);
}

extern "C" int ot_mixed_gemm_img(int mode, const float* A, int64_t lda, int K, const int32_t* in_rows,
                                 int a_xform, const float* a_rstd, const float* a_gamma,
                                 const float* W, int64_t w_gstride, int64_t ldw, int N,
                                 const int32_t* tile_group, int ntiles,
                                 const float* bias, int64_t bias_gstride,
                                 float* C, int64_t ldc, const int32_t* out_rows, int epi,
                                 const float* res, int64_t ldres, int res_tok,
                                 const float* aux, int64_t ldaux,
                                 uint32_t seed, uint32_t site, float drop_rate, int tail_K, int tail_I,
                                 const int32_t* tail_pos, const uint16_t* b_image, int image_ntn, int image_tn0,
                                 int precision, void* stream) {
  return mixed_gemm_impl(mode, A, lda, K, in_rows, a_xform, a_rstd, a_gamma, W, w_gstride, ldw, N, tile_group,
                         ntiles, bias, bias_gstride, C, ldc, out_rows, epi, res, ldres, res_tok, aux, ldaux, seed,
                         site, drop_rate, tail_K, tail_I, tail_pos, nullptr, b_image, image_ntn, image_tn0, precision, stream);
}

extern "C" size_t ot_split_image_elems(int G, int N, int K) {
  if (G <= 0 || N <= 0 || K <= 0 || K % 16) return 0;
  return (size_t)G * ceil_div(N, GT) * (K / 16) * (PG_B_BYTES / 2);
}

extern "C" int ot_split_images(const float* base, const int64_t* desc_dev, int ndesc, int64_t total_units,
                               uint16_t* img, int precision, void* stream) {
  OT_REQUIRE(base && desc_dev && img && ndesc > 0 && total_units >= 0, "ot_split_images: bad args");
  OT_REQUIRE(precision == OT_MATMUL_SPLIT_BF16 || precision == OT_MATMUL_BF16,
             "ot_split_images: precision %d has no plane images", precision);
  if (total_units == 0) return OT_OK;
  if (precision == OT_MATMUL_SPLIT_BF16) {
    hipLaunchKernelGGL(image_colscale_kernel, dim3((unsigned)total_units), dim3(256), 0, (hipStream_t)stream, base,
                       desc_dev, ndesc, img);
    OT_LAUNCH_CHECK("ot_split_images(column scales)");
  }
  hipLaunchKernelGGL(split_images_kernel, dim3((unsigned)total_units), dim3(256), 0, (hipStream_t)stream, base,
                     desc_dev, ndesc, img, precision == OT_MATMUL_BF16 ? 1 : 0);
  OT_LAUNCH_CHECK("ot_split_images");
  return OT_OK;
}

extern "C" size_t ot_mixed_gemm_rms_workspace_size(int ntiles, int N) {
  const int64_t parts = ntiles > 0 ? ntiles : 1;
  return (size_t)(parts * N + colsum_scratch_floats(parts, N)) * sizeof(float);
}

extern "C" int ot_mixed_gemm_rms(int mode, const float* A, int64_t lda, int K, const int32_t* in_rows,
                                 int a_xform, const float* a_rstd, const float* a_gamma,
                                 const float* W, int64_t w_gstride, int64_t ldw, int N,
                                 const int32_t* tile_group, int ntiles,
                                 const float* bias, int64_t bias_gstride,
                                 float* C, int64_t ldc, const int32_t* out_rows, int epi,
                                 const float* res, int64_t ldres, int res_tok,
                                 const float* aux, int64_t ldaux,
                                 uint32_t seed, uint32_t site, float drop_rate, int tail_K, int tail_I,
                                 const int32_t* tail_pos, const ot_rms_epilogue* rms, int precision, void* stream) {
  OT_REQUIRE(rms, "ot_mixed_gemm_rms: null epilogue operands");
  OT_REQUIRE(rms->struct_size == sizeof(ot_rms_epilogue),
             "ot_mixed_gemm_rms: ot_rms_epilogue.struct_size %zu != %zu (header of another ot_version)",
             rms->struct_size, sizeof(ot_rms_epilogue));
  return mixed_gemm_impl(mode, A, lda, K, in_rows, a_xform, a_rstd, a_gamma, W, w_gstride, ldw, N, tile_group,
                         ntiles, bias, bias_gstride, C, ldc, out_rows, epi, res, ldres, res_tok, aux, ldaux, seed,
                         site, drop_rate, tail_K, tail_I, tail_pos, rms, nullptr, 0, 0, precision, stream);
}

extern "C" int ot_mixed_gemm_rms_img(int mode, const float* A, int64_t lda, int K, const int32_t* in_rows,
                                     int a_xform, const float* a_rstd, const float* a_gamma,
                                     const float* W, int64_t w_gstride, int64_t ldw, int N,
                                     const int32_t* tile_group, int ntiles,
                                     const float* bias, int64_t bias_gstride,
                                     float* C, int64_t ldc, const int32_t* out_rows, int epi,
                                     const float* res, int64_t ldres, int res_tok,
                                     const float* aux, int64_t ldaux,
                                     uint32_t seed, uint32_t site, float drop_rate, int tail_K, int tail_I,
                                     const int32_t* tail_pos, const ot_rms_epilogue* rms, const uint16_t* b_image,
                                     int image_ntn, int image_tn0, int precision, void* stream) {
  OT_REQUIRE(rms, "ot_mixed_gemm_rms: null epilogue operands");
  OT_REQUIRE(rms->struct_size == sizeof(ot_rms_epilogue),
             "ot_mixed_gemm_rms: ot_rms_epilogue.struct_size %zu != %zu (header of another ot_version)",
             rms->struct_size, sizeof(ot_rms_epilogue));
  return mixed_gemm_impl(mode, A, lda, K, in_rows, a_xform, a_rstd, a_gamma, W, w_gstride, ldw, N, tile_group,
                         ntiles, bias, bias_gstride, C, ldc, out_rows, epi, res, ldres, res_tok, aux, ldaux, seed,
                         site, drop_rate, tail_K, tail_I, tail_pos, rms, b_image, image_ntn, image_tn0, precision, stream);
}


// process-wide choice of the bf16 weight-gradient tile (ot_wgrad_wide): 0 128 x 128, 1 auto (256 x 256 where K and N
// allow, else 128 x 256), 2 128 x 256, 3 256 x 256
static std::atomic<int> g_wgrad_wide{OT_WGRAD_WIDE};
extern "C" int ot_wgrad_wide(int on) {
  const int prev = g_wgrad_wide.load();
  if (on >= 0) g_wgrad_wide.store(on > 3 ? 3 : on);
  return prev;
}

extern "C" size_t ot_wgrad_workspace_size(int nchunks, int K, int N) {
  return ((size_t)nchunks * K * N + (size_t)nchunks * N) * sizeof(float);
}

static int wgrad_impl(const float* A, int64_t lda, const int32_t* a_rows, int a_xform,
                      const float* a_rstd, const float* a_gamma,
                      const float* D, int64_t ldd, const int32_t* d_rows, int K, int N,
                      const int32_t* chunks, int nchunks, const int32_t* gchunk, int ngroups,
                      float* dW, int64_t dw_gstride, float* db, int64_t db_gstride,
                      int accumulate, void* workspace, size_t ws_bytes, const float* a_bound, const float* d_bound,
                      int precision, void* stream) {
  OT_REQUIRE(precision == OT_MATMUL_F32 || precision == OT_MATMUL_SPLIT_BF16 || precision == OT_MATMUL_BF16,
             "ot_mixed_gemm_wgrad: unknown precision %d", precision);
  OT_REQUIRE(A && D && dW && chunks && gchunk && workspace, "ot_mixed_gemm_wgrad: null operand");
  OT_REQUIRE(K % 4 == 0 && N % 4 == 0 && lda % 4 == 0 && ldd % 4 == 0 && dw_gstride % 4 == 0,
             "ot_mixed_gemm_wgrad: K, N, lda, ldd, dw_gstride must be multiples of 4");
  OT_REQUIRE(ws_bytes >= ot_wgrad_workspace_size(nchunks, K, N), "ot_mixed_gemm_wgrad: workspace too small");
  const bool dbf = (a_xform & OT_WG_D_BF16) != 0;
  a_xform &= ~OT_WG_D_BF16;
  OT_REQUIRE(a_xform != OT_AX_RMSNORM || (a_rstd && a_gamma), "ot_mixed_gemm_wgrad: rmsnorm prologue needs rstd/gamma");
  OT_REQUIRE(!dbf || (precision == OT_MATMUL_BF16 &&
                      (a_xform == OT_AX_NONE || a_xform == OT_AX_RMSNORM || a_xform == OT_AX_BF16) &&
                      ((uintptr_t)D % 8) == 0),
             "ot_mixed_gemm_wgrad: OT_WG_D_BF16 needs the bf16 mode, A form OT_AX_NONE / OT_AX_RMSNORM and 8-B "
             "aligned D rows");
  hipStream_t s = (hipStream_t)stream;
  float* slab = (float*)workspace;
  float* bslab = db ? slab + (size_t)nchunks * K * N : nullptr;
  if (nchunks > 0) {
    WgradArgs p{A, lda, a_rows, a_xform, a_rstd, a_gamma, D, ldd, d_rows, K, N, chunks, nchunks, slab, bslab,
                (int)ceil_div(K, GT), (int)ceil_div(N, GT), a_bound, d_bound};
    // the scaled fp16 pair: split mode, f32 operands, D's bound given, and A's (or the RMSNorm prologue's own)
    const bool pair = precision == OT_MATMUL_SPLIT_BF16 && !dbf && d_bound &&
                      ((a_xform == OT_AX_RMSNORM) || ((a_xform == OT_AX_NONE || a_xform == OT_AX_GELU) && a_bound));
    const size_t shmem = (OT_WGRAD_DBUF ? 4 : 2) * WBR * WLD * sizeof(float);
    const bool split = precision != OT_MATMUL_F32;
    OT_REQUIRE(a_xform != OT_AX_BF16 || (precision != OT_MATMUL_F32 && lda % 4 == 0 && ((uintptr_t)A % 8) == 0),
               "ot_mixed_gemm_wgrad: OT_AX_BF16 needs the split / bf16 mode and 8-B aligned rows");
    // both operands bf16 with whole 16-B column chunks: the copy-staged kernel
    const bool copy = dbf && a_xform == OT_AX_BF16 && K % 8 == 0 && N % 8 == 0 && lda % 8 == 0 &&
                      ldd % 8 == 0 && ((uintptr_t)A % 16) == 0 && ((uintptr_t)D % 16) == 0 && a_rows == d_rows;
    void (*kern)(WgradArgs) =
        pair ? (a_xform == OT_AX_NONE      ? wgrad_split_kernel<OT_AX_NONE, 2>
                : a_xform == OT_AX_RMSNORM ? wgrad_split_kernel<OT_AX_RMSNORM, 2>
                                           : wgrad_split_kernel<OT_AX_GELU, 2>)
        : copy ? (a_rows ? wgrad_bf16_kernel<true> : wgrad_bf16_kernel<false>)
        : dbf ? (a_xform == OT_AX_NONE      ? wgrad_split_kernel<OT_AX_NONE, 1, true>
                 : a_xform == OT_AX_BF16    ? wgrad_split_kernel<OT_AX_BF16, 1, true>
                                            : wgrad_split_kernel<OT_AX_RMSNORM, 1, true>)
        : a_xform == OT_AX_BF16 ? (precision == OT_MATMUL_BF16 ? wgrad_split_kernel<OT_AX_BF16, 1>
                                                                : wgrad_split_kernel<OT_AX_BF16, SPLIT_TERMS>)
        : precision == OT_MATMUL_BF16
            ? (a_xform == OT_AX_NONE      ? wgrad_split_kernel<OT_AX_NONE, 1>
               : a_xform == OT_AX_RMSNORM ? wgrad_split_kernel<OT_AX_RMSNORM, 1>
               : a_xform == OT_AX_GELU    ? wgrad_split_kernel<OT_AX_GELU, 1>
                                          : wgrad_split_kernel<-1, 1>)
        : split ? (a_xform == OT_AX_NONE      ? wgrad_split_kernel<OT_AX_NONE, SPLIT_TERMS>
                 : a_xform == OT_AX_RMSNORM ? wgrad_split_kernel<OT_AX_RMSNORM, SPLIT_TERMS>
                 : a_xform == OT_AX_GELU    ? wgrad_split_kernel<OT_AX_GELU, SPLIT_TERMS>
                                            : wgrad_split_kernel<-1, SPLIT_TERMS>)
              : (a_xform == OT_AX_NONE      ? wgrad_kernel<OT_AX_NONE>
                 : a_xform == OT_AX_RMSNORM ? wgrad_kernel<OT_AX_RMSNORM>
                 : a_xform == OT_AX_GELU    ? wgrad_kernel<OT_AX_GELU>
                                            : wgrad_kernel<-1>);
    const size_t split_shmem = 2 * WSOP;
    static std::once_flag lds_once;
    std::call_once(lds_once, [] {
      for (void (*k)(WgradArgs) : {wgrad_kernel<OT_AX_NONE>, wgrad_kernel<OT_AX_RMSNORM>, wgrad_kernel<OT_AX_GELU>,
                                   wgrad_kernel<-1>})
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 4 * WBR * WLD * 4);
      (void)hipGetLastError();
    });
    const size_t copy_shmem = (size_t)WG_LDS;
    if (copy && copy_shmem > 64 * 1024) {
      static std::once_flag copy_once;
      std::call_once(copy_once, [] {
        for (void (*k)(WgradArgs) : {wgrad_bf16_kernel<true>, wgrad_bf16_kernel<false>})
          (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, WG_LDS);
        (void)hipGetLastError();
      });
    }
    const int wgw = g_wgrad_wide.load(std::memory_order_relaxed);
    if (copy && N % (2 * GT) == 0 && K % (2 * GT) == 0 && (wgw == 1 || wgw == 3)) {   // 256 x 256
      static std::once_flag sq_once;
      std::call_once(sq_once, [] {
        for (void (*k)(WgradArgs) : {wgrad_bf16_sq_kernel<true>, wgrad_bf16_sq_kernel<false>})
          (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, WS_LDS);
        (void)hipGetLastError();
      });
      hipLaunchKernelGGL(a_rows ? wgrad_bf16_sq_kernel<true> : wgrad_bf16_sq_kernel<false>,
                         dim3(wgrad_grid(nchunks, (K / (2 * GT)) * (N / (2 * GT)))), dim3(512), (size_t)WS_LDS, s, p);
    } else if (copy && N % (2 * GT) == 0 && wgw) {
      static std::once_flag wide_once;
      std::call_once(wide_once, [] {
        for (void (*k)(WgradArgs) : {wgrad_bf16_wide_kernel<true>, wgrad_bf16_wide_kernel<false>})
          (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, WW_LDS);
        (void)hipGetLastError();
      });
      hipLaunchKernelGGL(a_rows ? wgrad_bf16_wide_kernel<true> : wgrad_bf16_wide_kernel<false>,
                         dim3(wgrad_grid(nchunks, p.ntk * (N / (2 * GT)))), dim3(256), (size_t)WW_LDS, s, p);
    } else {
      hipLaunchKernelGGL(kern, dim3(wgrad_grid(nchunks, p.ntk * p.ntn)), dim3(256),
                         copy ? copy_shmem : split ? split_shmem : shmem, s, p);
    }
    OT_LAUNCH_CHECK("ot_mixed_gemm_wgrad");
  }
  const int wblocks = (int)ceil_div((int64_t)K * N / 4, 16);
  const int bblocks = (db && N % 4 == 0) ? (int)ceil_div((int64_t)N / 4, 16) : 0;
  dim3 rg(wblocks + bblocks, ngroups);
  hipLaunchKernelGGL(wgrad_reduce_kernel, rg, dim3(256), 0, s, slab, bslab, gchunk, K, N, dW, dw_gstride, db,
                     db_gstride, accumulate, wblocks);
  OT_LAUNCH_CHECK("ot_mixed_gemm_wgrad(reduce)");
  return OT_OK;
}

extern "C" int ot_mixed_gemm_wgrad(const float* A, int64_t lda, const int32_t* a_rows, int a_xform,
                                   const float* a_rstd, const float* a_gamma,
                                   const float* D, int64_t ldd, const int32_t* d_rows, int K, int N,
                                   const int32_t* chunks, int nchunks, const int32_t* gchunk, int ngroups,
                                   float* dW, int64_t dw_gstride, float* db, int64_t db_gstride,
                                   int accumulate, void* workspace, size_t ws_bytes, int precision,
                                   void* stream) {
  return wgrad_impl(A, lda, a_rows, a_xform, a_rstd, a_gamma, D, ldd, d_rows, K, N, chunks, nchunks, gchunk, ngroups,
                    dW, dw_gstride, db, db_gstride, accumulate, workspace, ws_bytes, nullptr, nullptr, precision,
                    stream);
}

extern "C" int ot_mixed_gemm_wgrad_ex(const float* A, int64_t lda, const int32_t* a_rows, int a_xform,
                                      const float* a_rstd, const float* a_gamma,
                                      const float* D, int64_t ldd, const int32_t* d_rows, int K, int N,
                                      const int32_t* chunks, int nchunks, const int32_t* gchunk, int ngroups,
                                      float* dW, int64_t dw_gstride, float* db, int64_t db_gstride,
                                      int accumulate, void* workspace, size_t ws_bytes, const float* a_bound,
                                      const float* d_bound, int precision, void* stream) {
  return wgrad_impl(A, lda, a_rows, a_xform, a_rstd, a_gamma, D, ldd, d_rows, K, N, chunks, nchunks, gchunk, ngroups,
                    dW, dw_gstride, db, db_gstride, accumulate, workspace, ws_bytes, a_bound, d_bound, precision,
                    stream);
}
