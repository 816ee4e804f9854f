/* onetrans_hip.h — C ABI of libonetrans_hip.so, the gfx950 (MI355X) kernels of the OneTrans
 * ranking training step (fwd + bwd + optimizer).
 *
 * The reference (ScottHCL/recommend, rank/scaling_up/oneTrans/practice) is TensorFlow/Keras with
 * no native code; every entry point below replaces a TF op call site of that model (cited per
 * function as file:line relative to rank/scaling_up/oneTrans/practice/).  The host-side mirror
 * of the reference interface (recommend_amd.OneTransModel / OneTransTrainer) binds this library
 * with ctypes.
 *
 * Conventions
 *  - All tensors are caller-allocated device memory (fp32 activations/weights, int32 row maps,
 *    int64 ids).  The library never allocates, never synchronises the device and keeps no global
 *    mutable state: every call is stream-ordered on `stream` (a hipStream_t passed as void*),
 *    so calls are graph-capturable and thread-safe on distinct streams.
 *  - Scratch memory is passed as (workspace, ws_bytes); size it with the matching
 *    *_workspace_size() function.
 *  - Return 0 (OT_OK) on success, else an OT_ERR_* code; ot_get_last_error_string() describes
 *    the last failure of the calling host thread.
 *  - Row-major 2-D operands are (pointer, leading dimension in elements).  Row maps (int32)
 *    list, per tile row, the source / destination row; -1 marks padding.
 *  - Dropout masks are counter-based: element (token t, column n) of site s is kept iff
 *    fmix32((t*width + n) * 0x9E3779B1 + seed ^ s * 0x85EBCA77) >= rate * 2^32, kept values are
 *    scaled by 1/(1-rate).  A compacted tail row r (the last K of I tokens per sample) maps to
 *    token t = (r / K) * I + (I - K) + r % K, or, when a kept-position map `tail_pos` [B*K]
 *    from ot_pyramid_select is passed, t = (r / K) * I + tail_pos[r].
 */
#ifndef ONETRANS_HIP_H
#define ONETRANS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OT_OK 0
#define OT_ERR_INVALID_ARG 1
#define OT_ERR_UNSUPPORTED 2
#define OT_ERR_HIP 3

/* GEMM modes */
#define OT_GEMM_NN 0 /* C = A @ W[g],   W[g] stored [K][N] (Keras Dense kernel layout) */
#define OT_GEMM_NT 1 /* C = A @ W[g]^T, W[g] stored [N][K] (dgrad through a Keras kernel) */

/* A-load prologues */
#define OT_AX_NONE 0
#define OT_AX_RMSNORM 1 /* a * rstd[in_row] * gamma[k]  (RMSNorm fused into the consumer GEMM) */
#define OT_AX_GELU 2    /* gelu_erf(a)                   (FFN hidden recomputed from its pre-activation) */
#define OT_AX_BF16 4    /* A holds bf16 values (uint16 bits, lda in elements), used as they are (the stored
                           GELU of ot_rms_epilogue.gelu_out).  ot_mixed_gemm_wgrad: OT_MATMUL_BF16 / split
                           modes; forward GEMMs: OT_MATMUL_BF16, NT mode, a B image (the plane GEMM), lda % 8
                           == 0, 16-B aligned A, epilogue OT_EPI_BIAS | OT_EPI_RESIDUAL [| OT_EPI_DROPOUT]
                           [| OT_EPI_ROW_RSTD] (the FFN2 GEMM) */
#define OT_AX_BF16_RMSNORM 5 /* plane GEMM, OT_MATMUL_BF16: A holds bf16 x (as OT_AX_BF16) and the RMSNorm is applied
                                as the RMSNorm prologue is there (gamma folded into the B image, rstd scales the
                                output rows): the QKV / FFN1 GEMMs from the bf16 copy of their input */

/* GEMM epilogue flags (applied in this order) */
#define OT_EPI_BIAS 1        /* + bias[g][n] */
#define OT_EPI_GELU_BWD 2    /* * gelu'(aux[out_row][n]) */
#define OT_EPI_GELU 4        /* gelu_erf(.) */
#define OT_EPI_DROPOUT 8     /* counter-based mask, index (token, n) */
#define OT_EPI_RESIDUAL 16   /* + res[res_tok ? token : out_row][n] */
#define OT_EPI_ACCUMULATE 32 /* C += result */
/* row-norm epilogues (ot_mixed_gemm_rms only): N == 128 (one tile holds whole output rows); OT_EPI_ROW_RSTD
 * also N = 256, 384, ... on the plane GEMM (split mode, ot_mixed_gemm_rms_img; per-tile row sums of
 * squares in the workspace, ot_mixed_gemm_rms_workspace_size(ntiles, N), then a finishing pass);
 * OT_EPI_RMSNORM_BWD also N = 256, 384, ... given the row dots' partials (ot_rms_epilogue.rowdot) */
#define OT_EPI_ROW_RSTD 64      /* rstd_out[out_row] = 1/sqrt(mean_n(C[out_row]^2) + eps), C as above */
#define OT_EPI_ROWDOT 256       /* with OT_EPI_GELU_BWD (ot_mixed_gemm_rms, N % 128 == 0): also
                                   rowdot[out_row * rowdot_n + n / 128] = sum over the tile's columns of
                                   C * (aux - bias[g]) — for the FFN2 dgrad (C = dU, aux = U, bias = b1)
                                   this is the FFN1 norm backward's row dot: sum_f dU_f (U_f - b1_f) =
                                   rstd * <gamma dy, x> (no row-wide reduction needed at d > 128) */
#define OT_EPI_RMSNORM_BWD 128  /* the product is dL/dy of y = RMSNorm(x) * gamma: C = dL/dx (+ dres);
                                   with OT_EPI_DROPOUT also dx_masked = mask(C) (C itself unmasked) */
#define OT_EPI_C_BF16 512       /* C is stored rounded to bf16 (uint16 bits, ldc in elements; 8-B aligned
                                   rows).  Plane GEMM in the bf16 mode, with OT_EPI_GELU_BWD [| OT_EPI_ROWDOT]
                                   [| OT_EPI_AUX_BF16] (the FFN2 dgrad: dU, whose consumers — the FFN1 dgrad
                                   and the W1 weight gradient — round it to bf16 anyway) or with OT_EPI_BIAS
                                   alone (the FFN1 forward: U, read only by the FFN2 dgrad's GELU') */
#define OT_EPI_AUX_BF16 1024    /* with OT_EPI_GELU_BWD: aux holds bf16 (uint16 bits, ldaux in elements) — the
                                   bf16 mode's stored pre-activation U (plane GEMM, OT_MATMUL_BF16 only) */
/* ot_mixed_gemm_wgrad: or'ed into a_xform, D holds bf16 values (uint16 bits, ldd in elements; 8-B aligned
 * rows; OT_MATMUL_BF16 / split modes) — dU stored by OT_EPI_C_BF16 */
#define OT_WG_D_BF16 8

int ot_version(void);
const char* ot_get_last_error_string(void);

/* ---- mixed-parameterisation grouped GEMM (gemm.hip) --------------------------------------
 * Replaces: per-token Q/K/V Dense loop model.py:84-92 (+ weights 38-54, group rule 67-74),
 * Wo model.py:117, per-token FFN loop model.py:154-161 (weights 136-147), tokenizer Dense layers
 * model.py:211-219/254/265, task-head Dense(d/2) model.py:325-330/391, and their gradients
 * (tape.gradient, train.py:131).  Tiles are 128 rows (ot_gemm_tile_rows()); tile i multiplies the
 * rows in_rows[128 i .. 128 i + 127] by W + tile_group[i] * w_gstride. */
int ot_gemm_tile_rows(void);
/* Matmul arithmetic: the `precision` argument of every GEMM, weight-gradient, plane-image and attention
 * entry point (per call: no process-wide state, so models of different precision share the library).
 *   OT_MATMUL_SPLIT_BF16 (default): every f32 operand is split exactly into three bf16 parts
 *     (x = x0 + x1 + x2, 8 significant bits each) and the product is sum_ij ai.bj over the six
 *     largest terms on v_mfma_f32_32x32x16_bf16 (each part product exact in the f32 accumulator;
 *     the dropped a1.b2 + a2.b1 + a2.b2 is below 2^-22 |a||b|, one f32 rounding).  Error vs an
 *     f64 product measured no larger than native f32 (tools/split_gemm_check.py).
 *   OT_MATMUL_F32: native v_mfma_f32_32x32x2_f32.
 *   OT_MATMUL_BF16: reduced precision (BASELINE C5's bf16 configuration, not the reference's f32):
 *     operands rounded to bf16 (nearest even), one v_mfma_f32_32x32x16_bf16 product, f32
 *     accumulation; attention forward and backward likewise.
 * Keras computes these Dense layers in f32 (model.py:38-57, 136-147; default float32 policy). */
#define OT_MATMUL_F32 0
#define OT_MATMUL_SPLIT_BF16 1
#define OT_MATMUL_BF16 2
int ot_mixed_gemm(int mode, const float* A, int64_t lda, int K, const int32_t* in_rows,
                  int a_xform, const float* a_rstd, const float* a_gamma,
                  const float* W, int64_t w_gstride, int64_t ldw, int N,
                  const int32_t* tile_group, int ntiles,
                  const float* bias, int64_t bias_gstride,
                  float* C, int64_t ldc, const int32_t* out_rows, int epi,
                  const float* res, int64_t ldres, int res_tok,
                  const float* aux, int64_t ldaux,
                  uint32_t seed, uint32_t site, float drop_rate, int tail_K, int tail_I,
                  const int32_t* tail_pos, int precision, void* stream);
/* Row-norm epilogue operands for ot_mixed_gemm_rms.  Replaces the RMSNorm layers around the GEMMs
 * (model.py:11-23 RMSNorm, applied at 191/196; their tape gradients): the forward GEMM producing the
 * residual stream emits the next norm's rstd, the dgrad GEMM feeding a norm applies its backward. */
typedef struct ot_rms_epilogue {
  size_t struct_size;                                  /* sizeof(ot_rms_epilogue) of the caller's header: the
                                                          library rejects any other value (OT_ERR_INVALID_ARG)
                                                          instead of reading fields a smaller struct lacks */
  float* rstd_out; float eps;                          /* OT_EPI_ROW_RSTD */
  const float* x; int64_t ldx;                         /* OT_EPI_RMSNORM_BWD: norm input rows (out_row) */
  const float* gamma; const float* rstd;               /*   gamma[N], rstd[out_row] */
  const float* dres; int64_t lddres;                   /*   + dres (row out_row, or through the tail map */
  int dres_tail_K, dres_tail_I;                        /*     b*I+p -> b*K+(p-(I-K)) when dres_tail_K > 0) */
  const int32_t* dres_tail_inv;                        /*     or b*I+p -> inv[b*I+p] (ot_pyramid_select) */
  float* dx_masked; int64_t lddxm;                     /*   with OT_EPI_DROPOUT: GEMM seed/site/rate/tail */
  float* dgamma; int accumulate_dgamma;                /*   dgamma (+)= sum_rows dy * x * rstd */
  void* workspace; size_t ws_bytes;                    /*   ot_mixed_gemm_rms_workspace_size(ntiles, N) */
  float* rowdot; int rowdot_n;                         /* OT_EPI_ROWDOT: output partials [out rows][rowdot_n];
                                                          OT_EPI_RMSNORM_BWD with N > 128: their input (the row
                                                          dot = sum_j rowdot[out_row][j] / rstd) */
  uint16_t* gelu_out; int64_t ldgelu;                  /* optional, whole tiles: also gelu_erf(aux) (with
                                                          OT_EPI_GELU_BWD) or gelu_erf(C) (epi == OT_EPI_BIAS: the
                                                          FFN1 forward, C = U) rounded to bf16 at [out_row][n] —
                                                          the FFN2 GEMM's and its weight gradient's A operand in
                                                          the bf16 mode (OT_AX_BF16): they neither read f32 U nor
                                                          re-evaluate erf.  No other row-norm field is needed */
  uint16_t* xn_out; int64_t ldxn;                      /* optional, with the RMSNorm prologue on the plane GEMM:
                                                          also bf16((A * gamma) * rstd) of every A row [in_row][k]
                                                          (written by the first column tile's workgroups) — the
                                                          normalised operand of the bf16-mode weight gradient
                                                          (OT_AX_BF16), so it neither re-reads f32 A nor
                                                          re-applies the norm */
  uint16_t* c16_out; int64_t ldc16;                    /* optional, bf16-mode plane GEMM (not with the norm-backward
                                                          or bf16-C epilogues): also C rounded to bf16 — the next
                                                          GEMM's OT_AX_BF16_RMSNORM operand */
  float* rowmax_out; int rowmax_n;                     /* optional, split-mode plane GEMM: each 128-column tile's
                                                          largest C value after the bias (signed) at
                                                          [out_row][tile] (rowmax_n = N / 128): the FFN1 forward's
                                                          row maxima of U for the FFN2 GEMM's a_rowmax */
  const float* a_rowmax; int a_rowmax_n;               /* optional, split-mode plane GEMM with the GELU prologue
                                                          (or none: then the parts are max |a|, e.g. rowabs_out /
                                                          ot_dropout_apply_ex / ot_rows_absmax of A's producer):
                                                          the A rows' partial maxima [in_row][a_rowmax_n] (as
                                                          rowmax_out wrote them); the GEMM then multiplies on the
                                                          scaled fp16 pair, the row scale from max(max_j a_rowmax,
                                                          0.17) >= max |gelu(a)|, and b_image must be a pair image
                                                          (desc kscale_off -2, ot_split_images) */
  float* amax_out;                                     /* optional, whole-tile kernels: *amax_out = max(*amax_out,
                                                          max |v|) over the values v the epilogue stores for the next
                                                          consumer (dx_masked when written, else C), by one atomic
                                                          per wave (order-independent, deterministic); the caller
                                                          zeroes it first.  The |D| / |A| bound of the fp16-pair
                                                          weight gradient (ot_mixed_gemm_wgrad_ex) */
  float* rowabs_out; int rowabs_n;                     /* optional, whole-tile kernels: each 128-column tile's max
                                                          |v| of every output row (v as for amax_out) at
                                                          [out_row][tile], rowabs_n = ceil(N / 128): the row bounds
                                                          (a_rowmax) of an fp16-pair consumer GEMM whose A this is */
} ot_rms_epilogue;
size_t ot_mixed_gemm_rms_workspace_size(int ntiles, int N);
int ot_mixed_gemm_rms(int mode, const float* A, int64_t lda, int K, const int32_t* in_rows,
                      int a_xform, const float* a_rstd, const float* a_gamma,
                      const float* W, int64_t w_gstride, int64_t ldw, int N,
                      const int32_t* tile_group, int ntiles,
                      const float* bias, int64_t bias_gstride,
                      float* C, int64_t ldc, const int32_t* out_rows, int epi,
                      const float* res, int64_t ldres, int res_tok,
                      const float* aux, int64_t ldaux,
                      uint32_t seed, uint32_t site, float drop_rate, int tail_K, int tail_I,
                      const int32_t* tail_pos, const ot_rms_epilogue* rms, int precision, void* stream);

/* dW[g] (+)= sum pro(A[a_rows])^T D[d_rows], db[g] (+)= sum D[d_rows] over the rows of every
 * chunk of group g.  chunks: [nchunks][3] {group, row_begin, row_count} indexing the row maps;
 * gchunk: [ngroups][2] {first chunk, chunk count} (a group's chunks are contiguous).
 * Deterministic: per-chunk partial slabs summed in chunk order. */
size_t ot_wgrad_workspace_size(int nchunks, int K, int N);
int ot_mixed_gemm_wgrad(const float* A, int64_t lda, const int32_t* a_rows, int a_xform,
                        const float* a_rstd, const float* a_gamma,
                        const float* D, int64_t ldd, const int32_t* d_rows, int K, int N,
                        const int32_t* chunks, int nchunks, const int32_t* gchunk, int ngroups,
                        float* dW, int64_t dw_gstride, float* db, int64_t db_gstride,
                        int accumulate, void* workspace, size_t ws_bytes, int precision, void* stream);

/* ot_mixed_gemm_wgrad on the scaled fp16 pair (OT_MATMUL_SPLIT_BF16, f32 operands, a_xform OT_AX_NONE /
 * OT_AX_RMSNORM / OT_AX_GELU): A column k and D are scaled by powers of two from magnitude bounds and split into an
 * fp16 pair (x s = h + l, 22 significant bits of each element down to 2^-16 of its bound), three f16 products per
 * f32 product instead of the six bf16 ones.  d_bound: one float >= max |D| over the rows used; a_bound: one float
 * >= max |A'| of the transformed A (GELU: >= max |A|, since |gelu(u)| <= |u|), not needed with OT_AX_RMSNORM
 * (|x_k rstd gamma_k| <= sqrt(K) |gamma_k|).  The bounds are device pointers, typically the amax outputs of the
 * operands' producers (ot_rms_epilogue.amax_out, ot_dropout_apply_ex, ot_attn_fwd_amax, ot_attn_bwd_amax).
 * With d_bound NULL (or a_bound NULL where needed, or another mode / form) the call is ot_mixed_gemm_wgrad. */
int ot_mixed_gemm_wgrad_ex(const float* A, int64_t lda, const int32_t* a_rows, int a_xform,
                           const float* a_rstd, const float* a_gamma,
                           const float* D, int64_t ldd, const int32_t* d_rows, int K, int N,
                           const int32_t* chunks, int nchunks, const int32_t* gchunk, int ngroups,
                           float* dW, int64_t dw_gstride, float* db, int64_t db_gstride,
                           int accumulate, void* workspace, size_t ws_bytes, const float* a_bound,
                           const float* d_bound, int precision, void* stream);

/* Transposed weight shadow for the forward GEMMs (NT staging reads k-contiguous rows):
 * dst[g][n][k] = src[g][k][n] per bank; banks_dev: [nbanks][6] int64 {src_off, dst_off, G, K, N,
 * first_tile}, a bank owning G*ceil(K/32)*ceil(N/32) consecutive 32x32 tiles of the launch. */
int ot_transpose_banks(const float* src, float* dst, const int64_t* banks_dev, int nbanks, int64_t total_tiles,
                       void* stream);

/* Pre-split B images for the plane GEMM (split-bf16 mode).  A weight bank used as the B operand
 * B[g][n][k] = src[g*gstride + n*sn + k*sk] (* kscale[k] when kscale_off >= 0: an RMSNorm gamma folded
 * into the weights, x*rstd*gamma @ W = rstd * (x @ (gamma W))) is written once per weight update as
 * its three exact bf16 planes, one 12-KiB block per (g, 128-column tile, 16-k stage) in the LDS image
 * the GEMM reads — except a gamma-folded bank (the RMSNorm-prologue GEMMs'), written as the scaled fp16
 * pair of B[g][n][k] s_n (s_n a power of two per column n putting its largest magnitude in [2^13, 2^14),
 * stored as 128 floats in the third plane of the tile's first block), which those GEMMs multiply with three
 * f16 products (A scaled per row from the bound |x| <= sqrt(K) / rstd).  desc_dev: [ndesc][10] int64 {src_off, sn, sk, gstride, kscale_off, dst_off
 * (elements of img), first_unit, G, N, K} (offsets into base; K % 16 == 0; kscale_off -1: none, -2: none
 * and the pair form — the FFN2 forward's W2 image, read with ot_rms_epilogue.a_rowmax); a bank owns
 * G*ceil(N/128)*(K/16) consecutive units of the launch; ot_split_image_elems gives its size. */
size_t ot_split_image_elems(int G, int N, int K);
int ot_split_images(const float* base, const int64_t* desc_dev, int ndesc, int64_t total_units, uint16_t* img,
                    int precision, void* stream);
/* ot_mixed_gemm / ot_mixed_gemm_rms with the B operand's pre-split image (b_image: the bank's image,
 * image_ntn column tiles per group, the GEMM's columns starting at tile image_tn0).  In split mode,
 * NT, whole tiles and 16-B aligned A rows the plane GEMM runs (B by global_load_lds from the image,
 * A split once per tile at fragment time); with a_xform = OT_AX_RMSNORM the image must carry gamma
 * (kscale) and only a_rstd is read.  Otherwise the call is ot_mixed_gemm / ot_mixed_gemm_rms. */
int ot_mixed_gemm_img(int mode, const float* A, int64_t lda, int K, const int32_t* in_rows,
                      int a_xform, const float* a_rstd, const float* a_gamma,
                      const float* W, int64_t w_gstride, int64_t ldw, int N,
                      const int32_t* tile_group, int ntiles,
                      const float* bias, int64_t bias_gstride,
                      float* C, int64_t ldc, const int32_t* out_rows, int epi,
                      const float* res, int64_t ldres, int res_tok,
                      const float* aux, int64_t ldaux,
                      uint32_t seed, uint32_t site, float drop_rate, int tail_K, int tail_I,
                      const int32_t* tail_pos, const uint16_t* b_image, int image_ntn, int image_tn0,
                      int precision, void* stream);
/* The bf16-mode plane GEMM's tile for N % 256 == 0, K % 32 == 0: 0 = 128 x 128, 1 = auto (default: 128 x 256 when
 * N <= K, else 128 x 128), 2 / 3 / 4 = 128 x 256 / 128 x 512 / 256 x 256 where the shape allows; every tile gives
 * the same outputs bit for bit (fewer L2 -> LDS bytes per MFMA on the larger ones).  Process-wide; on = -1 only
 * queries; returns the previous setting.  A tuning and test knob. */
int ot_plane_wide(int on);
/* The bf16 weight gradient's (OT_WG_D_BF16 with OT_AX_BF16 A) tile: 0 = 128 x 128, 1 = auto (default: 256 x 256
 * where K % 256 == N % 256 == 0, else 128 x 256 where N % 256 == 0), 2 = 128 x 256, 3 = 256 x 256; the same slabs
 * bit for bit.  Same switch semantics as ot_plane_wide. */
int ot_wgrad_wide(int on);
int ot_mixed_gemm_rms_img(int mode, const float* A, int64_t lda, int K, const int32_t* in_rows,
                          int a_xform, const float* a_rstd, const float* a_gamma,
                          const float* W, int64_t w_gstride, int64_t ldw, int N,
                          const int32_t* tile_group, int ntiles,
                          const float* bias, int64_t bias_gstride,
                          float* C, int64_t ldc, const int32_t* out_rows, int epi,
                          const float* res, int64_t ldres, int res_tok,
                          const float* aux, int64_t ldaux,
                          uint32_t seed, uint32_t site, float drop_rate, int tail_K, int tail_I,
                          const int32_t* tail_pos, const ot_rms_epilogue* rms, const uint16_t* b_image,
                          int image_ntn, int image_tn0, int precision, void* stream);

/* ---- causal attention with a query tail (attention.hip) ----------------------------------
 * Replaces model.py:100-114 (einsum QK^T/sqrt(hd), band_part mask with -1e9, softmax, einsum PV)
 * and the pyramid gather of queries model.py:356/371 (only the last K of I queries computed).
 * qkv: [B*I, ld] (q | k | v, head h at +h*head_dim); out: [B*K, H*head_dim]; lse: [B, H, K].
 * qpos: NULL (query j of a sample sits at position I - K + j) or the ascending kept positions
 * [B*K] of ot_pyramid_select (query j at qpos[b*K + j], causal limit key <= qpos). */
int ot_attn_fwd(const float* qkv, int64_t ld, int B, int H, int I, int K, const int32_t* qpos,
                int head_dim, float* out, float* lse, int precision, void* stream);
/* The same forward on block-scaled fp8 MFMA (attention_fp8.hip; BASELINE configs[4] "CDNA4 fp8 MFMA
 * attention"): K and Q quantised to OCP e4m3 with one e8m0 scale per (row, 32 dims), V with one scale
 * per (dim, 64 keys), P = exp(s - m) as e4m3 of P * 2^8; v_mfma_scale_f32_32x32x64_f8f6f4 for QK^T and
 * PV, softmax statistics and O accumulation in f32.  head_dim 64 or 128.  Reduced precision (not the
 * reference's f32): out / lse as ot_attn_fwd within the fp8 bounds of tests/test_attn_fp8_gpu.py.
 * workspace: ot_attn_fwd_fp8_workspace_size(B, H, I, head_dim) bytes, 16-B aligned (the packed
 * fp8 K / V^T images and their scales). */
size_t ot_attn_fwd_fp8_workspace_size(int B, int H, int I, int head_dim);
int ot_attn_fwd_fp8(const float* qkv, int64_t ld, int B, int H, int I, int K, const int32_t* qpos,
                    int head_dim, float* out, float* lse, void* workspace, size_t ws_bytes, void* stream);
/* flags of ot_attn_fwd_fp8_ex */
#define OT_FP8_DEQUANT 1 /* training: overwrite qkv's Q (kept query rows), K and V with their dequantised fp8
                          * values, so ot_attn_bwd in the bf16 GEMM mode recomputes S from (nearly) the operands
                          * the fp8 forward used.  One term (e4m3 x block scale) is exact in bf16 and the
                          * backward's P then matches this lse up to summation order.  With OT_FP8_TWO_TERM the
                          * dequantised value hi + lo has more than bf16's 8 significant bits (the bf16 backward
                          * rounds it) and the forward dropped the lo.lo product, so the recomputed S differs from
                          * the forward's by those two terms: the straight-through gradient is approximate
                          * (tests/test_attn_fp8_gpu.py: 0.5-1% of max|g| from the exact attention gradient) */
#define OT_FP8_TWO_TERM 2 /* two-term e4m3 operands: every Q / K / V / P element as hi = e4m3(x) plus lo =
                           * e4m3(x - hi), each with its own block scale; QK^T and PV as three fp8 MFMA
                           * products (hi.hi + hi.lo + lo.hi): ~7 significant bits per operand */
int ot_attn_fwd_fp8_ex(float* qkv, int64_t ld, int B, int H, int I, int K, const int32_t* qpos, int head_dim,
                       float* out, float* lse, void* workspace, size_t ws_bytes, int flags, void* stream);
/* ot_attn_fwd_fp8_ex with OT_FP8_DEQUANT implied and the dequantised Q (kept rows) / K / V written rounded to
 * bf16 into deq16 ([B*I][ld] uint16, the qkv layout; 16-B aligned, ld % 8 == 0) instead of in place: the
 * bf16 backward's operands (OT_ATTN_QKV_BF16), which it would round so anyway; qkv is only read */
int ot_attn_fwd_fp8_deq16(const float* qkv, int64_t ld, int B, int H, int I, int K, const int32_t* qpos,
                          int head_dim, float* out, float* lse, void* workspace, size_t ws_bytes, int flags,
                          uint16_t* deq16, void* stream);
/* dqkv: like qkv (dq written on the K kept query rows only; dk, dv on all rows);
 * ws: ot_attn_bwd_workspace_size(B, H, K) bytes (row stats padded to 32 queries per (b, h)) */
size_t ot_attn_bwd_workspace_size(int B, int H, int K);
int ot_attn_bwd(const float* qkv, int64_t ld, const float* out, const float* dout, const float* lse,
                int B, int H, int I, int K, const int32_t* qpos, int head_dim, float* dqkv, float* delta_ws,
                int precision, void* stream);
/* ot_attn_bwd with a sized workspace: given ot_attn_bwd_ex_workspace_size(B, H, I, K, head_dim,
 * qpos != NULL, precision) bytes, the bf16-mode backward splits each (sample, head)'s key blocks over several
 * waves when B*H alone cannot fill the chip (C5: 4 slices), their dQ partials summed in a fixed
 * order (deterministic); with ot_attn_bwd_workspace_size bytes it runs as ot_attn_bwd. */
size_t ot_attn_bwd_ex_workspace_size(int B, int H, int I, int K, int head_dim, int selected, int precision);
int ot_attn_bwd_ex(const float* qkv, int64_t ld, const float* out, const float* dout, const float* lse,
                   int B, int H, int I, int K, const int32_t* qpos, int head_dim, float* dqkv, void* workspace,
                   size_t ws_bytes, int precision, void* stream);
/* ot_attn_bwd_ex with output flags.  OT_ATTN_DQKV_BF16: dqkv holds bf16 (uint16 bits, ld in elements,
 * 8-B aligned) — the bf16 mode's consumers (the QKV dgrad's A operand, the Wqkv weight gradient's D) round
 * it to bf16 anyway, so the values they use are unchanged (each element is the f32 result rounded once).
 * Key-grouped backward only (ot_attn_bwd_dqkv_bf16_supported); workspace
 * ot_attn_bwd_flags_workspace_size (one more [B*K][H*head_dim] f32 dQ slot: slice 0's). */
#define OT_ATTN_DQKV_BF16 1
/* OT_ATTN_QKV_BF16: qkv holds bf16 (uint16 bits, ld in elements, 16-B aligned): the fp8 forward's dequantised
 * operands from ot_attn_fwd_fp8_deq16 (same key-grouped condition) */
#define OT_ATTN_QKV_BF16 2
/* OT_ATTN_DQ_PART_BF16 (with OT_ATTN_DQKV_BF16): the key slices' dQ partials are kept in bf16 (summed in f32,
 * then rounded: not the f32 sum rounded once — about one more bf16 rounding of each partial) */
#define OT_ATTN_DQ_PART_BF16 4
int ot_attn_bwd_dqkv_bf16_supported(int I, int K, int head_dim, int selected, int precision);
/* the OT_ATTN_*_BF16 flags the backward supports at this shape: all three on the key-grouped bf16 backward,
 * OT_ATTN_DQKV_BF16 alone on the short-tail kernel (K <= 4: the last layer after DCE), none otherwise */
int ot_attn_bwd_bf16_forms(int I, int K, int head_dim, int selected, int precision);
/* (in the f32-accurate mode it also covers the head_dim-64 slice backward's dS scratch: one causal block pair
 * store per co-resident workgroup, two per CU — one per CU for the long form, K <= 272 / I <= 544; a smaller
 * workspace shrinks that kernel's grid, and below one workgroup's share per CU the long forms (I > 144) are not
 * taken: the per-pair f32 backward runs instead) */
size_t ot_attn_bwd_flags_workspace_size(int B, int H, int I, int K, int head_dim, int selected, int flags, int precision);
/* 1 when the f32-accurate mode (OT_MATMUL_SPLIT_BF16) runs this shape's forward and backward as one
 * workgroup per (sample, head) slice on split MFMA (attention_slice.hip: head_dim 32 / 64, I <= 192,
 * tail queries for the backward, the slice's planes within LDS; the dS store in LDS at head_dim 32, in the
 * workspace at 64), else 0.  (The backward alone also takes head_dim 64 up to I 544 / K 272 on the slice
 * kernels, with a forward from attn_fwd_split_kernel: ot_attn_bwd_flags_workspace_size then exceeds
 * ot_attn_bwd_workspace_size by its dS scratch.) */
int ot_attn_slice_supported(int I, int K, int head_dim, int selected);
int ot_attn_bwd_flags(const float* qkv, int64_t ld, const float* out, const float* dout, const float* lse,
                      int B, int H, int I, int K, const int32_t* qpos, int head_dim, void* dqkv, int flags,
                      void* workspace, size_t ws_bytes, int precision, void* stream);
/* Output bounds for the fp16-pair weight gradients (ot_mixed_gemm_wgrad_ex): ot_attn_fwd / ot_attn_bwd_ex that also
 * fold max |O| (forward) or max |dQKV| (backward) into *amax (one float the caller zeroes; atomic max, deterministic).
 * Only where the slice kernels run the shape — ot_attn_amax_supported: bit 1 the forward (OT_MATMUL_SPLIT_BF16, K > 4,
 * the slice forward's shapes), bit 2 the backward (also qpos NULL, the slice backward's shapes; it needs
 * ot_attn_bwd_flags_workspace_size bytes) — elsewhere the call is refused. */
int ot_attn_amax_supported(int I, int K, int head_dim, int selected, int precision);
/* rowmax (optional, either may be NULL): per-row maxima of |output| for an fp16-pair dgrad consumer's a_rowmax —
 * forward [B*K][H] (row b*K + j, head h: max |O| over the head's columns), backward [B*I][3][H] (row b*I + p: the dQ,
 * dK, dV parts per head; with K < I the dQ part of the rows without a query is not written: zero the array first) */
int ot_attn_fwd_amax(const float* qkv, int64_t ld, int B, int H, int I, int K, const int32_t* qpos,
                     int head_dim, float* out, float* lse, float* amax, float* rowmax, int precision, void* stream);
int ot_attn_bwd_amax(const float* qkv, int64_t ld, const float* out, const float* dout, const float* lse,
                     int B, int H, int I, int K, const int32_t* qpos, int head_dim, float* dqkv,
                     void* workspace, size_t ws_bytes, float* amax, float* rowmax, int precision, void* stream);

/* Two-stage cached serving (paper §3.5.1; replaces the reference's defective cache path
 * model.py:94-98, 359-381, D6): candidate c (request req[c]) attends with the last Kq of its n
 * N-side rows (qkv [C*n, ld], q | k | v) over its request's Ic cached S-side rows (kv_cache
 * [R*Ic, ldc], k at col 0, v at col d) and its own n rows, causally (query j at absolute position
 * Ic + n - Kq + j).  out: [C*Kq, H*head_dim].  Forward only. */
int ot_attn_fwd_cached(const float* qkv, int64_t ld, const float* kv_cache, int64_t ldc, const int32_t* req,
                       int C, int H, int Ic, int n, int Kq, int head_dim, float* out, void* stream);

/* ---- pyramid query selection (pyramid.hip) -----------------------------------------------
 * Replaces PyramidScheduler.get_layer_config + tf.gather (model.py:287-302, 356, 371): per sample,
 * keep the K of I tokens with the largest key (score[b*I+p] * score_sign, ties to the later
 * position), the last `nforce` (<= K) positions always kept, positions emitted ascending.  score NULL =
 * every score equal = the reference's tail slice (range(I-K, I), D2-fixed).  One wavefront per
 * sample: bitwise radix select of the K-th key by ballot/popcount, ordered compaction by mbcnt.
 * pos [B*K]: kept positions; inv [B*I] (optional): compact row b*K+j of token row b*I+p, or -1;
 * map_rows (optional): map_rows[b*map_per_sample + j] = b*I + pos[b*K+j] for j < map_per_sample
 * (rewrites the shared-group part of a tail row map, layout.layer_maps).  I <= 4096. */
int ot_pyramid_select(const float* score, float score_sign, int B, int I, int K, int nforce,
                      int32_t* pos, int32_t* inv, int32_t* map_rows, int map_per_sample, void* stream);

/* ---- row-wise kernels (rowwise.hip) -------------------------------------------------------
 * RMSNorm model.py:19-23 (forward writes rstd, and y only when asked: the output norm
 * model.py:384); dropout model.py:184/193/198. */
int ot_rmsnorm_fwd(const float* x, int64_t ldx, const float* gamma, float* y, int64_t ldy, float* rstd,
                   int64_t rows, int d, float eps, void* stream);
size_t ot_rmsnorm_bwd_workspace_size(int64_t rows, int d);
/* dres (residual-branch gradient added to dx): when dres_tail_K > 0 it holds only the compact tail
 * rows (last dres_tail_K of every dres_tail_I rows of x); the other rows get no residual term. */
int ot_rmsnorm_bwd(const float* dy, int64_t lddy, const float* x, int64_t ldx, const float* gamma,
                   const float* rstd, const float* dres, int64_t lddres, int dres_tail_K, int dres_tail_I,
                   const int32_t* dres_tail_inv, float* dx, int64_t lddx,
                   float* dx_masked, int64_t lddxm, uint32_t seed, uint32_t site, float drop_rate,
                   int tail_K, int tail_I, const int32_t* tail_pos, float* dgamma, int accumulate_dgamma, int64_t rows, int d,
                   void* workspace, size_t ws_bytes, void* stream);
int ot_dropout_apply(const float* src, int64_t lds, float* dst, int64_t ldd, int64_t rows, int d,
                     uint32_t seed, uint32_t site, float drop_rate, int tail_K, int tail_I,
                     const int32_t* tail_pos, void* stream);
/* ot_dropout_apply that also reports the output's magnitude for fp16-pair consumers: amax (optional, one float the
 * caller zeroes) = max(*amax, max |out|) (atomic, order-independent); rowmax (optional, [rows][rowmax_n], rowmax_n =
 * ceil(d / 256), d / 4 a power of two or a multiple of 64) = max |out| of each row's 256-column parts */
int ot_dropout_apply_ex(const float* src, int64_t lds, float* dst, int64_t ldd, int64_t rows, int d,
                        uint32_t seed, uint32_t site, float drop_rate, int tail_K, int tail_I,
                        const int32_t* tail_pos, float* amax, float* rowmax, int rowmax_n, void* stream);
/* out[r][j] = max |x[r][c]| over c in [256 j, 256 j + 256) (parts = ceil(d / 256)): the row bounds (a_rowmax) of an
 * fp16-pair GEMM whose A has no producer that reports them */
int ot_rows_absmax(const float* x, int64_t ldx, int64_t rows, int d, float* out, int parts, void* stream);
/* ot_dropout_apply with the masked rows stored rounded to bf16 (uint16 bits, ldd in elements): the bf16
 * mode's dY of the FFN2 GEMM, whose consumers (the FFN2 dgrad's A operand, the W2 weight gradient's D)
 * round it to bf16 anyway */
int ot_dropout_apply_bf16(const float* src, int64_t lds, uint16_t* dst, int64_t ldd, int64_t rows, int d,
                          uint32_t seed, uint32_t site, float drop_rate, int tail_K, int tail_I,
                          const int32_t* tail_pos, void* stream);
size_t ot_rows_colsum_workspace_size(int64_t nrows, int ncols);
int ot_rows_colsum(const float* src, int64_t ld, const int32_t* rows, int64_t nrows, int ncols,
                   float* out, int accumulate, void* workspace, size_t ws_bytes, void* stream);

/* ---- tokenizer + heads + loss (model_io.hip) ---------------------------------------------- */
typedef struct {
  const float* dense;   /* [B] float feature (stride dense_stride) or NULL */
  const int64_t* ids;   /* [B] ids (stride ids_stride) for an embedding feature, or NULL */
  int64_t row_offset;   /* row of id 0 in the (concatenated) table */
  int64_t stride;       /* element stride between samples of `dense` / `ids` */
  int col;              /* first destination column */
  int width;            /* 1 for dense, embedding width for ids */
} ot_ns_field;
/* NS feature concat model.py:243-253 (+ embedding gather for id features):
 * out[b][col .. col+width) = table[row_offset + ids[b]] or dense[b]; columns >= F are untouched. */
int ot_ns_assemble(const ot_ns_field* fields_dev, int nfields, const float* table, int B, float* out,
                   int64_t ld_out, void* stream);
/* Pack the NS embedding-feature gradients of ot_ns_assemble: keys[f*B + b] = row_offset+ids[b],
 * grads[f*B + b][:] = dmat[b][col .. col+width) for the nsparse id fields (equal width). */
int ot_ns_grad_pack(const ot_ns_field* fields_dev, int nsparse, int width, const float* dmat, int64_t ld,
                    int B, int64_t* keys, float* grads, void* stream);
/* [SEP] placement model.py:270-272: dst[rows[i]][:] = vec[:] */
int ot_fill_rows(float* dst, int64_t ld, const int32_t* rows, int64_t nrows, const float* vec, int d,
                 void* stream);
/* Row maps of the per-sequence projection GEMM model.py:262-265: in_rows[m] = ids (item id) of
 * sequence element m; sequences concatenated, tiles padded to ot_gemm_tile_rows(). */
int ot_seq_rows(const int64_t* ids, int64_t ids_stride_b, int B, int L, int64_t vocab, int32_t* in_rows,
                void* stream);
/* Task heads model.py:388-391: logits[t][b] = gelu(pre1[t*B+b]) . w2[t] + b2[t], probs = sigmoid */
int ot_head_fwd(const float* pre1, const float* w2, const float* b2, int T, int B, int dh,
                float* logits, float* probs, void* stream);
size_t ot_head_bwd_workspace_size(int T, int B, int dh);
int ot_head_bwd(const float* pre1, const float* w2, const float* probs, const float* dprobs, int T, int B,
                int dh, float* dpre1, float* dw2, float* db2, int64_t task_stride_w2, int64_t task_stride_b2,
                int accumulate, void* workspace, size_t ws_bytes, void* stream);
/* ot_head_bwd with the loss gradient given w.r.t. the logits and / or the probabilities (either may be null):
 * dz = dlogits + dprobs * p (1 - p).  The model's training path passes dlogits (ot_task_loss_logits_bwd). */
int ot_head_bwd_ex(const float* pre1, const float* w2, const float* probs, const float* dprobs, const float* dlogits,
                   int T, int B, int dh, float* dpre1, float* dw2, float* db2, int64_t task_stride_w2,
                   int64_t task_stride_b2, int accumulate, void* workspace, size_t ws_bytes, void* stream);
/* The task loss of train.py:78-93 as the reference's Keras 2.12 evaluates it on its sigmoid heads (model.py:327-329,
 * train.py:84-87, 124-128): keras.activations.sigmoid caches its input as the output's _keras_logits and
 * keras.backend.binary_crossentropy(from_logits=False) then computes tf.nn.sigmoid_cross_entropy_with_logits:
 *   BCE task t:  mean_b  max(z, 0) - z y + log(1 + exp(-|z|))      (z = logits[t][b]; no clipping)
 *   MSE task t (bit t of mse_mask, tasks other than 'ctr' / 'cvr'):  mean_b (y - p)^2
 * loss = sum over the T <= 32 tasks.  Workspace: ot_bce_workspace_size.
 * bwd: dlogits = gscale[0] * d loss / d z = gscale (p - y) / B (BCE), gscale 2 (p - y) p (1 - p) / B (MSE). */
int ot_task_loss_logits_fwd(const float* logits, const float* probs, const float* labels, int T, int B,
                            unsigned mse_mask, float* loss, void* workspace, size_t ws_bytes, void* stream);
int ot_task_loss_logits_bwd(const float* probs, const float* labels, const float* gscale, int T, int B,
                            unsigned mse_mask, float* dlogits, void* stream);
/* The probability form (a caller holding only probabilities: Keras without a cached logit):
 * tf.keras.losses.BinaryCrossentropy(from_logits=False) summed over tasks,
 * loss = sum_t mean_b -(y log(clip(p)+eps) + (1-y) log(1-clip(p)+eps)). */
size_t ot_bce_workspace_size(int T, int B);
int ot_bce_fwd(const float* probs, const float* labels, int T, int B, float* loss, void* workspace,
               size_t ws_bytes, void* stream);
/* dprobs = gscale[0] * d loss / d probs (zero where p was clipped) */
int ot_bce_bwd(const float* probs, const float* labels, const float* gscale, int T, int B, float* dprobs,
               void* stream);
/* Per-task loss of train.py:78-93: task t is tf.keras.losses.MeanSquaredError (SUM_OVER_BATCH_SIZE:
 * mean_b (y - p)^2) when bit t of mse_mask is set (tasks other than 'ctr'/'cvr'), the BCE above
 * otherwise; loss = sum over the T <= 32 tasks.  ot_bce_* == mse_mask 0.  Workspace: ot_bce_workspace_size. */
int ot_task_loss_fwd(const float* probs, const float* labels, int T, int B, unsigned mse_mask, float* loss,
                     void* workspace, size_t ws_bytes, void* stream);
int ot_task_loss_bwd(const float* probs, const float* labels, const float* gscale, int T, int B,
                     unsigned mse_mask, float* dprobs, void* stream);

/* ---- sparse embedding update (embedding.hip) ----------------------------------------------
 * Build extension (no reference site; paper: sparse Adagrad, clip 120, complete_translation.md:190).
 * Keras-2.12 Adagrad on a de-duplicated gradient: rows sorted (rocPRIM radix sort, stable) and
 * summed per unique key in a fixed order (deterministic), clip_by_norm(clip) over the unique-row
 * gradient, then acc[r] += g^2; w[r] -= lr g / sqrt(acc[r] + eps). */
size_t ot_sparse_adagrad_workspace_size(int64_t n, int E);
int ot_sparse_adagrad(float* table, float* accum, int E, int64_t num_rows, const int64_t* keys,
                      const float* grads, int64_t n, float lr, float eps, float clip,
                      void* workspace, size_t ws_bytes, void* stream);
/* Data-parallel form for replicated tables small enough to exchange densely (all-reduce instead of
 * an all-gather of every rank's rows): dense[key] = sum of the rows of key (dense zeroed by the
 * caller; same de-duplication as ot_sparse_adagrad, workspace ot_sparse_adagrad_workspace_size),
 * then clip_by_norm + Keras Adagrad over all rows (zero-gradient rows stay bitwise unchanged, i.e.
 * the same update as the sparse path). */
int ot_sparse_grad_dense(int E, int64_t num_rows, const int64_t* keys, const float* grads, int64_t n,
                         float* dense, void* workspace, size_t ws_bytes, void* stream);
size_t ot_dense_adagrad_workspace_size(void);
int ot_dense_adagrad(float* table, float* accum, const float* grad, int64_t num_rows, int E, float lr,
                     float eps, float clip, void* workspace, size_t ws_bytes, void* stream);
/* Two-phase sparse update for row-sharded tables (the clip norm spans all owners): prepare
 * de-duplicates and writes this rank's squared norm to sumsq_out (device float); the caller
 * all-reduces it; finish applies clip_by_norm(clip) with the global norm + Keras Adagrad.  Same
 * workspace (ot_sparse_adagrad_workspace_size) for both calls. */
int ot_sparse_prepare(int E, int64_t num_rows, const int64_t* keys, const float* grads, int64_t n, float* sumsq_out,
                      void* workspace, size_t ws_bytes, void* stream);
int ot_sparse_finish(float* table, float* accum, int E, int64_t n, float lr, float eps, float clip,
                     const float* sumsq_total, void* workspace, size_t ws_bytes, void* stream);

/* ---- row-sharded embedding tables (shard.hip) ------------------------------
 * Row id lives on rank id % world at local row id / world.  ot_shard_route buckets n ids by owner
 * (stable): perm[j] = position of the j-th routed id, send_local[j] = its local row at the owner
 * (-1 for ids outside [0, num_rows)), counts[r] = ids routed to rank r.  The all-to-all exchanges
 * are the caller's (RCCL); ot_gather_rows / ot_permute_rows move the rows on each side. */
size_t ot_shard_route_workspace_size(int64_t n);
int ot_shard_route(const int64_t* ids, int64_t n, int64_t num_rows, int world, int32_t* perm, int64_t* send_local,
                   int32_t* counts, void* workspace, size_t ws_bytes, void* stream);
/* De-duplicating route (replaces ot_shard_route in ShardedTable.lookup; same owner rule): the n ids
 * sorted by (owner, local row), stable, with equal ids merged into U unique entries in owner order.
 * uniq_local[u] = local row of unique u at its owner (-1: every id outside [0, num_rows) merges into
 * one entry routed to rank 0); counts[r] = unique ids owned by rank r (U = their sum); inv[i] = the
 * unique entry of id i (int64: the idx of ot_gather_rows that expands the U fetched rows to the n
 * tokens); order[j] = position of the j-th id in sorted order and run_start[u] = first j of unique
 * u (run_start[U] = n), the runs of ot_segment_rows_sum.  Arrays sized n (run_start n + 1). */
size_t ot_shard_route_unique_workspace_size(int64_t n);
int ot_shard_route_unique(const int64_t* ids, int64_t n, int64_t num_rows, int world, int64_t* uniq_local,
                          int64_t* inv, int32_t* order, int32_t* run_start, int32_t* counts, void* workspace,
                          size_t ws_bytes, void* stream);
/* out[u] = sum of src[order[j]] for j in [run_start[u], run_start[u+1]), ascending j (deterministic):
 * the per-token gradient rows of a de-duplicated route summed per unique id before they travel */
int ot_segment_rows_sum(const float* src, const int32_t* order, const int32_t* run_start, int64_t U, int E,
                        float* out, void* stream);
/* The same sums, balanced for Zipf-hot ids (runs cut into pieces of <= 64 positions, piece partials added
 * in piece order: deterministic); n = the routed id count (run_start[U]).  ws:
 * ot_segment_rows_sum_workspace_size(U, n, E) bytes. */
size_t ot_segment_rows_sum_workspace_size(int64_t U, int64_t n, int E);
int ot_segment_rows_sum_ex(const float* src, const int32_t* order, const int32_t* run_start, int64_t U, int64_t n,
                           int E, float* out, void* workspace, size_t ws_bytes, void* stream);
/* out[i] = table[idx[i]] (zeros for idx < 0) */
int ot_gather_rows(const float* table, int E, const int64_t* idx, int64_t n, float* out, void* stream);
/* inverse = 0: dst[j] = src[perm[j]]; inverse = 1: dst[perm[j]] = src[j] */
int ot_permute_rows(const float* src, const int32_t* perm, int64_t n, int E, int inverse, float* dst, void* stream);
/* shard init U(lo, hi) from a counter-based hash of (global row, column): the same logical table
 * for every world size */
int ot_hash_uniform_rows(float* out, int64_t local_rows, int E, int rank, int world, uint32_t seed, float lo,
                         float hi, void* stream);

/* ---- dense optimizer (optim.hip) ----------------------------------------------------------
 * Per-variable tf.clip_by_norm (train.py:134-135) over 2-D strided segments of one flat
 * gradient buffer, then Keras-2.12 RMSprop(momentum) (train.py:64-70, 138):
 *   v = rho v + (1-rho) g^2; inc = lr g rsqrt(v + eps); m = mom m + inc; w -= m.
 * segs: [nseg][4] int64 {offset, rows, cols, row_stride}. */
size_t ot_clip_rmsprop_workspace_size(int nseg, int64_t max_seg_elems);
int ot_clip_rmsprop(float* w, float* g, float* v, float* m, const int64_t* segs_dev, int nseg,
                    int64_t max_seg_elems, float lr, float rho, float eps, float momentum, float clip,
                    void* workspace, size_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ONETRANS_HIP_H */
