// Causal attention forward on gfx950 block-scaled fp8 MFMA (v_mfma_scale_f32_32x32x64_f8f6f4, OCP
// e4m3 operands, one e8m0 scale per 32-element k block): BASELINE configs[4] "bf16, CDNA4 fp8 MFMA
// attention" (C5).  Replaces the same reference op as ot_attn_fwd: model.py:100-114 (QK^T/sqrt(hd),
// band_part mask with -1e9, softmax, PV) with the pyramid's tail / selected queries (model.py:356/371).
//
// Two launches:
//  1. attn_fp8_pack_kernel — per (sample, head, 64-key block): K rows quantised to e4m3 with one
//     scale per (key, 32 dims); V quantised with one scale per (dim, 64 keys) and written transposed
//     ([dim][key], keys permuted inside each 64-key block into the order the P operand holds them).
//  2. attn_fwd_fp8_kernel — one wave per (sample, head) as attn_fwd_split_kernel, 32 queries x 64 keys
//     per step:  S^T = K Q^T  (one 32x32x64 MFMA per 32-key tile and 64 dims; Q quantised in registers
//     once per query block with one scale per (query, 32 dims), the accumulator scaled by
//     log2(e)/sqrt(hd) in f32), online softmax in f32,
//     O^T += V^T P^T  (P^T is the two S^T accumulators converted to e4m3 in place: lane half hh, element
//     j = 16t + r <-> key 32t + acc_row(r, hh); the V^T image holds the same keys at byte 32hh + j).
//     P is kept as P * 2^8 (exp2(s - m + 8): [0, 256], inside e4m3's range, small values stay normal)
//     and the row sum l in the same units, so O = sum(P V) / l needs no extra scale.
//
// OT_FP8_DEQUANT (training): both launches also write the dequantised operands back into qkv (each
// Q / K / V element replaced by its dequantised value), so the backward (ot_attn_bwd in the bf16 GEMM
// mode) recomputes S from the operands the fp8 forward used.  One term: the e4m3 value times its block
// scale is exact in bf16, the recomputed P matches the forward's log-sum-exp up to summation order and
// delta = rowsum(dO o O) gives the straight-through gradient of the forward that ran (P's own e4m3
// rounding aside).  Two terms (the default): hi + lo needs more than bf16's 8 significant bits, so the
// bf16 backward (and ot_attn_fwd_fp8_deq16's copy) round it, and the forward summed hi.hi + hi.lo + lo.hi
// without lo.lo — the recomputed S is off by those terms and the gradient is approximate (0.5-1% of
// max|g| from the exact attention gradient, tests/test_attn_fp8_gpu.py).  Without OT_FP8_DEQUANT the
// backward would recompute S from unquantised operands against the fp8 forward's statistics.
//
// Operand layout of the 32x32x64 scaled MFMA, measured on the box (tools/micro/fp8_probe.hip): A lane l
// holds row l&31, B lane l column l&31; byte j of lane half h meets byte j of the other operand's lane
// half h (so any k assignment that agrees between A and B is a valid product); the e8m0 scale operand
// of lane half h covers k-block h = bytes [16h, 16h+16) of BOTH half-lanes of its row / column.  So a
// row's 64 k-elements sit as: half 0 = dims 0-15 | 32-47, half 1 = dims 16-31 | 48-63, and lane half h
// supplies the scale of dims 32h .. 32h+31.
#include "common.h"

namespace ot {

typedef int i32x8 __attribute__((ext_vector_type(8)));

namespace fp8 {

__device__ __forceinline__ int acc_row(int r, int hh) { return (r & 3) + 8 * (r >> 2) + 4 * hh; }

// scale exponent for a block with max |x| = amax: x * 2^-e lands in [-256, 256) (e4m3 max 448);
// e8m0 byte = e + 127.  amax = 0 -> the smallest scale (the block is zeros anyway).
__device__ __forceinline__ int block_exp(float amax) {
  const int E = (int)((__float_as_uint(amax) >> 23) & 0xff) - 127;   // amax in [2^E, 2^(E+1))
  int e = E - 7;
  e = e < -120 ? -120 : (e > 120 ? 120 : e);
  return e;
}
__device__ __forceinline__ float pow2f(int e) { return __uint_as_float((uint32_t)(127 + e) << 23); }

// 4 floats -> 4 e4m3 bytes (element 0 in the low byte)
__device__ __forceinline__ uint32_t pack4(float a, float b, float c, float d) {
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
  return (uint32_t)v;
}

__device__ __forceinline__ f32x16 mfma_fp8(const i32x8& a, const i32x8& b, f32x16 c, int sa, int sb) {
  return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, sa, 0, sb);
}

// e4m3 bytes of v (element 0 in the low byte) back to f32, times the block scale 2^e
__device__ __forceinline__ f32x4 unpack4(int v, float sc) {
  typedef float v2f __attribute__((ext_vector_type(2)));
  const v2f lo = __builtin_amdgcn_cvt_pk_f32_fp8(v, false), hi = __builtin_amdgcn_cvt_pk_f32_fp8(v, true);
  return f32x4{lo.x * sc, lo.y * sc, hi.x * sc, hi.y * sc};
}

// 16 bytes at p (operand bytes 0-15) and 16 at p + gap (bytes 16-31)
__device__ __forceinline__ i32x8 load32(const uint8_t* p, int gap = 16) {
  const i32x4 lo = *reinterpret_cast<const i32x4*>(p);
  const i32x4 hi = *reinterpret_cast<const i32x4*>(p + gap);
  return i32x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
}

}  // namespace fp8

// Workspace of one call (all u8), Ip = I rounded up to 64 keys, for each term t (hi; lo with T8 = 2):
//   k8 [BH][Ip][HD]   ks [BH][Ip][HD/32]   vt8 [BH][HD][Ip]   vs [BH][Ip/64][HD]
struct Fp8Pack {
  uint8_t *k8, *ks, *vt8, *vs;          // hi term
  uint8_t *k8l, *ksl, *vt8l, *vsl;      // lo term (two-term operands)
};

__host__ __device__ inline int64_t fp8_ipad(int I) { return ((int64_t)I + 63) / 64 * 64; }

inline size_t fp8_term_bytes(int64_t BH, int I, int HD) {
  const int64_t Ip = fp8_ipad(I);
  return (size_t)(BH * Ip * HD * 2 + BH * Ip * (HD / 32) + BH * (Ip / 64) * HD);
}

inline Fp8Pack fp8_pack_layout(void* ws, int64_t BH, int I, int HD) {
  const int64_t Ip = fp8_ipad(I);
  uint8_t* p = static_cast<uint8_t*>(ws);
  Fp8Pack f;
  uint8_t* q = p + fp8_term_bytes(BH, I, HD);
  f.k8 = p;  p += BH * Ip * HD;
  f.vt8 = p; p += BH * Ip * HD;
  f.ks = p;  p += BH * Ip * (HD / 32);
  f.vs = p;
  f.k8l = q;  q += BH * Ip * HD;
  f.vt8l = q; q += BH * Ip * HD;
  f.ksl = q;  q += BH * Ip * (HD / 32);
  f.vsl = q;
  return f;
}

// both terms' space (the one-term form uses the first half)
inline size_t fp8_pack_bytes(int64_t BH, int I, int HD) { return 2 * fp8_term_bytes(BH, I, HD); }

// 16 floats -> 16 e4m3 bytes at scale 2^-e, and their dequantised values into r (r = x - q(x) 2^e when
// resid: the lo term's input)
__device__ __forceinline__ i32x4 quant16(const float (&x)[16], int e, float (&r)[16], bool resid) {
  const float inv = fp8::pow2f(-e), sc = fp8::pow2f(e);
  i32x4 o;
  int* ow = reinterpret_cast<int*>(&o);
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    ow[w] = (int)fp8::pack4(x[4 * w] * inv, x[4 * w + 1] * inv, x[4 * w + 2] * inv, x[4 * w + 3] * inv);
    const f32x4 d = fp8::unpack4(ow[w], sc);
    r[4 * w] = resid ? x[4 * w] - d.x : d.x;
    r[4 * w + 1] = resid ? x[4 * w + 1] - d.y : d.y;
    r[4 * w + 2] = resid ? x[4 * w + 2] - d.z : d.z;
    r[4 * w + 3] = resid ? x[4 * w + 3] - d.w : d.w;
  }
  return o;
}

// grid (B*H, Ip/64), 256 threads (B*H on x: up to 2^31 - 1 heads).  Keys >= I are zeros (the causal mask removes them).
// T8 = 2: every element also gets a lo term, lo = e4m3(x - hi) with its own block scale (same blocks).
template <int HD, int T8>
__global__ __launch_bounds__(256) void attn_fp8_pack_kernel(float* qkv, int64_t ld, int H, int I, Fp8Pack f,
                                                            int dequant, uint16_t* deq16) {
  constexpr int VLD = HD + 1;
  __shared__ float vs_f[64 * VLD];
  __shared__ __attribute__((aligned(16))) uint8_t vt_img[T8][HD * 64];
  const int kb = blockIdx.y, bh = blockIdx.x;
  const int b = bh / H, h = bh % H, d = H * HD;
  const int64_t Ip = fp8_ipad(I);
  const int t = threadIdx.x;
  float* base = qkv + (int64_t)b * I * ld + h * HD;

  // ---- K: thread = (key, 16 dims); a 32-dim scale block = 2 adjacent lanes
  constexpr int TPK = HD / 16, KPP = 256 / TPK;
#pragma unroll
  for (int pass = 0; pass < 64 / KPP; ++pass) {
    const int kk = pass * KPP + t / TPK, part = t % TPK;
    const int key = 64 * kb + kk;
    float x[16], r[16];
    if (key < I) {
      const float* src = base + (int64_t)key * ld + d + 16 * part;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(src + 4 * q);
        x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) x[j] = 0.f;
    }
    float am = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) am = fmaxf(am, fabsf(x[j]));
    am = fmaxf(am, __shfl_xor(am, 1, 64));
    const int e = fp8::block_exp(am);
    const i32x4 o = quant16(x, e, r, T8 == 2);
    const int64_t row = (int64_t)bh * Ip + key;
    *reinterpret_cast<i32x4*>(f.k8 + row * HD + 16 * part) = o;
    if ((part & 1) == 0) f.ks[row * (HD / 32) + part / 2] = (uint8_t)(e + 127);
    if constexpr (T8 == 2) {
      float aml = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) aml = fmaxf(aml, fabsf(r[j]));
      aml = fmaxf(aml, __shfl_xor(aml, 1, 64));
      const int el = fp8::block_exp(aml);
      float rl[16];
      const i32x4 ol = quant16(r, el, rl, false);
      *reinterpret_cast<i32x4*>(f.k8l + row * HD + 16 * part) = ol;
      if ((part & 1) == 0) f.ksl[row * (HD / 32) + part / 2] = (uint8_t)(el + 127);
#pragma unroll
      for (int j = 0; j < 16; ++j) r[j] = x[j] - r[j] + rl[j];      // hi + lo (dequantised)
    }
    if (dequant && key < I) {
      if (deq16) {                                   // bf16 copy (the backward rounds to bf16 anyway)
        uint16_t* dst = deq16 + ((int64_t)b * I + key) * ld + h * HD + d + 16 * part;
#pragma unroll
        for (int q = 0; q < 4; q += 2) {
          const u32x2 lo = bf16_rne4(f32x4{r[4 * q], r[4 * q + 1], r[4 * q + 2], r[4 * q + 3]});
          const u32x2 hi = bf16_rne4(f32x4{r[4 * q + 4], r[4 * q + 5], r[4 * q + 6], r[4 * q + 7]});
          *reinterpret_cast<u32x4*>(dst + 4 * q) = u32x4{lo.x, lo.y, hi.x, hi.y};
        }
      } else {
        f32x4* dst = reinterpret_cast<f32x4*>(base + (int64_t)key * ld + d + 16 * part);
#pragma unroll
        for (int q = 0; q < 4; ++q) dst[q] = f32x4{r[4 * q], r[4 * q + 1], r[4 * q + 2], r[4 * q + 3]};
      }
    }
  }

  // ---- V: stage the [64 keys][HD] tile, then thread = (dim, KPT keys)
  for (int i = t; i < 64 * HD / 4; i += 256) {
    const int kk = i / (HD / 4), c4 = i % (HD / 4);
    const int key = 64 * kb + kk;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (key < I) v = *reinterpret_cast<const f32x4*>(base + (int64_t)key * ld + 2 * d + 4 * c4);
    float* dst = vs_f + kk * VLD + 4 * c4;
    dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;
  }
  __syncthreads();
  constexpr int G = 256 / HD, KPT = 64 / G;       // threads per dim, keys per thread
  {
    const int c = t / G, g = t % G;
    float am = 0.f;
#pragma unroll
    for (int i = 0; i < KPT; ++i) am = fmaxf(am, fabsf(vs_f[(g * KPT + i) * VLD + c]));
#pragma unroll
    for (int o = 1; o < G; o <<= 1) am = fmaxf(am, __shfl_xor(am, o, 64));
    const int e = fp8::block_exp(am);
    const float inv = fp8::pow2f(-e), sc = fp8::pow2f(e);
    float deq[KPT];                                  // this thread's keys' dequantised hi values
    auto put = [&](int term, int k0, int v2) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int k = k0 + u, kk = k & 31;
        // key k of the block sits at byte 32 hh + 16 t + (kk & 3) + 4 (kk >> 3) of the P order
        const int pos = 32 * ((kk >> 2) & 1) + 16 * (k >> 5) + (kk & 3) + 4 * (kk >> 3);
        vt_img[term][c * 64 + pos] = (uint8_t)((v2 >> (8 * u)) & 0xff);
      }
    };
#pragma unroll
    for (int i = 0; i < KPT; i += 2) {
      const int k0 = g * KPT + i;
      const int v2 = __builtin_amdgcn_cvt_pk_fp8_f32(vs_f[k0 * VLD + c] * inv, vs_f[(k0 + 1) * VLD + c] * inv, 0, false);
      const f32x4 dv = fp8::unpack4(v2, sc);
      deq[i] = dv.x;
      deq[i + 1] = dv.y;
      put(0, k0, v2);
    }
    if (g == 0) f.vs[((int64_t)bh * (Ip / 64) + kb) * HD + c] = (uint8_t)(e + 127);
    if constexpr (T8 == 2) {
      float aml = 0.f;
#pragma unroll
      for (int i = 0; i < KPT; ++i) aml = fmaxf(aml, fabsf(vs_f[(g * KPT + i) * VLD + c] - deq[i]));
#pragma unroll
      for (int o = 1; o < G; o <<= 1) aml = fmaxf(aml, __shfl_xor(aml, o, 64));
      const int el = fp8::block_exp(aml);
      const float invl = fp8::pow2f(-el), scl = fp8::pow2f(el);
#pragma unroll
      for (int i = 0; i < KPT; i += 2) {
        const int k0 = g * KPT + i;
        const float r0 = vs_f[k0 * VLD + c] - deq[i], r1 = vs_f[(k0 + 1) * VLD + c] - deq[i + 1];
        const int v2 = __builtin_amdgcn_cvt_pk_fp8_f32(r0 * invl, r1 * invl, 0, false);
        const f32x4 dv = fp8::unpack4(v2, scl);
        deq[i] += dv.x;
        deq[i + 1] += dv.y;
        put(1, k0, v2);
      }
      if (g == 0) f.vsl[((int64_t)bh * (Ip / 64) + kb) * HD + c] = (uint8_t)(el + 127);
    }
    if (dequant) {            // this thread owns (dim c, its keys) of the staged tile
#pragma unroll
      for (int i = 0; i < KPT; ++i) vs_f[(g * KPT + i) * VLD + c] = deq[i];
    }
  }
  __syncthreads();
  for (int i = t; i < HD * 4; i += 256) {
    const int c = i / 4, q = i % 4;
    *reinterpret_cast<i32x4*>(f.vt8 + ((int64_t)bh * HD + c) * Ip + 64 * kb + 16 * q) =
        *reinterpret_cast<const i32x4*>(vt_img[0] + c * 64 + 16 * q);
    if constexpr (T8 == 2)
      *reinterpret_cast<i32x4*>(f.vt8l + ((int64_t)bh * HD + c) * Ip + 64 * kb + 16 * q) =
          *reinterpret_cast<const i32x4*>(vt_img[T8 - 1] + c * 64 + 16 * q);
  }
  if (dequant) {
    for (int i = t; i < 64 * HD / 4; i += 256) {
      const int kk = i / (HD / 4), c4 = i % (HD / 4);
      const int key = 64 * kb + kk;
      const float* src = vs_f + kk * VLD + 4 * c4;
      if (key < I) {
        if (deq16)
          *reinterpret_cast<u32x2*>(deq16 + ((int64_t)b * I + key) * ld + h * HD + 2 * d + 4 * c4) =
              bf16_rne4(f32x4{src[0], src[1], src[2], src[3]});
        else
          *reinterpret_cast<f32x4*>(base + (int64_t)key * ld + 2 * d + 4 * c4) = f32x4{src[0], src[1], src[2], src[3]};
      }
    }
  }
}

struct Fp8AttnArgs {
  float* qkv; int64_t ld; int d;
  float* out; float* lse;
  int B, H, I, K;
  float scale;
  const int32_t* qpos;
  Fp8Pack f;
  int dequant;
  uint16_t* deq16;           // dequantised operands in bf16 here (ld as qkv) instead of in place, or null
};

// one wave per (b, h), 4 waves per block.  T8 = 2: two-term operands, S^T = Kh Qh + Kh Ql + Kl Qh and
// O^T += Vh Ph + Vh Pl + Vl Ph (the lo x lo products dropped: below the e4m3 pair's own rounding); P's lo
// term is e4m3((P 2^8 - Ph) 2^4) at MFMA scale 2^-4.
// PW > 1: one workgroup of PW waves per (b, h), wave w taking query blocks w, w + PW, ...: the waves sweep the
// pair's key blocks at about the same time, so its K / V packs are read from L2 by PW waves instead of
// from the Infinity Cache by one (PW = 1, one pair per wave, 4 per block: 21 GB of L3 fetch per C5 layer,
// the kernel bound at ~7 TB/s).
template <int HD, int T8, int PW>
__global__ __launch_bounds__(PW > 1 ? 64 * PW : 256) void attn_fwd_fp8_kernel(Fp8AttnArgs p) {
  static_assert(HD == 64 || HD == 128, "fp8 attention: head_dim 64 or 128");
  constexpr int NKS = HD / 64;                   // 64-dim k steps of S^T
  constexpr int NC = HD / 32;                    // 32-dim output chunks
  const int lane = threadIdx.x & 63, li = lane & 31, hh = lane >> 5;
  const int pair = PW > 1 ? (int)blockIdx.x : (int)(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (pair >= p.B * p.H) return;
  const int qb0 = PW > 1 ? (int)(threadIdx.x >> 6) : 0;
  const int b = pair / p.H, h = pair % p.H;
  const int I = p.I, K = p.K, q_off = I - K;
  const int64_t Ip = fp8_ipad(I);
  float* Q = p.qkv + (int64_t)b * I * p.ld + h * HD;
  const int64_t kofs = (int64_t)pair * Ip * HD + 16 * hh, ksofs = (int64_t)pair * Ip * (HD / 32) + hh;
  const int64_t vofs = (int64_t)pair * HD * Ip + 32 * hh, vsofs = (int64_t)pair * (Ip / 64) * HD;
  const uint8_t* k8[2] = {p.f.k8 + kofs, p.f.k8l + kofs};
  const uint8_t* ksc[2] = {p.f.ks + ksofs, p.f.ksl + ksofs};
  const uint8_t* vt8[2] = {p.f.vt8 + vofs, p.f.vt8l + vofs};
  const uint8_t* vsc[2] = {p.f.vs + vsofs, p.f.vsl + vsofs};
  const int32_t* qp = p.qpos ? p.qpos + (int64_t)b * K : nullptr;
  const int nqb = (K + 31) / 32;
  const float qscale = p.scale * 1.4426950408889634f;   // log2(e) / sqrt(hd)

  for (int qb = qb0; qb < nqb; qb += (PW > 1 ? PW : 1)) {
    const int j = 32 * qb + li;
    const int jc = j < K ? j : K - 1;
    const int qpos = qp ? qp[jc] : q_off + jc;
    // Q fragment of k-step ks: bytes 0-15 = dims 64 ks + 16 hh .. +15 (k-block 0), bytes 16-31 =
    // dims 64 ks + 32 + 16 hh .. +15 (k-block 1); each block's amax is completed across the two
    // half-lanes, and lane half hh supplies block hh's scale
    i32x8 qa[T8][NKS];
    int qs[T8][NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      float* src = Q + (int64_t)qpos * p.ld + 64 * ks + 16 * hh;
      float x[2][16];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(src + 4 * (q & 3) + 32 * (q >> 2));
        float* xx = x[q >> 2] + 4 * (q & 3);
        xx[0] = v.x; xx[1] = v.y; xx[2] = v.z; xx[3] = v.w;
      }
#pragma unroll
      for (int term = 0; term < T8; ++term) {
        float am[2] = {0.f, 0.f};
#pragma unroll
        for (int blk = 0; blk < 2; ++blk) {
#pragma unroll
          for (int s = 0; s < 16; ++s) am[blk] = fmaxf(am[blk], fabsf(x[blk][s]));
          am[blk] = fmaxf(am[blk], __shfl_xor(am[blk], 32, 64));
        }
        const int e0 = fp8::block_exp(am[0]), e1 = fp8::block_exp(am[1]);
        float r[2][16];
        const i32x4 o0 = quant16(x[0], e0, r[0], true), o1 = quant16(x[1], e1, r[1], true);
        qa[term][ks] = i32x8{o0.x, o0.y, o0.z, o0.w, o1.x, o1.y, o1.z, o1.w};
        qs[term][ks] = (hh ? e1 : e0) + 127;
#pragma unroll
        for (int blk = 0; blk < 2; ++blk)
#pragma unroll
          for (int s = 0; s < 16; ++s) x[blk][s] = r[blk][s];            // the residual: next term's input
      }
      if (p.dequant && j < K) {          // this lane's 32 elements of query row qpos, dequantised in place
        float dq[2][16];
#pragma unroll
        for (int blk = 0; blk < 2; ++blk)
#pragma unroll
          for (int s = 0; s < 16; ++s) dq[blk][s] = 0.f;
#pragma unroll
        for (int term = 0; term < T8; ++term) {
          // lane half hh holds block hh's scale; the other block's is the partner's
          const int eo = __shfl_xor(qs[term][ks], 32, 64);
          const float s0 = fp8::pow2f((hh ? eo : qs[term][ks]) - 127), s1 = fp8::pow2f((hh ? qs[term][ks] : eo) - 127);
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            const f32x4 a = fp8::unpack4(qa[term][ks][w], s0), c = fp8::unpack4(qa[term][ks][4 + w], s1);
            dq[0][4 * w] += a.x; dq[0][4 * w + 1] += a.y; dq[0][4 * w + 2] += a.z; dq[0][4 * w + 3] += a.w;
            dq[1][4 * w] += c.x; dq[1][4 * w + 1] += c.y; dq[1][4 * w + 2] += c.z; dq[1][4 * w + 3] += c.w;
          }
        }
        if (p.deq16) {
          uint16_t* d16 = p.deq16 + ((int64_t)b * I + qpos) * p.ld + h * HD + 64 * ks + 16 * hh;
#pragma unroll
          for (int blk = 0; blk < 2; ++blk)
#pragma unroll
            for (int w = 0; w < 4; w += 2) {
              const u32x2 lo = bf16_rne4(f32x4{dq[blk][4 * w], dq[blk][4 * w + 1], dq[blk][4 * w + 2], dq[blk][4 * w + 3]});
              const u32x2 hi = bf16_rne4(f32x4{dq[blk][4 * w + 4], dq[blk][4 * w + 5], dq[blk][4 * w + 6], dq[blk][4 * w + 7]});
              *reinterpret_cast<u32x4*>(d16 + 32 * blk + 4 * w) = u32x4{lo.x, lo.y, hi.x, hi.y};
            }
        } else {
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            *reinterpret_cast<f32x4*>(src + 4 * w) = f32x4{dq[0][4 * w], dq[0][4 * w + 1], dq[0][4 * w + 2], dq[0][4 * w + 3]};
            *reinterpret_cast<f32x4*>(src + 32 + 4 * w) =
                f32x4{dq[1][4 * w], dq[1][4 * w + 1], dq[1][4 * w + 2], dq[1][4 * w + 3]};
          }
        }
      }
    }
    f32x16 oacc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) oacc[c][r] = 0.f;
    float m = -INFINITY, l = 0.f;
    const int last_q = qp ? qp[min(32 * qb + 31, K - 1)] : q_off + min(32 * qb + 31, K - 1);
    const int nkb = last_q / 64 + 1;
    const int first_masked = (qp ? qp[32 * qb] : q_off + 32 * qb) / 64;

    // fragments of key block kb: K tiles t (keys 64 kb + 32 t + li), V^T chunks c (dims 32 c + li)
    i32x8 kf[T8][2][NKS], vf[T8][NC];
    int kscale[T8][2][NKS], vscale[T8][NC];
    auto load_kv = [&](int kb, i32x8 (&kf_)[T8][2][NKS], i32x8 (&vf_)[T8][NC], int (&ksc_)[T8][2][NKS],
                       int (&vsc_)[T8][NC]) {
#pragma unroll
      for (int term = 0; term < T8; ++term) {
#pragma unroll
        for (int t2 = 0; t2 < 2; ++t2) {
          const int64_t key = 64 * kb + 32 * t2 + li;
#pragma unroll
          for (int ks = 0; ks < NKS; ++ks) {
            kf_[term][t2][ks] = fp8::load32(k8[term] + key * HD + 64 * ks, 32);      // dims 16hh.. | 32+16hh..
            ksc_[term][t2][ks] = ksc[term][key * (HD / 32) + 2 * ks];
          }
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          vf_[term][c] = fp8::load32(vt8[term] + (int64_t)(32 * c + li) * Ip + 64 * kb);
          vsc_[term][c] = vsc[term][(int64_t)kb * HD + 32 * c + li];
        }
      }
    };
    load_kv(0, kf, vf, kscale, vscale);
    for (int kb = 0; kb < nkb; ++kb) {
      i32x8 kn[T8][2][NKS], vn[T8][NC];
      int kscn[T8][2][NKS], vscn[T8][NC];
      load_kv(min(kb + 1, nkb - 1), kn, vn, kscn, vscn);   // unconditional: the wait before this block's
                                                              // MFMAs can leave the prefetch in flight
      f32x16 s[2];
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2) {
#pragma unroll
        for (int r = 0; r < 16; ++r) s[t2][r] = 0.f;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          s[t2] = fp8::mfma_fp8(kf[0][t2][ks], qa[0][ks], s[t2], kscale[0][t2][ks], qs[0][ks]);
          if constexpr (T8 == 2) {
            s[t2] = fp8::mfma_fp8(kf[0][t2][ks], qa[1][ks], s[t2], kscale[0][t2][ks], qs[1][ks]);
            s[t2] = fp8::mfma_fp8(kf[1][t2][ks], qa[0][ks], s[t2], kscale[1][t2][ks], qs[0][ks]);
          }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) s[t2][r] *= qscale;          // log2 domain
      }
      if (kb >= first_masked) {
#pragma unroll
        for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            s[t2][r] = (64 * kb + 32 * t2 + fp8::acc_row(r, hh) <= qpos) ? s[t2][r] : -INFINITY;
      }
      float mloc = s[0][0];
#pragma unroll
      for (int r = 1; r < 16; ++r) mloc = fmaxf(mloc, s[0][r]);
#pragma unroll
      for (int r = 0; r < 16; ++r) mloc = fmaxf(mloc, s[1][r]);
      mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
      const float mnew = fmaxf(m, mloc);
      const float corr = __builtin_amdgcn_exp2f(m - mnew);
      const float moff = mnew - 8.f;                  // P * 2^8
      float lsum = 0.f;
#pragma unroll
      for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = __builtin_amdgcn_exp2f(s[t2][r] - moff);
          s[t2][r] = e;
          lsum += e;
        }
      lsum += __shfl_xor(lsum, 32, 64);
      l = l * corr + lsum;
      m = mnew;
      i32x8 pb[T8];
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        const int t2 = w >> 2, r = 4 * (w & 3);
        pb[0][w] = (int)fp8::pack4(s[t2][r], s[t2][r + 1], s[t2][r + 2], s[t2][r + 3]);
        if constexpr (T8 == 2) {
          const f32x4 q = fp8::unpack4(pb[0][w], 1.f);
          pb[T8 - 1][w] = (int)fp8::pack4((s[t2][r] - q.x) * 16.f, (s[t2][r + 1] - q.y) * 16.f,
                                          (s[t2][r + 2] - q.z) * 16.f, (s[t2][r + 3] - q.w) * 16.f);
        }
      }
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        oacc[c] *= corr;
        oacc[c] = fp8::mfma_fp8(vf[0][c], pb[0], oacc[c], vscale[0][c], 127);   // O^T += V^T P^T
        if constexpr (T8 == 2) {
          oacc[c] = fp8::mfma_fp8(vf[0][c], pb[T8 - 1], oacc[c], vscale[0][c], 127 - 4);
          oacc[c] = fp8::mfma_fp8(vf[T8 - 1][c], pb[0], oacc[c], vscale[T8 - 1][c], 127);
        }
      }
#pragma unroll
      for (int term = 0; term < T8; ++term) {
#pragma unroll
        for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
          for (int ks = 0; ks < NKS; ++ks) { kf[term][t2][ks] = kn[term][t2][ks]; kscale[term][t2][ks] = kscn[term][t2][ks]; }
#pragma unroll
        for (int c = 0; c < NC; ++c) { vf[term][c] = vn[term][c]; vscale[term][c] = vscn[term][c]; }
      }
    }
    if (j < K) {
      const float inv = 1.f / l;
      float* orow = p.out + ((int64_t)b * K + j) * p.d + h * HD;
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int dd = 32 * c + 8 * g + 4 * hh;
          f32x4 v = {oacc[c][4 * g] * inv, oacc[c][4 * g + 1] * inv, oacc[c][4 * g + 2] * inv,
                     oacc[c][4 * g + 3] * inv};
          *reinterpret_cast<f32x4*>(orow + dd) = v;
        }
      // l is in units of 2^8 (P * 2^8): lse = ln(sum exp(s)) = (m - 8) ln 2 + ln(l)
      if (hh == 0) p.lse[((int64_t)b * p.H + h) * K + j] = (m - 8.f) * 0.6931471805599453f + __logf(l);
    }
  }
}

}  // namespace ot

using namespace ot;

extern "C" size_t ot_attn_fwd_fp8_workspace_size(int B, int H, int I, int head_dim) {
  if (B <= 0 || H <= 0 || I <= 0 || (head_dim != 64 && head_dim != 128)) return 0;
  return fp8_pack_bytes((int64_t)B * H, I, head_dim);
}

static int attn_fwd_fp8_impl(float* qkv, int64_t ld, int B, int H, int I, int K, const int32_t* qpos, int head_dim,
                             float* out, float* lse, void* workspace, size_t ws_bytes, int flags, uint16_t* deq16,
                             void* stream);

extern "C" int ot_attn_fwd_fp8_ex(float* qkv, int64_t ld, int B, int H, int I, int K, const int32_t* qpos,
                                  int head_dim, float* out, float* lse, void* workspace, size_t ws_bytes, int flags,
                                  void* stream) {
  return attn_fwd_fp8_impl(qkv, ld, B, H, I, K, qpos, head_dim, out, lse, workspace, ws_bytes, flags, nullptr, stream);
}

extern "C" int ot_attn_fwd_fp8_deq16(const float* qkv, int64_t ld, int B, int H, int I, int K, const int32_t* qpos,
                                     int head_dim, float* out, float* lse, void* workspace, size_t ws_bytes,
                                     int flags, uint16_t* deq16, void* stream) {
  OT_REQUIRE(deq16 && ((uintptr_t)deq16 % 16) == 0 && ld % 8 == 0,
             "ot_attn_fwd_fp8_deq16: deq16 needs 16-B alignment and ld %% 8 == 0");
  return attn_fwd_fp8_impl(const_cast<float*>(qkv), ld, B, H, I, K, qpos, head_dim, out, lse, workspace, ws_bytes,
                           flags | OT_FP8_DEQUANT, deq16, stream);
}

static int attn_fwd_fp8_impl(float* qkv, int64_t ld, int B, int H, int I, int K, const int32_t* qpos, int head_dim,
                             float* out, float* lse, void* workspace, size_t ws_bytes, int flags, uint16_t* deq16,
                             void* stream) {
  OT_REQUIRE(qkv && out && lse, "ot_attn_fwd_fp8: null operand");
  OT_REQUIRE((flags & ~(OT_FP8_DEQUANT | OT_FP8_TWO_TERM)) == 0, "ot_attn_fwd_fp8: unknown flags 0x%x", flags);
  const int dq = (flags & OT_FP8_DEQUANT) ? 1 : 0;
  const bool two = (flags & OT_FP8_TWO_TERM) != 0;
  OT_REQUIRE(B >= 0 && H > 0 && I > 0 && K > 0 && K <= I, "ot_attn_fwd_fp8: bad sizes B=%d H=%d I=%d K=%d", B, H, I, K);
  OT_REQUIRE(head_dim == 64 || head_dim == 128, "ot_attn_fwd_fp8: head_dim %d (64 or 128)", head_dim);
  OT_REQUIRE(ld % 4 == 0 && ld >= 3 * H * head_dim, "ot_attn_fwd_fp8: ld must be >= 3d and a multiple of 4");
  if (B == 0) return OT_OK;
  OT_REQUIRE(workspace && ws_bytes >= ot_attn_fwd_fp8_workspace_size(B, H, I, head_dim) &&
             ((uintptr_t)workspace % 16) == 0, "ot_attn_fwd_fp8: workspace");
  const int64_t BH = (int64_t)B * H;
  const Fp8Pack f = fp8_pack_layout(workspace, BH, I, head_dim);
  OT_REQUIRE(BH < 2147483647LL && fp8_ipad(I) / 64 <= 65535, "ot_attn_fwd_fp8: B*H = %lld, I = %d out of range",
             (long long)BH, I);
  const dim3 pg((unsigned)BH, (unsigned)(fp8_ipad(I) / 64));
  hipStream_t s = (hipStream_t)stream;
  auto pk = head_dim == 64 ? (two ? attn_fp8_pack_kernel<64, 2> : attn_fp8_pack_kernel<64, 1>)
                           : (two ? attn_fp8_pack_kernel<128, 2> : attn_fp8_pack_kernel<128, 1>);
  hipLaunchKernelGGL(pk, pg, dim3(256), 0, s, qkv, ld, H, I, f, dq, deq16);
  OT_LAUNCH_CHECK("ot_attn_fwd_fp8(pack)");
  Fp8AttnArgs p{qkv, ld, H * head_dim, out, lse, B, H, I, K, 1.f / sqrtf((float)head_dim), qpos, f, dq, deq16};
  // one workgroup of 8 waves per (b, h) (measured faster than one pair per wave or 4 waves: DESIGN.md §5)
  auto fk = head_dim == 64 ? (two ? attn_fwd_fp8_kernel<64, 2, 8> : attn_fwd_fp8_kernel<64, 1, 8>)
                           : (two ? attn_fwd_fp8_kernel<128, 2, 8> : attn_fwd_fp8_kernel<128, 1, 8>);
  hipLaunchKernelGGL(fk, dim3((unsigned)BH), dim3(64 * 8), 0, s, p);
  OT_LAUNCH_CHECK("ot_attn_fwd_fp8");
  return OT_OK;
}

extern "C" int ot_attn_fwd_fp8(const float* qkv, int64_t ld, int B, int H, int I, int K, const int32_t* qpos,
                               int head_dim, float* out, float* lse, void* workspace, size_t ws_bytes, void* stream) {
  // flags 0: qkv is only read
  return ot_attn_fwd_fp8_ex(const_cast<float*>(qkv), ld, B, H, I, K, qpos, head_dim, out, lse, workspace, ws_bytes,
                            0, stream);
}
