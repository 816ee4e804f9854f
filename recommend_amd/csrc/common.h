// Shared helpers for the OneTrans gfx950 kernels (C-ABI in include/onetrans_hip.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "../../include/onetrans_hip.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

namespace ot {

// ---- split-bf16 arithmetic (OT_MATMUL_SPLIT_BF16) ------------------------------------
// f32x4 -> three planes of 4 bf16 (each packed into 2 dwords, element 0 in the low half):
// x = x0 + x1 + x2 exactly (x0 the top 8 significant bits, x1 the next 8, x2 the rest; truncation
// keeps every step exact)
// The subtractions run on packed-f32 adds (v_pk_add_f32, two elements each) and the planes are the high halves
// of x, r1, r2 (v_perm): the masked values are needed only as the subtrahends.
__device__ __forceinline__ void split3(f32x4 v, u32x2& p0, u32x2& p1, u32x2& p2) {
  typedef float f32x2_ __attribute__((ext_vector_type(2)));
  uint32_t a[4], b[4], c[4];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const f32x2_ x = {v[2 * k], v[2 * k + 1]};
    const f32x2_ x0 = {__uint_as_float(__float_as_uint(x.x) & 0xffff0000u), __uint_as_float(__float_as_uint(x.y) & 0xffff0000u)};
    const f32x2_ r1 = x - x0;
    const f32x2_ x1 = {__uint_as_float(__float_as_uint(r1.x) & 0xffff0000u), __uint_as_float(__float_as_uint(r1.y) & 0xffff0000u)};
    const f32x2_ r2 = r1 - x1;
    a[2 * k] = __float_as_uint(x.x); a[2 * k + 1] = __float_as_uint(x.y);
    b[2 * k] = __float_as_uint(r1.x); b[2 * k + 1] = __float_as_uint(r1.y);
    c[2 * k] = __float_as_uint(r2.x); c[2 * k + 1] = __float_as_uint(r2.y);
  }
  p0 = u32x2{__builtin_amdgcn_perm(a[1], a[0], 0x07060302u), __builtin_amdgcn_perm(a[3], a[2], 0x07060302u)};
  p1 = u32x2{__builtin_amdgcn_perm(b[1], b[0], 0x07060302u), __builtin_amdgcn_perm(b[3], b[2], 0x07060302u)};
  p2 = u32x2{__builtin_amdgcn_perm(c[1], c[0], 0x07060302u), __builtin_amdgcn_perm(c[3], c[2], 0x07060302u)};
}
// 8 floats -> three planes of one 32x32x16 operand fragment (8 bf16 = 4 dwords each)
__device__ __forceinline__ void split8(const float* v, u32x4 (&pl)[3]) {
  u32x2 a0, a1, a2, b0, b1, b2;
  split3(f32x4{v[0], v[1], v[2], v[3]}, a0, a1, a2);
  split3(f32x4{v[4], v[5], v[6], v[7]}, b0, b1, b2);
  pl[0] = u32x4{a0.x, a0.y, b0.x, b0.y};
  pl[1] = u32x4{a1.x, a1.y, b1.x, b1.y};
  pl[2] = u32x4{a2.x, a2.y, b2.x, b2.y};
}
// f32x4 -> 4 bf16 rounded to nearest even (OT_MATMUL_BF16: the one-plane form), packed like split3
// (v_cvt_pk_bf16_f32: one instruction per pair, round to nearest even — the integer form u + 0x7fff + lsb took
// about four per element and is the same for every finite value)
typedef __bf16 bf16x2_cvt_t __attribute__((ext_vector_type(2)));
typedef float f32x2_cvt_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u32x2 bf16_rne4(f32x4 v) {
  const bf16x2_cvt_t a = __builtin_convertvector(f32x2_cvt_t{v[0], v[1]}, bf16x2_cvt_t);
  const bf16x2_cvt_t b = __builtin_convertvector(f32x2_cvt_t{v[2], v[3]}, bf16x2_cvt_t);
  return u32x2{__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b)};
}
// TERMS = 6: split8; TERMS = 1: plane 0 = the rounded bf16 (planes 1, 2 unused)
template <int TERMS>
__device__ __forceinline__ void split8t(const float* v, u32x4 (&pl)[3]) {
  if constexpr (TERMS == 1) {
    const u32x2 a = bf16_rne4(f32x4{v[0], v[1], v[2], v[3]}), b = bf16_rne4(f32x4{v[4], v[5], v[6], v[7]});
    pl[0] = u32x4{a.x, a.y, b.x, b.y};
  } else {
    split8(v, pl);
  }
}
// XCD-aware bijective remap (cdna_hip_programming.md T1): blocks b and b+8 share an XCD, so give
// each XCD a contiguous range of logical ids (tiles / slices that share operands then share that XCD's L2).
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
  int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (b >> 3);
}

__device__ __forceinline__ f32x16 mfma_bf16(u32x4 a, u32x4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0,
                                                  0);
}
// a.b over the six largest plane products (smallest first): the dropped a1.b2 + a2.b1 + a2.b2 is
// below 2^-22 |a||b|, one f32 rounding of the product
__device__ __forceinline__ f32x16 mfma_split6(const u32x4 (&a)[3], const u32x4 (&b)[3], f32x16 c) {
  c = mfma_bf16(a[0], b[2], c);
  c = mfma_bf16(a[2], b[0], c);
  c = mfma_bf16(a[1], b[1], c);
  c = mfma_bf16(a[0], b[1], c);
  c = mfma_bf16(a[1], b[0], c);
  return mfma_bf16(a[0], b[0], c);
}
template <int TERMS>
__device__ __forceinline__ f32x16 mfma_terms(const u32x4 (&a)[3], const u32x4 (&b)[3], f32x16 c) {
  if constexpr (TERMS == 1) return mfma_bf16(a[0], b[0], c);
  else return mfma_split6(a, b, c);
}

// ---- scaled fp16 pair (the plane GEMM's split mode; attention_slice.hip has the 16x16 form) -----------------
// x s = h + l, h = fp16(x s), l = fp16(x s - h) (round to nearest even): 22 significant bits when the power-of-two
// scale s puts the operand's largest magnitude in [2^13, 2^14); a product is h h' + h l' + l h' (the dropped l l'
// is below 2^-22 |a||b|)
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float pow2_scale14(float m) {
  const int e = (int)((__float_as_uint(m) >> 23) & 255u);   // m in [2^(e-127), 2^(e-126))
  int se = 127 + 13 - (e - 127);
  se = e == 0 ? 127 : (se < 1 ? 1 : (se > 254 ? 254 : se));
  // an inf / NaN bound (a diverged producer) gives a NaN scale: the product turns NaN instead of silently 0
  return e == 255 ? __builtin_nanf("") : __uint_as_float((uint32_t)se << 23);
}
// 4 floats (already scaled) -> the fp16 pair's planes, 8 B each
__device__ __forceinline__ void pair4(f32x4 v, u32x2& hi, u32x2& lo) {
  const f32x2_t x0 = f32x2_t{v.x, v.y}, x1 = f32x2_t{v.z, v.w};
  const f16x2_t h0 = __builtin_convertvector(x0, f16x2_t), h1 = __builtin_convertvector(x1, f16x2_t);
  const f16x2_t l0 = __builtin_convertvector(x0 - __builtin_convertvector(h0, f32x2_t), f16x2_t);
  const f16x2_t l1 = __builtin_convertvector(x1 - __builtin_convertvector(h1, f32x2_t), f16x2_t);
  hi = u32x2{__builtin_bit_cast(uint32_t, h0), __builtin_bit_cast(uint32_t, h1)};
  lo = u32x2{__builtin_bit_cast(uint32_t, l0), __builtin_bit_cast(uint32_t, l1)};
}
// per-tensor magnitude bounds for the fp16-pair weight gradient: a producer max-reduces |value| over what it stores
// and folds it into *amax (zeroed by the caller) with one atomic per wave — max is order-independent, so the bound
// is deterministic.  Non-negative floats order like their bit patterns; NaNs are skipped by fmaxf.
__device__ __forceinline__ float amax4(float m, f32x4 v) {
  return fmaxf(fmaxf(m, fmaxf(fabsf(v.x), fabsf(v.y))), fmaxf(fabsf(v.z), fabsf(v.w)));
}
// One address takes every wave's max: the atomic is issued only when the wave's max exceeds the value the wave reads
// there (a plain, possibly stale load: stale is smaller, so at worst an atomic too many) — after the first waves the
// maximum is in and the rest skip it (a million unconditional atomics per launch serialised at one L2 channel:
// measured 9 ms per C2 step in the row-wise kernels and 4 in the attention forward)
__device__ __forceinline__ void amax_flush(float* amax, float m) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if (amax && (threadIdx.x & 63) == 0 && __float_as_uint(m) > *reinterpret_cast<volatile unsigned int*>(amax))
    atomicMax(reinterpret_cast<unsigned int*>(amax), __float_as_uint(m));
}
// x s is saturated to the fp16 range first (v_med3_f32): a row bound that under-estimates the operand (a stale or
// wrong a_rowmax) then gives a deterministic, finite, clipped product instead of an inf plane and inf - inf = NaN
__device__ __forceinline__ void pair8(const float* v, float s, u32x4 (&pl)[3]) {
  uint32_t a[4], b[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const f32x2_t x = f32x2_t{__builtin_amdgcn_fmed3f(v[2 * k] * s, -65504.f, 65504.f),
                              __builtin_amdgcn_fmed3f(v[2 * k + 1] * s, -65504.f, 65504.f)};
    const f16x2_t h = __builtin_convertvector(x, f16x2_t);
    const f16x2_t l = __builtin_convertvector(x - __builtin_convertvector(h, f32x2_t), f16x2_t);
    a[k] = __builtin_bit_cast(uint32_t, h);
    b[k] = __builtin_bit_cast(uint32_t, l);
  }
  pl[0] = u32x4{a[0], a[1], a[2], a[3]};
  pl[1] = u32x4{b[0], b[1], b[2], b[3]};
}
__device__ __forceinline__ f32x16 mfma_f16(u32x4 a, u32x4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c, 0, 0,
                                                 0);
}
__device__ __forceinline__ f32x16 mfma_pair(const u32x4 (&a)[3], const u32x4 (&b)[3], f32x16 c) {
  c = mfma_f16(a[0], b[1], c);
  c = mfma_f16(a[1], b[0], c);
  return mfma_f16(a[0], b[0], c);
}

// ---- error reporting (per host thread) ---------------------------------------------
void set_error(const char* fmt, ...);
int fail(int code, const char* fmt, ...);

#define OT_REQUIRE(cond, ...)                                   \
  do {                                                          \
    if (!(cond)) return ::ot::fail(OT_ERR_INVALID_ARG, __VA_ARGS__); \
  } while (0)

#define OT_LAUNCH_CHECK(name)                                                        \
  do {                                                                              \
    hipError_t _e = hipGetLastError();                                              \
    if (_e != hipSuccess)                                                           \
      return ::ot::fail(OT_ERR_HIP, "%s: %s", name, hipGetErrorString(_e));         \
  } while (0)

// ---- dropout: counter-based mask (oracle/keras_math.py::dropout_keep) ---------------
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
  return h;
}
// keep iff hash >= thr (thr = round(rate * 2^32)); index = (b*I + p)*d + n
__device__ __forceinline__ bool drop_keep(uint32_t seed, uint32_t site, uint32_t index, uint32_t thr) {
  uint32_t h = index * 0x9E3779B1u + seed;
  h ^= site * 0x85EBCA77u;
  return fmix32(h) >= thr;
}

// token index in the layer-input space for compacted row r of a layer keeping K of I tokens per
// sample: the tail (p = I - K + j) or, when `pos` is given (ot_pyramid_select), p = pos[r]
__device__ __forceinline__ int64_t tail_token(int64_t r, int K, int I, const int32_t* pos = nullptr) {
  if (pos) return (r / K) * I + pos[r];
  if (K == I) return r;
  int64_t b = r / K;
  return b * I + (I - K) + (r - b * K);
}

// inverse: compact row of input row o (b*I + p), or -1 when p is not kept (`inv` from
// ot_pyramid_select, else the tail rule)
__device__ __forceinline__ int64_t kept_row(int64_t o, int K, int I, const int32_t* inv = nullptr) {
  if (inv) return inv[o];
  const int64_t b = o / I, j = o - b * I - (I - K);
  return j >= 0 ? b * K + j : -1;
}

// erf for the GELU: branch-free rational minimax on [-4, 4] (|error| < 5e-7; erf(±4) rounds to ±1 in
// fp32).  This is the float erf TensorFlow's CPU kernels evaluate (Eigen's generic fast erf), so it
// is also the reference's own arithmetic; ~15 VALU ops instead of the two-regime libm erff.
// Every multiply-add is an explicit fma (no contraction left to the compiler) so the scalar form and the
// packed-pair form below give identical bits per element; the pair form runs the polynomials on
// v_pk_fma_f32 / v_pk_mul_f32 (half the VALU issue of four scalar evaluations: the GELU prologues and
// epilogues of the FFN GEMMs evaluate it once per element of a [rows, f] tensor).
typedef float f32x2 __attribute__((ext_vector_type(2)));
#define OT_ERF_P(V, T)                                                   \
  V = __builtin_elementwise_fma(V, x2, (T)(2.77068142495902e-08f));      \
  V = __builtin_elementwise_fma(V, x2, (T)(-2.10102402082508e-06f));     \
  V = __builtin_elementwise_fma(V, x2, (T)(-5.69250639462346e-05f));     \
  V = __builtin_elementwise_fma(V, x2, (T)(-7.34990630326855e-04f));     \
  V = __builtin_elementwise_fma(V, x2, (T)(-2.95459980854025e-03f));     \
  V = __builtin_elementwise_fma(V, x2, (T)(-1.60960333262415e-02f));
#define OT_ERF_Q(V, T)                                                   \
  V = __builtin_elementwise_fma(V, x2, (T)(-2.13374055278905e-04f));     \
  V = __builtin_elementwise_fma(V, x2, (T)(-1.68282697438203e-03f));     \
  V = __builtin_elementwise_fma(V, x2, (T)(-7.37332916720468e-03f));     \
  V = __builtin_elementwise_fma(V, x2, (T)(-1.42647390514189e-02f));
// 1 + erf(a)
__device__ __forceinline__ float one_plus_erf(float a) {
  const float x = fminf(fmaxf(a, -4.f), 4.f);
  const float x2 = x * x;
  float p = -2.72614225801306e-10f;
  OT_ERF_P(p, float)
  float q = -1.45660718464996e-05f;
  OT_ERF_Q(q, float)
  return __builtin_fmaf(x * p, __builtin_amdgcn_rcpf(q), 1.0f);
}
__device__ __forceinline__ f32x2 one_plus_erf2(f32x2 a) {
  const f32x2 x = __builtin_elementwise_min(__builtin_elementwise_max(a, (f32x2)(-4.f)), (f32x2)(4.f));
  const f32x2 x2 = x * x;
  f32x2 p = (f32x2)(-2.72614225801306e-10f);
  OT_ERF_P(p, f32x2)
  f32x2 q = (f32x2)(-1.45660718464996e-05f);
  OT_ERF_Q(q, f32x2)
  const f32x2 r = {__builtin_amdgcn_rcpf(q.x), __builtin_amdgcn_rcpf(q.y)};
  return __builtin_elementwise_fma(x * p, r, (f32x2)(1.0f));
}
#undef OT_ERF_P
#undef OT_ERF_Q
__device__ __forceinline__ float gelu_erf(float x) {
  return (0.5f * x) * one_plus_erf(x * 0.70710678118654752440f);
}
__device__ __forceinline__ float gelu_erf_grad(float x) {
  // d/dx 0.5 x (1 + erf(x/sqrt2)) = 0.5 (1 + erf(x/sqrt2)) + x * exp(-x^2/2) / sqrt(2 pi)
  return __builtin_fmaf(x * 0.39894228040143267794f, __builtin_amdgcn_exp2f((-0.72134752044448170368f * x) * x),
                        0.5f * one_plus_erf(x * 0.70710678118654752440f));
}
__device__ __forceinline__ f32x2 gelu_erf2(f32x2 x) {
  return (0.5f * x) * one_plus_erf2(x * 0.70710678118654752440f);
}
__device__ __forceinline__ f32x2 gelu_erf_grad2(f32x2 x) {
  const f32x2 t = (-0.72134752044448170368f * x) * x;
  const f32x2 e = {__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
  return __builtin_elementwise_fma(x * 0.39894228040143267794f, e, 0.5f * one_plus_erf2(x * 0.70710678118654752440f));
}
// four elements as two packed pairs (bit-identical to gelu_erf / gelu_erf_grad per element)
__device__ __forceinline__ f32x4 gelu_erf4(f32x4 v) {
  const f32x2 a = gelu_erf2(f32x2{v.x, v.y}), b = gelu_erf2(f32x2{v.z, v.w});
  return f32x4{a.x, a.y, b.x, b.y};
}
__device__ __forceinline__ f32x4 gelu_erf_grad4(f32x4 v) {
  const f32x2 a = gelu_erf_grad2(f32x2{v.x, v.y}), b = gelu_erf_grad2(f32x2{v.z, v.w});
  return f32x4{a.x, a.y, b.x, b.y};
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

inline unsigned ceil_div(int64_t a, int64_t b) { return (unsigned)((a + b - 1) / b); }

}  // namespace ot

namespace ot {
inline uint32_t drop_threshold(float rate) {
  double thr = (double)rate * 4294967296.0;
  return thr >= 4294967295.0 ? 4294967295u : (uint32_t)llround(thr);
}
}  // namespace ot

namespace ot {
// out[c] (+)= sum_b part[b][c], deterministic (rowwise.hip); shared by the fused row-norm epilogue
// (scratch: colsum_scratch_floats(nparts, ncols) floats, used when nparts > 256)
int64_t colsum_scratch_floats(int64_t nparts, int ncols);
void launch_colsum_reduce(const float* part, int64_t nparts, int ncols, float* out, int accumulate, hipStream_t s,
                          float* scratch);
}  // namespace ot
