// Short-sequence causal attention (I <= 192 keys) on split-bf16 MFMA, one workgroup per (sample, head)
// slice.  Replaces model.py:100-114 (QK^T / sqrt(hd), band_part causal mask, softmax, PV) and its
// gradient for the f32-accurate mode (OT_MATMUL_SPLIT_BF16) at head_dim 32 / 64; the backward also in two long
// forms at head_dim 64 (I <= 544, K <= 272: the query side in LDS, the key side from global; see bwd_form).
//
// Why a new kernel family: the per-(sample, head)-wave kernels of attention.hip
// walk (key block, query block) pairs and re-read the Q / dO block and read-modify-write the running
// dQ partial once per pair (about 2x the compulsory bytes through L2 at I = 140), on f32 MFMA
// (64 cycles per 32x32x2).  Here one workgroup owns a whole (sample, head) slice:
//   * every operand is read from HBM once and split once, exactly, into three bf16 planes
//     (x = x0 + x1 + x2, common.h split8) staged in LDS; every product is the sum of the six largest
//     plane products on v_mfma_f32_16x16x32_bf16 (f32-accurate, 2.7x fewer MFMA cycles than the f32 form);
//   * 16-row blocks: at I = 140 the causal triangle keeps 45 of 81 block pairs (useful fraction 0.86
//     against 0.64 for 32-row blocks);
//   * backward, phase 1 (key-block owners): dV, dK accumulate in registers over the query blocks,
//     dS of every causal block goes to an LDS store; phase 2 (query-block owners): dQ = dS K from the
//     store and a K image — Q / dO read once, dQ / dK / dV written once, no atomics, deterministic.
//
// Operand maps (cdna_hip_programming.md §3, 16x16x32 bf16): lane l holds A[row l&15][k 8(l>>4)+j] and
// B[k 8(l>>4)+j][col l&15]; C/D: col l&15, rows 4(l>>4)+i.  A product that sums over an accumulator's
// ROW index takes the accumulator registers as its B operand with the k order permuted: k-slot j of lane
// group g is row 4g + j of block a (j < 4) or of block a + 1 (j >= 4); the other operand, read from a
// row-major [row][dim] plane image by ds_read_b64_tr_b16 (two reads of 4 rows), follows the same order.
//
// LDS plane images are [row][HD] bf16, 16-byte chunks XOR-swizzled per row (poff) so that both the
// ds_read_b128 row reads (16 rows x one chunk per lane group) and the transposed reads are conflict-free.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <mutex>

#include "common.h"
#include "attn_slice.h"

namespace ot {
namespace slice {

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

constexpr int MAXKB = 12;                          // 16-key blocks per slice (I <= 192)
constexpr float L2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;
constexpr int LDS_MAX = 160 * 1024;

// byte offset of 16-byte chunk c of row `row` in a [rows][HD] bf16 plane image
template <int HD>
__device__ __forceinline__ int poff(int row, int c) {
  if constexpr (HD == 64) return row * 128 + 16 * (c ^ (((row >> 1) & 3) << 1));
  else return row * 64 + 16 * (c ^ ((-(row >> 2)) & 3));
}

__device__ __forceinline__ f32x4 mma(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                  0, 0);
}
// a.b over the six largest plane products, smallest first (as mfma_split6)
__device__ __forceinline__ f32x4 mma6(const u32x4 (&a)[3], const u32x4 (&b)[3], f32x4 c) {
  c = mma(a[0], b[2], c);
  c = mma(a[2], b[0], c);
  c = mma(a[1], b[1], c);
  c = mma(a[0], b[1], c);
  c = mma(a[1], b[0], c);
  return mma(a[0], b[0], c);
}

// lane (row, group g) <- dims 32t + 8g .. +7 of `row`, three planes (pb bytes apart)
template <int HD>
__device__ __forceinline__ void row_frag(u32x4 (&f)[3], const char* img, int pb, int row, int t, int g) {
  const int o = poff<HD>(row, 4 * t + g);
#pragma unroll
  for (int pl = 0; pl < 3; ++pl) f[pl] = *reinterpret_cast<const u32x4*>(img + pl * pb + o);
}

// lane (column i, group g) <- column 16m + i of rows ra + 4g + 0..3 (elements 0-3) and rb + 4g + 0..3
// (elements 4-7): lane 4q + p of each 16-lane group addresses row r + q, columns 16m + 4p .. +3
template <int HD>
__device__ __forceinline__ void tr_frag(u32x4 (&f)[3], const char* img, int pb, int ra, int rb, int m, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int c = 2 * m + (pp >> 1), e = 8 * (pp & 1);
  const int o0 = poff<HD>(ra + 4 * g + q, c) + e, o1 = poff<HD>(rb + 4 * g + q, c) + e;
#pragma unroll
  for (int pl = 0; pl < 3; ++pl) {
    const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(img + pl * pb + o0));
    const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(img + pl * pb + o1));
    const u32x2 x = __builtin_bit_cast(u32x2, lo), y = __builtin_bit_cast(u32x2, hi);
    f[pl] = u32x4{x.x, x.y, y.x, y.y};
  }
}

// the same reads from precomputed per-lane offsets: every plane image row block of 16 rows has the same
// swizzle (the XOR terms of poff depend on row mod 8 / 16 only), so the offset of (block, lane) is
// block * 16 * row bytes + a per-lane constant, and a loop adds one uniform term per block
__device__ __forceinline__ void frag_at(u32x4 (&f)[3], const char* p, int pb) {
#pragma unroll
  for (int pl = 0; pl < 3; ++pl) f[pl] = *reinterpret_cast<const u32x4*>(p + pl * pb);
}
__device__ __forceinline__ void tr_at(u32x4 (&f)[3], const char* p0, const char* p1, int pb) {
#pragma unroll
  for (int pl = 0; pl < 3; ++pl) {
    const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(p0 + pl * pb));
    const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(p1 + pl * pb));
    const u32x2 x = __builtin_bit_cast(u32x2, lo), y = __builtin_bit_cast(u32x2, hi);
    f[pl] = u32x4{x.x, x.y, y.x, y.y};
  }
}
// split8 with the two subtractions of each element pair on packed-f32 adds (v_pk_add_f32); the planes are
// the high halves of x, r1, r2 (v_perm), so only the residuals need the masked values.  Bit-identical to split8.
__device__ __forceinline__ void split8p(const float* v, u32x4 (&pl)[3]) {
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  uint32_t a[4], b[4], c[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const f32x2 x = {v[2 * k], v[2 * k + 1]};
    const f32x2 x0 = {__uint_as_float(__float_as_uint(x.x) & 0xffff0000u), __uint_as_float(__float_as_uint(x.y) & 0xffff0000u)};
    const f32x2 r1 = x - x0;
    const f32x2 x1 = {__uint_as_float(__float_as_uint(r1.x) & 0xffff0000u), __uint_as_float(__float_as_uint(r1.y) & 0xffff0000u)};
    const f32x2 r2 = r1 - x1;
    a[k] = __builtin_amdgcn_perm(__float_as_uint(x.y), __float_as_uint(x.x), 0x07060302u);
    b[k] = __builtin_amdgcn_perm(__float_as_uint(r1.y), __float_as_uint(r1.x), 0x07060302u);
    c[k] = __builtin_amdgcn_perm(__float_as_uint(r2.y), __float_as_uint(r2.x), 0x07060302u);
  }
  pl[0] = u32x4{a[0], a[1], a[2], a[3]};
  pl[1] = u32x4{b[0], b[1], b[2], b[3]};
  pl[2] = u32x4{c[0], c[1], c[2], c[3]};
}

// max / sum with the lane 16 and 32 apart (the 4 lane groups of a 16x16 accumulator column) on the VALU
// lane-swap instructions (no LDS round trip as ds_bpermute): each swap hands every lane its own value and
// its partner's, in some order — max and + are symmetric, so all four groups get identical results
__device__ __forceinline__ float group_max(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float group_sum(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

__device__ __forceinline__ void load8(float (&v)[8], const float* src) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(src), b = *reinterpret_cast<const f32x4*>(src + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// 8 floats -> planes written to three plane images at byte offset o
__device__ __forceinline__ void store_planes(char* img, int pb, int o, const float (&v)[8]) {
  u32x4 pl[3];
  split8(v, pl);
#pragma unroll
  for (int k = 0; k < 3; ++k) *reinterpret_cast<u32x4*>(img + k * pb + o) = pl[k];
}

// ---- two-plane fp16 form (NP = 2).  x s = h + l with h = fp16(x s), l = fp16(x s - h) (round to nearest even,
// v_cvt_pk_f16_f32): 22 significant bits, and a product is the sum of the three largest plane products
// (h h' + h l' + l h', v_mfma_f32_16x16x32_f16; the dropped l l' is below 2^-22 |a||b|).  The power-of-two scale s
// puts the operand's largest magnitude in [2^13, 2^14) so every plane is a normal fp16 (smaller elements keep an
// absolute error below 2^-25 of that scale).  Emulated against float64 at the C2 / T slice shapes this is as
// accurate as the three-plane bf16 split with six products (1e-7 - 4e-7 of max|x| on O, dQ, dK, dV), at half the
// MFMAs, two planes of LDS images instead of three and a cheaper split.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x4 mmh(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}
template <int NP>
__device__ __forceinline__ f32x4 mmaN(const u32x4 (&a)[NP], const u32x4 (&b)[NP], f32x4 c) {
  if constexpr (NP == 3) {
    return mma6(a, b, c);
  } else {
    c = mmh(a[0], b[1], c);
    c = mmh(a[1], b[0], c);
    return mmh(a[0], b[0], c);
  }
}
// 8 floats -> NP planes; NP = 2: of v * s (s a power of two); NP = 3: the exact bf16 split (s must be 1)
template <int NP>
__device__ __forceinline__ void splitN(const float* v, float s, u32x4 (&pl)[NP]) {
  if constexpr (NP == 3) {
    split8p(v, pl);
  } else {
    uint32_t a[4], b[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const f32x2 x = f32x2{v[2 * k], v[2 * k + 1]} * s;
      const f16x2 h = __builtin_convertvector(x, f16x2);
      const f16x2 l = __builtin_convertvector(x - __builtin_convertvector(h, f32x2), f16x2);
      a[k] = __builtin_bit_cast(uint32_t, h);
      b[k] = __builtin_bit_cast(uint32_t, l);
    }
    pl[0] = u32x4{a[0], a[1], a[2], a[3]};
    pl[1] = u32x4{b[0], b[1], b[2], b[3]};
  }
}
template <int NP>
__device__ __forceinline__ void frag_atN(u32x4 (&f)[NP], const char* p, int pb) {
#pragma unroll
  for (int pl = 0; pl < NP; ++pl) f[pl] = *reinterpret_cast<const u32x4*>(p + pl * pb);
}
template <int NP>
__device__ __forceinline__ void tr_atN(u32x4 (&f)[NP], const char* p0, const char* p1, int pb) {
#pragma unroll
  for (int pl = 0; pl < NP; ++pl) {
    const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(p0 + pl * pb));
    const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(p1 + pl * pb));
    const u32x2 x = __builtin_bit_cast(u32x2, lo), y = __builtin_bit_cast(u32x2, hi);
    f[pl] = u32x4{x.x, x.y, y.x, y.y};
  }
}
template <int NP>
__device__ __forceinline__ void store_planesN(char* img, int pb, int o, const float (&v)[8], float s) {
  u32x4 pl[NP];
  if constexpr (NP == 3) split8(v, pl);
  else splitN<2>(v, s, pl);
#pragma unroll
  for (int k = 0; k < NP; ++k) *reinterpret_cast<u32x4*>(img + k * pb + o) = pl[k];
}
// power-of-two scale putting a largest magnitude m in [2^13, 2^14) (1 for m = 0; clamped to the normal range)
__device__ __forceinline__ float pow2scale(float m) {
  const int e = (int)((__float_as_uint(m) >> 23) & 255u);   // m in [2^(e-127), 2^(e-126))
  int se = 127 + 13 - (e - 127);
  se = e == 0 ? 127 : (se < 1 ? 1 : (se > 254 ? 254 : se));
  return __uint_as_float((uint32_t)se << 23);
}
__device__ __forceinline__ float wave_maxf(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

// tail queries: first 16-query block whose last query sees key block kb (query blocks before the last
// end at 16f + 15 < K, so the first f with q_off + 16f + 15 >= 16 kb, capped at the last block)
__host__ __device__ inline int tail_qf(int kb, int q_off, int nqb) {
  const int num = 16 * kb - q_off - 15;
  const int f = num <= 0 ? 0 : (num + 15) / 16;
  return f < nqb - 1 ? f : nqb - 1;
}

// ------------------------------------------------------------------------------------------
// Plane images have compile-time strides (RMAX rows per plane), so every LDS address is a per-lane base
// plus an immediate.  hd 64: 144 rows (the backward's LDS limit at I = 140), hd 32: 192.
template <int HD>
constexpr int RMAX() { return HD == 64 ? 144 : 192; }
// key blocks a backward wave may own (its K planes are kept in registers for the phase-2 K image): at most
// RMAX / 16 key blocks (9 at hd 64, 12 at hd 32) over the workgroup's waves
__host__ __device__ constexpr int keep_slots(int hd, int nwv) {
  return ((hd == 64 ? 144 : 192) / 16 + nwv - 1) / nwv;
}

// the wave's schedule row as one uniform 64-bit value (a scalar load at kernel start: an in-loop vector
// load of the kernel argument would wait, in-order, for every prefetch load issued before it)
__device__ __forceinline__ uint64_t sched_row(const SliceArgs& p, int phase, int wave) {
  const uint64_t* rows = reinterpret_cast<const uint64_t*>(&p.sched[0][0][0]);
  const uint64_t r = rows[phase * 8 + wave];
  return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(r >> 32)) << 32) |
         (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)r);
}
__device__ __forceinline__ int sched_item(uint64_t row, int slot) {
  return slot < 8 ? (int)(int8_t)(row >> (8 * slot)) : -1;
}

// Diagnostic build only (-DOT_SLICE_STAMPS=1, a separate library: tools/slice_stamps.py): thread 0 of each
// workgroup records the shader clock at the phase boundaries of its first two slices.
#ifndef OT_SLICE_STAMPS
#define OT_SLICE_STAMPS 0
#endif
#if OT_SLICE_STAMPS
__device__ unsigned long long g_slice_stamps[2][2048][2][8];
#define SLICE_STAMP(kind, it, k)                                                                   \
  do {                                                                                           \
    if (threadIdx.x == 0 && (it) < 2 && blockIdx.x < 2048) g_slice_stamps[kind][blockIdx.x][it][k] = clock64(); \
  } while (0)
#else
#define SLICE_STAMP(kind, it, k) do {} while (0)
#endif

// The backward is persistent: a workgroup walks slices s = blockIdx.x, + gridDim.x, ... (grid = the co-resident
// workgroups); at head_dim 32 (one workgroup per CU by LDS) the next slice's operands are loaded into registers
// while the current slice computes, at head_dim 64 two workgroups per CU cover each other's loads.  The forward
// runs one slice per workgroup, two workgroups of 8 waves per CU (<= 128 VGPRs, <= 74 KiB of LDS): the other
// workgroup covers a slice's K / V loads.  (Round 5: the head_dim-64 forward as a persistent workgroup per CU
// with the next slice's K / V prefetched, 243 VGPRs, measured 574-631 us against 497-507 at B 4096 H 4 I 140.)

// ------------------------------------------------------------------------------------------
// Forward.  The slice's K and V planes are staged in LDS ([RMAX][HD] x 3 each); each wave takes whole
// 16-query blocks (host LPT schedule over the SIMDs, heaviest first).  Per query block the wave holds Q
// (pre-scaled by log2(e)/sqrt(hd), split) as the B operand of S^T = K Q^T (query on the lane) and
// computes S^T for every visible key block at once (<= 12 x 4 registers), so the softmax is exact in one
// pass (row max and sum over the 4 lane groups by shuffles, no rescaling); O^T = V^T P^T takes P^T from
// the S^T registers and V^T by transposed reads.  Loads in flight during compute: the next query block's Q.
// NP planes per operand: 3 = the exact bf16 split (6 products), 2 = the scaled fp16 pair (3 products, splitN): K and V
// each get a power-of-two scale per slice (the largest magnitude, reduced over the workgroup), Q one per query (lane)
template <int HD, int NWV, bool SEL, int NP>
__global__ __launch_bounds__(64 * NWV, 2) void attn_fwd_slice_kernel(SliceArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float am = 0.f;                                   // max |stored O| (p.amax)
  constexpr int NT = HD / 32, NM = HD / 16, CPR = HD / 8, NTH = 64 * NWV;
  constexpr int PB = RMAX<HD>() * HD * 2;
  constexpr int SR = (RMAX<HD>() * CPR + NTH - 1) / NTH;          // staging rounds
  const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // uniform
  const int I = p.I, K = p.K, q_off = I - K;
  const int nkb = (I + 15) >> 4, nqb = (K + 15) >> 4, IP = nkb * 16;
  const int nslices = p.B * p.H;
  char* kimg = smem;
  char* vimg = smem + NP * PB;
  int* qposl = reinterpret_cast<int*>(smem + 2 * NP * PB);           // SEL: the slice's kept positions
  float* red = reinterpret_cast<float*>(qposl + RMAX<HD>());          // NP = 2: per-wave K / V maxima
  const float qscale = p.scale * L2E;
  auto qkv_of = [&](int s) { return p.qkv + (int64_t)(s / p.H) * I * p.ld + (s % p.H) * HD; };
  // query positions: the tail rule, or (SEL) the slice's kept positions staged in LDS with K / V
  // staging rows past I (and tasks past IP) read row I - 1: finite, zeroed or skipped at store time
  float kr[SR][8], vr[SR][8], qr[NT][8];
  auto load_kv = [&](int s) {
    const float* Q = qkv_of(s);
#pragma unroll
    for (int r = 0; r < SR; ++r) {
      const int task = threadIdx.x + r * NTH, row = min(task / CPR, I - 1), c = task % CPR;
      load8(kr[r], Q + p.d + (int64_t)row * p.ld + 8 * c);
      load8(vr[r], Q + 2 * p.d + (int64_t)row * p.ld + 8 * c);
    }
  };
  auto qpos_of = [&](int j) { return SEL ? qposl[j] : q_off + j; };
  auto load_q = [&](int s, int idx) {
    const float* Q = qkv_of(s);
    const int j = min(16 * (nqb - 1 - idx) + li, K - 1);
    const int qp = qpos_of(j);
#pragma unroll
    for (int t = 0; t < NT; ++t) load8(qr[t], Q + (int64_t)qp * p.ld + 32 * t + 8 * g);
  };
  const uint64_t srow = sched_row(p, 0, wave);
  const int idx0 = sched_item(srow, 0);
  // per-lane LDS offsets of the fragment reads (see the backward): held opaque so each key block adds one
  // uniform term to a register instead of re-deriving image + plane constants per read
  int kbase[NT], vtbase[NM];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    kbase[t] = poff<HD>(li, 4 * t + g);
    asm volatile("" : "+v"(kbase[t]));
  }
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    vtbase[m] = poff<HD>(4 * g + ((lane >> 2) & 3), 2 * m + ((lane & 3) >> 1)) + 8 * (lane & 1) + NP * PB;
    asm volatile("" : "+v"(vtbase[m]));
  }
  const int s = blockIdx.x;
  if (s >= nslices) return;
  load_kv(s);
  if (!SEL && idx0 >= 0) load_q(s, idx0);
  {
    constexpr int it = 0;
    SLICE_STAMP(0, it, 0);
    float sk = 1.f, sv = 1.f;                                        // K / V scales (NP = 2)
    if constexpr (NP == 2) {
      float mk = 0.f, mv = 0.f;
#pragma unroll
      for (int r = 0; r < SR; ++r)
#pragma unroll
        for (int e = 0; e < 8; ++e) {                                 // (rows past I hold row I - 1)
          mk = fmaxf(mk, fabsf(kr[r][e]));
          mv = fmaxf(mv, fabsf(vr[r][e]));
        }
      mk = wave_maxf(mk);
      mv = wave_maxf(mv);
      if (lane == 0) {
        red[2 * wave] = mk;
        red[2 * wave + 1] = mv;
      }
      __syncthreads();
#pragma unroll
      for (int w = 0; w < NWV; ++w) {
        mk = fmaxf(mk, red[2 * w]);
        mv = fmaxf(mv, red[2 * w + 1]);
      }
      sk = pow2scale(mk);
      sv = pow2scale(mv);
    }
#pragma unroll
    for (int r = 0; r < SR; ++r) {
      const int task = threadIdx.x + r * NTH, row = task / CPR, c = task % CPR;
      if (task < IP * CPR) {
        if (row >= I) {
#pragma unroll
          for (int e = 0; e < 8; ++e) kr[r][e] = vr[r][e] = 0.f;
        }
        const int o = poff<HD>(row, c);
        store_planesN<NP>(kimg, PB, o, kr[r], sk);
        store_planesN<NP>(vimg, PB, o, vr[r], sv);
      }
    }
    if (SEL)
      for (int j = threadIdx.x; j < K; j += NTH) qposl[j] = p.qpos[(int64_t)(s / p.H) * K + j];
    __syncthreads();
    SLICE_STAMP(0, it, 1);
    if (SEL && idx0 >= 0) load_q(s, idx0);
    const int b = s / p.H, h = s % p.H;
#pragma unroll 1
    for (int slot = 0, idx = idx0; idx >= 0; ++slot) {
      const int qb = nqb - 1 - idx;
      const int j = 16 * qb + li;                                    // this lane's query
      const int qpos = qpos_of(j < K ? j : K - 1);
      const int kbl = qpos_of(min(16 * qb + 15, K - 1)) >> 4;        // last visible key block
      const int kbm = qpos_of(16 * qb) >> 4;                          // key blocks >= kbm may be masked
      u32x4 qp[NT][NP];
      float cs = 1.f;                                                 // NP = 2: S^T = acc * cs (this lane's query)
      if constexpr (NP == 2) {
        float mq = 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int e = 0; e < 8; ++e) mq = fmaxf(mq, fabsf(qr[t][e]));
        const float sq = pow2scale(group_max(mq) * qscale) * qscale;   // the query row is spread over 4 lane groups
#pragma unroll
        for (int t = 0; t < NT; ++t) splitN<2>(qr[t], sq, qp[t]);
        cs = qscale / (sk * sq);
      } else {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
#pragma unroll
          for (int e = 0; e < 8; ++e) qr[t][e] *= qscale;
          split8p(qr[t], qp[t]);
        }
      }
      const int idxn = sched_item(srow, slot + 1);
      if (idxn >= 0) load_q(s, idxn);                                // next block's Q, in flight meanwhile
      f32x4 sc[MAXKB];
      float mx = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < MAXKB; ++kb) {
        sc[kb] = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
        if (kb > kbl) continue;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          u32x4 fk[NP];
          frag_atN<NP>(fk, smem + 16 * HD * 2 * kb + kbase[t], PB);
          acc = mmaN<NP>(fk, qp[t], acc);                             // S^T: row = key, col = query
        }
        if (kb >= kbm) {
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i] = (16 * kb + 4 * g + i <= qpos) ? acc[i] : -INFINITY;
        }
        mx = fmaxf(mx, fmaxf(fmaxf(acc[0], acc[1]), fmaxf(acc[2], acc[3])));
        sc[kb] = acc;
      }
      mx = group_max(mx);
      // NP = 2: exp2 of the unscaled S^T, times 2^14 (P's scale, in the exponent: P' in [0, 2^14])
      const float mxc = NP == 2 ? 14.f - mx * cs : -mx;
      float l = 0.f;
#pragma unroll
      for (int kb = 0; kb < MAXKB; ++kb) {
        if (kb > kbl) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float e = __builtin_amdgcn_exp2f(NP == 2 ? fmaf(sc[kb][i], cs, mxc) : sc[kb][i] + mxc);
          sc[kb][i] = e;
          l += e;
        }
      }
      l = group_sum(l);
      f32x4 o[NM];
#pragma unroll
      for (int m = 0; m < NM; ++m) o[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < MAXKB; kb += 2) {
        if (kb > kbl) continue;
        const bool two = kb + 1 <= kbl;
        float v[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[i] = sc[kb][i];
          v[4 + i] = two ? sc[kb + 1][i] : 0.f;
        }
        u32x4 pp[NP];
        splitN<NP>(v, 1.f, pp);
#pragma unroll
        for (int m = 0; m < NM; ++m) {
          u32x4 fa[NP];
          const int ra = 16 * HD * 2 * kb, rb = two ? ra + 16 * HD * 2 : ra;
          tr_atN<NP>(fa, smem + ra + vtbase[m], smem + rb + vtbase[m], PB);
          o[m] = mmaN<NP>(fa, pp, o[m]);                              // O^T += V^T P^T
        }
      }
      float rm = 0.f;                                                 // this lane's max |O| (rowmax)
      if (j < K) {
        const float inv = 1.f / (NP == 2 ? l * sv : l);               // (NP = 2: l and O^T carry 2^14, O^T sv)
        float* orow = p.out + ((int64_t)b * K + j) * p.d + h * HD + 4 * g;
#pragma unroll
        for (int m = 0; m < NM; ++m) {
          *reinterpret_cast<f32x4*>(orow + 16 * m) = o[m] * inv;
          rm = amax4(rm, o[m] * inv);
        }
        am = fmaxf(am, rm);
        if (g == 0) p.lse[(int64_t)s * K + j] = NP == 2 ? (mx * cs - 14.f) * LN2 + __logf(l) : mx * LN2 + __logf(l);
      }
      if (p.rowmax) {                                                 // (uniform) the row's max |O| over its head
        rm = group_max(rm);
        if (j < K && g == 0) p.rowmax[((int64_t)b * K + j) * p.H + h] = rm;
      }
      idx = idxn;
    }
    SLICE_STAMP(0, it, 2);
  }
  if (p.amax) amax_flush(p.amax, am);               // |O| bound of the Wo weight gradient (fp16 pair)
}

// ------------------------------------------------------------------------------------------
// Backward (tail queries).  LDS: Q planes [RMAX][HD] x 3 (phase 2: the K image), dO planes x 3,
// lse (log2 units, +inf padding), delta = rowsum(dO o O) (formed here from one read of O), query
// positions, then the dS store: one 1 KiB [16 query][16 key] f32 block per causal block pair.
//   phase 1, key blocks (host LPT schedule), query steps of two 16-row blocks (a, a+1):
//     S = Q K^T, dP = dO V^T          A = Q / dO rows (ds_read_b128), B = K^T / V^T (registers)
//     P = exp2(S log2e/sqrt(hd) - lse), dS = P (dP - delta) / sqrt(hd)     (key on the lane)
//     dV^T += dO^T P, dK^T += Q^T dS  A = dO^T / Q^T (transposed reads), B = P / dS (registers)
//     dS -> store
//   phase 2, query blocks: dQ^T = K^T dS^T over the visible key blocks, two per step (K image re-read
//   from global — L2-warm — into the Q planes' space).
// Loads in flight during compute: the next key block's K / V (phase 1), the K image rows (issued by each
// wave as it leaves phase 1), and the next slice's Q / dO / O rows, lse and first K / V (phase 2).
// The next slice's loads are issued before phase 2 at head_dim 64 (overlapping it) and after it at head_dim
// 32 (measured: 1,688-1,697 vs 1,710-1,717 us at hd 64, 931-955 vs 943-1,019 us at hd 32; B 4096 H 4, I 140).
// Software pipelining of phase 1 (step a + 2's S / dP issued before step a's softmax gradient) measured
// 1-4% slower at hd 64 and within noise at hd 32; not kept.
// NP = 2 (the scaled fp16 pair): Q and dO get a power-of-two scale per slice and K / V per key block (the owner's),
// P is exp2(... + 14) (P' = P 2^14, in [0, 2^14]), phase 1's dS a per-key-block scale from the bound
// |dS| <= (hd max|dO| max|V| + max|delta|) / sqrt(hd); phase 2's K image and dS one slice scale each (maxima
// reduced through LDS at the phase-1 barrier).  Outputs are unscaled at their stores.
// G2: two workgroups per CU instead of one — the dS store goes to a per-workgroup global scratch (p.dsws,
// L2-resident) instead of LDS, so the LDS holds only the planes (75.7 KiB at hd 64); no cross-slice prefetch (its
// 120 registers do not fit the 256 of two waves per SIMD; the other workgroup's compute covers a slice's loads), the
// K image re-read from global (issued before the phase-1 barrier) instead of kept in registers, and phase 2's dS
// reads issued two key-block pairs ahead.
template <int HD, int NWV, int NP, bool LAT_ = NWV == 4, bool G2 = false, int RQ = RMAX<HD>(), int KR = RQ>
__global__ __launch_bounds__(64 * NWV, G2 ? 2 : 1) void attn_bwd_slice_kernel(SliceArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float am = 0.f;                                   // max |stored dQ / dK / dV| (p.amax)
  constexpr int NT = HD / 32, NM = HD / 16, CPR = HD / 8, NTH = 64 * NWV;
  constexpr int RM = RQ, PB = RM * HD * 2;
  // phase 2's K image: KR rows; past RQ (the long forms) its planes take twice the Q planes' stride, the second
  // plane over the dO planes (free after phase 1)
  static_assert(KR == RQ || (G2 && NP == 2 && KR <= 2 * RQ), "attn_bwd_slice_kernel: K image rows");
  constexpr int KPB = KR > RQ ? 2 * PB : PB;
  constexpr int SR = (RM * CPR + NTH - 1) / NTH;
  constexpr bool LAT = LAT_;                        // fragment reads one item ahead, fenced (one wave per SIMD)
  static_assert(NTH >= RM, "attn_bwd_slice_kernel: the staging gives each padded query row one thread");
  constexpr int RBY = HD * 2;                       // bytes per plane image row
  const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // uniform
  const int I = p.I, K = p.K, q_off = I - K;
  const int nkb = (I + 15) >> 4, nqb = (K + 15) >> 4, IP = nkb * 16, KP = nqb * 16;
  const int nslices = p.B * p.H;
  char* qimg = smem;
  char* oimg = smem + NP * PB;
  float* lse2 = reinterpret_cast<float*>(smem + 2 * NP * PB);
  float* dlt = lse2 + RM;
  int* qps = reinterpret_cast<int*>(dlt + RM);
  int* tab = qps + RM;                     // [TABN] first visible query block, [TABN] dS-store base per key block
  float* red = reinterpret_cast<float*>(tab + 2 * SLICE_TABN);   // NP = 2: per-wave maxima [3][8], [2][8]
  char* dss = G2 ? reinterpret_cast<char*>(p.dsws + (size_t)blockIdx.x * p.ds_floats) : reinterpret_cast<char*>(red + 32);
  const float c1 = p.scale * L2E;
  if (threadIdx.x < SLICE_TABN) {
    tab[threadIdx.x] = p.qf[threadIdx.x];
    tab[SLICE_TABN + threadIdx.x] = p.bbase[threadIdx.x];
  }
  const uint64_t srow1 = sched_row(p, 1, wave), srow2 = sched_row(p, 2, wave);
  // per-lane LDS offsets, held opaque (asm) so the compiler keeps one register per base and adds each
  // loop's uniform block offset to it once, instead of re-deriving image + plane constants past the
  // 16-bit immediate per read
  int rbase[NT], tbase[NM], orbase[NT], otbase[NM], dsw[4];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    rbase[t] = poff<HD>(li, 4 * t + g);
    orbase[t] = rbase[t] + NP * PB;
    asm volatile("" : "+v"(rbase[t]), "+v"(orbase[t]));
  }
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    tbase[m] = poff<HD>(4 * g + ((lane >> 2) & 3), 2 * m + ((lane & 3) >> 1)) + 8 * (lane & 1);
    otbase[m] = tbase[m] + NP * PB;
    asm volatile("" : "+v"(tbase[m]), "+v"(otbase[m]));
  }
  // dS block rows permuted within each group of four (row r at 4 (r / 4) + (r + r / 4) % 4): the phase-1 stores
  // of rows 4g + i (g = 0..3, one per 16-lane group) then fall in four different bank quarters (2 extra cycles
  // per store instruction otherwise); the phase-2 row reads stay conflict-free (tools/lds_conflicts.py)
  auto dsrow = [](int r) { return (r & ~3) | ((r + (r >> 2)) & 3); };
#pragma unroll
  for (int i = 0; i < 4; ++i) dsw[i] = poff<32>(dsrow(4 * g + i), li >> 2) + 4 * (li & 3);
  const int dsr = poff<32>(dsrow(li), g);
  auto qkv_of = [&](int s) { return p.qkv + (int64_t)(s / p.H) * I * p.ld + (s % p.H) * HD; };
  auto row_of = [&](int s) { return (int64_t)(s / p.H) * K * p.d + (s % p.H) * HD; };   // O / dO slice
  // rows past K / I read the last valid row (finite) and are zeroed at use, so no load is predicated
  float qr[SR][8], yr[SR][8], orr[SR][8], lsev;
  float kr[NT][8], vr[NT][8];
  auto load_kv = [&](int s, int kb) {
    const float* Kg = qkv_of(s) + p.d;
    const int krow = min(16 * kb + li, I - 1);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      load8(kr[t], Kg + (int64_t)krow * p.ld + 32 * t + 8 * g);
      load8(vr[t], Kg + p.d + (int64_t)krow * p.ld + 32 * t + 8 * g);
    }
  };
  const int kb0 = sched_item(srow1, 0);
  auto prefetch = [&](int s) {
    const float* Qg = qkv_of(s);
    const float* dOg = p.dout + row_of(s);
    const float* Og = p.o + row_of(s);
#pragma unroll
    for (int r = 0; r < SR; ++r) {
      const int task = threadIdx.x + r * NTH, j = min(task / CPR, K - 1), c = task % CPR;
      load8(qr[r], Qg + (int64_t)(q_off + j) * p.ld + 8 * c);
      load8(yr[r], dOg + (int64_t)j * p.d + 8 * c);
      load8(orr[r], Og + (int64_t)j * p.d + 8 * c);
    }
    lsev = p.lse_in[(int64_t)s * K + min((int)threadIdx.x, K - 1)];
  };
  int s = blockIdx.x;
  if (!G2 && s < nslices) prefetch(s);
#pragma unroll 1
  for (int it = 0; s < nslices; s += gridDim.x, ++it) {
    SLICE_STAMP(1, it, 0);
    if (G2) prefetch(s);                           // (G2: this slice's Q / dO / O rows, no cross-slice prefetch)
    // the first key block's K / V: issued here, not with the slice prefetch — loaded during phase 2, the
    // compiler parked them in AGPRs and drained every load (vmcnt(0)) to copy them out before phase 2.  Here
    // they stay in flight through the staging (which waits only for the older Q / dO / O loads)
    if (kb0 >= 0) load_kv(s, kb0);
    float* dQg = p.dqkv + (int64_t)(s / p.H) * I * p.ld + (s % p.H) * HD;
    float* dKg = dQg + p.d;
    float* dVg = dQg + 2 * p.d;
    const float* Kg = qkv_of(s) + p.d;

    // ---- stage the query side from the prefetched registers
    if ((int)threadIdx.x < KP) {
      const bool v = (int)threadIdx.x < K;
      qps[threadIdx.x] = v ? q_off + threadIdx.x : -1;
      lse2[threadIdx.x] = v ? lsev * L2E - (NP == 2 ? 14.f : 0.f) : INFINITY;   // (NP = 2: P' = P 2^14)
    }
    float sq = 1.f, so = 1.f, mo = 0.f, mdl = 0.f;                  // Q / dO scales, max|dO|, max|delta| (NP = 2)
#pragma unroll
    for (int r = 0; r < SR; ++r) {
      // query rows past K hold row K - 1 (finite): their P and dS are 0 (lse +inf, qpos -1) and their dQ is
      // not stored, so they need no zeroing
      const int task = threadIdx.x + r * NTH, j = task / CPR, c = task % CPR;
      float pd = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) pd = fmaf(yr[r][e], orr[r][e], pd);
#pragma unroll
      for (int off = 1; off < CPR; off <<= 1) pd += __shfl_xor(pd, off, 64);
      if (task < KP * CPR && c == 0) dlt[j] = pd;
      if constexpr (NP == 2) mdl = fmaxf(mdl, fabsf(pd));
    }
    if constexpr (NP == 2) {
      float mq = 0.f;
#pragma unroll
      for (int r = 0; r < SR; ++r)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          mq = fmaxf(mq, fabsf(qr[r][e]));
          mo = fmaxf(mo, fabsf(yr[r][e]));
        }
      mq = wave_maxf(mq);
      mo = wave_maxf(mo);
      mdl = wave_maxf(mdl);
      if (lane == 0) {
        red[wave] = mq;
        red[8 + wave] = mo;
        red[16 + wave] = mdl;
      }
      __syncthreads();
#pragma unroll
      for (int w = 0; w < NWV; ++w) {
        mq = fmaxf(mq, red[w]);
        mo = fmaxf(mo, red[8 + w]);
        mdl = fmaxf(mdl, red[16 + w]);
      }
      sq = pow2scale(mq);
      so = pow2scale(mo);
    }
#pragma unroll
    for (int r = 0; r < SR; ++r) {
      const int task = threadIdx.x + r * NTH, j = task / CPR, c = task % CPR;
      if (task < KP * CPR) {
        const int o = poff<HD>(j, c);
        store_planesN<NP>(qimg, PB, o, qr[r], sq);
        store_planesN<NP>(oimg, PB, o, yr[r], so);
      }
    }
    __syncthreads();
    SLICE_STAMP(1, it, 1);

    // ---- phase 1: key-block owners
    constexpr int KEEP = keep_slots(HD, NWV);
    // the owned key blocks' K planes (NP = 3) or K rows (NP = 2: split at the slice scale after phase 1), for the
    // phase-2 K image
    u32x4 keep[NP == 3 && !G2 ? KEEP : 1][NT][3];
    float keepf[NP == 2 && !G2 ? KEEP : 1][NT][8];      // (G2: the K image is re-read from global, L2-warm)
    float mkw = 0.f, mdsw = 0.f;                   // NP = 2: this wave's max |K| and max |dS| (phase 2's scales)
#pragma unroll 1
    for (int slot = 0, kb = kb0; kb >= 0; ++slot) {
      const int krow = 16 * kb + li;               // this lane's key
      // keys past I hold row I - 1 (finite): their S / dP columns are masked (P = dS = 0, a select) and
      // their dK / dV rows are not stored, so they need no zeroing
      u32x4 kp[NT][NP], vp[NT][NP];
      float sk = 1.f, sv = 1.f, cS = c1, cdp = 1.f, sds = 1.f, dsc = p.scale;
      if constexpr (NP == 2) {
        float mk = 0.f, mv = 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            mk = fmaxf(mk, fabsf(kr[t][e]));
            mv = fmaxf(mv, fabsf(vr[t][e]));
          }
        mk = wave_maxf(mk);
        mv = wave_maxf(mv);
        mkw = fmaxf(mkw, mk);
        sk = pow2scale(mk);
        sv = pow2scale(mv);
        cS = c1 / (sq * sk);
        cdp = 1.f / (so * sv);
        sds = pow2scale(((float)HD * mo * mv + mdl) * p.scale);     // bound on this key block's |dS|
        dsc = p.scale * (1.f / 16384.f);                            // dS = P' (dP - delta) / sqrt(hd) / 2^14
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        splitN<NP>(kr[t], sk, kp[t]);
        splitN<NP>(vr[t], sv, vp[t]);
      }
#pragma unroll
      for (int k2 = 0; k2 < (G2 ? 0 : KEEP); ++k2)   // uniform branch, static register index
        if (slot == k2) {
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            if constexpr (NP == 3) {
#pragma unroll
              for (int pl = 0; pl < 3; ++pl) keep[k2][t][pl] = kp[t][pl];
            } else {
#pragma unroll
              for (int e = 0; e < 8; ++e) keepf[k2][t][e] = kr[t][e];
            }
          }
        }
      const int kbn = sched_item(srow1, slot + 1);
      if (kbn >= 0) load_kv(s, kbn);                // next key block's K / V in flight meanwhile
      f32x4 dk[NM], dv[NM];
#pragma unroll
      for (int m = 0; m < NM; ++m) dk[m] = dv[m] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int a0 = tab[kb], blk0 = tab[SLICE_TABN + kb];
      // S and dP of query step a (blocks a, a + 1; the second zero past the last block).  With one wave per
      // SIMD nothing else hides LDS latency, so each (half, t) item's fragments are read one item ahead
      // (sched_barrier keeps the compiler from sinking the reads back to their MFMAs)
      auto sdp = [&](int a, bool two, f32x4 (&sc)[2], f32x4 (&dc)[2]) {
        constexpr int NI = 2 * NT;
        u32x4 fq[2][NP], fo[2][NP];
        frag_atN<NP>(fq[0], smem + 16 * RBY * a + rbase[0], PB);
        frag_atN<NP>(fo[0], smem + 16 * RBY * a + orbase[0], PB);
#pragma unroll
        for (int h = 0; h < 2; ++h) sc[h] = dc[h] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          if (i + 1 < NI) {
            const int qb1 = two ? a + (i + 1) / NT : a;            // past the last block: a harmless re-read
            frag_atN<NP>(fq[(i + 1) & 1], smem + 16 * RBY * qb1 + rbase[(i + 1) % NT], PB);
            frag_atN<NP>(fo[(i + 1) & 1], smem + 16 * RBY * qb1 + orbase[(i + 1) % NT], PB);
          }
          const int half = i / NT, t = i % NT;
          if (half == 0 || two) {
            sc[half] = mmaN<NP>(fq[i & 1], kp[t], sc[half]);        // S: row = query, col = key
            dc[half] = mmaN<NP>(fo[i & 1], vp[t], dc[half]);        // dP
          }
          if (LAT) __builtin_amdgcn_sched_barrier(0);
        }
      };
#pragma unroll 1
      for (int a = a0; a < nqb; a += 2) {
        const bool two = a + 1 < nqb;
        f32x4 sc[2], dc[2];
        sdp(a, two, sc, dc);
        float P[8], dS[8];
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const int qb = a + half;
#pragma unroll
          for (int i = 0; i < 4; ++i) P[4 * half + i] = dS[4 * half + i] = 0.f;
          if (half == 1 && !two) continue;
          const int q0 = 16 * qb + 4 * g;
          const f32x4 L = *reinterpret_cast<const f32x4*>(lse2 + q0);
          const f32x4 D = *reinterpret_cast<const f32x4*>(dlt + q0);
          char* blk = dss + 1024 * (blk0 + qb - a0);
          // the causal mask only on blocks the diagonal crosses (uniform): elsewhere every key of the block
          // precedes every query (padded queries have lse +inf, so P = 0 without it; the key block holding
          // keys past I is always on the diagonal)
          if (16 * kb + 15 > q_off + 16 * qb) {
            const i32x4 Qp = *reinterpret_cast<const i32x4*>(qps + q0);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float e = __builtin_amdgcn_exp2f(fmaf(sc[half][i], cS, -L[i]));
              const float pv = krow <= Qp[i] ? e : 0.f;
              const float ds = pv * (NP == 2 ? fmaf(dc[half][i], cdp, -D[i]) : dc[half][i] - D[i]) * dsc;
              P[4 * half + i] = pv;
              dS[4 * half + i] = ds;
              *reinterpret_cast<float*>(blk + dsw[i]) = ds;
              if constexpr (NP == 2) mdsw = fmaxf(mdsw, fabsf(ds));
            }
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float pv = __builtin_amdgcn_exp2f(fmaf(sc[half][i], cS, -L[i]));
              const float ds = pv * (NP == 2 ? fmaf(dc[half][i], cdp, -D[i]) : dc[half][i] - D[i]) * dsc;
              P[4 * half + i] = pv;
              dS[4 * half + i] = ds;
              *reinterpret_cast<float*>(blk + dsw[i]) = ds;
              if constexpr (NP == 2) mdsw = fmaxf(mdsw, fabsf(ds));
            }
          }
        }
        u32x4 pp[NP], sp[NP];
        splitN<NP>(P, 1.f, pp);
        splitN<NP>(dS, sds, sp);
        const int ra = 16 * RBY * a, rb = two ? ra + 16 * RBY : ra;
        u32x4 fa[2][NP], fb[2][NP];
        tr_atN<NP>(fa[0], smem + ra + otbase[0], smem + rb + otbase[0], PB);
        tr_atN<NP>(fb[0], smem + ra + tbase[0], smem + rb + tbase[0], PB);
#pragma unroll
        for (int m = 0; m < NM; ++m) {
          if (m + 1 < NM) {                                           // next dim tile's fragments in flight
            tr_atN<NP>(fa[(m + 1) & 1], smem + ra + otbase[m + 1], smem + rb + otbase[m + 1], PB);
            tr_atN<NP>(fb[(m + 1) & 1], smem + ra + tbase[m + 1], smem + rb + tbase[m + 1], PB);
          }
          dv[m] = mmaN<NP>(fa[m & 1], pp, dv[m]);                     // dV^T += dO^T P
          dk[m] = mmaN<NP>(fb[m & 1], sp, dk[m]);                     // dK^T += Q^T dS
          if (LAT) __builtin_amdgcn_sched_barrier(0);
        }
      }
      float rk = 0.f, rv = 0.f;                                      // this lane's max |dK|, |dV| (rowmax)
      if (krow < I) {
        const float uk = NP == 2 ? 1.f / (sq * sds) : 1.f, uv = NP == 2 ? 1.f / (so * 16384.f) : 1.f;
#pragma unroll
        for (int m = 0; m < NM; ++m) {
          *reinterpret_cast<f32x4*>(dKg + (int64_t)krow * p.ld + 16 * m + 4 * g) = dk[m] * uk;
          *reinterpret_cast<f32x4*>(dVg + (int64_t)krow * p.ld + 16 * m + 4 * g) = dv[m] * uv;
          rk = amax4(rk, dk[m] * uk);
          rv = amax4(rv, dv[m] * uv);
        }
        am = fmaxf(am, fmaxf(rk, rv));
      }
      if (p.rowmax) {                                // (uniform) [row][q / k / v part][head] maxima of dQKV rows
        rk = group_max(rk);
        rv = group_max(rv);
        if (krow < I && g == 0) {
          float* rr = p.rowmax + ((int64_t)(s / p.H) * I + krow) * 3 * p.H + (s % p.H);
          rr[p.H] = rk;
          rr[2 * p.H] = rv;
        }
      }
      kb = kbn;
    }
    // K image for phase 2, in the Q planes' space: each key-block owner stores the K planes it kept (rows past
    // I hold row I - 1, times dS = 0) — no re-read or re-split of K
    SLICE_STAMP(1, it, 2);
    // G2: the K rows for the phase-2 image, issued before the barrier (in flight while the other waves finish)
    constexpr int SRK = (KR * CPR + NTH - 1) / NTH;
    float kim[G2 ? SRK : 1][8];
    if constexpr (G2) {
#pragma unroll
      for (int r = 0; r < SRK; ++r) {
        const int task = threadIdx.x + r * NTH, j = min(task / CPR, I - 1), c = task % CPR;
        load8(kim[r], Kg + (int64_t)j * p.ld + 8 * c);
      }
    }
    if constexpr (NP == 2) {
      mdsw = wave_maxf(mdsw);
      if (lane == 0) {                             // (the staging maxima were read before phase 1)
        red[wave] = mkw;
        red[8 + wave] = mdsw;
      }
    }
    __syncthreads();                               // dS store complete, Q planes no longer read
    SLICE_STAMP(1, it, 3);
    float sks = 1.f, sdss = 1.f;                   // NP = 2: phase 2's K image and dS scales (slice-wide)
    if constexpr (NP == 2) {
      float mk = 0.f, md = 0.f;
#pragma unroll
      for (int w = 0; w < NWV; ++w) {
        mk = fmaxf(mk, red[w]);
        md = fmaxf(md, red[8 + w]);
      }
      sks = pow2scale(mk);
      sdss = pow2scale(md);
    }
    if constexpr (G2) {                            // the whole workgroup: K rows -> the image at the slice scale
#pragma unroll
      for (int r = 0; r < SRK; ++r) {
        const int task = threadIdx.x + r * NTH, j = task / CPR, c = task % CPR;
        if (task < IP * CPR) store_planesN<NP>(qimg, KPB, poff<HD>(j, c), kim[r], sks);
      }
    }
#pragma unroll
    for (int k2 = 0; k2 < (G2 ? 0 : KEEP); ++k2) {
      const int kb = sched_item(srow1, k2);
      if (kb >= 0) {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          u32x4 kp[NP];
          if constexpr (NP == 3) {
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) kp[pl] = keep[k2][t][pl];
          } else {
            splitN<2>(keepf[k2][t], sks, kp);
          }
#pragma unroll
          for (int pl = 0; pl < NP; ++pl)
            *reinterpret_cast<u32x4*>(qimg + pl * KPB + poff<HD>(16 * kb + li, 4 * t + g)) = kp[pl];
        }
      }
    }
    __syncthreads();
    SLICE_STAMP(1, it, 4);
    // the next slice's Q / dO / O rows: issued before phase 2 at head_dim 64, after it at 32.  Issuing them (~108
    // KiB per CU at head_dim 64) stalls the wave for about 7k cycles wherever they go — at the start of phase 1
    // measured the same, streamed a piece per phase-1 / phase-2 step slower (the waits for the next key block's
    // K / V then drain them too)
    constexpr bool EARLY = HD == 64;
    if (!G2 && EARLY && s + (int)gridDim.x < nslices) prefetch(s + gridDim.x);

    // ---- phase 2: query-block owners, dQ^T = K^T dS^T
#pragma unroll 1
    for (int slot = 0; slot < 8; ++slot) {
      const int idx = sched_item(srow2, slot);
      if (idx < 0) break;
      const int qb = nqb - 1 - idx;
      const int kbl = (q_off + min(16 * qb + 15, K - 1)) >> 4;
      f32x4 dq[NM];
#pragma unroll
      for (int m = 0; m < NM; ++m) dq[m] = f32x4{0.f, 0.f, 0.f, 0.f};
      // two independent accumulator sets over alternate key-block pairs (the pairs' dS reads, splits and
      // transposed reads overlap), added at the end
      f32x4 dq2[NM];
#pragma unroll
      for (int m = 0; m < NM; ++m) dq2[m] = f32x4{0.f, 0.f, 0.f, 0.f};
      auto ldds = [&](int k2, f32x4& x0, f32x4& x1) {
        x0 = *reinterpret_cast<const f32x4*>(dss + 1024 * (tab[SLICE_TABN + k2] + qb - tab[k2]) + dsr);
        x1 = f32x4{0.f, 0.f, 0.f, 0.f};
        if (k2 + 1 <= kbl)
          x1 = *reinterpret_cast<const f32x4*>(dss + 1024 * (tab[SLICE_TABN + 1 + k2] + qb - tab[k2 + 1]) + dsr);
      };
      auto stepx = [&](int k2, f32x4 x0, f32x4 x1, f32x4 (&acc)[NM]) {
        const bool two = k2 + 1 <= kbl;
        float v[8];
        const int ra = 16 * RBY * k2, rb = two ? ra + 16 * RBY : ra;
        u32x4 fa[2][NP];
        tr_atN<NP>(fa[0], smem + ra + tbase[0], smem + rb + tbase[0], KPB);   // in flight during the split
#pragma unroll
        for (int i = 0; i < 4; ++i) { v[i] = x0[i]; v[4 + i] = x1[i]; }
        u32x4 bp[NP];
        splitN<NP>(v, sdss, bp);
#pragma unroll
        for (int m = 0; m < NM; ++m) {
          if (m + 1 < NM) tr_atN<NP>(fa[(m + 1) & 1], smem + ra + tbase[m + 1], smem + rb + tbase[m + 1], KPB);
          acc[m] = mmaN<NP>(fa[m & 1], bp, acc[m]);
          if (LAT) __builtin_amdgcn_sched_barrier(0);
        }
      };
      if constexpr (G2) {                          // global dS: each pair's reads issued two pairs ahead
        f32x4 xa0, xa1, xb0, xb1;
        ldds(0, xa0, xa1);
        if (2 <= kbl) ldds(2, xb0, xb1);
#pragma unroll 1
        for (int k2 = 0; k2 <= kbl; k2 += 4) {
          const f32x4 c0 = xa0, c1 = xa1;
          if (k2 + 4 <= kbl) ldds(k2 + 4, xa0, xa1);
          stepx(k2, c0, c1, dq);
          if (k2 + 2 <= kbl) {
            const f32x4 d0 = xb0, d1 = xb1;
            if (k2 + 6 <= kbl) ldds(k2 + 6, xb0, xb1);
            stepx(k2 + 2, d0, d1, dq2);
          }
        }
      } else {
#pragma unroll 1
        for (int k2 = 0; k2 <= kbl; k2 += 4) {
          f32x4 x0, x1;
          ldds(k2, x0, x1);
          stepx(k2, x0, x1, dq);
          if (k2 + 2 <= kbl) {
            ldds(k2 + 2, x0, x1);
            stepx(k2 + 2, x0, x1, dq2);
          }
        }
      }
      const float uq = NP == 2 ? 1.f / (sks * sdss) : 1.f;
#pragma unroll
      for (int m = 0; m < NM; ++m) dq[m] = (dq[m] + dq2[m]) * uq;
      const int j = 16 * qb + li;
      float rq = 0.f;
      if (j < K) {
        float* drow = dQg + (int64_t)(q_off + j) * p.ld + 4 * g;
#pragma unroll
        for (int m = 0; m < NM; ++m) {
          *reinterpret_cast<f32x4*>(drow + 16 * m) = dq[m];
          rq = amax4(rq, dq[m]);
        }
        am = fmaxf(am, rq);
      }
      if (p.rowmax) {                                // (uniform) the dQ part of the row's maxima
        rq = group_max(rq);
        if (j < K && g == 0) p.rowmax[((int64_t)(s / p.H) * I + q_off + j) * 3 * p.H + (s % p.H)] = rq;
      }
    }
    SLICE_STAMP(1, it, 5);
    if (!G2 && !EARLY && s + (int)gridDim.x < nslices) prefetch(s + gridDim.x);
    __syncthreads();                               // LDS is restaged next slice
    SLICE_STAMP(1, it, 6);
  }
  if (p.amax) amax_flush(p.amax, am);               // |dQKV| bound of the Wqkv weight gradient (fp16 pair)
}

static int rmax(int hd) { return hd == 64 ? RMAX<64>() : RMAX<32>(); }
size_t fwd_lds(int I, int hd, int np = 3) { return (size_t)4 * np * rmax(hd) * hd + 4 * (size_t)rmax(hd) + 64; }

// causal 16 x 16 block pairs of the tail-query backward
int bwd_pairs(int I, int K) {
  const int nkb = (I + 15) / 16, nqb = (K + 15) / 16, q_off = I - K;
  int n = 0;
  for (int kb = 0; kb < nkb; ++kb) n += nqb - tail_qf(kb, q_off, nqb);
  return n;
}

size_t bwd_lds(int I, int K, int hd, int np = 3, bool g2 = false, int rq = 0) {
  const size_t r = rq ? rq : rmax(hd);
  return (size_t)4 * np * r * hd + 12 * r + 8 * SLICE_TABN + 128 + (g2 ? 0 : 1024 * (size_t)bwd_pairs(I, K));
}

static int device_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        n > 0)
      cus = n;
    else
      cus = 256;
    (void)hipGetLastError();
  }
  return cus;
}

// persistent grid: the workgroups that are co-resident (occupancy query, cached per kernel and LDS size),
// at most one per slice
static unsigned persistent_grid(const void* kernel, int threads, size_t lds, int64_t slices) {
  static std::mutex mu;
  static int cus = 0;
  static const void* last_k[8] = {};
  static size_t last_lds[8] = {};
  static int last_n[8] = {};
  std::lock_guard<std::mutex> lock(mu);
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  int per = 0;
  for (int i = 0; i < 8; ++i)
    if (last_k[i] == kernel && last_lds[i] == lds) per = last_n[i];
  if (!per) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, threads, lds) != hipSuccess || per <= 0) per = 1;
    (void)hipGetLastError();
    for (int i = 0; i < 8; ++i)
      if (!last_k[i]) { last_k[i] = kernel; last_lds[i] = lds; last_n[i] = per; break; }
  }
  return (unsigned)std::min<int64_t>(slices, (int64_t)per * cus);
}

// LPT over the SIMDs: waves w and w + 4 share SIMD w & 3 (a workgroup's waves go to the SIMDs
// cyclically, MI355X_MICROARCH.md §LDS), so each item (heaviest first) goes to the least-loaded SIMD,
// then to its less-loaded wave.  Returns false if a wave would get more than 8 items.
static bool lpt(int n, const int* load, int nwv, int8_t (&out)[8][8], int cap = 8) {
  std::memset(out, -1, sizeof out);
  int sl[4] = {0, 0, 0, 0}, wl[8] = {0, 0, 0, 0, 0, 0, 0, 0}, cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < n; ++i) {
    int w = -1;
    for (int k = 0; k < 4; ++k) {                  // least-loaded SIMD with a wave under the cap
      int c = -1;
      for (int v = k; v < nwv; v += 4)
        if (cnt[v] < cap && (c < 0 || wl[v] < wl[c])) c = v;
      if (c >= 0 && (w < 0 || sl[k] < sl[w & 3])) w = c;
    }
    if (w < 0) return false;
    sl[w & 3] += load[i];
    wl[w] += load[i];
    out[w][cnt[w]++] = (int8_t)i;
  }
  return true;
}

// forward: query blocks (heaviest first: the last); backward: key blocks (heaviest first: the first) in
// query steps of two blocks, then query blocks in steps of two key blocks; costs in MFMA groups
static bool make_schedule(SliceArgs& p, int hd, int nwv, int kcap) {
  const int I = p.I, K = p.K, q_off = I - K, nkb = (I + 15) / 16, nqb = (K + 15) / 16;
  const int NT = hd / 32, NM = hd / 16;
  if (nkb > SLICE_TABN) return false;
  int load[SLICE_TABN];
  for (int idx = 0; idx < nqb; ++idx) {
    const int kl = (q_off + std::min(16 * (nqb - 1 - idx) + 15, K - 1)) >> 4;
    load[idx] = NT * (kl + 1) + NM * (kl / 2 + 1);
  }
  if (!lpt(nqb, load, nwv, p.sched[0])) return false;
  int base = 0;
  for (int kb = 0; kb < nkb; ++kb) {
    const int f = tail_qf(kb, q_off, nqb);
    load[kb] = (nqb - f + 1) >> 1;
    p.qf[kb] = (int8_t)f;
    p.bbase[kb] = (int16_t)base;
    base += nqb - f;
  }
  if (!lpt(nkb, load, nwv, p.sched[1], kcap)) return false;   // (one workgroup per CU: the backward keeps K per slot)
  for (int idx = 0; idx < nqb; ++idx) load[idx] = (((q_off + std::min(16 * (nqb - 1 - idx) + 15, K - 1)) >> 4) + 2) >> 1;
  return lpt(nqb, load, nwv, p.sched[2]);
}

// Arithmetic (measured at B 4096 H 4 I 140, round 5): the scaled fp16 pair (NP 2) everywhere except the head_dim-32
// forward, where the three-plane bf16 split (NP 3) stays faster (286-302 vs 318-330 us: the per-slice K / V scale
// reduction costs more than the halved MFMAs save in that short, non-persistent kernel).  hd 64: forward 605-617 ->
// 550-561 us, backward 1,616-1,629 -> 1,515-1,523; hd 32 backward 936-950 -> 871-901.
constexpr int fwd_planes(int hd) { return hd == 64 ? 2 : 3; }
constexpr int BWD_PLANES = 2;

// waves per workgroup (measured, B 4096 H 4 I 140): forward 8 (hd 32: 4 waves / SIMD at 128 VGPRs); backward hd 32
// 8 (4 waves: 1,136-1,160 vs 928-965 us; again 1,066-1,093 vs 919-948 with the kept K planes and fenced
// fragment reads), hd 64 4 (one wave per SIMD with up to 512 registers; 8 waves spill at
// the 256-register limit: 1,971-2,095 vs 1,688-1,782 us)
#ifndef OT_SLICE_BWD32_WAVES
#define OT_SLICE_BWD32_WAVES 8
#endif
constexpr int FWD_WAVES = 8, BWD_WAVES32 = OT_SLICE_BWD32_WAVES, BWD_WAVES64 = 4;

template <typename F>
static void raise_lds_limit(F* k) {
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
}

// Backward forms.  Past I = 144 at head_dim 64 (C3's first two layers: I 524 / K 262, I 262 / K 131) the key
// side outgrows the Q planes' rows: the K / V blocks come from global per key block anyway, so only phase 2's K
// image needs room — it takes the Q and dO planes' space together (KR = 2 RQ rows), and dS goes to the workspace.
//   MID:  K <= 144, I <= 288 — the two-workgroup kernel (4 waves, 75.9 KiB of LDS) with a 288-row K image;
//   LONG: K <= 272, I <= 544 — one workgroup of 8 waves per CU (Q / dO planes of 272 rows: 139.6 KiB).
// (The MID shapes on the LONG form measured 7-8% slower: I 262 / K 131, B 2048 H 4 1,620-1,628 vs 1,503-1,552 us.)
enum BwdForm { BWD_NONE, BWD_32, BWD_64, BWD_MID, BWD_LONG };
constexpr int RQ_LONG = 272, BWD_WAVES_LONG = 8;
static BwdForm bwd_form(int I, int K, int hd) {
  if (K <= 0 || K > I) return BWD_NONE;
  if (hd == 32) return I <= RMAX<32>() && bwd_lds(I, K, 32, BWD_PLANES) <= (size_t)LDS_MAX ? BWD_32 : BWD_NONE;
  if (hd != 64) return BWD_NONE;
  if (I <= RMAX<64>()) return bwd_lds(I, K, 64, BWD_PLANES) <= (size_t)LDS_MAX ? BWD_64 : BWD_NONE;
  if (K <= RMAX<64>() && I <= 2 * RMAX<64>()) return BWD_MID;
  if (K <= RQ_LONG && I <= 2 * RQ_LONG && (I + 15) / 16 <= SLICE_TABN) return BWD_LONG;
  return BWD_NONE;
}

}  // namespace slice

bool attn_slice_fwd_supported(int I, int K, int head_dim) {
  return (head_dim == 32 || head_dim == 64) && I <= slice::rmax(head_dim) && K > 0 && K <= I &&
         slice::fwd_lds(I, head_dim, head_dim == 64 ? slice::fwd_planes(64) : slice::fwd_planes(32)) <=
             (size_t)slice::LDS_MAX;
}

bool attn_slice_bwd_supported(int I, int K, int head_dim, bool selected) {
  return !selected && slice::bwd_form(I, K, head_dim) != slice::BWD_NONE;
}

int attn_slice_fwd(const float* qkv, int64_t ld, int B, int H, int I, int K, const int32_t* qpos, int head_dim,
                   float* out, float* lse, hipStream_t stream, float* amax, float* rowmax) {
  using namespace slice;
  using KF = void (*)(SliceArgs);
  constexpr int P32 = fwd_planes(32), P64 = fwd_planes(64);
  static const KF table[2][2] = {
      {attn_fwd_slice_kernel<32, FWD_WAVES, false, P32>, attn_fwd_slice_kernel<32, FWD_WAVES, true, P32>},
      {attn_fwd_slice_kernel<64, FWD_WAVES, false, P64>, attn_fwd_slice_kernel<64, FWD_WAVES, true, P64>}};
  static std::once_flag once;
  std::call_once(once, [] {
    for (int a = 0; a < 2; ++a)
      for (int b = 0; b < 2; ++b) raise_lds_limit(table[a][b]);
    (void)hipGetLastError();
  });
  SliceArgs p{qkv, ld, H * head_dim, nullptr, nullptr, nullptr, out, lse, nullptr, B, H, I, K,
              1.f / sqrtf((float)head_dim), qpos};
  p.amax = amax;
  p.rowmax = rowmax;
  const size_t lds = fwd_lds(I, head_dim, head_dim == 64 ? P64 : P32);
  const int nw = FWD_WAVES;
  OT_REQUIRE(make_schedule(p, head_dim, nw, 8), "ot_attn_fwd(slice): schedule");
  const KF k = table[head_dim == 64][qpos != nullptr];
  const unsigned slices = (unsigned)((int64_t)B * H);
  const dim3 grid(slices), block(64 * nw);
  hipLaunchKernelGGL(k, grid, block, lds, stream, p);
  OT_LAUNCH_CHECK("ot_attn_fwd(slice)");
  return OT_OK;
}

// two workgroups per CU (global dS scratch) at head_dim 64.  Measured at B 4096 H 4 I 140 (round 5): hd 64 1,523 ->
// 1,385 us (with the K image's loads issued before the phase-1 barrier; the fenced one-item-ahead fragment reads
// (LAT) cost 40-60 us at two waves per SIMD; half a slice of start skew between the two workgroups changed nothing);
// hd 32 as two workgroups of 4 waves 868-879 us against 816-821 for one of 8 (kept)
constexpr bool bwd_g2(int hd) { return hd == 64; }

// workgroups per CU of the workspace-dS forms (0: dS in LDS only)
static int bwd_ws_wpc(slice::BwdForm f) {
  return f == slice::BWD_64 || f == slice::BWD_MID ? 2 : f == slice::BWD_LONG ? 1 : 0;
}

size_t attn_slice_bwd_ws_bytes(int B, int H, int I, int K, int head_dim) {
  using namespace slice;
  const int wpc = bwd_ws_wpc(bwd_form(I, K, head_dim));
  if (!wpc) return 0;
  const int64_t grid = std::min<int64_t>((int64_t)B * H, wpc * (int64_t)device_cus());
  return (size_t)grid * 1024 * bwd_pairs(I, K);
}

// the long forms keep dS only in the workspace: below one workgroup's share per CU (e.g. ot_attn_bwd's lse / delta
// workspace) the caller takes the per-pair f32 kernels instead of a starved grid
size_t attn_slice_bwd_min_ws(int B, int H, int I, int K, int head_dim) {
  using namespace slice;
  const BwdForm f = bwd_form(I, K, head_dim);
  if (f != BWD_MID && f != BWD_LONG) return 0;
  return (size_t)1024 * bwd_pairs(I, K) * (size_t)std::min<int64_t>((int64_t)B * H, device_cus());
}

int attn_slice_bwd(const float* qkv, int64_t ld, const float* out, const float* dout, const float* lse, int B, int H,
                   int I, int K, int head_dim, float* dqkv, float* ws, size_t ws_bytes, hipStream_t stream,
                   float* amax, float* rowmax) {
  using namespace slice;
  using KF = void (*)(SliceArgs);
  static const KF k32 = attn_bwd_slice_kernel<32, BWD_WAVES32, BWD_PLANES>,
                  k64 = attn_bwd_slice_kernel<64, BWD_WAVES64, BWD_PLANES>,
                  k64g = attn_bwd_slice_kernel<64, BWD_WAVES64, BWD_PLANES, false, true>,
                  kmid = attn_bwd_slice_kernel<64, BWD_WAVES64, BWD_PLANES, false, true, RMAX<64>(), 2 * RMAX<64>()>,
                  klong = attn_bwd_slice_kernel<64, BWD_WAVES_LONG, BWD_PLANES, false, true, RQ_LONG, 2 * RQ_LONG>;
  static std::once_flag once;
  std::call_once(once, [] {
    for (KF k : {k32, k64, k64g, kmid, klong}) raise_lds_limit(k);
    (void)hipGetLastError();
  });
  const BwdForm form = bwd_form(I, K, head_dim);
  OT_REQUIRE(form != BWD_NONE, "ot_attn_bwd(slice): I %d K %d head_dim %d unsupported", I, K, head_dim);
  SliceArgs p{qkv, ld, H * head_dim, out, dout, lse, nullptr, nullptr, dqkv, B, H, I, K,
              1.f / sqrtf((float)head_dim), nullptr};
  p.amax = amax;
  p.rowmax = rowmax;
  const size_t per_wg = (size_t)1024 * bwd_pairs(I, K);
  const bool wsok = ws && ws_bytes >= per_wg;
  const bool g2 = form == BWD_MID || form == BWD_LONG || (form == BWD_64 && bwd_g2(64) && wsok);
  OT_REQUIRE(!g2 || wsok, "ot_attn_bwd(slice): I %d K %d needs %zu bytes of workspace", I, K, per_wg);
  const int nw = form == BWD_32 ? BWD_WAVES32 : form == BWD_LONG ? BWD_WAVES_LONG : BWD_WAVES64;
  OT_REQUIRE(make_schedule(p, head_dim, nw, g2 ? 8 : keep_slots(head_dim, nw)), "ot_attn_bwd(slice): schedule");
  const KF k = form == BWD_32 ? k32 : form == BWD_MID ? kmid : form == BWD_LONG ? klong : g2 ? k64g : k64;
  const size_t lds = bwd_lds(I, K, head_dim, BWD_PLANES, g2, form == BWD_LONG ? RQ_LONG : 0);
  unsigned g = persistent_grid((const void*)k, 64 * nw, lds, (int64_t)B * H);
  if (g2) {
    g = (unsigned)std::min<size_t>(g, ws_bytes / per_wg);      // each workgroup owns per_wg bytes of scratch
    p.dsws = ws;
    p.ds_floats = (int)(per_wg / sizeof(float));
  }
  const dim3 grid(g), block(64 * nw);
  hipLaunchKernelGGL(k, grid, block, lds, stream, p);
  OT_LAUNCH_CHECK("ot_attn_bwd(slice)");
  return OT_OK;
}

}  // namespace ot

#if OT_SLICE_STAMPS
extern "C" int ot_slice_stamps_read(unsigned long long* host, size_t bytes) {
  if (bytes < sizeof(ot::slice::g_slice_stamps)) return -1;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(ot::slice::g_slice_stamps), sizeof(ot::slice::g_slice_stamps)) == hipSuccess ? 0 : -2;
}
#endif
