// Short-sequence causal attention (I <= 192 keys) on split-bf16 MFMA, one workgroup per (sample, head)
// slice.  Replaces model.py:100-114 (QK^T / sqrt(hd), band_part causal mask, softmax, PV) and its
// gradient for the f32-accurate mode (OT_MATMUL_SPLIT_BF16) at head_dim 32 / 64.
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

// Work schedule inside a workgroup of NWV waves (4 or 8).  Waves w and w + 4 share SIMD w & 3 (a
// workgroup's waves go to the SIMDs cyclically, MI355X_MICROARCH.md §LDS), so items (heaviest first) go
// to the least-loaded SIMD, then to its less-loaded wave (LPT).  Every wave runs the same uniform
// arithmetic; the result is the item index of `slot` of wave w, or -1.
template <int NWV, typename F>
__device__ __forceinline__ int lpt_pick(int slot, int w, int n, F load) {
  int s0 = 0, s1 = 0, s2 = 0, s3 = 0, w0 = 0, w1 = 0, w2 = 0, w3 = 0, w4 = 0, w5 = 0, w6 = 0, w7 = 0;
  int cnt = 0;
  for (int i = 0; i < n; ++i) {
    const int L = load(i);
    int s = 0, m = s0;
    if (s1 < m) { s = 1; m = s1; }
    if (s2 < m) { s = 2; m = s2; }
    if (s3 < m) { s = 3; m = s3; }
    int ww = s;
    if (NWV == 8) {
      const int a = s == 0 ? w0 : s == 1 ? w1 : s == 2 ? w2 : w3;
      const int b = s == 0 ? w4 : s == 1 ? w5 : s == 2 ? w6 : w7;
      ww = a <= b ? s : s + 4;
    }
    s0 += s == 0 ? L : 0; s1 += s == 1 ? L : 0; s2 += s == 2 ? L : 0; s3 += s == 3 ? L : 0;
    w0 += ww == 0 ? L : 0; w1 += ww == 1 ? L : 0; w2 += ww == 2 ? L : 0; w3 += ww == 3 ? L : 0;
    w4 += ww == 4 ? L : 0; w5 += ww == 5 ? L : 0; w6 += ww == 6 ? L : 0; w7 += ww == 7 ? L : 0;
    if (ww == w) {
      if (cnt == slot) return i;
      ++cnt;
    }
  }
  return -1;
}

// tail queries: first 16-query block whose last query sees key block kb
__device__ __forceinline__ int tail_qf(int kb, int q_off, int K, int nqb) {
  int f = 0;
  while (f < nqb && q_off + min(16 * f + 15, K - 1) < 16 * kb) ++f;
  return f;
}

// ------------------------------------------------------------------------------------------
// Forward.  The slice's K and V planes are staged in LDS ([IP][HD] x 3 each); each wave takes whole
// 16-query blocks (LPT over the SIMDs, heaviest first).  Per query block the wave holds Q (pre-scaled by
// log2(e)/sqrt(hd), split) as the B operand of S^T = K Q^T (query on the lane) and computes S^T for
// every visible key block at once (<= 12 x 4 registers), so the softmax is exact in one pass (row max
// and sum over the 4 lane groups by shuffles, no rescaling); O^T = V^T P^T takes P^T from the S^T
// registers and V^T by transposed reads.  Every global load is issued ahead of its use: the staging
// rounds all at once, each wave's first Q block before the staging barrier, the next one while the
// current block computes.
template <int HD, int NWV>
__global__ __launch_bounds__(64 * NWV, 1) void attn_fwd_slice_kernel(SliceArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NT = HD / 32, NM = HD / 16, CPR = HD / 8, NTH = 64 * NWV;
  constexpr int SR = (MAXKB * 16 * CPR + NTH - 1) / NTH;          // staging rounds (upper bound)
  const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // uniform: the schedule runs on SALU
  const int pair = blockIdx.x, b = pair / p.H, h = pair % p.H;
  const int I = p.I, K = p.K, q_off = I - K;
  const int nkb = (I + 15) >> 4, nqb = (K + 15) >> 4, IP = nkb * 16;
  const int PB = IP * HD * 2;
  char* kimg = smem;
  char* vimg = smem + 3 * PB;
  const int64_t tok0 = (int64_t)b * I;
  const float* Qg = p.qkv + tok0 * p.ld + h * HD;
  const float* Kg = Qg + p.d;
  const float* Vg = Qg + 2 * p.d;
  const int32_t* qsel = p.qpos ? p.qpos + (int64_t)b * K : nullptr;
  auto qpos_of = [&](int j) { return qsel ? qsel[j] : q_off + j; };
  // query block of item idx (heaviest first) and its last visible key block
  auto kbl_of = [&](int qb) { return qpos_of(min(16 * qb + 15, K - 1)) >> 4; };
  auto load_of = [&](int idx) { const int kl = kbl_of(nqb - 1 - idx); return NT * (kl + 1) + NM * (kl / 2 + 1); };

  float kr[SR][8], vr[SR][8];
#pragma unroll
  for (int r = 0; r < SR; ++r) {
    const int task = threadIdx.x + r * NTH, row = task / CPR, c = task % CPR;
    if (task < IP * CPR && row < I) {
      load8(kr[r], Kg + (int64_t)row * p.ld + 8 * c);
      load8(vr[r], Vg + (int64_t)row * p.ld + 8 * c);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) kr[r][e] = vr[r][e] = 0.f;
    }
  }
  float qr[NT][8];
  int idx = lpt_pick<NWV>(0, wave, nqb, load_of);
  auto load_q = [&](int ix) {
    const int j = 16 * (nqb - 1 - ix) + li;
    const int qp = qpos_of(j < K ? j : K - 1);
#pragma unroll
    for (int t = 0; t < NT; ++t) load8(qr[t], Qg + (int64_t)qp * p.ld + 32 * t + 8 * g);
  };
  if (idx >= 0) load_q(idx);
#pragma unroll
  for (int r = 0; r < SR; ++r) {
    const int task = threadIdx.x + r * NTH, row = task / CPR, c = task % CPR;
    if (task < IP * CPR) {
      const int o = poff<HD>(row, c);
      store_planes(kimg, PB, o, kr[r]);
      store_planes(vimg, PB, o, vr[r]);
    }
  }
  __syncthreads();
  const float qscale = p.scale * L2E;
#pragma unroll 1
  for (int slot = 0; idx >= 0; ++slot) {
    const int qb = nqb - 1 - idx;
    const int j = 16 * qb + li;                                      // this lane's query
    const int qpos = qpos_of(j < K ? j : K - 1);
    const int kbl = kbl_of(qb);
    u32x4 qp[NT][3];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
#pragma unroll
      for (int e = 0; e < 8; ++e) qr[t][e] *= qscale;
      split8(qr[t], qp[t]);
    }
    idx = lpt_pick<NWV>(slot + 1, wave, nqb, load_of);
    if (idx >= 0) load_q(idx);                                       // next block's Q, in flight meanwhile
    f32x4 s[MAXKB];
    float mx = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < MAXKB; ++kb) {
      s[kb] = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
      if (kb > kbl) continue;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        u32x4 fk[3];
        row_frag<HD>(fk, kimg, PB, 16 * kb + li, t, g);
        acc = mma6(fk, qp[t], acc);                                   // S^T: row = key, col = query
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        acc[i] = (16 * kb + 4 * g + i <= qpos) ? acc[i] : -INFINITY;
        mx = fmaxf(mx, acc[i]);
      }
      s[kb] = acc;
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float l = 0.f;
#pragma unroll
    for (int kb = 0; kb < MAXKB; ++kb) {
      if (kb > kbl) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float e = __builtin_amdgcn_exp2f(s[kb][i] - mx);
        s[kb][i] = e;
        l += e;
      }
    }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
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
        v[i] = s[kb][i];
        v[4 + i] = two ? s[kb + 1][i] : 0.f;
      }
      u32x4 pp[3];
      split8(v, pp);
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        u32x4 fa[3];
        tr_frag<HD>(fa, vimg, PB, 16 * kb, two ? 16 * kb + 16 : 16 * kb, m, lane);
        o[m] = mma6(fa, pp, o[m]);                                    // O^T += V^T P^T
      }
    }
    if (j < K) {
      const float inv = 1.f / l;
      float* orow = p.out + ((int64_t)b * K + j) * p.d + h * HD + 4 * g;
#pragma unroll
      for (int m = 0; m < NM; ++m) *reinterpret_cast<f32x4*>(orow + 16 * m) = o[m] * inv;
      if (g == 0) p.lse[(int64_t)pair * K + j] = mx * LN2 + __logf(l);
    }
  }
}

// ------------------------------------------------------------------------------------------
// Backward (tail queries).  LDS: Q planes [IP][HD] x 3 (phase 2: the K image), dO planes [KP][HD] x 3,
// lse (log2 units, +inf padding), delta = rowsum(dO o O) (formed here from one read of O), query
// positions, per key block its first visible query block and dS-store base, then the dS store: one
// 1 KiB [16 query][16 key] f32 block per causal block pair.
//   phase 1, key blocks (LPT over the SIMDs), query steps of two 16-row blocks (a, a+1):
//     S = Q K^T, dP = dO V^T          A = Q / dO rows (ds_read_b128), B = K^T / V^T (registers)
//     P = exp2(S log2e/sqrt(hd) - lse), dS = P (dP - delta) / sqrt(hd)     (key on the lane)
//     dV^T += dO^T P, dK^T += Q^T dS  A = dO^T / Q^T (transposed reads), B = P / dS (registers)
//     dS -> store
//   phase 2, query blocks: dQ^T = K^T dS^T over the visible key blocks, two per step (K image re-read
//   from global — L2-warm — into the Q planes' space).
// Global loads are issued ahead of use: the staging rounds and the first key block's K / V before the
// staging barrier, the next key block's during the current one, the K image's before the phase barrier.
template <int HD, int NWV>
__global__ __launch_bounds__(64 * NWV, 1) void attn_bwd_slice_kernel(SliceArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NT = HD / 32, NM = HD / 16, CPR = HD / 8, NTH = 64 * NWV;
  constexpr int SR = (MAXKB * 16 * CPR + NTH - 1) / NTH;
  const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // uniform: the schedule runs on SALU
  const int pair = blockIdx.x, b = pair / p.H, h = pair % p.H;
  const int I = p.I, K = p.K, q_off = I - K;
  const int nkb = (I + 15) >> 4, nqb = (K + 15) >> 4, IP = nkb * 16, KP = nqb * 16;
  const int PBQ = IP * HD * 2, PBO = KP * HD * 2;
  char* qimg = smem;
  char* oimg = qimg + 3 * PBQ;
  float* lse2 = reinterpret_cast<float*>(oimg + 3 * PBO);
  float* dlt = lse2 + KP;
  int* qps = reinterpret_cast<int*>(dlt + KP);
  int* qfb = qps + KP;
  int* bbase = qfb + MAXKB;
  char* dss = reinterpret_cast<char*>(bbase + MAXKB);
  const int64_t tok0 = (int64_t)b * I;
  const int hoff = h * HD;
  const float* Qg = p.qkv + tok0 * p.ld + hoff;
  const float* Kg = Qg + p.d;
  const float* Vg = Qg + 2 * p.d;
  const float* dOg = p.dout + (int64_t)b * K * p.d + hoff;
  const float* Og = p.o + (int64_t)b * K * p.d + hoff;
  float* dQg = p.dqkv + tok0 * p.ld + hoff;
  float* dKg = dQg + p.d;
  float* dVg = dQg + 2 * p.d;
  auto kload = [&](int kb) { return (nqb - tail_qf(kb, q_off, K, nqb) + 1) >> 1; };   // query steps
  auto qload = [&](int idx) { return ((q_off + min(16 * (nqb - 1 - idx) + 15, K - 1)) >> 5) + 1; };

  // ---- prologue: every load issued first
  float qr[SR][8], yr[SR][8], orr[SR][8];
#pragma unroll
  for (int r = 0; r < SR; ++r) {
    const int task = threadIdx.x + r * NTH, j = task / CPR, c = task % CPR;
    if (task < KP * CPR && j < K) {
      load8(qr[r], Qg + (int64_t)(q_off + j) * p.ld + 8 * c);
      load8(yr[r], dOg + (int64_t)j * p.d + 8 * c);
      load8(orr[r], Og + (int64_t)j * p.d + 8 * c);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) qr[r][e] = yr[r][e] = orr[r][e] = 0.f;
    }
  }
  // K / V rows of a key block: rows past I read row I - 1 (finite) and are zeroed at split time, so the
  // loads carry no branch (a branch here kept the arrays in scratch)
  float kr[NT][8], vr[NT][8];
  auto load_kv = [&](int kb) {
    const int krow = min(16 * kb + li, I - 1);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      load8(kr[t], Kg + (int64_t)krow * p.ld + 32 * t + 8 * g);
      load8(vr[t], Vg + (int64_t)krow * p.ld + 32 * t + 8 * g);
    }
  };
  int kb = lpt_pick<NWV>(0, wave, nkb, kload);
  if (HD <= 32 && kb >= 0) load_kv(kb);           // hd 64: after the staging stores (register pressure)
  for (int j = threadIdx.x; j < KP; j += NTH) {
    const bool v = j < K;
    qps[j] = v ? q_off + j : -1;
    lse2[j] = v ? p.lse_in[(int64_t)pair * K + j] * L2E : INFINITY;
  }
  if (threadIdx.x < nkb) {
    int base = 0;
    for (int k = 0; k < (int)threadIdx.x; ++k) base += nqb - tail_qf(k, q_off, K, nqb);
    qfb[threadIdx.x] = tail_qf(threadIdx.x, q_off, K, nqb);
    bbase[threadIdx.x] = base;
  }
#pragma unroll
  for (int r = 0; r < SR; ++r) {
    const int task = threadIdx.x + r * NTH, j = task / CPR, c = task % CPR;
    float pd = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) pd = fmaf(yr[r][e], orr[r][e], pd);
#pragma unroll
    for (int off = 1; off < CPR; off <<= 1) pd += __shfl_xor(pd, off, 64);
    if (task < KP * CPR) {
      if (c == 0) dlt[j] = pd;
      const int o = poff<HD>(j, c);
      store_planes(qimg, PBQ, o, qr[r]);
      store_planes(oimg, PBO, o, yr[r]);
    }
  }
  if (HD > 32 && kb >= 0) load_kv(kb);
  __syncthreads();

  // ---- phase 1: key-block owners
  const float c1 = p.scale * L2E;
#pragma unroll 1
  for (int slot = 0; kb >= 0; ++slot) {
    const int krow = 16 * kb + li;                 // this lane's key
    u32x4 kp[NT][3], vp[NT][3];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        kr[t][e] = krow < I ? kr[t][e] : 0.f;
        vr[t][e] = krow < I ? vr[t][e] : 0.f;
      }
      split8(kr[t], kp[t]);
      split8(vr[t], vp[t]);
    }
    const int kbn = lpt_pick<NWV>(slot + 1, wave, nkb, kload);
    if (kbn >= 0) load_kv(kbn);                    // next key block's K / V in flight meanwhile
    f32x4 dk[NM], dv[NM];
#pragma unroll
    for (int m = 0; m < NM; ++m) dk[m] = dv[m] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int a0 = qfb[kb], blk0 = bbase[kb];
#pragma unroll 1
    for (int a = a0; a < nqb; a += 2) {
      const bool two = a + 1 < nqb;
      float P[8], dS[8];
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int qb = a + half;
#pragma unroll
        for (int i = 0; i < 4; ++i) P[4 * half + i] = dS[4 * half + i] = 0.f;
        if (half == 1 && !two) continue;
        f32x4 s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          u32x4 fa[3], fb[3];
          row_frag<HD>(fa, qimg, PBQ, 16 * qb + li, t, g);
          row_frag<HD>(fb, oimg, PBO, 16 * qb + li, t, g);
          s = mma6(fa, kp[t], s);                                     // S: row = query, col = key
          dp = mma6(fb, vp[t], dp);                                   // dP
        }
        const int q0 = 16 * qb + 4 * g;
        const f32x4 L = *reinterpret_cast<const f32x4*>(lse2 + q0);
        const f32x4 D = *reinterpret_cast<const f32x4*>(dlt + q0);
        const i32x4 Qp = *reinterpret_cast<const i32x4*>(qps + q0);
        char* blk = dss + 1024 * (blk0 + qb - a0);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float e = __builtin_amdgcn_exp2f(fmaf(s[i], c1, -L[i]));
          const float pv = krow <= Qp[i] ? e : 0.f;
          const float ds = pv * (dp[i] - D[i]) * p.scale;
          P[4 * half + i] = pv;
          dS[4 * half + i] = ds;
          *reinterpret_cast<float*>(blk + poff<32>(4 * g + i, li >> 2) + 4 * (li & 3)) = ds;
        }
      }
      u32x4 pp[3], sp[3];
      split8(P, pp);
      split8(dS, sp);
      const int rb = two ? 16 * a + 16 : 16 * a;
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        u32x4 fa[3], fb[3];
        tr_frag<HD>(fa, oimg, PBO, 16 * a, rb, m, lane);
        tr_frag<HD>(fb, qimg, PBQ, 16 * a, rb, m, lane);
        dv[m] = mma6(fa, pp, dv[m]);                                  // dV^T += dO^T P
        dk[m] = mma6(fb, sp, dk[m]);                                  // dK^T += Q^T dS
      }
    }
    if (krow < I) {
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        *reinterpret_cast<f32x4*>(dKg + (int64_t)krow * p.ld + 16 * m + 4 * g) = dk[m];
        *reinterpret_cast<f32x4*>(dVg + (int64_t)krow * p.ld + 16 * m + 4 * g) = dv[m];
      }
    }
    kb = kbn;
  }
  // K image for phase 2: the rows re-read (L2-warm) before the barrier, stored into the Q planes' space after it
  constexpr int KR = (MAXKB * 16 * CPR + NTH - 1) / NTH;
  float kk[KR][8];
#pragma unroll
  for (int r = 0; r < KR; ++r) {
    const int task = threadIdx.x + r * NTH, row = task / CPR, c = task % CPR;
    if (task < IP * CPR && row < I) {
      load8(kk[r], Kg + (int64_t)row * p.ld + 8 * c);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) kk[r][e] = 0.f;
    }
  }
  __syncthreads();                                   // dS store complete, Q planes no longer read
#pragma unroll
  for (int r = 0; r < KR; ++r) {
    const int task = threadIdx.x + r * NTH, row = task / CPR, c = task % CPR;
    if (task < IP * CPR) store_planes(qimg, PBQ, poff<HD>(row, c), kk[r]);
  }
  __syncthreads();

  // ---- phase 2: query-block owners, dQ^T = K^T dS^T
#pragma unroll 1
  for (int slot = 0;; ++slot) {
    const int idx = lpt_pick<NWV>(slot, wave, nqb, qload);
    if (idx < 0) break;
    const int qb = nqb - 1 - idx;
    const int kbl = (q_off + min(16 * qb + 15, K - 1)) >> 4;
    f32x4 dq[NM];
#pragma unroll
    for (int m = 0; m < NM; ++m) dq[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int k2 = 0; k2 <= kbl; k2 += 2) {
      const bool two = k2 + 1 <= kbl;
      float v[8];
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(dss + 1024 * (bbase[k2] + qb - qfb[k2]) + poff<32>(li, g));
      f32x4 x1 = {0.f, 0.f, 0.f, 0.f};
      if (two) x1 = *reinterpret_cast<const f32x4*>(dss + 1024 * (bbase[k2 + 1] + qb - qfb[k2 + 1]) + poff<32>(li, g));
#pragma unroll
      for (int i = 0; i < 4; ++i) { v[i] = x0[i]; v[4 + i] = x1[i]; }
      u32x4 bp[3];
      split8(v, bp);
#pragma unroll
      for (int m = 0; m < NM; ++m) {
        u32x4 fa[3];
        tr_frag<HD>(fa, qimg, PBQ, 16 * k2, two ? 16 * k2 + 16 : 16 * k2, m, lane);
        dq[m] = mma6(fa, bp, dq[m]);
      }
    }
    const int j = 16 * qb + li;
    if (j < K) {
      float* drow = dQg + (int64_t)(q_off + j) * p.ld + 4 * g;
#pragma unroll
      for (int m = 0; m < NM; ++m) *reinterpret_cast<f32x4*>(drow + 16 * m) = dq[m];
    }
  }
}

size_t fwd_lds(int I, int hd) { return (size_t)6 * ((I + 15) / 16 * 16) * hd * 2; }

// causal 16 x 16 block pairs of the tail-query backward
int bwd_pairs(int I, int K) {
  const int nkb = (I + 15) / 16, nqb = (K + 15) / 16, q_off = I - K;
  int n = 0, f = 0;
  for (int kb = 0; kb < nkb; ++kb) {
    while (f < nqb && q_off + std::min(16 * f + 15, K - 1) < 16 * kb) ++f;
    n += nqb - f;
  }
  return n;
}

size_t bwd_lds(int I, int K, int hd) {
  const int IP = (I + 15) / 16 * 16, KP = (K + 15) / 16 * 16;
  return (size_t)3 * IP * hd * 2 + (size_t)3 * KP * hd * 2 + 12 * (size_t)KP + 8 * MAXKB + 1024 * (size_t)bwd_pairs(I, K);
}

static int g_enabled = [] {
  const char* e = std::getenv("ONETRANS_ATTN_SLICE");
  return e ? std::atoi(e) : 1;
}();

constexpr int FWD_WAVES = 8, BWD_WAVES = 8;
// A/B timing of the workgroup size (4 or 8 waves) per head_dim: ONETRANS_ATTN_SLICE_WAVES=fwd32,fwd64,bwd32,bwd64
static int g_waves[4] = {FWD_WAVES, FWD_WAVES, BWD_WAVES, BWD_WAVES};
static int g_waves_init = [] {
  if (const char* e = std::getenv("ONETRANS_ATTN_SLICE_WAVES"))
    std::sscanf(e, "%d,%d,%d,%d", &g_waves[0], &g_waves[1], &g_waves[2], &g_waves[3]);
  return 0;
}();

template <typename F>
static void raise_lds_limit(F* k) {
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
}

}  // namespace slice

bool attn_slice_fwd_supported(int I, int K, int head_dim) {
  return slice::g_enabled && (head_dim == 32 || head_dim == 64) && I <= 16 * slice::MAXKB && K > 0 && K <= I &&
         slice::fwd_lds(I, head_dim) <= (size_t)slice::LDS_MAX;
}

bool attn_slice_bwd_supported(int I, int K, int head_dim, bool selected) {
  return slice::g_enabled && !selected && (head_dim == 32 || head_dim == 64) && I <= 16 * slice::MAXKB && K > 0 &&
         K <= I && slice::bwd_lds(I, K, head_dim) <= (size_t)slice::LDS_MAX;
}

int attn_slice_fwd(const float* qkv, int64_t ld, int B, int H, int I, int K, const int32_t* qpos, int head_dim,
                   float* out, float* lse, hipStream_t stream) {
  using namespace slice;
  static std::once_flag once;
  std::call_once(once, [] {
    raise_lds_limit(attn_fwd_slice_kernel<32, 8>);
    raise_lds_limit(attn_fwd_slice_kernel<64, 8>);
    raise_lds_limit(attn_fwd_slice_kernel<32, 4>);
    raise_lds_limit(attn_fwd_slice_kernel<64, 4>);
    (void)hipGetLastError();
  });
  SliceArgs p{qkv, ld, H * head_dim, nullptr, nullptr, nullptr, out, lse, nullptr, B, H, I, K,
              1.f / sqrtf((float)head_dim), qpos};
  const size_t lds = fwd_lds(I, head_dim);
  const int nw = g_waves[head_dim == 32 ? 0 : 1] == 4 ? 4 : 8;
  const dim3 grid((unsigned)((int64_t)B * H)), block(64 * nw);
  if (head_dim == 32) {
    if (nw == 4) hipLaunchKernelGGL((attn_fwd_slice_kernel<32, 4>), grid, block, lds, stream, p);
    else hipLaunchKernelGGL((attn_fwd_slice_kernel<32, 8>), grid, block, lds, stream, p);
  } else {
    if (nw == 4) hipLaunchKernelGGL((attn_fwd_slice_kernel<64, 4>), grid, block, lds, stream, p);
    else hipLaunchKernelGGL((attn_fwd_slice_kernel<64, 8>), grid, block, lds, stream, p);
  }
  OT_LAUNCH_CHECK("ot_attn_fwd(slice)");
  return OT_OK;
}

int attn_slice_bwd(const float* qkv, int64_t ld, const float* out, const float* dout, const float* lse, int B, int H,
                   int I, int K, int head_dim, float* dqkv, hipStream_t stream) {
  using namespace slice;
  static std::once_flag once;
  std::call_once(once, [] {
    raise_lds_limit(attn_bwd_slice_kernel<32, 8>);
    raise_lds_limit(attn_bwd_slice_kernel<64, 8>);
    raise_lds_limit(attn_bwd_slice_kernel<32, 4>);
    raise_lds_limit(attn_bwd_slice_kernel<64, 4>);
    (void)hipGetLastError();
  });
  SliceArgs p{qkv, ld, H * head_dim, out, dout, lse, nullptr, nullptr, dqkv, B, H, I, K,
              1.f / sqrtf((float)head_dim), nullptr};
  const size_t lds = bwd_lds(I, K, head_dim);
  const int nw = g_waves[head_dim == 32 ? 2 : 3] == 4 ? 4 : 8;
  const dim3 grid((unsigned)((int64_t)B * H)), block(64 * nw);
  if (head_dim == 32) {
    if (nw == 4) hipLaunchKernelGGL((attn_bwd_slice_kernel<32, 4>), grid, block, lds, stream, p);
    else hipLaunchKernelGGL((attn_bwd_slice_kernel<32, 8>), grid, block, lds, stream, p);
  } else {
    if (nw == 4) hipLaunchKernelGGL((attn_bwd_slice_kernel<64, 4>), grid, block, lds, stream, p);
    else hipLaunchKernelGGL((attn_bwd_slice_kernel<64, 8>), grid, block, lds, stream, p);
  }
  OT_LAUNCH_CHECK("ot_attn_bwd(slice)");
  return OT_OK;
}

}  // namespace ot
