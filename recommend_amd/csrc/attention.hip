// Causal attention with a query tail offset on gfx950 fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces model.py:100-114 (einsum QK^T / sqrt(hd), band_part causal mask filled with -1e9,
// softmax, einsum PV).  The -1e9 fill equals -inf here because the diagonal is never masked.
// Only the last K queries of a layer with I tokens are computed (pyramid keep / last-layer DCE,
// exact), keys/values cover all I tokens.
//
// Layout: qkv [B*I, ld] token-major (q at col 0, k at col d, v at col 2d, head h at +h*hd);
// o / dO compact [B*K, d]; lse [B, H, K]; dqkv like qkv (dq only on the K tail rows).
// One wave per (sample, head); a block of 4 waves = 4 consecutive (b, h) pairs.
//
// Orientation: S^T = K Q^T puts the query on the MFMA column (lane) and keys in registers, so
// P^T (registers) is directly the B operand of O^T = V^T P^T (the accumulator-as-operand idiom,
// cdna_hip_programming.md §3) with the k index of step r = the key held in register r.
#include <algorithm>
#include <cstdlib>
#include <mutex>

#include "common.h"
#include "attn_slice.h"

#ifndef OT_ATTN_FWD_BRANCHLOAD
#define OT_ATTN_FWD_BRANCHLOAD 1
#endif
#ifndef OT_ATTN_BWD_BRANCHLOAD
#define OT_ATTN_BWD_BRANCHLOAD 1
#endif
#if OT_ATTN_BWD_BRANCHLOAD
#define BWD_LOAD load_frag
#else
#define BWD_LOAD load_frag_clamped
#endif
#ifndef OT_ATTN_KV_LDS_MAX
#define OT_ATTN_KV_LDS_MAX (80 * 1024)
#endif
#ifndef OT_ATTN_FWD_MASKALL
#define OT_ATTN_FWD_MASKALL 0
#endif

namespace ot {

struct AttnArgs {
  const float* qkv; int64_t ld; int d;
  const float* o; const float* dout; float* out; float* lse; float* dqkv; float* delta;
  int B, H, I, K;
  float scale;
  const int32_t* qpos;      // kept query positions [B*K] (ot_pyramid_select) or null: I - K + j
  // key-grouped backward (attn_bwd_group_kernel): kslices workgroups per (sample, head), workgroup s
  // owning key blocks kgroup*s .. kgroup*s + kgroup-1; slice 0 writes dQ into dqkv, slice s > 0 into
  // dqpart[s - 1] ([B*K][d]), summed into dqkv by attn_dq_reduce_kernel
  int kslices, kgroup; float* dqpart;
  // OT_ATTN_DQKV_BF16 (key-grouped backward only): dqkv holds bf16 (uint16 bits, ld in elements); every
  // slice s writes its dQ into dqpart[s] and attn_dq_reduce_kernel stores the rounded sum (slice 0 first,
  // then the later slices in order: the f32 path's sum, rounded once)
  int dq_bf16;
  // OT_ATTN_QKV_BF16 (key-grouped backward only): qkv holds bf16 (uint16 bits, ld in elements) — the fp8
  // forward's dequantised operands, which the bf16 backward would round to bf16 anyway
  int qkv_bf16;
  // OT_ATTN_DQ_PART_BF16 (with OT_ATTN_DQKV_BF16): the slices' dQ partials are stored rounded to bf16 (half the
  // partial traffic; summed in f32 by attn_dq_reduce_kernel, then rounded once more)
  int dq_part16;
  // short-tail backward, f32 dqkv (fp16-pair consumers' bounds): max |dQKV| folded in (one float, zeroed by the
  // caller) and the per-row maxima [B*I][3][H] (dQ / dK / dV part per head; the caller zeroes the array)
  float* amax; float* rowmax;
};

// position of kept query j (< K) of the sample whose qpos slice is qp (null: the tail rule)
__device__ __forceinline__ int query_pos(const int32_t* qp, int q_off, int j) { return qp ? qp[j] : q_off + j; }

__device__ __forceinline__ int acc_row(int r, int hh) { return (r & 3) + 8 * (r >> 2) + 4 * hh; }

// Fragment of a [32 rows x HD] operand for a product over HD: lane (li, hh) holds row li,
// dims (HD/2)*hh + s, s < HD/2 (the k permutation).  Rows >= nrows give zeros.
template <int HD>
__device__ __forceinline__ void load_frag(float (&f)[HD / 2], const float* base, int64_t ld, int row,
                                          int nrows, int hh) {
  if (row < nrows) {
    const float* p = base + (int64_t)row * ld + (HD / 2) * hh;
    if constexpr (HD >= 8) {
#pragma unroll
      for (int q = 0; q < HD / 8; ++q) {
        f32x4 v = *reinterpret_cast<const f32x4*>(p + 4 * q);
        f[4 * q] = v.x; f[4 * q + 1] = v.y; f[4 * q + 2] = v.z; f[4 * q + 3] = v.w;
      }
    }
  } else {
#pragma unroll
    for (int s = 0; s < HD / 2; ++s) f[s] = 0.f;
  }
}

template <int HD>
__device__ __forceinline__ f32x16 mm_frag(const float (&a)[HD / 2], const float (&b)[HD / 2]) {
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
  for (int s = 0; s < HD / 2; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b[s], acc, 0, 0, 0);
  return acc;
}

constexpr int NB(int hd) { return (hd + 31) / 32; }

// O^T[d][col] += sum_r X[row(r)][d0 + li] * P[r]   (X rows are the k index of register r)
template <int HD>
__device__ __forceinline__ void acc_xT_p(f32x16 (&acc)[NB(HD)], const float* xbase, int64_t ld, int row0,
                                         int nrows, const f32x16& p, int li, int hh) {
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = row0 + acc_row(r, hh);
#pragma unroll
    for (int c = 0; c < NB(HD); ++c) {
      const int dd = 32 * c + li;
      float a = 0.f;
      if (row < nrows && dd < HD) a = xbase[(int64_t)row * ld + dd];
      acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, p[r], acc[c], 0, 0, 0);
    }
  }
}

// Per-wave LDS tile [32][HD+4]: a block the wave holds as row fragments (lane li = row li) is
// written once and read transposed (lane li = column) as the A operand of the accumulator-as-
// operand products — no scalar global re-reads inside the MFMA chains.
template <int HD>
constexpr int TLD() { return HD + 4; }

template <int HD>
__device__ __forceinline__ void frag_to_lds(float* tile, const float (&f)[HD / 2], int li, int hh) {
#pragma unroll
  for (int q = 0; q < HD / 8; ++q)
    *reinterpret_cast<f32x4*>(tile + li * TLD<HD>() + (HD / 2) * hh + 4 * q) =
        f32x4{f[4 * q], f[4 * q + 1], f[4 * q + 2], f[4 * q + 3]};
}

// acc[c] (+)= sum_r tile[row(r)][32c + li] * p[r]
template <int HD>
__device__ __forceinline__ void acc_tile_p(f32x16 (&acc)[NB(HD)], const float* tile, const f32x16& p, int li,
                                           int hh) {
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = acc_row(r, hh);
#pragma unroll
    for (int c = 0; c < NB(HD); ++c) {
      const int dd = 32 * c + li;
      const float a = dd < HD ? tile[row * TLD<HD>() + dd] : 0.f;
      acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, p[r], acc[c], 0, 0, 0);
    }
  }
}

// Fragment as load_frag, but rows >= nrows read row nrows - 1 (finite data that the masks null).
template <int HD>
__device__ __forceinline__ void load_frag_clamped(float (&f)[HD / 2], const float* base, int64_t ld, int row,
                                                  int nrows, int hh) {
  const float* p = base + (int64_t)(row < nrows ? row : nrows - 1) * ld + (HD / 2) * hh;
#pragma unroll
  for (int q = 0; q < HD / 8; ++q) {
    f32x4 v = *reinterpret_cast<const f32x4*>(p + 4 * q);
    f[4 * q] = v.x; f[4 * q + 1] = v.y; f[4 * q + 2] = v.z; f[4 * q + 3] = v.w;
  }
}

// Forward.  Scores are kept in the log2 domain (q pre-scaled by log2(e)/sqrt(hd), one multiply per
// q element) so the online softmax uses v_exp_f32 directly; the causal mask is applied on the
// diagonal key block only (earlier blocks are fully visible); K/V rows past the end are loaded from
// a clamped row (finite) and removed by the mask, so the loads carry no branches.
template <int HD>
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnArgs p) {
  __shared__ __attribute__((aligned(16))) float lds[4][32 * TLD<HD>()];
  const int lane = threadIdx.x & 63, li = lane & 31, hh = lane >> 5;
  float* tV = lds[threadIdx.x >> 6];
  const int pair = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pair >= p.B * p.H) return;
  const int b = pair / p.H, h = pair % p.H;
  const int I = p.I, K = p.K, q_off = I - K;
  const float* Q = p.qkv + (int64_t)b * I * p.ld + h * HD;
  const float* Kp = Q + p.d;
  const float* V = Q + 2 * p.d;
  const int32_t* qp = p.qpos ? p.qpos + (int64_t)b * K : nullptr;
  const int nqb = (K + 31) / 32;
  const float qscale = p.scale * 1.4426950408889634f;   // log2(e) / sqrt(hd)
  for (int qb = 0; qb < nqb; ++qb) {
    const int j = 32 * qb + li;                     // this lane's query (kept index)
    const int qpos = query_pos(qp, q_off, j < K ? j : K - 1);
    float qf[HD / 2];
    load_frag_clamped<HD>(qf, Q, p.ld, qpos, I, hh);
#pragma unroll
    for (int s = 0; s < HD / 2; ++s) qf[s] *= qscale;
    f32x16 oacc[NB(HD)];
#pragma unroll
    for (int c = 0; c < NB(HD); ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) oacc[c][r] = 0.f;
    float m = -INFINITY, l = 0.f;
    const int last_q = query_pos(qp, q_off, min(32 * qb + 31, K - 1));   // positions ascend
    const int nkb = last_q / 32 + 1;
    const int first_masked = query_pos(qp, q_off, 32 * qb) / 32;       // key blocks >= this may be masked
    for (int kb = 0; kb < nkb; ++kb) {
      const int key0 = 32 * kb;
      float kf[HD / 2], vf[HD / 2];
#if OT_ATTN_FWD_BRANCHLOAD
      load_frag<HD>(kf, Kp, p.ld, key0 + li, I, hh);
      load_frag<HD>(vf, V, p.ld, key0 + li, I, hh);
#else
      load_frag_clamped<HD>(kf, Kp, p.ld, key0 + li, I, hh);
      load_frag_clamped<HD>(vf, V, p.ld, key0 + li, I, hh);
#endif
      frag_to_lds<HD>(tV, vf, li, hh);
      f32x16 s = mm_frag<HD>(kf, qf);               // S^T (log2 units): row = key, col = query
      if (OT_ATTN_FWD_MASKALL || kb >= first_masked) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          s[r] = (key0 + acc_row(r, hh) <= qpos) ? s[r] : -INFINITY;   // kpos <= qpos < I
      }
      float mloc = s[0];
#pragma unroll
      for (int r = 1; r < 16; ++r) mloc = fmaxf(mloc, s[r]);
      mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
      const float mnew = fmaxf(m, mloc);            // finite: key 0 is always visible
      const float corr = __builtin_amdgcn_exp2f(m - mnew);
      float lsum = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = __builtin_amdgcn_exp2f(s[r] - mnew);
        s[r] = e;
        lsum += e;
      }
      lsum += __shfl_xor(lsum, 32, 64);
      l = l * corr + lsum;
      m = mnew;
#pragma unroll
      for (int c = 0; c < NB(HD); ++c) oacc[c] *= corr;
      __builtin_amdgcn_wave_barrier();
      acc_tile_p<HD>(oacc, tV, s, li, hh);             // O^T += V^T P^T
      __builtin_amdgcn_wave_barrier();
    }
    if (j < K) {
      const float inv = 1.f / l;
      float* orow = p.out + ((int64_t)b * K + j) * p.d + h * HD;
#pragma unroll
      for (int c = 0; c < NB(HD); ++c)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int dd = 32 * c + 8 * g + 4 * hh;
          if (dd < HD) {
            f32x4 v = {oacc[c][4 * g] * inv, oacc[c][4 * g + 1] * inv, oacc[c][4 * g + 2] * inv,
                       oacc[c][4 * g + 3] * inv};
            *reinterpret_cast<f32x4*>(orow + dd) = v;
          }
        }
      // natural-log lse for the backward: m (log2 units) * ln 2 + ln l
      if (hh == 0) p.lse[((int64_t)b * p.H + h) * K + j] = m * 0.6931471805599453f + __logf(l);
    }
  }
}

// Forward, one workgroup per (sample, head) for short sequences: the (b, h) slice's K and V rows
// are staged in LDS once ([KP][HD+4], zero rows past I) and shared by the 4 waves, each of which
// takes whole query blocks (snake order from the heaviest causal block: balanced).  Every K/V byte
// is read from HBM once (the one-wave-per-head kernel re-reads them for every query block).
template <int HD>
__global__ __launch_bounds__(256) void attn_fwd_kv_kernel(AttnArgs p) {
  extern __shared__ __attribute__((aligned(16))) float kv[];   // Ks [KP][LD] then Vs [KP][LD]
  constexpr int LD = TLD<HD>();
  const int lane = threadIdx.x & 63, li = lane & 31, hh = lane >> 5, wave = threadIdx.x >> 6;
  const int pair = blockIdx.x;
  const int b = pair / p.H, h = pair % p.H;
  const int I = p.I, K = p.K, q_off = I - K;
  const int KP = (I + 31) / 32 * 32;
  float* Ks = kv;
  float* Vs = kv + KP * LD;
  const float* Q = p.qkv + (int64_t)b * I * p.ld + h * HD;
  // stage K and V: thread t copies float4 chunks (row, c4) of both, rows >= I zero
  constexpr int C4 = HD / 4;
  for (int i = threadIdx.x; i < KP * C4; i += 256) {
    const int row = i / C4, c = 4 * (i % C4);
    f32x4 kvv = {0.f, 0.f, 0.f, 0.f}, vvv = {0.f, 0.f, 0.f, 0.f};
    if (row < I) {
      const float* src = Q + (int64_t)row * p.ld + c;
      kvv = *reinterpret_cast<const f32x4*>(src + p.d);
      vvv = *reinterpret_cast<const f32x4*>(src + 2 * p.d);
    }
    *reinterpret_cast<f32x4*>(Ks + row * LD + c) = kvv;
    *reinterpret_cast<f32x4*>(Vs + row * LD + c) = vvv;
  }
  __syncthreads();
  const int32_t* qp = p.qpos ? p.qpos + (int64_t)b * K : nullptr;
  const int nqb = (K + 31) / 32;
  const float qscale = p.scale * 1.4426950408889634f;   // log2(e) / sqrt(hd)
  for (int i = 0; i < nqb; ++i) {
    const int slot = (i >> 2) & 1 ? 3 - (i & 3) : (i & 3);   // snake assignment
    if (slot != wave) continue;
    const int qb = nqb - 1 - i;
    const int j = 32 * qb + li;
    const int qpos = query_pos(qp, q_off, j < K ? j : K - 1);
    float qf[HD / 2];
    load_frag<HD>(qf, Q, p.ld, j < K ? qpos : I, I, hh);           // rows >= I: zeros
#pragma unroll
    for (int s2 = 0; s2 < HD / 2; ++s2) qf[s2] *= qscale;
    f32x16 oacc[NB(HD)];
#pragma unroll
    for (int c = 0; c < NB(HD); ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) oacc[c][r] = 0.f;
    float m = -INFINITY, l = 0.f;
    const int last_q = query_pos(qp, q_off, min(32 * qb + 31, K - 1));
    const int nkb = last_q / 32 + 1;
    const int first_masked = query_pos(qp, q_off, 32 * qb) / 32;
    for (int kb = 0; kb < nkb; ++kb) {
      const int key0 = 32 * kb;
      float kf[HD / 2];
#pragma unroll
      for (int q4 = 0; q4 < HD / 8; ++q4) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(Ks + (key0 + li) * LD + (HD / 2) * hh + 4 * q4);
        kf[4 * q4] = v.x; kf[4 * q4 + 1] = v.y; kf[4 * q4 + 2] = v.z; kf[4 * q4 + 3] = v.w;
      }
      f32x16 s = mm_frag<HD>(kf, qf);               // S^T (log2 units): row = key, col = query
      if (kb >= first_masked) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          s[r] = (key0 + acc_row(r, hh) <= qpos) ? s[r] : -INFINITY;
      }
      float mloc = s[0];
#pragma unroll
      for (int r = 1; r < 16; ++r) mloc = fmaxf(mloc, s[r]);
      mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
      const float mnew = fmaxf(m, mloc);
      const float corr = __builtin_amdgcn_exp2f(m - mnew);
      float lsum = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = __builtin_amdgcn_exp2f(s[r] - mnew);
        s[r] = e;
        lsum += e;
      }
      lsum += __shfl_xor(lsum, 32, 64);
      l = l * corr + lsum;
      m = mnew;
#pragma unroll
      for (int c = 0; c < NB(HD); ++c) oacc[c] *= corr;
      acc_tile_p<HD>(oacc, Vs + key0 * LD, s, li, hh);     // O^T += V^T P^T
    }
    if (j < K) {
      const float inv = 1.f / l;
      float* orow = p.out + ((int64_t)b * K + j) * p.d + h * HD;
#pragma unroll
      for (int c = 0; c < NB(HD); ++c)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int dd = 32 * c + 8 * g + 4 * hh;
          if (dd < HD) {
            f32x4 v = {oacc[c][4 * g] * inv, oacc[c][4 * g + 1] * inv, oacc[c][4 * g + 2] * inv,
                       oacc[c][4 * g + 3] * inv};
            *reinterpret_cast<f32x4*>(orow + dd) = v;
          }
        }
      if (hh == 0) p.lse[((int64_t)b * p.H + h) * K + j] = m * 0.6931471805599453f + __logf(l);
    }
  }
}

// ------------------------------------------------------------------------------------------
// XOR-swizzled byte offset in a bf16 image of RB-byte rows (the split forward's V planes, the key-grouped
// backward's [32][HD] and [32][32] images): row r's 16-B chunk index is XORed with (r / (256 / RB)) mod (RB / 16), so the rows that share LDS banks
// (256 B apart) spread over the chunks — the row-major fragment reads (one row per lane) and the transposed reads
// were 2- to 8-way bank-conflicted on the plain layout (C5: conflict cycles 68% of the LDS-active cycles).
#ifndef OT_BWDG_SWIZZLE
#define OT_BWDG_SWIZZLE 1
#endif
template <int RB>
__device__ __forceinline__ int gswz(int r, int b) {
  constexpr int P = 256 / RB, C = RB / 16;
  return OT_BWDG_SWIZZLE ? r * RB + (b ^ (((r / P) & (C - 1)) << 4)) : r * RB + b;
}
template <int RB>
__device__ __forceinline__ u32x4 tr16_frag_sw(const char* img, int ra, int rb, int colbase, int lane) {
  typedef short v4i16 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) v4i16 lds_v4i16;
  const int gi = lane & 15, q = gi >> 2, pp = gi & 3;
  const int c = colbase + 16 * ((lane >> 4) & 1) + 4 * pp;
  const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(img + gswz<RB>(ra + q, c * 2)));
  const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(img + gswz<RB>(rb + q, c * 2)));
  const u32x2 a = __builtin_bit_cast(u32x2, lo), b = __builtin_bit_cast(u32x2, hi);
  return u32x4{a.x, a.y, b.x, b.y};
}

// Split-bf16 forward (OT_MATMUL_SPLIT_BF16; HD >= 32): the same online softmax as attn_fwd_kernel,
// the two products on v_mfma_f32_32x32x16_bf16 with every f32 operand split exactly into three bf16
// planes and the six largest plane products summed (mfma_split6: f32-accurate, 2.7x fewer MFMA
// cycles than the 32x32x2 f32 form).
//   S^T = K Q^T: K (A, lane = key) and Q (B, lane = query) fragments split in registers; lane half
//     hh, k-step t, element j <-> dim (HD/2) hh + 8t + j on both sides.
//   O^T += V^T P^T: P^T is the S^T accumulator (k-step s = registers 8s..8s+7, element j <-> key
//     16s + 8(j>>2) + 4hh + (j&3)); V^T comes from the wave's row-major bf16 V plane images through
//     ds_read_b64_tr_b16 (4 key rows of the lane's dim column per read, two reads per k-step).
template <int HD>
__device__ __forceinline__ u32x4 vt_frag(const char* plane, int s, int c, int lane) {
  // lane 4q+p of each 16-lane group addresses key row r0 + q, dims c0 + 4p .. c0 + 4p + 3
  typedef short v4i16 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) v4i16 lds_v4i16;
  const int hh = lane >> 5, gi = lane & 15, q = gi >> 2, pp = gi & 3;
  const int c0 = 32 * c + 16 * ((lane >> 4) & 1) + 4 * pp;
  const int r0 = 16 * s + 4 * hh + q;
  const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(plane + gswz<HD * 2>(r0, c0 * 2)));
  const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(plane + gswz<HD * 2>(r0 + 8, c0 * 2)));
  const u32x2 a = __builtin_bit_cast(u32x2, lo), b = __builtin_bit_cast(u32x2, hi);
  return u32x4{a.x, a.y, b.x, b.y};
}

template <int HD, int TERMS>
__global__ __launch_bounds__(256) void attn_fwd_split_kernel(AttnArgs p) {
  static_assert(HD >= 32, "split forward: HD >= 32");
  constexpr int NS = HD / 16;                         // k-steps of S^T
  constexpr int PLANE = 32 * HD * 2;                  // bytes of one V plane image [32 keys][HD] bf16
  __shared__ __attribute__((aligned(16))) char lds[4][3 * PLANE];
  const int lane = threadIdx.x & 63, li = lane & 31, hh = lane >> 5;
  char* vimg = lds[threadIdx.x >> 6];
  const int pair = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pair >= p.B * p.H) return;
  const int b = pair / p.H, h = pair % p.H;
  const int I = p.I, K = p.K, q_off = I - K;
  const float* Q = p.qkv + (int64_t)b * I * p.ld + h * HD;
  const float* Kp = Q + p.d;
  const float* V = Q + 2 * p.d;
  const int32_t* qp = p.qpos ? p.qpos + (int64_t)b * K : nullptr;
  const int nqb = (K + 31) / 32;
  const float qscale = p.scale * 1.4426950408889634f;   // log2(e) / sqrt(hd)
  for (int qb = 0; qb < nqb; ++qb) {
    const int j = 32 * qb + li;
    const int qpos = query_pos(qp, q_off, j < K ? j : K - 1);
    u32x4 qs[NS][3];
    {
      float qf[HD / 2];
      load_frag_clamped<HD>(qf, Q, p.ld, qpos, I, hh);
#pragma unroll
      for (int s = 0; s < HD / 2; ++s) qf[s] *= qscale;
#pragma unroll
      for (int t = 0; t < NS; ++t) split8t<TERMS>(qf + 8 * t, qs[t]);
    }
    f32x16 oacc[NB(HD)];
#pragma unroll
    for (int c = 0; c < NB(HD); ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) oacc[c][r] = 0.f;
    float m = -INFINITY, l = 0.f;
    const int last_q = query_pos(qp, q_off, min(32 * qb + 31, K - 1));
    const int nkb = last_q / 32 + 1;
    const int first_masked = query_pos(qp, q_off, 32 * qb) / 32;
    // K/V fragments of key block kb + 1 are loaded while block kb computes (the global latency
    // would otherwise be exposed once per block)
    float kf[HD / 2], vf[HD / 2];
    load_frag<HD>(kf, Kp, p.ld, li, I, hh);
    load_frag<HD>(vf, V, p.ld, li, I, hh);
    for (int kb = 0; kb < nkb; ++kb) {
      const int key0 = 32 * kb;
      float kn[HD / 2], vn[HD / 2];
      load_frag<HD>(kn, Kp, p.ld, kb + 1 < nkb ? key0 + 32 + li : I, I, hh);    // rows >= I: no load
      load_frag<HD>(vn, V, p.ld, kb + 1 < nkb ? key0 + 32 + li : I, I, hh);
      f32x16 sacc;
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[r] = 0.f;
      {
        // V planes -> the wave's row-major images (row = key li, dims (HD/2) hh ..)
#pragma unroll
        for (int t = 0; t < NS; ++t) {
          u32x4 vp[3];
          split8t<TERMS>(vf + 8 * t, vp);
#pragma unroll
          for (int pl = 0; pl < (TERMS == 1 ? 1 : 3); ++pl)
            *reinterpret_cast<u32x4*>(vimg + pl * PLANE + gswz<HD * 2>(li, ((HD / 2) * hh + 8 * t) * 2)) = vp[pl];
        }
#pragma unroll
        for (int t = 0; t < NS; ++t) {
          u32x4 ks[3];
          split8t<TERMS>(kf + 8 * t, ks);
          sacc = mfma_terms<TERMS>(ks, qs[t], sacc);         // S^T (log2 units): row = key, col = query
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < HD / 2; ++s2) { kf[s2] = kn[s2]; vf[s2] = vn[s2]; }
      f32x16 s = sacc;
      if (kb >= first_masked) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          s[r] = (key0 + acc_row(r, hh) <= qpos) ? s[r] : -INFINITY;
      }
      float mloc = s[0];
#pragma unroll
      for (int r = 1; r < 16; ++r) mloc = fmaxf(mloc, s[r]);
      mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
      const float mnew = fmaxf(m, mloc);
      const float corr = __builtin_amdgcn_exp2f(m - mnew);
      float lsum = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = __builtin_amdgcn_exp2f(s[r] - mnew);
        s[r] = e;
        lsum += e;
      }
      lsum += __shfl_xor(lsum, 32, 64);
      l = l * corr + lsum;
      m = mnew;
#pragma unroll
      for (int c = 0; c < NB(HD); ++c) oacc[c] *= corr;
      u32x4 ps[2][3];
      {
        float pv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) pv[r] = s[r];
        split8t<TERMS>(pv, ps[0]);
        split8t<TERMS>(pv + 8, ps[1]);
      }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int c = 0; c < NB(HD); ++c)
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          u32x4 va[3];
#pragma unroll
          for (int pl = 0; pl < (TERMS == 1 ? 1 : 3); ++pl) va[pl] = vt_frag<HD>(vimg + pl * PLANE, st, c, lane);
          oacc[c] = mfma_terms<TERMS>(va, ps[st], oacc[c]);   // O^T += V^T P^T
        }
      __builtin_amdgcn_wave_barrier();
    }
    if (j < K) {
      const float inv = 1.f / l;
      float* orow = p.out + ((int64_t)b * K + j) * p.d + h * HD;
#pragma unroll
      for (int c = 0; c < NB(HD); ++c)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int dd = 32 * c + 8 * g + 4 * hh;
          f32x4 v = {oacc[c][4 * g] * inv, oacc[c][4 * g + 1] * inv, oacc[c][4 * g + 2] * inv,
                     oacc[c][4 * g + 3] * inv};
          *reinterpret_cast<f32x4*>(orow + dd) = v;
        }
      if (hh == 0) p.lse[((int64_t)b * p.H + h) * K + j] = m * 0.6931471805599453f + __logf(l);
    }
  }
}

// Row statistics of the backward, padded to KP = round_up(K, 32) queries per (b, h) so the main
// kernel reads them as aligned float4 without bounds checks:
//   ws[0 .. BH*KP)       lse  (padding +inf: P = exp(s - inf) = 0 masks the padded queries)
//   ws[BH*KP .. 2*BH*KP) delta[b,h,j] = sum_d dO[b*K+j][h*hd+d] * O[b*K+j][h*hd+d]   (padding 0)
//   (int) ws[2*BH*KP .. +B*KP) kept query positions qpos[b][j] padded with qpos[b][K-1] (only
//   when a selection map is given: the selected-query backward reads them as aligned int4)
// Threads of the first `main` blocks take one float4 of [B*K, d] each (coalesced rows), reduced over
// the hd/4 lanes of a head with shuffles; the remaining blocks fill the padding.
__host__ __device__ constexpr int attn_kpad(int K) { return (K + 31) / 32 * 32; }

__global__ __launch_bounds__(256) void attn_bwd_prep_kernel(const float* __restrict__ o, const float* __restrict__ dout,
                                                            const float* __restrict__ lse, float* ws, int B, int H,
                                                            int K, int hd, int main_blocks, int pad_blocks,
                                                            const int32_t* __restrict__ qpos) {
  const int d = H * hd, KP = attn_kpad(K);
  const int64_t BHKP = (int64_t)B * H * KP;
  if ((int)blockIdx.x >= main_blocks + pad_blocks) {
    const int64_t e = ((int64_t)blockIdx.x - main_blocks - pad_blocks) * blockDim.x + threadIdx.x;   // [B][KP]
    if (!qpos || e >= (int64_t)B * KP) return;
    const int64_t b = e / KP;
    const int j = (int)(e % KP);
    reinterpret_cast<int32_t*>(ws + 2 * BHKP)[e] = qpos[b * K + (j < K ? j : K - 1)];
    return;
  }
  if ((int)blockIdx.x >= main_blocks) {
    const int pad = KP - K;
    const int64_t e = ((int64_t)blockIdx.x - main_blocks) * blockDim.x + threadIdx.x;   // [B*H][pad]
    if (pad == 0 || e >= (int64_t)B * H * pad) return;
    const int64_t bh = e / pad, j = K + e % pad;
    ws[bh * KP + j] = INFINITY;
    ws[BHKP + bh * KP + j] = 0.f;
    return;
  }
  const int64_t i4 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;   // element index in [B*K, d]
  const bool live = i4 < (int64_t)B * K * d;
  float s = 0.f;
  if (live) {
    f32x4 x = *reinterpret_cast<const f32x4*>(o + i4);
    f32x4 y = *reinterpret_cast<const f32x4*>(dout + i4);
    s = x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
  }
  for (int off = (hd >> 3); off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  const int c = (int)(i4 % d);
  if (live && (c % hd) == 0) {
    const int64_t row = i4 / d;
    const int64_t b = row / K, j = row % K;
    const int64_t bh = b * H + c / hd;
    ws[bh * KP + j] = lse[bh * K + j];
    ws[BHKP + bh * KP + j] = s;
  }
}

// ------------------------------------------------------------------------------------------
// Backward, one pass per (sample, head) wave: key blocks outer, the query blocks that see them
// inner.  S and dP are computed with the key on the lane, so P and dS feed dV^T += dO^T P and
// dK^T += Q^T dS directly (dO and Q blocks read transposed from per-wave LDS tiles).  dS (pre-scaled
// by 1/sqrt(hd)) is also written to an LDS tile [query][key] and read back as the B operand of
// dQ^T += K^T dS^T (K block from its LDS tile); the dQ^T accumulator has the query on the lane, so
// the running partial in dqkv is read / written as whole float4 row pieces.  The wave owns its
// (b, h) slice: the first key block (seen by every query) stores, later ones read-modify-write the
// same lanes' addresses.  No atomics, no recompute pass, deterministic.
//
// Padding is branch-free: rows past the end (keys >= I, queries >= K) are loaded from a clamped
// in-bounds row; padded keys are removed by the causal select, padded queries by lse = +inf.

template <int HD>
constexpr int BWD_WAVES() { return HD >= 128 ? 2 : 4; }

// SEL: queries at selected positions (p.qpos, padded copy in the workspace) instead of the tail.
// DS = 2 (head_dim 2 HD, e.g. 64 as two waves of HD = 32): the two waves of a 128-thread block share
// one (sample, head) and each owns half of its dims — half the dK / dV / dQ accumulators, fragments
// and LDS tiles, so a wave has the HD = 32 kernel's footprint (2 waves / SIMD instead of 1).  S and dP
// are sums over all dims: each wave computes its half's partial and the two partials are summed
// through the wave's dS tile (an LDS exchange, four barriers per (key block, query block) pair); the
// softmax gradient is then computed identically in both waves.
// FDL (DS = 1, tail queries, K <= FDL_KP): the row statistics come from the kernel itself instead of
// attn_bwd_prep_kernel — at the first key block (which every query block sees) the wave forms
// delta = rowsum(dO * O) from the dO block it holds anyway and one read of the O block, and copies the
// block's lse (+inf past K); both go to a per-wave LDS row that the later key blocks read.  The prep
// launch and its re-read of dO disappear (C2: 87 us per layer).
constexpr int FDL_KP = 160;
template <int HD, bool SEL, int DS = 1, bool FDL = false>
__global__ __launch_bounds__(DS == 1 ? 64 * BWD_WAVES<HD>() : 64 * DS, 2)   // 2 waves per SIMD
void attn_bwd_kernel(AttnArgs p) {
  static_assert(!FDL || (DS == 1 && !SEL), "attn_bwd_kernel: in-kernel row statistics need DS = 1, tail queries");
  constexpr int LD = TLD<HD>();
  constexpr int SLD = 36;                  // dS tile row stride (32 keys + pad)
  constexpr int PER_WAVE = 3 * 32 * LD + 32 * SLD;
  constexpr int NW = DS == 1 ? BWD_WAVES<HD>() : DS;  // waves per block
  constexpr int HDF = HD * DS;             // head dim
  static_assert(DS == 1 || (DS == 2 && HD == 32), "attn_bwd_kernel: DS = 2 splits head_dim 64");
  // (HD <= 32: the dQ partial is loaded at the start of a pair; larger HD reads it at the end, as
  // the registers of a live seed would not fit next to the dK / dV accumulators)
  constexpr bool SEED_EARLY = HD <= 32;
  __shared__ __attribute__((aligned(16))) float lds[NW * PER_WAVE];
  __shared__ __attribute__((aligned(16))) float rstat[FDL ? NW * 2 * FDL_KP : 4];   // FDL: [wave][lse | delta][KP]
  const int lane = threadIdx.x & 63, li = lane & 31, hh = lane >> 5;
  const int wave = threadIdx.x >> 6;
  float* tO = lds + wave * PER_WAVE;                 // dO block   [query][dim]
  float* tQ = tO + 32 * LD;                          // Q block    [query][dim]
  float* tK = tQ + 32 * LD;                          // K block    [key][dim]
  float* tS = tK + 32 * LD;                          // dS block   [query][key]
  const float* tSp = lds + (wave ^ 1) * PER_WAVE + 3 * 32 * LD;   // DS = 2: the partner wave's dS tile
  const int pair = DS == 1 ? blockIdx.x * NW + wave : blockIdx.x;
  const int half = DS == 1 ? 0 : wave;
  if (pair >= p.B * p.H) return;
  const int b = pair / p.H, h = pair % p.H;
  const int I = p.I, K = p.K, q_off = I - K, KP = attn_kpad(K);
  const int64_t tok0 = (int64_t)b * I;
  const int hoff = h * HDF + half * HD;                // this wave's first dim of head h
  const float* Q = p.qkv + tok0 * p.ld + hoff;
  const float* Kp = Q + p.d;
  const float* V = Q + 2 * p.d;
  const float* Qt = Q + (int64_t)q_off * p.ld;
  const float* dO = p.dout + (int64_t)b * K * p.d + hoff;
  const int32_t* qpp = reinterpret_cast<const int32_t*>(p.delta + 2 * (int64_t)p.B * p.H * KP) + (int64_t)b * KP;
  const float* lsep = p.delta + (int64_t)pair * KP;                              // padded lse
  const float* dltp = p.delta + ((int64_t)p.B * p.H + pair) * KP;                // padded delta
  float* dQt = p.dqkv + (tok0 + q_off) * p.ld + hoff;
  float* dK = p.dqkv + tok0 * p.ld + p.d + hoff;
  float* dV = dK + p.d;
  // DS = 2: S / dP partial exchange through the dS tiles ([4 groups][64 lanes] float4, 4 KiB)
  auto exchange = [&](f32x16& v) {
    f32x4* mine = reinterpret_cast<f32x4*>(tS);
    const f32x4* theirs = reinterpret_cast<const f32x4*>(tSp);
#pragma unroll
    for (int g = 0; g < 4; ++g) mine[g * 64 + lane] = f32x4{v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]};
    __syncthreads();
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 o = theirs[g * 64 + lane];
      // fixed operand order (lower half's partial first): both waves get bit-identical sums
      const f32x4 m4 = {v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]};
      const f32x4 t4 = half == 0 ? m4 + o : o + m4;
      v[4 * g] = t4.x; v[4 * g + 1] = t4.y; v[4 * g + 2] = t4.z; v[4 * g + 3] = t4.w;
    }
    __syncthreads();                                   // the partner is done reading before the next write
  };
  const int nqb = KP / 32;
  const int nkb = (I + 31) / 32;

  for (int kb = 0; kb < nkb; ++kb) {
    const int key0 = 32 * kb;
    const int kpos = key0 + li;                        // this lane's key
    float kf[HD / 2], vf[HD / 2];
    BWD_LOAD<HD>(kf, Kp, p.ld, kpos, I, hh);
    BWD_LOAD<HD>(vf, V, p.ld, kpos, I, hh);
    frag_to_lds<HD>(tK, kf, li, hh);
    f32x16 dk[NB(HD)], dv[NB(HD)];
#pragma unroll
    for (int c = 0; c < NB(HD); ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) { dk[c][r] = 0.f; dv[c][r] = 0.f; }
    int qb0;                                           // first query block that sees key0
    if constexpr (SEL) {
      qb0 = 0;
      while (qb0 < nqb - 1 && qpp[32 * qb0 + 31] < key0) ++qb0;   // ascending positions, padded
    } else {
      qb0 = key0 - q_off; qb0 = qb0 < 0 ? 0 : qb0 / 32;
    }
    float qf[HD / 2], of[HD / 2];
    auto load_qblock = [&](int q0) {
      if constexpr (SEL) BWD_LOAD<HD>(qf, Q, p.ld, q0 + li < K ? qpp[q0 + li] : I, I, hh);
      else BWD_LOAD<HD>(qf, Qt, p.ld, q0 + li, K, hh);
      BWD_LOAD<HD>(of, dO, p.d, q0 + li, K, hh);
    };
    load_qblock(32 * qb0);
    // Per pair, in issue order (vmcnt stays counted, nothing waits early): this block's row stats and
    // dQ seed loads; S / dP chains on the prefetched q block; the next q block's prefetch; softmax
    // gradient; dV / dK chains; dQ chain; dQ store.
    for (int qb = qb0; qb < nqb; ++qb) {
      const int q0 = 32 * qb;
      f32x4 l4[4], d4[4];
      if constexpr (FDL) {
        float* rl = rstat + wave * 2 * FDL_KP;
        if (kb == 0) {                                 // lane li: query q0 + li, dims (HD / 2) hh ..
          float ofo[HD / 2];
          BWD_LOAD<HD>(ofo, p.o + (int64_t)b * K * p.d + hoff, p.d, q0 + li, K, hh);
          float pd = 0.f;
#pragma unroll
          for (int s2 = 0; s2 < HD / 2; ++s2) pd += of[s2] * ofo[s2];
          pd += __shfl_xor(pd, 32, 64);
          const int j = q0 + li;
          if (hh == 0) {
            rl[j] = j < K ? p.lse[(int64_t)pair * K + j] : INFINITY;
            rl[FDL_KP + j] = j < K ? pd : 0.f;
          }
          __builtin_amdgcn_wave_barrier();
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          l4[g] = *reinterpret_cast<const f32x4*>(rl + q0 + 8 * g + 4 * hh);
          d4[g] = *reinterpret_cast<const f32x4*>(rl + FDL_KP + q0 + 8 * g + 4 * hh);
        }
      } else {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          l4[g] = *reinterpret_cast<const f32x4*>(lsep + q0 + 8 * g + 4 * hh);
          d4[g] = *reinterpret_cast<const f32x4*>(dltp + q0 + 8 * g + 4 * hh);
        }
      }
      // dQ^T block: lane = query q0 + li, register r = dim 32c + acc_row(r, hh) (4 float4 per lane)
      const int jq = q0 + li;
      float* dqrow = SEL ? p.dqkv + (tok0 + qpp[jq]) * p.ld + hoff + 4 * hh
                         : dQt + (int64_t)(jq < K ? jq : K - 1) * p.ld + 4 * hh;
      f32x16 dq[NB(HD)];
#pragma unroll
      for (int c = 0; c < NB(HD); ++c)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int dd = 32 * c + 8 * g;
          f32x4 v = {0.f, 0.f, 0.f, 0.f};
          if (SEED_EARLY && kb > 0 && dd < HD) v = *reinterpret_cast<const f32x4*>(dqrow + dd);
          dq[c][4 * g] = v.x; dq[c][4 * g + 1] = v.y; dq[c][4 * g + 2] = v.z; dq[c][4 * g + 3] = v.w;
        }
      __builtin_amdgcn_wave_barrier();
      frag_to_lds<HD>(tO, of, li, hh);
      frag_to_lds<HD>(tQ, qf, li, hh);
      f32x16 s = mm_frag<HD>(qf, kf);                  // S: row = query, col = key
      f32x16 dp = mm_frag<HD>(of, vf);                 // dP: row = query, col = key
      if constexpr (DS == 2) {                         // whole-head S and dP from the two halves
        exchange(s);
        exchange(dp);
      }
      if (qb + 1 < nqb) load_qblock(q0 + 32);          // prefetch the next query block
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        // selected positions read here, not with the row stats: 16 registers fewer across the S / dP
        // chains (the DS = 2 selected-query variant spilled 19 registers holding them)
        i32x4 qv = {0, 0, 0, 0};
        if constexpr (SEL) qv = *reinterpret_cast<const i32x4*>(qpp + q0 + 8 * g + 4 * hh);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * g + e, j = q0 + 8 * g + 4 * hh + e;
          const float ex = __expf(s[r] * p.scale - l4[g][e]);
          const int qposj = SEL ? qv[e] : q_off + j;
          const float P = kpos <= qposj ? ex : 0.f;
          s[r] = P;
          dp[r] = P * (dp[r] - d4[g][e]) * p.scale;    // dS, pre-scaled by 1/sqrt(hd)
          tS[(8 * g + 4 * hh + e) * SLD + li] = dp[r];
        }
      }
      __builtin_amdgcn_wave_barrier();
      if constexpr (HD <= 32) {
        // dV^T += dO^T P and dK^T += Q^T dS: all 32 LDS operands read first, then the two chains
        // interleaved (independent accumulators) — no LDS round trip between consecutive MFMAs
        float ao[16], aq[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = acc_row(r, hh);
          ao[r] = li < HD ? tO[row * LD + li] : 0.f;
          aq[r] = li < HD ? tQ[row * LD + li] : 0.f;
        }
        __builtin_amdgcn_sched_barrier(0);             // keep the reads above: the scheduler sinks them
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          dv[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(ao[r], s[r], dv[0], 0, 0, 0);
          dk[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(aq[r], dp[r], dk[0], 0, 0, 0);
        }
        float bk[16];
        f32x4 a4[4];
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) a4[q4] = *reinterpret_cast<const f32x4*>(tS + li * SLD + 16 * hh + 4 * q4);
#pragma unroll
        for (int e = 0; e < 16; ++e) bk[e] = li < HD ? tK[(16 * hh + e) * LD + li] : 0.f;
        __builtin_amdgcn_sched_barrier(0);
        // dQ^T[d][q] += sum_key K[key][d] dS[q][key]: A = K^T (row = dim, k = key, from tK),
        // B = dS^T (k = key 16hh + s, col = query = lane, from tS)
#pragma unroll
        for (int e = 0; e < 16; ++e) dq[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(bk[e], a4[e >> 2][e & 3], dq[0], 0, 0, 0);
      } else {
        acc_tile_p<HD>(dv, tO, s, li, hh);             // dV^T += dO^T P
        acc_tile_p<HD>(dk, tQ, dp, li, hh);            // dK^T += Q^T dS
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
          const f32x4 a4 = *reinterpret_cast<const f32x4*>(tS + li * SLD + 16 * hh + 4 * q4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int key = 16 * hh + 4 * q4 + e;
#pragma unroll
            for (int c = 0; c < NB(HD); ++c) {
              const int dd = 32 * c + li;
              const float bkv = dd < HD ? tK[key * LD + dd] : 0.f;
              dq[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(bkv, a4[e], dq[c], 0, 0, 0);
            }
          }
        }
      }
      if (jq < K) {                                      // the running dQ partial
#pragma unroll
        for (int c = 0; c < NB(HD); ++c)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int dd = 32 * c + 8 * g;
            if (dd >= HD) continue;
            f32x4 v = {dq[c][4 * g], dq[c][4 * g + 1], dq[c][4 * g + 2], dq[c][4 * g + 3]};
            if (!SEED_EARLY && kb > 0) v = *reinterpret_cast<const f32x4*>(dqrow + dd) + v;
            *reinterpret_cast<f32x4*>(dqrow + dd) = v;
          }
      }
    }
    if (kpos < I) {
#pragma unroll
      for (int c = 0; c < NB(HD); ++c)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int dd = 32 * c + 8 * g + 4 * hh;
          if (dd < HD) {
            f32x4 a = {dk[c][4 * g], dk[c][4 * g + 1], dk[c][4 * g + 2], dk[c][4 * g + 3]};
            f32x4 v = {dv[c][4 * g], dv[c][4 * g + 1], dv[c][4 * g + 2], dv[c][4 * g + 3]};
            *reinterpret_cast<f32x4*>(dK + (int64_t)kpos * p.ld + dd) = a;
            *reinterpret_cast<f32x4*>(dV + (int64_t)kpos * p.ld + dd) = v;
          }
        }
    }
  }
}

// ------------------------------------------------------------------------------------------
// bf16 backward (TERMS = 1, OT_MATMUL_BF16; the kernel also builds with TERMS = 6 split planes, which
// measured slower than attn_bwd_kernel and is not dispatched).
// Same pass structure as attn_bwd_kernel (one wave per (sample, head), key blocks outer, the query
// blocks that see them inner, dQ partial read-modify-written in dqkv), all five products on
// v_mfma_f32_32x32x16_bf16:
//   S = Q K^T, dP = dO V^T        A = Q / dO (lane = query), B = K / V (lane = key): register planes
//   dV^T += dO^T P, dK^T += Q^T dS  A = dO^T / Q^T via ds_read_b64_tr_b16 from the wave's row-major
//                                  [query][dim] plane images (k = query in the accumulator order of
//                                  P / dS, which are the B operands straight from the registers)
//   dQ^T += K^T dS^T              A = K^T from the [key][dim] image, B = dS^T from a [key][query]
//                                  image the lanes write as 8-byte runs (k = key, natural order)
// K and V fragments (the B operands of S and dP) are re-read from the wave's [key][dim] plane images
// each pair instead of living in registers for the whole key block: at HD 64 the kernel fits 256
// registers, i.e. 2 waves / SIMD instead of 1 (C5 backward 17.4 -> see DESIGN.md).
// Planes: 3 (split, TERMS = 6) or 1 (bf16).  LDS per wave: (4 x 32 x HD + 32 x 32) x 2 B x planes.

// two ds_read_b64_tr_b16 reads -> one 32x32x16 operand fragment: elements 0-3 from rows ra .. ra+3,
// 4-7 from rows rb .. rb+3, the lane's column colbase + (lane & 31) (row stride rs bytes)
__device__ __forceinline__ u32x4 tr16_frag(const char* img, int rs, int ra, int rb, int colbase, int lane) {
  typedef short v4i16 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) v4i16 lds_v4i16;
  const int gi = lane & 15, q = gi >> 2, pp = gi & 3;
  const int c = colbase + 16 * ((lane >> 4) & 1) + 4 * pp;
  const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(img + (ra + q) * rs + c * 2));
  const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(img + (rb + q) * rs + c * 2));
  const u32x2 a = __builtin_bit_cast(u32x2, lo), b = __builtin_bit_cast(u32x2, hi);
  return u32x4{a.x, a.y, b.x, b.y};
}

template <int HD, int TERMS>
constexpr int BWDS_LDS() { return (TERMS == 1 ? 1 : 3) * (4 * 32 * HD + 32 * 32) * 2; }

template <int HD, int TERMS, bool SEL, int WAVES>
__global__ __launch_bounds__(64 * WAVES, TERMS == 1 ? 2 : 1) void attn_bwd_split_kernel(AttnArgs p) {
  static_assert(HD == 32 || HD == 64, "split backward: HD 32 or 64");
  constexpr int NPL = TERMS == 1 ? 1 : 3;
  constexpr int NS = HD / 16;                          // k-steps over the head dim
  constexpr int IMG = 32 * HD * 2;                     // bytes of one [32][HD] plane image
  constexpr int SIMG = 32 * 32 * 2;                    // bytes of one [32 keys][32 queries] plane
  extern __shared__ __attribute__((aligned(16))) char lds_b[];
  const int lane = threadIdx.x & 63, li = lane & 31, hh = lane >> 5;
  char* kimg = lds_b + (threadIdx.x >> 6) * BWDS_LDS<HD, TERMS>();
  char* qimg = kimg + NPL * IMG;
  char* oimg = qimg + NPL * IMG;
  char* simg = oimg + NPL * IMG;
  char* vimg = simg + NPL * SIMG;
  const int pair = blockIdx.x * WAVES + (threadIdx.x >> 6);
  if (pair >= p.B * p.H) return;                       // wave-uniform
  const int b = pair / p.H, h = pair % p.H;
  const int I = p.I, K = p.K, q_off = I - K, KP = attn_kpad(K);
  const int64_t tok0 = (int64_t)b * I;
  const float* Q = p.qkv + tok0 * p.ld + h * HD;
  const float* Kp = Q + p.d;
  const float* V = Q + 2 * p.d;
  const float* dO = p.dout + (int64_t)b * K * p.d + h * HD;
  const float* lsep = p.delta + (int64_t)pair * KP;
  const float* dltp = p.delta + ((int64_t)p.B * p.H + pair) * KP;
  const int32_t* qpp = reinterpret_cast<const int32_t*>(p.delta + 2 * (int64_t)p.B * p.H * KP) + (int64_t)b * KP;
  float* dK = p.dqkv + tok0 * p.ld + p.d + h * HD;
  float* dV = dK + p.d;
  const int nqb = KP / 32;
  const int nkb = (I + 31) / 32;
  auto qrow = [&](int j) { return SEL ? qpp[j < KP ? j : KP - 1] : q_off + (j < K ? j : K - 1); };

  for (int kb = 0; kb < nkb; ++kb) {
    const int key0 = 32 * kb;
    const int kpos = key0 + li;
    {
      float kf[HD / 2], vf[HD / 2];
      load_frag<HD>(kf, Kp, p.ld, kpos, I, hh);        // rows >= I: zeros (masked below)
      load_frag<HD>(vf, V, p.ld, kpos, I, hh);
#pragma unroll
      for (int t = 0; t < NS; ++t) {
        u32x4 kB[3], vB[3];
        split8t<TERMS>(kf + 8 * t, kB);
        split8t<TERMS>(vf + 8 * t, vB);
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) {
          *reinterpret_cast<u32x4*>(kimg + pl * IMG + (li * HD + (HD / 2) * hh + 8 * t) * 2) = kB[pl];
          *reinterpret_cast<u32x4*>(vimg + pl * IMG + (li * HD + (HD / 2) * hh + 8 * t) * 2) = vB[pl];
        }
      }
    }
    f32x16 dk[NB(HD)], dv[NB(HD)];
#pragma unroll
    for (int c = 0; c < NB(HD); ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) { dk[c][r] = 0.f; dv[c][r] = 0.f; }
    int qb0;
    if constexpr (SEL) {
      qb0 = 0;
      while (qb0 < nqb - 1 && qpp[32 * qb0 + 31] < key0) ++qb0;
    } else {
      qb0 = key0 - q_off; qb0 = qb0 < 0 ? 0 : qb0 / 32;
    }
    for (int qb = qb0; qb < nqb; ++qb) {
      const int q0 = 32 * qb;
      const int jq = q0 + li;
      // Q / dO rows of this lane's query: register planes (A of S / dP) and the plane images
      u32x4 qA[NS][3], oA[NS][3];
      {
        float qf[HD / 2], of[HD / 2];
        if constexpr (SEL) load_frag<HD>(qf, Q, p.ld, jq < K ? qpp[jq] : I, I, hh);
        else load_frag<HD>(qf, Q, p.ld, jq < K ? q_off + jq : I, I, hh);
        load_frag<HD>(of, dO, p.d, jq, K, hh);
#pragma unroll
        for (int t = 0; t < NS; ++t) {
          split8t<TERMS>(qf + 8 * t, qA[t]);
          split8t<TERMS>(of + 8 * t, oA[t]);
#pragma unroll
          for (int pl = 0; pl < NPL; ++pl) {
            *reinterpret_cast<u32x4*>(qimg + pl * IMG + (li * HD + (HD / 2) * hh + 8 * t) * 2) = qA[t][pl];
            *reinterpret_cast<u32x4*>(oimg + pl * IMG + (li * HD + (HD / 2) * hh + 8 * t) * 2) = oA[t][pl];
          }
        }
      }
      f32x16 s, dp;
#pragma unroll
      for (int r = 0; r < 16; ++r) { s[r] = 0.f; dp[r] = 0.f; }
#pragma unroll
      for (int t = 0; t < NS; ++t) {
        u32x4 kB[3], vB[3];                              // this lane's key row, dims 8t.. (its own writes)
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) {
          kB[pl] = *reinterpret_cast<const u32x4*>(kimg + pl * IMG + (li * HD + (HD / 2) * hh + 8 * t) * 2);
          vB[pl] = *reinterpret_cast<const u32x4*>(vimg + pl * IMG + (li * HD + (HD / 2) * hh + 8 * t) * 2);
        }
        s = mfma_terms<TERMS>(qA[t], kB, s);            // S: row = query, col = key
        dp = mfma_terms<TERMS>(oA[t], vB, dp);          // dP
      }
      // softmax gradient (rows = queries acc_row(r, hh), column = this lane's key)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 l4 = *reinterpret_cast<const f32x4*>(lsep + q0 + 8 * g + 4 * hh);
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(dltp + q0 + 8 * g + 4 * hh);
        i32x4 qv4;
        if constexpr (SEL) qv4 = *reinterpret_cast<const i32x4*>(qpp + q0 + 8 * g + 4 * hh);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * g + e, j = q0 + 8 * g + 4 * hh + e;
          const int qposj = SEL ? qv4[e] : q_off + j;
          const float ex = __expf(s[r] * p.scale - l4[e]);
          const float P = kpos <= qposj ? ex : 0.f;
          s[r] = P;
          dp[r] = P * (dp[r] - d4[e]) * p.scale;         // dS, pre-scaled by 1/sqrt(hd)
        }
      }
      u32x4 pB[2][3], sB[2][3];
      {
        float pv[16], sv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) { pv[r] = s[r]; sv[r] = dp[r]; }
        split8t<TERMS>(pv, pB[0]); split8t<TERMS>(pv + 8, pB[1]);
        split8t<TERMS>(sv, sB[0]); split8t<TERMS>(sv + 8, sB[1]);
        // dS^T image [key][query]: this lane's key row, registers 4g .. 4g+3 = queries 8g + 4hh + 0..3
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const u32x4 w = sB[g >> 1][pl];
            const u32x2 two = (g & 1) ? u32x2{w.z, w.w} : u32x2{w.x, w.y};
            *reinterpret_cast<u32x2*>(simg + pl * SIMG + (li * 32 + 8 * g + 4 * hh) * 2) = two;
          }
      }
      __builtin_amdgcn_wave_barrier();
      // dV^T += dO^T P, dK^T += Q^T dS  (k = query, accumulator order)
#pragma unroll
      for (int c = 0; c < NB(HD); ++c)
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          u32x4 oT[3], qT[3];
#pragma unroll
          for (int pl = 0; pl < NPL; ++pl) {
            oT[pl] = tr16_frag(oimg + pl * IMG, HD * 2, 16 * st + 4 * hh, 16 * st + 8 + 4 * hh, 32 * c, lane);
            qT[pl] = tr16_frag(qimg + pl * IMG, HD * 2, 16 * st + 4 * hh, 16 * st + 8 + 4 * hh, 32 * c, lane);
          }
          dv[c] = mfma_terms<TERMS>(oT, pB[st], dv[c]);
          dk[c] = mfma_terms<TERMS>(qT, sB[st], dk[c]);
        }
      // dQ^T += K^T dS^T  (k = key, natural order)
      f32x16 dq[NB(HD)];
#pragma unroll
      for (int c = 0; c < NB(HD); ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r) dq[c][r] = 0.f;
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        u32x4 sT[3];
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl)
          sT[pl] = tr16_frag(simg + pl * SIMG, 64, 16 * st + 8 * hh, 16 * st + 8 * hh + 4, 0, lane);
#pragma unroll
        for (int c = 0; c < NB(HD); ++c) {
          u32x4 kT[3];
#pragma unroll
          for (int pl = 0; pl < NPL; ++pl)
            kT[pl] = tr16_frag(kimg + pl * IMG, HD * 2, 16 * st + 8 * hh, 16 * st + 8 * hh + 4, 32 * c, lane);
          dq[c] = mfma_terms<TERMS>(kT, sT, dq[c]);
        }
      }
      __builtin_amdgcn_wave_barrier();                   // the images are rewritten by the next pair
      if (jq < K) {                                      // the running dQ partial (single owner)
        float* dqrow = p.dqkv + (tok0 + qrow(jq)) * p.ld + h * HD + 4 * hh;
#pragma unroll
        for (int c = 0; c < NB(HD); ++c)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int dd = 32 * c + 8 * g;
            f32x4 v = {dq[c][4 * g], dq[c][4 * g + 1], dq[c][4 * g + 2], dq[c][4 * g + 3]};
            if (kb > 0) v = *reinterpret_cast<const f32x4*>(dqrow + dd) + v;
            *reinterpret_cast<f32x4*>(dqrow + dd) = v;
          }
      }
    }
    if (kpos < I) {
#pragma unroll
      for (int c = 0; c < NB(HD); ++c)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int dd = 32 * c + 8 * g + 4 * hh;
          f32x4 a = {dk[c][4 * g], dk[c][4 * g + 1], dk[c][4 * g + 2], dk[c][4 * g + 3]};
          f32x4 v = {dv[c][4 * g], dv[c][4 * g + 1], dv[c][4 * g + 2], dv[c][4 * g + 3]};
          *reinterpret_cast<f32x4*>(dK + (int64_t)kpos * p.ld + dd) = a;
          *reinterpret_cast<f32x4*>(dV + (int64_t)kpos * p.ld + dd) = v;
        }
    }
  }
}

// Key-grouped bf16 backward for long tails (C5: 33 key blocks per (sample, head)).  The per-pair
// kernel above walks every key block with one wave and re-reads the (sample, head)'s Q / dO rows and
// read-modify-writes its dQ rows once per key block — at L = 1036 that is ~70 GB of L2-missing
// traffic per layer.  Here a workgroup of NW waves owns NW consecutive key blocks (one per wave: dK /
// dV accumulators in registers) and streams the query blocks once: each query block's Q / dO rows are
// loaded by the whole workgroup into shared bf16 images (the next block's loads in flight during the
// current block's MFMAs), every wave runs S / dP / softmax gradient / dV / dK for its key block, and
// the NW dQ contributions are summed through LDS in a fixed order and stored once per (slice, query
// block) — slice 0 into dqkv, slice s > 0 into dqpart[s - 1] (attn_dq_reduce_kernel adds them).
// Tail queries only (no selection map), TERMS = 1 (OT_MATMUL_BF16).
// XCD-aware slice placement: measured 4,523 us per C5 layer against 4,489 us without (within noise; the
// slices' Q / dO re-reads are not the bound) — kept as an option, off
#ifndef OT_BWDG_XCD
#define OT_BWDG_XCD 0
#endif
// Descending query blocks: every slice of a (sample, head) then streams the same query block at once (with
// OT_BWDG_XCD the slices share one L2; the kernel re-reads Q / dO once per slice, ~12 GB per C5 layer): 4,330 us
// against 4,387-4,489 us ascending (runs/r6ab.sh) — not kept: dK / dV would no longer sum the query blocks in the
// one-wave-per-pair backward's order (bit-identity, test_attn_bwd_key_slices) for ~0.3% of a C5 step
#ifndef OT_BWDG_DESC
#define OT_BWDG_DESC 0
#endif
// Cross-wave dQ (head_dim 64, 4 waves): after a barrier that publishes every wave's dS^T image, wave w forms dQ^T
// tile w & 1 over key blocks 2 (w >> 1) and 2 (w >> 1) + 1 of the group, and waves 2 / 3 hand theirs to waves 0 / 1
// through an 8 KiB buffer (a third barrier) — the [NW][2][4][64][4] f32 buffer (32 KiB) and its reduce pass go, LDS
// 64 -> 40 KiB per workgroup.  C5 layer (tools/attn_c5_bench.py, runs/r6ad.sh): 4,228-4,240 us against 4,405-4,435;
// dQ sums its four key blocks as (kb0 + kb1) + (kb2 + kb3) instead of one fixed-order pass (dK / dV unchanged, bit for
// bit).  Three workgroups per CU (OT_BWDG_MINWG 3, 168 VGPRs) spill 344 B per lane: 13.5 ms — two kept.
#ifndef OT_BWDG_DQX
#define OT_BWDG_DQX 1
#endif
#ifndef OT_BWDG_MINWG
#define OT_BWDG_MINWG 2
#endif
template <int HD, int NW>
constexpr bool bwdg_dqx() { return OT_BWDG_DQX && HD == 64 && (NW == 4 || NW == 8); }
template <int HD, int NW>
constexpr int BWDG_LDS() {
  return 2 * 32 * HD * 2 + NW * (32 * HD * 2 + 32 * 32 * 2) + (bwdg_dqx<HD, NW>() ? (NW - 2) * 64 * 16 * 4 : NW * 32 * HD * 4);
}

template <int HD, int NW, bool QB = false>
__global__ __launch_bounds__(64 * NW, NW >= 8 ? 1 : (bwdg_dqx<HD, NW>() ? OT_BWDG_MINWG : 2)) void attn_bwd_group_kernel(AttnArgs p) {
  constexpr bool DQX = bwdg_dqx<HD, NW>();
  static_assert(HD == 64 || HD == 32, "grouped backward: HD 32 or 64");
  constexpr int NS = HD / 16;                          // k-steps over the head dim
  constexpr int IMG = 32 * HD * 2;                     // one [32][HD] bf16 image
  constexpr int SIMG = 32 * 32 * 2;
  constexpr int NT = 64 * NW;
  constexpr int F4 = 32 * HD / 4;                      // float4 per [32][HD] block
  constexpr int PT = (F4 + NT - 1) / NT;               // float4 per thread per operand
  extern __shared__ __attribute__((aligned(16))) char lds_g[];
  // the wave index in a scalar register: the key-block conditions below are wave-uniform branches
  const int t = threadIdx.x, lane = t & 63, li = lane & 31, hh = lane >> 5, w = __builtin_amdgcn_readfirstlane(t >> 6);
  char* qimg = lds_g;                                  // shared [query][dim] images of the query block
  char* oimg = qimg + IMG;
  char* kimg = oimg + IMG + w * (IMG + SIMG);          // this wave's key block (its V fragments stay in registers)
  char* simg = kimg + IMG;                             // this wave's dS^T [key][query]
  float* dqbuf = reinterpret_cast<float*>(lds_g + 2 * IMG + NW * (IMG + SIMG));   // [NW][NB][4][64 lanes][4]
  const int S = p.kslices;
  // the S slices of one (sample, head) read the same query / dO blocks: consecutive logical ids on one XCD
  const int wg = OT_BWDG_XCD ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int pair = wg / S, slice = wg - pair * S;
  const int b = pair / p.H, h = pair % p.H;
  const int I = p.I, K = p.K, q_off = I - K, KP = attn_kpad(K);
  const int64_t tok0 = (int64_t)b * I;
  const float* Q = p.qkv + tok0 * p.ld + h * HD;
  const float* Kp = Q + p.d;
  const float* V = Q + 2 * p.d;
  const float* dO = p.dout + (int64_t)b * K * p.d + h * HD;
  const float* lsep = p.delta + (int64_t)pair * KP;
  const float* dltp = p.delta + ((int64_t)p.B * p.H + pair) * KP;
  float* dK = p.dqkv + tok0 * p.ld + p.d + h * HD;
  float* dV = dK + p.d;
  const int nqb = KP / 32;
  const int kb = slice * NW + w;                       // this wave's key block (>= nkb: an idle wave, P = 0)
  const int key0 = 32 * kb;
  const int kpos = key0 + li;
  const uint16_t* Q16 = reinterpret_cast<const uint16_t*>(p.qkv) + tok0 * p.ld + h * HD;
  // this lane's K / V fragments (row li, dims (HD / 2) hh + 8 st ..) for every query block: held in registers
  u32x4 kF[NS], vF[NS];
  if constexpr (QB) {                                  // bf16 operands: the images are copies
    const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      const int64_t o = (int64_t)kpos * p.ld + (HD / 2) * hh + 8 * st;
      const u32x4 kB = kpos < I ? *reinterpret_cast<const u32x4*>(Q16 + p.d + o) : z;
      const u32x4 vB = kpos < I ? *reinterpret_cast<const u32x4*>(Q16 + 2 * p.d + o) : z;
      *reinterpret_cast<u32x4*>(kimg + gswz<HD * 2>(li, ((HD / 2) * hh + 8 * st) * 2)) = kB;
      kF[st] = kB;
      vF[st] = vB;
    }
  } else {
    float kf[HD / 2], vf[HD / 2];
    load_frag<HD>(kf, Kp, p.ld, kpos, I, hh);          // rows >= I: zeros (masked below)
    load_frag<HD>(vf, V, p.ld, kpos, I, hh);
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      u32x4 kB[3], vB[3];
      split8t<1>(kf + 8 * st, kB);
      split8t<1>(vf + 8 * st, vB);
      *reinterpret_cast<u32x4*>(kimg + gswz<HD * 2>(li, ((HD / 2) * hh + 8 * st) * 2)) = kB[0];
      kF[st] = kB[0];
      vF[st] = vB[0];
    }
  }
  f32x16 dk[NB(HD)], dv[NB(HD)];
#pragma unroll
  for (int c = 0; c < NB(HD); ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) { dk[c][r] = 0.f; dv[c][r] = 0.f; }
  int qbs = 32 * slice * NW - q_off;                   // first query block that sees the group's first key
  qbs = qbs < 0 ? 0 : qbs / 32;
  // cooperative Q / dO block loads: thread t takes float4 e = t + NT i of the [32][HD] block
  f32x4 pq[PT], po[PT];
  u32x2 pq16[PT];
  // the block's lse (lanes 0-31) and delta (lanes 32-63), one float per lane, loaded with the Q / dO rows and
  // parked in the wave's dS^T image until the softmax reads them (that image is rewritten only after it)
  float plsd = 0.f;
  auto load_q = [&](int qb) {
    plsd = lane < 32 ? lsep[32 * qb + lane] : dltp[32 * qb + lane - 32];
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int e = t + NT * i;
      const int row = e / (HD / 4), c4 = e % (HD / 4);
      const int j = 32 * qb + row;
      const int jj = j < K ? j : K - 1;                // padded queries: a real row (lse = +inf masks it)
      if constexpr (QB)
        pq16[i] = e < F4 ? *reinterpret_cast<const u32x2*>(Q16 + (int64_t)(q_off + jj) * p.ld + 4 * c4) : u32x2{0u, 0u};
      else
        pq[i] = e < F4 ? *reinterpret_cast<const f32x4*>(Q + (int64_t)(q_off + jj) * p.ld + 4 * c4) : f32x4{0.f, 0.f, 0.f, 0.f};
      po[i] = e < F4 ? *reinterpret_cast<const f32x4*>(dO + (int64_t)jj * p.d + 4 * c4) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto store_q = [&]() {
    reinterpret_cast<float*>(simg)[lane] = plsd;
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int e = t + NT * i;
      if (e < F4) {
        const int io = gswz<HD * 2>(e / (HD / 4), (e % (HD / 4)) * 8);
        if constexpr (QB) *reinterpret_cast<u32x2*>(qimg + io) = pq16[i];
        else *reinterpret_cast<u32x2*>(qimg + io) = bf16_rne4(pq[i]);
        *reinterpret_cast<u32x2*>(oimg + io) = bf16_rne4(po[i]);
      }
    }
  };
  const int nit = nqb - qbs;
  load_q(OT_BWDG_DESC ? nqb - 1 : qbs);
  for (int it = 0; it < nit; ++it) {
    const int qb = OT_BWDG_DESC ? nqb - 1 - it : qbs + it;
    const int q0 = 32 * qb;
    store_q();
    __syncthreads();                                   // images of block qb (and the previous reduce done)
    if (it + 1 < nit) load_q(OT_BWDG_DESC ? qb - 1 : qb + 1);   // in flight during this block's MFMAs
    // a wave whose key block lies wholly after this query block (or past the end) contributes zeros
    if (key0 > q_off + q0 + 31 || key0 >= I) {
      if constexpr (!DQX) {
#pragma unroll
        for (int c = 0; c < NB(HD); ++c)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<f32x4*>(dqbuf + (((w * NB(HD) + c) * 4 + g) * 64 + lane) * 4) = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    } else {
    u32x4 qA[NS][3], oA[NS][3];
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      qA[st][0] = *reinterpret_cast<const u32x4*>(qimg + gswz<HD * 2>(li, ((HD / 2) * hh + 8 * st) * 2));
      oA[st][0] = *reinterpret_cast<const u32x4*>(oimg + gswz<HD * 2>(li, ((HD / 2) * hh + 8 * st) * 2));
    }
    f32x16 s, dp;
#pragma unroll
    for (int r = 0; r < 16; ++r) { s[r] = 0.f; dp[r] = 0.f; }
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      u32x4 kB[3], vB[3];
      kB[0] = kF[st];
      vB[0] = vF[st];
      s = mfma_terms<1>(qA[st], kB, s);                // S: row = query, col = key
      dp = mfma_terms<1>(oA[st], vB, dp);              // dP
    }
    // the causal mask only where the block pair straddles the diagonal (or holds keys past I): a wholly visible
    // pair skips the per-element compare / select (padded queries have lse = +inf: P = 0 either way)
    if (key0 + 31 <= q_off + q0) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 l4 = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(simg) + 8 * g + 4 * hh);
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(simg) + 32 + 8 * g + 4 * hh);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * g + e;
          const float P = __expf(s[r] * p.scale - l4[e]);
          s[r] = P;
          dp[r] = P * (dp[r] - d4[e]) * p.scale;        // dS, pre-scaled by 1/sqrt(hd)
        }
      }
    } else {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 l4 = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(simg) + 8 * g + 4 * hh);
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(simg) + 32 + 8 * g + 4 * hh);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * g + e, j = q0 + 8 * g + 4 * hh + e;
          const float ex = __expf(s[r] * p.scale - l4[e]);
          const float P = kpos <= q_off + j ? ex : 0.f;
          s[r] = P;
          dp[r] = P * (dp[r] - d4[e]) * p.scale;        // dS, pre-scaled by 1/sqrt(hd)
        }
      }
    }
    u32x4 pB[2][3], sB[2][3];
    {
      float pv[16], sv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) { pv[r] = s[r]; sv[r] = dp[r]; }
      split8t<1>(pv, pB[0]); split8t<1>(pv + 8, pB[1]);
      split8t<1>(sv, sB[0]); split8t<1>(sv + 8, sB[1]);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const u32x4 wv = sB[g >> 1][0];
        const u32x2 two = (g & 1) ? u32x2{wv.z, wv.w} : u32x2{wv.x, wv.y};
        *reinterpret_cast<u32x2*>(simg + gswz<64>(li, (8 * g + 4 * hh) * 2)) = two;
      }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int c = 0; c < NB(HD); ++c)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        u32x4 oT[3], qT[3];
        oT[0] = tr16_frag_sw<HD * 2>(oimg, 16 * st + 4 * hh, 16 * st + 8 + 4 * hh, 32 * c, lane);
        qT[0] = tr16_frag_sw<HD * 2>(qimg, 16 * st + 4 * hh, 16 * st + 8 + 4 * hh, 32 * c, lane);
        dv[c] = mfma_terms<1>(oT, pB[st], dv[c]);      // dV^T += dO^T P
        dk[c] = mfma_terms<1>(qT, sB[st], dk[c]);      // dK^T += Q^T dS
      }
    if constexpr (!DQX) {
    f32x16 dq[NB(HD)];
#pragma unroll
    for (int c = 0; c < NB(HD); ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) dq[c][r] = 0.f;
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      u32x4 sT[3];
      sT[0] = tr16_frag_sw<64>(simg, 16 * st + 8 * hh, 16 * st + 8 * hh + 4, 0, lane);
#pragma unroll
      for (int c = 0; c < NB(HD); ++c) {
        u32x4 kT[3];
        kT[0] = tr16_frag_sw<HD * 2>(kimg, 16 * st + 8 * hh, 16 * st + 8 * hh + 4, 32 * c, lane);
        dq[c] = mfma_terms<1>(kT, sT, dq[c]);           // dQ^T += K^T dS^T
      }
    }
#pragma unroll
    for (int c = 0; c < NB(HD); ++c)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<f32x4*>(dqbuf + (((w * NB(HD) + c) * 4 + g) * 64 + lane) * 4) =
            f32x4{dq[c][4 * g], dq[c][4 * g + 1], dq[c][4 * g + 2], dq[c][4 * g + 3]};
    }
    }
    // the dQ store of (slice, query block): float4 a = query jq, dims dd .. dd + 3
    auto store_dq = [&](const f32x4& a, int jq, int dd) {
      if (jq < K && dd < HD) {
        const int ps = p.dq_bf16 ? slice : slice - 1;  // dqpart slot (bf16 output: slice 0 too)
        const int64_t pe = ((int64_t)ps * p.B * K + (int64_t)b * K + jq) * p.d + h * HD + dd;
        if (p.dq_part16) {
          *reinterpret_cast<u32x2*>(reinterpret_cast<uint16_t*>(p.dqpart) + pe) = bf16_rne4(a);
        } else {
          float* dst = ps < 0 ? p.dqkv + (tok0 + q_off + jq) * p.ld + h * HD + dd : p.dqpart + pe;
          *reinterpret_cast<f32x4*>(dst) = a;
        }
      }
    };
    if constexpr (DQX) {
      __syncthreads();                                 // every wave's dS^T image is in LDS
      const int c = w & 1;
      f32x16 dq;
#pragma unroll
      for (int r = 0; r < 16; ++r) dq[r] = 0.f;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int v = 2 * (w >> 1) + j;                // key block v of the group (uniform)
        const int kv0 = 32 * (slice * NW + v);
        if (kv0 > q_off + q0 + 31 || kv0 >= I) continue;   // its dS is zero (no image written)
        const char* kimg_v = lds_g + 2 * IMG + v * (IMG + SIMG);
        const char* simg_v = kimg_v + IMG;
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          u32x4 sT[3], kT[3];
          sT[0] = tr16_frag_sw<64>(simg_v, 16 * st + 8 * hh, 16 * st + 8 * hh + 4, 0, lane);
          kT[0] = tr16_frag_sw<HD * 2>(kimg_v, 16 * st + 8 * hh, 16 * st + 8 * hh + 4, 32 * c, lane);
          dq = mfma_terms<1>(kT, sT, dq);              // dQ^T (dims 32c ..) += K_v^T dS_v^T
        }
      }
      float* xb = dqbuf;                               // [NW - 2][4][64 lanes][4]: waves w >= 2 -> wave w & 1
      if (w >= 2) {
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<f32x4*>(xb + (((w - 2) * 4 + g) * 64 + lane) * 4) =
              f32x4{dq[4 * g], dq[4 * g + 1], dq[4 * g + 2], dq[4 * g + 3]};
      }
      __syncthreads();
      if (w < 2) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          f32x4 a = f32x4{dq[4 * g], dq[4 * g + 1], dq[4 * g + 2], dq[4 * g + 3]};
#pragma unroll
          for (int k = 0; k < NW / 2 - 1; ++k)         // fixed order: key-block pairs 1, 2, ...
            a += *reinterpret_cast<const f32x4*>(xb + (((w + 2 * k) * 4 + g) * 64 + lane) * 4);
          store_dq(a, q0 + li, 32 * c + 8 * g + 4 * hh);
        }
      }
    } else {
      __syncthreads();                                 // every wave's dQ contribution is in LDS
      // fixed-order sum over the NW waves: float4 u = (lane, c, g) -> query q0 + (lane & 31), dims
      // 32c + 8g + 4 (lane >> 5) + 0..3; stored once per (slice, query block)
      for (int u = t; u < NB(HD) * 4 * 64; u += NT) {
        const int ln = u & 63, cg = u >> 6, c = cg >> 2, g = cg & 3;
        f32x4 a = {0.f, 0.f, 0.f, 0.f};
        for (int v = 0; v < NW; ++v) a += *reinterpret_cast<const f32x4*>(dqbuf + (((v * NB(HD) + c) * 4 + g) * 64 + ln) * 4);
        store_dq(a, q0 + (ln & 31), 32 * c + 8 * g + 4 * (ln >> 5));
      }
    }
  }
  if (kpos < I) {
#pragma unroll
    for (int c = 0; c < NB(HD); ++c)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int dd = 32 * c + 8 * g + 4 * hh;
        if (dd < HD) {
          f32x4 a = {dk[c][4 * g], dk[c][4 * g + 1], dk[c][4 * g + 2], dk[c][4 * g + 3]};
          f32x4 v = {dv[c][4 * g], dv[c][4 * g + 1], dv[c][4 * g + 2], dv[c][4 * g + 3]};
          if (p.dq_bf16) {
            uint16_t* dK16 = reinterpret_cast<uint16_t*>(p.dqkv) + tok0 * p.ld + p.d + h * HD;
            *reinterpret_cast<u32x2*>(dK16 + (int64_t)kpos * p.ld + dd) = bf16_rne4(a);
            *reinterpret_cast<u32x2*>(dK16 + p.d + (int64_t)kpos * p.ld + dd) = bf16_rne4(v);
          } else {
            *reinterpret_cast<f32x4*>(dK + (int64_t)kpos * p.ld + dd) = a;
            *reinterpret_cast<f32x4*>(dV + (int64_t)kpos * p.ld + dd) = v;
          }
        }
      }
  }
}

// dQ of the key-grouped backward: dqkv[q row] += sum over slices s = 1 .. S-1 whose first key block
// (kgroup * s) the query's block sees of dqpart[s - 1] (fixed slice order: deterministic).  One thread
// per float4 of the [B*K, d] tail dQ.
__global__ __launch_bounds__(256) void attn_dq_reduce_kernel(AttnArgs p) {
  const int64_t e4 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const int64_t n = (int64_t)p.B * p.K * p.d;
  if (e4 >= n) return;
  const int64_t row = e4 / p.d;
  const int col = (int)(e4 - row * p.d);
  const int b = (int)(row / p.K), j = (int)(row - (int64_t)b * p.K);
  const int q_off = p.I - p.K, qb = j / 32;
  const int o = p.dq_bf16 ? 0 : 1;                     // dqpart slot of slice s: s - o
  const uint16_t* part16 = reinterpret_cast<const uint16_t*>(p.dqpart);
  auto part = [&](int64_t i) -> f32x4 {
    if (!p.dq_part16) return *reinterpret_cast<const f32x4*>(p.dqpart + i);
    const u32x2 w = *reinterpret_cast<const u32x2*>(part16 + i);
    return f32x4{__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u), __uint_as_float(w.y << 16),
                 __uint_as_float(w.y & 0xffff0000u)};
  };
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  bool any = false;
  for (int s = 1; s < p.kslices; ++s) {
    const int f = 32 * p.kgroup * s - q_off;           // first query block that sees the slice's first key
    if ((f < 0 ? 0 : f / 32) > qb) break;              // later slices start later still
    acc += part((int64_t)(s - o) * n + e4);
    any = true;
  }
  const int64_t di = ((int64_t)b * p.I + q_off + j) * p.ld + col;
  if (p.dq_bf16) {
    const f32x4 d0 = part(e4);
    *reinterpret_cast<u32x2*>(reinterpret_cast<uint16_t*>(p.dqkv) + di) = bf16_rne4(any ? d0 + acc : d0);
    return;
  }
  if (!any) return;
  f32x4* dst = reinterpret_cast<f32x4*>(p.dqkv + di);
  *dst = *dst + acc;
}

// ------------------------------------------------------------------------------------------
// Backward for a short query tail (K <= SMALL_K, e.g. the last layer's single query after DCE):
// HBM-bound (read K/V rows, write dK/dV rows), so VALU instead of 32x32 MFMA tiles that would be
// 1/32 occupied.  One wave per (sample, head); HD/4 lanes per key (one float4 of dims each), 64/(HD/4)
// keys per pass; dot products reduced over the key's lanes with xor shuffles.  dQ partials are
// reduced over the wave's key slots at the end.
constexpr int SMALL_K = 4;

// KQ: the largest K the instance takes (1: the last layer's one query — a quarter of the registers, so more waves
// per SIMD keep more K / V rows in flight)
template <int HD, int KQ = SMALL_K>
__global__ __launch_bounds__(256) void attn_bwd_small_kernel(AttnArgs p) {
  constexpr int LPK = HD / 4, KPW = 64 / LPK;
  const int lane = threadIdx.x & 63, sub = lane % LPK, slot = lane / LPK;
  const int pair = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pair >= p.B * p.H) return;
  const int b = pair / p.H, h = pair % p.H;
  const int I = p.I, K = p.K, q_off = I - K;
  const int64_t tok0 = (int64_t)b * I;
  const float* Q = p.qkv + tok0 * p.ld + h * HD + 4 * sub;
  const float* Kp = Q + p.d;
  const float* V = Q + 2 * p.d;
  float* dK = p.dqkv + tok0 * p.ld + p.d + h * HD + 4 * sub;
  float* dV = dK + p.d;
  const int32_t* qp = p.qpos ? p.qpos + (int64_t)b * K : nullptr;
  float am = 0.f;                                      // max |stored dK / dV / dQ| (p.amax)
  f32x4 q[KQ], o[KQ], dq[KQ];
  float lse[KQ], delta[KQ];
  int qpos[KQ];
#pragma unroll
  for (int j = 0; j < KQ; ++j) {
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    q[j] = z; o[j] = z; dq[j] = z; lse[j] = 0.f; delta[j] = 0.f; qpos[j] = -1;
    if (j < K) {
      qpos[j] = query_pos(qp, q_off, j);
      q[j] = *reinterpret_cast<const f32x4*>(Q + (int64_t)qpos[j] * p.ld);
      o[j] = *reinterpret_cast<const f32x4*>(p.dout + ((int64_t)b * K + j) * p.d + h * HD + 4 * sub);
      lse[j] = p.delta[(int64_t)pair * attn_kpad(K) + j];
      delta[j] = p.delta[((int64_t)p.B * p.H + pair) * attn_kpad(K) + j];
    }
  }
  // each pass's K / V rows are loaded one pass ahead (two loads per lane in flight during a pass's math)
  f32x4 kvn = *reinterpret_cast<const f32x4*>(Kp + (int64_t)min(slot, I - 1) * p.ld);
  f32x4 vvn = *reinterpret_cast<const f32x4*>(V + (int64_t)min(slot, I - 1) * p.ld);
  for (int key0 = 0; key0 < I; key0 += KPW) {
    const int key = key0 + slot;
    const bool live = key < I;
    const int64_t ro = (int64_t)(live ? key : 0) * p.ld;
    const f32x4 kv = kvn, vv = vvn;
    if (key0 + KPW < I) {
      const int64_t rn = (int64_t)min(key + KPW, I - 1) * p.ld;
      kvn = *reinterpret_cast<const f32x4*>(Kp + rn);
      vvn = *reinterpret_cast<const f32x4*>(V + rn);
    }
    f32x4 dk = {0.f, 0.f, 0.f, 0.f}, dv = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < KQ; ++j) {
      if (j >= K) break;
      float sdot = q[j].x * kv.x + q[j].y * kv.y + q[j].z * kv.z + q[j].w * kv.w;
      float pdot = o[j].x * vv.x + o[j].y * vv.y + o[j].z * vv.z + o[j].w * vv.w;
#pragma unroll
      for (int off = 1; off < LPK; off <<= 1) {
        sdot += __shfl_xor(sdot, off, 64);
        pdot += __shfl_xor(pdot, off, 64);
      }
      const bool vis = live && key <= qpos[j];
      const float P = vis ? __expf(sdot * p.scale - lse[j]) : 0.f;
      const float ds = vis ? P * (pdot - delta[j]) * p.scale : 0.f;
      dv += P * o[j];
      dk += ds * q[j];
      dq[j] += ds * kv;
    }
    if (live) {
      if (p.dq_bf16) {                                 // bf16 dqkv (OT_ATTN_DQKV_BF16)
        uint16_t* dK16 = reinterpret_cast<uint16_t*>(p.dqkv) + tok0 * p.ld + p.d + h * HD + 4 * sub;
        *reinterpret_cast<u32x2*>(dK16 + ro) = bf16_rne4(dk);
        *reinterpret_cast<u32x2*>(dK16 + p.d + ro) = bf16_rne4(dv);
      } else {
        *reinterpret_cast<f32x4*>(dK + ro) = dk;
        *reinterpret_cast<f32x4*>(dV + ro) = dv;
      }
    }
    if (p.rowmax || p.amax) {                          // (uniform) magnitude bounds of the stored rows
      float rk = live ? amax4(0.f, dk) : 0.f, rv = live ? amax4(0.f, dv) : 0.f;
#pragma unroll
      for (int off = 1; off < LPK; off <<= 1) {
        rk = fmaxf(rk, __shfl_xor(rk, off, 64));
        rv = fmaxf(rv, __shfl_xor(rv, off, 64));
      }
      am = fmaxf(am, fmaxf(rk, rv));
      if (p.rowmax && live && sub == 0) {
        float* rr = p.rowmax + (tok0 + key) * 3 * p.H + h;
        rr[p.H] = rk;
        rr[2 * p.H] = rv;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < KQ; ++j) {
    if (j >= K) break;
    f32x4 v = dq[j];
#pragma unroll
    for (int off = LPK; off < 64; off <<= 1) {
      v.x += __shfl_xor(v.x, off, 64); v.y += __shfl_xor(v.y, off, 64);
      v.z += __shfl_xor(v.z, off, 64); v.w += __shfl_xor(v.w, off, 64);
    }
    if (slot == 0) {
      if (p.dq_bf16)
        *reinterpret_cast<u32x2*>(reinterpret_cast<uint16_t*>(p.dqkv) + (tok0 + qpos[j]) * p.ld + h * HD + 4 * sub) =
            bf16_rne4(v);
      else
        *reinterpret_cast<f32x4*>(p.dqkv + (tok0 + qpos[j]) * p.ld + h * HD + 4 * sub) = v;
    }
    if (p.rowmax || p.amax) {                          // (uniform) the dQ row's bound
      float rq = amax4(0.f, v);
#pragma unroll
      for (int off = 1; off < LPK; off <<= 1) rq = fmaxf(rq, __shfl_xor(rq, off, 64));
      am = fmaxf(am, rq);
      if (p.rowmax && slot == 0 && sub == 0) p.rowmax[(tok0 + qpos[j]) * 3 * p.H + h] = rq;
    }
  }
  if (p.amax) amax_flush(p.amax, am);
}

// Forward for a short query tail (K <= SMALL_K: the last layer's single query after DCE), the f32-accurate modes.
// HBM-bound (each K / V row read once; 2 K hd flops per row), so plain f32 FMAs on the VALU: the slice kernel's
// MFMA tiles would be 1/16 occupied and it would split all I K / V rows into planes for one query (as slow as a
// full layer).  One wave per (sample, head); HD/4 lanes per key (one float4 of dims each), 64/(HD/4) key slots
// per pass, each slot with its own online softmax (running max m, sum l, output o; scores in log2 units) over the
// keys it sees; the slots' states are merged at the end with xor shuffles (max, then rescaled sums).  Exact f32
// products — no split.
template <int HD, int KQ = SMALL_K>
__global__ __launch_bounds__(256) void attn_fwd_small_kernel(AttnArgs p) {
  constexpr int LPK = HD / 4, KPW = 64 / LPK;
  const int lane = threadIdx.x & 63, sub = lane % LPK, slot = lane / LPK;
  const int pair = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pair >= p.B * p.H) return;
  const int b = pair / p.H, h = pair % p.H;
  const int I = p.I, K = p.K, q_off = I - K;
  const int64_t tok0 = (int64_t)b * I;
  const float* Q = p.qkv + tok0 * p.ld + h * HD + 4 * sub;
  const float* Kp = Q + p.d;
  const float* V = Q + 2 * p.d;
  const int32_t* qp = p.qpos ? p.qpos + (int64_t)b * K : nullptr;
  const float c = p.scale * 1.4426950408889634f;      // scores in log2 units
  f32x4 q[KQ], o[KQ];
  float m[KQ], l[KQ];
  int qpos[KQ];
#pragma unroll
  for (int j = 0; j < KQ; ++j) {
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    q[j] = z; o[j] = z; m[j] = -INFINITY; l[j] = 0.f; qpos[j] = -1;
    if (j < K) {
      qpos[j] = query_pos(qp, q_off, j);
      q[j] = *reinterpret_cast<const f32x4*>(Q + (int64_t)qpos[j] * p.ld) * c;
    }
  }
  int last = 0;                                        // keys past every query's position are never visible
#pragma unroll
  for (int j = 0; j < KQ; ++j)
    if (j < K) last = max(last, qpos[j]);
  f32x4 kvn = *reinterpret_cast<const f32x4*>(Kp + (int64_t)min(slot, last) * p.ld);   // one pass ahead
  f32x4 vvn = *reinterpret_cast<const f32x4*>(V + (int64_t)min(slot, last) * p.ld);
  for (int key0 = 0; key0 <= last; key0 += KPW) {
    const int key = key0 + slot;
    const bool live = key <= last;
    const f32x4 kv = kvn, vv = vvn;
    if (key0 + KPW <= last) {
      const int64_t rn = (int64_t)min(key + KPW, last) * p.ld;
      kvn = *reinterpret_cast<const f32x4*>(Kp + rn);
      vvn = *reinterpret_cast<const f32x4*>(V + rn);
    }
#pragma unroll
    for (int j = 0; j < KQ; ++j) {
      if (j >= K) break;
      float s = q[j].x * kv.x + q[j].y * kv.y + q[j].z * kv.z + q[j].w * kv.w;
#pragma unroll
      for (int off = 1; off < LPK; off <<= 1) s += __shfl_xor(s, off, 64);
      if (live && key <= qpos[j]) {                   // (uniform over the key's lanes)
        const float mn = fmaxf(m[j], s);
        const float corr = __builtin_amdgcn_exp2f(m[j] - mn), e = __builtin_amdgcn_exp2f(s - mn);
        l[j] = l[j] * corr + e;
        o[j] = o[j] * corr + e * vv;
        m[j] = mn;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < KQ; ++j) {
    if (j >= K) break;
    // merge the key slots (lanes sub + LPK * slot): max of m, then the rescaled l and o summed
    float mx = m[j];
#pragma unroll
    for (int off = LPK; off < 64; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
    const float corr = m[j] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m[j] - mx);
    float lt = l[j] * corr;
    f32x4 v = o[j] * corr;
#pragma unroll
    for (int off = LPK; off < 64; off <<= 1) {
      lt += __shfl_xor(lt, off, 64);
      v.x += __shfl_xor(v.x, off, 64); v.y += __shfl_xor(v.y, off, 64);
      v.z += __shfl_xor(v.z, off, 64); v.w += __shfl_xor(v.w, off, 64);
    }
    if (slot == 0) {
      *reinterpret_cast<f32x4*>(p.out + ((int64_t)b * K + j) * p.d + h * HD + 4 * sub) = v * (1.f / lt);
      if (sub == 0) p.lse[(int64_t)pair * K + j] = mx * 0.6931471805599453f + __logf(lt);
    }
  }
}

// ------------------------------------------------------------------------------------------
// Serving (paper §3.5.1 two-stage KV cache; the reference's broken cache path model.py:94-98,
// 359-381): candidate c of request req[c] attends with its last Kq N-side queries over the request's
// cached S-side keys/values (Ic rows, computed once per request) and its own n N-side rows.
// Absolute positions: cache rows 0..Ic-1, N rows Ic..Ic+n-1; query j sits at Ic + n - Kq + j, so
// every cached key is visible and the causal mask only touches the N-side key blocks.  Same
// orientation and online softmax as attn_fwd_kernel; key rows come from two sources, so each lane
// resolves its key row's address (one pointer per lane per key block).  Forward only (no lse).
struct AttnCachedArgs {
  const float* qkv; int64_t ld;            // N-side rows [C*n, ld]: q | k | v
  const float* kc; const float* vc; int64_t ldc;   // cached S-side K / V rows [R*Ic, ldc]
  const int32_t* req;                      // [C] request of each candidate
  float* out;                              // [C*Kq, d]
  int C, H, Ic, n, Kq, d;
  float scale;
};

template <int HD>
__device__ __forceinline__ void load_row_frag(float (&f)[HD / 2], const float* row, int hh) {
  if (row) {
    const float* q = row + (HD / 2) * hh;
#pragma unroll
    for (int i = 0; i < HD / 8; ++i) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(q + 4 * i);
      f[4 * i] = v.x; f[4 * i + 1] = v.y; f[4 * i + 2] = v.z; f[4 * i + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int s = 0; s < HD / 2; ++s) f[s] = 0.f;
  }
}

template <int HD>
__global__ __launch_bounds__(256) void attn_fwd_cached_kernel(AttnCachedArgs p) {
  __shared__ __attribute__((aligned(16))) float lds[4][32 * TLD<HD>()];
  const int lane = threadIdx.x & 63, li = lane & 31, hh = lane >> 5;
  float* tV = lds[threadIdx.x >> 6];
  const int pair = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pair >= p.C * p.H) return;
  const int c = pair / p.H, h = pair % p.H;
  const int Ic = p.Ic, n = p.n, Kq = p.Kq, L = Ic + n;
  const int64_t r = p.req[c];
  const float* Nq = p.qkv + (int64_t)c * n * p.ld + h * HD;        // this candidate's N rows
  const float* Ck = p.kc + r * Ic * p.ldc + h * HD;
  const float* Cv = p.vc + r * Ic * p.ldc + h * HD;
  const int q_off = L - Kq;                                         // absolute position of query 0
  const float qscale = p.scale * 1.4426950408889634f;
  const int nqb = (Kq + 31) / 32;
  for (int qb = 0; qb < nqb; ++qb) {
    const int j = 32 * qb + li;
    const int qpos = q_off + (j < Kq ? j : Kq - 1);
    float qf[HD / 2];
    load_row_frag<HD>(qf, Nq + (int64_t)(qpos - Ic) * p.ld, hh);
#pragma unroll
    for (int s = 0; s < HD / 2; ++s) qf[s] *= qscale;
    f32x16 oacc[NB(HD)];
#pragma unroll
    for (int cc = 0; cc < NB(HD); ++cc)
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) oacc[cc][rr] = 0.f;
    float m = -INFINITY, l = 0.f;
    const int last_q = q_off + min(32 * qb + 31, Kq - 1);
    const int nkb = last_q / 32 + 1;
    const int first_masked = (q_off + 32 * qb) / 32;
    for (int kb = 0; kb < nkb; ++kb) {
      const int key = 32 * kb + li;                 // this lane's key row (absolute position)
      const float* kr = nullptr;
      const float* vr = nullptr;
      if (key < Ic) {
        kr = Ck + (int64_t)key * p.ldc;
        vr = Cv + (int64_t)key * p.ldc;
      } else if (key < L) {
        kr = Nq + (int64_t)(key - Ic) * p.ld + p.d;
        vr = kr + p.d;
      }
      float kf[HD / 2], vf[HD / 2];
      load_row_frag<HD>(kf, kr, hh);
      load_row_frag<HD>(vf, vr, hh);
      frag_to_lds<HD>(tV, vf, li, hh);
      f32x16 s = mm_frag<HD>(kf, qf);               // S^T (log2 units): row = key, col = query
      if (kb >= first_masked) {
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) s[rr] = (32 * kb + acc_row(rr, hh) <= qpos) ? s[rr] : -INFINITY;
      }
      float mloc = s[0];
#pragma unroll
      for (int rr = 1; rr < 16; ++rr) mloc = fmaxf(mloc, s[rr]);
      mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
      const float mnew = fmaxf(m, mloc);
      const float corr = __builtin_amdgcn_exp2f(m - mnew);
      float lsum = 0.f;
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        const float e = __builtin_amdgcn_exp2f(s[rr] - mnew);
        s[rr] = e;
        lsum += e;
      }
      lsum += __shfl_xor(lsum, 32, 64);
      l = l * corr + lsum;
      m = mnew;
#pragma unroll
      for (int cc = 0; cc < NB(HD); ++cc) oacc[cc] *= corr;
      __builtin_amdgcn_wave_barrier();
      acc_tile_p<HD>(oacc, tV, s, li, hh);           // O^T += V^T P^T
      __builtin_amdgcn_wave_barrier();
    }
    if (j < Kq) {
      const float inv = 1.f / l;
      float* orow = p.out + ((int64_t)c * Kq + j) * p.d + h * HD;
#pragma unroll
      for (int cc = 0; cc < NB(HD); ++cc)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int dd = 32 * cc + 8 * g + 4 * hh;
          if (dd < HD) {
            f32x4 v = {oacc[cc][4 * g] * inv, oacc[cc][4 * g + 1] * inv, oacc[cc][4 * g + 2] * inv,
                       oacc[cc][4 * g + 3] * inv};
            *reinterpret_cast<f32x4*>(orow + dd) = v;
          }
        }
    }
  }
}

}  // namespace ot

using namespace ot;

// (KERNEL<HD, 1>: the one-query instance of a short-tail kernel)
#define OT_ATTN_DISPATCH_K1(KERNEL, HD_, ...)                                                \
  switch (HD_) {                                                                             \
    case 16: hipLaunchKernelGGL((KERNEL<16, 1>), __VA_ARGS__); break;                        \
    case 32: hipLaunchKernelGGL((KERNEL<32, 1>), __VA_ARGS__); break;                        \
    case 64: hipLaunchKernelGGL((KERNEL<64, 1>), __VA_ARGS__); break;                        \
    case 128: hipLaunchKernelGGL((KERNEL<128, 1>), __VA_ARGS__); break;                      \
    default: return fail(OT_ERR_UNSUPPORTED, "attention: head_dim %d unsupported", HD_);     \
  }
#define OT_ATTN_DISPATCH(KERNEL, HD_, ...)                                                   \
  switch (HD_) {                                                                             \
    case 16: hipLaunchKernelGGL(KERNEL<16>, __VA_ARGS__); break;                             \
    case 32: hipLaunchKernelGGL(KERNEL<32>, __VA_ARGS__); break;                             \
    case 64: hipLaunchKernelGGL(KERNEL<64>, __VA_ARGS__); break;                             \
    case 128: hipLaunchKernelGGL(KERNEL<128>, __VA_ARGS__); break;                           \
    default: return fail(OT_ERR_UNSUPPORTED, "attention: head_dim %d unsupported", HD_);     \
  }

extern "C" int ot_attn_fwd_cached(const float* qkv, int64_t ld, const float* kv_cache, int64_t ldc,
                                  const int32_t* req, int C, int H, int Ic, int n, int Kq, int head_dim,
                                  float* out, void* stream) {
  OT_REQUIRE(qkv && out && req && (Ic == 0 || kv_cache), "ot_attn_fwd_cached: null operand");
  OT_REQUIRE(C >= 0 && H > 0 && Ic >= 0 && n > 0 && Kq > 0 && Kq <= n, "ot_attn_fwd_cached: bad sizes C=%d Ic=%d n=%d Kq=%d",
             C, Ic, n, Kq);
  const int d = H * head_dim;
  OT_REQUIRE(ld % 4 == 0 && ld >= 3 * d && (Ic == 0 || (ldc % 4 == 0 && ldc >= 2 * d)),
             "ot_attn_fwd_cached: ld/ldc must hold k|v and be multiples of 4");
  if (C == 0) return OT_OK;
  AttnCachedArgs p{qkv, ld, kv_cache, kv_cache ? kv_cache + d : nullptr, ldc, req, out, C, H, Ic, n, Kq, d,
                   1.f / sqrtf((float)head_dim)};
  const unsigned grid = ceil_div((int64_t)C * H, 4);
  OT_ATTN_DISPATCH(attn_fwd_cached_kernel, head_dim, dim3(grid), dim3(256), 0, (hipStream_t)stream, p);
  OT_LAUNCH_CHECK("ot_attn_fwd_cached");
  return OT_OK;
}


static int attn_fwd_impl(const float* qkv, int64_t ld, int B, int H, int I, int K, const int32_t* qpos,
                         int head_dim, float* out, float* lse, int precision, void* stream, float* amax,
                         float* rowmax = nullptr);

extern "C" int ot_attn_fwd(const float* qkv, int64_t ld, int B, int H, int I, int K, const int32_t* qpos,
                           int head_dim, float* out, float* lse, int precision, void* stream) {
  return attn_fwd_impl(qkv, ld, B, H, I, K, qpos, head_dim, out, lse, precision, stream, nullptr);
}

extern "C" int ot_attn_amax_supported(int I, int K, int head_dim, int selected, int precision) {
  // the slice kernels fold max |output| in as they store: bit 1 the forward (O), bit 2 the backward (dQKV, tail
  // queries; its long forms reach I 544 at head_dim 64)
  if (precision != OT_MATMUL_SPLIT_BF16) return 0;
  if (K <= SMALL_K) return (head_dim == 32 || head_dim == 64 || head_dim == 128) ? 2 : 0;   // the short-tail backward
  return (attn_slice_fwd_supported(I, K, head_dim) ? 1 : 0) |
         (!selected && attn_slice_bwd_supported(I, K, head_dim, false) ? 2 : 0);
}

extern "C" int ot_attn_fwd_amax(const float* qkv, int64_t ld, int B, int H, int I, int K, const int32_t* qpos,
                                int head_dim, float* out, float* lse, float* amax, float* rowmax, int precision,
                                void* stream) {
  OT_REQUIRE((amax || rowmax) && (ot_attn_amax_supported(I, K, head_dim, qpos != nullptr, precision) & 1),
             "ot_attn_fwd_amax: the output bound needs the slice forward (split mode, I %d K %d head_dim %d: see "
             "ot_attn_amax_supported)", I, K, head_dim);
  return attn_fwd_impl(qkv, ld, B, H, I, K, qpos, head_dim, out, lse, precision, stream, amax, rowmax);
}

static int attn_fwd_impl(const float* qkv, int64_t ld, int B, int H, int I, int K, const int32_t* qpos,
                         int head_dim, float* out, float* lse, int precision, void* stream, float* amax,
                         float* rowmax) {
  OT_REQUIRE(precision == OT_MATMUL_F32 || precision == OT_MATMUL_SPLIT_BF16 || precision == OT_MATMUL_BF16,
             "ot_attn_fwd: unknown precision %d", precision);
  OT_REQUIRE(qkv && out && lse, "ot_attn_fwd: null operand");
  OT_REQUIRE(B >= 0 && H > 0 && I > 0 && K > 0 && K <= I, "ot_attn_fwd: bad sizes B=%d H=%d I=%d K=%d", B, H, I, K);
  OT_REQUIRE(ld % 4 == 0 && ld >= 3 * H * head_dim, "ot_attn_fwd: ld must be >= 3d and a multiple of 4");
  if (B == 0) return OT_OK;
  AttnArgs p{qkv, ld, H * head_dim, nullptr, nullptr, out, lse, nullptr, nullptr, B, H, I, K,
             1.f / sqrtf((float)head_dim), qpos};
  const size_t kv_bytes = 2 * (size_t)((I + 31) / 32 * 32) * (head_dim + 4) * sizeof(float);
  const bool kv_fits = head_dim <= 64 && kv_bytes <= OT_ATTN_KV_LDS_MAX && (K + 31) / 32 >= 3;
  const int mm = precision;
  if (mm != OT_MATMUL_BF16 && K <= SMALL_K && (head_dim == 32 || head_dim == 64 || head_dim == 128)) {
    // a short query tail (the last layer's one query): f32 VALU, HBM-bound
    if (K == 1) {
      OT_ATTN_DISPATCH_K1(attn_fwd_small_kernel, head_dim, dim3(ceil_div((int64_t)B * H, 4)), dim3(256), 0,
                       (hipStream_t)stream, p);
    } else {
      OT_ATTN_DISPATCH(attn_fwd_small_kernel, head_dim, dim3(ceil_div((int64_t)B * H, 4)), dim3(256), 0,
                       (hipStream_t)stream, p);
    }
    OT_LAUNCH_CHECK("ot_attn_fwd(small)");
    return OT_OK;
  }
  if (mm == OT_MATMUL_SPLIT_BF16 && attn_slice_fwd_supported(I, K, head_dim)) {
    // short sequence, f32-accurate: one workgroup per (sample, head) slice on split-bf16 MFMA
    return attn_slice_fwd(qkv, ld, B, H, I, K, qpos, head_dim, out, lse, (hipStream_t)stream, amax, rowmax);
  }
  if (head_dim >= 32 && (mm == OT_MATMUL_BF16 || (mm == OT_MATMUL_SPLIT_BF16 && !kv_fits && I > 256))) {
    // split-bf16: long sequences (I > 256), with the next key block prefetched (short ones stay on
    // the f32 kernels below, which measure faster there: profiles/r01/attention_split.md);
    // bf16 mode: one rounded plane, every length
    const unsigned grid = ceil_div((int64_t)B * H, 4);
    void (*kern)(AttnArgs) = nullptr;
    const bool one = mm == OT_MATMUL_BF16;
    switch (head_dim) {
      case 32: kern = one ? attn_fwd_split_kernel<32, 1> : attn_fwd_split_kernel<32, 6>; break;
      case 64: kern = one ? attn_fwd_split_kernel<64, 1> : attn_fwd_split_kernel<64, 6>; break;
      case 128: kern = one ? attn_fwd_split_kernel<128, 1> : attn_fwd_split_kernel<128, 6>; break;
      default: return fail(OT_ERR_UNSUPPORTED, "attention: head_dim %d unsupported", head_dim);
    }
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, (hipStream_t)stream, p);
  } else if (kv_fits) {
    // short sequence: K/V of a head staged once in LDS, shared by 4 waves
    static std::once_flag once;
    std::call_once(once, [] {
      for (const void* k : {(const void*)attn_fwd_kv_kernel<16>, (const void*)attn_fwd_kv_kernel<32>,
                            (const void*)attn_fwd_kv_kernel<64>})
        (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, OT_ATTN_KV_LDS_MAX);
      (void)hipGetLastError();
    });
    switch (head_dim) {
      case 16: hipLaunchKernelGGL(attn_fwd_kv_kernel<16>, dim3(B * H), dim3(256), kv_bytes, (hipStream_t)stream, p); break;
      case 32: hipLaunchKernelGGL(attn_fwd_kv_kernel<32>, dim3(B * H), dim3(256), kv_bytes, (hipStream_t)stream, p); break;
      default: hipLaunchKernelGGL(attn_fwd_kv_kernel<64>, dim3(B * H), dim3(256), kv_bytes, (hipStream_t)stream, p); break;
    }
  } else {
    const unsigned grid = ceil_div((int64_t)B * H, 4);
    OT_ATTN_DISPATCH(attn_fwd_kernel, head_dim, dim3(grid), dim3(256), 0, (hipStream_t)stream, p);
  }
  OT_LAUNCH_CHECK("ot_attn_fwd");
  return OT_OK;
}

extern "C" size_t ot_attn_bwd_workspace_size(int B, int H, int K) {
  return (2 * (size_t)B * H + B) * attn_kpad(K) * sizeof(float);     // lse, delta (+ padded qpos)
}

// key-grouped bf16 backward (attn_bwd_group_kernel): long tails only — at C2-like lengths (<= 8 key
// blocks) the per-pair kernel re-reads little and has more parallelism
// (4 waves per workgroup measured faster than 8 at C5: 7.19 vs 8.66 ms per layer, 18.36 per pair)
#ifndef OT_BWDG_NW
#define OT_BWDG_NW 4
#endif
constexpr int ATTN_BWD_GROUP = OT_BWDG_NW, ATTN_BWD_GROUP_MIN_KB = 9;   // waves (key blocks) per group; from 9 key blocks
static int attn_bwd_kgroup(int I, int K, int head_dim, bool sel, int prec) {
  if (sel || K <= SMALL_K || prec != OT_MATMUL_BF16 || (head_dim != 32 && head_dim != 64)) return 0;
  if ((I + 31) / 32 < ATTN_BWD_GROUP_MIN_KB) return 0;
  return ATTN_BWD_GROUP;
}
static int attn_bwd_kslices(int B, int H, int I, int K, int head_dim, bool sel, int prec) {
  const int g = attn_bwd_kgroup(I, K, head_dim, sel, prec);
  return g ? ((I + 31) / 32 + g - 1) / g : 1;
}

extern "C" size_t ot_attn_bwd_ex_workspace_size(int B, int H, int I, int K, int head_dim, int selected,
                                                int precision) {
  const int S = attn_bwd_kslices(B, H, I, K, head_dim, selected != 0, precision);
  return ot_attn_bwd_workspace_size(B, H, K) + (size_t)(S - 1) * B * K * H * head_dim * sizeof(float);
}

extern "C" int ot_attn_bwd_dqkv_bf16_supported(int I, int K, int head_dim, int selected, int precision) {
  return attn_bwd_kgroup(I, K, head_dim, selected != 0, precision) != 0;
}

extern "C" int ot_attn_bwd_bf16_forms(int I, int K, int head_dim, int selected, int precision) {
  if (attn_bwd_kgroup(I, K, head_dim, selected != 0, precision))
    return OT_ATTN_DQKV_BF16 | OT_ATTN_QKV_BF16 | OT_ATTN_DQ_PART_BF16;
  if (K > 0 && K <= SMALL_K && (head_dim == 32 || head_dim == 64 || head_dim == 128)) return OT_ATTN_DQKV_BF16;
  return 0;
}

extern "C" int ot_attn_slice_supported(int I, int K, int head_dim, int selected) {
  return attn_slice_fwd_supported(I, K, head_dim) &&
         (K <= SMALL_K || attn_slice_bwd_supported(I, K, head_dim, selected != 0));
}

extern "C" size_t ot_attn_bwd_flags_workspace_size(int B, int H, int I, int K, int head_dim, int selected, int flags,
                                                   int precision) {
  const int S = attn_bwd_kslices(B, H, I, K, head_dim, selected != 0, precision);
  const int slots = (flags & OT_ATTN_DQKV_BF16) ? S : S - 1;
  const size_t n = ot_attn_bwd_workspace_size(B, H, K) + (size_t)slots * B * K * H * head_dim * sizeof(float);
  // the slice backward's dS scratch (two workgroups per CU), when that kernel takes the shape
  if (precision == OT_MATMUL_SPLIT_BF16 && flags == 0 && K > SMALL_K && !selected &&
      attn_slice_bwd_supported(I, K, head_dim, false))
    return std::max(n, attn_slice_bwd_ws_bytes(B, H, I, K, head_dim));
  return n;
}

static int attn_bwd_impl(const float* qkv, int64_t ld, const float* out, const float* dout, const float* lse,
                         int B, int H, int I, int K, const int32_t* qpos, int head_dim, float* dqkv,
                         float* delta_ws, size_t ws_bytes, int prec, void* stream, int flags = 0,
                         float* amax = nullptr, float* rowmax = nullptr);

extern "C" int ot_attn_bwd_amax(const float* qkv, int64_t ld, const float* out, const float* dout, const float* lse,
                                int B, int H, int I, int K, const int32_t* qpos, int head_dim, float* dqkv,
                                void* workspace, size_t ws_bytes, float* amax, float* rowmax, int precision,
                                void* stream) {
  OT_REQUIRE((amax || rowmax) && (ot_attn_amax_supported(I, K, head_dim, qpos != nullptr, precision) & 2) &&
                 ws_bytes >= ot_attn_bwd_flags_workspace_size(B, H, I, K, head_dim, qpos != nullptr, 0, precision),
             "ot_attn_bwd_amax: the dQKV bound needs the slice backward (split mode, tail queries, I %d K %d head_dim "
             "%d, ot_attn_bwd_flags_workspace_size bytes)", I, K, head_dim);
  return attn_bwd_impl(qkv, ld, out, dout, lse, B, H, I, K, qpos, head_dim, dqkv, (float*)workspace, ws_bytes,
                       precision, stream, 0, amax, rowmax);
}

extern "C" int ot_attn_bwd(const float* qkv, int64_t ld, const float* out, const float* dout, const float* lse,
                           int B, int H, int I, int K, const int32_t* qpos, int head_dim, float* dqkv,
                           float* delta_ws, int precision, void* stream) {
  return attn_bwd_impl(qkv, ld, out, dout, lse, B, H, I, K, qpos, head_dim, dqkv, delta_ws,
                       ot_attn_bwd_workspace_size(B, H, K), precision, stream);
}

extern "C" int ot_attn_bwd_ex(const float* qkv, int64_t ld, const float* out, const float* dout, const float* lse,
                              int B, int H, int I, int K, const int32_t* qpos, int head_dim, float* dqkv,
                              void* workspace, size_t ws_bytes, int precision, void* stream) {
  OT_REQUIRE(ws_bytes >= ot_attn_bwd_workspace_size(B, H, K), "ot_attn_bwd_ex: workspace too small");
  return attn_bwd_impl(qkv, ld, out, dout, lse, B, H, I, K, qpos, head_dim, dqkv, (float*)workspace, ws_bytes,
                       precision, stream);
}

extern "C" int ot_attn_bwd_flags(const float* qkv, int64_t ld, const float* out, const float* dout,
                                 const float* lse, int B, int H, int I, int K, const int32_t* qpos, int head_dim,
                                 void* dqkv, int flags, void* workspace, size_t ws_bytes, int precision,
                                 void* stream) {
  OT_REQUIRE(!(flags & ~(OT_ATTN_DQKV_BF16 | OT_ATTN_QKV_BF16 | OT_ATTN_DQ_PART_BF16)),
             "ot_attn_bwd_flags: unknown flags %d", flags);
  OT_REQUIRE(!(flags & OT_ATTN_DQ_PART_BF16) || (flags & OT_ATTN_DQKV_BF16),
             "ot_attn_bwd_flags: OT_ATTN_DQ_PART_BF16 goes with OT_ATTN_DQKV_BF16");
  OT_REQUIRE((flags & ot_attn_bwd_bf16_forms(I, K, head_dim, qpos != nullptr, precision)) == flags,
             "ot_attn_bwd_flags: flags %d not supported at I %d K %d head_dim %d (ot_attn_bwd_bf16_forms)", flags, I,
             K, head_dim);
  OT_REQUIRE(!(flags & OT_ATTN_QKV_BF16) || (ot_attn_bwd_dqkv_bf16_supported(I, K, head_dim, qpos != nullptr, precision) &&
                                             ((uintptr_t)qkv % 16) == 0 && ld % 8 == 0),
             "ot_attn_bwd_flags: OT_ATTN_QKV_BF16 needs the key-grouped bf16 backward, 16-B aligned qkv, ld %% 8 == 0");
  OT_REQUIRE(ws_bytes >= ot_attn_bwd_flags_workspace_size(B, H, I, K, head_dim, qpos != nullptr, flags, precision),
             "ot_attn_bwd_flags: workspace too small");
  OT_REQUIRE(!(flags & OT_ATTN_DQKV_BF16) || ((uintptr_t)dqkv % 8) == 0, "ot_attn_bwd_flags: dqkv alignment");
  return attn_bwd_impl(qkv, ld, out, dout, lse, B, H, I, K, qpos, head_dim, (float*)dqkv, (float*)workspace,
                       ws_bytes, precision, stream, flags);
}

static int attn_bwd_impl(const float* qkv, int64_t ld, const float* out, const float* dout, const float* lse,
                         int B, int H, int I, int K, const int32_t* qpos, int head_dim, float* dqkv,
                         float* delta_ws, size_t ws_bytes, int prec, void* stream, int flags, float* amax,
                         float* rowmax) {
  OT_REQUIRE(prec == OT_MATMUL_F32 || prec == OT_MATMUL_SPLIT_BF16 || prec == OT_MATMUL_BF16,
             "ot_attn_bwd: unknown precision %d", prec);
  OT_REQUIRE(qkv && out && dout && lse && dqkv && delta_ws, "ot_attn_bwd: null operand");
  OT_REQUIRE(B >= 0 && H > 0 && I > 0 && K > 0 && K <= I, "ot_attn_bwd: bad sizes");
  OT_REQUIRE(ld % 4 == 0 && ld >= 3 * H * head_dim, "ot_attn_bwd: bad ld");
  if (B == 0) return OT_OK;
  AttnArgs p{qkv, ld, H * head_dim, out, dout, nullptr, const_cast<float*>(lse), dqkv, delta_ws, B, H, I, K,
             1.f / sqrtf((float)head_dim), qpos};
  const int mm = prec;
  if (mm == OT_MATMUL_SPLIT_BF16 && flags == 0 && K > SMALL_K && attn_slice_bwd_supported(I, K, head_dim, qpos != nullptr) &&
      ws_bytes >= attn_slice_bwd_min_ws(B, H, I, K, head_dim))
    return attn_slice_bwd(qkv, ld, out, dout, lse, B, H, I, K, head_dim, dqkv, delta_ws, ws_bytes, (hipStream_t)stream,
                          amax, rowmax);
  OT_REQUIRE((!amax && !rowmax) || K <= SMALL_K, "ot_attn_bwd_amax: shape not on the slice / short-tail backward");
  p.amax = amax;
  p.rowmax = rowmax;
  // the f32 head_dim-32 backward over tail queries forms its own row statistics (no prep launch)
  const bool fdl = !qpos && head_dim == 32 && K > SMALL_K && attn_kpad(K) <= FDL_KP &&
                   mm != OT_MATMUL_BF16;
  if (fdl) {
    hipLaunchKernelGGL((attn_bwd_kernel<32, false, 1, true>), dim3(ceil_div((int64_t)B * H, BWD_WAVES<32>())),
                       dim3(64 * BWD_WAVES<32>()), 0, (hipStream_t)stream, p);
    OT_LAUNCH_CHECK("ot_attn_bwd");
    return OT_OK;
  }
  const int main_blocks = (int)ceil_div((int64_t)B * K * H * head_dim / 4, 256);
  const int pad_blocks = (int)ceil_div((int64_t)B * H * (attn_kpad(K) - K), 256);
  const int qpos_blocks = qpos ? (int)ceil_div((int64_t)B * attn_kpad(K), 256) : 0;
  hipLaunchKernelGGL(attn_bwd_prep_kernel, dim3(main_blocks + pad_blocks + qpos_blocks), dim3(256), 0,
                     (hipStream_t)stream, out, dout, lse, delta_ws, B, H, K, head_dim, main_blocks, pad_blocks, qpos);
  OT_LAUNCH_CHECK("ot_attn_bwd(prep)");
  p.dq_bf16 = (flags & OT_ATTN_DQKV_BF16) ? 1 : 0;
  if (K == 1) {
    OT_ATTN_DISPATCH_K1(attn_bwd_small_kernel, head_dim, dim3(ceil_div((int64_t)B * H, 4)), dim3(256), 0,
                     (hipStream_t)stream, p);
  } else if (K <= SMALL_K) {
    OT_ATTN_DISPATCH(attn_bwd_small_kernel, head_dim, dim3(ceil_div((int64_t)B * H, 4)), dim3(256), 0,
                     (hipStream_t)stream, p);
  } else if (mm == OT_MATMUL_BF16 && (head_dim == 32 || head_dim == 64) &&
             attn_bwd_kgroup(I, K, head_dim, qpos != nullptr, prec) &&
             ws_bytes >= ot_attn_bwd_ex_workspace_size(B, H, I, K, head_dim, 0, prec)) {
    // bf16 mode, long tails: key-grouped workgroups (dQ partials in the ot_attn_bwd_ex workspace)
    const int G = attn_bwd_kgroup(I, K, head_dim, false, prec), S = attn_bwd_kslices(B, H, I, K, head_dim, false, prec);
    p.kslices = S;
    p.kgroup = G;
    p.dqpart = delta_ws + ot_attn_bwd_workspace_size(B, H, K) / sizeof(float);
    p.dq_bf16 = (flags & OT_ATTN_DQKV_BF16) ? 1 : 0;
    p.qkv_bf16 = (flags & OT_ATTN_QKV_BF16) ? 1 : 0;
    p.dq_part16 = (flags & OT_ATTN_DQ_PART_BF16) ? 1 : 0;
    void (*kern)(AttnArgs) =
        p.qkv_bf16 ? (G == 8 ? (head_dim == 32 ? attn_bwd_group_kernel<32, 8, true> : attn_bwd_group_kernel<64, 8, true>)
                             : (head_dim == 32 ? attn_bwd_group_kernel<32, 4, true> : attn_bwd_group_kernel<64, 4, true>))
                   : (G == 8 ? (head_dim == 32 ? attn_bwd_group_kernel<32, 8> : attn_bwd_group_kernel<64, 8>)
                             : (head_dim == 32 ? attn_bwd_group_kernel<32, 4> : attn_bwd_group_kernel<64, 4>));
    const size_t lds = G == 8 ? (head_dim == 32 ? BWDG_LDS<32, 8>() : BWDG_LDS<64, 8>())
                              : (head_dim == 32 ? BWDG_LDS<32, 4>() : BWDG_LDS<64, 4>());
    static std::once_flag glds_once;
    std::call_once(glds_once, [] {
      for (void (*k)(AttnArgs) : {attn_bwd_group_kernel<32, 8>, attn_bwd_group_kernel<64, 8>,
                                  attn_bwd_group_kernel<32, 4>, attn_bwd_group_kernel<64, 4>,
                                  attn_bwd_group_kernel<32, 8, true>, attn_bwd_group_kernel<64, 8, true>,
                                  attn_bwd_group_kernel<32, 4, true>, attn_bwd_group_kernel<64, 4, true>})
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, BWDG_LDS<64, 8>());
      (void)hipGetLastError();
    });
    hipLaunchKernelGGL(kern, dim3((unsigned)((int64_t)B * H * S)), dim3(64 * G), lds, (hipStream_t)stream, p);
    if (S > 1 || p.dq_bf16) {
      OT_LAUNCH_CHECK("ot_attn_bwd");
      hipLaunchKernelGGL(attn_dq_reduce_kernel, dim3(ceil_div((int64_t)B * K * p.d / 4, 256)), dim3(256), 0,
                         (hipStream_t)stream, p);
    }
  } else if (mm == OT_MATMUL_BF16 && (head_dim == 32 || head_dim == 64)) {
    // bf16 mode: one-plane bf16 MFMA, one wave per (sample, head), 4 waves / block.  The six-term split
    // form of the same kernel measured slower than the f32 kernel at hd 32 (1.42 vs 1.34 ms at C2:
    // the pass is latency-bound, not MFMA-bound), so split mode keeps the f32 backward.
    void (*kern)(AttnArgs) = nullptr;
    const bool sel = qpos != nullptr;
    const int waves = 4, lds = head_dim == 32 ? BWDS_LDS<32, 1>() : BWDS_LDS<64, 1>();
    if (head_dim == 32) kern = sel ? attn_bwd_split_kernel<32, 1, true, 4> : attn_bwd_split_kernel<32, 1, false, 4>;
    else kern = sel ? attn_bwd_split_kernel<64, 1, true, 4> : attn_bwd_split_kernel<64, 1, false, 4>;
    const unsigned grid = ceil_div((int64_t)B * H, waves);
    static std::once_flag lds_once;                    // hd 64: 72 KiB per 4-wave block (> 64 KiB default)
    std::call_once(lds_once, [] {
      for (void (*k)(AttnArgs) : {attn_bwd_split_kernel<32, 1, true, 4>, attn_bwd_split_kernel<32, 1, false, 4>,
                                  attn_bwd_split_kernel<64, 1, true, 4>, attn_bwd_split_kernel<64, 1, false, 4>})
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 4 * BWDS_LDS<64, 1>());
      (void)hipGetLastError();
    });
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * waves), (size_t)waves * lds, (hipStream_t)stream, p);
  } else if (head_dim == 64) {
    // head_dim 64 as two 32-dim waves per (sample, head): 2 waves / SIMD instead of 1
    const bool sel = qpos != nullptr;
    void (*kern)(AttnArgs) = sel ? attn_bwd_kernel<32, true, 2> : attn_bwd_kernel<32, false, 2>;
    hipLaunchKernelGGL(kern, dim3((unsigned)((int64_t)B * H)), dim3(128), 0, (hipStream_t)stream, p);
  } else {
    const int waves = head_dim >= 128 ? 2 : 4;
    const unsigned grid = ceil_div((int64_t)B * H, waves);
    void (*kern)(AttnArgs) = nullptr;
    const bool sel = qpos != nullptr;
    switch (head_dim) {
      case 16: kern = sel ? attn_bwd_kernel<16, true> : attn_bwd_kernel<16, false>; break;
      case 32: kern = sel ? attn_bwd_kernel<32, true> : attn_bwd_kernel<32, false>; break;
      case 128: kern = sel ? attn_bwd_kernel<128, true> : attn_bwd_kernel<128, false>; break;
      default: return fail(OT_ERR_UNSUPPORTED, "attention: head_dim %d unsupported", head_dim);
    }
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * waves), 0, (hipStream_t)stream, p);
  }
  OT_LAUNCH_CHECK("ot_attn_bwd");
  return OT_OK;
}
