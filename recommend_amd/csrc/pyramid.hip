// Pyramid query selection on gfx950: per-sample top-K of I tokens with wavefront ballots.
//
// Replaces PyramidScheduler.get_layer_config + tf.gather (model.py:287-302, 356, 371).  The
// reference keeps the static tail range(L0 - keep, L0) (D2: against the original length; the build
// uses the current one).  Here the kept set is the K largest keys, key(p) = (score[p] * sign,
// position p), the last `nforce` positions forced in; with no score every key ties on the first
// component and the position decides: the kept set is exactly the tail (reference semantics).
//
// One 64-lane wavefront per sample, keys in registers (lane l holds positions l, l + 64, ...):
//  1. radix select of the K-th largest 64-bit key, one bit at a time from the top: the number of
//     keys >= candidate is a sum of popcounts of per-register ballots (no LDS, no shuffles);
//     bits between the position field and bit 32 are provably zero in the answer and skipped;
//  2. ordered compaction: register c of every lane is position 64c + lane, so the ballot of
//     "selected" over register c, counted below the lane with mbcnt, gives each kept position its
//     output slot in ascending order.
// HBM-bound and tiny (reads B*I scores, writes B*K positions + B*I inverse entries).
#include "common.h"

namespace ot {

__device__ __forceinline__ uint32_t ordered_bits(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);     // monotone: larger float -> larger uint
}

template <int PL>
__global__ __launch_bounds__(256) void pyramid_select_kernel(const float* __restrict__ score, float sign, int B,
                                                             int I, int K, int nforce, int32_t* __restrict__ pos,
                                                             int32_t* __restrict__ inv, int32_t* __restrict__ map_rows,
                                                             int mps) {
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;                                   // wave-uniform
  const int64_t row0 = (int64_t)b * I;
  uint64_t key[PL];
#pragma unroll
  for (int c = 0; c < PL; ++c) {
    const int p = 64 * c + lane;
    uint64_t k = 0;                                     // past the end: below every real key
    if (p < I) {
      uint32_t hi = 0;
      if (p >= I - nforce) hi = 0xFFFFFFFFu;
      else if (score) hi = min(ordered_bits(score[row0 + p] * sign), 0xFFFFFFFEu);
      k = ((uint64_t)hi << 32) | (uint32_t)(p + 1);     // ties -> the later position
    }
    key[c] = k;
  }
  // K-th largest key (keys are distinct: the position field)
  const int lb = 32 - __builtin_clz((unsigned)I);       // position field width (p + 1 <= I)
  uint64_t t = 0;
  for (int bit = 63; bit >= 0; --bit) {
    if (bit < 32 && bit >= lb) continue;
    const uint64_t cand = t | (1ull << bit);
    int cnt = 0;
#pragma unroll
    for (int c = 0; c < PL; ++c) cnt += __popcll(__ballot(key[c] >= cand));
    if (cnt >= K) t = cand;
  }
  // ordered compaction
  int base = 0;
#pragma unroll
  for (int c = 0; c < PL; ++c) {
    const int p = 64 * c + lane;
    const bool sel = key[c] >= t;                       // t >= 1, so padding (key 0) is never selected
    const uint64_t m = __ballot(sel);
    const int j = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (sel) {
      pos[(int64_t)b * K + j] = p;
      if (map_rows && j < mps) map_rows[(int64_t)b * mps + j] = (int32_t)(row0 + p);
    }
    if (inv && p < I) inv[row0 + p] = sel ? (int32_t)((int64_t)b * K + j) : -1;
    base += __popcll(m);
  }
}

}  // namespace ot

using namespace ot;

extern "C" int ot_pyramid_select(const float* score, float score_sign, int B, int I, int K, int nforce,
                                 int32_t* pos, int32_t* inv, int32_t* map_rows, int map_per_sample, void* stream) {
  OT_REQUIRE(pos, "ot_pyramid_select: null pos");
  OT_REQUIRE(B >= 0 && I > 0 && I <= 4096 && K > 0 && K <= I, "ot_pyramid_select: bad sizes B=%d I=%d K=%d", B, I, K);
  OT_REQUIRE(nforce >= 0 && nforce <= K, "ot_pyramid_select: nforce=%d out of range [0, K=%d]", nforce, K);
  OT_REQUIRE(!map_rows || (map_per_sample >= 0 && map_per_sample <= K), "ot_pyramid_select: bad map_per_sample");
  OT_REQUIRE((int64_t)B * I < (int64_t)INT32_MAX, "ot_pyramid_select: B*I exceeds int32 rows");
  if (B == 0) return OT_OK;
  const dim3 grid(ceil_div((int64_t)B, 4)), block(256);
  hipStream_t s = (hipStream_t)stream;
  const int pl = (I + 63) / 64;
#define OT_SEL_LAUNCH(PL_)                                                                               \
  hipLaunchKernelGGL(pyramid_select_kernel<PL_>, grid, block, 0, s, score, score_sign, B, I, K, nforce, pos, \
                     inv, map_rows, map_per_sample)
  if (pl <= 1) OT_SEL_LAUNCH(1);
  else if (pl <= 2) OT_SEL_LAUNCH(2);
  else if (pl <= 4) OT_SEL_LAUNCH(4);
  else if (pl <= 8) OT_SEL_LAUNCH(8);
  else if (pl <= 16) OT_SEL_LAUNCH(16);
  else if (pl <= 32) OT_SEL_LAUNCH(32);
  else OT_SEL_LAUNCH(64);
#undef OT_SEL_LAUNCH
  OT_LAUNCH_CHECK("ot_pyramid_select");
  return OT_OK;
}
