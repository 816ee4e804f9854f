// Short-sequence attention: one workgroup per (sample, head) slice on split MFMA (three bf16 planes or a scaled fp16
// pair per f32 operand)
// (attention_slice.hip).  Dispatched from ot_attn_fwd / ot_attn_bwd (attention.hip) in the
// f32-accurate mode (OT_MATMUL_SPLIT_BF16) when the slice fits LDS.
#pragma once
#include "common.h"

namespace ot {

constexpr int SLICE_TABN = 36;                // backward key blocks per slice (I <= 544 at head_dim 64)

struct SliceArgs {
  const float* qkv; int64_t ld; int d;        // qkv [B*I, ld]: q at col 0, k at d, v at 2d; head h at +h*hd
  const float* o; const float* dout; const float* lse_in;   // backward inputs: O, dO [B*K, d], lse [B*H*K]
  float* out; float* lse;                     // forward outputs
  float* dqkv;                                // backward output (dq on the K tail rows, dk / dv on all rows)
  int B, H, I, K;
  float scale;
  const int32_t* qpos;                        // forward only: kept query positions [B*K] or null (tail)
  // work schedule from the host (attention_slice.hip make_schedule): item of slot s of wave w, -1 = none;
  // [0] forward query blocks, [1] backward key blocks, [2] backward query blocks (items heaviest first)
  alignas(8) int8_t sched[3][8][8];            // rows read as one uint64 each (slot s = byte s)
  int8_t qf[SLICE_TABN];                      // backward: first query block that sees key block kb
  int16_t bbase[SLICE_TABN];                  // backward: dS-store block index of (qf[kb], kb)
  float* dsws; int ds_floats;                 // backward, two workgroups per CU: per-workgroup dS scratch
  float* amax;                                // optional: max |output| folded in atomically (fp16-pair bounds)
  float* rowmax;                              // optional: per-row max |output| parts: forward [B*K][H] (O, per
                                              // head), backward [B*I][3][H] (dQ / dK / dV, per head)
};

bool attn_slice_fwd_supported(int I, int K, int head_dim);
bool attn_slice_bwd_supported(int I, int K, int head_dim, bool selected);
// amax (optional): max |output| folded in atomically (the caller zeroes it; fp16-pair weight-gradient bounds)
int attn_slice_fwd(const float* qkv, int64_t ld, int B, int H, int I, int K, const int32_t* qpos, int head_dim,
                   float* out, float* lse, hipStream_t stream, float* amax = nullptr, float* rowmax = nullptr);
// ws / ws_bytes: scratch for the two-workgroups-per-CU backward (attn_slice_bwd_ws_bytes for the full grid; less
// shrinks its grid; below one workgroup's share the one-workgroup-per-CU kernel runs)
int attn_slice_bwd(const float* qkv, int64_t ld, const float* out, const float* dout, const float* lse, int B, int H,
                   int I, int K, int head_dim, float* dqkv, float* ws, size_t ws_bytes, hipStream_t stream,
                   float* amax = nullptr, float* rowmax = nullptr);
size_t attn_slice_bwd_ws_bytes(int B, int H, int I, int K, int head_dim);
// the workspace below which the backward's long forms are not taken (they keep dS only there; 0 otherwise)
size_t attn_slice_bwd_min_ws(int B, int H, int I, int K, int head_dim);

}  // namespace ot
