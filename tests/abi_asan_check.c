/* Host-side AddressSanitizer check of the C ABI (include/onetrans_hip.h), no GPU: every entry point
 * below is called with invalid arguments and must return a non-zero status with a non-empty error
 * string, before touching the device; the workspace-size queries are called at edge sizes.  Built and
 * run by tests/test_abi_asan.py against the host-only ASAN build (make -C recommend_amd/csrc asan). */
#include <stdio.h>
#include <string.h>

#include "onetrans_hip.h"

static int failures = 0;

static void expect_error(const char* what, int rc) {
  const char* msg = ot_get_last_error_string();
  if (rc == 0 || msg == NULL || msg[0] == '\0') {
    printf("FAIL %s: rc=%d msg='%s'\n", what, rc, msg ? msg : "(null)");
    ++failures;
  } else {
    printf("ok   %s: %s\n", what, msg);
  }
}

int main(void) {
  float f[64];
  int32_t ids[64];
  memset(f, 0, sizeof f);
  memset(ids, 0, sizeof ids);
  if (ot_version() <= 0 || ot_gemm_tile_rows() != 128) { printf("FAIL identity\n"); ++failures; }
  expect_error("ot_mixed_gemm null operands",
               ot_mixed_gemm(1, NULL, 4, 4, NULL, 0, NULL, NULL, NULL, 0, 4, 4, NULL, 1, NULL, 0, NULL, 4, NULL, 0,
                             NULL, 0, 0, NULL, 0, 0, 0, 0.f, 1, 1, NULL, OT_MATMUL_SPLIT_BF16, NULL));
  expect_error("ot_mixed_gemm K not a multiple of 4",
               ot_mixed_gemm(1, f, 4, 3, NULL, 0, NULL, NULL, f, 0, 4, 4, NULL, 1, NULL, 0, f, 4, NULL, 0,
                             NULL, 0, 0, NULL, 0, 0, 0, 0.f, 1, 1, NULL, OT_MATMUL_SPLIT_BF16, NULL));
  expect_error("ot_mixed_gemm bias flag without bias",
               ot_mixed_gemm(1, f, 4, 4, NULL, 0, NULL, NULL, f, 0, 4, 4, NULL, 1, NULL, 0, f, 4, NULL, OT_EPI_BIAS,
                             NULL, 0, 0, NULL, 0, 0, 0, 0.f, 1, 1, NULL, OT_MATMUL_SPLIT_BF16, NULL));
  expect_error("ot_mixed_gemm row-norm flag without epilogue operands",
               ot_mixed_gemm(1, f, 4, 4, NULL, 0, NULL, NULL, f, 0, 4, 128, NULL, 1, NULL, 0, f, 128, NULL,
                             OT_EPI_ROW_RSTD, NULL, 0, 0, NULL, 0, 0, 0, 0.f, 1, 1, NULL, OT_MATMUL_SPLIT_BF16, NULL));
  expect_error("ot_attn_fwd bad sizes (K > I)", ot_attn_fwd(f, 96, 1, 1, 4, 8, NULL, 32, f, f, OT_MATMUL_SPLIT_BF16, NULL));
  expect_error("ot_attn_fwd unsupported head_dim", ot_attn_fwd(f, 24, 1, 1, 4, 4, NULL, 8, f, f, OT_MATMUL_SPLIT_BF16, NULL));
  expect_error("ot_attn_fwd_fp8 head_dim 32", ot_attn_fwd_fp8(f, 96, 1, 1, 4, 4, NULL, 32, f, f, f, 64, NULL));
  expect_error("ot_attn_fwd_fp8 workspace too small", ot_attn_fwd_fp8(f, 192, 1, 1, 4, 4, NULL, 64, f, f, f, 16, NULL));
  expect_error("ot_attn_fwd_fp8_ex unknown flag", ot_attn_fwd_fp8_ex(f, 192, 1, 1, 4, 4, NULL, 64, f, f, f, 1 << 20, 2, NULL));
  expect_error("ot_attn_bwd null operand", ot_attn_bwd(f, 96, f, NULL, f, 1, 1, 4, 4, NULL, 32, f, f, OT_MATMUL_SPLIT_BF16, NULL));
  expect_error("ot_attn_bwd_ex workspace too small",
               ot_attn_bwd_ex(f, 96, f, f, f, 1, 1, 4, 4, NULL, 32, f, f, 16, OT_MATMUL_SPLIT_BF16, NULL));
  expect_error("ot_attn_fwd_cached bad sizes", ot_attn_fwd_cached(f, 96, f, 64, ids, 1, 1, 2, 4, 5, 32, f, NULL));
  expect_error("ot_pyramid_select K > I", ot_pyramid_select(NULL, 1.f, 1, 4, 5, 0, ids, NULL, NULL, 0, NULL));
  expect_error("ot_sparse_adagrad E not a multiple of 4",
               ot_sparse_adagrad(f, f, 3, 10, (const int64_t*)ids, f, 2, 0.1f, 1e-7f, 120.f, f, sizeof f, NULL));
  expect_error("ot_clip_rmsprop null segments",
               ot_clip_rmsprop(f, f, f, f, NULL, 1, 4, 0.1f, 0.9f, 1e-7f, 0.f, 90.f, f, sizeof f, NULL));
  expect_error("ot_attn_fwd unknown precision", ot_attn_fwd(f, 96, 1, 1, 4, 4, NULL, 32, f, f, 7, NULL));
  /* workspace queries at edge sizes (pure host arithmetic) */
  if (ot_attn_bwd_workspace_size(1, 1, 1) == 0 || ot_mixed_gemm_rms_workspace_size(0, 128) == 0 ||
      ot_attn_fwd_fp8_workspace_size(1, 1, 1, 64) == 0 || ot_attn_fwd_fp8_workspace_size(1, 1, 1, 32) != 0 ||
      ot_sparse_adagrad_workspace_size(0, 16) == 0 ||
      ot_attn_bwd_ex_workspace_size(1, 1, 4, 4, 32, 0, OT_MATMUL_BF16) < ot_attn_bwd_workspace_size(1, 1, 4)) {
    printf("FAIL workspace sizes\n");
    ++failures;
  }
  printf(failures ? "ABI ASAN CHECK FAILED (%d)\n" : "ABI ASAN CHECK OK\n", failures);
  return failures ? 1 : 0;
}
