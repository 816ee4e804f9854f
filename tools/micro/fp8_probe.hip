// Operand-layout probe of v_mfma_scale_f32_32x32x64_f8f6f4 (fp8 e4m3, scales 127 = 1.0 unless noted).
// 1. k pairing: A one-hot at (lane half ha, byte j) of row 0; B lane n has 1.0 at byte n (half 0) and
//    2.0 at byte n (half 1): C[0][n] tells which B (half, byte) meets A's (ha, j).
// 2. C layout: A = e_r (row r all-ones on k 0), B column c has k0 = c+1: C[r][c] = c+1 at reg/lane.
// 3. scales: A half-0 scale 128 (x2) on lane r: which outputs double.
// 4. cvt_pk_fp8_f32 byte order.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
__global__ void mm(const unsigned char* A, const unsigned char* B, const int* sa, const int* sb, float* C) {
  const int l = threadIdx.x;
  i32x8 a, b;
  memcpy(&a, A + 32 * l, 32);
  memcpy(&b, B + 32 * l, 32);
  f32x16 c = {};
  c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, sa[l], 0, sb[l]);
  for (int r = 0; r < 16; ++r) C[l * 16 + r] = c[r];
}
__global__ void cvt(const float* x, int* y) {
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(x[0], x[1], 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(x[2], x[3], v, true);
  y[0] = v;
}
static unsigned char hA[64 * 32], hB[64 * 32];
static int hsa[64], hsb[64];
static float hC[64 * 16];
unsigned char *dA, *dB; int *dsa, *dsb; float* dC;
void run() {
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  hipMemcpy(dsa, hsa, sizeof hsa, hipMemcpyHostToDevice);
  hipMemcpy(dsb, hsb, sizeof hsb, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(mm, dim3(1), dim3(64), 0, 0, dA, dB, dsa, dsb, dC);
  hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
}
// C[row][col] assuming row = (r&3) + 8(r>>2) + 4(l>>5), col = l&31
float Cat(int row, int col) {
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 16; ++r)
      if ((l & 31) == col && (r & 3) + 8 * (r >> 2) + 4 * (l >> 5) == row) return hC[l * 16 + r];
  return -999;
}
int main() {
  hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dsa, sizeof hsa); hipMalloc(&dsb, sizeof hsb);
  hipMalloc(&dC, sizeof hC);
  const unsigned char ONE = 0x38, TWO = 0x40;
  for (int i = 0; i < 64; ++i) hsa[i] = hsb[i] = 127;
  printf("[1] k pairing (A row 0, half ha, byte j) -> B (half, byte):\n");
  int same = 0;
  for (int ha = 0; ha < 2; ++ha)
    for (int j = 0; j < 32; ++j) {
      memset(hA, 0, sizeof hA); memset(hB, 0, sizeof hB);
      hA[32 * (32 * ha + 0) + j] = ONE;
      for (int n = 0; n < 32; ++n) { hB[32 * n + n] = ONE; hB[32 * (32 + n) + n] = TWO; }
      run();
      int hit = -1, hb = -1;
      for (int n = 0; n < 32; ++n) {
        const float v = Cat(0, n);
        if (v == 1.f) { hit = n; hb = 0; }
        if (v == 2.f) { hit = n; hb = 1; }
        if (v == 3.f) { hit = n; hb = 2; }
      }
      if (hb == ha && hit == j) ++same;
      else printf("  A(h%d,b%d) -> B(h%d,b%d)\n", ha, j, hb, hit);
    }
  printf("  %d of 64 positions pair with the same (half, byte)\n", same);
  // [2] C layout: A row r (lane r, half 0, byte 0) = 1; B column c (lane c, byte 0) = value (c%8)+1
  memset(hA, 0, sizeof hA); memset(hB, 0, sizeof hB);
  const unsigned char vals[8] = {0x38, 0x40, 0x44, 0x48, 0x4a, 0x4c, 0x4e, 0x50};   // 1,2,3,4,5,6,7,8
  for (int r = 0; r < 32; ++r) hA[32 * r] = (r < 16) ? ONE : TWO;
  for (int c = 0; c < 32; ++c) hB[32 * c] = vals[c % 8];
  run();
  int bad = 0;
  for (int row = 0; row < 32; ++row)
    for (int col = 0; col < 32; ++col) {
      const float want = (row < 16 ? 1.f : 2.f) * (float)(col % 8 + 1);
      if (Cat(row, col) != want) ++bad;
    }
  printf("[2] C layout mismatches under acc_row: %d of 1024\n", bad);
  // [3] scales: all A, B = 1.0 on every byte; A lane 5 (row 5, half 0) scale 128; B lane 32+7 scale 129
  memset(hA, ONE, sizeof hA); memset(hB, ONE, sizeof hB);
  hsa[5] = 128; hsb[39] = 129;
  run();
  printf("[3] scales: C[5][0]=%g (want 96: half0 x2), C[0][7]=%g (want 160: half1 x4), C[5][7]=%g (want 192), C[0][0]=%g (64)\n",
         Cat(5, 0), Cat(0, 7), Cat(5, 7), Cat(0, 0));
  for (int i = 0; i < 64; ++i) hsa[i] = hsb[i] = 127;
  // [5] which bytes a lane's scale covers: A all ones, lane 5's scale x2; B ones only in bytes 0-15
  //     of lane 32 (column 0, upper half).  C[5][0] = 32 if lane 5's scale also covers lane 37's bytes
  //     0-15 (scale block = bytes [16h, 16h+16) of both half-lanes), 16 if it covers only lane 5.
  memset(hA, ONE, sizeof hA); memset(hB, 0, sizeof hB);
  for (int j = 0; j < 16; ++j) hB[32 * 32 + j] = ONE;
  hsa[5] = 128;
  run();
  printf("[5] C[5][0] = %g (32: scale block = bytes [16h,16h+16) of lanes r and r+32; 16: the lane's own 32 bytes)\n",
         Cat(5, 0));
  hsa[5] = 127;
  float hx[4] = {1.f, 2.f, 3.f, 0.5f}, *dx; int hy, *dy;
  hipMalloc(&dx, 16); hipMalloc(&dy, 4);
  hipMemcpy(dx, hx, 16, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(cvt, dim3(1), dim3(1), 0, 0, dx, dy);
  hipMemcpy(&hy, dy, 4, hipMemcpyDeviceToHost);
  printf("[4] cvt_pk(1,2) lo + cvt_pk(3,0.5) hi = 0x%08x (want 0x30444038)\n", hy);
  return 0;
}
