// Probe: operand/result lane map of v_mfma_f32_16x16x4_f32 (one-hot A operand, distinct B values),
// checked against the fp32 chain's layout (chain32.hpp): A lane l = A[l%16][l/16], B lane l =
// B[l/16][l%16], D lane l reg r = D[4(l/16) + r][l%16] (the f64 16x16x4 form differs: D[4r + l/16]).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void probe(float* out) {
  int l = threadIdx.x;
  for (int p = 0; p < 64; ++p) {
    float a = (l == p) ? 1.f : 0.f, b = (float)(l + 1);
    f4 d = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, f4{0, 0, 0, 0}, 0, 0, 0);
    for (int r = 0; r < 4; ++r) out[(p * 64 + l) * 4 + r] = d[r];
  }
}
int main() {
  float* d; hipMalloc(&d, 64 * 64 * 4 * sizeof(float));
  float* h = new float[64 * 64 * 4];
  probe<<<1, 64>>>(d);
  hipMemcpy(h, d, 64 * 64 * 4 * sizeof(float), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int p = 0; p < 64; ++p) {
    int ai = p % 16, ak = p / 16;  // assumed A[i][k]
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < 4; ++r) {
        int di = 4 * (l / 16) + r, dj = l % 16;  // chain32.hpp's D[i][j]
        float expect = (di == ai) ? (float)(16 * ak + dj + 1) : 0.f;  // B[k][j] at lane 16k + j
        if (h[(p * 64 + l) * 4 + r] != expect) ++bad;
      }
    if (p < 4 || p == 17) {
      printf("p%02d:", p);
      for (int l = 0; l < 64; ++l) for (int r = 0; r < 4; ++r) { float v = h[(p * 64 + l) * 4 + r]; if (v != 0) printf(" %d.%d=%d", l, r, (int)v - 1); }
      printf("\n");
    }
  }
  printf("layout mismatches: %d\n", bad);
  return 0;
}
