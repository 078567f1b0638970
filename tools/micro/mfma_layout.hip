// Calibration (not product code): operand/result lane maps of v_mfma_f64_4x4x4f64 and
// v_mfma_f64_16x16x4f64 on gfx950, by one-hot probing with exact integer data.
// Prints, for each one-hot lane L of A (B = lane+1) and of B (A = lane+1), the nonzero outputs.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void probe4(double* out, int which) {
  const int L = blockIdx.x, l = threadIdx.x;
  const double a = which == 0 ? (l == L ? 1.0 : 0.0) : (double)(l + 1);
  const double b = which == 1 ? (l == L ? 1.0 : 0.0) : (double)(l + 1);
  out[L * 64 + l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
}

__global__ void probe16(double* out, int which) {
  const int L = blockIdx.x, l = threadIdx.x;
  const double a = which == 0 ? (l == L ? 1.0 : 0.0) : (double)(l + 1);
  const double b = which == 1 ? (l == L ? 1.0 : 0.0) : (double)(l + 1);
  d4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[(L * 64 + l) * 4 + r] = c[r];
}

int main() {
  double *d, h[64 * 64 * 4];
  (void)hipMalloc(&d, sizeof(h));
  for (int which = 0; which < 2; ++which) {
    probe4<<<64, 64>>>(d, which);
    (void)hipMemcpy(h, d, 64 * 64 * 8, hipMemcpyDeviceToHost);
    for (int L = 0; L < 64; ++L) {
      printf("4x4x4 %s L=%d:", which ? "B" : "A", L);
      for (int l = 0; l < 64; ++l)
        if (h[L * 64 + l] != 0) printf(" %d=%g", l, h[L * 64 + l]);
      printf("\n");
    }
  }
  for (int which = 0; which < 2; ++which) {
    probe16<<<64, 64>>>(d, which);
    (void)hipMemcpy(h, d, 64 * 64 * 4 * 8, hipMemcpyDeviceToHost);
    for (int L = 0; L < 64; ++L) {
      printf("16x16x4 %s L=%d:", which ? "B" : "A", L);
      for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 4; ++r)
          if (h[(L * 64 + l) * 4 + r] != 0) printf(" %d.%d=%g", l, r, h[(L * 64 + l) * 4 + r]);
      printf("\n");
    }
  }
  return 0;
}
