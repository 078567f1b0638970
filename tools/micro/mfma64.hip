// Calibration (not product code): FP64 MFMA issue rate on gfx950, and whether FP64 MFMA and
// FP64 VALU FMA issued from different waves of one SIMD add up.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int C>
__device__ __forceinline__ void mfma16_body(d4 (&acc)[C], double a, double b, int iters) {
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < C; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
  }
}

template <int C>
__device__ __forceinline__ void valu_body(double (&c)[C], double a, double b, int iters) {
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < C; ++j) c[j] = fma(a, b, c[j]);
  }
}

// mode 0: all waves MFMA 16x16x4; 1: all waves MFMA 4x4x4; 2: all waves VALU;
// 3: even waves MFMA16, odd waves VALU; 4: every wave interleaves MFMA16 + VALU
template <int MODE>
__global__ __launch_bounds__(256) void probe(double* out, int iters, int viters) {
  const double a = 1.0 + threadIdx.x * 1e-9, b = 0.999999;
  const int w = threadIdx.x >> 6;
  double s = 0;
  if (MODE == 0 || (MODE == 3 && (w & 1) == 0)) {
    d4 acc[4];
    for (int j = 0; j < 4; ++j) acc[j] = d4{(double)j, 0, 0, 0};
    mfma16_body<4>(acc, a, b, iters);
    for (int j = 0; j < 4; ++j) s += acc[j].x + acc[j].y + acc[j].z + acc[j].w;
  } else if (MODE == 1) {
    double acc[4] = {0, 1, 2, 3};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[j], 0, 0, 0);
    }
    for (int j = 0; j < 4; ++j) s += acc[j];
  } else if (MODE == 2 || MODE == 3) {
    double c[8];
    for (int j = 0; j < 8; ++j) c[j] = j;
    valu_body<8>(c, a, b, viters);
    for (int j = 0; j < 8; ++j) s += c[j];
  } else {
    d4 acc[4];
    double c[8];
    for (int j = 0; j < 4; ++j) acc[j] = d4{(double)j, 0, 0, 0};
    for (int j = 0; j < 8; ++j) c[j] = j;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) c[j] = fma(a, b, c[j]);
    }
    for (int j = 0; j < 4; ++j) s += acc[j].x + acc[j].y + acc[j].z + acc[j].w;
    for (int j = 0; j < 8; ++j) s += c[j];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE>
void run(double* out, int blocks, int iters, int viters, const char* tag) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  probe<MODE><<<blocks, 256>>>(out, iters, viters);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) probe<MODE><<<blocks, 256>>>(out, iters, viters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1000.0 / 5;
  const double waves = (double)blocks * 4;
  double mf = 0, vf = 0;
  if (MODE == 0) mf = waves * iters * 4 * 2048.0;
  if (MODE == 1) mf = waves * iters * 4 * 512.0;
  if (MODE == 2) vf = waves * viters * 8 * 128.0;
  if (MODE == 3) { mf = waves / 2 * iters * 4 * 2048.0; vf = waves / 2 * viters * 8 * 128.0; }
  if (MODE == 4) { mf = waves * iters * 4 * 2048.0; vf = waves * iters * 32 * 128.0; }
  printf("%-34s blocks=%5d %9.1f us  mfma %6.1f TF  valu %6.1f TF  total %6.1f TF\n", tag, blocks,
         us, mf / us / 1e6, vf / us / 1e6, (mf + vf) / us / 1e6);
}

int main() {
  double* out;
  (void)hipMalloc(&out, 64 << 20);
  for (int bpc : {1, 2, 4}) {
    const int blocks = 256 * bpc;
    char tag[64];
    snprintf(tag, 64, "mfma16 (%d wave/SIMD)", bpc);
    run<0>(out, blocks, 2000, 0, tag);
    snprintf(tag, 64, "mfma4x4 (%d wave/SIMD)", bpc);
    run<1>(out, blocks, 2000, 0, tag);
    snprintf(tag, 64, "valu fma (%d wave/SIMD)", bpc);
    run<2>(out, blocks, 0, 16000, tag);
  }
  // mixed: waves alternate; iteration counts chosen so both halves take similar time alone
  for (int vi : {4000, 8000, 16000, 32000}) {
    char tag[64];
    snprintf(tag, 64, "split mfma16|valu vi=%d", vi);
    run<3>(out, 512, 2000, vi, tag);
  }
  run<4>(out, 256, 2000, 0, "same-wave mfma16+valu (1w)");
  run<4>(out, 512, 2000, 0, "same-wave mfma16+valu (2w)");
  return 0;
}
