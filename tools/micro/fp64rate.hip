// Calibration: FP64 FMA issue rate vs waves per SIMD and independent chains (not product code).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int C>
__global__ void fma_chains(double* __restrict__ out, int iters) {
  double a = threadIdx.x * 1e-3, b = 1.0000001, c[C];
#pragma unroll
  for (int j = 0; j < C; ++j) c[j] = j;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < C; ++j) c[j] = fma(a, b, c[j]);
  }
  double s = 0;
#pragma unroll
  for (int j = 0; j < C; ++j) s += c[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int C>
void run(double* out, int blocks, int threads, const char* tag) {
  const int iters = 4000;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  fma_chains<C><<<blocks, threads>>>(out, iters);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int r = 0; r < 5; ++r) fma_chains<C><<<blocks, threads>>>(out, iters);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  const double us = ms * 1000.0 / 5;
  const double flops = 2.0 * C * iters * (double)blocks * threads;
  const double waves_per_simd = (double)blocks * threads / 64 / 1024;
  // cycles per wave-instruction per SIMD at 2.4 GHz
  const double insts_per_simd = (double)C * iters * waves_per_simd;
  printf("%-28s chains=%2d waves/SIMD=%5.2f  %8.1f us  %6.1f TFLOP/s  %5.2f cyc/inst@2.4GHz\n", tag, C,
         waves_per_simd, us, flops / us / 1e6, us * 2400.0 / insts_per_simd);
}

int main() {
  double* out;
  (void)hipMalloc(&out, 64 << 20);
  run<8>(out, 256, 256, "1 wave/SIMD");
  run<4>(out, 256, 256, "1 wave/SIMD");
  run<2>(out, 256, 256, "1 wave/SIMD");
  run<16>(out, 256, 256, "1 wave/SIMD");
  run<8>(out, 512, 256, "2 waves/SIMD");
  run<4>(out, 512, 256, "2 waves/SIMD");
  run<8>(out, 1024, 256, "4 waves/SIMD");
  run<4>(out, 1024, 256, "4 waves/SIMD");
  run<2>(out, 1024, 256, "4 waves/SIMD");
  run<8>(out, 2048, 256, "8 waves/SIMD");
  return 0;
}
