// Calibration: kernel-duration floor and memory latency on the GPU box (not product code).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void empty_k() {}
__global__ void load_store(const double* __restrict__ a, double* __restrict__ b, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = a[i] * 2.0;
}
__global__ void chase(const int* __restrict__ next, int* __restrict__ out, int steps) {
  int i = (blockIdx.x * blockDim.x + threadIdx.x) & 1023;
  for (int s = 0; s < steps; ++s) i = next[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = i;
}
__global__ void fma_loop(double* __restrict__ out, int iters) {
  double a = threadIdx.x * 1e-3, b = 1.0000001, c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0, c5 = 0, c6 = 0, c7 = 0;
  for (int i = 0; i < iters; ++i) {
    c0 = fma(a, b, c0); c1 = fma(a, b, c1); c2 = fma(a, b, c2); c3 = fma(a, b, c3);
    c4 = fma(a, b, c4); c5 = fma(a, b, c5); c6 = fma(a, b, c6); c7 = fma(a, b, c7);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
}

template <class F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  f();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a);
  for (int i = 0; i < reps; ++i) f();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / reps;
}

int main() {
  const int n = 1 << 24;
  double *a, *b;
  int *nx, *out;
  (void)hipMalloc(&a, n * 8);
  (void)hipMalloc(&b, n * 8);
  (void)hipMalloc(&nx, 1024 * 4);
  (void)hipMalloc(&out, n * 4);
  std::vector<int> h(1024);
  for (int i = 0; i < 1024; ++i) h[i] = (i * 337 + 11) & 1023;
  (void)hipMemcpy(nx, h.data(), 4096, hipMemcpyHostToDevice);
  (void)hipMemset(a, 0, n * 8);
  printf("empty <<<1,64>>>          %7.2f us/launch\n", timeit([] { empty_k<<<1, 64>>>(); }, 2000));
  printf("empty <<<1125,128>>>      %7.2f us/launch\n", timeit([] { empty_k<<<1125, 128>>>(); }, 2000));
  printf("empty <<<4500,256>>>      %7.2f us/launch\n", timeit([] { empty_k<<<4500, 256>>>(); }, 2000));
  for (int m : {1 << 16, 1 << 20, 1 << 22, 1 << 24})
    printf("load_store %8d dbl      %7.2f us/launch (%.0f GB/s)\n", m,
           timeit([&] { load_store<<<(m + 255) / 256, 256>>>(a, b, m); }, 500),
           16.0 * m / (timeit([&] { load_store<<<(m + 255) / 256, 256>>>(a, b, m); }, 500) * 1e3));
  for (int st : {1, 8, 32, 128})
    printf("chase %4d steps (L2)     %7.2f us/launch\n", st, timeit([&] { chase<<<1024, 64>>>(nx, out, st); }, 200));
  for (int it : {1000, 10000})
    printf("fma_loop %6d x8 f64 (1024x256 thr) %7.2f us -> %.1f TFLOP/s\n", it,
           timeit([&] { fma_loop<<<1024, 256>>>(b, it); }, 20),
           1024.0 * 256 * it * 16 / (timeit([&] { fma_loop<<<1024, 256>>>(b, it); }, 20) * 1e6));
  return 0;
}
