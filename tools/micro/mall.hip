// Calibration (not product code): does a write-then-read round trip of a region stay on die (the
// 256 MiB Infinity Cache) when the region is small, and what does it cost when it is not?  Models
// the large-K Y entries: 256-B entries (32 doubles) written scattered (entry order permuted), then
// read back in entry order, one 16-lane group per entry.
//   ./mall   -> one line per region size: write GB/s, read GB/s, write+read round trip GB/s (bytes
//               counted once per direction), each the median of several passes
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double d2 __attribute__((ext_vector_type(2)));

// 16 lanes per 256-B entry, 16 B per lane; entry e written at slot perm[e]
__global__ __launch_bounds__(256) void write_scatter(d2* __restrict__ y, const int* __restrict__ perm, long long n_ent,
                                                     double v) {
  const long long g = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long e = g >> 4;
  if (e >= n_ent) return;
  const int l = threadIdx.x & 15;
  y[(long long)perm[e] * 16 + l] = d2{v + l, v - l};
}

__global__ __launch_bounds__(256) void write_seq(d2* __restrict__ y, long long n_ent, double v) {
  const long long g = (long long)blockIdx.x * 256 + threadIdx.x;
  if ((g >> 4) >= n_ent) return;
  y[g] = d2{v, v + 1.0};
}

// 16 lanes per 256-B entry: entry e read from slot perm[e] (a gather of whole entries)
__global__ __launch_bounds__(256) void read_gather(const d2* __restrict__ y, const int* __restrict__ perm, long long n_ent,
                                                   double* __restrict__ out) {
  const long long g = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long e = g >> 4;
  if (e >= n_ent) return;
  const d2 a = y[(long long)perm[e] * 16 + (threadIdx.x & 15)];
  if (a.x == -1.2345) out[0] = a.y;
}

__global__ __launch_bounds__(256) void read_seq(const d2* __restrict__ y, long long n_ent, double* __restrict__ out) {
  const long long g = (long long)blockIdx.x * 256 + threadIdx.x;
  if ((g >> 4) >= n_ent) return;
  const d2 a = y[g];
  if (a.x == -1.2345) out[0] = a.y;  // keeps the load
}

template <class F>
float med_us(F f, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  std::vector<float> t;
  f();
  for (int i = 0; i < reps; ++i) {
    (void)hipEventRecord(a);
    f();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    t.push_back(ms * 1000.f);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main() {
  const long long MB = 1 << 20;
  const long long sizes[] = {16 * MB, 48 * MB, 96 * MB, 128 * MB, 192 * MB, 256 * MB, 512 * MB, 2048 * MB, 5120 * MB};
  const long long maxb = 5120 * MB;
  d2* y;
  int* perm;
  double* out;
  if (hipMalloc(&y, maxb) != hipSuccess || hipMalloc(&perm, maxb / 256 * 4) != hipSuccess ||
      hipMalloc(&out, 64) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  std::vector<int> h(maxb / 256);
  printf("%10s %12s %12s %12s %12s %14s %14s\n", "MB", "wr_seq GB/s", "wr_scat GB/s", "rd GB/s", "rd_gath GB/s",
         "scat+rd GB/s", "seq+gath GB/s");
  double base_rt = 0;
  std::vector<double> rts;
  for (long long S : sizes) {
    const long long n = S / 256;
    for (long long i = 0; i < n; ++i) h[i] = (int)i;
    srand(7);
    for (long long i = n - 1; i > 0; --i) std::swap(h[i], h[rand() % (i + 1)]);
    (void)hipMemcpy(perm, h.data(), n * 4, hipMemcpyHostToDevice);
    const unsigned nb = (unsigned)((n * 16 + 255) / 256);
    const float tw = med_us([&] { write_seq<<<nb, 256>>>(y, n, 1.0); }, 9);
    const float ts = med_us([&] { write_scatter<<<nb, 256>>>(y, perm, n, 1.0); }, 9);
    const float tr = med_us([&] { read_seq<<<nb, 256>>>(y, n, out); }, 9);
    const float tg = med_us([&] { read_gather<<<nb, 256>>>(y, perm, n, out); }, 9);
    const float trt = med_us([&] {
      write_scatter<<<nb, 256>>>(y, perm, n, 2.0);
      read_seq<<<nb, 256>>>(y, n, out);
    }, 9);
    const float trt2 = med_us([&] {
      write_seq<<<nb, 256>>>(y, n, 2.0);
      read_gather<<<nb, 256>>>(y, perm, n, out);
    }, 9);
    const double gb = S / 1e9;
    printf("%10lld %12.0f %12.0f %12.0f %12.0f %14.0f %14.0f\n", S / MB, gb / (tw * 1e-6), gb / (ts * 1e-6),
           gb / (tr * 1e-6), gb / (tg * 1e-6), 2 * gb / (trt * 1e-6), 2 * gb / (trt2 * 1e-6));
    rts.push_back(2 * gb / (trt * 1e-6));
  }
  // ring of two 96 MB regions against one 5 GB stream, same bytes: 52 write+read round trips
  {
    const long long S = 96 * MB, n = S / 256;
    for (long long i = 0; i < n; ++i) h[i] = (int)i;
    srand(9);
    for (long long i = n - 1; i > 0; --i) std::swap(h[i], h[rand() % (i + 1)]);
    (void)hipMemcpy(perm, h.data(), n * 4, hipMemcpyHostToDevice);
    const unsigned nb = (unsigned)((n * 16 + 255) / 256);
    const float t = med_us([&] {
      for (int k = 0; k < 52; ++k) {
        d2* r = y + (long long)(k & 1) * (S / 16);
        write_scatter<<<nb, 256>>>(r, perm, n, 3.0);
        read_seq<<<nb, 256>>>(r, n, out);
      }
    }, 3);
    printf("ring 2 x 96 MB, 52 round trips (%.2f GB each way): %.0f us, %.0f GB/s\n", 52 * S / 1e9, t,
           2 * 52 * S / 1e9 / (t * 1e-6));
  }
  return 0;
}
