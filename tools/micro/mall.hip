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

// The guide's load shape (MI355X_MICROARCH.md, indexed rows / Infinity Cache): 16 B per lane and
// U independent loads in flight per lane (U x 1 KiB per wave; 8 waves per 512-thread workgroup
// -> 64 KiB per workgroup in flight), the grid sized to a few workgroups per CU and striding
template <int U>
__global__ __launch_bounds__(512) void read_seq_u(const d2* __restrict__ y, long long n16, double* __restrict__ out) {
  const long long stride = (long long)gridDim.x * 512 * U;
  double acc = 0.0;
  for (long long base = (long long)blockIdx.x * 512 * U + threadIdx.x; base < n16; base += stride) {
    d2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = y[base + (long long)u * 512 < n16 ? base + (long long)u * 512 : base];
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y;
  }
  if (acc == -1.2345) out[0] = acc;  // keeps the loads
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
  const long long sizes[] = {16 * MB, 38 * MB, 48 * MB, 96 * MB, 128 * MB, 151 * MB, 192 * MB, 256 * MB, 512 * MB, 2048 * MB, 5120 * MB};
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
  printf("%10s %12s %12s %12s %12s %14s %14s %12s %12s\n", "MB", "wr_seq GB/s", "wr_scat GB/s", "rd GB/s", "rd_gath GB/s",
         "scat+rd GB/s", "seq+gath GB/s", "rd_u8 GB/s", "rd_u16 GB/s");
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
    // the guide's shape: 16 B per lane, 8 / 16 loads in flight per lane, 4 workgroups per CU
    const float tu8 = med_us([&] { read_seq_u<8><<<1024, 512>>>(y, n * 16, out); }, 9);
    const float tu16 = med_us([&] { read_seq_u<16><<<1024, 512>>>(y, n * 16, out); }, 9);
    const double gb = S / 1e9;
    printf("%10lld %12.0f %12.0f %12.0f %12.0f %14.0f %14.0f %12.0f %12.0f\n", S / MB, gb / (tw * 1e-6), gb / (ts * 1e-6),
           gb / (tr * 1e-6), gb / (tg * 1e-6), 2 * gb / (trt * 1e-6), 2 * gb / (trt2 * 1e-6), gb / (tu8 * 1e-6),
           gb / (tu16 * 1e-6));
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
