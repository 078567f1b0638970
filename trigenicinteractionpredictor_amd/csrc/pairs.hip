// pairs.hip — MI355X (gfx950) kernels + C ABI (include/mmsbm_pairs.h) for the pair lattice of the
// joint digenic + trigenic model, src/TrigenicInteractionPredictor_23.py (spec fix: DESIGN.md).
//
// The pair loop of make_iteration (:1608-1635) for one pair observation o = (i, j, r, n):
//   dd = eps + th_i^T q_r th_j,  c = n / dd
//   ntheta[i] += th_i (x) c (q_r th_j),  ntheta[j] += th_j (x) c (q_r^T th_i),  nqr_r += q_r (x) c th_i th_j^T
// Grouped by gene (the same regrouping as the triplet engine's pivot runs, one level lower):
//   W^s_{g,r} = sum_{o: slot-s gene of o is g, rating r} c_o th_other(o)       (K per entry)
//   ntheta[g] += q_r W^0_{g,r} + q_r^T W^1_{g,r}                               (2 K^2 per gene)
//   S2_r = sum_g th_g (x) W^0_{g,r},  nqr_r = q_r S2_r                           (K^2 per gene)
// Kernels per iteration (grid.y = sample):
//   pair_c_kernel<K, false>   one thread per observation: dd from q (all ratings staged in LDS),
//                             c written into both of the observation's gather entries
//   pair_gather_kernel<K>     one thread per (gene, slot, rating) run of entries, in entry order;
//                             per workgroup of 128/R genes: ntheta[g] += ..., and the workgroup's
//                             S2 partial sum_g th_g (x) W^0_g
//   pair_s2_kernel            S2 = fixed-order sum of the workgroup partials
// plus pair_qstep_kernel (qr M-step), pair_c_kernel<K, true> + pair_reduce_kernel (likelihood,
// :1549-1559) and pair_predict_kernel<K> (:957-962).  Every sum has a fixed order: results are
// bitwise reproducible and do not depend on the batch.  The pair work is O(K^2) per
// observation and the gather O(K) per entry (FP64 VALU; the 2 K^2 / K^3 gene terms are tiny),
// so no MFMA here: these kernels are latency / L2 bound.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <utility>
#include <vector>

#include "mmsbm_pairs.h"

int mmsbm_detail_fail(int code, const char* msg);  // mmsbm.hip: the library's error channel

namespace {

constexpr int PNT = 256;  // threads per workgroup of every pair kernel
constexpr int MAX_R = 8;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  return mmsbm_detail_fail(code, buf);
}

#define HIP_TRY(expr)                                                                          \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess) return fail(MMSBM_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

// per-iteration intermediates leave the XCD L2 while the kernel runs (mmsbm.hip, st_wt)
__device__ __forceinline__ void st_wt(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) v += __shfl_xor(v, s, 64);
  return v;
}

// genes per gather workgroup: one thread per (gene, slot, rating)
__host__ __device__ constexpr int gather_genes(int R) { return PNT / (2 * R); }

// ------------------------------------------------------------------------------------------
// c per observation (EM), or sum n log dd per workgroup (LL).  obs[o] = (i, j, n, r).
// ------------------------------------------------------------------------------------------
template <int K, bool LL>
__global__ __launch_bounds__(PNT) void pair_c_kernel(const int4* __restrict__ obs,
                                                     const int2* __restrict__ pos, int n_obs,
                                                     int n_ent, const double* __restrict__ theta,
                                                     const double* __restrict__ qr,
                                                     double* __restrict__ cent,
                                                     double* __restrict__ part, int P, int R,
                                                     double eps) {
  constexpr int K2 = K * K;
  extern __shared__ double qs[];  // q of every rating, [R][K][K]
  const int b = blockIdx.y;
  const double* __restrict__ q = qr + (size_t)b * R * K2;
  for (int t = threadIdx.x; t < R * K2; t += PNT) qs[t] = q[t];
  __syncthreads();
  const int o = blockIdx.x * PNT + threadIdx.x;
  double v = 0.0;
  if (o < n_obs) {
    const int4 ob = obs[o];
    const double* __restrict__ th = theta + (size_t)b * P * K;
    const double* __restrict__ ti = th + (size_t)ob.x * K;
    const double* __restrict__ tj = th + (size_t)ob.y * K;
    double rj[K];
#pragma unroll
    for (int x = 0; x < K; ++x) rj[x] = tj[x];
    const double* qq = qs + ob.w * K2;
    double dd = 0.0;
    for (int a = 0; a < K; ++a) {
      double u = 0.0;
#pragma unroll
      for (int x = 0; x < K; ++x) u = fma(qq[a * K + x], rj[x], u);
      dd = fma(ti[a], u, dd);
    }
    dd = eps + dd;
    if constexpr (LL) {
      v = (double)ob.z * log(dd);
    } else {
      const double c = (double)ob.z / dd;
      const int2 p = pos[o];
      double* ce = cent + (size_t)b * n_ent;
      st_wt(ce + p.x, c);
      st_wt(ce + p.y, c);
    }
  }
  if constexpr (LL) {
    __shared__ double red[PNT / 64];
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
      double s = 0.0;
      for (int w = 0; w < PNT / 64; ++w) s += red[w];
      part[(size_t)b * gridDim.x + blockIdx.x] = s;
    }
  }
}

// ------------------------------------------------------------------------------------------
// Gather.  Entries are ordered by (gene, slot, rating), then observation; gptr[(g 2 + s) R + r]
// opens each run.  Thread t of a workgroup owns run (gene gl = t / 2R, slot, rating) of the
// workgroup's G = 128 / R genes and sums c th_other over it in entry order (registers).
// LDS: q [R][K][K], W [G][2][R][K] (the runs' sums), th rows of the G genes.
// ------------------------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__(PNT) void pair_gather_kernel(const int* __restrict__ gptr,
                                                          const int* __restrict__ oth,
                                                          const double* __restrict__ cent,
                                                          const double* __restrict__ theta,
                                                          const double* __restrict__ qr,
                                                          double* __restrict__ nth,
                                                          double* __restrict__ s2part, int n_ent,
                                                          int P, int R) {
  constexpr int K2 = K * K;
  const int G = gather_genes(R), NR = 2 * R;
  extern __shared__ double sm[];
  double* qs = sm;                 // R K2
  double* ws = qs + R * K2;        // G NR K
  double* ths = ws + G * NR * K;   // G K
  const int b = blockIdx.y, tid = threadIdx.x;
  const double* __restrict__ q = qr + (size_t)b * R * K2;
  const double* __restrict__ th = theta + (size_t)b * P * K;
  const double* __restrict__ ce = cent + (size_t)b * n_ent;
  const int g0 = blockIdx.x * G;
  for (int t = tid; t < R * K2; t += PNT) qs[t] = q[t];
  for (int t = tid; t < G * K; t += PNT) {
    const int g = g0 + t / K;
    ths[t] = g < P ? th[(size_t)g * K + t % K] : 0.0;
  }
  {
    double acc[K];
#pragma unroll
    for (int x = 0; x < K; ++x) acc[x] = 0.0;
    const int gl = tid / NR, sr = tid % NR, g = g0 + gl;
    if (gl < G && g < P) {
      const int lo = gptr[(size_t)g * NR + sr], hi = gptr[(size_t)g * NR + sr + 1];
      int e = lo;
      for (; e + 1 < hi; e += 2) {  // two entries' loads in flight
        const int o0 = oth[e], o1 = oth[e + 1];
        const double c0 = ce[e], c1 = ce[e + 1];
        const double* __restrict__ t0 = th + (size_t)o0 * K;
        const double* __restrict__ t1 = th + (size_t)o1 * K;
        double r0[K], r1[K];
#pragma unroll
        for (int x = 0; x < K; ++x) {
          r0[x] = t0[x];
          r1[x] = t1[x];
        }
#pragma unroll
        for (int x = 0; x < K; ++x) acc[x] = fma(c1, r1[x], fma(c0, r0[x], acc[x]));
      }
      if (e < hi) {
        const double c0 = ce[e];
        const double* __restrict__ t0 = th + (size_t)oth[e] * K;
#pragma unroll
        for (int x = 0; x < K; ++x) acc[x] = fma(c0, t0[x], acc[x]);
      }
    }
    if (gl < G) {
#pragma unroll
      for (int x = 0; x < K; ++x) ws[(gl * NR + sr) * K + x] = acc[x];
    }
  }
  __syncthreads();
  // ntheta[g][a] += sum_r (q_r W^0_r)[a] + (q_r^T W^1_r)[a], rating order
  for (int t = tid; t < G * K; t += PNT) {
    const int gl = t / K, a = t % K, g = g0 + gl;
    if (g >= P) continue;
    const double* w = ws + gl * NR * K;
    double s = 0.0;
    for (int r = 0; r < R; ++r) {
      const double* qq = qs + r * K2;
      const double* w0 = w + r * K;
      const double* w1 = w + (R + r) * K;
#pragma unroll
      for (int y = 0; y < K; ++y) s = fma(qq[a * K + y], w0[y], s);
#pragma unroll
      for (int y = 0; y < K; ++y) s = fma(qq[y * K + a], w1[y], s);
    }
    double* dst = nth + ((size_t)b * P + g) * K + a;
    *dst = *dst + s;
  }
  // S2 partial of the workgroup's genes: cells (r, a, y)
  double* out = s2part + ((size_t)b * gridDim.x + blockIdx.x) * R * K2;
  for (int t = tid; t < R * K2; t += PNT) {
    const int r = t / K2, a = (t / K) % K, y = t % K;
    double s = 0.0;
    for (int gl = 0; gl < G; ++gl) s = fma(ths[gl * K + a], ws[(gl * NR + r) * K + y], s);
    st_wt(out + t, s);
  }
}

// S2[b][cell] = sum over gather workgroups of the partials, in workgroup order.
__global__ __launch_bounds__(PNT) void pair_s2_kernel(const double* __restrict__ s2part, int nblk,
                                                      int ncell, double* __restrict__ S2) {
  const int b = blockIdx.y, cell = blockIdx.x * PNT + threadIdx.x;
  if (cell >= ncell) return;
  const double* p = s2part + (size_t)b * nblk * ncell + cell;
  double s = 0.0;
  for (int k = 0; k < nblk; ++k) s += p[(size_t)k * ncell];
  S2[(size_t)b * ncell + cell] = s;
}

// qr <- qr S2 / (eps + sum_r qr S2)   (:1660-1666)
__global__ __launch_bounds__(PNT) void pair_qstep_kernel(double* __restrict__ qr,
                                                         const double* __restrict__ S2, int K2,
                                                         int R, double eps) {
  const int b = blockIdx.y, cell = blockIdx.x * PNT + threadIdx.x;
  if (cell >= K2) return;
  double nq[MAX_R];
  double den = eps;
  double* qc = qr + (size_t)b * R * K2 + cell;
  const double* sc = S2 + (size_t)b * R * K2 + cell;
  for (int r = 0; r < R; ++r) {
    nq[r] = qc[(size_t)r * K2] * sc[(size_t)r * K2];
    den += nq[r];
  }
  for (int r = 0; r < R; ++r) qc[(size_t)r * K2] = nq[r] / den;
}

__global__ __launch_bounds__(PNT) void pair_reduce_kernel(const double* __restrict__ part, int n,
                                                          double* __restrict__ out) {
  __shared__ double red[PNT / 64];
  const int b = blockIdx.x;
  double s = 0.0;
  for (int t = threadIdx.x; t < n; t += PNT) s += part[(size_t)b * n + t];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < PNT / 64; ++w) t += red[w];
    out[b] = t;
  }
}

// P(r = 1) of a pair (:957-962), no eps.  grid (ceil(n / 256), B).
template <int K>
__global__ __launch_bounds__(PNT) void pair_predict_kernel(const int* __restrict__ ids, long long n,
                                                           const double* __restrict__ theta,
                                                           const double* __restrict__ qr,
                                                           double* __restrict__ out, int P, int R) {
  constexpr int K2 = K * K;
  const int b = blockIdx.y;
  const long long row = (long long)blockIdx.x * PNT + threadIdx.x;
  if (row >= n) return;
  const int gi = ids[2 * row], gj = ids[2 * row + 1];
  if (gi < 0 || gi >= P || gj < 0 || gj >= P) {
    out[(size_t)b * n + row] = __builtin_nan("");
    return;
  }
  const double* __restrict__ th = theta + (size_t)b * P * K;
  const double* __restrict__ q = qr + ((size_t)b * R + 1) * K2;
  const double* ti = th + (size_t)gi * K;
  const double* tj = th + (size_t)gj * K;
  double rj[K];
#pragma unroll
  for (int x = 0; x < K; ++x) rj[x] = tj[x];
  double p = 0.0;
  for (int a = 0; a < K; ++a) {
    double u = 0.0;
#pragma unroll
    for (int x = 0; x < K; ++x) u = fma(q[a * K + x], rj[x], u);
    p = fma(ti[a], u, p);
  }
  out[(size_t)b * n + row] = p;
}

// ------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------
struct PairSet {
  bool present = false;
  int n_obs = 0, n_ent = 0;
  int4* obs = nullptr;   // (i, j, n, r)
  int2* pos = nullptr;   // the observation's two gather entries (train only)
  int* gptr = nullptr;   // [P 2 R + 1] (train only)
  int* oth = nullptr;    // [n_ent] the other gene of each entry (train only)
  void release() {
    void* ps[] = {obs, pos, gptr, oth};
    for (void* p : ps)
      if (p) (void)hipFree(p);
    *this = PairSet();
  }
};

}  // namespace

struct mmsbm_pairs_ctx {
  int device = 0;
  int K = 0, R = 0, B = 0, P = 0;
  double eps = 1e-10;
  PairSet sets[2];
  char* ws = nullptr;
  long long ws_bytes = 0;
  double *cent = nullptr, *s2part = nullptr, *llpart = nullptr;
  unsigned attr = 0;  // gather kernels opted in to > 64 KB of LDS
};

namespace {

size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

int gather_blocks(const mmsbm_pairs_ctx* c) {
  const int G = gather_genes(c->R);
  return (c->P + G - 1) / G;
}

int c_blocks(int n_obs) { return (n_obs + PNT - 1) / PNT; }

struct PairWs {
  size_t cent, s2part, llpart, total;
};

PairWs ws_layout(const mmsbm_pairs_ctx* c) {
  PairWs L{};
  const size_t B = c->B, K2 = (size_t)c->K * c->K;
  size_t off = 0;
  L.cent = off;
  off += align_up(B * std::max(c->sets[MMSBM_SET_TRAIN].n_ent, 1) * 8);
  L.s2part = off;
  off += align_up(B * gather_blocks(c) * c->R * K2 * 8);
  L.llpart = off;
  off += align_up(B * std::max({c_blocks(c->sets[0].n_obs), c_blocks(c->sets[1].n_obs), 1}) * 8);
  L.total = off;
  return L;
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

template <typename D, typename T>
int upload(D** dst, const std::vector<T>& src) {
  static_assert(sizeof(D) == sizeof(T), "element size");
  if (src.empty()) return MMSBM_OK;
  HIP_TRY(hipMalloc(reinterpret_cast<void**>(dst), src.size() * sizeof(T)));
  HIP_TRY(hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
  return MMSBM_OK;
}

struct PLaunch {
  int (*accumulate)(mmsbm_pairs_ctx*, const double*, const double*, double*, double*, hipStream_t);
  int (*loglik)(mmsbm_pairs_ctx*, int, const double*, const double*, double*, hipStream_t);
  int (*predict)(mmsbm_pairs_ctx*, const int*, long long, const double*, const double*, double*,
                 hipStream_t);
};

template <int K>
int launch_accumulate(mmsbm_pairs_ctx* c, const double* theta, const double* qr, double* nth,
                      double* S2, hipStream_t s) {
  const PairSet& ps = c->sets[MMSBM_SET_TRAIN];
  const int K2 = K * K, ncell = c->R * K2;
  if (ps.n_obs == 0) {
    HIP_TRY(hipMemsetAsync(S2, 0, sizeof(double) * c->B * ncell, s));
    return MMSBM_OK;
  }
  pair_c_kernel<K, false><<<dim3(c_blocks(ps.n_obs), c->B), PNT, ncell * 8, s>>>(
      ps.obs, ps.pos, ps.n_obs, ps.n_ent, theta, qr, c->cent, nullptr, c->P, c->R, c->eps);
  HIP_TRY(hipGetLastError());
  const int G = gather_genes(c->R), nblk = gather_blocks(c);
  const int lds = (ncell + G * 2 * c->R * K + G * K) * 8;
  if (lds > 64 * 1024 && !(c->attr & (1u << (K - 1)))) {
    HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&pair_gather_kernel<K>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    c->attr |= 1u << (K - 1);
  }
  pair_gather_kernel<K><<<dim3(nblk, c->B), PNT, lds, s>>>(ps.gptr, ps.oth, c->cent, theta, qr, nth,
                                                          c->s2part, ps.n_ent, c->P, c->R);
  HIP_TRY(hipGetLastError());
  pair_s2_kernel<<<dim3((ncell + PNT - 1) / PNT, c->B), PNT, 0, s>>>(c->s2part, nblk, ncell, S2);
  HIP_TRY(hipGetLastError());
  return MMSBM_OK;
}

template <int K>
int launch_loglik(mmsbm_pairs_ctx* c, int which, const double* theta, const double* qr, double* out,
                  hipStream_t s) {
  const PairSet& ps = c->sets[which];
  if (!ps.present || ps.n_obs == 0) {
    HIP_TRY(hipMemsetAsync(out, 0, sizeof(double) * c->B, s));
    return MMSBM_OK;
  }
  const int nb = c_blocks(ps.n_obs);
  pair_c_kernel<K, true><<<dim3(nb, c->B), PNT, c->R * K * K * 8, s>>>(
      ps.obs, nullptr, ps.n_obs, 0, theta, qr, nullptr, c->llpart, c->P, c->R, c->eps);
  HIP_TRY(hipGetLastError());
  pair_reduce_kernel<<<c->B, PNT, 0, s>>>(c->llpart, nb, out);
  HIP_TRY(hipGetLastError());
  return MMSBM_OK;
}

template <int K>
int launch_predict(mmsbm_pairs_ctx* c, const int* ids, long long n, const double* theta,
                   const double* qr, double* out, hipStream_t s) {
  if (n == 0) return MMSBM_OK;
  pair_predict_kernel<K><<<dim3((unsigned)((n + PNT - 1) / PNT), c->B), PNT, 0, s>>>(ids, n, theta, qr,
                                                                                     out, c->P, c->R);
  HIP_TRY(hipGetLastError());
  return MMSBM_OK;
}

template <int... Ks>
constexpr auto make_table(std::integer_sequence<int, Ks...>) {
  return std::array<PLaunch, sizeof...(Ks)>{
      PLaunch{&launch_accumulate<Ks + 1>, &launch_loglik<Ks + 1>, &launch_predict<Ks + 1>}...};
}

const auto kPTable = make_table(std::make_integer_sequence<int, MMSBM_MAX_K>{});

int check_shape(const mmsbm_pairs_ctx* c) {
  if (c->K < 1 || c->K > MMSBM_MAX_K)
    return fail(MMSBM_ERR_UNSUPPORTED, "K=%d outside [1, %d]: call mmsbm_pairs_set_shape", c->K,
                MMSBM_MAX_K);
  return MMSBM_OK;
}

}  // namespace

extern "C" {

int mmsbm_pairs_create(int device, mmsbm_pairs_ctx** out) {
  if (!out) return fail(MMSBM_ERR_INVALID, "out is null");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(MMSBM_ERR_INVALID, "device %d outside [0, %d)", device, ndev);
  auto* c = new mmsbm_pairs_ctx();
  c->device = device;
  *out = c;
  return MMSBM_OK;
}

int mmsbm_pairs_destroy(mmsbm_pairs_ctx* c) {
  if (!c) return MMSBM_OK;
  DeviceGuard g(c->device);
  for (auto& s : c->sets) s.release();
  delete c;
  return MMSBM_OK;
}

int mmsbm_pairs_set_shape(mmsbm_pairs_ctx* c, int32_t K, int32_t R, int32_t B, int32_t P, double eps) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  if (K < 1 || K > MMSBM_MAX_K) return fail(MMSBM_ERR_UNSUPPORTED, "K=%d outside [1, %d]", K, MMSBM_MAX_K);
  if (R < 2 || R > MAX_R) return fail(MMSBM_ERR_UNSUPPORTED, "R=%d outside [2, %d]", R, MAX_R);
  if (B < 1 || B > 65535) return fail(MMSBM_ERR_INVALID, "B=%d outside [1, 65535]", B);
  if (P < 1) return fail(MMSBM_ERR_INVALID, "P=%d < 1", P);
  if (!(eps >= 0.0)) return fail(MMSBM_ERR_INVALID, "eps must be >= 0");
  for (auto& s : c->sets)
    if (s.present && (c->P != P || c->R != R)) {
      DeviceGuard g(c->device);
      s.release();  // plans depend on P and R
    }
  c->K = K;
  c->R = R;
  c->B = B;
  c->P = P;
  c->eps = eps;
  c->ws = nullptr;
  return MMSBM_OK;
}

int mmsbm_pairs_set_links(mmsbm_pairs_ctx* c, int32_t which, const int32_t* ids_host,
                          const int32_t* counts_host, int64_t E) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  int rc = check_shape(c);
  if (rc) return rc;
  if (which != MMSBM_SET_TRAIN && which != MMSBM_SET_TEST) return fail(MMSBM_ERR_INVALID, "which=%d", which);
  if (E < 0 || (E > 0 && (!ids_host || !counts_host))) return fail(MMSBM_ERR_INVALID, "bad link table");
  if (E * c->R * 2 >= ((int64_t)1 << 31)) return fail(MMSBM_ERR_UNSUPPORTED, "E=%lld too large", (long long)E);
  for (int64_t q = 0; q < E * 2; ++q)
    if (ids_host[q] < 0 || ids_host[q] >= c->P)
      return fail(MMSBM_ERR_INVALID, "gene id %d outside [0, P=%d)", ids_host[q], c->P);
  for (int64_t q = 0; q < E * c->R; ++q)
    if (counts_host[q] < 0) return fail(MMSBM_ERR_INVALID, "negative count");
  DeviceGuard g(c->device);
  PairSet& ps = c->sets[which];
  ps.release();
  const int R = c->R, NR = 2 * R;
  // observations: every (link, r) with n > 0, in link order (a zero count adds exactly zero)
  std::vector<int4> obs;
  for (int64_t e = 0; e < E; ++e)
    for (int r = 0; r < R; ++r) {
      const int n = counts_host[e * R + r];
      if (n > 0) obs.push_back(make_int4(ids_host[2 * e], ids_host[2 * e + 1], n, r));
    }
  ps.n_obs = (int)obs.size();
  if ((rc = upload(&ps.obs, obs))) return rc;
  if (which == MMSBM_SET_TRAIN) {
    // gather entries: two per observation, counting-sorted by (gene, slot, rating), stable
    std::vector<int> gptr((size_t)c->P * NR + 1, 0);
    for (const int4& o : obs) {
      gptr[(size_t)o.x * NR + o.w + 1]++;
      gptr[(size_t)o.y * NR + R + o.w + 1]++;
    }
    for (size_t k = 1; k < gptr.size(); ++k) gptr[k] += gptr[k - 1];
    std::vector<int> fill(gptr.begin(), gptr.end() - 1);
    ps.n_ent = 2 * ps.n_obs;
    std::vector<int> oth(std::max(ps.n_ent, 1), 0);
    std::vector<int2> pos(std::max(ps.n_obs, 1));
    for (int o = 0; o < ps.n_obs; ++o) {
      const int4& ob = obs[o];
      const int p0 = fill[(size_t)ob.x * NR + ob.w]++;
      const int p1 = fill[(size_t)ob.y * NR + R + ob.w]++;
      oth[p0] = ob.y;
      oth[p1] = ob.x;
      pos[o] = make_int2(p0, p1);
    }
    if ((rc = upload(&ps.gptr, gptr))) return rc;
    if ((rc = upload(&ps.oth, oth))) return rc;
    if ((rc = upload(&ps.pos, pos))) return rc;
  }
  ps.present = true;
  c->ws = nullptr;  // the workspace layout changed
  return MMSBM_OK;
}

int mmsbm_pairs_workspace_bytes(const mmsbm_pairs_ctx* c, int64_t* bytes) {
  if (!c || !bytes) return fail(MMSBM_ERR_INVALID, "null argument");
  *bytes = (int64_t)ws_layout(c).total;
  return MMSBM_OK;
}

int mmsbm_pairs_set_workspace(mmsbm_pairs_ctx* c, void* ws, int64_t bytes) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  const PairWs L = ws_layout(c);
  if (bytes < (int64_t)L.total)
    return fail(MMSBM_ERR_INVALID, "workspace %lld < %lld bytes", (long long)bytes, (long long)L.total);
  if (((uintptr_t)ws) & 255) return fail(MMSBM_ERR_INVALID, "workspace not 256-B aligned");
  c->ws = (char*)ws;
  c->ws_bytes = bytes;
  c->cent = (double*)(c->ws + L.cent);
  c->s2part = (double*)(c->ws + L.s2part);
  c->llpart = (double*)(c->ws + L.llpart);
  return MMSBM_OK;
}

static int check_ready(const mmsbm_pairs_ctx* c) {
  int rc = check_shape(c);
  if (rc) return rc;
  if (!c->sets[MMSBM_SET_TRAIN].present) return fail(MMSBM_ERR_INVALID, "train pairs not set");
  if (!c->ws || c->ws_bytes < (long long)ws_layout(c).total)
    return fail(MMSBM_ERR_INVALID, "workspace missing or too small (mmsbm_pairs_workspace_bytes)");
  return MMSBM_OK;
}

int mmsbm_pairs_accumulate(mmsbm_pairs_ctx* c, const double* theta, const double* qr, double* nth,
                           double* S2, void* stream) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  int rc = check_ready(c);
  if (rc) return rc;
  if (!theta || !qr || !nth || !S2) return fail(MMSBM_ERR_INVALID, "null pointer");
  DeviceGuard g(c->device);
  return kPTable[c->K - 1].accumulate(c, theta, qr, nth, S2, (hipStream_t)stream);
}

int mmsbm_pairs_qstep(mmsbm_pairs_ctx* c, double* qr, const double* S2, void* stream) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  int rc = check_shape(c);
  if (rc) return rc;
  if (!qr || !S2) return fail(MMSBM_ERR_INVALID, "null pointer");
  DeviceGuard g(c->device);
  const int K2 = c->K * c->K;
  pair_qstep_kernel<<<dim3((K2 + PNT - 1) / PNT, c->B), PNT, 0, (hipStream_t)stream>>>(qr, S2, K2, c->R,
                                                                                       c->eps);
  HIP_TRY(hipGetLastError());
  return MMSBM_OK;
}

int mmsbm_pairs_loglik(mmsbm_pairs_ctx* c, int32_t which, const double* theta, const double* qr,
                       double* out, void* stream) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  int rc = check_shape(c);
  if (rc) return rc;
  if (which != MMSBM_SET_TRAIN && which != MMSBM_SET_TEST) return fail(MMSBM_ERR_INVALID, "which=%d", which);
  if (!c->ws) return fail(MMSBM_ERR_INVALID, "workspace missing");
  if (!theta || !qr || !out) return fail(MMSBM_ERR_INVALID, "null pointer");
  DeviceGuard g(c->device);
  return kPTable[c->K - 1].loglik(c, which, theta, qr, out, (hipStream_t)stream);
}

int mmsbm_pairs_predict(mmsbm_pairs_ctx* c, const int32_t* ids, int64_t n, const double* theta,
                        const double* qr, double* out, void* stream) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  int rc = check_shape(c);
  if (rc) return rc;
  if (n < 0 || (n > 0 && (!ids || !theta || !qr || !out))) return fail(MMSBM_ERR_INVALID, "bad arguments");
  DeviceGuard g(c->device);
  return kPTable[c->K - 1].predict(c, ids, n, theta, qr, out, (hipStream_t)stream);
}

int mmsbm_pairs_plan_info(const mmsbm_pairs_ctx* c, int32_t which, int64_t* info) {
  if (!c || !info || (which != MMSBM_SET_TRAIN && which != MMSBM_SET_TEST))
    return fail(MMSBM_ERR_INVALID, "bad arguments");
  const PairSet& ps = c->sets[which];
  info[0] = ps.n_obs;
  info[1] = ps.n_ent;
  info[2] = which == MMSBM_SET_TRAIN ? gather_blocks(c) : 0;
  info[3] = c_blocks(ps.n_obs);
  return MMSBM_OK;
}

}  // extern "C"
