// pairs.hip — MI355X (gfx950) kernels + C ABI (include/mmsbm_pairs.h) for the pair lattice of the
// joint digenic + trigenic model, src/TrigenicInteractionPredictor_23.py (spec fix: DESIGN.md).
//
// The pair loop of make_iteration (:1608-1635) for one pair observation o = (i, j, r, n):
//   dd = eps + th_i^T q_r th_j,  c = n / dd
//   ntheta[i] += th_i (x) c (q_r th_j),  ntheta[j] += th_j (x) c (q_r^T th_i),  nqr_r += q_r (x) c th_i th_j^T
// Grouped by gene (the triplet engine's pivot runs, one level lower).  A run = the gather entries
// of one (gene g, slot s, rating r); an entry = the observation's other gene and count:
//   V_{g,r} = q_r^T th_g (slot 0),  U_{g,r} = q_r th_g (slot 1)            2 K^2 per (gene, rating)
//   dd = eps + V.th_other (or U.th_other),  c = n / dd                      K per entry
//   W^s_{g,r} = sum over the run of c th_other                               K per entry
//   ntheta[g] += q_r W^0_{g,r} + q_r^T W^1_{g,r}                             2 K^2 per gene
//   S2_r = sum_g th_g (x) W^0_{g,r},  nqr_r = q_r S2_r                         K^2 per gene
// so one kernel does the whole pair half of an iteration (pair_em_kernel<K, MODE>): a workgroup
// owns a block of consecutive genes; V / U of its genes in LDS; one thread per *part* (a run is
// split into parts of <= 8 entries, at most 32 parts, so no thread walks a long serial chain)
// sums c th_other with NF entries' loads in flight; the parts of a run are added in order; the
// genes' ntheta terms and the block's S2 partial follow; the last workgroup of each sample (one
// agent-scope ticket) adds the S2 partials in workgroup order and writes S2 (MODE_ADD,
// mmsbm_pairs_accumulate); in the fused joint iteration (MODE_FUSED, mmsbm_joint_iterate) the
// partials are left for the q cells of the triplet engine's fin_kernel, which sums them and
// applies the qr M-step (no ticket, no serial tail).  pair_ll_kernel<K> + pair_reduce_kernel give the likelihood (:1549-1559),
// pair_predict_kernel<K> the prediction (:957-962).  Every sum has a fixed order: results are
// bitwise reproducible and do not depend on the batch.  The work is O(K) per entry and O(K^2)
// per gene (FP64 VALU; nothing GEMM-shaped enough for MFMA at these sizes): latency / L2 bound.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
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

// ------------------------------------------------------------------------------------------
// Likelihood: sum n log dd per workgroup (obs[o] = (i, j, n, r); q of every rating in LDS).
// ------------------------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__(PNT) void pair_ll_kernel(const int4* __restrict__ obs, int n_obs,
                                                      const double* __restrict__ theta,
                                                      const double* __restrict__ qr,
                                                      double* __restrict__ part, int P, int R,
                                                      double eps) {
  constexpr int K2 = K * K;
  extern __shared__ double qs[];  // [R][K][K]
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
    v = (double)ob.z * log(eps + dd);
  }
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

// ------------------------------------------------------------------------------------------
// The pair half of one EM iteration.  Workgroup w owns genes [wg_gene[w], wg_gene[w + 1]) and
// parts [wg_part[w], wg_part[w + 1]); part_desc[p] = (first entry, end entry, local run =
// (gene - g0) NR + s R + r); run_part_ptr = the parts of every global run (g NR + s R + r);
// ent[e] = (other gene, count).  LDS: q [R][K2], th [G][K], V/U [G][NR][K], run sums W [G][NR][K],
// part sums [NP][K].
// ------------------------------------------------------------------------------------------
enum { MODE_ADD = 0, MODE_FUSED = 1 };

template <int K, int MODE>
__global__ __launch_bounds__(PNT) void pair_em_kernel(
    const int2* __restrict__ ent, const int4* __restrict__ part_desc, const int* __restrict__ run_part_ptr,
    const int* __restrict__ wg_gene, const int* __restrict__ wg_part, const double* __restrict__ theta,
    double* __restrict__ qr, double* __restrict__ nth, double* __restrict__ s2part,
    double* __restrict__ S2, unsigned* __restrict__ counter, int P, int R, int n_wg, int max_genes,
    double eps) {
  constexpr int K2 = K * K, NF = K <= 10 ? 8 : (K <= 16 ? 4 : 2);  // entries in flight per part thread
  const int NR = 2 * R;
  extern __shared__ double sm[];
  const int b = blockIdx.y, w = blockIdx.x, tid = threadIdx.x;
  const int g0 = wg_gene[w], ng = wg_gene[w + 1] - g0;
  const int p0 = wg_part[w], np = wg_part[w + 1] - p0;
  double* qs = sm;                            // R K2
  double* ths = qs + R * K2;                  // G K
  double* vu = ths + max_genes * K;           // G NR K
  double* wr = vu + max_genes * NR * K;       // G NR K
  double* wp = wr + max_genes * NR * K;       // NP K
  const double* __restrict__ q = qr + (size_t)b * R * K2;
  const double* __restrict__ th = theta + (size_t)b * P * K;
  // the first part descriptor and run range of this thread go out with the staging loads
  const int4 pd0 = part_desc[p0 + (tid < np ? tid : (np > 0 ? np - 1 : 0))];
  const int run0 = g0 * NR + (tid / K < ng * NR ? tid / K : 0);
  const int rpa0 = run_part_ptr[run0], rpb0 = run_part_ptr[run0 + 1];
  for (int t = tid; t < R * K2; t += PNT) qs[t] = q[t];
  for (int t = tid; t < ng * K; t += PNT) ths[t] = th[(size_t)g0 * K + t];
  __syncthreads();
  // V_{g,r}[x] = sum_a th_g[a] q_r[a][x] (slot 0),  U_{g,r}[x] = sum_y q_r[x][y] th_g[y] (slot 1)
  for (int t = tid; t < ng * NR * K; t += PNT) {
    const int gl = t / (NR * K), sr = (t / K) % NR, x = t % K, r = sr % R;
    const double* qq = qs + r * K2;
    const double* tg = ths + gl * K;
    double v = 0.0;
    if (sr < R) {
#pragma unroll
      for (int a = 0; a < K; ++a) v = fma(tg[a], qq[a * K + x], v);
    } else {
#pragma unroll
      for (int y = 0; y < K; ++y) v = fma(qq[x * K + y], tg[y], v);
    }
    vu[t] = v;
  }
  __syncthreads();
  // part sums: c = n / (eps + vec . th_other), acc += c th_other over <= 8 entries
  for (int pi = tid; pi < np; pi += PNT) {
    const int4 pd = pi == tid ? pd0 : part_desc[p0 + pi];
    const double* vec = vu + pd.z * K;
    double acc[K];
#pragma unroll
    for (int x = 0; x < K; ++x) acc[x] = 0.0;
    for (int e = pd.x; e < pd.y; e += NF) {
      int2 en[NF];
#pragma unroll
      for (int u = 0; u < NF; ++u) en[u] = ent[e + u < pd.y ? e + u : pd.y - 1];
      double row[NF][K];
#pragma unroll
      for (int u = 0; u < NF; ++u)
#pragma unroll
        for (int x = 0; x < K; ++x) row[u][x] = th[(size_t)en[u].x * K + x];
#pragma unroll
      for (int u = 0; u < NF; ++u) {
        double dd = 0.0;
#pragma unroll
        for (int x = 0; x < K; ++x) dd = fma(vec[x], row[u][x], dd);
        const double c = e + u < pd.y ? (double)en[u].y / (eps + dd) : 0.0;
#pragma unroll
        for (int x = 0; x < K; ++x) acc[x] = fma(c, row[u][x], acc[x]);
      }
    }
#pragma unroll
    for (int x = 0; x < K; ++x) wp[pi * K + x] = acc[x];
  }
  __syncthreads();
  // W of every run of the block: its parts added in order
  for (int t = tid; t < ng * NR * K; t += PNT) {
    const int lr = t / K, x = t % K;
    const int run = g0 * NR + lr;
    const int a = (t == tid ? rpa0 : run_part_ptr[run]) - p0;
    const int e = (t == tid ? rpb0 : run_part_ptr[run + 1]) - p0;
    double v = 0.0;
    for (int pp = a; pp < e; ++pp) v += wp[pp * K + x];
    wr[t] = v;
  }
  __syncthreads();
  // ntheta[g][a] (+)= sum_r (q_r W^0_r)[a] + (q_r^T W^1_r)[a], rating order
  for (int t = tid; t < ng * K; t += PNT) {
    const int gl = t / K, a = t % K;
    const double* wg = wr + gl * NR * K;
    double v = 0.0;
    for (int r = 0; r < R; ++r) {
      const double* qq = qs + r * K2;
      const double* w0 = wg + r * K;
      const double* w1 = wg + (R + r) * K;
#pragma unroll
      for (int y = 0; y < K; ++y) v = fma(qq[a * K + y], w0[y], v);
#pragma unroll
      for (int y = 0; y < K; ++y) v = fma(qq[y * K + a], w1[y], v);
    }
    double* dst = nth + ((size_t)b * P + g0) * K + t;
    if constexpr (MODE == MODE_ADD) *dst = *dst + v;
    else *dst = v;
  }
  // the block's S2 partial: cells (r, a, y)
  double* out = s2part + ((size_t)b * n_wg + w) * R * K2;
  for (int t = tid; t < R * K2; t += PNT) {
    const int r = t / K2, a = (t / K) % K, y = t % K;
    double v = 0.0;
    for (int gl = 0; gl < ng; ++gl) v = fma(ths[gl * K + a], wr[(gl * NR + r) * K + y], v);
    st_wt(out + t, v);
  }
  // MODE_FUSED: the S2 partials are summed (in workgroup order) and qr updated by the q cells
  // of the triplet engine's fin_kernel, which runs next in the same joint iteration
  if constexpr (MODE == MODE_FUSED) return;
  // MODE_ADD: the last workgroup of this sample adds the partials in workgroup order
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  __shared__ unsigned last;
  if (tid == 0)
    last = __hip_atomic_fetch_add(counter + b, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
           (unsigned)(n_wg - 1);
  __syncthreads();
  if (!last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const double* __restrict__ sp = s2part + (size_t)b * n_wg * R * K2;
  for (int cell = tid; cell < K2; cell += PNT) {
    double sv[MAX_R];
    for (int r = 0; r < R; ++r) {
      double v = 0.0;
      int k = 0;
      for (; k + 8 <= n_wg; k += 8) {  // eight partials' loads in flight, added in order
        double l[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) l[u] = sp[(size_t)(k + u) * R * K2 + r * K2 + cell];
#pragma unroll
        for (int u = 0; u < 8; ++u) v += l[u];
      }
      for (; k < n_wg; ++k) v += sp[(size_t)k * R * K2 + r * K2 + cell];
      sv[r] = v;
    }
    for (int r = 0; r < R; ++r) S2[((size_t)b * R + r) * K2 + cell] = sv[r];
  }
  if (tid == 0) __hip_atomic_store(counter + b, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// qr <- qr S2 / (eps + sum_r qr S2)   (:1660-1666), from caller sums (mmsbm_pairs_qstep)
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
  int n_obs = 0, n_ent = 0, n_parts = 0, n_wg = 0, max_genes = 0, max_parts = 0;
  int4* obs = nullptr;        // (i, j, n, r): the likelihood's observations
  int2* ent = nullptr;        // train: gather entries (other gene, n), by (gene, slot, rating)
  int4* part_desc = nullptr;  // train: (first entry, end entry, local run, 0)
  int* run_part_ptr = nullptr;  // train: [P NR + 1] parts of each run
  int* wg_gene = nullptr;     // train: [n_wg + 1]
  int* wg_part = nullptr;     // train: [n_wg + 1]
  void release() {
    void* ps[] = {obs, ent, part_desc, run_part_ptr, wg_gene, wg_part};
    for (void* p : ps)
      if (p) (void)hipFree(p);
    *this = PairSet();
  }
};

// plan constants: a run is split into parts of >= 8 entries, at most 32 parts; a workgroup takes
// whole genes while it has <= GW(K) genes and <= 64 parts (a lone gene may exceed the part cap:
// the part loop strides by the workgroup size)
constexpr int PART_MIN = 8, PART_MAX = 32, WG_PARTS = 64;  // 64: sweep in DESIGN.md
constexpr int gather_wg_genes(int K) { return K <= 16 ? 64 : 32; }

}  // namespace

struct mmsbm_pairs_ctx {
  int device = 0;
  int K = 0, R = 0, B = 0, P = 0;
  double eps = 1e-10;
  PairSet sets[2];
  char* ws = nullptr;
  long long ws_bytes = 0;
  double *s2part = nullptr, *llpart = nullptr;
  unsigned* counter = nullptr;  // [B] tickets of the last-workgroup reduction (zero between launches)
  int attr[2][MMSBM_MAX_K] = {};  // dynamic LDS bytes pair_em_kernel<K, mode> is opted in to
};

namespace {

size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

int c_blocks(int n_obs) { return (n_obs + PNT - 1) / PNT; }

size_t em_lds_bytes(const mmsbm_pairs_ctx* c) {
  const PairSet& ps = c->sets[MMSBM_SET_TRAIN];
  const size_t K = c->K, NR = 2 * c->R;
  return 8 * (c->R * K * K + ps.max_genes * K + 2 * ps.max_genes * NR * K + ps.max_parts * K);
}

struct PairWs {
  size_t s2part, llpart, counter, total;
};

PairWs ws_layout(const mmsbm_pairs_ctx* c) {
  PairWs L{};
  const size_t B = c->B, K2 = (size_t)c->K * c->K;
  size_t off = 0;
  L.s2part = off;
  off += align_up(B * std::max(c->sets[MMSBM_SET_TRAIN].n_wg, 1) * c->R * K2 * 8);
  L.llpart = off;
  off += align_up(B * std::max({c_blocks(c->sets[0].n_obs), c_blocks(c->sets[1].n_obs), 1}) * 8);
  L.counter = off;
  off += align_up(B * sizeof(unsigned));
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
  int (*em)(mmsbm_pairs_ctx*, int mode, const double*, double*, double*, double*, hipStream_t);
  int (*loglik)(mmsbm_pairs_ctx*, int, const double*, const double*, double*, hipStream_t);
  int (*predict)(mmsbm_pairs_ctx*, const int*, long long, const double*, const double*, double*,
                 hipStream_t);
};

// mode MODE_ADD: nth += pair sums, S2 written.  MODE_FUSED: nth = pair sums, qr M-step in place.
template <int K>
int launch_em(mmsbm_pairs_ctx* c, int mode, const double* theta, double* qr, double* nth, double* S2,
              hipStream_t s) {
  const PairSet& ps = c->sets[MMSBM_SET_TRAIN];
  const int lds = (int)em_lds_bytes(c);
  if (lds > 160 * 1024)
    return fail(MMSBM_ERR_UNSUPPORTED, "pair plan needs %d B of LDS per workgroup", lds);
  auto kern = mode == MODE_ADD ? &pair_em_kernel<K, MODE_ADD> : &pair_em_kernel<K, MODE_FUSED>;
  if (lds > 64 * 1024 && c->attr[mode][K - 1] < lds) {  // opt in to this plan's dynamic LDS
    HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    c->attr[mode][K - 1] = lds;
  }
  kern<<<dim3(ps.n_wg, c->B), PNT, lds, s>>>(ps.ent, ps.part_desc, ps.run_part_ptr, ps.wg_gene, ps.wg_part,
                                             theta, qr, nth, c->s2part, S2, c->counter, c->P, c->R,
                                             ps.n_wg, ps.max_genes, c->eps);
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
  pair_ll_kernel<K><<<dim3(nb, c->B), PNT, c->R * K * K * 8, s>>>(ps.obs, ps.n_obs, theta, qr, c->llpart,
                                                                  c->P, c->R, c->eps);
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
      PLaunch{&launch_em<Ks + 1>, &launch_loglik<Ks + 1>, &launch_predict<Ks + 1>}...};
}

const auto kPTable = make_table(std::make_integer_sequence<int, MMSBM_MAX_K>{});

// Train plan: entries by (gene, slot, rating) run, parts, workgroups of whole genes.
int build_train_plan(mmsbm_pairs_ctx* c, PairSet& ps, const std::vector<int4>& obs) {
  const int R = c->R, NR = 2 * R, P = c->P, GW = gather_wg_genes(c->K);
  int wg_parts = WG_PARTS;  // MMSBM_PAIR_PARTS=n: parts per workgroup (measurement sweeps)
  if (const char* e = getenv("MMSBM_PAIR_PARTS")) {
    const int v = atoi(e);
    if (v >= 16 && v <= 1024) wg_parts = v;
  }
  const size_t nrun = (size_t)P * NR;
  std::vector<int> run_ptr(nrun + 1, 0);
  for (const int4& o : obs) {
    run_ptr[(size_t)o.x * NR + o.w + 1]++;
    run_ptr[(size_t)o.y * NR + R + o.w + 1]++;
  }
  for (size_t k = 1; k <= nrun; ++k) run_ptr[k] += run_ptr[k - 1];
  ps.n_ent = run_ptr[nrun];
  std::vector<int> fill(run_ptr.begin(), run_ptr.end() - 1);
  std::vector<int2> ent(std::max(ps.n_ent, 1), make_int2(0, 0));
  for (const int4& o : obs) {  // observation order inside each run
    ent[fill[(size_t)o.x * NR + o.w]++] = make_int2(o.y, o.z);
    ent[fill[(size_t)o.y * NR + R + o.w]++] = make_int2(o.x, o.z);
  }
  std::vector<int> run_part_ptr(nrun + 1, 0);
  std::vector<int4> parts;
  for (size_t run = 0; run < nrun; ++run) {
    const int e0 = run_ptr[run], n = run_ptr[run + 1] - e0;
    if (n > 0) {
      const int pl = std::max(PART_MIN, (n + PART_MAX - 1) / PART_MAX);
      for (int e = 0; e < n; e += pl) parts.push_back(make_int4(e0 + e, e0 + std::min(n, e + pl), 0, 0));
    }
    run_part_ptr[run + 1] = (int)parts.size();
  }
  ps.n_parts = (int)parts.size();
  std::vector<int> wg_gene{0}, wg_part{0};
  ps.max_genes = ps.max_parts = 0;
  for (int g = 0; g < P;) {  // whole genes per workgroup
    const int g0 = g;
    int np = 0;
    while (g < P) {
      const int gp = run_part_ptr[(size_t)(g + 1) * NR] - run_part_ptr[(size_t)g * NR];
      if (g > g0 && (g - g0 >= GW || np + gp > wg_parts)) break;
      np += gp;
      ++g;
    }
    for (size_t run = (size_t)g0 * NR; run < (size_t)g * NR; ++run)
      for (int q = run_part_ptr[run]; q < run_part_ptr[run + 1]; ++q) parts[q].z = (int)(run - (size_t)g0 * NR);
    ps.max_genes = std::max(ps.max_genes, g - g0);
    ps.max_parts = std::max(ps.max_parts, np);
    wg_gene.push_back(g);
    wg_part.push_back(run_part_ptr[(size_t)g * NR]);
  }
  ps.n_wg = (int)wg_gene.size() - 1;
  if (parts.empty()) parts.push_back(make_int4(0, 0, 0, 0));
  int rc;
  if ((rc = upload(&ps.ent, ent))) return rc;
  if ((rc = upload(&ps.part_desc, parts))) return rc;
  if ((rc = upload(&ps.run_part_ptr, run_part_ptr))) return rc;
  if ((rc = upload(&ps.wg_gene, wg_gene))) return rc;
  if ((rc = upload(&ps.wg_part, wg_part))) return rc;
  if (em_lds_bytes(c) > 160 * 1024)
    return fail(MMSBM_ERR_UNSUPPORTED, "pair plan needs %zu B of LDS per workgroup", em_lds_bytes(c));
  return MMSBM_OK;
}

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
  if (c->K != K || c->P != P || c->R != R) {  // plans depend on K (workgroup size), P and R
    DeviceGuard g(c->device);
    for (auto& s : c->sets) s.release();
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
  const int R = c->R;
  // observations: every (link, r) with n > 0, in link order (a zero count adds exactly zero)
  std::vector<int4> obs;
  for (int64_t e = 0; e < E; ++e)
    for (int r = 0; r < R; ++r) {
      const int n = counts_host[e * R + r];
      if (n > 0) obs.push_back(make_int4(ids_host[2 * e], ids_host[2 * e + 1], n, r));
    }
  ps.n_obs = (int)obs.size();
  if ((rc = upload(&ps.obs, obs))) return rc;
  if (which == MMSBM_SET_TRAIN && (rc = build_train_plan(c, ps, obs))) {
    ps.release();
    return rc;
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
  DeviceGuard g(c->device);
  c->ws = (char*)ws;
  c->ws_bytes = bytes;
  c->s2part = (double*)(c->ws + L.s2part);
  c->llpart = (double*)(c->ws + L.llpart);
  c->counter = (unsigned*)(c->ws + L.counter);
  HIP_TRY(hipMemset(c->counter, 0, sizeof(unsigned) * c->B));  // tickets start (and end) at zero
  HIP_TRY(hipDeviceSynchronize());
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
  return kPTable[c->K - 1].em(c, MODE_ADD, theta, const_cast<double*>(qr), nth, S2, (hipStream_t)stream);
}

}  // extern "C"

// Library-internal (mmsbm_joint_iterate, mmsbm.hip): the fused pair half of a joint iteration,
// nth2 = the pair sums (every gene written) and the S2 partials of its workgroups.
int mmsbm_detail_pairs_estep(mmsbm_pairs_ctx* c, const double* theta, const double* qr, double* nth2,
                             hipStream_t s, const double** s2part, int* n_wg) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null pair context");
  int rc = check_ready(c);
  if (rc) return rc;
  if (c->K < 1 || c->B < 1) return fail(MMSBM_ERR_INVALID, "pair context shape");
  *s2part = c->s2part;
  *n_wg = c->sets[MMSBM_SET_TRAIN].n_wg;
  return kPTable[c->K - 1].em(c, MODE_FUSED, theta, const_cast<double*>(qr), nth2, nullptr, s);
}

int mmsbm_detail_pairs_shape(const mmsbm_pairs_ctx* c, int* K, int* R, int* B, int* P) {
  *K = c->K;
  *R = c->R;
  *B = c->B;
  *P = c->P;
  return MMSBM_OK;
}

extern "C" {

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
  info[2] = ps.n_parts;
  info[3] = ps.n_wg;
  info[4] = ps.max_genes;
  info[5] = ps.max_parts;
  info[6] = c_blocks(ps.n_obs);
  return MMSBM_OK;
}

}  // extern "C"
