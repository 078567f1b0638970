// mmsbm.hip — MI355X (gfx950) MMSBM EM engine: kernels + C ABI (include/mmsbm.h).
//
// Hot path of AleixMT/TrigenicInteractionPredictor, src/TrigenicInteractionPredictor.py:
//   make_iteration      :984-1043   -> estep*_kernel, m1_kernel (S), m2_kernel (p, theta)
//   compute_likelihood  :952-974    -> loglik_kernel + reduce_kernel
//   do_prediction       :530-547    -> predict_kernel
//
// Algebra (per observed (link, r) with gene ids (i, j, k) and weight n = n_r):
//   T[abg]  = th_i[a] th_j[b] th_k[g] p_r[abg]
//   d       = eps + sum T                              (:990, :996-1000)
//   U[ab]   = sum_g p_r[abg] th_k[g]
//   Y[a]    = sum_b th_j[b] U[ab]        Z[b] = sum_a th_i[a] U[ab]
//   W[g]    = sum_ab th_i[a] th_j[b] p_r[abg]
//   d       = eps + sum_a th_i[a] Y[a]
//   c       = n / d
//   ntheta[i][a] += th_i[a] c Y[a],  ntheta[j][b] += th_j[b] c Z[b],  ntheta[k][g] += th_k[g] c W[g]
//   npr[abg r]   += p_r[abg] * S_r[abg],  S_r[abg] = sum_links c th_i[a] th_j[b] th_k[g]
// which is the reference's per-cell a = T/d scatter (:1002-1012) factorised: 3K^3 FMAs per
// observation instead of 2 * K^3 * R multiply-adds over the full lattice.
//
// Mapping (all FP64 on the vector ALUs; no MFMA — this is a normalise / outer-product path):
//   * one workgroup = one tile of MMSBM_TILE observations of ONE rating r, so p_r's address is
//     wave-uniform and the p reads are scalar loads (SGPR operands, no LDS, no VGPR traffic);
//   * phase A: one lane per observation, th_j / th_k rows and Z / W accumulators in VGPRs;
//     Y, Z, W rows are stored once per observation (plain stores), c = n/d per observation;
//   * phase B: S_r accumulation as a register-tiled outer-product GEMM over the tile's
//     observations staged in LDS (lane = (a, b-chunk) cell block x link group), reduced across
//     link groups through LDS in a fixed tree, one partial-S row per tile;
//   * M-step: theta by a per-gene gather over the gene's (observation, slot) incidence list
//     (store-then-gather instead of float atomics: deterministic, bitwise reproducible), p by a
//     fixed-order sum of the per-tile partials.
// Every reduction has a fixed order, so results are bitwise reproducible run to run.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "mmsbm.h"

namespace {

constexpr int TILE = MMSBM_TILE;
constexpr int MAX_R = 8;
constexpr int LDS_BUDGET = 64 * 1024;
constexpr int SACC_WGS = 256;      // default S-accumulation workgroups (MMSBM_SACC_WGS): 1 per CU
constexpr int SACC_WGS_MAX = 2048;

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) return fail(MMSBM_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

// ------------------------------------------------------------------------------------------
// Compile-time tiling of the S accumulation (phase B) for a given K.
// ------------------------------------------------------------------------------------------
constexpr int pick_nb(int K) {
  // cells per lane = NB * K <= 50 doubles (fits 3 waves/SIMD with phase A's live set);
  // prefer a divisor of K (no ragged b-chunk).
  int cap = 50 / K;
  if (cap < 1) cap = 1;
  if (cap > K) cap = K;
  int best = 1;
  for (int d = 1; d <= cap; ++d)
    if (K % d == 0) best = d;
  return (2 * best >= cap) ? best : cap;
}

// Phase-B (S accumulation) tiling for NT threads: lane = (cell block, link group).
// b-chunk per lane for a cell budget of `cells` doubles: a divisor of K when one comes close
// to the budget (no ragged chunk), else the largest chunk that fits.
constexpr int pick_nb_cap(int K, int cells) {
  int cap = cells / K;
  if (cap < 1) cap = 1;
  if (cap > K) cap = K;
  int best = 1;
  for (int d = 1; d <= cap; ++d)
    if (K % d == 0) best = d;
  return (4 * best >= 3 * cap) ? best : cap;
}

template <int K, int NT, int CELLS = 50>
struct SPlan {
  static constexpr int K3 = K * K * K;
  static constexpr int NB = pick_nb_cap(K, CELLS);  // b-chunk per lane
  static constexpr int NBC = (K + NB - 1) / NB;
  static constexpr int NBLK = K * NBC;     // cell blocks (a, b-chunk, all g)
  static constexpr int NSETS = (NBLK + NT - 1) / NT;
  static constexpr int LG_RAW = NBLK >= NT ? 1 : NT / NBLK;
  static constexpr int LG_RED = 2 * (LDS_BUDGET / (8 * K3)) + 1;  // keep the reduction in budget
  static constexpr int LG = LG_RAW < LG_RED ? LG_RAW : LG_RED;    // link groups
};

// Wave64 butterfly sum in a fixed order (bitwise reproducible).
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) v += __shfl_xor(v, s, 64);
  return v;
}

// Workgroup sum of one double per thread; result valid in thread 0.  `scratch` >= 4 doubles.
__device__ __forceinline__ double block_sum(double v, double* scratch) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) scratch[w] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0) {
    for (int q = 0; q < (int)(blockDim.x >> 6); ++q) s += scratch[q];
  }
  return s;
}

// ------------------------------------------------------------------------------------------
// Phase A: per-observation contractions.  One lane = one observation.  p_r is wave-uniform.
// Returns sum_a th_i[a] Y[a]; stores Y, Z, W (unscaled) into the rows ry, rz, rw.
// ------------------------------------------------------------------------------------------
template <int K>
__device__ __forceinline__ double phase_a(const double* __restrict__ th, const double* __restrict__ p,
                                          const int4 e, double* __restrict__ ry,
                                          double* __restrict__ rz, double* __restrict__ rw) {
  constexpr int K2 = K * K;
  const double* __restrict__ ri = th + (size_t)e.x * K;
  const double* __restrict__ rj = th + (size_t)e.y * K;
  const double* __restrict__ rk = th + (size_t)e.z * K;
  double tj[K], tk[K], zc[K];
#pragma unroll
  for (int g = 0; g < K; ++g) {
    tj[g] = rj[g];
    tk[g] = rk[g];
    zc[g] = 0.0;
  }
  double dsum = 0.0;
  if constexpr (K <= 16) {
    // single pass: each p element feeds two FMAs (U and W)
    double wc[K];
#pragma unroll
    for (int g = 0; g < K; ++g) wc[g] = 0.0;
    double ta_next = ri[0];
#pragma unroll 1
    for (int a = 0; a < K; ++a) {
      const double ta = ta_next;
      ta_next = ri[a + 1 < K ? a + 1 : a];  // prefetch: its latency hides under this iteration
      const double* __restrict__ pa = p + a * K2;
      double y = 0.0;
#pragma unroll
      for (int b = 0; b < K; ++b) {
        double u = 0.0;
#pragma unroll
        for (int g = 0; g < K; ++g) u = fma(pa[b * K + g], tk[g], u);
        y = fma(tj[b], u, y);
        zc[b] = fma(ta, u, zc[b]);
        const double t = ta * tj[b];
#pragma unroll
        for (int g = 0; g < K; ++g) wc[g] = fma(t, pa[b * K + g], wc[g]);
      }
      ry[a] = y;
      dsum = fma(ta, y, dsum);
    }
#pragma unroll
    for (int g = 0; g < K; ++g) {
      rz[g] = zc[g];
      rw[g] = wc[g];
    }
  } else {
    // two passes keep the live set at 3K (pass 1) / 2K (pass 2) doubles
    double ta_next = ri[0];
#pragma unroll 1
    for (int a = 0; a < K; ++a) {
      const double ta = ta_next;
      ta_next = ri[a + 1 < K ? a + 1 : a];
      const double* __restrict__ pa = p + a * K2;
      double y = 0.0;
#pragma unroll
      for (int b = 0; b < K; ++b) {
        double u = 0.0;
#pragma unroll
        for (int g = 0; g < K; ++g) u = fma(pa[b * K + g], tk[g], u);
        y = fma(tj[b], u, y);
        zc[b] = fma(ta, u, zc[b]);
      }
      ry[a] = y;
      dsum = fma(ta, y, dsum);
    }
#pragma unroll
    for (int g = 0; g < K; ++g) rz[g] = zc[g];
    double wc[K];
#pragma unroll
    for (int g = 0; g < K; ++g) wc[g] = 0.0;
    ta_next = ri[0];
#pragma unroll 1
    for (int a = 0; a < K; ++a) {
      const double ta = ta_next;
      ta_next = ri[a + 1 < K ? a + 1 : a];
      const double* __restrict__ pa = p + a * K2;
#pragma unroll
      for (int b = 0; b < K; ++b) {
        const double t = ta * tj[b];
#pragma unroll
        for (int g = 0; g < K; ++g) wc[g] = fma(t, pa[b * K + g], wc[g]);
      }
    }
#pragma unroll
    for (int g = 0; g < K; ++g) rw[g] = wc[g];
  }
  return dsum;
}

// Normaliser only (compute_likelihood / prediction): sum_a th_i[a] sum_b th_j[b] sum_g p th_k[g].
template <int K>
__device__ __forceinline__ double contract(const double* __restrict__ th, const double* __restrict__ p,
                                           int gi, int gj, int gk) {
  constexpr int K2 = K * K;
  const double* __restrict__ ri = th + (size_t)gi * K;
  const double* __restrict__ rj = th + (size_t)gj * K;
  const double* __restrict__ rk = th + (size_t)gk * K;
  double tj[K], tk[K];
#pragma unroll
  for (int g = 0; g < K; ++g) {
    tj[g] = rj[g];
    tk[g] = rk[g];
  }
  double dsum = 0.0;
  double ta_next = ri[0];
#pragma unroll 1
  for (int a = 0; a < K; ++a) {
    const double ta = ta_next;
    ta_next = ri[a + 1 < K ? a + 1 : a];
    const double* __restrict__ pa = p + a * K2;
    double y = 0.0;
#pragma unroll
    for (int b = 0; b < K; ++b) {
      double u = 0.0;
#pragma unroll
      for (int g = 0; g < K; ++g) u = fma(pa[b * K + g], tk[g], u);
      y = fma(tj[b], u, y);
    }
    dsum = fma(ta, y, dsum);
  }
  return dsum;
}

// ------------------------------------------------------------------------------------------
// E-step plan.  ET = 64 observations per workgroup, H lanes per observation (NT = 64*H).
//   K in {1..8, 10, 12}: p_r is staged in LDS once per workgroup and read with wave-uniform
//            ds_read_b128 (broadcast, conflict-free); H = 2: the two lanes of an observation
//            split the a-range and exchange their Z / W / d partials with one lane swap (twice
//            the waves of one lane per observation: a fold0-sized problem otherwise leaves ~1
//            wave per SIMD to hide every latency).
//   other K: p_r streams through the scalar cache (SGPR operands), H = 1.
// LDS: Ps = K slabs of K*KP doubles, the second half shifted by 16 B so that the two lanes'
//      reads of one instruction hit distinct banks; 8 doubles of block-sum scratch.
// ------------------------------------------------------------------------------------------
constexpr int ET = 64;

template <int K>
struct EPlan {
  static constexpr bool STAGE_P = K <= 12 && K != 9 && K != 11;
  static constexpr int H = STAGE_P ? 2 : 1;
  static constexpr int NT = ET * H;
  static constexpr int K3 = K * K * K;
  static constexpr int KP = (K + 1) & ~1;
  static constexpr int KH = (K + H - 1) / H;  // a-range per lane
  static constexpr int P_DBL = STAGE_P ? K * K * KP + 2 : 0;
  static constexpr int LDS_BYTES = (P_DBL + 8) * 8;
  // waves/SIMD the register allocator must leave room for (3 keeps a fold0 grid resident)
  static constexpr int OCC = STAGE_P ? 3 : 1;
  // observations per lane in the E-step (two halve the LDS reads per FMA and double the
  // independent FMA chains; the fold0 grid is then one wave per SIMD, latency covered by ILP)
  static constexpr int NO = STAGE_P && K >= 4 && K <= 10 ? 2 : 1;
  static constexpr int EOBS = ET * NO;  // observations per E-step workgroup
  static constexpr int E_OCC = NO == 2 ? 2 : OCC;
  __device__ static constexpr int slab(int a) { return a * K * KP + (a >= KH ? 2 : 0); }
};

template <int K>
__device__ __forceinline__ void stage_p(double* __restrict__ Ps, const double* __restrict__ p,
                                        int tid, int nt) {
  using EP = EPlan<K>;
  for (int idx = tid; idx < EP::K3; idx += nt) {
    const int a = idx / (K * K);
    Ps[EP::slab(a) + ((idx / K) % K) * EP::KP + idx % K] = p[idx];
  }
}

template <int K>
__device__ __forceinline__ void lds_row(double (&dst)[K], const double* __restrict__ src) {
#pragma unroll
  for (int g = 0; g < (K & ~1); g += 2) {
    const double2 v = *reinterpret_cast<const double2*>(src + g);
    dst[g] = v.x;
    dst[g + 1] = v.y;
  }
  if constexpr (K & 1) dst[K - 1] = src[K - 1];
}

// Phase A with p_r in LDS for NO observations per lane; lane h of 2 covers a in
// [h*KH, h*KH + KH).  Returns Y[a] of its own a-range in yv; on return zc / wc / dsum hold the
// FULL sums (partner partials added in a commutative, lane-symmetric order, so both lanes
// agree bitwise).  Every p value read from LDS feeds 2*NO FMAs.
template <int K, int NO>
__device__ __forceinline__ void phase_a_lds(const double* __restrict__ Ps,
                                            const double* __restrict__ const (&ri)[NO],
                                            const double* __restrict__ const (&rj)[NO],
                                            const double* __restrict__ const (&rk)[NO], int h,
                                            double (&yv)[NO][EPlan<K>::KH], double (&zc)[NO][K],
                                            double (&wc)[NO][K], double (&dsum)[NO]) {
  using EP = EPlan<K>;
  constexpr int KP = EP::KP, KH = EP::KH, NPAIR = (K + 1) / 2;
  double tj[NO][K], tk[NO][K], ti[NO][KH];
#pragma unroll
  for (int m = 0; m < NO; ++m) {
#pragma unroll
    for (int g = 0; g < K; ++g) {
      tj[m][g] = rj[m][g];
      tk[m][g] = rk[m][g];
      zc[m][g] = 0.0;
      wc[m][g] = 0.0;
    }
#pragma unroll
    for (int q = 0; q < KH; ++q) ti[m][q] = (h * KH + q < K) ? ri[m][h * KH + q] : 0.0;
    dsum[m] = 0.0;
  }
  // Two p rows per step: 2*NO independent U chains.
#pragma unroll
  for (int q = 0; q < KH; ++q) {
    const int a = h * KH + q;
    const bool valid = a < K;
    const double* __restrict__ pa = Ps + EP::slab(valid ? a : K - 1);
    double y[NO];
#pragma unroll
    for (int m = 0; m < NO; ++m) y[m] = 0.0;
#pragma unroll
    for (int bp = 0; bp < NPAIR; ++bp) {
      const int b0 = 2 * bp, b1 = 2 * bp + 1;
      double pv0[K], pv1[K];
      lds_row<K>(pv0, pa + b0 * KP);
      if (b1 < K) {
        lds_row<K>(pv1, pa + b1 * KP);
      } else {
#pragma unroll
        for (int g = 0; g < K; ++g) pv1[g] = 0.0;
      }
#pragma unroll
      for (int m = 0; m < NO; ++m) {
        const double ta = ti[m][q];
        double u0 = 0.0, u1 = 0.0;
#pragma unroll
        for (int g = 0; g < K; ++g) {
          u0 = fma(pv0[g], tk[m][g], u0);
          u1 = fma(pv1[g], tk[m][g], u1);
        }
        const double t0 = ta * tj[m][b0];
        y[m] = fma(tj[m][b0], u0, y[m]);
        zc[m][b0] = fma(ta, u0, zc[m][b0]);
        if (b1 < K) {
          const double t1 = ta * tj[m][b1];
          y[m] = fma(tj[m][b1], u1, y[m]);
          zc[m][b1] = fma(ta, u1, zc[m][b1]);
#pragma unroll
          for (int g = 0; g < K; ++g) wc[m][g] = fma(t1, pv1[g], fma(t0, pv0[g], wc[m][g]));
        } else {
#pragma unroll
          for (int g = 0; g < K; ++g) wc[m][g] = fma(t0, pv0[g], wc[m][g]);
        }
      }
    }
#pragma unroll
    for (int m = 0; m < NO; ++m) {
      yv[m][q] = y[m];
      dsum[m] = fma(ti[m][q], y[m], dsum[m]);
    }
  }
#pragma unroll
  for (int m = 0; m < NO; ++m) {
#pragma unroll
    for (int g = 0; g < K; ++g) {
      zc[m][g] += __shfl_xor(zc[m][g], 1, 64);
      wc[m][g] += __shfl_xor(wc[m][g], 1, 64);
    }
    dsum[m] += __shfl_xor(dsum[m], 1, 64);
  }
}

// ------------------------------------------------------------------------------------------
// E-step, four lanes per observation: lane h = (ha, hb) covers the a-half ha x b-half hb block
// of the (a, b) lattice (balanced for every even K), so a fold0-sized problem has ~4 waves per
// SIMD; FP64 FMA needs >= 4 resident waves with >= 4 independent chains each to approach its
// issue rate (one wave alone issues at most one per ~6.5 cycles; dependent latency ~40).
// p_r in LDS: the four lanes of an observation read four different (a, b) rows per
// instruction; the half offsets sa / sb place them in four distinct 4-bank slots.
// ------------------------------------------------------------------------------------------
constexpr int E4_NT = 256;  // 64 observations x 4 lanes

constexpr bool e4_slots_ok(int K, int sa, int sb) {
  const int KP = (K + 1) & ~1, KA = (K + 1) / 2, KB = (K + 1) / 2, SA = K * KP + 8;
  const int da = ((KA * SA + sa) / 2) % 16, db = ((KB * KP + sb) / 2) % 16;
  return da != 0 && db != 0 && da != db && (da + db) % 16 != 0;
}
constexpr int e4_pick_sa(int K) {
  for (int sa = 0; sa <= 30; sa += 2)
    for (int sb = 0; sb <= 6; sb += 2)
      if (e4_slots_ok(K, sa, sb)) return sa;
  return 0;
}
constexpr int e4_pick_sb(int K) {
  for (int sa = 0; sa <= 30; sa += 2)
    for (int sb = 0; sb <= 6; sb += 2)
      if (e4_slots_ok(K, sa, sb)) return sb;
  return 0;
}

template <int K>
struct E4Plan {
  static constexpr bool ON = K >= 2 && K <= 12 && K != 9 && K != 11;
  static constexpr int K3 = K * K * K;
  static constexpr int KP = (K + 1) & ~1;
  static constexpr int KA = (K + 1) / 2, KB = (K + 1) / 2;
  static constexpr int SA = K * KP + 8;  // a-slab stride (doubles): room for the b-half shift
  static constexpr int SHA = e4_pick_sa(K), SHB = e4_pick_sb(K);
  static constexpr int P_DBL = K * SA + SHA + 8;
  static constexpr int LDS_BYTES = (P_DBL + 8) * 8;
  __device__ static constexpr int off(int a, int b) {
    return a * SA + b * KP + (b >= KB ? SHB : 0) + (a >= KA ? SHA : 0);
  }
};

template <int K>
__device__ __forceinline__ void e4_stage_p(double* __restrict__ Ps, const double* __restrict__ p,
                                           int tid) {
  using EP = E4Plan<K>;
  for (int idx = tid; idx < EP::K3; idx += E4_NT) {
    const int a = idx / (K * K), b = (idx / K) % K;
    Ps[EP::off(a, b) + idx % K] = p[idx];
  }
}

// Lane (ha, hb): Y partials of its a-half over its b-half, Z partials of its b-half over its
// a-half, W and d partials over its block; exchanged with two lane swaps (xor 1: a-halves,
// xor 2: b-halves) in commutative, lane-symmetric order, so all lanes agree bitwise.
template <int K>
__device__ __forceinline__ double phase_a_e4(const double* __restrict__ Ps,
                                             const double* __restrict__ ri,
                                             const double* __restrict__ rj,
                                             const double* __restrict__ rk, int ha, int hb,
                                             double (&yv)[E4Plan<K>::KA],
                                             double (&zc)[E4Plan<K>::KB], double (&wc)[K]) {
  using EP = E4Plan<K>;
  constexpr int KA = EP::KA, KB = EP::KB;
  double ti[KA], tj[KB], tk[K];
#pragma unroll
  for (int s = 0; s < KA; ++s) ti[s] = (ha * KA + s < K) ? ri[ha * KA + s] : 0.0;
#pragma unroll
  for (int t = 0; t < KB; ++t) tj[t] = (hb * KB + t < K) ? rj[hb * KB + t] : 0.0;
#pragma unroll
  for (int g = 0; g < K; ++g) {
    tk[g] = rk[g];
    wc[g] = 0.0;
  }
#pragma unroll
  for (int t = 0; t < KB; ++t) zc[t] = 0.0;
  double dsum = 0.0;
#pragma unroll
  for (int s = 0; s < KA; ++s) {
    const int a = ha * KA + s < K ? ha * KA + s : K - 1;
    const double ta = ti[s];
    double y = 0.0;
#pragma unroll
    for (int t = 0; t < KB; ++t) {
      const int bb = hb * KB + t < K ? hb * KB + t : K - 1;
      double pv[K];
      lds_row<K>(pv, Ps + EP::off(a, bb));
      double u = 0.0;
#pragma unroll
      for (int g = 0; g < K; ++g) u = fma(pv[g], tk[g], u);
      y = fma(tj[t], u, y);
      zc[t] = fma(ta, u, zc[t]);
      const double tt = ta * tj[t];
#pragma unroll
      for (int g = 0; g < K; ++g) wc[g] = fma(tt, pv[g], wc[g]);
    }
    yv[s] = y;
    dsum = fma(ta, y, dsum);
  }
#pragma unroll
  for (int s = 0; s < KA; ++s) yv[s] += __shfl_xor(yv[s], 2, 64);
#pragma unroll
  for (int t = 0; t < KB; ++t) zc[t] += __shfl_xor(zc[t], 1, 64);
#pragma unroll
  for (int g = 0; g < K; ++g) {
    wc[g] += __shfl_xor(wc[g], 1, 64);
    wc[g] += __shfl_xor(wc[g], 2, 64);
  }
  dsum += __shfl_xor(dsum, 1, 64);
  dsum += __shfl_xor(dsum, 2, 64);
  return dsum;
}

template <int K>
__global__ __launch_bounds__(E4_NT, 4) void estep4_kernel(
    const int4* __restrict__ obs, const int4* __restrict__ pos, const int* __restrict__ tile_r,
    const double* __restrict__ theta, const double* __restrict__ pr, double* __restrict__ contrib,
    double* __restrict__ cvec, double* __restrict__ partL, int P, int R, long long n_obs_pad,
    long long nnz, int ntiles, double eps, int ablate) {
  using EP = E4Plan<K>;
  constexpr int K3 = EP::K3, KA = EP::KA, KB = EP::KB;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* Ps = smem;
  double* scratch = smem + EP::P_DBL;
  const int tid = threadIdx.x;
  const int lo = tid >> 2, h = tid & 3, ha = h & 1, hb = h >> 1;
  const int tile = blockIdx.x;
  const int b = blockIdx.y;
  const int r = __builtin_amdgcn_readfirstlane(tile_r[(tile * ET) / TILE]);
  const double* __restrict__ th = theta + (size_t)b * P * K;
  const double* __restrict__ p = pr + ((size_t)b * R + r) * K3;
  const size_t o = (size_t)tile * ET + lo;
  const int4 e = obs[o];
  const int4 q = pos[o];
  const double n = (double)e.w;
  e4_stage_p<K>(Ps, p, tid);
  __syncthreads();
  double yv[KA], zc[KB], wc[K], dsum = 1.0;
  // ablate (measurement builds only, MMSBM_ABLATE): bit 0 skips phase A
  if (!(ablate & 1))
    dsum = phase_a_e4<K>(Ps, th + (size_t)e.x * K, th + (size_t)e.y * K, th + (size_t)e.z * K,
                         ha, hb, yv, zc, wc);
  const double d = dsum + eps;
  const double c = n / d;
  if (q.x >= 0 && !(ablate & 9)) {  // bit 3: skip the row stores (measurement only)
    double* __restrict__ cb = contrib + (size_t)b * (nnz + 1) * K;
    if (hb == 0) {  // Y row, own a-half
      double* ry = cb + (size_t)q.x * K + ha * KA;
#pragma unroll
      for (int s = 0; s < KA; ++s)
        if (ha * KA + s < K) ry[s] = c * yv[s];
    }
    if (ha == 0) {  // Z row, own b-half
      double* rz = cb + (size_t)q.y * K + hb * KB;
#pragma unroll
      for (int t = 0; t < KB; ++t)
        if (hb * KB + t < K) rz[t] = c * zc[t];
    } else {  // W row, g-half hb
      double* rw = cb + (size_t)q.z * K;
#pragma unroll
      for (int g = 0; g < K; ++g)
        if ((g >= KB) == (hb == 1)) rw[g] = c * wc[g];
    }
  }
  if (h == 0) cvec[(size_t)b * n_obs_pad + o] = c;
  const double ll = block_sum(h == 0 ? n * log(d) : 0.0, scratch);
  if (tid == 0) partL[(size_t)b * ntiles + tile] = ll;
}

// ------------------------------------------------------------------------------------------
// E-step (phase A of :987-1012): grid (n_obs_pad / ET, B), block NT.
//   The three c-scaled contribution rows of an observation, c*Y -> ntheta[i], c*Z -> ntheta[j],
//   c*W -> ntheta[k], are stored at the observation's positions in the gene incidence CSR
//   (pos[o] = (q0, q1, q2)), so that M1 reads every gene's rows as one contiguous run.
//   cvec[b][o] <- c = n / d;  partL[b][tile] <- sum n log d (likelihood of the incoming
//   parameters, for free).
// ------------------------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__((EPlan<K>::NT), (EPlan<K>::E_OCC)) void estep_kernel(
    const int4* __restrict__ obs, const int4* __restrict__ pos, const int* __restrict__ tile_r,
    const double* __restrict__ theta, const double* __restrict__ pr, double* __restrict__ contrib,
    double* __restrict__ cvec, double* __restrict__ partL, int P, int R, long long n_obs_pad,
    long long nnz, int ntiles, double eps, int ablate) {
  using EP = EPlan<K>;
  constexpr int K3 = EP::K3, H = EP::H, NT = EP::NT, KH = EP::KH, NO = EP::NO;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* Ps = smem;
  double* scratch = smem + EP::P_DBL;

  const int tid = threadIdx.x;
  const int lo = tid / H;  // observation slot within the tile (x NO)
  const int h = tid % H;   // lane's share of the observation
  const int tile = blockIdx.x;
  const int b = blockIdx.y;
  const int r = __builtin_amdgcn_readfirstlane(tile_r[(tile * EP::EOBS) / TILE]);
  const double* __restrict__ th = theta + (size_t)b * P * K;
  const double* __restrict__ p = pr + ((size_t)b * R + r) * K3;
  double* __restrict__ cb = contrib + (size_t)b * (nnz + 1) * K;
  if constexpr (EP::STAGE_P) {
    size_t o[NO];
    int4 e[NO], q[NO];
    const double* ri[NO];
    const double* rj[NO];
    const double* rk[NO];
#pragma unroll
    for (int m = 0; m < NO; ++m) {
      o[m] = (size_t)tile * EP::EOBS + m * ET + lo;
      e[m] = obs[o[m]];
      q[m] = pos[o[m]];  // CSR rows of slots 0, 1, 2 (-1 for padding)
      ri[m] = th + (size_t)e[m].x * K;
      rj[m] = th + (size_t)e[m].y * K;
      rk[m] = th + (size_t)e[m].z * K;
    }
    stage_p<K>(Ps, p, tid, NT);
    __syncthreads();
    double yv[NO][KH], zc[NO][K], wc[NO][K], dsum[NO];
    // ablate (measurement builds only, MMSBM_ABLATE): bit 0 skips phase A
    if (!(ablate & 1)) {
      phase_a_lds<K, NO>(Ps, ri, rj, rk, h, yv, zc, wc, dsum);
    } else {
#pragma unroll
      for (int m = 0; m < NO; ++m) dsum[m] = 1.0;
    }
    double llsum = 0.0;
#pragma unroll
    for (int m = 0; m < NO; ++m) {
      const double n = (double)e[m].w;
      const double d = dsum[m] + eps;
      const double c = n / d;
      if (q[m].x >= 0 && !(ablate & 1)) {
        double* ry = cb + (size_t)q[m].x * K + h * KH;
#pragma unroll
        for (int t = 0; t < KH; ++t)
          if (h * KH + t < K) ry[t] = c * yv[m][t];
        double* rzw = cb + (size_t)(h == 0 ? q[m].y : q[m].z) * K;
#pragma unroll
        for (int g = 0; g < K; ++g) rzw[g] = c * (h == 0 ? zc[m][g] : wc[m][g]);
      }
      if (h == 0) {
        cvec[(size_t)b * n_obs_pad + o[m]] = c;
        llsum += n * log(d);
      }
    }
    const double ll = block_sum(llsum, scratch);
    if (tid == 0) partL[(size_t)b * ntiles + tile] = ll;
  } else {
    // scalar-p path (one lane per observation): Y, Z, W land unscaled in the CSR rows, then
    // are scaled in place
    const size_t o = (size_t)tile * ET + tid;
    const int4 e = obs[o];
    const int4 q = pos[o];
    const double n = (double)e.w;
    double dsum = 1.0;
    double* ry = cb + (size_t)(q.x >= 0 ? q.x : 0) * K;
    double* rz = cb + (size_t)(q.y >= 0 ? q.y : 0) * K;
    double* rw = cb + (size_t)(q.z >= 0 ? q.z : 0) * K;
    if (q.x >= 0 && !(ablate & 1)) dsum = phase_a<K>(th, p, e, ry, rz, rw);
    const double d = dsum + eps;
    const double c = n / d;
    if (q.x >= 0 && !(ablate & 1)) {
#pragma unroll
      for (int g = 0; g < K; ++g) {
        ry[g] *= c;
        rz[g] *= c;
        rw[g] *= c;
      }
    }
    cvec[(size_t)b * n_obs_pad + o] = c;
    const double ll = block_sum(n * log(d), scratch);
    if (tid == 0) partL[(size_t)b * ntiles + tile] = ll;
  }
}

// ------------------------------------------------------------------------------------------
// M1 = S accumulation (:1012 npr scatter, factorised), grid (G, B), block 1024:
//      S_r[a b g] = sum_obs c th_i[a] th_j[b] th_k[g]
// Workgroup w owns a contiguous, balanced run of 64-observation tiles (one workgroup per CU,
// 16 waves: 4 per SIMD, which FP64 FMA needs).  The run is processed in windows of
// rating-uniform tiles: the window's c*theta_i / theta_j / theta_k rows are staged in LDS at
// once and consumed by a register-tiled outer product (lane = (a, b-chunk) cell block x link
// group; a group strides the whole window, so its loop is long and balanced).  Accumulators
// stay in VGPRs across windows and are folded across link groups through LDS in a fixed order
// (up to RED_SLOTS partial copies per round) once per rating: G partial rows per rating.
// ------------------------------------------------------------------------------------------
constexpr int M1_NT = 1024;

template <int K>
struct S1Plan {
  // cell budget: accumulators + the staged theta_k row fit 128 VGPRs (4 waves/SIMD)
  static constexpr int CELLS = (50 - 2 * K) < 40 ? ((50 - 2 * K) < K ? K : 50 - 2 * K) : 40;
  using S = SPlan<K, M1_NT, CELLS>;
  static constexpr int K3 = K * K * K;
  static constexpr int KP = (K + 1) & ~1;
  static constexpr int RS = (KP % 4 == 2) ? KP : KP + 2;  // conflict-free 16-lane b128 rows
  static constexpr int LDS_CAP = 144 * 1024;               // one workgroup per CU
  // observations staged per window (multiple of ET): ~3/4 of the LDS
  static constexpr int WOBS_RAW = (LDS_CAP * 3 / 4) / (3 * RS * 8 + 16) / ET * ET;
  static constexpr int WOBS = WOBS_RAW > 8 * ET ? 8 * ET : (WOBS_RAW < ET ? ET : WOBS_RAW);
  static constexpr int STAGE_DBL = 3 * WOBS * RS;
  static constexpr int SLOTS_FIT = (LDS_CAP / 8 - 2 * WOBS) / K3;
  static constexpr int RED_SLOTS_RAW = S::LG / 2 < SLOTS_FIT ? S::LG / 2 : SLOTS_FIT;
  static constexpr int RED_SLOTS = S::LG < 2 ? 0 : (RED_SLOTS_RAW < 1 ? 1 : RED_SLOTS_RAW);
  static constexpr int RED_DBL = RED_SLOTS * K3;
  static constexpr int BODY_DBL = ((STAGE_DBL > RED_DBL ? STAGE_DBL : RED_DBL) + 1) & ~1;
  static constexpr int WREC_DBL = WOBS + (3 * WOBS + 1) / 2;  // c (double) + 3 gene ids (int)
  static constexpr int LDS_BYTES = (BODY_DBL + WREC_DBL) * 8;
  static_assert(LDS_BYTES <= LDS_CAP + 16 * 1024, "M1 LDS plan over budget");
};

template <int K>
__global__ __launch_bounds__(M1_NT) void m1_kernel(
    const int4* __restrict__ obs, const int* __restrict__ tile_r, const double* __restrict__ theta,
    const double* __restrict__ cvec, double* __restrict__ partS, int P, int R,
    long long n_obs_pad, int G, int ablate) {
  using PL = S1Plan<K>;
  using SP = typename PL::S;
  constexpr int K3 = PL::K3, RS = PL::RS, WOBS = PL::WOBS;
  constexpr int NB = SP::NB, NBC = SP::NBC, NBLK = SP::NBLK, LG = SP::LG;
  const int b = blockIdx.y;
  const int tid = threadIdx.x;
  const double* __restrict__ th = theta + (size_t)b * P * K;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* As = smem;  // [WOBS][RS] c * theta_i
  double* Bs = As + WOBS * RS;
  double* Gs = Bs + WOBS * RS;
  double* Wc = smem + PL::BODY_DBL;
  int* Wg = reinterpret_cast<int*>(Wc + WOBS);
  const int w = blockIdx.x;
  const int T = (int)(n_obs_pad / ET);
  const int t0 = (int)((long long)w * T / G), t1 = (int)((long long)(w + 1) * T / G);
  double* __restrict__ rows = partS + ((size_t)b * G + w) * R * K3;
  for (int idx = tid; idx < R * K3; idx += M1_NT) rows[idx] = 0.0;  // ratings this run lacks
  if (ablate & 2) return;

  for (int set = 0; set < SP::NSETS; ++set) {
    int blk, grp;
    if constexpr (SP::NSETS == 1) {
      blk = tid % NBLK;
      grp = tid / NBLK;
    } else {
      blk = set * M1_NT + tid;
      grp = 0;
    }
    const bool active = (grp < LG) && (blk < NBLK);
    const int alpha = blk / NBC;
    const int beta0 = (blk % NBC) * NB;
    double acc[NB][K];
#pragma unroll
    for (int q = 0; q < NB; ++q)
#pragma unroll
      for (int g = 0; g < K; ++g) acc[q][g] = 0.0;

    // fold the link groups' accumulators (fixed order) and store rating cur_r's row
    auto flush = [&](int cur_r) {
      if constexpr (LG > 1) {
        double* red = smem;  // the staged rows are dead here
        int ng = LG;
        while (ng > 1) {
          const int k = (ng / 2 < PL::RED_SLOTS) ? ng / 2 : PL::RED_SLOTS;
          __syncthreads();
          if (active && grp >= ng - k && grp < ng) {
            double* dst = red + (size_t)(grp - (ng - k)) * K3 + (alpha * K + beta0) * K;
#pragma unroll
            for (int q = 0; q < NB; ++q)
              if (NB * NBC == K || beta0 + q < K)
#pragma unroll
                for (int g = 0; g < K; ++g) dst[q * K + g] = acc[q][g];
          }
          __syncthreads();
          if (active && grp < k) {
            const double* src = red + (size_t)grp * K3 + (alpha * K + beta0) * K;
#pragma unroll
            for (int q = 0; q < NB; ++q)
              if (NB * NBC == K || beta0 + q < K)
#pragma unroll
                for (int g = 0; g < K; ++g) acc[q][g] += src[q * K + g];
          }
          ng -= k;
        }
      }
      if (active && grp == 0) {
        double* dst = rows + (size_t)cur_r * K3 + (alpha * K + beta0) * K;
#pragma unroll
        for (int q = 0; q < NB; ++q)
          if (NB * NBC == K || beta0 + q < K)
#pragma unroll
            for (int g = 0; g < K; ++g) dst[q * K + g] = acc[q][g];
      }
#pragma unroll
      for (int q = 0; q < NB; ++q)
#pragma unroll
        for (int g = 0; g < K; ++g) acc[q][g] = 0.0;
    };

    int cur_r = tile_r[(t0 * ET) / TILE];
    int t = t0;
    while (t < t1) {
      // window: up to WOBS/ET tiles of one rating
      const int rt = tile_r[(t * ET) / TILE];
      if (rt != cur_r) {  // workgroup-uniform
        flush(cur_r);
        cur_r = rt;
      }
      int tw = t + 1;
      while (tw < t1 && tw - t < WOBS / ET && tile_r[(tw * ET) / TILE] == rt) ++tw;
      const int nobs = (tw - t) * ET;
      __syncthreads();  // previous window's readers are done with the stage / records
#pragma unroll 1
      for (int idx = tid; idx < nobs; idx += M1_NT) {
        const size_t oo = (size_t)t * ET + idx;
        const int4 e = obs[oo];
        Wg[idx * 3 + 0] = e.x;
        Wg[idx * 3 + 1] = e.y;
        Wg[idx * 3 + 2] = e.z;
        Wc[idx] = cvec[(size_t)b * n_obs_pad + oo];
      }
      __syncthreads();
#pragma unroll 1
      for (int idx = tid; idx < 3 * nobs; idx += M1_NT) {  // gather the window's theta rows
        const int l = idx % nobs, slot = idx / nobs;
        const double sc = slot == 0 ? Wc[l] : 1.0;
        const double* __restrict__ src = th + (size_t)Wg[l * 3 + slot] * K;
        double* dst = smem + (size_t)slot * WOBS * RS + l * RS;
#pragma unroll
        for (int g = 0; g < K; ++g) dst[g] = sc * src[g];
      }
      __syncthreads();
      if (active) {
#pragma unroll 1
        for (int l = grp; l < nobs; l += LG) {
          const double av = As[l * RS + alpha];
          double gv[K];
          lds_row<K>(gv, Gs + l * RS);
#pragma unroll
          for (int q = 0; q < NB; ++q) {
            if (NB * NBC == K || beta0 + q < K) {
              const double ab = av * Bs[l * RS + beta0 + q];
#pragma unroll
              for (int g = 0; g < K; ++g) acc[q][g] = fma(ab, gv[g], acc[q][g]);
            }
          }
        }
      }
      t = tw;
    }
    flush(cur_r);
  }
}

// CSR inversion: pos[obs][slot] = the CSR row of (obs, slot); -1 stays on padding rows.
__global__ void csr_invert_kernel(const int* __restrict__ ginc, long long nnz, int* __restrict__ pos) {
  const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q < nnz) {
    const int inc = ginc[q];
    pos[(size_t)(inc / 3) * 4 + inc % 3] = (int)q;
  }
}

// ------------------------------------------------------------------------------------------
// Which S-partial rows hold rating r (M2's view of partS):
//   row(b, w, r) = partS + ((b * G + w) * rs + r * ro) * K3,  w in [wlo[r], whi[r])
//   M1 layout: every workgroup writes every rating (rs = R, ro = 1, w in [0, G));
//   fused MFMA layout: a workgroup owns one rating (rs = 1, ro = 0, w in that rating's range).
// The fused kernel also reads grp[r] = first 16-observation group of rating r.
// ------------------------------------------------------------------------------------------
struct SRows {
  int wlo[MAX_R], whi[MAX_R];
  int grp[MAX_R + 1];
  int rs, ro;
};

// ------------------------------------------------------------------------------------------
// Fused E-step + S accumulation on FP64 MFMA (:987-1012), grid (G, B), block 64 * NW.
//
// v_mfma_f64_4x4x4f64 computes four independent 4x4x4 products ("blocks") per wave; with
// lane = 16 * hi + 4 * blk + lo its operands are A[blk][m = lo][k = hi], B[blk][k = hi][n = lo]
// and its result D[blk][m = hi][n = lo] (probed: tools/micro/mfma_layout.hip).  A wave takes
// 16 observations at a time (a "group"); observation oA = lane & 15 feeds the A side, the
// result rows belong to observation oD = 4 * blk + hi.
//   U-phase   U[o][a][b] = sum_g p_r[a][b][g] th_k[o][g]: per (a, b-block) tile 1 MFMA per
//             g-block (A = th_k of oA, B = p_r from LDS, the same in all four blocks).  Lane
//             (oD, lo) keeps b = 4 bb + lo, so Z[b] = sum_a th_i[a] U[a][b] is complete in the
//             lane and Y[a] = sum_b th_j[b] U[a][b] needs one quad butterfly.
//             d = eps + sum_a th_i[a] Y[a], c = n / d.
//   KR        c th_i[a] th_j[b] of the group's observations written to a per-wave LDS image.
//   W-phase   W'[o][g] = sum_(a,b) KR[o][(a,b)] p_r[a][b][g] (= c W): k over the K^2 cells.
//   S-phase   S[(a,b)][g] += sum_o KR[o][(a,b)] th_k[o][g]: k over the group's observations,
//             accumulators stay in registers across all the wave's groups.
// Contributions c Y, c Z, c W go to the observation's three gene-CSR rows (M2 multiplies by
// theta and divides by deg).  At the end the NW waves' S accumulators are summed in LDS in a
// fixed order: one partial S row per workgroup (each workgroup owns one rating).  Every sum
// has a fixed order: bitwise reproducible.
// ------------------------------------------------------------------------------------------
constexpr int XG = 16;  // observations per wave group

// Measurement builds only (-DEMX_AB=mask): bit 0 U-phase MFMAs, 1 W-phase MFMAs, 2 S-phase
// MFMAs replaced by VALU adds of the same operands; 3 no contribution stores; 4 no KR stores.
#ifndef EMX_AB
#define EMX_AB 0
#endif

template <int K>
struct XPlan {
  static constexpr int NG = (K + 3) / 4;      // 4-wide blocks of a / b / g
  static constexpr int KP = 4 * NG;
  static constexpr int K2 = K * K, K3 = K * K * K;
  static constexpr int NC = (K2 + 3) / 4;     // W-phase k-steps over the (a, b) cells
  static constexpr int KRW = 4 * NC;          // KR cells per observation (zero padded)
  static constexpr int KRS = KRW + 2;         // row stride = 2 (mod 4): conflict-free W reads
  static constexpr int NT4 = (K2 + 15) / 16;  // S-phase 16-cell tiles
  static constexpr int SACC = NT4 * NG;       // S accumulators per lane
  static constexpr int PW_ROWS = K2 + KP;     // p_r image rows (a, b) = a K + b, zero padded
  static constexpr int P_DBL = PW_ROWS * KP;  // p_r image [(a, b)][g], g zero padded
  static constexpr int IMG = 3 * XG * KP;     // th_i / th_j / th_k rows of the wave's group
  static constexpr int WAVE_DBL = XG * KRS + IMG;
  static constexpr int NW = (P_DBL + 8 * WAVE_DBL + 8) * 8 <= 160 * 1024 ? 8 : 4;
  static constexpr int NT = 64 * NW;
  static constexpr int LDS_BYTES = (P_DBL + NW * WAVE_DBL + 8) * 8;
  static constexpr bool ON = K >= 2 && K <= 12;
  static_assert(!ON || SACC * 64 <= WAVE_DBL, "S reduction must fit the wave images");
  static_assert(!ON || LDS_BYTES <= 160 * 1024, "fused E-step LDS plan over budget");
};

__device__ __forceinline__ double mfma4(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

// v within a quad of lanes, permuted by the DPP quad_perm CTRL (0xB1: xor 1, 0x4E: xor 2).
template <int CTRL>
__device__ __forceinline__ double quad_perm(double v) {
  const long long x = __double_as_longlong(v);
  const int l = __builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, false);
  const int h = __builtin_amdgcn_mov_dpp((int)(x >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)h << 32) | (unsigned int)l);
}

// LDS writes of this wave visible to its own later reads (no workgroup barrier; a wave's LDS
// operations execute in order, the fence only keeps the compiler from reordering them).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Optional per-wave phase clock (measurement builds only: -DEMX_TRACE=1, then MMSBM_TRACE=1):
// [wave][16] cycle sums.  Compiled out of the product build: each clock read would split the
// loop body into separate basic blocks and keep the scheduler from moving loads across them.
#ifndef EMX_TRACE
#define EMX_TRACE 0
#endif
struct XTrace {
  unsigned long long* out;
  __device__ __forceinline__ unsigned long long now() const {
    if constexpr (EMX_TRACE) return out ? clock64() : 0ull;
    return 0ull;
  }
};

template <int K>
__global__ __launch_bounds__(XPlan<K>::NT) void emx_kernel(
    const int4* __restrict__ obs, const int4* __restrict__ pos, const double* __restrict__ theta,
    const double* __restrict__ pr, double* __restrict__ contrib, double* __restrict__ partS,
    double* __restrict__ partL, SRows rg, int P, int R, long long nnz, int G, double eps,
    XTrace tr) {
  using X = XPlan<K>;
  constexpr int NG = X::NG, KP = X::KP, K2 = X::K2, K3 = X::K3, NC = X::NC, NT4 = X::NT4;
  constexpr int KRS = X::KRS, KRW = X::KRW, NW = X::NW, NT = X::NT, SACC = X::SACC;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* Pw = smem;  // [K^2 + KP][KP] p_r, row a K + b, columns g
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  double* KR = smem + X::P_DBL + wv * X::WAVE_DBL;  // [XG][KRS]
  double* TI = KR + XG * KRS;                        // [XG][KP] th_i of the group's observations
  double* TJ = TI + XG * KP;
  double* TK = TJ + XG * KP;
  double* scratch = smem + X::P_DBL + NW * X::WAVE_DBL;
  const int hi = lane >> 4, lo = lane & 3;
  const int oA = lane & 15, oD = 4 * ((lane >> 2) & 3) + hi;
  const int w = blockIdx.x, b = blockIdx.y;
  unsigned long long tph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const unsigned long long t_start = tr.now();
  int r = 0;
  while (r + 1 < R && w >= rg.whi[r]) ++r;  // workgroup-uniform
  const int nwg = rg.whi[r] - rg.wlo[r], lw = w - rg.wlo[r];
  const int ng = rg.grp[r + 1] - rg.grp[r];
  const int g0 = rg.grp[r] + (int)((long long)lw * ng / nwg);
  const int g1 = rg.grp[r] + (int)((long long)(lw + 1) * ng / nwg);
  const double* __restrict__ th = theta + (size_t)b * P * K;
  const double* __restrict__ p = pr + ((size_t)b * R + r) * K3;
  double* __restrict__ cb = contrib + (size_t)b * (nnz + 1) * K;

  // the first group's records and theta values are in flight while p_r is staged
  int grp = g0 + wv;
  int4 eA = make_int4(0, 0, 0, 0), eD = eA, qD = eA, nA = eA, nD = eA, nQ = eA;
  // records: e* = this group, n* = next group (loaded one iteration earlier, i.e. before the
  // previous group's stores), m* = the group after (loaded at the top of this iteration)
  double aU[NG], tjD[NG], tiD4[NG];  // th_k[oA][4s+hi], th_j[oD][4j+lo], th_i[oD][4j+lo]
  auto load_theta = [&](const int4& a, const int4& d, double (&u)[NG], double (&tj)[NG],
                        double (&ti)[NG]) {
#pragma unroll
    for (int s = 0; s < NG; ++s) {
      const int g = 4 * s + hi, v = 4 * s + lo;
      u[s] = g < K ? th[(size_t)a.z * K + g] : 0.0;
      tj[s] = v < K ? th[(size_t)d.y * K + v] : 0.0;
      ti[s] = v < K ? th[(size_t)d.x * K + v] : 0.0;
    }
  };
  if (grp < g1) {
    const size_t r0 = (size_t)grp * XG;
    eA = obs[r0 + oA];
    eD = obs[r0 + oD];
    qD = pos[r0 + oD];
    load_theta(eA, eD, aU, tjD, tiD4);
    const size_t r1 = (size_t)(grp + NW < g1 ? grp + NW : grp) * XG;
    nA = obs[r1 + oA];
    nD = obs[r1 + oD];
    nQ = pos[r1 + oD];
  }

  for (int idx = tid; idx < X::P_DBL; idx += NT) {
    const int g = idx % KP, row = idx / KP;
    Pw[idx] = (g < K && row < K2) ? p[row * K + g] : 0.0;
  }
  if constexpr (KRW > K2) {  // pad cells of the W-phase k-steps stay 0
    for (int idx = lane; idx < XG * (KRW - K2); idx += 64)
      KR[(idx / (KRW - K2)) * KRS + K2 + idx % (KRW - K2)] = 0.0;
  }
  __syncthreads();
  unsigned long long t0 = tr.now();
  tph[0] = t0 - t_start;

  double sacc[NT4][NG];
#pragma unroll
  for (int t = 0; t < NT4; ++t)
#pragma unroll
    for (int u = 0; u < NG; ++u) sacc[t][u] = 0.0;
  int ngrp = 0;

  while (grp < g1) {
    ++ngrp;
    // ---- theta images of this group (LDS), then prefetch the next group
#pragma unroll
    for (int s = 0; s < NG; ++s) {
      TK[oA * KP + 4 * s + hi] = aU[s];
      TJ[oD * KP + 4 * s + lo] = tjD[s];
      TI[oD * KP + 4 * s + lo] = tiD4[s];
    }
    const int gn = grp + NW;
    int4 mA, mD, mQ;
    {  // records of the group after next; past the end the current group is re-read
      // (branch-free, unused)
      const size_t r2 = (size_t)(gn + NW < g1 ? gn + NW : grp) * XG;
      mA = obs[r2 + oA];
      mD = obs[r2 + oD];
      mQ = pos[r2 + oD];
    }
    wave_lds_sync();

    // ---- U-phase: per a, NG x NG MFMAs with the NG (b-block) accumulators innermost
    double yp[K], zp[NG];
#pragma unroll
    for (int bb = 0; bb < NG; ++bb) zp[bb] = 0.0;
#pragma unroll
    for (int a = 0; a < K; ++a) {
      double bf[NG][NG];
#pragma unroll
      for (int bb = 0; bb < NG; ++bb)
#pragma unroll
        for (int s = 0; s < NG; ++s)  // b = 4 bb + lo >= K reads the next row: finite, and
          bf[bb][s] = Pw[(a * K + 4 * bb + lo) * KP + 4 * s + hi];  // th_j[b] = 0 drops it
      double acc[NG];
#pragma unroll
      for (int bb = 0; bb < NG; ++bb) acc[bb] = 0.0;
#pragma unroll
      for (int s = 0; s < NG; ++s)
#pragma unroll
        for (int bb = 0; bb < NG; ++bb)
          acc[bb] = (EMX_AB & 1) ? acc[bb] + aU[s] + bf[bb][s] : mfma4(aU[s], bf[bb][s], acc[bb]);
      const double ta = TI[oD * KP + a];
      double y = 0.0;
#pragma unroll
      for (int bb = 0; bb < NG; ++bb) {
        y = fma(tjD[bb], acc[bb], y);
        zp[bb] = fma(ta, acc[bb], zp[bb]);
      }
      yp[a] = y;
    }
    unsigned long long t1 = tr.now();
    tph[1] += t1 - t0;
    // theta values of the next group: in flight through the rest of this one
    double aU2[NG], tjD2[NG], tiD42[NG];
    load_theta(nA, nD, aU2, tjD2, tiD42);
    // d = eps + sum_b th_j[b] Z[b]: this lane's three b, then the quad
    double dsum = 0.0;
#pragma unroll
    for (int j = 0; j < NG; ++j) dsum = fma(tjD[j], zp[j], dsum);
    dsum += quad_perm<0xB1>(dsum);
    dsum += quad_perm<0x4E>(dsum);
#pragma unroll
    for (int a = 0; a < K; ++a) {
      yp[a] += quad_perm<0xB1>(yp[a]);
      yp[a] += quad_perm<0x4E>(yp[a]);
    }
    const double c = (double)eD.w / (dsum + eps);

    // ---- KR image: c th_i[a] th_j[b] for observation oA, a = hi + 4 j
    const double cA = __shfl(c, 16 * (oA & 3) + 4 * (oA >> 2), 64);
    double tj[K];
#pragma unroll
    for (int bq = 0; bq < K; ++bq) tj[bq] = TJ[oA * KP + bq];
    double* KRo = KR + oA * KRS;
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      const int a = hi + 4 * j;
      if (a < K) {
        const double ct = cA * TI[oA * KP + a];
#pragma unroll
        for (int bq = 0; bq < K; ++bq)
          if (!(EMX_AB & 16)) KRo[a * K + bq] = ct * tj[bq];
      }
    }
    wave_lds_sync();
    unsigned long long t2 = tr.now();
    tph[2] += t2 - t1;

    // ---- W-phase: W' = c W for observation oD, g = 4 u + lo
    // two accumulator sets (even / odd k-steps): 2 NG independent MFMA chains in flight
    double wacc[NG], wacc2[NG];
#pragma unroll
    for (int u = 0; u < NG; ++u) {
      wacc[u] = 0.0;
      wacc2[u] = 0.0;
    }
#pragma unroll
    for (int s = 0; s < NC; ++s) {
      const int cell = 4 * s + hi;
      const double av = KRo[cell];
      const double* pb = Pw + cell * KP + lo;  // rows >= K^2 are zero (KR is zero there too)
      double (&wa)[NG] = (s & 1) ? wacc2 : wacc;
#pragma unroll
      for (int u = 0; u < NG; ++u)
        wa[u] = (EMX_AB & 2) ? wa[u] + av + pb[4 * u] : mfma4(av, pb[4 * u], wa[u]);
    }
#pragma unroll
    for (int u = 0; u < NG; ++u) wacc[u] += wacc2[u];
    unsigned long long t3 = tr.now();
    tph[3] += t3 - t2;

    // ---- contributions of observation oD: entries 4 j + lo of its three gene-CSR rows
    if (!(EMX_AB & 8)) {
      const bool real = qD.x >= 0;  // padding observations write the trash row (nnz)
      double* ri = cb + (size_t)(real ? qD.x : nnz) * K;
      double* rj = cb + (size_t)(real ? qD.y : nnz) * K;
      double* rk = cb + (size_t)(real ? qD.z : nnz) * K;
#pragma unroll
      for (int j = 0; j < NG; ++j) {
        const int v = 4 * j + lo;
        const int vs = v < K ? v : K - 1;  // the ragged block's extra lanes repeat entry K-1
        double y = yp[4 * j];
#pragma unroll
        for (int t = 1; t < 4; ++t)
          if (4 * j + t < K && lo == t) y = yp[4 * j + t];
        double* trash = cb + (size_t)nnz * K;
        (v < K ? ri : trash)[vs] = c * y;
        (v < K ? rj : trash)[vs] = c * zp[j];
        (v < K ? rk : trash)[vs] = wacc[j];
      }
    }
    unsigned long long t4 = tr.now();
    tph[4] += t4 - t3;

    // ---- S-phase: k over the group's observations o = 4 s + hi
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int o = 4 * s + hi;
      double bS[NG];
#pragma unroll
      for (int u = 0; u < NG; ++u) bS[u] = TK[o * KP + 4 * u + lo];
      const double* KRs = KR + o * KRS;
#pragma unroll
      for (int t = 0; t < NT4; ++t) {
        const int cell = 16 * t + oA;
        const double av = KRs[cell < KRW ? cell : 0];  // cells >= K2 feed discarded S entries
#pragma unroll
        for (int u = 0; u < NG; ++u)
          sacc[t][u] = (EMX_AB & 4) ? sacc[t][u] + av + bS[u] : mfma4(av, bS[u], sacc[t][u]);
      }
    }
    wave_lds_sync();  // this group's image reads complete before the next group's writes
    t0 = tr.now();
    tph[5] += t0 - t4;

    eA = nA;
    eD = nD;
    qD = nQ;
    nA = mA;
    nD = mD;
    nQ = mQ;
#pragma unroll
    for (int s = 0; s < NG; ++s) {
      aU[s] = aU2[s];
      tjD[s] = tjD2[s];
      tiD4[s] = tiD42[s];
    }
    grp = gn;
  }

  __syncthreads();
  double* red = smem + X::P_DBL;  // [NW][SACC][64] over the wave images
#pragma unroll
  for (int t = 0; t < NT4; ++t)
#pragma unroll
    for (int u = 0; u < NG; ++u) red[(wv * SACC + t * NG + u) * 64 + lane] = sacc[t][u];
  __syncthreads();
  double* __restrict__ rowS = partS + ((size_t)b * G + w) * K3;
  for (int idx = tid; idx < SACC * 64; idx += NT) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < NW; ++q) s += red[q * SACC * 64 + idx];
    const int t = idx >> 6, ln = idx & 63;
    const int cell = 16 * (t / NG) + 4 * ((ln >> 2) & 3) + (ln >> 4);
    const int g = 4 * (t % NG) + (ln & 3);
    if (cell < K2 && g < K) rowS[cell * K + g] = s;
  }
  if (EMX_TRACE && tr.out && lane == 0) {
    const unsigned long long t_end = tr.now();
    unsigned long long* o = tr.out + ((size_t)(b * gridDim.x + w) * NW + wv) * 16;
    for (int q = 0; q < 6; ++q) o[q] = tph[q];
    o[6] = t_end - t0;
    o[7] = (unsigned long long)ngrp;
    o[8] = t_end - t_start;
  }
}

// ------------------------------------------------------------------------------------------
// Lean fused E-step + S (MMSBM_ESTEP=5, K <= 12): the same MFMA algebra as emx_kernel without
// the per-wave KR image (EML_NW waves per workgroup, default 8): the W- and S-phase A operands
// th_i[a] th_j[b] are formed from the theta images (LDS reads and a multiply), c enters W at
// the store and S through its B operand (c_o th_k[o][g]).  The W-phase k index runs over
// (a, b = 4 bb + hi) with b padded to KP (th_j is zero there), so every operand address is a
// lane base plus a constant.  Y is reduced per a (the lane keeps its entries a = 4 j + lo).
// ------------------------------------------------------------------------------------------
#ifndef EML_NW
#define EML_NW 8
#endif
template <int K>
struct XLPlan {
  static constexpr int NG = (K + 3) / 4, KP = 4 * NG;
  static constexpr int K2 = K * K, K3 = K * K * K;
  static constexpr int NC = (K2 + 3) / 4;     // W-phase k-steps over the (a, b) cells
  static constexpr int NT4 = (K2 + 15) / 16;  // S-phase 16-cell tiles
  static constexpr int SACC = NT4 * NG;
  static constexpr int PW_ROWS = K2 + KP;
  static constexpr int P_DBL = PW_ROWS * KP;
  static constexpr int IS = KP + 1;           // image row stride (odd: conflict-free)
  static constexpr int IMG = 3 * XG * IS;     // th_i / th_j / th_k rows of the group
  static constexpr int NW = EML_NW;
  static constexpr int NT = 64 * NW;
  static constexpr int SLOT = IMG > SACC * 64 ? IMG : SACC * 64;
  static constexpr int LDS_BYTES = (P_DBL + NW * SLOT) * 8;
  static constexpr bool ON = K >= 2 && K <= 12 && LDS_BYTES <= 160 * 1024;
};

template <int K>
__global__ __launch_bounds__(XLPlan<K>::NT) void eml_kernel(
    const int4* __restrict__ obs, const int4* __restrict__ pos, const double* __restrict__ theta,
    const double* __restrict__ pr, double* __restrict__ contrib, double* __restrict__ partS,
    SRows rg, int P, int R, long long nnz, int G, double eps) {
  using X = XLPlan<K>;
  constexpr int NG = X::NG, KP = X::KP, K2 = X::K2, K3 = X::K3, NC = X::NC, NT4 = X::NT4;
  constexpr int IS = X::IS, NW = X::NW, NT = X::NT, SACC = X::SACC;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* Pw = smem;  // [K^2 + KP][KP]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  double* TI = smem + X::P_DBL + wv * X::SLOT;  // [XG][IS]
  double* TJ = TI + XG * IS;
  double* TK = TJ + XG * IS;
  const int hi = lane >> 4, lo = lane & 3;
  const int oA = lane & 15, oD = 4 * ((lane >> 2) & 3) + hi;
  const int w = blockIdx.x, b = blockIdx.y;
  int r = 0;
  while (r + 1 < R && w >= rg.whi[r]) ++r;  // workgroup-uniform
  const int nwg = rg.whi[r] - rg.wlo[r], lw = w - rg.wlo[r];
  const int ng = rg.grp[r + 1] - rg.grp[r];
  const int g0 = rg.grp[r] + (int)((long long)lw * ng / nwg);
  const int g1 = rg.grp[r] + (int)((long long)(lw + 1) * ng / nwg);
  const double* __restrict__ th = theta + (size_t)b * P * K;
  const double* __restrict__ p = pr + ((size_t)b * R + r) * K3;
  double* __restrict__ cb = contrib + (size_t)b * (nnz + 1) * K;

  int grp = g0 + wv;
  // records kept field by field: k gene of oA; i, j genes, weight and CSR rows of oD
  int kA = 0, iD = 0, jD = 0, nD = 0, q0 = -1, q1 = -1, q2 = -1;
  int kA2 = 0, iD2 = 0, jD2 = 0, nD2 = 0, q02 = -1, q12 = -1, q22 = -1;
  double aU[NG], tjD[NG], tiD4[NG];
  auto load_theta = [&](int k_a, int i_d, int j_d, double (&u)[NG], double (&tj)[NG],
                        double (&ti)[NG]) {
#pragma unroll
    for (int s = 0; s < NG; ++s) {
      const int g = 4 * s + hi, v = 4 * s + lo;
      u[s] = g < K ? th[(size_t)k_a * K + g] : 0.0;
      tj[s] = v < K ? th[(size_t)j_d * K + v] : 0.0;
      ti[s] = v < K ? th[(size_t)i_d * K + v] : 0.0;
    }
  };
  if (grp < g1) {
    const size_t r0 = (size_t)grp * XG;
    const int4 a = obs[r0 + oA], d = obs[r0 + oD], q = pos[r0 + oD];
    kA = a.z; iD = d.x; jD = d.y; nD = d.w; q0 = q.x; q1 = q.y; q2 = q.z;
    load_theta(kA, iD, jD, aU, tjD, tiD4);
  }
  for (int idx = tid; idx < X::P_DBL; idx += NT) {
    const int g = idx % KP, row = idx / KP;
    Pw[idx] = (g < K && row < K2) ? p[row * K + g] : 0.0;
  }
  __syncthreads();

  double sacc[NT4][NG];
#pragma unroll
  for (int t = 0; t < NT4; ++t)
#pragma unroll
    for (int u = 0; u < NG; ++u) sacc[t][u] = 0.0;

  while (grp < g1) {
#pragma unroll
    for (int s = 0; s < NG; ++s) {
      TK[oA * IS + 4 * s + hi] = aU[s];
      TJ[oD * IS + 4 * s + lo] = tjD[s];
      TI[oD * IS + 4 * s + lo] = tiD4[s];
    }
    const int gn = grp + NW;
    {
      const size_t r1 = (size_t)(gn < g1 ? gn : grp) * XG;
      const int4 a = obs[r1 + oA], d = obs[r1 + oD], q = pos[r1 + oD];
      kA2 = a.z; iD2 = d.x; jD2 = d.y; nD2 = d.w; q02 = q.x; q12 = q.y; q22 = q.z;
    }
    wave_lds_sync();

    // ---- U-phase (Y reduced per a; the lane keeps a = 4 j + lo)
    double ysel[NG], zp[NG];
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      ysel[j] = 0.0;
      zp[j] = 0.0;
    }
#pragma unroll
    for (int a = 0; a < K; ++a) {
      double bf[NG][NG];
#pragma unroll
      for (int bb = 0; bb < NG; ++bb)
#pragma unroll
        for (int s = 0; s < NG; ++s) bf[bb][s] = Pw[(a * K + 4 * bb + lo) * KP + 4 * s + hi];
      double acc[NG];
#pragma unroll
      for (int bb = 0; bb < NG; ++bb) acc[bb] = 0.0;
#pragma unroll
      for (int s = 0; s < NG; ++s)
#pragma unroll
        for (int bb = 0; bb < NG; ++bb) acc[bb] = mfma4(aU[s], bf[bb][s], acc[bb]);
      const double ta = TI[oD * IS + a];
      double y = 0.0;
#pragma unroll
      for (int bb = 0; bb < NG; ++bb) {
        y = fma(tjD[bb], acc[bb], y);
        zp[bb] = fma(ta, acc[bb], zp[bb]);
      }
      y += quad_perm<0xB1>(y);
      y += quad_perm<0x4E>(y);
      if (lo == (a & 3)) ysel[a >> 2] = y;
      __builtin_amdgcn_sched_barrier(0);
    }
    double aU2[NG], tjD2[NG], tiD42[NG];
    load_theta(kA2, iD2, jD2, aU2, tjD2, tiD42);

    // ---- W-phase: A = th_i[a] th_j[b] of oA, k = (a, b = 4 bb + hi) with b padded to KP
    //      (th_j = 0 there), B = p[a][b][g]
    double wacc[NG], tjA[NG];
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      tjA[j] = TJ[oA * IS + 4 * j + hi];
      wacc[j] = 0.0;
    }
#pragma unroll
    for (int a = 0; a < K; ++a) {
      const double tia = TI[oA * IS + a];
#pragma unroll
      for (int bb = 0; bb < NG; ++bb) {
        const double av = tia * tjA[bb];
        const double* pb = Pw + (a * K + 4 * bb + hi) * KP + lo;
#pragma unroll
        for (int u = 0; u < NG; ++u) wacc[u] = mfma4(av, pb[4 * u], wacc[u]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    double dsum = 0.0;
#pragma unroll
    for (int j = 0; j < NG; ++j) dsum = fma(tjD[j], zp[j], dsum);
    dsum += quad_perm<0xB1>(dsum);
    dsum += quad_perm<0x4E>(dsum);
    const double c = (double)nD / (dsum + eps);

    // ---- contributions of observation oD: entries 4 j + lo of its three gene-CSR rows
    {
      const bool real = q0 >= 0;
      double* ri = cb + (size_t)(real ? q0 : nnz) * K;
      double* rj = cb + (size_t)(real ? q1 : nnz) * K;
      double* rk = cb + (size_t)(real ? q2 : nnz) * K;
      double* trash = cb + (size_t)nnz * K;
#pragma unroll
      for (int j = 0; j < NG; ++j) {
        const int v = 4 * j + lo;
        const int vs = v < K ? v : K - 1;
        (v < K ? ri : trash)[vs] = c * ysel[j];
        (v < K ? rj : trash)[vs] = c * zp[j];
        (v < K ? rk : trash)[vs] = c * wacc[j];
      }
    }

    // ---- S-phase: A = th_i th_j of o = 4 s + hi at cell 16 t + oA, B = c_o th_k[o].  The
    //      image bases pass through an empty asm each group: the per-(s, t) addresses are then
    //      formed in the loop as base + offset(t) with s folded into the instruction offset,
    //      instead of 8 NT4 loop-invariant registers.
    int zb = 0, oAv = oA;
    asm volatile("" : "+v"(zb), "+v"(oAv));
    const double* TIs = TI + zb + hi * IS;
    const double* TJs = TJ + zb + hi * IS;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int o = 4 * s + hi;
      const double co = __shfl(c, 16 * (o & 3) + 4 * (o >> 2), 64);
      double bS[NG];
#pragma unroll
      for (int u = 0; u < NG; ++u) bS[u] = co * TK[o * IS + 4 * u + lo];
#pragma unroll
      for (int t = 0; t < NT4; ++t) {
        const int cell = 16 * t + oAv;
        const int cc = cell < K2 ? cell : K2 - 1;  // cells >= K2 feed discarded S entries
        const double av = TIs[cc / K + 4 * s * IS] * TJs[cc % K + 4 * s * IS];
#pragma unroll
        for (int u = 0; u < NG; ++u) sacc[t][u] = mfma4(av, bS[u], sacc[t][u]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    wave_lds_sync();
    kA = kA2; iD = iD2; jD = jD2; nD = nD2; q0 = q02; q1 = q12; q2 = q22;
#pragma unroll
    for (int s = 0; s < NG; ++s) {
      aU[s] = aU2[s];
      tjD[s] = tjD2[s];
      tiD4[s] = tiD42[s];
    }
    grp = gn;
  }

  __syncthreads();
  double* red = smem + X::P_DBL;  // wave q's accumulators at red + q * SLOT, [SACC][64]
#pragma unroll
  for (int t = 0; t < NT4; ++t)
#pragma unroll
    for (int u = 0; u < NG; ++u) red[wv * X::SLOT + (t * NG + u) * 64 + lane] = sacc[t][u];
  __syncthreads();
  double* __restrict__ rowS = partS + ((size_t)b * G + w) * K3;
  for (int idx = tid; idx < SACC * 64; idx += NT) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < NW; ++q) s += red[q * X::SLOT + idx];
    const int t = idx >> 6, ln = idx & 63;
    const int cell = 16 * (t / NG) + 4 * ((ln >> 2) & 3) + (ln >> 4);
    const int g = 4 * (t % NG) + (ln & 3);
    if (cell < K2 && g < K) rowS[cell * K + g] = s;
  }
}

// ------------------------------------------------------------------------------------------
// Large-K FP64-MFMA path (13 <= K <= 32): E-step kernel emb_kernel<K>
// (U, Y, Z, W; c) then S accumulation m1x_kernel<K>, then m2_kernel on the same partial-row
// layout as the fused path (fused_rows).  Operand layout as in emx_kernel (lane = 16 hi + 4 blk
// + lo; A[blk][lo][hi], B[blk][hi][lo], D[blk][hi][lo]).
//
// emb_kernel: one 16-observation group per wave per round; the workgroup's waves run in
// lockstep rounds because p_r is staged in LDS in chunks of CH a-values (K^2 K doubles do not
// fit above K ~ 22): per chunk, every wave accumulates
//   U[oD][a][b] = sum_g p[a][b][g] th_k[oD][g]        (NG x NG MFMAs per a; A = th_k of oA)
//   Y[oD][a] = sum_b th_j[b] U[a][b]  (quad butterfly; the lane keeps a = 4 j + lo)
//   Z[oD][b] += th_i[a] U[a][b]       (b = 4 bb + lo, complete in the lane)
//   W[oD][g] += sum_b th_i[oA][a] th_j[oA][b] p[a][b][g]   (k = b = 4 bb + hi, NG x NG MFMAs)
// and after the last chunk d = eps + sum_b th_j[b] Z[b], c = n / d; c Y, c Z, c W go to the
// observation's three gene-CSR rows and c to cvec (M1 input).  Rounds = ceil(groups / NW); a
// wave without a group in the last round computes on a repeated group and stores nothing.
// ------------------------------------------------------------------------------------------
template <int K>
struct BPlan {
  static constexpr int NG = (K + 3) / 4, KP = 4 * NG;
  static constexpr int K2 = K * K, K3 = K * K * K;
#ifndef EMB_NW_SMALL  // measurement builds: waves per workgroup where all of p_r fits (K <= 20)
#define EMB_NW_SMALL 12
#endif
  // K <= 20: all of p_r plus 12 waves' images fit in LDS (3 waves per SIMD; K=20 x 8 samples:
  // 599 -> 544 us against 8 waves, 16 waves 670 us); above, 8 waves and p_r staged in chunks
  static constexpr int NW = K <= 20 ? EMB_NW_SMALL : 8, NT = 64 * NW;
  static constexpr int IS = KP + 1;                  // image row stride (odd)
  static constexpr int IMG = 2 * XG * IS;            // th_i / th_j rows of the wave's group
  // p image row stride: PS = 4 (mod 8) doubles makes both fragment reads conflict-free
  // (U-phase rows 4 bb + lo, columns 4 s + hi; W-phase rows 4 bb + hi, columns 4 u + lo: the
  // 8 addresses of a 32-lane ds_read_b64 group land on 8 distinct bank pairs)
  static constexpr int PS = (KP % 8 == 4) ? KP : KP + 4;
  static constexpr int LDS_CAP = 160 * 1024 / 8;     // doubles
  static constexpr int PAD_ROWS = KP - K + 1;        // b reads past K in the last a of a chunk
  static constexpr int CH_FIT = (LDS_CAP - NW * IMG - PAD_ROWS * PS) / (K * PS);
  static constexpr int CH = CH_FIT < K ? CH_FIT : K; // a-values per staged chunk
  static constexpr int NCH = (K + CH - 1) / CH;
  static constexpr int PW_DBL = (CH * K + PAD_ROWS) * PS;
  static constexpr int LDS_BYTES = (PW_DBL + NW * IMG) * 8;
  static constexpr bool ON = K >= 13 && K <= 32 && CH >= 1;
  static_assert(!ON || LDS_BYTES <= 160 * 1024, "big-K E-step LDS plan over budget");
};

template <int K>
__global__ __launch_bounds__(BPlan<K>::NT) void emb_kernel(
    const int4* __restrict__ obs, const int4* __restrict__ pos, const double* __restrict__ theta,
    const double* __restrict__ pr, double* __restrict__ contrib, double* __restrict__ cvec,
    SRows rg, int P, int R, long long n_obs_pad, long long nnz, double eps) {
  using X = BPlan<K>;
  constexpr int NG = X::NG, KP = X::KP, K3 = X::K3, IS = X::IS, NW = X::NW, NT = X::NT;
  constexpr int CH = X::CH, NCH = X::NCH, PS = X::PS;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* Pw = smem;  // [CH K + PAD_ROWS][PS]: rows (a - a0) K + b, columns g (zero padded)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  double* TI = smem + X::PW_DBL + wv * X::IMG;  // [XG][IS]
  double* TJ = TI + XG * IS;
  const int hi = lane >> 4, lo = lane & 3;
  const int oA = lane & 15, oD = 4 * ((lane >> 2) & 3) + hi;
  const int w = blockIdx.x, b = blockIdx.y;
  int r = 0;
  while (r + 1 < R && w >= rg.whi[r]) ++r;  // workgroup-uniform
  const int nwg = rg.whi[r] - rg.wlo[r], lw = w - rg.wlo[r];
  const int ng = rg.grp[r + 1] - rg.grp[r];
  const int g0 = rg.grp[r] + (int)((long long)lw * ng / nwg);
  const int g1 = rg.grp[r] + (int)((long long)(lw + 1) * ng / nwg);
  const int rounds = (g1 - g0 + NW - 1) / NW;
  const double* __restrict__ th = theta + (size_t)b * P * K;
  const double* __restrict__ p = pr + ((size_t)b * R + r) * K3;
  double* __restrict__ cb = contrib + (size_t)b * (nnz + 1) * K;

  // chunk of a-values [a0, a0 + CH) (rows past K^2 are zero).  Loads go out in batches of
  // SB from clamped (always valid) addresses, then the batch is stored: SB loads in flight
  // per thread instead of one load-store round trip per element
  auto stage = [&](int a0) {
    constexpr int NPER = (X::PW_DBL + NT - 1) / NT, SB = 12;
#pragma unroll
    for (int j0 = 0; j0 < NPER; j0 += SB) {
      double v[SB];
#pragma unroll
      for (int j = 0; j < SB; ++j) {
        const int idx = tid + (j0 + j) * NT;
        const int g = idx % PS, row = idx / PS;
        const int src = a0 * K + row;  // (a, b) cell index
        const bool in = g < K && src < K * K;
        const double x = p[(size_t)(in ? src : 0) * K + (in ? g : 0)];
        v[j] = in ? x : 0.0;
      }
#pragma unroll
      for (int j = 0; j < SB; ++j) {
        const int idx = tid + (j0 + j) * NT;
        if (j0 + j < NPER && idx < X::PW_DBL) Pw[idx] = v[j];
      }
    }
  };
  if constexpr (NCH == 1) {
    stage(0);
    __syncthreads();
  }

  for (int rd = 0; rd < rounds; ++rd) {
    const int gq = g0 + rd * NW + wv;
    const bool active = gq < g1;
    const size_t r0 = (size_t)(active ? gq : g0) * XG;
    const int4 eA = obs[r0 + oA], eD = obs[r0 + oD], qD = pos[r0 + oD];
    double aU[NG], tjD[NG], tjA[NG];
#pragma unroll
    for (int s = 0; s < NG; ++s) {
      const int g = 4 * s + hi, v = 4 * s + lo;
      aU[s] = g < K ? th[(size_t)eA.z * K + g] : 0.0;
      tjD[s] = v < K ? th[(size_t)eD.y * K + v] : 0.0;
      TI[oD * IS + v] = v < K ? th[(size_t)eD.x * K + v] : 0.0;
      TJ[oD * IS + v] = tjD[s];
    }
    wave_lds_sync();
#pragma unroll
    for (int s = 0; s < NG; ++s) tjA[s] = TJ[oA * IS + 4 * s + hi];

    double ysel[NG], zp[NG], wacc[NG];
#pragma unroll
    for (int j = 0; j < NG; ++j) {
      ysel[j] = 0.0;
      zp[j] = 0.0;
      wacc[j] = 0.0;
    }
    for (int ci = 0; ci < NCH; ++ci) {
      // odd rounds walk the chunks backwards, so a round starts on the chunk the previous
      // round ended with, which is still staged: NCH - 1 stagings per round instead of NCH
      const int ch = (rd & 1) ? NCH - 1 - ci : ci;
      const int a0 = ch * CH;
      const int a1 = a0 + CH < K ? a0 + CH : K;
      if constexpr (NCH > 1) {
        if (ci > 0 || rd == 0) {  // workgroup-uniform
          __syncthreads();  // every wave is done with the previous chunk
          stage(a0);
          __syncthreads();
        }
      }
#pragma unroll 1
      for (int a = a0; a < a1; ++a) {
        const double* Pa = Pw + (size_t)(a - a0) * K * PS;
        // U-phase: acc[bb] = U[oD][a][4 bb + lo]
        double acc[NG];
#pragma unroll
        for (int bb = 0; bb < NG; ++bb) acc[bb] = 0.0;
#pragma unroll
        for (int s = 0; s < NG; ++s) {
          double bf[NG];
#pragma unroll
          for (int bb = 0; bb < NG; ++bb) bf[bb] = Pa[(4 * bb + lo) * PS + 4 * s + hi];
#pragma unroll
          for (int bb = 0; bb < NG; ++bb) acc[bb] = mfma4(aU[s], bf[bb], acc[bb]);
        }
        // W-phase: A = th_i[oA][a] th_j[oA][4 bb + hi], B = p[a][4 bb + hi][4 u + lo]
        const double tia = TI[oA * IS + a];
#pragma unroll
        for (int bb = 0; bb < NG; ++bb) {
          const double av = tia * tjA[bb];
          const double* pb = Pa + (4 * bb + hi) * PS + lo;
#pragma unroll
          for (int u = 0; u < NG; ++u) wacc[u] = mfma4(av, pb[4 * u], wacc[u]);
        }
        const double ta = TI[oD * IS + a];
        double y = 0.0;
#pragma unroll
        for (int bb = 0; bb < NG; ++bb) {
          y = fma(tjD[bb], acc[bb], y);
          zp[bb] = fma(ta, acc[bb], zp[bb]);
        }
        y += quad_perm<0xB1>(y);
        y += quad_perm<0x4E>(y);
#pragma unroll
        for (int j = 0; j < NG; ++j)
          if (a == 4 * j + lo) ysel[j] = y;
      }
    }
    double dsum = 0.0;
#pragma unroll
    for (int j = 0; j < NG; ++j) dsum = fma(tjD[j], zp[j], dsum);
    dsum += quad_perm<0xB1>(dsum);
    dsum += quad_perm<0x4E>(dsum);
    const double c = (double)eD.w / (dsum + eps);
    if (active) {
      const bool real = qD.x >= 0;  // padding observations write the trash row (nnz)
      double* ri = cb + (size_t)(real ? qD.x : nnz) * K;
      double* rj = cb + (size_t)(real ? qD.y : nnz) * K;
      double* rk = cb + (size_t)(real ? qD.z : nnz) * K;
      double* trash = cb + (size_t)nnz * K;
#pragma unroll
      for (int j = 0; j < NG; ++j) {
        const int v = 4 * j + lo;
        const int vs = v < K ? v : K - 1;
        (v < K ? ri : trash)[vs] = c * ysel[j];
        (v < K ? rj : trash)[vs] = c * zp[j];
        (v < K ? rk : trash)[vs] = c * wacc[j];
      }
      if (lo == 0) cvec[(size_t)b * n_obs_pad + r0 + oD] = c;  // one writer per observation
    }
    wave_lds_sync();  // image reads of this round done before the next round's writes
  }
}

// ------------------------------------------------------------------------------------------
// m1x_kernel<K>: S_r[a][b][g] = sum_o c_o th_i[o][a] th_j[o][b] th_k[o][g] on FP64 MFMA, grid
// (G, B) over the fused_rows workgroup ranges (one rating per workgroup), NW waves.  The
// workgroup works in rounds of SG groups (OBS = 16 SG observations): c th_i, th_j, th_k rows
// of the round in an LDS image (double buffered).  Staging is register-prefetched: thread
// (o = tid / 8, q = tid % 8) holds the observation record two rounds ahead and its theta
// entries v = q + 8 m one round ahead, so the gathers' latency hides under the MFMA work and
// each round costs one workgroup barrier.
// S is tiled in 4 x 4 (a, b) blocks (ta, tb) x 4 g: block blk of the MFMA takes a = 4 ta + blk,
// rows b = 4 tb + lo (A) / 4 tb + hi (D), k = 4 observations (o = 4 s + hi), g = 4 u + lo.
// Wave wv owns the tiles t = ta NG + tb with t % NW == wv: accumulators stay in registers for
// the whole range and each wave writes its own tiles of the partial row: no cross-wave sum.
// ------------------------------------------------------------------------------------------
#ifndef MX_BIG_ROUND  // measurement builds: 128-observation single-buffered rounds at K <= 20
#define MX_BIG_ROUND 0
#endif
#ifndef MX_STEP_UNROLL  // measurement builds: step-loop unroll of m1x_kernel
#define MX_STEP_UNROLL 1
#endif
#ifndef MX_OCC4  // measurement builds: -DMX_OCC4=0 keeps m1x_kernel at 2 waves per SIMD
#define MX_OCC4 1
#endif
template <int K>
struct MXPlan {
  static constexpr int NG = (K + 3) / 4, KP = 4 * NG, K3 = K * K * K;
  static constexpr int NW = 8, NT = 64 * NW;
  static constexpr int NTILE = NG * NG;
  static constexpr int TPW = (NTILE + NW - 1) / NW;  // tiles per wave (last ones may be empty)
  static constexpr int IS = (KP % 8 == 4) ? KP : KP + 4;  // = 4 (mod 8): conflict-free fragments
  // rounds of SG groups; a single image buffer (two barriers per round) where MX_BIG_ROUND
  // doubles the round at K <= 20 within the same LDS (measurement switch)
  static constexpr bool ONEBUF = MX_BIG_ROUND && K <= 20;
  static constexpr int NBUF = ONEBUF ? 1 : 2;
  static constexpr int SG = ONEBUF ? 8 : 4;          // groups per round
  static constexpr int OBS = SG * XG;                // observations per round
  static constexpr int TPO = NT / OBS;               // staging threads per observation
  static constexpr int NV = (KP + TPO - 1) / TPO;    // theta entries per thread and slot
  static constexpr int IMG = 3 * OBS * IS;
  static constexpr int LDS_BYTES = NBUF * IMG * 8;
  // waves per SIMD (__launch_bounds__ minimum): two workgroups per CU where their LDS fits (K <= 20)
  static constexpr int OCC = MX_OCC4 && 2 * LDS_BYTES <= 160 * 1024 ? 4 : 2;
  static_assert(NT % OBS == 0, "staging map needs whole observations per thread set");
  static constexpr bool ON = K >= 13 && K <= 32 && LDS_BYTES <= 160 * 1024;
};

template <int K>
__global__ __launch_bounds__(MXPlan<K>::NT, MXPlan<K>::OCC) void m1x_kernel(
    const int4* __restrict__ obs, const double* __restrict__ theta, const double* __restrict__ cvec,
    double* __restrict__ partS, SRows rg, int P, int R, long long n_obs_pad, int G) {
  using X = MXPlan<K>;
  constexpr int NG = X::NG, KP = X::KP, IS = X::IS, NW = X::NW, NT = X::NT, TPW = X::TPW;
  constexpr int K3 = X::K3, OBS = X::OBS, IMG = X::IMG, TPO = X::TPO, NV = X::NV, SG = X::SG;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 4, blk = (lane >> 2) & 3, lo = lane & 3;
  const int w = blockIdx.x, b = blockIdx.y;
  int r = 0;
  while (r + 1 < R && w >= rg.whi[r]) ++r;
  const int nwg = rg.whi[r] - rg.wlo[r], lw = w - rg.wlo[r];
  const int ng = rg.grp[r + 1] - rg.grp[r];
  const int g0 = rg.grp[r] + (int)((long long)lw * ng / nwg);
  const int g1 = rg.grp[r] + (int)((long long)(lw + 1) * ng / nwg);
  const double* __restrict__ th = theta + (size_t)b * P * K;
  const double* __restrict__ cv = cvec + (size_t)b * n_obs_pad;
  const int nrounds = (g1 - g0 + SG - 1) / SG;

  double acc[TPW][NG];
#pragma unroll
  for (int t = 0; t < TPW; ++t)
#pragma unroll
    for (int u = 0; u < NG; ++u) acc[t][u] = 0.0;

  // staging role: observation so of a round, entries v = sq + TPO m of each slot
  const int so = tid / TPO, sq = tid % TPO;
  auto load_rec = [&](int rd, int4& e, double& c) {  // record + c of round rd (zero if absent)
    const int grp = g0 + rd * SG + so / XG;
    const bool ok = rd < nrounds && grp < g1;
    const size_t row = (size_t)(ok ? grp : g0) * XG + so % XG;
    e = obs[row];
    c = ok ? cv[row] : 0.0;
  };
  auto load_vals = [&](const int4& e, double c, double (&v)[3][NV]) {
#pragma unroll
    for (int m = 0; m < NV; ++m) {
      const int q = sq + TPO * m;
      const bool in = q < K;
      const int qs = in ? q : 0;
      v[0][m] = in ? c * th[(size_t)e.x * K + qs] : 0.0;
      v[1][m] = in ? th[(size_t)e.y * K + qs] : 0.0;
      v[2][m] = in ? th[(size_t)e.z * K + qs] : 0.0;
    }
  };
  auto store_vals = [&](double* img, const double (&v)[3][NV]) {
#pragma unroll
    for (int m = 0; m < NV; ++m) {
      const int q = sq + TPO * m;
      if (q < KP) {
#pragma unroll
        for (int sl = 0; sl < 3; ++sl) img[sl * OBS * IS + so * IS + q] = v[sl][m];
      }
    }
  };

  double vals[3][NV];
  int4 e1;
  double c1;
  if (nrounds > 0) {
    int4 e0;
    double c0;
    load_rec(0, e0, c0);
    load_rec(1, e1, c1);
    load_vals(e0, c0, vals);
    store_vals(smem, vals);
  }
  __syncthreads();
#pragma unroll 1
  for (int rd = 0; rd < nrounds; ++rd) {
    const bool more = rd + 1 < nrounds;  // workgroup-uniform
    int4 e2;
    double c2;
    if (more) {
      load_vals(e1, c1, vals);  // next round's theta entries (in flight during the MFMAs)
      load_rec(rd + 2, e2, c2);
    }
    const double* img = smem + (X::NBUF == 2 ? (rd & 1) * IMG : 0);
    const double* TIc = img;
    const double* TJ = img + OBS * IS;
    const double* TK = img + 2 * OBS * IS;
    const int nrem = g1 - (g0 + rd * SG);
    const int nobs = (nrem < SG ? nrem : SG) * XG;
    // the step loop for a compile-time tile count (no per-tile branch, so the step's LDS
    // reads are issued together and waited on once)
    auto steps = [&](auto ntc) {
      constexpr int NTL = decltype(ntc)::value;
#pragma unroll MX_STEP_UNROLL
      for (int s = 0; s < nobs / 4; ++s) {
        const int o = 4 * s + hi;
        double bk[NG];
#pragma unroll
        for (int u = 0; u < NG; ++u) bk[u] = TK[o * IS + 4 * u + lo];
#pragma unroll
        for (int t = 0; t < NTL; ++t) {
          const int tile = t * NW + wv;
          const int ta = tile / NG, tb = tile % NG;
          const double av = TIc[o * IS + 4 * ta + blk] * TJ[o * IS + 4 * tb + lo];
#pragma unroll
          for (int u = 0; u < NG; ++u) acc[t][u] = mfma4(av, bk[u], acc[t][u]);
        }
      }
    };
    // tiles t < TPW - 1 exist for every wave; the last one only where t NW + wv < NTILE
    if (X::NTILE % NW == 0 || (TPW - 1) * NW + wv < X::NTILE)
      steps(std::integral_constant<int, TPW>{});
    else
      steps(std::integral_constant<int, TPW - 1>{});
    if constexpr (X::NBUF == 1) __syncthreads();  // every wave is done with the image
    if (more) {
      // double buffered: the buffer last read in round rd - 1; single: the one just read
      store_vals(smem + (X::NBUF == 2 ? ((rd + 1) & 1) * IMG : 0), vals);
      e1 = e2;
      c1 = c2;
    }
    __syncthreads();
  }
  double* __restrict__ rowS = partS + ((size_t)b * G + w) * K3;
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int tile = t * NW + wv;
    if (tile < X::NTILE) {
      const int a = 4 * (tile / NG) + blk, bq = 4 * (tile % NG) + hi;
#pragma unroll
      for (int u = 0; u < NG; ++u) {
        const int g = 4 * u + lo;
        if (a < K && bq < K && g < K) rowS[((size_t)a * K + bq) * K + g] = acc[t][u];
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// M2, grid (p_blocks + P, B), block 256.
//  blocks [0, p_blocks): p (:1021-1028), 8 cells x 32 row slices per block.  Partial row n
//    (n < NR = G * rs) sits at partS + (b * NR + n) * K3 and belongs to rating n % R (M1
//    layout) or to the rating whose workgroup range holds n (fused layout).  Each thread loads
//    its rows MP_UNROLL at a time (one memory round trip for up to 256 rows), keeps a sum per
//    rating, then the 32 slices are added in a fixed order; npr_r = p_r S_r;
//    p_r <- npr_r / (eps + sum_r npr_r).
//  blocks [p_blocks, ...): theta (:1016-1018), in place, one workgroup per gene:
//      theta[g][a] <- theta[g][a] * (sum of the gene's contiguous c-scaled rows)[a] / deg[g]
//    thread = (row slot, entry a); fixed slot / accumulator / combine order: reproducible.
// ------------------------------------------------------------------------------------------
constexpr int MP_CELLS = 8, MP_SLICES = 32, MP_UNROLL = 8;

template <int K>
__global__ __launch_bounds__(256) void m2_kernel(double* __restrict__ pr, double* __restrict__ theta,
                                                 const double* __restrict__ partS,
                                                 const double* __restrict__ contrib,
                                                 const int* __restrict__ gptr,
                                                 const int* __restrict__ deg, SRows rg, int P,
                                                 int R, int G, long long nnz, int p_blocks,
                                                 double eps, int ablate,
                                                 double* __restrict__ nth_out,
                                                 double* __restrict__ S_out) {
  constexpr int K3 = K * K * K;
  const int b = blockIdx.y;
  const int tid = threadIdx.x;
  if ((int)blockIdx.x >= p_blocks) {  // --------------------------------------------- theta
    const int g = (int)blockIdx.x - p_blocks;
    if (g >= P || (ablate & 4)) return;  // workgroup-uniform
    constexpr int NS = 256 / K;          // row slots
    __shared__ double tred[256];
    const int slot = tid / K, k = tid % K;
    const int q0 = gptr[g], q1 = gptr[g + 1];
    double* row = theta + (size_t)b * P * K + (size_t)g * K;
    // the final update's operands load now, beside the row pointers, not after the reduction
    double th_old = 0.0, dg = 1.0;
    if (tid < K && !nth_out) {
      th_old = row[tid];
      dg = (double)deg[g];
    }
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    if (slot < NS) {
      const double* __restrict__ src = contrib + (size_t)b * (nnz + 1) * K + k;
      int q = q0 + slot;
      for (; q + 3 * NS < q1; q += 4 * NS) {
        a0 += src[(size_t)q * K];
        a1 += src[(size_t)(q + NS) * K];
        a2 += src[(size_t)(q + 2 * NS) * K];
        a3 += src[(size_t)(q + 3 * NS) * K];
      }
      for (; q < q1; q += NS) a0 += src[(size_t)q * K];
    }
    tred[tid] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    if (tid < K) {
      double sum = 0.0;
#pragma unroll
      for (int q = 0; q < NS; ++q) sum += tred[q * K + tid];
      if (nth_out) {  // link-sharded: this rank's sum, applied after the cross-rank reduction
        nth_out[(size_t)b * P * K + (size_t)g * K + tid] = sum;
      } else {
        row[tid] = th_old * sum / dg;
      }
    }
    return;
  }
  // ------------------------------------------------------------------------------------ p
  __shared__ double red[MAX_R][MP_SLICES][MP_CELLS];
  const int cl = tid % MP_CELLS, sl = tid / MP_CELLS;
  const int cell = blockIdx.x * MP_CELLS + cl;
  const int cc = cell < K3 ? cell : K3 - 1;
  const int NR = G * rg.rs;
  const double* __restrict__ base = partS + (size_t)b * NR * K3 + cc;
  double acc[MAX_R];
#pragma unroll
  for (int q = 0; q < MAX_R; ++q) acc[q] = 0.0;
  for (int n0 = 0; n0 < NR; n0 += MP_SLICES * MP_UNROLL) {
    double v[MP_UNROLL];
#pragma unroll
    for (int j = 0; j < MP_UNROLL; ++j) {
      const int n = n0 + sl + j * MP_SLICES;
      v[j] = n < NR ? base[(size_t)n * K3] : 0.0;
    }
#pragma unroll
    for (int j = 0; j < MP_UNROLL; ++j) {
      const int n = n0 + sl + j * MP_SLICES;
      if (n < NR) {
        int rr = 0;
        if (rg.rs == 1) {
#pragma unroll
          for (int q = 1; q < MAX_R; ++q)
            if (q < R && n >= rg.wlo[q]) rr = q;
        } else {
          rr = n % R;
        }
#pragma unroll
        for (int q = 0; q < MAX_R; ++q)
          if (q == rr) acc[q] += v[j];
      }
    }
  }
#pragma unroll
  for (int q = 0; q < MAX_R; ++q)
    if (q < R) red[q][sl][cl] = acc[q];
  __syncthreads();
  if (sl == 0 && cell < K3 && S_out) {  // link-sharded: this rank's S sums
    for (int q = 0; q < R; ++q) {
      double s = 0.0;
#pragma unroll
      for (int z = 0; z < MP_SLICES; ++z) s += red[q][z][cl];
      S_out[((size_t)b * R + q) * K3 + cell] = s;
    }
  } else if (sl == 0 && cell < K3) {
    double npr[MAX_R];
    double den = eps;
    double* pc = pr + (size_t)b * R * K3 + cell;
    for (int q = 0; q < R; ++q) {
      double s = 0.0;
#pragma unroll
      for (int z = 0; z < MP_SLICES; ++z) s += red[q][z][cl];
      npr[q] = pc[(size_t)q * K3] * s;
      den += npr[q];
    }
    for (int q = 0; q < R; ++q) pc[(size_t)q * K3] = npr[q] / den;
  }
}

// ------------------------------------------------------------------------------------------
// M-step from summed accumulators (link-sharded iteration, after the cross-rank all-reduce):
//   theta[g][a] <- theta[g][a] * nth[g][a] / deg[g]                          (:1016-1018)
//   p_r <- p_r S_r / (eps + sum_r p_r S_r)                                      (:1021-1028)
// with the same operation order as m2_kernel.  Grid (ceil((P K + K^3) / 256), B).
// ------------------------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__(256) void mapply_kernel(double* __restrict__ theta, double* __restrict__ pr,
                                                     const double* __restrict__ nth,
                                                     const double* __restrict__ S,
                                                     const int* __restrict__ deg, int P, int R,
                                                     double eps) {
  constexpr int K3 = K * K * K;
  const int b = blockIdx.y;
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long PK = (long long)P * K;
  if (idx < PK) {
    const int g = (int)(idx / K);
    double* t = theta + (size_t)b * PK + idx;
    *t = *t * nth[(size_t)b * PK + idx] / (double)deg[g];
  } else if (idx < PK + K3) {
    const int cell = (int)(idx - PK);
    double npr[MAX_R];
    double den = eps;
    double* pc = pr + (size_t)b * R * K3 + cell;
    const double* sc = S + (size_t)b * R * K3 + cell;
    for (int q = 0; q < R; ++q) {
      npr[q] = pc[(size_t)q * K3] * sc[(size_t)q * K3];
      den += npr[q];
    }
    for (int q = 0; q < R; ++q) pc[(size_t)q * K3] = npr[q] / den;
  }
}

// ------------------------------------------------------------------------------------------
// Log-likelihood partials (:958-969), one per 64-observation tile: grid (n_obs_pad/64, B).
//  K in the LDS plan: 128 threads, p_r staged in LDS, two lanes per observation (a halves);
//  otherwise 64 threads, p_r through the scalar cache.
// ------------------------------------------------------------------------------------------
constexpr int LL_TS = ET;

template <int K>
__global__ __launch_bounds__((EPlan<K>::NT)) void loglik_kernel(
    const int4* __restrict__ obs, const int* __restrict__ tile_r, const double* __restrict__ theta,
    const double* __restrict__ pr, double* __restrict__ partL, int P, int R, int ntiles,
    double eps) {
  using EP = EPlan<K>;
  constexpr int K3 = K * K * K, KP = EP::KP, KH = EP::KH, H = EP::H, NT = EP::NT;
  __shared__ __attribute__((aligned(16))) double Ps[EP::STAGE_P ? EP::P_DBL : 2];
  __shared__ double scratch[8];
  const int tile = blockIdx.x;
  const int b = blockIdx.y;
  const int tid = threadIdx.x;
  const int lo = tid / H, h = tid % H;
  const int r = __builtin_amdgcn_readfirstlane(tile_r[(tile * LL_TS) / TILE]);
  const double* __restrict__ th = theta + (size_t)b * P * K;
  const double* __restrict__ p = pr + ((size_t)b * R + r) * K3;
  const int4 e = obs[(size_t)tile * LL_TS + lo];
  double dsum;
  if constexpr (EP::STAGE_P) {
    stage_p<K>(Ps, p, tid, NT);
    __syncthreads();
    const double* __restrict__ ri = th + (size_t)e.x * K;
    const double* __restrict__ rj = th + (size_t)e.y * K;
    const double* __restrict__ rk = th + (size_t)e.z * K;
    double tj[K], tk[K];
#pragma unroll
    for (int g = 0; g < K; ++g) {
      tj[g] = rj[g];
      tk[g] = rk[g];
    }
    dsum = 0.0;
#pragma unroll 1
    for (int q = 0; q < KH; ++q) {
      const int a = h * KH + q;
      const bool valid = a < K;
      const int ac = valid ? a : K - 1;
      const double ta = valid ? ri[ac] : 0.0;
      const double* __restrict__ pa = Ps + EP::slab(ac);
      double y0 = 0.0, y1 = 0.0;
#pragma unroll
      for (int bb = 0; bb < K; bb += 2) {
        double u0 = 0.0, u1 = 0.0;
#pragma unroll
        for (int g = 0; g < (K & ~1); g += 2) {
          const double2 v0 = *reinterpret_cast<const double2*>(pa + bb * KP + g);
          u0 = fma(v0.y, tk[g + 1], fma(v0.x, tk[g], u0));
          if (bb + 1 < K) {
            const double2 v1 = *reinterpret_cast<const double2*>(pa + (bb + 1) * KP + g);
            u1 = fma(v1.y, tk[g + 1], fma(v1.x, tk[g], u1));
          }
        }
        if constexpr (K & 1) {
          u0 = fma(pa[bb * KP + K - 1], tk[K - 1], u0);
          if (bb + 1 < K) u1 = fma(pa[(bb + 1) * KP + K - 1], tk[K - 1], u1);
        }
        y0 = fma(tj[bb], u0, y0);
        if (bb + 1 < K) y1 = fma(tj[bb + 1], u1, y1);
      }
      dsum = fma(ta, y0 + y1, dsum);
    }
    dsum += __shfl_xor(dsum, 1, 64);  // partner lane's a-half (commutative: lanes agree)
  } else {
    dsum = contract<K>(th, p, e.x, e.y, e.z);
  }
  const double d = dsum + eps;
  const double ll = block_sum(h == 0 ? (double)e.w * log(d) : 0.0, scratch);
  if (tid == 0) partL[(size_t)b * ntiles + tile] = ll;
}

// Fixed-order sum of per-tile partials: grid (B), block 256.
__global__ __launch_bounds__(256) void reduce_kernel(const double* __restrict__ partL, int ntiles,
                                                     double* __restrict__ out) {
  __shared__ double scratch[4];
  const int b = blockIdx.x;
  double s = 0.0;
  for (int t = threadIdx.x; t < ntiles; t += blockDim.x) s += partL[(size_t)b * ntiles + t];
  s = block_sum(s, scratch);
  if (threadIdx.x == 0) out[b] = s;
}

// ------------------------------------------------------------------------------------------
// Prediction (:530-547): P(r=1) = sum th th th p[..][1], no eps.  grid (ceil(n/256), B).
// ------------------------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__(256) void predict_kernel(const int* __restrict__ ids, long long n,
                                                      const double* __restrict__ theta,
                                                      const double* __restrict__ pr,
                                                      double* __restrict__ out, int P, int R) {
  constexpr int K3 = K * K * K;
  const int b = blockIdx.y;
  const long long row = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= n) return;
  const double* __restrict__ th = theta + (size_t)b * P * K;
  const double* __restrict__ p = pr + ((size_t)b * R + 1) * K3;
  out[(size_t)b * n + row] = contract<K>(th, p, ids[3 * row], ids[3 * row + 1], ids[3 * row + 2]);
}

// ------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------
struct LinkSet {
  const int4* obs = nullptr;
  long long n_obs_pad = 0;
  int ntiles = 0;
  std::vector<int64_t> seg;  // row offsets, R+1
  int* tile_r = nullptr;     // device, owned
};

size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

struct Launch {
  bool fused;  // emx_kernel compiled for this K
  bool lean;   // eml_kernel is the default fused kernel for this K
  bool big;    // large-K MFMA path (emb_kernel + m1x_kernel) compiled for this K
  int (*emb)(mmsbm_ctx*, hipStream_t);
  int (*m1x)(mmsbm_ctx*, hipStream_t);
  int (*emx)(mmsbm_ctx*, hipStream_t);
  int (*estep)(mmsbm_ctx*, hipStream_t);
  int (*m1)(mmsbm_ctx*, hipStream_t);
  int (*m2)(mmsbm_ctx*, hipStream_t, bool);
  int (*mapply)(mmsbm_ctx*, double*, double*, const double*, const double*, hipStream_t);
  int (*loglik)(mmsbm_ctx*, int, const double*, const double*, hipStream_t);
  int (*predict)(mmsbm_ctx*, const int*, long long, const double*, const double*, double*,
                 hipStream_t);
};

}  // namespace

struct mmsbm_ctx {
  int device = 0;
  int K = 0, R = 0, B = 0, P = 0;
  double eps = 1e-10;
  LinkSet sets[2];
  const int* gptr = nullptr;
  const int* ginc = nullptr;
  int* pos = nullptr;  // device, owned: [n_obs_pad][4] CSR rows of each observation's slots
  const int* deg = nullptr;
  long long nnz = 0;
  bool genes_set = false;
  bool zero_degree = false;
  char* ws = nullptr;
  long long ws_bytes = 0;
  double* contrib = nullptr;
  double* cvec = nullptr;
  double* partS = nullptr;
  double* partL = nullptr;
  double* nth_out = nullptr;  // set only inside mmsbm_accumulate (link-sharded sums)
  double* S_out = nullptr;
  // current iterate (only valid during a call)
  double* theta_mut = nullptr;
  double* pr_mut = nullptr;
  // optional per-kernel timing: HIP event pairs recorded around each launch on its stream
  bool timing = false;
  int timing_stride = 1;  // time every n-th iteration
  int ablate = 0;  // MMSBM_ABLATE (measurement only)
  int sacc_wgs = SACC_WGS;  // S-accumulation workgroups requested (MMSBM_SACC_WGS)
  bool sacc_set = false;    // MMSBM_SACC_WGS given: per-sample count fixed, not batch-scaled
  // MMSBM_ESTEP: 0 fused MFMA E-step + S where compiled (else 2); 1 two-lane VALU E-step + M1;
  // 2 four-lane VALU E-step + M1
  int estep_variant = 0;
  std::vector<hipEvent_t> ev[3];  // start/stop pairs per kernel id (E, M1, M2)
  // MMSBM_TRACE (measurement only): per-wave phase cycles of the fused kernel's last launch
  unsigned long long* trace = nullptr;
  long long trace_waves = 0;
  size_t nev[3] = {0, 0, 0};
};

namespace {

struct WsLayout {
  size_t contrib, cvec, partS, partL, total;
};

// S-accumulation workgroups actually launched: never more than the train set's tiles.
int sacc_groups(const mmsbm_ctx* c) {
  const long long T = c->sets[MMSBM_SET_TRAIN].n_obs_pad / ET;
  long long G = c->sacc_wgs < SACC_WGS_MAX ? c->sacc_wgs : SACC_WGS_MAX;
  if (G > T) G = T;
  return (int)(G > 0 ? G : 1);
}

// Workgroups per sample of the group-range kernels (emx / eml / emb / m1x): the launch is
// (G, B), so G = ceil(target / B) keeps the grid near `target` workgroups whatever the batch
// (target = workgroups resident at once: one per CU, two for m1x at K <= 20).  Fewer, longer
// workgroup ranges remove the 16-observation quantization tail of short ranges and restage p
// less often (K=10 x 8 samples: 40.5k -> 48.5k sample-iterations/s; K=20 x 8: 8.8k -> 10.7k).
// MMSBM_SACC_WGS fixes the per-sample count instead.
long long range_wgs(const mmsbm_ctx* c, int target) {
  long long req = c->sacc_set ? c->sacc_wgs : (target + c->B - 1) / c->B;
  if (req > SACC_WGS_MAX) req = SACC_WGS_MAX;
  return req > 0 ? req : 1;
}
constexpr int RANGE_TARGET = SACC_WGS;       // emx / eml / emb: one workgroup per CU
constexpr int RANGE_TARGET_MAX = 2 * SACC_WGS;
template <int K>
constexpr int mx_target() {  // m1x: two workgroups per CU where their LDS fits
  return MXPlan<K>::OCC == 4 ? RANGE_TARGET_MAX : RANGE_TARGET;
}
enum class EPath { VALU, FUSED, BIG };
EPath epath(const mmsbm_ctx* c);

// Workgroups of the fused kernel: each owns one rating; a rating gets a share of the requested
// count proportional to its 16-observation groups (at least 1 when it has any, at most its
// group count).  Returns the row description M2 reads and the total in *G.
SRows fused_rows(const mmsbm_ctx* c, int* G, int target = RANGE_TARGET) {
  SRows rg{};
  const LinkSet& tr = c->sets[MMSBM_SET_TRAIN];
  const long long T = tr.n_obs_pad / XG;
  const long long req = range_wgs(c, target);
  int w = 0;
  rg.grp[0] = 0;
  for (int r = 0; r < c->R; ++r) {
    const long long lo = tr.seg.size() > (size_t)r ? tr.seg[r] / XG : 0;
    const long long hi = tr.seg.size() > (size_t)r + 1 ? tr.seg[r + 1] / XG : 0;
    const long long ng = hi - lo;
    long long gr = 0;
    if (ng > 0) {
      gr = (long long)((double)req * (double)ng / (double)T + 0.5);
      if (gr < 1) gr = 1;
      if (gr > ng) gr = ng;
    }
    rg.grp[r + 1] = (int)hi;
    rg.wlo[r] = w;
    w += (int)gr;
    rg.whi[r] = w;
  }
  rg.rs = 1;
  rg.ro = 0;
  *G = w > 0 ? w : 1;
  return rg;
}

// M1 layout: every workgroup writes one row per rating.
SRows m1_rows(const mmsbm_ctx* c) {
  SRows rg{};
  const int G = sacc_groups(c);
  for (int r = 0; r < c->R; ++r) {
    rg.wlo[r] = 0;
    rg.whi[r] = G;
  }
  rg.rs = c->R;
  rg.ro = 1;
  return rg;
}

WsLayout ws_layout(const mmsbm_ctx* c) {
  WsLayout L{};
  int GX = 1;
  (void)fused_rows(c, &GX, RANGE_TARGET_MAX);  // the most rows any range kernel writes
  const LinkSet& tr = c->sets[MMSBM_SET_TRAIN];
  const LinkSet& te = c->sets[MMSBM_SET_TEST];
  const size_t K3 = (size_t)c->K * c->K * c->K;
  size_t off = 0;
  // c-scaled (Y, Z, W) rows in gene-CSR order, 3 per observation, + one trash row per sample
  // (row nnz: the fused kernel's stores for padding observations land there, branch-free)
  L.contrib = off;
  off += align_up((size_t)c->B * (tr.n_obs_pad * 3 + 1) * c->K * sizeof(double));
  L.cvec = off;
  off += align_up((size_t)c->B * tr.n_obs_pad * sizeof(double));
  L.partS = off;  // partial S rows: [B][G][R][K3] (M1) or [B][GX][K3] (fused)
  const size_t srows = std::max((size_t)sacc_groups(c) * c->R, (size_t)GX);
  off += align_up((size_t)c->B * srows * K3 * sizeof(double));
  L.partL = off;  // one log-likelihood partial per 64-observation tile / fused workgroup
  long long nt = (tr.n_obs_pad > te.n_obs_pad ? tr.n_obs_pad : te.n_obs_pad) / ET;
  if (nt < GX) nt = GX;
  off += align_up((size_t)c->B * (nt > 0 ? nt : 1) * sizeof(double));
  L.total = off;
  return L;
}

template <int K>
int launch_estep(mmsbm_ctx* c, hipStream_t s) {
  using EP = EPlan<K>;
  const LinkSet& tr = c->sets[MMSBM_SET_TRAIN];
  if (tr.ntiles == 0) return MMSBM_OK;
  if constexpr (E4Plan<K>::ON) {
    if (c->estep_variant != 1) {
      const int nt = (int)(tr.n_obs_pad / ET);
      estep4_kernel<K><<<dim3(nt, c->B), E4_NT, E4Plan<K>::LDS_BYTES, s>>>(
          tr.obs, reinterpret_cast<const int4*>(c->pos), tr.tile_r, c->theta_mut, c->pr_mut,
          c->contrib, c->cvec, c->partL, c->P, c->R, tr.n_obs_pad, c->nnz, nt, c->eps,
          c->ablate);
      HIP_TRY(hipGetLastError());
      return MMSBM_OK;
    }
  }
  const int nt = (int)(tr.n_obs_pad / EP::EOBS);
  estep_kernel<K><<<dim3(nt, c->B), EP::NT, EP::LDS_BYTES, s>>>(
      tr.obs, reinterpret_cast<const int4*>(c->pos), tr.tile_r, c->theta_mut, c->pr_mut,
      c->contrib, c->cvec, c->partL, c->P, c->R, tr.n_obs_pad, c->nnz, nt, c->eps, c->ablate);
  HIP_TRY(hipGetLastError());
  return MMSBM_OK;
}

template <int K>
int launch_m1(mmsbm_ctx* c, hipStream_t s) {
  const LinkSet& tr = c->sets[MMSBM_SET_TRAIN];
  if (tr.ntiles == 0) return MMSBM_OK;
  const int G = sacc_groups(c);
  static bool attr = false;  // LDS above 64 KB needs the opt-in once per kernel
  if (!attr) {
    HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&m1_kernel<K>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, S1Plan<K>::LDS_BYTES));
    attr = true;
  }
  m1_kernel<K><<<dim3(G, c->B), M1_NT, S1Plan<K>::LDS_BYTES, s>>>(
      tr.obs, tr.tile_r, c->theta_mut, c->cvec, c->partS, c->P, c->R, tr.n_obs_pad, G, c->ablate);
  HIP_TRY(hipGetLastError());
  return MMSBM_OK;
}

// Fused kernel choice: MMSBM_ESTEP=5 forces the lean kernel; by default it runs where the
// KR-image kernel only fits 4 waves per workgroup (K = 11, 12: measured 14-16 % faster there).
template <int K>
constexpr bool lean_default() {
  return XLPlan<K>::ON && (!XPlan<K>::ON || XPlan<K>::NW < 8);
}
template <int K>
bool use_lean(int variant) {
  return XLPlan<K>::ON && (variant == 5 || (variant == 0 && lean_default<K>()));
}

template <int K>
int launch_eml(mmsbm_ctx* c, hipStream_t s) {
  if constexpr (XLPlan<K>::ON) {
    const LinkSet& tr = c->sets[MMSBM_SET_TRAIN];
    if (tr.ntiles == 0) return MMSBM_OK;
    int G = 1;
    const SRows rg = fused_rows(c, &G);
    static bool attr = false;
    if (!attr) {
      HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&eml_kernel<K>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, XLPlan<K>::LDS_BYTES));
      attr = true;
    }
    eml_kernel<K><<<dim3(G, c->B), XLPlan<K>::NT, XLPlan<K>::LDS_BYTES, s>>>(
        tr.obs, reinterpret_cast<const int4*>(c->pos), c->theta_mut, c->pr_mut, c->contrib,
        c->partS, rg, c->P, c->R, c->nnz, G, c->eps);
    HIP_TRY(hipGetLastError());
    return MMSBM_OK;
  } else {
    return fail(MMSBM_ERR_UNSUPPORTED, "lean fused E-step not compiled for K=%d", K);
  }
}

template <int K>
int launch_emb(mmsbm_ctx* c, hipStream_t s) {
  if constexpr (BPlan<K>::ON) {
    const LinkSet& tr = c->sets[MMSBM_SET_TRAIN];
    if (tr.ntiles == 0) return MMSBM_OK;
    int G = 1;
    const SRows rg = fused_rows(c, &G);
    static bool attr = false;
    if (!attr) {
      HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&emb_kernel<K>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, BPlan<K>::LDS_BYTES));
      attr = true;
    }
    emb_kernel<K><<<dim3(G, c->B), BPlan<K>::NT, BPlan<K>::LDS_BYTES, s>>>(
        tr.obs, reinterpret_cast<const int4*>(c->pos), c->theta_mut, c->pr_mut, c->contrib,
        c->cvec, rg, c->P, c->R, tr.n_obs_pad, c->nnz, c->eps);
    HIP_TRY(hipGetLastError());
    return MMSBM_OK;
  } else {
    return fail(MMSBM_ERR_UNSUPPORTED, "large-K MFMA E-step not compiled for K=%d", K);
  }
}

template <int K>
int launch_m1x(mmsbm_ctx* c, hipStream_t s) {
  if constexpr (MXPlan<K>::ON) {
    const LinkSet& tr = c->sets[MMSBM_SET_TRAIN];
    if (tr.ntiles == 0) return MMSBM_OK;
    int G = 1;
    const SRows rg = fused_rows(c, &G, mx_target<K>());
    static bool attr = false;
    if (!attr) {
      HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&m1x_kernel<K>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, MXPlan<K>::LDS_BYTES));
      attr = true;
    }
    m1x_kernel<K><<<dim3(G, c->B), MXPlan<K>::NT, MXPlan<K>::LDS_BYTES, s>>>(
        tr.obs, c->theta_mut, c->cvec, c->partS, rg, c->P, c->R, tr.n_obs_pad, G);
    HIP_TRY(hipGetLastError());
    return MMSBM_OK;
  } else {
    return fail(MMSBM_ERR_UNSUPPORTED, "large-K MFMA S accumulation not compiled for K=%d", K);
  }
}

template <int K>
int launch_emx(mmsbm_ctx* c, hipStream_t s) {
  if constexpr (XLPlan<K>::ON) {
    if (use_lean<K>(c->estep_variant)) return launch_eml<K>(c, s);
  }
  if constexpr (XPlan<K>::ON) {
    const LinkSet& tr = c->sets[MMSBM_SET_TRAIN];
    if (tr.ntiles == 0) return MMSBM_OK;
    int G = 1;
    const SRows rg = fused_rows(c, &G);
    static bool attr = false;  // LDS above 64 KB needs the opt-in once per kernel
    if (!attr) {
      HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&emx_kernel<K>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, XPlan<K>::LDS_BYTES));
      attr = true;
    }
    emx_kernel<K><<<dim3(G, c->B), XPlan<K>::NT, XPlan<K>::LDS_BYTES, s>>>(
        tr.obs, reinterpret_cast<const int4*>(c->pos), c->theta_mut, c->pr_mut, c->contrib,
        c->partS, c->partL, rg, c->P, c->R, c->nnz, G, c->eps, XTrace{c->trace});
    c->trace_waves = (long long)G * c->B * XPlan<K>::NW;
    HIP_TRY(hipGetLastError());
    return MMSBM_OK;
  } else {
    return fail(MMSBM_ERR_UNSUPPORTED, "fused E-step not compiled for K=%d", K);
  }
}

template <int K>
int launch_m2(mmsbm_ctx* c, hipStream_t s, bool fused) {
  constexpr int K3 = K * K * K;
  const LinkSet& tr = c->sets[MMSBM_SET_TRAIN];
  if (tr.ntiles == 0) {
    if (c->nth_out) {  // a rank without train links contributes zeros
      HIP_TRY(hipMemsetAsync(c->nth_out, 0, sizeof(double) * c->B * c->P * K, s));
      HIP_TRY(hipMemsetAsync(c->S_out, 0, sizeof(double) * c->B * c->R * K3, s));
    }
    return MMSBM_OK;
  }
  int G = sacc_groups(c);
  SRows rg;
  if (fused) {  // the rows the S kernel wrote: emx / eml, or m1x on the large-K path
    int target = RANGE_TARGET;
    if constexpr (MXPlan<K>::ON) {
      if (epath(c) == EPath::BIG) target = mx_target<K>();
    }
    rg = fused_rows(c, &G, target);
  } else {
    rg = m1_rows(c);
  }
  const int p_blocks = (K3 + MP_CELLS - 1) / MP_CELLS;
  const int theta_blocks = c->P;  // one workgroup per gene
  m2_kernel<K><<<dim3(p_blocks + theta_blocks, c->B), 256, 0, s>>>(
      c->pr_mut, c->theta_mut, c->partS, c->contrib, c->gptr, c->deg, rg, c->P, c->R, G,
      c->nnz, p_blocks, c->eps, c->ablate, c->nth_out, c->S_out);
  HIP_TRY(hipGetLastError());
  return MMSBM_OK;
}

template <int K>
int launch_mapply(mmsbm_ctx* c, double* theta, double* pr, const double* nth, const double* S,
                  hipStream_t s) {
  const long long n = (long long)c->P * K + (long long)K * K * K;
  mapply_kernel<K><<<dim3((unsigned)((n + 255) / 256), c->B), 256, 0, s>>>(theta, pr, nth, S, c->deg,
                                                                           c->P, c->R, c->eps);
  HIP_TRY(hipGetLastError());
  return MMSBM_OK;
}

template <int K>
int launch_loglik(mmsbm_ctx* c, int which, const double* theta, const double* pr, hipStream_t s) {
  const LinkSet& ls = c->sets[which];
  if (ls.ntiles == 0) return MMSBM_OK;
  const int nt = (int)(ls.n_obs_pad / LL_TS);
  loglik_kernel<K><<<dim3(nt, c->B), EPlan<K>::NT, 0, s>>>(
      ls.obs, ls.tile_r, theta, pr, c->partL, c->P, c->R, nt, c->eps);
  HIP_TRY(hipGetLastError());
  return MMSBM_OK;
}

template <int K>
int launch_predict(mmsbm_ctx* c, const int* ids, long long n, const double* theta,
                   const double* pr, double* out, hipStream_t s) {
  if (n == 0) return MMSBM_OK;
  const long long nb = (n + 255) / 256;
  predict_kernel<K><<<dim3((unsigned)nb, c->B), 256, 0, s>>>(ids, n, theta, pr, out, c->P, c->R);
  HIP_TRY(hipGetLastError());
  return MMSBM_OK;
}

template <int... Ks>
constexpr auto make_table(std::integer_sequence<int, Ks...>) {
  return std::array<Launch, sizeof...(Ks)>{
      Launch{XPlan<Ks + 1>::ON, lean_default<Ks + 1>(), BPlan<Ks + 1>::ON && MXPlan<Ks + 1>::ON,
             &launch_emb<Ks + 1>, &launch_m1x<Ks + 1>, &launch_emx<Ks + 1>, &launch_estep<Ks + 1>, &launch_m1<Ks + 1>,
             &launch_m2<Ks + 1>, &launch_mapply<Ks + 1>, &launch_loglik<Ks + 1>, &launch_predict<Ks + 1>}...};
}

const auto kTable = make_table(std::make_integer_sequence<int, MMSBM_MAX_K>{});

// Which E-step path mmsbm_iterate runs (MMSBM_ESTEP: 0 default, 1/2 VALU, 5 lean fused):
//   FUSED  E-step + S in one kernel (emx / eml, K <= 12), then M2
//   BIG    emb_kernel (E) + m1x_kernel (S) on FP64 MFMA (13 <= K <= 32), then M2
//   VALU   estep_kernel + m1_kernel, then M2
EPath epath(const mmsbm_ctx* c) {
  const Launch& L = kTable[c->K - 1];
  if (L.fused && (c->estep_variant == 0 || c->estep_variant == 5)) return EPath::FUSED;
  if (L.big && c->estep_variant == 0) return EPath::BIG;
  return EPath::VALU;
}
int run_estep(mmsbm_ctx* c, EPath path, hipStream_t s) {
  const Launch& L = kTable[c->K - 1];
  return path == EPath::FUSED ? L.emx(c, s) : path == EPath::BIG ? L.emb(c, s) : L.estep(c, s);
}
int run_m1(mmsbm_ctx* c, EPath path, hipStream_t s) {
  const Launch& L = kTable[c->K - 1];
  return path == EPath::FUSED ? MMSBM_OK : path == EPath::BIG ? L.m1x(c, s) : L.m1(c, s);
}

int check_shape(const mmsbm_ctx* c) {
  if (c->K < 1 || c->K > MMSBM_MAX_K)
    return fail(MMSBM_ERR_UNSUPPORTED, "K=%d outside [1, %d]", c->K, MMSBM_MAX_K);
  return MMSBM_OK;
}
}  // namespace

namespace {
// Records one event of kernel `kid`'s next start/stop pair (grows the pool on demand).
int timing_mark(mmsbm_ctx* c, int kid, hipStream_t s) {
  if (!c->timing) return MMSBM_OK;
  auto& v = c->ev[kid];
  if (c->nev[kid] == v.size()) {
    hipEvent_t e;
    HIP_TRY(hipEventCreate(&e));
    v.push_back(e);
  }
  HIP_TRY(hipEventRecord(v[c->nev[kid]++], s));
  return MMSBM_OK;
}
}  // namespace

extern "C" {

int mmsbm_version(void) { return 1; }
int mmsbm_tile(void) { return TILE; }
const char* mmsbm_last_error(void) { return g_err.c_str(); }

int mmsbm_create(int device, mmsbm_ctx** out) {
  if (!out) return fail(MMSBM_ERR_INVALID, "out is null");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev)
    return fail(MMSBM_ERR_INVALID, "device %d outside [0, %d)", device, ndev);
  auto* c = new mmsbm_ctx();
  c->device = device;
  if (const char* ab = getenv("MMSBM_ABLATE")) c->ablate = atoi(ab);
  if (const char* v = getenv("MMSBM_ESTEP")) c->estep_variant = atoi(v);
  if (EMX_TRACE && getenv("MMSBM_TRACE")) {
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipMalloc(&c->trace, sizeof(unsigned long long) * 16 * 65536));
  }
  if (const char* t = getenv("MMSBM_SACC_WGS")) {
    const int v = atoi(t);
    if (v >= 1) {
      c->sacc_wgs = v;
      c->sacc_set = true;
    }
  }
  *out = c;
  return MMSBM_OK;
}

int mmsbm_destroy(mmsbm_ctx* c) {
  if (!c) return MMSBM_OK;
  (void)hipSetDevice(c->device);
  for (auto& s : c->sets)
    if (s.tile_r) (void)hipFree(s.tile_r);
  if (c->pos) (void)hipFree(c->pos);
  if (c->trace) (void)hipFree(c->trace);
  for (auto& v : c->ev)
    for (hipEvent_t e : v) (void)hipEventDestroy(e);
  delete c;
  return MMSBM_OK;
}

int mmsbm_set_shape(mmsbm_ctx* c, int32_t K, int32_t R, int32_t B, int32_t P, double eps) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  if (K < 1 || K > MMSBM_MAX_K)
    return fail(MMSBM_ERR_UNSUPPORTED, "K=%d outside [1, %d]", K, MMSBM_MAX_K);
  if (R < 2 || R > MAX_R) return fail(MMSBM_ERR_UNSUPPORTED, "R=%d outside [2, %d]", R, MAX_R);
  if (B < 1 || B > 65535) return fail(MMSBM_ERR_INVALID, "B=%d outside [1, 65535]", B);
  if (P < 1) return fail(MMSBM_ERR_INVALID, "P=%d < 1", P);
  if (!(eps >= 0.0)) return fail(MMSBM_ERR_INVALID, "eps must be >= 0");
  c->K = K;
  c->R = R;
  c->B = B;
  c->P = P;
  c->eps = eps;
  return MMSBM_OK;
}

int mmsbm_set_links(mmsbm_ctx* c, int32_t which, const int32_t* obs, int64_t n_obs_pad,
                    const int64_t* seg_host) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  if (c->R < 2) return fail(MMSBM_ERR_INVALID, "call mmsbm_set_shape first");
  if (which != MMSBM_SET_TRAIN && which != MMSBM_SET_TEST)
    return fail(MMSBM_ERR_INVALID, "which=%d", which);
  if (n_obs_pad < 0 || n_obs_pad % TILE != 0)
    return fail(MMSBM_ERR_INVALID, "n_obs_pad=%lld not a multiple of %d", (long long)n_obs_pad, TILE);
  if (n_obs_pad > 0 && (!obs || !seg_host)) return fail(MMSBM_ERR_INVALID, "null obs/seg");
  if (n_obs_pad * 3 >= (int64_t)1 << 31)
    return fail(MMSBM_ERR_UNSUPPORTED, "n_obs_pad=%lld too large for int32 incidences",
                (long long)n_obs_pad);
  LinkSet& ls = c->sets[which];
  HIP_TRY(hipSetDevice(c->device));
  std::vector<int> tr;
  std::vector<int64_t> seg(c->R + 1, 0);
  if (n_obs_pad > 0) {
    if (seg_host[0] != 0 || seg_host[c->R] != n_obs_pad)
      return fail(MMSBM_ERR_INVALID, "seg must run from 0 to n_obs_pad");
    for (int r = 0; r <= c->R; ++r) {
      seg[r] = seg_host[r];
      if (seg[r] % TILE) return fail(MMSBM_ERR_INVALID, "seg[%d] not tile aligned", r);
      if (r > 0 && seg[r] < seg[r - 1]) return fail(MMSBM_ERR_INVALID, "seg not monotone");
    }
    for (int r = 0; r < c->R; ++r)
      for (int64_t t = seg[r] / TILE; t < seg[r + 1] / TILE; ++t) tr.push_back(r);
  }
  if (ls.tile_r) {
    HIP_TRY(hipFree(ls.tile_r));
    ls.tile_r = nullptr;
  }
  if (!tr.empty()) {
    HIP_TRY(hipMalloc(&ls.tile_r, tr.size() * sizeof(int)));
    HIP_TRY(hipMemcpy(ls.tile_r, tr.data(), tr.size() * sizeof(int), hipMemcpyHostToDevice));
  }
  ls.obs = reinterpret_cast<const int4*>(obs);
  if (which == MMSBM_SET_TRAIN) c->genes_set = false;  // the incidence CSR must follow
  ls.n_obs_pad = n_obs_pad;
  ls.ntiles = (int)(n_obs_pad / TILE);
  ls.seg = seg;
  return MMSBM_OK;
}

int mmsbm_set_genes(mmsbm_ctx* c, const int32_t* gene_ptr, const int32_t* gene_inc, int64_t nnz,
                    const int32_t* deg) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  if (c->P < 1) return fail(MMSBM_ERR_INVALID, "call mmsbm_set_shape first");
  if (!gene_ptr || !deg || (nnz > 0 && !gene_inc)) return fail(MMSBM_ERR_INVALID, "null CSR");
  HIP_TRY(hipSetDevice(c->device));
  std::vector<int32_t> hdeg(c->P);
  HIP_TRY(hipMemcpy(hdeg.data(), deg, sizeof(int32_t) * c->P, hipMemcpyDeviceToHost));
  c->zero_degree = false;
  for (int g = 0; g < c->P; ++g)
    if (hdeg[g] <= 0) c->zero_degree = true;
  const LinkSet& tr = c->sets[MMSBM_SET_TRAIN];
  if (nnz > 3 * tr.n_obs_pad)
    return fail(MMSBM_ERR_INVALID, "nnz=%lld exceeds 3 x train rows: call mmsbm_set_links(TRAIN) first",
                (long long)nnz);
  if (c->pos) {
    HIP_TRY(hipFree(c->pos));
    c->pos = nullptr;
  }
  if (tr.n_obs_pad > 0) {
    HIP_TRY(hipMalloc(&c->pos, sizeof(int) * 4 * tr.n_obs_pad));
    HIP_TRY(hipMemset(c->pos, 0xFF, sizeof(int) * 4 * tr.n_obs_pad));
    if (nnz > 0) {
      csr_invert_kernel<<<(unsigned)((nnz + 255) / 256), 256>>>(gene_inc, nnz, c->pos);
      HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipDeviceSynchronize());
  }
  c->gptr = gene_ptr;
  c->ginc = gene_inc;
  c->deg = deg;
  c->nnz = nnz;
  c->genes_set = true;
  if (c->zero_degree)
    return fail(MMSBM_ERR_ZERO_DEGREE, "a gene has no train link (float division by zero)");
  return MMSBM_OK;
}

int mmsbm_workspace_bytes(const mmsbm_ctx* c, int64_t* bytes) {
  if (!c || !bytes) return fail(MMSBM_ERR_INVALID, "null argument");
  *bytes = (int64_t)ws_layout(c).total;
  return MMSBM_OK;
}

int mmsbm_set_workspace(mmsbm_ctx* c, void* ws, int64_t bytes) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  const WsLayout L = ws_layout(c);
  if (bytes < (int64_t)L.total)
    return fail(MMSBM_ERR_INVALID, "workspace %lld < %lld bytes", (long long)bytes,
                (long long)L.total);
  if (((uintptr_t)ws) & 255) return fail(MMSBM_ERR_INVALID, "workspace not 256-B aligned");
  c->ws = (char*)ws;
  c->ws_bytes = bytes;
  c->contrib = (double*)(c->ws + L.contrib);
  c->cvec = (double*)(c->ws + L.cvec);
  c->partS = (double*)(c->ws + L.partS);
  c->partL = (double*)(c->ws + L.partL);
  return MMSBM_OK;
}

int mmsbm_iterate(mmsbm_ctx* c, double* theta, double* pr, int32_t n_iters, void* stream) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  int rc = check_shape(c);
  if (rc) return rc;
  if (!c->genes_set) return fail(MMSBM_ERR_INVALID, "call mmsbm_set_genes first");
  if (c->zero_degree)
    return fail(MMSBM_ERR_ZERO_DEGREE, "a gene has no train link (float division by zero)");
  if (!c->ws || c->ws_bytes < (long long)ws_layout(c).total)
    return fail(MMSBM_ERR_INVALID, "workspace missing or too small");
  if (!theta || !pr) return fail(MMSBM_ERR_INVALID, "null theta/pr");
  if (n_iters < 0) return fail(MMSBM_ERR_INVALID, "n_iters < 0");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  const Launch& L = kTable[c->K - 1];
  c->theta_mut = theta;
  c->pr_mut = pr;
  const EPath path = epath(c);
  const bool fused = path == EPath::FUSED;
  const bool fused_rows_layout = path != EPath::VALU;  // partial S rows per fused_rows workgroup
  for (int it = 0; it < n_iters; ++it) {
    const bool mark = c->timing && (it % c->timing_stride == 0);
    if (mark && (rc = timing_mark(c, 0, s))) return rc;
    if ((rc = run_estep(c, path, s))) return rc;
    if (mark && (rc = timing_mark(c, 0, s))) return rc;
    if (!fused) {
      if (mark && (rc = timing_mark(c, 1, s))) return rc;
      if ((rc = run_m1(c, path, s))) return rc;
      if (mark && (rc = timing_mark(c, 1, s))) return rc;
    }
    if (mark && (rc = timing_mark(c, 2, s))) return rc;
    if ((rc = L.m2(c, s, fused_rows_layout))) return rc;
    if (mark && (rc = timing_mark(c, 2, s))) return rc;
  }
  if (c->trace && fused && n_iters > 0) {  // measurement only: phase cycles of the last launch
    const long long nw = c->trace_waves < 65536 ? c->trace_waves : 65536;
    std::vector<unsigned long long> h(nw * 16);
    HIP_TRY(hipStreamSynchronize(s));
    HIP_TRY(hipMemcpy(h.data(), c->trace, h.size() * 8, hipMemcpyDeviceToHost));
    double sum[9] = {0};
    unsigned long long mx = 0;
    for (long long i = 0; i < nw; ++i) {
      for (int q = 0; q < 9; ++q) sum[q] += (double)h[i * 16 + q];
      mx = std::max(mx, h[i * 16 + 8]);
    }
    fprintf(stderr,
            "[mmsbm trace] waves=%lld avg cycles: prologue %.0f  U %.0f  KR %.0f  W %.0f  "
            "stores %.0f  S %.0f  epilogue %.0f  groups %.2f  total %.0f (max %llu)\n",
            nw, sum[0] / nw, sum[1] / nw, sum[2] / nw, sum[3] / nw, sum[4] / nw, sum[5] / nw,
            sum[6] / nw, sum[7] / nw, sum[8] / nw, mx);
  }
  return MMSBM_OK;
}

int mmsbm_accumulate(mmsbm_ctx* c, const double* theta, const double* pr, double* nth, double* S,
                     void* stream) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  int rc = check_shape(c);
  if (rc) return rc;
  if (!c->genes_set) return fail(MMSBM_ERR_INVALID, "call mmsbm_set_genes first");
  if (!c->ws || c->ws_bytes < (long long)ws_layout(c).total)
    return fail(MMSBM_ERR_INVALID, "workspace missing or too small");
  if (!theta || !pr || !nth || !S) return fail(MMSBM_ERR_INVALID, "null pointer");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  const Launch& L = kTable[c->K - 1];
  // the E-step kernels only read theta / pr; m2 in sums-out mode writes nth / S, not them
  c->theta_mut = const_cast<double*>(theta);
  c->pr_mut = const_cast<double*>(pr);
  const EPath path = epath(c);
  if ((rc = run_estep(c, path, s))) return rc;
  if ((rc = run_m1(c, path, s))) return rc;
  c->nth_out = nth;
  c->S_out = S;
  rc = L.m2(c, s, path != EPath::VALU);
  c->nth_out = nullptr;
  c->S_out = nullptr;
  return rc;
}

int mmsbm_mstep(mmsbm_ctx* c, double* theta, double* pr, const double* nth, const double* S,
                void* stream) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  int rc = check_shape(c);
  if (rc) return rc;
  if (!c->genes_set) return fail(MMSBM_ERR_INVALID, "call mmsbm_set_genes first");
  if (c->zero_degree)
    return fail(MMSBM_ERR_ZERO_DEGREE, "a gene has no train link (float division by zero)");
  if (!theta || !pr || !nth || !S) return fail(MMSBM_ERR_INVALID, "null pointer");
  HIP_TRY(hipSetDevice(c->device));
  return kTable[c->K - 1].mapply(c, theta, pr, nth, S, (hipStream_t)stream);
}

int mmsbm_loglik(mmsbm_ctx* c, int32_t which, const double* theta, const double* pr, double* out,
                 void* stream) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  int rc = check_shape(c);
  if (rc) return rc;
  if (which != MMSBM_SET_TRAIN && which != MMSBM_SET_TEST)
    return fail(MMSBM_ERR_INVALID, "which=%d", which);
  if (!c->ws) return fail(MMSBM_ERR_INVALID, "workspace missing");
  if (!theta || !pr || !out) return fail(MMSBM_ERR_INVALID, "null pointer");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  const LinkSet& ls = c->sets[which];
  if (ls.ntiles == 0) {
    HIP_TRY(hipMemsetAsync(out, 0, sizeof(double) * c->B, s));
    return MMSBM_OK;
  }
  if ((rc = kTable[c->K - 1].loglik(c, which, theta, pr, s))) return rc;
  reduce_kernel<<<c->B, 256, 0, s>>>(c->partL, (int)(ls.n_obs_pad / LL_TS), out);
  HIP_TRY(hipGetLastError());
  return MMSBM_OK;
}

int mmsbm_predict(mmsbm_ctx* c, const int32_t* ids, int64_t n, const double* theta,
                  const double* pr, double* out, void* stream) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  int rc = check_shape(c);
  if (rc) return rc;
  if (n < 0 || (n > 0 && (!ids || !theta || !pr || !out)))
    return fail(MMSBM_ERR_INVALID, "bad arguments");
  HIP_TRY(hipSetDevice(c->device));
  return kTable[c->K - 1].predict(c, ids, n, theta, pr, out, (hipStream_t)stream);
}

int mmsbm_fused(const mmsbm_ctx* c, int32_t* fused) {
  if (!c || !fused) return fail(MMSBM_ERR_INVALID, "null argument");
  int rc = check_shape(c);
  if (rc) return rc;
  const Launch& L = kTable[c->K - 1];
  const EPath path = epath(c);
  *fused = path == EPath::BIG ? 3 : path == EPath::VALU ? 0 : (c->estep_variant == 5 || L.lean) ? 2 : 1;
  return MMSBM_OK;
}

int mmsbm_timing(mmsbm_ctx* c, int32_t stride) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  c->timing = stride > 0;
  c->timing_stride = stride > 0 ? stride : 1;
  for (auto& n : c->nev) n = 0;
  return MMSBM_OK;
}

int mmsbm_time_estep(mmsbm_ctx* c, double* theta, double* pr, int32_t n, void* stream,
                     double* avg_ms) {
  if (!c || !theta || !pr || !avg_ms || n < 1) return fail(MMSBM_ERR_INVALID, "bad arguments");
  int rc = check_shape(c);
  if (rc) return rc;
  if (!c->genes_set || !c->ws) return fail(MMSBM_ERR_INVALID, "links / workspace not set");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  const Launch& L = kTable[c->K - 1];
  const EPath path = epath(c);
  c->theta_mut = theta;
  c->pr_mut = pr;
  hipEvent_t e0, e1;
  HIP_TRY(hipEventCreate(&e0));
  HIP_TRY(hipEventCreate(&e1));
  HIP_TRY(hipEventRecord(e0, s));
  for (int i = 0; i < n && rc == MMSBM_OK; ++i) rc = run_estep(c, path, s);
  HIP_TRY(hipEventRecord(e1, s));
  HIP_TRY(hipEventSynchronize(e1));
  float ms = 0.f;
  HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (rc) return rc;
  *avg_ms = (double)ms / n;
  return MMSBM_OK;
}

int mmsbm_timing_result(mmsbm_ctx* c, int32_t kernel, double* total_ms, int64_t* count) {
  if (!c || !total_ms || !count) return fail(MMSBM_ERR_INVALID, "null argument");
  if (kernel < 0 || kernel > 2) return fail(MMSBM_ERR_INVALID, "kernel id %d", kernel);
  const size_t n = c->nev[kernel] / 2;
  double tot = 0.0;
  if (n) HIP_TRY(hipEventSynchronize(c->ev[kernel][2 * n - 1]));
  for (size_t i = 0; i < n; ++i) {
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, c->ev[kernel][2 * i], c->ev[kernel][2 * i + 1]));
    tot += ms;
  }
  *total_ms = tot;
  *count = (int64_t)n;
  return MMSBM_OK;
}

}  // extern "C"
