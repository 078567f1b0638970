// mmsbm.hip — MI355X (gfx950) MMSBM EM engine: kernels + C ABI (include/mmsbm.h).
//
// Hot path of AleixMT/TrigenicInteractionPredictor, src/TrigenicInteractionPredictor.py:
//   make_iteration      :984-1043   -> estep_kernel + mstep_kernel (theta and p halves)
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

#include <array>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "mmsbm.h"

namespace {

constexpr int TILE = MMSBM_TILE;
constexpr int MAX_R = 8;
constexpr int LDS_BUDGET = 64 * 1024;
constexpr int MIN_TS = 64;  // smallest E-step tile (observations per workgroup)

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
  // cells per lane = NB * K <= 64 doubles; prefer a divisor of K (no ragged b-chunk).
  int cap = 64 / K;
  if (cap < 1) cap = 1;
  if (cap > K) cap = K;
  int best = 1;
  for (int d = 1; d <= cap; ++d)
    if (K % d == 0) best = d;
  return (2 * best >= cap) ? best : cap;
}

// Phase-B (S accumulation) tiling for NT threads: lane = (cell block, link group).
template <int K, int NT>
struct SPlan {
  static constexpr int K3 = K * K * K;
  static constexpr int NB = pick_nb(K);    // b-chunk per lane
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
// Returns sum_a th_i[a] Y[a]; stores Y, Z, W (unscaled) into crow[0:K], [K:2K], [2K:3K].
// ------------------------------------------------------------------------------------------
template <int K>
__device__ __forceinline__ double phase_a(const double* __restrict__ th, const double* __restrict__ p,
                                          const int4 e, double* __restrict__ crow) {
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
      crow[a] = y;
      dsum = fma(ta, y, dsum);
    }
#pragma unroll
    for (int g = 0; g < K; ++g) {
      crow[K + g] = zc[g];
      crow[2 * K + g] = wc[g];
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
      crow[a] = y;
      dsum = fma(ta, y, dsum);
    }
#pragma unroll
    for (int g = 0; g < K; ++g) crow[K + g] = zc[g];
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
    for (int g = 0; g < K; ++g) crow[2 * K + g] = wc[g];
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
// E-step plan.  TS observations per workgroup, H lanes per observation (NT = TS*H threads).
//   K <= 12: p_r is staged in LDS once per workgroup and read with ds_read_b128 (broadcast);
//            H = 2: the two lanes of an observation split the a-range and exchange their
//            Z / W / d partials with one lane swap (2x the waves of one-lane-per-observation:
//            a fold0-sized problem otherwise leaves ~1 wave per SIMD to hide all latency).
//   K > 12:  p_r streams through the scalar cache (SGPR operands), H = 1.
// LDS: Ps [K slabs of K*KP, second half shifted by 16 B so the two lanes' reads hit distinct
//      banks], Ri/Rj/Rk [TS][RS] theta rows of every observation (RS = 2 mod 4 doubles:
//      conflict-free 16-lane ds_read_b128), Cv [TS] c = n/d, red (phase-B reduction, aliases
//      the rows once accumulation is done), 8 doubles of block-sum scratch.
// ------------------------------------------------------------------------------------------
template <int K, int TS>
struct EPlan {
  static constexpr bool STAGE_P = K <= 12;
  static constexpr int H = STAGE_P ? 2 : 1;
  static constexpr int NT = TS * H;
  using S = SPlan<K, NT>;
  static constexpr int K3 = K * K * K;
  static constexpr int KP = (K + 1) & ~1;
  static constexpr int KH = (K + H - 1) / H;   // a-range per lane
  static constexpr int RS = (KP % 4 == 2) ? KP : KP + 2;
  static constexpr int P_DBL = STAGE_P ? K * K * KP + 2 : 0;
  static constexpr int CS_DBL = STAGE_P ? TS * 3 * K : 0;  // contrib rows, written out coalesced
  static constexpr int ROWS_DBL = 3 * TS * RS;
  static constexpr int RED_DBL = (S::LG / 2) * K3;
  static constexpr int BODY_DBL = ROWS_DBL + TS > RED_DBL ? ROWS_DBL + TS : RED_DBL;
  static constexpr int LDS_BYTES = (P_DBL + CS_DBL + BODY_DBL + 8) * 8;
  static constexpr bool FITS = LDS_BYTES <= LDS_BUDGET;
  __device__ static constexpr int slab(int a) { return a * K * KP + (a >= KH ? 2 : 0); }
};

// Phase A, LDS-staged p_r, lane h of 2 covers a in [h*KH, h*KH + KH).  On return zc / wc /
// dsum hold the FULL sums (partner partials added in a commutative, lane-symmetric order).
template <int K, int TS>
__device__ __forceinline__ double phase_a_lds(const double* __restrict__ Ps,
                                              const double* __restrict__ ri,
                                              const double* __restrict__ rj,
                                              const double* __restrict__ rk, int h,
                                              double* __restrict__ crow, double (&zc)[K],
                                              double (&wc)[K]) {
  using EP = EPlan<K, TS>;
  constexpr int KP = EP::KP, KH = EP::KH;
  constexpr int KE = K & ~1;  // even part of a row (double2 reads)
  double tj[K], tk[K];
#pragma unroll
  for (int g = 0; g < K; ++g) {
    tj[g] = rj[g];
    tk[g] = rk[g];
    zc[g] = 0.0;
    wc[g] = 0.0;
  }
  // p rows are software-pipelined: row (a, b+1) is in flight while row (a, b) is consumed.
  auto load_row = [&](double (&dst)[K], const double* __restrict__ src) {
#pragma unroll
    for (int g = 0; g < KE; g += 2) {
      const double2 v = *reinterpret_cast<const double2*>(src + g);
      dst[g] = v.x;
      dst[g + 1] = v.y;
    }
    if constexpr (K & 1) dst[K - 1] = src[K - 1];
  };
  // Two p rows per step (two independent U chains for ILP); the next pair is in flight while
  // the current one is consumed.  Odd K: the last row of a slab pairs with a zero row.
  constexpr int NPAIR = (K + 1) / 2;
  double dsum = 0.0;
  double pv0[K], pv1[K];
  auto load_pair = [&](double (&d0)[K], double (&d1)[K], const double* __restrict__ slab, int bp) {
    load_row(d0, slab + (2 * bp) * KP);
    if (2 * bp + 1 < K) {
      load_row(d1, slab + (2 * bp + 1) * KP);
    } else {
#pragma unroll
      for (int g = 0; g < K; ++g) d1[g] = 0.0;
    }
  };
  load_pair(pv0, pv1, Ps + EP::slab(h * KH < K ? h * KH : K - 1), 0);
#pragma unroll 1
  for (int q = 0; q < KH; ++q) {
    const int a = h * KH + q;
    const bool valid = a < K;
    const int ac = valid ? a : K - 1;
    const double ta = valid ? ri[ac] : 0.0;
    const double* __restrict__ pa = Ps + EP::slab(ac);
    const int an = (a + 1 < K && q + 1 < KH) ? a + 1 : ac;  // next slab (clamped)
    const double* __restrict__ pn_slab = Ps + EP::slab(an);
    double y = 0.0;
#pragma unroll
    for (int bp = 0; bp < NPAIR; ++bp) {
      const int b0 = 2 * bp, b1 = 2 * bp + 1;
      double pn0[K], pn1[K];
      if (bp + 1 < NPAIR)
        load_pair(pn0, pn1, pa, bp + 1);
      else
        load_pair(pn0, pn1, pn_slab, 0);
      double u0 = 0.0, u1 = 0.0;
#pragma unroll
      for (int g = 0; g < K; ++g) {
        u0 = fma(pv0[g], tk[g], u0);
        u1 = fma(pv1[g], tk[g], u1);
      }
      const double t0 = ta * tj[b0];
      y = fma(tj[b0], u0, y);
      zc[b0] = fma(ta, u0, zc[b0]);
      if (b1 < K) {
        const double t1 = ta * tj[b1];
        y = fma(tj[b1], u1, y);
        zc[b1] = fma(ta, u1, zc[b1]);
#pragma unroll
        for (int g = 0; g < K; ++g) wc[g] = fma(t1, pv1[g], fma(t0, pv0[g], wc[g]));
      } else {
#pragma unroll
        for (int g = 0; g < K; ++g) wc[g] = fma(t0, pv0[g], wc[g]);
      }
#pragma unroll
      for (int g = 0; g < K; ++g) {
        pv0[g] = pn0[g];
        pv1[g] = pn1[g];
      }
    }
    if (valid) crow[a] = y;
    dsum = fma(ta, y, dsum);
  }
  // partner exchange (lanes 2l, 2l+1): a + b == b + a exactly, so both lanes agree bitwise
#pragma unroll
  for (int g = 0; g < K; ++g) {
    zc[g] += __shfl_xor(zc[g], 1, 64);
    wc[g] += __shfl_xor(wc[g], 1, 64);
  }
  dsum += __shfl_xor(dsum, 1, 64);
  return dsum;
}

// ------------------------------------------------------------------------------------------
// E-step: grid (n_obs_pad / TS, B), block NT = TS*H.
// ------------------------------------------------------------------------------------------
template <int K, int TS>
__global__ __launch_bounds__((EPlan<K, TS>::NT)) void estep_kernel(
    const int4* __restrict__ obs, const int* __restrict__ tile_r, const double* __restrict__ theta,
    const double* __restrict__ pr, double* __restrict__ contrib, double* __restrict__ cvec,
    double* __restrict__ partS, double* __restrict__ partL, int P, int R, long long n_obs_pad,
    int ntiles, double eps, int ablate) {
  using EP = EPlan<K, TS>;
  using SP = typename EP::S;
  constexpr int K3 = EP::K3, KP = EP::KP, RS = EP::RS, NT = EP::NT, H = EP::H;
  constexpr int NB = SP::NB, NBC = SP::NBC, NBLK = SP::NBLK, LG = SP::LG;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* Ps = smem;
  double* Cs = smem + EP::P_DBL;
  double* Ri = Cs + EP::CS_DBL;
  double* Rj = Ri + TS * RS;
  double* Rk = Rj + TS * RS;
  double* Cv = Rk + TS * RS;
  double* scratch = Ri + EP::BODY_DBL;

  const int tid = threadIdx.x;
  const int lo = tid / H;  // observation within the tile
  const int h = tid % H;   // lane's share of the observation
  const int tile = blockIdx.x;
  const int b = blockIdx.y;
  const int r = __builtin_amdgcn_readfirstlane(tile_r[(tile * TS) / TILE]);
  const double* __restrict__ th = theta + (size_t)b * P * K;
  const double* __restrict__ p = pr + ((size_t)b * R + r) * K3;
  const size_t o = (size_t)tile * TS + lo;
  const int4 e = obs[o];
  const double n = (double)e.w;

  // ---- stage p_r and the observations' theta rows
  if constexpr (EP::STAGE_P) {
    for (int idx = tid; idx < K3; idx += NT) {
      const int a = idx / (K * K);
      Ps[EP::slab(a) + ((idx / K) % K) * KP + idx % K] = p[idx];
    }
  }
  if (h == 0) {
    const double* __restrict__ gi = th + (size_t)e.x * K;
    const double* __restrict__ gj = th + (size_t)e.y * K;
#pragma unroll
    for (int g = 0; g < K; ++g) {
      Ri[lo * RS + g] = gi[g];
      Rj[lo * RS + g] = gj[g];
    }
  }
  if (h == H - 1) {
    const double* __restrict__ gk = th + (size_t)e.z * K;
#pragma unroll
    for (int g = 0; g < K; ++g) Rk[lo * RS + g] = gk[g];
  }
  __syncthreads();

  // ---- phase A (LDS path: Y/Z/W rows staged in Cs, written out as one contiguous block)
  double* __restrict__ crow =
      EP::STAGE_P ? Cs + lo * 3 * K : contrib + ((size_t)b * n_obs_pad + o) * 3 * K;
  double dsum = 1.0;
  // ablate (measurement builds only, MMSBM_ABLATE): bit 0 skips phase A, bit 1 phase B
  if (!(ablate & 1)) {
    if constexpr (EP::STAGE_P) {
      double zc[K], wc[K];
      dsum = phase_a_lds<K, TS>(Ps, Ri + lo * RS, Rj + lo * RS, Rk + lo * RS, h, crow, zc, wc);
      if (h == 0) {
#pragma unroll
        for (int g = 0; g < K; ++g) crow[K + g] = zc[g];
      } else {
#pragma unroll
        for (int g = 0; g < K; ++g) crow[2 * K + g] = wc[g];
      }
    } else {
      dsum = phase_a<K>(th, p, e, crow);
    }
  }
  const double d = dsum + eps;
  const double c = n / d;
  if (h == 0) {
    cvec[(size_t)b * n_obs_pad + o] = c;
    Cv[lo] = c;
  }
  const double ll = block_sum(h == 0 ? n * log(d) : 0.0, scratch);  // barrier for phase B
  if (tid == 0) partL[(size_t)b * ntiles + tile] = ll;
  if constexpr (EP::STAGE_P) {
    // the tile's TS contrib rows are one contiguous block: coalesced 16-B stores
    double2* __restrict__ dst =
        reinterpret_cast<double2*>(contrib + ((size_t)b * n_obs_pad + (size_t)tile * TS) * 3 * K);
    const double2* src = reinterpret_cast<const double2*>(Cs);
    if (!(ablate & 4))
      for (int idx = tid; idx < TS * 3 * K / 2; idx += NT) dst[idx] = src[idx];
  }

  // ---- phase B: S_r[a b g] = sum_l c_l th_i[a] th_j[b] th_k[g] over this tile
  double* __restrict__ sdst = partS + ((size_t)b * ntiles + tile) * K3;
  for (int set = 0; set < ((ablate & 2) ? 0 : SP::NSETS); ++set) {
    int blk, grp;
    if constexpr (SP::NSETS == 1) {
      blk = tid % NBLK;
      grp = tid / NBLK;
    } else {
      blk = set * NT + tid;
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
    if (active) {
#pragma unroll 2
      for (int l = grp; l < TS; l += LG) {
        const double av = Cv[l] * Ri[l * RS + alpha];
        double gv[K];
#pragma unroll
        for (int g = 0; g < (K & ~1); g += 2) {
          const double2 v = *reinterpret_cast<const double2*>(Rk + l * RS + g);
          gv[g] = v.x;
          gv[g + 1] = v.y;
        }
        if constexpr (K & 1) gv[K - 1] = Rk[l * RS + K - 1];
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          if (NB * NBC == K || beta0 + q < K) {
            const double ab = av * Rj[l * RS + beta0 + q];
#pragma unroll
            for (int g = 0; g < K; ++g) acc[q][g] = fma(ab, gv[g], acc[q][g]);
          }
        }
      }
    }
    if constexpr (LG > 1) {
      double* red = Ri;  // rows are dead once every group has accumulated
      int ng = LG;
      while (ng > 1) {
        const int half = (ng + 1) / 2;
        __syncthreads();
        if (active && grp >= half && grp < ng) {
          double* dst = red + (size_t)(grp - half) * K3 + (alpha * K + beta0) * K;
#pragma unroll
          for (int q = 0; q < NB; ++q)
            if (NB * NBC == K || beta0 + q < K)
#pragma unroll
              for (int g = 0; g < K; ++g) dst[q * K + g] = acc[q][g];
        }
        __syncthreads();
        if (active && grp < ng - half) {
          const double* src = red + (size_t)grp * K3 + (alpha * K + beta0) * K;
#pragma unroll
          for (int q = 0; q < NB; ++q)
            if (NB * NBC == K || beta0 + q < K)
#pragma unroll
              for (int g = 0; g < K; ++g) acc[q][g] += src[q * K + g];
        }
        ng = half;
      }
    }
    if (active && grp == 0) {
      double* dst = sdst + (alpha * K + beta0) * K;
#pragma unroll
      for (int q = 0; q < NB; ++q)
        if (NB * NBC == K || beta0 + q < K)
#pragma unroll
          for (int g = 0; g < K; ++g) dst[q * K + g] = acc[q][g];
    }
  }
}

struct Segs {
  int t[MAX_R + 1];  // tile offsets of each rating group
};

constexpr int MP_CELLS = 4;   // p M-step: cells per block
constexpr int MP_PARTS = 64;  // p M-step: tile stripes per cell
constexpr int MT_BATCH = 4;   // theta M-step: incidences in flight per lane

// ------------------------------------------------------------------------------------------
// Fused M-step, grid (theta_blocks + ceil(K3 / MP_CELLS), B), block 256.
//  blocks [0, theta_blocks): theta (:1016-1018), one wave per gene:
//      theta[g][a] <- theta[g][a] * (sum over the gene's incidences of c * row[a]) / deg[g]
//    lanes stride the incidence list MT_BATCH entries at a time (all loads of a batch in
//    flight together), each keeps K partial sums, then a fixed butterfly.
//  blocks [theta_blocks, ...): p (:1021-1028), MP_CELLS cells x MP_PARTS tile stripes:
//      S_r = sum of the per-tile partials of rating r; npr_r = p_r S_r;
//      p_r <- npr_r / (eps + sum_r npr_r).
// Both halves read only E-step outputs and write disjoint parameters, so they share a launch.
// Every sum has a fixed order (bitwise reproducible).
// ------------------------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__(256) void mstep_kernel(
    double* __restrict__ theta, double* __restrict__ pr, const double* __restrict__ contrib,
    const double* __restrict__ cvec, const int* __restrict__ gptr, const int* __restrict__ ginc,
    const int* __restrict__ deg, const double* __restrict__ partS, Segs segs, int P, int R,
    int ntiles, long long n_obs_pad, int theta_blocks, double eps) {
  constexpr int K3 = K * K * K;
  const int b = blockIdx.y;
  if ((int)blockIdx.x < theta_blocks) {
    const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (g >= P) return;  // wave-uniform
    const double* __restrict__ cb = contrib + (size_t)b * n_obs_pad * 3 * K;
    const double* __restrict__ cv = cvec + (size_t)b * n_obs_pad;
    double acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0.0;
    const int q0 = gptr[g], q1 = gptr[g + 1];
    for (int qb = q0; qb < q1; qb += 64 * MT_BATCH) {
      int inc[MT_BATCH];
#pragma unroll
      for (int j = 0; j < MT_BATCH; ++j) {
        const int q = qb + j * 64 + lane;
        inc[j] = q < q1 ? ginc[q] : -1;
      }
      double cc[MT_BATCH], row[MT_BATCH][K];
#pragma unroll
      for (int j = 0; j < MT_BATCH; ++j) {
        const int ij = inc[j] < 0 ? 0 : inc[j];
        cc[j] = inc[j] < 0 ? 0.0 : cv[ij / 3];
        const double* __restrict__ src = cb + (size_t)ij * K;
#pragma unroll
        for (int k = 0; k < K; ++k) row[j][k] = src[k];
      }
#pragma unroll
      for (int j = 0; j < MT_BATCH; ++j)
#pragma unroll
        for (int k = 0; k < K; ++k) acc[k] = fma(cc[j], row[j][k], acc[k]);
    }
    double mine = 0.0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const double t = wave_sum(acc[k]);
      if (lane == k) mine = t;
    }
    if (lane < K) {
      double* th = theta + (size_t)b * P * K + (size_t)g * K;
      th[lane] = th[lane] * mine / (double)deg[g];
    }
    return;
  }
  __shared__ double red[MP_PARTS][MP_CELLS];
  const int cl = threadIdx.x % MP_CELLS;
  const int part = threadIdx.x / MP_CELLS;
  const int cell = ((int)blockIdx.x - theta_blocks) * MP_CELLS + cl;
  const double* __restrict__ ps = partS + (size_t)b * ntiles * K3 + cell;
  double S[MAX_R];
  for (int r = 0; r < R; ++r) {
    double s = 0.0;
    if (cell < K3) {
      const int end = segs.t[r + 1];
      int t = segs.t[r] + part;
      for (; t + 3 * MP_PARTS < end; t += 4 * MP_PARTS) {
        const double a0 = ps[(size_t)t * K3], a1 = ps[(size_t)(t + MP_PARTS) * K3];
        const double a2 = ps[(size_t)(t + 2 * MP_PARTS) * K3], a3 = ps[(size_t)(t + 3 * MP_PARTS) * K3];
        s += (a0 + a1) + (a2 + a3);
      }
      for (; t < end; t += MP_PARTS) s += ps[(size_t)t * K3];
    }
    red[part][cl] = s;
    __syncthreads();
    double tot = 0.0;
    if (part == 0)
      for (int q = 0; q < MP_PARTS; ++q) tot += red[q][cl];
    S[r] = tot;
    __syncthreads();
  }
  if (part == 0 && cell < K3) {
    double* pc = pr + (size_t)b * R * K3;
    double npr[MAX_R];
    double den = eps;
    for (int r = 0; r < R; ++r) {
      npr[r] = pc[(size_t)r * K3 + cell] * S[r];
      den += npr[r];
    }
    for (int r = 0; r < R; ++r) pc[(size_t)r * K3 + cell] = npr[r] / den;
  }
}

// ------------------------------------------------------------------------------------------
// Log-likelihood tile partials (:958-969): grid (ntiles, B), block TILE.
// ------------------------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__(TILE) void loglik_kernel(const int4* __restrict__ obs,
                                                      const int* __restrict__ tile_r,
                                                      const double* __restrict__ theta,
                                                      const double* __restrict__ pr,
                                                      double* __restrict__ partL, int P, int R,
                                                      int ntiles, double eps) {
  __shared__ double scratch[TILE / 64];
  constexpr int K3 = K * K * K;
  const int tile = blockIdx.x;
  const int b = blockIdx.y;
  const int r = __builtin_amdgcn_readfirstlane(tile_r[tile]);
  const double* __restrict__ th = theta + (size_t)b * P * K;
  const double* __restrict__ p = pr + ((size_t)b * R + r) * K3;
  const int4 e = obs[(size_t)tile * TILE + threadIdx.x];
  const double d = contract<K>(th, p, e.x, e.y, e.z) + eps;
  const double ll = block_sum((double)e.w * log(d), scratch);
  if (threadIdx.x == 0) partL[(size_t)b * ntiles + tile] = ll;
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
  int (*estep)(mmsbm_ctx*, const double*, const double*, hipStream_t);
  int (*mstep)(mmsbm_ctx*, hipStream_t);
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
  // current iterate (only valid during a call)
  double* theta_mut = nullptr;
  double* pr_mut = nullptr;
  // optional per-kernel timing: HIP event pairs recorded around each launch on its stream
  bool timing = false;
  int ablate = 0;  // MMSBM_ABLATE (measurement only)
  int ts = 64;     // E-step tile (observations per workgroup): MMSBM_ESTEP_TILE = 64/128/256
  std::vector<hipEvent_t> ev[2];  // start/stop pairs per kernel id
  size_t nev[2] = {0, 0};
};

namespace {

struct WsLayout {
  size_t contrib, cvec, partS, partL, total;
};

WsLayout ws_layout(const mmsbm_ctx* c) {
  WsLayout L{};
  const LinkSet& tr = c->sets[MMSBM_SET_TRAIN];
  const LinkSet& te = c->sets[MMSBM_SET_TEST];
  const size_t K3 = (size_t)c->K * c->K * c->K;
  size_t off = 0;
  L.contrib = off;
  off += align_up((size_t)c->B * tr.n_obs_pad * 3 * c->K * sizeof(double));
  L.cvec = off;
  off += align_up((size_t)c->B * tr.n_obs_pad * sizeof(double));
  L.partS = off;  // one row per E-step tile; sized for the smallest tile (MIN_TS)
  const long long et = tr.n_obs_pad / MIN_TS;
  off += align_up((size_t)c->B * et * K3 * sizeof(double));
  L.partL = off;
  long long nt = et > te.ntiles ? et : te.ntiles;
  off += align_up((size_t)c->B * (nt > 0 ? nt : 1) * sizeof(double));
  L.total = off;
  return L;
}

// E-step tile actually used for a requested one: the largest that fits the LDS plan.
template <int K>
int estep_tile(int requested) {
  if (requested >= 256 && EPlan<K, 256>::FITS) return 256;
  if (requested >= 128 && EPlan<K, 128>::FITS) return 128;
  return 64;
}

template <int K, int TS>
int launch_estep_ts(mmsbm_ctx* c, hipStream_t s) {
  using T = EPlan<K, TS>;
  static_assert(T::FITS, "E-step LDS plan over budget");
  const LinkSet& tr = c->sets[MMSBM_SET_TRAIN];
  const int et = (int)(tr.n_obs_pad / TS);
  estep_kernel<K, TS><<<dim3(et, c->B), T::NT, T::LDS_BYTES, s>>>(
      tr.obs, tr.tile_r, c->theta_mut, c->pr_mut, c->contrib, c->cvec, c->partS, c->partL, c->P,
      c->R, tr.n_obs_pad, et, c->eps, c->ablate);
  HIP_TRY(hipGetLastError());
  return MMSBM_OK;
}

template <int K>
int launch_estep(mmsbm_ctx* c, const double*, const double*, hipStream_t s) {
  const LinkSet& tr = c->sets[MMSBM_SET_TRAIN];
  if (tr.ntiles == 0) return MMSBM_OK;
  switch (estep_tile<K>(c->ts)) {
    case 256:
      if constexpr (EPlan<K, 256>::FITS) return launch_estep_ts<K, 256>(c, s);
      break;
    case 128:
      if constexpr (EPlan<K, 128>::FITS) return launch_estep_ts<K, 128>(c, s);
      break;
    default:
      break;
  }
  return launch_estep_ts<K, 64>(c, s);
}

template <int K>
int launch_mstep(mmsbm_ctx* c, hipStream_t s) {
  constexpr int K3 = K * K * K;
  const LinkSet& tr = c->sets[MMSBM_SET_TRAIN];
  const int ts = estep_tile<K>(c->ts);
  Segs segs{};  // rating groups in units of E-step tiles
  for (int r = 0; r <= c->R; ++r) segs.t[r] = (int)(tr.seg.empty() ? 0 : tr.seg[r] / ts);
  const int theta_blocks = (c->P + 3) / 4;
  const int p_blocks = (K3 + MP_CELLS - 1) / MP_CELLS;
  mstep_kernel<K><<<dim3(theta_blocks + p_blocks, c->B), 256, 0, s>>>(
      c->theta_mut, c->pr_mut, c->contrib, c->cvec, c->gptr, c->ginc, c->deg, c->partS, segs,
      c->P, c->R, (int)(tr.n_obs_pad / ts), tr.n_obs_pad, theta_blocks, c->eps);
  HIP_TRY(hipGetLastError());
  return MMSBM_OK;
}

template <int K>
int launch_loglik(mmsbm_ctx* c, int which, const double* theta, const double* pr, hipStream_t s) {
  const LinkSet& ls = c->sets[which];
  if (ls.ntiles == 0) return MMSBM_OK;
  loglik_kernel<K><<<dim3(ls.ntiles, c->B), TILE, 0, s>>>(ls.obs, ls.tile_r, theta, pr, c->partL,
                                                         c->P, c->R, ls.ntiles, c->eps);
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
      Launch{&launch_estep<Ks + 1>, &launch_mstep<Ks + 1>, &launch_loglik<Ks + 1>, &launch_predict<Ks + 1>}...};
}

const auto kTable = make_table(std::make_integer_sequence<int, MMSBM_MAX_K>{});

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
  if (const char* t = getenv("MMSBM_ESTEP_TILE")) {
    const int v = atoi(t);
    if (v == 64 || v == 128 || v == 256) c->ts = v;
  }
  *out = c;
  return MMSBM_OK;
}

int mmsbm_destroy(mmsbm_ctx* c) {
  if (!c) return MMSBM_OK;
  (void)hipSetDevice(c->device);
  for (auto& s : c->sets)
    if (s.tile_r) (void)hipFree(s.tile_r);
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
  for (int it = 0; it < n_iters; ++it) {
    if ((rc = timing_mark(c, 0, s))) return rc;
    if ((rc = L.estep(c, theta, pr, s))) return rc;
    if ((rc = timing_mark(c, 0, s))) return rc;
    if ((rc = timing_mark(c, 1, s))) return rc;
    if ((rc = L.mstep(c, s))) return rc;
    if ((rc = timing_mark(c, 1, s))) return rc;
  }
  return MMSBM_OK;
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
  reduce_kernel<<<c->B, 256, 0, s>>>(c->partL, ls.ntiles, out);
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

int mmsbm_timing(mmsbm_ctx* c, int32_t enable) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  c->timing = enable != 0;
  for (auto& n : c->nev) n = 0;
  return MMSBM_OK;
}

int mmsbm_timing_result(mmsbm_ctx* c, int32_t kernel, double* total_ms, int64_t* count) {
  if (!c || !total_ms || !count) return fail(MMSBM_ERR_INVALID, "null argument");
  if (kernel < 0 || kernel > 1) return fail(MMSBM_ERR_INVALID, "kernel id %d", kernel);
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
