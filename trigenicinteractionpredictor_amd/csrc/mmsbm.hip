// mmsbm.hip — MI355X (gfx950) MMSBM EM engine: kernels + C ABI (include/mmsbm.h).
//
// Hot path of AleixMT/TrigenicInteractionPredictor, src/TrigenicInteractionPredictor.py:
//   make_iteration      :984-1043   -> K <= 12 (sk.h): sk_pass_kernel<K, SK_U> (or sky_pass_kernel<K>)
//                                      + sk_fin_kernel<K>; K > 12: pass_kernel<K, PASS_A>,
//                                      gm_kernel<K>, upd_kernel<K>
//   compute_likelihood  :952-974    -> sk_pass_kernel<K, SK_LL> / pass_kernel<K, PASS_LL> + reduce_kernel
//   do_prediction       :530-547    -> predict_kernel<K>
//
// Pivot-run factorisation.  The reference spends K^3 work per observed (link, rating):
//   T[a][b][h] = th_i[a] th_j[b] th_k[h] p_r[a][b][h],  d = eps + sum T,  c = n / d,
//   ntheta[i] += c sum_bh T,  ntheta[j] += c sum_ah T,  ntheta[k] += c sum_ab T,  npr += c T.
// Grouping the same sums by gene moves every K^3 term from the observation to the gene.  Order the
// observations of rating r by their slot-s gene g (the pivot, s = 0, 1, 2) and let u, v be the two
// other slots:
//   V_g[b][h]   = sum_a th_g[a] p_r[a][b][h]                         per gene (stream 0 only)
//   Z_o[b]      = sum_h V_g[b][h] th_k(o)[h],  d_o = eps + sum_b th_j(o)[b] Z_o[b],  c_o = n_o / d_o
//   M^s_g[x][y] = sum_{o with pivot g} c_o th_u(o)[x] th_v(o)[y]      K^2 per observation
// and per gene (the update kernels):
//   X^0_g[a] = sum_bh p[a][b][h] M^0_g[b][h],  X^1_g[b] = sum_ah p M^1_g[a][h],  X^2_g[h] = sum_ab p M^2_g[a][b]
//   theta'_g = theta_g (sum_r X^0 + X^1 + X^2) / deg_g                          (:1009-1018)
//   S_r = sum_g theta_g (x) M^0_g,  p' = p S / (eps + sum_r p S)               (:1012, :1021-1028)
// (tests/pivot_model.py restates this in numpy and checks it against the C oracle.)
//
// Per observation the GPU does K^2 work (Z, and M for each of the three slots) on FP64 MFMA
// (v_mfma_f64_4x4x4f64 / 16x16x4f64); the K^3 work is per pivot gene.  A large-K iteration is three
// launches:
//   PASS_A  stream 0 (pivot = slot 0): V in LDS per workgroup, then per 4-observation chunk Z, Z',
//           d, c; the j / k slots' sums as Y entries c Z, c Z'; M^0 flushed as a partial row per
//           gene stretch
//   gm      X rows (M^0 p) and S partials (theta (x) M^0) in one pass over the partial rows
//   upd     per gene: X rows + Y entries summed in a fixed order, theta'; per cell: S summed, p'
// The small-K family (sk.h) fuses the E-step into one launch per iteration plus its update.
// Every sum has a fixed order: results are bitwise reproducible run to run.

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
#include "mmsbm_pairs.h"
#include "plan.h"

namespace {

using mmsbm_plan::CH;
using mmsbm_plan::NW;
constexpr int MAX_R = 8;
constexpr int NT = 64 * NW;     // pass workgroup: one unit per wave
constexpr int FIN_NT = 256;

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
// Compile-time shape of one K.
// ------------------------------------------------------------------------------------------
// Pass-A LDS budget (V tables of GMAX genes + the wave images): two workgroups per CU at every K.
// Measured (tools/gpu_r02c_gcap.sh): a 150 KB budget (one workgroup per CU, GMAX 22 at K = 20,
// 13 at K = 30) ran pass A at 156 us (K = 20 x 8) and 2088 us (K = 30, 10M links); 78 KB
// (GMAX 9 / 4) at 125 us and 1794 us.
// From K = MMSBM_LDS_BIG up the pass kernel takes more than 128 VGPRs (130-140 at K = 25-32), so it
// runs one workgroup per CU whatever its LDS: there the budget is 150 KB (GMAX 13 at K = 30 instead
// of 5; pass A 2,761 -> 2,531 us at K=30 on 10M links, profiles/r04s_large_ab.txt)
#ifndef MMSBM_LDS_BIG
#define MMSBM_LDS_BIG 25
#endif
// Waves per pass workgroup from K = MMSBM_LDS_BIG (MMSBM_PNW; below LDS_BIG always NW = 8) and
// the V operands in registers (MMSBM_VREG, pass_kernel).  Measured at K=30 on 10M links, one box
// (profiles/r05_vreg_ab.txt): 8-wave workgroups with V in registers (~245 VGPRs, one workgroup per
// CU) are fastest; 4-wave workgroups (MMSBM_PNW=4: 52 KB, three per CU at <= 168 VGPRs with U=4 /
// DT=1, profiles/r05_pnw4_ab.txt) beat 8-wave ones only while V is read from LDS, and with V in
// registers (two per CU) they lose.
#ifndef MMSBM_PNW
#define MMSBM_PNW 8
#endif
#ifndef MMSBM_VREG
#define MMSBM_VREG 1
#endif
#ifndef MMSBM_ZSPLIT
#define MMSBM_ZSPLIT 1
#endif
#ifndef MMSBM_VREG_MIN
#define MMSBM_VREG_MIN MMSBM_LDS_BIG
#endif
#ifndef MMSBM_PNW_U
#define MMSBM_PNW_U 4
#endif
#ifndef MMSBM_PNW_DT
#define MMSBM_PNW_DT 1
#endif
#ifndef MMSBM_PNW_WPE
#define MMSBM_PNW_WPE 3
#endif
#ifndef MMSBM_LDS_BIGKB
#define MMSBM_LDS_BIGKB (MMSBM_PNW == 8 ? 150 : 52)
#endif
constexpr int pnw_for(int K) { return K >= MMSBM_LDS_BIG ? MMSBM_PNW : NW; }
constexpr int lds_target(int K) {
  return K >= MMSBM_LDS_BIG ? MMSBM_LDS_BIGKB * 1024 : K <= 16 ? 76 * 1024 : 78 * 1024;
}

// Pass-A ablations for measurement builds only (results invalid): 1 = no Y stores, 2 = theta
// gathers from 64 hot rows (L2 hits), 4 = no partial-row stores
#ifndef MMSBM_ABL
#define MMSBM_ABL 0
#endif

// Large-K Y entries: row stride K rounded up to MMSBM_YALIGN doubles (4 = one 32-B sector), so no
// entry starts inside a sector another entry also writes (the pad words hold zeros or never-read
// values).  K=30 on 10M links: pass A 3,695 us at stride 30, 3,402 at 32; K=20 x 8 (already
// sector-aligned at 20): 139.8 us at 20, 152.5 at 24 and 197.0 at 32, the pad being pure extra
// bytes there (profiles/r04p_large_ab.txt).
#ifndef MMSBM_YALIGN
#define MMSBM_YALIGN 4
#endif
constexpr int y_stride(int K) { return (K + MMSBM_YALIGN - 1) / MMSBM_YALIGN * MMSBM_YALIGN; }
// Y entry stores (pass A) and loads (upd) plain or non-temporal: bit 1 stores, bit 2 loads.
// Non-temporal loads in upd: K=30 on 10M links upd 895 -> 807 us (the 5.1 GB stream no longer
// displaces the L2's theta / X-row lines); non-temporal stores in pass A within noise, and
// non-temporal loads of the small-K SK_Y entries (92 MB, just written, on die) slower (fin 19.5 ->
// 21.8 us at K=10 x 8): profiles/r06p_fin_ynt_ab.txt, r06q_fin_butterfly_ab.txt
#ifndef MMSBM_YNT
#define MMSBM_YNT 2
#endif
__device__ __forceinline__ void y_st(double* p, double v) {
  if constexpr (MMSBM_YNT & 1) __builtin_nontemporal_store(v, p);
  else *p = v;
}
typedef double yd2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ yd2 y_ld2(const yd2* p) {
  if constexpr (MMSBM_YNT & 2) return __builtin_nontemporal_load(p);
  else return *p;
}

// Pass-kernel occupancy hint: 1 leaves the compiler free (K = 25-32 take 132-134 VGPRs, so one
// 8-wave workgroup per CU although the LDS would fit two); 4 caps it at 128 VGPRs (4 waves per
// SIMD) at the price of 3-21 spilled VGPRs: K=30 pass A 3,402 us capped vs 3,306 free
// (profiles/r04p_large_ab.txt), so the default stays free.
#ifndef MMSBM_PASS_WPE
#define MMSBM_PASS_WPE 1
#endif
constexpr int PASS_WPE = MMSBM_PASS_WPE;

// Row strides of pass A's V tables and of their genes' theta rows: odd (1) or the round-3 even
// strides (0, measurement).  The compiler pairs the chunk loop's V reads into ds_read2_b64, whose
// 16-lane groups bank on (a/4) mod 32: an odd stride puts the 16 rows of a Z read (b = 4 blk + lo)
// on distinct banks, and the 4 theta rows of a V-prologue read (4 t + lo) likewise; the Z' reads
// walk one row and stay conflict-free at any stride.
#ifndef MMSBM_VR_ODD
#define MMSBM_VR_ODD 1
#endif

template <int K>
struct KT {
  static constexpr int NG = (K + 3) / 4;          // 4-wide tiles of one K axis
  static constexpr int KP = 4 * NG;
  static constexpr int K2 = K * K, K3 = K * K * K;
  static constexpr int NBG = (NG + 3) / 4;        // Z phase: groups of 4 b-tiles (one per block)
  static constexpr int VROWS = 16 * NBG;          // V image rows (b); zero from K on
  static constexpr int VR = MMSBM_VR_ODD ? KP + 1 : KP + 2;  // V row stride (above)
  static constexpr int VDBL = VROWS * VR;         // one gene's V image
  static constexpr int TGR = MMSBM_VR_ODD ? KP + 1 : KP;     // theta row stride of the V genes
  // doubles of g genes' theta rows, even so the wave images after them stay 16-byte aligned
  static constexpr int tg_dbl(int g) { return (g * TGR + 1) & ~1; }
  static constexpr int TR = KP + 2;               // theta image row stride
  static constexpr int IMG = 8 * TR;              // one chunk: th_u rows of obs 0-3, th_v rows
  static constexpr int SW = (K % 2 == 0) ? 2 : 1;  // staging width: double2 pieces when K is even
  static constexpr int NPC = (8 * KP / SW + 63) / 64;  // staged pieces per lane per chunk
  static constexpr int IMGW = 2 * IMG + 2;        // per wave: double buffer + a dummy piece slot
  static constexpr int NWK = pnw_for(K), NTK = 64 * NWK;  // pass_kernel's waves / threads
  // occupancy hint: 4-wave workgroups three per CU (<= 168 VGPRs), else PASS_WPE
  static constexpr int WPE = NWK == 4 ? MMSBM_PNW_WPE : PASS_WPE;
  static constexpr int IMG_BYTES = NWK * IMGW * 8;
  static constexpr int GMAX_RAW = (lds_target(K) - IMG_BYTES - 64 - 8) / ((VDBL + TGR) * 8);
  static constexpr int GMAX = GMAX_RAW > 64 ? 64 : (GMAX_RAW < 4 ? 4 : GMAX_RAW);
  static constexpr int LDS_A = GMAX * VDBL * 8 + tg_dbl(GMAX) * 8 + IMG_BYTES + 64;
  static constexpr int LDS_B = IMG_BYTES + 64;
  // S partials: (a-tile, group of 4 cell tiles) items over the 8 waves
  static constexpr int NCT = (K2 + 3) / 4;
  static constexpr int NCG = (NCT + 3) / 4;
  static_assert(LDS_A <= 160 * 1024, "pass A LDS over budget");
  static_assert(64 * KP * 8 <= IMG_BYTES, "S partial staging over the pass B LDS");
};

int gmax_for(int K);  // host view of KT<K>::GMAX (table below)
int pnw_host(int K) { return pnw_for(K); }

__device__ __forceinline__ double mfma4(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

// v_mfma_f64_16x16x4_f64: lane l holds A[l & 15][l >> 4], B[l >> 4][l & 15]; D[(l >> 4) + 4 i][l & 15]
// in element i (MI355X guide: the f64 C/D map differs from the f32 one)
typedef double d4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ d4v mfma16(double a, double b, d4v c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// Stores of the large-K intermediates (partial rows, S partials): plain (0), or written through
// the XCD L2 (1: agent-scope relaxed atomic store = global_store sc1, so their bytes leave L2
// while the kernel runs instead of at the kernel boundary).  Write-through won 2-3 % at fold0 in
// round 2, when the large-K kernels ran the headline with c and the S partials among these
// stores; since round 4 (stream 0 + Y entries) it costs: pass A 3,402 -> 2,776 us at K=30 on 10M
// links and 152.5 -> 128.3 us at K=20 x 8 with plain stores (profiles/r04p_large_ab.txt), a
// partial row's K x K words being written as scattered 4 x 16-word pieces.
#ifndef MMSBM_WT
#define MMSBM_WT 0
#endif
__device__ __forceinline__ void st_wt(double* p, double v) {
  if constexpr (MMSBM_WT) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) v += __shfl_xor(v, s, 64);
  return v;
}

// LDS writes of this wave visible to its own later reads (the fence only keeps the compiler from
// reordering; a wave's LDS operations execute in order).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Measurement builds only (-DMMSBM_STAMP=1, then MMSBM_STAMP=1 at run time): every wave records
// s_memtime at its phase boundaries; mmsbm_iterate prints per-kernel phase averages.  The
// product build compiles all of it out.
#ifndef MMSBM_STAMP
#define MMSBM_STAMP 0
#endif
__device__ unsigned long long* g_stamp = nullptr;
constexpr int STAMP_SLOTS = 10;  // 0-7 s_memtime phase marks; 8, 9 s_memrealtime (100 MHz, chip-wide) at 0 and 7
constexpr long long STAMP_WAVES = 1 << 16;  // per kernel id
struct Stamp {
  unsigned long long t[STAMP_SLOTS];
  __device__ __forceinline__ void mark(int i) {
    if constexpr (MMSBM_STAMP) {
      t[i] = __builtin_amdgcn_s_memtime();
      if (i == 0) t[8] = __builtin_amdgcn_s_memrealtime();
      if (i == 7) t[9] = __builtin_amdgcn_s_memrealtime();
    }
  }
  __device__ __forceinline__ void flush(int kid, long long wave, int lane) {
    if constexpr (MMSBM_STAMP) {
      if (g_stamp && lane == 0 && wave < STAMP_WAVES)
        for (int i = 0; i < STAMP_SLOTS; ++i) g_stamp[((long long)kid * STAMP_WAVES + wave) * STAMP_SLOTS + i] = t[i];
    }
  }
};

// v of another lane of the same 16-lane row, by DPP (no LDS round trip): CTRL 0xB1 / 0x4E swap
// neighbours / pairs of a quad, 0x141 mirrors each half-row, 0x140 mirrors the row.
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
  const long long x = __double_as_longlong(v);
  const int l = __builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, false);
  const int h = __builtin_amdgcn_mov_dpp((int)(x >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)h << 32) | (unsigned int)l);
}

// Sum over the 16 lanes of a row; every lane gets the same bits (each step adds a lane pair
// that is symmetric under the step's permutation).
// n / d by v_rcp_f64 and two Newton steps plus a residual correction (within an ulp or two of the
// IEEE quotient; d > 0 here): 8 FP64 instructions instead of the IEEE division's 11 (scale / fixup
// sequence), in the chunk loops of sk.h and (MMSBM_PDIV, round 5) pass_kernel.  Deterministic, so
// results stay bitwise reproducible.
__device__ __forceinline__ double sk_div(double n, double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = fma(fma(-d, r, 1.0), r, r);
  r = fma(fma(-d, r, 1.0), r, r);
  const double q = n * r;
  return fma(fma(-d, q, n), r, q);
}

#ifndef MMSBM_PDIV
#define MMSBM_PDIV 1
#endif

__device__ __forceinline__ double row16_sum(double v) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  v += dpp<0x141>(v);
  v += dpp<0x140>(v);
  return v;
}

enum { PASS_A = 0, PASS_LL = 1, PASS_B = 2 };  // (PASS_B: the small-K family's stream-1/2 pass)

// ------------------------------------------------------------------------------------------
// Pass kernel, grid (workgroups, B), block 512 = one unit (contiguous chunks) per wave; stream 0
// only (the plan's large-K layout, plan.h).  MODE PASS_A: the EM E-step; PASS_LL: the likelihood.
// MFMA lane map (v_mfma_f64_4x4x4f64, lane = 16 hi + 4 blk + lo): A[blk][m = lo][k = hi],
// B[blk][k = hi][n = lo], D[blk][m = hi][n = lo] (tools/micro/mfma_layout.hip).
//   Z   (blocks = b tiles, k = h):  A = th_v[obs lo][4 hs + hi], B = V_g[b][4 hs + hi]  -> Z[obs hi][b]
//   Z'  (blocks = h tiles, k = b):  A = th_u[obs lo][4 bs + hi], B = V_g[4 bs + hi][h] -> Z'[obs hi][h]
//   M   (v_mfma_f64_16x16x4, k = the chunk's 4 observations): M[x][y] += c th_u[x] th_v[y]
// Per observation (u = j, v = k; src/TrigenicInteractionPredictor.py:996-1012):
//   d = eps + th_j . Z,  c = n / d,  Y[entry j] = c Z  (= ntheta_j / th_j),  Y[entry k] = c Z'
// and per gene stretch the M^0 partial row (K^2) for X^0 and S (gene_kernel).
// ------------------------------------------------------------------------------------------
template <int K, int MODE>
__global__ __launch_bounds__(KT<K>::NTK) __attribute__((amdgpu_waves_per_eu(KT<K>::WPE))) void pass_kernel(
    const int4* __restrict__ rows, const int* __restrict__ chunk_prow,
    const int* __restrict__ chunk_vslot, const int* __restrict__ row_y, const int* __restrict__ wg_units,
    const int* __restrict__ wg_code, const int* __restrict__ wg_gene, const int* __restrict__ vgenes,
    const double* __restrict__ theta, const double* __restrict__ pr, double* __restrict__ ybuf,
    double* __restrict__ prows, double* __restrict__ partL, int P, int R, long long n_y,
    long long n_prows, int n_wg, double eps, int gcap, int merge) {
  using T = KT<K>;
  constexpr int NG = T::NG, TR = T::TR, VR = T::VR;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 4, blk = (lane >> 2) & 3, lo = lane & 3;
  const int w = blockIdx.x, b = blockIdx.y;
  const double* __restrict__ th = theta + (size_t)b * P * K;
  Stamp st_{};
  st_.mark(0);
  const long long wave_id = ((long long)b * gridDim.x + w) * T::NWK + wv;

  const int code = wg_code[w];
  const int r = code & 15;
  const double* __restrict__ p = pr + ((size_t)b * R + r) * T::K3;
  double* Vt = smem;
  // LDS: [gcap V tables][gcap theta rows][per-wave images]; gcap (<= GMAX) = the plan's most
  // genes per workgroup
  double* Tg = smem + gcap * T::VDBL;  // theta rows of the V genes
  double* img = smem + gcap * T::VDBL + T::tg_dbl(gcap) + wv * T::IMGW;

  // this wave's unit, and the first records of its pipeline (in flight during the V prologue).
  // Record stream: lane l < 16 holds int l of the chunk's 4 records (i, j, k, w), lane 16 the
  // chunk's partial row, lane 17 its V slot, lanes 18-25 the 4 rows' Y entries (slot 1, slot 2);
  // the other lanes read them by readlane / shuffle, so no register array is indexed at run time.
  // Ring of U record registers: the loop below is unrolled U times so each ring slot keeps a
  // fixed register (a rotation by register moves would wait for every load in flight).
  constexpr int U = T::NWK == 4 ? MMSBM_PNW_U : 6;  // records U - 1 chunks ahead
  constexpr int DT = T::NWK == 4 ? MMSBM_PNW_DT : 2;  // theta values DT chunks ahead (ring of U slots, DT + 1 live)
  constexpr bool EM = MODE == PASS_A;
  const int c0 = wg_units[w * (T::NWK + 1) + wv], c1 = wg_units[w * (T::NWK + 1) + wv + 1];
  const int* __restrict__ rows_i = reinterpret_cast<const int*>(rows);
  // Every load in the chunk loop is issued by every lane on every path (addresses clamped, values
  // selected afterwards): an exec-masked load behind a branch would make the compiler's vmcnt
  // accounting assume it may be missing and wait for everything in flight.
  const int lr = lane & 31;  // this lane's record word: base and stride fixed once
  const bool ylane = EM && lr >= 18 && lr < 26;
  const int* __restrict__ rbase = lr < 16 ? rows_i + lr : lr == 16 ? chunk_prow : lr == 17 ? chunk_vslot
                                  : ylane ? row_y + (lr - 18) : rows_i;
  const int rstride = lr < 16 ? 16 : lr < 18 ? 1 : ylane ? 2 * CH : 16;
  auto ld_rec = [&](int q) -> int { return rbase[(size_t)q * rstride]; };
  auto clampq = [&](int q) { return q < c1 ? q : c1 - 1; };
  const bool any = c0 < c1;
  // Merged partial rows (Plan::merge, K >= MMSBM_LDS_BIG, where one workgroup runs per CU and the
  // registers are there): one row per (workgroup, gene).  A wave's first stretch may continue the
  // previous wave's run (first_cont: its M goes to the workgroup's LDS after the chunk loops) and
  // its last may be continued by the next waves (last_cont: it adds their parts, in wave order,
  // before the one store).
  constexpr bool MG = EM && K >= MMSBM_LDS_BIG;
  bool first_cont = false, last_cont = false;
  if (MG && merge && any) {
    const int wc0 = wg_units[w * (T::NWK + 1)], wc1 = wg_units[w * (T::NWK + 1) + T::NWK];
    first_cont = c0 > wc0 && __builtin_amdgcn_readfirstlane(chunk_prow[c0 - 1]) ==
                                 __builtin_amdgcn_readfirstlane(chunk_prow[c0]);
    last_cont = c1 < wc1 && __builtin_amdgcn_readfirstlane(chunk_prow[c1]) ==
                                __builtin_amdgcn_readfirstlane(chunk_prow[c1 - 1]);
  }
  int rv[U];
#pragma unroll
  for (int i = 0; i < U - 1; ++i) rv[i] = any ? ld_rec(clampq(c0 + i)) : 0;
  rv[U - 1] = 0;

  {
    // ---- V_g[b][h] = sum_a th_g[a] p_r[a][b][h] for the workgroup's pivot genes (LDS)
    // vgenes holds GMAX (padded) genes per workgroup, so the theta loads do not wait for
    // wg_gene; p_r is staged in the image region when it fits.  All loads go out together.
    const int ng = wg_gene[w + 1] - wg_gene[w];
    const int* __restrict__ vgw = vgenes + (size_t)w * gcap;
    constexpr bool PV = T::K3 <= T::NWK * T::IMGW;
    double* Ps = smem + gcap * T::VDBL + T::tg_dbl(gcap);
    constexpr int NTG = (T::GMAX * T::KP + T::NTK - 1) / T::NTK, NPV = PV ? (T::K3 + T::NTK - 1) / T::NTK : 1;
    double tg[NTG], pv[NPV];
#pragma unroll
    for (int i = 0; i < NTG; ++i) {
      const int idx = tid + T::NTK * i, gl = idx / T::KP, a = idx % T::KP;
      const int g = vgw[gl < gcap ? gl : 0];
      tg[i] = th[(size_t)g * K + (a < K ? a : 0)];
    }
    if constexpr (PV) {
#pragma unroll
      for (int i = 0; i < NPV; ++i) pv[i] = p[tid + T::NTK * i < T::K3 ? tid + T::NTK * i : 0];
    }
    constexpr int ZR = (T::VROWS - K) * VR;  // rows b >= K read as zero
    if constexpr (ZR > 0)
      for (int idx = tid; idx < ng * ZR; idx += T::NTK)
        Vt[(idx / ZR) * T::VDBL + K * VR + idx % ZR] = 0.0;
#pragma unroll
    for (int i = 0; i < NTG; ++i) {  // theta rows, zero padded
      const int idx = tid + T::NTK * i, gl = idx / T::KP, a = idx % T::KP;
      if (idx < gcap * T::KP) Tg[gl * T::TGR + a] = (gl < ng && a < K) ? tg[i] : 0.0;
    }
    if constexpr (PV) {
#pragma unroll
      for (int i = 0; i < NPV; ++i)
        if (tid + T::NTK * i < T::K3) Ps[tid + T::NTK * i] = pv[i];
    }
    const double* __restrict__ pv_src = PV ? Ps : p;
    __syncthreads();
    st_.mark(6);
    constexpr int CT = K * NG;  // (b, h tile) cell tiles
    constexpr int CG = (CT + 3) / 4;
    const int GT = (ng + 3) / 4;
    constexpr int GTM = (T::GMAX + 3) / 4;
    // wave wv owns cell groups (4 cell tiles) cg = wv, wv + T::NWK, ..., CPR per round, for every
    // gene tile: each p value is loaded once and feeds GT MFMAs (A = the tile's theta rows)
    constexpr int CPR = K <= 12 ? 1 : 2;
    // software pipeline over the rounds: the next round's p values (from L2 when K > 12) are in
    // flight during this round's MFMAs; every load is unconditional (clamped address, value
    // selected afterwards), a round past the last cell group only loads
    auto v_load = [&](int cr, double (&bv)[CPR][NG], int (&ctv)[CPR]) {
#pragma unroll
      for (int u = 0; u < CPR; ++u) {
        const int ct = 4 * (cr + u * T::NWK) + blk;
        const bool cv = cr + u * T::NWK < CG && ct < CT;
        const int bb = cv ? ct / NG : 0, hh = cv ? 4 * (ct % NG) + lo : 0;
        ctv[u] = cv ? ct : -1;
#pragma unroll
        for (int as = 0; as < NG; ++as) {
          const int a = 4 * as + hi;
          const bool ok = cv && a < K && hh < K;
          const double v = pv_src[ok ? (a * K + bb) * K + hh : 0];
          bv[u][as] = ok ? v : 0.0;
        }
      }
    };
    auto v_round = [&](const double (&bv)[CPR][NG], const int (&ctv)[CPR]) {
#pragma unroll
      for (int u = 0; u < CPR; ++u) {
        double acc[GTM];
#pragma unroll
        for (int t = 0; t < GTM; ++t) acc[t] = 0.0;
#pragma unroll
        for (int as = 0; as < NG; ++as)
#pragma unroll
          for (int t = 0; t < GTM; ++t)
            if (t < GT) acc[t] = mfma4(Tg[(4 * t + lo) * T::TGR + 4 * as + hi], bv[u][as], acc[t]);
        const int ct = ctv[u];
#pragma unroll
        for (int t = 0; t < GTM; ++t) {
          const int go = 4 * t + hi;
          if (t < GT && ct >= 0 && go < ng) Vt[go * T::VDBL + (ct / NG) * VR + 4 * (ct % NG) + lo] = acc[t];
        }
      }
    };
    constexpr int CST = CPR * T::NWK;  // cell groups per round (all waves)
    double bvA[CPR][NG], bvB[CPR][NG];
    int ctA[CPR], ctB[CPR];
    v_load(wv, bvA, ctA);
    for (int cr = wv; cr < CG; cr += 2 * CST) {
      v_load(cr + CST, bvB, ctB);
      v_round(bvA, ctA);
      v_load(cr + 2 * CST, bvA, ctA);
      if (cr + CST < CG) v_round(bvB, ctB);
    }
    __syncthreads();
  }
  st_.mark(1);

  double* __restrict__ pb = prows + (size_t)b * n_prows * T::K2;
  constexpr int YS = y_stride(K);
  static_assert(YS <= 16 * T::NBG, "Y stride within the Z / Z' lanes");
  double* __restrict__ yb = ybuf + (size_t)b * (n_y + 1) * YS;
  // staged pieces of one chunk: piece pc = 64 t + lane is SW doubles of row8 = pc / (KP / SW)
  // (rows 0-3: th_u = th_j of obs 0-3, rows 4-7: th_v = th_k), columns SW (pc % (KP / SW)) ..
  typedef double d2v __attribute__((ext_vector_type(2)));  // a native vector: SROA-friendly
  using SV = typename std::conditional<T::SW == 2, d2v, double>::type;
  constexpr int PR = T::KP / T::SW;  // pieces per image row
  // A piece outside the image (lanes past 8 PR) or in the zero pad columns is still loaded (from
  // a clamped address) and stored, to a per-wave dummy slot: no select, so the load cannot be
  // sunk behind an exec mask.
  double* dummy = img + 2 * T::IMG;
  int soff[T::NPC];  // image offset of each piece, or -1 for the dummy slot
#pragma unroll
  for (int t = 0; t < T::NPC; ++t) {
    const int pc = 64 * t + lane, col = T::SW * (pc % PR);
    soff[t] = (pc < 8 * PR && col < K) ? (pc / PR) * TR + col : -1;
  }
  auto stage_load = [&](int rv, SV (&v)[T::NPC]) {
#pragma unroll
    for (int t = 0; t < T::NPC; ++t) {
      const int pc = 64 * t + lane;
      const int row8 = pc < 8 * PR ? pc / PR : 0, col = T::SW * (pc % PR);
      int g = __shfl(rv, (row8 & 3) * 4 + ((row8 >> 2) ? 2 : 1), 64);
      if constexpr (MMSBM_ABL & 2) g &= 63;
      v[t] = *reinterpret_cast<const SV*>(th + (size_t)g * K + (col < K ? col : K - T::SW));
    }
  };
  auto stage_store = [&](double* I, const SV (&v)[T::NPC]) {
#pragma unroll
    for (int t = 0; t < T::NPC; ++t)
      *reinterpret_cast<SV*>(soff[t] >= 0 ? I + soff[t] : dummy) = v[t];
  };

  constexpr int NX16 = (K + 15) / 16;  // 16-wide tiles of each M axis
  d4v m16[NX16 * NX16];
#pragma unroll
  for (int t = 0; t < NX16 * NX16; ++t) m16[t] = d4v{0.0, 0.0, 0.0, 0.0};
  d4v mc[MG ? NX16 * NX16 : 1];  // MG: the first stretch's M when it continues a run
#pragma unroll
  for (int t = 0; t < (MG ? NX16 * NX16 : 1); ++t) mc[t] = d4v{0.0, 0.0, 0.0, 0.0};
  bool first_st = true, kept = false;  // kept: the last stretch heads a merged row
  double ll = 0.0;
  // the image's pad columns are read (times a zero Z entry) by the d dot product and are the Z'
  // operand's k >= K rows: keep them 0
  for (int idx = lane; idx < 2 * T::IMG; idx += 64) img[idx] = 0.0;
  wave_lds_sync();

  // w of observation hi (its count n_r) of a record register
  auto rec_w = [&](int rr) { return __shfl(rr, hi * 4 + 3, 64); };
  // VREG (MMSBM_VREG, K >= MMSBM_VREG_MIN = MMSBM_LDS_BIG): the pivot gene's Z / Z' operands of the V table kept in
  // registers for the whole stretch (reloaded at a gene change) instead of read from LDS per chunk
  constexpr bool VREG = MMSBM_VREG && K >= MMSBM_VREG_MIN && EM;
  constexpr bool ZSPLIT = MMSBM_ZSPLIT && K >= MMSBM_VREG_MIN;  // (K = 20: -7 %, r05_zsplit_ab.txt)
  double vz[VREG ? T::NBG : 1][VREG ? NG : 1], vzp[VREG ? T::NBG : 1][VREG ? NG : 1];
  int cur_vs = -1;
  if (any) {
    // Software pipeline: records U - 1 chunks ahead, theta values DT ahead; the LDS image of
    // chunk q + 1 is written at the end of chunk q (double buffer).
    SV st[U][T::NPC];  // theta values of chunk q in slot (q - c0) % U
#pragma unroll
    for (int i = 0; i < DT; ++i) stage_load(rv[i], st[i]);
    stage_store(img, st[0]);
    for (int q0 = c0; q0 < c1; q0 += U) {
#pragma unroll
      for (int ph = 0; ph < U; ++ph) {
        const int q = q0 + ph;
        if (q >= c1) break;
        const int buf = ph & 1;  // U is even: the image buffer alternates with q
        // prefetch: records of chunk q + U - 1 into the slot chunk q - 1 used, theta of q + DT
        rv[(ph + U - 1) % U] = ld_rec(clampq(q + U - 1));
        stage_load(rv[(ph + DT) % U], st[(ph + DT) % U]);
        wave_lds_sync();
        const double* I = img + buf * T::IMG;
        const int rq = rv[ph % U];
        const int pr0 = __builtin_amdgcn_readlane(rq, 16);
        const int pr1 = __builtin_amdgcn_readlane(rv[(ph + 1) % U], 16);

        // ---- Z[obs hi][b] for b = 4 (4 bg + blk) + lo, then d, c
        const int nw = rec_w(rq);
        const int vsl = __builtin_amdgcn_readlane(rq, 17);
        const double* __restrict__ V = Vt + vsl * T::VDBL;
        if constexpr (VREG) {
          if (vsl != cur_vs) {  // (uniform) a new pivot gene: its V operands into registers
            cur_vs = vsl;
#pragma unroll
            for (int bg = 0; bg < T::NBG; ++bg)
#pragma unroll
              for (int hs = 0; hs < NG; ++hs) {
                vz[bg][hs] = V[(16 * bg + 4 * blk + lo) * VR + 4 * hs + hi];
                vzp[bg][hs] = V[(4 * hs + hi) * VR + 16 * bg + 4 * blk + lo];
              }
          }
        }
        double az[NG];  // th_v[obs lo][4 hs + hi]: the A operand of every b group
#pragma unroll
        for (int hs = 0; hs < NG; ++hs) az[hs] = I[(4 + lo) * TR + 4 * hs + hi];
        double zb[T::NBG];
        double dp = 0.0;
#pragma unroll
        for (int bg = 0; bg < T::NBG; ++bg) {
          // MMSBM_ZSPLIT: even and odd h steps in two accumulators (shorter dependent MFMA chains)
          double z = 0.0, zo = 0.0;
#pragma unroll
          for (int hs = 0; hs < NG; ++hs) {
            const double vv = VREG ? vz[bg][hs] : V[(16 * bg + 4 * blk + lo) * VR + 4 * hs + hi];
            if (ZSPLIT && (hs & 1)) zo = mfma4(az[hs], vv, zo);
            else z = mfma4(az[hs], vv, z);
          }
          if (ZSPLIT) z += zo;
          zb[bg] = z;
          dp = fma(I[hi * TR + 16 * bg + 4 * blk + lo], z, dp);
        }
        const double d = row16_sum(dp) + eps;
        if constexpr (MODE == PASS_LL) {
          if ((lane & 15) == 0) ll += (double)nw * log(d);
        } else {
          const double c = MMSBM_PDIV ? sk_div((double)nw, d) : (double)nw / d;
          // ---- the j- and k-slot sums of this observation (:1009-1011): Y[entry j][b] = c Z[b]
          // and Y[entry k][h] = c Z'[h], Z'[h] = sum_b th_j[b] V[b][h]; 16 lanes of row hi write
          // 16 consecutive words of observation hi's entry
          const int e1 = __shfl(rq, 18 + 2 * hi, 64), e2 = __shfl(rq, 19 + 2 * hi, 64);
          double au[NG];  // th_u[obs lo][4 bs + hi]: the A operand of Z'
#pragma unroll
          for (int bs = 0; bs < NG; ++bs) au[bs] = I[lo * TR + 4 * bs + hi];
#pragma unroll
          for (int bg = 0; bg < T::NBG; ++bg) {
            const int bb = 16 * bg + 4 * blk + lo;
            if (bb < YS && !(MMSBM_ABL & 1)) y_st(yb + (size_t)e1 * YS + bb, c * zb[bg]);
          }
#pragma unroll
          for (int hg = 0; hg < T::NBG; ++hg) {
            double z2 = 0.0, z2o = 0.0;
            // (columns h in [K, KP) of V are zero; the pad column and the next row's words past
            // KP reach only Y pad words, which nothing reads)
#pragma unroll
            for (int bs = 0; bs < NG; ++bs) {
              const double vv = VREG ? vzp[hg][bs] : V[(4 * bs + hi) * VR + 16 * hg + 4 * blk + lo];
              if (ZSPLIT && (bs & 1)) z2o = mfma4(au[bs], vv, z2o);
              else z2 = mfma4(au[bs], vv, z2);
            }
            if (ZSPLIT) z2 += z2o;
            const int hh = 16 * hg + 4 * blk + lo;
            if (hh < YS && !(MMSBM_ABL & 1)) y_st(yb + (size_t)e2 * YS + hh, c * z2);
            else if (MMSBM_ABL & 1) ll += z2;  // (keep Z' live)
          }
          // ---- M += c th_u (x) th_v over the chunk's 4 observations: one v_mfma_f64_16x16x4 per
          // 16 x 16 tile of M, k = the 4 observations.  Lane l holds A[x = l & 15][o = l >> 4] =
          // th_u(obs hi)[x] and B[o = l >> 4][y = l & 15] = c_hi th_v(obs hi)[y]: both come from
          // this lane's own observation hi, whose c it already holds; D[x = hi + 4 i][y = l & 15]
          // in accumulator element i.
          const int col = lane & 15;
          double a16[NX16], b16[NX16];
#pragma unroll
          for (int t = 0; t < NX16; ++t) {
            const int x = 16 * t + col;
            const bool ok = x < K;
            const double va = I[hi * TR + (ok ? x : 0)];
            const double vb = I[(4 + hi) * TR + (ok ? x : 0)];
            a16[t] = ok ? va : 0.0;
            b16[t] = ok ? c * vb : 0.0;
          }
#pragma unroll
          for (int tx = 0; tx < NX16; ++tx)
#pragma unroll
            for (int ty = 0; ty < NX16; ++ty)
              m16[tx * NX16 + ty] = mfma16(a16[tx], b16[ty], m16[tx * NX16 + ty]);
          if (q + 1 >= c1 || pr1 != pr0) {  // end of this gene stretch: its partial row
            const bool to_mc = MG && first_st && first_cont;       // (uniform)
            const bool keep = MG && !to_mc && q + 1 >= c1 && last_cont;
            first_st = false;
            kept = keep;
            if (to_mc) {
#pragma unroll
              for (int t = 0; t < NX16 * NX16; ++t) {
                mc[MG ? t : 0] = m16[t];
                m16[t] = d4v{0.0, 0.0, 0.0, 0.0};
              }
            } else if (!keep) {  // (keep: the loop ends here, m16 stays for the merge)
              double* __restrict__ out = pb + (size_t)pr0 * T::K2;
#pragma unroll
              for (int tx = 0; tx < NX16; ++tx)
#pragma unroll
                for (int ty = 0; ty < NX16; ++ty)
#pragma unroll
                  for (int i = 0; i < 4; ++i) {
                    const int x = 16 * tx + hi + 4 * i, y = 16 * ty + col;
                    if (x < K && y < K && !(MMSBM_ABL & 4)) st_wt(out + x * K + y, m16[tx * NX16 + ty][i]);
                    else if (MMSBM_ABL & 4) ll += m16[tx * NX16 + ty][i];
                    m16[tx * NX16 + ty][i] = 0.0;
                  }
            }
          }
        }
        // next chunk's image into the other buffer (its reads of this buffer are done)
        wave_lds_sync();
        stage_store(img + (buf ^ 1) * T::IMG, st[(ph + 1) % U]);
      }
    }
  }
  st_.mark(2);
  if constexpr (MG) {
    if (merge) {  // (workgroup-uniform) the V tables and images are dead: T::NWK slots of K^2 words
      static_assert((4 * T::VDBL + T::tg_dbl(4)) * 8 + T::IMG_BYTES >= T::NWK * T::K2 * 8,
                    "merge slots within the smallest gene cap's LDS");
      const int col = lane & 15;
      __syncthreads();
      if (first_cont) {
#pragma unroll
        for (int tx = 0; tx < NX16; ++tx)
#pragma unroll
          for (int ty = 0; ty < NX16; ++ty)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int x = 16 * tx + hi + 4 * i, y = 16 * ty + col;
              if (x < K && y < K) smem[wv * T::K2 + x * K + y] = mc[tx * NX16 + ty][i];
            }
      }
      __syncthreads();
      if (kept) {
        const int mypr = __builtin_amdgcn_readfirstlane(chunk_prow[c1 - 1]);
        for (int nx = wv + 1; nx < T::NWK; ++nx) {  // the continuing waves, in order
          const int n0 = wg_units[w * (T::NWK + 1) + nx], n1 = wg_units[w * (T::NWK + 1) + nx + 1];
          if (n0 == n1) continue;  // (an empty unit)
          if (__builtin_amdgcn_readfirstlane(chunk_prow[n0]) != mypr) break;
#pragma unroll
          for (int tx = 0; tx < NX16; ++tx)
#pragma unroll
            for (int ty = 0; ty < NX16; ++ty)
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const int x = 16 * tx + hi + 4 * i, y = 16 * ty + col;
                if (x < K && y < K) m16[tx * NX16 + ty][i] += smem[nx * T::K2 + x * K + y];
              }
          if (__builtin_amdgcn_readfirstlane(chunk_prow[n1 - 1]) != mypr) break;
        }
        double* __restrict__ out = pb + (size_t)mypr * T::K2;
#pragma unroll
        for (int tx = 0; tx < NX16; ++tx)
#pragma unroll
          for (int ty = 0; ty < NX16; ++ty)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int x = 16 * tx + hi + 4 * i, y = 16 * ty + col;
              if (x < K && y < K) st_wt(out + x * K + y, m16[tx * NX16 + ty][i]);
            }
      }
    }
  }
  if constexpr (MMSBM_ABL != 0 && EM)  // ablation builds: keep the skipped stores' values live
    if (ll == -1.2345e300) partL[0] = ll;
  st_.t[5] = (unsigned long long)(c1 - c0);
  st_.t[4] = (unsigned long long)(wg_gene[w + 1] - wg_gene[w]);
  if constexpr (MODE == PASS_LL) {
    // fixed-order workgroup sum of the log-likelihood terms
    __shared__ double red[T::NWK];
    ll = wave_sum(ll);
    __syncthreads();
    if (lane == 0) red[wv] = ll;
    __syncthreads();
    if (tid == 0) {
      double t = 0.0;
      for (int q = 0; q < T::NWK; ++q) t += red[q];
      partL[(size_t)b * n_wg + w] = t;
    }
  }
  st_.mark(3);
  st_.flush(MODE == PASS_A ? 0 : 4, wave_id, lane);
}

struct SpRange {  // per rating: the S partials [lo, hi) of the train plan
  int lo[MAX_R], hi[MAX_R];
};

// ------------------------------------------------------------------------------------------
// gm_kernel (round 5; launch 2 of a large-K iteration): both contractions of the stream-0 partial
// rows in ONE pass over them, as two GEMMs on v_mfma_f64_16x16x4f64:
//   X_q[a]       = sum_cell M_q[cell] p_r[a][cell]        per partial row q  (-> xrow[CS][B][n_prows][K];
//                  upd sums a gene's rows, so x0_g = sum_r sum_{q of (r, g)} X_q, :1009 / :1016)
//   S_w[a][cell] = sum_{q in w} th_g(q)[a] M_q[cell]       per part w         (-> spart, :1012)
// grid (n_sp x CS, B), block 512.  Part w = the rows [q0, q1) of one rating (Plan::sp_desc, 128 rows
// a part); its cells are split into CS groups of whole 64-cell chunks, one workgroup each (CS = 2
// from 9 chunks, K >= 24: the S accumulators of one group then fit the registers of two workgroups
// per CU).  A workgroup walks its rows in tiles of 64 and, in a tile, its chunks: the chunk's M tile
// (64 x 64, from HBM), p_r's 64 cells of every a (L2) and the tile's theta rows sit in LDS; every M
// word is read from HBM once and feeds both products.  Wave wv owns one 16 x 16 X tile (row tile,
// a tile) of the row tile, over the group's chunks (its part of X_q: upd adds the CS groups), and
// one S tile (cell tile, a tile) of every chunk of the group, over all the part's rows (K <= 16:
// 4 tiles each for 8 waves, so two waves split each tile's k-steps and add their parts in wave
// order).  The next chunk's loads are in flight during the current chunk's MFMAs (register
// staging, one LDS buffer).  LDS (72 KB): M tile [64 rows][64] and p chunk [32 a][64], columns
// XOR-swizzled by the row (gm_swz: the X operand reads 16 rows x 2 cells, the S operand 2 rows x 16
// cells, both conflict-free ds_read_b64; addresses formed per k-step, not hoisted, so they take no
// registers), theta tile [64][48] (stride = 16 mod 32 doubles).  Replaces round 4's gene_kernel x0
// workgroups (16 genes each, all of p_r re-read from L2 per workgroup) and gene_sy's S workgroups
// (a second read of every partial row).
// ------------------------------------------------------------------------------------------
// gm_kernel occupancy hint: 4 waves per SIMD (<= 128 VGPRs, two 72 KB workgroups per CU) where
// that does not spill (K <= 16); above, the S accumulators and staging take up to 254 VGPRs and the
// hint is free (one workgroup per CU; 128 spilled 58-120 VGPRs at K = 20-32)
template <int K>
struct GM {
  static constexpr int K2 = K * K;
  static constexpr int NA = (K + 15) / 16;   // 16-wide a tiles
  static constexpr int AP = 16 * NA;
  static constexpr int RT = 64, CW = 64;     // rows per row tile, cells per chunk
  static constexpr int NCH = (K2 + CW - 1) / CW;
  // X rows in NQ fixed groups of QC chunks ([j QC, min((j + 1) QC, NCH))), whatever the launch
  // (round 6): a part's cells run as CS workgroups of NQ / CS consecutive groups each (CS = 1, 2 when
  // NQ is even, NQ) with the same bits, so the launch can choose CS per batch (upd adds the groups
  // in order).  Up to four groups at K = 17-24 (one wave forms a whole X tile, written at the
  // group's last chunk); two at K <= 16, where two waves split each tile's k-steps and add their
  // parts through LDS after the row tile's chunks (two groups' parts fit the freed M tile), and at
  // K >= MMSBM_LDS_BIG (XPOST below)
  // X rows written after a row tile's chunks (two groups) where two waves split an X tile's k-steps
  // (K <= 16) or where one workgroup's S accumulators fill the registers (K >= MMSBM_LDS_BIG: a group
  // written at its last chunk cost K = 30 eight spilled VGPRs, 0.7 %); else at each group's last chunk
  static constexpr bool XPOST = 8 / (4 * NA) == 2 || K >= MMSBM_LDS_BIG;
  static constexpr int QC = XPOST ? (NCH + 1) / 2 : (NCH + 3) / 4;  // chunks per X group
  static constexpr int NQ = (NCH + QC - 1) / QC;          // X groups (all non-empty)
  // Q4 (K >= MMSBM_LDS_BIG, plans with fewer parts than CUs, SetDev::gm_q4): the four-group layout
  // of K = 17-24 there too (written at each group's last chunk; its CS = 2 form spills, but such
  // plans run four workgroups per part)
  static constexpr bool Q4OK = K >= MMSBM_LDS_BIG && 8 / (4 * NA) == 1;
  static constexpr int QC4 = (NCH + 3) / 4, NQ4 = (NCH + QC4 - 1) / QC4;
  static constexpr int qc(bool q4) { return q4 && Q4OK ? QC4 : QC; }
  static constexpr int nq(bool q4) { return q4 && Q4OK ? NQ4 : NQ; }
  static constexpr bool ONE = NCH <= 8;                   // CS = 1 possible (its S accumulators fit)
  static constexpr bool cs_ok(int cs, bool q4 = false) {  // a valid workgroups-per-part count
    return cs >= 1 && cs <= nq(q4) && nq(q4) % cs == 0 && (cs > 1 || ONE) && (nq(q4) / cs) * qc(q4) <= 8;
  }
  static constexpr int TST = AP == 32 ? 48 : 16;  // theta tile row stride (= 16 mod 32 doubles)
  static constexpr int XT = 4 * NA, XK = 8 / XT;  // X tiles per row tile, k-splits per tile
  static constexpr int NXR = NQ;                  // X row sets (one per group; nq(true) under Q4)
  static constexpr int ST = 4 * NA, SK = 8 / ST;  // S tiles per chunk, row splits per tile
  static constexpr int MW = K2 % 2 == 0 ? 2 : 1;  // staging width (a row starts 16-B aligned)
  static constexpr int NM = RT * CW / MW / 512;   // M staging loads per thread
  static constexpr int NP = (AP * CW / MW + 511) / 512;
  static constexpr int NTH = RT * AP / 512;       // theta staging loads per thread
  static constexpr int LDS = (RT * CW + AP * CW + RT * TST) * 8;
  static constexpr int WPE = K <= 16 ? 4 : 1;
  static_assert(XT * XK == 8 && ST * SK == 8, "gm: 8 waves");
  static_assert(RT * CW % (MW * 512) == 0 && RT * AP % 512 == 0, "gm staging");
};

// host view of GM<K>::NXR (the X row sets gm_kernel writes)
constexpr int gm_nxr(int K) {  // (the most of either layout)
  const int nch = (K * K + 63) / 64, xk = 8 / (4 * ((K + 15) / 16));
  const int qc = xk == 2 ? (nch + 1) / 2 : (nch + 3) / 4;
  return (nch + qc - 1) / qc;
}
static_assert(gm_nxr(30) == GM<30>::nq(true) && gm_nxr(16) == GM<16>::NXR && gm_nxr(13) == GM<13>::NXR &&
                  gm_nxr(20) == GM<20>::NXR && gm_nxr(24) == GM<24>::NXR && gm_nxr(25) == GM<25>::nq(true), "gm_nxr");

// column swizzle of the 64-wide LDS tiles: bit 4 <- row bit 0, bits 1-3 <- row bits 1-3
__device__ __forceinline__ int gm_swz(int r) { return ((r & 1) << 4) | (((r >> 1) & 7) << 1); }

template <int K, int CS, bool Q4 = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(GM<K>::WPE))) void gm_kernel(const double* __restrict__ theta, const double* __restrict__ pr,
                                                  const double* __restrict__ prows,
                                                  const int* __restrict__ prow_gene,
                                                  const int* __restrict__ sp_desc, double* __restrict__ xrow,
                                                  double* __restrict__ spart, int P, int R, long long n_prows,
                                                  int n_sp, long long xgs) {
  using G = GM<K>;
  constexpr int K2 = G::K2, K3 = K * K * K, CW = G::CW, RT = G::RT, TST = G::TST, AP = G::AP;
  extern __shared__ __attribute__((aligned(16))) double gsm[];
  double* Ml = gsm;                  // [RT][CW] swizzled
  double* Pt = gsm + RT * CW;        // [AP][CW] swizzled
  double* Tl = Pt + AP * CW;         // [RT][TST]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  static_assert(G::cs_ok(CS, Q4) && (!Q4 || G::Q4OK), "gm_kernel: workgroups per part");
  constexpr int NXH = G::nq(Q4) / CS;               // X groups this workgroup forms
  constexpr int QC = G::qc(Q4);
  constexpr int CPG = NXH * QC;                     // its chunks (the last workgroup's may end early)
  const int w = blockIdx.x / CS, grp = blockIdx.x % CS, b = blockIdx.y;
  const int cb = grp * CPG;          // its first chunk (0 for CS = 1)
  const int l15 = lane & 15, l4 = lane >> 4;
  const int* d = sp_desc + 3 * w;
  const int r = d[0], q0 = d[1], q1 = d[2];
  const double* __restrict__ th = theta + (size_t)b * P * K;
  const double* __restrict__ p = pr + ((size_t)b * R + r) * K3;
  const double* __restrict__ mb = prows + (size_t)b * n_prows * K2;
  double* __restrict__ xb = xrow + (size_t)b * n_prows * K;  // xgs: one group's X rows
  // this wave's X tile (row tile xr, a tile xa, k-split xk) and S tile (cell tile sc, a tile sa,
  // row split sk) of every chunk
  const int xt = wv % G::XT, xk = wv / G::XT, xr = xt % 4, xa = xt / 4;
  const int st = wv % G::ST, sk = wv / G::ST, sc = st % 4, sa = st / 4;
  constexpr int XKS = 16 / G::XK, SKS = 16 / G::SK;  // k-steps per split
  d4v sacc[CPG];
#pragma unroll
  for (int c = 0; c < CPG; ++c) sacc[c] = d4v{0.0, 0.0, 0.0, 0.0};
  typedef double d2v __attribute__((ext_vector_type(2)));
  using MV = typename std::conditional<G::MW == 2, d2v, double>::type;

  // staging of chunk c of the row tile starting at row qt: M words (rows past q1 and cells past
  // K2 load a clamped address and are zeroed), p_r's cells of the chunk for every a
  auto load_m = [&](int qt, int c, MV (&mv)[G::NM]) {
#pragma unroll
    for (int u = 0; u < G::NM; ++u) {
      const int idx = tid + 512 * u, row = idx / (CW / G::MW), col = G::MW * (idx % (CW / G::MW));
      const int q = qt + row, cell = c * CW + col;
      const bool ok = q < q1 && cell < K2;
      const MV v = *reinterpret_cast<const MV*>(mb + (size_t)(ok ? q : q0) * K2 + (ok ? cell : 0));
      mv[u] = ok ? v : MV{};
    }
  };
  auto load_p = [&](int c, MV (&pv)[G::NP]) {
#pragma unroll
    for (int u = 0; u < G::NP; ++u) {
      const int idx = tid + 512 * u, a = idx / (CW / G::MW), col = G::MW * (idx % (CW / G::MW));
      const int cell = c * CW + col;
      const bool ok = idx < AP * CW / G::MW && a < K && cell < K2;
      const MV v = *reinterpret_cast<const MV*>(p + (ok ? (size_t)a * K2 + cell : 0));
      pv[u] = ok ? v : MV{};
    }
  };
  auto store_mp = [&](const MV (&mv)[G::NM], const MV (&pv)[G::NP]) {
#pragma unroll
    for (int u = 0; u < G::NM; ++u) {
      const int idx = tid + 512 * u, row = idx / (CW / G::MW), col = G::MW * (idx % (CW / G::MW));
      *reinterpret_cast<MV*>(Ml + row * CW + (col ^ gm_swz(row))) = mv[u];
    }
#pragma unroll
    for (int u = 0; u < G::NP; ++u) {
      const int idx = tid + 512 * u, a = idx / (CW / G::MW), col = G::MW * (idx % (CW / G::MW));
      if (idx < AP * CW / G::MW) *reinterpret_cast<MV*>(Pt + a * CW + (col ^ gm_swz(a))) = pv[u];
    }
  };
  auto load_t = [&](int qt, double (&tv)[G::NTH]) {
#pragma unroll
    for (int u = 0; u < G::NTH; ++u) {
      const int idx = tid + 512 * u, row = idx / AP, a = idx % AP;
      const int q = qt + row;
      const bool ok = q < q1 && a < K;
      const int g = prow_gene[ok ? q : q0];
      const double v = th[(size_t)g * K + (ok ? a : 0)];
      tv[u] = ok ? v : 0.0;
    }
  };
  auto store_t = [&](const double (&tv)[G::NTH]) {
#pragma unroll
    for (int u = 0; u < G::NTH; ++u) {
      const int idx = tid + 512 * u;
      Tl[(idx / AP) * TST + idx % AP] = tv[u];
    }
  };
  // per-lane LDS bases and swizzles of the operands (the k-step's address is formed in the loop)
  const int xrow_l = 16 * xr + l15, xa_l = 16 * xa + l15;
  const int xsw_m = gm_swz(xrow_l), xsw_p = gm_swz(xa_l);
  const double* xm = Ml + xrow_l * CW;
  const double* xp = Pt + xa_l * CW;
  const double* sT = Tl + 16 * sa + l15;
  const int scell = 16 * sc + l15;

  MV mv[G::NM], pv[G::NP];
  double tv[G::NTH];
  if (q0 < q1) {
    load_t(q0, tv);
    load_m(q0, cb, mv);
    load_p(cb, pv);
  }
  constexpr bool XPOST = G::XPOST && !Q4;
  constexpr int NXA = XPOST ? NXH : 1;  // X accumulators held over the row tile's chunks
  for (int qt = q0; qt < q1; qt += RT) {
    d4v xacc[NXA];
#pragma unroll
    for (int j = 0; j < NXA; ++j) xacc[j] = d4v{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int i = 0; i < CPG; ++i) {
      const int c = cb + i;
      if (c >= G::NCH) break;  // (uniform: the last group may hold fewer chunks)
      __syncthreads();  // the previous chunk's reads of the LDS tiles are done
      store_mp(mv, pv);
      if (i == 0) store_t(tv);
      __syncthreads();
      // next chunk (or the next row tile's first chunk and theta rows) in flight
      if (i + 1 < CPG && c + 1 < G::NCH) {
        load_m(qt, c + 1, mv);
        load_p(c + 1, pv);
      } else if (qt + RT < q1) {
        load_m(qt + RT, cb, mv);
        load_p(cb, pv);
        load_t(qt + RT, tv);
      }
      // X tile: rows 16 xr + i, a 16 xa + j; k = the chunk's cells (this wave's k-split of them)
      const int hx = XPOST ? i / QC : 0;  // (compile-time: i is unrolled, cb a multiple of QC)
#pragma unroll 4
      for (int s = xk * XKS; s < (xk + 1) * XKS; ++s) {
        const int cell = 4 * s + l4;
        xacc[hx] = mfma16(xm[cell ^ xsw_m], xp[cell ^ xsw_p], xacc[hx]);
      }
      // K > 16: the chunk ends its X group (QC chunks; the part's last chunk ends the last group),
      // whose X rows go out at once (no register holds a group past its chunks)
      if constexpr (!XPOST) {
        constexpr int ILAST = (G::NCH - 1) - (CS - 1) * CPG;  // the part's last chunk, in the last workgroup
        if (i % QC == QC - 1 || (i == ILAST && grp == CS - 1)) {  // (uniform; i is compile-time)
          const int xs = grp * NXH + i / QC;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int row = 16 * xr + l4 + 4 * e, a = 16 * xa + l15;
            if (qt + row < q1 && a < K) xb[xs * xgs + (size_t)(qt + row) * K + a] = xacc[0][e];
          }
          xacc[0] = d4v{0.0, 0.0, 0.0, 0.0};
        }
      }
      // S tile: a 16 sa + i, cells 16 sc + j of the chunk; k = the tile's rows
#pragma unroll 4
      for (int s = sk * SKS; s < (sk + 1) * SKS; ++s) {
        const int row = 4 * s + l4;
        sacc[i] = mfma16(sT[row * TST], Ml[row * CW + (scell ^ gm_swz(row))], sacc[i]);
      }
    }
    if constexpr (XPOST && G::XK == 1) {
#pragma unroll
      for (int j = 0; j < NXH; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = 16 * xr + l4 + 4 * e, a = 16 * xa + l15;
          if (qt + row < q1 && a < K) xb[(grp * NXH + j) * xgs + (size_t)(qt + row) * K + a] = xacc[j][e];
        }
    }
    if constexpr (G::XK == 2) {
      // K <= 16: the row tile's X rows per group, the k-splits' parts added in wave order through
      // LDS (Ml is free: group j's parts at 2048 j)
      static_assert(NXH <= 2, "two groups' parts in the M tile");
      __syncthreads();
      if (xk == 1)
#pragma unroll
        for (int j = 0; j < NXH; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) Ml[2048 * j + (xt * 4 + e) * 64 + lane] = xacc[j][e];
      __syncthreads();
      if (xk == 0)
#pragma unroll
        for (int j = 0; j < NXH; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int row = 16 * xr + l4 + 4 * e, a = 16 * xa + l15;
            const double v = xacc[j][e] + Ml[2048 * j + (xt * 4 + e) * 64 + lane];
            if (qt + row < q1 && a < K) xb[(grp * NXH + j) * xgs + (size_t)(qt + row) * K + a] = v;
          }
    }
  }
  // the part's S partial over the group's cells: the row splits' parts added in wave order
  double* __restrict__ out = spart + ((size_t)b * n_sp + w) * K3;
  if constexpr (G::SK == 2) __syncthreads();
#pragma unroll
  for (int i = 0; i < CPG; ++i) {
    const int c = cb + i;
    if (c >= G::NCH) break;
    if constexpr (G::SK == 2) {
      if (sk == 1)
#pragma unroll
        for (int e = 0; e < 4; ++e) Ml[(st * 4 + e) * 64 + lane] = sacc[i][e];
      __syncthreads();
      if (sk == 0)
#pragma unroll
        for (int e = 0; e < 4; ++e) sacc[i][e] += Ml[(st * 4 + e) * 64 + lane];
      __syncthreads();
    }
    if (sk == 0) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int a = 16 * sa + l4 + 4 * e, cell = c * CW + 16 * sc + l15;
        if (a < K && cell < K2) out[(size_t)a * K2 + cell] = sacc[i][e];
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// upd_kernel (launch 3), grid (theta workgroups + cell workgroups + q workgroups, B), block 512:
//   theta workgroups: one wave per gene, lane a: X = the gene's gm_kernel X rows + its Y entries
//     (+ the joint model's pair sums);
//     theta' = theta X / deg (:1016-1018), or SUMS: nth = X
//   cell workgroups: 64 cells x 8 parts; S_r = sum of the rating's S partials (fixed order);
//     p' = p S / (eps + sum_r p S) in place (:1021-1028), or SUMS: S_out = S
//   q workgroups (joint model, include/mmsbm_pairs.h): qr from the pair launch's S2 partials
// ------------------------------------------------------------------------------------------
constexpr int UPD_NT = 512;

template <int K, bool SUMS>
__global__ __launch_bounds__(UPD_NT) void upd_kernel(
    double* __restrict__ theta, double* __restrict__ pr, const double* __restrict__ spart,
    const int* __restrict__ deg,
    SpRange spr, int P, int R, int n_sp, int n_th_wg, double eps, double* __restrict__ nth_out,
    double* __restrict__ S_out, const double* __restrict__ nth_add, const double* __restrict__ q_part,
    double* __restrict__ q_out, int n_qwg, const double* __restrict__ xrow, const int* __restrict__ prow_ptr,
    long long n_prows, long long xgs, const double* __restrict__ ybuf, const int* __restrict__ yptr,
    long long n_y, int nxr) {
  constexpr int K2 = K * K, K3 = K * K * K;
  constexpr int NCW = (K3 + 63) / 64, NPART = UPD_NT / 64;
  __shared__ double red[MAX_R * NPART * 64];
  const int tid = threadIdx.x, b = blockIdx.y, w = blockIdx.x;
  if (w < n_th_wg) {
    // one wave per gene (round 6): its X rows (lanes a < K), then its Y entries with 16-byte loads
    // over the whole wave (the wide coalesced form; a gene's entries are one contiguous block and
    // YS is a multiple of 4 doubles): lane l < LW reads words 2 l, 2 l + 1 of each WW-word step,
    // components 2 l mod YS and 2 l + 1 mod YS (WW = EPI YS, whole entries; pad components are
    // summed apart and never used), YU2 steps in flight; the lanes of one component are then
    // added in order through LDS
    const int lane = tid & 63, wv = tid >> 6;
    const int g = w * (UPD_NT / 64) + wv;
    if (g >= P) return;  // (wave-uniform; no barrier in this branch)
    const int a = lane < K ? lane : 0;
    const size_t o = ((size_t)b * P + g) * K + a;
    const double th = theta[o];
    const int dg = deg[g];
    const double ad = nth_add ? nth_add[o] : 0.0;
    // the gene's X rows (gm_kernel), rating then row order, cell groups in order
    const double* __restrict__ xb = xrow + (size_t)b * n_prows * K + a;
    double X = 0.0;
    for (int r = 0; r < R; ++r)
      for (int q = prow_ptr[(size_t)r * (P + 1) + g], qe = prow_ptr[(size_t)r * (P + 1) + g + 1]; q < qe; ++q) {
        double x = xb[(size_t)q * K];
#pragma unroll
        for (int h = 1; h < (GM<K>::Q4OK ? nxr : GM<K>::NXR); ++h) x += xb[h * xgs + (size_t)q * K];
        X += x;
      }
    constexpr int YS = y_stride(K), EPI = 128 / YS, WW = EPI * YS, LW = WW / 2, YU2 = 8;
    typedef double d2 __attribute__((ext_vector_type(2)));
    const double* __restrict__ yb = ybuf + (size_t)b * (n_y + 1) * YS;
    const long long w0 = (long long)yptr[g] * YS, w1 = (long long)yptr[g + 1] * YS;
    const long long wf = w0 + 2 * (lane < LW ? lane : 0);
    double Sa = 0.0, Sb = 0.0;
    if (lane < LW) {
      for (long long wd = wf; wd < w1; wd += (long long)YU2 * WW) {
        d2 v[YU2];
#pragma unroll
        for (int u = 0; u < YU2; ++u)
          v[u] = y_ld2(reinterpret_cast<const d2*>(yb + (wd + (long long)u * WW < w1 ? wd + (long long)u * WW : wf)));
#pragma unroll
        for (int u = 0; u < YU2; ++u)
          if (wd + (long long)u * WW < w1) {
            Sa += v[u].x;
            Sb += v[u].y;
          }
      }
    }
    double* __restrict__ yr = red + wv * 128;
    yr[2 * lane] = Sa;
    yr[2 * lane + 1] = Sb;
    wave_lds_sync();
    if (lane < K) {
      double Y = yr[lane];
#pragma unroll
      for (int jj = 1; jj < EPI; ++jj) Y += yr[lane + jj * YS];
      X += Y;
      if (nth_add) X += ad;
      if constexpr (SUMS) nth_out[o] = X;
      else theta[o] = th * X / (double)dg;
    }
    return;
  }
  const int cl = tid & 63, part = tid >> 6;
  if (w < n_th_wg + NCW) {
    // NPART threads per cell, each summing a share of every rating's S partials (16 loads in
    // flight), the shares combined in order through LDS
    const int cell = (w - n_th_wg) * 64 + cl;
    const bool cv = cell < K3;
    const int cc = cv ? cell : 0;
    double po[MAX_R];
#pragma unroll
    for (int r = 0; r < MAX_R; ++r) po[r] = pr[((size_t)b * R + (r < R ? r : R - 1)) * K3 + cc];
    for (int r = 0; r < R; ++r) {
      const int n = spr.hi[r] - spr.lo[r];
      const int s0 = spr.lo[r] + n * part / NPART, s1 = spr.lo[r] + n * (part + 1) / NPART;
      double S = 0.0;
      for (int sp = s0; sp < s1; sp += 16) {
        double v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const double x = spart[((size_t)b * n_sp + (sp + u < s1 ? sp + u : s0)) * K3 + cc];
          v[u] = sp + u < s1 ? x : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) S += v[u];
      }
      red[(r * NPART + part) * 64 + cl] = S;
    }
    __syncthreads();
    if (part == 0 && cv) {
      double npr[MAX_R];
      double den = eps;
#pragma unroll
      for (int r = 0; r < MAX_R; ++r) {
        if (r < R) {
          double S = red[r * NPART * 64 + cl];
#pragma unroll
          for (int q = 1; q < NPART; ++q) S += red[(r * NPART + q) * 64 + cl];
          if constexpr (SUMS) {
            S_out[((size_t)b * R + r) * K3 + cell] = S;
          } else {
            npr[r] = po[r] * S;
            den += npr[r];
          }
        }
      }
      if constexpr (!SUMS) {
#pragma unroll
        for (int r = 0; r < MAX_R; ++r)
          if (r < R) pr[((size_t)b * R + r) * K3 + cell] = npr[r] / den;
      }
    }
    return;
  }
  // joint model q cells: 64 cells of qr per workgroup, NPART threads per cell each summing a share
  // of the pair launch's S2 partials [B][n_qwg][R][K2] (16 loads in flight), the shares combined in
  // order; qr <- qr S2 / (eps + sum_r qr S2) (src/TrigenicInteractionPredictor_23.py:1660-1666)
  const int cell = (w - n_th_wg - NCW) * 64 + cl;
  const bool cv = cell < K2;
  const int cc = cv ? cell : 0;
  double qo[MAX_R];
#pragma unroll
  for (int r = 0; r < MAX_R; ++r) qo[r] = q_out[((size_t)b * R + (r < R ? r : R - 1)) * K2 + cc];
  const int s0 = n_qwg * part / NPART, s1 = n_qwg * (part + 1) / NPART;
  for (int r = 0; r < R; ++r) {
    double S = 0.0;
    for (int ww = s0; ww < s1; ww += 16) {
      double v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const double x = q_part[(((size_t)b * n_qwg + (ww + u < s1 ? ww + u : s0)) * R + r) * K2 + cc];
        v[u] = ww + u < s1 ? x : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) S += v[u];
    }
    red[(r * NPART + part) * 64 + cl] = S;
  }
  __syncthreads();
  if (part == 0 && cv) {
    double nq[MAX_R];
    double den = eps;
#pragma unroll
    for (int r = 0; r < MAX_R; ++r) {
      if (r < R) {
        double S = red[r * NPART * 64 + cl];
#pragma unroll
        for (int q = 1; q < NPART; ++q) S += red[(r * NPART + q) * 64 + cl];
        nq[r] = qo[r] * S;
        den += nq[r];
      }
    }
#pragma unroll
    for (int r = 0; r < MAX_R; ++r)
      if (r < R) q_out[((size_t)b * R + r) * K2 + cell] = nq[r] / den;
  }
}

// ------------------------------------------------------------------------------------------
// M-step from summed accumulators (link-sharded iteration, after the cross-rank all-reduce):
//   theta[g][a] <- theta[g][a] * nth[g][a] / deg[g]                          (:1016-1018)
//   p_r <- p_r S_r / (eps + sum_r p_r S_r)                                      (:1021-1028)
// with the same operation order as upd_kernel.  Grid (ceil((P K + K^3) / 256), B).
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

// Fixed-order sum of per-workgroup partials: grid (B), block 256.
__global__ __launch_bounds__(256) void reduce_kernel(const double* __restrict__ part, int n,
                                                     double* __restrict__ out) {
  __shared__ double red[4];
  const int b = blockIdx.x;
  double s = 0.0;
  for (int t = threadIdx.x; t < n; t += blockDim.x) s += part[(size_t)b * n + t];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[b] = red[0] + red[1] + red[2] + red[3];
}

// ------------------------------------------------------------------------------------------
// Prediction (:530-547): P(r=1) = sum th th th p[..][1], no eps.  grid (ceil(n/256), B).
// Ids outside [0, P) give NaN (the host wrapper raises IndexError before that, like :537).
// ------------------------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__(256) void predict_kernel(const int* __restrict__ ids, long long n,
                                                      const double* __restrict__ theta,
                                                      const double* __restrict__ pr,
                                                      double* __restrict__ out, int P, int R) {
  constexpr int K2 = K * K, K3 = K * K * K;
  const int b = blockIdx.y;
  const long long row = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= n) return;
  const int gi = ids[3 * row], gj = ids[3 * row + 1], gk = ids[3 * row + 2];
  if (gi < 0 || gi >= P || gj < 0 || gj >= P || gk < 0 || gk >= P) {
    out[(size_t)b * n + row] = __builtin_nan("");
    return;
  }
  const double* __restrict__ th = theta + (size_t)b * P * K;
  const double* __restrict__ p = pr + ((size_t)b * R + 1) * K3;
  const double* ri = th + (size_t)gi * K;
  const double* rj = th + (size_t)gj * K;
  const double* rk = th + (size_t)gk * K;
  double tk[K];
#pragma unroll
  for (int h = 0; h < K; ++h) tk[h] = rk[h];
  double dsum = 0.0;
  for (int a = 0; a < K; ++a) {
    double y = 0.0;
    for (int bb = 0; bb < K; ++bb) {
      double u = 0.0;
#pragma unroll
      for (int h = 0; h < K; ++h) u = fma(p[a * K2 + bb * K + h], tk[h], u);
      y = fma(rj[bb], u, y);
    }
    dsum = fma(ri[a], y, dsum);
  }
  out[(size_t)b * n + row] = dsum;
}

#include "sk.h"  // the small-K (K <= 12) kernel family

// ------------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------------
struct SetDev {  // device copy of one link set's plan
  mmsbm_plan::Plan h;
  bool present = false;
  int4* rows = nullptr;
  int* chunk_prow = nullptr;
  int* chunk_vslot = nullptr;
  int* wg_units = nullptr;
  int* wg_code = nullptr;
  int* wg_gene = nullptr;
  int* vgenes = nullptr;
  int* prow_ptr = nullptr;
  int* prow_gene = nullptr;
  int* sp_desc = nullptr;
  int* row_y = nullptr;                 // large-K EM plans: Y entries of each stream-0 row,
  int* yptr = nullptr;                  // and each gene's entry range
  int* gptr = nullptr;                  // small-K: each gene's gene-major X partial rows
  int* sku[2] = {nullptr, nullptr};     // small-K plans (sk.h): slot descriptors of each group,
  int4* skr[2] = {nullptr, nullptr};    // slot-major records,
  int* skrow12 = nullptr;               // slot-major row12 of group 0
  int ncu = 0;                          // CUs the fused plan's unit target came from (0: none)
  int unit_target = 0;
  bool gm_q4 = false;                   // K >= MMSBM_LDS_BIG: gm_kernel's four-group X layout (GM<K>::Q4OK)
  void release() {
    void* ps[] = {rows, chunk_prow, chunk_vslot, wg_units, wg_code, wg_gene, vgenes, prow_ptr, prow_gene, sp_desc,
                  row_y, yptr, gptr, sku[0], sku[1], skr[0], skr[1], skrow12};
    for (void* p : ps)
      if (p) (void)hipFree(p);
    *this = SetDev();
  }
};

size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

using PassFn = int (*)(mmsbm_ctx*, int mode, int which, const double*, const double*, hipStream_t);
using FinFn = int (*)(mmsbm_ctx*, bool sums, double*, double*, double*, double*, hipStream_t);

struct Launch {
  PassFn pass;
  FinFn fin;
  int (*mapply)(mmsbm_ctx*, double*, double*, const double*, const double*, hipStream_t);
  int (*predict)(mmsbm_ctx*, const int*, long long, const double*, const double*, double*, hipStream_t);
  int gmax;
  PassFn sk_pass;  // small-K kernels (sk.h), K <= 12; nullptr above
  FinFn sk_fin;
  int (*gm_groups)(const mmsbm_ctx*, int, bool);  // gm_kernel's workgroups per part (gm_cs<K>)
};

}  // namespace

struct mmsbm_ctx {
  unsigned long long* stamp = nullptr;  // MMSBM_STAMP measurement builds
  int device = 0;
  int K = 0, R = 0, B = 0, P = 0;
  double eps = 1e-10;
  int gcap = 0;                  // most pivot genes per stream-0 workgroup (<= KT<K>::GMAX)
  bool sk = false;               // K <= 12: the small-K kernels of sk.h (MMSBM_SK=0: the large-K ones)
  bool sk_fused = false;         // small-K: one fused E-step launch (SK_U) instead of pass A + pass B
  bool sk_y = false;             // small-K fused: the stream-0 E-step with Y entries (SK_Y)
  int family = MMSBM_FAMILY_AUTO;  // mmsbm_set_family: SK_U / SK_Y, or from B (AUTO)
  int nact = 0;                  // mmsbm_set_active: samples [0, nact) run (0: all B)
  SetDev sets[2];
  int* deg = nullptr;            // device, owned
  std::vector<int> deg_host;
  bool deg_pending = false;      // mmsbm_set_degree: the next set_links(TRAIN) keeps this degree
  bool zero_degree = false;
  char* ws = nullptr;
  long long ws_bytes = 0;
  // workspace views: cbuf = small-K c / large-K Y entries, prows = small-K X / large-K M^0 partial
  // rows, spart = S partials
  double *cbuf = nullptr, *prows = nullptr, *spart = nullptr, *partL = nullptr;
  double *nth_tmp = nullptr, *S_tmp = nullptr;  // fin_kernel sums-out scratch (kernel timing)
  const double* nth_add = nullptr;  // joint model: pair sums added before the degree division
  const double* q_part = nullptr;   // joint model: S2 partials for fin's q cells (null = none)
  double* q_out = nullptr;          // joint model: qr, updated in place by fin's q cells
  int n_qwg = 0;                    // joint model: S2 partials per sample
  unsigned attr = 0;             // dynamic-LDS opt-ins done on this context's device
  bool timing = false;
  int timing_stride = 1;
  std::vector<hipEvent_t> ev[3];
  size_t nev[3] = {0, 0, 0};
  // hipGraph replay of mmsbm_iterate (MMSBM_GRAPH=G: G iterations per graph, 0 = direct launches).
  // The graph bakes in every kernel argument, so each setter bumps `gen` and a stale graph is
  // re-captured.
  int graph_iters = 0;
  unsigned long long gen = 1;
  bool warm = false;                 // a direct iteration ran (LDS opt-ins done before capture)
  hipStream_t cap = nullptr;         // capture stream (torch's default stream cannot be captured)
  hipGraphExec_t gexec = nullptr;
  double* xrows = nullptr;       // gm_kernel's X rows [GM<K>::NXR groups][B][n_prows][K]
  int ncu = 256;                 // the device's compute units (gm_kernel's split rule)
  int gm_cs = 0;                 // MMSBM_GM_CS: force gm_kernel's workgroups per part (0: by batch)
  const double *g_theta = nullptr, *g_pr = nullptr;
  unsigned long long g_gen = 0;
  int g_iters = 0;
};

namespace {

// samples the launches cover (grid.y): the active prefix of the B (mmsbm_set_active)
inline int nb_of(const mmsbm_ctx* c) { return c->nact > 0 && c->nact < c->B ? c->nact : c->B; }

struct WsLayout {
  size_t cbuf, prows, spart, partL, nth, S, xrows, total;
};

WsLayout ws_layout(const mmsbm_ctx* c) {
  WsLayout L{};
  const auto& tr = c->sets[MMSBM_SET_TRAIN].h;
  const auto& te = c->sets[MMSBM_SET_TEST].h;
  const size_t K2 = (size_t)c->K * c->K, K3 = K2 * c->K, B = c->B;
  size_t off = 0;
  if (c->sk) {
    // small-K: c at the stream-1/2 rows, X partials (K per partial row), S partials (K^3 per
    // stream-0 workgroup), likelihood partials, fin's sums-out scratch
    // (SK_Y: the Y entries instead of c)
    L.cbuf = off;
    off += align_up(c->sk_y ? B * (tr.n_y + 1) * c->K * 8
                            : B * std::max<long long>(tr.sk_slots[1] * 4 * tr.sk_L[1], 1) * 8);
    L.prows = off;  // (SK_Y: the X rows are Y entries)
    off += align_up(c->sk_y ? 8 : B * std::max<long long>(tr.n_prows, 1) * c->K * 8);
    L.spart = off;
    off += align_up(B * std::max(tr.n_wg_a, 1) * K3 * 8);
    L.partL = off;
    off += align_up(B * std::max({tr.n_wg_a, te.n_wg_a, 1}) * 8);
    L.nth = off;
    off += align_up(B * (size_t)c->P * c->K * 8);
    L.S = off;
    off += align_up(B * c->R * K3 * 8);
    L.total = off;
    return L;
  }
  // large-K: Y entries (+ the dummy entry of padding rows), M^0 partial rows, S partials,
  // likelihood partials, fin's sums-out scratch, gm_kernel's X rows
  L.cbuf = off;
  off += align_up(B * (tr.n_y + 1) * y_stride(c->K) * 8);
  L.prows = off;
  off += align_up(B * std::max<long long>(tr.n_prows, 1) * K2 * 8);
  L.spart = off;
  off += align_up(B * std::max(tr.n_sp, 1) * K3 * 8);
  L.partL = off;
  off += align_up(B * std::max({tr.n_wg_a, te.n_wg_a, 1}) * 8);
  L.nth = off;
  off += align_up(B * (size_t)c->P * c->K * 8);
  L.S = off;
  off += align_up(B * c->R * K3 * 8);
  L.xrows = off;  // gm_kernel's X row groups (GM<K>::NXR <= 4)
  off += align_up(gm_nxr(c->K) * B * std::max<long long>(tr.n_prows, 1) * c->K * 8);
  L.total = off;
  return L;
}

// Saves and restores the caller's current device around an ABI call (every call runs on the
// context's device; torch's notion of the current device is left as it was).
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

template <typename KernelT>
int lds_opt_in(mmsbm_ctx* c, unsigned bit, KernelT* kern, int bytes) {
  if (bytes > 64 * 1024 && !(c->attr & (1u << bit))) {
    HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
    c->attr |= 1u << bit;
  }
  return MMSBM_OK;
}

// gm_kernel's workgroups per part, CS (the bits are the same for every valid CS: GM<K>::NQ fixed X
// groups): the largest valid CS whose grid still fits one round of resident workgroups (one sample
// at K = 13-32: the grid is a few dozen to a few hundred parts; r05: two per part at K=20 +24 %),
// else the smallest valid one (K=20 x 8: -6 % with two; one is invalid where one workgroup's S
// accumulators would not fit, NCH > 8).  MMSBM_GM_CS=n forces a valid n (tests, measurement).
template <int K>
int gm_cs(const mmsbm_ctx* c, int nsp, bool q4) {
  using G = GM<K>;
  q4 = q4 && G::Q4OK;
  if (c->gm_cs > 0 && G::cs_ok(c->gm_cs, q4)) return c->gm_cs;
  const long long slots = (long long)c->ncu * (G::WPE >= 4 ? 2 : 1);
  int lo = 0, best = 0;
  for (int cs = 1; cs <= G::nq(q4); ++cs) {
    if (!G::cs_ok(cs, q4)) continue;
    if (!lo) lo = cs;
    if ((long long)cs * nsp * nb_of(c) <= slots) best = cs;
  }
  return best ? best : lo;
}

// one gm_kernel launch with CS workgroups per part (a CS GM<K> does not allow is never chosen)
template <int K, int CS, bool Q4>
int launch_gm(mmsbm_ctx* c, const SetDev& sd, int nsp, const double* theta, const double* pr,
              hipStream_t s) {
  if constexpr (GM<K>::cs_ok(CS, Q4) && (!Q4 || GM<K>::Q4OK)) {
    int rc;
    if ((rc = lds_opt_in(c, (Q4 ? 13 : 9) + CS, &gm_kernel<K, CS, Q4>, GM<K>::LDS))) return rc;
    gm_kernel<K, CS, Q4><<<dim3(CS * nsp, nb_of(c)), 512, GM<K>::LDS, s>>>(
        theta, pr, c->prows, sd.prow_gene, sd.sp_desc, c->xrows, c->spart, c->P, c->R, sd.h.n_prows, nsp,
        (long long)c->B * sd.h.n_prows * K);
  }
  return MMSBM_OK;
}

template <int K>
int launch_pass(mmsbm_ctx* c, int mode, int which, const double* theta, const double* pr,
                hipStream_t s) {
  using T = KT<K>;
  const SetDev& sd = c->sets[which];
  const auto& h = sd.h;
  int rc;
  if (mode == PASS_B) {  // launch 2: gm_kernel (X rows + S partials in one pass); upd sums Y
    const int nsp = std::max(h.n_sp, 1);
    const bool q4 = sd.gm_q4 && GM<K>::Q4OK;
    switch (gm_cs<K>(c, nsp, q4) + (q4 ? 4 : 0)) {
      case 1: rc = launch_gm<K, 1, false>(c, sd, nsp, theta, pr, s); break;
      case 2: rc = launch_gm<K, 2, false>(c, sd, nsp, theta, pr, s); break;
      case 3: rc = launch_gm<K, 3, false>(c, sd, nsp, theta, pr, s); break;
      case 4: rc = launch_gm<K, 4, false>(c, sd, nsp, theta, pr, s); break;
      case 6: rc = launch_gm<K, 2, true>(c, sd, nsp, theta, pr, s); break;
      default: rc = launch_gm<K, 4, true>(c, sd, nsp, theta, pr, s); break;
    }
    if (rc) return rc;
  } else {
    if (h.n_wg_a == 0) return MMSBM_OK;
    // dynamic LDS for the context's gene cap (<= the compile-time GMAX the opt-in covers)
    const int lds = (c->gcap * T::VDBL + T::tg_dbl(c->gcap)) * 8 + T::IMG_BYTES + 64;
    if (mode == PASS_A) {
      if ((rc = lds_opt_in(c, 0, &pass_kernel<K, PASS_A>, T::LDS_A))) return rc;
      pass_kernel<K, PASS_A><<<dim3(h.n_wg_a, nb_of(c)), T::NTK, lds, s>>>(
          sd.rows, sd.chunk_prow, sd.chunk_vslot, sd.row_y, sd.wg_units, sd.wg_code, sd.wg_gene, sd.vgenes,
          theta, pr, c->cbuf, c->prows, c->partL, c->P, c->R, h.n_y, h.n_prows, h.n_wg_a, c->eps, c->gcap,
          h.merge ? 1 : 0);
    } else {
      if ((rc = lds_opt_in(c, 1, &pass_kernel<K, PASS_LL>, T::LDS_A))) return rc;
      pass_kernel<K, PASS_LL><<<dim3(h.n_wg_a, nb_of(c)), T::NTK, lds, s>>>(
          sd.rows, sd.chunk_prow, sd.chunk_vslot, nullptr, sd.wg_units, sd.wg_code, sd.wg_gene, sd.vgenes,
          theta, pr, c->cbuf, c->prows, c->partL, c->P, c->R, 0, h.n_prows, h.n_wg_a, c->eps, c->gcap, 0);
    }
  }
  HIP_TRY(hipGetLastError());
  return MMSBM_OK;
}

// launch 3: upd_kernel (theta from the X rows + Y entries, p from the S partials; sums-out mode for the
// link-sharded accumulate and kernel timing)
template <int K>
int launch_fin(mmsbm_ctx* c, bool sums, double* theta, double* pr, double* nth, double* S,
               hipStream_t s) {
  const SetDev& sd = c->sets[MMSBM_SET_TRAIN];
  const auto& h = sd.h;
  const int nthw = (c->P + UPD_NT / 64 - 1) / (UPD_NT / 64);  // one wave per gene
  const int ncw = (K * K * K + 63) / 64;
  SpRange spr{};
  for (int r = 0; r < c->R; ++r) {
    spr.lo[r] = h.sp_lo[r];
    spr.hi[r] = h.sp_hi[r];
  }
  // joint model: the q cells (qr M-step from the pair launch's S2 partials), theta update only
  const int nqc = (!sums && c->q_part) ? (K * K + 63) / 64 : 0;
  const double* xr = c->xrows;  // gm_kernel's X rows; the theta workgroups sum the Y entries (cbuf)
  const double* yb = c->cbuf;
  if (sums)
    upd_kernel<K, true><<<dim3(nthw + ncw, nb_of(c)), UPD_NT, 0, s>>>(
        theta, pr, c->spart, c->deg, spr, c->P, c->R, std::max(h.n_sp, 1), nthw, c->eps,
        nth, S, c->nth_add, nullptr, nullptr, 0, xr, sd.prow_ptr, h.n_prows, (long long)c->B * h.n_prows * K,
        yb, sd.yptr, h.n_y, GM<K>::nq(sd.gm_q4));
  else
    upd_kernel<K, false><<<dim3(nthw + ncw + nqc, nb_of(c)), UPD_NT, 0, s>>>(
        theta, pr, c->spart, c->deg, spr, c->P, c->R, std::max(h.n_sp, 1), nthw, c->eps,
        nth, S, c->nth_add, c->q_part, c->q_out, c->n_qwg, xr, sd.prow_ptr, h.n_prows,
        (long long)c->B * h.n_prows * K, yb, sd.yptr, h.n_y, GM<K>::nq(sd.gm_q4));
  HIP_TRY(hipGetLastError());
  return MMSBM_OK;
}

template <int K>
int launch_mapply(mmsbm_ctx* c, double* theta, double* pr, const double* nth, const double* S,
                  hipStream_t s) {
  const long long n = (long long)c->P * K + (long long)K * K * K;
  mapply_kernel<K><<<dim3((unsigned)((n + 255) / 256), nb_of(c)), 256, 0, s>>>(theta, pr, nth, S, c->deg,
                                                                           c->P, c->R, c->eps);
  HIP_TRY(hipGetLastError());
  return MMSBM_OK;
}

template <int K>
int launch_predict(mmsbm_ctx* c, const int* ids, long long n, const double* theta,
                   const double* pr, double* out, hipStream_t s) {
  if (n == 0) return MMSBM_OK;
  const long long nb = (n + 255) / 256;
  predict_kernel<K><<<dim3((unsigned)nb, nb_of(c)), 256, 0, s>>>(ids, n, theta, pr, out, c->P, c->R);
  HIP_TRY(hipGetLastError());
  return MMSBM_OK;
}

template <int K>
int launch_sk_pass(mmsbm_ctx* c, int mode, int which, const double* theta, const double* pr,
                   hipStream_t s) {
  using T = SKT<K>;
  const SetDev& sd = c->sets[which];
  const auto& h = sd.h;
  const auto& tr = c->sets[MMSBM_SET_TRAIN].h;
  const long long n_cb = std::max<long long>(tr.sk_slots[1] * 4 * tr.sk_L[1], 1);  // pass B's c layout
  SkSec sec{};
  for (int i = 0; i < 3 * MAX_R; ++i) sec.wg_end[i] = h.sk_wg_end[i];
  const int2* r12 = reinterpret_cast<const int2*>(sd.skrow12);
  int rc;
  if (mode == PASS_B) {
    if (h.n_wg_b == 0 || c->sk_fused) return MMSBM_OK;  // fused: streams 1, 2 ran in "pass A"
    if ((rc = lds_opt_in(c, 5, &sk_pass_kernel<K, SK_B>, T::LDS_B))) return rc;
    sk_pass_kernel<K, SK_B><<<dim3(h.n_wg_b, nb_of(c)), NT, T::LDS_B, s>>>(
        sd.skr[1], sd.sku[1], r12, theta, pr, c->cbuf, c->prows, c->spart, c->partL, sec, h.n_wg_a,
        h.sk_L[1], c->P, c->R, n_cb, h.n_prows, h.n_wg_b, c->eps, nullptr, nullptr, 0);
  } else if (mode == PASS_A && c->sk_y) {  // SK_Y: the stream-0 E-step with Y entries
    if (h.n_wg_a == 0) return MMSBM_OK;
    if ((rc = lds_opt_in(c, 9, &sky_pass_kernel<K>, SKY<K>::LDS))) return rc;
    sky_pass_kernel<K><<<dim3(h.n_wg_a, nb_of(c)), NT, SKY<K>::LDS, s>>>(
        sd.skr[0], sd.sku[0], r12, theta, pr, c->cbuf, c->prows, c->spart, sec, h.sk_L[0], c->P, c->R,
        h.n_y, h.n_prows, h.n_wg_a, c->eps);
  } else if (mode == PASS_A && c->sk_fused) {  // the fused E-step: every stream in one launch
    if (h.n_wg_a + h.n_wg_b == 0) return MMSBM_OK;
    if ((rc = lds_opt_in(c, 7, &sk_pass_kernel<K, SK_U>, T::LDS_U))) return rc;
    sk_pass_kernel<K, SK_U><<<dim3(h.n_wg_a + h.n_wg_b, nb_of(c)), NT, T::LDS_U, s>>>(
        sd.skr[0], sd.sku[0], r12, theta, pr, c->cbuf, c->prows, c->spart, c->partL, sec, 0,
        h.sk_L[0], c->P, c->R, n_cb, h.n_prows, h.n_wg_a, c->eps, sd.skr[1], sd.sku[1], h.sk_L[1]);
  } else if (mode == PASS_A) {
    if (h.n_wg_a == 0) return MMSBM_OK;
    if ((rc = lds_opt_in(c, 4, &sk_pass_kernel<K, SK_A>, T::LDS))) return rc;
    sk_pass_kernel<K, SK_A><<<dim3(h.n_wg_a, nb_of(c)), NT, T::LDS, s>>>(
        sd.skr[0], sd.sku[0], r12, theta, pr, c->cbuf, c->prows, c->spart, c->partL, sec, 0,
        h.sk_L[0], c->P, c->R, n_cb, h.n_prows, h.n_wg_a, c->eps, nullptr, nullptr, 0);
  } else {
    if (h.n_wg_a == 0) return MMSBM_OK;
    if ((rc = lds_opt_in(c, 6, &sk_pass_kernel<K, SK_LL>, T::LDS))) return rc;
    sk_pass_kernel<K, SK_LL><<<dim3(h.n_wg_a, nb_of(c)), NT, T::LDS, s>>>(
        sd.skr[0], sd.sku[0], r12, theta, pr, c->cbuf, c->prows, c->spart, c->partL, sec, 0,
        h.sk_L[0], c->P, c->R, n_cb, h.n_prows, h.n_wg_a, c->eps, nullptr, nullptr, 0);
  }
  HIP_TRY(hipGetLastError());
  return MMSBM_OK;
}

template <int K>
int launch_sk_fin(mmsbm_ctx* c, bool sums, double* theta, double* pr, double* nth, double* S,
                  hipStream_t s) {
  const SetDev& sd = c->sets[MMSBM_SET_TRAIN];
  const auto& h = sd.h;
  // gene workgroups: threads per (gene, component), or (SK_Y) one wave per gene
  const int ngw = c->sk_y ? (c->P + SKF_NT / 64 - 1) / (SKF_NT / 64) : (c->P * K + SKF_NT - 1) / SKF_NT;
  const int ncw = (K * K * K + SKF_CW - 1) / SKF_CW;
  const double* yb = c->sk_y ? c->cbuf : nullptr;
  SpRange spr{};
  for (int r = 0; r < c->R; ++r) {
    spr.lo[r] = h.sp_lo[r];
    spr.hi[r] = h.sp_hi[r];
  }
  const int nqc = (!sums && c->q_part) ? (K * K + 63) / 64 : 0;
  if (sums)
    sk_fin_kernel<K, true><<<dim3(ngw + ncw, nb_of(c)), SKF_NT, 0, s>>>(
        theta, pr, c->prows, sd.gptr, c->spart, c->deg, spr, c->P, c->R, h.n_prows,
        std::max(h.n_wg_a, 1), ngw, c->eps, nth, S, c->nth_add, nullptr, nullptr, 0, yb, sd.yptr, h.n_y);
  else
    sk_fin_kernel<K, false><<<dim3(ngw + ncw + nqc, nb_of(c)), SKF_NT, 0, s>>>(
        theta, pr, c->prows, sd.gptr, c->spart, c->deg, spr, c->P, c->R, h.n_prows,
        std::max(h.n_wg_a, 1), ngw, c->eps, nth, S, c->nth_add, c->q_part, c->q_out, c->n_qwg, yb, sd.yptr,
        h.n_y);
  HIP_TRY(hipGetLastError());
  return MMSBM_OK;
}

template <int K>
constexpr PassFn sk_pass_fn() {
  if constexpr (K <= 12) return &launch_sk_pass<K>;
  else return nullptr;
}
template <int K>
constexpr FinFn sk_fin_fn() {
  if constexpr (K <= 12) return &launch_sk_fin<K>;
  else return nullptr;
}

template <int... Ks>
constexpr auto make_table(std::integer_sequence<int, Ks...>) {
  return std::array<Launch, sizeof...(Ks)>{Launch{&launch_pass<Ks + 1>, &launch_fin<Ks + 1>,
                                                  &launch_mapply<Ks + 1>, &launch_predict<Ks + 1>,
                                                  KT<Ks + 1>::GMAX, sk_pass_fn<Ks + 1>(),
                                                  sk_fin_fn<Ks + 1>(), &gm_cs<Ks + 1>}...};
}


const auto kTable = make_table(std::make_integer_sequence<int, MMSBM_MAX_K>{});

// the pass / fin launchers of this context (the small-K kernels of sk.h when c->sk)
PassFn pass_of(const mmsbm_ctx* c) { return c->sk ? kTable[c->K - 1].sk_pass : kTable[c->K - 1].pass; }
FinFn fin_of(const mmsbm_ctx* c) { return c->sk ? kTable[c->K - 1].sk_fin : kTable[c->K - 1].fin; }

int gmax_for(int K) { return kTable[K - 1].gmax; }

int check_shape(const mmsbm_ctx* c) {
  if (c->K < 1 || c->K > MMSBM_MAX_K)
    return fail(MMSBM_ERR_UNSUPPORTED, "K=%d outside [1, %d]: call mmsbm_set_shape", c->K, MMSBM_MAX_K);
  return MMSBM_OK;
}

int check_ready(const mmsbm_ctx* c) {
  int rc = check_shape(c);
  if (rc) return rc;
  if (!c->sets[MMSBM_SET_TRAIN].present) return fail(MMSBM_ERR_INVALID, "train links not set");
  if (!c->ws || c->ws_bytes < (long long)ws_layout(c).total)
    return fail(MMSBM_ERR_INVALID, "workspace missing or too small (mmsbm_workspace_bytes)");
  return MMSBM_OK;
}

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

template <typename D, typename T>
int upload(D** dst, const std::vector<T>& src) {
  static_assert(sizeof(D) == sizeof(T), "element size");
  if (src.empty()) return MMSBM_OK;
  HIP_TRY(hipMalloc(reinterpret_cast<void**>(dst), src.size() * sizeof(T)));
  HIP_TRY(hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
  return MMSBM_OK;
}

int set_degree(mmsbm_ctx* c, const std::vector<int>& deg) {
  ++c->gen;
  c->deg_host = deg;
  c->zero_degree = false;
  for (int v : deg)
    if (v <= 0) c->zero_degree = true;
  if (c->deg) {
    HIP_TRY(hipFree(c->deg));
    c->deg = nullptr;
  }
  return upload(&c->deg, deg);
}

// The small-K kernel family (include/mmsbm.h mmsbm_set_family): the stream-0 E-step with Y entries
// (SK_Y) or the three-stream fused E-step (SK_U).  Same-box A/B (profiles/r04j_sky_ab.txt): SK_Y
// does less than half SK_U's work and wins where the grid is throughput-bound (fold0 K=10, 8
// samples: 78.2k vs 62.1k sample-iter/s) but loses at one sample, where both are bound by one
// wave's latency chain (25.1 vs 23.2 us per iteration), hence AUTO = SK_Y from B = 2.  The two
// order their sums differently, so the family is part of a sample's bits: drivers fix it per run.
void apply_family(mmsbm_ctx* c) {
  bool sky = c->family == MMSBM_FAMILY_SKY || (c->family == MMSBM_FAMILY_AUTO && c->B >= 2);
  if (const char* y = getenv("MMSBM_SK_Y")) sky = y[0] == '1';  // measurement override
  sky = sky && c->sk_fused;
  if (sky != c->sk_y) {  // the plans hold different streams: set links again
    DeviceGuard g(c->device);
    for (auto& sd : c->sets) sd.release();
    c->ws = nullptr;
    c->ws_bytes = 0;
  }
  c->sk_y = sky;
}

}  // namespace

// pairs.hip (same library): the fused pair half of a joint iteration and the pair context shape
int mmsbm_detail_pairs_estep(mmsbm_pairs_ctx* c, const double* theta, const double* qr, double* nth2,
                             hipStream_t s, const double** s2part, int* n_wg);
int mmsbm_detail_pairs_shape(const mmsbm_pairs_ctx* c, int* K, int* R, int* B, int* P);

// One error channel for the whole library: pairs.hip (the joint model's pair lattice, same .so)
// reports through mmsbm_last_error too.
int mmsbm_detail_fail(int code, const char* msg) {
  g_err = msg;
  return code;
}

extern "C" {

int mmsbm_version(void) { return 2; }
int mmsbm_chunk(void) { return CH; }
const char* mmsbm_last_error(void) { return g_err.c_str(); }

int mmsbm_create(int device, mmsbm_ctx** out) {
  if (!out) return fail(MMSBM_ERR_INVALID, "out is null");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev)
    return fail(MMSBM_ERR_INVALID, "device %d outside [0, %d)", device, ndev);
  auto* c = new mmsbm_ctx();
  c->device = device;
  if (const char* gi = getenv("MMSBM_GRAPH")) c->graph_iters = std::max(0, atoi(gi));
  if (const char* gc = getenv("MMSBM_GM_CS")) c->gm_cs = atoi(gc);
  {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0)
      c->ncu = ncu;
  }
  if (MMSBM_STAMP && getenv("MMSBM_STAMP")) {
    DeviceGuard g(device);
    const size_t bytes = sizeof(unsigned long long) * 5 * STAMP_WAVES * STAMP_SLOTS;
    HIP_TRY(hipMalloc(&c->stamp, bytes));
    HIP_TRY(hipMemset(c->stamp, 0, bytes));
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_stamp), &c->stamp, sizeof(c->stamp)));
  }
  *out = c;
  return MMSBM_OK;
}

int mmsbm_destroy(mmsbm_ctx* c) {
  if (!c) return MMSBM_OK;
  DeviceGuard g(c->device);
  for (auto& s : c->sets) s.release();
  if (c->deg) (void)hipFree(c->deg);
  if (c->stamp) (void)hipFree(c->stamp);
  if (c->gexec) (void)hipGraphExecDestroy(c->gexec);
  if (c->cap) (void)hipStreamDestroy(c->cap);
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
  if (K != c->K || R != c->R || P != c->P) {
    // the link plans (gene caps, partial-row sizes), the degree and the workspace were built for
    // the old shape: the caller sets links (and the workspace) again
    DeviceGuard g(c->device);
    for (auto& sd : c->sets) sd.release();
    if (c->deg) (void)hipFree(c->deg);
    c->deg = nullptr;
    c->deg_host.clear();
    c->deg_pending = false;
    c->zero_degree = false;
    c->ws = nullptr;
    c->ws_bytes = 0;
  }
  if (B != c->B) {  // the workspace holds B samples' scratch
    c->ws = nullptr;
    c->ws_bytes = 0;
  }
  c->K = K;
  c->R = R;
  c->B = B;
  c->P = P;
  c->eps = eps;
  {
    const char* e = getenv("MMSBM_SK");  // MMSBM_SK=0: the large-K kernels at every K (measurement)
    const bool sk = K <= 12 && !(e && e[0] == '0');
    if (sk != c->sk) {  // the plans are built for one kernel family
      DeviceGuard g(c->device);
      for (auto& sd : c->sets) sd.release();
      c->ws = nullptr;
      c->ws_bytes = 0;
    }
    c->sk = sk;
    const char* f = getenv("MMSBM_SK_FUSED");  // the fused E-step (SK_U); 0: pass A + pass B
    const bool fused = sk && !(f && f[0] == '0');
    if (fused != c->sk_fused) {  // the fused plan packs its units differently: set links again
      DeviceGuard g(c->device);
      for (auto& sd : c->sets) sd.release();
      c->ws = nullptr;
      c->ws_bytes = 0;
    }
    c->sk_fused = fused;
  }
  c->nact = 0;
  apply_family(c);
  ++c->gen;
  c->attr = 0;      // the dynamic-LDS opt-ins are per kernel, and the kernels depend on K
  c->warm = false;
  // genes per stream-0 workgroup: the LDS budget's GMAX; MMSBM_GCAP=n lowers it (measurement:
  // smaller V tables let more workgroups share a CU)
  c->gcap = gmax_for(K);
  if (const char* g = getenv("MMSBM_GCAP")) {
    const int v = atoi(g);
    if (v >= 4 && v < c->gcap) c->gcap = v;
  }
  return MMSBM_OK;
}

int mmsbm_set_links(mmsbm_ctx* c, int32_t which, const int32_t* ids_host, const int32_t* counts_host,
                    int64_t E) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  int rc = check_shape(c);
  if (rc) return rc;
  if (which != MMSBM_SET_TRAIN && which != MMSBM_SET_TEST)
    return fail(MMSBM_ERR_INVALID, "which=%d", which);
  if (E < 0 || (E > 0 && (!ids_host || !counts_host))) return fail(MMSBM_ERR_INVALID, "bad link table");
  if (E * 3 * 4 >= ((int64_t)1 << 31)) return fail(MMSBM_ERR_UNSUPPORTED, "E=%lld too large", (long long)E);
  for (int64_t q = 0; q < E * 3; ++q)
    if (ids_host[q] < 0 || ids_host[q] >= c->P)
      return fail(MMSBM_ERR_INVALID, "gene id %d outside [0, P=%d)", ids_host[q], c->P);
  for (int64_t q = 0; q < E * c->R; ++q)
    if (counts_host[q] < 0) return fail(MMSBM_ERR_INVALID, "negative count");
  DeviceGuard g(c->device);
  SetDev& sd = c->sets[which];
  sd.release();
  const bool em = which == MMSBM_SET_TRAIN;
  // unit counts do not depend on B, so a sample's sums (and its bits) are the same whatever its
  // batch; MMSBM_UNITS="a,b" overrides them (tests: tiny units force every split path).  The fused
  // small-K launch packs full units (as few as the chunk cap allows: the grid must be resident).
  int units_a = 1536, units_b = 3072;
  int ncu = 0;
  if (c->sk_fused) {  // about the waves resident at once: 15 per CU (two 8-wave workgroups, some
                      // headroom for units the stretch cap or a section's end leave short).  The
                      // unit length sets the sums' order: bits depend on the device's CU count
                      // (plan_info[12]), not on B or the rank
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess || ncu < 1)
      ncu = 256;
    units_a = units_b = 15 * ncu;
    // SK_Y (stream 0 only, the batched family): half as many, twice as long units, 7.5 per CU
    // (fold0 K=10 x 8: 78.2k sample-iter/s at 1,920 units vs 62.2k at 3,840,
    // profiles/r04j_sky_ab.txt)
    if (c->sk_y) units_a = units_b = 15 * ncu / 2;
  }
  if (const char* u = getenv("MMSBM_UNITS")) {
    int a = 0, b = 0;
    const int n = sscanf(u, "%d,%d", &a, &b);
    if (n == 1) b = a;  // (one number: both targets)
    if (n >= 1 && a > 0 && b > 0) {
      units_a = a;
      units_b = b;
    }
  }
  int rho = 85;  // stream-0 unit length, % of the others' (fused plans; plan.h)
  if (const char* e = getenv("MMSBM_SK_RHO")) rho = std::max(10, std::min(100, atoi(e)));
  // large-K workgroups: units of even length (plan.h pack_balanced); MMSBM_BALANCE=0 packs whole
  // runs per unit as in round 3 (measurement)
  const char* bal = getenv("MMSBM_BALANCE");
  const bool balance = !(bal && bal[0] == '0');
  // one partial row per (workgroup, gene) where the pass kernel merges its waves' parts (K >=
  // MMSBM_LDS_BIG); MMSBM_MERGE=0: one per unit stretch (measurement)
  const char* mg = getenv("MMSBM_MERGE");
  const bool merge = !c->sk && c->K >= MMSBM_LDS_BIG && !(mg && mg[0] == '0');
  // stream-0 partial rows per S partial at large K (each S partial is K^3 words the update sums);
  // MMSBM_SP_ROWS=n overrides it (measurement)
  // gm_kernel (round 5): 128 rows (two 64-row tiles) per part, at most 1,024 parts per rating
  // (longer parts beyond that: gm_kernel walks any number of 64-row tiles), so the S partials take
  // at most R x 1,024 x K^3 doubles per sample whatever E (2 x 1,024 x 27,000 x 8 B = 442 MB at K=30)
  // Round 6: a link set whose 128-row parts number fewer than the device's CUs (a fold0-sized set:
  // 32 parts at K = 20) takes 64-row parts (one row tile each), twice the gm_kernel workgroups:
  // one sample at K = 13-32 +12-28 %, 8 samples -1-2 % (profiles/r06sp_rows64_ab.txt).  The rule
  // reads the links and the CU count alone, never B, so a sample's bits do not depend on its batch.
  int sp_rows = c->K <= 12 ? 16 : 128;
  const char* sp_env = getenv("MMSBM_SP_ROWS");
  if (sp_env) sp_rows = std::max(4, atoi(sp_env));
  const int sp_cap = c->sk ? 256 : 1024;
  auto build_plan = [&]() {
    return mmsbm_plan::build(ids_host, counts_host, E, c->R, c->P, em, units_a, units_b, c->gcap, sp_rows,
                             c->sk, 1024, c->sk_fused, mmsbm_plan::sk_gu(c->K), rho, c->sk_y, balance, merge,
                             sp_cap, pnw_host(c->K));
  };
  sd.h = build_plan();
  bool small_plan = false;
  if (em && !c->sk && !sp_env && sd.h.n_sp < c->ncu) {
    sp_rows = 64;
    sd.h = build_plan();
    small_plan = true;
  }
  // such a plan at K >= MMSBM_LDS_BIG also takes gm_kernel's four-group X layout (GM<K>::Q4OK):
  // one sample runs four workgroups per part there (MMSBM_GM_Q4=0/1 forces the choice)
  const char* q4_env = getenv("MMSBM_GM_Q4");
  const bool gm_q4 = q4_env ? q4_env[0] == '1' : small_plan;
  const auto& h = sd.h;
  sd.ncu = c->sk_fused ? ncu : 0;
  sd.gm_q4 = em && !c->sk && gm_q4;
  sd.unit_target = c->sk_fused ? units_a : 0;
  if ((rc = upload(&sd.rows, h.rows))) return rc;
  if ((rc = upload(&sd.chunk_prow, h.chunk_prow))) return rc;
  if ((rc = upload(&sd.chunk_vslot, h.chunk_vslot))) return rc;
  if ((rc = upload(&sd.wg_units, h.wg_units))) return rc;
  if ((rc = upload(&sd.wg_code, h.wg_code))) return rc;
  if ((rc = upload(&sd.wg_gene, h.wg_gene))) return rc;
  {  // pivot genes padded to GMAX per stream-0 workgroup (the pass prologue indexes w GMAX + slot)
    const int gm = c->gcap;
    const size_t nw = h.wg_gene.empty() ? 0 : h.wg_gene.size() - 1;
    std::vector<int> vpad(std::max<size_t>(nw * gm, 1), 0);
    for (size_t w = 0; w < nw; ++w) {
      const int g0 = h.wg_gene[w], ng = h.wg_gene[w + 1] - g0;
      if (ng > gm) return fail(MMSBM_ERR_INVALID, "plan: %d genes in a workgroup (max %d)", ng, gm);
      for (int i = 0; i < gm; ++i) vpad[w * gm + i] = ng ? h.vgenes[g0 + (i < ng ? i : ng - 1)] : 0;
    }
    if ((rc = upload(&sd.vgenes, vpad))) return rc;
  }
  if ((rc = upload(&sd.prow_ptr, h.prow_ptr))) return rc;
  if ((rc = upload(&sd.prow_gene, h.prow_gene))) return rc;
  if ((rc = upload(&sd.sp_desc, h.sp_desc))) return rc;
  if ((rc = upload(&sd.row_y, h.row_y))) return rc;
  if ((rc = upload(&sd.yptr, h.yptr))) return rc;
  if ((rc = upload(&sd.gptr, h.gptr))) return rc;
  for (int g = 0; g < 2; ++g) {
    if ((rc = upload(&sd.sku[g], h.sk_udesc[g]))) return rc;
    if ((rc = upload(&sd.skr[g], h.sk_urec[g]))) return rc;
  }
  if ((rc = upload(&sd.skrow12, h.sk_urow12))) return rc;
  sd.present = true;
  ++c->gen;
  c->ws = nullptr;  // the workspace layout changed: mmsbm_set_workspace again
  if (em) {
    if (!c->deg_pending) {  // no mmsbm_set_degree since the last train set: count this one
      std::vector<int> deg(c->P, 0);  // the reference's `counter` (:986-994)
      for (int64_t q = 0; q < E * 3; ++q) deg[ids_host[q]]++;
      if ((rc = set_degree(c, deg))) return rc;
    }
    c->deg_pending = false;
  }
  return MMSBM_OK;
}

int mmsbm_set_degree(mmsbm_ctx* c, const int32_t* deg_host) {
  if (!c || !deg_host) return fail(MMSBM_ERR_INVALID, "null argument");
  int rc = check_shape(c);
  if (rc) return rc;
  DeviceGuard g(c->device);
  c->deg_pending = true;
  return set_degree(c, std::vector<int>(deg_host, deg_host + c->P));
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
    return fail(MMSBM_ERR_INVALID, "workspace %lld < %lld bytes", (long long)bytes, (long long)L.total);
  if (((uintptr_t)ws) & 255) return fail(MMSBM_ERR_INVALID, "workspace not 256-B aligned");
  DeviceGuard g(c->device);
  c->ws = (char*)ws;
  c->ws_bytes = bytes;
  ++c->gen;
  c->cbuf = (double*)(c->ws + L.cbuf);
  c->prows = (double*)(c->ws + L.prows);
  c->spart = (double*)(c->ws + L.spart);
  c->partL = (double*)(c->ws + L.partL);
  c->nth_tmp = (double*)(c->ws + L.nth);
  c->S_tmp = (double*)(c->ws + L.S);
  c->xrows = c->sk ? nullptr : (double*)(c->ws + L.xrows);
  // small-K: the c vector's last slot (stream-1/2 padding rows read it) and the S partials stay
  // zero; large-K: Y and the S partials start zeroed (every word read is written each iteration)
  HIP_TRY(hipMemset(c->ws + L.cbuf, 0, L.prows - L.cbuf));
  HIP_TRY(hipMemset(c->ws + L.spart, 0, L.partL - L.spart));
  HIP_TRY(hipDeviceSynchronize());
  return MMSBM_OK;
}

// One EM iteration = pass A, pass B, fin (theta / p in place).
static int one_iteration(mmsbm_ctx* c, double* theta, double* pr, bool mark, hipStream_t s) {
  const PassFn pass = pass_of(c);
  const FinFn fin = fin_of(c);
  int rc;
  if (mark && (rc = timing_mark(c, 0, s))) return rc;
  if ((rc = pass(c, PASS_A, MMSBM_SET_TRAIN, theta, pr, s))) return rc;
  if (mark && (rc = timing_mark(c, 0, s))) return rc;
  if (mark && (rc = timing_mark(c, 1, s))) return rc;
  if ((rc = pass(c, PASS_B, MMSBM_SET_TRAIN, theta, pr, s))) return rc;
  if (mark && (rc = timing_mark(c, 1, s))) return rc;
  if (mark && (rc = timing_mark(c, 2, s))) return rc;
  if ((rc = fin(c, false, theta, pr, nullptr, nullptr, s))) return rc;
  if (mark && (rc = timing_mark(c, 2, s))) return rc;
  c->warm = true;
  return MMSBM_OK;
}

// G iterations as one hipGraph launch on s (captured once per theta / pr / context generation).
static int graph_iterations(mmsbm_ctx* c, double* theta, double* pr, int G, hipStream_t s) {
  if (!c->gexec || c->g_theta != theta || c->g_pr != pr || c->g_gen != c->gen || c->g_iters != G) {
    if (c->gexec) {
      HIP_TRY(hipGraphExecDestroy(c->gexec));
      c->gexec = nullptr;
    }
    if (!c->cap) HIP_TRY(hipStreamCreateWithFlags(&c->cap, hipStreamNonBlocking));
    HIP_TRY(hipStreamBeginCapture(c->cap, hipStreamCaptureModeRelaxed));
    int rc = MMSBM_OK;
    for (int i = 0; i < G && rc == MMSBM_OK; ++i) rc = one_iteration(c, theta, pr, false, c->cap);
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(c->cap, &g);
    if (rc == MMSBM_OK && e != hipSuccess)
      rc = fail(MMSBM_ERR_HIP, "hipStreamEndCapture: %s", hipGetErrorString(e));
    if (rc == MMSBM_OK) {
      const hipError_t ei = hipGraphInstantiate(&c->gexec, g, nullptr, nullptr, 0);
      if (ei != hipSuccess) {
        c->gexec = nullptr;
        rc = fail(MMSBM_ERR_HIP, "hipGraphInstantiate: %s", hipGetErrorString(ei));
      }
    }
    if (g) (void)hipGraphDestroy(g);
    if (rc) return rc;
    c->g_theta = theta;
    c->g_pr = pr;
    c->g_gen = c->gen;
    c->g_iters = G;
  }
  HIP_TRY(hipGraphLaunch(c->gexec, s));
  return MMSBM_OK;
}

int mmsbm_iterate(mmsbm_ctx* c, double* theta, double* pr, int32_t n_iters, void* stream) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  int rc = check_ready(c);
  if (rc) return rc;
  if (c->zero_degree)
    return fail(MMSBM_ERR_ZERO_DEGREE, "a gene has no train link (float division by zero)");
  if (!theta || !pr) return fail(MMSBM_ERR_INVALID, "null theta/pr");
  if (n_iters < 0) return fail(MMSBM_ERR_INVALID, "n_iters < 0");
  DeviceGuard g(c->device);
  hipStream_t s = (hipStream_t)stream;
  int it = 0;
  const int G = c->graph_iters;
  if (G > 0 && !c->timing && !c->stamp) {
    if (!c->warm && n_iters > 0) {
      if ((rc = one_iteration(c, theta, pr, false, s))) return rc;
      ++it;
    }
    for (; n_iters - it >= G; it += G)
      if ((rc = graph_iterations(c, theta, pr, G, s))) return rc;
  }
  for (; it < n_iters; ++it)
    if ((rc = one_iteration(c, theta, pr, c->timing && it % c->timing_stride == 0, s))) return rc;
  if (c->stamp && n_iters > 0) {  // measurement: phase cycles of the last iteration's waves
    std::vector<unsigned long long> h((size_t)5 * STAMP_WAVES * STAMP_SLOTS);
    HIP_TRY(hipStreamSynchronize(s));
    HIP_TRY(hipMemcpy(h.data(), c->stamp, h.size() * 8, hipMemcpyDeviceToHost));
    if (const char* path = getenv("MMSBM_STAMP_DUMP")) {  // raw [kernel][wave][slot] words
      if (FILE* f = fopen(path, "wb")) {
        fwrite(h.data(), 8, h.size(), f);
        fclose(f);
      }
    }
    const char* names[5] = {"passA", "passB", "fin", "spart", "passLL"};
    for (int k = 0; k < 5; ++k) {
      double sum[4] = {0, 0, 0, 0}, chunks = 0;
      unsigned long long mx = 0, t0min = ~0ull, t3max = 0;
      long long n = 0;
      for (long long wv = 0; wv < STAMP_WAVES; ++wv) {
        const unsigned long long* t = &h[((size_t)k * STAMP_WAVES + wv) * STAMP_SLOTS];
        if (t[0] == 0) continue;
        ++n;
        sum[0] += (double)(t[1] - t[0]);
        sum[1] += (double)(t[2] - t[1]);
        sum[2] += (double)(t[3] - t[2]);
        sum[3] += (double)(t[3] - t[0]);
        chunks += (double)t[5];
        mx = std::max(mx, t[3] - t[0]);
        t0min = std::min(t0min, t[0]);
        t3max = std::max(t3max, t[3]);
      }
      if (n)
        fprintf(stderr, "[mmsbm stamp] %-6s waves %6lld  avg cycles: phase1 %8.0f  phase2 %8.0f  "
                "phase3 %8.0f  life %8.0f  (max %llu, first start -> last end %llu, chunks/wave %.1f)\n",
                names[k], n, sum[0] / n, sum[1] / n, sum[2] / n, sum[3] / n, mx, t3max - t0min,
                chunks / n);
    }
    HIP_TRY(hipMemset(c->stamp, 0, h.size() * 8));
  }
  return MMSBM_OK;
}

int mmsbm_accumulate(mmsbm_ctx* c, const double* theta, const double* pr, double* nth, double* S,
                     void* stream) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  int rc = check_ready(c);
  if (rc) return rc;
  if (!theta || !pr || !nth || !S) return fail(MMSBM_ERR_INVALID, "null pointer");
  DeviceGuard g(c->device);
  hipStream_t s = (hipStream_t)stream;
  const PassFn pass = pass_of(c);
  double* th = const_cast<double*>(theta);  // the passes only read theta / pr; fin in sums mode
  double* p = const_cast<double*>(pr);      // writes nth / S and leaves them untouched
  if (c->sets[MMSBM_SET_TRAIN].h.n_obs == 0) {  // a rank without train links adds zeros
    if (c->nth_add)  // the joint model's pair sums still count (fin would add them)
      HIP_TRY(hipMemcpyAsync(nth, c->nth_add, sizeof(double) * c->B * c->P * c->K,
                             hipMemcpyDeviceToDevice, s));
    else
      HIP_TRY(hipMemsetAsync(nth, 0, sizeof(double) * c->B * c->P * c->K, s));
    HIP_TRY(hipMemsetAsync(S, 0, sizeof(double) * c->B * c->R * c->K * c->K * c->K, s));
    return MMSBM_OK;
  }
  if ((rc = pass(c, PASS_A, MMSBM_SET_TRAIN, th, p, s))) return rc;
  if ((rc = pass(c, PASS_B, MMSBM_SET_TRAIN, th, p, s))) return rc;
  return fin_of(c)(c, true, th, p, nth, S, s);
}

int mmsbm_mstep(mmsbm_ctx* c, double* theta, double* pr, const double* nth, const double* S,
                void* stream) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  int rc = check_shape(c);
  if (rc) return rc;
  if (c->deg_host.empty()) return fail(MMSBM_ERR_INVALID, "train links / degree not set");
  if (c->zero_degree)
    return fail(MMSBM_ERR_ZERO_DEGREE, "a gene has no train link (float division by zero)");
  if (!theta || !pr || !nth || !S) return fail(MMSBM_ERR_INVALID, "null pointer");
  DeviceGuard g(c->device);
  return kTable[c->K - 1].mapply(c, theta, pr, nth, S, (hipStream_t)stream);
}

int mmsbm_loglik(mmsbm_ctx* c, int32_t which, const double* theta, const double* pr, double* out,
                 void* stream) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  int rc = check_shape(c);
  if (rc) return rc;
  if (which != MMSBM_SET_TRAIN && which != MMSBM_SET_TEST)
    return fail(MMSBM_ERR_INVALID, "which=%d", which);
  if (!c->ws || c->ws_bytes < (long long)ws_layout(c).total)
    return fail(MMSBM_ERR_INVALID, "workspace missing or too small (mmsbm_workspace_bytes)");
  if (!theta || !pr || !out) return fail(MMSBM_ERR_INVALID, "null pointer");
  DeviceGuard g(c->device);
  hipStream_t s = (hipStream_t)stream;
  const SetDev& sd = c->sets[which];
  if (!sd.present || sd.h.n_wg_a == 0) {
    HIP_TRY(hipMemsetAsync(out, 0, sizeof(double) * c->B, s));
    return MMSBM_OK;
  }
  if ((rc = pass_of(c)(c, PASS_LL, which, theta, pr, s))) return rc;
  reduce_kernel<<<nb_of(c), 256, 0, s>>>(c->partL, sd.h.n_wg_a, out);
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
  DeviceGuard g(c->device);
  return kTable[c->K - 1].predict(c, ids, n, theta, pr, out, (hipStream_t)stream);
}

// Joint digenic + trigenic iterations (include/mmsbm_pairs.h), all on `stream`: per iteration the
// pair launch (nth2 and the S2 partials), then pass A, pass B and fin, whose gene part adds nth2
// before the division by the joint counter and whose q cells sum the S2 partials and update qr.
int mmsbm_joint_iterate(mmsbm_ctx* c, mmsbm_pairs_ctx* pairs, double* theta, double* pr, double* qr,
                        double* nth2, int32_t n_iters, void* stream) {
  if (!c || !pairs) return fail(MMSBM_ERR_INVALID, "null context");
  int rc = check_ready(c);
  if (rc) return rc;
  int pK, pR, pB, pP;
  mmsbm_detail_pairs_shape(pairs, &pK, &pR, &pB, &pP);
  if (pK != c->K || pR != c->R || pB != c->B || pP != c->P)
    return fail(MMSBM_ERR_INVALID, "pair context shape differs from the triplet context");
  if (nb_of(c) != c->B) return fail(MMSBM_ERR_INVALID, "joint iterations run all B samples (mmsbm_set_active)");
  if (c->zero_degree)
    return fail(MMSBM_ERR_ZERO_DEGREE, "a gene has no train link (float division by zero)");
  if (!theta || !pr || !qr || !nth2) return fail(MMSBM_ERR_INVALID, "null pointer");
  if (n_iters < 0) return fail(MMSBM_ERR_INVALID, "n_iters < 0");
  DeviceGuard g(c->device);
  hipStream_t s = (hipStream_t)stream;
  const double* keep = c->nth_add;
  c->nth_add = nth2;
  c->q_out = qr;
  for (int it = 0; it < n_iters && rc == MMSBM_OK; ++it) {
    if ((rc = mmsbm_detail_pairs_estep(pairs, theta, qr, nth2, s, &c->q_part, &c->n_qwg))) break;
    rc = one_iteration(c, theta, pr, c->timing && it % c->timing_stride == 0, s);
  }
  c->nth_add = keep;
  c->q_part = nullptr;
  c->q_out = nullptr;
  c->n_qwg = 0;
  return rc;
}

int mmsbm_set_family(mmsbm_ctx* c, int32_t family) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  if (family != MMSBM_FAMILY_AUTO && family != MMSBM_FAMILY_SKU && family != MMSBM_FAMILY_SKY)
    return fail(MMSBM_ERR_INVALID, "family=%d", family);
  c->family = family;
  apply_family(c);
  ++c->gen;
  return MMSBM_OK;
}

int mmsbm_set_active(mmsbm_ctx* c, int32_t n) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  if (n < 0) return fail(MMSBM_ERR_INVALID, "active samples %d < 0", n);
  c->nact = n >= c->B ? 0 : n;
  ++c->gen;  // a captured graph bakes in the grids
  return MMSBM_OK;
}

int mmsbm_set_theta_addend(mmsbm_ctx* c, const double* nth_add) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  c->nth_add = nth_add;
  ++c->gen;
  return MMSBM_OK;
}

int mmsbm_plan_info(const mmsbm_ctx* c, int32_t which, int64_t* info) {
  if (!c || !info || (which != MMSBM_SET_TRAIN && which != MMSBM_SET_TEST))
    return fail(MMSBM_ERR_INVALID, "bad arguments");
  const auto& h = c->sets[which].h;
  info[0] = h.n_obs;
  info[1] = (int64_t)h.rows.size();
  info[2] = h.n_rows0;
  info[3] = h.n_wg_a;
  info[4] = h.n_wg_b;
  info[5] = h.n_sp;
  info[6] = h.n_prows;
  info[9] = h.prow_ptr.empty() ? 0 : h.prow_ptr[(size_t)h.R * (h.P + 1)];  // stream-0 partial rows
  info[7] = h.small ? h.gu : h.gmax;
  info[8] = h.small ? info[9] : (int64_t)h.vgenes.size();  // small-K: one V table per stream-0 stretch
  info[10] = h.small ? (c->sk_y ? 3 : c->sk_fused ? 2 : 1) : 0;
  info[11] = h.small ? h.n_units : (int64_t)(h.n_wg_a + h.n_wg_b) * h.nw;
  info[12] = c->sets[which].ncu;
  info[13] = c->sets[which].unit_target;
  info[14] = h.n_y;
  info[15] = h.small ? 0 : kTable[c->K - 1].gm_groups(c, std::max(h.n_sp, 1), c->sets[which].gm_q4);
  return MMSBM_OK;
}

int mmsbm_timing(mmsbm_ctx* c, int32_t stride) {
  if (!c) return fail(MMSBM_ERR_INVALID, "null context");
  c->timing = stride > 0;
  c->timing_stride = stride > 0 ? stride : 1;
  for (auto& n : c->nev) n = 0;
  return MMSBM_OK;
}

int mmsbm_time_kernel(mmsbm_ctx* c, int32_t kernel, double* theta, double* pr, int32_t n,
                      void* stream, double* avg_ms) {
  if (!c || !theta || !pr || !avg_ms || n < 1 || kernel < 0 || kernel > 2)
    return fail(MMSBM_ERR_INVALID, "bad arguments");
  int rc = check_ready(c);
  if (rc) return rc;
  DeviceGuard g(c->device);
  hipStream_t s = (hipStream_t)stream;
  const PassFn pass = pass_of(c);
  const FinFn fin = fin_of(c);
  hipEvent_t e0, e1;
  HIP_TRY(hipEventCreate(&e0));
  HIP_TRY(hipEventCreate(&e1));
  HIP_TRY(hipEventRecord(e0, s));
  // pass A / pass B only read theta / p; fin runs in sums mode into workspace scratch
  for (int i = 0; i < n && rc == MMSBM_OK; ++i)
    rc = kernel == 2 ? fin(c, true, theta, pr, c->nth_tmp, c->S_tmp, s)
                     : pass(c, kernel == 0 ? PASS_A : PASS_B, MMSBM_SET_TRAIN, theta, pr, s);
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
  DeviceGuard g(c->device);
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
