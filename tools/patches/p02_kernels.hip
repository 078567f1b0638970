// ------------------------------------------------------------------------------------------
// Fused E-step + S accumulation on FP64 MFMA (:987-1012), grid (G, B), block 64 * NW.
//
// v_mfma_f64_4x4x4f64 computes four independent 4x4x4 products ("blocks") per wave; with
// lane = 16 * hi + 4 * blk + lo its operands are A[blk][m = lo][k = hi], B[blk][k = hi][n = lo]
// and its result D[blk][m = hi][n = lo] (probed: tools/micro/mfma_layout.hip).  A wave takes
// 16 observations at a time (a "group"); observation oA = lane & 15 feeds the A side, the
// result rows belong to observation oD = 4 * blk + hi.  Per group:
//   images    th_i / th_j / th_k rows of the 16 observations in a per-wave LDS image (double
//             buffered), from 9 global loads per lane issued one group ahead.
//   U-phase   U[o][a][b] = sum_g p_r[a][b][g] th_k[o][g]: per (a, b-block) tile 1 MFMA per
//             g-block (A = th_k of oA, B = p_r, the same in all four blocks).  Lane (oD, lo)
//             keeps b = 4 bb + lo, so Z[b] = sum_a th_i[a] U[a][b] is complete in the lane and
//             Y[a] = sum_b th_j[b] U[a][b] needs one quad butterfly.  d = eps + sum_b th_j Z.
//   W-phase   W0[o][g] = sum_(a,b) th_i[a] th_j[b] p_r[a][b][g]: k over the K^2 cells, the A
//             operand formed from the images (independent of U, so the two interleave).
//   S-phase   S[(a,b)][g] += sum_o th_i[a] th_j[b] (c th_k[g]): k over the group's
//             observations, c folded into the B operand; run one group late (software
//             pipelined under the next group's U/W MFMAs), accumulators in registers across all
//             the wave's groups.
// Contributions c Y, c Z, c W0 go to the observation's three gene-CSR rows (M2 multiplies by
// theta and divides by deg).  At the end the NW waves' S accumulators are summed in LDS in a
// fixed order: one partial S row per workgroup (each workgroup owns one rating).  Every sum
// has a fixed order: bitwise reproducible.
// ------------------------------------------------------------------------------------------
constexpr int XG = 16;  // observations per wave group

// RP = p_r's U-phase fragments register-resident: one wave per SIMD (4 waves, up to 512
// registers), otherwise two waves per SIMD reading them from LDS.
template <int K, bool RP>
struct XPlan {
  static constexpr int NG = (K + 3) / 4;      // 4-wide blocks of a / b / g
  static constexpr int KP = 4 * NG;
  static constexpr int K2 = K * K, K3 = K * K * K;
  static constexpr int NC = (K2 + 3) / 4;     // W-phase k-steps over the (a, b) cells
  static constexpr int NT4 = (K2 + 15) / 16;  // S-phase 16-cell tiles
  static constexpr int NSU = 4 * NT4;         // S-phase units (k-step, tile) per group
  static constexpr int SACC = NT4 * NG;       // S accumulators per lane
  static constexpr int P_DBL = K * KP * KP;   // p_r image [a][b][g], b and g zero padded
  static constexpr int IS = KP + 1;           // theta image row stride (odd: conflict-free)
  static constexpr int IMG1 = 3 * XG * IS;    // th_i / th_j / th_k rows of one group
  static constexpr int WAVE_DBL = 2 * IMG1;   // double buffered: S reads the previous group's
  static constexpr int RED_DBL = SACC * 64;   // the wave's S accumulators in the epilogue
  static constexpr int SLOT = WAVE_DBL > RED_DBL ? WAVE_DBL : RED_DBL;
  static constexpr int NW = RP ? 4 : 8;
  static constexpr int WPE = RP ? 1 : 2;      // waves per SIMD the allocator plans for
  static constexpr int NT = 64 * NW;
  static constexpr int LDS_BYTES = (P_DBL + NW * SLOT) * 8;
  static constexpr bool ON = K >= 2 && K <= 12;
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

// Optional per-wave phase clock (MMSBM_TRACE, measurement only): [wave][16] cycle sums.
struct XTrace {
  unsigned long long* out;
  __device__ __forceinline__ unsigned long long now() const { return out ? clock64() : 0ull; }
};

// S-phase units [U0, U1) of one group: unit = (k-step s4, 16-cell tile t); A = th_i th_j of
// observation o = 4 s4 + hi at cell 16 t + oA (cells past K^2 feed discarded S entries), B =
// c_o th_k[o][4 u + lo] (reloaded at each k-step's first unit).
template <int K, bool RP, int U0, int U1>
__device__ __forceinline__ void s_units(double (&sacc)[XPlan<K, RP>::NT4][XPlan<K, RP>::NG],
                                        double (&bS)[XPlan<K, RP>::NG], const double* TIp,
                                        const double* TJp, const double* TKp, double cprev,
                                        int hi, int lo, int oA) {
  using X = XPlan<K, RP>;
  constexpr int NG = X::NG, NT4 = X::NT4, IS = X::IS, K2 = X::K2;
#pragma unroll
  for (int su = U0; su < U1; ++su) {
    const int s4 = su / NT4, t = su % NT4;
    const int o = 4 * s4 + hi;
    if (t == 0) {
      const double co = __shfl(cprev, 16 * (o & 3) + 4 * (o >> 2), 64);
#pragma unroll
      for (int u = 0; u < NG; ++u) bS[u] = co * TKp[o * IS + 4 * u + lo];
    }
    const int cell = 16 * t + oA;
    const int cc = cell < K2 ? cell : K2 - 1;
    const double av = TIp[o * IS + cc / K] * TJp[o * IS + cc % K];
#pragma unroll
    for (int u = 0; u < NG; ++u) sacc[t][u] = mfma4(av, bS[u], sacc[t][u]);
  }
}

// One a-step of the U-phase with its share of the W-phase and of the previous group's S-phase.
template <int K, bool RP, int A>
__device__ __forceinline__ void uws_step(
    const double* Pl, const double (&pU)[RP ? K : 1][XPlan<K, RP>::NG][XPlan<K, RP>::NG],
    const double (&aU)[XPlan<K, RP>::NG], const double (&tjD)[XPlan<K, RP>::NG],
    const double* TIc, const double* TJc, const double* TIp, const double* TJp,
    const double* TKp, double cprev, double (&yp)[K], double (&zp)[XPlan<K, RP>::NG],
    double (&wacc)[XPlan<K, RP>::NG], double (&sacc)[XPlan<K, RP>::NT4][XPlan<K, RP>::NG],
    double (&bS)[XPlan<K, RP>::NG], int hi, int lo, int oA, int oD) {
  using X = XPlan<K, RP>;
  constexpr int NG = X::NG, KP = X::KP, K2 = X::K2, NC = X::NC, IS = X::IS, NSU = X::NSU;
  double acc[NG];
#pragma unroll
  for (int bb = 0; bb < NG; ++bb) acc[bb] = 0.0;
#pragma unroll
  for (int s = 0; s < NG; ++s)
#pragma unroll
    for (int bb = 0; bb < NG; ++bb) {
      const double f = RP ? pU[RP ? A : 0][bb][s] : Pl[(A * KP + 4 * bb + lo) * KP + 4 * s + hi];
      acc[bb] = mfma4(aU[s], f, acc[bb]);
    }
#pragma unroll
  for (int s = A * NC / K; s < (A + 1) * NC / K; ++s) {  // this a's share of the W steps
    const int cell = 4 * s + hi;
    const int cc = cell < K2 ? cell : K2 - 1;
    const int ca = cc / K, cbq = cc % K;
    const double av = cell < K2 ? TIc[oA * IS + ca] * TJc[oA * IS + cbq] : 0.0;
    const double* pb = Pl + (ca * KP + cbq) * KP + lo;
#pragma unroll
    for (int u = 0; u < NG; ++u) wacc[u] = mfma4(av, pb[4 * u], wacc[u]);
  }
  s_units<K, RP, A * NSU / K, (A + 1) * NSU / K>(sacc, bS, TIp, TJp, TKp, cprev, hi, lo, oA);
  const double ta = TIc[oD * IS + A];
  double y = 0.0;
#pragma unroll
  for (int bb = 0; bb < NG; ++bb) {
    y = fma(tjD[bb], acc[bb], y);
    zp[bb] = fma(ta, acc[bb], zp[bb]);
  }
  yp[A] = y;
}

template <int K, bool RP, int... As>
__device__ __forceinline__ void uws_all(
    std::integer_sequence<int, As...>, const double* Pl,
    const double (&pU)[RP ? K : 1][XPlan<K, RP>::NG][XPlan<K, RP>::NG],
    const double (&aU)[XPlan<K, RP>::NG], const double (&tjD)[XPlan<K, RP>::NG],
    const double* TIc, const double* TJc, const double* TIp, const double* TJp,
    const double* TKp, double cprev, double (&yp)[K], double (&zp)[XPlan<K, RP>::NG],
    double (&wacc)[XPlan<K, RP>::NG], double (&sacc)[XPlan<K, RP>::NT4][XPlan<K, RP>::NG],
    double (&bS)[XPlan<K, RP>::NG], int hi, int lo, int oA, int oD) {
  (uws_step<K, RP, As>(Pl, pU, aU, tjD, TIc, TJc, TIp, TJp, TKp, cprev, yp, zp, wacc, sacc, bS,
                       hi, lo, oA, oD),
   ...);
}

template <int K, bool RP>
__global__ __launch_bounds__((XPlan<K, RP>::NT))
__attribute__((amdgpu_waves_per_eu(XPlan<K, RP>::WPE, XPlan<K, RP>::WPE))) void emx_kernel(
    const int4* __restrict__ obs, const int4* __restrict__ pos, const double* __restrict__ theta,
    const double* __restrict__ pr, double* __restrict__ contrib, double* __restrict__ partS,
    SRows rg, int P, int R, long long nnz, int G, double eps, XTrace tr) {
  using X = XPlan<K, RP>;
  constexpr int NG = X::NG, KP = X::KP, K2 = X::K2, K3 = X::K3, NT4 = X::NT4, NSU = X::NSU;
  constexpr int IS = X::IS, NW = X::NW, NT = X::NT, SACC = X::SACC;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* Pl = smem;  // [K][KP][KP]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  double* IMG = smem + X::P_DBL + wv * X::SLOT;  // [2][3][XG][IS] theta images
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
  }

  for (int idx = tid; idx < X::P_DBL; idx += NT) {
    const int g = idx % KP, bq = (idx / KP) % KP, a = idx / (KP * KP);
    Pl[idx] = (g < K && bq < K) ? p[(a * K + bq) * K + g] : 0.0;
  }
  // both image buffers start at 0: the first group's pipelined S-phase adds exact zeros
  for (int idx = lane; idx < X::WAVE_DBL; idx += 64) IMG[idx] = 0.0;
  __syncthreads();
  double pU[RP ? K : 1][NG][NG];  // U-phase B fragments, register-resident when RP
  if constexpr (RP) {
#pragma unroll
    for (int a = 0; a < K; ++a)
#pragma unroll
      for (int bb = 0; bb < NG; ++bb)
#pragma unroll
        for (int s = 0; s < NG; ++s) pU[a][bb][s] = Pl[(a * KP + 4 * bb + lo) * KP + 4 * s + hi];
  }
  unsigned long long t0 = tr.now();
  tph[0] = t0 - t_start;

  double sacc[NT4][NG];
#pragma unroll
  for (int t = 0; t < NT4; ++t)
#pragma unroll
    for (int u = 0; u < NG; ++u) sacc[t][u] = 0.0;
  double bS[NG];
  double cprev = 0.0;  // c of the previous group's observation oD
  int cur = 0, ngrp = 0;

  while (grp < g1) {
    ++ngrp;
    double* TIc = IMG + cur * X::IMG1;
    double* TJc = TIc + XG * IS;
    double* TKc = TJc + XG * IS;
    const double* TIp = IMG + (cur ^ 1) * X::IMG1;
    const double* TJp = TIp + XG * IS;
    const double* TKp = TJp + XG * IS;
    // ---- theta images of this group, then the next group's records
#pragma unroll
    for (int s = 0; s < NG; ++s) {
      TKc[oA * IS + 4 * s + hi] = aU[s];
      TJc[oD * IS + 4 * s + lo] = tjD[s];
      TIc[oD * IS + 4 * s + lo] = tiD4[s];
    }
    const int gn = grp + NW;
    {  // past the end the current group is re-read (branch-free, unused)
      const size_t r1 = (size_t)(gn < g1 ? gn : grp) * XG;
      nA = obs[r1 + oA];
      nD = obs[r1 + oD];
      nQ = pos[r1 + oD];
    }
    wave_lds_sync();
    unsigned long long t1 = tr.now();
    tph[2] += t1 - t0;

    // ---- U-phase + W-phase of this group, S-phase of the previous one, interleaved per a
    double yp[K], zp[NG], wacc[NG];
#pragma unroll
    for (int bb = 0; bb < NG; ++bb) {
      zp[bb] = 0.0;
      wacc[bb] = 0.0;
    }
    uws_all<K, RP>(std::make_integer_sequence<int, K>{}, Pl, pU, aU, tjD, TIc, TJc, TIp, TJp, TKp,
                   cprev, yp, zp, wacc, sacc, bS, hi, lo, oA, oD);
    unsigned long long t2 = tr.now();
    tph[1] += t2 - t1;
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
    unsigned long long t3 = tr.now();
    tph[3] += t3 - t2;

    // ---- contributions of observation oD: entries 4 j + lo of its three gene-CSR rows
    {
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
        (v < K ? rk : trash)[vs] = c * wacc[j];
      }
    }
    unsigned long long t4 = tr.now();
    tph[4] += t4 - t3;

    cprev = c;
    cur ^= 1;
    wave_lds_sync();  // this group's image reads are ordered before the next group's writes
    eA = nA;
    eD = nD;
    qD = nQ;
#pragma unroll
    for (int s = 0; s < NG; ++s) {
      aU[s] = aU2[s];
      tjD[s] = tjD2[s];
      tiD4[s] = tiD42[s];
    }
    grp = gn;
    t0 = tr.now();
    tph[5] += t0 - t4;
  }
  if (ngrp > 0) {  // drain: the last group's S-phase
    const double* TIp = IMG + (cur ^ 1) * X::IMG1;
    s_units<K, RP, 0, NSU>(sacc, bS, TIp, TIp + XG * IS, TIp + 2 * XG * IS, cprev, hi, lo, oA);
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
  if (tr.out && lane == 0) {
    const unsigned long long t_end = tr.now();
    unsigned long long* o = tr.out + ((size_t)(b * gridDim.x + w) * NW + wv) * 16;
    for (int q = 0; q < 6; ++q) o[q] = tph[q];
    o[6] = t_end - t0;
    o[7] = (unsigned long long)ngrp;
    o[8] = t_end - t_start;
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
                                                 double eps, int ablate) {
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
      double* row = theta + (size_t)b * P * K + (size_t)g * K;
      row[tid] = row[tid] * sum / (double)deg[g];
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
  if (sl == 0 && cell < K3) {
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

