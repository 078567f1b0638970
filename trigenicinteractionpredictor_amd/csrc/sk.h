// sk.h — the small-K (K <= 12) EM kernels of mmsbm.hip: one EM iteration
// (src/TrigenicInteractionPredictor.py make_iteration :984-1043) as sk_pass_kernel<K, SK_A>,
// sk_pass_kernel<K, SK_B> and sk_fin_kernel<K>; compute_likelihood (:952-974) as
// sk_pass_kernel<K, SK_LL> + reduce_kernel.  Same pivot-run algebra as the large-K kernels
// (mmsbm.hip header), laid out for latency instead of throughput:
//
//  * one unit (<= GUK gene stretches, <= LCAP_SK chunks of 4 observations) per wave, and no
//    workgroup barrier between a wave's start and its end: the wave stages its unit's records in
//    its own LDS with one coalesced load, computes the V tables of its own <= 4 pivot genes
//    (one MFMA per (a tile, cell group), p_r staged once per workgroup), and gathers the theta
//    values of every chunk straight into the registers its MFMA operands need, SKD chunks ahead;
//  * a gene stretch's M row (K x K) never leaves the wave: at the unit's end the wave contracts
//    its <= 4 rows with p (X, K values per row, one MFMA per cell step) and, on stream 0, forms
//    its share of S = sum_g theta_g (x) M0_g in registers; a workgroup adds its 8 waves' S in a
//    fixed order and writes ONE K^3 partial;
//  * pass A stores each observation's c = n / d at its stream-1 and stream-2 rows (plan row12),
//    so pass B reads c coalesced with its records;
//  * fin sums the X partials per gene (theta update) and the S partials per cell (p update).
// Bytes per iteration: records + c + X partials (K per partial row) + S partials (K^3 per stream-0
// workgroup), against K^2 per partial row written and read back by the large-K path.  These are
// plain stores: the scattered 8-byte c / X writes as write-through (sc1) stores cost 6-10 us per
// pass at fold0 (each lane a separate fabric write), the kernel-boundary write-back of the few MB
// of dirty lines far less (profiles/r03_wt_ab.txt).
//
// MFMA lane maps as in mmsbm.hip: v_mfma_f64_4x4x4f64 (lane = 16 hi + 4 blk + lo) takes
// A[blk][m = lo][k = hi], B[blk][k = hi][n = lo] and gives D[blk][m = hi][n = lo];
// v_mfma_f64_16x16x4f64 takes A[m = l & 15][k = l >> 4], B[k = l >> 4][n = l & 15] and gives
// D[m = (l >> 4) + 4 i][n = l & 15] in element i.

// SK_U (the fused E-step): every stream in ONE launch, each observation's d (and c = n / d) computed
// by the wave of every stream it sits in (stream s contracts V^s_g, the lattice with the pivot slot
// s summed against theta_g), so nothing waits for another workgroup: pass A's c stores, pass B's c
// loads and one dependent launch per iteration go away for 2x the Z / d / c work.
enum { SK_A = 0, SK_LL = 1, SK_B = 2, SK_U = 3 };
#ifndef MMSBM_SK_TRSWZ
#define MMSBM_SK_TRSWZ 1  // the Z operand transpose with a bank swizzle (r03u A/B: 38.5k vs 38.1k iter/s)
#endif
#ifndef MMSBM_SK_SCOOP
#define MMSBM_SK_SCOOP 1  // the workgroup's S partial in one cooperative pass (0: per-wave shares + tree)
#endif
#ifndef MMSBM_SK_MRED
#define MMSBM_SK_MRED 0  // 1: d's sum over b on MFMA, four chunks at a time (measured slower than the DPP row sum)
#endif
#ifndef MMSBM_SK_PVS
#define MMSBM_SK_PVS 1  // P^s rows at an odd stride (0: K^2, round 3), see SKT::PVS
#endif
#ifndef MMSBM_SK_GHOIST
#define MMSBM_SK_GHOIST 0  // 1: the first block's theta gathers before the V tables (after the barrier)
#endif

constexpr int LC = mmsbm_plan::SK_BLOCK;          // chunks of one block (gathered at once)
constexpr int SK_ROWS = 4 * mmsbm_plan::SK_BLOCK;  // records staged per wave (one block, one per lane)
static_assert(SK_ROWS == 64, "one record per lane");

template <int K>
struct SKT {
  static constexpr int NG = (K + 3) / 4;          // 4-wide tiles of one K axis (<= 3)
  static constexpr int K2 = K * K, K3 = K * K * K;
  static constexpr int NCT = (K2 + 3) / 4;        // 4-cell tiles of a dense K x K row
  static constexpr int NCG = (NCT + 3) / 4;       // groups of 4 cell tiles (one MFMA, 4 blocks)
  static constexpr int SLOT = 4 * NCT;            // doubles per stretch slot (V table, then M row)
  // P^s_r staged per workgroup, [z][cell] rows of PVS words (zero past K^2 and past the last row,
  // up to the last word the unguarded V-operand reads touch: rows a >= K of the 4-wide a tiles,
  // cells up to 16 NCG).  The X contraction's B reads take 16 rows z at once, paired into
  // ds_read2_b64 (16-lane groups, bank (a/4) mod 32): at the K^2 stride (100 at K = 10) rows
  // z, z + 4, z + 8 shared banks, an odd stride puts the 16 rows on distinct banks.
  static constexpr int PVS = MMSBM_SK_PVS ? (K2 | 1) : K2;
  static constexpr int PVR = (K - 1) * PVS + 16 * NCG;  // (V-operand rows a >= K read row K - 1)
  static constexpr int PSD = ((PVR > K * PVS ? PVR : K * PVS) + 1) & ~1;
  static constexpr int GUK = mmsbm_plan::sk_gu(K);  // stretches per unit (slots per wave): 8 or 4
  static constexpr int NT2 = GUK / 4;                // 4-row MFMA tiles of the unit's stretches
  static constexpr int THL = GUK * 4 * NG;          // the unit's pivot-gene theta rows (S operand)
  // per wave: slots, the block's (u, v) gene pairs, pivot rows, aux (row12 / c), two transposes,
  // d / c words
  static constexpr int WAVE = GUK * SLOT + SK_ROWS + THL + SK_ROWS + 2 * 64 + SK_ROWS;
  static constexpr int WAVE_B = WAVE - 2 * 64 - SK_ROWS;  // pass B: c arrives in aux
  static constexpr int LDS_B = (PSD + NW * WAVE_B) * 8;
  static constexpr int WAVE_U = WAVE - SK_ROWS;   // fused: no row12 / c staging
  static constexpr int NPV = (PSD + NT - 1) / NT; // staged words per thread
  static constexpr int LDS_U = (PSD + NW * WAVE_U) * 8;
  static constexpr int NS = NG * NCG;             // S accumulators per lane
  static constexpr int LDS = (PSD + NW * WAVE) * 8;
  static_assert(K <= 12, "small-K kernels: K <= 12");
  static_assert(4 * NS * 64 <= PSD + NW * WAVE_U, "S reduction buffer over the LDS");
  static_assert(LDS_U <= 80 * 1024, "two fused / likelihood workgroups per CU");
  static_assert(LDS <= 160 * 1024, "pass A LDS");
  static_assert(GUK % 4 == 0 && GUK <= mmsbm_plan::GU, "stretch tiles");

  static_assert(SLOT >= 4 * NCT, "slot holds a V table / M row");
  // the unguarded V / M reads stay inside the slots and the records (finite words)
  static_assert((GUK - 1) * SLOT + 15 * K + 4 * NG <= GUK * SLOT + SK_ROWS + THL,
                "V reads past the wave's slots and records");
  static_assert(16 * NCG <= SLOT + SK_ROWS + THL, "S operand reads past the slots and records");
};

// p index of P^s[z][cell] (s = the pivot slot z sits in; cell = x K + y over the two other
// slots u, v in order): s = 0 p[z][x][y], s = 1 p[x][z][y], s = 2 p[x][y][z]
template <int K>
__device__ __forceinline__ int sk_pidx(int s, int z, int x, int y) {
  return s == 0 ? (z * K + x) * K + y : s == 1 ? (x * K + z) * K + y : (x * K + y) * K + z;
}

struct SkSec {  // workgroup sections of a small-K plan (Plan::sk_wg_end)
  int wg_end[3 * MAX_R];
};

// grid (the group's workgroups, B), block 512; group 0 (SK_A, SK_LL) = stream 0, group 1 (SK_B) =
// streams 1 and 2; SK_U: both groups, group 0's n_wg workgroups first, then group 1's (urec1,
// udesc1, L1).  Wave wv of workgroup w of a group owns unit slot w NW + wv (Plan::sk_*).
template <int K, int MODE>
// (4 waves per SIMD: two workgroups per CU, the LDS budget of the fused launch)
__global__ __launch_bounds__(NT, 4) void sk_pass_kernel(
    const int4* __restrict__ urec, const int* __restrict__ udesc, const int2* __restrict__ urow12,
    const double* __restrict__ theta, const double* __restrict__ pr, double* __restrict__ cB,
    double* __restrict__ xpart, double* __restrict__ spart, double* __restrict__ partL, SkSec sec,
    int wg_base, int L, int P, int R, long long n_cb, long long n_prows, int n_wg,
    double eps, const int4* __restrict__ urec1, const int* __restrict__ udesc1, int L1) {
  using T = SKT<K>;
  constexpr int NG = T::NG, K2 = T::K2, K3 = T::K3, NCT = T::NCT, NCG = T::NCG, SLOT = T::SLOT;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 4, blk = (lane >> 2) & 3, lo = lane & 3, col = lane & 15;
  const int wx = blockIdx.x, b = blockIdx.y;
  const bool g1 = MODE == SK_U && wx >= n_wg;  // SK_U: a group-1 (stream 1 / 2) workgroup
  const int w = g1 ? wx - n_wg : wx;            // workgroup within its group
  if (g1) {
    urec = urec1;
    udesc = udesc1;
    L = L1;
  }
  int sr = 0;  // this workgroup's (stream, rating) section, from the launch arguments alone
#pragma unroll
  for (int i = 0; i < 3 * MAX_R - 1; ++i)  // (constant indices: the argument array stays in SGPRs)
    if (i + 1 < 3 * R && wg_base + wx >= sec.wg_end[i]) sr = i + 1;
  const int s = __builtin_amdgcn_readfirstlane(sr / R), r = __builtin_amdgcn_readfirstlane(sr % R);
  const double* __restrict__ th = theta + (size_t)b * P * K;
  const double* __restrict__ p = pr + ((size_t)b * R + r) * K3;
  double* PV = smem;  // P^s_r[z][cell] (cell = x K + y over the u, v slots), rows of SKT::PVS words
  double* wl = smem + T::PSD + wv * (MODE == SK_B ? T::WAVE_B : MODE == SK_U ? T::WAVE_U : T::WAVE);
  constexpr int GUK = T::GUK, NT2 = T::NT2;
  double* MSl = wl;                                                 // GUK slots: V, then M
  int2* REC = reinterpret_cast<int2*>(wl + GUK * SLOT);             // the block's (u, v) genes
  double* THl = wl + GUK * SLOT + SK_ROWS;                          // pivot theta rows [GUK][4 NG]
  double* AUX = THl + T::THL;                                       // row12 (A) / c (B)
  double* TRl = MODE == SK_U ? AUX : AUX + SK_ROWS;                 // Z operand transpose
  double* DL = TRl + 2 * 64;                                        // d, then c, per observation
  double* __restrict__ cBb = cB + (size_t)b * n_cb;
  double* __restrict__ xb = xpart + (size_t)b * n_prows * K;
  Stamp st_{};
  st_.mark(0);
#ifdef MMSBM_SK_EXIT  // measurement builds: leave after phase MMSBM_SK_EXIT (0 = at once)
  if (MMSBM_SK_EXIT == 0 && b >= 0) return;
#endif

  // P^s_r once per workgroup (every unit of a workgroup has its stream and rating): its loads go
  // out first, so the barrier that publishes it (before the V tables) waits about one round trip.
  double pvv[T::NPV];
#pragma unroll
  for (int i = 0; i < T::NPV; ++i) {
    const int e = tid + NT * i, z = e / T::PVS, cell = e % T::PVS;
    const bool ok = z < K && cell < K2;
    const int x = ok ? cell / K : 0, y = ok ? cell % K : 0;
    const double v = p[ok ? sk_pidx<K>(s, z, x, y) : 0];
    pvv[i] = ok ? v : 0.0;
  }

  // One slot's descriptor and pivot-gene theta, with its first block's records (+ row12 / c).
  // A unit of c1 chunks runs in blocks of LC chunks (SK_ROWS records, one per lane); the next
  // block's records are loaded while the current one computes.
  const long long slot = (long long)w * NW + wv;
  struct Unit {
    int nst, c1, ds[GUK], prow[NT2];
    double tv[NT2][NG];     // theta_{gene 4 tt + lo}[4 as + hi] (A of V; zero past nst and K)
  };
  struct Blk {
    int4 rv;
    int2 r12;
    double cv;
  };
  auto load_block = [&](int bi, Blk& bk) {  // (rows past the slot's capacity: its last, valid row)
    const int idx = SK_ROWS * bi + lane;
    const long long row = slot * 4 * L + (idx < 4 * L ? idx : 4 * L - 1);
    bk.rv = urec[row];
    if constexpr (MODE == SK_A) bk.r12 = urow12[row];
    if constexpr (MODE == SK_B) bk.cv = cBb[row];
  };
  int wlane = 0;  // the count n of this lane's observation in the current block
  auto stage_block = [&](const Blk& bk) {
    REC[lane] = make_int2(bk.rv.x, bk.rv.y);
    wlane = bk.rv.w;
    if constexpr (MODE == SK_A) reinterpret_cast<int2*>(AUX)[lane] = bk.r12;
    if constexpr (MODE == SK_B) AUX[lane] = bk.cv;
  };
  auto load_unit = [&](Unit& un) {
    const int* __restrict__ d = udesc + slot * mmsbm_plan::UD;
    un.nst = __builtin_amdgcn_readfirstlane(d[mmsbm_plan::D_NST]);  // wave-uniform (scalar control flow)
    un.c1 = __builtin_amdgcn_readfirstlane(d[mmsbm_plan::D_END]);
#pragma unroll
    for (int t = 0; t < GUK; ++t) un.ds[t] = __builtin_amdgcn_readfirstlane(d[t]);
#pragma unroll
    for (int tt = 0; tt < NT2; ++tt) un.prow[tt] = d[mmsbm_plan::D_PROW + 4 * tt + hi];
    if constexpr (MODE != SK_B) {
#pragma unroll
      for (int tt = 0; tt < NT2; ++tt) {
        const int glo = d[mmsbm_plan::D_GENE + 4 * tt + lo];
#pragma unroll
        for (int as = 0; as < NG; ++as) {
          const int a1 = 4 * as + hi;
          const double v1 = th[(size_t)glo * K + (a1 < K ? a1 : 0)];
          un.tv[tt][as] = (4 * tt + lo < un.nst && a1 < K) ? v1 : 0.0;
        }
      }
    }
  };
  Blk bk;
  load_block(0, bk);  // (the block loads do not wait for the descriptor)
  Unit un;
  load_unit(un);

#pragma unroll
  for (int i = 0; i < T::NPV; ++i)
    if (tid + NT * i < T::PSD) PV[tid + NT * i] = pvv[i];
  stage_block(bk);  // the first block's records (and row12 / c) into this wave's LDS
  // pass B reads P^s only in the X contraction, behind the barrier after its chunk loop; the
  // passes that form V tables publish it here
  if constexpr (MODE == SK_B) wave_lds_sync();
  else __syncthreads();
  st_.mark(6);
#ifdef MMSBM_SK_EXIT
  if (MMSBM_SK_EXIT == 1 && b >= 0) return;
#endif

  double sacc[NG][NCG];  // SK_A: this wave's share of S_r[a][cell], a = 4 at + hi
#pragma unroll
  for (int at = 0; at < NG; ++at)
#pragma unroll
    for (int cg = 0; cg < NCG; ++cg) sacc[at][cg] = 0.0;
  double ll = 0.0;

  if (un.nst > 0) {  // an empty slot only joins the workgroup's barriers
    const int nst = un.nst;
    const int c0 = 0, c1 = un.c1;
    st_.t[5] = (unsigned long long)(c1 - c0);
    st_.t[4] = (unsigned long long)nst;
    const auto& ds = un.ds;
    const int2* __restrict__ rec = REC;
    const int colc = col < K ? col : K - 1;
    const unsigned cb = (unsigned)colc * 8u;
    const bool kcol = col < K;
    const auto& tv = un.tv;  // (array references: the indices stay compile-time constants)
    // ---- theta gathers: every value of a block at once, straight into the registers of the
    // MFMA operands (lane (obs hi, col): theta_u and theta_v of its observation, column col);
    // columns col >= K are zeroed where a product needs it (the Z operand and d), at first use,
    // so no select waits for a load here
    double ga[LC], gv[LC];
    auto gather = [&](int nb) {
      // Every chunk of the block loads, a short block too (chunks past the unit's end read the
      // clamped records load_block staged: valid genes, values never used): with no branch between
      // them the 16 record reads go out together and each chunk waits for its own two loads only
      // (round 6: per-chunk guards made the compiler wait for every load of the block before the
      // first chunk, and read the records one LDS round trip at a time)
      (void)nb;
      int2 rh[LC];
#pragma unroll
      for (int i = 0; i < LC; ++i) rh[i] = rec[i * 4 + hi];  // (u gene, v gene): make_slots orders them
#pragma unroll
      for (int i = 0; i < LC; ++i) {
        // (32-bit byte offsets from the sample's theta base: one 24-bit multiply-add per address;
        // col >= K reads a finite copy of column K - 1)
        const char* __restrict__ thb = reinterpret_cast<const char*>(th);
        ga[i] = *reinterpret_cast<const double*>(thb + (__umul24((unsigned)rh[i].x, K * 8u) + cb));
        gv[i] = *reinterpret_cast<const double*>(thb + (__umul24((unsigned)rh[i].y, K * 8u) + cb));
      }
    };
    if constexpr (MMSBM_SK_GHOIST) gather(c1 < LC ? c1 : LC);  // (in flight during the V tables)
    if constexpr (MODE != SK_B) {
      // ---- V_g[cell] = sum_a theta_g[a] P^s[a][cell] for the unit's genes (m = gene, k = a, B
      // from the staged lattice: rows a >= K meet zero theta, words past K^3 are zero), into slot g
      // of the wave's LDS (cell = b K + h).  Every word of the GU slots is written (zero past K^2
      // and for absent stretches), so the unguarded V / M reads below see finite values.  The
      // unit's pivot theta rows go to THl (the S contraction's A operand).
#pragma unroll
      for (int tt = 0; tt < NT2; ++tt) {
        const bool live = tt == 0 || nst > 4 * tt;  // (uniform) a tile without stretches: zeros
#pragma unroll
        for (int cg = 0; cg < NCG; ++cg) {
          const int cell = 4 * (4 * cg + blk) + lo;
          double v = 0.0;
          if (live) {
#pragma unroll
            for (int as = 0; as < NG; ++as)  // (rows a >= K: zero theta times row K - 1)
              v = mfma4(tv[tt][as], PV[(4 * as + hi < K ? 4 * as + hi : K - 1) * T::PVS + cell], v);
          }
          if (cell < SLOT) MSl[(4 * tt + hi) * SLOT + cell] = cell < K2 ? v : 0.0;
        }
#pragma unroll
        for (int as = 0; as < NG; ++as)
          if (blk == 0) THl[(4 * tt + lo) * 4 * NG + 4 * as + hi] = tv[tt][as];
        __builtin_amdgcn_sched_barrier(0);  // (one tile's operand reads in flight at a time)
      }
    } else {
      // pass B forms no V tables: the slots' words past each M row stay finite (zero)
#pragma unroll
      for (int i = 0; i < (GUK * SLOT + 63) / 64; ++i)
        if (lane + 64 * i < GUK * SLOT) MSl[lane + 64 * i] = 0.0;
#pragma unroll
      for (int i = 0; i < (T::THL + 63) / 64; ++i)
        if (lane + 64 * i < T::THL) THl[lane + 64 * i] = 0.0;
    }
    if constexpr (MODE != SK_B) TRl[64 + lane] = 0.0;  // (load_v's zero words)
    wave_lds_sync();
    st_.mark(1);

    const double* __restrict__ vrow = MSl + col * K + hi;
    const double* __restrict__ cw = MODE == SK_B ? AUX : DL;
    d4v m16 = d4v{0.0, 0.0, 0.0, 0.0};  // the running stretch's M (persists across blocks)
    int t = 0;                          // the running stretch (phase 2)
    double vb[NG];  // B of Z: V_vt[b = col][h = 4 hs + hi] of the running stretch (phase 1)
    // The V operand's LDS word per (lane, h tile): the running stretch's slot where b = col < K and
    // h = 4 hs + hi < K, else a zeroed word (the second transpose buffer, TRl + 64, zeroed before
    // the V tables and never written after), so the loads need neither a mask nor a select: plain
    // ds_reads issued at a stretch change and first waited on by the next chunk's MFMA (round 6:
    // the masked form made each stretch change wait an LDS round trip inside the chunk chain)
    int voff[NG], vstr[NG];
#pragma unroll
    for (int hs = 0; hs < NG; ++hs) {
      const bool ok = kcol && 4 * hs + hi < K;
      voff[hs] = ok ? (int)(MSl - smem) + col * K + hi + 4 * hs : (int)(TRl + 64 - smem);
      vstr[hs] = ok ? SLOT : 0;
    }
    auto load_v = [&](int tv_) {
#pragma unroll
      for (int hs = 0; hs < NG; ++hs) vb[hs] = smem[voff[hs] + tv_ * vstr[hs]];
    };
    int vt = 0;  // the running stretch (phase 1: its V operand)
    if constexpr (MODE != SK_B) load_v(0);
    for (int b0 = 0; b0 < c1; b0 += LC) {  // (uniform; one block for units of <= LC chunks)
      const int nb = c1 - b0;               // chunks left (this block: min(nb, LC))
      // bit q: chunk b0 + q ends a stretch other than the unit's last (one scalar test per chunk
      // instead of tracking the next stretch's end through a select chain over ds[]; round 6)
      unsigned endm = 0;
#pragma unroll
      for (int i = 1; i < GUK; ++i) {
        const int e = ds[i] - 1 - b0;
        if (i < nst && e >= 0 && e < LC) endm |= 1u << e;
      }
      endm = __builtin_amdgcn_readfirstlane(endm);
      if (b0 > 0) {  // this block's records (loaded during the last one) into the wave's LDS
        wave_lds_sync();
        stage_block(bk);
        wave_lds_sync();
      }
      if (!MMSBM_SK_GHOIST || b0 > 0) gather(nb);
      if (nb > LC) load_block(b0 / LC + 1, bk);  // the next block's records, in flight meanwhile
      if constexpr (MODE != SK_B) {
        // ---- d of every observation of the block.  Per chunk: Z[obs hi][b = col] =
        // sum_h theta_v(obs hi)[h] V_t[b][h] on MFMA (A = theta_v(obs lo)[4 hs + hi], the transpose
        // of the gathered tile, through the wave's LDS; B = the running stretch's V operand, zero for
        // b >= K and h >= K), d = eps + sum_b theta_u[b] Z[b], parked at DL[4 q + obs] (one word per
        // observation = per lane of the wave).  A chunk past the end has zero theta (never used).
#if MMSBM_SK_MRED
        // d of a group of 4 chunks: w_u[obs][col] = theta_u[col] Z[col] (zero for col >= K), then
        // one v_mfma_f64_16x16x4 per chunk against a 0/1 selector, R += w_u E_u with
        // E_u[k = obs][n] = [n == 4 u + obs], moves chunk u's observation obs to column n = 4 u + obs:
        // lane (hi, n) receives the columns col = hi + 4 i (i = 0..3) of observation n; summed in
        // the lane, then over the four rows by two lane swaps (xor 32, then 16: commutative, so
        // every row gets the same bits).  d of (chunk 4 g + n / 4, obs n % 4) = DL[16 g + n].
#pragma unroll
        for (int g4 = 0; g4 < LC / 4; ++g4) {
          if (4 * g4 < nb) {
            d4v R = d4v{0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int q = 4 * g4 + u;
              TRl[lane] = gv[q];  // (h >= K: finite, against zero V)
              wave_lds_sync();
              double z = 0.0;
#pragma unroll
              for (int hs = 0; hs < NG; ++hs) z = mfma4(TRl[16 * lo + 4 * hs + hi], vb[hs], z);
              R = mfma16(ga[q] * z, col == 4 * u + hi ? 1.0 : 0.0, R);
              if (q < nb && ((endm >> q) & 1u)) {  // the next stretch's V operand
                ++vt;
                load_v(vt);
              }
            }
            double sr = (R[0] + R[1]) + (R[2] + R[3]);
            sr += __shfl_xor(sr, 32, 64);
            sr += __shfl_xor(sr, 16, 64);
            DL[16 * g4 + col] = sr + eps;
          }
        }
#else  // d by a DPP row sum per chunk (r03s same-box A/B: 38.2k vs 37.4k iter/s with the MFMA sum)
#pragma unroll
        for (int q = 0; q < LC; ++q) {
          if (q < nb) {
#if MMSBM_SK_TRSWZ  // column swizzle c ^ 4 o (o = the observation row): the compiler pairs the
                    // reads of hs = 0, 2 into ds_read2_b64, whose 16-lane groups bank on (a/4) mod
                    // 32, where the 4 rows (16 doubles apart) coincide; c ^ 4 o moves each row to
                    // its own 8 banks (round 3's c ^ 4 (o >> 1) left rows 0 / 1 and 2 / 3 sharing:
                    // 56 % of the kernel's LDS conflict cycles, profiles/r05h_lds_attribution.txt)
            TRl[16 * hi + (col ^ (4 * hi))] = gv[q];
            wave_lds_sync();
            double z = 0.0;
#pragma unroll
            for (int hs = 0; hs < NG; ++hs)
              z = mfma4(TRl[16 * lo + ((4 * hs + hi) ^ (4 * lo))], vb[hs], z);
#else
            TRl[lane] = gv[q];
            wave_lds_sync();
            double z = 0.0;
#pragma unroll
            for (int hs = 0; hs < NG; ++hs) z = mfma4(TRl[16 * lo + 4 * hs + hi], vb[hs], z);
#endif
            // (the 16 lanes of a row hold the same bits and store the same word; storing from one
            // lane per row measured no faster, r03u)
            DL[q * 4 + hi] = row16_sum(ga[q] * z) + eps;
            if ((endm >> q) & 1u) {  // the next stretch's V operand
              ++vt;
              load_v(vt);
            }
          }
        }
#endif
        wave_lds_sync();
        // ---- one observation per lane: c = n / d (or n log d), once per observation instead of
        // once per 16 lanes of it
        const double dl = DL[lane];
        const double wn = (double)wlane;
        const bool real = lane < 4 * nb;
        if constexpr (MODE == SK_LL) {
          if (real) ll += wn * log(dl);
        } else {
          const double cl = sk_div(wn, dl);
          DL[lane] = cl;
          if (MODE == SK_A && real) {
            const int2 rr = reinterpret_cast<const int2*>(AUX)[lane];
            if (rr.x >= 0) {
              cBb[rr.x] = cl;
              cBb[rr.y] = cl;
            }
          }
        }
        wave_lds_sync();
      }
      if constexpr (MODE != SK_LL) {
        // ---- M^s += c theta_u (x) theta_v over each chunk's 4 observations (k = observation), c
        // broadcast from the observation's word; a stretch's M row replaces its V table in slot t
#pragma unroll
        for (int q = 0; q < LC; ++q) {
          if (q < nb) {
            m16 = mfma16(ga[q], cw[q * 4 + hi] * gv[q], m16);
            if (((endm >> q) & 1u) || b0 + q + 1 == c1) {  // stretch t done: its M row into slot t
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                const int x = hi + 4 * i;
                if (x < K && kcol) MSl[t * SLOT + x * K + col] = m16[i];
              }
              m16 = d4v{0.0, 0.0, 0.0, 0.0};
              ++t;
            }
          }
        }
      }
    }
    st_.mark(2);
  }
  // pass B staged P^s without a barrier (it forms no V tables): publish it before X; the other
  // modes published it before the V tables, so their waves run X and S without waiting
  if constexpr (MODE == SK_B) __syncthreads();
  if (un.nst > 0) {
    const int nst = un.nst;
    if constexpr (MODE != SK_LL) {
      // ---- X_q[z] = sum_cell P^s[z][cell] M_q[cell] for the unit's rows q (m = q, n = z in the
      // block's z tile, k = 4 cells per step)
      // (four independent accumulator chains over the cell steps, added in a fixed order)
      const int z = 4 * blk + lo;
      const double* __restrict__ pz = PV + (z < K ? z : K - 1) * T::PVS + hi;  // B: P^s[z][4 ks + hi]
#pragma unroll
      for (int tt = 0; tt < NT2; ++tt) {
        if (tt == 0 || nst > 4 * tt) {  // (uniform)
          double xa[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int ks = 0; ks < NCT; ++ks) {
            // (M words past K^2 are zero; rows q >= nst and columns z >= K are not stored)
            xa[ks & 3] = mfma4(MSl[(4 * tt + lo) * SLOT + 4 * ks + hi], pz[4 * ks], xa[ks & 3]);
          }
          const double xacc = (xa[0] + xa[1]) + (xa[2] + xa[3]);
          if (4 * tt + hi < nst && blk < NG && z < K) xb[(size_t)un.prow[tt] * K + z] = xacc;
        }
      }
      if (!MMSBM_SK_SCOOP && (MODE == SK_A || (MODE == SK_U && s == 0))) {
        // ---- S_r[a][cell] += sum_q theta_{g_q}[a] M_q[cell] (m = a, k = q, n = cell), the
        // unit's row tiles in order
#pragma unroll
        for (int tt = 0; tt < NT2; ++tt) {
          if (tt == 0 || nst > 4 * tt) {
#pragma unroll
            for (int cg = 0; cg < NCG; ++cg) {
              // (ts is zero for q >= nst; cells >= K^2 are not stored)
              const double mb = MSl[(4 * tt + hi) * SLOT + 4 * (4 * cg + blk) + lo];
#pragma unroll
              for (int at = 0; at < NG; ++at)  // A: theta_{g_q}[4 at + lo] for q = 4 tt + hi
                sacc[at][cg] = mfma4(THl[(4 * tt + hi) * 4 * NG + 4 * at + lo], mb, sacc[at][cg]);
            }
          }
        }
      }
      st_.mark(3);
    }
  }

#if MMSBM_SK_SCOOP
  if (MODE == SK_A || (MODE == SK_U && s == 0)) {  // (workgroup-uniform)
    // ---- the workgroup's S partial in one pass over all its stretches: S_r[a][cell] =
    // sum_q theta_{g_q}[a] M_q[cell] over the rows q = (wave, slot) of every wave, in that order
    // (m = a, k = q, n = cell; A from the waves' pivot theta rows, B from their M rows).  Rows of
    // absent stretches are zero (V zeros, zero theta); an empty slot zeroes its own first.  One
    // barrier, then each wave takes (a tile, cell group) items and stores its cells directly.
    constexpr int WV = MODE == SK_U ? T::WAVE_U : T::WAVE;
    if (un.nst == 0) {
#pragma unroll
      for (int i = 0; i < (GUK * SLOT + 63) / 64; ++i)
        if (lane + 64 * i < GUK * SLOT) MSl[lane + 64 * i] = 0.0;
#pragma unroll
      for (int i = 0; i < (T::THL + 63) / 64; ++i)
        if (lane + 64 * i < T::THL) THl[lane + 64 * i] = 0.0;
    }
    __syncthreads();
    double* __restrict__ out = spart + ((size_t)b * n_wg + w) * K3;
    constexpr int NI = NG * NCG, NIW = (NI + NW - 1) / NW, QS = NW * GUK / 4;
    double acc[NIW];
#pragma unroll
    for (int j = 0; j < NIW; ++j) acc[j] = 0.0;
#pragma unroll 4
    for (int qs = 0; qs < QS; ++qs) {
      const int qw = (4 * qs) / GUK, qt = (4 * qs) % GUK + hi;  // (wave qw uniform per step)
      const double* __restrict__ wq = smem + T::PSD + qw * WV;
      const double* __restrict__ thq = wq + GUK * SLOT + SK_ROWS + qt * 4 * NG + lo;
      const double* __restrict__ mq = wq + qt * SLOT + 4 * blk + lo;
#pragma unroll
      for (int j = 0; j < NIW; ++j) {
        const int it = wv + NW * j;
        if (j + 1 < NIW || it < NI) {  // (uniform)
          const int at = it / NCG, cg = it % NCG;
          acc[j] = mfma4(thq[4 * at], mq[16 * cg], acc[j]);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < NIW; ++j) {
      const int it = wv + NW * j;
      const int a = 4 * (it / NCG) + hi, cell = 16 * (it % NCG) + 4 * blk + lo;
      if (it < NI && a < K && cell < K2) out[a * K2 + cell] = acc[j];
    }
  }
#else
  if (MODE == SK_A || (MODE == SK_U && s == 0)) {  // (workgroup-uniform)
    // ---- the workgroup's S partial: the 8 waves' shares added in a fixed order,
    // ((w0 + w4) + (w2 + w6)) + ((w1 + w5) + (w3 + w7)), through LDS: waves 4-7 park theirs, waves
    // 0-3 add them to their own and park the pair sums, then every thread combines the four pairs
    // for its share of the K^3 partial and stores it
    constexpr int NE = NG * NCG * 64;  // (a tile, cell group, lane) entries of one share
    double* red = smem;
    auto put = [&](int slot) {
#pragma unroll
      for (int at = 0; at < NG; ++at)
#pragma unroll
        for (int cg = 0; cg < NCG; ++cg) red[slot * NE + (at * NCG + cg) * 64 + lane] = sacc[at][cg];
    };
    __syncthreads();
    if (wv >= 4) put(wv - 4);
    __syncthreads();
    if (wv < 4) {
#pragma unroll
      for (int at = 0; at < NG; ++at)
#pragma unroll
        for (int cg = 0; cg < NCG; ++cg) sacc[at][cg] += red[wv * NE + (at * NCG + cg) * 64 + lane];
      put(wv);
    }
    __syncthreads();
    double* __restrict__ out = spart + ((size_t)b * n_wg + w) * K3;
#pragma unroll
    for (int i = 0; i < (NE + NT - 1) / NT; ++i) {
      const int e = tid + NT * i;
      if (e < NE) {
        const int l = e & 63, ac = e >> 6;
        const int a = 4 * (ac / NCG) + (l >> 4), cell = 4 * (4 * (ac % NCG) + ((l >> 2) & 3)) + (l & 3);
        const double v = (red[e] + red[2 * NE + e]) + (red[NE + e] + red[3 * NE + e]);
        if (a < K && cell < K2) out[a * K2 + cell] = v;
      }
    }
  }
#endif
  if constexpr (MODE == SK_LL) {
    __shared__ double redl[NW];
    ll = wave_sum(ll);
    __syncthreads();
    if (lane == 0) redl[wv] = ll;
    __syncthreads();
    if (tid == 0) {
      double tt = 0.0;
      for (int q = 0; q < NW; ++q) tt += redl[q];
      partL[(size_t)b * n_wg + w] = tt;
    }
  }
  st_.mark(7);
  st_.flush(MODE == SK_B ? 1 : MODE == SK_LL ? 4 : 0, ((long long)b * gridDim.x + wx) * NW + wv, lane);
}

// ------------------------------------------------------------------------------------------
// SK_Y (round 4; the family for B >= 2 under MMSBM_FAMILY_AUTO, or as a driver fixes it per run with
// mmsbm_set_family; SK_U serves one sample): ONE launch over the stream-0 slots only.  The j- and
// k-slot sums of an observation factor through its stream-0 pivot's V table (mmsbm.hip header,
// tests/pivot_model.py::iterate_y):
//   sum_ah T = th_j[b] Z[b],  Z[b] = sum_h V_i[b][h] th_k[h];   sum_ab T = th_k[h] Z'[h],
//   Z'[h] = sum_b th_j[b] V_i[b][h]
// so per chunk the wave forms Z and Z' (two 4x4x4 MFMA chains over the V table, read row- and
// column-wise from its slot), d = eps + th_j . Z, c = n / d, writes the Y entries c Z (gene j)
// and c Z' (gene k) and accumulates M^0 += c th_j (x) th_k.  Streams 1 and 2 — their records,
// their theta gathers, V tables, c and M work and their X contractions — do not exist.  At the
// unit's end: X^0 of its stretches (into the stretch's own Y entry, Plan::prow_y) and the
// workgroup's S partial, as SK_U does for stream 0; sk_fin_kernel then sums each gene's Y range
// (Plan::yptr: its observation entries, then its X^0 rows) in one pass.
// Each chunk runs start to end (Z, Z', d, c in its 16 lanes, Y, M): the block's 32 theta gathers
// all go out first, as in SK_U, and no chunk's Z / Z' has to stay live until a batched division.
// ------------------------------------------------------------------------------------------
template <int K>
struct SKY {
  using T = SKT<K>;
  // per wave: slots, the block's (u, v) genes, pivot rows, the block's Y entries, one transpose
  // buffer
  static constexpr int WAVE = T::GUK * T::SLOT + SK_ROWS + T::THL + SK_ROWS + 64 + 16;  // (+ zero words)
  static constexpr int LDS = (T::PSD + NW * WAVE) * 8;
  static_assert(LDS <= 80 * 1024, "two SK_Y workgroups per CU");
  // the unguarded Z' operand reads (rows b < 4 NG of the last slot, columns up to 15) stay inside
  // the wave's slots, records and pivot rows (finite words)
  static_assert((T::GUK - 1) * T::SLOT + (4 * T::NG - 1) * K + 15 < T::GUK * T::SLOT + SK_ROWS + T::THL,
                "Z' reads past the wave's slots");
};

template <int K>
__global__ __launch_bounds__(NT, 4) void sky_pass_kernel(
    const int4* __restrict__ urec, const int* __restrict__ udesc, const int2* __restrict__ urowy,
    const double* __restrict__ theta, const double* __restrict__ pr, double* __restrict__ ybuf,
    double* __restrict__ xpart, double* __restrict__ spart, SkSec sec, int L, int P, int R,
    long long n_y, long long n_prows, int n_wg, double eps) {
  using T = SKT<K>;
  using Y = SKY<K>;
  constexpr int NG = T::NG, K2 = T::K2, K3 = T::K3, NCT = T::NCT, NCG = T::NCG, SLOT = T::SLOT;
  constexpr int GUK = T::GUK, NT2 = T::NT2;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 4, blk = (lane >> 2) & 3, lo = lane & 3, col = lane & 15;
  const int w = blockIdx.x, b = blockIdx.y;
  int sr = 0;  // this workgroup's (stream 0, rating) section, from the launch arguments alone
#pragma unroll
  for (int i = 0; i < MAX_R - 1; ++i)
    if (i + 1 < R && w >= sec.wg_end[i]) sr = i + 1;
  const int r = __builtin_amdgcn_readfirstlane(sr);
  const double* __restrict__ th = theta + (size_t)b * P * K;
  const double* __restrict__ p = pr + ((size_t)b * R + r) * K3;
  double* PV = smem;  // P^0_r[z][cell] (cell = x K + y), rows of SKT::PVS words
  double* wl = smem + T::PSD + wv * Y::WAVE;
  double* MSl = wl;                                        // GUK slots: V, then M
  int2* REC = reinterpret_cast<int2*>(wl + GUK * SLOT);    // the block's (u, v) genes
  double* THl = wl + GUK * SLOT + SK_ROWS;                 // pivot theta rows [GUK][4 NG]
  int2* YE = reinterpret_cast<int2*>(THl + T::THL);        // the block's Y entries (slot 1, slot 2)
  double* TRl = THl + T::THL + SK_ROWS;                    // the Z / Z' operand transpose
  double* ZRl = TRl + 64;                                  // 16 zero words (load_v's masked lanes)
  double* __restrict__ yb = ybuf + (size_t)b * (n_y + 1) * K;
  (void)xpart;
  (void)n_prows;
  Stamp st_{};
  st_.mark(0);

  // P^0_r once per workgroup (plain copy: the pivot slot is slot 0)
  double pvv[T::NPV];
#pragma unroll
  for (int i = 0; i < T::NPV; ++i) {
    const int e = tid + NT * i, z = e / T::PVS, cell = e % T::PVS;
    const bool ok = z < K && cell < K2;
    const double v = p[ok ? z * K2 + cell : 0];
    pvv[i] = ok ? v : 0.0;
  }

  const long long slot = (long long)w * NW + wv;
  struct Unit {
    int nst, c1, ds[GUK], prow[NT2];
    double tv[NT2][NG];
  };
  struct Blk {
    int4 rv;
    int2 ry;
  };
  auto load_block = [&](int bi, Blk& bk) {
    const int idx = SK_ROWS * bi + lane;
    const long long row = slot * 4 * L + (idx < 4 * L ? idx : 4 * L - 1);
    bk.rv = urec[row];
    bk.ry = urowy[row];
  };
  int wlane = 0;
  auto stage_block = [&](const Blk& bk) {
    REC[lane] = make_int2(bk.rv.x, bk.rv.y);
    wlane = bk.rv.w;
    YE[lane] = bk.ry;
  };
  auto load_unit = [&](Unit& un) {
    const int* __restrict__ d = udesc + slot * mmsbm_plan::UD;
    un.nst = __builtin_amdgcn_readfirstlane(d[mmsbm_plan::D_NST]);
    un.c1 = __builtin_amdgcn_readfirstlane(d[mmsbm_plan::D_END]);
#pragma unroll
    for (int t = 0; t < GUK; ++t) un.ds[t] = __builtin_amdgcn_readfirstlane(d[t]);
#pragma unroll
    for (int tt = 0; tt < NT2; ++tt) un.prow[tt] = d[mmsbm_plan::D_PROW + 4 * tt + hi];
#pragma unroll
    for (int tt = 0; tt < NT2; ++tt) {
      const int glo = d[mmsbm_plan::D_GENE + 4 * tt + lo];
#pragma unroll
      for (int as = 0; as < NG; ++as) {
        const int a1 = 4 * as + hi;
        const double v1 = th[(size_t)glo * K + (a1 < K ? a1 : 0)];
        un.tv[tt][as] = (4 * tt + lo < un.nst && a1 < K) ? v1 : 0.0;
      }
    }
  };
  Blk bk;
  load_block(0, bk);
  Unit un;
  load_unit(un);
  // the first block's theta gathers go out as soon as its records are in the wave's LDS, before
  // P^0 is staged and the V tables are formed: a unit is only a few chunks long, so the gathers'
  // latency would otherwise sit on the wave's path once per unit
  stage_block(bk);
  wave_lds_sync();
  const int colc = col < K ? col : K - 1;
  const unsigned cb = (unsigned)colc * 8u;
  const bool kcol = col < K;
  double ga[LC], gv[LC];
  auto gather = [&](int nb) {  // (every chunk of the block, as in sk_pass_kernel; nb = 0: none)
    if (nb > 0) {  // (uniform)
      int2 rh[LC];
#pragma unroll
      for (int i = 0; i < LC; ++i) rh[i] = REC[i * 4 + hi];
#pragma unroll
      for (int i = 0; i < LC; ++i) {
        const char* __restrict__ thb = reinterpret_cast<const char*>(th);
        ga[i] = *reinterpret_cast<const double*>(thb + (__umul24((unsigned)rh[i].x, K * 8u) + cb));
        gv[i] = *reinterpret_cast<const double*>(thb + (__umul24((unsigned)rh[i].y, K * 8u) + cb));
      }
    } else {
#pragma unroll
      for (int i = 0; i < LC; ++i) ga[i] = gv[i] = 0.0;
    }
  };
  gather(un.nst > 0 ? (un.c1 < LC ? un.c1 : LC) : 0);
#pragma unroll
  for (int i = 0; i < T::NPV; ++i)
    if (tid + NT * i < T::PSD) PV[tid + NT * i] = pvv[i];
  __syncthreads();  // P^0_r published (the V tables below read it)
  st_.mark(6);

  if (un.nst > 0) {
    const int nst = un.nst;
    const int c1 = un.c1;
    st_.t[5] = (unsigned long long)c1;
    st_.t[4] = (unsigned long long)nst;
    const auto& ds = un.ds;
    const auto& tv = un.tv;
    // ---- V_g[cell] = sum_a theta_g[a] P^0[a][cell] for the unit's genes into their slots (every
    // word of the GUK slots written: zero past K^2 and for absent stretches); pivot theta rows to
    // THl for the S pass
#pragma unroll
    for (int tt = 0; tt < NT2; ++tt) {
      const bool live = tt == 0 || nst > 4 * tt;
#pragma unroll
      for (int cg = 0; cg < NCG; ++cg) {
        const int cell = 4 * (4 * cg + blk) + lo;
        double v = 0.0;
        if (live) {
#pragma unroll
          for (int as = 0; as < NG; ++as)
            v = mfma4(tv[tt][as], PV[(4 * as + hi < K ? 4 * as + hi : K - 1) * T::PVS + cell], v);
        }
        if (cell < SLOT) MSl[(4 * tt + hi) * SLOT + cell] = cell < K2 ? v : 0.0;
      }
#pragma unroll
      for (int as = 0; as < NG; ++as)
        if (blk == 0) THl[(4 * tt + lo) * 4 * NG + 4 * as + hi] = tv[tt][as];
      __builtin_amdgcn_sched_barrier(0);
    }
    if (lane < 16) ZRl[lane] = 0.0;
    wave_lds_sync();
    st_.mark(1);

    // Z operand V[b = col][h = 4 hs + hi] (zero for b >= K, h >= K); Z' operand V[b = 4 bs + hi]
    // [h = col] (rows b >= K meet a zero theta_j; columns h >= K are never stored)
    const double* __restrict__ vrow = MSl + col * K + hi;
    const double* __restrict__ vcol = MSl + hi * K + col;
    d4v m16 = d4v{0.0, 0.0, 0.0, 0.0};
    int t = 0;
    double vb[NG], vbt[NG];
    // (the Z operand from the slot or a zero word, as in sk_pass_kernel; Z' needs no mask)
    int voff[NG], vstr[NG];
#pragma unroll
    for (int hs = 0; hs < NG; ++hs) {
      const bool ok = kcol && 4 * hs + hi < K;
      voff[hs] = ok ? (int)(MSl - smem) + col * K + hi + 4 * hs : (int)(ZRl - smem);
      vstr[hs] = ok ? SLOT : 0;
    }
    auto load_v = [&](int tv_) {
#pragma unroll
      for (int hs = 0; hs < NG; ++hs) {
        vb[hs] = smem[voff[hs] + tv_ * vstr[hs]];
        vbt[hs] = vcol[tv_ * SLOT + 4 * hs * K];
      }
    };
    int vt = 0;
    load_v(0);
    for (int b0 = 0; b0 < c1; b0 += LC) {
      const int nb = c1 - b0;
      unsigned endm = 0;  // bit q: chunk b0 + q ends a stretch other than the unit's last
#pragma unroll
      for (int i = 1; i < GUK; ++i) {
        const int e = ds[i] - 1 - b0;
        if (i < nst && e >= 0 && e < LC) endm |= 1u << e;
      }
      endm = __builtin_amdgcn_readfirstlane(endm);
      // ---- theta gathers: every value of the block at once, straight into the registers of the
      // MFMA operands (lane (obs hi, col): theta_j and theta_k of its observation, column col;
      // col >= K a finite copy of column K - 1, masked where a product needs it); the first
      // block's went out in the prologue
      if (b0 > 0) {
        wave_lds_sync();
        stage_block(bk);
        wave_lds_sync();
        gather(nb);
      }
      if (nb > LC) load_block(b0 / LC + 1, bk);  // the next block's records, in flight meanwhile
      // ---- per chunk: Z and Z' on MFMA (A = the transposed theta_k / theta_j tile through the
      // wave's LDS, bank-swizzled; theta_j zeroed past K), d by a DPP row sum, c = n / d in the 16
      // lanes of each observation, the Y entries c Z (gene j) and c Z' (gene k), M += c theta_j (x)
      // theta_k (k = observation); a finished stretch's M row replaces its V table in slot t
#pragma unroll
      for (int q = 0; q < LC; ++q) {
        if (q < nb) {
          TRl[16 * hi + (col ^ (4 * hi))] = gv[q];
          wave_lds_sync();
          double z = 0.0;
#pragma unroll
          for (int hs = 0; hs < NG; ++hs)
            z = mfma4(TRl[16 * lo + ((4 * hs + hi) ^ (4 * lo))], vb[hs], z);
          // (a wave's LDS accesses execute in order: the reads above precede this write)
          TRl[16 * hi + (col ^ (4 * hi))] = kcol ? ga[q] : 0.0;
          wave_lds_sync();
          double zp = 0.0;
#pragma unroll
          for (int bs = 0; bs < NG; ++bs)
            zp = mfma4(TRl[16 * lo + ((4 * bs + hi) ^ (4 * lo))], vbt[bs], zp);
          // the count of observation hi of this chunk (lane 4 q + hi's record), by scalar reads
          const int n0 = __builtin_amdgcn_readlane(wlane, 4 * q), n1 = __builtin_amdgcn_readlane(wlane, 4 * q + 1);
          const int n2 = __builtin_amdgcn_readlane(wlane, 4 * q + 2), n3 = __builtin_amdgcn_readlane(wlane, 4 * q + 3);
          const int nq = hi == 0 ? n0 : hi == 1 ? n1 : hi == 2 ? n2 : n3;
          const double d = row16_sum(ga[q] * z) + eps;
          const double c = sk_div((double)nq, d);
          const int2 ey = YE[q * 4 + hi];
          if (kcol) {
            yb[(size_t)ey.x * K + col] = c * z;
            yb[(size_t)ey.y * K + col] = c * zp;
          }
          m16 = mfma16(ga[q], c * gv[q], m16);
          const bool ends = (endm >> q) & 1u;
          if (ends) {  // the next stretch's V operands
            ++vt;
            load_v(vt);
          }
          if (ends || b0 + q + 1 == c1) {  // stretch t done: its M row into slot t
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int x = hi + 4 * i;
              if (x < K && kcol) MSl[t * SLOT + x * K + col] = m16[i];
            }
            m16 = d4v{0.0, 0.0, 0.0, 0.0};
            ++t;
          }
        }
      }
    }
    st_.mark(2);
    // ---- X_q[z] = sum_cell P^0[z][cell] M_q[cell] for the unit's rows q
    const int z = 4 * blk + lo;
    const double* __restrict__ pz = PV + (z < K ? z : K - 1) * T::PVS + hi;
#pragma unroll
    for (int tt = 0; tt < NT2; ++tt) {
      if (tt == 0 || nst > 4 * tt) {
        double xa[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int ks = 0; ks < NCT; ++ks)
          xa[ks & 3] = mfma4(MSl[(4 * tt + lo) * SLOT + 4 * ks + hi], pz[4 * ks], xa[ks & 3]);
        const double xacc = (xa[0] + xa[1]) + (xa[2] + xa[3]);
        // (the stretch's Y entry: fin sums it with the gene's observation entries)
        if (4 * tt + hi < nst && blk < NG && z < K) yb[(size_t)un.prow[tt] * K + z] = xacc;
      }
    }
    st_.mark(3);
  }

  // ---- the workgroup's S partial in one pass over all its stretches (as SK_U's stream 0)
  {
    if (un.nst == 0) {
#pragma unroll
      for (int i = 0; i < (GUK * SLOT + 63) / 64; ++i)
        if (lane + 64 * i < GUK * SLOT) MSl[lane + 64 * i] = 0.0;
#pragma unroll
      for (int i = 0; i < (T::THL + 63) / 64; ++i)
        if (lane + 64 * i < T::THL) THl[lane + 64 * i] = 0.0;
    }
    __syncthreads();
    double* __restrict__ out = spart + ((size_t)b * n_wg + w) * K3;
    constexpr int NI = NG * NCG, NIW = (NI + NW - 1) / NW, QS = NW * GUK / 4;
    double acc[NIW];
#pragma unroll
    for (int j = 0; j < NIW; ++j) acc[j] = 0.0;
#pragma unroll 4
    for (int qs = 0; qs < QS; ++qs) {
      const int qw = (4 * qs) / GUK, qt = (4 * qs) % GUK + hi;
      const double* __restrict__ wq = smem + T::PSD + qw * Y::WAVE;
      const double* __restrict__ thq = wq + GUK * SLOT + SK_ROWS + qt * 4 * NG + lo;
      const double* __restrict__ mq = wq + qt * SLOT + 4 * blk + lo;
#pragma unroll
      for (int j = 0; j < NIW; ++j) {
        const int it = wv + NW * j;
        if (j + 1 < NIW || it < NI) {
          const int at = it / NCG, cg = it % NCG;
          acc[j] = mfma4(thq[4 * at], mq[16 * cg], acc[j]);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < NIW; ++j) {
      const int it = wv + NW * j;
      const int a = 4 * (it / NCG) + hi, cell = 16 * (it % NCG) + 4 * blk + lo;
      if (it < NI && a < K && cell < K2) out[a * K2 + cell] = acc[j];
    }
  }
  st_.mark(7);
  st_.flush(0, ((long long)b * gridDim.x + w) * NW + wv, lane);
}

// ------------------------------------------------------------------------------------------
// sk_fin_kernel, grid (gene workgroups + cell workgroups + q workgroups, B), block 256.
//   gene part, SK_U plans: thread (g, x): X = the sum of g's X partials (gene-major: (stream,
//     rating, row) order) (+ the joint model's pair sums); theta' = theta X / deg (:1016-1018)
//     or, SUMS, nth = X.
//   gene part, SK_Y plans (ybuf set): one wave per gene; its Y entries (one contiguous
//     block of K-word rows, Plan::yptr) are summed by lanes l < K floor(64 / K), lane l taking
//     words l, l + LY, ... (component l mod K), the lanes of one component then added in lane
//     order; lane x < K adds that to its X^0 partial rows (stream 0) and updates theta.
//   cell part: SKF_CW cells x SKF_NPART parts per workgroup: S_r[cell] = sum of the rating's S
//     partials (one per stream-0 workgroup), parts combined in order, two ratings' loads in one
//     round; p' = p S / (eps + sum_r p S)
//     (:1021-1028) in place, or, SUMS, S_out = S.
//   q part (joint model): as in fin_kernel.
// ------------------------------------------------------------------------------------------
// cell part: SKF_CW cells x SKF_NPART parts per workgroup, SKF_SB partial loads per batch (round 6:
// 8 x 32 x 4 instead of 16 x 16 x 16: a part's few partials (fold0: 2-3 of 88 per rating) without
// the clamped duplicate loads that kept the address units of each cell workgroup's CU busy; the
// 32 parts are added by a butterfly in each wave, then the 4 waves in order)
constexpr int SKF_NT = 256, SKF_CW = 8, SKF_NPART = 32, SKF_SB = 4;
static_assert(SKF_CW * SKF_NPART == SKF_NT, "fin cell part: one (cell, part) per thread");

// sum of gene g's X partials (component x): its gene-major range [gptr[g], gptr[g + 1]) of
// partial rows ((stream, rating, row) order, Plan::prow_g), 8 loads in flight (a hub gene's pivot
// runs span many units); one dependent round for the range, then the rows
__device__ __forceinline__ double sk_gene_sum(const double* __restrict__ xb, const int* __restrict__ gptr,
                                              int g, int x, int K) {
  const int q0 = gptr[g], q1 = gptr[g + 1];
  double X = 0.0;
  for (int q = q0; q < q1; q += 8) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = xb[(size_t)(q + u < q1 ? q + u : q) * K + x];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (q + u < q1) X += v[u];
  }
  return X;
}

template <int K, bool SUMS>
__global__ __launch_bounds__(SKF_NT) void sk_fin_kernel(
    double* __restrict__ theta, double* __restrict__ pr, const double* __restrict__ xpart,
    const int* __restrict__ gptr, const double* __restrict__ spart, const int* __restrict__ deg,
    SpRange spr, int P, int R, long long n_prows, int n_wg_a, int n_gene_wg, double eps,
    double* __restrict__ nth_out, double* __restrict__ S_out, const double* __restrict__ nth_add,
    const double* __restrict__ q_part, double* __restrict__ q_out, int n_qwg,
    const double* __restrict__ ybuf, const int* __restrict__ yptr, long long n_y) {
  constexpr int K2 = K * K, K3 = K * K * K;
  constexpr int NCW = (K3 + SKF_CW - 1) / SKF_CW;
  __shared__ double red[MAX_R * SKF_NPART * SKF_CW];
  const int tid = threadIdx.x, b = blockIdx.y;
  const int wgx = blockIdx.x;
  Stamp st_{};
  st_.mark(0);
#ifdef MMSBM_FIN_EMPTY  // measurement builds only (results invalid): the launch without its work
  if (b >= 0) return;
#endif
#ifdef MMSBM_FIN_ONLY  // measurement builds only (results invalid): 1 = gene workgroups only, 2 = cell only
  if ((MMSBM_FIN_ONLY == 1) != (wgx < n_gene_wg)) return;
#endif
  if (wgx < n_gene_wg && ybuf) {
    constexpr int LPX = 64 / K, LY = K * LPX, YU = 16;  // lanes per component, lanes used
    const int lane = tid & 63, wv = tid >> 6;
    const int g = wgx * (SKF_NT / 64) + wv;
    if (g >= P) return;  // (wave-uniform; no barrier in this branch)
    const long long w0 = (long long)yptr[g] * K, w1 = (long long)yptr[g + 1] * K;
    const double* __restrict__ yb = ybuf + (size_t)b * (n_y + 1) * K;
    const int x = lane < K ? lane : 0;
    const double th = theta[((size_t)b * P + g) * K + x];
    const double ad = nth_add ? nth_add[((size_t)b * P + g) * K + x] : 0.0;
    const int dg = deg[g];
    // the gene's Y range holds its observation entries and its X^0 partial rows (at fold0 ~100
    // entries of K words: one round of YU loads over LY lanes for most genes)
    double S = 0.0;
    if constexpr (K % 2 == 0) {
      // even K (round 6): 16-byte loads (the wide coalesced form the memory pipe moves at full
      // rate; the range and the sample's Y block start at even words).  Lane l < LW reads words
      // 2 l, 2 l + 1 of each WW-word step, components 2 l mod K and 2 l + 1 mod K (WW = EPI K, a
      // whole number of entries); YU2 steps in flight.
      constexpr int EPI = 128 / K, WW = EPI * K, LW = WW / 2, YU2 = 8;
      typedef double d2 __attribute__((ext_vector_type(2)));
      const long long wf = w0 + 2 * (lane < LW ? lane : 0);
      double Sa = 0.0, Sb = 0.0;
      if (lane < LW) {
        for (long long wd = wf; wd < w1; wd += (long long)YU2 * WW) {
          d2 v[YU2];
#pragma unroll
          for (int u = 0; u < YU2; ++u)
            v[u] = *reinterpret_cast<const d2*>(yb + (wd + (long long)u * WW < w1 ? wd + (long long)u * WW : wf));
#pragma unroll
          for (int u = 0; u < YU2; ++u)
            if (wd + (long long)u * WW < w1) {
              Sa += v[u].x;
              Sb += v[u].y;
            }
        }
      }
      double* __restrict__ yr2 = red + wv * 128;
      yr2[2 * lane] = Sa;
      yr2[2 * lane + 1] = Sb;
      wave_lds_sync();
      if (lane < K) {  // component x: words x + j K of a step, j in order
        double Y = yr2[lane];
#pragma unroll
        for (int jj = 1; jj < EPI; ++jj) Y += yr2[lane + jj * K];
        double X = Y;
        if (nth_add) X += ad;
        const size_t o = ((size_t)b * P + g) * K + lane;
        if constexpr (SUMS) nth_out[o] = X;
        else theta[o] = th * X / (double)dg;
      }
      return;
    }
    const long long wf = w0 + (lane < LY ? lane : 0);
    double v0[YU];
#pragma unroll
    for (int u = 0; u < YU; ++u) v0[u] = yb[wf + (long long)u * LY < w1 ? wf + (long long)u * LY : wf];
    if (lane < LY) {
#pragma unroll
      for (int u = 0; u < YU; ++u)
        if (wf + (long long)u * LY < w1) S += v0[u];
      for (long long wd = wf + YU * LY; wd < w1; wd += YU * LY) {
        double v[YU];
#pragma unroll
        for (int u = 0; u < YU; ++u) v[u] = yb[wd + (long long)u * LY < w1 ? wd + (long long)u * LY : wd];
#pragma unroll
        for (int u = 0; u < YU; ++u)
          if (wd + (long long)u * LY < w1) S += v[u];
      }
    }
    double* __restrict__ yr = red + wv * 64;
    yr[lane] = S;
    wave_lds_sync();
    if (lane < K) {
      double Y = yr[lane];
#pragma unroll
      for (int j = 1; j < LPX; ++j) Y += yr[lane + j * K];
      double X = Y;
      if (nth_add) X += ad;
      const size_t o = ((size_t)b * P + g) * K + lane;
      if constexpr (SUMS) nth_out[o] = X;
      else theta[o] = th * X / (double)dg;
    }
    return;
  }
  if (wgx < n_gene_wg) {
    const int item = wgx * SKF_NT + tid;
    if (item >= P * K) return;  // no barrier in this branch
    const int g = item / K, x = item % K;
    const double* __restrict__ xb = xpart + (size_t)b * n_prows * K;
    const double th = theta[((size_t)b * P + g) * K + x];
    const double ad = nth_add ? nth_add[((size_t)b * P + g) * K + x] : 0.0;
    const int dg = deg[g];
    double X = sk_gene_sum(xb, gptr, g, x, K);
    st_.mark(1);
    if (nth_add) X += ad;
    const size_t o = ((size_t)b * P + g) * K + x;
    if constexpr (SUMS) nth_out[o] = X;
    else theta[o] = th * X / (double)dg;
    st_.mark(7);
    st_.flush(2, ((long long)b * gridDim.x + wgx) * (SKF_NT / 64) + (tid >> 6), tid & 63);
    return;
  }
  if (wgx < n_gene_wg + NCW) {
    const int cl = tid % SKF_CW, part = tid / SKF_CW;
    const int cell = (wgx - n_gene_wg) * SKF_CW + cl;
    const int cc = cell < K3 ? cell : 0;
    // the S partial loads of two ratings go out together (round 6: one dependent round for R = 2
    // instead of one per rating, with the same sums: each rating's parts and their order are
    // unchanged); p (for p') is loaded after them, off their path
    auto part_sum = [&](int r, double (&v)[SKF_SB], int& s0, int& s1) {  // loads of rating r's part
      const int n = spr.hi[r] - spr.lo[r];
      s0 = spr.lo[r] + n * part / SKF_NPART;
      s1 = spr.lo[r] + n * (part + 1) / SKF_NPART;
#pragma unroll
      for (int u = 0; u < SKF_SB; ++u)
        v[u] = spart[((size_t)b * n_wg_a + (s0 + u < s1 ? s0 + u : s0)) * K3 + cc];
    };
    // a part's sum, then the wave's 8 parts (lane bits 3-5) by a butterfly (commutative pairs: every
    // lane gets the same bits), parked per (wave, rating, cell) for the in-order sum over waves
    auto finish = [&](int r, const double (&v)[SKF_SB], int s0, int s1) {
      double S = 0.0;
#pragma unroll
      for (int u = 0; u < SKF_SB; ++u) S += s0 + u < s1 ? v[u] : 0.0;
      for (int sp = s0 + SKF_SB; sp < s1; sp += SKF_SB) {  // (parts longer than one batch)
        double w[SKF_SB];
#pragma unroll
        for (int u = 0; u < SKF_SB; ++u) {
          const double xv = spart[((size_t)b * n_wg_a + (sp + u < s1 ? sp + u : s0)) * K3 + cc];
          w[u] = sp + u < s1 ? xv : 0.0;
        }
#pragma unroll
        for (int u = 0; u < SKF_SB; ++u) S += w[u];
      }
      S += __shfl_xor(S, 8, 64);
      S += __shfl_xor(S, 16, 64);
      S += __shfl_xor(S, 32, 64);
      if ((tid & 63) < SKF_CW) red[((tid >> 6) * MAX_R + r) * SKF_CW + cl] = S;
    };
    for (int r = 0; r < R; r += 2) {
      double va[SKF_SB], vb[SKF_SB];
      int a0, a1, b0 = 0, b1 = 0;
      part_sum(r, va, a0, a1);
      const bool two = r + 1 < R;  // (uniform)
      if (two) part_sum(r + 1, vb, b0, b1);
      finish(r, va, a0, a1);
      if (two) finish(r + 1, vb, b0, b1);
      st_.mark(1 + (r < 1 ? 0 : 1));
    }
    double po[MAX_R];
#pragma unroll
    for (int r = 0; r < MAX_R; ++r) po[r] = pr[((size_t)b * R + (r < R ? r : R - 1)) * K3 + cc];
    __syncthreads();
    st_.mark(3);
    if (part == 0 && cell < K3) {
      double npr[MAX_R];
      double den = eps;
#pragma unroll
      for (int r = 0; r < MAX_R; ++r) {
        if (r < R) {
          double S = red[r * SKF_CW + cl];
#pragma unroll
          for (int q = 1; q < SKF_NT / 64; ++q) S += red[(q * MAX_R + r) * SKF_CW + cl];
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
    st_.mark(7);
    st_.flush(2, ((long long)b * gridDim.x + wgx) * (SKF_NT / 64) + (tid >> 6), tid & 63);
    return;
  }
  // joint model q cells (include/mmsbm_pairs.h): 64 cells of qr per workgroup, 4 threads per cell
  // each summing a share of the pair launch's S2 partials, combined in order (:1660-1666)
  {
    constexpr int NPART = SKF_NT / 64;
    const int cl = tid & 63, part = tid >> 6;
    const int cell = (wgx - n_gene_wg - NCW) * 64 + cl;
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
          const double xv = q_part[(((size_t)b * n_qwg + (ww + u < s1 ? ww + u : s0)) * R + r) * K2 + cc];
          v[u] = ww + u < s1 ? xv : 0.0;
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
}
