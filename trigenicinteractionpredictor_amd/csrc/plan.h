// plan.h — host-side work plan of the pivot-run EM engine (built once per link set).
//
// Input: the reference's link table in `links` insertion order (src/TrigenicInteractionPredictor.py
// :321-423): ids[E][3] in the string-sorted key order (:349-358), counts[E][R] (:360-368).  One
// OBSERVATION = one (link, rating r) with n = counts[e][r] > 0 (an unobserved rating adds exactly
// +0.0 in the reference loop, :1002-1012).
//
// For every slot s in {0, 1, 2} ("stream" s) and rating r, the observations are ordered by their
// slot-s gene (the PIVOT; stable, so ties keep link order).  A pivot run is padded to a multiple of
// CH = 4 rows with zero-weight rows, so every CHUNK of 4 rows has one pivot gene.  Chunks are
// grouped into UNITS (one wave each: whole runs where they fit, long runs split) and units into
// WORKGROUPS of NW units.  Inside a unit, every maximal stretch of one pivot gene accumulates into
// one PARTIAL ROW (K x K doubles of M^s, see mmsbm.hip); partial rows are numbered in stream
// order, so the partial rows of one (stream, rating, gene) are contiguous.
//
// Row record (int4): (i, j, k, w); stream 0: w = n_r (0 on padding rows); streams 1, 2: w = the
// stream-0 row of the same observation (its c = n / d lives there), padding rows: w = n_rows0 (a
// slot that always holds 0).
//
// Large-K EM plans (mmsbm.hip) hold stream 0 only: the pass over the stream-0 rows writes, per
// observation, the j-slot and k-slot contributions c Z and c Z' (K words each) into Y ENTRIES, and
// the gene kernel sums each gene's entries.  The entries of one gene are contiguous: ordered by
// gene, then slot (1, 2), rating and link order; `yptr` [P + 1] delimits them and `row_y`
// [n_rows0][2] names the slot-1 / slot-2 entry of every stream-0 row (n_y on padding rows: a
// dummy entry nobody reads).
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

namespace mmsbm_plan {

constexpr int CH = 4;   // observations per chunk (one MFMA k-step)
constexpr int NW = 8;   // waves (units) per workgroup
// Small-K plans (K <= 12, the register-direct kernels of sk.h): a unit has at most `gu` <= GU gene
// stretches (one wave keeps their V tables and M rows, and contracts them with p at its end; gu is
// the kernel's LDS budget: 8 at K <= 10, 4 above) and at most LCAP_SK chunks, processed in blocks of
// SK_BLOCK chunks (one block's records are staged in the wave's LDS at a time).
constexpr int GU = 8;
constexpr int SK_BLOCK = 16;
constexpr int LCAP_SK = 128;
// unit descriptor: stretch start chunks [0, GU) (unused ones = the end), end chunk [D_END], stretches
// [D_NST], partial rows [D_PROW, +GU), pivot genes [D_GENE, +GU), stream * 16 + rating [D_CODE]
constexpr int D_END = GU, D_NST = GU + 1, D_PROW = GU + 2, D_GENE = 2 * GU + 2, D_CODE = 3 * GU + 2;
constexpr int UD = 32;  // ints per unit descriptor
static_assert(D_CODE < UD, "descriptor layout");
// stretches per unit of the small-K kernels at K (their LDS budget: GU * K^2 words of V tables / M
// rows per wave fit two workgroups per CU up to K = 10)
constexpr int sk_gu(int K) { return K <= 10 ? 8 : 4; }

struct I4 {
  int x, y, z, w;
};

struct Plan {
  int R = 0, P = 0;
  int streams = 0;                 // 3 (train: EM) or 1 (likelihood only)
  std::vector<I4> rows;            // all streams, stream-major then rating-major
  std::vector<int> chunk_prow;     // partial row of each chunk (-1: likelihood-only plan)
  std::vector<int> chunk_vslot;    // stream 0: the chunk's pivot gene in its workgroup's gene list
  std::vector<int> wg_units;       // [n_wg][nw + 1] chunk boundaries of the workgroup's units
  std::vector<int> wg_code;        // [n_wg] stream * 16 + rating
  std::vector<int> wg_gene;        // [n_wg + 1] offsets into vgenes (stream-0 workgroups)
  std::vector<int> vgenes;         // pivot genes of each stream-0 workgroup, ascending
  std::vector<int> prow_ptr;       // [3][R][P + 1] partial rows of (stream, rating, gene)
  std::vector<int> prow_gene;      // [n_prows]
  std::vector<int> sp_desc;        // S-partial workgroups: [n_sp][3] (rating, prow begin, end)
  int sp_lo[8] = {0}, sp_hi[8] = {0};  // S-partial workgroups of each rating
  // small-K plans only (sk.h):
  bool small = false;
  int gu = GU;                     // most stretches per unit (<= GU)
  std::vector<int> udesc;          // [n_units][UD]: the unit descriptors (D_* offsets above)
  std::vector<int> wg_ustart;      // [n_wg + 1] units of each workgroup (rounds of NW)
  std::vector<int> row12;          // [n_rows0][2] the observation's stream-1 / stream-2 row
                                   // (relative to n_rows0; -1 on padding rows)
  // large-K EM plans only: Y entries (see the header)
  std::vector<int> row_y;          // [n_rows0][2] slot-1 / slot-2 entry of each stream-0 row
  std::vector<int> yptr;           // [P + 1] entries of each gene
  long long n_y = 0;               // 2 x observations (+ the partial rows of a small-K SK_Y plan)
  std::vector<int> prow_y;         // small-K SK_Y plans: the Y entry of each (stream-0) partial row
  // small-K three-stream plans: the X partial rows gene-major (a gene's rows of every (stream,
  // rating) in one range, (stream, rating, row) order inside: fin sums one range per gene)
  std::vector<int> prow_g;         // [n_prows] gene-major position of each partial row
  std::vector<int> gptr;           // [P + 1] each gene's range of gene-major positions
  bool merge = false;              // large-K: one partial row per (workgroup, gene) (see build)
  int nw = NW;                     // units (waves) per large-K workgroup (small-K plans: NW)
  int rounds_a = 1, rounds_b = 1;  // unit rounds per workgroup (stream 0 / streams 1, 2)
  long long n_units = 0;
  // slot layout the small-K kernels read (make_slots below); group 0 = stream 0 (pass A), group 1 =
  // streams 1, 2 (pass B).  Workgroup w of a group owns slots [w rounds NW, (w + 1) rounds NW) (round
  // major, then wave); a slot holds one unit or nothing.  Records are copied slot-major with a fixed
  // capacity of 4 L rows per slot, so a wave finds its unit's records from its slot number alone.
  int sk_L[2] = {0, 0};            // chunks per slot (the group's longest unit)
  int lmax[2] = {0, 0};            // the unit length the packing aimed at (stream 0, streams 1 / 2)
  long long sk_slots[2] = {0, 0};
  std::vector<int> sk_udesc[2];    // [slots][UD]: unit descriptors with the stretch starts and end
                                   // relative to the slot's first chunk (D_NST 0: empty slot)
  std::vector<I4> sk_urec[2];      // [slots][4 L] records
  std::vector<int> sk_urow12;      // [slots_0][4 L][2] slot-major row of the stream-1 / stream-2 copy
                                   // of each stream-0 row (-1: padding), the index of its c in pass B
  int sk_wg_end[3 * 8] = {0};      // section (s, r) = s R + r ends at workgroup sk_wg_end[s R + r]
  int n_wg_a = 0;                  // stream-0 workgroups (the first n_wg_a)
  int n_wg_b = 0;                  // stream-1/2 workgroups (the next n_wg_b)
  int n_sp = 0;
  int gmax = 0;                    // most genes of one stream-0 workgroup
  long long n_rows0 = 0;           // rows of stream 0 (the c vector)
  long long n_prows = 0;
  long long n_obs = 0;             // real observations (one stream)
};

// Greedy unit packing over the runs of one (stream, rating): a unit takes whole runs while they
// fit in `lmax` chunks (and, on stream 0, `gcap` genes), a run longer than `lmax` is split.  With
// `fill`, a run that does not fit is split at the unit's end instead, so every unit but the last of
// a section holds exactly `lmax` chunks unless it reached `gcap` genes first (the fused small-K
// launch: fewest units, so the whole grid is resident at once).
// Returns unit boundaries (chunk offsets relative to the stream section).
inline void pack_units(const std::vector<int>& run_chunks, int lmax, int gcap, std::vector<int>& ub,
                       bool fill = false) {
  ub.clear();
  ub.push_back(0);
  int cur = 0, genes = 0, pos = 0;
  for (int nch : run_chunks) {
    if (cur > 0 && (genes + 1 > gcap || cur >= lmax || (!fill && cur + nch > lmax))) {
      ub.push_back(pos);
      cur = 0;
      genes = 0;
    }
    while (nch > 0) {
      const int take = std::min(nch, lmax - cur);
      cur += take;
      pos += take;
      nch -= take;
      if (nch > 0) {  // split: the run continues in the next unit
        ub.push_back(pos);
        cur = 0;
        genes = 0;
      }
    }
    genes += 1;
  }
  if (cur > 0) ub.push_back(pos);
}

// Large-K stream-0 packing (the pass kernel's one unit per wave): WORKGROUPS first — whole runs while
// the workgroup holds at most `gcap` genes (its V tables) and NW * lmax chunks, a run longer than
// that split into workgroup-sized pieces — then each workgroup's chunks split evenly over its NW
// units, across gene boundaries (a unit may hold several stretches; a run may span units).  A
// workgroup lives as long as its longest wave: with one run per unit (pack_units at K = 30 on 10M
// links: ~5 genes of ~50 chunks per workgroup) 3 of the 8 waves had nothing to do.
// Returns NW unit boundaries per workgroup (units may be empty when a workgroup has < NW chunks).
inline void pack_balanced(const std::vector<int>& run_chunks, int lmax, int gcap, std::vector<int>& ub,
                          int nw = NW) {
  ub.assign(1, 0);
  const int cap = nw * std::max(lmax, 1);
  int pos = 0, cur = 0, genes = 0, w0 = 0;
  auto close = [&]() {
    const long long n = pos - w0;
    for (int i = 1; i <= nw; ++i) ub.push_back(w0 + (int)(i * n / nw));
    w0 = pos;
    cur = 0;
    genes = 0;
  };
  for (int nch : run_chunks) {
    if (cur > 0 && (genes + 1 > gcap || cur + nch > cap)) close();
    while (nch > 0) {
      const int take = std::min(nch, cap - cur);
      cur += take;
      pos += take;
      nch -= take;
      if (nch > 0) close();  // the run continues in the next workgroup
    }
    genes += 1;
  }
  if (cur > 0) close();
}

// Slot layout of a small-K plan (see Plan::sk_*), from the per-unit descriptors and row12.
inline void make_slots(Plan& pl) {
  const int R = pl.R;
  const int n_wg = (int)pl.wg_code.size();
  // section ends
  {
    int sec = 0;
    for (int w = 0; w < n_wg; ++w) {
      const int code = (pl.wg_code[w] >> 4) * R + (pl.wg_code[w] & 15);
      while (sec < code) pl.sk_wg_end[sec++] = w;
    }
    while (sec < 3 * R) pl.sk_wg_end[sec++] = n_wg;
  }
  std::vector<long long> pos(pl.rows.size(), -1);  // slot-major position of every real row
  for (int g = 0; g < 2; ++g) {
    const int w0 = g == 0 ? 0 : pl.n_wg_a, w1 = g == 0 ? pl.n_wg_a : n_wg;
    const int per = NW * (g == 0 ? pl.rounds_a : pl.rounds_b);
    int L = 1;
    for (int w = w0; w < w1; ++w)
      for (int u = pl.wg_ustart[w]; u < pl.wg_ustart[w + 1]; ++u) {
        const int* d = &pl.udesc[(size_t)u * UD];
        L = std::max(L, d[D_END] - d[0]);
      }
    pl.sk_L[g] = L;
    pl.sk_slots[g] = (long long)(w1 - w0) * per;
    pl.sk_udesc[g].assign((size_t)pl.sk_slots[g] * UD, 0);
    pl.sk_urec[g].assign((size_t)pl.sk_slots[g] * 4 * L, I4{0, 0, 0, 0});
    for (int w = w0; w < w1; ++w)
      for (int k = 0; k < per; ++k) {
        const long long slot = (long long)(w - w0) * per + k;
        int* sd = &pl.sk_udesc[g][(size_t)slot * UD];
        const int u = pl.wg_ustart[w] + k;
        if (u >= pl.wg_ustart[w + 1]) {  // empty slot
          sd[D_CODE] = pl.wg_code[w];
          continue;
        }
        const int* d = &pl.udesc[(size_t)u * UD];
        const int c0 = d[0];
        for (int t = 0; t < UD; ++t) sd[t] = d[t];
        for (int t = 0; t <= D_END; ++t) sd[t] = d[t] - c0;
        if (!pl.prow_y.empty())  // SK_Y: a stretch's X^0 row goes to its Y entry
          for (int t = 0; t < d[D_NST]; ++t) sd[D_PROW + t] = pl.prow_y[(size_t)d[D_PROW + t]];
        else if (!pl.prow_g.empty())  // a stretch's X row goes to its gene-major position
          for (int t = 0; t < d[D_NST]; ++t) sd[D_PROW + t] = pl.prow_g[(size_t)d[D_PROW + t]];
        I4* rec = &pl.sk_urec[g][(size_t)slot * 4 * L];
        const long long row0 = 4LL * c0, nrow = 4LL * (d[D_END] - c0);
        for (long long i = 0; i < 4LL * L; ++i) {
          const long long row = row0 + (i < nrow ? i : nrow - 1);  // padding: the unit's last row
          // (u gene, v gene, pivot gene, n) in the slot's stream order: stream 0 (j, k, i),
          // stream 1 (i, k, j), stream 2 (i, j, k); n = the count (streams 1, 2: the stream-0 row's
          // w, 0 on padding rows; pass B reads c by position and ignores it)
          const I4 x = pl.rows[row];
          const int st = pl.wg_code[w] >> 4;
          const int n = g == 0 ? x.w : (x.w < pl.n_rows0 ? pl.rows[x.w].w : 0);
          rec[i] = st == 0 ? I4{x.y, x.z, x.x, n} : st == 1 ? I4{x.x, x.z, x.y, n} : I4{x.x, x.y, x.z, n};
          if (i < nrow) pos[row] = slot * 4 * L + i;
        }
      }
  }
  if (!pl.row_y.empty()) {  // SK_Y: each slot row's Y entries (n_y: padding, never a real store)
    const int L = pl.sk_L[0];
    pl.sk_urow12.assign((size_t)pl.sk_slots[0] * 4 * L * 2, (int)pl.n_y);
    for (long long q = 0; q < pl.n_rows0; ++q)
      if (pos[q] >= 0)
        for (int k = 0; k < 2; ++k) pl.sk_urow12[(size_t)2 * pos[q] + k] = pl.row_y[(size_t)2 * q + k];
  }
  if (!pl.row12.empty()) {
    const int L = pl.sk_L[0];
    pl.sk_urow12.assign((size_t)pl.sk_slots[0] * 4 * L * 2, -1);
    for (long long q = 0; q < pl.n_rows0; ++q) {
      if (pos[q] < 0) continue;
      for (int k = 0; k < 2; ++k) {
        const int t = pl.row12[(size_t)2 * q + k];
        pl.sk_urow12[(size_t)2 * pos[q] + k] = t < 0 ? -1 : (int)pos[pl.n_rows0 + t];
      }
    }
  }
}

// Builds the plan.  units_a / units_b: the number of units to aim for in stream 0 and in streams
// 1 + 2 together (about 8 waves per CU); gcap: most distinct genes per stream-0 workgroup (its
// V table lives in LDS); sp_rows: stream-0 partial rows per S-partial workgroup (each writes a
// K^3 partial, so large K wants more rows per partial), at most sp_cap of them per rating.
inline Plan build(const int32_t* ids, const int32_t* counts, long long E, int R, int P, bool em,
                  int units_a, int units_b, int gcap, int sp_rows = 16, bool small = false,
                  int wg_target = 1024, bool fill = false, int gu = GU, int rho_pct = 85,
                  bool yent = false, bool balance = true, bool merge = false, int sp_cap = 256,
                  int nw = NW) {
  Plan pl;
  pl.nw = small ? NW : std::max(1, std::min(nw, NW));
  pl.merge = merge && balance && !small && em;
  pl.gu = std::max(1, std::min(gu, GU));
  pl.R = R;
  pl.P = P;
  // large-K EM plans, and small-K EM plans with `yent` (sk.h SK_Y): stream 0 + Y entries
  const bool ymode = em && (!small || yent);
  pl.streams = (em && !ymode) ? 3 : 1;
  pl.small = small;
  // observations of each rating in link order
  std::vector<std::vector<int>> obs(R);
  for (long long e = 0; e < E; ++e)
    for (int r = 0; r < R; ++r)
      if (counts[e * R + r] > 0) obs[r].push_back((int)e);
  for (int r = 0; r < R; ++r) pl.n_obs += (long long)obs[r].size();

  // stream-0 row of each observation (e, r): for the c index of streams 1, 2
  std::vector<std::vector<int>> row0(R);
  if (em) pl.prow_ptr.assign((size_t)3 * R * (P + 1), 0);

  // chunk counts of every (stream, rating) for the unit length
  auto sorted_by = [&](int s, int r) {
    // counting sort by pivot gene (stable)
    const std::vector<int>& o = obs[r];
    std::vector<int> cnt(P + 1, 0);
    for (int e : o) cnt[ids[(size_t)e * 3 + s] + 1]++;
    for (int g = 0; g < P; ++g) cnt[g + 1] += cnt[g];
    std::vector<int> out(o.size());
    for (int e : o) out[cnt[ids[(size_t)e * 3 + s]]++] = e;
    return out;
  };

  long long chunks_a = 0, chunks_b = 0;
  std::vector<std::vector<int>> order((size_t)3 * R);
  for (int s = 0; s < pl.streams; ++s)
    for (int r = 0; r < R; ++r) {
      order[s * R + r] = sorted_by(s, r);
      const auto& o = order[s * R + r];
      long long nch = 0;
      for (size_t q = 0; q < o.size();) {
        const int g = ids[(size_t)o[q] * 3 + s];
        size_t q1 = q;
        while (q1 < o.size() && ids[(size_t)o[q1] * 3 + s] == g) ++q1;
        nch += (long long)((q1 - q + CH - 1) / CH);
        q = q1;
      }
      (s == 0 ? chunks_a : chunks_b) += nch;
    }
  // unit length: the work spread over about units_* units, but no unit longer than LCAP chunks
  // (large link sets get more units rather than longer ones, so a few long units do not set
  // the kernel's duration).  Fill-packed small plans (the fused launch) take units_a as the
  // number of units for all streams together (about the waves that are resident at once); a
  // stream-0 unit is rho_pct % of the others' length (it also owns its genes' X contraction and
  // S outer products, so a shorter chunk loop evens the waves' finish; 85 % measured best of
  // 55 / 70 / 85 / 100 on fold0 K=10, profiles/r03ad_rho_ab.txt), streams 1 / 2 at least one block.
  const long long LCAP = small ? LCAP_SK : 64;
  int lmax_a = (int)std::min(LCAP, std::max<long long>(2, (chunks_a + units_a - 1) / std::max(units_a, 1)));
  int lmax_b = (int)std::min(LCAP, std::max<long long>(2, (chunks_b + units_b - 1) / std::max(units_b, 1)));
  if (small && fill) {
    const double rho = std::max(10, std::min(100, rho_pct)) / 100.0;
    const double lb = ((double)chunks_a / rho + (double)chunks_b) / std::max(units_a, 1);
    lmax_b = (int)std::min<double>(LCAP, std::max<double>(SK_BLOCK, std::ceil(lb)));
    lmax_a = (int)std::min<double>(LCAP, std::max<double>(rho < 1.0 ? 4.0 : SK_BLOCK, std::ceil(rho * lb)));
  }
  pl.lmax[0] = lmax_a;
  pl.lmax[1] = lmax_b;
  if (small) {  // one unit per wave: rounds stay 1 (wg_target is kept for the plan checker)
    pl.rounds_a = pl.rounds_b = 1;
    (void)wg_target;
    pl.wg_ustart.push_back(0);
  }

  std::vector<int> wg_stream;
  for (int s = 0; s < pl.streams; ++s) {
    for (int r = 0; r < R; ++r) {
      const auto& o = order[s * R + r];
      const long long row_base = (long long)pl.rows.size();
      const int chunk_base = (int)(row_base / CH);
      // rows + runs
      std::vector<int> run_chunks, run_gene;
      std::vector<int> pos0;  // stream-0 row of each obs of rating r, indexed like obs[r]
      for (size_t q = 0; q < o.size();) {
        const int g = ids[(size_t)o[q] * 3 + s];
        size_t q1 = q;
        while (q1 < o.size() && ids[(size_t)o[q1] * 3 + s] == g) ++q1;
        for (size_t t = q; t < q1; ++t) {
          const int e = o[t];
          I4 rec{ids[(size_t)e * 3], ids[(size_t)e * 3 + 1], ids[(size_t)e * 3 + 2], 0};
          if (s == 0) {
            rec.w = counts[(size_t)e * R + r];
          } else {
            rec.w = -1;  // filled below from the stream-0 row map
          }
          pl.rows.push_back(rec);
        }
        const int n = (int)(q1 - q);
        const int pad = (CH - n % CH) % CH;
        for (int t = 0; t < pad; ++t) pl.rows.push_back(I4{g, g, g, s == 0 ? 0 : -2});
        run_chunks.push_back((n + pad) / CH);
        run_gene.push_back(g);
        q = q1;
      }
      // units
      std::vector<int> ub;
      const bool bal = balance && !small && s == 0;  // units NW per workgroup, even lengths
      if (bal)
        pack_balanced(run_chunks, lmax_a, gcap, ub, pl.nw);
      else
        pack_units(run_chunks, s == 0 ? lmax_a : lmax_b, small ? pl.gu : s == 0 ? gcap : (1 << 30), ub,
                   small && fill);
      const int nunits = (int)ub.size() - 1;
      // chunk -> gene
      const int nch = ub.empty() ? 0 : ub.back();
      std::vector<int> cgene(nch);
      {
        int c = 0;
        for (size_t k = 0; k < run_chunks.size(); ++k)
          for (int t = 0; t < run_chunks[k]; ++t) cgene[c++] = run_gene[k];
      }
      if (small) {
        // workgroups: rounds of NW consecutive units of this (stream, rating); unit descriptors
        const int per = NW * (s == 0 ? pl.rounds_a : pl.rounds_b);
        const long long u_first = pl.n_units;
        for (int u = 0; u < nunits; ++u) {
          int d[UD];
          const int c0 = ub[u], c1 = ub[u + 1];
          int nst = 0;
          for (int c = c0; c < c1; ++c)
            if (c == c0 || cgene[c] != cgene[c - 1]) {
              d[nst] = chunk_base + c;      // stretch start
              d[D_GENE + nst] = cgene[c];   // its pivot gene
              ++nst;
            }
          for (int t = nst; t < GU; ++t) {
            d[t] = chunk_base + c1;
            d[D_GENE + t] = cgene[c0];
          }
          d[D_END] = chunk_base + c1;
          d[D_NST] = nst;
          for (int t = 0; t < GU; ++t) d[D_PROW + t] = -1;  // partial rows: filled below (em plans)
          d[D_CODE] = s * 16 + r;
          for (int t = D_CODE + 1; t < UD; ++t) d[t] = 0;
          pl.udesc.insert(pl.udesc.end(), d, d + UD);
        }
        pl.n_units += nunits;
        for (int u = 0; u < nunits; u += per) {
          pl.wg_ustart.push_back((int)(u_first + std::min(u + per, nunits)));
          pl.wg_code.push_back(s * 16 + r);
          wg_stream.push_back(s);
        }
      } else {
        // workgroups: NW consecutive units; stream 0 also caps the distinct genes (V table)
        std::vector<int> wstart;  // unit index where each workgroup starts
        if (bal) {
          for (int u = 0; u < nunits; u += pl.nw) wstart.push_back(u);
        } else {
          int u = 0;
          while (u < nunits) {
            wstart.push_back(u);
            int taken = 0, genes = 0, last = -1;
            while (u < nunits && taken < pl.nw) {
              int ug = 0, lg = last;
              for (int c = ub[u]; c < ub[u + 1]; ++c)
                if (cgene[c] != lg) {
                  ++ug;
                  lg = cgene[c];
                }
              if (s == 0 && taken > 0 && genes + ug > gcap) break;
              genes += ug;
              last = lg;
              ++taken;
              ++u;
            }
          }
        }
        for (size_t w = 0; w < wstart.size(); ++w) {
          const int u0 = wstart[w];
          const int u1 = w + 1 < wstart.size() ? wstart[w + 1] : nunits;
          for (int i = 0; i <= pl.nw; ++i) {
            const int u = std::min(u0 + i, u1);
            pl.wg_units.push_back(chunk_base + ub[u]);
          }
          pl.wg_code.push_back(s * 16 + r);
          wg_stream.push_back(s);
          if (s == 0) {
            pl.wg_gene.push_back((int)pl.vgenes.size());
            const int first = (int)pl.vgenes.size();
            for (int c = ub[u0]; c < ub[u1]; ++c)
              if ((int)pl.vgenes.size() == first || pl.vgenes.back() != cgene[c]) pl.vgenes.push_back(cgene[c]);
            for (int c = ub[u0]; c < ub[u1]; ++c) {
              // genes ascend within the stream, so the slot is a lower_bound in this list
              const auto it = std::lower_bound(pl.vgenes.begin() + first, pl.vgenes.end(), cgene[c]);
              pl.chunk_vslot.push_back((int)(it - (pl.vgenes.begin() + first)));
            }
            pl.gmax = std::max(pl.gmax, (int)pl.vgenes.size() - first);
          }
        }
      }
      if (s != 0) pl.chunk_vslot.resize(pl.chunk_vslot.size() + nch, 0);
      // partial rows: a new one at every unit start and every gene change inside a unit; with
      // `merge` (balanced large-K plans) at every workgroup start and gene change: the waves that
      // share a gene's run add their parts in the workgroup (pass kernel) before one store
      if (em) {
        int* ptr = &pl.prow_ptr[((size_t)s * R + r) * (P + 1)];
        const long long first_prow = pl.n_prows;
        int u = 0;
        for (int c = 0; c < nch; ++c) {
          while (u + 1 < (int)ub.size() && ub[u + 1] <= c) ++u;
          const int start = (bal && merge) ? ub[(u / pl.nw) * pl.nw] : ub[u];
          if (c == start || cgene[c] != cgene[c - 1]) {
            pl.prow_gene.push_back(cgene[c]);
            ++pl.n_prows;
          }
          pl.chunk_prow.push_back((int)(pl.n_prows - 1));
        }
        if (small) {  // each unit stretch's partial row
          const long long u_first = pl.n_units - (long long)(ub.size() - 1);
          for (int u = 0; u + 1 < (int)ub.size(); ++u) {
            int* d = &pl.udesc[(size_t)(u_first + u) * UD];
            for (int t = 0; t < d[D_NST]; ++t) d[D_PROW + t] = pl.chunk_prow[(size_t)d[t]];
          }
        }
        // CSR over genes: prows of stream (s, r) ascend by gene
        std::vector<int> cnt(P + 1, 0);
        for (long long q = first_prow; q < pl.n_prows; ++q) cnt[pl.prow_gene[q] + 1]++;
        ptr[0] = (int)first_prow;
        for (int g = 0; g < P; ++g) ptr[g + 1] = ptr[g] + cnt[g + 1];
      } else {
        pl.chunk_prow.resize(pl.chunk_prow.size() + nch, -1);
      }
      if (s == 0) {
        // stream-0 row of every observation of rating r
        std::vector<int>& m = row0[r];
        m.assign(E, -1);
        long long rr = row_base;
        for (size_t q = 0; q < o.size();) {
          const int g = ids[(size_t)o[q] * 3];
          size_t q1 = q;
          while (q1 < o.size() && ids[(size_t)o[q1] * 3] == g) ++q1;
          for (size_t t = q; t < q1; ++t) m[o[t]] = (int)(rr++);
          rr += (CH - (long long)(q1 - q) % CH) % CH;
          q = q1;
        }
        pl.n_rows0 = (long long)pl.rows.size();
        if (small && em && !ymode) pl.row12.resize((size_t)2 * pl.n_rows0, -1);
      } else {
        // c index of every row of this stream section
        size_t rr = (size_t)row_base;
        for (size_t q = 0; q < o.size();) {
          const int g = ids[(size_t)o[q] * 3 + s];
          size_t q1 = q;
          while (q1 < o.size() && ids[(size_t)o[q1] * 3 + s] == g) ++q1;
          for (size_t t = q; t < q1; ++t) {
            const int r0 = row0[r][o[t]];
            if (small) pl.row12[(size_t)2 * r0 + (s - 1)] = (int)((long long)rr - pl.n_rows0);
            pl.rows[rr++].w = r0;
          }
          const int pad = (CH - (int)(q1 - q) % CH) % CH;
          for (int t = 0; t < pad; ++t) pl.rows[rr++].w = -2;
          q = q1;
        }
      }
    }
    if (s == 0) pl.n_wg_a = (int)pl.wg_code.size();
  }
  pl.n_wg_b = (int)pl.wg_code.size() - pl.n_wg_a;
  pl.wg_gene.push_back((int)pl.vgenes.size());
  if (ymode) {
    // Y entries: every observation's slot-1 and slot-2 gene, grouped by gene (counting sort,
    // stable over slot, rating, link order)
    pl.yptr.assign((size_t)P + 1, 0);
    for (int s = 1; s <= 2; ++s)
      for (int r = 0; r < R; ++r)
        for (int e : obs[r]) pl.yptr[(size_t)ids[(size_t)e * 3 + s] + 1]++;
    // small-K SK_Y plans: a gene's X^0 partial rows (K words each, written by the pass at its
    // stretch ends) follow its observation entries, rating then row order, so fin sums one range
    if (small)
      for (long long q = 0; q < pl.n_prows; ++q) pl.yptr[(size_t)pl.prow_gene[q] + 1]++;
    for (int g = 0; g < P; ++g) pl.yptr[g + 1] += pl.yptr[g];
    pl.n_y = pl.yptr[P];
    std::vector<int> pos(pl.yptr.begin(), pl.yptr.end() - 1);
    pl.row_y.assign((size_t)2 * pl.n_rows0, (int)pl.n_y);
    for (int s = 1; s <= 2; ++s)
      for (int r = 0; r < R; ++r)
        for (int e : obs[r]) pl.row_y[(size_t)2 * row0[r][e] + (s - 1)] = pos[ids[(size_t)e * 3 + s]]++;
    if (small) {
      pl.prow_y.assign((size_t)pl.n_prows, -1);
      for (int r = 0; r < R; ++r)
        for (int g = 0; g < P; ++g) {
          const int* ptr = &pl.prow_ptr[(size_t)r * (P + 1)];
          for (int q = ptr[g]; q < ptr[g + 1]; ++q) pl.prow_y[q] = pos[g]++;
        }
    }
  }
  for (auto& rec : pl.rows)
    if (rec.w == -2) rec.w = (int)pl.n_rows0;  // padding rows of streams 1, 2: the zero c slot
  if (small) {
    // S partials: one per stream-0 workgroup; those of rating r are workgroups [sp_lo, sp_hi)
    for (int r = 0; r < R; ++r) {
      pl.sp_lo[r] = pl.sp_hi[r] = 0;
      bool seen = false;
      for (int w = 0; w < pl.n_wg_a; ++w)
        if ((pl.wg_code[w] & 15) == r) {
          if (!seen) pl.sp_lo[r] = w;
          seen = true;
          pl.sp_hi[r] = w + 1;
        }
    }
    pl.n_sp = pl.n_wg_a;
    if (em && !ymode) {  // gene-major X partial rows
      pl.gptr.assign((size_t)P + 1, 0);
      for (long long q = 0; q < pl.n_prows; ++q) pl.gptr[(size_t)pl.prow_gene[q] + 1]++;
      for (int g = 0; g < P; ++g) pl.gptr[g + 1] += pl.gptr[g];
      std::vector<int> at(pl.gptr.begin(), pl.gptr.end() - 1);
      pl.prow_g.assign((size_t)pl.n_prows, -1);
      for (int c = 0; c < 3 * R; ++c)
        for (int g = 0; g < P; ++g) {
          const int* ptr = &pl.prow_ptr[(size_t)c * (P + 1)];
          for (int q = ptr[g]; q < ptr[g + 1]; ++q) pl.prow_g[q] = at[g]++;
        }
    }
    make_slots(pl);
    return pl;
  }
  // S-partial workgroups over the stream-0 partial rows of each rating
  if (em) {
    for (int r = 0; r < R; ++r) {
      const int q0 = pl.prow_ptr[(size_t)r * (P + 1)];
      const int q1 = pl.prow_ptr[(size_t)r * (P + 1) + P];
      pl.sp_lo[r] = pl.n_sp;
      const int n = q1 - q0;
      const int parts = n <= 0 ? 0 : std::min(sp_cap, std::max(1, (n + sp_rows - 1) / std::max(sp_rows, 1)));
      for (int k = 0; k < parts; ++k) {
        pl.sp_desc.push_back(r);
        pl.sp_desc.push_back(q0 + (int)((long long)n * k / parts));
        pl.sp_desc.push_back(q0 + (int)((long long)n * (k + 1) / parts));
        ++pl.n_sp;
      }
      pl.sp_hi[r] = pl.n_sp;
    }
    if (pl.n_sp == 0) {  // no observation at all: one empty S workgroup still snapshots p
      pl.sp_desc.insert(pl.sp_desc.end(), {0, 0, 0});
      pl.n_sp = 1;
      pl.sp_hi[0] = 1;
    }
  }
  return pl;
}

}  // namespace mmsbm_plan
