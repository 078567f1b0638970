// Host-side check of the engine's work plan (csrc/plan.h), built and run by tests/test_plan.py
// on the CPU.  Reads a link table on stdin:
//   E R P units_a units_b gcap sp_rows
//   then E lines of "i j k n_0 .. n_{R-1}"
// builds the EM plan and checks its invariants; prints "ok <rows> <units> <wgs> <prows> <n_sp>"
// or "FAIL <what>" (exit 1).
#include <cstdio>
#include <cstdlib>
#include <map>
#include <set>
#include <tuple>
#include <vector>

#include "../trigenicinteractionpredictor_amd/csrc/plan.h"

using namespace mmsbm_plan;

static int fail(const char* what, long long a = 0, long long b = 0) {
  printf("FAIL %s %lld %lld\n", what, a, b);
  return 1;
}

// Y entries (large-K EM plans and small-K SK_Y plans, stream 0 only): yptr tiles
// [0, n_y = 2 x observations), an entry of gene g's range is named by exactly one (stream-0 row,
// slot 1 / 2) whose slot gene is g, and padding rows name the dummy entry n_y
static int check_y(const Plan& pl, int P, long long n_obs) {

  const bool py = !pl.prow_y.empty();  // SK_Y: the partial rows are Y entries too
  if (pl.n_y != 2 * n_obs + (py ? pl.n_prows : 0) || (int)pl.yptr.size() != P + 1 || pl.yptr[0] != 0 ||
      pl.yptr[P] != pl.n_y)
    return fail("yptr", pl.n_y, 2 * n_obs);
  if ((long long)pl.row_y.size() != 2 * pl.n_rows0) return fail("row_y size");
  {
    std::vector<int> owner(pl.n_y, -1), hits(pl.n_y, 0);
    for (int g = 0; g < P; ++g) {
      if (pl.yptr[g + 1] < pl.yptr[g]) return fail("yptr order", g);
      for (int e = pl.yptr[g]; e < pl.yptr[g + 1]; ++e) owner[e] = g;
    }
    for (long long q = 0; q < pl.n_rows0; ++q) {
      const I4& x = pl.rows[q];
      for (int k = 0; k < 2; ++k) {
        const int e = pl.row_y[2 * q + k];
        if (x.w <= 0) {
          if (e != pl.n_y) return fail("row_y padding", q, e);
          continue;
        }
        if (e < 0 || e >= pl.n_y) return fail("row_y range", q, e);
        if (owner[e] != (k == 0 ? x.y : x.z)) return fail("row_y gene", q, e);
        hits[e]++;
      }
    }
    for (long long q = 0; py && q < pl.n_prows; ++q) {
      const int e = pl.prow_y[q];
      if (e < 0 || e >= pl.n_y || owner[e] != pl.prow_gene[q]) return fail("prow_y gene", q, e);
      hits[e]++;
    }
    for (long long e = 0; e < pl.n_y; ++e)
      if (hits[e] != 1) return fail("y entry coverage", e, hits[e]);
  }
  return 0;
}

// Small-K plan: units of at most GU stretches and LCAP_SK chunks covering every chunk once, their
// descriptors (stretch starts, pivot genes, partial rows), workgroup unit ranges of one
// (stream, rating), the c scatter map row12, and the S-partial workgroup ranges.
static int check_small(const Plan& pl, int R, int P, long long nch) {
  if ((long long)pl.udesc.size() != pl.n_units * UD) return fail("udesc size");
  const int n_wg = pl.n_wg_a + pl.n_wg_b;
  if ((int)pl.wg_ustart.size() != n_wg + 1 || pl.wg_ustart[0] != 0 || pl.wg_ustart[n_wg] != pl.n_units)
    return fail("wg_ustart");
  std::vector<int> covered(nch, 0);
  for (int w = 0; w < n_wg; ++w) {
    const int s = pl.wg_code[w] >> 4, r = pl.wg_code[w] & 15;
    if ((w < pl.n_wg_a) != (s == 0)) return fail("stream order", w, s);
    const int rounds = s == 0 ? pl.rounds_a : pl.rounds_b;
    if (pl.wg_ustart[w + 1] - pl.wg_ustart[w] > NW * rounds || pl.wg_ustart[w + 1] <= pl.wg_ustart[w])
      return fail("wg units", w, pl.wg_ustart[w + 1] - pl.wg_ustart[w]);
    for (int u = pl.wg_ustart[w]; u < pl.wg_ustart[w + 1]; ++u) {
      const int* d = &pl.udesc[(size_t)u * UD];
      if (d[D_CODE] != pl.wg_code[w]) return fail("unit code", u, d[D_CODE]);
      const int nst = d[D_NST], c0 = d[0], c1 = d[D_END];
      if (nst < 1 || nst > pl.gu) return fail("stretches", u, nst);
      if (c1 - c0 > LCAP_SK || c1 <= c0) return fail("unit length", u, c1 - c0);
      for (int t = 0; t < GU; ++t) {
        const int a = d[t], b = t + 1 < nst ? d[t + 1] : c1;
        if (t >= nst) {
          if (a != c1) return fail("empty stretch start", u, t);
          continue;
        }
        if (b <= a) return fail("stretch order", u, t);
        const int q = d[D_PROW + t], g = d[D_GENE + t];
        if (q < 0 || q >= pl.n_prows || pl.prow_gene[q] != g) return fail("stretch prow", u, t);
        if (t > 0 && d[D_GENE + t - 1] == g) return fail("stretch not maximal", u, t);
        for (int c = a; c < b; ++c) {
          covered[c]++;
          if (pl.chunk_prow[c] != q) return fail("chunk prow", c, q);
          for (int k = 0; k < CH; ++k) {
            const I4& x = pl.rows[(long long)c * CH + k];
            if ((s == 0 ? x.x : s == 1 ? x.y : x.z) != g) return fail("stretch gene", c, k);
          }
        }
      }
    }
    (void)r;
  }
  for (long long c = 0; c < nch; ++c)
    if (covered[c] != 1) return fail("chunk coverage", c, covered[c]);
  // row12: the stream-1 / stream-2 rows of each real stream-0 row hold the same triple and point
  // back at it; padding rows map to -1
  const bool yent = !pl.row_y.empty();
  if (!yent && (long long)pl.row12.size() != 2 * pl.n_rows0) return fail("row12 size");
  for (long long q = 0; q < (yent ? 0 : pl.n_rows0); ++q) {
    const I4& x = pl.rows[q];
    for (int k = 0; k < 2; ++k) {
      const int t = pl.row12[2 * q + k];
      if (x.w <= 0) {
        if (t != -1) return fail("row12 padding", q, t);
        continue;
      }
      if (t < 0 || pl.n_rows0 + t >= (long long)pl.rows.size()) return fail("row12 range", q, t);
      const I4& y = pl.rows[pl.n_rows0 + t];
      if (y.x != x.x || y.y != x.y || y.z != x.z || y.w != q) return fail("row12 target", q, t);
    }
  }
  for (int r = 0; r < R; ++r)
    for (int w = 0; w < pl.n_wg_a; ++w)
      if (((pl.wg_code[w] & 15) == r) != (w >= pl.sp_lo[r] && w < pl.sp_hi[r])) return fail("sp range", r, w);
  // slots: every unit once, in its workgroup's slot range, records copied slot-major; the slot-major
  // row12 points at the pass-B slot row holding the same observation
  long long units_seen = 0;
  for (int g = 0; g < 2; ++g) {
    const int L = pl.sk_L[g];
    const int w0 = g == 0 ? 0 : pl.n_wg_a, w1 = g == 0 ? pl.n_wg_a : n_wg;
    const int per = NW * (g == 0 ? pl.rounds_a : pl.rounds_b);
    if (pl.sk_slots[g] != (long long)(w1 - w0) * per) return fail("slots", g, pl.sk_slots[g]);
    for (long long slot = 0; slot < pl.sk_slots[g]; ++slot) {
      const int* d = &pl.sk_udesc[g][(size_t)slot * UD];
      const int w = w0 + (int)(slot / per);
      if (d[D_CODE] != pl.wg_code[w]) return fail("slot code", slot, d[D_CODE]);
      if (d[D_NST] == 0) continue;
      ++units_seen;
      const int u = pl.wg_ustart[w] + (int)(slot % per);
      const int* du = &pl.udesc[(size_t)u * UD];
      if (d[D_END] != du[D_END] - du[0] || d[D_END] > L || d[0] != 0) return fail("slot extent", slot, d[D_END]);
      for (int i = 0; i < 4 * d[D_END]; ++i) {
        const I4& a = pl.sk_urec[g][(size_t)slot * 4 * L + i];
        const I4& b = pl.rows[4LL * du[0] + i];
        // (u, v, pivot, n) in the stream's order; group 1 (streams 1, 2) carries the observation's
        // count n = its stream-0 row's w (0: padding)
        const int bw = g == 0 ? b.w : (b.w < pl.n_rows0 ? pl.rows[b.w].w : 0);
        const int st = d[D_CODE] >> 4;
        const I4 e = st == 0 ? I4{b.y, b.z, b.x, bw} : st == 1 ? I4{b.x, b.z, b.y, bw} : I4{b.x, b.y, b.z, bw};
        if (a.x != e.x || a.y != e.y || a.z != e.z || a.w != e.w) return fail("slot record", slot, i);
        if (g == 1 && b.w < pl.n_rows0 && bw <= 0) return fail("slot count", slot, i);
      }
    }
  }
  if (units_seen != pl.n_units) return fail("slot units", units_seen, pl.n_units);
  if (yent) {  // SK_Y: the slot-major urow12 holds each stream-0 row's Y entries
    if (int rc = check_y(pl, P, pl.n_obs)) return rc;
    if (pl.n_wg_b != 0 || (long long)pl.rows.size() != pl.n_rows0) return fail("SK_Y streams", pl.n_wg_b);
    const int L = pl.sk_L[0];
    const int per = NW * pl.rounds_a;
    for (long long slot = 0; slot < pl.sk_slots[0]; ++slot) {
      const int* d = &pl.sk_udesc[0][(size_t)slot * UD];
      if (d[D_NST] == 0) continue;
      const int u = pl.wg_ustart[(int)(slot / per)] + (int)(slot % per);
      const int* du = &pl.udesc[(size_t)u * UD];
      for (int t = 0; t < d[D_NST]; ++t)
        if (d[D_PROW + t] != pl.prow_y[du[D_PROW + t]]) return fail("SK_Y stretch entry", slot, t);
      for (int i = 0; i < 4 * d[D_END]; ++i)
        for (int k = 0; k < 2; ++k)
          if (pl.sk_urow12[((size_t)slot * 4 * L + i) * 2 + k] != pl.row_y[(4LL * du[0] + i) * 2 + k])
            return fail("SK_Y urow12", slot, i);
    }
  } else {
    // gene-major X partial rows: gptr tiles [0, n_prows), each row's position lies in its gene's
    // range, ranges follow (stream, rating, row) order, and the slot descriptors name positions
    if ((int)pl.gptr.size() != P + 1 || pl.gptr[P] != pl.n_prows || (long long)pl.prow_g.size() != pl.n_prows)
      return fail("gptr", pl.n_prows);
    std::vector<int> seen(pl.n_prows, 0);
    for (long long q = 0; q < pl.n_prows; ++q) {
      const int g = pl.prow_gene[q], e = pl.prow_g[q];
      if (e < pl.gptr[g] || e >= pl.gptr[g + 1]) return fail("prow_g range", q, e);
      if (seen[e]++) return fail("prow_g twice", q, e);
      if (q > 0 && pl.prow_gene[q - 1] == g && pl.prow_g[q - 1] != e - 1) return fail("prow_g order", q, e);
    }
    for (int g2 = 0; g2 < 2; ++g2) {
      const int per = NW * (g2 == 0 ? pl.rounds_a : pl.rounds_b);
      const int w0 = g2 == 0 ? 0 : pl.n_wg_a;
      for (long long slot = 0; slot < pl.sk_slots[g2]; ++slot) {
        const int* d = &pl.sk_udesc[g2][(size_t)slot * UD];
        if (d[D_NST] == 0) continue;
        const int u = pl.wg_ustart[w0 + (int)(slot / per)] + (int)(slot % per);
        const int* du = &pl.udesc[(size_t)u * UD];
        for (int t = 0; t < d[D_NST]; ++t)
          if (d[D_PROW + t] != pl.prow_g[du[D_PROW + t]]) return fail("slot prow_g", slot, t);
      }
    }
    const int La = pl.sk_L[0], Lb = pl.sk_L[1];
    for (long long i = 0; i < pl.sk_slots[0] * 4 * La; ++i) {
      const I4& a = pl.sk_urec[0][i];
      for (int k = 0; k < 2; ++k) {
        const int t = pl.sk_urow12[2 * i + k];
        if (t < 0) continue;
        if (t >= pl.sk_slots[1] * 4 * Lb) return fail("urow12 range", i, t);
        const I4& b = pl.sk_urec[1][t];
        // the same triple (stream 0 holds (j, k, i), streams 1 / 2 (i, k, j) / (i, j, k)) and count
        const int ti = a.z, tj = a.x, tk = a.y;
        const bool same = (b.x == ti && ((b.y == tk && b.z == tj) || (b.y == tj && b.z == tk)));
        if (!same || a.w <= 0 || b.w != a.w) return fail("urow12 target", i, t);
      }
    }
  }
  for (int sec = 0; sec < 3 * R; ++sec) {
    const int lo = sec == 0 ? 0 : pl.sk_wg_end[sec - 1], hi = pl.sk_wg_end[sec];
    for (int w = lo; w < hi; ++w)
      if (((pl.wg_code[w] >> 4) * R + (pl.wg_code[w] & 15)) != sec) return fail("section", sec, w);
  }
  (void)P;
  printf("ok %zu %lld %d %lld %d\n", pl.rows.size(), pl.n_units, n_wg, pl.n_prows, pl.n_sp);
  return 0;
}

int main() {
  long long E;
  int R, P, ua, ub, gcap, sp_rows;
  if (scanf("%lld %d %d %d %d %d %d", &E, &R, &P, &ua, &ub, &gcap, &sp_rows) != 7) return fail("input");
  std::vector<int32_t> ids(E * 3), counts(E * R);
  for (long long e = 0; e < E; ++e) {
    for (int t = 0; t < 3; ++t)
      if (scanf("%d", &ids[e * 3 + t]) != 1) return fail("ids");
    for (int r = 0; r < R; ++r)
      if (scanf("%d", &counts[e * R + r]) != 1) return fail("counts");
  }
  // gcap <= 0: the small-K plans of sk.h (sp_rows = their wg_target): 0 = 4 stretches per unit
  // (K 11-12), -3 = 8 (K <= 10); fill-packed (the fused launch) -1 = 8, -2 = 4; -4 = fill-packed
  // stream-0 plans with Y entries (SK_Y), 8 stretches
  const bool small = gcap <= 0, fill = gcap == -1 || gcap == -2 || gcap == -4, yent = gcap == -4;
  // PLAN_NO_BALANCE=1: the large-K units packed whole-run-wise (round 3, MMSBM_BALANCE=0)
  const bool balance = !getenv("PLAN_NO_BALANCE");
  // PLAN_MERGE=1: one partial row per (workgroup, gene) (the K >= 25 pass kernel merges its waves' parts)
  const bool merge = getenv("PLAN_MERGE") != nullptr;
  const int gu = (gcap == 0 || gcap == -2) ? 4 : 8;
  // PLAN_NW=n: n units per large-K workgroup (the K >= 25 pass kernel runs 4-wave workgroups)
  const int nw_env = getenv("PLAN_NW") ? atoi(getenv("PLAN_NW")) : NW;
  // PLAN_SP_CAP=n: at most n S-partial parts per rating (the large-K product plans take 1,024)
  const int sp_cap = getenv("PLAN_SP_CAP") ? atoi(getenv("PLAN_SP_CAP")) : 256;
  const Plan pl = small ? build(ids.data(), counts.data(), E, R, P, true, ua, ub, 0, 16, true, sp_rows, fill, gu,
                                85, yent)
                        : build(ids.data(), counts.data(), E, R, P, true, ua, ub, gcap, sp_rows, false, 1024,
                                false, GU, 85, false, balance, merge, sp_cap, nw_env);
  if (fill) {  // every unit but the last of its (stream, rating) section is full: LCAP_SK chunks or GU stretches
    for (long long u = 0; u + 1 < pl.n_units; ++u) {
      const int* d = &pl.udesc[(size_t)u * UD];
      const int* dn = &pl.udesc[(size_t)(u + 1) * UD];
      if (dn[D_CODE] != d[D_CODE]) continue;  // the section's last unit
      const int lm = pl.lmax[(d[D_CODE] >> 4) == 0 ? 0 : 1];
      if (d[D_END] - d[0] != lm && d[D_NST] != pl.gu) return fail("fill", (int)u, d[D_END] - d[0]);
    }
  }

  // 1. every observation appears once per stream (small-K plans: 3 streams; large-K: stream 0),
  //    with its count on stream 0 and its stream-0 row on streams 1 / 2; padding rows carry a zero
  //    count / the zero c slot
  long long n_obs = 0;
  for (long long e = 0; e < E; ++e)
    for (int r = 0; r < R; ++r) n_obs += counts[e * R + r] > 0;
  if (pl.n_obs != n_obs) return fail("n_obs", pl.n_obs, n_obs);
  if ((long long)pl.rows.size() % CH) return fail("rows not chunked");
  const long long nch = (long long)pl.rows.size() / CH;
  std::map<std::tuple<int, int, int, int>, long long> seen0;  // (i, j, k, count) multiset
  long long real0 = 0;
  for (long long q = 0; q < pl.n_rows0; ++q) {
    const I4& x = pl.rows[q];
    if (x.w > 0) {
      ++real0;
      ++seen0[{x.x, x.y, x.z, x.w}];
    }
  }
  if (real0 != n_obs) return fail("stream-0 rows", real0, n_obs);
  std::map<std::tuple<int, int, int, int>, long long> want;
  for (long long e = 0; e < E; ++e)
    for (int r = 0; r < R; ++r)
      if (counts[e * R + r] > 0) ++want[{ids[e * 3], ids[e * 3 + 1], ids[e * 3 + 2], counts[e * R + r]}];
  if (seen0 != want) return fail("stream-0 multiset");
  for (long long q = pl.n_rows0; q < (long long)pl.rows.size(); ++q) {
    const I4& x = pl.rows[q];
    if (x.w < 0 || x.w > pl.n_rows0) return fail("c index", q, x.w);
    if (x.w < pl.n_rows0) {  // a real observation: the same triple as its stream-0 row
      const I4& y = pl.rows[x.w];
      if (y.x != x.x || y.y != x.y || y.z != x.z || y.w <= 0) return fail("c row mismatch", q, x.w);
    }
  }

  if (small) return check_small(pl, R, P, nch);
  const int NW = pl.nw;  // units per large-K workgroup
  if (NW != nw_env) return fail("plan nw", NW, nw_env);

  // 2. a chunk has one pivot gene; pivots ascend inside each (stream, rating) section
  // 3. workgroups: NW + 1 nondecreasing unit bounds, units at most 64 chunks, stream-0
  //    workgroups within the gene cap, and chunk_vslot naming the chunk's gene
  const int n_wg = pl.n_wg_a + pl.n_wg_b;
  if ((int)pl.wg_units.size() != n_wg * (NW + 1)) return fail("wg_units size");
  if ((long long)pl.chunk_prow.size() != nch || (long long)pl.chunk_vslot.size() != nch)
    return fail("chunk arrays", pl.chunk_prow.size(), nch);
  std::vector<int> covered(nch, 0);
  for (int w = 0; w < n_wg; ++w) {
    const int s = pl.wg_code[w] >> 4;
    if ((w < pl.n_wg_a) != (s == 0)) return fail("stream order", w, s);
    int umin = 1 << 30, umax = 0;
    for (int u = 0; u < NW; ++u) {
      const int c0 = pl.wg_units[w * (NW + 1) + u], c1 = pl.wg_units[w * (NW + 1) + u + 1];
      if (c1 < c0) return fail("unit bounds", w, u);
      if (c1 - c0 > 64) return fail("unit over 64 chunks", w, c1 - c0);
      umin = std::min(umin, c1 - c0);
      umax = std::max(umax, c1 - c0);
      for (int c = c0; c < c1; ++c) covered[c]++;
    }
    // balanced packing: a workgroup's NW units differ by at most one chunk
    if (balance && umax - umin > 1) return fail("unbalanced units", w, umax - umin);
    if (s == 0) {
      const int g0 = pl.wg_gene[w], g1 = pl.wg_gene[w + 1];
      if (g1 - g0 > gcap || g1 - g0 > pl.gmax) return fail("gene cap", w, g1 - g0);
      for (int c = pl.wg_units[w * (NW + 1)]; c < pl.wg_units[w * (NW + 1) + NW]; ++c) {
        const int vs = pl.chunk_vslot[c];
        if (vs < 0 || vs >= g1 - g0) return fail("vslot range", c, vs);
        if (pl.vgenes[g0 + vs] != pl.rows[(long long)c * CH].x) return fail("vslot gene", c, vs);
      }
    }
  }
  std::vector<int> cstream(nch, -1);
  for (int w = 0; w < n_wg; ++w)
    for (int c = pl.wg_units[w * (NW + 1)]; c < pl.wg_units[w * (NW + 1) + NW]; ++c)
      cstream[c] = pl.wg_code[w] >> 4;
  for (long long c = 0; c < nch; ++c) {
    if (covered[c] != 1) return fail("chunk coverage", c, covered[c]);
    const int s = cstream[c];
    auto comp = [&](const I4& x) { return s == 0 ? x.x : s == 1 ? x.y : x.z; };
    const int g = comp(pl.rows[c * CH]);
    for (int t = 1; t < CH; ++t)
      if (comp(pl.rows[c * CH + t]) != g) return fail("chunk pivot", c, t);
    if (c > 0 && cstream[c - 1] == s && comp(pl.rows[(c - 1) * CH]) > g) {
      // pivots ascend inside a (stream, rating) section; a drop must start a workgroup (the
      // next rating's section)
      bool next_rating = false;
      for (int w = 0; w < n_wg; ++w)
        if (pl.wg_units[w * (NW + 1)] == c) next_rating = true;
      if (!next_rating) return fail("pivot order", c, g);
    }
  }

  // 4. partial rows: one per gene stretch per unit, contiguous per (stream, rating, gene) in
  //    prow_ptr, and a chunk's partial row belongs to the chunk's pivot gene
  for (long long c = 0; c < nch; ++c) {
    const int q = pl.chunk_prow[c];
    if (q < 0 || q >= pl.n_prows) return fail("chunk_prow", c, q);
    if (c * CH < pl.n_rows0 && pl.prow_gene[q] != pl.rows[c * CH].x) return fail("prow gene", c, q);
  }
  for (int s = 0; s < 3; ++s)
    for (int r = 0; r < R; ++r) {
      const int* ptr = &pl.prow_ptr[((size_t)s * R + r) * (P + 1)];
      for (int g = 0; g < P; ++g) {
        if (ptr[g + 1] < ptr[g]) return fail("prow_ptr order", s * R + r, g);
        for (int q = ptr[g]; q < ptr[g + 1]; ++q)
          if (pl.prow_gene[q] != g) return fail("prow_ptr gene", q, g);
      }
    }

  // 4b. merged plans: a partial row's chunks lie in one workgroup, and inside a workgroup a gene's
  //     chunks share one row
  if (merge != pl.merge || (merge && !balance)) return fail("merge flag", pl.merge);
  if (pl.merge) {
    std::vector<int> prow_wg(pl.n_prows, -1);
    for (int w = 0; w < n_wg; ++w) {
      const int c0 = pl.wg_units[w * (NW + 1)], c1 = pl.wg_units[w * (NW + 1) + NW];
      for (int c = c0; c < c1; ++c) {
        const int q = pl.chunk_prow[c];
        if (prow_wg[q] >= 0 && prow_wg[q] != w) return fail("merged row spans workgroups", q, w);
        prow_wg[q] = w;
        if (c > c0) {
          const bool same = pl.rows[(long long)c * CH].x == pl.rows[(long long)(c - 1) * CH].x;
          if (same != (q == pl.chunk_prow[c - 1])) return fail("merged row per gene", c, q);
        }
      }
    }
  }

  // 5. S-partial descriptors tile each rating's stream-0 partial rows
  for (int r = 0; r < R; ++r) {
    const int q0 = pl.prow_ptr[(size_t)r * (P + 1)], q1 = pl.prow_ptr[(size_t)r * (P + 1) + P];
    int at = q0;
    for (int sp = pl.sp_lo[r]; sp < pl.sp_hi[r]; ++sp) {
      if (pl.sp_desc[3 * sp] != r || pl.sp_desc[3 * sp + 1] != at) return fail("sp tiling", r, sp);
      at = pl.sp_desc[3 * sp + 2];
    }
    if (q1 > q0 && at != q1) return fail("sp end", r, at);
  }
  if (int rc = check_y(pl, P, n_obs)) return rc;
  if (pl.n_wg_b != 0 || (long long)pl.rows.size() != pl.n_rows0) return fail("large-K streams", pl.n_wg_b);
  printf("ok %zu %d %d %lld %d\n", pl.rows.size(), n_wg * NW, n_wg, pl.n_prows, pl.n_sp);
  return 0;
}
