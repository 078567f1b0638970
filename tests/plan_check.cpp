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
  const Plan pl = build(ids.data(), counts.data(), E, R, P, true, ua, ub, gcap, sp_rows);

  // 1. every observation appears once per stream, with its count on stream 0 and its stream-0
  //    row on streams 1 / 2; padding rows carry a zero count / the zero c slot
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
    for (int u = 0; u < NW; ++u) {
      const int c0 = pl.wg_units[w * (NW + 1) + u], c1 = pl.wg_units[w * (NW + 1) + u + 1];
      if (c1 < c0) return fail("unit bounds", w, u);
      if (c1 - c0 > 64) return fail("unit over 64 chunks", w, c1 - c0);
      for (int c = c0; c < c1; ++c) covered[c]++;
    }
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
  printf("ok %zu %d %d %lld %d\n", pl.rows.size(), n_wg * NW, n_wg, pl.n_prows, pl.n_sp);
  return 0;
}
