"""Fused kernel: one cell-major p_r image Pw[(a,b)][g] (rows K^2 + KP, zero padded) shared by the
U- and W-phases, so every fragment address is a lane base plus a compile-time offset."""
P = '/root/repo/trigenicinteractionpredictor_amd/csrc/mmsbm.hip'
s = open(P).read()
reps = [
('''  static constexpr int P_DBL = K * KP * KP;   // p_r image [a][b][g], b and g zero padded''',
 '''  static constexpr int PW_ROWS = K2 + KP;     // p_r image rows (a, b) = a K + b, zero padded
  static constexpr int P_DBL = PW_ROWS * KP;  // p_r image [(a, b)][g], g zero padded'''),
('''  double* Pl = smem;  // [K][KP][KP]''',
 '''  double* Pw = smem;  // [K^2 + KP][KP] p_r, row a K + b, columns g'''),
('''  for (int idx = tid; idx < X::P_DBL; idx += NT) {
    const int g = idx % KP, bq = (idx / KP) % KP, a = idx / (KP * KP);
    Pl[idx] = (g < K && bq < K) ? p[(a * K + bq) * K + g] : 0.0;
  }''',
 '''  for (int idx = tid; idx < X::P_DBL; idx += NT) {
    const int g = idx % KP, row = idx / KP;
    Pw[idx] = (g < K && row < K2) ? p[row * K + g] : 0.0;
  }'''),
('''        for (int s = 0; s < NG; ++s) bf[bb][s] = Pl[(a * KP + 4 * bb + lo) * KP + 4 * s + hi];''',
 '''        for (int s = 0; s < NG; ++s)  // b = 4 bb + lo >= K reads the next row: finite, and
          bf[bb][s] = Pw[(a * K + 4 * bb + lo) * KP + 4 * s + hi];  // th_j[b] = 0 drops it'''),
('''      const double* pb = Pl + ((cc / K) * KP + cc % K) * KP + lo;''',
 '''      const double* pb = Pw + cell * KP + lo;  // rows >= K^2 are zero (KR is zero there too)'''),
]
for old, new in reps:
    assert old in s, old[:70]
    s = s.replace(old, new)
open(P, 'w').write(s)
print('ok')
