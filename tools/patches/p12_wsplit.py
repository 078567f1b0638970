"""W-phase: two accumulator sets (even / odd k-steps) so six MFMA chains are in flight."""
R = '/root/repo/'


def sub(path, old, new, count=1):
    s = open(R + path).read()
    assert s.count(old) >= count, (path, old[:70])
    open(R + path, 'w').write(s.replace(old, new, count))


H = 'trigenicinteractionpredictor_amd/csrc/mmsbm.hip'
sub(H, '''    double wacc[NG];
#pragma unroll
    for (int u = 0; u < NG; ++u) wacc[u] = 0.0;
#pragma unroll
    for (int s = 0; s < NC; ++s) {
      const int cell = 4 * s + hi;
      const double av = KRo[cell];
      const double* pb = Pw + cell * KP + lo;  // rows >= K^2 are zero (KR is zero there too)
#pragma unroll
      for (int u = 0; u < NG; ++u)
        wacc[u] = (EMX_AB & 2) ? wacc[u] + av + pb[4 * u] : mfma4(av, pb[4 * u], wacc[u]);
    }''', '''    // two accumulator sets (even / odd k-steps): 2 NG independent MFMA chains in flight
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
    for (int u = 0; u < NG; ++u) wacc[u] += wacc2[u];''')
print('ok')
