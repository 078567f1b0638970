"""Compile-time ablation switches for the fused kernel (EMX_AB, measurement builds only) and an
MMSBM_LIB override of the library path (measurement)."""
R = '/root/repo/'


def sub(path, old, new):
    s = open(R + path).read()
    assert old in s, (path, old[:60])
    open(R + path, 'w').write(s.replace(old, new, 1))


H = 'trigenicinteractionpredictor_amd/csrc/mmsbm.hip'
sub(H, '''constexpr int XG = 16;  // observations per wave group''', '''constexpr int XG = 16;  // observations per wave group

// Measurement builds only (-DEMX_AB=mask): bit 0 U-phase MFMAs, 1 W-phase MFMAs, 2 S-phase
// MFMAs replaced by VALU adds of the same operands; 3 no contribution stores; 4 no KR stores.
#ifndef EMX_AB
#define EMX_AB 0
#endif''')
sub(H, '''        for (int bb = 0; bb < NG; ++bb) acc[bb] = mfma4(aU[s], bf[bb][s], acc[bb]);''',
    '''        for (int bb = 0; bb < NG; ++bb)
          acc[bb] = (EMX_AB & 1) ? acc[bb] + aU[s] + bf[bb][s] : mfma4(aU[s], bf[bb][s], acc[bb]);''')
sub(H, '''        for (int bq = 0; bq < K; ++bq) KRo[a * K + bq] = ct * tj[bq];''',
    '''        for (int bq = 0; bq < K; ++bq)
          if (!(EMX_AB & 16)) KRo[a * K + bq] = ct * tj[bq];''')
sub(H, '''      for (int u = 0; u < NG; ++u) wacc[u] = mfma4(av, pb[4 * u], wacc[u]);
    }
    unsigned long long t3 = tr.now();''', '''      for (int u = 0; u < NG; ++u)
        wacc[u] = (EMX_AB & 2) ? wacc[u] + av + pb[4 * u] : mfma4(av, pb[4 * u], wacc[u]);
    }
    unsigned long long t3 = tr.now();''')
sub(H, '''    {
      const bool real = qD.x >= 0;  // padding observations write the trash row (nnz)''',
    '''    if (!(EMX_AB & 8)) {
      const bool real = qD.x >= 0;  // padding observations write the trash row (nnz)''')
sub(H, '''        for (int u = 0; u < NG; ++u) sacc[t][u] = mfma4(av, bS[u], sacc[t][u]);''',
    '''        for (int u = 0; u < NG; ++u)
          sacc[t][u] = (EMX_AB & 4) ? sacc[t][u] + av + bS[u] : mfma4(av, bS[u], sacc[t][u]);''')
sub('trigenicinteractionpredictor_amd/_lib.py', '''    if _lib is not None:
        return _lib''', '''    if _lib is not None:
        return _lib
    path = os.environ.get("MMSBM_LIB", path)  # measurement builds (tools/); default: in-tree build''')
print('ok')
