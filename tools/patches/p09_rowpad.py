"""Fused path: contribution rows padded to 128 B (one cache line each, CROW doubles)."""
R = '/root/repo/'


def sub(path, old, new, count=1):
    s = open(R + path).read()
    assert s.count(old) >= count, (path, old[:70])
    open(R + path, 'w').write(s.replace(old, new, count))


H = 'trigenicinteractionpredictor_amd/csrc/mmsbm.hip'
sub(H, '''constexpr int XG = 16;  // observations per wave group''', '''constexpr int XG = 16;  // observations per wave group

// Row stride (doubles) of the fused path's contribution rows: one 128-B line per row for
// K <= 16, so every line is written whole by the wave that owns the observation.
template <int K>
constexpr int crow() {
  return K <= 16 ? 16 : K;
}''')
sub(H, '''  double* __restrict__ cb = contrib + (size_t)b * (nnz + 1) * K;

  // the first group's records''', '''  constexpr int CR = crow<K>();
  double* __restrict__ cb = contrib + (size_t)b * (nnz + 1) * CR;

  // the first group's records''')
sub(H, '''      double* ri = cb + (size_t)(real ? qD.x : nnz) * K;
      double* rj = cb + (size_t)(real ? qD.y : nnz) * K;
      double* rk = cb + (size_t)(real ? qD.z : nnz) * K;''', '''      double* ri = cb + (size_t)(real ? qD.x : nnz) * CR;
      double* rj = cb + (size_t)(real ? qD.y : nnz) * CR;
      double* rk = cb + (size_t)(real ? qD.z : nnz) * CR;''')
sub(H, '''        double* trash = cb + (size_t)nnz * K;''', '''        double* trash = cb + (size_t)nnz * CR;''')
sub(H, '''template <int K>
__global__ __launch_bounds__(256) void m2_kernel(''', '''template <int K, int CR>
__global__ __launch_bounds__(256) void m2_kernel(''')
sub(H, '''      const double* __restrict__ src = contrib + (size_t)b * (nnz + 1) * K + k;''',
    '''      const double* __restrict__ src = contrib + (size_t)b * (nnz + 1) * CR + k;''')
sub(H, '''        a0 += src[(size_t)q * K];
        a1 += src[(size_t)(q + NS) * K];
        a2 += src[(size_t)(q + 2 * NS) * K];
        a3 += src[(size_t)(q + 3 * NS) * K];
      }
      for (; q < q1; q += NS) a0 += src[(size_t)q * K];''', '''        a0 += src[(size_t)q * CR];
        a1 += src[(size_t)(q + NS) * CR];
        a2 += src[(size_t)(q + 2 * NS) * CR];
        a3 += src[(size_t)(q + 3 * NS) * CR];
      }
      for (; q < q1; q += NS) a0 += src[(size_t)q * CR];''')
sub(H, '''  m2_kernel<K><<<dim3(p_blocks + theta_blocks, c->B), 256, 0, s>>>(
      c->pr_mut, c->theta_mut, c->partS, c->contrib, c->gptr, c->deg, rg, c->P, c->R, G,
      c->nnz, p_blocks, c->eps, c->ablate);''', '''  if (fused)
    m2_kernel<K, crow<K>()><<<dim3(p_blocks + theta_blocks, c->B), 256, 0, s>>>(
        c->pr_mut, c->theta_mut, c->partS, c->contrib, c->gptr, c->deg, rg, c->P, c->R, G,
        c->nnz, p_blocks, c->eps, c->ablate);
  else
    m2_kernel<K, K><<<dim3(p_blocks + theta_blocks, c->B), 256, 0, s>>>(
        c->pr_mut, c->theta_mut, c->partS, c->contrib, c->gptr, c->deg, rg, c->P, c->R, G,
        c->nnz, p_blocks, c->eps, c->ablate);''')
sub(H, '''  off += align_up((size_t)c->B * (tr.n_obs_pad * 3 + 1) * c->K * sizeof(double));''',
    '''  const size_t crow_max = c->K <= 16 ? 16 : c->K;  // crow<K>() of the fused path
  off += align_up((size_t)c->B * (tr.n_obs_pad * 3 + 1) * crow_max * sizeof(double));''')
print('ok')
