"""Fused path: contribution rows in observation-major order (row = obs_row * 3 + slot, the gene
incidence CSR's own entry values), so each wave writes its group's 48 rows as one contiguous
block; M2 gathers each gene's rows through the CSR (gene_inc) instead of reading a run."""
R = '/root/repo/'


def sub(path, old, new, count=1):
    s = open(R + path).read()
    assert s.count(old) >= 1, (path, old[:70])
    open(R + path, 'w').write(s.replace(old, new, count))


H = 'trigenicinteractionpredictor_amd/csrc/mmsbm.hip'
# --- emx: no pos records; stores to obs-major rows; trash row = crow (= 3 n_obs_pad)
sub(H, '''  int4 eA = make_int4(0, 0, 0, 0), eD = eA, qD = eA, nA = eA, nD = eA, nQ = eA;''',
    '''  int4 eA = make_int4(0, 0, 0, 0), eD = eA, nA = eA, nD = eA;''')
sub(H, '''    eD = obs[r0 + oD];
    qD = pos[r0 + oD];
    load_theta(eA, eD, aU, tjD, tiD4);''', '''    eD = obs[r0 + oD];
    load_theta(eA, eD, aU, tjD, tiD4);''')
sub(H, '''      nD = obs[r1 + oD];
      nQ = pos[r1 + oD];''', '''      nD = obs[r1 + oD];''')
sub(H, '''      const bool real = qD.x >= 0;  // padding observations write the trash row (nnz)
      double* ri = cb + (size_t)(real ? qD.x : nnz) * K;
      double* rj = cb + (size_t)(real ? qD.y : nnz) * K;
      double* rk = cb + (size_t)(real ? qD.z : nnz) * K;''', '''      // rows (obs, slot) of the group: one contiguous 3 x 16 x K block per wave
      double* ri = cb + ((size_t)grp * XG + oD) * 3 * K;
      double* rj = ri + K;
      double* rk = rj + K;''')
sub(H, '''        double* trash = cb + (size_t)nnz * K;''', '''        double* trash = cb + (size_t)nnz * K;  // row 3 n_obs_pad: never read''')
sub(H, '''    qD = nQ;
''', '')
# --- M2: GATHER variant
sub(H, '''template <int K>
__global__ __launch_bounds__(256) void m2_kernel(double* __restrict__ pr, double* __restrict__ theta,
                                                 const double* __restrict__ partS,
                                                 const double* __restrict__ contrib,
                                                 const int* __restrict__ gptr,''', '''template <int K, bool GATHER>
__global__ __launch_bounds__(256) void m2_kernel(double* __restrict__ pr, double* __restrict__ theta,
                                                 const double* __restrict__ partS,
                                                 const double* __restrict__ contrib,
                                                 const int* __restrict__ ginc,
                                                 const int* __restrict__ gptr,''')
sub(H, '''    if (slot < NS) {
      const double* __restrict__ src = contrib + (size_t)b * (nnz + 1) * K + k;
      int q = q0 + slot;
      for (; q + 3 * NS < q1; q += 4 * NS) {
        a0 += src[(size_t)q * K];
        a1 += src[(size_t)(q + NS) * K];
        a2 += src[(size_t)(q + 2 * NS) * K];
        a3 += src[(size_t)(q + 3 * NS) * K];
      }
      for (; q < q1; q += NS) a0 += src[(size_t)q * K];
    }''', '''    if (slot < NS) {
      const double* __restrict__ src = contrib + (size_t)b * (nnz + 1) * K + k;
      // GATHER (fused path): the gene's rows sit at its incidence entries obs_row * 3 + slot;
      // otherwise they are the contiguous run [q0, q1)
      auto row = [&](int q) -> size_t { return GATHER ? (size_t)ginc[q] : (size_t)q; };
      int q = q0 + slot;
      for (; q + 3 * NS < q1; q += 4 * NS) {
        const size_t r0 = row(q), r1 = row(q + NS), r2 = row(q + 2 * NS), r3 = row(q + 3 * NS);
        a0 += src[r0 * K];
        a1 += src[r1 * K];
        a2 += src[r2 * K];
        a3 += src[r3 * K];
      }
      for (; q < q1; q += NS) a0 += src[row(q) * K];
    }''')
sub(H, '''//  blocks [p_blocks, ...): theta (:1016-1018), in place, one workgroup per gene:
//      theta[g][a] <- theta[g][a] * (sum of the gene's contiguous c-scaled rows)[a] / deg[g]''',
    '''//  blocks [p_blocks, ...): theta (:1016-1018), in place, one workgroup per gene:
//      theta[g][a] <- theta[g][a] * (sum of the gene's c-scaled rows)[a] / deg[g]
//    rows: the gene's contiguous CSR run (VALU path) or, GATHER (fused path), the
//    observation-major rows its incidence entries name;''')
# --- host launches
sub(H, '''        tr.obs, reinterpret_cast<const int4*>(c->pos), c->theta_mut, c->pr_mut, c->contrib,
        c->partS, c->partL, rg, c->P, c->R, c->nnz, G, c->eps, XTrace{c->trace});''',
    '''        tr.obs, reinterpret_cast<const int4*>(c->pos), c->theta_mut, c->pr_mut, c->contrib,
        c->partS, c->partL, rg, c->P, c->R, 3 * tr.n_obs_pad, G, c->eps, XTrace{c->trace});''')
sub(H, '''  m2_kernel<K><<<dim3(p_blocks + theta_blocks, c->B), 256, 0, s>>>(
      c->pr_mut, c->theta_mut, c->partS, c->contrib, c->gptr, c->deg, rg, c->P, c->R, G,
      c->nnz, p_blocks, c->eps, c->ablate);''', '''  if (fused)  // observation-major rows (3 n_obs_pad + trash per sample), gathered through gene_inc
    m2_kernel<K, true><<<dim3(p_blocks + theta_blocks, c->B), 256, 0, s>>>(
        c->pr_mut, c->theta_mut, c->partS, c->contrib, c->ginc, c->gptr, c->deg, rg, c->P, c->R,
        G, 3 * tr.n_obs_pad, p_blocks, c->eps, c->ablate);
  else
    m2_kernel<K, false><<<dim3(p_blocks + theta_blocks, c->B), 256, 0, s>>>(
        c->pr_mut, c->theta_mut, c->partS, c->contrib, c->ginc, c->gptr, c->deg, rg, c->P, c->R,
        G, c->nnz, p_blocks, c->eps, c->ablate);''')
print('ok')
