"""Slot-0 run pre-reduction: observations are sorted by slot-0 gene within each rating, so a
16-observation group holds few runs of equal slot-0 genes; the fused kernel sums each run's
c*Y rows in LDS and stores one row per run; the gene CSR lists only the run heads for slot 0."""
R = '/root/repo/'


def sub(path, old, new, count=1):
    s = open(R + path).read()
    assert s.count(old) >= count, (path, old[:70])
    open(R + path, 'w').write(s.replace(old, new, count))


L = 'trigenicinteractionpredictor_amd/layout.py'
sub(L, '''TILE = 256''', '''TILE = 256
GROUP = 16   # observations per wave group of the fused kernel (XG in csrc/mmsbm.hip)''')
sub(L, '''def build_gene_csr(layout: ObsLayout, ids: np.ndarray, P: int) -> GeneCSR:
    real = np.nonzero(layout.link_of_row >= 0)[0]
    genes = layout.obs[real, :3].astype(np.int64)          # [n_obs][3]
    entry = (real[:, None] * 3 + np.arange(3)[None, :])     # row*3 + slot
    g_flat = genes.ravel()
    e_flat = entry.ravel()''', '''def build_gene_csr(layout: ObsLayout, ids: np.ndarray, P: int, run_group: int = 0) -> GeneCSR:
    """run_group > 0 (fused kernel): within each group of run_group rows, consecutive real rows
    with the same slot-0 gene form a run whose slot-0 rows the kernel sums into the run head's
    row; only the heads' slot-0 entries are listed (deg is unchanged: the reference's counter)."""
    real = np.nonzero(layout.link_of_row >= 0)[0]
    genes = layout.obs[real, :3].astype(np.int64)          # [n_obs][3]
    entry = (real[:, None] * 3 + np.arange(3)[None, :])     # row*3 + slot
    keep = np.ones(genes.shape, dtype=bool)
    if run_group and real.size:
        is_real = layout.link_of_row >= 0
        g0 = layout.obs[:, 0]
        prev = real - 1
        nonhead = (real % run_group != 0) & is_real[np.maximum(prev, 0)] & \\
            (g0[np.maximum(prev, 0)] == g0[real])
        keep[:, 0] = ~nonhead
    g_flat = genes[keep]
    e_flat = entry[keep]''')
E = 'trigenicinteractionpredictor_amd/engine.py'
sub(E, '''from .layout import TILE, build_gene_csr, build_obs''', '''from .layout import GROUP, TILE, build_gene_csr, build_obs''')
sub(E, '''            csr = build_gene_csr(lay, ids, self.P)''', '''            csr = build_gene_csr(lay, ids, self.P, run_group=GROUP if self.fused else 0)''')
H = 'trigenicinteractionpredictor_amd/csrc/mmsbm.hip'
sub(H, '''    // ---- contributions of observation oD: entries 4 j + lo of its three gene-CSR rows
    if (!(EMX_AB & 8)) {''', '''    // ---- slot-0 runs: the observations are sorted by slot-0 gene, so equal genes are adjacent;
    //      c Y rows and genes staged in LDS (TI / TJ are free after the KR phase), each run's
    //      head sums its run in order (the CSR lists only run heads for slot 0; the other
    //      rows' pos is -1 and they store to the trash row)
    double ysum[NG];
    {
      int* G0 = reinterpret_cast<int*>(TJ);
#pragma unroll
      for (int j = 0; j < NG; ++j) {
        const int v = 4 * j + lo;
        double y = yp[4 * j];
#pragma unroll
        for (int t = 1; t < 4; ++t)
          if (4 * j + t < K && lo == t) y = yp[4 * j + t];
        if (v < K) TI[oD * KP + v] = c * y;
        ysum[j] = 0.0;
      }
      if (lo == 0) G0[oD] = qD.x >= 0 ? eD.x : -1 - oD;  // padding never joins a run
      wave_lds_sync();
      const int gme = G0[oD];
      if (qD.x >= 0) {
        for (int o2 = oD; o2 < XG && G0[o2] == gme; ++o2) {
#pragma unroll
          for (int j = 0; j < NG; ++j)
            if (4 * j + lo < K) ysum[j] += TI[o2 * KP + 4 * j + lo];
        }
      }
    }

    // ---- contributions of observation oD: entries 4 j + lo of its three gene-CSR rows
    if (!(EMX_AB & 8)) {''')
sub(H, '''        double* trash = cb + (size_t)nnz * K;
        (v < K ? ri : trash)[vs] = c * y;''', '''        double* trash = cb + (size_t)nnz * K;
        (void)y;
        (v < K ? ri : trash)[vs] = ysum[j];''')
print('ok')
