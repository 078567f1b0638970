"""On the committed fused kernel: the mmsbm_fused query and the single-round-trip M2."""
P = '/root/repo/trigenicinteractionpredictor_amd/csrc/mmsbm.hip'
s = open(P).read()
old = '''int mmsbm_timing(mmsbm_ctx* c, int32_t stride) {'''
assert old in s
s = s.replace(old, '''int mmsbm_fused(const mmsbm_ctx* c, int32_t* fused) {
  if (!c || !fused) return fail(MMSBM_ERR_INVALID, "null argument");
  int rc = check_shape(c);
  if (rc) return rc;
  *fused = kTable[c->K - 1].fused && c->estep_variant == 0 ? 1 : 0;
  return MMSBM_OK;
}

int mmsbm_timing(mmsbm_ctx* c, int32_t stride) {''')
new_m2 = open('/root/repo/tools/patches/p02_kernels.hip').read()
m2 = new_m2[new_m2.index('// M2, grid (p_blocks + P, B), block 256.'):]
m2 = m2[:m2.rindex('}') + 1] + '\n\n'
a = s.index('// M2, grid (p_blocks + theta_blocks, B), block 256.')
b = s.index('// Log-likelihood partials (:958-969)')
b = s.rfind('// ----', 0, b)
s = s[:a] + m2 + s[b:]
old = '''  const int theta_blocks = (c->P + 3) / 4;'''
assert old in s
s = s.replace(old, '''  const int theta_blocks = c->P;  // one workgroup per gene''')
open(P, 'w').write(s)
print('ok')
