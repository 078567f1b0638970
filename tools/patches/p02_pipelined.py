"""Replace the fused kernel (and its header comment) with the software-pipelined version and
M2 with the single-round-trip reductions."""
P = '/root/repo/trigenicinteractionpredictor_amd/csrc/mmsbm.hip'
s = open(P).read()
a = s.index('// Fused E-step + S accumulation on FP64 MFMA (:987-1012), grid (G, B), block 64 * NW.')
a = s.rfind('// ----', 0, a)
b = s.index('// Log-likelihood partials (:958-969)')
b = s.rfind('// ----', 0, b)
NEW = open('/root/repo/tools/patches/p02_kernels.hip').read()
s = s[:a] + NEW + s[b:]
old = '''        c->partS, c->partL, rg, c->P, c->R, c->nnz, G, c->eps, XTrace{c->trace});'''
assert old in s
s = s.replace(old, '''        c->partS, rg, c->P, c->R, c->nnz, G, c->eps, XTrace{c->trace});''')
old = '''            "[mmsbm trace] waves=%lld avg cycles: prologue %.0f  U %.0f  KR %.0f  W %.0f  "
            "stores %.0f  S %.0f  epilogue %.0f  groups %.2f  total %.0f (max %llu)\\n",'''
assert old in s, 'trace'
s = s.replace(old, '''            "[mmsbm trace] waves=%lld avg cycles: prologue %.0f  U+W+S' %.0f  images %.0f  "
            "reduce/c %.0f  stores %.0f  tail %.0f  epilogue %.0f  groups %.2f  total %.0f "
            "(max %llu)\\n",''')
open(P, 'w').write(s)
print('ok')
