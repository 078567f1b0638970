"""One-off source edit: mmsbm_fused ABI query, engine.fused, bench roofline for the fused path."""
R = '/root/repo/'


def sub(path, old, new):
    s = open(R + path).read()
    assert old in s, (path, old[:60])
    open(R + path, 'w').write(s.replace(old, new, 1))


sub('trigenicinteractionpredictor_amd/engine.py', '''    def timing(self, stride: int = 1):''', '''    @property
    def fused(self) -> bool:
        """True when iterate() runs the fused FP64-MFMA E-step (E-step + S in one kernel)."""
        v = ctypes.c_int32()
        _lib.check(self.lib.mmsbm_fused(self.ctx, ctypes.byref(v)))
        return bool(v.value)

    def timing(self, stride: int = 1):''')
sub('trigenicinteractionpredictor_amd/_lib.py', '''    "mmsbm_timing": (_c_int, [_vp, _c_i32]),''', '''    "mmsbm_fused": (_c_int, [_vp, ctypes.POINTER(_c_i32)]),
    "mmsbm_timing": (_c_int, [_vp, _c_i32]),''')
sub('include/mmsbm.h', '''/* Kernel timing for measurement (bench.py)''', '''/* *fused = 1 when mmsbm_iterate runs the fused FP64-MFMA E-step (E-step and S accumulation in
 * one kernel, then M2), 0 when it runs the VALU E-step + M1 + M2 (MMSBM_ESTEP, or K outside the
 * fused kernel's range). */
int mmsbm_fused(const mmsbm_ctx *ctx, int32_t *fused);

/* Kernel timing for measurement (bench.py)''')
sub('trigenicinteractionpredictor_amd/csrc/mmsbm.hip', '''int mmsbm_timing(mmsbm_ctx* c, int32_t stride) {''', '''int mmsbm_fused(const mmsbm_ctx* c, int32_t* fused) {
  if (!c || !fused) return fail(MMSBM_ERR_INVALID, "null argument");
  int rc = check_shape(c);
  if (rc) return rc;
  *fused = kTable[c->K - 1].fused && (c->estep_variant == 0 || c->estep_variant == 3) ? 1 : 0;
  return MMSBM_OK;
}

int mmsbm_timing(mmsbm_ctx* c, int32_t stride) {''')
sub('bench.py', '''        # roofline of the dominant kernel (E-step), per launch; SURVEY.md §8d figures
        est_avg_s = est_ms / 1e3 / est_n if est_n else float("nan")
        flops = 8.0 * K ** 3 * E_obs * B''', '''        # roofline of the dominant kernel (the E-step), per launch; SURVEY.md §8d figures.
        # Fused path (FP64 MFMA): the E-step launch does Y, Z, W and S = 8 K^3 per observation;
        # VALU path: the E-step does Y, Z, W = 6 K^3 (S is M1's 2 K^3).
        fused = eng.fused
        est_avg_s = est_ms / 1e3 / est_n if est_n else float("nan")
        flops = (8.0 if fused else 6.0) * K ** 3 * E_obs * B''')
sub('bench.py', '''            if rec.get("E_obs") == E_obs and rec.get("B") == B:''',
    '''            if rec.get("E_obs") == E_obs and rec.get("B") == B and rec.get("fused") == fused:''')
sub('bench.py', '''            "roofline": {"bound": "fp64-valu", "achieved": achieved_tf, "peak": FP64_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": achieved_tf / FP64_PEAK_TFLOPS, "traffic": traffic,
                         "kernel": "estep_kernel<%d>" % K, "avg_launch_us": est_avg_s * 1e6,''', '''            "roofline": {"bound": "mfma" if fused else "fp64-valu", "achieved": achieved_tf,
                         "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved_tf / FP64_PEAK_TFLOPS, "traffic": traffic,
                         "kernel": ("emx_kernel<%d> (E-step + S, FP64 MFMA)" if fused
                                    else "estep_kernel<%d> (VALU)") % K,
                         "avg_launch_us": est_avg_s * 1e6,''')
sub('bench.py', '''FP64_PEAK_TFLOPS = 78.6     # MI355X FP64 vector: 256 CU x 128 FLOP/clk x 2.4 GHz (spec)''',
    '''FP64_PEAK_TFLOPS = 78.6     # MI355X FP64 vector and matrix: 256 CU x 128 FLOP/clk x 2.4 GHz (spec)''')
print("ok")
