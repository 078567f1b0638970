P = '/root/repo/trigenicinteractionpredictor_amd/csrc/mmsbm.hip'
s = open(P).read()
reps = [
('''template <int K, bool RP, int U0, int U1>
__device__ __forceinline__ void s_units(double (&sacc)[XPlan<K, RP>::NT4][XPlan<K, RP>::NG],
                                        double (&bS)[XPlan<K, RP>::NG], const double* TIp,''',
 '''template <int K, bool RP, int U0, int U1, int NT4_, int NG_>
__device__ __forceinline__ void s_units(double (&sacc)[NT4_][NG_], double (&bS)[NG_],
                                        const double* TIp,'''),
('''template <int K, bool RP, int A>
__device__ __forceinline__ void uws_step(
    const double* Pl, const double (&pU)[RP ? K : 1][XPlan<K, RP>::NG][XPlan<K, RP>::NG],
    const double (&aU)[XPlan<K, RP>::NG], const double (&tjD)[XPlan<K, RP>::NG],
    const double* TIc, const double* TJc, const double* TIp, const double* TJp,
    const double* TKp, double cprev, double (&yp)[K], double (&zp)[XPlan<K, RP>::NG],
    double (&wacc)[XPlan<K, RP>::NG], double (&sacc)[XPlan<K, RP>::NT4][XPlan<K, RP>::NG],
    double (&bS)[XPlan<K, RP>::NG], int hi, int lo, int oA, int oD) {''',
 '''template <int K, bool RP, int A, int KU_, int NT4_, int NG_>
__device__ __forceinline__ void uws_step(
    const double* Pl, const double (&pU)[KU_][NG_][NG_], const double (&aU)[NG_],
    const double (&tjD)[NG_], const double* TIc, const double* TJc, const double* TIp,
    const double* TJp, const double* TKp, double cprev, double (&yp)[K], double (&zp)[NG_],
    double (&wacc)[NG_], double (&sacc)[NT4_][NG_], double (&bS)[NG_], int hi, int lo, int oA,
    int oD) {'''),
('''template <int K, bool RP, int... As>
__device__ __forceinline__ void uws_all(
    std::integer_sequence<int, As...>, const double* Pl,
    const double (&pU)[RP ? K : 1][XPlan<K, RP>::NG][XPlan<K, RP>::NG],
    const double (&aU)[XPlan<K, RP>::NG], const double (&tjD)[XPlan<K, RP>::NG],
    const double* TIc, const double* TJc, const double* TIp, const double* TJp,
    const double* TKp, double cprev, double (&yp)[K], double (&zp)[XPlan<K, RP>::NG],
    double (&wacc)[XPlan<K, RP>::NG], double (&sacc)[XPlan<K, RP>::NT4][XPlan<K, RP>::NG],
    double (&bS)[XPlan<K, RP>::NG], int hi, int lo, int oA, int oD) {''',
 '''template <int K, bool RP, int KU_, int NT4_, int NG_, int... As>
__device__ __forceinline__ void uws_all(
    std::integer_sequence<int, As...>, const double* Pl, const double (&pU)[KU_][NG_][NG_],
    const double (&aU)[NG_], const double (&tjD)[NG_], const double* TIc, const double* TJc,
    const double* TIp, const double* TJp, const double* TKp, double cprev, double (&yp)[K],
    double (&zp)[NG_], double (&wacc)[NG_], double (&sacc)[NT4_][NG_], double (&bS)[NG_],
    int hi, int lo, int oA, int oD) {'''),
]
for old, new in reps:
    assert old in s, old[:80]
    s = s.replace(old, new)
open(P, 'w').write(s)
print('ok')
