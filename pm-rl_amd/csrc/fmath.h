// fmath.h — exp in f64 written out, bit for bit the device library's.
//
// The ROCm 7.2 device library's exp(double) for gfx950, as hipcc emits it (the sequence read
// from the compiled kernels): t = rint(x log2 e); a two-constant Cody-Waite reduction
// r = x - t ln2; a degree-11 polynomial in Horner form, then two fma steps with 1; ldexp by
// t; +inf above x = 1024 and +0 below -1075 (NaN propagates). Written out with the same
// constants and the same fma order it gives the same bits for every input
// (tools/exp_check.hip checks 2^28 inputs on the GPU, the edges of both range checks, rint's
// half-way points and every special value). What it changes is the code: called from an
// unrolled loop it runs without a branch per element and its constants are materialised
// once, where the library call re-materialised ten 64-bit constants into VGPR pairs per
// call (SQ_INSTS_VALU: profiles/ab_r04/f2_pmc_r04n.txt).
#pragma once
#include <hip/hip_runtime.h>

namespace pmenv_dev {

__device__ __forceinline__ double exp_f64(double x) {
    const double t = __builtin_rint(x * 0x1.71547652b82fep+0);
    double r = __builtin_fma(-0x1.62e42fefa39efp-1, t, x);
    r = __builtin_fma(-0x1.abc9e3b39803fp-56, t, r);
    double p = __builtin_fma(0x1.ade156a5dcb37p-26, r, 0x1.28af3fca7ab0cp-22);
    p = __builtin_fma(r, p, 0x1.71dee623fde64p-19);
    p = __builtin_fma(r, p, 0x1.a01997c89e6b0p-16);
    p = __builtin_fma(r, p, 0x1.a01a014761f6ep-13);
    p = __builtin_fma(r, p, 0x1.6c16c1852b7b0p-10);
    p = __builtin_fma(r, p, 0x1.1111111122322p-7);
    p = __builtin_fma(r, p, 0x1.55555555502a1p-5);
    p = __builtin_fma(r, p, 0x1.5555555555511p-3);
    p = __builtin_fma(r, p, 0x1.000000000000bp-1);
    p = __builtin_fma(r, p, 1.0);
    p = __builtin_fma(r, p, 1.0);
    // t is integral; clamped so the conversion is defined for every input (|t| > 2000 and
    // NaN only reach the selects below, which replace the result)
    const int n = (int)__builtin_fmin(__builtin_fmax(t, -2000.0), 2000.0);
    double y = __builtin_ldexp(p, n);
    y = x > 1024.0 ? __builtin_inf() : y;
    y = x < -1075.0 ? 0.0 : y;
    return y;
}

}  // namespace pmenv_dev
