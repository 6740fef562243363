// fmath.h — TOOLS ONLY: exp in f64 written out, bit for bit the device library's.
//
// The ROCm 7.2 device library's exp(double) for gfx950, as hipcc emits it (the sequence read
// from the compiled kernels): t = rint(x log2 e); a two-constant Cody-Waite reduction
// r = x - t ln2; a degree-11 polynomial in Horner form, then two fma steps with 1; ldexp by
// t; +inf above x = 1024 and +0 below -1075 (NaN propagates). Written out with the same
// constants and the same fma order it gives the same bits for every input: tools/exp_check.hip
// found 0 mismatches in 2^28 inputs on the GPU (random doubles over the range checks, random
// bit patterns, both edges, rint's half-way points, the special values), and the batched
// reward's and the env step's fingerprints (tools/f2_bits.py, tools/step_bits.py) did not move
// (profiles/ab_r04/exp_r04o/). What it changes is the code: the library call re-materialised
// ten 64-bit constants into VGPR pairs per call (14 VALU moves); here they are scalar
// operands. Measured in the batched reward and the env step's softmax (round 4): 112 fewer
// VALU instructions per wave in batch_reward_rows_quad_kernel (1,117 -> 1,005) and
// batch_reward_grad_quad_kernel (653 -> 541), and no faster — the rows kernel 8.93 -> 8.96 us,
// config 5's 8-asset scalar step 38.5 -> 38.1 us — so the product keeps the library call.
#pragma once
#include <hip/hip_runtime.h>

namespace pmenv_dev {

// a 64-bit constant built in an SGPR pair by an opaque scalar move, and the Horner step
// fma(r, p, c) with c as the scalar operand of a VOP3 v_fma_f64: given a literal or an SGPR
// addend the compiler emits v_fmac_f64 and copies the addend into a VGPR pair first, two
// VALU moves per step. Neither asm has side effects (repeated constants are CSE'd across the
// unrolled calls of a kernel); fma rounds once, so the bits are those of __builtin_fma.
__device__ __forceinline__ double sconst(uint32_t hi, uint32_t lo) {
    uint32_t h, l;
    asm("s_mov_b32 %0, %1" : "=s"(h) : "i"(hi));
    asm("s_mov_b32 %0, %1" : "=s"(l) : "i"(lo));
    return __hiloint2double((int)h, (int)l);
}
__device__ __forceinline__ double fma_s(double a, double b, double c_sgpr) {
    double d;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(c_sgpr));
    return d;
}
__device__ __forceinline__ double exp_f64(double x) {
    const double t = __builtin_rint(x * sconst(0x3ff71547u, 0x652b82feu));                 // log2 e
    double r = __builtin_fma(sconst(0xbfe62e42u, 0xfefa39efu), t, x);                        // -ln2 hi
    r = __builtin_fma(sconst(0xbc7abc9eu, 0x3b39803fu), t, r);                               // -ln2 lo
    double p = __builtin_fma(sconst(0x3e5ade15u, 0x6a5dcb37u), r, sconst(0x3e928af3u, 0xfca7ab0cu));
    p = fma_s(r, p, sconst(0x3ec71deeu, 0x623fde64u));
    p = fma_s(r, p, sconst(0x3efa0199u, 0x7c89e6b0u));
    p = fma_s(r, p, sconst(0x3f2a01a0u, 0x14761f6eu));
    p = fma_s(r, p, sconst(0x3f56c16cu, 0x1852b7b0u));
    p = fma_s(r, p, sconst(0x3f811111u, 0x11122322u));
    p = fma_s(r, p, sconst(0x3fa55555u, 0x555502a1u));
    p = fma_s(r, p, sconst(0x3fc55555u, 0x55555511u));
    p = fma_s(r, p, sconst(0x3fe00000u, 0x0000000bu));
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
