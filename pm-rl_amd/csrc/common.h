// common.h — shared device helpers and the kernel parameter block.
#pragma once
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>

#include "../../include/pmenv.h"

namespace pmenv_dev {

constexpr int kWideMaxAssets = 512;   // the widest env the packed scalar step and the wide flat step take
// polls of a missing relay word before a tile defers (step_relay.h): each is an s_sleep plus an
// agent-scope load round trip (~1 us under the stream), so ~1 ms — two orders of magnitude above
// the scalar blocks' whole run, reached only when they were not dispatched ahead of the tile
constexpr uint32_t kRelaySpin = 1024;

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));   // dword-aligned 16-B access

// ---------------------------------------------------------------- fast division
// q = floor(n / d) for 0 <= n < 2^31 by multiply-high (Granlund & Montgomery).
struct FastDiv {
    uint32_t mul, shift, d;
};

inline FastDiv make_fastdiv(uint32_t d) {
    FastDiv f;
    f.d = d;
    uint32_t s = 0;
    while ((1ull << s) < d) ++s;
    f.shift = s;
    f.mul = (uint32_t)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
    return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
    uint32_t hi = __umulhi(n, f.mul);
    return (uint32_t)(((uint64_t)hi + n) >> f.shift);
}

// ---------------------------------------------------------------- parameter block
struct StepParams {
    int B, N, W, F, close_ch;
    int reward_kind, norm_mode, ring_mode, ret_mode, mu_max_iter;
    int rows_per_tile;     // LDS kernel: asset rows per staged tile
    int tile_floats;       // LDS kernel: floats reserved for the tile region (multiple of 4)
    int unit_rows;         // streaming kernel: asset rows per workgroup
    int units_per_env;
    double init_cash, commission, scale, rf, eta, mu_tol;
    const float* action;
    const float* prices;
    const float* bar;      // [B, N, F-1], or the series base when `day` is set
    const int32_t* day;    // resident-series mode: env b's bar is series[day[b]] ([T, N, F-1] shared)
    int32_t series_days;   // T of the resident series (days outside [0, T) read NaN)
    float* obs;
    float* obs_out;        // advance mode: destination window (== obs when in place)
    float* reward;
    double* ret;
    float* weights;
    // env state (handle-owned)
    double* value;
    int32_t* k;
    float* ring;
    float* last_close;
    float* w_new;          // [B, N] post-drift weights of the latest step (dense copy of the ring slot)
    double* sa;
    double* sb;
    unsigned long long* nonfinite;
    // in-place flat advance: the scalar step kernel copies every flat workgroup's
    // first two chunks here (advance_flat_inplace_kernel's halo); null: no copy
    float* halo;
    uint32_t halo_wgs, halo_block, halo_qtot;
    uint32_t halo_hs;      // log2 of the two-chunk items per workgroup boundary: 0 (two chunks,
                           // every F <= 8 stream), 1 (four: the generic stream past F = 8)
    // one-launch flat step (step_flat.h): the state snapshot the scalar step reads
    // (parity p: value, counter, get_last(), last close) and the one the env's owner
    // writes for the next step (parity 1 - p); in place, the halo of this step and the
    // one this step leaves for the next
    const double* sv_in;
    const int32_t* sk_in;
    const float* sw_in;
    const float* slc_in;
    double* sv_out;
    int32_t* sk_out;
    float* sw_out;
    float* slc_out;
    const float* halo_in;
    float* halo_out;
    uint32_t per4;         // 16-B chunks per env window
    // device-sequenced flat step (hipGraph-safe; step_flat.h): null = the host chose the
    // parity. Else seq = {D, C, V, pad, HOBS lo, HOBS hi}: D the parity the next step
    // reads, C the parity of the step in flight, V = 1 when snapshot D mirrors the state,
    // HOBS the window whose halo halo[D] holds; *_in / halo_in are parity 0, *_out /
    // halo_out parity 1, swapped by the kernel when C == 1
    int32_t* seq;
    FastDiv div_wf, div_f, div_w, div_units;
};

// the host-I/O step's staging outputs (env_step.h surface_body<true>, pmenv_step_host)
struct HostIO {
    const float* close_in;   // [B, N] obs[b, n, W-1, close] gathered by the host
    float* chan;             // [B, N, W] channel F-1 out
    double* value_out;       // [B] the value after the step (TradingEnv.value)
    uint32_t* done;          // [B] completion words: env b's outputs are all in host memory once
    uint32_t seq;            //     done[b] == seq (written last, system scope)
};


// The day's bar [N, F-1] of env b: a row of the per-env bar batch, or — resident
// series mode — day[b] of a market series shared by all envs. Returns null for an
// out-of-range day (the caller then reads NaN: the env's reward turns non-finite
// and is counted, no memory outside the series is touched).
__device__ __forceinline__ const float* env_bar(const StepParams& p, int b) {
    const size_t row = (size_t)p.N * (p.F - 1);
    if (!p.day) return p.bar + (size_t)b * row;
    const int32_t d = p.day[b];
    return (d >= 0 && d < p.series_days) ? p.bar + (size_t)d * row : nullptr;
}

// the ring slot (1 + k) % W of weight_buffer.py:32-44 for the step counter k >= 0 (it starts
// at 0 on reset and only counts up): 32-bit unsigned arithmetic, the 64-bit remainder's
// ~100 instructions were on the register step's critical path
__device__ __forceinline__ int ring_slot(int32_t k, int W) { return (int)(((uint32_t)k + 1u) % (uint32_t)W); }

// branch-free float select (bit masks: keeps element loops free of control flow)
__device__ __forceinline__ float pick(bool c, float a, float b) {
    const int m = -(int)c;
    return __int_as_float((__float_as_int(a) & m) | (__float_as_int(b) & ~m));
}

// ---------------------------------------------------------------- buffer access
// Range-checked buffer loads/stores (CDNA SRSRC descriptors): a lane whose byte
// offset falls outside [0, bytes) reads 0 / stores nothing, so prologues need no
// per-lane branches (and no control-flow joins that force early vmcnt waits).
// Build descriptors from wave-uniform values only (kernel args, blockIdx).
typedef unsigned int u4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
// AUX = the instruction's cache-policy bits (gfx950: 1 = sc0, 2 = nt, 16 = sc1)
template <int AUX = 0>
__device__ __forceinline__ f4 buf_load4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    const u4v v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX);
    return f4{__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w)};
}
__device__ __forceinline__ float buf_load1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ double buf_load_f64(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    typedef unsigned int u2v __attribute__((ext_vector_type(2)));
    const u2v v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
    return __hiloint2double((int)v.y, (int)v.x);
}
template <int AUX = 0>
__device__ __forceinline__ void buf_store4(__amdgpu_buffer_rsrc_t r, uint32_t off, f4 v) {
    const u4v u = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
    __builtin_amdgcn_raw_buffer_store_b128(u, r, off, 0, AUX);
}

// ---------------------------------------------------------------- wave reductions
// f64 reductions over one wave with DPP row shifts (no LDS crossbar): four
// row_shr steps leave each 16-lane row's total in its lane 15, and the four row
// totals are combined in a fixed order from v_readlane — so every lane gets
// bitwise the same value and every branch taken on it is wave-uniform.
template <int CTRL>
__device__ __forceinline__ double dpp_shift(double v, double fill) {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    const int flo = __double2loint(fill), fhi = __double2hiint(fill);
    const int rlo = __builtin_amdgcn_update_dpp(flo, lo, CTRL, 0xF, 0xF, false);
    const int rhi = __builtin_amdgcn_update_dpp(fhi, hi, CTRL, 0xF, 0xF, false);
    return __hiloint2double(rhi, rlo);
}

__device__ __forceinline__ double lane_value(double v, int lane) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}

constexpr int kRowShr1 = 0x111, kRowShr2 = 0x112, kRowShr4 = 0x114, kRowShr8 = 0x118;

__device__ __forceinline__ double wave_sum(double v) {
    v += dpp_shift<kRowShr1>(v, 0.0);
    v += dpp_shift<kRowShr2>(v, 0.0);
    v += dpp_shift<kRowShr4>(v, 0.0);
    v += dpp_shift<kRowShr8>(v, 0.0);
    return (lane_value(v, 15) + lane_value(v, 31)) + (lane_value(v, 47) + lane_value(v, 63));
}
__device__ __forceinline__ double wave_max(double v) {
    v = fmax(v, dpp_shift<kRowShr1>(v, -INFINITY));
    v = fmax(v, dpp_shift<kRowShr2>(v, -INFINITY));
    v = fmax(v, dpp_shift<kRowShr4>(v, -INFINITY));
    v = fmax(v, dpp_shift<kRowShr8>(v, -INFINITY));
    return fmax(fmax(lane_value(v, 15), lane_value(v, 31)), fmax(lane_value(v, 47), lane_value(v, 63)));
}
__device__ __forceinline__ double wave_min(double v) {
    v = fmin(v, dpp_shift<kRowShr1>(v, INFINITY));
    v = fmin(v, dpp_shift<kRowShr2>(v, INFINITY));
    v = fmin(v, dpp_shift<kRowShr4>(v, INFINITY));
    v = fmin(v, dpp_shift<kRowShr8>(v, INFINITY));
    return fmin(fmin(lane_value(v, 15), lane_value(v, 31)), fmin(lane_value(v, 47), lane_value(v, 63)));
}

// quad (4-lane group) reductions by DPP quad_perm: xor 1 then xor 2. Every lane of
// the quad ends with bitwise the same value ((a0+a1)+(a2+a3) in each, by commutativity).
constexpr int kQuadXor1 = 0xB1, kQuadXor2 = 0x4E;
__device__ __forceinline__ double quad_sum(double v) {
    v += dpp_shift<kQuadXor1>(v, 0.0);
    return v + dpp_shift<kQuadXor2>(v, 0.0);
}
__device__ __forceinline__ double quad_max(double v) {
    v = fmax(v, dpp_shift<kQuadXor1>(v, -INFINITY));
    return fmax(v, dpp_shift<kQuadXor2>(v, -INFINITY));
}
__device__ __forceinline__ double quad_min(double v) {
    v = fmin(v, dpp_shift<kQuadXor1>(v, INFINITY));
    return fmin(v, dpp_shift<kQuadXor2>(v, INFINITY));
}

}  // namespace pmenv_dev
