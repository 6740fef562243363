// step_split.h — the whole env step in ONE launch with the scalar step decoupled from the
// window stream (in place).
//
// TradingEnv.step (zachramsey/pm-rl env/sim/trading_env.py:44-105) and the one-day window
// advance (data/instrument.py:339-356) for every env of the batch. step_flat_kernel runs
// an env's scalar step in every tile the env straddles, and a tile's stores wait (one
// barrier) for that step's w'. Where the window sits in the Infinity Cache its loads land
// before the f64 reduction chain ends, so the chain sets the tile's time.
// Here a launch holds two kinds of workgroup, neither of which waits for the other:
//   * stream tiles (BLOCK x V chunks: the in-place flat stream's geometry and side data)
//     compose every output chunk except the w' dword of each asset row — the row's last-day
//     weight, or (storage order, ring full) its ring slot — which they leave unwritten: a
//     chunk holding it is stored as its three other dwords;
//   * scalar workgroups, one wave per env, one every R workgroups of the grid, run the env's
//     whole scalar step on the canonical state (the two-launch path's order of operations:
//     the same bits) and store w' into the window's slot themselves.
// The tiles read two things the scalar workgroups overwrite during the launch, so they
// take them from the per-step snapshot (parity p in, 1 - p written by the scalar
// workgroup): the env's counter (sk), and — in shift mode, where day W-2's weight is the
// old last-day weight that the new w' replaces — that old weight (sw: a copy of the window's
// last-day weight dwords, which the prime takes from the window itself). The halo of the
// in-place tiles is step_flat_kernel's (parity p in, 1 - p out; its w' dwords are never
// read: the snapshot replaces them), as are the device sequencing and the priming.
#pragma once
#include "step_flat.h"

namespace pmenv_dev {

__device__ __forceinline__ void buf_store1(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, 0);
}

// flat_compose with the w' dword left out (`hole` = its element, -1 if the chunk has
// none) and, in shift mode, day W-2's weight from the snapshot (sd.xwp = the row's old
// last-day weight) instead of the window, whose copy the scalar workgroup overwrites
__device__ __forceinline__ f4 split_compose(const StepParams& p, const FlatSide& sd, const float (&un)[4],
                                            const float (&sh)[4], int& hole) {
    constexpr int F = 5;
    const int W = p.W, WF = W * F;
    const bool shift_w = !(p.ring_mode == PMENV_RING_STORAGE && sd.k >= W - 1);
    const int slot_w = (int)(((uint32_t)(1 + sd.k) - fdiv((uint32_t)(1 + sd.k), p.div_w) * (uint32_t)W) * F + (F - 1));
    int f = sd.kk - (int)fdiv((uint32_t)sd.kk, p.div_f) * F;
    float v[4];
    hole = -1;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int pos = sd.kk + e;
        const bool in_row = pos < WF;
        const bool lastday = in_row && pos >= WF - F;
        const bool is_w = in_row && f == F - 1;
        const float bsel = pick(sd.bar_nan, __int_as_float(0x7fc00000),
                                pick(f == 0, sd.xb.x, pick(f == 1, sd.xb.y, pick(f == 2, sd.xb.z, sd.xb.w))));
        const bool w_here = shift_w ? lastday : pos == slot_w;
        const bool from_snap = shift_w && pos == WF - F - 1;
        const float wv = pick(from_snap, sd.xwp, pick(shift_w, sh[e], un[e]));
        v[e] = pick(is_w, wv, pick(lastday, bsel, sh[e]));
        if (is_w && w_here) hole = e;
        f = f == F - 1 ? 0 : f + 1;
    }
    return f4{v[0], v[1], v[2], v[3]};
}

// a stream tile: chunks [CPW tile, CPW tile + CPW) of the flat window, in place
// (ABL, timing-only variants of the tools build, 0 in the product: 1 = whole 16-B stores)
template <int BLOCK, int V, int POL, int ABL = 0>
__device__ __forceinline__ void split_tile(const StepParams& p, uint32_t qtot, uint32_t tile, uint32_t ntiles,
                                           f4* sh4) {
    constexpr int kAux = POL == 1 ? 2 : 0;
    constexpr int CPW = BLOCK * V;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t c0 = tile * (uint32_t)CPW;
    const uint32_t nblk = min((uint32_t)CPW, qtot - c0);
    const auto rs = make_rsrc(p.obs + (size_t)c0 * 4, nblk * 16u);
    f4 own[V];
#pragma unroll
    for (int v = 0; v < V; ++v) own[v] = buf_load4<kAux>(rs, (uint32_t)(64 * V * wave + 64 * v + lane) * 16u);
    const uint32_t nh = tile + 1 < ntiles ? min(2u, qtot - c0 - nblk) : 0u;
    const f4 hal = buf_load4<0>(make_rsrc(p.halo_in + (size_t)tile * 8, nh * 16u),
                                tid < 2 ? (uint32_t)tid * 16u : 0xFFFFFFF0u);
    __builtin_amdgcn_sched_barrier(0);
    // side data: the bar rows as the two-launch stream, the counter and the old last-day
    // weights from the snapshot
    StepParams ps = p;
    ps.k = const_cast<int32_t*>(p.sk_in);
    ps.w_new = const_cast<float*>(p.sw_in);
    const uint32_t qw = __builtin_amdgcn_readfirstlane(c0 + (uint32_t)(64 * V * wave));
    const WaveSide ws = wave_side_load(ps, qw, 64u * V, qtot);
    FlatSide sd[V];
#pragma unroll
    for (int v = 0; v < V; ++v) sd[v] = flat_side_from_wave<0, 0>(ps, ws, min(qw + 64u * v + lane, qtot - 1u));
#pragma unroll
    for (int v = 0; v < V; ++v) sh4[64 * V * wave + 64 * v + lane] = own[v];
    if (tid < 2) sh4[CPW + tid] = hal;
    __syncthreads();
    const bool first_out = tile > 0;                                    // feeds the previous tile's halo
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int j = 64 * V * wave + 64 * v + lane;
        const f4 n1 = sh4[j + 1], n2 = sh4[j + 2];
        const float sh[4] = {n1.y, n1.z, n1.w, n2.x};
        const float un[4] = {own[v].x, own[v].y, own[v].z, own[v].w};
        int hole;
        const f4 o = split_compose(p, sd[v], un, sh, hole);
        const uint32_t off = (uint32_t)j * 16u;
        if (ABL & 1) hole = -1;
        buf_store4<kAux>(rs, hole < 0 ? off : 0xFFFFFFF0u, o);           // past the end: dropped
        if (hole >= 0) {                                                 // the three other dwords
            buf_store1(rs, hole == 0 ? 0xFFFFFFF0u : off, o.x);
            buf_store1(rs, hole == 1 ? 0xFFFFFFF0u : off + 4u, o.y);
            buf_store1(rs, hole == 2 ? 0xFFFFFFF0u : off + 8u, o.z);
            buf_store1(rs, hole == 3 ? 0xFFFFFFF0u : off + 12u, o.w);
        }
        if (first_out && j < 2) reinterpret_cast<f4*>(p.halo_out)[2 * (tile - 1) + j] = o;
    }
}

// a scalar workgroup: envs WAVES s .. WAVES s + WAVES - 1, one per wave (ABL: 2 = no w'
// store into the window, 4 = no scalar step at all)
template <int BLOCK, int ABL = 0>
__device__ __forceinline__ void split_scalar(const StepParams& p, uint32_t s) {
    if (ABL & 4) return;
    constexpr int WAVES = BLOCK / 64, F = 5;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int b = (int)s * WAVES + wave;
    if (b >= p.B) return;
    const ScalarIn in = scalar_load_row(p, b, lane);
    const ScalarMid m = scalar_core<64, true>(p, b, lane, in);
    const int N = p.N, W = p.W;
    if (lane < N && !(ABL & 2)) {
        // w' into the window's slot: the last day, or (storage order, ring full) the ring slot
        const bool shift_w = !(p.ring_mode == PMENV_RING_STORAGE && m.k >= W - 1);
        const int day = shift_w ? W - 1 : (int)((1 + (int64_t)m.k) % W);
        p.obs[((size_t)b * N + lane) * (size_t)(W * F) + (size_t)day * F + (F - 1)] = m.wp;
        p.sw_out[(size_t)b * N + lane] = m.wp;
    }
    if (lane == 0) p.sk_out[b] = m.k + 1;
    scalar_tail<64, false>(p, b, lane, in, m);
}

// grid: nscalar groups of R workgroups (one scalar workgroup, then R - 1 tiles), then the
// remaining tiles; every workgroup has an exit (tiles past ntiles return at once)
template <int BLOCK, int V, int POL, int ABL = 0>
__global__ __launch_bounds__(BLOCK) void step_split_kernel(StepParams p, uint32_t qtot, uint32_t ntiles,
                                                           uint32_t nscalar, uint32_t R) {
    __shared__ f4 sh4[BLOCK * V + 2];
    flat_seq_enter<false>(p);
    const uint32_t g = blockIdx.x;
    const uint32_t grp = g / R, r = g - grp * R;
    uint32_t tile;
    if (grp < nscalar) {
        if (r == 0) {
            split_scalar<BLOCK, ABL>(p, grp);
            return;
        }
        tile = grp * (R - 1) + r - 1;
    } else {
        tile = nscalar * (R - 1) + (g - nscalar * R);
    }
    if (tile >= ntiles) return;
    split_tile<BLOCK, V, POL, ABL>(p, qtot, tile, ntiles, sh4);
}

}  // namespace pmenv_dev
