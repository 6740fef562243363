// step_env.h — the whole env step in ONE launch: one workgroup per env.
//
// TradingEnv.step (zachramsey/pm-rl env/sim/trading_env.py:44-105) plus the
// one-day window advance of the fused path (data/instrument.py:79 price relatives,
// :339-356 sliding window), for every env of the batch in a single kernel:
//
//   workgroup b owns env b's whole [N, W, F] window (per4 = N*W*F/4 16-B chunks).
//   1. wave 0 issues the env's scalar loads (action, w_last = get_last(), the
//      window's last close, the day's bar row, value / counter / reward statistics;
//      scalar_load_row, branch-free buffer loads);
//   2. every wave issues its aligned 16-B window loads (wave w owns V of the env's
//      1 KiB-aligned 64-chunk blocks, lane l chunk l of each: each load one aligned,
//      coalesced 1 KiB) — nothing waits in between;
//   3. wave 0 runs the scalar step up to w' (scalar_core: normalisation :54-60,
//      commission fixed point :62-75, value :77-79, w' :83-84) while the window is in
//      flight, and leaves w', the bar rows and the counter in LDS;
//   4. every wave parks its chunks in the LDS image of the window; one barrier;
//   5. each lane composes its output chunk from LDS neighbours (the shifted source
//      floats 4c+5 .. 4c+8 = chunks c+1, c+2) and the env's w' / bar row, and stores
//      it with one 16-B store (flat_compose, env_step.h);
//   6. wave 0 finishes the step (scalar_tail: w' into the ring / w_new, return and
//      reward :87-100, counter) after its stores, off the barrier's critical path.
//
// The workgroup owns the whole env, so the in-place advance needs no halo and no
// inter-workgroup ordering: every load of the env lands before any of its stores
// (the barrier), and the shifted source never crosses the env's end at a position
// that is kept (the last chunks' reads past the env are last-day positions, which
// take the bar). No second launch, no scalar-step kernel boundary, no halo copy.
//
// Requirements (host-checked): F == 5, W >= 2, N <= 64 (the scalar step is one
// asset per lane of wave 0), N*W*F % 4 == 0, the env's 64-chunk blocks <= 16 waves x V.
#pragma once
#include "env_step.h"

namespace pmenv_dev {

// POL: cache policy of the window stream (0 default, 1 nt); OUT: double-buffered;
// ABL (timing-only ablation, tools build): 1 = no scalar step (constant w' / bar),
// 2 = every chunk reads the bar / w' from LDS (the unconditional form), 4 = XCD-contiguous
// env ranges, 8 = default-policy loads (nt stores)
template <int V, bool OUT, int POL, int ABL>
__device__ __forceinline__ void step_env_body(const StepParams& p, uint32_t per4) {
    constexpr int kAux = POL == 1 ? 2 : 0;
    constexpr int F = 5;
    extern __shared__ __attribute__((aligned(16))) f4 sh4[];        // [64 * V * waves + 2] window image
    __shared__ f4 sh_bar[64];
    __shared__ float sh_wp[64];
    __shared__ int32_t sh_k;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int b = blockIdx.x;
    if (ABL & 4) {   // A/B: XCD-contiguous env ranges (workgroups go round-robin over the 8 XCDs)
        const int G = gridDim.x, q = G >> 3, r = G & 7, x = b & 7, i = b >> 3;
        b = x < r ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
    }
    const int WF = p.W * F;
    // The env's chunks [e0, e0 + per4) of the flat [B, N, W, F] tensor, covered by the
    // 1 KiB-aligned 64-chunk blocks from g0 = e0 / 64 on: slot s of the workgroup is
    // global chunk 64 * g0 + s, env-local chunk s - a (a = e0 - 64 * g0 < 64). Every wave
    // instruction then reads / writes one aligned 1 KiB line run (an env-aligned mapping
    // leaves most of them straddling 128-B lines: 706 against 615 us per launch at the
    // BASELINE shape); lanes outside the env fall outside the descriptor's range (read 0,
    // store nothing), so the two blocks an env shares with its neighbours are split, not raced.
    const uint64_t e0 = (uint64_t)b * per4;
    const uint32_t a = (uint32_t)(e0 & 63u);
    float* env_in = p.obs + e0 * 4;
    const auto rs = make_rsrc(env_in, per4 * 16u);
    // 1. the scalar step's loads (wave-uniform branch)
    ScalarIn sin;
    if (!(ABL & 1) && wave == 0) sin = scalar_load_row(p, b, lane);
    __builtin_amdgcn_sched_barrier(0);
    // 2. the window stream (offsets relative to the env: negative ones wrap out of range)
    f4 own[V];
#pragma unroll
    for (int v = 0; v < V; ++v)
        own[v] = buf_load4<(ABL & 8) ? 0 : kAux>(rs, ((uint32_t)(64 * V * wave + 64 * v + lane) - a) * 16u);
    __builtin_amdgcn_sched_barrier(0);
    // 3. the scalar step, on wave 0, while the window is in flight
    if ((ABL & 1) && wave == 0) {
        sh_wp[lane] = 0.5f;
        sh_bar[lane] = f4{1.f, 1.f, 1.f, 1.f};
        if (lane == 0) sh_k = 0;
    }
    ScalarMid mid;
    if (!(ABL & 1) && wave == 0) {
        mid = scalar_core<64, true>(p, b, lane, sin);
        sh_wp[lane] = mid.wp;
        sh_bar[lane] = sin.bar_ok ? sin.bar : f4{NAN, NAN, NAN, NAN};   // day outside the series: NaN bar
        if (lane == 0) sh_k = mid.k;
    }
    // 4. the window image
#pragma unroll
    for (int v = 0; v < V; ++v) sh4[64 * V * wave + 64 * v + lane] = own[v];
    __syncthreads();
    // 5. compose and store; only the chunks holding a row's last day or (ring full,
    // storage order) its weight slot read the env's bar / w' from LDS
    const int32_t k = sh_k;
    const bool shift_w = !(p.ring_mode == PMENV_RING_STORAGE && k >= p.W - 1);
    const int slot_w = (int)(((uint32_t)(1 + k) - fdiv((uint32_t)(1 + k), p.div_w) * (uint32_t)p.W) * F + (F - 1));
    const auto rd = OUT ? make_rsrc(p.obs_out + e0 * 4, per4 * 16u) : rs;
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const uint32_t slot = (uint32_t)(64 * V * wave + 64 * v + lane);
        const uint32_t c = slot - a;                                         // env-local chunk (wraps if < 0)
        const uint32_t j0 = 4u * min(c, per4 - 1u);                          // lanes outside the env: any row
        const uint32_t row = fdiv(j0, p.div_wf);
        FlatSide sd;
        sd.kk = (int)(j0 - row * (uint32_t)WF);
        sd.bar_nan = false;
        if (ABL & 2) {
            sd.xb = sh_bar[row];
            sd.xwp = sh_wp[row];
        } else {
            const bool need = sd.kk + 3 >= WF - F || (!shift_w && (uint32_t)(slot_w - sd.kk) <= 3u);
            sd.xb = f4{0.f, 0.f, 0.f, 0.f};
            sd.xwp = 0.f;
            if (need) {
                sd.xb = sh_bar[row];
                sd.xwp = sh_wp[row];
            }
        }
        sd.k = k;
        const f4 n1 = sh4[slot + 1], n2 = sh4[slot + 2];
        const float sh[4] = {n1.y, n1.z, n1.w, n2.x};
        const float un[4] = {own[v].x, own[v].y, own[v].z, own[v].w};
        buf_store4<kAux>(rd, c * 16u, flat_compose(p, sd, un, sh));          // outside the env: dropped
    }
    // 6. the rest of the scalar step after the stores: state, ring slot, return, reward
    if (!(ABL & 1) && wave == 0) scalar_tail<64>(p, b, lane, sin, mid);
}

// Held to 80 SGPRs (the compiler spills ~20 to VGPR lanes): gfx950 admits
// floor(800 / (ceil(sgpr / 16) * 16 + 16)) waves per SIMD — 7 at 82-96 SGPRs, 8 at
// <= 80 (MI355X_MICROARCH.md, Residency); measured 647-651 against 651-658 us per step
// uncapped at the BASELINE shape (profiles/ab_r02/r02e_*, r02f_*, r02j_*).
template <int V, bool OUT, int POL, int ABL = 0>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_num_sgpr(80))) void step_env_kernel(StepParams p,
                                                                                             uint32_t per4) {
    step_env_body<V, OUT, POL, ABL>(p, per4);
}

// tools build: the same kernel without the SGPR cap
template <int V, bool OUT, int POL, int ABL = 0>
__global__ __launch_bounds__(1024) void step_env_nocap_kernel(StepParams p, uint32_t per4) {
    step_env_body<V, OUT, POL, ABL>(p, per4);
}

}  // namespace pmenv_dev
