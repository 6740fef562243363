// step_flat.h — the whole env step in ONE launch over the flat window stream.
//
// TradingEnv.step (zachramsey/pm-rl env/sim/trading_env.py:44-105) and the one-day
// window advance (data/instrument.py:79 price relatives, :339-356 sliding window) for
// every env of the batch, with the workgroup geometry of the fastest window stream
// (advance_flat_inplace_kernel: fixed 16 KiB tiles of the flat [B, N, W, F] tensor,
// independent of the env size) and the scalar step folded in:
//
//   workgroup g owns output chunks [1024 g, 1024 g + 1024) of the flat tensor (16 KiB;
//   256 threads x 4 chunks), which touch envs e_lo .. e_hi (at most one per wave;
//   host-checked).
//   1. wave w < ne issues env (e_lo + w)'s scalar loads (action, bar row, and the
//      state snapshot: value, counter, get_last(), last close);
//   2. every wave issues its aligned 16-B window loads (one coalesced 1 KiB per wave
//      instruction), and lanes 0-1 the two chunks past the tile (the halo);
//   3. wave w < ne runs env (e_lo + w)'s scalar step up to w' (scalar_core: f64 DPP
//      reductions, bitwise the same as every other step path) while the window is in
//      flight, and leaves w', the bar rows and the counter in LDS;
//   4. the window image goes to LDS; ONE barrier;
//   5. each lane composes its output chunks (shifted source from LDS neighbours, the
//      env's bar / w' where a row's last day or weight slot falls) and stores them;
//   6. wave w < ne finishes env (e_lo + w)'s step after the stores (scalar_tail: the
//      state, ring slot and snapshot writes, lane 0's return and reward), so the barrier
//      of step 4 waits only for what the compose needs (scalar_core: w').
//
// Several workgroups run the scalar step of an env that straddles their tiles; only the
// workgroup holding the env's first chunk (its owner) writes the env's state, reward and
// ring slot. The others must read the state from before the step whatever the owner's
// timing, and a launch has no ordering between workgroups (cdna_hip_programming.md
// Guideline 16), so the state the scalar step reads — value, counter, get_last() and the
// window's last close — is a per-step snapshot: read from parity p, written by the owner
// into parity 1 - p; the host flips p every step (pmenv.hip). In place, the two chunks
// past a tile belong to the next tile, which may already have advanced them: they are
// the next tile's first two output chunks of the previous step, which that tile also
// stored into the halo buffer of parity 1 - p. After anything else touched the state or
// the window (reset, set_state, another step path, a different obs), the host primes
// the snapshot and the halo from the canonical state and the window (flat_prime_kernel)
// before the step. Under hipGraph capture the host-chosen parity would be frozen: from the
// first captured step on, the handle runs flat_seq_kernel before each step, which reads
// the parity and the snapshot's validity from device words and primes on the device; the
// kernel then reads the parity from memory (below).
#pragma once
#include "scalar_vec.h"

namespace pmenv_dev {

// the snapshot loads of scalar_load_row: value / counter / get_last() / last close from
// parity p, the rest as scalar_load_row (reward statistics: only the owner uses them)
__device__ __forceinline__ ScalarIn scalar_load_snap(const StepParams& p, int b, int lane) {
    const int N = p.N;
    const uint32_t nb = (uint32_t)N * 4u, off = (uint32_t)lane * 4u;
    ScalarIn in;
    in.k = p.sk_in[b];
    in.v_prev = p.sv_in[b];
    in.sa = p.sa[b];
    in.sb = p.sb[b];
    in.a = buf_load1(make_rsrc(p.action + (size_t)b * N, nb), off);
    // get_last() only feeds the commission fixed point (a handle constant): without it
    // the snapshot carries no weights (the descriptor has no records: no traffic)
    in.wlf = buf_load1(make_rsrc(p.sw_in + (size_t)b * N, p.commission > 0.0 ? nb : 0u), off);
    in.pl = buf_load1(make_rsrc((p.prices ? p.prices : p.slc_in) + (size_t)b * N, nb), off);
    const float* barb = env_bar(p, b);            // null: out-of-range day -> the descriptor reads 0
    in.bar = buf_load4(make_rsrc(barb ? barb : p.bar, barb ? nb * 4u : 0u), off * 4u);
    in.bar_ok = barb != nullptr;
    in.cn = 0.0f;
    return in;
}

// What a tile needs from memory: its window chunks, the two chunks past it (halo), and
// wave w's env scalar inputs (w < ne).
template <int V>
struct FlatTile {
    uint32_t c0, nblk, e_lo;
    int ne;
    f4 own[V];
    f4 hal;
    ScalarIn sin;
};

// AUX: the window loads' buffer cache-policy bits (0 default, 2 nt)
template <int BLOCK, int V, int AUX, bool OUT>
__device__ __forceinline__ void flat1_load(const StepParams& p, uint32_t qtot, uint32_t tile, FlatTile<V>& t) {
    constexpr int CPW = BLOCK * V;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    t.c0 = tile * (uint32_t)CPW;
    t.nblk = min((uint32_t)CPW, qtot - t.c0);
    t.e_lo = fdiv(t.c0, p.div_units);                                  // div_units: per4
    t.ne = (int)(fdiv(t.c0 + t.nblk - 1u, p.div_units) - t.e_lo) + 1;  // <= BLOCK / 64 (host-checked)
    // 1. the scalar step's loads (wave-uniform branch), 2. the window stream and the halo
    if (wave < t.ne) t.sin = scalar_load_snap(p, (int)t.e_lo + wave, lane);
    __builtin_amdgcn_sched_barrier(0);
    const auto rs = make_rsrc(p.obs + (size_t)t.c0 * 4, t.nblk * 16u);
#pragma unroll
    for (int v = 0; v < V; ++v) t.own[v] = buf_load4<AUX>(rs, (uint32_t)(64 * V * wave + 64 * v + lane) * 16u);
    const uint32_t ntiles = (qtot + CPW - 1) / CPW;
    const uint32_t nh = tile + 1 < ntiles ? min(2u, qtot - t.c0 - t.nblk) : 0u;
    const float* hsrc = OUT ? p.obs + (size_t)(t.c0 + t.nblk) * 4 : p.halo_in + (size_t)tile * 8;
    t.hal = buf_load4<0>(make_rsrc(hsrc, nh * 16u), tid < 2 ? (uint32_t)tid * 16u : 0xFFFFFFF0u);
    __builtin_amdgcn_sched_barrier(0);
}

// AUX: the window stores' buffer cache-policy bits (0 default, 2 nt)
template <int BLOCK, int V, int AUX, bool OUT>
__device__ __forceinline__ void flat1_process(const StepParams& p, uint32_t qtot, uint32_t tile, const FlatTile<V>& t,
                                              f4* sh4, f4 (*sh_bar)[64], float (*sh_wp)[64], int32_t* sh_k) {
    constexpr int CPW = BLOCK * V, F = 5;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t per4 = p.per4;
    // 3. the scalar steps' cores, one env per wave (their tails run after the stores)
    ScalarMid mid;
    if (wave < t.ne) {
        mid = scalar_core<64, true>(p, (int)t.e_lo + wave, lane, t.sin);
        sh_wp[wave][lane] = mid.wp;
        sh_bar[wave][lane] = t.sin.bar_ok ? t.sin.bar : f4{NAN, NAN, NAN, NAN};   // day outside the series
        if (lane == 0) sh_k[wave] = mid.k;
    }
    // 4. the window image
#pragma unroll
    for (int v = 0; v < V; ++v) sh4[64 * V * wave + 64 * v + lane] = t.own[v];
    if (tid < 2) sh4[CPW + tid] = t.hal;
    __syncthreads();
    // 5. compose and store; only chunks holding a row's last day or (ring full, storage
    // order) its weight slot read the env's bar / w' from LDS
    const int WF = p.W * F;
    const auto rd = make_rsrc((OUT ? p.obs_out : p.obs) + (size_t)t.c0 * 4, t.nblk * 16u);
    const bool first_out = !OUT && tile > 0;                            // feeds the previous tile's halo
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int j = 64 * V * wave + 64 * v + lane;
        const uint32_t q = min(t.c0 + (uint32_t)j, qtot - 1u);          // lanes past the end: any chunk
        const uint32_t e = fdiv(q, p.div_units);
        const int le = (int)(e - t.e_lo);
        const uint32_t j0 = 4u * (q - e * per4);
        const uint32_t row = fdiv(j0, p.div_wf);
        const int kk = (int)(j0 - row * (uint32_t)WF);
        const f4 n1 = sh4[j + 1], n2 = sh4[j + 2];
        const float sh[4] = {n1.y, n1.z, n1.w, n2.x};
        const float un[4] = {t.own[v].x, t.own[v].y, t.own[v].z, t.own[v].w};
        // the two-level compose: only chunks holding a row's last day or ring slot read the
        // env's bar / w' from LDS
        const f4 o = compose2(p, kk, sh_k[le], un, sh, [&](f4& xb, float& xwp) {
            xb = sh_bar[le][row];
            xwp = sh_wp[le][row];
        });
        buf_store4<AUX>(rd, (uint32_t)j * 16u, o);                     // past the end: dropped
        if (first_out && j < 2) reinterpret_cast<f4*>(p.halo_out)[2 * (tile - 1) + j] = o;
    }
    // 6. the scalar steps' tails: state, ring slot, snapshot and reward (the owner only)
    if (wave < t.ne) {
        const int b = (int)t.e_lo + wave;
        const bool owner = (uint64_t)b * per4 >= t.c0;                 // the env's first chunk is ours
        scalar_tail<64, true>(p, b, lane, t.sin, mid, owner);
    }
}

// The device-sequenced step (p.seq set): take the parity C that flat_seq_kernel published
// (nothing writes C during this launch) — swap the *_in / *_out snapshot and halo pointers
// when it is 1 — and from workgroup 0 publish the next step's D, V and HOBS (nothing reads
// them during this launch).
template <bool OUT>
__device__ __forceinline__ void flat_seq_enter(StepParams& p) {
    if (!p.seq) return;
    const int c = __builtin_amdgcn_readfirstlane(p.seq[1]);
    if (c) {
        const double* v = p.sv_in; p.sv_in = p.sv_out; p.sv_out = const_cast<double*>(v);
        const int32_t* k = p.sk_in; p.sk_in = p.sk_out; p.sk_out = const_cast<int32_t*>(k);
        const float* w = p.sw_in; p.sw_in = p.sw_out; p.sw_out = const_cast<float*>(w);
        const float* l = p.slc_in; p.slc_in = p.slc_out; p.slc_out = const_cast<float*>(l);
        const float* h = p.halo_in; p.halo_in = p.halo_out; p.halo_out = const_cast<float*>(h);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const uint64_t hobs = OUT ? 0ull : (uint64_t)(uintptr_t)p.obs;
        p.seq[0] = 1 - c;
        p.seq[2] = 1;
        p.seq[4] = (int32_t)(uint32_t)hobs;
        p.seq[5] = (int32_t)(uint32_t)(hobs >> 32);
    }
}

// POL: cache policy of the window stream, loads and stores (0 default, 1 nt); OUT:
// double-buffered (the two chunks past a tile are read straight from obs, no halo).
// BLOCK x V: 128 x 8 / 256 x 4 (env windows of >= 511 chunks) or 512 x 2 (148 .. 510),
// host-chosen. Held to 80 SGPRs where the compiler can (512 x 2: 8 waves per SIMD
// instead of 7). (The tile orders and per-direction policies measured against it are
// the tools build's step_flat_ab_kernel, tools/ab/ab_kernels.h.)
template <int BLOCK, int V, int POL, bool OUT>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_num_sgpr(80))) void step_flat_kernel(StepParams p,
                                                                                              uint32_t qtot) {
    constexpr int CPW = BLOCK * V, WAVES = BLOCK / 64, AUX = POL == 1 ? 2 : 0;
    __shared__ f4 sh4[CPW + 2];
    __shared__ f4 sh_bar[WAVES][64];
    __shared__ float sh_wp[WAVES][64];
    __shared__ int32_t sh_k[WAVES];
    flat_seq_enter<OUT>(p);
    FlatTile<V> t;
    flat1_load<BLOCK, V, AUX, OUT>(p, qtot, blockIdx.x, t);
    flat1_process<BLOCK, V, AUX, OUT>(p, qtot, blockIdx.x, t, sh4, sh_bar, sh_wp, sh_k);
}

// ---------------------------------------------------------------- wide envs (64 < N <= 512)
// step_flat_kernel with the packed scalar step (scalar_vec.h: A strided assets per lane,
// the two-launch path's own loads and reductions, so the two give the same bits): an env
// window there spans 4,000 - 32,000 chunks, so a 16 KiB tile holds parts of at most two
// envs and most tiles one. Each tile runs the scalar step of the env(s) it holds — the
// reductions need every asset — but stages only the rows it touches: the bar rows and w'
// of at most 64 rows per env (host-checked), the same LDS as the narrow kernel. The
// snapshot, the halo and the device sequencing are step_flat_kernel's.
template <int A, int BLOCK, int V, int POL, bool OUT>
__global__ __launch_bounds__(BLOCK) void step_flat_vec_kernel(StepParams p, uint32_t qtot) {
    constexpr int kAuxL = POL == 1 ? 2 : 0, kAuxS = POL == 1 ? 2 : 0;
    constexpr int CPW = BLOCK * V, WAVES = BLOCK / 64, F = 5;
    __shared__ f4 sh4[CPW + 2];
    __shared__ f4 sh_bar[WAVES][64];
    __shared__ float sh_wp[WAVES][64];
    __shared__ int32_t sh_k[WAVES], sh_rlo[WAVES];
    const uint32_t tile = blockIdx.x;
    flat_seq_enter<OUT>(p);
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int N = p.N, WF = p.W * F;
    const uint32_t per4 = p.per4;
    const uint32_t c0 = tile * (uint32_t)CPW;
    const uint32_t nblk = min((uint32_t)CPW, qtot - c0);
    const uint32_t e_lo = fdiv(c0, p.div_units);
    const int ne = (int)(fdiv(c0 + nblk - 1u, p.div_units) - e_lo) + 1;   // <= WAVES (host-checked)
    // 1. wave w < ne: env (e_lo + w)'s scalar loads and the bar rows the tile touches
    VecIn<A> vin;
    f4 brow = f4{0.f, 0.f, 0.f, 0.f};
    int rlo = 0;
    bool bar_ok = false;
    const int b = (int)e_lo + wave;
    if (wave < ne) {
        vin = vec_load<64, A, true, true>(p, b, lane);
        const uint64_t eb = (uint64_t)b * per4;
        const uint32_t qa = (uint32_t)(max((uint64_t)c0, eb) - eb);                          // env-local chunks
        const uint32_t qb = (uint32_t)(min((uint64_t)c0 + nblk - 1u, eb + per4 - 1u) - eb);  // in this tile
        rlo = (int)fdiv(4u * qa, p.div_wf);
        const int rhi = min((int)fdiv(4u * qb + 3u, p.div_wf), N - 1);
        const float* barb = env_bar(p, b);
        bar_ok = barb != nullptr;
        const auto rb = make_rsrc(barb ? barb : p.bar, barb ? (uint32_t)(rhi + 1) * 16u : 0u);
        brow = buf_load4<0>(rb, (uint32_t)(rlo + lane) * 16u);                             // rows past rhi: 0
    }
    __builtin_amdgcn_sched_barrier(0);
    // 2. the window stream and the halo
    const auto rs = make_rsrc(p.obs + (size_t)c0 * 4, nblk * 16u);
    f4 own[V];
#pragma unroll
    for (int v = 0; v < V; ++v) own[v] = buf_load4<kAuxL>(rs, (uint32_t)(64 * V * wave + 64 * v + lane) * 16u);
    const uint32_t ntiles = (qtot + CPW - 1) / CPW;
    const uint32_t nh = tile + 1 < ntiles ? min(2u, qtot - c0 - nblk) : 0u;
    const float* hsrc = OUT ? p.obs + (size_t)(c0 + nblk) * 4 : p.halo_in + (size_t)tile * 8;
    const f4 hal = buf_load4<0>(make_rsrc(hsrc, nh * 16u), tid < 2 ? (uint32_t)tid * 16u : 0xFFFFFFF0u);
    __builtin_amdgcn_sched_barrier(0);
    // 3. the scalar steps (state, ring slot, snapshot and reward by the env's owner only)
    if (wave < ne) {
        const VecMid<A> mid = vec_core<64, A, true>(p, b, lane, vin);
#pragma unroll
        for (int e = 0; e < A; ++e) {
            const int n = lane + 64 * e;
            if ((unsigned)(n - rlo) < 64u) sh_wp[wave][n - rlo] = mid.wp[e];
        }
        sh_bar[wave][lane] = bar_ok ? brow : f4{NAN, NAN, NAN, NAN};                      // day outside the series
        if (lane == 0) {
            sh_k[wave] = vin.k;
            sh_rlo[wave] = rlo;
        }
        const bool owner = (uint64_t)b * per4 >= c0;                    // the env's first chunk is ours
        vec_tail<64, A, true, true>(p, b, lane, vin, mid, owner);
    }
    // 4. the window image
#pragma unroll
    for (int v = 0; v < V; ++v) sh4[64 * V * wave + 64 * v + lane] = own[v];
    if (tid < 2) sh4[CPW + tid] = hal;
    __syncthreads();
    // 5. compose and store
    const auto rd = make_rsrc((OUT ? p.obs_out : p.obs) + (size_t)c0 * 4, nblk * 16u);
    const bool first_out = !OUT && tile > 0;                            // feeds the previous tile's halo
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int j = 64 * V * wave + 64 * v + lane;
        const uint32_t q = min(c0 + (uint32_t)j, qtot - 1u);            // lanes past the end: any chunk
        const uint32_t e = fdiv(q, p.div_units);
        const int le = (int)(e - e_lo);
        const uint32_t j0 = 4u * (q - e * per4);
        const uint32_t row = fdiv(j0, p.div_wf);
        const int kk = (int)(j0 - row * (uint32_t)WF);
        const f4 n1 = sh4[j + 1], n2 = sh4[j + 2];
        const float sh[4] = {n1.y, n1.z, n1.w, n2.x};
        const float un[4] = {own[v].x, own[v].y, own[v].z, own[v].w};
        const f4 o = compose2(p, kk, sh_k[le], un, sh, [&](f4& xb, float& xwp) {
            const int r = (int)row - sh_rlo[le];
            xb = sh_bar[le][r];
            xwp = sh_wp[le][r];
        });
        buf_store4<kAuxS>(rd, (uint32_t)j * 16u, o);                    // past the end: dropped
        if (first_out && j < 2) reinterpret_cast<f4*>(p.halo_out)[2 * (tile - 1) + j] = o;
    }
}

// The snapshot copy (sv_out .. slc_out <- the canonical state, when `snap`) and the halo
// copy (copy_halo, when p.halo is set), grid-stride over the launch.
__device__ __forceinline__ void flat_prime(const StepParams& p, bool snap) {
    copy_halo(p);
    if (!snap) return;
    const uint32_t nthr = gridDim.x * blockDim.x;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    const size_t BN = (size_t)p.B * p.N;
    for (size_t i = tid; i < (size_t)p.B; i += nthr) {
        p.sv_out[i] = p.value[i];
        p.sk_out[i] = p.k[i];
    }
    for (size_t i = tid; i < BN; i += nthr) {
        p.sw_out[i] = p.w_new[i];
        p.slc_out[i] = p.last_close[i];
    }
}

// The device-sequenced form's first node (hipGraph-safe: every decision is read from
// device memory, none is a launch argument): reads D, V and HOBS (nothing writes them
// during this launch), re-primes the snapshot of parity D from the canonical state when
// V == 0 and — in place — the halo of parity D from the window when HOBS is not this
// step's window, and publishes C = D for the flat kernel (which reads nothing else of
// seq). *_out / halo point at parity 0, the kernel adds parity D's offset (`stride`
// bytes between the parities).
static __global__ __launch_bounds__(256) void flat_seq_kernel(StepParams p, int out, uint64_t stride) {
    const int d = __builtin_amdgcn_readfirstlane(p.seq[0]);
    const int valid = __builtin_amdgcn_readfirstlane(p.seq[2]);
    const uint64_t hobs = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(p.seq[4]) |
                          ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(p.seq[5]) << 32);
    const bool snap = !valid;
    const bool halo = !out && (!valid || hobs != (uint64_t)(uintptr_t)p.obs);
    if (snap || halo) {
        const uint64_t off = d ? stride : 0ull;
        StepParams q = p;
        q.sv_out = (double*)((char*)p.sv_out + off);
        q.sk_out = (int32_t*)((char*)p.sk_out + off);
        q.sw_out = (float*)((char*)p.sw_out + off);
        q.slc_out = (float*)((char*)p.slc_out + off);
        q.halo = halo ? (float*)((char*)p.halo + off) : nullptr;
        flat_prime(q, snap);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) p.seq[1] = d;
}

// Prime the snapshot (parity p) from the canonical state and, in place, the halo of
// parity p from the window: halo[i] = chunks (i+1)*CPW and (i+1)*CPW + 1 (copy_halo).
static __global__ __launch_bounds__(256) void flat_prime_kernel(StepParams p) { flat_prime(p, true); }

}  // namespace pmenv_dev
