// rollout.h — rollout return pass and advantage moments.
// The reference's replay/rollout_buffer.py stores (s, a, v, r) (:43-57) and computes
// no returns; the north star asks for its GAE / discounted-return pass on device.
#pragma once
#include "common.h"

namespace pmenv_dev {

// ---------------------------------------------------------------- GAE / moments
// One thread per env walks its column of the [T, B] rollout backwards; for a fixed
// t the B threads touch B consecutive floats, so every access is coalesced.
static __global__ void gae_kernel(const float* r, const float* v, const uint8_t* dones, float* adv, float* ret,
                           int T, int B, float gamma, float lam) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    double a = 0.0;
    for (int t = T - 1; t >= 0; --t) {
        size_t i = (size_t)t * B + b;
        double nd = dones ? (dones[i] ? 0.0 : 1.0) : 1.0;
        double vt = (double)v[i];
        double delta = (double)r[i] + (double)gamma * nd * (double)v[i + B] - vt;
        a = delta + (double)gamma * (double)lam * nd * a;
        adv[i] = (float)a;
        ret[i] = (float)(a + vt);
    }
}

// GAE as a parallel scan for few envs x long horizons: one wave per env, the
// horizon cut into 64 chunks (one per lane). The recursion A_t = d_t + c_t A_{t+1}
// (c_t = gamma*lambda*(1-done_t)) makes each chunk an affine map f(x) = D + C x from
// the advantage after the chunk to the advantage at its start; a suffix scan of
// the 64 maps (composition (C, D) o (C', D') = (C C', D + C D'), six shuffle steps)
// gives every lane its carry-in, and each lane then re-walks its chunk.
__device__ __forceinline__ void gae_delta(const float* r, const float* v, const uint8_t* dones, int t, int B, int b,
                                          float gamma, float lam, double* delta, double* c) {
    const size_t i = (size_t)t * B + b;
    const double nd = dones ? (dones[i] ? 0.0 : 1.0) : 1.0;
    *delta = (double)r[i] + (double)gamma * nd * (double)v[i + B] - (double)v[i];
    *c = (double)gamma * (double)lam * nd;
}

static __global__ __launch_bounds__(256) void gae_scan_kernel(const float* r, const float* v, const uint8_t* dones,
                                                       float* adv, float* ret, int T, int B, float gamma, float lam) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= B) return;
    const int L = (T + 63) / 64;
    const int t0 = min(lane * L, T), t1 = min(t0 + L, T);
    double C = 1.0, D = 0.0;
    for (int t = t1 - 1; t >= t0; --t) {
        double dl, c;
        gae_delta(r, v, dones, t, B, b, gamma, lam, &dl, &c);
        D = dl + c * D;
        C = c * C;
    }
    // suffix composition g_l = f_l o f_{l+1} o ... o f_63
    for (int o = 1; o < 64; o <<= 1) {
        const double C2 = __shfl_down(C, o, 64), D2 = __shfl_down(D, o, 64);
        if (lane + o < 64) {
            D = D + C * D2;
            C = C * C2;
        }
    }
    double a = __shfl_down(D, 1, 64);             // advantage at the start of the next chunk
    if (lane == 63) a = 0.0;
    for (int t = t1 - 1; t >= t0; --t) {
        double dl, c;
        gae_delta(r, v, dones, t, B, b, gamma, lam, &dl, &c);
        a = dl + c * a;
        const size_t i = (size_t)t * B + b;
        adv[i] = (float)a;
        ret[i] = (float)(a + (double)v[i]);
    }
}

// GAE as a tiled scan for many envs: a workgroup owns 64 envs (one per lane, so
// every load and store is a coalesced 256-B row of the time-major rollout) and
// walks the horizon backwards in segments of NW x U steps; wave w holds sub-chunk
// w of the segment in registers (each input read exactly once), reduces it to its
// affine map (C, D), and after one LDS exchange composes the later sub-chunks'
// maps onto the segment's carry to get its own carry-in, then re-walks its
// registers writing adv / ret. f64 throughout, like the sequential recursion.
// Loads are buffer loads with the lane's env as the (only) VGPR offset and the
// wave-uniform row as the SGPR offset, so U rows in flight cost no address VGPRs.
// Needs every array below 2 GiB (the host checks).
// SP: cache-policy bits of the adv / ret stores (0 in the product; tools A/B)
template <int NW, int U, int OCC = 1, int SP = 0>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(OCC))) void gae_tile_kernel(
    const float* r, const float* v, const uint8_t* dones, float* adv, float* ret, int T, int B, float gamma,
    float lam) {
    __shared__ double shC[NW][64], shD[NW][64];
    constexpr int S = NW * U;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: rows go in SGPRs
    const int b = blockIdx.x * 64 + lane;
    const bool ok = b < B;
    const uint32_t voff = (uint32_t)(ok ? b : B - 1) * 4u;
    const uint32_t row = (uint32_t)B * 4u;
    const auto rs_r = make_rsrc(r, (uint32_t)T * row);
    const auto rs_v = make_rsrc(v, (uint32_t)(T + 1) * row);
    const auto rs_d = make_rsrc(dones ? (const void*)dones : (const void*)r, dones ? (uint32_t)T * (uint32_t)B : 0u);
    const auto rs_adv = make_rsrc(adv, (uint32_t)T * row);
    const auto rs_ret = make_rsrc(ret, (uint32_t)T * row);
    const uint32_t voff_st = ok ? voff : 0x80000000u;
    const double g = (double)gamma, gl = (double)gamma * (double)lam;
    double carry = 0.0;                           // advantage just after the current segment
    for (int seg_end = T; seg_end > 0; seg_end -= S) {
        const int seg_start = max(seg_end - S, 0);
        const int t0 = seg_start + w * U;
        float vv[U + 1], rr[U];
        uint32_t alive = 0;                       // bit u: 1 - done_t
#pragma unroll
        for (int u = 0; u <= U; ++u) {            // v has T + 1 rows: row seg_end is the bootstrap
            const uint32_t t = (uint32_t)min(t0 + u, seg_end);
            vv[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_v, voff, t * row, 0));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t t = (uint32_t)min(t0 + u, seg_end - 1);
            rr[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_r, voff, t * row, 0));
            // no dones: the descriptor has no records and every load reads 0 (alive)
            const uint32_t dn = __builtin_amdgcn_raw_buffer_load_b8(rs_d, voff >> 2, t * (uint32_t)B, 0);
            alive |= (dn ? 0u : 1u) << u;
        }
        // delta_t, kept for the second walk (OCC >= 8: recomputed there, the same bits, so
        // the kernel fits 64 VGPRs)
        constexpr bool RECOMP = OCC >= 8;
        double dl[RECOMP ? 1 : U];
        double C = 1.0, D = 0.0;
#pragma unroll
        for (int u = U - 1; u >= 0; --u) {
            const double n = (alive >> u) & 1u ? 1.0 : 0.0;
            const double d = (double)rr[u] + g * n * (double)vv[u + 1] - (double)vv[u];
            if (!RECOMP) dl[u] = d;
            if (t0 + u < seg_end) {
                D = d + gl * n * D;
                C = gl * n * C;
            }
        }
        shC[w][lane] = C;
        shD[w][lane] = D;
        __syncthreads();
        if (RECOMP) {                             // opaque to the optimiser: no delta stays live
#pragma unroll
            for (int u = 0; u < U; ++u) asm volatile("" : "+v"(rr[u]));
#pragma unroll
            for (int u = 0; u <= U; ++u) asm volatile("" : "+v"(vv[u]));
        }
        double a = carry;
        for (int j = NW - 1; j > w; --j) a = shD[j][lane] + shC[j][lane] * a;
#pragma unroll
        for (int u = U - 1; u >= 0; --u) {
            const int t = t0 + u;
            if (t < seg_end) {
                const double n = (alive >> u) & 1u ? 1.0 : 0.0;
                const double d = RECOMP ? (double)rr[u] + g * n * (double)vv[u + 1] - (double)vv[u] : dl[RECOMP ? 0 : u];
                a = d + gl * n * a;
                // lanes past B: voff is out of range for the store descriptors -> dropped
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)a), rs_adv, voff_st, (uint32_t)t * row, SP);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)(a + (double)vv[u])), rs_ret, voff_st,
                                                      (uint32_t)t * row, SP);
            }
        }
        for (int j = NW - 1; j >= 0; --j) carry = shD[j][lane] + shC[j][lane] * carry;
        __syncthreads();                          // the LDS maps are rewritten next segment
    }
}

// GAE as a pipelined per-env walk for many envs (B / 64 waves fill the SIMDs): one lane
// per env, so a wave's rows are coalesced 256-B runs of the time-major rollout; the
// horizon walked backwards in blocks of P days whose loads are issued one block ahead
// (P rows of r, v and done in flight per wave while the previous block is consumed), no
// LDS, no barrier, no second pass. The recursion is gae_kernel's, in f64.
template <int P>
__device__ __forceinline__ void gae_stream_load(__amdgpu_buffer_rsrc_t rs_r, __amdgpu_buffer_rsrc_t rs_v,
                                                __amdgpu_buffer_rsrc_t rs_d, uint32_t voff, uint32_t row, int B,
                                                int tb, float* rr, float* vv, uint32_t& alive) {
    alive = 0;
#pragma unroll
    for (int u = 0; u < P; ++u) {
        const uint32_t t = (uint32_t)max(tb - P + u, 0);          // days before 0: row 0 again, unused
        rr[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_r, voff, t * row, 0));
        vv[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_v, voff, t * row, 0));
        const uint32_t dn = __builtin_amdgcn_raw_buffer_load_b8(rs_d, voff >> 2, t * (uint32_t)B, 0);
        alive |= (dn ? 0u : 1u) << u;
    }
}

template <int P>
__device__ __forceinline__ void gae_stream_block(__amdgpu_buffer_rsrc_t rs_adv, __amdgpu_buffer_rsrc_t rs_ret,
                                                 uint32_t voff_st, uint32_t row, int tb, const float* rr,
                                                 const float* vv, uint32_t alive, double g, double gl, double& a,
                                                 float& vnext) {
#pragma unroll
    for (int u = P - 1; u >= 0; --u) {
        const int t = tb - P + u;
        if (t >= 0) {
            const double n = (alive >> u) & 1u ? 1.0 : 0.0;
            const double vt = (double)vv[u];
            const double delta = (double)rr[u] + g * n * (double)vnext - vt;
            a = delta + gl * n * a;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)a), rs_adv, voff_st, (uint32_t)t * row, 0);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)(a + vt)), rs_ret, voff_st, (uint32_t)t * row,
                                                  0);
            vnext = vv[u];
        }
    }
}

template <int P>
__global__ __launch_bounds__(64) void gae_stream_kernel(const float* r, const float* v, const uint8_t* dones,
                                                       float* adv, float* ret, int T, int B, float gamma, float lam) {
    const int lane = threadIdx.x;
    const int b = blockIdx.x * 64 + lane;
    const bool ok = b < B;
    const uint32_t voff = (uint32_t)(ok ? b : B - 1) * 4u;
    const uint32_t row = (uint32_t)B * 4u;
    const auto rs_r = make_rsrc(r, (uint32_t)T * row);
    const auto rs_v = make_rsrc(v, (uint32_t)(T + 1) * row);
    const auto rs_d = make_rsrc(dones ? (const void*)dones : (const void*)r, dones ? (uint32_t)T * (uint32_t)B : 0u);
    const auto rs_adv = make_rsrc(adv, (uint32_t)T * row);
    const auto rs_ret = make_rsrc(ret, (uint32_t)T * row);
    const uint32_t voff_st = ok ? voff : 0x80000000u;
    const double g = (double)gamma, gl = (double)gamma * (double)lam;
    float cr[P], cv[P], nr[P], nv[P];
    uint32_t ca, na;
    float vnext = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_v, voff, (uint32_t)T * row, 0));
    double a = 0.0;
    gae_stream_load<P>(rs_r, rs_v, rs_d, voff, row, B, T, cr, cv, ca);
    for (int tb = T; tb > 0; tb -= 2 * P) {
        if (tb - P > 0) gae_stream_load<P>(rs_r, rs_v, rs_d, voff, row, B, tb - P, nr, nv, na);
        gae_stream_block<P>(rs_adv, rs_ret, voff_st, row, tb, cr, cv, ca, g, gl, a, vnext);
        if (tb - P <= 0) break;
        if (tb - 2 * P > 0) gae_stream_load<P>(rs_r, rs_v, rs_d, voff, row, B, tb - 2 * P, cr, cv, ca);
        gae_stream_block<P>(rs_adv, rs_ret, voff_st, row, tb - P, nr, nv, na, g, gl, a, vnext);
    }
}

// The horizon split in ONE pass for rollouts with too few envs to fill the chip: grid (env
// blocks of 64) x (chunks of S = NW x U days), the LATER chunks dispatched first. A
// workgroup loads its chunk once into registers (the tile kernel's loads), reduces it to the
// per-env affine map A(chunk start) = D + C A(after the chunk), and publishes it: the maps
// with agent-scope atomic stores, then — after an order-only fence (workgroup-scope release
// and s_waitcnt vmcnt(0), no L2 write-back) — a 64-bit flag holding the call's epoch (the
// pattern of rocPRIM's look-back scan state on gfx942 / gfx950). It then composes every
// later chunk's map into its carry — the NW waves each take a contiguous part of the later
// chunks, waiting for their flags and reading their maps through agent-scope atomic loads,
// and the parts are composed in order through LDS — and walks its registers writing adv /
// ret (nt stores: written once, read by the learner later). Inputs are read once (17 B
// per element, against 26 for the maps + apply split).
//
// Forward progress does not rest on dispatch order: a wave that has waited kLbSpin polls for
// a later chunk's flag computes that chunk's map itself, from the inputs, with the producer's
// own code and association order (lb_wave_map folded as the publisher folds), so the bits are
// the producer's and the wait always ends — whatever order the hardware dispatches workgroups
// in (with the usual later-chunks-first dispatch the fallback never runs; the tools build's
// SPIN = 0 form takes it on the first poll that finds a flag missing, and gives the product's
// bits: tools/ab_gae_fallback.py).
constexpr int kLbSpin = 4096;

template <int U>
__device__ __forceinline__ void lb_load_wave(const __amdgpu_buffer_rsrc_t& rs_r, const __amdgpu_buffer_rsrc_t& rs_v,
                                             const __amdgpu_buffer_rsrc_t& rs_d, uint32_t voff, uint32_t row, int B,
                                             int t0, int seg_end, float* vv, float* rr, uint32_t& alive) {
    alive = 0;
#pragma unroll
    for (int u = 0; u <= U; ++u) {                // v has T + 1 rows: row seg_end closes the chunk
        const uint32_t t = (uint32_t)min(t0 + u, seg_end);
        vv[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_v, voff, t * row, 0));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t t = (uint32_t)min(t0 + u, seg_end - 1);
        rr[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_r, voff, t * row, 0));
        const uint32_t dn = __builtin_amdgcn_raw_buffer_load_b8(rs_d, voff >> 2, t * (uint32_t)B, 0);
        alive |= (dn ? 0u : 1u) << u;
    }
}

// one wave's U days reduced to its map (C, D) and the days' deltas
template <int U>
__device__ __forceinline__ void lb_wave_map(const float* vv, const float* rr, uint32_t alive, int t0, int seg_end,
                                            double g, double gl, double* dl, double& C, double& D) {
    C = 1.0;
    D = 0.0;
#pragma unroll
    for (int u = U - 1; u >= 0; --u) {
        const double n = (alive >> u) & 1u ? 1.0 : 0.0;
        dl[u] = (double)rr[u] + g * n * (double)vv[u + 1] - (double)vv[u];
        if (t0 + u < seg_end) {
            D = dl[u] + gl * n * D;
            C = gl * n * C;
        }
    }
}

// the publisher's fold of the NW waves' maps (wave NW-1 first)
__device__ __forceinline__ void lb_fold(double Cj, double Dj, double& Ca, double& Da) {
    Da = Dj + Cj * Da;
    Ca = Cj * Ca;
}

template <int NW, int U, int SPIN = kLbSpin>
__global__ __launch_bounds__(64 * NW) void gae_lookback_kernel(const float* r, const float* v, const uint8_t* dones,
                                                              float* adv, float* ret, int T, int B, float gamma,
                                                              float lam, int nC, double* maps, uint64_t* flags,
                                                              uint64_t epoch) {
    __shared__ double shC[NW][64], shD[NW][64];     // the chunk's per-wave maps
    __shared__ double sxC[NW][64], sxD[NW][64];     // the later chunks' maps, a part per wave
    constexpr int S = NW * U;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nEB = (B + 63) / 64;
    const int c = nC - 1 - (int)(blockIdx.x / (unsigned)nEB);
    const int eb = (int)(blockIdx.x % (unsigned)nEB);
    const int b = eb * 64 + lane;
    const bool ok = b < B;
    const uint32_t voff = (uint32_t)(ok ? b : B - 1) * 4u;
    const uint32_t row = (uint32_t)B * 4u;
    const auto rs_r = make_rsrc(r, (uint32_t)T * row);
    const auto rs_v = make_rsrc(v, (uint32_t)(T + 1) * row);
    const auto rs_d = make_rsrc(dones ? (const void*)dones : (const void*)r, dones ? (uint32_t)T * (uint32_t)B : 0u);
    const auto rs_adv = make_rsrc(adv, (uint32_t)T * row);
    const auto rs_ret = make_rsrc(ret, (uint32_t)T * row);
    const uint32_t voff_st = ok ? voff : 0x80000000u;
    const double g = (double)gamma, gl = (double)gamma * (double)lam;
    const int seg_start = c * S, seg_end = min(T, seg_start + S);
    const int t0 = seg_start + w * U;
    float vv[U + 1], rr[U];
    uint32_t alive;
    lb_load_wave<U>(rs_r, rs_v, rs_d, voff, row, B, t0, seg_end, vv, rr, alive);
    double dl[U];
    double C, D;
    lb_wave_map<U>(vv, rr, alive, t0, seg_end, g, gl, dl, C, D);
    shC[w][lane] = C;
    shD[w][lane] = D;
    __syncthreads();
    double* mapC = maps;
    double* mapD = maps + (size_t)nC * B;
    if (w == 0) {                                 // publish the chunk's map
        double Ca = 1.0, Da = 0.0;
        for (int j = NW - 1; j >= 0; --j) lb_fold(shC[j][lane], shD[j][lane], Ca, Da);
        if (ok) {
            __hip_atomic_store(mapC + (size_t)c * B + b, Ca, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(mapD + (size_t)c * B + b, Da, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_s_waitcnt(0 | (0x7 << 4) | (0xf << 8));          // vmcnt(0): the maps are written
        if (lane == 0) __hip_atomic_store(flags + (size_t)c * nEB + eb, epoch, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
    }
    // this wave's part of the later chunks: [j0, j1)
    const int nl = nC - 1 - c, m = (nl + NW - 1) / NW;
    const int j0 = c + 1 + w * m, j1 = min(nC, j0 + m);
    double Cw = 1.0, Dw = 0.0;
    if (j0 < j1) {
        for (int base = j0; base < j1; base += 64) {
            const int j = base + lane;
            bool ready = j >= j1 || __hip_atomic_load(flags + (size_t)j * nEB + eb, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT) == epoch;
            for (int spin = 0; !__all(ready); ++spin) {
                if (spin >= SPIN) {
                    // the producers of the chunks still missing may not be running: compute
                    // their maps here (all 64 lanes, one chunk at a time), as they would
                    uint64_t miss = __ballot(!ready);
                    while (miss) {
                        const int jm = base + (int)__builtin_ctzll(miss);
                        miss &= miss - 1;
                        double Ca = 1.0, Da = 0.0;
                        const int s0 = jm * S, s1 = min(T, s0 + S);
                        for (int jw = NW - 1; jw >= 0; --jw) {
                            float fv[U + 1], fr[U];
                            uint32_t fa;
                            double fdl[U], Cj, Dj;
                            lb_load_wave<U>(rs_r, rs_v, rs_d, voff, row, B, s0 + jw * U, s1, fv, fr, fa);
                            lb_wave_map<U>(fv, fr, fa, s0 + jw * U, s1, g, gl, fdl, Cj, Dj);
                            lb_fold(Cj, Dj, Ca, Da);
                        }
                        if (ok) {                 // the producer's values: a race of equal stores
                            __hip_atomic_store(mapC + (size_t)jm * B + b, Ca, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                            __hip_atomic_store(mapD + (size_t)jm * B + b, Da, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                        }
                    }
                    ready = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                if (!ready)
                    ready = __hip_atomic_load(flags + (size_t)j * nEB + eb, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT) == epoch;
            }
        }
        __builtin_amdgcn_s_waitcnt(0 | (0x7 << 4) | (0xf << 8));
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const size_t bb = (size_t)(ok ? b : B - 1);
        for (int hi = j1 - 1; hi >= j0; hi -= 8) {    // eight maps in flight, composed in order
            double cq[8], dq[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int j = max(hi - k, j0);
                cq[k] = __hip_atomic_load(mapC + (size_t)j * B + bb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                dq[k] = __hip_atomic_load(mapD + (size_t)j * B + bb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (hi - k >= j0) {
                    Dw = dq[k] + cq[k] * Dw;
                    Cw = cq[k] * Cw;
                }
            }
        }
    }
    sxC[w][lane] = Cw;
    sxD[w][lane] = Dw;
    __syncthreads();
    double a = 0.0;                               // the advantage just after the chunk
    for (int j = NW - 1; j >= 0; --j) a = sxD[j][lane] + sxC[j][lane] * a;
    for (int j = NW - 1; j > w; --j) a = shD[j][lane] + shC[j][lane] * a;
#pragma unroll
    for (int u = U - 1; u >= 0; --u) {
        const int t = t0 + u;
        if (t < seg_end) {
            const double n = (alive >> u) & 1u ? 1.0 : 0.0;
            a = dl[u] + gl * n * a;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)a), rs_adv, voff_st, (uint32_t)t * row, 2);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)(a + (double)vv[u])), rs_ret, voff_st,
                                                  (uint32_t)t * row, 2);
        }
    }
}

constexpr int kMomBlock = 256;
constexpr int kMomBlocks = 1024;

// {sum, sum of squares} per block into work[2 * block]: 16-B loads (after a scalar
// head up to the first 16-B boundary), four in flight per thread, f64 accumulation,
// fixed thread -> element assignment (deterministic for a given n).
static __global__ __launch_bounds__(kMomBlock) void moments_partial_kernel(const float* x, int64_t n, double* work) {
    __shared__ double sh[2][kMomBlock / 64];
    const int64_t head = min<int64_t>(n, (int64_t)(((16u - ((uintptr_t)x & 15u)) & 15u) / 4u));
    const f4* x4 = reinterpret_cast<const f4*>(x + head);
    const int64_t n4 = (n - head) / 4;
    const int64_t tail0 = head + n4 * 4;
    const int64_t stride = (int64_t)gridDim.x * kMomBlock;
    double s0 = 0.0, s1 = 0.0, q0 = 0.0, q1 = 0.0;
    auto add4 = [&](f4 v) {
        const double a = v.x, b = v.y, c = v.z, d = v.w;
        s0 += a + b;
        s1 += c + d;
        q0 += a * a + b * b;
        q1 += c * c + d * d;
    };
    int64_t i = (int64_t)blockIdx.x * kMomBlock + threadIdx.x;
    for (; i + 3 * stride < n4; i += 4 * stride) {
        const f4 a = x4[i], b = x4[i + stride], c = x4[i + 2 * stride], d = x4[i + 3 * stride];
        add4(a);
        add4(b);
        add4(c);
        add4(d);
    }
    for (; i < n4; i += stride) add4(x4[i]);
    if (blockIdx.x == 0) {                        // head and tail elements
        const int64_t k = threadIdx.x;
        if (k < head) { const double v = x[k]; s0 += v; q0 += v * v; }
        if (tail0 + k < n) { const double v = x[tail0 + k]; s1 += v; q1 += v * v; }
    }
    double s = s0 + s1, q = q0 + q1;
    for (int o = 32; o > 0; o >>= 1) { s += __shfl_xor(s, o, 64); q += __shfl_xor(q, o, 64); }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sh[0][w] = s; sh[1][w] = q; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double ts = 0.0, tq = 0.0;
        for (int j = 0; j < kMomBlock / 64; ++j) { ts += sh[0][j]; tq += sh[1][j]; }
        work[blockIdx.x * 2 + 0] = ts;
        work[blockIdx.x * 2 + 1] = tq;
    }
}

// one workgroup folds the block partials in a fixed shape: thread t adds partials
// t, t + 256, ... in order, then a DPP/shuffle tree per wave and the 4 wave totals
// in order
static __global__ __launch_bounds__(kMomBlock) void moments_final_kernel(int nblocks, int64_t n, const double* work,
                                                                  double* out) {
    __shared__ double sh[2][kMomBlock / 64];
    double s = 0.0, q = 0.0;
    for (int i = threadIdx.x; i < nblocks; i += kMomBlock) { s += work[i * 2 + 0]; q += work[i * 2 + 1]; }
    for (int o = 32; o > 0; o >>= 1) { s += __shfl_xor(s, o, 64); q += __shfl_xor(q, o, 64); }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sh[0][w] = s; sh[1][w] = q; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double ts = 0.0, tq = 0.0;
        for (int j = 0; j < kMomBlock / 64; ++j) { ts += sh[0][j]; tq += sh[1][j]; }
        out[0] = (double)n;
        out[1] = ts;
        out[2] = tq;
    }
}

}  // namespace pmenv_dev
