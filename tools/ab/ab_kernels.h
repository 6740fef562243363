// ab_kernels.h — device kernels of the tools build only (tools/libpmenv_ab.so): the
// alternatives the product measured against and replaced. Moved out of
// pm-rl_amd/csrc/replay.h and trainer.h, whose device helpers they use.
#pragma once
#include "../../pm-rl_amd/csrc/env_step.h"
#include "../../pm-rl_amd/csrc/replay.h"
#include "../../pm-rl_amd/csrc/trainer.h"

namespace pmenv_dev {

// from replay.h: tools build: one thread per output float ([S, N, W, F], coalesced stores)
static __global__ void rollout_gather_kernel(const float* series, int T, int N, int F, int W, const int32_t* start,
                                      const float* weights, int T_rec, int B, int ring_mode, const int32_t* t_idx,
                                      const int32_t* env, int S, float* s) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per = (int64_t)N * W * F;
    if (i >= (int64_t)S * per) return;
    const int Fm = F - 1;
    const int j = (int)(i / per);
    int rem = (int)(i - (int64_t)j * per);
    const int n = rem / (W * F);
    rem -= n * W * F;
    const int p = rem / F, f = rem - p * F;
    const int b = env[j], t = t_idx[j];
    float v;
    if (f < Fm) {
        const int d = start[b] + t + p;
        v = (d >= 0 && d < T) ? series[((size_t)d * N + n) * Fm + f] : NAN;
    } else {
        const bool storage = ring_mode == PMENV_RING_STORAGE && t >= W - 1;
        const int c = storage ? (((p - t - 1) % W) + W) % W : p;
        const int r = t + c;                       // history row
        if (r < W - 1) v = 0.0f;
        else if (r == W - 1) v = n == 0 ? 1.0f : 0.0f;
        else v = weights[((size_t)(r - W) * B + b) * N + n];
    }
    s[i] = v;
}

// from replay.h: tools build: the thread-per-env walk (the fused kernel replaced it)
// one thread per env walks its column of the trajectory (coalesced across envs)
//   out[b] = {sharpe, sortino, max drawdown, average turnover, final value}
static __global__ void metrics_kernel(const double* returns, const double* values, int T, int B, double rf,
                               double periods, double* out) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    // qs.stats.sharpe / sortino: excess returns over the per-period rate
    // (1 + rf)^(1/periods) - 1, annualised by sqrt(periods)
    const double rfp = rf != 0.0 ? pow(1.0 + rf, 1.0 / periods) - 1.0 : 0.0;
    double mean = 0.0, m2 = 0.0, down = 0.0;
    for (int t = 0; t < T; ++t) {
        const double x = returns[(size_t)t * B + b] - rfp;
        const double d = x - mean;
        mean += d / (t + 1);
        m2 += d * (x - mean);
        down += x < 0.0 ? x * x : 0.0;
    }
    const double sd = T > 1 ? sqrt(m2 / (T - 1)) : NAN;
    const double sharpe = mean / sd * sqrt(periods);
    const double sortino = mean / sqrt(down / T) * sqrt(periods);
    // qs.stats.max_drawdown on the value curve: min_t (V_t / max_{s<=t} V_s - 1)
    double peak = -INFINITY, mdd = 0.0;
    for (int t = 0; t <= T; ++t) {
        const double v = values[(size_t)t * B + b];
        peak = fmax(peak, v);
        mdd = fmin(mdd, v / peak - 1.0);
    }
    out[(size_t)b * 5 + 0] = sharpe;
    out[(size_t)b * 5 + 1] = sortino;
    out[(size_t)b * 5 + 2] = mdd;
    out[(size_t)b * 5 + 4] = values[(size_t)T * B + b];
}

// from replay.h: tools build: the two-launch form of metrics_fused_kernel
static __global__ __launch_bounds__(256) void metrics_seg_kernel(const double* returns, const double* values, int T, int B,
                                                          double rf, double periods, double* out) {
    metrics_seg_body(returns, values, T, B, rf, periods, out, (int)blockIdx.x);
}

// from replay.h
static __global__ __launch_bounds__(256) void metrics_turnover_kernel(const float* weights, int T, int B, int N, int tpe,
                                                               int eb, double* out) {
    metrics_turnover_body(weights, T, B, N, tpe, eb, out, (int)blockIdx.x);
}

// from trainer.h
// ---------------------------------------------------------------- tools: the forward in one launch
// The row blocks write their partials as above; then every block takes a ticket from a
// device-scope counter (work[6B + 6], zeroed by the host before the launch), and the block
// that draws the last ticket folds all partials with final_fold — the same code and
// order as batch_reward_final_kernel, so both forms give the same bits. Release: the
// partials' writers fence before the block barrier and the ticket; acquire: the last
// block fences before reading the other blocks' partials (they live in other XCDs' L2).
// No block waits for another: blocks that are not last simply exit. Measured: the
// agent-scope fences (an L2 write-back per block) cost more than the second launch they
// save, at every shape and grid tried — kept here as that evidence.
__device__ __forceinline__ uint32_t* batch_reward_ticket(double* work, int B) {
    return reinterpret_cast<uint32_t*>(work + 6 * (size_t)B + 6);
}

// FENCE 0: every thread fences its own stores; 1: only thread 0 (after the barrier that
// orders the block's stores, all of which thread 0 made in the quad form)
template <int FENCE>
__device__ __forceinline__ bool drew_last_ticket(uint32_t* ticket) {
    __shared__ uint32_t last;
    if (FENCE == 0) __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) {
        if (FENCE == 1) __threadfence();
        last = atomicAdd(ticket, 1u) == gridDim.x - 1u ? 1u : 0u;
    }
    __syncthreads();
    if (!last) return false;
    __threadfence();
    return true;
}

// nblk row blocks over the grid (grid-stride: a block may produce several partials)
template <int EPL, int FENCE>
__global__ __launch_bounds__(kTrainBlock) void batch_reward_fwd_quad_kernel(const float* a, const float* v_prev,
                                                                            const float* p, int B, int N, int kind,
                                                                            int norm, double scale, double* work,
                                                                            float* reward_out, int nblk) {
    __shared__ double rec_w[4][kPartStride];
    for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
        rows_quad_partial<EPL>(a, v_prev, p, B, N, kind, norm, work, rec_w, blk, nblk);
        __syncthreads();                                          // rec_w is reused
    }
    if (drew_last_ticket<FENCE>(batch_reward_ticket(work, B)))
        final_fold(B, kind, norm, scale, work, reward_out, nblk);
}

// the ticketed one-launch forward without a fence or a per-call memset (PMENV_BR_TICKET): the
// record goes out with agent-scope atomic stores, thread 0 waits for them (vmcnt(0), no L2
// write-back) and draws a ticket with one fetch-add on a 64-bit word {epoch, count}; the block
// that draws count nblk - 1 folds the records through agent-scope atomic loads
// (final_fold<true>: the same bits) and re-arms the word as {epoch + 1, 0} for the next call
// (the host steps the epoch by one per call; the word starts as {first epoch, 0}). (A CAS loop
// that restarted the count on a stale epoch serialised 1,024 blocks: 2.7 ms at 65,536 rows.)
__device__ __forceinline__ bool drew_last_ticket_epoch(uint64_t* t, uint32_t epoch, uint32_t nblk) {
    __shared__ uint32_t last;
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_s_waitcnt(0 | (0x7 << 4) | (0xf << 8));          // vmcnt(0): the record is written
        const uint64_t old = __hip_atomic_fetch_add(t, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = (uint32_t)(old >> 32) == epoch && (uint32_t)old == nblk - 1u ? 1u : 0u;
    }
    __syncthreads();
    return last != 0;
}

template <int EPL>
__global__ __launch_bounds__(kTrainBlock) void batch_reward_fwd_ticket_kernel(const float* a, const float* v_prev,
                                                                              const float* p, int B, int N, int kind,
                                                                              int norm, double scale, double* work,
                                                                              float* reward_out, uint64_t* ticket,
                                                                              uint32_t epoch) {
    __shared__ double rec_w[4][kPartStride];
    const int nblk = (int)gridDim.x;
    rows_quad_partial<EPL, true>(a, v_prev, p, B, N, kind, norm, work, rec_w, (int)blockIdx.x, nblk);
    if (!drew_last_ticket_epoch(ticket, epoch, (uint32_t)nblk)) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    final_fold<true>(B, kind, norm, scale, work, reward_out, nblk);
    if (threadIdx.x == 0)
        __hip_atomic_store(ticket, (uint64_t)(epoch + 1u) << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int EPL, int FENCE>
__global__ __launch_bounds__(kTrainBlock) void batch_reward_fwd_rows_kernel(const float* a, const float* v_prev,
                                                                            const float* p, int B, int N, int kind,
                                                                            int norm, double scale, double* work,
                                                                            float* reward_out, int nblk) {
    __shared__ double sh[4][kRowsPerBlock];
    for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
        rows_wave_partial<EPL>(a, v_prev, p, B, N, kind, norm, work, sh, blk, nblk);
        __syncthreads();
    }
    if (drew_last_ticket<FENCE == 1 ? 0 : FENCE>(batch_reward_ticket(work, B)))   // several writer lanes
        final_fold(B, kind, norm, scale, work, reward_out, nblk);
}


// scalar_step_vec_kernel held to OCC waves per SIMD (PMENV_K1_OCC; the 8-assets-per-lane
// form takes 102 VGPRs, 4 waves per SIMD, unconstrained)
template <int L, int A, bool STR, int OCC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC))) void scalar_step_vec_occ_kernel(
    StepParams p) {
    const HaloRegs halo = halo_load(p);
    constexpr int EPW = 64 / L;
    const int lane = threadIdx.x & 63;
    const int w = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
    const int b = w * EPW + lane / L;
    const VecIn<A> in = vec_load<L, A, STR>(p, b, lane);
    const VecMid<A> m = vec_core<L, A, STR>(p, b, lane, in);
    vec_tail<L, A, STR>(p, b, lane, in, m);
    halo_store(p, halo);
}

// The forward in one launch without a ticket (PMENV_BR_RELAY): every row block writes its
// partial record with agent-scope atomic stores, then (after an order-only fence: a
// workgroup-scope release and s_waitcnt vmcnt(0), no L2 write-back) a 64-bit flag with the
// call's epoch; the LAST block, dispatched last, waits for every flag and folds the records
// through agent-scope atomic loads — final_fold's code and order, so the same bits.
template <int EPL>
__global__ __launch_bounds__(kTrainBlock) void batch_reward_fwd_relay_kernel(const float* a, const float* v_prev,
                                                                             const float* p, int B, int N, int kind,
                                                                             int norm, double scale, double* work,
                                                                             float* reward_out, uint64_t* flags,
                                                                             uint64_t epoch) {
    __shared__ double rec_w[4][kPartStride];
    const int nblk = (int)gridDim.x;
    rows_quad_partial<EPL, true>(a, v_prev, p, B, N, kind, norm, work, rec_w, (int)blockIdx.x, nblk);
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_s_waitcnt(0 | (0x7 << 4) | (0xf << 8));          // vmcnt(0): the record is written
        __hip_atomic_store(flags + blockIdx.x, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (blockIdx.x != (unsigned)nblk - 1) return;
    for (int k = threadIdx.x; k < nblk; k += blockDim.x)
        while (__hip_atomic_load(flags + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch)
            __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_s_waitcnt(0 | (0x7 << 4) | (0xf << 8));
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    __syncthreads();
    final_fold<true>(B, kind, norm, scale, work, reward_out, nblk);
}

// The in-place flat stream without the LDS image (PMENV_FLAT_DIRECT): each lane loads its
// own chunk and its shifted source (floats 4j+5 .. 4j+8) straight from memory with a
// dword-aligned 16-B load; the workgroup's last two chunks take theirs from the next chunk
// and the halo. One barrier (every load of the workgroup before any store), then compose
// and store. ABL: flat_side_load's SKIP bits (timing only).
template <int BLOCK, int V, int POL, int ABL>
__global__ __launch_bounds__(BLOCK) void advance_flat_direct_kernel(StepParams p, uint32_t qtot) {
    constexpr int kAux = POL == 1 ? 2 : 0;
    constexpr int CPW = BLOCK * V;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t c0 = blockIdx.x * CPW;
    const uint32_t nblk = min((uint32_t)CPW, qtot - c0);
    const auto rs = make_rsrc(p.obs + (size_t)c0 * 4, nblk * 16u);
    const uint32_t nh = blockIdx.x + 1 < gridDim.x ? min(2u, qtot - c0 - nblk) : 0u;
    const auto rh = make_rsrc(p.halo + (size_t)blockIdx.x * 8, nh * 16u);
    f4 own[V], shf[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const uint32_t j = (uint32_t)(64 * V * wave + 64 * v + lane);
        own[v] = buf_load4<kAux>(rs, j * 16u);
        // floats 4j+5 .. 4j+8 lie inside the workgroup's range for j + 3 <= nblk
        shf[v] = buf_load4<kAux>(rs, j + 3u <= nblk ? j * 16u + 20u : 0xFFFFFFF0u);
    }
    // the last two chunks' sources: chunk j+1 (in range) or the halo
    const uint32_t je = nblk >= 2 ? nblk - 2u : 0u;
    const bool edge = tid < 2 && nblk >= 2;
    f4 ea = f4{0.f, 0.f, 0.f, 0.f}, eb = f4{0.f, 0.f, 0.f, 0.f};
    if (edge) {
        const uint32_t j = je + (uint32_t)tid;                        // nblk - 2, nblk - 1
        ea = j + 1u < nblk ? buf_load4<0>(rs, (j + 1u) * 16u) : buf_load4<0>(rh, 0u);
        eb = j + 1u < nblk ? buf_load4<0>(rh, 0u) : buf_load4<0>(rh, 16u);
    }
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t qw = __builtin_amdgcn_readfirstlane(c0 + (uint32_t)(64 * V * wave));
    WaveSide ws;
    ws.ok = false;
    ws = wave_side_load(p, qw, 64u * V, qtot);
    FlatSide sd[V];
#pragma unroll
    for (int v = 0; v < V; ++v) sd[v] = flat_side_from_wave<ABL & 15>(p, ws, min(qw + 64u * v + lane, qtot - 1u));
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    __shared__ f4 sh_edge[2][2];
    if (edge) { sh_edge[tid][0] = ea; sh_edge[tid][1] = eb; }
    __syncthreads();
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const uint32_t j = (uint32_t)(64 * V * wave + 64 * v + lane);
        float sh[4] = {shf[v].x, shf[v].y, shf[v].z, shf[v].w};
        if (j + 3u > nblk && j < nblk) {
            const int k = (int)(j - je);
            const f4 a = sh_edge[k][0], b = sh_edge[k][1];
            sh[0] = a.y; sh[1] = a.z; sh[2] = a.w; sh[3] = b.x;
        }
        const float un[4] = {own[v].x, own[v].y, own[v].z, own[v].w};
        buf_store4<kAux>(rs, j * 16u, flat_compose(p, sd[v], un, sh));
    }
}

// step_flat_kernel (csrc/step_flat.h) with the alternatives it was measured against:
// per-direction cache policies (POL 3 nt loads only, 4 nt stores only, 5 sc0 nt, 6 sc1 nt,
// 7 nt loads + sc1 nt stores) and XCD-contiguous tile ranges (XCD x takes workgroups
// x, x + 8, ... as one contiguous range of tiles)
template <int BLOCK, int V, int POL, bool OUT, bool XCD>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_num_sgpr(80))) void step_flat_ab_kernel(StepParams p,
                                                                                                 uint32_t qtot) {
    constexpr int CPW = BLOCK * V, WAVES = BLOCK / 64;
    constexpr int kAuxL = (POL == 1 || POL == 3 || POL == 7) ? 2 : POL == 5 ? 3 : POL == 6 ? 18 : 0;
    constexpr int kAuxS = (POL == 1 || POL == 4) ? 2 : POL == 5 ? 3 : (POL == 6 || POL == 7) ? 18 : 0;
    __shared__ f4 sh4[CPW + 2];
    __shared__ f4 sh_bar[WAVES][64];
    __shared__ float sh_wp[WAVES][64];
    __shared__ int32_t sh_k[WAVES];
    uint32_t tile = blockIdx.x;
    if (XCD) {
        const uint32_t G = gridDim.x, q = G >> 3, r = G & 7, x = tile & 7, i = tile >> 3;
        tile = x < r ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
    }
    flat_seq_enter<OUT>(p);
    FlatTile<V> t;
    flat1_load<BLOCK, V, kAuxL, OUT>(p, qtot, tile, t);
    flat1_process<BLOCK, V, kAuxS, OUT>(p, qtot, tile, t, sh4, sh_bar, sh_wp, sh_k);
}

// Round 3's horizon split (PMENV_GAE=split; the product runs gae_lookback_kernel in one
// pass since round 4). The tiled scan with the horizon also split across workgroups, for rollouts with
// too few envs to fill the chip (B / 64 workgroups): grid (B / 64, chunks), chunk c
// covering days [c*Lc, (c+1)*Lc), Lc a multiple of the NW*U segment.
//   MAPS  pass: each workgroup reduces its chunk to the per-env affine map
//               A(chunk start) = D + C * A(after the chunk) -> maps[2][chunks][B] (f64)
//   apply pass: each workgroup composes the maps of every later chunk into its
//               carry-in, then runs the tiled scan over its chunk writing adv / ret.
// The inputs are read twice (26 B per element instead of 17) in exchange for
// chunks x the workgroups; selected by the host only where B / 64 leaves the CUs idle.
// SP: cache-policy bits of the apply pass's adv / ret stores
template <int NW, int U, bool MAPS, int SP = 0>
__global__ __launch_bounds__(64 * NW) void gae_chunk_kernel(const float* r, const float* v, const uint8_t* dones,
                                                           float* adv, float* ret, int T, int B, float gamma,
                                                           float lam, int Lc, double* maps) {
    __shared__ double shC[NW][64], shD[NW][64];
    constexpr int S = NW * U;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int b = blockIdx.x * 64 + lane;
    const int chunk = blockIdx.y, nchunks = gridDim.y;
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
    const int c0 = chunk * Lc, c1 = min(T, c0 + Lc);
    double* mapC = maps;
    double* mapD = maps + (size_t)nchunks * B;
    const int bb = ok ? b : B - 1;
    double carry = 0.0, Cc = 1.0;                 // apply: advantage after the segment; maps: A = carry + Cc x
    if (!MAPS)
        for (int j = nchunks - 1; j > chunk; --j)
            carry = mapD[(size_t)j * B + bb] + mapC[(size_t)j * B + bb] * carry;
    for (int seg_end = c1; seg_end > c0; seg_end -= S) {
        const int seg_start = max(seg_end - S, c0);
        const int t0 = seg_start + w * U;
        float vv[U + 1], rr[U];
        uint32_t alive = 0;
#pragma unroll
        for (int u = 0; u <= U; ++u) {
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
        double dl[U];
        double C = 1.0, D = 0.0;
#pragma unroll
        for (int u = U - 1; u >= 0; --u) {
            const double n = (alive >> u) & 1u ? 1.0 : 0.0;
            dl[u] = (double)rr[u] + g * n * (double)vv[u + 1] - (double)vv[u];
            if (t0 + u < seg_end) {
                D = dl[u] + gl * n * D;
                C = gl * n * C;
            }
        }
        shC[w][lane] = C;
        shD[w][lane] = D;
        __syncthreads();
        if (!MAPS) {
            double a = carry;
            for (int j = NW - 1; j > w; --j) a = shD[j][lane] + shC[j][lane] * a;
#pragma unroll
            for (int u = U - 1; u >= 0; --u) {
                const int t = t0 + u;
                if (t < seg_end) {
                    const double n = (alive >> u) & 1u ? 1.0 : 0.0;
                    a = dl[u] + gl * n * a;
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)a), rs_adv, voff_st,
                                                          (uint32_t)t * row, SP);
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)(a + (double)vv[u])), rs_ret,
                                                          voff_st, (uint32_t)t * row, SP);
                }
            }
        }
        for (int j = NW - 1; j >= 0; --j) {
            carry = shD[j][lane] + shC[j][lane] * carry;
            if (MAPS) Cc = shC[j][lane] * Cc;
        }
        __syncthreads();
    }
    if (MAPS && w == 0 && ok) {
        mapC[(size_t)chunk * B + b] = Cc;
        mapD[(size_t)chunk * B + b] = carry;
    }
}


// the look-back pieces (tools copies of rollout.h gae_lookback_kernel's steps) and the paired form
template <int NW, int U>
struct LbChunk {
    float vv[U + 1], rr[U];
    uint32_t alive;
};

template <int NW, int U>
__device__ __forceinline__ void lb_load(const float* r, const float* v, const uint8_t* dones, int T, int B, int c,
                                        int w, uint32_t voff, LbChunk<NW, U>& k) {
    constexpr int S = NW * U;
    const uint32_t row = (uint32_t)B * 4u;
    const auto rs_r = make_rsrc(r, (uint32_t)T * row);
    const auto rs_v = make_rsrc(v, (uint32_t)(T + 1) * row);
    const auto rs_d = make_rsrc(dones ? (const void*)dones : (const void*)r, dones ? (uint32_t)T * (uint32_t)B : 0u);
    const int seg_start = c * S, seg_end = min(T, seg_start + S);
    const int t0 = seg_start + w * U;
#pragma unroll
    for (int u = 0; u <= U; ++u) {
        const uint32_t t = (uint32_t)min(t0 + u, seg_end);
        k.vv[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_v, voff, t * row, 0));
    }
    k.alive = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t t = (uint32_t)min(t0 + u, seg_end - 1);
        k.rr[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_r, voff, t * row, 0));
        const uint32_t dn = __builtin_amdgcn_raw_buffer_load_b8(rs_d, voff >> 2, t * (uint32_t)B, 0);
        k.alive |= (dn ? 0u : 1u) << u;
    }
}

// reduce the chunk (dl kept), publish its map and flag; returns nothing, fills dl and LDS
template <int NW, int U>
__device__ __forceinline__ void lb_reduce_publish(const LbChunk<NW, U>& k, double (&dl)[U], int T, int B, int c, int w,
                                                  int lane, int b, bool ok, int nEB, int eb, double g, double gl,
                                                  double (*shC)[64], double (*shD)[64], double* maps, int nC,
                                                  uint64_t* flags, uint64_t epoch) {
    constexpr int S = NW * U;
    const int seg_start = c * S, seg_end = min(T, seg_start + S);
    const int t0 = seg_start + w * U;
    double C = 1.0, D = 0.0;
#pragma unroll
    for (int u = U - 1; u >= 0; --u) {
        const double n = (k.alive >> u) & 1u ? 1.0 : 0.0;
        dl[u] = (double)k.rr[u] + g * n * (double)k.vv[u + 1] - (double)k.vv[u];
        if (t0 + u < seg_end) {
            D = dl[u] + gl * n * D;
            C = gl * n * C;
        }
    }
    shC[w][lane] = C;
    shD[w][lane] = D;
    __syncthreads();
    double* mapC = maps;
    double* mapD = maps + (size_t)nC * B;
    if (w == 0) {
        double Ca = 1.0, Da = 0.0;
        for (int j = NW - 1; j >= 0; --j) {
            Da = shD[j][lane] + shC[j][lane] * Da;
            Ca = shC[j][lane] * Ca;
        }
        if (ok) {
            __hip_atomic_store(mapC + (size_t)c * B + b, Ca, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(mapD + (size_t)c * B + b, Da, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_s_waitcnt(0 | (0x7 << 4) | (0xf << 8));
        if (lane == 0) __hip_atomic_store(flags + (size_t)c * nEB + eb, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// the later chunks' maps composed into the advantage just after this wave's segment of chunk c
template <int NW, int U>
__device__ __forceinline__ double lb_lookback(int B, int c, int w, int lane, int b, bool ok, int nEB, int eb,
                                              double (*shC)[64], double (*shD)[64], double (*sxC)[64],
                                              double (*sxD)[64], const double* maps, int nC, const uint64_t* flags,
                                              uint64_t epoch) {
    const double* mapC = maps;
    const double* mapD = maps + (size_t)nC * B;
    const int nl = nC - 1 - c, m = (nl + NW - 1) / NW;
    const int j0 = c + 1 + w * m, j1 = min(nC, j0 + m);
    double Cw = 1.0, Dw = 0.0;
    if (j0 < j1) {
        for (int base = j0; base < j1; base += 64) {
            const int j = base + lane;
            bool ready = j >= j1 || __hip_atomic_load(const_cast<uint64_t*>(flags) + (size_t)j * nEB + eb, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT) == epoch;
            while (!__all(ready)) {
                __builtin_amdgcn_s_sleep(1);
                if (!ready)
                    ready = __hip_atomic_load(const_cast<uint64_t*>(flags) + (size_t)j * nEB + eb, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT) == epoch;
            }
        }
        __builtin_amdgcn_s_waitcnt(0 | (0x7 << 4) | (0xf << 8));
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const size_t bb = (size_t)(ok ? b : B - 1);
        for (int hi = j1 - 1; hi >= j0; hi -= 8) {
            double cq[8], dq[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int j = max(hi - q, j0);
                cq[q] = __hip_atomic_load(const_cast<double*>(mapC) + (size_t)j * B + bb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                dq[q] = __hip_atomic_load(const_cast<double*>(mapD) + (size_t)j * B + bb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                if (hi - q >= j0) {
                    Dw = dq[q] + cq[q] * Dw;
                    Cw = cq[q] * Cw;
                }
            }
        }
    }
    sxC[w][lane] = Cw;
    sxD[w][lane] = Dw;
    __syncthreads();
    double a = 0.0;
    for (int j = NW - 1; j >= 0; --j) a = sxD[j][lane] + sxC[j][lane] * a;
    for (int j = NW - 1; j > w; --j) a = shD[j][lane] + shC[j][lane] * a;
    return a;
}

template <int NW, int U>
__device__ __forceinline__ void lb_walk(const LbChunk<NW, U>& k, const double (&dl)[U], double a, float* adv, float* ret,
                                        int T, int B, int c, int w, bool ok, uint32_t voff, double gl) {
    constexpr int S = NW * U;
    const uint32_t row = (uint32_t)B * 4u;
    const auto rs_adv = make_rsrc(adv, (uint32_t)T * row);
    const auto rs_ret = make_rsrc(ret, (uint32_t)T * row);
    const uint32_t voff_st = ok ? voff : 0x80000000u;
    const int seg_start = c * S, seg_end = min(T, seg_start + S);
    const int t0 = seg_start + w * U;
#pragma unroll
    for (int u = U - 1; u >= 0; --u) {
        const int t = t0 + u;
        if (t < seg_end) {
            const double n = (k.alive >> u) & 1u ? 1.0 : 0.0;
            a = dl[u] + gl * n * a;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)a), rs_adv, voff_st, (uint32_t)t * row, 2);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((float)(a + (double)k.vv[u])), rs_ret, voff_st,
                                                  (uint32_t)t * row, 2);
        }
    }
}

// gae_lookback_kernel with TWO adjacent chunks per workgroup (PMENV_GAE=lb2): pair p holds
// chunk A = 2p + 1 and B = 2p; B's loads are issued after A's look-back, so they are in
// flight while A's adv / ret are stored — the read and write phases of the chip overlap
// instead of all workgroups loading, then all storing. The same look-back and walk as the
// product kernel (the same bits). Waits: A needs chunks > 2p + 1, B needs A and chunks
// > 2p + 1 — all published by this workgroup or by pairs dispatched before it (later pairs
// first), so every wait ends whatever the residency.
template <int NW, int U>
__global__ __launch_bounds__(64 * NW) void gae_lookback2_kernel(const float* r, const float* v, const uint8_t* dones,
                                                               float* adv, float* ret, int T, int B, float gamma,
                                                               float lam, int nC, double* maps, uint64_t* flags,
                                                               uint64_t epoch) {
    __shared__ double shC[NW][64], shD[NW][64];
    __shared__ double sxC[NW][64], sxD[NW][64];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nEB = (B + 63) / 64;
    const int nP = (nC + 1) / 2;                   // pairs: B chunk 2p, A chunk 2p + 1 (if < nC)
    const int pr = nP - 1 - (int)(blockIdx.x / (unsigned)nEB);
    const int eb = (int)(blockIdx.x % (unsigned)nEB);
    const int b = eb * 64 + lane;
    const bool ok = b < B;
    const uint32_t voff = (uint32_t)(ok ? b : B - 1) * 4u;
    const double g = (double)gamma, gl = (double)gamma * (double)lam;
    const int cA = 2 * pr + 1, cB = 2 * pr;
    LbChunk<NW, U> kB;
    double dl[U];
    if (cA < nC) {
        LbChunk<NW, U> kA;
        lb_load<NW, U>(r, v, dones, T, B, cA, w, voff, kA);
        lb_reduce_publish<NW, U>(kA, dl, T, B, cA, w, lane, b, ok, nEB, eb, g, gl, shC, shD, maps, nC, flags, epoch);
        const double a = lb_lookback<NW, U>(B, cA, w, lane, b, ok, nEB, eb, shC, shD, sxC, sxD, maps, nC, flags, epoch);
        // B's loads go out after the last wait of A (a wait on anything issued later would wait
        // for them too: vmcnt counts in order), so they are in flight while A's stores drain
        lb_load<NW, U>(r, v, dones, T, B, cB, w, voff, kB);
        lb_walk<NW, U>(kA, dl, a, adv, ret, T, B, cA, w, ok, voff, gl);
        __syncthreads();                            // shC / shD / sxC / sxD are reused by B
    } else {
        lb_load<NW, U>(r, v, dones, T, B, cB, w, voff, kB);
    }
    lb_reduce_publish<NW, U>(kB, dl, T, B, cB, w, lane, b, ok, nEB, eb, g, gl, shC, shD, maps, nC, flags, epoch);
    const double a = lb_lookback<NW, U>(B, cB, w, lane, b, ok, nEB, eb, shC, shD, sxC, sxD, maps, nC, flags, epoch);
    lb_walk<NW, U>(kB, dl, a, adv, ret, T, B, cB, w, ok, voff, gl);
}


// (round 5's env-aligned relay tiles, step_relay_env_kernel — measured 3-6 % slower at 2,048 -
// 6,144 x 30 and 20 % at N = 8 / 16, profiles/ab_r05/relay_env_r05g.err — are in the git history)

// The register step (env_step.h step_small_kernel, REG form) with wall-clock stamps and
// timing-only ablations (PMENV_SMALL_ABL): where config 1's 1 x 5 x 50 x 5 step spends its
// time. Thread 0 reads s_memrealtime (100 MHz) at each phase and stores the stamps with one
// vector store per stamp into g_small_stamps[slot][0..7]; the last wave stamps its entry in
// [7]. ABL: 2 no scalar step (w' = 0, no tail), 4 no window loads / stores, 8 return at once,
// 16 no tail. The stamps are read back by pmenv_tools_small_stamps (pmenv_ab.hip).
__device__ uint64_t g_small_stamps[1024 * 8];

__device__ __forceinline__ uint64_t stamp_now() {
    uint64_t t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
    return t;
}

template <int BLOCK, int E, int ABL>
__global__ __launch_bounds__(BLOCK) void small_stamp_kernel(StepParams p, uint32_t slot_id) {
    static_assert(E <= 8, "the stamped copy keeps the product's small-E form only");
    __shared__ float sh_wp[64];
    uint64_t ts[7] = {0, 0, 0, 0, 0, 0, 0};
    const int tid = threadIdx.x;
    if (tid == 0) ts[0] = stamp_now();
    if (tid == BLOCK - 64) {
        const uint64_t t = stamp_now();
        g_small_stamps[(slot_id & 1023) * 8 + 7] = t;
    }
    if (ABL & 8) {
        if (tid == 0) g_small_stamps[(slot_id & 1023) * 8] = ts[0];
        return;
    }
    const int b = blockIdx.x;
    const int N = p.N, W = p.W, F = p.F, Fm = F - 1;
    const uint32_t WF = (uint32_t)(W * F), NWF = (uint32_t)N * WF;
    constexpr uint32_t kOut = 0x80000000u;
    const auto rs_in = make_rsrc(p.obs + (size_t)b * NWF, NWF * 4u);
    const auto rs_out = make_rsrc(p.obs_out + (size_t)b * NWF, NWF * 4u);
    const float* barg = env_bar(p, b);
    const auto rs_bar = make_rsrc(barg ? barg : p.obs, barg ? (uint32_t)(N * Fm) * 4u : 0u);
    const float nanv = __int_as_float(0x7fc00000);
    uint32_t z = 0u;
    asm volatile("" : "+v"(z));
    const ScalarIn sin = scalar_load<64, true>(p, b, tid, z);
    const int32_t k0 = sin.k;
    uint32_t xr[E], xt[E], xf[E];
    float src[E], cur[E];
    if (!(ABL & 4)) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const uint32_t j = (uint32_t)tid + (uint32_t)(BLOCK * e);
            const uint32_t row = fdiv(j, p.div_wf);
            const uint32_t kk = j - row * WF;
            const uint32_t t = fdiv(kk, p.div_f);
            const uint32_t f = kk - t * (uint32_t)F;
            xr[e] = row;
            xt[e] = t;
            xf[e] = f;
            const bool mkt = j < NWF && (int)f < Fm, last = (int)t == W - 1;
            const float sh = buf_load1(rs_in, mkt && !last ? (j + (uint32_t)F) * 4u : kOut);
            const float bv = buf_load1(rs_bar, mkt && last ? (row * (uint32_t)Fm + f) * 4u : kOut);
            src[e] = last ? (barg ? bv : nanv) : sh;
        }
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const uint32_t j = (uint32_t)tid + (uint32_t)(BLOCK * e);
            const bool wch = j < NWF && (int)xf[e] == Fm;
            const float ws = buf_load1(rs_in, wch && (int)xt[e] < W - 1 ? (j + (uint32_t)F) * 4u : kOut);
            cur[e] = buf_load1(rs_in, wch ? j * 4u : kOut);
            src[e] = wch ? ws : src[e];
        }
    }
    const bool shift_w = p.ring_mode == PMENV_RING_CHRONO || k0 < W - 1;
    ScalarMid mid{};
    if (tid < 64) {
        if (!(ABL & 2)) {
            mid = scalar_core<64>(p, b, tid, sin);
        } else {
            mid.wp = sin.a;
            mid.k = sin.k;
        }
        sh_wp[tid] = mid.wp;
    }
    if (tid == 0) {
        asm volatile("" ::"v"(mid.wp));
        ts[1] = stamp_now();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tid == 0) ts[2] = stamp_now();
    __syncthreads();
    if (tid == 0) ts[3] = stamp_now();
    const int slot = ring_slot(k0, W);
    if (!(ABL & 4)) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const uint32_t j = (uint32_t)tid + (uint32_t)(BLOCK * e);
            const uint32_t row = xr[e], t = xt[e], f = xf[e];
            const float v = src[e];
            const float wp = sh_wp[min(row, (uint32_t)N - 1u)];
            const float wv = pick(shift_w, pick((int)t == W - 1, wp, v), pick((int)t == slot, wp, cur[e]));
            const float o = pick((int)f == Fm && j < NWF, wv, v);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o), rs_out, j < NWF ? j * 4u : kOut, 0, 0);
        }
    }
    if (tid == 0) ts[4] = stamp_now();
    if (!(ABL & 18) && tid < 64) scalar_tail<64>(p, b, tid, sin, mid);
    if (tid == 0) ts[5] = stamp_now();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tid == 0) {
        ts[6] = stamp_now();
        uint64_t* d = g_small_stamps + (slot_id & 1023) * 8;
#pragma unroll
        for (int i = 0; i < 7; ++i) d[i] = ts[i];
    }
}
}  // namespace pmenv_dev
