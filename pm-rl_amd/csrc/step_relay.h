// step_relay.h — the advance step in ONE launch whose scalar steps run once per env, in
// dedicated workgroups, and reach the window-stream tiles through relay words.
//
// The two-launch step (scalar-step kernel, then the flat window stream) pays a kernel
// boundary: the stream cannot start before the last env's scalar step has ended. The flat
// one-launch step (step_flat.h) removes the boundary but runs the scalar step inside every
// tile an env straddles, which lengthens every tile's life. Here one launch carries both
// roles: blocks [0, S) are the scalar blocks, blocks [S, S + T) the tiles (dispatch order):
//   * a scalar block runs the two-launch path's own scalar step (the same code, so the same
//     bits) for its envs and relays each lane's w' as a 64-bit word {epoch, w'} — an
//     agent-scope relaxed atomic store, coherent across the XCDs' L2s without an L2
//     write-back fence — then writes the state (scalar_tail) and the counter's next-step
//     copy (kp_out, read by the next launch);
//   * a tile streams its 16-B chunks of the flat window exactly as the in-place stream does
//     (the two-level compose of flat_wg_body_patch), staging its rows' bar, w' and counter
//     from the relay words and its rows' counter from the parity copy kp_in; a word whose
//     epoch is not this step's is not yet written, and the lane re-reads it (s_sleep between
//     tries). Each word validates itself, so no flag and no ordering between words is needed
//     (the pattern rocPRIM's look-back scan state uses on gfx942 / gfx950: atomic loads /
//     stores that bypass the non-coherent L2).
// Forward progress does not rest on dispatch order. A tile polls its rows' words at most `spin`
// times; if one is still missing it DEFERS: it stores nothing, appends its index to the step's
// deferral list ({epoch, count} word + entries), re-checks its words once and exits. A deferred
// tile is run exactly once — under its own claim word {epoch} — by itself on that re-check if every
// word has arrived by then, or else by a scalar block: after its units, every scalar block reads
// the list and runs each listed tile whose words have all arrived. No workgroup ever waits without
// bound, so every scalar block is eventually dispatched, and a listed tile is never missed: the
// tile's append and re-check and each scalar block's word stores and list read are ordered by
// completion waits (a store-buffering pair), so either the re-check sees the last of its words or
// that word's scalar block sees the entry. The same tile code runs in either case (the same bits).
// In the hardware's dispatch order (blockIdx order, round-robin over the XCDs) the scalar blocks
// come first and no tile defers; the normal path's cost is the bounded poll, one LDS vote, and
// one list read per scalar block. (The first fallback built — tiles running the missing
// scalar-step units themselves under per-unit claims — put the scalar step into the tile's path:
// 106 SGPRs, 7 waves per SIMD, +4 % at 4,096 x 30 and +10 % at 8,192 x 30; profiles/r06/. An
// ordered ticket, one agent-scope fetch-add per workgroup on one counter — rocPRIM's ordered block
// id — ran 4.7x slower: the ~15,900 same-address atomics of a 4,096 x 30 step serialise at ~10 ns
// each, 194.9 against 41.0 us; profiles/ab_r05/ticket_r05b.*.)
//
// Epoch and parity: eager steps take them from the host (launch arguments). A handle seen under
// stream capture sequences its relay steps on the device instead (graph replays must not
// replay frozen arguments): relay_prime_kernel, launched before every such step, reads the
// device words {D, E, V, HOBS}, re-primes the copies of parity D when V / HOBS say so, and
// publishes {C = D, EC = E + 1} for the step, which reads only C and EC and writes D = 1 - C,
// E = EC, V = 1 and HOBS for the next one (no launch reads a word it or a concurrent block
// writes).
//
// In place, the two chunks past a tile belong to the next tile, which may already have
// stored them: they come from a halo the next tile wrote in the previous step (its first
// two output chunks, parity-buffered like step_flat_kernel's), primed from the window by
// the host when anything else wrote it. Double-buffered tiles read them from obs.
//
// Reference semantics as the two-launch path (env_step.h scalar_core / scalar_tail,
// scalar_vec.h vec_*, compose2): env/sim/trading_env.py:54-105, weight_buffer.py:13-44,
// data/instrument.py:79, :339-356.
#pragma once
#include "env_step.h"
#include "scalar_vec.h"

namespace pmenv_dev {

struct RelayParams {
    uint32_t scal;           // scalar blocks (the first `scal` blocks of the grid)
    uint32_t epoch;          // eager: this step's tag (never 0: the words start zeroed)
    uint64_t* w;             // [B * N] {epoch, w' bits}
    uint64_t* list;          // the deferral list: [0] {epoch, count}, [1 + i] {epoch, tile}
    uint32_t* done;          // [tiles] the epoch of the step in which a deferred tile last ran
    uint32_t spin;           // tools build (ANY): polls of a missing word before a tile defers
    uint32_t rot;            // tools build (ANY): blockIdx rotated by `rot` (tiles first: no order)
    uint32_t grid;           // the launch's workgroups
    // eager: this step's copies (parity p: the counter before the step and, in place, its input
    // chunks past each tile; parity 1 - p: the same for the next step, written by this one)
    const int32_t* kp_in;
    int32_t* kp_out;
    const float* halo_in;    // [tiles - 1][2] float4
    float* halo_out;
    // device-sequenced (step_relay_kernel<..., SEQ = true>): the parity-0 bases, parity 1 at
    // +B / +halo_stride, and the words {D, E, V, C, EC, pad, HOBS lo, HOBS hi}
    uint32_t* seq;
    int32_t* kp;
    float* halo;
    uint32_t B;
    uint32_t halo_stride;
    const float* obs;        // the window (HOBS of a device-sequenced in-place step)
    uint32_t par;            // eager: this step's parity (relay_prime_kernel's copies)
};
enum { kSeqD = 0, kSeqE = 1, kSeqV = 2, kSeqC = 3, kSeqEC = 4, kSeqHobs = 6 };

// this step's epoch and parity copies: eager from the launch arguments, device-sequenced from the
// words relay_prime_kernel published (C, EC: nothing writes them during the launch)
struct RelayCtx {
    uint32_t epoch;
    const int32_t* kp_in;
    int32_t* kp_out;
    const float* halo_in;
    float* halo_out;
};
template <bool SEQ>
__device__ __forceinline__ RelayCtx relay_ctx(const RelayParams& r) {
    RelayCtx c{r.epoch, r.kp_in, r.kp_out, r.halo_in, r.halo_out};
    if constexpr (SEQ) {
        const uint32_t par = __builtin_amdgcn_readfirstlane(r.seq[kSeqC]);
        c.epoch = __builtin_amdgcn_readfirstlane(r.seq[kSeqEC]);
        c.kp_in = r.kp + (size_t)par * r.B;
        c.kp_out = r.kp + (size_t)(par ^ 1u) * r.B;
        c.halo_in = r.halo + (size_t)par * r.halo_stride;
        c.halo_out = r.halo + (size_t)(par ^ 1u) * r.halo_stride;
    }
    return c;
}

// step_relay_kernel's arguments read afresh from the kernel-argument segment, through a pointer
// the compiler cannot see through: the deferral paths (relay_defer, relay_adopt) run a second
// copy of the tile's code after the first attempt or the scalar step, and the compiler hoists
// every argument load to the kernel's entry — values held from there through the first code
// would push the kernel past the SGPR budget of its occupancy (81 SGPRs without the deferral
// paths, 106 with them on the hoisted arguments: 7 waves per SIMD instead of 8)
struct KArgs {
    StepParams p;
    RelayParams r;
    uint32_t qtot;
};
__device__ __forceinline__ KArgs kargs() {
    typedef __attribute__((address_space(4))) const uint32_t KWord;
    KWord* ka = (KWord*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ka));
    uint32_t w[sizeof(KArgs) / 4];
#pragma unroll
    for (size_t i = 0; i < sizeof(KArgs) / 4; ++i) w[i] = ka[i];
    KArgs k;
    __builtin_memcpy(&k, w, sizeof(KArgs));                   // not a punned store: well-defined
    return k;
}

// Tools build only (step_relay_kernel<..., ANY = 2>, PMENV_RELAY_STAMPS: the product's order and
// polls): thread 0 of each workgroup reads s_memrealtime (100 MHz) at the phases of its role — each
// read issued once `dep` (a value of the phase's last load) has arrived, DRAIN: once the wave's
// stores have completed — holds the stamps in scalar registers and stores them at its end into
// g_relay_stamps[epoch % kStampSlots][bid][k] (tools/relay_stamps.py); a null pointer stores none.
// The product's instantiations (ANY = 0) hold no stamp code.
constexpr uint32_t kStampSlots = 16, kStampMaxWg = 40960;
static __device__ uint64_t* g_relay_stamps;
template <bool ST, bool DRAIN = false>
__device__ __forceinline__ uint64_t relay_clock(uint32_t dep) {
    uint64_t t = 0;
    if constexpr (ST) {
        if constexpr (DRAIN)
            asm volatile("s_waitcnt vmcnt(0)\n\ts_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : "v"(dep) : "memory");
        else
            asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : "v"(dep) : "memory");
    }
    return t;
}
template <bool ST, int K>
__device__ __forceinline__ void relay_stamps_put(uint32_t bid, uint32_t epoch, const uint64_t (&ts)[K]) {
    if constexpr (ST) {
        uint64_t* s = g_relay_stamps;
        if (s && threadIdx.x == 0 && bid < kStampMaxWg) {
#pragma unroll
            for (int k = 0; k < K; ++k) s[((size_t)(epoch % kStampSlots) * kStampMaxWg + bid) * 8 + k] = ts[k];
        }
    }
}

__device__ __forceinline__ void relay_put(uint64_t* w, uint32_t epoch, uint32_t bits) {
    __hip_atomic_store(w, ((uint64_t)epoch << 32) | bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t relay_get(const uint64_t* w) {
    return __hip_atomic_load(const_cast<uint64_t*>(w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A scalar wave's read of the deferral list's count, once its relay words have completed (the
// store-buffering pair with relay_defer: step_relay.h's head)
__device__ __forceinline__ uint32_t relay_list_read(const RelayParams& r, uint32_t epoch) {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    const uint64_t lw = relay_get(r.list);
    return (uint32_t)(lw >> 32) == epoch ? (uint32_t)lw : 0u;
}

// The scalar role: the two-launch path's scalar step for envs [s * EPB, (s + 1) * EPB).
// KA = 0: the register form, KL lanes per env (scalar_step_reg_kernel); KA > 0: the packed
// form, KL lanes x KA strided assets (scalar_step_vec_kernel<KL, KA, true>). Only w' goes
// through the relay words; the counter of the next step goes to kp_out (read after this
// launch has ended).
template <int BLOCK, int KL, int KA, bool ST = false>
__device__ __forceinline__ uint32_t relay_scalar(const StepParams& p, const RelayParams& r, int s, uint32_t epoch,
                                                 int32_t* kp_out, uint64_t t_entry = 0) {
    uint64_t ts[3] = {t_entry, 0, 0};
    constexpr int EPW = 64 / KL, EPB = (BLOCK / 64) * EPW;
    const int lane = threadIdx.x & 63;
    const int b = s * EPB + (int)(threadIdx.x >> 6) * EPW + lane / KL;
    const int j = lane % KL;
    const int N = p.N;
    const bool env_ok = b < p.B;
    // after the words: the wave's list read (relay_list_read), its round trip under the tail's stores
    uint32_t listed;
    if constexpr (KA == 0) {
        const ScalarIn in = scalar_load<KL>(p, b, lane);
        const ScalarMid m = scalar_core<KL>(p, b, lane, in);
        if (env_ok && j < N) relay_put(r.w + (size_t)b * N + j, epoch, __float_as_uint(m.wp));
        if (env_ok && j == 0) kp_out[b] = m.k + 1;
        listed = relay_list_read(r, epoch);
        ts[1] = relay_clock<ST>(listed);                            // its words published
        scalar_tail<KL>(p, b, lane, in, m);
    } else {
        const VecIn<KA> in = vec_load<KL, KA, true>(p, b, lane);
        const VecMid<KA> m = vec_core<KL, KA, true>(p, b, lane, in);
#pragma unroll
        for (int e = 0; e < KA; ++e) {
            const int n = j + e * KL;
            if (env_ok && n < N) relay_put(r.w + (size_t)b * N + n, epoch, __float_as_uint(m.wp[e]));
        }
        if (env_ok && j == 0) kp_out[b] = in.k + 1;
        listed = relay_list_read(r, epoch);
        ts[1] = relay_clock<ST>(listed);
        vec_tail<KL, KA, true>(p, b, lane, in, m);
    }
    ts[2] = relay_clock<ST, true>(0);                               // its state written
    relay_stamps_put<ST>((uint32_t)s, epoch, ts);
    return listed;
}

// The tile role: flat_wg_body_patch's stream of tile t, its rows' bar and counter (kp_in)
// staged with the window and their w' from the relay words. (A form that stored every chunk
// needing neither bar nor w' before reading the relay words, and the last-day / slot chunks
// after, ran 1.1-1.4x slower: the deferred 16-B chunks leave partly written lines between the
// two store waves — profiles/ab_r04/relay_split_r04s.err.)
// OUT: double-buffered (the chunks past the tile read straight from obs).
// ADOPT = false: the tile's own attempt, which polls `spin` times at most and returns false — having
// stored nothing — when a wave still misses a word; ADOPT = true: a deferred tile's run (by itself
// after the re-check, or by a scalar block), which polls once, returns false if a word is missing,
// and else runs only under the tile's claim (one run per step: in place, a second run would shift
// the window twice).
template <int BLOCK, int V, int POL, bool OUT, bool ADOPT, bool ST = false>
__device__ __forceinline__ bool relay_tile(const StepParams& p, const RelayParams& r, uint32_t qtot, uint32_t spin, uint32_t t,
                                           uint32_t epoch, const int32_t* kp_in, const float* halo_in,
                                           float* halo_out, f4* sh4, f4* sh_bar, float* sh_wp, int32_t* sh_kc,
                                           int32_t* sh_ok, uint64_t t_entry = 0) {
    uint64_t ts[6] = {t_entry, 0, 0, 0, 0, 0};
    constexpr int kAux = POL == 1 ? 2 : 0;
    constexpr int CPW = BLOCK * V, F = 5;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t c0 = t * CPW;
    const uint32_t nblk = min((uint32_t)CPW, qtot - c0);
    const auto rs = make_rsrc(p.obs + (size_t)c0 * 4, nblk * 16u);
    f4 own[V];
#pragma unroll
    for (int v = 0; v < V; ++v) own[v] = buf_load4<kAux>(rs, (uint32_t)(64 * V * wave + 64 * v + lane) * 16u);
    const uint32_t ntiles = (qtot + CPW - 1) / CPW;
    const uint32_t nh = t + 1 < ntiles ? min(2u, qtot - c0 - nblk) : 0u;
    const float* hsrc = OUT ? p.obs + (size_t)(c0 + nblk) * 4 : halo_in + (size_t)t * 8;
    const f4 hal = buf_load4<0>(make_rsrc(hsrc, nh * 16u), tid < 2 ? (uint32_t)tid * 16u : 0xFFFFFFF0u);
    __builtin_amdgcn_sched_barrier(0);
    // the tile's rows g_lo .. g_hi (global row = b N + n): thread i stages row g_lo + i
    const int N = p.N, W = p.W, WF = W * F;
    const uint32_t per4 = (uint32_t)(N * WF) >> 2;
    const uint32_t b_lo = fdiv(c0, p.div_units);
    const uint32_t g_lo = b_lo * (uint32_t)N + fdiv(4u * (c0 - b_lo * per4), p.div_wf);
    const uint32_t ql = c0 + nblk - 1u;
    const uint32_t b_hi = fdiv(ql, p.div_units);
    const uint32_t g_hi = b_hi * (uint32_t)N + fdiv(4u * (ql - b_hi * per4) + 3u, p.div_wf);
    const bool mine = (uint32_t)tid <= g_hi - g_lo;
    const uint32_t g = g_lo + (mine ? (uint32_t)tid : 0u);
    const uint32_t b = g / (uint32_t)N, n = g - b * (uint32_t)N;
    const float* barb = env_bar(p, (int)b);                         // null: a day outside the series
    const float nanv = __int_as_float(0x7fc00000);
    f4 xb = f4{nanv, nanv, nanv, nanv};
    int32_t kc = 0;
    uint64_t ww = 0;
    if (barb) xb = *reinterpret_cast<const f4*>(barb + (size_t)n * 4);
    kc = kp_in[b];
    // w': relayed by the scalar blocks, polled `spin` times at most (ADOPT: once)
    ww = relay_get(r.w + g);
    bool ready = !mine || (uint32_t)(ww >> 32) == epoch;
    ts[1] = relay_clock<ST>((uint32_t)ww);                          // its loads returned
    for (uint32_t polls = 0; !ADOPT && !__all(ready) && polls < spin; ++polls) {
        __builtin_amdgcn_s_sleep(2);
        if (!ready) {
            ww = relay_get(r.w + g);
            ready = (uint32_t)(ww >> 32) == epoch;
        }
    }
    const bool wave_ok = __all(ready);                              // the whole wave, before any branch
    ts[2] = relay_clock<ST>((uint32_t)ww);                          // wave 0's words arrived
    if (mine) {
        sh_bar[tid] = xb;
        sh_wp[tid] = __uint_as_float((uint32_t)ww);
        sh_kc[tid] = kc;
    }
#pragma unroll
    for (int v = 0; v < V; ++v) sh4[64 * V * wave + 64 * v + lane] = own[v];
    if (tid < 2) sh4[CPW + tid] = hal;
    if (lane == 0) sh_ok[wave] = wave_ok ? 1 : 0;
    __syncthreads();
    ts[3] = relay_clock<ST>(0);                                     // every wave staged
    if constexpr (ADOPT) {                                          // polled once; then the tile's claim
        bool tile_ok = true;
#pragma unroll
        for (int w = 0; w < BLOCK / 64; ++w) tile_ok = tile_ok && sh_ok[w] != 0;
        if (!tile_ok) return false;                                 // the whole workgroup: nothing stored
        if (tid == 0)
            sh_ok[BLOCK / 64] = __hip_atomic_exchange(r.done + t, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch;
        __syncthreads();
        if (!sh_ok[BLOCK / 64]) return true;                        // ran elsewhere
    }
    const auto rd = OUT ? make_rsrc(p.obs_out + (size_t)c0 * 4, nblk * 16u) : rs;
    const bool first_out = !OUT && t > 0;                           // feeds the previous tile's halo
    bool ok = true;
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int j = 64 * V * wave + 64 * v + lane;
        const uint32_t q = min(c0 + (uint32_t)j, qtot - 1u);
        const uint32_t bq = fdiv(q, p.div_units);
        const uint32_t j0 = 4u * (q - bq * per4);
        const uint32_t row = fdiv(j0, p.div_wf);
        const int kk = (int)(j0 - row * (uint32_t)WF);
        const int i = (int)(bq * (uint32_t)N + row - g_lo);
        const f4 n1 = sh4[j + 1], n2 = sh4[j + 2];
        const float sh[4] = {n1.y, n1.z, n1.w, n2.x};
        const float un[4] = {own[v].x, own[v].y, own[v].z, own[v].w};
        f4 o = compose2(p, kk, sh_kc[i], un, sh, [&](f4& x, float& xwp) {
            x = sh_bar[i];
            xwp = sh_wp[i];
        });
        if (!ADOPT && v == 0) {
            // the first attempt's vote: no branch on it ahead of the compose (that would put one more
            // LDS round trip on every tile's path), only the stores' offsets — a tile that gives up
            // drops its stores (out-of-range buffer offsets) and returns false
            int32_t okv = 1;
#pragma unroll
            for (int w = 0; w < BLOCK / 64; ++w) okv &= sh_ok[w];
            ok = __builtin_amdgcn_readfirstlane(okv) != 0;
        }
        buf_store4<kAux>(rd, ok ? (uint32_t)j * 16u : 0x80000000u, o);  // past the end: dropped
        if (ok && first_out && j < 2) reinterpret_cast<f4*>(halo_out)[2 * (t - 1) + j] = o;
    }
    ts[4] = relay_clock<ST>(0);                                     // its stores issued
    ts[5] = relay_clock<ST, true>(0);                               // its stores completed
    relay_stamps_put<ST>(r.scal + t, epoch, ts);
    return ok;
}

// A scalar block, after its units: every tile on the step's deferral list (as far as any of its
// waves read it, each after its own relay words completed: relay_list_read) whose words have all
// arrived, run under its claim. With the deferring tile's append-then-re-check, no listed tile is
// missed (step_relay.h's head). The normal case — an empty list — costs one LDS vote.
template <int BLOCK, int V, int POL, bool OUT, bool SEQ>
__device__ __forceinline__ void relay_adopt(f4* sh4, f4* sh_bar, float* sh_wp, int32_t* sh_kc, int32_t* sh_ok,
                                            uint32_t listed) {
    constexpr int kB = BLOCK / 64 + 1;                              // sh_ok's broadcast slot (the tile's: below)
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) sh_ok[wave] = (int32_t)__builtin_amdgcn_readfirstlane(listed);
    __syncthreads();
    uint32_t n = 0;
#pragma unroll
    for (int w = 0; w < BLOCK / 64; ++w) n = max(n, (uint32_t)sh_ok[w]);
    if (n == 0) return;
    const KArgs ka = kargs();
    const RelayCtx c = relay_ctx<SEQ>(ka.r);
    for (uint32_t i = 0; i < n; ++i) {
        __syncthreads();                                            // sh_ok / the tile's LDS are free
        if (threadIdx.x == 0) {
            const uint64_t e = relay_get(ka.r.list + 1 + i);        // its tile may not have stored it yet
            int32_t t = (uint32_t)(e >> 32) == c.epoch ? (int32_t)(uint32_t)e : -1;
            if (t >= 0 && __hip_atomic_load(ka.r.done + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == c.epoch)
                t = -1;                                             // ran already
            sh_ok[kB] = t;
        }
        __syncthreads();
        const int32_t t = __builtin_amdgcn_readfirstlane(sh_ok[kB]);
        if (t >= 0)
            (void)relay_tile<BLOCK, V, POL, OUT, true>(ka.p, ka.r, ka.qtot, 0u, (uint32_t)t, c.epoch, c.kp_in, c.halo_in,
                                                       c.halo_out, sh4, sh_bar, sh_wp, sh_kc, sh_ok);
    }
}

// A tile that gave up: append it to the deferral list, wait for that store, re-check once (and run
// under its claim if every word has arrived), exit
template <int BLOCK, int V, int POL, bool OUT, bool SEQ>
__device__ __forceinline__ void relay_defer(uint32_t t, f4* sh4, f4* sh_bar, float* sh_wp, int32_t* sh_kc,
                                            int32_t* sh_ok) {
    const KArgs ka = kargs();
    const RelayCtx c = relay_ctx<SEQ>(ka.r);
    if (threadIdx.x == 0) {
        uint64_t lw = relay_get(ka.r.list), nw;
        do {                                                        // {epoch, count}: a stale epoch restarts it
            nw = (uint32_t)(lw >> 32) == c.epoch ? lw + 1 : ((uint64_t)c.epoch << 32) | 1u;
        } while (!__hip_atomic_compare_exchange_strong(ka.r.list, &lw, nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT));
        const uint32_t slot = (uint32_t)(lw >> 32) == c.epoch ? (uint32_t)lw : 0u;
        relay_put(ka.r.list + 1 + slot, c.epoch, t);
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        __builtin_amdgcn_s_waitcnt(0);                              // the entry is stored before the re-check
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
    }
    __syncthreads();
    (void)relay_tile<BLOCK, V, POL, OUT, true>(ka.p, ka.r, ka.qtot, 0u, t, c.epoch, c.kp_in, c.halo_in, c.halo_out, sh4,
                                               sh_bar, sh_wp, sh_kc, sh_ok);
}

// BLOCK x V tiles (the flat stream's 256 x 2 / 512 x 2), POL the window stream's cache
// policy (0 default, 1 nt), (KL, KA) the scalar step's form (relay_scalar), OCC the waves
// per SIMD the kernel is held to (the 8-assets-per-lane form would otherwise take 84 VGPRs
// and cut the tiles to 5 waves per SIMD)
// ANY (tools build only): 1 — the dispatch order and the polls before a tile defers from the launch
// arguments (r.rot, r.spin), to force the deferral paths; 2 — the product's code with wall-clock
// stamps (relay_clock). The product (0) takes blockIdx order and kRelaySpin.
template <int BLOCK, int V, int POL, bool OUT, int KL, int KA, int OCC = 1, bool SEQ = false, int ANY = 0>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(OCC))) void step_relay_kernel(
    StepParams p, RelayParams r, uint32_t qtot) {
    __shared__ f4 sh4[BLOCK * V + 2];
    __shared__ f4 sh_bar[BLOCK];
    __shared__ float sh_wp[BLOCK];
    __shared__ int32_t sh_kc[BLOCK];
    __shared__ int32_t sh_ok[BLOCK / 64 + 2];   // the waves' votes | the claim | a broadcast
    const RelayCtx c = relay_ctx<SEQ>(r);
    if constexpr (SEQ) {                         // relay_prime_kernel published C and EC
        if (blockIdx.x == 0 && threadIdx.x == 0) {   // what the next step finds
            const uint64_t hobs = OUT ? 0ull : (uint64_t)(uintptr_t)r.obs;
            r.seq[kSeqD] = (uint32_t)((c.kp_in - r.kp) / r.B) ^ 1u;
            r.seq[kSeqE] = c.epoch;
            r.seq[kSeqV] = 1u;
            r.seq[kSeqHobs] = (uint32_t)hobs;
            r.seq[kSeqHobs + 1] = (uint32_t)(hobs >> 32);
        }
    }
    constexpr bool kSt = ANY == 2;
    const uint64_t t_entry = relay_clock<kSt>(0);
    uint32_t bid = blockIdx.x;
    if constexpr (ANY == 1) {
        bid += r.rot;
        if (bid >= r.grid) bid -= r.grid;
    }
    if (bid < r.scal) {
        const uint32_t listed = relay_scalar<BLOCK, KL, KA, kSt>(p, r, (int)bid, c.epoch, c.kp_out, t_entry);
        relay_adopt<BLOCK, V, POL, OUT, SEQ>(sh4, sh_bar, sh_wp, sh_kc, sh_ok, listed);
    } else if (!relay_tile<BLOCK, V, POL, OUT, false, kSt>(p, r, qtot, ANY == 1 ? r.spin : kRelaySpin, bid - r.scal, c.epoch,
                                                           c.kp_in, c.halo_in, c.halo_out, sh4, sh_bar, sh_wp, sh_kc,
                                                           sh_ok, t_entry)) {
        relay_defer<BLOCK, V, POL, OUT, SEQ>(bid - r.scal, sh4, sh_bar, sh_wp, sh_kc, sh_ok);
    }
}

// The relay step's copies of parity D (eager: r.par; device-sequenced: the word D): kp[D] <- the
// state's counter (when `prime_kp`), and in place halo[D][i] <- chunks (i + 1) * CPW and + 1 of
// the window (when p.halo, the parity-0 base). Device-sequenced (`seq`): V == 0 re-primes both,
// HOBS != this window the halo, and block 0 publishes C = D and EC = E + 1 for the step.
static __global__ __launch_bounds__(256) void relay_prime_kernel(StepParams p, RelayParams r, int prime_kp, int seq) {
    uint32_t d = r.par;
    bool kp = prime_kp != 0, halo = p.halo != nullptr;
    if (seq) {
        d = __builtin_amdgcn_readfirstlane(r.seq[kSeqD]);
        const uint32_t e = __builtin_amdgcn_readfirstlane(r.seq[kSeqE]);
        const uint32_t v = __builtin_amdgcn_readfirstlane(r.seq[kSeqV]);
        const uint64_t hobs = (uint64_t)__builtin_amdgcn_readfirstlane(r.seq[kSeqHobs]) |
                              ((uint64_t)__builtin_amdgcn_readfirstlane(r.seq[kSeqHobs + 1]) << 32);
        kp = v == 0;
        halo = halo && (v == 0 || hobs != (uint64_t)(uintptr_t)p.obs);
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            r.seq[kSeqC] = d;
            r.seq[kSeqEC] = e + 1u == 0u ? 1u : e + 1u;     // never the zeroed words' 0
        }
    }
    if (halo) {
        p.halo += (size_t)d * r.halo_stride;
        copy_halo(p);
    }
    if (kp) {
        int32_t* kpd = r.kp + (size_t)d * r.B;
        for (int b = blockIdx.x * blockDim.x + threadIdx.x; b < p.B; b += gridDim.x * blockDim.x) kpd[b] = p.k[b];
    }
}

}  // namespace pmenv_dev
