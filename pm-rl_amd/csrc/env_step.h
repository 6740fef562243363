// env_step.h — the env step and reset kernels.
//
// Reference semantics restated (zachramsey/pm-rl):
//   env/sim/trading_env.py:21-41 reset, :44-105 step
//   env/sim/weight_buffer.py:13-51 ring update / get_last / get_all
//   env/reward.py:20-31 returns / log_returns / sharpe_ratio
//   data/instrument.py:79 price relatives, :339-356 sliding window
//
// Advance mode (north-star fused path) runs as two launches on the caller's stream:
//   scalar_step_kernel  — one wave per env: normalisation, commission fixed point,
//                         value (f64), return, reward, weight drift; writes w' into
//                         the ring slot. Latency-bound, so it is kept out of the
//                         streaming kernel where it would stall every workgroup.
//   advance_rows_kernel — pure HBM streaming: each workgroup advances a unit of
//                         whole asset rows of one env's [N, W, F] window by one day
//                         in place and appends the bar and w'.
// step_advance_lds_kernel is the single-launch fallback for shapes the streaming
// kernel does not cover (F < 5, env blocks that are not 16-B granular, rows too long).
#pragma once
#include "common.h"

namespace pmenv_dev {

constexpr int kBlock = 256;         // threads per env workgroup (LDS / surface / reset kernels)
constexpr int kMaxVec = 8;          // float4 per thread for one LDS tile
constexpr int kTileFloats = kBlock * kMaxVec * 4;  // 8192 floats = 32 KiB LDS tile
constexpr int kScalarWaves = 4;     // envs (waves) per scalar_step_kernel workgroup
constexpr int kStreamBlock = 512;   // threads per advance_rows_kernel workgroup

// LDS carve of the per-env scalar scratch, behind an optional 16-B aligned tile region.
struct Scratch {
    double* wv;   // [N] target weights, then portfolio values
    double* yv;   // [N] price relatives
    float* wl;    // [N] w_last (ring.get_last())
    float* wp;    // [N] post-drift weights w'
    float* bar;   // [N * (F-1)] new bar (LDS kernel)
    int* ints;    // [3] shift_weights, slot, counter after the step
    int wp_off, bar_off;  // float offsets of wp / bar inside the LDS float array
};

__device__ __forceinline__ Scratch carve(float* lds, int tile_floats, int N, int F) {
    Scratch s;
    s.wv = reinterpret_cast<double*>(lds + tile_floats);
    s.yv = s.wv + N;
    s.wl = reinterpret_cast<float*>(s.yv + N);
    s.wp = s.wl + N;
    s.bar = s.wp + N;
    s.ints = reinterpret_cast<int*>(s.bar + N * (F - 1));
    s.wp_off = tile_floats + 4 * N + N;
    s.bar_off = s.wp_off + N;
    return s;
}

inline size_t scratch_bytes(int tile_floats, int N, int F) {
    return (size_t)tile_floats * 4 + (size_t)N * 16 + (size_t)N * 8 + (size_t)N * (F - 1) * 4 + 16;
}

// ---------------------------------------------------------------- the scalar step
// The per-env scalar part of TradingEnv.step (trading_env.py:54-100), on one wave,
// split in two so the loads can be issued early:
//   gather_inputs  — action, price relatives, w_last -> LDS scratch
//   scalar_compute — everything else, from LDS, in f64.
__device__ __forceinline__ void gather_inputs(const StepParams& p, int b, Scratch& s, int32_t k) {
    const int lane = threadIdx.x & 63;
    const int N = p.N, W = p.W, Fm = p.F - 1;
    // w_last = ActionBuffer.get_last() = ring slot k % W (weight_buffer.py:28-30), kept
    // densely in w_new so no load depends on the step counter
    const float* wlast = p.w_new + (size_t)b * N;
    (void)W; (void)k;
    const float* barb = p.bar ? env_bar(p, b) : nullptr;
    for (int n = lane; n < N; n += 64) {
        const size_t i = (size_t)b * N + n;
        const float a = p.action[i];
        double y = 0.0;
        if (p.bar) {
            // instrument.py:79 divides float32 tensors: the relative is the correctly
            // rounded fp32 quotient of today's close over the window's last close
            const float cn = barb ? barb[(size_t)n * Fm + p.close_ch] : NAN;
            y = p.prices ? (double)p.prices[i] : (double)(cn / p.last_close[i]);
            p.last_close[i] = cn;
        } else {
            y = (double)p.prices[i];
        }
        s.wv[n] = (double)a;
        s.yv[n] = y;
        s.wl[n] = wlast[n];
    }
}

// returns the portfolio value after the step (every lane)
__device__ __forceinline__ double scalar_compute(const StepParams& p, int b, Scratch& s, int32_t k,
                                                 double v_prev) {
    const int lane = threadIdx.x & 63;
    const int N = p.N, W = p.W;

    // :54-55 flatten; :58 isclose(sum) / min(action)
    double sum = 0.0, mn = INFINITY;
    int nan_seen = 0;
    for (int n = lane; n < N; n += 64) {
        const double a = s.wv[n];
        sum += a;
        mn = fmin(mn, a);
        nan_seen |= isnan(a);
    }
    sum = wave_sum(sum);
    mn = wave_min(mn);
    if (__any(nan_seen)) mn = NAN;               // torch.min propagates NaN

    // :58 normalise iff !isclose(sum, 1, atol=1e-6) AND (OR for the trainer) min < 0
    const bool not_close = !(fabs(sum - 1.0) <= 1e-6 + 1e-5);
    const bool negative = mn < 0.0;
    const bool norm = p.norm_mode == PMENV_NORM_AND ? (not_close && negative) : (not_close || negative);
    if (norm) {
        double shift = 0.0;
        if (p.norm_mode == PMENV_NORM_OR) {      // torch.softmax is max-shifted
            double m = -INFINITY;
            for (int n = lane; n < N; n += 64) m = fmax(m, s.wv[n]);
            shift = wave_max(m);
        }
        double z = 0.0;
        for (int n = lane; n < N; n += 64) {
            double e = exp(s.wv[n] - shift);      // :59 exp(w) (no max-shift in AND mode)
            s.wv[n] = e;
            z += e;
        }
        z = wave_sum(z);
        for (int n = lane; n < N; n += 64) s.wv[n] = s.wv[n] / z;   // :60
    }

    // :67-75 transaction remainder factor mu (PGPortfolio fixed point), f64, capped
    double V = v_prev;
    if (p.commission > 0.0) {
        const double c = p.commission;
        double mu_last = 1.0, mu = 1.0 - 2.0 * c + c * c;
        const double w0 = s.wv[0];
        const double wl0 = (double)s.wl[0];
        int it = 0;
        while (fabs(mu - mu_last) > p.mu_tol && it < p.mu_max_iter) {
            mu_last = mu;
            double part = 0.0;
            for (int n = lane; n < N; n += 64) {
                if (n == 0) continue;
                double d = (double)s.wl[n] - mu * s.wv[n];
                part += d > 0.0 ? d : 0.0;        // torch.maximum(x, 0) as intended
            }
            double tot = wave_sum(part);
            mu = (1.0 - c * wl0 - (2.0 * c - c * c) * tot) / (1.0 - c * w0);
            ++it;
        }
        V = mu * V;
    }

    // :78-79 portfolio = V * (w * y); value = sum(portfolio)
    double part = 0.0;
    for (int n = lane; n < N; n += 64) {
        double pv = V * (s.wv[n] * s.yv[n]);
        s.wv[n] = pv;
        part += pv;
    }
    const double value = wave_sum(part);

    // :83-84 w' = portfolio / value ; ring.update(w') at slot idx = (1 + k) % W
    const int slot = ring_slot(k, W);
    float* ring_row = p.ring + (size_t)b * W * N + (size_t)slot * N;
    for (int n = lane; n < N; n += 64) {
        float w = (float)(s.wv[n] / value);
        s.wp[n] = w;
        ring_row[n] = w;
        p.w_new[(size_t)b * N + n] = w;
        if (p.weights) p.weights[(size_t)b * N + n] = w;
    }

    if (lane == 0) {
        // :88 ret = value / self.value (mu-scaled: excludes commission) ; :89
        const double ret = p.ret_mode == PMENV_RET_GROSS ? value / V : value / v_prev;
        double r;
        switch (p.reward_kind) {
        case PMENV_REWARD_RETURN:
            r = ret * p.scale;
            break;
        case PMENV_REWARD_SHARPE: {              // reward.py:26-31 as running moments
            double m = (double)(k + 1);
            double mean = p.sa[b], m2 = p.sb[b];
            double d = ret - mean;
            mean += d / m;
            m2 += d * (ret - mean);
            p.sa[b] = mean;
            p.sb[b] = m2;
            r = m < 2.0 ? NAN : (mean - p.rf) / sqrt(m2 / (m - 1.0)) * p.scale;
            break;
        }
        case PMENV_REWARD_DIFF_SHARPE: {         // Moody & Saffell (1998)
            double R = ret - 1.0, A = p.sa[b], Bm = p.sb[b];
            double dA = R - A, dB = R * R - Bm, var = Bm - A * A;
            r = var > 1e-12 ? (Bm * dA - 0.5 * A * dB) / (var * sqrt(var)) * p.scale : 0.0;
            p.sa[b] = A + p.eta * dA;
            p.sb[b] = Bm + p.eta * dB;
            break;
        }
        default:
            r = log(ret) * p.scale;              // :99
        }
        p.value[b] = value;
        p.k[b] = k + 1;
        if (p.reward) p.reward[b] = (float)r;
        if (p.ret) p.ret[b] = ret;
        if (!isfinite(r) || !isfinite(value)) atomicAdd(p.nonfinite, 1ull);
        // weight channel: shift with the window until the ring is full, then
        // (reference storage order) overwrite slot `slot` in place
        s.ints[0] = (p.ring_mode == PMENV_RING_CHRONO) || (k < W - 1);
        s.ints[1] = slot;
        s.ints[2] = k + 1;
    }
    return value;
}

// ---------------------------------------------------------------- K1: scalar step
// One wave per env, kScalarWaves envs per workgroup, no barriers.
__device__ __forceinline__ void copy_halo(const StepParams& p);

static __global__ __launch_bounds__(64 * kScalarWaves) void scalar_step_kernel(StepParams p, int scratch_floats) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    copy_halo(p);
    const int wave = threadIdx.x >> 6;
    const int b = blockIdx.x * kScalarWaves + wave;
    if (b >= p.B) return;
    Scratch s = carve(lds + wave * scratch_floats, 0, p.N, p.F);
    const int32_t k = p.k[b];
    const double v_prev = p.value[b];
    gather_inputs(p, b, s, k);
    scalar_compute(p, b, s, k, v_prev);
}

// ---------------------------------------------------------------- K1, register form (N <= 64)
// L lanes per env (L = 32: two envs per wave for N <= 32; L = 64: one), one asset
// per lane, every per-asset value in VGPRs. Reductions are DPP row shifts plus a
// fixed-order combine of the row totals of the lane's group, so each group's lanes
// hold bitwise the same value. No LDS, no barrier, one memory round trip.
template <int L>
__device__ __forceinline__ double group_combine(double r0, double r1, double r2, double r3, int lane) {
    if (L == 64) return (r0 + r1) + (r2 + r3);
    return lane < 32 ? r0 + r1 : r2 + r3;
}
// After the row shifts, DPP row_bcast:15 on rows 1 and 3 (row_mask 0xA) adds the previous
// row's total into them: lane 31 holds r1 + r0 and lane 63 r3 + r2, the pair sums of
// group_combine, in the same order (f64 addition commutes bitwise) — two readlanes per
// half instead of four, the same bits.
constexpr int kRowBcast15 = 0x142;
template <int L>
__device__ __forceinline__ double group_sum(double v, int lane) {
    v += dpp_shift<kRowShr1>(v, 0.0);
    v += dpp_shift<kRowShr2>(v, 0.0);
    v += dpp_shift<kRowShr4>(v, 0.0);
    v += dpp_shift<kRowShr8>(v, 0.0);
    const int lo = __double2loint(v), hi = __double2hiint(v);
    const double prev = __hiloint2double(__builtin_amdgcn_update_dpp(0, hi, kRowBcast15, 0xA, 0xF, false),
                                         __builtin_amdgcn_update_dpp(0, lo, kRowBcast15, 0xA, 0xF, false));
    v += prev;                                    // rows 0 and 2: + 0.0
    const double p01 = lane_value(v, 31), p23 = lane_value(v, 63);
    if (L == 64) return p01 + p23;
    return lane < 32 ? p01 : p23;
}
template <int L>
__device__ __forceinline__ double group_max(double v, int lane) {
    v = fmax(v, dpp_shift<kRowShr1>(v, -INFINITY));
    v = fmax(v, dpp_shift<kRowShr2>(v, -INFINITY));
    v = fmax(v, dpp_shift<kRowShr4>(v, -INFINITY));
    v = fmax(v, dpp_shift<kRowShr8>(v, -INFINITY));
    const double r0 = lane_value(v, 15), r1 = lane_value(v, 31), r2 = lane_value(v, 47), r3 = lane_value(v, 63);
    if (L == 64) return fmax(fmax(r0, r1), fmax(r2, r3));
    return lane < 32 ? fmax(r0, r1) : fmax(r2, r3);
}
template <int L>
__device__ __forceinline__ double group_min(double v, int lane) {
    v = fmin(v, dpp_shift<kRowShr1>(v, INFINITY));
    v = fmin(v, dpp_shift<kRowShr2>(v, INFINITY));
    v = fmin(v, dpp_shift<kRowShr4>(v, INFINITY));
    v = fmin(v, dpp_shift<kRowShr8>(v, INFINITY));
    const double r0 = lane_value(v, 15), r1 = lane_value(v, 31), r2 = lane_value(v, 47), r3 = lane_value(v, 63);
    if (L == 64) return fmin(fmin(r0, r1), fmin(r2, r3));
    return lane < 32 ? fmin(r0, r1) : fmin(r2, r3);
}

// lane 0 of the lane's L-lane group (0 or 32), read through the scalar unit
template <int L>
__device__ __forceinline__ int group_lane0_i(int v, int lane) {
    const int a = __builtin_amdgcn_readlane(v, 0);
    if (L == 64) return a;
    const int b = __builtin_amdgcn_readlane(v, 32);
    return lane < 32 ? a : b;
}
template <int L>
__device__ __forceinline__ double group_lane0(double v, int lane) {
    return __hiloint2double(group_lane0_i<L>(__double2hiint(v), lane), group_lane0_i<L>(__double2loint(v), lane));
}

// The per-env step of lane group (b, lane % L) in two halves, so a caller can put
// other loads between them: a load half issues every load (none dependent on
// another, no data-dependent branch), scalar_finish computes and returns the
// lane's w' (0 past N) and the counter before the step.
struct ScalarIn {
    int32_t k;
    int bar_ok;      // bar4: the day is inside the series
    double v_prev;
    double sa, sb;   // reward statistics (Sharpe moments / differential-Sharpe EMAs)
    float a, wlf;
    float cn;        // today's close (not bar4)
    float pl;        // caller prices (advance with prices / surface) or the window's last close
    f4 bar;          // bar4: the lane's whole bar row
};

// K1 form: L lanes per env, every load unconditional from a clamped (always
// valid) address and masked afterwards, so several envs' loads can be in flight
// together without control-flow joins between them
//
// LV (the register step, one env per workgroup): the env's counter, value and statistics are
// read as lane values at a lane-varying zero offset `zoff` — a load the compiler sees as
// uniform gets its value moved to an SGPR right after issue, and the wait for that would hold
// every load issued after it back by a memory round trip
template <int L, bool LV = false>
__device__ __forceinline__ ScalarIn scalar_load(const StepParams& p, int b, int lane, uint32_t zoff = 0u) {
    const int n = lane % L;
    const int N = p.N, Fm = p.F - 1;
    const bool env_ok = b < p.B;
    const bool act = env_ok && n < N;
    const int bc = env_ok ? b : 0;
    const int nc = act ? n : 0;
    const size_t i = (size_t)bc * N + nc;
    ScalarIn in;
    if constexpr (LV) {
        in.k = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(make_rsrc(p.k + bc, 4u), zoff, 0, 0);
        in.v_prev = buf_load_f64(make_rsrc(p.value + bc, 8u), zoff);
        in.sa = buf_load_f64(make_rsrc(p.sa + bc, 8u), zoff);
        in.sb = buf_load_f64(make_rsrc(p.sb + bc, 8u), zoff);
    } else {
        in.k = p.k[bc];
        in.v_prev = p.value[bc];
        in.sa = p.sa[bc];
        in.sb = p.sb[bc];
    }
    const float a = p.action[i];
    const float wl = p.w_new[i];                                       // get_last() (weight_buffer.py:28-30)
    const float* barb = p.bar ? env_bar(p, bc) : nullptr;
    const float cv = *(barb ? barb + (size_t)nc * Fm + p.close_ch : p.action + i);
    const float pl = *((p.prices ? p.prices : p.last_close) + i);
    in.a = act ? a : 0.0f;
    in.wlf = act ? wl : 0.0f;
    in.cn = barb ? cv : NAN;
    in.pl = act ? pl : 1.0f;
    in.bar_ok = 0;
    in.bar = f4{0.f, 0.f, 0.f, 0.f};
    return in;
}

// fused form (advance mode, F = 5, one env per wave): branch-free buffer loads
// (lanes past N read 0) and the lane's whole bar row (16 B)
__device__ __forceinline__ ScalarIn scalar_load_row(const StepParams& p, int b, int lane) {
    const int N = p.N;
    const uint32_t nb = (uint32_t)N * 4u, off = (uint32_t)lane * 4u;
    ScalarIn in;
    in.k = p.k[b];
    in.v_prev = p.value[b];
    in.sa = p.sa[b];
    in.sb = p.sb[b];
    in.a = buf_load1(make_rsrc(p.action + (size_t)b * N, nb), off);
    in.wlf = buf_load1(make_rsrc(p.w_new + (size_t)b * N, nb), off);
    in.pl = buf_load1(make_rsrc((p.prices ? p.prices : p.last_close) + (size_t)b * N, nb), off);
    const float* barb = env_bar(p, b);            // null: out-of-range day -> the descriptor reads 0
    in.bar = buf_load4(make_rsrc(barb ? barb : p.bar, barb ? nb * 4u : 0u), off * 4u);
    in.bar_ok = barb != nullptr;
    in.cn = 0.0f;
    return in;
}

// The scalar step in two halves. scalar_core computes what the window's compose needs
// — the normalised weights, the commission factor, the portfolio value and w' — and
// nothing else; scalar_tail does every state write and the return / reward (lane 0's
// f64 division, log and statistics). The one-launch steps run the tail after the
// window's barrier and stores, so the barrier waits for the core only.
struct ScalarMid {
    double value, V;   // portfolio value after the step, mu-scaled value before it
    float wp, cn;      // the lane's w' (0 past N) and today's close
    int32_t k;         // the counter before the step
};

template <int L, bool ROW = false>
__device__ __forceinline__ ScalarMid scalar_core(const StepParams& p, int b, int lane, const ScalarIn& in) {
    const int n = lane % L;
    const int N = p.N;
    const bool env_ok = b < p.B;
    const bool act = env_ok && n < N;
    const double v_prev = in.v_prev;
    const double a = (double)in.a;
    const float wlf = in.wlf;
    // instrument.py:79 divides float32 tensors: the relative is the correctly
    // rounded fp32 quotient of today's close over the window's last close
    double y = 1.0;
    float cn = 0.0f;
    if (act) {
        if (p.bar) {
            if (ROW) {
                const int c = p.close_ch;
                // bit-mask selects: a nested ?: chain on the runtime channel was miscompiled in
                // one kernel (ROCm 7.2 clang: channel 3 read the .y component)
                cn = pick(in.bar_ok, pick(c == 0, in.bar.x, pick(c == 1, in.bar.y, pick(c == 2, in.bar.z, in.bar.w))),
                          __int_as_float(0x7fc00000));
            } else {
                cn = in.cn;
            }
            y = p.prices ? (double)in.pl : (double)(cn / in.pl);
        } else {
            y = (double)in.pl;
        }
    }

    // :58 normalise iff !isclose(sum, 1, atol=1e-6) AND (OR: trainer) min(action) < 0.
    // AND mode with every group's sum close to 1 (simplex actions) cannot normalise:
    // the min reduction is skipped (wave-uniform), the result is the same
    const double sum = group_sum<L>(act ? a : 0.0, lane);
    const bool not_close = !(fabs(sum - 1.0) <= 1e-6 + 1e-5);
    bool norm = false;
    if (p.norm_mode != PMENV_NORM_AND || __any(not_close)) {
        double mn = group_min<L>(act ? a : INFINITY, lane);
        const bool nan_here = act && isnan(a);
        const uint64_t nan_mask = __ballot(nan_here);
        const uint64_t gmask = L == 64 ? ~0ull : (lane < 32 ? 0xFFFFFFFFull : 0xFFFFFFFF00000000ull);
        if (nan_mask & gmask) mn = NAN;           // torch.min propagates NaN
        const bool negative = mn < 0.0;
        norm = p.norm_mode == PMENV_NORM_AND ? (not_close && negative) : (not_close || negative);
    }
    double w = a;
    if (__any(norm)) {
        double shift = 0.0;
        if (p.norm_mode == PMENV_NORM_OR) shift = group_max<L>(act ? a : -INFINITY, lane);
        const double e = act ? exp(a - shift) : 0.0;             // :59 (no max-shift in AND mode)
        const double z = group_sum<L>(e, lane);
        if (norm) w = e / z;                                      // :60
    }

    // :67-75 commission fixed point (f64, capped), per env group: the reference's iteration
    // mu <- (1 - c wl0 - (2c - c^2) S(mu)) / (1 - c w0), S(mu) = sum_{n>=1} max(wl_n - mu w_n, 0),
    // with S in active-set form: S(mu) = A - mu Bw over the assets P(mu) where wl_n > mu w_n
    // (the same set the max keeps). P is one ballot per iteration; A and Bw are reduced only
    // when P changes — in practice on the first one or two iterations — so the later
    // iterations are a few scalar f64 operations instead of a group reduction each. The
    // iterates equal the reference's up to f64 rounding of S (parity: value rtol 1e-12).
    // The division by 1 - c w0 (fixed over the iterations) is a multiplication by its
    // reciprocal, and the group's asset-0 values are read with v_readlane (SALU path) rather
    // than a cross-lane shuffle through LDS.
    double V = v_prev;
    if (p.commission > 0.0) {
        const double c = p.commission;
        const double w0 = group_lane0<L>(w, lane);
        const double wl0 = (double)__int_as_float(group_lane0_i<L>(__float_as_int(wlf), lane));
        const double K = 1.0 - c * wl0, Dc = 2.0 * c - c * c, invE = 1.0 / (1.0 - c * w0);
        const uint64_t gmask = L == 64 ? ~0ull : (lane < 32 ? 0xFFFFFFFFull : 0xFFFFFFFF00000000ull);
        const bool cand = act && n > 0;
        const double wld = (double)wlf;
        double mu_last = 1.0, mu = 1.0 - 2.0 * c + c * c;
        double Aw = 0.0, Bw = 0.0;
        uint64_t pset = 0;
        bool have = false;
        int it = 0;
        bool done = !(fabs(mu - mu_last) > p.mu_tol) || p.mu_max_iter <= 0;
        while (__any(!done)) {
            const bool in_p = cand && wld - mu * w > 0.0;            // torch.maximum(x, 0) as intended
            const uint64_t m = __ballot(in_p) & gmask;
            if (__any(!done && (!have || m != pset))) {             // a group's active set changed
                Aw = group_sum<L>(in_p ? wld : 0.0, lane);
                Bw = group_sum<L>(in_p ? w : 0.0, lane);
                pset = m;
                have = true;
            }
            if (!done) {
                mu_last = mu;
                mu = (K - Dc * (Aw - mu * Bw)) * invE;
                ++it;
                done = !(fabs(mu - mu_last) > p.mu_tol) || it >= p.mu_max_iter;
            }
        }
        V = mu * V;
    }

    // :78-79 portfolio value; :83-84 w' = portfolio / value
    const double pv = act ? V * (w * y) : 0.0;
    ScalarMid m;
    m.value = group_sum<L>(pv, lane);
    m.V = V;
    m.wp = act ? (float)(pv / m.value) : 0.0f;
    m.cn = cn;
    m.k = in.k;
    return m;
}

// trading_env.py:88 ret = value / self.value (gross: mu-scaled, excludes commission)
__device__ __forceinline__ double step_ret(const StepParams& p, const ScalarIn& in, const ScalarMid& m) {
    return p.ret_mode == PMENV_RET_GROSS ? m.value / m.V : m.value / in.v_prev;
}

// the step's reward from its return (trading_env.py:89-99, reward.py); the Sharpe forms
// update their running statistics sa / sb (stats = true). k: the counter before the step
__device__ __forceinline__ double step_reward(const StepParams& p, int32_t k, double ret, double& sa, double& sb,
                                              bool& stats) {
    switch (p.reward_kind) {
    case PMENV_REWARD_RETURN:
        return ret * p.scale;
    case PMENV_REWARD_SHARPE: {              // reward.py:26-31 as running moments
        double mm = (double)(k + 1);
        double mean = sa, m2 = sb;
        double d = ret - mean;
        mean += d / mm;
        m2 += d * (ret - mean);
        sa = mean;
        sb = m2;
        stats = true;
        return mm < 2.0 ? NAN : (mean - p.rf) / sqrt(m2 / (mm - 1.0)) * p.scale;
    }
    case PMENV_REWARD_DIFF_SHARPE: {         // Moody & Saffell (1998)
        double R = ret - 1.0, A = sa, Bm = sb;
        double dA = R - A, dB = R * R - Bm, var = Bm - A * A;
        const double r = var > 1e-12 ? (Bm * dA - 0.5 * A * dB) / (var * sqrt(var)) * p.scale : 0.0;
        sa = A + p.eta * dA;
        sb = Bm + p.eta * dB;
        stats = true;
        return r;
    }
    default:
        return log(ret) * p.scale;           // :99
    }
}

// SNAP (step_flat_kernel): only the env's owner workgroup (`owner`) writes the state,
// reward and ring slot, and it also writes the next step's snapshot (sv_out .. slc_out)
template <int L, bool SNAP = false>
__device__ __forceinline__ void scalar_tail(const StepParams& p, int b, int lane, const ScalarIn& in,
                                            const ScalarMid& m, bool owner = true) {
    const int n = lane % L;
    const int N = p.N, W = p.W;
    const bool env_ok = b < p.B;
    const bool act = env_ok && n < N;
    const size_t i = (size_t)(env_ok ? b : 0) * N + (act ? n : 0);
    const int32_t k = m.k;
    const double value = m.value;
    // :83-84 ring.update(w') at slot idx = (1 + k) % W
    const int slot = ring_slot(k, W);
    const bool wr = !SNAP || owner;
    if (act && wr) {
        const float wp = m.wp;
        p.ring[(size_t)b * W * N + (size_t)slot * N + n] = wp;
        p.w_new[i] = wp;
        if (p.weights) p.weights[i] = wp;
        if (p.bar) p.last_close[i] = m.cn;
        if (SNAP) {
            if (p.commission > 0.0) p.sw_out[i] = wp;      // get_last() feeds only the fixed point
            p.slc_out[i] = m.cn;
        }
    }
    if (env_ok && n == 0 && wr) {
        // :88 ret = value / self.value (mu-scaled: excludes commission) ; :89
        const double ret = step_ret(p, in, m);
        double sa = in.sa, sb = in.sb;
        bool stats = false;
        const double r = step_reward(p, k, ret, sa, sb, stats);
        if (stats) {
            p.sa[b] = sa;
            p.sb[b] = sb;
        }
        p.value[b] = value;
        p.k[b] = k + 1;
        if (SNAP) {
            p.sv_out[b] = value;
            p.sk_out[b] = k + 1;
        }
        if (p.reward) p.reward[b] = (float)r;
        if (p.ret) p.ret[b] = ret;
        if (!isfinite(r) || !isfinite(value)) atomicAdd(p.nonfinite, 1ull);
    }
}

// the whole scalar step: core, then tail; returns the lane's w' (0 past N) and the
// counter before the step
template <int L, bool ROW = false, bool SNAP = false>
__device__ __forceinline__ float scalar_finish(const StepParams& p, int b, int lane, const ScalarIn& in,
                                               int32_t& k_before, bool owner = true) {
    const ScalarMid m = scalar_core<L, ROW>(p, b, lane, in);
    scalar_tail<L, SNAP>(p, b, lane, in, m, owner);
    k_before = m.k;
    return m.wp;
}

// The in-place flat advance's halo (copy_halo in env_step.h) in two halves: the
// loads go out with the step's own loads, the stores after its compute, so the copy
// costs the wave no extra memory round trip. Items past two per thread (grids
// smaller than half the halo) take the plain loop at the end.
struct HaloRegs {
    f4 v[4];
    bool d0, d1;
};

// halo item i (two chunks): boundary i >> halo_hs, chunks 2 (i & (2^hs - 1)) + {0, 1} past it
__device__ __forceinline__ uint32_t halo_src(const StepParams& p, uint32_t i) {
    return ((i >> p.halo_hs) + 1u) * p.halo_block + 2u * (i & ((1u << p.halo_hs) - 1u));
}

__device__ __forceinline__ HaloRegs halo_load(const StepParams& p) {
    HaloRegs h;
    const uint32_t nthr = gridDim.x * blockDim.x, gid = blockIdx.x * blockDim.x + threadIdx.x;
    h.d0 = p.halo && gid < p.halo_wgs;
    h.d1 = p.halo && gid + nthr < p.halo_wgs;
    const f4* src = reinterpret_cast<const f4*>(p.obs);
    const f4 z = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const bool d = t ? h.d1 : h.d0;
        const uint32_t q = halo_src(p, gid + t * nthr);
        h.v[2 * t] = d && q < p.halo_qtot ? src[q] : z;
        h.v[2 * t + 1] = d && q + 1 < p.halo_qtot ? src[q + 1] : z;
    }
    return h;
}

__device__ __forceinline__ void halo_store(const StepParams& p, const HaloRegs& h) {
    if (!p.halo) return;
    const uint32_t nthr = gridDim.x * blockDim.x, gid = blockIdx.x * blockDim.x + threadIdx.x;
    f4* dst = reinterpret_cast<f4*>(p.halo);
    if (h.d0) { dst[2 * gid] = h.v[0]; dst[2 * gid + 1] = h.v[1]; }
    if (h.d1) { dst[2 * (gid + nthr)] = h.v[2]; dst[2 * (gid + nthr) + 1] = h.v[3]; }
    const f4* src = reinterpret_cast<const f4*>(p.obs);
    for (uint32_t i = gid + 2 * nthr; i < p.halo_wgs; i += nthr) {
        const uint32_t q = halo_src(p, i);
        dst[2 * i] = q < p.halo_qtot ? src[q] : f4{0.f, 0.f, 0.f, 0.f};
        dst[2 * i + 1] = q + 1 < p.halo_qtot ? src[q + 1] : f4{0.f, 0.f, 0.f, 0.f};
    }
}

// P env groups per wave in sequence, all their loads issued first: P times the
// bytes in flight per wave for a latency-bound kernel; the in-place stream's halo copy
// loads with them and stores at the end (HaloRegs)
template <int L, int P>
__global__ __launch_bounds__(256) void scalar_step_reg_kernel(StepParams p) {
    const HaloRegs halo = halo_load(p);
    constexpr int EPW = 64 / L;                   // envs per wave and group
    const int lane = threadIdx.x & 63;
    const int w = blockIdx.x * 4 + (int)(threadIdx.x >> 6);
    ScalarIn in[P];
#pragma unroll
    for (int j = 0; j < P; ++j) in[j] = scalar_load<L>(p, (w * P + j) * EPW + lane / L, lane);
#pragma unroll
    for (int j = 0; j < P; ++j) {
        int32_t k;
        (void)scalar_finish<L>(p, (w * P + j) * EPW + lane / L, lane, in[j], k);
    }
    halo_store(p, halo);
}

// ---------------------------------------------------------------- K2: window advance
// A workgroup owns `unit_rows` whole asset rows of one env (a unit never straddles
// an env; rows only ever read themselves, so units are independent). F = 5
// ([open, high, low, close, weight], the BASELINE layout; other F take the LDS
// fallback). Thread q owns output chunk q = floats 4q..4q+3 of the unit:
//   out[n, t, f]   = t < W-1 ? in[n, t+1, f] : bar[n, f]               (market)
//   out[n, t, F-1] = shifted with w'[n] appended at t = W-1, or — ring full,
//                    storage order (weight_buffer.py:38-39) — in[n, t, F-1] with
//                    w'[n] at t == slot.
// Everything a chunk can need is loaded straight into VGPRs before the one
// barrier, with no dependency on the step counter: the shifted source
// in[4q+5 .. 4q+8] (one dword-aligned 16-B load), the bar row of the chunk's
// asset (16 B, only if the chunk touches the last day), w'[n] and the chunk's
// unshifted weight float. After the barrier — which closes the in-place
// read-before-write window of the unit — the chunk is pure selects and one 16-B
// store: a workgroup lives one memory round trip plus its store issue, which is
// what bounds this kernel (bytes in flight per CU = residency x unit size).
// ABL (timing-only ablation builds, tools/ab_advance.py; 0 in the product):
//   1 = skip the bar / w' loads, 2 = skip the unshifted-weight load, 4 = store xs as is.
// FUSED (whole-env units, N <= 64): the workgroup also runs the env's scalar step
// on its first wave, after every streaming load is in flight, and hands w' and the
// counter to the other waves through LDS — one launch per step instead of two.
// POL: cache policy of the 16-B window stream (the shifted-source loads and the
// stores), every byte of which is touched once per step: 0 = default, 1 = nt,
// 2 = sc0 nt (aux bits 2 / 3). The small bar / w' / unshifted-weight loads re-read
// lines other lanes fetch and keep the default policy.
template <int BLOCK, int V, bool INPLACE, int ABL = 0, bool FUSED = false, int POL = 0>
__global__ __launch_bounds__(BLOCK) void advance_rows_kernel(StepParams p) {
    constexpr int kAux = POL == 1 ? 2 : POL == 2 ? 3 : 0;
    constexpr int F = 5;
    const int tid = threadIdx.x;
    const int N = p.N, W = p.W;
    const int WF = W * F;
    const int R = p.unit_rows;
    const int b = (int)fdiv(blockIdx.x, p.div_units);
    const int r0 = (int)(blockIdx.x - (uint32_t)b * (uint32_t)p.units_per_env) * R;
    const int rows = min(R, N - r0);
    const uint32_t nf = (uint32_t)(rows * WF);
    const uint32_t nq = nf >> 2;
    // descriptors: the env's window (loads may run past the unit into the env,
    // never past the env), this unit's rows (stores), the env's bar and w' rows
    float* env_obs = p.obs + (size_t)b * N * WF;
    const uint32_t unit_off = (uint32_t)(r0 * WF) * 4u;
    const auto rs_env = make_rsrc(env_obs, (uint32_t)(N * WF) * 4u);
    float* env_out = p.obs_out + (size_t)b * N * WF;
    const auto rs_unit = make_rsrc(env_out + (size_t)r0 * WF, nf * 4u);
    const float* barb = env_bar(p, b);            // null: out-of-range day -> NaN bar (wave-uniform)
    const auto rs_bar = make_rsrc(barb ? barb : p.bar, barb ? (uint32_t)(rows + r0) * 16u : 0u);
    const auto rs_wp = make_rsrc(p.w_new + (size_t)b * N, (uint32_t)(rows + r0) * 4u);

    f4 xs[V], xb[V];
    float xwp[V], xun[V];
    int kk0[V];
    // FUSED: the first wave's scalar loads go out ahead of its streaming loads
    ScalarIn sin;
    if (FUSED && tid < 64) sin = scalar_load_row(p, b, tid);
#pragma unroll
    for (int i = 0; i < V; ++i) {
        const uint32_t q = (uint32_t)(tid + i * BLOCK);
        const uint32_t j0 = 4u * q;
        const uint32_t row = fdiv(j0, p.div_wf);
        const int kk = (int)(j0 - row * (uint32_t)WF);   // position of the chunk's first float in its row
        const int f0 = kk - (int)fdiv((uint32_t)kk, p.div_f) * F;
        const int ew = min(F - 1 - f0, 3);                // element holding the weight channel
        kk0[i] = kk;
        xs[i] = buf_load4<kAux>(rs_env, unit_off + (j0 + F) * 4u);           // shifted source
        xb[i] = f4{0.f, 0.f, 0.f, 0.f};
        xwp[i] = 0.f;
        xun[i] = 0.f;
        if (FUSED) {
            kk0[i] |= (int)min(row, 63u) << 16;                             // asset: bar and w' from LDS
        } else if (!(ABL & 1)) {
            xb[i] = barb ? buf_load4(rs_bar, (uint32_t)(r0 + (int)row) * 16u)   // the asset's new bar
                         : f4{NAN, NAN, NAN, NAN};                              // day outside the series
            xwp[i] = buf_load1(rs_wp, (uint32_t)(r0 + (int)row) * 4u);      // its new weight w'
        }
        if (!(ABL & 2)) xun[i] = buf_load1(rs_env, unit_off + (j0 + (uint32_t)ew) * 4u);   // unshifted weight
    }
    int32_t k;
    if (FUSED) {
        __shared__ f4 sh_bar[64];
        __shared__ float sh_wp[64];
        __shared__ int32_t sh_k;
        if (tid < 64) {
            int32_t kb;
            const float wp = scalar_finish<64, true>(p, b, tid, sin, kb);
            sh_wp[tid] = wp;
            sh_bar[tid] = sin.bar_ok ? sin.bar : f4{NAN, NAN, NAN, NAN};
            if (tid == 0) sh_k = kb;
        }
        if (INPLACE) __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        k = sh_k;
#pragma unroll
        for (int i = 0; i < V; ++i) {
            xwp[i] = sh_wp[kk0[i] >> 16];
            xb[i] = sh_bar[kk0[i] >> 16];
            kk0[i] &= 0xFFFF;
        }
    } else {
        k = p.k[b] - 1;                              // scalar_step_kernel already counted this step
        if (INPLACE) {
            // in place: every load of the unit lands before the unit's first store
            __builtin_amdgcn_s_waitcnt(0);
            __syncthreads();
        }
    }

    const bool shift_w = !(p.ring_mode == PMENV_RING_STORAGE && k >= W - 1);
    const int slotF = ring_slot(k, W) * F;
#pragma unroll
    for (int i = 0; i < V; ++i) {
        const uint32_t q = (uint32_t)(tid + i * BLOCK);
        float v[4] = {xs[i].x, xs[i].y, xs[i].z, xs[i].w};
        const float bv[4] = {xb[i].x, xb[i].y, xb[i].z, xb[i].w};
        int kk = kk0[i];
        int f = kk - (int)fdiv((uint32_t)kk, p.div_f) * F;
#pragma unroll
        for (int e = 0; e < ((ABL & 4) ? 0 : 4); ++e) {
            const bool lastday = kk >= WF - F;        // false after wrapping into the next row
            if (f == F - 1) {
                const bool w_here = shift_w ? lastday : (kk - f == slotF);
                v[e] = w_here ? xwp[i] : (shift_w ? v[e] : xun[i]);
            } else {
                const float bf = f == 0 ? bv[0] : f == 1 ? bv[1] : f == 2 ? bv[2] : bv[3];
                v[e] = lastday ? bf : v[e];
            }
            ++kk;
            if (++f == F) f = 0;
            if (kk == WF) kk = 0;
        }
        if (ABL & 4) v[0] += bv[0] + xwp[i] + xun[i];
        buf_store4<kAux>(rs_unit, q * 16u, f4{v[0], v[1], v[2], v[3]});  // lanes past the unit: dropped
    }
    (void)nq;
}

// ---------------------------------------------------------------- K2, double-buffered: flat stream
// The out-of-place advance as a flat 16-B stream over the whole [B, N, W, F] tensor
// (obs -> obs_out): lane q of the grid owns output chunk q (floats 4q..4q+3) and
// loads only the ALIGNED input chunk q. The shifted source of chunk q, floats
// 4q+5..4q+8, is elements 1..3 of chunk q+1 and element 0 of chunk q+2 — the own
// chunks of lanes l+1 and l+2, moved across the wave with ds_bpermute; lanes 62 and
// 63 take chunks wbase+64 and wbase+65 from one wave-uniform 32-B load. Each input
// line is thus fetched by one wave instruction and the workgroup holds one chunk per
// thread (4 KiB at 256 threads): the shape of the fastest plain copy measured on this
// chip (tools/copybench.hip). Per element, at row position pos = kk + e of the
// chunk's asset row (pos >= WF: the chunk has wrapped into the next row, whose
// positions 0..2 are never a last day or a weight slot for W >= 2, so they take the
// shifted value):
//   market:  pos >= WF-F (last day) ? bar[f] : shifted
//   weight:  shift mode: last day ? w' : shifted;  storage mode: pos == slot ? w' : own
// The bar is fetched only by lanes whose chunk touches the row's last day (the other
// lanes' offsets are out of the descriptor's range: no traffic).
// Requirements (host-checked): F == 5, W >= 2, N*W*F % 4 == 0, B*N*W*F/4 < 2^31.

// What chunk q of the flat stream needs besides its input chunks: its position in
// its asset row, the row's bar (only lanes whose chunk touches the last day load it;
// the others' offsets are out of range: no traffic), w' and the env's counter.
struct FlatSide {
    int kk;            // row position of the chunk's first float
    bool bar_nan;      // resident series: a day outside the series -> NaN bar
    f4 xb;
    float xwp;
    int32_t k;
};

// SKIP (timing-only ablation bits, 0 in the product): 1 bar, 2 w', 4 counter, 8 day
template <int SKIP = 0>
__device__ __forceinline__ FlatSide flat_side_load(const StepParams& p, uint32_t q) {
    constexpr int F = 5;
    const int N = p.N, WF = p.W * F;
    const uint32_t per4 = (uint32_t)(N * WF) >> 2;                        // chunks per env
    FlatSide sd;
    const uint32_t b = fdiv(q, p.div_units);                              // div_units: per4 here
    const uint32_t j0 = 4u * (q - b * per4);
    const uint32_t row = fdiv(j0, p.div_wf);
    sd.kk = (int)(j0 - row * (uint32_t)WF);
    const bool touch_last = sd.kk + 3 >= WF - F;
    // branch-free: without a day index the day descriptor has no records (reads 0), so
    // no control flow can hold the streaming loads behind the day's latency
    // the day index only in resident-series mode: a wave-uniform branch on the kernel
    // argument, taken after the caller has issued its streaming loads, so the bar
    // load of the bar-batch mode depends on no other load
    const bool by_day = p.day != nullptr;
    int32_t d = 0;
    if (!(SKIP & 8) && by_day) d = p.day[b];
    sd.bar_nan = by_day && (d < 0 || d >= p.series_days);
    const uint32_t bar_bytes = (uint32_t)(by_day ? p.series_days : p.B) * (uint32_t)N * 16u;
    const uint32_t bar_row = by_day ? (uint32_t)d : b;
    const uint32_t bar_off = touch_last && !sd.bar_nan ? (bar_row * (uint32_t)N + row) * 16u : 0xFFFFFFF0u;
    sd.xb = (SKIP & 1) ? f4{1.f, 1.f, 1.f, 1.f} : buf_load4<0>(make_rsrc(p.bar, bar_bytes), bar_off);
    sd.xwp = (SKIP & 2) ? 0.5f : p.w_new[(size_t)b * N + row];
    sd.k = (SKIP & 4) ? 0 : p.k[b] - 1;                                   // scalar_step_kernel counted this step
    return sd;
}

// flat_side_load for a whole wave through the scalar cache. The wave's 64 chunks
// touch at most a few consecutive global rows (b*N + row); when they span <= 4 rows
// (WF >= ~86 floats, N >= 4, bar-batch mode), ONE s_load_dwordx16 fetches those rows'
// bars, one s_load_dwordx4 their w' and one s_load_dwordx2 the counters of the (at
// most two) envs, and each lane selects its row's values from SGPRs: no vector
// memory instruction, no texture-address work, for the side data of the stream.
// Other waves fall back to the per-lane loads. The 4-row window is clamped inside
// the arrays (rows g0 .. g0+3 with g0 <= rows - 4), so no load runs past them; the
// counter pair may read the state blob's next word (the ring follows the counters).
typedef int i16v_t __attribute__((ext_vector_type(16)));
typedef int i4v_t __attribute__((ext_vector_type(4)));
typedef int i2v_t __attribute__((ext_vector_type(2)));

struct WaveSide {
    bool ok;           // the wave's rows fit one 4-row scalar window
    bool two;          // resident series: the wave spans two envs (two days, two bar windows)
    bool nan_a, nan_b; // resident series: the env's day is outside the series
    uint32_t g0, b0;   // first row of the window, first env of the wave
    uint32_t ca;       // resident series: first asset row of env b0's bar window
    i16v_t bar16, bar16b;
    i4v_t w4;
    i2v_t k2;
};

// qa_in: the wave's first chunk, nq: chunks the wave covers (both wave-uniform)
__device__ __forceinline__ WaveSide wave_side_load(const StepParams& p, uint32_t qa_in, uint32_t nq, uint32_t qtot) {
    constexpr int F = 5;
    const int N = p.N, WF = p.W * F;
    const uint32_t per4 = (uint32_t)(N * WF) >> 2;
    const uint32_t qa = min(qa_in, qtot - 1u), qb = min(qa_in + nq - 1u, qtot - 1u);
    const uint32_t ba = fdiv(qa, p.div_units), bb = fdiv(qb, p.div_units);
    const uint32_t ga = ba * (uint32_t)N + fdiv(4u * (qa - ba * per4), p.div_wf);
    const uint32_t gb = bb * (uint32_t)N + fdiv(4u * (qb - bb * per4), p.div_wf);
    const uint32_t rows = (uint32_t)p.B * (uint32_t)N;
    WaveSide ws;
    ws.ok = gb - ga <= 3u && N >= 4 && rows >= 4u;
    ws.two = false;
    ws.nan_a = ws.nan_b = false;
    if (!ws.ok) return ws;
    ws.g0 = __builtin_amdgcn_readfirstlane(min(ga, rows - 4u));
    ws.b0 = __builtin_amdgcn_readfirstlane(ba);
    const float* bar_p = p.bar + (size_t)ws.g0 * 4;
    if (p.day) {
        // resident series: the bar rows are env b's asset rows of the series block of
        // day[b]. Env b0's window is asset rows ca .. ca+3; a wave that runs into env
        // b0+1 (at most 3 rows further: its rows there are 0 .. 2) takes that env's
        // rows 0 .. 3 of its own day as a second window. Out-of-range days load row 0
        // (never used: NaN bar).
        ws.two = bb != ba;
        ws.ca = __builtin_amdgcn_readfirstlane(min(ga - ws.b0 * (uint32_t)N, (uint32_t)N - 4u));
        const int32_t* d_p = p.day + ws.b0;
        int32_t d0, d1 = 0;
        if (ws.two) {
            i2v_t dd;
            asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=&s"(dd) : "s"(d_p) : "memory");
            d0 = dd[0];
            d1 = dd[1];
        } else {
            asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=&s"(d0) : "s"(d_p) : "memory");
        }
        ws.nan_a = d0 < 0 || d0 >= p.series_days;
        ws.nan_b = d1 < 0 || d1 >= p.series_days;
        const uint32_t ra = ws.nan_a ? 0u : (uint32_t)d0 * (uint32_t)N + ws.ca;
        bar_p = p.bar + (size_t)__builtin_amdgcn_readfirstlane(ra) * 4;
        // the second window is fetched in the same scalar batch (env b0's again when
        // the wave stays in one env)
        const uint32_t rb = ws.two && !ws.nan_b ? (uint32_t)d1 * (uint32_t)N : ra;
        const float* bar_b = p.bar + (size_t)__builtin_amdgcn_readfirstlane(rb) * 4;
        const float* w_p = p.w_new + ws.g0;
        const int32_t* k_p = p.k + ws.b0;
        asm volatile(
            "s_load_dwordx16 %0, %4, 0x0\n\t"
            "s_load_dwordx16 %1, %5, 0x0\n\t"
            "s_load_dwordx4 %2, %6, 0x0\n\t"
            "s_load_dwordx2 %3, %7, 0x0\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&s"(ws.bar16), "=&s"(ws.bar16b), "=&s"(ws.w4), "=&s"(ws.k2)
            : "s"(bar_p), "s"(bar_b), "s"(w_p), "s"(k_p)
            : "memory");
        return ws;
    }
    const float* w_p = p.w_new + ws.g0;
    const int32_t* k_p = p.k + ws.b0;
    asm volatile(
        "s_load_dwordx16 %0, %3, 0x0\n\t"
        "s_load_dwordx4 %1, %4, 0x0\n\t"
        "s_load_dwordx2 %2, %5, 0x0\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&s"(ws.bar16), "=&s"(ws.w4), "=&s"(ws.k2)       // early clobber: no output may reuse an address SGPR
        : "s"(bar_p), "s"(w_p), "s"(k_p)
        : "memory");
    return ws;
}

// two-level selects on the bits of i (0..3) with constant SGPR indices (a runtime index
// into the SGPR tuple lowers to a 16-way compare chain per value)
__device__ __forceinline__ int sel4(int i, int r0, int r1, int r2, int r3) {
    const int m1 = -(i & 1), m2 = -((i >> 1) & 1);
    const int lo = (r1 & m1) | (r0 & ~m1), hi = (r3 & m1) | (r2 & ~m1);
    return (hi & m2) | (lo & ~m2);
}

__device__ __forceinline__ f4 sel_bar(int i, const i16v_t& r) {
    return f4{__int_as_float(sel4(i, r[0], r[4], r[8], r[12])), __int_as_float(sel4(i, r[1], r[5], r[9], r[13])),
              __int_as_float(sel4(i, r[2], r[6], r[10], r[14])), __int_as_float(sel4(i, r[3], r[7], r[11], r[15]))};
}

template <int SKIP = 0>
__device__ __forceinline__ FlatSide flat_side_from_wave(const StepParams& p, const WaveSide& ws, uint32_t q) {
    if (!ws.ok) return flat_side_load<SKIP>(p, q);
    constexpr int F = 5;
    const int N = p.N, WF = p.W * F;
    const uint32_t per4 = (uint32_t)(N * WF) >> 2;
    FlatSide sd;
    const uint32_t b = fdiv(q, p.div_units);
    const uint32_t j0 = 4u * (q - b * per4);
    const uint32_t row = fdiv(j0, p.div_wf);
    sd.kk = (int)(j0 - row * (uint32_t)WF);
    const int i = (int)(b * (uint32_t)N + row - ws.g0);               // 0 .. 3
    const bool in_b = b != ws.b0;
    if (p.day) {                                                       // kernel argument: uniform
        const int ib = in_b ? (int)row : (int)(row - ws.ca);            // 0 .. 3 in the env's window
        sd.bar_nan = in_b ? ws.nan_b : ws.nan_a;
        if (!(SKIP & 1)) {
            const f4 xa = sel_bar(ib, ws.bar16);
            sd.xb = xa;
            if (ws.two) {
                const f4 xb2 = sel_bar(ib, ws.bar16b);
                sd.xb = f4{pick(in_b, xb2.x, xa.x), pick(in_b, xb2.y, xa.y), pick(in_b, xb2.z, xa.z),
                           pick(in_b, xb2.w, xa.w)};
            }
        } else {
            sd.xb = f4{1.f, 1.f, 1.f, 1.f};
        }
    } else {
        sd.bar_nan = false;
        sd.xb = (SKIP & 1) ? f4{1.f, 1.f, 1.f, 1.f} : sel_bar(i, ws.bar16);
    }
    sd.xwp = (SKIP & 2) ? 0.5f : __int_as_float(sel4(i, ws.w4[0], ws.w4[1], ws.w4[2], ws.w4[3]));
    const int mk = -(int)in_b;
    sd.k = (SKIP & 4) ? 0 : ((ws.k2[1] & mk) | (ws.k2[0] & ~mk)) - 1;   // scalar_step_kernel counted this step
    return sd;
}

// flat_side_from_wave without the bar row and w' (bar-batch mode, the wave's rows in one
// 4-row window): `ri` = the chunk's row in that window (0 .. 3), for a stream that reads
// the row's bar and w' from LDS after its barrier (flat_wg_body<..., LSIDE>, tools A/B)
__device__ __forceinline__ FlatSide flat_side_rows(const StepParams& p, const WaveSide& ws, uint32_t q, int& ri) {
    constexpr int F = 5;
    const int N = p.N, WF = p.W * F;
    const uint32_t per4 = (uint32_t)(N * WF) >> 2;
    FlatSide sd;
    const uint32_t b = fdiv(q, p.div_units);
    const uint32_t j0 = 4u * (q - b * per4);
    const uint32_t row = fdiv(j0, p.div_wf);
    sd.kk = (int)(j0 - row * (uint32_t)WF);
    ri = (int)(b * (uint32_t)N + row - ws.g0);
    sd.bar_nan = false;
    sd.xb = f4{0.f, 0.f, 0.f, 0.f};
    sd.xwp = 0.f;
    const int mk = -(int)(b != ws.b0);
    sd.k = ((ws.k2[1] & mk) | (ws.k2[0] & ~mk)) - 1;   // scalar_step_kernel counted this step
    return sd;
}

// the output chunk from the unshifted input un (chunk q) and the shifted source sh
// (floats 4q+5 .. 4q+8), per element at row position pos = kk + e (pos >= WF: the
// chunk has wrapped into the next row, whose positions 0..2 are never a last day or
// a weight slot for W >= 2, so they take the shifted value):
//   market:  last day ? bar[f] : shifted
//   weight:  shift mode: last day ? w' : shifted;  storage mode: pos == slot ? w' : own
__device__ __forceinline__ f4 flat_compose(const StepParams& p, const FlatSide& sd, const float (&un)[4],
                                           const float (&sh)[4]) {
    constexpr int F = 5;
    const int W = p.W, WF = W * F;
    const bool shift_w = !(p.ring_mode == PMENV_RING_STORAGE && sd.k >= W - 1);
    const int slot_w = (int)(((uint32_t)(1 + sd.k) - fdiv((uint32_t)(1 + sd.k), p.div_w) * (uint32_t)W) * F + (F - 1));
    int f = sd.kk - (int)fdiv((uint32_t)sd.kk, p.div_f) * F;
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int pos = sd.kk + e;
        const bool in_row = pos < WF;
        const bool lastday = in_row && pos >= WF - F;
        const bool is_w = in_row && f == F - 1;
        const float bsel = pick(sd.bar_nan, __int_as_float(0x7fc00000),
                                pick(f == 0, sd.xb.x, pick(f == 1, sd.xb.y, pick(f == 2, sd.xb.z, sd.xb.w))));
        const bool w_here = shift_w ? lastday : pos == slot_w;
        const float wv = pick(w_here, sd.xwp, pick(shift_w, sh[e], un[e]));
        v[e] = pick(is_w, wv, pick(lastday, bsel, sh[e]));
        f = f == F - 1 ? 0 : f + 1;
    }
    return f4{v[0], v[1], v[2], v[3]};
}

// flat_compose in two levels, the same values element by element: every chunk takes the
// common form — the shifted source, or (storage order, ring full) its own weight dwords —
// and only a chunk holding a row's last day or its ring slot (a divergent branch: a few
// lanes per wave instruction) fetches the row's bar and w' (`side(xb, xwp)`, NaN bar for a
// day outside the series) and patches those elements. k: the counter before the step. The
// conditions are bitwise (`&`, `|`), not short-circuit: no exec-mask branches inside the patch
// (round 6: 8,192 x 30 relay 77.5 vs 78.5 us, the same bits; profiles/r06/relay_v4/compose_v4_*).
template <typename Side>
__device__ __forceinline__ f4 compose2(const StepParams& p, int kk, int32_t k, const float (&un)[4],
                                       const float (&sh)[4], Side side) {
    constexpr int F = 5;
    const int W = p.W, WF = W * F;
    const bool shift_w = !(p.ring_mode == PMENV_RING_STORAGE && k >= W - 1);
    const int f0 = kk - (int)fdiv((uint32_t)kk, p.div_f) * F;
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int f = f0 + e >= F ? f0 + e - F : f0 + e;
        o[e] = pick(!shift_w & (f == F - 1), un[e], sh[e]);
    }
    const int slot_w = (int)(((uint32_t)(1 + k) - fdiv((uint32_t)(1 + k), p.div_w) * (uint32_t)W) * F + (F - 1));
    if ((kk + 3 >= WF - F) | (!shift_w & ((uint32_t)(slot_w - kk) <= 3u))) {   // a last day or the slot
        f4 xb;
        float xwp;
        side(xb, xwp);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int pos = kk + e;
            const int f = f0 + e >= F ? f0 + e - F : f0 + e;
            const bool in_row = pos < WF;
            const bool lastday = in_row & (pos >= WF - F);
            const float bsel = pick(f == 0, xb.x, pick(f == 1, xb.y, pick(f == 2, xb.z, xb.w)));
            o[e] = pick(lastday & (f < F - 1), bsel, o[e]);
            o[e] = pick((shift_w & lastday & (f == F - 1)) | (!shift_w & in_row & (pos == slot_w)), xwp, o[e]);
        }
    }
    return f4{o[0], o[1], o[2], o[3]};
}

template <int BLOCK, int POL>
__global__ __launch_bounds__(BLOCK) void advance_flat_kernel(StepParams p, uint32_t qtot) {
    constexpr int kAux = POL == 1 ? 2 : POL == 2 ? 3 : 0;
    const int lane = threadIdx.x & 63;
    // wave-uniform by construction; readfirstlane lets the descriptors live in SGPRs
    const uint32_t wbase = __builtin_amdgcn_readfirstlane(blockIdx.x * BLOCK + (threadIdx.x & ~63u));
    if (wbase >= qtot) return;
    const uint32_t nwave = min(64u, qtot - wbase);
    const auto rs_src = make_rsrc(p.obs + (size_t)wbase * 4, nwave * 16u);
    const f4 own = buf_load4<kAux>(rs_src, (uint32_t)lane * 16u);
    // chunks wbase+64 and wbase+65, into lanes 62 and 63 (range-checked: past the
    // tensor's end they read 0 — only last-day positions, which the bar replaces,
    // would take them)
    const uint32_t qx = wbase + 64u;
    const auto rs_ext = make_rsrc(p.obs + (size_t)qx * 4, qx < qtot ? min(2u, qtot - qx) * 16u : 0u);
    const f4 ext = buf_load4<0>(rs_ext, lane >= 62 ? (uint32_t)(lane - 62) * 16u : 0xFFFFFFF0u);
    // lanes past the tensor's end (last wave) index as its last chunk: loads stay in
    // bounds, their stores are dropped by the range check
    __builtin_amdgcn_sched_barrier(0);
    const FlatSide sd = flat_side_load(p, min(wbase + (uint32_t)lane, qtot - 1u));
    // every load is in flight before the first cross-lane move waits on one
    __builtin_amdgcn_sched_barrier(0);
    // neighbours' chunks
    const int l1 = min(lane + 1, 63) * 4, l2 = min(lane + 2, 63) * 4;
    float n1y = __int_as_float(__builtin_amdgcn_ds_bpermute(l1, __float_as_int(own.y)));
    float n1z = __int_as_float(__builtin_amdgcn_ds_bpermute(l1, __float_as_int(own.z)));
    float n1w = __int_as_float(__builtin_amdgcn_ds_bpermute(l1, __float_as_int(own.w)));
    float n2x = __int_as_float(__builtin_amdgcn_ds_bpermute(l2, __float_as_int(own.x)));
    const float x62 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ext.x), 62));
    const float y62 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ext.y), 62));
    const float z62 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ext.z), 62));
    const float w62 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ext.w), 62));
    const float x63 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ext.x), 63));
    n1y = pick(lane == 63, y62, n1y);
    n1z = pick(lane == 63, z62, n1z);
    n1w = pick(lane == 63, w62, n1w);
    n2x = pick(lane == 63, x63, pick(lane == 62, x62, n2x));
    const float sh[4] = {n1y, n1z, n1w, n2x};
    const float un[4] = {own.x, own.y, own.z, own.w};
    const auto rs_dst = make_rsrc(p.obs_out + (size_t)wbase * 4, nwave * 16u);
    buf_store4<kAux>(rs_dst, (uint32_t)lane * 16u, flat_compose(p, sd, un, sh));
}

// ---------------------------------------------------------------- K2, in place: flat stream + halo
// The same flat stream advancing the window IN PLACE. A workgroup owns chunks
// [c0, c0 + BLOCK): every lane loads its chunk into LDS, one barrier (every load of
// the workgroup lands before any of its stores), then each lane composes its chunk
// from LDS neighbours. The two chunks past the workgroup's end belong to the next
// workgroup, which may already have advanced them: they come from `halo`, a copy of
// every workgroup's first two chunks taken by the scalar step kernel of the same step
// (copy_halo below), before any advance store.
// V chunks per thread: wave w covers the contiguous chunks [c0 + 64V*w, +64V), lane
// l its chunks 64v + l, so each load and store instruction is a coalesced 1 KiB and
// the wave's side data is one scalar window.
// ABL (timing-only ablation, PMENV_ABLATE = 64 + ABL with the flat path; 0 in the
// product): flat_side_load's SKIP bits (1 bar, 2 w', 4 counter, 8 day), 16 = no halo,
// 32 = per-lane side loads instead of the wave's scalar loads, 128 = no compose (the
// shifted chunk stored as it is: PMENV_STREAM_BARE)
// OUT = true: the same workgroup body double-buffered (obs -> obs_out); the two
// chunks past the workgroup are then read straight from obs (no halo copy).
template <int BLOCK, int V, int POL, bool OUT, int ABL, bool LSIDE = false>
__device__ __forceinline__ void flat_wg_body(StepParams& p, uint32_t qtot, f4* sh4) {
    __shared__ f4 sh_side[LSIDE ? BLOCK / 64 : 1][5];   // LSIDE: per wave its 4 bar rows, then their w'
    constexpr int kAux = POL == 1 ? 2 : POL == 2 ? 3 : 0;
    constexpr int CPW = BLOCK * V;                  // chunks per workgroup
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t c0 = blockIdx.x * CPW;
    const uint32_t nblk = min((uint32_t)CPW, qtot - c0);
    const auto rs = make_rsrc(p.obs + (size_t)c0 * 4, nblk * 16u);
    f4 own[V];
#pragma unroll
    for (int v = 0; v < V; ++v) own[v] = buf_load4<kAux>(rs, (uint32_t)(64 * V * wave + 64 * v + lane) * 16u);
    // halo of this workgroup = first two chunks of the next one (none for the last)
    const uint32_t nh = blockIdx.x + 1 < gridDim.x ? min(2u, qtot - c0 - nblk) : 0u;
    const float* hsrc = OUT ? p.obs + (size_t)(c0 + nblk) * 4 : p.halo + (size_t)blockIdx.x * 8;
    const f4 hal = (ABL & 16) ? own[0] : buf_load4<0>(make_rsrc(hsrc, nh * 16u),
                                                      tid < 2 ? (uint32_t)tid * 16u : 0xFFFFFFF0u);
    // the window and halo loads go out before anything else (a halo issued after the
    // own chunk's wait costs every workgroup a second memory round trip)
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t qw = __builtin_amdgcn_readfirstlane(c0 + (uint32_t)(64 * V * wave));
    WaveSide ws;
    ws.ok = false;
    if (!(ABL & 32)) ws = wave_side_load(p, qw, 64u * V, qtot);
    const bool lside = LSIDE && ABL == 0 && ws.ok && !p.day;
    if (lside && lane == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
            sh_side[wave][r] = f4{__int_as_float(ws.bar16[4 * r]), __int_as_float(ws.bar16[4 * r + 1]),
                                  __int_as_float(ws.bar16[4 * r + 2]), __int_as_float(ws.bar16[4 * r + 3])};
        sh_side[wave][4] = f4{__int_as_float(ws.w4[0]), __int_as_float(ws.w4[1]), __int_as_float(ws.w4[2]),
                              __int_as_float(ws.w4[3])};
    }
    FlatSide sd[V];
    int ri[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const uint32_t q = min(qw + 64u * v + lane, qtot - 1u);
        if (lside) sd[v] = flat_side_rows(p, ws, q, ri[v]);
        else sd[v] = flat_side_from_wave<ABL & 15>(p, ws, q);
    }
#pragma unroll
    for (int v = 0; v < V; ++v) sh4[64 * V * wave + 64 * v + lane] = own[v];
    if (tid < 2) sh4[CPW + tid] = hal;
    __syncthreads();
    const auto rd = OUT ? make_rsrc(p.obs_out + (size_t)c0 * 4, nblk * 16u) : rs;
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int j = 64 * V * wave + 64 * v + lane;
        if (lside) {
            sd[v].xb = sh_side[wave][ri[v]];
            sd[v].xwp = reinterpret_cast<const float*>(&sh_side[wave][4])[ri[v]];
        }
        const f4 n1 = sh4[j + 1], n2 = sh4[j + 2];
        const float sh[4] = {n1.y, n1.z, n1.w, n2.x};
        const float un[4] = {own[v].x, own[v].y, own[v].z, own[v].w};
        if (ABL & 128) buf_store4<kAux>(rd, (uint32_t)j * 16u, f4{sh[0], sh[1], sh[2], sh[3]});   // timing only
        else buf_store4<kAux>(rd, (uint32_t)j * 16u, flat_compose(p, sd[v], un, sh));
    }
}

// The same workgroup body with a two-level compose. Every chunk takes the common form —
// its shifted source, or (storage order, ring full) its own weight dwords — and only the
// chunks holding a row's last day or its ring slot patch those elements from the row's bar
// and w' (a divergent branch a few lanes per wave instruction take). The workgroup's rows'
// bar, w' and counter come into LDS before the barrier, one row per thread (per-lane
// loads: no scalar window, no per-chunk selects). The same values as flat_compose, element
// by element: the common form is flat_compose's result wherever neither a last day nor the
// slot is involved, and the patch applies flat_compose's rule to exactly those elements.
// Needs at most BLOCK rows per workgroup: 4 V <= W F (W >= 2 at V = 2: the flat stream's
// shape rule, pmenv.hip).
template <int BLOCK, int V, int POL, bool OUT>
__device__ __forceinline__ void flat_wg_body_patch(StepParams& p, uint32_t qtot, f4* sh4) {
    constexpr int kAux = POL == 1 ? 2 : POL == 2 ? 3 : 0;
    constexpr int CPW = BLOCK * V, F = 5;
    __shared__ f4 sh_bar[BLOCK];
    __shared__ float sh_wp[BLOCK];
    __shared__ int32_t sh_kc[BLOCK];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t c0 = blockIdx.x * CPW;
    const uint32_t nblk = min((uint32_t)CPW, qtot - c0);
    const auto rs = make_rsrc(p.obs + (size_t)c0 * 4, nblk * 16u);
    f4 own[V];
#pragma unroll
    for (int v = 0; v < V; ++v) own[v] = buf_load4<kAux>(rs, (uint32_t)(64 * V * wave + 64 * v + lane) * 16u);
    const uint32_t nh = blockIdx.x + 1 < gridDim.x ? min(2u, qtot - c0 - nblk) : 0u;
    const float* hsrc = OUT ? p.obs + (size_t)(c0 + nblk) * 4 : p.halo + (size_t)blockIdx.x * 8;
    const f4 hal = buf_load4<0>(make_rsrc(hsrc, nh * 16u), tid < 2 ? (uint32_t)tid * 16u : 0xFFFFFFF0u);
    __builtin_amdgcn_sched_barrier(0);
    // the workgroup's rows g_lo .. g_hi (global row = b N + n): thread t stages row g_lo + t
    const int N = p.N, W = p.W, WF = W * F;
    const uint32_t per4 = (uint32_t)(N * WF) >> 2;
    const uint32_t b_lo = fdiv(c0, p.div_units);
    const uint32_t g_lo = b_lo * (uint32_t)N + fdiv(4u * (c0 - b_lo * per4), p.div_wf);
    const uint32_t ql = c0 + nblk - 1u;
    const uint32_t b_hi = fdiv(ql, p.div_units);
    const uint32_t g_hi = b_hi * (uint32_t)N + fdiv(4u * (ql - b_hi * per4) + 3u, p.div_wf);
    if ((uint32_t)tid <= g_hi - g_lo) {
        const uint32_t g = g_lo + (uint32_t)tid;
        const uint32_t b = g / (uint32_t)N, n = g - b * (uint32_t)N;
        const float* barb = env_bar(p, (int)b);                     // null: a day outside the series
        const float nanv = __int_as_float(0x7fc00000);
        sh_bar[tid] = barb ? *reinterpret_cast<const f4*>(barb + (size_t)n * 4) : f4{nanv, nanv, nanv, nanv};
        sh_wp[tid] = p.w_new[g];
        sh_kc[tid] = p.k[b] - 1;                                     // scalar_step_kernel counted this step
    }
#pragma unroll
    for (int v = 0; v < V; ++v) sh4[64 * V * wave + 64 * v + lane] = own[v];
    if (tid < 2) sh4[CPW + tid] = hal;
    __syncthreads();
    const auto rd = OUT ? make_rsrc(p.obs_out + (size_t)c0 * 4, nblk * 16u) : rs;
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int j = 64 * V * wave + 64 * v + lane;
        const uint32_t q = min(c0 + (uint32_t)j, qtot - 1u);
        const uint32_t b = fdiv(q, p.div_units);
        const uint32_t j0 = 4u * (q - b * per4);
        const uint32_t row = fdiv(j0, p.div_wf);
        const int kk = (int)(j0 - row * (uint32_t)WF);
        const int t = (int)(b * (uint32_t)N + row - g_lo);
        const f4 n1 = sh4[j + 1], n2 = sh4[j + 2];
        const float sh[4] = {n1.y, n1.z, n1.w, n2.x};
        const float un[4] = {own[v].x, own[v].y, own[v].z, own[v].w};
        const f4 o = compose2(p, kk, sh_kc[t], un, sh, [&](f4& xb, float& xwp) {
            xb = sh_bar[t];
            xwp = sh_wp[t];
        });
        buf_store4<kAux>(rd, (uint32_t)j * 16u, o);
    }
}

// The in-place flat stream: the two-level compose in the product (ABL = 0); the tools
// build's timing-only ablations run the per-element compose with their SKIP bits.
// Round 3, in-process interleaved against the per-element compose, the same bits:
// 8,192 x 30 81.5 vs 82.8 us, 65,536 x 30 637.0 vs 646.5, double-buffered 84.6 vs 87.1 and
// 641.8 vs 648.5; 4,096 x 30, 8,192 x 16, 16,384 x 8, 4,096 x 48 within 0.3 %
// (profiles/ab_r03/patch_r03p.err)
template <int BLOCK, int V, int POL, int ABL = 0>
__global__ __launch_bounds__(BLOCK) void advance_flat_inplace_kernel(StepParams p, uint32_t qtot) {
    __shared__ f4 sh4[BLOCK * V + 2];
    if constexpr (ABL == 0) flat_wg_body_patch<BLOCK, V, POL, false>(p, qtot, sh4);
    else flat_wg_body<BLOCK, V, POL, false, ABL>(p, qtot, sh4);
}

// tools A/B: the in-place / double-buffered stream with the per-element compose
template <int BLOCK, int V, int POL>
__global__ __launch_bounds__(BLOCK) void advance_flat_inplace_perelem_kernel(StepParams p, uint32_t qtot) {
    __shared__ f4 sh4[BLOCK * V + 2];
    flat_wg_body<BLOCK, V, POL, false, 0>(p, qtot, sh4);
}
template <int BLOCK, int V, int POL>
__global__ __launch_bounds__(BLOCK) void advance_flat_wg_perelem_kernel(StepParams p, uint32_t qtot) {
    __shared__ f4 sh4[BLOCK * V + 2];
    flat_wg_body<BLOCK, V, POL, true, 0>(p, qtot, sh4);
}

// tools A/B: the stream reading each chunk's bar and w' from LDS rows staged per wave
template <int BLOCK, int V, int POL>
__global__ __launch_bounds__(BLOCK) void advance_flat_inplace_lside_kernel(StepParams p, uint32_t qtot) {
    __shared__ f4 sh4[BLOCK * V + 2];
    flat_wg_body<BLOCK, V, POL, false, 0, true>(p, qtot, sh4);
}

// the same kernel held to 80 SGPRs (8 waves per SIMD instead of 7; tools A/B)
template <int BLOCK, int V, int POL>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_num_sgpr(80))) void advance_flat_inplace_s80_kernel(
    StepParams p, uint32_t qtot) {
    __shared__ f4 sh4[BLOCK * V + 2];
    flat_wg_body<BLOCK, V, POL, false, 0>(p, qtot, sh4);
}

// the double-buffered twin of advance_flat_inplace_kernel (same body, OUT = true)
template <int BLOCK, int V, int POL>
__global__ __launch_bounds__(BLOCK) void advance_flat_wg_kernel(StepParams p, uint32_t qtot) {
    __shared__ f4 sh4[BLOCK * V + 2];
    flat_wg_body_patch<BLOCK, V, POL, true>(p, qtot, sh4);
}

// Taken by the scalar step kernels before the in-place flat advance of the same step:
// halo[i] = chunks (i+1)*B_flat and (i+1)*B_flat + 1 of the window (0 past its end).
__device__ __forceinline__ void copy_halo(const StepParams& p) {
    if (!p.halo) return;
    const uint32_t nthr = gridDim.x * blockDim.x;
    const f4* src = reinterpret_cast<const f4*>(p.obs);
    f4* dst = reinterpret_cast<f4*>(p.halo);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < p.halo_wgs; i += nthr) {
        const uint32_t q = halo_src(p, i);
        dst[2 * i] = q < p.halo_qtot ? src[q] : f4{0.f, 0.f, 0.f, 0.f};
        dst[2 * i + 1] = q + 1 < p.halo_qtot ? src[q + 1] : f4{0.f, 0.f, 0.f, 0.f};
    }
}

// ---------------------------------------------------------------- K2 for F != 5: the generic stream
// The two-launch step's window stream for the channel counts the F = 5 streams do not take
// (2 <= F <= 16, F != 5; 16-B granular env windows): flat_wg_body_patch's workgroup layout —
// BLOCK x V chunks of the flat [B, N, W, F] tensor staged in LDS, the HC chunks past the
// workgroup that a shift by F floats reads (two for F <= 8, four up to 16: FMAX — the
// reference loader's width grows past 8 with every indicator of config/base.py:30-44,
// data/data_loader.py:48) read from `halo` in place (copied by the scalar step of the same step) or from
// obs double-buffered — with the shift by F floats read from LDS dword-wise and every
// element composed from its own (day, channel) (weight_buffer.py:32-44, instrument.py:339-356):
//   market f < F-1:  t < W-1 ? in[n, t+1, f] : bar[n, f]
//   weight f = F-1:  shift order ? (t < W-1 ? in[n, t+1, F-1] : w'[n])
//                                : (t == slot ? w'[n] : in[n, t, F-1])
// The workgroup's rows' bar (F - 1 floats, NaN for a day outside the series), w' and
// counter come into LDS before the barrier, one row per thread (at most BLOCK rows per
// workgroup: the plan's rule 4 V BLOCK / (W F) + 2 <= BLOCK). An env window is a whole
// number of chunks, so a chunk spans at most two rows of one env.
// SHV: the shifted source's LDS reads — 4 (F % 4 == 0: one 16-B read), 2 (F % 4 == 2: two
// 8-B reads), 1 (dword reads). TWO (the product): the two-level compose of flat_wg_body_patch —
// every chunk takes the common form (the shifted source, or in place its own weight float once
// the storage-order ring is full), and only chunks holding a row's last day or its ring slot
// (a divergent branch) read the rows' bar / w' / slot and compose element by element; TWO =
// false (tools build): every element composed from its row's LDS values. The same values.
// POL: the window stream's cache policy (the own-chunk loads and the stores), as the F = 5
// streams: 0 default, 1 nt (windows past the Infinity Cache). ABL (tools build, timing
// only): 1 no side-data loads, 2 no compose (the shifted source stored), 4 no shifted read.
template <int BLOCK, int V, bool OUT, int SHV = 1, bool TWO = true, int POL = 0, int ABL = 0, int FMAX = 8>
__global__ __launch_bounds__(BLOCK) void advance_gen_kernel(StepParams p, uint32_t qtot, uint32_t rows) {
    constexpr int kAux = POL == 1 ? 2 : 0;
    constexpr int CPW = BLOCK * V;
    constexpr int kFm = FMAX - 1;                            // bar floats per staged row (F <= FMAX)
    constexpr int HC = FMAX > 8 ? 4 : 2;                     // chunks past the workgroup the shift reads
    static_assert(FMAX == 8 || FMAX == 16, "F <= 8: two chunks past a workgroup; F <= 16: four");
    __shared__ f4 sh4[CPW + HC];
    // the rows' side data, sized by the plan's bound on rows per workgroup (4 CPW / (W F) + 2:
    // a dozen at W F = 400) rather than BLOCK — more workgroups per CU, more bytes in flight
    extern __shared__ float gside[];
    float* sh_wp = gside;                                    // [rows] w'
    int32_t* sh_sl = reinterpret_cast<int32_t*>(gside + rows);   // [rows] ring slot, or -1 while it shifts
    float* sh_bar = gside + 2 * rows;                        // [rows][kFm] bar
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t c0 = blockIdx.x * CPW;
    const uint32_t nblk = min((uint32_t)CPW, qtot - c0);
    const auto rs = make_rsrc(p.obs + (size_t)c0 * 4, nblk * 16u);
    f4 own[V];
#pragma unroll
    for (int v = 0; v < V; ++v) own[v] = buf_load4<kAux>(rs, (uint32_t)(64 * V * wave + 64 * v + lane) * 16u);
    // (no halo buffer in place: nothing is read, the HC chunks stay 0)
    const uint32_t nh = blockIdx.x + 1 < gridDim.x && (OUT || p.halo) ? min((uint32_t)HC, qtot - c0 - nblk) : 0u;
    const float* hsrc = OUT ? p.obs + (size_t)(c0 + nblk) * 4 : (p.halo ? p.halo + (size_t)blockIdx.x * 4 * HC : p.obs);
    const f4 hal = buf_load4<0>(make_rsrc(hsrc, nh * 16u), tid < HC ? (uint32_t)tid * 16u : 0xFFFFFFF0u);
    __builtin_amdgcn_sched_barrier(0);
    const int N = p.N, W = p.W, F = p.F, Fm = F - 1, WF = W * F;
    const uint32_t per4 = (uint32_t)(N * WF) >> 2;
    const uint32_t b_lo = fdiv(c0, p.div_units);
    const uint32_t g_lo = b_lo * (uint32_t)N + fdiv(4u * (c0 - b_lo * per4), p.div_wf);
    const uint32_t ql = c0 + nblk - 1u;
    const uint32_t b_hi = fdiv(ql, p.div_units);
    const uint32_t g_hi = b_hi * (uint32_t)N + fdiv(4u * (ql - b_hi * per4) + 3u, p.div_wf);
    if ((ABL & 1) && (uint32_t)tid <= g_hi - g_lo) {
#pragma unroll
        for (int f = 0; f < kFm; ++f) sh_bar[tid * kFm + f] = 0.0f;
        sh_wp[tid] = 0.0f;
        sh_sl[tid] = -1;
    } else if ((uint32_t)tid <= g_hi - g_lo) {
        const uint32_t g = g_lo + (uint32_t)tid;
        const uint32_t b = g / (uint32_t)N, n = g - b * (uint32_t)N;
        const float* barb = env_bar(p, (int)b);                     // null: a day outside the series
        // plain per-lane loads: a buffer resource built from a per-lane base costs a
        // readfirstlane loop per load, each with its own wait (584 -> 396 us at F = 3, r05ga)
        const float* rowp = barb + (size_t)n * Fm;
        float x[kFm];
#pragma unroll
        for (int f = 0; f < kFm; ++f) x[f] = f < Fm && barb ? rowp[f] : __int_as_float(0x7fc00000);
#pragma unroll
        for (int f = 0; f < kFm; ++f) sh_bar[tid * kFm + f] = x[f];
        sh_wp[tid] = p.w_new[g];
        const int32_t kc = p.k[b] - 1;                               // the scalar step counted this step
        const bool shift_w = !(p.ring_mode == PMENV_RING_STORAGE && kc >= W - 1);
        sh_sl[tid] = shift_w ? -1 : (int)((uint32_t)(1 + kc) - fdiv((uint32_t)(1 + kc), p.div_w) * (uint32_t)W);
    }
#pragma unroll
    for (int v = 0; v < V; ++v) sh4[64 * V * wave + 64 * v + lane] = own[v];
    if (tid < HC) sh4[CPW + tid] = hal;
    __syncthreads();
    const float* shf = reinterpret_cast<const float*>(sh4);
    const auto rd = OUT ? make_rsrc(p.obs_out + (size_t)c0 * 4, nblk * 16u) : rs;
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int j = 64 * V * wave + 64 * v + lane;
        const uint32_t q = min(c0 + (uint32_t)j, qtot - 1u);
        const uint32_t b = fdiv(q, p.div_units);
        const uint32_t j0 = 4u * (q - b * per4);
        const uint32_t row = fdiv(j0, p.div_wf);
        const uint32_t kk = j0 - row * (uint32_t)WF;
        const int t0 = (int)fdiv(kk, p.div_f);
        const int f0 = (int)kk - t0 * F;
        const int r0 = (int)(b * (uint32_t)N + row - g_lo);          // the chunk's first row in the workgroup
        const float un[4] = {own[v].x, own[v].y, own[v].z, own[v].w};
        const float* src = shf + 4 * j + F;                           // floats 4j+F .. 4j+F+3
        float sh[4];
        if constexpr ((ABL & 4) != 0) {
            sh[0] = un[0]; sh[1] = un[1]; sh[2] = un[2]; sh[3] = un[3];
        } else if constexpr (SHV == 4) {
            const f4 x = *reinterpret_cast<const f4*>(src);
            sh[0] = x.x; sh[1] = x.y; sh[2] = x.z; sh[3] = x.w;
        } else if constexpr (SHV == 2) {
            typedef float f2 __attribute__((ext_vector_type(2)));
            const f2 x0 = *reinterpret_cast<const f2*>(src), x1 = *reinterpret_cast<const f2*>(src + 2);
            sh[0] = x0.x; sh[1] = x0.y; sh[2] = x1.x; sh[3] = x1.y;
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) sh[e] = src[e];
        }
        float o[4];
        bool patch = true;
        int sl0 = 0;
        if constexpr (TWO) {
            sl0 = sh_sl[r0];
            int f = f0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                o[e] = sl0 >= 0 && f == Fm ? un[e] : sh[e];
                f = f == Fm ? 0 : f + 1;
            }
            // a last day (every chunk that reaches the row's end holds one) or the ring slot
            patch = (int)kk + 3 >= WF - F || (sl0 >= 0 && (uint32_t)(sl0 * F + Fm - (int)kk) <= 3u);
        }
        if constexpr ((ABL & 2) != 0) {
            o[0] = sh[0]; o[1] = sh[1]; o[2] = sh[2]; o[3] = sh[3];
            patch = false;
        }
        if (patch) {
            const int r1 = min(r0 + 1, (int)rows - 1);
            if constexpr (!TWO) sl0 = sh_sl[r0];
            const int sl1 = sh_sl[r1];
            const float wp0 = sh_wp[r0], wp1 = sh_wp[r1];
            int t = t0, f = f0;
            bool nx = false;                                          // past the first row's end
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int slot = nx ? sl1 : sl0;
                const float wp = nx ? wp1 : wp0;
                const bool last = t == W - 1;
                const float bf = last && f < Fm ? sh_bar[(r0 + (nx ? 1 : 0)) * kFm + f] : 0.0f;
                const float wv = slot < 0 ? (last ? wp : sh[e]) : (t == slot ? wp : un[e]);
                o[e] = f == Fm ? wv : (last ? bf : sh[e]);
                // the next element: channel, day, row
                const bool fw = f == Fm;
                f = fw ? 0 : f + 1;
                t += fw ? 1 : 0;
                const bool tw = t == W;
                t = tw ? 0 : t;
                nx = nx || tw;
            }
        }
        buf_store4<kAux>(rd, (uint32_t)j * 16u, f4{o[0], o[1], o[2], o[3]});
    }
}

// ---------------------------------------------------------------- single-launch fallback
// The whole step in one workgroup per env with the obs staged through an LDS tile
// (rows of any length up to kTileFloats, any F >= 2, any alignment).
template <int BLOCK, int MAXV, bool VEC>
__device__ __forceinline__ void stage_tile(const float* __restrict__ src, float* lds, int nf, int tid) {
    if (VEC) {
        f4 reg[MAXV];
        const int nq = nf >> 2;
#pragma unroll
        for (int i = 0; i < MAXV; ++i) {
            int q = tid + i * BLOCK;
            reg[i] = q < nq ? reinterpret_cast<const f4*>(src)[q] : f4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int i = 0; i < MAXV; ++i) {
            int q = tid + i * BLOCK;
            if (q < nq) reinterpret_cast<f4*>(lds)[q] = reg[i];
        }
    } else {
        float reg[MAXV * 4];
#pragma unroll
        for (int i = 0; i < MAXV * 4; ++i) {
            int j = tid + i * BLOCK;
            reg[i] = j < nf ? src[j] : 0.0f;
        }
#pragma unroll
        for (int i = 0; i < MAXV * 4; ++i) {
            int j = tid + i * BLOCK;
            if (j < nf) lds[j] = reg[i];
        }
    }
}

template <bool VEC>
__global__ __launch_bounds__(kBlock) void step_advance_lds_kernel(StepParams p) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int N = p.N, W = p.W, F = p.F, Fm = F - 1;
    const int WF = W * F;
    const int R = p.rows_per_tile;
    Scratch s = carve(lds, p.tile_floats, N, F);
    float* obs = p.obs + (size_t)b * N * WF;

    const float* barg = env_bar(p, b);
    for (int i = tid; i < N * Fm; i += kBlock) s.bar[i] = barg ? barg[i] : NAN;
    if (tid < 64) {
        const int32_t k = p.k[b];
        const double v_prev = p.value[b];
        gather_inputs(p, b, s, k);
        scalar_compute(p, b, s, k, v_prev);
    }
    __syncthreads();
    const int shift_w = s.ints[0];
    const int slot = s.ints[1];

    for (int r0 = 0; r0 < N; r0 += R) {
        const int rows = min(R, N - r0);
        const int nf = rows * WF;
        if (r0 > 0) __syncthreads();
        stage_tile<kBlock, kMaxVec, VEC>(obs + (size_t)r0 * WF, lds, nf, tid);
        __syncthreads();
        float* dst = p.obs_out + (size_t)b * N * WF + (size_t)r0 * WF;
        for (int j = tid; j < nf; j += kBlock) {
            uint32_t row = fdiv((uint32_t)j, p.div_wf);
            uint32_t kk = (uint32_t)j - row * (uint32_t)WF;
            uint32_t t = fdiv(kk, p.div_f);
            uint32_t f = kk - t * (uint32_t)F;
            const int n = r0 + (int)row;
            const bool lastday = (int)t == W - 1;
            int idx;
            if ((int)f == F - 1)
                idx = shift_w ? (lastday ? s.wp_off + n : j + F) : ((int)t == slot ? s.wp_off + n : j);
            else
                idx = lastday ? s.bar_off + n * Fm + (int)f : j + F;
            dst[j] = lds[idx];
        }
    }
}

// ---------------------------------------------------------------- register step (any F, any alignment)
// The whole advance-mode step in one workgroup per env, for the windows the 16-B streams do
// not take (F != 5, or env windows that are not 16-B granular: config 1's 1 x 5 x 50 x 5 is
// 250 floats per asset row) with at most BLOCK x E floats per env. Every float the step reads
// is loaded straight into VGPRs, before the scalar step: thread i owns floats j = i + BLOCK e
// of the env's [N, W, F] block and loads in[j + F] (the same row's next day), or on the last
// day the bar's [n, f] (f < F-1); for the weight channel in[j + F] while the ring shifts and
// in[j] once the storage-order ring is full (it then stays in place) — the one read that
// waits for the step counter (a scalar load issued with the market loads).
// Wave 0 runs the env's scalar step meanwhile (N <= 64: the register form, one asset per lane,
// its state writes and reward after the window's stores as in step_env_kernel; wider envs the
// LDS-scratch form of gather_inputs / scalar_compute); every wave then waits for its loads to have RETURNED
// (vmcnt(0)) before the barrier, which closes the in-place read-before-write window of the
// env — one workgroup owns one env, no other workgroup touches it — and composes and stores
// dword-wise. Replaces step_advance_lds_kernel's stage-through-LDS rounds (two barriers per
// row tile, the window loads issued only after the scalar step) for these shapes.
template <int BLOCK, int E, bool REG>
__global__ __launch_bounds__(BLOCK) void step_small_kernel(StepParams p) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    __shared__ float sh_wp[REG ? 64 : 1];
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int N = p.N, W = p.W, F = p.F, Fm = F - 1;
    const uint32_t WF = (uint32_t)(W * F), NWF = (uint32_t)N * WF;
    constexpr uint32_t kOut = 0x80000000u;                // a byte offset past every buffer: reads 0, stores nothing
    Scratch s = carve(lds, 0, N, F);
    const auto rs_in = make_rsrc(p.obs + (size_t)b * NWF, NWF * 4u);
    const auto rs_out = make_rsrc(p.obs_out + (size_t)b * NWF, NWF * 4u);
    const float* barg = env_bar(p, b);                    // null: a day outside the series (NaN bar)
    const auto rs_bar = make_rsrc(barg ? barg : p.obs, barg ? (uint32_t)(N * Fm) * 4u : 0u);
    const float nanv = __int_as_float(0x7fc00000);
    // the step counter as a lane value, read at a lane-varying zero offset: a load the compiler
    // sees as uniform has its value moved to an SGPR right after it is issued, and the wait for
    // that held every load below back by one memory round trip
    uint32_t z = 0u;
    asm volatile("" : "+v"(z));
    ScalarIn sin;
    int32_t k0;
    if constexpr (REG) {
        sin = scalar_load<64, true>(p, b, tid, z);        // every wave (lane % 64 = asset): no branch before the window loads
        k0 = sin.k;
    } else {
        k0 = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(make_rsrc(p.k + b, 4u), z, 0, 0);
    }
    // thread i owns floats j = i + BLOCK e; small E keeps their (row, day, channel) in registers
    // for the stores, large E recomputes them (fewer live registers)
    constexpr bool BOTH = E <= 8;
    uint32_t xr[BOTH ? E : 1], xt[BOTH ? E : 1], xf[BOTH ? E : 1];
    auto decomp = [&](uint32_t j, uint32_t& row, uint32_t& t, uint32_t& f) {
        row = fdiv(j, p.div_wf);
        const uint32_t kk = j - row * WF;
        t = fdiv(kk, p.div_f);
        f = kk - t * (uint32_t)F;
    };
    float src[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {                         // the market channels: in[j + F] or the bar
        const uint32_t j = (uint32_t)tid + (uint32_t)(BLOCK * e);
        uint32_t row, t, f;
        decomp(j, row, t, f);
        if constexpr (BOTH) {
            xr[e] = row;
            xt[e] = t;
            xf[e] = f;
        }
        const bool mkt = j < NWF && (int)f < Fm, last = (int)t == W - 1;
        const float sh = buf_load1(rs_in, mkt && !last ? (j + (uint32_t)F) * 4u : kOut);
        const float bv = buf_load1(rs_bar, mkt && last ? (row * (uint32_t)Fm + f) * 4u : kOut);
        src[e] = last ? (barg ? bv : nanv) : sh;
    }
    // the weight channel: shifted with the window until the ring is full, then (storage order)
    // in place (weight_buffer.py:32-44). Small E: both candidates are read at once (no wait for
    // the counter, one memory round trip); large E: the counter picks the one float to read
    // (half the registers, the weight loads a round trip later)
    float cur[BOTH ? E : 1];
    const bool shift_w = p.ring_mode == PMENV_RING_CHRONO || k0 < W - 1;
    uint32_t tid2 = (uint32_t)tid;
    asm volatile("" : "+v"(tid2));                        // recompute the indices, do not keep E of them live
#pragma unroll
    for (int e = 0; e < E; ++e) {
        if constexpr (BOTH) {
            const uint32_t j = (uint32_t)tid + (uint32_t)(BLOCK * e);
            const bool wch = j < NWF && (int)xf[e] == Fm;
            const float ws = buf_load1(rs_in, wch && (int)xt[e] < W - 1 ? (j + (uint32_t)F) * 4u : kOut);
            cur[e] = buf_load1(rs_in, wch ? j * 4u : kOut);
            src[e] = wch ? ws : src[e];
        } else {
            const uint32_t j = tid2 + (uint32_t)(BLOCK * e);
            uint32_t row, t, f;
            decomp(j, row, t, f);
            const bool wch = j < NWF && (int)f == Fm;
            const uint32_t off = !wch ? kOut : !shift_w ? j * 4u : (int)t < W - 1 ? (j + (uint32_t)F) * 4u : kOut;
            const float wv = buf_load1(rs_in, off);
            src[e] = wch ? wv : src[e];
        }
    }
    ScalarMid mid;
    if (REG) {
        if (tid < 64) {
            mid = scalar_core<64>(p, b, tid, sin);
            sh_wp[tid] = mid.wp;
        }
    } else if (tid < 64) {
        const double v_prev = p.value[b];
        gather_inputs(p, b, s, k0);
        scalar_compute(p, b, s, k0, v_prev);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");              // this wave's window reads are in
    __syncthreads();
    const int slot = ring_slot(k0, W);
    const float* wps = REG ? sh_wp : s.wp;
    uint32_t tid3 = (uint32_t)tid;
    asm volatile("" : "+v"(tid3));
#pragma unroll
    for (int e = 0; e < E; ++e) {
        uint32_t j, row, t, f;
        if constexpr (BOTH) {
            j = (uint32_t)tid + (uint32_t)(BLOCK * e);
            row = xr[e];
            t = xt[e];
            f = xf[e];
        } else {
            j = tid3 + (uint32_t)(BLOCK * e);
            decomp(j, row, t, f);
        }
        // branch-free: every lane reads a w' (its row clamped), the selects pick
        const float v = src[e];
        const float wp = wps[min(row, (uint32_t)N - 1u)];
        const float kept = BOTH ? cur[e] : v;
        const float wv = pick(shift_w, pick((int)t == W - 1, wp, v), pick((int)t == slot, wp, kept));
        const float o = pick((int)f == Fm && j < NWF, wv, v);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o), rs_out, j < NWF ? j * 4u : kOut, 0, 0);
    }
    // the state writes and the reward after the window's stores (the barrier waited for the core only)
    if (REG && tid < 64) scalar_tail<64>(p, b, tid, sin, mid);
}

// The register step for the smallest windows (env windows of at most BLOCK x E floats, E <= 8,
// N <= 64: config 1's 1 x 5 x 50 x 5), staged through LDS: every thread issues its 16-B loads
// of the env block (dword-aligned: env windows need not be 16-B granular) and the bar, all
// with the scalar step's loads and none waiting for another; wave 0 runs the whole scalar
// step up to the reward while they are in flight (the return, log and statistics included:
// only stores are left after the barrier); the window's floats then come from LDS — the
// shifted source at j + F, the own weight float at j — and leave as coalesced dword stores,
// followed by the state's stores. A quarter of step_small_kernel's load instructions per
// wave, and no f64 tail after the window's stores. Same values, element by element.
template <int BLOCK, int E>
__global__ __launch_bounds__(BLOCK) void step_tiny_kernel(StepParams p) {
    static_assert(E % 4 == 0 && E <= 8 && BLOCK >= 256, "16-B chunks, at most two per thread");
    constexpr int Q = E / 4;                               // chunks per thread
    extern __shared__ __attribute__((aligned(16))) float lds[];   // [NWF + 8] window | [N (F-1)] bar
    __shared__ float sh_wp[64];
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int N = p.N, W = p.W, F = p.F, Fm = F - 1;
    const uint32_t WF = (uint32_t)(W * F), NWF = (uint32_t)N * WF, nq = NWF >> 2;
    constexpr uint32_t kOut = 0x80000000u;
    const auto rs_in = make_rsrc(p.obs + (size_t)b * NWF, NWF * 4u);
    const auto rs_out = make_rsrc(p.obs_out + (size_t)b * NWF, NWF * 4u);
    const float* barg = env_bar(p, b);                     // null: a day outside the series (NaN bar)
    const uint32_t nbar = (uint32_t)(N * Fm);
    const auto rs_bar = make_rsrc(barg ? barg : p.obs, barg ? nbar * 4u : 0u);
    uint32_t z = 0u;
    asm volatile("" : "+v"(z));
    const ScalarIn sin = scalar_load<64, true>(p, b, tid, z);   // every wave: no branch before the loads
    f4 ch[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const uint32_t c = (uint32_t)tid + (uint32_t)(BLOCK * q);
        ch[q] = buf_load4<0>(rs_in, c < nq ? c * 16u : kOut);
    }
    const uint32_t jt = nq * 4u + (uint32_t)tid;            // the block's last NWF % 4 floats
    const float tl = buf_load1(rs_in, jt < NWF ? jt * 4u : kOut);
    // the bar: N (F - 1) <= 2 BLOCK floats (the plan: pmenv.hip), two per thread
    const float bv0 = buf_load1(rs_bar, (uint32_t)tid < nbar ? (uint32_t)tid * 4u : kOut);
    const float bv1 = buf_load1(rs_bar, (uint32_t)(tid + BLOCK) < nbar ? (uint32_t)(tid + BLOCK) * 4u : kOut);
    float* lbar = lds + NWF + 8;
    const int32_t k0 = sin.k;
    ScalarMid mid;
    double ret = 0.0, rwd = 0.0, sa = sin.sa, sb = sin.sb;
    bool stats = false;
    if (tid < 64) {
        mid = scalar_core<64>(p, b, tid, sin);
        sh_wp[tid] = mid.wp;
        ret = step_ret(p, sin, mid);
        rwd = step_reward(p, mid.k, ret, sa, sb, stats);
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const uint32_t c = (uint32_t)tid + (uint32_t)(BLOCK * q);
        if (c < nq) reinterpret_cast<f4*>(lds)[c] = ch[q];
    }
    if (jt < NWF + 8u) lds[jt] = jt < NWF ? tl : 0.0f;      // and 8 floats past the block (read only by last days)
    if ((uint32_t)tid < nbar) lbar[tid] = barg ? bv0 : __int_as_float(0x7fc00000);
    if ((uint32_t)(tid + BLOCK) < nbar) lbar[tid + BLOCK] = barg ? bv1 : __int_as_float(0x7fc00000);
    // every load of every wave has returned before any store: the counter the waves past the
    // first read (for the ring slot) is one wave 0 rewrites after the barrier
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const bool shift_w = p.ring_mode == PMENV_RING_CHRONO || k0 < W - 1;
    const int slot = ring_slot(k0, W);
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const uint32_t j = (uint32_t)tid + (uint32_t)(BLOCK * e);
        const uint32_t jc = j < NWF ? j : 0u;
        const uint32_t row = fdiv(jc, p.div_wf);
        const uint32_t kk = jc - row * WF;
        const uint32_t t = fdiv(kk, p.div_f);
        const int f = (int)(kk - t * (uint32_t)F);
        const bool last = (int)t == W - 1;
        const float sh = lds[jc + (uint32_t)F];
        const float un = lds[jc];
        const float wp = sh_wp[row];
        const float bf = lbar[row * (uint32_t)Fm + (uint32_t)min(f, Fm - 1 < 0 ? 0 : Fm - 1)];
        const float wv = shift_w ? (last ? wp : sh) : ((int)t == slot ? wp : un);
        const float o = f == Fm ? wv : (last ? bf : sh);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o), rs_out, j < NWF ? j * 4u : kOut, 0, 0);
    }
    // the state's stores (scalar_tail's, the reward computed before the barrier)
    if (tid < 64) {
        const int n = tid;
        const bool act = n < N;
        const size_t i = (size_t)b * N + (act ? n : 0);
        if (act) {
            const float wp = mid.wp;
            p.ring[(size_t)b * W * N + (size_t)ring_slot(mid.k, W) * N + n] = wp;
            p.w_new[i] = wp;
            if (p.weights) p.weights[i] = wp;
            if (p.bar) p.last_close[i] = mid.cn;
        }
        if (n == 0) {
            if (stats) {
                p.sa[b] = sa;
                p.sb[b] = sb;
            }
            p.value[b] = mid.value;
            p.k[b] = mid.k + 1;
            if (p.reward) p.reward[b] = (float)rwd;
            if (p.ret) p.ret[b] = ret;
            if (!isfinite(rwd) || !isfinite(mid.value)) atomicAdd(p.nonfinite, 1ull);
        }
    }
}

// ---------------------------------------------------------------- surface kernel
// The reference contract: obs is the caller's next-day window; only channel F-1
// is rewritten with ActionBuffer.get_all() (trading_env.py:103).
//
// Host-I/O form (pmenv_step_host, the reference driver's CPU tensors, train/on_policy.py:
// 59-67): `io` is non-null and every per-step input and output lives in pinned,
// device-mapped host staging — action / prices (p.action, p.prices) and the window's last
// closes (io.close_in) are read straight over PCIe, and the channel goes out as a dense
// [B, N, W] block (io.chan) beside the reward, return, post-drift weights and value
// (io.value_out), which the host scatters into the caller's window after one stream sync.
// The window itself never crosses the bus: only channel F-1 is the env's to write.
// HostIO: common.h


// the host-I/O kernels' last act: every wave's stores into the mapped staging have completed
// (vmcnt(0)) before the barrier, then one system-scope release and the env's completion word
__device__ __forceinline__ void hostio_done(const HostIO& io, int b) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 && io.done) {
        __threadfence_system();
        __hip_atomic_store(io.done + b, io.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

template <bool HOST>
__device__ __forceinline__ void surface_body(const StepParams& p, const HostIO& io, const int b) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int tid = threadIdx.x;
    const int N = p.N, W = p.W, F = p.F;
    Scratch s = carve(lds, 0, N, F);
    // Everything the step reads that does not depend on its own results is issued up front,
    // none waiting for another: the counter and value as lane values (a load the compiler sees
    // as uniform is moved to an SGPR at once, and the wait for it would hold the rest back by a
    // round trip), the window's last closes (host I/O: over PCIe) and the ring rows the channel
    // is rebuilt from — every slot but the one this step writes (weight_buffer.py:32-44).
    uint32_t z = 0u;
    asm volatile("" : "+v"(z));
    const int32_t k = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(make_rsrc(p.k + b, 4u), z, 0, 0);
    const double v_prev = buf_load_f64(make_rsrc(p.value + b, 8u), z);
    const bool out = HOST ? io.chan != nullptr : p.obs != nullptr;
    const float cl = HOST && out && tid < N ? io.close_in[(size_t)b * N + tid] : 0.0f;
    constexpr int PF = 4;                          // channel floats per thread prefetched (N W <= 1,024)
    const int32_t k1 = k + 1;                      // updates since reset, after this step
    const int slot = ring_slot(k, W), idx = ring_slot(k1, W);
    const bool full = (int64_t)k1 >= W - 1;
    const float* ringb = p.ring + (size_t)b * W * N;
    auto ring_src = [&](int i, int& n) {           // the ring slot feeding channel float i, or -1 (zero padding)
        n = (int)fdiv((uint32_t)i, p.div_w);
        const int t = i - n * W;
        if (!full) return t < W - idx ? -1 : t - (W - idx);
        return p.ring_mode == PMENV_RING_STORAGE ? t : (idx + t) % W;
    };
    float pv[PF];
#pragma unroll
    for (int e = 0; e < PF; ++e) {
        const int i = tid + kBlock * e;
        int n = 0;
        const int rs = out && i < N * W ? ring_src(i, n) : -1;
        pv[e] = rs >= 0 && rs != slot ? ringb[(size_t)rs * N + n] : 0.0f;
    }
    if (tid < 64) {
        if (N <= 64) {
            // the register-form scalar step (one asset per lane, DPP reductions, scalar_tail's
            // state writes), its loads issued inside the branch that consumes them; w' to LDS
            // for the channel's ring slot
            const ScalarIn sin = scalar_load<64, true>(p, b, tid, z);
            const ScalarMid mid = scalar_core<64>(p, b, tid, sin);
            if (tid < N) s.wp[tid] = mid.wp;
            scalar_tail<64>(p, b, tid, sin, mid);
            if (HOST && tid == 0) io.value_out[b] = mid.value;
        } else {
            gather_inputs(p, b, s, k);
            const double value = scalar_compute(p, b, s, k, v_prev);
            if (HOST && tid == 0) io.value_out[b] = value;      // the value scalar_compute stored
        }
    }
    __syncthreads();
    if (!out) {
        if (HOST) hostio_done(io, b);
        return;
    }
    float* obs = HOST ? io.chan + (size_t)b * N * W : p.obs + (size_t)b * N * W * F;
    const int fs = HOST ? 1 : F, fo = HOST ? 0 : F - 1;
#pragma unroll
    for (int e = 0; e < PF; ++e) {
        const int i = tid + kBlock * e;
        if (i < N * W) {
            int n;
            const int rs = ring_src(i, n);
            obs[(size_t)i * fs + fo] = rs < 0 ? 0.0f : (rs == slot ? s.wp[n] : pv[e]);
        }
    }
    for (int i = tid + kBlock * PF; i < N * W; i += kBlock) {   // windows past 1,024 channel floats
        int n;
        const int rs = ring_src(i, n);
        obs[(size_t)i * fs + fo] = rs < 0 ? 0.0f : (rs == slot ? s.wp[n] : ringb[(size_t)rs * N + n]);
    }
    // keep the advance-mode close in step with the caller's window
    for (int n = tid; n < N; n += kBlock)
        p.last_close[(size_t)b * N + n] = HOST ? (n == tid ? cl : io.close_in[(size_t)b * N + n])
                                               : obs[((size_t)n * W + (W - 1)) * F + p.close_ch];
    if (HOST) hostio_done(io, b);
}

static __global__ __launch_bounds__(kBlock) void step_surface_kernel(StepParams p) {
    surface_body<false>(p, HostIO{}, (int)blockIdx.x);
}
static __global__ __launch_bounds__(kBlock) void step_surface_host_kernel(StepParams p, HostIO io) {
    surface_body<true>(p, io, (int)blockIdx.x);
}

// The host-I/O step without a launch per call (pmenv_step_host, the reference driver's loop:
// train/on_policy.py:59-67 steps ONE env with CPU tensors). One resident workgroup polls the
// staging block's `go` word (system scope, over PCIe) and, each time the host posts a new tag
// there after writing the call's inputs, runs step_surface_host_kernel's body for every env —
// the same code, so the same bits — whose completion words the host spins on. It exits on the
// tag 0 (the host's stop) or after `idle` ticks of s_memrealtime (100 MHz) without a new tag,
// and stores the last tag it ran, so a relaunch picks up a tag posted as it left. Every call
// starts with a system-scope acquire (this call's inputs, and state other launches wrote) and
// ends with hostio_done's system-scope release (state visible to later launches on any XCD).
struct HostRes {
    const uint32_t* go;      // in the staging block: the tag of the call to run (0: stop)
    uint32_t* last;          // device memory: the last tag run (read at start, written at exit)
    uint32_t idle;           // ticks without a new tag before the workgroup exits
};
static __global__ __launch_bounds__(kBlock) void step_host_resident_kernel(StepParams p, HostIO io, HostRes rs) {
    __shared__ uint32_t s_go;
    uint32_t last = __builtin_amdgcn_readfirstlane(*rs.last);
    for (;;) {
        if (threadIdx.x == 0) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            uint32_t g;
            for (;;) {
                g = __hip_atomic_load(rs.go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (g != last) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > (uint64_t)rs.idle) {
                    g = 0u;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            s_go = g;
        }
        __syncthreads();
        const uint32_t g = __builtin_amdgcn_readfirstlane(s_go);
        __syncthreads();                                   // s_go is free for the next poll
        if (g == 0u) break;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");      // system scope
        HostIO c = io;
        c.seq = g;
        for (int b = 0; b < p.B; ++b) surface_body<true>(p, c, b);
        last = g;
    }
    if (threadIdx.x == 0) *rs.last = last;
}

// ---------------------------------------------------------------- the surface stream (two launches)
// The reference surface contract on windows past the Infinity Cache: the scalar step (K1, which
// also writes this step's ring slot), then this stream over the flat [B, N, W, F] window in
// 16-B chunks — no shift, so no halo and no LDS: every chunk is loaded, its (at most two)
// weight-channel floats are replaced by the ring floats they show (weight_buffer.py:32-44,
// the slot K1 just wrote included), and it is stored whole; the chunk holding a row's close on
// the last day also writes the advance-mode close (last_close). The per-env workgroup form
// (step_surface_kernel) waits for its env's scalar step before any store; here the stream
// streams. POL: the stream's cache policy (1 nt).
template <int BLOCK, int V, int POL>
__global__ __launch_bounds__(BLOCK) void surface_stream_kernel(StepParams p, uint32_t qtot) {
    constexpr int kAux = POL == 1 ? 2 : 0;
    constexpr int CPW = BLOCK * V;
    // the workgroup's rows' ring columns, [row][slot]: the ring is [B][W][N] (slot-major), so a
    // row's days are N floats apart and a chunk-per-lane gather touches a line per lane — staged
    // instead slot by slot, the rows of a slot adjacent (launch_surface_stream sizes it)
    extern __shared__ float sring[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t c0 = blockIdx.x * CPW;
    const uint32_t nblk = min((uint32_t)CPW, qtot - c0);
    const auto rs = make_rsrc(p.obs + (size_t)c0 * 4, nblk * 16u);
    const int N = p.N, W = p.W, F = p.F, Fm = F - 1;
    const uint32_t WF = (uint32_t)(W * F), per4 = (uint32_t)N * WF >> 2;
    const int close_pos = (W - 1) * F + p.close_ch;          // the last day's close in a row
    f4 x[V];
#pragma unroll
    for (int v = 0; v < V; ++v) x[v] = buf_load4<kAux>(rs, (uint32_t)(64 * V * wave + 64 * v + lane) * 16u);
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t b_lo = fdiv(c0, p.div_units);
    const uint32_t g_lo = b_lo * (uint32_t)N + fdiv(4u * (c0 - b_lo * per4), p.div_wf);
    const uint32_t ql = c0 + nblk - 1u;
    const uint32_t b_hi = fdiv(ql, p.div_units);
    const uint32_t g_hi = b_hi * (uint32_t)N + fdiv(4u * (ql - b_hi * per4) + 3u, p.div_wf);
    const uint32_t nrows = g_hi - g_lo + 1u;
    // each row's counter (after the scalar step) staged beside its ring columns, so that no
    // global load is left after the barrier; the element walk (slot i / nrows, row i % nrows)
    // keeps its quotient and remainder by increments (a division per thread, none per element)
    int32_t* sk = reinterpret_cast<int32_t*>(sring + (4u * CPW / WF + 2u) * (uint32_t)W);
    if ((uint32_t)tid < nrows) {
        const uint32_t g = g_lo + (uint32_t)tid;
        sk[tid] = p.k[g / (uint32_t)N];
    }
    {
        const uint32_t dq = (uint32_t)BLOCK / nrows, dr = (uint32_t)BLOCK - dq * nrows;
        uint32_t sl = (uint32_t)tid / nrows, r = (uint32_t)tid - sl * nrows;
        for (uint32_t i = (uint32_t)tid; i < nrows * (uint32_t)W; i += BLOCK) {
            const uint32_t g = g_lo + r, b = g / (uint32_t)N, n = g - b * (uint32_t)N;
            sring[r * (uint32_t)W + sl] = p.ring[((size_t)b * W + sl) * N + n];
            sl += dq;
            r += dr;
            if (r >= nrows) {
                r -= nrows;
                ++sl;
            }
        }
    }
    __syncthreads();
    float r[V][2];
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const uint32_t q = min(c0 + (uint32_t)(64 * V * wave + 64 * v + lane), qtot - 1u);
        const uint32_t b = fdiv(q, p.div_units);
        const uint32_t j0 = 4u * (q - b * per4);
        const uint32_t row = fdiv(j0, p.div_wf);
        const uint32_t kk = j0 - row * WF;
        const int f0 = (int)(kk - fdiv(kk, p.div_f) * (uint32_t)F);
        const uint32_t r0 = b * (uint32_t)N + row - g_lo;        // the chunk's row in the workgroup
        const int32_t k1 = sk[r0];                               // after the scalar step (one env per chunk)
        const int idx = ring_slot(k1, W);
        const bool full = (int64_t)k1 >= W - 1;
#pragma unroll
        for (int kth = 0; kth < 2; ++kth) {
            const int c = (Fm - f0) + kth * F;                   // the chunk's kth weight float (>= 4: none)
            int rsl = -1, rr = (int)r0;
            if (c < 4) {
                int pos = (int)kk + c;
                if (pos >= (int)WF) { pos -= (int)WF; ++rr; }
                const int t = (int)fdiv((uint32_t)pos, p.div_f);   // pos = t F + F - 1
                rsl = !full ? (t < W - idx ? -1 : t - (W - idx))
                            : (p.ring_mode == PMENV_RING_STORAGE ? t : (idx + t) % W);
            }
            r[v][kth] = rsl >= 0 ? sring[rr * W + rsl] : 0.0f;
        }
    }
    const auto rd = rs;
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const int j = 64 * V * wave + 64 * v + lane;
        const uint32_t q = min(c0 + (uint32_t)j, qtot - 1u);
        const uint32_t b = fdiv(q, p.div_units);
        const uint32_t j0 = 4u * (q - b * per4);
        const uint32_t row = fdiv(j0, p.div_wf);
        const uint32_t kk = j0 - row * WF;
        const int f0 = (int)(kk - fdiv(kk, p.div_f) * (uint32_t)F);
        float e[4] = {x[v].x, x[v].y, x[v].z, x[v].w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            int pos = (int)kk + c, rr = (int)row;
            if (pos >= (int)WF) { pos -= (int)WF; ++rr; }
            if (pos == close_pos && c0 + (uint32_t)j < qtot) p.last_close[(size_t)b * N + rr] = e[c];
        }
        const int ca = Fm - f0, cb = ca + F;                       // the weight floats' places (>= 4: none)
#pragma unroll
        for (int c = 0; c < 4; ++c) e[c] = c == ca ? r[v][0] : (c == cb ? r[v][1] : e[c]);
        buf_store4<kAux>(rd, (uint32_t)j * 16u, f4{e[0], e[1], e[2], e[3]});
    }
}

// ---------------------------------------------------------------- reset kernel
// io non-null: the host-I/O form (pmenv_reset_host) — the channel goes to io.chan [B, N, W]
// and the last closes come from io.close_in, as in step_surface_host_kernel.
static __global__ __launch_bounds__(kBlock) void reset_kernel(StepParams p, float* obs, const uint8_t* mask,
                                                              HostIO io = HostIO{}) {
    const int b = blockIdx.x;
    if (mask && !mask[b]) return;
    const int tid = threadIdx.x;
    const int N = p.N, W = p.W, F = p.F;
    if (tid == 0) {
        p.value[b] = p.init_cash;                 // trading_env.py:28
        p.k[b] = 0;                               // weight_buffer.py:49 idx = 1
        p.sa[b] = 0.0;
        p.sb[b] = 0.0;
        if (io.value_out) io.value_out[b] = p.init_cash;
    }
    float* ringb = p.ring + (size_t)b * W * N;     // weight_buffer.py:47-48 e0 in slot 0
    for (int i = tid; i < W * N; i += kBlock) ringb[i] = i == 0 ? 1.0f : 0.0f;
    for (int n = tid; n < N; n += kBlock) p.w_new[(size_t)b * N + n] = n == 0 ? 1.0f : 0.0f;   // get_last()
    if (io.chan) {
        float* ch = io.chan + (size_t)b * N * W;   // the same channel, dense, for the host to scatter
        for (int i = tid; i < N * W; i += kBlock) ch[i] = i == W - 1 ? 1.0f : 0.0f;
        for (int n = tid; n < N; n += kBlock) p.last_close[(size_t)b * N + n] = io.close_in[(size_t)b * N + n];
    }
    if (io.done) {                                 // host I/O: the completion word
        hostio_done(io, b);
        return;
    }
    if (!obs) return;
    float* ob = obs + (size_t)b * N * W * F;       // trading_env.py:31-32 get_all() at idx = 1
    for (int i = tid; i < N * W; i += kBlock) {
        const int n = (int)fdiv((uint32_t)i, p.div_w);
        const int t = i - n * W;
        ob[((size_t)n * W + t) * F + (F - 1)] = (n == 0 && t == W - 1) ? 1.0f : 0.0f;
    }
    for (int n = tid; n < N; n += kBlock)
        p.last_close[(size_t)b * N + n] = ob[((size_t)n * W + (W - 1)) * F + p.close_ch];
}

}  // namespace pmenv_dev
