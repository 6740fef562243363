// scalar_vec.h — the per-env scalar step (K1) in packed form, for the two-launch
// advance path (included by pmenv.hip after env_step.h).
//
// L lanes per env and A assets per lane (L*A >= N): 64/L envs per wave, so a wave
// carries A times the envs of the one-asset-per-lane form. Lane j holds the
// consecutive assets j*A .. j*A+A-1 (one dwordx{A} per array: small N), or — STR —
// the strided assets j, j+L, .. (each dword instruction a coalesced run: large N).
// Reductions: the lane's A values in order, then an all-lane butterfly inside the
// group — DPP quad_perm xor 1 / xor 2, row_half_mirror (8 lanes), row_mirror (16) —
// whose every level combines a value with its partner's in commutative pairs, so all
// L lanes hold bitwise the same total and every branch on it is group-uniform;
// L = 32 / 64 use the row-shift + readlane form of the register kernel.
//
// Reference semantics (zachramsey/pm-rl), as scalar_finish in env_step.h:
//   env/sim/trading_env.py:54-100 normalisation, commission mu, value, return, reward
//   env/sim/weight_buffer.py:13-30 ring update / get_last
//   env/reward.py:20-31 returns / sharpe_ratio;  data/instrument.py:79 price relatives
#pragma once
#include "env_step.h"

namespace pmenv_dev {

constexpr int kHalfMirror = 0x141, kRowMirror = 0x140;

// L-lane group reduction, bitwise the same in every lane of the group
template <int L, int OP>   // OP 0 sum, 1 max, 2 min
__device__ __forceinline__ double gred(double v, int lane) {
    if constexpr (L >= 32) {
        return OP == 0 ? group_sum<L>(v, lane) : OP == 1 ? group_max<L>(v, lane) : group_min<L>(v, lane);
    } else {
        auto op = [](double a, double b) { return OP == 0 ? a + b : OP == 1 ? fmax(a, b) : fmin(a, b); };
        v = op(v, dpp_shift<kQuadXor1>(v, 0.0));
        v = op(v, dpp_shift<kQuadXor2>(v, 0.0));
        if (L >= 8) v = op(v, dpp_shift<kHalfMirror>(v, 0.0));
        if (L >= 16) v = op(v, dpp_shift<kRowMirror>(v, 0.0));
        return v;
    }
}

// A floats of a [B*N] array for lane j of an env row starting at element `row`: the
// consecutive elements j*A .. j*A+A-1 (one dwordx{A}), or — STR — the strided
// elements j, j+L, .. (A dword loads, each a coalesced run across the group's lanes).
// Past the array's end the buffer descriptor reads 0 (never a fault); lanes mask
// what is not theirs.
template <int L, int A, bool STR>
__device__ __forceinline__ void load_packed(const float* base, uint32_t bytes, size_t row, int j, float (&x)[A]) {
    const auto r = make_rsrc(base, bytes);
    if constexpr (STR || A == 1) {
#pragma unroll
        for (int e = 0; e < A; ++e) x[e] = buf_load1(r, (uint32_t)(row + j + e * L) * 4u);
    } else if constexpr (A == 2) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, (uint32_t)(row + j * A) * 4u, 0, 0);
        x[0] = __uint_as_float(v[0]);
        x[1] = __uint_as_float(v[1]);
    } else {
        const uint32_t off = (uint32_t)(row + j * A) * 4u;
#pragma unroll
        for (int h = 0; h < A / 4; ++h) {
            const f4 v = buf_load4<0>(r, off + 16u * h);
            x[4 * h] = v.x; x[4 * h + 1] = v.y; x[4 * h + 2] = v.z; x[4 * h + 3] = v.w;
        }
    }
}


// The packed scalar step in three parts, so the one-launch walk step (step_walk.h) can
// put its window loads between the loads and the compute and run the state writes
// after its stores: vec_load issues every load (none dependent on another; the bar
// rows of a resident series follow the env's day index), vec_core computes the
// normalised weights, mu, the value and the lanes' w', vec_tail writes the state and
// the reward. scalar_step_vec_kernel runs the three in a row.
template <int A>
struct VecIn {
    int32_t k;
    double v_prev, sa, sb;
    float a[A], wl[A], pl[A], cn[A];
};

template <int A>
struct VecMid {
    double value, V;
    float wp[A];       // the lane's w' (0 for assets past N)
};

// SNAP (step_flat_vec_kernel): value, counter, get_last() and the last close from the
// flat step's state snapshot of parity p (sv_in .. slc_in) instead of the canonical state.
// get_last() feeds only the commission fixed point: without commission it is not read
// (the descriptor has no records: no traffic), and vec_core never looks at it.
template <int L, int A, bool STR, bool SNAP = false>
__device__ __forceinline__ VecIn<A> vec_load(const StepParams& p, int b, int lane) {
    const int j = lane % L;
    const int N = p.N, Fm = p.F - 1;
    const bool env_ok = b < p.B;
    const int bc = env_ok ? b : 0;
    const size_t row = (size_t)bc * N;
    const uint32_t nbytes = (uint32_t)p.B * (uint32_t)N * 4u;
    VecIn<A> in;
    in.k = SNAP ? p.sk_in[bc] : p.k[bc];
    in.v_prev = SNAP ? p.sv_in[bc] : p.value[bc];
    // reward statistics: only the tail's lane 0 reads them; the snapshot form (a tile's
    // registers are scarce there) loads them in the tail
    in.sa = SNAP ? 0.0 : p.sa[bc];
    in.sb = SNAP ? 0.0 : p.sb[bc];
    load_packed<L, A, STR>(p.action, nbytes, row, j, in.a);
    load_packed<L, A, STR>(SNAP ? p.sw_in : p.w_new, p.commission > 0.0 ? nbytes : 0u, row, j,
                           in.wl);                                        // get_last() (weight_buffer.py:28-30)
    load_packed<L, A, STR>(p.prices ? p.prices : SNAP ? p.slc_in : p.last_close, nbytes, row, j, in.pl);
    const float* barb = p.bar ? env_bar(p, bc) : nullptr;
#pragma unroll
    for (int e = 0; e < A; ++e) {
        const int n = STR ? j + e * L : j * A + e;
        const int nc = env_ok && n < N ? n : 0;
        in.cn[e] = barb ? barb[(size_t)nc * Fm + p.close_ch] : NAN;
    }
    return in;
}

template <int L, int A, bool STR>
__device__ __forceinline__ VecMid<A> vec_core(const StepParams& p, int b, int lane, const VecIn<A>& in) {
    const int j = lane % L;
    const int N = p.N;
    const bool env_ok = b < p.B;
    int nn[A];                                    // the lane's assets
    bool act[A];
#pragma unroll
    for (int e = 0; e < A; ++e) {
        nn[e] = STR ? j + e * L : j * A + e;
        act[e] = env_ok && nn[e] < N;
    }
    double x[A];
    double s_loc = 0.0, mn_loc = INFINITY;
    bool nan_here = false;
#pragma unroll
    for (int e = 0; e < A; ++e) {
        x[e] = act[e] ? (double)in.a[e] : 0.0;
        s_loc += x[e];
        mn_loc = fmin(mn_loc, act[e] ? x[e] : INFINITY);
        nan_here |= act[e] && isnan(in.a[e]);
    }
    // trading_env.py:58 normalise iff !isclose(sum, 1, atol=1e-6) AND (OR: trainer) min < 0;
    // AND mode with every group's sum close to 1 cannot normalise (the min is skipped)
    const double sum = gred<L, 0>(s_loc, lane);
    const bool not_close = !(fabs(sum - 1.0) <= 1e-6 + 1e-5);
    bool norm = false;
    if (p.norm_mode != PMENV_NORM_AND || __any(not_close)) {
        double mn = gred<L, 2>(mn_loc, lane);
        const uint64_t gmask = L == 64 ? ~0ull : (((1ull << (L & 63)) - 1ull) << (lane & ~(L - 1)));
        if (__ballot(nan_here) & gmask) mn = NAN;     // torch.min propagates NaN
        const bool negative = mn < 0.0;
        norm = p.norm_mode == PMENV_NORM_AND ? (not_close && negative) : (not_close || negative);
    }
    double wv[A];
#pragma unroll
    for (int e = 0; e < A; ++e) wv[e] = x[e];
    if (__any(norm)) {
        double shift = 0.0;
        if (p.norm_mode == PMENV_NORM_OR) {       // torch.softmax is max-shifted
            double m = -INFINITY;
#pragma unroll
            for (int e = 0; e < A; ++e) m = fmax(m, act[e] ? x[e] : -INFINITY);
            shift = gred<L, 1>(m, lane);
        }
        double ex[A], z_loc = 0.0;
#pragma unroll
        for (int e = 0; e < A; ++e) {
            ex[e] = act[e] ? exp(x[e] - shift) : 0.0;   // :59 (no max-shift in AND mode)
            z_loc += ex[e];
        }
        const double z = gred<L, 0>(z_loc, lane);
        if (norm) {
#pragma unroll
            for (int e = 0; e < A; ++e) wv[e] = ex[e] / z;   // :60
        }
    }

    // :67-75 commission fixed point (f64, capped), per env group, in the active-set form of
    // scalar_core (env_step.h): S(mu) = A - mu Bw over the assets where wl_n > mu w_n, A and
    // Bw reduced only when that set changes (A ballots per iteration)
    double V = in.v_prev;
    if (p.commission > 0.0) {
        const double c = p.commission;
        const int g0 = lane & ~(L - 1);
        const double w0 = L == 64 ? group_lane0<64>(wv[0], lane) : __shfl(wv[0], g0, 64);
        const double wl0 = L == 64 ? (double)__int_as_float(group_lane0_i<64>(__float_as_int(in.wl[0]), lane))
                                   : (double)__shfl(in.wl[0], g0, 64);
        const double K = 1.0 - c * wl0, Dc = 2.0 * c - c * c, invE = 1.0 / (1.0 - c * w0);
        const uint64_t gmask = L == 64 ? ~0ull : (((1ull << (L & 63)) - 1ull) << (lane & ~(L - 1)));
        double mu_last = 1.0, mu = 1.0 - 2.0 * c + c * c;
        double Aw = 0.0, Bw = 0.0;
        uint64_t pset[A];
#pragma unroll
        for (int e = 0; e < A; ++e) pset[e] = 0;
        bool have = false;
        int it = 0;
        bool done = !(fabs(mu - mu_last) > p.mu_tol) || p.mu_max_iter <= 0;
        while (__any(!done)) {
            bool in_p[A];
            bool changed = !have;
            uint64_t m[A];
#pragma unroll
            for (int e = 0; e < A; ++e) {
                in_p[e] = act[e] && nn[e] > 0 && (double)in.wl[e] - mu * wv[e] > 0.0;   // max(x, 0) as intended
                m[e] = __ballot(in_p[e]) & gmask;
                changed |= m[e] != pset[e];
            }
            if (__any(!done && changed)) {
                double pa = 0.0, pb = 0.0;
#pragma unroll
                for (int e = 0; e < A; ++e) {
                    pa += in_p[e] ? (double)in.wl[e] : 0.0;
                    pb += in_p[e] ? wv[e] : 0.0;
                    pset[e] = m[e];
                }
                Aw = gred<L, 0>(pa, lane);
                Bw = gred<L, 0>(pb, lane);
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

    // :78-79 portfolio value; :83-84 w' = portfolio / value. instrument.py:79: the price
    // relative is the correctly rounded fp32 quotient of today's close over the window's
    // last close (caller prices when given), formed here where it is used
    double pv[A], pv_loc = 0.0;
#pragma unroll
    for (int e = 0; e < A; ++e) {
        const double y = !act[e] ? 1.0 : (p.bar && !p.prices) ? (double)(in.cn[e] / in.pl[e]) : (double)in.pl[e];
        pv[e] = act[e] ? V * (wv[e] * y) : 0.0;
        pv_loc += pv[e];
    }
    VecMid<A> m;
    m.value = gred<L, 0>(pv_loc, lane);
    m.V = V;
#pragma unroll
    for (int e = 0; e < A; ++e) m.wp[e] = act[e] ? (float)(pv[e] / m.value) : 0.0f;
    return m;
}

// SNAP: only the env's owner workgroup (`owner`) writes, and it also writes the next
// step's snapshot (sv_out .. slc_out), as scalar_tail
template <int L, int A, bool STR, bool SNAP = false>
__device__ __forceinline__ void vec_tail(const StepParams& p, int b, int lane, const VecIn<A>& in,
                                         const VecMid<A>& m, bool owner = true) {
    if (SNAP && !owner) return;
    const int j = lane % L;
    const int N = p.N, W = p.W;
    const bool env_ok = b < p.B;
    const int bc = env_ok ? b : 0;
    const int32_t k = in.k;
    const double value = m.value, V = m.V;
    // :83-84 ring.update(w') at slot (1 + k) % W
    const int slot = ring_slot(k, W);
    float* ring_row = p.ring + (size_t)bc * W * N + (size_t)slot * N;
#pragma unroll
    for (int e = 0; e < A; ++e) {
        const int n = STR ? j + e * L : j * A + e;
        if (!(env_ok && n < N)) continue;
        const float wp = m.wp[e];
        ring_row[n] = wp;
        p.w_new[(size_t)bc * N + n] = wp;
        if (p.weights) p.weights[(size_t)bc * N + n] = wp;
        if (p.bar) p.last_close[(size_t)bc * N + n] = in.cn[e];
        if (SNAP) {
            if (p.commission > 0.0) p.sw_out[(size_t)bc * N + n] = wp;
            p.slc_out[(size_t)bc * N + n] = in.cn[e];
        }
    }
    if (env_ok && j == 0) {
        const double in_sa = SNAP ? p.sa[b] : in.sa, in_sb = SNAP ? p.sb[b] : in.sb;
        // :88 ret = value / self.value (mu-scaled: excludes commission) ; :89
        const double ret = p.ret_mode == PMENV_RET_GROSS ? value / V : value / in.v_prev;
        double r;
        switch (p.reward_kind) {
        case PMENV_REWARD_RETURN:
            r = ret * p.scale;
            break;
        case PMENV_REWARD_SHARPE: {              // reward.py:26-31 as running moments
            const double mm = (double)(k + 1);
            double mean = in_sa, m2 = in_sb;
            const double d = ret - mean;
            mean += d / mm;
            m2 += d * (ret - mean);
            p.sa[b] = mean;
            p.sb[b] = m2;
            r = mm < 2.0 ? NAN : (mean - p.rf) / sqrt(m2 / (mm - 1.0)) * p.scale;
            break;
        }
        case PMENV_REWARD_DIFF_SHARPE: {         // Moody & Saffell (1998)
            const double R = ret - 1.0, Am = in_sa, Bm = in_sb;
            const double dA = R - Am, dB = R * R - Bm, var = Bm - Am * Am;
            r = var > 1e-12 ? (Bm * dA - 0.5 * Am * dB) / (var * sqrt(var)) * p.scale : 0.0;
            p.sa[b] = Am + p.eta * dA;
            p.sb[b] = Bm + p.eta * dB;
            break;
        }
        default:
            r = log(ret) * p.scale;              // :99
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

template <int L, int A, bool STR>
__global__ __launch_bounds__(256) void scalar_step_vec_kernel(StepParams p) {
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

}  // namespace pmenv_dev
