// pmenv.hip — MI355X (gfx950) vectorised portfolio environment: HIP kernels + C ABI.
//
// One workgroup owns one env per launch. The env's [N, W, F] observation block is
// staged through LDS, so the one-day window advance (a shift by F floats inside
// every asset row: 20 B for F = 5, not 16-B aligned) is done with aligned 16-B
// global loads and stores and arbitrary-offset LDS reads. The per-env scalar work
// (normalisation, commission fixed point, value, return, reward, weight drift)
// runs on wave 0 with 64-lane shuffle reductions in f64.
//
// Reference semantics restated (zachramsey/pm-rl):
//   env/sim/trading_env.py:21-41 reset, :44-105 step
//   env/sim/weight_buffer.py:13-51 ring update / get_last / get_all
//   env/reward.py:20-31 returns / log_returns / sharpe_ratio
//   data/instrument.py:79 price relatives, :339-356 sliding window
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/pmenv.h"

namespace {

constexpr int kBlock = 256;         // threads per env workgroup (4 waves)
constexpr int kMaxVec = 8;          // float4 registers per thread for one tile
constexpr int kTileFloats = kBlock * kMaxVec * 4;  // 8192 floats = 32 KiB LDS tile

// ---------------------------------------------------------------- fast division
// q = floor(n / d) for 0 <= n < 2^31 by multiply-high (Granlund & Montgomery).
struct FastDiv {
    uint32_t mul, shift, d;
};

FastDiv make_fastdiv(uint32_t d) {
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

// ---------------------------------------------------------------- params
struct StepParams {
    int B, N, W, F, close_ch;
    int reward_kind, norm_mode, ring_mode, ret_mode, mu_max_iter;
    int rows_per_tile;     // asset rows per LDS tile
    int tile_floats;       // floats reserved for the tile region (multiple of 4)
    double init_cash, commission, scale, rf, eta, mu_tol;
    const float* action;
    const float* prices;
    const float* bar;
    float* obs;
    float* reward;
    double* ret;
    float* weights;
    double* value;
    int32_t* k;
    float* ring;
    double* sa;
    double* sb;
    unsigned long long* nonfinite;
    FastDiv div_wf, div_f, div_w;
};

// ---------------------------------------------------------------- wave reductions
// Butterfly over 64 lanes then broadcast lane 0, so every lane holds bitwise the
// same value and every branch taken on it is wave-uniform.
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return __shfl(v, 0, 64);
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return __shfl(v, 0, 64);
}
__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
    return __shfl(v, 0, 64);
}

// LDS carve of the per-env scratch, behind the (16-B aligned) tile region.
struct Scratch {
    double* wv;   // [N] target weights, then portfolio values
    double* yv;   // [N] price relatives
    float* wl;    // [N] w_last (ring.get_last())
    float* wp;    // [N] post-drift weights w'
    float* bar;   // [N * (F-1)] new bar (advance mode)
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

size_t scratch_bytes(int tile_floats, int N, int F) {
    return (size_t)tile_floats * 4 + (size_t)N * 16 + (size_t)N * 8 + (size_t)N * (F - 1) * 4 + 16;
}

// ---------------------------------------------------------------- phase A
// The per-env scalar part of TradingEnv.step (trading_env.py:54-100), on wave 0.
// `tile` is the env's staged obs block in LDS (advance mode, single tile) or null.
__device__ __forceinline__ void env_scalar_step(const StepParams& p, int b, Scratch& s, const float* tile) {
    const int lane = threadIdx.x;
    const int N = p.N, W = p.W, F = p.F, Fm = F - 1;
    const size_t env_off = (size_t)b * N * W * F;
    const int32_t k = p.k[b];
    const double v_prev = p.value[b];
    const float* ringb = p.ring + (size_t)b * W * N;
    const int last = k % W;                        // weight_buffer.py:30 (idx-1) % W

    // :54-55 flatten; price relatives (given, or instrument.py:79 from the close channel)
    double sum = 0.0, mn = INFINITY;
    int nan_seen = 0;
    for (int n = lane; n < N; n += 64) {
        double a = (double)p.action[(size_t)b * N + n];
        double y;
        if (p.prices) {
            y = (double)p.prices[(size_t)b * N + n];
        } else {
            // instrument.py:79 divides float32 tensors: correctly rounded fp32 quotient
            float cn = s.bar[n * Fm + p.close_ch];
            size_t o = (size_t)n * W * F + (size_t)(W - 1) * F + p.close_ch;
            float co = tile ? tile[o] : p.obs[env_off + o];
            y = (double)(cn / co);  // IEEE division (hipcc default: correctly rounded)
        }
        s.wv[n] = a;
        s.yv[n] = y;
        s.wl[n] = ringb[(size_t)last * N + n];
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
        double w0 = __shfl(lane == 0 ? s.wv[0] : 0.0, 0, 64);
        double wl0 = (double)s.wl[0];
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
    const int slot = (int)((1 + (int64_t)k) % W);
    float* ring_slot = p.ring + (size_t)b * W * N + (size_t)slot * N;
    for (int n = lane; n < N; n += 64) {
        float w = (float)(s.wv[n] / value);
        s.wp[n] = w;
        ring_slot[n] = w;
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
}

// Copy nf floats of one tile HBM -> registers -> LDS. All loads are issued before
// the first LDS store so up to kMaxVec 16-B loads per lane are in flight.
typedef float f4 __attribute__((ext_vector_type(4)));

template <bool VEC>
__device__ __forceinline__ void stage_tile(const float* __restrict__ src, float* lds, int nf, int tid) {
    if (VEC) {
        f4 reg[kMaxVec];
        const int nq = nf >> 2;
#pragma unroll
        for (int i = 0; i < kMaxVec; ++i) {
            int q = tid + i * kBlock;
            reg[i] = q < nq ? reinterpret_cast<const f4*>(src)[q] : f4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int i = 0; i < kMaxVec; ++i) {
            int q = tid + i * kBlock;
            if (q < nq) reinterpret_cast<f4*>(lds)[q] = reg[i];
        }
    } else {
        float reg[kMaxVec * 4];
#pragma unroll
        for (int i = 0; i < kMaxVec * 4; ++i) {
            int j = tid + i * kBlock;
            reg[i] = j < nf ? src[j] : 0.0f;
        }
#pragma unroll
        for (int i = 0; i < kMaxVec * 4; ++i) {
            int j = tid + i * kBlock;
            if (j < nf) lds[j] = reg[i];
        }
    }
}

// ---------------------------------------------------------------- advance kernel
// out[n, t, f] = t < W-1 ? in[n, t+1, f] : bar[n, f]           (market channels)
// out[n, t, F-1] = shifted like the market channels with w' appended, or, once the
// ring is full in storage mode, in[n, t, F-1] with w' at t == slot.
template <bool VEC>
__global__ __launch_bounds__(kBlock) void step_advance_kernel(StepParams p) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int N = p.N, W = p.W, F = p.F, Fm = F - 1;
    const int WF = W * F;
    const int R = p.rows_per_tile;
    const bool single = R >= N;
    Scratch s = carve(lds, p.tile_floats, N, F);
    float* obs = p.obs + (size_t)b * N * WF;

    // the new bar -> LDS (N * Fm floats, coalesced)
    const float* barg = p.bar + (size_t)b * N * Fm;
    for (int i = tid; i < N * Fm; i += kBlock) s.bar[i] = barg[i];

    if (single) stage_tile<VEC>(obs, lds, N * WF, tid);
    __syncthreads();
    if (tid < 64) env_scalar_step(p, b, s, single ? lds : nullptr);
    __syncthreads();
    const int shift_w = s.ints[0];
    const int slot = s.ints[1];

    for (int r0 = 0; r0 < N; r0 += R) {
        const int rows = min(R, N - r0);
        const int nf = rows * WF;
        if (!single) {
            if (r0 > 0) __syncthreads();
            stage_tile<VEC>(obs + (size_t)r0 * WF, lds, nf, tid);
            __syncthreads();
        }
        float* dst = obs + (size_t)r0 * WF;
        if (VEC) {
            const int nq = nf >> 2;
            for (int q = tid; q < nq; q += kBlock) {
                uint32_t j = (uint32_t)q * 4u;
                uint32_t row = fdiv(j, p.div_wf);
                uint32_t kk = j - row * (uint32_t)WF;
                uint32_t t = fdiv(kk, p.div_f);
                uint32_t f = kk - t * (uint32_t)F;
                float v[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int n = r0 + (int)row;
                    const bool lastday = (int)t == W - 1;
                    int idx;
                    if ((int)f == F - 1)
                        idx = shift_w ? (lastday ? s.wp_off + n : (int)j + F)
                                      : ((int)t == slot ? s.wp_off + n : (int)j);
                    else
                        idx = lastday ? s.bar_off + n * Fm + (int)f : (int)j + F;
                    v[e] = lds[idx];
                    ++j;
                    if (++f == (uint32_t)F) {
                        f = 0;
                        if (++t == (uint32_t)W) { t = 0; ++row; }
                    }
                }
                reinterpret_cast<f4*>(dst)[q] = f4{v[0], v[1], v[2], v[3]};
            }
        } else {
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
}

// ---------------------------------------------------------------- surface kernel
// The reference contract: obs is the caller's next-day window; only channel F-1
// is rewritten with ActionBuffer.get_all() (trading_env.py:103).
__global__ __launch_bounds__(kBlock) void step_surface_kernel(StepParams p) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int N = p.N, W = p.W, F = p.F;
    Scratch s = carve(lds, 0, N, F);
    if (tid < 64) env_scalar_step(p, b, s, nullptr);
    __syncthreads();
    if (!p.obs) return;
    const int slot = s.ints[1];
    const int32_t k1 = s.ints[2];                 // updates since reset, after this step
    const int idx = (int)((1 + (int64_t)k1) % W);
    const bool full = (int64_t)k1 >= W - 1;
    const float* ringb = p.ring + (size_t)b * W * N;
    float* obs = p.obs + (size_t)b * N * W * F;
    for (int i = tid; i < N * W; i += kBlock) {
        const int n = (int)fdiv((uint32_t)i, p.div_w);
        const int t = i - n * W;
        int rs;  // ring slot feeding position t, or -1 for zero padding (weight_buffer.py:38-44)
        if (!full) rs = t < W - idx ? -1 : t - (W - idx);
        else rs = p.ring_mode == PMENV_RING_STORAGE ? t : (idx + t) % W;
        float v = rs < 0 ? 0.0f : (rs == slot ? s.wp[n] : ringb[(size_t)rs * N + n]);
        obs[((size_t)n * W + t) * F + (F - 1)] = v;
    }
}

// ---------------------------------------------------------------- reset kernel
__global__ __launch_bounds__(kBlock) void reset_kernel(StepParams p, float* obs, const uint8_t* mask) {
    const int b = blockIdx.x;
    if (mask && !mask[b]) return;
    const int tid = threadIdx.x;
    const int N = p.N, W = p.W, F = p.F;
    if (tid == 0) {
        p.value[b] = p.init_cash;                 // trading_env.py:28
        p.k[b] = 0;                               // weight_buffer.py:49 idx = 1
        p.sa[b] = 0.0;
        p.sb[b] = 0.0;
    }
    float* ringb = p.ring + (size_t)b * W * N;     // weight_buffer.py:47-48 e0 in slot 0
    for (int i = tid; i < W * N; i += kBlock) ringb[i] = i == 0 ? 1.0f : 0.0f;
    if (!obs) return;
    float* ob = obs + (size_t)b * N * W * F;       // trading_env.py:31-32 get_all() at idx = 1
    for (int i = tid; i < N * W; i += kBlock) {
        const int n = (int)fdiv((uint32_t)i, p.div_w);
        const int t = i - n * W;
        ob[((size_t)n * W + t) * F + (F - 1)] = (n == 0 && t == W - 1) ? 1.0f : 0.0f;
    }
}

// ---------------------------------------------------------------- Philox + synthetic data
__device__ __forceinline__ void philox4x32(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint32_t lo0 = 0xD2511F53u * c[0], hi0 = __umulhi(0xD2511F53u, c[0]);
        uint32_t lo1 = 0xCD9E8D57u * c[2], hi1 = __umulhi(0xCD9E8D57u, c[2]);
        uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}

__device__ __forceinline__ double u01(uint32_t x) { return ((double)(x >> 8) + 0.5) * (1.0 / 16777216.0); }

__device__ __forceinline__ void normals4(uint32_t c0, uint32_t c1, uint64_t g, uint64_t seed, double z[4]) {
    uint32_t c[4] = {c0, c1, (uint32_t)g, (uint32_t)(g >> 32)};
    philox4x32(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const double two_pi = 6.283185307179586476925286766559;
    double r0 = sqrt(-2.0 * log(u01(c[0]))), r1 = sqrt(-2.0 * log(u01(c[2])));
    z[0] = r0 * cos(two_pi * u01(c[1]));
    z[1] = r0 * sin(two_pi * u01(c[1]));
    z[2] = r1 * cos(two_pi * u01(c[3]));
    z[3] = r1 * sin(two_pi * u01(c[3]));
}

// One thread per (env, asset): close_t = close_{t-1} exp(sigma z - sigma^2/2), OHLC
// around it (SURVEY.md §8d synthetic inputs). series [T][B][N][4].
__global__ void synth_series_kernel(float4* series, int T, int B, int N, int64_t env_offset,
                                    uint64_t seed, double sigma) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)B * N) return;
    const int b = (int)(i / N), n = (int)(i % N);
    const uint64_t g = (uint64_t)(env_offset + b);
    double z[4];
    normals4(0u, (uint32_t)n, g, seed, z);
    double close = 100.0 * exp(0.2 * z[0]);
    for (int t = 0; t < T; ++t) {
        normals4((uint32_t)(t + 1), (uint32_t)n, g, seed, z);
        double cl = close * exp(sigma * z[0] - 0.5 * sigma * sigma);
        double op = close * exp(0.3 * sigma * z[1]);
        double hi = fmax(op, cl) * exp(fabs(0.5 * sigma * z[2]));
        double lo = fmin(op, cl) * exp(-fabs(0.5 * sigma * z[3]));
        series[((size_t)t * B + b) * N + n] = make_float4((float)op, (float)hi, (float)lo, (float)cl);
        close = cl;
    }
}

// One thread per (t, env): softmax of N(0,1) logits over the N assets.
__global__ void synth_actions_kernel(float* actions, int T, int B, int N, int64_t env_offset, uint64_t seed) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)T * B) return;
    const int t = (int)(i / B), b = (int)(i % B);
    const uint64_t g = (uint64_t)(env_offset + b);
    float* out = actions + (size_t)i * N;
    double mx = -INFINITY;
    for (int n = 0; n < N; ++n) {
        double z[4];
        normals4((uint32_t)t, 0x80000000u | (uint32_t)n, g, seed, z);
        out[n] = (float)z[0];
        mx = fmax(mx, z[0]);
    }
    double sum = 0.0;
    for (int n = 0; n < N; ++n) {
        double z[4];
        normals4((uint32_t)t, 0x80000000u | (uint32_t)n, g, seed, z);
        sum += exp(z[0] - mx);
    }
    for (int n = 0; n < N; ++n) {
        double z[4];
        normals4((uint32_t)t, 0x80000000u | (uint32_t)n, g, seed, z);
        out[n] = (float)(exp(z[0] - mx) / sum);
    }
}

__global__ void window_init_kernel(float* obs, const float4* series, int B, int N, int W, int F) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // over B*N*W
    if (i >= (int64_t)B * N * W) return;
    const int t = (int)(i % W);
    const int64_t bn = i / W;
    const int n = (int)(bn % N), b = (int)(bn / N);
    float4 v = series[((size_t)t * B + b) * N + n];
    float* o = obs + (size_t)i * F;
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
    for (int f = 4; f < F; ++f) o[f] = 0.0f;
}

// ---------------------------------------------------------------- GAE / moments
// One thread per env walks its column of the [T, B] rollout backwards; for a fixed
// t the B threads touch B consecutive floats, so every access is coalesced.
__global__ void gae_kernel(const float* r, const float* v, const uint8_t* dones, float* adv, float* ret,
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

constexpr int kMomBlocks = 1024;
__device__ double g_mom_partial[kMomBlocks * 3];

__global__ __launch_bounds__(kBlock) void moments_partial_kernel(const float* x, int64_t n) {
    __shared__ double sh[2][kBlock / 64];
    double s = 0.0, q = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        double v = (double)x[i];
        s += v;
        q += v * v;
    }
    for (int o = 32; o > 0; o >>= 1) { s += __shfl_xor(s, o, 64); q += __shfl_xor(q, o, 64); }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sh[0][w] = s; sh[1][w] = q; }
    __syncthreads();
    if (threadIdx.x == 0) {
        double ts = 0.0, tq = 0.0;
        for (int i = 0; i < kBlock / 64; ++i) { ts += sh[0][i]; tq += sh[1][i]; }
        g_mom_partial[blockIdx.x * 3 + 0] = ts;
        g_mom_partial[blockIdx.x * 3 + 1] = tq;
    }
}

__global__ void moments_final_kernel(int nblocks, int64_t n, double* out) {
    if (threadIdx.x != 0) return;
    double s = 0.0, q = 0.0;
    for (int i = 0; i < nblocks; ++i) { s += g_mom_partial[i * 3 + 0]; q += g_mom_partial[i * 3 + 1]; }
    out[0] = (double)n;
    out[1] = s;
    out[2] = q;
}

}  // namespace

// ================================================================ host side / C ABI
struct pmenv {
    pmenv_cfg cfg;
    int device;
    void* state;          // one allocation: value | sa | sb | k | ring | nonfinite
    size_t state_bytes;
    double* value;
    double* sa;
    double* sb;
    int32_t* k;
    float* ring;
    unsigned long long* nonfinite;
    int rows_per_tile, tile_floats;
    bool vec;
    bool owns_state;
    size_t lds_advance, lds_surface;
    char err[512];
};

namespace {

thread_local char g_create_err[512] = "";

void set_err(pmenv* h, const char* fmt, ...) {
    if (!h) return;
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(h->err, sizeof(h->err), fmt, ap);
    va_end(ap);
}

struct DeviceGuard {
    int prev = -1;
    bool changed = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) == hipSuccess && prev != dev) {
            changed = hipSetDevice(dev) == hipSuccess;
        }
    }
    ~DeviceGuard() {
        if (changed) (void)hipSetDevice(prev);
    }
};

StepParams base_params(const pmenv* h) {
    StepParams p;
    memset(&p, 0, sizeof(p));
    const pmenv_cfg& c = h->cfg;
    p.B = c.num_envs; p.N = c.num_assets; p.W = c.window; p.F = c.features;
    p.close_ch = c.close_channel;
    p.reward_kind = c.reward_kind; p.norm_mode = c.norm_mode; p.ring_mode = c.ring_mode;
    p.ret_mode = c.ret_mode; p.mu_max_iter = c.mu_max_iter;
    p.rows_per_tile = h->rows_per_tile;
    p.tile_floats = h->tile_floats;
    p.init_cash = c.init_cash; p.commission = c.commission; p.scale = c.reward_scale;
    p.rf = c.risk_free_rate; p.eta = c.sharpe_eta; p.mu_tol = c.mu_tol;
    p.value = h->value; p.k = h->k; p.ring = h->ring; p.sa = h->sa; p.sb = h->sb;
    p.nonfinite = h->nonfinite;
    p.div_wf = make_fastdiv((uint32_t)(c.window * c.features));
    p.div_f = make_fastdiv((uint32_t)c.features);
    p.div_w = make_fastdiv((uint32_t)c.window);
    return p;
}

inline bool aligned4(const void* ptr) { return ((uintptr_t)ptr & 3u) == 0; }

int check_launch(pmenv* h, const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_err(h, "%s launch failed: %s", what, hipGetErrorString(e));
        return PMENV_ERR_HIP;
    }
    return PMENV_OK;
}

}  // namespace

extern "C" {

int32_t pmenv_abi_version(void) { return PMENV_ABI_VERSION; }

void pmenv_cfg_default(pmenv_cfg* cfg, int32_t num_envs, int32_t num_assets, int32_t window, int32_t features) {
    if (!cfg) return;
    memset(cfg, 0, sizeof(*cfg));
    cfg->num_envs = num_envs;
    cfg->num_assets = num_assets;
    cfg->window = window;
    cfg->features = features;
    cfg->close_channel = features >= 5 ? 3 : 0;
    cfg->reward_kind = PMENV_REWARD_LOG_RETURN;
    cfg->norm_mode = PMENV_NORM_AND;
    cfg->ring_mode = PMENV_RING_STORAGE;
    cfg->ret_mode = PMENV_RET_GROSS;
    cfg->mu_max_iter = 100;
    cfg->init_cash = 25000.0;
    cfg->commission = 0.0;
    cfg->reward_scale = 1.0;
    cfg->risk_free_rate = 0.04;
    cfg->sharpe_eta = 0.01;
    cfg->mu_tol = 1e-10;
}

const char* pmenv_last_error(const pmenv* h) { return h ? h->err : g_create_err; }

int pmenv_get_cfg(const pmenv* h, pmenv_cfg* out) {
    if (!h || !out) return PMENV_ERR_ARG;
    *out = h->cfg;
    return PMENV_OK;
}

int pmenv_state_layout(const pmenv_cfg* cfg, size_t off[6]) {
    if (!cfg || !off || cfg->num_envs < 1 || cfg->num_assets < 1 || cfg->window < 1) return PMENV_ERR_ARG;
    const size_t B = (size_t)cfg->num_envs;
    const size_t ring_elems = B * (size_t)cfg->window * (size_t)cfg->num_assets;
    auto up16 = [](size_t x) { return (x + 15) / 16 * 16; };
    size_t o = 0;
    off[0] = o; o = up16(o + B * 8);
    off[1] = o; o = up16(o + B * 8);
    off[2] = o; o = up16(o + B * 8);
    off[3] = o; o = up16(o + B * 4);
    off[4] = o; o = up16(o + ring_elems * 4);
    off[5] = o;
    return PMENV_OK;
}

size_t pmenv_state_bytes_for(const pmenv_cfg* cfg) {
    size_t off[6];
    if (pmenv_state_layout(cfg, off) != PMENV_OK) return 0;
    return off[5] + 16;
}

int pmenv_create(const pmenv_cfg* cfg, int device, pmenv** out) {
    return pmenv_create_in(cfg, device, nullptr, 0, out);
}

int pmenv_create_in(const pmenv_cfg* cfg, int device, void* state, size_t state_bytes, pmenv** out) {
    if (!cfg || !out) return PMENV_ERR_ARG;
    *out = nullptr;
    pmenv* h = (pmenv*)calloc(1, sizeof(pmenv));
    if (!h) return PMENV_ERR_ARG;
    h->cfg = *cfg;
    h->device = device;
    const pmenv_cfg& c = h->cfg;
    auto fail = [&](int code) {
        // no handle reaches the caller: pmenv_last_error(NULL) reports this one
        snprintf(g_create_err, sizeof(g_create_err), "%s", h->err);
        if (h->state && h->owns_state) (void)hipFree(h->state);
        free(h);
        return code;
    };
    if (c.num_envs < 1 || c.num_assets < 1 || c.window < 1 || c.features < 2) {
        set_err(h, "invalid shape B=%d N=%d W=%d F=%d (need B,N,W >= 1, F >= 2)", c.num_envs, c.num_assets,
                c.window, c.features);
        return fail(PMENV_ERR_ARG);
    }
    if (c.close_channel < 0 || c.close_channel >= c.features - 1) {
        set_err(h, "close_channel %d must be a market channel in [0, F-2]", c.close_channel);
        return fail(PMENV_ERR_ARG);
    }
    if (c.reward_kind < 0 || c.reward_kind > 3 || c.norm_mode < 0 || c.norm_mode > 1 || c.ring_mode < 0 ||
        c.ring_mode > 1 || c.ret_mode < 0 || c.ret_mode > 1 || c.mu_max_iter < 0 || c.commission < 0.0 ||
        c.commission >= 1.0) {
        set_err(h, "invalid mode/commission value in cfg");
        return fail(PMENV_ERR_ARG);
    }
    const int64_t WF = (int64_t)c.window * c.features;
    if (WF > kTileFloats) {
        set_err(h, "window*features = %lld exceeds the %d-float LDS tile", (long long)WF, kTileFloats);
        return fail(PMENV_ERR_ARG);
    }
    if ((int64_t)c.num_assets * WF >= (1ll << 31)) {
        set_err(h, "per-env obs block too large");
        return fail(PMENV_ERR_ARG);
    }
    // tile geometry: whole asset rows, 16-B granular when every env block is
    int R = (int)(kTileFloats / WF);
    if (R > c.num_assets) R = c.num_assets;
    bool vec = ((int64_t)c.num_assets * WF) % 4 == 0;
    if (vec && R < c.num_assets) {
        while (R > 0 && ((int64_t)R * WF) % 4 != 0) --R;
        if (R == 0) { vec = false; R = (int)(kTileFloats / WF); }
    }
    h->rows_per_tile = R;
    h->vec = vec;
    h->tile_floats = (int)((((int64_t)R * WF) + 3) / 4 * 4);
    h->lds_advance = scratch_bytes(h->tile_floats, c.num_assets, c.features);
    h->lds_surface = scratch_bytes(0, c.num_assets, c.features);
    if (h->lds_advance > 160 * 1024) {
        set_err(h, "num_assets %d needs %zu B of LDS (> 160 KiB)", c.num_assets, h->lds_advance);
        return fail(PMENV_ERR_ARG);
    }

    DeviceGuard g(device);
    size_t off[6];
    pmenv_state_layout(&c, off);
    h->state_bytes = off[5] + 16;
    if (state) {
        if (state_bytes < h->state_bytes || ((uintptr_t)state & 15u)) {
            set_err(h, "caller state buffer too small (%zu < %zu) or not 16-B aligned", state_bytes, h->state_bytes);
            return fail(PMENV_ERR_ARG);
        }
        h->state = state;
        h->owns_state = false;
    } else {
        hipError_t ae = hipMalloc(&h->state, h->state_bytes);
        if (ae != hipSuccess) {
            set_err(h, "hipMalloc(%zu) failed: %s", h->state_bytes, hipGetErrorString(ae));
            h->state = nullptr;
            return fail(PMENV_ERR_HIP);
        }
        h->owns_state = true;
    }
    char* base = (char*)h->state;
    h->value = (double*)(base + off[0]);
    h->sa = (double*)(base + off[1]);
    h->sb = (double*)(base + off[2]);
    h->k = (int32_t*)(base + off[3]);
    h->ring = (float*)(base + off[4]);
    h->nonfinite = (unsigned long long*)(base + off[5]);
    hipError_t e;
    if (hipFuncSetAttribute((const void*)step_advance_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)h->lds_advance) != hipSuccess ||
        hipFuncSetAttribute((const void*)step_advance_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)h->lds_advance) != hipSuccess ||
        hipFuncSetAttribute((const void*)step_surface_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)h->lds_surface) != hipSuccess) {
        (void)hipGetLastError();  // attribute is advisory below 64 KiB
    }
    e = hipMemset(h->nonfinite, 0, 16);
    if (e != hipSuccess) {
        set_err(h, "hipMemset failed: %s", hipGetErrorString(e));
        return fail(PMENV_ERR_HIP);
    }
    StepParams p = base_params(h);
    reset_kernel<<<c.num_envs, kBlock, 0, nullptr>>>(p, nullptr, nullptr);
    e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        set_err(h, "initial reset failed: %s", hipGetErrorString(e));
        return fail(PMENV_ERR_HIP);
    }
    *out = h;
    return PMENV_OK;
}

int pmenv_destroy(pmenv* h) {
    if (!h) return PMENV_ERR_ARG;
    DeviceGuard g(h->device);
    if (h->state && h->owns_state) (void)hipFree(h->state);
    free(h);
    return PMENV_OK;
}

int pmenv_reset(pmenv* h, float* obs, const uint8_t* mask, hipStream_t stream) {
    if (!h) return PMENV_ERR_ARG;
    if (obs && !aligned4(obs)) { set_err(h, "obs not 4-byte aligned"); return PMENV_ERR_ALIGN; }
    DeviceGuard g(h->device);
    StepParams p = base_params(h);
    reset_kernel<<<h->cfg.num_envs, kBlock, 0, stream>>>(p, obs, mask);
    return check_launch(h, "reset_kernel");
}

int pmenv_step_ex(pmenv* h, const pmenv_step_args* a, hipStream_t stream) {
    if (!h) return PMENV_ERR_ARG;
    if (!a || !a->action) { set_err(h, "action is required"); return PMENV_ERR_ARG; }
    if (!a->bar && !a->prices) { set_err(h, "surface mode (bar == NULL) needs prices"); return PMENV_ERR_ARG; }
    if (a->bar && !a->obs) { set_err(h, "advance mode (bar != NULL) needs obs"); return PMENV_ERR_ARG; }
    if (!aligned4(a->action) || (a->prices && !aligned4(a->prices)) || (a->bar && !aligned4(a->bar)) ||
        (a->obs && !aligned4(a->obs)) || (a->reward && !aligned4(a->reward)) ||
        (a->weights && !aligned4(a->weights)) || (a->ret && ((uintptr_t)a->ret & 7u))) {
        set_err(h, "unaligned pointer");
        return PMENV_ERR_ALIGN;
    }
    DeviceGuard g(h->device);
    StepParams p = base_params(h);
    p.action = a->action; p.prices = a->prices; p.bar = a->bar; p.obs = a->obs;
    p.reward = a->reward; p.ret = a->ret; p.weights = a->weights;
    const int B = h->cfg.num_envs;
    if (a->bar) {
        const bool vec = h->vec && (((uintptr_t)a->obs & 15u) == 0);
        if (vec)
            step_advance_kernel<true><<<B, kBlock, h->lds_advance, stream>>>(p);
        else
            step_advance_kernel<false><<<B, kBlock, h->lds_advance, stream>>>(p);
        return check_launch(h, "step_advance_kernel");
    }
    step_surface_kernel<<<B, kBlock, h->lds_surface, stream>>>(p);
    return check_launch(h, "step_surface_kernel");
}

int pmenv_step(pmenv* h, const float* action, const float* prices, const float* bar, float* obs, float* reward,
               hipStream_t stream) {
    pmenv_step_args a;
    memset(&a, 0, sizeof(a));
    a.action = action; a.prices = prices; a.bar = bar; a.obs = obs; a.reward = reward;
    return pmenv_step_ex(h, &a, stream);
}

double* pmenv_value(pmenv* h) { return h ? h->value : nullptr; }
float* pmenv_ring(pmenv* h) { return h ? h->ring : nullptr; }
int32_t* pmenv_counter(pmenv* h) { return h ? h->k : nullptr; }
size_t pmenv_state_bytes(const pmenv* h) { return h ? h->state_bytes : 0; }

int pmenv_get_state(pmenv* h, void* dst, hipStream_t stream) {
    if (!h || !dst) return PMENV_ERR_ARG;
    DeviceGuard g(h->device);
    hipError_t e = hipMemcpyAsync(dst, h->state, h->state_bytes, hipMemcpyDeviceToDevice, stream);
    if (e != hipSuccess) { set_err(h, "get_state: %s", hipGetErrorString(e)); return PMENV_ERR_HIP; }
    return PMENV_OK;
}

int pmenv_set_state(pmenv* h, const void* src, hipStream_t stream) {
    if (!h || !src) return PMENV_ERR_ARG;
    DeviceGuard g(h->device);
    hipError_t e = hipMemcpyAsync(h->state, src, h->state_bytes, hipMemcpyDeviceToDevice, stream);
    if (e != hipSuccess) { set_err(h, "set_state: %s", hipGetErrorString(e)); return PMENV_ERR_HIP; }
    return PMENV_OK;
}

int pmenv_nonfinite_count(pmenv* h, uint64_t* out, hipStream_t stream) {
    if (!h || !out) return PMENV_ERR_ARG;
    DeviceGuard g(h->device);
    unsigned long long v = 0;
    hipError_t e = hipMemcpyAsync(&v, h->nonfinite, 8, hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) { set_err(h, "nonfinite_count: %s", hipGetErrorString(e)); return PMENV_ERR_HIP; }
    *out = v;
    return PMENV_OK;
}

int pmenv_synth_series(float* series, int32_t T, int32_t B, int32_t N, int64_t env_offset, uint64_t seed,
                       float sigma, hipStream_t stream) {
    if (!series || T < 1 || B < 1 || N < 1 || ((uintptr_t)series & 15u)) return PMENV_ERR_ARG;
    const int64_t threads = (int64_t)B * N;
    synth_series_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, stream>>>(
        reinterpret_cast<float4*>(series), T, B, N, env_offset, seed, (double)sigma);
    return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
}

int pmenv_synth_actions(float* actions, int32_t T, int32_t B, int32_t N, int64_t env_offset, uint64_t seed,
                        hipStream_t stream) {
    if (!actions || T < 1 || B < 1 || N < 1) return PMENV_ERR_ARG;
    const int64_t threads = (int64_t)T * B;
    synth_actions_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, stream>>>(actions, T, B, N, env_offset, seed);
    return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
}

int pmenv_window_init(float* obs, const float* series, int32_t B, int32_t N, int32_t W, int32_t F,
                      hipStream_t stream) {
    if (!obs || !series || B < 1 || N < 1 || W < 1 || F != 5 || ((uintptr_t)series & 15u)) return PMENV_ERR_ARG;
    const int64_t threads = (int64_t)B * N * W;
    window_init_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, stream>>>(
        obs, reinterpret_cast<const float4*>(series), B, N, W, F);
    return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
}

int pmenv_gae(const float* rewards, const float* values, const uint8_t* dones, float* adv, float* ret, int32_t T,
              int32_t B, float gamma, float lam, hipStream_t stream) {
    if (!rewards || !values || !adv || !ret || T < 1 || B < 1) return PMENV_ERR_ARG;
    gae_kernel<<<(B + 255) / 256, 256, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam);
    return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
}

int pmenv_moments(const float* x, int64_t n, double* out, hipStream_t stream) {
    if (!x || !out || n < 0) return PMENV_ERR_ARG;
    int64_t want = (n + kBlock * 4 - 1) / (kBlock * 4);
    int blocks = (int)(want < 1 ? 1 : (want > kMomBlocks ? kMomBlocks : want));
    moments_partial_kernel<<<blocks, kBlock, 0, stream>>>(x, n);
    moments_final_kernel<<<1, 64, 0, stream>>>(blocks, n, out);
    return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
}

}  // extern "C"
