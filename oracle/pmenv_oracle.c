/*
 * pmenv_oracle.c — TEST INFRASTRUCTURE ONLY (see pmenv_oracle.h).
 *
 * A scalar, obviously-correct restatement of the reference's env step, written
 * straight from the reference text, one env at a time, in f64:
 *   env/sim/trading_env.py:44-105   TradingEnv.step
 *   env/sim/trading_env.py:21-41    TradingEnv.reset
 *   env/sim/weight_buffer.py:13-51  ActionBuffer.update / get_last / get_all / reset
 *   env/reward.py:20-31             returns / log_returns / sharpe_ratio
 *   data/instrument.py:79           price relatives; :339-356 sliding window
 * The obs of "advance" mode is built the reference way — next window = old
 * window shifted one day + the new bar, channel F-1 = get_all() — not the way
 * the HIP kernel derives it, so the kernel's shortcut is actually checked.
 */
#include "pmenv_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

or_env* or_create(const pmenv_cfg* cfg) {
    or_env* e = (or_env*)calloc(1, sizeof(or_env));
    e->cfg = *cfg;
    /* PMENV_RET_AUTO: trading_env.py:88 (gross) for the log-return reward,
     * env/reward.py:20-31 over info["values"] (net) for the others */
    if (e->cfg.ret_mode == PMENV_RET_AUTO)
        e->cfg.ret_mode = cfg->reward_kind == PMENV_REWARD_LOG_RETURN ? PMENV_RET_GROSS : PMENV_RET_NET;
    size_t B = (size_t)cfg->num_envs, W = (size_t)cfg->window, N = (size_t)cfg->num_assets;
    e->value = (double*)calloc(B, sizeof(double));
    e->k = (int32_t*)calloc(B, sizeof(int32_t));
    e->ring = (float*)calloc(B * W * N, sizeof(float));
    e->sa = (double*)calloc(B, sizeof(double));
    e->sb = (double*)calloc(B, sizeof(double));
    or_reset(e, NULL, NULL);
    return e;
}

void or_destroy(or_env* e) {
    if (!e) return;
    free(e->value); free(e->k); free(e->ring); free(e->sa); free(e->sb); free(e);
}

/* ActionBuffer.get_all() (weight_buffer.py:32-44), after `k` updates since reset,
 * transposed to [N, W]: returns the weight of asset n at window position t. */
static float get_all_at(const pmenv_cfg* c, const float* ring, int32_t k, int n, int t) {
    int W = c->window, N = c->num_assets;
    int idx = (int)((1 + (int64_t)k) % W);          /* weight_buffer.py:22 */
    int full = (int64_t)k >= W - 1;                 /* weight_buffer.py:25-26 */
    if (!full) {                                    /* :40-42 zero padding in front */
        int pad = W - idx;
        return t < pad ? 0.0f : ring[(size_t)(t - pad) * N + n];
    }
    if (c->ring_mode == PMENV_RING_STORAGE)         /* :38-39 storage order */
        return ring[(size_t)t * N + n];
    return ring[(size_t)((idx + t) % W) * N + n];   /* chronological */
}

static void write_weight_channel(const pmenv_cfg* c, const float* ring, int32_t k, float* obs_env) {
    int N = c->num_assets, W = c->window, F = c->features;
    for (int n = 0; n < N; ++n)
        for (int t = 0; t < W; ++t)
            obs_env[((size_t)n * W + t) * F + (F - 1)] = get_all_at(c, ring, k, n, t);
}

static void reset_env(or_env* e, int b, float* obs) {
    const pmenv_cfg* c = &e->cfg;
    size_t WN = (size_t)c->window * c->num_assets;
    float* ring = e->ring + (size_t)b * WN;
    memset(ring, 0, WN * sizeof(float));            /* weight_buffer.py:47 */
    ring[0] = 1.0f;                                 /* :48 all cash */
    e->k[b] = 0;                                    /* :49 idx = 1 */
    e->value[b] = c->init_cash;                     /* trading_env.py:28 */
    e->sa[b] = 0.0; e->sb[b] = 0.0;                 /* info reset :34-39 */
    if (obs) write_weight_channel(c, ring, 0, obs + (size_t)b * c->num_assets * c->window * c->features);
}

void or_reset(or_env* e, float* obs, const uint8_t* mask) {
    for (int b = 0; b < e->cfg.num_envs; ++b)
        if (!mask || mask[b]) reset_env(e, b, obs);
}

static void step_env(or_env* e, int b, const float* action, const float* prices, const float* bar,
                     float* obs, float* reward, double* ret_out, float* weights_out,
                     double* w, double* y) {
    const pmenv_cfg* c = &e->cfg;
    const int N = c->num_assets, W = c->window, F = c->features, Fm = F - 1;
    const size_t env_obs = (size_t)N * W * F;
    float* ring = e->ring + (size_t)b * W * N;
    float* ob = obs ? obs + (size_t)b * env_obs : NULL;
    const float* a = action + (size_t)b * N;

    /* trading_env.py:54-55 flatten; :57-60 normalisation */
    double sum = 0.0, mn = INFINITY;
    int has_nan = 0;
    for (int n = 0; n < N; ++n) {
        w[n] = (double)a[n];
        sum += w[n];
        if (isnan(w[n])) has_nan = 1;
        if (w[n] < mn) mn = w[n];
    }
    if (has_nan) mn = NAN;
    int not_close = !(fabs(sum - 1.0) <= 1e-6 + 1e-5 * 1.0);   /* torch.isclose defaults */
    int negative = mn < 0.0;
    int norm = c->norm_mode == PMENV_NORM_AND ? (not_close && negative) : (not_close || negative);
    if (norm) {
        double shift = 0.0;
        if (c->norm_mode == PMENV_NORM_OR) {            /* torch.softmax subtracts the max */
            shift = -INFINITY;
            for (int n = 0; n < N; ++n) if (w[n] > shift) shift = w[n];
        }
        double z = 0.0;
        for (int n = 0; n < N; ++n) { w[n] = exp(w[n] - shift); z += w[n]; }
        for (int n = 0; n < N; ++n) w[n] /= z;         /* :59-60 exp(w)/sum(exp(w)) */
    }

    /* price relatives: given, or instrument.py:79 close_t / close_{t-1} */
    for (int n = 0; n < N; ++n) {
        if (prices) y[n] = (double)prices[(size_t)b * N + n];
        else {
            /* instrument.py:79 divides float32 tensors: the relative is fp32-rounded */
            float cn = bar[((size_t)b * N + n) * Fm + c->close_channel];
            float co = ob[((size_t)n * W + (W - 1)) * F + c->close_channel];
            y[n] = (double)(cn / co);
        }
    }

    /* :63 w_last = ring.get_last() = slot (idx-1) % W = k % W */
    const int32_t k = e->k[b];
    const float* wl = ring + (size_t)(k % W) * N;
    double V_prev = e->value[b];
    double V = V_prev;
    /* :67-75 commission fixed point (max(x, 0) as intended; the reference's
     * torch.maximum(x, ) raises TypeError — parity unpinned by the reference) */
    if (c->commission > 0.0) {
        double cm = c->commission;
        double mu_last = 1.0, mu = 1.0 - 2.0 * cm + cm * cm;
        int it = 0;
        while (fabs(mu - mu_last) > c->mu_tol && it < c->mu_max_iter) {
            mu_last = mu;
            double s = 0.0;
            for (int n = 1; n < N; ++n) {
                double d = (double)wl[n] - mu * w[n];
                s += d > 0.0 ? d : 0.0;
            }
            mu = (1.0 - cm * (double)wl[0] - (2.0 * cm - cm * cm) * s) / (1.0 - cm * w[0]);
            ++it;
        }
        V = mu * V;                                    /* :75 */
    }

    /* :78-79 portfolio = V * (w * y); value = sum */
    double value = 0.0;
    for (int n = 0; n < N; ++n) { w[n] = V * (w[n] * y[n]); value += w[n]; }
    /* :83 w' = portfolio / value ; :84 ring.update(w') */
    int slot = (int)((1 + (int64_t)k) % W);           /* weight_buffer.py:21 idx */
    for (int n = 0; n < N; ++n) {
        float wp = (float)(w[n] / value);
        ring[(size_t)slot * N + n] = wp;
        if (weights_out) weights_out[(size_t)b * N + n] = wp;
    }
    e->k[b] = k + 1;
    /* :88 ret = value / self.value (mu-scaled), :89 V <- value */
    double ret = c->ret_mode == PMENV_RET_GROSS ? value / V : value / V_prev;
    e->value[b] = value;

    /* reward: :99 log(ret) * REWARD_SCALE, or env/reward.py variants */
    double r;
    switch (c->reward_kind) {
    case PMENV_REWARD_RETURN: r = ret * c->reward_scale; break;
    case PMENV_REWARD_SHARPE: {
        /* reward.py:26-31 over the full history of ratios, as running (Welford) moments */
        double m = (double)(k + 1);
        double d = ret - e->sa[b];
        e->sa[b] += d / m;
        e->sb[b] += d * (ret - e->sa[b]);
        r = m < 2.0 ? NAN : (e->sa[b] - c->risk_free_rate) / sqrt(e->sb[b] / (m - 1.0)) * c->reward_scale;
        break;
    }
    case PMENV_REWARD_DIFF_SHARPE: {
        /* Moody & Saffell (1998): D_t = (B dA - A dB / 2) / (B - A^2)^{3/2} */
        double R = ret - 1.0, A = e->sa[b], Bm = e->sb[b];
        double dA = R - A, dB = R * R - Bm, var = Bm - A * A;
        r = var > 1e-12 ? (Bm * dA - 0.5 * A * dB) / (var * sqrt(var)) * c->reward_scale : 0.0;
        e->sa[b] = A + c->sharpe_eta * dA;
        e->sb[b] = Bm + c->sharpe_eta * dB;
        break;
    }
    default: r = log(ret) * c->reward_scale;
    }
    if (reward) reward[b] = (float)r;
    if (ret_out) ret_out[b] = ret;

    /* :103 obs update */
    if (!ob) return;
    if (bar) {
        /* sliding window (instrument.py:339-356): drop day 0, append the bar */
        for (int n = 0; n < N; ++n) {
            float* row = ob + (size_t)n * W * F;
            memmove(row, row + F, (size_t)(W - 1) * F * sizeof(float));
            for (int f = 0; f < Fm; ++f) row[(size_t)(W - 1) * F + f] = bar[((size_t)b * N + n) * Fm + f];
        }
    }
    write_weight_channel(c, ring, k + 1, ob);
}

static void step_range(or_env* e, const float* action, const float* prices, const float* bar,
                       float* obs, float* reward, double* ret, float* weights, int threads) {
    const int B = e->cfg.num_envs, N = e->cfg.num_assets;
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel num_threads(threads)
#endif
    {
        double* w = (double*)malloc(sizeof(double) * (size_t)N);
        double* y = (double*)malloc(sizeof(double) * (size_t)N);
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
        for (int b = 0; b < B; ++b) step_env(e, b, action, prices, bar, obs, reward, ret, weights, w, y);
        free(w); free(y);
    }
    (void)threads;
}

void or_step(or_env* e, const float* action, const float* prices, const float* bar,
             float* obs, float* reward, double* ret, float* weights) {
    step_range(e, action, prices, bar, obs, reward, ret, weights, 1);
}

void or_step_mt(or_env* e, const float* action, const float* prices, const float* bar,
                float* obs, float* reward, double* ret, float* weights, int threads) {
    step_range(e, action, prices, bar, obs, reward, ret, weights, threads);
}

/* GAE(gamma, lambda) reverse recursion — no reference counterpart is runnable
 * (rollout_buffer.py stores r/v but computes no returns; the nearest recursions,
 * dreamer.py:134-141 and td3.py:92-97, do not import). Parity unpinned. */
void or_gae(const float* rewards, const float* values, const uint8_t* dones,
            float* adv, float* ret, int32_t T, int32_t B, float gamma, float lam) {
    for (int b = 0; b < B; ++b) {
        double a = 0.0;
        for (int t = T - 1; t >= 0; --t) {
            size_t i = (size_t)t * B + b;
            double nd = dones ? (dones[i] ? 0.0 : 1.0) : 1.0;
            double delta = (double)rewards[i] + (double)gamma * nd * (double)values[i + B] - (double)values[i];
            a = delta + (double)gamma * (double)lam * nd * a;
            adv[i] = (float)a;
            ret[i] = (float)(a + (double)values[i]);
        }
    }
}

void or_moments(const float* x, int64_t n, double* out) {
    double s = 0.0, q = 0.0;
    for (int64_t i = 0; i < n; ++i) { s += x[i]; q += (double)x[i] * x[i]; }
    out[0] = (double)n; out[1] = s; out[2] = q;
}

/* Batched trainer reward: agent/pg/pg.py:40-82 `_reward`, written straight from the
 * reference text in f64; the gradient is the hand-derived chain rule of the same
 * expression (checked against torch autograd of the reference in the tests). */
double or_batch_reward(const float* a, const float* v_prev, const float* p, int32_t B, int32_t N,
                       int32_t kind, int32_t norm, double scale, float* ret_out, float* grad_a) {
    double tot = 0.0, mn = INFINITY;
    int nan_seen = 0;
    for (int64_t i = 0; i < (int64_t)B * N; ++i) {
        tot += a[i];
        if (isnan(a[i])) nan_seen = 1;
        if (a[i] < mn) mn = a[i];
    }
    if (nan_seen) mn = NAN;
    /* :52 if not isclose(sum(a), 1, atol=1e-6) or min(a) < 0: a = softmax(a, dim=1) */
    int glob = !(fabs(tot - 1.0) <= 1e-6 + 1e-5) || mn < 0.0;
    double* w = (double*)malloc(sizeof(double) * (size_t)B * N);
    double* ret = (double*)malloc(sizeof(double) * (size_t)B);
    int* nb = (int*)malloc(sizeof(int) * (size_t)B);
    for (int b = 0; b < B; ++b) {
        const float* ab = a + (size_t)b * N;
        double rs = 0.0, rmn = INFINITY, mx = -INFINITY;
        int rn = 0;
        for (int n = 0; n < N; ++n) {
            rs += ab[n];
            if (isnan(ab[n])) rn = 1;
            if (ab[n] < rmn) rmn = ab[n];
            if (ab[n] > mx) mx = ab[n];
        }
        if (rn) rmn = NAN;
        nb[b] = norm == 0 ? glob : norm == 1 ? (!(fabs(rs - 1.0) <= 1e-6 + 1e-5) || rmn < 0.0 || isnan(rmn)) : 0;
        double z = 0.0;
        for (int n = 0; n < N; ++n) z += exp(ab[n] - mx);
        double v = v_prev[b], pv = 0.0;
        for (int n = 0; n < N; ++n) {
            w[(size_t)b * N + n] = nb[b] ? exp(ab[n] - mx) / z : (double)ab[n];
            pv += v * (w[(size_t)b * N + n] * (double)p[(size_t)b * N + n]);   /* :68-69 */
        }
        ret[b] = pv / v;                                                        /* :72 */
        if (ret_out) ret_out[b] = (float)ret[b];
    }
    double sf = 0.0, sr = 0.0;
    for (int b = 0; b < B; ++b) { sf += kind == PMENV_REWARD_LOG_RETURN ? log(ret[b]) : ret[b]; sr += ret[b]; }
    double mean = sr / B, dev = 0.0;
    for (int b = 0; b < B; ++b) dev += (ret[b] - mean) * (ret[b] - mean);
    double sd = B > 1 ? sqrt(dev / (B - 1)) : NAN;
    double R = kind == PMENV_REWARD_SHARPE ? mean / sd * scale : sf / B * scale;   /* :75-80 */
    if (grad_a) {
        for (int b = 0; b < B; ++b) {
            double dr = kind == PMENV_REWARD_LOG_RETURN ? scale / ((double)B * ret[b])
                      : kind == PMENV_REWARD_RETURN ? scale / (double)B
                      : scale * (1.0 / ((double)B * sd) - mean * (ret[b] - mean) / ((double)(B - 1) * sd * sd * sd));
            double v = v_prev[b], wg = 0.0;
            for (int n = 0; n < N; ++n) wg += w[(size_t)b * N + n] * (dr * (v * (double)p[(size_t)b * N + n]) / v);
            for (int n = 0; n < N; ++n) {
                double g = dr * (v * (double)p[(size_t)b * N + n]) / v;
                grad_a[(size_t)b * N + n] = (float)(nb[b] ? w[(size_t)b * N + n] * (g - wg) : g);
            }
        }
    }
    free(w); free(ret); free(nb);
    return R;
}

/* ---- Philox4x32-10 (Salmon et al., SC'11) ---- */
static inline void mulhilo(uint32_t a, uint32_t b, uint32_t* hi, uint32_t* lo) {
    uint64_t p = (uint64_t)a * b;
    *hi = (uint32_t)(p >> 32); *lo = (uint32_t)p;
}

void or_philox4x32(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                   uint32_t k0, uint32_t k1, uint32_t out[4]) {
    for (int r = 0; r < 10; ++r) {
        uint32_t hi0, lo0, hi1, lo1;
        mulhilo(0xD2511F53u, c0, &hi0, &lo0);
        mulhilo(0xCD9E8D57u, c2, &hi1, &lo1);
        uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static inline double u01(uint32_t x) { return ((double)(x >> 8) + 0.5) * (1.0 / 16777216.0); }

static void normals4(uint32_t c0, uint32_t c1, uint64_t g, uint64_t seed, double z[4]) {
    uint32_t o[4];
    or_philox4x32(c0, c1, (uint32_t)g, (uint32_t)(g >> 32), (uint32_t)seed, (uint32_t)(seed >> 32), o);
    const double two_pi = 6.283185307179586476925286766559;
    double r0 = sqrt(-2.0 * log(u01(o[0]))), r1 = sqrt(-2.0 * log(u01(o[2])));
    z[0] = r0 * cos(two_pi * u01(o[1])); z[1] = r0 * sin(two_pi * u01(o[1]));
    z[2] = r1 * cos(two_pi * u01(o[3])); z[3] = r1 * sin(two_pi * u01(o[3]));
}

void or_synth_series(float* series, int32_t T, int32_t B, int32_t N,
                     int64_t env_offset, uint64_t seed, float sigma) {
    const double s = (double)sigma;
    for (int b = 0; b < B; ++b)
        for (int n = 0; n < N; ++n) {
            uint64_t g = (uint64_t)(env_offset + b);
            double z[4];
            normals4(0u, (uint32_t)n, g, seed, z);
            double close = 100.0 * exp(0.2 * z[0]);
            for (int t = 0; t < T; ++t) {
                normals4((uint32_t)(t + 1), (uint32_t)n, g, seed, z);
                double cl = close * exp(s * z[0] - 0.5 * s * s);
                double op = close * exp(0.3 * s * z[1]);
                double hi = (op > cl ? op : cl) * exp(fabs(0.5 * s * z[2]));
                double lo = (op < cl ? op : cl) * exp(-fabs(0.5 * s * z[3]));
                float* o = series + (((size_t)t * B + b) * N + n) * 4;
                o[0] = (float)op; o[1] = (float)hi; o[2] = (float)lo; o[3] = (float)cl;
                close = cl;
            }
        }
}

void or_synth_actions(float* actions, int32_t T, int32_t B, int32_t N,
                      int64_t env_offset, uint64_t seed) {
    double* z = (double*)malloc(sizeof(double) * (size_t)N);
    for (int t = 0; t < T; ++t)
        for (int b = 0; b < B; ++b) {
            uint64_t g = (uint64_t)(env_offset + b);
            double mx = -INFINITY, sum = 0.0;
            for (int n = 0; n < N; ++n) {
                double zz[4];
                normals4((uint32_t)t, 0x80000000u | (uint32_t)n, g, seed, zz);
                z[n] = zz[0];
                if (z[n] > mx) mx = z[n];
            }
            for (int n = 0; n < N; ++n) { z[n] = exp(z[n] - mx); sum += z[n]; }
            for (int n = 0; n < N; ++n) actions[((size_t)t * B + b) * N + n] = (float)(z[n] / sum);
        }
    free(z);
}
