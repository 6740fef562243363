// replay.h — device replay gather and trajectory metrics.
//
// replay_gather_kernel restates replay/buffer.py:39-79 (ReplayBuffer.sample) for
// vectorised envs: the buffer keeps, per recorded step h and env b, only the day
// index of the window the agent acted on, the action and the reward; a sample
// (h0, b) re-materialises
//   s  = window ending at day[h0+W-1, b]      with channel F-1 = actions[h0 .. h0+W-1, b]
//   s' = window ending at day[h0+W-1, b] + 1  with channel F-1 = actions[h0+1 .. h0+W, b]
//   a  = actions[h0+W, b],  r = rewards[h0+W-1, b]                (buffer.py:59-72)
// from the resident market series [T, N, F-1]. Recorded steps are a ring of H rows.
//
// metrics_kernel restates util/eval.py:14-37 per env over a [T, B] trajectory with
// quantstats' published definitions (quantstats is not installed here: parity unpinned).
#pragma once
#include "common.h"

namespace pmenv_dev {

// one thread per output float of s and s' (both [S, N, W, F]); a/r by the first threads
__global__ void replay_gather_kernel(const float* series, int T, int N, int F, int W, const int32_t* days,
                                     const float* actions, const float* rewards, int H, int B, const int32_t* h0,
                                     const int32_t* env, int S, float* s, float* s_next, float* a_out,
                                     float* r_out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per = (int64_t)N * W * F;
    const int Fm = F - 1;
    if (i < (int64_t)S * N) {                     // a = actions[h0+W], r = rewards[h0+W-1]
        const int j = (int)(i / N), n = (int)(i % N);
        const int b = env[j];
        const int ha = (h0[j] + W) % H;
        a_out[i] = actions[((size_t)ha * B + b) * N + n];
        if (n == 0) r_out[j] = rewards[(size_t)((h0[j] + W - 1) % H) * B + b];
    }
    if (i >= (int64_t)S * per) return;
    const int j = (int)(i / per);
    int rem = (int)(i - (int64_t)j * per);
    const int n = rem / (W * F);
    rem -= n * W * F;
    const int t = rem / F, f = rem - t * F;
    const int b = env[j];
    const int hl = (h0[j] + W - 1) % H;           // the step whose window is s
    const int dlast = days[(size_t)hl * B + b];
    float v, vn;
    if (f < Fm) {
        const int d = dlast - (W - 1) + t;        // window of day dlast, and of dlast + 1 for s'
        v = (d >= 0 && d < T) ? series[((size_t)d * N + n) * Fm + f] : NAN;
        vn = (d + 1 >= 0 && d + 1 < T) ? series[((size_t)(d + 1) * N + n) * Fm + f] : NAN;
    } else {
        v = actions[((size_t)((h0[j] + t) % H) * B + b) * N + n];
        vn = actions[((size_t)((h0[j] + t + 1) % H) * B + b) * N + n];
    }
    s[i] = v;
    s_next[i] = vn;
}

// one thread per env walks its column of the trajectory (coalesced across envs)
//   out[b] = {sharpe, sortino, max drawdown, average turnover, final value}
__global__ void metrics_kernel(const double* returns, const double* values, const float* weights, int T, int B,
                               int N, double rf, double periods, double* out) {
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
    // util/eval.py:32-37 average turnover over the weight history
    double turn = 0.0;
    for (int t = 1; t <= T; ++t)
        for (int n = 0; n < N; ++n)
            turn += fabs((double)weights[((size_t)t * B + b) * N + n] - (double)weights[((size_t)(t - 1) * B + b) * N + n]);
    out[(size_t)b * 5 + 0] = sharpe;
    out[(size_t)b * 5 + 1] = sortino;
    out[(size_t)b * 5 + 2] = mdd;
    out[(size_t)b * 5 + 3] = T > 0 ? turn / T : NAN;
    out[(size_t)b * 5 + 4] = values[(size_t)T * B + b];
}

}  // namespace pmenv_dev
