// trainer.h — the trainer-side twin of the env step: the differentiable batched
// portfolio reward of the PG / A2C agents (agent/pg/pg.py:40-82 `_reward`,
// agent/a2c.py/a2c.py:40-82 `_loss`), forward and backward, in f64.
//
//   a [B, N] raw policy scores, v_prev [B], p [B, N] price relatives
//   normalise: softmax over assets iff !isclose(sum(a), 1) OR min(a) < 0, where the
//              reference takes sum/min over the WHOLE batch (pg.py:52); per-row and
//              none are offered as well
//   ret_b  = sum_n(v_b * (w_bn * p_bn)) / v_b                         (pg.py:68-72)
//   R      = mean(ret * s) | mean(log(ret) * s) | mean(ret) / std(ret) * s  (pg.py:75-80)
// The commission branch (pg.py:57-65) raises TypeError in the reference and is not
// part of this op.
#pragma once
#include "common.h"

namespace pmenv_dev {

// work layout (f64): [0,B) ret chosen, [B,2B) row sum, [2B,3B) row min, [3B,4B) ret raw,
// [4B,5B) ret softmax, [5B,6B) row normalised flag, [6B..6B+8) globals:
// +0 normalised (global), +1 mean, +2 std, +3 reward
constexpr int kTrainBlock = 256;

// one wave per row; N <= 64 lanes per pass, looping for larger N
__global__ __launch_bounds__(256) void batch_reward_rows_kernel(const float* a, const float* v_prev, const float* p,
                                                                int B, int N, double* work) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= B) return;
    const double v = (double)v_prev[b];
    double s = 0.0, mn = INFINITY, mx = -INFINITY, raw = 0.0;
    int nan_seen = 0;
    for (int n = lane; n < N; n += 64) {
        const double x = (double)a[(size_t)b * N + n];
        s += x;
        mn = fmin(mn, x);
        mx = fmax(mx, x);
        nan_seen |= isnan(x);
        raw += v * (x * (double)p[(size_t)b * N + n]);
    }
    s = wave_sum(s);
    mn = wave_min(mn);
    mx = wave_max(mx);
    raw = wave_sum(raw);
    if (__any(nan_seen)) mn = NAN;
    double z = 0.0, sm = 0.0;
    for (int n = lane; n < N; n += 64) z += exp((double)a[(size_t)b * N + n] - mx);
    z = wave_sum(z);
    for (int n = lane; n < N; n += 64) {
        const double w = exp((double)a[(size_t)b * N + n] - mx) / z;     // torch.softmax(a, dim=1)
        sm += v * (w * (double)p[(size_t)b * N + n]);
    }
    sm = wave_sum(sm);
    if (lane == 0) {
        work[(size_t)B + b] = s;
        work[2 * (size_t)B + b] = mn;
        work[3 * (size_t)B + b] = raw / v;
        work[4 * (size_t)B + b] = sm / v;
    }
}

// single workgroup: the normalisation decision, the chosen returns and the reward
__global__ __launch_bounds__(kTrainBlock) void batch_reward_final_kernel(int B, int kind, int norm, double scale,
                                                                         double* work, float* reward_out,
                                                                         float* ret_out) {
    __shared__ double sh[kTrainBlock / 64][2];
    const int tid = threadIdx.x;
    auto block_sum2 = [&](double x, double y, double* ox, double* oy) {
        x = wave_sum(x);
        y = wave_sum(y);
        if ((tid & 63) == 0) { sh[tid >> 6][0] = x; sh[tid >> 6][1] = y; }
        __syncthreads();
        double sx = 0.0, sy = 0.0;
        for (int w = 0; w < kTrainBlock / 64; ++w) { sx += sh[w][0]; sy += sh[w][1]; }
        __syncthreads();
        *ox = sx;
        *oy = sy;
    };
    // global sum / min of a (pg.py:52 sums the whole [B, N, 1] tensor)
    double s = 0.0, mn = INFINITY;
    int nan_seen = 0;
    for (int b = tid; b < B; b += kTrainBlock) {
        s += work[(size_t)B + b];
        const double m = work[2 * (size_t)B + b];
        nan_seen |= isnan(m);
        mn = fmin(mn, m);
    }
    double mn_all;
    {
        double m = wave_min(mn);
        int has_nan = __any(nan_seen);
        if ((tid & 63) == 0) { sh[tid >> 6][0] = m; sh[tid >> 6][1] = has_nan; }
        __syncthreads();
        double mm = INFINITY, hn = 0.0;
        for (int w = 0; w < kTrainBlock / 64; ++w) { mm = fmin(mm, sh[w][0]); hn += sh[w][1]; }
        __syncthreads();
        mn_all = hn > 0.0 ? NAN : mm;
    }
    double s_all, dummy;
    block_sum2(s, 0.0, &s_all, &dummy);
    const bool glob = !(fabs(s_all - 1.0) <= 1e-6 + 1e-5) || mn_all < 0.0;
    // chosen returns
    double fs = 0.0, rs = 0.0;
    for (int b = tid; b < B; b += kTrainBlock) {
        bool nb;
        if (norm == PMENV_BNORM_GLOBAL_OR) nb = glob;
        else if (norm == PMENV_BNORM_ROW_OR) {
            const double rsum = work[(size_t)B + b], rmin = work[2 * (size_t)B + b];
            nb = !(fabs(rsum - 1.0) <= 1e-6 + 1e-5) || rmin < 0.0 || isnan(rmin);
        } else nb = false;
        const double r = nb ? work[4 * (size_t)B + b] : work[3 * (size_t)B + b];
        work[b] = r;
        work[5 * (size_t)B + b] = nb ? 1.0 : 0.0;
        if (ret_out) ret_out[b] = (float)r;
        fs += kind == PMENV_REWARD_LOG_RETURN ? log(r) : r;
        rs += r;
    }
    double f_all, r_all;
    block_sum2(fs, rs, &f_all, &r_all);
    const double mean = r_all / B;
    double dev = 0.0;
    for (int b = tid; b < B; b += kTrainBlock) { const double d = work[b] - mean; dev += d * d; }
    double dev_all;
    block_sum2(dev, 0.0, &dev_all, &dummy);
    const double sd = B > 1 ? sqrt(dev_all / (B - 1)) : NAN;           // torch.std: unbiased
    double R;
    if (kind == PMENV_REWARD_SHARPE) R = mean / sd * scale;               // pg.py:80
    else R = f_all / B * scale;                                           // pg.py:76, :78
    if (tid == 0) {
        work[6 * (size_t)B + 0] = glob ? 1.0 : 0.0;
        work[6 * (size_t)B + 1] = mean;
        work[6 * (size_t)B + 2] = sd;
        work[6 * (size_t)B + 3] = R;
        *reward_out = (float)R;
    }
}

// one wave per row: dR/da through the (optional) softmax
__global__ __launch_bounds__(256) void batch_reward_grad_kernel(const float* a, const float* v_prev, const float* p,
                                                                int B, int N, int kind, double scale,
                                                                const double* work, const float* grad_out,
                                                                float* grad_a) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= B) return;
    const double go = (double)*grad_out;
    const double r = work[b];
    double dr;
    if (kind == PMENV_REWARD_LOG_RETURN) dr = scale / ((double)B * r);
    else if (kind == PMENV_REWARD_RETURN) dr = scale / (double)B;
    else {
        const double m = work[6 * (size_t)B + 1], sd = work[6 * (size_t)B + 2];
        dr = scale * (1.0 / ((double)B * sd) - m * (r - m) / ((double)(B - 1) * sd * sd * sd));
    }
    dr *= go;
    const double v = (double)v_prev[b];
    const bool nb = work[5 * (size_t)B + b] != 0.0;
    if (!nb) {
        for (int n = lane; n < N; n += 64)
            grad_a[(size_t)b * N + n] = (float)(dr * (v * (double)p[(size_t)b * N + n]) / v);
        return;
    }
    double mx = -INFINITY;
    for (int n = lane; n < N; n += 64) mx = fmax(mx, (double)a[(size_t)b * N + n]);
    mx = wave_max(mx);
    double z = 0.0;
    for (int n = lane; n < N; n += 64) z += exp((double)a[(size_t)b * N + n] - mx);
    z = wave_sum(z);
    double wg = 0.0;                               // sum_m w_m g_m
    for (int n = lane; n < N; n += 64) {
        const double w = exp((double)a[(size_t)b * N + n] - mx) / z;
        wg += w * (dr * (v * (double)p[(size_t)b * N + n]) / v);
    }
    wg = wave_sum(wg);
    for (int n = lane; n < N; n += 64) {
        const double w = exp((double)a[(size_t)b * N + n] - mx) / z;
        const double gn = dr * (v * (double)p[(size_t)b * N + n]) / v;
        grad_a[(size_t)b * N + n] = (float)(w * (gn - wg));
    }
}

}  // namespace pmenv_dev
