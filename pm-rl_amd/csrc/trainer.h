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
// +0 normalised (global), +1 mean, +2 std, +3 reward; then one partial record of
// kPartStride doubles per block of kRowsPerBlock rows.
constexpr int kTrainBlock = 256;
constexpr int kRowsPerBlock = 16;   // 4 waves x 4 rows
constexpr int kPartStride = 16;     // sum a, min a, nan, then 3 x {n, mean, M2, sum f}
constexpr int kCandRaw = 0, kCandSoftmax = 1, kCandRow = 2;

__host__ __device__ inline size_t batch_reward_blocks(int B) { return ((size_t)B + kRowsPerBlock - 1) / kRowsPerBlock; }
__host__ __device__ inline size_t batch_reward_work_doubles(int B) {
    return (size_t)6 * B + 8 + batch_reward_blocks(B) * kPartStride;
}

__device__ __forceinline__ bool row_normalises(double rsum, double rmin) {
    return !(fabs(rsum - 1.0) <= 1e-6 + 1e-5) || rmin < 0.0 || isnan(rmin);
}

// Chan et al. parallel merge of (n, mean, M2) — fixed operand order, deterministic
__device__ __forceinline__ void chan_merge(double& n, double& mean, double& m2, double n2, double mean2, double m22) {
    if (n2 == 0.0) return;
    if (n == 0.0) { n = n2; mean = mean2; m2 = m22; return; }
    const double nn = n + n2, d = mean2 - mean;
    mean += d * (n2 / nn);
    m2 += m22 + d * d * (n * n2 / nn);
    n = nn;
}

// one wave per row (4 rows per wave, 16 per block); N <= 64 lanes per pass, looping
// for larger N. Wave 0 then folds the block's rows into one partial record:
// sums / min for the normalisation decision and, for each candidate return vector
// (raw, softmax, per-row choice), count, mean, M2 (two-pass inside the block) and
// the sum of f(ret) (log for the log-return reward).
__global__ __launch_bounds__(kTrainBlock) void batch_reward_rows_kernel(const float* a, const float* v_prev,
                                                                        const float* p, int B, int N, int kind,
                                                                        double* work) {
    __shared__ double sh[4][kRowsPerBlock];       // row sum, row min, raw, softmax
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int j = 0; j < kRowsPerBlock / 4; ++j) {
        const int rl = wave * (kRowsPerBlock / 4) + j;
        const int b = blockIdx.x * kRowsPerBlock + rl;
        if (b >= B) break;
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
            sh[0][rl] = s;
            sh[1][rl] = mn;
            sh[2][rl] = raw / v;
            sh[3][rl] = sm / v;
        }
    }
    __syncthreads();
    if (wave != 0) return;
    const int b = blockIdx.x * kRowsPerBlock + lane;
    const bool ok = lane < kRowsPerBlock && b < B;
    const double cnt = (double)min(kRowsPerBlock, B - (int)blockIdx.x * kRowsPerBlock);
    double* part = work + (size_t)6 * B + 8 + (size_t)blockIdx.x * kPartStride;
    const int li = ok ? lane : 0;
    const double rs = ok ? sh[0][li] : 0.0, rm = ok ? sh[1][li] : INFINITY;
    const double s_all = wave_sum(rs);
    const int has_nan = __any(ok && isnan(rm));
    const double mn_all = wave_min(ok && !isnan(rm) ? rm : INFINITY);
    double x[3];
    x[kCandRaw] = ok ? sh[2][li] : 0.0;
    x[kCandSoftmax] = ok ? sh[3][li] : 0.0;
    x[kCandRow] = row_normalises(rs, rm) ? x[kCandSoftmax] : x[kCandRaw];
    double rec[kPartStride];
    rec[0] = s_all;
    rec[1] = mn_all;
    rec[2] = has_nan ? 1.0 : 0.0;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const double mean = wave_sum(ok ? x[c] : 0.0) / cnt;
        const double d = ok ? x[c] - mean : 0.0;
        const double m2 = wave_sum(d * d);
        const double f = wave_sum(ok ? (kind == PMENV_REWARD_LOG_RETURN ? log(x[c]) : x[c]) : 0.0);
        rec[3 + 4 * c + 0] = cnt;
        rec[3 + 4 * c + 1] = mean;
        rec[3 + 4 * c + 2] = m2;
        rec[3 + 4 * c + 3] = f;
    }
    rec[15] = 0.0;
    if (lane < kPartStride) {
        double val = rec[0];
#pragma unroll
        for (int i = 1; i < kPartStride; ++i) val = lane == i ? rec[i] : val;
        part[lane] = val;
    }
}

// single workgroup over the block partials: the normalisation decision, the reward
// and the chosen candidate's mean / std. Thread t folds partials t, t + 256, ... in
// order, then a fixed-shape LDS tree folds the 256 threads: deterministic.
__global__ __launch_bounds__(kTrainBlock) void batch_reward_final_kernel(int B, int kind, int norm, double scale,
                                                                         double* work, float* reward_out) {
    __shared__ double sh[kTrainBlock][kPartStride];
    const int tid = threadIdx.x;
    const size_t nblk = batch_reward_blocks(B);
    const double* parts = work + (size_t)6 * B + 8;
    double acc[kPartStride];
    acc[0] = 0.0; acc[1] = INFINITY; acc[2] = 0.0;
    for (int c = 0; c < 3; ++c) { acc[3 + 4 * c] = 0.0; acc[4 + 4 * c] = 0.0; acc[5 + 4 * c] = 0.0; acc[6 + 4 * c] = 0.0; }
    acc[15] = 0.0;
    auto fold = [&](const double* q) {
        acc[0] += q[0];
        acc[1] = fmin(acc[1], q[1]);
        acc[2] += q[2];
        for (int c = 0; c < 3; ++c) {
            chan_merge(acc[3 + 4 * c], acc[4 + 4 * c], acc[5 + 4 * c], q[3 + 4 * c], q[4 + 4 * c], q[5 + 4 * c]);
            acc[6 + 4 * c] += q[6 + 4 * c];
        }
    };
    for (size_t k = tid; k < nblk; k += kTrainBlock) fold(parts + k * kPartStride);
    for (int i = 0; i < kPartStride; ++i) sh[tid][i] = acc[i];
    __syncthreads();
    for (int o = kTrainBlock / 2; o > 0; o >>= 1) {
        if (tid < o) {
            for (int i = 0; i < kPartStride; ++i) acc[i] = sh[tid][i];
            fold(sh[tid + o]);
            for (int i = 0; i < kPartStride; ++i) sh[tid][i] = acc[i];
        }
        __syncthreads();
    }
    if (tid != 0) return;
    for (int i = 0; i < kPartStride; ++i) acc[i] = sh[0][i];
    // pg.py:52 sums / mins the WHOLE [B, N, 1] tensor; torch.min propagates NaN
    const double mn_all = acc[2] > 0.0 ? NAN : acc[1];
    const bool glob = !(fabs(acc[0] - 1.0) <= 1e-6 + 1e-5) || mn_all < 0.0;
    const int c = norm == PMENV_BNORM_GLOBAL_OR ? (glob ? kCandSoftmax : kCandRaw)
                : norm == PMENV_BNORM_ROW_OR ? kCandRow : kCandRaw;
    const double mean = acc[4 + 4 * c];
    const double sd = B > 1 ? sqrt(acc[5 + 4 * c] / (B - 1)) : NAN;     // torch.std: unbiased
    double R;
    if (kind == PMENV_REWARD_SHARPE) R = mean / sd * scale;               // pg.py:80
    else R = acc[6 + 4 * c] / B * scale;                                  // pg.py:76, :78
    work[6 * (size_t)B + 0] = glob ? 1.0 : 0.0;
    work[6 * (size_t)B + 1] = mean;
    work[6 * (size_t)B + 2] = sd;
    work[6 * (size_t)B + 3] = R;
    *reward_out = (float)R;
}

// elementwise: each row's chosen return and normalisation flag (for the backward)
__global__ __launch_bounds__(256) void batch_reward_select_kernel(int B, int norm, double* work, float* ret_out) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= B) return;
    bool nb;
    if (norm == PMENV_BNORM_GLOBAL_OR) nb = work[6 * (size_t)B] != 0.0;
    else if (norm == PMENV_BNORM_ROW_OR) nb = row_normalises(work[(size_t)B + b], work[2 * (size_t)B + b]);
    else nb = false;
    const double r = nb ? work[4 * (size_t)B + b] : work[3 * (size_t)B + b];
    work[b] = r;
    work[5 * (size_t)B + b] = nb ? 1.0 : 0.0;
    if (ret_out) ret_out[b] = (float)r;
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
