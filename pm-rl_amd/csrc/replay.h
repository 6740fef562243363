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
static __global__ void replay_gather_kernel(const float* series, int T, int N, int F, int W, const int32_t* days,
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

// The compact on-policy rollout (the device rollout keeps actions,
// rewards and values, not windows): env b's window after t steps is re-materialised
// from the resident market series and the env's post-drift weight history —
//   market f < F-1:  series[start[b] + t + p, n, f]          (p = day in the window)
//   weight f = F-1:  ActionBuffer.get_all() after t updates (weight_buffer.py:32-44)
// with the history rows r = 0 .. T_rec+W-1 of env b: rows < W-1 zero, row W-1 = e0 (the
// reset ring, weight_buffer.py:46-51), row W-1+j = w' of update j (weights [T_rec, B, N]).
// Chronological position c of the window after u = t updates reads row t + c; once the
// ring is full (u >= W-1) the reference returns it in storage order (:38-39): position
// p holds update j with j % W == p, i.e. chronological c = (p - u - 1) mod W.
// Days outside the series read NaN.

constexpr int kRowGatherUnroll = 8;   // rows of W*F <= 512 floats: all loads first

// The map above, one wave per (sample, asset) row of W*F floats: a lane writes floats
// lane, lane + 64, ... of the row (each store one contiguous 256-B run), the day and
// channel from the row offset by one multiply-shift, the sample's env / step / start
// wave-uniform. The float-per-thread form (tools build) spends its time in 64-bit divisions.
static __global__ __launch_bounds__(256) void rollout_gather_rows_kernel(const float* series, int T, int N, int F, int W,
                                                                  const int32_t* start, const float* weights,
                                                                  int B, int ring_mode, const int32_t* t_idx,
                                                                  const int32_t* env, int S, float* s, FastDiv div_f) {
    const int64_t rowi = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (rowi >= (int64_t)S * N) return;
    const int lane = threadIdx.x & 63;
    const int j = __builtin_amdgcn_readfirstlane((int)(rowi / N));
    const int n = __builtin_amdgcn_readfirstlane((int)(rowi - (int64_t)j * N));
    const int b = env[j], t = t_idx[j];
    const int d0 = start[b] + t;
    const int Fm = F - 1, WF = W * F;
    const bool storage = ring_mode == PMENV_RING_STORAGE && t >= W - 1;
    float* out = s + rowi * WF;
    // the value of row float i: a series or a weight-history float, or a constant
    auto fetch = [&](int i) -> float {
        const int p = (int)fdiv((uint32_t)i, div_f), f = i - p * F;
        if (f < Fm) {
            const int d = d0 + p;
            return (d >= 0 && d < T) ? series[((size_t)d * N + n) * Fm + f] : NAN;
        }
        const int c = storage ? (((p - t - 1) % W) + W) % W : p;
        const int r = t + c;                       // history row
        if (r < W - 1) return 0.0f;
        if (r == W - 1) return n == 0 ? 1.0f : 0.0f;
        return weights[((size_t)(r - W) * B + b) * N + n];
    };
    if (WF <= 64 * kRowGatherUnroll) {             // every load of the row in flight before the stores
        float v[kRowGatherUnroll];
#pragma unroll
        for (int k = 0; k < kRowGatherUnroll; ++k) v[k] = lane + 64 * k < WF ? fetch(lane + 64 * k) : 0.0f;
#pragma unroll
        for (int k = 0; k < kRowGatherUnroll; ++k)
            if (lane + 64 * k < WF) out[lane + 64 * k] = v[k];
        return;
    }
    for (int i = lane; i < WF; i += 64) out[i] = fetch(i);
}

// One workgroup per sample (F = 5, the sample's [W, N] weight block and [W, N, 4] market
// block fit LDS): both blocks are staged with coalesced reads — the market block is W
// consecutive series days, contiguous in [T, N, 4]; each history row's N weights are one
// contiguous run of [T_rec, B, N] — and the [N, W, 5] window is written as 16-B chunks
// from LDS (a lane's four floats walk (asset, day, channel) incrementally). Every weight
// line is fetched once per sample, where the per-row form fetches it per asset row.
// NT: cache-policy bits of the window stores (0: plain stores; the product: 16, sc1, for
// windows <= 128 MiB, else 2, nt; the tools build A/Bs the others)
template <int NT = 0>
__global__ __launch_bounds__(256) void rollout_gather_tile_kernel(const float* series, int T, int N, int W,
                                                                  const int32_t* start, const float* weights, int B,
                                                                  int ring_mode, const int32_t* t_idx,
                                                                  const int32_t* env, float* s, FastDiv div_n,
                                                                  FastDiv div_wf, FastDiv div_f) {
    constexpr int F = 5;
    extern __shared__ __attribute__((aligned(16))) float sh[];   // market [W][N][4], then weights [W][N]
    float* sh_m = sh;
    float* sh_w = sh + (size_t)W * N * 4;
    const int tid = threadIdx.x;
    const int j = blockIdx.x;
    const int b = env[j], t = t_idx[j];
    const int d0 = start[b] + t;
    const bool storage = ring_mode == PMENV_RING_STORAGE && t >= W - 1;
    const int nd = W * N;                          // market: one f4 per (day, asset); weights: one float
    const f4* src = reinterpret_cast<const f4*>(series) + (size_t)d0 * N;
    f4* sh_m4 = reinterpret_cast<f4*>(sh_m);
    // every load of a round in flight before its LDS writes (4 per thread and array)
    for (int i0 = 0; i0 < nd; i0 += 4 * 256) {
        f4 m[4];
        float w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = i0 + k * 256 + tid;
            m[k] = f4{NAN, NAN, NAN, NAN};
            w[k] = 0.0f;
            if (i < nd) {
                const int p = (int)fdiv((uint32_t)i, div_n), n = i - p * N;
                const int d = d0 + p;
                if (d >= 0 && d < T) m[k] = src[i];        // days outside the series read NaN
                const int c = storage ? (((p - t - 1) % W) + W) % W : p;
                const int r = t + c;                       // history row
                if (r == W - 1) w[k] = n == 0 ? 1.0f : 0.0f;
                else if (r > W - 1) w[k] = weights[((size_t)(r - W) * B + b) * N + n];
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = i0 + k * 256 + tid;
            if (i < nd) {
                sh_m4[i] = m[k];
                sh_w[i] = w[k];
            }
        }
    }
    __syncthreads();
    const int WF = W * F;
    const int nq = N * WF / 4;
    f4* out = reinterpret_cast<f4*>(s + (size_t)j * N * WF);
    for (int q = tid; q < nq; q += 256) {
        const int e = 4 * q;
        int n = (int)fdiv((uint32_t)e, div_wf);
        int rem = e - n * WF;
        int p = (int)fdiv((uint32_t)rem, div_f);
        int f = rem - p * F;
        float v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v[k] = f < F - 1 ? sh_m[(p * N + n) * 4 + f] : sh_w[p * N + n];
            if (++f == F) {
                f = 0;
                if (++p == W) {
                    p = 0;
                    ++n;
                }
            }
        }
        if constexpr (NT == 0) out[q] = f4{v[0], v[1], v[2], v[3]};
        else buf_store4<NT>(make_rsrc(out, (uint32_t)nq * 16u), (uint32_t)q * 16u, f4{v[0], v[1], v[2], v[3]});
    }
}



// The same per-env metrics with the horizon split over the four waves of a
// workgroup (lane = env: every load is a coalesced 512-B row; four times the waves
// in flight of the thread-per-env walk). Wave w walks days [w*T/4, (w+1)*T/4):
//   sharpe / sortino: shifted sums S1 = sum(x - K), S2 = sum((x - K)^2) with K the
//   env's first excess return (no division in the loop), and sum(min(x, 0)^2);
//   max drawdown: each wave's segment maximum goes through LDS, then the wave
//   re-walks its segment (an L2 re-read) with the running peak seeded by the
//   maximum of every earlier segment.
// Wave 0 adds the four segments' sums in wave order: deterministic.
__device__ __forceinline__ void metrics_seg_body(const double* returns, const double* values, int T, int B, double rf,
                                                 double periods, double* out, int bid) {
    __shared__ double sh[5][4][64];              // S1, S2, down, segment max (of values), mdd
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int b = bid * 64 + lane;
    const bool ok = b < B;
    const int bb = ok ? b : B - 1;
    const double rfp = rf != 0.0 ? pow(1.0 + rf, 1.0 / periods) - 1.0 : 0.0;
    const double K = returns[bb] - rfp;
    // returns: T rows, values: T + 1 rows; split both the same way
    const int r0 = (int)((int64_t)T * w / 4), r1 = (int)((int64_t)T * (w + 1) / 4);
    double s1 = 0.0, s2 = 0.0, dn = 0.0;
    int t = r0;
    for (; t + 4 <= r1; t += 4) {
        double x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) x[u] = returns[(size_t)(t + u) * B + bb] - rfp;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const double d = x[u] - K;
            s1 += d;
            s2 += d * d;
            dn += x[u] < 0.0 ? x[u] * x[u] : 0.0;
        }
    }
    for (; t < r1; ++t) {
        const double x = returns[(size_t)t * B + bb] - rfp;
        const double d = x - K;
        s1 += d;
        s2 += d * d;
        dn += x < 0.0 ? x * x : 0.0;
    }
    const int v0 = (int)((int64_t)(T + 1) * w / 4), v1 = (int)((int64_t)(T + 1) * (w + 1) / 4);
    double vmax = -INFINITY;
    for (t = v0; t < v1; ++t) vmax = fmax(vmax, values[(size_t)t * B + bb]);
    sh[0][w][lane] = s1;
    sh[1][w][lane] = s2;
    sh[2][w][lane] = dn;
    sh[3][w][lane] = vmax;
    __syncthreads();
    // qs.stats.max_drawdown: min_t (V_t / max_{s<=t} V_s - 1), the peak seeded by
    // every earlier segment
    double peak = -INFINITY;
    for (int j = 0; j < w; ++j) peak = fmax(peak, sh[3][j][lane]);
    double mdd = 0.0;
    for (t = v0; t < v1; ++t) {
        const double v = values[(size_t)t * B + bb];
        peak = fmax(peak, v);
        mdd = fmin(mdd, v / peak - 1.0);
    }
    sh[4][w][lane] = mdd;
    __syncthreads();
    if (w != 0 || !ok) return;
    double S1 = 0.0, S2 = 0.0, DN = 0.0, MDD = 0.0;
    for (int j = 0; j < 4; ++j) {
        S1 += sh[0][j][lane];
        S2 += sh[1][j][lane];
        DN += sh[2][j][lane];
        MDD = fmin(MDD, sh[4][j][lane]);
    }
    const double mean = K + S1 / T;
    const double sd = T > 1 ? sqrt(fmax(S2 - S1 * S1 / T, 0.0) / (T - 1)) : NAN;
    out[(size_t)b * 5 + 0] = mean / sd * sqrt(periods);
    out[(size_t)b * 5 + 1] = mean / sqrt(DN / T) * sqrt(periods);
    out[(size_t)b * 5 + 2] = MDD;
    out[(size_t)b * 5 + 4] = values[(size_t)T * B + b];
}


// util/eval.py:32-37 average turnover, element-parallel: a workgroup owns `eb` whole
// envs (N <= 256: one thread per (env, asset), so each day's read is eb*N contiguous
// floats) and every thread walks the days keeping the previous weight in a
// register; the env's assets are then summed in a fixed order. N > 256: one env
// per workgroup, threads stride over the assets.
__device__ __forceinline__ void metrics_turnover_body(const float* weights, int T, int B, int N, int tpe, int eb,
                                                      double* out, int bid) {
    __shared__ double sh[256];
    const int tid = threadIdx.x;
    const int el = tid % tpe, le = tid / tpe;
    const int b = bid * eb + le;
    double acc = 0.0;
    if (le < eb && b < B) {
        for (int n = el; n < N; n += tpe) {
            const float* w = weights + (size_t)b * N + n;
            const size_t step = (size_t)B * N;
            float prev = w[0];
            int t = 1;
            for (; t + 3 <= T; t += 4) {
                const float x1 = w[(size_t)t * step], x2 = w[(size_t)(t + 1) * step];
                const float x3 = w[(size_t)(t + 2) * step], x4 = w[(size_t)(t + 3) * step];
                acc += fabs((double)x1 - (double)prev) + fabs((double)x2 - (double)x1) +
                       fabs((double)x3 - (double)x2) + fabs((double)x4 - (double)x3);
                prev = x4;
            }
            for (; t <= T; ++t) {
                const float x = w[(size_t)t * step];
                acc += fabs((double)x - (double)prev);
                prev = x;
            }
        }
    }
    sh[tid] = acc;
    __syncthreads();
    if (el == 0 && le < eb && b < B) {
        double tot = 0.0;
        for (int i = 0; i < tpe; ++i) tot += sh[le * tpe + i];
        out[(size_t)b * 5 + 3] = tot / T;
    }
}


// Both metric passes in one launch: they read disjoint inputs and write disjoint
// fields of out, so the latency-bound segment walk (returns, values) runs beside the
// bandwidth-bound turnover stream (weights) instead of before it. Blocks [0, nseg)
// take the segment walk when seg_first, else the turnover blocks come first.
static __global__ __launch_bounds__(256) void metrics_fused_kernel(const double* returns, const double* values,
                                                            const float* weights, int T, int B, int N, double rf,
                                                            double periods, int tpe, int eb, int nseg, int nturn,
                                                            int seg_first, double* out) {
    const int bid = (int)blockIdx.x;
    const bool seg = seg_first ? bid < nseg : bid >= nturn;
    if (seg) metrics_seg_body(returns, values, T, B, rf, periods, out, seg_first ? bid : bid - nturn);
    else metrics_turnover_body(weights, T, B, N, tpe, eb, out, seg_first ? bid - nseg : bid);
}

// replay/buffer.py:53-79, one workgroup per sample: the W+1 days the pair (s, s')
// spans — market channels from the series, channel F-1 from the recorded actions —
// are staged in LDS as [N][W+1][F], then s (days 0..W-1) and s' (days 1..W) are
// written as whole 16-B chunks when the sample block is 16-B granular.
static __global__ __launch_bounds__(256) void replay_gather_lds_kernel(const float* series, int T, int N, int F, int W,
                                                                const int32_t* days, const float* actions,
                                                                const float* rewards, int H, int B,
                                                                const int32_t* h0, const int32_t* env, float* s,
                                                                float* s_next, float* a_out, float* r_out) {
    extern __shared__ __attribute__((aligned(16))) float ext[];
    const int j = blockIdx.x, tid = threadIdx.x;
    const int b = env[j], hj = h0[j];
    const int Fm = F - 1, W1 = W + 1;
    const int dlast = days[(size_t)((hj + W - 1) % H) * B + b];
    for (int it = tid; it < N * W1; it += 256) {                 // t-major: a day's assets are contiguous
        const int t = it / N, n = it - t * N;
        const int d = dlast - (W - 1) + t;
        float* dst = ext + ((size_t)n * W1 + t) * F;
        const bool in = d >= 0 && d < T;
        const float* src = series + ((size_t)(in ? d : 0) * N + n) * Fm;
        for (int f = 0; f < Fm; ++f) dst[f] = in ? src[f] : NAN;
        dst[Fm] = actions[((size_t)((hj + t) % H) * B + b) * N + n];
    }
    if (tid < N) a_out[(size_t)j * N + tid] = actions[((size_t)((hj + W) % H) * B + b) * N + tid];
    if (tid == 0) r_out[j] = rewards[(size_t)((hj + W - 1) % H) * B + b];
    __syncthreads();
    const int WF = W * F, per = N * WF;
    float* so = s + (size_t)j * per;
    float* sn = s_next + (size_t)j * per;
    if ((per & 3) == 0) {
        for (int q = tid; q < per / 4; q += 256) {
            float v0[4], v1[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int e = 4 * q + k;
                const int n = e / WF, rem = e - n * WF;
                const float* x = ext + (size_t)n * W1 * F + rem;
                v0[k] = x[0];
                v1[k] = x[F];
            }
            reinterpret_cast<f4*>(so)[q] = f4{v0[0], v0[1], v0[2], v0[3]};
            reinterpret_cast<f4*>(sn)[q] = f4{v1[0], v1[1], v1[2], v1[3]};
        }
    } else {
        for (int e = tid; e < per; e += 256) {
            const int n = e / WF, rem = e - n * WF;
            const float* x = ext + (size_t)n * W1 * F + rem;
            so[e] = x[0];
            sn[e] = x[F];
        }
    }
}

// F = 5 form of the LDS gather with every load in flight before the first LDS
// write. Workgroup (j, g) stages sample j's assets [g*R, (g+1)*R) — a few asset
// rows, so the LDS image is ~10 KiB and many workgroups share a CU — thread i
// taking the (day, asset) pairs i, i + 256, ... (PPT at most): the pair's four
// market floats as ONE 16-B load from the [T, N, 4] series and its action as one
// dword; then the image [R][W+1][5] in LDS; then its rows of s and s' as whole
// 16-B chunks (R*W*5 is a multiple of 4, so every group starts 16-B aligned).
// Index divisions by R and W*F are multiply-high.
// NT: cache policy of the s / s' stores (written once, read by the learner later:
// 0 default, 2 nt); TPB threads per workgroup.
template <int PPT, int NT = 0, int TPB = 256>
__global__ __launch_bounds__(TPB) void replay_gather_f5_kernel(const float* series, int T, int N, int W,
                                                               const int32_t* days, const float* actions,
                                                               const float* rewards, int H, int B,
                                                               const int32_t* h0, const int32_t* env, float* s,
                                                               float* s_next, float* a_out, float* r_out, int R,
                                                               FastDiv div_r, FastDiv div_wf) {
    constexpr int F = 5;
    extern __shared__ __attribute__((aligned(16))) float ext[];
    const int j = blockIdx.x, tid = threadIdx.x;
    const int n0 = blockIdx.y * R;
    const int b = env[j], hj = h0[j];
    const int W1 = W + 1;
    // the day index goes out first, the actions (which need only b and hj) behind it,
    // so the wait for the day leaves the action loads in flight
    const int dlast = days[(size_t)((hj + W - 1) % H) * B + b];
    const int P = R * W1;
    f4 mk[PPT];
    float ac[PPT];
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
        const int it = min(tid + k * TPB, P - 1);
        const int t = (int)fdiv((uint32_t)it, div_r), n = n0 + it - t * R;
        int h = hj + t;
        h = h >= H ? h - H : h;
        ac[k] = actions[((size_t)h * B + b) * N + n];
    }
    const int d0 = dlast - (W - 1);
    const auto rs_ser = make_rsrc(series, (uint32_t)T * (uint32_t)N * 16u);
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
        const int it = min(tid + k * TPB, P - 1);
        const int t = (int)fdiv((uint32_t)it, div_r), n = n0 + it - t * R;
        const int d = d0 + t;
        const bool in = tid + k * TPB < P && d >= 0 && d < T;   // days off the series read NaN below
        mk[k] = buf_load4(rs_ser, in ? ((uint32_t)d * (uint32_t)N + (uint32_t)n) * 16u : 0xFFFFFFF0u);
    }
    if (tid < R) a_out[(size_t)j * N + n0 + tid] = actions[((size_t)((hj + W) % H) * B + b) * N + n0 + tid];
    if (tid == 0 && blockIdx.y == 0) r_out[j] = rewards[(size_t)((hj + W - 1) % H) * B + b];
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
        const int it = tid + k * TPB;
        if (it < P) {
            const int t = (int)fdiv((uint32_t)it, div_r), nl = it - t * R;
            const int d = d0 + t;
            const bool in = d >= 0 && d < T;
            float* dst = ext + ((size_t)nl * W1 + t) * F;
            dst[0] = in ? mk[k].x : NAN;
            dst[1] = in ? mk[k].y : NAN;
            dst[2] = in ? mk[k].z : NAN;
            dst[3] = in ? mk[k].w : NAN;
            dst[4] = ac[k];
        }
    }
    __syncthreads();
    const int WF = W * F, per = R * WF;
    float* so = s + (size_t)j * N * WF + (size_t)n0 * WF;
    float* sn = s_next + (size_t)j * N * WF + (size_t)n0 * WF;
    const auto rso = make_rsrc(so, (uint32_t)per * 4u), rsn = make_rsrc(sn, (uint32_t)per * 4u);
    for (int q = tid; q < per / 4; q += TPB) {
        float v0[4], v1[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int e = 4 * q + k;
            const int n = (int)fdiv((uint32_t)e, div_wf);
            const float* x = ext + (size_t)n * F + e;       // LDS row n starts n*F floats later than in s
            v0[k] = x[0];
            v1[k] = x[F];
        }
        buf_store4<NT>(rso, (uint32_t)q * 16u, f4{v0[0], v0[1], v0[2], v0[3]});
        buf_store4<NT>(rsn, (uint32_t)q * 16u, f4{v1[0], v1[1], v1[2], v1[3]});
    }
}


// The F = 5 gather as a persistent loop: workgroup g takes samples g, g + G, g + 2G, ..
// and keeps the pipeline full across them — the next sample's staging loads go out
// (into the same registers, once the current image is in LDS) before the current
// sample's write-out, and its index chain (env / h0, then the day) is fetched two and
// one samples ahead — so a sample costs its write-out, not three dependent memory
// round trips plus the write-out. Same image and write-out as replay_gather_f5_kernel.
template <int PPT, int NT>
__global__ __launch_bounds__(256) void replay_gather_f5p_kernel(const float* series, int T, int N, int W,
                                                                const int32_t* days, const float* actions,
                                                                const float* rewards, int H, int B,
                                                                const int32_t* h0, const int32_t* env, int S, float* s,
                                                                float* s_next, float* a_out, float* r_out, int R,
                                                                FastDiv div_r, FastDiv div_wf) {
    constexpr int F = 5;
    extern __shared__ __attribute__((aligned(16))) float ext[];
    const int tid = threadIdx.x;
    const int n0 = blockIdx.y * R;
    const int W1 = W + 1, P = R * W1, WF = W * F, per = R * WF;
    const int G = gridDim.x;
    int j = blockIdx.x;
    if (j >= S) return;                                    // uniform per workgroup
    const auto rs_ser = make_rsrc(series, (uint32_t)T * (uint32_t)N * 16u);
    auto day_of = [&](int bb, int hh) { return days[(size_t)((hh + W - 1) % H) * B + bb]; };
    f4 mk[PPT];
    float ac[PPT];
    auto issue = [&](int bb, int hh, int dl) {            // the sample's staging loads, nothing waited
        const int d0 = dl - (W - 1);
#pragma unroll
        for (int k = 0; k < PPT; ++k) {
            const int it = min(tid + k * 256, P - 1);
            const int t = (int)fdiv((uint32_t)it, div_r), n = n0 + it - t * R;
            int h = hh + t;
            h = h >= H ? h - H : h;
            ac[k] = actions[((size_t)h * B + bb) * N + n];
            const int d = d0 + t;
            const bool in = tid + k * 256 < P && d >= 0 && d < T;
            mk[k] = buf_load4(rs_ser, in ? ((uint32_t)d * (uint32_t)N + (uint32_t)n) * 16u : 0xFFFFFFF0u);
        }
    };
    // index pipeline: (b0, h0, d0) current; (b1, h1, d1) next; (b2, h2) the one after
    int bc = env[j], hc = h0[j];
    int dc = day_of(bc, hc);
    bool m1 = j + G < S, m2 = j + 2 * G < S;
    int b1 = 0, h1 = 0, d1 = 0, b2 = 0, h2 = 0;
    if (m1) { b1 = env[j + G]; h1 = h0[j + G]; }
    if (m2) { b2 = env[j + 2 * G]; h2 = h0[j + 2 * G]; }
    if (m1) d1 = day_of(b1, h1);
    issue(bc, hc, dc);
    while (true) {
        if (tid < R) a_out[(size_t)j * N + n0 + tid] = actions[((size_t)((hc + W) % H) * B + bc) * N + n0 + tid];
        if (tid == 0 && blockIdx.y == 0) r_out[j] = rewards[(size_t)((hc + W - 1) % H) * B + bc];
        const int dfirst = dc - (W - 1);
#pragma unroll
        for (int k = 0; k < PPT; ++k) {
            const int it = tid + k * 256;
            if (it < P) {
                const int t = (int)fdiv((uint32_t)it, div_r), nl = it - t * R;
                const int d = dfirst + t;
                const bool in = d >= 0 && d < T;
                float* dst = ext + ((size_t)nl * W1 + t) * F;
                dst[0] = in ? mk[k].x : NAN;
                dst[1] = in ? mk[k].y : NAN;
                dst[2] = in ? mk[k].z : NAN;
                dst[3] = in ? mk[k].w : NAN;
                dst[4] = ac[k];
            }
        }
        __syncthreads();
        if (m1) issue(b1, h1, d1);                          // the next sample's loads fly during the write-out
        float* so = s + (size_t)j * N * WF + (size_t)n0 * WF;
        float* sn = s_next + (size_t)j * N * WF + (size_t)n0 * WF;
        const auto rso = make_rsrc(so, (uint32_t)per * 4u), rsn = make_rsrc(sn, (uint32_t)per * 4u);
        for (int q = tid; q < per / 4; q += 256) {
            float v0[4], v1[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int e = 4 * q + k;
                const int n = (int)fdiv((uint32_t)e, div_wf);
                const float* x = ext + (size_t)n * F + e;
                v0[k] = x[0];
                v1[k] = x[F];
            }
            buf_store4<NT>(rso, (uint32_t)q * 16u, f4{v0[0], v0[1], v0[2], v0[3]});
            buf_store4<NT>(rsn, (uint32_t)q * 16u, f4{v1[0], v1[1], v1[2], v1[3]});
        }
        // index chain ahead: the day of the sample after next, env / h0 of the one after that
        const int j3 = j + 3 * G;
        const bool m3 = j3 < S;
        const int d2 = m2 ? day_of(b2, h2) : 0;
        int b3 = 0, h3 = 0;
        if (m3) { b3 = env[j3]; h3 = h0[j3]; }
        __syncthreads();                                   // the image is rewritten next
        if (!m1) break;
        j += G;
        bc = b1; hc = h1; dc = d1;
        b1 = b2; h1 = h2; d1 = d2; m1 = m2;
        b2 = b3; h2 = h3; m2 = m3;
    }
}

}  // namespace pmenv_dev
