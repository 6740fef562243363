// data.h — on-device synthetic market data: Philox4x32-10
// counter-based normals, OHLC random walk, softmax actions, initial window.
// Replaces the reference's network data path (data/load_yf.py, instrument.py:79,
// :339-356) for benchmarks; keyed by (seed, global env id, asset, day) so a sharded
// run generates exactly its slice of the unsharded data.
#pragma once
#include "common.h"

namespace pmenv_dev {

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
static __global__ void synth_series_kernel(f4* series, int T, int B, int N, int64_t env_offset,
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
        series[((size_t)t * B + b) * N + n] = f4{(float)op, (float)hi, (float)lo, (float)cl};
        close = cl;
    }
}

// One thread per (t, env): softmax of N(0,1) logits over the N assets.
static __global__ void synth_actions_kernel(float* actions, int T, int B, int N, int64_t env_offset, uint64_t seed) {
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

static __global__ void window_init_kernel(float* obs, const f4* series, int B, int N, int W, int F) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // over B*N*W
    if (i >= (int64_t)B * N * W) return;
    const int t = (int)(i % W);
    const int64_t bn = i / W;
    const int n = (int)(bn % N), b = (int)(bn / N);
    f4 v = series[((size_t)t * B + b) * N + n];
    float* o = obs + (size_t)i * F;
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
    for (int f = 4; f < F; ++f) o[f] = 0.0f;
}

// obs[b, n, t, f] = series[start[b] + t, n, f]; one thread per (b, n, t) row of F floats
static __global__ void window_init_days_kernel(float* obs, const float* series, int T, int N, int F,
                                        const int32_t* start, int B, int W) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // over B*N*W
    if (i >= (int64_t)B * N * W) return;
    const int t = (int)(i % W);
    const int64_t bn = i / W;
    const int n = (int)(bn % N), b = (int)(bn / N);
    const int Fm = F - 1;
    const int64_t d = (int64_t)start[b] + t;
    float* o = obs + (size_t)i * F;
    const bool ok = start[b] >= 0 && d < T;
    for (int f = 0; f < Fm; ++f) o[f] = ok ? series[((size_t)d * N + n) * Fm + f] : NAN;
    o[Fm] = 0.0f;
}

}  // namespace pmenv_dev
