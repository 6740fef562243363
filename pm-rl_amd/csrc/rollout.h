// rollout.h — rollout return pass and advantage moments.
// The reference's replay/rollout_buffer.py stores (s, a, v, r) (:43-57) and computes
// no returns; the north star asks for its GAE / discounted-return pass on device.
#pragma once
#include "common.h"

namespace pmenv_dev {

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

constexpr int kMomBlock = 256;
constexpr int kMomBlocks = 1024;
__device__ double g_mom_partial[kMomBlocks * 3];

__global__ __launch_bounds__(kMomBlock) void moments_partial_kernel(const float* x, int64_t n) {
    __shared__ double sh[2][kMomBlock / 64];
    double s = 0.0, q = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kMomBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kMomBlock) {
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
        for (int i = 0; i < kMomBlock / 64; ++i) { ts += sh[0][i]; tq += sh[1][i]; }
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

}  // namespace pmenv_dev
