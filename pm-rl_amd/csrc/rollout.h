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

// GAE as a parallel scan for few envs x long horizons: one wave per env, the
// horizon cut into 64 chunks (one per lane). The recursion A_t = d_t + c_t A_{t+1}
// (c_t = gamma*lambda*(1-done_t)) makes each chunk an affine map f(x) = D + C x from
// the advantage after the chunk to the advantage at its start; a suffix scan of
// the 64 maps (composition (C, D) o (C', D') = (C C', D + C D'), six shuffle steps)
// gives every lane its carry-in, and each lane then re-walks its chunk.
__device__ __forceinline__ void gae_delta(const float* r, const float* v, const uint8_t* dones, int t, int B, int b,
                                          float gamma, float lam, double* delta, double* c) {
    const size_t i = (size_t)t * B + b;
    const double nd = dones ? (dones[i] ? 0.0 : 1.0) : 1.0;
    *delta = (double)r[i] + (double)gamma * nd * (double)v[i + B] - (double)v[i];
    *c = (double)gamma * (double)lam * nd;
}

__global__ __launch_bounds__(256) void gae_scan_kernel(const float* r, const float* v, const uint8_t* dones,
                                                       float* adv, float* ret, int T, int B, float gamma, float lam) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= B) return;
    const int L = (T + 63) / 64;
    const int t0 = min(lane * L, T), t1 = min(t0 + L, T);
    double C = 1.0, D = 0.0;
    for (int t = t1 - 1; t >= t0; --t) {
        double dl, c;
        gae_delta(r, v, dones, t, B, b, gamma, lam, &dl, &c);
        D = dl + c * D;
        C = c * C;
    }
    // suffix composition g_l = f_l o f_{l+1} o ... o f_63
    for (int o = 1; o < 64; o <<= 1) {
        const double C2 = __shfl_down(C, o, 64), D2 = __shfl_down(D, o, 64);
        if (lane + o < 64) {
            D = D + C * D2;
            C = C * C2;
        }
    }
    double a = __shfl_down(D, 1, 64);             // advantage at the start of the next chunk
    if (lane == 63) a = 0.0;
    for (int t = t1 - 1; t >= t0; --t) {
        double dl, c;
        gae_delta(r, v, dones, t, B, b, gamma, lam, &dl, &c);
        a = dl + c * a;
        const size_t i = (size_t)t * B + b;
        adv[i] = (float)a;
        ret[i] = (float)(a + (double)v[i]);
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
