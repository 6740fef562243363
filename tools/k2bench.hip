// k2bench.hip — ablation of the streaming window-advance kernel (not product code).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/k2bench tools/k2bench.hip
// Each variant removes one ingredient of advance_rows_kernel; results are only
// timed, not checked (variants other than FULL compute wrong windows).
#include <algorithm>
#include <vector>
#include <stdio.h>
#include <stdlib.h>

#include "../pm-rl_amd/csrc/common.h"

using namespace pmenv_dev;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

enum : int { XW = 1, STAGE = 2, COMPOSE = 4, KLOAD = 8, BIGARGS = 16 };

struct Small {
    float* obs; const float* bar; const float* wnew; const int* k;
    int N, W, F, R, units;
    FastDiv div_units, div_wf, div_f;
};

template <int BLOCK, int FLAGS>
__global__ __launch_bounds__(BLOCK) void k2(Small p) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int tid = threadIdx.x;
    const int N = p.N, W = p.W, F = p.F, Fm = F - 1, WF = W * F, R = p.R;
    const int b = (int)fdiv(blockIdx.x, p.div_units);
    const int r0 = (int)(blockIdx.x - (uint32_t)b * (uint32_t)p.units) * R;
    const int rows = min(R, N - r0);
    const int nf = rows * WF, nq = nf >> 2;
    float* obs = p.obs + (size_t)b * N * WF + (size_t)r0 * WF;
    f4 xs = f4{0.f, 0.f, 0.f, 0.f};
    float xw = 0.f;
    const int q = tid;
    const int j = 4 * q + F;
    if (j + 3 < nf) {
        const f4u v = *reinterpret_cast<const f4u*>(obs + j);
        xs = f4{v.x, v.y, v.z, v.w};
    } else if (q < nq) {
        xs.x = j < nf ? obs[j] : 0.f;
        xs.y = j + 1 < nf ? obs[j + 1] : 0.f;
        xs.z = j + 2 < nf ? obs[j + 2] : 0.f;
    }
    if ((FLAGS & XW) && q < nq) {
        const uint32_t j0 = (uint32_t)(4 * q);
        const int e = F - 1 - (int)(j0 - fdiv(j0, p.div_f) * (uint32_t)F);
        if (e < 4) xw = obs[4 * q + e];
    }
    float* sbar = lds;
    float* swp = lds + R * Fm;
    if (FLAGS & STAGE) {
        const float* barg = p.bar + ((size_t)b * N + r0) * Fm;
        for (int i = tid; i < rows * Fm; i += BLOCK) sbar[i] = barg[i];
        const float* wpg = p.wnew + (size_t)b * N + r0;
        for (int i = tid; i < rows; i += BLOCK) swp[i] = wpg[i];
    }
    int k = 60;
    if (FLAGS & KLOAD) k = p.k[b] - 1;
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (q < nq) {
        float v[4] = {xs.x, xs.y, xs.z, xs.w};
        if (FLAGS & COMPOSE) {
            const bool storage_full = k >= W - 1, shift_w = !storage_full;
            const int slotF = ((1 + k) % W) * F;
            const uint32_t j0 = (uint32_t)q * 4u;
            const uint32_t row = fdiv(j0, p.div_wf);
            int kk = (int)(j0 - row * (uint32_t)WF);
            int f = kk - (int)fdiv((uint32_t)kk, p.div_f) * F;
            int n = (int)row;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const bool lastday = kk >= WF - F;
                if (f == F - 1) {
                    if (shift_w ? lastday : (kk - f == slotF)) v[e] = swp[n];
                    else if (!shift_w) v[e] = xw;
                } else if (lastday) {
                    v[e] = sbar[n * Fm + f];
                }
                ++kk;
                if (++f == F) f = 0;
                if (kk == WF) { kk = 0; ++n; }
            }
        } else {
            v[0] += xw;
        }
        reinterpret_cast<f4*>(obs)[q] = f4{v[0], v[1], v[2], v[3]};
    }
}

template <typename Fn>
double timeit(Fn f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(a)); f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2] * 1e-3;
}

int main() {
    const int B = 65536, N = 30, W = 50, F = 5;
    const size_t nfl = (size_t)B * N * W * F;
    float *obs, *bar, *wn; int* k;
    CK(hipMalloc(&obs, nfl * 4 + 64)); CK(hipMemset(obs, 0, nfl * 4 + 64));
    CK(hipMalloc(&bar, (size_t)B * N * 4 * 4)); CK(hipMemset(bar, 0, (size_t)B * N * 16));
    CK(hipMalloc(&wn, (size_t)B * N * 4)); CK(hipMemset(wn, 0, (size_t)B * N * 4));
    CK(hipMalloc(&k, B * 4)); CK(hipMemset(k, 0, B * 4));
    const double bytes = 8.0 * nfl;
    for (int R : {8, 6, 4}) {
        Small p{obs, bar, wn, k, N, W, F, R, (N + R - 1) / R, make_fastdiv((N + R - 1) / R), make_fastdiv(W * F), make_fastdiv(F)};
        const unsigned grid = B * p.units;
        const size_t lds = R * F * 4;
        auto run = [&](const char* nm, auto kern) {
            double s = timeit([&] { kern<<<grid, 512, lds>>>(p); }, 15);
            printf("R=%d %-28s %8.1f us  %7.1f GB/s\n", R, nm, s * 1e6, bytes / s / 1e9);
        };
        run("bare (shifted copy)", k2<512, 0>);
        run("+xw", k2<512, XW>);
        run("+stage", k2<512, STAGE>);
        run("+kload", k2<512, KLOAD>);
        run("+compose", k2<512, COMPOSE>);
        run("full", k2<512, XW | STAGE | COMPOSE | KLOAD>);
        run("full - xw", k2<512, STAGE | COMPOSE | KLOAD>);
    }
    return 0;
}
