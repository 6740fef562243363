/*
 * c_abi_step.c — TEST INFRASTRUCTURE: a plain C caller of the C ABI (include/pmenv.h),
 * no Python and no torch: the shape a non-Python host (a C/C++ trainer, a cgo / JNI /
 * N-API binding) drives. It generates the synthetic workload on the device
 * (pmenv_synth_series / _actions / pmenv_window_init), steps B envs in place through
 * each advance-step implementation (AUTO, FLAT = step_flat_kernel, ONE_LAUNCH,
 * TWO_LAUNCH) and checks every step's rewards and values, and the final window, against
 * the CPU restatement (oracle/liboracle.so, the parity checker) on the same inputs.
 *
 *   tests/c_abi/c_abi_step [B N W T]        (built by pm-rl_amd/build.py; run by
 *                                             tests/test_gpu_c_abi.py on the GPU box)
 * Exit status 0 = every path matched; the reference tolerances of tests/ (reward
 * |d| <= 1e-6 |r| + 1e-9, value rel 1e-12, market channels bit-exact, weights rel 2e-7).
 */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pmenv.h"
#include "pmenv_oracle.h"

#define HIP(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); exit(2); } } while (0)

static int run_path(int path, const char* name, int B, int N, int W, int T, const float* d_series,
                    const float* d_actions, const float* h_series, const float* h_actions, const float* h_obs0) {
    const int F = 5;
    const size_t nobs = (size_t)B * N * W * F;
    pmenv_cfg cfg;
    pmenv_cfg_default(&cfg, B, N, W, F);
    pmenv* h = NULL;
    if (pmenv_create(&cfg, 0, &h) != PMENV_OK) { fprintf(stderr, "create: %s\n", pmenv_last_error(NULL)); return 1; }
    if (pmenv_set_step_path(h, path) != PMENV_OK) {
        fprintf(stderr, "%s: %s\n", name, pmenv_last_error(h));
        pmenv_destroy(h);
        return 1;
    }
    float *d_obs = NULL, *d_rew = NULL;
    HIP(hipMalloc((void**)&d_obs, nobs * sizeof(float)));
    HIP(hipMalloc((void**)&d_rew, (size_t)B * sizeof(float)));
    HIP(hipMemcpy(d_obs, h_obs0, nobs * sizeof(float), hipMemcpyHostToDevice));
    float* c_obs = malloc(nobs * sizeof(float));
    memcpy(c_obs, h_obs0, nobs * sizeof(float));
    or_env* o = or_create(&cfg);
    float* g_rew = malloc((size_t)B * sizeof(float));
    float* c_rew = malloc((size_t)B * sizeof(float));
    double* g_val = malloc((size_t)B * sizeof(double));
    int bad = 0;
    if (pmenv_reset(h, d_obs, NULL, NULL) != PMENV_OK) { fprintf(stderr, "reset: %s\n", pmenv_last_error(h)); bad = 1; }
    or_reset(o, c_obs, NULL);
    for (int t = 0; t < T && !bad; ++t) {
        const size_t bar_off = (size_t)(W + t) * B * N * 4, act_off = (size_t)t * B * N;
        if (pmenv_step(h, d_actions + act_off, NULL, d_series + bar_off, d_obs, d_rew, NULL) != PMENV_OK) {
            fprintf(stderr, "%s step %d: %s\n", name, t, pmenv_last_error(h));
            bad = 1;
            break;
        }
        or_step(o, h_actions + act_off, NULL, h_series + bar_off, c_obs, c_rew, NULL, NULL);
        HIP(hipMemcpy(g_rew, d_rew, (size_t)B * sizeof(float), hipMemcpyDeviceToHost));
        HIP(hipMemcpy(g_val, pmenv_value(h), (size_t)B * sizeof(double), hipMemcpyDeviceToHost));
        for (int b = 0; b < B; ++b) {
            const double d = fabs((double)g_rew[b] - (double)c_rew[b]);
            if (!(d <= 1e-6 * fabs((double)c_rew[b]) + 1e-9)) {
                fprintf(stderr, "%s step %d env %d: reward %.9g vs %.9g\n", name, t, b, g_rew[b], c_rew[b]);
                bad = 1;
                break;
            }
            if (!(fabs(g_val[b] / o->value[b] - 1.0) <= 1e-12)) {
                fprintf(stderr, "%s step %d env %d: value %.17g vs %.17g\n", name, t, b, g_val[b], o->value[b]);
                bad = 1;
                break;
            }
        }
    }
    if (!bad) {
        float* g_obs = malloc(nobs * sizeof(float));
        HIP(hipMemcpy(g_obs, d_obs, nobs * sizeof(float), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < nobs; ++i) {
            const int f = (int)(i % F);
            const int ok = f < F - 1 ? memcmp(&g_obs[i], &c_obs[i], 4) == 0
                                     : fabsf(g_obs[i] - c_obs[i]) <= 2e-7f * fabsf(c_obs[i]) + 1e-12f;
            if (!ok) {
                fprintf(stderr, "%s: window float %zu: %.9g vs %.9g\n", name, i, g_obs[i], c_obs[i]);
                bad = 1;
                break;
            }
        }
        free(g_obs);
    }
    if (!bad) printf("c_abi ok %-10s %s\n", name, pmenv_step_path(h));
    or_destroy(o);
    free(c_obs); free(g_rew); free(c_rew); free(g_val);
    HIP(hipFree(d_obs));
    HIP(hipFree(d_rew));
    pmenv_destroy(h);
    return bad;
}

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 600, N = argc > 2 ? atoi(argv[2]) : 30;
    const int W = argc > 3 ? atoi(argv[3]) : 50, T = argc > 4 ? atoi(argv[4]) : 60;
    const int F = 5;
    if (pmenv_abi_version() != PMENV_ABI_VERSION) { fprintf(stderr, "ABI version mismatch\n"); return 1; }
    const size_t nser = (size_t)(W + T) * B * N * 4, nact = (size_t)T * B * N, nobs = (size_t)B * N * W * F;
    float *d_series = NULL, *d_actions = NULL, *d_obs = NULL;
    HIP(hipMalloc((void**)&d_series, nser * sizeof(float)));
    HIP(hipMalloc((void**)&d_actions, nact * sizeof(float)));
    HIP(hipMalloc((void**)&d_obs, nobs * sizeof(float)));
    if (pmenv_synth_series(d_series, W + T, B, N, 0, 42, 0.015f, NULL) != PMENV_OK ||
        pmenv_synth_actions(d_actions, T, B, N, 0, 43, NULL) != PMENV_OK ||
        pmenv_window_init(d_obs, d_series, B, N, W, F, NULL) != PMENV_OK) {
        fprintf(stderr, "synthetic data: %s\n", pmenv_last_error(NULL));
        return 1;
    }
    HIP(hipDeviceSynchronize());
    float* h_series = malloc(nser * sizeof(float));
    float* h_actions = malloc(nact * sizeof(float));
    float* h_obs0 = malloc(nobs * sizeof(float));
    HIP(hipMemcpy(h_series, d_series, nser * sizeof(float), hipMemcpyDeviceToHost));
    HIP(hipMemcpy(h_actions, d_actions, nact * sizeof(float), hipMemcpyDeviceToHost));
    HIP(hipMemcpy(h_obs0, d_obs, nobs * sizeof(float), hipMemcpyDeviceToHost));
    const struct { int path; const char* name; } paths[] = {
        {PMENV_STEP_PATH_AUTO, "auto"}, {PMENV_STEP_PATH_FLAT, "flat"},
        {PMENV_STEP_PATH_ONE_LAUNCH, "one_launch"}, {PMENV_STEP_PATH_TWO_LAUNCH, "two_launch"}};
    int bad = 0;
    for (size_t i = 0; i < sizeof paths / sizeof paths[0]; ++i)
        bad |= run_path(paths[i].path, paths[i].name, B, N, W, T, d_series, d_actions, h_series, h_actions, h_obs0);
    free(h_series); free(h_actions); free(h_obs0);
    HIP(hipFree(d_series));
    HIP(hipFree(d_actions));
    HIP(hipFree(d_obs));
    return bad;
}
