/*
 * sanitize_main.c — TEST INFRASTRUCTURE ONLY (SURVEY.md §5 "race detection /
 * sanitizers"): built with -fsanitize=address,undefined by oracle/sanitize/build.sh and
 * run by tests/test_sanitizers.py on the CPU.
 *
 * 1. Drives every entry point of the CPU restatement (oracle/pmenv_oracle.c) through
 *    every mode — reward kinds, ring and norm modes, commission, surface and advance
 *    steps, masked resets, GAE, moments, the batched trainer reward, the synthetic
 *    generators — on random inputs, so ASan / UBSan see every index path.
 * 2. Emulates, on the host, the two in-place window-advance schedules of the HIP path
 *    with workgroups executed in a random order and every store visible at once (the
 *    worst interleaving), and proves them race-free and exact against an out-of-place
 *    advance:
 *      - the flat stream (env_step.h flat_wg_body + copy_halo): a workgroup owns chunks
 *        [c0, c0 + CPW); the two chunks past it come from the halo the scalar-step
 *        kernel copied before any store. Every memory read of a workgroup is checked
 *        to hit a chunk no workgroup has stored yet (read-before-write).
 *      - the one-launch step (step_env.h): a workgroup owns one env; its slots are the
 *        env's 1 KiB-aligned 64-chunk blocks, lanes outside the env read 0 and store
 *        nothing. Reads outside the env are checked never to feed a kept position.
 * 3. Emulates the flat one-launch step (step_flat.h) over consecutive steps: tiles in a
 *    random order, the halo and the state snapshot by parity, one owner per env (below).
 * Exit status 0 = clean (UBSan built with -fno-sanitize-recover: any report aborts).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../pmenv_oracle.h"

static uint64_t g_rng = 0x9E3779B97F4A7C15ull;
static double urand(void) {
    g_rng ^= g_rng << 13; g_rng ^= g_rng >> 7; g_rng ^= g_rng << 17;
    return (double)(g_rng >> 11) * (1.0 / 9007199254740992.0);
}
static double nrand(void) { return sqrt(-2.0 * log(urand() + 1e-300)) * cos(6.283185307179586 * urand()); }
static int fails = 0;
#define CHECK(c, ...) do { if (!(c)) { ++fails; fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); } } while (0)

/* ------------------------------------------------------------ 1. the restatement */
static void drive_oracle(int B, int N, int W, int F, int T, int kind, int norm, int ring, int ret, double c) {
    pmenv_cfg cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.num_envs = B; cfg.num_assets = N; cfg.window = W; cfg.features = F;
    cfg.close_channel = F >= 5 ? 3 : F - 2;
    cfg.reward_kind = kind; cfg.norm_mode = norm; cfg.ring_mode = ring; cfg.ret_mode = ret;
    cfg.mu_max_iter = 100; cfg.init_cash = 25000.0; cfg.commission = c; cfg.reward_scale = 1.0;
    cfg.risk_free_rate = 0.04; cfg.sharpe_eta = 0.05; cfg.mu_tol = 1e-10;
    or_env* e = or_create(&cfg);
    const int Fm = F - 1;
    float* obs = calloc((size_t)B * N * W * F, sizeof(float));
    float* act = malloc((size_t)B * N * sizeof(float));
    float* bar = malloc((size_t)B * N * Fm * sizeof(float));
    float* pr = malloc((size_t)B * N * sizeof(float));
    float* rew = malloc((size_t)B * sizeof(float));
    double* rets = malloc((size_t)B * sizeof(double));
    float* wts = malloc((size_t)B * N * sizeof(float));
    uint8_t* mask = malloc((size_t)B);
    for (size_t i = 0; i < (size_t)B * N * W * F; ++i) obs[i] = (float)(100.0 * (1.0 + 0.01 * nrand()));
    or_reset(e, obs, NULL);
    for (int t = 0; t < T; ++t) {
        for (int i = 0; i < B * N; ++i) {
            act[i] = (float)(norm ? nrand() : (t % 3 == 0 ? nrand() : urand() / N * 2.0));
            pr[i] = (float)(1.0 + 0.01 * nrand());
        }
        for (int i = 0; i < B * N * Fm; ++i) bar[i] = (float)(100.0 * (1.0 + 0.01 * nrand()));
        if (t % 4 == 3) or_step(e, act, pr, NULL, obs, rew, rets, wts);        /* surface */
        else if (t % 4 == 2) or_step(e, act, pr, bar, obs, rew, rets, wts);    /* advance, caller prices */
        else or_step_mt(e, act, NULL, bar, obs, rew, rets, NULL, 1 + t % 3);  /* advance, derived prices */
        if (t == T / 2) {
            for (int b = 0; b < B; ++b) mask[b] = (uint8_t)(urand() < 0.4);
            or_reset(e, obs, mask);
        }
    }
    for (int b = 0; b < B; ++b) CHECK(isfinite(e->value[b]), "value not finite (kind %d)", kind);
    or_destroy(e);
    free(obs); free(act); free(bar); free(pr); free(rew); free(rets); free(wts); free(mask);
}

static void drive_rows(void) {
    const int T = 37, B = 19;
    float* r = malloc(sizeof(float) * T * B);
    float* v = malloc(sizeof(float) * (T + 1) * B);
    float* adv = malloc(sizeof(float) * T * B);
    float* ret = malloc(sizeof(float) * T * B);
    uint8_t* d = malloc((size_t)T * B);
    for (int i = 0; i < T * B; ++i) { r[i] = (float)nrand(); d[i] = urand() < 0.05; }
    for (int i = 0; i < (T + 1) * B; ++i) v[i] = (float)nrand();
    or_gae(r, v, d, adv, ret, T, B, 0.99f, 0.95f);
    or_gae(r, v, NULL, adv, ret, T, B, 0.99f, 1.0f);
    double m[3];
    or_moments(r, (int64_t)T * B, m);
    CHECK(m[0] == T * B, "moments count");
    or_moments(r, 0, m);
    const int BB = 11, NN = 7;
    float* a = malloc(sizeof(float) * BB * NN);
    float* p = malloc(sizeof(float) * BB * NN);
    float* vp = malloc(sizeof(float) * BB);
    float* ro = malloc(sizeof(float) * BB);
    float* ga = malloc(sizeof(float) * BB * NN);
    for (int i = 0; i < BB * NN; ++i) { a[i] = (float)nrand(); p[i] = (float)(1.0 + 0.01 * nrand()); }
    for (int i = 0; i < BB; ++i) vp[i] = 25000.0f;
    for (int kind = 0; kind < 3; ++kind)
        for (int norm = 0; norm < 3; ++norm) {
            double R = or_batch_reward(a, vp, p, BB, NN, kind, norm, 1.0, ro, ga);
            /* unnormalised raw scores can give a negative portfolio return: log -> NaN, as torch */
            CHECK(isfinite(R) || kind == 2 || norm == 2, "batch reward kind %d norm %d", kind, norm);
        }
    float* ser = malloc(sizeof(float) * 9 * 5 * 3 * 4);
    float* acts = malloc(sizeof(float) * 9 * 5 * 3);
    or_synth_series(ser, 9, 5, 3, 11, 42, 0.015f);
    or_synth_actions(acts, 9, 5, 3, 11, 43);
    free(r); free(v); free(adv); free(ret); free(d); free(a); free(p); free(vp); free(ro); free(ga); free(ser);
    free(acts);
}

/* ------------------------------------------------------------ 2. schedule emulation */
/* The out-of-place reference advance of one step, F = 5: out[n, t, f] = in[n, t+1, f]
 * for t < W-1; day W-1 = the bar (market) and w' (weight channel); storage-order ring
 * (ring full) keeps the weight channel in place except slot `slot`, which takes w'. */
static void advance_ref(const float* in, float* out, int B, int N, int W, const float* bar, const float* wp,
                        int shift_w, int slot) {
    const int F = 5, WF = W * F;
    for (int b = 0; b < B; ++b)
        for (int n = 0; n < N; ++n) {
            const float* r = in + ((size_t)b * N + n) * WF;
            float* o = out + ((size_t)b * N + n) * WF;
            const float* br = bar + ((size_t)b * N + n) * 4;
            const float w = wp[(size_t)b * N + n];
            for (int t = 0; t < W; ++t)
                for (int f = 0; f < F; ++f) {
                    const int pos = t * F + f;
                    float v;
                    if (f == F - 1) v = shift_w ? (t == W - 1 ? w : r[pos + F]) : (t == slot ? w : r[pos]);
                    else v = t == W - 1 ? br[f] : r[pos + F];
                    o[pos] = v;
                }
        }
}

/* the value of output float j (flat index in the env-local or global float space)
 * composed the way flat_compose does: from the unshifted own float, the shifted source
 * (float j + 5) and the row's bar / w' */
static float compose_float(int64_t j, float un, float sh, int N, int W, const float* bar, const float* wp,
                           int64_t env, int shift_w, int slot) {
    const int F = 5, WF = W * F;
    const int64_t row_g = j / WF;                     /* global row = env * N + n */
    const int pos = (int)(j - row_g * WF), f = pos % F, t = pos / F;
    const int n = (int)(row_g - env * N);
    const float w = wp[env * N + n];
    if (f == F - 1) return shift_w ? (t == W - 1 ? w : sh) : (t == slot ? w : un);
    return t == W - 1 ? bar[(env * N + n) * 4 + f] : sh;
}

static void shuffle(int* order, int n) {
    for (int i = 0; i < n; ++i) order[i] = i;
    for (int i = n - 1; i > 0; --i) {
        const int j = (int)(urand() * (i + 1));
        const int t = order[i]; order[i] = order[j]; order[j] = t;
    }
}

static void emulate(int B, int N, int W, int CPW, int shift_w, int slot) {
    const int F = 5;
    const int64_t per = (int64_t)N * W * F, tot = per * B;
    if (per % 4) return;
    const int64_t per4 = per / 4, qtot = tot / 4;
    float* mem = malloc(sizeof(float) * tot);
    float* init = malloc(sizeof(float) * tot);
    float* ref = malloc(sizeof(float) * tot);
    float* bar = malloc(sizeof(float) * B * N * 4);
    float* wp = malloc(sizeof(float) * B * N);
    uint8_t* stored = calloc((size_t)qtot, 1);
    for (int64_t i = 0; i < tot; ++i) init[i] = (float)nrand();
    for (int i = 0; i < B * N * 4; ++i) bar[i] = (float)nrand();
    for (int i = 0; i < B * N; ++i) wp[i] = (float)urand();
    advance_ref(init, ref, B, N, W, bar, wp, shift_w, slot);

    /* --- flat in-place stream with the halo --- */
    memcpy(mem, init, sizeof(float) * tot);
    const int64_t nwg = (qtot + CPW - 1) / CPW;
    float* halo = malloc(sizeof(float) * 8 * (size_t)nwg);
    for (int64_t i = 0; i + 1 < nwg; ++i)            /* copy_halo: the scalar kernel, before any store */
        for (int h = 0; h < 2; ++h) {
            const int64_t q = (i + 1) * CPW + h;
            for (int e = 0; e < 4; ++e) halo[i * 8 + h * 4 + e] = q < qtot ? mem[q * 4 + e] : 0.0f;
        }
    int* order = malloc(sizeof(int) * (size_t)(nwg > B ? nwg : B));
    shuffle(order, (int)nwg);
    float* lds = malloc(sizeof(float) * 4 * (CPW + 2));
    for (int o = 0; o < nwg; ++o) {
        const int64_t wg = order[o], c0 = wg * CPW;
        const int64_t nblk = qtot - c0 < CPW ? qtot - c0 : CPW;
        for (int64_t q = 0; q < CPW + 2; ++q) {         /* every load lands before the barrier */
            for (int e = 0; e < 4; ++e) lds[q * 4 + e] = 0.0f;
            if (q < nblk) {
                CHECK(!stored[c0 + q], "flat: chunk %lld read after a store", (long long)(c0 + q));
                for (int e = 0; e < 4; ++e) lds[q * 4 + e] = mem[(c0 + q) * 4 + e];
            } else if (q >= CPW && wg + 1 < nwg) {
                for (int e = 0; e < 4; ++e) lds[q * 4 + e] = halo[wg * 8 + (q - CPW) * 4 + e];
            }
        }
        for (int64_t q = 0; q < nblk; ++q) {            /* compose and store */
            const int64_t gq = c0 + q;
            const int64_t env = gq / per4;
            for (int e = 0; e < 4; ++e) {
                const int64_t j = gq * 4 + e;
                const float sh = lds[q * 4 + e + 5];    /* floats 4q+5 .. 4q+8: chunks q+1, q+2 */
                const float v = compose_float(j, lds[q * 4 + e], sh, N, W, bar, wp, env, shift_w, slot);
                mem[j] = v;
            }
            stored[gq] = 1;
        }
    }
    for (int64_t i = 0; i < tot; ++i)
        if (memcmp(&mem[i], &ref[i], 4)) { CHECK(0, "flat: float %lld differs (B%d N%d W%d CPW%d)", (long long)i, B, N, W, CPW); break; }

    /* --- one workgroup per env, 1 KiB-aligned blocks (step_env.h) --- */
    memcpy(mem, init, sizeof(float) * tot);
    memset(stored, 0, (size_t)qtot);
    const int64_t blocks = (per4 + 126) / 64, slots = ((blocks + 3) / 4) * 4 * 64;
    float* img = malloc(sizeof(float) * 4 * (size_t)(slots + 2));
    shuffle(order, B);
    for (int o = 0; o < B; ++o) {
        const int64_t b = order[o], e0 = b * per4, a = e0 & 63;
        for (int64_t s = 0; s < slots + 2; ++s) {
            const int64_t c = s - a;                      /* env-local chunk */
            for (int e = 0; e < 4; ++e) img[s * 4 + e] = 0.0f;
            if (s < slots && c >= 0 && c < per4) {
                CHECK(!stored[e0 + c], "one: chunk %lld read after a store", (long long)(e0 + c));
                for (int e = 0; e < 4; ++e) img[s * 4 + e] = mem[(e0 + c) * 4 + e];
            }
        }
        for (int64_t s = 0; s < slots; ++s) {
            const int64_t c = s - a;
            if (c < 0 || c >= per4) continue;             /* outside the env: the store is dropped */
            for (int e = 0; e < 4; ++e) {
                const int64_t jl = c * 4 + e;               /* env-local float */
                const float sh = img[s * 4 + e + 5];
                /* a shifted source outside the env (read as 0) may only feed a last-day position */
                if (jl + 5 >= per) {
                    const int pos = (int)(jl % (W * F));
                    CHECK(pos / F == W - 1, "one: a kept position reads past the env");
                }
                mem[e0 * 4 + jl] = compose_float(e0 * 4 + jl, img[s * 4 + e], sh, N, W, bar, wp, b, shift_w, slot);
            }
            stored[e0 + c] = 1;
        }
    }
    for (int64_t i = 0; i < tot; ++i)
        if (memcmp(&mem[i], &ref[i], 4)) { CHECK(0, "one: float %lld differs (B%d N%d W%d)", (long long)i, B, N, W); break; }
    free(mem); free(init); free(ref); free(bar); free(wp); free(stored); free(halo); free(order); free(lds); free(img);
}

/* ------------------------------------------------------------ 3. the flat one-launch step */
/* step_flat.h over T consecutive steps: tiles of CPW chunks in a random order each step,
 * every store visible at once. A tile reads only its own chunks from the window (checked:
 * no chunk read after a store), the two chunks past it from the halo of parity p (checked:
 * nothing writes parity p during the step) and each env's scalar inputs from the state
 * snapshot of parity p (checked likewise); the env's owner — the tile holding its first
 * chunk, exactly one per env (checked) — writes the canonical state and the snapshot of
 * parity 1 - p, and every tile its first two output chunks into the halo of parity 1 - p.
 * w' and the counter that every tile of an env uses come from the snapshot, so all tiles of
 * an env must agree with the owner (checked through the result). Mid-run the canonical
 * state changes outside the step (a reset) and the snapshot and halo are re-primed. The
 * window after each step must equal the out-of-place advance, bit for bit. */
static float flat1_wp(double v, int32_t k, int64_t b, int n) {          /* stands in for w' */
    return (float)(fmod(v * 1e-3 + 0.37 * n + 0.11 * k + 0.05 * (double)b, 1.0));
}

static void emulate_flat1(int B, int N, int W, int CPW, int T, int storage) {
    const int F = 5, WF = W * F;
    const int64_t per = (int64_t)N * WF, tot = per * B;
    if (per % 4) return;
    const int64_t per4 = per / 4, qtot = tot / 4, ntiles = (qtot + CPW - 1) / CPW;
    float* mem = malloc(sizeof(float) * tot);
    float* ref = malloc(sizeof(float) * tot);
    float* nxt = malloc(sizeof(float) * tot);
    float* bar = malloc(sizeof(float) * B * N * 4);
    float* wp = malloc(sizeof(float) * B * N);
    double* value = malloc(sizeof(double) * B);
    int32_t* k = malloc(sizeof(int32_t) * B);
    double* sv[2] = {malloc(sizeof(double) * B), malloc(sizeof(double) * B)};
    int32_t* sk[2] = {malloc(sizeof(int32_t) * B), malloc(sizeof(int32_t) * B)};
    float* halo[2] = {calloc((size_t)ntiles * 8, sizeof(float)), calloc((size_t)ntiles * 8, sizeof(float))};
    uint8_t* halo_w[2] = {calloc((size_t)ntiles, 1), calloc((size_t)ntiles, 1)};   /* written this step */
    uint8_t* snap_w[2] = {calloc((size_t)B, 1), calloc((size_t)B, 1)};
    uint8_t* owners = calloc((size_t)B, 1);
    uint8_t* stored = calloc((size_t)qtot, 1);
    int* order = malloc(sizeof(int) * (size_t)ntiles);
    float* lds = malloc(sizeof(float) * 4 * (CPW + 2));
    for (int64_t i = 0; i < tot; ++i) mem[i] = ref[i] = (float)nrand();
    for (int b = 0; b < B; ++b) { value[b] = 25000.0 + b; k[b] = (int32_t)(urand() * 2 * W); }
    int par = 0, primed = 0;
    for (int t = 0; t < T; ++t) {
        if (t == T / 2) {                               /* a reset outside the step: re-prime */
            for (int b = 0; b < B; b += 2) { value[b] = 25000.0; k[b] = 0; }
            primed = 0;
        }
        if (!primed) {                                  /* flat_prime_kernel */
            for (int b = 0; b < B; ++b) { sv[par][b] = value[b]; sk[par][b] = k[b]; }
            for (int64_t i = 0; i + 1 < ntiles; ++i)
                for (int h = 0; h < 2; ++h) {
                    const int64_t q = (i + 1) * CPW + h;
                    for (int e = 0; e < 4; ++e) halo[par][i * 8 + h * 4 + e] = q < qtot ? mem[q * 4 + e] : 0.0f;
                }
            primed = 1;
        }
        for (int i = 0; i < B * N * 4; ++i) bar[i] = (float)nrand();
        /* the expected result: the out-of-place advance with each env's own counter */
        for (int b = 0; b < B; ++b) {
            for (int n = 0; n < N; ++n) wp[b * N + n] = flat1_wp(value[b], k[b], b, n);
            const int shift_w = !(storage && k[b] >= W - 1), slot = (int)((1 + (int64_t)k[b]) % W);
            advance_ref(ref + (size_t)b * per, nxt + (size_t)b * per, 1, N, W, bar + (size_t)b * N * 4,
                        wp + (size_t)b * N, shift_w, slot);
        }
        memset(stored, 0, (size_t)qtot);
        for (int h = 0; h < 2; ++h) {
            memset(halo_w[h], 0, (size_t)ntiles);
            memset(snap_w[h], 0, (size_t)B);
        }
        memset(owners, 0, (size_t)B);
        shuffle(order, (int)ntiles);
        for (int o = 0; o < ntiles; ++o) {
            const int64_t tile = order[o], c0 = tile * CPW;
            const int64_t nblk = qtot - c0 < CPW ? qtot - c0 : CPW;
            const int64_t e_lo = c0 / per4, e_hi = (c0 + nblk - 1) / per4;
            for (int64_t q = 0; q < CPW + 2; ++q) {
                for (int e = 0; e < 4; ++e) lds[q * 4 + e] = 0.0f;
                if (q < nblk) {
                    CHECK(!stored[c0 + q], "flat1: chunk %lld read after a store", (long long)(c0 + q));
                    for (int e = 0; e < 4; ++e) lds[q * 4 + e] = mem[(c0 + q) * 4 + e];
                } else if (q >= CPW && tile + 1 < ntiles) {
                    CHECK(!halo_w[par][tile], "flat1: halo %lld read after this step wrote it", (long long)tile);
                    for (int e = 0; e < 4; ++e) lds[q * 4 + e] = halo[par][tile * 8 + (q - CPW) * 4 + e];
                }
            }
            /* the scalar steps of the tile's envs, from the snapshot of parity p */
            float* twp = malloc(sizeof(float) * (size_t)(e_hi - e_lo + 1) * N);
            int32_t* tk = malloc(sizeof(int32_t) * (size_t)(e_hi - e_lo + 1));
            for (int64_t b = e_lo; b <= e_hi; ++b) {
                CHECK(!snap_w[par][b], "flat1: env %lld snapshot read after this step wrote it", (long long)b);
                tk[b - e_lo] = sk[par][b];
                for (int n = 0; n < N; ++n) twp[(b - e_lo) * N + n] = flat1_wp(sv[par][b], sk[par][b], b, n);
                if (b * per4 >= c0) {                   /* the owner */
                    CHECK(!owners[b]++, "flat1: env %lld has two owners", (long long)b);
                    value[b] = value[b] * 1.0001 + 1.0;
                    k[b] = k[b] + 1;
                    sv[1 - par][b] = value[b];
                    sk[1 - par][b] = k[b];
                    snap_w[1 - par][b] = 1;
                }
            }
            for (int64_t q = 0; q < nblk; ++q) {
                const int64_t gq = c0 + q;
                for (int e = 0; e < 4; ++e) {
                    const int64_t j = gq * 4 + e, env = j / per;
                    const int32_t kb = tk[env - e_lo];
                    const int shift_w = !(storage && kb >= W - 1), slot = (int)((1 + (int64_t)kb) % W);
                    const float sh = lds[q * 4 + e + 5];
                    /* compose_float reads w' from a [B, N] array: hand it the tile's copy */
                    const float v = compose_float(j - env * per + 0, lds[q * 4 + e], sh, N, W,
                                                  bar + (size_t)env * N * 4, twp + (env - e_lo) * N, 0, shift_w, slot);
                    mem[j] = v;
                    if (tile > 0 && q < 2) halo[1 - par][(tile - 1) * 8 + q * 4 + e] = v;
                }
                stored[gq] = 1;
            }
            if (tile > 0) halo_w[1 - par][tile - 1] = 1;
            free(twp);
            free(tk);
        }
        for (int b = 0; b < B; ++b) CHECK(owners[b] == 1, "flat1: env %d owned %d times", b, owners[b]);
        par = 1 - par;
        float* sw = ref; ref = nxt; nxt = sw;
        for (int64_t i = 0; i < tot; ++i)
            if (memcmp(&mem[i], &ref[i], 4)) {
                CHECK(0, "flat1: step %d float %lld differs (B%d N%d W%d CPW%d)", t, (long long)i, B, N, W, CPW);
                break;
            }
    }
    free(mem); free(ref); free(nxt); free(bar); free(wp); free(value); free(k); free(sv[0]); free(sv[1]);
    free(sk[0]); free(sk[1]); free(halo[0]); free(halo[1]); free(halo_w[0]); free(halo_w[1]);
    free(snap_w[0]); free(snap_w[1]); free(owners); free(stored);
    free(order); free(lds);
}

int main(void) {
    /* every reward kind x norm x ring x ret mode, with and without commission */
    for (int kind = 0; kind < 4; ++kind)
        for (int norm = 0; norm < 2; ++norm)
            for (int ring = 0; ring < 2; ++ring)
                for (int ret = 0; ret < 3; ++ret)
                    drive_oracle(5, 7, 6, 5, 15, kind, norm, ring, ret, (kind + ring) % 2 ? 0.0025 : 0.0);
    drive_oracle(3, 30, 50, 5, 60, 0, 0, 0, 2, 0.0);      /* BASELINE row shape through the ring wrap */
    drive_oracle(2, 9, 4, 3, 9, 1, 1, 1, 1, 0.01);        /* F = 3 (close channel 1) */
    drive_rows();
    /* schedules: rows of 20 .. 250 floats, W = 2, single-asset envs, 1 KiB seams at every
     * env offset, both weight-channel modes, the product's 1024-chunk workgroups and a
     * small one that puts many seams inside each env */
    const int shapes[][3] = {{37, 30, 50}, {13, 5, 4}, {7, 4, 2}, {9, 1, 4}, {3, 64, 16}, {600, 4, 50}, {1, 12, 10}};
    for (size_t i = 0; i < sizeof shapes / sizeof shapes[0]; ++i)
        for (int mode = 0; mode < 2; ++mode)
            for (int cpw = 0; cpw < 2; ++cpw)
                emulate(shapes[i][0], shapes[i][1], shapes[i][2], cpw ? 1024 : 96, mode == 0,
                        mode ? (int)(urand() * shapes[i][2]) : 0);
    /* the flat one-launch step: the product's 1,024-chunk tiles (256 x 4 and 512 x 2) and
     * small tiles that put several tiles in one env and several envs in one tile, both ring
     * orders, through the wrap and a re-prime */
    const int fshapes[][3] = {{37, 30, 50}, {301, 4, 30}, {3, 64, 47}, {13, 5, 4}, {9, 1, 4}, {130, 2, 60}};
    for (size_t i = 0; i < sizeof fshapes / sizeof fshapes[0]; ++i)
        for (int storage = 0; storage < 2; ++storage)
            for (int cpw = 0; cpw < 2; ++cpw)
                emulate_flat1(fshapes[i][0], fshapes[i][1], fshapes[i][2], cpw ? 1024 : 96, 2 * fshapes[i][2] + 3,
                              storage);
    if (fails) { fprintf(stderr, "%d check(s) failed\n", fails); return 1; }
    printf("sanitize ok\n");
    return 0;
}
