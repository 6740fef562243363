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
 *    - the generic stream for F != 5, F <= 16 (env_step.h advance_gen_kernel): the same workgroup
 *      and halo, the shift by F floats, the element walk over rows and the staged rows.
 * 3. Emulates the flat one-launch step (step_flat.h) over consecutive steps: tiles in a
 *    random order, the halo and the state snapshot by parity, one owner per env (below).
 * 4. Emulates the relayed step (step_relay.h) over consecutive steps: workgroups dispatched
 *    in a random, non-monotone order with one to 64 resident at once, each taking its role
 *    from the ordered ticket on arrival, a tile runnable only once every relay word it stages
 *    carries the step's epoch (the kernel's wait) — any schedule in which every resident
 *    workgroup waits is a deadlock and fails — through the epoch's wrap, caller edits, a
 *    state write and a step of another path; the tile's staged rows are checked to fit its
 *    BLOCK threads and every LDS / halo / counter index to stay in its buffer.
 * 5. Emulates the one-pass look-back GAE (rollout.h gae_lookback_kernel) with the kernel's
 *    indexing: workgroups dispatched in blockIdx order or a random permutation with a
 *    residency limit, publishing and composing subject to the flag waits, a waiting
 *    workgroup taking the kernel's fallback (the missing maps computed itself, checked
 *    bitwise against the producer's) when no resident one can move; on a workspace of
 *    exactly pmenv_gae_workspace's size holding garbage or the previous call's maps and
 *    flags; the result is checked against the restatement.
 * 6. Audits, without data, the addresses of the in-place stream's halo copy
 *    (env_step.h halo_load / halo_store / copy_halo) for every scalar-step grid, and of
 *    the tools build's advance_flat_direct_kernel (the kernel of the round-3 record
 *    profiles/ab_r03/direct_r03d.err), at the shapes of that record.
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

/* ------------------------------------------------------------ 2b. the generic stream (F != 5) */
/* env_step.h advance_gen_kernel in place: workgroups of CPW chunks in a random order, every
 * store visible at once; the HC chunks past a workgroup (two for F <= 8, four up to F = 16)
 * from the halo, copied before any store as the scalar step does (halo_src: two-chunk items,
 * item i of boundary i >> hs), the shift by F floats read from the staged image (checked: never past it), the
 * workgroup's rows g_lo .. g_hi staged one per thread (checked: at most BLOCK rows, and the
 * element walk's row index inside them), and each element's (day, channel, row) from the
 * chunk's first element plus the kernel's increments. Exact against the out-of-place advance. */
static void emulate_gen(int B, int N, int W, int F, int BLOCK, int CPW, int shift_w, int slot) {
    const int Fm = F - 1, WF = W * F;
    const int64_t per = (int64_t)N * WF, tot = per * B;
    if (per % 4) return;
    const int64_t per4 = per / 4, qtot = tot / 4;
    float* mem = malloc(sizeof(float) * tot);
    float* ref = malloc(sizeof(float) * tot);
    float* bar = malloc(sizeof(float) * B * N * Fm);
    float* wp = malloc(sizeof(float) * B * N);
    uint8_t* stored = calloc((size_t)qtot, 1);
    for (int64_t i = 0; i < tot; ++i) mem[i] = (float)nrand();
    for (int i = 0; i < B * N * Fm; ++i) bar[i] = (float)nrand();
    for (int i = 0; i < B * N; ++i) wp[i] = (float)urand();
    for (int64_t g = 0; g < (int64_t)B * N; ++g)         /* the out-of-place reference */
        for (int t = 0; t < W; ++t)
            for (int f = 0; f < F; ++f) {
                const int64_t j = g * WF + t * F + f;
                float v;
                if (f == Fm) v = shift_w ? (t == W - 1 ? wp[g] : mem[j + F]) : (t == slot ? wp[g] : mem[j]);
                else v = t == W - 1 ? bar[g * Fm + f] : mem[j + F];
                ref[j] = v;
            }
    const int64_t nwg = (qtot + CPW - 1) / CPW;
    const int hs = F > 8 ? 1 : 0, HC = 2 << hs;
    float* halo = malloc(sizeof(float) * 4 * HC * (size_t)nwg);
    for (int64_t i = 0; i < (nwg - 1) << hs; ++i)       /* the scalar step's halo copy, before any store */
        for (int h = 0; h < 2; ++h) {
            const int64_t q = ((i >> hs) + 1) * CPW + 2 * (i & ((1 << hs) - 1)) + h;
            CHECK(i * 8 + h * 4 + 3 < 4 * HC * nwg, "gen: halo item %lld past the buffer", (long long)i);
            for (int e = 0; e < 4; ++e) halo[i * 8 + h * 4 + e] = q < qtot ? mem[q * 4 + e] : 0.0f;
        }
    int* order = malloc(sizeof(int) * (size_t)nwg);
    shuffle(order, (int)nwg);
    float* lds = malloc(sizeof(float) * 4 * (CPW + HC));
    for (int o = 0; o < nwg; ++o) {
        const int64_t wg = order[o], c0 = wg * CPW;
        const int64_t nblk = qtot - c0 < CPW ? qtot - c0 : CPW;
        for (int64_t q = 0; q < CPW + HC; ++q) {
            for (int e = 0; e < 4; ++e) lds[q * 4 + e] = 0.0f;
            if (q < nblk) {
                CHECK(!stored[c0 + q], "gen: chunk %lld read after a store", (long long)(c0 + q));
                for (int e = 0; e < 4; ++e) lds[q * 4 + e] = mem[(c0 + q) * 4 + e];
            } else if (q >= CPW && wg + 1 < nwg) {
                for (int e = 0; e < 4; ++e) lds[q * 4 + e] = halo[wg * 4 * HC + (q - CPW) * 4 + e];
            }
        }
        const int64_t b_lo = c0 / per4, ql = c0 + nblk - 1, b_hi = ql / per4;
        const int64_t g_lo = b_lo * N + (4 * (c0 - b_lo * per4)) / WF;
        const int64_t g_hi = b_hi * N + (4 * (ql - b_hi * per4) + 3) / WF;
        CHECK(g_hi - g_lo < BLOCK, "gen: %lld rows in a workgroup of %d threads", (long long)(g_hi - g_lo + 1), BLOCK);
        for (int64_t q = 0; q < nblk; ++q) {
            const int64_t gq = c0 + q, b = gq / per4;
            const int64_t j0 = 4 * (gq - b * per4), row = j0 / WF, kk = j0 - row * WF;
            int t = (int)(kk / F), f = (int)(kk - (int64_t)t * F);
            int64_t r = b * N + row - g_lo;
            for (int e = 0; e < 4; ++e) {
                CHECK(r >= 0 && r <= g_hi - g_lo, "gen: row %lld outside the staged rows", (long long)r);
                CHECK(q * 4 + e + F < 4 * (CPW + HC), "gen: shifted read past the image");
                const int64_t g = g_lo + r;
                const float sh = lds[q * 4 + e + F], un = lds[q * 4 + e];
                const int last = t == W - 1;
                const float wv = shift_w ? (last ? wp[g] : sh) : (t == slot ? wp[g] : un);
                mem[gq * 4 + e] = f == Fm ? wv : (last ? bar[g * Fm + (f < Fm ? f : 0)] : sh);
                const int fw = f == Fm;
                f = fw ? 0 : f + 1;
                t += fw;
                const int tw = t == W;
                t = tw ? 0 : t;
                r += tw;
            }
            stored[gq] = 1;
        }
    }
    for (int64_t i = 0; i < tot; ++i)
        if (memcmp(&mem[i], &ref[i], 4)) {
            CHECK(0, "gen: float %lld differs (B%d N%d W%d F%d CPW%d)", (long long)i, B, N, W, F, CPW);
            break;
        }
    free(mem); free(ref); free(bar); free(wp); free(stored); free(halo); free(order); free(lds);
}

/* ------------------------------------------------------------ 2c. the surface stream's ring columns */
/* env_step.h surface_stream_kernel: a workgroup of CPW chunks stages its rows' ring columns
 * (ring [B][W][N], slot-major) in LDS as [row][slot], rows g_lo .. g_hi; checked: the staged
 * floats within launch_surface_stream's size ((4 CPW / (W F) + 2) W), every weight float's row
 * (the chunk's row, or the next one when the chunk crosses a row's end) inside the staged rows,
 * and the staged float it reads equal to the ring's (row, slot) — for every slot. */
static void emulate_surf(int B, int N, int W, int F, int CPW) {
    const int Fm = F - 1, WF = W * F;
    const int64_t per = (int64_t)N * WF;
    if (per % 4) return;
    const int64_t per4 = per / 4, qtot = per4 * B;
    float* ring = malloc(sizeof(float) * (size_t)B * W * N);
    for (int64_t i = 0; i < (int64_t)B * W * N; ++i) ring[i] = (float)nrand();
    const int64_t cap = (int64_t)(4 * CPW / WF + 2) * W;
    float* sring = malloc(sizeof(float) * (size_t)cap);
    uint8_t* seen = malloc((size_t)cap);
    for (int64_t c0 = 0; c0 < qtot; c0 += CPW) {
        const int64_t nblk = qtot - c0 < CPW ? qtot - c0 : CPW;
        const int64_t b_lo = c0 / per4, ql = c0 + nblk - 1, b_hi = ql / per4;
        const int64_t g_lo = b_lo * N + (4 * (c0 - b_lo * per4)) / WF;
        const int64_t g_hi = b_hi * N + (4 * (ql - b_hi * per4) + 3) / WF;
        const int64_t nrows = g_hi - g_lo + 1;
        CHECK(nrows * W <= cap, "surf: %lld staged floats past %lld", (long long)(nrows * W), (long long)cap);
        if (nrows * W > cap) break;
        /* the kernel's walk: thread t from (t / nrows, t % nrows), stepping BLOCK elements by
         * quotient / remainder increments; every (row, slot) staged exactly once */
        const int BLOCK = 256;
        memset(seen, 0, (size_t)cap);
        for (int t = 0; t < BLOCK; ++t) {
            const int64_t dq = BLOCK / nrows, dr = BLOCK - dq * nrows;
            int64_t sl = t / nrows, r = t - sl * nrows;
            for (int64_t i = t; i < nrows * W; i += BLOCK) {
                CHECK(sl * nrows + r == i && sl < W && r < nrows, "surf: walk at %lld gives (%lld, %lld)", (long long)i,
                      (long long)sl, (long long)r);
                const int64_t g = g_lo + r, b = g / N, n = g - b * N;
                sring[r * W + sl] = ring[(b * W + sl) * N + n];
                ++seen[r * W + sl];
                sl += dq;
                r += dr;
                if (r >= nrows) { r -= nrows; ++sl; }
            }
        }
        for (int64_t i = 0; i < nrows * W; ++i) CHECK(seen[i] == 1, "surf: staged float %lld written %d times", (long long)i, seen[i]);
        for (int64_t q = c0; q < c0 + nblk; ++q) {
            const int64_t b = q / per4, j0 = 4 * (q - b * per4), row = j0 / WF, kk = j0 - row * WF;
            const int f0 = (int)(kk % F);
            const int64_t r0 = b * N + row - g_lo;           /* the staged counter the chunk reads */
            CHECK(r0 >= 0 && r0 < nrows && (g_lo + r0) / N == b, "surf: chunk %lld reads row %lld's counter",
                  (long long)q, (long long)r0);
            for (int kth = 0; kth < 2; ++kth) {
                const int c = (Fm - f0) + kth * F;
                if (c >= 4) continue;
                int64_t pos = kk + c, rr = b * N + row - g_lo;
                if (pos >= WF) { pos -= WF; ++rr; }
                CHECK((pos % F) == Fm, "surf: weight float at channel %lld", (long long)(pos % F));
                CHECK(rr >= 0 && rr < nrows, "surf: row %lld outside the %lld staged", (long long)rr, (long long)nrows);
                const int64_t g = g_lo + rr, gb = g / N, gn = g - gb * N;
                CHECK(gb == b, "surf: a chunk's weight float in another env");
                for (int sl = 0; sl < W; ++sl)
                    if (memcmp(&sring[rr * W + sl], &ring[(gb * W + sl) * N + gn], 4)) {
                        CHECK(0, "surf: staged (row %lld, slot %d) differs (B%d N%d W%d F%d)", (long long)rr, sl, B, N, W, F);
                        break;
                    }
            }
        }
    }
    free(ring); free(sring); free(seen);
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

/* ------------------------------------------------------------ 4. the relayed step */
/* step_relay.h: blocks [0, scal) are scalar blocks (EPB envs each), the rest tiles of CPW =
 * BLOCK x V chunks. A scalar block writes each env's w' as {epoch, w'} words, the counter's
 * next-step copy (kp parity 1 - q) and the canonical state. A tile stages one row per thread
 * (g_lo .. g_hi), the rows' w' from the words and their counter from kp parity q; in place, the
 * two chunks past it from the halo of parity q, and it writes its first two output chunks into
 * the halo of parity 1 - q. A tile whose words are still missing after `spin` polls DEFERS: it
 * stores nothing, appends itself to the step's list, re-checks once (and runs under its claim if
 * every word arrived) and exits; every scalar block, after its units, runs each listed tile whose
 * words have all arrived, under the tile's claim. Events are sequentially consistent here — the
 * order the kernel builds with completion waits around the list (step_relay.h's head).
 * Dispatch models (a polling tile holds its slot; a finished or deferred workgroup frees one):
 *   0  blockIdx order, 1 to 64 workgroups resident (the hardware's order);
 *   1  a random order with every workgroup resident;
 *   2  a random order with ONE resident;
 *   3  tiles first (the tools build's PMENV_RELAY_TILES_FIRST), 1 to 4 resident.
 * Every tile must run exactly once per step, every env be stepped once, in every model. spin < 0
 * removes the deferral (round 5's kernel): under model 2 it returns 1 on the first deadlock — the
 * negative control that shows the detection works. */
typedef struct { uint64_t* w; int32_t* kp[2]; float* halo[2]; uint32_t epoch; int par, kp_ok; const float* obs; } relay_st;

static void relay_prime(relay_st* r, const float* obs, int B, const int32_t* k, int64_t ntiles, int64_t CPW,
                        int64_t qtot, int need_halo) {
    if (need_halo)
        for (int64_t i = 0; i + 1 < ntiles; ++i)
            for (int h = 0; h < 2; ++h) {
                const int64_t q = (i + 1) * CPW + h;
                for (int e = 0; e < 4; ++e) r->halo[r->par][i * 8 + h * 4 + e] = q < qtot ? obs[q * 4 + e] : 0.0f;
            }
    if (!r->kp_ok)
        for (int b = 0; b < B; ++b) r->kp[r->par][b] = k[b];
}

/* one step's context for the tile runs */
typedef struct {
    relay_st* r;
    int B, N, W, BLOCK, storage, dbuf, q;
    int64_t per4, qtot, CPW, ntiles, nhal;
    const float* in; float* out; const float* bar;
    const double* v0; const int32_t* k0;
    uint8_t* stored; uint8_t* halo_w[2]; uint8_t* ran;
    float* lds; float* s_wp; int32_t* s_kc;
} relay_ctx;

static void relay_rows(const relay_ctx* c, int64_t tile, int64_t* g_lo, int64_t* g_hi) {
    const int WF = c->W * 5;
    const int64_t c0 = tile * c->CPW, nb = c->qtot - c0 < c->CPW ? c->qtot - c0 : c->CPW;
    const int64_t b_lo = c0 / c->per4, ql = c0 + nb - 1, b_hi = ql / c->per4;
    *g_lo = b_lo * c->N + 4 * (c0 - b_lo * c->per4) / WF;
    *g_hi = b_hi * c->N + (4 * (ql - b_hi * c->per4) + 3) / WF;
}

static int relay_ready(const relay_ctx* c, int64_t tile) {
    int64_t g_lo, g_hi;
    relay_rows(c, tile, &g_lo, &g_hi);
    for (int64_t g = g_lo; g <= g_hi; ++g)
        if ((uint32_t)(c->r->w[g] >> 32) != c->r->epoch) return 0;
    return 1;
}

static void relay_run_tile(relay_ctx* c, int64_t tile) {
    relay_st* r = c->r;
    const int N = c->N, W = c->W, F = 5, WF = W * F, q = c->q;
    CHECK(!c->ran[tile]++, "relay: tile %lld ran twice", (long long)tile);
    const int64_t c0 = tile * c->CPW, CPW = c->CPW, qtot = c->qtot, per4 = c->per4;
    const int64_t nblk = qtot - c0 < CPW ? qtot - c0 : CPW;
    const int64_t nh = tile + 1 < c->ntiles ? (qtot - c0 - nblk < 2 ? qtot - c0 - nblk : 2) : 0;
    for (int64_t j = 0; j < CPW + 2; ++j) {
        for (int e = 0; e < 4; ++e) c->lds[j * 4 + e] = 0.0f;
        if (j < nblk) {
            CHECK(c->dbuf || !c->stored[c0 + j], "relay: chunk %lld read after a store", (long long)(c0 + j));
            for (int e = 0; e < 4; ++e) c->lds[j * 4 + e] = c->in[(c0 + j) * 4 + e];
        } else if (j >= CPW && j - CPW < nh) {
            if (c->dbuf) {
                for (int e = 0; e < 4; ++e) c->lds[j * 4 + e] = c->in[(c0 + nblk + j - CPW) * 4 + e];
            } else {
                CHECK(!c->halo_w[q][tile], "relay: halo %lld read after this step wrote it", (long long)tile);
                CHECK(tile * 8 + (j - CPW) * 4 + 3 < c->nhal, "relay: halo index past its buffer");
                for (int e = 0; e < 4; ++e) c->lds[j * 4 + e] = r->halo[q][tile * 8 + (j - CPW) * 4 + e];
            }
        }
    }
    int64_t g_lo, g_hi;
    relay_rows(c, tile, &g_lo, &g_hi);
    CHECK(g_hi - g_lo < c->BLOCK, "relay: tile %lld stages %lld rows > %d threads", (long long)tile,
          (long long)(g_hi - g_lo + 1), c->BLOCK);
    for (int64_t g = g_lo; g <= g_hi && g - g_lo < c->BLOCK; ++g) {
        const int64_t b = g / N;
        CHECK(g < (int64_t)c->B * N, "relay: row %lld past the batch", (long long)g);
        CHECK((uint32_t)(r->w[g] >> 32) == r->epoch, "relay: tile %lld ran before row %lld's word", (long long)tile,
              (long long)g);
        c->s_kc[g - g_lo] = r->kp[q][b];
        c->s_wp[g - g_lo] = flat1_wp(c->v0[b], c->k0[b], b, (int)(g - b * N));   /* what the word carries */
    }
    for (int64_t j = 0; j < nblk; ++j) {
        const int64_t gq = c0 + j, bq = gq / per4, j0 = 4 * (gq - bq * per4), row = j0 / WF;
        const int kk = (int)(j0 - row * WF);
        const int64_t li = bq * N + row - g_lo;
        CHECK(li >= 0 && li <= g_hi - g_lo, "relay: chunk %lld row index %lld", (long long)gq, (long long)li);
        const int32_t kc = c->s_kc[li];
        CHECK(kc == c->k0[bq], "relay: env %lld counter copy %d != %d", (long long)bq, kc, c->k0[bq]);
        const int shift_w = !(c->storage && kc >= W - 1), slot = (int)((1 + (int64_t)kc) % W);
        for (int e = 0; e < 4; ++e) {
            const int pos = kk + e;
            const int64_t jg = gq * 4 + e, rg = jg / WF;
            const int f = (int)((jg - rg * WF) % F), td = (int)((jg - rg * WF) / F);
            const float un = c->lds[j * 4 + e], sh = c->lds[j * 4 + e + 5];
            float v;
            if (pos >= WF) v = sh;                                   /* the next row's positions 0..2 */
            else if (f == F - 1) v = shift_w ? (td == W - 1 ? c->s_wp[li] : sh) : (td == slot ? c->s_wp[li] : un);
            else v = td == W - 1 ? c->bar[rg * 4 + f] : sh;
            c->out[jg] = v;
            if (!c->dbuf && tile > 0 && j < 2) {
                CHECK((tile - 1) * 8 + j * 4 + e < c->nhal, "relay: halo_out index past its buffer");
                r->halo[1 - q][(tile - 1) * 8 + j * 4 + e] = v;
            }
        }
        c->stored[gq] = 1;
    }
    if (!c->dbuf && tile > 0) c->halo_w[1 - q][tile - 1] = 1;
}

/* a deferred tile's run (relay_tile<ADOPT>): all words arrived and the claim won */
static void relay_adopt_one(relay_ctx* c, uint32_t* done, int64_t tile) {
    if (!relay_ready(c, tile)) return;
    if (done[tile] == c->r->epoch) return;                  /* the claim: ran elsewhere */
    done[tile] = c->r->epoch;
    relay_run_tile(c, tile);
}

static int emulate_relay(int B, int N, int W, int BLOCK, int V, int KL, int T, int storage, int dbuf, int model,
                         int spin) {
    const int F = 5, WF = W * F;
    const int64_t per = (int64_t)N * WF, tot = per * B;
    if (per % 4 || W < 2) return 0;
    const int64_t per4 = per / 4, qtot = tot / 4, CPW = (int64_t)BLOCK * V, ntiles = (qtot + CPW - 1) / CPW;
    const int EPB = (BLOCK / 64) * (64 / KL), scal = (B + EPB - 1) / EPB;
    /* the host plan's closed form (pmenv.hip: at most BLOCK rows per tile) */
    CHECK(4 * CPW / WF + 2 <= BLOCK, "relay: plan admits %lld rows per tile > %d", (long long)(4 * CPW / WF + 2), BLOCK);
    float* buf[2] = {malloc(sizeof(float) * tot), malloc(sizeof(float) * tot)};
    float* ref = malloc(sizeof(float) * tot);
    float* nxt = malloc(sizeof(float) * tot);
    float* bar = malloc(sizeof(float) * B * N * 4);
    float* wp = malloc(sizeof(float) * B * N);
    double* value = malloc(sizeof(double) * B);
    int32_t* k = malloc(sizeof(int32_t) * B);
    int32_t* k0 = malloc(sizeof(int32_t) * B);
    double* v0 = malloc(sizeof(double) * B);
    relay_st r;
    r.w = calloc((size_t)B * N, sizeof(uint64_t));
    r.kp[0] = malloc(sizeof(int32_t) * B); r.kp[1] = malloc(sizeof(int32_t) * B);
    const int64_t nhal = ntiles > 1 ? (ntiles - 1) * 8 : 1;               /* [tiles - 1][2] float4 */
    r.halo[0] = malloc(sizeof(float) * nhal); r.halo[1] = malloc(sizeof(float) * nhal);
    const int grid = scal + (int)ntiles;
    r.epoch = 0xFFFFFFFDu; r.par = 0; r.kp_ok = 0; r.obs = NULL;
    int deadlocked = 0, deferred = 0;
    uint32_t* done = calloc((size_t)ntiles, sizeof(uint32_t));
    int64_t* list = malloc(sizeof(int64_t) * (size_t)ntiles);
    uint8_t* stored = calloc((size_t)qtot, 1);
    uint8_t* halo_w[2] = {calloc((size_t)ntiles, 1), calloc((size_t)ntiles, 1)};   /* written this step, per parity */
    uint8_t* ran = calloc((size_t)ntiles, 1);
    uint8_t* scal_owner = calloc((size_t)B, 1);
    int* polls = malloc(sizeof(int) * (size_t)grid);
    int* order = malloc(sizeof(int) * (size_t)grid);
    int* res_idx = malloc(sizeof(int) * (size_t)grid);  /* resident workgroups */
    relay_ctx c;
    c.r = &r; c.B = B; c.N = N; c.W = W; c.BLOCK = BLOCK; c.storage = storage; c.dbuf = dbuf;
    c.per4 = per4; c.qtot = qtot; c.CPW = CPW; c.ntiles = ntiles; c.nhal = nhal; c.bar = bar; c.v0 = v0; c.k0 = k0;
    c.stored = stored; c.halo_w[0] = halo_w[0]; c.halo_w[1] = halo_w[1]; c.ran = ran;
    c.lds = malloc(sizeof(float) * 4 * (CPW + 2)); c.s_wp = malloc(sizeof(float) * BLOCK);
    c.s_kc = malloc(sizeof(int32_t) * BLOCK);
    int cur = 0;
    for (int64_t i = 0; i < tot; ++i) buf[0][i] = ref[i] = (float)nrand();
    for (int b = 0; b < B; ++b) { value[b] = 25000.0 + b; k[b] = (int32_t)(urand() * 2 * W); }
    for (int t = 0; t < T; ++t) {
        float* in = buf[cur];
        float* out = dbuf ? buf[1 - cur] : buf[cur];
        if (t == T / 3 && !dbuf) {                      /* a caller edit of the window: window_written */
            for (int64_t i = 0; i < tot; i += 7) { in[i] *= 0.5f; ref[i] = in[i]; }
            r.obs = NULL;
        }
        if (t == T / 2) {                               /* a state write: pmenv_state_written */
            for (int b = 0; b < B; b += 3) { value[b] = 25000.0; k[b] = 0; }
            r.kp_ok = 0;
        }
        for (int i = 0; i < B * N * 4; ++i) bar[i] = (float)nrand();
        for (int b = 0; b < B; ++b) {
            k0[b] = k[b]; v0[b] = value[b];
            for (int n = 0; n < N; ++n) wp[b * N + n] = flat1_wp(value[b], k[b], b, n);
            const int shift_w = !(storage && k[b] >= W - 1), slot = (int)((1 + (int64_t)k[b]) % W);
            advance_ref(ref + (size_t)b * per, nxt + (size_t)b * per, 1, N, W, bar + (size_t)b * N * 4,
                        wp + (size_t)b * N, shift_w, slot);
        }
        if (t == 2 * T / 3) {                           /* a step of another path: both copies stale */
            memcpy(out, nxt, sizeof(float) * tot);
            for (int b = 0; b < B; ++b) { value[b] = value[b] * 1.0001 + 1.0; k[b] += 1; }
            r.obs = NULL; r.kp_ok = 0;
        } else {
            /* launch_relay: prime, next epoch (the words, list and claims restart at 0 on the wrap) */
            relay_prime(&r, in, B, k, ntiles, CPW, qtot, !dbuf && r.obs != in);
            if (++r.epoch == 0) {
                memset(r.w, 0, sizeof(uint64_t) * (size_t)B * N);
                memset(done, 0, sizeof(uint32_t) * (size_t)ntiles);
                r.epoch = 1;
            }
            const int q = r.par;
            c.q = q; c.in = in; c.out = out;
            int nlist = 0;
            if (model == 0) for (int i = 0; i < grid; ++i) order[i] = i;
            else if (model == 3) for (int i = 0; i < grid; ++i) order[i] = (i + scal) % grid;   /* blockIdx + rot */
            else shuffle(order, grid);
            const int resident = model == 0 ? 1 + (int)(urand() * (t % 3 == 0 ? 4 : 64))
                               : model == 1 ? grid : model == 2 ? 1 : 1 + (int)(urand() * 4);
            int next = 0, live = 0;
            memset(stored, 0, (size_t)qtot); memset(halo_w[0], 0, (size_t)ntiles); memset(halo_w[1], 0, (size_t)ntiles);
            memset(scal_owner, 0, (size_t)B); memset(ran, 0, (size_t)ntiles);
            for (int i = 0; i < grid; ++i) polls[i] = 0;
            for (int left = grid; left > 0;) {
                while (live < resident && next < grid) res_idx[live++] = order[next++];
                /* a workgroup that can move: a scalar block, or a tile (it runs, polls or defers); without
                 * the deferral (spin < 0) a tile whose words are missing cannot */
                int s2 = (int)(urand() * live), moved = 0;
                for (int tries = 0; tries < live && !moved; ++tries) {
                    if (tries) s2 = (s2 + 1) % live;
                    const int i = res_idx[s2];
                    if (i < scal) {                     /* relay_scalar, then relay_adopt */
                        for (int j = 0; j < EPB; ++j) {
                            const int b = i * EPB + j;
                            if (b >= B) continue;
                            CHECK(!scal_owner[b]++, "relay: env %d stepped twice", b);
                            for (int n = 0; n < N; ++n) r.w[(size_t)b * N + n] = ((uint64_t)r.epoch << 32) | 0u;
                            r.kp[1 - q][b] = k[b] + 1;          /* parity 1 - q: no tile reads it */
                            value[b] = value[b] * 1.0001 + 1.0; /* scalar_tail */
                            k[b] += 1;
                        }
                        for (int e = 0; e < nlist; ++e) relay_adopt_one(&c, done, list[e]);
                    } else {
                        const int64_t tile = i - scal;
                        if (polls[i] <= spin && relay_ready(&c, tile)) {
                            relay_run_tile(&c, tile);
                        } else if (spin < 0) {
                            continue;                   /* waits without bound */
                        } else if (polls[i]++ <= spin) {
                            moved = 1;                  /* a poll (the last one gives up): the tile stays */
                            break;
                        } else {                        /* relay_defer, a later event: append, re-check once, exit */
                            CHECK(nlist < ntiles, "relay: deferral list past its %lld entries", (long long)ntiles);
                            list[nlist++] = tile;
                            ++deferred;
                            relay_adopt_one(&c, done, tile);
                        }
                    }
                    res_idx[s2] = res_idx[--live]; --left;
                    moved = 1;
                }
                if (!moved && spin < 0 && model == 2) { deadlocked = 1; break; }
                CHECK(moved, "relay: deadlock, %d resident workgroups all wait (B%d N%d W%d model %d spin %d)", live, B,
                      N, W, model, spin);
                if (!moved) break;
            }
            if (deadlocked) break;
            for (int b = 0; b < B; ++b) CHECK(scal_owner[b] == 1, "relay: env %d stepped %d times", b, scal_owner[b]);
            for (int64_t i = 0; i < ntiles; ++i) CHECK(ran[i] == 1, "relay: tile %lld ran %d times (model %d)", (long long)i,
                                                       ran[i], model);
            r.par = 1 - q; r.kp_ok = 1; r.obs = dbuf ? NULL : out;
        }
        float* sw = ref; ref = nxt; nxt = sw;
        for (int64_t i = 0; i < tot; ++i)
            if (memcmp(&out[i], &ref[i], 4)) {
                CHECK(0, "relay: step %d float %lld differs (B%d N%d W%d %dx%d db%d model %d)", t, (long long)i, B, N, W,
                      BLOCK, V, dbuf, model);
                break;
            }
        if (dbuf) cur = 1 - cur;
    }
    free(buf[0]); free(buf[1]); free(ref); free(nxt); free(bar); free(wp); free(value); free(k); free(k0); free(v0);
    free(r.w); free(r.kp[0]); free(r.kp[1]); free(r.halo[0]); free(r.halo[1]); free(stored); free(halo_w[0]);
    free(halo_w[1]); free(ran); free(done); free(list); free(scal_owner); free(polls); free(order); free(res_idx);
    free(c.lds); free(c.s_wp); free(c.s_kc);
    if (model >= 2 && spin >= 0) CHECK(deferred > 0, "relay: model %d never exercised the deferral", model);
    return deadlocked;
}

/* ------------------------------------------------------------ 5. the look-back GAE */
/* pmenv.hip gae_lb_seg / gae_lb_chunks / pmenv_gae_workspace, restated */
static int lb_seg(int T, int B) { return (int64_t)((T + 127) / 128) * ((B + 63) / 64) >= 128 ? 128 : 64; }
static int lb_chunks(int T, int B, int seg) {
    if (B >= 8192 || T < 512 || (size_t)(T + 1) * (size_t)B * 4u >= (1ull << 31)) return 0;
    return (T + seg - 1) / seg;
}

/* chunk c's map for env lane of block eb, as a publisher reduces it (lb_wave_map per wave, folded
 * from wave NW - 1); st_* (may be NULL) receive the days' deltas / alive bits / values */
static void lb_map_lane(const float* r, const float* v, const uint8_t* d, int T, int B, double g, double gl, int NW,
                        int U, int c, int eb, int lane, double* Ca_out, double* Da_out, double* wc, double* wd,
                        double* st_dl, uint8_t* st_al, double* st_vv) {
    const int S = NW * U, seg_start = c * S, seg_end = seg_start + S < T ? seg_start + S : T;
    const int b = eb * 64 + lane, bb = b < B ? b : B - 1;
    double Ca = 1.0, Da = 0.0;
    for (int w = 0; w < NW; ++w) {
        const int t0 = seg_start + w * U;
        double C = 1.0, D = 0.0;
        for (int u = U - 1; u >= 0; --u) {
            const int tv = t0 + u + 1 < seg_end ? t0 + u + 1 : seg_end;     /* vv[u + 1] */
            const int tu = t0 + u < seg_end ? t0 + u : seg_end;             /* vv[u] */
            const int tr = t0 + u < seg_end - 1 ? t0 + u : seg_end - 1;
            CHECK((size_t)tv * B + bb < (size_t)(T + 1) * B && (size_t)tr * B + bb < (size_t)T * B, "gae_lb: load index");
            const double n = d && d[(size_t)tr * B + bb] ? 0.0 : 1.0;
            const double dl = (double)r[(size_t)tr * B + bb] + g * n * (double)v[(size_t)tv * B + bb] -
                              (double)v[(size_t)tu * B + bb];
            if (st_dl) {
                const size_t si = (size_t)w * U + u;
                st_dl[si] = dl; st_al[si] = (uint8_t)n; st_vv[si] = (double)v[(size_t)tu * B + bb];
            }
            if (t0 + u < seg_end) { D = dl + gl * n * D; C = gl * n * C; }
        }
        wc[w] = C; wd[w] = D;
    }
    for (int w = NW - 1; w >= 0; --w) { Da = wd[w] + wc[w] * Da; Ca = wc[w] * Ca; }
    *Ca_out = Ca; *Da_out = Da;
}

/* one call of gae_lookback_kernel<NW, U> on a workspace `ws` of exactly the ABI's size. Workgroups
 * are dispatched in blockIdx order (later chunks first) or in a random permutation, at most
 * `resident` on the device at once (a finished one frees its slot); a resident workgroup
 * waiting for flags holds its slot. When every resident workgroup waits (its producers not
 * dispatched), one of them takes the kernel's fallback: it computes the missing chunks' maps
 * itself (the producers' code; they must agree bit for bit when a producer publishes later). */
static void lb_call(const float* r, const float* v, const uint8_t* d, float* adv, float* ret, int T, int B, double g,
                    double gl, int NW, int U, int nC, double* ws, size_t ws_doubles, uint64_t epoch, int resident,
                    int random_order) {
    const int S = NW * U, nEB = (B + 63) / 64, nblk = nC * nEB;
    double* mapC = ws;
    double* mapD = ws + (size_t)nC * B;
    uint64_t* flags = (uint64_t*)(ws + (size_t)2 * nC * B);
    CHECK((size_t)2 * nC * B + (size_t)nC * nEB <= ws_doubles, "gae_lb: workspace too small");
    /* per block: its registers (dl, alive, vv) and LDS maps between the two phases */
    double* st_dl = malloc(sizeof(double) * (size_t)nblk * 64 * S);
    double* st_vv = malloc(sizeof(double) * (size_t)nblk * 64 * S);
    uint8_t* st_al = malloc((size_t)nblk * 64 * S);
    double* shC = malloc(sizeof(double) * (size_t)nblk * NW * 64);
    double* shD = malloc(sizeof(double) * (size_t)nblk * NW * 64);
    int* phase = calloc((size_t)nblk, sizeof(int));
    int* runnable = malloc(sizeof(int) * (size_t)nblk);
    int* order = malloc(sizeof(int) * (size_t)nblk);
    uint8_t* res = calloc((size_t)nblk, 1);
    uint8_t* forced = calloc((size_t)nblk, 1);         /* took the fallback: composes without flags */
    uint8_t* fb = calloc((size_t)nC * nEB, 1);          /* a chunk's map written by a fallback */
    if (random_order) shuffle(order, nblk);
    else for (int i = 0; i < nblk; ++i) order[i] = i;
    int next = 0, live = 0, fallbacks = 0;
    double wc[64], wd[64];
    for (int left = 2 * nblk; left > 0; --left) {
        while (live < resident && next < nblk) { res[order[next++]] = 1; ++live; }
        int nr = 0;
        for (int bi = 0; bi < nblk; ++bi) {
            if (!res[bi] || phase[bi] == 2) continue;
            if (phase[bi] == 1 && !forced[bi]) {
                const int c = nC - 1 - bi / nEB, eb = bi % nEB;
                int ready = 1;
                for (int j = c + 1; j < nC && ready; ++j) ready = flags[(size_t)j * nEB + eb] == epoch;
                if (!ready) continue;
            }
            runnable[nr++] = bi;
        }
        if (!nr) {                                      /* every resident waits: a spin bound expires */
            int waiting = 0;
            for (int bi = 0; bi < nblk; ++bi) if (res[bi] && phase[bi] == 1) runnable[waiting++] = bi;
            CHECK(waiting > 0, "gae_lb: no workgroup can run and none waits");
            if (!waiting) break;
            const int bi = runnable[(int)(urand() * waiting)];
            const int c = nC - 1 - bi / nEB, eb = bi % nEB;
            for (int j = c + 1; j < nC; ++j) {
                if (flags[(size_t)j * nEB + eb] == epoch) continue;
                for (int lane = 0; lane < 64; ++lane) {
                    const int b = eb * 64 + lane;
                    double Ca, Da;
                    lb_map_lane(r, v, d, T, B, g, gl, NW, U, j, eb, lane, &Ca, &Da, wc, wd, NULL, NULL, NULL);
                    if (b < B) { mapC[(size_t)j * B + b] = Ca; mapD[(size_t)j * B + b] = Da; }
                }
                fb[(size_t)j * nEB + eb] = 1;
                ++fallbacks;
            }
            forced[bi] = 1;
            runnable[0] = bi;
            nr = 1;
        }
        const int bi = runnable[(int)(urand() * nr)];
        const int c = nC - 1 - bi / nEB, eb = bi % nEB;
        const int seg_start = c * S, seg_end = seg_start + S < T ? seg_start + S : T;
        if (phase[bi] == 0) {                           /* load, reduce, publish */
            for (int lane = 0; lane < 64; ++lane) {
                const int b = eb * 64 + lane, ok = b < B;
                double Ca, Da;
                const size_t si = ((size_t)bi * 64 + lane) * S;
                lb_map_lane(r, v, d, T, B, g, gl, NW, U, c, eb, lane, &Ca, &Da, wc, wd, st_dl + si, st_al + si,
                            st_vv + si);
                for (int w = 0; w < NW; ++w) {
                    shC[((size_t)bi * NW + w) * 64 + lane] = wc[w];
                    shD[((size_t)bi * NW + w) * 64 + lane] = wd[w];
                }
                if (ok && fb[(size_t)c * nEB + eb])
                    CHECK(!memcmp(&mapC[(size_t)c * B + b], &Ca, 8) && !memcmp(&mapD[(size_t)c * B + b], &Da, 8),
                          "gae_lb: a fallback map differs from the producer's (chunk %d env %d)", c, b);
                if (ok) { mapC[(size_t)c * B + b] = Ca; mapD[(size_t)c * B + b] = Da; }
            }
            flags[(size_t)c * nEB + eb] = epoch;
            phase[bi] = 1;
            continue;
        }
        /* compose the later chunks' maps (a part per wave), then walk and store */
        for (int lane = 0; lane < 64; ++lane) {
            const int b = eb * 64 + lane, ok = b < B, bb = ok ? b : B - 1;
            const int nl = nC - 1 - c, m = (nl + NW - 1) / NW;
            double sxC[64], sxD[64];
            for (int w = 0; w < NW; ++w) {
                const int j0 = c + 1 + w * m, j1 = j0 + m < nC ? j0 + m : nC;
                double Cw = 1.0, Dw = 0.0;
                for (int j = j1 - 1; j >= j0; --j) {
                    Dw = mapD[(size_t)j * B + bb] + mapC[(size_t)j * B + bb] * Dw;
                    Cw = mapC[(size_t)j * B + bb] * Cw;
                }
                sxC[w] = Cw; sxD[w] = Dw;
            }
            for (int w = 0; w < NW; ++w) {
                double a = 0.0;
                for (int j = NW - 1; j >= 0; --j) a = sxD[j] + sxC[j] * a;
                for (int j = NW - 1; j > w; --j)
                    a = shD[((size_t)bi * NW + j) * 64 + lane] + shC[((size_t)bi * NW + j) * 64 + lane] * a;
                const int t0 = seg_start + w * U;
                for (int u = U - 1; u >= 0; --u) {
                    const int t = t0 + u;
                    if (t >= seg_end) continue;
                    const size_t si = ((size_t)bi * 64 + lane) * S + (size_t)w * U + u;
                    a = st_dl[si] + gl * (double)st_al[si] * a;
                    if (ok) { adv[(size_t)t * B + b] = (float)a; ret[(size_t)t * B + b] = (float)(a + st_vv[si]); }
                }
            }
        }
        phase[bi] = 2;
        res[bi] = 0;
        --live;
    }
    for (int bi = 0; bi < nblk; ++bi) CHECK(phase[bi] == 2, "gae_lb: workgroup %d never finished", bi);
    CHECK(random_order || resident < nblk || !fallbacks, "gae_lb: a fallback under blockIdx dispatch with every workgroup resident");
    free(st_dl); free(st_vv); free(st_al); free(shC); free(shD); free(phase); free(runnable);
    free(order); free(res); free(forced); free(fb);
}

/* gae_lookback2_kernel (tools build, PMENV_GAE=lb2 / lb2x16): pairs of adjacent chunks (B = 2p, A = 2p + 1)
 * per workgroup, later pairs dispatched first, at most `resident` workgroups on the device at
 * once (a finished one frees its slot for the next in dispatch order). Phases: 0 load A and B,
 * publish A; 1 look back A (waits for chunks > A) and store it; 2 publish B; 3 look back B
 * (waits for chunks > B) and store it. Every wait must be on a published chunk or on a
 * workgroup already resident: a schedule in which no resident workgroup can move is a
 * deadlock, which the kernel must never have. Checks the result against the restatement. */
static void emulate_gae_lb2(int T, int B, int NW, int U, int resident) {
    const int S = NW * U, nC = (T + S - 1) / S, nEB = (B + 63) / 64, nP = (nC + 1) / 2, nblk = nP * nEB;
    float* r = malloc(sizeof(float) * (size_t)T * B);
    float* v = malloc(sizeof(float) * (size_t)(T + 1) * B);
    uint8_t* d = malloc((size_t)T * B);
    float* adv = malloc(sizeof(float) * (size_t)T * B);
    float* ret = malloc(sizeof(float) * (size_t)T * B);
    float* oa = malloc(sizeof(float) * (size_t)T * B);
    float* orr = malloc(sizeof(float) * (size_t)T * B);
    for (size_t i = 0; i < (size_t)T * B; ++i) { r[i] = (float)nrand(); d[i] = urand() < 0.01; }
    for (size_t i = 0; i < (size_t)(T + 1) * B; ++i) v[i] = (float)nrand();
    const double g = 0.99, gl = 0.99 * (double)0.95f;
    /* per chunk: the published map (C, D per env) and whether it is published */
    double* mC = malloc(sizeof(double) * (size_t)nC * B);
    double* mD = malloc(sizeof(double) * (size_t)nC * B);
    uint8_t* pub = calloc((size_t)nC * nEB, 1);
    int* phase = calloc((size_t)nblk, sizeof(int));
    int* runnable = malloc(sizeof(int) * (size_t)nblk);
    int next = 0, live = 0;                          /* dispatch cursor, resident count */
    uint8_t* res = calloc((size_t)nblk, 1);
    /* the chunk's reduction and walk, as the kernel's lanes do them, straight on the arrays */
    #define LB_MAP(c, eb) do { \
        for (int lane = 0; lane < 64; ++lane) { const int b_ = (eb) * 64 + lane; if (b_ >= B) continue; \
            const int s0 = (c) * S, s1 = s0 + S < T ? s0 + S : T; double Ca = 1.0, Da = 0.0; \
            for (int w = NW - 1; w >= 0; --w) { double C = 1.0, D = 0.0; \
                for (int u = U - 1; u >= 0; --u) { const int t = s0 + w * U + u; if (t >= s1) continue; \
                    const double n = d[(size_t)t * B + b_] ? 0.0 : 1.0; \
                    const double dl = (double)r[(size_t)t * B + b_] + g * n * (double)v[(size_t)(t + 1) * B + b_] - (double)v[(size_t)t * B + b_]; \
                    D = dl + gl * n * D; C = gl * n * C; } \
                Da = D + C * Da; Ca = C * Ca; } \
            mC[(size_t)(c) * B + b_] = Ca; mD[(size_t)(c) * B + b_] = Da; } \
        pub[(size_t)(c) * nEB + (eb)] = 1; } while (0)
    #define LB_WALK(c, eb) do { \
        for (int lane = 0; lane < 64; ++lane) { const int b_ = (eb) * 64 + lane; if (b_ >= B) continue; \
            double a = 0.0; for (int j = nC - 1; j > (c); --j) a = mD[(size_t)j * B + b_] + mC[(size_t)j * B + b_] * a; \
            const int s0 = (c) * S, s1 = s0 + S < T ? s0 + S : T; \
            for (int t = s1 - 1; t >= s0; --t) { const double n = d[(size_t)t * B + b_] ? 0.0 : 1.0; \
                const double dl = (double)r[(size_t)t * B + b_] + g * n * (double)v[(size_t)(t + 1) * B + b_] - (double)v[(size_t)t * B + b_]; \
                a = dl + gl * n * a; adv[(size_t)t * B + b_] = (float)a; ret[(size_t)t * B + b_] = (float)(a + (double)v[(size_t)t * B + b_]); } } } while (0)
    for (;;) {
        while (live < resident && next < nblk) { res[next++] = 1; ++live; }
        int nr = 0, left = 0;
        for (int bi = 0; bi < nblk; ++bi) {
            if (phase[bi] == 4) continue;
            ++left;
            if (!res[bi]) continue;
            const int pr = nP - 1 - bi / nEB, eb = bi % nEB, cA = 2 * pr + 1, cB = 2 * pr;
            int ok = 1;
            if (phase[bi] == 1 || phase[bi] == 3) {
                const int c = phase[bi] == 1 ? cA : cB;
                for (int j = c + 1; j < nC && ok; ++j) ok = pub[(size_t)j * nEB + eb];
            }
            if (ok) runnable[nr++] = bi;
        }
        if (!left) break;
        CHECK(nr > 0, "gae_lb2: deadlock (T%d B%d %dx%d, %d resident)", T, B, NW, U, resident);
        if (!nr) break;
        const int bi = runnable[(int)(urand() * nr)];
        const int pr = nP - 1 - bi / nEB, eb = bi % nEB, cA = 2 * pr + 1, cB = 2 * pr;
        switch (phase[bi]) {
        case 0: if (cA < nC) LB_MAP(cA, eb); phase[bi] = cA < nC ? 1 : 2; break;
        case 1: LB_WALK(cA, eb); phase[bi] = 2; break;
        case 2: LB_MAP(cB, eb); phase[bi] = 3; break;
        default: LB_WALK(cB, eb); phase[bi] = 4; res[bi] = 0; --live; break;
        }
    }
    #undef LB_MAP
    #undef LB_WALK
    or_gae(r, v, d, oa, orr, T, B, 0.99f, 0.95f);
    for (size_t i = 0; i < (size_t)T * B; ++i)
        if (!(fabsf(adv[i] - oa[i]) <= 1e-5f * (1.0f + fabsf(oa[i])))) {
            CHECK(0, "gae_lb2: T%d B%d element %zu: %g vs %g", T, B, i, adv[i], oa[i]);
            break;
        }
    free(r); free(v); free(d); free(adv); free(ret); free(oa); free(orr); free(mC); free(mD); free(pub); free(phase);
    free(runnable); free(res);
}

static void emulate_gae_lb(int T, int B, int NW, int U, int resident, int random_order) {
    const int seg = NW * U, nC = (T + seg - 1) / seg, nEB = (B + 63) / 64;
    const size_t ws_doubles = (size_t)2 * nC * B + (size_t)nC * nEB;
    double* ws = malloc(sizeof(double) * ws_doubles);
    for (size_t i = 0; i < ws_doubles; ++i) ((uint64_t*)ws)[i] = ((uint64_t)(urand() * 4294967296.0) << 32) ^ (uint64_t)(urand() * 4294967296.0);
    float* r = malloc(sizeof(float) * (size_t)T * B);
    float* v = malloc(sizeof(float) * (size_t)(T + 1) * B);
    uint8_t* d = malloc((size_t)T * B);
    float* adv = malloc(sizeof(float) * (size_t)T * B);
    float* ret = malloc(sizeof(float) * (size_t)T * B);
    float* oa = malloc(sizeof(float) * (size_t)T * B);
    float* orr = malloc(sizeof(float) * (size_t)T * B);
    uint64_t epoch = 0x51ED270B00000001ull;
    for (int call = 0; call < 2; ++call, ++epoch) {    /* the second call finds the first's maps and flags */
        for (size_t i = 0; i < (size_t)T * B; ++i) { r[i] = (float)nrand(); d[i] = urand() < 0.01; }
        for (size_t i = 0; i < (size_t)(T + 1) * B; ++i) v[i] = (float)nrand();
        const float gamma = 0.99f, lam = call ? 1.0f : 0.95f;
        lb_call(r, v, call ? NULL : d, adv, ret, T, B, (double)gamma, (double)gamma * (double)lam, NW, U, nC, ws,
                ws_doubles, epoch, resident, random_order);
        or_gae(r, v, call ? NULL : d, oa, orr, T, B, gamma, lam);
        for (size_t i = 0; i < (size_t)T * B; ++i)
            if (!(fabsf(adv[i] - oa[i]) <= 1e-5f * (1.0f + fabsf(oa[i]))) ||
                !(fabsf(ret[i] - orr[i]) <= 1e-5f * (1.0f + fabsf(orr[i])))) {
                CHECK(0, "gae_lb: T%d B%d %dx%d call %d element %zu: %g vs %g", T, B, NW, U, call, i, adv[i], oa[i]);
                break;
            }
    }
    free(ws); free(r); free(v); free(d); free(adv); free(ret); free(oa); free(orr);
}

/* ------------------------------------------------------------ 6. address audits (no data) */
/* the scalar-step grids of launch.h launch_scalar_kernels (threads), per form */
static int64_t scalar_threads(int B, int N, int form) {
    if (form == 801) return ((int64_t)(B + 7) / 8 + 3) / 4 * 256;
    if (form == 1601) return ((int64_t)(B + 3) / 4 + 3) / 4 * 256;
    if (form == 1602) return ((int64_t)(B + 3) / 4 + 3) / 4 * 256;          /* tools: scalar_step_vec_kernel<16, 2> */
    if (form == 6402 || form == 6404 || form == 6408) return ((int64_t)B + 3) / 4 * 256;
    if (N <= 64) return ((int64_t)(B + (N <= 32 ? 1 : 0)) / (N <= 32 ? 2 : 1) + 3) / 4 * 256;
    return (int64_t)B * 64;                                                  /* scalar_step_kernel: a wave per env */
}

static void audit_halo_and_direct(int B, int N, int W, int block, int vec, int form) {
    const int64_t per4 = (int64_t)N * W * 5 / 4, qtot = (int64_t)B * per4, cpw = (int64_t)block * vec;
    const int64_t wgs = (qtot + cpw - 1) / cpw, halo_wgs = wgs > 0 ? wgs - 1 : 0;
    const int64_t halo_f4 = 2 * (halo_wgs + 1);                               /* hipMalloc((halo_wgs + 1) * 32) */
    CHECK(qtot < (1ll << 31) - 1024, "audit: %d x %d past the flat stream's index", B, N);
    uint8_t* written = calloc((size_t)halo_wgs + 1, 1);
    const uint32_t nthr = (uint32_t)scalar_threads(B, N, form);
    /* halo_load / halo_store (the register-held copy: two entries per thread, a loop beyond) */
    for (uint32_t gid = 0; gid < nthr; ++gid) {
        for (int t = 0; t < 2; ++t) {
            const uint64_t i = (uint64_t)gid + (uint64_t)t * nthr;
            if (i >= (uint64_t)halo_wgs) continue;
            const uint64_t q = (i + 1) * (uint64_t)cpw;
            CHECK(q <= 0xFFFFFFFFull, "audit: uint32 chunk index overflows");
            CHECK(2 * i + 1 < (uint64_t)halo_f4, "audit: halo store past its buffer");
            CHECK(q + 1 < (uint64_t)qtot, "audit: halo source past the window (%llu)", (unsigned long long)q);
            CHECK(!written[i]++, "audit: halo %llu written twice", (unsigned long long)i);
        }
    }
    for (uint64_t i = (uint64_t)2 * nthr; i < (uint64_t)halo_wgs; ++i) {    /* halo_store's loop */
        CHECK(2 * i + 1 < (uint64_t)halo_f4 && (i + 1) * (uint64_t)cpw + 1 < (uint64_t)qtot, "audit: halo loop index");
        CHECK(!written[i]++, "audit: halo %llu written twice", (unsigned long long)i);
    }
    for (int64_t i = 0; i < halo_wgs; ++i) CHECK(written[i] == 1, "audit: halo %lld not copied", (long long)i);
    /* advance_flat_direct_kernel<block, vec>: descriptors and the halo pointer per tile */
    for (int64_t t = 0; t < wgs; ++t) {
        const int64_t c0 = t * cpw, nblk = qtot - c0 < cpw ? qtot - c0 : cpw;
        CHECK(nblk > 0 && c0 + nblk <= qtot, "audit: direct tile %lld range", (long long)t);
        const int64_t nh = t + 1 < wgs ? (qtot - c0 - nblk < 2 ? qtot - c0 - nblk : 2) : 0;
        CHECK(nh == 0 || (t < halo_wgs && 2 * t + nh <= halo_f4), "audit: direct tile %lld halo", (long long)t);
        for (int64_t j = 0; j < cpw; ++j)                          /* shifted source: j + 3 <= nblk */
            if (j + 3 <= nblk) CHECK(j * 16 + 20 + 16 <= nblk * 16, "audit: direct shifted load past its range");
        if (nblk >= 2) CHECK(nblk - 2 + 1 <= nblk, "audit: direct edge");
    }
    free(written);
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
    /* the generic stream (F != 5): the product's 512 x 2 and 256 x 2 tiles (and 256 x 4, the
     * tools build's), and small ones (64 threads x 1) that put many envs and rows in one tile,
     * both weight-channel modes */
    const int gshp[][4] = {{4, 30, 50, 8}, {11, 8, 10, 3}, {9, 5, 12, 2}, {13, 9, 8, 4}, {7, 3, 20, 6},
                           {5, 11, 4, 7}, {3, 64, 16, 8}, {2, 65, 16, 4}, {40, 2, 10, 6},
                           /* past F = 8: the four-chunk halo */
                           {3, 30, 50, 12}, {5, 7, 10, 16}, {9, 5, 4, 9}, {11, 3, 6, 10}, {4, 13, 3, 13},
                           {6, 9, 2, 14}, {3, 20, 8, 11}, {2, 16, 32, 15}};
    for (size_t i = 0; i < sizeof gshp / sizeof gshp[0]; ++i)
        for (int mode = 0; mode < 2; ++mode) {
            const int B = gshp[i][0], N = gshp[i][1], W = gshp[i][2], F = gshp[i][3];
            const int sl = mode ? (int)(urand() * W) : 0;
            if (4 * 1024 / (W * F) + 2 <= 256) emulate_gen(B, N, W, F, 256, 1024, mode == 0, sl);
            if (4 * 1024 / (W * F) + 2 <= 512) emulate_gen(B, N, W, F, 512, 1024, mode == 0, sl);
            if (4 * 512 / (W * F) + 2 <= 256) emulate_gen(B, N, W, F, 256, 512, mode == 0, sl);
            if (4 * 64 / (W * F) + 2 <= 64) emulate_gen(B, N, W, F, 64, 64, mode == 0, sl);
        }
    /* the surface stream's staged ring columns: rows of 20 .. 400 floats, tiles spanning
     * many envs, the product's 1,024-chunk tiles and small ones */
    const int sshp[][4] = {{9, 30, 50, 5}, {51, 4, 5, 4}, {13, 16, 12, 8}, {7, 5, 50, 8}, {300, 4, 5, 4},
                           {5, 30, 50, 3}, {2, 64, 50, 6}};
    for (size_t i = 0; i < sizeof sshp / sizeof sshp[0]; ++i) {
        emulate_surf(sshp[i][0], sshp[i][1], sshp[i][2], sshp[i][3], 1024);
        emulate_surf(sshp[i][0], sshp[i][1], sshp[i][2], sshp[i][3], 64);
    }
    /* the flat one-launch step: the product's 1,024-chunk tiles (256 x 4 and 512 x 2) and
     * small tiles that put several tiles in one env and several envs in one tile, both ring
     * orders, through the wrap and a re-prime */
    const int fshapes[][3] = {{37, 30, 50}, {301, 4, 30}, {3, 64, 47}, {13, 5, 4}, {9, 1, 4}, {130, 2, 60}};
    for (size_t i = 0; i < sizeof fshapes / sizeof fshapes[0]; ++i)
        for (int storage = 0; storage < 2; ++storage)
            for (int cpw = 0; cpw < 2; ++cpw)
                emulate_flat1(fshapes[i][0], fshapes[i][1], fshapes[i][2], cpw ? 1024 : 96, 2 * fshapes[i][2] + 3,
                              storage);
    /* the relayed step: the product's 256 x 2 and 512 x 2 tiles (256 x 4 below), small tiles that put many
     * rows and envs in one tile, the register (32 / 64 lanes) and packed (8 / 16 lanes)
     * scalar forms' blocks, W = 2 (every day a last day), both ring orders, in place and
     * double-buffered; every dispatch model, the fallback after 0 to 3 polls */
    const int rshapes[][4] = {{37, 30, 50, 32}, {301, 8, 12, 8}, {97, 16, 20, 16}, {9, 64, 47, 64}, {400, 30, 2, 32},
                              {13, 5, 48, 8}, {3, 1, 600, 8}, {61, 24, 3, 32}};
    const int bks[3] = {256, 512, 64};
    for (size_t i = 0; i < sizeof rshapes / sizeof rshapes[0]; ++i)
        for (int storage = 0; storage < 2; ++storage)
            for (int db = 0; db < 2; ++db)
                for (int model = 0; model < 4; ++model)
                    for (int bk = 0; bk < 3; ++bk)
                        emulate_relay(rshapes[i][0], rshapes[i][1], rshapes[i][2], bks[bk], 2, rshapes[i][3], 12, storage,
                                      db, model, (int)(urand() * 4));
    /* the 256 x 4 tiles AUTO gives the largest cache-resident in-place windows (register form,
     * 17 <= N <= 32) */
    for (size_t i = 0; i < sizeof rshapes / sizeof rshapes[0]; ++i)
        if (rshapes[i][3] == 32 && 4 * 256 * 4 / (rshapes[i][2] * 5) + 2 <= 256)
            for (int storage = 0; storage < 2; ++storage)
                for (int model = 0; model < 4; ++model)
                    emulate_relay(rshapes[i][0], rshapes[i][1], rshapes[i][2], 256, 4, 32, 12, storage, 0, model,
                                  (int)(urand() * 4));
    /* negative control: without the fallback (round 5's kernel), a non-monotone dispatch order with
     * one workgroup resident deadlocks (a tile dispatched before its scalar block waits forever) —
     * the detection above sees a deadlock when there is one */
    int dl = 0;
    for (int rep = 0; rep < 8 && !dl; ++rep) dl = emulate_relay(37, 30, 50, 64, 2, 32, 3, 1, 0, 2, -1);
    CHECK(dl, "relay: no deadlock without the fallback under a non-monotone order, one resident (negative control)");
    /* the look-back GAE: the product's rule and both chunk lengths, ragged B and T, one chunk */
    const int gshapes[][2] = {{700, 67}, {513, 3}, {1000, 130}, {600, 64}, {130, 5}};
    for (size_t i = 0; i < sizeof gshapes / sizeof gshapes[0]; ++i) {
        /* every workgroup resident in any order; blockIdx order at a few resident; a random,
         * non-monotone dispatch order at one to a few resident (the fallback's case) */
        emulate_gae_lb(gshapes[i][0], gshapes[i][1], 8, 8, 1 << 30, 0);
        emulate_gae_lb(gshapes[i][0], gshapes[i][1], 8, 16, 1 << 30, 0);
        emulate_gae_lb(gshapes[i][0], gshapes[i][1], 8, 8, 3, 0);
        emulate_gae_lb(gshapes[i][0], gshapes[i][1], 8, 16, 1, 1);
        emulate_gae_lb(gshapes[i][0], gshapes[i][1], 8, 8, 5, 1);
    }
    /* the paired kernel (tools build) under every residency, down to one workgroup */
    for (int res = 1; res <= 9; res += 4) {
        emulate_gae_lb2(700, 67, 8, 8, res);
        emulate_gae_lb2(1000, 130, 8, 16, res);
        emulate_gae_lb2(130, 5, 8, 8, res);
    }
    {   /* the rule's choice at the shapes the GPU tests run */
        const int rs[][2] = {{512, 64}, {4096, 512}, {1000, 200}, {5000, 3}, {2048, 4096}, {700, 4099}, {16384, 64}};
        for (size_t i = 0; i < sizeof rs / sizeof rs[0]; ++i)
            CHECK(lb_chunks(rs[i][0], rs[i][1], lb_seg(rs[i][0], rs[i][1])) > 0 || rs[i][0] < 512,
                  "gae_lb: rule declines %d x %d", rs[i][0], rs[i][1]);
    }
    /* addresses of the halo copy and the tools build's direct stream at the r03d record's
     * shapes (16,384 x 30 included) and the BASELINE ones, every scalar grid */
    const int ashapes[][3] = {{8192, 30, 50}, {4096, 30, 50}, {16384, 30, 50}, {65536, 30, 50}, {8192, 16, 50},
                              {8192, 500, 50}, {4096, 8, 50}, {3, 1, 2}};
    const int forms[] = {0, 801, 1601, 1602, 6402, 6408};
    for (size_t i = 0; i < sizeof ashapes / sizeof ashapes[0]; ++i)
        for (size_t f = 0; f < sizeof forms / sizeof forms[0]; ++f)
            for (int g = 0; g < 2; ++g)
                audit_halo_and_direct(ashapes[i][0], ashapes[i][1], ashapes[i][2], g ? 512 : 256, 2, forms[f]);
    if (fails) { fprintf(stderr, "%d check(s) failed\n", fails); return 1; }
    printf("sanitize ok\n");
    return 0;
}
