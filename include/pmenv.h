/*
 * pmenv.h — C ABI of the MI355X-native vectorised portfolio environment.
 *
 * This is the drop-in boundary for the hot path of zachramsey/pm-rl:
 *   env/sim/trading_env.py   (TradingEnv.__init__ :8-18, reset :21-41, step :44-105)
 *   env/sim/weight_buffer.py (ActionBuffer :5-51 — the W x N weight ring)
 *   env/reward.py            (Reward :6-31 — returns / log_returns / sharpe_ratio)
 *   data/instrument.py:79    (price relatives y_t = close_t / close_{t-1})
 *   data/instrument.py:339-356 (sliding window; fused here as an in-place window advance)
 *
 * The reference is a single-env Python class driven from train/on_policy.py:59-67;
 * here B lockstep envs share one handle and one HIP kernel launch per step.
 *
 * Conventions
 *   - every entry point returns 0 (PMENV_OK) or a negative pmenv_status;
 *     pmenv_last_error(h) then holds a message.
 *   - every data pointer passed to reset/step is a DEVICE pointer owned by the
 *     caller (e.g. a torch tensor's data_ptr()); env state is owned by the handle.
 *   - layouts are dense row-major: obs [B, N, W, F] fp32, action [B, N] fp32,
 *     prices [B, N] fp32, bar [B, N, F-1] fp32, reward [B] fp32.
 *   - one handle belongs to one device; calls on a handle are not thread-safe;
 *     reset/step enqueue on `stream` and never synchronise the host, allocate,
 *     or free (they are hipGraph-capturable).
 */
#ifndef PMENV_H
#define PMENV_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: pmenv_window_written / pmenv_state_written and PMENV_STEP_PATH_RELAY added;
 *    pmenv_cfg_default's ret_mode is PMENV_RET_GROSS (trading_env.py:88 for every reward
 *    kind; was AUTO in 1) */
/* 3: pmenv_step_host / pmenv_reset_host (host buffers, the reference driver's call shape) */
#define PMENV_ABI_VERSION 3

/* Opaque HIP stream (identical to HIP's own typedef); NULL = default stream. */
typedef struct ihipStream_t* hipStream_t;

typedef struct pmenv pmenv; /* opaque handle */

typedef enum pmenv_status {
    PMENV_OK = 0,
    PMENV_ERR_ARG = -1,    /* bad config value or NULL where a pointer is required */
    PMENV_ERR_SHAPE = -2,  /* shape mismatch; weight_buffer.py:18-19 raises ValueError */
    PMENV_ERR_HIP = -3,    /* a HIP runtime call failed */
    PMENV_ERR_ALIGN = -4   /* pointer not 4-byte aligned */
} pmenv_status;

/* Reward kinds. The reference step() hard-codes log_returns (trading_env.py:99);
 * REWARD switch at trading_env.py:93-98 is commented out; env/reward.py:15-31
 * restates returns/log_returns/sharpe_ratio; differential Sharpe is absent from
 * the reference (north star addition, parity unpinned by the reference). */
typedef enum pmenv_reward_kind {
    PMENV_REWARD_LOG_RETURN = 0,  /* r = log(ret) * scale           trading_env.py:99 */
    PMENV_REWARD_RETURN = 1,      /* r = ret * scale                reward.py:20-21   */
    PMENV_REWARD_SHARPE = 2,      /* (mean(ret_1..t) - rf) / std(ret_1..t, ddof=1) * scale, reward.py:26-31 (NaN while t < 2, as numpy) */
    PMENV_REWARD_DIFF_SHARPE = 3  /* Moody-Saffell differential Sharpe on R = ret - 1, EMA rate eta */
} pmenv_reward_kind;

/* Action normalisation predicate (trading_env.py:58 vs agent/pg/pg.py:52). */
typedef enum pmenv_norm_mode {
    PMENV_NORM_AND = 0, /* reference env: normalise iff !isclose(sum,1) AND min<0; exp(w)/sum(exp(w)) */
    PMENV_NORM_OR = 1   /* batched trainer: normalise iff !isclose(sum,1) OR min<0; softmax */
} pmenv_norm_mode;

/* Weight-history channel order once the ring has wrapped (weight_buffer.py:38-44). */
typedef enum pmenv_ring_mode {
    PMENV_RING_STORAGE = 0, /* reference: ring returned in storage order after wrap */
    PMENV_RING_CHRONO = 1   /* intended: oldest..newest always */
} pmenv_ring_mode;

/* Which value the return uses (trading_env.py:75,88). The reference has two answers:
 * step() takes log(value / (mu * V_prev)) (trading_env.py:75,88,99 — the commission is
 * excluded) and records that ratio as info["returns"] (:90), while env/reward.py:20-31
 * forms returns / log_returns / sharpe_ratio from info["values"], i.e. V_t / V_{t-1}
 * (trading_env.py:80 — commission included). GROSS, the default, is step()'s answer for
 * every reward kind, so info["returns"] and every reward match trading_env.py whatever
 * the commission. NET and AUTO are opt-in; with commission 0 all three agree. */
typedef enum pmenv_ret_mode {
    PMENV_RET_GROSS = 0, /* ret = value / (mu * V_prev): excludes commission (trading_env.py:88) — default */
    PMENV_RET_NET = 1,   /* ret = value / V_prev: includes commission (reward.py:20-31 over info["values"]) */
    PMENV_RET_AUTO = 2   /* opt-in: GROSS for PMENV_REWARD_LOG_RETURN (step()'s hard-coded reward,
                            trading_env.py:99), NET for the kinds only reward.py defines (returns,
                            sharpe_ratio) and for diff_sharpe (resolved at create) */
} pmenv_ret_mode;

typedef struct pmenv_cfg {
    int32_t num_envs;       /* B */
    int32_t num_assets;     /* N  (config/base.py:29 NUM_ASSETS) — asset 0 is cash */
    int32_t window;         /* W  (config/base.py:28 WINDOW_SIZE) */
    int32_t features;       /* F  (last channel F-1 carries the weight history, trading_env.py:103) */
    int32_t close_channel;  /* channel of the close price in obs / bar (price relatives) */
    int32_t reward_kind;    /* pmenv_reward_kind */
    int32_t norm_mode;      /* pmenv_norm_mode */
    int32_t ring_mode;      /* pmenv_ring_mode */
    int32_t ret_mode;       /* pmenv_ret_mode, default GROSS (AUTO is resolved at create; pmenv_get_cfg returns the result) */
    int32_t mu_max_iter;    /* cap on the commission fixed point (trading_env.py:70 has none) */
    double init_cash;       /* config/base.py:47 INITIAL_CASH = 25000 */
    double commission;      /* config/base.py:48 COMISSION = 0.0 */
    double reward_scale;    /* config/base.py:52 REWARD_SCALE = 1 */
    double risk_free_rate;  /* config/base.py:53 RISK_FREE_RATE = 0.04 (sharpe_ratio only) */
    double sharpe_eta;      /* EMA rate of the differential Sharpe reward */
    double mu_tol;          /* fixed-point tolerance, trading_env.py:70 uses 1e-10 */
} pmenv_cfg;

/* Fills cfg with the reference defaults for the given shapes
 * (close_channel = 3 for [open, high, low, close, weight] when F >= 5, else 0). */
void pmenv_cfg_default(pmenv_cfg* cfg, int32_t num_envs, int32_t num_assets,
                       int32_t window, int32_t features);

int32_t pmenv_abi_version(void);

/* Allocates per-env state on `device` (value f64, update counter, W x N weight
 * ring, reward-statistic pair) and puts every env in the reset state.
 * Replaces TradingEnv.__init__ (trading_env.py:8-18) + ActionBuffer.__init__ (weight_buffer.py:6-11). */
int pmenv_create(const pmenv_cfg* cfg, int device, pmenv** out);
/* Same, with the state living in caller-provided device memory of at least
 * pmenv_state_bytes_for(cfg) bytes, 16-B aligned (e.g. a torch uint8 tensor, so
 * the host wrapper gets zero-copy views); the handle never frees it. */
size_t pmenv_state_bytes_for(const pmenv_cfg* cfg);
int pmenv_create_in(const pmenv_cfg* cfg, int device, void* state, size_t state_bytes, pmenv** out);
/* Byte offsets of the state fields inside the state blob:
 * [0] value f64[B], [1] stat_a f64[B], [2] stat_b f64[B], [3] counter i32[B],
 * [4] ring f32[B,W,N], [5] nonfinite u64, [6] last_close f32[B,N] (the close of
 * the window's last day, i.e. obs[b, n, W-1, close_channel], kept by reset/step
 * so the advance path never re-reads the window to form price relatives),
 * [7] w_new f32[B,N] (post-drift weights of the latest step = the ring slot just
 * written, stored densely for the streaming kernel). */
#define PMENV_STATE_FIELDS 8
int pmenv_state_layout(const pmenv_cfg* cfg, size_t offsets[PMENV_STATE_FIELDS]);
int pmenv_destroy(pmenv* h);
const char* pmenv_last_error(const pmenv* h);
int pmenv_get_cfg(const pmenv* h, pmenv_cfg* out);

/* TradingEnv.reset (trading_env.py:21-41): value <- init_cash, ring <- e0, and
 * obs[:, :, :, F-1] <- get_all() (weight_buffer.py:32-44) in place.
 * mask [B] (uint8, device) selects which envs reset; NULL resets all.
 * obs may be NULL (state-only reset). */
int pmenv_reset(pmenv* h, float* obs, const uint8_t* mask, hipStream_t stream);

/* Optional per-step outputs (the reference's info dict, trading_env.py:80,85,90,100). */
typedef struct pmenv_step_args {
    const float* action;   /* [B, N]  target weights (raw policy output)            */
    const float* prices;   /* [B, N]  price relatives y_t, or NULL (needs bar)       */
    const float* bar;      /* [B, N, F-1] new day's market channels, or NULL; with `day`
                              set: a market series [series_days, N, F-1] shared by all envs */
    const int32_t* day;    /* NULL, or [B] device day index: env b's bar is bar[day[b]]
                              (resident-series data path; a day outside
                              [0, series_days) reads NaN and is counted non-finite)   */
    int32_t series_days;
    float* obs;            /* [B, N, W, F] in/out                                     */
    float* obs_out;        /* advance mode only: NULL = advance obs in place; else the
                              advanced window is written here and obs is left untouched
                              (double-buffered windows; must not overlap obs)           */
    float* reward;         /* [B] out, may be NULL                                    */
    double* ret;           /* [B] out (info["returns"]), may be NULL                  */
    float* weights;        /* [B, N] out post-drift weights (info["actions"]), may be NULL */
    uint32_t phases;       /* 0 = whole step; PMENV_PHASE_SCALAR / PMENV_PHASE_ADVANCE run
                              one launch of the two-launch advance path (the advance
                              phase must follow the scalar phase of the same step;
                              used to time the streaming kernel on its own). Where the
                              step is one launch (step_flat_kernel, step_env_kernel,
                              step_relay_kernel, the per-env surface step) the scalar
                              phase runs all of it, the advance phase nothing; the
                              surface step past the Infinity Cache is two launches (the
                              scalar step, then surface_stream_kernel rewriting channel
                              F-1), so its scalar phase alone leaves that channel stale */
} pmenv_step_args;

#define PMENV_PHASE_SCALAR 1u
#define PMENV_PHASE_ADVANCE 2u

/* TradingEnv.step (trading_env.py:44-105) for all B envs in one kernel.
 *  - bar == NULL  ("surface" mode, the reference's own contract): obs is the
 *    caller's next-day window; only channel F-1 is rewritten from the ring.
 *    prices must be given.
 *  - bar != NULL  ("advance" mode, the north-star fused path): obs is the
 *    env-owned window returned by the previous reset/step; it is advanced one
 *    day in place (instrument.py:339-356 sliding window), the bar is appended
 *    at t = W-1, and if prices == NULL the relatives are
 *    bar[close] / obs[W-1, close] (instrument.py:79), with obs[W-1, close]
 *    taken from the env's last_close state (equal to it by construction).
 *    The window's channel F-1 is the ring itself here: the step shifts it with
 *    the window (or, storage order with the ring full, rewrites only the slot),
 *    so an edit the caller makes to that channel persists, where surface mode
 *    rewrites the whole channel from the ring; market-channel edits are honoured
 *    in both modes (announce in-place edits with pmenv_window_written).
 * Portfolio value (f64, env-owned) is readable through pmenv_value(). */
int pmenv_step_ex(pmenv* h, const pmenv_step_args* args, hipStream_t stream);
int pmenv_step(pmenv* h, const float* action, const float* prices, const float* bar,
               float* obs, float* reward, hipStream_t stream);

/* TradingEnv.step / reset with HOST buffers — the call shape of the reference's own driver,
 * which hands the env the data loader's CPU tensors (train/on_policy.py:59-67, :81-89;
 * trading_env.py:21-41, :44-105). Surface contract only: action [B, N], prices [B, N] and
 * the caller's window obs [B, N, W, F] are host memory (pageable is fine); channel F-1 of
 * obs is rewritten in place, exactly as trading_env.py:32 / :103 do. Outputs, each
 * optional (NULL): reward [B] f32, value [B] f64 (TradingEnv.value after the call), ret [B]
 * f64 (info["returns"]), weights [B, N] f32 (info["actions"]).
 * The step kernel reads the action, the prices and the window's last closes (N floats per
 * env) straight from pinned, device-mapped staging, and writes the [N, W] weight channel
 * and the outputs back into it; the market channels never cross PCIe. SYNCHRONOUS: the
 * outputs are in place when the call returns (so not graph-capturable: PMENV_ERR_ARG under
 * capture). Up to 8 envs, and when this handle has enqueued no device work since its last
 * host-buffer call, pmenv_step_host runs in one resident workgroup that polls the staging (no
 * launch per call; it exits after 20 ms without a call or at pmenv_destroy); otherwise it is
 * one launch on `stream`, ordered after the handle's earlier work there. Other kernels that
 * read or write this handle's state must be complete before a host-buffer call. The staging is
 * allocated on the first call. The host side (the last closes gathered, the channel scattered
 * into obs) is serial on the calling thread: B*N*W strided stores per call. */
int pmenv_step_host(pmenv* h, const float* action, const float* prices, float* obs, float* reward, double* value,
                    double* ret, float* weights, hipStream_t stream);
int pmenv_reset_host(pmenv* h, float* obs, double* value, hipStream_t stream);

/* Which kernels the advance path launches for this handle's shape (diagnostics):
 * "<obs_out path> (obs_out) | <in-place path> (in place)", each either
 * "step_flat_kernel" (the whole step in one launch over 16 KiB window tiles),
 * "step_flat_vec_kernel" (the same for 64 < N <= 512),
 * "step_env_kernel" (the whole step in one launch, one workgroup per env) or
 * "<scalar step>+<window stream>"
 * (two launches; for F != 5 the stream is advance_gen_kernel); or, for F != 5 or windows that
 * are not 16-B granular, "step_tiny_kernel" (one workgroup per env, the window staged in LDS:
 * env windows of at most 2,048 floats, N <= 64), "step_small_kernel" (one workgroup per env,
 * the window in registers: env windows of at most 16,384 floats) or "step_advance_lds_kernel" (the LDS-tiled
 * fallback, any F). */
const char* pmenv_step_path(const pmenv* h);

/* Advance-mode step implementation. AUTO (the default) picks per shape and window
 * mode; ONE_LAUNCH forces step_env_kernel (one workgroup per env: F = 5, W >= 2,
 * N <= 64, the env window within 64 KiB of LDS); TWO_LAUNCH forces the scalar-step
 * kernel followed by the window stream (F = 5, 16-B granular env windows; or the generic
 * stream advance_gen_kernel for 2 <= F <= 16, F != 5, 16-B granular env windows with
 * W F >= 17, which AUTO also takes for such windows above 2 MiB in both modes, 16 MiB
 * where the env window is at most 2,048 floats with N <= 64); FLAT forces
 * step_flat_kernel (the whole step in one launch over fixed 16 KiB tiles of the window:
 * F = 5, W >= 2, env windows of >= 148 16-B chunks, N <= 64 — or, as step_flat_vec_kernel,
 * 64 < N <= 512 with W >= 14). Returns PMENV_ERR_ARG
 * (handle unchanged) when the shape does not fit the requested path. For N <= 64 every
 * path gives the same bits; the N > 64 scalar-step forms reduce in another order.
 *
 * FLAT keeps a per-step snapshot of the state its scalar step reads and, in place, the
 * halo of its tiles, both produced by the previous step: a caller that writes the state
 * blob (pmenv_create_in, e.g. the value) or an in-place window outside this API — or that
 * hands in a different window at the address of the last one — must say so before the
 * next step: pmenv_state_written / pmenv_window_written (pmenv_set_state and pmenv_reset
 * do it themselves; so does every other step path). The reference keeps no copy of the
 * caller's features (trading_env.py:102-105), so every such edit is honoured.
 * From the first FLAT step, reset or invalidation enqueued while `stream` is being captured
 * into a hipGraph on, the handle sequences its FLAT steps on the device (a small
 * flat_seq_kernel before each step_flat_kernel reads the parity and the snapshot's
 * validity from device memory, so graph replays and eager calls interleave freely;
 * pmenv_step_path then says "device-sequenced").
 *
 * RELAY forces step_relay_kernel: the two-launch path's scalar step and window stream in
 * ONE launch — scalar workgroups (one run per env) relay w' and the counter to the stream
 * tiles through epoch-tagged words in handle memory (F = 5, W >= 2, 16-B granular env
 * windows, N <= 512; the same bits as TWO_LAUNCH). In place it keeps the tiles' halo from
 * the previous step, under the same pmenv_window_written rule as FLAT. From the first call of
 * a handle enqueued while a stream is being captured into a hipGraph on, its relay steps are
 * device-sequenced (a small relay_prime_kernel before each step_relay_kernel reads the epoch,
 * the parity and the copies' validity from device memory), so captured and eager relay steps
 * interleave freely; pmenv_step_path then says "relay steps device-sequenced".
 * No dispatch-order assumption: a tile polls its rows' relay words a bounded number of times
 * and, if one is still missing (its scalar block not yet dispatched), defers — it stores
 * nothing, lists itself for the step and exits; the scalar blocks run the listed tiles once
 * their words have arrived (one run per tile, under a claim word). In blockIdx dispatch order
 * no tile defers; with every tile dispatched before every scalar block the step completes with
 * the same bits. (pmenv_gae_ex's look-back pass likewise: a wave that waits too
 * long computes the map itself.) */
typedef enum pmenv_step_path_kind {
    PMENV_STEP_PATH_AUTO = 0,
    PMENV_STEP_PATH_ONE_LAUNCH = 1,
    PMENV_STEP_PATH_TWO_LAUNCH = 2,
    PMENV_STEP_PATH_FLAT = 3,
    PMENV_STEP_PATH_RELAY = 4
} pmenv_step_path_kind;
int pmenv_set_step_path(pmenv* h, int32_t path);

/* The caller wrote the in-place window `obs` between steps (features it owns and may
 * edit, trading_env.py:102-105), or hands in a new window at a previous one's address:
 * the next FLAT step re-reads the tile halo from the window (enqueued on `stream`; a
 * no-op for the other step paths, which keep nothing of the window). */
int pmenv_window_written(pmenv* h, const float* obs, hipStream_t stream);
/* The caller wrote the state blob (pmenv_value, pmenv_counter, pmenv_ring or any field of
 * pmenv_state_layout) outside pmenv_set_state: the next FLAT step re-primes its snapshot
 * from the state (and its halo from the window). */
int pmenv_state_written(pmenv* h, hipStream_t stream);

/* Device pointer to the env-owned portfolio values [B] f64 (TradingEnv.value). */
double* pmenv_value(pmenv* h);
/* Device pointer to the weight ring [B, W, N] f32 (ActionBuffer.buffer) and
 * update counters [B] i32 (ActionBuffer.idx = (1 + k) % W, is_full = k >= W-1). */
float* pmenv_ring(pmenv* h);
int32_t* pmenv_counter(pmenv* h);

/* Checkpoint: the whole env state as one opaque device blob. */
size_t pmenv_state_bytes(const pmenv* h);
int pmenv_get_state(pmenv* h, void* dst_device, hipStream_t stream);
int pmenv_set_state(pmenv* h, const void* src_device, hipStream_t stream);

/* Count of envs whose reward or value came out non-finite since create
 * (synchronises `stream`). */
int pmenv_nonfinite_count(pmenv* h, uint64_t* out, hipStream_t stream);

/* ---- synthetic data path (Philox4x32-10, key = seed) ---- */

/* OHLC random walk: series [T, B, Fm=4 ... ] written as [T][B][N][4] =
 * [open, high, low, close]; env ids are env_offset .. env_offset+B-1 so a
 * sharded run generates exactly the slice of the unsharded series. */
int pmenv_synth_series(float* series, int32_t T, int32_t B, int32_t N,
                       int64_t env_offset, uint64_t seed, float sigma, hipStream_t stream);
/* Softmax-of-N(0,1) simplex actions [T][B][N]. */
int pmenv_synth_actions(float* actions, int32_t T, int32_t B, int32_t N,
                        int64_t env_offset, uint64_t seed, hipStream_t stream);
/* obs[b, n, t, f] = series[t, b, n, f] for t < W, f < 4; channel F-1 left for reset. F must be 5. */
int pmenv_window_init(float* obs, const float* series, int32_t B, int32_t N,
                      int32_t W, int32_t F, hipStream_t stream);
/* Resident market series (data/instrument.py:339-356 windows over one shared series):
 * obs[b, n, t, f] = series[start[b] + t, n, f] for t < W, f < F-1 (channel F-1 = 0,
 * written by reset). series [T, N, F-1]; start [B] device int32 with
 * 0 <= start[b] <= T - W (envs outside get NaN windows). */
int pmenv_window_init_days(float* obs, const float* series, int32_t T, int32_t N, int32_t F,
                           const int32_t* start, int32_t B, int32_t W, hipStream_t stream);

/* ---- rollout returns (north star: replay/rollout_buffer.py's GAE / discounted
 * return pass as a device scan; the reference stores (s,a,v,r) but computes no
 * returns, rollout_buffer.py:43-57) ---- */

/* adv[t,b] = delta_t + gamma*lambda*(1-done[t,b])*adv[t+1,b],
 * delta_t = r[t,b] + gamma*(1-done[t,b])*v[t+1,b] - v[t,b];  ret = adv + v.
 * rewards/dones [T,B], values [T+1,B]; dones may be NULL. */
int pmenv_gae(const float* rewards, const float* values, const uint8_t* dones,
              float* adv, float* ret, int32_t T, int32_t B, float gamma, float lam,
              hipStream_t stream);
/* The same pass with caller-owned device scratch of pmenv_gae_workspace(T, B) bytes
 * (0 when the shape does not use it): rollouts with few envs (B < 8192) and long
 * horizons (T >= 512) also split the horizon across workgroups in ONE launch — each
 * chunk publishes its affine map and an epoch-tagged flag in `work`, then composes the
 * later chunks' maps (replaces round 3's two launches). `work` must be 8-B aligned; it
 * may be reused by later calls (each call tags its flags with a fresh epoch) but not
 * shared by two calls in flight. work == NULL, too small or misaligned: as pmenv_gae. */
size_t pmenv_gae_workspace(int32_t T, int32_t B);
int pmenv_gae_ex(const float* rewards, const float* values, const uint8_t* dones,
                 float* adv, float* ret, int32_t T, int32_t B, float gamma, float lam,
                 double* work, size_t work_bytes, hipStream_t stream);

/* Per-rank advantage moments {count, sum, sum of squares} in f64 into out[3]
 * (the only cross-GPU exchange: a 24-byte all-reduce over xGMI). `work` is
 * caller-owned device scratch of pmenv_moments_workspace() bytes (per-block
 * partials; two calls in flight need two workspaces). Deterministic. */
size_t pmenv_moments_workspace(void);
int pmenv_moments(const float* x, int64_t n, double* out, double* work, hipStream_t stream);

/* ---- trainer-side twin: the differentiable batched portfolio reward of the
 * PG / A2C agents (agent/pg/pg.py:40-82 `_reward`, agent/a2c.py/a2c.py:40-82 `_loss`
 * = -_reward), forward and backward in f64 over a [B, N] batch. ---- */
typedef enum pmenv_batch_norm {
    PMENV_BNORM_GLOBAL_OR = 0, /* reference: softmax over assets iff !isclose(sum over the WHOLE batch, 1)
                                  OR min < 0 (pg.py:52) */
    PMENV_BNORM_ROW_OR = 1,    /* the same decision per row */
    PMENV_BNORM_NONE = 2
} pmenv_batch_norm;

/* f64 scratch the forward fills and the backward reads: (6*B + 8 + 16*ceil(B/16)) * 8 bytes. */
size_t pmenv_batch_reward_workspace(int32_t B);
/* a, p [B, N]; v_prev [B] (the _v of pg.py); reward_kind LOG_RETURN / RETURN / SHARPE
 * (batch mean / std, pg.py:80); writes reward_out[0] (device) and optionally the
 * per-row gross returns ret_out [B]. */
int pmenv_batch_reward_forward(const float* a, const float* v_prev, const float* p, int32_t B, int32_t N,
                               int32_t reward_kind, int32_t norm, double scale, double* work,
                               float* reward_out, float* ret_out, hipStream_t stream);
/* grad_a [B, N] = grad_out[0] * dR/da (grad_out is a device scalar). */
int pmenv_batch_reward_backward(const float* a, const float* v_prev, const float* p, int32_t B, int32_t N,
                                int32_t reward_kind, double scale, const double* work,
                                const float* grad_out, float* grad_a, hipStream_t stream);

/* ---- device replay and trajectory metrics ---- */

/* replay/buffer.py:39-79 ReplayBuffer.sample for vectorised envs over a ring of H
 * recorded steps (days [H, B] int32 = last day of the window acted on, actions
 * [H, B, N], rewards [H, B]): for each of the S samples (h0[j], env[j]) writes
 * s, s_next [S, N, W, F] (market channels from series [T, N, F-1], channel F-1 = the
 * W actions h0..h0+W-1, resp. h0+1..h0+W), a_out [S, N] = actions[h0+W],
 * r_out [S] = rewards[h0+W-1]. Days outside the series read NaN. */
int pmenv_replay_gather(const float* series, int32_t T, int32_t N, int32_t F, int32_t W,
                        const int32_t* days, const float* actions, const float* rewards,
                        int32_t H, int32_t B, const int32_t* h0, const int32_t* env, int32_t S,
                        float* s, float* s_next, float* a_out, float* r_out, hipStream_t stream);

/* The compact on-policy rollout (replay/rollout_buffer.py:43-57 stores s per step;
 * here the windows are re-materialised instead): for each of the S
 * samples (t_idx[j], env[j]) writes s[j] = env b's window after t updates, [N, W, F]:
 * market channels from series [T, N, F-1] at days start[b] + t .. start[b] + t + W - 1
 * (start [B] = first day of the reset window; days outside read NaN), channel F-1 =
 * ActionBuffer.get_all() rebuilt from the post-drift weights [T_rec, B, N] of updates
 * 1 .. T_rec (weight_buffer.py:32-44; ring_mode = pmenv_ring_mode). t_idx <= T_rec. */
int pmenv_rollout_gather(const float* series, int32_t T, int32_t N, int32_t F, int32_t W, const int32_t* start,
                         const float* weights, int32_t T_rec, int32_t B, int32_t ring_mode,
                         const int32_t* t_idx, const int32_t* env, int32_t S, float* s, hipStream_t stream);

/* util/eval.py:14-37 per env over a trajectory: returns [T, B] (simple returns),
 * values [T+1, B] f64, weights [T+1, B, N]; out [B, 5] f64 =
 * {sharpe, sortino, max drawdown, average turnover, final value} from f64 simple
 * returns [T, B], values [T+1, B] f64 and weights [T+1, B, N] f32, quantstats
 * definitions with per-period risk-free (1+rf)^(1/periods)-1 (parity unpinned:
 * quantstats is absent). */
int pmenv_metrics(const double* returns, const double* values, const float* weights, int32_t T, int32_t B,
                  int32_t N, double risk_free_rate, double periods, double* out, hipStream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* PMENV_H */
