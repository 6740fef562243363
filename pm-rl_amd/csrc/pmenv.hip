// pmenv.hip — host side and C ABI (include/pmenv.h) of the MI355X-native vectorised
// portfolio environment: the product library, libpmenv.so. Device code lives in
// step_flat.h (the one-launch step over fixed window tiles), step_env.h (the one-launch
// step, one workgroup per env), env_step.h (scalar step, window streams, reset,
// fallbacks), scalar_vec.h (packed scalar step), data.h (synthetic market data),
// rollout.h (GAE, moments), replay.h (replay gather, metrics) and trainer.h (batched
// reward); the step's launchers in launch.h, the handle and its shape planning in handle.h.
//
// Every entry point enqueues on the caller's stream and never synchronises, allocates or
// frees (graph-capturable), except create / destroy / the explicit synchronous queries
// documented in the header. Kernel choice is a function of the shape and of
// pmenv_set_step_path only: this library reads no environment variable. The A/B
// alternatives measured while choosing live in the tools build (tools/ab/pmenv_ab.hip,
// linked with this file into tools/libpmenv_ab.so), behind the pmenv_tools hooks whose
// definitions here, at the end of the file, do nothing.
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>

#include "../../include/pmenv.h"
#include "data.h"
#include "handle.h"
#include "launch.h"
#include "replay.h"
#include "rollout.h"
#include "trainer.h"

using namespace pmenv_dev;
using namespace pmenv_host;

namespace {

thread_local char g_create_err[512] = "";

// K1 shape per asset count: N <= 64 keeps one asset per lane, with reductions bitwise
// those of the one-launch steps' scalar part (so the paths, and sharded and unsharded
// runs whose path can differ by env count, give the same bits): N <= 16 the packed form
// with 8 / 16 lanes per env (8 / 4 envs per wave instead of 2; its butterfly pairs the
// lanes as the row shifts do, every pair sum commutes bitwise, and the all-zero padding
// lanes of the register form only add +0.0, which the packed form's 0.0 + x seed
// reproduces), 16 < N <= 64 the register form; 64 < N <= 512 the packed strided form
// (64 lanes x A assets, every dword load a coalesced run; step_flat_vec_kernel shares
// it); N > 512 the LDS form.
int pick_k1_vec(const pmenv_cfg& c) {
    const int N = c.num_assets;
    if ((int64_t)c.num_envs * N * 4 >= (1ll << 32)) return 0;     // descriptors span the [B*N] arrays
    if (N <= 8) return kK1Str + 801;
    if (N <= 16) return kK1Str + 1601;
    if (N <= 64) return 0;
    if (N <= 128) return kK1Str + 6402;
    if (N <= 256) return kK1Str + 6404;
    if (N <= 512) return kK1Str + 6408;
    return 0;
}

// the stream is being captured into a hipGraph: step_flat_kernel's host-chosen parity
// would be frozen under replay, so the handle switches to the device-sequenced form
bool capturing(hipStream_t stream) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &st) != hipSuccess) {
        (void)hipGetLastError();
        return true;
    }
    return st != hipStreamCaptureStatusNone;
}

// Anything but step_flat_kernel that writes the state or a window leaves the snapshot and
// the halo stale (`what` = the device words to clear: V, the snapshot-valid word, or HOBS,
// the window the halo belongs to). The host flags cover eager steps; device-sequenced
// handles also clear the device word on the stream. An invalidation enqueued while the
// stream is being captured switches the handle to the device-sequenced form first: a
// graph of [reset, flat steps] replays the reset's clear before every replay's steps,
// where host flags set once at capture time would let replay 2 on read the snapshot the
// previous replay left (flat_seq_kernel then re-primes from the reset state).
enum { kInvalSnap = 1, kInvalHalo = 2 };
// Once any call of this handle is enqueued while `stream` is being captured into a hipGraph,
// replays may write the window or the state where the host does not see it: from then on the
// flat and the relay steps keep the validity of their copies (snapshot, counter copy, halo) in
// device words that every invalidation clears on the stream — whatever path is current when the
// capture is seen, since a later switch of path must not find host flags a replay outdated.
void note_capture(pmenv* h, hipStream_t stream) {
    if (((h->flat1_ok && !h->device_seq) || (h->relay_ok && !h->relay_dseq)) && capturing(stream)) {
        if (h->flat1_ok) h->device_seq = true;
        if (h->relay_ok) h->relay_dseq = true;
    }
}

// the relay step's copies go stale (kInvalSnap: the counter copy and the halo; kInvalHalo: the halo)
int relay_invalidate(pmenv* h, hipStream_t stream, int what) {
    h->relay_obs = nullptr;
    if (what & kInvalSnap) h->relay_kp_ok = false;
    if (!h->relay_dseq || !h->relay_mem) return PMENV_OK;
    // V = 0 re-primes both, HOBS = 0 the halo
    const hipError_t e = (what & kInvalSnap) ? hipMemsetAsync(h->relay_seq + 2, 0, 4, stream)
                                             : hipMemsetAsync(h->relay_seq + 6, 0, 8, stream);
    if (e != hipSuccess) {
        set_err(h, "invalidating the relay step's copies: %s", hipGetErrorString(e));
        return PMENV_ERR_HIP;
    }
    return PMENV_OK;
}

int flat1_invalidate(pmenv* h, hipStream_t stream, int what = kInvalSnap | kInvalHalo, bool host_only = false,
                     bool keep_relay = false) {
    if (what & kInvalSnap) h->snap_ok = false;
    h->halo1_obs = nullptr;
    if (!host_only) note_capture(h, stream);
    if (!keep_relay) {
        if (host_only) {
            h->relay_obs = nullptr;
            if (what & kInvalSnap) h->relay_kp_ok = false;
        } else if (const int rc = relay_invalidate(h, stream, what)) {
            return rc;
        }
    }
    if (host_only || !h->device_seq) return PMENV_OK;
    // V = 0 clears both (a stale V re-primes the halo too); HOBS = 0 only the halo
    const hipError_t e = (what & kInvalSnap) ? hipMemsetAsync(h->seq + 2, 0, 4, stream)
                                             : hipMemsetAsync(h->seq + 4, 0, 8, stream);
    if (e != hipSuccess) {
        set_err(h, "invalidating the flat step's snapshot: %s", hipGetErrorString(e));
        return PMENV_ERR_HIP;
    }
    return PMENV_OK;
}

// The relay step's memory (zeroed: the device-sequenced words, no relay word, deferral list or tile
// claim of any epoch), allocated when AUTO gives the shape the relay step or pmenv_set_step_path asks
// for it — not on a step. The deferral list and claims (step_relay.h) follow the relay words, so
// one memset clears all three when the eager epoch wraps.
int relay_alloc(pmenv* h) {
    if (h->relay_mem || !h->relay_ok) return PMENV_OK;
    const pmenv_cfg& c = h->cfg;
    const uint64_t B = (uint64_t)c.num_envs, BN = B * (uint64_t)c.num_assets;
    auto up16 = [](size_t x) { return (x + 15) / 16 * 16; };
    const size_t ctl_b = 64, words_b = up16(BN * 8) + relay_list_bytes(h), kp_b = up16(B * 4);
    const size_t hal = up16((size_t)h->relay_tiles * 32);
    const size_t bytes = ctl_b + words_b + 2 * kp_b + 2 * hal;
    DeviceGuard g(h->device);
    void* m = nullptr;
    hipError_t ae = hipMalloc(&m, bytes);
    if (ae != hipSuccess) {
        set_err(h, "hipMalloc(relay) failed: %s", hipGetErrorString(ae));
        return PMENV_ERR_HIP;
    }
    ae = hipMemset(m, 0, ctl_b + words_b);
    if (ae != hipSuccess) {
        (void)hipFree(m);
        set_err(h, "relay words: %s", hipGetErrorString(ae));
        return PMENV_ERR_HIP;
    }
    char* b = (char*)m;
    h->relay_mem = m;
    h->relay_seq = (uint32_t*)b;
    h->relay_w = (uint64_t*)(b + ctl_b);
    h->relay_list = (uint64_t*)(b + ctl_b + up16(BN * 8));
    h->relay_done = (uint32_t*)(b + ctl_b + up16(BN * 8) + up16(((size_t)h->relay_tiles + 1) * 8));
    h->relay_kp = (int32_t*)(b + ctl_b + words_b);
    h->relay_halo = (float*)(b + ctl_b + words_b + 2 * kp_b);
    h->relay_halo_stride = (uint32_t)(hal / 4);
    h->relay_obs = nullptr;
    h->relay_kp_ok = false;
    h->relay_par = 0;
    h->relay_epoch = 0;
    return PMENV_OK;
}

// which windows take the one-launch steps under `path`
int one_bits(const pmenv* h, int path) {
    if (path == PMENV_STEP_PATH_ONE_LAUNCH) return h->one_ok ? (PMENV_FUSE_DB | PMENV_FUSE_INPLACE) : -1;
    if (path == PMENV_STEP_PATH_TWO_LAUNCH) return h->streaming || h->gen_ok ? 0 : -1;
    if (path == PMENV_STEP_PATH_FLAT) return h->flat1_ok ? 0 : -1;
    if (path == PMENV_STEP_PATH_RELAY) return h->relay_ok ? 0 : -1;
    return h->one_auto;
}
int relay_bits(const pmenv* h, int path) {
    if (path == PMENV_STEP_PATH_RELAY) return h->relay_ok ? (PMENV_FUSE_DB | PMENV_FUSE_INPLACE) : -1;
    if (path == PMENV_STEP_PATH_AUTO) return h->relay_auto;
    return 0;
}
int gen_bits(const pmenv* h, int path) {
    if (path == PMENV_STEP_PATH_TWO_LAUNCH) return h->gen_ok ? (PMENV_FUSE_DB | PMENV_FUSE_INPLACE) : 0;
    if (path == PMENV_STEP_PATH_AUTO) return h->gen_auto;
    return 0;
}
int flat1_bits(const pmenv* h, int path) {
    if (path == PMENV_STEP_PATH_FLAT) return h->flat1_ok ? (PMENV_FUSE_DB | PMENV_FUSE_INPLACE) : -1;
    if (path == PMENV_STEP_PATH_AUTO) return h->flat1_auto;
    return 0;
}

}  // namespace

extern "C" {

int32_t pmenv_abi_version(void) { return PMENV_ABI_VERSION; }

void pmenv_cfg_default(pmenv_cfg* cfg, int32_t num_envs, int32_t num_assets, int32_t window, int32_t features) {
    if (!cfg) return;
    memset(cfg, 0, sizeof(*cfg));
    cfg->num_envs = num_envs;
    cfg->num_assets = num_assets;
    cfg->window = window;
    cfg->features = features;
    cfg->close_channel = features >= 5 ? 3 : 0;
    cfg->reward_kind = PMENV_REWARD_LOG_RETURN;
    cfg->norm_mode = PMENV_NORM_AND;
    cfg->ring_mode = PMENV_RING_STORAGE;
    cfg->ret_mode = PMENV_RET_GROSS;
    cfg->mu_max_iter = 100;
    cfg->init_cash = 25000.0;
    cfg->commission = 0.0;
    cfg->reward_scale = 1.0;
    cfg->risk_free_rate = 0.04;
    cfg->sharpe_eta = 0.01;
    cfg->mu_tol = 1e-10;
}

const char* pmenv_last_error(const pmenv* h) { return h ? h->err : g_create_err; }

int pmenv_get_cfg(const pmenv* h, pmenv_cfg* out) {
    if (!h || !out) return PMENV_ERR_ARG;
    *out = h->cfg;
    return PMENV_OK;
}

int pmenv_state_layout(const pmenv_cfg* cfg, size_t off[PMENV_STATE_FIELDS]) {
    if (!cfg || !off || cfg->num_envs < 1 || cfg->num_assets < 1 || cfg->window < 1) return PMENV_ERR_ARG;
    const size_t B = (size_t)cfg->num_envs, N = (size_t)cfg->num_assets;
    const size_t ring_elems = B * (size_t)cfg->window * N;
    auto up16 = [](size_t x) { return (x + 15) / 16 * 16; };
    size_t o = 0;
    off[0] = o; o = up16(o + B * 8);           // value
    off[1] = o; o = up16(o + B * 8);           // stat_a
    off[2] = o; o = up16(o + B * 8);           // stat_b
    off[3] = o; o = up16(o + B * 4);           // counter
    off[4] = o; o = up16(o + ring_elems * 4);  // ring
    off[5] = o; o = up16(o + 8);               // nonfinite
    off[6] = o; o = up16(o + B * N * 4);       // last_close
    off[7] = o;                                // w_new
    return PMENV_OK;
}

size_t pmenv_state_bytes_for(const pmenv_cfg* cfg) {
    size_t off[PMENV_STATE_FIELDS];
    if (pmenv_state_layout(cfg, off) != PMENV_OK) return 0;
    return (off[7] + (size_t)cfg->num_envs * cfg->num_assets * 4 + 15) / 16 * 16;
}

int pmenv_create(const pmenv_cfg* cfg, int device, pmenv** out) {
    return pmenv_create_in(cfg, device, nullptr, 0, out);
}

int pmenv_create_in(const pmenv_cfg* cfg, int device, void* state, size_t state_bytes, pmenv** out) {
    if (!cfg || !out) return PMENV_ERR_ARG;
    *out = nullptr;
    pmenv* h = (pmenv*)calloc(1, sizeof(pmenv));
    if (!h) return PMENV_ERR_ARG;
    h->cfg = *cfg;
    h->device = device;
    const pmenv_cfg& c = h->cfg;
    auto fail = [&](int code) {
        // no handle reaches the caller: pmenv_last_error(NULL) reports this one
        snprintf(g_create_err, sizeof(g_create_err), "%s", h->err);
        pmenv_tools::release(h);
        if (h->state && h->owns_state) (void)hipFree(h->state);
        if (h->halo) (void)hipFree(h->halo);
        if (h->snap) (void)hipFree(h->snap);
        if (h->relay_mem) (void)hipFree(h->relay_mem);
        free(h);
        return code;
    };
    if (c.num_envs < 1 || c.num_assets < 1 || c.window < 1 || c.features < 2) {
        set_err(h, "invalid shape B=%d N=%d W=%d F=%d (need B,N,W >= 1, F >= 2)", c.num_envs, c.num_assets,
                c.window, c.features);
        return fail(PMENV_ERR_ARG);
    }
    if (c.close_channel < 0 || c.close_channel >= c.features - 1) {
        set_err(h, "close_channel %d must be a market channel in [0, F-2]", c.close_channel);
        return fail(PMENV_ERR_ARG);
    }
    if (c.reward_kind < 0 || c.reward_kind > 3 || c.norm_mode < 0 || c.norm_mode > 1 || c.ring_mode < 0 ||
        c.ring_mode > 1 || c.ret_mode < 0 || c.ret_mode > 2 || c.mu_max_iter < 0 || !(c.commission >= 0.0) ||
        !(c.commission < 1.0)) {
        set_err(h, "invalid mode/commission value in cfg");
        return fail(PMENV_ERR_ARG);
    }
    if (h->cfg.ret_mode == PMENV_RET_AUTO)
        h->cfg.ret_mode = c.reward_kind == PMENV_REWARD_LOG_RETURN ? PMENV_RET_GROSS : PMENV_RET_NET;
    const int64_t WF = (int64_t)c.window * c.features;
    if (WF > kTileFloats) {
        set_err(h, "window*features = %lld exceeds the %d-float LDS tile", (long long)WF, kTileFloats);
        return fail(PMENV_ERR_ARG);
    }
    if ((int64_t)c.num_assets * WF >= (1ll << 31)) {
        set_err(h, "per-env obs block too large");
        return fail(PMENV_ERR_ARG);
    }
    // LDS fallback tile geometry: whole asset rows, 16-B granular when every env block is
    int R = (int)(kTileFloats / WF);
    if (R > c.num_assets) R = c.num_assets;
    bool vec = ((int64_t)c.num_assets * WF) % 4 == 0;
    if (vec && R < c.num_assets) {
        while (R > 0 && ((int64_t)R * WF) % 4 != 0) --R;
        if (R == 0) { vec = false; R = (int)(kTileFloats / WF); }
    }
    h->rows_per_tile = R;
    h->vec = vec;
    // the register step: the env's window within BLOCK x E floats (one workgroup per env)
    {
        const int64_t nwf = (int64_t)c.num_assets * WF;
        h->small_block = nwf <= 256 * 16 ? 256 : nwf <= 512 * 16 ? 512 : nwf <= 1024 * 16 ? 1024 : 0;
        h->small_e = nwf <= 256 * 8 ? 8 : 16;
        // config 1's 1 x 5 x 50 x 5: 4.1 us (step_small_kernel) -> see DESIGN.md §3
        // (step_tiny_kernel stages the day's bar two floats per thread: N (F - 1) <= 2 x 256)
        h->tiny = h->small_block == 256 && h->small_e == 8 && c.num_assets <= 64 &&
                  (int64_t)c.num_assets * (c.features - 1) <= 2 * 256;
    }
    // surface steps on windows past the Infinity Cache with 16-B granular env blocks: the scalar
    // step, then surface_stream_kernel (65,536 x 30 x 50 x 5 723 us with the ring columns staged
    // in LDS, against 939 on the per-env kernel's dword writes, 892 with its writes in whole
    // chunks; cache-resident windows keep the per-env kernel: 4,096 x 30 38.3 against 48.6 in
    // whole chunks — ab_r05/surface_stream_r05s4_*, surface_ringlds_r05sr.*); the staged
    // columns (rows x W floats) and counters (rows) within 64 KiB
    h->surf_lds = (size_t)(4 * 1024 / WF + 2) * (c.window + 1) * 4;   // + each row's counter
    h->surf_stream = window_bytes(c) > (256ll << 20) && ((int64_t)c.num_assets * WF) % 4 == 0 &&
                     (int64_t)c.num_envs * ((int64_t)c.num_assets * WF / 4) < (1ll << 31) - 1024 &&
                     h->surf_lds <= (64u << 10) && 4 * 1024 / WF + 2 <= 256;   // a thread per row's counter
    h->tile_floats = (int)((((int64_t)R * WF) + 3) / 4 * 4);
    h->lds_tile = scratch_bytes(h->tile_floats, c.num_assets, c.features);
    h->lds_surface = scratch_bytes(0, c.num_assets, c.features);

    // ---- the two-launch stream: row-kernel geometry (fallback) and the flat stream
    static const int kInplaceOrder[3] = {2, 4, 1}, kDoubleOrder[3] = {4, 2, 1};
    h->streaming = plan_streaming(c, kInplaceOrder, kStreamBlock, 0, &h->unit_rows, &h->stream_vec) &&
                   plan_streaming(c, kDoubleOrder, kStreamBlock, 0, &h->unit_rows_db, &h->stream_vec_db);
    const int64_t per = (int64_t)c.num_assets * c.window * c.features;
    const int64_t win = window_bytes(c);
    // Flat 16-B stream (F = 5, W >= 2, 16-B granular envs, chunk count < 2^31) in place
    // (with the halo) and double-buffered: 512 threads x 2 chunks, side data through the
    // scalar unit (6.38 TB/s against 5.37 for whole-row units).
    h->flat_ok = h->streaming && c.features == 5 && c.window >= 2 && per % 4 == 0 &&
                 (int64_t)c.num_envs * (per / 4) < (1ll << 31) - 1024;
    h->flat = h->flat_inplace = h->flat_ok;
    // in place, cache-resident windows (<= 256 MiB) take 8 KiB workgroups: 80.2 vs 83.2 us
    // at 8,192 x 30, 44.4 vs 44.7 at 4,096 (profiles/ab_r02/r02w_smallip_*); above, 16 KiB
    // (round 1: 512 x 2 against 256 x 1 / 2 / 4, 512 x 1, 1024 x 1)
    h->flat_ip_block = win <= (256ll << 20) ? 256 : 512;
    h->flat_ip_vec = 2;
    h->flat_qtot = h->flat_ok ? (uint32_t)((int64_t)c.num_envs * (per / 4)) : 0u;
    // nt unless the stream's working set fits the 256 MiB Infinity Cache: the window in
    // place (<= 256 MiB), the window and its double buffer otherwise (<= 128 MiB each).
    // Step at 4,096 x 30 x 50 x 5 (123 MB) 44.4 us with the default policy against 46.5
    // nt; 8,192 envs (246 MB) in place 84.6 / 86.1 but double-buffered 91.2 / 86.5;
    // 16,384: 199.6 / 164.6 (profiles/ab_r01/pol_small_r01j.log, pol_ip_r01m.log)
    h->flat_pol = win <= (128ll << 20) ? 0 : 1;
    h->flat_ip_pol = win <= (256ll << 20) ? 0 : 1;
    h->k1_vec = pick_k1_vec(c);
    h->per4 = (uint32_t)(per / 4);

    // ---- the one-launch step (step_env_kernel, one workgroup per env): F = 5, W >= 2,
    // N <= 64 (the scalar step on one wave), 16-B granular env windows whose 1 KiB
    // blocks fit 16 waves and 64 KiB of LDS, 4 chunks per lane (650 us against 662-666
    // for 8, 762 for 3, 860 for 2 at the BASELINE shape). AUTO gives it the windows of at
    // most 48 MiB, where launch latency dominates and it wins by 7-38 % (tools/gpu_ab_smallb.sh,
    // profiles/ab_r02/r02u_*: N = 8..64, 256..4,096 envs; N = 30: 64 envs 6.5 vs 9.6 us,
    // 1,024: 13.1 vs 18.2). Larger windows take the two-launch stream: its fixed 16 KiB
    // workgroups run 640-670 us on a 2 GB window at every asset count measured, while the
    // one-workgroup-per-env geometry ties it only at N = 30 (650-658 us) and loses 4-15 %
    // at N = 8, 16, 24, 32, 40, 48, 60, 64 (profiles/ab_r02/r02r_*, r02s_*, r02t_*).
    // (Also beyond the flat stream's 2^31-chunk index, where the two-launch path would
    // fall back to the whole-row stream.)
    plan_one(h, kOneV);
    h->one_auto = h->one_ok && (win <= (48ll << 20) || !h->flat_inplace) ? (PMENV_FUSE_DB | PMENV_FUSE_INPLACE) : 0;

    // ---- the one-launch flat step (step_flat_kernel; step_flat_vec_kernel for 64 < N <=
    // 512): the flat stream's shape rules, the scalar step on one wave per env, at most one
    // env per wave in a tile (flat1_fits). Geometry: 256 threads x 4 chunks (16 KiB tiles,
    // 4 waves) where env windows have >= 511 chunks, 512 x 2 (8 waves) from 148 chunks.
    // 256 x 4 against 512 x 2 / 512 x 4 / 1024 x 2 / 256 x 8 / 256 x 2 / 128 x 8 / 128 x 4 at
    // 65,536 x 30 in place: 629.5 against 714 / 678 / 790 / 695 / 675 / 624 / 641 us; 128 x 8
    // loses 15 % at N = 16 and 64 where 256 x 4 wins (profiles/ab_r02/r02w_flat1b_*,
    // r02w_flat1c_*). A persistent form that keeps the next tile's loads in flight needs
    // 160 VGPRs (3 waves per SIMD): 2x slower.
    // 128 x 8 (2 waves, 8 chunks per lane, the same 16 KiB tiles) where every tile holds at
    // most two envs (1,023 .. 1,999 chunks per env: N = 20 .. 39 at W = 50) and the window
    // streams through HBM: 0.5-1.1 % ahead of 256 x 4 from 49,152 envs at N = 30 (65,536:
    // 625.7 vs 629.4 and 628.8 vs 631.6 us; 98,304: 941.1 vs 951.6), N = 20 / 24 / 28 by
    // 1.0 / 0.7 / 0.5 %; behind it at 16,384 envs (162.9 vs 161.4) and at N = 16 / 64
    // (profiles/ab_r02/r02w_flat1k_*, r02w_flat1l_*, r02w_flat1c_*). Wide envs: 256 x 4.
    const bool band128 = c.num_assets <= 64 && h->per4 >= 1023u && h->per4 < 2000u && win > (1ll << 30);
    if (band128 && flat1_fits(h, 128, 8)) { h->flat1_block = 128; h->flat1_vec = 8; }
    else if (flat1_fits(h, 256, 4)) { h->flat1_block = 256; h->flat1_vec = 4; }
    else { h->flat1_block = 512; h->flat1_vec = 2; }
    h->flat1_ok = flat1_fits(h, h->flat1_block, h->flat1_vec) && (c.num_assets <= 64 || h->flat1_block == 256);
    // AUTO: above the one-launch-per-env windows (48 MiB) the flat step beats the two-launch
    // stream by 1-3.5 % for env windows of >= 1,000 chunks (N >= 16 at W = 50): 65,536 x 30
    // 629.5 / 639.7 against 642.4 / 648.8 us on two boxes, N = 24 / 40 / 48 / 64 by 1-3.4 %,
    // N = 16 681 vs 689; it loses at N = 8 (500 chunks, 4 envs per tile: 713 vs 691) and in
    // place on cache-resident windows (4,096 envs: 46.3 vs 44.2 us, 8,192: 85.2 vs 84.2);
    // double-buffered it wins from 2,048 envs (25.4 vs 27.0) (profiles/ab_r02/r02w_flat1d_*).
    // Commission > 0: every tile an env straddles runs the capped fixed point. With the
    // active-set iteration (scalar_core), a uniform wave index (no waterfall loops around
    // the scalar loads) and the reciprocal of 1 - c w0, the flat step leads there too:
    // 65,536 x 30 at 0.0025 642.8 vs 661.9 us on two launches (profiles/ab_r03/comm3_r03.err;
    // in round 2 the fixed point cost it 6-8 %: 701 vs 662).
    h->flat1_auto = 0;
    if (h->flat1_ok && c.num_assets <= 64 && h->flat1_block <= 256 && h->per4 >= 1000u) {
        if (win > (48ll << 20)) h->flat1_auto |= PMENV_FUSE_DB;
        if (win > (256ll << 20)) h->flat1_auto |= PMENV_FUSE_INPLACE;
        h->one_auto &= ~h->flat1_auto;
    }
    // Wide envs (step_flat_vec_kernel, 64 < N <= 512): every tile an env straddles runs the
    // env's whole packed scalar step, which costs more than the kernel boundary it saves
    // from 4 assets per lane on: 8,192 x 500 in place 1,512 (128 x 8) / 1,605 (256 x 4)
    // against 1,381 us on two launches, 2,048 x 200 143.5 vs 140.0; at 2 assets per lane
    // it wins on HBM-streamed windows: 16,384 x 100 532.9 vs 549.7 us (profiles/ab_r03/
    // wide_r03wide.err). AUTO gives it in-place windows > 1 GiB at N <= 128 without commission.
    if (h->flat1_ok && c.num_assets > 64 && c.num_assets <= 128 && win > (1ll << 30) && !(c.commission > 0.0))
        h->flat1_auto |= PMENV_FUSE_INPLACE;
    // In place, 24-100 MiB: a one-launch step beats the two-launch stream there (round 3,
    // in-process interleaved, profiles/ab_r03/band_r03u.err, band_r03w.err; µs per step,
    // two launches / one WG per env / flat step): N = 30 at 2,048 envs 27.2 / 24.7 / 25.9,
    // 3,072 36.3 / 34.7 / 36.3; N = 16 at 4,096 28.8 / 28.1 / 26.8, 6,144 38.1 / 39.8 / 36.9;
    // N = 8 at 4,096 19.4 / 18.9 / 16.3, 8,192 29.1 / 30.5 / 27.2; N = 32 at 3,072 37.9 /
    // 38.4 / 36.7; N = 64 at 1,024 28.6 / - / 26.8. From ~115 MiB the two-launch stream
    // leads (N = 30 at 4,096 44.8 / 45.7 / 47.2, N = 32 / 16 / 8 at 125 MiB, N = 48 at 188).
    // Which one-launch form: the one-WG-per-env step where its waves' chunk slots hold the
    // env with >= 90 % occupancy (N = 30: 1,875 of 2,048; it wins by 5-8 % there), else
    // the flat step (N = 8 / 16 / 32: 65 / 78 / 87 %, the flat step wins by 4-14 %) — the
    // same rule from 24 MiB, where the flat step also wins at N = 8 and 16 (4,096 x 8:
    // 16.3 vs 18.9 us; 3,072 x 16: 21.6 vs 22.6).
    if (win > (24ll << 20) && win <= (100ll << 20)) {
        const double one_fill = h->one_ok ? (double)h->per4 / (256.0 * h->one_waves) : 0.0;
        if (h->one_ok && one_fill >= 0.9) {
            h->one_auto |= PMENV_FUSE_INPLACE;
        } else if (h->flat1_ok && c.num_assets <= 64) {
            h->flat1_auto |= PMENV_FUSE_INPLACE;
            h->one_auto &= ~PMENV_FUSE_INPLACE;
        } else if (h->one_ok) {
            h->one_auto |= PMENV_FUSE_INPLACE;
        }
    }

    // ---- the relayed one-launch step (step_relay_kernel): the flat stream's shapes (F = 5,
    // W >= 2, 16-B granular env windows) with the two-launch path's scalar step forms
    // (N <= 512, the packed forms' [B*N] descriptors under 2^32 bytes), the stream's tile
    // geometry; at most BLOCK rows per tile (4 * 2 <= W * F).
    {
        const int N = c.num_assets;
        const int kv = h->k1_vec >= kK1Str ? h->k1_vec - kK1Str : h->k1_vec;
        h->relay_block = h->flat_ip_block;
        h->relay_v = 2;
        // a tile stages one row per thread: 4 CPW / (W F) + 2 rows must fit its BLOCK threads
        // (for V = 2: W >= 2; the host schedule emulation under tests/ checks it per tile)
        const bool rows_fit = 4 * h->relay_block * h->relay_v / (c.window * 5) + 2 <= h->relay_block;
        h->relay_ok = h->flat_ok && c.window >= 2 && rows_fit && N <= 512 && (N <= 64 || h->k1_vec != 0);
        h->relay_kl = kv ? kv / 100 : (N <= 32 ? 32 : 64);
        h->relay_ka = kv ? kv % 100 : 0;
        h->relay_auto = 0;
    }
    // AUTO gives the relay step the cache-resident windows where the kernel boundary of two
    // launches, or the scalar step inside every tile, is what a step pays for (N <= 64,
    // round 4, in-process interleaved, profiles/ab_r04/relay_band_r04b.err; us per step,
    // AUTO's previous choice / relay): in place 24-256 MiB — N = 30 at 2,048 / 3,072 / 4,096 /
    // 6,144 / 8,192 envs 24.9 / 23.7, 34.5 / 32.1, 44.3 / 40.6, 62.1 / 58.3, 81.9 / 80.0 (with
    // commission 83.6 / 80.6), N = 8 at 4,096 / 8,192 / 16,384 16.2 / 14.5, 27.7 / 24.3, 46.4 /
    // 42.7, N = 16 at 4,096 / 8,192 27.6 / 24.4, 46.4 / 42.4, N = 64 at 2,048 / 4,096 46.6 /
    // 43.1, 85.9 / 84.3 — except 24-48 MiB where the one-workgroup-per-env step holds the env
    // at >= 90 % (1,024 x 30: 13.5 / 14.9); double-buffered 48-128 MiB (2,048 / 4,096 x 30:
    // 27.2 / 23.2, 49.1 / 41.6; 8,192: 83.2 / 90.6). From 256 MiB in place the flat step leads
    // (12,288 / 16,384 / 65,536 x 30: 119.0 / 120.5, 156.8 / 159.9, 625.5 / 641.7), and at
    // config 5 two launches (1,324.6 / 1,360.3).
    if (h->relay_ok && c.num_assets <= 64) {
        const double one_fill = h->one_ok ? (double)h->per4 / (256.0 * h->one_waves) : 0.0;
        const bool one_holds = h->one_ok && one_fill >= 0.9 && win <= (48ll << 20);
        if (win > (24ll << 20) && win <= (256ll << 20) && !one_holds) h->relay_auto |= PMENV_FUSE_INPLACE;
        if (win > (48ll << 20) && win <= (128ll << 20)) h->relay_auto |= PMENV_FUSE_DB;
        h->one_auto &= ~h->relay_auto;
        h->flat1_auto &= ~h->relay_auto;
        // 256 x 4 tiles (16 KiB) for the largest cache-resident in-place windows, 192-256 MiB,
        // with the register-form scalar step of 17 <= N <= 32: config 4's 8-GPU share, 8,192 x
        // 30 in place, 78.6 vs 81.5 us (profiles/r06/relay_stamps/geom_8192x30.err; round 4: 76.8
        // vs 79.5 and 77.5 vs 78.1, ab_r04/relay_geom*); at 4,096 x 30 (123 MB) they lose
        // (42.3 vs 41.1), so 256 x 2 stays below
        const bool rows_fit4 = 4 * 256 * 4 / (c.window * 5) + 2 <= 256;
        if ((h->relay_auto & PMENV_FUSE_INPLACE) && win > (192ll << 20) && h->relay_block == 256 &&
            h->relay_kl == 32 && h->relay_ka == 0 && rows_fit4)
            h->relay_v = 4;
    }
    // ---- the generic stream (advance_gen_kernel, F != 5): 2 <= F <= 16 (its halo is the two
    // chunks past a workgroup, four past F = 8), 16-B granular env windows, at most BLOCK rows
    // per workgroup.
    // AUTO gives it every window above 2 MiB (16 MiB where step_tiny_kernel would take it),
    // both modes: against the register step / the LDS fallback, one process, the same bits
    // (profiles/ab_r05/gen_few_r05gf2.*), 64 / 256 x 30 x 50 x 8 in place 9.2 / 11.2 against
    // 12.8 / 14.2 us, 128 x 30 x 50 x 3 8.7 vs 9.2, 32 x 64 x 50 x 8 8.6 vs 16.4, 64 x 100 x 50 x 8
    // 10.9 vs 24.4 (LDS fallback), 2,048 x 128 x 50 x 4 double-buffered 76.8 vs 91.8; ties at 1-2
    // MiB (128 x 16 x 32 x 8 8.9 / 8.9, 64 x 16 x 32 x 8 9.0 vs 8.8); over tiny windows 1,024 x 5 x
    // 50 x 8 (8 MiB) 9.9 vs 7.8, 4,096 x 5 x 50 x 8 17.1 / 17.0, 4,096 x 8 x 32 x 6 14.9 vs 16.7
    {
        const int F = c.features;
        // 512 x 2 chunks per workgroup for windows past 128 MiB, 256 x 2 below (gen_geom_*_r05gg.*,
        // against 256 x 4: 65,536 x 30 x 50 x 8 in place / double-buffered 1,015.5 / 1,033.2 vs
        // 1,061.6 / 1,069.0 us, F = 3 / 4 388.8 / 514.9 vs 406.9 / 537.4, 16,384 x 30 x 50 x 8
        // 254.1 vs 268.3; within 2 % of 256 x 2 at 4,096 envs and below)
        h->gen_block = win > (128ll << 20) ? 512 : 256;
        h->gen_v = 2;
        const int64_t cpw = 1024;                           // the shape rule at the larger tile
        h->gen_ok = F != 5 && F >= 2 && F <= 16 && per % 4 == 0 &&
                    (int64_t)c.num_envs * (per / 4) < (1ll << 31) - 1024 && 4 * cpw / WF + 2 <= 256;
        h->gen_qtot = h->gen_ok ? (uint32_t)((int64_t)c.num_envs * (per / 4)) : 0u;
        h->gen_auto = h->gen_ok && win > (h->tiny ? (16ll << 20) : (2ll << 20)) ? (PMENV_FUSE_DB | PMENV_FUSE_INPLACE) : 0;
    }
    pmenv_tools::plan(h);     // the tools build's PMENV_* knobs (nothing in the product library)
    if (h->streaming) {
        h->units_per_env = (c.num_assets + h->unit_rows - 1) / h->unit_rows;
        h->units_per_env_db = (c.num_assets + h->unit_rows_db - 1) / h->unit_rows_db;
    }
    h->path = PMENV_STEP_PATH_AUTO;
    h->one = h->one_auto;
    h->flat1 = h->flat1_auto;
    h->relay = h->relay_ok ? h->relay_auto : 0;
    h->gen = h->gen_ok ? h->gen_auto : 0;

    h->scalar_scratch_floats = (int)((scratch_bytes(0, c.num_assets, c.features) / 4 + 3) / 4 * 4);
    h->lds_scalar = (size_t)kScalarWaves * h->scalar_scratch_floats * 4;
    if (h->lds_tile > 160 * 1024 || h->lds_scalar > 160 * 1024) {
        set_err(h, "num_assets %d needs more than 160 KiB of LDS", c.num_assets);
        return fail(PMENV_ERR_ARG);
    }
    if ((int64_t)c.num_envs * (h->streaming ? (h->units_per_env > h->units_per_env_db ? h->units_per_env
                                                                                    : h->units_per_env_db)
                                               : 1) >= (1ll << 31)) {
        set_err(h, "too many envs for one launch");
        return fail(PMENV_ERR_ARG);
    }

    DeviceGuard g(device);
    size_t off[PMENV_STATE_FIELDS];
    pmenv_state_layout(&c, off);
    h->state_bytes = pmenv_state_bytes_for(&c);
    if (state) {
        if (state_bytes < h->state_bytes || ((uintptr_t)state & 15u)) {
            set_err(h, "caller state buffer too small (%zu < %zu) or not 16-B aligned", state_bytes, h->state_bytes);
            return fail(PMENV_ERR_ARG);
        }
        h->state = state;
        h->owns_state = false;
    } else {
        hipError_t ae = hipMalloc(&h->state, h->state_bytes);
        if (ae != hipSuccess) {
            set_err(h, "hipMalloc(%zu) failed: %s", h->state_bytes, hipGetErrorString(ae));
            h->state = nullptr;
            return fail(PMENV_ERR_HIP);
        }
        h->owns_state = true;
    }
    if (h->flat_inplace || h->gen_ok) {
        const uint32_t cpw = (uint32_t)(h->flat_inplace ? h->flat_ip_block * h->flat_ip_vec : h->gen_block * h->gen_v);
        const uint32_t qtot = h->flat_inplace ? h->flat_qtot : h->gen_qtot;
        const uint32_t wgs = (qtot + cpw - 1) / cpw;
        h->halo_wgs = wgs > 0 ? wgs - 1 : 0;
        const size_t per_wg = !h->flat_inplace && c.features > 8 ? 64 : 32;   // four chunks past F = 8
        hipError_t ae = hipMalloc(&h->halo, (size_t)(h->halo_wgs + 1) * per_wg);
        if (ae != hipSuccess) {
            set_err(h, "hipMalloc(halo) failed: %s", hipGetErrorString(ae));
            h->halo = nullptr;
            return fail(PMENV_ERR_HIP);
        }
    }
    if (h->flat1_ok) {
        // two parities of the snapshot (16-B aligned fields) and of the tile halo
        const size_t B = (size_t)c.num_envs, BN = B * (size_t)c.num_assets;
        auto up16 = [](size_t x) { return (x + 15) / 16 * 16; };
        const size_t one = up16(B * 8) + up16(B * 4) + 2 * up16(BN * 4);
        const uint32_t cpw = (uint32_t)(h->flat1_block * h->flat1_vec);
        const uint32_t wgs = (h->flat_qtot + cpw - 1) / cpw;
        h->halo1_wgs = wgs > 0 ? wgs - 1 : 0;
        const size_t hal = up16(((size_t)h->halo1_wgs + 1) * 32);
        hipError_t ae = hipMalloc(&h->snap, 2 * (one + hal) + 64);
        if (ae != hipSuccess) {
            set_err(h, "hipMalloc(snapshot) failed: %s", hipGetErrorString(ae));
            h->snap = nullptr;
            return fail(PMENV_ERR_HIP);
        }
        for (int q = 0; q < 2; ++q) {
            char* sb = (char*)h->snap + (size_t)q * (one + hal);
            h->sv[q] = (double*)sb;
            h->sk[q] = (int32_t*)(sb + up16(B * 8));
            h->sw[q] = (float*)(sb + up16(B * 8) + up16(B * 4));
            h->slc[q] = (float*)(sb + up16(B * 8) + up16(B * 4) + up16(BN * 4));
            h->halo1[q] = (float*)(sb + one);
        }
        h->snap_stride = one + hal;
        h->seq = (int32_t*)((char*)h->snap + 2 * (one + hal));
        if (hipMemset(h->seq, 0, 64) != hipSuccess) {
            set_err(h, "hipMemset(seq) failed");
            return fail(PMENV_ERR_HIP);
        }
    }
    if (h->relay_ok) {
        const uint32_t cpw = (uint32_t)(h->relay_block * h->relay_v);
        h->relay_epb = (h->relay_block / 64) * (64 / h->relay_kl);
        h->relay_tiles = (h->flat_qtot + cpw - 1) / cpw;
        h->relay_scal = (uint32_t)(((uint64_t)c.num_envs + (uint64_t)h->relay_epb - 1) / (uint64_t)h->relay_epb);
        if (h->relay && relay_alloc(h) != PMENV_OK) return fail(PMENV_ERR_HIP);
    }
    (void)flat1_invalidate(h, nullptr, kInvalSnap | kInvalHalo, true);   // no device sequencing yet
    char* base = (char*)h->state;
    h->value = (double*)(base + off[0]);
    h->sa = (double*)(base + off[1]);
    h->sb = (double*)(base + off[2]);
    h->k = (int32_t*)(base + off[3]);
    h->ring = (float*)(base + off[4]);
    h->nonfinite = (unsigned long long*)(base + off[5]);
    h->last_close = (float*)(base + off[6]);
    h->w_new = (float*)(base + off[7]);
    const struct { const void* fn; size_t lds; } attrs[] = {
        {(const void*)step_advance_lds_kernel<true>, h->lds_tile},
        {(const void*)step_advance_lds_kernel<false>, h->lds_tile},
        {(const void*)step_surface_kernel, h->lds_surface},
        {(const void*)step_surface_host_kernel, h->lds_surface},
        {(const void*)step_host_resident_kernel, h->lds_surface},
        {(const void*)step_small_kernel<64, 32, false>, h->lds_surface},
        {(const void*)step_small_kernel<256, 8, false>, h->lds_surface},
        {(const void*)step_small_kernel<256, 16, false>, h->lds_surface},
        {(const void*)step_small_kernel<512, 16, false>, h->lds_surface},
        {(const void*)step_small_kernel<1024, 16, false>, h->lds_surface},
        {(const void*)scalar_step_kernel, h->lds_scalar},
    };
    for (const auto& a : attrs)   // only needed above 64 KiB; failures surface at launch
        if (hipFuncSetAttribute(a.fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)a.lds) != hipSuccess)
            (void)hipGetLastError();
    hipError_t e = hipMemset(h->state, 0, h->state_bytes);
    if (e != hipSuccess) {
        set_err(h, "hipMemset failed: %s", hipGetErrorString(e));
        return fail(PMENV_ERR_HIP);
    }
    StepParams p = base_params(h);
    reset_kernel<<<c.num_envs, kBlock, 0, nullptr>>>(p, nullptr, nullptr);
    e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        set_err(h, "initial reset failed: %s", hipGetErrorString(e));
        return fail(PMENV_ERR_HIP);
    }
    *out = h;
    return PMENV_OK;
}

namespace {
void res_stop(pmenv* h);    // the resident host-I/O step (below)
}

int pmenv_destroy(pmenv* h) {
    if (!h) return PMENV_ERR_ARG;
    DeviceGuard g(h->device);
    pmenv_tools::release(h);
    if (h->state && h->owns_state) (void)hipFree(h->state);
    if (h->halo) (void)hipFree(h->halo);
    if (h->snap) (void)hipFree(h->snap);
    if (h->relay_mem) (void)hipFree(h->relay_mem);
    if (h->hio) {
        res_stop(h);
        (void)hipHostFree(h->hio);
    }
    if (h->res_stream) {
        (void)hipEventDestroy(h->res_ev);
        (void)hipStreamDestroy(h->res_stream);
        (void)hipFree(h->res_last);
    }
    free(h);
    return PMENV_OK;
}

int pmenv_set_step_path(pmenv* h, int32_t path) {
    if (!h) return PMENV_ERR_ARG;
    if (path < PMENV_STEP_PATH_AUTO || path > PMENV_STEP_PATH_RELAY) {
        set_err(h, "unknown step path %d", path);
        return PMENV_ERR_ARG;
    }
    const int bits = one_bits(h, path);
    const int fbits = flat1_bits(h, path);
    const int rbits = relay_bits(h, path);
    if (bits < 0 || fbits < 0 || rbits < 0) {
        set_err(h, "step path %d does not fit this shape (one launch: F = 5, W >= 2, N <= 64, window <= 64 KiB "
                   "of LDS; two launches: F = 5, 16-B granular env windows; flat: F = 5, W >= 2, N <= 64, "
                   "16-B granular env windows of >= 148 chunks, N > 64 up to 512 with W >= 14; relay: F = 5, "
                   "W >= 2, 16-B granular env windows, N <= 512)", path);
        return PMENV_ERR_ARG;
    }
    if (rbits && relay_alloc(h) != PMENV_OK) return PMENV_ERR_HIP;
    h->path = path;
    h->one = bits;
    h->flat1 = fbits;
    h->relay = rbits;
    h->gen = gen_bits(h, path);
    return PMENV_OK;
}

int pmenv_reset(pmenv* h, float* obs, const uint8_t* mask, hipStream_t stream) {
    if (!h) return PMENV_ERR_ARG;
    h->dev_pending = true;                          // device work of this handle may be in flight
    if (obs && !aligned4(obs)) { set_err(h, "obs not 4-byte aligned"); return PMENV_ERR_ALIGN; }
    DeviceGuard g(h->device);
    StepParams p = base_params(h);
    if (const int rc = flat1_invalidate(h, stream)) return rc;
    reset_kernel<<<h->cfg.num_envs, kBlock, 0, stream>>>(p, obs, mask);
    return check_launch(h, "reset_kernel");
}

int pmenv_step_ex(pmenv* h, const pmenv_step_args* a, hipStream_t stream) {
    if (!h) return PMENV_ERR_ARG;
    h->dev_pending = true;                          // device work of this handle may be in flight
    if (!a || !a->action) { set_err(h, "action is required"); return PMENV_ERR_ARG; }
    if (!a->bar && !a->prices) { set_err(h, "surface mode (bar == NULL) needs prices"); return PMENV_ERR_ARG; }
    if (a->bar && !a->obs) { set_err(h, "advance mode (bar != NULL) needs obs"); return PMENV_ERR_ARG; }
    if (!aligned4(a->action) || (a->prices && !aligned4(a->prices)) || (a->bar && !aligned4(a->bar)) ||
        (a->obs && !aligned4(a->obs)) || (a->reward && !aligned4(a->reward)) ||
        (a->weights && !aligned4(a->weights)) || (a->ret && ((uintptr_t)a->ret & 7u))) {
        set_err(h, "unaligned pointer");
        return PMENV_ERR_ALIGN;
    }
    DeviceGuard g(h->device);
    StepParams p = base_params(h);
    if (a->day && (!a->bar || a->series_days < 1)) {
        set_err(h, "day[] needs the series in bar and series_days >= 1");
        return PMENV_ERR_ARG;
    }
    p.action = a->action; p.prices = a->prices; p.bar = a->bar; p.obs = a->obs;
    p.day = a->day; p.series_days = a->series_days;
    p.obs_out = a->obs_out ? a->obs_out : a->obs;
    if (a->obs_out && a->bar) {
        const size_t bytes = (size_t)h->cfg.num_envs * h->cfg.num_assets * h->cfg.window * h->cfg.features * 4;
        const char *o0 = (const char*)a->obs, *o1 = (const char*)a->obs_out;
        if (!aligned4(a->obs_out) || (o1 < o0 + bytes && o0 < o1 + bytes)) {
            set_err(h, "obs_out must be 4-byte aligned and must not overlap obs");
            return PMENV_ERR_ARG;
        }
    }
    p.reward = a->reward; p.ret = a->ret; p.weights = a->weights;
    const int B = h->cfg.num_envs;
    const bool obs16 = (((uintptr_t)a->obs | (uintptr_t)p.obs_out) & 15u) == 0;
    const int fuse_bit = p.obs_out == p.obs ? PMENV_FUSE_INPLACE : PMENV_FUSE_DB;
    if (a->bar && h->streaming && obs16 && (h->flat1 & fuse_bit)) {
        // one launch over the flat stream: the whole step runs in the scalar phase
        const uint32_t ph = a->phases ? a->phases : (PMENV_PHASE_SCALAR | PMENV_PHASE_ADVANCE);
        if (!(ph & PMENV_PHASE_SCALAR)) return PMENV_OK;
        // a step captured into a hipGraph replays with frozen arguments: from then on this
        // handle sequences its flat steps on the device (flat_seq_kernel + the kernel)
        if (!h->device_seq && capturing(stream)) h->device_seq = true;
        note_capture(h, stream);
        // the relay step's halo and counter copy go stale
        if (const int rc = relay_invalidate(h, stream, kInvalSnap | kInvalHalo)) return rc;
        launch_flat1(h, p, stream);
        return check_launch(h, "step_flat_kernel");
    }
    if (a->bar && h->streaming && obs16 && (h->relay & fuse_bit)) {
        // one launch, the scalar work relaying to the stream tiles (captured: device-sequenced)
        const uint32_t ph = a->phases ? a->phases : (PMENV_PHASE_SCALAR | PMENV_PHASE_ADVANCE);
        if (!(ph & PMENV_PHASE_SCALAR)) return PMENV_OK;
        if (const int rc = flat1_invalidate(h, stream, kInvalSnap | kInvalHalo, false, true)) return rc;
        if (launch_relay(h, p, stream) != PMENV_OK) {
            set_err(h, "relay step: hipMemsetAsync failed");
            return PMENV_ERR_HIP;
        }
        return check_launch(h, "step_relay_kernel");
    }
    if (const int rc = flat1_invalidate(h, stream)) return rc;   // every other path skips the snapshot
    if (!a->bar && h->surf_stream && (((uintptr_t)a->obs) & 15u) == 0) {
        // past the Infinity Cache: the scalar step, then the surface stream
        const uint32_t ph = a->phases ? a->phases : (PMENV_PHASE_SCALAR | PMENV_PHASE_ADVANCE);
        if (ph & PMENV_PHASE_SCALAR) {
            launch_scalar_kernels(h, p, stream);
            if (const int rc = check_launch(h, "scalar_step_kernel")) return rc;
        }
        if (ph & PMENV_PHASE_ADVANCE) {
            launch_surface_stream(h, p, stream);
            return check_launch(h, "surface_stream_kernel");
        }
        return PMENV_OK;
    }
    if (!a->bar) {
        if (a->phases == PMENV_PHASE_ADVANCE) return PMENV_OK;   // single launch: done in the scalar phase
        step_surface_kernel<<<B, kBlock, h->lds_surface, stream>>>(p);
        return check_launch(h, "step_surface_kernel");
    }
    if (h->streaming && obs16) {
        const uint32_t ph = a->phases ? a->phases : (PMENV_PHASE_SCALAR | PMENV_PHASE_ADVANCE);
        if (h->one & fuse_bit) {       // one launch: the whole step runs in the scalar phase
            if (!(ph & PMENV_PHASE_SCALAR)) return PMENV_OK;
            launch_one(h, p, stream);
            return check_launch(h, "step_env_kernel");
        }
        if (pmenv_tools::launch_fused(h, p, fuse_bit, ph, stream)) return check_launch(h, "tools: fused step");
        if (ph & PMENV_PHASE_SCALAR) {
            launch_scalar(h, p, stream);
            const int rc = check_launch(h, "scalar_step_kernel");
            if (rc) return rc;
        }
        if (ph & PMENV_PHASE_ADVANCE) {
            launch_advance(h, p, stream);
            return check_launch(h, "advance kernel");
        }
        return PMENV_OK;
    }
    if (h->gen_ok && (h->gen & fuse_bit) && obs16) {
        // F != 5: the scalar step (copying the in-place stream's halo), then the generic stream
        const uint32_t ph = a->phases ? a->phases : (PMENV_PHASE_SCALAR | PMENV_PHASE_ADVANCE);
        if (ph & PMENV_PHASE_SCALAR) {
            launch_scalar(h, p, stream);
            const int rc = check_launch(h, "scalar_step_kernel");
            if (rc) return rc;
        }
        if (ph & PMENV_PHASE_ADVANCE) {
            launch_gen(h, p, stream);
            return check_launch(h, "advance_gen_kernel");
        }
        return PMENV_OK;
    }
    if (a->phases == PMENV_PHASE_ADVANCE) return PMENV_OK;   // single-launch path: all done in the scalar phase
    if (h->small_block) {
        launch_small(h, p, stream);
        return check_launch(h, h->tiny ? "step_tiny_kernel" : "step_small_kernel");
    }
    if (h->vec && obs16)
        step_advance_lds_kernel<true><<<B, kBlock, h->lds_tile, stream>>>(p);
    else
        step_advance_lds_kernel<false><<<B, kBlock, h->lds_tile, stream>>>(p);
    return check_launch(h, "step_advance_lds_kernel");
}

int pmenv_step(pmenv* h, const float* action, const float* prices, const float* bar, float* obs, float* reward,
               hipStream_t stream) {
    pmenv_step_args a;
    memset(&a, 0, sizeof(a));
    a.action = action; a.prices = prices; a.bar = bar; a.obs = obs; a.reward = reward;
    return pmenv_step_ex(h, &a, stream);
}

}  // extern "C"

namespace {
// The host-I/O staging block (allocated on first use, freed by destroy): f32 action |
// prices | closes [B*N] each, channel [B*N*W], weights [B*N], reward [B]; f64 return |
// value [B]; u32 completion words [B]; the resident step's go word. Pinned and device-mapped,
// so the kernels read and write it over PCIe directly.
int hio_ensure(pmenv* h) {
    if (h->hio) return PMENV_OK;
    const size_t B = (size_t)h->cfg.num_envs, BN = B * (size_t)h->cfg.num_assets;
    auto up64 = [](size_t x) { return (x + 63) / 64 * 64; };
    size_t o = 0;
    const size_t sizes[10] = {BN * 4, BN * 4, BN * 4, BN * (size_t)h->cfg.window * 4, BN * 4, B * 4, B * 8, B * 8,
                              B * 4, 4};
    for (int i = 0; i < 10; ++i) {
        h->hio_off[i] = o;
        o = up64(o + sizes[i]);
    }
    void* p = nullptr;
    // coherent (fine-grained): the GPU never caches it, so each step reads what the host
    // just wrote and the host reads the kernel's stores after the stream sync
    hipError_t e = hipHostMalloc(&p, o, hipHostMallocMapped | hipHostMallocCoherent);
    if (e != hipSuccess) {
        set_err(h, "hipHostMalloc(%zu) for host-I/O staging failed: %s", o, hipGetErrorString(e));
        return PMENV_ERR_HIP;
    }
    void* d = nullptr;
    e = hipHostGetDevicePointer(&d, p, 0);
    if (e != hipSuccess) {
        (void)hipHostFree(p);
        set_err(h, "hipHostGetDevicePointer: %s", hipGetErrorString(e));
        return PMENV_ERR_HIP;
    }
    h->hio = (char*)p;
    h->hio_dev = (char*)d;
    memset(h->hio + h->hio_off[8], 0, B * 4);      // completion words: no call yet (tags start at 1)
    memset(h->hio + h->hio_off[9], 0, 4);          // the go word: no tag posted
    h->hio_seq = 0;
    return PMENV_OK;
}
enum { kHioAct, kHioPri, kHioClose, kHioChan, kHioW, kHioRew, kHioRet, kHioVal, kHioDone, kHioGo };
template <class T>
T* hio_host(const pmenv* h, int f) { return reinterpret_cast<T*>(h->hio + h->hio_off[f]); }
template <class T>
T* hio_dev(const pmenv* h, int f) { return reinterpret_cast<T*>(h->hio_dev + h->hio_off[f]); }

// the window's last closes obs[b, n, W-1, close] -> staging (the only window bytes the step reads)
void hio_gather_closes(pmenv* h, const float* obs) {
    const pmenv_cfg& c = h->cfg;
    const size_t BN = (size_t)c.num_envs * c.num_assets, row = (size_t)c.window * c.features;
    const float* src = obs + (size_t)(c.window - 1) * c.features + c.close_channel;
    float* dst = hio_host<float>(h, kHioClose);
    for (size_t i = 0; i < BN; ++i) dst[i] = src[i * row];
}
// the [B, N, W] channel the kernel wrote -> obs[..., F-1] of the caller's window
void hio_scatter_channel(const pmenv* h, float* obs) {
    const pmenv_cfg& c = h->cfg;
    const size_t BNW = (size_t)c.num_envs * c.num_assets * c.window;
    const int F = c.features;
    const float* src = hio_host<float>(h, kHioChan);
    float* dst = obs + (F - 1);
    for (size_t i = 0; i < BNW; ++i) dst[i * F] = src[i];
}
// The call's completion: every env's completion word carries the call's tag once its outputs
// are in host memory (the kernels write it last, at system scope, after every store of the
// workgroup has completed). The host spins on the words — they turn a few us after the
// launch — instead of synchronising the stream: 12.3 / 14.8 us per pmenv_step_host call
// against 18.2 / 20.1 with hipStreamSynchronize at 1 x 5 x 50 x 5 / 1 x 32 x 32 x 5
// (profiles/hostio_r05/hostio_r05h*.json). Past ~2 ms (a large batch, or a kernel that
// failed) it synchronises the stream, which also reports an error.
int hio_sync(pmenv* h, hipStream_t stream, const char* what) {
    if (const int rc = check_launch(h, what)) return rc;
    const volatile uint32_t* done = hio_host<volatile uint32_t>(h, kHioDone);
    const uint32_t seq = h->hio_seq;
    const int B = h->cfg.num_envs;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t it = 0;; ++it) {
        int b = 0;
        while (b < B && done[b] == seq) ++b;
        if (b == B) {
            __atomic_thread_fence(__ATOMIC_ACQUIRE);        // the outputs are read after the words
            return PMENV_OK;
        }
        if ((it & 255u) == 255u && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) break;
    }
    const hipError_t e = hipStreamSynchronize(stream);
    if (e != hipSuccess) {
        set_err(h, "%s: %s", what, hipGetErrorString(e));
        return PMENV_ERR_HIP;
    }
    return PMENV_OK;
}

// ---- the resident host-I/O step (step_host_resident_kernel): no launch per call
constexpr int kResMaxEnvs = 8;             // one workgroup steps every env in turn
constexpr uint32_t kResIdle = 2000000u;    // 20 ms of s_memrealtime (100 MHz) without a call: it exits

// the workgroup exits (the stop tag) and the handle forgets it (destroy, or its launch
// arguments no longer match the call's)
void res_stop(pmenv* h) {
    if (!h->res_live) return;
    __atomic_store_n(hio_host<uint32_t>(h, kHioGo), 0u, __ATOMIC_RELEASE);
    (void)hipEventSynchronize(h->res_ev);
    h->res_live = false;
}

int res_launch(pmenv* h, const StepParams& p, const HostIO& io) {
    if (!h->res_stream) {
        if (hipStreamCreateWithFlags(&h->res_stream, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&h->res_ev, hipEventDisableTiming) != hipSuccess ||
            hipMalloc((void**)&h->res_last, 64) != hipSuccess || hipMemset(h->res_last, 0, 64) != hipSuccess) {
            set_err(h, "resident host-I/O step: stream / event / memory");
            return PMENV_ERR_HIP;
        }
    }
    // the go word holds the last tag posted (or 0): a fresh workgroup starts from what the
    // previous one ran, so an unseen tag is run and a seen one is not run twice
    HostRes rs;
    rs.go = hio_dev<uint32_t>(h, kHioGo);
    rs.last = h->res_last;
    rs.idle = kResIdle;
    step_host_resident_kernel<<<1, kBlock, h->lds_surface, h->res_stream>>>(p, io, rs);
    if (const int rc = check_launch(h, "step_host_resident_kernel")) return rc;
    if (hipEventRecord(h->res_ev, h->res_stream) != hipSuccess) {
        set_err(h, "resident host-I/O step: event record");
        return PMENV_ERR_HIP;
    }
    h->res_live = true;
    h->res_p = p;
    h->res_io = io;
    return PMENV_OK;
}

// post the call's tag (its inputs are in the staging: stored before, released with the tag) and
// spin on the completion words; a workgroup that exited idle before it saw the tag is relaunched
int res_step(pmenv* h, const StepParams& p, const HostIO& io) {
    const bool same = h->res_live && memcmp(&h->res_p, &p, sizeof p) == 0 &&
                      h->res_io.close_in == io.close_in && h->res_io.chan == io.chan &&
                      h->res_io.value_out == io.value_out && h->res_io.done == io.done;
    if (!same) res_stop(h);
    if (!h->res_live || hipEventQuery(h->res_ev) == hipSuccess)
        if (const int rc = res_launch(h, p, io)) return rc;
    __atomic_store_n(hio_host<uint32_t>(h, kHioGo), io.seq, __ATOMIC_RELEASE);
    const volatile uint32_t* done = hio_host<volatile uint32_t>(h, kHioDone);
    const int B = h->cfg.num_envs;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t it = 1;; ++it) {
        int b = 0;
        while (b < B && done[b] == io.seq) ++b;
        if (b == B) {
            __atomic_thread_fence(__ATOMIC_ACQUIRE);        // the outputs are read after the words
            return PMENV_OK;
        }
        if ((it & 1023u) == 0u) {
            const hipError_t q = hipEventQuery(h->res_ev);
            if (q == hipSuccess) {                          // exited idle as the tag arrived: relaunch
                if (const int rc = res_launch(h, p, io)) return rc;
            } else if (q != hipErrorNotReady) {
                set_err(h, "step_host_resident_kernel: %s", hipGetErrorString(q));
                return PMENV_ERR_HIP;
            }
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
                set_err(h, "step_host_resident_kernel: no completion within 2 s");
                return PMENV_ERR_HIP;
            }
        }
    }
}
}  // namespace

extern "C" {

int pmenv_step_host(pmenv* h, const float* action, const float* prices, float* obs, float* reward, double* value,
                    double* ret, float* weights, hipStream_t stream) {
    if (!h) return PMENV_ERR_ARG;
    if (!action || !prices) { set_err(h, "host step: action and prices are required"); return PMENV_ERR_ARG; }
    DeviceGuard g(h->device);
    if (capturing(stream)) {          // the host waits on the kernel's words: nothing runs under capture
        set_err(h, "pmenv_step_host is not graph-capturable (the stream is being captured)");
        return PMENV_ERR_ARG;
    }
    if (const int rc = hio_ensure(h)) return rc;
    // the resident workgroup (no launch per call) for a few envs when none of this handle's own
    // device work can be pending (what the call would otherwise be ordered after on `stream`);
    // else one launch on `stream`
    // (dev_pending: this handle enqueued device work since its last synchronous call — the
    // ordering a launch on `stream` gives; hipStreamQuery would cost ~9 us per call)
    const bool resident = h->cfg.num_envs <= kResMaxEnvs && !h->dev_pending;
    const pmenv_cfg& c = h->cfg;
    const size_t B = (size_t)c.num_envs, BN = B * (size_t)c.num_assets;
    memcpy(hio_host<float>(h, kHioAct), action, BN * 4);
    memcpy(hio_host<float>(h, kHioPri), prices, BN * 4);
    if (obs) hio_gather_closes(h, obs);
    if (const int rc = flat1_invalidate(h, stream)) return rc;   // the snapshot / halos go stale
    StepParams p = base_params(h);
    p.action = hio_dev<float>(h, kHioAct);
    p.prices = hio_dev<float>(h, kHioPri);
    p.reward = hio_dev<float>(h, kHioRew);
    p.ret = hio_dev<double>(h, kHioRet);
    p.weights = hio_dev<float>(h, kHioW);
    HostIO io;
    io.close_in = hio_dev<float>(h, kHioClose);
    io.chan = obs ? hio_dev<float>(h, kHioChan) : nullptr;
    io.value_out = hio_dev<double>(h, kHioVal);
    io.done = hio_dev<uint32_t>(h, kHioDone);
    io.seq = h->hio_seq = h->hio_seq + 1u == 0u ? 1u : h->hio_seq + 1u;
    if (resident) {
        if (const int rc = res_step(h, p, io)) return rc;
    } else {
        step_surface_host_kernel<<<c.num_envs, kBlock, h->lds_surface, stream>>>(p, io);
        if (const int rc = hio_sync(h, stream, "step_surface_host_kernel")) return rc;
        h->dev_pending = false;                     // everything before it on `stream` has run
    }
    if (obs) hio_scatter_channel(h, obs);
    if (reward) memcpy(reward, hio_host<float>(h, kHioRew), B * 4);
    if (ret) memcpy(ret, hio_host<double>(h, kHioRet), B * 8);
    if (value) memcpy(value, hio_host<double>(h, kHioVal), B * 8);
    if (weights) memcpy(weights, hio_host<float>(h, kHioW), BN * 4);
    return PMENV_OK;
}

int pmenv_reset_host(pmenv* h, float* obs, double* value, hipStream_t stream) {
    if (!h) return PMENV_ERR_ARG;
    DeviceGuard g(h->device);
    if (capturing(stream)) {
        set_err(h, "pmenv_reset_host is not graph-capturable (the stream is being captured)");
        return PMENV_ERR_ARG;
    }
    if (const int rc = hio_ensure(h)) return rc;
    if (obs) hio_gather_closes(h, obs);
    if (const int rc = flat1_invalidate(h, stream)) return rc;
    StepParams p = base_params(h);
    HostIO io;
    io.close_in = hio_dev<float>(h, kHioClose);
    io.chan = obs ? hio_dev<float>(h, kHioChan) : nullptr;
    io.value_out = hio_dev<double>(h, kHioVal);
    io.done = hio_dev<uint32_t>(h, kHioDone);
    io.seq = h->hio_seq = h->hio_seq + 1u == 0u ? 1u : h->hio_seq + 1u;
    reset_kernel<<<h->cfg.num_envs, kBlock, 0, stream>>>(p, nullptr, nullptr, io);
    if (const int rc = hio_sync(h, stream, "reset_kernel (host I/O)")) return rc;
    h->dev_pending = false;
    if (obs) hio_scatter_channel(h, obs);
    if (value) memcpy(value, hio_host<double>(h, kHioVal), (size_t)h->cfg.num_envs * 8);
    return PMENV_OK;
}

double* pmenv_value(pmenv* h) { return h ? h->value : nullptr; }
float* pmenv_ring(pmenv* h) { return h ? h->ring : nullptr; }
int32_t* pmenv_counter(pmenv* h) { return h ? h->k : nullptr; }
size_t pmenv_state_bytes(const pmenv* h) { return h ? h->state_bytes : 0; }

const char* pmenv_step_path(const pmenv* h) {
    if (!h) return "";
    // per window mode: the one-launch kernel, or the scalar step (K1) then the stream
    const char* k1 = h->k1_vec ? "scalar_step_vec_kernel"
                   : h->cfg.num_assets <= 64 ? "scalar_step_reg_kernel" : "scalar_step_kernel";
    if (!h->streaming) {
        const char* one = h->tiny ? "step_tiny_kernel" : h->small_block ? "step_small_kernel" : "step_advance_lds_kernel";
        if (!h->gen) return one;
        static thread_local char gout[320];
        char g2[96];
        snprintf(g2, sizeof g2, "%s+advance_gen_kernel", k1);
        snprintf(gout, sizeof gout, "%s (obs_out) | %s (in place)", (h->gen & PMENV_FUSE_DB) ? g2 : one,
                 (h->gen & PMENV_FUSE_INPLACE) ? g2 : one);
        return gout;
    }
    const char* db2 = h->flat ? "advance_flat_wg_kernel" : "advance_rows_kernel";
    const char* ip2 = h->flat_inplace ? "advance_flat_inplace_kernel" : "advance_rows_kernel";
    static thread_local char buf[2][128], out[320];
    const char* part[2];
    for (int m = 0; m < 2; ++m) {          // 0 = double-buffered (obs_out), 1 = in place
        const int bit = m ? PMENV_FUSE_INPLACE : PMENV_FUSE_DB;
        if (h->relay & bit) part[m] = "step_relay_kernel";
        else if (h->flat1 & bit) part[m] = h->cfg.num_assets > 64 ? "step_flat_vec_kernel" : "step_flat_kernel";
        else if (h->one & bit) part[m] = "step_env_kernel";
        else {
            snprintf(buf[m], sizeof buf[m], "%s+%s", k1, m ? ip2 : db2);
            part[m] = buf[m];
        }
    }
    snprintf(out, sizeof out, "%s (obs_out) | %s (in place)%s%s", part[0], part[1],
             h->device_seq && h->flat1 ? " [flat steps device-sequenced]" : "",
             h->relay_dseq && h->relay ? " [relay steps device-sequenced]" : "");
    return out;
}

int pmenv_get_state(pmenv* h, void* dst, hipStream_t stream) {
    if (!h || !dst) return PMENV_ERR_ARG;
    h->dev_pending = true;                          // device work of this handle may be in flight
    DeviceGuard g(h->device);
    hipError_t e = hipMemcpyAsync(dst, h->state, h->state_bytes, hipMemcpyDeviceToDevice, stream);
    if (e != hipSuccess) { set_err(h, "get_state: %s", hipGetErrorString(e)); return PMENV_ERR_HIP; }
    return PMENV_OK;
}

int pmenv_set_state(pmenv* h, const void* src, hipStream_t stream) {
    if (!h || !src) return PMENV_ERR_ARG;
    h->dev_pending = true;                          // device work of this handle may be in flight
    DeviceGuard g(h->device);
    if (const int rc = flat1_invalidate(h, stream)) return rc;
    hipError_t e = hipMemcpyAsync(h->state, src, h->state_bytes, hipMemcpyDeviceToDevice, stream);
    if (e != hipSuccess) { set_err(h, "set_state: %s", hipGetErrorString(e)); return PMENV_ERR_HIP; }
    return PMENV_OK;
}

int pmenv_window_written(pmenv* h, const float* obs, hipStream_t stream) {
    if (!h) return PMENV_ERR_ARG;
    h->dev_pending = true;                          // device work of this handle may be in flight
    (void)obs;                                 // any window: the halo is dropped whichever it was
    DeviceGuard g(h->device);
    return flat1_invalidate(h, stream, kInvalHalo);
}

int pmenv_state_written(pmenv* h, hipStream_t stream) {
    if (!h) return PMENV_ERR_ARG;
    h->dev_pending = true;                          // device work of this handle may be in flight
    DeviceGuard g(h->device);
    return flat1_invalidate(h, stream, kInvalSnap | kInvalHalo);
}

int pmenv_nonfinite_count(pmenv* h, uint64_t* out, hipStream_t stream) {
    if (!h || !out) return PMENV_ERR_ARG;
    h->dev_pending = true;                          // device work of this handle may be in flight
    DeviceGuard g(h->device);
    unsigned long long v = 0;
    hipError_t e = hipMemcpyAsync(&v, h->nonfinite, 8, hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) { set_err(h, "nonfinite_count: %s", hipGetErrorString(e)); return PMENV_ERR_HIP; }
    *out = v;
    return PMENV_OK;
}

int pmenv_synth_series(float* series, int32_t T, int32_t B, int32_t N, int64_t env_offset, uint64_t seed,
                       float sigma, hipStream_t stream) {
    if (!series || T < 1 || B < 1 || N < 1 || ((uintptr_t)series & 15u)) return PMENV_ERR_ARG;
    const int64_t threads = (int64_t)B * N;
    synth_series_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, stream>>>(
        reinterpret_cast<f4*>(series), T, B, N, env_offset, seed, (double)sigma);
    return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
}

int pmenv_synth_actions(float* actions, int32_t T, int32_t B, int32_t N, int64_t env_offset, uint64_t seed,
                        hipStream_t stream) {
    if (!actions || T < 1 || B < 1 || N < 1) return PMENV_ERR_ARG;
    const int64_t threads = (int64_t)T * B;
    synth_actions_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, stream>>>(actions, T, B, N, env_offset, seed);
    return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
}

int pmenv_window_init(float* obs, const float* series, int32_t B, int32_t N, int32_t W, int32_t F,
                      hipStream_t stream) {
    if (!obs || !series || B < 1 || N < 1 || W < 1 || F != 5 || ((uintptr_t)series & 15u)) return PMENV_ERR_ARG;
    const int64_t threads = (int64_t)B * N * W;
    window_init_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, stream>>>(
        obs, reinterpret_cast<const f4*>(series), B, N, W, F);
    return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
}

int pmenv_window_init_days(float* obs, const float* series, int32_t T, int32_t N, int32_t F, const int32_t* start,
                           int32_t B, int32_t W, hipStream_t stream) {
    if (!obs || !series || !start || T < 1 || B < 1 || N < 1 || W < 1 || F < 2) return PMENV_ERR_ARG;
    const int64_t threads = (int64_t)B * N * W;
    window_init_days_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, stream>>>(obs, series, T, N, F, start, B, W);
    return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
}

int pmenv_gae(const float* rewards, const float* values, const uint8_t* dones, float* adv, float* ret, int32_t T,
              int32_t B, float gamma, float lam, hipStream_t stream) {
    if (!rewards || !values || !adv || !ret || T < 1 || B < 1) return PMENV_ERR_ARG;
    int rc = PMENV_OK;
    if (pmenv_tools::gae(rewards, values, dones, adv, ret, T, B, gamma, lam, stream, &rc)) return rc;
    // measured on MI355X (tools/bench_rows.py, profiles/rows_r01.json): the tiled scan
    // beats the per-env loop 2.7x at T = 256 x B = 65536 and 14x at 2048 x 8192; the
    // wave-per-env scan only for a handful of envs with long horizons
    const bool fits = (size_t)(T + 1) * (size_t)B * 4u < (1ull << 31);   // gae_tile_kernel's buffer offsets
    const bool scan = B < 64 && T >= 256;
    const bool tile = fits && !scan;
    const int U = B >= 16384 ? 8 : 16;           // steps per lane and segment
    // many envs and at least four 64-day segments: the tile held to 64 VGPRs (8 waves per
    // SIMD, so a 65,536-env rollout's 1,024 workgroups are resident at once; the same bits):
    // 56.7 vs 58.5 us at 256 x 65,536, 110.1 vs 114.7 at 512 x 65,536; slower below 65,536
    // envs or 256 days (profiles/ab_r02/gae_occ8_r02zl.json)
    // adv / ret are written once and read by the learner later: nt stores where they measured
    // faster (the same bits): 62.3 -> 45.7 us at 256 x 65,536, 9.0 -> 8.4 at 256 x 4,096,
    // 80.2 -> 58.9 at 2,048 x 8,192 on the tile; at 256 x 16,384 (the U = 8 tile, a cache-
    // resident rollout) 14.1 vs 14.5, so that form keeps plain stores
    // (profiles/rows_r03ad/rows_nt2.json)
    if (tile && U == 8 && B >= 65536 && T >= 256)
        gae_tile_kernel<8, 8, 8, 2><<<(B + 63) / 64, 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma,
                                                                      lam);
    else if (tile && U == 16)
        gae_tile_kernel<8, 16, 1, 2><<<(B + 63) / 64, 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma,
                                                                       lam);
    else if (tile)
        gae_tile_kernel<8, 8><<<(B + 63) / 64, 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma,
                                                                lam);
    else if (scan)
        gae_scan_kernel<<<(B + 3) / 4, 256, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam);
    else
        gae_kernel<<<(B + 255) / 256, 256, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam);
    return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
}

// Horizon split of the tiled GAE scan: used when the B / 64 env blocks leave CUs idle (few
// envs, long horizons). Round 4: one pass (gae_lookback_kernel, 64- or 128-day chunks, every chunk
// composing the later chunks' published maps) in place of the round-3 maps + apply passes
// (gae_chunk_kernel, now in the tools build).
namespace {
// chunk length S = NW x U days: 8 waves x 16 days where that still makes 128 workgroups, else
// 8 x 8 (fewer composes per chunk against fewer workgroups). T x B = 4,096 x 512: 9.85 us for
// 128-day chunks against 12.7 for 64-day; 16,384 x 64: 10.3 vs 11.2; 2,048 x 4,096: 31.5 vs
// 32.4; 1,000 x 200 (32 workgroups): 8.7 vs 7.7 (profiles/ab_r04/gae_geom_r04h.err)
int gae_lb_seg(int32_t T, int32_t B) {
    const int64_t wg16 = (int64_t)((T + 127) / 128) * ((B + 63) / 64);
    return wg16 >= 128 ? 128 : 64;
}
int gae_lb_chunks(int32_t T, int32_t B) {
    // from 8,192 envs (128 workgroups) the one-pass tile with nt stores wins: 2,048 x 8,192
    // 59.0 vs 74.2 us for the round-3 split (profiles/rows_r03af/rows_r03af.json)
    if (B >= 8192 || T < 512) return 0;
    if ((size_t)(T + 1) * (size_t)B * 4u >= (1ull << 31)) return 0;
    const int seg = gae_lb_seg(T, B);
    return (T + seg - 1) / seg;
}
// the look-back flags' epochs: a process-wide counter from a clock-mixed start, so a flag word
// left in a reused workspace (an older epoch) or garbage (2^-64) never passes for this call's
std::atomic<uint64_t> g_gae_epoch{0};
uint64_t gae_next_epoch() {
    uint64_t e = g_gae_epoch.load();
    if (e == 0) {
        const uint64_t seed = ((uint64_t)std::chrono::steady_clock::now().time_since_epoch().count() *
                               0x9E3779B97F4A7C15ull) | 1ull;
        g_gae_epoch.compare_exchange_strong(e, seed);
    }
    return g_gae_epoch.fetch_add(1) + 1;
}
}  // namespace

size_t pmenv_gae_workspace(int32_t T, int32_t B) {
    const int n = (T < 1 || B < 1) ? 0 : gae_lb_chunks(T, B);
    return n ? ((size_t)2 * n * B + (size_t)n * ((B + 63) / 64)) * sizeof(double) : 0;
}

int pmenv_gae_ex(const float* rewards, const float* values, const uint8_t* dones, float* adv, float* ret, int32_t T,
                 int32_t B, float gamma, float lam, double* work, size_t work_bytes, hipStream_t stream) {
    if (!rewards || !values || !adv || !ret || T < 1 || B < 1) return PMENV_ERR_ARG;
    const int n = gae_lb_chunks(T, B);
    int rc = PMENV_OK;
    if (pmenv_tools::gae(rewards, values, dones, adv, ret, T, B, gamma, lam, stream, &rc)) return rc;
    if (!n || !work || work_bytes < pmenv_gae_workspace(T, B) || ((uintptr_t)work & 7u))
        return pmenv_gae(rewards, values, dones, adv, ret, T, B, gamma, lam, stream);
    const int neb = (B + 63) / 64;
    uint64_t* flags = reinterpret_cast<uint64_t*>(work + (size_t)2 * n * B);
    if (gae_lb_seg(T, B) == 128)
        gae_lookback_kernel<8, 16><<<(unsigned)(n * neb), 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B,
                                                                          gamma, lam, n, work, flags, gae_next_epoch());
    else
        gae_lookback_kernel<8, 8><<<(unsigned)(n * neb), 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B,
                                                                         gamma, lam, n, work, flags, gae_next_epoch());
    return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
}

size_t pmenv_moments_workspace(void) { return (size_t)kMomBlocks * 2 * sizeof(double); }

int pmenv_moments(const float* x, int64_t n, double* out, double* work, hipStream_t stream) {
    if ((!x && n > 0) || !out || !work || n < 0) return PMENV_ERR_ARG;
    const int64_t want = (n + kMomBlock * 16 - 1) / (kMomBlock * 16);   // >= 16 floats per thread
    const int blocks = (int)(want < 1 ? 1 : (want > kMomBlocks ? kMomBlocks : want));
    moments_partial_kernel<<<blocks, kMomBlock, 0, stream>>>(x, n, work);
    moments_final_kernel<<<1, kMomBlock, 0, stream>>>(blocks, n, work, out);
    return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
}

int pmenv_replay_gather(const float* series, int32_t T, int32_t N, int32_t F, int32_t W, const int32_t* days,
                        const float* actions, const float* rewards, int32_t H, int32_t B, const int32_t* h0,
                        const int32_t* env, int32_t S, float* s, float* s_next, float* a_out, float* r_out,
                        hipStream_t stream) {
    if (!series || !days || !actions || !rewards || !h0 || !env || !s || !s_next || !a_out || !r_out || T < 1 ||
        N < 1 || F < 2 || W < 1 || H < W + 1 || B < 1 || S < 1)
        return PMENV_ERR_ARG;
    int rc = PMENV_OK;
    if (pmenv_tools::replay_gather(series, T, N, F, W, days, actions, rewards, H, B, h0, env, S, s, s_next, a_out,
                                   r_out, stream, &rc))
        return rc;
    // F = 5: vector staging per asset group (replay_gather_f5p_kernel, persistent; or
    // replay_gather_f5_kernel, one workgroup per sample); otherwise one workgroup per
    // sample with the W+1 staged days in LDS when they fit in 64 KiB, else one thread per
    // output float. Measured at S = 8,192, N = 30, W = 50: 96-102 us for the persistent
    // f5 form, 117 us one workgroup per sample, 204 us for the per-element staging
    // (tools/ab_replay.py, bench_rows.py)
    const size_t lds = (size_t)N * (W + 1) * F * sizeof(float);
    const bool al16 = ((uintptr_t)s & 15u) == 0 && ((uintptr_t)s_next & 15u) == 0 && ((uintptr_t)series & 15u) == 0;
    // F = 5 vector staging over asset groups of R rows: R divides N, R*W*F is a multiple
    // of 4 (16-B aligned groups), R*(W+1) <= 2,048 (day, asset) pairs (at most 8 per
    // thread); N = 30, W = 50: R = 30, one group per sample
    int R = 0;
    if (F == 5 && al16) {
        // the largest group within 2,048 pairs: whole samples measured faster than
        // 10-asset groups (131 vs 148 us at N = 30, W = 50) — every workgroup pays the
        // sample's dependent index loads once
        for (int r = N; r >= 1; --r)
            if (N % r == 0 && ((int64_t)r * W * F) % 4 == 0 && (int64_t)r * (W + 1) <= 2048 && r <= 256) {
                R = r;
                break;
            }
    }
    if (R > 0) {
        const FastDiv dr = make_fastdiv((uint32_t)R), dwf = make_fastdiv((uint32_t)(W * F));
        const size_t glds = (size_t)R * (W + 1) * F * sizeof(float);
        const int pairs = R * (W + 1);
        // s / s' are written once per sample: nt stores, 129.6 -> 118.6 us at S = 8,192
        // (tools/ab_replay.py, profiles/ab_r01/replay_nt_tpb_r01h.log). Persistent form
        // (replay_gather_f5p_kernel): one workgroup per CU loops over the samples with the
        // next sample's loads in flight. One per CU is the measured optimum (S = 8,192:
        // 96 us at 256 workgroups; 114-121 us at 192, 288, 512, 768, 1,280 and one
        // workgroup per sample, 117 us; profiles/ab_r01/replay_grid_r01j.log).
        static int cus = 0;
        if (!cus) {
            int dev = 0;
            if (hipGetDevice(&dev) != hipSuccess ||
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
                cus = 256;
        }
        const int gy = N / R;
        const int G = cus / gy > 0 ? cus / gy : 1;
        const dim3 pgrid((unsigned)(S < G ? S : G), (unsigned)(N / R));
        const int ppt = pairs <= 2 * 256 ? 2 : pairs <= 4 * 256 ? 4 : 8;
#define PMENV_RGP(PPT)                                                                                        \
    replay_gather_f5p_kernel<PPT, 2><<<pgrid, 256, glds, stream>>>(series, T, N, W, days, actions, rewards, H, B, \
                                                                   h0, env, S, s, s_next, a_out, r_out, R, dr, dwf)
        if (ppt == 2) PMENV_RGP(2); else if (ppt == 4) PMENV_RGP(4); else PMENV_RGP(8);
#undef PMENV_RGP
    } else if (lds <= 64 * 1024 && N <= 256 && ((uintptr_t)s & 15u) == 0 && ((uintptr_t)s_next & 15u) == 0) {
        replay_gather_lds_kernel<<<(unsigned)S, 256, lds, stream>>>(series, T, N, F, W, days, actions, rewards, H, B,
                                                                   h0, env, s, s_next, a_out, r_out);
    } else {
        const int64_t threads = (int64_t)S * N * W * F;
        replay_gather_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, stream>>>(
            series, T, N, F, W, days, actions, rewards, H, B, h0, env, S, s, s_next, a_out, r_out);
    }
    return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
}

int pmenv_rollout_gather(const float* series, int32_t T, int32_t N, int32_t F, int32_t W, const int32_t* start,
                         const float* weights, int32_t T_rec, int32_t B, int32_t ring_mode, const int32_t* t_idx,
                         const int32_t* env, int32_t S, float* s, hipStream_t stream) {
    if (!series || !start || (!weights && T_rec > 0) || !t_idx || !env || !s || T < 1 || N < 1 || F < 2 || W < 1 ||
        T_rec < 0 || B < 1 || S < 1 || ring_mode < 0 || ring_mode > 1)
        return PMENV_ERR_ARG;
    int rc = PMENV_OK;
    if (pmenv_tools::rollout_gather(series, T, N, F, W, start, weights, T_rec, B, ring_mode, t_idx, env, S, s,
                                    stream, &rc))
        return rc;
    const size_t lds = (size_t)W * N * F * sizeof(float);
    // market [W][N][4] + weights [W][N]; the tile's 16-B series loads and window stores need
    // 16-B aligned series / s (C callers may pass sliced views: those take the row form)
    const bool al16 = (((uintptr_t)series | (uintptr_t)s) & 15u) == 0;
    const bool tile = F == 5 && (N * W * F) % 4 == 0 && lds <= 64 * 1024 && al16;
    // the windows are written once and read by the learner later: nt stores (the tile's
    // bits unchanged), per call 29.0 -> 27.5 us at 4,096 samples, 235.1 -> 196.9 at 32,768,
    // 74.4 -> 54.3 at 8,192 from a 65,536 x 64 buffer; windows that fit well inside the
    // Infinity Cache (<= 128 MiB) take sc1 stores instead: 24.1-24.5 us at 4,096 samples
    // (123 MB), which lose 1.5-2x from 245 MB up (profiles/rows_r03ad/, rows_r03ae/)
    if (tile) {                                            // one workgroup per sample, staged in LDS
        const bool small = (size_t)S * N * W * F * sizeof(float) <= ((size_t)128 << 20);
        auto go = [&](auto kern) {
            kern<<<(unsigned)S, 256, lds, stream>>>(series, T, N, W, start, weights, B, ring_mode, t_idx, env, s,
                                                   make_fastdiv((uint32_t)N), make_fastdiv((uint32_t)(W * F)),
                                                   make_fastdiv((uint32_t)F));
        };
        if (small) go(rollout_gather_tile_kernel<16>);
        else go(rollout_gather_tile_kernel<2>);
        return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
    }
    const int64_t rows = (int64_t)S * N;                 // one wave per (sample, asset) row
    rollout_gather_rows_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, stream>>>(
        series, T, N, F, W, start, weights, B, ring_mode, t_idx, env, S, s, make_fastdiv((uint32_t)F));
    return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
}

int pmenv_metrics(const double* returns, const double* values, const float* weights, int32_t T, int32_t B, int32_t N,
                  double risk_free_rate, double periods, double* out, hipStream_t stream) {
    if (!returns || !values || !weights || !out || T < 1 || B < 1 || N < 1 || !(periods > 0.0)) return PMENV_ERR_ARG;
    int rc = PMENV_OK;
    if (pmenv_tools::metrics(returns, values, weights, T, B, N, risk_free_rate, periods, out, stream, &rc)) return rc;
    // measured on MI355X (tools/bench_rows.py): the segment walk (the horizon split over
    // four waves per 64 envs) beside the turnover stream, in one launch — against the
    // thread-per-env walk and the two-launch form (profiles/rows_r01*/)
    const int tpe = N <= 256 ? N : 256, eb = 256 / tpe;
    const int nseg = (B + 63) / 64, nturn = (B + eb - 1) / eb;
    metrics_fused_kernel<<<(unsigned)(nseg + nturn), 256, 0, stream>>>(returns, values, weights, T, B, N,
                                                                       risk_free_rate, periods, tpe, eb, nseg,
                                                                       nturn, 1, out);
    return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
}

size_t pmenv_batch_reward_workspace(int32_t B) { return B < 1 ? 0 : batch_reward_work_doubles(B) * 8; }

int pmenv_batch_reward_forward(const float* a, const float* v_prev, const float* p, int32_t B, int32_t N,
                               int32_t reward_kind, int32_t norm, double scale, double* work,
                               float* reward_out, float* ret_out, hipStream_t stream) {
    if (!a || !v_prev || !p || !work || !reward_out || B < 1 || N < 1) return PMENV_ERR_ARG;
    if (reward_kind != PMENV_REWARD_LOG_RETURN && reward_kind != PMENV_REWARD_RETURN &&
        reward_kind != PMENV_REWARD_SHARPE)
        return PMENV_ERR_ARG;
    if (norm < PMENV_BNORM_GLOBAL_OR || norm > PMENV_BNORM_NONE) return PMENV_ERR_ARG;
    int rc = PMENV_OK;
    if (pmenv_tools::batch_reward_forward(a, v_prev, p, B, N, reward_kind, norm, scale, work, reward_out, ret_out,
                                          stream, &rc))
        return rc;
    // at most 64 rows (the agents' BATCH_SIZE, config/pg.py:7): one workgroup, one launch
    if (B <= kQuadRows && N <= kQuadMaxN) {
        if (N <= 32)
            batch_reward_small_kernel<8><<<1, kTrainBlock, 0, stream>>>(a, v_prev, p, B, N, reward_kind, norm, scale,
                                                                         work, reward_out, ret_out);
        else
            batch_reward_small_kernel<16><<<1, kTrainBlock, 0, stream>>>(a, v_prev, p, B, N, reward_kind, norm, scale,
                                                                          work, reward_out, ret_out);
        return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
    }
    // two launches: the row blocks' partials, then the final fold (a one-launch form with a
    // last-block ticket measured slower at every shape: DESIGN.md §7 f2)
    int nparts;
    if (N <= kQuadMaxN) {         // a quad of lanes per row
        nparts = (B + kQuadRows - 1) / kQuadRows;
        if (N <= 32)
            batch_reward_rows_quad_kernel<8><<<(unsigned)nparts, kTrainBlock, 0, stream>>>(a, v_prev, p, B, N,
                                                                                           reward_kind, norm, work);
        else
            batch_reward_rows_quad_kernel<16><<<(unsigned)nparts, kTrainBlock, 0, stream>>>(a, v_prev, p, B, N,
                                                                                            reward_kind, norm, work);
    } else {                      // wave per row, registers up to N = 512
        nparts = (int)batch_reward_blocks(B);
        const unsigned g = (unsigned)nparts;
        if (N <= 128) batch_reward_rows_kernel<2><<<g, kTrainBlock, 0, stream>>>(a, v_prev, p, B, N, reward_kind, norm, work);
        else if (N <= 256) batch_reward_rows_kernel<4><<<g, kTrainBlock, 0, stream>>>(a, v_prev, p, B, N, reward_kind, norm, work);
        else if (N <= 512) batch_reward_rows_kernel<8><<<g, kTrainBlock, 0, stream>>>(a, v_prev, p, B, N, reward_kind, norm, work);
        else batch_reward_rows_kernel<0><<<g, kTrainBlock, 0, stream>>>(a, v_prev, p, B, N, reward_kind, norm, work);
    }
    batch_reward_final_kernel<<<1, kTrainBlock, 0, stream>>>(B, reward_kind, norm, scale, work, reward_out, nparts);
    // the chosen per-row return, when asked for (the backward takes each row's choice itself)
    if (ret_out) batch_reward_select_kernel<<<(B + 255) / 256, 256, 0, stream>>>(B, norm, work, ret_out);
    return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
}

int pmenv_batch_reward_backward(const float* a, const float* v_prev, const float* p, int32_t B, int32_t N,
                                int32_t reward_kind, double scale, const double* work, const float* grad_out,
                                float* grad_a, hipStream_t stream) {
    if (!a || !v_prev || !p || !work || !grad_out || !grad_a || B < 1 || N < 1) return PMENV_ERR_ARG;
    const unsigned qgrid = (unsigned)((B + kQuadRows - 1) / kQuadRows);
    if (N <= 32)
        batch_reward_grad_quad_kernel<8><<<qgrid, kTrainBlock, 0, stream>>>(a, v_prev, p, B, N, reward_kind, scale,
                                                                           work, grad_out, grad_a);
    else if (N <= kQuadMaxN)
        batch_reward_grad_quad_kernel<16><<<qgrid, kTrainBlock, 0, stream>>>(a, v_prev, p, B, N, reward_kind, scale,
                                                                            work, grad_out, grad_a);
    else if (N <= 128)
        batch_reward_grad_kernel<2><<<(B + 3) / 4, 256, 0, stream>>>(a, v_prev, p, B, N, reward_kind, scale, work,
                                                                     grad_out, grad_a);
    else if (N <= 256)
        batch_reward_grad_kernel<4><<<(B + 3) / 4, 256, 0, stream>>>(a, v_prev, p, B, N, reward_kind, scale, work,
                                                                     grad_out, grad_a);
    else if (N <= 512)
        batch_reward_grad_kernel<8><<<(B + 3) / 4, 256, 0, stream>>>(a, v_prev, p, B, N, reward_kind, scale, work,
                                                                     grad_out, grad_a);
    else
        batch_reward_grad_kernel<0><<<(B + 3) / 4, 256, 0, stream>>>(a, v_prev, p, B, N, reward_kind, scale, work,
                                                                     grad_out, grad_a);
    return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
}

}  // extern "C"

// ---------------------------------------------------------------- tools-build hooks
// The product library's hooks do nothing; tools/ab/pmenv_ab.hip (linked only into
// tools/libpmenv_ab.so) overrides these weak definitions.
namespace pmenv_tools {
__attribute__((weak, noinline)) void plan(pmenv*) {}
__attribute__((weak, noinline)) void release(pmenv*) {}
__attribute__((weak, noinline)) bool launch_scalar(const pmenv*, const StepParams&, hipStream_t) { return false; }
__attribute__((weak, noinline)) bool launch_advance(const pmenv*, const StepParams&, hipStream_t) { return false; }
__attribute__((weak, noinline)) bool launch_one(const pmenv*, const StepParams&, hipStream_t) { return false; }
__attribute__((weak, noinline)) bool launch_small(const pmenv*, const StepParams&, hipStream_t) { return false; }
__attribute__((weak, noinline)) bool launch_gen(const pmenv*, const StepParams&, hipStream_t) { return false; }
__attribute__((weak, noinline)) bool launch_fused(const pmenv*, const StepParams&, int, uint32_t, hipStream_t) {
    return false;
}
__attribute__((weak, noinline)) bool launch_relay(const pmenv*, const StepParams&, const RelayParams&, unsigned,
                                                  hipStream_t) {
    return false;
}
__attribute__((weak, noinline)) bool launch_flat1(const pmenv*, const StepParams&, unsigned, bool, int,
                                                  hipStream_t) {
    return false;
}
__attribute__((weak, noinline)) bool gae(const float*, const float*, const uint8_t*, float*, float*, int32_t,
                                         int32_t, float, float, hipStream_t, int*) {
    return false;
}
__attribute__((weak, noinline)) bool replay_gather(const float*, int32_t, int32_t, int32_t, int32_t, const int32_t*,
                                                   const float*, const float*, int32_t, int32_t, const int32_t*,
                                                   const int32_t*, int32_t, float*, float*, float*, float*,
                                                   hipStream_t, int*) {
    return false;
}
__attribute__((weak, noinline)) bool rollout_gather(const float*, int32_t, int32_t, int32_t, int32_t, const int32_t*,
                                                    const float*, int32_t, int32_t, int32_t, const int32_t*,
                                                    const int32_t*, int32_t, float*, hipStream_t, int*) {
    return false;
}
__attribute__((weak, noinline)) bool metrics(const double*, const double*, const float*, int32_t, int32_t, int32_t,
                                             double, double, double*, hipStream_t, int*) {
    return false;
}
__attribute__((weak, noinline)) bool batch_reward_forward(const float*, const float*, const float*, int32_t, int32_t,
                                                          int32_t, int32_t, double, double*, float*, float*,
                                                          hipStream_t, int*) {
    return false;
}
}  // namespace pmenv_tools
