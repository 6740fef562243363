// pmenv.hip — host side and C ABI (include/pmenv.h) of the MI355X-native
// vectorised portfolio environment. Device code lives in step_env.h (the one-launch
// step), env_step.h (scalar step, window streams, reset, fallbacks), scalar_vec.h
// (packed scalar step), data.h (synthetic market data), rollout.h / gae_vec.h (GAE,
// moments), replay.h (replay gather, metrics) and trainer.h (batched reward).
//
// Every entry point enqueues on the caller's stream and never synchronises,
// allocates or frees (graph-capturable), except create / destroy / the explicit
// synchronous queries documented in the header.
//
// Kernel choice is a function of the shape only (and of pmenv_set_step_path). The
// A/B variants measured while choosing — other geometries, cache policies, the
// timing-only ablations that skip work — exist only in the tools build
// (-DPMENV_AB -> tools/libpmenv_ab.so), which alone reads the PMENV_* knobs.
#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/pmenv.h"
#include "common.h"
#include "data.h"
#include "env_step.h"
#include "scalar_vec.h"
#include "step_env.h"
#include "step_flat.h"
#include "rollout.h"
#include "gae_vec.h"
#include "replay.h"
#include "trainer.h"

using namespace pmenv_dev;

#ifdef PMENV_AB
static const char* ab_knob(const char* name) { return getenv(name); }
static int ab_int(const char* name, int dflt) {
    const char* v = getenv(name);
    return v ? atoi(v) : dflt;
}
#else
static inline const char* ab_knob(const char*) { return nullptr; }
static inline int ab_int(const char*, int dflt) { return dflt; }
#endif

struct pmenv {
    pmenv_cfg cfg;
    int device;
    void* state;          // value | stat_a | stat_b | counter | ring | nonfinite | last_close | w_new
    size_t state_bytes;
    bool owns_state;
    double* value;
    double* sa;
    double* sb;
    int32_t* k;
    float* ring;
    float* last_close;
    float* w_new;
    unsigned long long* nonfinite;
    // LDS single-launch fallback geometry
    int rows_per_tile, tile_floats;
    bool vec;
    size_t lds_tile, lds_surface;
    // two-launch streaming path geometry
    bool streaming;       // scalar step kernel + window stream
    int unit_rows, units_per_env, stream_vec;          // row-kernel advance in place
    int unit_rows_db, units_per_env_db, stream_vec_db; // row-kernel advance double-buffered (obs_out)
    int stream_block, stream_block_db;                 // threads per row-kernel workgroup (tools: 128 | 256)
    int stream_pol;       // cache policy of the row kernel
    bool flat;            // double-buffered advance as the flat 16-B stream
    int flat_block, flat_pol, flat_ip_pol;   // cache policy: double-buffered / in-place stream
    bool flat_inplace;    // in-place advance as the flat stream + halo (advance_flat_inplace_kernel)
    int flat_ip_block, flat_ip_vec;   // threads per workgroup, chunks per thread
    bool flat_db_wg;      // double-buffered flat stream in the workgroup form (tools: ds_bpermute form)
    float* halo;          // [halo_wgs][2] float4: first two chunks of every in-place flat workgroup
    uint32_t halo_wgs, flat_qtot;
    int scalar_scratch_floats;
    int k1_groups;        // env groups per wave in scalar_step_reg_kernel
    int k1_vec;           // scalar_step_vec_kernel shape 100 * L + A (0: register / LDS form)
    // one launch per step
    bool one_ok;          // the shape fits step_env_kernel
    int one_auto;         // PMENV_FUSE_* bits the automatic choice gives step_env_kernel
    int one;              // PMENV_FUSE_* bits: which windows take step_env_kernel now
    int one_v, one_waves; // step_env_kernel: chunks per lane, waves per workgroup
    uint32_t per4;        // 16-B chunks per env window
    // one launch over the flat stream (step_flat_kernel)
    bool flat1_ok;        // the shape fits step_flat_kernel
    int flat1_auto;       // PMENV_FUSE_* bits the automatic choice gives step_flat_kernel
    int flat1;            // PMENV_FUSE_* bits: which windows take step_flat_kernel now
    void* snap;           // the state snapshot, two parities: value f64 | counter i32 | get_last() | last close
    double* sv[2];
    int32_t* sk[2];
    float* sw[2];
    float* slc[2];
    float* halo1[2];      // [halo1_wgs][2] float4 per parity: the next tile's first two chunks
    uint32_t halo1_wgs;
    int flat1_block, flat1_vec;   // threads per workgroup, chunks per thread (tools: PMENV_FLAT1_GEOM)
    bool flat1_xcd;               // tools: XCD-contiguous tile ranges (PMENV_FLAT1_XCD)
    int flat1_pol;                // tools: 3 nt loads only, 4 nt stores only, 5 sc0 nt, 6 sc1 nt, 7 nt loads + sc1 nt stores
    int par;              // parity of the snapshot / halo the next step reads
    bool snap_ok;         // sv[par] .. slc[par] equal the canonical state
    const float* halo1_obs;   // the window whose halo halo1[par] holds (null: none)
    // device-sequenced form (hipGraph-safe): from the first flat step enqueued under
    // stream capture on, every flat step is flat_seq_kernel + step_flat_kernel reading
    // the parity and the validity from seq (device words) instead of the host fields above
    bool device_seq;
    int32_t* seq;         // {D, C, V, pad, HOBS lo, HOBS hi} (step_flat.h)
    uint64_t snap_stride; // bytes between the two parities of the snapshot / halo
    int path;             // pmenv_step_path_kind
    // tools build only
    int fused;            // PMENV_FUSE_* bits: advance_rows_kernel<fused> (PMENV_FUSED)
    int fused_vec;
    int ablate;           // PMENV_ABLATE timing-only variants
    bool one_nocap, flat_s80;
    int flat1_lds_pad;
    size_t lds_scalar, lds_stream;
    char err[512];
};

namespace {

thread_local char g_create_err[512] = "";

void set_err(pmenv* h, const char* fmt, ...) {
    if (!h) return;
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(h->err, sizeof(h->err), fmt, ap);
    va_end(ap);
}

struct DeviceGuard {
    int prev = -1;
    bool changed = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) == hipSuccess && prev != dev) changed = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (changed) (void)hipSetDevice(prev);
    }
};

StepParams base_params(const pmenv* h) {
    StepParams p;
    memset(&p, 0, sizeof(p));
    const pmenv_cfg& c = h->cfg;
    p.B = c.num_envs; p.N = c.num_assets; p.W = c.window; p.F = c.features;
    p.close_ch = c.close_channel;
    p.reward_kind = c.reward_kind; p.norm_mode = c.norm_mode; p.ring_mode = c.ring_mode;
    p.ret_mode = c.ret_mode; p.mu_max_iter = c.mu_max_iter;
    p.rows_per_tile = h->rows_per_tile;
    p.tile_floats = h->tile_floats;
    p.unit_rows = h->unit_rows;
    p.units_per_env = h->units_per_env;
    p.init_cash = c.init_cash; p.commission = c.commission; p.scale = c.reward_scale;
    p.rf = c.risk_free_rate; p.eta = c.sharpe_eta; p.mu_tol = c.mu_tol;
    p.value = h->value; p.k = h->k; p.ring = h->ring; p.last_close = h->last_close;
    p.w_new = h->w_new;
    p.sa = h->sa; p.sb = h->sb;
    p.nonfinite = h->nonfinite;
    p.div_wf = make_fastdiv((uint32_t)(c.window * c.features));
    p.div_f = make_fastdiv((uint32_t)c.features);
    p.div_w = make_fastdiv((uint32_t)c.window);
    p.div_units = make_fastdiv((uint32_t)(h->units_per_env > 0 ? h->units_per_env : 1));
    return p;
}

inline bool aligned4(const void* ptr) { return ((uintptr_t)ptr & 3u) == 0; }

int check_launch(pmenv* h, const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_err(h, "%s launch failed: %s", what, hipGetErrorString(e));
        return PMENV_ERR_HIP;
    }
    return PMENV_OK;
}

constexpr int PMENV_FUSE_DB = 1, PMENV_FUSE_INPLACE = 2;

// Geometry of the row-kernel stream (the fallback of the flat stream): units of R
// whole asset rows per `block`-thread workgroup, R*W*F floats <= 4*block*V (V float4
// per thread) and R*W*F % 4 == 0 so every unit starts 16-B aligned. `v_order` lists V
// in preference order. Returns false when the shape needs the LDS fallback.
bool plan_streaming(const pmenv_cfg& c, const int* v_order, int block, int* unit_rows, int* vec_per_thread) {
    const int64_t WF = (int64_t)c.window * c.features;
    if (c.features != 5 || ((int64_t)c.num_assets * WF) % 4 != 0) return false;
    int align = 1;                       // rows per unit must be a multiple of this
    while ((align * WF) % 4 != 0) ++align;
    const int want = ab_int("PMENV_UNIT_ROWS", 0);
    static const int kAscending[3] = {1, 2, 4};
    if (want > 0) v_order = kAscending;   // a forced unit takes the fewest float4 per thread that hold it
    for (int vi = 0; vi < 3; ++vi) {
        const int V = v_order[vi];
        const int64_t cap = (int64_t)block * 4 * V;
        int R = (int)(cap / WF);
        if (R >= c.num_assets) R = c.num_assets;
        else R -= R % align;
        if (R < 1 || (int64_t)R * WF > cap) continue;
        if (want > 0) {
            if (want > R) continue;
            if (want != c.num_assets && want % align) return false;
            R = want;
        }
        *unit_rows = R;
        *vec_per_thread = V;
        return true;
    }
    return false;
}

// ---------------------------------------------------------------- launchers
// the row-kernel stream (fallback of the flat stream: W = 1, or windows past 2^31 chunks)
template <int BLOCK, int V, int ABL, int POL>
void launch_advance_bv(const StepParams& p, unsigned grid, hipStream_t stream) {
    if (p.obs_out == p.obs)
        advance_rows_kernel<BLOCK, V, true, ABL, false, POL><<<grid, BLOCK, 0, stream>>>(p);
    else
        advance_rows_kernel<BLOCK, V, false, ABL, false, POL><<<grid, BLOCK, 0, stream>>>(p);
}

template <int BLOCK, int ABL, int POL>
void launch_advance_b(int vec, const StepParams& p, unsigned grid, hipStream_t stream) {
    if (vec == 1) launch_advance_bv<BLOCK, 1, ABL, POL>(p, grid, stream);
    else if (vec == 2) launch_advance_bv<BLOCK, 2, ABL, POL>(p, grid, stream);
    else launch_advance_bv<BLOCK, 4, ABL, POL>(p, grid, stream);
}

template <int POL>
void launch_advance_p(int block, int vec, const StepParams& p, unsigned grid, hipStream_t stream) {
#ifdef PMENV_AB
    if (block == 128) { launch_advance_b<128, 0, POL>(vec, p, grid, stream); return; }
    if (block == 256) { launch_advance_b<256, 0, POL>(vec, p, grid, stream); return; }
#endif
    (void)block;
    launch_advance_b<kStreamBlock, 0, POL>(vec, p, grid, stream);
}

// the double-buffered flat stream: the workgroup (LDS) form, 512 threads x 2 chunks
void launch_flat(const pmenv* h, StepParams p, hipStream_t stream) {
    const pmenv_cfg& c = h->cfg;
    const uint32_t per4 = (uint32_t)((int64_t)c.num_assets * c.window * c.features / 4);
    const uint32_t qtot = (uint32_t)((int64_t)c.num_envs * per4);
    p.div_units = make_fastdiv(per4);
#ifdef PMENV_AB
    if (!h->flat_db_wg) {        // the ds_bpermute form, one chunk per thread
        const int bk = h->flat_block;
        const unsigned grid = (unsigned)((qtot + bk - 1) / bk);
#define PMENV_FLATB(BK)                                                                             \
        if (bk == BK) {                                                                             \
            if (h->flat_pol == 1) advance_flat_kernel<BK, 1><<<grid, BK, 0, stream>>>(p, qtot);      \
            else if (h->flat_pol == 2) advance_flat_kernel<BK, 2><<<grid, BK, 0, stream>>>(p, qtot); \
            else advance_flat_kernel<BK, 0><<<grid, BK, 0, stream>>>(p, qtot);                       \
            return;                                                                                 \
        }
        PMENV_FLATB(128) PMENV_FLATB(512) PMENV_FLATB(256)
#undef PMENV_FLATB
    }
    if (h->flat_pol == 2) {
        advance_flat_wg_kernel<512, 2, 2><<<(unsigned)((qtot + 1023) / 1024), 512, 0, stream>>>(p, qtot);
        return;
    }
#endif
    const unsigned g = (unsigned)((qtot + 1023) / 1024);
    if (h->flat_pol == 0) advance_flat_wg_kernel<512, 2, 0><<<g, 512, 0, stream>>>(p, qtot);
    else advance_flat_wg_kernel<512, 2, 1><<<g, 512, 0, stream>>>(p, qtot);
}

// the in-place flat stream: 512 threads x 2 chunks, the halo copied by the scalar step
void launch_flat_inplace(const pmenv* h, StepParams p, hipStream_t stream) {
    const pmenv_cfg& c = h->cfg;
    const uint32_t per4 = (uint32_t)((int64_t)c.num_assets * c.window * c.features / 4);
    p.div_units = make_fastdiv(per4);
    p.halo = h->halo;
    const int cpw = h->flat_ip_block * h->flat_ip_vec;
    const unsigned grid = (unsigned)((h->flat_qtot + cpw - 1) / cpw);
#ifdef PMENV_AB
    const int key = h->flat_ip_block * 10 + h->flat_ip_vec;
    const int pol = h->flat_ip_pol;
    if (h->ablate >= 64 && h->ablate < 128) {     // timing-only ablations (PMENV_ABLATE = 64 + SKIP bits)
        const unsigned g1 = (unsigned)((h->flat_qtot + 511) / 512);
#define PMENV_ABL(X) case 64 + X: advance_flat_inplace_kernel<512, 1, 1, X><<<g1, 512, 0, stream>>>(p, h->flat_qtot); break;
        switch (h->ablate) {
            PMENV_ABL(1) PMENV_ABL(2) PMENV_ABL(4) PMENV_ABL(6) PMENV_ABL(15) PMENV_ABL(31) PMENV_ABL(32)
            PMENV_ABL(33)
            default: break;
        }
#undef PMENV_ABL
        return;
    }
    if (h->flat_s80 && key == 5122) {
        if (pol == 1) advance_flat_inplace_s80_kernel<512, 2, 1><<<grid, 512, 0, stream>>>(p, h->flat_qtot);
        else advance_flat_inplace_s80_kernel<512, 2, 0><<<grid, 512, 0, stream>>>(p, h->flat_qtot);
        return;
    }
#define PMENV_FIP(BK, V)                                                                                      \
    if (key == BK * 10 + V) {                                                                                 \
        if (pol == 1) advance_flat_inplace_kernel<BK, V, 1><<<grid, BK, 0, stream>>>(p, h->flat_qtot);         \
        else if (pol == 2) advance_flat_inplace_kernel<BK, V, 2><<<grid, BK, 0, stream>>>(p, h->flat_qtot);    \
        else advance_flat_inplace_kernel<BK, V, 0><<<grid, BK, 0, stream>>>(p, h->flat_qtot);                  \
        return;                                                                                               \
    }
    PMENV_FIP(256, 1) PMENV_FIP(256, 2) PMENV_FIP(256, 4) PMENV_FIP(512, 1) PMENV_FIP(1024, 1)
#undef PMENV_FIP
#endif
    if (h->flat_ip_block == 256) advance_flat_inplace_kernel<256, 2, 0><<<grid, 256, 0, stream>>>(p, h->flat_qtot);
    else if (h->flat_ip_pol == 1) advance_flat_inplace_kernel<512, 2, 1><<<grid, 512, 0, stream>>>(p, h->flat_qtot);
    else advance_flat_inplace_kernel<512, 2, 0><<<grid, 512, 0, stream>>>(p, h->flat_qtot);
}

// the second launch of the two-launch step
void launch_advance(const pmenv* h, StepParams p, hipStream_t stream) {
    const bool db = p.obs_out != p.obs;
    if (db && h->flat && !h->ablate) {
        launch_flat(h, p, stream);
        return;
    }
    if (!db && h->flat_inplace && (!h->ablate || (h->ablate >= 64 && h->ablate < 128))) {
        launch_flat_inplace(h, p, stream);
        return;
    }
    p.unit_rows = db ? h->unit_rows_db : h->unit_rows;
    p.units_per_env = db ? h->units_per_env_db : h->units_per_env;
    p.div_units = make_fastdiv((uint32_t)p.units_per_env);
    const int vec = db ? h->stream_vec_db : h->stream_vec;
    const int block = db ? h->stream_block_db : h->stream_block;
    const unsigned grid = (unsigned)(h->cfg.num_envs * p.units_per_env);
#ifdef PMENV_AB
    switch (h->ablate) {     // timing-only builds: 512-thread geometry, default policy
    case 1: launch_advance_b<kStreamBlock, 1, 0>(vec, p, grid, stream); return;
    case 2: launch_advance_b<kStreamBlock, 2, 0>(vec, p, grid, stream); return;
    case 3: launch_advance_b<kStreamBlock, 3, 0>(vec, p, grid, stream); return;
    case 7: launch_advance_b<kStreamBlock, 7, 0>(vec, p, grid, stream); return;
    default: break;
    }
    if (h->stream_pol == 2) { launch_advance_p<2>(block, vec, p, grid, stream); return; }
#endif
    if (h->stream_pol == 1) launch_advance_p<1>(block, vec, p, grid, stream);
    else launch_advance_p<0>(block, vec, p, grid, stream);
}

// K1, the first launch of the two-launch step: the register form (N <= 64)
template <int L>
void launch_scalar_reg_l(int groups, const StepParams& p, hipStream_t stream) {
    const int per_wave = (64 / L) * groups;
    const unsigned waves = (unsigned)((p.B + per_wave - 1) / per_wave);
    const unsigned grid = (waves + 3) / 4;
#ifdef PMENV_AB
    if (groups == 4) { scalar_step_reg_kernel<L, 4><<<grid, 256, 0, stream>>>(p); return; }
    if (groups == 2) { scalar_step_reg_kernel<L, 2><<<grid, 256, 0, stream>>>(p); return; }
#endif
    scalar_step_reg_kernel<L, 1><<<grid, 256, 0, stream>>>(p);
}

void launch_scalar_reg(const pmenv* h, const StepParams& p, hipStream_t stream) {
    if (p.N <= 32) launch_scalar_reg_l<32>(h->k1_groups, p, stream);
    else launch_scalar_reg_l<64>(h->k1_groups, p, stream);
}

// K1 packed form (scalar_vec.h): L lanes x A assets per env, consecutive or strided
// (STR); h->k1_vec = 100 * L + A (+ kK1Str for the strided layout)
constexpr int kK1Str = 100000;

template <int L, int A, bool STR>
void launch_scalar_vec_la(const StepParams& p, hipStream_t stream) {
    const unsigned waves = (unsigned)((p.B + 64 / L - 1) / (64 / L));
    scalar_step_vec_kernel<L, A, STR><<<(waves + 3) / 4, 256, 0, stream>>>(p);
}

bool launch_scalar_vec(int vec, const StepParams& p, hipStream_t stream) {
    switch (vec) {   // the shapes pick_k1_vec chooses per asset count (N > 64)
    case kK1Str + 6402: launch_scalar_vec_la<64, 2, true>(p, stream); return true;
    case kK1Str + 6404: launch_scalar_vec_la<64, 4, true>(p, stream); return true;
    case kK1Str + 6408: launch_scalar_vec_la<64, 8, true>(p, stream); return true;
#ifdef PMENV_AB
    case 801: launch_scalar_vec_la<8, 1, false>(p, stream); return true;
    case 802: launch_scalar_vec_la<8, 2, false>(p, stream); return true;
    case 1602: launch_scalar_vec_la<16, 2, false>(p, stream); return true;
    case 1604: launch_scalar_vec_la<16, 4, false>(p, stream); return true;
    case 804: launch_scalar_vec_la<8, 4, false>(p, stream); return true;
    case 1601: launch_scalar_vec_la<16, 1, false>(p, stream); return true;
    case 1608: launch_scalar_vec_la<16, 8, false>(p, stream); return true;
    case 3202: launch_scalar_vec_la<32, 2, false>(p, stream); return true;
    case 3204: launch_scalar_vec_la<32, 4, false>(p, stream); return true;
    case kK1Str + 3202: launch_scalar_vec_la<32, 2, true>(p, stream); return true;
    case kK1Str + 3204: launch_scalar_vec_la<32, 4, true>(p, stream); return true;
#endif
    default: return false;
    }
}

// K1 shape per asset count (tools build: the PMENV_K1 knob "reg" | "LxA" | "LxAs"
// strided, e.g. "16x2", "64x8s"). 0: the register form (N <= 64) or the LDS form (N > 512).
// N <= 64 takes the register form: its reductions (one asset per lane, DPP row shifts,
// the fixed-order row combine) are bitwise those of the one-launch step's scalar part,
// so the two paths — and therefore sharded and unsharded runs, whose path can differ
// by env count — give the same bits. It costs 4.6 us at 65,536 envs over the packed
// 16 x 2 form (29.1 vs 24.5 us), and the two-launch path runs for N <= 64 only on
// cache-resident in-place windows (<= 8,192 envs at N = 30): < 1 us per step.
int pick_k1_vec(const pmenv_cfg& c) {
    const int N = c.num_assets;
    if ((int64_t)c.num_envs * N * 4 >= (1ll << 32)) return 0;     // descriptors span the [B*N] arrays
    int v = 0;
#ifdef PMENV_AB
    if (N <= 8) v = 801;
    else if (N <= 16) v = 802;
    else if (N <= 32) v = 1602;
    else if (N <= 64) v = 1604;
    else
#endif
    if (N <= 64) v = 0;
    else if (N <= 128) v = kK1Str + 6402;
    else if (N <= 256) v = kK1Str + 6404;
    else if (N <= 512) v = kK1Str + 6408;
    if (const char* knob = ab_knob("PMENV_K1")) {
        static const int kK1Vec[] = {801, 802, 804, 1601, 1602, 1604, 1608, 3202, 3204,
                                     kK1Str + 3202, kK1Str + 3204, kK1Str + 6402, kK1Str + 6404, kK1Str + 6408};
        int L = 0, A = 0;
        char s = 0;
        if (!strcmp(knob, "reg")) return 0;
        if (sscanf(knob, "%dx%d%c", &L, &A, &s) >= 2) {
            const int want = 100 * L + A + (s == 's' ? kK1Str : 0);
            for (int k : kK1Vec)
                if (k == want && L * A >= N) return k;
        }
    }
    return v;
}

// the first launch of the two-launch step (with the in-place stream's halo copy)
int launch_scalar(pmenv* h, StepParams p, hipStream_t stream) {
    if (p.obs_out == p.obs && h->flat_inplace && !h->ablate) {   // the in-place advance's halo
        p.halo = h->halo;
        p.halo_wgs = h->halo_wgs;
        p.halo_block = (uint32_t)(h->flat_ip_block * h->flat_ip_vec);
        p.halo_qtot = h->flat_qtot;
    }
    const int N = h->cfg.num_assets;
    if (h->k1_vec && launch_scalar_vec(h->k1_vec, p, stream)) {
        // packed form
    } else if (N <= 64) {
        launch_scalar_reg(h, p, stream);
    } else {
        const int B = h->cfg.num_envs;
        scalar_step_kernel<<<(B + kScalarWaves - 1) / kScalarWaves, 64 * kScalarWaves, h->lds_scalar, stream>>>(
            p, h->scalar_scratch_floats);
    }
    return check_launch(h, "scalar_step_kernel");
}

// the whole step in one launch, one workgroup per env (step_env.h)
template <int V>
void launch_one_v(const pmenv* h, const StepParams& p, hipStream_t stream) {
    const bool out = p.obs_out != p.obs;
    const int pol = out ? h->flat_pol : h->flat_ip_pol;
    const unsigned threads = 64u * (unsigned)h->one_waves;
    size_t lds = ((size_t)threads * V + 2) * 16;
    const unsigned grid = (unsigned)h->cfg.num_envs;
#ifdef PMENV_AB
    lds += (size_t)ab_int("PMENV_ONE_LDS_PAD", 0);    // occupancy study: fewer workgroups per CU
    if (h->ablate >= 128 && h->ablate < 144) {    // timing-only / A/B bits (step_env.h ABL), nt policy
#define PMENV_ONEABL(X)                                                                                     \
        case 128 + X:                                                                                     \
            if (out) step_env_kernel<V, true, 1, X><<<grid, threads, lds, stream>>>(p, h->per4);            \
            else step_env_kernel<V, false, 1, X><<<grid, threads, lds, stream>>>(p, h->per4);               \
            return;
        switch (h->ablate) {
            PMENV_ONEABL(1) PMENV_ONEABL(2) PMENV_ONEABL(4) PMENV_ONEABL(8) PMENV_ONEABL(12)
            default: break;
        }
#undef PMENV_ONEABL
    }
    if (h->one_nocap) {
        if (out && pol == 1) step_env_nocap_kernel<V, true, 1><<<grid, threads, lds, stream>>>(p, h->per4);
        else if (out) step_env_nocap_kernel<V, true, 0><<<grid, threads, lds, stream>>>(p, h->per4);
        else if (pol == 1) step_env_nocap_kernel<V, false, 1><<<grid, threads, lds, stream>>>(p, h->per4);
        else step_env_nocap_kernel<V, false, 0><<<grid, threads, lds, stream>>>(p, h->per4);
        return;
    }
#endif
    if (out) {
        if (pol == 1) step_env_kernel<V, true, 1><<<grid, threads, lds, stream>>>(p, h->per4);
        else step_env_kernel<V, true, 0><<<grid, threads, lds, stream>>>(p, h->per4);
    } else {
        if (pol == 1) step_env_kernel<V, false, 1><<<grid, threads, lds, stream>>>(p, h->per4);
        else step_env_kernel<V, false, 0><<<grid, threads, lds, stream>>>(p, h->per4);
    }
}

void launch_one(const pmenv* h, const StepParams& p, hipStream_t stream) {
#ifdef PMENV_AB
    switch (h->one_v) {
    case 1: launch_one_v<1>(h, p, stream); return;
    case 2: launch_one_v<2>(h, p, stream); return;
    case 3: launch_one_v<3>(h, p, stream); return;
    case 6: launch_one_v<6>(h, p, stream); return;
    case 8: launch_one_v<8>(h, p, stream); return;
    default: break;
    }
#endif
    launch_one_v<4>(h, p, stream);
}

#ifdef PMENV_AB
// tools build: the previous one-launch form (whole-env row units, scalar step inside)
void launch_fused(const pmenv* h, StepParams p, hipStream_t stream) {
    p.unit_rows = h->cfg.num_assets;
    p.units_per_env = 1;
    p.div_units = make_fastdiv(1u);
    const unsigned grid = (unsigned)h->cfg.num_envs;
    const bool inplace = p.obs_out == p.obs;
#define PMENV_FUSED_LAUNCH(V)                                                                        \
    if (inplace) advance_rows_kernel<kStreamBlock, V, true, 0, true><<<grid, kStreamBlock, 0, stream>>>(p); \
    else advance_rows_kernel<kStreamBlock, V, false, 0, true><<<grid, kStreamBlock, 0, stream>>>(p);
    if (h->fused_vec == 1) { PMENV_FUSED_LAUNCH(1) }
    else if (h->fused_vec == 2) { PMENV_FUSED_LAUNCH(2) }
    else { PMENV_FUSED_LAUNCH(4) }
#undef PMENV_FUSED_LAUNCH
}
#endif

// step_flat_vec_kernel (64 < N <= 512): A strided assets per lane, as pick_k1_vec's
// packed two-launch scalar step, so the two paths give the same bits
template <int A, int BK, int VV>
void launch_flat1_vec_g(const StepParams& p, uint32_t qtot, unsigned grid, bool out, int pol, hipStream_t stream) {
    if (out) {
        if (pol == 1) step_flat_vec_kernel<A, BK, VV, 1, true><<<grid, BK, 0, stream>>>(p, qtot);
        else step_flat_vec_kernel<A, BK, VV, 0, true><<<grid, BK, 0, stream>>>(p, qtot);
    } else {
        if (pol == 1) step_flat_vec_kernel<A, BK, VV, 1, false><<<grid, BK, 0, stream>>>(p, qtot);
        else step_flat_vec_kernel<A, BK, VV, 0, false><<<grid, BK, 0, stream>>>(p, qtot);
    }
}

template <int A>
void launch_flat1_vec_a(const pmenv* h, const StepParams& p, unsigned grid, bool out, int pol, hipStream_t stream) {
#ifdef PMENV_AB
    if (h->flat1_block == 128) { launch_flat1_vec_g<A, 128, 8>(p, h->flat_qtot, grid, out, pol, stream); return; }
#endif
    launch_flat1_vec_g<A, 256, 4>(p, h->flat_qtot, grid, out, pol, stream);
}

void launch_flat1_vec(const pmenv* h, const StepParams& p, unsigned grid, bool out, int pol, hipStream_t stream) {
    const int N = h->cfg.num_assets;
    if (N <= 128) launch_flat1_vec_a<2>(h, p, grid, out, pol, stream);
    else if (N <= 256) launch_flat1_vec_a<4>(h, p, grid, out, pol, stream);
    else launch_flat1_vec_a<8>(h, p, grid, out, pol, stream);
}

// the whole step in one launch over the flat stream (step_flat.h): prime the snapshot
// and the halo when something other than this kernel touched them, then one launch
void launch_flat1(pmenv* h, StepParams p, hipStream_t stream) {
    const bool out = p.obs_out != p.obs;
    const int q = h->par;
    p.per4 = h->per4;
    p.div_units = make_fastdiv(h->per4);
    const bool need_halo = !out && h->halo1_obs != p.obs;
    if (h->device_seq) {
        // parity 0 in *_in / halo_in, parity 1 in *_out / halo_out; the sequencer primes
        // parity D if needed and publishes it, the kernel swaps when it is 1
        p.sv_in = h->sv[0]; p.sk_in = h->sk[0]; p.sw_in = h->sw[0]; p.slc_in = h->slc[0];
        p.sv_out = h->sv[1]; p.sk_out = h->sk[1]; p.sw_out = h->sw[1]; p.slc_out = h->slc[1];
        p.halo_in = h->halo1[0];
        p.halo_out = h->halo1[1];
        p.seq = h->seq;
        StepParams pp = p;
        pp.sv_out = h->sv[0]; pp.sk_out = h->sk[0]; pp.sw_out = h->sw[0]; pp.slc_out = h->slc[0];
        pp.halo = h->halo1[0];
        pp.halo_wgs = h->halo1_wgs;
        pp.halo_block = (uint32_t)(h->flat1_block * h->flat1_vec);
        pp.halo_qtot = h->flat_qtot;
        const int64_t work = (int64_t)h->cfg.num_envs * h->cfg.num_assets;
        const unsigned g = (unsigned)(work / 256 + 1 < 2048 ? work / 256 + 1 : 2048);
        flat_seq_kernel<<<g, 256, 0, stream>>>(pp, out ? 1 : 0, h->snap_stride);
    } else if (!h->snap_ok || need_halo) {
        StepParams pp = p;
        pp.sv_out = h->sv[q]; pp.sk_out = h->sk[q]; pp.sw_out = h->sw[q]; pp.slc_out = h->slc[q];
        pp.halo = need_halo ? h->halo1[q] : nullptr;
        pp.halo_wgs = h->halo1_wgs;
        pp.halo_block = (uint32_t)(h->flat1_block * h->flat1_vec);
        pp.halo_qtot = h->flat_qtot;
        const int64_t work = (int64_t)h->cfg.num_envs * h->cfg.num_assets;
        const unsigned g = (unsigned)(work / 256 + 1 < 2048 ? work / 256 + 1 : 2048);
        flat_prime_kernel<<<g, 256, 0, stream>>>(pp);
    }
    if (!h->device_seq) {
        p.sv_in = h->sv[q]; p.sk_in = h->sk[q]; p.sw_in = h->sw[q]; p.slc_in = h->slc[q];
        p.sv_out = h->sv[1 - q]; p.sk_out = h->sk[1 - q]; p.sw_out = h->sw[1 - q]; p.slc_out = h->slc[1 - q];
        p.halo_in = h->halo1[q];
        p.halo_out = h->halo1[1 - q];
    }
    const int pol = out ? h->flat_pol : h->flat_ip_pol;
    const unsigned grid = (h->flat_qtot + (uint32_t)(h->flat1_block * h->flat1_vec) - 1) /
                          (uint32_t)(h->flat1_block * h->flat1_vec);
    if (h->cfg.num_assets > 64) {                 // wide envs: the packed scalar step per tile
        launch_flat1_vec(h, p, grid, out, pol, stream);
        h->par = 1 - q;
        h->snap_ok = true;
        h->halo1_obs = out ? nullptr : p.obs;
        return;
    }
    size_t pad = 0;                               // tools: extra LDS per workgroup (occupancy study)
#ifdef PMENV_AB
    pad = (size_t)h->flat1_lds_pad;
#endif
#define PMENV_FLAT1_LAUNCH(BK, VV)                                                                           \
    if (out) {                                                                                              \
        if (pol == 1) step_flat_kernel<BK, VV, 1, true><<<grid, BK, pad, stream>>>(p, h->flat_qtot);        \
        else step_flat_kernel<BK, VV, 0, true><<<grid, BK, pad, stream>>>(p, h->flat_qtot);                 \
    } else {                                                                                                \
        if (pol == 1) step_flat_kernel<BK, VV, 1, false><<<grid, BK, pad, stream>>>(p, h->flat_qtot);       \
        else step_flat_kernel<BK, VV, 0, false><<<grid, BK, pad, stream>>>(p, h->flat_qtot);                \
    }
    const int key = h->flat1_block * 100 + h->flat1_vec;
#ifdef PMENV_AB
    if (key == 25604 && h->flat1_pol >= 3 && h->flat1_pol <= 7) {   // other cache policies
#define PMENV_FLAT1_POLV(PV)                                                                      \
        if (h->flat1_pol == PV) {                                                                 \
            if (out) step_flat_kernel<256, 4, PV, true><<<grid, 256, 0, stream>>>(p, h->flat_qtot);  \
            else step_flat_kernel<256, 4, PV, false><<<grid, 256, 0, stream>>>(p, h->flat_qtot);     \
        }
        PMENV_FLAT1_POLV(3) PMENV_FLAT1_POLV(4) PMENV_FLAT1_POLV(5) PMENV_FLAT1_POLV(6) PMENV_FLAT1_POLV(7)
#undef PMENV_FLAT1_POLV
    }
    else if (key == 25604 && h->flat1_xcd) {
        if (out) step_flat_kernel<256, 4, 1, true, true><<<grid, 256, 0, stream>>>(p, h->flat_qtot);
        else step_flat_kernel<256, 4, 1, false, true><<<grid, 256, 0, stream>>>(p, h->flat_qtot);
    }
    else if (key == 51204) { PMENV_FLAT1_LAUNCH(512, 4) }
    else if (key == 102402) { PMENV_FLAT1_LAUNCH(1024, 2) }
    else if (key == 25608) { PMENV_FLAT1_LAUNCH(256, 8) }
    else if (key == 25602) { PMENV_FLAT1_LAUNCH(256, 2) }
    else if (key == 12804) { PMENV_FLAT1_LAUNCH(128, 4) }
    else
#endif
    if (key == 25604) { PMENV_FLAT1_LAUNCH(256, 4) }
    else if (key == 12808) { PMENV_FLAT1_LAUNCH(128, 8) }
    else { PMENV_FLAT1_LAUNCH(512, 2) }
#undef PMENV_FLAT1_LAUNCH
    h->par = 1 - q;
    h->snap_ok = true;
    h->halo1_obs = out ? nullptr : p.obs;
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
int flat1_invalidate(pmenv* h, hipStream_t stream, int what = kInvalSnap | kInvalHalo, bool host_only = false) {
    if (what & kInvalSnap) h->snap_ok = false;
    h->halo1_obs = nullptr;
    if (host_only || !h->flat1_ok) return PMENV_OK;
    if (!h->device_seq && h->flat1 && capturing(stream)) h->device_seq = true;
    if (!h->device_seq) return PMENV_OK;
    // V = 0 clears both (a stale V re-primes the halo too); HOBS = 0 only the halo
    const hipError_t e = (what & kInvalSnap) ? hipMemsetAsync(h->seq + 2, 0, 4, stream)
                                             : hipMemsetAsync(h->seq + 4, 0, 8, stream);
    if (e != hipSuccess) {
        set_err(h, "invalidating the flat step's snapshot: %s", hipGetErrorString(e));
        return PMENV_ERR_HIP;
    }
    return PMENV_OK;
}

// which windows take the one-launch steps under `path`
int one_bits(const pmenv* h, int path) {
    if (path == PMENV_STEP_PATH_ONE_LAUNCH) return h->one_ok ? (PMENV_FUSE_DB | PMENV_FUSE_INPLACE) : -1;
    if (path == PMENV_STEP_PATH_TWO_LAUNCH) return h->streaming ? 0 : -1;
    if (path == PMENV_STEP_PATH_FLAT) return h->flat1_ok ? 0 : -1;
    return h->one_auto;
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
        if (h->state && h->owns_state) (void)hipFree(h->state);
        if (h->halo) (void)hipFree(h->halo);
        if (h->snap) (void)hipFree(h->snap);
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
    h->tile_floats = (int)((((int64_t)R * WF) + 3) / 4 * 4);
    h->lds_tile = scratch_bytes(h->tile_floats, c.num_assets, c.features);
    h->lds_surface = scratch_bytes(0, c.num_assets, c.features);

    // ---- the two-launch stream: row-kernel geometry (fallback) and the flat stream
    static const int kInplaceOrder[3] = {2, 4, 1}, kDoubleOrder[3] = {4, 2, 1};
    h->stream_block = h->stream_block_db = kStreamBlock;
    {
        const int bk = ab_int("PMENV_STREAM_BLOCK", kStreamBlock);   // tools: 128 | 256
        if (bk == 128 || bk == 256) h->stream_block = h->stream_block_db = bk;
    }
    h->streaming = plan_streaming(c, kInplaceOrder, h->stream_block, &h->unit_rows, &h->stream_vec) &&
                   plan_streaming(c, kDoubleOrder, h->stream_block_db, &h->unit_rows_db, &h->stream_vec_db);
    const int64_t per = (int64_t)c.num_assets * c.window * c.features;
    const int64_t win = (int64_t)c.num_envs * per * 4;
    // Flat 16-B stream (F = 5, W >= 2, 16-B granular envs, chunk count < 2^31) in place
    // (with the halo) and double-buffered: 512 threads x 2 chunks, side data through the
    // scalar unit (6.38 TB/s against 5.37 for whole-row units).
    const bool flat_ok = h->streaming && c.features == 5 && c.window >= 2 && per % 4 == 0 &&
                         (int64_t)c.num_envs * (per / 4) < (1ll << 31) - 1024;
    h->flat = h->flat_inplace = flat_ok;
    h->flat_db_wg = true;
    h->flat_block = 512;
    // in place, cache-resident windows (<= 256 MiB) take 8 KiB workgroups: 80.2 vs 83.2 us
    // at 8,192 x 30, 44.4 vs 44.7 at 4,096 (profiles/ab_r02/r02w_smallip_*); above, 16 KiB
    // (round 1: 512 x 2 against 256 x 1 / 2 / 4, 512 x 1, 1024 x 1)
    h->flat_ip_block = (int64_t)c.num_envs * per * 4 <= (256ll << 20) ? 256 : 512;
    h->flat_ip_vec = 2;
    h->flat_qtot = flat_ok ? (uint32_t)((int64_t)c.num_envs * (per / 4)) : 0u;
    // nt unless the stream's working set fits the 256 MiB Infinity Cache: the window in
    // place (<= 256 MiB), the window and its double buffer otherwise (<= 128 MiB each).
    // Step at 4,096 x 30 x 50 x 5 (123 MB) 44.4 us with the default policy against 46.5
    // nt; 8,192 envs (246 MB) in place 84.6 / 86.1 but double-buffered 91.2 / 86.5;
    // 16,384: 199.6 / 164.6 (profiles/ab_r01/pol_small_r01j.log, pol_ip_r01m.log)
    h->flat_pol = win <= (128ll << 20) ? 0 : 1;
    h->flat_ip_pol = win <= (256ll << 20) ? 0 : 1;
    h->stream_pol = 0;
    if (const char* knob = ab_knob("PMENV_STREAM_POL")) {       // tools: 0 | 1 (nt) | 2 (sc0 nt)
        const int pol = atoi(knob);
        if (pol >= 0 && pol <= 2) h->stream_pol = h->flat_pol = h->flat_ip_pol = pol;
    }
#ifdef PMENV_AB
    if (const char* knob = ab_knob("PMENV_FLAT")) h->flat = flat_ok && atoi(knob) != 0;
    if (const char* knob = ab_knob("PMENV_FLAT_INPLACE")) h->flat_inplace = flat_ok && atoi(knob) != 0;
    h->flat_db_wg = ab_int("PMENV_FLAT_DB_WG", 1) != 0;
    h->flat_ip_block = ab_int("PMENV_FLAT_IP_BLOCK", h->flat_ip_block);
    h->flat_ip_vec = ab_int("PMENV_FLAT_IP_VEC", 2);
    {   // the launcher's (block, vec) table: anything else takes the default 512 x 2
        const int key = h->flat_ip_block * 10 + h->flat_ip_vec;
        if (key != 2561 && key != 2562 && key != 2564 && key != 5121 && key != 5122 && key != 10241) {
            h->flat_ip_block = 512;
            h->flat_ip_vec = 2;
        }
    }
    {
        const int bk = ab_int("PMENV_FLAT_BLOCK", 512);
        if (bk == 128 || bk == 256 || bk == 512) h->flat_block = bk;
    }
    if (const char* knob = ab_knob("PMENV_ADVANCE"))   // force the single-launch LDS kernel
        if (!strcmp(knob, "lds")) h->streaming = h->flat = h->flat_inplace = false;
    h->ablate = ab_int("PMENV_ABLATE", 0);
    h->one_nocap = ab_int("PMENV_ONE_NOCAP", 0) != 0;
    h->flat1_lds_pad = ab_int("PMENV_FLAT1_LDS_PAD", 0);
    h->flat_s80 = ab_int("PMENV_FLAT_S80", 0) != 0;
#endif
    h->k1_groups = ab_int("PMENV_K1_GROUPS", 1);
    if (h->k1_groups != 2 && h->k1_groups != 4) h->k1_groups = 1;
    h->k1_vec = pick_k1_vec(c);
    if (h->streaming) {
        h->units_per_env = (c.num_assets + h->unit_rows - 1) / h->unit_rows;
        h->units_per_env_db = (c.num_assets + h->unit_rows_db - 1) / h->unit_rows_db;
        h->lds_stream = 0;
    }

    // ---- the one-launch step (step_env_kernel, one workgroup per env): F = 5, W >= 2,
    // N <= 64 (the scalar step on one wave), 16-B granular env windows whose 1 KiB
    // blocks fit 16 waves and 64 KiB of LDS. AUTO gives it the windows of at most
    // 48 MiB, where launch latency dominates and it wins by 7-38 % (tools/gpu_ab_smallb.sh,
    // profiles/ab_r02/r02u_*: N = 8..64, 256..4,096 envs; N = 30: 64 envs 6.5 vs 9.6 us,
    // 1,024: 13.1 vs 18.2). Larger windows take the two-launch stream: its fixed 16 KiB
    // workgroups run 640-670 us on a 2 GB window at every asset count measured, while the
    // one-workgroup-per-env geometry ties it only at N = 30 (650-658 us) and loses 4-15 %
    // at N = 8, 16, 24, 32, 40, 48, 60, 64 (profiles/ab_r02/r02r_*, r02s_*, r02t_*).
    h->per4 = (uint32_t)(per / 4);
    // 4 chunks per lane (tools: PMENV_ONE_V = 1 | 2 | 3 | 6 | 8; 4 measured best: 650 us
    // against 662-666 for 8, 762 for 3, 860 for 2 at the BASELINE shape)
    h->one_v = ab_int("PMENV_ONE_V", 4);
    if (h->one_v != 1 && h->one_v != 2 && h->one_v != 3 && h->one_v != 6 && h->one_v != 8) h->one_v = 4;
    {
        // the env's chunks start anywhere in a 64-chunk block: up to 63 slots ahead of it
        const uint32_t blocks = (h->per4 + 63u + 63u) / 64u;
        h->one_waves = (int)((blocks + (uint32_t)h->one_v - 1) / (uint32_t)h->one_v);
    }
    h->one_ok = h->streaming && c.features == 5 && c.window >= 2 && c.num_assets <= 64 && per % 4 == 0 &&
                h->one_waves <= 16 && ((int64_t)64 * h->one_v * h->one_waves + 2) * 16 <= 65536;
    // (also beyond the flat stream's 2^31-chunk index, where the two-launch path would fall
    // back to the whole-row stream)
    h->one_auto = h->one_ok && (win <= (48ll << 20) || !h->flat_inplace) ? (PMENV_FUSE_DB | PMENV_FUSE_INPLACE) : 0;
#ifdef PMENV_AB
    if (const char* knob = ab_knob("PMENV_ONE")) {    // 0 | db | ip | all
        if (!h->one_ok || !strcmp(knob, "0")) h->one_auto = 0;
        else if (!strcmp(knob, "db")) h->one_auto = PMENV_FUSE_DB;
        else if (!strcmp(knob, "ip")) h->one_auto = PMENV_FUSE_INPLACE;
        else if (!strcmp(knob, "all")) h->one_auto = PMENV_FUSE_DB | PMENV_FUSE_INPLACE;
    }
    {   // the previous one-launch form (advance_rows_kernel<fused>), PMENV_FUSED = db | all
        int fused_rows = 0;
        const bool fusable = h->streaming && c.num_assets <= 64 && !h->ablate &&
                             plan_streaming(c, kDoubleOrder, kStreamBlock, &fused_rows, &h->fused_vec) &&
                             fused_rows == c.num_assets;
        if (const char* knob = ab_knob("PMENV_FUSED")) {
            if (fusable && !strcmp(knob, "db")) h->fused = PMENV_FUSE_DB;
            else if (fusable && !strcmp(knob, "all")) h->fused = PMENV_FUSE_DB | PMENV_FUSE_INPLACE;
            if (h->fused) h->one_auto &= ~h->fused;
        }
    }
#endif
    // ---- the one-launch flat step (step_flat_kernel): the flat stream's shape rules, the
    // scalar step on one wave per env (N <= 64), at most one env per wave in a tile.
    // Geometry: 256 threads x 4 chunks (16 KiB tiles, 4 waves) where env windows have
    // >= 511 chunks, 512 x 2 (8 waves) from 148 chunks. 256 x 4 against 512 x 2 / 512 x 4 /
    // 1024 x 2 / 256 x 8 / 256 x 2 / 128 x 8 / 128 x 4 at 65,536 x 30 in place: 629.5 against
    // 714 / 678 / 790 / 695 / 675 / 624 / 641 us; 128 x 8 loses 15 % at N = 16 and 64 where
    // 256 x 4 wins (profiles/ab_r02/r02w_flat1b_*, r02w_flat1c_*). A persistent form that
    // keeps the next tile's loads in flight needs 160 VGPRs (3 waves per SIMD): 2x slower.
    // Wide envs (64 < N <= 512, step_flat_vec_kernel) also need the rows a tile touches
    // per env to fit one wave's 64 staged bar rows (W >= 14 at F = 5 for 16 KiB tiles).
    auto flat1_fits = [&](int block, int vec) {
        const uint32_t cpw = (uint32_t)(block * vec);
        const uint32_t ne_max = h->per4 ? (cpw + h->per4 - 2u) / h->per4 + 1u : 0u;
        const int64_t span_rows = (4ll * cpw - 1) / (WF > 0 ? WF : 1) + 2;
        const bool wide_ok = c.num_assets <= kWideMaxAssets && span_rows <= 64;
        return flat_ok && (c.num_assets <= 64 || wide_ok) && ne_max <= (uint32_t)(block / 64);
    };
    // 128 x 8 (2 waves, 8 chunks per lane, the same 16 KiB tiles) where every tile holds at
    // most two envs (1,023 .. 1,999 chunks per env: N = 20 .. 39 at W = 50) and the window
    // streams through HBM: 0.5-1.1 % ahead of 256 x 4 from 49,152 envs at N = 30 (65,536:
    // 625.7 vs 629.4 and 628.8 vs 631.6 us; 98,304: 941.1 vs 951.6), N = 20 / 24 / 28 by
    // 1.0 / 0.7 / 0.5 %; behind it at 16,384 envs (162.9 vs 161.4) and at N = 16 / 64
    // (profiles/ab_r02/r02w_flat1k_*, r02w_flat1l_*, r02w_flat1c_*)
    const bool band128 = h->per4 >= 1023u && h->per4 < 2000u && win > (1ll << 30);
    if (band128 && flat1_fits(128, 8)) { h->flat1_block = 128; h->flat1_vec = 8; }
    else if (flat1_fits(256, 4)) { h->flat1_block = 256; h->flat1_vec = 4; }
    else { h->flat1_block = 512; h->flat1_vec = 2; }
    h->flat1_ok = flat1_fits(h->flat1_block, h->flat1_vec);
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
    const int one_auto_base = h->one_auto;   // tools: PMENV_FLAT1=0 restores it
    (void)one_auto_base;
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
#ifdef PMENV_AB
    if (const char* knob = ab_knob("PMENV_FLAT1")) {   // tools: 1 = the flat step for every window, 0 = never
        h->flat1_auto = h->flat1_ok && atoi(knob) ? (PMENV_FUSE_DB | PMENV_FUSE_INPLACE) : 0;
        h->one_auto = h->flat1_auto ? 0 : one_auto_base;
    }
    h->flat1_xcd = ab_int("PMENV_FLAT1_XCD", 0) != 0;
    h->flat1_pol = ab_int("PMENV_FLAT1_POL", 0);
    if (const char* knob = ab_knob("PMENV_FLAT1_GEOM")) {   // "512x2" | "512x4" | "1024x2" | "256x8" | ...
        int bk = 0, vv = 0;
        if (sscanf(knob, "%dx%d", &bk, &vv) == 2) {
            const int key = bk * 100 + vv;
            if ((key == 51202 || key == 51204 || key == 102402 || key == 25604 || key == 25608 || key == 25602 ||
                 key == 12808 || key == 12804) && flat1_fits(bk, vv)) {
                h->flat1_block = bk;
                h->flat1_vec = vv;
            }
        }
    }
#endif
    h->path = PMENV_STEP_PATH_AUTO;
    h->one = h->one_auto;
    h->flat1 = h->flat1_auto;

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
    if (h->flat_inplace) {
        const uint32_t cpw = (uint32_t)(h->flat_ip_block * h->flat_ip_vec);
        const uint32_t wgs = (h->flat_qtot + cpw - 1) / cpw;
        h->halo_wgs = wgs > 0 ? wgs - 1 : 0;
        hipError_t ae = hipMalloc(&h->halo, (size_t)(h->halo_wgs + 1) * 32);
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

int pmenv_destroy(pmenv* h) {
    if (!h) return PMENV_ERR_ARG;
    DeviceGuard g(h->device);
    if (h->state && h->owns_state) (void)hipFree(h->state);
    if (h->halo) (void)hipFree(h->halo);
    if (h->snap) (void)hipFree(h->snap);
    free(h);
    return PMENV_OK;
}

int pmenv_set_step_path(pmenv* h, int32_t path) {
    if (!h) return PMENV_ERR_ARG;
    if (path < PMENV_STEP_PATH_AUTO || path > PMENV_STEP_PATH_FLAT) {
        set_err(h, "unknown step path %d", path);
        return PMENV_ERR_ARG;
    }
    const int bits = one_bits(h, path);
    const int fbits = flat1_bits(h, path);
    if (bits < 0 || fbits < 0) {
        set_err(h, "step path %d does not fit this shape (one launch: F = 5, W >= 2, N <= 64, window <= 64 KiB "
                   "of LDS; two launches: F = 5, 16-B granular env windows; flat: F = 5, W >= 2, N <= 64, "
                   "16-B granular env windows of >= 148 chunks, N > 64 up to 512 with W >= 14)", path);
        return PMENV_ERR_ARG;
    }
    h->path = path;
    h->one = bits;
    h->flat1 = fbits;
    return PMENV_OK;
}

int pmenv_reset(pmenv* h, float* obs, const uint8_t* mask, hipStream_t stream) {
    if (!h) return PMENV_ERR_ARG;
    if (obs && !aligned4(obs)) { set_err(h, "obs not 4-byte aligned"); return PMENV_ERR_ALIGN; }
    DeviceGuard g(h->device);
    StepParams p = base_params(h);
    if (const int rc = flat1_invalidate(h, stream)) return rc;
    reset_kernel<<<h->cfg.num_envs, kBlock, 0, stream>>>(p, obs, mask);
    return check_launch(h, "reset_kernel");
}

int pmenv_step_ex(pmenv* h, const pmenv_step_args* a, hipStream_t stream) {
    if (!h) return PMENV_ERR_ARG;
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
        launch_flat1(h, p, stream);
        return check_launch(h, "step_flat_kernel");
    }
    if (const int rc = flat1_invalidate(h, stream)) return rc;   // every other path skips the snapshot
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

#ifdef PMENV_AB
        if (ph == (PMENV_PHASE_SCALAR | PMENV_PHASE_ADVANCE) && (h->fused & fuse_bit)) {
            launch_fused(h, p, stream);
            return check_launch(h, "advance_rows_kernel<fused>");
        }
#endif
        if (ph & PMENV_PHASE_SCALAR) {
            const int rc = launch_scalar(h, p, stream);
            if (rc) return rc;
        }
        if (ph & PMENV_PHASE_ADVANCE) {
            launch_advance(h, p, stream);
            return check_launch(h, "advance kernel");
        }
        return PMENV_OK;
    }
    if (a->phases == PMENV_PHASE_ADVANCE) return PMENV_OK;   // single-launch path: all done in the scalar phase
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

double* pmenv_value(pmenv* h) { return h ? h->value : nullptr; }
float* pmenv_ring(pmenv* h) { return h ? h->ring : nullptr; }
int32_t* pmenv_counter(pmenv* h) { return h ? h->k : nullptr; }
size_t pmenv_state_bytes(const pmenv* h) { return h ? h->state_bytes : 0; }

const char* pmenv_step_path(const pmenv* h) {
    if (!h) return "";
    if (!h->streaming) return "step_advance_lds_kernel";
    // per window mode: the one-launch kernel, or the scalar step (K1) then the stream
    const char* k1 = h->k1_vec ? "scalar_step_vec_kernel"
                   : h->cfg.num_assets <= 64 ? "scalar_step_reg_kernel" : "scalar_step_kernel";
    const char* db2 = h->flat ? (h->flat_db_wg ? "advance_flat_wg_kernel" : "advance_flat_kernel")
                    : "advance_rows_kernel";
    const char* ip2 = h->flat_inplace ? "advance_flat_inplace_kernel" : "advance_rows_kernel";
    static thread_local char buf[2][128], out[320];
    const char* part[2];
    for (int m = 0; m < 2; ++m) {          // 0 = double-buffered (obs_out), 1 = in place
        const int bit = m ? PMENV_FUSE_INPLACE : PMENV_FUSE_DB;
        if (h->flat1 & bit) part[m] = h->cfg.num_assets > 64 ? "step_flat_vec_kernel" : "step_flat_kernel";
        else if (h->one & bit) part[m] = "step_env_kernel";
        else if (h->fused & bit) part[m] = "advance_rows_kernel<fused>";
        else {
            snprintf(buf[m], sizeof buf[m], "%s+%s", k1, m ? ip2 : db2);
            part[m] = buf[m];
        }
    }
    snprintf(out, sizeof out, "%s (obs_out) | %s (in place)%s", part[0], part[1],
             h->device_seq && h->flat1 ? " [flat steps device-sequenced]" : "");
    return out;
}

int pmenv_get_state(pmenv* h, void* dst, hipStream_t stream) {
    if (!h || !dst) return PMENV_ERR_ARG;
    DeviceGuard g(h->device);
    hipError_t e = hipMemcpyAsync(dst, h->state, h->state_bytes, hipMemcpyDeviceToDevice, stream);
    if (e != hipSuccess) { set_err(h, "get_state: %s", hipGetErrorString(e)); return PMENV_ERR_HIP; }
    return PMENV_OK;
}

int pmenv_set_state(pmenv* h, const void* src, hipStream_t stream) {
    if (!h || !src) return PMENV_ERR_ARG;
    DeviceGuard g(h->device);
    if (const int rc = flat1_invalidate(h, stream)) return rc;
    hipError_t e = hipMemcpyAsync(h->state, src, h->state_bytes, hipMemcpyDeviceToDevice, stream);
    if (e != hipSuccess) { set_err(h, "set_state: %s", hipGetErrorString(e)); return PMENV_ERR_HIP; }
    return PMENV_OK;
}

int pmenv_window_written(pmenv* h, const float* obs, hipStream_t stream) {
    if (!h) return PMENV_ERR_ARG;
    (void)obs;                                 // any window: the halo is dropped whichever it was
    DeviceGuard g(h->device);
    return flat1_invalidate(h, stream, kInvalHalo);
}

int pmenv_state_written(pmenv* h, hipStream_t stream) {
    if (!h) return PMENV_ERR_ARG;
    DeviceGuard g(h->device);
    return flat1_invalidate(h, stream, kInvalSnap | kInvalHalo);
}

int pmenv_nonfinite_count(pmenv* h, uint64_t* out, hipStream_t stream) {
    if (!h || !out) return PMENV_ERR_ARG;
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
    // measured on MI355X (tools/bench_rows.py, profiles/rows_r01.json): the tiled scan
    // beats the per-env loop 2.7x at T = 256 x B = 65536 and 14x at 2048 x 8192; the
    // wave-per-env scan only for a handful of envs with long horizons
    const char* knob = ab_knob("PMENV_GAE");      // tools: loop | scan | tile
    const bool fits = (size_t)(T + 1) * (size_t)B * 4u < (1ull << 31);   // gae_tile_kernel's buffer offsets
    const bool scan = knob ? !strcmp(knob, "scan") : (B < 64 && T >= 256);
    const bool tile = fits && (knob ? !strcmp(knob, "tile") : !scan);
    const int U = ab_int("PMENV_GAE_U", B >= 16384 ? 8 : 16);   // tools: steps per lane and segment
#ifdef PMENV_AB
    // PMENV_GAE_E: envs per lane of the pipelined tile (gae_tile_vec_kernel; 1, 2 or 4,
    // needs B % E == 0); 0 = gae_tile_kernel
    int E = ab_int("PMENV_GAE_E", 0);
    if (E != 1 && E != 2 && E != 4) E = 0;
    if (E && B % E) E = 0;
    if (knob && !strcmp(knob, "tile8") && fits) {   // tools: the tile held to 64 VGPRs (8 waves per SIMD)
        gae_tile_kernel<8, 8, 8><<<(B + 63) / 64, 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam);
        return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
    }
    if (knob && !strcmp(knob, "stream") && fits) {   // PMENV_GAE_P: days per block (16 or 32)
        const unsigned g = (unsigned)((B + 63) / 64);
        if (ab_int("PMENV_GAE_P", 16) == 32)
            gae_stream_kernel<32><<<g, 64, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam);
        else if (ab_int("PMENV_GAE_P", 16) == 8)
            gae_stream_kernel<8><<<g, 64, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam);
        else
            gae_stream_kernel<16><<<g, 64, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam);
        return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
    }
    if (tile && E) {
        const unsigned g = (unsigned)((B + 64 * E - 1) / (64 * E));
#define PMENV_GAEV(U_, E_) \
    gae_tile_vec_kernel<8, U_, E_><<<g, 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam)
        if (E == 1 && U == 16) PMENV_GAEV(16, 1);
        else if (E == 1) PMENV_GAEV(8, 1);
        else if (E == 2 && U == 4) PMENV_GAEV(4, 2);
        else if (E == 2) PMENV_GAEV(8, 2);
        else PMENV_GAEV(4, 4);                    // E = 4 at U = 8 spills
#undef PMENV_GAEV
        return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
    }
#endif
    // many envs and at least four 64-day segments: the tile held to 64 VGPRs (8 waves per
    // SIMD, so a 65,536-env rollout's 1,024 workgroups are resident at once; the same bits):
    // 56.7 vs 58.5 us at 256 x 65,536, 110.1 vs 114.7 at 512 x 65,536; slower below 65,536
    // envs or 256 days (profiles/ab_r02/gae_occ8_r02zl.json)
    if (tile && U == 8 && B >= 65536 && T >= 256)
        gae_tile_kernel<8, 8, 8><<<(B + 63) / 64, 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma,
                                                                   lam);
    else if (tile && U == 16)
        gae_tile_kernel<8, 16><<<(B + 63) / 64, 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma,
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

// Horizon split of the tiled GAE scan (gae_chunk_kernel): used when the B / 64 env
// blocks leave CUs idle; chunks sized so blocks x chunks ~ 1024 workgroups, each
// chunk a whole number of 128-day segments (NW = 8, U = 16) and at least 2 of them.
namespace {
constexpr int kGaeSeg = 8 * 16;
int gae_chunks(int32_t T, int32_t B, int* Lc) {
    const int blocks = (B + 63) / 64;
    if (B >= 16384 || T < 4 * kGaeSeg) return 0;
    if ((size_t)(T + 1) * (size_t)B * 4u >= (1ull << 31)) return 0;
    int want = (1024 + blocks - 1) / blocks;                    // chunks for ~1024 workgroups
    int lc = (T + want - 1) / want;
    lc = (lc + kGaeSeg - 1) / kGaeSeg * kGaeSeg;
    lc = lc < 2 * kGaeSeg ? 2 * kGaeSeg : lc;
    const int n = (T + lc - 1) / lc;
    if (n < 2) return 0;
    *Lc = lc;
    return n;
}
}  // namespace

size_t pmenv_gae_workspace(int32_t T, int32_t B) {
    int lc = 0;
    const int n = (T < 1 || B < 1) ? 0 : gae_chunks(T, B, &lc);
    return n ? (size_t)2 * n * B * sizeof(double) : 0;
}

int pmenv_gae_ex(const float* rewards, const float* values, const uint8_t* dones, float* adv, float* ret, int32_t T,
                 int32_t B, float gamma, float lam, double* work, size_t work_bytes, hipStream_t stream) {
    if (!rewards || !values || !adv || !ret || T < 1 || B < 1) return PMENV_ERR_ARG;
    int lc = 0;
    const int n = gae_chunks(T, B, &lc);
    const char* knob = ab_knob("PMENV_GAE");      // tools: an explicit kernel choice wins
    if (!n || knob || !work || work_bytes < (size_t)2 * n * B * sizeof(double))
        return pmenv_gae(rewards, values, dones, adv, ret, T, B, gamma, lam, stream);
    const dim3 grid((unsigned)((B + 63) / 64), (unsigned)n);
    gae_chunk_kernel<8, 16, true><<<grid, 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam, lc,
                                                            work);
    gae_chunk_kernel<8, 16, false><<<grid, 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam, lc,
                                                             work);
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
    if (F == 5 && al16 && !ab_knob("PMENV_REPLAY_LDS")) {   // tools: the per-element staging kernel
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
        const dim3 grid((unsigned)S, (unsigned)(N / R));
        const int pairs = R * (W + 1);
        // s / s' are written once per sample: nt stores, 129.6 -> 118.6 us at S = 8,192
        // (tools/ab_replay.py, profiles/ab_r01/replay_nt_tpb_r01h.log). Persistent form
        // (replay_gather_f5p_kernel): one workgroup per CU loops over the samples with the
        // next sample's loads in flight. One per CU is the measured optimum (S = 8,192:
        // 96 us at 256 workgroups; 114-121 us at 192, 288, 512, 768, 1,280 and one
        // workgroup per sample, 117 us; profiles/ab_r01/replay_grid_r01j.log). Tools knobs:
        // PMENV_REPLAY_NT=0 (default-policy stores), PMENV_REPLAY_PERSIST=0 (one workgroup
        // per sample), PMENV_REPLAY_TPB=512, PMENV_REPLAY_GRID=G.
        const bool nt = ab_int("PMENV_REPLAY_NT", 1) != 0;
        const bool t512 = ab_int("PMENV_REPLAY_TPB", 256) == 512;
        const bool persist = !t512 && ab_int("PMENV_REPLAY_PERSIST", 1) != 0;
        if (persist) {
            static int cus = 0;
            if (!cus) {
                int dev = 0;
                if (hipGetDevice(&dev) != hipSuccess ||
                    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
                    cus = 256;
            }
            const int gy = N / R;
            int G = cus / gy > 0 ? cus / gy : 1;
            G = ab_int("PMENV_REPLAY_GRID", G) > 0 ? ab_int("PMENV_REPLAY_GRID", G) : G;
            const dim3 pgrid((unsigned)(S < G ? S : G), (unsigned)(N / R));
            const int ppt = pairs <= 2 * 256 ? 2 : pairs <= 4 * 256 ? 4 : 8;
#define PMENV_RGP(PPT, NTV)                                                                                   \
    replay_gather_f5p_kernel<PPT, NTV><<<pgrid, 256, glds, stream>>>(series, T, N, W, days, actions, rewards, H, B, \
                                                                     h0, env, S, s, s_next, a_out, r_out, R, dr, dwf)
#ifdef PMENV_AB
            if (!nt) {
                if (ppt == 2) PMENV_RGP(2, 0); else if (ppt == 4) PMENV_RGP(4, 0); else PMENV_RGP(8, 0);
                return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
            }
#endif
            if (ppt == 2) PMENV_RGP(2, 2); else if (ppt == 4) PMENV_RGP(4, 2); else PMENV_RGP(8, 2);
#undef PMENV_RGP
            return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
        }
#ifdef PMENV_AB
        const int tpb = t512 ? 512 : 256;
        const int ppt = pairs <= 2 * tpb ? 2 : pairs <= 4 * tpb ? 4 : 8;
#define PMENV_RG(PPT, NTV, TPB)                                                                              \
    replay_gather_f5_kernel<PPT, NTV, TPB><<<grid, TPB, glds, stream>>>(series, T, N, W, days, actions, rewards, \
                                                                        H, B, h0, env, s, s_next, a_out, r_out, \
                                                                        R, dr, dwf)
        if (t512) {
            if (nt) { if (ppt == 2) PMENV_RG(2, 2, 512); else if (ppt == 4) PMENV_RG(4, 2, 512); else PMENV_RG(8, 2, 512); }
            else { if (ppt == 2) PMENV_RG(2, 0, 512); else if (ppt == 4) PMENV_RG(4, 0, 512); else PMENV_RG(8, 0, 512); }
        } else {
            if (nt) { if (ppt == 2) PMENV_RG(2, 2, 256); else if (ppt == 4) PMENV_RG(4, 2, 256); else PMENV_RG(8, 2, 256); }
            else { if (ppt == 2) PMENV_RG(2, 0, 256); else if (ppt == 4) PMENV_RG(4, 0, 256); else PMENV_RG(8, 0, 256); }
        }
#undef PMENV_RG
#else
        (void)grid;
        (void)nt;
#endif
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
#ifdef PMENV_AB
    if (ab_knob("PMENV_RGATHER_ELEM")) {          // tools: one thread per output float
        const int64_t threads = (int64_t)S * N * W * F;
        rollout_gather_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, stream>>>(
            series, T, N, F, W, start, weights, T_rec, B, ring_mode, t_idx, env, S, s);
        return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
    }
#endif
    const size_t lds = (size_t)W * N * F * sizeof(float);
    // market [W][N][4] + weights [W][N]; the tile's 16-B series loads and window stores need
    // 16-B aligned series / s (C callers may pass sliced views: those take the row form)
    const bool al16 = (((uintptr_t)series | (uintptr_t)s) & 15u) == 0;
    bool tile = F == 5 && (N * W * F) % 4 == 0 && lds <= 64 * 1024 && al16;
#ifdef PMENV_AB
    if (ab_knob("PMENV_RGATHER_ROWS")) tile = false;      // tools: the wave-per-row form
#endif
    if (tile) {                                            // one workgroup per sample, staged in LDS
        rollout_gather_tile_kernel<<<(unsigned)S, 256, lds, stream>>>(
            series, T, N, W, start, weights, B, ring_mode, t_idx, env, s, make_fastdiv((uint32_t)N),
            make_fastdiv((uint32_t)(W * F)), make_fastdiv((uint32_t)F));
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
    // measured on MI355X (tools/bench_rows.py): the horizon split over four waves per
    // 64 envs against the thread-per-env walk — see profiles/rows_r01*/
    const int tpe = N <= 256 ? N : 256, eb = 256 / tpe;
    const int nseg = (B + 63) / 64, nturn = (B + eb - 1) / eb;
    // one launch for both passes (metrics_fused_kernel); A/B knobs: PMENV_METRICS_FUSED=0
    // (two launches), PMENV_METRICS_SEG_FIRST=0 (turnover blocks dispatched first)
    const bool walk = ab_knob("PMENV_METRICS_WALK") != nullptr;  // tools: the thread-per-env walk
    const bool fused = !walk && ab_int("PMENV_METRICS_FUSED", 1) != 0;
    if (fused) {
        const int seg_first = ab_int("PMENV_METRICS_SEG_FIRST", 1) != 0;
        metrics_fused_kernel<<<(unsigned)(nseg + nturn), 256, 0, stream>>>(returns, values, weights, T, B, N,
                                                                           risk_free_rate, periods, tpe, eb, nseg,
                                                                           nturn, seg_first, out);
        return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
    }
#ifdef PMENV_AB
    if (walk)
        metrics_kernel<<<(B + 255) / 256, 256, 0, stream>>>(returns, values, T, B, risk_free_rate, periods, out);
    else
        metrics_seg_kernel<<<(unsigned)nseg, 256, 0, stream>>>(returns, values, T, B, risk_free_rate, periods, out);
    metrics_turnover_kernel<<<(unsigned)nturn, 256, 0, stream>>>(weights, T, B, N, tpe, eb, out);
#endif
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
    // one launch: the row blocks' partials and, in the block that finishes last, the
    // final fold (batch_reward_fwd_*_kernel; the ticket it counts on is zeroed first)
#ifdef PMENV_AB
    // tools: the forward in one launch (batch_reward_fwd_*_kernel: the block that draws
    // the last ticket folds the partials). Measured slower than the two launches below at
    // every shape, so the product keeps the two.
    if (ab_knob("PMENV_BR_ONE")) {
        if (hipMemsetAsync(work + 6 * (size_t)B + 6, 0, sizeof(uint32_t), stream) != hipSuccess) return PMENV_ERR_HIP;
        const bool quad = N <= kQuadMaxN;
        const int nblk = quad ? (B + kQuadRows - 1) / kQuadRows : (int)batch_reward_blocks(B);
        int grid = nblk, fence = 1;
        if (const char* knob = ab_knob("PMENV_BR_GRID")) grid = std::max(1, std::min(nblk, atoi(knob)));
        if (const char* knob = ab_knob("PMENV_BR_FENCE")) fence = atoi(knob);
        const unsigned g = (unsigned)grid;
#define PMENV_FWD_ARGS a, v_prev, p, B, N, reward_kind, norm, scale, work, reward_out, nblk
        if (quad) {
            if (fence == 0) {
                if (N <= 32) batch_reward_fwd_quad_kernel<8, 0><<<g, kTrainBlock, 0, stream>>>(PMENV_FWD_ARGS);
                else batch_reward_fwd_quad_kernel<16, 0><<<g, kTrainBlock, 0, stream>>>(PMENV_FWD_ARGS);
            } else if (N <= 32) batch_reward_fwd_quad_kernel<8, 1><<<g, kTrainBlock, 0, stream>>>(PMENV_FWD_ARGS);
            else batch_reward_fwd_quad_kernel<16, 1><<<g, kTrainBlock, 0, stream>>>(PMENV_FWD_ARGS);
        } else {
            if (N <= 128) batch_reward_fwd_rows_kernel<2, 0><<<g, kTrainBlock, 0, stream>>>(PMENV_FWD_ARGS);
            else if (N <= 256) batch_reward_fwd_rows_kernel<4, 0><<<g, kTrainBlock, 0, stream>>>(PMENV_FWD_ARGS);
            else if (N <= 512) batch_reward_fwd_rows_kernel<8, 0><<<g, kTrainBlock, 0, stream>>>(PMENV_FWD_ARGS);
            else batch_reward_fwd_rows_kernel<0, 0><<<g, kTrainBlock, 0, stream>>>(PMENV_FWD_ARGS);
        }
#undef PMENV_FWD_ARGS
        if (ret_out) batch_reward_select_kernel<<<(B + 255) / 256, 256, 0, stream>>>(B, norm, work, ret_out);
        return hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
    }
#endif
    int nparts;
    if (N <= kQuadMaxN) {         // a quad of lanes per row
        nparts = (B + kQuadRows - 1) / kQuadRows;
        if (N <= 32)
            batch_reward_rows_quad_kernel<8><<<(unsigned)nparts, kTrainBlock, 0, stream>>>(a, v_prev, p, B, N,
                                                                                           reward_kind, work);
        else
            batch_reward_rows_quad_kernel<16><<<(unsigned)nparts, kTrainBlock, 0, stream>>>(a, v_prev, p, B, N,
                                                                                            reward_kind, work);
    } else {                      // wave per row, registers up to N = 512
        nparts = (int)batch_reward_blocks(B);
        const unsigned g = (unsigned)nparts;
        if (N <= 128) batch_reward_rows_kernel<2><<<g, kTrainBlock, 0, stream>>>(a, v_prev, p, B, N, reward_kind, work);
        else if (N <= 256) batch_reward_rows_kernel<4><<<g, kTrainBlock, 0, stream>>>(a, v_prev, p, B, N, reward_kind, work);
        else if (N <= 512) batch_reward_rows_kernel<8><<<g, kTrainBlock, 0, stream>>>(a, v_prev, p, B, N, reward_kind, work);
        else batch_reward_rows_kernel<0><<<g, kTrainBlock, 0, stream>>>(a, v_prev, p, B, N, reward_kind, work);
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
