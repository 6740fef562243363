// handle.h — the env handle (struct pmenv) and the host-side shape planning, shared by the
// product library (pmenv.hip, launch.h) and the tools build (tools/ab/pmenv_ab.hip).
//
// The tools build — tools/libpmenv_ab.so, the A/B harnesses' library — is the product's
// translation unit linked with tools/ab/pmenv_ab.hip, which defines the pmenv_tools hooks
// below: it reads the PMENV_* knobs and launches the alternatives the product was measured
// against. The product library's definitions of the hooks (weak, at the end of pmenv.hip)
// do nothing, and it reads no environment variable.
#pragma once
#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/pmenv.h"
#include "common.h"

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
    // the register step (step_small_kernel<small_block, small_e>): any F, any alignment, env
    // windows of at most 1,024 x 16 floats; 0: the LDS fallback
    int small_block, small_e;
    bool tiny;            // ... of at most 256 x 8 floats and N <= 64: step_tiny_kernel (LDS-staged)
    bool surf_stream;     // surface steps as two launches: the scalar step, then surface_stream_kernel
    size_t surf_lds;      // its workgroup's rows' ring columns (rows x W floats)
    // LDS single-launch fallback geometry
    int rows_per_tile, tile_floats;
    bool vec;
    size_t lds_tile, lds_surface;
    // two-launch path: the scalar step, then the window stream
    bool streaming;       // F = 5, 16-B granular env windows: the streams below apply
    int unit_rows, units_per_env, stream_vec;          // row-kernel advance in place
    int unit_rows_db, units_per_env_db, stream_vec_db; // row-kernel advance double-buffered (obs_out)
    bool flat_ok;         // the flat 16-B stream's shape rules hold
    bool flat;            // double-buffered advance as the flat 16-B stream
    int flat_pol, flat_ip_pol;   // cache policy (0 default, 1 nt): double-buffered / in-place stream
    bool flat_inplace;    // in-place advance as the flat stream + halo (advance_flat_inplace_kernel)
    int flat_ip_block, flat_ip_vec;   // threads per workgroup, chunks per thread
    float* halo;          // [halo_wgs][2] float4: first two chunks of every in-place flat workgroup
    uint32_t halo_wgs, flat_qtot;
    int scalar_scratch_floats;
    size_t lds_scalar;
    // two-launch path for F != 5 (2 <= F <= 8, 16-B granular env windows): the scalar step,
    // then the generic stream (advance_gen_kernel<gen_block, gen_v>)
    bool gen_ok;          // the shape fits the generic stream
    int gen_auto;         // PMENV_FUSE_* bits the automatic choice gives it
    int gen;              // PMENV_FUSE_* bits: which windows take it now
    int gen_block, gen_v; // threads per workgroup, chunks per thread
    uint32_t gen_qtot;    // chunks of the whole [B, N, W, F] window
    int k1_vec;           // scalar_step_vec_kernel shape 100 * L + A (+ kK1Str), 0: register / LDS form
    // one launch per step, one workgroup per env (step_env_kernel)
    bool one_ok;          // the shape fits step_env_kernel
    int one_auto;         // PMENV_FUSE_* bits the automatic choice gives step_env_kernel
    int one;              // PMENV_FUSE_* bits: which windows take step_env_kernel now
    int one_waves;        // waves per workgroup
    uint32_t per4;        // 16-B chunks per env window
    // one launch over the flat stream (step_flat_kernel / step_flat_vec_kernel)
    bool flat1_ok;        // the shape fits the flat one-launch step
    int flat1_auto;       // PMENV_FUSE_* bits the automatic choice gives it
    int flat1;            // PMENV_FUSE_* bits: which windows take it now
    int flat1_block, flat1_vec;   // threads per workgroup, chunks per thread
    void* snap;           // the state snapshot, two parities: value f64 | counter i32 | get_last() | last close
    double* sv[2];
    int32_t* sk[2];
    float* sw[2];
    float* slc[2];
    float* halo1[2];      // [halo1_wgs][2] float4 per parity: the next tile's first two chunks
    uint32_t halo1_wgs;
    int par;              // parity of the snapshot / halo the next step reads
    bool snap_ok;         // sv[par] .. slc[par] equal the canonical state
    const float* halo1_obs;   // the window whose halo halo1[par] holds (null: none)
    // device-sequenced form (hipGraph-safe): from the first flat step enqueued under
    // stream capture on, every flat step is flat_seq_kernel + the kernel reading the
    // parity and the validity from seq (device words) instead of the host fields above
    bool device_seq;
    int32_t* seq;         // {D, C, V, pad, HOBS lo, HOBS hi} (step_flat.h)
    uint64_t snap_stride; // bytes between the two parities of the snapshot / halo
    // one launch, scalar blocks relaying w' and the counter to the stream tiles (step_relay.h)
    bool relay_ok;        // the shape fits step_relay_kernel
    int relay_auto;       // PMENV_FUSE_* bits the automatic choice gives it
    int relay;            // PMENV_FUSE_* bits: which windows take it now
    int relay_kl, relay_ka;   // the scalar step's form: KL lanes per env, KA strided assets per lane (0: register)
    int relay_block, relay_v; // the tiles' geometry: relay_block threads x relay_v 16-B chunks
    int relay_epb;        // envs per scalar block (relay_block / 64 waves x 64 / relay_kl envs)
    uint32_t relay_tiles, relay_scal;
    void* relay_mem;      // control words | relay words, deferral list, tile claims | counter copy x 2 | halo x 2 (allocated when
                          // AUTO gives the shape the relay step or pmenv_set_step_path asks for it)
    uint32_t* relay_seq;  // device-sequenced words {D, E, V, C, EC, pad, HOBS lo, HOBS hi} (step_relay.h)
    uint64_t* relay_w;    // [B * N] {epoch, w'}
    uint64_t* relay_list; // the deferral list: [0] {epoch, count}, [1 .. relay_tiles] {epoch, tile}
    uint32_t* relay_done; // [relay_tiles] the epoch in which each deferred tile last ran
    int32_t* relay_kp;    // [2][B] the counter copies, per parity
    float* relay_halo;    // in place: [2][relay_halo_stride] floats
    uint32_t relay_halo_stride;
    bool relay_kp_ok;     // eager: relay_kp[relay_par] equals the state's counter
    const float* relay_obs;   // eager: the window whose halo relay_halo[relay_par] holds (null: none)
    int relay_par;        // eager: parity of the counter copy / halo the next relay step reads
    uint32_t relay_epoch; // eager: the last step's tag
    bool relay_dseq;      // device-sequenced: from the first call of this handle enqueued under stream
                          // capture on, epoch, parity and the copies' validity live in relay_seq
    // host-I/O staging (pmenv_step_host / pmenv_reset_host): one pinned, device-mapped block,
    // allocated on the first host-I/O call — action | prices | last closes | channel [B,N,W] |
    // weights | reward (f32), then return | value (f64), then the completion words (u32);
    // `hio_dev` is its device address
    char* hio;
    char* hio_dev;
    size_t hio_off[10];
    uint32_t hio_seq;     // the last host-I/O call's completion tag
    // the resident host-I/O step (step_host_resident_kernel): its own stream, an event recorded
    // after its launch (complete = the workgroup has exited), the last tag it ran (device u32)
    hipStream_t res_stream;
    hipEvent_t res_ev;
    uint32_t* res_last;
    bool res_live;        // launched and not yet seen exited
    bool dev_pending;     // an asynchronous call of this handle since its last synchronous host call
    pmenv_dev::StepParams res_p;   // its launch arguments
    pmenv_dev::HostIO res_io;
    int path;             // pmenv_step_path_kind
    void* tools;        // tools build: its knob state (null in the product library)
    char err[512];
};

namespace pmenv_host {

constexpr int PMENV_FUSE_DB = 1, PMENV_FUSE_INPLACE = 2;
constexpr int kOneV = 4;              // step_env_kernel: 16-B chunks per lane
constexpr int kK1Str = 100000;        // k1_vec: the strided layout of scalar_step_vec_kernel

inline void set_err(pmenv* h, const char* fmt, ...) {
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

inline pmenv_dev::StepParams base_params(const pmenv* h) {
    using pmenv_dev::make_fastdiv;
    pmenv_dev::StepParams p;
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

// the relay step's deferral list ({epoch, count} + one entry per tile) and tile claims, 16-B padded
inline size_t relay_list_bytes(const pmenv* h) {
    const size_t tiles = h->relay_tiles;
    return ((tiles + 1) * 8 + 15) / 16 * 16 + (tiles * 4 + 15) / 16 * 16;
}

inline int check_launch(pmenv* h, const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_err(h, "%s launch failed: %s", what, hipGetErrorString(e));
        return PMENV_ERR_HIP;
    }
    return PMENV_OK;
}

// Geometry of the row-kernel stream (the fallback of the flat stream): units of R whole
// asset rows per `block`-thread workgroup, R*W*F floats <= 4*block*V (V float4 per
// thread) and R*W*F % 4 == 0 so every unit starts 16-B aligned. `v_order` lists V in
// preference order; want_rows > 0 forces R (tools A/B). Returns false when the shape
// needs the LDS fallback.
inline bool plan_streaming(const pmenv_cfg& c, const int* v_order, int block, int want_rows, int* unit_rows,
                           int* vec_per_thread) {
    const int64_t WF = (int64_t)c.window * c.features;
    if (c.features != 5 || ((int64_t)c.num_assets * WF) % 4 != 0) return false;
    int align = 1;                       // rows per unit must be a multiple of this
    while ((align * WF) % 4 != 0) ++align;
    static const int kAscending[3] = {1, 2, 4};
    if (want_rows > 0) v_order = kAscending;   // a forced unit takes the fewest float4 per thread that hold it
    for (int vi = 0; vi < 3; ++vi) {
        const int V = v_order[vi];
        const int64_t cap = (int64_t)block * 4 * V;
        int R = (int)(cap / WF);
        if (R >= c.num_assets) R = c.num_assets;
        else R -= R % align;
        if (R < 1 || (int64_t)R * WF > cap) continue;
        if (want_rows > 0) {
            if (want_rows > R) continue;
            if (want_rows != c.num_assets && want_rows % align) return false;
            R = want_rows;
        }
        *unit_rows = R;
        *vec_per_thread = V;
        return true;
    }
    return false;
}

// The one-workgroup-per-env step with V chunks per lane: waves per workgroup and whether
// the shape fits (F = 5, W >= 2, N <= 64: the scalar step on one wave; the env's 1 KiB
// blocks in at most 16 waves and 64 KiB of LDS)
inline void plan_one(pmenv* h, int V) {
    const pmenv_cfg& c = h->cfg;
    const int64_t per = (int64_t)c.num_assets * c.window * c.features;
    // the env's chunks start anywhere in a 64-chunk block: up to 63 slots ahead of it
    const uint32_t blocks = (h->per4 + 63u + 63u) / 64u;
    h->one_waves = (int)((blocks + (uint32_t)V - 1) / (uint32_t)V);
    h->one_ok = h->streaming && c.features == 5 && c.window >= 2 && c.num_assets <= 64 && per % 4 == 0 &&
                h->one_waves <= 16 && ((int64_t)64 * V * h->one_waves + 2) * 16 <= 65536;
}

// The flat one-launch step in `block` x `vec` tiles: the flat stream's shape rules, at
// most one env per wave in a tile, N <= 64 — or, for wide envs (64 < N <= 512,
// step_flat_vec_kernel), the rows a tile touches per env within one wave's 64 staged bar
// rows (W >= 14 at F = 5 for 16 KiB tiles)
inline bool flat1_fits(const pmenv* h, int block, int vec) {
    const pmenv_cfg& c = h->cfg;
    const int64_t WF = (int64_t)c.window * c.features;
    const uint32_t cpw = (uint32_t)(block * vec);
    const uint32_t ne_max = h->per4 ? (cpw + h->per4 - 2u) / h->per4 + 1u : 0u;
    const int64_t span_rows = (4ll * cpw - 1) / (WF > 0 ? WF : 1) + 2;
    const bool wide_ok = c.num_assets <= pmenv_dev::kWideMaxAssets && span_rows <= 64;
    return h->flat_ok && (c.num_assets <= 64 || wide_ok) && ne_max <= (uint32_t)(block / 64);
}

inline int64_t window_bytes(const pmenv_cfg& c) {
    return (int64_t)c.num_envs * c.num_assets * c.window * c.features * 4;
}

}  // namespace pmenv_host

// ---------------------------------------------------------------- tools-build hooks
// Defined weak (doing nothing) in pmenv.hip; tools/ab/pmenv_ab.hip defines them for
// tools/libpmenv_ab.so. A launch hook returns true when it enqueued the launch itself.
namespace pmenv_dev {
struct RelayParams;
}

namespace pmenv_tools {
void plan(pmenv* h);        // after the product's shape plan, before any allocation
void release(pmenv* h);
bool launch_scalar(const pmenv* h, const pmenv_dev::StepParams& p, hipStream_t stream);
bool launch_advance(const pmenv* h, const pmenv_dev::StepParams& p, hipStream_t stream);
bool launch_one(const pmenv* h, const pmenv_dev::StepParams& p, hipStream_t stream);
bool launch_small(const pmenv* h, const pmenv_dev::StepParams& p, hipStream_t stream);
bool launch_gen(const pmenv* h, const pmenv_dev::StepParams& p, hipStream_t stream);
bool launch_fused(const pmenv* h, const pmenv_dev::StepParams& p, int fuse_bit, uint32_t phases, hipStream_t stream);
bool launch_relay(const pmenv* h, const pmenv_dev::StepParams& p, const pmenv_dev::RelayParams& r, unsigned grid,
                  hipStream_t stream);
bool launch_flat1(const pmenv* h, const pmenv_dev::StepParams& p, unsigned grid, bool out, int pol,
                  hipStream_t stream);
bool gae(const float* rewards, const float* values, const uint8_t* dones, float* adv, float* ret, int32_t T,
         int32_t B, float gamma, float lam, hipStream_t stream, int* rc);
bool replay_gather(const float* series, int32_t T, int32_t N, int32_t F, int32_t W, const int32_t* days,
                   const float* actions, const float* rewards, int32_t H, int32_t B, const int32_t* h0,
                   const int32_t* env, int32_t S, float* s, float* s_next, float* a_out, float* r_out,
                   hipStream_t stream, int* rc);
bool rollout_gather(const float* series, int32_t T, int32_t N, int32_t F, int32_t W, const int32_t* start,
                    const float* weights, int32_t T_rec, int32_t B, int32_t ring_mode, const int32_t* t_idx,
                    const int32_t* env, int32_t S, float* s, hipStream_t stream, int* rc);
bool metrics(const double* returns, const double* values, const float* weights, int32_t T, int32_t B, int32_t N,
             double risk_free_rate, double periods, double* out, hipStream_t stream, int* rc);
bool batch_reward_forward(const float* a, const float* v_prev, const float* p, int32_t B, int32_t N,
                          int32_t reward_kind, int32_t norm, double scale, double* work, float* reward_out,
                          float* ret_out, hipStream_t stream, int* rc);
}  // namespace pmenv_tools
