// pmenv_ab.hip — the tools build's half of tools/libpmenv_ab.so (linked with the product's
// pm-rl_amd/csrc/pmenv.hip): the pmenv_tools hooks of handle.h, which read the PMENV_*
// A/B knobs and launch the alternatives the product was measured against — other
// workgroup geometries, cache policies, the ds_bpermute stream, the packed scalar-step
// shapes for N <= 64, the previous one-launch form (advance_rows_kernel<fused>), the
// timing-only ablations that skip work, the pipelined / multi-env GAE tiles, the
// non-persistent replay gathers, the two-launch metrics, the one-launch batched reward.
// The tools/ab_*.py harnesses load this library; bench.py and the tests never do (the
// product library reads no environment variable: tests/test_abi.py).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../pm-rl_amd/csrc/data.h"
#include "../../pm-rl_amd/csrc/gae_vec.h"
#include "../../pm-rl_amd/csrc/handle.h"
#include "../../pm-rl_amd/csrc/launch.h"
#include "../../pm-rl_amd/csrc/replay.h"
#include "../../pm-rl_amd/csrc/rollout.h"
#include "../../pm-rl_amd/csrc/trainer.h"
#include "ab_kernels.h"

using namespace pmenv_dev;
using namespace pmenv_host;

namespace {

const char* knob(const char* name) { return getenv(name); }
int knob_int(const char* name, int dflt) {
    const char* v = getenv(name);
    return v ? atoi(v) : dflt;
}

// the knob state of one handle (pmenv::tools)
struct Tools {
    int k1_occ = 0;             // PMENV_K1_OCC: the 8-asset packed scalar step held to 6 / 8 waves per SIMD
    int ablate = 0;             // PMENV_ABLATE: timing-only variants (64 + SKIP: flat stream, 128 + ABL: step_env)
    bool one_nocap = false;     // PMENV_ONE_NOCAP: step_env_kernel without the 80-SGPR cap
    bool flat_s80 = false;      // PMENV_FLAT_S80: the in-place flat stream held to 80 SGPRs
    int flat1_lds_pad = 0;      // PMENV_FLAT1_LDS_PAD: extra LDS per flat-step workgroup (occupancy study)
    bool flat1_xcd = false;     // PMENV_FLAT1_XCD: XCD-contiguous tile ranges
    int flat1_pol = 0;          // PMENV_FLAT1_POL: 3 nt loads only, 4 nt stores only, 5 sc0 nt, 6 sc1 nt, 7 nt + sc1 nt
    int fused = 0, fused_vec = 4;   // PMENV_FUSED: advance_rows_kernel<fused> (db | all)
    int stream_block = 512;     // PMENV_STREAM_BLOCK: row-kernel workgroup (128 | 256)
    int relay_spin = -1;        // PMENV_RELAY_SPIN: a tile's polls before it runs a missing unit (-1: product's)
    bool relay_tiles_first = false;   // PMENV_RELAY_TILES_FIRST: the tiles at blockIdx 0.., the scalar blocks last
    bool relay_stamps = false;  // PMENV_RELAY_STAMPS: the product's relay step with wall-clock stamps (step_relay.h)
    int stream_pol = 0;         // PMENV_STREAM_POL: 0 | 1 (nt) | 2 (sc0 nt)
    int flat_block = 512;       // PMENV_FLAT_BLOCK: the ds_bpermute stream's workgroup
    bool flat_db_wg = true;     // PMENV_FLAT_DB_WG=0: the ds_bpermute double-buffered stream
    int k1_groups = 1;          // PMENV_K1_GROUPS: env groups per wave of scalar_step_reg_kernel
    int one_v = kOneV;          // PMENV_ONE_V: step_env_kernel chunks per lane
    // in-place stream variants, read at create like every knob here (ab_libs.py sets them
    // only while it creates the handle): PMENV_FLAT_DIRECT (+ _ABL SKIP bits), PMENV_STREAM_BARE
    // (1: no compose, no side data; 2: no compose), PMENV_FLAT_LSIDE (bar rows / w' via LDS)
    int flat_direct = 0, flat_direct_abl = 0, stream_bare = 0;
    bool flat_lside = false;
    bool flat_perelem = false;  // PMENV_FLAT_PERELEM: the stream's per-element compose (flat_wg_body)
    int small_abl = -1;         // PMENV_SMALL_ABL: small_stamp_kernel (stamps, + ablation bits), -1 = product
    bool tiny_off = false;      // PMENV_TINY_OFF: step_small_kernel where the product runs step_tiny_kernel
    bool gen_perelem = false;   // PMENV_GEN_PERELEM: advance_gen_kernel's per-element compose, dword reads
    bool gen_pol0 = false;      // PMENV_GEN_POL0: advance_gen_kernel with the default cache policy everywhere
    int gen_abl = 0;            // PMENV_GEN_ABL: advance_gen_kernel's timing-only ablations (in place, nt)
    uint32_t small_slot = 0;    // its stamp slot, one per launch
};

Tools* tools(const pmenv* h) { return static_cast<Tools*>(h->tools); }

bool is_product_k1(int v) { return v == 0 || v == kK1Str + 801 || v == kK1Str + 1601 || v == kK1Str + 6402 || v == kK1Str + 6404 || v == kK1Str + 6408; }

// ---------------------------------------------------------------- the two-launch stream
template <int BLOCK, int V, int ABL, int POL>
void advance_rows_bv(const StepParams& p, unsigned grid, hipStream_t stream) {
    if (p.obs_out == p.obs)
        advance_rows_kernel<BLOCK, V, true, ABL, false, POL><<<grid, BLOCK, 0, stream>>>(p);
    else
        advance_rows_kernel<BLOCK, V, false, ABL, false, POL><<<grid, BLOCK, 0, stream>>>(p);
}
template <int BLOCK, int ABL, int POL>
void advance_rows_b(int vec, const StepParams& p, unsigned grid, hipStream_t stream) {
    if (vec == 1) advance_rows_bv<BLOCK, 1, ABL, POL>(p, grid, stream);
    else if (vec == 2) advance_rows_bv<BLOCK, 2, ABL, POL>(p, grid, stream);
    else advance_rows_bv<BLOCK, 4, ABL, POL>(p, grid, stream);
}
template <int POL>
void advance_rows_p(int block, int vec, const StepParams& p, unsigned grid, hipStream_t stream) {
    if (block == 128) advance_rows_b<128, 0, POL>(vec, p, grid, stream);
    else if (block == 256) advance_rows_b<256, 0, POL>(vec, p, grid, stream);
    else advance_rows_b<kStreamBlock, 0, POL>(vec, p, grid, stream);
}

// double-buffered: the ds_bpermute form (one chunk per thread) or the sc0 nt policy;
// false: the product's stream
bool flat_db(const pmenv* h, const Tools* t, StepParams p, hipStream_t stream) {
    const pmenv_cfg& c = h->cfg;
    const uint32_t per4 = (uint32_t)((int64_t)c.num_assets * c.window * c.features / 4);
    const uint32_t qtot = (uint32_t)((int64_t)c.num_envs * per4);
    p.div_units = make_fastdiv(per4);
    if (t->flat_perelem) {                        // the per-element compose, the product's 512 x 2 geometry
        const unsigned gp = (unsigned)((qtot + 1023) / 1024);
        if (h->flat_pol == 1) advance_flat_wg_perelem_kernel<512, 2, 1><<<gp, 512, 0, stream>>>(p, qtot);
        else advance_flat_wg_perelem_kernel<512, 2, 0><<<gp, 512, 0, stream>>>(p, qtot);
        return true;
    }
    if (!t->flat_db_wg) {
        const int bk = t->flat_block;
        const unsigned grid = (unsigned)((qtot + bk - 1) / bk);
#define PMENV_FLATB(BK)                                                                             \
        if (bk == BK) {                                                                             \
            if (h->flat_pol == 1) advance_flat_kernel<BK, 1><<<grid, BK, 0, stream>>>(p, qtot);      \
            else if (h->flat_pol == 2) advance_flat_kernel<BK, 2><<<grid, BK, 0, stream>>>(p, qtot); \
            else advance_flat_kernel<BK, 0><<<grid, BK, 0, stream>>>(p, qtot);                       \
            return true;                                                                            \
        }
        PMENV_FLATB(128) PMENV_FLATB(512) PMENV_FLATB(256)
#undef PMENV_FLATB
    }
    if (h->flat_pol == 2) {
        advance_flat_wg_kernel<512, 2, 2><<<(unsigned)((qtot + 1023) / 1024), 512, 0, stream>>>(p, qtot);
        return true;
    }
    return false;
}

// in place: the timing-only ablations, the 80-SGPR form, other geometries and policies
bool flat_inplace(const pmenv* h, const Tools* t, StepParams p, hipStream_t stream) {
    const pmenv_cfg& c = h->cfg;
    const uint32_t per4 = (uint32_t)((int64_t)c.num_assets * c.window * c.features / 4);
    p.div_units = make_fastdiv(per4);
    p.halo = h->halo;
    const int cpw = h->flat_ip_block * h->flat_ip_vec;
    const unsigned grid = (unsigned)((h->flat_qtot + cpw - 1) / cpw);
    const int key = h->flat_ip_block * 10 + h->flat_ip_vec;
    const int pol = h->flat_ip_pol;
    if (key == 2562 && t->stream_bare) {                      // timing only: no compose (and no side data)
        if (t->stream_bare == 2) advance_flat_inplace_kernel<256, 2, 0, 128><<<grid, 256, 0, stream>>>(p, h->flat_qtot);
        else advance_flat_inplace_kernel<256, 2, 0, 128 + 15><<<grid, 256, 0, stream>>>(p, h->flat_qtot);
        return true;
    }
    if (t->flat_perelem && (key == 2562 || key == 5122)) {     // the per-element compose (before round 3)
        if (key == 2562) advance_flat_inplace_perelem_kernel<256, 2, 0><<<grid, 256, 0, stream>>>(p, h->flat_qtot);
        else if (pol == 1) advance_flat_inplace_perelem_kernel<512, 2, 1><<<grid, 512, 0, stream>>>(p, h->flat_qtot);
        else advance_flat_inplace_perelem_kernel<512, 2, 0><<<grid, 512, 0, stream>>>(p, h->flat_qtot);
        return true;
    }
    if (key == 2562 && t->flat_lside) {                       // bar rows and w' staged in LDS per wave
        advance_flat_inplace_lside_kernel<256, 2, 0><<<grid, 256, 0, stream>>>(p, h->flat_qtot);
        return true;
    }
    if (key == 2562 && t->ablate > 64 && t->ablate < 80) {   // the product's cache-resident geometry, side data skipped
        switch (t->ablate - 64) {
            case 1: advance_flat_inplace_kernel<256, 2, 0, 1><<<grid, 256, 0, stream>>>(p, h->flat_qtot); break;
            case 2: advance_flat_inplace_kernel<256, 2, 0, 2><<<grid, 256, 0, stream>>>(p, h->flat_qtot); break;
            case 4: advance_flat_inplace_kernel<256, 2, 0, 4><<<grid, 256, 0, stream>>>(p, h->flat_qtot); break;
            default: advance_flat_inplace_kernel<256, 2, 0, 15><<<grid, 256, 0, stream>>>(p, h->flat_qtot); break;
        }
        return true;
    }
    if (t->ablate >= 64 && t->ablate < 128 && cpw != 512) return false;   // its 512 x 1 tiles need the 512-chunk halo
    if (t->ablate >= 64 && t->ablate < 128) {     // PMENV_ABLATE = 64 + SKIP bits
        const unsigned g1 = (unsigned)((h->flat_qtot + 511) / 512);
#define PMENV_ABL(X) case 64 + X: advance_flat_inplace_kernel<512, 1, 1, X><<<g1, 512, 0, stream>>>(p, h->flat_qtot); break;
        switch (t->ablate) {
            PMENV_ABL(1) PMENV_ABL(2) PMENV_ABL(4) PMENV_ABL(6) PMENV_ABL(15) PMENV_ABL(31) PMENV_ABL(32)
            PMENV_ABL(33)
            default: break;
        }
#undef PMENV_ABL
        return true;
    }
    if (t->flat_s80 && key == 5122) {
        if (pol == 1) advance_flat_inplace_s80_kernel<512, 2, 1><<<grid, 512, 0, stream>>>(p, h->flat_qtot);
        else advance_flat_inplace_s80_kernel<512, 2, 0><<<grid, 512, 0, stream>>>(p, h->flat_qtot);
        return true;
    }
    const bool product = (key == 2562 && pol == 0) || (key == 5122 && pol <= 1);
    if (product) return false;
#define PMENV_FIP(BK, V)                                                                                      \
    if (key == BK * 10 + V) {                                                                                 \
        if (pol == 1) advance_flat_inplace_kernel<BK, V, 1><<<grid, BK, 0, stream>>>(p, h->flat_qtot);         \
        else if (pol == 2) advance_flat_inplace_kernel<BK, V, 2><<<grid, BK, 0, stream>>>(p, h->flat_qtot);    \
        else advance_flat_inplace_kernel<BK, V, 0><<<grid, BK, 0, stream>>>(p, h->flat_qtot);                  \
        return true;                                                                                          \
    }
    PMENV_FIP(256, 1) PMENV_FIP(256, 2) PMENV_FIP(256, 4) PMENV_FIP(512, 1) PMENV_FIP(512, 2) PMENV_FIP(1024, 1)
#undef PMENV_FIP
    return false;
}

bool advance_rows(const pmenv* h, const Tools* t, StepParams p, hipStream_t stream) {
    const bool db = p.obs_out != p.obs;
    p.unit_rows = db ? h->unit_rows_db : h->unit_rows;
    p.units_per_env = db ? h->units_per_env_db : h->units_per_env;
    p.div_units = make_fastdiv((uint32_t)p.units_per_env);
    const int vec = db ? h->stream_vec_db : h->stream_vec;
    const unsigned grid = (unsigned)(h->cfg.num_envs * p.units_per_env);
    switch (t->ablate) {     // timing-only builds: 512-thread geometry, default policy
    case 1: advance_rows_b<kStreamBlock, 1, 0>(vec, p, grid, stream); return true;
    case 2: advance_rows_b<kStreamBlock, 2, 0>(vec, p, grid, stream); return true;
    case 3: advance_rows_b<kStreamBlock, 3, 0>(vec, p, grid, stream); return true;
    case 7: advance_rows_b<kStreamBlock, 7, 0>(vec, p, grid, stream); return true;
    default: break;
    }
    if (t->stream_pol == 0 && t->stream_block == kStreamBlock) return false;
    if (t->stream_pol == 2) advance_rows_p<2>(t->stream_block, vec, p, grid, stream);
    else if (t->stream_pol == 1) advance_rows_p<1>(t->stream_block, vec, p, grid, stream);
    else advance_rows_p<0>(t->stream_block, vec, p, grid, stream);
    return true;
}

// ---------------------------------------------------------------- the first launch: packed shapes for N <= 64
template <int L, int A, bool STR>
void scalar_vec_la(const StepParams& p, hipStream_t stream) {
    const unsigned waves = (unsigned)((p.B + 64 / L - 1) / (64 / L));
    scalar_step_vec_kernel<L, A, STR><<<(waves + 3) / 4, 256, 0, stream>>>(p);
}

bool scalar_vec_ab(int vec, const StepParams& p, hipStream_t stream) {
    switch (vec) {
    case 801: scalar_vec_la<8, 1, false>(p, stream); return true;
    case 802: scalar_vec_la<8, 2, false>(p, stream); return true;
    case 804: scalar_vec_la<8, 4, false>(p, stream); return true;
    case 1601: scalar_vec_la<16, 1, false>(p, stream); return true;
    case 1602: scalar_vec_la<16, 2, false>(p, stream); return true;
    case 1604: scalar_vec_la<16, 4, false>(p, stream); return true;
    case 1608: scalar_vec_la<16, 8, false>(p, stream); return true;
    case 3202: scalar_vec_la<32, 2, false>(p, stream); return true;
    case 3204: scalar_vec_la<32, 4, false>(p, stream); return true;
    case kK1Str + 3202: scalar_vec_la<32, 2, true>(p, stream); return true;
    case kK1Str + 3204: scalar_vec_la<32, 4, true>(p, stream); return true;
    default: return false;
    }
}

template <int L>
void scalar_reg_groups(int groups, const StepParams& p, hipStream_t stream) {
    const int per_wave = (64 / L) * groups;
    const unsigned waves = (unsigned)((p.B + per_wave - 1) / per_wave);
    const unsigned grid = (waves + 3) / 4;
    if (groups == 4) scalar_step_reg_kernel<L, 4><<<grid, 256, 0, stream>>>(p);
    else if (groups == 2) scalar_step_reg_kernel<L, 2><<<grid, 256, 0, stream>>>(p);
    else scalar_step_reg_kernel<L, 1><<<grid, 256, 0, stream>>>(p);
}

// ---------------------------------------------------------------- one workgroup per env
template <int V>
void one_v(const pmenv* h, const Tools* t, const StepParams& p, hipStream_t stream) {
    const bool out = p.obs_out != p.obs;
    const int pol = out ? h->flat_pol : h->flat_ip_pol;
    const unsigned threads = 64u * (unsigned)h->one_waves;
    const size_t lds = ((size_t)threads * V + 2) * 16 + (size_t)knob_int("PMENV_ONE_LDS_PAD", 0);
    const unsigned grid = (unsigned)h->cfg.num_envs;
    if (t->ablate >= 128 && t->ablate < 144) {    // timing-only / A/B bits (step_env.h ABL), nt policy
#define PMENV_ONEABL(X)                                                                                     \
        case 128 + X:                                                                                     \
            if (out) step_env_kernel<V, true, 1, X><<<grid, threads, lds, stream>>>(p, h->per4);            \
            else step_env_kernel<V, false, 1, X><<<grid, threads, lds, stream>>>(p, h->per4);               \
            return;
        switch (t->ablate) {
            PMENV_ONEABL(1) PMENV_ONEABL(2) PMENV_ONEABL(4) PMENV_ONEABL(8) PMENV_ONEABL(12)
            default: break;
        }
#undef PMENV_ONEABL
    }
    if (t->one_nocap) {
        if (out && pol == 1) step_env_nocap_kernel<V, true, 1><<<grid, threads, lds, stream>>>(p, h->per4);
        else if (out) step_env_nocap_kernel<V, true, 0><<<grid, threads, lds, stream>>>(p, h->per4);
        else if (pol == 1) step_env_nocap_kernel<V, false, 1><<<grid, threads, lds, stream>>>(p, h->per4);
        else step_env_nocap_kernel<V, false, 0><<<grid, threads, lds, stream>>>(p, h->per4);
        return;
    }
    if (out) {
        if (pol == 1) step_env_kernel<V, true, 1><<<grid, threads, lds, stream>>>(p, h->per4);
        else step_env_kernel<V, true, 0><<<grid, threads, lds, stream>>>(p, h->per4);
    } else {
        if (pol == 1) step_env_kernel<V, false, 1><<<grid, threads, lds, stream>>>(p, h->per4);
        else step_env_kernel<V, false, 0><<<grid, threads, lds, stream>>>(p, h->per4);
    }
}

// ---------------------------------------------------------------- the flat one-launch step
template <int BK, int VV>
void flat1_pad(const pmenv* h, const StepParams& p, unsigned grid, bool out, int pol, size_t pad, hipStream_t stream) {
    if (out) {
        if (pol == 1) step_flat_kernel<BK, VV, 1, true><<<grid, BK, pad, stream>>>(p, h->flat_qtot);
        else step_flat_kernel<BK, VV, 0, true><<<grid, BK, pad, stream>>>(p, h->flat_qtot);
    } else {
        if (pol == 1) step_flat_kernel<BK, VV, 1, false><<<grid, BK, pad, stream>>>(p, h->flat_qtot);
        else step_flat_kernel<BK, VV, 0, false><<<grid, BK, pad, stream>>>(p, h->flat_qtot);
    }
}

template <int A>
void flat1_vec_128(const StepParams& p, uint32_t qtot, unsigned grid, bool out, int pol, hipStream_t stream) {
    if (out) {
        if (pol == 1) step_flat_vec_kernel<A, 128, 8, 1, true><<<grid, 128, 0, stream>>>(p, qtot);
        else step_flat_vec_kernel<A, 128, 8, 0, true><<<grid, 128, 0, stream>>>(p, qtot);
    } else {
        if (pol == 1) step_flat_vec_kernel<A, 128, 8, 1, false><<<grid, 128, 0, stream>>>(p, qtot);
        else step_flat_vec_kernel<A, 128, 8, 0, false><<<grid, 128, 0, stream>>>(p, qtot);
    }
}

}  // namespace

// ---------------------------------------------------------------- the hooks
namespace pmenv_tools {

void plan(pmenv* h) {
    Tools* t = new Tools;
    h->tools = t;
    const pmenv_cfg& c = h->cfg;
    const int64_t win = window_bytes(c);
    static const int kInplaceOrder[3] = {2, 4, 1}, kDoubleOrder[3] = {4, 2, 1};
    // the row-kernel stream: workgroup size and forced unit rows
    {
        const int bk = knob_int("PMENV_STREAM_BLOCK", kStreamBlock);
        if (bk == 128 || bk == 256) t->stream_block = bk;
        const int want = knob_int("PMENV_UNIT_ROWS", 0);
        if (want > 0 || t->stream_block != kStreamBlock) {
            h->streaming = plan_streaming(c, kInplaceOrder, t->stream_block, want, &h->unit_rows, &h->stream_vec) &&
                           plan_streaming(c, kDoubleOrder, t->stream_block, want, &h->unit_rows_db, &h->stream_vec_db);
            h->flat_ok = h->flat_ok && h->streaming;
        }
    }
    if (const char* k = knob("PMENV_STREAM_POL")) {       // 0 | 1 (nt) | 2 (sc0 nt), every stream
        const int pol = atoi(k);
        if (pol >= 0 && pol <= 2) t->stream_pol = h->flat_pol = h->flat_ip_pol = pol;
    }
    if (const char* k = knob("PMENV_FLAT")) h->flat = h->flat_ok && atoi(k) != 0;
    if (const char* k = knob("PMENV_FLAT_INPLACE")) h->flat_inplace = h->flat_ok && atoi(k) != 0;
    t->flat_db_wg = knob_int("PMENV_FLAT_DB_WG", 1) != 0;
    h->flat_ip_block = knob_int("PMENV_FLAT_IP_BLOCK", h->flat_ip_block);
    h->flat_ip_vec = knob_int("PMENV_FLAT_IP_VEC", h->flat_ip_vec);
    {   // the launcher's (block, vec) table: anything else takes the default 512 x 2
        const int key = h->flat_ip_block * 10 + h->flat_ip_vec;
        if (key != 2561 && key != 2562 && key != 2564 && key != 5121 && key != 5122 && key != 10241) {
            h->flat_ip_block = 512;
            h->flat_ip_vec = 2;
        }
    }
    {
        const int bk = knob_int("PMENV_FLAT_BLOCK", 512);
        if (bk == 128 || bk == 256 || bk == 512) t->flat_block = bk;
    }
    t->ablate = knob_int("PMENV_ABLATE", 0);
    t->k1_occ = knob_int("PMENV_K1_OCC", 0);
    if (const char* k = knob("PMENV_RELAY_GEOM")) {   // BLOCK x V of relay_geom's table: N <= 64 forms only
        int bk = 0, v = 0;
        const int g = sscanf(k, "%dx%d", &bk, &v) == 2 ? bk * 10 + v : 0;
        const int form = h->relay_kl * 100 + h->relay_ka;
        const bool rows_fit = g && 4 * bk * v / (h->cfg.window * 5) + 2 <= bk;   // one staged row per thread
        if ((g == 1282 || g == 1284 || g == 2564 || g == 2561 || g == 2568 || g == 5124) && rows_fit &&
            (form == 801 || form == 1601 || form == 3200 || form == 6400)) {
            h->relay_block = bk;
            h->relay_v = v;
        }
    }
    t->relay_spin = knob_int("PMENV_RELAY_SPIN", -1);
    t->relay_tiles_first = knob_int("PMENV_RELAY_TILES_FIRST", 0) != 0;
    t->relay_stamps = knob_int("PMENV_RELAY_STAMPS", 0) != 0;
    if (const char* k = knob("PMENV_SMALL_GEOM")) {   // step_small_kernel's BLOCK x E: 64x32 | 256x8 | 256x16 | ...
        int bk = 0, e = 0;
        const int64_t nwf = (int64_t)c.num_assets * c.window * c.features;
        if (sscanf(k, "%dx%d", &bk, &e) == 2 && (int64_t)bk * e >= nwf &&
            (bk * 100 + e == 6432 || bk * 100 + e == 25608 || bk * 100 + e == 25616 || bk * 100 + e == 51216 ||
             bk * 100 + e == 102416)) {
            h->small_block = bk;
            h->small_e = e;
        }
    }
    t->small_abl = knob_int("PMENV_SMALL_ABL", -1);
    t->tiny_off = knob_int("PMENV_TINY_OFF", 0) != 0;
    if (const char* k = knob("PMENV_SURF_STREAM")) h->surf_stream = h->surf_stream && atoi(k) != 0;
    t->gen_perelem = knob_int("PMENV_GEN_PERELEM", 0) != 0;
    t->gen_pol0 = knob_int("PMENV_GEN_POL0", 0) != 0;
    t->gen_abl = knob_int("PMENV_GEN_ABL", 0);
    if (knob_int("PMENV_GEN_OFF", 0)) h->gen_auto = 0;   // AUTO keeps the register step for F != 5
    if (const char* k = knob("PMENV_GEN_GEOM")) {     // advance_gen_kernel's BLOCK x V: 256x4 | 256x2 | 512x2 | 512x4 | 1024x2
        int bk = 0, v = 0;
        const int g = sscanf(k, "%dx%d", &bk, &v) == 2 ? bk * 10 + v : 0;
        if (h->gen_ok && (g == 2564 || g == 2562 || g == 5122 || g == 5124 || g == 10242)) {
            h->gen_block = bk;
            h->gen_v = v;
        }
    }
    t->one_nocap = knob_int("PMENV_ONE_NOCAP", 0) != 0;
    t->flat1_lds_pad = knob_int("PMENV_FLAT1_LDS_PAD", 0);
    t->flat_s80 = knob_int("PMENV_FLAT_S80", 0) != 0;
    t->k1_groups = knob_int("PMENV_K1_GROUPS", 1);
    if (t->k1_groups != 2 && t->k1_groups != 4) t->k1_groups = 1;
    // K1: the packed shapes for N <= 64 (this build's default there, as measured in round 2:
    // they reduce in another order than the one-launch steps), or the PMENV_K1 knob
    // ("reg" | "LxA" | "LxAs" strided, e.g. "16x2", "64x8s")
    if ((int64_t)c.num_envs * c.num_assets * 4 < (1ll << 32)) {
        const int N = c.num_assets;
        if (N <= 8) h->k1_vec = 801;
        else if (N <= 16) h->k1_vec = 802;
        else if (N <= 32) h->k1_vec = 1602;
        else if (N <= 64) h->k1_vec = 1604;
        if (const char* k = knob("PMENV_K1")) {
            static const int kK1Vec[] = {801, 802, 804, 1601, 1602, 1604, 1608, 3202, 3204,
                                         kK1Str + 3202, kK1Str + 3204, kK1Str + 6402, kK1Str + 6404, kK1Str + 6408};
            int L = 0, A = 0;
            char s = 0;
            if (!strcmp(k, "reg")) {
                h->k1_vec = 0;
            } else if (sscanf(k, "%dx%d%c", &L, &A, &s) >= 2) {
                const int want = 100 * L + A + (s == 's' ? kK1Str : 0);
                for (int v : kK1Vec)
                    if (v == want && L * A >= N) h->k1_vec = v;
            }
        }
    }
    if (const char* k = knob("PMENV_ADVANCE"))   // "lds": force the single-launch LDS kernel
        if (!strcmp(k, "lds")) {
            h->streaming = h->flat = h->flat_inplace = false;
            h->one_ok = h->flat1_ok = false;
            h->one_auto = h->flat1_auto = 0;
        }
    // the one-workgroup-per-env step: chunks per lane, forced windows
    const int one_rule = [&] {
        return h->one_ok && (win <= (48ll << 20) || !h->flat_inplace) ? (PMENV_FUSE_DB | PMENV_FUSE_INPLACE) : 0;
    }();
    t->flat_direct = knob_int("PMENV_FLAT_DIRECT", 0);
    t->flat_direct_abl = knob_int("PMENV_FLAT_DIRECT_ABL", 0);
    t->stream_bare = knob_int("PMENV_STREAM_BARE", 0);
    t->flat_lside = knob_int("PMENV_FLAT_LSIDE", 0) != 0;
    t->flat_perelem = knob_int("PMENV_FLAT_PERELEM", 0) != 0;
    t->one_v = knob_int("PMENV_ONE_V", kOneV);
    if (t->one_v != 1 && t->one_v != 2 && t->one_v != 3 && t->one_v != 6 && t->one_v != 8) t->one_v = kOneV;
    if (t->one_v != kOneV) {
        plan_one(h, t->one_v);
        h->one_auto = (h->one_ok && (win <= (48ll << 20) || !h->flat_inplace) ? (PMENV_FUSE_DB | PMENV_FUSE_INPLACE)
                                                                              : 0) & ~h->flat1_auto;
    }
    if (const char* k = knob("PMENV_ONE")) {    // 0 | db | ip | all
        if (!h->one_ok || !strcmp(k, "0")) h->one_auto = 0;
        else if (!strcmp(k, "db")) h->one_auto = PMENV_FUSE_DB;
        else if (!strcmp(k, "ip")) h->one_auto = PMENV_FUSE_INPLACE;
        else if (!strcmp(k, "all")) h->one_auto = PMENV_FUSE_DB | PMENV_FUSE_INPLACE;
    }
    {   // the previous one-launch form (advance_rows_kernel<fused>), PMENV_FUSED = db | all
        int fused_rows = 0;
        const bool fusable = h->streaming && c.num_assets <= 64 && !t->ablate &&
                             plan_streaming(c, kDoubleOrder, kStreamBlock, 0, &fused_rows, &t->fused_vec) &&
                             fused_rows == c.num_assets;
        if (const char* k = knob("PMENV_FUSED")) {
            if (fusable && !strcmp(k, "db")) t->fused = PMENV_FUSE_DB;
            else if (fusable && !strcmp(k, "all")) t->fused = PMENV_FUSE_DB | PMENV_FUSE_INPLACE;
            if (t->fused) h->one_auto &= ~t->fused;
        }
    }
    // the flat one-launch step: forced on / off, tile order, cache policies, geometry
    if (const char* k = knob("PMENV_FLAT1")) {   // 1 = the flat step for every window, 0 = never
        h->flat1_auto = h->flat1_ok && atoi(k) ? (PMENV_FUSE_DB | PMENV_FUSE_INPLACE) : 0;
        h->one_auto = h->flat1_auto ? 0 : one_rule;
    }
    t->flat1_xcd = knob_int("PMENV_FLAT1_XCD", 0) != 0;
    t->flat1_pol = knob_int("PMENV_FLAT1_POL", 0);
    if (const char* k = knob("PMENV_FLAT1_GEOM")) {   // "512x2" | "512x4" | "1024x2" | "256x8" | ...
        int bk = 0, vv = 0;
        if (sscanf(k, "%dx%d", &bk, &vv) == 2) {
            const int key = bk * 100 + vv;
            const bool narrow = c.num_assets <= 64 &&
                                (key == 51202 || key == 51204 || key == 102402 || key == 25604 || key == 25608 ||
                                 key == 25602 || key == 12808 || key == 12804);
            const bool wide = c.num_assets > 64 && (key == 25604 || key == 12808);
            if ((narrow || wide) && flat1_fits(h, bk, vv)) {
                h->flat1_block = bk;
                h->flat1_vec = vv;
                h->flat1_ok = true;
            }
        }
    }
}

void release(pmenv* h) {
    delete tools(h);
    h->tools = nullptr;
}

bool launch_scalar(const pmenv* h, const StepParams& p, hipStream_t stream) {
    const Tools* t = tools(h);
    if (!t) return false;
    const bool ab_vec = !is_product_k1(h->k1_vec);
    const bool groups = t->k1_groups != 1 && h->cfg.num_assets <= 64 && h->k1_vec == 0;
    if (t->k1_occ > 0 && h->k1_vec == kK1Str + 6408 && !t->ablate) {   // the wide form held to 6 / 8 waves
        StepParams q = p;
        const unsigned grid = (unsigned)((p.B + 3) / 4);
        if (t->k1_occ >= 8) scalar_step_vec_occ_kernel<64, 8, true, 8><<<grid, 256, 0, stream>>>(q);
        else scalar_step_vec_occ_kernel<64, 8, true, 6><<<grid, 256, 0, stream>>>(q);
        return true;
    }
    if (!t->ablate && !ab_vec && !groups) return false;
    StepParams q = p;
    // the ablations of the stream skip its halo copy too, except the side-data-only ones
    // at the product's cache-resident geometry (PMENV_ABLATE = 64 + 1 / 2 / 4 / 15, 256 x 2)
    const bool side_only = t->ablate > 64 && t->ablate < 80 && h->flat_ip_block * h->flat_ip_vec == 512 &&
                           h->flat_ip_block == 256;
    if (t->ablate && !side_only) q.halo = nullptr;
    if (ab_vec) scalar_vec_ab(h->k1_vec, q, stream);
    else if (groups) {
        if (h->cfg.num_assets <= 32) scalar_reg_groups<32>(t->k1_groups, q, stream);
        else scalar_reg_groups<64>(t->k1_groups, q, stream);
    } else launch_scalar_kernels(h, q, stream);
    return true;
}

template <int BLOCK, int E>
void small_stamp(int abl, const StepParams& p, uint32_t slot, hipStream_t stream) {
    const unsigned grid = (unsigned)p.B;
    switch (abl) {
    case 0: small_stamp_kernel<BLOCK, E, 0><<<grid, BLOCK, 0, stream>>>(p, slot); break;
    case 2: small_stamp_kernel<BLOCK, E, 2><<<grid, BLOCK, 0, stream>>>(p, slot); break;
    case 4: small_stamp_kernel<BLOCK, E, 4><<<grid, BLOCK, 0, stream>>>(p, slot); break;
    case 6: small_stamp_kernel<BLOCK, E, 6><<<grid, BLOCK, 0, stream>>>(p, slot); break;
    case 8: small_stamp_kernel<BLOCK, E, 8><<<grid, BLOCK, 0, stream>>>(p, slot); break;
    default: small_stamp_kernel<BLOCK, E, 16><<<grid, BLOCK, 0, stream>>>(p, slot); break;
    }
}

bool launch_small(const pmenv* h, const StepParams& p, hipStream_t stream) {
    Tools* t = tools(h);
    if (t->tiny_off && h->tiny && t->small_abl < 0) {
        step_small_kernel<256, 8, true><<<(unsigned)h->cfg.num_envs, 256, 0, stream>>>(p);
        return true;
    }
    if (t->small_abl < 0 || h->cfg.num_assets > 64) return false;
    const uint32_t slot = t->small_slot++;
    switch (h->small_block * 100 + h->small_e) {
    case 25608: small_stamp<256, 8>(t->small_abl, p, slot, stream); break;
    default: return false;
    }
    return true;
}

// the generic stream's tools variants at the product's tile (256 x 4 as in round 5's first
// form, or 512 x 2 past 128 MiB)
template <int BLOCK, int V>
bool launch_gen_t(const pmenv* h, const StepParams& p, hipStream_t stream) {
    const unsigned grid = (unsigned)((h->gen_qtot + BLOCK * V - 1) / (BLOCK * V));
    const uint32_t rows = gen_rows(h, BLOCK * V);
    const size_t lds = (size_t)rows * 9 * 4;
    const int fm4 = h->cfg.features % 4;
    const bool ip = p.obs_out == p.obs;
    if (tools(h)->gen_pol0) {
        if (fm4 == 0 && ip) advance_gen_kernel<BLOCK, V, false, 4><<<grid, BLOCK, lds, stream>>>(p, h->gen_qtot, rows);
        else if (fm4 == 0) advance_gen_kernel<BLOCK, V, true, 4><<<grid, BLOCK, lds, stream>>>(p, h->gen_qtot, rows);
        else if (ip) advance_gen_kernel<BLOCK, V, false, 1><<<grid, BLOCK, lds, stream>>>(p, h->gen_qtot, rows);
        else advance_gen_kernel<BLOCK, V, true, 1><<<grid, BLOCK, lds, stream>>>(p, h->gen_qtot, rows);
        return true;
    }
    if (const int a = tools(h)->gen_abl; a > 0 && ip) {
#define GEN_ABL(A)                                                                                       \
    case A:                                                                                              \
        if (fm4 == 0) advance_gen_kernel<BLOCK, V, false, 4, true, 1, A><<<grid, BLOCK, lds, stream>>>(p, h->gen_qtot, rows); \
        else advance_gen_kernel<BLOCK, V, false, 1, true, 1, A><<<grid, BLOCK, lds, stream>>>(p, h->gen_qtot, rows);      \
        break;
        switch (a) { GEN_ABL(1) GEN_ABL(2) GEN_ABL(3) GEN_ABL(6) GEN_ABL(7) default: return false; }
#undef GEN_ABL
        return true;
    }
    if (!tools(h)->gen_perelem) return false;
    if (ip) advance_gen_kernel<BLOCK, V, false, 1, false><<<grid, BLOCK, lds, stream>>>(p, h->gen_qtot, rows);
    else advance_gen_kernel<BLOCK, V, true, 1, false><<<grid, BLOCK, lds, stream>>>(p, h->gen_qtot, rows);
    return true;
}

bool launch_gen(const pmenv* h, const StepParams& p, hipStream_t stream) {
    if (h->cfg.features > 8) return false;      // the tools variants stage F <= 8 (the product takes F <= 16)
    if (h->gen_block == 256 && h->gen_v == 4) return launch_gen_t<256, 4>(h, p, stream);
    if (h->gen_block == 512 && h->gen_v == 2) return launch_gen_t<512, 2>(h, p, stream);
    // tiles the product does not instantiate (PMENV_GEN_GEOM=512x4 | 1024x2)
    if (h->gen_block == 512 && h->gen_v == 4) {
        if (!launch_gen_t<512, 4>(h, p, stream)) launch_gen_g<512, 4>(h, p, stream);
        return true;
    }
    if (h->gen_block == 1024 && h->gen_v == 2) {
        if (!launch_gen_t<1024, 2>(h, p, stream)) launch_gen_g<1024, 2>(h, p, stream);
        return true;
    }
    return false;
}

bool launch_advance(const pmenv* h, const StepParams& p, hipStream_t stream) {
    const Tools* t = tools(h);
    if (!t) return false;
    const bool db = p.obs_out != p.obs;
    if (!db && h->flat_inplace && t->flat_direct) {                 // the stream without the LDS image
        StepParams q = p;
        const pmenv_cfg& c = h->cfg;
        q.div_units = make_fastdiv((uint32_t)((int64_t)c.num_assets * c.window * c.features / 4));
        q.halo = h->halo;
        const int cpw = h->flat_ip_block * h->flat_ip_vec;
        const unsigned grid = (unsigned)((h->flat_qtot + cpw - 1) / cpw);
        const int abl = t->flat_direct_abl;
        if (h->flat_ip_block == 256) {
            if (abl == 15) advance_flat_direct_kernel<256, 2, 0, 15><<<grid, 256, 0, stream>>>(q, h->flat_qtot);
            else advance_flat_direct_kernel<256, 2, 0, 0><<<grid, 256, 0, stream>>>(q, h->flat_qtot);
        } else if (h->flat_ip_pol == 1) {
            advance_flat_direct_kernel<512, 2, 1, 0><<<grid, 512, 0, stream>>>(q, h->flat_qtot);
        } else {
            advance_flat_direct_kernel<512, 2, 0, 0><<<grid, 512, 0, stream>>>(q, h->flat_qtot);
        }
        return true;
    }
    if (db && h->flat && !t->ablate) return flat_db(h, t, p, stream);
    if (!db && h->flat_inplace && (!t->ablate || (t->ablate >= 64 && t->ablate < 128)))
        return flat_inplace(h, t, p, stream);
    if ((db && h->flat) || (!db && h->flat_inplace)) {   // an ablation of the row stream on a flat shape
        if (!advance_rows(h, t, p, stream)) launch_advance_rows(h, p, stream);
        return true;
    }
    return advance_rows(h, t, p, stream);
}

bool launch_one(const pmenv* h, const StepParams& p, hipStream_t stream) {
    const Tools* t = tools(h);
    if (!t) return false;
    const bool pad = knob("PMENV_ONE_LDS_PAD") != nullptr;
    if (t->one_v == kOneV && !pad && !t->one_nocap && !(t->ablate >= 128 && t->ablate < 144)) return false;
    switch (t->one_v) {
    case 1: one_v<1>(h, t, p, stream); break;
    case 2: one_v<2>(h, t, p, stream); break;
    case 3: one_v<3>(h, t, p, stream); break;
    case 6: one_v<6>(h, t, p, stream); break;
    case 8: one_v<8>(h, t, p, stream); break;
    default: one_v<kOneV>(h, t, p, stream); break;
    }
    return true;
}

bool launch_fused(const pmenv* h, const StepParams& p0, int fuse_bit, uint32_t phases, hipStream_t stream) {
    const Tools* t = tools(h);
    if (!t || phases != (PMENV_PHASE_SCALAR | PMENV_PHASE_ADVANCE) || !(t->fused & fuse_bit)) return false;
    StepParams p = p0;
    p.unit_rows = h->cfg.num_assets;
    p.units_per_env = 1;
    p.div_units = make_fastdiv(1u);
    const unsigned grid = (unsigned)h->cfg.num_envs;
    const bool inplace = p.obs_out == p.obs;
#define PMENV_FUSED_LAUNCH(V)                                                                        \
    if (inplace) advance_rows_kernel<kStreamBlock, V, true, 0, true><<<grid, kStreamBlock, 0, stream>>>(p); \
    else advance_rows_kernel<kStreamBlock, V, false, 0, true><<<grid, kStreamBlock, 0, stream>>>(p);
    if (t->fused_vec == 1) { PMENV_FUSED_LAUNCH(1) }
    else if (t->fused_vec == 2) { PMENV_FUSED_LAUNCH(2) }
    else { PMENV_FUSED_LAUNCH(4) }
#undef PMENV_FUSED_LAUNCH
    return true;
}

// PMENV_RELAY_GEOM: the relay step's tiles in other geometries (the N <= 64 scalar forms)
template <int BK, int V, bool OUT>
static void relay_geom_o(const pmenv* h, const StepParams& p, const RelayParams& r, uint32_t q, unsigned grid,
                         hipStream_t stream) {
    switch (h->relay_kl * 100 + h->relay_ka) {
    case 801: step_relay_kernel<BK, V, 0, OUT, 8, 1><<<grid, BK, 0, stream>>>(p, r, q); break;
    case 1601: step_relay_kernel<BK, V, 0, OUT, 16, 1><<<grid, BK, 0, stream>>>(p, r, q); break;
    case 3200: step_relay_kernel<BK, V, 0, OUT, 32, 0><<<grid, BK, 0, stream>>>(p, r, q); break;
    default: step_relay_kernel<BK, V, 0, OUT, 64, 0><<<grid, BK, 0, stream>>>(p, r, q); break;
    }
}
template <int BK, int V>
static void relay_geom(const pmenv* h, const StepParams& p, const RelayParams& r, uint32_t q, unsigned grid, bool out,
                       hipStream_t stream) {
    if (out) relay_geom_o<BK, V, true>(h, p, r, q, grid, stream);
    else relay_geom_o<BK, V, false>(h, p, r, q, grid, stream);
}
bool launch_relay(const pmenv* h, const StepParams& p, const RelayParams& r, unsigned grid, hipStream_t stream) {
    const int g = h->relay_block * 10 + h->relay_v;
    const Tools* tt = tools(h);
    // the forward-progress fallback exercised: PMENV_RELAY_SPIN=0 (a tile runs a missing unit on
    // its first miss) and / or PMENV_RELAY_TILES_FIRST=1 (blockIdx rotated so every tile precedes
    // every scalar block: the tiles fill the chip and run the scalar steps themselves)
    RelayParams rr = r;
    const bool mod = tt && (tt->relay_spin >= 0 || tt->relay_tiles_first || tt->relay_stamps);
    if (tt && tt->relay_spin >= 0) rr.spin = (uint32_t)tt->relay_spin;
    if (tt && tt->relay_tiles_first) rr.rot = r.scal;
    const bool out = p.obs_out != p.obs;
    const uint32_t q = h->flat_qtot;
    // the product's geometries (256 x 2, 512 x 2, and 256 x 4 for the register form of N <= 32:
    // launch_relay_g's own rule) take the modified launches; other geometries only the A/B ones
    const bool prod_geom = g == 2562 || g == 5122 || (g == 2564 && h->relay_kl == 32 && h->relay_ka == 0);
    if (mod && prod_geom) {
        if (tt->relay_stamps && tt->relay_spin < 0 && !tt->relay_tiles_first) {   // the product's code, stamped
            if (h->relay_block == 256) launch_relay_b<256, 0, 2>(h, p, rr, grid, out, false, stream);
            else launch_relay_b<512, 1, 2>(h, p, rr, grid, out, false, stream);
        } else if (h->relay_block == 256) launch_relay_b<256, 0, 1>(h, p, rr, grid, out, false, stream);
        else launch_relay_b<512, 1, 1>(h, p, rr, grid, out, false, stream);
        return true;
    }
    switch (g) {
    case 1282: relay_geom<128, 2>(h, p, rr, q, grid, out, stream); return true;
    case 1284: relay_geom<128, 4>(h, p, rr, q, grid, out, stream); return true;
    case 2564: relay_geom<256, 4>(h, p, rr, q, grid, out, stream); return true;
    case 2561: relay_geom<256, 1>(h, p, rr, q, grid, out, stream); return true;
    case 2568: relay_geom<256, 8>(h, p, rr, q, grid, out, stream); return true;
    case 5124: relay_geom<512, 4>(h, p, rr, q, grid, out, stream); return true;
    default: return false;
    }
}

bool launch_flat1(const pmenv* h, const StepParams& p, unsigned grid, bool out, int pol, hipStream_t stream) {
    const Tools* t = tools(h);
    if (!t) return false;
    if (h->cfg.num_assets > 64) {
        if (h->flat1_block != 128) return false;
        const int N = h->cfg.num_assets;
        if (N <= 128) flat1_vec_128<2>(p, h->flat_qtot, grid, out, pol, stream);
        else if (N <= 256) flat1_vec_128<4>(p, h->flat_qtot, grid, out, pol, stream);
        else flat1_vec_128<8>(p, h->flat_qtot, grid, out, pol, stream);
        return true;
    }
    const size_t pad = (size_t)t->flat1_lds_pad;
    const int key = h->flat1_block * 100 + h->flat1_vec;
    if (key == 25604 && t->flat1_pol >= 3 && t->flat1_pol <= 7) {   // other cache policies
#define PMENV_FLAT1_POLV(PV)                                                                      \
        if (t->flat1_pol == PV) {                                                                 \
            if (out) step_flat_ab_kernel<256, 4, PV, true, false><<<grid, 256, 0, stream>>>(p, h->flat_qtot);  \
            else step_flat_ab_kernel<256, 4, PV, false, false><<<grid, 256, 0, stream>>>(p, h->flat_qtot);     \
        }
        PMENV_FLAT1_POLV(3) PMENV_FLAT1_POLV(4) PMENV_FLAT1_POLV(5) PMENV_FLAT1_POLV(6) PMENV_FLAT1_POLV(7)
#undef PMENV_FLAT1_POLV
        return true;
    }
    if (key == 25604 && t->flat1_xcd) {
        if (out) step_flat_ab_kernel<256, 4, 1, true, true><<<grid, 256, 0, stream>>>(p, h->flat_qtot);
        else step_flat_ab_kernel<256, 4, 1, false, true><<<grid, 256, 0, stream>>>(p, h->flat_qtot);
        return true;
    }
    if (key == 51204) flat1_pad<512, 4>(h, p, grid, out, pol, pad, stream);
    else if (key == 102402) flat1_pad<1024, 2>(h, p, grid, out, pol, pad, stream);
    else if (key == 25608) flat1_pad<256, 8>(h, p, grid, out, pol, pad, stream);
    else if (key == 25602) flat1_pad<256, 2>(h, p, grid, out, pol, pad, stream);
    else if (key == 12804) flat1_pad<128, 4>(h, p, grid, out, pol, pad, stream);
    else if (!pad) return false;                   // a product geometry at the product's LDS
    else if (key == 25604) flat1_pad<256, 4>(h, p, grid, out, pol, pad, stream);
    else if (key == 12808) flat1_pad<128, 8>(h, p, grid, out, pol, pad, stream);
    else flat1_pad<512, 2>(h, p, grid, out, pol, pad, stream);
    return true;
}

// GAE: PMENV_GAE = loop | scan | tile | tile8 | stream, PMENV_GAE_U (steps per lane and
// segment), PMENV_GAE_E (envs per lane of the pipelined tile), PMENV_GAE_P (days per block)
bool gae(const float* rewards, const float* values, const uint8_t* dones, float* adv, float* ret, int32_t T,
         int32_t B, float gamma, float lam, hipStream_t stream, int* rc) {
    const char* k = knob("PMENV_GAE");
    if (const char* sp = knob("PMENV_GAE_SP")) {   // the product's tile choice, stores with policy 2 (nt) / 16 (sc1)
        const int a = atoi(sp);
        const bool big = B >= 65536 && T >= 256;
        const unsigned g = (unsigned)((B + 63) / 64);
#define PMENV_GAESP(A_)                                                                                        \
    do {                                                                                                       \
        if (big) gae_tile_kernel<8, 8, 8, A_><<<g, 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam); \
        else if (B < 16384) gae_tile_kernel<8, 16, 1, A_><<<g, 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam); \
        else gae_tile_kernel<8, 8, 1, A_><<<g, 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam); \
    } while (0)
        if (a == 2) PMENV_GAESP(2);
        else PMENV_GAESP(16);
#undef PMENV_GAESP
        *rc = hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
        return true;
    }
    if (k && !strcmp(k, "lbfb")) {   // the product's look-back, its fallback taken on the first missing flag (SPIN = 0)
        const int seg = (int64_t)((T + 127) / 128) * ((B + 63) / 64) >= 128 ? 128 : 64;
        const int n = (T + seg - 1) / seg, neb = (B + 63) / 64;
        static double* ws = nullptr;
        static size_t ws_n = 0;
        const size_t need = (size_t)2 * n * B + (size_t)n * neb;
        if (need > ws_n) {
            if (ws) (void)hipFree(ws);
            if (hipMalloc(&ws, need * 8) != hipSuccess) { *rc = PMENV_ERR_HIP; return true; }
            ws_n = need;
        }
        static uint64_t epoch = 0x7a13ull << 48;
        ++epoch;
        uint64_t* flags = reinterpret_cast<uint64_t*>(ws + (size_t)2 * n * B);
        const unsigned g = (unsigned)(n * neb);
        if (seg == 128) gae_lookback_kernel<8, 16, 0><<<g, 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam, n, ws, flags, epoch);
        else gae_lookback_kernel<8, 8, 0><<<g, 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam, n, ws, flags, epoch);
        *rc = hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
        return true;
    }
    if (k && (!strcmp(k, "lb2") || !strcmp(k, "lb2x16"))) {   // two chunks per workgroup (64- / 128-day chunks)
        const int u = !strcmp(k, "lb2x16") ? 16 : 8;
        const int seg = 8 * u, n = (T + seg - 1) / seg, neb = (B + 63) / 64;
        static double* ws = nullptr;
        static size_t ws_n = 0;
        const size_t need = (size_t)2 * n * B + (size_t)n * neb;
        if (need > ws_n) {
            if (ws) (void)hipFree(ws);
            if (hipMalloc(&ws, need * 8) != hipSuccess) { *rc = PMENV_ERR_HIP; return true; }
            ws_n = need;
        }
        static uint64_t epoch = 0x7a12ull << 48;
        ++epoch;
        uint64_t* flags = reinterpret_cast<uint64_t*>(ws + (size_t)2 * n * B);
        const unsigned g = (unsigned)(((n + 1) / 2) * neb);
        if (u == 16) gae_lookback2_kernel<8, 16><<<g, 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam, n, ws, flags, epoch);
        else gae_lookback2_kernel<8, 8><<<g, 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam, n, ws, flags, epoch);
        *rc = hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
        return true;
    }
    if (k && (!strcmp(k, "lb16") || !strcmp(k, "lb4x16") || !strcmp(k, "lb16x4") || !strcmp(k, "lb8o1") ||
              !strcmp(k, "lb4o1") || !strcmp(k, "lb16o1") || !strcmp(k, "lb16x8"))) {   // look-back geometries; o1: one workgroup per CU
        const bool o1 = strstr(k, "o1") != nullptr;
        const int nw = !strcmp(k, "lb4x16") ? 4 : (!strcmp(k, "lb16x4") || !strcmp(k, "lb16x8")) ? 16 : 8;
        const int u = !strcmp(k, "lb16x4") || !strcmp(k, "lb4o1") ? 4 : (!strcmp(k, "lb8o1") || !strcmp(k, "lb16x8")) ? 8 : 16;
        const int seg = nw * u, n = (T + seg - 1) / seg, neb = (B + 63) / 64;
        static double* ws = nullptr;
        static size_t ws_n = 0;
        const size_t need = (size_t)2 * n * B + (size_t)n * neb;
        if (need > ws_n) {
            if (ws) (void)hipFree(ws);
            if (hipMalloc(&ws, need * 8) != hipSuccess) { *rc = PMENV_ERR_HIP; return true; }
            ws_n = need;
        }
        static uint64_t epoch = 0x7a11ull << 48;
        ++epoch;
        uint64_t* flags = reinterpret_cast<uint64_t*>(ws + (size_t)2 * n * B);
        const unsigned g = (unsigned)(n * neb);
        const size_t pad = 96 * 1024;         // LDS that holds a CU to one workgroup
        if (o1) {
            (void)hipFuncSetAttribute((const void*)gae_lookback_kernel<8, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pad);
            (void)hipFuncSetAttribute((const void*)gae_lookback_kernel<8, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pad);
            (void)hipFuncSetAttribute((const void*)gae_lookback_kernel<8, 16>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pad);
        }
        if (o1 && u == 4) gae_lookback_kernel<8, 4><<<g, 512, pad, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam, n, ws, flags, epoch);
        else if (o1 && u == 8) gae_lookback_kernel<8, 8><<<g, 512, pad, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam, n, ws, flags, epoch);
        else if (o1) gae_lookback_kernel<8, 16><<<g, 512, pad, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam, n, ws, flags, epoch);
        else if (nw == 4) gae_lookback_kernel<4, 16><<<g, 256, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam, n, ws, flags, epoch);
        else if (nw == 16 && u == 8) gae_lookback_kernel<16, 8><<<g, 1024, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam, n, ws, flags, epoch);
        else if (nw == 16) gae_lookback_kernel<16, 4><<<g, 1024, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam, n, ws, flags, epoch);
        else gae_lookback_kernel<8, 16><<<g, 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam, n, ws, flags, epoch);
        *rc = hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
        return true;
    }
    if (k && !strcmp(k, "split")) {               // the round-3 horizon split: maps pass + apply pass
        const int blocks = (B + 63) / 64;
        int want = (1024 + blocks - 1) / blocks, lc = (T + want - 1) / want;
        lc = (lc + 127) / 128 * 128;
        lc = lc < 256 ? 256 : lc;
        const int n = (T + lc - 1) / lc;
        static double* ws = nullptr;
        static size_t ws_n = 0;
        const size_t need = (size_t)2 * n * B;
        if (need > ws_n) {
            if (ws) (void)hipFree(ws);
            if (hipMalloc(&ws, need * 8) != hipSuccess) { *rc = PMENV_ERR_HIP; return true; }
            ws_n = need;
        }
        const dim3 grid((unsigned)blocks, (unsigned)n);
        gae_chunk_kernel<8, 16, true><<<grid, 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam, lc, ws);
        gae_chunk_kernel<8, 16, false, 2><<<grid, 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam, lc,
                                                                 ws);
        *rc = hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
        return true;
    }
    if (!k && !knob("PMENV_GAE_U") && !knob("PMENV_GAE_E")) return false;
    const bool fits = (size_t)(T + 1) * (size_t)B * 4u < (1ull << 31);
    const bool scan = k ? !strcmp(k, "scan") : (B < 64 && T >= 256);
    const bool tile = fits && (k ? (!strcmp(k, "tile") || !strcmp(k, "tile8") || !strcmp(k, "stream")) : !scan);
    const int U = knob_int("PMENV_GAE_U", B >= 16384 ? 8 : 16);
    int E = knob_int("PMENV_GAE_E", 0);
    if (E != 1 && E != 2 && E != 4) E = 0;
    if (E && B % E) E = 0;
    if (k && !strcmp(k, "tile8") && fits) {
        gae_tile_kernel<8, 8, 8><<<(B + 63) / 64, 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam);
    } else if (k && !strcmp(k, "stream") && fits) {
        const unsigned g = (unsigned)((B + 63) / 64);
        const int P = knob_int("PMENV_GAE_P", 16);
        if (P == 32) gae_stream_kernel<32><<<g, 64, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam);
        else if (P == 8) gae_stream_kernel<8><<<g, 64, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam);
        else gae_stream_kernel<16><<<g, 64, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam);
    } else if (tile && E) {
        const unsigned g = (unsigned)((B + 64 * E - 1) / (64 * E));
#define PMENV_GAEV(U_, E_) \
    gae_tile_vec_kernel<8, U_, E_><<<g, 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam)
        if (E == 1 && U == 16) PMENV_GAEV(16, 1);
        else if (E == 1) PMENV_GAEV(8, 1);
        else if (E == 2 && U == 4) PMENV_GAEV(4, 2);
        else if (E == 2) PMENV_GAEV(8, 2);
        else PMENV_GAEV(4, 4);                    // E = 4 at U = 8 spills
#undef PMENV_GAEV
    } else if (tile && U == 8 && B >= 65536 && T >= 256 && !k) {
        gae_tile_kernel<8, 8, 8><<<(B + 63) / 64, 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam);
    } else if (tile && U == 16) {
        gae_tile_kernel<8, 16><<<(B + 63) / 64, 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam);
    } else if (tile) {
        gae_tile_kernel<8, 8><<<(B + 63) / 64, 512, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam);
    } else if (scan) {
        gae_scan_kernel<<<(B + 3) / 4, 256, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam);
    } else {
        gae_kernel<<<(B + 255) / 256, 256, 0, stream>>>(rewards, values, dones, adv, ret, T, B, gamma, lam);
    }
    *rc = hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
    return true;
}

// replay gather: PMENV_REPLAY_LDS (the per-element staging kernel), PMENV_REPLAY_NT=0
// (default-policy stores), PMENV_REPLAY_PERSIST=0 (one workgroup per sample),
// PMENV_REPLAY_TPB=512, PMENV_REPLAY_GRID=G
bool replay_gather(const float* series, int32_t T, int32_t N, int32_t F, int32_t W, const int32_t* days,
                   const float* actions, const float* rewards, int32_t H, int32_t B, const int32_t* h0,
                   const int32_t* env, int32_t S, float* s, float* s_next, float* a_out, float* r_out,
                   hipStream_t stream, int* rc) {
    if (!knob("PMENV_REPLAY_LDS") && !knob("PMENV_REPLAY_NT") && !knob("PMENV_REPLAY_PERSIST") &&
        !knob("PMENV_REPLAY_TPB") && !knob("PMENV_REPLAY_GRID"))
        return false;
    const size_t lds = (size_t)N * (W + 1) * F * sizeof(float);
    const bool al16 = ((uintptr_t)s & 15u) == 0 && ((uintptr_t)s_next & 15u) == 0 && ((uintptr_t)series & 15u) == 0;
    int R = 0;
    if (F == 5 && al16 && !knob("PMENV_REPLAY_LDS")) {
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
        const bool nt = knob_int("PMENV_REPLAY_NT", 1) != 0;
        const bool t512 = knob_int("PMENV_REPLAY_TPB", 256) == 512;
        const bool persist = !t512 && knob_int("PMENV_REPLAY_PERSIST", 1) != 0;
        if (persist) {
            int cus = 0, dev = 0;
            if (hipGetDevice(&dev) != hipSuccess ||
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
                cus = 256;
            const int gy = N / R;
            int G = cus / gy > 0 ? cus / gy : 1;
            G = knob_int("PMENV_REPLAY_GRID", G) > 0 ? knob_int("PMENV_REPLAY_GRID", G) : G;
            const dim3 pgrid((unsigned)(S < G ? S : G), (unsigned)(N / R));
            const int ppt = pairs <= 2 * 256 ? 2 : pairs <= 4 * 256 ? 4 : 8;
#define PMENV_RGP(PPT, NTV)                                                                                   \
    replay_gather_f5p_kernel<PPT, NTV><<<pgrid, 256, glds, stream>>>(series, T, N, W, days, actions, rewards, H, B, \
                                                                     h0, env, S, s, s_next, a_out, r_out, R, dr, dwf)
            if (nt) { if (ppt == 2) PMENV_RGP(2, 2); else if (ppt == 4) PMENV_RGP(4, 2); else PMENV_RGP(8, 2); }
            else { if (ppt == 2) PMENV_RGP(2, 0); else if (ppt == 4) PMENV_RGP(4, 0); else PMENV_RGP(8, 0); }
#undef PMENV_RGP
        } else {
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
        }
    } else if (lds <= 64 * 1024 && N <= 256 && ((uintptr_t)s & 15u) == 0 && ((uintptr_t)s_next & 15u) == 0) {
        replay_gather_lds_kernel<<<(unsigned)S, 256, lds, stream>>>(series, T, N, F, W, days, actions, rewards, H, B,
                                                                   h0, env, s, s_next, a_out, r_out);
    } else {
        const int64_t threads = (int64_t)S * N * W * F;
        replay_gather_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, stream>>>(
            series, T, N, F, W, days, actions, rewards, H, B, h0, env, S, s, s_next, a_out, r_out);
    }
    *rc = hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
    return true;
}

// rollout gather: PMENV_RGATHER_ELEM (one thread per output float), PMENV_RGATHER_ROWS (the
// wave-per-row form), PMENV_RGATHER_NT=2|16|18 (the product's tile, window stores with those
// cache-policy bits)
bool rollout_gather(const float* series, int32_t T, int32_t N, int32_t F, int32_t W, const int32_t* start,
                    const float* weights, int32_t T_rec, int32_t B, int32_t ring_mode, const int32_t* t_idx,
                    const int32_t* env, int32_t S, float* s, hipStream_t stream, int* rc) {
    if (knob("PMENV_RGATHER_ELEM")) {
        const int64_t threads = (int64_t)S * N * W * F;
        rollout_gather_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, stream>>>(
            series, T, N, F, W, start, weights, T_rec, B, ring_mode, t_idx, env, S, s);
    } else if (const char* nt = knob("PMENV_RGATHER_NT")) {      // the tile with nt (2) / sc1 (16) stores
        const size_t lds = (size_t)W * N * F * sizeof(float);
        const int aux = atoi(nt);
        auto go = [&](auto kern) {
            kern<<<(unsigned)S, 256, lds, stream>>>(series, T, N, W, start, weights, B, ring_mode, t_idx, env, s,
                                                   make_fastdiv((uint32_t)N), make_fastdiv((uint32_t)(W * F)),
                                                   make_fastdiv((uint32_t)F));
        };
        if (aux == 2) go(rollout_gather_tile_kernel<2>);
        else if (aux == 16) go(rollout_gather_tile_kernel<16>);
        else go(rollout_gather_tile_kernel<18>);
    } else if (knob("PMENV_RGATHER_ROWS")) {
        const int64_t rows = (int64_t)S * N;
        rollout_gather_rows_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, stream>>>(
            series, T, N, F, W, start, weights, B, ring_mode, t_idx, env, S, s, make_fastdiv((uint32_t)F));
    } else {
        return false;
    }
    *rc = hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
    return true;
}

// metrics: PMENV_METRICS_WALK (the thread-per-env walk), PMENV_METRICS_FUSED=0 (two
// launches), PMENV_METRICS_SEG_FIRST=0 (turnover blocks dispatched first)
bool metrics(const double* returns, const double* values, const float* weights, int32_t T, int32_t B, int32_t N,
             double risk_free_rate, double periods, double* out, hipStream_t stream, int* rc) {
    const bool walk = knob("PMENV_METRICS_WALK") != nullptr;
    if (!walk && !knob("PMENV_METRICS_FUSED") && !knob("PMENV_METRICS_SEG_FIRST")) return false;
    const int tpe = N <= 256 ? N : 256, eb = 256 / tpe;
    const int nseg = (B + 63) / 64, nturn = (B + eb - 1) / eb;
    if (!walk && knob_int("PMENV_METRICS_FUSED", 1) != 0) {
        const int seg_first = knob_int("PMENV_METRICS_SEG_FIRST", 1) != 0;
        metrics_fused_kernel<<<(unsigned)(nseg + nturn), 256, 0, stream>>>(returns, values, weights, T, B, N,
                                                                           risk_free_rate, periods, tpe, eb, nseg,
                                                                           nturn, seg_first, out);
    } else {
        if (walk)
            metrics_kernel<<<(B + 255) / 256, 256, 0, stream>>>(returns, values, T, B, risk_free_rate, periods, out);
        else
            metrics_seg_kernel<<<(unsigned)nseg, 256, 0, stream>>>(returns, values, T, B, risk_free_rate, periods, out);
        metrics_turnover_kernel<<<(unsigned)nturn, 256, 0, stream>>>(weights, T, B, N, tpe, eb, out);
    }
    *rc = hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
    return true;
}

// the batched reward's forward in one launch (PMENV_BR_ONE; PMENV_BR_GRID, PMENV_BR_FENCE):
// the block that draws the last ticket folds the partials. Slower than the product's two
// launches at every shape.
bool batch_reward_forward(const float* a, const float* v_prev, const float* p, int32_t B, int32_t N,
                          int32_t reward_kind, int32_t norm, double scale, double* work, float* reward_out,
                          float* ret_out, hipStream_t stream, int* rc) {
    if (knob("PMENV_BR_TICKET") && N <= kQuadMaxN) {   // one launch, an epoch-tagged ticket, no fence
        static uint64_t* ticket = nullptr;
        static uint32_t epoch = 0x7e11u;
        if (!ticket) {                            // armed once as {first epoch, 0}; each call re-arms it
            if (hipMalloc(&ticket, 8) != hipSuccess) { *rc = PMENV_ERR_HIP; return true; }
            const uint64_t armed = (uint64_t)(epoch + 1u) << 32;
            (void)hipMemcpy(ticket, &armed, 8, hipMemcpyHostToDevice);
        }
        ++epoch;
        const int nblk = (B + kQuadRows - 1) / kQuadRows;
        if (N <= 32)
            batch_reward_fwd_ticket_kernel<8><<<(unsigned)nblk, kTrainBlock, 0, stream>>>(
                a, v_prev, p, B, N, reward_kind, norm, scale, work, reward_out, ticket, epoch);
        else
            batch_reward_fwd_ticket_kernel<16><<<(unsigned)nblk, kTrainBlock, 0, stream>>>(
                a, v_prev, p, B, N, reward_kind, norm, scale, work, reward_out, ticket, epoch);
        if (ret_out) batch_reward_select_kernel<<<(B + 255) / 256, 256, 0, stream>>>(B, norm, work, ret_out);
        *rc = hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
        return true;
    }
    if (knob("PMENV_BR_RELAY") && N <= kQuadMaxN) {   // one launch, flags instead of a ticket
        static uint64_t* flags = nullptr;
        static size_t nflags = 0;
        static uint64_t epoch = 0x5eed000000000000ull ^ (uint64_t)(uintptr_t)&flags;
        const int nblk = (B + kQuadRows - 1) / kQuadRows;
        if ((size_t)nblk > nflags) {
            if (flags) (void)hipFree(flags);
            if (hipMalloc(&flags, (size_t)nblk * 8) != hipSuccess) { *rc = PMENV_ERR_HIP; return true; }
            (void)hipMemset(flags, 0, (size_t)nblk * 8);
            nflags = (size_t)nblk;
        }
        ++epoch;
        if (N <= 32)
            batch_reward_fwd_relay_kernel<8><<<(unsigned)nblk, kTrainBlock, 0, stream>>>(
                a, v_prev, p, B, N, reward_kind, norm, scale, work, reward_out, flags, epoch);
        else
            batch_reward_fwd_relay_kernel<16><<<(unsigned)nblk, kTrainBlock, 0, stream>>>(
                a, v_prev, p, B, N, reward_kind, norm, scale, work, reward_out, flags, epoch);
        if (ret_out) batch_reward_select_kernel<<<(B + 255) / 256, 256, 0, stream>>>(B, norm, work, ret_out);
        *rc = hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
        return true;
    }
    if (!knob("PMENV_BR_ONE")) return false;
    if (hipMemsetAsync(work + 6 * (size_t)B + 6, 0, sizeof(uint32_t), stream) != hipSuccess) {
        *rc = PMENV_ERR_HIP;
        return true;
    }
    const bool quad = N <= kQuadMaxN;
    const int nblk = quad ? (B + kQuadRows - 1) / kQuadRows : (int)batch_reward_blocks(B);
    int grid = nblk, fence = 1;
    if (const char* k = knob("PMENV_BR_GRID")) grid = std::max(1, std::min(nblk, atoi(k)));
    if (const char* k = knob("PMENV_BR_FENCE")) fence = atoi(k);
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
    *rc = hipGetLastError() == hipSuccess ? PMENV_OK : PMENV_ERR_HIP;
    return true;
}

}  // namespace pmenv_tools

// the relay step's stamps (PMENV_RELAY_STAMPS, step_relay.h relay_clock): `buf` (device, kStampSlots x
// kStampMaxWg x 8 u64, zeroed by the caller) receives them from the next launches on; null stops them
extern "C" int pmenv_tools_relay_stamps(uint64_t* buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(pmenv_dev::g_relay_stamps), &buf, sizeof(buf), 0, hipMemcpyHostToDevice) ==
                   hipSuccess ? 0 : 1;
}
extern "C" int pmenv_tools_relay_stamp_dims(uint32_t* slots, uint32_t* max_wg) {
    *slots = pmenv_dev::kStampSlots;
    *max_wg = pmenv_dev::kStampMaxWg;
    return 0;
}

// the stamps of small_stamp_kernel (PMENV_SMALL_ABL), 1024 launches x 8 u64 (100 MHz ticks)
extern "C" int pmenv_tools_small_stamps(uint64_t* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(pmenv_dev::g_small_stamps), sizeof(uint64_t) * 1024 * 8, 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
