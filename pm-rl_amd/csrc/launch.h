// launch.h — the product's kernel launchers for the env step (host side), shared by the
// product library (pmenv.hip) and the tools build. Kernel choice is a function of the
// shape planned at create (pmenv_create_in) and of pmenv_set_step_path. Each step-phase
// launcher first offers the launch to the tools hook (a no-op in the product library).
#pragma once
#include "env_step.h"
#include "handle.h"
#include "scalar_vec.h"
#include "step_env.h"
#include "step_flat.h"
#include "step_relay.h"

namespace pmenv_host {

using namespace pmenv_dev;

// ---------------------------------------------------------------- the two-launch step
// the row-kernel stream (fallback of the flat stream: W = 1, or windows past 2^31 chunks)
template <int V>
inline void launch_advance_rows_v(const StepParams& p, unsigned grid, hipStream_t stream) {
    if (p.obs_out == p.obs)
        advance_rows_kernel<kStreamBlock, V, true><<<grid, kStreamBlock, 0, stream>>>(p);
    else
        advance_rows_kernel<kStreamBlock, V, false><<<grid, kStreamBlock, 0, stream>>>(p);
}

inline void launch_advance_rows(const pmenv* h, StepParams p, hipStream_t stream) {
    const bool db = p.obs_out != p.obs;
    p.unit_rows = db ? h->unit_rows_db : h->unit_rows;
    p.units_per_env = db ? h->units_per_env_db : h->units_per_env;
    p.div_units = make_fastdiv((uint32_t)p.units_per_env);
    const int vec = db ? h->stream_vec_db : h->stream_vec;
    const unsigned grid = (unsigned)(h->cfg.num_envs * p.units_per_env);
    if (vec == 1) launch_advance_rows_v<1>(p, grid, stream);
    else if (vec == 2) launch_advance_rows_v<2>(p, grid, stream);
    else launch_advance_rows_v<4>(p, grid, stream);
}

// the double-buffered flat stream: the workgroup (LDS) form, 512 threads x 2 chunks
inline void launch_flat_db(const pmenv* h, StepParams p, hipStream_t stream) {
    const pmenv_cfg& c = h->cfg;
    const uint32_t per4 = (uint32_t)((int64_t)c.num_assets * c.window * c.features / 4);
    const uint32_t qtot = (uint32_t)((int64_t)c.num_envs * per4);
    p.div_units = make_fastdiv(per4);
    const unsigned g = (unsigned)((qtot + 1023) / 1024);
    if (h->flat_pol == 0) advance_flat_wg_kernel<512, 2, 0><<<g, 512, 0, stream>>>(p, qtot);
    else advance_flat_wg_kernel<512, 2, 1><<<g, 512, 0, stream>>>(p, qtot);
}

// the in-place flat stream, the halo copied by the scalar step: 512 threads x 2 chunks,
// 256 x 2 for cache-resident windows
inline void launch_flat_inplace(const pmenv* h, StepParams p, hipStream_t stream) {
    const pmenv_cfg& c = h->cfg;
    const uint32_t per4 = (uint32_t)((int64_t)c.num_assets * c.window * c.features / 4);
    p.div_units = make_fastdiv(per4);
    p.halo = h->halo;
    const int cpw = h->flat_ip_block * h->flat_ip_vec;
    const unsigned grid = (unsigned)((h->flat_qtot + cpw - 1) / cpw);
    if (h->flat_ip_block == 256) advance_flat_inplace_kernel<256, 2, 0><<<grid, 256, 0, stream>>>(p, h->flat_qtot);
    else if (h->flat_ip_pol == 1) advance_flat_inplace_kernel<512, 2, 1><<<grid, 512, 0, stream>>>(p, h->flat_qtot);
    else advance_flat_inplace_kernel<512, 2, 0><<<grid, 512, 0, stream>>>(p, h->flat_qtot);
}

// the second launch of the two-launch step
inline void launch_advance(const pmenv* h, const StepParams& p, hipStream_t stream) {
    if (pmenv_tools::launch_advance(h, p, stream)) return;
    const bool db = p.obs_out != p.obs;
    if (db && h->flat) launch_flat_db(h, p, stream);
    else if (!db && h->flat_inplace) launch_flat_inplace(h, p, stream);
    else launch_advance_rows(h, p, stream);
}

// the first launch: the packed one-asset-per-lane form (N <= 16, L = 8 / 16 lanes per env),
// the register form (16 < N <= 64, L = 32 / 64), the packed strided form (64 < N <= 512),
// the LDS form (N > 512)
template <int L, int A>
inline void launch_scalar_vec_la(const StepParams& p, hipStream_t stream) {
    const unsigned waves = (unsigned)((p.B + 64 / L - 1) / (64 / L));
    scalar_step_vec_kernel<L, A, true><<<(waves + 3) / 4, 256, 0, stream>>>(p);
}

inline void launch_scalar_kernels(const pmenv* h, const StepParams& p, hipStream_t stream) {
    const int N = h->cfg.num_assets;
    if (h->k1_vec == kK1Str + 801) launch_scalar_vec_la<8, 1>(p, stream);
    else if (h->k1_vec == kK1Str + 1601) launch_scalar_vec_la<16, 1>(p, stream);
    else if (h->k1_vec == kK1Str + 6402) launch_scalar_vec_la<64, 2>(p, stream);
    else if (h->k1_vec == kK1Str + 6404) launch_scalar_vec_la<64, 4>(p, stream);
    else if (h->k1_vec == kK1Str + 6408) launch_scalar_vec_la<64, 8>(p, stream);
    else if (N <= 64) {
        const int per_wave = N <= 32 ? 2 : 1;
        const unsigned waves = (unsigned)((p.B + per_wave - 1) / per_wave);
        if (N <= 32) scalar_step_reg_kernel<32, 1><<<(waves + 3) / 4, 256, 0, stream>>>(p);
        else scalar_step_reg_kernel<64, 1><<<(waves + 3) / 4, 256, 0, stream>>>(p);
    } else {
        const int B = h->cfg.num_envs;
        scalar_step_kernel<<<(B + kScalarWaves - 1) / kScalarWaves, 64 * kScalarWaves, h->lds_scalar, stream>>>(
            p, h->scalar_scratch_floats);
    }
}

// the in-place flat stream reads its workgroups' halo, which this launch copies first
inline void launch_scalar(const pmenv* h, StepParams p, hipStream_t stream) {
    if (p.obs_out == p.obs && h->flat_inplace) {
        p.halo = h->halo;
        p.halo_wgs = h->halo_wgs;
        p.halo_block = (uint32_t)(h->flat_ip_block * h->flat_ip_vec);
        p.halo_qtot = h->flat_qtot;
    } else if (p.obs_out == p.obs && (h->gen & PMENV_FUSE_INPLACE)) {   // the generic stream's halo
        p.halo = h->halo;
        p.halo_hs = h->cfg.features > 8 ? 1u : 0u;   // four chunks per workgroup past F = 8
        p.halo_wgs = h->halo_wgs << p.halo_hs;
        p.halo_block = (uint32_t)(h->gen_block * h->gen_v);
        p.halo_qtot = h->gen_qtot;
    }
    if (pmenv_tools::launch_scalar(h, p, stream)) return;
    launch_scalar_kernels(h, p, stream);
}

// ---------------------------------------------------------------- the surface stream
inline void launch_surface_stream(const pmenv* h, StepParams p, hipStream_t stream) {
    const pmenv_cfg& c = h->cfg;
    const uint32_t per4 = (uint32_t)((int64_t)c.num_assets * c.window * c.features / 4);
    const uint32_t qtot = (uint32_t)((int64_t)c.num_envs * per4);
    p.div_units = make_fastdiv(per4);
    const unsigned grid = (qtot + 1023u) / 1024u;
    surface_stream_kernel<256, 4, 1><<<grid, 256, h->surf_lds, stream>>>(p, qtot);
}

// ---------------------------------------------------------------- the generic stream (F != 5)
// rows of the [B N, W F] window a workgroup of cpw chunks can touch (the plan keeps it <= BLOCK)
inline uint32_t gen_rows(const pmenv* h, int cpw) {
    return (uint32_t)(4 * (int64_t)cpw / ((int64_t)h->cfg.window * h->cfg.features) + 2);
}
template <int BLOCK, int V, int SHV, int FMAX>
inline void launch_gen_s(const pmenv* h, const StepParams& p, hipStream_t stream) {
    const unsigned grid = (unsigned)((h->gen_qtot + BLOCK * V - 1) / (BLOCK * V));
    const uint32_t rows = gen_rows(h, BLOCK * V);
    const size_t lds = (size_t)rows * (2 + (FMAX - 1)) * 4;
    // nt past the Infinity Cache: the F = 5 streams' rule (flat_ip_pol / flat_pol, pmenv.hip)
    if (p.obs_out == p.obs) {
        if (h->flat_ip_pol)
            advance_gen_kernel<BLOCK, V, false, SHV, true, 1, 0, FMAX><<<grid, BLOCK, lds, stream>>>(p, h->gen_qtot, rows);
        else
            advance_gen_kernel<BLOCK, V, false, SHV, true, 0, 0, FMAX><<<grid, BLOCK, lds, stream>>>(p, h->gen_qtot, rows);
    } else {
        if (h->flat_pol)
            advance_gen_kernel<BLOCK, V, true, SHV, true, 1, 0, FMAX><<<grid, BLOCK, lds, stream>>>(p, h->gen_qtot, rows);
        else
            advance_gen_kernel<BLOCK, V, true, SHV, true, 0, 0, FMAX><<<grid, BLOCK, lds, stream>>>(p, h->gen_qtot, rows);
    }
}
template <int BLOCK, int V, int FMAX>
inline void launch_gen_f(const pmenv* h, const StepParams& p, hipStream_t stream) {
    const int fm4 = h->cfg.features % 4;   // the shifted source's LDS reads: 16 B (F % 4 = 0), 8 B (F % 4 = 2), dwords
    if (fm4 == 0) launch_gen_s<BLOCK, V, 4, FMAX>(h, p, stream);
    else if (fm4 == 2) launch_gen_s<BLOCK, V, 2, FMAX>(h, p, stream);
    else launch_gen_s<BLOCK, V, 1, FMAX>(h, p, stream);
}
template <int BLOCK, int V>
inline void launch_gen_g(const pmenv* h, const StepParams& p, hipStream_t stream) {
    if (h->cfg.features > 8) launch_gen_f<BLOCK, V, 16>(h, p, stream);
    else launch_gen_f<BLOCK, V, 8>(h, p, stream);
}
inline void launch_gen(const pmenv* h, StepParams p, hipStream_t stream) {
    p.div_units = make_fastdiv(h->per4);
    p.halo = h->halo;                      // in place: the chunks past each workgroup (the scalar step's copy)
    if (pmenv_tools::launch_gen(h, p, stream)) return;
    switch (h->gen_block * 10 + h->gen_v) {
    case 2562: launch_gen_g<256, 2>(h, p, stream); break;
    case 5122: launch_gen_g<512, 2>(h, p, stream); break;
    default: launch_gen_g<256, 4>(h, p, stream); break;
    }
}

// ---------------------------------------------------------------- the register step (any F)
template <bool REG>
inline void launch_small_r(const pmenv* h, const StepParams& p, hipStream_t stream) {
    const unsigned grid = (unsigned)h->cfg.num_envs;
    const size_t lds = REG ? 0 : h->lds_surface;
    switch (h->small_block * 100 + h->small_e) {
    case 6432: step_small_kernel<64, 32, REG><<<grid, 64, lds, stream>>>(p); break;
    case 25608: step_small_kernel<256, 8, REG><<<grid, 256, lds, stream>>>(p); break;
    case 25616: step_small_kernel<256, 16, REG><<<grid, 256, lds, stream>>>(p); break;
    case 51216: step_small_kernel<512, 16, REG><<<grid, 512, lds, stream>>>(p); break;
    default: step_small_kernel<1024, 16, REG><<<grid, 1024, lds, stream>>>(p); break;
    }
}
inline void launch_small(const pmenv* h, const StepParams& p, hipStream_t stream) {
    if (pmenv_tools::launch_small(h, p, stream)) return;
    if (h->tiny) {
        const pmenv_cfg& c = h->cfg;
        const size_t lds = ((size_t)c.num_assets * c.window * c.features + 8 + (size_t)c.num_assets * (c.features - 1)) * 4;
        step_tiny_kernel<256, 8><<<(unsigned)c.num_envs, 256, lds, stream>>>(p);
        return;
    }
    if (h->cfg.num_assets <= 64) launch_small_r<true>(h, p, stream);
    else launch_small_r<false>(h, p, stream);
}

// ---------------------------------------------------------------- one launch, one workgroup per env
inline void launch_one(const pmenv* h, const StepParams& p, hipStream_t stream) {
    if (pmenv_tools::launch_one(h, p, stream)) return;
    const bool out = p.obs_out != p.obs;
    const int pol = out ? h->flat_pol : h->flat_ip_pol;
    const unsigned threads = 64u * (unsigned)h->one_waves;
    const size_t lds = ((size_t)threads * kOneV + 2) * 16;
    const unsigned grid = (unsigned)h->cfg.num_envs;
    if (out) {
        if (pol == 1) step_env_kernel<kOneV, true, 1><<<grid, threads, lds, stream>>>(p, h->per4);
        else step_env_kernel<kOneV, true, 0><<<grid, threads, lds, stream>>>(p, h->per4);
    } else {
        if (pol == 1) step_env_kernel<kOneV, false, 1><<<grid, threads, lds, stream>>>(p, h->per4);
        else step_env_kernel<kOneV, false, 0><<<grid, threads, lds, stream>>>(p, h->per4);
    }
}

// ---------------------------------------------------------------- one launch over the flat stream
template <int BK, int VV>
inline void launch_flat1_g(const StepParams& p, uint32_t qtot, unsigned grid, bool out, int pol,
                           hipStream_t stream) {
    if (out) {
        if (pol == 1) step_flat_kernel<BK, VV, 1, true><<<grid, BK, 0, stream>>>(p, qtot);
        else step_flat_kernel<BK, VV, 0, true><<<grid, BK, 0, stream>>>(p, qtot);
    } else {
        if (pol == 1) step_flat_kernel<BK, VV, 1, false><<<grid, BK, 0, stream>>>(p, qtot);
        else step_flat_kernel<BK, VV, 0, false><<<grid, BK, 0, stream>>>(p, qtot);
    }
}

// step_flat_vec_kernel (64 < N <= 512): A strided assets per lane, as the packed
// two-launch scalar step, so the two paths give the same bits
template <int A>
inline void launch_flat1_vec_a(const StepParams& p, uint32_t qtot, unsigned grid, bool out, int pol,
                               hipStream_t stream) {
    if (out) {
        if (pol == 1) step_flat_vec_kernel<A, 256, 4, 1, true><<<grid, 256, 0, stream>>>(p, qtot);
        else step_flat_vec_kernel<A, 256, 4, 0, true><<<grid, 256, 0, stream>>>(p, qtot);
    } else {
        if (pol == 1) step_flat_vec_kernel<A, 256, 4, 1, false><<<grid, 256, 0, stream>>>(p, qtot);
        else step_flat_vec_kernel<A, 256, 4, 0, false><<<grid, 256, 0, stream>>>(p, qtot);
    }
}

inline void launch_flat1_kernels(const pmenv* h, const StepParams& p, unsigned grid, bool out, int pol,
                                 hipStream_t stream) {
    const int N = h->cfg.num_assets;
    if (N > 64) {                                 // wide envs: the packed scalar step per tile
        if (N <= 128) launch_flat1_vec_a<2>(p, h->flat_qtot, grid, out, pol, stream);
        else if (N <= 256) launch_flat1_vec_a<4>(p, h->flat_qtot, grid, out, pol, stream);
        else launch_flat1_vec_a<8>(p, h->flat_qtot, grid, out, pol, stream);
    } else if (h->flat1_block == 256) {
        launch_flat1_g<256, 4>(p, h->flat_qtot, grid, out, pol, stream);
    } else if (h->flat1_block == 128) {
        launch_flat1_g<128, 8>(p, h->flat_qtot, grid, out, pol, stream);
    } else {
        launch_flat1_g<512, 2>(p, h->flat_qtot, grid, out, pol, stream);
    }
}

// the whole step in one launch over the flat stream (step_flat.h): prime the snapshot and
// the halo when something other than this kernel touched them, then one launch
inline void launch_flat1(pmenv* h, StepParams p, hipStream_t stream) {
    const bool out = p.obs_out != p.obs;
    const int q = h->par;
    p.per4 = h->per4;
    p.div_units = make_fastdiv(h->per4);
    const bool need_halo = !out && h->halo1_obs != p.obs;
    const int64_t work = (int64_t)h->cfg.num_envs * h->cfg.num_assets;
    const unsigned prime_grid = (unsigned)(work / 256 + 1 < 2048 ? work / 256 + 1 : 2048);
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
        flat_seq_kernel<<<prime_grid, 256, 0, stream>>>(pp, out ? 1 : 0, h->snap_stride);
    } else if (!h->snap_ok || need_halo) {
        StepParams pp = p;
        pp.sv_out = h->sv[q]; pp.sk_out = h->sk[q]; pp.sw_out = h->sw[q]; pp.slc_out = h->slc[q];
        pp.halo = need_halo ? h->halo1[q] : nullptr;
        pp.halo_wgs = h->halo1_wgs;
        pp.halo_block = (uint32_t)(h->flat1_block * h->flat1_vec);
        pp.halo_qtot = h->flat_qtot;
        flat_prime_kernel<<<prime_grid, 256, 0, stream>>>(pp);
    }
    if (!h->device_seq) {
        p.sv_in = h->sv[q]; p.sk_in = h->sk[q]; p.sw_in = h->sw[q]; p.slc_in = h->slc[q];
        p.sv_out = h->sv[1 - q]; p.sk_out = h->sk[1 - q]; p.sw_out = h->sw[1 - q]; p.slc_out = h->slc[1 - q];
        p.halo_in = h->halo1[q];
        p.halo_out = h->halo1[1 - q];
    }
    const int pol = out ? h->flat_pol : h->flat_ip_pol;
    const uint32_t cpw = (uint32_t)(h->flat1_block * h->flat1_vec);
    const unsigned grid = (h->flat_qtot + cpw - 1) / cpw;
    if (!pmenv_tools::launch_flat1(h, p, grid, out, pol, stream)) launch_flat1_kernels(h, p, grid, out, pol, stream);
    h->par = 1 - q;
    h->snap_ok = true;
    h->halo1_obs = out ? nullptr : p.obs;
}

// ---------------------------------------------------------------- one launch, relayed (step_relay.h)
template <int BLOCK, int POL, bool OUT, bool SEQ, int ANY = 0>
inline void launch_relay_g(const pmenv* h, const StepParams& p, const RelayParams& r, unsigned grid,
                           hipStream_t stream) {
    const uint32_t q = h->flat_qtot;
    if constexpr (BLOCK == 256) {
        if (h->relay_v == 4) {                      // 16 KiB tiles: the register form of 17 <= N <= 32 only
            step_relay_kernel<256, 4, POL, OUT, 32, 0, 1, SEQ, ANY><<<grid, BLOCK, 0, stream>>>(p, r, q);
            return;
        }
    }
    switch (h->relay_kl * 100 + h->relay_ka) {
    case 801: step_relay_kernel<BLOCK, 2, POL, OUT, 8, 1, 1, SEQ, ANY><<<grid, BLOCK, 0, stream>>>(p, r, q); break;
    case 1601: step_relay_kernel<BLOCK, 2, POL, OUT, 16, 1, 1, SEQ, ANY><<<grid, BLOCK, 0, stream>>>(p, r, q); break;
    case 3200: step_relay_kernel<BLOCK, 2, POL, OUT, 32, 0, 1, SEQ, ANY><<<grid, BLOCK, 0, stream>>>(p, r, q); break;
    case 6400: step_relay_kernel<BLOCK, 2, POL, OUT, 64, 0, 1, SEQ, ANY><<<grid, BLOCK, 0, stream>>>(p, r, q); break;
    case 6402: step_relay_kernel<BLOCK, 2, POL, OUT, 64, 2, 1, SEQ, ANY><<<grid, BLOCK, 0, stream>>>(p, r, q); break;
    case 6404: step_relay_kernel<BLOCK, 2, POL, OUT, 64, 4, 1, SEQ, ANY><<<grid, BLOCK, 0, stream>>>(p, r, q); break;
    default: step_relay_kernel<BLOCK, 2, POL, OUT, 64, 8, 8, SEQ, ANY><<<grid, BLOCK, 0, stream>>>(p, r, q); break;
    }
}
template <int BLOCK, int POL, int ANY = 0>
inline void launch_relay_b(const pmenv* h, const StepParams& p, const RelayParams& r, unsigned grid, bool out,
                           bool seq, hipStream_t stream) {
    if (out) {
        if (seq) launch_relay_g<BLOCK, POL, true, true, ANY>(h, p, r, grid, stream);
        else launch_relay_g<BLOCK, POL, true, false, ANY>(h, p, r, grid, stream);
    } else {
        if (seq) launch_relay_g<BLOCK, POL, false, true, ANY>(h, p, r, grid, stream);
        else launch_relay_g<BLOCK, POL, false, false, ANY>(h, p, r, grid, stream);
    }
}

// prime the counter copy and the in-place halo when the previous relay step's do not hold (eager:
// the host's flags say so; device-sequenced: the prime kernel reads the validity words, so a
// replayed graph decides per replay), tag the step with the next epoch, then one launch
inline int launch_relay(pmenv* h, StepParams p, hipStream_t stream) {
    const bool out = p.obs_out != p.obs;
    const uint32_t cpw = (uint32_t)(h->relay_block * h->relay_v);
    const bool dseq = h->relay_dseq;
    p.per4 = h->per4;
    p.div_units = make_fastdiv(h->per4);
    if (!dseq && ++h->relay_epoch == 0) {           // the words, list and claims restart at 0 when the counter wraps
        const size_t words = (size_t)((char*)h->relay_list - (char*)h->relay_w) + relay_list_bytes(h);
        if (hipMemsetAsync(h->relay_w, 0, words, stream) != hipSuccess) return PMENV_ERR_HIP;
        h->relay_epoch = 1;
    }
    RelayParams r;
    const int q = h->relay_par;
    r.scal = h->relay_scal;
    r.epoch = h->relay_epoch;
    r.par = (uint32_t)q;
    r.kp_in = h->relay_kp + (size_t)q * h->cfg.num_envs;
    r.kp_out = h->relay_kp + (size_t)(1 - q) * h->cfg.num_envs;
    r.halo_in = h->relay_halo + (size_t)q * h->relay_halo_stride;
    r.halo_out = h->relay_halo + (size_t)(1 - q) * h->relay_halo_stride;
    r.seq = dseq ? h->relay_seq : nullptr;
    r.w = h->relay_w;
    r.list = h->relay_list;
    r.done = h->relay_done;
    r.spin = pmenv_dev::kRelaySpin;
    r.rot = 0;
    r.grid = h->relay_tiles + h->relay_scal;
    r.kp = h->relay_kp;
    r.halo = h->relay_halo;
    r.B = (uint32_t)h->cfg.num_envs;
    r.halo_stride = h->relay_halo_stride;
    r.obs = p.obs;
    const bool need_halo = !out && (dseq || h->relay_obs != p.obs);
    const bool need_kp = dseq || !h->relay_kp_ok;
    if (need_halo || need_kp) {
        StepParams pp = p;
        pp.halo = need_halo ? h->relay_halo : nullptr;
        pp.halo_wgs = h->relay_tiles > 0 ? h->relay_tiles - 1 : 0;
        pp.halo_block = cpw;
        pp.halo_qtot = h->flat_qtot;
        const uint32_t work = pp.halo_wgs > (uint32_t)h->cfg.num_envs ? pp.halo_wgs : (uint32_t)h->cfg.num_envs;
        const unsigned g = work / 256 + 1 < 2048 ? work / 256 + 1 : 2048;
        relay_prime_kernel<<<g, 256, 0, stream>>>(pp, r, need_kp ? 1 : 0, dseq ? 1 : 0);
    }
    const unsigned grid = h->relay_tiles + h->relay_scal;
    if (dseq || !pmenv_tools::launch_relay(h, p, r, grid, stream)) {
        if (h->relay_block == 256) launch_relay_b<256, 0>(h, p, r, grid, out, dseq, stream);
        else launch_relay_b<512, 1>(h, p, r, grid, out, dseq, stream);
    }
    // eager: every relay step flips the parity; the halo of the next parity belongs to this
    // window only when this step ran in place (and wrote it)
    h->relay_par = 1 - h->relay_par;
    h->relay_kp_ok = true;
    h->relay_obs = out ? nullptr : p.obs;
    return PMENV_OK;
}

}  // namespace pmenv_host
