// gae_vec.h — the tiled GAE scan with E envs per lane and a software-pipelined
// segment loop (included by pmenv.hip after rollout.h).
//
// E consecutive envs per lane in one dword{E} load (the workgroup owns 64*E envs, so
// a wave instruction moves a 64*E*4-byte row run, and the done flags of the lane's
// envs are one E-byte load), with the NEXT segment's loads issued right after the
// LDS exchange, before the current segment's store walk: a segment's stores and the
// following segment's loads overlap instead of alternating. The per-env arithmetic
// (segment cuts, compose order) is the same as gae_tile_kernel's (rollout.h), so at
// the same (NW, U) the results are bitwise identical. The host guarantees
// B % E == 0 (aligned dword{E} rows) and every array below 2 GiB.
#pragma once
#include "rollout.h"

namespace pmenv_dev {

typedef unsigned int u2v __attribute__((ext_vector_type(2)));

template <int E>
__device__ __forceinline__ void gae_ld(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff, float (&x)[E]) {
    if constexpr (E == 1) {
        x[0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, 0));
    } else if constexpr (E == 2) {
        const u2v q = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0);
        x[0] = __uint_as_float(q.x); x[1] = __uint_as_float(q.y);
    } else {
        const u4v q = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0);
        x[0] = __uint_as_float(q.x); x[1] = __uint_as_float(q.y);
        x[2] = __uint_as_float(q.z); x[3] = __uint_as_float(q.w);
    }
}

template <int E>
__device__ __forceinline__ void gae_st(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff, const float (&x)[E]) {
    if constexpr (E == 1) {
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x[0]), rs, voff, soff, 0);
    } else if constexpr (E == 2) {
        const u2v q = {__float_as_uint(x[0]), __float_as_uint(x[1])};
        __builtin_amdgcn_raw_buffer_store_b64(q, rs, voff, soff, 0);
    } else {
        const u4v q = {__float_as_uint(x[0]), __float_as_uint(x[1]), __float_as_uint(x[2]), __float_as_uint(x[3])};
        __builtin_amdgcn_raw_buffer_store_b128(q, rs, voff, soff, 0);
    }
}

template <int E>
__device__ __forceinline__ uint32_t gae_ld_done(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff) {
    if constexpr (E == 1) return __builtin_amdgcn_raw_buffer_load_b8(rs, voff, soff, 0);
    else if constexpr (E == 2) return __builtin_amdgcn_raw_buffer_load_b16(rs, voff, soff, 0);
    else return __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, 0);
}

template <int NW, int U, int E>
__global__ __launch_bounds__(64 * NW) void gae_tile_vec_kernel(const float* r, const float* v, const uint8_t* dones,
                                                              float* adv, float* ret, int T, int B, float gamma,
                                                              float lam) {
    __shared__ double shC[NW][E][64], shD[NW][E][64];
    constexpr int S = NW * U;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: rows go in SGPRs
    const int b0 = (blockIdx.x * 64 + lane) * E;
    const bool ok = b0 < B;
    const uint32_t voff = (uint32_t)(ok ? b0 : B - E) * 4u;
    const uint32_t row = (uint32_t)B * 4u;
    const auto rs_r = make_rsrc(r, (uint32_t)T * row);
    const auto rs_v = make_rsrc(v, (uint32_t)(T + 1) * row);
    const auto rs_d = make_rsrc(dones ? (const void*)dones : (const void*)r, dones ? (uint32_t)T * (uint32_t)B : 0u);
    const auto rs_adv = make_rsrc(adv, (uint32_t)T * row);
    const auto rs_ret = make_rsrc(ret, (uint32_t)T * row);
    const uint32_t voff_st = ok ? voff : 0x80000000u;
    const double g = (double)gamma, gl = (double)gamma * (double)lam;
    float vv[U + 1][E], rr[U][E];
    uint32_t dn[U];                               // the lane's E done bytes per step
    auto load_seg = [&](int seg_end) {
        const int t0 = max(seg_end - S, 0) + w * U;
#pragma unroll
        for (int u = 0; u <= U; ++u) gae_ld<E>(rs_v, voff, (uint32_t)min(t0 + u, seg_end) * row, vv[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t t = (uint32_t)min(t0 + u, seg_end - 1);
            gae_ld<E>(rs_r, voff, t * row, rr[u]);
            dn[u] = gae_ld_done<E>(rs_d, voff >> 2, t * (uint32_t)B);   // no dones: reads 0 (alive)
        }
    };
    double carry[E];                              // advantage just after the current segment
#pragma unroll
    for (int e = 0; e < E; ++e) carry[e] = 0.0;
    load_seg(T);
    for (int seg_end = T; seg_end > 0; seg_end -= S) {
        const int t0 = max(seg_end - S, 0) + w * U;
        double dl[U][E];                          // delta_t, then A_t
        float vc[U][E];                           // v_t, kept for ret = A_t + v_t
        uint32_t alive[E];                        // bit u: 1 - done_t
#pragma unroll
        for (int e = 0; e < E; ++e) {
            alive[e] = 0;
#pragma unroll
            for (int u = 0; u < U; ++u) alive[e] |= (((dn[u] >> (8 * e)) & 0xFFu) ? 0u : 1u) << u;
            double C = 1.0, D = 0.0;
#pragma unroll
            for (int u = U - 1; u >= 0; --u) {
                const double n = (alive[e] >> u) & 1u ? 1.0 : 0.0;
                dl[u][e] = (double)rr[u][e] + g * n * (double)vv[u + 1][e] - (double)vv[u][e];
                vc[u][e] = vv[u][e];
                if (t0 + u < seg_end) {
                    D = dl[u][e] + gl * n * D;
                    C = gl * n * C;
                }
            }
            shC[w][e][lane] = C;
            shD[w][e][lane] = D;
        }
        __syncthreads();
        if (seg_end - S > 0) load_seg(seg_end - S);   // the next segment's loads fly during the stores
#pragma unroll
        for (int e = 0; e < E; ++e) {
            double a = carry[e];
            for (int j = NW - 1; j > w; --j) a = shD[j][e][lane] + shC[j][e][lane] * a;
#pragma unroll
            for (int u = U - 1; u >= 0; --u) {
                if (t0 + u < seg_end) {
                    const double n = (alive[e] >> u) & 1u ? 1.0 : 0.0;
                    a = dl[u][e] + gl * n * a;
                    dl[u][e] = a;
                }
            }
        }
#pragma unroll
        for (int u = U - 1; u >= 0; --u) {
            const int t = t0 + u;
            if (t < seg_end) {
                float ao[E], ro[E];
#pragma unroll
                for (int e = 0; e < E; ++e) {
                    ao[e] = (float)dl[u][e];
                    ro[e] = (float)(dl[u][e] + (double)vc[u][e]);
                }
                // lanes past B: voff is out of range for the store descriptors -> dropped
                gae_st<E>(rs_adv, voff_st, (uint32_t)t * row, ao);
                gae_st<E>(rs_ret, voff_st, (uint32_t)t * row, ro);
            }
        }
#pragma unroll
        for (int e = 0; e < E; ++e)
            for (int j = NW - 1; j >= 0; --j) carry[e] = shD[j][e][lane] + shC[j][e][lane] * carry[e];
        __syncthreads();                          // the LDS maps are rewritten next segment
    }
}

}  // namespace pmenv_dev
