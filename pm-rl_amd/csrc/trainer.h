// trainer.h — the trainer-side twin of the env step: the differentiable batched
// portfolio reward of the PG / A2C agents (agent/pg/pg.py:40-82 `_reward`,
// agent/a2c.py/a2c.py:40-82 `_loss`), forward and backward, in f64.
//
//   a [B, N] raw policy scores, v_prev [B], p [B, N] price relatives
//   normalise: softmax over assets iff !isclose(sum(a), 1) OR min(a) < 0, where the
//              reference takes sum/min over the WHOLE batch (pg.py:52); per-row and
//              none are offered as well
//   ret_b  = sum_n(v_b * (w_bn * p_bn)) / v_b                         (pg.py:68-72)
//   R      = mean(ret * s) | mean(log(ret) * s) | mean(ret) / std(ret) * s  (pg.py:75-80)
// The commission branch (pg.py:57-65) raises TypeError in the reference and is not
// part of this op.
#pragma once
#include "common.h"

namespace pmenv_dev {

// work layout (f64): [0,B) ret chosen and [5B,6B) row normalised flag (the select pass,
// run when the caller asks for the per-row returns), [B,2B) row sum, [2B,3B) row min,
// [3B,4B) ret raw, [4B,5B) ret softmax, [6B..6B+8) globals:
// +0 normalised (global), +1 mean, +2 std, +3 reward, +4 norm mode, +6 the tools build's
// one-launch forward's ticket (a u32, zeroed by the host before the launch); then the partial
// records of the row blocks (kRowsPerBlock or kQuadRows rows each), field-major:
// field i of block k at [6B+8 + i*nblocks + k].
constexpr int kTrainBlock = 256;
constexpr int kRowsPerBlock = 16;   // 4 waves x 4 rows
constexpr int kPartStride = 16;     // sum a, min a, nan, then 3 x {n, mean, M2, sum f}
constexpr int kCandRaw = 0, kCandSoftmax = 1, kCandRow = 2;

__host__ __device__ inline size_t batch_reward_blocks(int B) { return ((size_t)B + kRowsPerBlock - 1) / kRowsPerBlock; }
__host__ __device__ inline size_t batch_reward_work_doubles(int B) {
    return (size_t)6 * B + 8 + batch_reward_blocks(B) * kPartStride;
}

__device__ __forceinline__ bool row_normalises(double rsum, double rmin) {
    return !(fabs(rsum - 1.0) <= 1e-6 + 1e-5) || rmin < 0.0 || isnan(rmin);
}

// Chan et al. parallel merge of (n, mean, M2) — fixed operand order, deterministic
__device__ __forceinline__ void chan_merge(double& n, double& mean, double& m2, double n2, double mean2, double m22) {
    if (n2 == 0.0) return;
    if (n == 0.0) { n = n2; mean = mean2; m2 = m22; return; }
    const double nn = n + n2, d = mean2 - mean;
    mean += d * (n2 / nn);
    m2 += m22 + d * d * (n * n2 / nn);
    n = nn;
}

// The candidate return vectors the norm mode can choose — GLOBAL_OR: raw or softmax (the
// whole batch decides, in the final fold); ROW_OR: the per-row choice; NONE: raw — and the
// statistics the reward kind needs of them: Sharpe the count, mean and M2 (pg.py:80), the
// others the sum of f(ret) (pg.py:76, :78). The partial records carry only those (the other
// fields 0), and the folds skip the rest: no Chan merge (two f64 divisions per candidate and
// step) outside Sharpe.
__device__ __forceinline__ bool cand_used(int norm, int c) {
    return norm == PMENV_BNORM_GLOBAL_OR ? c != kCandRow : norm == PMENV_BNORM_ROW_OR ? c == kCandRow : c == kCandRaw;
}
__device__ __forceinline__ bool field_used(int kind, int norm, int i) {
    if (i < 3) return true;                                  // sum a, min a, nan
    if (i >= 15) return false;
    const int c = (i - 3) >> 2, f = (i - 3) & 3;
    if (!cand_used(norm, c)) return false;
    return kind == PMENV_REWARD_SHARPE ? f < 3 : f == 3;
}

// the candidate fields of one record (count, mean, M2 | sum f) over this wave's rows:
// `own` lanes hold a row's candidates x[c], cnt rows in all
__device__ __forceinline__ void cand_record(int kind, int norm, bool own, double cnt, const double (&x)[3],
                                            double (&rec)[kPartStride]) {
    const bool sharpe = kind == PMENV_REWARD_SHARPE;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        rec[3 + 4 * c + 0] = 0.0;
        rec[3 + 4 * c + 1] = 0.0;
        rec[3 + 4 * c + 2] = 0.0;
        rec[3 + 4 * c + 3] = 0.0;
        if (!cand_used(norm, c)) continue;                   // uniform
        if (sharpe) {
            const double mean = cnt > 0.0 ? wave_sum(own ? x[c] : 0.0) / cnt : 0.0;
            const double d = own ? x[c] - mean : 0.0;
            rec[3 + 4 * c + 0] = cnt;
            rec[3 + 4 * c + 1] = mean;
            rec[3 + 4 * c + 2] = wave_sum(d * d);
        } else {
            rec[3 + 4 * c + 3] = wave_sum(own ? (kind == PMENV_REWARD_LOG_RETURN ? log(x[c]) : x[c]) : 0.0);
        }
    }
    rec[15] = 0.0;
}

// fold record q into acc (fields the kind / norm mode use only)
__device__ __forceinline__ void fold_record(int kind, int norm, double (&acc)[kPartStride], const double* q) {
    acc[0] += q[0];
    acc[1] = fmin(acc[1], q[1]);
    acc[2] += q[2];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        if (!cand_used(norm, c)) continue;
        if (kind == PMENV_REWARD_SHARPE)
            chan_merge(acc[3 + 4 * c], acc[4 + 4 * c], acc[5 + 4 * c], q[3 + 4 * c], q[4 + 4 * c], q[5 + 4 * c]);
        else
            acc[6 + 4 * c] += q[6 + 4 * c];
    }
}

// one wave per row (4 rows per wave, 16 per block). EPL > 0 (N <= 64*EPL): the wave
// loads all four rows' elements into registers up front (lane l holds elements
// l + 64k: coalesced 256-B rows, every load in flight before the first reduction) and
// reads memory once; EPL = 0: any N, looping over the row in passes. Wave 0 then
// folds the block's rows into one partial record: sums / min for the normalisation
// decision and, for each candidate return vector (raw, softmax, per-row choice),
// count, mean, M2 (two-pass inside the block) and the sum of f(ret) (log for the
// log-return reward).
template <int EPL>
__device__ __forceinline__ void rows_wave_partial(const float* a, const float* v_prev, const float* p, int B, int N,
                                                  int kind, int norm, double* work, double (*sh)[kRowsPerBlock],
                                                  int blk, int nblk) {
    constexpr int RPW = kRowsPerBlock / 4;        // rows per wave
    constexpr int E = EPL > 0 ? EPL : 1;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float ra[RPW][E], rp[RPW][E];
    if (EPL > 0) {
        const uint32_t bytes = (uint32_t)B * (uint32_t)N * 4u;
        const auto rsa = make_rsrc(a, bytes), rsp = make_rsrc(p, bytes);
#pragma unroll
        for (int j = 0; j < RPW; ++j) {
            const int b = blk * kRowsPerBlock + wave * RPW + j;
#pragma unroll
            for (int k = 0; k < E; ++k) {
                const int n = lane + 64 * k;
                // lanes past the row (or rows past B) read out of range: 0, no traffic
                const uint32_t off = (n < N && b < B) ? ((uint32_t)b * (uint32_t)N + (uint32_t)n) * 4u : 0xFFFFFFF0u;
                ra[j][k] = buf_load1(rsa, off);
                rp[j][k] = buf_load1(rsp, off);
            }
        }
    }
    for (int j = 0; j < RPW; ++j) {
        const int rl = wave * RPW + j;
        const int b = blk * kRowsPerBlock + rl;
        if (b >= B) break;
        const double v = (double)v_prev[b];
        double s = 0.0, mn = INFINITY, mx = -INFINITY, raw = 0.0;
        int nan_seen = 0;
        if (EPL > 0) {
#pragma unroll
            for (int k = 0; k < E; ++k) {
                if (lane + 64 * k < N) {
                    const double x = (double)ra[j][k];
                    s += x;
                    mn = fmin(mn, x);
                    mx = fmax(mx, x);
                    nan_seen |= isnan(x);
                    raw += v * (x * (double)rp[j][k]);
                }
            }
        } else {
            for (int n = lane; n < N; n += 64) {
                const double x = (double)a[(size_t)b * N + n];
                s += x;
                mn = fmin(mn, x);
                mx = fmax(mx, x);
                nan_seen |= isnan(x);
                raw += v * (x * (double)p[(size_t)b * N + n]);
            }
        }
        s = wave_sum(s);
        mn = wave_min(mn);
        mx = wave_max(mx);
        raw = wave_sum(raw);
        if (__any(nan_seen)) mn = NAN;
        double z = 0.0, sm = 0.0;
        if (EPL > 0) {
            double e[E];
#pragma unroll
            for (int k = 0; k < E; ++k) {
                e[k] = lane + 64 * k < N ? exp((double)ra[j][k] - mx) : 0.0;
                z += e[k];
            }
            z = wave_sum(z);
            const double rz = 1.0 / z;
#pragma unroll
            for (int k = 0; k < E; ++k) sm += v * ((e[k] * rz) * (double)rp[j][k]);   // torch.softmax(a, dim=1)
        } else {
            for (int n = lane; n < N; n += 64) z += exp((double)a[(size_t)b * N + n] - mx);
            z = wave_sum(z);
            for (int n = lane; n < N; n += 64) {
                const double w = exp((double)a[(size_t)b * N + n] - mx) / z;     // torch.softmax(a, dim=1)
                sm += v * (w * (double)p[(size_t)b * N + n]);
            }
        }
        sm = wave_sum(sm);
        if (lane == 0) {
            work[(size_t)B + b] = s;
            work[2 * (size_t)B + b] = mn;
            work[3 * (size_t)B + b] = raw / v;
            work[4 * (size_t)B + b] = sm / v;
            sh[0][rl] = s;
            sh[1][rl] = mn;
            sh[2][rl] = raw / v;
            sh[3][rl] = sm / v;
        }
    }
    __syncthreads();
    if (wave != 0) return;                                          // (no barrier follows in this function)
    const int b = blk * kRowsPerBlock + lane;
    const bool ok = lane < kRowsPerBlock && b < B;
    const double cnt = (double)min(kRowsPerBlock, B - blk * kRowsPerBlock);
    double* part = work + (size_t)6 * B + 8 + blk;
    const int li = ok ? lane : 0;
    const double rs = ok ? sh[0][li] : 0.0, rm = ok ? sh[1][li] : INFINITY;
    const double s_all = wave_sum(rs);
    const int has_nan = __any(ok && isnan(rm));
    const double mn_all = wave_min(ok && !isnan(rm) ? rm : INFINITY);
    double x[3];
    x[kCandRaw] = ok ? sh[2][li] : 0.0;
    x[kCandSoftmax] = ok ? sh[3][li] : 0.0;
    x[kCandRow] = row_normalises(rs, rm) ? x[kCandSoftmax] : x[kCandRaw];
    double rec[kPartStride];
    rec[0] = s_all;
    rec[1] = mn_all;
    rec[2] = has_nan ? 1.0 : 0.0;
    cand_record(kind, norm, ok, cnt, x, rec);
    if (lane < kPartStride) {
        double val = rec[0];
#pragma unroll
        for (int i = 1; i < kPartStride; ++i) val = lane == i ? rec[i] : val;
        part[(size_t)lane * nblk] = val;                      // field-major: coalesced final fold
    }
}

template <int EPL>
__global__ __launch_bounds__(kTrainBlock) void batch_reward_rows_kernel(const float* a, const float* v_prev,
                                                                        const float* p, int B, int N, int kind,
                                                                        int norm, double* work) {
    __shared__ double sh[4][kRowsPerBlock];       // row sum, row min, raw, softmax
    rows_wave_partial<EPL>(a, v_prev, p, B, N, kind, norm, work, sh, (int)blockIdx.x, (int)gridDim.x);
}

// ---------------------------------------------------------------- N <= 64: a quad per row
// Four lanes per row (64 rows per 256-thread workgroup, B/64 workgroups: four waves
// per SIMD at B = 65,536), lane g of a row holding elements [g*EPL, g*EPL + EPL) in
// registers from dword-aligned 16-B loads of the contiguous row (range-checked: the
// batch's last row never reads past the tensor). The row's sums, min, max and
// softmax go through DPP quad reductions; each wave then folds its 16 rows and
// thread 0 merges the four wave records in wave order (Chan): deterministic, one
// partial per 64 rows for the final fold.
constexpr int kQuadRows = 64;
constexpr int kQuadMaxN = 64;

template <int EPL>
struct RowQuad {
    float a[EPL], p[EPL];
};

template <int EPL>
__device__ __forceinline__ RowQuad<EPL> load_row_quad(const float* a, const float* p, int B, int N, int b, int g) {
    RowQuad<EPL> q;
    const uint32_t bytes = (uint32_t)B * (uint32_t)N * 4u;
    const auto ra = make_rsrc(a, bytes), rp = make_rsrc(p, bytes);
    const uint32_t base = ((uint32_t)b * (uint32_t)N + (uint32_t)(g * EPL)) * 4u;
#pragma unroll
    for (int c = 0; c < EPL / 4; ++c) {
        const f4 va = buf_load4(ra, base + 16u * c), vp = buf_load4(rp, base + 16u * c);
        q.a[4 * c] = va.x; q.a[4 * c + 1] = va.y; q.a[4 * c + 2] = va.z; q.a[4 * c + 3] = va.w;
        q.p[4 * c] = vp.x; q.p[4 * c + 1] = vp.y; q.p[4 * c + 2] = vp.z; q.p[4 * c + 3] = vp.w;
    }
    return q;
}

// COH (tools A/B: the one-launch forward): the partial record is written with agent-scope
// atomic stores, coherent across the XCDs' L2s for a fold in the same launch
template <int EPL, bool COH = false>
__device__ __forceinline__ void rows_quad_partial(const float* a, const float* v_prev, const float* p, int B, int N,
                                                  int kind, int norm, double* work, double (*rec_w)[kPartStride],
                                                  int blk, int nblk, double* rec_dst = nullptr) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = tid & 3;
    const int r0 = blk * kQuadRows;
    const int nrows = min(kQuadRows, B - r0);
    const bool ok = (tid >> 2) < nrows;
    const int b = r0 + (ok ? tid >> 2 : 0);
    const RowQuad<EPL> q = load_row_quad<EPL>(a, p, B, N, b, g);
    const double v = (double)v_prev[b];
    double s = 0.0, mn = INFINITY, mx = -INFINITY, raw = 0.0;
    bool nan_seen = false;
#pragma unroll
    for (int i = 0; i < EPL; ++i) {
        if (g * EPL + i < N) {
            const double x = (double)q.a[i];
            s += x;
            mn = fmin(mn, x);
            mx = fmax(mx, x);
            nan_seen |= isnan(x);
            raw += v * (x * (double)q.p[i]);
        }
    }
    s = quad_sum(s);
    mn = quad_min(mn);
    mx = quad_max(mx);
    raw = quad_sum(raw);
    if (quad_sum(nan_seen ? 1.0 : 0.0) > 0.0) mn = NAN;            // torch.min propagates NaN
    double e[EPL];
    double z = 0.0;
#pragma unroll
    for (int i = 0; i < EPL; ++i) {
        e[i] = g * EPL + i < N ? exp((double)q.a[i] - mx) : 0.0;
        z += e[i];
    }
    z = quad_sum(z);
    const double rz = 1.0 / z;
    double sm = 0.0;
#pragma unroll
    for (int i = 0; i < EPL; ++i)
        if (g * EPL + i < N) sm += v * ((e[i] * rz) * (double)q.p[i]);   // torch.softmax(a, dim=1)
    sm = quad_sum(sm);
    const double x_raw = raw / v, x_sm = sm / v;
    if (ok && g == 0) {
        work[(size_t)B + b] = s;
        work[2 * (size_t)B + b] = mn;
        work[3 * (size_t)B + b] = x_raw;
        work[4 * (size_t)B + b] = x_sm;
    }
    // this wave's record over its 16 rows (lane g == 0 of each quad contributes)
    const bool own = ok && g == 0;
    const double cnt = (double)max(0, min(16, nrows - 16 * wave));
    double x[3];
    x[kCandRaw] = own ? x_raw : 0.0;
    x[kCandSoftmax] = own ? x_sm : 0.0;
    x[kCandRow] = row_normalises(s, mn) ? x[kCandSoftmax] : x[kCandRaw];
    double rec[kPartStride];
    rec[0] = wave_sum(own ? s : 0.0);
    rec[1] = wave_min(own && !isnan(mn) ? mn : INFINITY);
    rec[2] = __any(own && isnan(mn)) ? 1.0 : 0.0;
    cand_record(kind, norm, own, cnt, x, rec);
    if (lane < kPartStride) {
        double val = rec[0];
#pragma unroll
        for (int i = 1; i < kPartStride; ++i) val = lane == i ? rec[i] : val;
        rec_w[wave][lane] = val;
    }
    __syncthreads();
    if (tid != 0) return;
    double acc[kPartStride];
    for (int i = 0; i < kPartStride; ++i) acc[i] = rec_w[0][i];
    for (int w = 1; w < 4; ++w) fold_record(kind, norm, acc, rec_w[w]);
    double* part = rec_dst ? rec_dst + blk : work + (size_t)6 * B + 8 + blk;   // field-major: coalesced final fold
    for (int i = 0; i < kPartStride; ++i) {
        if (COH) __hip_atomic_store(part + (size_t)i * nblk, acc[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else part[(size_t)i * nblk] = acc[i];
    }
}

template <int EPL>
__global__ __launch_bounds__(kTrainBlock) void batch_reward_rows_quad_kernel(const float* a, const float* v_prev,
                                                                             const float* p, int B, int N, int kind,
                                                                             int norm, double* work) {
    __shared__ double rec_w[4][kPartStride];
    rows_quad_partial<EPL>(a, v_prev, p, B, N, kind, norm, work, rec_w, (int)blockIdx.x, (int)gridDim.x);
}

// backward, N <= 64, a quad per row: dR/da through the (optional) softmax. The
// per-row choice (softmax or raw) is taken here from the forward's workspace (its
// norm mode at work[6B+4]), so the backward needs no select pass. Whole 16-B chunks
// of the row are stored as such, the row's tail element by element.
template <int EPL>
__global__ __launch_bounds__(kTrainBlock) void batch_reward_grad_quad_kernel(const float* a, const float* v_prev,
                                                                             const float* p, int B, int N, int kind,
                                                                             double scale, const double* work,
                                                                             const float* grad_out, float* grad_a) {
    const int tid = threadIdx.x, g = tid & 3;
    const int r0 = blockIdx.x * kQuadRows;
    const int nrows = min(kQuadRows, B - r0);
    const bool ok = (tid >> 2) < nrows;
    const int b = r0 + (ok ? tid >> 2 : 0);
    const RowQuad<EPL> q = load_row_quad<EPL>(a, p, B, N, b, g);
    const int norm = (int)work[6 * (size_t)B + 4];                // the forward's mode
    bool nb;
    if (norm == PMENV_BNORM_GLOBAL_OR) nb = work[6 * (size_t)B] != 0.0;
    else if (norm == PMENV_BNORM_ROW_OR) nb = row_normalises(work[(size_t)B + b], work[2 * (size_t)B + b]);
    else nb = false;
    const double r = nb ? work[4 * (size_t)B + b] : work[3 * (size_t)B + b];
    double dr;
    if (kind == PMENV_REWARD_LOG_RETURN) dr = scale / ((double)B * r);
    else if (kind == PMENV_REWARD_RETURN) dr = scale / (double)B;
    else {
        const double m = work[6 * (size_t)B + 1], sd = work[6 * (size_t)B + 2];
        dr = scale * (1.0 / ((double)B * sd) - m * (r - m) / ((double)(B - 1) * sd * sd * sd));
    }
    dr *= (double)*grad_out;
    const double v = (double)v_prev[b];
    float out[EPL];
    // nb is uniform per quad (a row's lanes agree), so the quad reductions below see
    // every lane of the quad on the same branch
    if (!nb) {
#pragma unroll
        for (int i = 0; i < EPL; ++i) out[i] = (float)(dr * (v * (double)q.p[i]) / v);
    } else {
        double mx = -INFINITY;
#pragma unroll
        for (int i = 0; i < EPL; ++i)
            if (g * EPL + i < N) mx = fmax(mx, (double)q.a[i]);
        mx = quad_max(mx);
        double e[EPL], z = 0.0;
#pragma unroll
        for (int i = 0; i < EPL; ++i) {
            e[i] = g * EPL + i < N ? exp((double)q.a[i] - mx) : 0.0;
            z += e[i];
        }
        z = quad_sum(z);
        const double rz = 1.0 / z;
        double wg = 0.0;                                          // sum_m w_m g_m
#pragma unroll
        for (int i = 0; i < EPL; ++i) wg += (e[i] * rz) * (dr * (v * (double)q.p[i]) / v);
        wg = quad_sum(wg);
#pragma unroll
        for (int i = 0; i < EPL; ++i) out[i] = (float)((e[i] * rz) * (dr * (v * (double)q.p[i]) / v - wg));
    }
    if (!ok) return;
    const auto rg = make_rsrc(grad_a, (uint32_t)B * (uint32_t)N * 4u);
    const int n0 = g * EPL;
    const uint32_t base = ((uint32_t)b * (uint32_t)N + (uint32_t)n0) * 4u;
#pragma unroll
    for (int c = 0; c < EPL / 4; ++c) {
        if (n0 + 4 * c + 4 <= N) {
            buf_store4(rg, base + 16u * c, f4{out[4 * c], out[4 * c + 1], out[4 * c + 2], out[4 * c + 3]});
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (n0 + 4 * c + k < N) grad_a[(size_t)b * N + n0 + 4 * c + k] = out[4 * c + k];
        }
    }
}

// single workgroup over the `nparts` block partials: the normalisation decision, the reward
// and the chosen candidate's mean / std. Thread t folds partials t, t + 256, ... in
// order, then a fixed-shape LDS tree folds the 256 threads: deterministic.
template <bool COH = false>
__device__ __forceinline__ void final_fold(int B, int kind, int norm, double scale, double* work, float* reward_out,
                                           int nparts, const double* parts_src = nullptr, int* glob_out = nullptr) {
    __shared__ double sh[4][kPartStride];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const size_t nblk = (size_t)nparts;
    const double* parts = parts_src ? parts_src : work + (size_t)6 * B + 8;
    double acc[kPartStride];
    acc[0] = 0.0; acc[1] = INFINITY; acc[2] = 0.0;
    for (int c = 0; c < 3; ++c) { acc[3 + 4 * c] = 0.0; acc[4 + 4 * c] = 0.0; acc[5 + 4 * c] = 0.0; acc[6 + 4 * c] = 0.0; }
    acc[15] = 0.0;
    auto fold = [&](const double* q) { fold_record(kind, norm, acc, q); };
    // thread t folds partials t, t + 256, ... in order; then a shift-down tree inside
    // each wave (lane i takes lane i + o) and the four wave records in wave order
    // partials are field-major (field i of block k at parts[i * nparts + k]): every
    // load below is a coalesced row, and a thread's four partials are all in flight
    // before the first fold
    for (size_t k0 = tid; k0 < nblk; k0 += 4 * kTrainBlock) {
        double q[4][kPartStride];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const size_t k = k0 + (size_t)j * kTrainBlock;
#pragma unroll
            for (int i = 0; i < kPartStride; ++i)
                q[j][i] = !(k < nblk && field_used(kind, norm, i)) ? 0.0
                          : COH ? __hip_atomic_load(const_cast<double*>(parts) + (size_t)i * nblk + k, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT)
                                : parts[(size_t)i * nblk + k];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (k0 + (size_t)j * kTrainBlock < nblk) fold(q[j]);
    }
    for (int o = 32; o > 0; o >>= 1) {
        double q[kPartStride];
#pragma unroll
        for (int i = 0; i < kPartStride; ++i)
            q[i] = field_used(kind, norm, i) ? __hiloint2double(__shfl_down(__double2hiint(acc[i]), o, 64),
                                                                __shfl_down(__double2loint(acc[i]), o, 64))
                                             : 0.0;
        if (lane < o) fold(q);
    }
    if (lane == 0)
        for (int i = 0; i < kPartStride; ++i) sh[wave][i] = acc[i];
    __syncthreads();
    if (tid != 0) return;
    for (int w = 1; w < 4; ++w) fold(sh[w]);
    // pg.py:52 sums / mins the WHOLE [B, N, 1] tensor; torch.min propagates NaN
    const double mn_all = acc[2] > 0.0 ? NAN : acc[1];
    const bool glob = !(fabs(acc[0] - 1.0) <= 1e-6 + 1e-5) || mn_all < 0.0;
    const int c = norm == PMENV_BNORM_GLOBAL_OR ? (glob ? kCandSoftmax : kCandRaw)
                : norm == PMENV_BNORM_ROW_OR ? kCandRow : kCandRaw;
    // constant indices only (a runtime index into acc would put it in scratch memory)
    const double mean = c == kCandRaw ? acc[4] : c == kCandSoftmax ? acc[8] : acc[12];
    const double m2 = c == kCandRaw ? acc[5] : c == kCandSoftmax ? acc[9] : acc[13];
    const double fsum = c == kCandRaw ? acc[6] : c == kCandSoftmax ? acc[10] : acc[14];
    const bool sharpe = kind == PMENV_REWARD_SHARPE;
    const double sd = B > 1 ? sqrt(m2 / (B - 1)) : NAN;                  // torch.std: unbiased
    double R;
    if (sharpe) R = mean / sd * scale;                                    // pg.py:80
    else R = fsum / B * scale;                                            // pg.py:76, :78
    work[6 * (size_t)B + 0] = glob ? 1.0 : 0.0;
    work[6 * (size_t)B + 1] = sharpe ? mean : 0.0;                        // only the Sharpe backward reads them
    work[6 * (size_t)B + 2] = sharpe ? sd : 0.0;
    work[6 * (size_t)B + 3] = R;
    work[6 * (size_t)B + 4] = (double)norm;
    *reward_out = (float)R;
    if (glob_out) *glob_out = glob ? 1 : 0;
}

// the second launch of the forward: one workgroup folds the row blocks' partials
static __global__ __launch_bounds__(kTrainBlock) void batch_reward_final_kernel(int B, int kind, int norm, double scale,
                                                                         double* work, float* reward_out,
                                                                         int nparts) {
    final_fold(B, kind, norm, scale, work, reward_out, nparts);
}


// The whole forward in ONE workgroup for a batch of at most 64 rows (N <= 64) — the PG / A2C
// agents' own BATCH_SIZE = 64 (config/pg.py:7), where the two-launch forward is two kernel
// latencies for a few KiB of work: the row block's partial record goes to LDS, the same
// final_fold reads it from there (one record: the same folds, the same bits), and with
// `ret_out` the rows' choice is made here too (no select launch).
template <int EPL>
__global__ __launch_bounds__(kTrainBlock) void batch_reward_small_kernel(const float* a, const float* v_prev,
                                                                         const float* p, int B, int N, int kind,
                                                                         int norm, double scale, double* work,
                                                                         float* reward_out, float* ret_out) {
    __shared__ double rec_w[4][kPartStride];
    __shared__ double rec[kPartStride];
    __shared__ int glob;
    rows_quad_partial<EPL>(a, v_prev, p, B, N, kind, norm, work, rec_w, 0, 1, rec);
    __syncthreads();
    final_fold(B, kind, norm, scale, work, reward_out, 1, rec, &glob);
    if (!ret_out) return;
    __syncthreads();
    const int b = threadIdx.x;                       // batch_reward_select_kernel's row, B <= 64
    if (b >= B) return;
    bool nb;
    if (norm == PMENV_BNORM_GLOBAL_OR) nb = glob != 0;
    else if (norm == PMENV_BNORM_ROW_OR) nb = row_normalises(work[(size_t)B + b], work[2 * (size_t)B + b]);
    else nb = false;
    const double r = nb ? work[4 * (size_t)B + b] : work[3 * (size_t)B + b];
    work[b] = r;
    work[5 * (size_t)B + b] = nb ? 1.0 : 0.0;
    ret_out[b] = (float)r;
}

// elementwise: each row's chosen return and normalisation flag (for the backward)
static __global__ __launch_bounds__(256) void batch_reward_select_kernel(int B, int norm, double* work, float* ret_out) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= B) return;
    bool nb;
    if (norm == PMENV_BNORM_GLOBAL_OR) nb = work[6 * (size_t)B] != 0.0;
    else if (norm == PMENV_BNORM_ROW_OR) nb = row_normalises(work[(size_t)B + b], work[2 * (size_t)B + b]);
    else nb = false;
    const double r = nb ? work[4 * (size_t)B + b] : work[3 * (size_t)B + b];
    work[b] = r;
    work[5 * (size_t)B + b] = nb ? 1.0 : 0.0;
    if (ret_out) ret_out[b] = (float)r;
}

// one wave per row: dR/da through the (optional) softmax. EPL > 0 (N <= 64*EPL):
// the row is loaded once into registers (lane l: elements l + 64k) and every pass
// runs from them; EPL = 0: any N, re-reading the row per pass.
template <int EPL>
__global__ __launch_bounds__(256) void batch_reward_grad_kernel(const float* a, const float* v_prev, const float* p,
                                                                int B, int N, int kind, double scale,
                                                                const double* work, const float* grad_out,
                                                                float* grad_a) {
    constexpr int E = EPL > 0 ? EPL : 1;
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= B) return;
    float ra[E], rp[E];
    if (EPL > 0) {
        const uint32_t bytes = (uint32_t)B * (uint32_t)N * 4u;
        const auto rsa = make_rsrc(a, bytes), rsp = make_rsrc(p, bytes);
#pragma unroll
        for (int k = 0; k < E; ++k) {
            const int n = lane + 64 * k;
            const uint32_t off = n < N ? ((uint32_t)b * (uint32_t)N + (uint32_t)n) * 4u : 0xFFFFFFF0u;
            ra[k] = buf_load1(rsa, off);
            rp[k] = buf_load1(rsp, off);
        }
    }
    const double go = (double)*grad_out;
    // the per-row choice from the forward's workspace (its norm mode at work[6B+4]), as
    // the quad backward does: the forward needs no select pass for this kernel
    const int norm = (int)work[6 * (size_t)B + 4];
    bool nb;
    if (norm == PMENV_BNORM_GLOBAL_OR) nb = work[6 * (size_t)B] != 0.0;
    else if (norm == PMENV_BNORM_ROW_OR) nb = row_normalises(work[(size_t)B + b], work[2 * (size_t)B + b]);
    else nb = false;
    const double r = nb ? work[4 * (size_t)B + b] : work[3 * (size_t)B + b];
    double dr;
    if (kind == PMENV_REWARD_LOG_RETURN) dr = scale / ((double)B * r);
    else if (kind == PMENV_REWARD_RETURN) dr = scale / (double)B;
    else {
        const double m = work[6 * (size_t)B + 1], sd = work[6 * (size_t)B + 2];
        dr = scale * (1.0 / ((double)B * sd) - m * (r - m) / ((double)(B - 1) * sd * sd * sd));
    }
    dr *= go;
    const double v = (double)v_prev[b];
    if (EPL > 0) {
        float out[E];
        if (!nb) {
#pragma unroll
            for (int k = 0; k < E; ++k) out[k] = (float)(dr * (v * (double)rp[k]) / v);
        } else {
            double mx = -INFINITY;
#pragma unroll
            for (int k = 0; k < E; ++k)
                if (lane + 64 * k < N) mx = fmax(mx, (double)ra[k]);
            mx = wave_max(mx);
            double e[E], z = 0.0;
#pragma unroll
            for (int k = 0; k < E; ++k) {
                e[k] = lane + 64 * k < N ? exp((double)ra[k] - mx) : 0.0;
                z += e[k];
            }
            z = wave_sum(z);
            const double rz = 1.0 / z;
            double wg = 0.0;                           // sum_m w_m g_m
#pragma unroll
            for (int k = 0; k < E; ++k) wg += (e[k] * rz) * (dr * (v * (double)rp[k]) / v);
            wg = wave_sum(wg);
#pragma unroll
            for (int k = 0; k < E; ++k) out[k] = (float)((e[k] * rz) * (dr * (v * (double)rp[k]) / v - wg));
        }
#pragma unroll
        for (int k = 0; k < E; ++k)
            if (lane + 64 * k < N) grad_a[(size_t)b * N + lane + 64 * k] = out[k];
        return;
    }
    if (!nb) {
        for (int n = lane; n < N; n += 64)
            grad_a[(size_t)b * N + n] = (float)(dr * (v * (double)p[(size_t)b * N + n]) / v);
        return;
    }
    double mx = -INFINITY;
    for (int n = lane; n < N; n += 64) mx = fmax(mx, (double)a[(size_t)b * N + n]);
    mx = wave_max(mx);
    double z = 0.0;
    for (int n = lane; n < N; n += 64) z += exp((double)a[(size_t)b * N + n] - mx);
    z = wave_sum(z);
    double wg = 0.0;                               // sum_m w_m g_m
    for (int n = lane; n < N; n += 64) {
        const double w = exp((double)a[(size_t)b * N + n] - mx) / z;
        wg += w * (dr * (v * (double)p[(size_t)b * N + n]) / v);
    }
    wg = wave_sum(wg);
    for (int n = lane; n < N; n += 64) {
        const double w = exp((double)a[(size_t)b * N + n] - mx) / z;
        const double gn = dr * (v * (double)p[(size_t)b * N + n]) / v;
        grad_a[(size_t)b * N + n] = (float)(w * (gn - wg));
    }
}

}  // namespace pmenv_dev
