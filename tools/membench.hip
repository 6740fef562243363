// membench.hip — calibration of the memory patterns behind the fused env step
// (not product code). Build: hipcc --offload-arch=gfx950 -O3 -o membench membench.hip
// Every variant moves 2 x `bytes` (read + write); reported as GB/s of that sum.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

// 1. out-of-place grid-stride float4 copy
__global__ void copy_gs(const f4* __restrict__ a, f4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

// 2. out-of-place, one block per env block of `per` float4, all loads then all stores
template <int BLOCK, int V>
__global__ __launch_bounds__(BLOCK) void copy_env(const f4* __restrict__ a, f4* __restrict__ b, int per) {
    const f4* src = a + (size_t)blockIdx.x * per;
    f4* dst = b + (size_t)blockIdx.x * per;
    f4 r[V];
#pragma unroll
    for (int i = 0; i < V; ++i) { int q = threadIdx.x + i * BLOCK; if (q < per) r[i] = src[q]; }
#pragma unroll
    for (int i = 0; i < V; ++i) { int q = threadIdx.x + i * BLOCK; if (q < per) dst[q] = r[i]; }
}

// 3. in-place, one block per env, loads, barrier, stores (aligned: shift 0)
template <int BLOCK, int V, int SHIFT, bool NT>
__global__ __launch_bounds__(BLOCK) void inplace_env(float* x, int per) {
    float* e = x + (size_t)blockIdx.x * per * 4;
    f4 r[V];
    const int nq = per;
#pragma unroll
    for (int i = 0; i < V; ++i) {
        int q = threadIdx.x + i * BLOCK;
        int j = 4 * q + SHIFT;
        if (j + 3 < 4 * nq) {
            if (SHIFT % 4 == 0) r[i] = NT ? __builtin_nontemporal_load(reinterpret_cast<const f4*>(e + j)) : *reinterpret_cast<const f4*>(e + j);
            else { f4u v = *reinterpret_cast<const f4u*>(e + j); r[i] = f4{v.x, v.y, v.z, v.w}; }
        } else r[i] = f4{0, 0, 0, 0};
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < V; ++i) {
        int q = threadIdx.x + i * BLOCK;
        if (q < nq) {
            if (NT) __builtin_nontemporal_store(r[i], reinterpret_cast<f4*>(e) + q);
            else reinterpret_cast<f4*>(e)[q] = r[i];
        }
    }
}

// 4. persistent in-place: grid = k per CU, each block walks envs, double-buffered in registers
template <int BLOCK, int V>
__global__ __launch_bounds__(BLOCK) void inplace_persist(float* x, int per, int nenv) {
    f4 r0[V], r1[V];
    int b = blockIdx.x;
    auto load = [&](f4* r, int env) {
        const float* e = x + (size_t)env * per * 4;
#pragma unroll
        for (int i = 0; i < V; ++i) {
            int q = threadIdx.x + i * BLOCK;
            int j = 4 * q + 5;
            if (j + 3 < 4 * per) { f4u v = *reinterpret_cast<const f4u*>(e + j); r[i] = f4{v.x, v.y, v.z, v.w}; }
            else r[i] = f4{0, 0, 0, 0};
        }
    };
    auto store = [&](const f4* r, int env) {
        float* e = x + (size_t)env * per * 4;
#pragma unroll
        for (int i = 0; i < V; ++i) { int q = threadIdx.x + i * BLOCK; if (q < per) reinterpret_cast<f4*>(e)[q] = r[i]; }
    };
    if (b >= nenv) return;
    load(r0, b);
    while (true) {
        int nb = b + gridDim.x;
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        if (nb < nenv) load(r1, nb);
        store(r0, b);
        if (nb >= nenv) break;
        b = nb;
        nb = b + gridDim.x;
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        if (nb < nenv) load(r0, nb);
        store(r1, b);
        if (nb >= nenv) break;
        b = nb;
    }
}


// 5. grid-stride copy, U independent loads in flight per thread
template <int U>
__global__ __launch_bounds__(256) void copy_gs_u(const f4* __restrict__ a, f4* __restrict__ b, size_t n) {
    size_t stride = (size_t)gridDim.x * 256;
    size_t i = blockIdx.x * (size_t)256 + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        f4 r[U];
#pragma unroll
        for (int u = 0; u < U; ++u) r[u] = a[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) b[i + u * stride] = r[u];
    }
    for (; i < n; i += stride) b[i] = a[i];
}
// 6. contiguous chunk per block: block copies CH float4 consecutive, U in flight
template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_chunk(const f4* __restrict__ a, f4* __restrict__ b, size_t n) {
    const size_t base = (size_t)blockIdx.x * 256 * U;
    f4 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { size_t i = base + u * 256 + threadIdx.x; if (i < n) r[u] = NT ? __builtin_nontemporal_load(a + i) : a[i]; }
#pragma unroll
    for (int u = 0; u < U; ++u) { size_t i = base + u * 256 + threadIdx.x; if (i < n) { if (NT) __builtin_nontemporal_store(r[u], b + i); else b[i] = r[u]; } }
}
__global__ void read_only(const f4* __restrict__ a, size_t n, float* out) {
    f4 acc = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc += a[i];
    if (acc.x == 1234.5f) out[0] = acc.y;
}
template <int U>
__global__ __launch_bounds__(256) void read_chunk(const f4* __restrict__ a, size_t n, float* out) {
    const size_t base = (size_t)blockIdx.x * 256 * U;
    f4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u) { size_t i = base + u * 256 + threadIdx.x; if (i < n) acc += a[i]; }
    if (acc.x == 1234.5f) out[0] = acc.y;
}
__global__ void write_only(f4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = f4{1, 2, 3, 4};
}


// 7. in-place shifted copy, block = `unit` float4 (whole rows of 250 floats), V loads per thread
template <int BLOCK, int V>
__global__ __launch_bounds__(BLOCK) void inplace_unit(float* x, int unit) {
    float* e = x + (size_t)blockIdx.x * unit * 4;
    const int nf = unit * 4;
    f4 r[V];
#pragma unroll
    for (int i = 0; i < V; ++i) {
        int q = threadIdx.x + i * BLOCK;
        int j = 4 * q + 5;
        r[i] = f4{0, 0, 0, 0};
        if (j + 3 < nf) { f4u v = *reinterpret_cast<const f4u*>(e + j); r[i] = f4{v.x, v.y, v.z, v.w}; }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < V; ++i) {
        int q = threadIdx.x + i * BLOCK;
        if (q < unit) reinterpret_cast<f4*>(e)[q] = r[i];
    }
}
// 8. same, wave-contiguous mapping: wave w owns chunks [w*64*V, (w+1)*64*V)
template <int BLOCK, int V>
__global__ __launch_bounds__(BLOCK) void inplace_unit_wc(float* x, int unit) {
    float* e = x + (size_t)blockIdx.x * unit * 4;
    const int nf = unit * 4;
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    f4 r[V];
#pragma unroll
    for (int i = 0; i < V; ++i) {
        int q = w * 64 * V + i * 64 + l;
        int j = 4 * q + 5;
        r[i] = f4{0, 0, 0, 0};
        if (j + 3 < nf) { f4u v = *reinterpret_cast<const f4u*>(e + j); r[i] = f4{v.x, v.y, v.z, v.w}; }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < V; ++i) {
        int q = w * 64 * V + i * 64 + l;
        if (q < unit) reinterpret_cast<f4*>(e)[q] = r[i];
    }
}

// 9. in-place shifted copy through an LDS image (the product stream's structure, no side
// data, no halo): aligned own chunks -> LDS, barrier, two 16-B LDS reads, shift, store
template <int BLOCK, int V>
__global__ __launch_bounds__(BLOCK) void inplace_lds(float* x, int unit) {
    __shared__ f4 img[BLOCK * V + 2];
    f4* e = reinterpret_cast<f4*>(x) + (size_t)blockIdx.x * unit;
    f4 r[V];
#pragma unroll
    for (int i = 0; i < V; ++i) {
        const int q = threadIdx.x + i * BLOCK;
        r[i] = q < unit ? e[q] : f4{0, 0, 0, 0};
    }
#pragma unroll
    for (int i = 0; i < V; ++i) img[threadIdx.x + i * BLOCK] = r[i];
    if (threadIdx.x < 2) img[BLOCK * V + threadIdx.x] = f4{0, 0, 0, 0};
    __syncthreads();
#pragma unroll
    for (int i = 0; i < V; ++i) {
        const int q = threadIdx.x + i * BLOCK;
        const f4 a = img[q + 1], b = img[q + 2];
        if (q < unit) e[q] = f4{a.y, a.z, a.w, b.x};
    }
}

// fills the buffer with non-zero data (the product's windows are prices, not zeros)
__global__ void fill(float* x, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        x[i] = 100.0f + (float)(i % 977) * 0.013f;
}

template <typename F>
double timeit(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(a));
        f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2] * 1e-3;
}

int main(int argc, char** argv) {
    const int nenv = argc > 1 ? atoi(argv[1]) : 65536;
    const int per = 1875;                 // float4 per env: 30 x 50 x 5 floats
    const size_t n4 = (size_t)nenv * per;
    const double bytes = 2.0 * n4 * 16;
    f4 *a, *b;
    CK(hipMalloc(&a, n4 * 16 + 256));
    CK(hipMalloc(&b, n4 * 16 + 256));
    CK(hipMemset(a, 0, n4 * 16 + 256));
    CK(hipMemset(b, 0, n4 * 16 + 256));
    int reps = 20;
    if (argc > 2 && atoi(argv[2]) == 1) {    // the LDS-image probe only, on non-zero data
        fill<<<4096, 256>>>((float*)a, n4 * 4);
        CK(hipDeviceSynchronize());
        auto rep2 = [&](const char* name, double s) { printf("%-40s %8.1f us  %7.1f GB/s\n", name, s * 1e6, bytes / s / 1e9); };
        char nm[80];
#define RUNL(BL, V, UNIT) snprintf(nm, sizeof nm, "inplace lds  %4d f4 %4dx%d", UNIT, BL, V); \
        rep2(nm, timeit([&] { inplace_lds<BL, V><<<(unsigned)(n4 / UNIT), BL>>>((float*)a, UNIT); }, reps));
#define RUNU(BL, V, UNIT) snprintf(nm, sizeof nm, "inplace unit %4d f4 %4dx%d", UNIT, BL, V); \
        rep2(nm, timeit([&] { inplace_unit<BL, V><<<(unsigned)(n4 / UNIT), BL>>>((float*)a, UNIT); }, reps));
        RUNU(256, 2, 500) RUNU(512, 1, 500) RUNU(512, 4, 1875) RUNU(1024, 2, 1875)
        RUNL(256, 2, 512) RUNL(512, 1, 512) RUNL(512, 2, 1024) RUNL(256, 4, 1024) RUNL(1024, 2, 2048)
        RUNL(256, 2, 500) RUNL(512, 4, 1875) RUNL(1024, 2, 1875)
        CK(hipFree(a)); CK(hipFree(b));
        return 0;
    }
    auto rep = [&](const char* name, double s) { printf("%-40s %8.1f us  %7.1f GB/s\n", name, s * 1e6, bytes / s / 1e9); };
    float* dummy; CK(hipMalloc(&dummy, 64));
    {
        struct U { int unit; } units[] = {{375}, {500}, {625}, {750}, {1875}};
        (void)units;
        char nm[80];
#define RUN(BL, V, UNIT) snprintf(nm, sizeof nm, "inplace unit %4d f4 %4dx%d", UNIT, BL, V); \
        rep(nm, timeit([&] { inplace_unit<BL, V><<<(unsigned)(n4 / UNIT), BL>>>((float*)a, UNIT); }, reps));
        RUN(128, 3, 375) RUN(192, 2, 375) RUN(64, 6, 375) RUN(384, 1, 375)
        RUN(256, 2, 500) RUN(128, 4, 500) RUN(512, 1, 500)
        RUN(320, 2, 625) RUN(256, 3, 625) RUN(640, 1, 625)
        RUN(384, 2, 750) RUN(256, 3, 750) RUN(768, 1, 750)
        RUN(512, 4, 1875) RUN(1024, 2, 1875) RUN(640, 3, 1875)
#define RUNW(BL, V, UNIT) snprintf(nm, sizeof nm, "inplace unit wc %4d f4 %4dx%d", UNIT, BL, V); \
        rep(nm, timeit([&] { inplace_unit_wc<BL, V><<<(unsigned)(n4 / UNIT), BL>>>((float*)a, UNIT); }, reps));
        RUNW(256, 8, 1875) RUNW(512, 4, 1875) RUNW(128, 4, 500) RUNW(256, 2, 500)
    }
    rep("hipMemcpyAsync D2D", timeit([&] { CK(hipMemcpyAsync(b, a, n4 * 16, hipMemcpyDeviceToDevice, 0)); }, reps));
    rep("copy gs U4 2048x256", timeit([&] { copy_gs_u<4><<<2048, 256>>>(a, b, n4); }, reps));
    rep("copy gs U8 1024x256", timeit([&] { copy_gs_u<8><<<1024, 256>>>(a, b, n4); }, reps));
    rep("copy gs U4 8192x256", timeit([&] { copy_gs_u<4><<<8192, 256>>>(a, b, n4); }, reps));
    rep("copy chunk U4", timeit([&] { copy_chunk<4, false><<<(n4 + 1023) / 1024, 256>>>(a, b, n4); }, reps));
    rep("copy chunk U8", timeit([&] { copy_chunk<8, false><<<(n4 + 2047) / 2048, 256>>>(a, b, n4); }, reps));
    rep("copy chunk U16", timeit([&] { copy_chunk<16, false><<<(n4 + 4095) / 4096, 256>>>(a, b, n4); }, reps));
    rep("copy chunk U8 nt", timeit([&] { copy_chunk<8, true><<<(n4 + 2047) / 2048, 256>>>(a, b, n4); }, reps));
    rep("copy chunk U2", timeit([&] { copy_chunk<2, false><<<(n4 + 511) / 512, 256>>>(a, b, n4); }, reps));
    rep("(x2) read-only gs 4096x256", timeit([&] { read_only<<<4096, 256>>>(a, n4, dummy); }, reps) * 2);
    rep("(x2) read chunk U8", timeit([&] { read_chunk<8><<<(n4 + 2047) / 2048, 256>>>(a, n4, dummy); }, reps) * 2);
    rep("(x2) write-only gs 4096x256", timeit([&] { write_only<<<4096, 256>>>(b, n4); }, reps) * 2);
    rep("copy grid-stride 2048x256", timeit([&] { copy_gs<<<2048, 256>>>(a, b, n4); }, reps));
    rep("copy grid-stride 8192x256", timeit([&] { copy_gs<<<8192, 256>>>(a, b, n4); }, reps));
    rep("copy env-block 256x8", timeit([&] { copy_env<256, 8><<<nenv, 256>>>(a, b, per); }, reps));
    rep("copy env-block 512x4", timeit([&] { copy_env<512, 4><<<nenv, 512>>>(a, b, per); }, reps));
    rep("inplace env 256x8 shift0", timeit([&] { inplace_env<256, 8, 0, false><<<nenv, 256>>>((float*)a, per); }, reps));
    rep("inplace env 256x8 shift0 nt", timeit([&] { inplace_env<256, 8, 0, true><<<nenv, 256>>>((float*)a, per); }, reps));
    rep("inplace env 256x8 shift5", timeit([&] { inplace_env<256, 8, 5, false><<<nenv, 256>>>((float*)a, per); }, reps));
    rep("inplace env 512x4 shift5", timeit([&] { inplace_env<512, 4, 5, false><<<nenv, 512>>>((float*)a, per); }, reps));
    rep("inplace env 1024x2 shift5", timeit([&] { inplace_env<1024, 2, 5, false><<<nenv, 1024>>>((float*)a, per); }, reps));
    for (int g : {256, 512, 1024, 2048}) {
        char nm[64];
        snprintf(nm, sizeof nm, "inplace persist 256x8 grid %d", g);
        rep(nm, timeit([&] { inplace_persist<256, 8><<<g, 256>>>((float*)a, per, nenv); }, reps));
    }
    for (int g : {512, 1024}) {
        char nm[64];
        snprintf(nm, sizeof nm, "inplace persist 512x4 grid %d", g);
        rep(nm, timeit([&] { inplace_persist<512, 4><<<g, 512>>>((float*)a, per, nenv); }, reps));
    }
    CK(hipFree(a)); CK(hipFree(b));
    return 0;
}
