// copybench.hip — is the out-of-place stream ceiling of this chip above the 5.8 TB/s
// the advance kernel is calibrated against? (not product code)
// Build: hipcc --offload-arch=gfx950 -O3 -o copybench copybench.hip
// Variants of a 2 x `bytes` float4 copy (2.0 GB -> 2.0 GB, the advance kernel's size):
// block size, chunk per workgroup, cache-policy bits on the loads and stores
// (aux: 1 = sc0, 2 = nt, 16 = sc1), LDS-DMA loads, persistent software pipeline.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

typedef unsigned int u4v __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

// one workgroup copies BLOCK*U float4 (contiguous), all loads first
template <int BLOCK, int U, int LAUX, int SAUX>
__global__ __launch_bounds__(BLOCK) void copy_chunk(const u4v* a, u4v* b, size_t n) {
    const size_t base = (size_t)blockIdx.x * BLOCK * U;
    const uint32_t bytes = (uint32_t)(min((size_t)BLOCK * U, n - base) * 16);
    const auto ra = rsrc(a + base, bytes);
    const auto rb = rsrc(b + base, bytes);
    u4v r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = __builtin_amdgcn_raw_buffer_load_b128(ra, (uint32_t)(u * BLOCK + threadIdx.x) * 16u, 0, LAUX);
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_amdgcn_raw_buffer_store_b128(r[u], rb, (uint32_t)(u * BLOCK + threadIdx.x) * 16u, 0, SAUX);
}

// wave-contiguous variant: each wave owns U consecutive KiB
template <int BLOCK, int U, int LAUX, int SAUX>
__global__ __launch_bounds__(BLOCK) void copy_wave(const u4v* a, u4v* b, size_t n) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const size_t base = (size_t)blockIdx.x * BLOCK * U + (size_t)w * 64 * U;
    const uint32_t bytes = base < n ? (uint32_t)(min((size_t)64 * U, n - base) * 16) : 0u;
    const auto ra = rsrc(a + base, bytes);
    const auto rb = rsrc(b + base, bytes);
    u4v r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = __builtin_amdgcn_raw_buffer_load_b128(ra, (uint32_t)(u * 64 + l) * 16u, 0, LAUX);
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_amdgcn_raw_buffer_store_b128(r[u], rb, (uint32_t)(u * 64 + l) * 16u, 0, SAUX);
}

// persistent: grid of G workgroups walks chunks of BLOCK*U float4, next chunk's loads
// issued before the current chunk's stores
template <int BLOCK, int U, int LAUX, int SAUX>
__global__ __launch_bounds__(BLOCK) void copy_persist(const u4v* a, u4v* b, size_t n) {
    const size_t nch = (n + (size_t)BLOCK * U - 1) / ((size_t)BLOCK * U);
    size_t c = blockIdx.x;
    if (c >= nch) return;
    u4v r0[U], r1[U];
    auto ld = [&](u4v* r, size_t ch) {
        const size_t base = ch * BLOCK * U;
        const auto ra = rsrc(a + base, (uint32_t)(min((size_t)BLOCK * U, n - base) * 16));
#pragma unroll
        for (int u = 0; u < U; ++u) r[u] = __builtin_amdgcn_raw_buffer_load_b128(ra, (uint32_t)(u * BLOCK + threadIdx.x) * 16u, 0, LAUX);
    };
    auto st = [&](const u4v* r, size_t ch) {
        const size_t base = ch * BLOCK * U;
        const auto rb = rsrc(b + base, (uint32_t)(min((size_t)BLOCK * U, n - base) * 16));
#pragma unroll
        for (int u = 0; u < U; ++u) __builtin_amdgcn_raw_buffer_store_b128(r[u], rb, (uint32_t)(u * BLOCK + threadIdx.x) * 16u, 0, SAUX);
    };
    ld(r0, c);
    while (true) {
        size_t nc = c + gridDim.x;
        if (nc < nch) ld(r1, nc);
        st(r0, c);
        if (nc >= nch) break;
        c = nc;
        nc = c + gridDim.x;
        if (nc < nch) ld(r0, nc);
        st(r1, c);
        if (nc >= nch) break;
        c = nc;
    }
}

// read-only and write-only references
template <int BLOCK, int U, int LAUX>
__global__ __launch_bounds__(BLOCK) void read_chunk(const u4v* a, size_t n, unsigned* out) {
    const size_t base = (size_t)blockIdx.x * BLOCK * U;
    const auto ra = rsrc(a + base, (uint32_t)(min((size_t)BLOCK * U, n - base) * 16));
    u4v acc = {0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= __builtin_amdgcn_raw_buffer_load_b128(ra, (uint32_t)(u * BLOCK + threadIdx.x) * 16u, 0, LAUX);
    if (acc.x == 0x12345u && acc.y == 0x777u) out[0] = acc.z;
}
template <int BLOCK, int U, int SAUX>
__global__ __launch_bounds__(BLOCK) void write_chunk(u4v* b, size_t n) {
    const size_t base = (size_t)blockIdx.x * BLOCK * U;
    const auto rb = rsrc(b + base, (uint32_t)(min((size_t)BLOCK * U, n - base) * 16));
    const u4v v = {1u, 2u, 3u, (unsigned)threadIdx.x};
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_amdgcn_raw_buffer_store_b128(v, rb, (uint32_t)(u * BLOCK + threadIdx.x) * 16u, 0, SAUX);
}

__global__ void fill_random(u4v* a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t)(i * 2654435761u) ^ (uint32_t)(i >> 32);
        u4v v;
        for (int k = 0; k < 4; ++k) {
            h ^= h >> 16; h *= 0x7feb352du; h ^= h >> 15; h *= 0x846ca68bu; h ^= h >> 16;
            v[k] = 0x3f000000u | (h & 0x007fffffu);     // floats in [0.5, 1)
        }
        a[i] = v;
    }
}

template <typename F>
double timeit(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f(); f();
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
    const size_t mb = argc > 1 ? (size_t)atol(argv[1]) : 1967;      // MB per buffer (advance kernel: 1.97 GB)
    const size_t n4 = mb * 1000000 / 16;
    const double bytes = 2.0 * n4 * 16;
    u4v *a, *b;
    CK(hipMalloc(&a, n4 * 16 + 4096));
    CK(hipMalloc(&b, n4 * 16 + 4096));
    CK(hipMemset(a, 1, n4 * 16 + 4096));
    CK(hipMemset(b, 0, n4 * 16 + 4096));
    const bool rnd = argc > 2 && atoi(argv[2]) != 0;        // random float data instead of a byte pattern
    if (rnd) { fill_random<<<4096, 256>>>(a, n4 + 256); CK(hipDeviceSynchronize()); }
    unsigned* dummy; CK(hipMalloc(&dummy, 64));
    const int reps = 15;
    printf("buffers: %zu MB each, %s data\n", mb, rnd ? "random" : "0x01-byte");
    auto rep = [&](const char* name, double s, double mult = 1.0) { printf("%-44s %8.1f us  %7.1f GB/s\n", name, s * 1e6, bytes * mult / s / 1e9); };
#define CH(BL, U, LA, SA) rep("chunk " #BL "x" #U " l" #LA " s" #SA, timeit([&] { copy_chunk<BL, U, LA, SA><<<(unsigned)((n4 + BL * U - 1) / (BL * U)), BL>>>(a, b, n4); }, reps));
#define WV(BL, U, LA, SA) rep("wave " #BL "x" #U " l" #LA " s" #SA, timeit([&] { copy_wave<BL, U, LA, SA><<<(unsigned)((n4 + BL * U - 1) / (BL * U)), BL>>>(a, b, n4); }, reps));
#define PS(BL, U, G, LA, SA) rep("persist " #BL "x" #U " g" #G " l" #LA " s" #SA, timeit([&] { copy_persist<BL, U, LA, SA><<<G, BL>>>(a, b, n4); }, reps));
    CH(256, 2, 0, 0) CH(256, 1, 0, 0) CH(128, 2, 0, 0) CH(64, 4, 0, 0) CH(512, 2, 0, 0) CH(256, 4, 0, 0)
    CH(512, 4, 0, 0) CH(1024, 2, 0, 0)
    CH(256, 2, 2, 0) CH(256, 2, 0, 2) CH(256, 2, 2, 2) CH(256, 2, 0, 16) CH(256, 2, 2, 16) CH(256, 2, 16, 0)
    CH(256, 2, 1, 0) CH(256, 2, 0, 1) CH(256, 2, 3, 3) CH(256, 2, 2, 18)
    CH(512, 4, 2, 0) CH(512, 4, 0, 16)
    WV(256, 4, 0, 0) WV(256, 8, 0, 0) WV(256, 2, 0, 0) WV(512, 4, 0, 0) WV(256, 4, 2, 0) WV(256, 4, 0, 16)
    PS(256, 4, 2048, 0, 0) PS(256, 4, 4096, 0, 0) PS(256, 8, 2048, 0, 0) PS(512, 4, 1024, 0, 0) PS(256, 4, 2048, 2, 0)
    PS(256, 2, 4096, 0, 0) PS(256, 4, 1024, 0, 0)
    rep("memcpy D2D", timeit([&] { CK(hipMemcpyAsync(b, a, n4 * 16, hipMemcpyDeviceToDevice, 0)); }, reps));
#define RD(BL, U, LA) rep("(x2) read " #BL "x" #U " l" #LA, timeit([&] { read_chunk<BL, U, LA><<<(unsigned)((n4 + BL * U - 1) / (BL * U)), BL>>>(a, n4, dummy); }, reps) * 2);
#define WR(BL, U, SA) rep("(x2) write " #BL "x" #U " s" #SA, timeit([&] { write_chunk<BL, U, SA><<<(unsigned)((n4 + BL * U - 1) / (BL * U)), BL>>>(b, n4); }, reps) * 2);
    RD(256, 2, 0) RD(256, 8, 0) RD(256, 2, 2) RD(256, 8, 2)
    WR(256, 2, 0) WR(256, 8, 0) WR(256, 2, 2) WR(256, 2, 16) WR(256, 8, 16)
    CK(hipFree(a)); CK(hipFree(b));
    return 0;
}
