// exp_check.hip — TOOLS: tools/ab/fmath.h's exp_f64 against the device library's exp(double), bit
// for bit, on the GPU: random doubles over the whole range checks, random bit patterns
// (every exponent: NaN, inf, subnormals), dense sweeps around the range checks' edges and
// rint's half-way points (x log2 e near k + 1/2), and the special values.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/exp_check tools/exp_check.hip
//   ./tools/exp_check            -> "exp_check: N inputs, M mismatches"
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "ab/fmath.h"

__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// mode 0: uniform in [-1100, 1100]; 1: random bits; 2: near the edges; 3: rint half-way points
__device__ double input(uint64_t i, int mode) {
    const uint64_t z = mix(i * 4 + (uint64_t)mode);
    if (mode == 0) return -1100.0 + 2200.0 * (double)(z >> 11) * 0x1p-53;
    if (mode == 1) { double d; uint64_t b = z; memcpy(&d, &b, 8); return d; }
    if (mode == 2) {
        const double edges[] = {1024.0, -1075.0, 709.782712893384, -708.3964185322641, -745.1332191019412, 0.0,
                                -1074.5, 1023.5, 1e-300, -1e-300};
        const double e = edges[z % 10];
        const int64_t k = (int64_t)((z >> 8) % 200001) - 100000;          // +-1e5 ulps
        double d = e;
        uint64_t b; memcpy(&b, &d, 8);
        if (e != 0.0) b += (uint64_t)k; else b = (uint64_t)(k < 0 ? -k : k) | (k < 0 ? 0x8000000000000000ull : 0);
        memcpy(&d, &b, 8);
        return d;
    }
    const int64_t kk = (int64_t)((z >> 20) % 3000) - 1500;               // x log2 e = kk + 1/2 +- a few ulps
    double d = ((double)kk + 0.5) / 0x1.71547652b82fep+0;
    uint64_t b; memcpy(&b, &d, 8);
    b += (uint64_t)((int64_t)(z % 9) - 4);
    memcpy(&d, &b, 8);
    return d;
}

__global__ void check(uint64_t n, int mode, unsigned long long* bad, double* first) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const double x = input(i, mode);
        const double a = exp(x), b = pmenv_dev::exp_f64(x);
        uint64_t ua, ub;
        memcpy(&ua, &a, 8);
        memcpy(&ub, &b, 8);
        if (ua != ub) {
            if (atomicAdd(bad, 1ull) == 0) first[0] = x;
        }
    }
}

__global__ void specials(unsigned long long* bad) {
    const double xs[] = {0.0, -0.0, 1.0, -1.0, INFINITY, -INFINITY, NAN, -NAN, 1024.0, -1075.0, 709.0, 710.0,
                         -745.0, -746.0, 1e-320, -1e-320, 0x1p-1074, 1e308, -1e308};
    for (double x : xs) {
        const double a = exp(x), b = pmenv_dev::exp_f64(x);
        uint64_t ua, ub;
        memcpy(&ua, &a, 8);
        memcpy(&ub, &b, 8);
        if (ua != ub) atomicAdd(bad, 1ull);
    }
}

int main() {
    unsigned long long* bad;
    double* first;
    if (hipMalloc(&bad, 8) != hipSuccess || hipMalloc(&first, 8) != hipSuccess) return 2;
    unsigned long long total = 0, nin = 0;
    const uint64_t n = 1ull << 26;
    for (int mode = 0; mode < 4; ++mode) {
        unsigned long long h = 0;
        double f = 0;
        (void)hipMemset(bad, 0, 8);
        check<<<4096, 256>>>(n, mode, bad, first);
        if (hipDeviceSynchronize() != hipSuccess) return 3;
        (void)hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(&f, first, 8, hipMemcpyDeviceToHost);
        printf("exp_check mode %d: %llu inputs, %llu mismatches%s", mode, (unsigned long long)n, h, h ? "" : "\n");
        if (h) printf(" (first at x = %.17g)\n", f);
        total += h;
        nin += n;
    }
    (void)hipMemset(bad, 0, 8);
    specials<<<1, 1>>>(bad);
    unsigned long long hs = 0;
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    (void)hipMemcpy(&hs, bad, 8, hipMemcpyDeviceToHost);
    printf("exp_check specials: %llu mismatches\n", hs);
    printf("exp_check: %llu inputs, %llu mismatches\n", nin + 19, total + hs);
    return total + hs ? 1 : 0;
}
