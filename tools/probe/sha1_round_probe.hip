// sha1_round_probe.hip -- what bounds one SHA-1 round chain on a gfx950 SIMD?
//
// Each wave runs ITERS x 80 SHA-1 rounds on register-resident K+W words (no
// memory), lane-parallel (64 independent chains).  Per wave it records
// s_memtime (shader clock) and s_memrealtime (100 MHz) around the loop, so
// the output is cycles per round and the clock.  Modes:
//   0: the round as sha1_gpu.hip writes it, the compiler picking the order
//      (with K+W in registers it emits e + K+W off the chain, then add3)
//   1: X = add3(e, K+W, f) first (off the chain), then a' = rotl5(a) + X
//      (two dependent instructions), forced with inline asm
//   2: the order the compiler emits in sha1_kernel, where K+W arrives from LDS
//      late: y = rotl5(a) + e, then a' = add3(y, K+W, f) (three dependent)
//   3: 80 distinct K+W registers (as many live registers as sha1_kernel's rows)
//   4: per block, the 80 K+W words read from LDS (20 ds_read_b128, as sha1_kernel)
//   5: mode 4 plus one __syncthreads() per block (the kernel's hand-over barrier)
// Launching 1, 4 and 8 waves per workgroup (one workgroup) puts 1 wave on one
// SIMD, 1 wave on each of 4 SIMDs, and 2 waves on each SIMD: if two waves on
// one SIMD take no longer per round than one, a lone chain is latency-bound,
// not issue-bound.
//
// Build: hipcc -O3 --offload-arch=gfx950 -o sha1_round_probe sha1_round_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { if ((x) != hipSuccess) { printf("hip error line %d\n", __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }

__device__ __forceinline__ void rounds80(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d, uint32_t &e,
                                         const uint32_t *kw, int mode)
{
#pragma unroll
    for (int r = 0; r < 80; ++r) {
        uint32_t f;
        if (r < 20) {
            f = __builtin_amdgcn_bitop3_b32(b, c, d, 0xCA);
        } else if (r < 40 || r >= 60) {
            f = __builtin_amdgcn_bitop3_b32(b, c, d, 0x96);
        } else {
            f = __builtin_amdgcn_bitop3_b32(b, c, d, 0xE8);
        }
        const uint32_t k = kw[mode == 0 || mode == 1 || mode == 2 ? (r & 15) : r];
        uint32_t tmp;
        if (mode == 2) {
            uint32_t y, r5 = rotl(a, 5);
            asm volatile("v_add_u32 %0, %1, %2" : "=v"(y) : "v"(r5), "v"(e));
            asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(tmp) : "v"(y), "v"(k), "v"(f));
        } else if (mode == 1) {
            uint32_t x, r5;
            asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(x) : "v"(e), "v"(k), "v"(f));
            r5 = rotl(a, 5);
            asm volatile("v_add_u32 %0, %1, %2" : "=v"(tmp) : "v"(r5), "v"(x));
        } else {
            tmp = rotl(a, 5) + f + e + k;
        }
        e = d;
        d = c;
        c = rotl(b, 30);
        b = a;
        a = tmp;
    }
}

template <int MODE>
__global__ void __launch_bounds__(512) probe(uint32_t *out, unsigned long long *t, int iters)
{
    __shared__ uint4 lds[20][512];
    uint32_t kw[80];
#pragma unroll
    for (int k = 0; k < 80; ++k) {
        kw[k] = threadIdx.x * 0x9E3779B9u + k * 0x7F4A7C15u;
    }
    if (MODE >= 4) {
        for (int r = 0; r < 20; ++r) {
            lds[r][threadIdx.x] = make_uint4(kw[4 * r], kw[4 * r + 1], kw[4 * r + 2], kw[4 * r + 3]);
        }
        __syncthreads();
    }
    uint32_t a = threadIdx.x, b = a * 3u, c = a * 5u, d = a * 7u, e = a * 11u;
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
        if (MODE >= 4) {
            uint32_t w[80];
#pragma unroll
            for (int r = 0; r < 20; ++r) {
                const uint4 q = lds[r][threadIdx.x];
                w[4 * r] = q.x; w[4 * r + 1] = q.y; w[4 * r + 2] = q.z; w[4 * r + 3] = q.w;
            }
            rounds80(a, b, c, d, e, w, 3);
            if (MODE == 5) {
                __syncthreads();
            }
        } else {
            rounds80(a, b, c, d, e, kw, MODE);
        }
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = a ^ b ^ c ^ d ^ e;
    if ((threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        t[2 * w] = c1 - c0;
        t[2 * w + 1] = r1 - r0;
    }
}

template <int MODE>
static int run(uint32_t *out, unsigned long long *t, int iters, int waves, double *cyc, double *real)
{
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(probe<MODE>, dim3(1), dim3(64 * waves), 0, 0, out, t, iters);
        CK(hipDeviceSynchronize());
    }
    unsigned long long h[2 * 8];
    CK(hipMemcpy(h, t, 2 * waves * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    *cyc = 0;
    *real = 0;
    for (int w = 0; w < waves; ++w) {
        *cyc += (double) h[2 * w];
        *real += (double) h[2 * w + 1];
    }
    *cyc /= waves;
    *real /= waves;
    return 0;
}

int main()
{
    const int iters = 2000;
    uint32_t *out;
    unsigned long long *t;
    CK(hipMalloc(&out, 512 * 16 * sizeof(uint32_t)));
    CK(hipMalloc(&t, 2 * 8 * 16 * sizeof(unsigned long long)));
    for (int mode = 0; mode < 6; ++mode) {
        for (int waves : {1, 4, 8}) {
            double cyc = 0, real = 0;
            int rc = 0;
            switch (mode) {
            case 0: rc = run<0>(out, t, iters, waves, &cyc, &real); break;
            case 1: rc = run<1>(out, t, iters, waves, &cyc, &real); break;
            case 2: rc = run<2>(out, t, iters, waves, &cyc, &real); break;
            case 3: rc = run<3>(out, t, iters, waves, &cyc, &real); break;
            case 4: rc = run<4>(out, t, iters, waves, &cyc, &real); break;
            default: rc = run<5>(out, t, iters, waves, &cyc, &real); break;
            }
            if (rc) {
                return rc;
            }
            const double rounds = 80.0 * iters;
            printf("mode %d waves %d: %.2f cycles/round (s_memtime), %.2f ns/round, clock %.3f GHz\n", mode, waves,
                   cyc / rounds, real * 10.0 / rounds, cyc / (real * 10.0));
        }
    }
    hipError_t e = hipGetLastError();
    printf("status %s\n", hipGetErrorString(e));
    return e == hipSuccess ? 0 : 1;
}
