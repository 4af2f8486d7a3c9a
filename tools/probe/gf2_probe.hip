// Latency of one wave's GF(2) products (the fold arithmetic at a wave's range
// end runs on the kernel's critical path with the rest of the CU idle).
//   hipcc -O3 --offload-arch=gfx950 -o build/gf2_probe tools/probe/gf2_probe.hip
// Prints ns per product for each form, one wave alone on the GPU, chained
// (each product's input depends on the previous output).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define POLY 0xedb88320u

__host__ __device__ constexpr uint32_t cx_mult(uint32_t a, uint32_t b)
{
    uint32_t p = 0;
    for (int i = 31; i >= 0; --i) {
        if ((a >> i) & 1u) p ^= b;
        b = (b & 1u) ? (b >> 1) ^ POLY : (b >> 1);
    }
    return p;
}
constexpr uint32_t cx_xpow8n(uint64_t n)
{
    uint32_t r = 0x80000000u, sq = 0x00800000u;
    while (n) {
        if (n & 1u) r = cx_mult(sq, r);
        sq = cx_mult(sq, sq);
        n >>= 1;
    }
    return r;
}

__device__ __forceinline__ uint32_t serial(uint32_t a, uint32_t b)
{
    uint32_t p = 0;
#pragma unroll
    for (int i = 31; i >= 0; --i) {
        p ^= b & (0u - ((a >> i) & 1u));
        b = (b >> 1) ^ (POLY & (0u - (b & 1u)));
    }
    return p;
}

template <uint32_t C> struct Cols {
    uint32_t v[32];
    constexpr Cols() : v{} { for (int j = 0; j < 32; ++j) v[j] = cx_mult(C, 1u << j); }
};

template <uint32_t C>
__device__ __forceinline__ uint32_t mulconst_tree(uint32_t b)
{
    constexpr Cols<C> K;
    uint32_t p[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        p[j & 3] = __builtin_amdgcn_bitop3_b32(p[j & 3], 0u - ((b >> j) & 1u), K.v[j], 0x78);
    }
    return __builtin_amdgcn_bitop3_b32(p[0], p[1], p[2], 0x96) ^ p[3];
}

template <uint32_t C>
__device__ __forceinline__ uint32_t mulconst_serial(uint32_t b)
{
    constexpr Cols<C> K;
    uint32_t p = 0;
#pragma unroll
    for (int j = 0; j < 32; ++j) p ^= K.v[j] & (0u - ((b >> j) & 1u));
    return p;
}

// a * b with four independent 8-step chains from b, b x^8, b x^16, b x^24.
__device__ __forceinline__ uint32_t split4(uint32_t a, uint32_t b)
{
    uint32_t bk[4] = {b, mulconst_tree<cx_xpow8n(1)>(b), mulconst_tree<cx_xpow8n(2)>(b),
                      mulconst_tree<cx_xpow8n(3)>(b)};
    uint32_t p[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            p[k] = __builtin_amdgcn_bitop3_b32(p[k], 0u - ((a >> (31 - 8 * k - j)) & 1u), bk[k], 0x78);
            bk[k] = __builtin_amdgcn_bitop3_b32(bk[k] >> 1, 0u - (bk[k] & 1u), POLY, 0x78);
        }
    }
    return __builtin_amdgcn_bitop3_b32(p[0], p[1], p[2], 0x96) ^ p[3];
}

template <int V>
__global__ void probe(const uint32_t *in, uint32_t *out, unsigned long long *t, int reps)
{
    uint32_t a = in[threadIdx.x], b = in[64 + threadIdx.x];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int r = 0; r < reps; ++r) {
        uint32_t x;
        if (V == 0) x = serial(a, b);
        else if (V == 1) x = split4(a, b);
        else if (V == 2) x = mulconst_serial<cx_xpow8n(1024)>(b);
        else if (V == 3) x = mulconst_tree<cx_xpow8n(1024)>(b);
        else x = serial(cx_xpow8n(1024), b);
        b = x ^ (uint32_t) r;
        asm volatile("" : "+v"(b), "+v"(a));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    out[threadIdx.x] = b;
    if (threadIdx.x == 0) *t = t1 - t0;
}

int main()
{
    uint32_t h[128];
    for (int i = 0; i < 128; ++i) h[i] = 0x9e3779b9u * (i + 1);
    uint32_t *in, *out;
    unsigned long long *t;
    hipMalloc(&in, sizeof h);
    hipMalloc(&out, 64 * 4);
    hipMalloc(&t, 8);
    hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice);
    const int reps = 1000;
    const char *names[] = {"serial multmodp(a, b)", "split4 multmodp(a, b)", "mulconst serial", "mulconst tree",
                           "serial multmodp(const, b)"};
    void (*ks[])(const uint32_t *, uint32_t *, unsigned long long *, int) = {probe<0>, probe<1>, probe<2>, probe<3>, probe<4>};
    uint32_t ref[64];
    for (int v = 0; v < 5; ++v) {
        unsigned long long best = ~0ull, tt;
        for (int it = 0; it < 5; ++it) {
            hipLaunchKernelGGL(ks[v], dim3(1), dim3(64), 0, 0, in, out, t, reps);
            hipMemcpy(&tt, t, 8, hipMemcpyDeviceToHost);
            best = tt < best ? tt : best;
        }
        uint32_t o[64];
        hipMemcpy(o, out, sizeof o, hipMemcpyDeviceToHost);
        if (v == 0) for (int i = 0; i < 64; ++i) ref[i] = o[i];
        if (v == 1) {
            bool same = true;
            for (int i = 0; i < 64; ++i) same &= o[i] == ref[i];
            printf("split4 == serial: %s\n", same ? "yes" : "NO");
        }
        printf("%-28s %7.1f ns per product (one wave alone)\n", names[v], best * 10.0 / reps);
    }
    return 0;
}
