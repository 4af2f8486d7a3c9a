// crc_probe.hip -- isolation probe for the CRC stream kernel's inner loop.
//
// Standalone (not part of libchunkio_amd.so).  Every variant streams the same
// byte range (total bytes split evenly over the persistent waves of one
// 1024-thread workgroup per CU, LDS sized like the product kernel) and
// differs only in the access pattern / compute, so their GB/s isolates the
// limiter:
//   0 strided64-nt  + CRC   lane owns 64 contiguous bytes of a 4 KiB step
//   1 strided64     + CRC   same, plain loads
//   2 compute only          CRC on register data, no loads
//   3 strided64 loads only  XOR of the loaded words
//   4 coalesced loads only  lane l reads bytes [16 l, 16 l + 16) of each 1 KiB
//   5 coalesced     + CRC4  4 sub-chains per lane (16 B each), 4080-B shift
//   6 coalesced-nt loads only
// Build: hipcc -O3 --offload-arch=gfx950 -o crc_probe crc_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

constexpr uint32_t POLY = 0xEDB88320u;
constexpr int kThreads = 1024;
constexpr int kStep = 4096;
constexpr uint32_t kSlice = 131072;
constexpr uint32_t kShiftOff = kSlice;            // 32 KiB replicated shift table
constexpr uint32_t kLdsBytes = kSlice + 32768;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld(const uint8_t *p)
{
    if (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    return *reinterpret_cast<const u32x4 *>(p);
}

template <int K>
__device__ __forceinline__ uint32_t tl(const char *lds, uint32_t lb, uint32_t b)
{
    return *reinterpret_cast<const uint32_t *>(lds + ((K >> 1) << 16) + ((K & 1) << 7) + ((b << 8) | lb));
}

__device__ __forceinline__ uint32_t word_step(const char *lds, uint32_t lb, uint32_t s, uint32_t w)
{
    const uint32_t x = s ^ w;
    return tl<3>(lds, lb, x & 0xffu) ^ tl<2>(lds, lb, (x >> 8) & 0xffu) ^
           tl<1>(lds, lb, (x >> 16) & 0xffu) ^ tl<0>(lds, lb, x >> 24);
}

// v_perm_b32 address path: D.byte[i] = {S0,S1}.byte[sel.byte[i]], S1 = bytes 0-3,
// S0 = bytes 4-7, selector 0x0c -> 0x00.  addr = {0, table-hi, x.byte_k, lane*4}
template <int K>
__device__ __forceinline__ uint32_t tlp(const char *lds, uint32_t x, uint32_t lbase)
{
    // lbase = (lane & 31) * 4 | (K >> 1) << 16 ; byte K of x goes to address byte 1
    constexpr uint32_t sel = 0x0c020000u | ((4u + (3 - K)) << 8);   // K: which table; byte (3-K) of x
    const uint32_t a = __builtin_amdgcn_perm(x, lbase, sel);
    return *reinterpret_cast<const uint32_t *>(lds + a + ((K & 1) << 7));
}

// word step: s' = T3[x.b0] ^ T2[x.b1] ^ T1[x.b2] ^ T0[x.b3]
__device__ __forceinline__ uint32_t word_step_p(const char *lds, uint32_t lb0, uint32_t lb1,
                                                uint32_t s, uint32_t w)
{
    const uint32_t x = s ^ w;
    return tlp<3>(lds, x, lb1) ^ tlp<2>(lds, x, lb1) ^ tlp<1>(lds, x, lb0) ^ tlp<0>(lds, x, lb0);
}

// replicated shift table: same layout as one slice table, at kShiftOff
__device__ __forceinline__ uint32_t shift_rep(const char *lds, uint32_t lb, uint32_t s)
{
    const char *t = lds + kShiftOff;
    // 32 KiB holds 256 entries x 32 replicas of ONE combined table indexed by a
    // single byte; a 4-byte shift needs 4 tables, so use 8 replicas x 4 tables:
    // addr = k*8192 + b*32 + (lane&7)*4   (8-way replicated, 2-way conflicts)
    const uint32_t r = (lb >> 2) & 7u;
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t b = (s >> (8 * k)) & 0xffu;
        v ^= *reinterpret_cast<const uint32_t *>(t + k * 8192 + b * 32 + r * 4);
    }
    return v;
}

template <int MODE>
__global__ void __launch_bounds__(kThreads, 1)
probe(const uint8_t *__restrict__ base, uint64_t total, const uint32_t *__restrict__ slice,
      const uint32_t *__restrict__ shift, uint32_t *__restrict__ out)
{
    __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];
    const uint32_t tid = threadIdx.x;
    {
        const uint32_t k = tid >> 8, b = tid & 255u;
        const uint32_t v = slice[tid];
        uint4 *dst = reinterpret_cast<uint4 *>(lds + ((k >> 1) << 16) + (b << 8) + ((k & 1u) << 7));
        for (int q = 0; q < 8; ++q) dst[q] = make_uint4(v, v, v, v);
        const uint32_t sv = shift[tid];     // [k][b]
        uint4 *sd = reinterpret_cast<uint4 *>(lds + kShiftOff + k * 8192 + b * 32);
        sd[0] = make_uint4(sv, sv, sv, sv);
        sd[1] = make_uint4(sv, sv, sv, sv);
    }
    __syncthreads();
    const uint32_t W = gridDim.x * (kThreads / 64);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (kThreads / 64) + (tid >> 6));
    const uint32_t lane = tid & 63u;
    const uint32_t lb = (lane & 31u) << 2;
    const uint32_t lb0 = lb, lb1 = lb | 0x10000u;
    const uint64_t S = total / kStep;
    const uint64_t g0 = (uint64_t) wave * S / W, g1 = (uint64_t) (wave + 1) * S / W;
    uint32_t s = 0, s1 = 0, s2 = 0, s3 = 0;
    const uint8_t *p = base + g0 * kStep;
    for (uint64_t g = g0; g < g1; ++g, p += kStep) {
        u32x4 a, b, c, d;
        if (MODE == 0 || MODE == 1 || MODE == 3 || MODE == 10) {
            const uint8_t *q = p + lane * 64;
            a = ld<MODE == 0>(q); b = ld<MODE == 0>(q + 16); c = ld<MODE == 0>(q + 32); d = ld<MODE == 0>(q + 48);
        } else if (MODE == 4 || MODE == 5 || MODE == 6 || MODE == 7 || MODE == 8) {
            const uint8_t *q = p + lane * 16;
            constexpr bool nt = MODE == 6 || MODE == 7 || MODE == 8;
            a = ld<nt>(q); b = ld<nt>(q + 1024); c = ld<nt>(q + 2048); d = ld<nt>(q + 3072);
        } else if (MODE == 11) {
            const uint8_t *q = p + lane * 32;
            a = ld<true>(q); b = ld<true>(q + 16); c = ld<true>(q + 2048); d = ld<true>(q + 2048 + 16);
        } else {
            const uint32_t x = (uint32_t) g * 0x9E3779B9u + lane;   // modes 2, 9
            a = u32x4{x, x ^ 1, x ^ 2, x ^ 3}; b = a + 7u; c = a * 3u; d = a ^ 0x5555u;
        }
        if (MODE == 3 || MODE == 4 || MODE == 6 || MODE == 11) {
            s ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
        } else if (MODE == 8 || MODE == 9) {
            s = shift_rep(lds, lb, s);   s1 = shift_rep(lds, lb, s1);
            s2 = shift_rep(lds, lb, s2); s3 = shift_rep(lds, lb, s3);
            s = word_step_p(lds, lb0, lb1, s, a.x);  s1 = word_step_p(lds, lb0, lb1, s1, b.x);
            s2 = word_step_p(lds, lb0, lb1, s2, c.x); s3 = word_step_p(lds, lb0, lb1, s3, d.x);
            s = word_step_p(lds, lb0, lb1, s, a.y);  s1 = word_step_p(lds, lb0, lb1, s1, b.y);
            s2 = word_step_p(lds, lb0, lb1, s2, c.y); s3 = word_step_p(lds, lb0, lb1, s3, d.y);
            s = word_step_p(lds, lb0, lb1, s, a.z);  s1 = word_step_p(lds, lb0, lb1, s1, b.z);
            s2 = word_step_p(lds, lb0, lb1, s2, c.z); s3 = word_step_p(lds, lb0, lb1, s3, d.z);
            s = word_step_p(lds, lb0, lb1, s, a.w);  s1 = word_step_p(lds, lb0, lb1, s1, b.w);
            s2 = word_step_p(lds, lb0, lb1, s2, c.w); s3 = word_step_p(lds, lb0, lb1, s3, d.w);
        } else if (MODE == 10) {
            s = shift_rep(lds, lb, s);
            s = word_step_p(lds, lb0, lb1, s, a.x); s = word_step_p(lds, lb0, lb1, s, a.y);
            s = word_step_p(lds, lb0, lb1, s, a.z); s = word_step_p(lds, lb0, lb1, s, a.w);
            s = word_step_p(lds, lb0, lb1, s, b.x); s = word_step_p(lds, lb0, lb1, s, b.y);
            s = word_step_p(lds, lb0, lb1, s, b.z); s = word_step_p(lds, lb0, lb1, s, b.w);
            s = word_step_p(lds, lb0, lb1, s, c.x); s = word_step_p(lds, lb0, lb1, s, c.y);
            s = word_step_p(lds, lb0, lb1, s, c.z); s = word_step_p(lds, lb0, lb1, s, c.w);
            s = word_step_p(lds, lb0, lb1, s, d.x); s = word_step_p(lds, lb0, lb1, s, d.y);
            s = word_step_p(lds, lb0, lb1, s, d.z); s = word_step_p(lds, lb0, lb1, s, d.w);
        } else if (MODE == 5 || MODE == 7) {
            s = shift_rep(lds, lb, s);   s1 = shift_rep(lds, lb, s1);
            s2 = shift_rep(lds, lb, s2); s3 = shift_rep(lds, lb, s3);
            s = word_step(lds, lb, s, a.x);  s1 = word_step(lds, lb, s1, b.x);
            s2 = word_step(lds, lb, s2, c.x); s3 = word_step(lds, lb, s3, d.x);
            s = word_step(lds, lb, s, a.y);  s1 = word_step(lds, lb, s1, b.y);
            s2 = word_step(lds, lb, s2, c.y); s3 = word_step(lds, lb, s3, d.y);
            s = word_step(lds, lb, s, a.z);  s1 = word_step(lds, lb, s1, b.z);
            s2 = word_step(lds, lb, s2, c.z); s3 = word_step(lds, lb, s3, d.z);
            s = word_step(lds, lb, s, a.w);  s1 = word_step(lds, lb, s1, b.w);
            s2 = word_step(lds, lb, s2, c.w); s3 = word_step(lds, lb, s3, d.w);
        } else {
            s = shift_rep(lds, lb, s);
            s = word_step(lds, lb, s, a.x); s = word_step(lds, lb, s, a.y);
            s = word_step(lds, lb, s, a.z); s = word_step(lds, lb, s, a.w);
            s = word_step(lds, lb, s, b.x); s = word_step(lds, lb, s, b.y);
            s = word_step(lds, lb, s, b.z); s = word_step(lds, lb, s, b.w);
            s = word_step(lds, lb, s, c.x); s = word_step(lds, lb, s, c.y);
            s = word_step(lds, lb, s, c.z); s = word_step(lds, lb, s, c.w);
            s = word_step(lds, lb, s, d.x); s = word_step(lds, lb, s, d.y);
            s = word_step(lds, lb, s, d.z); s = word_step(lds, lb, s, d.w);
        }
    }
    out[blockIdx.x * kThreads + tid] = s ^ s1 ^ s2 ^ s3;
}

typedef void (*Kern)(const uint8_t *, uint64_t, const uint32_t *, const uint32_t *, uint32_t *);

int main(int argc, char **argv)
{
    const uint64_t total = 1024ull * 409600;   // cfg2 bytes per launch
    const int nrot = 4, iters = 20;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int grid = prop.multiProcessorCount;
    std::vector<uint8_t *> bufs(nrot);
    for (auto &b : bufs) {
        CK(hipMalloc(&b, total));
        std::vector<uint32_t> r(total / 4);
        uint64_t z = 0x12345678ull + (uint64_t) (&b - &bufs[0]);
        for (auto &v : r) { z = z * 6364136223846793005ull + 1442695040888963407ull; v = (uint32_t) (z >> 32); }
        CK(hipMemcpy(b, r.data(), total, hipMemcpyHostToDevice));
    }
    std::vector<uint32_t> tab(1024);
    for (uint32_t i = 0; i < 1024; i++) tab[i] = i * 2654435761u ^ (i << 7);
    uint32_t *slice, *shift, *out;
    CK(hipMalloc(&slice, 4096)); CK(hipMalloc(&shift, 4096)); CK(hipMalloc(&out, grid * kThreads * 4));
    CK(hipMemcpy(slice, tab.data(), 4096, hipMemcpyHostToDevice));
    CK(hipMemcpy(shift, tab.data(), 4096, hipMemcpyHostToDevice));
    Kern ks[] = {probe<0>, probe<1>, probe<2>, probe<3>, probe<4>, probe<5>, probe<6>, probe<7>,
                 probe<8>, probe<9>, probe<10>, probe<11>};
    const char *names[] = {"strided64-nt+crc", "strided64+crc", "compute-only", "strided64 loads",
                           "coalesced loads", "coalesced+crc4", "coalesced-nt loads",
                           "coalesced-nt+crc4", "coalesced-nt+crc4perm", "compute-only crc4perm",
                           "strided64+crc perm", "strided32-nt loads"};
    const int NM = 12;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int round = 0; round < 2; round++) {
        for (int m = 0; m < NM; m++) {
            for (int w = 0; w < 3; w++) hipLaunchKernelGGL(ks[m], dim3(grid), dim3(kThreads), 0, 0, bufs[w % nrot], total, slice, shift, out);
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            for (int it = 0; it < iters; it++)
                hipLaunchKernelGGL(ks[m], dim3(grid), dim3(kThreads), 0, 0, bufs[it % nrot], total, slice, shift, out);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / iters;
            std::vector<uint32_t> h(grid * kThreads);
            CK(hipMemcpy(h.data(), out, h.size() * 4, hipMemcpyDeviceToHost));
            uint32_t x = 0;
            for (uint32_t v : h) x ^= v;
            printf("round %d mode %2d %-24s %8.2f us/launch %8.1f GB/s  xor=%08x\n", round, m, names[m], us,
                   total / (us * 1e-6) / 1e9, x);
        }
    }
    return 0;
}
