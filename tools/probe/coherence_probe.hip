// coherence_probe.hip -- do the CRC kernel's cross-wave protocols hold across
// XCDs?  Standalone; 256 workgroups x 1024 threads (one per CU).
//
//  test 1 (accumulate): wave w XORs v(w) into acc[w % NC] and counts into
//          cnt[w % NC]; the arrival completing the count (64 per chunk, from
//          workgroups on different XCDs) reads acc and writes out.
//          mode 0: fetch_xor relaxed + fetch_add acq_rel (the kernel's form)
//          mode 1: fetch_xor relaxed + s_waitcnt + fetch_add relaxed
//          mode 2: returning fetch_xor + fetch_add acq_rel
//  test 2 (claims): every wave owns K units and claims them from the front
//          (+1) while the waves of its 64-wave group steal halves from the
//          back (+n << 28) of 64-bit words; every unit bumps done[] once.
//
// Build: hipcc -O3 --offload-arch=gfx950 -o coherence_probe coherence_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

constexpr uint32_t NC = 64;

__device__ __host__ inline uint32_t hv(uint32_t w, uint32_t it)
{
    uint32_t x = w * 0x9E3779B9u + it * 0x85EBCA6Bu + 1u;
    x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
    return x;
}

template <int MODE>
__global__ void __launch_bounds__(1024, 1) acc_probe(uint32_t *acc, uint32_t *cnt, uint32_t *out, uint32_t it,
                                                   uint32_t per)
{
    const uint32_t w = blockIdx.x * 16 + (threadIdx.x >> 6);
    if ((threadIdx.x & 63) != 0) {
        return;
    }
    const uint32_t c = w % NC;
    const uint32_t v = hv(w, it);
    uint32_t old;
    if (MODE == 0) {
        __hip_atomic_fetch_xor(&acc[c], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        old = __hip_atomic_fetch_add(&cnt[c], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    } else if (MODE == 1) {
        __hip_atomic_fetch_xor(&acc[c], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        old = __hip_atomic_fetch_add(&cnt[c], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        const uint32_t x = __hip_atomic_fetch_xor(&acc[c], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        old = __hip_atomic_fetch_add(&cnt[c], 1u + (x & 0u), __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (old + 1 == per) {
        out[c] = __hip_atomic_load(&acc[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&acc[c], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&cnt[c], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ void __launch_bounds__(1024, 1) claim_probe(unsigned long long *words, uint32_t *done, uint32_t K,
                                                     uint32_t gen, uint32_t W)
{
    const uint32_t w = blockIdx.x * 16 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    if (lane == 0) {
        __hip_atomic_store(&words[w], (unsigned long long) gen << 56, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // owner: claim from the front, with some work between claims
    for (uint32_t t = 0; t < K; ++t) {
        unsigned long long o = 0;
        if (lane == 0) {
            o = __hip_atomic_fetch_add(&words[w], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        o = __shfl(o, 0);
        const uint32_t hi = (uint32_t) ((o >> 28) & ((1u << 28) - 1));
        if (t + hi >= K) {
            break;
        }
        if (lane == 0) {
            atomicAdd(&done[(uint64_t) w * K + t], 1u);
        }
        for (uint32_t z = 0; z < 1 + (w * 7) % 4; ++z) { __builtin_amdgcn_s_sleep(20); }
    }
    // thief: steal halves of the largest remaining in the group
    const uint32_t grp = w & ~63u;
    for (;;) {
        const uint32_t cand = grp + lane;
        uint32_t lo = 0, hi = 0, rem = 0;
        if (cand < W) {
            const unsigned long long v = __hip_atomic_load(&words[cand], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            lo = (uint32_t) (v & ((1u << 28) - 1));
            hi = (uint32_t) ((v >> 28) & ((1u << 28) - 1));
            if ((uint32_t) (v >> 56) == gen && lo + hi < K) {
                rem = K - lo - hi;
            }
        }
        uint32_t key = (rem << 6) | lane;
        for (int o = 32; o >= 1; o >>= 1) {
            key = max(key, (uint32_t) __shfl_xor(key, o));
        }
        if ((key >> 6) == 0) {
            break;
        }
        const uint32_t bl = key & 63, v = grp + bl;
        const uint32_t n = ((key >> 6) + 1) / 2;
        unsigned long long o = 0;
        if (lane == 0) {
            o = __hip_atomic_fetch_add(&words[v], (unsigned long long) n << 28, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
        }
        o = __shfl(o, 0);
        const uint32_t lo_o = (uint32_t) (o & ((1u << 28) - 1));
        const uint32_t hi_o = (uint32_t) ((o >> 28) & ((1u << 28) - 1));
        if ((uint32_t) (o >> 56) != gen || lo_o + hi_o >= K) {
            continue;
        }
        const uint32_t tb = K - hi_o;
        const uint32_t ta = max(lo_o, tb - min(n, tb));
        for (uint32_t t = ta; t < tb; ++t) {
            if (lane == 0) {
                atomicAdd(&done[(uint64_t) v * K + t], 1u);
            }
            __builtin_amdgcn_s_sleep(20);
        }
    }
}

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 50;
    const uint32_t W = 256 * 16, per = W / NC;
    uint32_t *acc, *cnt, *out;
    CK(hipMalloc(&acc, NC * 4));
    CK(hipMalloc(&cnt, NC * 4));
    CK(hipMalloc(&out, NC * 4));
    CK(hipMemset(acc, 0, NC * 4));
    CK(hipMemset(cnt, 0, NC * 4));
    for (int mode = 0; mode < 3; ++mode) {
        int bad = 0;
        for (int it = 0; it < iters; ++it) {
            CK(hipMemset(out, 0, NC * 4));
            if (mode == 0) hipLaunchKernelGGL(acc_probe<0>, dim3(256), dim3(1024), 0, 0, acc, cnt, out, it, per);
            if (mode == 1) hipLaunchKernelGGL(acc_probe<1>, dim3(256), dim3(1024), 0, 0, acc, cnt, out, it, per);
            if (mode == 2) hipLaunchKernelGGL(acc_probe<2>, dim3(256), dim3(1024), 0, 0, acc, cnt, out, it, per);
            CK(hipDeviceSynchronize());
            std::vector<uint32_t> h(NC), want(NC, 0);
            CK(hipMemcpy(h.data(), out, NC * 4, hipMemcpyDeviceToHost));
            for (uint32_t w = 0; w < W; ++w) want[w % NC] ^= hv(w, it);
            for (uint32_t c = 0; c < NC; ++c) bad += h[c] != want[c];
        }
        printf("accumulate mode %d: %d bad of %d\n", mode, bad, iters * (int) NC);
    }
    for (uint32_t K : {8u, 16u, 64u}) {
        unsigned long long *words;
        uint32_t *done;
        CK(hipMalloc(&words, W * 8));
        CK(hipMemset(words, 0, W * 8));
        CK(hipMalloc(&done, (size_t) W * K * 4));
        int bad = 0;
        for (int it = 0; it < iters; ++it) {
            CK(hipMemset(done, 0, (size_t) W * K * 4));
            hipLaunchKernelGGL(claim_probe, dim3(256), dim3(1024), 0, 0, words, done, K, (uint32_t) (it % 255 + 1), W);
            CK(hipDeviceSynchronize());
            std::vector<uint32_t> h((size_t) W * K);
            CK(hipMemcpy(h.data(), done, h.size() * 4, hipMemcpyDeviceToHost));
            for (auto x : h) bad += x != 1;
        }
        printf("claims K=%u: %d units not done exactly once of %d\n", K, bad, iters * (int) (W * K));
        CK(hipFree(words));
        CK(hipFree(done));
    }
    return 0;
}
