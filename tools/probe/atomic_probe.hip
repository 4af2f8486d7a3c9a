// atomic_probe.hip -- cost model of the atomics a dynamic work queue would use.
//
// Standalone.  256 workgroups x 1024 threads (one per CU, like the CRC
// kernel); lane 0 of every wave performs K agent-scope fetch_adds, each
// dependent on the previous result, on an address chosen by the mode:
//   0 one address for all 4096 waves
//   1 one address per XCD (blockIdx % 8)
//   2 one address per workgroup
//   3 one address per wave (no contention: latency only)
//   4 LDS atomic on one per-workgroup LDS word (workgroup-local queue)
// Prints the kernel time and the time per atomic per wave.
// Build: hipcc -O3 --offload-arch=gfx950 -o atomic_probe atomic_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

template <int MODE>
__global__ void __launch_bounds__(1024, 1) probe(uint32_t *ctr, uint32_t K, uint32_t *sink)
{
    __shared__ uint32_t lq;
    if (threadIdx.x == 0) {
        lq = 0;
    }
    __syncthreads();
    const uint32_t wave = blockIdx.x * 16 + (threadIdx.x >> 6);
    uint32_t *a;
    switch (MODE) {
    case 0: a = ctr; break;
    case 1: a = ctr + 64 * (blockIdx.x & 7); break;
    case 2: a = ctr + 64 * blockIdx.x; break;
    default: a = ctr + 64 * wave; break;
    }
    uint32_t acc = 0;
    if ((threadIdx.x & 63) == 0) {
        for (uint32_t k = 0; k < K; ++k) {
            uint32_t v;
            if (MODE == 4) {
                v = __hip_atomic_fetch_add(&lq, 1u + (acc & 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else {
                v = __hip_atomic_fetch_add(a + (acc & 0), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            acc += v;
        }
        sink[wave] = acc;
    }
}

template <int MODE>
static float run(uint32_t *ctr, uint32_t K, uint32_t *sink)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CK(hipMemset(ctr, 0, 64 * 4096 * sizeof(uint32_t)));
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(probe<MODE>, dim3(256), dim3(1024), 0, 0, ctr, K, sink);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    return best;
}

int main()
{
    uint32_t *ctr, *sink;
    CK(hipMalloc(&ctr, 64 * 4096 * sizeof(uint32_t)));
    CK(hipMalloc(&sink, 4096 * sizeof(uint32_t)));
    const char *names[] = {"one address", "per-XCD address", "per-WG address", "per-wave address",
                           "LDS per-WG"};
    for (uint32_t K : {1u, 4u, 16u}) {
        float t[5] = {run<0>(ctr, K, sink), run<1>(ctr, K, sink), run<2>(ctr, K, sink),
                      run<3>(ctr, K, sink), run<4>(ctr, K, sink)};
        for (int m = 0; m < 5; ++m) {
            printf("K=%2u %-18s kernel %9.2f us  per atomic per wave %8.1f ns  (4096 waves)\n", K,
                   names[m], t[m] * 1e3, t[m] * 1e6 / K);
        }
    }
    return 0;
}
