// wave_place_probe.hip -- where the dispatcher puts a small grid's waves.
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/probe/wave_place_probe tools/probe/wave_place_probe.hip
//   tools/probe/wave_place_probe
//
// The SHA-1 kernel runs one latency-bound round wave per workgroup, so its
// speed depends on that wave having a SIMD (and a CU's LDS) to itself.  This
// launches grids shaped like its variants (threads, LDS bytes, workgroups),
// keeps every wave resident for ~200 us, and prints for each workgroup the
// XCC / SE / CU / SIMD of each of its waves (HW_ID and XCC_ID registers).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <map>
#include <set>
#include <tuple>
#include <vector>

__global__ void place_kernel(uint32_t *out, uint32_t waves_per_wg)
{
    extern __shared__ uint32_t lds[];
    const uint32_t w = threadIdx.x >> 6;
    if ((threadIdx.x & 63u) == 0) {
        // HW_ID (id 4, all 32 bits) and XCC_ID (id 20, all 32 bits)
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
        const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 20);
        lds[w] = hw;
        out[(blockIdx.x * waves_per_wg + w) * 2 + 0] = hw;
        out[(blockIdx.x * waves_per_wg + w) * 2 + 1] = xcc;
    }
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < 20000) {   // 100 MHz: 200 us
        __builtin_amdgcn_s_sleep(10);
    }
}

int main()
{
    struct Cfg {
        const char *name;
        uint32_t threads, lds, wgs;
    };
    const Cfg cfgs[] = {
        {"c64s2 (192 thr, 160 KiB, 16 WG)", 192, 163840, 16},
        {"c32s1 (128 thr, 80 KiB, 32 WG)", 128, 81920, 32},
        {"c32s1g8 (128 thr, 160 KiB, 32 WG)", 128, 163840, 32},
        {"c32s2 (192 thr, 80 KiB, 32 WG)", 192, 81920, 32},
        {"c16s1 (128 thr, 40 KiB, 64 WG)", 128, 40960, 64},
        {"c64s2 x4 (192 thr, 160 KiB, 64 WG)", 192, 163840, 64},
    };
    for (const Cfg &c : cfgs) {
        const uint32_t wpw = c.threads / 64;
        uint32_t *d = nullptr;
        const size_t n = (size_t) c.wgs * wpw * 2;
        if (hipMalloc(&d, n * 4) != hipSuccess) {
            return 1;
        }
        hipFuncSetAttribute((const void *) place_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
        hipLaunchKernelGGL(place_kernel, dim3(c.wgs), dim3(c.threads), c.lds, 0, d, wpw);
        if (hipDeviceSynchronize() != hipSuccess) {
            printf("%s: launch failed\n", c.name);
            return 1;
        }
        std::vector<uint32_t> h(n);
        hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost);
        hipFree(d);
        std::map<std::tuple<int, int, int, int>, int> cu_wgs;      // (xcc, se, sh, cu) -> WGs
        std::map<std::tuple<int, int, int, int, int>, int> simd_waves;
        int shared_simd_in_wg = 0;
        printf("== %s\n", c.name);
        for (uint32_t g = 0; g < c.wgs; ++g) {
            std::set<int> simds;
            printf("  wg %2u:", g);
            std::tuple<int, int, int, int> cu0;
            for (uint32_t w = 0; w < wpw; ++w) {
                const uint32_t hw = h[(g * wpw + w) * 2], xcc = h[(g * wpw + w) * 2 + 1] & 0xf;
                const int simd = (hw >> 4) & 3, cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
                printf(" [x%u se%d sh%d cu%2d simd%d]", xcc, se, sh, cu, simd);
                simds.insert(simd);
                cu0 = std::make_tuple((int) xcc, se, sh, cu);
                simd_waves[std::make_tuple((int) xcc, se, sh, cu, simd)]++;
            }
            printf("\n");
            cu_wgs[cu0]++;
            shared_simd_in_wg += simds.size() < wpw;
        }
        int multi = 0, maxw = 0;
        for (auto &kv : cu_wgs) {
            multi += kv.second > 1;
        }
        for (auto &kv : simd_waves) {
            maxw = kv.second > maxw ? kv.second : maxw;
        }
        printf("  -> %zu CUs used, %d CUs with >1 WG, %d WGs with two waves on one SIMD, max waves on one SIMD %d\n",
               cu_wgs.size(), multi, shared_simd_in_wg, maxw);
    }
    return 0;
}
