// crc32_gpu.hip -- batched CRC-32 over independent chunk content buffers,
// hand-written for CDNA4 (gfx950, MI355X).  C ABI in
// include/chunkio_amd/cio_crc32_gpu.h.
//
// Reference behaviour reproduced (fluent/chunkio):
//   crc_update(state, buf, len)  deps/crc32/crc32.c:337-390 — CRC-32/IEEE,
//   reflected poly 0xEDB88320, raw (un-finalized) state in and out.  Each
//   chunk i of a batch yields crc_update(seed_i, base + off_i, len_i), i.e.
//   cio_file_calculate_checksum() (src/cio_file.c:66-94) over that chunk.
//
// Algorithm (see DESIGN.md for the derivation and the roofline):
//   The CRC is affine over GF(2):  crc(s, A||B) = shift(crc(s, A), |B|) ^
//   crc(0, B), shift(s, n) = s * x^(8n) mod P.  Every chunk is cut into
//   4 KiB wave-steps; step j of a chunk covers virtual bytes [4096 j, 4096 j
//   + 4096) where the virtual chunk is the content prefixed by its (off & 15)
//   misalignment bytes, which are zeroed (a zero-seeded CRC ignores leading
//   zeros) so every load is an aligned 16-byte global_load_dwordx4.  Lane l of
//   a wave owns the 64 contiguous bytes [64 l, 64 l + 64) of a step and runs
//   a slice-by-4 chain over them with lookup tables held in LDS, replicated
//   32 times so lane l always hits bank (l & 31): no data-dependent bank
//   conflicts.  Between two steps a lane's state jumps over the 4032 bytes of
//   the other 63 lanes (one 4-lookup shift table).  The seed is folded into
//   the first 4 content bytes.  At the end of a piece (the steps of one chunk
//   that one wave owns) each lane shifts its state to the piece end
//   (x^(8d) table + GF(2) multiply) and the wave XOR-reduces with __shfl_xor.
//   A small second kernel folds a chunk's pieces in order (Horner with
//   x^(8 bytes)) -> one raw CRC per chunk.
//
//   Work partition: the S wave-steps of the whole batch are split evenly over
//   the W persistent waves of the grid (one 1024-thread workgroup per CU), so
//   every wave streams the same number of bytes whatever the chunk sizes —
//   the load-balanced persistent kernel of BASELINE config 3.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <stdlib.h>
#include <mutex>
#include <vector>
#include <string>
#include <algorithm>

#include "crc32_host.h"
#include "chunkio_amd/cio_crc32_gpu.h"

namespace {

constexpr int kWave = 64;
constexpr int kBPL = 64;                    // bytes per lane per step
constexpr int kStep = kWave * kBPL;         // 4096 bytes per wave-step
constexpr int kThreads = 1024;              // one workgroup per CU
constexpr int kWavesPerWG = kThreads / kWave;
constexpr int kX8Count = 2 * kStep;         // x^(8m), m in [0, 8192)
constexpr uint32_t kSliceBytes = 131072;    // 4 tables x 256 x 32 replicas x 4 B
constexpr uint32_t kShiftWordOff = kSliceBytes / 4;
constexpr uint32_t kLdsWords = (kSliceBytes + 4096) / 4;

struct ChunkDesc {
    uint64_t a;        // aligned-down start offset from the batch base
    uint64_t vlen;     // virtual length = (off & 15) + len
    uint64_t g;        // first global wave-step of this chunk
    uint32_t nsteps;   // ceil(vlen / kStep); 0 for chunks handled by the finisher
    uint32_t h;        // off & 15 (zeroed head bytes)
};
static_assert(sizeof(ChunkDesc) == 32, "desc layout");

// ---------------------------------------------------------------- device math

__device__ __forceinline__ uint32_t multmodp(uint32_t a, uint32_t b)
{
    uint32_t p = 0;
#pragma unroll
    for (int i = 31; i >= 0; --i) {
        p ^= b & (0u - ((a >> i) & 1u));
        b = (b >> 1) ^ (CIOA_POLY & (0u - (b & 1u)));
    }
    return p;
}

__device__ __forceinline__ uint64_t wave_start(uint64_t w, uint64_t S, uint64_t W)
{
    return (w * S) / W;
}

__device__ __forceinline__ uint64_t wave_of_step(uint64_t g, uint64_t S, uint64_t W)
{
    return ((g + 1) * W + S - 1) / S - 1;
}

// Slice-table lookup in the replicated LDS image.
//   byte address(k, b, lane) = (k>>1)*65536 + b*256 + (k&1)*128 + (lane&31)*4
template <int K>
__device__ __forceinline__ uint32_t tl(const uint32_t *lds, uint32_t lb, uint32_t b)
{
    const char *p = reinterpret_cast<const char *>(lds) + ((K >> 1) << 16) + ((K & 1) << 7);
    return *reinterpret_cast<const uint32_t *>(p + ((b << 8) | lb));
}

// crc_update(s, 4 little-endian bytes of w)
__device__ __forceinline__ uint32_t word_step(const uint32_t *lds, uint32_t lb, uint32_t s, uint32_t w)
{
    const uint32_t x = s ^ w;
    return tl<3>(lds, lb, x & 0xffu) ^ tl<2>(lds, lb, (x >> 8) & 0xffu) ^
           tl<1>(lds, lb, (x >> 16) & 0xffu) ^ tl<0>(lds, lb, x >> 24);
}

__device__ __forceinline__ uint32_t byte_step(const uint32_t *lds, uint32_t lb, uint32_t s, uint32_t byte)
{
    return tl<0>(lds, lb, (s ^ byte) & 0xffu) ^ (s >> 8);
}

// shift(s, kStep - kBPL): jump over the other lanes' bytes of one step.
__device__ __forceinline__ uint32_t step_shift(const uint32_t *lds, uint32_t s)
{
    const uint32_t *sh = lds + kShiftWordOff;
    return sh[s & 0xffu] ^ sh[256 + ((s >> 8) & 0xffu)] ^
           sh[512 + ((s >> 16) & 0xffu)] ^ sh[768 + (s >> 24)];
}

__device__ __forceinline__ uint32_t block64(const uint32_t *lds, uint32_t lb, uint32_t s,
                                            const uint4 &v0, const uint4 &v1,
                                            const uint4 &v2, const uint4 &v3)
{
    s = word_step(lds, lb, s, v0.x); s = word_step(lds, lb, s, v0.y);
    s = word_step(lds, lb, s, v0.z); s = word_step(lds, lb, s, v0.w);
    s = word_step(lds, lb, s, v1.x); s = word_step(lds, lb, s, v1.y);
    s = word_step(lds, lb, s, v1.z); s = word_step(lds, lb, s, v1.w);
    s = word_step(lds, lb, s, v2.x); s = word_step(lds, lb, s, v2.y);
    s = word_step(lds, lb, s, v2.z); s = word_step(lds, lb, s, v2.w);
    s = word_step(lds, lb, s, v3.x); s = word_step(lds, lb, s, v3.y);
    s = word_step(lds, lb, s, v3.z); s = word_step(lds, lb, s, v3.w);
    return s;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 ldg16(const uint8_t *p)
{
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

// Generic step: partial blocks, first step of a chunk (head zeroing + seed fold).
__device__ __forceinline__ void slow_step(const uint32_t *lds, uint32_t lb, const uint8_t *cbase,
                                       uint64_t jj, uint64_t vlen, uint32_t h, uint32_t seed,
                                       uint32_t lane, uint32_t &s, uint64_t &lane_end)
{
    const uint64_t bstart = jj * kStep + (uint64_t) lane * kBPL;
    const uint32_t vb = bstart >= vlen ? 0u : (uint32_t) min(vlen - bstart, (uint64_t) kBPL);
    if (vb == 0) {
        return;
    }
    uint32_t w[16];
    const uint8_t *p = cbase + bstart;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if ((uint32_t) (q * 16) < vb) {
            v = *reinterpret_cast<const uint4 *>(p + q * 16);
        }
        w[4 * q + 0] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
    }
    if (jj == 0 && lane == 0) {
        // Zero the alignment head [0, h) and fold the seed into bytes [h, h+4).
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const int off = 4 * i - (int) h;
            if (off <= -4) {
                w[i] = 0u;
            } else if (off < 0) {
                w[i] = (w[i] & (~0u << (8 * -off))) ^ (seed << (8 * -off));
            } else if (off == 0) {
                w[i] ^= seed;
            } else if (off < 4) {
                w[i] ^= seed >> (8 * off);
            }
        }
    }
    s = step_shift(lds, s);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        if ((uint32_t) (4 * i + 4) <= vb) {
            s = word_step(lds, lb, s, w[i]);
        } else if ((uint32_t) (4 * i) < vb) {
            for (uint32_t t = 4 * i; t < vb; ++t) {
                s = byte_step(lds, lb, s, (w[i] >> (8 * (t - 4 * i))) & 0xffu);
            }
        }
    }
    lane_end = bstart + vb;
}

__global__ void __launch_bounds__(kThreads, 1)
crc32_piece_kernel(const uint8_t *__restrict__ base, const ChunkDesc *__restrict__ desc,
                   const uint32_t *__restrict__ wave_chunk0, const uint32_t *__restrict__ seeds,
                   uint32_t *__restrict__ partials, const uint32_t *__restrict__ g_slice,
                   const uint32_t *__restrict__ g_shift, const uint32_t *__restrict__ g_x8,
                   const uint32_t *__restrict__ cid, uint64_t S, uint32_t W, uint32_t n)
{
    __shared__ __attribute__((aligned(16))) uint32_t lds[kLdsWords];
    const uint32_t tid = threadIdx.x;

    {   // Build the replicated slice tables and the step-shift table.
        const uint32_t k = tid >> 8, b = tid & 255u;
        const uint32_t v = g_slice[tid];
        const uint4 v4 = make_uint4(v, v, v, v);
        uint4 *dst = reinterpret_cast<uint4 *>(reinterpret_cast<char *>(lds) +
                                               ((k >> 1) << 16) + (b << 8) + ((k & 1u) << 7));
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            dst[q] = v4;
        }
        lds[kShiftWordOff + tid] = g_shift[tid];
    }
    __syncthreads();

    const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * kWavesPerWG + (tid >> 6));
    const uint32_t lane = tid & 63u;
    const uint32_t lb = (lane & 31u) << 2;

    uint64_t g = wave_start(wave, S, W);
    const uint64_t gend = wave_start((uint64_t) wave + 1, S, W);
    if (g >= gend) {
        return;
    }
    uint32_t c = wave_chunk0[wave];
    ChunkDesc d = desc[c];
    uint64_t j = g - d.g;

    for (;;) {
        const uint64_t jend = min((uint64_t) d.nsteps, j + (gend - g));
        const uint64_t full_end = d.vlen / kStep;
        const uint8_t *cbase = base + d.a;
        const uint32_t seed = (j == 0) ? (seeds ? seeds[cid ? cid[c] : c] : 0xffffffffu) : 0u;
        uint32_t s = 0;
        uint64_t lane_end = 0;
        uint64_t jj = j;

        if (jj == 0) {
            slow_step(lds, lb, cbase, 0, d.vlen, d.h, seed, lane, s, lane_end);
            jj = 1;
        }
        const uint64_t fe = min(jend, full_end);
        if (jj < fe) {
            const uint8_t *lp = cbase + jj * kStep + lane * kBPL;
            uint4 c0 = ldg16(lp), c1 = ldg16(lp + 16), c2 = ldg16(lp + 32), c3 = ldg16(lp + 48);
            for (; jj < fe; ++jj) {
                uint4 n0 = c0, n1 = c1, n2 = c2, n3 = c3;
                if (jj + 1 < fe) {
                    lp += kStep;
                    n0 = ldg16(lp); n1 = ldg16(lp + 16); n2 = ldg16(lp + 32); n3 = ldg16(lp + 48);
                }
                s = step_shift(lds, s);
                s = block64(lds, lb, s, c0, c1, c2, c3);
                c0 = n0; c1 = n1; c2 = n2; c3 = n3;
            }
            lane_end = (fe - 1) * kStep + (uint64_t) (lane + 1) * kBPL;
        }
        if (jj < jend) {
            slow_step(lds, lb, cbase, jj, d.vlen, d.h, 0u, lane, s, lane_end);
        }

        // Shift every lane's state to the piece end, XOR-reduce over the wave.
        const uint64_t pend = min(jend * kStep, d.vlen);
        const uint64_t dist = lane_end < pend ? pend - lane_end : 0;
        uint32_t contrib = s ? multmodp(g_x8[min(dist, (uint64_t) (kX8Count - 1))], s) : 0u;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            contrib ^= __shfl_xor(contrib, o);
        }
        if (lane == 0) {
            partials[(uint64_t) wave + c] = contrib;
        }

        g += jend - j;
        if (g >= gend) {
            break;
        }
        do {
            if (++c >= n) {
                return;     // unreachable for a consistent plan; never read past desc[n-1]
            }
            d = desc[c];
        } while (d.nsteps == 0);
        j = 0;
    }
}

__device__ __forceinline__ uint32_t xpow8_bytes(uint64_t bytes, const uint32_t *x8, const uint32_t *x4k)
{
    const uint64_t m = bytes / kStep;
    const uint32_t r = (uint32_t) (bytes % kStep);
    return m == 0 ? x8[r] : multmodp(x4k[m], x8[r]);
}

__global__ void __launch_bounds__(256)
crc32_finish_kernel(const uint8_t *__restrict__ base, const ChunkDesc *__restrict__ desc,
                    const uint32_t *seeds, const uint32_t *__restrict__ partials,
                    uint32_t *out, const uint32_t *__restrict__ g_byte,
                    const uint32_t *__restrict__ g_x8, const uint32_t *__restrict__ g_x4k,
                    const uint32_t *__restrict__ cid, uint64_t S, uint32_t W, uint32_t n)
{
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) {
        return;
    }
    const uint32_t oc = cid ? cid[c] : c;   // output / seed slot
    const ChunkDesc d = desc[c];
    if (d.nsteps == 0) {
        // Tiny (len < 4) or empty chunk: byte-serial with the seed directly.
        uint32_t s = seeds ? seeds[oc] : 0xffffffffu;
        const uint8_t *p = base + d.a + d.h;
        const uint32_t len = (uint32_t) (d.vlen - d.h);
        for (uint32_t i = 0; i < len; ++i) {
            s = g_byte[(s ^ p[i]) & 0xffu] ^ (s >> 8);
        }
        out[oc] = s;
        return;
    }
    const uint64_t w0 = wave_of_step(d.g, S, W);
    const uint64_t w1 = wave_of_step(d.g + d.nsteps - 1, S, W);
    uint32_t acc = partials[w0 + c];
    for (uint64_t w = w0 + 1; w <= w1; ++w) {
        const uint64_t st = wave_start(w, S, W);
        const uint64_t en = wave_start(w + 1, S, W);
        if (st == en) {
            continue;   // empty wave (S < W)
        }
        const uint64_t ps = st - d.g;
        const uint64_t pe = min(en - d.g, (uint64_t) d.nsteps);
        const uint64_t bytes = (w == w1) ? d.vlen - ps * kStep : (pe - ps) * kStep;
        acc = multmodp(xpow8_bytes(bytes, g_x8, g_x4k), acc) ^ partials[w + c];
    }
    out[oc] = acc;
}

// ---------------------------------------------------------------- synthetic fill

__device__ __forceinline__ uint64_t splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void __launch_bounds__(256)
fill_kernel(uint8_t *__restrict__ base, const uint64_t *__restrict__ offs,
            const uint64_t *__restrict__ lens, const uint64_t *__restrict__ ids, uint64_t seed,
            uint32_t n)
{
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        const uint64_t off = offs[i], len = lens[i];
        if (len == 0) {
            continue;
        }
        const uint64_t id = ids ? ids[i] : (uint64_t) i;
        const uint64_t key = seed ^ (0x9E3779B97F4A7C15ull * (id + 1));
        const uint64_t first = off & ~15ull;
        const uint64_t ngran = ((off + len + 15) & ~15ull) - first;
        for (uint64_t gi = threadIdx.x; gi < ngran / 16; gi += blockDim.x) {
            const uint64_t gaddr = first + gi * 16;
            const int64_t t0 = (int64_t) gaddr - (int64_t) off;  // chunk-relative byte of granule start
            if (t0 >= 0 && (uint64_t) t0 + 16 <= len) {
                const uint64_t k0 = (uint64_t) t0 >> 3;
                const uint32_t sh = (uint32_t) (t0 & 7) * 8;
                const uint64_t w0 = splitmix64(key + k0), w1 = splitmix64(key + k0 + 1);
                uint64_t lo, hi;
                if (sh == 0) {
                    lo = w0; hi = w1;
                } else {
                    const uint64_t w2 = splitmix64(key + k0 + 2);
                    lo = (w0 >> sh) | (w1 << (64 - sh));
                    hi = (w1 >> sh) | (w2 << (64 - sh));
                }
                *reinterpret_cast<uint4 *>(base + gaddr) =
                    make_uint4((uint32_t) lo, (uint32_t) (lo >> 32), (uint32_t) hi, (uint32_t) (hi >> 32));
            } else {
                for (int b = 0; b < 16; ++b) {
                    const int64_t t = t0 + b;
                    if (t >= 0 && (uint64_t) t < len) {
                        const uint64_t w = splitmix64(key + ((uint64_t) t >> 3));
                        base[gaddr + b] = (uint8_t) (w >> (8 * (t & 7)));
                    }
                }
            }
        }
    }
}

// ---------------------------------------------------------------- host side

thread_local std::string g_err;

int fail(const char *what, hipError_t e = hipSuccess)
{
    char buf[512];
    if (e != hipSuccess) {
        snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(e));
    } else {
        snprintf(buf, sizeof(buf), "%s", what);
    }
    g_err = buf;
    return CIO_ERROR;
}

}  // namespace

extern "C" int cioa_fail_msg(const char *what, const char *detail)
{
    g_err = std::string(what) + (detail ? std::string(": ") + detail : std::string());
    return CIO_ERROR;
}

namespace {

#define HIP_TRY(expr, what)                         \
    do {                                            \
        hipError_t e_ = (expr);                     \
        if (e_ != hipSuccess) return fail(what, e_); \
    } while (0)

struct DeviceState {
    bool ready = false;
    int cus = 0;
    uint32_t *slice = nullptr;   // [4][256] compact
    uint32_t *shift = nullptr;   // [4][256] shift by kStep - kBPL
    uint32_t *x8 = nullptr;      // [kX8Count]
};

std::mutex g_mu;
std::vector<DeviceState> g_dev;

int device_state(DeviceState **out)
{
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev), "hipGetDevice");
    std::lock_guard<std::mutex> lk(g_mu);
    if ((int) g_dev.size() <= dev) {
        g_dev.resize(dev + 1);
    }
    DeviceState &st = g_dev[dev];
    if (!st.ready) {
        hipDeviceProp_t prop;
        HIP_TRY(hipGetDeviceProperties(&prop, dev), "hipGetDeviceProperties");
        if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
            char msg[256];
            snprintf(msg, sizeof(msg), "chunkio_amd kernels are built for gfx950, device is %s",
                     prop.gcnArchName);
            return fail(msg);
        }
        st.cus = prop.multiProcessorCount;
        static uint32_t slice[4][256], shift[4][256];
        std::vector<uint32_t> x8(kX8Count);
        cioa_gen_slice4(slice);
        cioa_gen_shift_table(shift, (uint64_t) (kStep - kBPL));
        cioa_gen_xpow8_table(x8.data(), kX8Count, 1);
        HIP_TRY(hipMalloc(&st.slice, sizeof(slice)), "hipMalloc(slice)");
        HIP_TRY(hipMalloc(&st.shift, sizeof(shift)), "hipMalloc(shift)");
        HIP_TRY(hipMalloc(&st.x8, kX8Count * sizeof(uint32_t)), "hipMalloc(x8)");
        HIP_TRY(hipMemcpy(st.slice, slice, sizeof(slice), hipMemcpyHostToDevice), "upload slice");
        HIP_TRY(hipMemcpy(st.shift, shift, sizeof(shift), hipMemcpyHostToDevice), "upload shift");
        HIP_TRY(hipMemcpy(st.x8, x8.data(), kX8Count * sizeof(uint32_t), hipMemcpyHostToDevice),
                "upload x8");
        st.ready = true;
    }
    *out = &st;
    return CIO_OK;
}

}  // namespace

struct cio_crc32_plan {
    int device = 0;
    uint32_t n = 0;
    uint64_t S = 0;            // total wave-steps
    uint32_t W = 0;            // waves in the grid
    uint32_t grid = 0;         // workgroups
    uint64_t bytes = 0;        // sum of lens
    ChunkDesc *desc = nullptr;
    uint32_t *wave_chunk0 = nullptr;
    uint32_t *partials = nullptr;
    uint32_t *x4k = nullptr;
    DeviceState *st = nullptr;
};

extern "C" {

const char *cio_gpu_last_error(void)
{
    return g_err.c_str();
}

const char *cio_gpu_version(void)
{
    return "chunkio_amd crc32 v1 gfx950 lane64B-step4K slice4-lds32x";
}

int cio_gpu_init(void)
{
    DeviceState *st;
    return device_state(&st);
}

void cio_crc32_plan_destroy(cio_crc32_plan *p)
{
    if (!p) {
        return;
    }
    (void) hipFree(p->desc);
    (void) hipFree(p->wave_chunk0);
    (void) hipFree(p->partials);
    (void) hipFree(p->x4k);
    delete p;
}

int cio_crc32_plan_create(cio_crc32_plan **out, const uint64_t *offs, const uint64_t *lens, size_t n)
{
    if (!out || (n && (!offs || !lens))) {
        return fail("cio_crc32_plan_create: null argument");
    }
    if (n >= 0xffffffffull) {
        return fail("cio_crc32_plan_create: too many chunks");
    }
    *out = nullptr;
    DeviceState *st;
    if (device_state(&st) != CIO_OK) {
        return CIO_ERROR;
    }
    cio_crc32_plan *p = new cio_crc32_plan();
    p->st = st;
    p->n = (uint32_t) n;
    p->grid = (uint32_t) st->cus;
    p->W = p->grid * kWavesPerWG;

    std::vector<ChunkDesc> desc(n ? n : 1);
    uint64_t S = 0, bytes = 0, max_steps = 0;
    for (size_t i = 0; i < n; i++) {
        ChunkDesc &d = desc[i];
        d.a = offs[i] & ~15ull;
        d.h = (uint32_t) (offs[i] & 15u);
        d.vlen = d.h + lens[i];
        d.g = S;
        const uint64_t ns = lens[i] >= 4 ? (d.vlen + kStep - 1) / kStep : 0;
        if (ns > 0xffffffffull) {
            delete p;
            return fail("cio_crc32_plan_create: chunk too large");
        }
        d.nsteps = (uint32_t) ns;
        S += ns;
        bytes += lens[i];
        max_steps = std::max(max_steps, ns);
    }
    p->S = S;
    p->bytes = bytes;

    // First non-empty chunk of every wave's step range.
    std::vector<uint32_t> wc(p->W, 0);
    {
        size_t c = 0;
        for (uint32_t w = 0; w < p->W; w++) {
            const uint64_t g0 = (S == 0) ? 0 : ((uint64_t) w * S) / p->W;
            while (c < n && (desc[c].nsteps == 0 || desc[c].g + desc[c].nsteps <= g0)) {
                c++;
            }
            wc[w] = (uint32_t) std::min(c, n ? n - 1 : 0);
        }
    }
    const uint64_t per_wave = S / p->W + 2;
    const uint64_t nx4k = std::min(max_steps, per_wave) + 2;
    std::vector<uint32_t> x4k(nx4k);
    cioa_gen_xpow8_table(x4k.data(), nx4k, (uint64_t) kStep);

    hipError_t e;
    if ((e = hipMalloc(&p->desc, desc.size() * sizeof(ChunkDesc))) != hipSuccess ||
        (e = hipMalloc(&p->wave_chunk0, wc.size() * sizeof(uint32_t))) != hipSuccess ||
        (e = hipMalloc(&p->partials, ((size_t) p->W + n + 1) * sizeof(uint32_t))) != hipSuccess ||
        (e = hipMalloc(&p->x4k, nx4k * sizeof(uint32_t))) != hipSuccess ||
        (e = hipMemcpy(p->desc, desc.data(), desc.size() * sizeof(ChunkDesc), hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(p->wave_chunk0, wc.data(), wc.size() * sizeof(uint32_t), hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(p->x4k, x4k.data(), nx4k * sizeof(uint32_t), hipMemcpyHostToDevice)) != hipSuccess) {
        cio_crc32_plan_destroy(p);
        return fail("cio_crc32_plan_create: device allocation/upload", e);
    }
    *out = p;
    return CIO_OK;
}

uint64_t cio_crc32_plan_bytes(const cio_crc32_plan *p)
{
    return p ? p->bytes : 0;
}

static int plan_exec_impl(const cio_crc32_plan *p, const void *dev_base, const uint32_t *dev_seeds,
                          uint32_t *dev_out, const uint32_t *cid, hipStream_t s,
                          hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);

int cio_crc32_plan_exec_events(const cio_crc32_plan *p, const void *dev_base,
                               const uint32_t *dev_seeds, uint32_t *dev_out, void *stream,
                               void *ev_piece_start, void *ev_piece_stop)
{
    return plan_exec_impl(p, dev_base, dev_seeds, dev_out, nullptr,
                          reinterpret_cast<hipStream_t>(stream),
                          reinterpret_cast<hipEvent_t>(ev_piece_start),
                          reinterpret_cast<hipEvent_t>(ev_piece_stop));
}

int cio_crc32_plan_exec(const cio_crc32_plan *p, const void *dev_base, const uint32_t *dev_seeds,
                        uint32_t *dev_out, void *stream)
{
    return plan_exec_impl(p, dev_base, dev_seeds, dev_out, nullptr,
                          reinterpret_cast<hipStream_t>(stream));
}

}  // extern "C"

static int plan_exec_impl(const cio_crc32_plan *p, const void *dev_base, const uint32_t *dev_seeds,
                          uint32_t *dev_out, const uint32_t *cid, hipStream_t s,
                          hipEvent_t ev0, hipEvent_t ev1)
{
    if (!p) {
        return fail("cio_crc32_plan_exec: null plan");
    }
    if (p->n == 0) {
        return CIO_OK;
    }
    if (!dev_base || !dev_out) {
        return fail("cio_crc32_plan_exec: null buffer");
    }
    const DeviceState *st = p->st;
    if (ev0) {
        HIP_TRY(hipEventRecord(ev0, s), "hipEventRecord");
    }
    if (p->S > 0) {
        hipLaunchKernelGGL(crc32_piece_kernel, dim3(p->grid), dim3(kThreads), 0, s,
                           reinterpret_cast<const uint8_t *>(dev_base), p->desc, p->wave_chunk0,
                           dev_seeds, p->partials, st->slice, st->shift, st->x8, cid, p->S, p->W, p->n);
        HIP_TRY(hipGetLastError(), "crc32_piece_kernel launch");
    }
    if (ev1) {
        HIP_TRY(hipEventRecord(ev1, s), "hipEventRecord");
    }
    const uint32_t fb = 256;
    hipLaunchKernelGGL(crc32_finish_kernel, dim3((p->n + fb - 1) / fb), dim3(fb), 0, s,
                       reinterpret_cast<const uint8_t *>(dev_base), p->desc, dev_seeds,
                       p->partials, dev_out, st->slice, st->x8, p->x4k, cid, p->S, p->W, p->n);
    HIP_TRY(hipGetLastError(), "crc32_finish_kernel launch");
    return CIO_OK;
}

extern "C" {

int cio_crc32_batch_dev(const void *dev_base, const uint64_t *offs, const uint64_t *lens,
                        const uint32_t *dev_seeds, uint32_t *dev_out, size_t n, void *stream)
{
    cio_crc32_plan *p = nullptr;
    if (cio_crc32_plan_create(&p, offs, lens, n) != CIO_OK) {
        return CIO_ERROR;
    }
    int rc = cio_crc32_plan_exec(p, dev_base, dev_seeds, dev_out, stream);
    if (rc == CIO_OK) {
        hipError_t e = hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream));
        if (e != hipSuccess) {
            rc = fail("cio_crc32_batch_dev: stream sync", e);
        }
    }
    cio_crc32_plan_destroy(p);
    return rc;
}

int cio_gpu_fill_synthetic(void *dev_base, const uint64_t *offs, const uint64_t *lens,
                           const uint64_t *ids, size_t n, uint64_t seed, void *stream)
{
    if (n == 0) {
        return CIO_OK;
    }
    DeviceState *st;
    if (device_state(&st) != CIO_OK) {
        return CIO_ERROR;
    }
    uint64_t *d_meta = nullptr;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    HIP_TRY(hipMalloc(&d_meta, 3 * n * sizeof(uint64_t)), "fill: hipMalloc");
    uint64_t *d_offs = d_meta, *d_lens = d_meta + n, *d_ids = ids ? d_meta + 2 * n : nullptr;
    hipError_t e = hipMemcpy(d_offs, offs, n * sizeof(uint64_t), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_lens, lens, n * sizeof(uint64_t), hipMemcpyHostToDevice);
    if (e == hipSuccess && ids) e = hipMemcpy(d_ids, ids, n * sizeof(uint64_t), hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        const uint32_t grid = (uint32_t) std::min<size_t>(n, 65535);
        hipLaunchKernelGGL(fill_kernel, dim3(grid), dim3(256), 0, s,
                           reinterpret_cast<uint8_t *>(dev_base), d_offs, d_lens, d_ids, seed,
                           (uint32_t) n);
        e = hipGetLastError();
    }
    if (e == hipSuccess) {
        e = hipStreamSynchronize(s);
    }
    (void) hipFree(d_meta);
    if (e != hipSuccess) {
        return fail("fill_kernel", e);
    }
    return CIO_OK;
}

void *cio_gpu_event_create(void)
{
    hipEvent_t ev = nullptr;
    if (hipEventCreate(&ev) != hipSuccess) {
        return nullptr;
    }
    return ev;
}

void cio_gpu_event_destroy(void *ev)
{
    if (ev) {
        (void) hipEventDestroy(reinterpret_cast<hipEvent_t>(ev));
    }
}

int cio_gpu_event_record(void *ev, void *stream)
{
    HIP_TRY(hipEventRecord(reinterpret_cast<hipEvent_t>(ev), reinterpret_cast<hipStream_t>(stream)),
            "hipEventRecord");
    return CIO_OK;
}

float cio_gpu_event_elapsed_ms(void *start, void *stop)
{
    float ms = -1.0f;
    if (hipEventSynchronize(reinterpret_cast<hipEvent_t>(stop)) != hipSuccess) {
        return -1.0f;
    }
    if (hipEventElapsedTime(&ms, reinterpret_cast<hipEvent_t>(start),
                            reinterpret_cast<hipEvent_t>(stop)) != hipSuccess) {
        return -1.0f;
    }
    return ms;
}

int cio_gpu_stream_sync(void *stream)
{
    HIP_TRY(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)), "hipStreamSynchronize");
    return CIO_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- host-memory batch
//
// End-to-end path for chunks that live in host memory (mmap'd chunk files,
// src/cio_file_unix.c:100): the batch is cut into segments of at most
// kStage bytes, packed into groups; each group is copied by host threads into
// one of two pinned staging buffers, sent with hipMemcpyAsync to one of two
// device buffers, and CRC'd by a plan whose seeds/outputs go through a
// chunk-id map into one running-state array on the device, so a chunk split
// over several groups chains its state on the GPU with no host round trip.
// Copies of group g+1 overlap the kernels of group g.

#include <thread>

namespace {

constexpr size_t kStage = 64ull << 20;

struct HostGroup {
    std::vector<const uint8_t *> src;
    std::vector<uint64_t> offs, lens;
    std::vector<uint32_t> cid;
    uint64_t bytes = 0;
    cio_crc32_plan *plan = nullptr;
    uint32_t *d_cid = nullptr;
};

void parallel_copy(uint8_t *dst, const HostGroup &g)
{
    const size_t nthreads = std::min<size_t>(8, std::max<size_t>(1, g.bytes >> 22));
    if (nthreads <= 1) {
        for (size_t k = 0; k < g.src.size(); k++) {
            memcpy(dst + g.offs[k], g.src[k], g.lens[k]);
        }
        return;
    }
    // Split the group's byte range evenly; each thread copies its slice.
    std::vector<std::thread> th;
    const uint64_t per = (g.bytes + nthreads - 1) / nthreads;
    for (size_t t = 0; t < nthreads; t++) {
        th.emplace_back([&, t]() {
            const uint64_t lo = t * per, hi = std::min<uint64_t>(g.bytes, lo + per);
            for (size_t k = 0; k < g.src.size(); k++) {
                const uint64_t a = g.offs[k], b = a + g.lens[k];
                const uint64_t x = std::max(a, lo), y = std::min(b, hi);
                if (x < y) {
                    memcpy(dst + x, g.src[k] + (x - a), y - x);
                }
            }
        });
    }
    for (auto &t : th) {
        t.join();
    }
}

}  // namespace

extern "C" int cio_crc32_batch_host(const void *const *bufs, const size_t *lens, const uint32_t *seeds,
                                    uint32_t *out_raw, size_t n)
{
    if (n == 0) {
        return CIO_OK;
    }
    if (!bufs || !lens || !out_raw) {
        return fail("cio_crc32_batch_host: null argument");
    }
    DeviceState *st;
    if (device_state(&st) != CIO_OK) {
        return CIO_ERROR;
    }
    // Build groups of <= kStage bytes, 16-byte aligned segment placement.
    std::vector<HostGroup> groups(1);
    for (size_t i = 0; i < n; i++) {
        const uint8_t *p = reinterpret_cast<const uint8_t *>(bufs[i]);
        uint64_t left = lens[i], done = 0;
        do {
            HostGroup *g = &groups.back();
            uint64_t at = (g->bytes + 15) & ~15ull;
            if (at >= kStage) {
                groups.emplace_back();
                g = &groups.back();
                at = 0;
            }
            const uint64_t take = std::min<uint64_t>(left, kStage - at);
            g->src.push_back(p + done);
            g->offs.push_back(at);
            g->lens.push_back(take);
            g->cid.push_back((uint32_t) i);
            g->bytes = at + take;
            left -= take;
            done += take;
        } while (left > 0);
    }

    int rc = CIO_OK;
    uint8_t *pinned[2] = {nullptr, nullptr};
    uint8_t *dbuf[2] = {nullptr, nullptr};
    uint32_t *d_state = nullptr;
    hipStream_t stream[2] = {nullptr, nullptr};
    hipEvent_t copied[2] = {nullptr, nullptr}, done_k[2] = {nullptr, nullptr};
    std::vector<uint32_t> init(n);
    for (size_t i = 0; i < n; i++) {
        init[i] = seeds ? seeds[i] : 0xffffffffu;
    }
    hipError_t e = hipSuccess;
    for (int b = 0; b < 2 && e == hipSuccess; b++) {
        if ((e = hipHostMalloc(&pinned[b], kStage, hipHostMallocDefault)) != hipSuccess) break;
        if ((e = hipMalloc(&dbuf[b], kStage + 64)) != hipSuccess) break;
        if ((e = hipStreamCreateWithFlags(&stream[b], hipStreamNonBlocking)) != hipSuccess) break;
        if ((e = hipEventCreateWithFlags(&copied[b], hipEventDisableTiming)) != hipSuccess) break;
        if ((e = hipEventCreateWithFlags(&done_k[b], hipEventDisableTiming)) != hipSuccess) break;
    }
    if (e == hipSuccess) e = hipMalloc(&d_state, n * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemcpy(d_state, init.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice);
    for (size_t gi = 0; gi < groups.size() && e == hipSuccess && rc == CIO_OK; gi++) {
        HostGroup &g = groups[gi];
        if (cio_crc32_plan_create(&g.plan, g.offs.data(), g.lens.data(), g.offs.size()) != CIO_OK) {
            rc = CIO_ERROR;
            break;
        }
        if ((e = hipMalloc(&g.d_cid, g.cid.size() * sizeof(uint32_t))) != hipSuccess) break;
        e = hipMemcpy(g.d_cid, g.cid.data(), g.cid.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
    }
    for (size_t gi = 0; gi < groups.size() && e == hipSuccess && rc == CIO_OK; gi++) {
        const int b = (int) (gi & 1);
        HostGroup &g = groups[gi];
        if (gi >= 2) {
            // pinned[b] is free once the H2D of group gi-2 has completed.
            if ((e = hipEventSynchronize(copied[b])) != hipSuccess) break;
        }
        parallel_copy(pinned[b], g);
        if (gi >= 1) {
            // Chained states: this group's kernels run after the previous group's.
            if ((e = hipStreamWaitEvent(stream[b], done_k[b ^ 1], 0)) != hipSuccess) break;
        }
        if ((e = hipMemcpyAsync(dbuf[b], pinned[b], g.bytes, hipMemcpyHostToDevice, stream[b])) != hipSuccess) break;
        if ((e = hipEventRecord(copied[b], stream[b])) != hipSuccess) break;
        if (plan_exec_impl(g.plan, dbuf[b], d_state, d_state, g.d_cid, stream[b]) != CIO_OK) {
            rc = CIO_ERROR;
            break;
        }
        if ((e = hipEventRecord(done_k[b], stream[b])) != hipSuccess) break;
    }
    if (e == hipSuccess && rc == CIO_OK) {
        for (int b = 0; b < 2 && e == hipSuccess; b++) {
            e = hipStreamSynchronize(stream[b]);
        }
        if (e == hipSuccess) {
            e = hipMemcpy(out_raw, d_state, n * sizeof(uint32_t), hipMemcpyDeviceToHost);
        }
    }
    for (auto &g : groups) {
        cio_crc32_plan_destroy(g.plan);
        (void) hipFree(g.d_cid);
    }
    for (int b = 0; b < 2; b++) {
        if (stream[b]) (void) hipStreamSynchronize(stream[b]);
        (void) hipHostFree(pinned[b]);
        (void) hipFree(dbuf[b]);
        if (stream[b]) (void) hipStreamDestroy(stream[b]);
        if (copied[b]) (void) hipEventDestroy(copied[b]);
        if (done_k[b]) (void) hipEventDestroy(done_k[b]);
    }
    (void) hipFree(d_state);
    if (e != hipSuccess) {
        return fail("cio_crc32_batch_host", e);
    }
    return rc;
}
