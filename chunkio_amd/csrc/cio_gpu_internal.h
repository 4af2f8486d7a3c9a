// cio_gpu_internal.h -- declarations shared by the HIP translation units of
// libchunkio_amd.so (crc32_gpu.hip: kernels, device state, plans;
// host_pipeline.hip: the host-memory / file batch pipeline).  Not installed.
#ifndef CIOA_GPU_INTERNAL_H
#define CIOA_GPU_INTERNAL_H

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <vector>

#include "cio_diag.h"
#include "crc32_host.h"
#include "chunkio_amd/cio_crc32_gpu.h"

namespace cioa {

constexpr int kWave = 64;
constexpr int kGran = 16;                   // bytes per lane per sub-chain per step
constexpr int kSub = 4;                     // sub-chains per lane
constexpr int kRow = kWave * kGran;         // 1024: one coalesced wave-instruction
constexpr int kStep = kSub * kRow;          // 4096 bytes per wave-step
constexpr int kThreads = 1024;              // one workgroup per CU
constexpr uint32_t kWavesPerWg = kThreads / kWave;   // 16
// Per-wave flags (the plan's pfac array continues with one word per wave):
//   bit 0: the wave's first chunk began in an earlier wave of this workgroup
//          and ends in this wave's range (the wave folds it through LDS);
//   bits 8..15: how many waves before this one hold its earlier pieces;
//   bit 1: the range ends inside a chunk whose pieces all lie in this
//          workgroup (the wave hands that piece over through LDS).
constexpr uint32_t kWfFold = 1u, kWfPublish = 2u;
constexpr int kX8Count = 2 * kStep;         // x^(8m), m in [0, 8192)
constexpr uint32_t kSliceBytes = 131072;    // 4 tables x 256 x 32 replicas x 4 B
constexpr uint32_t kShiftBytes = 32768;     // 4 tables x 256 x 8 replicas x 4 B
constexpr uint32_t kShiftOff = kSliceBytes;
constexpr uint32_t kLdsBytes = kSliceBytes + kShiftBytes;   // all 160 KiB of the CU
constexpr int kStampWords = 16;             // diagnostic stamps per wave (CIO_GPU_STAMPS)

struct ChunkDesc {
    uint64_t a;        // aligned-down start offset from the batch base
    uint64_t vlen;     // virtual length = (off & 15) + len
    uint64_t g;        // first global wave-step of this chunk
    uint32_t nsteps;   // ceil(vlen / kStep); 0 for tiny chunks (len < 4)
    uint32_t h;        // off & 15 (zeroed head bytes)
    uint32_t npieces;  // waves holding a piece of this chunk
    uint32_t w0, w1;   // first and last wave holding a piece (npieces > 0)
    uint32_t pad;
};
static_assert(sizeof(ChunkDesc) == 48, "desc layout");

// Where each wave's step range begins: its first chunk and that chunk's
// descriptor, so a wave starts streaming after ONE scalar load.
struct WaveStart {
    ChunkDesc d;
    uint32_t c;
    uint32_t pad[3];
};
static_assert(sizeof(WaveStart) == 64, "wave start layout");

// Per-device constant tables (global memory), built once per process.
struct DeviceState {
    bool ready = false;
    int cus = 0;
    uint32_t *slice = nullptr;   // [4][256] compact
    uint32_t *shift = nullptr;   // [4][256] shift by kStep - kGran
    uint32_t *x8 = nullptr;      // [kX8Count]
    uint32_t *xinv8 = nullptr;   // [kStep]: x^(-8 d) (d bytes un-shifted)
};

// Host image of everything a launch reads besides the data.
struct PlanHost {
    std::vector<ChunkDesc> desc;
    std::vector<WaveStart> ws;
    std::vector<uint32_t> tiny;
    std::vector<uint32_t> pfac;   // per piece slot (wave + chunk), then W wave flags, then W last-piece factors
    uint64_t S = 0, bytes = 0;
};

constexpr int kMaxDev = 64;          // device ordinals with per-device state

// The calling thread's last error message (cio_gpu_last_error).
extern thread_local std::string g_err;
// Record the message for cio_gpu_last_error(); returns CIO_ERROR.
int fail(const char *what, hipError_t e = hipSuccess);
// The calling thread's current device's state (built on first use).
int device_state(DeviceState **out);
// Plan geometry and knobs for n chunks on st's device.
void plan_init(cio_crc32_plan *p, DeviceState *st, size_t n);
// Descriptors, split, piece counts and fold factors; nullptr or an error message.
const char *plan_build(PlanHost &ph, const uint64_t *offs, const uint64_t *lens, size_t n, uint32_t W);
// One launch of plan p over dev_base (chunk-id map cid: outputs and seeds by id).
int plan_exec_impl(const cio_crc32_plan *p, const void *dev_base, const uint32_t *dev_seeds,
                   uint32_t *dev_out, const uint32_t *cid, hipStream_t s,
                   hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);

}  // namespace cioa

#define HIP_TRY(expr, what)                                \
    do {                                                   \
        hipError_t e_ = (expr);                            \
        if (e_ != hipSuccess) return cioa::fail(what, e_); \
    } while (0)

struct cio_crc32_plan {
    uint32_t n = 0;
    uint64_t S = 0;            // total wave-steps
    uint32_t W = 0;            // waves in the grid
    uint32_t grid = 0;         // workgroups
    uint32_t ntiny = 0;        // chunks with len < 4 (byte-serial)
    int prio = 1;              // CIO_GPU_PRIO: 0 none, 1 per-step rotation (2/3, time-sliced, measured slower and removed)
    uint64_t ustride = 0, ua0 = 0, uvlen = 0;   // uniform batch geometry (unsteps > 0)
    uint32_t unsteps = 0, uh = 0;
    bool small = false;        // every chunk fits one wave-step: crc32_small_kernel
    bool ahead = false;        // uniform, 16-B aligned, whole 4 KiB steps: issue-ahead stream kernel
    bool l64 = false;          // stream kernels: one 64-byte chain per lane (CIO_GPU_L64)
    bool l64_small = false;    // the same layout in the small-chunk kernel
    unsigned long long *stamps = nullptr;   // CIO_GPU_STAMPS=1: diagnostic timestamps
    uint64_t bytes = 0;        // sum of lens
    cioa::ChunkDesc *desc = nullptr;
    cioa::WaveStart *wstart = nullptr;
    uint32_t *tiny = nullptr;
    unsigned long long *partials = nullptr;
    uint32_t *counters = nullptr;
    uint32_t *pfac = nullptr;   // per piece slot: x^(8 * chunk bytes after the piece)
    cioa::DeviceState *st = nullptr;
};

#endif
