// host_pipeline.hip -- the batch path for chunks in host memory or in files
// (cio_crc32_batch_host[_multi], cio_crc32_batch_fd_multi, registered ranges,
// device selection).  Kernels, plans and device state: crc32_gpu.hip.
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include "cio_gpu_internal.h"

using namespace cioa;

// ---------------------------------------------------------------- host-memory batch
//
// End-to-end path for chunks that live in host memory (mmap'd chunk files,
// src/cio_file_unix.c:100).  The batch is cut into segments of at most kStage
// bytes packed into groups.  A persistent per-device pipeline of kSlots slots
// (pinned staging buffer, pinned plan image, device buffer, device plan
// arena, stream) carries the groups: host threads copy group g into a free
// slot while the DMA engine moves group g-1 and the GPU CRCs group g-2.  Each
// group's plan is built on the host straight into the slot's pinned image and
// uploaded with the data, so steady-state calls allocate nothing.  Seeds and
// outputs go through a chunk-id map into one running-state array on the
// device, so a chunk split over several groups chains its state on the GPU.

#include <atomic>
#include <ctype.h>
#include <pthread.h>
#include <sched.h>
#include <thread>
#include <condition_variable>
#include <errno.h>
#include <time.h>
#include <unistd.h>

namespace {

// Slot size: CIO_GPU_STAGE_MB (read once, when the pipeline is created),
// default 64 MiB.  Smaller groups shorten the pipeline's fill and drain (the
// first group's host copy and the last group's DMA are not overlapped).
static size_t stage_bytes()
{
    static const size_t v = [] {
        size_t mb = 64;
        if (const char *r = cioa_diag_getenv("CIO_GPU_STAGE_MB")) {
            const long x = atol(r);
            if (x >= 1 && x <= 1024) {
                mb = (size_t) x;
            }
        }
        return mb << 20;
    }();
    return v;
}
#define kStage (stage_bytes())

// Capacity of a call's first staging group (CIO_GPU_STAGE_FIRST_MB, default 4);
// each later group doubles it up to kStage.
static size_t first_stage_bytes()
{
    static const size_t v = [] {
        size_t mb = 4;
        if (const char *r = cioa_diag_getenv("CIO_GPU_STAGE_FIRST_MB")) {
            const long x = atol(r);
            if (x >= 1 && x <= 1024) {
                mb = (size_t) x;
            }
        }
        return mb << 20;
    }();
    return v;
}
constexpr int kSlots = CIO_PIPE_SLOTS;   // 3 (cio_diag.h)

// One staging group.  A source is host memory (src[k]) or, for batches read
// straight from files, a file range (fd[k], foff[k]) that the copy threads
// pread() into the pinned buffer: no mapping, no page faults, no TLB
// shootdowns at unmap.
struct HostGroup {
    std::vector<const uint8_t *> src;
    std::vector<int> fd;               // empty for memory sources
    std::vector<uint64_t> foff;
    std::vector<uint64_t> offs, lens;
    std::vector<uint32_t> cid;
    uint64_t bytes = 0;
};

// Persistent host copy workers (the box's CPU share per GPU is 16 threads).
// copy() cuts a group's byte range into pieces that the workers and the
// caller claim through one atomic counter, so a slow or descheduled thread
// delays the group by one piece, not by a 1/16 slice.  Pieces are 1 MiB, or
// smaller for small groups so every thread gets about two (a call's first
// 4 MiB group in 1 MiB pieces kept 12 of the 16 threads idle while the DMA
// engine waited for it).  The caller first runs `before` (the group's plan
// build), overlapping it with the workers' copying.
// CPUs of the NUMA node whose PCIe root the device hangs off, within this
// process's affinity (empty when unknown: no sysfs node, node -1, or no
// overlap).  *node_out = that node or -1.
std::vector<int> device_local_cpus(int dev, int *node_out)
{
    *node_out = -1;
    char bdf[64] = {0};
    if (hipDeviceGetPCIBusId(bdf, (int) sizeof(bdf) - 1, dev) != hipSuccess) {
        return {};
    }
    for (char *c = bdf; *c; ++c) {
        *c = (char) tolower((unsigned char) *c);
    }
    char path[192];
    snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/numa_node", bdf);
    int node = -1;
    if (FILE *f = fopen(path, "r")) {
        if (fscanf(f, "%d", &node) != 1) {
            node = -1;
        }
        fclose(f);
    }
    if (node < 0) {
        return {};
    }
    *node_out = node;
    snprintf(path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", node);
    std::vector<int> cpus;
    if (FILE *f = fopen(path, "r")) {
        int a, b;
        char sep;
        while (fscanf(f, "%d", &a) == 1) {
            b = a;
            if (fscanf(f, "%c", &sep) == 1 && sep == '-') {
                if (fscanf(f, "%d", &b) != 1) {
                    break;
                }
                if (fscanf(f, "%c", &sep) != 1) {
                    sep = '\n';
                }
            }
            for (int c = a; c <= b; c++) {
                cpus.push_back(c);
            }
            if (sep != ',') {
                break;
            }
        }
        fclose(f);
    }
    cpu_set_t mine;
    CPU_ZERO(&mine);
    if (sched_getaffinity(0, sizeof(mine), &mine) != 0) {
        return {};
    }
    std::vector<int> out;
    for (int c : cpus) {
        if (c >= 0 && c < CPU_SETSIZE && CPU_ISSET(c, &mine)) {
            out.push_back(c);
        }
    }
    return out;
}

class CopyPool {
public:
    static constexpr uint64_t kPieceMax = 1ull << 20;
    static constexpr uint64_t kPieceMin = 64ull << 10;

    uint64_t piece_bytes(uint64_t bytes) const
    {
        static const uint64_t fixed = [] {
            const char *r = cioa_diag_getenv("CIO_GPU_COPY_PIECE_KB");   // A/B knob: a fixed piece size
            const long v = r ? atol(r) : 0;
            return v >= 4 && v <= 65536 ? (uint64_t) v << 10 : 0;
        }();
        if (fixed) {
            return fixed;
        }
        const uint64_t per = bytes / (2 * (workers_.size() + 1));
        return std::min(kPieceMax, std::max(kPieceMin, (per + kPieceMin - 1) & ~(kPieceMin - 1)));
    }

    // Workers run on the CPUs of the device's NUMA node when that is known
    // (CIO_GPU_COPY_NUMA=0: wherever the scheduler puts them): the staging
    // copy writes pinned memory the device DMAs from, and a copy thread on
    // the far socket sends every byte over the inter-socket link first.
    explicit CopyPool(int dev)
    {
        const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
        const unsigned nw = std::min(15u, hw > 1 ? hw - 1 : 0u);
        static const bool numa = [] {
            const char *r = cioa_diag_getenv("CIO_GPU_COPY_NUMA");
            return !(r && r[0] == '0');
        }();
        int node = -1;
        const std::vector<int> local = numa ? device_local_cpus(dev, &node) : std::vector<int>();
        for (unsigned t = 0; t < nw; t++) {
            workers_.emplace_back([this]() { run(); });
            if (!local.empty()) {
                cpu_set_t set;
                CPU_ZERO(&set);
                for (int c : local) {
                    CPU_SET(c, &set);
                }
                (void) pthread_setaffinity_np(workers_.back().native_handle(), sizeof(set), &set);
            }
        }
    }
    ~CopyPool()
    {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &w : workers_) {
            w.join();
        }
    }
    // false if a file source could not be read in full
    template <typename F>
    bool copy(uint8_t *dst, const HostGroup &g, F before)
    {
        const uint64_t piece = piece_bytes(g.bytes);
        const uint64_t npieces = (g.bytes + piece - 1) / piece;
        if (npieces <= 1 || workers_.empty()) {
            before();
            const bool ok = range(dst, g, 0, g.bytes);
            cioa_stage_fence();
            return ok;
        }
        {
            std::lock_guard<std::mutex> lk(mu_);
            dst_ = dst;
            g_ = &g;
            npieces_ = npieces;
            piece_ = piece;
            next_.store(0, std::memory_order_relaxed);
            pending_ = workers_.size();
            failed_ = false;
            ++gen_;
        }
        cv_.notify_all();
        before();
        const bool ok = drain(dst, g, npieces, piece);
        cioa_stage_fence();
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [this] { return pending_ == 0; });
        return ok && !failed_;
    }

private:
    bool drain(uint8_t *dst, const HostGroup &g, uint64_t npieces, uint64_t piece)
    {
        bool ok = true;
        for (;;) {
            const uint64_t p = next_.fetch_add(1, std::memory_order_relaxed);
            if (p >= npieces) {
                return ok;
            }
            ok &= range(dst, g, p * piece, std::min<uint64_t>(g.bytes, (p + 1) * piece));
        }
    }
    static constexpr uint64_t kBounce = 256u << 10;
    static uint8_t *bounce_buffer()
    {
        thread_local std::unique_ptr<uint8_t[]> b(new uint8_t[kBounce]);
        return b.get();
    }
    // Bytes [lo, hi) of the group's staging image.
    static bool range(uint8_t *dst, const HostGroup &g, uint64_t lo, uint64_t hi)
    {
        // first chunk ending after lo (offs increase along the group)
        size_t k = (size_t) (std::upper_bound(g.offs.begin(), g.offs.end(), lo) - g.offs.begin());
        k = k ? k - 1 : 0;
        bool ok = true;
        for (; k < g.offs.size() && g.offs[k] < hi; k++) {
            const uint64_t a = g.offs[k], b = a + g.lens[k];
            const uint64_t x = std::max(a, lo), y = std::min(b, hi);
            if (x >= y) {
                continue;
            }
            if (g.fd.empty()) {
                cioa_stage_copy(dst + x, g.src[k] + (x - a), y - x);
                continue;
            }
            // File source: pread through a per-thread, cache-resident bounce
            // buffer, then the streaming copy into staging -- a pread straight
            // into the pinned image would read every destination line first.
            uint8_t *bounce = cioa_stage_nt() ? bounce_buffer() : nullptr;
            uint64_t done = 0;
            while (done < y - x) {
                uint8_t *to = bounce ? bounce : dst + x + done;
                const uint64_t want = bounce ? std::min<uint64_t>(y - x - done, kBounce) : y - x - done;
                const ssize_t r = pread(g.fd[k], to, want, (off_t) (g.foff[k] + (x - a) + done));
                if (r <= 0) {
                    if (r < 0 && errno == EINTR) {
                        continue;
                    }
                    ok = false;
                    break;
                }
                if (bounce) {
                    cioa_stage_copy(dst + x + done, bounce, (size_t) r);
                }
                done += (uint64_t) r;
            }
        }
        return ok;
    }
    void run()
    {
        uint64_t seen = 0;
        for (;;) {
            uint8_t *dst;
            const HostGroup *g;
            uint64_t npieces, piece;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) {
                    return;
                }
                seen = gen_;
                dst = dst_;
                g = g_;
                npieces = npieces_;
                piece = piece_;
            }
            const bool ok = drain(dst, *g, npieces, piece);
            cioa_stage_fence();
            std::lock_guard<std::mutex> lk(mu_);
            failed_ = failed_ || !ok;
            if (--pending_ == 0) {
                done_cv_.notify_one();
            }
        }
    }
    std::vector<std::thread> workers_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    bool stop_ = false;
    bool failed_ = false;
    uint64_t gen_ = 0;
    uint8_t *dst_ = nullptr;
    const HostGroup *g_ = nullptr;
    uint64_t npieces_ = 0;
    uint64_t piece_ = kPieceMax;
    std::atomic<uint64_t> next_{0};
    size_t pending_ = 0;
};

size_t align256(size_t x)
{
    return (x + 255) & ~(size_t) 255;
}

struct PipeSlot {
    uint8_t *pinned = nullptr;       // kStage data
    uint8_t *dbuf = nullptr;         // kStage + 64
    uint8_t *meta_h = nullptr;       // pinned plan image
    uint8_t *meta_d = nullptr;       // device plan image
    size_t meta_cap = 0;
    unsigned long long *partials = nullptr;
    size_t part_cap = 0;
    uint32_t *counters = nullptr;    // zero between launches (self-resetting)
    size_t cnt_cap = 0;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;       // after the slot's kernel
    bool busy = false;
};

// A built plan image (the bytes stage_plan copies into a slot's pinned
// arena) and the geometry it was built for.  Batches of the same geometry
// recur -- the chunk layer's syncs of equal-sized chunks, a scan of
// equal-sized files, a benchmark's repeated batch -- and building a group's
// plan (ChunkDesc / WaveStart / fold factors for 4096 waves, ~0.1 ms) then
// costs more than copying its ~330 KB image.  The key is a 128-bit digest of
// the whole geometry (offsets, lengths, chunk ids, wave count: two
// independent 64-bit hashes), not a copy of it, so an entry holds only its
// image.  Entries are admitted on a geometry's SECOND sighting (a stream of
// never-repeating batches -- the chunk layer's varying sync batches -- stores
// nothing) and the cache is capped in bytes per pipeline.
struct GeoKey {
    uint64_t a = 0, b = 0;
    uint32_t W = 0;
    uint64_t n = 0;
    bool operator==(const GeoKey &o) const { return a == o.a && b == o.b && W == o.W && n == o.n; }
};

struct PlanImage {
    GeoKey key;
    std::vector<uint64_t> offs, lens;   // the geometry itself (cached entries): a hit compares it whole
    std::vector<uint8_t> image;
    size_t o_desc = 0, o_ws = 0, o_tiny = 0, o_pfac = 0, o_cid = 0, npfac = 0;
    uint64_t S = 0, bytes = 0;
    uint32_t ntiny = 0;
    uint64_t used = 0;               // LRU clock
};

constexpr int kSeen = 64;            // recent misses remembered for admission

struct HostPipe {
    bool ready = false;
    CopyPool *pool = nullptr;
    PipeSlot slot[kSlots];
    uint32_t *state = nullptr;       // running raw CRC per chunk of the call
    size_t state_cap = 0;
    std::vector<PlanImage> plans;    // plan image cache (one pipeline = one caller at a time)
    size_t plan_bytes = 0;           // sum of the cached images and their geometries
    uint64_t plan_clock = 0;
    GeoKey seen[kSeen];              // ring of geometries seen once (admission filter)
    int seen_next = 0;
    uint64_t hits = 0, misses = 0, stores = 0, evictions = 0;
};

// Plan image cache limits per pipeline: CIO_GPU_PLAN_CACHE entries (default
// 32, 0 = off) and CIO_GPU_PLAN_CACHE_MB megabytes (default 16; an image
// larger than a quarter of it is never cached).  A 64 MiB group of 400 KB
// chunks is ~330 KB; of 4 KiB chunks ~1.3 MB.
static size_t plan_cache_entries()
{
    static const size_t v = [] {
        long k = 32;
        if (const char *r = getenv("CIO_GPU_PLAN_CACHE")) {
            k = atol(r);
            if (k < 0 || k > 1024) {
                k = 32;
            }
        }
        return (size_t) k;
    }();
    return v;
}

static size_t plan_cache_bytes()
{
    static const size_t v = [] {
        long mb = 16;
        if (const char *r = getenv("CIO_GPU_PLAN_CACHE_MB")) {
            mb = atol(r);
            if (mb < 0 || mb > 4096) {
                mb = 16;
            }
        }
        return (size_t) mb << 20;
    }();
    return v;
}

static GeoKey geometry_key(const HostGroup &g, uint32_t W)
{
    // FNV-1a-style and a multiply-xorshift over the same words, different
    // constants: a false match needs both 64-bit digests to collide.
    uint64_t h1 = 0xcbf29ce484222325ull ^ W, h2 = 0x9E3779B97F4A7C15ull + W;
    auto mix = [&](uint64_t x) {
        h1 ^= x;
        h1 *= 0x100000001b3ull;
        h1 ^= h1 >> 29;
        h2 += x * 0xbf58476d1ce4e5b9ull;
        h2 ^= h2 >> 31;
        h2 *= 0x94d049bb133111ebull;
    };
    const size_t n = g.offs.size();
    mix(n);
    for (size_t i = 0; i < n; i++) {
        mix(g.offs[i]);
        mix(g.lens[i]);
        mix(g.cid[i]);
    }
    GeoKey k;
    k.a = h1;
    k.b = h2;
    k.W = W;
    k.n = n;
    return k;
}

// Pipelines are pooled per device: a call takes an idle one (or builds one,
// up to CIO_GPU_PIPES_PER_DEV, default 4) and gives it back when done, so
// concurrent callers on one device, and callers on different devices, run
// in parallel.  Nothing global is held while a batch runs.
struct DevPipes {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<HostPipe *> idle;
    int count = 0;
};
DevPipes g_pipes[kMaxDev];

int pipes_per_dev()
{
    static const int v = [] {
        int k = 4;
        if (const char *r = getenv("CIO_GPU_PIPES_PER_DEV")) {
            const int x = atoi(r);
            if (x >= 1 && x <= 64) {
                k = x;
            }
        }
        return k;
    }();
    return v;
}

hipError_t pipe_acquire(int dev, HostPipe **out)
{
    DevPipes &dp = g_pipes[dev];
    std::unique_lock<std::mutex> lk(dp.mu);
    dp.cv.wait(lk, [&] { return !dp.idle.empty() || dp.count < pipes_per_dev(); });
    if (!dp.idle.empty()) {
        *out = dp.idle.back();
        dp.idle.pop_back();
        return hipSuccess;
    }
    dp.count++;
    *out = new HostPipe();
    return hipSuccess;
}

void pipe_release(int dev, HostPipe *hp)
{
    DevPipes &dp = g_pipes[dev];
    {
        std::lock_guard<std::mutex> lk(dp.mu);
        dp.idle.push_back(hp);
    }
    dp.cv.notify_one();
}

// Releases whatever a slot holds (safe on a partly built slot).
void slot_free(PipeSlot &s)
{
    if (s.done) (void) hipEventDestroy(s.done);
    if (s.stream) (void) hipStreamDestroy(s.stream);
    if (s.dbuf) (void) hipFree(s.dbuf);
    if (s.pinned) (void) hipHostFree(s.pinned);
    if (s.meta_h) (void) hipHostFree(s.meta_h);
    if (s.meta_d) (void) hipFree(s.meta_d);
    if (s.partials) (void) hipFree(s.partials);
    if (s.counters) (void) hipFree(s.counters);
    s = PipeSlot();
}

hipError_t pipe_init(HostPipe &hp, int dev)
{
    hipError_t e = hipSuccess;
    for (int b = 0; b < kSlots && e == hipSuccess; b++) {
        PipeSlot &s = hp.slot[b];
        if ((e = hipHostMalloc(&s.pinned, kStage, hipHostMallocDefault)) != hipSuccess) break;
        if ((e = hipMalloc(&s.dbuf, kStage + 64)) != hipSuccess) break;
        if ((e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking)) != hipSuccess) break;
        e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
    }
    if (e != hipSuccess) {
        // A partial set-up is undone, so the next call's pipe_init starts
        // from empty slots instead of overwriting (leaking) these.
        for (int b = 0; b < kSlots; b++) {
            slot_free(hp.slot[b]);
        }
        hp.ready = false;
        return e;
    }
    hp.pool = new CopyPool(dev);
    hp.ready = true;
    return e;
}

template <typename T>
hipError_t grow_dev(T **p, size_t *cap, size_t need, bool zero, hipStream_t s)
{
    if (need <= *cap) {
        return hipSuccess;
    }
    need = std::max(need, *cap * 2);
    (void) hipFree(*p);
    *p = nullptr;
    *cap = 0;
    hipError_t e = hipMalloc(p, need * sizeof(T));
    if (e == hipSuccess && zero) {
        e = hipMemsetAsync(*p, 0, need * sizeof(T), s);
    }
    if (e == hipSuccess) {
        *cap = need;
    }
    return e;
}

hipError_t grow_meta(PipeSlot &s, size_t need)
{
    if (need <= s.meta_cap) {
        return hipSuccess;
    }
    need = std::max(need, s.meta_cap * 2);
    (void) hipHostFree(s.meta_h);
    (void) hipFree(s.meta_d);
    s.meta_h = s.meta_d = nullptr;
    s.meta_cap = 0;
    hipError_t e = hipHostMalloc(&s.meta_h, need, hipHostMallocDefault);
    if (e == hipSuccess) {
        e = hipMalloc(&s.meta_d, need);
    }
    if (e == hipSuccess) {
        s.meta_cap = need;
    }
    return e;
}

// Build group g's plan into slot s (pinned image + device arenas) and return
// a launchable plan view over the slot's device memory.  A geometry seen
// before on this pipeline copies its cached image instead of rebuilding it.
hipError_t stage_plan(HostPipe &hp, PipeSlot &s, const HostGroup &g, DeviceState *st, cio_crc32_plan &view,
                      uint32_t **d_cid, size_t *meta_bytes, const char **err)
{
    const size_t n = g.offs.size();
    plan_init(&view, st, n);
    const size_t ncache = plan_cache_entries();
    GeoKey key;
    PlanImage *hit = nullptr;
    if (ncache) {
        key = geometry_key(g, view.W);
        // The digest only finds a candidate; the entry's stored geometry must
        // match in full (offsets, lengths, chunk ids), so a digest collision
        // can never hand a group another geometry's descriptors.
        for (auto &pi : hp.plans) {
            if (pi.key == key && pi.offs.size() == n &&
                memcmp(pi.offs.data(), g.offs.data(), n * sizeof(uint64_t)) == 0 &&
                memcmp(pi.lens.data(), g.lens.data(), n * sizeof(uint64_t)) == 0 &&
                memcmp(pi.image.data() + pi.o_cid, g.cid.data(), n * sizeof(uint32_t)) == 0) {
                hit = &pi;
                break;
            }
        }
        hit ? hp.hits++ : hp.misses++;
    }
    PlanImage built;
    if (!hit) {
        PlanHost ph;
        if ((*err = plan_build(ph, g.offs.data(), g.lens.data(), n, view.W)) != nullptr) {
            return hipSuccess;
        }
        PlanImage &pi = built;
        pi.o_desc = 0;
        pi.o_ws = pi.o_desc + align256(ph.desc.size() * sizeof(ChunkDesc));
        pi.o_tiny = pi.o_ws + align256(ph.ws.size() * sizeof(WaveStart));
        pi.o_pfac = pi.o_tiny + align256(std::max<size_t>(1, ph.tiny.size()) * sizeof(uint32_t));
        pi.o_cid = pi.o_pfac + align256(ph.pfac.size() * sizeof(uint32_t));
        pi.npfac = ph.pfac.size();
        pi.S = ph.S;
        pi.bytes = ph.bytes;
        pi.ntiny = (uint32_t) ph.tiny.size();
        pi.image.assign(pi.o_cid + align256(n * sizeof(uint32_t)), 0);
        memcpy(pi.image.data() + pi.o_desc, ph.desc.data(), ph.desc.size() * sizeof(ChunkDesc));
        memcpy(pi.image.data() + pi.o_ws, ph.ws.data(), ph.ws.size() * sizeof(WaveStart));
        if (!ph.tiny.empty()) {
            memcpy(pi.image.data() + pi.o_tiny, ph.tiny.data(), ph.tiny.size() * sizeof(uint32_t));
        }
        memcpy(pi.image.data() + pi.o_pfac, ph.pfac.data(), ph.pfac.size() * sizeof(uint32_t));
        memcpy(pi.image.data() + pi.o_cid, g.cid.data(), n * sizeof(uint32_t));
        hit = &built;
    }
    const PlanImage &pi = *hit;
    const size_t total = pi.image.size();
    hipError_t e = grow_meta(s, total);
    if (e == hipSuccess) e = grow_dev(&s.partials, &s.part_cap, pi.npfac, false, s.stream);
    if (e == hipSuccess) e = grow_dev(&s.counters, &s.cnt_cap, std::max<size_t>(1, n), true, s.stream);
    if (e != hipSuccess) {
        return e;
    }
    memcpy(s.meta_h, pi.image.data(), total);
    view.S = pi.S;
    view.bytes = pi.bytes;
    view.ntiny = pi.ntiny;
    view.desc = reinterpret_cast<ChunkDesc *>(s.meta_d + pi.o_desc);
    view.wstart = reinterpret_cast<WaveStart *>(s.meta_d + pi.o_ws);
    view.tiny = reinterpret_cast<uint32_t *>(s.meta_d + pi.o_tiny);
    view.pfac = reinterpret_cast<uint32_t *>(s.meta_d + pi.o_pfac);
    view.partials = s.partials;
    view.counters = s.counters;
    *d_cid = reinterpret_cast<uint32_t *>(s.meta_d + pi.o_cid);
    *meta_bytes = total;
    hit->used = ++hp.plan_clock;
    if (hit == &built && ncache) {
        // Admit on the second sighting only, then evict least recently used
        // entries until both the entry and the byte caps hold.
        bool seen_before = false;
        for (const auto &k : hp.seen) {
            seen_before |= (k == key);
        }
        const size_t sz = built.image.size() + 2 * n * sizeof(uint64_t);
        if (!seen_before) {
            hp.seen[hp.seen_next] = key;
            hp.seen_next = (hp.seen_next + 1) % kSeen;
        } else if (sz <= plan_cache_bytes() / 4) {
            while (!hp.plans.empty() &&
                   (hp.plans.size() >= ncache || hp.plan_bytes + sz > plan_cache_bytes())) {
                auto lru = std::min_element(hp.plans.begin(), hp.plans.end(),
                                            [](const PlanImage &a, const PlanImage &b) { return a.used < b.used; });
                hp.plan_bytes -= lru->image.size() + (lru->offs.size() + lru->lens.size()) * sizeof(uint64_t);
                std::iter_swap(lru, hp.plans.end() - 1);
                hp.plans.pop_back();
                hp.evictions++;
            }
            built.key = key;
            built.offs = g.offs;
            built.lens = g.lens;
            hp.plan_bytes += sz;
            hp.plans.push_back(std::move(built));
            hp.stores++;
        }
    }
    return hipSuccess;
}

// Host ranges pinned in place by cio_crc32_host_register (long-lived chunk
// mappings).  A group whose every source lies inside one of them skips the
// staging copy: the DMA engine reads the caller's pages directly.  Batches
// hold the registry shared for their whole run (so a range cannot be
// unregistered under queued DMAs); register/unregister take it exclusively.
std::shared_mutex g_reg_mu;
std::vector<std::pair<uintptr_t, size_t>> g_reg;   // (start, length)

bool in_registered(const uint8_t *p, uint64_t len)
{
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    for (const auto &r : g_reg) {
        if (a >= r.first && a + len <= r.first + r.second) {
            return true;
        }
    }
    return false;
}

bool group_registered(const HostGroup &g)
{
    if (g_reg.empty() || !g.fd.empty()) {
        return false;
    }
    for (size_t k = 0; k < g.src.size(); k++) {
        if (g.lens[k] && !in_registered(g.src[k], g.lens[k])) {
            return false;
        }
    }
    return true;
}

// Direct DMAs of a registered group into the slot's device buffer, one per
// run of chunks that are adjacent both in host memory and in the group.
hipError_t dma_registered(const HostGroup &g, uint8_t *dbuf, hipStream_t stream)
{
    size_t k = 0;
    while (k < g.src.size()) {
        if (g.lens[k] == 0) {
            k++;
            continue;
        }
        const uint8_t *src = g.src[k];
        const uint64_t at = g.offs[k];
        uint64_t len = g.lens[k];
        size_t j = k + 1;
        while (j < g.src.size() && g.src[j] == src + len && g.offs[j] == at + len) {
            len += g.lens[j];
            j++;
        }
        const hipError_t e = hipMemcpyAsync(dbuf + at, src, len, hipMemcpyHostToDevice, stream);
        if (e != hipSuccess) {
            return e;
        }
        k = j;
    }
    return hipSuccess;
}

// The host legs of host batches, for cio_gpu_pipe_last_timing(): the calling
// thread's own last single-device batch, and the last one any thread
// finished (what a *_multi caller sees: its devices run on internal threads,
// so the record is the device pipeline that finished last).
struct PipeTiming {
    double total_ms = 0, copy_ms = 0, slot_wait_ms = 0, plan_ms = 0, groups = 0, bytes = 0;
    bool valid = false;
};
std::mutex g_timing_mu;
PipeTiming g_last_timing;
thread_local PipeTiming t_last_timing;

double wall_s()
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double) t.tv_sec + (double) t.tv_nsec * 1e-9;
}

// The single-device host batch on the calling thread's current device.
// Sources are bufs[i] (host memory), or file ranges (fds[i], foffs[i]) when
// fds is given.
int batch_host_current(const void *const *bufs, const int *fds, const uint64_t *foffs, const size_t *lens,
                       const uint32_t *seeds, uint32_t *out_raw, size_t n)
{
    DeviceState *st;
    if (device_state(&st) != CIO_OK) {
        return CIO_ERROR;
    }
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev), "hipGetDevice");
    // Groups of <= kStage bytes, 16-byte aligned segment placement.  The
    // first groups are smaller (first_stage_bytes(), doubling up to kStage):
    // the DMA engine starts after a short copy instead of a full slot's.
    std::vector<HostGroup> groups(1);
    uint64_t cap = std::min<uint64_t>(first_stage_bytes(), kStage);
    for (size_t i = 0; i < n; i++) {
        const uint8_t *p = fds ? nullptr : reinterpret_cast<const uint8_t *>(bufs[i]);
        uint64_t left = lens[i], done = 0;
        do {
            HostGroup *g = &groups.back();
            uint64_t at = (g->bytes + 15) & ~15ull;
            if (at >= cap) {
                groups.emplace_back();
                g = &groups.back();
                at = 0;
                cap = std::min<uint64_t>(cap * 2, kStage);
            }
            const uint64_t take = std::min<uint64_t>(left, cap - at);
            if (fds) {
                g->fd.push_back(fds[i]);
                g->foff.push_back(foffs[i] + done);
            }
            g->src.push_back(p ? p + done : nullptr);
            g->offs.push_back(at);
            g->lens.push_back(take);
            g->cid.push_back((uint32_t) i);
            g->bytes = at + take;
            left -= take;
            done += take;
        } while (left > 0);
    }

    HostPipe *hp = nullptr;
    hipError_t e = pipe_acquire(dev, &hp);
    if (e != hipSuccess) {
        return fail("cio_crc32_batch_host: device", e);
    }
    struct Release {
        int dev;
        HostPipe *hp;
        ~Release() { pipe_release(dev, hp); }
    } release{dev, hp};
    if (!hp->ready && (e = pipe_init(*hp, dev)) != hipSuccess) {
        return fail("cio_crc32_batch_host: pipeline setup", e);
    }
    std::vector<uint32_t> init(n);
    for (size_t i = 0; i < n; i++) {
        init[i] = seeds ? seeds[i] : 0xffffffffu;
    }
    PipeSlot &s0 = hp->slot[0];
    // Every slot is idle between calls (the previous call synchronised them).
    e = grow_dev(&hp->state, &hp->state_cap, n, false, s0.stream);
    if (e == hipSuccess) {
        // Ordered before every kernel: group 0 runs on slot 0's stream after
        // it, and each later group's kernel waits for the previous one's.
        // (init outlives the call's final synchronisation.)
        e = hipMemcpyAsync(hp->state, init.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice, s0.stream);
    }
    std::shared_lock<std::shared_mutex> rlk(g_reg_mu);
    int rc = CIO_OK;
    hipEvent_t prev = nullptr;
    // Per-call breakdown, kept for cio_gpu_pipe_last_timing() (a few clock
    // reads per group); CIO_GPU_PIPE_TIMING=1 also prints it on stderr.
    static const bool print_timing = getenv("CIO_GPU_PIPE_TIMING") != nullptr;
    constexpr bool timing = true;
    double t_copy = 0, t_wait = 0, t_plan = 0;
    const double t_start = wall_s();
    for (size_t gi = 0; gi < groups.size() && e == hipSuccess && rc == CIO_OK; gi++) {
        PipeSlot &s = hp->slot[gi % kSlots];
        const HostGroup &g = groups[gi];
        const bool direct = group_registered(g);
        double t = timing ? wall_s() : 0;
        if (s.busy) {
            // The slot's previous group (gi - kSlots) must be fully done.
            if ((e = hipEventSynchronize(s.done)) != hipSuccess) break;
            s.busy = false;
        }
        if (timing) {
            t_wait += wall_s() - t;
        }
        cio_crc32_plan view;
        uint32_t *d_cid = nullptr;
        size_t meta_bytes = 0;
        const char *err = nullptr;
        // the group's plan (host image into the slot's pinned arena)
        auto build = [&] {
            const double tp = timing ? wall_s() : 0;
            e = stage_plan(*hp, s, g, st, view, &d_cid, &meta_bytes, &err);
            if (timing) {
                t_plan += wall_s() - tp;
            }
        };
        if (direct) {
            // The data DMA needs no plan: queue it first and build the plan
            // while the engine moves the group (the plan only has to precede
            // the metadata copy and the kernel on this stream).
            if ((e = dma_registered(g, s.dbuf, s.stream)) != hipSuccess) break;
            build();
        } else {
            // staged: the plan is built while the copy workers fill the slot
            const double tc = timing ? wall_s() : 0;
            if (!hp->pool->copy(s.pinned, g, build)) {
                rc = fail("cio_crc32_batch: short read from a file source");
                break;
            }
            if (timing) {
                t_copy += wall_s() - tc;
            }
        }
        if (e != hipSuccess) break;
        if (err) {
            rc = fail(err);
            break;
        }
        if ((e = hipMemcpyAsync(s.meta_d, s.meta_h, meta_bytes, hipMemcpyHostToDevice, s.stream)) != hipSuccess) break;
        if (!direct) {
            if ((e = hipMemcpyAsync(s.dbuf, s.pinned, g.bytes, hipMemcpyHostToDevice, s.stream)) != hipSuccess) break;
        }
        if (prev && (e = hipStreamWaitEvent(s.stream, prev, 0)) != hipSuccess) break;   // chained states
        if (plan_exec_impl(&view, s.dbuf, hp->state, hp->state, d_cid, s.stream) != CIO_OK) {
            rc = CIO_ERROR;
            break;
        }
        if ((e = hipEventRecord(s.done, s.stream)) != hipSuccess) break;
        s.busy = true;
        prev = s.done;
    }
    for (int b = 0; b < kSlots; b++) {
        PipeSlot &s = hp->slot[b];
        const hipError_t e2 = hipStreamSynchronize(s.stream);
        if (e == hipSuccess) {
            e = e2;
        }
        s.busy = false;
    }
    if (e == hipSuccess && rc == CIO_OK) {
        e = hipMemcpy(out_raw, hp->state, n * sizeof(uint32_t), hipMemcpyDeviceToHost);
    }
    {
        uint64_t total = 0;
        for (const auto &g : groups) {
            total += g.bytes;
        }
        PipeTiming &pt = t_last_timing;
        pt.total_ms = (wall_s() - t_start) * 1e3;
        pt.copy_ms = t_copy * 1e3;
        pt.slot_wait_ms = t_wait * 1e3;
        pt.plan_ms = t_plan * 1e3;
        pt.groups = (double) groups.size();
        pt.bytes = (double) total;
        pt.valid = true;
        if (print_timing) {
            fprintf(stderr, "batch_host: dev %d, %zu chunks, %zu groups, %.1f MB: total %.2f ms, copy %.2f ms, "
                            "slot waits %.2f ms, plans %.2f ms\n", dev, n, groups.size(), total / 1e6,
                    pt.total_ms, pt.copy_ms, pt.slot_wait_ms, pt.plan_ms);
        }
        std::lock_guard<std::mutex> lk(g_timing_mu);
        g_last_timing = pt;
    }
    if (e != hipSuccess) {
        return fail("cio_crc32_batch_host", e);
    }
    return rc;
}

// Runs fn with `dev` as the calling thread's current device and restores the
// previous one afterwards.
template <typename F>
int on_device(int dev, F fn)
{
    int prev = 0;
    HIP_TRY(hipGetDevice(&prev), "hipGetDevice");
    if (prev != dev) {
        HIP_TRY(hipSetDevice(dev), "hipSetDevice");
    }
    const int rc = fn();
    if (prev != dev) {
        (void) hipSetDevice(prev);
    }
    return rc;
}

}  // namespace

extern "C" int cio_crc32_host_register(const void *p, size_t len)
{
    if (!p || len == 0) {
        return fail("cio_crc32_host_register: empty range");
    }
    DeviceState *st;
    if (device_state(&st) != CIO_OK) {
        return CIO_ERROR;
    }
    std::unique_lock<std::shared_mutex> lk(g_reg_mu);
    for (const auto &r : g_reg) {
        if (r.first == reinterpret_cast<uintptr_t>(p)) {
            return fail("cio_crc32_host_register: already registered");
        }
    }
    // Portable: the pinned range is DMA-able by every device of the process,
    // so multi-device batches take the direct path for it too.
    const hipError_t e = hipHostRegister(const_cast<void *>(p), len, hipHostRegisterPortable);
    if (e != hipSuccess) {
        return fail("cio_crc32_host_register", e);
    }
    g_reg.emplace_back(reinterpret_cast<uintptr_t>(p), len);
    return CIO_OK;
}

extern "C" int cio_crc32_host_unregister(const void *p)
{
    std::unique_lock<std::shared_mutex> lk(g_reg_mu);
    for (size_t i = 0; i < g_reg.size(); i++) {
        if (g_reg[i].first == reinterpret_cast<uintptr_t>(p)) {
            const hipError_t e = hipHostUnregister(const_cast<void *>(p));
            g_reg.erase(g_reg.begin() + (long) i);
            return e == hipSuccess ? CIO_OK : fail("cio_crc32_host_unregister", e);
        }
    }
    return fail("cio_crc32_host_unregister: not registered");
}

extern "C" int cio_crc32_batch_host(const void *const *bufs, const size_t *lens, const uint32_t *seeds,
                                    uint32_t *out_raw, size_t n)
{
    if (n == 0) {
        return CIO_OK;
    }
    if (!bufs || !lens || !out_raw) {
        return fail("cio_crc32_batch_host: null argument");
    }
    if (n >= 0xffffffffull) {
        return fail("cio_crc32_batch_host: too many chunks");
    }
    return batch_host_current(bufs, nullptr, nullptr, lens, seeds, out_raw, n);
}

namespace {

// Chunk i -> devices[i % G]: one host thread per device entry, each with its
// own pipeline, stream and device buffers; no collective, results are
// scattered back by chunk index.
int batch_multi(const void *const *bufs, const int *fds, const uint64_t *foffs, const size_t *lens,
                const uint32_t *seeds, uint32_t *out_raw, size_t n, const int *devices, int ndev,
                const char *what)
{
    if (ndev <= 0) {
        return batch_host_current(bufs, fds, foffs, lens, seeds, out_raw, n);
    }
    int visible = 0;
    HIP_TRY(hipGetDeviceCount(&visible), "hipGetDeviceCount");
    for (int d = 0; d < ndev; d++) {
        if (devices[d] < 0 || devices[d] >= visible || devices[d] >= kMaxDev) {
            return cioa_fail_msg(what, "device ordinal out of range");
        }
    }
    const int G = (int) std::min<size_t>((size_t) ndev, n);
    if (G == 1) {
        return on_device(devices[0], [&] {
            return batch_host_current(bufs, fds, foffs, lens, seeds, out_raw, n);
        });
    }
    std::vector<int> rcs(G, CIO_OK);
    std::vector<std::string> errs(G);
    std::vector<std::thread> th;
    th.reserve(G);
    for (int d = 0; d < G; d++) {
        th.emplace_back([&, d]() {
            std::vector<const void *> b;
            std::vector<int> f;
            std::vector<uint64_t> fo;
            std::vector<size_t> l;
            std::vector<uint32_t> sd, o;
            for (size_t i = (size_t) d; i < n; i += (size_t) G) {
                if (fds) {
                    f.push_back(fds[i]);
                    fo.push_back(foffs[i]);
                } else {
                    b.push_back(bufs[i]);
                }
                l.push_back(lens[i]);
                if (seeds) {
                    sd.push_back(seeds[i]);
                }
            }
            o.resize(l.size());
            if (hipSetDevice(devices[d]) != hipSuccess) {
                rcs[d] = CIO_ERROR;
                errs[d] = "hipSetDevice";
                return;
            }
            rcs[d] = batch_host_current(fds ? nullptr : b.data(), fds ? f.data() : nullptr,
                                        fds ? fo.data() : nullptr, l.data(), seeds ? sd.data() : nullptr,
                                        o.data(), l.size());
            if (rcs[d] != CIO_OK) {
                errs[d] = g_err;
                return;
            }
            size_t k = 0;
            for (size_t i = (size_t) d; i < n; i += (size_t) G) {
                out_raw[i] = o[k++];
            }
        });
    }
    for (auto &t : th) {
        t.join();
    }
    for (int d = 0; d < G; d++) {
        if (rcs[d] != CIO_OK) {
            char msg[96];
            snprintf(msg, sizeof(msg), "%s: device %d", what, devices[d]);
            return cioa_fail_msg(msg, errs[d].c_str());
        }
    }
    return CIO_OK;
}

}  // namespace

extern "C" int cio_crc32_batch_fd_multi(const int *fds, const uint64_t *foffs, const size_t *lens,
                                        const uint32_t *seeds, uint32_t *out_raw, size_t n,
                                        const int *devices, int ndev)
{
    if (n == 0) {
        return CIO_OK;
    }
    if (!fds || !foffs || !lens || !out_raw || (ndev > 0 && !devices)) {
        return fail("cio_crc32_batch_fd_multi: null argument");
    }
    if (n >= 0xffffffffull) {
        return fail("cio_crc32_batch_fd_multi: too many chunks");
    }
    return batch_multi(nullptr, fds, foffs, lens, seeds, out_raw, n, devices, ndev, "cio_crc32_batch_fd_multi");
}

extern "C" int cio_crc32_batch_host_multi(const void *const *bufs, const size_t *lens, const uint32_t *seeds,
                                          uint32_t *out_raw, size_t n, const int *devices, int ndev)
{
    if (n == 0) {
        return CIO_OK;
    }
    if (!bufs || !lens || !out_raw || (ndev > 0 && !devices)) {
        return fail("cio_crc32_batch_host_multi: null argument");
    }
    if (n >= 0xffffffffull) {
        return fail("cio_crc32_batch_host_multi: too many chunks");
    }
    return batch_multi(bufs, nullptr, nullptr, lens, seeds, out_raw, n, devices, ndev,
                       "cio_crc32_batch_host_multi");
}

extern "C" int cio_crc32_split_host_multi(const void *buf, size_t len, uint32_t seed, uint32_t *out_raw,
                                          const int *devices, int ndev)
{
    if (!out_raw || (len && !buf) || (ndev > 0 && !devices)) {
        return fail("cio_crc32_split_host_multi: null argument");
    }
    if (len == 0) {
        *out_raw = seed;
        return CIO_OK;
    }
    const size_t G = ndev > 0 ? (size_t) ndev : 1;
    // pieces of a 4 KiB multiple (whole wave-steps on each device), the last short
    const size_t piece = std::max<size_t>(4096, ((len + G - 1) / G + 4095) & ~(size_t) 4095);
    std::vector<const void *> bufs;
    std::vector<size_t> lens;
    std::vector<uint32_t> seeds, out;
    for (size_t at = 0; at < len; at += piece) {
        bufs.push_back(static_cast<const uint8_t *>(buf) + at);
        lens.push_back(std::min(piece, len - at));
        seeds.push_back(at == 0 ? seed : 0u);
    }
    out.resize(bufs.size());
    const int rc = cio_crc32_batch_host_multi(bufs.data(), lens.data(), seeds.data(), out.data(), bufs.size(),
                                              ndev > 0 ? devices : nullptr, ndev > 0 ? (int) std::min(G, bufs.size()) : 0);
    if (rc != CIO_OK) {
        return rc;
    }
    uint32_t acc = out[0];
    for (size_t i = 1; i < out.size(); i++) {
        acc = cio_crc32_combine(acc, out[i], lens[i]);
    }
    *out_raw = acc;
    return CIO_OK;
}

/* Diagnostic (not in the public header): the H2D DMA rate from `host`
 * (pinned, registered or pageable) into a device buffer, `reps` copies of
 * `bytes` on one stream; GB/s, or a negative value on error.  bench.py puts
 * it beside the registered-in-place E2E rate: registration pins the
 * caller's own (4 KiB) pages, and the engine's rate from them is the
 * registered path's real ceiling. */
extern "C" double cioa_debug_h2d_gbps(const void *host, size_t bytes, int reps)
{
    void *d = nullptr;
    hipStream_t s = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    double r = -1.0;
    if (!host || bytes == 0 || reps <= 0 || hipMalloc(&d, bytes) != hipSuccess) {
        return -1.0;
    }
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess &&
        hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess &&
        hipMemcpyAsync(d, host, bytes, hipMemcpyHostToDevice, s) == hipSuccess &&
        hipStreamSynchronize(s) == hipSuccess && hipEventRecord(e0, s) == hipSuccess) {
        bool ok = true;
        for (int i = 0; i < reps && ok; i++) {
            ok = hipMemcpyAsync(d, host, bytes, hipMemcpyHostToDevice, s) == hipSuccess;
        }
        float ms = 0.f;
        if (ok && hipEventRecord(e1, s) == hipSuccess && hipEventSynchronize(e1) == hipSuccess &&
            hipEventElapsedTime(&ms, e0, e1) == hipSuccess && ms > 0.f) {
            r = (double) bytes * reps / (ms * 1e-3) / 1e9;
        }
    }
    if (e0) (void) hipEventDestroy(e0);
    if (e1) (void) hipEventDestroy(e1);
    if (s) (void) hipStreamDestroy(s);
    (void) hipFree(d);
    return r;
}

// The split route (crc_route.c) runs the GPU part on a helper thread and
// hands its record to the calling thread, so cio_gpu_pipe_last_timing there
// reports that part.
extern "C" void cioa_pipe_timing_set(const double *v)
{
    PipeTiming pt;
    pt.total_ms = v[0];
    pt.copy_ms = v[1];
    pt.slot_wait_ms = v[2];
    pt.plan_ms = v[3];
    pt.groups = v[4];
    pt.bytes = v[5];
    pt.valid = true;
    t_last_timing = pt;
}

extern "C" int cio_gpu_pipe_last_timing(double *out, int n)
{
    if (!out || n <= 0) {
        return fail("cio_gpu_pipe_last_timing: null argument");
    }
    PipeTiming pt = t_last_timing;
    if (!pt.valid) {
        std::lock_guard<std::mutex> lk(g_timing_mu);
        pt = g_last_timing;
    }
    const double v[6] = {pt.total_ms, pt.copy_ms, pt.slot_wait_ms, pt.plan_ms, pt.groups, pt.bytes};
    for (int i = 0; i < n && i < 6; i++) {
        out[i] = v[i];
    }
    return CIO_OK;
}

extern "C" int cio_gpu_plan_cache_stats(uint64_t *out, int n)
{
    if (!out) {
        return cioa::fail("cio_gpu_plan_cache_stats: null pointer");
    }
    uint64_t v[7] = {0, 0, 0, 0, 0, 0, 0};
    for (int d = 0; d < kMaxDev; d++) {
        DevPipes &dp = g_pipes[d];
        std::lock_guard<std::mutex> lk(dp.mu);
        for (const HostPipe *hp : dp.idle) {
            v[0] += hp->plans.size();
            v[1] += hp->plan_bytes;
            v[2] += hp->hits;
            v[3] += hp->misses;
            v[4] += hp->stores;
            v[5] += hp->evictions;
            v[6] += 1;
        }
    }
    for (int i = 0; i < n && i < 7; i++) {
        out[i] = v[i];
    }
    return CIO_OK;
}

extern "C" int cio_gpu_numa_node(int dev)
{
    int node = -1;
    (void) device_local_cpus(dev, &node);
    return node;
}

extern "C" int cio_gpu_pci_bus_id(int dev, char *buf, int len)
{
    if (!buf || len < 13) {
        return cioa::fail("cio_gpu_pci_bus_id: buffer shorter than 13 bytes");
    }
    HIP_TRY(hipDeviceGetPCIBusId(buf, len, dev), "hipDeviceGetPCIBusId");
    return CIO_OK;
}

extern "C" int cio_gpu_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        return 0;
    }
    return n;
}

extern "C" int cio_gpu_set_device(int dev)
{
    HIP_TRY(hipSetDevice(dev), "hipSetDevice");
    return CIO_OK;
}

extern "C" int cio_gpu_get_device(void)
{
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess) {
        return -1;
    }
    return dev;
}
