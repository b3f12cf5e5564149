// rc4_hooks_device.cpp -- the gfx950 Rc4Hooks (include/zsummerx_amd/rc4_hooks.h)
// over the C-ABI of libzrc4.so (include/zrc4.h).
//
// Memory ("pinned SessionBlock pool"): every SessionBlock
// slab is pinned host memory (hipHostMalloc) that the kernels read and write
// in place -- no staging copies and no per-session calls.  The batch tables
// (slot ids, offsets, lengths, keys) are pinned too.  Payload addressing:
// kernels take one base pointer and 64-bit per-entry offsets; the base is the
// first pinned allocation and an entry's offset is its address minus the base
// in two's complement, so slabs anywhere in the address space share one launch.
//
// Every launch is a zrc4_crypt_grouped_declared batch (the groups built here
// are declared with it): entries sorted by slot, one
// 256-entry bucket per 256-slot group touched, so each bucket moves its
// group's S-boxes as one coalesced 64 KiB image whatever subset of the group
// the iteration touches (the kIds gather path is never used here).
//
// Two modes:
//   direct     one grouped launch per engine iteration over the spans
//              themselves, then a wait.  A span's latency is its serial RC4
//              chain: ~40 ns per byte on one lane (rc4_encryption.h:83-88 is
//              byte-serial), so small batches wait on the chain.
//   reservoir  (default) RC4's keystream does not depend on the data, so each
//              slot's keystream is generated AHEAD by the GPU -- a background
//              stream runs zrc4_crypt over the slot's ring bytes (kept zero:
//              0 ^ k = k) -- into a ring of `ring` bytes in PINNED HOST memory
//              (written over PCIe by the kernel).  The hook then XORs each
//              span with committed ring bytes on the host: no GPU round trip
//              on the latency path.  Only a slot whose committed keystream
//              does not cover its span goes to the GPU synchronously, and only
//              for the missing tail (the slot's state sits exactly at the end
//              of its committed keystream).  The RC4 state never leaves the
//              device; keystream bytes are consumed strictly in order, so the
//              wire bytes are the reference's.
// Ordering rules (streams: A = synchronous work, B = background refill):
//   * the host reads only ring bytes of COMMITTED refills (their event has
//     completed), and zeroes them as it consumes them; a refill writes only
//     ring bytes past the committed end -- the two never touch the same bytes;
//   * kernels that touch slot state (ksa, tail crypt, refill) never run on A
//     and B at once: a grouped kernel stores its whole group image, so A
//     waits for every queued refill on B before a seed or a tail crypt;
//   * refills on B run in stream order, at most kRefillDepth queued.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "zrc4.h"
#include "zsummerx_amd/rc4_hooks.h"

namespace zsummerx_amd {
namespace {

// Pinned host allocations shared with the kernels (blocks, rings, batch
// tables) are COHERENT (fine-grained).  HIP dispatches kernels with
// agent-scope acquire/release, so a kernel can hit lines of NON-coherent host
// memory still held in the GPU L2 from an earlier kernel after the host has
// rewritten them (stale batch tables, SessionBlocks, zeroed ring bytes): the
// hooks_check run at 2 048 sessions failed that way with hipHostMallocDefault
// (profiles/r02/hooks_diag.jsonl).  Diagnostic knob:
// ZSX_HOST_ALLOC=coherent|noncoherent|default.
unsigned hostAllocFlags()
{
    static const unsigned f = [] {
        const char *e = std::getenv("ZSX_HOST_ALLOC");
        if (!e) return (unsigned)hipHostMallocCoherent;
        if (!std::strcmp(e, "default")) return (unsigned)hipHostMallocDefault;
        if (!std::strcmp(e, "coherent")) return (unsigned)hipHostMallocCoherent;
        if (!std::strcmp(e, "noncoherent")) return (unsigned)hipHostMallocNonCoherent;
        return (unsigned)hipHostMallocCoherent;
    }();
    return f;
}

template <class T>
struct PinnedArray {
    T *p = nullptr;
    size_t cap = 0;
    void reserve(size_t n)
    {
        if (n <= cap) return;
        size_t c = cap ? cap : 1024;
        while (c < n) c *= 2;
        T *q = nullptr;
        if (hipHostMalloc(reinterpret_cast<void **>(&q), c * sizeof(T), hostAllocFlags()) != hipSuccess)
            throw std::bad_alloc();
        if (p) {
            std::memcpy(q, p, cap * sizeof(T));   // keep the entries already pushed
            (void)hipHostFree(p);
        }
        p = q;
        cap = c;
    }
    ~PinnedArray()
    {
        if (p) (void)hipHostFree(p);
    }
};

// One grouped batch table (ids / offsets / lengths) in pinned memory.
struct Table {
    PinnedArray<uint32_t> ids, len;
    PinnedArray<uint64_t> off;
    std::vector<uint32_t> groups;   // each bucket's group, declared to zrc4_crypt_grouped_declared
    uint32_t n = 0;
    void clear()
    {
        n = 0;
        groups.clear();
    }
    void push(uint32_t id, uint64_t o, uint32_t l)
    {
        if (n == ids.cap || n == off.cap || n == len.cap) {
            ids.reserve(n + 1);
            off.reserve(n + 1);
            len.reserve(n + 1);
        }
        ids.p[n] = id;
        off.p[n] = o;
        len.p[n] = l;
        ++n;
    }
};

// A grouped launch over table t: the groups built here are declared with it
// up to 256 buckets, where the kernels take them in their arguments and load
// each bucket's state with its entries; above that the persistent kernel
// prefetches every bucket's ids a bucket ahead anyway, and a declaration
// would only add the library's up-front check (include/zrc4.h).
int launchGrouped(zrc4_ctx *ctx, const Table &t, uint8_t *base, const zrc4_frame_args *fa, hipStream_t s)
{
    if (t.groups.size() <= 256u)
        return zrc4_crypt_grouped_declared(ctx, t.ids.p, t.groups.data(), base, t.off.p, t.len.p, t.n, fa, s);
    return fa ? zrc4_crypt_grouped_frame(ctx, t.ids.p, base, t.off.p, t.len.p, t.n, fa, s)
              : zrc4_crypt_grouped(ctx, t.ids.p, base, t.off.p, t.len.p, t.n, s);
}

struct Entry {
    uint32_t slot;
    uint32_t len;
    uint64_t off;
    uint32_t idx = 0;     // the caller's span index (framed calls)
    uint32_t flen = 0;    // frame block length (framed calls)
    uint64_t foff = 0;    // frame block offset from the base (framed calls)
};

// Per-entry framing tables of a framed grouped launch (pinned).
struct FrameTable {
    PinnedArray<uint64_t> off;
    PinnedArray<uint32_t> len, npk, used, status, pkt;
    std::vector<int64_t> idx;   // batch entry -> span index (-1: padding)
    void reserve(size_t n)
    {
        off.reserve(n);
        len.reserve(n);
        npk.reserve(n);
        used.reserve(n);
        status.reserve(n);
        pkt.reserve(n * Rc4Frame::kMaxPackets);
    }
};

// zrc4_crypt_grouped layout: entries sorted by slot, a new 256-entry bucket
// at every group change (each group holds at most 256 distinct slots, so one
// bucket per group).
void buildGrouped(Table &t, std::vector<Entry> &es, FrameTable *ft = nullptr)
{
    std::sort(es.begin(), es.end(), [](const Entry &a, const Entry &b) { return a.slot < b.slot; });
    t.clear();
    if (ft) ft->idx.clear();
    auto push = [&](uint32_t slot, uint64_t off, uint32_t len, const Entry *e) {
        t.push(slot, off, len);
        if (ft) {
            ft->reserve(t.n);
            ft->off.p[t.n - 1] = e ? e->foff : 0;
            ft->len.p[t.n - 1] = e ? e->flen : 0;
            ft->idx.push_back(e ? (int64_t)e->idx : -1);
        }
    };
    uint32_t cur = ZRC4_IDLE_SLOT;
    for (const Entry &e : es) {
        const uint32_t g = e.slot >> 8;
        if (g != cur) {
            while (t.n % ZRC4_GROUP_SLOTS) push(ZRC4_IDLE_SLOT, 0, 0, nullptr);
            cur = g;
            t.groups.push_back(g);
        }
        push(e.slot, e.off, e.len, &e);
    }
}

struct Level {
    uint64_t gen = 0;    // keystream bytes generated and committed (absolute stream position)
    uint64_t use = 0;    // keystream bytes consumed
    uint64_t pend = 0;   // end of the last queued refill (== gen when none is in flight)
};

// One background refill launch: its grouped table, its completion event and
// the (slot, end position) pairs it commits.
struct Refill {
    Table t;
    hipEvent_t ev = nullptr;
    std::vector<std::pair<uint32_t, uint64_t>> ends;
};

// dst ^= src for n bytes, then src = 0 (word-wise where possible).
void xorAndClear(uint8_t *__restrict dst, uint8_t *__restrict src, size_t n)
{
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t a, b;
        std::memcpy(&a, dst + i, 8);
        std::memcpy(&b, src + i, 8);
        a ^= b;
        std::memcpy(dst + i, &a, 8);
    }
    for (; i < n; ++i) dst[i] ^= src[i];
    std::memset(src, 0, n);
}

// One piece of a reservoir call's host work: span bytes ^= committed ring
// bytes, ring bytes = 0.
struct XorJob {
    uint8_t *dst;
    uint8_t *src;
    uint32_t n;
};

// The reservoir's host XOR for large batches, spread over worker threads.
// At 2 048 sessions x 2 in flight one call XORs 4 MiB (4 096 spans) and the
// event loop spends ~1 ms in it on one core (profiles/r02/frame_loopback_v2.jsonl:
// 975 us per call, slower than the direct GPU path).  Only the keystream XOR
// is parallel: keystream generation stays on the GPU, and every piece of
// bookkeeping stays on the calling thread.  Threads: $ZSX_XOR_THREADS
// (default min(4, hardware threads / 2); 0 or 1 = inline); batches under
// $ZSX_XOR_MIN_BYTES (default kParallelBytes) run inline.
class XorPool {
public:
    static constexpr size_t kParallelBytes = 256u << 10;

    XorPool()
    {
        if (const char *m = std::getenv("ZSX_XOR_MIN_BYTES")) minBytes_ = (size_t)std::strtoull(m, nullptr, 10);
        const char *e = std::getenv("ZSX_XOR_THREADS");
        unsigned hw = std::thread::hardware_concurrency();
        unsigned t = e ? (unsigned)std::atoi(e) : std::min(4u, hw / 2u);
        workers_ = t > 1u ? t - 1u : 0u;          // the calling thread is one of them
        for (unsigned i = 0; i < workers_; ++i) threads_.emplace_back([this, i] { loop(i + 1u); });
    }
    ~XorPool()
    {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
            ++gen_;
        }
        cv_.notify_all();
        for (std::thread &t : threads_) t.join();
    }
    unsigned threads() const { return workers_ + 1u; }

    void run(const std::vector<XorJob> &jobs, size_t bytes)
    {
        if (!workers_ || bytes < minBytes_ || jobs.size() < 2) {
            for (const XorJob &j : jobs) xorAndClear(j.dst, j.src, j.n);
            return;
        }
        // contiguous job ranges of about equal bytes, one per thread
        const unsigned parts = workers_ + 1u;
        bounds_.assign(parts + 1u, jobs.size());
        bounds_[0] = 0;
        size_t acc = 0, k = 1;
        for (size_t i = 0; i < jobs.size() && k < parts; ++i) {
            acc += jobs[i].n;
            if (acc * parts >= bytes * k) bounds_[k++] = i + 1;
        }
        jobs_ = &jobs;
        pending_.store(workers_, std::memory_order_relaxed);
        {
            std::lock_guard<std::mutex> g(mu_);
            ++gen_;
        }
        cv_.notify_all();
        work(0);
        while (pending_.load(std::memory_order_acquire) != 0) std::this_thread::yield();
    }

private:
    void work(unsigned part)
    {
        const std::vector<XorJob> &jobs = *jobs_;
        for (size_t i = bounds_[part]; i < bounds_[part + 1]; ++i) xorAndClear(jobs[i].dst, jobs[i].src, jobs[i].n);
    }
    void loop(unsigned part)
    {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> l(mu_);
                cv_.wait(l, [&] { return gen_ != seen; });
                seen = gen_;
                if (stop_) return;
            }
            work(part);
            pending_.fetch_sub(1, std::memory_order_release);
        }
    }
    unsigned workers_ = 0;
    size_t minBytes_ = kParallelBytes;
    std::vector<std::thread> threads_;
    std::mutex mu_;
    std::condition_variable cv_;
    uint64_t gen_ = 0;
    bool stop_ = false;
    const std::vector<XorJob> *jobs_ = nullptr;
    std::vector<size_t> bounds_;
    std::atomic<unsigned> pending_{0};
};

class DeviceRc4Hooks final : public Rc4Hooks {
public:
    DeviceRc4Hooks(int device, uint32_t capacity, uint32_t ringBytes) : ringCap_(ringBytes)
    {
        const int rc = zrc4_create(&ctx_, device, capacity);
        if (rc != ZRC4_OK)
            throw std::runtime_error(std::string("makeDeviceRc4Hooks: zrc4_create: ") + zrc4_strerror(rc));
        bool ok = hipSetDevice(device) == hipSuccess &&
                  hipStreamCreateWithFlags(&sA_, hipStreamNonBlocking) == hipSuccess &&
                  hipStreamCreateWithFlags(&sB_, hipStreamNonBlocking) == hipSuccess;
        for (Refill &r : refill_) ok = ok && hipEventCreateWithFlags(&r.ev, hipEventDisableTiming) == hipSuccess;
        if (!ok) {
            release();
            throw std::runtime_error("makeDeviceRc4Hooks: HIP stream/event creation failed");
        }
        seen_.assign(zrc4_capacity(ctx_), 0u);
        if (ringCap_) {
            level_.resize(zrc4_capacity(ctx_));
            ringSlab_.assign(zrc4_capacity(ctx_) / ZRC4_GROUP_SLOTS, nullptr);
            hungryMark_.assign(zrc4_capacity(ctx_), 0u);
            // $ZSX_REFILL_CHUNK (A/B knob): bytes per slot per refill, at most a
            // quarter of the ring (two refills in flight leave half of it readable)
            const char *rc = std::getenv("ZSX_REFILL_CHUNK");
            const uint32_t want = rc ? (uint32_t)std::strtoul(rc, nullptr, 10) : kRefillChunk;
            refillChunk_ = std::max<uint32_t>(256u, std::min<uint32_t>(want, ringCap_ / 4));
        }
    }
    ~DeviceRc4Hooks() override { release(); }

    const char *name() const override { return ringCap_ ? "zrc4-gfx950" : "zrc4-gfx950-direct"; }
    uint32_t capacity() const override { return zrc4_capacity(ctx_); }

    void *allocBlocks(size_t bytes) override
    {
        void *p = nullptr;
        if (hipHostMalloc(&p, bytes, hostAllocFlags()) != hipSuccess) throw std::bad_alloc();
        if (!base_) base_ = static_cast<uint8_t *>(p);
        return p;
    }
    void freeBlocks(void *p) override
    {
        if (p) (void)hipHostFree(p);
    }

    int seed(const uint32_t *slots, uint32_t n, const std::string &key) override
    {
        // Only the first 256 key bytes reach the S-box (rc4_encryption.h:60-70).
        const uint32_t kl = (uint32_t)std::min<size_t>(key.size(), 256);
        const uint64_t ko = keyBytes_.size();
        keyBytes_.insert(keyBytes_.end(), key.data(), key.data() + kl);
        for (uint32_t i = 0; i < n; ++i) {
            if (slots[i] >= capacity()) return ZRC4_ERR_SLOT_RANGE;
            seedIds_.push_back(slots[i]);
            seedOff_.push_back(ko);
            seedLen_.push_back(kl);
        }
        return ZRC4_OK;
    }

    int crypt(const Rc4Span *spans, uint32_t n) override
    {
        int rc = flushSeeds();
        if (rc != ZRC4_OK) return rc;
        if (n == 0) return ZRC4_OK;
        // Each slot at most once per call (rc4_hooks.h contract): a second span
        // of one slot would consume keystream the first already accounted for.
        if (++callStamp_ == 0) {
            std::fill(seen_.begin(), seen_.end(), 0u);
            callStamp_ = 1;
        }
        for (uint32_t i = 0; i < n; ++i) {
            const uint32_t s = spans[i].slot;
            if (s >= seen_.size() || seen_[s] == callStamp_) return ZRC4_ERR_INVALID_ARG;
            seen_[s] = callStamp_;
        }
        return ringCap_ ? cryptReservoir(spans, n) : cryptDirect(spans, n);
    }

    // Device framing rides on the direct mode's launch (the reservoir mode
    // decrypts on the host, so there is no device pass to fuse with).
    bool canFrame() const override { return ringCap_ == 0; }

    int cryptFrame(const Rc4Span *spans, uint32_t n, Rc4Frame *frames, uint32_t bound) override
    {
        if (ringCap_) return ZRC4_ERR_INVALID_ARG;
        int rc = flushSeeds();
        if (rc != ZRC4_OK) return rc;
        if (n == 0) return ZRC4_OK;
        if (++callStamp_ == 0) {
            std::fill(seen_.begin(), seen_.end(), 0u);
            callStamp_ = 1;
        }
        es_.clear();
        for (uint32_t i = 0; i < n; ++i) {
            const uint32_t s = spans[i].slot;
            if (s >= seen_.size() || seen_[s] == callStamp_) return ZRC4_ERR_INVALID_ARG;
            seen_[s] = callStamp_;
            Entry e{s, spans[i].len, offOf(spans[i].data)};
            e.idx = i;
            e.flen = frames[i].len;
            e.foff = frames[i].len ? offOf(frames[i].block) : 0;
            es_.push_back(e);
            tailBytes_ += spans[i].len;
        }
        buildGrouped(tt_, es_, &ft_);
        zrc4_frame_args fa{ft_.off.p, ft_.len.p, bound, Rc4Frame::kMaxPackets, ft_.npk.p, ft_.used.p,
                           ft_.status.p, ft_.pkt.p};
        rc = launchGrouped(ctx_, tt_, base_, &fa, sA_);
        if (rc != ZRC4_OK) return rc;
        ++tailLaunches_;
        if ((rc = zrc4_sync(ctx_, sA_)) != ZRC4_OK) return rc;
        for (uint32_t b = 0; b < tt_.n; ++b) {
            const int64_t i = ft_.idx[b];
            if (i < 0 || !frames[i].len) continue;
            Rc4Frame &f = frames[i];
            f.npk = ft_.npk.p[b];
            f.used = ft_.used.p[b];
            f.status = ft_.status.p[b];
            const uint32_t k = std::min(f.npk, Rc4Frame::kMaxPackets);
            std::memcpy(f.pkt, ft_.pkt.p + (size_t)b * Rc4Frame::kMaxPackets, k * sizeof(uint32_t));
            ++framed_;
        }
        return ZRC4_OK;
    }

    std::string stats() const override
    {
        char b[768];
        std::snprintf(b, sizeof b,
                      "{\"ring_bytes\": %llu, \"tail_bytes\": %llu, \"tail_launches\": %llu, "
                      "\"refill_bytes\": %llu, \"refill_launches\": %llu, \"refill_waits\": %llu, "
                      "\"ring_cap\": %u, \"refill_chunk\": %u, \"device_framed\": %llu, \"xor_threads\": %u, "
                      "\"direct_calls\": %llu, \"direct_bytes\": %llu}",
                      ringBytes_, tailBytes_, tailLaunches_, refillBytes_, refillLaunches_, refillWaits_, ringCap_,
                      refillChunk_, framed_, xor_.threads(), directCalls_, (unsigned long long)directBytes_);
        return b;
    }

private:
    uint64_t offOf(const void *p)
    {
        if (!base_) base_ = static_cast<uint8_t *>(const_cast<void *>(p));
        return (uint64_t)((uintptr_t)p - (uintptr_t)base_);
    }

    // The ring of slot s: pinned host memory, one slab of 256 rings per group,
    // allocated on first use and zeroed (the zero invariant of the refills).
    uint8_t *ringOf(uint32_t s)
    {
        uint8_t *&slab = ringSlab_[s / ZRC4_GROUP_SLOTS];
        if (!slab) {
            const size_t bytes = (size_t)ZRC4_GROUP_SLOTS * ringCap_;
            void *p = nullptr;
            if (hipHostMalloc(&p, bytes, hostAllocFlags()) != hipSuccess) throw std::bad_alloc();
            std::memset(p, 0, bytes);
            slab = static_cast<uint8_t *>(p);
        }
        return slab + (size_t)(s % ZRC4_GROUP_SLOTS) * ringCap_;
    }

    // One grouped launch on A over `es`, then the wait.
    int runTail(std::vector<Entry> &es)
    {
        if (es.empty()) return ZRC4_OK;
        buildGrouped(tt_, es);
        int rc = launchGrouped(ctx_, tt_, base_, nullptr, sA_);
        if (rc != ZRC4_OK) return rc;
        ++tailLaunches_;
        return zrc4_sync(ctx_, sA_);
    }

    int cryptDirect(const Rc4Span *spans, uint32_t n)
    {
        es_.clear();
        for (uint32_t i = 0; i < n; ++i)
            if (spans[i].len) es_.push_back({spans[i].slot, spans[i].len, offOf(spans[i].data)});
        for (const Entry &e : es_) tailBytes_ += e.len;
        return runTail(es_);
    }

    // Adaptive mode (r03).  The reservoir wins while an iteration is small
    // (a host XOR, no GPU round trip on the latency path); with megabytes per
    // iteration the host XOR of every span dominates and one grouped launch
    // over the spans in place (zero-copy pinned blocks) wins: 2048 x 2
    // sessions (~4 MB per call) 134k vs 172k echo/s, 512 x 4 (~1.8 MB) 210k vs
    // 223k, while 512 x 1 (~0.45 MB) runs 228k vs 212k the other way
    // (profiles/r02/frame_loopback_win_v17.jsonl).  So the hooks follow a
    // moving average of the bytes per call: at or above $ZSX_RC4_DIRECT_BYTES
    // (default 1 MiB; 0 = never) they stop refilling -- each slot drains
    // what its ring holds, then its spans go to the device as tails, which
    // is exactly the direct mode's launch -- and below half of it refills
    // resume.  The keystream order is the same either way.
    void updateMode(const Rc4Span *spans, uint32_t n)
    {
        uint64_t bytes = 0;
        for (uint32_t i = 0; i < n; ++i) bytes += spans[i].len;
        emaBytes_ = emaBytes_ == 0.0 ? (double)bytes : 0.875 * emaBytes_ + 0.125 * (double)bytes;
        if (directBytes_ && !direct_ && emaBytes_ >= (double)directBytes_) direct_ = true;
        else if (direct_ && emaBytes_ < 0.5 * (double)directBytes_) direct_ = false;
        if (direct_) ++directCalls_;
    }

    int cryptReservoir(const Rc4Span *spans, uint32_t n)
    {
        updateMode(spans, n);
        int rc = pollRefills(false);
        if (rc != ZRC4_OK) return rc;
        // A slot short of committed keystream while refills are queued: wait
        // for them in order until it is covered or none is left (their bytes
        // are the ones it needs, and a tail crypt may not run beside them).
        for (;;) {
            bool wait = false;
            for (uint32_t i = 0; i < n && !wait; ++i) {
                const Level &L = level_[spans[i].slot];
                if (L.gen - L.use < spans[i].len && L.pend > L.gen) wait = true;
            }
            if (!wait || !inFlight_) break;      // nothing queued: the span goes to the tail path
            ++refillWaits_;
            if ((rc = commitOldest(true)) != ZRC4_OK) return rc;
        }
        // Host XOR with the committed ring bytes (XorPool, after this pass:
        // before any refill is launched, since a refill may write the ring
        // bytes consumed here); collect the uncovered tails.
        es_.clear();
        xj_.clear();
        size_t xjBytes = 0;
        for (uint32_t i = 0; i < n; ++i) {
            const Rc4Span &sp = spans[i];
            if (!sp.len) continue;
            Level &L = level_[sp.slot];
            const uint32_t have = (uint32_t)std::min<uint64_t>(L.gen - L.use, sp.len);
            if (have) {
                uint8_t *r = ringOf(sp.slot);
                uint32_t done = 0;
                while (done < have) {
                    const uint32_t at = (uint32_t)((L.use + done) % ringCap_);
                    const uint32_t k = std::min(have - done, ringCap_ - at);
                    xj_.push_back({sp.data + done, r + at, k});
                    done += k;
                }
                L.use += have;
                ringBytes_ += have;
                xjBytes += have;
            }
            if (have < sp.len) {
                // the slot's device state is at position L.gen == L.use
                es_.push_back({sp.slot, sp.len - have, offOf(sp.data + have)});
                L.use += sp.len - have;
                L.gen = L.pend = L.use;
                tailBytes_ += sp.len - have;
            }
            if (!direct_ && !hungryMark_[sp.slot]) {
                hungryMark_[sp.slot] = 1;
                hungry_.push_back(sp.slot);
            }
        }
        xor_.run(xj_, xjBytes);
        if (!es_.empty()) {
            if ((rc = drainRefills()) != ZRC4_OK) return rc;     // slot state must be quiet
            if ((rc = runTail(es_)) != ZRC4_OK) return rc;
        }
        while (!direct_ && inFlight_ < refillDepth_) {
            const uint32_t before = inFlight_;
            if ((rc = launchRefill()) != ZRC4_OK) return rc;
            if (inFlight_ == before) break;
        }
        return ZRC4_OK;
    }

    // Background refill of the slots used since the last one, each up to a
    // full ring (counting what is already queued), in one piece of at most
    // refillChunk_ bytes per slot (one chunk's chain ~ refillChunk_ x 40 ns),
    // written straight into the pinned host rings.  Up to kRefillDepth
    // refills are queued back to back on stream B, so a stream's keystream
    // generation does not pause between launches (stream order keeps each
    // slot's pieces sequential).
    int launchRefill()
    {
        if (inFlight_ >= refillDepth_ || debugNoRefill_ || hungry_.empty()) return ZRC4_OK;
        Refill &R = refill_[(head_ + inFlight_) % kRefillDepth];
        rs_.clear();
        R.ends.clear();
        std::vector<uint32_t> keep;
        for (uint32_t s : hungry_) {
            Level &L = level_[s];
            const uint64_t level = L.pend - L.use;
            // Whole chunks only: a launch lasts as long as its longest piece
            // (one lane per slot), so every slot it carries gets a full chunk
            // (or the piece up to the ring end).  A slot without room for one
            // leaves the hungry list until it is consumed from again.
            if (ringCap_ - level < refillChunk_) {
                hungryMark_[s] = 0;
                continue;
            }
            const uint32_t at = (uint32_t)(L.pend % ringCap_);
            const uint32_t amt = std::min(ringCap_ - at, refillChunk_);
            rs_.push_back({s, amt, offOf(ringOf(s) + at)});
            L.pend += amt;
            R.ends.push_back({s, L.pend});
            keep.push_back(s);                      // re-examined at the next launch
        }
        hungry_.swap(keep);
        if (rs_.empty()) return ZRC4_OK;
        buildGrouped(R.t, rs_);
        int rc = launchGrouped(ctx_, R.t, base_, nullptr, sB_);
        if (rc != ZRC4_OK) {
            // nothing queued: the levels go back (pend > gen with no refill in
            // flight would make cryptReservoir wait for bytes that never come)
            for (const Entry &e : rs_) level_[e.slot].pend -= e.len;
            R.ends.clear();
            return rc;
        }
        ++refillLaunches_;
        if (hipEventRecord(R.ev, sB_) != hipSuccess) {
            // the refill is queued but cannot be tracked: wait for stream B
            // and commit its bytes now
            if (hipStreamSynchronize(sB_) != hipSuccess) return ZRC4_ERR_HIP;
            for (const auto &se : R.ends) {
                Level &L = level_[se.first];
                if (se.second > L.gen) {
                    refillBytes_ += se.second - L.gen;
                    L.gen = se.second;
                }
            }
            R.ends.clear();
            return zrc4_poll_faults(ctx_);
        }
        ++inFlight_;
        if (debugSyncRefill_) return drainRefills();
        return ZRC4_OK;
    }

    // Commit the oldest queued refill if it has finished (wait = block until
    // it has).  Refills complete in stream order.
    int commitOldest(bool wait)
    {
        if (!inFlight_) return ZRC4_OK;
        Refill &R = refill_[head_];
        if (wait) {
            if (hipEventSynchronize(R.ev) != hipSuccess) return ZRC4_ERR_HIP;
        } else {
            const hipError_t q = hipEventQuery(R.ev);
            if (q == hipErrorNotReady) return ZRC4_ERR_NOT_READY_;
            if (q != hipSuccess) return ZRC4_ERR_HIP;
        }
        for (const auto &se : R.ends) {
            Level &L = level_[se.first];
            if (se.second > L.gen) {
                refillBytes_ += se.second - L.gen;
                L.gen = se.second;
            }
        }
        R.ends.clear();
        head_ = (head_ + 1) % kRefillDepth;
        --inFlight_;
        return ZRC4_OK;
    }

    // Commit every finished refill (wait = every queued one), then report
    // latched device faults of stream B.
    int pollRefills(bool wait)
    {
        bool any = false;
        while (inFlight_) {
            const int rc = commitOldest(wait);
            if (rc == ZRC4_ERR_NOT_READY_) break;
            if (rc != ZRC4_OK) return rc;
            any = true;
        }
        // committed refills have completed: their faults are in the latch
        // (no stream wait -- a second queued refill keeps running)
        return any ? zrc4_poll_faults(ctx_) : ZRC4_OK;
    }
    int drainRefills() { return pollRefills(true); }

    // Queued makeSBox calls: one zrc4_ksa ahead of the hook work on A.  In
    // reservoir mode a reseeded slot's unconsumed keystream is dropped (its
    // ring bytes zeroed on the host) and its counters restart.
    int flushSeeds()
    {
        const uint32_t m = (uint32_t)seedIds_.size();
        if (m == 0) return ZRC4_OK;
        int rc;
        if (ringCap_) {
            if ((rc = drainRefills()) != ZRC4_OK) return rc;
            for (uint32_t s : seedIds_) {
                Level &L = level_[s];
                if (L.gen > L.use) {
                    uint8_t *r = ringOf(s);
                    for (uint64_t p = L.use; p < L.gen;) {
                        const uint32_t at = (uint32_t)(p % ringCap_);
                        const uint32_t k = (uint32_t)std::min<uint64_t>(L.gen - p, ringCap_ - at);
                        std::memset(r + at, 0, k);
                        p += k;
                    }
                }
                L = Level();
            }
        } else if ((rc = zrc4_sync(ctx_, sA_)) != ZRC4_OK) {
            return rc;
        }
        kIds_.reserve(m);
        kOff_.reserve(m);
        kLen_.reserve(m);
        kBytes_.reserve(std::max<size_t>(keyBytes_.size(), 1));
        std::memcpy(kIds_.p, seedIds_.data(), m * sizeof(uint32_t));
        std::memcpy(kOff_.p, seedOff_.data(), m * sizeof(uint64_t));
        std::memcpy(kLen_.p, seedLen_.data(), m * sizeof(uint32_t));
        if (!keyBytes_.empty()) std::memcpy(kBytes_.p, keyBytes_.data(), keyBytes_.size());
        seedIds_.clear();
        seedOff_.clear();
        seedLen_.clear();
        keyBytes_.clear();
        rc = zrc4_ksa(ctx_, kIds_.p, kBytes_.p, kOff_.p, kLen_.p, m, sA_);
        if (rc != ZRC4_OK) return rc;
        // The key tables are reused by the next flush: wait for this one (seeds
        // happen at connect / accept, not per packet).
        return zrc4_sync(ctx_, sA_);
    }

    void release()
    {
        if (sB_) (void)hipStreamSynchronize(sB_);
        if (sA_) (void)hipStreamSynchronize(sA_);
        for (Refill &r : refill_)
            if (r.ev) {
                (void)hipEventDestroy(r.ev);
                r.ev = nullptr;
            }
        if (sA_) (void)hipStreamDestroy(sA_);
        if (sB_) (void)hipStreamDestroy(sB_);
        for (uint8_t *&slab : ringSlab_)
            if (slab) {
                (void)hipHostFree(slab);
                slab = nullptr;
            }
        if (ctx_) zrc4_destroy(ctx_);
        sA_ = sB_ = nullptr;
        ctx_ = nullptr;
    }

    // 16 KiB per slot per refill (r06; 8 KiB before): a refill launch pays
    // ~6 us of launch, state load and store around its serial chain, and a
    // few-session engine is bound by that chain (config 1: 113.3k -> 117.0k
    // echo/s, scripts/r06_refill_ab.sh)
    static constexpr uint32_t kRefillChunk = 16384;
    static constexpr uint32_t kRefillDepth = 2;
    const uint32_t refillDepth_ = std::getenv("ZSX_REFILL_DEPTH") ? std::max(1, std::min(2, std::atoi(std::getenv("ZSX_REFILL_DEPTH")))) : kRefillDepth;
    static constexpr int ZRC4_ERR_NOT_READY_ = 1;   // internal: oldest refill still running
    const uint64_t directBytes_ = std::getenv("ZSX_RC4_DIRECT_BYTES")
                                     ? std::strtoull(std::getenv("ZSX_RC4_DIRECT_BYTES"), nullptr, 10)
                                     : (1ull << 20);
    double emaBytes_ = 0.0;
    bool direct_ = false;
    unsigned long long directCalls_ = 0;
    const bool debugNoRefill_ = std::getenv("ZSX_RESERVOIR_NO_REFILL") != nullptr;   // test knobs
    const bool debugSyncRefill_ = std::getenv("ZSX_RESERVOIR_SYNC_REFILL") != nullptr;

    zrc4_ctx *ctx_ = nullptr;
    hipStream_t sA_ = nullptr, sB_ = nullptr;
    Refill refill_[kRefillDepth];
    uint32_t head_ = 0, inFlight_ = 0;
    uint8_t *base_ = nullptr;
    uint32_t ringCap_;
    uint32_t refillChunk_ = 0;
    std::vector<uint8_t *> ringSlab_;
    std::vector<Level> level_;
    std::vector<uint32_t> seen_;
    uint32_t callStamp_ = 0;
    std::vector<uint8_t> hungryMark_;
    std::vector<uint32_t> hungry_;
    std::vector<XorJob> xj_;
    XorPool xor_;
    std::vector<Entry> es_, rs_;
    Table tt_;                                    // tail grouped table
    FrameTable ft_;                               // framing tables of cryptFrame
    PinnedArray<uint32_t> kIds_, kLen_;
    PinnedArray<uint64_t> kOff_;
    PinnedArray<uint8_t> kBytes_;
    std::vector<uint32_t> seedIds_, seedLen_;
    std::vector<uint64_t> seedOff_;
    std::vector<uint8_t> keyBytes_;
    unsigned long long ringBytes_ = 0, tailBytes_ = 0, tailLaunches_ = 0, refillBytes_ = 0, refillLaunches_ = 0,
                       refillWaits_ = 0, framed_ = 0;
};

}  // namespace

std::unique_ptr<Rc4Hooks> makeDeviceRc4Hooks(int device, uint32_t capacity, uint32_t ringBytes)
{
    return std::unique_ptr<Rc4Hooks>(new DeviceRc4Hooks(device, capacity, ringBytes));
}

}  // namespace zsummerx_amd
