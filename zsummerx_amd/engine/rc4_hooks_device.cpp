// rc4_hooks_device.cpp -- the gfx950 Rc4Hooks (include/zsummerx_amd/rc4_hooks.h)
// over the C-ABI of libzrc4.so (include/zrc4.h).
//
// Memory ("pinned SessionBlock pool"): every SessionBlock
// slab is pinned host memory (hipHostMalloc) that the crypt kernel reads and
// writes in place, so one engine iteration costs one zrc4_ksa (only when
// sessions were seeded) + one zrc4_crypt launch + one wait -- no staging
// copies and no per-session calls.  The batch tables (slot ids, offsets,
// lengths, keys) are pinned too; the kernel reads them over PCIe.
//
// Payload addressing: zrc4_crypt takes one base pointer and 64-bit per-entry
// offsets; the base is the first slab and an entry's offset is its address
// minus the base in two's complement, so slabs anywhere in the address space
// share one launch (the kernel adds base + off in 64-bit arithmetic).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "zrc4.h"
#include "zsummerx_amd/rc4_hooks.h"

namespace zsummerx_amd {
namespace {

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
        if (hipHostMalloc(reinterpret_cast<void **>(&q), c * sizeof(T), hipHostMallocDefault) != hipSuccess)
            throw std::bad_alloc();
        if (p) (void)hipHostFree(p);
        p = q;
        cap = c;
    }
    ~PinnedArray()
    {
        if (p) (void)hipHostFree(p);
    }
};

class DeviceRc4Hooks final : public Rc4Hooks {
public:
    DeviceRc4Hooks(int device, uint32_t capacity) : device_(device)
    {
        const int rc = zrc4_create(&ctx_, device, capacity);
        if (rc != ZRC4_OK)
            throw std::runtime_error(std::string("makeDeviceRc4Hooks: zrc4_create: ") + zrc4_strerror(rc));
        if (hipSetDevice(device) != hipSuccess ||
            hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess) {
            zrc4_destroy(ctx_);
            throw std::runtime_error("makeDeviceRc4Hooks: cannot create a HIP stream");
        }
    }
    ~DeviceRc4Hooks() override
    {
        if (stream_) {
            (void)hipStreamSynchronize(stream_);
            (void)hipStreamDestroy(stream_);
        }
        if (ctx_) zrc4_destroy(ctx_);
    }

    const char *name() const override { return "zrc4-gfx950"; }
    uint32_t capacity() const override { return zrc4_capacity(ctx_); }

    void *allocBlocks(size_t bytes) override
    {
        void *p = nullptr;
        if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) throw std::bad_alloc();
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
        if (!base_) return ZRC4_ERR_INVALID_ARG;
        ids_.reserve(n);
        off_.reserve(n);
        len_.reserve(n);
        for (uint32_t i = 0; i < n; ++i) {
            ids_.p[i] = spans[i].slot;
            off_.p[i] = (uint64_t)((uintptr_t)spans[i].data - (uintptr_t)base_);
            len_.p[i] = spans[i].len;
        }
        rc = zrc4_crypt(ctx_, ids_.p, base_, off_.p, len_.p, n, stream_);
        if (rc != ZRC4_OK) return rc;
        return zrc4_sync(ctx_, stream_);
    }

private:
    // Queued makeSBox calls go out as one zrc4_ksa launch ahead of the crypt
    // on the same stream; the crypt's wait covers both.
    int flushSeeds()
    {
        const uint32_t m = (uint32_t)seedIds_.size();
        if (m == 0) return ZRC4_OK;
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
        return zrc4_ksa(ctx_, kIds_.p, kBytes_.p, kOff_.p, kLen_.p, m, stream_);
    }

    int device_;
    zrc4_ctx *ctx_ = nullptr;
    hipStream_t stream_ = nullptr;
    uint8_t *base_ = nullptr;
    PinnedArray<uint32_t> ids_, len_, kIds_, kLen_;
    PinnedArray<uint64_t> off_, kOff_;
    PinnedArray<uint8_t> kBytes_;
    std::vector<uint32_t> seedIds_, seedLen_;
    std::vector<uint64_t> seedOff_;
    std::vector<uint8_t> keyBytes_;
};

}  // namespace

std::unique_ptr<Rc4Hooks> makeDeviceRc4Hooks(int device, uint32_t capacity)
{
    return std::unique_ptr<Rc4Hooks>(new DeviceRc4Hooks(device, capacity));
}

}  // namespace zsummerx_amd
