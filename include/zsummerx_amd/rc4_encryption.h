// zsummerx_amd/rc4_encryption.h -- C++ host mirror of the reference RC4 class,
// backed by the gfx950 C-ABI library (include/zrc4.h, libzrc4.so).
//
// Drop-in for /root/reference/depends/rc4/rc4_encryption.h:43-99:
//   class RC4Encryption {
//     void makeSBox(std::string obscure);            // :46-72
//     void encryption(unsigned char *data, int len); // :74-93
//   };
// Same names, argument meaning and (absent) error reporting: the reference
// has no error channel, so a device failure here throws std::runtime_error
// (the reference session would have crashed on garbage instead; see
// INTEGRATION.md for the batched, error-returning path the hooks should use).
//
// Each RC4Encryption owns one slot (stream) of a process-wide device arena.
// A TcpSession owns two (_rc4StateRead/_rc4StateWrite, session.h:115-116).
// The per-call path copies host<->device, so it is a correctness drop-in; the
// throughput path is Rc4Batch (one launch per event-loop iteration).
#pragma once

#include <cstdint>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "zrc4.h"

namespace zsummerx_amd {

inline void zrc4_throw(int rc, const char *what)
{
    if (rc != ZRC4_OK)
        throw std::runtime_error(std::string(what) + ": " + zrc4_strerror(rc));
}

// Process-wide arena with a free list of slots.
class Rc4Arena {
public:
    static Rc4Arena &instance(uint32_t capacity = 1u << 17, int device = 0)
    {
        static Rc4Arena a(capacity, device);
        return a;
    }
    zrc4_ctx *ctx() const { return ctx_; }
    uint32_t acquire()
    {
        std::lock_guard<std::mutex> g(mu_);
        if (!free_.empty()) {
            uint32_t s = free_.back();
            free_.pop_back();
            return s;
        }
        if (next_ >= zrc4_capacity(ctx_)) throw std::runtime_error("zrc4 arena out of slots");
        return next_++;
    }
    void release(uint32_t s)
    {
        std::lock_guard<std::mutex> g(mu_);
        free_.push_back(s);
    }
    ~Rc4Arena()
    {
        if (ctx_) zrc4_destroy(ctx_);
    }

private:
    Rc4Arena(uint32_t capacity, int device)
    {
        zrc4_throw(zrc4_create(&ctx_, device, capacity), "zrc4_create");
    }
    zrc4_ctx *ctx_ = nullptr;
    std::mutex mu_;
    std::vector<uint32_t> free_;
    uint32_t next_ = 0;
};

class RC4Encryption {
public:
    RC4Encryption() : slot_(Rc4Arena::instance().acquire()) {}
    ~RC4Encryption() { Rc4Arena::instance().release(slot_); }
    RC4Encryption(const RC4Encryption &) = delete;
    RC4Encryption &operator=(const RC4Encryption &) = delete;

    // rc4_encryption.h:46-72 -- the key is taken by value as a std::string, so
    // embedded NULs count (length(), not strlen) and an empty key means the
    // identity box with x = y = 0.
    void makeSBox(std::string obscure)
    {
        zrc4_throw(zrc4_make_sbox(Rc4Arena::instance().ctx(), slot_,
                                  reinterpret_cast<const uint8_t *>(obscure.data()),
                                  obscure.size()),
                   "RC4Encryption::makeSBox");
    }

    // rc4_encryption.h:74-93 -- in place; length <= 0 does nothing.
    void encryption(unsigned char *data, int length)
    {
        zrc4_throw(zrc4_encryption(Rc4Arena::instance().ctx(), slot_, data, length),
                   "RC4Encryption::encryption");
    }

    uint32_t slot() const { return slot_; }

private:
    uint32_t slot_;
};

// Batched hook path: collect (slot, buffer, len) for one event-loop
// iteration, then crypt them all with one launch.  Host buffers are gathered
// into one pinned staging copy by zrc4_crypt_host.  Entries are crypted in
// insertion order per slot; a slot may appear once per flush.
class Rc4Batch {
public:
    explicit Rc4Batch(zrc4_ctx *ctx = Rc4Arena::instance().ctx()) : ctx_(ctx) {}
    void add(uint32_t slot, unsigned char *data, unsigned len)
    {
        if (!len) return;
        ptrs_.push_back(data);
        ids_.push_back(slot);
        off_.push_back(bytes_.size());
        len_.push_back(len);
        bytes_.insert(bytes_.end(), data, data + len);
    }
    // Returns ZRC4_OK or the error; on error the caller closes the sessions
    // (the reference's BCT_CORRUPTION path, src/frame/session.cpp:355-361).
    int flush()
    {
        if (ids_.empty()) return ZRC4_OK;
        int rc = zrc4_crypt_host(ctx_, ids_.data(), bytes_.data(), bytes_.size(), off_.data(),
                                 len_.data(), (uint32_t)ids_.size());
        if (rc == ZRC4_OK)
            for (size_t i = 0; i < ids_.size(); ++i)
                std::copy(bytes_.begin() + off_[i], bytes_.begin() + off_[i] + len_[i], ptrs_[i]);
        ptrs_.clear();
        ids_.clear();
        off_.clear();
        len_.clear();
        bytes_.clear();
        return rc;
    }

private:
    zrc4_ctx *ctx_;
    std::vector<unsigned char *> ptrs_;
    std::vector<uint32_t> ids_;
    std::vector<uint64_t> off_;
    std::vector<uint32_t> len_;
    std::vector<uint8_t> bytes_;
};

}  // namespace zsummerx_amd
