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
// Each RC4Encryption owns one slot (stream) of a process-wide device arena
// that grows in 65 536-stream chunks.  A TcpSession owns two
// (_rc4StateRead/_rc4StateWrite, session.h:115-116).  Every call goes through
// the chunk's keystream reservoir (zrc4_ks_*, include/zrc4.h): the device
// generates each slot's keystream ahead into a ring of pinned host memory
// ($ZSX_RC4_RING bytes per slot, default 8192; 0 = no reservoir), so a call
// is a host XOR with committed keystream and goes to the device only for
// bytes the ring does not cover (a slot's first call after makeSBox, or a
// burst larger than the ring).  Rc4Batch gathers one event-loop iteration's
// calls into one reservoir call.
#pragma once

#include <cstdint>
#include <cstdlib>
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

// Process-wide arena: device contexts of kChunk streams each, created on
// demand (a 100K-connection server needs 200K streams; each chunk is a 16 MiB
// S-box arena), with a free list of slots.  Slot id = chunk * kChunk + local.
// Device: $ZSX_RC4_DEVICE (default 0).  Thread-safe.
class Rc4Arena {
public:
    static constexpr uint32_t kChunk = 1u << 16;

    static Rc4Arena &instance()
    {
        static Rc4Arena a;
        return a;
    }
    zrc4_ctx *ctx(uint32_t slot)
    {
        std::lock_guard<std::mutex> g(mu_);
        return chunks_[slot / kChunk];
    }
    // The chunk's keystream reservoir: every state change of a slot goes
    // through it (zrc4.h: once used through a reservoir, a slot's device
    // state runs ahead of its stream position).
    zrc4_ks *ks(uint32_t slot)
    {
        std::lock_guard<std::mutex> g(mu_);
        return ks_[slot / kChunk];
    }
    static uint32_t local(uint32_t slot) { return slot % kChunk; }

    // A slot for a new RC4Encryption.  *recycled: the slot comes back from a
    // destroyed instance and still holds that stream's state; its new owner
    // resets it lazily (RC4Encryption::prepare), so a destructor makes no GPU
    // call and a new owner that starts with makeSBox pays for no reset.
    uint32_t acquire(bool *recycled)
    {
        std::lock_guard<std::mutex> g(mu_);
        if (!free_.empty()) {
            const uint32_t s = free_.back();
            free_.pop_back();
            *recycled = true;
            return s;
        }
        if (next_ == (uint64_t)chunks_.size() * kChunk) {
            zrc4_ctx *c = nullptr;
            zrc4_throw(zrc4_create(&c, device_, kChunk), "zrc4_create");
            zrc4_ks *k = nullptr;
            const int rc = zrc4_ks_create(c, ring_, &k);
            if (rc != ZRC4_OK) zrc4_destroy(c);
            zrc4_throw(rc, "zrc4_ks_create");
            chunks_.push_back(c);
            ks_.push_back(k);
        }
        *recycled = false;                 // a fresh slot holds the empty-key state
        return (uint32_t)next_++;
    }
    // Back to the free list; no GPU call (destructors may run during static
    // destruction, and a session teardown should not wait on the device).
    void release(uint32_t s)
    {
        std::lock_guard<std::mutex> g(mu_);
        free_.push_back(s);
    }
    // The empty-key state (identity box, x = y = 0: makeSBox(""),
    // rc4_encryption.h:48-56), ring emptied.
    static void reset(uint32_t s)
    {
        zrc4_throw(zrc4_ks_make_sbox(instance().ks(s), local(s), nullptr, 0), "RC4Encryption reset");
    }
    ~Rc4Arena()
    {
        for (zrc4_ks *k : ks_) zrc4_ks_destroy(k);
        for (zrc4_ctx *c : chunks_) zrc4_destroy(c);
    }

private:
    Rc4Arena()
    {
        const char *d = std::getenv("ZSX_RC4_DEVICE");
        device_ = d ? std::atoi(d) : 0;
        const char *r = std::getenv("ZSX_RC4_RING");
        ring_ = r ? (uint32_t)std::strtoul(r, nullptr, 10) : 8192u;
    }
    int device_ = 0;
    uint32_t ring_ = 8192;
    std::mutex mu_;
    std::vector<zrc4_ctx *> chunks_;
    std::vector<zrc4_ks *> ks_;
    std::vector<uint32_t> free_;
    uint64_t next_ = 0;
};

class RC4Encryption {
public:
    RC4Encryption() : slot_(Rc4Arena::instance().acquire(&stale_)) {}
    ~RC4Encryption()
    {
        if (slot_ != kNoSlot) Rc4Arena::instance().release(slot_);
    }
    // A value type like the reference (an int[256] + x + y member block): a
    // copy owns its own slot holding the same state.
    RC4Encryption(const RC4Encryption &o) : slot_(Rc4Arena::instance().acquire(&stale_)) { copyState(o); }
    RC4Encryption &operator=(const RC4Encryption &o)
    {
        if (this != &o) copyState(o);
        return *this;
    }
    RC4Encryption(RC4Encryption &&o) noexcept : stale_(o.stale_), slot_(o.slot_) { o.slot_ = kNoSlot; }
    RC4Encryption &operator=(RC4Encryption &&o) noexcept
    {
        if (this != &o) {
            if (slot_ != kNoSlot) Rc4Arena::instance().release(slot_);
            slot_ = o.slot_;
            stale_ = o.stale_;
            o.slot_ = kNoSlot;
        }
        return *this;
    }

    // rc4_encryption.h:46-72 -- the key is taken by value as a std::string, so
    // embedded NULs count (length(), not strlen) and an empty key means the
    // identity box with x = y = 0.
    void makeSBox(std::string obscure)
    {
        zrc4_throw(zrc4_ks_make_sbox(Rc4Arena::instance().ks(slot_), Rc4Arena::local(slot_),
                                     reinterpret_cast<const uint8_t *>(obscure.data()), obscure.size()),
                   "RC4Encryption::makeSBox");
        stale_ = false;
    }

    // rc4_encryption.h:74-93 -- in place; length <= 0 does nothing.
    void encryption(unsigned char *data, int length)
    {
        if (length <= 0) return;
        prepare();
        const uint32_t id = Rc4Arena::local(slot_), n = (uint32_t)length;
        uint8_t *d = data;
        zrc4_throw(zrc4_ks_crypt(Rc4Arena::instance().ks(slot_), &id, &d, &n, 1), "RC4Encryption::encryption");
    }

    // A recycled slot still holds its previous owner's stream until this
    // object seeds it: used before makeSBox, it starts from the empty-key
    // state like a fresh slot (the reset happens here, once).
    void prepare() const
    {
        if (stale_) {
            Rc4Arena::reset(slot_);
            stale_ = false;
        }
    }

    uint32_t slot() const { return slot_; }

private:
    static constexpr uint32_t kNoSlot = 0xFFFFFFFFu;
    // device state + the keystream already buffered for the source
    void copyState(const RC4Encryption &o)
    {
        o.prepare();
        Rc4Arena &a = Rc4Arena::instance();
        zrc4_throw(zrc4_ks_copy(a.ks(slot_), Rc4Arena::local(slot_), a.ks(o.slot_), Rc4Arena::local(o.slot_)),
                   "RC4Encryption copy");
        stale_ = false;
    }
    // stale_ is declared (and initialised) before slot_: slot_'s initialiser,
    // acquire(&stale_), sets it
    mutable bool stale_ = false;
    uint32_t slot_;
};

// Batched hook path: collect (slot, buffer, len) for one event-loop
// iteration, then crypt them all with one reservoir call (host XOR for the
// buffered keystream, one grouped launch for the uncovered tails).  A slot may
// appear once per flush.  `slot` is a slot of the reservoir's chunk (for
// RC4Encryption objects: Rc4Arena::local(r.slot()) with
// Rc4Arena::instance().ks(r.slot())).
class Rc4Batch {
public:
    explicit Rc4Batch(zrc4_ks *ks) : ks_(ks) {}
    // An RC4Encryption of this batch's reservoir (a recycled slot used before
    // its makeSBox is reset first, as RC4Encryption::encryption does).
    void add(const RC4Encryption &r, unsigned char *data, unsigned len)
    {
        if (!len) return;
        r.prepare();
        add(Rc4Arena::local(r.slot()), data, len);
    }
    // A raw slot of the reservoir's chunk that the caller has seeded.
    void add(uint32_t slot, unsigned char *data, unsigned len)
    {
        if (!len) return;
        ids_.push_back(slot);
        ptrs_.push_back(data);
        len_.push_back(len);
    }
    // Returns ZRC4_OK or the error; on error the caller closes the sessions
    // (the reference's BCT_CORRUPTION path, src/frame/session.cpp:355-361).
    int flush()
    {
        if (ids_.empty()) return ZRC4_OK;
        const int rc = zrc4_ks_crypt(ks_, ids_.data(), ptrs_.data(), len_.data(), (uint32_t)ids_.size());
        ids_.clear();
        ptrs_.clear();
        len_.clear();
        return rc;
    }

private:
    zrc4_ks *ks_;
    std::vector<uint32_t> ids_;
    std::vector<uint8_t *> ptrs_;
    std::vector<uint32_t> len_;
};

}  // namespace zsummerx_amd
