// zsummerx_amd/rc4_hooks.h -- the RC4 hook interface of the batched session
// engine (include/zsummerx_amd/frame.h).
//
// The reference runs RC4 synchronously, one session at a time, at five hook
// sites of TcpSession:
//   seeding  _rc4StateRead/_rc4StateWrite.makeSBox(key)   src/frame/session.cpp:110-111
//   decrypt  _rc4StateRead.encryption(recv tail)          src/frame/session.cpp:313-323
//   encrypt  _rc4StateWrite.encryption(_sending)          src/frame/session.cpp:496-499,
//                                                         535-538, 603-606
// The engine instead collects every hook of one event-loop iteration and hands
// them to an Rc4Hooks object at once: seeds are queued, then ONE crypt() call
// covers every recv tail and every outgoing _sending block of the iteration.
//
// The product implementation is makeDeviceRc4Hooks(): one zrc4 context
// (include/zrc4.h) on a gfx950 device; SessionBlocks live in pinned host
// memory that the kernels read and write in place (zero-copy, no staging
// copies).  Keystream is generated on the GPU ahead of need into pinned host
// rings, so a hook call is a host-side XOR unless a stream runs short (see
// rc4_hooks_device.cpp).  There is no CPU fallback: without a device the
// factory throws.
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>

namespace zsummerx_amd {

// One RC4Encryption::encryption(data, len) call (rc4_encryption.h:74-93):
// crypt data[0..len) in place with stream `slot`, advancing it by len bytes.
struct Rc4Span {
    uint32_t slot;
    uint32_t len;
    uint8_t *data;   // inside memory returned by Rc4Hooks::allocBlocks
};

// Device-side framing request for one span: after the
// span is decrypted, frame block[0 .. len) -- the whole receive block, which
// may start before the span -- with proto4z HasRawPacket
// (depends/proto4z/proto4z.h:704-748) as TcpSession::onRecv's loop does
// (src/frame/session.cpp:329-371).  len == 0: no framing for this span.
struct Rc4Frame {
    static constexpr uint32_t kMaxPackets = 16;
    const uint8_t *block = nullptr;
    uint32_t len = 0;
    // results
    uint32_t npk = 0;                 // complete packets from the block start
    uint32_t used = 0;                // bytes they cover
    uint32_t status = 0;              // 1 stopped on shortage, 2 on corruption
    uint32_t pkt[kMaxPackets] = {};   // the first min(npk, kMaxPackets) lengths
};

class Rc4Hooks {
public:
    virtual ~Rc4Hooks() = default;
    virtual const char *name() const = 0;
    // Number of RC4 streams (slots); a session uses two (read and write).
    virtual uint32_t capacity() const = 0;
    // Memory that crypt() may touch in place (SessionBlocks come from here).
    virtual void *allocBlocks(size_t bytes) = 0;
    virtual void freeBlocks(void *p) = 0;
    // Queue RC4Encryption::makeSBox(key) (rc4_encryption.h:46-72) for each of
    // slots[0..n); it takes effect before the next crypt() touches them.
    virtual int seed(const uint32_t *slots, uint32_t n, const std::string &key) = 0;
    // Run every span (each slot at most once per call: a repeated slot is
    // ZRC4_ERR_INVALID_ARG); returns when the results are in place.  0 = ok,
    // otherwise a negative zrc4 status.
    virtual int crypt(const Rc4Span *spans, uint32_t n) = 0;
    // Decrypt and frame in one device pass: crypt() semantics for the spans,
    // then frames[i] (parallel to spans[i]) filled as Rc4Frame describes,
    // with `bound` the blocks' size (SESSION_BLOCK_SIZE).  Only when
    // canFrame(); otherwise the engine frames on the host.
    virtual bool canFrame() const { return false; }
    virtual int cryptFrame(const Rc4Span *spans, uint32_t n, Rc4Frame *frames, uint32_t bound)
    {
        (void)spans;
        (void)n;
        (void)frames;
        (void)bound;
        return -1;   // ZRC4_ERR_INVALID_ARG
    }
    // Implementation counters as one JSON object (diagnostics).
    virtual std::string stats() const { return "{}"; }
};

// The gfx950 implementation over libzrc4.so (throws std::runtime_error when no
// usable device exists or the context cannot be created).  ringBytes > 0
// selects the keystream-reservoir mode (per-slot keystream rings of that many
// bytes in pinned host memory, filled by the GPU; see rc4_hooks_device.cpp),
// 0 the direct mode (one grouped zrc4 launch over the spans per iteration).
std::unique_ptr<Rc4Hooks> makeDeviceRc4Hooks(int device, uint32_t capacity, uint32_t ringBytes = 65536);

// Hooks for an engine whose sessions all have RC4 off (empty
// _rc4TcpEncryption): plain host blocks; seed()/crypt() fail with
// ZRC4_ERR_NO_DEVICE if a keyed session ever reaches them.
std::unique_ptr<Rc4Hooks> makeKeylessHooks();

}  // namespace zsummerx_amd
