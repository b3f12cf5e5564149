/*
 * zrc4.h -- C-ABI of the MI355X-native RC4 payload-encryption path for
 * zsummerX (the drop-in behind SessionOptions::_rc4TcpEncryption).
 *
 * Reference interface this boundary replaces
 * (/root/reference, read-only):
 *   class RC4Encryption                      depends/rc4/rc4_encryption.h:43-99
 *     void makeSBox(std::string obscure)     depends/rc4/rc4_encryption.h:46-72
 *     void encryption(unsigned char*, int)   depends/rc4/rc4_encryption.h:74-93
 *     int _x, _y, _box[256]                  depends/rc4/rc4_encryption.h:96-98
 *   reached only from TcpSession:
 *     seeding  _rc4StateRead/_rc4StateWrite.makeSBox   src/frame/session.cpp:110-111
 *     decrypt  _rc4StateRead.encryption(recv tail)     src/frame/session.cpp:313-323
 *     encrypt  _rc4StateWrite.encryption(_sending)     src/frame/session.cpp:496-499,
 *                                                      535-538, 603-606
 *   switch    SessionOptions::_rc4TcpEncryption (empty = off)
 *                                                      include/zsummerX/frame/config.h:196
 *
 * Model.  A context owns one device (HIP/gfx950) and a device-resident arena of
 * `capacity` RC4 streams ("slots"; a TcpSession owns two: read and write).  A
 * slot's state is the reference state (S-box + x + y) held as 258 bytes.  The
 * batched entry points take DEVICE pointers and are stream-ordered and
 * asynchronous; the *_host entry points take host pointers and block.
 *
 * Conventions (all functions):
 *   - return 0 (ZRC4_OK) or a negative ZRC4_ERR_* code; nothing throws across
 *     the ABI; zrc4_strerror() names a code.
 *   - ids == NULL means the identity map (batch entry i -> slot i).
 *   - a slot may appear at most once per call; len == 0 is a no-op for that
 *     slot (reference: `length <= 0` never enters the loop, :81).
 *   - calls on one context are serialised by the caller (one event-loop
 *     thread, as the reference: include/zsummerX/frame/manager.h:98-110);
 *     concurrent calls on different streams must touch disjoint 256-slot
 *     groups (slot / 256).
 *   - no CPU fallback: with no usable gfx950 device zrc4_create fails with
 *     ZRC4_ERR_NO_DEVICE.
 *   - device-side faults of a batched call (a slot id >= capacity) are latched
 *     and reported by the next zrc4_sync() as ZRC4_ERR_SLOT_RANGE; the affected
 *     entries are skipped (caller closes those sessions, as the reference does
 *     on BCT_CORRUPTION, src/frame/session.cpp:355-361).  The latch belongs to
 *     the CONTEXT, not to a stream: zrc4_sync on any stream reports (and
 *     clears) faults of every kernel of the context that has completed, so a
 *     caller that uses several streams syncs them all before acting on a
 *     fault.
 */
#ifndef ZRC4_H
#define ZRC4_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZRC4_OK 0
#define ZRC4_ERR_INVALID_ARG (-1)
#define ZRC4_ERR_NO_DEVICE (-2)
#define ZRC4_ERR_OUT_OF_MEMORY (-3)
#define ZRC4_ERR_LAUNCH (-4)
#define ZRC4_ERR_SLOT_RANGE (-5)
#define ZRC4_ERR_HIP (-6)
#define ZRC4_ERR_GROUP (-7)    /* zrc4_crypt_grouped: a bucket broke the bucket contract */
#define ZRC4_ERR_INTERNAL (-8) /* kernel self-check failed (LDS layout) */
#define ZRC4_ERR_STATE (-9)    /* zrc4_ks_crypt / zrc4_ks_copy: the slot's stream position
                                  was lost by a failed zrc4_ks_crypt; reseed it
                                  (zrc4_ks_make_sbox) or copy into it (zrc4_ks_copy) */

/* Slots are grouped 256 to a 64 KiB device image (the LDS image of one
 * workgroup); capacity is rounded up to a multiple of this. */
#define ZRC4_GROUP_SLOTS 256u
#define ZRC4_STATE_BYTES 258u

typedef struct zrc4_ctx zrc4_ctx;

/* Create a context on HIP device `device` with room for `capacity` streams.
 * Replaces: the per-session RC4Encryption members (session.h:115-116). */
int zrc4_create(zrc4_ctx **out, int device, uint32_t capacity);
int zrc4_destroy(zrc4_ctx *ctx);
uint32_t zrc4_capacity(const zrc4_ctx *ctx);

/* Batched KSA (RC4Encryption::makeSBox, rc4_encryption.h:46-72) for n slots.
 * Entry i seeds slot ids[i] from keys[key_off[i] .. key_off[i]+key_len[i]);
 * key bytes may be NUL; key_len 0 gives the identity S-box with x = y = 0.
 * Device pointers; asynchronous on `stream` (hipStream_t, NULL = default). */
int zrc4_ksa(zrc4_ctx *ctx, const uint32_t *ids, const uint8_t *keys,
             const uint64_t *key_off, const uint32_t *key_len, uint32_t n,
             void *stream);

/* Batched PRGA+XOR (RC4Encryption::encryption, rc4_encryption.h:74-93), in
 * place: entry i crypts payload[off[i] .. off[i]+len[i]) with slot ids[i] and
 * advances that slot by len[i] bytes.  Device pointers; asynchronous. */
int zrc4_crypt(zrc4_ctx *ctx, const uint32_t *ids, uint8_t *payload,
               const uint64_t *off, const uint32_t *len, uint32_t n,
               void *stream);

/* Contiguous-slot variants: entry i uses slot first_slot + i (no ids array).
 * When first_slot is a multiple of 256 every workgroup owns a whole slot
 * group and moves its state as one coalesced 64 KiB image: the fast path for
 * a session engine that allocates its streams in groups.  Requires
 * first_slot + n <= capacity.  Device pointers; asynchronous. */
int zrc4_ksa_range(zrc4_ctx *ctx, uint32_t first_slot, const uint8_t *keys,
                   const uint64_t *key_off, const uint32_t *key_len, uint32_t n,
                   void *stream);
int zrc4_crypt_range(zrc4_ctx *ctx, uint32_t first_slot, uint8_t *payload,
                     const uint64_t *off, const uint32_t *len, uint32_t n,
                     void *stream);

/* Grouped-ids variant: the fast path for arbitrary slot subsets.  Entries
 * are taken in buckets of 256 (bucket b = entries [256b, 256b + 256)); the
 * caller promises that every busy entry (len > 0) of a bucket uses a slot of
 * ONE 256-slot group (slot / 256), that no other bucket of the call touches
 * that group, and that a slot appears at most once.  Entries may come in any
 * order; padding entries carry ids[i] = ZRC4_IDLE_SLOT or len 0.  Each bucket
 * then moves its group's state as one coalesced 64 KiB image, exactly like a
 * whole-group zrc4_crypt_range.  Refusals, reported by zrc4_sync as
 * ZRC4_ERR_GROUP (no payload byte, S-box or x/y of a refused bucket is
 * touched; every other bucket runs):
 *   - a bucket whose busy entries span two groups, or name a slot twice;
 *   - a bucket naming a group another bucket of the same call holds: every
 *     workgroup claims the PART of its bucket's group it moves (a dword
 *     column on the window kernel, <= 32 buckets; a half on the half-group
 *     and persistent kernels; the whole group otherwise), and the first
 *     claimant of a part runs.  Claims and refusals therefore apply per part:
 *     two buckets naming one group may each run some parts of it (each slot
 *     is still all or nothing: crypted with its state advanced, or untouched).
 *     Where the claim is taken: the window kernel (<= 32 buckets) claims
 *     only after its bucket's table check has passed, so a bucket it
 *     refuses claims nothing.  The half- and whole-group kernels (at most
 *     one bucket per CU) claim while the check runs, on the bucket's first
 *     busy id (zrc4_crypt_grouped_declared: on the declared group), and the
 *     persistent kernel (more buckets than CUs) claims a bucket's group
 *     before its slot table can refuse a slot named twice.  So on those
 *     kernels a bucket that breaks the one-group or once-per-slot rule may
 *     also block a valid bucket of a group it names.
 * An id >= capacity other than ZRC4_IDLE_SLOT is skipped and reported as
 * ZRC4_ERR_SLOT_RANGE (the rest of its bucket runs).  The claims carry a
 * per-call tag chosen on the host: a grouped call must not be captured into
 * a HIP graph and replayed (the replay would find its own tags and refuse
 * every bucket).  n <= 0xFFF00000.  Device pointers; asynchronous. */
#define ZRC4_IDLE_SLOT 0xFFFFFFFFu
int zrc4_crypt_grouped(zrc4_ctx *ctx, const uint32_t *ids, uint8_t *payload,
                       const uint64_t *off, const uint32_t *len, uint32_t n,
                       void *stream);

/* zrc4_crypt_grouped with each bucket's group declared by the caller, who
 * built the buckets on the host and so already knows them (the session
 * engine, zrc4_crypt_host).  bucket_group is HOST memory of ceil(n / 256)
 * entries, read during the call: bucket b's group (slot / 256 of its busy
 * entries), or ZRC4_IDLE_SLOT for a bucket with no busy entry.  A group
 * >= capacity / 256 returns ZRC4_ERR_INVALID_ARG and launches nothing.
 * Semantics are zrc4_crypt_grouped's, plus one refusal: a bucket with a busy
 * entry outside its declared group is refused (ZRC4_ERR_GROUP, nothing of it
 * written).  Why: with at most 256 buckets (at most one bucket per CU, where
 * the launch is one keystream chain long) the groups travel in the kernel
 * arguments, so each bucket's state image is loaded with its entries instead
 * of after a dependent read of the bucket's ids.  With more buckets the
 * declared groups are checked by a short kernel on the same stream just
 * before the crypt launch (it reads them from pinned memory the call fills);
 * a disagreeing bucket's own ids then also block the groups they name, so
 * another bucket naming one of those groups is refused too (the rule for two
 * buckets naming one group).  Callers that build their buckets themselves
 * gain nothing from the declaration above 256 buckets: there the persistent
 * kernel already prefetches each bucket's ids a bucket ahead.  frame: NULL for
 * no framing, else zrc4_crypt_grouped_frame's framing (below).  Device
 * pointers apart from bucket_group; asynchronous. */
struct zrc4_frame_args;
int zrc4_crypt_grouped_declared(zrc4_ctx *ctx, const uint32_t *ids,
                                const uint32_t *bucket_group, uint8_t *payload,
                                const uint64_t *off, const uint32_t *len,
                                uint32_t n, const struct zrc4_frame_args *frame,
                                void *stream);

/* Host-pointer variants: copy to the device (pinned staging), run, copy back,
 * block until done.  payload_bytes bounds the host payload buffer.
 * zrc4_crypt_host checks every id on the host first: an id >= capacity
 * (ZRC4_IDLE_SLOT included) returns ZRC4_ERR_SLOT_RANGE and crypts nothing.
 * With several ids it buckets them by group itself and runs the
 * zrc4_crypt_grouped path (a slot may appear once per call: a repeated slot
 * returns ZRC4_ERR_INVALID_ARG and crypts nothing). */
int zrc4_ksa_host(zrc4_ctx *ctx, const uint32_t *ids, const uint8_t *keys,
                  size_t keys_bytes, const uint64_t *key_off,
                  const uint32_t *key_len, uint32_t n);
int zrc4_crypt_host(zrc4_ctx *ctx, const uint32_t *ids, uint8_t *payload,
                    size_t payload_bytes, const uint64_t *off,
                    const uint32_t *len, uint32_t n);

/* Single-stream drop-ins with the reference's exact argument meaning:
 *   zrc4_make_sbox  == RC4Encryption::makeSBox(std::string(key, keylen))
 *   zrc4_encryption == RC4Encryption::encryption(data, length) (host data,
 *                      in place, length <= 0 is a no-op) */
int zrc4_make_sbox(zrc4_ctx *ctx, uint32_t id, const uint8_t *key,
                   size_t keylen);
int zrc4_encryption(zrc4_ctx *ctx, uint32_t id, uint8_t *data, int length);

/* Keystream reservoirs (the session engine's low-latency hook path,
 * zsummerx_amd/engine/rc4_hooks_device.cpp).  RC4's keystream does not depend
 * on the data, so a slot's keystream can be generated ahead into a device
 * ring of ring_cap bytes (ring r at ring + r * ring_cap) by zrc4_crypt over
 * ZEROED ring bytes (0 ^ k = k; the slot's state advances as usual).
 * zrc4_xor_ring then XORs entry i's payload[off[i] .. off[i]+len[i]) with
 * ring rid[i] from position pos[i] on (wrapping mod ring_cap) and zeroes the
 * ring bytes it used.  Requires len[i] <= ring_cap and pos[i] < ring_cap; the
 * caller tracks which ring bytes hold keystream.  Device (or pinned host)
 * pointers; asynchronous on `stream`.  Touches no slot state. */
int zrc4_xor_ring(zrc4_ctx *ctx, uint8_t *ring, uint32_t ring_cap,
                  const uint32_t *rid, const uint32_t *pos, uint8_t *payload,
                  const uint64_t *off, const uint32_t *len, uint32_t n,
                  void *stream);

/* Device-side proto4z framing of decrypted session buffers (the step after
 * the recv decrypt, src/frame/session.cpp:329-371, with HasRawPacket,
 * depends/proto4z/proto4z.h:704-748, as the check): entry i walks
 * buf[off[i] .. off[i]+len[i]) from its start with the reference's
 * check(begin+used, len-used, bound-used, bound) until it stops, and writes
 *   npk[i]     complete packets found,
 *   used[i]    bytes they cover (the reference memmoves the rest down),
 *   status[i]  1 = stopped on shortage, 2 = on corruption (close the session),
 *   pkt_len[i * max_packets + k]  the first max_packets packet lengths
 *              (pkt_len may be NULL when max_packets == 0).
 * bound is the receive block size (SESSION_BLOCK_SIZE = 20480 in the
 * reference, config.h:100).  Device pointers; asynchronous on `stream`. */
int zrc4_frame_scan(zrc4_ctx *ctx, const uint8_t *buf, const uint64_t *off,
                    const uint32_t *len, uint32_t bound, uint32_t n,
                    uint32_t max_packets, uint32_t *npk, uint32_t *used,
                    uint32_t *status, uint32_t *pkt_len, void *stream);

/* Decrypt + frame in ONE launch (the recv hook followed by onRecv's framing
 * loop, src/frame/session.cpp:313-371): zrc4_crypt_range / zrc4_crypt_grouped
 * semantics for the crypt, then for every entry i the zrc4_frame_scan walk of
 * payload[frame->off[i] .. frame->off[i] + frame->len[i]) (the whole receive
 * block, which may start before the decrypted tail) into npk/used/status/
 * pkt_len[i] exactly as zrc4_frame_scan defines them.  One launch at every
 * size: in the chain-bound regime (at most one slot group per CU) each lane
 * frames its own session in the crypt kernel's epilogue; larger batches run
 * the persistent throughput kernel, whose workgroups frame the entries of the
 * 256-entry chunks they decrypted in their tail.  Framing outputs of a bucket
 * refused with ZRC4_ERR_GROUP are unspecified, with one guarantee on launches
 * of at most one bucket per CU (the window, half- and whole-group kernels,
 * declared or not): its busy entries (the ones it would have decrypted) are
 * never framed over their undecrypted bytes.  (The persistent kernel's tail
 * walks every chunk, a refused bucket's included, on its bytes as they
 * stand.)  Device pointers; asynchronous. */
typedef struct zrc4_frame_args {
    const uint64_t *off;
    const uint32_t *len;
    uint32_t bound;
    uint32_t max_packets;
    uint32_t *npk;
    uint32_t *used;
    uint32_t *status;
    uint32_t *pkt_len;
} zrc4_frame_args;
int zrc4_crypt_range_frame(zrc4_ctx *ctx, uint32_t first_slot, uint8_t *payload,
                           const uint64_t *off, const uint32_t *len, uint32_t n,
                           const zrc4_frame_args *frame, void *stream);
int zrc4_crypt_grouped_frame(zrc4_ctx *ctx, const uint32_t *ids, uint8_t *payload,
                             const uint64_t *off, const uint32_t *len, uint32_t n,
                             const zrc4_frame_args *frame, void *stream);

/* Wait for `stream`, then report (and clear) any latched device-side fault. */
/* Keystream reservoir over a context (the C++ mirror's per-call path):
 * per-slot rings of ring_bytes in pinned host memory that the device fills
 * ahead with the slot's keystream (background stream, one grouped launch for
 * every slot used since the last refill).  zrc4_ks_crypt XORs host spans with
 * committed ring bytes on the host and crypts only what the rings do not
 * cover on the device, so steady-state calls make no GPU round trip; output
 * bytes are exactly RC4Encryption::encryption's.  Once a slot is used through
 * a reservoir, every state change of it must go through the same reservoir
 * (its device state runs ahead of its stream position by the buffered bytes):
 * zrc4_ks_make_sbox == makeSBox, zrc4_ks_copy == copying the RC4Encryption
 * value (device state + buffered keystream).  ring_bytes 0: no buffering
 * (every call crypts on the device).  Thread-safe per reservoir; a slot at
 * most once per zrc4_ks_crypt call.  stats: ring bytes, tail bytes, tail
 * launches, refill bytes, refill launches, refill waits.
 * Failure: a zrc4_ks_crypt whose device tail fails returns the error and
 * leaves EVERY slot of that call lost (some spans may already be crypted
 * from their rings, some not): zrc4_ks_crypt and zrc4_ks_copy return
 * ZRC4_ERR_STATE for them until zrc4_ks_make_sbox reseeds a slot or
 * zrc4_ks_copy copies a live one into it; the call's data must be treated as
 * consumed, not retried. */
typedef struct zrc4_ks zrc4_ks;
int zrc4_ks_create(zrc4_ctx *ctx, uint32_t ring_bytes, zrc4_ks **out);
int zrc4_ks_destroy(zrc4_ks *ks);
int zrc4_ks_crypt(zrc4_ks *ks, const uint32_t *ids, uint8_t *const *data,
                  const uint32_t *len, uint32_t n);
int zrc4_ks_make_sbox(zrc4_ks *ks, uint32_t id, const uint8_t *key,
                      size_t keylen);
int zrc4_ks_copy(zrc4_ks *dst_ks, uint32_t dst, zrc4_ks *src_ks, uint32_t src);
int zrc4_ks_stats(zrc4_ks *ks, uint64_t out[6]);

int zrc4_sync(zrc4_ctx *ctx, void *stream);

/* Report (and clear) faults latched by kernels that have already completed
 * (e.g. after an event query succeeded), without waiting for any stream. */
int zrc4_poll_faults(zrc4_ctx *ctx);

/* Export / import one slot's state: S-box bytes + x + y (the reference's
 * int _box[256], _x, _y narrowed to bytes; values are always in [0,255]). */
int zrc4_get_state(zrc4_ctx *ctx, uint32_t id, uint8_t sbox[256], uint8_t *x,
                   uint8_t *y);
int zrc4_set_state(zrc4_ctx *ctx, uint32_t id, const uint8_t sbox[256],
                   uint8_t x, uint8_t y);
/* Bulk export of slots [first_slot, first_slot + n): sbox[256 i .. 256 i +
 * 255], x[i], y[i] for slot first_slot + i (host memory; blocks).  One copy of
 * the groups' images instead of a strided copy per slot (checkpointing the
 * sessions of a shard, the parity tests' state checks). */
int zrc4_get_states(zrc4_ctx *ctx, uint32_t first_slot, uint32_t n,
                    uint8_t *sbox, uint8_t *x, uint8_t *y);

const char *zrc4_strerror(int code);
const char *zrc4_version(void);

#ifdef __cplusplus
}
#endif
#endif /* ZRC4_H */
