/*
 * oracle/rc4_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the zsummerX RC4 path, used as the parity checker for the
 * HIP product path and as the `cpu_baseline` ("port") leg of bench.py.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product library (zsummerx_amd/libzrc4.so) never links or calls this.
 *
 * Reference algorithm: /root/reference/depends/rc4/rc4_encryption.h
 *   RC4Encryption::makeSBox   :46-72   (KSA)
 *   RC4Encryption::encryption :74-93   (PRGA + XOR, in place)
 *   state int _x, _y, _box[256] :96-98
 *
 * Parity is pinned against the real header: oracle/Makefile compiles
 * oracle/ref_shim.cpp (which #includes the reference header where it lies) into
 * oracle/_ref/libzrc4_ref.so, and tests/golden/make_golden.py generates the
 * committed fixtures from it (plus the published RFC 6229 / Wikipedia KATs).
 */
#ifndef ZRC4_ORACLE_H
#define ZRC4_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same encoding as the reference state (rc4_encryption.h:96-98): ints. */
typedef struct oracle_rc4_state {
    int x;
    int y;
    int box[256];
} oracle_rc4_state;

/* rc4_encryption.h:46-72.  key may contain NULs; keylen==0 -> identity box. */
void oracle_make_sbox(oracle_rc4_state *st, const uint8_t *key, size_t keylen);

/* rc4_encryption.h:74-93.  length <= 0 is a no-op (loop never runs). */
void oracle_encryption(oracle_rc4_state *st, uint8_t *data, long length);

/* Batch helpers (test/bench infrastructure, not reference functions). */
void oracle_make_sbox_batch(oracle_rc4_state *st, const uint8_t *keys,
                            const uint64_t *key_off, const uint32_t *key_len,
                            uint32_t n);
/* crypt session i's payload[off[i] .. off[i]+len[i]) with st[i];
 * threads>1 splits sessions round-robin over pthreads (BASELINE.md plan). */
void oracle_crypt_batch(oracle_rc4_state *st, uint8_t *payload,
                        const uint64_t *off, const uint32_t *len, uint32_t n,
                        int threads);

/* Export/import between the int reference state and the 258-byte form. */
void oracle_state_to_bytes(const oracle_rc4_state *st, uint8_t sbox[256],
                           uint8_t *x, uint8_t *y);
void oracle_state_from_bytes(oracle_rc4_state *st, const uint8_t sbox[256],
                             uint8_t x, uint8_t y);

/* proto4z framing of n decrypted session buffers, as TcpSession::onRecv does
 * after decrypting (src/frame/session.cpp:329-371 with HasRawPacket,
 * depends/proto4z/proto4z.h:704-748): status 1 = stopped on shortage, 2 = on
 * corruption; npk / used / pkt_len as zrc4_frame_scan (include/zrc4.h). */
void oracle_frame_scan(const uint8_t *buf, const uint64_t *off, const uint32_t *len, uint32_t bound,
                       uint32_t n, uint32_t max_packets, uint32_t *npk, uint32_t *used,
                       uint32_t *status, uint32_t *pkt_len);

/* Wall-clock seconds (CLOCK_MONOTONIC) for the cpu_baseline timer. */
double oracle_now(void);

/* CPU-baseline timing: payload bytes per second of `threads` workers
 * re-crypting their contiguous share of the n sessions for `seconds`. */
double oracle_crypt_rate(oracle_rc4_state *st, uint8_t *payload, const uint64_t *off, const uint32_t *len,
                         uint32_t n, int threads, double seconds);

#ifdef __cplusplus
}
#endif
#endif
