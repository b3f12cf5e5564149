/*
 * oracle/rc4_oracle.c -- TEST INFRASTRUCTURE ONLY (see rc4_oracle.h).
 *
 * A plain-C restatement of RC4Encryption from
 * /root/reference/depends/rc4/rc4_encryption.h.  The per-byte work keeps the
 * reference's shape (int S-box, read S[x], update y, swap, keystream read) so
 * that, compiled -O3, it is a faithful single-core timing baseline; the
 * release flags of the reference are -O3 (CMakeLists.txt:109-111).
 */
#define _POSIX_C_SOURCE 200809L
#include "rc4_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* KSA.  Follows rc4_encryption.h:46-72:
 *   x = y = 0; box = identity;
 *   if key non-empty: for i in 0..255:
 *       j = (u8)(j + box[i] + key[k]); swap(box[i], box[j]); k = (k+1) % len
 * Key bytes are read as unsigned char (:63); an empty key leaves the identity
 * box (:56); only the first 256 key bytes can influence the result. */
void oracle_make_sbox(oracle_rc4_state *st, const uint8_t *key, size_t keylen)
{
    st->x = 0;
    st->y = 0;
    for (int i = 0; i < 256; ++i)
        st->box[i] = i;
    if (keylen == 0)
        return;
    unsigned j = 0;
    size_t k = 0;
    for (int i = 0; i < 256; ++i) {
        int v = st->box[i];
        j = (j + (unsigned)v + key[k]) & 0xFFu;
        st->box[i] = st->box[j];
        st->box[j] = v;
        if (++k == keylen)
            k = 0;
    }
}

/* PRGA + XOR, in place.  Follows rc4_encryption.h:74-93: for each byte
 *   x = (u8)(x+1); a = box[x]; y = (u8)(y+a);
 *   b = box[x] = box[y]; box[y] = a; data[i] ^= box[(u8)(a+b)]
 * x and y are loaded from / stored back to the state around the loop
 * (:78-79, :91-92).  length <= 0 leaves data and state untouched. */
void oracle_encryption(oracle_rc4_state *st, uint8_t *data, long length)
{
    int x = st->x, y = st->y;
    for (long i = 0; i < length; ++i) {
        x = (unsigned char)(x + 1);
        int a = st->box[x];
        y = (unsigned char)(y + a);
        int b = st->box[x] = st->box[y];
        st->box[y] = a;
        data[i] ^= (uint8_t)st->box[(unsigned char)(a + b)];
    }
    st->x = x;
    st->y = y;
}

void oracle_make_sbox_batch(oracle_rc4_state *st, const uint8_t *keys,
                            const uint64_t *key_off, const uint32_t *key_len,
                            uint32_t n)
{
    for (uint32_t i = 0; i < n; ++i)
        oracle_make_sbox(&st[i], keys + key_off[i], key_len[i]);
}

typedef struct {
    oracle_rc4_state *st;
    uint8_t *payload;
    const uint64_t *off;
    const uint32_t *len;
    uint32_t n;
    int tid, nthreads;
} crypt_job;

static void *crypt_worker(void *arg)
{
    crypt_job *j = (crypt_job *)arg;
    for (uint32_t i = (uint32_t)j->tid; i < j->n; i += (uint32_t)j->nthreads)
        oracle_encryption(&j->st[i], j->payload + j->off[i], (long)j->len[i]);
    return NULL;
}

void oracle_crypt_batch(oracle_rc4_state *st, uint8_t *payload,
                        const uint64_t *off, const uint32_t *len, uint32_t n,
                        int threads)
{
    if (threads <= 1) {
        crypt_job j = {st, payload, off, len, n, 0, 1};
        crypt_worker(&j);
        return;
    }
    if (threads > 256)
        threads = 256;
    pthread_t tids[256];
    crypt_job jobs[256];
    for (int t = 0; t < threads; ++t) {
        crypt_job j = {st, payload, off, len, n, t, threads};
        jobs[t] = j;
        pthread_create(&tids[t], NULL, crypt_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; ++t)
        pthread_join(tids[t], NULL);
}

/* CPU-baseline timing (bench.py cpu_baseline): `threads` workers, each
 * re-crypting its round-robin share of the n sessions pass after pass until
 * `seconds` have elapsed (one thread start per worker, not per pass).
 * Returns payload bytes per second over the wall time from the common start
 * to the last worker's finish. */
typedef struct {
    crypt_job job;
    pthread_barrier_t *bar;
    double deadline;
    unsigned long long bytes;
} timed_job;

static void *timed_worker(void *arg)
{
    timed_job *t = (timed_job *)arg;
    crypt_job *j = &t->job;
    pthread_barrier_wait(t->bar);
    unsigned long long bytes = 0;     /* local: the job records share cache lines */
    /* a contiguous share per worker: neighbouring states (1032 B each) and
     * payloads then belong to the same worker, no cache line ping-pong */
    const uint32_t lo = (uint32_t)((uint64_t)j->n * (uint32_t)j->tid / (uint32_t)j->nthreads);
    const uint32_t hi = (uint32_t)((uint64_t)j->n * ((uint32_t)j->tid + 1u) / (uint32_t)j->nthreads);
    do {
        for (uint32_t i = lo; i < hi; ++i) {
            oracle_encryption(&j->st[i], j->payload + j->off[i], (long)j->len[i]);
            bytes += j->len[i];
        }
    } while (oracle_now() < t->deadline);
    t->bytes = bytes;
    return NULL;
}

double oracle_crypt_rate(oracle_rc4_state *st, uint8_t *payload, const uint64_t *off, const uint32_t *len,
                         uint32_t n, int threads, double seconds)
{
    if (threads < 1)
        threads = 1;
    if ((uint32_t)threads > n)
        threads = (int)n;
    pthread_t *tids = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    timed_job *jobs = (timed_job *)calloc((size_t)threads, sizeof(timed_job));
    pthread_barrier_t bar;
    if (!tids || !jobs || pthread_barrier_init(&bar, NULL, (unsigned)threads + 1) != 0) {
        free(tids);
        free(jobs);
        return -1.0;
    }
    int started = 0;
    for (int t = 0; t < threads; ++t) {
        crypt_job j = {st, payload, off, len, n, t, threads};
        jobs[t].job = j;
        jobs[t].bar = &bar;
        jobs[t].deadline = 0.0;
        jobs[t].bytes = 0;
    }
    /* deadline set before the start, read by workers only after the barrier */
    for (int t = 0; t < threads; ++t) {
        if (pthread_create(&tids[t], NULL, timed_worker, &jobs[t]) != 0)
            break;
        ++started;
    }
    if (started != threads) {   /* cannot release the barrier: give up */
        abort();
    }
    const double t0 = oracle_now();
    for (int t = 0; t < threads; ++t)
        jobs[t].deadline = t0 + seconds;
    pthread_barrier_wait(&bar);
    const double tb = oracle_now();
    unsigned long long bytes = 0;
    for (int t = 0; t < threads; ++t) {
        pthread_join(tids[t], NULL);
        bytes += jobs[t].bytes;
    }
    const double t1 = oracle_now();
    pthread_barrier_destroy(&bar);
    free(tids);
    free(jobs);
    return (double)bytes / (t1 - tb);
}

void oracle_state_to_bytes(const oracle_rc4_state *st, uint8_t sbox[256],
                           uint8_t *x, uint8_t *y)
{
    for (int i = 0; i < 256; ++i)
        sbox[i] = (uint8_t)st->box[i];
    *x = (uint8_t)st->x;
    *y = (uint8_t)st->y;
}

void oracle_state_from_bytes(oracle_rc4_state *st, const uint8_t sbox[256],
                             uint8_t x, uint8_t y)
{
    for (int i = 0; i < 256; ++i)
        st->box[i] = sbox[i];
    st->x = x;
    st->y = y;
}

double oracle_now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* proto4z HasRawPacket (depends/proto4z/proto4z.h:704-748), restated:
 * 0 intact (*plen = packet length), 1 shortage, 2 corrupted.  The header
 * length it checks against is sizeof(LenInteger) + sizeof(ProtoInteger) = 6,
 * and the length field is a little-endian u32 (ReadPodData, :684-689). */
static int has_raw_packet(const uint8_t *b, uint32_t cur, uint32_t boundLen, uint32_t maxLen, uint32_t *plen)
{
    if (boundLen < cur || maxLen < boundLen)
        return 2;
    if (cur < 6)
        return 1;
    uint32_t pl = (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
    if (pl < 6)
        return 2;
    if (pl > boundLen)
        return pl > maxLen ? 2 : 1;
    if (pl > maxLen)
        return 2;
    if (pl <= cur) {
        *plen = pl;
        return 0;
    }
    return 1;
}

/* TcpSession::onRecv's framing loop (src/frame/session.cpp:329-371, PT_TCP):
 * walk session i's buffer buf[off[i] .. off[i]+len[i]) with
 * check(begin+used, len-used, bound-used, bound) until shortage (status 1) or
 * corruption (status 2); npk = packets found, used = bytes they cover, the
 * first max_packets lengths go to pkt_len[i*max_packets ..]. */
void oracle_frame_scan(const uint8_t *buf, const uint64_t *off, const uint32_t *len, uint32_t bound,
                       uint32_t n, uint32_t max_packets, uint32_t *npk, uint32_t *used,
                       uint32_t *status, uint32_t *pkt_len)
{
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t *b = buf + off[i];
        uint32_t u = 0, k = 0, st;
        for (;;) {
            uint32_t pl = 0;
            st = (uint32_t)has_raw_packet(b + u, len[i] - u, bound - u, bound, &pl);
            if (st != 0)
                break;
            if (pkt_len && k < max_packets)
                pkt_len[(size_t)i * max_packets + k] = pl;
            ++k;
            u += pl;
        }
        npk[i] = k;
        used[i] = u;
        status[i] = st;
    }
}
