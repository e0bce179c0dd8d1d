/*
 * bup_oracle.c -- CPU restatement of szilu/syncr's content-defined chunker.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity *checker* (and the timed
 * CPU baseline, "kind": "port").  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product (syncr_amd /
 * libsyncr_cdc.so) never links, loads or calls anything under oracle/.
 *
 * What it restates (all citations relative to /root/reference):
 *   - parameters          src/chunking.rs:7,10,13  (CHUNK_BITS=20, MAX=16 MiB)
 *   - rollsum::Bup        third-party crate `rollsum = "0.3"` (Cargo.toml:24),
 *                         NOT present on disk (no Cargo.lock, no registry).  Its
 *                         published algorithm (bup's bupsplit.c: WINDOW=64,
 *                         CHAR_OFFSET=31, digest=(s1<<16)|(s2&0xffff), edge at
 *                         i+1 when digest&mask==mask) is restated in bup_*()
 *                         below; call sites src/protocol/file_operations.rs:
 *                         748,754-755 and tests/chunking_test.rs:176,179.
 *   - production driver   compute_file_chunks, file_operations.rs:721-788,
 *                         including tokio's <=2 MiB-per-read behaviour
 *                         (tokio "1", Cargo.toml:29; DEFAULT_MAX_BUF_SIZE).
 *   - ideal driver        tests/chunking_test.rs:170-192 (chunk_data).
 *
 * Two independent formulations live here:
 *   (i)  orc_chunk_production / orc_chunk_ideal: byte-at-a-time Bup state
 *        machine driven literally like the reference loops (16 MiB buffer,
 *        emulated reads, copy_within).
 *   (ii) orc_chunk_closed_form: prefix-sum closed form of the window sums plus
 *        a serial resolve with the chunk-head (first 63 bytes) fix-up -- the
 *        same decomposition the GPU engine uses, computed on the CPU.
 * They must agree; tests/test_oracle.py checks them against each other and
 * against the Appendix-A known-answer vectors of SURVEY.md.
 *
 * Parity status: pinned by the reference's own structural tests
 * (tests/chunking_test.rs, tests/protocol_list_test.rs:305-400) and by two
 * independent restatements; no reference-produced cut offsets exist
 * (rollsum is absent and Rust cannot run here) -- see DESIGN.md "Oracle".
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#define BUP_WINDOW 64u
#define BUP_CHAR_OFFSET 31u

/* ---------------------------------------------------------------------- */
/* (i) literal rollsum::Bup state machine                                 */
/* ---------------------------------------------------------------------- */
typedef struct {
    uint64_t s1, s2;             /* usize in the crate */
    uint8_t window[BUP_WINDOW];
    uint32_t wofs;
    uint32_t chunk_bits;
} bup_t;

/* Bup::new_with_chunk_bits (file_operations.rs:748) */
static void bup_init(bup_t *b, uint32_t bits) {
    b->s1 = BUP_WINDOW * BUP_CHAR_OFFSET;                        /* 1984   */
    b->s2 = BUP_WINDOW * (BUP_WINDOW - 1) * BUP_CHAR_OFFSET;     /* 124992 */
    memset(b->window, 0, sizeof b->window);
    b->wofs = 0;
    b->chunk_bits = bits;
}

/* Bup::roll_byte / Bup::add */
static inline void bup_roll_byte(bup_t *b, uint8_t newch) {
    uint8_t prevch = b->window[b->wofs];
    b->s1 += newch;
    b->s1 -= prevch;
    b->s2 += b->s1;
    b->s2 -= BUP_WINDOW * ((uint64_t)prevch + BUP_CHAR_OFFSET);
    b->window[b->wofs] = newch;
    b->wofs = (b->wofs + 1) & (BUP_WINDOW - 1);
}

/* Bup::digest */
static inline uint32_t bup_digest(const bup_t *b) {
    return ((uint32_t)b->s1 << 16) | ((uint32_t)b->s2 & 0xffffu);
}

/* Bup::find_chunk_edge: returns i+1 of the first edge, 0 if none. */
static uint64_t bup_find_chunk_edge(bup_t *b, const uint8_t *buf, uint64_t len) {
    const uint32_t mask = (uint32_t)((1ull << b->chunk_bits) - 1);
    for (uint64_t i = 0; i < len; i++) {
        bup_roll_byte(b, buf[i]);
        if ((bup_digest(b) & mask) == mask) {
            bup_init(b, b->chunk_bits); /* reset() */
            return i + 1;
        }
    }
    return 0;
}

/* Emitted cut: we store END offsets (offset+size); offsets follow. */
typedef struct {
    uint64_t *ends;
    uint64_t cap;
    uint64_t n;
} sink_t;

static inline void sink_push(sink_t *s, uint64_t end) {
    if (s->n < s->cap) s->ends[s->n] = end;
    s->n++;
}

/* tokio::fs::File::read emulation: min(space, read_cap, remaining). */
static uint64_t emu_read(const uint8_t *file, uint64_t F, uint64_t *fpos,
                         uint8_t *dst, uint64_t space, uint64_t read_cap) {
    uint64_t want = space;
    if (read_cap && want > read_cap) want = read_cap;
    if (want > F - *fpos) want = F - *fpos;
    if (want) memcpy(dst, file + *fpos, want);
    *fpos += want;
    return want;
}

/*
 * compute_file_chunks (file_operations.rs:721-788), literally: a MAX-byte
 * buffer (:737), first read (:738), fresh Bup per chunk (:748),
 * endofs=min(MAX,n) (:749-752), edge or endofs (:754-755), copy_within (:771),
 * refill read (:776).  read_cap = 0 means unlimited reads.
 * Returns the number of chunks; writes up to ends_cap end offsets.
 */
uint64_t orc_chunk_production(const uint8_t *file, uint64_t F, uint32_t bits,
                              uint64_t max_chunk, uint64_t read_cap,
                              uint64_t *ends, uint64_t ends_cap) {
    sink_t sk = {ends, ends_cap, 0};
    if (F == 0) return 0;
    uint8_t *buf = (uint8_t *)malloc(max_chunk);
    if (!buf) return UINT64_MAX;
    uint64_t fpos = 0;
    uint64_t n = emu_read(file, F, &fpos, buf, max_chunk, read_cap);
    uint64_t offset = 0;
    bup_t b;
    while (n > 0) {
        bup_init(&b, bits);
        uint64_t endofs = max_chunk;
        if (endofs > n) endofs = n;
        uint64_t edge = bup_find_chunk_edge(&b, buf, endofs);
        uint64_t count = edge ? edge : endofs;
        sink_push(&sk, offset + count);
        memmove(buf, buf + count, n - count);
        offset += count;
        n -= count;
        n += emu_read(file, F, &fpos, buf + n, max_chunk - n, read_cap);
    }
    free(buf);
    return sk.n;
}

/*
 * compute_file_chunks over a file whose bytes from offset P on cannot be read:
 * each read returns the bytes before P it asks for (a short read at P), and a
 * non-empty read starting at P fails, which breaks the loop (:776-782) and drops
 * whatever was buffered but not yet cut.  P = 0: the first read fails (:738-743),
 * no chunks.  Checks the ingest pipeline's read_error_keep rule (ingest_logic.h).
 */
uint64_t orc_chunk_production_read_error(const uint8_t *file, uint64_t P, uint32_t bits,
                                         uint64_t max_chunk, uint64_t read_cap,
                                         uint64_t *ends, uint64_t ends_cap) {
    sink_t sk = {ends, ends_cap, 0};
    if (P == 0) return 0;
    uint8_t *buf = (uint8_t *)malloc(max_chunk);
    if (!buf) return UINT64_MAX;
    uint64_t fpos = 0;
    uint64_t n = emu_read(file, P, &fpos, buf, max_chunk, read_cap);
    uint64_t offset = 0;
    bup_t b;
    while (n > 0) {
        bup_init(&b, bits);
        uint64_t endofs = max_chunk;
        if (endofs > n) endofs = n;
        uint64_t edge = bup_find_chunk_edge(&b, buf, endofs);
        uint64_t count = edge ? edge : endofs;
        sink_push(&sk, offset + count);
        memmove(buf, buf + count, n - count);
        offset += count;
        n -= count;
        if (max_chunk - n > 0 && fpos == P) break;       /* the read at P fails */
        n += emu_read(file, P, &fpos, buf + n, max_chunk - n, read_cap);
    }
    free(buf);
    return sk.n;
}

/*
 * The same loop with the buffer as a window into the file instead of a
 * memmove'd copy: buf[0..n) of the literal loop is always file[offset ..
 * offset + n) (reads are sequential), so the Bup state machine, the reads and
 * the cuts are identical; only copy_within's O(n) move per chunk is gone.  The
 * literal loop costs ~max_chunk bytes of memmove per chunk, which on data with a
 * cut every 64 bytes (the dense workload) is ~2^18 x the scan itself; tests use
 * this variant for such inputs, and test_oracle.py checks it against the literal
 * loop.
 */
uint64_t orc_chunk_production_window(const uint8_t *file, uint64_t F, uint32_t bits,
                                     uint64_t max_chunk, uint64_t read_cap,
                                     uint64_t *ends, uint64_t ends_cap) {
    sink_t sk = {ends, ends_cap, 0};
    const uint64_t cap = read_cap ? read_cap : UINT64_MAX;
    uint64_t R = F < max_chunk ? F : max_chunk;             /* bytes read so far (:738) */
    if (R > cap) R = cap;
    uint64_t offset = 0;
    bup_t b;
    while (R > offset) {                                      /* n = R - offset > 0 (:747) */
        bup_init(&b, bits);
        const uint64_t n = R - offset;
        const uint64_t endofs = n < max_chunk ? n : max_chunk;
        const uint64_t edge = bup_find_chunk_edge(&b, file + offset, endofs);
        const uint64_t count = edge ? edge : endofs;
        offset += count;
        sink_push(&sk, offset);
        uint64_t want = max_chunk - (R - offset);             /* f.read(&mut buf[n..]) (:776) */
        if (want > cap) want = cap;
        if (want > F - R) want = F - R;
        R += want;
    }
    return sk.n;
}

/* chunk_data (tests/chunking_test.rs:170-192): in-memory "ideal" semantics. */
uint64_t orc_chunk_ideal(const uint8_t *data, uint64_t len, uint32_t bits,
                         uint64_t max_chunk, uint64_t *ends, uint64_t ends_cap) {
    sink_t sk = {ends, ends_cap, 0};
    uint64_t pos = 0;
    bup_t b;
    while (pos < len) {
        bup_init(&b, bits);
        uint64_t end = pos + max_chunk < len ? pos + max_chunk : len;
        uint64_t edge = bup_find_chunk_edge(&b, data + pos, end - pos);
        uint64_t count = edge ? edge : end - pos;
        pos += count;
        sink_push(&sk, pos);
    }
    return sk.n;
}

/* Digest of a fresh Bup after rolling buf[0..n) (rollsum selftest style). */
uint32_t orc_digest_after(const uint8_t *buf, uint64_t n) {
    bup_t b;
    bup_init(&b, 20);
    for (uint64_t i = 0; i < n; i++) bup_roll_byte(&b, buf[i]);
    return bup_digest(&b);
}

/* ---------------------------------------------------------------------- */
/* (ii) closed form + serial resolve                                      */
/* ---------------------------------------------------------------------- */
/*
 * With S = sum of the last 64 bytes and W = sum (age+1)*byte (bytes before the
 * chunk start read as 0): s1 = 1984 + S, s2 = 124992 + W.  Edge iff
 * ((s1<<16)|(s2&0xffff)) & mask == mask.
 */
static inline int hit_sw(uint32_t S, uint32_t W, uint32_t mask) {
    uint32_t dg = ((1984u + S) << 16) | ((124992u + W) & 0xffffu);
    return (dg & mask) == mask;
}

/* First chunk-local hit in [s, min(s+63, lim)) with zeros before s. */
static uint64_t head_hit(const uint8_t *x, uint64_t s, uint64_t lim, uint32_t mask) {
    uint32_t S = 0, W = 0;
    uint64_t e = s + 63 < lim ? s + 63 : lim;
    for (uint64_t p = s; p < e; p++) {
        S += x[p];
        W += S;
        if (hit_sw(S, W & 0xffffu, mask)) return p;
    }
    return UINT64_MAX;
}

static uint64_t closed_form_impl(const uint8_t *x, uint64_t F, uint32_t bits,
                                 uint64_t max_chunk, uint64_t read_cap,
                                 uint64_t *ends, uint64_t ends_cap, int head_fixup) {
    sink_t sk = {ends, ends_cap, 0};
    if (F == 0) return 0;
    const uint32_t mask = (uint32_t)((1ull << bits) - 1);
    /* G(p) for every p from prefix sums: P1 = sum x, P2 = sum q*x (mod 2^64). */
    uint8_t *G = (uint8_t *)calloc(F, 1);
    uint64_t *P1 = (uint64_t *)malloc((F + 1) * 8), *P2 = (uint64_t *)malloc((F + 1) * 8);
    if (!G || !P1 || !P2) { free(G); free(P1); free(P2); return UINT64_MAX; }
    P1[0] = P2[0] = 0;
    for (uint64_t q = 0; q < F; q++) {
        P1[q + 1] = P1[q] + x[q];
        P2[q + 1] = P2[q] + (q + 1) * (uint64_t)x[q];   /* weight (q+1) */
    }
    for (uint64_t p = 0; p < F; p++) {
        uint64_t lo = p + 1 >= 64 ? p + 1 - 64 : 0;     /* window [lo, p] */
        uint64_t S = P1[p + 1] - P1[lo];
        /* W = sum_{q} (p - q + 1) x_q = (p+2) S - sum (q+1) x_q */
        uint64_t W = (p + 2) * S - (P2[p + 1] - P2[lo]);
        G[p] = (uint8_t)hit_sw((uint32_t)S, (uint32_t)(W & 0xffffu), mask);
    }
    free(P1); free(P2);
    const uint64_t cap = read_cap ? read_cap : UINT64_MAX;
    uint64_t R = F < max_chunk ? F : max_chunk;
    if (R > cap) R = cap;
    uint64_t s = 0;
    while (s < R) {
        uint64_t lim = R, e = UINT64_MAX;
        /* head: positions s..s+62 need zeros before s (none needed at s==0). */
        if (s > 0 && head_fixup) e = head_hit(x, s, lim, mask);
        if (e == UINT64_MAX)
            for (uint64_t p = (s > 0 && head_fixup ? s + 63 : s); p < lim; p++)
                if (G[p]) { e = p; break; }
        uint64_t cut = e != UINT64_MAX ? e + 1 : lim;
        sink_push(&sk, cut);
        s = cut;
        uint64_t room = max_chunk - (R - s), rd = room;
        if (rd > cap) rd = cap;
        if (rd > F - R) rd = F - R;
        R += rd;
    }
    free(G);
    return sk.n;
}

uint64_t orc_chunk_closed_form(const uint8_t *x, uint64_t F, uint32_t bits,
                               uint64_t max_chunk, uint64_t read_cap,
                               uint64_t *ends, uint64_t ends_cap) {
    return closed_form_impl(x, F, bits, max_chunk, read_cap, ends, ends_cap, 1);
}

/* DELIBERATELY WRONG variant (uses the file-global G at every position, i.e.
 * skips the chunk-head fix-up).  Only used to SEARCH for adversarial inputs
 * on which the head fix-up changes the cuts (tests/golden/make_golden.py). */
uint64_t orc_chunk_no_head_fixup(const uint8_t *x, uint64_t F, uint32_t bits,
                                 uint64_t max_chunk, uint64_t read_cap,
                                 uint64_t *ends, uint64_t ends_cap) {
    return closed_form_impl(x, F, bits, max_chunk, read_cap, ends, ends_cap, 0);
}

/* ---------------------------------------------------------------------- */
/* data generators and digests (test/bench fixtures)                       */
/* ---------------------------------------------------------------------- */
/* xorshift64 (13,7,17); byte = (x>>32)&0xff after each step. */
void orc_xorshift_fill(uint64_t seed, uint64_t discard, uint8_t *out, uint64_t n) {
    uint64_t x = seed;
    for (uint64_t i = 0; i < discard; i++) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; }
    for (uint64_t i = 0; i < n; i++) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        out[i] = (uint8_t)(x >> 32);
    }
}

/* Corpus file seed: 0x9E3779B97F4A7C15 * (i+1) mod 2^64, 64 outputs discarded. */
uint64_t orc_corpus_seed(uint64_t i) { return 0x9E3779B97F4A7C15ull * (i + 1); }

void orc_corpus_fill(const uint64_t *offs, const uint64_t *lens, uint64_t nfiles,
                     uint64_t first_index, uint8_t *base) {
    for (uint64_t i = 0; i < nfiles; i++)
        orc_xorshift_fill(orc_corpus_seed(first_index + i), 64, base + offs[i], lens[i]);
}

/* FNV-1a-64 over cut end offsets (KAT 4/5). */
uint64_t orc_fnv_ends(const uint64_t *ends, uint64_t n) {
    uint64_t h = 0xcbf29ce484222325ull;
    for (uint64_t i = 0; i < n; i++) h = (h ^ ends[i]) * 0x100000001b3ull;
    return h;
}

/* ---------------------------------------------------------------------- */
/* batch driver over threads (full-size parity + CPU baseline)             */
/* ---------------------------------------------------------------------- */
typedef struct {
    const uint8_t *base;
    const uint64_t *offs, *lens, *out_base, *out_cap;
    uint64_t *counts, *ends;
    uint64_t nfiles;
    uint32_t bits;
    uint64_t max_chunk, read_cap;
    int mode;               /* 0 production (literal), 1 ideal (literal), 2 closed form,
                               3 production without copy_within's memmove (window) */
    uint64_t next;          /* work queue (atomic) */
} batch_t;

static void *batch_worker(void *arg) {
    batch_t *B = (batch_t *)arg;
    for (;;) {
        uint64_t i = __atomic_fetch_add(&B->next, 1, __ATOMIC_RELAXED);
        if (i >= B->nfiles) break;
        const uint8_t *f = B->base + B->offs[i];
        uint64_t *e = B->ends + B->out_base[i];
        uint64_t c;
        if (B->mode == 1)
            c = orc_chunk_ideal(f, B->lens[i], B->bits, B->max_chunk, e, B->out_cap[i]);
        else if (B->mode == 2)
            c = orc_chunk_closed_form(f, B->lens[i], B->bits, B->max_chunk, B->read_cap, e, B->out_cap[i]);
        else if (B->mode == 3)
            c = orc_chunk_production_window(f, B->lens[i], B->bits, B->max_chunk, B->read_cap, e, B->out_cap[i]);
        else
            c = orc_chunk_production(f, B->lens[i], B->bits, B->max_chunk, B->read_cap, e, B->out_cap[i]);
        B->counts[i] = c;
    }
    return NULL;
}

/* Files are taken in the given order by a shared counter (callers pass
 * largest-first for balance).  Returns 0. */
int orc_chunk_batch(const uint8_t *base, const uint64_t *offs, const uint64_t *lens,
                    uint64_t nfiles, uint32_t bits, uint64_t max_chunk, uint64_t read_cap,
                    int mode, const uint64_t *out_base, const uint64_t *out_cap,
                    uint64_t *ends, uint64_t *counts, int nthreads) {
    batch_t B = {base, offs, lens, out_base, out_cap, counts, ends, nfiles, bits,
                 max_chunk, read_cap, mode, 0};
    if (nthreads < 1) nthreads = 1;
    if (nthreads == 1) { batch_worker(&B); return 0; }
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * nthreads);
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, batch_worker, &B);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
    return 0;
}
