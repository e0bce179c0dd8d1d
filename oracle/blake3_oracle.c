/*
 * blake3_oracle.c -- CPU restatement of BLAKE3 (unkeyed hash, 32-byte output).
 *
 * TEST INFRASTRUCTURE ONLY.  Linked into liborc_bup.so and loaded by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker of the
 * HIP chunk hasher; the product (syncr_amd, libsyncr_cdc.so) never loads it.
 *
 * What it restates: szilu/syncr hashes every chunk with
 *     util::hash_binary(buf) = *blake3::hash(buf).as_bytes()      src/util.rs:57-59
 * called per chunk at src/protocol/file_operations.rs:757 (and :224 on the dead
 * path), base64url-encoded by util::hash_to_base64 (src/util.rs:62-64).  The
 * `blake3 = "1.8"` crate (Cargo.toml:14) is a third-party dependency absent from
 * /root/reference (no Cargo.lock, no registry, no Rust toolchain here), so this
 * file restates the published BLAKE3 algorithm (the BLAKE3 paper / spec,
 * version 1.x of the crate): 1024-byte chunks of 64-byte blocks compressed with
 * CHUNK_START / CHUNK_END flags, chunk chaining values merged in a left-balanced
 * binary tree of PARENT nodes, the root compressed with ROOT.  It is written in
 * the spec's sequential form (one chunk state + a CV stack), deliberately not in
 * the GPU's leaf / subtree / level decomposition, so the two are independent.
 *
 * Pinning: tests/test_blake3.py checks it against the official BLAKE3 test
 * vectors (input byte i = i % 251; test_vectors.json of the BLAKE3 repository)
 * committed in tests/golden/blake3_vectors.json.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define B3_BLOCK 64
#define B3_CHUNK 1024
enum { CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8 };

static const uint32_t IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                               0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
static const uint8_t PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};

static inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

static inline void g(uint32_t *v, int a, int b, int c, int d, uint32_t mx, uint32_t my) {
    v[a] = v[a] + v[b] + mx;
    v[d] = rotr(v[d] ^ v[a], 16);
    v[c] = v[c] + v[d];
    v[b] = rotr(v[b] ^ v[c], 12);
    v[a] = v[a] + v[b] + my;
    v[d] = rotr(v[d] ^ v[a], 8);
    v[c] = v[c] + v[d];
    v[b] = rotr(v[b] ^ v[c], 7);
}

/* compression function; out[0..8) = the new chaining value */
static void compress(const uint32_t cv[8], const uint8_t block[B3_BLOCK], uint64_t counter,
                     uint32_t block_len, uint32_t flags, uint32_t out[8]) {
    uint32_t m[16], v[16], t[16];
    for (int i = 0; i < 16; i++)
        m[i] = (uint32_t)block[4 * i] | (uint32_t)block[4 * i + 1] << 8 |
               (uint32_t)block[4 * i + 2] << 16 | (uint32_t)block[4 * i + 3] << 24;
    for (int i = 0; i < 8; i++) v[i] = cv[i];
    for (int i = 0; i < 4; i++) v[8 + i] = IV[i];
    v[12] = (uint32_t)counter;
    v[13] = (uint32_t)(counter >> 32);
    v[14] = block_len;
    v[15] = flags;
    for (int r = 0; r < 7; r++) {
        g(v, 0, 4, 8, 12, m[0], m[1]);
        g(v, 1, 5, 9, 13, m[2], m[3]);
        g(v, 2, 6, 10, 14, m[4], m[5]);
        g(v, 3, 7, 11, 15, m[6], m[7]);
        g(v, 0, 5, 10, 15, m[8], m[9]);
        g(v, 1, 6, 11, 12, m[10], m[11]);
        g(v, 2, 7, 8, 13, m[12], m[13]);
        g(v, 3, 4, 9, 14, m[14], m[15]);
        for (int i = 0; i < 16; i++) t[i] = m[PERM[i]];
        memcpy(m, t, sizeof m);
    }
    for (int i = 0; i < 8; i++) out[i] = v[i] ^ v[i + 8];
}

static void words_to_bytes(const uint32_t w[8], uint8_t out[32]) {
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)w[i];
        out[4 * i + 1] = (uint8_t)(w[i] >> 8);
        out[4 * i + 2] = (uint8_t)(w[i] >> 16);
        out[4 * i + 3] = (uint8_t)(w[i] >> 24);
    }
}

/* A node's output before it is known whether it is the root: the inputs of its
 * last compression (the root flag is only added to the final one). */
typedef struct {
    uint32_t cv[8];
    uint8_t block[B3_BLOCK];
    uint64_t counter;
    uint32_t block_len, flags;
} node_t;

static void node_cv(const node_t *n, uint32_t out[8]) {
    compress(n->cv, n->block, n->counter, n->block_len, n->flags, out);
}

/* chunk `index` of the input: bytes [p, p+len), len <= 1024 (len 0 only for
 * the empty input) */
static void chunk_node(const uint8_t *p, size_t len, uint64_t index, node_t *n) {
    uint32_t cv[8];
    memcpy(cv, IV, sizeof cv);
    size_t nblocks = len ? (len + B3_BLOCK - 1) / B3_BLOCK : 1;
    for (size_t b = 0; b + 1 < nblocks; b++) {
        const uint32_t fl = b == 0 ? CHUNK_START : 0;
        compress(cv, p + b * B3_BLOCK, index, B3_BLOCK, fl, cv);
    }
    const size_t last = (nblocks - 1) * B3_BLOCK;
    memcpy(n->cv, cv, sizeof cv);
    memset(n->block, 0, B3_BLOCK);
    memcpy(n->block, p + last, len - last);
    n->counter = index;
    n->block_len = (uint32_t)(len - last);
    n->flags = (nblocks == 1 ? CHUNK_START : 0) | CHUNK_END;
}

static void parent_node(const uint32_t l[8], const uint32_t r[8], node_t *n) {
    memcpy(n->cv, IV, sizeof n->cv);
    words_to_bytes(l, n->block);
    words_to_bytes(r, n->block + 32);
    n->counter = 0;
    n->block_len = B3_BLOCK;
    n->flags = PARENT;
}

/* blake3::hash(in) -> out[32].  Sequential form: chunk CVs pushed on a stack;
 * after chunk k (k >= 1 chunks done, more input to come) merge while the
 * number of completed chunks has trailing zero bits (the spec's lazy merge). */
void orc_blake3(const uint8_t *in, uint64_t len, uint8_t out[32]) {
    uint32_t stack[64][8];
    int depth = 0;
    uint64_t index = 0;
    uint64_t pos = 0;
    while (len - pos > B3_CHUNK) {          /* every chunk except the last */
        node_t n;
        chunk_node(in + pos, B3_CHUNK, index, &n);
        uint32_t cv[8];
        node_cv(&n, cv);
        ++index;
        uint64_t total = index;
        while ((total & 1) == 0) {          /* merge completed subtrees */
            node_t pn;
            parent_node(stack[--depth], cv, &pn);
            node_cv(&pn, cv);
            total >>= 1;
        }
        memcpy(stack[depth++], cv, sizeof cv);
        pos += B3_CHUNK;
    }
    node_t n;
    chunk_node(in + pos, len - pos, index, &n);
    while (depth > 0) {                     /* fold the stack right to left */
        uint32_t cv[8];
        node_cv(&n, cv);
        parent_node(stack[--depth], cv, &n);
    }
    uint32_t w[8];
    compress(n.cv, n.block, n.counter, n.block_len, n.flags | ROOT, w);
    words_to_bytes(w, out);
}

/* Batch: out[32*i] = blake3(base + off[i], len[i]); nthreads workers. */
typedef struct {
    const uint8_t *base;
    const uint64_t *off;
    const uint64_t *len;
    uint64_t n;
    uint8_t *out;
    uint64_t next;
    pthread_mutex_t mu;
} b3job_t;

static void *b3_worker(void *arg) {
    b3job_t *j = (b3job_t *)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        const uint64_t i = j->next;
        j->next += 64;
        pthread_mutex_unlock(&j->mu);
        if (i >= j->n) return NULL;
        const uint64_t e = i + 64 < j->n ? i + 64 : j->n;
        for (uint64_t k = i; k < e; k++) orc_blake3(j->base + j->off[k], j->len[k], j->out + 32 * k);
    }
}

int orc_blake3_batch(const uint8_t *base, const uint64_t *off, const uint64_t *len, uint64_t n,
                     uint8_t *out, int nthreads) {
    b3job_t j = {base, off, len, n, out, 0, PTHREAD_MUTEX_INITIALIZER};
    if (nthreads <= 1) {
        b3_worker(&j);
        return 0;
    }
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nthreads);
    if (!th) return -1;
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, b3_worker, &j);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
    return 0;
}
