/*
 * syncr_cdc.h -- C ABI of the MI355X-native Bup content-defined chunker.
 *
 * Drop-in boundary for szilu/syncr's chunk scan.  The reference has no plugin
 * API for this path; its seam is the inline call pair
 *     Bup::new_with_chunk_bits(CHUNK_BITS)          src/protocol/file_operations.rs:748
 *     bup.find_chunk_edge(&buf[..endofs])           src/protocol/file_operations.rs:754-755
 * inside the driver loop compute_file_chunks()     src/protocol/file_operations.rs:721-788
 * (and its dead duplicate get_file_chunks(), :190-248).  The entry points below
 * replace that loop: bytes in, chunk boundaries (offset, size) out, bit-exact.
 * The *_hashed variants also return each chunk's BLAKE3 hash, computed on the GPU
 * (util::hash_binary, src/util.rs:57-59, called per chunk at file_operations.rs:757),
 * i.e. complete ChunkInfo records; the caller keeps feeding DumpState::add_chunk
 * (src/serve.rs:36-42) exactly as before.
 *
 * Conventions: every function returns 0 on success or a negative errno-style
 * code (SYNCR_CDC_E*); no C++ exception crosses this boundary.  Inputs and
 * outputs are caller-allocated; the handle owns its device scratch.  A handle is
 * single-threaded (one per device / host thread).  `stream` arguments are HIP
 * streams passed as void* (NULL = the handle's own stream).
 */
#ifndef SYNCR_CDC_H
#define SYNCR_CDC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SYNCR_CDC_ABI_VERSION 3

/* error codes (negative errno values) */
#define SYNCR_CDC_OK 0
#define SYNCR_CDC_EINVAL (-22) /* bad argument / parameter out of range          */
#define SYNCR_CDC_ENOMEM (-12) /* host or device allocation failed               */
#define SYNCR_CDC_ERANGE (-34) /* output capacity too small; *n_out = required   */
#define SYNCR_CDC_ENODEV (-19) /* no such HIP device / HIP runtime unavailable   */
#define SYNCR_CDC_EIO (-5)     /* HIP runtime error while running                 */
#define SYNCR_CDC_ESTATE (-71) /* call out of order (e.g. launch before plan)    */
#define SYNCR_CDC_ENOENT (-2)  /* chunk cache: no valid entry                     */
#define SYNCR_CDC_EBUSY (-16)  /* chunk cache: the log is locked by another handle */

/* Chunker parameters.  Defaults mirror src/chunking.rs:7-13 and the production
 * read path of file_operations.rs:737-776.  `flags` selects an exact
 * alternative resolve (same cuts; for cross-checks only): */
#define SYNCR_CDC_FLAG_RESOLVE_LANE 1u    /* one lane per file instead of one wave */
#define SYNCR_CDC_FLAG_RESOLVE_NOBURST 2u /* wave resolve without the chained-hop burst */
#define SYNCR_CDC_FLAG_RESOLVE_NOSPLIT 4u /* wave resolve without split walks of long files */
#define SYNCR_CDC_FLAG_SPLIT_NOWAIT 8u    /* testing: split-walk workers give up at once, so
                                             every file walker walks its whole file itself */
typedef struct syncr_cdc_params {
    uint32_t chunk_bits; /* CHUNK_BITS, 1..31 (default 20; reference validates 8..32) */
    uint32_t flags;      /* 0, or SYNCR_CDC_FLAG_* (other bits: SYNCR_CDC_EINVAL)     */
    uint64_t max_chunk;  /* MAX_CHUNK_SIZE, 1..2^32-1 (default 16 MiB)                  */
    uint64_t read_cap;   /* bytes per tokio File::read (default 2 MiB); 0 = "ideal"
                            in-memory semantics of tests/chunking_test.rs:170-192       */
} syncr_cdc_params;

/* One chunk: the (offset, size) pair of ChunkInfo (src/protocol/types.rs:24-29)
 * plus the index of the file it belongs to within the call's batch. */
typedef struct syncr_cut {
    uint64_t offset; /* byte offset within its file */
    uint32_t len;    /* chunk size (<= max_chunk)   */
    uint32_t file;   /* file index in the batch     */
} syncr_cut;

/* One chunk with its hash: ChunkInfo{hash: [u8; 32], offset: u64, size: u32}
 * (src/protocol/types.rs:24-29) plus the file index.  hash = blake3::hash of the
 * chunk's bytes (util::hash_binary, src/util.rs:57-59). */
typedef struct syncr_chunk_info {
    uint64_t offset;  /* byte offset within its file */
    uint32_t len;     /* chunk size                  */
    uint32_t file;    /* file index in the batch     */
    uint8_t hash[32]; /* BLAKE3-256 of the chunk     */
} syncr_chunk_info;

typedef struct syncr_cdc syncr_cdc;

int32_t syncr_cdc_abi_version(void);
const char *syncr_cdc_strerror(int32_t code);
/* chunk_bits=20, max_chunk=16 MiB, read_cap=2 MiB (production semantics) */
void syncr_cdc_default_params(syncr_cdc_params *p);
int32_t syncr_cdc_device_count(int32_t *n);

/* Replaces Bup::new_with_chunk_bits: one handle per device, parameters fixed.
 * The library reads no environment variables: its results depend only on the
 * parameters and the bytes.  Handles on one device are independent: several
 * handles = several batches in flight, the next batch's scan taking the GPU as
 * the previous scan's last work units end. */
int32_t syncr_cdc_open(int32_t device, const syncr_cdc_params *p, syncr_cdc **out);
void syncr_cdc_close(syncr_cdc *h);
int32_t syncr_cdc_get_params(const syncr_cdc *h, syncr_cdc_params *p);

/* --- host-memory entry points (end to end: H2D, scan, resolve, D2H) ---------- */
/* One file (compute_file_chunks' loop, file_operations.rs:746-784).  Empty input
 * gives 0 chunks.  If cap is too small returns SYNCR_CDC_ERANGE, *n_out = needed. */
int32_t syncr_cdc_chunk_host(syncr_cdc *h, const uint8_t *data, uint64_t len,
                             syncr_cut *out, uint64_t cap, uint64_t *n_out);
/* Many files laid out in one host buffer of `span` bytes.  Chunks are written
 * file by file (file order of the table); per_file_count[i] gets file i's count. */
int32_t syncr_cdc_chunk_batch_host(syncr_cdc *h, const uint8_t *data, uint64_t span,
                                   const uint64_t *file_off, const uint64_t *file_len,
                                   uint32_t nfiles, syncr_cut *out, uint64_t cap,
                                   uint64_t *per_file_count, uint64_t *n_out);

/* As above, with each chunk's BLAKE3 hash (compute_file_chunks' ChunkInfo list,
 * file_operations.rs:746-784 including the hash_binary call at :757). */
int32_t syncr_cdc_chunk_host_hashed(syncr_cdc *h, const uint8_t *data, uint64_t len,
                                    syncr_chunk_info *out, uint64_t cap, uint64_t *n_out);
int32_t syncr_cdc_chunk_batch_host_hashed(syncr_cdc *h, const uint8_t *data, uint64_t span,
                                          const uint64_t *file_off, const uint64_t *file_len,
                                          uint32_t nfiles, syncr_chunk_info *out, uint64_t cap,
                                          uint64_t *per_file_count, uint64_t *n_out);

/* --- device-resident entry points (what the throughput metric times) ------- */
/* plan: validate + upload the file table (host arrays) for bytes that will be
 * resident in device memory at [d_bytes, d_bytes+span).  Files must not overlap.
 * The host arrays may be reused as soon as plan returns; the device copy of the
 * tables may still be in flight on the handle's own stream, and any launch
 * (on whatever stream) is ordered after it.  Reusable for any number of
 * launches. */
int32_t syncr_cdc_plan(syncr_cdc *h, const uint64_t *file_off, const uint64_t *file_len,
                       uint32_t nfiles, uint64_t span);
/* launch: scan + resolve on `stream`, asynchronous: no host synchronisation and
 * no allocation.  d_bytes must be 16-byte aligned device memory.
 * Buffer lifetime: the bytes at [d_bytes, d_bytes + span) must stay resident
 * and UNMODIFIED until the fetch of this launch returns -- fetch may launch the
 * scan again over the same bytes (a capacity re-run, see
 * syncr_cdc_fetch_reruns), so e.g. the next batch's H2D copy into the same
 * buffer must be ordered after that fetch, not merely after this launch.
 * Streams: all launches of one handle share its device tables.  A launch on a
 * stream other than the previous launch's waits (on the device) for all work
 * enqueued on that previous stream, so launches of one handle never overlap,
 * whatever streams the caller alternates between; a stream passed here must
 * stay valid until the next launch or fetch of the handle.  Because results
 * are only known to be complete at fetch time (re-runs happen inside fetch), a
 * launch captured into a HIP graph still needs syncr_cdc_fetch afterwards; the
 * engine makes no claim beyond that. */
int32_t syncr_cdc_launch(syncr_cdc *h, const uint8_t *d_bytes, void *stream);
/* fetch: wait for the last launch, copy cuts to the host (file by file).  May
 * re-run the launch on its stream first (grown capacities), reading d_bytes
 * again.  The launch's results stay on the host until the next plan or launch:
 * fetching again (e.g. cap 0 for the total, then into a buffer of that size)
 * does not wait for the device again. */
int32_t syncr_cdc_fetch(syncr_cdc *h, syncr_cut *out, uint64_t cap,
                        uint64_t *per_file_count, uint64_t *n_out);
/* launch_hashed: launch, then BLAKE3 of every chunk on the same stream
 * (asynchronous, allocation-free).  fetch_hashed: like fetch, with hashes;
 * returns SYNCR_CDC_ESTATE unless the last launch was a launch_hashed. */
int32_t syncr_cdc_launch_hashed(syncr_cdc *h, const uint8_t *d_bytes, void *stream);
int32_t syncr_cdc_fetch_hashed(syncr_cdc *h, syncr_chunk_info *out, uint64_t cap,
                               uint64_t *per_file_count, uint64_t *n_out);
/* plan + launch + fetch */
int32_t syncr_cdc_chunk_batch_device(syncr_cdc *h, const uint8_t *d_bytes, uint64_t span,
                                     const uint64_t *file_off, const uint64_t *file_len,
                                     uint32_t nfiles, syncr_cut *out, uint64_t cap,
                                     uint64_t *per_file_count, uint64_t *n_out, void *stream);

/* --- wire / on-disk text of chunk lists ---------------------------------------
 * Byte-identical with what the reference emits for a ChunkInfo list
 * (hash = util::hash_to_base64, base64 URL_SAFE with padding, src/util.rs:62-64):
 *   SYNCR_FMT_LIST_LINES  LIST reply, one line per chunk (src/protocol/v3_server.rs:146-182:
 *                         serde_json::to_string(&json!({"typ","off","len","hsh"})) + "\n";
 *                         serde_json's default Map is a BTreeMap, so keys come sorted):
 *                         {"hsh":"<b64>","len":<size>,"off":<offset>,"typ":"C"}\n
 *   SYNCR_FMT_HASHCHUNKS  the "ch" array of a profile FileData (HashChunk's Serialize,
 *                         src/types.rs:117-129, through json5::to_string at
 *                         src/sync_impl/mod.rs:1167-1172): [{"h":"<b64>","of":<offset>,"sz":<size>},...]
 * Writes at most cap bytes (no terminating NUL); *len_out = bytes needed;
 * SYNCR_CDC_ERANGE if cap is too small. */
#define SYNCR_FMT_LIST_LINES 1
#define SYNCR_FMT_HASHCHUNKS 2
int32_t syncr_cdc_format_chunks(const syncr_chunk_info *chunks, uint64_t n, int32_t format, char *out,
                                uint64_t cap, uint64_t *len_out);

/* --- batched ingest pipeline (a whole directory walk) ------------------------
 * Replaces the serial per-file loop of traverse_and_stream
 * (src/protocol/file_operations.rs:544-715, which awaits compute_file_chunks per
 * file at :599-605): files are appended to pinned staging batches of
 * `batch_bytes`; a full batch is copied to the device and chunked + BLAKE3-hashed
 * on its own stream while the next one fills (`depth` batches in flight).  Each
 * file's ChunkInfo list comes back through `cb`, in submission order, on the
 * thread that called submit / flush.  `status` is 0, or -errno for a file that
 * could not be opened or read, following compute_file_chunks: when the open or
 * the first read fails n = 0 (the reference's empty list,
 * file_operations.rs:727-744); when a later read fails, the chunks the
 * reference cuts before its loop breaks (:776-782).  A file is read at its
 * fstat size: one that shrinks while being read is chunked at the length read
 * (status 0); bytes appended after the fstat are not read (the reference reads
 * to EOF).  In callbacks chunk.file
 * is 0.  A file larger than batch_bytes gets a batch of its own.  copy_threads:
 * host threads used for large copies / reads into pinned memory (1 = the caller
 * only). */
typedef struct syncr_ingest syncr_ingest;
typedef void (*syncr_ingest_cb)(void *ctx, uint64_t tag, int32_t status, const syncr_chunk_info *chunks,
                                uint64_t n);
int32_t syncr_ingest_open(int32_t device, const syncr_cdc_params *p, uint64_t batch_bytes, uint32_t depth,
                          uint32_t copy_threads, syncr_ingest_cb cb, void *ctx, syncr_ingest **out);
/* One pipeline over several devices of this process (the reference's host is
 * one process, src/protocol/factory.rs:116-125): devices[k] is the HIP device
 * of sub-pipeline k (a device may repeat: two sub-pipelines on one GPU).  Each
 * sub-pipeline has its own `depth` staging batches, engine handles and streams,
 * and its own worker thread, which reads / copies its files and runs its
 * batches.  Each file goes whole to the sub-pipeline with the fewest bytes
 * assigned so far (files are independent, file_operations.rs:721-788: the
 * online form of LPT by size; no cross-device traffic).  Callbacks still arrive
 * in submission order, on the thread that called submit / flush.  Every
 * syncr_ingest_* call takes the returned handle; syncr_ingest_open is the
 * one-device case (no worker thread).  The copy_threads threads form one pool
 * that the sub-pipelines take turns on. */
int32_t syncr_ingest_open_multi(const int32_t *devices, uint32_t ndevices, const syncr_cdc_params *p,
                                uint64_t batch_bytes, uint32_t depth, uint32_t copy_threads,
                                syncr_ingest_cb cb, void *ctx, syncr_ingest **out);
/* bytes already in memory (copied into the staging batch before returning) */
int32_t syncr_ingest_submit(syncr_ingest *g, const uint8_t *data, uint64_t len, uint64_t tag);
/* a file read with pread straight into pinned staging: opened and sized on the
 * calling thread, read by the copy_threads pool while the caller goes on (the
 * batch waits for its reads when it is sealed).  A file's descriptor stays open
 * until its reads are done; at most 64 files per device are open at once (past
 * that, submit_file runs queued reads on the calling thread, or waits, before it
 * opens the next file), so a walk of many small files never exhausts the
 * process's descriptors. */
int32_t syncr_ingest_submit_file(syncr_ingest *g, const char *path, uint64_t tag);
/* zero-copy: reserve `len` bytes of pinned staging, fill them, then commit */
int32_t syncr_ingest_reserve(syncr_ingest *g, uint64_t len, uint8_t **dst);
int32_t syncr_ingest_commit(syncr_ingest *g, uint64_t tag);
/* seal the current batch and deliver every outstanding file; staging grown
 * past 2 x batch_bytes for an oversized file is released (an idle pipeline
 * holds at most depth x 2 x batch_bytes of pinned and device memory) */
int32_t syncr_ingest_flush(syncr_ingest *g);
/* [files, bytes, batches, chunks] so far */
int32_t syncr_ingest_stats(const syncr_ingest *g, uint64_t *stats4);
/* per sub-pipeline k: stats[4k..4k+3] = [device, files, bytes, batches];
 * SYNCR_CDC_ERANGE if n < 4 * ndevices */
int32_t syncr_ingest_device_stats(const syncr_ingest *g, uint64_t *stats, uint32_t n);
/* Host seconds spent so far, summed over sub-pipelines, per stage: sec[0] copying
 * submitted bytes into pinned staging, [1] waiting for (and helping with) the
 * reads of a batch's files before its H2D (submit_file queues each file's preads
 * on the copy_threads pool, 2 MiB per task, and returns),
 * [2] sealing batches (plan + H2D and kernel enqueue), [3] waiting for a batch's
 * results (fetch: the device side -- H2D, kernels, D2H -- not yet done), [4]
 * per-file delivery (callbacks).  Diagnostics of where an end-to-end run is
 * bound; the first n entries are written. */
int32_t syncr_ingest_timing(const syncr_ingest *g, double *sec, uint32_t n);
/* Fault injection (tests of the read-error contract, file_operations.rs:
 * 727-744, 776-782): every later submit_file reads only the bytes before file
 * offset `offset`; the read that would cross it fails with errno `err`
 * (err = 0: it returns EOF there, as if the file shrank to `offset`).
 * offset = UINT64_MAX (the default) turns it off. Applies to every
 * sub-pipeline; set it before submitting the files it is meant for. */
int32_t syncr_ingest_set_read_fault(syncr_ingest *g, uint64_t offset, int32_t err);
/* release everything; files not yet delivered (no flush since their submit)
 * get no callback */
void syncr_ingest_close(syncr_ingest *g);

/* --- chunk cache (skip re-chunking unchanged files) ---------------------------
 * Restates ChildCache (src/cache.rs:138-260): one entry per key (file path) with
 * the file's mtime, size and ChunkInfo list; valid when mtime (cache.rs:167-179)
 * and size both match.  A cache holds chunk lists cut under ONE set of chunking
 * parameters `p` (NULL = defaults; flags are ignored): the reference's are
 * compile-time constants (src/chunking.rs:7-13), these are runtime values, so
 * they are part of the cache's identity.  Persistent in an append-only log at
 * `path` (NULL = in memory only) that records them in its header; opening a log
 * written under other parameters gives SYNCR_CDC_EINVAL, a file that is not a
 * cache log SYNCR_CDC_EIO, a log locked by another open handle SYNCR_CDC_EBUSY.
 * An empty file (or one torn while its header was written) is a new cache, and
 * so is a log of the ABI-v2 format (magic SYNCRCC1, which did not record the
 * parameters, so none of its lists can be trusted): it is rewritten with the
 * current header on open; a torn tail is dropped on open; a failed append is rolled back and makes later
 * puts fail with SYNCR_CDC_EIO.  get: 0 on a hit, SYNCR_CDC_ENOENT on a miss,
 * SYNCR_CDC_ERANGE (n_out = needed) if cap is short.  Attached to an ingest
 * pipeline (same parameters, else SYNCR_CDC_EINVAL), submit_file serves
 * unchanged files from it and stores every freshly chunked file in it. */
typedef struct syncr_cache syncr_cache;
int32_t syncr_cache_open(const char *path, const syncr_cdc_params *p, syncr_cache **out);
int32_t syncr_cache_get_params(const syncr_cache *c, syncr_cdc_params *p);
int32_t syncr_cache_get(syncr_cache *c, const char *key, uint32_t mtime, uint64_t size, syncr_chunk_info *out,
                        uint64_t cap, uint64_t *n_out);
int32_t syncr_cache_put(syncr_cache *c, const char *key, uint32_t mtime, uint64_t size,
                        const syncr_chunk_info *chunks, uint64_t n);
int32_t syncr_cache_sync(syncr_cache *c);
/* [hits, misses, puts, entries] */
int32_t syncr_cache_stats(syncr_cache *c, uint64_t *stats4);
void syncr_cache_close(syncr_cache *c);
int32_t syncr_ingest_set_cache(syncr_ingest *g, syncr_cache *c);
int32_t syncr_ingest_cache_hits(const syncr_ingest *g, uint64_t *hits);

/* --- device memory / stream / timing helpers (hosts without a GPU framework) -- */
int32_t syncr_cdc_device_alloc(syncr_cdc *h, uint64_t bytes, void **d_ptr);
int32_t syncr_cdc_device_free(syncr_cdc *h, void *d_ptr);
int32_t syncr_cdc_host_alloc_pinned(syncr_cdc *h, uint64_t bytes, void **ptr);
int32_t syncr_cdc_host_free_pinned(syncr_cdc *h, void *ptr);
int32_t syncr_cdc_memcpy_h2d(syncr_cdc *h, void *d_dst, const void *src, uint64_t bytes, void *stream);
int32_t syncr_cdc_memcpy_d2h(syncr_cdc *h, void *dst, const void *d_src, uint64_t bytes, void *stream);
/* Device-to-device copy on the handle's device (building device-resident
 * batches from shared pieces, e.g. the dedup corpus of SURVEY.md §8d config 5). */
int32_t syncr_cdc_memcpy_d2d(syncr_cdc *h, void *d_dst, const void *d_src, uint64_t bytes, void *stream);
/* wait for the handle's work: its own stream and its last launch's stream */
int32_t syncr_cdc_synchronize(syncr_cdc *h);
void *syncr_cdc_stream(syncr_cdc *h);
/* Fill [d_bytes + file_off[i], +file_len[i]) with corpus file number
 * file_index[i] (or first_index+i when file_index is NULL) of the synthetic
 * corpus: xorshift64 seeded 0x9E3779B97F4A7C15*(index+1), 64 outputs discarded,
 * byte=(x>>32)&0xff.  Synchronous. */
int32_t syncr_cdc_gen_corpus(syncr_cdc *h, uint8_t *d_bytes, const uint64_t *file_off,
                             const uint64_t *file_len, const uint64_t *file_index,
                             uint32_t nfiles, uint64_t first_index, void *stream);
/* Streaming-read probe (roofline denominator): reads
 * [d_bytes, d_bytes + bytes) once per pass with 16-byte loads (nt != 0: the
 * non-temporal policy the scan uses), writes nothing, `reps` timed passes on
 * the handle's stream after one warm-up.  ms2 = [best, mean] ms per pass. */
int32_t syncr_cdc_read_probe(syncr_cdc *h, const uint8_t *d_bytes, uint64_t bytes, uint32_t reps,
                             int32_t nt, double *ms2);
/* Per-kernel timing (kernel_times: summed ms of [scan, dense + compaction,
 * resolve] since the last set_timing, and the number of launches):
 *   enable = 1  every phase of each launch bracketed by HIP events on the launch stream;
 *   enable = 2  the scan kernel only, by HIP events bound to its dispatch (as in ABI v2);
 *   enable = 3  the same as 2;
 *   enable = 4  the scan kernel only, by the device's own clock: its first waves
 *               stamp their entry, every wave its exit (wall_clock64, the constant
 *               clock HIP events read), the launch's resolve adds last exit - first
 *               entry to device-side sums -- no packets in the queue, so the timed
 *               launches run exactly as untimed ones (an event pair costs a 1 GiB
 *               batch ~6 % of its step in queue idle);
 *   enable = 0  off.
 * set_timing(4) and kernel_times wait for this handle's streams only (not the
 * whole device). */
int32_t syncr_cdc_set_timing(syncr_cdc *h, int32_t enable);
int32_t syncr_cdc_kernel_times(syncr_cdc *h, double *ms3, uint64_t *launches);
/* The same for up to 4 phases: [scan, dense+compaction, resolve, hash]. */
int32_t syncr_cdc_kernel_times_ex(syncr_cdc *h, double *ms, uint32_t n, uint64_t *launches);
/* Diagnostics of the last fetched launch: [candidates, dense_tiles, tiles, overflow]. */
int32_t syncr_cdc_last_stats(syncr_cdc *h, uint64_t *stats4);
/* Split walks of long files (wave resolve) in the last fetched launch:
 * [worker waves launched (0: none), files_split, segments, segments walked by the split
 * workers, segments adopted by their file's walker, worker give-ups].  A worker
 * waits only for file walkers to publish their segments; it gives up (and
 * leaves the rest to the file walkers, which never wait) after ~100 ms. */
int32_t syncr_cdc_split_stats(syncr_cdc *h, uint64_t *stats6);
/* Capacity re-runs the fetches since the handle's last launch performed before
 * their results were complete (0: that launch fitted every capacity). A caller
 * timing launches it has not yet fetched checks this: launches before a re-run
 * ran with the smaller capacities. */
int32_t syncr_cdc_fetch_reruns(syncr_cdc *h, uint64_t *reruns);
/* Which scan kernel the last launch ran (the library's own choice, made per
 * launch from the batch size and the handle's history; a capacity re-run inside
 * fetch counts as a launch).  kind: one of SYNCR_CDC_SCAN_*; info4 (may be NULL) =
 * [kind, tiles, scan waves launched, segments per stream of a stream-tile scan
 * (9; 0 for the other scans)]; *name (may be NULL) = the kernel's symbol
 * name as a profiler shows it. */
#define SYNCR_CDC_SCAN_NONE 0         /* no launch yet, or an empty batch             */
#define SYNCR_CDC_SCAN_STREAM_TILES 1 /* cdc_scan_st_kernel: batches >= 24 tiles/wave  */
#define SYNCR_CDC_SCAN_CU 2           /* cdc_scan_kernel, CU schedule: small batches  */
#define SYNCR_CDC_SCAN_TILES 3        /* cdc_scan_kernel, dynamic tile groups: large
                                         batches after a >= 1 % dense-tile batch      */
#define SYNCR_CDC_SCAN_DEV 255        /* development library variant                  */
int32_t syncr_cdc_last_scan(const syncr_cdc *h, uint64_t *info4, const char **name);
/* Engine geometry: [run_bytes, tile_bytes, scan_grid, compute_units,
 * scan_blocks_per_cu, lds_bytes_per_scan_block, device, abi_version]. */
int32_t syncr_cdc_get_info(const syncr_cdc *h, uint64_t *info8);

#ifdef __cplusplus
}
#endif

#endif /* SYNCR_CDC_H */
