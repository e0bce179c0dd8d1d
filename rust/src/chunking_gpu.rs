//! GPU chunking for syncr: the MI355X engine (libsyncr_cdc.so) behind
//! `compute_file_chunks` (src/protocol/file_operations.rs:721-788).
//!
//! Drop this file and `chunking_gpu_ffi.rs` into syncr's `src/`, apply
//! `integration/file_operations.diff` (adds the `gpu` cargo feature, the
//! `build.rs` link step and the two call sites: the batched walk in
//! traverse_and_stream, `GpuWalk`, and compute_file_chunks per file) and build
//! with `--features gpu`.  Without the feature syncr is unchanged.
//!
//! What it replaces: the rollsum loop of compute_file_chunks -- a fresh
//! `Bup::new_with_chunk_bits(CHUNK_BITS)` per chunk (:748), `find_chunk_edge`
//! over at most `min(MAX_CHUNK_SIZE, buffered)` bytes (:749-755), BLAKE3 of the
//! chunk (:757), tokio reads of <= 2 MiB (:738,776).  The engine returns the
//! same `ChunkInfo` list bit for bit (boundaries and hashes) and follows the
//! loop's read-error behaviour: open or first read fails -> no chunks
//! (:727-744), a later read fails -> the chunks cut before it (:776-782).
//!
//! Safety: the crate is `#![deny(unsafe_code)]` (src/lib.rs:36); this module
//! opts out locally, as src/util.rs:16-23 does for `geteuid`.  Every unsafe
//! block is a call into the C ABI with pointers that outlive the call.
//!
//! Threading: a handle (`SyncrCdc`, `SyncrIngest`) is single-threaded.  The
//! async caller runs the blocking calls on tokio's blocking pool
//! (`spawn_blocking`), taking a pipeline from a small pool so that each is used
//! by one thread at a time (compute_file_chunks runs on a dedicated runtime
//! thread for local nodes, src/protocol/factory.rs:118-125, or on the main
//! runtime under `syncr serve`, src/serve.rs:273-279).
#![allow(unsafe_code)]

use std::collections::VecDeque;
use std::ffi::{CStr, CString};
use std::fs;
use std::os::raw::c_void;
use std::os::unix::ffi::OsStrExt;
use std::os::unix::fs::MetadataExt;
use std::path::{Path, PathBuf};
use std::sync::atomic::{AtomicUsize, Ordering};
use std::sync::Mutex;

use tracing::warn;

use crate::chunking;
use crate::protocol::types::{ChunkInfo, FileSystemEntry, FileSystemEntryType};
use crate::serve::DumpState;
use crate::util;

#[path = "chunking_gpu_ffi.rs"]
mod ffi;
use ffi::*;

/// Bytes one tokio `File::read` returns at most (its DEFAULT_MAX_BUF_SIZE): the
/// lookahead of the production loop (file_operations.rs:738,776), which cuts at
/// the read boundary when no edge is buffered.  The saved profile state
/// (src/sync_impl/mod.rs:1167-1172) holds these cuts, so they are kept.
pub const TOKIO_READ_CAP: u64 = 2 * 1024 * 1024;

/// Staging batch of a per-file pipeline: files up to this size share it, a
/// larger file gets a batch of its own.
const FILE_BATCH_BYTES: u64 = 64 << 20;

/// The chunking parameters of src/chunking.rs:7-13 with the production read cap.
pub fn params() -> SyncrCdcParams {
    SyncrCdcParams {
        chunk_bits: chunking::CHUNK_BITS,
        flags: 0,
        max_chunk: chunking::MAX_CHUNK_SIZE as u64,
        read_cap: TOKIO_READ_CAP,
    }
}

/// A failure of the native engine (negative errno, SYNCR_CDC_E*).  The caller
/// falls back to the rollsum loop: the listing never fails because of the GPU.
#[derive(Debug, Clone, Copy, PartialEq, Eq)]
pub struct GpuError(pub i32);

impl std::fmt::Display for GpuError {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        // SAFETY: syncr_cdc_strerror returns a static NUL-terminated string for any code.
        let s = unsafe { CStr::from_ptr(syncr_cdc_strerror(self.0)) };
        write!(f, "syncr_cdc: {} ({})", s.to_string_lossy(), self.0)
    }
}

impl std::error::Error for GpuError {}

fn check(rc: i32) -> Result<(), GpuError> {
    if rc == SYNCR_CDC_OK {
        Ok(())
    } else {
        Err(GpuError(rc))
    }
}

fn to_chunk_info(c: &SyncrChunkInfo) -> ChunkInfo {
    ChunkInfo { hash: c.hash, offset: c.offset, size: c.len }
}

/// Number of HIP devices (0 when the runtime or the GPU is absent).
pub fn device_count() -> i32 {
    let mut n = 0i32;
    // SAFETY: n outlives the call.
    if unsafe { syncr_cdc_device_count(&mut n) } == SYNCR_CDC_OK {
        n
    } else {
        0
    }
}

// ---------------------------------------------------------------------------
// Bytes already in memory: one engine handle (Bup::new_with_chunk_bits).
// ---------------------------------------------------------------------------

/// One engine handle on one device, for callers that hold a file's bytes.
pub struct GpuChunker {
    h: *mut SyncrCdc,
}

// SAFETY: the handle is used by one thread at a time (&mut self); it may move
// between threads.
unsafe impl Send for GpuChunker {}

impl GpuChunker {
    pub fn open(device: i32) -> Result<Self, GpuError> {
        let mut h = std::ptr::null_mut();
        // SAFETY: params() and h outlive the call.
        check(unsafe { syncr_cdc_open(device, &params(), &mut h) })?;
        Ok(GpuChunker { h })
    }

    /// compute_file_chunks' `ChunkInfo` list for `data` (boundaries of the
    /// rollsum loop, hashes of blake3::hash).  The output capacity is a guess;
    /// on SYNCR_CDC_ERANGE the engine reports the exact count and the call is
    /// repeated once with that capacity.
    pub fn chunk(&mut self, data: &[u8]) -> Result<Vec<ChunkInfo>, GpuError> {
        let blank = SyncrChunkInfo { offset: 0, len: 0, file: 0, hash: [0; 32] };
        let mut out = vec![blank; data.len() / (1 << 16) + 16];
        let mut n = 0u64;
        for _ in 0..2 {
            // SAFETY: data and out are live for the call; cap is out's length.
            let rc = unsafe {
                syncr_cdc_chunk_host_hashed(self.h, data.as_ptr(), data.len() as u64, out.as_mut_ptr(),
                                            out.len() as u64, &mut n)
            };
            if rc == SYNCR_CDC_ERANGE {
                out.resize(n as usize, blank);
                continue;
            }
            check(rc)?;
            return Ok(out[..n as usize].iter().map(to_chunk_info).collect());
        }
        Err(GpuError(SYNCR_CDC_ERANGE))
    }
}

impl Drop for GpuChunker {
    fn drop(&mut self) {
        // SAFETY: h came from syncr_cdc_open and is closed once.
        unsafe { syncr_cdc_close(self.h) }
    }
}

// ---------------------------------------------------------------------------
// Files by path: the ingest pipeline reads them (pread into pinned staging).
// ---------------------------------------------------------------------------

/// What the pipeline delivered for one file: its status (0, or -errno when the
/// open or a read failed) and the chunks the reference keeps in that case.
#[derive(Debug)]
pub struct FileResult {
    pub tag: u64,
    pub status: i32,
    pub chunks: Vec<ChunkInfo>,
}

/// Results land here from the engine's callback, on the thread that called
/// submit / flush, in submission order.
#[derive(Default)]
struct Inbox {
    done: VecDeque<FileResult>,
}

extern "C" fn deliver(ctx: *mut c_void, tag: u64, status: i32, chunks: *const SyncrChunkInfo, n: u64) {
    // SAFETY: ctx is the Box<Inbox> of the pipeline that registered this callback,
    // alive until its close; the engine calls back only inside submit / flush.
    let inbox = unsafe { &mut *(ctx as *mut Inbox) };
    let list = if n == 0 {
        Vec::new()
    } else {
        // SAFETY: the engine passes n valid records for the duration of the call.
        unsafe { std::slice::from_raw_parts(chunks, n as usize) }.iter().map(to_chunk_info).collect()
    };
    inbox.done.push_back(FileResult { tag, status, chunks: list });
}

/// A batched ingest pipeline: `syncr_ingest_open` on one device, or
/// `syncr_ingest_open_multi` over several (each file goes whole to the
/// least-loaded device; files are independent, file_operations.rs:721-788).
pub struct GpuPipeline {
    g: *mut SyncrIngest,
    inbox: Box<Inbox>,
}

// SAFETY: one thread at a time (&mut self); the pipeline may move between threads.
unsafe impl Send for GpuPipeline {}

impl GpuPipeline {
    /// One device, `depth` batches in flight.
    pub fn open(device: i32, batch_bytes: u64, depth: u32, copy_threads: u32) -> Result<Self, GpuError> {
        let mut inbox = Box::new(Inbox::default());
        let ctx = &mut *inbox as *mut Inbox as *mut c_void;
        let mut g = std::ptr::null_mut();
        // SAFETY: params(), g and the boxed inbox (ctx) outlive the call; the inbox
        // lives as long as the pipeline.
        check(unsafe { syncr_ingest_open(device, &params(), batch_bytes, depth, copy_threads, deliver, ctx, &mut g) })?;
        Ok(GpuPipeline { g, inbox })
    }

    /// Every GPU of the node from this one process (src/protocol/factory.rs:116-125).
    pub fn open_all_devices(batch_bytes: u64, depth: u32, copy_threads: u32) -> Result<Self, GpuError> {
        let devices: Vec<i32> = (0..device_count()).collect();
        if devices.is_empty() {
            return Err(GpuError(SYNCR_CDC_ENODEV));
        }
        let mut inbox = Box::new(Inbox::default());
        let ctx = &mut *inbox as *mut Inbox as *mut c_void;
        let mut g = std::ptr::null_mut();
        // SAFETY: as in open(); devices outlives the call.
        check(unsafe {
            syncr_ingest_open_multi(devices.as_ptr(), devices.len() as u32, &params(), batch_bytes, depth,
                                    copy_threads, deliver, ctx, &mut g)
        })?;
        Ok(GpuPipeline { g, inbox })
    }

    /// Queue a file (read with pread into pinned staging).  Results of earlier
    /// files may be delivered meanwhile: collect them with `take_done`.
    pub fn submit_file(&mut self, path: &Path, tag: u64) -> Result<(), GpuError> {
        let p = CString::new(path.as_os_str().as_bytes()).map_err(|_| GpuError(SYNCR_CDC_EINVAL))?;
        // SAFETY: p outlives the call.
        check(unsafe { syncr_ingest_submit_file(self.g, p.as_ptr(), tag) })
    }

    /// Seal the current batch and deliver every outstanding file.
    pub fn flush(&mut self) -> Result<(), GpuError> {
        // SAFETY: g is open.
        check(unsafe { syncr_ingest_flush(self.g) })
    }

    /// Results delivered so far, in submission order.
    pub fn take_done(&mut self) -> impl Iterator<Item = FileResult> + '_ {
        self.inbox.done.drain(..)
    }

    /// compute_file_chunks(path) on this pipeline: submit, flush, the one result.
    pub fn chunk_file(&mut self, path: &Path) -> Result<FileResult, GpuError> {
        self.inbox.done.clear();
        self.submit_file(path, 0)?;
        self.flush()?;
        self.inbox.done.pop_front().ok_or(GpuError(SYNCR_CDC_EIO))
    }
}

impl Drop for GpuPipeline {
    fn drop(&mut self) {
        // SAFETY: g came from syncr_ingest_open(_multi) and is closed once; the
        // inbox is dropped after the close returns (no callback after it).
        unsafe { syncr_ingest_close(self.g) }
    }
}

// ---------------------------------------------------------------------------
// The call site in compute_file_chunks (see integration/file_operations.diff).
// ---------------------------------------------------------------------------

/// Idle per-file pipelines (depth 1), one taken per blocking call.  The walk's
/// semaphore (file_operations.rs:599) bounds how many are ever open.
static POOL: Mutex<Vec<GpuPipeline>> = Mutex::new(Vec::new());
static NEXT_DEVICE: AtomicUsize = AtomicUsize::new(0);
/// Set once a pipeline could not be opened (no GPU): later calls go straight
/// to the rollsum loop.
static UNAVAILABLE: Mutex<Option<GpuError>> = Mutex::new(None);

fn take_pipeline() -> Result<GpuPipeline, GpuError> {
    if let Some(e) = *UNAVAILABLE.lock().unwrap_or_else(|p| p.into_inner()) {
        return Err(e);
    }
    if let Some(p) = POOL.lock().unwrap_or_else(|p| p.into_inner()).pop() {
        return Ok(p);
    }
    let n = device_count().max(1) as usize;
    let device = (NEXT_DEVICE.fetch_add(1, Ordering::Relaxed) % n) as i32;
    GpuPipeline::open(device, FILE_BATCH_BYTES, 1, 4).map_err(|e| {
        *UNAVAILABLE.lock().unwrap_or_else(|p| p.into_inner()) = Some(e);
        e
    })
}

fn chunk_file_blocking(path: PathBuf) -> Result<FileResult, GpuError> {
    let mut p = take_pipeline()?;
    let r = p.chunk_file(&path);
    if r.is_ok() {
        POOL.lock().unwrap_or_else(|p| p.into_inner()).push(p);       // an engine error drops the pipeline
    }
    r
}

/// compute_file_chunks (file_operations.rs:721-788) on the GPU: the same
/// `ChunkInfo` list, every chunk registered with `DumpState::add_chunk`
/// (:761-762), the reference's warnings on a failed open or read.  `None` when
/// the engine is unavailable or failed: the caller runs its rollsum loop.
pub async fn compute_file_chunks_gpu(path: &Path, state: &DumpState) -> Option<Vec<ChunkInfo>> {
    let owned = path.to_path_buf();
    let res = match tokio::task::spawn_blocking(move || chunk_file_blocking(owned)).await {
        Ok(Ok(r)) => r,
        Ok(Err(e)) => {
            warn!("GPU chunking of {} failed ({}); using the CPU loop", path.display(), e);
            return None;
        }
        Err(_) => return None,
    };
    if needs_cpu(&res) {
        return None;
    }
    warn_read_status(path, &res);
    for c in &res.chunks {
        state.add_chunk(util::hash_to_base64(&c.hash), path.to_path_buf(), c.offset, c.size as usize).await;
    }
    Some(res.chunks)
}

/// A file the engine could not take for lack of memory (its pinned staging and
/// device buffer are sized to the file: a file larger than what can be pinned
/// or allocated on the GPU gets SYNCR_CDC_ENOMEM and no chunks).  That is not a
/// read error of the reference's loop, which streams the file through 16 MiB,
/// so the file goes to the rollsum loop.
fn needs_cpu(res: &FileResult) -> bool {
    res.status == SYNCR_CDC_ENOMEM && res.chunks.is_empty()
}

/// The reference's warning for a file the engine could not read completely
/// (its status is -errno).  With no chunks the open (:730) or the first read
/// (:741) failed: the two are told apart by opening the file again (only on
/// this error path).  With chunks a later read failed (:780) and the chunks cut
/// before it are kept, as the reference's loop keeps them (:776-782): a failed
/// later read always follows a first read of >= 1 byte, which yields a chunk.
fn warn_read_status(path: &Path, res: &FileResult) {
    if res.status == 0 {
        return;
    }
    let err = std::io::Error::from_raw_os_error(-res.status);
    if !res.chunks.is_empty() {
        warn!("Error reading file {}: {}", path.display(), err);
    } else if fs::File::open(path).is_err() {
        warn!("Cannot open file {}: {}", path.display(), err);
    } else {
        warn!("Cannot read file {}: {}", path.display(), err);
    }
}

// ---------------------------------------------------------------------------
// The walk's call site: traverse_and_stream (file_operations.rs:544-715), see
// integration/file_operations.diff.  Instead of awaiting compute_file_chunks
// per file (:599-605), every regular file goes to ONE batched pipeline over all
// GPUs of the node, and the entries are sent (:707) in the walk's order as the
// files' ChunkInfo lists come back.
// ---------------------------------------------------------------------------

/// The walk's pipeline: 256 MiB staging batches (~5 ms of H2D each), three in
/// flight (reads of one, H2D + kernels of another, results of a third), 16
/// threads for the reads into pinned staging.
const WALK_BATCH_BYTES: u64 = 256 << 20;
const WALK_DEPTH: u32 = 3;
const WALK_COPY_THREADS: u32 = 16;

/// The FileSystemEntry traverse_and_stream builds for a file, symlink or
/// directory (:608-620, :668-680, :683-695), chunks still empty.
pub fn walk_entry(path: &Path, relative_path: PathBuf, meta: &fs::Metadata) -> FileSystemEntry {
    let (entry_type, size, target) = if meta.is_file() {
        (FileSystemEntryType::File, meta.size(), None)
    } else if meta.is_symlink() {
        (FileSystemEntryType::SymLink, 0, fs::read_link(path).ok())
    } else {
        (FileSystemEntryType::Directory, 0, None)
    };
    FileSystemEntry {
        entry_type,
        path: relative_path,
        mode: meta.mode(),
        user_id: meta.uid(),
        group_id: meta.gid(),
        created_time: meta.ctime() as u32,
        modified_time: meta.mtime() as u32,
        size,
        target,
        needs_data_transfer: None,
        chunks: Vec::new(),
    }
}

/// What the walk sends next (pop_ready).
pub enum WalkItem {
    /// the entry, complete (a file's chunks filled in, each registered with
    /// DumpState::add_chunk)
    Ready(FileSystemEntry),
    /// a file the engine could not chunk (it failed, or the file does not fit
    /// its memory): the caller runs the rollsum loop on the path and sends the
    /// entry with those chunks
    Cpu(FileSystemEntry, PathBuf),
}

enum Slot {
    Ready,
    Waiting,
    Done(FileResult),
    Cpu,
}

struct Queued {
    entry: FileSystemEntry,
    path: PathBuf,
    slot: Slot,
}

/// The batched walk.  Entries are queued in walk order; a file's entry is
/// ready once its result is back, and pop_ready only ever hands out the head
/// of the queue, so the listing's order is the reference's.  The pipeline's
/// blocking calls run on tokio's blocking pool (spawn_blocking), moving the
/// pipeline there and back: one thread uses it at a time.
pub struct GpuWalk {
    pipe: Option<GpuPipeline>,
    queue: VecDeque<Queued>,
    /// walk positions of the submitted files still without a result, in
    /// submission order = the order the pipeline delivers them
    waiting: VecDeque<u64>,
    /// entries popped so far (walk position of the queue's head)
    popped: u64,
}

impl GpuWalk {
    /// A pipeline over every GPU of the node; None (the walk then awaits the
    /// rollsum loop per file, as the reference does) when there is none.
    pub async fn open() -> Option<GpuWalk> {
        let opened = tokio::task::spawn_blocking(|| {
            GpuPipeline::open_all_devices(WALK_BATCH_BYTES, WALK_DEPTH, WALK_COPY_THREADS)
        })
        .await;
        match opened {
            Ok(Ok(pipe)) => Some(GpuWalk { pipe: Some(pipe), queue: VecDeque::new(), waiting: VecDeque::new(), popped: 0 }),
            Ok(Err(e)) => {
                warn!("GPU chunking unavailable ({}); chunking on the CPU", e);
                None
            }
            Err(_) => None,
        }
    }

    /// A regular file met by the walk: submitted to the pipeline, which reads
    /// it on its own threads (and may run a full batch and deliver earlier
    /// files meanwhile).
    pub async fn push_file(&mut self, path: PathBuf, entry: FileSystemEntry) {
        let pos = self.popped + self.queue.len() as u64;
        let mut pipe = match self.pipe.take() {
            Some(p) => p,
            None => {
                self.queue.push_back(Queued { entry, path, slot: Slot::Cpu });
                return;
            }
        };
        self.queue.push_back(Queued { entry, path: path.clone(), slot: Slot::Waiting });
        self.waiting.push_back(pos);
        let done = tokio::task::spawn_blocking(move || {
            let r = pipe.submit_file(&path, pos);
            (pipe, r)
        })
        .await;
        match done {
            Ok((pipe, r)) => {
                self.pipe = Some(pipe);
                self.collect();
                match r {
                    Ok(()) => {}
                    // this file alone could not be staged (its buffers, sized to the
                    // file, did not fit): the call returned without queueing it, so no
                    // result will come for it -- it goes to the rollsum loop, the walk
                    // goes on on the GPU
                    Err(GpuError(SYNCR_CDC_ENOMEM)) if self.waiting.back() == Some(&pos) => {
                        self.waiting.pop_back();
                        let i = (pos - self.popped) as usize;
                        self.queue[i].slot = Slot::Cpu;
                    }
                    Err(e) => self.engine_failed(e),
                }
            }
            Err(_) => self.engine_failed(GpuError(SYNCR_CDC_EIO)),   // the pipeline went down with the task
        }
    }

    /// A directory or symlink entry: sent in its place in the walk's order.
    pub fn push_entry(&mut self, entry: FileSystemEntry) {
        self.queue.push_back(Queued { entry, path: PathBuf::new(), slot: Slot::Ready });
    }

    /// The head of the queue once it is ready, in walk order.
    pub async fn pop_ready(&mut self, state: &DumpState) -> Option<WalkItem> {
        match self.queue.front() {
            Some(q) if !matches!(q.slot, Slot::Waiting) => {}
            _ => return None,
        }
        let Queued { mut entry, path, slot } = self.queue.pop_front()?;
        self.popped += 1;
        match slot {
            Slot::Done(res) if needs_cpu(&res) => Some(WalkItem::Cpu(entry, path)),
            Slot::Done(res) => {
                warn_read_status(&path, &res);
                for c in &res.chunks {
                    state.add_chunk(util::hash_to_base64(&c.hash), path.clone(), c.offset, c.size as usize).await;
                }
                entry.chunks = res.chunks;
                Some(WalkItem::Ready(entry))
            }
            Slot::Cpu => Some(WalkItem::Cpu(entry, path)),
            Slot::Ready | Slot::Waiting => Some(WalkItem::Ready(entry)),
        }
    }

    /// The walk is over: flush the pipeline so that every entry becomes ready.
    pub async fn finish(&mut self) {
        let mut pipe = match self.pipe.take() {
            Some(p) => p,
            None => return,
        };
        let done = tokio::task::spawn_blocking(move || {
            let r = pipe.flush();
            (pipe, r)
        })
        .await;
        match done {
            Ok((pipe, r)) => {
                self.pipe = Some(pipe);
                self.collect();
                if let Err(e) = r {
                    self.engine_failed(e);
                } else if !self.waiting.is_empty() {
                    self.engine_failed(GpuError(SYNCR_CDC_EIO));   // flush delivers every file
                }
            }
            Err(_) => self.engine_failed(GpuError(SYNCR_CDC_EIO)),
        }
    }

    /// Results delivered by the last pipeline call, matched to their files.
    fn collect(&mut self) {
        if let Some(pipe) = self.pipe.as_mut() {
            for r in pipe.take_done() {
                if let Some(pos) = self.waiting.pop_front() {
                    let i = (pos - self.popped) as usize;
                    self.queue[i].slot = Slot::Done(r);
                }
            }
        }
    }

    /// The engine failed: the pipeline is closed, and every file still without
    /// a result (and every later one) goes to the rollsum loop -- the listing
    /// never fails because of the GPU (file_operations.rs:622-643).
    fn engine_failed(&mut self, e: GpuError) {
        warn!("GPU chunking failed ({}); the rest of the walk is chunked on the CPU", e);
        self.pipe = None;
        for pos in self.waiting.drain(..) {
            let i = (pos - self.popped) as usize;
            self.queue[i].slot = Slot::Cpu;
        }
    }
}
