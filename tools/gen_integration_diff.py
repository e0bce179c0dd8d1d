#!/usr/bin/env python3
"""integration/file_operations.diff: the patch a syncr maintainer applies
(`patch -p1` at syncr's root) to put the MI355X chunker behind
compute_file_chunks (src/protocol/file_operations.rs:721-788).

The patch is computed from syncr's own files (read as text) and the edits
below, each anchored on text that must occur exactly once -- so a check run
proves the patch still applies to the reference as it is.  It only adds: the
`gpu` cargo feature and the build script, `mod chunking_gpu`, the batched walk
in traverse_and_stream (every regular file submitted to `GpuWalk`, entries sent
in walk order as results return, a file the engine failed on chunked by the
rollsum loop), and a `compute_file_chunks` that tries the GPU first and
otherwise runs the unchanged rollsum loop, renamed `compute_file_chunks_cpu`.
With the feature off the program is the reference's.  rust/src/chunking_gpu.rs,
rust/src/chunking_gpu_ffi.rs and rust/build.rs are the new files it expects
next to them.

    python tools/gen_integration_diff.py --write   # needs the reference checkout
    python tools/gen_integration_diff.py --check   # exit 1 if the committed diff is stale
"""
import difflib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("SYNCR_REFERENCE", "/root/reference")
OUT = os.path.join(ROOT, "integration", "file_operations.diff")

# (file, anchor, replacement) -- the anchor must occur exactly once in the file
EDITS = [
    ("Cargo.toml",
     'edition = "2018"\n',
     'edition = "2018"\n'
     'build = "build.rs"         # links libsyncr_cdc.so when the `gpu` feature is on\n'),
    ("Cargo.toml",
     'tui = ["ratatui", "crossterm"]\n',
     'tui = ["ratatui", "crossterm"]\n'
     '# MI355X chunk scan + BLAKE3 (libsyncr_cdc.so, src/chunking_gpu.rs); falls back to rollsum\n'
     'gpu = []\n'),
    ("src/lib.rs",
     "pub mod chunking;\n",
     "pub mod chunking;\n"
     "#[cfg(feature = \"gpu\")]\n"
     "pub mod chunking_gpu;\n"),
    # the batched walk: traverse_and_stream (:544-715) hands every regular file
    # to GpuWalk (one pipeline over all GPUs) instead of awaiting
    # compute_file_chunks per file (:599-605); entries still leave in walk order
    ("src/protocol/file_operations.rs",
     "/// Traverses directory tree and streams entries through a channel\n",
     "/// Sends the GPU walk's ready entries in walk order (feature `gpu`); a file the\n"
     "/// engine could not chunk goes through the rollsum loop here.  false when the\n"
     "/// receiver is gone.\n"
     "#[cfg(feature = \"gpu\")]\n"
     "async fn send_ready_gpu_entries(\n"
     "\twalk: &mut crate::chunking_gpu::GpuWalk,\n"
     "\tstate: &DumpState,\n"
     "\tsender: &super::streaming::ListingSender,\n"
     ") -> bool {\n"
     "\twhile let Some(item) = walk.pop_ready(state).await {\n"
     "\t\tlet entry = match item {\n"
     "\t\t\tcrate::chunking_gpu::WalkItem::Ready(e) => e,\n"
     "\t\t\tcrate::chunking_gpu::WalkItem::Cpu(mut e, path) => {\n"
     "\t\t\t\te.chunks = compute_file_chunks_cpu(&path, state).await.unwrap_or_default();\n"
     "\t\t\t\te\n"
     "\t\t\t}\n"
     "\t\t};\n"
     "\t\tif sender.send(Ok(entry)).await.is_err() {\n"
     "\t\t\tdebug!(\"Receiver dropped, terminating directory stream\");\n"
     "\t\t\treturn false;\n"
     "\t\t}\n"
     "\t}\n"
     "\ttrue\n"
     "}\n"
     "\n"
     "/// Traverses directory tree and streams entries through a channel\n"),
    ("src/protocol/file_operations.rs",
     "\tlet mut stack = vec![base_path.clone()];\n",
     "\tlet mut stack = vec![base_path.clone()];\n"
     "\t// GPU chunking (feature `gpu`): every regular file goes to one batched\n"
     "\t// pipeline; entries leave in walk order as their chunk lists come back\n"
     "\t#[cfg(feature = \"gpu\")]\n"
     "\tlet mut gpu_walk = crate::chunking_gpu::GpuWalk::open().await;\n"),
    ("src/protocol/file_operations.rs",
     "\t\t\t// Prepare entry based on type\n",
     "\t\t\t#[cfg(feature = \"gpu\")]\n"
     "\t\t\t{\n"
     "\t\t\t\tif let Some(walk) = gpu_walk.as_mut() {\n"
     "\t\t\t\t\tif !(meta.is_file() || meta.is_symlink() || meta.is_dir()) {\n"
     "\t\t\t\t\t\tcontinue;\n"
     "\t\t\t\t\t}\n"
     "\t\t\t\t\tlet entry = crate::chunking_gpu::walk_entry(&path, relative_path, &meta);\n"
     "\t\t\t\t\tif meta.is_file() {\n"
     "\t\t\t\t\t\twalk.push_file(path, entry).await;\n"
     "\t\t\t\t\t} else {\n"
     "\t\t\t\t\t\tif meta.is_dir() {\n"
     "\t\t\t\t\t\t\tstack.push(path);\n"
     "\t\t\t\t\t\t}\n"
     "\t\t\t\t\t\twalk.push_entry(entry);\n"
     "\t\t\t\t\t}\n"
     "\t\t\t\t\tif !send_ready_gpu_entries(walk, &state, &sender).await {\n"
     "\t\t\t\t\t\treturn Ok(());\n"
     "\t\t\t\t\t}\n"
     "\t\t\t\t\tcontinue;\n"
     "\t\t\t\t}\n"
     "\t\t\t}\n"
     "\n"
     "\t\t\t// Prepare entry based on type\n"),
    ("src/protocol/file_operations.rs",
     "\t\t}\n\t}\n\n\tOk(())\n}\n\n/// Compute chunks for a file using rolling hash\n",
     "\t\t}\n\t}\n\n"
     "\t// the walk's last files: flush the pipeline, send the rest in walk order\n"
     "\t#[cfg(feature = \"gpu\")]\n"
     "\t{\n"
     "\t\tif let Some(mut walk) = gpu_walk {\n"
     "\t\t\twalk.finish().await;\n"
     "\t\t\tsend_ready_gpu_entries(&mut walk, &state, &sender).await;\n"
     "\t\t}\n"
     "\t}\n"
     "\n"
     "\tOk(())\n}\n\n/// Compute chunks for a file using rolling hash\n"),
    ("src/protocol/file_operations.rs",
     "/// Compute chunks for a file using rolling hash\n"
     "///\n"
     "/// This is extracted from get_file_chunks() to be reusable by both\n"
     "/// the blocking and streaming paths.\n"
     "async fn compute_file_chunks(\n",
     "/// Compute chunks for a file: on the GPU (feature `gpu`, src/chunking_gpu.rs),\n"
     "/// falling back to the rollsum loop when the engine is unavailable or fails.\n"
     "#[cfg(feature = \"gpu\")]\n"
     "async fn compute_file_chunks(\n"
     "\tpath: &Path,\n"
     "\tstate: &DumpState,\n"
     ") -> Result<Vec<ChunkInfo>, ProtocolError> {\n"
     "\tif let Some(chunks) = crate::chunking_gpu::compute_file_chunks_gpu(path, state).await {\n"
     "\t\treturn Ok(chunks);\n"
     "\t}\n"
     "\tcompute_file_chunks_cpu(path, state).await\n"
     "}\n"
     "\n"
     "#[cfg(not(feature = \"gpu\"))]\n"
     "async fn compute_file_chunks(\n"
     "\tpath: &Path,\n"
     "\tstate: &DumpState,\n"
     ") -> Result<Vec<ChunkInfo>, ProtocolError> {\n"
     "\tcompute_file_chunks_cpu(path, state).await\n"
     "}\n"
     "\n"
     "/// Compute chunks for a file using rolling hash\n"
     "///\n"
     "/// This is extracted from get_file_chunks() to be reusable by both\n"
     "/// the blocking and streaming paths.\n"
     "async fn compute_file_chunks_cpu(\n"),
]


def make_diff() -> str:
    files = []
    for f, _, _ in EDITS:
        if f not in files:
            files.append(f)
    out = []
    for f in files:
        src = open(os.path.join(REF, f)).read()
        new = src
        for g, anchor, repl in EDITS:
            if g != f:
                continue
            if new.count(anchor) != 1:
                raise SystemExit(f"{f}: anchor occurs {new.count(anchor)} times: {anchor[:60]!r}")
            new = new.replace(anchor, repl)
        out += difflib.unified_diff(src.splitlines(keepends=True), new.splitlines(keepends=True),
                                    fromfile=f"a/{f}", tofile=f"b/{f}", n=3)
    return "".join(out)


def main():
    if not os.path.isdir(REF):
        print(f"{REF} absent: nothing to check", file=sys.stderr)
        return 0
    d = make_diff()
    if "--check" in sys.argv:
        if not os.path.exists(OUT) or open(OUT).read() != d:
            print("integration/file_operations.diff is stale: run tools/gen_integration_diff.py --write",
                  file=sys.stderr)
            return 1
        return 0
    if "--write" in sys.argv:
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        open(OUT, "w").write(d)
        return 0
    sys.stdout.write(d)
    return 0


if __name__ == "__main__":
    sys.exit(main())
