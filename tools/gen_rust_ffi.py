#!/usr/bin/env python3
"""Rust `extern "C"` declarations for every entry point of include/syncr_cdc.h.

INTEGRATION.md's appendix is this script's output; tests/test_capi.py checks
that the appendix matches the header, so a new entry point cannot be left out
of the binding a syncr maintainer would add.

    python tools/gen_rust_ffi.py            # print the block
    python tools/gen_rust_ffi.py --check    # exit 1 if INTEGRATION.md is stale
"""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "syncr_cdc.h")
DOC = os.path.join(ROOT, "INTEGRATION.md")
BEGIN = "<!-- rust-ffi:begin (tools/gen_rust_ffi.py) -->"
END = "<!-- rust-ffi:end -->"

SCALAR = {"int32_t": "i32", "uint32_t": "u32", "uint64_t": "u64", "uint8_t": "u8", "double": "f64",
          "char": "c_char", "void": "c_void"}
STRUCT = {"syncr_cdc_params": "SyncrCdcParams", "syncr_cut": "SyncrCut", "syncr_chunk_info": "SyncrChunkInfo",
          "syncr_cdc": "SyncrCdc", "syncr_ingest": "SyncrIngest", "syncr_cache": "SyncrCache",
          "syncr_ingest_cb": "IngestCb"}


def prototypes(text: str):
    """(return type, name, [(type, name)]) of every syncr_* function declaration."""
    text = re.sub(r"//[^\n]*", "", text)
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    out = []
    for m in re.finditer(r"(^|[;}\n])\s*([A-Za-z_][\w\s\*]*?)\b(syncr_\w+)\s*\(([^;{]*?)\)\s*;", text):
        ret, name, args = m.group(2).strip(), m.group(3), " ".join(m.group(4).split())
        if ret.startswith("typedef"):
            continue
        params = []
        if args and args != "void":
            for a in args.split(","):
                a = a.strip()
                pm = re.match(r"(.*?)([A-Za-z_]\w*)$", a)
                params.append((pm.group(1).strip(), pm.group(2)))
        out.append((ret, name, params))
    return out


def rust_type(c: str) -> str:
    c = " ".join(c.replace("*", " * ").split())
    stars = c.count("*")
    base = c.replace("*", "").strip()
    const = base.startswith("const ")
    base = base.replace("const ", "").strip()
    r = SCALAR.get(base) or STRUCT.get(base)
    if r is None:
        raise SystemExit(f"unmapped C type: {c!r}")
    if stars == 0:
        return "()" if r == "c_void" else r
    # innermost pointer carries the const of the pointee; outer pointers are mutable
    t = ("*const " if const else "*mut ") + r
    for _ in range(stars - 1):
        t = "*mut " + t
    return t


def rust_block(protos) -> str:
    lines = ["```rust", "#[link(name = \"syncr_cdc\")]", "extern \"C\" {"]
    for ret, name, params in protos:
        args = ", ".join(f"{n}: {rust_type(t)}" for t, n in params)
        r = rust_type(ret)
        lines.append(f"    pub fn {name}({args})" + ("" if r == "()" else f" -> {r}") + ";")
    lines += ["}", "```"]
    return "\n".join(lines)


def main():
    block = rust_block(prototypes(open(HEADER).read()))
    if "--check" in sys.argv:
        doc = open(DOC).read()
        i, j = doc.find(BEGIN), doc.find(END)
        cur = doc[i + len(BEGIN):j].strip() if i >= 0 and j > i else None
        if cur != block:
            print("INTEGRATION.md's Rust FFI appendix is stale: run tools/gen_rust_ffi.py --write", file=sys.stderr)
            return 1
        return 0
    if "--write" in sys.argv:
        doc = open(DOC).read()
        i, j = doc.find(BEGIN), doc.find(END)
        if i < 0 or j < i:
            raise SystemExit("INTEGRATION.md has no rust-ffi markers")
        open(DOC, "w").write(doc[:i + len(BEGIN)] + "\n" + block + "\n" + doc[j:])
        return 0
    print(block)
    return 0


if __name__ == "__main__":
    sys.exit(main())
