#!/usr/bin/env python3
"""Rust FFI of include/syncr_cdc.h, generated from the header.

Two outputs, both checked by tests/test_capi.py so that a new or changed entry
point cannot be left out of the binding a syncr maintainer adds:

  * rust/src/chunking_gpu_ffi.rs -- the complete module: constants, #[repr(C)]
    structs, opaque handle types, the callback type and the extern "C" block
    (included by rust/src/chunking_gpu.rs as `mod ffi`);
  * INTEGRATION.md's appendix -- the extern "C" block alone.

    python tools/gen_rust_ffi.py            # print the extern block
    python tools/gen_rust_ffi.py --write    # rewrite both outputs
    python tools/gen_rust_ffi.py --check    # exit 1 if either is stale
"""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "syncr_cdc.h")
DOC = os.path.join(ROOT, "INTEGRATION.md")
FFI_RS = os.path.join(ROOT, "rust", "src", "chunking_gpu_ffi.rs")
BEGIN = "<!-- rust-ffi:begin (tools/gen_rust_ffi.py) -->"
END = "<!-- rust-ffi:end -->"

SCALAR = {"int32_t": "i32", "uint32_t": "u32", "uint64_t": "u64", "uint8_t": "u8", "double": "f64",
          "char": "c_char", "void": "c_void"}
STRUCT = {"syncr_cdc_params": "SyncrCdcParams", "syncr_cut": "SyncrCut", "syncr_chunk_info": "SyncrChunkInfo",
          "syncr_cdc": "SyncrCdc", "syncr_ingest": "SyncrIngest", "syncr_cache": "SyncrCache",
          "syncr_ingest_cb": "IngestCb"}


def strip_comments(text: str) -> str:
    text = re.sub(r"//[^\n]*", "", text)
    return re.sub(r"/\*.*?\*/", "", text, flags=re.S)


def split_params(args: str):
    params = []
    if args and args != "void":
        for a in args.split(","):
            a = a.strip()
            pm = re.match(r"(.*?)([A-Za-z_]\w*)$", a)
            params.append((pm.group(1).strip(), pm.group(2)))
    return params


def prototypes(text: str):
    """(return type, name, [(type, name)]) of every syncr_* function declaration."""
    text = strip_comments(text)
    out = []
    for m in re.finditer(r"(^|[;}\n])\s*([A-Za-z_][\w\s\*]*?)\b(syncr_\w+)\s*\(([^;{]*?)\)\s*;", text):
        ret, name, args = m.group(2).strip(), m.group(3), " ".join(m.group(4).split())
        if ret.startswith("typedef"):
            continue
        out.append((ret, name, split_params(args)))
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


def extern_lines(protos, pub: bool = True):
    lines = ["#[link(name = \"syncr_cdc\")]", "extern \"C\" {"]
    for ret, name, params in protos:
        args = ", ".join(f"{n}: {rust_type(t)}" for t, n in params)
        r = rust_type(ret)
        lines.append(f"    {'pub ' if pub else ''}fn {name}({args})" + ("" if r == "()" else f" -> {r}") + ";")
    lines.append("}")
    return lines


def rust_block(protos) -> str:
    return "\n".join(["```rust", *extern_lines(protos), "```"])


def defines(text: str):
    """(name, rust type, value) of every integer #define (not include guards)."""
    out = []
    for m in re.finditer(r"^#define\s+(SYNCR_\w+)\s+\(?(-?\d+)(u?)\)?", text, flags=re.M):
        name, val, uns = m.group(1), int(m.group(2)), m.group(3)
        out.append((name, "u32" if uns else "i32", val))
    return out


def structs(text: str):
    """(rust name, [(rust type, field)]) of every `typedef struct x { ... } x;`."""
    text = strip_comments(text)
    out = []
    for m in re.finditer(r"typedef\s+struct\s+(\w+)\s*\{(.*?)\}\s*(\w+)\s*;", text, flags=re.S):
        fields = []
        for f in m.group(2).split(";"):
            f = " ".join(f.split())
            if not f:
                continue
            fm = re.match(r"(.*?)([A-Za-z_]\w*)\s*(\[(\d+)\])?$", f)
            ty = rust_type(fm.group(1))
            if fm.group(3):
                ty = f"[{ty}; {fm.group(4)}]"
            fields.append((ty, fm.group(2)))
        out.append((STRUCT[m.group(3)], fields))
    return out


def opaque(text: str):
    return [STRUCT[m.group(2)] for m in re.finditer(r"typedef\s+struct\s+(\w+)\s+(\w+)\s*;", strip_comments(text))]


def callbacks(text: str):
    out = []
    for m in re.finditer(r"typedef\s+(\w+)\s*\(\*\s*(\w+)\)\s*\(([^)]*)\)\s*;", strip_comments(text)):
        args = ", ".join(f"{n}: {rust_type(t)}" for t, n in split_params(" ".join(m.group(3).split())))
        r = rust_type(m.group(1))
        out.append(f"pub type {STRUCT[m.group(2)]} = extern \"C\" fn({args})" + ("" if r == "()" else f" -> {r}") + ";")
    return out


def ffi_module(text: str) -> str:
    L = ["// @generated by tools/gen_rust_ffi.py from include/syncr_cdc.h -- do not edit;",
         "// tests/test_capi.py fails when this file and the header disagree.",
         "//",
         "// Raw bindings of libsyncr_cdc.so (the MI355X chunker's C ABI).  The safe",
         "// wrappers are in chunking_gpu.rs, which includes this file as `mod ffi`.",
         "#![allow(dead_code, non_camel_case_types)]",
         "",
         "use std::os::raw::{c_char, c_void};",
         ""]
    for name, ty, val in defines(text):
        L.append(f"pub const {name}: {ty} = {val};")
    L.append("")
    for name, fields in structs(text):
        derive = "#[derive(Clone, Copy, Debug)]"
        L += ["#[repr(C)]", derive, f"pub struct {name} {{"]
        L += [f"    pub {f}: {t}," for t, f in fields]
        L += ["}", ""]
    for name in opaque(text):
        L += ["#[repr(C)]", f"pub struct {name} {{", "    _private: [u8; 0],", "}", ""]
    L += callbacks(text)
    L.append("")
    L += extern_lines(prototypes(text))
    return "\n".join(L) + "\n"


def doc_block_current():
    doc = open(DOC).read()
    i, j = doc.find(BEGIN), doc.find(END)
    return doc[i + len(BEGIN):j].strip() if i >= 0 and j > i else None


def main():
    text = open(HEADER).read()
    block = rust_block(prototypes(text))
    mod = ffi_module(text)
    if "--check" in sys.argv:
        rc = 0
        if doc_block_current() != block:
            print("INTEGRATION.md's Rust FFI appendix is stale: run tools/gen_rust_ffi.py --write", file=sys.stderr)
            rc = 1
        if not os.path.exists(FFI_RS) or open(FFI_RS).read() != mod:
            print("rust/src/chunking_gpu_ffi.rs is stale: run tools/gen_rust_ffi.py --write", file=sys.stderr)
            rc = 1
        return rc
    if "--write" in sys.argv:
        doc = open(DOC).read()
        i, j = doc.find(BEGIN), doc.find(END)
        if i < 0 or j < i:
            raise SystemExit("INTEGRATION.md has no rust-ffi markers")
        open(DOC, "w").write(doc[:i + len(BEGIN)] + "\n" + block + "\n" + doc[j:])
        os.makedirs(os.path.dirname(FFI_RS), exist_ok=True)
        open(FFI_RS, "w").write(mod)
        return 0
    print(block)
    return 0


if __name__ == "__main__":
    sys.exit(main())
