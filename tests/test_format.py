"""Wire / on-disk text of chunk lists (syncr_cdc_format_chunks, host code: no GPU).

LIST reply lines: the reference writes serde_json::to_string(&json!({"typ": "C",
"off": offset, "len": size, "hsh": hash_to_base64(hash)})) + "\\n" per chunk
(src/protocol/v3_server.rs:146-182).  serde_json = "1.0" (Cargo.toml:26) is
built without `preserve_order` (no crate in Cargo.toml enables it), so json!
objects are BTreeMaps and serialize with sorted keys, compact.  Profile state:
HashChunk serializes fields h, of, sz in that order (src/types.rs:117-129)
through json5::to_string (src/sync_impl/mod.rs:1167-1172).  The serde_json /
json5 crates are absent here, so this restates their documented output;
consumers parse by key (src/protocol/v3_client.rs:272-300), so only key order
and number/string spelling matter.  Parity unpinned beyond that restatement."""
import base64
import json

import numpy as np

import syncr_amd


def sample(n=5, seed=1):
    rng = np.random.default_rng(seed)
    a = np.zeros(n, syncr_amd.CHUNK_INFO_DTYPE)
    a["offset"] = np.cumsum(rng.integers(1, 1 << 24, n)) - 1
    a["offset"][-1] = (1 << 40) + 7                    # > 32-bit offsets
    a["len"] = rng.integers(1, 1 << 24, n)
    a["len"][0] = 0xFFFFFFFF
    a["hash"] = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    a["hash"][1] = 0xFB                                # '-' / '_' of the URL-safe alphabet
    return a


def b64(h):
    return base64.urlsafe_b64encode(bytes(h)).decode()   # util::hash_to_base64 (util.rs:62-64)


def test_list_lines_match_serde_json_semantics():
    a = sample()
    want = "".join(json.dumps({"typ": "C", "off": int(c["offset"]), "len": int(c["len"]), "hsh": b64(c["hash"])},
                              sort_keys=True, separators=(",", ":")) + "\n" for c in a)
    assert syncr_amd.format_chunks(a, syncr_amd.FMT_LIST_LINES).decode() == want
    assert "-" in want or "_" in want


def test_hashchunk_array():
    a = sample(4, 2)
    want = "[" + ",".join('{"h":"%s","of":%d,"sz":%d}' % (b64(c["hash"]), c["offset"], c["len"]) for c in a) + "]"
    got = syncr_amd.format_chunks(a, syncr_amd.FMT_HASHCHUNKS).decode()
    assert got == want
    assert json.loads(got)[0]["h"] == b64(a["hash"][0])


def test_empty_and_capacity():
    e = np.zeros(0, syncr_amd.CHUNK_INFO_DTYPE)
    assert syncr_amd.format_chunks(e, syncr_amd.FMT_LIST_LINES) == b""
    assert syncr_amd.format_chunks(e, syncr_amd.FMT_HASHCHUNKS) == b"[]"
    import ctypes
    L = syncr_amd.library()
    a = sample(2)
    n = ctypes.c_uint64(0)
    buf = ctypes.create_string_buffer(10)
    assert L.syncr_cdc_format_chunks(a.ctypes.data, 2, 1, buf, 10, ctypes.byref(n)) == syncr_amd.E_RANGE
    assert n.value == len(syncr_amd.format_chunks(a))
    assert L.syncr_cdc_format_chunks(a.ctypes.data, 2, 7, None, 0, ctypes.byref(n)) == -22
