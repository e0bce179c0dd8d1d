import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(TESTS, "golden")


def pytest_configure(config):
    if os.environ.get("SYNCR_TEST_DEV_LIBRARY"):       # diagnostics: run the suite on libsyncr_cdc_dev.so
        import syncr_amd
        syncr_amd.use_dev_library()
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests of the HIP engine")
    config.addinivalue_line("markers", "slow: long-running (full BASELINE sizes)")


@pytest.fixture(scope="session")
def kat_cases():
    with open(os.path.join(GOLDEN, "kat_cases.json")) as f:
        return json.load(f)["cases"]


@pytest.fixture(scope="session")
def uniform_corpus_golden():
    with open(os.path.join(GOLDEN, "corpus_uniform_1024x1MiB.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def chunkers():
    """Cache of syncr_amd.Chunker handles keyed by (bits, max_chunk, read_cap)."""
    import syncr_amd

    cache = {}

    def get(bits=20, max_chunk=16 << 20, read_cap=2 << 20):
        key = (bits, max_chunk, read_cap)
        if key not in cache:
            cache[key] = syncr_amd.Chunker(bits, max_chunk, read_cap)
        return cache[key]

    yield get
    for c in cache.values():
        c.close()
