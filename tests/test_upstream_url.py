"""build_upstream_url behaviour (reference tunnel/src/serve.rs:296-359) + quirk Q1."""
import pytest

CASES = [
    ("http://localhost:3001", "/", "/models", "http://localhost:3001/models"),          # default prefix
    ("http://localhost:3001", "/v1", "/v1/models", "http://localhost:3001/models"),     # with prefix
    ("http://localhost:3001/", "/v1/", "/v1/models", "http://localhost:3001/models"),   # trailing slashes
    ("http://localhost:3001", "", "/chat/completions", "http://localhost:3001/chat/completions"),  # empty
    ("http://localhost:3001", "/v1", "/v1", "http://localhost:3001/"),                  # exact prefix
    ("http://localhost:3001", "/v1", "/health", "http://localhost:3001/health"),        # no match
    ("http://localhost:3001", "/api/v1", "/api/v1/chat/completions",
     "http://localhost:3001/chat/completions"),                                         # nested
]


@pytest.mark.parametrize("base,prefix,path,want", CASES)
def test_build_upstream_url(native, base, prefix, path, want):
    assert native.build_upstream_url(base, prefix, path) == want


def test_prefix_strip_has_no_segment_boundary(native):
    # Q1 (serve.rs:177-179): "/v1beta" with prefix "/v1" strips to "beta". Kept for parity.
    assert native.build_upstream_url("http://h:1", "/v1", "/v1beta/x") == "http://h:1beta/x"


def test_query_string_preserved(native):
    assert native.build_upstream_url("http://h:1", "/v1", "/v1/models?x=1") == "http://h:1/models?x=1"
