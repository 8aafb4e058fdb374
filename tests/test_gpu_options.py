"""hlc_ctx_set_option / hlc_ctx_get_option (include/hlc.h HLC_OPT_*): every option's documented range.
Each endpoint is accepted and reads back as set, and one value on each side outside the range is
rejected with HLC_EINVAL and leaves the value unchanged.  Options that take any non-negative value or
act as booleans are checked at representative values.  (A range check that slipped onto the wrong
option, as happened to HLC_OPT_POOL_BIND during round 6, fails here.)"""
import pytest

from hashgraph_like_consensus import _ffi

pytestmark = pytest.mark.gpu

# name: (valid values, values rejected); the read-back of a valid value is the value itself unless
# READBACK says otherwise
RANGES = {
    "host_threads": ([1, 16, 64], [0, 65, -1]),
    "pool_bind": ([0, 1, 2], [-1, 3]),
    "host_trace": ([0, 1, 2], [-1, 3]),
    "first_batch": ([0, 1, 8, 64], [-1, 65]),
    "rest_pieces": ([1, 3, 64], [0, 65]),
    "wire_front_cap": ([0, 1536, 1 << 20], [-1]),
    "wire_walk": ([-1, 0, 1], [-2, 2]),
    "early_comb": ([0, 1, 2, 3], [-1, 4]),
    "split_votes": ([0, 98304], [-2]),
    "wire_split_bytes": ([0, 8 << 20], [-2]),
    "wire_chunk": ([4096, 4 << 20], [0, -1]),
}
READBACK = {("wire_chunk", 1): 4096}
BOOLEANS = ("nt_copy", "rec_force_exact", "serial_stages", "wire_pipeline")


def test_gpu_option_ranges(engine):
    names = set(RANGES) | set(BOOLEANS) | {"split_votes_append", "wire_split_bytes_append"}
    assert names == set(_ffi.OPTIONS), "every option is covered"
    for name, (good, bad) in RANGES.items():
        before = engine.get_option(name)
        try:
            for v in good:
                engine.set_option(name, v)
                assert engine.get_option(name) == READBACK.get((name, v), v), (name, v)
            last = engine.get_option(name)
            for v in bad:
                with pytest.raises(_ffi.HlcError):
                    engine.set_option(name, v)
                assert engine.get_option(name) == last, (name, v)
        finally:
            engine.set_option(name, -1 if name in _ffi.LIST_OPTIONS else before)
    for name in BOOLEANS:
        before = engine.get_option(name)
        try:
            for v, want in ((0, 0), (1, 1), (7, 1)):
                engine.set_option(name, v)
                assert engine.get_option(name) == want, (name, v)
        finally:
            engine.set_option(name, before)
    # wire_chunk below 4 KiB reads as 4 KiB (as the environment's value does)
    engine.set_option("wire_chunk", 1)
    assert engine.get_option("wire_chunk") == 4096
    engine.set_option("wire_chunk", 4 << 20)


def test_gpu_option_lists_and_defaults(engine):
    """The range-size lists take appended entries (at most 16) and reset to the library default with
    -1; a fresh context's defaults are the documented ones."""
    from hashgraph_like_consensus.engine import Engine
    engine.set_option("split_votes", [1000, 2000, 4000])
    assert engine.get_option("split_votes") == 1000
    for _ in range(13):
        engine.set_option("split_votes_append", 5)
    with pytest.raises(_ffi.HlcError):  # the 17th entry
        engine.set_option("split_votes_append", 5)
    engine.set_option("split_votes", -1)
    assert engine.get_option("split_votes") == 98304
    fresh = Engine(0)
    try:
        assert fresh.get_option("early_comb") == 1
        assert fresh.get_option("wire_front_cap") == 1536
        assert fresh.get_option("rest_pieces") == 3
        assert fresh.get_option("wire_split_bytes") == 8 << 20
        assert fresh.get_option("wire_walk") == -1
    finally:
        fresh.close()
