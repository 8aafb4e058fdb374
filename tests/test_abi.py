"""The drop-in boundary: libhlc.so loads (no GPU needed), exports every entry point include/hlc.h
declares, and the ctypes / numpy layouts match the C structs; ABI constants agree with the oracle."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import pyoracle as po
from hashgraph_like_consensus import _ffi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "hlc.h")


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|void|uint64_t|const char\*)\s+(hlc_[a-z0-9_]+)\(", text, re.M)))


def header_defines():
    text = open(HEADER).read()
    return {m.group(1): int(m.group(2)) for m in re.finditer(r"#define\s+(HLC_[A-Z0-9_]+)\s+\(?(-?\d+)\)?", text)}


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_ffi.LIB_PATH)
    names = declared_functions()
    assert len(names) >= 13
    for name in names:
        assert hasattr(lib, name), f"libhlc.so does not export {name}"
    assert set(names) == set(_ffi.EXPORTED_SYMBOLS)


def test_abi_version():
    lib = _ffi.load_library()
    assert lib.hlc_abi_version() == header_defines()["HLC_ABI_VERSION"]


def test_status_codes_match_oracle():
    d = header_defines()
    pairs = {
        "HLC_OK": po.OK, "HLC_PROPOSAL_EXPIRED": po.PROPOSAL_EXPIRED,
        "HLC_VOTE_PROPOSAL_ID_MISMATCH": po.VOTE_PROPOSAL_ID_MISMATCH, "HLC_EMPTY_VOTE_OWNER": po.EMPTY_VOTE_OWNER,
        "HLC_EMPTY_VOTE_HASH": po.EMPTY_VOTE_HASH, "HLC_EMPTY_SIGNATURE": po.EMPTY_SIGNATURE,
        "HLC_INVALID_VOTE_HASH": po.INVALID_VOTE_HASH, "HLC_SIGNATURE_SCHEME": po.SIGNATURE_SCHEME,
        "HLC_INVALID_VOTE_SIGNATURE": po.INVALID_VOTE_SIGNATURE,
        "HLC_TIMESTAMP_OLDER_THAN_CREATION": po.TIMESTAMP_OLDER_THAN_CREATION, "HLC_VOTE_EXPIRED": po.VOTE_EXPIRED,
        "HLC_RECEIVED_HASH_MISMATCH": po.RECEIVED_HASH_MISMATCH, "HLC_PARENT_HASH_MISMATCH": po.PARENT_HASH_MISMATCH,
        "HLC_DUPLICATE_VOTE": po.DUPLICATE_VOTE, "HLC_MAX_ROUNDS_EXCEEDED": po.MAX_ROUNDS_EXCEEDED,
        "HLC_PROPOSAL_ALREADY_EXIST": po.PROPOSAL_ALREADY_EXIST, "HLC_SCHEME_SIG_LEN": po.SCHEME_SIG_LEN,
        "HLC_SCHEME_ID_LEN": po.SCHEME_ID_LEN, "HLC_SCHEME_BAD_PARITY": po.SCHEME_BAD_PARITY,
        "HLC_SCHEME_SCALAR_RANGE": po.SCHEME_SCALAR_RANGE, "HLC_SCHEME_NO_POINT": po.SCHEME_NO_POINT,
        "HLC_SCHEME_INFINITY": po.SCHEME_INFINITY, "HLC_STILL_ACTIVE": po.STILL_ACTIVE,
        "HLC_REACHED_NO": po.REACHED_NO, "HLC_REACHED_YES": po.REACHED_YES,
    }
    for k, v in pairs.items():
        assert d[k] == v, k


PROBE = r"""
#include <stdio.h>
#include <stddef.h>
#include "hlc.h"
int main(void) {
  printf("%zu %zu %zu\n", sizeof(hlc_votes), sizeof(hlc_proposal), sizeof(hlc_result));
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\n", offsetof(hlc_proposal, vote_begin),
         offsetof(hlc_proposal, vote_count), offsetof(hlc_proposal, proposal_id), offsetof(hlc_proposal, timestamp),
         offsetof(hlc_proposal, expiration_timestamp), offsetof(hlc_proposal, expected_voters_count),
         offsetof(hlc_proposal, max_rounds), offsetof(hlc_proposal, consensus_threshold),
         offsetof(hlc_proposal, use_gossipsub_rounds), offsetof(hlc_proposal, liveness_criteria_yes));
  printf("%zu %zu %zu %zu %zu %zu\n", offsetof(hlc_result, status), offsetof(hlc_result, transition),
         offsetof(hlc_result, scheme_reason), offsetof(hlc_result, bad_index), offsetof(hlc_result, yes),
         offsetof(hlc_result, total));
  return 0;
}
"""


def test_struct_layout_matches_c(tmp_path):
    src = tmp_path / "probe.c"
    src.write_text(PROBE)
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    lines = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    sv, sp, sr = map(int, lines[0].split())
    assert (sv, sp, sr) == (ctypes.sizeof(_ffi.hlc_votes), ctypes.sizeof(_ffi.hlc_proposal),
                            ctypes.sizeof(_ffi.hlc_result))
    offs = list(map(int, lines[1].split()))
    names = ["vote_begin", "vote_count", "proposal_id", "timestamp", "expiration_timestamp",
             "expected_voters_count", "max_rounds", "consensus_threshold", "use_gossipsub_rounds",
             "liveness_criteria_yes"]
    assert offs == [_ffi.PROPOSAL_DTYPE.fields[n][1] for n in names]
    assert offs == [getattr(_ffi.hlc_proposal, n).offset for n in names]
    roffs = list(map(int, lines[2].split()))
    assert roffs == [_ffi.RESULT_DTYPE.fields[n][1] for n in
                     ["status", "transition", "scheme_reason", "bad_index", "yes", "total"]]


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(_ffi.HlcUnavailable):
        _ffi._lib_saved = _ffi._lib
        _ffi._lib = None
        try:
            _ffi.load_library(str(tmp_path / "nope.so"))
        finally:
            _ffi._lib = _ffi._lib_saved


def test_ctx_create_without_gpu_reports_error():
    """On a host without a gfx950 device the context refuses to start (no CPU fallback)."""
    lib = _ffi.load_library()
    h = ctypes.c_void_p()
    rc = lib.hlc_ctx_create(0, ctypes.byref(h))
    if rc == 0:  # running on a GPU box: nothing to check here
        lib.hlc_ctx_destroy(h)
        pytest.skip("a gfx950 device is present")
    assert rc == header_defines()["HLC_ENODEV"]
    assert lib.hlc_last_error()


WIRE_PROBE = r"""
#include <stdio.h>
#include <stddef.h>
#include "hlc.h"
int main(void) {
  printf("%zu %zu\n", sizeof(hlc_scope_config), sizeof(hlc_wire_proposal));
  printf("%zu %zu %zu\n", offsetof(hlc_scope_config, consensus_threshold), offsetof(hlc_scope_config, max_rounds),
         offsetof(hlc_scope_config, use_gossipsub_rounds));
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu\n", offsetof(hlc_wire_proposal, name_off),
         offsetof(hlc_wire_proposal, payload_off), offsetof(hlc_wire_proposal, owner_off),
         offsetof(hlc_wire_proposal, name_len), offsetof(hlc_wire_proposal, payload_len),
         offsetof(hlc_wire_proposal, owner_len), offsetof(hlc_wire_proposal, round),
         offsetof(hlc_wire_proposal, bad_vote), offsetof(hlc_wire_proposal, decode_status));
  return 0;
}
"""


def test_wire_struct_layout_and_codes(tmp_path):
    """hlc_scope_config / hlc_wire_proposal layouts and HLC_WIRE_* codes match the Python side
    (numpy dtypes, oracle/wire_oracle.py reason codes)."""
    import wire_oracle as wo
    src = tmp_path / "wprobe.c"
    src.write_text(WIRE_PROBE)
    exe = tmp_path / "wprobe"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    lines = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    assert list(map(int, lines[0].split())) == [_ffi.SCOPE_CONFIG_DTYPE.itemsize, _ffi.WIRE_PROPOSAL_DTYPE.itemsize]
    assert list(map(int, lines[1].split())) == [_ffi.SCOPE_CONFIG_DTYPE.fields[n][1] for n in
                                                ("consensus_threshold", "max_rounds", "use_gossipsub_rounds")]
    assert list(map(int, lines[2].split())) == [_ffi.WIRE_PROPOSAL_DTYPE.fields[n][1] for n in
                                                ("name_off", "payload_off", "owner_off", "name_len", "payload_len",
                                                 "owner_len", "round", "bad_vote", "decode_status")]
    d = header_defines()
    for name in ("OK", "INVALID_VARINT", "INVALID_KEY", "INVALID_WIRE_TYPE", "INVALID_TAG", "WIRE_TYPE_MISMATCH",
                 "BUFFER_UNDERFLOW", "DELIMITED_EXCEEDED", "INVALID_UTF8", "UNEXPECTED_END_GROUP",
                 "RECURSION_LIMIT"):
        assert d["HLC_WIRE_" + name] == getattr(wo, name), name
    assert d["HLC_PROPOSAL_DECODE_ERROR"] == 17 and d["HLC_ERANGE"] == -5


def _threads_in_child(env_extra):
    """hlc_host_threads() in a fresh process with `env_extra` set (no GPU call is made)."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); from hashgraph_like_consensus import _ffi; "
            "print(_ffi.load_library().hlc_host_threads())" % os.path.join(ROOT, "hashgraph-like-consensus_amd", "python"))
    env = {k: v for k, v in os.environ.items() if k not in ("HLC_HOST_THREADS", "LOCAL_WORLD_SIZE")}
    env.update(env_extra)
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    return int(out.stdout.strip())


def _cpu_share():
    """The CPUs this process may use by the library's rule: the cgroup v2 quota, else the hardware threads."""
    hw = os.cpu_count() or 1
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
        if q != "max":
            return min(float(q) / float(per), hw), hw
    except (OSError, ValueError):
        pass
    return float(hw), hw


def test_host_threads_default_is_rank_aware():
    """the host-buffer entries' staging threads default to min(16, hardware
    threads, the CPU quota / the ranks on the node), so 8 ranks on one node do not run 8 x 16 staging
    threads on one quota; HLC_HOST_THREADS overrides (clamped to 1..64)."""
    share, hw = _cpu_share()
    for ranks in (1, 2, 8, 64):
        want = max(1, min(16, hw, int(share / ranks + 1e-9)))
        assert _threads_in_child({"LOCAL_WORLD_SIZE": str(ranks)}) == want, ranks
    assert _threads_in_child({}) == max(1, min(16, hw, int(share + 1e-9)))
    assert _threads_in_child({"HLC_HOST_THREADS": "5", "LOCAL_WORLD_SIZE": "8"}) == 5
    assert _threads_in_child({"HLC_HOST_THREADS": "500"}) == 64


def test_options_match_header_and_no_per_call_getenv():
    """the tunables are context options (hlc_ctx_set_option); the environment is
    read in one function (read_env, called by hlc_ctx_create / hlc_host_threads) and nowhere else."""
    d = header_defines()
    for name, code in _ffi.OPTIONS.items():
        assert d["HLC_OPT_" + name.upper()] == code, name
    assert {k for k in d if k.startswith("HLC_OPT_")} == {"HLC_OPT_" + n.upper() for n in _ffi.OPTIONS}
    assert (d["HLC_POOL_BIND_NONE"], d["HLC_POOL_BIND_GPU"], d["HLC_POOL_BIND_SOURCE"]) == (
        _ffi.POOL_BIND_NONE, _ffi.POOL_BIND_GPU, _ffi.POOL_BIND_SOURCE)
    csrc = os.path.join(ROOT, "hashgraph-like-consensus_amd", "csrc")
    for f in sorted(os.listdir(csrc)):
        if not f.endswith((".cpp", ".hip", ".hpp", ".h")):
            continue
        text = open(os.path.join(csrc, f)).read()
        calls = [m.start() for m in re.finditer(r"std::getenv\(|\bgetenv\(", text)]
        if f != "hlc_api.cpp":
            assert not calls, f
            continue
        body = text[text.index("Options read_env() {"):]
        body = body[:body.index("\n}\n")]
        start = text.index(body)
        assert calls and all(start <= c < start + len(body) for c in calls), "getenv outside read_env"
