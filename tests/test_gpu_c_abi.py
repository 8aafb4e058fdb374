"""The C ABI from plain C (tests/c/hlc_abi_demo.c, built by the package Makefile with gcc against
include/hlc.h and libhlc.so only): what a non-Python embedder -- INTEGRATION.md's Rust hlc-sys, a
cgo or JNI stub -- links.  On the GPU it signs, identifies and verifies a batch through the ABI
and classifies broken items as signing/ethereum.rs:66-97 does; without a GPU it must fail loudly
(context creation), never fall back."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEMO = os.path.join(ROOT, "tests", "c", "hlc_abi_demo")


def _demo():
    if not os.path.exists(DEMO):  # built by the package Makefile (gcc only, seconds)
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "hashgraph-like-consensus_amd"),
                        "../tests/c/hlc_abi_demo"], check=False, capture_output=True)
    if not os.path.exists(DEMO):
        pytest.fail("tests/c/hlc_abi_demo is not built (python __graft_entry__.py build / make -C "
                    "hashgraph-like-consensus_amd)")
    return DEMO


@pytest.mark.gpu
def test_gpu_c_abi_demo():
    r = subprocess.run([_demo()], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "hlc_abi_demo ok" in r.stdout


def test_c_abi_demo_links_only_libhlc():
    """The demo needs libhlc.so (found through its RUNPATH) and libc -- no HIP or torch library."""
    out = subprocess.run(["readelf", "-d", _demo()], capture_output=True, text=True, check=True).stdout
    needed = sorted(line.split("[")[1].rstrip("]") for line in out.splitlines() if "(NEEDED)" in line)
    assert needed == ["libc.so.6", "libhlc.so"], needed


def test_c_abi_demo_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present (the GPU test covers this box)")
    r = subprocess.run([_demo()], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "hlc_ctx_create" in r.stderr
