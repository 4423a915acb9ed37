"""Whole-stream SHA-256 (zc_sha256_*, the Sha256 the feed loop keeps: sha256.hh:14-35,
zutils.cc:119,134).  Host code, so these run on the CPU.  The reference's SHA-256 is
OpenSSL's SHA256_Init/Update/Final (sha256.cc:8-21); Python's hashlib is that same
OpenSSL implementation, and FIPS 180-4's published vectors pin both."""
import hashlib
import os

import numpy as np
import pytest

from zbackup_amd import _build
from zbackup_amd.chunker import Sha256


@pytest.fixture(scope="module", autouse=True)
def built():
    _build.build()


FIPS = [  # FIPS 180-4 / NIST CAVP examples
    (b"", "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"),
    (b"abc", "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"),
    (b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
     "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"),
    (b"a" * 1000000, "cdc76e5c9914fb9281a1c7e284d73e67f1809a48a497200e046d39ccc7112cd0"),
]


@pytest.mark.parametrize("impl", ["auto", "scalar"])
def test_fips_vectors(impl, monkeypatch):
    if impl == "scalar":
        monkeypatch.setenv("ZC_SHA256_SCALAR", "1")
    for msg, hexd in FIPS:
        h = Sha256()
        if impl == "scalar":
            assert not h.uses_sha_extensions
        h.add(msg)
        assert h.finish().hex() == hexd


@pytest.mark.parametrize("impl", ["auto", "scalar"])
def test_incremental_feeds_match_hashlib(impl, monkeypatch):
    """Buffers of every length around the 64-byte block and the 55/56-byte padding
    split, fed in ragged pieces the way zutils.cc's read loop hands them over."""
    if impl == "scalar":
        monkeypatch.setenv("ZC_SHA256_SCALAR", "1")
    rng = np.random.default_rng(7)
    data = rng.integers(0, 256, 70000, dtype=np.uint8).tobytes()
    for n in list(range(0, 200)) + [4095, 4096, 4097, 65536, 70000]:
        cuts = sorted(rng.integers(0, n + 1, 5)) if n else []
        h = Sha256()
        prev = 0
        for c in list(cuts) + [n]:
            h.add(data[prev:c])
            prev = c
        assert h.finish() == hashlib.sha256(data[:n]).digest(), n


def test_finish_once_and_add_after_finish_fail():
    from zbackup_amd import ZcError
    h = Sha256()
    h.add(b"x")
    h.finish()
    with pytest.raises(ZcError):
        h.finish()
    with pytest.raises(ZcError):
        h.add(b"y")


def test_extensions_used_when_the_host_has_them():
    flags = open("/proc/cpuinfo").read() if os.path.exists("/proc/cpuinfo") else ""
    if " sha_ni" not in flags:
        pytest.skip("host has no SHA extensions")
    assert Sha256().uses_sha_extensions
