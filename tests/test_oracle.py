"""CPU tests: pin the oracle (the checker) against the reference-built golden
fixtures and known answers before anything is compared with it."""
import numpy as np
import pytest

from oracle import oracle
from tests import golden_io

CASES = golden_io.case_names()


@pytest.fixture(scope="module", autouse=True)
def _built():
    oracle.build()


def _case(name):
    return golden_io.load_case(f"{golden_io.GOLDEN}/{name}.txt")


def test_kat_digests():
    # digest("") = 1, digest(0^65536) = 257^65536 mod 2^64, plus
    # random slices, all computed by the reference's rolling_hash.cc
    for name, spec, want in golden_io.kats():
        assert oracle.digest(oracle.gen(spec)) == want, name


def test_kat_closed_form():
    # H = 257^n + sum b_i 257^(n-1-i) (mod 2^64), rolling_hash.hh:10-38
    rng = np.random.default_rng(7)
    for n in (0, 1, 2, 17, 255, 1000):
        b = rng.integers(0, 256, n, dtype=np.uint8)
        acc = 0
        for x in b:
            acc = (acc * 257 + int(x)) % (1 << 64)
        assert oracle.digest(b) == (pow(257, n, 1 << 64) + acc) % (1 << 64)


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_golden(name):
    meta, seeds, want = _case(name)
    data = oracle.gen(meta["spec"])
    assert data.size == meta["n"]
    got = oracle.chunk(data, meta["W"], seeds=seeds)
    assert got == want


@pytest.mark.parametrize("feed", [1, 7, 4096, 65535, 1 << 20])
def test_records_independent_of_input_framing(feed):
    # backup_creator.cc:56-108: records depend on the bytes, not on how fread
    # split them (SURVEY §3.3 rule 6)
    meta, seeds, want = _case("mixed" if feed >= 4096 else "w4096_shift")
    data = oracle.gen(meta["spec"])
    assert oracle.chunk(data, meta["W"], seeds=seeds, feed_max=feed) == want


def test_splitmix_stream_recipe():
    # byte k = byte (k mod 8) of splitmix64 word k // 8 (shared with the GPU filler)
    n = 1003
    got = oracle.splitmix64(n, 42)
    words = []
    for i in range(n // 8 + 1):
        z = (42 + (i + 1) * 0x9E3779B97F4A7C15) % (1 << 64)
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) % (1 << 64)
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) % (1 << 64)
        words.append(z ^ (z >> 31))
    ref = np.frombuffer(b"".join(w.to_bytes(8, "little") for w in words), dtype=np.uint8)[:n]
    assert np.array_equal(got, ref)


def test_zero_stream_survey_facts():
    # SURVEY §8c, from a run of the real backup_creator.cc: 16 MiB of zeros ->
    # 256 records, all with hash 0x172aeaff81000001; the first saved, 255 matches
    meta, _, recs = _case("zero16m")
    assert len(recs) == 256
    assert {r[3] for r in recs} == {0x172AEAFF81000001}
    assert [r[0] for r in recs] == ["N"] + ["D"] * 255


def test_dup_stream_survey_facts():
    # two concatenated 8 MiB copies: the second half re-emits the first half's ids
    _, _, recs = _case("dup16m")
    first, second = recs[:128], recs[128:]
    assert all(r[0] == "N" for r in first) and all(r[0] == "D" for r in second)
    assert [(r[3], r[4]) for r in first] == [(r[3], r[4]) for r in second]
