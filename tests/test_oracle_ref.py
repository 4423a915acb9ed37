"""CPU tests: pinning hygiene for the oracle (the checker), run wherever
/root/reference exists (this container; never the GPU box, which has no copy).

(a) the reference's own hot-path test, tests/rolling_hash/test_rolling_hash.cc
    (:27-68 roll-in vs rotate equivalence on 5,000 slices, :78-115 no collision
    in 500,000 slice hashes), compiled from where it lies (oracle/Makefile ref)
    and run here: its success lines are required;
(b) the committed fixtures tests/golden/* regenerated from oracle/_ref (the
    restated state machine over the reference's own rolling_hash.cc) into a
    temporary directory and compared file by file: no drift between the
    fixtures and their generator;
(c) the restated oracle (liboracle.so, the checker every other test uses)
    against the reference-built one (_ref/liboracle_ref.so) on 50 fresh seeded
    random streams and chunk sizes: every record equal.
"""
import filecmp
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_DIR = os.path.join(HERE, "..", "oracle")

pytestmark = pytest.mark.skipif(not os.path.isfile(os.path.join(REF, "rolling_hash.cc")),
                                reason="needs the reference sources (/root/reference)")


@pytest.fixture(scope="module", autouse=True)
def _built():
    oracle.build(ref=True)


def test_reference_rolling_hash_test_passes():
    exe = os.path.join(ORACLE_DIR, "_ref", "test_rolling_hash")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "Rolling hash test produced equal results" in out.stderr
    assert "Collisions: 0.0000% (0 in " in out.stderr
    assert "Rolling hash test succeeded" in out.stderr
    # every equivalence iteration printed its digest (5,000) plus one line per
    # 1,000 collision iterations (500)
    assert out.stdout.count("Iteration ") == 5000 + 500


def test_golden_fixtures_regenerate_identically(tmp_path):
    script = os.path.join(HERE, "golden", "make_golden.py")
    subprocess.run([sys.executable, script, str(tmp_path)], check=True, capture_output=True, timeout=600)
    golden = os.path.join(HERE, "golden")
    committed = sorted(f for f in os.listdir(golden) if f.endswith(".txt"))
    fresh = sorted(f for f in os.listdir(tmp_path) if f.endswith(".txt"))
    assert committed == fresh
    _, mismatch, errors = filecmp.cmpfiles(golden, str(tmp_path), committed, shallow=False)
    assert not mismatch and not errors, (mismatch, errors)


def _random_spec(rng, W):
    segs, n = [], 0
    for _ in range(int(rng.integers(1, 10))):
        t = int(rng.integers(0, 6))
        ln = int(rng.integers(1, 6 * W + 2))
        if t <= 1 or n == 0:
            segs.append(f"R{int(rng.integers(1, 1 << 30))}:{ln}")
        elif t == 2:
            segs.append(f"Z:{ln}")
        elif t == 3:
            segs.append(f"B{int(rng.integers(0, 256))}:{ln}")
        else:
            segs.append(f"C{int(rng.integers(0, n))}:{ln}")
        n += ln
    return ",".join(segs)


@pytest.mark.parametrize("seed", range(50))
def test_restated_oracle_equals_reference_built(seed):
    rng = np.random.default_rng(90000 + seed)
    W = int(rng.choice([1, 7, 64, 127, 128, 129, 257, 1000, 4096, 4097, 65536, int(rng.integers(2, 70000))]))
    spec = _random_spec(rng, W)
    data = oracle.gen(spec)
    assert np.array_equal(data, oracle.gen(spec, ref=True))
    seeds = []
    if seed % 5 == 0 and data.size >= W:
        # an index holding some of the stream's own W-byte windows (ChunkIndex::loadIndex)
        for off in rng.integers(0, data.size - W + 1, 4):
            win = data[int(off):int(off) + W]
            seeds.append((bytes(oracle.sha1(win)[:16]), oracle.digest(win), W))
    want = oracle.chunk(data, W, seeds=seeds, ref=True)
    assert oracle.chunk(data, W, seeds=seeds) == want, spec
    if seed % 7 == 0:  # the input framing (fread piece sizes) changes nothing
        assert oracle.chunk(data, W, seeds=seeds, feed_max=int(rng.integers(1, 3 * W + 2))) == want, spec
