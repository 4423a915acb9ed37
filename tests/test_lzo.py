"""CPU tests of the bundle writer offload (§8(f)-4):

* zc_lzo_core.h -- the LZO1X-1 parse, staging and bundle assembly the GPU
  kernels run -- compiled for the host and compared byte for byte with
  liblzo2 2.10's own lzo1x_1_compress (the library zbackup calls,
  compression.cc:586-606) on 600 payloads of six kinds and edge sizes, plus
  every length up to 160 and every short last block (49152 + 21 .. 63);
* the oracle's framing round-trips through lzo1x_decompress_safe;
* zc_bundle_plan (host bookkeeping) equals the restated Writer::add rule
  (chunk_storage.cc:31-46), including a chunk larger than the bundle limit."""
import os
import subprocess

import numpy as np
import pytest

from oracle import lzo_oracle
from tests.lzo_inputs import KINDS, payload

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LZO_INC = "/opt/conda/include"
LZO_SO = "/opt/conda/lib/liblzo2.so.2"

needs_lzo = pytest.mark.skipif(not os.path.exists(LZO_SO) or not os.path.exists(os.path.join(LZO_INC, "lzo")),
                               reason="liblzo2 not in this image")


@needs_lzo
def test_lzo_core_matches_liblzo2(tmp_path):
    exe = str(tmp_path / "lzo_core_check")
    subprocess.run(["g++", "-O2", "-Wall", "-Werror", "-std=c++17", "-I" + os.path.join(ROOT, "zbackup_amd", "csrc"),
                    "-I" + LZO_INC, os.path.join(ROOT, "tests", "lzo", "lzo_core_check.cpp"), LZO_SO,
                    "-Wl,-rpath," + os.path.dirname(LZO_SO), "-o", exe], check=True)
    out = subprocess.run([exe, "600"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("ok ") and int(out.stdout.split()[1]) >= 600 + 6 * 204


@needs_lzo
@pytest.mark.parametrize("kind", KINDS)
def test_oracle_frame_round_trip(kind):
    data = payload(kind, 200003, 7).tobytes()
    framed = lzo_oracle.frame(data)
    assert framed[4:8] == b"EFGH" and framed[12:16] == b"MNOP"
    assert int.from_bytes(framed[0:4], "little") == len(data)
    assert int.from_bytes(framed[8:12], "little") == len(framed) - 16
    assert lzo_oracle.unframe(framed) == data


def test_bundle_plan_matches_writer_add():
    from zbackup_amd.bundle import plan_bundles
    rng = np.random.default_rng(3)
    for trial in range(20):
        n = int(rng.integers(0, 400))
        sizes = rng.integers(128, 70000, n)
        if trial % 3 == 0 and n:
            sizes[rng.integers(0, n)] = 3_000_000  # larger than a bundle: finishes even an empty one
        max_payload = int(rng.choice([0x200000, 1 << 20, 300000]))
        want = lzo_oracle.writer_bundles([(i, int(s)) for i, s in enumerate(sizes)], max_payload)
        got, nb = plan_bundles(sizes, max_payload)
        assert nb == len(want)
        for b, members in enumerate(want):
            assert list(np.nonzero(got == b)[0]) == members


def test_bundle_plan_first_chunk_over_the_limit():
    from zbackup_amd.bundle import plan_bundles
    got, nb = plan_bundles([5_000_000, 10], 0x200000)
    # Writer::add: the empty current bundle is finished first (bundle 0 stays
    # empty), and the next chunk does not fit beside the oversized one
    assert nb == 3 and list(got) == [1, 2]
    assert lzo_oracle.writer_bundles([(0, 5_000_000), (1, 10)]) == [[], [0], [1]]
