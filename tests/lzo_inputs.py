"""Synthetic bundle payloads for the LZO parity tests and the bench (numpy,
seeded): the same six kinds tests/lzo/lzo_core_check.cpp draws."""
import numpy as np

KINDS = ("random", "zeros", "text", "repeats", "alphabet3", "runs")
_WORDS = [b"the ", b"backup ", b"chunk ", b"index ", b"bundle ", b"of ", b"and ", b"zbackup ", b"rolling ",
          b"hash ", b"\n", b"data ", b"stream "]


def text(n, rng):
    """words from a small vocabulary (compresses ~3x)"""
    lens = np.array([len(w) for w in _WORDS])
    table = np.frombuffer(b"".join(_WORDS), dtype=np.uint8)
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
    m = n // 3 + 16
    idx = rng.integers(0, len(_WORDS), m)
    ln = lens[idx]
    total = int(ln.sum())
    first = np.repeat(np.cumsum(ln) - ln, ln)
    src = np.repeat(starts[idx], ln) + (np.arange(total) - first)
    return table[src[:n]].copy()


def payload(kind, n, seed):
    rng = np.random.default_rng(seed)
    if kind == "random":
        return rng.integers(0, 256, n, dtype=np.uint8)
    if kind == "zeros":
        return np.zeros(n, dtype=np.uint8)
    if kind == "text":
        return text(n, rng)
    if kind == "repeats":  # random bytes with pieces copied from up to 60000 back
        v = rng.integers(0, 256, n, dtype=np.uint8)
        i = 0
        while i + 64 < n:
            ln, back = int(rng.integers(4, 204)), int(rng.integers(1, 60001))
            if i >= back and i + ln < n:
                v[i:i + ln] = v[i - back:i - back + ln].copy()
            i += 1 + int(rng.integers(0, 300))
        return v
    if kind == "alphabet3":
        return (97 + rng.integers(0, 3, n)).astype(np.uint8)
    if kind == "runs":  # runs of one value, 1 in 8 bytes random
        v = np.empty(n, dtype=np.uint8)
        lens = rng.integers(1, 2000, n // 500 + 2)
        vals = rng.integers(0, 256, len(lens), dtype=np.uint8)
        rep = np.repeat(vals, lens)
        while len(rep) < n:
            rep = np.concatenate([rep, rep])
        v[:] = rep[:n]
        noise = rng.integers(0, 8, n) == 0
        v[noise] = rng.integers(0, 256, int(noise.sum()), dtype=np.uint8)
        return v
    raise ValueError(kind)
