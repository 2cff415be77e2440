"""Deterministic synthetic stripe contents shared by the golden generator and the tests.

* ``affine(k, C)``: D_j[b] = (j*131 + b*7 + 1) mod 256 -- the input of the known-answer
  anchors recorded in SURVEY.md §8c.
* ``splitmix(seed, n)``: the splitmix64 byte stream of SURVEY.md §8d (seed 0x4C53544F5245).
"""
import numpy as np

SEED = 0x4C53544F5245


def affine(k, size):
    j = np.arange(k, dtype=np.int64)[:, None]
    b = np.arange(size, dtype=np.int64)[None, :]
    return ((j * 131 + b * 7 + 1) % 256).astype(np.uint8)


def splitmix(seed, nbytes, counter0=0):
    n = (nbytes + 7) // 8
    with np.errstate(over="ignore"):
        i = np.arange(counter0 + 1, counter0 + n + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.view(np.uint8)[:nbytes].copy()


def stripe(k, size, stripe_index=0, seed=SEED):
    """k data chunks of one stripe; stripe s uses counter base s*k*C/8."""
    return splitmix(seed, k * size, counter0=stripe_index * k * size // 8).reshape(k, size)
