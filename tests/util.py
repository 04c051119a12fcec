import pathlib

import numpy as np

GOLDEN = pathlib.Path(__file__).resolve().parent / "golden"


def real_frames():
    z = np.load(GOLDEN / "frames.npz")
    return {k: z[k] for k in z.files}


def near_duplicate_descriptors(rng, n_train, n_query, frac=0.6, p_flip=0.08):
    """C3 generator: 60% of queries are train rows with
    Binomial(256, p) bit flips, the rest uniform random bits."""
    t = rng.integers(0, 256, size=(n_train, 32), dtype=np.uint8)
    q = rng.integers(0, 256, size=(n_query, 32), dtype=np.uint8)
    k = int(frac * n_query)
    src = rng.integers(0, n_train, size=k)
    bits = np.unpackbits(t[src], axis=1)
    flips = rng.random(bits.shape) < p_flip
    q[:k] = np.packbits(bits ^ flips, axis=1)
    return q, t
