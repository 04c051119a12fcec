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


def bow_case(seed, n_kf=1000, n_f=1000, n_nodes=100, zipf=1.2, live=0.7, dup=0.6, flips=0.08, rot=20.0):
    """Synthetic SearchByBoW input: NodeIds from a Zipf
    over n_nodes, 70 % live MapPoints, dup of the F rows are KF rows with
    Binomial(256, flips) bit flips in the same node, angles rotated by `rot`
    degrees plus noise.  Returns (kf_desc, kf_angle, kf_live, kf_fv, f_desc,
    f_angle, f_fv) with fv = {node: [indices ascending]}."""
    rng = np.random.default_rng(seed)
    w = 1.0 / np.arange(1, n_nodes + 1) ** zipf
    w /= w.sum()
    node_ids = np.sort(rng.choice(100000, n_nodes, replace=False))
    kf_desc = rng.integers(0, 256, (n_kf, 32), dtype=np.uint8)
    kf_node = node_ids[rng.choice(n_nodes, n_kf, p=w)]
    kf_angle = rng.uniform(0, 360, n_kf).astype(np.float32)
    kf_live = (rng.random(n_kf) < live).astype(np.uint8)
    f_desc = rng.integers(0, 256, (n_f, 32), dtype=np.uint8)
    f_node = node_ids[rng.choice(n_nodes, n_f, p=w)]
    f_angle = rng.uniform(0, 360, n_f).astype(np.float32)
    nd = int(dup * n_f)
    src = rng.choice(n_kf, nd, replace=True)
    bits = np.unpackbits(kf_desc[src], axis=1)
    bits ^= (rng.random(bits.shape) < flips).astype(np.uint8)
    f_desc[:nd] = np.packbits(bits, axis=1)
    f_node[:nd] = kf_node[src]
    f_angle[:nd] = np.mod(kf_angle[src] - rot + rng.normal(0, 3, nd), 360).astype(np.float32)
    perm = rng.permutation(n_f)
    f_desc, f_node, f_angle = f_desc[perm], f_node[perm], f_angle[perm]

    def fv(nodes):
        d = {}
        for i, n in enumerate(nodes):
            d.setdefault(int(n), []).append(i)
        return d
    return kf_desc, kf_angle, kf_live, fv(kf_node), f_desc, f_angle, fv(f_node)
