"""DBoW2 vocabulary: loadFromTextFile + transform(features, BowVector&,
FeatureVector&, levelsup) (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:
1126-1259, 1338-1424), the ORB vocabulary step of Frame::ComputeBoW
(src/Frame.cc:1115-1122).

Parity unpinned: the reference has no vocabulary tests and its ORBvoc.txt
is absent.  The C++ oracle (oracle/bow_oracle.cpp, std::map containers and
iostream parsing like the reference) is cross-checked here against a second,
pure-Python restatement on small irregular trees and hand-built known
answers; the HIP path is then compared with the oracle bit-exactly (word
ids, double values, FeatureVector CSR)."""
import math

import numpy as np
import pytest

import oracle_lib
from plvi import synth


def _popc(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def py_transform(parent, is_leaf, desc, weight, scoring, weighting, L, feats, levelsup):
    """Second restatement (pure Python, small cases): TemplatedVocabulary.h:1126-1259."""
    n = len(parent) + 1
    children = [[] for _ in range(n)]
    word = [0] * n
    nw = 0
    for i, p in enumerate(parent):
        children[p].append(i + 1)
        if is_leaf[i]:
            word[i + 1] = nw
            nw += 1
    D = np.vstack([np.zeros((1, 32), np.uint8), desc])
    W = [0.0] + list(weight)
    if nw == 0:
        return {}, {}
    must, l2 = scoring != 5, scoring == 1
    tf = weighting in (0, 1)
    bow, fv = {}, {}
    for i, f in enumerate(feats):
        nid_level = L - levelsup
        nid = 0
        node, level = 0, 0
        while True:
            level += 1
            kids = children[node]
            node = kids[0]
            best = _popc(f, D[node])
            for c in kids[1:]:
                d = _popc(f, D[c])
                if d < best:
                    best, node = d, c
            if level == nid_level:
                nid = node
            if not children[node]:
                break
        w = W[node]
        if w > 0:
            wid = word[node]
            if tf:
                bow[wid] = bow[wid] + w if wid in bow else w
            elif wid not in bow:
                bow[wid] = w
            fv.setdefault(nid, []).append(i)
    bow = dict(sorted(bow.items()))
    if tf and bow and not must:
        nd = float(len(bow))
        bow = {k: v / nd for k, v in bow.items()}
    if must:
        nrm = 0.0
        for v in bow.values():
            nrm += abs(v) if not l2 else v * v
        if l2:
            nrm = math.sqrt(nrm)
        if nrm > 0:
            bow = {k: v / nrm for k, v in bow.items()}
    return bow, dict(sorted(fv.items()))


def _as_dicts(bw, bv, fn, fo, fi):
    bow = {int(w): float(v) for w, v in zip(bw, bv)}
    fv = {int(fn[i]): [int(x) for x in fi[fo[i]:fo[i + 1]]] for i in range(len(fn))}
    return bow, fv


def _write(tmp_path, text, name="voc.txt"):
    p = tmp_path / name
    p.write_text(text)
    return p


KAT_TEXT = ("2 2  0 0\n"
            "0 0 " + " ".join(["0"] * 32) + "  0\n"            # node 1: children 3, 4
            "0 0 " + " ".join(["255"] * 32) + "  0\n"          # node 2: children 5, 6
            "1 1 " + " ".join(["1"] + ["0"] * 31) + "  0.5\n"  # node 3: word 0
            "1 1 " + " ".join(["3"] + ["0"] * 31) + "  0\n"    # node 4: word 1 (stopped)
            "2 1 " + " ".join(["255"] * 31 + ["127"]) + "  2\n"  # node 5: word 2
            "2 1 " + " ".join(["255"] * 31 + ["127"]) + "  4\n")  # node 6: word 3 (tie with 5)


def test_oracle_loader_known_answers(tmp_path):
    p = _write(tmp_path, KAT_TEXT)
    v = oracle_lib.Vocab.load_text(p, emulate_tail=True)
    assert (v.k, v.L, v.scoring, v.weighting) == (2, 2, 0, 0)
    assert v.n_words == 4
    assert v.n_nodes == 8  # root + 6 lines + the empty tail after the final newline
    parent, nchild, word, weight, desc = v.nodes()
    assert list(parent[1:7]) == [0, 0, 1, 1, 2, 2] and parent[7] == 0
    assert list(nchild[:3]) == [3, 2, 2] and nchild[7] == 0 and weight[7] == 0
    assert list(word[3:7]) == [0, 1, 2, 3]
    v2 = oracle_lib.Vocab.load_text(p, emulate_tail=False)
    assert v2.n_nodes == 7
    p2 = _write(tmp_path, KAT_TEXT.rstrip("\n"), "nonl.txt")  # no final newline: no tail node
    assert oracle_lib.Vocab.load_text(p2, emulate_tail=True).n_nodes == 7
    with pytest.raises(ValueError):  # k > 20: "not a correct text file"
        oracle_lib.Vocab.load_text(_write(tmp_path, "30 2 0 0\n", "bad.txt"))


def test_oracle_transform_known_answers(tmp_path):
    v = oracle_lib.Vocab.load_text(_write(tmp_path, KAT_TEXT), emulate_tail=False)
    f = np.zeros((5, 32), np.uint8)
    f[0, 0] = 1      # -> node 1 (d 1 vs 255) -> node 3 (d 0): word 0, w 0.5
    f[1, 0] = 3      # -> node 1 -> node 4 (d 0): stopped (w 0)
    f[2] = 255       # -> node 2 -> 5 vs 6 tie (d 1 each): first wins -> word 2, w 2
    f[3, 0] = 1      # word 0 again
    f[4] = 254       # -> node 2 -> node 5 (tie again): word 2
    bw, bv, fn, fo, fi, fw, fwt, fni = v.transform(f, levelsup=1)  # nid level 1
    assert list(fw) == [0, 1, 2, 0, 2]
    assert list(fni) == [1, 1, 2, 1, 2]
    # BowVector: word0 = 0.5+0.5, word2 = 2+2, L1-normalised by 5
    assert list(bw) == [0, 2] and np.allclose(bv, [1.0 / 5.0, 4.0 / 5.0])
    assert list(fn) == [1, 2] and list(fo) == [0, 2, 4] and list(fi) == [0, 3, 2, 4]


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("scoring,weighting", [(0, 0), (1, 1), (5, 1), (5, 0), (0, 2), (3, 3)])
def test_oracle_matches_python_restatement(seed, scoring, weighting):
    parent, leaf, desc, weight = synth.vocabulary_irregular(k=5, L=4, seed=seed)
    v = oracle_lib.Vocab.create(5, 4, scoring, weighting, parent, leaf, desc, weight)
    feats = synth.vocab_features(parent, leaf, desc, 60, seed=seed)
    for levelsup in (0, 2, 4):
        got = _as_dicts(*v.transform(feats, levelsup)[:5])
        exp = py_transform(parent, leaf, desc, weight, scoring, weighting, 4, feats, levelsup)
        assert got == exp


# ------------------------------------------------------------------ GPU


def _gpu_vs_oracle(vg, vo, feats, levelsup):
    got = vg.transform_arrays(feats, levelsup)
    exp = vo.transform(feats, levelsup)
    for g, e, name in zip(got, exp[:5], ("bow_word", "bow_value", "fv_node", "fv_off", "fv_idx")):
        np.testing.assert_array_equal(g, e, err_msg=name)
    w, nid = vg.transform_features(feats, levelsup)
    np.testing.assert_array_equal(w, exp[5])
    np.testing.assert_array_equal(nid, exp[7])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("scoring,weighting", [(0, 0), (1, 1), (5, 1), (0, 2), (4, 3)])
def test_vocab_text_transform_matches_oracle(tmp_path, seed, scoring, weighting):
    import plvi
    parent, leaf, desc, weight = synth.vocabulary_irregular(k=8, L=5, seed=100 + seed)
    p = _write(tmp_path, synth.vocabulary_text(8, 5, scoring, weighting, parent, leaf, desc, weight))
    for tail in (True, False):
        vg = plvi.ORBVocabulary.loadFromTextFile(p, emulate_tail=tail)
        vo = oracle_lib.Vocab.load_text(p, emulate_tail=tail)
        assert (vg.n_nodes, vg.n_words) == (vo.n_nodes, vo.n_words)
        feats = synth.vocab_features(parent, leaf, desc, 700 + 13 * seed, seed=seed)
        feats[:20] = 0  # near the zero-descriptor tail node
        for levelsup in (4, 0, 5, 9):
            _gpu_vs_oracle(vg, vo, feats, levelsup)


@pytest.mark.gpu
def test_vocab_edge_cases(tmp_path):
    import plvi
    # no words: BowVector / FeatureVector stay empty (empty(), :1134-1137)
    p = _write(tmp_path, "3 2  0 0\n0 0 " + " ".join(["7"] * 32) + "  0\n", "nowords.txt")
    vg = plvi.ORBVocabulary.loadFromTextFile(p, emulate_tail=False)
    bow, fv = vg.transform(np.ones((10, 32), np.uint8))
    assert bow == {} and fv == {}
    # zero features, one feature, capacity above the LDS sort width
    parent, leaf, desc, weight = synth.vocabulary_irregular(k=6, L=4, seed=7)
    vg = plvi.ORBVocabulary.from_nodes(6, 4, 0, 0, parent, leaf, desc, weight)
    vo = oracle_lib.Vocab.create(6, 4, 0, 0, parent, leaf, desc, weight)
    assert vg.transform(np.zeros((0, 32), np.uint8)) == ({}, {})
    for n in (1, 255, 256, 257, 2500):
        _gpu_vs_oracle(vg, vo, synth.vocab_features(parent, leaf, desc, n, seed=n), 2)


@pytest.mark.gpu
def test_vocab_batch_orb_descriptors_full_tree():
    """k=10, L=6 (ORBvoc.txt's shape, 1.1M nodes) on real ORB descriptors of
    synthetic frames through the batched device API."""
    import ctypes
    import plvi
    parent, leaf, desc, weight = synth.vocabulary(10, 6, seed=1)
    vg = plvi.ORBVocabulary.from_nodes(10, 6, 0, 0, parent, leaf, desc, weight)
    vo = oracle_lib.Vocab.create(10, 6, 0, 0, parent, leaf, desc, weight)
    B = 4
    frames = synth.batch(B, seed0=50)
    orb = plvi.ORBextractor(1000, 1.2, 8, 20, 7, 640, 480, max_batch=B)
    dfr = plvi.DeviceBuffer(frames.nbytes)
    dfr.upload(frames)
    orb.extract_batch(dfr.ptr, B, 640 * 480, 640)
    lib = plvi.load()
    lib.plvi_device_synchronize()  # the extractor runs on its own stream
    kp, de, co, mo, cap = orb.outputs()
    outs = {k: plvi.DeviceBuffer(B * (cap + 1) * s) for k, s in
            (("bw", 4), ("bv", 8), ("bn", 4), ("fn", 4), ("fo", 4), ("fi", 4), ("fc", 4), ("w", 4), ("ni", 4))}
    ptr = {k: ctypes.c_void_p(b.ptr) for k, b in outs.items()}
    rc = lib.plvi_vocab_transform_batch(vg._h, ctypes.c_void_p(de), ctypes.c_void_p(co), cap, B, 4, ptr["bw"],
                                        ptr["bv"], ptr["bn"], ptr["fn"], ptr["fo"], ptr["fi"], ptr["fc"], ptr["w"],
                                        ptr["ni"], None)
    assert rc == 0
    lib.plvi_device_synchronize()
    counts = plvi.download(co, np.zeros(B, np.int32))
    D = plvi.download(de, np.zeros((B, cap, 32), np.uint8))
    get = lambda k, dt, shape: outs[k].download(np.zeros(shape, dt))
    bw, bv, bn = get("bw", np.uint32, (B, cap)), get("bv", np.float64, (B, cap)), get("bn", np.int32, B)
    fn, fo, fi, fc = (get("fn", np.uint32, (B, cap)), get("fo", np.int32, (B, cap + 1)), get("fi", np.uint32, (B, cap)),
                      get("fc", np.int32, B))
    for f in range(B):
        n = counts[f]
        assert n > 500
        e = vo.transform(D[f, :n], 4)
        assert bn[f] == len(e[0]) and fc[f] == len(e[2])
        np.testing.assert_array_equal(bw[f, :bn[f]], e[0])
        np.testing.assert_array_equal(bv[f, :bn[f]], e[1])
        np.testing.assert_array_equal(fn[f, :fc[f]], e[2])
        np.testing.assert_array_equal(fo[f, :fc[f] + 1], e[3])
        np.testing.assert_array_equal(fi[f, :fo[f, fc[f]]], e[4])
