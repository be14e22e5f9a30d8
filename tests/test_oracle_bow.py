"""CPU checks of the bag-of-words oracle (oracle/bow_oracle.cpp): DBoW2
TemplatedVocabulary::loadFromTextFile / transform (Frame::ComputeBoW,
src/Frame.cc:495-502) and ORBmatcher::SearchByBoW (src/ORBmatcher.cc:159-288).

Parity anchors: the reference ships no vocabulary (ORBvoc.txt is missing,
.MISSING_LARGE_BLOBS:2) and no fixtures, so the oracle is checked against an
independent pure-Python transcription (tests/bow_common.py) on the in-repo
vocabulary and synthetic ORB features, and against hand-built vocabularies
with known answers (ties, stop words, the trailing-newline phantom node,
levelsup above the tree depth)."""
import numpy as np
import pytest

import bow_common as BC
import oracle_bow


@pytest.fixture(scope="module")
def vocabs():
    t = BC.vocab_text()
    return oracle_bow.Vocabulary(t), BC.PyVocab(t)


@pytest.fixture(scope="module")
def feats():
    return BC.frames(3)


def test_loader_counts(vocabs):
    ov, pv = vocabs
    assert (ov.k, ov.L) == (6, 6)
    assert ov.n_nodes == len(pv.children) and ov.n_words == pv.n_words
    # the file ends with a newline: one phantom leaf under the root, weight 0, not a word
    assert pv.children[0][-1] == ov.n_nodes - 1 and pv.weight[-1] == 0.0


def _same(a, b):
    for k in ("words", "values", "nodes", "start", "features"):
        assert a[k].tobytes() == np.asarray(b[k], a[k].dtype).tobytes(), k


def test_transform_matches_transcription(vocabs, feats):
    ov, pv = vocabs
    for kps, desc in feats:
        o = ov.transform(desc)
        _same(o, pv.transform(desc))
        assert len(o["words"]) > 300 and 10 <= len(o["nodes"]) <= 36  # FeatureVector at level 2 of a k=6 tree
        assert abs(o["values"].sum() - 1.0) < 1e-12                     # L1-normalised (L1_NORM scoring)
        w, wt, nid = ov.words(desc)
        for i in range(0, len(desc), 97):
            assert (int(w[i]), float(wt[i]), int(nid[i])) == pv.word_of(desc[i]), i


def test_search_by_bow_matches_transcription(vocabs, feats):
    ov, _ = vocabs
    rng = np.random.default_rng(4)
    tot = 0
    for a, b in ((0, 1), (1, 2), (0, 2)):
        (kk, kd), (fk, fd) = feats[a], feats[b]
        kfv, ffv = ov.transform(kd), ov.transform(fd)
        has = (rng.random(len(kd)) < 0.8).astype(np.uint8)
        for nn, ori in ((0.7, True), (0.75, True), (0.7, False)):
            m, n = oracle_bow.search_by_bow(kd, kk["angle"], has, kfv, fd, fk["angle"], ffv, nn, ori)
            pm, pn = BC.py_search_by_bow(kd, kk["angle"], has, kfv, fd, fk["angle"], ffv, nn, ori)
            assert n == pn and np.array_equal(m, pm), (a, b, nn, ori)
            assert n == int((m >= 0).sum())
            tot += n
    assert tot > 100


def _tiny(newline=True, scoring=0, weighting=0):
    """k=2, L=2 vocabulary: root -> A (0x00..), B (0xff..); A -> a0, a1 (leaves), B -> b0 (leaf, stop word)."""
    z, o = " ".join(["0"] * 32), " ".join(["255"] * 32)
    a1 = " ".join(["15"] + ["0"] * 31)
    rows = [f"2 2  {scoring} {weighting}", f"0 0 {z} 0", f"0 0 {o} 0", f"1 1 {z} 1.5", f"1 1 {a1} 0.5",
            f"2 1 {o} 0"]
    return ("\n".join(rows) + ("\n" if newline else "")).encode()


def test_tiny_vocabulary_known_answers():
    v = oracle_bow.Vocabulary(_tiny())
    assert (v.n_nodes, v.n_words) == (7, 3)  # root + 5 + the phantom node
    f = np.zeros((5, 32), np.uint8)
    f[1, 0] = 0x0f          # word 1 (a1) exactly
    f[2, 0] = 0x03          # distance 2 to a0 and 2 to a1: first minimum -> a0
    f[3] = 0xff             # b0: a stop word (weight 0) -> in neither vector
    f[4, :20] = 0xff        # 160 bits: closer to B (96) than to A (160) -> b0, stopped
    w, wt, nid = v.words(f, levelsup=1)
    assert list(w) == [0, 1, 0, 2, 2] and list(wt) == [1.5, 0.5, 1.5, 0.0, 0.0]
    assert list(nid) == [1, 1, 1, 2, 2]     # level L - levelsup = 1
    o = v.transform(f, levelsup=1)
    assert list(o["words"]) == [0, 1]
    np.testing.assert_array_equal(o["values"], np.array([3.0, 0.5]) / 3.5)
    assert list(o["nodes"]) == [1] and list(o["features"]) == [0, 1, 2]
    o = v.transform(f, levelsup=4)          # levelsup >= L: every feature in node 0 (the root)
    assert list(o["nodes"]) == [0]
    # IDF weighting: addIfNotExist keeps the first weight, no summing
    o = oracle_bow.Vocabulary(_tiny(weighting=2)).transform(f, levelsup=1)
    np.testing.assert_array_equal(o["values"], np.array([1.5, 0.5]) / 2.0)
    # DOT_PRODUCT scoring does not normalise; TF_IDF then divides by the BowVector size
    o = oracle_bow.Vocabulary(_tiny(scoring=5)).transform(f, levelsup=1)
    np.testing.assert_array_equal(o["values"], np.array([3.0, 0.5]) / 2.0)
    # without the final newline there is no phantom node
    assert oracle_bow.Vocabulary(_tiny(newline=False)).n_nodes == 6
    for t in (_tiny(), _tiny(weighting=2), _tiny(scoring=5), _tiny(scoring=1)):
        pv, ov = BC.PyVocab(t), oracle_bow.Vocabulary(t)
        _same(ov.transform(f, levelsup=1), pv.transform(f, levelsup=1))


def test_empty_inputs(vocabs):
    ov, _ = vocabs
    o = ov.transform(np.zeros((0, 32), np.uint8))
    assert len(o["words"]) == 0 and len(o["nodes"]) == 0 and list(o["start"]) == [0]
    with pytest.raises(ValueError):
        oracle_bow.Vocabulary(b"30 6 0 0\n")
