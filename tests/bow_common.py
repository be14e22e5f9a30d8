"""Shared inputs of the bag-of-words tests: the in-repo DBoW2 vocabulary
(tests/golden/vocab_k6_l6.txt.gz, trained by tools/make_vocab.py), ORB
features of synthetic frames (CPU oracle), and an independent pure-Python
transcription of DBoW2's loadFromTextFile / transform and of
ORBmatcher::SearchByBoW used to pin the C++ oracle."""
import gzip
import math
import pathlib

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
VOCAB = ROOT / "tests" / "golden" / "vocab_k6_l6.txt.gz"
POP = np.array([bin(i).count("1") for i in range(256)], np.int32)


def vocab_text():
    return gzip.open(VOCAB, "rb").read()


def shape_vocab_text(k=10, L=6):
    """ORBvoc.txt's shape (k = 10, L = 6, 10^6 words): the harness's generated vocabulary
    (sp-slam_amd/synth.py shape_vocabulary_text)."""
    import synth
    return synth.shape_vocabulary_text(k, L)


def frames(n=4, seq=0, step=5, n_boxes=3, nfeatures=1000):
    """(keypoints, descriptors) of n synthetic frames, CPU oracle ORB."""
    import oracle_ctypes
    import synth
    orb = oracle_ctypes.OrbOracle(nfeatures=nfeatures)
    sc = synth.Scene(seq, n_boxes=n_boxes)
    out = []
    for i in range(n):
        g, _, _ = sc.render(sc.pose(step * i), noise_seed=step * i)
        out.append(orb.extract(g))
    return out


class PyVocab:
    """TemplatedVocabulary::loadFromTextFile, restated in Python (TemplatedVocabulary.h:1338-1424)."""

    def __init__(self, text: bytes):
        lines = text.decode().split("\n")
        k, L, sc, wt = (int(x) for x in lines[0].split())
        self.k, self.L, self.scoring, self.weighting = k, L, sc, wt
        self.children, self.desc, self.weight, self.word = [[]], [bytes(32)], [0.0], [0]
        nw = 0
        for ln in lines[1:]:  # split() yields the empty string after a final newline: the phantom node
            tok = ln.split()
            pid = int(tok[0]) if tok else 0
            leaf = int(tok[1]) if len(tok) > 1 else 0
            d = bytes(int(x) for x in tok[2:34]) if len(tok) >= 34 else bytes(32)
            w = float(tok[34]) if len(tok) > 34 else 0.0
            nid = len(self.children)
            self.children.append([])
            self.children[pid].append(nid)
            self.desc.append(d)
            self.weight.append(w)
            self.word.append(nw if leaf > 0 else 0)
            nw += leaf > 0
        self.n_words = nw
        self.D = np.frombuffer(b"".join(self.desc), np.uint8).reshape(-1, 32)

    def word_of(self, f, levelsup=4):
        """transform(feature, word_id, weight, &nid, levelsup) (:1217-1259)."""
        nid_level = self.L - levelsup
        node, level, nid = 0, 0, (0 if nid_level <= 0 else None)
        while True:
            level += 1
            ch = self.children[node]
            d = POP[self.D[ch] ^ f].sum(1)
            node = ch[int(np.argmin(d))]  # first minimum
            if level == nid_level:
                nid = node
            if not self.children[node]:
                break
        return self.word[node], self.weight[node], node if nid is None else nid

    def transform(self, desc, levelsup=4):
        bv, fv = {}, {}
        tf = self.weighting in (0, 1)
        for i, f in enumerate(np.asarray(desc, np.uint8).reshape(-1, 32)):
            w, wt, nid = self.word_of(f, levelsup)
            if wt > 0:
                if w in bv:
                    if tf:
                        bv[w] += wt
                else:
                    bv[w] = wt
                fv.setdefault(nid, []).append(i)
        words = sorted(bv)
        must = self.scoring != 5
        if tf and bv and not must:
            for w in words:
                bv[w] /= float(len(bv))
        if must:
            if self.scoring == 1:
                norm = math.sqrt(sum(bv[w] * bv[w] for w in words)) if words else 0.0
            else:
                norm = 0.0
                for w in words:
                    norm += abs(bv[w])
            if norm > 0:
                for w in words:
                    bv[w] /= norm
        nodes = sorted(fv)
        start = np.cumsum([0] + [len(fv[n]) for n in nodes]).astype(np.int32)
        feats = np.array([i for n in nodes for i in fv[n]], np.int32)
        return dict(words=np.array(words, np.uint32), values=np.array([bv[w] for w in words], np.float64),
                    nodes=np.array(nodes, np.uint32), start=start, features=feats)


def py_search_by_bow(kd, ka, has, kfv, fd, fa, ffv, nn_ratio=0.7, check_ori=True):
    """ORBmatcher::SearchByBoW (src/ORBmatcher.cc:159-288), restated in Python."""
    f32 = np.float32
    match = np.full(len(fd), -1, np.int32)
    hist = [[] for _ in range(30)]
    n = 0
    kpos = {int(x): j for j, x in enumerate(kfv["nodes"])}
    for b, node in enumerate(ffv["nodes"]):
        a = kpos.get(int(node))
        if a is None:
            continue
        for p in range(kfv["start"][a], kfv["start"][a + 1]):
            i = int(kfv["features"][p])
            if not has[i]:
                continue
            b1, bi, b2 = 256, -1, 256
            for q in range(ffv["start"][b], ffv["start"][b + 1]):
                j = int(ffv["features"][q])
                if match[j] >= 0:
                    continue
                d = int(POP[kd[i] ^ fd[j]].sum())
                if d < b1:
                    b2, b1, bi = b1, d, j
                elif d < b2:
                    b2 = d
            if b1 <= 50 and f32(b1) < f32(f32(nn_ratio) * f32(b2)):
                match[bi] = i
                if check_ori:
                    rot = f32(f32(ka[i]) - f32(fa[bi]))
                    if rot < 0:
                        rot = f32(rot + f32(360.0))
                    x = f32(rot * f32(1.0 / 30))
                    bn = int(math.floor(abs(float(x)) + 0.5)) * (1 if x >= 0 else -1)  # roundf
                    if bn == 30:
                        bn = 0
                    hist[bn].append(bi)
                n += 1
    if check_ori:
        m1 = m2 = m3 = 0
        i1 = i2 = i3 = -1
        for i in range(30):
            s = len(hist[i])
            if s > m1:
                m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, i
            elif s > m2:
                m3, m2, i3, i2 = m2, s, i2, i
            elif s > m3:
                m3, i3 = s, i
        if m2 < f32(0.1) * f32(m1):
            i2 = i3 = -1
        elif m3 < f32(0.1) * f32(m1):
            i3 = -1
        for i in range(30):
            if i in (i1, i2, i3):
                continue
            for j in hist[i]:
                match[j] = -1
                n -= 1
    return match, n
