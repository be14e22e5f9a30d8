#!/usr/bin/env python3
"""Train the in-repo DBoW2 vocabulary (tests/golden/vocab_k6_l6.txt.gz).

The reference loads ORBvoc.txt (k = 10, L = 6, ~1M words) with
TemplatedVocabulary::loadFromTextFile (src/System.cc:64), but that blob is not
vendored (.MISSING_LARGE_BLOBS:2).  The BoW path (Frame::ComputeBoW,
ORBmatcher::SearchByBoW) only needs *a* vocabulary in DBoW2's format, so this
script trains one the way DBoW2's TemplatedVocabulary::create does
(Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h):

  * HKmeansStep (:642-811): per node, <= k descriptors -> one child each, else
    k-majority: k-means++ seeding (initiateClustersKMpp), assign to the nearest
    center (first minimum), FORB::meanValue (bitwise majority, ties -> 1,
    FORB.cpp) until the assignment stops changing; children get consecutive ids,
    then the recursion runs child by child (depth first), skipping children
    with <= 1 descriptor;
  * setNodeWeights (:943-996): TF-IDF, weight = log(NDocs / Ni) per word, Ni =
    training images whose descriptors reach the word;
  * saveToTextFile (:1429-1455): "k L scoring weighting", then per node
    "parent isLeaf d0 .. d31 weight" (weight as `ostream << double`, 6
    significant digits), one line each, trailing newline.

Training data: ORB descriptors (CPU oracle, nFeatures 1000) of synthetic
frames from several scenes (sp-slam_amd/synth.py).  Deterministic (seeded).
k = 6, L = 6 keeps the file small while Frame::ComputeBoW's levelsup = 4 still
puts the FeatureVector at level 2, as with ORBvoc (36 nodes instead of 100).

    python tools/make_vocab.py [--out tests/golden/vocab_k6_l6.txt.gz]
"""
from __future__ import annotations

import argparse
import gzip
import math
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "sp-slam_amd"), str(ROOT / "oracle")]

POP = np.array([bin(i).count("1") for i in range(256)], np.uint8)


def hamming(a, b):
    """(n, 32) x (m, 32) u8 -> (n, m) Hamming distances."""
    out = np.zeros((len(a), len(b)), np.int32)
    for j in range(0, len(b), 16):
        out[:, j:j + 16] = POP[a[:, None, :] ^ b[None, j:j + 16, :]].sum(-1)
    return out


def majority(desc):
    """FORB::meanValue: bit set iff set in >= ceil(n / 2) descriptors (MSB first in each byte)."""
    if len(desc) == 1:
        return desc[0].copy()
    bits = np.unpackbits(desc, axis=1).astype(np.int32).sum(0)
    n2 = len(desc) // 2 + len(desc) % 2
    return np.packbits((bits >= n2).astype(np.uint8))


def kmeanspp(desc, k, rng):
    """initiateClustersKMpp: first center uniform, then each next one with probability ~ its distance to the
    closest chosen center."""
    centers = [desc[rng.integers(len(desc))]]
    dmin = hamming(desc, centers[0][None])[:, 0].astype(np.float64)
    while len(centers) < k:
        s = dmin.sum()
        if s <= 0:
            break
        i = int(np.searchsorted(np.cumsum(dmin), rng.random() * s, side="right"))
        i = min(i, len(desc) - 1)
        centers.append(desc[i])
        dmin = np.minimum(dmin, hamming(desc, desc[i][None])[:, 0])
    return np.array(centers, np.uint8)


class Tree:
    def __init__(self, k, L):
        self.k, self.L = k, L
        self.parent, self.desc, self.children = [0], [np.zeros(32, np.uint8)], [[]]

    def add(self, parent, d):
        nid = len(self.parent)
        self.parent.append(parent)
        self.desc.append(d)
        self.children.append([])
        self.children[parent].append(nid)
        return nid

    def step(self, parent, desc, level, rng):
        """HKmeansStep(parent_id, descriptors, current_level)."""
        if len(desc) == 0:
            return
        if len(desc) <= self.k:
            clusters = [d for d in desc]
            groups = [np.array([i]) for i in range(len(desc))]
        else:
            clusters = kmeanspp(desc, self.k, rng)
            last = None
            for _ in range(30):
                assign = hamming(desc, clusters).argmin(1)  # first minimum, as the `d < best` loop
                if last is not None and np.array_equal(assign, last):
                    break
                last = assign
                clusters = np.array([majority(desc[assign == c]) if (assign == c).any() else clusters[c]
                                     for c in range(len(clusters))], np.uint8)
            groups = [np.nonzero(assign == c)[0] for c in range(len(clusters))]
        ids = [self.add(parent, np.asarray(c, np.uint8)) for c in clusters]
        if level < self.L:
            for nid, g in zip(ids, groups):
                if len(g) > 1:
                    self.step(nid, desc[g], level + 1, rng)

    def word(self, d):
        """transform(feature) -> leaf node id (first minimum per level)."""
        node = 0
        while self.children[node]:
            ch = self.children[node]
            node = ch[int(hamming(d[None], np.array([self.desc[c] for c in ch]))[0].argmin())]
        return node


def training_descriptors(n_frames, seeds):
    import oracle_ctypes
    import synth
    orb = oracle_ctypes.OrbOracle()
    docs = []
    per = max(1, n_frames // len(seeds))
    for s in seeds:
        sc = synth.Scene(s, n_boxes=3 + s % 5)
        for i in range(per):
            g, _, _ = sc.render(sc.pose(7 * i + s), noise_seed=100 + 7 * i)
            _, d = orb.extract(g)
            docs.append(np.asarray(d, np.uint8))
    return docs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=str(ROOT / "tests" / "golden" / "vocab_k6_l6.txt.gz"))
    ap.add_argument("--k", type=int, default=6)
    ap.add_argument("--L", type=int, default=6)
    ap.add_argument("--frames", type=int, default=240)
    args = ap.parse_args()
    rng = np.random.default_rng(0xB0E)
    docs = training_descriptors(args.frames, seeds=list(range(8)))
    alld = np.concatenate(docs)
    print(f"{len(alld)} training descriptors from {len(docs)} frames", flush=True)
    T = Tree(args.k, args.L)
    T.step(0, alld, 1, rng)
    leaves = [n for n in range(1, len(T.parent)) if not T.children[n]]
    wid = {n: i for i, n in enumerate(leaves)}
    ni = np.zeros(len(leaves), np.int64)
    for d in docs:  # setNodeWeights: images reaching each word
        seen = {wid[T.word(x)] for x in d}
        for w in seen:
            ni[w] += 1
    weight = np.zeros(len(T.parent))
    for n, w in wid.items():
        if ni[w] > 0:
            weight[n] = math.log(len(docs) / ni[w])
    lines = [f"{args.k} {args.L}  0 0"]  # saveToTextFile writes two spaces before the scoring type
    for n in range(1, len(T.parent)):
        leaf = 0 if T.children[n] else 1
        lines.append(f"{T.parent[n]} {leaf} " + "".join(f"{int(b)} " for b in T.desc[n]) + f"{weight[n]:g}")
    text = "\n".join(lines) + "\n"
    with gzip.open(args.out, "wt", compresslevel=9) as f:
        f.write(text)
    depth_ok = all(T.children[c] for c in T.children[0])  # no leaf at level 1 (FeatureVector level 2 reached)
    print(f"{len(T.parent)} nodes, {len(leaves)} words, level-1 leaves: {not depth_ok}, {len(text) / 1e6:.1f} MB text "
          f"-> {args.out}", flush=True)


if __name__ == "__main__":
    main()
