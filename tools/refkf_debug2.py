"""Diagnostic: a tracked C2 batch with and without the TrackReferenceKeyFrame machinery: identical?"""
import pathlib
import sys
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "sp-slam_amd"), str(ROOT)]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import pipeline  # noqa: E402
import sequence  # noqa: E402

out = {}
for fbk in (False, True):
    sp = sequence.SequencePath(4, 23, n_sequences=2, pipelined=False, refkf_fallback=fbk, **pipeline.CONFIGS["c2"])
    for k in range(21):
        sp.step()
    out[fbk] = (sp.trajectory(), sp.history())
    sp.close()
a, b = out[False], out[True]
for t in range(1, 22):
    same = a[0][t].tobytes() == b[0][t].tobytes()
    print(t, "pose same" if same else "POSE DIFF", "hist", a[1][t].tolist(), b[1][t].tolist(), flush=True)
