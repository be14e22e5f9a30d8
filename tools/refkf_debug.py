"""Diagnostic: per-frame TrackWithMotionModel verdicts of a tracked C2 batch (fallback flags, matches, BoW)."""
import pathlib
import sys
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "sp-slam_amd"), str(ROOT)]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import pipeline  # noqa: E402
import sequence  # noqa: E402

sp = sequence.SequencePath(4, 23, n_sequences=2, pipelined=False, **pipeline.CONFIGS["c2"])
for k in range(21):
    sp.step()
    torch.cuda.synchronize()
    fb = sp.fb
    print(k + 1, "nmatch", sp.d_nmatch.cpu().numpy(), "fallback", fb["fallback"].cpu().numpy(), "apply",
          fb["apply"].cpu().numpy(), "bow_n", fb["bow_n"].cpu().numpy(), flush=True)
sp.close()
