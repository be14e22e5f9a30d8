"""Diagnostic: determinism of tracked sequences -- the same sequences run twice (and with a different length)
must give bit-identical trajectories.   python tools/ate_probe3.py n"""
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "sp-slam_amd"), str(ROOT / "oracle"), str(ROOT)]


def run(n, T):
    import pipeline
    import sequence
    sp = sequence.SequencePath(2, T, n_sequences=2, render_workers=16, **pipeline.CONFIGS["c2"])
    for _ in range(n):
        sp.step()
    tr, h = sp.trajectory(), sp.history()
    sp.close()
    return tr, h


def main(n):
    a = run(n, n + 1)
    b = run(n, n + 1)
    c = run(n, 2 * n + 1)
    for name, (x, y) in (("repeat", (a, b)), ("longer", (a, c))):
        for slot in range(2):
            d = [t for t in range(1, n + 1) if x[0][t, slot].tobytes() != y[0][t, slot].tobytes()]
            e = [t for t in range(1, n + 1) if not np.array_equal(x[1][t, slot], y[1][t, slot])]
            print(f"{name} slot {slot}: frame {n - 9} {x[1][n - 9, slot]} vs {y[1][n - 9, slot]}; first pose difference {d[:1]}, first decision difference {e[:1]}"
                  + (f" {x[1][e[0], slot]} vs {y[1][e[0], slot]}" if e else ""), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]))
