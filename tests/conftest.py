"""Test configuration.

Markers:
  gpu -- needs a HIP device (MI355X); run with `pytest -m gpu` on the GPU box.
Everything else runs on the CPU-only build container.
"""
import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
for p in (ROOT / "sp-slam_amd", ROOT / "oracle", ROOT):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs a HIP GPU (MI355X)")


@pytest.fixture(scope="session")
def synth_frames():
    """Four 640x480 frames of synthetic sequence 0 (gray, depth u16, Twc)."""
    import synth
    sc = synth.Scene(0)
    out = []
    for i in (0, 7, 19, 40):
        T = sc.pose(i)
        g, d, _ = sc.render(T, noise_seed=i)
        out.append((g, d, T))
    return out
