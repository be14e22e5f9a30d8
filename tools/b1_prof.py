"""Diagnostic: the reference's call pattern (one sequence, B = 1: Examples/RGB-D/SPSLAM.cc:90-136) -- the
single_sequence line of bench.py alone, for a rocprofv3 kernel trace.
    python tools/b1_prof.py [--frames 120] [--serial] [--config c2]
Prints frames/s (pipelined: frame k+1's extraction beside frame k's tail) or per-frame latency (serial)."""
import argparse
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "sp-slam_amd"), str(ROOT)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=120)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--serial", action="store_true")
    ap.add_argument("--config", default="c2")
    ap.add_argument("--lookahead", type=int, default=1)
    ap.add_argument("--max-inflight", type=int, default=0)
    ap.add_argument("--no-refkf", action="store_true", help="without the TrackReferenceKeyFrame failure branch")
    ap.add_argument("--cprofile", default="", help="write the timed loop's host profile (pstats text) here")
    a = ap.parse_args()
    import numpy as np
    import torch
    import pipeline
    import sequence
    cfg = pipeline.CONFIGS[a.config]
    sp = sequence.SequencePath(1, a.frames + a.warmup + 2, n_sequences=1, device=0, pipelined=not a.serial,
                               lookahead=a.lookahead, max_inflight=a.max_inflight,
                               refkf_fallback=False if a.no_refkf else None,
                               render_workers=min(16, os.cpu_count() or 1), **cfg)
    try:
        for _ in range(a.warmup):
            sp.step()
        torch.cuda.synchronize()
        lat = []
        prof = None
        if a.cprofile:
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        t0 = time.perf_counter()
        for _ in range(a.frames):
            ts = time.perf_counter()
            sp.step()
            if a.serial:
                torch.cuda.synchronize()
                lat.append(time.perf_counter() - ts)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if prof is not None:
            import io
            import pstats
            prof.disable()
            buf = io.StringIO()
            st = pstats.Stats(prof, stream=buf)
            st.sort_stats("tottime").print_stats(40)
            st.sort_stats("cumulative").print_stats(40)
            pathlib.Path(a.cprofile).write_text(f"{a.frames} frames, {el:.3f} s\n" + buf.getvalue())
    finally:
        sp.close()
    msg = f"B=1{' no-refkf' if a.no_refkf else ''} {'serial' if a.serial else f'pipelined lookahead {a.lookahead} inflight {a.max_inflight}'}: {a.frames / el:.1f} frames/s"
    if lat:
        msg += f", latency p50 {np.percentile(lat, 50) * 1e3:.2f} ms p99 {np.percentile(lat, 99) * 1e3:.2f} ms"
    print(msg, flush=True)


if __name__ == "__main__":
    main()
