"""The C++ step chain (oracle/step_oracle.cpp, bench.py's cpu_baseline) equals the Python stage-by-stage
oracle (oracle/oracle_step.py, the GPU step's checker) on the same frame: same keypoint / plane / match counts
and the same poses after both PoseOptimizations -- so the CPU baseline times the work the parity tests check."""
import numpy as np
import pytest

import oracle_step
import oracle_step_cpp
import synth


@pytest.mark.parametrize("seq,frame,K,min_size", [(0, 6, synth.TUM3, 500), (1, 9, synth.ICL, 1000)])
def test_cpp_chain_equals_python_chain(seq, frame, K, min_size):
    import oracle_ctypes
    import oracle_planes
    import spslam_gpu as G
    cfg = G.PlaneConfig(1.0, 100.0, 0.5, 0.5, 1000.0, 200.0) if K is synth.ICL else None
    fi = oracle_step.synthetic(seq, frame, K=K, min_size=min_size, pose_cfg=cfg)
    py = oracle_step.run(fi, oracle_ctypes.OrbOracle(nfeatures=1000), oracle_planes.PlaneOracle(), supp_cap=16)
    cc = oracle_step_cpp.run_frame(fi, supp_cap=16)
    assert cc["n_kps"] == len(py["kps"]) and cc["nmatches"] == py["nmatches"]
    assert cc["n_planes"] == len(py["planes"]["coef"]) and cc["n_supposed"] == min(16, len(py["supposed"]["coef"]))
    assert cc["local_nmatches"] == py["local_nmatches"]
    assert cc["inliers1"] == py["pose1"][0]["n_inliers"] and cc["inliers2"] == py["pose2"][0]["n_inliers"]
    assert np.array_equal(cc["Tcw1"].reshape(16), py["pose1"][0]["Tcw"])
    assert np.array_equal(cc["Tcw2"].reshape(16), py["pose2"][0]["Tcw"])
    assert cc["nmatches"] > 100 and cc["inliers2"] > 100


def test_bench_loop_threads():
    fi = [oracle_step.synthetic(0, f) for f in (6, 9)]
    el, outs = oracle_step_cpp.bench(fi, 1000, warmup=1, timed=2, threads=2)
    assert (el > 0).all() and len(outs) == 2
    one = oracle_step_cpp.run_frame(fi[1])
    assert np.array_equal(outs[1]["Tcw2"], one["Tcw2"])
