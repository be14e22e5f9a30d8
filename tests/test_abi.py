"""CPU checks of the drop-in boundary (include/spslam_gpu.h): the built HIP
library loads, exports every declared entry point, its struct layouts match
the Python bindings, it does not depend on the oracle, and it fails loudly
(an error code, no CPU fallback) when no GPU is present.  No compute calls.
"""
import ctypes
import pathlib
import re
import subprocess

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "spslam_gpu.h"
LIB = ROOT / "sp-slam_amd" / "libspslam_gpu.so"


def declared_functions():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\**\s*(spslam_\w+)\s*\(", text, flags=re.M)))


def test_library_exports_every_declared_symbol():
    import spslam_assoc  # noqa: F401  (each binding module registers its entry points)
    import spslam_gpu
    import spslam_match  # noqa: F401
    import spslam_track  # noqa: F401
    lib = spslam_gpu.load_library()
    names = declared_functions()
    assert len(names) >= 19, names
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(spslam_gpu.EXPORTED) <= set(names)


def test_library_has_no_oracle_dependency():
    out = subprocess.run(["readelf", "-d", str(LIB)], capture_output=True, text=True, check=True).stdout
    needed = re.findall(r"\(NEEDED\).*\[(.*)\]", out)
    assert any("amdhip64" in n for n in needed), needed
    assert not any("oracle" in n for n in needed), needed
    syms = subprocess.run(["nm", "-D", "--defined-only", str(LIB)], capture_output=True, text=True, check=True).stdout
    assert "oracle_" not in syms
    for py in (ROOT / "sp-slam_amd").glob("*.py"):
        assert "oracle" not in re.sub(r"#.*|\"\"\".*?\"\"\"", "", py.read_text(), flags=re.S), \
            f"{py.name} references the oracle"


LAYOUT_C = r"""
#include <stddef.h>
#include <stdio.h>
#include "spslam_gpu.h"
#define S(T) printf(#T " %zu\n", sizeof(T));
#define O(T, f) printf(#T "." #f " %zu\n", offsetof(T, f));
int main(void) {
  S(spslam_keypoint) O(spslam_keypoint, octave) O(spslam_keypoint, class_id)
  S(spslam_point_obs) O(spslam_point_obs, xw) O(spslam_point_obs, kp_index)
  S(spslam_plane_obs) O(spslam_plane_obs, kind)
  S(spslam_pose_problem) O(spslam_pose_problem, point_offset) O(spslam_pose_problem, plane_offset)
  S(spslam_pose_result) S(spslam_plane) O(spslam_plane, n_inliers) O(spslam_plane, contour_offset)
  S(spslam_orb_params) S(spslam_plane_params) S(spslam_plane_config)
  S(spslam_supposed_plane) O(spslam_supposed_plane, line) O(spslam_supposed_plane, source_plane)
  O(spslam_supposed_plane, patch_offset)
  S(spslam_line_candidate) O(spslam_line_candidate, n_inliers) O(spslam_line_candidate, idx_offset)
  S(spslam_map_plane) O(spslam_map_plane, id) O(spslam_map_plane, boundary_offset) O(spslam_map_plane, n_boundary)
  S(spslam_assoc_frame) O(spslam_assoc_frame, map_offset) O(spslam_assoc_frame, n_map) O(spslam_assoc_frame, carry)
  S(spslam_assoc_params)
  S(spslam_proj_point) O(spslam_proj_point, angle) O(spslam_proj_point, n_obs) O(spslam_proj_point, id)
  O(spslam_proj_point, desc)
  S(spslam_proj_frame) O(spslam_proj_frame, Tlw) O(spslam_proj_frame, point_offset) S(spslam_match_params)
  S(spslam_local_point) O(spslam_local_point, normal) O(spslam_local_point, max_dist) O(spslam_local_point, desc)
  S(spslam_local_frame) O(spslam_local_frame, n_points) O(spslam_local_frame, stamp) S(spslam_local_params)
  O(spslam_local_point, n_obs)
  S(spslam_track_batch) O(spslam_track_batch, cap) O(spslam_track_batch, proj_frames)
  O(spslam_track_batch, stride_a) O(spslam_track_batch, cap_b) O(spslam_track_batch, map)
  O(spslam_track_batch, point_outlier) O(spslam_track_batch, fx) O(spslam_track_batch, bf)
  O(spslam_track_batch, plane_outlier) O(spslam_track_batch, next_vertical) O(spslam_track_batch, problems)
  O(spslam_track_batch, seen) O(spslam_track_batch, velocity)
  S(spslam_refkf_batch) O(spslam_refkf_batch, refkf_counts) O(spslam_refkf_batch, rows_stride)
  O(spslam_refkf_batch, refkf_sets) O(spslam_refkf_batch, state) O(spslam_refkf_batch, refkf_assoc)
  S(spslam_frame_region) O(spslam_frame_region, frame_bytes) O(spslam_frame_region, src_stride)
  S(spslam_refkf_vote) O(spslam_refkf_vote, ids_per_kf) O(spslam_refkf_vote, new_kf) O(spslam_refkf_vote, state)
  O(spslam_refkf_vote, refkf_sets) O(spslam_refkf_vote, refkf_pairs)
  return 0;
}
"""


def test_struct_layouts_match_bindings(tmp_path):
    import spslam_assoc
    import spslam_gpu
    import spslam_match
    import spslam_planes
    src = tmp_path / "layout.c"
    src.write_text(LAYOUT_C)
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", str(ROOT / "include"), str(src), "-o", str(exe)], check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                         check=True).stdout.splitlines())
    got = {k: int(v) for k, v in got.items()}
    checks = {
        "spslam_keypoint": spslam_gpu.KEYPOINT_DTYPE, "spslam_point_obs": spslam_gpu.POINT_OBS_DTYPE,
        "spslam_plane_obs": spslam_gpu.PLANE_OBS_DTYPE, "spslam_pose_problem": spslam_gpu.POSE_PROBLEM_DTYPE,
        "spslam_pose_result": spslam_gpu.POSE_RESULT_DTYPE, "spslam_plane": spslam_planes.PLANE_DTYPE,
        "spslam_supposed_plane": spslam_planes.SUPPOSED_DTYPE, "spslam_line_candidate": spslam_planes.LINE_CAND_DTYPE,
        "spslam_map_plane": spslam_assoc.MAP_PLANE_DTYPE, "spslam_assoc_frame": spslam_assoc.ASSOC_FRAME_DTYPE,
        "spslam_proj_point": spslam_match.PROJ_POINT_DTYPE, "spslam_proj_frame": spslam_match.PROJ_FRAME_DTYPE,
        "spslam_local_point": spslam_match.LOCAL_POINT_DTYPE, "spslam_local_frame": spslam_match.LOCAL_FRAME_DTYPE,
    }
    for name, dt in checks.items():
        assert got[name] == dt.itemsize, (name, got[name], dt.itemsize)
        for key, off in got.items():
            if key.startswith(name + "."):
                field = key.split(".", 1)[1]
                assert dt.fields[field][1] == off, (key, off, dt.fields[field][1])
    assert got["spslam_orb_params"] == ctypes.sizeof(spslam_gpu.OrbParams)
    assert got["spslam_plane_params"] == ctypes.sizeof(spslam_planes.PlaneParams)
    assert got["spslam_plane_config"] == 6 * 8
    assert got["spslam_assoc_params"] == ctypes.sizeof(spslam_assoc.AssocParams)
    assert got["spslam_match_params"] == ctypes.sizeof(spslam_match.MatchParams)
    assert got["spslam_local_params"] == ctypes.sizeof(spslam_match.LocalParams)
    assert got["spslam_keypoint"] == 28  # cv::KeyPoint
    import spslam_track
    tb = spslam_track.TrackBatch
    assert got["spslam_track_batch"] == ctypes.sizeof(tb)
    for key, off in got.items():
        if key.startswith("spslam_track_batch."):
            assert getattr(tb, key.split(".", 1)[1]).offset == off, key
    for name, st in (("spslam_refkf_batch", spslam_track.RefkfBatch), ("spslam_frame_region", spslam_track.FrameRegion),
                     ("spslam_refkf_vote", spslam_track.RefkfVote)):
        assert got[name] == ctypes.sizeof(st), name
        for key, off in got.items():
            if key.startswith(name + "."):
                assert getattr(st, key.split(".", 1)[1]).offset == off, key


def test_fails_loudly_without_gpu():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import spslam_gpu
    with pytest.raises(spslam_gpu.SpslamError):
        spslam_gpu.OrbExtractor()
    lib = spslam_gpu.load_library()
    lib.spslam_kernel_name.restype = ctypes.c_char_p
    assert lib.spslam_kernel_name(0) == b"level_kernel"
    assert np.dtype(spslam_gpu.KEYPOINT_DTYPE).itemsize == 28
