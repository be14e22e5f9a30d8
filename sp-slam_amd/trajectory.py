"""Trajectory output and the ATE evaluation of the BASELINE metric (host side).

* save_trajectory_tum -- System::SaveTrajectoryTUM's file format
  (src/System.cc:329-384): one line per tracked frame, `fixed` notation,
  timestamp with 6 decimals, then twc (3) and the quaternion of Rwc (x y z w,
  Converter::toQuaternion, src/Converter.cc:134-144, i.e. Eigen's
  Quaterniond(Matrix3d)) with 9 decimals; Rwc = Rcw^T, twc = -Rwc * tcw in
  float like the cv::Mat arithmetic there.
* ate_rmse -- absolute trajectory error as the TUM RGB-D benchmark's
  evaluate_ate.py computes it (Horn's closed-form rigid alignment of the
  estimated camera centres onto the reference ones, then the RMSE of the
  translational residuals).  The reference repository ships no evaluator; this
  is the tool its TUM numbers are quoted with.
"""
from __future__ import annotations

import numpy as np


def quaternion_xyzw(R) -> np.ndarray:
    """Eigen::Quaterniond(const Matrix3d&) (Eigen/src/Geometry/Quaternion.h, quaternionbase_assign_impl):
    returns (x, y, z, w) as Converter::toQuaternion does."""
    m = np.asarray(R, np.float64)
    t = m[0, 0] + m[1, 1] + m[2, 2]
    q = np.zeros(4)  # x y z w
    if t > 0:
        t = np.sqrt(t + 1.0)
        q[3] = 0.5 * t
        t = 0.5 / t
        q[0] = (m[2, 1] - m[1, 2]) * t
        q[1] = (m[0, 2] - m[2, 0]) * t
        q[2] = (m[1, 0] - m[0, 1]) * t
    else:
        i = 0
        if m[1, 1] > m[0, 0]:
            i = 1
        if m[2, 2] > m[i, i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        t = np.sqrt(m[i, i] - m[j, j] - m[k, k] + 1.0)
        q[i] = 0.5 * t
        t = 0.5 / t
        q[3] = (m[k, j] - m[j, k]) * t
        q[j] = (m[j, i] + m[i, j]) * t
        q[k] = (m[k, i] + m[i, k]) * t
    return q


def camera_center(Tcw) -> np.ndarray:
    """twc = -Rcw^T tcw in float32 (System.cc:371-372)."""
    T = np.asarray(Tcw, np.float32).reshape(4, 4)
    Rwc = T[:3, :3].T
    return (-Rwc @ T[:3, 3]).astype(np.float32)


def tum_lines(timestamps, poses_cw):
    """The lines System::SaveTrajectoryTUM writes for the given frame poses (Tcw, world = first keyframe)."""
    out = []
    for ts, T in zip(timestamps, poses_cw):
        T = np.asarray(T, np.float32).reshape(4, 4)
        twc = camera_center(T)
        q = quaternion_xyzw(T[:3, :3].T.astype(np.float64)).astype(np.float32)
        out.append(f"{ts:.6f} " + " ".join(f"{v:.9f}" for v in (*twc, *q)))
    return out


def save_trajectory_tum(path, timestamps, poses_cw):
    with open(path, "w") as f:
        for line in tum_lines(timestamps, poses_cw):
            f.write(line + "\n")


def load_trajectory_tum(path):
    """Returns (timestamps, centres Nx3, quaternions Nx4 xyzw)."""
    a = np.loadtxt(path, ndmin=2)
    return a[:, 0], a[:, 1:4], a[:, 4:8]


def horn_align(model, data):
    """Rotation R, translation t minimising sum |R model_i + t - data_i|^2 (evaluate_ate.py align())."""
    model = np.asarray(model, np.float64).T  # 3xN
    data = np.asarray(data, np.float64).T
    mz = model - model.mean(1, keepdims=True)
    dz = data - data.mean(1, keepdims=True)
    W = mz @ dz.T
    U, _, Vt = np.linalg.svd(W.T)
    S = np.eye(3)
    if np.linalg.det(U) * np.linalg.det(Vt) < 0:
        S[2, 2] = -1
    R = U @ S @ Vt
    t = data.mean(1) - R @ model.mean(1)
    return R, t


def ate_rmse(estimated_centres, reference_centres, align=True) -> float:
    """RMSE of the camera-centre residuals after (optional) Horn alignment."""
    e = np.asarray(estimated_centres, np.float64).reshape(-1, 3)
    r = np.asarray(reference_centres, np.float64).reshape(-1, 3)
    if len(e) == 0:
        return float("nan")
    if align and len(e) >= 3:
        R, t = horn_align(e, r)
        e = (R @ e.T).T + t
    return float(np.sqrt(np.mean(np.sum((e - r) ** 2, axis=1))))
