"""Deterministic, synchronous LocalMapping for the tracked sequences (sp-slam_amd/sequence.py, C3), the stand-in
SURVEY.md Appendix A item 10 asks for: the reference's LocalMapping thread runs LocalBundleAdjustment
asynchronously (src/LocalMapping.cc:48-124, abortable), so a full-pipeline ATE comparison needs a mode where it
runs at a fixed point of the tracking loop, identically in the GPU loop and in the CPU oracle's.

Per sequence, a host-side map model (keyframes, map point observations, map planes) mirrors what the tracking
tail produces, and after every keyframe frame (synth.KEYFRAME_STEP) it

  * inserts the keyframe (Tracking::CreateNewKeyFrame + LocalMapping::ProcessNewKeyFrame, Tracking.cc:1251-1373,
    LocalMapping.cc:126-170): its pose is the frame's tracked pose; its map point matches are the frame's final
    tracked matches (the next frame's last-frame points), each becoming an observation of that point; its
    keypoints without a match take the keyframe's own new points (synth.keyframe_points, one observation each);
    its plane observations are the final PoseOptimization's inlier plane edges (EdgePlane / parallel / vertical);
  * once the map holds more than two keyframes (LocalMapping.cc:82-86), collects the local graph exactly as
    Optimizer::LocalBundleAdjustment does (Optimizer.cc:1156-1298: the keyframe and its covisible keyframes,
    their map points and planes, the fixed cameras that see them; KeyFrame::UpdateConnections' covisibility,
    KeyFrame.cc: >= 15 shared points or the best one, ordered by weight), flattened for the spslam_lba ABI in
    the reference's edge order (std::map<KeyFrame*> iteration by keyframe id);
  * applies the result (Optimizer.cc:1909-1977): outlier point observations erased, local keyframe poses, point
    positions (+ MapPoint::UpdateNormalAndDepth, MapPoint.cc:357-400) and plane coefficients written back -- into
    the local-map point table the next frames' SearchLocalPoints reads, the last frame's map points and, through
    UpdateLastFrame (Tracking.cc:1055-1062: mLastFrame.SetPose(Tlr * pRef->GetPose()) with Tlr = I for the
    keyframe's own frame), the last frame's pose the motion model starts from.

Deviations (both loops share them): keyframes on a fixed schedule; no MapPointCulling / CreateNewMapPoints /
SearchInNeighbors / KeyFrameCulling; no bad flags (MapPoint::EraseObservation's nObs <= 2 discard, MapPoint.cc:129-136); the keyframe's final PoseOptimization outliers are dropped before it becomes
a keyframe (the reference passes them on for the local BA to judge); keyframe 0 is fixed (mnId == 0).

The CPU oracle's loop does not run this module: oracle/oracle_local_map.py states the same bookkeeping
independently (scalar, from the reference), and tests/test_local_mapping_host.py holds the two bit-exact.
"""
from __future__ import annotations

import numpy as np

import spslam_lba as L
import spslam_match as SM
import synth


def camera_center(Tcw):
    T = np.asarray(Tcw, np.float32).reshape(4, 4)
    return (-(T[:3, :3].T.astype(np.float64) @ T[:3, 3].astype(np.float64))).astype(np.float32)


def norm64(v):
    """cv::norm of float 3-vectors (rows of v): squares summed in double in element order, then sqrt (OpenCV's
    normL2Sqr accumulation: ((x^2 + y^2) + z^2))."""
    d = np.asarray(v, np.float32).astype(np.float64)
    return np.sqrt((d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2])


class SeqMap:
    """One sequence's map.  table: every keyframe's own points (spslam_local_point records, keyframe order) --
    the local-map point table SearchLocalPoints reads; planes: the sequence's map planes (spslam_map_plane)."""

    COVIS_TH = 15

    def __init__(self, kf_points, cap, cam, scale_factors, inv_sigma2, map_planes):
        self.cap = cap
        self.fx, self.fy, self.cx, self.cy, self.bf = (float(x) for x in cam)
        self.scale = np.asarray(scale_factors, np.float32)
        self.inv_sigma2 = np.asarray(inv_sigma2, np.float32)
        self.table = np.concatenate(kf_points).copy()
        self.kf_rows = []      # keyframe j's own points: rows [a, b) of the table
        o = 0
        for P in kf_points:
            self.kf_rows.append((o, o + len(P)))
            o += len(P)
        self.row_of = {int(pid): r for r, pid in enumerate(self.table["id"])}
        self.planes = np.asarray(map_planes).copy()
        self.plane_row = {int(pid): r for r, pid in enumerate(self.planes["id"])}
        self.kfs = {}          # j -> dict(Tcw, keys (n, 2), ur, octave, mp {kp: pid}, planes [(kind, row, meas)])
        self.obs = {}          # pid -> {j: kp}
        self.ref = {}          # pid -> reference keyframe (the one that created it)
        self.plane_obs = {}    # plane row -> {kind: {j: meas}}

    # ---- keyframe insertion
    def insert_keyframe(self, j, Tcw, keys_un, uright, octave, matched, plane_edges):
        """matched: {keypoint index: map point id} (the frame's final tracked matches); plane_edges: [(kind,
        map plane id, frame plane coefficients)] of its final PoseOptimization's inlier plane edges."""
        n = len(keys_un)
        kf = dict(Tcw=np.asarray(Tcw, np.float32).reshape(4, 4).copy(),
                  keys=np.asarray(keys_un, np.float32).reshape(n, -1)[:, :2].copy(),
                  ur=np.asarray(uright, np.float32)[:n].copy(), octave=np.asarray(octave, np.int32)[:n].copy(),
                  mp={}, planes=[])
        a, b = self.kf_rows[j]
        own = {pid - j * self.cap: pid for pid in self.table["id"][a:b].tolist()}
        for kp in range(n):
            pid = matched.get(kp)
            if pid is None:
                pid = own.get(kp)
                if pid is None:
                    continue
                self.ref[pid] = j
            kf["mp"][kp] = pid
            self.obs.setdefault(pid, {})[j] = kp
        for kind, plane_id, meas in plane_edges:
            r = self.plane_row[int(plane_id)]
            kf["planes"].append((int(kind), r))
            self.plane_obs.setdefault(r, {}).setdefault(int(kind), {})[j] = np.asarray(meas, np.float32).copy()
        self.kfs[j] = kf

    def covisible(self, j):
        """KeyFrame::UpdateConnections + GetVectorCovisibleKeyFrames: keyframes sharing >= 15 map points with j
        (else the best one: the first maximum in keyframe order, KeyFrame.cc:353), by weight descending (ties: the
        higher id first -- sort + push_front in pointer order, KeyFrame.cc:371-378)."""
        cnt = {}
        for kp, pid in self.kfs[j]["mp"].items():
            for i in self.obs.get(pid, {}):
                if i != j:
                    cnt[i] = cnt.get(i, 0) + 1
        if not cnt:
            return []
        pairs = [(w, i) for i, w in cnt.items() if w >= self.COVIS_TH]
        if not pairs:
            i, w = max(cnt.items(), key=lambda kv: (kv[1], -kv[0]))
            pairs = [(w, i)]
        return [i for w, i in sorted(pairs, reverse=True)]

    # ---- Optimizer::LocalBundleAdjustment's graph collection (:1156-1298), flattened for spslam_lba
    def lba_problem(self, j):
        local = [j] + self.covisible(j)
        lset = set(local)
        points, seen = [], set()
        planes, pseen = [], set()
        for k in local:
            for kp in sorted(self.kfs[k]["mp"]):  # GetMapPointMatches(): keypoint order
                pid = self.kfs[k]["mp"][kp]
                if pid not in seen:
                    seen.add(pid)
                    points.append(pid)
            for kind, r in self.kfs[k]["planes"]:
                if kind == 0 and r not in pseen:  # mvpMapPlanes (the plane edges' planes)
                    pseen.add(r)
                    planes.append(r)
        fixed, fset = [], set()

        def see(i):
            if i not in lset and i not in fset:
                fset.add(i)
                fixed.append(i)
        for pid in points:
            for i in sorted(self.obs[pid]):
                see(i)
        for r in planes:
            for kind in (0, 2, 1):  # GetObservations, GetVerObservations, GetParObservations
                for i in sorted(self.plane_obs.get(r, {}).get(kind, {})):
                    see(i)
        kfs_order = local + fixed
        kidx = {k: n for n, k in enumerate(kfs_order)}
        K = np.zeros(len(kfs_order), L.LBA_KEYFRAME_DTYPE)
        for n, k in enumerate(kfs_order):
            K[n]["Tcw"] = self.kfs[k]["Tcw"].reshape(16)
            K[n]["fx"], K[n]["fy"], K[n]["cx"], K[n]["cy"], K[n]["bf"] = self.fx, self.fy, self.cx, self.cy, self.bf
            K[n]["id"] = k
            K[n]["fixed"] = 1 if (k not in lset or k == 0) else 0  # fixed cameras; KF 0 setFixed(mnId == 0)
        P = np.zeros(len(points), L.LBA_POINT_DTYPE)
        # observations in point order, each point's keyframes ascending; gathered from the keyframes' arrays at once
        src, ob_kf, ob_kp, n_obs = [], [], [], np.zeros(len(points), np.int32)
        for n, pid in enumerate(points):
            obs = self.obs[pid]
            ks = sorted(obs)
            n_obs[n] = len(ks)
            for i in ks:
                src.append((pid, i))
                ob_kf.append(i)
                ob_kp.append(obs[i])
        rows = np.fromiter((self.row_of[pid] for pid in points), np.int64, len(points))
        P["xw"] = self.table["xw"][rows]
        P["id"] = np.asarray(points, np.int64)
        P["n_obs"] = n_obs
        P["obs_offset"] = np.concatenate([[0], np.cumsum(n_obs)[:-1]]) if len(points) else n_obs
        po = np.zeros(len(src), L.LBA_POINT_OBS_DTYPE)
        if src:
            keys, ur, octv, base = self._kf_arrays()
            g = base[np.asarray(ob_kf, np.int64)] + np.asarray(ob_kp, np.int64)
            po["kf"] = np.fromiter((kidx[i] for i in ob_kf), np.int32, len(ob_kf))
            po["u"], po["v"], po["ur"] = keys[g, 0], keys[g, 1], ur[g]
            po["inv_sigma2"] = self.inv_sigma2[octv[g]]
        Q = np.zeros(len(planes), L.LBA_PLANE_DTYPE)
        QO = []
        for n, r in enumerate(planes):
            Q[n]["world"] = self.planes[r]["world"]
            Q[n]["id"] = self.planes[r]["id"]
            Q[n]["obs_offset"] = len(QO)
            for kind, code in ((0, 0), (2, 2), (1, 1)):  # observations, vertical, parallel (kind codes: spslam)
                for i, meas in sorted(self.plane_obs.get(r, {}).get(kind, {}).items()):
                    QO.append((kidx[i], code, meas))
            Q[n]["n_obs"] = len(QO) - Q[n]["obs_offset"]
        qo = np.zeros(len(QO), L.LBA_PLANE_OBS_DTYPE)
        for n, (k, code, meas) in enumerate(QO):
            qo[n]["kf"], qo[n]["kind"], qo[n]["meas"] = k, code, meas
        prob = np.zeros((), L.LBA_PROBLEM_DTYPE)
        prob["n_kf"], prob["n_points"], prob["n_planes"] = len(K), len(P), len(Q)
        prob["n_point_obs"], prob["n_plane_obs"] = len(po), len(qo)
        book = dict(kfs=kfs_order, n_local=len(local), points=points, planes=planes, src=src)
        return (prob, K, P, po, Q, qo), book

    def _kf_arrays(self):
        """Every keyframe's keypoints, mvuRight and octaves concatenated (keyframe id order) and each keyframe's
        first row (indexed by keyframe id)."""
        ids = sorted(self.kfs)
        base = np.zeros(ids[-1] + 1, np.int64)
        o = 0
        for k in ids:
            base[k] = o
            o += len(self.kfs[k]["ur"])
        return (np.concatenate([self.kfs[k]["keys"] for k in ids]), np.concatenate([self.kfs[k]["ur"] for k in ids]),
                np.concatenate([self.kfs[k]["octave"] for k in ids]), base)

    # ---- the result (Optimizer.cc:1909-1977)
    def apply(self, book, kf_out, pt_out, pl_out, point_outlier, stopped):
        """Returns the table rows whose points moved (for the device copy of the table)."""
        if stopped == 1:
            return np.zeros(0, np.int64)
        src = book["src"]
        for b in np.flatnonzero(np.asarray(point_outlier)[:len(src)]):
            pid, i = src[b]  # pKFi->EraseMapPointMatch(pMPi); pMPi->EraseObservation(pKFi)
            kp = self.obs[pid].pop(i)
            self.kfs[i]["mp"].pop(kp, None)
            if self.ref.get(pid) == i and self.obs[pid]:
                self.ref[pid] = min(self.obs[pid])  # MapPoint::EraseObservation: mpRefKF = first observation
        kf_out = np.asarray(kf_out, np.float32).reshape(-1, 16)
        for n in range(book["n_local"]):
            k = book["kfs"][n]
            self.kfs[k]["Tcw"] = kf_out[n].reshape(4, 4).copy()
        points = book["points"]
        rows = np.fromiter((self.row_of[pid] for pid in points), np.int64, len(points))
        self.table["xw"][rows] = np.asarray(pt_out, np.float32).reshape(-1, 3)[:len(points)]
        self.update_normals_and_depths(points, rows)
        pls = np.asarray(pl_out, np.float32).reshape(-1, 4)
        for n, r in enumerate(book["planes"]):
            self.planes[r]["world"] = pls[n]
        return rows

    def update_normals_and_depths(self, pids, rows):
        """update_normal_and_depth for many points at once (same float operations in the same order: the
        normal's terms are added keyframe by keyframe, one observation slot at a time over all points)."""
        ids = sorted(self.kfs)
        C = np.zeros((ids[-1] + 1, 3), np.float32)
        for k in ids:
            C[k] = camera_center(self.kfs[k]["Tcw"])  # (the updated poses)
        keep, start, okf, rkf, rlev = [], [], [], [], []
        for n, pid in enumerate(pids):
            obs = self.obs.get(pid)
            if not obs:
                continue
            ks = sorted(obs)
            keep.append(n)
            start.append(len(okf))
            okf.extend(ks)
            ref = self.ref.get(pid, ks[0])
            if ref not in obs:
                ref = ks[0]
            rkf.append(ref)
            rlev.append(int(self.kfs[ref]["octave"][obs[ref]]))
        if not keep:
            return
        r = np.asarray(rows, np.int64)[np.asarray(keep)]
        start = np.asarray(start, np.int64)
        cnt = np.diff(np.append(start, len(okf)))
        X = self.table["xw"][r].astype(np.float32)
        V = np.repeat(X, cnt, axis=0) - C[np.asarray(okf, np.int64)]
        T = V / norm64(V).astype(np.float32)[:, None]
        normal = np.zeros_like(X)
        for m in range(int(cnt.max())):
            sel = np.flatnonzero(cnt > m)
            normal[sel] = normal[sel] + T[start[sel] + m]
        dist = norm64(X - C[np.asarray(rkf, np.int64)]).astype(np.float32)
        maxd = (dist * self.scale[np.asarray(rlev, np.int64)]).astype(np.float32)
        self.table["max_dist"][r] = maxd
        self.table["min_dist"][r] = (maxd / self.scale[-1]).astype(np.float32)
        self.table["normal"][r] = normal / cnt.astype(np.float32)[:, None]

    def update_normal_and_depth(self, pid, r, centers=None):
        """MapPoint::UpdateNormalAndDepth (MapPoint.cc:357-400) for one point, float arithmetic (the scalar
        statement update_normals_and_depths follows).  centers: the keyframes' camera centres, when the caller
        has them."""
        obs = self.obs.get(pid, {})
        if not obs:
            return
        center = (lambda i: centers[i]) if centers is not None else (lambda i: camera_center(self.kfs[i]["Tcw"]))
        X = self.table[r]["xw"].astype(np.float32)
        normal = np.zeros(3, np.float32)
        for i in sorted(obs):
            v = X - center(i)
            normal = normal + v / np.float32(norm64(v))
        ref = self.ref.get(pid, min(obs))
        if ref not in obs:
            ref = min(obs)
        PC = X - center(ref)
        dist = np.float32(norm64(PC))
        level = int(self.kfs[ref]["octave"][obs[ref]])
        maxd = np.float32(dist * self.scale[level])
        self.table[r]["max_dist"] = maxd
        self.table[r]["min_dist"] = np.float32(maxd / self.scale[-1])
        self.table[r]["normal"] = normal / np.float32(len(obs))

    def local_points(self, t):
        """Frame t's local map: the own points of the two latest keyframes before it (sequence.py)."""
        j = (t - 1) // synth.KEYFRAME_STEP
        a = self.kf_rows[max(j - 1, 0)][0]
        return self.table[a:self.kf_rows[j][1]]

    def refresh_last_frame(self, P):
        """The last frame's map points after the write-back: positions from the table (by id)."""
        P = P.copy()
        r = np.fromiter((self.row_of.get(i, -1) for i in P["id"].tolist()), np.int64, len(P))
        k = np.flatnonzero(r >= 0)
        P["xw"][k] = self.table["xw"][r[k]]
        return P


def insert_initial_keyframe(m, Tcw, kps, depth_u16, depth_factor, bf):
    """StereoInitialization's keyframe 0 (Tracking.cc:529-595): the frame's pose, every keypoint with depth
    mapping its own point; mvuRight from the depth (Frame::ComputeStereoFromRGBD, Frame.cc:743-764, on
    GrabImageRGBD's float depth)."""
    z = np.asarray(depth_u16)[kps["y"].astype(np.int64), kps["x"].astype(np.int64)].astype(np.float32) * \
        (np.float32(1.0) / np.float32(depth_factor))
    with np.errstate(divide="ignore"):
        ur = np.where(z > 0, kps["x"] - np.float32(bf) / z, np.float32(-1)).astype(np.float32)
    m.insert_keyframe(0, Tcw, np.stack([kps["x"], kps["y"]], 1), ur, kps["octave"], {}, [])


def frame_keyframe_inputs(P_next, keys_un, uright, n_kp, pls, plout):
    """A tracked frame's keyframe data: its final matches (the next frame's last-frame points: keypoint index ->
    map point id), keypoints, mvuRight, octaves, and its final PoseOptimization's inlier plane edges."""
    matched = dict(zip(P_next["last_index"].tolist(), P_next["id"].tolist()))
    k = np.asarray(keys_un)[:n_kp]
    octave = k["octave"] if k.dtype.names else np.asarray(k[:, 5]).view(np.int32)
    keys = np.stack([k["x"], k["y"]], 1) if k.dtype.names else np.asarray(k[:, :2], np.float32)
    edges = [(int(e["kind"]), int(e["map_plane_id"]), e["meas"]) for e, o in zip(pls, plout) if not o]
    return matched, keys, np.asarray(uright, np.float32)[:n_kp], octave, edges


__all__ = ["SeqMap", "frame_keyframe_inputs", "camera_center", "SM"]
