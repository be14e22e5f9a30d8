"""Synthetic RGB-D sequences for parity tests and the throughput bench.

The reference datasets (TUM fr1/fr3, ICL-NUIM) are not available in the build
container or on the GPU box, so every test/bench input is generated here
("Synthetic inputs"):

* a textured room (6 planes) plus axis-aligned boxes on the floor (each box
  face is an extra plane; the C5-style dense scene uses >= 10 visible planes),
* random-block texture on every face, blurred (sigma 1.5 texels) and stretched
  to [10, 245] so FAST finds corners at iniThFAST = 20,
* a smooth camera trajectory (about 0.3 m/s, 15 deg/s at 30 Hz),
* depth as u16 = round(z * 5000) with N(0, 1 mm) noise and 2 % dropout to 0,
* TUM3 intrinsics (zero distortion) by default.

Everything is a pure function of (seq_id, frame index) through
numpy.random.Generator(PCG64(0x5EED0000 + seq_id)).
"""
from __future__ import annotations

import dataclasses

import numpy as np

TUM3 = dict(fx=535.4, fy=539.2, cx=320.1, cy=247.6, bf=40.0, depth_factor=5000.0, th_depth=40.0)
# Examples/RGB-D/ICL.yaml (ICL-NUIM): note the negative fy -- the organized cloud's y, the image bounds test and
# every projection flip sign (Frame.cc:864-865, ORBmatcher.cc:1370-1371)
ICL = dict(fx=481.2, fy=-480.0, cx=319.5, cy=239.5, bf=40.0, depth_factor=5000.0, th_depth=40.0)


@dataclasses.dataclass
class Face:
    axis: int          # normal axis 0/1/2 (world)
    offset: float      # plane: X[axis] = offset
    lo: np.ndarray     # bounds on the two other axes (in axis order)
    hi: np.ndarray
    tex: int           # texture index


def _jolts(rng: np.random.Generator, n_frames: int = 4096, gap=(18, 34), hold=(3, 7), deg=(9.0, 14.0)):
    """Hand-held jolts of the "shaky" motion: (first frame, frame it ends, camera-frame axis-angle) -- a turn of
    `deg` degrees about a random axis near the image plane's axes (yaw / pitch), held for `hold` frames, one
    every `gap` frames."""
    out, k = [], int(rng.integers(*gap))
    while k < n_frames:
        h = int(rng.integers(*hold))
        ax = np.array([rng.normal(0, 1), rng.normal(0, 1), rng.normal(0, 0.2)])
        ax /= np.linalg.norm(ax)
        out.append((k, k + h, ax * np.deg2rad(rng.uniform(*deg))))
        k += h + int(rng.integers(*gap))
    return out


def _texture(rng: np.random.Generator, size: int = 1024) -> np.ndarray:
    cells = rng.integers(0, 256, size=(size // 8, size // 8)).astype(np.float32)
    img = np.kron(cells, np.ones((8, 8), np.float32))
    # random dots
    n = size * size // 200
    ys, xs = rng.integers(2, size - 2, n), rng.integers(2, size - 2, n)
    vals = rng.integers(0, 256, n).astype(np.float32)
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            img[ys + dy, xs + dx] = vals
    # separable gaussian blur sigma 1.5 texels
    r = np.arange(-4, 5, dtype=np.float32)
    k = np.exp(-r * r / (2 * 1.5 ** 2)); k /= k.sum()
    pad = np.pad(img, 4, mode="wrap")
    tmp = sum(k[i] * pad[:, i:i + size] for i in range(9))
    img = sum(k[i] * tmp[i:i + size, :] for i in range(9))
    lo, hi = np.percentile(img, 0.5), np.percentile(img, 99.5)
    return np.clip(10 + (img - lo) * (235.0 / max(hi - lo, 1e-3)), 10, 245).astype(np.float32)


def _wrap_blur(img: np.ndarray, sigma: float) -> np.ndarray:
    """Periodic Gaussian blur (FFT; the textures tile the faces)."""
    n = img.shape[0]
    f = np.fft.fftfreq(n)
    g = np.exp(-2.0 * (np.pi * sigma) ** 2 * f * f)
    return np.real(np.fft.ifft2(np.fft.fft2(img) * np.outer(g, g))).astype(np.float32)


def _texture_low(rng: np.random.Generator, size: int = 1024, amp: float = 4.0, spots: int = 25) -> np.ndarray:
    """A nearly untextured face (the C1 proxy, TUM fr3 structure_notexture_far): a flat albedo in [70, 190], a
    smooth +-`amp` gray-level shading (blocks of 32 texels blurred with sigma 10 texels: no FAST corner at
    minThFAST = 7 on its own) and `spots` faint stains (Gaussian blobs of 2-4 texels, contrast 10-30), so the
    ORB features come from the structure's edges and corners plus a few stains and the per-cell FAST retry at
    minThFAST (ORBextractor.cc:812-816) decides most cells."""
    base = rng.uniform(70, 190)
    cells = rng.normal(0, 1, (size // 32, size // 32)).astype(np.float32)
    img = _wrap_blur(np.kron(cells, np.ones((32, 32), np.float32)), 10.0)
    img *= amp / max(float(img.std()), 1e-6)
    for _ in range(spots):
        cy, cx = rng.uniform(0, size, 2)
        r = rng.uniform(2.0, 4.0)
        c = rng.uniform(10, 30) * rng.choice([-1, 1])
        R = int(np.ceil(4 * r))
        iy, ix = np.arange(int(cy) - R, int(cy) + R + 2), np.arange(int(cx) - R, int(cx) + R + 2)
        d2 = (iy - cy)[:, None] ** 2 + (ix - cx)[None, :] ** 2
        img[np.ix_(iy % size, ix % size)] += (c * np.exp(-d2 / (2 * r * r))).astype(np.float32)
    return np.clip(base + img, 5, 250).astype(np.float32)


class Scene:
    """Room 5 x 2.6 x 4 m (x right, y down, z forward) plus boxes on the floor.

    texture: "dots" (random-block texture: the C2-C5 scenes) or "low" (nearly untextured faces, _texture_low:
    the C1 proxy); the geometry is the same for one seq_id either way.
    motion: "smooth" (the C2-C5 trajectory) or "shaky" (the same trajectory with hand-held jolts, _jolts: the
    camera turns by a few degrees from one frame to the next and back a few frames later -- the abrupt velocity
    changes under which TrackWithMotionModel fails and TrackReferenceKeyFrame takes over, Tracking.cc:318-324)."""

    def __init__(self, seq_id: int = 0, n_boxes: int = 3, texel: float = 0.006, texture: str = "dots",
                 motion: str = "smooth"):
        self.rng = np.random.Generator(np.random.PCG64(0x5EED0000 + seq_id))
        self.texel = texel
        if texture not in ("dots", "low"):
            raise ValueError(f"texture {texture!r}")
        if motion not in ("smooth", "shaky"):
            raise ValueError(f"motion {motion!r}")
        self.texture, self.motion = texture, motion
        # jolts from their own generator: the scene (geometry, textures) does not depend on the motion
        self.jolts = _jolts(np.random.Generator(np.random.PCG64(0x10175000 + seq_id))) if motion == "shaky" else []
        X0, X1, Y0, Y1, Z0, Z1 = -2.5, 2.5, -1.3, 1.3, -2.0, 3.5
        faces = [
            Face(0, X0, np.array([Y0, Z0]), np.array([Y1, Z1]), 0),
            Face(0, X1, np.array([Y0, Z0]), np.array([Y1, Z1]), 1),
            Face(1, Y0, np.array([X0, Z0]), np.array([X1, Z1]), 2),
            Face(1, Y1, np.array([X0, Z0]), np.array([X1, Z1]), 3),
            Face(2, Z0, np.array([X0, Y0]), np.array([X1, Y1]), 4),
            Face(2, Z1, np.array([X0, Y0]), np.array([X1, Y1]), 5),
        ]
        ntex = 6
        for b in range(n_boxes):
            sx, sy, sz = self.rng.uniform(0.4, 0.9), self.rng.uniform(0.4, 1.0), self.rng.uniform(0.4, 0.9)
            cx = self.rng.uniform(-1.8, 1.8)
            cz = self.rng.uniform(0.6, 2.6)
            lo = np.array([cx - sx / 2, Y1 - sy, cz - sz / 2])
            hi = np.array([cx + sx / 2, Y1, cz + sz / 2])
            for axis in range(3):
                o = [a for a in range(3) if a != axis]
                for off in (lo[axis], hi[axis]):
                    faces.append(Face(axis, float(off), lo[o].copy(), hi[o].copy(), ntex))
                    ntex += 1
        self.faces = faces
        make = _texture if texture == "dots" else _texture_low
        self.textures = [make(self.rng) for _ in range(ntex)]

    def pose(self, i: int) -> np.ndarray:
        """Camera-to-world 4x4 at frame i (30 Hz)."""
        T = self._smooth_pose(i)
        for k0, k1, rv in self.jolts:
            if k0 <= i < k1:  # the camera turned by rv (axis-angle, camera frame) at k0 and back at k1
                T[:3, :3] = T[:3, :3] @ _rot(rv)
        return T

    def _smooth_pose(self, i: int) -> np.ndarray:
        t = i / 30.0
        yaw = 0.26 * np.sin(0.5 * t)
        pitch = -0.32 + 0.08 * np.sin(0.7 * t + 0.3)  # looking down at the floor and boxes
        roll = 0.05 * np.sin(0.9 * t + 1.0)
        cy, sy = np.cos(yaw), np.sin(yaw)
        cp, sp = np.cos(pitch), np.sin(pitch)
        cr, sr = np.cos(roll), np.sin(roll)
        Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
        Rx = np.array([[1, 0, 0], [0, cp, -sp], [0, sp, cp]])
        Rz = np.array([[cr, -sr, 0], [sr, cr, 0], [0, 0, 1]])
        T = np.eye(4)
        T[:3, :3] = Ry @ Rx @ Rz
        T[:3, 3] = [0.4 * np.sin(0.3 * t), -0.3 + 0.1 * np.sin(0.5 * t), -1.2 + 0.3 * np.sin(0.2 * t)]
        return T

    def render(self, Twc: np.ndarray, w: int = 640, h: int = 480, K=TUM3, noise_seed: int = 0,
               depth_noise: float = 0.0012, dropout: float = 0.0005, gray_noise: float = 1.0,
               holes: int = 12):
        """Returns (gray u8 HxW, depth u16 HxW, plane id int16 HxW).

        Depth noise is Kinect-like, N(0, depth_noise * z^2); invalid depth (0)
        appears as salt (`dropout`), at occlusion edges, and in `holes` random
        blobs of 2-8 px radius."""
        fx, fy, cx, cy = K["fx"], K["fy"], K["cx"], K["cy"]
        if w != 640:  # scaled intrinsics for other resolutions
            s = w / 640.0
            fx, fy, cx, cy = fx * s, fy * s, cx * s, cy * s
        u, v = np.meshgrid(np.arange(w, dtype=np.float64), np.arange(h, dtype=np.float64))
        dc = np.stack([(u - cx) / fx, (v - cy) / fy, np.ones_like(u)], -1)
        R, o = Twc[:3, :3], Twc[:3, 3]
        dw = dc @ R.T
        best = np.full((h, w), np.inf)
        fid = np.full((h, w), -1, np.int32)
        for k, f in enumerate(self.faces):
            den = dw[..., f.axis]
            with np.errstate(divide="ignore", invalid="ignore"):
                t = (f.offset - o[f.axis]) / den
            ok = (t > 1e-6) & (t < best)
            oth = [a for a in range(3) if a != f.axis]
            for j, a in enumerate(oth):
                pa = o[a] + t * dw[..., a]
                ok &= (pa >= f.lo[j] - 1e-9) & (pa <= f.hi[j] + 1e-9)
            best = np.where(ok, t, best)
            fid = np.where(ok, k, fid)
        z = np.where(np.isfinite(best), best, 0.0)  # dc has unit z, so t == camera depth
        P = o + dw * z[..., None]
        gray = np.zeros((h, w), np.float32)
        for k, f in enumerate(self.faces):
            m = fid == k
            if not m.any():
                continue
            oth = [a for a in range(3) if a != f.axis]
            tu = P[..., oth[0]][m] / self.texel + 300.0
            tv = P[..., oth[1]][m] / self.texel + 300.0
            tex = self.textures[f.tex]
            n = tex.shape[0]
            iu, iv = np.floor(tu), np.floor(tv)
            au, av = (tu - iu).astype(np.float32), (tv - iv).astype(np.float32)
            iu = iu.astype(np.int64) % n
            iv = iv.astype(np.int64) % n
            iu1, iv1 = (iu + 1) % n, (iv + 1) % n
            val = ((1 - au) * (1 - av) * tex[iv, iu] + au * (1 - av) * tex[iv, iu1]
                   + (1 - au) * av * tex[iv1, iu] + au * av * tex[iv1, iu1])
            gray[m] = val
        nrng = np.random.Generator(np.random.PCG64(0x5EED0000 + 7919 * (noise_seed + 1)))
        gray = np.clip(np.rint(gray + nrng.normal(0, gray_noise, gray.shape)), 0, 255).astype(np.uint8)
        zn = z + nrng.normal(0, 1.0, z.shape) * depth_noise * z * z
        depth = np.clip(np.rint(zn * K["depth_factor"]), 0, 65535).astype(np.uint16)
        depth[nrng.random(z.shape) < dropout] = 0
        # occlusion-edge shadows (1 px band where depth jumps by > 10 cm)
        jump = np.zeros(z.shape, bool)
        jump[:, 1:] |= np.abs(np.diff(z, axis=1)) > 0.1
        jump[1:, :] |= np.abs(np.diff(z, axis=0)) > 0.1
        depth[jump & (nrng.random(z.shape) < 0.7)] = 0
        yy, xx = np.mgrid[0:h, 0:w]
        for _ in range(holes):
            r = nrng.uniform(2, 8)
            hy, hx = nrng.uniform(0, h), nrng.uniform(0, w)
            depth[(yy - hy) ** 2 + (xx - hx) ** 2 < r * r] = 0
        depth[fid < 0] = 0
        return gray, depth, fid.astype(np.int16)


def sequence(seq_id: int, n_frames: int, w: int = 640, h: int = 480, n_boxes: int = 3, texture: str = "dots",
             motion: str = "smooth"):
    """Yields (Twc, gray, depth_u16) for n_frames frames of sequence seq_id."""
    sc = Scene(seq_id, n_boxes=n_boxes, texture=texture, motion=motion)
    for i in range(n_frames):
        T = sc.pose(i)
        g, d, _ = sc.render(T, w, h, noise_seed=seq_id * 100003 + i)
        yield T, g, d


# ---------------------------------------------------------------------------
# PoseOptimization problems.  In the reference, the inputs of
# Optimizer::PoseOptimization come from ORBmatcher::SearchByProjection and
# Map::AssociatePlanesByBoundary (both outside this hot path).
# Here they are synthesized from the scene ground truth: each ORB keypoint of
# the frame gets a map point (its back-projection with the true depth, 5 mm
# noise, a fraction replaced by gross outliers), each visible face gets a
# plane edge, and some faces a parallel / perpendicular edge to another face.

def face_plane(face: Face) -> np.ndarray:
    """World plane (a, b, c, d) of a face with the reference's d >= 0 sign."""
    n = np.zeros(3)
    n[face.axis] = 1.0
    p = np.array([*n, -face.offset])
    return -p if p[3] < 0 else p


def transform_plane(Tcw: np.ndarray, p: np.ndarray) -> np.ndarray:
    R, t = Tcw[:3, :3], Tcw[:3, 3]
    n = R @ p[:3]
    out = np.array([*n, p[3] - t @ n])
    return -out if out[3] < 0 else out


def _rot(axis_angle):
    th = np.linalg.norm(axis_angle)
    if th < 1e-12:
        return np.eye(3)
    k = axis_angle / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def pose_problem(scene: Scene, frame: int, kps, depth_u16, fid, inv_level_sigma2, rng, K=TUM3,
                 match_frac=0.8, outlier_frac=0.08, rot_noise_deg=1.0, trans_noise=0.03,
                 with_planes=True, min_face_px=4000):
    """Returns (problem record, point obs, plane obs, Tcw_gt) with the dtypes of spslam_gpu."""
    import spslam_gpu as G
    Twc = scene.pose(frame)
    Tcw = np.linalg.inv(Twc)
    fx, fy, cx, cy, bf = K["fx"], K["fy"], K["cx"], K["cy"], K["bf"]
    h, w = depth_u16.shape
    if w != 640:
        s = w / 640.0
        fx, fy, cx, cy = fx * s, fy * s, cx * s, cy * s
    pts = []
    for i, kp in enumerate(kps):
        if rng.random() > match_frac:
            continue
        u, v = float(kp["x"]), float(kp["y"])
        d = depth_u16[int(v), int(u)] / K["depth_factor"]
        ur = u - bf / d if d > 0 else -1.0
        # true depth along the ray from the noise-free scene
        ray = np.array([(u - cx) / fx, (v - cy) / fy, 1.0])
        zt = d if d > 0 else 2.0
        Xc = ray * (zt + rng.normal(0, 0.005))
        Xw = Twc[:3, :3] @ Xc + Twc[:3, 3]
        if rng.random() < outlier_frac:
            Xw = Xw + rng.normal(0, 0.3, 3)
        pts.append((u, v, ur, inv_level_sigma2[int(kp["octave"])], Xw.astype(np.float32), i))
    points = np.array(pts, G.POINT_OBS_DTYPE) if pts else np.zeros(0, G.POINT_OBS_DTYPE)
    planes = []
    if with_planes:
        counts = np.bincount(fid[fid >= 0].ravel(), minlength=len(scene.faces))
        vis = [k for k in range(len(scene.faces)) if counts[k] >= min_face_px]
        edges = {0: [], 1: [], 2: []}
        for j, k in enumerate(vis):
            wp = face_plane(scene.faces[k])
            cp = transform_plane(Tcw, wp)
            Rn = _rot(rng.normal(0, np.deg2rad(0.3), 3))
            meas = np.array([*(Rn @ cp[:3]), cp[3] + rng.normal(0, 0.005)])
            edges[0].append((meas, wp, j, k))
            par = [m for m in range(len(scene.faces)) if m != k and scene.faces[m].axis == scene.faces[k].axis]
            ver = [m for m in range(len(scene.faces)) if scene.faces[m].axis != scene.faces[k].axis]
            if par and rng.random() < 0.5:
                m = par[rng.integers(len(par))]
                edges[1].append((meas, face_plane(scene.faces[m]), j, m))
            if ver and rng.random() < 0.5:
                m = ver[rng.integers(len(ver))]
                edges[2].append((meas, face_plane(scene.faces[m]), j, m))
        for kind in (0, 1, 2):
            for meas, wp, j, mid in edges[kind]:
                planes.append((meas.astype(np.float32), wp.astype(np.float32), kind, j, mid, 0))
    planes = np.array(planes, G.PLANE_OBS_DTYPE) if planes else np.zeros(0, G.PLANE_OBS_DTYPE)
    # motion-model initial guess: perturbed ground truth
    T0 = Tcw.copy()
    T0[:3, :3] = _rot(rng.normal(0, np.deg2rad(rot_noise_deg), 3)) @ Tcw[:3, :3]
    T0[:3, 3] = Tcw[:3, 3] + rng.normal(0, trans_noise, 3)
    prob = np.zeros((), G.POSE_PROBLEM_DTYPE)
    prob["Tcw"] = T0.astype(np.float32).ravel()
    prob["fx"], prob["fy"], prob["cx"], prob["cy"], prob["bf"] = fx, fy, cx, cy, bf
    prob["n_points"], prob["n_planes"] = len(points), len(planes)
    return prob, points, planes, Tcw


def lba_problem(scene: Scene, kf_frames, rng, n_fixed=2, n_points=1500, K=TUM3, stereo_frac=0.9,
                outlier_frac=0.04, pix_noise=1.0, pose_rot_deg=0.4, pose_trans=0.02, point_noise=0.02,
                plane_noise_deg=0.5, plane_noise_d=0.01, first_kf_id=1, with_planes=True):
    """A LocalBundleAdjustment graph over keyframes at `kf_frames` (the first
    len - n_fixed are local, the rest fixed cameras): map points sampled on the
    scene faces, observed by every keyframe that sees them in the image,
    room / box planes with observation, parallel and vertical edges.  Returns
    (problem, keyframes, points, point_obs, planes, plane_obs, ground truth)
    in the record types of spslam_lba."""
    import spslam_lba as L
    fx, fy, cx, cy, bf = K["fx"], K["fy"], K["cx"], K["cy"], K["bf"]
    n_kf = len(kf_frames)
    Tcw_gt = [np.linalg.inv(scene.pose(f)) for f in kf_frames]
    kfs = np.zeros(n_kf, L.LBA_KEYFRAME_DTYPE)
    for k, f in enumerate(kf_frames):
        T = Tcw_gt[k].copy()
        fixed = k >= n_kf - n_fixed
        if not fixed:
            T[:3, :3] = _rot(rng.normal(0, np.deg2rad(pose_rot_deg), 3)) @ T[:3, :3]
            T[:3, 3] = T[:3, 3] + rng.normal(0, pose_trans, 3)
        kfs[k]["Tcw"] = T.astype(np.float32).ravel()
        kfs[k]["fx"], kfs[k]["fy"], kfs[k]["cx"], kfs[k]["cy"], kfs[k]["bf"] = fx, fy, cx, cy, bf
        kfs[k]["id"] = first_kf_id + k
        kfs[k]["fixed"] = int(fixed)
    inv_s2 = [1.0 / (1.2 ** (2 * o)) for o in range(8)]
    # map points on faces in front of the cameras
    pts, obs = [], []
    faces = scene.faces
    tries = 0
    while len(pts) < n_points and tries < 50 * n_points:
        tries += 1
        face = faces[rng.integers(len(faces))]
        o = [a for a in range(3) if a != face.axis]
        X = np.zeros(3)
        X[face.axis] = face.offset
        X[o] = rng.uniform(face.lo, face.hi)
        seen = []
        for k in range(n_kf):
            Xc = Tcw_gt[k][:3, :3] @ X + Tcw_gt[k][:3, 3]
            if Xc[2] < 0.3:
                continue
            u, v = fx * Xc[0] / Xc[2] + cx, fy * Xc[1] / Xc[2] + cy
            if 10 <= u < 630 and 10 <= v < 470 and rng.random() < 0.85:
                seen.append((k, u, v, Xc[2]))
        if len(seen) < 2:
            continue
        pid = len(pts)
        off = len(obs)
        for k, u, v, z in seen:
            oc = int(rng.integers(8))
            if rng.random() < outlier_frac:
                u, v = rng.uniform(10, 630), rng.uniform(10, 470)
            else:
                u, v = u + rng.normal(0, pix_noise), v + rng.normal(0, pix_noise)
            ur = u - bf / (z + rng.normal(0, 0.002 * z * z)) if rng.random() < stereo_frac else -1.0
            obs.append((k, u, v, ur, inv_s2[oc]))
        Xn = X + rng.normal(0, point_noise, 3)
        pts.append((Xn.astype(np.float32), 1000 + 3 * pid, off, len(seen)))
    points = np.array(pts, L.LBA_POINT_DTYPE)
    point_obs = np.array(obs, L.LBA_POINT_OBS_DTYPE)
    # planes: faces seen (plane passing in front) by at least two keyframes
    planes, pobs = [], []
    if with_planes:
        room = list(range(min(6, len(faces)))) + list(range(6, len(faces)))[:4]
        vis = {}
        for j in room:
            wp = face_plane(faces[j])
            ks = [k for k in range(n_kf) if transform_plane(Tcw_gt[k], wp)[3] > 0.3]
            if len(ks) >= 2:
                vis[j] = ks
        for j, ks in vis.items():
            wp = face_plane(faces[j])
            off = len(pobs)
            cnt = 0
            for kind in (0, 2, 1):  # observations, vertical, parallel (Optimizer.cc:1501-1613)
                for k in ks:
                    if kind == 0:
                        m = j
                    else:
                        cand = [q for q in vis if q != j and ((faces[q].axis == faces[j].axis) == (kind == 1))]
                        if not cand or rng.random() < 0.6:
                            continue
                        m = cand[rng.integers(len(cand))]
                    cp = transform_plane(Tcw_gt[k], face_plane(faces[m]))
                    Rn = _rot(rng.normal(0, np.deg2rad(plane_noise_deg), 3))
                    meas = np.array([*(Rn @ cp[:3]), cp[3] + rng.normal(0, plane_noise_d)])
                    pobs.append((k, kind, meas.astype(np.float32)))
                    cnt += 1
            Rn = _rot(rng.normal(0, np.deg2rad(plane_noise_deg), 3))
            wn = np.array([*(Rn @ wp[:3]), wp[3] + rng.normal(0, plane_noise_d)])
            planes.append((wn.astype(np.float32), 7 + j, off, cnt, 0))
    planes = np.array(planes, L.LBA_PLANE_DTYPE) if planes else np.zeros(0, L.LBA_PLANE_DTYPE)
    plane_obs = np.array(pobs, L.LBA_PLANE_OBS_DTYPE) if pobs else np.zeros(0, L.LBA_PLANE_OBS_DTYPE)
    prob = np.zeros((), L.LBA_PROBLEM_DTYPE)
    prob["n_kf"], prob["n_points"], prob["n_planes"] = n_kf, len(points), len(planes)
    prob["n_point_obs"], prob["n_plane_obs"] = len(point_obs), len(plane_obs)
    return prob, kfs, points, point_obs, planes, plane_obs, dict(Tcw=np.array(Tcw_gt))


# ---------------------------------------------------------------- plane association
def map_planes(scene: Scene, rng, boundary_step=0.02, boundary_noise=0.005, coef_noise_deg=0.5,
               coef_noise_d=0.01, max_faces=None):
    """Map planes (MapPlane world coefficients + mvBoundaryPoints) for the scene's
    faces, in id order: the boundary cloud samples the face rectangle's border
    every `boundary_step` metres with Gaussian noise.  Returns (records in the
    spslam_map_plane layout as a dict of arrays, boundary xyz float32)."""
    faces = scene.faces if max_faces is None else scene.faces[:max_faces]
    world, offs, counts, pts = [], [], [], []
    n = 0
    for face in faces:
        p = face_plane(face)
        ax = rng.normal(size=3)
        ax *= np.deg2rad(coef_noise_deg) * rng.uniform() / max(np.linalg.norm(ax), 1e-12)
        nrm = _rot(ax) @ p[:3]
        world.append([*nrm, p[3] + rng.normal() * coef_noise_d])
        o = [a for a in range(3) if a != face.axis]
        (u0, v0), (u1, v1) = face.lo, face.hi
        nu, nv = max(int((u1 - u0) / boundary_step), 1), max(int((v1 - v0) / boundary_step), 1)
        us, vs = np.linspace(u0, u1, nu + 1), np.linspace(v0, v1, nv + 1)
        border = np.concatenate([np.stack([us, np.full_like(us, v0)], 1), np.stack([us, np.full_like(us, v1)], 1),
                                 np.stack([np.full_like(vs, u0), vs], 1), np.stack([np.full_like(vs, u1), vs], 1)])
        xyz = np.zeros((len(border), 3))
        xyz[:, face.axis] = face.offset
        xyz[:, o[0]], xyz[:, o[1]] = border[:, 0], border[:, 1]
        xyz += rng.normal(size=xyz.shape) * boundary_noise
        offs.append(n)
        counts.append(len(xyz))
        pts.append(xyz)
        n += len(xyz)
    return (dict(world=np.array(world, np.float32), boundary_offset=np.array(offs, np.int32),
                 n_boundary=np.array(counts, np.int32), id=np.arange(1, len(faces) + 1, dtype=np.int32)),
            np.concatenate(pts).astype(np.float32))


def assoc_frame_planes(scene: Scene, frame: int, rng, n_faces=6, n_random=2, far_frac=0.25, noise_deg=1.0,
                       noise_d=0.02):
    """A frame's mvPlaneCoefficients for AssociatePlanesByBoundary: camera-frame
    coefficients of `n_faces` scene faces (noisy; a fraction shifted 0.3-1 m so
    they only qualify as parallel), plus random planes.  Returns (Tcw float32,
    coefs float32 (n, 4) with d >= 0, source face index or -1)."""
    Tcw = np.linalg.inv(scene.pose(frame))
    idx = rng.choice(len(scene.faces), size=min(n_faces, len(scene.faces)), replace=False)
    coefs, src = [], []
    for f in idx:
        p = face_plane(scene.faces[f]).copy()
        if rng.uniform() < far_frac:
            p[3] += rng.choice([-1, 1]) * rng.uniform(0.3, 1.0)
        ax = rng.normal(size=3)
        ax *= np.deg2rad(noise_deg) * rng.uniform() / max(np.linalg.norm(ax), 1e-12)
        q = np.array([*(_rot(ax) @ p[:3]), p[3] + rng.normal() * noise_d])
        coefs.append(transform_plane(Tcw, q))
        src.append(int(f))
    for _ in range(n_random):
        n = rng.normal(size=3)
        n /= np.linalg.norm(n)
        coefs.append(np.array([*n, rng.uniform(0.2, 3.0)]))
        src.append(-1)
    return Tcw.astype(np.float32), np.array(coefs, np.float32).reshape(-1, 4), np.array(src, np.int32)


# ---------------------------------------------------------------- projection matching
def proj_problem(scene: Scene, last_fi: int, cur_fi: int, last_kps, last_desc, last_depth_u16, rng, K=TUM3,
                 map_frac=0.8, flip_bits=6, zero_obs_frac=0.05, rot_noise_deg=0.3, trans_noise=0.01):
    """TrackWithMotionModel inputs: the last frame's map points (its keypoints with
    depth, back-projected with the true pose, descriptors with a few flipped bits,
    a fraction without observations) and the current pose prediction (true pose
    with a small error).  Returns (spslam_proj_frame record, spslam_proj_point
    records)."""
    import spslam_match as M
    fx, fy, cx, cy = K["fx"], K["fy"], K["cx"], K["cy"]
    Twl = scene.pose(last_fi)
    Tcw = np.linalg.inv(scene.pose(cur_fi))
    ax = rng.normal(size=3)
    ax *= np.deg2rad(rot_noise_deg) / max(np.linalg.norm(ax), 1e-12)
    dT = np.eye(4)
    dT[:3, :3] = _rot(ax)
    dT[:3, 3] = rng.normal(size=3) * trans_noise
    Tcw = dT @ Tcw
    pts = []
    for i, kp in enumerate(last_kps):
        if rng.uniform() > map_frac:
            continue
        x, y = int(kp["x"]), int(kp["y"])
        z = float(last_depth_u16[y, x]) / K["depth_factor"]
        if z <= 0:
            continue
        Xc = np.array([(kp["x"] - cx) * z / fx, (kp["y"] - cy) * z / fy, z, 1.0])
        Xw = Twl @ Xc
        d = np.array(last_desc[i], np.uint8).copy()
        bits = np.unpackbits(d)
        flip = rng.choice(256, size=flip_bits, replace=False)
        bits[flip] ^= 1
        pts.append((Xw[:3], float(kp["angle"]), int(kp["octave"]),
                    0 if rng.uniform() < zero_obs_frac else int(rng.integers(1, 6)), i, np.packbits(bits)))
    P = np.zeros(len(pts), M.PROJ_POINT_DTYPE)
    for j, (xw, ang, octv, nobs, i, d) in enumerate(pts):
        P[j]["xw"], P[j]["angle"], P[j]["octave"], P[j]["n_obs"], P[j]["last_index"], P[j]["desc"] = \
            xw, ang, octv, nobs, i, d
    fr = np.zeros((), M.PROJ_FRAME_DTYPE)
    fr["Tcw"] = Tcw.astype(np.float32).reshape(16)
    fr["Tlw"] = np.linalg.inv(Twl).astype(np.float32).reshape(16)
    fr["n_points"] = len(P)
    return fr, P


def local_problem(scene: Scene, kf_fi: int, cur_fi: int, kf_kps, kf_desc, kf_depth_u16, rng, K=TUM3,
                  map_frac=0.9, flip_bits=6, rot_noise_deg=0.2, trans_noise=0.005, scale=1.2, n_levels=8):
    """SearchLocalPoints inputs: local map points built from a nearby keyframe's
    keypoints (true depth), with MapPoint::UpdateNormalAndDepth's normal and
    distance range (mfMaxDistance = dist * 1.2^octave, mfMinDistance =
    mfMaxDistance / 1.2^7), descriptors with flipped bits, and the current pose
    after the motion-model optimisation (true pose, small error).  Returns
    (spslam_local_frame record, spslam_local_point records)."""
    import spslam_match as M
    fx, fy, cx, cy = K["fx"], K["fy"], K["cx"], K["cy"]
    Twk = scene.pose(kf_fi)
    Tcw = np.linalg.inv(scene.pose(cur_fi))
    ax = rng.normal(size=3)
    ax *= np.deg2rad(rot_noise_deg) / max(np.linalg.norm(ax), 1e-12)
    dT = np.eye(4)
    dT[:3, :3] = _rot(ax)
    dT[:3, 3] = rng.normal(size=3) * trans_noise
    Tcw = dT @ Tcw
    sf = np.float32(scale) ** np.arange(n_levels, dtype=np.float32)
    rows = []
    for i, kp in enumerate(kf_kps):
        if rng.uniform() > map_frac:
            continue
        x, y = int(kp["x"]), int(kp["y"])
        z = float(kf_depth_u16[y, x]) / K["depth_factor"]
        if z <= 0:
            continue
        Xw = (Twk @ np.array([(kp["x"] - cx) * z / fx, (kp["y"] - cy) * z / fy, z, 1.0]))[:3]
        PC = Xw - Twk[:3, 3]
        dist = np.linalg.norm(PC)
        maxd = np.float32(dist) * sf[int(kp["octave"])]
        bits = np.unpackbits(np.array(kf_desc[i], np.uint8))
        bits[rng.choice(256, size=flip_bits, replace=False)] ^= 1
        rows.append((Xw, PC / dist, maxd / sf[-1], maxd, i, np.packbits(bits)))
    P = np.zeros(len(rows), M.LOCAL_POINT_DTYPE)
    for j, (xw, nrm, mind, maxd, i, d) in enumerate(rows):
        P[j]["xw"], P[j]["normal"], P[j]["min_dist"], P[j]["max_dist"], P[j]["id"], P[j]["desc"] = \
            xw, nrm, mind, maxd, i, d
    fr = np.zeros((), M.LOCAL_FRAME_DTYPE)
    fr["Tcw"] = Tcw.astype(np.float32).reshape(16)
    fr["n_points"] = len(P)
    return fr, P


# Per-face colour tints (R, G, B gains) for colour frames; the background stays gray.
_TINTS = np.array([[1.00, 0.92, 0.85], [0.85, 0.95, 1.00], [0.95, 1.00, 0.88], [1.00, 0.86, 0.95],
                   [0.90, 0.90, 1.00], [0.97, 0.97, 0.90], [0.88, 1.00, 1.00], [1.00, 0.95, 0.80]], np.float32)


def colorize(gray: np.ndarray, fid: np.ndarray) -> np.ndarray:
    """An interleaved RGB u8 frame (HxWx3, R,G,B order) from a rendered gray frame: each face's texture
    tinted by a per-face gain, so cvtColor's weights matter (TUM frames are colour, rgbd_tum reads them
    with imread and GrabImageRGBD converts them, src/Tracking.cc:214-224)."""
    tint = np.where((fid >= 0)[..., None], _TINTS[np.maximum(fid, 0) % len(_TINTS)], 1.0).astype(np.float32)
    return np.clip(np.rint(gray[..., None].astype(np.float32) * tint), 0, 255).astype(np.uint8)


# ---------------------------------------------------------------- tracked sequences
KEYFRAME_STEP = 10  # fixed keyframe schedule of the sequence harness (sp-slam_amd/sequence.py)


def keyframe_points(scene: Scene, kf_fi: int, kf_kps, kf_desc, kf_depth_u16, id_base: int, K=TUM3, scale=1.2,
                    n_levels=8, th_depth=None):
    """The map points a keyframe contributes (StereoInitialization / CreateNewKeyFrame, src/Tracking.cc:544-560,
    1315-1345: one MapPoint per keypoint with depth, at the keyframe's pose -- here the true pose), with
    MapPoint::UpdateNormalAndDepth's normal and distance range (src/MapPoint.cc:357-400), the keyframe's
    descriptor (one observation: ComputeDistinctiveDescriptors keeps it), Observations() = 1 + id % 3 and ids
    id_base + keypoint index.  Returns spslam_local_point records."""
    import spslam_match as M
    fx, fy, cx, cy = K["fx"], K["fy"], K["cx"], K["cy"]
    Twk = scene.pose(kf_fi)
    sf = np.float32(scale) ** np.arange(n_levels, dtype=np.float32)
    rows = []
    for i, kp in enumerate(kf_kps):
        x, y = int(kp["x"]), int(kp["y"])
        z = float(kf_depth_u16[y, x]) / K["depth_factor"]
        if z <= 0 or (th_depth is not None and z > th_depth):
            continue
        Xw = (Twk @ np.array([(kp["x"] - cx) * z / fx, (kp["y"] - cy) * z / fy, z, 1.0]))[:3]
        PC = Xw - Twk[:3, 3]
        dist = np.linalg.norm(PC)
        maxd = np.float32(dist) * sf[int(kp["octave"])]
        rows.append((Xw, PC / dist, maxd / sf[-1], maxd, id_base + i, np.asarray(kf_desc[i], np.uint8)))
    P = np.zeros(len(rows), M.LOCAL_POINT_DTYPE)
    for j, (xw, nrm, mind, maxd, pid, d) in enumerate(rows):
        P[j]["xw"], P[j]["normal"], P[j]["min_dist"], P[j]["max_dist"], P[j]["id"], P[j]["desc"] = \
            xw, nrm, mind, maxd, pid, d
        P[j]["n_obs"] = 1 + pid % 3
    return P


def as_last_frame_points(points, kps, id_base):
    """A keyframe's own map points as the last frame's (its mvpMapPoints, keypoint i = id - id_base):
    spslam_proj_point records in keypoint order with the keypoint's angle and octave."""
    import spslam_match as M
    P = np.zeros(len(points), M.PROJ_POINT_DTYPE)
    for j, p in enumerate(points):
        i = int(p["id"]) - id_base
        P[j]["xw"], P[j]["angle"], P[j]["octave"] = p["xw"], kps[i]["angle"], kps[i]["octave"]
        P[j]["n_obs"], P[j]["last_index"], P[j]["id"], P[j]["desc"] = p["n_obs"], i, p["id"], p["desc"]
    return P


def render_sequence_frames(seq_id, n_frames, w, h, K, n_boxes, first=0, texture="dots", motion="smooth"):
    """(colour RGB u8, depth u16) of frames first .. first + n_frames - 1 of a sequence (worker-pool friendly)."""
    sc = Scene(seq_id, n_boxes=n_boxes, texture=texture, motion=motion)
    out = []
    for t in range(first, first + n_frames):
        g, d, fid = sc.render(sc.pose(t), w, h, K=K, noise_seed=seq_id * 100003 + t)
        out.append((colorize(g, fid), d))
    return out


def shape_vocabulary_text(k=10, L=6, seed=0x0B0C):
    """A complete DBoW2 text vocabulary of ORBvoc.txt's shape (k = 10, L = 6: 1,111,111 nodes, 10^6 words),
    built in memory (the trained ORBvoc.txt is not vendored, .MISSING_LARGE_BLOBS:2, and a k-means tree of
    that size is not trainable here).  Level-1 nodes are random 256-bit descriptors; each child is its parent
    with a few random bits flipped (fewer at deeper levels), so a feature and its re-observation tend to
    descend alike, as in a trained tree.  The vocabulary of the tracked sequences' TrackReferenceKeyFrame
    (sp-slam_amd/sequence.py) and of the ORBvoc-shape BoW tests.  Leaves carry TF-IDF-like weights in
    [0.5, 5.5); nodes are listed level by level (parents precede children, which loadFromTextFile needs).
    Whitespace-aligned fields: the same text any istream-based loader reads."""
    rng = np.random.default_rng(seed)
    levels = [rng.integers(0, 256, (k, 32), dtype=np.uint8)]
    flips = {2: 24, 3: 12, 4: 6, 5: 3, 6: 2, 7: 1, 8: 1}
    for lv in range(2, L + 1):
        par = np.repeat(levels[-1], k, axis=0)
        bits = np.zeros((len(par), 256), np.uint8)
        pos = rng.integers(0, 256, (len(par), flips.get(lv, 1)))
        np.put_along_axis(bits, pos, 1, axis=1)
        levels.append(par ^ np.packbits(bits, axis=1))
    desc = np.concatenate(levels)
    n = len(desc)
    first = np.cumsum([1] + [k ** l for l in range(1, L + 1)])  # id of each level's first node
    ids = np.arange(1, n + 1)
    lvl = np.searchsorted(first, ids, side="right")              # 1..L
    parent = np.where(lvl == 1, 0, first[lvl - 2] + (ids - first[lvl - 1]) // k)
    leaf = (lvl == L).astype(np.int64)
    weight = np.where(leaf == 1, rng.integers(500000, 5500000, n), 0)  # micro-units

    def digits(v, width):  # right-aligned decimal, space padded, as a (len(v), width) byte matrix
        out = np.full((len(v), width), ord(" "), np.uint8)
        v = v.copy()
        for c in range(width - 1, -1, -1):
            nz = (v > 0) | (c == width - 1)
            out[nz, c] = ord("0") + v[nz] % 10
            v //= 10
        return out
    lut = np.array([digits(np.array([b]), 3)[0].tolist() + [ord(" ")] for b in range(256)], np.uint8)
    sp = np.full((n, 1), ord(" "), np.uint8)
    w_int, w_frac = weight // 1000000, weight % 1000000
    frac = digits(w_frac + 1000000, 7)[:, 1:]                    # 6 zero-padded fraction digits
    body = np.concatenate([digits(parent, 7), sp, digits(leaf, 1), sp, lut[desc].reshape(n, 128),
                           digits(w_int, 1), np.full((n, 1), ord("."), np.uint8), frac,
                           np.full((n, 1), ord("\n"), np.uint8)], axis=1)
    return f"{k} {L}  0 0\n".encode() + body.tobytes()
