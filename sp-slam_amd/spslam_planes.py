"""ctypes binding of the plane-extraction part of include/spslam_gpu.h
(Frame::ComputePlanesFromOrganizedPointCloud on gfx950)."""
from __future__ import annotations

import ctypes

import numpy as np

import spslam_gpu

PLANE_DTYPE = np.dtype([("coef", "<f4", 4), ("n_inliers", "<i4"), ("inlier_offset", "<i4"), ("n_contour", "<i4"),
                        ("contour_offset", "<i4")])
assert PLANE_DTYPE.itemsize == 32


class PlaneParams(ctypes.Structure):
    _fields_ = [("cloud_dis", ctypes.c_int), ("min_size", ctypes.c_int), ("angle_threshold", ctypes.c_float),
                ("distance_threshold", ctypes.c_float), ("fx", ctypes.c_float), ("fy", ctypes.c_float),
                ("cx", ctypes.c_float), ("cy", ctypes.c_float), ("width", ctypes.c_int), ("height", ctypes.c_int),
                ("line_ratio", ctypes.c_double), ("line_distance_threshold", ctypes.c_float),
                ("image_bounds", ctypes.c_float * 4)]


SUPPOSED_DTYPE = np.dtype([("coef", "<f4", 4), ("line", "<f4", 6), ("source_plane", "<i4"), ("n_line", "<i4"),
                           ("line_offset", "<i4"), ("n_patch", "<i4"), ("patch_offset", "<i4"), ("pad", "<i4")])
assert SUPPOSED_DTYPE.itemsize == 64
LINE_CAND_DTYPE = np.dtype([("line", "<f4", 6), ("n_inliers", "<i4"), ("iterations", "<i4"), ("flags", "<i4"),
                            ("idx_offset", "<i4")])


spslam_gpu.EXPORTED += ["spslam_planes_configure", "spslam_planes_capacity", "spslam_planes_extract",
                        "spslam_planes_extract_batch_device", "spslam_planes_debug", "spslam_debug_plane_labels",
                        "spslam_supposed_capacity",
                        "spslam_planes_generate_from_boundaries",
                        "spslam_planes_generate_from_boundaries_batch_device", "spslam_supposed_debug",
                        "spslam_planes_select_cloud_set",
                        "spslam_debug_plane_not_seen"]


def _bind(lib):
    vp, ip = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)
    lib.spslam_planes_configure.argtypes = [vp, ctypes.POINTER(PlaneParams)]
    lib.spslam_planes_capacity.argtypes = [vp, ip, ip, ip]
    lib.spslam_planes_extract.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, ip, vp,
                                          vp]
    lib.spslam_planes_extract_batch_device.argtypes = [vp, vp, ctypes.c_int, ctypes.c_size_t, ctypes.c_int, vp, vp,
                                                       vp, vp, vp]
    lib.spslam_planes_debug.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, ip]
    lib.spslam_supposed_capacity.argtypes = [vp, ip, ip, ip]
    lib.spslam_planes_generate_from_boundaries.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp,
                                                           ctypes.c_int, ip, vp, vp]
    lib.spslam_planes_generate_from_boundaries_batch_device.argtypes = [vp, vp, ctypes.c_int, ctypes.c_size_t,
                                                                        ctypes.c_int, vp, vp, vp, vp, vp, vp, vp, vp]
    lib.spslam_supposed_debug.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, ip, vp, ctypes.c_int]
    lib.spslam_planes_select_cloud_set.argtypes = [vp, ctypes.c_int]
    lib.spslam_debug_plane_not_seen.argtypes = [vp, vp, ctypes.c_int, vp, ctypes.c_int, vp]


def plane_not_seen(ex: spslam_gpu.OrbExtractor, planes, coefs):
    """Frame::PlaneNotSeen (src/Frame.cc:1116-1130) of each candidate against the planes, through the
    device predicate the extraction kernels use (test hook).  Returns a bool per candidate."""
    _bind(ex.lib)
    p = np.ascontiguousarray(planes, np.float32).reshape(-1, 4)
    c = np.ascontiguousarray(coefs, np.float32).reshape(-1, 4)
    out = np.zeros(max(len(c), 1), np.int32)
    ex._check(ex.lib.spslam_debug_plane_not_seen(ex.ctx, p.ctypes.data if len(p) else None, len(p),
                                                 c.ctypes.data if len(c) else None, len(c), out.ctypes.data))
    return out[:len(c)].astype(bool)


class PlaneExtractor:
    """GPU Frame::ComputePlanesFromOrganizedPointCloud on a context (shares its stream/device)."""

    def __init__(self, ex: spslam_gpu.OrbExtractor, fx, fy, cx, cy, width=640, height=480, cloud_dis=3,
                 min_size=500, angle_threshold=3.0, distance_threshold=0.05, line_ratio=0.2,
                 line_distance_threshold=0.01, image_bounds=(0.0, 0.0, 0.0, 0.0)):
        self.ex = ex
        _bind(ex.lib)
        self.params = PlaneParams(cloud_dis, min_size, angle_threshold, distance_threshold, fx, fy, cx, cy, width,
                                  height, line_ratio, line_distance_threshold, (ctypes.c_float * 4)(*image_bounds))
        ex._check(ex.lib.spslam_planes_configure(ex.ctx, ctypes.byref(self.params)))
        pc, ic, cc = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        ex._check(ex.lib.spslam_planes_capacity(ex.ctx, ctypes.byref(pc), ctypes.byref(ic), ctypes.byref(cc)))
        self.planes_cap, self.inlier_cap, self.contour_cap = pc.value, ic.value, cc.value
        self.W = -(-width // cloud_dis)
        self.H = -(-height // cloud_dis)
        self._supp_caps()

    def _supp_caps(self):
        a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self.ex._check(self.ex.lib.spslam_supposed_capacity(self.ex.ctx, ctypes.byref(a), ctypes.byref(b),
                                                            ctypes.byref(c)))
        self.supp_cap, self.line_cap, self.patch_points = a.value, b.value, c.value

    def configure(self, **kw):
        """Change Plane.* parameters (min_size, angle_threshold, distance_threshold, ...) in place."""
        for k, v in kw.items():
            if k == "image_bounds":
                v = (ctypes.c_float * 4)(*v)
            setattr(self.params, k, v)
        self.ex._check(self.ex.lib.spslam_planes_configure(self.ex.ctx, ctypes.byref(self.params)))
        self._supp_caps()

    def __call__(self, depth_f32: np.ndarray):
        """Returns dict(coef=[...], inliers=[...], contour=[...]) like the oracle."""
        d = np.ascontiguousarray(depth_f32, np.float32)
        planes = np.zeros(self.planes_cap, PLANE_DTYPE)
        inl = np.zeros(self.inlier_cap, np.int32)
        con = np.zeros(self.contour_cap, np.int32)
        n = ctypes.c_int()
        self.ex._check(self.ex.lib.spslam_planes_extract(self.ex.ctx, d.ctypes.data, d.shape[1], d.shape[0],
                                                         d.shape[1], planes.ctypes.data, self.planes_cap,
                                                         ctypes.byref(n), inl.ctypes.data, con.ctypes.data))
        out = dict(coef=[], inliers=[], contour=[])
        for p in planes[:n.value]:
            out["coef"].append(p["coef"].copy())
            out["inliers"].append(inl[p["inlier_offset"]:p["inlier_offset"] + p["n_inliers"]].copy())
            out["contour"].append(con[p["contour_offset"]:p["contour_offset"] + p["n_contour"]].copy())
        return out

    def extract_batch_device(self, depth_ptr, n_frames, frame_stride, stride, planes_ptr, counts_ptr, inliers_ptr,
                             contours_ptr, stream=0):
        self.ex._check(self.ex.lib.spslam_planes_extract_batch_device(
            self.ex.ctx, depth_ptr, n_frames, frame_stride, stride, planes_ptr, counts_ptr, inliers_ptr,
            contours_ptr, stream or None))

    def keep_labels(self, on=True):
        """Test hook: store the connected-component labels (debug(frame, 3)) on later extractions."""
        self.ex.lib.spslam_debug_plane_labels.argtypes = [ctypes.c_void_p, ctypes.c_int]
        self.ex._check(self.ex.lib.spslam_debug_plane_labels(self.ex.ctx, int(on)))

    def debug(self, frame, what):
        N = self.W * self.H
        shape, dt = {0: ((N, 3), np.float32), 1: ((N, 3), np.float32), 2: (N, np.float32), 3: (N, np.uint32)}[what]
        out = np.zeros(shape, dt)
        n = ctypes.c_int()
        self.ex._check(self.ex.lib.spslam_planes_debug(self.ex.ctx, frame, what, out.ctypes.data, ctypes.byref(n)))
        return out

    def generate_from_boundaries(self, depth_f32: np.ndarray):
        """Frame::GeneratePlanesFromBoundries on the planes of the last __call__ (same depth).
        Returns dict(coef, line, source, line_idx, patch) lists, one entry per appended plane."""
        d = np.ascontiguousarray(depth_f32, np.float32)
        out = np.zeros(self.supp_cap, SUPPOSED_DTYPE)
        lines = np.zeros(self.line_cap, np.int32)
        patch = np.zeros((self.supp_cap * self.patch_points, 3), np.float32)
        n = ctypes.c_int()
        self.ex._check(self.ex.lib.spslam_planes_generate_from_boundaries(
            self.ex.ctx, d.ctypes.data, d.shape[1], d.shape[0], d.shape[1], out.ctypes.data, self.supp_cap,
            ctypes.byref(n), lines.ctypes.data, patch.ctypes.data))
        res = dict(coef=[], line=[], source=[], line_idx=[], patch=[])
        for o in out[:n.value]:
            res["coef"].append(o["coef"].copy())
            res["line"].append(o["line"].copy())
            res["source"].append(int(o["source_plane"]))
            res["line_idx"].append(lines[o["line_offset"]:o["line_offset"] + o["n_line"]].copy())
            res["patch"].append(patch[o["patch_offset"]:o["patch_offset"] + o["n_patch"]].copy())
        return res

    def select_cloud_set(self, cloud_set):
        """The organized-cloud set of the extraction / supposed-plane calls enqueued next (0 or 1)."""
        self.ex._check(self.ex.lib.spslam_planes_select_cloud_set(self.ex.ctx, cloud_set))

    def generate_batch_device(self, depth_ptr, n_frames, frame_stride, stride, planes_ptr, counts_ptr, contours_ptr,
                              out_ptr, out_counts_ptr, line_ptr, patch_ptr, stream=0):
        self.ex._check(self.ex.lib.spslam_planes_generate_from_boundaries_batch_device(
            self.ex.ctx, depth_ptr, n_frames, frame_stride, stride, planes_ptr, counts_ptr, contours_ptr, out_ptr,
            out_counts_ptr, line_ptr, patch_ptr, stream or None))

    def line_candidates(self, frame, plane):
        """RANSAC line candidates of one boundary in the last supposed-plane call (parity access)."""
        cand = np.zeros(4, LINE_CAND_DTYPE)
        n = ctypes.c_int()
        idx = np.zeros(self.line_cap, np.int32)
        self.ex._check(self.ex.lib.spslam_supposed_debug(self.ex.ctx, frame, plane, cand.ctypes.data, ctypes.byref(n),
                                                         idx.ctypes.data, self.line_cap))
        out = []
        for c in cand[:n.value]:
            o = int(c["idx_offset"])
            out.append(dict(line=c["line"].copy(), n_inliers=int(c["n_inliers"]), iterations=int(c["iterations"]),
                            flags=int(c["flags"]),
                            cloud_idx=idx[o:o + c["n_inliers"]].copy() if o >= 0 else np.zeros(0, np.int32)))
        return out
