"""Dataset readers and trajectory IO around the tracking front end.

Host-side, like the reference's IO/ layer (it is not on the device path):
  * TumDataset  <- IO/DatasetTUM.cpp:28-89 (associations.txt, camera picked from the "freiburgN"
                   part of the path, depth factor 5000 / fr2 5208)
  * IclDataset  <- IO/DatasetICL.cpp:28-60 (associations.txt, fx 481.2, fy -480, no distortion)
  * CorbsDataset <- IO/DatasetCORBS.cpp:28-60 (associations.txt, fx 468.6, fy 468.61, cx 318.27,
                   cy 243.99, no distortion, depth factor 5000)
  * frames are read as cv::imread would hand them to Frame::Frame (Core/RGBDcamera.cpp:89-97):
    colour IMREAD_COLOR -> BGR u8, depth IMREAD_UNCHANGED -> u16
  * write_tum_trajectory   <- Tracking::saveCameraTrajectory (System/Tracking.cpp:286-317): "t tx ty tz
    qx qy qz qw" with precision 6 / 9 and the quaternion of Converter::toQuaternion (Eigen's
    Quaterniond(Matrix3d) assignment)
  * read_tum_trajectory / associate: the TUM benchmark's groundtruth format and associate.py rule
    (greedy closest pairs within max_difference), for tools/ate.py.
PNG decoding uses Pillow; a missing Pillow raises on first use.
"""
from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

# IO/DatasetTUM.cpp:61-89 (IntrinsicMatrix::setDistortion(k1, k2, k3, p1, p2), Core/IntrinsicMatrix.cpp:36)
TUM_CAMERAS = {
    "1": dict(fx=517.306408, fy=516.469215, cx=318.643040, cy=255.313989,
              k1=0.262383, k2=-0.953104, p1=-0.005358, p2=0.002628, k3=1.163314, factor=5000.0),
    "2": dict(fx=520.908620, fy=521.007327, cx=325.141442, cy=249.701764,
              k1=0.231222, k2=-0.784899, p1=-0.003257, p2=-0.000105, k3=0.917205, factor=5208.0),
    "3": dict(fx=535.4, fy=539.2, cx=320.1, cy=247.6,
              k1=0.0, k2=0.0, p1=0.0, p2=0.0, k3=0.0, factor=5000.0),
}
# IO/DatasetICL.cpp:37-38
ICL_CAMERA = dict(fx=481.2, fy=-480.0, cx=319.5, cy=239.5, k1=0.0, k2=0.0, p1=0.0, p2=0.0, k3=0.0,
                  factor=5000.0)
# IO/DatasetCORBS.cpp:37-39 (RGBDcamera(pIntrinsic, 40, 40, 5000, 30, 640, 480): depth factor 5000)
CORBS_CAMERA = dict(fx=468.6, fy=468.61, cx=318.27, cy=243.99, k1=0.0, k2=0.0, p1=0.0, p2=0.0, k3=0.0,
                    factor=5000.0)


def _pil():
    from PIL import Image  # noqa: WPS433 (optional dependency of the IO layer only)
    return Image


def read_associations(path: str):
    """associations.txt lines 't_rgb rgb_file t_depth depth_file' (DatasetTUM::open, :38-55): the
    frame timestamp is the RGB one."""
    times, rgb, dep = [], [], []
    with open(path) as f:
        for line in f:
            p = line.split()
            if len(p) < 4 or line.lstrip().startswith("#"):
                continue
            times.append(float(p[0]))
            rgb.append(p[1])
            dep.append(p[3])
    return np.array(times, np.float64), rgb, dep


class _Dataset:
    name = "dataset"

    def __init__(self, base_dir: str, camera: dict):
        self.base = base_dir if base_dir.endswith(os.sep) else base_dir + os.sep
        path = self.base + "associations.txt"
        if not os.path.exists(path):
            raise FileNotFoundError(f"{self.name}: no associations.txt in {base_dir}")
        self.times, self.rgb_files, self.depth_files = read_associations(path)
        self.camera = dict(camera)
        self.W, self.H = 640, 480   # RGBDcamera(..., 640, 480) for every dataset of the reference

    def __len__(self):
        return len(self.rgb_files)

    def frame(self, i: int):
        """(bgr [H, W, 3] u8, depth [H, W] u16) as cv::imread(IMREAD_COLOR / IMREAD_UNCHANGED)."""
        Image = _pil()
        with Image.open(self.base + self.rgb_files[i]) as im:
            rgb = np.asarray(im.convert("RGB"))
        with Image.open(self.base + self.depth_files[i]) as im:
            d = np.asarray(im)
        if d.dtype != np.uint16:
            d = d.astype(np.uint16)
        return np.ascontiguousarray(rgb[:, :, ::-1]), np.ascontiguousarray(d)

    def load(self, i0: int, n: int, threads: int = 8):
        """Frames i0 .. i0+n-1 as (bgr [n, H, W, 3] u8, depth [n, H, W] u16, times [n])."""
        n = max(0, min(n, len(self) - i0))
        bgr = np.empty((n, self.H, self.W, 3), np.uint8)
        dep = np.empty((n, self.H, self.W), np.uint16)

        def one(k):
            bgr[k], dep[k] = self.frame(i0 + k)

        with ThreadPoolExecutor(max_workers=max(1, threads)) as ex:
            list(ex.map(one, range(n)))
        return bgr, dep, self.times[i0:i0 + n].copy()


class TumDataset(_Dataset):
    """IO/DatasetTUM.cpp: the camera is chosen by the digit after "freiburg" in the path (:62-88)."""
    name = "TUM"

    def __init__(self, base_dir: str, camera: str | None = None):
        if camera is None:
            idx = base_dir.find("freiburg")
            if idx < 0 or idx + 8 >= len(base_dir) or base_dir[idx + 8] not in TUM_CAMERAS:
                raise ValueError(f"TUM: cannot detect the camera from {base_dir!r} (expects 'freiburg1/2/3')")
            camera = base_dir[idx + 8]
        super().__init__(base_dir, TUM_CAMERAS[camera])


class IclDataset(_Dataset):
    """IO/DatasetICL.cpp."""
    name = "ICL"

    def __init__(self, base_dir: str):
        super().__init__(base_dir, ICL_CAMERA)


class CorbsDataset(_Dataset):
    """IO/DatasetCORBS.cpp (same associations.txt layout as ICL; its own camera)."""
    name = "CORBS"

    def __init__(self, base_dir: str):
        super().__init__(base_dir, CORBS_CAMERA)


def open_dataset(base_dir: str, kind: str | None = None):
    """The reader main.cpp's DatasetType names (main.cpp:17-22): `kind` 'tum' / 'icl' / 'corbs', or by
    path when None: 'freiburg' -> TUM, 'corbs' (any case) -> CORBS, else ICL."""
    if kind is None:
        kind = "tum" if "freiburg" in base_dir else ("corbs" if "corbs" in base_dir.lower() else "icl")
    readers = {"tum": TumDataset, "icl": IclDataset, "corbs": CorbsDataset}
    if kind not in readers:
        raise ValueError(f"dataset kind must be one of {sorted(readers)}, not {kind!r}")
    return readers[kind](base_dir)


# ---------------------------------------------------------------- trajectories

def quaternion_eigen(R: np.ndarray):
    """Eigen::Quaterniond(Matrix3d) (quaternionbase_assign_impl: Shepperd's method on the trace or
    the largest diagonal entry), returned as (x, y, z, w) like Converter::toQuaternion."""
    m = np.asarray(R, np.float64)
    t = m[0, 0] + m[1, 1] + m[2, 2]
    if t > 0:
        t = np.sqrt(t + 1.0)
        w = 0.5 * t
        t = 0.5 / t
        x = (m[2, 1] - m[1, 2]) * t
        y = (m[0, 2] - m[2, 0]) * t
        z = (m[1, 0] - m[0, 1]) * t
        return x, y, z, w
    i = 0
    if m[1, 1] > m[0, 0]:
        i = 1
    if m[2, 2] > m[i, i]:
        i = 2
    j, k = (i + 1) % 3, (i + 2) % 3
    t = np.sqrt(m[i, i] - m[j, j] - m[k, k] + 1.0)
    q = [0.0, 0.0, 0.0]
    q[i] = 0.5 * t
    t = 0.5 / t
    w = (m[k, j] - m[j, k]) * t
    q[j] = (m[j, i] + m[i, j]) * t
    q[k] = (m[k, i] + m[i, k]) * t
    return q[0], q[1], q[2], w


def _rot_from_quat(x, y, z, w):
    n = np.sqrt(x * x + y * y + z * z + w * w)
    x, y, z, w = x / n, y / n, z / n, w / n
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def tum_trajectory_lines(times, Tcw):
    """Tracking::saveCameraTrajectory lines: camera centre twc = -Rwc t and the quaternion of Rwc in
    float (the reference's cv::Mat is CV_32F), printed with precision 6 (time) / 9 (pose)."""
    out = []
    for t, T in zip(times, Tcw):
        T = np.asarray(T, np.float32)
        Rwc = T[:3, :3].T
        twc = -(Rwc.astype(np.float64) @ T[:3, 3].astype(np.float64)).astype(np.float32)
        q = quaternion_eigen(Rwc.astype(np.float64))
        vals = [float(v) for v in twc] + [float(np.float32(v)) for v in q]
        out.append("%.6f " % t + " ".join("%.9f" % v for v in vals))
    return out


def _mat_mul_f32(A, B):
    """cv::Mat CV_32F product (gemm: double accumulation in k order, one rounding)."""
    A = np.asarray(A, np.float32).astype(np.float64)
    B = np.asarray(B, np.float32).astype(np.float64)
    C = np.zeros((A.shape[0], B.shape[1]), np.float64)
    for k in range(A.shape[1]):
        C += A[:, k:k + 1] * B[k:k + 1, :]
    return C.astype(np.float32)


def _pose_inverse_f32(T):
    """Frame::getPoseInverse (Core/Frame.cpp:137-153): [R^T | -R^T t], the translation one gemm."""
    T = np.asarray(T, np.float32)
    Ti = np.eye(4, dtype=np.float32)
    Ti[:3, :3] = T[:3, :3].T
    for i in range(3):
        s = 0.0
        for k in range(3):
            s += float(T[k, i]) * float(T[k, 3])
        Ti[i, 3] = np.float32(s * -1.0)
    return Ti


def camera_trajectory_poses(rel, keyframe, poses):
    """The poses Tracking::saveCameraTrajectory writes (System/Tracking.cpp:286-317) from a
    rgbd_track_batch_kf run: frame i's Tcw = mRelativeFramePoses[i] * (pose(its reference keyframe) *
    Two), Two = the first keyframe's getPoseInverse(), every product a float cv::Mat gemm.  A keyframe's
    pose at save time is the one updateLastFrame left it (Tcr * pose at its own step; no pose graph), except
    a keyframe at the last frame, which no later step rewrites."""
    rel = np.asarray(rel, np.float32).reshape(-1, 4, 4)
    poses = np.asarray(poses, np.float32).reshape(-1, 4, 4)
    kf = np.asarray(keyframe).astype(bool)
    n = len(rel)
    if n == 0:
        return np.zeros((0, 4, 4), np.float32)
    if not kf[0]:
        raise ValueError("frame 0 must be a keyframe (Tracking::initialize)")
    kf_pose = {}
    for i in np.nonzero(kf)[0]:
        # updateLastFrame at the keyframe's next step rewrites its pose to Tcr * pose; the sequence's last
        # frame has no next step, so a keyframe there keeps its pose as tracked
        kf_pose[i] = _mat_mul_f32(rel[i], poses[i]) if i < n - 1 else poses[i]
    Two = _pose_inverse_f32(kf_pose[0])
    out = np.zeros((n, 4, 4), np.float32)
    ref = 0
    for i in range(n):
        if kf[i]:
            ref = i
        Trw = _mat_mul_f32(_mat_mul_f32(np.eye(4, dtype=np.float32), kf_pose[ref]), Two)
        out[i] = _mat_mul_f32(rel[i], Trw)
    return out


def write_tum_trajectory(path: str, times, Tcw):
    with open(path, "w") as f:
        for line in tum_trajectory_lines(times, Tcw):
            f.write(line + "\n")


def read_tum_trajectory(path: str):
    """TUM 'timestamp tx ty tz qx qy qz qw' lines -> (times [n], Twc [n, 4, 4] f64)."""
    times, poses = [], []
    with open(path) as f:
        for line in f:
            if not line.strip() or line.lstrip().startswith("#"):
                continue
            v = [float(x) for x in line.replace(",", " ").split()]
            T = np.eye(4)
            T[:3, :3] = _rot_from_quat(v[4], v[5], v[6], v[7])
            T[:3, 3] = v[1:4]
            times.append(v[0])
            poses.append(T)
    return np.array(times, np.float64), np.array(poses, np.float64).reshape(-1, 4, 4)


def associate(first, second, offset: float = 0.0, max_difference: float = 0.02):
    """TUM associate.py: all (|a - (b + offset)|, a, b) pairs within max_difference, taken greedily
    from the closest, each stamp used once; returned as index pairs sorted by the first stamp."""
    first = np.asarray(first, np.float64)
    second = np.asarray(second, np.float64)
    cand = []
    for i, a in enumerate(first):
        d = np.abs(a - (second + offset))
        for j in np.nonzero(d < max_difference)[0]:
            cand.append((d[j], i, int(j)))
    cand.sort()
    used_a, used_b, pairs = set(), set(), []
    for _, i, j in cand:
        if i in used_a or j in used_b:
            continue
        used_a.add(i)
        used_b.add(j)
        pairs.append((i, j))
    pairs.sort()
    return pairs


def write_dataset(base_dir: str, bgr, depth, times, gt_Tcw=None):
    """A TUM-layout sequence (rgb/*.png, depth/*.png 16 bit, associations.txt, groundtruth.txt):
    used to feed synthetic sequences through the same reader as real ones."""
    Image = _pil()
    os.makedirs(os.path.join(base_dir, "rgb"), exist_ok=True)
    os.makedirs(os.path.join(base_dir, "depth"), exist_ok=True)
    lines = []
    for k, t in enumerate(times):
        rn, dn = "rgb/%.6f.png" % t, "depth/%.6f.png" % t
        Image.fromarray(np.ascontiguousarray(bgr[k][:, :, ::-1]), "RGB").save(os.path.join(base_dir, rn))
        Image.fromarray(np.ascontiguousarray(depth[k]).astype(np.uint16)).save(os.path.join(base_dir, dn))
        lines.append("%.6f %s %.6f %s" % (t, rn, t, dn))
    with open(os.path.join(base_dir, "associations.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    if gt_Tcw is not None:
        write_tum_trajectory(os.path.join(base_dir, "groundtruth.txt"), times, gt_Tcw)
