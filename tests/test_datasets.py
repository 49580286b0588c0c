"""Dataset readers and trajectory IO (rgbd-slam_amd/datasets.py; IO/DatasetTUM.cpp, IO/DatasetICL.cpp,
System/Tracking.cpp:286-317).  CPU only: synthetic sequences are written in the TUM layout and read back."""
import os

import numpy as np
import pytest

from conftest import load_pkg, synth_seq



def _ds():
    load_pkg()
    from rgbd_slam_amd import datasets
    return datasets


def test_tum_round_trip_and_camera(tmp_path):
    D = _ds()
    bgr, depth, gt, cam = synth_seq(3, seed=5, preset="fr1")
    base = str(tmp_path / "rgbd_dataset_freiburg1_synth") + os.sep
    times = 1305031102.175304 + 0.033 * np.arange(3)
    D.write_dataset(base, bgr, depth, times, gt)
    ds = D.open_dataset(base)
    assert isinstance(ds, D.TumDataset) and len(ds) == 3
    assert ds.camera == D.TUM_CAMERAS["1"]
    for k in ("fx", "fy", "cx", "cy", "k1", "k2", "p1", "p2", "k3", "factor"):
        assert ds.camera[k] == pytest.approx(cam[k])    # the synthetic presets are the reference's cameras
    b2, d2, t2 = ds.load(0, 3, threads=2)
    assert np.array_equal(b2, bgr) and np.array_equal(d2, depth)
    assert np.allclose(t2, np.round(times, 6))
    # groundtruth written in the reference's trajectory format reads back as the same poses
    gt_t, gt_Twc = D.read_tum_trajectory(base + "groundtruth.txt")
    assert np.allclose(np.linalg.inv(gt_Twc), gt, atol=2e-6)


def test_camera_detection_and_icl(tmp_path):
    D = _ds()
    bgr, depth, _, _ = synth_seq(2, seed=17, preset="icl")
    for digit in "123":
        base = str(tmp_path / f"rgbd_dataset_freiburg{digit}_x") + os.sep
        D.write_dataset(base, bgr, depth, [0.0, 0.03])
        assert D.TumDataset(base).camera == D.TUM_CAMERAS[digit]
    assert D.TUM_CAMERAS["2"]["factor"] == 5208.0           # IO/DatasetTUM.cpp:78
    base = str(tmp_path / "living_room_traj0") + os.sep
    D.write_dataset(base, bgr, depth, [0.0, 0.03])
    ds = D.open_dataset(base)
    assert isinstance(ds, D.IclDataset) and ds.camera["fy"] == -480.0   # IO/DatasetICL.cpp:37
    with pytest.raises(ValueError):
        D.TumDataset(str(tmp_path / "living_room_traj0"))
    with pytest.raises(FileNotFoundError):
        D.IclDataset(str(tmp_path / "missing"))


def test_corbs_reader(tmp_path):
    """IO/DatasetCORBS.cpp:37-39: fx 468.6, fy 468.61, cx 318.27, cy 243.99, no distortion, factor 5000."""
    D = _ds()
    bgr, depth, _, cam = synth_seq(2, seed=19, preset="corbs")
    base = str(tmp_path / "CORBS" / "D1") + os.sep
    D.write_dataset(base, bgr, depth, [0.0, 0.033])
    ds = D.open_dataset(base)
    assert isinstance(ds, D.CorbsDataset) and ds.name == "CORBS"
    assert ds.camera == dict(fx=468.6, fy=468.61, cx=318.27, cy=243.99, k1=0.0, k2=0.0, p1=0.0, p2=0.0, k3=0.0,
                             factor=5000.0)
    assert ds.camera == {k: pytest.approx(v) for k, v in cam.items()}
    b2, d2, _ = ds.load(0, 2, threads=1)
    assert np.array_equal(b2, bgr) and np.array_equal(d2, depth)
    assert isinstance(D.open_dataset(base, kind="icl"), D.IclDataset)
    with pytest.raises(ValueError):
        D.open_dataset(base, kind="kitti")


def test_quaternion_and_trajectory_lines():
    D = _ds()
    rs = np.random.default_rng(0)
    for _ in range(200):
        A = rs.normal(size=(3, 3))
        Q, _ = np.linalg.qr(A)
        if np.linalg.det(Q) < 0:
            Q[:, 0] *= -1
        x, y, z, w = D.quaternion_eigen(Q)
        assert np.allclose(D._rot_from_quat(x, y, z, w), Q, atol=1e-9)
        assert x * x + y * y + z * z + w * w == pytest.approx(1.0)
    T = np.eye(4, dtype=np.float32)
    T[:3, 3] = [1, 2, 3]
    line = D.tum_trajectory_lines([12.5], [T])[0].split()
    assert line[0] == "12.500000" and [float(v) for v in line[1:4]] == [-1.0, -2.0, -3.0]
    assert line[4:] == ["0.000000000", "0.000000000", "0.000000000", "1.000000000"]


def test_associate_and_batches():
    D = _ds()
    a = [0.0, 0.033, 0.066, 0.5]
    b = [0.001, 0.034, 0.030, 0.07, 0.9]
    assert D.associate(a, b) == [(0, 0), (1, 1), (2, 3)]
    load_pkg()
    from rgbd_slam_amd.sequence import batch_starts
    assert batch_starts(9, 5) == [0, 4]
    assert batch_starts(10, 5) == [0, 4, 8]
    assert batch_starts(1, 5) == [0] and batch_starts(0, 5) == []
    import pytest
    with pytest.raises(ValueError):   # batches overlap by one frame: B = 1 would never advance
        batch_starts(9, 1)


def test_camera_trajectory_poses_compose_like_save_camera_trajectory(pkg):
    """datasets.camera_trajectory_poses (System/Tracking.cpp:286-317): Tcw_i = Tcr_i * pose(KF) * Two
    with Two = the first keyframe's inverse; with consistent inputs it is Tcw_i * Tcw_0^-1 (the
    trajectory relative to the first keyframe) up to float rounding, and frame 0 maps to ~identity."""
    import importlib
    DS = importlib.import_module("rgbd_slam_amd.datasets")
    rs = np.random.RandomState(7)
    n = 9
    poses = np.zeros((n, 4, 4), np.float32)
    for i in range(n):
        a = 0.05 * i
        R = np.array([[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]])
        poses[i] = np.eye(4)
        poses[i][:3, :3] = R
        poses[i][:3, 3] = [0.1 * i, 0.02 * i * i, 1.0 + 0.01 * rs.randn()]
    kf = np.zeros(n, np.int32)
    kf[[0, 4, 7]] = 1
    rel = np.zeros_like(poses)
    ref = 0
    for i in range(n):
        if kf[i]:
            ref = i
        rel[i] = (poses[i].astype(np.float64) @ np.linalg.inv(poses[ref].astype(np.float64))).astype(np.float32)
    out = DS.camera_trajectory_poses(rel, kf, poses)
    want = poses.astype(np.float64) @ np.linalg.inv(poses[0].astype(np.float64))
    assert np.allclose(out, want, atol=1e-5)
    assert np.allclose(out[0], np.eye(4), atol=1e-6)
    with pytest.raises(ValueError):
        DS.camera_trajectory_poses(rel, np.zeros(n, np.int32), poses)
    # the last frame as a keyframe: no later updateLastFrame rewrites it, so its own pose is used as tracked
    kf2 = kf.copy()
    kf2[n - 1] = 1
    rel2 = rel.copy()
    rel2[n - 1] = (poses[n - 1].astype(np.float64) @ np.linalg.inv(poses[n - 1].astype(np.float64))).astype(np.float32)
    out2 = DS.camera_trajectory_poses(rel2, kf2, poses)
    assert np.array_equal(out2[:n - 1], out[:n - 1])
    Two = DS._pose_inverse_f32(DS._mat_mul_f32(rel[0], poses[0]))
    Trw = DS._mat_mul_f32(DS._mat_mul_f32(np.eye(4, dtype=np.float32), poses[n - 1]), Two)
    assert np.array_equal(out2[n - 1], DS._mat_mul_f32(rel2[n - 1], Trw))
