"""On-disk formats (lo_io.cpp) against the reference's documented stream semantics.
No reference binary or data file is run here (Eigen is absent, the datasets are external), so expected outputs
are derived from the reference source; quirks are asserted explicitly.  Host-only: runs without a GPU."""
import numpy as np
import pytest

from lidar_odometry_amd import io


def test_kitti_bin_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    rec = rng.normal(size=(1234, 4)).astype(np.float32)
    p = tmp_path / "000000.bin"
    p.write_bytes(rec.tobytes() + b"\x01\x02\x03")          # trailing partial record is ignored (:41-42)
    pts = io.load_kitti_bin(p)
    np.testing.assert_array_equal(pts, rec[:, :3])
    (tmp_path / "empty.bin").write_bytes(b"")
    assert io.load_kitti_bin(tmp_path / "empty.bin").shape == (0, 3)
    with pytest.raises(OSError):
        io.load_kitti_bin(tmp_path / "missing.bin")


def _ply_ascii(rows, props=("x", "y", "z", "intensity"), newline="\n"):
    head = ["ply", "format ascii 1.0", f"element vertex {len(rows)}"] + [f"property float {n}" for n in props] + ["end_header"]
    body = [" ".join(str(v) for v in r) for r in rows]
    return newline.join(head + body) + newline


def test_ply_ascii(tmp_path):
    rows = [[1.5, -2.25, 3.0, 7], [4.0, 5.0, 6.0, 8], [7.0, 8.0], [0.125, 1e-3, -1e5, 1]]   # short line skipped
    p = tmp_path / "a.ply"
    p.write_text(_ply_ascii(rows))
    pts = io.load_ply(p)
    np.testing.assert_array_equal(pts, np.array([[1.5, -2.25, 3.0], [4.0, 5.0, 6.0], [0.125, 1e-3, -1e5]], np.float32))
    p2 = tmp_path / "noz.ply"
    p2.write_text(_ply_ascii([[1, 2, 3]], props=("x", "y", "w")))
    assert io.load_ply(p2).shape == (0, 3)                    # parse_ply_header fails -> empty cloud
    p3 = tmp_path / "crlf.ply"
    p3.write_bytes(_ply_ascii([[1, 2, 3, 4]]).replace("\n", "\r\n").encode())
    assert io.load_ply(p3).shape == (0, 3)                    # quirk: "end_header\r" never matches


def test_ply_binary_and_quirks(tmp_path):
    rng = np.random.default_rng(1)
    xyz = rng.normal(size=(500, 3)).astype(np.float32)
    rgb = rng.integers(0, 255, size=(500, 3)).astype(np.uint8)
    head = ("ply\nformat binary_little_endian 1.0\nelement vertex 500\nproperty float x\nproperty float y\n"
            "property float z\nproperty uchar red\nproperty uchar green\nproperty uchar blue\nend_header\n")
    rec = np.zeros(500, dtype=[("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("r", "u1"), ("g", "u1"), ("b", "u1")])
    rec["x"], rec["y"], rec["z"] = xyz.T
    rec["r"], rec["g"], rec["b"] = rgb.T
    p = tmp_path / "b.ply"
    p.write_bytes(head.encode() + rec.tobytes())
    np.testing.assert_array_equal(io.load_ply(p), xyz)
    # quirk: a "double x" property is still read as the first 4 bytes of the 8-byte value
    head_d = ("ply\nformat binary_little_endian 1.0\nelement vertex 3\nproperty double x\nproperty float y\n"
              "property float z\nend_header\n")
    recd = np.zeros(3, dtype=[("x", "<f8"), ("y", "<f4"), ("z", "<f4")])
    recd["x"] = [1.0, 2.0, 3.0]
    recd["y"], recd["z"] = [4, 5, 6], [7, 8, 9]
    pd = tmp_path / "d.ply"
    pd.write_bytes(head_d.encode() + recd.tobytes())
    got = io.load_ply(pd)
    lo32 = np.frombuffer(recd["x"].tobytes(), dtype="<f4")[0::2]
    np.testing.assert_array_equal(got[:, 0], lo32)
    np.testing.assert_array_equal(got[:, 1:], np.array([[4, 7], [5, 8], [6, 9]], np.float32))
    # quirk: properties of later elements (face lists) still count toward the vertex stride
    head_f = ("ply\nformat binary_little_endian 1.0\nelement vertex 2\nproperty float x\nproperty float y\n"
              "property float z\nelement face 0\nproperty uchar n\nend_header\n")
    vals = np.array([1, 2, 3, 4, 5, 6], np.float32).tobytes() + b"\x00\x00"
    pf = tmp_path / "f.ply"
    pf.write_bytes(head_f.encode() + vals)
    got = io.load_ply(pf)                                     # stride 13 bytes: the second vertex is shifted
    assert got.shape[0] == 2
    np.testing.assert_array_equal(got[0], [1, 2, 3])
    np.testing.assert_array_equal(got[1], np.frombuffer(vals[13:25], "<f4"))


def test_kitti_trajectory(tmp_path):
    assert io.kitti_pose_line(np.eye(4)) == " ".join(
        ["1.000000000", "0.000000000", "0.000000000", "0.000000000",
         "0.000000000", "1.000000000", "0.000000000", "0.000000000",
         "0.000000000", "0.000000000", "1.000000000", "0.000000000"])
    from lidar_odometry_amd import synth
    rng = np.random.default_rng(2)
    poses = [synth.se3(synth.rot_z(a), rng.normal(size=3) * 10) for a in rng.uniform(-3, 3, 20)]
    A = np.array([[0, -1, 0, 0], [0, 0, -1, 0], [1, 0, 0, 0], [0, 0, 0, 1]], np.float64)
    for T in poses[:5]:
        want = (A @ np.asarray(T, np.float32).astype(np.float64) @ A.T)[:3, :4].reshape(12)
        got = np.array([float(v) for v in io.kitti_pose_line(T).split()])
        np.testing.assert_allclose(got, want, atol=5e-10)
    f = tmp_path / "07.txt"
    io.save_trajectory_kitti(f, poses)
    back = io.load_trajectory_kitti(f)
    np.testing.assert_allclose(back, np.stack(poses).astype(np.float32), atol=1e-8)
