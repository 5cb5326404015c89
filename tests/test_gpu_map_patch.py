"""Incremental device map (SURVEY.md §8f-1, §8b lo_map_patch_surfels): a context kept in sync with a growing,
pruned voxel map by in-place table patches (lo_map_sync_voxelmap) answers every surfel lookup exactly as a
context that re-uploads the whole map after each update (lo_map_set_from_voxelmap): identical correspondence sets
and bit-identical fp64 residuals, across keyframes that insert, refit, lose and prune surfels.
"""
import ctypes as C

import numpy as np
import pytest

from lidar_odometry_amd import synth

pytestmark = pytest.mark.gpu


def _ctx():
    from lidar_odometry_amd import IterativeClosestPointOptimizer
    return IterativeClosestPointOptimizer(max_points=1 << 16)


def _sync(icp, vm):
    from lidar_odometry_amd import lib
    patched = C.c_int(0)
    rc = lib().lo_map_sync_voxelmap(icp.ctx, vm.handle, C.byref(patched))
    assert rc == 0, rc
    return patched.value


def _full(icp, vm):
    from lidar_odometry_amd import lib
    assert lib().lo_map_set_from_voxelmap(icp.ctx, vm.handle) == 0


def _same_lookups(a, b, pts, poses):
    for T in poses:
        na, va, ra = a.find_correspondences(pts, T)
        nb, vb, rb = b.find_correspondences(pts, T)
        assert na == nb
        np.testing.assert_array_equal(va, vb)
        np.testing.assert_array_equal(ra, rb)


def test_patched_table_matches_full_upload():
    from lidar_odometry_amd.voxelmap import VoxelMap, voxel_filter
    seq = synth.KittiLikeSequence(seed=7, n_frames=62)
    vm = VoxelMap(0.5, 3, 0.1, True)
    A, B = _ctx(), _ctx()
    try:
        kinds = []
        for k in range(0, 61, 2):
            T = seq.poses[k]
            pts = voxel_filter(seq.scan(k), 0.5, 8)
            # 60 m pruning radius: surfels leave the map as the sensor moves on (erase -> tombstones)
            vm.update(synth.transform(T, pts), T[:3, 3], 60.0, True)
            p = _sync(A, vm)
            _full(B, vm)
            kinds.append(p)
            assert A.surfel_count() == B.surfel_count() == vm.surfel_count()
            if k % 10 == 0:
                f = k + 1
                scan = voxel_filter(seq.scan(f), 0.5, 8)
                rng = np.random.default_rng(k)
                poses = [seq.poses[f][:3].astype(np.float32).reshape(12)] + \
                        [synth.perturb(seq.poses[f], rng, 0.3, 0.03)[:3].astype(np.float32).reshape(12) for _ in range(2)]
                _same_lookups(A, B, scan, poses)
        # the first sync uploads everything; while the map grows fast the table outgrows its headroom a few times,
        # after that keyframes are patched in place
        assert kinds[0] == -1
        assert sum(p >= 0 for p in kinds[len(kinds) // 2:]) >= len(kinds) // 4, kinds
    finally:
        A.close()
        B.close()


def test_patch_capacity_falls_back_to_full_upload():
    """Churn (a sensor jumping between two far places with a small radius) fills the table with tombstones: the
    sync then re-uploads the whole map (-1) and lookups still agree."""
    from lidar_odometry_amd.voxelmap import VoxelMap
    sc = synth.patch_scene(n_patches=80, seed=11, extent=30.0)
    vm = VoxelMap(0.5, 3, 0.1, True)
    A, B = _ctx(), _ctx()
    try:
        results = []
        for k in range(12):
            off = np.array([0.0 if k % 2 == 0 else 500.0, 0.0, 0.0], np.float32)
            w = synth.sample_patches(sc, 40000, 100 + k, outlier_frac=0.0) + off
            vm.update(w, off.astype(np.float64), 45.0, True)
            results.append(_sync(A, vm))
            _full(B, vm)
            assert A.surfel_count() == B.surfel_count()
        assert -1 in results[1:], results
        q = synth.sample_patches(sc, 5000, 999, outlier_frac=0.0) + np.array([500.0, 0.0, 0.0], np.float32)
        I = np.eye(3, 4, dtype=np.float32).reshape(12)
        _same_lookups(A, B, q, [I])
    finally:
        A.close()
        B.close()


def test_sync_after_apply_transform_uploads_the_rehashed_map():
    """ApplyTransformAndRehash restarts the map's journal: the next sync is a full upload, then patching resumes."""
    from lidar_odometry_amd.voxelmap import VoxelMap, voxel_filter
    seq = synth.KittiLikeSequence(seed=7, n_frames=30)
    vm = VoxelMap(0.5, 3, 0.1, True)
    A, B = _ctx(), _ctx()
    try:
        for k in range(0, 21, 2):
            vm.update(synth.transform(seq.poses[k], voxel_filter(seq.scan(k), 0.5, 8)), seq.poses[k][:3, 3], 120.0, True)
            _sync(A, vm)
        T = synth.se3(synth.rot_z(0.05), [0.4, -0.3, 0.02])
        vm.apply_transform(T[:3].astype(np.float32))
        assert _sync(A, vm) == -1
        _full(B, vm)
        f = 21
        scan = voxel_filter(seq.scan(f), 0.5, 8)
        Tf = (T @ seq.poses[f])[:3].astype(np.float32).reshape(12)
        _same_lookups(A, B, scan, [Tf])
        vm.update(synth.transform(T @ seq.poses[22], voxel_filter(seq.scan(22), 0.5, 8)), (T @ seq.poses[22])[:3, 3],
                  120.0, True)
        assert _sync(A, vm) >= 0
        _full(B, vm)
        _same_lookups(A, B, scan, [Tf])
    finally:
        A.close()
        B.close()


def test_device_fit_matches_host_fit():
    """lo_voxelmap_set_device_fit: the touched voxels' refits run on the device inside the sync (k_surfel_fit patches
    the table) and come back to the host map.  Against a map fitting on the host and fully re-uploaded each
    keyframe: identical host maps (surfel keys / normals / centroids / planarity bitwise, L0 and L1 counts) and
    identical lookups, across keyframes that insert, refit, lose and prune surfels."""
    from lidar_odometry_amd.voxelmap import VoxelMap, voxel_filter
    seq = synth.KittiLikeSequence(seed=7, n_frames=42)
    va, vb = VoxelMap(0.5, 3, 0.1, True), VoxelMap(0.5, 3, 0.1, True)
    va.set_device_fit(True)
    A, B = _ctx(), _ctx()
    try:
        patched = []
        for k in range(0, 41, 2):
            T = seq.poses[k]
            w = synth.transform(T, voxel_filter(seq.scan(k), 0.5, 8))
            va.update(w, T[:3, 3], 60.0, True)
            vb.update(w, T[:3, 3], 60.0, True)
            patched.append(_sync(A, va))
            _full(B, vb)
            if k % 8 == 0:
                f = k + 1
                scan = voxel_filter(seq.scan(f), 0.5, 8)
                _same_lookups(A, B, scan, [seq.poses[f][:3].astype(np.float32).reshape(12)])
            sa, sb = va.surfels(), vb.surfels()
            for x, y in zip(sa, sb):
                np.testing.assert_array_equal(np.asarray(x).view(np.uint32), np.asarray(y).view(np.uint32))
            assert (va.l0_count(), va.l1_count()) == (vb.l0_count(), vb.l1_count())
            assert A.surfel_count() == B.surfel_count() == vb.surfel_count()
        assert sum(p > 0 for p in patched[1:]) >= len(patched) // 2, patched
    finally:
        A.close()
        B.close()


def test_sync_of_a_new_map_on_the_same_context_uploads_it():
    """A context that mirrored map M1 and then syncs a NEW map M2 (possibly at M1's recycled address, with the same
    epoch and a journal at least as long) must upload M2, not patch M1's table: maps are named by a process-unique
    id, not by their address."""
    from lidar_odometry_amd.voxelmap import VoxelMap, voxel_filter
    seq = synth.KittiLikeSequence(seed=7, n_frames=30)
    A, B = _ctx(), _ctx()
    try:
        v1 = VoxelMap(0.5, 3, 0.1, True)
        for k in range(0, 9, 2):
            v1.update(synth.transform(seq.poses[k], voxel_filter(seq.scan(k), 0.5, 8)), seq.poses[k][:3, 3], 60.0, True)
            _sync(A, v1)
        v1.close()
        v2 = VoxelMap(0.5, 3, 0.1, True)
        for k in range(20, 29, 2):          # a different place: M1's surfels must not survive in A's table
            v2.update(synth.transform(seq.poses[k], voxel_filter(seq.scan(k), 0.5, 8)), seq.poses[k][:3, 3], 60.0, True)
        assert _sync(A, v2) == -1
        _full(B, v2)
        assert A.surfel_count() == B.surfel_count() == v2.surfel_count()
        for f in (1, 25):
            scan = voxel_filter(seq.scan(f), 0.5, 8)
            _same_lookups(A, B, scan, [seq.poses[f][:3].astype(np.float32).reshape(12)])
        v2.close()
    finally:
        A.close()
        B.close()


def test_patch_duplicate_keys_last_record_wins():
    """lo_map_patch_surfels with a key given twice (insert then erase, two payloads): the last record decides, as on
    the host side, and the resident count agrees with the table."""
    from lidar_odometry_amd import lib
    A = _ctx()
    try:
        keys0 = np.array([[0, 0, 0], [5, 0, 0]], np.int32)
        n0 = np.tile(np.array([0, 0, 1], np.float32), (2, 1))
        c0 = np.array([[0.7, 0.7, 0.7], [7.9, 0.7, 0.7]], np.float32)
        A.set_surfels(keys0, n0, c0)
        fp = C.POINTER(C.c_float)
        keys = np.array([[1, 0, 0], [1, 0, 0], [0, 0, 0], [0, 0, 0], [5, 0, 0], [5, 0, 0]], np.int32)
        nrm = np.tile(np.array([0, 0, 1], np.float32), (6, 1))
        nrm[3] = [1, 0, 0]
        cen = np.array([[2.2, .7, .7], [2.2, .7, .7], [.7, .7, .7], [.7, .7, .9], [7.9, .7, .7], [7.9, .7, .7]], np.float32)
        present = np.array([1, 0, 0, 1, 1, 0], np.uint8)    # key 1: inserted then erased; key 0: erased then re-set
        rc = lib().lo_map_patch_surfels(A.ctx, keys.ctypes.data_as(C.POINTER(C.c_int32)), nrm.ctypes.data_as(fp),
                                        cen.ctypes.data_as(fp), present.ctypes.data_as(C.POINTER(C.c_uint8)), 6)
        assert rc == 0
        assert A.surfel_count() == 1                       # key 0 only
        I = np.eye(3, 4, dtype=np.float32).reshape(12)
        pts = np.array([[0.7, 0.7, 0.7], [2.2, 0.7, 0.7], [7.9, 0.7, 0.7]], np.float32)
        n, v, r = A.find_correspondences(pts, I)
        assert n == 1 and v.tolist() == [True, False, False]
        assert r[0] == 0.0                                 # key 0's LAST payload: normal x, centroid x = 0.7
    finally:
        A.close()


def test_device_fit_count_before_the_map_is_read():
    """With device fits pending, the context's surfel count already excludes the fits that failed planarity (no
    reader of the host map has run yet)."""
    from lidar_odometry_amd.voxelmap import VoxelMap, voxel_filter
    seq = synth.KittiLikeSequence(seed=7, n_frames=22)
    va, vb = VoxelMap(0.5, 3, 0.1, True), VoxelMap(0.5, 3, 0.1, True)
    va.set_device_fit(True)
    A = _ctx()
    try:
        for k in range(0, 21, 2):
            w = synth.transform(seq.poses[k], voxel_filter(seq.scan(k), 0.5, 8))
            va.update(w, seq.poses[k][:3, 3], 60.0, True)
            vb.update(w, seq.poses[k][:3, 3], 60.0, True)
            _sync(A, va)
            assert A.surfel_count() == vb.surfel_count()     # before va is read
    finally:
        A.close()


def test_sync_surfels_sends_only_the_difference():
    """lo_map_sync_surfels (the reference-side sync of a caller that keeps its own VoxelMap): the whole current surfel
    set goes in, only the changed voxels reach the device, and every lookup equals a full upload's."""
    from lidar_odometry_amd.voxelmap import VoxelMap, voxel_filter
    seq = synth.KittiLikeSequence(seed=7, n_frames=42)
    vm = VoxelMap(0.5, 3, 0.1, True)
    A, B = _ctx(), _ctx()
    try:
        prev = None
        for k in range(0, 41, 2):
            T = seq.poses[k]
            vm.update(synth.transform(T, voxel_filter(seq.scan(k), 0.5, 8)), T[:3, 3], 60.0, True)
            keys, nrm, ctr, _ = vm.surfels()
            p = A.sync_surfels(keys, nrm, ctr)
            B.set_surfels(keys, nrm, ctr)
            cur = {tuple(kk): (tuple(nn), tuple(cc)) for kk, nn, cc in zip(keys.tolist(), nrm.tolist(), ctr.tolist())}
            if prev is None:
                assert p == -1                                  # first sync: full upload
            else:
                changed = sum(1 for kk, v in cur.items() if prev.get(kk) != v) + sum(1 for kk in prev if kk not in cur)
                assert p == -1 or p == changed, (p, changed)
            assert A.sync_surfels(keys, nrm, ctr) == 0          # nothing changed since
            assert A.surfel_count() == B.surfel_count() == len(cur)
            prev = cur
            if k % 8 == 0:
                f = k + 1
                pts = voxel_filter(seq.scan(f), 0.5, 8)
                _same_lookups(A, B, pts, [seq.poses[f][:3, :].astype(np.float32).reshape(12)])
        # a table changed by anything else (a plain upload) makes the next sync a full one
        A.set_surfels(keys[:10], nrm[:10], ctr[:10])
        assert A.sync_surfels(keys, nrm, ctr) == -1
        _same_lookups(A, B, pts, [seq.poses[41][:3, :].astype(np.float32).reshape(12)])
    finally:
        A.close()
        B.close()


def test_update_config_keeps_the_device_map():
    """update_config (IterativeClosestPointOptimizer.h:220) replaces the parameters only: the next optimize runs on the
    same device map, equal to a fresh context made with the new parameters."""
    from lidar_odometry_amd import ICPConfig, IterativeClosestPointOptimizer
    from tests import _data
    m, pts, Ti, _ = _data.kitti_case(15, seed=5, sigma_t=0.3, sigma_r=0.03)
    k, n, c = _data.surfels(m)
    A = IterativeClosestPointOptimizer(max_points=1 << 16)
    B = IterativeClosestPointOptimizer(ICPConfig(max_iterations=2, min_correspondence_points=20), max_points=1 << 16)
    try:
        A.set_surfels(k, n, c)
        B.set_surfels(k, n, c)
        ok4, _ = A.optimize(None, pts, Ti)
        assert ok4 and A.get_last_stats().num_iterations >= 3
        A.update_config(ICPConfig(max_iterations=2, min_correspondence_points=20))
        okA, TA = A.optimize(None, pts, Ti)
        okB, TB = B.optimize(None, pts, Ti)
        assert okA and okB and A.get_last_stats().num_iterations == 2
        np.testing.assert_array_equal(np.asarray(TA, np.float32).view(np.uint32), np.asarray(TB, np.float32).view(np.uint32))
        from lidar_odometry_amd import MapGeometry
        with pytest.raises(RuntimeError):                     # the voxel geometry is fixed at creation
            cfg = ICPConfig()
            A.geometry = MapGeometry(voxel_size=0.4)
            A.update_config(cfg)
    finally:
        A.close()
        B.close()


def test_keyed_sync_of_changed_voxels_matches_full_upload():
    """The adapter's keyed sync_map(vm, changed), mirrored by sync_changed: after one whole upload,
    each keyframe patches only the L1 keys the update changed (lo_voxelmap_changed_l1 = the reference hook's list),
    each looked up with GetSurfelAtPoint at its voxel centre -- the device table answers every lookup as a full
    upload does, across inserts, refits, planarity losses and the 60 m prune."""
    from lidar_odometry_amd.voxelmap import VoxelMap, voxel_filter
    seq = synth.KittiLikeSequence(seed=7, n_frames=62)
    vm = VoxelMap(0.5, 3, 0.1, True)
    A, B = _ctx(), _ctx()
    try:
        sent = []
        for k in range(0, 61, 2):
            T = seq.poses[k]
            pts = voxel_filter(seq.scan(k), 0.5, 8)
            vm.update(synth.transform(T, pts), T[:3, 3], 60.0, True)
            if k == 0:
                s = vm.surfels()
                A.set_surfels(s[0], s[1], s[2])
            else:
                sent.append(A.sync_changed(vm, vm.changed_l1()))
            _full(B, vm)
            assert A.surfel_count() == B.surfel_count() == vm.surfel_count()
            if k % 10 == 0:
                f = k + 1
                _same_lookups(A, B, voxel_filter(seq.scan(f), 0.5, 8), [seq.poses[f]])
        keyed = [x for x in sent if x >= 0]             # -1: a table full of tombstones was uploaded whole
        assert len(keyed) > len(sent) // 2 and 0 < np.mean(keyed) < vm.surfel_count()
    finally:
        A.close()
        B.close()
