"""Host cost of a keyframe's map update and of bringing the device table up to date: full re-upload
(lo_map_set_from_voxelmap: host re-hash of every surfel + blocking copy of the whole table) against the in-place
patch (lo_map_sync_voxelmap: the L1 voxels the update changed, async).  KITTI-like sequence, keyframe every 2 frames,
pruning radius 120 m; times per keyframe over the second half (the map at its steady size).  Third column: the
same map with device surfel fits (lo_voxelmap_set_device_fit: update without fits + patch + k_surfel_fit, the
results applied at the next update).  Fourth: the reference-side sync (the adapter's sync_map ->
lo_map_sync_surfels): the map's whole surfel set handed over each keyframe, diffed against the context's resident
set, only the difference patched.  Fifth (r06): the adapter's keyed sync_map(vm, changed) -- only the L1 keys the
update changed (the INTEGRATION.md hook's list, here lo_voxelmap_changed_l1), GetSurfelAtPoint at each key's centre,
lo_map_patch_surfels; its host part is the Python mirror sync_changed (the C++ adapter does the same loop)."""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lidar_odometry_amd import IterativeClosestPointOptimizer, lib, synth  # noqa: E402
from lidar_odometry_amd.voxelmap import VoxelMap, voxel_filter  # noqa: E402

import torch  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
dev = "cuda:0" if torch.cuda.is_available() else None
seq = synth.KittiLikeSequence(seed=7, n_frames=n + 2)
vm = VoxelMap(0.5, 3, 0.1, True)
vd = VoxelMap(0.5, 3, 0.1, True)
vd.set_device_fit(True)
A, B = IterativeClosestPointOptimizer(max_points=1 << 16), IterativeClosestPointOptimizer(max_points=1 << 16)
D = IterativeClosestPointOptimizer(max_points=1 << 16)
E = IterativeClosestPointOptimizer(max_points=1 << 16)
F = IterativeClosestPointOptimizer(max_points=1 << 16)
t_upd, t_full, t_patch, kinds, t_dev, t_ref, sent = [], [], [], [], [], [], []
t_key, sent_key, t_key_host, t_key_list = [], [], [], []
patched = C.c_int(0)
for k in range(0, n + 1, 2):
    T = seq.poses[k]
    w = synth.transform(T, voxel_filter(seq.scan(k, device=dev), 0.5, 8))
    t0 = time.perf_counter()
    vm.update(w, T[:3, 3], 120.0, True)
    t1 = time.perf_counter()
    assert lib().lo_map_set_from_voxelmap(B.ctx, vm.handle) == 0
    t2 = time.perf_counter()
    assert lib().lo_map_sync_voxelmap(A.ctx, vm.handle, C.byref(patched)) == 0
    lib().lo_sync(A.ctx)
    t3 = time.perf_counter()
    t4 = time.perf_counter()
    vd.update(w, T[:3, 3], 120.0, True)
    assert lib().lo_map_sync_voxelmap(D.ctx, vd.handle, C.byref(patched)) == 0
    lib().lo_sync(D.ctx)
    t5 = time.perf_counter()
    keys, normals, cents, _ = vm.surfels()
    t6 = time.perf_counter()
    sent.append(E.sync_surfels(keys, normals, cents))
    lib().lo_sync(E.ctx)
    t7 = time.perf_counter()
    # the adapter's keyed sync_map(vm, changed): only the keys the update changed (the reference hook's list),
    # GetSurfelAtPoint at each key's centre, lo_map_patch_surfels (C++ in the adapter; the Python mirror here)
    t8 = time.perf_counter()
    t8a = t8
    if k == 0:
        F.set_surfels(keys, normals, cents)
    else:
        ch = vm.changed_l1()                     # the hook's key list (a ctypes call + array here; a vector in C++)
        t8a = time.perf_counter()
        sent_key.append(F.sync_changed(vm, ch))
    t8b = time.perf_counter()                    # host work only: the patch is queued on the context stream
    lib().lo_sync(F.ctx)
    t9 = time.perf_counter()
    t_key.append(t9 - t8)
    t_key_host.append(t8b - t8)
    t_key_list.append(t8a - t8)
    t_upd.append(t1 - t0); t_full.append(t2 - t1); t_patch.append(t3 - t2); kinds.append(patched.value)
    t_dev.append(t5 - t4)
    t_ref.append(t7 - t6)
h = len(t_upd) // 2
ms = lambda v: 1e3 * float(np.mean(v[h:]))  # noqa: E731
print(f"keyframes {len(t_upd)}, surfels {vm.surfel_count()}, L0 {vm.l0_count()}: per keyframe (second half) "
      f"host map update {ms(t_upd):.3f} ms, full upload {ms(t_full):.3f} ms, patch {ms(t_patch):.3f} ms "
      f"(incl. stream sync); patched voxels per keyframe {np.mean([p for p in kinds[h:] if p >= 0]):.0f}, "
      f"full re-uploads in the second half {sum(p < 0 for p in kinds[h:])}; with device fits: update + sync "
      f"{ms(t_dev):.3f} ms (host fits: {ms(t_upd) + ms(t_patch):.3f} ms); reference-side sync_surfels of the full "
      f"surfel set {ms(t_ref):.3f} ms, {np.mean([x for x in sent[h:] if x >= 0]):.0f} records sent per keyframe "
      f"(full uploads in the second half: {sum(x < 0 for x in sent[h:])}); keyed sync of the changed keys "
      f"{ms(t_key):.3f} ms incl. the stream sync, {ms(t_key_host):.3f} ms of host work (the patch queued on the "
      f"stream; of it {ms(t_key_list):.3f} ms fetching the key list, {ms(t_key_host) - ms(t_key_list):.3f} ms the "
      f"lookups + patch), {np.mean([x for x in sent_key[h:] if x >= 0]):.0f} keys per keyframe (full uploads in the second "
      f"half: {sum(x < 0 for x in sent_key[h:])})")
assert F.surfel_count() == vm.surfel_count()
assert vd.surfel_count() == vm.surfel_count()
