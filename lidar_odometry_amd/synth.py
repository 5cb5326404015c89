"""Deterministic synthetic LiDAR data for the benchmark configs (no datasets are reachable offline).

* ``KittiLikeSequence``  — HDL-64E-like spinning scanner (64 rings, -24.9..+2 deg, 1800 azimuth steps,
  ~115k returns, 100 m range, sigma 0.02 m) driving a meandering street (ground plane, building
  facades, poles, parked cars) at ~6 m/s, 10 Hz, 1101 frames (KITTI seq 07 length).  SURVEY.md §8d C1/C2/C4.
* ``mid360_like_scan``   — Livox-MID360-like non-repetitive scan (~20k pts, FoV 360 x -7..52 deg, <= 40 m).  C3.
* ``patch_scene``        — 1M-point scans of 1000 random planar patches + 10 % outliers.  C5.

Poses are 4x4 float64 world-from-sensor matrices; clouds are (N, 3) float32 in the sensor frame.
"""
from __future__ import annotations

import math

import numpy as np


# ----------------------------------------------------------------------------------------------------
# geometry helpers
# ----------------------------------------------------------------------------------------------------
def rot_z(yaw: float) -> np.ndarray:
    c, s = math.cos(yaw), math.sin(yaw)
    return np.array([[c, -s, 0.0], [s, c, 0.0], [0.0, 0.0, 1.0]])


def se3(R: np.ndarray, t) -> np.ndarray:
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = t
    return T


def exp_so3(w) -> np.ndarray:
    w = np.asarray(w, dtype=np.float64)
    th = np.linalg.norm(w)
    if th < 1e-12:
        return np.eye(3)
    k = w / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + math.sin(th) * K + (1 - math.cos(th)) * K @ K


def perturb(T: np.ndarray, rng: np.random.Generator, sigma_t=0.05, sigma_r=0.01) -> np.ndarray:
    """Right-perturb a pose by t ~ N(0, sigma_t), w ~ N(0, sigma_r) (SURVEY.md §8d parity micro-inputs)."""
    d = se3(exp_so3(rng.normal(0.0, sigma_r, 3)), rng.normal(0.0, sigma_t, 3))
    return T @ d


def transform(T: np.ndarray, pts: np.ndarray) -> np.ndarray:
    return (pts.astype(np.float64) @ T[:3, :3].T + T[:3, 3]).astype(np.float32)


class Scene:
    """Ground plane z = 0, yaw-rotated boxes, vertical cylinders."""

    def __init__(self, boxes: np.ndarray, cyls: np.ndarray, ground: bool = True):
        self.boxes = boxes    # (B, 7): cx, cy, cz, hx, hy, hz, yaw
        self.cyls = cyls      # (C, 5): cx, cy, r, z0, z1
        self.ground = ground

    def raycast(self, origin: np.ndarray, dirs: np.ndarray, max_range: float, near: float = 120.0) -> np.ndarray:
        """Distance along each unit ray to the first hit (inf = none)."""
        n = len(dirs)
        best = np.full(n, np.inf)
        o = origin
        if self.ground:
            dz = dirs[:, 2]
            with np.errstate(divide="ignore", invalid="ignore"):
                t = -o[2] / dz
            t[(dz >= -1e-9) | (t <= 0)] = np.inf
            best = np.minimum(best, t)
        if len(self.boxes):
            b = self.boxes
            dist = np.hypot(b[:, 0] - o[0], b[:, 1] - o[1]) - np.hypot(b[:, 3], b[:, 4])
            b = b[dist < near]
            for j0 in range(0, len(b), 16):
                bb = b[j0:j0 + 16]
                c, s = np.cos(-bb[:, 6]), np.sin(-bb[:, 6])
                ox = o[0] - bb[:, 0]; oy = o[1] - bb[:, 1]; oz = o[2] - bb[:, 2]
                lox = c * ox - s * oy; loy = s * ox + c * oy
                dx = dirs[:, 0:1] * c[None] - dirs[:, 1:2] * s[None]
                dy = dirs[:, 0:1] * s[None] + dirs[:, 1:2] * c[None]
                dzz = np.repeat(dirs[:, 2:3], len(bb), axis=1)
                with np.errstate(divide="ignore", invalid="ignore"):
                    tn = np.full((n, len(bb)), -np.inf)
                    tf = np.full((n, len(bb)), np.inf)
                    for lo_, d_, h in ((lox, dx, bb[:, 3]), (loy, dy, bb[:, 4]), (oz, dzz, bb[:, 5])):
                        t1 = (-h[None] - lo_[None]) / d_
                        t2 = (h[None] - lo_[None]) / d_
                        tmin = np.minimum(t1, t2)
                        tmax = np.maximum(t1, t2)
                        par = np.abs(d_) < 1e-12
                        inside = (np.abs(lo_) <= h)[None].repeat(n, 0)
                        tmin = np.where(par, np.where(inside, -np.inf, np.inf), tmin)
                        tmax = np.where(par, np.where(inside, np.inf, -np.inf), tmax)
                        tn = np.maximum(tn, tmin)
                        tf = np.minimum(tf, tmax)
                hit = (tn <= tf) & (tn > 0)
                tt = np.where(hit, tn, np.inf).min(axis=1)
                best = np.minimum(best, tt)
        if len(self.cyls):
            cy = self.cyls
            dist = np.hypot(cy[:, 0] - o[0], cy[:, 1] - o[1])
            cy = cy[dist < near]
            if len(cy):
                ox = o[0] - cy[:, 0]; oy = o[1] - cy[:, 1]
                a = dirs[:, 0:1] ** 2 + dirs[:, 1:2] ** 2
                bq = 2 * (dirs[:, 0:1] * ox[None] + dirs[:, 1:2] * oy[None])
                cq = (ox ** 2 + oy ** 2 - cy[:, 2] ** 2)[None]
                disc = bq * bq - 4 * a * cq
                with np.errstate(invalid="ignore", divide="ignore"):
                    sq = np.sqrt(np.maximum(disc, 0))
                    t1 = (-bq - sq) / (2 * a)
                z = o[2] + t1 * dirs[:, 2:3]
                ok = (disc > 0) & (t1 > 0) & (z >= cy[:, 3][None]) & (z <= cy[:, 4][None])
                best = np.minimum(best, np.where(ok, t1, np.inf).min(axis=1))
        best[best > max_range] = np.inf
        return best

    def raycast_torch(self, origin: np.ndarray, dirs: np.ndarray, max_range: float, device, near: float = 120.0):
        """raycast() with torch (float64) on `device` -- the same geometry, for generating long sequences quickly
        (bench maps); results agree with the numpy path to rounding.  Benchmark data only, never the product."""
        import torch
        d = torch.as_tensor(dirs, dtype=torch.float64, device=device)
        o = [float(v) for v in origin]
        n = d.shape[0]
        inf = torch.tensor(float("inf"), dtype=torch.float64, device=device)
        best = torch.full((n,), float("inf"), dtype=torch.float64, device=device)
        if self.ground:
            dz = d[:, 2]
            t = -o[2] / dz
            t = torch.where((dz >= -1e-9) | (t <= 0), inf, t)
            best = torch.minimum(best, t)
        if len(self.boxes):
            b = self.boxes
            dist = np.hypot(b[:, 0] - o[0], b[:, 1] - o[1]) - np.hypot(b[:, 3], b[:, 4])
            b = b[dist < near]
            for j0 in range(0, len(b), 64):
                bb = torch.as_tensor(b[j0:j0 + 64], dtype=torch.float64, device=device)
                c, sn = torch.cos(-bb[:, 6]), torch.sin(-bb[:, 6])
                ox = o[0] - bb[:, 0]; oy = o[1] - bb[:, 1]; oz = o[2] - bb[:, 2]
                lox = c * ox - sn * oy; loy = sn * ox + c * oy
                dx = d[:, 0:1] * c[None] - d[:, 1:2] * sn[None]
                dy = d[:, 0:1] * sn[None] + d[:, 1:2] * c[None]
                dzz = d[:, 2:3].expand(n, bb.shape[0])
                tn = torch.full((n, bb.shape[0]), -float("inf"), dtype=torch.float64, device=device)
                tf = torch.full((n, bb.shape[0]), float("inf"), dtype=torch.float64, device=device)
                for lo_, d_, h in ((lox, dx, bb[:, 3]), (loy, dy, bb[:, 4]), (oz, dzz, bb[:, 5])):
                    t1 = (-h[None] - lo_[None]) / d_
                    t2 = (h[None] - lo_[None]) / d_
                    tmin = torch.minimum(t1, t2)
                    tmax = torch.maximum(t1, t2)
                    par = d_.abs() < 1e-12
                    inside = (lo_.abs() <= h)[None].expand(n, -1)
                    tmin = torch.where(par, torch.where(inside, -inf, inf), tmin)
                    tmax = torch.where(par, torch.where(inside, inf, -inf), tmax)
                    tn = torch.maximum(tn, tmin)
                    tf = torch.minimum(tf, tmax)
                hit = (tn <= tf) & (tn > 0)
                best = torch.minimum(best, torch.where(hit, tn, inf).min(dim=1).values)
        if len(self.cyls):
            cy = self.cyls
            dist = np.hypot(cy[:, 0] - o[0], cy[:, 1] - o[1])
            cy = cy[dist < near]
            if len(cy):
                cy = torch.as_tensor(cy, dtype=torch.float64, device=device)
                ox = o[0] - cy[:, 0]; oy = o[1] - cy[:, 1]
                a = d[:, 0:1] ** 2 + d[:, 1:2] ** 2
                bq = 2 * (d[:, 0:1] * ox[None] + d[:, 1:2] * oy[None])
                cq = (ox ** 2 + oy ** 2 - cy[:, 2] ** 2)[None]
                disc = bq * bq - 4 * a * cq
                sq = torch.sqrt(torch.clamp(disc, min=0))
                t1 = (-bq - sq) / (2 * a)
                z = o[2] + t1 * d[:, 2:3]
                ok = (disc > 0) & (t1 > 0) & (z >= cy[:, 3][None]) & (z <= cy[:, 4][None])
                best = torch.minimum(best, torch.where(ok, t1, inf).min(dim=1).values)
        best = torch.where(best > max_range, inf, best)
        return best.cpu().numpy()


# ----------------------------------------------------------------------------------------------------
# KITTI-07-like sequence
# ----------------------------------------------------------------------------------------------------
class KittiLikeSequence:
    N_FRAMES = 1101
    HZ = 10.0
    SENSOR_H = 1.73

    def __init__(self, seed: int = 7, n_frames: int | None = None, ramp_s: float = 0.0):
        """ramp_s > 0: the vehicle starts from rest and reaches cruise speed after ramp_s seconds."""
        self.seed = seed
        self.n_frames = n_frames or self.N_FRAMES
        rng = np.random.default_rng(seed)
        # meandering trajectory (no self intersection), ~6 m/s with turns
        dt = 1.0 / self.HZ
        t = np.arange(self.n_frames) * dt
        heading = 0.6 * np.sin(2 * np.pi * t / 60.0) + 0.3 * np.sin(2 * np.pi * t / 23.0 + 0.7)
        speed = 6.0 + 1.0 * np.sin(2 * np.pi * t / 37.0)
        if ramp_s > 0.0:
            speed = speed * np.minimum(1.0, t / ramp_s)
        x = np.cumsum(speed * np.cos(heading) * dt)
        y = np.cumsum(speed * np.sin(heading) * dt)
        self.poses = []
        for i in range(self.n_frames):
            self.poses.append(se3(rot_z(heading[i]), [x[i], y[i], self.SENSOR_H]))
        # scene along the path
        boxes, cyls = [], []
        s_along = np.concatenate([[0.0], np.cumsum(np.hypot(np.diff(x), np.diff(y)))])
        total = s_along[-1] + 80.0
        sp = np.linspace(-80.0, total, int((total + 80.0) / 2.0))
        hx = np.interp(sp, np.concatenate([[-80.0], s_along]), np.concatenate([[x[0] - 80 * np.cos(heading[0])], x]))
        hy = np.interp(sp, np.concatenate([[-80.0], s_along]), np.concatenate([[y[0] - 80 * np.sin(heading[0])], y]))
        hh = np.interp(sp, np.concatenate([[-80.0], s_along]), np.concatenate([[heading[0]], heading]))

        def at(s):
            return np.interp(s, sp, hx), np.interp(s, sp, hy), np.interp(s, sp, hh)

        s = -80.0
        while s < total:                      # building facades on both sides
            for side in (-1.0, 1.0):
                if rng.random() < 0.12:
                    continue
                L = rng.uniform(8.0, 24.0)
                D = rng.uniform(6.0, 14.0)
                H = rng.uniform(4.0, 20.0)
                off = rng.uniform(9.0, 15.0) + D / 2
                px, py, ph = at(s + L / 2)
                nx, ny = -math.sin(ph), math.cos(ph)
                yaw = ph + rng.normal(0.0, 0.08)
                boxes.append([px + side * off * nx, py + side * off * ny, H / 2, L / 2, D / 2, H / 2, yaw])
            s += rng.uniform(14.0, 30.0)
        s = -80.0
        while s < total:                      # poles
            px, py, ph = at(s)
            nx, ny = -math.sin(ph), math.cos(ph)
            side = 1.0 if rng.random() < 0.5 else -1.0
            off = rng.uniform(5.0, 7.0)
            cyls.append([px + side * off * nx, py + side * off * ny, rng.uniform(0.12, 0.3), 0.0, rng.uniform(4, 9)])
            s += rng.uniform(12.0, 30.0)
        s = -80.0
        while s < total:                      # parked cars
            px, py, ph = at(s)
            nx, ny = -math.sin(ph), math.cos(ph)
            side = 1.0 if rng.random() < 0.5 else -1.0
            boxes.append([px + side * 4.0 * nx, py + side * 4.0 * ny, 0.75, 2.25, 0.9, 0.75, ph + rng.normal(0, 0.05)])
            s += rng.uniform(8.0, 40.0)
        s = -80.0
        while s < total:                      # vegetation: trunks + crowns, hedges
            px, py, ph = at(s)
            nx, ny = -math.sin(ph), math.cos(ph)
            side = 1.0 if rng.random() < 0.5 else -1.0
            off = rng.uniform(6.0, 30.0)
            cx, cyy = px + side * off * nx, py + side * off * ny
            cyls.append([cx, cyy, rng.uniform(0.15, 0.4), 0.0, rng.uniform(2.0, 4.0)])
            cr = rng.uniform(1.0, 2.5)
            boxes.append([cx, cyy, rng.uniform(3.5, 5.5), cr, cr, rng.uniform(0.8, 1.8), rng.uniform(0, np.pi)])
            if rng.random() < 0.5:
                boxes.append([cx + rng.uniform(-3, 3), cyy + rng.uniform(-3, 3), 0.5, rng.uniform(1, 4),
                              rng.uniform(0.4, 1.0), 0.5, ph + rng.normal(0, 0.3)])
            s += rng.uniform(3.0, 9.0)
        self.scene = Scene(np.array(boxes, dtype=np.float64), np.array(cyls, dtype=np.float64))
        # HDL-64E-like ray pattern, ring-major order like KITTI .bin files (each laser ring a full sweep)
        elev = np.deg2rad(np.linspace(-24.9, 2.0, 64))
        az = np.linspace(0.0, 2 * np.pi, 1800, endpoint=False)
        E, A = np.meshgrid(elev, az, indexing="ij")
        self.dirs = np.stack([np.cos(E) * np.cos(A), np.cos(E) * np.sin(A), np.sin(E)], axis=-1).reshape(-1, 3)

    def scan(self, i: int, device=None) -> np.ndarray:
        """Raw HDL-64-like scan of frame i (local frame).  device: raycast with torch there (raycast_torch)."""
        T = self.poses[i]
        rng = np.random.default_rng(1007 + i)
        dw = self.dirs @ T[:3, :3].T
        if device is None:
            r = self.scene.raycast(T[:3, 3], dw, max_range=100.0)
        else:
            r = self.scene.raycast_torch(T[:3, 3], dw, max_range=100.0, device=device)
        ok = np.isfinite(r)
        r = r[ok] + rng.normal(0.0, 0.02, ok.sum())
        pts = self.dirs[ok] * r[:, None]
        return pts.astype(np.float32)


class KittiCitySequence(KittiLikeSequence):
    """The same HDL-64E-like scanner driving a serpentine through a city grid: legs of `leg` m along parallel
    streets `spacing` m apart, joined by 90 degree turns (radius 8 m) through cross streets, facades, parked cars,
    poles and trees along every street.  Unlike the single meandering street of KittiLikeSequence, the 120 m
    pruning radius then holds several streets at once, so the keyframed map reaches the surfel count of an urban
    KITTI drive (~10^4 L1 surfels).  Benchmark data only."""

    def __init__(self, seed: int = 7, n_frames: int = 900, leg: float = 110.0, spacing: float = 44.0):
        self.seed = seed
        self.n_frames = n_frames
        rng = np.random.default_rng(seed + 500)
        dt, r_turn = 1.0 / self.HZ, 8.0
        t = np.arange(n_frames) * dt
        speed = 6.0 + 1.0 * np.sin(2 * np.pi * t / 37.0)
        s_frames = np.concatenate([[0.0], np.cumsum(speed[:-1] * dt)])
        total = s_frames[-1] + 1.0
        # path: straight leg, two quarter turns the same way, next leg back; alternate left / right
        segs, length, k = [], 0.0, 0
        while length < total:
            turn = 1.0 if k % 2 == 0 else -1.0
            for seg in ((leg, 0.0), (0.5 * np.pi * r_turn, turn / r_turn), (spacing - 2 * r_turn, 0.0),
                        (0.5 * np.pi * r_turn, turn / r_turn)):
                segs.append(seg)
                length += seg[0]
            k += 1
        n_legs = k + 1
        ds = 0.05
        xs, ys, hs = [0.0], [0.0], [0.0]
        for L, curv in segs:
            for _ in range(int(round(L / ds))):
                h = hs[-1] + curv * ds
                hm = 0.5 * (hs[-1] + h)
                xs.append(xs[-1] + ds * math.cos(hm))
                ys.append(ys[-1] + ds * math.sin(hm))
                hs.append(h)
        sp = np.arange(len(xs)) * ds
        x = np.interp(s_frames, sp, xs)
        y = np.interp(s_frames, sp, ys)
        heading = np.interp(s_frames, sp, hs)
        self.poses = [se3(rot_z(heading[i]), [x[i], y[i], self.SENSOR_H]) for i in range(n_frames)]
        # scene: along every horizontal street y = j * spacing, x in [-70, leg + 70], cross streets at the turns
        boxes, cyls = [], []
        cross = (-r_turn, leg + r_turn)
        max_back = spacing / 2 - 1.0
        for j in range(-1, n_legs + 1):
            y0 = j * spacing
            for side in (-1.0, 1.0):
                xa = -70.0
                while xa < leg + 70.0:
                    L = rng.uniform(8.0, 22.0)
                    if rng.random() < 0.12 or any(xa - 12.0 < c < xa + L + 12.0 for c in cross):
                        xa += L + rng.uniform(2.0, 8.0)
                        continue
                    off = rng.uniform(9.0, 12.0)
                    D = rng.uniform(6.0, max_back - off)
                    H = rng.uniform(4.0, 20.0)
                    boxes.append([xa + L / 2, y0 + side * (off + D / 2), H / 2, L / 2, D / 2, H / 2, rng.normal(0.0, 0.04)])
                    xa += L + rng.uniform(1.0, 6.0)
                xa = -70.0 + rng.uniform(0.0, 10.0)
                while xa < leg + 70.0:                # parked cars, poles, trees
                    u = rng.random()
                    if any(abs(xa - c) < 10.0 for c in cross):
                        pass
                    elif u < 0.45:
                        boxes.append([xa, y0 + side * rng.uniform(3.6, 4.4), 0.75, 2.25, 0.9, 0.75, rng.normal(0.0, 0.05)])
                    elif u < 0.65:
                        cyls.append([xa, y0 + side * rng.uniform(5.0, 7.0), rng.uniform(0.12, 0.3), 0.0, rng.uniform(4, 9)])
                    else:
                        cx, cy = xa, y0 + side * rng.uniform(5.5, 7.5)
                        cyls.append([cx, cy, rng.uniform(0.15, 0.4), 0.0, rng.uniform(2.0, 4.0)])
                        cr = rng.uniform(1.0, 2.5)
                        boxes.append([cx, cy, rng.uniform(3.5, 5.5), cr, cr, rng.uniform(0.8, 1.8), rng.uniform(0, np.pi)])
                    xa += rng.uniform(5.0, 14.0)
        self.scene = Scene(np.array(boxes, dtype=np.float64), np.array(cyls, dtype=np.float64))
        elev = np.deg2rad(np.linspace(-24.9, 2.0, 64))
        az = np.linspace(0.0, 2 * np.pi, 1800, endpoint=False)
        E, A = np.meshgrid(elev, az, indexing="ij")
        self.dirs = np.stack([np.cos(E) * np.cos(A), np.cos(E) * np.sin(A), np.sin(E)], axis=-1).reshape(-1, 3)


# ----------------------------------------------------------------------------------------------------
# MID360-like scan (C3)
# ----------------------------------------------------------------------------------------------------
def mid360_scene(seed: int = 107) -> Scene:
    rng = np.random.default_rng(seed)
    boxes = []
    # a courtyard of walls + furniture-like boxes within 40 m
    for k in range(4):
        yaw = k * np.pi / 2
        c = rot_z(yaw) @ np.array([18.0, 0.0, 0.0])
        boxes.append([c[0], c[1], 4.0, 0.4, 18.0, 4.0, yaw])
    # furniture stands on the floor, at most 1.4 m tall, and keeps >= 2.5 m clear of the sensor path
    # (x, y) = 0.3 k, 0.1 k, k < 42 (bench.py, tests): a sensor boxed in by tall clutter sees only the nearest
    # faces (a few hundred filtered points instead of the rosette's thousands)
    def clear(x, y, radius):
        t = np.clip((x * 12.3 + y * 4.1) / (12.3 ** 2 + 4.1 ** 2), 0.0, 1.0)
        return math.hypot(x - 12.3 * t, y - 4.1 * t) - radius > 2.5
    while len(boxes) < 28:
        hz = rng.uniform(0.3, 0.7)
        b = [rng.uniform(-15, 15), rng.uniform(-15, 15), hz,
             rng.uniform(0.3, 1.2), rng.uniform(0.3, 1.2), hz, rng.uniform(0, np.pi)]
        if clear(b[0], b[1], math.hypot(b[3], b[4])):
            boxes.append(b)
    cyls = []
    while len(cyls) < 12:
        c = [rng.uniform(-15, 15), rng.uniform(-15, 15), rng.uniform(0.15, 0.35), 0.0, rng.uniform(3, 8)]
        if clear(c[0], c[1], c[2]):
            cyls.append(c)
    return Scene(np.array(boxes), np.array(cyls))


def mid360_like_scan(scene: Scene, T: np.ndarray, frame: int, n_rays: int = 24000) -> np.ndarray:
    """Non-repetitive pattern over the MID360 field of view (360 deg x [-7, 52] deg): the R2 low-discrepancy
    sequence in (azimuth, elevation), continued across frames.  (A golden-angle azimuth with a 7x golden-ratio
    elevation phase puts every ray on one 7-petal curve -- 11k returns in ~350 voxels of 0.4 m.)"""
    k = np.arange(n_rays) + frame * n_rays
    az = 2.0 * np.pi * ((k * 0.7548776662466927) % 1.0)
    phase = (k * 0.5698402909980532) % 1.0
    el = np.deg2rad(-7.0 + 59.0 * phase)
    dirs = np.stack([np.cos(el) * np.cos(az), np.cos(el) * np.sin(az), np.sin(el)], axis=-1)
    rng = np.random.default_rng(1107 + frame)
    r = scene.raycast(T[:3, 3], dirs @ T[:3, :3].T, max_range=40.0, near=60.0)
    ok = np.isfinite(r) & (r > 0.1)
    r = r[ok] + rng.normal(0.0, 0.02, ok.sum())
    return (dirs[ok] * r[:, None]).astype(np.float32)


# ----------------------------------------------------------------------------------------------------
# C5: 1M-point planar-patch scans
# ----------------------------------------------------------------------------------------------------
def patch_scene(n_patches: int = 1000, seed: int = 1000, extent: float = 100.0):
    """Random planar patches (2-6 m squares) in a [-extent, extent]^2 x [0, 20] volume."""
    rng = np.random.default_rng(seed)
    centers = np.stack([rng.uniform(-extent, extent, n_patches), rng.uniform(-extent, extent, n_patches),
                        rng.uniform(0.0, 20.0, n_patches)], axis=1)
    normals = rng.normal(size=(n_patches, 3))
    normals /= np.linalg.norm(normals, axis=1, keepdims=True)
    a = np.cross(normals, np.array([0.0, 0.0, 1.0]))
    bad = np.linalg.norm(a, axis=1) < 1e-3
    a[bad] = np.cross(normals[bad], np.array([1.0, 0.0, 0.0]))
    a /= np.linalg.norm(a, axis=1, keepdims=True)
    b = np.cross(normals, a)
    size = rng.uniform(2.0, 6.0, n_patches)
    return {"c": centers, "n": normals, "a": a, "b": b, "size": size, "extent": extent}


def azimuth_order(local_pts) -> np.ndarray:
    """Reorder sensor-frame points by azimuth (then range), the acquisition order of a spinning LiDAR."""
    p = np.asarray(local_pts)
    az = np.arctan2(p[:, 1], p[:, 0])
    rg = np.einsum("ij,ij->i", p[:, :2], p[:, :2])
    return np.ascontiguousarray(p[np.lexsort((rg, az))])


def sample_patches(sc, n_points: int, seed: int, sigma: float = 0.01, outlier_frac: float = 0.1) -> np.ndarray:
    """World-frame samples: (1 - outlier_frac) on patches (area-weighted), the rest uniform in the volume."""
    rng = np.random.default_rng(seed)
    n_in = int(n_points * (1.0 - outlier_frac))
    w = sc["size"] ** 2
    idx = rng.choice(len(w), size=n_in, p=w / w.sum())
    u = rng.uniform(-0.5, 0.5, n_in) * sc["size"][idx]
    v = rng.uniform(-0.5, 0.5, n_in) * sc["size"][idx]
    p = sc["c"][idx] + u[:, None] * sc["a"][idx] + v[:, None] * sc["b"][idx]
    p += sc["n"][idx] * rng.normal(0.0, sigma, n_in)[:, None]
    e = sc["extent"]
    out = np.stack([rng.uniform(-e, e, n_points - n_in), rng.uniform(-e, e, n_points - n_in),
                    rng.uniform(0.0, 20.0, n_points - n_in)], axis=1)
    allp = np.concatenate([p, out], axis=0)
    return allp[rng.permutation(len(allp))].astype(np.float32)
