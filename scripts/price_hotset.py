"""Price the staged (LDS) set of a hybrid sphere walk stream before changing it.

C4's stream (random-10k, 1.6 MB) is staged in LDS only in part: the node parts the builder ranks likeliest to
be reached (scene.cpp walk_place_and_write: largest parent box surface first, 77 KB), the rest read through a
buffer from L2/MALL.  This script measures, on real segments of a lane-simulated render (tests/native/
lane_sim.hip lane_sim_segments: origin, direction, final closest), which node parts a walk visits (a node is
visited iff every ancestor's box is hit on [t_min, closest], the boxes being nested), and compares the share
of visits that land in the staged set for
  - the builder's staged set (the stream as placed: offsets below walk_hot), and
  - the most-visited node parts of a training set of segments (other rows of the same frame),
both evaluated on held-out segments.  Slab tests in f64 on the stored C +- E boxes (pricing, not parity).

  python scripts/price_hotset.py [--preset random_10k] [--width 3840 --height 2160] [--rays 20000]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hyper-ray-tracer_amd"), ROOT, os.path.join(ROOT, "scripts")]
import hrt  # noqa: E402
from price_hierarchy import segments  # noqa: E402
from price_wide import build  # noqa: E402


def parse_tree(blob, info):
    """node parts of the (32-B) walk stream: offsets, boxes, parent index, leaf flag; pre-order from the root"""
    raw = bytes(blob)[info.off_walk:info.off_walk + info.walk_bytes]
    offs, boxes, parent, leaf = [], [], [], []
    stack = [(0, -1)]
    while stack:
        off, par = stack.pop()
        f = np.frombuffer(raw[off:off + 32], np.float32).astype(np.float64)
        u = np.frombuffer(raw[off:off + 32], np.uint32)
        k = len(offs)
        offs.append(off)
        boxes.append(np.r_[f[:3] - f[4:7], f[:3] + f[4:7]])
        parent.append(par)
        is_leaf = bool(u[7] & 0x80000000)
        leaf.append(is_leaf)
        if not is_leaf:
            first = int(u[7])
            second = int(np.frombuffer(raw[first:first + 16], np.uint32)[3])
            stack.append((second, k))
            stack.append((first, k))
    return np.asarray(offs), np.asarray(boxes), np.asarray(parent), np.asarray(leaf)


def hits(box, o, inv, tmin, tmax):
    t0 = (box[:3][None, :] - o) * inv
    t1 = (box[3:][None, :] - o) * inv
    lo = np.nanmax(np.minimum(t0, t1), axis=1)
    hi = np.nanmin(np.maximum(t0, t1), axis=1)
    return (np.maximum(lo, tmin) <= np.minimum(hi, tmax))


def visits(boxes, parent, rays, tmin=0.001):
    o = rays[:, :3].astype(np.float64)
    d = rays[:, 3:6].astype(np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / d
    cl = rays[:, 6].astype(np.float64)
    n = len(boxes)
    hit = np.zeros((n, len(rays)), bool)
    vis = np.zeros((n, len(rays)), bool)
    for k in range(n):  # pre-order: a parent comes before its children
        vis[k] = True if parent[k] < 0 else (vis[parent[k]] & hit[parent[k]])
        if vis[k].any():
            hit[k] = vis[k] & hits(boxes[k], o, inv, tmin, cl)
    return vis


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="random_10k")
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--rays", type=int, default=20000)
    ap.add_argument("--view", action="store_true", help="commit with hrt_scene_set_view(the preset camera): the "
                    "'builder' line then prices the library's view-ranked staged set")
    a = ap.parse_args()
    L = build()
    L.lane_sim_segments.restype = ctypes.c_int
    s = hrt.preset(a.preset, 1, None)
    if a.view:
        s.set_view(hrt.preset_camera(s.info, a.width, a.height))
    blob, info = hrt.scene_blob(s)
    assert info.walk_hot and not info.walk_c16, "a hybrid 32-B stream"
    offs, boxes, parent, leaf = parse_tree(blob, info)
    n_hot_parts = int((offs < info.walk_hot).sum())
    rng = np.random.default_rng(5)
    rows = rng.choice(a.height, 12, replace=False)
    tr = segments(L, s, blob, info, a.width, a.height, 2, [int(y) for y in rows[:6]])
    te = segments(L, s, blob, info, a.width, a.height, 2, [int(y) for y in rows[6:]], seed=9)
    tr = tr[rng.choice(len(tr), min(a.rays, len(tr)), replace=False)]
    te = te[rng.choice(len(te), min(a.rays, len(te)), replace=False)]
    print(f"{a.preset}: {len(offs)} node parts ({leaf.sum()} leaves), {n_hot_parts} staged ({info.walk_hot} B); "
          f"{len(tr)} training / {len(te)} test segments", flush=True)
    v_tr = visits(boxes, parent, tr).sum(axis=1)
    v_te_m = visits(boxes, parent, te)
    v_te = v_te_m.sum(axis=1)
    per_ray = v_te.sum() / len(te)
    built = offs < info.walk_hot
    freq = np.zeros(len(offs), bool)
    freq[np.argsort(-v_tr, kind="stable")[:n_hot_parts]] = True
    for name, hot in (("the library's staged set", built), ("training-visit ranked", freq)):
        lds = v_te[hot].sum() / len(te)
        print(f"  {name:32s}: node visits per segment {per_ray:.2f}, in LDS {lds:.2f}, global {per_ray - lds:.2f}")
    # lockstep view: a wave step reads global memory if any of its lanes' node is not staged (64 consecutive segments)
    sph = spheres_of(blob, info, offs, leaf)
    cam = hrt.preset_camera(s.info, a.width, a.height)
    for bounces in (0, 1, 2):
        pr = proxy_rays(sph, cam, a.width, a.height, a.rays, bounces, rng)
        v_pr = visits(boxes, parent, pr).sum(axis=1)
        hot = np.zeros(len(offs), bool)
        hot[np.argsort(-v_pr, kind="stable")[:n_hot_parts]] = True
        lds = v_te[hot].sum() / len(te)
        print(f"  proxy: camera rays + {bounces} diffuse bounces ({len(pr)} rays): in LDS {lds:.2f}, global {per_ray - lds:.2f}",
              flush=True)
    # what the library can compute without the leaves' geometry: camera rays stopped at the nearest LEAF BOX
    lb = boxes[leaf]
    u, v = rng.random(a.rays), rng.random(a.rays)
    org = np.array(cam.origin, np.float64)
    d = (np.array(cam.lower_left_corner) + u[:, None] * np.array(cam.horizontal) + v[:, None] * np.array(cam.vertical)) - org
    o = np.tile(org, (a.rays, 1))
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / d
        tb = np.full(a.rays, np.inf)
        for c0 in range(0, len(lb), 256):
            bx = lb[c0:c0 + 256]
            t0 = (bx[None, :, :3] - o[:, None, :]) * inv[:, None, :]
            t1 = (bx[None, :, 3:] - o[:, None, :]) * inv[:, None, :]
            lo = np.maximum(np.nanmax(np.minimum(t0, t1), axis=2), 0.001)
            hi = np.nanmin(np.maximum(t0, t1), axis=2)
            t = np.where(lo <= hi, lo, np.inf)
            tb = np.minimum(tb, t.min(axis=1))
    pr = np.c_[o, d, tb].astype(np.float32)
    v_pr = visits(boxes, parent, pr).sum(axis=1)
    hot = np.zeros(len(offs), bool)
    hot[np.argsort(-v_pr, kind="stable")[:n_hot_parts]] = True
    lds = v_te[hot].sum() / len(te)
    print(f"  proxy: camera rays to the nearest leaf box ({len(pr)} rays): in LDS {lds:.2f}, global {per_ray - lds:.2f}",
          flush=True)
    # + one bounce off the entered leaf box: from the entry point, a random direction about the entered face's normal
    hit = np.isfinite(tb)
    ob = o[hit] + tb[hit, None] * d[hit]
    ib = inv[hit]
    # the entered face: the axis whose slab entry is the latest
    lbh = None
    nrm = np.zeros_like(ob)
    with np.errstate(divide="ignore", invalid="ignore"):
        best = np.full(len(ob), -1)
        tbest = np.full(len(ob), np.inf)
        for c0 in range(0, len(lb), 256):
            bx = lb[c0:c0 + 256]
            t0 = (bx[None, :, :3] - o[hit][:, None, :]) * ib[:, None, :]
            t1 = (bx[None, :, 3:] - o[hit][:, None, :]) * ib[:, None, :]
            lo = np.maximum(np.nanmax(np.minimum(t0, t1), axis=2), 0.001)
            hi = np.nanmin(np.maximum(t0, t1), axis=2)
            t = np.where(lo <= hi, lo, np.inf)
            k = t.argmin(axis=1)
            tk = t[np.arange(len(ob)), k]
            bet = tk < tbest
            tbest[bet], best[bet] = tk[bet], c0 + k[bet]
        bx = lb[best]
        t0 = (bx[:, :3] - o[hit]) * ib
        t1 = (bx[:, 3:] - o[hit]) * ib
        ax = np.nanargmax(np.minimum(t0, t1), axis=1)
    nrm[np.arange(len(ob)), ax] = -np.sign(d[hit][np.arange(len(ob)), ax])
    g = rng.normal(size=ob.shape)
    db = nrm + g / np.linalg.norm(g, axis=1, keepdims=True)
    with np.errstate(divide="ignore", invalid="ignore"):
        ibb = 1.0 / db
        tb2 = np.full(len(ob), np.inf)
        for c0 in range(0, len(lb), 256):
            bx = lb[c0:c0 + 256]
            t0 = (bx[None, :, :3] - ob[:, None, :]) * ibb[:, None, :]
            t1 = (bx[None, :, 3:] - ob[:, None, :]) * ibb[:, None, :]
            lo = np.maximum(np.nanmax(np.minimum(t0, t1), axis=2), 0.01)
            hi = np.nanmin(np.maximum(t0, t1), axis=2)
            t = np.where(lo <= hi, lo, np.inf)
            tb2 = np.minimum(tb2, t.min(axis=1))
    pr2 = np.concatenate([pr, np.c_[ob, db, tb2].astype(np.float32)])
    v_pr = visits(boxes, parent, pr2).sum(axis=1)
    hot = np.zeros(len(offs), bool)
    hot[np.argsort(-v_pr, kind="stable")[:n_hot_parts]] = True
    lds = v_te[hot].sum() / len(te)
    print(f"  proxy: leaf-box camera rays + one bounce off the entered face ({len(pr2)} rays): in LDS {lds:.2f}, "
          f"global {per_ray - lds:.2f}", flush=True)
    for nr in (1000, 4000):
        v_pr = visits(boxes, parent, pr[:nr]).sum(axis=1)
        hot = np.zeros(len(offs), bool)
        hot[np.argsort(-v_pr, kind="stable")[:n_hot_parts]] = True
        lds = v_te[hot].sum() / len(te)
        print(f"  proxy: the same, {nr} rays: in LDS {lds:.2f}, global {per_ray - lds:.2f}", flush=True)
    m = (len(te) // 64) * 64
    for name, hot in (("builder", built), ("training-visit ranked", freq)):
        cold = (v_te_m[~hot, :m]).reshape(-1, m // 64, 64).any(axis=2).sum() if (~hot).any() else 0
        print(f"  {name:32s}: node parts x 64-segment groups with a global read: {cold / (m // 64):.2f} per group")


def spheres_of(blob, info, offs, leaf):
    """(centre at t0, radius) of every leaf's sphere (payload: mn,w | mx,r | c0,t0 | dc,dt | ...)"""
    raw = bytes(blob)[info.off_walk:info.off_walk + info.walk_bytes]
    out = []
    for off, lf in zip(offs, leaf):
        if not lf:
            continue
        p = int(np.frombuffer(raw[off + 28:off + 32], np.uint32)[0]) & 0x7FFFFFFF
        f = np.frombuffer(raw[p:p + 96], np.float32).astype(np.float64)
        out.append(np.r_[f[8:11], f[7]])
    return np.asarray(out)


def trace(sph, o, d, tmin=0.001, chunk=512):
    """closest sphere hit (t, index) per ray, brute force"""
    t_best = np.full(len(o), np.inf)
    i_best = np.full(len(o), -1)
    for a in range(0, len(sph), chunk):
        c, r = sph[a:a + chunk, :3], sph[a:a + chunk, 3]
        oc = o[:, None, :] - c[None, :, :]
        A = (d * d).sum(1)[:, None]
        hb = (oc * d[:, None, :]).sum(2)
        C = (oc * oc).sum(2) - r[None, :] ** 2
        disc = hb * hb - A * C
        sq = np.sqrt(np.maximum(disc, 0))
        t1 = (-hb - sq) / A
        t2 = (-hb + sq) / A
        t = np.where(t1 > tmin, t1, np.where(t2 > tmin, t2, np.inf))
        t = np.where(disc >= 0, t, np.inf)
        k = t.argmin(1)
        tk = t[np.arange(len(o)), k]
        better = tk < t_best
        t_best[better] = tk[better]
        i_best[better] = a + k[better]
    return t_best, i_best


def proxy_rays(sph, cam, W, H, n, bounces, rng):
    """camera rays through random pixels (pinhole), then `bounces` diffuse bounces off the hit spheres"""
    u, v = rng.random(n), rng.random(n)
    org = np.array(cam.origin, np.float64)
    d = (np.array(cam.lower_left_corner) + u[:, None] * np.array(cam.horizontal) + v[:, None] * np.array(cam.vertical)) - org
    o = np.tile(org, (n, 1))
    out = []
    for b in range(bounces + 1):
        t, i = trace(sph, o, d)
        out.append(np.c_[o, d, t])
        hit = np.isfinite(t)
        if b == bounces or not hit.any():
            break
        o, d, i = o[hit] + t[hit, None] * d[hit], d[hit], i[hit]
        nrm = (o - sph[i, :3]) / sph[i, 3:4]
        g = rng.normal(size=o.shape)
        d = nrm + g / np.linalg.norm(g, axis=1, keepdims=True)
    return np.concatenate(out).astype(np.float32)


if __name__ == "__main__":
    main()
