"""Estimate SIMT lane utilization of traversal schedules on real path-traced rays.

Rays come from the oracle path-tracing a pixel sample of a scene (so the mix
of camera, extension and shadow rays is the real one); for each ray the
oracle records its (descent node fetches, leaf size) visit sequence.  Costs
are in abstract units: Cd per descent step, Cl per 2-entry leaf step, Cp per
leaf visit overhead (pop/fetch).
usage: python tools/simt_sim.py [scene] [pixels]
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("isaklm-raytracer_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import helpers  # noqa: E402
import oracle  # noqa: E402

Cd, Cl, Cp = 1.0, 3.0, 1.0


def load(scene, npix):
    L = oracle.lib()
    L.or_log_rays.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_int] * 2 + [ctypes.c_void_p, ctypes.c_int,
                                                                            ctypes.c_void_p, ctypes.c_int]
    L.or_trace_visits.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_int]
    sc = oracle.OracleScene(helpers.scene_path(scene))
    W, H = 1920, 1080
    rng = np.random.default_rng(0)
    # 8x8 tiles of pixels (the kernels' wave shape), spread over the frame
    tiles = rng.integers(0, (W // 8) * (H // 8), npix // 64)
    pix = []
    for t in tiles:
        tx, ty = t % (W // 8), t // (W // 8)
        for j in range(64):
            pix.append((ty * 8 + j // 8) * W + tx * 8 + j % 8)
    pix = np.array(pix, np.int32)
    cap = len(pix) * 64
    rays = np.zeros((cap, 6), np.float32)
    n = L.or_log_rays(sc.h, sc.camera.ctypes.data, W, H, pix.ctypes.data, len(pix), rays.ctypes.data, cap)
    rays = rays[:n]
    offs = np.zeros(n + 1, np.int32)
    vis = np.zeros(200_000_000, np.int32)
    L.or_trace_visits(sc.h, rays.ctypes.data, n, offs.ctypes.data, vis.ctypes.data, len(vis))
    vis = vis[:2 * offs[-1]].reshape(-1, 2)
    seqs = [vis[offs[i]:offs[i + 1]] for i in range(n)]
    return rays, seqs


def visit_cost(v):
    d, c = v
    return d * Cd + ((c + 1) // 2) * Cl + Cp


def ideal(seqs):
    return sum(sum(visit_cost(v) for v in s) for s in seqs)


def static_sched(seqs):
    """waves of 64 consecutive rays; each outer iteration = one leaf visit per active lane."""
    total = 0.0
    for w in range(0, len(seqs), 64):
        grp = seqs[w:w + 64]
        K = max(len(s) for s in grp)
        for i in range(K):
            act = [s[i] for s in grp if i < len(s)]
            total += max(a[0] for a in act) * Cd + max((a[1] + 1) // 2 for a in act) * Cl + Cp
    return total


def dynamic_sched(seqs, coop_leaf=False):
    """lanes refill from the ray stream at leaf boundaries."""
    total = 0.0
    stream = iter(range(len(seqs)))
    lanes = [[next(stream, None), 0] for _ in range(64)]
    while True:
        act = []
        for l in lanes:
            while l[0] is not None and l[1] >= len(seqs[l[0]]):
                l[0], l[1] = next(stream, None), 0
            if l[0] is not None:
                act.append(seqs[l[0]][l[1]])
                l[1] += 1
        if not act:
            break
        dmax = max(a[0] for a in act)
        leaf = (sum((a[1] + 1) // 2 for a in act) + 63) // 64 if coop_leaf else max((a[1] + 1) // 2 for a in act)
        total += dmax * Cd + leaf * Cl + Cp
    return total


def postponed_sched(seqs, K, T):
    """dynamic fetch + cooperative leaves, with the descent capped at K steps
    per round and the cooperative leaf test run only once T lanes hold a
    leaf (or no lane is still descending)."""
    total = 0.0
    stream = iter(range(len(seqs)))
    # lane: [ray, visit index, descent steps left, pending leaf size or -1]
    lanes = []
    for _ in range(64):
        r = next(stream, None)
        lanes.append([r, 0, seqs[r][0][0] if r is not None and len(seqs[r]) else 0, -1])

    def advance(l):
        while l[0] is not None and l[1] >= len(seqs[l[0]]):
            l[0], l[1] = next(stream, None), 0
            if l[0] is not None and len(seqs[l[0]]):
                l[2] = seqs[l[0]][0][0]
        return l[0] is not None

    while True:
        live = [l for l in lanes if advance(l)]
        if not live:
            break
        desc = [l for l in live if l[3] < 0]
        if desc:
            steps = min(K, max(l[2] for l in desc))
            total += steps * Cd
            for l in desc:
                l[2] -= steps
                if l[2] <= 0:
                    l[3] = seqs[l[0]][l[1]][1]
        pend = [l for l in live if l[3] >= 0]
        if pend and (len(pend) >= T or len(pend) == len(live)):
            total += (sum((l[3] + 1) // 2 for l in pend) + 63) // 64 * Cl + Cp
            for l in pend:
                l[3] = -1
                l[1] += 1
                if l[1] < len(seqs[l[0]]):
                    l[2] = seqs[l[0]][l[1]][0]
    return total


def main():
    scene = sys.argv[1] if len(sys.argv) > 1 else "room2m"
    npix = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    rays, seqs = load(scene, npix)
    per_lane = ideal(seqs) / 64
    st = static_sched(seqs)
    dy = dynamic_sched(seqs)
    co = dynamic_sched(seqs, coop_leaf=True)
    print(f"rays {len(seqs)}  visits/ray {np.mean([len(s) for s in seqs]):.1f}  "
          f"leaf size/visit {np.mean([v[1] for s in seqs for v in s]):.1f}  "
          f"descent/visit {np.mean([v[0] for s in seqs for v in s]):.2f}")
    print(f"utilization  static {per_lane / st:.3f}  dynamic-fetch {per_lane / dy:.3f}  "
          f"dynamic+coop-leaf {per_lane / co:.3f}")
    for K in (2, 4, 8, 64):
        print(f"  postponed K={K}: " + "  ".join(f"T={T} {per_lane / postponed_sched(seqs, K, T):.3f}"
                                                for T in (16, 32, 48, 64)))


if __name__ == "__main__":
    main()
