"""Driver for tools/leaf_cull_probe.c: dumps a scene's reference-layout KD
tree / indices / triangles and a ray list (rays from the camera position in
random directions, plus diffuse-like bounce rays from their hit points), then
runs the probe.  usage: python tools/leaf_cull_probe.py SCENE [MARGIN] [N]
(MARGIN < 0: the product's leaf-box growth and float slab test, coop_trace.h leaf_box_maybe)"""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("isaklm-raytracer_amd", "tests", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import helpers  # noqa: E402
import oracle  # noqa: E402


def main():
    scene = sys.argv[1] if len(sys.argv) > 1 else "room2m"
    margin = sys.argv[2] if len(sys.argv) > 2 else "0.001"
    N = int(sys.argv[3]) if len(sys.argv) > 3 else 20000
    osc = oracle.OracleScene(helpers.scene_path(scene))
    tris, nodes, idx, _, bounds = osc.arrays()
    g = np.random.default_rng(5)
    cam = np.asarray(osc.camera[:3], np.float32)
    d = g.normal(size=(N, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    prim = np.concatenate([np.repeat(cam[None], N, 0), d], 1).astype(np.float32)
    h = osc.trace_rays(prim)
    ok = h[:, 0] == 1
    pos, nrm = h[ok, 2:5], h[ok, 5:8]
    b = g.normal(size=pos.shape).astype(np.float32)
    b /= np.linalg.norm(b, axis=1, keepdims=True)
    b = np.where((b * nrm).sum(1, keepdims=True) < 0, -b, b) + nrm
    b /= np.linalg.norm(b, axis=1, keepdims=True)
    sec = np.concatenate([pos, b], 1).astype(np.float32)
    rays = np.concatenate([prim, sec]).astype(np.float32)
    with tempfile.TemporaryDirectory() as t:
        paths = [os.path.join(t, n) for n in ("nodes", "idx", "tris", "rays")]
        for pth, data in zip(paths, (nodes, idx.astype(np.int32).tobytes(), tris, rays.tobytes())):
            open(pth, "wb").write(data)
        exe = os.path.join(t, "probe")
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fopenmp", os.path.join(ROOT, "tools", "leaf_cull_probe.c"), "-o", exe, "-lm"],
                       check=True)
        print(subprocess.run([exe, *paths, margin], check=True, capture_output=True, text=True).stdout.strip())


if __name__ == "__main__":
    main()
