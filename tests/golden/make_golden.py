"""Regenerates tests/golden/oracle_regression.json.

The reference cannot be built in this image (it needs the CUDA toolkit and
GLFW/GL headers; see oracle/rt_oracle.h), so these vectors come from the CPU
oracle (oracle/rt_oracle.c) and pin it against regressions; the GPU tests
check the HIP path against the same vectors.  The reference-owned fixtures
are the material files in tests/golden/materials/ (copied data) and the
known answers quoted in tests/test_oracle.py.

usage: python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in ("isaklm-raytracer_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))

import helpers  # noqa: E402
import oracle  # noqa: E402

CASES = [
    # scene, W, H, passes, calls, adaptive, min_samples, max_depth, seed_skip
    ("cornell", 32, 32, 4, 1, False, 100, 0, 0),
    ("cornell", 24, 20, 12, 2, True, 5, 0, 0),
    ("cornell", 17, 13, 3, 1, False, 100, 2, 7 * 17 * 13),
    ("cornell_blob", 32, 18, 2, 1, False, 100, 0, 0),
    ("room_small", 32, 18, 2, 1, False, 100, 0, 0),
]


def sha(b):
    return hashlib.sha256(b).hexdigest()


def accum_digest(fb, sq, cnt, rng):
    return sha(np.ascontiguousarray(fb, np.float32).tobytes() + np.ascontiguousarray(sq, np.float32).tobytes() +
               np.ascontiguousarray(cnt, np.int32).tobytes() + np.ascontiguousarray(rng, np.uint32).tobytes())


def case_key(c):
    return "{}_{}x{}_p{}_c{}_a{}_m{}_d{}_s{}".format(*c)


def main():
    out = {"scenes": {}, "renders": {}}
    for name in ("cornell", "cornell_blob", "room_small"):
        sc = oracle.OracleScene(helpers.scene_path(name))
        tris, nodes, idx, lights, bounds = sc.arrays()
        out["scenes"][name] = {"triangles": sc.ntris, "nodes": sc.nnodes, "indices": sc.nindices,
                               "lights": sc.nlights, "triangles_sha256": sha(tris), "nodes_sha256": sha(nodes),
                               "indices_sha256": sha(idx.tobytes()), "bounds": [float(b) for b in bounds]}
    for c in CASES:
        name, W, H, P, calls, adaptive, ms, md, skip = c
        (fb, sq, cnt, rng), counters = helpers.oracle_render(helpers.scene_path(name), W, H, P, calls=calls,
                                                             adaptive=adaptive, min_samples=ms, max_depth=md,
                                                             seed_skip=skip)
        out["renders"][case_key(c)] = {"case": list(c), "sha256": accum_digest(fb, sq, cnt, rng),
                                      "counters": counters, "sum_count": int(cnt.sum()),
                                      "mean_radiance": float(fb.sum() / max(cnt.sum(), 1))}
    with open(os.path.join(HERE, "oracle_regression.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", os.path.join(HERE, "oracle_regression.json"))


if __name__ == "__main__":
    main()
