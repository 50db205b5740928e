"""Render a scene's frame with the bounded traversal and the run-time guard on
every ray (check_interval 1) and print the guard's statistics: the first
mismatching ray (o, d as hex floats) is what tests/native/bvh_trace_check's
`ray` mode replays on the host.  usage: python tools/mismatch_ray.py SCENE|adversarial:VARIANT [W H P]"""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "isaklm-raytracer_amd"), os.path.join(ROOT, "oracle")]
import hazards  # noqa: E402
import helpers  # noqa: E402
import rt  # noqa: E402

arg = sys.argv[1]
W, H, P = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (320, 240, 4)
path = hazards.adversarial_scene(tempfile.mkdtemp(), arg.split(":")[1]) if arg.startswith("adversarial:") else \
    helpers.scene_path(arg)
run = helpers.GpuRun(path)
rt.deviation_stats(reset=True)
run.render(W, H, [P, P], kernel=rt.KERNEL_WAVEFRONT, traversal=rt.TRAVERSAL_BOUNDED, check_interval=1)
dev = rt.deviation_stats(reset=True)
print("checked", dev["bounded_checked"], "mismatches", dev["bounded_mismatches"])
print("ray", " ".join(float(v).hex() for v in dev["mismatch_ray"]))
