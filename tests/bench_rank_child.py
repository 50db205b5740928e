"""TEST INFRASTRUCTURE: one rank of bench.py's multi-rank branch over the
CPU stand-in binding (tests/bench_stub_rt.py); RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT come from the environment as under
torch.distributed.run."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "isaklm-raytracer_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

import bench  # noqa: E402
import bench_stub_rt  # noqa: E402

if __name__ == "__main__":
    sys.exit(bench.main(sys.argv[1:], binding=bench_stub_rt))
