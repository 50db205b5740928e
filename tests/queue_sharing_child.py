"""Child process of test_gpu_parity.test_long_handoff_with_shared_hw_queues.

Occupies the process's hardware queues with extra streams BEFORE the
library creates its pipeline streams (as RCCL's streams do in a multi-GPU
bench), so the runtime must map the caller's stream and pipeline streams onto
shared hardware queues.  The wf_long slices must neither deadlock nor change
a bit.  Prints "OK" on success.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, os.path.join(ROOT, "isaklm-raytracer_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import helpers  # noqa: E402
import rt  # noqa: E402


def main():
    torch.cuda.set_device(0)
    streams = [torch.cuda.Stream() for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 8)]
    keep = []
    for s in streams:  # a launch on every stream makes the runtime bind it to a hardware queue
        with torch.cuda.stream(s):
            keep.append(torch.ones(1024, device="cuda") * 2)
    torch.cuda.synchronize()
    run = helpers.GpuRun("room_small")
    W, H, P = 48, 27, 3
    gpu, gcnt, _ = run.render(W, H, P, calls=2, count=True, kernel=rt.KERNEL_WAVEFRONT, wf_long_depth=1,
                              wf_pipelines=3)
    ref, rcnt = helpers.oracle_render(run.path, W, H, P, calls=2)
    helpers.assert_bitwise(gpu, ref, what="shared hardware queues")
    assert gcnt == rcnt, (gcnt, rcnt)
    print("OK", flush=True)


if __name__ == "__main__":
    main()
