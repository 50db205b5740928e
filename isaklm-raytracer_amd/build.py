"""Builds the in-tree HIP library libisaklm_rt.so for gfx950 (and nothing else).

Host C++ (scene loading, exact KD build, prepare) is compiled by g++, the
kernels and the C-ABI by hipcc --offload-arch=gfx950; everything with
-ffp-contract=off so host-precomputed constants and
GPU arithmetic round identically.  Rebuilds only what changed.
"""
import glob
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libisaklm_rt.so")
APP = os.path.join(HERE, "rt_render")  # C++ driver binary (apps/rt_render_main.cpp)
ROOT = os.path.dirname(HERE)
INCLUDE = os.path.join(ROOT, "include")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")

HOST_SOURCES = ["host/mesh_loading.cpp", "host/kd_build.cpp", "host/scene_prepare.cpp", "host/misc.cpp", "host/image_decode.cpp",
                "host/scenes.cpp", "host/bvh_build.cpp"]
HIP_SOURCES = ["path_kernel.hip", "wavefront.hip", "abi.hip", "shards.hip"]
# every header under csrc/ (a header missing here would not trigger a rebuild)
HEADERS = sorted(os.path.relpath(f, os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc"))
                 for f in glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc", "**", "*.h"),
                                    recursive=True))

COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-I" + INCLUDE, "-I" + CSRC]
# -fwrapv: the JPEG IDCT wraps on corrupt coefficients as stb_image's does on
# the reference's x86 build, instead of signed-overflow UB
HOST_FLAGS = ["-fopenmp", "-Wall", "-Wno-unused-function", "-fwrapv"]
HIP_FLAGS = ["--offload-arch=gfx950", "-fno-gpu-rdc", "-munsafe-fp-atomics", "-Wno-unused-command-line-argument"]


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("build failed: " + " ".join(cmd[:2]) + " ...")
    elif verbose and (r.stdout or r.stderr):
        sys.stderr.write(r.stdout + r.stderr)


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


STAMP = LIB + ".stamp"


def _digest(extra_hip_flags):
    h = hashlib.sha256()
    files = [os.path.join(CSRC, f) for f in HOST_SOURCES + HIP_SOURCES + HEADERS] + [
        os.path.join(INCLUDE, "isaklm_rt.h"), os.path.join(HERE, "apps", "rt_render_main.cpp")]
    for f in files:
        with open(f, "rb") as fh:
            h.update(os.path.relpath(f, ROOT).encode() + fh.read())
    flags = [x for x in COMMON + HOST_FLAGS + HIP_FLAGS + list(extra_hip_flags) if not x.startswith("-I")]
    h.update(" ".join(flags).encode())
    return h.hexdigest()


def build(verbose=False, extra_hip_flags=()):
    """Builds libisaklm_rt.so unless the stamp shows it was built from these exact sources."""
    digest = _digest(extra_hip_flags)
    if os.path.exists(LIB) and os.path.exists(APP) and os.path.exists(STAMP) and open(STAMP).read().strip() == digest:
        return LIB
    os.makedirs(BUILD, exist_ok=True)
    headers = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(INCLUDE, "isaklm_rt.h")]
    objs = []
    for src in HOST_SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(BUILD, os.path.basename(src) + ".o")
        if _stale(o, [s] + headers):
            _run(["g++"] + COMMON + HOST_FLAGS + ["-c", s, "-o", o], verbose)
        objs.append(o)
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    # the HIP objects remember the extra flags they were compiled with: a build
    # with other flags (an A/B variant, or the default after one) recompiles
    # them all even though their sources are older than the objects
    flags_file = os.path.join(BUILD, "hip_flags")
    want = " ".join(extra_hip_flags)
    have = open(flags_file).read() if os.path.exists(flags_file) else None
    for src in HIP_SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(BUILD, os.path.basename(src) + ".o")
        if _stale(o, [s] + headers) or have != want:
            _run([hipcc] + COMMON + HIP_FLAGS + list(extra_hip_flags) + ["-c", s, "-o", o], verbose)
        objs.append(o)
    with open(flags_file, "w") as fh:
        fh.write(want)
    if _stale(LIB, objs):
        _run(["g++", "-shared", "-o", LIB] + objs +
             ["-L" + os.path.join(ROCM, "lib"), "-lamdhip64", "-lrccl", "-fopenmp",
              "-Wl,-rpath," + os.path.join(ROCM, "lib")], verbose)
    # the C++ driver (the reference's main() without GLFW) over the C-ABI
    app_src = os.path.join(HERE, "apps", "rt_render_main.cpp")
    if _stale(APP, [LIB, app_src, os.path.join(INCLUDE, "isaklm_rt.h")]):
        _run(["g++", "-O2", "-std=c++17", "-Wall", "-I" + INCLUDE, app_src, "-o", APP, "-L" + HERE, "-lisaklm_rt",
              "-Wl,-rpath,$ORIGIN", "-Wl,-rpath," + os.path.join(ROCM, "lib")], verbose)
    with open(STAMP, "w") as fh:
        fh.write(digest + "\n")
    return LIB


if __name__ == "__main__":
    print(build(verbose=True))
