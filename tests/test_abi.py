"""The C-ABI library (CPU only): it loads without a GPU, exports every
function include/isaklm_rt.h declares, its structs have the reference's byte
layout, and argument errors are reported, not crashed on."""
import ctypes
import os
import re
import subprocess

import pytest

import rt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "isaklm_rt.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", text)))


def test_exports_every_declared_symbol():
    names = declared_functions()
    assert len(names) >= 30
    out = subprocess.run(["nm", "-D", "--defined-only", rt.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (rt_\w+)", out))
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    lib = rt.lib()
    for n in names:
        getattr(lib, n)


def test_struct_layouts_match_reference():
    # sizes from SURVEY §8b (measured on the reference with g++ x86-64)
    assert ctypes.sizeof(rt.Camera) == 28
    assert ctypes.sizeof(rt.G_Buffer) == 32
    assert ctypes.sizeof(rt.Scene) == 72
    assert ctypes.sizeof(rt.KD_Tree) == 40
    assert rt.Scene.light_indicies.offset == 16 and rt.Scene.kd_tree.offset == 32
    assert rt.Camera.FOV.offset == 20
    assert rt.TRIANGLE_BYTES == 152 and rt.NODE_BYTES == 20


def test_header_compiles_as_c_and_cpp(tmp_path):
    src = tmp_path / "t.c"
    src.write_text('#include "isaklm_rt.h"\n'
                   "_Static_assert(sizeof(Triangle) == 152, \"t\");\n"
                   "_Static_assert(sizeof(Material) == 56, \"m\");\n"
                   "_Static_assert(sizeof(KD_Tree_Node) == 20, \"n\");\n"
                   "int main(void){ RtOptions o; rt_default_options(&o); return o.width == 1920 ? 0 : 1; }\n")
    inc = os.path.join(ROOT, "include")
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-I", inc, "-c", str(src), "-o", str(tmp_path / "t.o")],
                   check=True)
    cpp = tmp_path / "t.cpp"
    cpp.write_text('#include "isaklm_rt.h"\nint main(){ return sizeof(Scene) == 72 ? 0 : 1; }\n')
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-I", inc, "-c", str(cpp), "-o", str(tmp_path / "u.o")],
                   check=True)


def test_default_options_are_the_reference_macros():
    o = rt.RtOptions()
    rt.lib().rt_default_options(ctypes.byref(o))
    assert (o.width, o.height, o.passes, o.adaptive, o.min_samples) == (1920, 1080, 1, 1, 100)
    assert abs(o.tolerance - 0.05) < 1e-9 and o.max_depth == 0


def test_argument_errors_are_reported():
    L = rt.lib()
    o = rt.RtOptions()
    L.rt_default_options(ctypes.byref(o))
    rc = L.rt_render(None, rt.G_Buffer(), rt.Camera(), 0, ctypes.byref(o))
    assert rc == -1 and b"null" in L.rt_last_error()
    assert L.rt_gbuffer_create(0, 10, 0, ctypes.byref(rt.G_Buffer())) == -1
    assert L.rt_generate_scene(b"no_such_scene", b"/tmp", None, 0) == -1
    assert L.rt_build_kd_tree(None, 0, None, None, None, None, None) == -1


def test_version_string():
    assert b"gfx950" in rt.lib().rt_version()


def test_ctypes_binding_matches_header_layout(tmp_path):
    """rt.py's RtOptions / RtProfile / RtDeviations must mirror
    include/isaklm_rt.h field by field: compile a probe with gcc and compare
    every offset and the size."""
    structs = {"RtOptions": rt.RtOptions, "RtProfile": rt.RtProfile, "RtDeviations": rt.RtDeviations}
    lines = ['#include <stddef.h>', '#include <stdio.h>', '#include "isaklm_rt.h"', "int main(void){"]
    for cname, cls in structs.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in cls._fields_:
            lines.append(f'printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0;}")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines) + "\n")
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    for line in filter(None, out):
        cname, fname, val = line.split()
        cls = structs[cname]
        want = ctypes.sizeof(cls) if fname == "size" else getattr(cls, fname).offset
        assert int(val) == want, (cname, fname, int(val), want)


def test_gbuffer_checkpoint_errors(tmp_path):
    """rt_gbuffer_load rejects what is not a matching checkpoint before touching
    the device (no GPU needed)."""
    import struct

    L = rt.lib()
    g = rt.G_Buffer()
    sc = ctypes.c_int()
    assert L.rt_gbuffer_load(str(tmp_path / "missing.gbuf").encode(), g, 4, 4, ctypes.byref(sc)) == -3
    (tmp_path / "junk.gbuf").write_bytes(b"not a checkpoint at all")
    assert L.rt_gbuffer_load(str(tmp_path / "junk.gbuf").encode(), g, 4, 4, ctypes.byref(sc)) == -4
    (tmp_path / "other.gbuf").write_bytes(b"RTGBUF01" + struct.pack("<4i", 5, 5, 7, 0) + bytes(25 * 24))
    assert L.rt_gbuffer_load(str(tmp_path / "other.gbuf").encode(), g, 4, 4, ctypes.byref(sc)) == -1  # RT_E_INVALID


MAIN_SHAPE = os.path.join(ROOT, "tests", "native", "ref_main_shape.cpp")


def build_main_shape(out_dir):
    """Compile + link the reference-main-shaped TU (its own reference-layout
    types, then isaklm_rt.h with ISAKLM_RT_CALLER_TYPES) against the library."""
    exe = os.path.join(str(out_dir), "ref_main_shape")
    lib_dir = os.path.dirname(rt.LIB_PATH)
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), MAIN_SHAPE,
                    "-o", exe, "-L", lib_dir, "-lisaklm_rt", "-Wl,-rpath," + lib_dir,
                    "-Wl,-rpath,/opt/rocm/lib"], check=True, capture_output=True, text=True)
    return exe


def test_reference_shaped_main_compiles_and_links(tmp_path):
    """INTEGRATION.md's drop-in: a TU that already defines the reference's
    Vec2D / Vec3D / Texture / Material / Triangle / KD_Tree_Node /
    Bounding_Box / KD_Tree / Scene / G_Buffer / Camera (anonymous unions,
    constructors, member functions as in rt/*.cuh) includes isaklm_rt.h after
    them with ISAKLM_RT_CALLER_TYPES: it compiles (the header's static_asserts
    check the caller's layouts), links, and runs up to its usage check."""
    exe = build_main_shape(tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "usage: ref_main_shape" in r.stderr


def test_caller_types_layout_mismatch_is_a_compile_error(tmp_path):
    """A caller type with another layout (Camera without aperture_radius)
    fails the header's static_asserts instead of corrupting rt_render's
    arguments at run time."""
    src = tmp_path / "bad.cpp"
    src.write_text(open(MAIN_SHAPE).read().replace("    float FOV;\n    float aperture_radius;\n", "    float FOV;\n"))
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I", os.path.join(ROOT, "include"), str(src)],
                       capture_output=True, text=True)
    assert r.returncode != 0 and "Camera" in r.stderr


def test_abi_version_matches_header():
    import re as _re

    text = open(HEADER).read()
    assert rt.lib().rt_abi_version() == int(_re.search(r"#define RT_ABI_VERSION (\d+)", text).group(1)) == rt.ABI_VERSION
