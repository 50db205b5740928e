"""Second, independent restatement of the rest of the render hot path (TEST
INFRASTRUCTURE ONLY), written directly from the reference source in numpy
float32 scalars, without looking at or calling oracle/rt_oracle.c — the
counterpart of tests/independent.py (which restates the BSDF, NEE and the KD
builder; this module uses those, and restates everything between them):

  * camera ray + random_point_in_pinhole   rt/path_tracing.cuh:327-336,381-391
    with Camera::rotation / rotation_matrix rt/camera.cuh:22-25,
                                           rt/math_library.cuh:337-408
  * the adaptive-sampling test             rt/path_tracing.cuh:352-376
  * trace_path (emission rule, NEE after   rt/path_tracing.cuh:268-325
    diffuse events, roulette, accumulation)
  * trace_ray traversal                    rt/trace_ray.cuh:174-318
    (ray_behind_plane, intersect_plane, intersect_bounding_box, the
     node / entry / exit stack, first leaf with a hit wins)
  * trace_leaf_node + intersect_triangle   rt/trace_ray.cuh:48-172
    + calculate_barycentric_coordinates
  * sample_texture (texel index)           rt/trace_ray.cuh:31-46,
                                           mod rt/math_library.cuh:32-35

Inputs: reference-layout triangles (152 B, from the product's loader), the KD
tree from independent.create_kd_tree, G-buffer seeds from numpy's own
MT19937 (RandomState(5489), the std::mt19937 default seed).  Conventions the
build defines where the reference reads out of bounds (both sides): a light
pick with xi == 1.0 takes the last light; a texel index past the
image reads 0 (the w + 1 zero texels after each texture).
Scalar Python: for frames of a few hundred samples.
"""
import struct

import numpy as np

import independent as ind

f32 = np.float32
PRIMARY, DIFFUSE = 0, 1  # Ray_Type (rt/path_tracing.cuh:18-25)


def reference_seeds(n, skip=0):
    """G_Buffer seeds (rt/screen.cuh:34-45): std::mt19937 with its default
    seed 5489, uniform_int_distribution<uint32_t>(0, UINT32_MAX) = the raw
    words — numpy's legacy MT19937 seeding is init_genrand(5489), and a
    full-range uint32 draw takes one raw word each"""
    rs = np.random.RandomState(5489)
    return rs.randint(0, 1 << 32, size=skip + n, dtype=np.uint64).astype(np.uint32)[skip:]


# ------------------------------------------------------------ scalar math
def v(x, y, z):
    return (f32(x), f32(y), f32(z))


def add(a, b):
    return (a[0] + b[0], a[1] + b[1], a[2] + b[2])


def sub(a, b):
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def mul(a, b):  # component-wise Vec3D * Vec3D
    return (a[0] * b[0], a[1] * b[1], a[2] * b[2])


def scale(s, a):  # float * Vec3D
    return (s * a[0], s * a[1], s * a[2])


def dot(a, b):
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]


def cross(a, b):
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


def normalize(a):
    r = f32(1) / np.sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2])
    return (a[0] * r, a[1] * r, a[2] * r)


def luminance(c):  # rt/math_library.cuh:263-266
    return dot(c, v(0.2126, 0.7152, 0.0722))


def mat_vec(m, x):
    """Matrix3X3 * Vec3D = x.x * i + x.y * j + x.z * k (rt/math_library.cuh:348-351)"""
    return add(add(scale(x[0], m[0]), scale(x[1], m[1])), scale(x[2], m[2]))


def mat_mat(m2, m1):
    return (mat_vec(m2, m1[0]), mat_vec(m2, m1[1]), mat_vec(m2, m1[2]))


def rotation_matrix(yaw, pitch):
    """rt/math_library.cuh:384-408 with roll 0; cos / sin of float arguments"""
    cy, sy = ind.cosf(yaw)[()], ind.sinf(yaw)[()]
    cp, sp = ind.cosf(pitch)[()], ind.sinf(pitch)[()]
    c0, s0 = ind.cosf(f32(0))[()], ind.sinf(f32(0))[()]
    y_rot = ((cy, f32(0), -sy), (f32(0), f32(1), f32(0)), (sy, f32(0), cy))
    x_rot = ((f32(1), f32(0), f32(0)), (f32(0), cp, sp), (f32(0), -sp, cp))
    z_rot = ((c0, s0, f32(0)), (-s0, c0, f32(0)), (f32(0), f32(0), f32(1)))
    return mat_mat(mat_mat(z_rot, y_rot), x_rot)


def rng_draw(state):
    """get_random_unilateral (rt/path_tracing.cuh:34-43) on a Python int"""
    s = (state * 747796405 + 2891336453) & 0xFFFFFFFF
    w = (((s >> ((s >> 28) + 4)) ^ s) * 277803737) & 0xFFFFFFFF
    r = ((w >> 22) ^ w) & 0xFFFFFFFF
    return f32(r) / f32(4294967295.0), r


def erfinvf(x):
    from scipy.special import erfinv

    return f32(erfinv(np.float64(x)))


# ------------------------------------------------------------ scene
class Scene:
    """Reference-layout triangles (n, 152) uint8 + the independent KD tree."""

    def __init__(self, tri_bytes, textures=None):
        self.raw = np.frombuffer(tri_bytes, np.uint8).reshape(-1, 152)
        n = len(self.raw)
        fl = self.raw[:, :96].copy().view(f32).reshape(n, 24)
        self.P = [tuple((f32(a), f32(b), f32(c)) for a, b, c in fl[i, :9].reshape(3, 3)) for i in range(n)]
        self.N = [tuple((f32(a), f32(b), f32(c)) for a, b, c in fl[i, 9:18].reshape(3, 3)) for i in range(n)]
        self.UV = [tuple((f32(a), f32(b)) for a, b in fl[i, 18:24].reshape(3, 2)) for i in range(n)]
        m = self.raw[:, 96:136].copy().view(f32).reshape(n, 10)
        self.albedo = [tuple(f32(x) for x in m[i, 0:3]) for i in range(n)]
        self.emit = [tuple(f32(x) for x in m[i, 3:6]) for i in range(n)]
        self.rough = [f32(m[i, 6]) for i in range(n)]
        self.ior = [f32(m[i, 7]) for i in range(n)]
        self.ext = [f32(m[i, 8]) for i in range(n)]
        self.transparent = [bool(self.raw[i, 132]) for i in range(n)]
        tex = self.raw[:, 136:152].copy()
        self.tex_key = [int.from_bytes(tex[i, 0:8].tobytes(), "little") for i in range(n)]
        self.tex_wh = [struct.unpack("<ii", tex[i, 8:16].tobytes()) for i in range(n)]
        self.textures = textures or {}  # texture pointer -> (h, w, 4) uint8
        nodes, self.indices, bounds = ind.create_kd_tree(self.raw)
        self.nodes = [struct.unpack("<iiB3xf?3x", nodes[k:k + 20]) for k in range(0, len(nodes), 20)]
        self.bmin = tuple(f32(x) for x in bounds[:3])
        self.bmax = tuple(f32(x) for x in bounds[3:])
        self.lights = [i for i in range(n) if any(e > 0 for e in self.emit[i])]  # rt/create_scene.cuh:40-64

    # ---- sample_texture (rt/trace_ray.cuh:31-46)
    def sample_texture(self, tri, blend, uv):
        key = self.tex_key[tri]
        if key == 0 or key not in self.textures:
            return blend
        img = self.textures[key]
        w, h = self.tex_wh[tri]
        u = uv[0] - f32(1) * np.floor(uv[0] / f32(1))  # mod(x, 1) = x - 1 * floorf(x / 1)
        vv = uv[1] - f32(1) * np.floor(uv[1] / f32(1))
        # int(v * h) * w is an int; + (u * w) makes the sum a float; the assignment truncates
        idx = int(f32(f32(int(vv * f32(h)) * w) + u * f32(w)))
        flat = img.reshape(-1, 4)
        c = flat[idx] if idx < len(flat) else np.zeros(4, np.uint8)  # the zero pad past the image (H10)
        col = (f32(c[0]) / f32(255), f32(c[1]) / f32(255), f32(c[2]) / f32(255))
        return mul(col, blend)

    # ---- intersect_triangle + barycentrics (rt/trace_ray.cuh:48-113)
    def intersect_triangle(self, o, d, tri):
        p1, p2, p3 = self.P[tri]
        with np.errstate(all="ignore"):
            nrm = normalize(cross(sub(p2, p1), sub(p3, p1)))
            ddn = dot(d, nrm)
            if ddn == 0:
                return False, None, None
            s = (dot(nrm, p1) - dot(o, nrm)) / ddn
            if s < f32(0.00001):
                return False, None, None
            p = add(o, scale(s, d))
            v0, v1, v2 = sub(p2, p1), sub(p3, p1), sub(p, p1)
            d00, d01, d11 = dot(v0, v0), dot(v0, v1), dot(v1, v1)
            d20, d21 = dot(v2, v0), dot(v2, v1)
            rden = f32(1) / (d00 * d11 - d01 * d01)
            by = (d11 * d20 - d01 * d21) * rden
            bz = (d00 * d21 - d01 * d20) * rden
            bx = f32(1) - by - bz
        inside = f32(0) <= bx <= f32(1) and f32(0) <= by <= f32(1) and f32(0) <= bz <= f32(1)
        return inside, s, (bx, by, bz)

    # ---- trace_leaf_node (rt/trace_ray.cuh:115-172)
    def trace_leaf(self, o, d, max_t, off, count):
        smallest, best, bary = max_t, -1, None
        for k in range(off, off + count):
            tri = int(self.indices[k])
            ok, t, b = self.intersect_triangle(o, d, tri)
            if ok and t < smallest:
                smallest, best, bary = t, tri, b
        if best < 0:
            return None
        bx, by, bz = bary
        uv1, uv2, uv3 = self.UV[best]
        uv = ((uv1[0] * bx + uv2[0] * by) + uv3[0] * bz, (uv1[1] * bx + uv2[1] * by) + uv3[1] * bz)
        p1, p2, p3 = self.P[best]
        n1, n2, n3 = self.N[best]
        s = {"tri": best,
             "albedo": self.sample_texture(best, self.albedo[best], uv),
             "emittance": self.sample_texture(best, self.emit[best], uv),
             "position": add(add(scale(bx, p1), scale(by, p2)), scale(bz, p3))}
        nrm = normalize(add(add(scale(bx, n1), scale(by, n2)), scale(bz, n3)))
        s["tangent"] = normalize(cross(sub(p2, p1), nrm))
        s["bitangent"] = normalize(cross(nrm, s["tangent"]))
        if dot(d, nrm) > 0:
            nrm = (-nrm[0], -nrm[1], -nrm[2])
        s["normal"] = nrm
        return s

    # ---- trace_ray (rt/trace_ray.cuh:212-318)
    def trace_ray(self, o, d):
        with np.errstate(all="ignore"):
            tmin = [(self.bmin[a] - o[a]) / d[a] for a in range(3)]
            tmax = [(self.bmax[a] - o[a]) / d[a] for a in range(3)]
        s1 = [np.fmin(tmin[a], tmax[a]) for a in range(3)]
        s2 = [np.fmax(tmin[a], tmax[a]) for a in range(3)]
        t1 = np.fmax(np.fmax(s1[0], s1[1]), s1[2])
        t2 = np.fmin(np.fmin(s2[0], s2[1]), s2[2])
        if not t1 <= t2:
            return None
        stack = [(0, t1, t2)]
        while stack:
            idx, entry, exit_ = stack.pop()
            a, b, axis, off, leaf = self.nodes[idx]
            while not leaf:
                near, far = (b, a) if o[axis] >= f32(off) else (a, b)  # ray_behind_plane (:174-188)
                with np.errstate(all="ignore"):
                    t = (f32(off) - o[axis]) / d[axis]  # intersect_plane (:190-210)
                if t >= exit_ or t < 0:
                    nxt = near
                elif t <= entry:
                    nxt = far
                else:
                    stack.append((far, t, exit_))
                    nxt = near
                    exit_ = t
                a, b, axis, off, leaf = self.nodes[nxt]
            if b > 0:
                s = self.trace_leaf(o, d, exit_, a, b)
                if s is not None:
                    return s
        return None

    # ---- sample_direct_light's ray query (independent.direct_light's `trace`)
    def trace_batch(self, rays6):
        hit, tri, nrm, emit = [], [], [], []
        zero = (f32(0), f32(0), f32(0))
        for r in rays6:
            s = self.trace_ray(tuple(f32(x) for x in r[:3]), tuple(f32(x) for x in r[3:]))
            hit.append(s is not None)
            tri.append(s["tri"] if s else -1)
            nrm.append(s["normal"] if s else zero)
            emit.append(s["emittance"] if s else zero)
        return np.array(hit), np.array(tri), np.array(nrm, f32), np.array(emit, f32)

    # ---- trace_path (rt/path_tracing.cuh:268-325); returns (L, rng)
    def trace_path(self, o, d, rng):
        L = v(0, 0, 0)
        T = v(1, 1, 1)
        inside = False
        typ = PRIMARY
        while True:
            s = self.trace_ray(o, d)
            if s is None:
                break
            if typ != DIFFUSE:
                L = add(L, mul(s["emittance"], T))
            a = lambda x: np.array([x], f32)  # noqa: E731  (independent.scatter works on arrays)
            pos, nd, w, t, ins, r = ind.scatter(
                a(d), np.array([inside]), np.array([rng], np.uint32), a(s["albedo"]), a(self.rough[s["tri"]]),
                a(self.ior[s["tri"]]), a(self.ext[s["tri"]]), np.array([self.transparent[s["tri"]]]), a(s["position"]),
                a(s["normal"]), a(s["tangent"]), a(s["bitangent"]))
            typ, inside, rng = int(t[0]), bool(ins[0]), int(r[0])
            o = s["position"]
            d = tuple(f32(x) for x in nd[0])
            T = mul(T, tuple(f32(x) for x in w[0]))
            if typ == DIFFUSE:
                lights = np.array(self.lights, np.int64)
                direct, r2 = ind.direct_light(self.raw, lights, self.trace_batch, a(o), a(s["normal"]),
                                              np.array([rng], np.uint32))
                rng = int(r2[0])
                L = add(L, mul(tuple(f32(x) for x in direct[0]), T))
            p = np.fmax(T[0], np.fmax(T[1], T[2]))
            xi, rng = rng_draw(rng)
            if xi > p:
                break
            T = scale(f32(1) / p, T)
        return L, rng


# ------------------------------------------------------------ path_tracing kernel
def render(scene, camera, W, H, passes, fb, sq, cnt, rng, adaptive=False, min_samples=100, tolerance=f32(0.05)):
    """path_tracing (rt/path_tracing.cuh:338-395) for `passes` passes on
    G_Buffer-layout arrays (fb (n, 3) float32, sq, cnt, rng), in place"""
    pos = tuple(f32(x) for x in camera[:3])
    yaw, pitch, fov, aperture = (f32(x) for x in camera[3:7])
    R = rotation_matrix(yaw, pitch)
    tan_half = f32(np.tan(np.float64(fov / f32(2))))  # tanf(camera.FOV / 2), correctly rounded
    z = np.sqrt(f32(2)) * erfinvf(f32(1) - f32(tolerance))
    hw, hh = W // 2, H // 2  # SCREEN_W / 2, SCREEN_H / 2 (int)
    for _ in range(passes):
        for y in range(H):
            for x in range(W):
                i = y * W + x
                n = int(cnt[i])
                run = True
                if adaptive and n >= min_samples:
                    tl = luminance(tuple(fb[i]))
                    mean = tl / f32(n)
                    var = (sq[i] - (tl * tl) / f32(n)) / f32(n - 1)
                    iw = z * np.sqrt(var / f32(n))
                    run = bool(iw > mean * f32(tolerance))
                if not run:
                    continue
                st = int(rng[i])
                rx, st = rng_draw(st)
                ry, st = rng_draw(st)
                dx = tan_half * (f32(f32(x) + rx) - f32(hw)) / f32(hw)
                dy = tan_half * (f32(f32(y) + ry) - f32(hh)) / f32(hw)
                d = mat_vec(R, normalize((dx, dy, f32(1))))
                th, st = rng_draw(st)
                theta = th * ind.TAU
                rr, st = rng_draw(st)
                r = np.sqrt(rr) * aperture
                ox = r * ind.cosf(theta)[()]
                oy = r * ind.sinf(theta)[()]
                o = add(add(pos, mat_vec(R, (ox, f32(0), f32(0)))), mat_vec(R, (f32(0), oy, f32(0))))
                L, st = scene.trace_path(o, d, st)
                fb[i] = np.array(add(tuple(fb[i]), L), f32)  # frame_buffer += L
                lum = luminance(L)
                sq[i] = sq[i] + lum * lum
                cnt[i] += 1
                rng[i] = st
