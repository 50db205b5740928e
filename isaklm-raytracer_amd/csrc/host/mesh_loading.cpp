// mesh_loading.cpp — OBJ + .mat loading, restating rt/mesh_loading.cuh.
//
// Same tokenisation (split on ' ' only, empty tokens dropped; '/'-split keeps
// empty middle tokens, rt/mesh_loading.cuh:73-103), same float parsing
// (std::stof == strtof, correctly rounded), same fan triangulation, face
// normals, smooth normals, ZERO_VEC2D = {1,1} default UVs,
// re-centring on the mesh AABB and M*p + offset transform.  The parser reads
// the file in one block instead of std::getline + std::list, which makes the
// 2M-triangle OBJ load in well under a second.
#include <errno.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <cfloat>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "rt_host.h"

namespace rt_host {
namespace {

bool read_file(const std::string &path, std::string &out)
{
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) return false;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    out.resize(n > 0 ? (size_t)n : 0);
    size_t got = n > 0 ? fread(&out[0], 1, (size_t)n, f) : 0;
    fclose(f);
    return got == out.size();
}

// split_string(line, ' ') with include_empty = false (rt/mesh_loading.cuh:73-103):
// tokens are the maximal runs of non-' ' characters.  Tokens are written
// NUL-terminated into `scratch` so strtof/strtol can parse them.
struct Tokens {
    std::vector<const char *> t;
    std::string scratch;
    void split(const char *b, const char *e)
    {
        t.clear();
        scratch.assign(b, e);
        scratch.push_back(' ');
        char *s = &scratch[0];
        size_t n = scratch.size();
        size_t i = 0;
        while (i < n) {
            while (i < n && s[i] == ' ') ++i;
            if (i >= n) break;
            size_t j = i;
            while (j < n && s[j] != ' ') ++j;
            s[j] = 0;
            t.push_back(s + i);
            i = j + 1;
        }
    }
};

bool parse_float(const char *s, float &v)
{
    char *end;
    v = strtof(s, &end); // std::stof (rt/mesh_loading.cuh:260-286)
    return end != s;
}
bool parse_int(const char *s, int &v)
{
    char *end;
    long l = strtol(s, &end, 10); // std::stoi
    v = (int)l;
    return end != s;
}

struct ObjVertex { int p = -1, t = -1, n = -1; };                 // OBJ::Vertex (:27-32)
struct ObjTriangle { ObjVertex v1, v2, v3; int material; };      // OBJ::Triangle (:34-39)

// create_vertex (:105-150): "p", "p/t", "p//n", "p/t/n"; negative = relative
bool create_vertex(const char *tok, int npos, int ntex, int nnor, ObjVertex &v)
{
    v = ObjVertex();
    // split_string(tok, '/', include_empty = true)
    std::vector<std::string> d;
    std::string cur;
    for (const char *c = tok; *c; ++c) {
        if (*c == '/') {
            d.push_back(cur);
            cur.clear();
        } else {
            cur.push_back(*c);
        }
    }
    if (!cur.empty()) d.push_back(cur);
    int idx;
    if (d.size() > 0) {
        if (!parse_int(d[0].c_str(), idx)) return false;
        v.p = idx > 0 ? idx - 1 : npos + idx;
    }
    if (d.size() > 1 && !d[1].empty()) {
        if (!parse_int(d[1].c_str(), idx)) return false;
        v.t = idx > 0 ? idx - 1 : ntex + idx;
    }
    if (d.size() > 2) {
        if (!parse_int(d[2].c_str(), idx)) return false;
        v.n = idx > 0 ? idx - 1 : nnor + idx;
    }
    return true;
}

} // namespace

static std::string dir_of(const std::string &p)
{
    const size_t k = p.find_last_of('/');
    return k == std::string::npos ? std::string() : p.substr(0, k + 1);
}

static bool file_exists(const std::string &p)
{
    FILE *f = fopen(p.c_str(), "rb");
    if (f) fclose(f);
    return f != nullptr;
}

// make_texture (rt/scene.cuh:25-63): stbi_load(path, ..., 4) -> RGBA8 texels.
// The reference opens `file` relative to the working directory; a path that
// does not exist there is also looked up next to the .mat file and in its
// parent directory (the reference's layout: materials/x.mat, textures/y.png).
// A texture file that exists nowhere leaves the material untextured, as in the
// reference (stbi_load fails, a 0x0 texture whose cudaMalloc(0) buffer is
// NULL).  A file that exists but does not decode is an error.
static int make_texture(RtHostScene &scene, const std::string &mat_path, const std::string &file, Texture &tex)
{
    memset(&tex, 0, sizeof tex);
    std::string found;
    const std::string d = dir_of(mat_path);
    const std::string up = d.empty() ? std::string("../") : dir_of(d.substr(0, d.size() - 1));
    for (const std::string &c : {file, d + file, up + file})
        if (!c.empty() && file_exists(c)) {
            found = c;
            break;
        }
    if (found.empty()) return RT_OK;
    for (const auto &t : scene.textures) // one decode per file per scene
        if (t->path == found) {
            tex.buffer = t->texels.data();
            tex.width = t->width;
            tex.height = t->height;
            return RT_OK;
        }
    std::vector<uint8_t> rgba;
    int w = 0, h = 0;
    std::string err;
    const int rc = decode_image_file(found, rgba, w, h, err);
    if (rc != RT_OK) {
        rt_set_error("%s: texture %s: %s", mat_path.c_str(), found.c_str(), err.c_str());
        return rc;
    }
    std::unique_ptr<RtHostTexture> t(new RtHostTexture);
    t->path = found;
    t->width = w;
    t->height = h;
    // + (width + 1) zero texels: mod(uv, 1) can return 1.0, so sample_texture's
    // index reaches width * height + width (the reference reads past
    // its buffer there)
    t->texels.assign((size_t)w * h + (size_t)w + 1, RtUChar4{0, 0, 0, 0});
    memcpy(t->texels.data(), rgba.data(), (size_t)w * h * 4);
    tex.buffer = t->texels.data();
    tex.width = w;
    tex.height = h;
    scene.textures.push_back(std::move(t));
    return RT_OK;
}

// load_material (rt/mesh_loading.cuh:152-219)
static int load_material(RtHostScene &scene, const std::string &path, const std::string &name, Material &m)
{
    memset(&m, 0, sizeof m); // { ZERO_VEC3D, ZERO_VEC3D, 0, 0, 0, false, NO_TEXTURE }
    std::string text;
    if (!read_file(path, text)) {
        // std::ifstream on a missing file reads nothing: the material stays zero
        return RT_OK;
    }
    const std::string header = "material " + name;
    bool found = false;
    Tokens tk;
    size_t pos = 0;
    while (pos <= text.size()) {
        size_t e = text.find('\n', pos);
        if (e == std::string::npos) {
            if (pos == text.size()) break;
            e = text.size();
        }
        std::string line = text.substr(pos, e - pos);
        pos = e + 1;
        if (line == header) {
            found = true;
        } else if (found) {
            if (line.empty()) break;
            tk.split(line.data(), line.data() + line.size());
            if (tk.t.empty()) {
                rt_set_error("%s: blank property line in material %s", path.c_str(), name.c_str());
                return RT_E_PARSE;
            }
            const std::string key = tk.t[0];
            bool ok = true;
            if (key == "albedo" && tk.t.size() >= 4) {
                ok = parse_float(tk.t[1], m.albedo.x) && parse_float(tk.t[2], m.albedo.y) &&
                     parse_float(tk.t[3], m.albedo.z);
            } else if (key == "emittance" && tk.t.size() >= 4) {
                ok = parse_float(tk.t[1], m.emittance.x) && parse_float(tk.t[2], m.emittance.y) &&
                     parse_float(tk.t[3], m.emittance.z);
            } else if (key == "roughness" && tk.t.size() >= 2) {
                ok = parse_float(tk.t[1], m.roughness);
            } else if (key == "n" && tk.t.size() >= 2) {
                ok = parse_float(tk.t[1], m.refractive_index);
            } else if (key == "k" && tk.t.size() >= 2) {
                ok = parse_float(tk.t[1], m.extinction);
            } else if (key == "transparent") {
                m.transparent = true;
            } else if (key == "texture" && tk.t.size() >= 2) {
                const int rc = make_texture(scene, path, tk.t[1], m.texture);
                if (rc != RT_OK) return rc;
            }
            if (!ok) {
                rt_set_error("%s: bad number in material %s", path.c_str(), name.c_str());
                return RT_E_PARSE;
            }
        }
    }
    return RT_OK;
}

static inline float tmin3(const Triangle &t, int a)
{
    const float *p1 = &t.p1.x, *p2 = &t.p2.x, *p3 = &t.p3.x;
    return fminf(p1[a], fminf(p2[a], p3[a]));
}
static inline float tmax3(const Triangle &t, int a)
{
    const float *p1 = &t.p1.x, *p2 = &t.p2.x, *p3 = &t.p3.x;
    return fmaxf(p1[a], fmaxf(p2[a], p3[a]));
}

int load_mesh(RtHostScene &scene, const std::string &obj_path, const std::string &mat_path, Vec3D offset,
              RtM3 matrix, bool smooth)
{
    std::string text;
    if (!read_file(obj_path, text)) {
        rt_set_error("cannot read %s", obj_path.c_str());
        return RT_E_IO;
    }
    std::vector<Vec3D> positions, normals;
    std::vector<Vec2D> texcoords;
    std::vector<char> false_normal;
    std::vector<ObjTriangle> mesh;
    std::map<std::string, int> material_ids;
    std::vector<Material> materials;
    int current = -1; // "" before any usemtl -> value-initialised Material
    Tokens tk;
    const char *b = text.data(), *end = b + text.size();
    long line_no = 0;
    while (b < end) {
        const char *e = (const char *)memchr(b, '\n', (size_t)(end - b));
        if (!e) e = end;
        ++line_no;
        tk.split(b, e);
        b = e + 1;
        if (tk.t.empty()) continue;
        const char *k = tk.t[0];
        bool ok = true;
        if (!strcmp(k, "v")) {
            Vec3D p = rt_v3(0.0f, 0.0f, 0.0f);
            ok = tk.t.size() >= 4 && parse_float(tk.t[1], p.x) && parse_float(tk.t[2], p.y) &&
                 parse_float(tk.t[3], p.z);
            positions.push_back(p);
        } else if (!strcmp(k, "vn")) {
            Vec3D n = rt_v3(0.0f, 0.0f, 0.0f);
            ok = tk.t.size() >= 4 && parse_float(tk.t[1], n.x) && parse_float(tk.t[2], n.y) &&
                 parse_float(tk.t[3], n.z);
            false_normal.push_back(n.x == 0 && n.y == 0 && n.z == 0); // :274-277
            normals.push_back(n);
        } else if (!strcmp(k, "vt")) {
            Vec2D t = rt_v2(1.0f, 1.0f); // ZERO_VEC2D
            float v = 0.0f;
            ok = tk.t.size() >= 3 && parse_float(tk.t[1], t.x) && parse_float(tk.t[2], v);
            t.y = 1.0f - v; // :286
            texcoords.push_back(t);
        } else if (!strcmp(k, "usemtl")) {
            ok = tk.t.size() >= 2;
            if (ok) {
                std::string name = tk.t[1];
                auto it = material_ids.find(name);
                if (it == material_ids.end()) {
                    Material m;
                    int rc = load_material(scene, mat_path, name, m);
                    if (rc != RT_OK) return rc;
                    int id = (int)materials.size();
                    materials.push_back(m);
                    it = material_ids.emplace(name, id).first;
                }
                current = it->second;
            }
        } else if (!strcmp(k, "f")) {
            ObjVertex v1, v2, v3;
            int np = (int)positions.size(), nt = (int)texcoords.size(), nn = (int)normals.size();
            ok = tk.t.size() >= 2 && create_vertex(tk.t[1], np, nt, nn, v1);
            bool is_false = ok && v1.n >= 0 && v1.n < nn && false_normal[v1.n];
            if (ok && !is_false) {
                for (size_t i = 3; i < tk.t.size() && ok; ++i) {
                    ok = create_vertex(tk.t[i - 1], np, nt, nn, v2) && create_vertex(tk.t[i], np, nt, nn, v3);
                    mesh.push_back({v1, v2, v3, current});
                }
            }
        }
        if (!ok) {
            rt_set_error("%s:%ld: malformed line", obj_path.c_str(), line_no);
            return RT_E_PARSE;
        }
    }
    const int np = (int)positions.size(), nt = (int)texcoords.size(), nn = (int)normals.size();
    for (const ObjTriangle &t : mesh) {
        for (const ObjVertex *v : {&t.v1, &t.v2, &t.v3}) {
            if (v->p < 0 || v->p >= np || v->t < -1 || v->t >= nt || v->n < -1 || v->n >= nn) {
                rt_set_error("%s: face index out of range", obj_path.c_str());
                return RT_E_PARSE;
            }
        }
    }
    // computed_normals (:328-342): unnormalised sums of face normals
    std::vector<Vec3D> computed(positions.size(), rt_v3(0.0f, 0.0f, 0.0f));
    for (const ObjTriangle &t : mesh) {
        Vec3D p1 = positions[t.v1.p], p2 = positions[t.v2.p], p3 = positions[t.v3.p];
        Vec3D n = rt_normalize(rt_cross(p2 - p1, p3 - p1));
        computed[t.v1.p] = computed[t.v1.p] + n;
        computed[t.v2.p] = computed[t.v2.p] + n;
        computed[t.v3.p] = computed[t.v3.p] + n;
    }
    const size_t prior = scene.tris.size();
    scene.tris.resize(prior + mesh.size());
    Material empty;
    memset(&empty, 0, sizeof empty);
    for (size_t i = 0; i < mesh.size(); ++i) { // :349-415
        const ObjTriangle &o = mesh[i];
        Triangle t;
        memset(&t, 0, sizeof t);
        t.p1 = positions[o.v1.p];
        t.p2 = positions[o.v2.p];
        t.p3 = positions[o.v3.p];
        Vec3D n = rt_normalize(rt_cross(t.p2 - t.p1, t.p3 - t.p1));
        t.n1 = n; t.n2 = n; t.n3 = n;
        if (o.v1.n != -1) t.n1 = normals[o.v1.n]; else if (smooth) t.n1 = computed[o.v1.p];
        if (o.v2.n != -1) t.n2 = normals[o.v2.n]; else if (smooth) t.n2 = computed[o.v2.p];
        if (o.v3.n != -1) t.n3 = normals[o.v3.n]; else if (smooth) t.n3 = computed[o.v3.p];
        t.uv1 = rt_v2(1.0f, 1.0f); t.uv2 = t.uv1; t.uv3 = t.uv1;
        if (o.v1.t != -1) t.uv1 = texcoords[o.v1.t];
        if (o.v2.t != -1) t.uv2 = texcoords[o.v2.t];
        if (o.v3.t != -1) t.uv3 = texcoords[o.v3.t];
        t.material = o.material >= 0 ? materials[o.material] : empty;
        scene.tris[prior + i] = t;
    }
    // transform (:418-439)
    Bounding_Box bb;
    bb.min = rt_v3(FLT_MAX, FLT_MAX, FLT_MAX);
    bb.max = -rt_v3(FLT_MAX, FLT_MAX, FLT_MAX);
    for (size_t i = prior; i < scene.tris.size(); ++i) {
        const Triangle &t = scene.tris[i];
        bb.min.x = fminf(tmin3(t, 0), bb.min.x);
        bb.min.y = fminf(tmin3(t, 1), bb.min.y);
        bb.min.z = fminf(tmin3(t, 2), bb.min.z);
        bb.max.x = fmaxf(tmax3(t, 0), bb.max.x);
        bb.max.y = fmaxf(tmax3(t, 1), bb.max.y);
        bb.max.z = fmaxf(tmax3(t, 2), bb.max.z);
    }
    Vec3D center = rt_v3((bb.min.x + bb.max.x) * 0.5f, (bb.min.y + bb.max.y) * 0.5f, (bb.min.z + bb.max.z) * 0.5f);
    for (size_t i = prior; i < scene.tris.size(); ++i) {
        Triangle &t = scene.tris[i];
        t.p1 = t.p1 - center;
        t.p2 = t.p2 - center;
        t.p3 = t.p3 - center;
        t.p1 = matrix * t.p1 + offset;
        t.p2 = matrix * t.p2 + offset;
        t.p3 = matrix * t.p3 + offset;
        t.n1 = rt_normalize(matrix * t.n1);
        t.n2 = rt_normalize(matrix * t.n2);
        t.n3 = rt_normalize(matrix * t.n3);
    }
    return RT_OK;
}

static std::string resolve(const std::string &dir, const std::string &p)
{
    return (!p.empty() && p[0] == '/') ? p : dir + p;
}

int load_scene_file(RtHostScene &scene, const std::string &path, Camera *camera_out)
{
    std::string text;
    if (!read_file(path, text)) {
        rt_set_error("cannot read scene %s", path.c_str());
        return RT_E_IO;
    }
    const std::string dir = dir_of(path);
    Tokens tk;
    size_t pos = 0;
    bool have_camera = false;
    while (pos < text.size()) {
        size_t e = text.find('\n', pos);
        if (e == std::string::npos) e = text.size();
        tk.split(text.data() + pos, text.data() + e);
        pos = e + 1;
        if (tk.t.empty() || tk.t[0][0] == '#') continue;
        std::string k = tk.t[0];
        if (k == "mesh" && tk.t.size() == 10) {
            float v[6];
            int smooth = 0;
            bool ok = true;
            for (int i = 0; i < 6; ++i) ok = ok && parse_float(tk.t[3 + i], v[i]);
            ok = ok && parse_int(tk.t[9], smooth);
            if (!ok) {
                rt_set_error("%s: bad mesh line", path.c_str());
                return RT_E_PARSE;
            }
            // create_models: { offset, rotation_matrix(yaw, pitch) * scale } (rt/create_models.cuh:21-39)
            RtM3 m = rt_rotation_matrix(v[3], v[4]) * v[5];
            int rc = load_mesh(scene, resolve(dir, tk.t[1]), resolve(dir, tk.t[2]), rt_v3(v[0], v[1], v[2]), m,
                               smooth != 0);
            if (rc != RT_OK) return rc;
        } else if (k == "camera" && tk.t.size() == 8) {
            float v[7];
            for (int i = 0; i < 7; ++i)
                if (!parse_float(tk.t[1 + i], v[i])) {
                    rt_set_error("%s: bad camera line", path.c_str());
                    return RT_E_PARSE;
                }
            if (camera_out) {
                camera_out->position = rt_v3(v[0], v[1], v[2]);
                camera_out->yaw = v[3];
                camera_out->pitch = v[4];
                camera_out->FOV = v[5];
                camera_out->aperture_radius = v[6];
            }
            have_camera = true;
        } else {
            rt_set_error("%s: unknown line '%s'", path.c_str(), k.c_str());
            return RT_E_PARSE;
        }
    }
    if (!have_camera && camera_out) {
        // rt/main.cu:101-104
        camera_out->position = rt_v3(-2.1f, 1.7f, -1.2f);
        camera_out->yaw = 0.975f;
        camera_out->pitch = 0.3f;
        camera_out->FOV = RT_HALF_PI;
        camera_out->aperture_radius = 0.002f;
    }
    if (scene.tris.empty()) {
        rt_set_error("%s: scene has no triangles", path.c_str());
        return RT_E_INVALID;
    }
    return RT_OK;
}

std::vector<int> light_list(const Triangle *tris, int n)
{
    std::vector<int> l;
    for (int i = 0; i < n; ++i) {
        Vec3D e = tris[i].material.emittance;
        if (e.x > 0 || e.y > 0 || e.z > 0) l.push_back(i);
    }
    return l;
}

} // namespace rt_host
