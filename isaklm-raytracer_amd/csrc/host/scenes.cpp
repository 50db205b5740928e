// scenes.cpp — deterministic synthetic scenes for BASELINE.json's configs.
//
// The reference's scene (rt/create_models.cuh:17-43) loads OBJ models that
// were never published (.gitignore:78 ignores *.obj), so every config runs on
// a generated scene.  The generator writes ordinary OBJ + .mat +
// scene files, which then go through the same load_mesh / create_scene path
// as any user scene.  Geometry uses only IEEE +,-,*,/ and rt_libm's
// double-precision sin/cos, and floats are printed with %.9g (round-trips
// through strtof), so the files are byte-identical on every machine.
//
//   name          config (BASELINE.json)            triangles
//   cornell       1: Cornell box, 256x256            36
//   cornell_blob  2: + displaced sphere (gold)       36 + 50,700
//   room2m        3/4: room + 2M displaced mesh       12+2 + 1,997,568 + 2 x 20,172 glass
//                    (dragon.mat gold) + 2 glass spheres + emissive quad
//   room2m_glass  5: as room2m, the big mesh glass with smooth normals
//   room_small    test-size room (blob 20,172 tris) for fast parity tests
// Meshes are displaced cube-spheres (12 n^2 near-uniform triangles).
#include <stdio.h>
#include <string.h>
#include <sys/stat.h>

#include <cmath>
#include <map>
#include <string>
#include <vector>

#include "rt_host.h"

namespace {

struct Obj {
    std::string text;
    int nverts = 0;
    char buf[256];
    int v(double x, double y, double z)
    {
        snprintf(buf, sizeof buf, "v %.9g %.9g %.9g\n", (double)(float)x, (double)(float)y, (double)(float)z);
        text += buf;
        return ++nverts; // 1-based
    }
    void use(const char *m) { text += "usemtl "; text += m; text += "\n"; }
    void tri(int a, int b, int c)
    {
        snprintf(buf, sizeof buf, "f %d %d %d\n", a, b, c);
        text += buf;
    }
    void quad(int a, int b, int c, int d) // fan-triangulated by load_mesh (:305-313)
    {
        snprintf(buf, sizeof buf, "f %d %d %d %d\n", a, b, c, d);
        text += buf;
    }
    void box_face(double x0, double y0, double z0, double ux, double uy, double uz, double vx, double vy, double vz)
    {
        int a = v(x0, y0, z0);
        int b = v(x0 + ux, y0 + uy, z0 + uz);
        int c = v(x0 + ux + vx, y0 + uy + vy, z0 + uz + vz);
        int d = v(x0 + vx, y0 + vy, z0 + vz);
        quad(a, b, c, d);
    }
};

bool write_text(const std::string &path, const std::string &text)
{
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) return false;
    bool ok = fwrite(text.data(), 1, text.size(), f) == text.size();
    return (fclose(f) == 0) && ok;
}

// axis-aligned room interior: floor/ceiling/4 walls as quads
void room_box(Obj &o, double x0, double x1, double y0, double y1, double z0, double z1, const char *wall_mat,
              const char *floor_mat, const char *ceil_mat, bool open_front)
{
    o.use(floor_mat);
    o.box_face(x0, y0, z0, x1 - x0, 0, 0, 0, 0, z1 - z0);
    o.use(ceil_mat);
    o.box_face(x0, y1, z0, 0, 0, z1 - z0, x1 - x0, 0, 0);
    o.use(wall_mat);
    o.box_face(x0, y0, z1, x1 - x0, 0, 0, 0, y1 - y0, 0); // back (+z)
    if (!open_front) o.box_face(x0, y0, z0, 0, y1 - y0, 0, x1 - x0, 0, 0);
}

// rotated rectangular block, 6 quads
void block(Obj &o, double cx, double cy, double cz, double sx, double sy, double sz, double angle)
{
    const double c = rt_cos_d(angle), s = rt_sin_d(angle);
    double P[8][3];
    for (int k = 0; k < 8; ++k) {
        double lx = ((k & 1) ? 0.5 : -0.5) * sx, ly = ((k & 2) ? 0.5 : -0.5) * sy, lz = ((k & 4) ? 0.5 : -0.5) * sz;
        P[k][0] = cx + c * lx + s * lz;
        P[k][1] = cy + ly;
        P[k][2] = cz - s * lx + c * lz;
    }
    int id[8];
    for (int k = 0; k < 8; ++k) id[k] = o.v(P[k][0], P[k][1], P[k][2]);
    const int f[6][4] = {{0, 1, 3, 2}, {4, 6, 7, 5}, {0, 4, 5, 1}, {2, 3, 7, 6}, {0, 2, 6, 4}, {1, 5, 7, 3}};
    for (auto &q : f) o.quad(id[q[0]], id[q[1]], id[q[2]], id[q[3]]);
}

// displaced cube-sphere: the 6 faces of [-1,1]^3 cut into n x n quads, vertices
// pushed onto the unit sphere and displaced radially; 12 n^2 triangles of
// near-uniform size, shared vertices, no pole fans (a UV sphere's poles put
// ~1,400 slivers in one KD leaf, nothing like a scanned model)
void cube_blob(Obj &o, int n, double amp)
{
    std::map<long long, int> ids;
    auto key = [&](int i, int j, int k) { return ((long long)i * (n + 1) + j) * (n + 1) + k; };
    auto vert = [&](int i, int j, int k) {
        auto it = ids.find(key(i, j, k));
        if (it != ids.end()) return it->second;
        double x = -1.0 + 2.0 * i / n, y = -1.0 + 2.0 * j / n, z = -1.0 + 2.0 * k / n;
        double len = sqrt(x * x + y * y + z * z);
        x /= len; y /= len; z /= len;
        double r = 1.0 + amp * (0.10 * rt_sin_d(3.1 * x + 1.7) * rt_cos_d(2.3 * y - 0.4) +
                                0.05 * rt_sin_d(9.7 * y + 0.3) * rt_sin_d(8.9 * z + 1.1) +
                                0.02 * rt_cos_d(27.1 * z - 0.2) * rt_sin_d(23.3 * x + 0.9));
        int id = o.v(r * x, r * y, r * z);
        ids.emplace(key(i, j, k), id);
        return id;
    };
    // each face: fixed axis a at value s (0 or n), the other two axes u, v
    for (int a = 0; a < 3; ++a) {
        for (int side = 0; side < 2; ++side) {
            const int s = side ? n : 0;
            for (int u = 0; u < n; ++u) {
                for (int v = 0; v < n; ++v) {
                    int c[4][3];
                    const int uu[4] = {u, u + 1, u + 1, u}, vv[4] = {v, v, v + 1, v + 1};
                    for (int q = 0; q < 4; ++q) {
                        c[q][a] = s;
                        c[q][(a + 1) % 3] = uu[q];
                        c[q][(a + 2) % 3] = vv[q];
                    }
                    int id[4];
                    for (int q = 0; q < 4; ++q) id[q] = vert(c[q][0], c[q][1], c[q][2]);
                    if (side) o.quad(id[0], id[1], id[2], id[3]);
                    else o.quad(id[0], id[3], id[2], id[1]);
                }
            }
        }
    }
}

// displaced UV sphere: 2*slices*(stacks-1) triangles, unit radius before displacement
void blob(Obj &o, int slices, int stacks, double amp)
{
    const double pi = 3.14159265358979323846;
    auto radius = [&](double th, double ph) {
        return 1.0 + amp * (0.12 * rt_sin_d(3 * th) * rt_cos_d(4 * ph) + 0.05 * rt_sin_d(11 * th) * rt_sin_d(13 * ph) +
                            0.02 * rt_sin_d(31 * th) * rt_cos_d(29 * ph));
    };
    const int top = o.v(0.0, radius(0.0, 0.0), 0.0);
    std::vector<int> ring((size_t)(stacks - 1) * slices);
    for (int i = 1; i < stacks; ++i) {
        double th = pi * i / stacks;
        for (int j = 0; j < slices; ++j) {
            double ph = 2 * pi * j / slices;
            double r = radius(th, ph);
            ring[(size_t)(i - 1) * slices + j] =
                o.v(r * rt_sin_d(th) * rt_cos_d(ph), r * rt_cos_d(th), r * rt_sin_d(th) * rt_sin_d(ph));
        }
    }
    const int bottom = o.v(0.0, -radius(pi, 0.0), 0.0);
    auto at = [&](int i, int j) { return ring[(size_t)i * slices + (j % slices)]; };
    for (int j = 0; j < slices; ++j) o.tri(top, at(0, j + 1), at(0, j));
    for (int i = 0; i + 1 < stacks - 1; ++i)
        for (int j = 0; j < slices; ++j) o.quad(at(i, j), at(i, j + 1), at(i + 1, j + 1), at(i + 1, j));
    for (int j = 0; j < slices; ++j) o.tri(bottom, at(stacks - 2, j), at(stacks - 2, j + 1));
}

// material files: values from the reference's rt/materials/*.mat; the
// room's wall/floor textures (rt/materials/room.mat:5,11) are replaced by
// constant albedo because the texture images are absent (.MISSING_LARGE_BLOBS)
const char *kCornellMat =
    "material white\nalbedo 0.73 0.73 0.73\nroughness 0.5\nn 1.5\n\n"
    "material red\nalbedo 0.65 0.05 0.05\nroughness 0.5\nn 1.5\n\n"
    "material green\nalbedo 0.12 0.45 0.15\nroughness 0.5\nn 1.5\n\n"
    "material light\nalbedo 0.78 0.78 0.78\nemittance 15.0 15.0 15.0\nroughness 0.5\nn 1.5\n";
const char *kRoomMat =
    "material walls\nalbedo 0.8 0.8 0.78\nroughness 0.2\nn 1.25\n\n"
    "material floor\nalbedo 0.62 0.45 0.3\nroughness 0.05\nn 1.6\n\n"
    "material ceiling_lamp\nalbedo 0.972 0.96 0.915\nroughness 0.02\nn 1.1978\nk 7.0488\n\n"
    "material emissive\nalbedo 0.7 0.7 0.7\nemittance 100.0 90.0 65.0\nroughness 0.2\nn 1.2\n";
const char *kDragonMat = "material dragon\nalbedo 0.9709 0.7429 0.3268\nroughness 0.01\nn 0.27732\nk 2.9278\n";
const char *kGlassMat = "material glass\nalbedo 0.995 0.995 0.995\nroughness 0.001\nn 1.51\ntransparent\n";

std::string cornell_obj()
{
    Obj o;
    room_box(o, -1, 1, 0, 2, -1, 1, "white", "white", "white", true);
    o.use("red");
    o.box_face(-1, 0, -1, 0, 0, 2, 0, 2, 0);
    o.use("green");
    o.box_face(1, 0, -1, 0, 2, 0, 0, 0, 2);
    o.use("light");
    o.box_face(-0.3, 1.98, -0.3, 0.6, 0, 0, 0, 0, 0.6);
    o.use("white");
    block(o, 0.35, 0.3, -0.3, 0.6, 0.6, 0.6, -0.3);
    block(o, -0.35, 0.6, 0.35, 0.6, 1.2, 0.6, 0.3);
    return o.text;
}

std::string room_obj()
{
    Obj o;
    room_box(o, -2.5, 2.5, 0, 3, -2, 2, "walls", "floor", "walls", false);
    o.use("emissive");
    o.box_face(-0.5, 2.98, -0.4, 1.0, 0, 0, 0, 0, 0.8);
    return o.text;
}

std::string blob_obj(const char *mat, int n, double amp)
{
    Obj o;
    o.text.reserve((size_t)n * n * 6 * 80);
    o.use(mat);
    cube_blob(o, n, amp);
    return o.text;
}

} // namespace

extern "C" int rt_generate_scene(const char *name, const char *out_dir, char *scene_path_out, size_t cap)
{
    if (!name || !out_dir) {
        rt_set_error("rt_generate_scene: null argument");
        return RT_E_INVALID;
    }
    std::string dir = out_dir;
    if (!dir.empty() && dir.back() != '/') dir += '/';
    mkdir(dir.c_str(), 0755);
    std::string n = name, scene;
    struct File { std::string name, text; };
    std::vector<File> files;
    // cameras: rt/main.cu:101-104 for the room; the Cornell camera sits off
    // every root split plane and is rotated with the room (yaw 0.1)
    if (n == "cornell" || n == "cornell_blob") {
        files.push_back({"cornell.obj", cornell_obj()});
        files.push_back({"cornell.mat", kCornellMat});
        scene = "# BASELINE config " + std::string(n == "cornell" ? "1" : "2") + "\n"
                "mesh cornell.obj cornell.mat 0 1 0 0.1 0 1 0\n";
        if (n == "cornell_blob") {
            files.push_back({"blob50k.obj", blob_obj("dragon", 65, 1.0)});
            files.push_back({"dragon.mat", kDragonMat});
            scene += "mesh blob50k.obj dragon.mat 0.27 0.93 -0.33 2.1 0 0.33 0\n";
        }
        scene += "camera -0.3458 1.0 -3.5834 0.1 0 0.8 0\n";
    } else if (n == "room2m" || n == "room2m_glass" || n == "room_small") {
        const bool big = n != "room_small";
        const bool glass = n == "room2m_glass";
        files.push_back({"room.obj", room_obj()});
        files.push_back({"room.mat", kRoomMat});
        files.push_back({"dragon.mat", kDragonMat});
        files.push_back({"glass.mat", kGlassMat});
        const char *blob_name = big ? "blob2m.obj" : "blob20k.obj";
        files.push_back({blob_name, big ? blob_obj(glass ? "glass" : "dragon", 408, 1.0)
                                        : blob_obj("dragon", 41, 1.0)});
        files.push_back({"glass_sphere.obj", blob_obj("glass", 41, 0.0)});
        scene = "# BASELINE config " + std::string(glass ? "5" : (big ? "3/4" : "test")) + "\n";
        scene += "mesh room.obj room.mat 0 1.5 0 0.1 0 1 0\n";
        scene += std::string("mesh ") + blob_name + (glass ? " glass.mat" : " dragon.mat") +
                 " -0.3 0.9 0.7 2.1 0 0.5 " + (glass ? "1" : "0") + "\n";
        scene += "mesh glass_sphere.obj glass.mat -1.0 0.45 -0.1 2.1 0 0.25 1\n";
        scene += "mesh glass_sphere.obj glass.mat 0.5 0.45 -0.5 2.1 0 0.25 1\n";
        scene += "camera -2.1 1.7 -1.2 0.975 0.3 1.5707963705062866 0.002\n";
    } else {
        rt_set_error("unknown scene '%s' (cornell, cornell_blob, room2m, room2m_glass, room_small)", name);
        return RT_E_INVALID;
    }
    if (n == "room2m_glass") {
        // the glass blob uses the dragon geometry file name of its own
        files[4].name = "blob2m_glass.obj";
        size_t p = scene.find("blob2m.obj");
        scene.replace(p, strlen("blob2m.obj"), "blob2m_glass.obj");
    }
    files.push_back({"scene.txt", scene});
    for (const File &f : files) {
        if (!write_text(dir + f.name, f.text)) {
            rt_set_error("cannot write %s%s", dir.c_str(), f.name.c_str());
            return RT_E_IO;
        }
    }
    std::string path = dir + "scene.txt";
    if (scene_path_out && cap > path.size()) memcpy(scene_path_out, path.c_str(), path.size() + 1);
    return RT_OK;
}
