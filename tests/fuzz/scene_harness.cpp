// Test harness (tests/test_loader_fuzz.py): loads every scene file named on
// the command line with the product's host path (load_scene_file: OBJ + .mat
// + textures, rt/mesh_loading.cuh:221-440) and builds the KD tree of what it
// loaded (create_kd_tree, rt/create_kd_tree.cuh:267-328), built with ASan +
// UBSan.  Prints one "<rc> <triangles> <nodes>" line per file; any memory
// error or undefined behaviour aborts.
#include <stdio.h>

#include <string>
#include <vector>

#include "host/rt_host.h"

void rt_set_error(const char *, ...) {}

int main(int argc, char **argv)
{
    for (int i = 1; i < argc; ++i) {
        RtHostScene scene;
        Camera cam{};
        const int rc = rt_host::load_scene_file(scene, argv[i], &cam);
        int nodes_n = 0;
        if (rc == 0 && !scene.tris.empty()) {
            std::vector<KD_Tree_Node> nodes;
            std::vector<int> indices;
            Bounding_Box bounds;
            if (rt_host::build_kd_tree(scene.tris.data(), (int)scene.tris.size(), nodes, indices, bounds) != 0) {
                printf("%d %zu kd-failed\n", rc, scene.tris.size());
                continue;
            }
            for (int k : indices)
                if (k < 0 || k >= (int)scene.tris.size()) {
                    fprintf(stderr, "%s: KD index out of range\n", argv[i]);
                    return 2;
                }
            nodes_n = (int)nodes.size();
        }
        printf("%d %zu %d\n", rc, scene.tris.size(), nodes_n);
    }
    return 0;
}
