// Test driver for include/rtracer_amd.hpp: builds a scene through the reference's C++
// API (rtracer::SceneBuilder, scene_builder.h:51-117), renders it with
// rtracer::gpu::update_scene (raytracer.h:18-22) and writes the canvas, read through
// scene->get_environment().get_canvas() (main.cc:91), as raw uint32 words.
//
//   shim_world DESC OUT
// DESC (text, written by tests/test_gpu_cli.py):
//   W H fov unit depth
//   px py pz qi qj qk qr          camera pose
//   da0 da1 da2 am0 am1 am2 am3   distance attenuation, ambience
//   N  then N lines of 26 floats  cube materials (Ke Ka Kd Ks Kt Kr alpha eta)
//   M  then M lines: mesh px py pz
//   K  then K lines: dx dy dz r g b a   directional lights
//   P  then P lines: px py pz r g b a   point lights
#include <cstdio>
#include <vector>

#include "rtracer_amd.hpp"

int main(int argc, char** argv) {
    if (argc != 3) return 2;
    FILE* f = std::fopen(argv[1], "r");
    if (!f) return 2;
    int W, H, depth;
    float fov, unit, cp[3], cq[4], da[3], am[4];
    if (std::fscanf(f, "%d %d %f %f %d", &W, &H, &fov, &unit, &depth) != 5) return 3;
    if (std::fscanf(f, "%f %f %f %f %f %f %f", cp, cp + 1, cp + 2, cq, cq + 1, cq + 2, cq + 3) != 7) return 3;
    if (std::fscanf(f, "%f %f %f %f %f %f %f", da, da + 1, da + 2, am, am + 1, am + 2, am + 3) != 7) return 3;

    rtracer::SceneBuilder b("assets/sus.png");
    int n;
    if (std::fscanf(f, "%d", &n) != 1) return 3;
    std::vector<int> meshes;
    for (int i = 0; i < n; i++) {
        float m[26];
        for (float& x : m) if (std::fscanf(f, "%f", &x) != 1) return 3;
        rmath::Vec4<float> c[6];
        for (int a = 0; a < 6; a++) c[a] = {m[4 * a], m[4 * a + 1], m[4 * a + 2], m[4 * a + 3]};
        rprimitives::Material mat(c[0], c[1], c[2], c[3], c[4], c[5], m[24], m[25]);
        meshes.push_back(b.build_cube(0.999f, rprimitives::TextureCoords{}, mat));   // cube_world.cc:146-160
    }
    if (std::fscanf(f, "%d", &n) != 1) return 3;
    for (int i = 0; i < n; i++) {
        int mesh;
        float p[3];
        if (std::fscanf(f, "%d %f %f %f", &mesh, p, p + 1, p + 2) != 4) return 3;
        int t = b.add_trans(b.get_mesh_builder(meshes[mesh]));
        b.get_transformation(t).set_position({p[0], p[1], p[2]});
    }
    for (int kind = 0; kind < 2; kind++) {
        if (std::fscanf(f, "%d", &n) != 1) return 3;
        for (int i = 0; i < n; i++) {
            float v[7];
            for (float& x : v) if (std::fscanf(f, "%f", &x) != 1) return 3;
            if (kind == 0) b.add_directional_light({v[0], v[1], v[2]}, {v[3], v[4], v[5], v[6]});
            else b.add_point_light({v[0], v[1], v[2]}, {v[3], v[4], v[5], v[6]});
        }
    }
    std::fclose(f);

    renv::Canvas canvas(W, H);
    renv::Camera camera(fov, unit, canvas);
    camera.set_position({cp[0], cp[1], cp[2]});
    camera.set_orientation(rmath::Quat<float>(cq[0], cq[1], cq[2], cq[3]));
    renv::gpu::Scene* scene = b.build_gpu_scene(canvas, camera, depth, {da[0], da[1], da[2]}, {am[0], am[1], am[2], am[3]});

    rtracer::gpu::update_scene(scene, 16, true);
    renv::Canvas& cv = scene->get_environment().get_canvas();
    FILE* o = std::fopen(argv[2], "wb");
    if (!o) return 4;
    std::fwrite(cv.get_buffer(), 4, (size_t)cv.get_width() * cv.get_height(), o);
    std::fclose(o);
    const renv::Color c = cv.get_color(W / 2, H - 1);
    std::printf("center-bottom %u %u %u %u\n", c.red(), c.green(), c.blue(), c.alpha());
    renv::gpu::Scene::free(*scene);
    delete scene;
    return 0;
}
