// rt_scene.h — host-side scene model and its HBM layout.
//
// Host side of the drop-in boundary: a SceneBuilder with the reference's
// semantics (include/scene_builder.h:29-117, src/scene_builder.{cc,cu}) and the
// worldN.json cube-world generator (src/procedural/cube_world.cc:38-191,
// perlin.cu).  `flatten()` produces the flat, device-ready arrays the kernels
// read (the reference's device-side `new Trimesh/Light` with virtual dispatch,
// scene_builder.cu:29-81, is replaced by these plain arrays).
#pragma once

#include <stdint.h>
#include <string>
#include <vector>

#include "rt_math.h"

namespace rt {

struct Material {                        // include/rayprimitives/material.h:14-31
    rtm::V4 Ke{0, 0, 0, 0}, Ka{0, 0, 0, 0}, Kd{0, 0, 0, 0}, Ks{0, 0, 0, 0}, Kt{0, 0, 0, 0}, Kr{0, 0, 0, 0};
    float alpha = 0.0f, eta = 1.0f;
};

struct MeshDesc { rtm::Q rot{0, 0, 0, 1}; rtm::V3 pos{0, 0, 0}; std::vector<int> tris; };
// rprimitives::TextureCoords (texture_coords.h:12-29): atlas texel of a hit with
// barycentric weights (u, v) of vertices 1 and 2 = (tx, ty) + u * (ux, uy) + v * (vx, vy).
// Build-defined: the reference stores these but never samples them (phong.cu:18-23).
struct TexDesc { int has = 0; float tx = 0, ty = 0, ux = 0, uy = 0, vx = 0, vy = 0; };
struct TriDesc { int i0, i1, i2, mat; TexDesc tex; };
struct InstDesc { rtm::Q rot{0, 0, 0, 1}; rtm::V3 pos{0, 0, 0}; int mesh; };
struct LightDesc { int type; rtm::V3 v; rtm::V4 col; };   // 0 point(pos), 1 directional(normalized dir)

struct CameraDesc {
    float fov = 0.785398163f, unit = 200, near_ = 0;
    int W = 640, H = 480;
    rtm::V3 pos{0, 0, 0};
    rtm::Q rot{0, 0, 0, 1};
};

// ---- device-ready records (all plain-old-data, 16-byte aligned) ----
struct alignas(16) DTri {              // 128 B: the plane filter's (pn, a) first (one 32-B scalar load)
    rtm::V3 pn, a, b, c;               // normalized plane normal, vertices (mesh-local)
    float area;                        // |cross(b-a, c-a)|
    float inv_area;                    // fl(1/area): only used by the filtered test's estimate
    rtm::V3 n0, n1, n2;                // vertex normals (generate_normals)
    int mat, tex;                      // tex: 1 if the texture coordinates below are set
    float tx, ty, ux, uy, vx, vy;      // TexDesc (textured shading mode only)
    int pad[2];
};
struct alignas(16) DMesh { rtm::Pose pose; int tri_begin, tri_count, pad[2]; };
struct alignas(16) DInst { rtm::Pose pose; int mesh, pad[3]; };
struct alignas(16) DMat { rtm::V4 Ke, Ka, Kd, Ks, Kt, Kr; float alpha, eta; int reflective, refractive; };
struct alignas(16) DLight { rtm::V3 v; int type; rtm::V4 col; };
struct alignas(16) DNode { float mnx, mny, mnz, mxx, mxy, mxz; int nd, inst; };   // 32 B BVH node

struct DCamera {                       // Camera::at (camera.cu:33-42) with the per-pixel-invariant parts hoisted
    rtm::V3 pos, r, u, f;
    float near_, unit, W, H;
};

struct Scene {
    // builder state (SceneBuilder)
    std::string atlas;                 // atlas path as given (JSON "atlas" / SceneBuilder{atlas})
    std::string base_dir;              // directory of the scene file (atlas paths resolve here first)
    std::vector<uint8_t> atlas_rgba;   // RGBA8 texels, row-major (empty: no atlas loaded)
    int atlas_w = 0, atlas_h = 0;
    std::vector<rtm::V3> verts, norms;
    std::vector<TriDesc> tris;
    std::vector<Material> mats;
    std::vector<MeshDesc> meshes;
    std::vector<InstDesc> insts;
    std::vector<LightDesc> points, dirs;
    CameraDesc cam;
    rtm::V3 dist_atten{0, 0, 0};
    rtm::V4 ambience{0, 0, 0, 0};
    int depth = 0;

    // flattened (valid after flatten())
    std::vector<DTri> d_tris;
    std::vector<DMesh> d_meshes;
    std::vector<DInst> d_insts;
    std::vector<DMat> d_mats;
    std::vector<DLight> d_lights;      // points first, then directional (scene_builder.cu:61-81)
    DCamera d_cam{};
    std::vector<float> verts_norm;     // generate_normals() output, xyz per vertex

    // builder API (scene_builder.h:58-112)
    int add_vertex(rtm::V3 v) { verts.push_back(v); return (int)verts.size() - 1; }
    int create_mesh(rtm::V3 pos, rtm::Q rot) { MeshDesc m; m.pos = pos; m.rot = rot; meshes.push_back(m); return (int)meshes.size() - 1; }
    int add_material(const Material& m) { mats.push_back(m); return (int)mats.size() - 1; }
    void add_triangle(int mesh, int i0, int i1, int i2, int mat, const TexDesc& tex = TexDesc{}) {
        tris.push_back(TriDesc{i0, i1, i2, mat, tex});
        meshes[mesh].tris.push_back((int)tris.size() - 1);
    }
    int add_trans(int mesh) { InstDesc t; t.mesh = mesh; insts.push_back(t); return (int)insts.size() - 1; }
    // tile (optional, build-defined): {tx, ty, size} maps every face onto that atlas square
    int build_cube(float scale, const Material& mat, const float* tile = nullptr);
    void add_point_light(rtm::V3 pos, rtm::V4 col) { points.push_back(LightDesc{0, pos, col}); }
    void add_directional_light(rtm::V3 dir, rtm::V4 col) { dirs.push_back(LightDesc{1, rtm::normalized(dir), col}); }

    void generate_normals();           // scene_builder.cc:11-29
    void set_camera(int W, int H, float fov, float unit);   // camera.cu:6-9
    void update_camera_basis();        // to_Mat3 columns (camera.cu:33-42)
    int flatten(std::string* err);     // -> d_* arrays
};

// worldN.json -> Scene (cube_world.cc:38-191).  width/height > 0 override the JSON.
int load_cube_world(const std::string& path, int width, int height, Scene* out, std::string* err);

// 8-bit RGBA/RGB non-interlaced PNG -> RGBA8 (the atlas format assets.cc:11-57 reads
// through libpng; here with zlib).  Returns 0 or -1 with *err set.
int load_png_rgba8(const std::string& path, std::vector<uint8_t>* out, int* w, int* h, std::string* err);

// Build-defined spp sample offsets: R2 sequence in IEEE double, k=0 -> (0,0).
void spp_offset(int k, float* dx, float* dy);

}  // namespace rt
