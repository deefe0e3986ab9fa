/*
 * rt_oracle.h — C ABI of the CPU ORACLE (test infrastructure only).
 *
 * This library is the parity checker for the MI355X ray-tracing core.  It is a
 * plain C++ restatement of wtzhang23/gpu-ray-tracer's render path (every
 * function cites the reference file:line it follows).  It is NEVER linked into
 * or called by the product path: only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it.
 *
 * Parity pinning: the math primitives are pinned by
 * known-answer vectors produced by the reference's own raymath headers and
 * z_order.cu compiled unmodified with g++ (oracle/ref_kat, outputs in
 * oracle/_ref).  The integrator / BVH / scene-loader glue lives in reference
 * files that need CUDA, Thrust, rapidjson and SDL headers absent from this
 * image (not built here); it is pinned by the reference's own recorded outputs
 * in SURVEY.md Appendix D (ray / node / leaf / triangle-test totals, CPU-vs-GPU
 * pixel-difference counts, CPU-path ray totals), all reproduced exactly
 * (tests/test_oracle.py).  Per-pixel images have no reference fixture: they are
 * pinned only through those statistics and the committed oracle frames.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_scene orc_scene;

/* Integrator semantics */
enum { ORC_SEM_GPU = 0,   /* renv::gpu::propagate_ray (scene.cu:92-188) — the north-star semantics */
       ORC_SEM_CPU = 1 }; /* renv::cpu::Scene::propagate_helper (scene.cu:222-268) + ropt::cpu::BVH */

/* Load a worldN.json (cube_world.cc:38-191).  width/height <= 0 keep the JSON's values. */
int orc_load(const char* json_path, int width, int height, orc_scene** out);
void orc_free(orc_scene* s);
/* Build extension (not in the reference): textured shading -- a hit on a triangle with
 * TextureCoords takes its diffuse colour from the point-sampled atlas texel (byte/255),
 * JSON cubes' "texture": [tx, ty, size] map every face onto that square. */
int orc_set_atlas(orc_scene* s, const uint8_t* rgba8, int width, int height);
int orc_set_textures(orc_scene* s, int on);
const char* orc_last_error(void);

/* SceneBuilder (scene_builder.h:29-117): an empty scene, then the builder calls, then
 * finish (build_gpu_scene with Canvas W x H and Camera(fov radians, unit), Environment).
 * Index-returning calls return the new index (>= 0) or -1.  material26 as rt_amd.h. */
int orc_scene_create(orc_scene** out);
int orc_builder_add_vertex(orc_scene* s, float x, float y, float z);
int orc_builder_create_mesh(orc_scene* s, const float* pos3, const float* quat4);
int orc_builder_add_triangle(orc_scene* s, int mesh, int i0, int i1, int i2, const float* material26, const float* tex6);
int orc_builder_add_trans(orc_scene* s, int mesh);
int orc_builder_build_cube(orc_scene* s, float scale, const float* material26, const float* tile3);
int orc_builder_add_point_light(orc_scene* s, const float* pos3, const float* col4);
int orc_builder_add_directional_light(orc_scene* s, const float* dir3, const float* col4);
int orc_builder_finish(orc_scene* s, int width, int height, float fov, float unit, const float* cam_pos3,
                       const float* cam_quat4, const float* dist_atten3, const float* ambience4, int depth);
/* Camera / instance poses (Entity::set_position / set_orientation, entity.h:49-74) and
 * the Environment (ambience, distance attenuation, depth).  NULL leaves a field as is. */
int orc_set_camera(orc_scene* s, const float* pos3, const float* quat4);
int orc_set_trans(orc_scene* s, int trans, const float* pos3, const float* quat4);
int orc_set_env(orc_scene* s, const float* ambience4, const float* dist_atten3, int depth);

/* Scene introspection: counts = {W, H, n_vertices, n_tris, n_meshes, n_instances, n_lights, n_point, depth, n_mats} */
int orc_scene_counts(const orc_scene* s, int32_t* counts10);
/* float dumps of the scene exactly as the reference builds it */
int orc_scene_vertices(const orc_scene* s, float* xyz);        /* n_vertices*3 */
int orc_scene_normals(const orc_scene* s, float* xyz);         /* n_vertices*3 (generate_normals) */
int orc_scene_tris(const orc_scene* s, int32_t* idx4);         /* n_tris*4: i0,i1,i2,mat */
int orc_scene_materials(const orc_scene* s, float* m26);       /* n_mats*26: Ke,Ka,Kd,Ks,Kt,Kr (4 each), alpha, eta */
int orc_scene_instances(const orc_scene* s, float* q4p3, int32_t* mesh); /* n_instances*7 + n_instances */
int orc_scene_lights(const orc_scene* s, float* l8);           /* n_lights*8: (pos|dir)xyz, type(0 pt,1 dir), col rgba */
/* camera: pos(3) quat(4) near unit W H  r(3) u(3) f(3) ; env: dist_atten(3) ambience(4) */
int orc_scene_camera(const orc_scene* s, float* cam21, float* env7);

/* BVH exactly as ropt::gpu::BVH builds it (bvh.cu:74-91, raytracer.cu:54-89).
 * boxes: (2n-1)*7 floats: min xyz, max xyz, nondegenerate flag; storage order (root last).
 * ordering: n ints.  Returns n (padded leaf count). */
int orc_build_bvh(const orc_scene* s, float* boxes, int32_t* ordering, int max_n);

/* Render.  Rows rendered: y = row0, row0+row_step, ... < H.  Output arrays are
 * indexed by the full-frame pixel (y*W+x) and only the rendered rows are written.
 * rgba: packed R<<24|G<<16|B<<8|A (color.cu:23-26); radiance: float4 mean of
 * unclamped samples; hit_inst/hit_tri: primary hit of sample 0 (-1 on miss).
 * stats[4] = {rays (cast_ray calls), nodes (BVH node tests), leaves (cast_local calls), tri tests}.
 * Any output pointer may be NULL.  nthreads <= 0 -> 1. */
int orc_render(const orc_scene* s, int semantics, int use_bvh, int spp,
               int row0, int row_step, int nthreads,
               uint32_t* rgba, float* radiance, int32_t* hit_inst, int32_t* hit_tri,
               uint64_t* stats);

/* debug_cast (raytracer.cu:91-100): the event log ("shooting a ray", "preparing to shoot a
 * reflection ray", "preparing to shoot a refraction ray", "shooting shadow ray", one per line,
 * scene.cu:107-153 / light.cu:38-39) of pixel (x, y)'s ray, into buf (NUL-terminated). */
int orc_debug_cast(const orc_scene* s, int x, int y, int use_bvh, char* buf, int64_t cap);

/* Sub-pixel sample offset table (build-defined spp extension). */
void orc_spp_offset(int k, float* dx, float* dy);

/* ---- Known-answer entry points (element-wise over n inputs) ---- */
void orc_kat_normalize3(int n, const float* v, float* out);
void orc_kat_cross(int n, const float* a, const float* b, float* out);
void orc_kat_reflect(int n, const float* d, const float* nrm, float* out);
void orc_kat_refract(int n, const float* d, const float* nrm, const float* n1n2, float* out, int32_t* tir);
void orc_kat_quat_rotate(int n, const float* q, const float* v, float* out);   /* Quat*Vec3 */
void orc_kat_quat_inverse(int n, const float* q, float* out);
void orc_kat_quat_mul(int n, const float* a, const float* b, float* out);
void orc_kat_tri_hit(int n, const float* tri9, const float* ray6, int32_t* hit, float* t_uv3); /* ray built with Ray(o,d) */
void orc_kat_box_hit(int n, const float* box7, const float* ray6, int32_t* hit, float* t);
void orc_kat_zorder(int n, const float* v, uint64_t* out);
void orc_kat_box_from_local(int n, const float* box7, const float* entity7, float* out6, int32_t* nd);  /* from_local */
void orc_kat_box_merge(int n, const float* a7, const float* b7, float* out6, int32_t* nd);              /* merge */
void orc_kat_entity(int n, const float* entity7, const float* v3, float* out12);  /* Entity p/v to/from local */
/* Hitable::hit's pose step (HitHandle) around a local hit (t, n): local ray 6, time, normal 3 */
void orc_kat_hitable(int n, const float* entity7, const float* ray6, const float* hit4, float* out10);
void orc_kat_axis_angle(int n, const float* axis_theta4, float* out);          /* Quat(axis, theta), g++-TU cos/sin */
void orc_kat_to_mat3(int n, const float* q, float* out9);
void orc_kat_ray_ctor(int n, const float* ray6, float* out6);                   /* Ray(o,d): normalizes d */

#ifdef __cplusplus
}
#endif
#endif
