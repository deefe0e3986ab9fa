// rtracer_amd.hpp — the reference's C++ API for the render path, over the C ABI.
//
// A caller of wtzhang23/gpu-ray-tracer's
//   rtracer::gpu::update_scene / debug_cast          (include/raytracer.h:18-22)
//   procedural::gpu::generate                        (include/procedural/cube_world.h:20-23)
//   rtracer::SceneBuilder / MeshBuilder              (include/scene_builder.h:29-117)
//   renv::gpu::Scene::free, scene->get_environment().get_canvas() / get_camera()
//                                                    (include/rayenv/gpu/scene.h:55-69, environment.h:75-83,
//                                                     canvas.h:17-44, entity.h:49-74)
// compiles against this header unchanged in the calls its GPU path makes (main.cc:61-77, 81-216,
// including the camera moves and Canvas::get_surface when SDL.h comes first).  The CPU
// renderer (rtracer::cpu, procedural::cpu, renv::cpu::Scene; main.cc:45-60) is not shipped
// and not declared here: a caller drops its `-s` branch.
// The reference asserts on errors; so does this shim (message from rt_last_error()).
// Header-only; link with librt_amd.so.  Types are the reference's names with just the
// members these calls use.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <initializer_list>
#include <cstdlib>
#include <string>
#include <vector>

#include "rt_amd.h"

namespace rtamd_detail {
inline void check(int rc, const char* what) {
    if (rc != RT_OK) {
        std::fprintf(stderr, "%s failed (%d): %s\n", what, rc, rt_last_error());
        std::abort();
    }
}
}  // namespace rtamd_detail

namespace rmath {
// The vector / quaternion / ray operations the reference's callers use on the host
// (main.cc:140-180 moves and turns the camera with them), with linear.h / geometry.h's
// semantics: Vec(initializer_list) fills leading coordinates, normalized() returns the zero
// vector below the 1e-5 threshold (linear.h:159-167), Quat(axis, theta) = (axis sin(theta/2),
// cos(theta/2)) (geometry.h:36-41), Quat * Quat is the Hamilton product (geometry.h:150-170),
// Ray's direction is normalized at construction (geometry.h:216).
constexpr double THRESHOLD = 1E-5f;
template <class T, int Dim> class Vec {
    T c_[Dim];
public:
    Vec() { for (int i = 0; i < Dim; i++) c_[i] = T(0); }
    Vec(std::initializer_list<T> l) : Vec() { int i = 0; for (T x : l) { if (i >= Dim) break; c_[i++] = x; } }
    static Vec zero() { return Vec(); }
    T operator[](int i) const { return c_[i]; }
    T& operator[](int i) { return c_[i]; }
    friend Vec operator+(const Vec& a, const Vec& b) { Vec r; for (int i = 0; i < Dim; i++) r.c_[i] = a.c_[i] + b.c_[i]; return r; }
    friend Vec operator-(const Vec& a, const Vec& b) { Vec r; for (int i = 0; i < Dim; i++) r.c_[i] = a.c_[i] - b.c_[i]; return r; }
    friend Vec operator*(T k, const Vec& v) { Vec r; for (int i = 0; i < Dim; i++) r.c_[i] = k * v.c_[i]; return r; }
    friend Vec operator-(const Vec& v) { return T(-1) * v; }
    T squared_norm() const { T s = 0; for (int i = 0; i < Dim; i++) s += c_[i] * c_[i]; return s; }
    T len() const { return std::sqrt(squared_norm()); }
    Vec normalized() const { const T l = len(); return l > THRESHOLD ? (1 / l) * *this : Vec(); }
};
template <class T> using Vec3 = Vec<T, 3>;
template <class T> using Vec4 = Vec<T, 4>;
template <class T> struct Quat {          // (i, j, k, r) as geometry.h:20-181
    T i = 0, j = 0, k = 0, r = 1;
    Quat() = default;
    Quat(T i_, T j_, T k_, T r_) : i(i_), j(j_), k(k_), r(r_) {}
    // geometry.h:36-41 as a g++ translation unit compiles it (main.cc:175-176, cube_world.cc:173):
    // unqualified cos / sin of the float 0.5f * theta resolve to the C double functions there,
    // and the result is rounded to T.  std::cos(float) would round differently for some theta.
    Quat(Vec3<T> axis, T theta) {
        const T hc = static_cast<T>(::cos(static_cast<double>(0.5f * theta)));
        const T hs = static_cast<T>(::sin(static_cast<double>(0.5f * theta)));
        i = axis[0] * hs; j = axis[1] * hs; k = axis[2] * hs; r = hc;
    }
    static Quat identity() { return Quat(); }
    friend Quat operator*(const Quat& a, const Quat& b) {
        return Quat(a.i * b.r + a.r * b.i + a.j * b.k - a.k * b.j, a.j * b.r + a.r * b.j + a.k * b.i - a.i * b.k,
                    a.k * b.r + a.r * b.k + a.i * b.j - a.j * b.i, a.r * b.r - a.i * b.i - a.j * b.j - a.k * b.k);
    }
};
template <class T> class Ray {
    Vec3<T> o_, d_;
public:
    Ray() = default;
    Ray(Vec3<T> origin, Vec3<T> direction) : o_(origin), d_(direction.normalized()) {}
    Vec3<T> origin() const { return o_; }
    Vec3<T> direction() const { return d_; }
};
}  // namespace rmath

namespace rprimitives {
struct TextureCoords {};                  // atlas coordinates: accepted, not sampled
class Material {                          // material.h:14-31
public:
    rmath::Vec4<float> Ke, Ka, Kd, Ks, Kt, Kr;
    float alpha = 0, eta = 1;
    Material() = default;
    Material(rmath::Vec4<float> Ke_, rmath::Vec4<float> Ka_, rmath::Vec4<float> Kd_, rmath::Vec4<float> Ks_,
             rmath::Vec4<float> Kt_, rmath::Vec4<float> Kr_, float alpha_, float eta_)
        : Ke(Ke_), Ka(Ka_), Kd(Kd_), Ks(Ks_), Kt(Kt_), Kr(Kr_), alpha(alpha_), eta(eta_) {}
    void pack(float m[26]) const {
        const rmath::Vec4<float>* c[6] = {&Ke, &Ka, &Kd, &Ks, &Kt, &Kr};
        for (int a = 0; a < 6; a++) for (int b = 0; b < 4; b++) m[4 * a + b] = (*c[a])[b];
        m[24] = alpha; m[25] = eta;
    }
};
}  // namespace rprimitives

namespace renv {
struct Color {                            // color.h: RGBA8
    std::uint8_t r, g, b, a;
    std::uint8_t red() const { return r; }
    std::uint8_t green() const { return g; }
    std::uint8_t blue() const { return b; }
    std::uint8_t alpha() const { return a; }
};

class Canvas {                            // canvas.h:17-44
    rt_scene* s_ = nullptr;
    int w_, h_;
    friend class Environment;
    friend class SceneAccess;
public:
    Canvas(int width, int height) : w_(width), h_(height) {}
    int get_width() const { return w_; }
    int get_height() const { return h_; }
    Color get_color(int x, int y) const {
        std::uint8_t c[4];
        rtamd_detail::check(rt_canvas_get_color(s_, x, y, c), "Canvas::get_color");
        return Color{c[0], c[1], c[2], c[3]};
    }
    // The packed RGBA8 framebuffer (R<<24|G<<16|B<<8|A, row-major), the buffer the
    // reference hands to SDL in get_surface (canvas.cu:23-29).
    const std::uint32_t* get_buffer() const { return rt_canvas_host_ptr(s_); }
#if defined(SDL_h_)
    // Canvas::get_surface (canvas.cu:23-29), declared when SDL.h is included first (main.cc:1
    // does): an SDL surface over the host framebuffer, 32 bits per pixel, R in bits 31..24
    // (Color::rmask..amask, color.cu:38-56).  The buffer stays put across frames: each
    // update_scene refreshes what the surface shows, as the reference's managed canvas does.
    void get_surface(SDL_Surface** surface) {
        *surface = SDL_CreateRGBSurfaceFrom(const_cast<std::uint32_t*>(get_buffer()), w_, h_, 32, 4 * w_,
                                            0xff000000u, 0x00ff0000u, 0x0000ff00u, 0x000000ffu);
    }
#endif
};

class Camera {                            // camera.h (an Entity)
    rt_scene* s_ = nullptr;
    friend class Environment;
    friend class SceneAccess;
public:
    float fov, unit_to_pixels;
    rmath::Vec3<float> init_pos;
    rmath::Quat<float> init_rot;
    Camera(float fov_, float unit_to_pixels_, const Canvas&) : fov(fov_), unit_to_pixels(unit_to_pixels_) {}
    void translate(rmath::Vec3<float> dp) {           // Entity::translate: p += vec_to_local(dp)
        float d[3] = {dp[0], dp[1], dp[2]};
        if (s_) rtamd_detail::check(rt_camera_translate(s_, d), "Camera::translate");
        else for (int i = 0; i < 3; i++) init_pos[i] += dp[i];
    }
    void translate_global(rmath::Vec3<float> dp) {
        float p[3], q[4];
        rtamd_detail::check(rt_camera_get(s_, p, q), "Camera::translate_global");
        for (int i = 0; i < 3; i++) p[i] += dp[i];
        rtamd_detail::check(rt_camera_set(s_, p, nullptr), "Camera::translate_global");
    }
    void rotate(rmath::Quat<float> dr) {              // Entity::rotate: o = dr * o
        float q[4] = {dr.i, dr.j, dr.k, dr.r};
        rtamd_detail::check(rt_camera_rotate(s_, q), "Camera::rotate");
    }
    void set_position(rmath::Vec3<float> p) {
        float a[3] = {p[0], p[1], p[2]};
        if (s_) rtamd_detail::check(rt_camera_set(s_, a, nullptr), "Camera::set_position");
        else init_pos = p;
    }
    void set_orientation(rmath::Quat<float> o) {
        float q[4] = {o.i, o.j, o.k, o.r};
        if (s_) rtamd_detail::check(rt_camera_set(s_, nullptr, q), "Camera::set_orientation");
        else init_rot = o;
    }
    rmath::Vec3<float> pos() const {
        float p[3], q[4];
        rtamd_detail::check(rt_camera_get(s_, p, q), "Camera::pos");
        return {p[0], p[1], p[2]};
    }
    rmath::Ray<float> right() const { return axis(0); }
    rmath::Ray<float> up() const { return axis(1); }
    rmath::Ray<float> forward() const { return axis(2); }
private:
    rmath::Ray<float> axis(int which) const {    // camera.cu:11-31: Ray(pos, axis)
        float a[3][3];
        rtamd_detail::check(rt_camera_axes(s_, a[0], a[1], a[2]), "Camera axes");
        return rmath::Ray<float>(pos(), {a[which][0], a[which][1], a[which][2]});
    }
};

class Environment {                       // environment.h:19-93 (canvas + camera of a scene)
    Canvas canvas_;
    Camera camera_;
    friend class SceneAccess;
public:
    Environment(rt_scene* s, int w, int h) : canvas_(w, h), camera_(0, 0, canvas_) { canvas_.s_ = s; camera_.s_ = s; }
    Canvas& get_canvas() { return canvas_; }
    Camera& get_camera() { return camera_; }
};

namespace gpu {
class Scene {                             // rayenv/gpu/scene.h:32-110
    rt_scene* h_;
    Environment env_;
public:
    explicit Scene(rt_scene* h) : h_(h), env_(h, info(h, 0), info(h, 1)) {}
    Environment& get_environment() { return env_; }
    rt_scene* handle() const { return h_; }
    // Scene::free (scene.h:55-69): releases the device data; the Scene object itself is
    // the caller's, as in the reference.
    static void free(Scene& s) {
        if (s.h_) rtamd_detail::check(rt_scene_free(s.h_), "Scene::free");
        s.h_ = nullptr;
    }
private:
    static int info(rt_scene* h, int i) {
        int32_t v[10];
        rtamd_detail::check(rt_scene_info(h, v), "rt_scene_info");
        return v[i];
    }
};
}  // namespace gpu
}  // namespace renv

namespace rtracer {
namespace gpu {
// raytracer.cu:102-120: BVH rebuilt when `optimize`, one frame, synchronized; the
// framebuffer is host-readable through get_canvas() afterwards.
inline void update_scene(renv::gpu::Scene* scene, int kernel_dim, bool optimize) {
    rtamd_detail::check(rt_update_scene(scene->handle(), kernel_dim, optimize ? 1 : 0), "update_scene");
}
// Build extension: every later update_scene of `scene` renders row-cyclic
// slices on `devices` (n_ranks slices, default one per device) and gathers them to
// devices[0] with RCCL; the canvas is the whole frame as before (rt_scene_set_devices).
inline void use_devices(renv::gpu::Scene* scene, const std::vector<int>& devices, int n_ranks = 0) {
    rtamd_detail::check(rt_scene_set_devices(scene->handle(), devices.data(), (int)devices.size(),
                                             n_ranks > 0 ? n_ranks : (int)devices.size()), "use_devices");
}
// raytracer.cu:91-100: one-pixel trace with the reference's event log on stdout.
inline void debug_cast(renv::gpu::Scene* scene, int x, int y) {
    std::vector<char> buf(1 << 16);
    rtamd_detail::check(rt_debug_cast(scene->handle(), x, y, buf.data(), (int64_t)buf.size()), "debug_cast");
    std::fputs(buf.data(), stdout);
}
}  // namespace gpu

class SceneBuilder;
class MeshBuilder {                       // scene_builder.h:29-49
    int mesh_;
    std::vector<std::vector<int>> tris_;
    std::vector<rprimitives::Material> mats_;
    friend class SceneBuilder;
public:
    explicit MeshBuilder(int mesh) : mesh_(mesh) {}
    void add_triangle(rmath::Vec3<int> tri, rprimitives::TextureCoords, rprimitives::Material mat) {
        tris_.push_back({tri[0], tri[1], tri[2]});
        mats_.push_back(mat);
    }
};

class Transformation {                    // renv::Transformation (an Entity + mesh index)
    rt_scene* s_;
    int idx_;
public:
    Transformation(rt_scene* s, int idx) : s_(s), idx_(idx) {}
    void set_position(rmath::Vec3<float> p) {
        float a[3] = {p[0], p[1], p[2]};
        rtamd_detail::check(rt_builder_set_trans(s_, idx_, a, nullptr), "set_position");
    }
    void set_orientation(rmath::Quat<float> o) {
        float q[4] = {o.i, o.j, o.k, o.r};
        rtamd_detail::check(rt_builder_set_trans(s_, idx_, nullptr, q), "set_orientation");
    }
};

class SceneBuilder {                      // scene_builder.h:51-117
    rt_scene* s_ = nullptr;
    std::vector<MeshBuilder> meshes_;
    std::vector<Transformation> trans_;
    std::vector<int> flushed_;            // triangles of each mesh already handed to the C ABI
    void flush() {
        for (size_t m = 0; m < meshes_.size(); m++) {
            MeshBuilder& b = meshes_[m];
            for (size_t t = flushed_[m]; t < b.tris_.size(); t++) {
                float mat[26];
                b.mats_[t].pack(mat);
                rtamd_detail::check(rt_builder_add_triangle(s_, b.mesh_, b.tris_[t][0], b.tris_[t][1], b.tris_[t][2], mat),
                                    "add_triangle");
            }
            flushed_[m] = (int)b.tris_.size();
        }
    }
public:
    explicit SceneBuilder(std::string atlas_path) {
        rtamd_detail::check(rt_scene_create(atlas_path.c_str(), &s_), "SceneBuilder");
    }
    int add_vertex(rmath::Vec3<float> v) { return add_vertex(v[0], v[1], v[2]); }
    int add_vertex(float x, float y, float z) {
        int i;
        rtamd_detail::check(rt_builder_add_vertex(s_, x, y, z, &i), "add_vertex");
        return i;
    }
    int create_mesh(rmath::Vec3<float> pos, rmath::Quat<float> rot) {
        float p[3] = {pos[0], pos[1], pos[2]}, q[4] = {rot.i, rot.j, rot.k, rot.r};
        int m;
        rtamd_detail::check(rt_builder_create_mesh(s_, p, q, &m), "create_mesh");
        meshes_.emplace_back(m);
        flushed_.push_back(0);
        return m;
    }
    int create_mesh() { return create_mesh(rmath::Vec3<float>(), rmath::Quat<float>::identity()); }
    MeshBuilder& get_mesh_builder(int idx) { return meshes_[idx]; }
    Transformation& get_transformation(int idx) { return trans_[idx]; }
    int add_trans(const MeshBuilder& builder) {
        flush();
        int t;
        rtamd_detail::check(rt_builder_add_trans(s_, builder.mesh_, &t), "add_trans");
        trans_.emplace_back(s_, t);
        return t;
    }
    int build_cube(float scale, rprimitives::TextureCoords, rprimitives::Material mat) {
        flush();
        float m[26];
        mat.pack(m);
        int mesh;
        rtamd_detail::check(rt_builder_build_cube(s_, scale, m, &mesh), "build_cube");
        meshes_.emplace_back(mesh);
        flushed_.push_back(0);
        return mesh;
    }
    void add_directional_light(rmath::Vec3<float> dir, rmath::Vec4<float> col) {
        float d[3] = {dir[0], dir[1], dir[2]}, c[4] = {col[0], col[1], col[2], col[3]};
        rtamd_detail::check(rt_builder_add_directional_light(s_, d, c), "add_directional_light");
    }
    void add_point_light(rmath::Vec3<float> pos, rmath::Vec4<float> col) {
        float p[3] = {pos[0], pos[1], pos[2]}, c[4] = {col[0], col[1], col[2], col[3]};
        rtamd_detail::check(rt_builder_add_point_light(s_, p, c), "add_point_light");
    }
    // build_gpu_scene(Canvas, Camera) (scene_builder.cu:29-81).  The reference's
    // Environment defaults: no distance attenuation, no ambience; `depth` is this
    // build's explicit recursion depth (the reference takes it from the JSON).
    renv::gpu::Scene* build_gpu_scene(renv::Canvas canvas, renv::Camera camera, int depth = 0,
                                      rmath::Vec3<float> dist_atten = {}, rmath::Vec4<float> ambience = {}) {
        flush();
        float p[3] = {camera.init_pos[0], camera.init_pos[1], camera.init_pos[2]};
        float q[4] = {camera.init_rot.i, camera.init_rot.j, camera.init_rot.k, camera.init_rot.r};
        float da[3] = {dist_atten[0], dist_atten[1], dist_atten[2]};
        float am[4] = {ambience[0], ambience[1], ambience[2], ambience[3]};
        rtamd_detail::check(rt_builder_finish(s_, canvas.get_width(), canvas.get_height(), camera.fov,
                                              camera.unit_to_pixels, p, q, da, am, depth), "build_gpu_scene");
        rt_scene* h = s_;
        s_ = nullptr;
        return new renv::gpu::Scene(h);
    }
};
}  // namespace rtracer

namespace procedural {
namespace gpu {
// cube_world.cc:195-207: worldN.json -> scene (device upload happens at the first frame).
inline renv::gpu::Scene* generate(std::string config_path) {
    rt_scene* s = nullptr;
    rtamd_detail::check(rt_scene_load_json(config_path.c_str(), 0, 0, &s), "procedural::gpu::generate");
    return new renv::gpu::Scene(s);
}
}  // namespace gpu
}  // namespace procedural
