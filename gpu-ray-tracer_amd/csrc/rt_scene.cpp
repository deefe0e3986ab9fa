// rt_scene.cpp — worldN.json loader, cube-world generator and SceneBuilder
// semantics of wtzhang23/gpu-ray-tracer, producing the flat HBM layout.
//
// Float-exactness notes (they decide which instances exist and where the camera
// is, so they are part of parity):
//  * cube_world.cc and scene_builder.cc are g++ translation units in the
//    reference: `cos`/`sin` of a float there are the C double functions, and
//    `floor` runs in double (cube_world.cc:159).
//  * perlin.cu and camera.cu are nvcc translation units: acos/cos/sin/floor/tan
//    of floats are the float functions (perlin.cu:40-42, 90-92; camera.cu:7).
//  * rapidjson's GetFloat is (float)GetDouble; numbers are parsed with strtod.
//  * std::mt19937 / uniform_real_distribution<float> / uniform_int_distribution
//    come from libstdc++ exactly as in the reference build (perlin.cu:84-101).
#include "rt_scene.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <map>
#include <random>
#include <sstream>
#include <stdexcept>

#include <zlib.h>

namespace rt {
using namespace rtm;

namespace {

// ---- small JSON reader (the subset cube_world.cc reads through rapidjson) ----
struct Json {
    enum Kind { Null, Num, Str, Arr, Obj, Bool } kind = Null;
    double num = 0;
    std::string str;
    std::vector<Json> arr;
    std::vector<std::pair<std::string, Json>> obj;
    const Json* get(const char* k) const {
        if (kind != Obj) return nullptr;
        for (auto& kv : obj) if (kv.first == k) return &kv.second;
        return nullptr;
    }
    bool has(const char* k) const { return get(k) != nullptr; }
    const Json& at(const char* k) const {
        const Json* j = get(k);
        if (!j) throw std::runtime_error(std::string("missing key '") + k + "'");
        return *j;
    }
    const Json& at(int i) const {
        if (kind != Arr || i < 0 || (size_t)i >= arr.size()) throw std::runtime_error("array index out of range");
        return arr[i];
    }
    double number() const {
        if (kind != Num) throw std::runtime_error("expected a number");
        return num;
    }
};

class JsonReader {
  public:
    JsonReader(const char* b, const char* e) : p_(b), e_(e) {}
    Json document() { Json j = value(); skip(); if (p_ != e_) fail("trailing characters"); return j; }

  private:
    const char* p_; const char* e_;
    [[noreturn]] void fail(const char* what) { throw std::runtime_error(std::string("json: ") + what); }
    void skip() { while (p_ < e_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) ++p_; }
    bool lit(const char* s) { size_t n = strlen(s); if ((size_t)(e_ - p_) >= n && !memcmp(p_, s, n)) { p_ += n; return true; } return false; }
    std::string string_token() {
        if (*p_ != '"') fail("expected string");
        ++p_;
        std::string s;
        while (p_ < e_ && *p_ != '"') {
            if (*p_ == '\\' && p_ + 1 < e_) { ++p_; char c = *p_; s.push_back(c == 'n' ? '\n' : c == 't' ? '\t' : c); ++p_; continue; }
            s.push_back(*p_++);
        }
        if (p_ >= e_) fail("unterminated string");
        ++p_;
        return s;
    }
    Json value() {
        skip();
        if (p_ >= e_) fail("unexpected end of input");
        Json j;
        if (*p_ == '{') {
            j.kind = Json::Obj; ++p_; skip();
            if (*p_ == '}') { ++p_; return j; }
            for (;;) {
                skip(); std::string k = string_token(); skip();
                if (p_ >= e_ || *p_ != ':') fail("expected ':'");
                ++p_;
                j.obj.emplace_back(k, value());
                skip();
                if (p_ < e_ && *p_ == ',') { ++p_; continue; }
                if (p_ < e_ && *p_ == '}') { ++p_; break; }
                fail("expected ',' or '}'");
            }
        } else if (*p_ == '[') {
            j.kind = Json::Arr; ++p_; skip();
            if (*p_ == ']') { ++p_; return j; }
            for (;;) {
                j.arr.push_back(value()); skip();
                if (p_ < e_ && *p_ == ',') { ++p_; continue; }
                if (p_ < e_ && *p_ == ']') { ++p_; break; }
                fail("expected ',' or ']'");
            }
        } else if (*p_ == '"') {
            j.kind = Json::Str; j.str = string_token();
        } else if (lit("true")) { j.kind = Json::Bool; j.num = 1; }
        else if (lit("false")) { j.kind = Json::Bool; }
        else if (lit("null")) { j.kind = Json::Null; }
        else {
            std::string tok;
            while (p_ < e_ && (isdigit((unsigned char)*p_) || *p_ == '-' || *p_ == '+' || *p_ == '.' || *p_ == 'e' || *p_ == 'E')) tok.push_back(*p_++);
            if (tok.empty()) fail("unexpected character");
            char* end = nullptr;
            j.kind = Json::Num; j.num = strtod(tok.c_str(), &end);
            if (!end || *end) fail("bad number");
        }
        return j;
    }
};

float get_float(const Json& j) { return (float)j.number(); }            // rapidjson GetFloat
V3 read_vec3(const Json& v) { return v3(get_float(v.at(0)), get_float(v.at(1)), get_float(v.at(2))); }
V4 read_vec4(const Json& v) { return v4(get_float(v.at(0)), get_float(v.at(1)), get_float(v.at(2)), get_float(v.at(3))); }

// ---- Perlin height field (perlin.cu; float transcendental overloads) ----
class Perlin {
  public:
    Perlin(int seed, int n) : n_(n) {
        std::mt19937 gen(seed);
        auto rng = std::bind(std::uniform_real_distribution<float>{}, gen);   // binds a COPY of gen
        dirs_.resize(n); perm_.resize(n);
        for (int i = 0; i < n; i++) {
            float theta = acosf(2 * rng() - 1);
            float phi = (float)(2 * rng() * M_PI);
            dirs_[i] = normalized(v3(cosf(phi) * sinf(theta), sinf(phi) * sinf(theta), cosf(theta)));
            perm_[i] = i;
        }
        auto rng_int = std::bind(std::uniform_int_distribution<unsigned>{}, gen);  // restarts from the seed state
        for (int i = 0; i < n; i++) std::swap(perm_[i], perm_[rng_int() % n]);
    }
    float amplitude = 1.0f, period = 1.0f;

    float sample(float x, float y, float z) const {
        float gx = x * n_ / period, gy = y * n_ / period, gz = z * n_ / period;
        int ix = (int)floorf(gx) % n_, iy = (int)floorf(gy) % n_, iz = (int)floorf(gz) % n_;
        float mx = smooth(gx - floorf(gx)), my = smooth(gy - floorf(gy)), mz = smooth(gz - floorf(gz));
        auto weight = [&](int dx, int dy, int dz) {
            float cx = ix + dx, cy = iy + dy, cz = iz + dz;
            V3 off = v3(dx - mx, dy - my, dz - mz);
            return dot(corner((int)cx, (int)cy, (int)cz), normalized(off));
        };
        float w000 = weight(0, 0, 0), w001 = weight(0, 0, 1), w010 = weight(0, 1, 0), w011 = weight(0, 1, 1);
        float w100 = weight(1, 0, 0), w101 = weight(1, 0, 1), w110 = weight(1, 1, 0), w111 = weight(1, 1, 1);
        float x00 = lerp(w000, w100, mx), x01 = lerp(w001, w101, mx), x10 = lerp(w010, w110, mx), x11 = lerp(w011, w111, mx);
        float xy0 = lerp(x00, x10, my), xy1 = lerp(x01, x11, my);
        return amplitude * lerp(xy0, xy1, mz);
    }

  private:
    int n_;
    std::vector<V3> dirs_;
    std::vector<int> perm_;
    static float smooth(float d) { return d * d * (3 - 2 * d); }
    static float lerp(float a, float b, float w) { return w * a + (1 - w) * b; }
    const V3& corner(int x, int y, int z) const {
        int hx = x % n_, hxy = (perm_[hx] + y) % n_, hxyz = (perm_[hxy] + z) % n_;
        return dirs_[perm_[hxyz]];
    }
};

}  // namespace

// SceneBuilder::build_cube (scene_builder.cu:181-239): 12 triangles, 36 unshared vertices.
int Scene::build_cube(float scale, const Material& mat, const float* tile) {
    const V3 A = scale * v3(-0.5f, 0.5f, -0.5f), B = scale * v3(0.5f, 0.5f, -0.5f);
    const V3 C = scale * v3(-0.5f, -0.5f, -0.5f), D = scale * v3(0.5f, -0.5f, -0.5f);
    const V3 E = scale * v3(-0.5f, 0.5f, 0.5f), F = scale * v3(0.5f, 0.5f, 0.5f);
    const V3 G = scale * v3(-0.5f, -0.5f, 0.5f), Hh = scale * v3(0.5f, -0.5f, 0.5f);
    int m = create_mesh(v3(0, 0, 0), Q{0, 0, 0, 1});
    int mi = add_material(mat);
    const V3* faces[12][3] = {{&D, &A, &B}, {&C, &A, &D},     // front
                              {&A, &E, &B}, {&E, &F, &B},     // top
                              {&D, &B, &Hh}, {&B, &F, &Hh},   // right
                              {&C, &G, &A}, {&A, &G, &E},     // left
                              {&G, &Hh, &E}, {&E, &Hh, &F},   // back
                              {&G, &C, &D}, {&D, &Hh, &G}};   // bottom
    // Texture tile (build-defined): face-local (s, t) in [-scale/2, scale/2] -> the
    // square [tx, tx+size] x [ty, ty+size] of the atlas, image rows downwards.
    // Faces in the order above: front/back use (x, y), top/bottom (x, z), right/left (z, y).
    static const int face_axes[6][2] = {{0, 1}, {0, 2}, {2, 1}, {2, 1}, {0, 1}, {0, 2}};
    for (int k = 0; k < 12; k++) {
        const V3* const* f = faces[k];
        int i0 = add_vertex(*f[0]), i1 = add_vertex(*f[1]), i2 = add_vertex(*f[2]);
        TexDesc tex;
        if (tile) {
            const int* ax = face_axes[k / 2];
            auto T = [&](const V3& p, float* o) {
                const float c[3] = {p.x, p.y, p.z};
                o[0] = tile[0] + (c[ax[0]] / scale + 0.5f) * tile[2];
                o[1] = tile[1] + (0.5f - c[ax[1]] / scale) * tile[2];
            };
            float t0[2], t1[2], t2[2];
            T(*f[0], t0); T(*f[1], t1); T(*f[2], t2);
            tex.has = 1;
            tex.tx = t0[0]; tex.ty = t0[1];
            tex.ux = t1[0] - t0[0]; tex.uy = t1[1] - t0[1];
            tex.vx = t2[0] - t0[0]; tex.vy = t2[1] - t0[1];
        }
        add_triangle(m, i0, i1, i2, mi, tex);
    }
    return m;
}

void Scene::generate_normals() {
    norms.assign(verts.size(), v3(0, 0, 0));
    for (const MeshDesc& m : meshes)
        for (int t : m.tris) {
            const TriDesc& tr = tris[t];
            V3 n = normalized(cross(verts[tr.i1] - verts[tr.i0], verts[tr.i2] - verts[tr.i0]));
            norms[tr.i0] = norms[tr.i0] + n;
            norms[tr.i1] = norms[tr.i1] + n;
            norms[tr.i2] = norms[tr.i2] + n;
        }
    for (V3& n : norms) n = normalized(n);
}

void Scene::set_camera(int W, int H, float fov, float unit) {
    cam.W = W; cam.H = H; cam.fov = fov; cam.unit = unit;
    cam.near_ = 0.5f * W / unit / tanf(fov);                     // camera.cu:7 (float tan)
}

void Scene::update_camera_basis() {
    float m[3][3];
    to_mat3(cam.rot, m);
    d_cam.pos = cam.pos;
    d_cam.r = normalized(v3(m[0][0], m[1][0], m[2][0]));
    d_cam.u = normalized(v3(m[0][1], m[1][1], m[2][1]));
    d_cam.f = normalized(v3(m[0][2], m[1][2], m[2][2]));
    d_cam.near_ = cam.near_; d_cam.unit = cam.unit;
    d_cam.W = (float)cam.W; d_cam.H = (float)cam.H;
}

int Scene::flatten(std::string* err) {
    for (const TriDesc& t : tris)
        if (t.i0 < 0 || t.i1 < 0 || t.i2 < 0 || t.i0 >= (int)verts.size() || t.i1 >= (int)verts.size() ||
            t.i2 >= (int)verts.size() || t.mat < 0 || t.mat >= (int)mats.size()) {
            if (err) *err = "triangle references a missing vertex or material";
            return -1;
        }
    for (const InstDesc& t : insts)
        if (t.mesh < 0 || t.mesh >= (int)meshes.size()) { if (err) *err = "instance references a missing mesh"; return -1; }
    if (depth >= 10) { if (err) *err = "depth must be <= 9 (the reference's frame stack holds MAX_DEPTH=10 frames)"; return -1; }
    generate_normals();
    d_tris.clear(); d_meshes.clear(); d_insts.clear(); d_mats.clear(); d_lights.clear();
    for (const MeshDesc& m : meshes) {
        DMesh dm{};
        dm.pose = make_pose(m.rot, m.pos);
        dm.tri_begin = (int)d_tris.size();
        dm.tri_count = (int)m.tris.size();
        for (int t : m.tris) {
            const TriDesc& tr = tris[t];
            DTri d{};
            d.a = verts[tr.i0]; d.b = verts[tr.i1]; d.c = verts[tr.i2];
            V3 pn = cross(d.b - d.a, d.c - d.a);                 // Triangle::hit (geometry.h:275-276)
            d.pn = normalized(pn);                               // Plane ctor (geometry.h:233)
            d.area = len(pn);                                    // geometry.h:280
            d.inv_area = 1.0f / d.area;
            d.mat = tr.mat;
            d.tex = tr.tex.has;
            d.tx = tr.tex.tx; d.ty = tr.tex.ty; d.ux = tr.tex.ux; d.uy = tr.tex.uy; d.vx = tr.tex.vx; d.vy = tr.tex.vy;
            d.n0 = norms[tr.i0]; d.n1 = norms[tr.i1]; d.n2 = norms[tr.i2];
            d_tris.push_back(d);
        }
        d_meshes.push_back(dm);
    }
    for (const InstDesc& t : insts) { DInst di{}; di.pose = make_pose(t.rot, t.pos); di.mesh = t.mesh; d_insts.push_back(di); }
    for (const Material& m : mats) {
        DMat d{};
        d.Ke = m.Ke; d.Ka = m.Ka; d.Kd = m.Kd; d.Ks = m.Ks; d.Kt = m.Kt; d.Kr = m.Kr; d.alpha = m.alpha; d.eta = m.eta;
        d.reflective = m.Kr.x > 0.0f || m.Kr.y > 0.0f || m.Kr.z > 0.0f || m.Kr.w > 0.0f;   // material.h:106-108
        d.refractive = m.Kt.x > 0.0f || m.Kt.y > 0.0f || m.Kt.z > 0.0f || m.Kt.w > 0.0f;   // material.h:110-112
        d_mats.push_back(d);
    }
    for (const LightDesc& l : points) d_lights.push_back(DLight{l.v, 0, l.col});
    for (const LightDesc& l : dirs) d_lights.push_back(DLight{l.v, 1, l.col});
    verts_norm.clear();
    for (const V3& n : norms) { verts_norm.push_back(n.x); verts_norm.push_back(n.y); verts_norm.push_back(n.z); }
    update_camera_basis();
    return 0;
}

int load_cube_world(const std::string& path, int width, int height, Scene* s, std::string* err) {
    try {
        std::ifstream f(path);
        if (!f) { if (err) *err = "cannot open " + path; return -2; }
        std::stringstream ss; ss << f.rdbuf();
        std::string txt = ss.str();
        Json doc = JsonReader(txt.data(), txt.data() + txt.size()).document();
        if (doc.kind != Json::Obj) throw std::runtime_error("top level is not an object");

        int seed = 42, grid = 8, W = 640, H = 480;                 // cube_world.cc:14-20 defaults
        float fov = (float)M_PI / 4, unit = 200;
        if (doc.has("seed")) seed = (int)doc.at("seed").number();
        if (doc.has("grid_size")) grid = (int)doc.at("grid_size").number();
        if (doc.has("width")) W = (int)doc.at("width").number();
        if (doc.has("height")) H = (int)doc.at("height").number();
        if (doc.has("fov")) fov = (float)(doc.at("fov").number() * M_PI) / 180;
        if (doc.has("unit_length")) unit = (float)doc.at("unit_length").number();
        if (width > 0) W = width;
        if (height > 0) H = height;
        if (W <= 0 || H <= 0) throw std::runtime_error("canvas size must be positive");
        if (grid < 0) throw std::runtime_error("grid_size must be >= 0");
        s->atlas = doc.has("atlas") ? doc.at("atlas").str : std::string();
        const size_t slash = path.find_last_of('/');
        s->base_dir = slash == std::string::npos ? std::string(".") : path.substr(0, slash);
        s->set_camera(W, H, fov, unit);

        const float inv255 = 1.0f / 255;                          // 1.0f / UINT8_MAX
        int n_cubes = 0;
        if (doc.has("cubes")) {
            const Json& cubes = doc.at("cubes");
            n_cubes = (int)cubes.arr.size();
            for (int i = 0; i < n_cubes; i++) {
                const Json& c = cubes.at(i);
                Material m;
                if (c.has("Ke")) m.Ke = inv255 * read_vec4(c.at("Ke"));
                if (c.has("Ka")) m.Ka = inv255 * read_vec4(c.at("Ka"));
                if (c.has("Kd")) m.Kd = inv255 * read_vec4(c.at("Kd"));
                if (c.has("Ks")) m.Ks = inv255 * read_vec4(c.at("Ks"));
                if (c.has("Kt")) m.Kt = read_vec4(c.at("Kt"));
                if (c.has("Kr")) m.Kr = read_vec4(c.at("Kr"));
                if (c.has("alpha")) m.alpha = (float)c.at("alpha").number();
                if (c.has("eta")) m.eta = (float)c.at("eta").number();
                // "texture": [tx, ty, size] (build-defined; the reference leaves this key a
                // TODO, cube_world.cc:79-81, so it changes nothing unless textures are on)
                float tile[3];
                const bool tex = c.has("texture") && c.at("texture").arr.size() == 3;
                if (tex) for (int k = 0; k < 3; k++) tile[k] = (float)c.at("texture").at(k).number();
                s->build_cube(.999f, m, tex ? tile : nullptr);
            }
        }
        if (doc.has("lights")) {
            const Json& L = doc.at("lights");
            if (L.has("directional"))
                for (const Json& l : L.at("directional").arr) s->add_directional_light(read_vec3(l.at("dir")), inv255 * read_vec4(l.at("col")));
            if (L.has("point"))
                for (const Json& l : L.at("point").arr) s->add_point_light(read_vec3(l.at("pos")), inv255 * read_vec4(l.at("col")));
        }
        float amplitude = 1.0f;
        if (doc.has("amplitude")) amplitude = (float)doc.at("amplitude").number();
        std::vector<float> last((size_t)grid * grid, 0.0f);
        float max_h = 0.0f;
        for (int c = 0; c < n_cubes; c++) {                       // cube_world.cc:149-170 (same seed every layer)
            Perlin perlin(seed, (grid + 4) / 5);
            perlin.amplitude = amplitude;
            perlin.period = (float)grid;
            for (int i = 0; i < grid; i++)
                for (int j = 0; j < grid; j++) {
                    float x = i - grid / 2.0f, z = j - grid / 2.0f;
                    float y_off = (float)(floor((double)(0.5f * (perlin.sample((float)i, (float)j, 0.0f) + amplitude))) + 1);
                    for (int d = 0; d < y_off; d++) {
                        int t = s->add_trans(c);
                        s->insts[t].pos = v3(x, last[(size_t)i * grid + j] + d, z);
                    }
                    last[(size_t)i * grid + j] += y_off;
                    max_h = std::max(max_h, last[(size_t)i * grid + j]);
                }
        }
        s->cam.pos = v3(0.0f, max_h + 10.0f, -(float)grid / 2);      // cube_world.cc:172
        s->cam.rot = axis_angle_gxx(v3(1.0f, 0.0f, 0.0f), 45);      // cube_world.cc:173 (45 radians)
        if (doc.has("ambience")) s->ambience = read_vec4(doc.at("ambience"));   // finish_env :177-191
        if (doc.has("depth")) s->depth = (int)doc.at("depth").number();
        if (doc.has("distance_attenuation")) {
            const Json& a = doc.at("distance_attenuation");
            s->dist_atten = v3((float)a.at("constant_term").number(), (float)a.at("linear_term").number(),
                               (float)a.at("quadratic_term").number());
        }
        return s->flatten(err) == 0 ? 0 : -3;
    } catch (const std::exception& e) {
        if (err) *err = e.what();
        return -3;
    }
}

void spp_offset(int k, float* dx, float* dy) {
    const double a1 = 0.7548776662466927, a2 = 0.5698402909980532;   // 1/phi2, 1/phi2^2 (R2 sequence)
    double u = (double)k * a1, v = (double)k * a2;
    *dx = (float)(u - floor(u));
    *dy = (float)(v - floor(v));
}

// Atlas PNG (assets.cc:11-57 reads it with libpng; this build uses zlib directly).
// Supports what the reference's atlas is: 8-bit RGBA (colour type 6) or RGB (2),
// non-interlaced; RGB gets alpha 255.
int load_png_rgba8(const std::string& path, std::vector<uint8_t>* out, int* w, int* h, std::string* err) {
    auto fail = [&](const std::string& m) { if (err) *err = path + ": " + m; return -1; };
    std::ifstream f(path, std::ios::binary);
    if (!f) return fail("cannot open");
    std::vector<uint8_t> d((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0d, 0x0a, 0x1a, 0x0a};
    if (d.size() < 8 || memcmp(d.data(), sig, 8) != 0) return fail("not a PNG file");
    auto be32 = [&](size_t o) { return (uint32_t)d[o] << 24 | (uint32_t)d[o + 1] << 16 | (uint32_t)d[o + 2] << 8 | d[o + 3]; };
    uint32_t W = 0, H = 0;
    int depth = 0, ctype = 0, interlace = 0;
    std::vector<uint8_t> idat;
    for (size_t o = 8; o + 12 <= d.size();) {
        const uint32_t n = be32(o);
        if (o + 12 + (size_t)n > d.size()) return fail("truncated chunk");
        const std::string type(reinterpret_cast<const char*>(&d[o + 4]), 4);
        const uint8_t* c = &d[o + 8];
        if (type == "IHDR" && n >= 13) {
            W = be32(o + 8); H = be32(o + 12); depth = c[8]; ctype = c[9]; interlace = c[12];
        } else if (type == "IDAT") {
            idat.insert(idat.end(), c, c + n);
        } else if (type == "IEND") {
            break;
        }
        o += 12 + (size_t)n;
    }
    if (!W || !H || W > 16384 || H > 16384) return fail("bad image size");
    if (depth != 8 || (ctype != 6 && ctype != 2) || interlace) return fail("only 8-bit RGB/RGBA non-interlaced PNGs");
    const int bpp = ctype == 6 ? 4 : 3;
    const size_t stride = (size_t)W * bpp;
    std::vector<uint8_t> raw((stride + 1) * H);
    uLongf raw_len = (uLongf)raw.size();
    if (uncompress(raw.data(), &raw_len, idat.data(), (uLong)idat.size()) != Z_OK || raw_len != raw.size())
        return fail("corrupt image data");
    std::vector<uint8_t> img(stride * H);
    for (uint32_t y = 0; y < H; y++) {                       // undo the scanline filters (PNG spec 9.2)
        const uint8_t* src = &raw[y * (stride + 1)];
        uint8_t* row = &img[y * stride];
        const uint8_t* up = y ? &img[(y - 1) * stride] : nullptr;
        for (size_t x = 0; x < stride; x++) {
            const int a = x >= (size_t)bpp ? row[x - bpp] : 0, b = up ? up[x] : 0;
            const int c = (up && x >= (size_t)bpp) ? up[x - bpp] : 0;
            int v = src[1 + x];
            switch (src[0]) {
                case 0: break;
                case 1: v += a; break;
                case 2: v += b; break;
                case 3: v += (a + b) / 2; break;
                case 4: {
                    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
                    v += (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
                    break;
                }
                default: return fail("bad filter type");
            }
            row[x] = (uint8_t)v;
        }
    }
    out->assign((size_t)W * H * 4, 255);
    for (size_t i = 0; i < (size_t)W * H; i++)
        for (int k = 0; k < bpp; k++) (*out)[4 * i + k] = img[i * bpp + k];
    *w = (int)W; *h = (int)H;
    return 0;
}

}  // namespace rt
