// Test driver for include/rtracer_amd.hpp: the calls the reference's GPU front end makes
// (main.cc:61-77 load/bench/free, :81-92 the SDL surface over the canvas, :140-180 camera
// moves and turns, :184 debug_cast), against the shim, in this build's own program.  SDL is
// absent from the image, so a minimal test double of the three SDL names get_surface uses is
// declared first (SDL_h_ is SDL2's include guard: the shim then declares get_surface).
//
//   shim_main CONFIG W H OUT
// Renders CONFIG (canvas resized to W x H), then moves the camera the way main.cc's key and
// mouse handlers do and renders again.  OUT (raw): the second frame's W*H uint32 words, then
// the camera pose (px py pz qi qj qk qr, float32).  The test renders the oracle at that pose.
#define SDL_h_ 1
#include <cstdint>
struct SDL_Surface {
    void* pixels;
    int w, h, depth, pitch;
    std::uint32_t rmask, gmask, bmask, amask;
};
static SDL_Surface g_surface;
static SDL_Surface* SDL_CreateRGBSurfaceFrom(void* pixels, int w, int h, int depth, int pitch, std::uint32_t rm,
                                             std::uint32_t gm, std::uint32_t bm, std::uint32_t am) {
    g_surface = SDL_Surface{pixels, w, h, depth, pitch, rm, gm, bm, am};
    return &g_surface;
}

#include <cstdio>
#include <cstring>

#include "rtracer_amd.hpp"

int main(int argc, char** argv) {
    if (argc != 5) return 2;
    const int W = std::atoi(argv[2]), H = std::atoi(argv[3]);
    // procedural::gpu::generate keeps the JSON's canvas; this test wants a small frame, so it
    // loads through the C ABI with a size and wraps the handle the way generate() does
    rt_scene* h = nullptr;
    if (rt_scene_load_json(argv[1], W, H, &h) != RT_OK) { std::fprintf(stderr, "%s\n", rt_last_error()); return 3; }
    renv::gpu::Scene* scene = new renv::gpu::Scene(h);
    renv::Environment& env = scene->get_environment();
    std::printf("Loaded scene\n");
    rtracer::gpu::update_scene(scene, 16, true);

    SDL_Surface* surface = nullptr;
    env.get_canvas().get_surface(&surface);                  // main.cc:90-92
    if (!surface || surface->pixels != (const void*)env.get_canvas().get_buffer() || surface->w != W ||
        surface->h != H || surface->depth != 32 || surface->pitch != 4 * W || surface->rmask != 0xff000000u ||
        surface->amask != 0x000000ffu) {
        std::fprintf(stderr, "get_surface does not wrap the canvas\n");
        return 4;
    }
    const std::uint32_t first = env.get_canvas().get_buffer()[(H / 2) * W + W / 2];

    // key handler (main.cc:144-165): w / a, then d and s with the same speed
    const float MOVE = 0.2f, ROT = 0.01f;
    renv::Camera& cam = env.get_camera();
    cam.translate(rmath::Vec3<float>{0, 0, MOVE});
    cam.translate(rmath::Vec3<float>{-MOVE, 0, 0});
    cam.translate(rmath::Vec3<float>{0, 0, MOVE});
    // mouse handler (main.cc:169-178), relative motion (7, -3)
    rmath::Vec<float, 2> rel = rmath::Vec<float, 2>({7.0f, -3.0f}).normalized();
    rmath::Vec3<float> global = rel[0] * cam.right().direction() + rel[1] * cam.up().direction();
    (void)global;
    rmath::Quat<float> rot = rmath::Quat<float>(cam.up().direction(), ROT * rel[0]) *
                             rmath::Quat<float>(cam.right().direction(), ROT * rel[1]);
    cam.rotate(rot);
    rtracer::gpu::update_scene(scene, 16, true);             // the window loop's draw()
    rtracer::gpu::debug_cast(scene, W / 2, H / 2);           // main.cc:181-185

    FILE* o = std::fopen(argv[4], "wb");
    if (!o) return 5;
    // the surface still shows the canvas: the second frame is what SDL would blit
    std::fwrite(surface->pixels, 4, (size_t)W * H, o);
    float p[3], q[4];
    if (rt_camera_get(scene->handle(), p, q) != RT_OK) return 6;
    std::fwrite(p, 4, 3, o);
    std::fwrite(q, 4, 4, o);
    std::fclose(o);
    std::printf("centre pixel %08x -> %08x\n", first, env.get_canvas().get_buffer()[(H / 2) * W + W / 2]);
    renv::gpu::Scene::free(*scene);
    delete scene;
    return 0;
}
