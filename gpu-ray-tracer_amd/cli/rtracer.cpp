// rtracer — headless front end with the reference's command line (src/main.cc:31-79).
//
//   rtracer -c world8.json [-b] [-r] [-s] [-d DIM] [--frames N] [--spp K]
//           [--width W --height H] [--out frame.ppm] [--debug X,Y] [--textures [ATLAS.png]]
//           [--gpus N [--ranks R]] [--in-flight D]
//
// -c config (worldN.json), -b benchmark (one timed frame, "Time: X ms" as main.cc:210-216),
// -r unoptimize (brute force, no BVH), -d kernel dimension (accepted; the HIP path
// tiles itself), -s serial CPU path: not part of this build (the CPU restatement lives
// in oracle/ as test infrastructure), so it is rejected.  Without -b the reference
// opens an SDL window and renders continuously; headless, this renders --frames frames
// (default 1) through rtracer::gpu::update_scene and prints the frame rate.  --spp > 1
// uses the build's multi-sample extension (rt_render).  --debug X,Y runs debug_cast.
// --textures turns on the build-defined textured shading mode with the scene's atlas
// (or the given PNG).  --gpus N splits every frame row-cyclically over devices 0..N-1 of this
// process (R slices, default N; RCCL gather to device 0: rtracer::gpu::use_devices).
// --in-flight D (timing, build extension): --frames frames issued asynchronously with D in
// flight (rt_scene_set_frame_slots), each into its own device buffer on its own stream, then
// one wait; prints the time per frame and per slice.  --out then writes the last frame.
// --overlap sets the frames' grid policy (rt_scene_set_overlap; default stream).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <string>
#include <vector>

#include "rtracer_amd.hpp"

static void usage() {
    std::fprintf(stderr,
                 "usage: rtracer -c CONFIG [-b] [-r] [-s] [-d DIM] [--frames N] [--spp K] [--width W --height H]\n"
                 "               [--out FILE.ppm] [--debug X,Y] [--textures [ATLAS.png]] [--gpus N [--ranks R]]\n"
                 "               [--in-flight D [--readback] [--overlap stream|half|full]]\n");
}

static bool write_ppm(const char* path, const uint32_t* px, int w, int h) {
    FILE* f = std::fopen(path, "wb");
    if (!f) return false;
    std::fprintf(f, "P6\n%d %d\n255\n", w, h);
    std::vector<unsigned char> row(3 * (size_t)w);
    for (int y = 0; y < h; y++) {
        for (int x = 0; x < w; x++) {
            const uint32_t v = px[(size_t)y * w + x];
            row[3 * x] = (unsigned char)(v >> 24); row[3 * x + 1] = (unsigned char)(v >> 16);
            row[3 * x + 2] = (unsigned char)(v >> 8);
        }
        std::fwrite(row.data(), 1, row.size(), f);
    }
    return std::fclose(f) == 0;
}

int main(int argc, char** argv) {
    std::string config, out;
    bool bench = false, unopt = false, serial = false, textures = false, readback = false;
    std::string atlas, overlap = "stream";
    int dim = 16, frames = 1, spp = 1, width = 0, height = 0, dbg_x = -1, dbg_y = -1, gpus = 1, ranks = 0, in_flight = 0;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        auto val = [&](const char* name) -> const char* {
            if (i + 1 >= argc) { std::fprintf(stderr, "%s needs a value\n", name); usage(); std::exit(2); }
            return argv[++i];
        };
        if (a == "-c" || a == "--config") config = val("-c");
        else if (a == "-b" || a == "--bench") bench = true;
        else if (a == "-r" || a == "--unoptimize") unopt = true;
        else if (a == "-s" || a == "--serial") serial = true;
        else if (a == "-d" || a == "--dim") dim = std::atoi(val("-d"));
        else if (a == "--frames") frames = std::atoi(val("--frames"));
        else if (a == "--spp") spp = std::atoi(val("--spp"));
        else if (a == "--width") width = std::atoi(val("--width"));
        else if (a == "--height") height = std::atoi(val("--height"));
        else if (a == "--out") out = val("--out");
        else if (a == "--gpus") gpus = std::atoi(val("--gpus"));
        else if (a == "--ranks") ranks = std::atoi(val("--ranks"));
        else if (a == "--in-flight") in_flight = std::atoi(val("--in-flight"));
        else if (a == "--readback") readback = true;
        else if (a == "--overlap") {
            overlap = val("--overlap");
            if (overlap != "stream" && overlap != "half" && overlap != "full") { usage(); return 2; }
        }
        else if (a == "--textures") {
            textures = true;
            if (i + 1 < argc && argv[i + 1][0] != '-') atlas = argv[++i];
        }
        else if (a == "--debug") {
            if (std::sscanf(val("--debug"), "%d,%d", &dbg_x, &dbg_y) != 2) { usage(); return 2; }
        } else { std::fprintf(stderr, "unknown option %s\n", a.c_str()); usage(); return 2; }
    }
    if (config.empty()) { usage(); return 2; }
    if (serial) {
        std::fprintf(stderr, "-s (serial CPU path) is not part of this build: the reference CPU path is "
                             "restated in oracle/ for testing only\n");
        return 2;
    }
    if (frames < 1 || spp < 1 || gpus < 1 || ranks < 0 || in_flight < 0 || in_flight > 8) { usage(); return 2; }
    // frames in flight use a stream each: HIP maps streams round-robin onto GPU_MAX_HW_QUEUES
    // hardware queues (4 by default), and streams sharing a queue serialise.
    // The HIP runtime reads it when librt_amd.so's kernels are registered, before main: set it
    // in the environment (GPU_MAX_HW_QUEUES=16 rtracer ... --in-flight 8).
    if (in_flight > 1 && !getenv("GPU_MAX_HW_QUEUES"))
        std::fprintf(stderr, "note: GPU_MAX_HW_QUEUES is not set; with the HIP default of 4 hardware queues "
                             "frames in flight share queues\n");

    // procedural::gpu::generate with optional canvas override; a bad config is reported
    // and exits (the reference asserts)
    rt_scene* handle = nullptr;
    if (rt_scene_load_json(config.c_str(), width, height, &handle) != RT_OK) {
        std::fprintf(stderr, "cannot load %s: %s\n", config.c_str(), rt_last_error());
        return 1;
    }
    if (textures && rt_scene_load_atlas(handle, atlas.empty() ? nullptr : atlas.c_str()) != RT_OK) {
        std::fprintf(stderr, "cannot load the atlas: %s\n", rt_last_error());
        return 1;
    }
    renv::gpu::Scene* scene = new renv::gpu::Scene(handle);
    renv::Environment& env = scene->get_environment();
    std::printf("Loaded scene\n");
    const int W = env.get_canvas().get_width(), H = env.get_canvas().get_height();
    if (gpus > 1 || ranks > 1) {
        std::vector<int> devs(gpus);
        for (int d = 0; d < gpus; d++) devs[d] = d;
        rtracer::gpu::use_devices(scene, devs, ranks > 0 ? ranks : gpus);
        std::printf("Frames split over %d GPU(s), %d slices\n", gpus, ranks > 0 ? ranks : gpus);
    }

    std::vector<uint32_t> host;
    if (in_flight > 0) {                                   // timing: D frames in flight
        const int D = in_flight;
        const bool split = gpus > 1 || ranks > 1;
        rtamd_detail::check(rt_scene_set_frame_slots(handle, D), "rt_scene_set_frame_slots");
        // the frames are issued back to back: every frame on half the CUs, the first of the
        // stream included (RT_OVERLAP_STREAM, include/rt_amd.h; bench.py's default --grid)
        const int policy = overlap == "full" ? RT_OVERLAP_FULL : overlap == "half" ? RT_OVERLAP_HALF : RT_OVERLAP_STREAM;
        rtamd_detail::check(rt_scene_set_overlap(handle, policy), "rt_scene_set_overlap");
        // --readback (the reference's post-condition for every frame, main.cc's loop blits each
        // canvas): each frame is copied into pinned host memory by a copy engine once it is
        // complete -- the host waits for frame f - (D - 1) as it issues frame f and copies it then,
        // and copies any frame it sees complete -- on one copy stream; frame
        // buffers are 2 D deep so a buffer is rewritten long after its copy.  Single device.
        const bool rb = readback && !split;
        const int NB = rb ? 2 * D : D;
        std::vector<hipStream_t> st(D);
        std::vector<uint32_t*> buf(NB);
        std::vector<uint32_t*> hbuf(rb ? NB : 0);
        std::vector<hipEvent_t> ev_done(NB), ev_copy(NB);
        std::vector<char> copied(NB, 0);
        // the frames' copies alternate over two copy streams (RT_CLI_COPY_STREAMS: 1-4): on one
        // copy-engine queue consecutive copies left ~85-us gaps and a growing backlog
        // (profiles/r06/cli_api/); two queues: world8 +4-12% -> +0.3-2% (profiles/r06/cli_cs/)
        const int ncs = !rb ? 1 : getenv("RT_CLI_COPY_STREAMS") ? std::max(1, std::min(4, atoi(getenv("RT_CLI_COPY_STREAMS")))) : 2;
        std::vector<hipStream_t> csts(ncs, nullptr);
        for (int k = 0; k < D; k++)
            if (hipStreamCreateWithFlags(&st[k], hipStreamNonBlocking) != hipSuccess) { std::fprintf(stderr, "HIP stream failed\n"); return 1; }
        for (int k = 0; k < NB; k++) {
            if (hipMalloc((void**)&buf[k], (size_t)W * H * 4) != hipSuccess) { std::fprintf(stderr, "HIP allocation failed\n"); return 1; }
            if (rb) {
                void* hp = nullptr;
                rtamd_detail::check(rt_host_alloc((int64_t)W * H * 4, &hp), "rt_host_alloc");
                hbuf[k] = static_cast<uint32_t*>(hp);
                if (hipEventCreateWithFlags(&ev_done[k], hipEventDisableTiming) != hipSuccess ||
                    hipEventCreateWithFlags(&ev_copy[k], hipEventDisableTiming) != hipSuccess) { std::fprintf(stderr, "HIP event failed\n"); return 1; }
            }
        }
        if (rb) {
            for (auto& c : csts)
                if (hipStreamCreateWithFlags(&c, hipStreamNonBlocking) != hipSuccess) { std::fprintf(stderr, "HIP stream failed\n"); return 1; }
            std::vector<void*> ws(csts.begin(), csts.end());
            for (auto x : st) ws.push_back(x);
            rtamd_detail::check(rt_copy_engines_warm(ws.data(), (int)ws.size()), "rt_copy_engines_warm");
        }
        long long f = 0;
        std::deque<long long> uncopied;                        // issued frames whose copies are not yet issued
        const long long lag = D > 1 ? D - 1 : 0;
        // Frames in flight complete out of order (several share the GPU), so a copy is issued as
        // soon as its own frame is seen complete, not after the older ones: in order only, the
        // copies trailed their frames by ~4 ms and ~6 of them were left after the last frame
        // (profiles/r06/cli_window/).  Each frame has its own host buffer.
        auto copy_frame = [&](long long fr) -> bool {          // frame fr's copy, if the frame is complete
            const int b = (int)(fr % NB);
            if (hipEventQuery(ev_done[b]) != hipSuccess) return false;
            hipStream_t c = csts[fr % ncs];
            rtamd_detail::check(rt_copy_to_host_async(hbuf[b], buf[b], (int64_t)W * H * 4, c), "rt_copy_to_host_async");
            if (hipEventRecord(ev_copy[b], c) != hipSuccess) std::exit(1);
            copied[b] = 1;
            return true;
        };
        auto copy_done_frames = [&]() {                        // every frame seen complete, oldest first
            for (auto it = uncopied.begin(); it != uncopied.end();)
                it = copy_frame(*it) ? uncopied.erase(it) : it + 1;
        };
        auto issue = [&]() {
            const int b = (int)(f % NB);
            rt_render_opts o;
            rt_render_opts_default(&o);
            o.spp = spp; o.use_bvh = unopt ? 0 : 1; o.kernel_dim = dim; o.textures = textures ? 1 : 0;
            o.rgba = buf[b]; o.sync = 0;                       // asynchronous: frames overlap
            // single device: frame f on stream f % D.  Split frames (use_devices) run on the
            // library's per-slot streams; a caller stream would only add event waits, which block
            // whatever else HIP mapped onto that stream's hardware queue
            o.stream = split ? nullptr : st[f % D];
            if (rb && copied[b] && hipStreamWaitEvent(st[f % D], ev_copy[b], 0) != hipSuccess) std::exit(1);
            rtamd_detail::check(rt_render(handle, &o, nullptr), "rt_render");
            if (rb) {
                if (hipEventRecord(ev_done[b], st[f % D]) != hipSuccess) std::exit(1);
                uncopied.push_back(f);
                f++;
                // wait (polling, so younger frames that complete meanwhile are copied too) until
                // frame f - lag is copied: lag + 1 frames stay in flight
                do copy_done_frames(); while (!uncopied.empty() && uncopied.front() < f - lag);
                return;
            }
            f++;
        };
        auto wait_all = [&]() {
            if (split) {                                       // every device of the split
                for (int d = gpus - 1; d >= 0; d--) { (void)hipSetDevice(d); (void)hipDeviceSynchronize(); }
            }
            else if (rb) {
                // the frames still in flight: each copy as soon as its frame completes, so the
                // last copies overlap the last frames instead of following all of them
                while (!uncopied.empty()) copy_done_frames();  // polls: any frame's copy as it completes
                for (auto c : csts) (void)hipStreamSynchronize(c);   // every frame is on the host
            }
            else for (int k = 0; k < D; k++) (void)hipStreamSynchronize(st[k]);
        };
        for (int k = 0; k < 2 * D; k++) issue();          // warm-up: slots, streams, scheduling history
        wait_all();
        auto from = std::chrono::high_resolution_clock::now();
        for (int k = 0; k < frames; k++) issue();
        wait_all();
        auto to = std::chrono::high_resolution_clock::now();
        const double ms = std::chrono::duration<double, std::milli>(to - from).count() / frames;
        const int slices = (gpus > 1 || ranks > 1) ? (ranks > 0 ? ranks : gpus) : 1;
        std::printf("In flight %d%s: %.4f ms/frame, %.4f ms per slice (%d slices on %d GPU(s), %d frames)\n", D,
                    rb ? " (host-readable)" : "", ms, ms * gpus / slices, slices, gpus, frames);
        if (!out.empty()) {
            const uint32_t* px = nullptr;
            if (rb) px = hbuf[(f - 1) % NB];
            else {
                host.resize((size_t)W * H);
                if (hipMemcpy(host.data(), buf[(f - 1) % NB], host.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) px = nullptr;
                else px = host.data();
            }
            if (!px || !write_ppm(out.c_str(), px, W, H)) { std::fprintf(stderr, "cannot write %s\n", out.c_str()); return 1; }
        }
        for (int k = 0; k < D; k++) (void)hipStreamDestroy(st[k]);
        for (int k = 0; k < NB; k++) {
            (void)hipFree(buf[k]);
            if (rb) { (void)rt_host_free(hbuf[k]); (void)hipEventDestroy(ev_done[k]); (void)hipEventDestroy(ev_copy[k]); }
        }
        for (auto c : csts) if (c) (void)hipStreamDestroy(c);
        renv::gpu::Scene::free(*scene);
        delete scene;
        return 0;
    }
    // spp > 1 / textures (build extensions): the frame as update_scene leaves it -- rendered into a
    // device buffer, copied by a copy engine into pinned host memory, waited for -- with the
    // buffers made before any timing, as the reference's canvas is made with the scene
    uint32_t* dframe = nullptr;
    uint32_t* hframe = nullptr;
    hipStream_t dst = nullptr;
    if (spp != 1 || textures) {
        void* hp = nullptr;
        if (hipMalloc((void**)&dframe, (size_t)W * H * 4) != hipSuccess ||
            hipStreamCreateWithFlags(&dst, hipStreamNonBlocking) != hipSuccess) { std::fprintf(stderr, "HIP allocation failed\n"); return 1; }
        rtamd_detail::check(rt_host_alloc((int64_t)W * H * 4, &hp), "rt_host_alloc");
        hframe = static_cast<uint32_t*>(hp);
    }
    auto draw = [&]() {
        if (spp == 1 && !textures) {
            rtracer::gpu::update_scene(scene, dim, !unopt);
        } else {
            rt_render_opts o;
            rt_render_opts_default(&o);
            o.spp = spp; o.use_bvh = unopt ? 0 : 1; o.kernel_dim = dim; o.textures = textures ? 1 : 0;
            o.rgba = dframe; o.stream = dst; o.sync = 0;
            rtamd_detail::check(rt_render(scene->handle(), &o, nullptr), "rt_render");
            rtamd_detail::check(rt_copy_to_host_async(hframe, dframe, (int64_t)W * H * 4, dst), "rt_copy_to_host_async");
            if (hipStreamSynchronize(dst) != hipSuccess) { std::fprintf(stderr, "HIP stream failed\n"); std::exit(1); }
        }
    };
    if (bench) {
        auto from = std::chrono::high_resolution_clock::now();
        draw();
        auto to = std::chrono::high_resolution_clock::now();
        std::printf("Time: %g ms\n", std::chrono::duration<double, std::milli>(to - from).count());
    } else {
        auto from = std::chrono::high_resolution_clock::now();
        for (int f = 0; f < frames; f++) draw();
        auto to = std::chrono::high_resolution_clock::now();
        std::printf("FPS: %g\n", frames / std::chrono::duration<double>(to - from).count());
    }
    if (dbg_x >= 0) {
        std::printf("shooting debug ray at %d, %d\n", dbg_x, dbg_y);
        rtracer::gpu::debug_cast(scene, dbg_x, dbg_y);
    }
    if (!out.empty()) {
        const uint32_t* px = (spp == 1 && !textures) ? env.get_canvas().get_buffer() : hframe;
        if (!px || !write_ppm(out.c_str(), px, W, H)) { std::fprintf(stderr, "cannot write %s\n", out.c_str()); return 1; }
    }
    if (dframe) { (void)hipStreamDestroy(dst); (void)hipFree(dframe); (void)rt_host_free(hframe); }
    renv::gpu::Scene::free(*scene);
    delete scene;
    return 0;
}
