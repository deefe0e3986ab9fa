/*
 * rt_amd.h — C ABI of the MI355X-native ray-tracing core (the drop-in boundary).
 *
 * Replaces the render path of wtzhang23/gpu-ray-tracer:
 *   rtracer::gpu::update_scene(Scene*, int kernel_dim, bool optimize)   include/raytracer.h:18-22, src/raytracer.cu:102-120
 *   rtracer::gpu::debug_cast(Scene*, int x, int y)                      include/raytracer.h:21,       src/raytracer.cu:91-100
 *   procedural::gpu::generate(std::string config_path)                  include/procedural/cube_world.h:20-23, src/procedural/cube_world.cc:195-207
 *   rtracer::SceneBuilder {add_vertex, create_mesh, add_triangle, add_trans, build_cube,
 *                          add_point_light, add_directional_light, build_gpu_scene}  include/scene_builder.h:29-117
 *   renv::gpu::Scene::free(Scene&)                                       include/rayenv/gpu/scene.h:55-69
 *   Camera/Entity translate/rotate/set_position/set_orientation          include/rayprimitives/entity.h:49-74
 *   Canvas::get_color / the framebuffer SDL wraps                        include/rayenv/canvas.h:17-44, src/rayenv/canvas.cu:10-29
 * Plain pointers and sizes only; every call returns an RT_* status and sets a
 * thread-local message readable with rt_last_error() (the reference asserts).
 */
#ifndef RT_AMD_H
#define RT_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 3: rt_work gained the query-occupancy fields; RT_EXPORT_TRIS / RT_EXPORT_TEXCOORDS list
 *    triangles in the flattened mesh order (the index space of hit_tri)
 * 4: rt_host_alloc / rt_host_free / rt_copy_to_host_async / rt_copy_engines_warm (host-readable
 *    frames through a copy engine); a finished scene is uploaded and warmed at creation when a gfx950 device is present */
#define RT_ABI_VERSION 4

enum {
    RT_OK = 0,
    RT_ERR_ARG = -1,      /* bad argument / out-of-range index */
    RT_ERR_IO = -2,       /* file cannot be opened */
    RT_ERR_PARSE = -3,    /* malformed scene description */
    RT_ERR_HIP = -4,      /* HIP runtime error (message has the hipError string) */
    RT_ERR_STATE = -5,    /* call not valid in the current state */
    RT_ERR_NODEV = -6,    /* no usable gfx950 device */
    RT_ERR_LIMIT = -7     /* scene exceeds a build limit (see rt_last_error) */
};

typedef struct rt_scene rt_scene;

/* ---- library ---- */
int rt_abi_version(void);
const char* rt_last_error(void);
int rt_device_count(int* count);
/* Select the HIP device for subsequent scene uploads on this thread. */
int rt_set_device(int device);

/* ---- scene creation ----
 * A finished scene (rt_scene_load_json, rt_builder_finish) goes to the current device at once
 * when a gfx950 device is present, as procedural::gpu::generate / build_gpu_scene do
 * (cube_world.cc:195-207, scene_builder.cu:29-81), and one untimed 1-spp frame warms the code
 * object, the scene's stream and the frame buffers; the first rt_update_scene then only renders.
 * Without a device the scene stays host-only and render calls return RT_ERR_NODEV.
 * RT_NO_WARM=1 (environment) defers the upload to the first render. */
/* worldN.json -> scene (cube_world.cc:38-191).  width/height <= 0 keep the JSON's canvas size. */
int rt_scene_load_json(const char* path, int width, int height, rt_scene** out);
/* Empty scene for the builder API (SceneBuilder{atlas_path}, scene_builder.h:51-56). */
int rt_scene_create(const char* atlas_path, rt_scene** out);
int rt_scene_free(rt_scene* s);

/* SceneBuilder (scene_builder.h:58-112).  Indices are returned through out-params. */
int rt_builder_add_vertex(rt_scene* s, float x, float y, float z, int* idx);
int rt_builder_create_mesh(rt_scene* s, const float pos3[3], const float quat4[4], int* mesh);
/* material26: Ke[4] Ka[4] Kd[4] Ks[4] Kt[4] Kr[4] alpha eta (material.h:14-31) */
int rt_builder_add_triangle(rt_scene* s, int mesh, int i0, int i1, int i2, const float material26[26]);
/* add_triangle with rprimitives::TextureCoords (texture_coords.h:12-29): tex6 = {tx, ty, ux, uy, vx, vy};
 * a hit with barycentric weights (u, v) of vertices i1, i2 reads atlas texel (tx, ty) + u (ux, uy) + v (vx, vy)
 * in the textured shading mode (build-defined: the reference never samples, phong.cu:18-23). */
int rt_builder_add_triangle_tex(rt_scene* s, int mesh, int i0, int i1, int i2, const float material26[26],
                                const float tex6[6]);
int rt_builder_add_trans(rt_scene* s, int mesh, int* trans);
int rt_builder_set_trans(rt_scene* s, int trans, const float pos3[3], const float quat4[4]);  /* either may be NULL */
int rt_builder_build_cube(rt_scene* s, float scale, const float material26[26], int* mesh);
/* build_cube with every face mapped onto the atlas square tile3 = {tx, ty, size} (texels). */
int rt_builder_build_cube_tex(rt_scene* s, float scale, const float material26[26], const float tile3[3], int* mesh);
int rt_builder_add_point_light(rt_scene* s, const float pos3[3], const float col4[4]);
int rt_builder_add_directional_light(rt_scene* s, const float dir3[3], const float col4[4]);
/* Canvas + Camera (camera.cu:6-9) + Environment (environment.h:19-93); finalises the builder. */
int rt_builder_finish(rt_scene* s, int width, int height, float fov_radians, float unit_to_pixels,
                      const float cam_pos3[3], const float cam_quat4[4],
                      const float dist_atten3[3], const float ambience4[4], int depth);

/* ---- texture atlas (assets.cc:61-81, gputils TextureBuffer4D alloc.h:24-80) ----
 * Texels are float RGBA = byte / 255 in HBM, point-sampled with clamp addressing as the
 * reference's texture object (gfx950 has no texture units).  Only read when
 * rt_render_opts.textures = 1. */
int rt_scene_set_atlas(rt_scene* s, const uint8_t* rgba8, int width, int height);
/* Decode an 8-bit RGB/RGBA PNG.  png_path NULL: the scene's own atlas entry (JSON "atlas"
 * or SceneBuilder{atlas}), resolved against the scene file's directory, then the CWD. */
int rt_scene_load_atlas(rt_scene* s, const char* png_path);
/* atlas3 = {width, height, loaded} */
int rt_scene_atlas_info(const rt_scene* s, int32_t atlas3[3]);

/* info10 = {W, H, n_vertices, n_tris, n_meshes, n_instances, n_lights, n_point_lights, depth, n_materials} */
int rt_scene_info(const rt_scene* s, int32_t info10[10]);
/* Host copies of the scene arrays (layouts as in oracle/rt_oracle.h) for parity checks.
 * Triangles (and their texture coordinates) are listed in the flattened mesh order, the
 * index space of rt_render_opts.hit_tri. */
enum { RT_EXPORT_VERTICES = 0, RT_EXPORT_NORMALS = 1, RT_EXPORT_TRIS = 2, RT_EXPORT_MATERIALS = 3,
       RT_EXPORT_INSTANCES = 4, RT_EXPORT_INST_MESH = 5, RT_EXPORT_LIGHTS = 6, RT_EXPORT_CAMERA = 7, RT_EXPORT_ENV = 8,
       RT_EXPORT_TEXCOORDS = 9,   /* per triangle float7 {has, tx, ty, ux, uy, vx, vy} */
       RT_EXPORT_ATLAS = 10 };    /* atlas RGBA8 bytes, width*height*4 (rt_scene_atlas_info) */
int rt_scene_export(const rt_scene* s, int what, void* dst, int64_t dst_bytes);

/* ---- camera / environment (entity.h:49-74, environment.h:30-44) ---- */
int rt_camera_get(const rt_scene* s, float pos3[3], float quat4[4]);
int rt_camera_set(rt_scene* s, const float pos3[3], const float quat4[4]);      /* either may be NULL */
int rt_camera_translate(rt_scene* s, const float d3[3]);                        /* Entity::translate: p += o*d */
int rt_camera_rotate(rt_scene* s, const float dq4[4]);                          /* Entity::rotate: o = dq*o */
/* Camera::up()/right()/forward() unit directions (camera.cu:11-31) */
int rt_camera_axes(const rt_scene* s, float right3[3], float up3[3], float forward3[3]);
int rt_env_set(rt_scene* s, const float ambience4[4], const float dist_atten3[3], int depth);

/* ---- rendering ---- */
typedef struct rt_render_opts {
    int spp;            /* samples per pixel, >= 1 (1 == reference) */
    int use_bvh;        /* reference `optimize`: 1 BVH traversal, 0 brute force over instances */
    int rebuild_bvh;    /* 1: rebuild the BVH in this call (reference per-frame semantics); 0: reuse if built */
    int row0, row_step; /* render rows y = row0 + j*row_step (row-cyclic multi-GPU slice); 0,1 = full frame */
    int compact;        /* 0: outputs indexed by full-frame pixel y*W+x; 1: by slice row j*W+x */
    int kernel_dim;     /* reference's block edge (-d); accepted, the HIP path picks its own tiling */
    void* stream;       /* hipStream_t to launch on; NULL = the scene's own stream */
    uint32_t* rgba;     /* device outputs (NULL = internal canvas for rgba, skipped for the others) */
    float* radiance;    /* float4 per pixel: mean of unclamped sample radiance */
    int32_t* hit_inst;  /* primary hit of sample 0: instance index, -1 on miss */
    int32_t* hit_tri;   /* primary hit of sample 0: global triangle index, -1 on miss */
    int sync;           /* 1: wait for completion before returning (required for stats) */
    int host_outputs;   /* 1: rgba/radiance/hit_* are HOST pointers; results are copied back (implies sync) */
    int timing;         /* 1: time the BVH build and the trace kernel with start/stop events on the
                           dispatches themselves (hipExtLaunchKernel; no marker packets, no sync);
                           totals via rt_timing_collect */
    int textures;       /* 1: textured shading (build-defined, parity-unpinned): the diffuse colour of a
                           hit on a triangle with texture coordinates is its atlas texel instead of Kd
                           (the TODO branch of phong.cu:18-23).  0 (default) = the reference. */
} rt_render_opts;

typedef struct rt_stats {
    uint64_t rays;       /* closest-hit queries (= reference cast_ray calls) */
    uint64_t nodes;      /* BVH node tests, single-ray semantics */
    uint64_t leaves;     /* instance tests (= cast_local calls) */
    uint64_t tri_tests;  /* triangle tests */
    double bvh_ms;       /* BVH build kernel time (device events) */
    double trace_ms;     /* trace kernel time (device events) */
} rt_stats;

void rt_render_opts_default(rt_render_opts* o);
int rt_render(rt_scene* s, const rt_render_opts* opts, rt_stats* stats);

/* The work the fast (statistics-free) kernels do for one frame of `opts`, from a profiling
 * run of the fast kernel with wave-level counters (not timed, outputs discarded).  rt_stats
 * counts the reference's units (every cast_ray of propagate_ray, raytracer.cu:17-43); the
 * fast kernel proves some of them unnecessary and skips them (unlit shadow rays, pruned
 * subtrees, occluded-shadow early exits): this is what it does instead. */
typedef struct rt_work {
    uint64_t queries;       /* closest-hit queries issued: one per primary sample, reflection /
                               refraction ray and traced shadow segment */
    uint64_t wave_queries;  /* wave-level query steps (64 lanes each) */
    uint64_t pair_steps;    /* wave-level BVH child-pair tests */
    uint64_t leaf_visits;   /* wave-level leaf (instance) visits */
    uint64_t leaf_lanes;    /* lane-level leaf visits (cast_local calls) */
    uint64_t tri_iters;     /* wave-level triangle-loop iterations */
    uint64_t scene_bytes;   /* the scene the fast kernel reads: ordered-tree records, instance records,
                               triangles, meshes, materials, lights (staged into each block's LDS) */
    /* Query occupancy (ABI 3).  Lanes by integrator phase over every wave query: */
    uint64_t lanes_primary;    /* primary-ray queries (sample's first NORMAL frame) */
    uint64_t lanes_secondary;  /* reflection / refraction NORMAL-frame queries */
    uint64_t lanes_shadow;     /* traced shadow segments */
    uint64_t lanes_unlit;      /* shadow steps the unlit skip answers without a query */
    /* Over the wave queries of live groups only (some primary enters the tree's root; the sky
     * groups the pre-pass answers are left out): */
    uint64_t live_wave_queries;
    uint64_t live_lanes;       /* queries issued in them: occupancy = live_lanes / (64 live_wave_queries) */
    uint64_t hist_wave_queries[8];  /* live wave queries by active lanes: 1-8, 9-16, ..., 57-64 */
    uint64_t hist_pair_steps[8];    /* their child-pair steps */
    uint64_t hist_leaf_visits[8];   /* their leaf visits */
} rt_work;
/* BVH frames with 1 <= spp <= 64, untextured; RT_ERR_STATE when the scene has no profiling
 * variant (the fast kernel needs the ordered tree in LDS). */
int rt_frame_work(rt_scene* s, const rt_render_opts* opts, rt_work* work);

/* Frame slots (1 = default, up to 8).  The reference rebuilds its BVH inside every
 * update_scene call (raytracer.cu:103-119), so a frame owns per-frame state: BVH, work
 * counters and scheduling history.  With n slots, consecutive rt_render calls rotate
 * through n copies of that state.  Frames issued on other streams then overlap the
 * previous frames' tails on the CUs they have freed.  Each call waits (stream-ordered, no
 * host sync) for the last frame of its slot.  The caller gives frames in flight distinct
 * outputs.  Images are identical either way.  Waits for the device when changed. */
int rt_scene_set_frame_slots(rt_scene* s, int n_slots);

/* Grid of a frame issued while another frame of the scene is still running (four frame
 * slots): RT_OVERLAP_HALF (default) = half the CUs, so that two frames' persistent blocks
 * share the GPU and a block's tail (its slowest wave) holds fewer CUs; RT_OVERLAP_FULL =
 * every CU, as a frame issued alone gets.  HALF measured faster for device-resident
 * pipelines (frame -3%, row slices -4..-11%); FULL was faster for pipelines whose host copies
 * ran as blit kernels on the CUs (round 3), not for copy-engine copies (rt_copy_to_host_async,
 * DESIGN.md §4.2).  RT_OVERLAP_STREAM = half the CUs for every frame, the
 * first of a stream included, for callers that issue frames back to back: the first two
 * frames then run side by side instead of the second waiting for the first's tail (20-frame
 * streams -2%), but a frame issued alone takes half the GPU, so set it for the stream only.
 * Images are identical either way.  Host-side state. */
enum { RT_OVERLAP_HALF = 0, RT_OVERLAP_FULL = 1, RT_OVERLAP_STREAM = 2 };
int rt_scene_set_overlap(rt_scene* s, int policy);

/* Multi-GPU frames from one host process (the reference's single-device
 * update_scene, raytracer.cu:102-120, split over a node's GPUs).  After this call every
 * whole-frame rt_render / rt_update_scene of the scene renders n_ranks row-cyclic slices
 * (slice r = rows r, r + n_ranks, ...), ranks [i k, (i+1) k) on devices[i] (k = n_ranks /
 * n_devices; each device holds a replica of the scene and rebuilds the same BVH), gathers
 * them to devices[0] with RCCL (ncclGather over ncclCommInitAll communicators) and
 * un-permutes the rows there: the caller sees one frame, RGBA8 only.  devices[0] is the
 * scene's device.  n_ranks > n_devices gives several slices per device (on one GPU the
 * whole sequence runs with a one-rank communicator).  n_devices = n_ranks = 1 returns to
 * single-device frames.  Camera, instance and environment changes reach every replica. */
int rt_scene_set_devices(rt_scene* s, const int* devices, int n_devices, int n_ranks);

/* Sum of the event-timed kernel durations of all rt_render calls with timing=1
 * since the last collect (synchronizes those events), then resets. */
int rt_timing_collect(rt_scene* s, double* bvh_ms_total, double* trace_ms_total, int* n_frames);

/* ---- host-readable frames (the post-condition of update_scene, raytracer.cu:102-120 /
 * canvas.cu:23-29: the canvas is host memory the caller reads after the call) ---- */
/* Pinned (page-locked) host memory: the copy engines write it directly over PCIe. */
int rt_host_alloc(int64_t bytes, void** out);
int rt_host_free(void* p);
/* Enqueue a device -> host copy of `bytes` on `stream` (a hipStream_t; NULL = the null stream)
 * on a DMA copy engine: no compute unit is taken from frames in flight.  host_dst should come
 * from rt_host_alloc (pageable memory is staged by the runtime).  Stream-ordered: record an
 * event after it, or synchronize the stream, before reading host_dst. */
int rt_copy_to_host_async(void* host_dst, const void* dev_src, int64_t bytes, void* stream);
/* Start the device's SDMA copy engines a host-copy pipeline will use, once per process and
 * device: one gated copy from each of the n streams (hipStream_t; the streams the pipeline
 * copies from or orders copies behind).  The runtime gives a copy queued while earlier copies
 * are still pending the next idle engine, and a copy's first use of an engine creates that
 * engine's queue (~7 ms of host time inside the enqueue): a pipeline with frames in flight
 * would pay that inside its first timed frames.  Blocks until done. */
int rt_copy_engines_warm(void* const* streams, int n_streams);

/* Reference-equivalent frame: rebuild BVH if optimize, trace 1 spp, copy the frame into the
 * pinned host canvas on a copy engine, wait for that stream; the framebuffer is host-readable
 * afterwards (raytracer.cu:102-120). */
int rt_update_scene(rt_scene* s, int kernel_dim, int optimize);
/* Host framebuffer (RGBA8 packed R<<24|G<<16|B<<8|A, row-major W*H) after rt_update_scene. */
int rt_canvas_read(const rt_scene* s, uint32_t* dst, int64_t n_pixels);
const uint32_t* rt_canvas_host_ptr(const rt_scene* s);
/* Canvas::get_color(x, y) of the last rt_update_scene frame (canvas.cu:14-17). */
int rt_canvas_get_color(const rt_scene* s, int x, int y, uint8_t rgba4[4]);

/* debug_cast (raytracer.cu:91-100): trace pixel (x, y) and write an event log
 * ("shooting a ray", "preparing to shoot a reflection ray", ...) into buf. */
int rt_debug_cast(rt_scene* s, int x, int y, char* buf, int64_t cap);

/* Device-side math known-answer entry (test hook): evaluates `op` element-wise on
 * the GPU.  op names as in oracle/rt_oracle.h's orc_kat_*, plus the filtered variants
 * tri_hit_f, box_hit_f and box_pair (two boxes per element, two int results), and
 * box_from_local / box_merge (box7 = min3 max3 nondegenerate; entity7 = quat4 pos3 -> box6 +
 * int) and entity (entity7, v3 -> point/vec to/from local, 12 floats). 
 * Host pointers in/out. */
int rt_kat_device(const char* op, int n, const float* in0, const float* in1, const float* in2,
                  float* out_f, int32_t* out_i, uint64_t* out_u);

/* Profiling hook: launches an empty marker kernel of `tag` (1..64) workgroups on `stream` (a
 * hipStream_t; NULL = the default stream), so a rocprofv3 kernel or counter trace can find the
 * caller's timed region between two markers (bench.py --pmc-window, tools/pmc_step.py). */
int rt_profile_marker(int tag, void* stream);

/* Sample offset table of the build-defined spp extension (k=0 -> (0,0)). */
int rt_spp_offset(int k, float* dx, float* dy);

#ifdef __cplusplus
}
#endif
#endif
