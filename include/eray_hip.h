/*
 * eray_hip.h — the C-ABI drop-in boundary of the MI355X (gfx950) implementation of
 * HoloTheDrunk/eray's per-pixel ray-tracing hot path.
 *
 * Everything here is plain C: opaque context pointer, plain pointers, sizes and status codes.
 * It is what the reference's Rust host (Engine / Scene / Material / shader Graph) would bind
 * with one `extern "C"` block, and what this repository's own C++ host
 * (include/eray/ headers) and Python tooling (eray_amd/) call.
 *
 * Entry points and the reference interface each one replaces (paths relative to the
 * reference checkout, src/...):
 *
 *   eray_node_wave          lib shaderlib/wave.rs:100-137        (wave::node closure)
 *   eray_node_rgb           shaderlib/rgb.rs:64-103              (rgb::node closure)
 *   eray_node_flat_color    shaderlib/flat_color.rs:65-95        (flat_color::node closure)
 *   eray_node_mix_color     shaderlib/mix_color.rs:57-102        (mix_color::node closure)
 *   eray_material_example   main.rs:80-144 + lib/material.rs:35-53 (Graph::run of main's graph,
 *                           all four nodes fused into one pass)
 *   eray_scene_*            lib/scene.rs:39-54 (add_object / add_light / set_camera) and
 *                           lib/object.rs:213-230 (Object::build -> device triangle arrays);
 *                           eray_scene_set_object_texel_graph: lib/material.rs:35-94 +
 *                           lib/shader/graph.rs:499-609 (Material::update's Graph::run over the
 *                           shaderlib nodes, evaluated at the texel Material::get reads);
 *                           eray_scene_set_object_example_material: lib/material.rs:56-94
 *                           (Material::get) over main.rs:80-144's graph, per hit texel
 *   eray_render_camera_path lib/scene.rs:39-54 Scene::set_camera + lib/engine.rs:46-81 per frame
 *   eray_render             lib/engine.rs:46-81 (Engine::render: camera rays, first-hit
 *                           Object::intersects object.rs:58-81, Triangle::intersects
 *                           primitives.rs:41-72, cast_ray shading engine.rs:112-216,
 *                           reaches_light engine.rs:218-228) fused with the PPM byte pack
 *   eray_pack_ppm           lib/image.rs:48-74 + lib/color.rs:31-37 (save_as_ppm body bytes)
 *   eray_gather_rows        lib/engine.rs:85-98 + lib/image.rs:48-74 across GPUs (row tiles, RCCL)
 *   eray_gather_frames      the same for a batch of frames (a frame ring), optionally sync-free
 *   eray_ppm_header         lib/image.rs:56
 *   eray_camera_size        lib/camera.rs:36-38
 *
 * Conventions
 *   - Every function returns an eray_status (0 = OK, < 0 = error) unless stated otherwise.
 *     The reference's Result errors and panics map onto these codes; a message is available
 *     from eray_last_error(ctx).  No C++ exception ever crosses this boundary.
 *   - "device" pointers are HIP device allocations (eray_device_alloc or any other allocator
 *     on the context's device).  Work is enqueued on the context's stream and is asynchronous;
 *     call eray_synchronize (or synchronise the stream) before reading results on the host.
 *   - Images are row-major f32: an IValue image holds 1 float per pixel, an IColor image 3
 *     (r, g, b), exactly like Image<f32> / Image<Color> (#[repr(C)] Color, color.rs:12-22).
 *   - One context per GPU; a context is used from one host thread at a time.
 */
#ifndef ERAY_HIP_H
#define ERAY_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ERAY_ABI_VERSION 6

typedef enum eray_status {
    ERAY_OK = 0,
    ERAY_E_INVALID_ARGUMENT = -1,
    ERAY_E_HIP = -2,            /* a HIP runtime call failed (message has the HIP error) */
    ERAY_E_OUT_OF_MEMORY = -3,
    ERAY_E_MISSING = -4,        /* shader::Error::Missing / graph::Error::Missing          */
    ERAY_E_MISSING_MANY = -5,   /* shader::Error::MissingMany (utils.rs:15-34)             */
    ERAY_E_INVALID_TYPE = -6,   /* shader::Error::InvalidType (shader.rs:140-178)          */
    ERAY_E_OUT_OF_BOUNDS = -7,  /* an index the reference would panic on (image.rs:36-43,
                                   rgb.rs:89-95, `% 0` in mod_get)                         */
    ERAY_E_IO = -8,
    ERAY_E_PARSE = -9,          /* Object::load_obj panics (object.rs:101-186,396-421)     */
    ERAY_E_BUILD = -10,         /* Object::build Err (object.rs:213-218)                   */
    ERAY_E_UNSUPPORTED = -11,   /* a reference feature this build does not offer (yet)     */
    ERAY_E_CYCLE = -12          /* graph::Error::Cycle (graph.rs:326-338)                  */
} eray_status;

typedef struct eray_ctx eray_ctx;

/* ------------------------------------------------------------------ context & memory --- */
int eray_abi_version(void);                      /* returns ERAY_ABI_VERSION */
int eray_ctx_create(int device, eray_ctx** out);
int eray_ctx_destroy(eray_ctx* ctx);
/* Last error message of ctx (or of the calling thread when ctx is NULL); never NULL. */
const char* eray_last_error(const eray_ctx* ctx);
/* Enqueue all further work on `hip_stream` (e.g. PyTorch's current stream).  NULL selects
 * HIP's null (default) stream; a new context starts on a stream of its own. */
int eray_set_stream(eray_ctx* ctx, void* hip_stream);
void* eray_get_stream(eray_ctx* ctx);
int eray_synchronize(eray_ctx* ctx);
int eray_device_alloc(eray_ctx* ctx, size_t bytes, void** dev_ptr);
int eray_device_free(eray_ctx* ctx, void* dev_ptr);
int eray_memset(eray_ctx* ctx, void* dev_ptr, int value, size_t bytes);
int eray_copy_to_device(eray_ctx* ctx, void* dev_dst, const void* host_src, size_t bytes);
int eray_copy_to_host(eray_ctx* ctx, void* host_dst, const void* dev_src, size_t bytes);

/* ------------------------------------------------------------------ images -------------- */
/* A read-only view of a device image socket value.  data == NULL means "no value" (the
 * Option is None).  For IValue images channels are implied 1, for IColor 3. */
typedef struct eray_image {
    const float* data;
    uint32_t width;
    uint32_t height;
} eray_image;

/* ------------------------------------------------------------------ shaderlib nodes ----- *
 * Each node writes its output image into a caller-allocated device buffer of
 * width*height pixels (the reference's node allocates `Image::new(width, height, ..)` and
 * `out.replace`s it; ownership stays with the caller here).  `width`/`height` are the node's
 * Value inputs already converted with Rust's saturating `as u32`.                           */

/* wave.rs:123-130: out[y*w+x] = |cosf((x*x_fac + y*y_fac)/10)| (glibc cosf, bit-exact). */
int eray_node_wave(eray_ctx* ctx, uint32_t width, uint32_t height, float x_fac, float y_fac,
                   float* out_value);
/* rgb.rs:89-95: out[i] = (red[i], green[i], blue[i]); each input must hold >= width*height
 * pixels (the reference indexes the input's pixel vector with the output's index). */
int eray_node_rgb(eray_ctx* ctx, uint32_t width, uint32_t height, eray_image red,
                  eray_image green, eray_image blue, float* out_color);
/* flat_color.rs:88: a width x height image filled with (r, g, b). */
int eray_node_flat_color(eray_ctx* ctx, uint32_t width, uint32_t height, float r, float g,
                         float b, float* out_color);
/* mix_color.rs:85-95: out = left.mod_get(x,y)*(1-factor) + right.mod_get(x,y)*factor. */
int eray_node_mix_color(eray_ctx* ctx, uint32_t width, uint32_t height, eray_image left,
                        eray_image right, float factor, float* out_color);
/* main.rs:80-144 evaluated in one pass: color = mix(rgb(w,w,w), flat(r,g,b), factor),
 * diffuse = w with w = wave(x_fac, y_fac).  Either output may be NULL. */
int eray_material_example(eray_ctx* ctx, uint32_t width, uint32_t height, float x_fac,
                          float y_fac, float r, float g, float b, float factor,
                          float* out_color, float* out_diffuse);

/* ------------------------------------------------------------------ scene --------------- */
typedef struct eray_camera {        /* camera.rs:15-31 (target/up are unused by the path) */
    float center[3];
    float fov[2];                   /* Fov(f32, f32); only fov[0]/fov[1] is used */
    uint32_t width;
    float z_dist;
} eray_camera;

typedef enum eray_light_variant {   /* light.rs:20-25 */
    ERAY_LIGHT_POINT = 0,
    ERAY_LIGHT_AMBIENT = 1
} eray_light_variant;

typedef struct eray_light {         /* light.rs:7-16 */
    float position[3];              /* transform.translation() */
    int32_t variant;                /* eray_light_variant */
    float color[3];
    float brightness;
} eray_light;

typedef struct eray_material {      /* Material::get's selected outputs (material.rs:56-94) */
    eray_image color;               /* IColor output or data == NULL */
    eray_image diffuse;             /* IValue outputs or data == NULL */
    eray_image specular;
    eray_image specular_power;
    eray_image reflection;
} eray_material;

typedef struct eray_object {        /* Object<Built> (object.rs:30-52) */
    const float* positions;         /* host, T x 9: face vertices a.xyz b.xyz c.xyz */
    const float* normals;           /* host, T x 9: per-vertex normals of a, b, c   */
    const float* uvs;               /* host, T x 6: per-vertex uv of a, b, c        */
    uint32_t triangle_count;        /* T (faces in file order: first hit is by index) */
    float bbox_min[3];              /* bounding_box x/y/z range starts (0 for load_obj meshes) */
    float bbox_max[3];              /* ... range ends */
    eray_material material;         /* device textures; must outlive the scene */
} eray_object;

/* main.rs:80-144's material graph (wave -> rgb -> mix with flat_color) evaluated at the hit
 * texel instead of sampled from its textures: Material::get reads texel
 * ((u*width) as u32 % width, (v*height) as u32 % height) of width x height images, so computing
 * that one texel (wave.rs:127, mix_color.rs:89) is bit-identical to eray_material_example's
 * textures and needs neither the 16 B/texel images nor a memory round trip per hit. */
typedef struct eray_material_example_params {
    uint32_t width;                 /* the graph's "width" / "height" inputs (as u32) */
    uint32_t height;
    float x_fac, y_fac;             /* wave inputs */
    float r, g, b;                  /* flat_color inputs */
    float factor;                   /* mix_color input */
} eray_material_example_params;

/* A material shader graph of the four shaderlib nodes, evaluated at the hit texel instead of
 * sampled from the textures Graph::run would produce (graph.rs:499-609, material.rs:35-94).
 * Material::get reads texel ((u*W) as u32 % W, (v*H) as u32 % H) of an output's W x H image; a
 * node's value at a texel depends only on its inputs' values at texels its own formula picks —
 * mix_color's mod_get (mix_color.rs:85-91: the input's (x % w, y % h)), rgb's pixel index
 * (rgb.rs:89-95: pixels[y * W + x] of each input), wave's (x, y) (wave.rs:127) — so evaluating
 * the graph at that one texel is bit-identical to the texture path, with no image at all.     */
typedef enum eray_texel_node_kind {
    ERAY_TEXEL_WAVE = 0,            /* IValue; param = x_fac, y_fac (wave.rs:100-137)          */
    ERAY_TEXEL_RGB = 1,             /* IColor; input = red, green, blue (IValue nodes)         */
    ERAY_TEXEL_FLAT_COLOR = 2,      /* IColor; param = r, g, b (flat_color.rs:65-95)           */
    ERAY_TEXEL_MIX_COLOR = 3        /* IColor; input = left, right (IColor nodes), param[0] =
                                       factor (default 0.5 is the caller's: mix_color.rs:83)   */
} eray_texel_node_kind;

typedef struct eray_texel_node {
    uint32_t kind;                  /* eray_texel_node_kind */
    uint32_t width, height;         /* the node's width / height inputs (as u32)               */
    float param[3];
    int32_t input[3];               /* indices of EARLIER nodes of the array (a DAG in order)   */
} eray_texel_node;

typedef struct eray_texel_graph {
    const eray_texel_node* nodes;
    uint32_t count;
    /* node index of each Material output, or -1 to keep the object's texture / default; an
     * output whose node has the wrong type reads as None (Material::get, material.rs:61-88:
     * the default then applies, as in the reference) */
    int32_t color, diffuse, specular, specular_power, reflection;
} eray_texel_graph;

int eray_scene_reset(eray_ctx* ctx);
int eray_scene_set_camera(eray_ctx* ctx, const eray_camera* camera);
int eray_scene_add_light(eray_ctx* ctx, const eray_light* light);
/* Copies the host arrays; *object_index (optional) receives the object's position.  A scene
 * holds at most 2^26 - 1 triangles over all its objects (the kernels address triangle records
 * with 32-bit byte offsets): ERAY_E_INVALID_ARGUMENT beyond, with nothing added. */
int eray_scene_add_object(eray_ctx* ctx, const eray_object* object, uint32_t* object_index);
/* The object's color and diffuse outputs become main.rs's graph evaluated per hit (see
 * eray_material_example_params); its other outputs stay as given. */
int eray_scene_set_object_example_material(eray_ctx* ctx, uint32_t object_index,
                                           const eray_material_example_params* params);
/* The object's material outputs named by `graph` become that graph evaluated per hit texel
 * (see eray_texel_graph); the others stay as given.  Errors: a node input that is not an
 * earlier node or has the wrong type (shader::Error::InvalidType), a zero-sized mix input
 * (`% 0`) or an rgb input with fewer pixels than the rgb image (rgb.rs indexes past the end:
 * ERAY_E_OUT_OF_BOUNDS), more than 32 nodes in one output's expansion (ERAY_E_UNSUPPORTED).
 * graph == NULL removes a previous graph. */
int eray_scene_set_object_texel_graph(eray_ctx* ctx, uint32_t object_index, const eray_texel_graph* graph);
/* Camera::size(): (width, (width as f32 / (fov0/fov1)) as u32) */
int eray_camera_size(const eray_camera* camera, uint32_t* width, uint32_t* height);

/* ------------------------------------------------------------------ render -------------- */
typedef struct eray_render_params {
    uint32_t image_width;           /* the Engine's image size (Engine::new((w, h), ..))    */
    uint32_t image_height;
    uint32_t row0;                  /* render camera rows [row0, row0 + rows)               */
    uint32_t rows;
    uint32_t bounces;               /* Engine::bounces (reflection recursion depth, <= 16)  */
    uint32_t anti_aliasing;         /* Engine::anti_aliasing: extra jittered rays per pixel */
    float* out_rgb;                 /* device or NULL: rows x image_width x 3 f32, pixel
                                       (x, row0 + j) at ((j * image_width) + x) * 3         */
    uint8_t* out_ppm;               /* device or NULL: the PPM body bytes of these rows, in
                                       file (bottom-up) order: rows x image_width x 3 bytes,
                                       byte row k holds camera row row0 + rows - 1 - k      */
    int32_t* out_face;              /* device or NULL: rows x image_width, the face index of
                                       the closest object's first hit, -1 for a miss        */
    uint32_t flags;                 /* ERAY_RENDER_* */
    uint64_t aa_seed;               /* anti-aliasing jitter stream: Philox4x32-10 keyed by
                                       aa_seed, counter (x, y, sample, 0) — replaces the
                                       reference's OS-seeded rand::thread_rng (engine.rs:49) */
    uint32_t band_rows;             /* 0: the rows are camera rows [row0, row0 + rows).  Else
                                       interleaved bands (a multi-GPU rank's share): local row j
                                       is camera row row0 + (j / band_rows) * band_stride +
                                       j % band_rows; band_rows a power of two >= 4,
                                       band_stride and row0 multiples of 4.  The outputs hold the local rows (out_ppm in local
                                       file order: byte row k = local row rows - 1 - k). */
    uint32_t band_stride;
} eray_render_params;

#define ERAY_RENDER_DEFAULT 0u
#define ERAY_RENDER_BRUTE_FORCE 1u  /* disable the exact per-wave triangle culling and the general tracer's background skip (A/B) */
/* Launch-shape overrides (tests / tuning; every choice renders the same image).  By default the
 * library picks them from the frame's detail sub-block count. */
#define ERAY_RENDER_DENSE_DETAIL 2u      /* large meshes: the 3-workgroups-per-CU detail build      */
#define ERAY_RENDER_NO_DENSE_DETAIL 4u   /* large meshes: the 2-workgroups-per-CU detail build      */
#define ERAY_RENDER_SEPARATE_FILL 8u     /* dense build: background fill in a second, parallel kernel */
#define ERAY_RENDER_NO_SEPARATE_FILL 16u /* dense build: background fill inside the frame kernel     */
#define ERAY_RENDER_SHARED_DETAIL 32u    /* binned meshes: every detail sub-block's search shared by its
                                            workgroup (default: only the heavy ones; the light ones
                                            search their own bins without workgroup barriers)     */

int eray_render(eray_ctx* ctx, const eray_render_params* params);
/* Renders `frames` frames back to back with the same parameters (a serving / animation loop
 * without a host round trip per frame): the frame launches are replayed from a HIP graph of up
 * to 64 frames, captured on the context's stream and cached for these parameters.  When
 * mean_frame_ms is not NULL, two HIP events on the stream bracket the frames and the mean
 * device time per frame is returned — the frame kernel back to back, within the graph's
 * inter-kernel gap of its own duration (this call then waits). */
int eray_render_frames(eray_ctx* ctx, const eray_render_params* params, uint32_t frames,
                       float* mean_frame_ms);
/* Builds (and caches) the launch plan eray_render_frames uses for these parameters and frame
 * count, without rendering: the one-time capture cost stays out of a timed or serving loop. */
int eray_render_prepare(eray_ctx* ctx, const eray_render_params* params, uint32_t frames);
/* Renders one frame per camera of `cameras` (host array of n), in order, into the same outputs —
 * Scene::set_camera + Engine::render per frame (scene.rs:39-54, engine.rs:46-81), e.g. an
 * animation or a serving loop whose camera moves every frame.  Every camera must have the scene
 * camera's Camera::size.  Each frame's camera setup (culling records, pixel rectangles, screen
 * bins, detail list) runs on the device right before its frame, with no host round trip, and the
 * frames are replayed from cached HIP graphs (the cameras are re-read every call).  When
 * mean_frame_ms is not NULL the call waits and returns the mean device time per frame, setup
 * included.  The scene camera (eray_scene_set_camera) is unchanged. */
int eray_render_camera_path(eray_ctx* ctx, const eray_render_params* params, const eray_camera* cameras,
                            uint32_t n, float* mean_frame_ms);

/* Frames in flight.  A serving or animation loop renders a stream of independent frames; the
 * ring variants below give frame k of a call its own outputs — ring slot k % slots, at
 * out_rgb + (k % slots) * rgb_stride (bytes; likewise out_ppm / out_face) — so that several frames
 * can be rendered by ONE kernel launch (frames_per_launch): one frame's latency-bound shading
 * chains then overlap the other frames' background stores instead of ending the launch alone.
 * Every frame is rendered in full, bit-identical to eray_render's; a slot stays valid until frame
 * k + slots of the same call overwrites it.  The plain eray_render_frames /
 * eray_render_camera_path are the ring calls with one slot (every frame into the same outputs,
 * one frame per launch). */
typedef struct eray_frame_ring {
    uint32_t slots;                 /* a power of two <= 64 */
    uint32_t frames_per_launch;     /* a power of two <= slots; 0: the library's choice (frames of
                                       up to 3840x2160 pixels together per launch, at most 8;
                                       anti-aliasing / bounces: 1) */
    uint64_t rgb_stride;            /* bytes between slots of each non-NULL output: a multiple of */
    uint64_t ppm_stride;            /* 16 and at least one slot's size (ignored when slots == 1) */
    uint64_t face_stride;
} eray_frame_ring;
int eray_render_frames_ring(eray_ctx* ctx, const eray_render_params* params, const eray_frame_ring* ring,
                            uint32_t frames, float* mean_frame_ms);
int eray_render_prepare_ring(eray_ctx* ctx, const eray_render_params* params, const eray_frame_ring* ring,
                             uint32_t frames);
/* The frames per launch the library picks (frames_per_launch = 0) for these parameters, the scene
 * camera and a ring of `slots` slots — e.g. to size a ring of exactly that many slots. */
uint32_t eray_frames_per_launch(eray_ctx* ctx, const eray_render_params* params, uint32_t slots);
/* Measurement: renders frames as eray_render_frames_ring does (same kernels, same ring slots;
 * max(1, frames / frames_per_launch) full launches, as plain launches, then waits) with every
 * frame kernel launched through hipExtLaunchKernel's start / stop events, which carry the
 * dispatch's own begin / end timestamps — the durations rocprofv3's kernel trace reports, free
 * of launch and graph gaps.  Frame kernel durations per launch (mean, min, max), the separate
 * background fill kernel's (0 when the launch shape has none) and each launch's span from the
 * first kernel's start to the last one's end. */
typedef struct eray_kernel_times {
    uint32_t launches;
    uint32_t frames_per_launch;
    float frame_kernel_ms;          /* mean over the launches */
    float frame_kernel_min_ms;
    float frame_kernel_max_ms;
    float fill_kernel_ms;
    float launch_span_ms;           /* mean */
} eray_kernel_times;
int eray_time_frames_ring(eray_ctx* ctx, const eray_render_params* params, const eray_frame_ring* ring,
                          uint32_t frames, eray_kernel_times* out);
/* Measurement: the write ceiling of the same launches — every frame's background bytes (the
 * frame kernel's fill with nothing to render) written into the same ring slots, frames per
 * launch and launch count as eray_time_frames_ring, by a plain block-strided store stream with
 * `wgs_per_cu` (1..8) workgroups per CU and no other work, dispatch-timed the same way
 * (frame_kernel_* fields).  The chip's own write rate for this ring in this process: the
 * reference point of the frame kernel's fill floor.  The slots hold background frames afterwards
 * (tagged as such: eray_gather_frames refuses them).  Whole 64 x 4 blocks only (image_width %
 * 64 == 0, rows % 4 == 0, aligned outputs), else ERAY_E_UNSUPPORTED. */
int eray_time_write_ceiling(eray_ctx* ctx, const eray_render_params* params, const eray_frame_ring* ring,
                            uint32_t frames, uint32_t wgs_per_cu, eray_kernel_times* out);
/* Camera paths of scenes whose per-camera setups are batched (no mesh over 256 faces) render
 * frames_per_launch frames per launch; others one (each camera rebuilds the screen bins). */
int eray_render_camera_path_ring(eray_ctx* ctx, const eray_render_params* params, const eray_frame_ring* ring,
                                 const eray_camera* cameras, uint32_t n, float* mean_frame_ms);

/* ------------------------------------------------------------------ multi-GPU ----------- *
 * One process (one context) per GPU; a frame is split into row tiles and gathered on rank 0
 * (SURVEY.md §8(e)).  Rank r of n renders the r-th block of PPM file rows — camera rows
 * [H - (r+1)*rows, H - r*rows) with out_ppm set — and eray_gather_rows concatenates the blocks on
 * rank 0 in rank order, which is the PPM body of Image::save_as_ppm (image.rs:48-74).  The gather
 * is one RCCL collective (xGMI) on the context's stream.  `nccl_comm` is an ncclComm_t: the
 * caller's own, or one made with eray_comm_init from an id that rank 0 got from
 * eray_comm_unique_id and sent to the other ranks by any means. */
#define ERAY_COMM_ID_BYTES 128
int eray_comm_unique_id(uint8_t* id /* ERAY_COMM_ID_BYTES */);
int eray_comm_init(eray_ctx* ctx, int nranks, int rank, const uint8_t* id, void** nccl_comm);
int eray_comm_destroy(void* nccl_comm);
/* The PPM body of a height x width frame on rank 0 (frame: device, height x width x 3 bytes),
 * from every rank's fused out_ppm rows (local: device).  band_rows == 0: rank r rendered the
 * r-th of nranks equal blocks of file rows (camera rows [H - (r+1) h, H - r h), h = height /
 * nranks), and the gather is a concatenation in rank order.  band_rows > 0: rank r rendered the
 * interleaved bands r, r + nranks, ... of band_rows camera rows (eray_render_params row0 =
 * r * band_rows, band_stride = nranks * band_rows) — equal work per rank wherever the scene
 * sits — into a local buffer of eray_band_rows(height, band_rows, nranks, 0) rows (rank 0 has
 * the most), and rank 0 puts the rows in file order.  With bands the rows travel coded: each
 * 64-pixel row segment whose pixels are all equal as one 4-byte word, the others as their bytes
 * (a frame is mostly the miss colour, engine.rs:212), so the transfer into rank 0 shrinks with
 * the background; the packed sizes are exchanged first and the call synchronises the context's
 * stream once (not capturable in a graph).  Without bands the ranks exchange a status word
 * first (one small all-gather, one stream synchronisation, every call).  Either way every rank
 * learns every rank's verdict on its own buffers before any rows move: a rank with a null `local`
 * (or rank 0 with a null `frame`, or no memory for its staging buffer) still takes part, and every
 * rank returns an error.  The words of those exchanges live in a block allocated with the context,
 * so no rank can fail to enter them.  At most 64 ranks (ERAY_E_UNSUPPORTED on every rank beyond).
 * Replaces the reference's single-process image write (engine.rs:85-98 render_to_path ->
 * save_as_ppm). */
int eray_gather_rows(eray_ctx* ctx, void* nccl_comm, const uint8_t* local, uint8_t* frame, uint32_t height,
                     uint32_t width, uint32_t band_rows);
/* `nframes` frames at once (frame k: local + k * local_stride on every rank, frames + k *
 * frame_stride on rank 0, or on its root with ERAY_GATHER_ROTATE_ROOT), e.g. a ring of
 * eray_render_frames_ring slots gathered while the next frames render on another stream.  flags:
 *   ERAY_GATHER_DEFAULT       — eray_gather_rows per frame.
 *   ERAY_GATHER_SCENE_CAMERA  — the local rows are this context's renders of its scene camera
 *     (eray_render / eray_render_frames[_ring] without anti-aliasing or bounces, over this rank's
 *     share: the band or block split above).  The frame kernel writes the miss colour (engine.rs:
 *     212) at every pixel outside the objects' pixel rectangles, where no primary ray can hit a
 *     face, so only the bytes inside those rectangles travel: each rank packs them, rank 0
 *     receives them with fixed-size point-to-point transfers and writes every frame row.  The
 *     ranks exchange their rectangles once per camera setup (the first call after a new setup
 *     synchronises the context's stream; a batch size's first call allocates); every later call
 *     only enqueues kernels and transfers — no host round trip, capturable in a HIP graph.
 *     Needs width % 16 == 0 (else ERAY_E_INVALID_ARGUMENT on every rank) and 16-byte aligned
 *     buffers and strides.  The frames must be of this context's latest render of its scene
 *     camera or of a camera path (anti-aliased, reflecting and brute-force renders do not count):
 *     the plan is made for that render, so older frames are refused.  Collective safety: every
 *     rank chooses what it does from the shared arguments and that render history (the same on
 *     every rank when the ranks make the same calls: SPMD), never from its own buffers; a rank
 *     whose own buffers or frames are unusable still takes part — in a new plan's exchange, whose
 *     verdict every rank then returns, or in a cached plan's transfers, whose headers carry its
 *     error — and returns its error.  A batch size's first call agrees on every rank's transfer
 *     buffer before any transfer (one stream synchronisation; a rank without the memory makes
 *     every rank return an error).  A root assembles a batch only when every transfer's header
 *     says ERAY_OK and the plan's source, otherwise it writes none of the batch's frames and its
 *     context's next eray_gather_frames (which first waits for that assembly) returns
 *     ERAY_E_INVALID_ARGUMENT; batches replayed from a captured graph are reported by the first
 *     call after them.  At most 64 ranks.
 *   ERAY_GATHER_ROTATE_ROOT   — with ERAY_GATHER_SCENE_CAMERA: frame k of the batch is assembled
 *     on rank k % nranks instead of rank 0, so the assembly writes and the inbound xGMI traffic of
 *     a stream of frames spread over every GPU.  Rank r's frames k = r, r + nranks, ... land at
 *     frames + j * frame_stride, j = (k - r) / nranks (every rank with r < nframes passes
 *     `frames`).  Each frame is still one complete PPM body on one GPU. */
#define ERAY_GATHER_DEFAULT 0u
#define ERAY_GATHER_SCENE_CAMERA 1u
#define ERAY_GATHER_ROTATE_ROOT 2u
int eray_gather_frames(eray_ctx* ctx, void* nccl_comm, const uint8_t* local, uint64_t local_stride, uint8_t* frames,
                       uint64_t frame_stride, uint32_t nframes, uint32_t height, uint32_t width, uint32_t band_rows,
                       uint32_t flags);
/* Camera rows of rank `rank` in the interleaved band split of a frame of `height` rows. */
uint32_t eray_band_rows(uint32_t height, uint32_t band_rows, uint32_t nranks, uint32_t rank);

/* ------------------------------------------------------------------ PPM ----------------- */
/* Body bytes of Image<Color>::save_as_ppm for a width x height device image: rows bottom-up,
 * each channel (c * 255.) as u8 (saturating, NaN -> 0). out: device, width*height*3 bytes. */
int eray_pack_ppm(eray_ctx* ctx, const float* rgb, uint32_t width, uint32_t height,
                  uint8_t* out);
/* Writes "P6 {width} {height} 255\n" into buf; *len receives its length (buf may be NULL). */
int eray_ppm_header(uint32_t width, uint32_t height, char* buf, size_t cap, size_t* len);

/* ------------------------------------------------------------------ .obj input ---------- */
/* Object::load_obj + Object::build (object.rs:101-230, 396-421): the .obj file at `path` in the
 * reference's dialect, as eray_object's per-face arrays (faces copy their vertices by value).
 * ERAY_E_IO: unreadable; ERAY_E_PARSE: an input the reference panics on; ERAY_E_BUILD: no
 * vertices or no normals.  The arrays are malloc'd; release them with eray_obj_free. */
typedef struct eray_obj_mesh {
    float* positions;    /* triangles x 9 (a, b, c) */
    float* normals;      /* triangles x 9 */
    float* uvs;          /* triangles x 6 */
    uint32_t triangles;
} eray_obj_mesh;
int eray_obj_load(const char* path, eray_obj_mesh* out);
void eray_obj_free(eray_obj_mesh* mesh);

#ifdef __cplusplus
}
#endif
#endif /* ERAY_HIP_H */
