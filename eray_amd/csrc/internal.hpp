// internal.hpp — descriptors shared by the C-ABI layer (capi.cpp) and the gfx950 kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <array>
#include <vector>

namespace eray {
namespace gpu {

// Hot per-triangle record of the exact test, 48 B (three 16-B loads), computed on the device
// from the face vertices with the reference's own operations (primitives.rs:44-46):
//   q0 = (e1.x, e1.y, e1.z, e2.x)   q1 = (e2.y, e2.z, n.x, n.y)   q2 = (n.z, a.x, a.y, a.z)
struct __align__(16) TriHot {
    float4 q0, q1, q2;
};

// Cold per-triangle shading record, 64 B, read only for the hit face:
//   s0 = (na.x, na.y, na.z, nb.x)  s1 = (nb.y, nb.z, nc.x, nc.y)
//   s2 = (nc.z, uva.u, uva.v, uvb.u)  s3 = (uvb.v, uvc.u, uvc.v, 0)
struct __align__(16) TriShade {
    float4 s0, s1, s2, s3;
};

// Camera-dependent culling record of a triangle for primary rays (see render.hip,
// "exact wave culling").  For each of the four conditions k in {u, v, w, n}:
//   f_k(x', y') = K_k + A_k x' + B_k y'   (a real-valued bound of the reference's test value
//   along the camera ray through viewport coordinate (x', y')), rejected for a whole pixel
//   rectangle when max f_k < -T_k.
struct __align__(16) TriCull {
    float4 A;  // A_u, A_v, A_w, A_n
    float4 B;
    float4 K;
    float4 T;  // thresholds (>= 0; +inf disables the condition)
};

struct TexView {
    const float* data;  // nullptr: the output is absent (Option::None)
    uint32_t w, h;
};

// One node of a material output's expression tree, evaluated per hit texel (hit.hpp
// texel_program): the host expands the shader graph (eray_texel_graph) per output into a tree in
// pre-order — a node shared along different paths is evaluated at each path's texel — where
// every node's texel derives from its parent's.
struct TexelInstr {  // 48 B
    uint32_t kind;    // eray_texel_node_kind
    uint32_t w, h;    // the node's image size
    uint32_t parent;  // instruction index of the parent (0: the root itself)
    uint32_t xform;   // kTexelMod: parent texel mod (w, h) (mix's mod_get); kTexelIndex: the
                      // parent's pixel index y * w_parent + x as (i % w, i / w) (rgb's pixels[i])
    float p[3];
    uint32_t c[3];    // children (later instructions; rgb's identical inputs share one)
    uint32_t pad;
};
constexpr uint32_t kTexelMod = 0, kTexelIndex = 1;
constexpr uint32_t kTexelMaxNodes = 32;  // per output tree
// Program header (uint32 words): first instruction and count per Material output (color,
// diffuse, specular, specular_power, reflection), count 0 = not a program output; then the
// instructions from word kTexelHeaderWords (48-B records).
constexpr uint32_t kTexelHeaderWords = 12;

struct MaterialDesc {
    TexView color;  // IColor, 3 floats per texel
    TexView diffuse, specular, specular_power, reflection;  // IValue
    // example: 1 = color and diffuse are main.rs's graph evaluated at the hit texel
    uint32_t example, ex_w, ex_h;
    float ex_xf, ex_yf, ex_r, ex_g, ex_b, ex_factor;
    // a shader graph per hit texel (eray_scene_set_object_texel_graph), or null
    const uint32_t* prog;
};

// Scenes up to these sizes are preloaded whole into each frame workgroup's LDS.
constexpr uint32_t kCacheTris = 256, kCacheObjects = 16, kCacheLights = 16;
// Objects with more faces than this are not scanned per wave: screen bins / LDS tiles.
constexpr uint32_t kDirectMax = 256;
// Screen bins of large objects' faces: kBinW x kBinH pixels (one wave's 16 x 4 sub-block).
constexpr uint32_t kBinW = 16, kBinH = 4;
// Bins of 65 to this many entries are sorted by face index (bins.hip bin_sort_kernel); longer
// ones keep the scatter's order.  In a sorted bin each full 64-entry chunk but the last also
// carries, in the pad words of its first two entries (low, high half), the union of the pixel
// masks of every later chunk: the frame kernel stops the bin once no pixel that can still improve
// is covered by what is left (render.hip first_hit_binned_wave).
constexpr uint32_t kBinSortMax = 1024;
// Detail rectangles carried in the kernel arguments (more objects: merged into the last one).
constexpr int kMaxRects = 8;
// Deepest reflection recursion the general tracer keeps frames for (Engine::bounces).
constexpr uint32_t kMaxBounces = 16;
// Frames one launch may render (eray_frame_ring::frames_per_launch <= slots <= 64).
constexpr uint32_t kMaxFramesPerLaunch = 64;
// The frame kernel reads triangle records (TriHot 48 B, TriShade 64 B) and bin entries (64 B) by
// buffer loads with 32-bit byte offsets (render.hip load_rec): a scene holds fewer than 2^26
// triangles (eray_scene_add_object refuses more) and a bin buffer at most 2^26 entries (a setup
// that needs more overflows: its objects are scanned through LDS tiles, still exact).
constexpr uint64_t kMaxSceneTris = (1ull << 26) - 1;
constexpr size_t kMaxBinEntries = (size_t)1 << 26;
// The multi-GPU gathers (comm.cpp) serve at most this many ranks, and every buffer a rank needs
// to take part in their status exchanges (status and count words, the plan records, the plan's
// rank table) lives in a scratch block allocated with the context — so no rank can fail to enter
// a collective its peers have entered for want of memory.
constexpr int kMaxGatherRanks = 64;
constexpr size_t kCollScratchBytes = 32u << 10;
// The MI355X Infinity Cache (the die's last-level cache, MI355X_MICROARCH.md).
constexpr uint64_t kInfinityCacheBytes = 256ull << 20;

// One entry of a screen bin (bins.hip): a face that may be hit in the bin, its intersection
// record, the bin's pixels it may cover (bit row * kBinW + column) and its index relative to the
// object's first face — one 64-B line, so the scatter that places an entry in its bin writes one
// line and a detail wave reads a 64-entry chunk as 4 KB of consecutive lines.
struct alignas(16) BinEntry {
    TriHot hot;
    unsigned long long mask;
    uint32_t tri;
    uint32_t pad;  // sorted bins: half of the later chunks' mask union (kBinSortMax), else 0
};
static_assert(sizeof(BinEntry) == 64, "one 64-B line per bin entry");

struct ObjGeom {  // what the triangle scans need of an object, 64 B
    uint32_t tri_begin, tri_count;
    // Camera pixels whose primary ray can hit the object: x0..x1 x y0..y1 (inclusive, camera
    // rows), from the culling records (tri_rect_kernel); empty when x0 > x1.
    int32_t rect[4];
    float bb_lo[3], bb_hi[3];
    // Screen bins of a large object's faces (bins.hip), or null: bin b's entries are
    // bin_ent[bin_start[b] .. bin_start[b + 1]) (bins of 65..kBinSortMax entries in increasing
    // face index, with the later chunks' mask unions, BinEntry).
    const uint32_t* bin_start;
    const BinEntry* bin_ent;
};

struct alignas(16) ObjectDesc {  // 192 B: the LDS scene copy moves whole 16-B words
    ObjGeom g;
    MaterialDesc mat;
};

struct LightDesc {
    float pos[3];
    int32_t variant;  // 0 point, 1 ambient
    float color[3];
    float brightness;
};

// A camera as the kernels use it (camera.rs:57-76): centre, Fov ratio fov0 / fov1 (computed on
// the host in f32, as Fov::ratio does) and z_dist.  Camera::size is fixed per frame plan.
struct CamDev {
    float cx, cy, cz, ratio, z_dist;
    uint32_t pad[3];
};

// Per-camera frame setup in device memory, written by the setup kernels (setup.hip, bins.hip)
// and read by the frame kernel in device-camera mode (FrameParams::cam_state): no host round
// trip between a camera change and its frame.
struct alignas(16) CamState {
    CamDev cam;                   // the camera of the setup (copied by the setup kernel)
    uint32_t nrect;               // detail rectangles (sub-block units, rank-local rows, disjoint)
    uint32_t total_sub;           // detail sub-blocks (rectangles' area, or the detail list's length)
    uint32_t bin_entries;         // (face, bin) entries the bins needed (host capacity sizing)
    uint32_t bin_overflow;        // the bins did not fit: binned objects fall back to LDS tiles
    // a split detail list (FrameParams::dlist_split, camera paths): heavy sub-blocks appended from
    // the front, light ones from the back (bins.hip detail_list_kernel)
    uint32_t heavy_sub, light_sub;
    int32_t rects[kMaxRects][4];  // x0, x1, y0, y1 (inclusive)
};

constexpr uint32_t kTraceSkipTris = 256;  // general tracer: largest scene with the background skip
// general tracer: a binned sub-block whose bin holds more entries is searched by a whole
// workgroup (trace.hip; the tracer's setup lists those first, bins.hip detail_flags_kernel)
constexpr uint32_t kTraceHeavyMin = 192;

struct FrameParams {
    // camera (camera.rs:57-76)
    float cx, cy, cz;
    float ratio;  // fov0 / fov1
    float z_dist;
    uint32_t cam_w, cam_h;
    // output
    uint32_t img_w, img_h;
    uint32_t row0, rows;
    // interleaved row bands (multi-GPU balance): local row j is camera row
    // row0 + (j >> band_shift) * band_stride + (j & band_mask) (band_rows = 1 << band_shift, a
    // power of two); a contiguous block is band_shift = 31, band_mask = 0x7fffffff (row0 + j)
    uint32_t band_shift, band_mask, band_stride;
    float* out_rgb;
    uint8_t* out_ppm;
    int32_t* out_face;
    uint32_t aligned;  // img_w % 16 == 0 and 16-byte aligned outputs: 16-byte row stores
    // scene
    const TriHot* tris;
    const TriShade* shade;
    const TriCull* cull;  // nullptr: brute force
    const ObjectDesc* objects;
    const LightDesc* lights;
    uint32_t nobj, nlights;
    uint32_t max_object_tris;  // selects the kernel variant with LDS triangle tiles
    uint32_t total_tris;
    uint32_t lds_scene;        // the scene is small enough to preload into LDS (kCache*)
    uint32_t nrect;            // detail rectangles (sub-block units: 16 px x 4 rank-local rows,
    uint32_t total_sub;        // inclusive) and the number of sub-blocks they cover, counting
    int32_t rects[kMaxRects][4];  // overlaps once: x0, x1, y0, y1
    uint32_t spec_pow;         // some material has a specular-power output (powf != identity)
    uint32_t example_mat;      // some material evaluates main.rs's graph per hit (example)
    uint32_t tiles_x;    // 64 x 4 pixel blocks per row
    uint32_t bins_x;     // screen bins per row
    uint32_t bin_phase;  // bins start at camera rows bin_phase + k * kBinH (row0 % kBinH)
    // Detail sub-block list (scenes with binned objects, bins.hip detail_list_kernel): the j-th
    // detail sub-block is detail_list[j] = sy << 16 | sx (sub-block units, rank-local rows) and
    // bit i of detail_occ[block] marks sub-block i of 64 x 4 block `block` as listed.  Null: the
    // detail rectangles enumerate the sub-blocks.
    const uint32_t* detail_list;
    const uint8_t* detail_occ;
    // the ordered detail list's heavy sub-blocks (its first detail_heavy[0] entries: a bin of more
    // than one 64-entry chunk), or null (an unordered list: every sub-block treated as heavy)
    const uint32_t* detail_heavy;
    uint32_t detail_wgs;  // most workgroups of the frame kernel's grid doing detail work (0: all)
    uint32_t fill_first;  // the fill workgroups take the grid's first block indices (dispatched first)
    uint32_t separate_fill;  // the frame kernel does detail work only; fill_kernel writes the background
    uint32_t fill_cap;       // at most this many workgroups write the background (0: no cap)
    // device-camera mode: camera, detail rectangles and detail count come from the setup
    // kernels' CamState (the host has not read them back); null: the fields above hold them
    const CamState* cam_state;
    // device-camera mode's fill reservation (launch_frame_kernel computes it on the host in
    // args mode): detail workgroups at the default share and at the small-scene share used
    // when the detail sub-blocks exceed one round (frame_kernel decides from the count)
    uint32_t detail_wgs_alt;
    uint32_t launch_flags;  // ERAY_RENDER_* launch overrides (dense / separate fill), part of the plan key
    // general tracer (trace.hip): anti-aliasing rays per pixel, reflection depth, jitter seed;
    // aa == 0 && bounces == 0 selects the frame kernel
    uint32_t aa, bounces;
    uint32_t seed_lo, seed_hi;
    // trace_kernel's culling records for this camera (scenes of at most kTraceSkipTris faces;
    // null: no background skip), written by trace_cull_kernel when the camera or the scene changes
    TriCull* trace_cull;
    // trace_kernel's camera rays scan the binned objects' screen bins (a setup with
    // SetupParams::keep_all; the descriptors' bin views and rectangles), else every face
    uint32_t trace_bins;
    // ... over the setup's detail list (the sub-blocks some ray of which may hit a face; detail_occ
    // per 64 x 4 block): trace_heavy_kernel's workgroups take the heavy head of the list, a
    // workgroup per sub-block; trace_binned_kernel's first trace_fill_wgs workgroups write the
    // background of the unlisted sub-blocks and the next trace_light_wgs the light list, a wave
    // per sub-block
    uint32_t trace_heavy_wgs, trace_fill_wgs, trace_light_wgs;
    // Frames in flight: one launch renders `nframes` (>= 1) independent frames, its workgroups
    // dealt round-robin over them (frame_kernel).  Frame f writes out_* + f * *_stride (bytes,
    // multiples of 16) and, with dev_slots, reads the batched per-camera setup of slot f
    // (cam_state + f, cull + f * total_tris, objects + f * nobj: launch_camera_setup_batch) and,
    // for scenes with binned objects (the multi-camera setup), its detail list at detail_list +
    // f * dlist_stride and occupancy at detail_occ + f * dlist_stride / 4.
    uint32_t nframes;
    uint32_t dev_slots;
    uint32_t dlist_stride;
    // device-camera mode with a split detail list of this capacity (0: none): list position j of
    // CamState::heavy_sub heavy sub-blocks is j, of a light one dlist_split - 1 - (j - heavy_sub)
    uint32_t dlist_split;
    uint64_t rgb_stride, ppm_stride, face_stride;
    // frame stores also non-temporal (launch_render: a launch whose outputs exceed the 256 MiB
    // Infinity Cache — the frame's lines then do not evict what the detail waves read back)
    uint32_t store_nt;
};

// Camera row of rank-local row j (FrameParams::band_shift; shifts and masks: no division in the
// kernels' per-pixel paths).
__host__ __device__ inline uint32_t band_camera_row(uint32_t row0, uint32_t band_shift, uint32_t band_mask,
                                                    uint32_t band_stride, uint32_t j) {
    return row0 + (j >> band_shift) * band_stride + (j & band_mask);
}
// The rank-local rows [*lo, *hi] whose camera rows lie in [y0, y1] (empty: *lo > *hi); the
// mapping is monotonic, so a camera row range is a local row range.
__host__ __device__ inline void band_local_range(uint32_t row0, uint32_t band_shift, uint32_t band_stride, int32_t y0,
                                                 int32_t y1, int32_t* lo, int32_t* hi) {
    if (band_shift >= 31) {
        *lo = y0 - (int32_t)row0;
        *hi = y1 - (int32_t)row0;
        return;
    }
    const int64_t B = (int64_t)1 << band_shift, S = band_stride, off = row0;
    auto floordiv = [](int64_t a, int64_t b) { return a >= 0 ? a / b : -((-a + b - 1) / b); };
    // first local row at or after camera row y0
    int64_t i = floordiv((int64_t)y0 - off, S), w = (int64_t)y0 - off - i * S;
    const int64_t l0 = w < B ? i * B + w : (i + 1) * B;
    // last local row at or before camera row y1
    i = floordiv((int64_t)y1 - off, S);
    w = (int64_t)y1 - off - i * S;
    const int64_t l1 = w < B ? i * B + w : i * B + B - 1;
    *lo = (int32_t)(l0 < -1 ? -1 : (l0 > 0x7fffffff ? 0x7fffffff : l0));
    *hi = (int32_t)(l1 < -1 ? -1 : (l1 > 0x7fffffff ? 0x7fffffff : l1));
}

// Byte offsets of the LDS scene copy: [ObjectDesc x nobj | LightDesc x nl | TriCull x n (if
// culling) | TriHot x n | TriShade x n]; every section is a whole number of 16-B words.
struct SceneLdsLayout {
    uint32_t objs, lights, cull, hot, shade, bytes;
};
__host__ __device__ inline SceneLdsLayout scene_lds_layout(uint32_t nobj, uint32_t nl, uint32_t n, bool cull) {
    SceneLdsLayout L;
    L.objs = 0;
    L.lights = L.objs + nobj * (uint32_t)sizeof(ObjectDesc);
    L.cull = L.lights + nl * (uint32_t)sizeof(LightDesc);
    L.hot = L.cull + (cull ? n * (uint32_t)sizeof(TriCull) : 0u);
    L.shade = L.hot + n * (uint32_t)sizeof(TriHot);
    L.bytes = L.shade + n * (uint32_t)sizeof(TriShade);
    return L;
}
static_assert(sizeof(ObjectDesc) % 16 == 0 && sizeof(LightDesc) % 16 == 0, "16-B words");

// ------------------------------------------------------------- launchers (.hip files) ------
hipError_t launch_tri_precompute(const float* pos, const float* nrm, const float* uv, uint32_t T,
                                 TriHot* hot, TriShade* shade, hipStream_t s);
// ------------------------------------------------------------- per-camera setup (setup.hip)
// Everything a camera change needs before its frame, enqueued on the stream with no host round
// trip (so a camera path can be graph-replayed): per triangle the culling record (TriCull) and
// its conservative pixel rectangle, per object the union of those (ObjGeom::rect, written into
// the device descriptors), for binned objects each face's bin rectangle (bins.hip), and, for
// scenes without binned objects, the merged detail rectangles of the rendered rows (CamState).
// camera_setup_kernel's grid: at most this many workgroups, each a contiguous chunk of triangles —
// the workgroups resident at once on MI355X (its chunk pass holds 131 VGPRs and 36.9 KB of LDS:
// 3 per CU x 256 CUs), so a multi-camera setup runs in one round, not 1.33 (1024: a tail round of
// 256 workgroups; same-box A/B profiles/r06/ab/ab_r06q_setup_grid.txt: moving 3840x2160 / 70k
// 46.2 -> 44.7 us, moving 1M faces 268.6 -> 255.5 us per frame)
constexpr uint32_t kSetupMaxBlocks = 768;
// camera_setup_kernel's chunk workgroups for T triangles (each a contiguous chunk of
// ceil(T / blocks) faces)
inline uint32_t setup_blocks(uint32_t T) {
    const uint32_t b = (T + 255u) / 256u;
    return T ? (b < kSetupMaxBlocks ? b : kSetupMaxBlocks) : 1u;
}
struct SetupParams {
    const TriHot* hot;
    TriCull* cull;
    uint32_t T;                 // all triangles of the scene
    ObjectDesc* objs;           // device descriptors (rect written)
    uint32_t nobj;
    const uint32_t* obj_begin;  // nobj + 1: first triangle of each object, then T
    const uint32_t* objkey;     // nobj: the object's binned-object index, or ~0u
    const CamDev* cam;          // the camera to set up (device)
    CamState* state;
    uint32_t W, H;              // Camera::size
    uint32_t row0, rows;        // rendered camera rows (the merged rectangles are rank-local)
    uint32_t band_shift, band_mask, band_stride;  // interleaved bands (FrameParams)
    uint32_t* acc;              // 4 x nobj rectangle accumulators, zero between setups
    uint32_t* done;             // workgroup counter (last-workgroup finalisation), zero between setups
    uint32_t* part;             // kSetupMaxBlocks x 10: each workgroup's boundary objects' partials
    uint32_t binned;            // some object is binned: bins.hip narrows rects + builds the detail list
    // binned objects' faces (bins.hip): bin rectangle and its number of units per face (bin_segments:
    // rows of the rectangle, else its bins; zero for other faces), the binned-object index per face
    int4* range;
    unsigned long long* area;
    uint32_t* fkey;
    uint32_t bins_x, phase;
    // the general tracer's setup (trace.hip): culling records and rectangles over the viewport
    // its jittered anti-aliasing rays reach, bin masks of the pixels any of whose rays may pass
    // (face_rect.hpp bin_pixels_jittered)
    uint32_t keep_all;
    uint32_t rect_pairs;  // (diagnostics) the rectangle-pair form where segments apply (bin_segments)
    // Several cameras in one setup (ncam > 1: camera paths of scenes with binned objects): the
    // cameras sp.cam[0 .. ncam), T = ncam * T1 "faces" (face i is face i % T1 of camera i / T1:
    // its culling record, bin rectangle and pairs), nobj = ncam * nobj1 descriptors (camera k's
    // copy of object o at k * nobj1 + o), ncam * nb1 binned objects (camera k's copy of binned
    // object j is k * nb1 + j), ncam CamStates; the bins and their detail lists per camera.
    uint32_t ncam, T1, nobj1, nb1;
    const ObjectDesc* objs_src;  // batched setups: the scene's descriptors, copied into each slot
    // binned faces' first unit: the exclusive scan of `area`, as each chunk workgroup's own scan
    // (first_local) plus its chunk's offset boff[b] (kSetupMaxBlocks + 1 entries; boff[nparts] =
    // all units) — bins.hip bin_segments_kernel / bin_pairs_kernel read them
    unsigned long long* first_local;
    unsigned long long* boff;
    // Camera paths (eray_gather_frames' layout of path frames): every camera's final object
    // rectangles also fold into this union (object o % union_nobj: x0, y0 minimised at
    // path_union[2 o ..], x1, y1 maximised at path_union[2 union_nobj + 2 o ..]), or null
    int32_t* path_union;
    uint32_t union_nobj;
};
hipError_t launch_camera_setup(const SetupParams& sp, hipStream_t s);
// The units the setup enumerates per binned face (`area`, and the scan first_local / boff over
// them): its bin rectangle's rows (bins.hip bin_segments_kernel) for the frame kernel's bins, its
// (face, bin) pairs for the general tracer's (bin_pairs_kernel) and for frames wider than the
// segments' 16-bit columns.
__host__ __device__ inline bool bin_segments(const SetupParams& sp) {
    return !sp.keep_all && !sp.rect_pairs && sp.W <= 65535u;
}
// The setups of `ncam` cameras sp.cam[0 .. ncam) at once, one workgroup each, into per-camera
// slots: culling records sp.cull + k * T, descriptors sp.objs + k * nobj (sp.objs_src with the
// camera's rectangles), state sp.state + k.  Scenes without binned objects and at most
// kSetupBatchMaxObjects objects (every object's union stays in the workgroup's LDS).
constexpr uint32_t kSetupBatchMaxObjects = 256;
hipError_t launch_camera_setup_batch(const SetupParams& sp, uint32_t ncam, hipStream_t s);
// A camera path's rectangle union (SetupParams::path_union, 4 nobj words) copied to `host` (mapped
// pinned memory, read by the host after the stream passes this point) and reset for the next
// path: x0, y0 to INT_MAX, x1, y1 to INT_MIN.  host null: the reset alone.
hipError_t launch_union_flush(int32_t* acc, uint32_t nobj, int32_t* host, hipStream_t s);
// Folds an object's final pixel rectangle r (x0, x1, y0, y1; skipped when empty) into the union.
__device__ __forceinline__ void union_rect(int32_t* u, uint32_t nobj, uint32_t o, const int32_t* r) {
    if (r[0] > r[1] || r[2] > r[3]) return;
    atomicMin(u + 2 * o, r[0]);
    atomicMin(u + 2 * o + 1, r[2]);
    atomicMax(u + 2 * nobj + 2 * o, r[1]);
    atomicMax(u + 2 * nobj + 2 * o + 1, r[3]);
}
// Writes `cam` into the device camera slot (kernel arguments: no host staging buffer to race).
hipError_t launch_set_camera(const CamDev& cam, CamDev* slot, hipStream_t s);
// Launch overrides of eray_render_params::flags (eray_hip.h ERAY_RENDER_*) the frame launcher reads.
constexpr uint32_t kLaunchDense = 2u, kLaunchNoDense = 4u, kLaunchSeparateFill = 8u, kLaunchNoSeparateFill = 16u,
                   kLaunchSharedDetail = 32u;
// (internal, set per launch by the ring plan: the ring's slots together exceed the Infinity Cache)
constexpr uint32_t kLaunchRingBeyondCache = 1u << 16;
// Per-context launch resources: the separate fill kernel's stream and its fork / join events.
// Measurement (eray_time_frames_ring): when frame_t[0] is set, the frame kernel is launched with
// hipExtLaunchKernel's start / stop events, which take the dispatch's own begin / end timestamps
// (the figures rocprofv3's kernel trace reports); fill_t likewise for the separate fill kernel.
struct LaunchCtx {
    hipStream_t side;
    hipEvent_t fork, join;
    hipEvent_t frame_t[2] = {nullptr, nullptr};
    hipEvent_t fill_t[2] = {nullptr, nullptr};
    uint32_t* fill_used = nullptr;  // set to 1 when the launch ran the separate fill kernel
};
// The frame kernel, or the general tracer (trace.hip) when p.aa or p.bounces is set.
hipError_t launch_render(const FrameParams& p, const LaunchCtx& lc, hipStream_t s);
hipError_t launch_trace(const FrameParams& p, const LaunchCtx& lc, hipStream_t s);
// Measurement (eray_time_write_ceiling): the frames' background bytes as one plain block-strided
// write stream of wgs_per_cu workgroups per CU (render.hip ceiling_fill_kernel), timed by t.
hipError_t launch_write_ceiling(const FrameParams& p, uint32_t wgs_per_cu, const hipEvent_t (&t)[2], hipStream_t s);
hipError_t launch_trace_cull(const FrameParams& p, hipStream_t s);

// ------------------------------------------------------------- screen bins (bins.hip)
// Device arrays of the binned objects' screen bins for one layout (camera size, row phase, the
// binned objects), all preallocated: a camera's bins are rebuilt on the stream with no host
// round trip.  Bin key = k * nbins + bin for binned object k; a bin's entries (face relative to
// the object, pixel mask, intersection record) are unordered — the frame kernel keeps the
// smallest face index that hits, which is the reference's first hit (object.rs:63-78).
struct BinBuffers {
    uint32_t nb = 0, nbins = 0, bins_x = 0, bins_y = 0, phase = 0, T = 0;
    size_t cap = 0;                       // entry capacity
    unsigned long long* first = nullptr;  // SetupParams::first_local (T)
    unsigned long long* boff = nullptr;   // SetupParams::boff (kSetupMaxBlocks + 1)
    uint32_t nparts = 0, chunk = 0;       // the setup's chunk workgroups and faces per chunk
    uint32_t* count = nullptr;            // per key (nb * nbins + 1), zero between builds
    uint32_t* start = nullptr;            // per key + 1
    uint32_t* kbegin = nullptr;           // tri_begin per binned object
    uint32_t* kobj = nullptr;             // object index per binned object
    uint32_t* n = nullptr;                // entries found (device counter, reset by the finaliser)
    uint32_t* done = nullptr;             // workgroup counter of the finaliser
    uint32_t* acc = nullptr;              // rectangle accumulators of the non-empty bins (a line per object)
    uint32_t* part = nullptr;             // 10 per finaliser workgroup: its end objects' partials
    uint32_t* ekey = nullptr;             // unscattered entries (cap)
    uint32_t* eface = nullptr;
    unsigned long long* emask = nullptr;
    uint32_t* erank = nullptr;            // the entry's place among its bin's entries (count's old value)
    BinEntry* ent = nullptr;              // bin entries in key order (cap)
    // detail sub-block list of the rendered rows
    uint8_t* dflags = nullptr;            // listed sub-blocks whose bin holds more than one chunk
    uint8_t* dflags_light = nullptr;      // ... and the other listed ones
    uint32_t* dpacked = nullptr;
    uint32_t* dlist = nullptr;
    uint32_t* dlight = nullptr;           // the light ones, appended to dlist after the heavy ones
    uint32_t* dcount = nullptr;           // [heavy, light] counts
    uint8_t* docc = nullptr;
    uint32_t* sortq = nullptr;            // bins to sort by face index (bins.hip bin_sort_kernel)
    uint32_t* nsort = nullptr;            // their count, zero between builds
    size_t nsub = 0;
    void* temp = nullptr;                 // hipcub scratch
    size_t temp_bytes = 0;
};
// (Re)allocates `b` for T triangles, nb binned objects (kbegin / kobj: host arrays), a W x H
// camera, row phase and `rows` rendered rows, entry capacity `cap` (synchronises `s` when it
// reallocates); the detail lists of `ncam` cameras (a multi-camera setup, SetupParams::ncam).
hipError_t bins_alloc(BinBuffers& b, uint32_t T, uint32_t nb, const uint32_t* kbegin, const uint32_t* kobj, uint32_t W,
                      uint32_t H, uint32_t phase, uint32_t tiles_x, uint32_t rows, size_t cap, hipStream_t s,
                      uint32_t ncam = 1);
void bins_free(BinBuffers& b);
// After launch_camera_setup: the bins of the setup's camera, the binned objects' rectangles
// narrowed to their non-empty bins and their bin views in the descriptors (or none when the
// entries overflow the capacity: the frame kernel then scans those objects through LDS tiles),
// and the detail sub-block list of rows [row0, row0 + rows) with CamState::total_sub.
hipError_t launch_bins_build(const SetupParams& sp, BinBuffers& b, uint32_t tiles_x, bool ordered, hipStream_t s);
hipError_t launch_pack_ppm(const float* rgb, uint32_t w, uint32_t h, uint8_t* out, hipStream_t s);

// ------------------------------------------------------------- capi.cpp internals for comm.cpp
// Where a frame in an output buffer came from (eray_gather_frames' scene-camera transport): the
// context tags every PPM output slot it renders into with the render's kind and key.  kind
// kSrcScene: a frame kernel render of the scene camera, key = a hash of (camera, scene
// generation, Camera::size) — the same on every rank that made the same scene calls, whatever
// internal re-setups (bin capacity growth) a rank did; kSrcPath: a frame of a camera path, key =
// the context's path call counter; kSrcOther: anti-aliasing / bounces / brute force.
constexpr uint32_t kSrcNone = 0, kSrcScene = 1, kSrcPath = 2, kSrcOther = 3;
struct FrameSource {
    uint32_t kind = kSrcNone;
    uint64_t key = 0;
    uint32_t W = 0, H = 0;
    uint32_t row0 = 0, rows = 0, band_shift = 0, band_stride = 0;  // the rendered rows
};
// The pixel rectangles of a source (every object's ObjGeom::rect: x0, x1, y0, y1 inclusive, camera
// rows; empty when x0 > x1; for a camera path the union over its cameras) — outside them every
// frame of the source is the background colour.
struct SceneLayout {
    FrameSource src;
    std::vector<std::array<int32_t, 4>> rects;
};

hipError_t launch_wave(uint32_t w, uint32_t h, float xf, float yf, float* out, hipStream_t s);
hipError_t launch_rgb(uint32_t w, uint32_t h, const float* r, const float* g, const float* b,
                      float* out, hipStream_t s);
hipError_t launch_flat(uint32_t w, uint32_t h, float r, float g, float b, float* out,
                       hipStream_t s);
hipError_t launch_mix(uint32_t w, uint32_t h, TexView left, TexView right, float factor,
                      float* out, hipStream_t s);
hipError_t launch_material_example(uint32_t w, uint32_t h, float xf, float yf, float r, float g,
                                   float b, float factor, float* color, float* diffuse,
                                   hipStream_t s);

}  // namespace gpu
}  // namespace eray
