// capi.cpp — implementation of include/eray_hip.h: context, device memory, scene upload and
// kernel launches.  Host code only; the kernels live in render.hip and shaderlib.hip.
//
// Error policy: every HIP call is checked; failures and every case where the reference would
// panic become a status code plus a message (eray_last_error).  Nothing here falls back to a
// CPU path: without a usable GPU the calls fail loudly.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <cstddef>
#include <string>
#include <vector>

#include "../../include/eray_hip.h"
#include "internal.hpp"

using namespace eray::gpu;

namespace {
thread_local std::string g_thread_error;
constexpr size_t kMaxTags = 512;
constexpr uint32_t kUnionRing = 4;

struct HostObject {
    std::vector<float> raw;  // T*9 positions | T*9 normals | T*6 uvs
    uint32_t T = 0;
    float lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
    eray_material mat{};
    bool example = false;  // color + diffuse from main.rs's graph at the hit texel
    eray_material_example_params ex{};
    std::vector<eray_texel_node> tnodes;  // a shader graph per hit texel (texel_graph)
    int32_t tout[5] = {-1, -1, -1, -1, -1};
};

// Node types of the shaderlib outputs: wave's is IValue, rgb / flat_color / mix_color's IColor.
bool texel_is_color(uint32_t kind) { return kind != ERAY_TEXEL_WAVE; }

// Expands node `idx` of `nodes` (evaluated at a texel derived from instruction `parent` by
// `xform`) into pre-order instructions; indices are relative to `first`.
uint32_t texel_emit(const std::vector<eray_texel_node>& nodes, uint32_t idx, uint32_t parent, uint32_t xform,
                    size_t first, std::vector<TexelInstr>& ins) {
    const eray_texel_node& nd = nodes[idx];
    const uint32_t k = (uint32_t)(ins.size() - first);
    TexelInstr t{};
    t.kind = nd.kind;
    t.w = nd.width;
    t.h = nd.height;
    t.parent = parent;
    t.xform = xform;
    for (int j = 0; j < 3; ++j) t.p[j] = nd.param[j];
    ins.push_back(t);
    if (ins.size() - first > kTexelMaxNodes) return k;  // the caller reports the size
    if (nd.kind == ERAY_TEXEL_RGB) {
        uint32_t c[3];
        for (int j = 0; j < 3; ++j) {
            int same = -1;  // rgb's inputs at the same node read the same pixel index: share
            for (int q = 0; q < j; ++q)
                if (nd.input[q] == nd.input[j]) same = q;
            c[j] = same >= 0 ? c[same] : texel_emit(nodes, (uint32_t)nd.input[j], k, kTexelIndex, first, ins);
        }
        for (int j = 0; j < 3; ++j) ins[first + k].c[j] = c[j];
    } else if (nd.kind == ERAY_TEXEL_MIX_COLOR) {
        const uint32_t l = texel_emit(nodes, (uint32_t)nd.input[0], k, kTexelMod, first, ins);
        const uint32_t r = texel_emit(nodes, (uint32_t)nd.input[1], k, kTexelMod, first, ins);
        ins[first + k].c[0] = l;
        ins[first + k].c[1] = r;
    }
    return k;
}
}  // namespace

struct eray_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::string err;

    eray_camera camera{{0.0f, 0.0f, 0.0f}, {60.0f, 60.0f}, 1024u, 1.0f};  // Camera::default()
    std::vector<eray_light> lights;
    std::vector<HostObject> objects;

    bool geom_dirty = true, desc_dirty = true;
    uint64_t scene_gen = 0;  // bumped whenever geometry or descriptors are uploaded
    TriHot* d_hot = nullptr;
    TriShade* d_shade = nullptr;
    TriCull* d_cull = nullptr;
    TriCull* d_tcull = nullptr;  // kTraceSkipTris records: trace.hip's background skip
    size_t tri_cap = 0;
    float* d_raw = nullptr;
    size_t raw_cap = 0;
    ObjectDesc* d_objs = nullptr;
    size_t objs_cap = 0;
    LightDesc* d_lights = nullptr;
    size_t lights_cap = 0;
    // launch plans of eray_render_frames / eray_render_camera_path: HIP graphs of back-to-back
    // frames (chunks of up to kGraphFrames frames and remainders), each cached for the frame
    // parameters + stream + length + kind it was captured with; the least recently used is
    // evicted beyond kGraphCache
    struct FrameGraph {
        hipGraph_t graph = nullptr;
        hipGraphExec_t exec = nullptr;
        std::vector<unsigned char> key;
        uint64_t used = 0;
    };
    std::vector<FrameGraph> graphs;
    uint64_t graph_clock = 0;
    uint32_t* d_prog = nullptr;  // every object's texel program (MaterialDesc::prog), concatenated
    size_t prog_cap = 0;
    std::vector<uint32_t> h_prog;
    std::vector<ObjectDesc> h_objs;  // kept alive for the async uploads
    std::vector<LightDesc> h_lights;
    std::vector<float> h_raw;
    std::vector<uint32_t> h_begin;   // obj_begin (nobj + 1) | objkey (nobj), uploaded with the descriptors
    uint32_t total_tris = 0;
    bool spec_pow = false;     // some material has a specular-power output
    bool example_mat = false;  // some material is main.rs's graph evaluated per hit
    // ---- per-camera setup (setup.hip, bins.hip), all on the device
    CamDev* d_cam = nullptr;      // the context camera's device slot
    CamState* d_state = nullptr;  // the last setup's results
    CamState* h_state = nullptr;  // pinned host copy, valid once state_ev has completed
    hipEvent_t state_ev = nullptr;
    bool state_pending = false;   // a copy into h_state is in flight
    bool state_known = false;     // h_state holds the results of the setup of setup_key
    std::vector<uint64_t> setup_key;  // camera, size, rows and scene generation of the last setup
    std::vector<uint64_t> tcull_key;  // camera, size, scene generation and stream of d_tcull's records
    FrameSource setup_src;        // the last enqueued scene-camera setup: its source key and rows
    ObjectDesc* h_objs_state = nullptr;  // pinned copy of the descriptors after that setup (pixel rectangles)
    size_t h_objs_state_cap = 0;
    // where the frames in output buffers came from (eray_gather_frames): PPM slot address -> the
    // source of the last render enqueued into it, most recent last (at most kMaxTags)
    struct SlotTag {
        uintptr_t ppm;
        FrameSource src;
    };
    std::vector<SlotTag> slot_tags;
    // camera paths: call counter (kSrcPath keys) and the union of every path camera's object
    // rectangles — accumulated on the device (d_union_acc, captured into path graphs), then copied
    // into ring entry seq % kUnionRing on the device and the host, with an event per entry
    uint64_t path_seq = 0;
    int32_t* d_union_acc = nullptr;
    size_t union_cap = 0;  // objects per entry
    int32_t* h_union = nullptr;
    int32_t* d_union_host = nullptr;  // h_union's device address (mapped)
    uint64_t union_seq[4] = {0, 0, 0, 0};
    FrameSource union_src[4];
    uint32_t union_nobj[4] = {0, 0, 0, 0};  // objects and scene generation the entry's union covers
    uint64_t union_gen[4] = {0, 0, 0, 0};
    hipEvent_t union_ev[4] = {nullptr, nullptr, nullptr, nullptr};
    // eray_gather_frames' plan (comm.cpp owns it)
    void* gather_plan = nullptr;
    void (*gather_plan_free)(void*) = nullptr;
    uint32_t* d_acc = nullptr;    // setup counter, partials and rectangle accumulators (enqueue_setup)
    size_t acc_cap = 0;
    uint32_t* d_begin = nullptr;  // obj_begin | objkey
    size_t begin_cap = 0;
    int4* d_range = nullptr;      // binned faces' bin rectangles, areas, binned-object index
    unsigned long long* d_area = nullptr;
    uint32_t* d_fkey = nullptr;
    size_t face_cap = 0;
    BinBuffers bins;
    std::vector<uint64_t> bins_layout;
    uint64_t bins_gen = 0;        // bumped whenever bins_alloc (re)allocates the bin buffers
    size_t bin_cap = 0;           // entry capacity to allocate (grown when a setup overflows)
    bool rect_pairs = false;      // (diagnostics) setups walk the bin rectangles' pairs (bins.hip)
    // camera paths (eray_render_camera_path): the cameras of the current graph chunk on the
    // device, the whole path staged in pinned memory
    CamDev* d_path = nullptr;
    size_t path_cap = 0;
    CamDev* d_path_all = nullptr;
    size_t path_all_cap = 0;
    // two pinned staging buffers used in turn: a call waits only for the upload two calls back
    // (not for the previous call's frames, which its upload is queued behind)
    CamDev* h_path[2] = {nullptr, nullptr};
    size_t h_path_cap[2] = {0, 0};
    hipEvent_t path_ev[2] = {nullptr, nullptr};  // each buffer's last upload (reusable once complete)
    uint32_t path_buf = 0;
    // batched setups of a path chunk's cameras (scenes without binned objects): per camera slot
    // its culling records, object descriptors and setup state
    TriCull* d_bcull = nullptr;
    size_t bcull_cap = 0;
    ObjectDesc* d_bobjs = nullptr;
    size_t bobjs_cap = 0;
    CamState* d_bstate = nullptr;
    size_t bstate_cap = 0;
    // camera paths of scenes with binned objects: the setups of up to mc_k cameras in one
    // multi-camera build (SetupParams::ncam), into per-camera slices of a buffer set; two sets, so
    // that the next cameras' build (on mc_stream) runs beside the current cameras' frames
    struct MultiSet {
        TriCull* cull = nullptr;
        ObjectDesc* objs = nullptr;
        CamState* state = nullptr;
        uint32_t* acc = nullptr;
        int4* range = nullptr;
        unsigned long long* area = nullptr;
        uint32_t* fkey = nullptr;
        BinBuffers bins;
    };
    MultiSet mc[2];
    uint32_t mc_k = 0;
    std::vector<uint64_t> mc_layout;
    uint64_t mc_gen = 0;          // bumped whenever the multi-camera buffers are (re)allocated
    hipStream_t mc_stream = nullptr;
    hipEvent_t mc_fork = nullptr, mc_ready[2] = {nullptr, nullptr}, mc_free[2] = {nullptr, nullptr};
    // the latest render of the scene camera or of a camera path (tag_frames): what a scene-camera
    // gather plans for — state every rank holds alike when the ranks make the same render calls
    FrameSource gather_src;
    uint8_t* d_coll = nullptr;     // kCollScratchBytes: the gathers' status exchanges (comm.cpp)
    uint8_t* d_staging = nullptr;  // eray_gather_rows' banded staging (rank 0)
    size_t staging_cap = 0;
    LaunchCtx lc{nullptr, nullptr, nullptr};  // the separate fill's stream and events
};

namespace {

int set_error(eray_ctx* ctx, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (ctx)
        ctx->err = buf;
    else
        g_thread_error = buf;
    return code;
}

#define HIP_TRY(ctx, expr)                                                                   \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return set_error((ctx), e_ == hipErrorOutOfMemory ? ERAY_E_OUT_OF_MEMORY : ERAY_E_HIP, \
                             "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
    } while (0)

int use_device(eray_ctx* ctx) {
    if (!ctx) return set_error(nullptr, ERAY_E_INVALID_ARGUMENT, "null context");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    return ERAY_OK;
}

template <typename T>
int ensure(eray_ctx* ctx, T** ptr, size_t* cap, size_t need) {
    if (need <= *cap && *ptr) return ERAY_OK;
    if (*ptr) {
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        HIP_TRY(ctx, hipFree(*ptr));
        *ptr = nullptr;
        *cap = 0;
    }
    size_t n = need ? need : 1;
    HIP_TRY(ctx, hipMalloc((void**)ptr, n * sizeof(T)));
    *cap = n;
    return ERAY_OK;
}

uint32_t sat_u32_host(float f) {
    if (!(f > 0.0f)) return 0u;
    if (f >= 4294967296.0f) return 0xffffffffu;
    return (uint32_t)f;
}

bool image_ok(const eray_image& im) { return !im.data || (im.width > 0 && im.height > 0); }
TexView tex(const eray_image& im) { return TexView{im.data, im.width, im.height}; }

int sync_scene(eray_ctx* ctx) {
    int st;
    // The host staging vectors below feed async copies: drain earlier ones before reuse.
    if (ctx->geom_dirty || ctx->desc_dirty) HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (ctx->geom_dirty) {
        uint32_t T = 0;
        for (auto& o : ctx->objects) T += o.T;
        ctx->total_tris = T;
        if ((st = ensure(ctx, &ctx->d_hot, &ctx->tri_cap, T))) return st;
        size_t shade_cap = ctx->tri_cap;
        // shade shares the capacity bookkeeping of hot: (re)allocate alongside
        if (ctx->d_shade) {
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
            HIP_TRY(ctx, hipFree(ctx->d_shade));
            ctx->d_shade = nullptr;
        }
        HIP_TRY(ctx, hipMalloc((void**)&ctx->d_shade, shade_cap * sizeof(TriShade)));
        if (ctx->d_cull) {
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
            HIP_TRY(ctx, hipFree(ctx->d_cull));
            ctx->d_cull = nullptr;
        }
        HIP_TRY(ctx, hipMalloc((void**)&ctx->d_cull, shade_cap * sizeof(TriCull)));
        if (!ctx->d_tcull)  // the general tracer's per-frame culling records (small scenes)
            HIP_TRY(ctx, hipMalloc((void**)&ctx->d_tcull, kTraceSkipTris * sizeof(TriCull)));

        ctx->h_raw.assign((size_t)T * 24, 0.0f);
        size_t off = 0;
        for (auto& o : ctx->objects) {
            std::memcpy(&ctx->h_raw[off * 9], o.raw.data(), sizeof(float) * 9 * o.T);
            std::memcpy(&ctx->h_raw[(size_t)T * 9 + off * 9], o.raw.data() + 9 * (size_t)o.T,
                        sizeof(float) * 9 * o.T);
            std::memcpy(&ctx->h_raw[(size_t)T * 18 + off * 6], o.raw.data() + 18 * (size_t)o.T,
                        sizeof(float) * 6 * o.T);
            off += o.T;
        }
        if ((st = ensure(ctx, &ctx->d_raw, &ctx->raw_cap, (size_t)T * 24))) return st;
        if (T) {
            HIP_TRY(ctx, hipMemcpyAsync(ctx->d_raw, ctx->h_raw.data(), sizeof(float) * 24 * (size_t)T,
                                        hipMemcpyHostToDevice, ctx->stream));
            HIP_TRY(ctx, launch_tri_precompute(ctx->d_raw, ctx->d_raw + 9 * (size_t)T,
                                               ctx->d_raw + 18 * (size_t)T, T, ctx->d_hot,
                                               ctx->d_shade, ctx->stream));
        }
        ctx->geom_dirty = false;
        ctx->desc_dirty = true;
    }
    if (ctx->desc_dirty) {
        ctx->h_objs.clear();
        uint32_t begin = 0;
        ctx->spec_pow = false;
        ctx->example_mat = false;
        // texel programs: per object a header + its outputs' expression trees (48-B records)
        ctx->h_prog.clear();
        std::vector<size_t> prog_at(ctx->objects.size(), SIZE_MAX);
        for (size_t i = 0; i < ctx->objects.size(); ++i) {
            const HostObject& o = ctx->objects[i];
            if (o.tnodes.empty()) continue;
            std::vector<TexelInstr> ins;
            uint32_t head[kTexelHeaderWords] = {};
            for (int out = 0; out < 5; ++out) {
                const int32_t idx = o.tout[out];
                if (idx < 0 || texel_is_color(o.tnodes[idx].kind) != (out == 0)) continue;  // kept / None
                const size_t first = ins.size();
                texel_emit(o.tnodes, (uint32_t)idx, 0, kTexelMod, first, ins);
                if (ins.size() - first > kTexelMaxNodes)
                    return set_error(ctx, ERAY_E_UNSUPPORTED, "object %zu: output %d expands to more than %u texel nodes",
                                     i, out, kTexelMaxNodes);
                head[out] = (uint32_t)first;
                head[5 + out] = (uint32_t)(ins.size() - first);
            }
            prog_at[i] = ctx->h_prog.size();
            ctx->h_prog.insert(ctx->h_prog.end(), head, head + kTexelHeaderWords);
            const uint32_t* w = reinterpret_cast<const uint32_t*>(ins.data());
            ctx->h_prog.insert(ctx->h_prog.end(), w, w + ins.size() * (sizeof(TexelInstr) / 4));
        }
        if (!ctx->h_prog.empty()) {
            if ((st = ensure(ctx, &ctx->d_prog, &ctx->prog_cap, ctx->h_prog.size()))) return st;
            HIP_TRY(ctx, hipMemcpyAsync(ctx->d_prog, ctx->h_prog.data(), 4 * ctx->h_prog.size(), hipMemcpyHostToDevice,
                                        ctx->stream));
        }
        for (size_t i = 0; i < ctx->objects.size(); ++i) {
            const HostObject& o = ctx->objects[i];
            ObjectDesc d{};
            d.g.tri_begin = begin;
            d.g.tri_count = o.T;
            d.g.rect[0] = d.g.rect[2] = 0;  // every pixel until the culling pass computes it
            d.g.rect[1] = d.g.rect[3] = INT32_MAX;
            for (int k = 0; k < 3; ++k) {
                d.g.bb_lo[k] = o.lo[k];
                d.g.bb_hi[k] = o.hi[k];
            }
            d.mat = MaterialDesc{tex(o.mat.color), tex(o.mat.diffuse), tex(o.mat.specular),
                                 tex(o.mat.specular_power), tex(o.mat.reflection)};
            if (o.example) {
                d.mat.color = TexView{nullptr, 0, 0};
                d.mat.diffuse = TexView{nullptr, 0, 0};
                d.mat.example = 1;
                d.mat.ex_w = o.ex.width;
                d.mat.ex_h = o.ex.height;
                d.mat.ex_xf = o.ex.x_fac;
                d.mat.ex_yf = o.ex.y_fac;
                d.mat.ex_r = o.ex.r;
                d.mat.ex_g = o.ex.g;
                d.mat.ex_b = o.ex.b;
                d.mat.ex_factor = o.ex.factor;
            }
            if (prog_at[i] != SIZE_MAX) {  // graph outputs replace the textures (None: defaults)
                d.mat.prog = ctx->d_prog + prog_at[i];
                TexView* tv[5] = {&d.mat.color, &d.mat.diffuse, &d.mat.specular, &d.mat.specular_power,
                                  &d.mat.reflection};
                for (int out = 0; out < 5; ++out)
                    if (o.tout[out] >= 0) *tv[out] = TexView{nullptr, 0, 0};
                ctx->example_mat = true;
                if (o.tout[3] >= 0 && !texel_is_color(o.tnodes[o.tout[3]].kind)) ctx->spec_pow = true;
            }
            ctx->h_objs.push_back(d);
            ctx->spec_pow |= d.mat.specular_power.data != nullptr;
            ctx->example_mat |= d.mat.example != 0;
            begin += o.T;
        }
        ctx->h_lights.clear();
        for (auto& l : ctx->lights) {
            LightDesc d{};
            for (int k = 0; k < 3; ++k) {
                d.pos[k] = l.position[k];
                d.color[k] = l.color[k];
            }
            d.variant = l.variant;
            d.brightness = l.brightness;
            ctx->h_lights.push_back(d);
        }
        if ((st = ensure(ctx, &ctx->d_objs, &ctx->objs_cap, ctx->h_objs.size()))) return st;
        if ((st = ensure(ctx, &ctx->d_lights, &ctx->lights_cap, ctx->h_lights.size()))) return st;
        if (!ctx->h_objs.empty())
            HIP_TRY(ctx, hipMemcpyAsync(ctx->d_objs, ctx->h_objs.data(), sizeof(ObjectDesc) * ctx->h_objs.size(),
                                        hipMemcpyHostToDevice, ctx->stream));
        if (!ctx->h_lights.empty())
            HIP_TRY(ctx, hipMemcpyAsync(ctx->d_lights, ctx->h_lights.data(),
                                        sizeof(LightDesc) * ctx->h_lights.size(), hipMemcpyHostToDevice,
                                        ctx->stream));
        // setup.hip's object ranges and binned-object indices
        const uint32_t nobj = (uint32_t)ctx->objects.size();
        ctx->h_begin.assign(2 * (size_t)nobj + 1, 0u);
        uint32_t nb = 0;
        for (uint32_t i = 0; i < nobj; ++i) {
            ctx->h_begin[i] = ctx->h_objs[i].g.tri_begin;
            ctx->h_begin[nobj + 1 + i] = ctx->objects[i].T > kDirectMax ? nb++ : ~0u;
        }
        ctx->h_begin[nobj] = ctx->total_tris;
        if ((st = ensure(ctx, &ctx->d_begin, &ctx->begin_cap, ctx->h_begin.size()))) return st;
        HIP_TRY(ctx, hipMemcpyAsync(ctx->d_begin, ctx->h_begin.data(), 4 * ctx->h_begin.size(), hipMemcpyHostToDevice,
                                    ctx->stream));
        // rectangle accumulators + the setup's workgroup counter, zero between setups
        const size_t acc_words = 4 * (size_t)nobj + 1 + 10 * (size_t)kSetupMaxBlocks;
        if (ctx->acc_cap < acc_words || !ctx->d_acc) {
            if ((st = ensure(ctx, &ctx->d_acc, &ctx->acc_cap, acc_words))) return st;
            HIP_TRY(ctx, hipMemsetAsync(ctx->d_acc, 0, 4 * ctx->acc_cap, ctx->stream));
        }
        ctx->desc_dirty = false;
        ++ctx->scene_gen;
    }
    return ERAY_OK;
}

uint32_t binned_objects(const eray_ctx* ctx) {
    uint32_t nb = 0;
    for (auto& o : ctx->objects) nb += o.T > kDirectMax;
    return nb;
}

// The device buffers of the binned objects' bins for this camera size, row phase and rows
// (reallocated, with a stream synchronisation, only when that layout or the capacity changes).
// The rendered rows of a call: camera rows [row0, row0 + rows), or rows local rows of
// interleaved bands (eray_render_params::band_rows).
struct RowSpan {
    uint32_t row0, rows, band_shift, band_mask, band_stride;
};
// eray_render_params' band fields as FrameParams encodes them (contiguous: shift 31)
RowSpan row_span(const eray_render_params* rp) {
    if (!rp->band_rows) return RowSpan{rp->row0, rp->rows, 31u, 0x7fffffffu, 0u};
    uint32_t shift = 0;
    while ((1u << shift) < rp->band_rows) ++shift;
    return RowSpan{rp->row0, rp->rows, shift, rp->band_rows - 1u, rp->band_stride};
}

uint64_t fnv1a(const void* data, size_t n, uint64_t h = 1469598103934665603ull) {
    const unsigned char* p = static_cast<const unsigned char*>(data);
    for (size_t i = 0; i < n; ++i) {
        h ^= p[i];
        h *= 1099511628211ull;
    }
    return h;
}

// The source tag of a render of the scene camera over rows rs: a hash of the camera's value, the
// scene generation (uploads since the context was made) and Camera::size — what every rank that
// made the same scene calls computes alike.
FrameSource scene_source(const eray_ctx* ctx, uint32_t W, uint32_t H, const RowSpan& rs) {
    FrameSource s;
    s.kind = kSrcScene;
    uint64_t h = fnv1a(&ctx->camera, sizeof ctx->camera);
    h = fnv1a(&ctx->scene_gen, sizeof ctx->scene_gen, h);
    const uint32_t wh[2] = {W, H};
    s.key = fnv1a(wh, sizeof wh, h);
    s.W = W;
    s.H = H;
    s.row0 = rs.row0;
    s.rows = rs.rows;
    s.band_shift = rs.band_shift;
    s.band_stride = rs.band_stride;
    return s;
}

// A tagged slot's PPM bytes: [ppm, ppm + rows * W * 3).
uintptr_t tag_end(const eray_ctx::SlotTag& t) { return t.ppm + (uintptr_t)t.src.rows * t.src.W * 3u; }
// Forgets the source of every tagged slot whose bytes meet [a, a + bytes): memory written (or
// freed) by anything but a render of that source no longer holds its frame.
void untag_range(eray_ctx* ctx, uintptr_t a, size_t bytes) {
    if (!bytes) return;
    auto& v = ctx->slot_tags;
    v.erase(std::remove_if(v.begin(), v.end(),
                           [&](const eray_ctx::SlotTag& t) { return t.ppm < a + bytes && a < std::max(tag_end(t), t.ppm + 1); }),
            v.end());
}
// Records `s` as the source of the n PPM slots ppm + k * stride (k < n); any other tag whose
// bytes the new frames overwrite is dropped.
void tag_frames(eray_ctx* ctx, const uint8_t* ppm, uint64_t stride, uint32_t n, const FrameSource& s) {
    if (!ppm) return;
    if (s.kind == kSrcScene || s.kind == kSrcPath) ctx->gather_src = s;
    auto& v = ctx->slot_tags;
    for (uint32_t k = 0; k < n; ++k) {
        const uintptr_t a = reinterpret_cast<uintptr_t>(ppm) + (uintptr_t)(k * stride);
        untag_range(ctx, a, std::max<size_t>((size_t)s.rows * s.W * 3u, 1));
        if (v.size() >= kMaxTags) v.erase(v.begin());
        v.push_back({a, s});
    }
}

// The binned objects' first triangles and object indices (bins_alloc's key tables).
void binned_lists(const eray_ctx* ctx, std::vector<uint32_t>* kbegin, std::vector<uint32_t>* kobj) {
    for (uint32_t i = 0; i < ctx->objects.size(); ++i)
        if (ctx->objects[i].T > kDirectMax) {
            kbegin->push_back(ctx->h_objs[i].g.tri_begin);
            kobj->push_back(i);
        }
}

int ensure_bins(eray_ctx* ctx, uint32_t W, uint32_t H, const RowSpan& rs) {
    const uint32_t row0 = rs.row0, rows = rs.rows;
    const uint32_t nb = binned_objects(ctx);
    const uint32_t T = ctx->total_tris;
    if (ctx->face_cap < T || !ctx->d_range) {
        int st;
        if ((st = ensure(ctx, &ctx->d_range, &ctx->face_cap, T))) return st;
        size_t c1 = 0, c2 = 0;
        if ((st = ensure(ctx, &ctx->d_area, &c1, T)) || (st = ensure(ctx, &ctx->d_fkey, &c2, T))) return st;
    }
    size_t binned_tris = 0;
    for (auto& o : ctx->objects)
        if (o.T > kDirectMax) binned_tris += o.T;
    if (!ctx->bin_cap) ctx->bin_cap = std::min(std::max<size_t>(2 * binned_tris, 1u << 16), kMaxBinEntries);
    const uint32_t phase = row0 % kBinH, tiles_x = (W + 63) / 64;
    std::vector<uint64_t> layout{T, nb, W, H, phase, rows, ctx->bin_cap, ctx->scene_gen};
    if (layout == ctx->bins_layout) return ERAY_OK;
    std::vector<uint32_t> kbegin, kobj;
    binned_lists(ctx, &kbegin, &kobj);
    HIP_TRY(ctx, bins_alloc(ctx->bins, T, nb, kbegin.data(), kobj.data(), W, H, phase, tiles_x, rows, ctx->bin_cap,
                            ctx->stream));
    ctx->bins_layout = std::move(layout);
    ++ctx->bins_gen;         // graphs that captured the old buffers must not be replayed
    ctx->setup_key.clear();  // the bins must be rebuilt
    return ERAY_OK;
}

// Enqueues the per-camera setup of `d_camera` (device) for camera rows [row0, row0 + rows): no
// host round trip (setup.hip, bins.hip).
SetupParams setup_params(eray_ctx* ctx, const CamDev* d_camera, uint32_t W, uint32_t H, const RowSpan& rs) {
    SetupParams sp{};
    sp.hot = ctx->d_hot;
    sp.cull = ctx->d_cull;
    sp.T = ctx->total_tris;
    sp.objs = ctx->d_objs;
    sp.nobj = (uint32_t)ctx->objects.size();
    sp.obj_begin = ctx->d_begin;
    sp.objkey = ctx->d_begin + sp.nobj + 1;
    sp.cam = d_camera;
    sp.state = ctx->d_state;
    sp.W = W;
    sp.H = H;
    sp.row0 = rs.row0;
    sp.rows = rs.rows;
    sp.band_shift = rs.band_shift;
    sp.band_mask = rs.band_mask;
    sp.band_stride = rs.band_stride;
    // [done counter | kSetupMaxBlocks x 10 partials | 4 x nobj accumulators]: the counter and the
    // accumulators are zero between setups whatever the object count (partials are rewritten)
    sp.done = ctx->d_acc;
    sp.part = ctx->d_acc + 1;
    sp.acc = ctx->d_acc + 1 + 10 * (size_t)kSetupMaxBlocks;
    const bool binned = binned_objects(ctx) > 0;
    sp.binned = binned ? 1u : 0u;
    sp.rect_pairs = ctx->rect_pairs ? 1u : 0u;
    if (binned) {
        sp.range = ctx->d_range;
        sp.area = ctx->d_area;
        sp.fkey = ctx->d_fkey;
        sp.bins_x = ctx->bins.bins_x;
        sp.phase = ctx->bins.phase;
        sp.first_local = ctx->bins.first;
        sp.boff = ctx->bins.boff;
    }
    return sp;
}

// ordered: the detail list in raster order (one-camera setups, whose list serves many frames);
// camera paths append it in one launch instead (bins.hip detail_list_kernel)
// keep_all: the general tracer's bins (SetupParams::keep_all)
int enqueue_setup(eray_ctx* ctx, const CamDev* d_camera, uint32_t W, uint32_t H, const RowSpan& rs, bool ordered,
                  bool keep_all = false, int32_t* path_union = nullptr) {
    SetupParams sp = setup_params(ctx, d_camera, W, H, rs);
    sp.keep_all = keep_all ? 1u : 0u;
    sp.path_union = path_union;
    sp.union_nobj = sp.nobj;
    HIP_TRY(ctx, launch_camera_setup(sp, ctx->stream));
    if (sp.binned) HIP_TRY(ctx, launch_bins_build(sp, ctx->bins, (W + 63) / 64, ordered, ctx->stream));
    return ERAY_OK;
}

// The multi-camera setup buffers (camera paths of scenes with binned objects) for the current
// bins layout (ensure_bins ran first): two sets of mc_k copies of every per-camera array, camera
// k's descriptors initialised with the scene's; reallocated when the layout or the scene changes
// (mc_gen keys the captured path graphs).
int ensure_multi(eray_ctx* ctx, uint32_t W, uint32_t H, const RowSpan& rs) {
    // cameras per build: the chain's kernels are latency bound at tens of thousands of faces (16
    // cameras share one chain), work bound at millions (fewer: the buffers grow with K x faces)
    const uint32_t K = std::max(1u, std::min(16u, (1u << 22) / std::max(ctx->total_tris, 1u)));
    std::vector<uint64_t> layout = ctx->bins_layout;
    layout.push_back(ctx->scene_gen);
    if (layout == ctx->mc_layout) return ERAY_OK;
    if (!ctx->mc_stream) {
        // (a priority of its own: HIP deals its hardware queues to streams round-robin per priority,
        // and on the frames' queue the setup chain serialised with them — moving C5 frame 416 ->
        // 375 us, 3840x2160 / 70k 60.6 -> 55.7 us, profiles/r04/ab/ab_r04m.txt)
        HIP_TRY(ctx, hipStreamCreateWithPriority(&ctx->mc_stream, hipStreamNonBlocking, -1));
        for (hipEvent_t* ev : {&ctx->mc_fork, &ctx->mc_ready[0], &ctx->mc_ready[1], &ctx->mc_free[0], &ctx->mc_free[1]})
            HIP_TRY(ctx, hipEventCreateWithFlags(ev, hipEventDisableTiming));
    }
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->mc_stream));
    ctx->mc_layout.clear();
    const uint32_t T = ctx->total_tris, nobj = (uint32_t)ctx->objects.size(), nb = binned_objects(ctx);
    const size_t t = (size_t)K * (T ? T : 1);
    const size_t acc_words = 4 * (size_t)K * nobj + 1 + 10 * (size_t)kSetupMaxBlocks;
    // camera k's copy of binned object j: key k * nb + j, its faces from k * T + tri_begin
    std::vector<uint32_t> kbegin, kobj, mbegin, mobj;
    binned_lists(ctx, &kbegin, &kobj);
    for (uint32_t k = 0; k < K; ++k)
        for (uint32_t j = 0; j < nb; ++j) {
            mbegin.push_back(k * T + kbegin[j]);
            mobj.push_back(k * nobj + kobj[j]);
        }
    for (auto& m : ctx->mc) {
        for (void* b : {(void*)m.cull, (void*)m.objs, (void*)m.state, (void*)m.acc, (void*)m.range, (void*)m.area,
                        (void*)m.fkey})
            if (b) HIP_TRY(ctx, hipFree(b));
        m.cull = nullptr;
        m.objs = nullptr;
        m.state = nullptr;
        m.acc = nullptr;
        m.range = nullptr;
        m.area = nullptr;
        m.fkey = nullptr;
        HIP_TRY(ctx, hipMalloc((void**)&m.cull, sizeof(TriCull) * t));
        HIP_TRY(ctx, hipMalloc((void**)&m.objs, sizeof(ObjectDesc) * K * (nobj ? nobj : 1)));
        HIP_TRY(ctx, hipMalloc((void**)&m.state, sizeof(CamState) * K));
        HIP_TRY(ctx, hipMalloc((void**)&m.acc, 4 * acc_words));
        HIP_TRY(ctx, hipMalloc((void**)&m.range, sizeof(int4) * t));
        HIP_TRY(ctx, hipMalloc((void**)&m.area, sizeof(unsigned long long) * t));
        HIP_TRY(ctx, hipMalloc((void**)&m.fkey, sizeof(uint32_t) * t));
        HIP_TRY(ctx, hipMemsetAsync(m.acc, 0, 4 * acc_words, ctx->stream));
        HIP_TRY(ctx, hipMemsetAsync(m.state, 0, sizeof(CamState) * K, ctx->stream));
        for (uint32_t k = 0; k < K && nobj; ++k)  // (each setup rewrites the rectangles and bin views)
            HIP_TRY(ctx, hipMemcpyAsync(m.objs + (size_t)k * nobj, ctx->d_objs, sizeof(ObjectDesc) * nobj,
                                        hipMemcpyDeviceToDevice, ctx->stream));
        HIP_TRY(ctx, bins_alloc(m.bins, K * T, K * nb, mbegin.data(), mobj.data(), W, H, rs.row0 % kBinH, (W + 63) / 64,
                                rs.rows, std::min((size_t)K * ctx->bin_cap, kMaxBinEntries), ctx->stream, K));
    }
    ctx->mc_layout = std::move(layout);
    ctx->mc_k = K;
    ++ctx->mc_gen;
    return ERAY_OK;
}

// Enqueues on `s` the setups of the `ncam` cameras at d_cams (ncam <= mc_k) into buffer set `m`:
// camera k's culling records at m.cull + k T, descriptors at m.objs + k nobj, state m.state + k,
// detail list m.bins.dlist + k nsub (occupancy m.bins.docc + k nsub / 4).
int enqueue_multi_setup(eray_ctx* ctx, eray_ctx::MultiSet& m, const CamDev* d_cams, uint32_t ncam, uint32_t W,
                        uint32_t H, const RowSpan& rs, hipStream_t s, int32_t* path_union = nullptr) {
    const uint32_t T = ctx->total_tris, nobj = (uint32_t)ctx->objects.size();
    SetupParams sp = setup_params(ctx, d_cams, W, H, rs);
    sp.ncam = ncam;
    sp.T1 = T;
    sp.nobj1 = nobj;
    sp.nb1 = binned_objects(ctx);
    sp.T = ncam * T;
    sp.nobj = ncam * nobj;
    sp.cull = m.cull;
    sp.objs = m.objs;
    sp.state = m.state;
    sp.done = m.acc;
    sp.part = m.acc + 1;
    sp.acc = m.acc + 1 + 10 * (size_t)kSetupMaxBlocks;
    sp.range = m.range;
    sp.area = m.area;
    sp.fkey = m.fkey;
    sp.bins_x = m.bins.bins_x;
    sp.phase = m.bins.phase;
    sp.first_local = m.bins.first;
    sp.boff = m.bins.boff;
    sp.path_union = path_union;
    sp.union_nobj = nobj;
    HIP_TRY(ctx, launch_camera_setup(sp, s));
    HIP_TRY(ctx, launch_bins_build(sp, m.bins, (W + 63) / 64, false, s));
    return ERAY_OK;
}

// Camera paths of scenes without binned objects set up a whole graph chunk's cameras in one
// launch (one workgroup per camera, into per-camera slots) instead of one setup per frame: the
// setup of a small scene is one workgroup's latency chain (culling records, the double-precision
// clip of face_rect, the rectangle merge), which as its own launch per frame cost about as much
// as the frame.  Up to kBatchTris triangles (the slots hold kGraphFrames x T culling records).
constexpr uint32_t kBatchTris = 16384;
bool batch_setup_ok(const eray_ctx* ctx) {
    return !binned_objects(ctx) && ctx->objects.size() <= kSetupBatchMaxObjects && ctx->total_tris <= kBatchTris;
}

CamDev cam_dev(const eray_camera& c) {
    return CamDev{c.center[0], c.center[1], c.center[2], c.fov[0] / c.fov[1], c.z_dist, {0u, 0u, 0u}};
}

// A copy of the setup state has reached the host (h_state): grow the bins' capacity when some
// setup since the last reallocation needed more entries (they then fell back to LDS tiles).
void state_arrived(eray_ctx* ctx) {
    ctx->state_pending = false;
    ctx->state_known = true;
    if (ctx->h_state->bin_entries > ctx->bin_cap && ctx->bin_cap < kMaxBinEntries) {
        // (at most kMaxBinEntries: beyond, the setups keep overflowing into the exact LDS-tile scan)
        ctx->bin_cap = std::min(2 * (size_t)ctx->h_state->bin_entries, kMaxBinEntries);
        ctx->state_known = false;
        ctx->setup_key.clear();  // rebuilt with the larger capacity
    }
}

// Makes the per-camera setup of the context camera current for rows [row0, row0 + rows):
// enqueued when the camera, the rows or the scene changed, its results copied to the host
// asynchronously.  *known: the host has them (args-mode frames); `wait`: block until it does.
// trace_bins: the general tracer's setup (every pair of each face's bin rectangle binned).
int sync_setup(eray_ctx* ctx, uint32_t W, uint32_t H, const RowSpan& rs, bool wait, bool* known,
               bool trace_bins = false) {
    for (int attempt = 0; attempt < 3; ++attempt) {
        if (ctx->state_pending) {
            const hipError_t q = hipEventQuery(ctx->state_ev);
            if (q == hipSuccess) state_arrived(ctx);
            else if (q != hipErrorNotReady) return set_error(ctx, ERAY_E_HIP, "setup event: %s", hipGetErrorString(q));
        }
        auto bins_ready = [&]() -> int {
            if (!binned_objects(ctx)) return ERAY_OK;
            const std::vector<uint64_t> before = ctx->bins_layout;
            if (int st = ensure_bins(ctx, W, H, rs)) return st;
            if (ctx->bins_layout != before)  // new buffers: the bin statistics start over
                HIP_TRY(ctx, hipMemsetAsync(ctx->d_state, 0, sizeof(CamState), ctx->stream));
            return ERAY_OK;
        };
        if (int st = bins_ready()) return st;
        std::vector<uint64_t> key(sizeof(eray_camera) / 4 + 5);
        std::memcpy(key.data(), &ctx->camera, sizeof(eray_camera));
        key[key.size() - 5] = trace_bins ? 1u : 0u;
        key[key.size() - 4] = ((uint64_t)rs.row0 << 32) | rs.band_shift;
        key[key.size() - 3] = ((uint64_t)rs.rows << 32) | rs.band_stride;
        key[key.size() - 2] = ctx->scene_gen;
        key[key.size() - 1] = ((uint64_t)W << 32) | H;
        if (key != ctx->setup_key) {
            if (ctx->state_pending) {  // h_state is about to be rewritten
                HIP_TRY(ctx, hipEventSynchronize(ctx->state_ev));
                state_arrived(ctx);
                if (int st = bins_ready()) return st;  // (a grown capacity)
            }
            HIP_TRY(ctx, launch_set_camera(cam_dev(ctx->camera), ctx->d_cam, ctx->stream));
            if (int st = enqueue_setup(ctx, ctx->d_cam, W, H, rs, true, trace_bins)) return st;
            HIP_TRY(ctx, hipMemcpyAsync(ctx->h_state, ctx->d_state, sizeof(CamState), hipMemcpyDeviceToHost,
                                        ctx->stream));
            // the objects' pixel rectangles of this camera (eray_gather_frames' transfer layout);
            // no copy into the pinned buffer is in flight here (state_pending was drained above)
            const size_t nobj = ctx->objects.size();
            if (ctx->h_objs_state_cap < nobj) {
                if (ctx->h_objs_state) HIP_TRY(ctx, hipHostFree(ctx->h_objs_state));
                ctx->h_objs_state = nullptr;
                ctx->h_objs_state_cap = 0;
                HIP_TRY(ctx, hipHostMalloc((void**)&ctx->h_objs_state, sizeof(ObjectDesc) * nobj, hipHostMallocDefault));
                ctx->h_objs_state_cap = nobj;
            }
            if (nobj)
                HIP_TRY(ctx, hipMemcpyAsync(ctx->h_objs_state, ctx->d_objs, sizeof(ObjectDesc) * nobj,
                                            hipMemcpyDeviceToHost, ctx->stream));
            ctx->setup_src = scene_source(ctx, W, H, rs);
            HIP_TRY(ctx, hipEventRecord(ctx->state_ev, ctx->stream));
            ctx->setup_key = std::move(key);
            ctx->state_pending = true;
            ctx->state_known = false;
        }
        if (ctx->state_pending && wait) {
            HIP_TRY(ctx, hipEventSynchronize(ctx->state_ev));
            state_arrived(ctx);  // (may ask for a larger capacity: set up again)
        }
        if (ctx->state_known || !wait) break;
    }
    *known = ctx->state_known;
    return ERAY_OK;
}

}  // namespace

extern "C" {

int eray_abi_version(void) { return ERAY_ABI_VERSION; }

int eray_ctx_create(int device, eray_ctx** out) {
    if (!out) return set_error(nullptr, ERAY_E_INVALID_ARGUMENT, "out is null");
    *out = nullptr;
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count == 0)
        return set_error(nullptr, ERAY_E_HIP, "no HIP device available (%s)",
                         e == hipSuccess ? "0 devices" : hipGetErrorString(e));
    if (device < 0 || device >= count)
        return set_error(nullptr, ERAY_E_INVALID_ARGUMENT, "device %d out of range (%d devices)", device, count);
    eray_ctx* ctx = new (std::nothrow) eray_ctx();
    if (!ctx) return set_error(nullptr, ERAY_E_OUT_OF_MEMORY, "context allocation failed");
    ctx->device = device;
    e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking);
    // the separate fill kernel's stream and fork / join events (render.hip launch_frame_kernel);
    // low priority, so that it never shares a hardware queue with a caller's normal-priority
    // stream (the fill would then wait for the frame kernel it runs beside)
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&ctx->lc.side, hipStreamNonBlocking, 1);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->lc.fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->lc.join, hipEventDisableTiming);
    // the per-camera setup's device state and its pinned host copy
    if (e == hipSuccess) e = hipMalloc((void**)&ctx->d_cam, sizeof(CamDev));
    if (e == hipSuccess) e = hipMalloc((void**)&ctx->d_state, sizeof(CamState));
    if (e == hipSuccess) e = hipMemset(ctx->d_state, 0, sizeof(CamState));
    if (e == hipSuccess) e = hipMalloc((void**)&ctx->d_coll, kCollScratchBytes);

    if (e == hipSuccess) e = hipHostMalloc((void**)&ctx->h_state, sizeof(CamState), hipHostMallocDefault);
    if (e == hipSuccess) std::memset(ctx->h_state, 0, sizeof(CamState));
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->state_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->path_ev[0], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->path_ev[1], hipEventDisableTiming);
    if (e != hipSuccess) {
        ctx->stream = ctx->own_stream;
        eray_ctx_destroy(ctx);
        return set_error(nullptr, ERAY_E_HIP, "context init: %s", hipGetErrorString(e));
    }
    ctx->stream = ctx->own_stream;
    *out = ctx;
    return ERAY_OK;
}

int eray_ctx_destroy(eray_ctx* ctx) {
    if (!ctx) return ERAY_OK;
    hipSetDevice(ctx->device);
    if (ctx->stream) hipStreamSynchronize(ctx->stream);
    if (ctx->own_stream) hipStreamSynchronize(ctx->own_stream);
    bins_free(ctx->bins);
    if (ctx->mc_stream) hipStreamSynchronize(ctx->mc_stream);
    for (auto& m : ctx->mc) {
        bins_free(m.bins);
        for (void* b : {(void*)m.cull, (void*)m.objs, (void*)m.state, (void*)m.acc, (void*)m.range, (void*)m.area,
                        (void*)m.fkey})
            if (b) hipFree(b);
    }
    for (hipEvent_t ev : {ctx->mc_fork, ctx->mc_ready[0], ctx->mc_ready[1], ctx->mc_free[0], ctx->mc_free[1]})
        if (ev) hipEventDestroy(ev);
    if (ctx->mc_stream) hipStreamDestroy(ctx->mc_stream);
    void* bufs[] = {ctx->d_hot,   ctx->d_shade, ctx->d_cull,  ctx->d_raw,  ctx->d_objs,  ctx->d_lights,
                    ctx->d_prog,  ctx->d_cam,   ctx->d_state, ctx->d_acc,  ctx->d_begin, ctx->d_range,
                    ctx->d_area,  ctx->d_fkey,  ctx->d_path,  ctx->d_path_all, ctx->d_staging,
                    ctx->d_bcull, ctx->d_bobjs, ctx->d_bstate, ctx->d_tcull, ctx->d_union_acc, ctx->d_coll};
    for (void* b : bufs)
        if (b) hipFree(b);
    if (ctx->h_state) hipHostFree(ctx->h_state);
    for (CamDev* h : ctx->h_path)
        if (h) hipHostFree(h);
    if (ctx->h_objs_state) hipHostFree(ctx->h_objs_state);
    if (ctx->h_union) hipHostFree(ctx->h_union);
    for (hipEvent_t ev : ctx->union_ev)
        if (ev) hipEventDestroy(ev);
    if (ctx->gather_plan && ctx->gather_plan_free) ctx->gather_plan_free(ctx->gather_plan);
    for (auto& g : ctx->graphs) {
        if (g.exec) hipGraphExecDestroy(g.exec);
        if (g.graph) hipGraphDestroy(g.graph);
    }
    for (hipEvent_t ev : {ctx->state_ev, ctx->path_ev[0], ctx->path_ev[1], ctx->lc.fork, ctx->lc.join})
        if (ev) hipEventDestroy(ev);
    if (ctx->lc.side) hipStreamDestroy(ctx->lc.side);
    if (ctx->own_stream) hipStreamDestroy(ctx->own_stream);
    delete ctx;
    return ERAY_OK;
}

const char* eray_last_error(const eray_ctx* ctx) {
    return ctx ? ctx->err.c_str() : g_thread_error.c_str();
}

int eray_set_stream(eray_ctx* ctx, void* stream) {
    if (int st = use_device(ctx)) return st;
    ctx->stream = (hipStream_t)stream;
    return ERAY_OK;
}

void* eray_get_stream(eray_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int eray_synchronize(eray_ctx* ctx) {
    if (int st = use_device(ctx)) return st;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return ERAY_OK;
}

int eray_device_alloc(eray_ctx* ctx, size_t bytes, void** dev_ptr) {
    if (int st = use_device(ctx)) return st;
    if (!dev_ptr) return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "dev_ptr is null");
    HIP_TRY(ctx, hipMalloc(dev_ptr, bytes ? bytes : 1));
    return ERAY_OK;
}

int eray_device_free(eray_ctx* ctx, void* dev_ptr) {
    if (int st = use_device(ctx)) return st;
    if (!dev_ptr) return ERAY_OK;
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, dev_ptr) == hipSuccess)  // (frames in it lose their source)
        untag_range(ctx, reinterpret_cast<uintptr_t>(base), size);
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    HIP_TRY(ctx, hipFree(dev_ptr));
    return ERAY_OK;
}

int eray_memset(eray_ctx* ctx, void* dev_ptr, int value, size_t bytes) {
    if (int st = use_device(ctx)) return st;
    if (!bytes) return ERAY_OK;
    if (!dev_ptr) return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "dev_ptr is null");
    untag_range(ctx, reinterpret_cast<uintptr_t>(dev_ptr), bytes);
    HIP_TRY(ctx, hipMemsetAsync(dev_ptr, value, bytes, ctx->stream));
    return ERAY_OK;
}

int eray_copy_to_device(eray_ctx* ctx, void* dst, const void* src, size_t bytes) {
    if (int st = use_device(ctx)) return st;
    if (!bytes) return ERAY_OK;
    if (!dst || !src) return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "null pointer");
    untag_range(ctx, reinterpret_cast<uintptr_t>(dst), bytes);
    HIP_TRY(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return ERAY_OK;
}

int eray_copy_to_host(eray_ctx* ctx, void* dst, const void* src, size_t bytes) {
    if (int st = use_device(ctx)) return st;
    if (!bytes) return ERAY_OK;
    if (!dst || !src) return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "null pointer");
    HIP_TRY(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return ERAY_OK;
}

// ------------------------------------------------------------------------ shaderlib ---------
int eray_node_wave(eray_ctx* ctx, uint32_t w, uint32_t h, float x_fac, float y_fac, float* out) {
    if (int st = use_device(ctx)) return st;
    if ((size_t)w * h && !out) return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "wave: out is null");
    HIP_TRY(ctx, launch_wave(w, h, x_fac, y_fac, out, ctx->stream));
    return ERAY_OK;
}

int eray_node_rgb(eray_ctx* ctx, uint32_t w, uint32_t h, eray_image r, eray_image g, eray_image b,
                  float* out) {
    if (int st = use_device(ctx)) return st;
    const size_t n = (size_t)w * h;
    const eray_image* in[3] = {&r, &g, &b};
    const char* names[3] = {"red", "green", "blue"};
    for (int k = 0; k < 3; ++k) {
        if (!in[k]->data)
            return set_error(ctx, ERAY_E_MISSING, "rgb: missing input `%s`", names[k]);
        if ((size_t)in[k]->width * in[k]->height < n)
            return set_error(ctx, ERAY_E_OUT_OF_BOUNDS,
                             "rgb: input `%s` has %zu pixels, the %ux%u output indexes %zu",
                             names[k], (size_t)in[k]->width * in[k]->height, w, h, n);
    }
    if (n && !out) return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "rgb: out is null");
    HIP_TRY(ctx, launch_rgb(w, h, r.data, g.data, b.data, out, ctx->stream));
    return ERAY_OK;
}

int eray_node_flat_color(eray_ctx* ctx, uint32_t w, uint32_t h, float r, float g, float b,
                         float* out) {
    if (int st = use_device(ctx)) return st;
    if ((size_t)w * h && !out) return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "flat_color: out is null");
    HIP_TRY(ctx, launch_flat(w, h, r, g, b, out, ctx->stream));
    return ERAY_OK;
}

int eray_node_mix_color(eray_ctx* ctx, uint32_t w, uint32_t h, eray_image left, eray_image right,
                        float factor, float* out) {
    if (int st = use_device(ctx)) return st;
    if (!left.data) return set_error(ctx, ERAY_E_MISSING, "mix_color: missing input `left`");
    if (!right.data) return set_error(ctx, ERAY_E_MISSING, "mix_color: missing input `right`");
    const size_t n = (size_t)w * h;
    if (n && (!left.width || !left.height || !right.width || !right.height))
        return set_error(ctx, ERAY_E_OUT_OF_BOUNDS, "mix_color: empty input image (mod_get by 0)");
    if (n && !out) return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "mix_color: out is null");
    HIP_TRY(ctx, launch_mix(w, h, tex(left), tex(right), factor, out, ctx->stream));
    return ERAY_OK;
}

int eray_material_example(eray_ctx* ctx, uint32_t w, uint32_t h, float x_fac, float y_fac, float r,
                          float g, float b, float factor, float* out_color, float* out_diffuse) {
    if (int st = use_device(ctx)) return st;
    HIP_TRY(ctx, launch_material_example(w, h, x_fac, y_fac, r, g, b, factor, out_color, out_diffuse,
                                         ctx->stream));
    return ERAY_OK;
}

// ------------------------------------------------------------------------ scene -------------
int eray_scene_reset(eray_ctx* ctx) {
    if (!ctx) return set_error(nullptr, ERAY_E_INVALID_ARGUMENT, "null context");
    ctx->objects.clear();
    ctx->lights.clear();
    ctx->camera = eray_camera{{0.0f, 0.0f, 0.0f}, {60.0f, 60.0f}, 1024u, 1.0f};
    ctx->geom_dirty = ctx->desc_dirty = true;
    return ERAY_OK;
}

int eray_scene_set_camera(eray_ctx* ctx, const eray_camera* camera) {
    if (!ctx || !camera) return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "null argument");
    if (std::memcmp(&ctx->camera, camera, sizeof(eray_camera)) != 0) {
        ctx->camera = *camera;  // (the next culled render sets it up: sync_setup)
    }
    return ERAY_OK;
}

int eray_scene_add_light(eray_ctx* ctx, const eray_light* light) {
    if (!ctx || !light) return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "null argument");
    if (light->variant != ERAY_LIGHT_POINT && light->variant != ERAY_LIGHT_AMBIENT)
        return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "unknown light variant %d", light->variant);
    ctx->lights.push_back(*light);
    ctx->desc_dirty = true;
    return ERAY_OK;
}

int eray_scene_set_object_example_material(eray_ctx* ctx, uint32_t index, const eray_material_example_params* m) {
    if (!ctx || !m) return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "null argument");
    if (index >= ctx->objects.size())
        return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "object %u out of range (%zu objects)", index,
                         ctx->objects.size());
    if (!m->width || !m->height)  // Image::mod_get by 0 panics (image.rs:36-38)
        return set_error(ctx, ERAY_E_OUT_OF_BOUNDS, "example material of zero width or height");
    ctx->objects[index].example = true;
    ctx->objects[index].ex = *m;
    ctx->desc_dirty = true;
    return ERAY_OK;
}

int eray_scene_set_object_texel_graph(eray_ctx* ctx, uint32_t index, const eray_texel_graph* g) {
    if (!ctx) return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "null context");
    if (index >= ctx->objects.size())
        return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "object %u out of range (%zu objects)", index,
                         ctx->objects.size());
    HostObject& o = ctx->objects[index];
    if (!g) {
        o.tnodes.clear();
        std::fill(o.tout, o.tout + 5, -1);
        ctx->desc_dirty = true;
        return ERAY_OK;
    }
    if (g->count && !g->nodes) return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "nodes is null");
    for (uint32_t i = 0; i < g->count; ++i) {
        const eray_texel_node& n = g->nodes[i];
        if (n.kind > ERAY_TEXEL_MIX_COLOR) return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "node %u: kind %u", i, n.kind);
        // every image a Material::get lookup can reach is indexed by mod_get or by pixel index:
        // a zero-sized one panics there (image.rs:36-38)
        if (!n.width || !n.height)
            return set_error(ctx, ERAY_E_OUT_OF_BOUNDS, "node %u: zero width or height", i);
        const int inputs = n.kind == ERAY_TEXEL_RGB ? 3 : n.kind == ERAY_TEXEL_MIX_COLOR ? 2 : 0;
        for (int j = 0; j < inputs; ++j) {
            const int32_t in = n.input[j];
            if (in < 0 || (uint32_t)in >= i)  // unconnected (MissingMany) or not an earlier node
                return set_error(ctx, ERAY_E_MISSING_MANY, "node %u: input %d is not an earlier node", i, j);
            const eray_texel_node& src = g->nodes[in];
            // rgb takes IValue images, mix_color IColor ones (get_sv!, shader.rs:140-178)
            if (texel_is_color(src.kind) != (n.kind == ERAY_TEXEL_MIX_COLOR))
                return set_error(ctx, ERAY_E_INVALID_TYPE, "node %u: input %d has the wrong image type", i, j);
            // rgb reads pixels[y * width + x] of each input (rgb.rs:89-95): it panics past the end
            if (n.kind == ERAY_TEXEL_RGB && (uint64_t)src.width * src.height < (uint64_t)n.width * n.height)
                return set_error(ctx, ERAY_E_OUT_OF_BOUNDS, "node %u: input %d has fewer pixels than the node", i, j);
        }
    }
    const int32_t outs[5] = {g->color, g->diffuse, g->specular, g->specular_power, g->reflection};
    for (int k = 0; k < 5; ++k)
        if (outs[k] < -1 || outs[k] >= (int32_t)g->count)
            return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "output %d: node %d out of range", k, outs[k]);
    o.tnodes.assign(g->nodes, g->nodes + g->count);
    std::copy(outs, outs + 5, o.tout);
    ctx->desc_dirty = true;
    return ERAY_OK;
}

int eray_scene_add_object(eray_ctx* ctx, const eray_object* obj, uint32_t* index) {
    if (!ctx || !obj) return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "null argument");
    const uint32_t T = obj->triangle_count;
    if (T && (!obj->positions || !obj->normals || !obj->uvs))
        return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "object arrays are null");
    const eray_material& m = obj->material;
    if (!image_ok(m.color) || !image_ok(m.diffuse) || !image_ok(m.specular) ||
        !image_ok(m.specular_power) || !image_ok(m.reflection))
        return set_error(ctx, ERAY_E_OUT_OF_BOUNDS, "material image with zero width or height (mod_get by 0)");
    uint64_t total = T;
    for (auto& o : ctx->objects) total += o.T;
    if (total > kMaxSceneTris)
        return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "too many triangles: %llu in the scene (at most %llu)",
                         (unsigned long long)total, (unsigned long long)kMaxSceneTris);
    HostObject h;
    h.T = T;
    h.raw.resize((size_t)T * 24);
    if (T) {
        std::memcpy(h.raw.data(), obj->positions, sizeof(float) * 9 * (size_t)T);
        std::memcpy(h.raw.data() + 9 * (size_t)T, obj->normals, sizeof(float) * 9 * (size_t)T);
        std::memcpy(h.raw.data() + 18 * (size_t)T, obj->uvs, sizeof(float) * 6 * (size_t)T);
    }
    for (int k = 0; k < 3; ++k) {
        h.lo[k] = obj->bbox_min[k];
        h.hi[k] = obj->bbox_max[k];
    }
    h.mat = m;
    ctx->objects.push_back(std::move(h));
    if (index) *index = (uint32_t)(ctx->objects.size() - 1);
    ctx->geom_dirty = ctx->desc_dirty = true;
    return ERAY_OK;
}

int eray_camera_size(const eray_camera* c, uint32_t* w, uint32_t* h) {
    if (!c || !w || !h) return set_error(nullptr, ERAY_E_INVALID_ARGUMENT, "null argument");
    *w = c->width;
    *h = sat_u32_host((float)c->width / (c->fov[0] / c->fov[1]));
    return ERAY_OK;
}

// ------------------------------------------------------------------------ render ------------
namespace {
enum class SetupWait { kNo, kYes };
// Frame parameters of a render call.  Culled frames need the camera's setup: when its results
// are on the host (or `wait`), the detail rectangles / count travel in the kernel arguments
// (args mode); otherwise the frame kernel reads them from the setup's CamState (device-camera
// mode) and the call never waits for the setup.
int prepare_render(eray_ctx* ctx, const eray_render_params* rp, FrameParams* out, bool* empty,
                   SetupWait wait = SetupWait::kNo) {
    if (int st = use_device(ctx)) return st;
    if (!rp) return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "params is null");
    // anti-aliasing and reflection bounces take the general tracer (trace.hip); bounces only
    // matter when some material has a reflection output (engine.rs:181-182)
    bool reflective = false;
    for (auto& o : ctx->objects) {
        const int32_t r = o.tout[4];  // a graph output replaces the texture (None if mistyped)
        reflective |= r >= 0 ? !texel_is_color(o.tnodes[r].kind) : o.mat.reflection.data != nullptr;
    }
    const uint32_t bounces = reflective ? rp->bounces : 0u;
    if (bounces > kMaxBounces)
        return set_error(ctx, ERAY_E_UNSUPPORTED, "bounces = %u: at most %u reflection levels", rp->bounces,
                         kMaxBounces);
    const uint32_t known_flags = ERAY_RENDER_BRUTE_FORCE | ERAY_RENDER_DENSE_DETAIL | ERAY_RENDER_NO_DENSE_DETAIL |
                                 ERAY_RENDER_SEPARATE_FILL | ERAY_RENDER_NO_SEPARATE_FILL | ERAY_RENDER_SHARED_DETAIL;
    if (rp->flags & ~known_flags) return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "unknown render flags 0x%x", rp->flags);
    const bool general = rp->anti_aliasing > 0 || bounces > 0;
    uint32_t W, H;
    eray_camera_size(&ctx->camera, &W, &H);
    if (!rp->band_rows && (uint64_t)rp->row0 + rp->rows > H)
        return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "rows [%u, %u) exceed the camera height %u", rp->row0,
                         rp->row0 + rp->rows, H);
    // Image::set indexes y * image.width + x and panics past the end (image.rs:41-43)
    if (W && H &&
        (uint64_t)(H - 1) * rp->image_width + (W - 1) >= (uint64_t)rp->image_width * rp->image_height)
        return set_error(ctx, ERAY_E_OUT_OF_BOUNDS,
                         "camera size %ux%u does not fit the %ux%u engine image (Image::set panics)", W, H,
                         rp->image_width, rp->image_height);
    if (rp->out_ppm && (W != rp->image_width || H != rp->image_height))
        return set_error(ctx, ERAY_E_INVALID_ARGUMENT,
                         "fused PPM output needs camera size == image size; use eray_pack_ppm");
    if (rp->band_rows) {  // interleaved bands: aligned to the 4-row sub-blocks, inside the camera
        if (rp->band_rows % 4 || (rp->band_rows & (rp->band_rows - 1)) || rp->band_stride % 4 || rp->row0 % 4 ||
            rp->band_stride < rp->band_rows)
            return set_error(ctx, ERAY_E_INVALID_ARGUMENT,
                             "bands: band_rows (%u) must be a power of two >= 4, band_stride (%u) and row0 (%u) "
                             "multiples of 4, band_stride >= band_rows", rp->band_rows, rp->band_stride, rp->row0);
        const RowSpan rs = row_span(rp);
        if (rp->rows && (uint64_t)rp->row0 + (uint64_t)((rp->rows - 1) >> rs.band_shift) * rp->band_stride +
                                ((rp->rows - 1) & rs.band_mask) >= H)
            return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "bands: %u local rows reach past the camera height %u",
                             rp->rows, H);
    }
    const bool cull = !general && !(rp->flags & ERAY_RENDER_BRUTE_FORCE);
    if (int st = sync_scene(ctx)) return st;
    *empty = !rp->rows || !W;
    if (*empty) return ERAY_OK;
    // the general tracer's camera rays scan the binned objects' bins (a setup of its own kind)
    const bool trace_bins = general && !(rp->flags & ERAY_RENDER_BRUTE_FORCE) && binned_objects(ctx) > 0;
    bool known = true;
    if (cull || trace_bins)
        if (int st = sync_setup(ctx, W, H, row_span(rp), wait == SetupWait::kYes, &known, trace_bins)) return st;

    FrameParams& p = *out;
    std::memset(&p, 0, sizeof p);  // padding too: the launch-plan cache compares the bytes
    p.nframes = 1;
    const eray_camera& c = ctx->camera;
    p.cx = c.center[0];
    p.cy = c.center[1];
    p.cz = c.center[2];
    p.ratio = c.fov[0] / c.fov[1];
    p.z_dist = c.z_dist;
    p.cam_w = W;
    p.cam_h = H;
    p.img_w = rp->image_width;
    p.img_h = rp->image_height;
    p.row0 = rp->row0;
    p.rows = rp->rows;
    const RowSpan span = row_span(rp);
    p.band_shift = span.band_shift;
    p.band_mask = span.band_mask;
    p.band_stride = span.band_stride;
    p.out_rgb = rp->out_rgb;
    p.out_ppm = rp->out_ppm;
    p.out_face = rp->out_face;
    // 16-byte row stores: 16-byte aligned rows, and byte offsets of the largest output (f32 RGB)
    // within 32 bits (the kernels store through buffer resources, render.hip stream16)
    p.aligned = (p.img_w % 16) == 0 && (uint64_t)p.rows * p.img_w * 12u < (1ull << 32) &&
                ((reinterpret_cast<uintptr_t>(p.out_rgb) | reinterpret_cast<uintptr_t>(p.out_ppm) |
                  reinterpret_cast<uintptr_t>(p.out_face)) & 15) == 0;
    p.tris = ctx->d_hot;
    p.shade = ctx->d_shade;
    p.cull = cull ? ctx->d_cull : nullptr;
    p.objects = ctx->d_objs;
    p.lights = ctx->d_lights;
    p.nobj = (uint32_t)ctx->objects.size();
    p.nlights = (uint32_t)ctx->lights.size();
    p.max_object_tris = 0;
    for (auto& o : ctx->objects) p.max_object_tris = o.T > p.max_object_tris ? o.T : p.max_object_tris;
    p.total_tris = ctx->total_tris;
    p.lds_scene = (ctx->total_tris <= kCacheTris && p.nobj <= kCacheObjects && p.nlights <= kCacheLights) ? 1u : 0u;
    p.spec_pow = ctx->spec_pow ? 1u : 0u;
    p.example_mat = ctx->example_mat ? 1u : 0u;
    p.tiles_x = (W + 63) / 64;
    p.bins_x = (W + kBinW - 1) / kBinW;
    p.bin_phase = rp->row0 % kBinH;
    p.aa = rp->anti_aliasing;
    p.bounces = bounces;
    p.seed_lo = (uint32_t)rp->aa_seed;
    p.seed_hi = (uint32_t)(rp->aa_seed >> 32);
    p.trace_cull = (general && !(rp->flags & ERAY_RENDER_BRUTE_FORCE) && ctx->total_tris <= kTraceSkipTris)
                       ? ctx->d_tcull : nullptr;
    if (p.trace_cull) {  // the tracer's culling records of this camera (enqueued when it or the scene changed)
        std::vector<uint64_t> key(sizeof(eray_camera) / 4 + 3);
        std::memcpy(key.data(), &ctx->camera, sizeof(eray_camera));
        key[key.size() - 3] = ctx->scene_gen;
        key[key.size() - 2] = ((uint64_t)W << 32) | H;
        key[key.size() - 1] = (uint64_t)reinterpret_cast<uintptr_t>(ctx->stream);
        if (key != ctx->tcull_key) {
            ctx->tcull_key.clear();
            HIP_TRY(ctx, launch_trace_cull(p, ctx->stream));
            ctx->tcull_key = std::move(key);
        }
    }
    p.trace_bins = trace_bins ? 1u : 0u;
    if (trace_bins) {  // the setup's detail list (trace.hip trace_binned_kernel, trace_heavy_kernel)
        p.detail_list = ctx->bins.dlist;
        p.detail_heavy = ctx->bins.dcount;
        p.detail_occ = ctx->bins.docc;
    }
    p.launch_flags = rp->flags & ~(ERAY_RENDER_BRUTE_FORCE | kLaunchRingBeyondCache);
    if (!cull) {  // every pixel in detail: one rectangle, the frame (sub-block units)
        if (p.nobj) {
            p.nrect = 1;
            p.rects[0][0] = 0;
            p.rects[0][1] = (int32_t)((W - 1) / 16);
            p.rects[0][2] = 0;
            p.rects[0][3] = (int32_t)((rp->rows - 1) / 4);
            p.total_sub = (uint32_t)(p.rects[0][1] + 1) * (uint32_t)(p.rects[0][3] + 1);
        }
        return ERAY_OK;
    }
    if (binned_objects(ctx)) {  // the detail sub-block list of the setup (ordered: heavy ones first)
        p.detail_list = ctx->bins.dlist;
        p.detail_occ = ctx->bins.docc;
        p.detail_heavy = ctx->bins.dcount;
    }
    if (known) {  // args mode
        const CamState& h = *ctx->h_state;
        p.nrect = h.nrect;
        p.total_sub = h.total_sub;
        std::memcpy(p.rects, h.rects, sizeof p.rects);
    } else {  // device-camera mode (the last known count only steers the launch shape)
        p.cam_state = ctx->d_state;
        p.total_sub = ctx->h_state ? ctx->h_state->total_sub : 0u;
    }
    return ERAY_OK;
}

hipError_t launch_frame(eray_ctx* ctx, const FrameParams& p) { return launch_render(p, ctx->lc, ctx->stream); }

// The source tag of frames rendered with p (prepare_render of rp): the scene camera through the
// frame kernel with its culling setup, or another kind.
FrameSource render_source(const eray_ctx* ctx, const FrameParams& p, const eray_render_params* rp) {
    if (p.cull && !p.aa && !p.bounces) return scene_source(ctx, p.cam_w, p.cam_h, row_span(rp));
    FrameSource s;
    s.kind = kSrcOther;
    return s;
}
}  // namespace

int eray_render(eray_ctx* ctx, const eray_render_params* rp) {
    FrameParams p;
    bool empty = false;
    if (int st = prepare_render(ctx, rp, &p, &empty)) return st;
    if (!empty) {
        HIP_TRY(ctx, launch_frame(ctx, p));
        tag_frames(ctx, p.out_ppm, 0, 1, render_source(ctx, p, rp));
    }
    return ERAY_OK;
}

}  // extern "C"

namespace {
constexpr uint32_t kGraphFrames = 64;

constexpr size_t kGraphCache = 6;

// The graph of n back-to-back frames, frame f enqueued by body(f), for `key` (+ n and the
// stream), captured unless cached.
template <typename Body>
int ensure_graph(eray_ctx* ctx, std::vector<unsigned char> key, uint32_t n, Body&& body, hipGraphExec_t* out) {
    const size_t at = key.size();
    key.resize(at + sizeof n + sizeof ctx->stream);
    std::memcpy(key.data() + at, &n, sizeof n);
    std::memcpy(key.data() + at + sizeof n, &ctx->stream, sizeof ctx->stream);
    for (auto& G : ctx->graphs)
        if (G.key == key) {
            G.used = ++ctx->graph_clock;
            *out = G.exec;
            return ERAY_OK;
        }
    if (ctx->graphs.size() >= kGraphCache) {  // evict the least recently used
        size_t lru = 0;
        for (size_t i = 1; i < ctx->graphs.size(); ++i)
            if (ctx->graphs[i].used < ctx->graphs[lru].used) lru = i;
        auto& G = ctx->graphs[lru];
        if (G.exec) hipGraphExecDestroy(G.exec);
        if (G.graph) hipGraphDestroy(G.graph);
        ctx->graphs.erase(ctx->graphs.begin() + (std::ptrdiff_t)lru);
    }
    HIP_TRY(ctx, hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
    int st = ERAY_OK;
    for (uint32_t f = 0; f < n && st == ERAY_OK; ++f) st = body(f, n);
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamEndCapture(ctx->stream, &g);
    if (st != ERAY_OK) {
        if (g) hipGraphDestroy(g);
        return st;
    }
    hipGraphExec_t exec = nullptr;
    if (e == hipSuccess) e = hipGraphInstantiate(&exec, g, nullptr, nullptr, 0);
    // the executable's packets and arguments go to the device now, not at its first launch (a
    // plan prepared ahead of a timed loop otherwise pays ~20 us at its first replay)
    if (e == hipSuccess) e = hipGraphUpload(exec, ctx->stream);
    if (e != hipSuccess) {
        if (g) hipGraphDestroy(g);
        return set_error(ctx, ERAY_E_HIP, "frame graph capture: %s", hipGetErrorString(e));
    }
    eray_ctx::FrameGraph G;
    G.graph = g;
    G.exec = exec;
    G.key = std::move(key);
    G.used = ++ctx->graph_clock;
    ctx->graphs.push_back(std::move(G));
    *out = exec;
    return ERAY_OK;
}

std::vector<unsigned char> params_key(const FrameParams& p, uint32_t kind) {
    std::vector<unsigned char> key(sizeof p + sizeof kind);
    std::memcpy(key.data(), &p, sizeof p);
    std::memcpy(key.data() + sizeof p, &kind, sizeof kind);
    return key;
}

// The launch plan of `frames` frames: a graph of `chunk` = min(frames, kGraphFrames) frames,
// replayed frames / chunk times, and a graph of the remainder (no plain launches, whose host
// cost can exceed a frame's device time).  chunk = 0: plain launches (null stream, 1 frame).
struct Plan {
    uint32_t chunk = 0, rest = 0;
    hipGraphExec_t chunk_exec = nullptr, rest_exec = nullptr;
};
template <typename Body>
int ensure_plan(eray_ctx* ctx, const std::vector<unsigned char>& key, uint32_t frames, Body&& body, Plan* plan) {
    *plan = Plan{};
    if (!ctx->stream || frames < 2) return ERAY_OK;  // the null stream cannot be captured
    const uint32_t n = frames < kGraphFrames ? frames : kGraphFrames;
    if (int st = ensure_graph(ctx, key, n, body, &plan->chunk_exec)) return st;
    plan->chunk = n;
    const uint32_t r = frames % n;
    if (r > 1) {
        if (int st = ensure_graph(ctx, key, r, body, &plan->rest_exec)) return st;
        plan->rest = r;
    }
    return ERAY_OK;
}

// Replays `plan` for `frames` frames (before_chunk(first frame, count) runs ahead of each graph
// launch, plain(f) renders frames the plan does not cover); mean device time per frame when asked.
template <typename Before, typename Plain>
int replay(eray_ctx* ctx, const Plan& plan, uint32_t frames, Before&& before_chunk, Plain&& plain, float* mean_ms) {
    hipEvent_t ev[2] = {nullptr, nullptr};
    if (mean_ms) {
        *mean_ms = 0.0f;
        for (auto& e : ev) {
            hipError_t he = hipEventCreate(&e);
            if (he != hipSuccess) {
                if (ev[0]) hipEventDestroy(ev[0]);
                return set_error(ctx, ERAY_E_HIP, "hipEventCreate: %s", hipGetErrorString(he));
            }
        }
    }
    int st = ERAY_OK;
    hipError_t he = mean_ms ? hipEventRecord(ev[0], ctx->stream) : hipSuccess;
    uint32_t done = 0;
    for (; plan.chunk && done + plan.chunk <= frames && he == hipSuccess && !st; done += plan.chunk) {
        st = before_chunk(done, plan.chunk);
        if (!st) he = hipGraphLaunch(plan.chunk_exec, ctx->stream);
    }
    if (plan.rest && done + plan.rest == frames && he == hipSuccess && !st) {
        st = before_chunk(done, plan.rest);
        if (!st) he = hipGraphLaunch(plan.rest_exec, ctx->stream);
        done += plan.rest;
    }
    for (; done < frames && he == hipSuccess && !st; ++done) st = plain(done);
    if (mean_ms && he == hipSuccess && !st) {
        he = hipEventRecord(ev[1], ctx->stream);
        if (he == hipSuccess) he = hipEventSynchronize(ev[1]);
        float ms = 0.0f;
        if (he == hipSuccess) he = hipEventElapsedTime(&ms, ev[0], ev[1]);
        if (he == hipSuccess) *mean_ms = ms / (float)frames;
    }
    for (auto e : ev)
        if (e) hipEventDestroy(e);
    if (st) return st;
    if (he != hipSuccess) return set_error(ctx, ERAY_E_HIP, "render loop: %s", hipGetErrorString(he));
    return ERAY_OK;
}
// Frames in flight (eray_frame_ring): frames of one call are rendered `per_launch` to a kernel
// launch (FrameParams::nframes), frame k into ring slot k % slots.
struct Ring {
    uint32_t slots = 1, per_launch = 1;
    uint64_t rgb = 0, ppm = 0, face = 0;  // bytes between slots
};
// One launch renders at most this many pixels (frames x rows x width) when the library picks the
// frames per launch, at most kMaxInFlight frames.  Measured (scripts/frames_in_flight.py,
// profiles/r03/frames_in_flight.jsonl, device us per frame by frames per launch): the cube at
// 1920x1080 9.3 / 7.6 / 5.4 / 5.0 for 1 / 2 / 4 / 8, at 3840x2160 22.9 / 19.6 for 1 / 2; the 70k
// stand-in (screen bins, heavier detail work) at 1920x1080 14.2 / 9.2 / 8.2 / 9.2, at 3840x2160
// 29.1 / 34.5 for 1 / 2.  So two frames of 3840x2160 pixels for small scenes, one for scenes with
// binned meshes.
constexpr uint64_t kInFlightPixels = 2ull * 3840ull * 2160ull, kInFlightPixelsBinned = 3840ull * 2160ull;
constexpr uint32_t kMaxInFlight = 8;

// The library's frames per launch for frames of cam_w x rows pixels and a ring of `slots`.
uint32_t auto_frames(uint64_t cam_w, uint64_t rows, uint32_t slots, bool binned) {
    const uint64_t cap = binned ? kInFlightPixelsBinned : kInFlightPixels;
    uint32_t F = 1;
    while (F * 2 <= kMaxInFlight && F * 2 <= slots && (uint64_t)(F * 2) * cam_w * rows <= cap) F *= 2;
    return F;
}

int make_ring(eray_ctx* ctx, const eray_render_params* rp, const FrameParams& p, const eray_frame_ring* r, Ring* out) {
    *out = Ring{};
    if (!r) return ERAY_OK;
    if (!r->slots || r->slots > 64 || (r->slots & (r->slots - 1)))
        return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "ring: slots (%u) must be a power of two <= 64", r->slots);
    const uint64_t px = (uint64_t)rp->rows * rp->image_width;
    const uint64_t need[3] = {px * 12u, px * 3u, px * 4u};
    const uint64_t stride[3] = {r->rgb_stride, r->ppm_stride, r->face_stride};
    const void* ptr[3] = {rp->out_rgb, rp->out_ppm, rp->out_face};
    for (int k = 0; k < 3; ++k) {
        if (!ptr[k] || r->slots == 1) continue;
        if (stride[k] % 16 || stride[k] < need[k])
            return set_error(ctx, ERAY_E_INVALID_ARGUMENT,
                             "ring: output %d's slot stride %llu must be a multiple of 16 of at least %llu bytes", k,
                             (unsigned long long)stride[k], (unsigned long long)need[k]);
    }
    if (r->frames_per_launch && (r->frames_per_launch > r->slots || (r->frames_per_launch & (r->frames_per_launch - 1))))
        return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "ring: frames_per_launch (%u) must be a power of two <= slots (%u)",
                         r->frames_per_launch, r->slots);
    out->slots = r->slots;
    out->rgb = r->slots > 1 ? r->rgb_stride : 0;
    out->ppm = r->slots > 1 ? r->ppm_stride : 0;
    out->face = r->slots > 1 ? r->face_stride : 0;
    uint32_t F = 1;
    if (p.aa || p.bounces || r->slots == 1) {
        F = 1;  // the general tracer renders one frame per launch
    } else if (r->frames_per_launch) {
        F = r->frames_per_launch;
    } else {
        F = auto_frames(p.cam_w, p.rows, r->slots, p.max_object_tris > kDirectMax);
    }
    out->per_launch = F;
    return ERAY_OK;
}

// The launch parameters of frames [f, f + count) of a call: ring slot f % slots onwards (slots is
// a multiple of per_launch, so a launch's frames never wrap).
FrameParams ring_frames(const FrameParams& p, const Ring& r, uint32_t f, uint32_t count) {
    FrameParams q = p;
    const uint64_t slot = f % r.slots;
    q.nframes = count;
    q.rgb_stride = r.rgb;
    q.ppm_stride = r.ppm;
    q.face_stride = r.face;
    if (q.out_rgb) q.out_rgb = reinterpret_cast<float*>(reinterpret_cast<char*>(q.out_rgb) + slot * r.rgb);
    if (q.out_ppm) q.out_ppm += slot * r.ppm;
    if (q.out_face) q.out_face = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(q.out_face) + slot * r.face);
    const uint64_t ring_bytes = (uint64_t)r.slots * ((q.out_rgb ? r.rgb : 0) + (q.out_ppm ? r.ppm : 0) + (q.out_face ? r.face : 0));
    if (ring_bytes > kInfinityCacheBytes) q.launch_flags |= kLaunchRingBeyondCache;
    return q;
}

std::vector<unsigned char> ring_key(std::vector<unsigned char> key, const Ring& r) {
    const size_t at = key.size();
    key.resize(at + sizeof r);
    std::memcpy(key.data() + at, &r, sizeof r);
    return key;
}
}  // namespace

// The camera-path rectangle union (eray_gather_frames' layout of path frames): the device
// accumulator for nobj objects (SetupParams::path_union: the path's setup kernels fold every
// camera's rectangles into it) and a ring of kUnionRing finished unions in mapped pinned memory.
int ensure_union(eray_ctx* ctx, uint32_t nobj) {
    if (ctx->d_union_acc && ctx->union_cap >= nobj) return ERAY_OK;
    for (hipEvent_t& ev : ctx->union_ev) {
        if (!ev) HIP_TRY(ctx, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        HIP_TRY(ctx, hipEventSynchronize(ev));  // (a flush into the ring still in flight)
    }
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (ctx->d_union_acc) HIP_TRY(ctx, hipFree(ctx->d_union_acc));
    if (ctx->h_union) HIP_TRY(ctx, hipHostFree(ctx->h_union));
    ctx->d_union_acc = nullptr;
    ctx->h_union = nullptr;
    ctx->d_union_host = nullptr;
    ctx->union_cap = 0;
    const uint32_t n = std::max<uint32_t>(nobj, 1u);
    HIP_TRY(ctx, hipMalloc((void**)&ctx->d_union_acc, 4 * sizeof(int32_t) * n));
    HIP_TRY(ctx, hipHostMalloc((void**)&ctx->h_union, 4 * sizeof(int32_t) * n * kUnionRing, hipHostMallocMapped));
    HIP_TRY(ctx, hipHostGetDevicePointer((void**)&ctx->d_union_host, ctx->h_union, 0));
    HIP_TRY(ctx, launch_union_flush(ctx->d_union_acc, n, nullptr, ctx->stream));  // the initial reset
    for (auto& s : ctx->union_seq) s = 0;
    ctx->union_cap = n;
    return ERAY_OK;
}
// After path call `seq`'s frames: its union into ring entry seq % kUnionRing (and the accumulator
// reset for the next path), one kernel on the stream.
int finish_union(eray_ctx* ctx, uint64_t seq, const FrameSource& src, uint32_t nobj) {
    const uint32_t e = (uint32_t)(seq % kUnionRing);
    HIP_TRY(ctx, hipEventSynchronize(ctx->union_ev[e]));  // the entry's flush kUnionRing paths back
    HIP_TRY(ctx, launch_union_flush(ctx->d_union_acc, std::max(nobj, 1u),
                                    ctx->d_union_host + (size_t)e * 4 * ctx->union_cap, ctx->stream));
    HIP_TRY(ctx, hipEventRecord(ctx->union_ev[e], ctx->stream));
    ctx->union_seq[e] = seq;
    ctx->union_src[e] = src;
    ctx->union_nobj[e] = nobj;
    ctx->union_gen[e] = ctx->scene_gen;
    return ERAY_OK;
}

extern "C" {

int eray_render_prepare_ring(eray_ctx* ctx, const eray_render_params* rp, const eray_frame_ring* ring, uint32_t frames) {
    FrameParams p;
    bool empty = false;
    if (int st = prepare_render(ctx, rp, &p, &empty, SetupWait::kYes)) return st;
    if (empty) return ERAY_OK;
    Ring r;
    if (int st = make_ring(ctx, rp, p, ring, &r)) return st;
    Plan plan;
    auto body = [&](uint32_t f, uint32_t n) -> int {
        if (f % r.per_launch) return ERAY_OK;  // rendered by the launch of frame f - f % per_launch
        HIP_TRY(ctx, launch_frame(ctx, ring_frames(p, r, f, std::min(r.per_launch, n - f))));
        return ERAY_OK;
    };
    return ensure_plan(ctx, ring_key(params_key(p, 0), r), frames, body, &plan);
}

uint32_t eray_frames_per_launch(eray_ctx* ctx, const eray_render_params* rp, uint32_t slots) {
    if (!ctx || !rp || !slots) return 1u;
    if (rp->anti_aliasing || rp->bounces) return 1u;
    uint32_t W, H;
    eray_camera_size(&ctx->camera, &W, &H);
    bool binned = false;
    for (auto& o : ctx->objects) binned |= o.T > kDirectMax;
    return auto_frames(W, rp->rows, slots, binned);
}

int eray_render_prepare(eray_ctx* ctx, const eray_render_params* rp, uint32_t frames) {
    return eray_render_prepare_ring(ctx, rp, nullptr, frames);
}

int eray_render_frames_ring(eray_ctx* ctx, const eray_render_params* rp, const eray_frame_ring* ring, uint32_t frames,
                            float* mean_frame_ms) {
    FrameParams p;
    bool empty = false;
    if (mean_frame_ms) *mean_frame_ms = 0.0f;
    if (int st = prepare_render(ctx, rp, &p, &empty, SetupWait::kYes)) return st;
    if (empty || !frames) return ERAY_OK;
    Ring r;
    if (int st = make_ring(ctx, rp, p, ring, &r)) return st;
    Plan plan;
    auto body = [&](uint32_t f, uint32_t n) -> int {
        if (f % r.per_launch) return ERAY_OK;
        HIP_TRY(ctx, launch_frame(ctx, ring_frames(p, r, f, std::min(r.per_launch, n - f))));
        return ERAY_OK;
    };
    if (int st = ensure_plan(ctx, ring_key(params_key(p, 0), r), frames, body, &plan)) return st;
    auto none = [](uint32_t, uint32_t) { return (int)ERAY_OK; };
    auto plain = [&](uint32_t f) { return body(f, frames); };
    const int st = replay(ctx, plan, frames, none, plain, mean_frame_ms);
    if (!st) tag_frames(ctx, p.out_ppm, r.ppm, std::min(frames, r.slots), render_source(ctx, p, rp));
    return st;
}

int eray_render_frames(eray_ctx* ctx, const eray_render_params* rp, uint32_t frames, float* mean_frame_ms) {
    return eray_render_frames_ring(ctx, rp, nullptr, frames, mean_frame_ms);
}

int eray_time_frames_ring(eray_ctx* ctx, const eray_render_params* rp, const eray_frame_ring* ring, uint32_t frames,
                          eray_kernel_times* out) {
    if (!out) return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "kernel timing: out is null");
    *out = eray_kernel_times{};
    FrameParams p;
    bool empty = false;
    if (int st = prepare_render(ctx, rp, &p, &empty, SetupWait::kYes)) return st;
    if (empty || !frames) return ERAY_OK;
    if (p.aa || p.bounces)
        return set_error(ctx, ERAY_E_UNSUPPORTED, "kernel timing: the frame kernel only (no anti-aliasing or bounces)");
    Ring r;
    if (int st = make_ring(ctx, rp, p, ring, &r)) return st;
    const uint32_t F = r.per_launch, L = std::max(1u, frames / F);
    std::vector<hipEvent_t> ev(4 * (size_t)L, nullptr);
    auto drop = [&]() {
        for (auto e : ev)
            if (e) hipEventDestroy(e);
    };
    int st = ERAY_OK;
    std::vector<uint32_t> fill_used(L, 0u);
    for (uint32_t l = 0; l < L && !st; ++l) {
        LaunchCtx lc = ctx->lc;
        for (int k = 0; k < 4 && !st; ++k) {
            const hipError_t e = hipEventCreate(&ev[4 * (size_t)l + k]);
            if (e != hipSuccess) st = set_error(ctx, ERAY_E_HIP, "hipEventCreate: %s", hipGetErrorString(e));
        }
        if (st) break;
        lc.frame_t[0] = ev[4 * (size_t)l];
        lc.frame_t[1] = ev[4 * (size_t)l + 1];
        lc.fill_t[0] = ev[4 * (size_t)l + 2];
        lc.fill_t[1] = ev[4 * (size_t)l + 3];
        lc.fill_used = &fill_used[l];
        const hipError_t e = launch_render(ring_frames(p, r, l * F, F), lc, ctx->stream);
        if (e != hipSuccess) st = set_error(ctx, ERAY_E_HIP, "timed frame launch: %s", hipGetErrorString(e));
    }
    hipError_t e = st ? hipSuccess : hipStreamSynchronize(ctx->stream);
    double sum = 0.0, fill = 0.0, span = 0.0;
    float lo = 0.0f, hi = 0.0f;
    uint32_t nfill = 0;
    for (uint32_t l = 0; l < L && !st && e == hipSuccess; ++l) {
        hipEvent_t* q = &ev[4 * (size_t)l];
        float k = 0.0f;
        if ((e = hipEventElapsedTime(&k, q[0], q[1])) != hipSuccess) break;
        sum += k;
        lo = l ? std::min(lo, k) : k;
        hi = l ? std::max(hi, k) : k;
        float s = k;
        if (fill_used[l]) {  // the separate fill beside it: both kernels' span, from the frame kernel's start
            float f0 = 0.0f, f1 = 0.0f, fk = 0.0f;
            if ((e = hipEventElapsedTime(&fk, q[2], q[3])) != hipSuccess ||
                (e = hipEventElapsedTime(&f0, q[0], q[2])) != hipSuccess ||
                (e = hipEventElapsedTime(&f1, q[0], q[3])) != hipSuccess)
                break;
            fill += fk;
            ++nfill;
            s = std::max(k, f1) - std::min(0.0f, f0);
        }
        span += s;
    }
    drop();
    if (st) return st;
    if (e != hipSuccess) return set_error(ctx, ERAY_E_HIP, "kernel timing: %s", hipGetErrorString(e));
    tag_frames(ctx, p.out_ppm, r.ppm, std::min(L * F, r.slots), render_source(ctx, p, rp));
    out->launches = L;
    out->frames_per_launch = F;
    out->frame_kernel_ms = (float)(sum / L);
    out->frame_kernel_min_ms = lo;
    out->frame_kernel_max_ms = hi;
    out->fill_kernel_ms = nfill ? (float)(fill / nfill) : 0.0f;
    out->launch_span_ms = (float)(span / L);
    return ERAY_OK;
}

int eray_time_write_ceiling(eray_ctx* ctx, const eray_render_params* rp, const eray_frame_ring* ring, uint32_t frames,
                            uint32_t wgs_per_cu, eray_kernel_times* out) {
    if (!out) return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "write ceiling: out is null");
    *out = eray_kernel_times{};
    if (wgs_per_cu < 1 || wgs_per_cu > 8)
        return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "write ceiling: %u workgroups per CU (1..8)", wgs_per_cu);
    FrameParams p;
    bool empty = false;
    if (int st = prepare_render(ctx, rp, &p, &empty, SetupWait::kYes)) return st;
    if (empty || !frames) return ERAY_OK;
    if (!p.aligned || p.img_w % 64u || p.rows % 4u)
        return set_error(ctx, ERAY_E_UNSUPPORTED, "write ceiling: whole 64x4 blocks only (%ux%u, aligned %u)", p.img_w,
                         p.rows, p.aligned);
    Ring r;
    if (int st = make_ring(ctx, rp, p, ring, &r)) return st;
    const uint32_t F = r.per_launch, L = std::max(1u, frames / F);
    std::vector<hipEvent_t> ev(2 * (size_t)L, nullptr);
    int st = ERAY_OK;
    hipError_t e = hipSuccess;
    for (size_t k = 0; k < ev.size() && e == hipSuccess; ++k) e = hipEventCreate(&ev[k]);
    for (uint32_t l = 0; l < L && e == hipSuccess; ++l) {
        const hipEvent_t t[2] = {ev[2 * (size_t)l], ev[2 * (size_t)l + 1]};
        e = launch_write_ceiling(ring_frames(p, r, l * F, F), wgs_per_cu, t, ctx->stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    double sum = 0.0;
    float lo = 0.0f, hi = 0.0f;
    for (uint32_t l = 0; l < L && e == hipSuccess; ++l) {
        float k = 0.0f;
        if ((e = hipEventElapsedTime(&k, ev[2 * (size_t)l], ev[2 * (size_t)l + 1])) != hipSuccess) break;
        sum += k;
        lo = l ? std::min(lo, k) : k;
        hi = l ? std::max(hi, k) : k;
    }
    for (auto x : ev)
        if (x) hipEventDestroy(x);
    if (e != hipSuccess) st = set_error(ctx, ERAY_E_HIP, "write ceiling: %s", hipGetErrorString(e));
    if (st) return st;
    // the slots now hold background frames, not renders of the scene
    tag_frames(ctx, p.out_ppm, r.ppm, std::min(L * F, r.slots), FrameSource{kSrcOther});
    out->launches = L;
    out->frames_per_launch = F;
    out->frame_kernel_ms = (float)(sum / L);
    out->frame_kernel_min_ms = lo;
    out->frame_kernel_max_ms = hi;
    out->launch_span_ms = out->frame_kernel_ms;
    return ERAY_OK;
}

int eray_render_camera_path_ring(eray_ctx* ctx, const eray_render_params* rp, const eray_frame_ring* ring,
                                 const eray_camera* cameras, uint32_t n, float* mean_frame_ms) {
    if (int st = use_device(ctx)) return st;
    if (mean_frame_ms) *mean_frame_ms = 0.0f;
    if (!rp) return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "params is null");
    if (n && !cameras) return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "cameras is null");
    uint32_t W, H;
    eray_camera_size(&ctx->camera, &W, &H);
    for (uint32_t f = 0; f < n; ++f) {  // one engine image: every camera has the scene camera's size
        uint32_t w, h;
        eray_camera_size(&cameras[f], &w, &h);
        if (w != W || h != H)
            return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "camera %u: size %ux%u differs from the scene camera's %ux%u",
                             f, w, h, W, H);
    }
    FrameParams p;
    bool empty = false;
    // the scene camera's setup (scene upload, bins layout; the last known detail count steers the
    // launch shape) — enqueued, not waited for: the path's frames read their own cameras' setups
    if (int st = prepare_render(ctx, rp, &p, &empty, SetupWait::kNo)) return st;
    if (empty || !n) return ERAY_OK;
    Ring r;
    if (int st = make_ring(ctx, rp, p, ring, &r)) return st;
    if (!p.cull) {  // anti-aliasing, bounces, brute force: no per-camera setup, camera in the arguments
        const eray_camera saved = ctx->camera;
        hipEvent_t ev[2] = {nullptr, nullptr};  // mean device ms per frame, as replay() times it
        if (mean_frame_ms) {
            for (auto& e : ev) HIP_TRY(ctx, hipEventCreate(&e));
            HIP_TRY(ctx, hipEventRecord(ev[0], ctx->stream));
        }
        auto drop = [&]() {
            for (auto e : ev)
                if (e) hipEventDestroy(e);
        };
        for (uint32_t f = 0; f < n; ++f) {
            ctx->camera = cameras[f];
            FrameParams q;
            int st = prepare_render(ctx, rp, &q, &empty);
            if (!st && !empty) {
                const hipError_t e = launch_frame(ctx, ring_frames(q, r, f, 1));
                if (e != hipSuccess) st = set_error(ctx, ERAY_E_HIP, "render: %s", hipGetErrorString(e));
            }
            if (st) {
                ctx->camera = saved;
                drop();
                return st;
            }
        }
        ctx->camera = saved;
        FrameSource other;
        other.kind = kSrcOther;
        tag_frames(ctx, p.out_ppm, r.ppm, std::min(n, r.slots), other);
        if (mean_frame_ms) {
            hipError_t e = hipEventRecord(ev[1], ctx->stream);
            float ms = 0.0f;
            if (e == hipSuccess) e = hipEventSynchronize(ev[1]);
            if (e == hipSuccess) e = hipEventElapsedTime(&ms, ev[0], ev[1]);
            drop();
            if (e != hipSuccess) return set_error(ctx, ERAY_E_HIP, "camera path timing: %s", hipGetErrorString(e));
            *mean_frame_ms = ms / (float)n;
        }
        return ERAY_OK;
    }
    // device-camera mode: every frame reads its setup's CamState; the per-frame detail lists are
    // appended split (heavy sub-blocks from the front, light ones from the back: CamState counts)
    p.cam_state = ctx->d_state;
    p.detail_heavy = nullptr;
    p.dlist_split = p.detail_list ? (uint32_t)ctx->bins.nsub : 0u;
    p.nrect = 0;
    std::memset(p.rects, 0, sizeof p.rects);
    // the cameras: staged in pinned memory, copied to the device once per call; each graph chunk
    // reads its cameras from d_path (a device-to-device copy of its slice before each replay)
    const uint32_t hb = ctx->path_buf;
    ctx->path_buf ^= 1u;
    CamDev*& h_path = ctx->h_path[hb];
    if (ctx->h_path_cap[hb] < n) {
        HIP_TRY(ctx, hipEventSynchronize(ctx->path_ev[hb]));
        if (h_path) HIP_TRY(ctx, hipHostFree(h_path));
        h_path = nullptr;
        HIP_TRY(ctx, hipHostMalloc((void**)&h_path, sizeof(CamDev) * n, hipHostMallocDefault));
        ctx->h_path_cap[hb] = n;
    }
    HIP_TRY(ctx, hipEventSynchronize(ctx->path_ev[hb]));  // the upload two calls back has read this buffer
    for (uint32_t f = 0; f < n; ++f) h_path[f] = cam_dev(cameras[f]);
    if (int st = ensure(ctx, &ctx->d_path_all, &ctx->path_all_cap, n)) return st;
    if (int st = ensure(ctx, &ctx->d_path, &ctx->path_cap, kGraphFrames)) return st;
    // a path of one graph chunk goes straight into the chunk's camera slots (no per-chunk copy)
    const bool one_chunk = n <= kGraphFrames;
    HIP_TRY(ctx, hipMemcpyAsync(one_chunk ? ctx->d_path : ctx->d_path_all, h_path, sizeof(CamDev) * n,
                                hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipEventRecord(ctx->path_ev[hb], ctx->stream));
    const bool batched = batch_setup_ok(ctx);
    // scenes with binned objects: the setups of up to mc_k cameras at once (one chain of
    // kernels for all of them, ensure_multi), then their frames, each from its camera's slices
    const bool multi = !batched && binned_objects(ctx) > 0;
    const RowSpan rs = row_span(rp);
    if (multi)
        if (int st = ensure_multi(ctx, W, H, rs)) return st;
    if (multi) {  // frames in flight within one multi-camera build: per_launch divides mc_k
        while (ctx->mc_k % r.per_launch) r.per_launch /= 2;
    } else if (!batched) {
        r.per_launch = 1;  // a setup (screen bins) per frame: one frame per launch
    }
    const uint32_t T = ctx->total_tris, nobj = (uint32_t)ctx->objects.size();
    // this call's frames are camera-path frames (eray_gather_frames): every camera's object
    // rectangles fold into the union of the call
    FrameSource psrc;
    psrc.kind = kSrcPath;
    psrc.key = ++ctx->path_seq;
    psrc.W = W;
    psrc.H = H;
    psrc.row0 = rs.row0;
    psrc.rows = rs.rows;
    psrc.band_shift = rs.band_shift;
    psrc.band_stride = rs.band_stride;
    if (int st = ensure_union(ctx, nobj)) return st;
    if (batched) {
        if (int st = ensure(ctx, &ctx->d_bcull, &ctx->bcull_cap, (size_t)kGraphFrames * T)) return st;
        if (int st = ensure(ctx, &ctx->d_bobjs, &ctx->bobjs_cap, (size_t)kGraphFrames * nobj)) return st;
        if (int st = ensure(ctx, &ctx->d_bstate, &ctx->bstate_cap, kGraphFrames)) return st;
    }
    // frame `slot` of a batch whose setups started at camera `cams` (count cameras) — the batch
    // is enqueued with its first frame; frames in flight: the launch of slot s (s % per_launch ==
    // 0) renders slots [s, s + per_launch) of the batch, each from its own setup slot; `f` is the
    // frame's index in the call (its ring slot)
    auto batch_frame = [&](const CamDev* cams, uint32_t slot, uint32_t count, uint32_t f) -> int {
        if (slot == 0) {
            SetupParams sp = setup_params(ctx, cams, W, H, row_span(rp));
            sp.cull = ctx->d_bcull;
            sp.objs = ctx->d_bobjs;
            sp.objs_src = ctx->d_objs;
            sp.state = ctx->d_bstate;
            sp.path_union = ctx->d_union_acc;
            sp.union_nobj = nobj;
            HIP_TRY(ctx, launch_camera_setup_batch(sp, count, ctx->stream));
        }
        if (slot % r.per_launch) return ERAY_OK;
        FrameParams q = ring_frames(p, r, f, std::min(r.per_launch, count - slot));
        q.cam_state = ctx->d_bstate + slot;
        q.cull = ctx->d_bcull + (size_t)slot * T;
        q.objects = ctx->d_bobjs + (size_t)slot * nobj;
        q.dev_slots = 1;
        HIP_TRY(ctx, launch_frame(ctx, q));
        return ERAY_OK;
    };
    // frame `slot` of a run of `count` cameras at `cams` (f: its index in the call, its ring slot):
    // batch b = slot / K of the run is built into set b % 2; the first batch's build on the main
    // stream, every later one on mc_stream while the previous batch's frames render (it waits for
    // the frames of batch b - 2, the set's previous users), the frames wait for their build;
    // frames in flight: the launch of slot s (s % per_launch == 0) renders slots [s, s + n) of
    // the batch (per_launch divides K, so a launch never spans two builds), each from its slices
    auto multi_frame = [&](const CamDev* cams, uint32_t slot, uint32_t count, uint32_t f) -> int {
        const uint32_t K = ctx->mc_k, k = slot % K, b = slot / K;
        auto& m = ctx->mc[b & 1u];
        if (k == 0) {
            if (b == 0) {
                if (int st = enqueue_multi_setup(ctx, m, cams, std::min(K, count), W, H, rs, ctx->stream, ctx->d_union_acc))
                    return st;
                HIP_TRY(ctx, hipEventRecord(ctx->mc_fork, ctx->stream));
            } else {
                HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->mc_ready[b & 1u], 0));
            }
            if ((b + 1) * K < count) {  // the next batch's build, beside this batch's frames
                auto& m2 = ctx->mc[(b + 1) & 1u];
                HIP_TRY(ctx, hipStreamWaitEvent(ctx->mc_stream, b == 0 ? ctx->mc_fork : ctx->mc_free[(b + 1) & 1u], 0));
                if (int st = enqueue_multi_setup(ctx, m2, cams + (b + 1) * K, std::min(K, count - (b + 1) * K), W, H, rs,
                                                 ctx->mc_stream, ctx->d_union_acc))
                    return st;
                HIP_TRY(ctx, hipEventRecord(ctx->mc_ready[(b + 1) & 1u], ctx->mc_stream));
            }
        }
        if (slot % r.per_launch) return ERAY_OK;  // rendered by the launch of slot - slot % per_launch
        const uint32_t nsub = (uint32_t)m.bins.nsub, nf = std::min(r.per_launch, count - slot);
        FrameParams q = ring_frames(p, r, f, nf);
        q.cam_state = m.state + k;
        q.cull = m.cull + (size_t)k * T;
        q.objects = m.objs + (size_t)k * nobj;
        q.detail_list = m.bins.dlist + (size_t)k * nsub;
        q.detail_occ = m.bins.docc + (size_t)k * (nsub / 4);
        q.dev_slots = nf > 1 ? 1u : 0u;
        q.dlist_stride = nf > 1 ? nsub : 0u;
        q.dlist_split = nsub;
        HIP_TRY(ctx, launch_frame(ctx, q));
        if (k + nf >= K || slot + nf >= count) HIP_TRY(ctx, hipEventRecord(ctx->mc_free[b & 1u], ctx->stream));
        return ERAY_OK;
    };
    auto frame = [&](const CamDev* cam, uint32_t f) -> int {
        if (multi) return multi_frame(cam, 0, 1, f);
        if (batched) {
            const Ring keep = r;
            r.per_launch = 1;
            const int st = batch_frame(cam, 0, 1, f);
            r = keep;
            return st;
        }
        if (int st = enqueue_setup(ctx, cam, W, H, row_span(rp), false, false, ctx->d_union_acc)) return st;
        HIP_TRY(ctx, launch_frame(ctx, ring_frames(p, r, f, 1)));
        return ERAY_OK;
    };
    auto body = [&](uint32_t f, uint32_t count) {
        if (multi) return multi_frame(ctx->d_path, f, count, f);
        return batched ? batch_frame(ctx->d_path, f, count, f) : frame(ctx->d_path + f, f);
    };
    std::vector<unsigned char> key = ring_key(params_key(p, batched ? 2 : 1), r);
    for (const void* ptr : {(const void*)ctx->d_path, (const void*)ctx->d_bcull, (const void*)ctx->d_bobjs,
                            (const void*)ctx->d_bstate, (const void*)ctx->d_union_acc})
        key.insert(key.end(), reinterpret_cast<const unsigned char*>(&ptr),
                   reinterpret_cast<const unsigned char*>(&ptr) + sizeof ptr);
    // the captured setup and bins kernels hold every bin buffer's address: a reallocation (a grown
    // capacity) must never replay a graph of the old buffers, even if some addresses recur
    key.insert(key.end(), reinterpret_cast<const unsigned char*>(&ctx->bins_gen),
               reinterpret_cast<const unsigned char*>(&ctx->bins_gen) + sizeof ctx->bins_gen);
    const uint64_t mc_gen = multi ? ctx->mc_gen : 0u;  // (likewise the multi-camera buffers)
    key.insert(key.end(), reinterpret_cast<const unsigned char*>(&mc_gen),
               reinterpret_cast<const unsigned char*>(&mc_gen) + sizeof mc_gen);
    auto before = [&](uint32_t first, uint32_t count) -> int {
        if (one_chunk) return ERAY_OK;
        HIP_TRY(ctx, hipMemcpyAsync(ctx->d_path, ctx->d_path_all + first, sizeof(CamDev) * count,
                                    hipMemcpyDeviceToDevice, ctx->stream));
        return ERAY_OK;
    };
    // multi-camera builds on two streams: enqueued directly, chunk by chunk, not replayed from a
    // captured graph (the graph executor left the GPU idle for milliseconds after a path's first
    // builds; same-box A/B, scripts/ab_multi.sh: C5's frame 475-485 -> 468 us, 3840x2160 / 70k
    // 88-91 -> 57-58 us per moving frame)
    if (multi) {
        hipEvent_t ev[2] = {nullptr, nullptr};
        if (mean_frame_ms) {
            for (auto& e : ev) HIP_TRY(ctx, hipEventCreate(&e));
            HIP_TRY(ctx, hipEventRecord(ev[0], ctx->stream));
        }
        int st = ERAY_OK;
        for (uint32_t first = 0; first < n && !st; first += kGraphFrames) {
            const uint32_t count = std::min(kGraphFrames, n - first);
            st = before(first, count);
            for (uint32_t f = 0; f < count && !st; ++f) st = multi_frame(ctx->d_path, f, count, first + f);
        }
        if (!st) st = finish_union(ctx, psrc.key, psrc, nobj);
        if (!st) tag_frames(ctx, p.out_ppm, r.ppm, std::min(n, r.slots), psrc);
        if (mean_frame_ms && !st) {
            float ms = 0.0f;
            hipError_t e = hipEventRecord(ev[1], ctx->stream);
            if (e == hipSuccess) e = hipEventSynchronize(ev[1]);
            if (e == hipSuccess) e = hipEventElapsedTime(&ms, ev[0], ev[1]);
            if (e != hipSuccess) st = set_error(ctx, ERAY_E_HIP, "camera path timing: %s", hipGetErrorString(e));
            else *mean_frame_ms = ms / (float)n;
        }
        for (auto e : ev)
            if (e) hipEventDestroy(e);
        return st;
    }
    Plan plan;
    if (int st = ensure_plan(ctx, key, n, body, &plan)) return st;
    auto plain = [&](uint32_t f) { return frame((one_chunk ? ctx->d_path : ctx->d_path_all) + f, f); };
    int st = replay(ctx, plan, n, before, plain, mean_frame_ms);
    if (!st) st = finish_union(ctx, psrc.key, psrc, nobj);
    if (!st) tag_frames(ctx, p.out_ppm, r.ppm, std::min(n, r.slots), psrc);
    if (batched || multi) return st;  // (per-camera slots: the context's setup is still the scene camera's)
    // the device state now belongs to the path's last camera: the scene camera is set up again at
    // its next render (whose count copy also grows the bins' capacity when a camera needed more;
    // no copy here: waiting for an earlier one would wait for that call's frames)
    ctx->setup_key.clear();
    ctx->state_known = false;
    return st;
}

int eray_render_camera_path(eray_ctx* ctx, const eray_render_params* rp, const eray_camera* cameras, uint32_t n,
                            float* mean_frame_ms) {
    return eray_render_camera_path_ring(ctx, rp, nullptr, cameras, n, mean_frame_ms);
}

int eray_pack_ppm(eray_ctx* ctx, const float* rgb, uint32_t w, uint32_t h, uint8_t* out) {
    if (int st = use_device(ctx)) return st;
    if ((size_t)w * h && (!rgb || !out)) return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "null pointer");
    untag_range(ctx, reinterpret_cast<uintptr_t>(out), (size_t)w * h * 3u);
    HIP_TRY(ctx, launch_pack_ppm(rgb, w, h, out, ctx->stream));
    return ERAY_OK;
}

int eray_ppm_header(uint32_t w, uint32_t h, char* buf, size_t cap, size_t* len) {
    char tmp[64];
    int n = std::snprintf(tmp, sizeof tmp, "P6 %u %u %u\n", w, h, 255u);
    if (n < 0) return set_error(nullptr, ERAY_E_INVALID_ARGUMENT, "format failed");
    if (len) *len = (size_t)n;
    if (buf) {
        if (cap < (size_t)n + 1) return set_error(nullptr, ERAY_E_INVALID_ARGUMENT, "buffer too small");
        std::memcpy(buf, tmp, (size_t)n + 1);
    }
    return ERAY_OK;
}

}  // extern "C"

// The source of the n frames local + k * stride (k < n) as this context last rendered them
// (tag_frames); every frame must have the same one.
int eray_internal_frame_source(eray_ctx* ctx, const uint8_t* local, uint64_t stride, uint32_t n, FrameSource* out) {
    if (!ctx || !out) return ERAY_E_INVALID_ARGUMENT;
    *out = FrameSource{};
    for (uint32_t k = 0; k < n; ++k) {
        const uintptr_t a = reinterpret_cast<uintptr_t>(local) + (uintptr_t)(k * stride);
        const eray_ctx::SlotTag* t = nullptr;
        for (auto it = ctx->slot_tags.rbegin(); it != ctx->slot_tags.rend(); ++it)
            if (it->ppm == a) {
                t = &*it;
                break;
            }
        if (!t)
            return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "gather: frame %u at %p was not rendered by this context", k,
                             (const void*)a);
        if (k == 0) {
            *out = t->src;
        } else if (t->src.kind != out->kind || t->src.key != out->key) {
            return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "gather: frames 0 and %u come from different renders", k);
        }
    }
    if (out->kind == kSrcOther)
        return set_error(ctx, ERAY_E_INVALID_ARGUMENT,
                         "gather: the frames were rendered with anti-aliasing, bounces or brute force (no pixel rectangles)");
    return ERAY_OK;
}

// The pixel rectangles of `src` (waits for their host copy): the last scene-camera setup when it
// is src's (same camera, scene and rows), or the union of camera path src.key's cameras while it
// is among the last kUnionRing paths.
int eray_internal_source_layout(eray_ctx* ctx, const FrameSource& src, SceneLayout* out) {
    if (!ctx || !out) return ERAY_E_INVALID_ARGUMENT;
    auto same_rows = [](const FrameSource& a, const FrameSource& b) {
        return a.W == b.W && a.H == b.H && a.row0 == b.row0 && a.rows == b.rows && a.band_shift == b.band_shift &&
               a.band_stride == b.band_stride;
    };
    out->src = src;
    out->rects.clear();
    const size_t nobj = ctx->objects.size();
    if (src.kind == kSrcScene) {
        const FrameSource& s = ctx->setup_src;
        if (s.kind != kSrcScene || s.key != src.key || !same_rows(s, src))
            return set_error(ctx, ERAY_E_INVALID_ARGUMENT,
                             "gather: the scene camera's last setup is not the one these frames were rendered with");
        if (ctx->state_pending) {
            HIP_TRY(ctx, hipEventSynchronize(ctx->state_ev));
            state_arrived(ctx);
        }
        for (size_t i = 0; i < nobj; ++i) {
            const int32_t* r = ctx->h_objs_state[i].g.rect;
            out->rects.push_back({r[0], r[1], r[2], r[3]});
        }
        return ERAY_OK;
    }
    if (src.kind == kSrcPath) {
        const uint32_t e = (uint32_t)(src.key % kUnionRing);
        if (ctx->union_seq[e] != src.key || !same_rows(ctx->union_src[e], src))
            return set_error(ctx, ERAY_E_INVALID_ARGUMENT,
                             "gather: these camera-path frames are older than the last %u paths", kUnionRing);
        // (the union covers the objects of the scene the path was rendered from; a scene change
        // since makes the path's frames ungatherable, as their objects no longer exist)
        if (ctx->union_nobj[e] != nobj || ctx->union_gen[e] != ctx->scene_gen || nobj > ctx->union_cap)
            return set_error(ctx, ERAY_E_INVALID_ARGUMENT,
                             "gather: the scene changed after these camera-path frames were rendered");
        HIP_TRY(ctx, hipEventSynchronize(ctx->union_ev[e]));
        const int32_t* u = ctx->h_union + (size_t)e * 4 * ctx->union_cap;
        for (size_t i = 0; i < nobj; ++i)
            out->rects.push_back({u[2 * i], u[2 * nobj + 2 * i], u[2 * i + 1], u[2 * nobj + 2 * i + 1]});
        return ERAY_OK;
    }
    return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "gather: frames of an unknown source");
}
// The source of the scene camera's last setup (diagnostics: eray_debug_scene_gather).
int eray_internal_scene_setup_source(eray_ctx* ctx, FrameSource* out) {
    if (!ctx || !out) return ERAY_E_INVALID_ARGUMENT;
    if (ctx->setup_src.kind != kSrcScene)
        return set_error(ctx, ERAY_E_INVALID_ARGUMENT, "no setup of the scene camera: render it first");
    *out = ctx->setup_src;
    return ERAY_OK;
}
// The context's latest render of the scene camera or of a camera path (kind kSrcNone: none yet).
void eray_internal_gather_source(const eray_ctx* ctx, FrameSource* out) { *out = ctx->gather_src; }
// The context's collective scratch block (kCollScratchBytes of device memory, made with it).
uint8_t* eray_internal_coll_scratch(eray_ctx* ctx) { return ctx->d_coll; }
void** eray_internal_gather_plan(eray_ctx* ctx, void (*free_fn)(void*)) {
    ctx->gather_plan_free = free_fn;
    return &ctx->gather_plan;
}
int eray_internal_use_device(eray_ctx* ctx) { return use_device(ctx); }

// Error reporting and the gather's staging buffer for the other translation units (comm.cpp).
int eray_internal_error(eray_ctx* ctx, int code, const char* msg) { return set_error(ctx, code, "%s", msg); }
void eray_internal_untag(eray_ctx* ctx, const void* p, size_t bytes) {
    if (ctx && p) untag_range(ctx, reinterpret_cast<uintptr_t>(p), bytes);
}
void* eray_internal_staging(eray_ctx* ctx, size_t bytes) {
    if (!ctx) return nullptr;
    if (ensure(ctx, &ctx->d_staging, &ctx->staging_cap, bytes)) return nullptr;
    return ctx->d_staging;
}

// Diagnostics (not part of include/eray_hip.h): the screen bins of object `index` as built for
// the last setup — out[0] bins, out[1] entries, out[2] (face, pixel) pairs (mask bits),
// out[3] most entries in one bin, out[4] non-empty bins, out[5] most pairs in one bin,
// out[6..9] the object's pixel rectangle (x0, x1, y0, y1; int32 as uint64), out[10] the bin with
// the most entries, out[11] / out[12] the bins of more than 64 / kTraceHeavyMin entries, out[13]
// the units the pair pass walked: the faces' bin-rectangle rows (segments) or their (face, bin)
// pairs (the tracer's setups, eray_debug_set_bin_form) (out: 14 words).  Synchronises.
extern "C" int eray_debug_bin_stats(eray_ctx* ctx, uint32_t index, uint64_t* out) {
    if (!ctx || !out || index >= ctx->objects.size() || ctx->objects[index].T <= kDirectMax || !ctx->bins.start)
        return ERAY_E_INVALID_ARGUMENT;
    const BinBuffers& b = ctx->bins;
    uint32_t k = 0;
    for (uint32_t i = 0; i < index; ++i) k += ctx->objects[i].T > kDirectMax;
    std::vector<uint32_t> start(b.nbins + 1);
    ObjectDesc d{};
    if (hipStreamSynchronize(ctx->stream) != hipSuccess ||
        hipMemcpy(start.data(), b.start + (size_t)k * b.nbins, start.size() * 4, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&d, ctx->d_objs + index, sizeof d, hipMemcpyDeviceToHost) != hipSuccess)
        return set_error(ctx, ERAY_E_HIP, "bin stats copy failed");
    const size_t n = start[b.nbins] - start[0];
    std::vector<unsigned long long> mask(n);  // the entries' masks (a strided copy out of the 64-B entries)
    if (n && hipMemcpy2D(mask.data(), 8, reinterpret_cast<const char*>(b.ent + start[0]) + offsetof(BinEntry, mask),
                         sizeof(BinEntry), 8, n, hipMemcpyDeviceToHost) != hipSuccess)
        return set_error(ctx, ERAY_E_HIP, "bin stats copy failed");
    uint64_t pairs = 0, most = 0, nonempty = 0, most_pairs = 0, most_at = 0, over64 = 0, over192 = 0;
    for (size_t i = 0; i < b.nbins; ++i) {
        const uint64_t e = start[i + 1] - start[i];
        over64 += e > 64;
        over192 += e > kTraceHeavyMin;
        if (e > most) most_at = i;
        most = e > most ? e : most;
        nonempty += e != 0;
        uint64_t pb = 0;
        for (uint32_t j = start[i]; j < start[i + 1]; ++j) pb += (uint64_t)__builtin_popcountll(mask[j - start[0]]);
        pairs += pb;
        most_pairs = pb > most_pairs ? pb : most_pairs;
    }
    out[0] = b.nbins;
    out[1] = n;
    out[2] = pairs;
    out[3] = most;
    out[4] = nonempty;
    out[5] = most_pairs;
    for (int q = 0; q < 4; ++q) out[6 + q] = (uint64_t)(int64_t)d.g.rect[q];
    out[10] = most_at;
    out[11] = over64;
    out[12] = over192;
    // out[13]: the units of the faces' bin rectangles (every object)
    unsigned long long pairs_all = 0;
    if (hipMemcpy(&pairs_all, b.boff + setup_blocks(ctx->total_tris), sizeof pairs_all, hipMemcpyDeviceToHost) != hipSuccess)
        return set_error(ctx, ERAY_E_HIP, "bin stats copy failed");
    out[13] = pairs_all;
    return ERAY_OK;
}

// Diagnostics: the entries of bin `bin` of object `index` in bin order (faces relative to the
// object, pixel masks, pad words: a sorted bin's later-chunk mask unions, BinEntry), at most
// `cap`; *n = the bin's entry count; `pad` may be null.  Synchronises.
extern "C" int eray_debug_bin_entries(eray_ctx* ctx, uint32_t index, uint32_t bin, uint32_t* tri, uint64_t* mask,
                                      uint32_t* pad, uint32_t cap, uint32_t* n) {
    if (!ctx || !n || index >= ctx->objects.size() || ctx->objects[index].T <= kDirectMax || !ctx->bins.start ||
        bin >= ctx->bins.nbins)
        return ERAY_E_INVALID_ARGUMENT;
    const BinBuffers& b = ctx->bins;
    uint32_t k = 0;
    for (uint32_t i = 0; i < index; ++i) k += ctx->objects[i].T > kDirectMax;
    uint32_t se[2];
    if (hipStreamSynchronize(ctx->stream) != hipSuccess ||
        hipMemcpy(se, b.start + (size_t)k * b.nbins + bin, 8, hipMemcpyDeviceToHost) != hipSuccess)
        return set_error(ctx, ERAY_E_HIP, "bin dump copy failed");
    *n = se[1] - se[0];
    const uint32_t m = std::min(*n, cap);
    std::vector<BinEntry> ent(m);
    if (m && hipMemcpy(ent.data(), b.ent + se[0], sizeof(BinEntry) * (size_t)m, hipMemcpyDeviceToHost) != hipSuccess)
        return set_error(ctx, ERAY_E_HIP, "bin dump copy failed");
    for (uint32_t i = 0; i < m; ++i) {
        tri[i] = ent[i].tri;
        mask[i] = ent[i].mask;
        if (pad) pad[i] = ent[i].pad;
    }
    return ERAY_OK;
}

// Diagnostics: eray_debug_bin_entries without the pad words.
extern "C" int eray_debug_bin_dump(eray_ctx* ctx, uint32_t index, uint32_t bin, uint32_t* tri, uint64_t* mask,
                                   uint32_t cap, uint32_t* n) {
    return eray_debug_bin_entries(ctx, index, bin, tri, mask, nullptr, cap, n);
}

// Diagnostics: the entry count of every bin of object `index` (bins.nbins of them, row-major over
// the camera's bin rows, at most `cap`); *nbins = the object's bin count.  Synchronises.
extern "C" int eray_debug_bin_counts(eray_ctx* ctx, uint32_t index, uint32_t* counts, uint32_t cap, uint32_t* nbins) {
    if (!ctx || !nbins || index >= ctx->objects.size() || ctx->objects[index].T <= kDirectMax || !ctx->bins.start)
        return ERAY_E_INVALID_ARGUMENT;
    const BinBuffers& b = ctx->bins;
    uint32_t k = 0;
    for (uint32_t i = 0; i < index; ++i) k += ctx->objects[i].T > kDirectMax;
    *nbins = b.nbins;
    const uint32_t m = std::min(b.nbins, cap);
    std::vector<uint32_t> st((size_t)m + 1);
    if (hipStreamSynchronize(ctx->stream) != hipSuccess ||
        (m && hipMemcpy(st.data(), b.start + (size_t)k * b.nbins, sizeof(uint32_t) * ((size_t)m + 1),
                        hipMemcpyDeviceToHost) != hipSuccess))
        return set_error(ctx, ERAY_E_HIP, "bin counts copy failed");
    for (uint32_t i = 0; i < m; ++i) counts[i] = st[i + 1] - st[i];
    return ERAY_OK;
}

// Diagnostics (not part of include/eray_hip.h): the screen bins' entry capacity.  Setting it
// reallocates the bins at the next setup; a setup whose entries exceed it renders its binned
// objects through LDS tiles and the capacity grows once the host sees the count (tests).
extern "C" int eray_debug_set_bin_capacity(eray_ctx* ctx, uint64_t entries) {
    if (!ctx || !entries) return ERAY_E_INVALID_ARGUMENT;
    ctx->bin_cap = std::min((size_t)entries, kMaxBinEntries);
    ctx->setup_key.clear();
    return ERAY_OK;
}
extern "C" uint64_t eray_debug_bin_capacity(const eray_ctx* ctx) { return ctx ? (uint64_t)ctx->bins.cap : 0u; }
// Diagnostics: the frame setups' pair pass walks every (face, bin) pair of the faces' bin
// rectangles (rect_pairs != 0) instead of the rectangles' rows (bins.hip bin_segments_kernel);
// the next setup rebuilds the bins (tests compare the two forms' entries).
extern "C" int eray_debug_set_bin_form(eray_ctx* ctx, int rect_pairs) {
    if (!ctx) return ERAY_E_INVALID_ARGUMENT;
    ctx->rect_pairs = rect_pairs != 0;
    ctx->setup_key.clear();
    ctx->mc_layout.clear();
    return ERAY_OK;
}
// Diagnostics: the last setup's device state (CamState, 192 B) and object `index`'s pixel
// rectangle as the frame kernel reads them (synchronises).
extern "C" int eray_debug_setup_state(eray_ctx* ctx, uint32_t index, void* state_out, int32_t* rect_out) {
    if (!ctx || !state_out || !rect_out || index >= ctx->objects.size()) return ERAY_E_INVALID_ARGUMENT;
    ObjectDesc d{};
    if (hipStreamSynchronize(ctx->stream) != hipSuccess ||
        hipMemcpy(state_out, ctx->d_state, sizeof(CamState), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&d, ctx->d_objs + index, sizeof d, hipMemcpyDeviceToHost) != hipSuccess)
        return set_error(ctx, ERAY_E_HIP, "setup state copy failed");
    std::memcpy(rect_out, d.g.rect, sizeof d.g.rect);
    return ERAY_OK;
}
