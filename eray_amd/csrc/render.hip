// render.hip — the per-pixel ray-tracing hot path on gfx950 (CDNA4).
//
// Replaces Engine::render (src/lib/engine.rs:46-81) with the PPM byte pack of
// Image::save_as_ppm (src/lib/image.rs:48-74) fused in.  One thread per pixel; a 256-thread
// workgroup owns a 64x4 pixel tile and each 64-lane wave a 16x4 sub-tile; the tile's f32 RGB
// and PPM rows leave through LDS as 16-byte coalesced stores.
//
// First-hit search (Object::intersects, object.rs:58-81): the workgroup streams the object's
// triangles in index order through LDS in tiles of kTriTile records; each ray keeps the FIRST
// face (by index) whose Triangle::intersects (primitives.rs:41-72) passes — the reference's
// semantics, not the nearest hit.  The loop ends as soon as no ray of the workgroup is still
// searching (__syncthreads_or).
//
// Exact wave culling (primary rays only; disabled by ERAY_RENDER_BRUTE_FORCE).  For a camera
// ray the reference's test quantities are linear in the (unnormalised) ray direction, and the
// camera directions of a 16x4 pixel block span a small convex cone.  Per camera, each triangle
// gets four affine bounds f_k(x', y') of those quantities with float-error margins T_k
// (camera_setup_kernel in setup.hip, see the derivation there).  A wave evaluates them triangle-parallel —
// lane j takes triangle j of a 64-triangle chunk — and __ballot()s the survivors; only the
// survivors are tested ray-parallel, in index order, with the reference's exact arithmetic.
// The margins make the cull conservative: a triangle the exact test could accept for any ray
// of the block is never dropped, so results are identical to the brute-force scan
// (tests/test_render_gpu.py checks this bit-for-bit).
//
// Shadow rays (engine.rs:136-142, 218-228) go through the same LDS tiles without culling; the
// reference's degenerate bounding box rejects almost all of them before the scan.
#include <hip/hip_ext.h>

#include <mutex>

#include "cull_record.hpp"
#include "device_math.hpp"
#include "glibc_cosf.hpp"
#include "internal.hpp"
#include "hit.hpp"

// Per-workgroup timestamps for a diagnostics build (scripts/microbench/render_trace.hip defines
// it before including this file); nothing in the product build.
#ifndef ERAY_TRACE_POINT
#define ERAY_TRACE_POINT(k)
#define ERAY_TRACE_WAVE0(k)
#define ERAY_TRACE_VALUE(k, v)
#endif

namespace eray {
namespace gpu {
namespace {

using namespace eray::dev;

constexpr int kWG = 256;
constexpr int kTriTile = 256;

// Scene descriptors and triangle records are read-only for the whole frame: reading them
// through the constant address space lets wave-uniform reads become scalar (s_load) loads.
// Texture pointers come out of the descriptors: say they are global (no flat loads).
__device__ __forceinline__ const __attribute__((address_space(1))) float* as_global(const float* ptr) {
    return (const __attribute__((address_space(1))) float*)ptr;
}
template <typename T>
__device__ __forceinline__ T as_global_rec(const T* ptr) {  // per-lane record read, global
    static_assert(sizeof(T) % 16 == 0, "16-byte records only");
    using v4 = unsigned int __attribute__((ext_vector_type(4)));
    using gv4 = const __attribute__((address_space(1))) v4;
    gv4* src = (gv4*)ptr;
    T out;
    v4* dst = reinterpret_cast<v4*>(&out);
#pragma unroll
    for (size_t k = 0; k < sizeof(T) / 16; ++k) dst[k] = src[k];
    return out;
}

// Record `index` of a wave-uniform array by buffer loads: the array base lives in SGPRs (the
// buffer resource) and each lane only carries a 32-bit byte offset — no 64-bit per-lane address
// arithmetic or registers (arrays below 4 GB: triangle records, bin entries).
template <typename T>
__device__ __forceinline__ T load_rec(const T* base, uint32_t index) {
    static_assert(sizeof(T) % 16 == 0, "16-byte records only");
    using v4 = unsigned int __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(base), 0, -1, 0x00020000);
    T out;
    v4* dst = reinterpret_cast<v4*>(&out);
#pragma unroll
    for (uint32_t k = 0; k < sizeof(T) / 16; ++k)
        dst[k] = __builtin_amdgcn_raw_buffer_load_b128(r, index * (uint32_t)sizeof(T) + 16u * k, 0, 0);
    return out;
}

// --------------------------------------------------------------------- triangle setup ------
// Triangle::intersects recomputes e1 = b - a, e2 = c - a, n = e1 x e2 for every test
// (primitives.rs:44-46); they do not depend on the ray, so they are computed once here with
// the same f32 operations (bit-identical values).
__global__ void __launch_bounds__(256) tri_precompute_kernel(const float* __restrict__ pos,
                                                             const float* __restrict__ nrm,
                                                             const float* __restrict__ uv,
                                                             uint32_t T, TriHot* __restrict__ hot,
                                                             TriShade* __restrict__ shade) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= T) return;
    const float* P = pos + 9 * (size_t)i;
    f3 a = mk3(P[0], P[1], P[2]), b = mk3(P[3], P[4], P[5]), c = mk3(P[6], P[7], P[8]);
    f3 e1 = sub(b, a), e2 = sub(c, a);
    f3 n = cross(e1, e2);
    hot[i].q0 = make_float4(e1.x, e1.y, e1.z, e2.x);
    hot[i].q1 = make_float4(e2.y, e2.z, n.x, n.y);
    hot[i].q2 = make_float4(n.z, a.x, a.y, a.z);
    const float* N = nrm + 9 * (size_t)i;
    const float* U = uv + 6 * (size_t)i;
    shade[i].s0 = make_float4(N[0], N[1], N[2], N[3]);
    shade[i].s1 = make_float4(N[4], N[5], N[6], N[7]);
    shade[i].s2 = make_float4(N[8], U[0], U[1], U[2]);
    shade[i].s3 = make_float4(U[3], U[4], U[5], 0.0f);
}

struct Bundle {  // a wave's pixel rectangle in viewport coordinates
    float xlo, xhi, ylo, yhi;
};

// --------------------------------------------------------------------- scene views ---------
// Read paths of the frame's scene data (descriptors, lights, triangle records).
//  * SceneGlobal reads the device arrays; uniform reads go through the constant address
//    space and become scalar loads.
//  * SceneLds reads a copy of the whole scene that each workgroup preloads into LDS in one
//    round trip (small scenes: kCacheTris triangles, kCacheObjects objects, kCacheLights
//    lights).  Uniform reads are LDS broadcasts moved to SGPRs with readfirstlane.
// Either way one instantiation touches one address space (no generic "flat" loads).
template <typename T>
__device__ __forceinline__ T lds_uniform(const T* ptr) {
    static_assert(sizeof(T) % 4 == 0, "dword-sized records only");
    T out;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(ptr);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&out);
#pragma unroll
    for (size_t k = 0; k < sizeof(T) / 4; ++k) dst[k] = __builtin_amdgcn_readfirstlane(src[k]);
    return out;
}

// The frame kernel's first reads, passed as leading scalar kernel arguments: the compiler
// preloads them into SGPRs (-amdgpu-kernarg-preload-count, build.py), so the scene preload's
// loads issue without a kernel-argument round trip first.
struct FrameHot {
    const ObjectDesc* objects;
    const LightDesc* lights;
    const TriCull* cull;
    const TriHot* tris;
    const TriShade* shade;
    uint32_t counts;      // nobj | nlights << 16
    uint32_t total_tris;
    uint32_t total_sub;   // detail sub-blocks
    uint32_t grid;        // workgroups launched
};

struct SceneGlobal {
    const FrameParams& p;
    const ObjectDesc* objects;  // the frame's descriptors and culling records (a batched camera
    const TriCull* culls;       // setup's slot: FrameParams::dev_slots)
    __device__ ObjGeom geom(uint32_t i) const { return load_const(&objects[i].g, 0); }
    __device__ const ObjGeom* geom_ptr(uint32_t i) const { return &objects[i].g; }
    __device__ MaterialDesc mat(uint32_t i) const { return load_const(&objects[i].mat, 0); }
    __device__ LightDesc light(uint32_t i) const { return load_const(p.lights, i); }
    __device__ TriCull cull(uint32_t g) const { return culls[g]; }          // per lane
    __device__ const TriCull* cull_array() const { return culls; }
    __device__ TriHot hot(uint32_t g) const { return load_const(p.tris, g); }  // uniform
    __device__ TriHot hot_lane(uint32_t g) const { return load_rec(p.tris, g); }  // per lane
    __device__ TriShade shade(uint32_t g) const { return load_rec(p.shade, g); }  // per lane
};

struct SceneLds {
    const ObjectDesc* objs;
    const LightDesc* lights;
    const TriCull* culls;
    const TriHot* hots;
    const TriShade* shades;
    const ObjectDesc* g_objs;  // the device arrays (scalar loads of uniform records)
    const LightDesc* g_lights;
    const TriHot* g_tris;
    const TriCull* g_cull;
    // Wave-uniform records (objects, materials, lights) by scalar loads from the device arrays,
    // not LDS reads + readfirstlane: C2 8.67 -> 8.40 us per frame (profiles/ab/ab_c2chain.log),
    // though one wave's chain alone is 0.2 us longer (7.26 -> 7.44 us, a 4-row frame).
    __device__ ObjGeom geom(uint32_t i) const { return load_const(&g_objs[i].g, 0); }
    __device__ const ObjGeom* geom_ptr(uint32_t i) const { return &g_objs[i].g; }
    __device__ MaterialDesc mat(uint32_t i) const { return load_const(&g_objs[i].mat, 0); }
    __device__ LightDesc light(uint32_t i) const { return load_const(g_lights, i); }
    __device__ TriCull cull(uint32_t g) const { return culls[g]; }
    __device__ const TriCull* cull_array() const { return g_cull; }
    __device__ TriHot hot(uint32_t g) const { return hots[g]; }  // broadcast read (VGPRs)
    __device__ TriHot hot_lane(uint32_t g) const { return hots[g]; }
    __device__ TriShade shade(uint32_t g) const { return shades[g]; }
};

// Copies the scene into LDS (layout: scene_lds_layout, internal.hpp): every 16-byte word is
// loaded before any is stored, four per thread per pass, so a small scene costs one round trip.
// `meanwhile()` runs once while the first pass's loads are in flight.
template <typename Meanwhile>
__device__ SceneLds preload_scene(const FrameHot& p, char* dyn, Meanwhile&& meanwhile) {
    const SceneLdsLayout L = scene_lds_layout(p.counts & 0xffffu, p.counts >> 16, p.total_tris, p.cull != nullptr);
    const uint32_t n_obj = L.lights / 16, n_light = (L.cull - L.lights) / 16;
    const uint32_t n_cull = (L.hot - L.cull) / 16, n_hot = (L.shade - L.hot) / 16;
    const uint32_t total = L.bytes / 16;
    using v4 = unsigned int __attribute__((ext_vector_type(4)));
    using gv4 = const __attribute__((address_space(1))) v4;
    gv4* src_obj = (gv4*)p.objects;
    gv4* src_light = (gv4*)p.lights;
    gv4* src_cull = (gv4*)p.cull;
    gv4* src_hot = (gv4*)p.tris;
    gv4* src_shade = (gv4*)p.shade;
    v4* dst = reinterpret_cast<v4*>(dyn);
    for (uint32_t base = 0; base < total; base += 4 * kWG) {
        v4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // branch-free (clamped index): the loads issue back to back
            const uint32_t i = min(base + k * kWG + threadIdx.x, total - 1);
            const uint32_t i1 = i - n_obj, i2 = i1 - n_light, i3 = i2 - n_cull, i4 = i3 - n_hot;
            gv4* src = i < n_obj ? src_obj + i
                     : i1 < n_light ? src_light + i1
                     : i2 < n_cull ? src_cull + i2
                     : i3 < n_hot ? src_hot + i3
                     : src_shade + i4;
            v[k] = *src;
        }
        if (base == 0) {
            meanwhile();
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t i = base + k * kWG + threadIdx.x;
            if (i < total) dst[i] = v[k];
        }
    }
    return SceneLds{reinterpret_cast<const ObjectDesc*>(dyn + L.objs), reinterpret_cast<const LightDesc*>(dyn + L.lights),
                    reinterpret_cast<const TriCull*>(dyn + L.cull), reinterpret_cast<const TriHot*>(dyn + L.hot),
                    reinterpret_cast<const TriShade*>(dyn + L.shade), p.objects, p.lights, p.tris, p.cull};
}

// A word of a read-only array through the vector memory path (buffer load; every lane the same
// address): its wait counts with the wave's vector loads (vmcnt, in order), not with its LDS
// operations (lgkmcnt, which an outstanding scalar load would hold up) — for loads issued one
// sub-block ahead and used in the next.
__device__ __forceinline__ uint32_t vload_u32(const uint32_t* base, uint32_t i) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(base), 0, -1, 0x00020000);
    return __builtin_amdgcn_raw_buffer_load_b32(r, 4u * i, 0, 0);
}

// A bin range [lo, hi) loaded ahead (render_sub's pipelining), or none (ok false).
struct PreRange {
    uint32_t lo, hi;
    bool ok;
};

// Lanes whose Triangle::intersects could pass: the det and t conditions of exact_test, from the
// same expressions (so the same values).  t = dot(ao, n) * (1 / det) is >= 0 exactly when
// dot(ao, n) >= 0, except where the product underflows to -0 or 1 / det is 0 — those lanes are
// kept.  A lane that fails here fails the exact test; a face no lane keeps is skipped.
__device__ __forceinline__ bool plane_may_hit(f3 n, f3 a, f3 o, f3 d) {
    const float det = -dot0(d, n);
    const float dn = dot0(sub(o, a), n);
    return (det >= 1e-6f) & !((dn < -1e-18f) & (det < 1e19f));
}

// Faces [0, n) (n <= 64; lane j holds face j's record) that some searching lane may hit
// (plane_may_hit), as a bit mask.  The planes are broadcast from the lanes that hold them, four
// faces per step.
__device__ __forceinline__ unsigned long long plane_mask(const TriHot& mine, uint32_t n, bool searching, f3 o, f3 d) {
    const float pn[6] = {mine.q1.z, mine.q1.w, mine.q2.x, mine.q2.y, mine.q2.z, mine.q2.w};
    unsigned long long mask = 0;
    for (uint32_t i = 0; i < n; i += 4) {
        bool keep[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            const uint32_t f = min(i + k, n - 1);
            const f3 nn = mk3(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(pn[0]), f)),
                              __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pn[1]), f)),
                              __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pn[2]), f)));
            const f3 a = mk3(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(pn[3]), f)),
                             __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pn[4]), f)),
                             __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pn[5]), f)));
            keep[k] = searching && plane_may_hit(nn, a, o, d);
        }
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k)
            if (i + k < n && __any(keep[k])) mask |= 1ull << (i + k);
    }
    return mask;
}

// --------------------------------------------------------------------- first hit -----------
// Per-ray search state: kUndecided (ray and bounding-box test not evaluated yet), kSearching,
// kDone (hit found, bbox rejected, or not a pixel of the image).
constexpr int kUndecided = 0, kSearching = 1, kDone = 2;

// Objects with at most kDirectMax (internal.hpp) triangles are searched by each wave on its
// own (no LDS tiles, no barrier); larger ones through their screen bins (primary rays, culled)
// or workgroup-shared LDS tiles (shadow rays, brute force).
// Candidate triangles tested together per step (independent, branch-free tests: their long
// dependent chains, division included, overlap).
constexpr int kBatch = 4;
constexpr int kLargeTestBatch = 1;  // the large-mesh builds: one candidate per step (no spills)

// Tests the next kB candidates of `mask` (kB <= its population) in index order.
template <int kB, typename Face, typename Hot>
__device__ __forceinline__ void test_step(unsigned long long& mask, Face&& face, Hot&& hot, int& st, const f3& o,
                                          const f3& d, int& found, float& hu, float& hv, float& ht) {
    uint32_t ids[kB];
    bool has[kB];
    TriHot h[kB];
#pragma unroll
    for (int k = 0; k < kB; ++k) {
        has[k] = mask != 0;
        ids[k] = has[k] ? (uint32_t)(__ffsll(mask) - 1) : 0u;
        mask &= mask - 1;
        h[k] = hot(ids[k]);
    }
    bool hit[kB];
    float u[kB], v[kB], t[kB];
#pragma unroll
    for (int k = 0; k < kB; ++k) hit[k] = has[k] && exact_test_flat(h[k], o, d, u[k], v[k], t[k]);
#pragma unroll
    for (int k = 0; k < kB; ++k) {
        if (st == kSearching && hit[k]) {
            found = (int)face(ids[k]);
            hu = u[k];
            hv = v[k];
            ht = t[k];
            st = kDone;
        }
    }
}

// Tests the candidates of `mask` in index order, up to kBatch at a time: bit i stands for face
// face(i) (relative to the object) whose record is hot(i).  Returns false once no lane is
// searching.
template <int kB = kBatch, typename Face, typename Hot>
__device__ __forceinline__ bool test_candidates(unsigned long long mask, Face&& face, Hot&& hot, int& st,
                                                const f3& o, const f3& d, int& found, float& hu, float& hv,
                                                float& ht) {
    while (mask) {
        const int n = __popcll(mask);
        if (kB >= 4 && n >= 4)
            test_step<4>(mask, face, hot, st, o, d, found, hu, hv, ht);
        else if (kB >= 2 && n >= 2)
            test_step<2>(mask, face, hot, st, o, d, found, hu, hv, ht);
        else
            test_step<1>(mask, face, hot, st, o, d, found, hu, hv, ht);
        if (!__any(st == kSearching)) return false;
    }
    return true;
}

// First-hit search over triangles [begin, begin + count) (Object::intersects' face loop,
// object.rs:63-78).  A ray still kUndecided when the wave meets its first candidate triangle is
// resolved by activate(), which must generate its direction (into `d`) and return the
// bounding-box verdict (object.rs:59-61).  `found` receives the face index relative to
// `begin`, or stays -1.  kLds: every thread of the workgroup must call it.
template <bool kCull, bool kLds, bool kPlane = false, int kB = kBatch, typename Scene, typename Activate>
__device__ void first_hit(const FrameParams& p, const Scene& sc, uint32_t begin, uint32_t count, int& st,
                          const f3& o, const f3& d, const Bundle& bd, TriHot* s_hot, TriCull* s_cull,
                          Activate&& activate, int& found, float& hu, float& hv, float& ht) {
    const uint32_t lane = threadIdx.x & 63;
    // false when no ray of the wave can hit anything in this object any more
    auto resolve = [&]() -> bool {
        if (__any(st == kUndecided)) {
            const bool a = activate();
            if (st == kUndecided) st = a ? kSearching : kDone;
        }
        return __any(st == kSearching);
    };
    if (!kLds) {
        for (uint32_t base = 0; base < count; base += 64) {
            if (!__any(st != kDone)) break;
            unsigned long long mask;
            if (kCull) {
                const uint32_t j = base + lane;
                bool keep = false;
                if (j < count) keep = !cull_rejects(sc.cull(begin + j), bd.xlo, bd.xhi, bd.ylo, bd.yhi);
                mask = __ballot(keep);
            } else if (kPlane) {  // rays already resolved (shadow rays): faces some lane may hit
                const uint32_t n = min(64u, count - base);
                mask = plane_mask(sc.hot_lane(begin + base + min(lane, n - 1)), n, st == kSearching, o, d);
            } else {
                const uint32_t n = min(64u, count - base);
                mask = n == 64 ? ~0ull : ((1ull << n) - 1ull);
            }
            if (!mask) continue;
            if (!resolve()) break;
            auto face = [&](uint32_t i) { return base + i; };
            auto hot = [&](uint32_t i) { return sc.hot(begin + base + i); };
            if (!test_candidates<kB>(mask, face, hot, st, o, d, found, hu, hv, ht)) return;
        }
        return;
    }
    for (uint32_t base = 0; base < count; base += kTriTile) {
        if (!__syncthreads_or(st != kDone)) break;  // also orders the LDS reuse below
        const uint32_t n = min((uint32_t)kTriTile, count - base);
        if (threadIdx.x < n) {
            s_hot[threadIdx.x] = p.tris[begin + base + threadIdx.x];
            if (kCull) s_cull[threadIdx.x] = sc.cull_array()[begin + base + threadIdx.x];
        }
        __syncthreads();
        if (!__any(st != kDone)) continue;
        for (uint32_t c = 0; c < n; c += 64) {
            unsigned long long mask;
            if (kCull) {
                const uint32_t j = c + lane;
                mask = __ballot(j < n && !cull_rejects(s_cull[j], bd.xlo, bd.xhi, bd.ylo, bd.yhi));
            } else {
                const uint32_t m = min(64u, n - c);
                mask = m == 64 ? ~0ull : ((1ull << m) - 1ull);
            }
            if (!mask) continue;
            if (!resolve()) break;
            auto face = [&](uint32_t i) { return base + c + i; };
            auto hot = [&](uint32_t i) { return s_hot[c + i]; };
            if (!test_candidates<kB>(mask, face, hot, st, o, d, found, hu, hv, ht)) break;
        }
    }
    __syncthreads();  // the tiles' LDS is reused (aliased by the binned search)
}

constexpr uint32_t kBlkW = 64, kBlkH = 4;  // pixel block
constexpr uint32_t kSubW = 16;             // sub-block width (x kBlkH rows): one wave's pixels
static_assert(kSubW == kBinW && kBlkH == kBinH, "a screen bin is one wave's sub-block");

constexpr uint32_t kWide = 16;  // candidates that may cover more pixels are tested by the whole wave

// Per-wave LDS of the binned primary search.
struct BinLds {
    float dir[3][64];         // each pixel's camera ray (lane = pixel)
    // each pixel's first hit so far as an order key, 0xffffffff = none: its bin position in a
    // sorted bin (positions grow with the face index), its face index in a longer one
    uint32_t best[64];
    TriHot cand[64];          // the chunk's candidate records (slot = lane that loaded it)
    uint32_t key[64];         // ... and their order keys
    // (candidate slot << 6) | pixel, for every pixel a narrow candidate (<= kWide pixels) may hit
    uint16_t pairs[64 * kWide];
};
constexpr uint32_t kBinLdsBytes = (sizeof(BinLds) + 15) / 16 * 16;

// Primary-ray first hit of a binned object (bins.hip), all four waves of the workgroup together
// (every wave calls it; workgroup-uniform).  The reference's first hit is the smallest face index
// whose Triangle::intersects passes (object.rs:63-78), so each pixel keeps the smallest hitting
// face seen so far (LDS atomicMin of an order key).  A bin of 65 to kBinSortMax entries lists its
// faces in index order (bins.hip sort_bins): the key is the bin position, and a chunk none of
// whose pixels is still without a hit before the chunk's first position is skipped before its
// entries are read.  Other bins are in no particular order (one chunk, or too long to sort): the
// key is the face index, and a chunk is skipped when every pixel's best face is below the
// chunk's smallest.  Each wave's
// sub-block bin is cut into chunks of 64 entries and the workgroup's chunks are dealt round-robin
// over its waves — a bin at a dense spot (thousands of faces) is shared four ways.  A chunk is
// tested as (face, pixel) pairs: each entry carries the pixels where its four culling bounds can
// pass (bin_pixels), restricted to the live pixels; narrow faces' pairs are compacted in LDS and
// tested one per lane, wide ones by the whole wave, and a pair whose key is not below the pixel's
// best so far is skipped.
// Work follows the pixels a face can cover, not 64 lanes per face.  Each wave then re-tests its
// pixels' winners for u, v, t.
template <typename Activate>
__device__ void first_hit_binned(const FrameParams& p, const ObjGeom& ob, uint32_t bin, int& st, const f3& o,
                                 const f3& d, Activate&& activate, int& found, float& hu, float& hv, float& ht,
                                 char* s_bins, PreRange pre) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr uint32_t kWaves = kWG / 64;
    BinLds& L = *reinterpret_cast<BinLds*>(s_bins + wave * kBinLdsBytes);
    uint32_t* s_range = reinterpret_cast<uint32_t*>(s_bins + kWaves * kBinLdsBytes);  // [lo, hi] per wave
    // the bin's entries [lo, hi): loaded one sub-block ahead when the caller has them (pre)
    uint32_t lo = pre.ok ? pre.lo : load_const(ob.bin_start, bin), hi = pre.ok ? pre.hi : load_const(ob.bin_start, bin + 1);
    if (lo != hi && __any(st == kUndecided)) {  // every pixel's ray and bbox verdict, up front
        const bool a = activate();
        if (st == kUndecided) st = a ? kSearching : kDone;
    }
    if (!__any(st == kSearching)) hi = lo;  // nothing to search in this sub-block
    ERAY_TRACE_WAVE0(8);
    L.dir[0][lane] = d.x;
    L.dir[1][lane] = d.y;
    L.dir[2][lane] = d.z;
    L.best[lane] = st == kSearching ? 0xffffffffu : 0u;  // 0: never improved
    if (lane == 0) {
        s_range[2 * wave] = lo;
        s_range[2 * wave + 1] = hi;
    }
    __syncthreads();
    ERAY_TRACE_WAVE0(9);
    uint32_t chunks[kWaves], total = 0;
#pragma unroll
    for (uint32_t w = 0; w < kWaves; ++w) {
        chunks[w] = (s_range[2 * w + 1] - s_range[2 * w] + 63) / 64;
        total += chunks[w];
    }
    for (uint32_t item = wave; item < total; item += kWaves) {  // this wave's chunks
        uint32_t w = 0, c = item;
        while (c >= chunks[w]) c -= chunks[w++];
        BinLds& T = *reinterpret_cast<BinLds*>(s_bins + w * kBinLdsBytes);  // the chunk's sub-block
        const uint32_t lo_w = s_range[2 * w], end = s_range[2 * w + 1];
        const uint32_t base = lo_w + 64 * c;
        const bool sorted = end - lo_w > 64 && end - lo_w <= kBinSortMax;  // workgroup-uniform
        const uint32_t j = base + lane;
        uint32_t fj = 0xffffffffu;  // the entry's order key
        unsigned long long pm = 0;
        unsigned long long live;  // pixels of that sub-block this chunk can still improve
        if (sorted) {
            live = __ballot(T.best[lane] > base);
            if (!live) continue;
            if (j < end) {
                const BinEntry x = as_global_rec(ob.bin_ent + j);  // (one 64-B line per entry)
                fj = j;
                pm = x.mask;
                L.cand[lane] = x.hot;
                L.key[lane] = j;
            }
        } else {
            if (j < end) {
                const BinEntry x = as_global_rec(ob.bin_ent + j);
                fj = x.tri;
                pm = x.mask;
                L.cand[lane] = x.hot;
                L.key[lane] = fj;
            }
            uint32_t cmin = fj;  // the chunk's smallest face
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) cmin = min(cmin, (uint32_t)__shfl_xor((int)cmin, off));
            live = __ballot(T.best[lane] > cmin);
            if (!live) continue;
        }
        const unsigned long long pix = pm & live;  // live pixels this face may hit
        const uint32_t cnt = (uint32_t)__popcll(pix);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // L.cand / L.key of this chunk visible to the wave
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // wide candidates (many pixels): the whole wave tests them, each lane its own pixel
        unsigned long long wide = __ballot(cnt > kWide);
        while (wide) {
            const uint32_t s = (uint32_t)(__ffsll(wide) - 1);
            wide &= wide - 1;
            const unsigned long long ps =
                ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(pix >> 32), (int)s) << 32) |
                (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)pix, (int)s);
            const uint32_t fc = (uint32_t)__builtin_amdgcn_readlane((int)fj, (int)s);
            if (((ps >> lane) & 1ull) && fc < T.best[lane]) {
                float u, v, t;
                const f3 dd = mk3(T.dir[0][lane], T.dir[1][lane], T.dir[2][lane]);
                if (exact_test(L.cand[s], o, dd, u, v, t)) atomicMin(&T.best[lane], fc);
            }
        }
        // narrow candidates: (candidate, pixel) pairs compacted in LDS, one test per lane
        const uint32_t ncnt = cnt > kWide ? 0u : cnt;
        uint32_t incl = ncnt;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off);
            if ((int)lane >= off) incl += y;
        }
        const uint32_t npairs = __shfl(incl, 63);
        uint32_t at = incl - ncnt;
        unsigned long long np = ncnt ? pix : 0ull;
        while (np) {
            const uint32_t bpos = (uint32_t)(__ffsll(np) - 1);
            np &= np - 1;
            L.pairs[at++] = (uint16_t)((lane << 6) | bpos);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t q = 0; q < npairs; q += 64) {
            if (q + lane < npairs) {
                const uint32_t pr = L.pairs[q + lane];
                const uint32_t slot = pr >> 6, px = pr & 63;
                const uint32_t fc = L.key[slot];
                if (fc < T.best[px]) {  // a pixel already hit by an earlier face needs no test
                    float u, v, t;
                    const f3 dd = mk3(T.dir[0][px], T.dir[1][px], T.dir[2][px]);
                    if (exact_test(L.cand[slot], o, dd, u, v, t)) atomicMin(&T.best[px], fc);
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // L.cand / L.key / L.pairs are rewritten by the next chunk
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    ERAY_TRACE_WAVE0(10);
    __syncthreads();  // every chunk of every sub-block is done
    ERAY_TRACE_WAVE0(11);
    const uint32_t mine = L.best[lane];
    if (st == kSearching && mine != 0xffffffffu) {
        float u, v, t;
        if (hi - lo > 64 && hi - lo <= kBinSortMax) {  // the winner again, for u, v, t
            const BinEntry x = as_global_rec(ob.bin_ent + mine);
            exact_test(x.hot, o, d, u, v, t);
            found = (int)x.tri;
        } else {
            exact_test(as_global_rec(p.tris + ob.tri_begin + mine), o, d, u, v, t);
            found = (int)mine;
        }
        hu = u;
        hv = v;
        ht = t;
        st = kDone;
    }
    ERAY_TRACE_WAVE0(12);
    __syncthreads();  // the LDS is reused by the next object / sub-block
}

// Faces of an object the per-wave binned search takes (its keys pack face << 6 | slot).
constexpr uint32_t kWaveBinMaxTris = (1u << 26) - 1u;

// Primary-ray first hit of a binned object by ONE wave over its own sub-block's bin, with no
// workgroup barrier (the light sub-blocks of a frame's ordered detail list: their bins hold at
// most one 64-entry chunk, so sharing chunks across the workgroup's waves, as first_hit_binned
// does, buys nothing and its barriers tie four sub-blocks' latency chains together).  The same
// (face, pixel) pair tests; each pixel keeps the smallest order key of a hitting pair (LDS
// atomicMin), so the smallest hitting face index wins (object.rs:63-78) and its record is still
// in the wave's LDS: the winner's u, v, t are recomputed from there after each chunk, not re-read
// from memory.  Keys: face << 6 | slot in a bin in no order; in a sorted bin (65..kBinSortMax
// entries, bins.hip bin_sort_kernel) the position, which grows with the face index — a pixel
// whose best position precedes a chunk cannot improve there, and after each chunk the bin ends
// once no pixel that still can is in the later chunks' mask union (BinEntry::pad): a heavy bin's
// wave stops at the chunk that settles its last pixel, not at the bin's end.
template <typename Activate>
__device__ void first_hit_binned_wave(const ObjGeom& ob, uint32_t bin, int& st, const f3& o, const f3& d,
                                      Activate&& activate, int& found, float& hu, float& hv, float& ht, char* s_bins,
                                      PreRange pre) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    BinLds& L = *reinterpret_cast<BinLds*>(s_bins + wave * kBinLdsBytes);
    const uint32_t lo = pre.ok ? pre.lo : load_const(ob.bin_start, bin), hi = pre.ok ? pre.hi : load_const(ob.bin_start, bin + 1);
    if (lo == hi) return;
    if (__any(st == kUndecided)) {  // every pixel's ray and bbox verdict, up front
        const bool a = activate();
        if (st == kUndecided) st = a ? kSearching : kDone;
    }
    ERAY_TRACE_WAVE0(8);
    if (!__any(st == kSearching)) return;
    L.dir[0][lane] = d.x;
    L.dir[1][lane] = d.y;
    L.dir[2][lane] = d.z;
    uint32_t best = st == kSearching ? 0xffffffffu : 0u;  // this lane's pixel: its winning key so far
    L.best[lane] = best;
    const bool sorted = hi - lo > 64 && hi - lo <= kBinSortMax;  // (wave-uniform)
    for (uint32_t base = lo; base < hi; base += 64) {
        const uint32_t j = base + lane;
        uint32_t fj = 0xffffffffu, sfx = 0;
        unsigned long long pm = 0;
        if (j < hi) {
            const BinEntry x = load_rec(ob.bin_ent, j);
            fj = x.tri;
            pm = x.mask;
            sfx = x.pad;
            L.cand[lane] = x.hot;
        }
        unsigned long long live;  // pixels this chunk can still improve
        uint32_t key;
        if (sorted) {
            live = __ballot(best > base - lo);
            if (!live) break;  // (and none in any later chunk)
            key = j - lo;
        } else {
            uint32_t cmin = fj;  // the chunk's smallest face
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) cmin = min(cmin, (uint32_t)__shfl_xor((int)cmin, off));
            live = __ballot((best >> 6) > cmin);
            if (!live) continue;
            key = (fj << 6) | lane;
        }
        ERAY_TRACE_WAVE0(9);
        const unsigned long long pix = pm & live;
        const uint32_t cnt = (uint32_t)__popcll(pix);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // L.cand / L.dir / L.best visible to the wave
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        unsigned long long wide = __ballot(cnt > kWide);
        while (wide) {  // wide candidates: the whole wave tests them, each lane its own pixel
            const uint32_t sl = (uint32_t)(__ffsll(wide) - 1);
            wide &= wide - 1;
            const unsigned long long ps =
                ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(pix >> 32), (int)sl) << 32) |
                (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)pix, (int)sl);
            const uint32_t kc = (uint32_t)__builtin_amdgcn_readlane((int)key, (int)sl);
            if (((ps >> lane) & 1ull) && kc < L.best[lane]) {
                float u, v, t;
                if (exact_test(L.cand[sl], o, d, u, v, t)) atomicMin(&L.best[lane], kc);
            }
        }
        // narrow candidates: (candidate, pixel) pairs compacted in LDS, one test per lane
        const uint32_t ncnt = cnt > kWide ? 0u : cnt;
        uint32_t incl = ncnt;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off);
            if ((int)lane >= off) incl += y;
        }
        const uint32_t npairs = __shfl(incl, 63);
        uint32_t at = incl - ncnt;
        unsigned long long np = ncnt ? pix : 0ull;
        while (np) {
            const uint32_t bpos = (uint32_t)(__ffsll(np) - 1);
            np &= np - 1;
            L.pairs[at++] = (uint16_t)((lane << 6) | bpos);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t q = 0; q < npairs; q += 64) {
            const bool in = q + lane < npairs;
            const uint32_t pr = in ? L.pairs[q + lane] : 0u;
            const uint32_t sl = pr >> 6, px = pr & 63;
            const uint32_t kc = (uint32_t)__shfl((int)key, (int)sl);  // the pair's key, from the lane that loaded it
            if (in && kc < L.best[px]) {  // a pixel already hit by an earlier face needs no test
                float u, v, t;
                const f3 dd = mk3(L.dir[0][px], L.dir[1][px], L.dir[2][px]);
                if (exact_test(L.cand[sl], o, dd, u, v, t)) atomicMin(&L.best[px], kc);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // every pair of the chunk tested
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t nb = L.best[lane];
        const uint32_t fwin = sorted ? (uint32_t)__shfl((int)fj, (int)(nb & 63u)) : nb >> 6;  // its face
        if (nb != best) {  // improved by this chunk: the winner's record is still L.cand[slot]
            best = nb;
            exact_test(L.cand[nb & 63u], o, d, hu, hv, ht);
            found = (int)fwin;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // L.cand / L.pairs are rewritten by the next chunk
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (sorted) {  // the later chunks' masks (this chunk's first two entries): anything left?
            const unsigned long long later = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)sfx, 1) << 32) |
                                             (uint32_t)__builtin_amdgcn_readlane((int)sfx, 0);
            if (!(__ballot(best > base + 64 - lo) & later)) break;
        }
    }
    ERAY_TRACE_WAVE0(10);
    ERAY_TRACE_VALUE(15, (hi - lo + 63) / 64);
    if (st == kSearching && found >= 0) st = kDone;
}

__device__ const float g_texel_dummy[4] = {0.0f, 0.0f, 0.0f, 0.0f};

// The frame's camera: the kernel arguments, or the setup kernel's copy in device-camera mode
// (FrameParams::cam_state; wave-uniform, scalar loads).
template <bool kDev>
__device__ __forceinline__ CamDev frame_camera(const FrameParams& p, const CamState* cs) {
    if (kDev) return load_const(&cs->cam, 0);
    return CamDev{p.cx, p.cy, p.cz, p.ratio, p.z_dist, {0u, 0u, 0u}};
}

// Camera::pixel_to_ray(x / W, y / H).dir (engine.rs:100-109, camera.rs:57-76, Ray::new)
__device__ __forceinline__ f3 camera_dir(const CamDev& cam, const FrameParams& p, uint32_t px, uint32_t y) {
    const f3 C = mk3(cam.cx, cam.cy, cam.cz);
    const float xf = (float)px / (float)p.cam_w;
    const float yf = (float)y / (float)p.cam_h;
    const float vw = cam.ratio * 2.0f;
    const f3 horizontal = mk3(vw, 0.0f, 0.0f), vertical = mk3(0.0f, 2.0f, 0.0f);
    const f3 botleft = sub(sub(sub(C, divs(horizontal, 2.0f)), divs(vertical, 2.0f)),
                           mk3(0.0f, 0.0f, cam.z_dist));
    return normalize(sub(add(add(botleft, mul(horizontal, xf)), mul(vertical, yf)), C));
}

// ---------------------------------------------------------------------- frame kernel -------
// The image (rank-local rows) is cut into 64 x 4 pixel blocks of four 16 x 4 sub-blocks.  A
// sub-block inside one of the frame's detail rectangles (FrameParams::rects: the objects' pixel
// rectangles, ObjectDesc::rect, in sub-block units) is "detail": one wave runs Engine::cast_ray
// for its 64 pixels, one pixel per lane.  Every other sub-block is background
// (engine.rs:211-213) with no test at all.  One persistent launch does both:
//  * detail: the detail sub-blocks are enumerated rectangle by rectangle (the host makes the
//    rectangles disjoint) and dealt out round-robin over the first
//    workgroups, four consecutive ones per workgroup, so the latency-bound shading is spread
//    over all CUs instead of clustering on the CUs that own the object's screen region;
//  * fill: the remaining workgroups stride over the 64 x 4 blocks and write the background of
//    the non-detail sub-blocks — a whole block as 3 + 1 + 1 wave-contiguous 16-byte stores.
//    This is the frame's HBM-write floor.  Keeping it off the detail workgroups matters: their
//    loads must not wait behind their own stores (a CDNA wave's vmcnt counts both).

// Rank-local row -> camera row (interleaved bands or a contiguous block), from the frame kernel's
// band word (h_band: shift | stride << 5) and row0.
struct RowMap {
    uint32_t row0, shift, stride;
};
__device__ __forceinline__ uint32_t cam_row(const RowMap& m, uint32_t j) {
    return band_camera_row(m.row0, m.shift, 0xffffffffu >> (32u - m.shift), m.stride, j);
}

__device__ __forceinline__ Bundle make_bundle(const FrameParams& p, const RowMap& rm, uint32_t x0, uint32_t xe,
                                              uint32_t py0, uint32_t pye) {
    // the pixel rectangle in viewport coordinates, widened to contain every pixel's x' = x/W and
    // y' = y/H (approximate reciprocal, then 2^-20 outward; x', y' >= 0)
    const float rw = __builtin_amdgcn_rcpf((float)p.cam_w), rh = __builtin_amdgcn_rcpf((float)p.cam_h);
    const float lo = 1.0f - 0x1p-20f, hi = 1.0f + 0x1p-20f;
    const uint32_t y0 = cam_row(rm, py0);  // (a sub-block's rows lie in one band)
    return Bundle{((float)x0 * rw) * lo, ((float)xe * rw) * hi, ((float)y0 * rh) * lo,
                  ((float)(y0 + (pye - py0)) * rh) * hi};
}

// One frame's output arrays (FrameParams::out_* of the frame: frames in flight write their own).
struct FrameOut {
    float* rgb;
    uint8_t* ppm;
    int32_t* face;
    bool nt;  // stores also non-temporal (FrameParams::store_nt)
};
__device__ __forceinline__ FrameOut frame_out(const FrameParams& p, uint32_t fr) {
    return FrameOut{p.out_rgb ? reinterpret_cast<float*>(reinterpret_cast<char*>(p.out_rgb) + fr * p.rgb_stride) : nullptr,
                    p.out_ppm ? p.out_ppm + fr * p.ppm_stride : nullptr,
                    p.out_face ? reinterpret_cast<int32_t*>(reinterpret_cast<char*>(p.out_face) + fr * p.face_stride)
                               : nullptr,
                    p.store_nt != 0};
}

// background (engine.rs:211-213) and its bytes: sat_u8(0.1*255) = 25, sat_u8(0.2*255) = 51
__device__ __forceinline__ float4 bg_rgb4(uint32_t phase) {  // 16-byte word at float offset 4c
    const float a = 0.1f, b = 0.2f;
    return phase == 0 ? make_float4(a, a, b, a) : phase == 1 ? make_float4(a, b, a, a) : make_float4(b, a, a, b);
}
__device__ __forceinline__ uint4 bg_ppm16(uint32_t phase) {  // 16-byte word at byte offset 16c
    const uint32_t c01 = sat_u8(0.1f * 255.0f), c02 = sat_u8(0.2f * 255.0f);
    const uint32_t w0 = c01 | (c01 << 8) | (c02 << 16) | (c01 << 24);  // 25 25 51 25
    const uint32_t w1 = c01 | (c02 << 8) | (c01 << 16) | (c01 << 24);  // 25 51 25 25
    const uint32_t w2 = c02 | (c01 << 8) | (c01 << 16) | (c02 << 24);  // 51 25 25 51
    return phase == 0 ? make_uint4(w0, w1, w2, w0) : phase == 1 ? make_uint4(w1, w2, w0, w1) : make_uint4(w2, w0, w1, w2);
}

// Background for the pixels [x0, x0 + w) x rows [py0, py0 + kBlkH) (w = 64 or 16), wave-wide.
// (kNt: non-temporal stores, FrameOut::nt — a template argument, not a per-store select)
template <uint32_t kW, bool kNt = false>
__device__ __forceinline__ void fill_background(const FrameParams& p, const FrameOut& o, uint32_t x0, uint32_t py0, bool aligned,
                                                uint32_t lane) {
    if (aligned && x0 + kW <= p.cam_w && py0 + kBlkH <= p.rows) {
        constexpr uint32_t kRow4 = kW * 3 / 4;    // float4 per RGB row
        constexpr uint32_t kRow16 = kW * 3 / 16;  // 16-byte words per PPM row
        constexpr uint32_t kFace4 = kW / 4;       // int4 per face row
        if (o.rgb) {
#pragma unroll
            for (uint32_t i = lane; i < kBlkH * kRow4; i += 64) {
                const uint32_t r = i / kRow4, c = i % kRow4;
                stream16(o.rgb, reinterpret_cast<float4*>(o.rgb + 3 * ((size_t)(py0 + r) * p.img_w + x0)) + c,
                         bg_rgb4(c % 3), kNt);
            }
        }
        if (o.ppm && lane < kBlkH * kRow16) {
            const uint32_t r = lane / kRow16, c = lane % kRow16;
            const size_t row = (size_t)(p.rows - py0 - kBlkH + r);  // file rows, bottom-up
            stream16(o.ppm, reinterpret_cast<uint4*>(o.ppm + 3 * (row * p.img_w + x0)) + c, bg_ppm16(c % 3), kNt);
        }
        if (o.face && lane < kBlkH * kFace4) {
            const uint32_t r = lane / kFace4, c = lane % kFace4;
            stream16(o.face, reinterpret_cast<int4*>(o.face + (size_t)(py0 + r) * p.img_w + x0) + c,
                     make_uint4(~0u, ~0u, ~0u, ~0u), kNt);
        }
    } else {  // image edge or unaligned output: per pixel
        const float4 b = bg_rgb4(0);
        const uint32_t c01 = sat_u8(0.1f * 255.0f), c02 = sat_u8(0.2f * 255.0f);
        for (uint32_t k = lane; k < kW * kBlkH; k += 64) {
            const uint32_t px = x0 + k % kW, py = py0 + k / kW;
            if (px >= p.cam_w || py >= p.rows) continue;
            const size_t idx = (size_t)py * p.img_w + px;
            if (o.rgb) {
                float* q = o.rgb + 3 * idx;
                q[0] = b.x;
                q[1] = b.y;
                q[2] = b.z;
            }
            if (o.ppm) {
                uint8_t* q = o.ppm + 3 * ((size_t)(p.rows - 1 - py) * p.img_w + px);
                q[0] = (uint8_t)c01;
                q[1] = (uint8_t)c01;
                q[2] = (uint8_t)c02;
            }
            if (o.face) o.face[idx] = -1;
        }
    }
}

// A full 64 x 4 background block's stores (fill_background<kBlkW> for aligned blocks inside the
// frame), per lane: the 16-B words it writes and their byte offsets from the block's first byte in
// each output array.  They are the same for every block, so the fill loop adds a wave-uniform
// block base as the buffer store's scalar offset and issues the stores: no per-store address
// arithmetic or pattern selects (the fill waves share their SIMDs' issue slots with the detail
// waves, and a frame's background is ~99 % of its stores).
struct BlockFill {
    uint4 rgb[3];
    uint32_t rgb_off[3];
    uint4 ppm;
    uint32_t ppm_off;
    uint32_t face_off;
};
__device__ __forceinline__ BlockFill block_fill(uint32_t img_w, uint32_t lane) {
    constexpr uint32_t kRow4 = kBlkW * 3 / 4;    // float4 per RGB row (48)
    constexpr uint32_t kRow16 = kBlkW * 3 / 16;  // 16-byte words per PPM row (12)
    constexpr uint32_t kFace4 = kBlkW / 4;       // int4 per face row (16)
    BlockFill b;
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) {
        const uint32_t i = lane + 64u * k, r = i / kRow4, c = i % kRow4;
        b.rgb_off[k] = r * img_w * 12u + c * 16u;
        const float4 v = bg_rgb4(c % 3u);
        b.rgb[k] = make_uint4(__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w));
    }
    const uint32_t r = lane / kRow16, c = lane % kRow16;  // lanes < kBlkH * kRow16 store
    b.ppm_off = r * img_w * 3u + c * 16u;
    b.ppm = bg_ppm16(c % 3u);
    b.face_off = (lane / kFace4) * img_w * 4u + (lane % kFace4) * 16u;
    return b;
}
template <bool kNt = false, typename B>
__device__ __forceinline__ void stream16_at(B* base, uint32_t voff, uint32_t soff, uint4 v) {
    stream16_pol<kNt>(base, voff, __builtin_amdgcn_readfirstlane(soff), v);
}
// The block (bx, by) (block units, rank-local rows; wave-uniform) from the lane constants.
template <bool kNt>
__device__ __forceinline__ void fill_block_fast(const FrameParams& p, const FrameOut& o, const BlockFill& bf, uint32_t bx,
                                                uint32_t by, uint32_t lane) {
    const uint32_t x0 = bx * kBlkW, py0 = by * kBlkH;
    if (o.rgb) {
        const uint32_t base = (py0 * p.img_w + x0) * 12u;
#pragma unroll
        for (uint32_t k = 0; k < 3; ++k) stream16_at<kNt>(o.rgb, bf.rgb_off[k], base, bf.rgb[k]);
    }
    if (o.ppm && lane < kBlkH * (kBlkW * 3 / 16))
        stream16_at<kNt>(o.ppm, bf.ppm_off, ((p.rows - py0 - kBlkH) * p.img_w + x0) * 3u, bf.ppm);
    if (o.face) stream16_at<kNt>(o.face, bf.face_off, (py0 * p.img_w + x0) * 4u, make_uint4(~0u, ~0u, ~0u, ~0u));
}

// the pixel rectangle of `ob` (camera rows) meets the sub-block's pixels
__device__ __forceinline__ bool rect_meets(const ObjGeom& ob, const RowMap& rm, uint32_t wx0, uint32_t py0) {
    const int32_t x0 = (int32_t)wx0, y0 = (int32_t)cam_row(rm, py0);
    return ob.rect[0] <= x0 + (int32_t)kSubW - 1 && ob.rect[1] >= x0 && ob.rect[2] <= y0 + (int32_t)kBlkH - 1 &&
           ob.rect[3] >= y0;
}

// Engine::cast_ray for the 16 x 4 pixels at (wx0, py0) (rank-local rows), one pixel per lane;
// `active` false: the wave only takes part in the workgroup's LDS-tile barriers.
// kMat: material features some object of the scene uses — kMatSpecPow (a specular-power output:
// powf is not the identity), kMatExample (main.rs's graph evaluated per hit texel); a kernel
// without them carries none of their code or registers.
constexpr int kMatSpecPow = 1, kMatExample = 2;
// Pipelining across a wave's sub-blocks (binned meshes): `pre` (or null) holds the bin range of
// this sub-block for object `pre_obj`, loaded during the wave's previous sub-block; `mid()` runs
// once the first hits are known (the next sub-block's range loads are issued there).
struct NoMid {
    __device__ void operator()() const {}
};

// Staged outputs of a wave's sub-block: its 16 x 4 pixels' f32 RGB rows (768 B) and PPM byte rows
// (192 B, file order) in an LDS slice.
constexpr uint32_t kWavePix = kSubW * kBlkH;
constexpr uint32_t kSliceRgbBytes = 3 * 4 * kWavePix, kSlicePpmBytes = 3 * kWavePix;
// The 16-B row stores of a staged slice (sub-block at (wx0, py0), rank-local rows).
// (wave-uniform sub-block: 32-bit lane offsets, the sub-block's base as the scalar offset)
__device__ __forceinline__ void store_slice(const FrameParams& p, const FrameOut& fo, uint32_t wx0, uint32_t py0,
                                            const float* wrgb, const uint8_t* wppm, uint32_t lane) {
    constexpr uint32_t kRgbRow4 = kSubW * 3 / 4;    // float4 per wave row (12)
    constexpr uint32_t kPpmRow16 = kSubW * 3 / 16;  // 16-byte words per wave row (3)
    // (the lane offsets are recomputed here, a few instructions, rather than kept live across the
    // detail rounds, where the 4-per-CU build would spill them)
    asm volatile("" : "+v"(lane));
    if (fo.rgb && lane < kBlkH * kRgbRow4) {
        const uint32_t r = lane / kRgbRow4, c = lane % kRgbRow4;
        const float4 v = reinterpret_cast<const float4*>(wrgb)[lane];
        const uint4 w = make_uint4(__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w));
        if (fo.nt)
            stream16_at<true>(fo.rgb, r * p.img_w * 12u + c * 16u, (py0 * p.img_w + wx0) * 12u, w);
        else
            stream16_at<false>(fo.rgb, r * p.img_w * 12u + c * 16u, (py0 * p.img_w + wx0) * 12u, w);
    }
    if (fo.ppm && lane < kBlkH * kPpmRow16) {
        const uint32_t r = lane / kPpmRow16, c = lane % kPpmRow16;  // r-th byte row of the block
        const uint4 w = reinterpret_cast<const uint4*>(wppm)[lane];
        if (fo.nt)
            stream16_at<true>(fo.ppm, r * p.img_w * 3u + c * 16u, ((p.rows - py0 - kBlkH) * p.img_w + wx0) * 3u, w);
        else
            stream16_at<false>(fo.ppm, r * p.img_w * 3u + c * 16u, ((p.rows - py0 - kBlkH) * p.img_w + wx0) * 3u, w);
    }
}

// kStaging: the build keeps the LDS-staged output path (only the dense large-mesh builds, whose
// 4-slot north-star frames use it; the others store per lane only and carry none of its registers)
template <bool kCull, bool kLdsTiles, int kMat, bool kStaging = true, typename Scene, typename Mid = NoMid>
__device__ __forceinline__ void render_sub(const FrameParams& p, const FrameOut& fo, const CamDev& cam, const RowMap& rm,
                                           const Scene& sc, uint32_t wx0, uint32_t py0,
                                           bool active, TriHot* s_hot, TriCull* s_cull, char* s_bins, float4* s_rgb,
                                           uint32_t* s_ppm, bool aligned, bool has_given = false,
                                           f3 given_d = f3{0.0f, 0.0f, 0.0f}, bool coop = true,
                                           PreRange pre = PreRange{0u, 0u, false}, uint32_t pre_obj = ~0u,
                                           Mid&& mid = Mid{}) {
    // coop (workgroup-uniform): the workgroup's four sub-blocks share their large objects' work —
    // binned chunks dealt over the waves, shadow rays through shared LDS tiles — with barriers;
    // otherwise (light sub-blocks) every wave searches its own bins and shadow rays alone
    // Culled large-mesh builds (screen bins): every sub-block is searched by its own wave
    // (first_hit_binned_wave handles bins of any length), the cooperative paths are compiled out —
    // 139 instead of 161 VGPRs and 1.5-2.7 % faster frames at 3840x2160 / 70k, C3, C5 and moving
    // cameras, where switching them off at run time gained nothing (profiles/r04/ab/ab_r04am.txt,
    // ab_r04an.txt).  A large object without bins (a bin-capacity overflow's fallback frame) is
    // then scanned by each wave alone; brute-force builds (!kCull) keep the LDS tiles.
    if constexpr (kCull && kLdsTiles) coop = false;
    wx0 = __builtin_amdgcn_readfirstlane(wx0);  // (wave-uniform: scalar registers)
    py0 = __builtin_amdgcn_readfirstlane(py0);
    constexpr bool kSpecPow = (kMat & kMatSpecPow) != 0, kExample = (kMat & kMatExample) != 0;
    // candidates tested together by the per-wave scans (small objects, shadow rays): four for ILP,
    // one in the large-mesh builds, whose registers bound their resident waves
    constexpr int kTestB = kLdsTiles ? kLargeTestBatch : kBatch;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const f3 C = mk3(cam.cx, cam.cy, cam.cz);
    const uint32_t px = wx0 + (lane % kSubW), ly = lane / kSubW;
    const uint32_t py = py0 + ly;
    const bool valid = active && px < p.cam_w && py < p.rows;
    const uint32_t y = cam_row(rm, py);
    const Bundle bd = make_bundle(p, rm, wx0, min(wx0 + kSubW - 1, p.cam_w - 1), py0, min(py0 + kBlkH - 1, p.rows - 1));

    // ---- cast_ray (engine.rs:112-216): closest object among first hits -----------
    ERAY_TRACE_WAVE0(4);
    f3 d = given_d;  // the camera ray, when the caller has it (has_given)
    bool ray_ready = has_given;
    bool have = false;
    float closest = 0.0f, bu = 0.0f, bv = 0.0f, bt = 0.0f;
    uint32_t best_obj = 0;
    int best_face = -1;
    for (uint32_t oi = 0; oi < p.nobj; ++oi) {
        const ObjGeom ob = sc.geom(oi);  // uniform
        ERAY_TRACE_WAVE0(16);
        const bool direct = !kLdsTiles || ob.tri_count <= kDirectMax;
        const bool wave_bins = kCull && !direct && !coop && ob.bin_start && ob.tri_count <= kWaveBinMaxTris;
        // outside the object's pixel rectangle no primary ray can hit it (only where skipping
        // keeps the workgroup's barriers uniform: without coop nothing here has a barrier)
        if (kCull && (direct || !coop) && !rect_meets(ob, rm, wx0, py0)) continue;
        auto activate = [&]() {
            if (!ray_ready) {
                uint32_t pxo = px, yo = y;  // opaque: keep ray generation on this path
                asm volatile("" : "+v"(pxo), "+v"(yo));
                d = camera_dir(cam, p, pxo, yo);
                ray_ready = true;
            }
            const bool bb = bbox_hit(ob, C, d);
            return bb;
        };
        int st = valid ? kUndecided : kDone, f = -1;
        float u, v, t;
        if (direct) {
            first_hit<kCull, false, false, kTestB>(p, sc, ob.tri_begin, ob.tri_count, st, C, d, bd, s_hot, s_cull, activate, f, u,
                                    v, t);
        } else if (wave_bins) {  // this wave's own bin, no barrier
            const uint32_t bin = ((cam_row(rm, py0) + kBinH - p.bin_phase) / kBinH) * p.bins_x + wx0 / kBinW;
            first_hit_binned_wave(ob, bin, st, C, d, activate, f, u, v, t, s_bins,
                                  oi == pre_obj ? pre : PreRange{0u, 0u, false});
        } else if (kCull && ob.bin_start && coop) {  // the workgroup's four sub-blocks together
            const uint32_t bin = ((cam_row(rm, py0) + kBinH - p.bin_phase) / kBinH) * p.bins_x + wx0 / kBinW;
            first_hit_binned(p, ob, bin, st, C, d, activate, f, u, v, t, s_bins,
                             oi == pre_obj ? pre : PreRange{0u, 0u, false});
        } else if (!coop) {  // no bins (or too many faces for the wave's keys): this wave scans alone
            first_hit<kCull, false, false, kTestB>(p, sc, ob.tri_begin, ob.tri_count, st, C, d, bd, s_hot, s_cull,
                                                   activate, f, u, v, t);
        } else {
            first_hit<kCull, kLdsTiles, false, kTestB>(p, sc, ob.tri_begin, ob.tri_count, st, C, d, bd, s_hot, s_cull, activate,
                                        f, u, v, t);
        }
        if (f >= 0) {
            const f3 P = add(C, mul(d, t));
            const float dsq = len_sq(sub(P, C));
            if (!have || dsq < closest) {  // strict `<`: the first object wins ties
                have = true;
                closest = dsq;
                best_obj = oi;
                best_face = f;
                bu = u;
                bv = v;
                bt = t;
            }
        }
    }

    mid();
    ERAY_TRACE_WAVE0(5);
    // ---- hit data and Material::get (material.rs:56-94) --------------------------
    // The object loop only finds each lane's texel addresses; the loads are issued once after
    // it and first used by the shading, so their latency overlaps the shadow rays.
    f3 P = mk3(0.0f, 0.0f, 0.0f), N = mk3(0.0f, 0.0f, 0.0f);
    rgb color{0.0f, 0.0f, 0.0f};
    float kd = 0.5f, ks = 0.5f, sp = 1.0f;
    const float *tc = nullptr, *tkd = nullptr, *tks = nullptr, *tsp = nullptr;  // texels, if any
    // every hit lane's shading record in one load from a wave-uniform point (a lane without a
    // hit reads record 0)
    TriShade sh = TriShade{};
    if (__any(have)) {
        uint32_t g = 0;
        for (uint32_t oi = 0; oi < p.nobj; ++oi) {
            if (!__any(have && best_obj == oi)) continue;
            const uint32_t tb = load_const(&sc.geom_ptr(oi)->tri_begin, 0);
            if (have && best_obj == oi) g = tb + (uint32_t)best_face;
        }
        sh = sc.shade(g);
    }
    for (uint32_t oi = 0; oi < p.nobj; ++oi) {  // per-lane object, read from uniform copies
        if (!__any(have && best_obj == oi)) continue;
        const MaterialDesc mat = sc.mat(oi);
        ERAY_TRACE_WAVE0(17);
        if (!(have && best_obj == oi)) continue;
        P = add(C, mul(d, bt));
        const f3 na = mk3(sh.s0.x, sh.s0.y, sh.s0.z), nb = mk3(sh.s0.w, sh.s1.x, sh.s1.y);
        const f3 nc = mk3(sh.s1.z, sh.s1.w, sh.s2.x);
        N = normalize(add(add(mul(na, bu), mul(nb, bv)), mul(nc, bt)));
        const float w = 1.0f - bu - bv;
        const float uv0 = ((sh.s2.y * w) + (sh.s2.w * bu)) + (sh.s3.y * bv);
        const float uv1 = ((sh.s2.z * w) + (sh.s3.x * bu)) + (sh.s3.z * bv);
        if (kExample && mat.example) {  // main.rs's graph at the texel Material::get would read
            const uint32_t ix = mod_size(sat_u32(uv0 * (float)mat.ex_w), mat.ex_w);
            const uint32_t iy = mod_size(sat_u32(uv1 * (float)mat.ex_h), mat.ex_h);
            const float wv = __builtin_fabsf(libm::cosf_glibc(libm::div10_f32((float)ix * mat.ex_xf + (float)iy * mat.ex_yf)));
            const float omf = 1.0f - mat.ex_factor;  // mix_color.rs:89 (material_example_kernel)
            color = rgb{wv * omf + mat.ex_r * mat.ex_factor, wv * omf + mat.ex_g * mat.ex_factor,
                        wv * omf + mat.ex_b * mat.ex_factor};
            kd = wv;
        }
        if (kExample && mat.prog) {  // a shader graph at the texel (its outputs have no texture)
            float t3[3];
            if (texel_program(mat.prog, 0, uv0, uv1, t3)) color = rgb{t3[0], t3[1], t3[2]};
            if (texel_program(mat.prog, 1, uv0, uv1, t3)) kd = t3[0];
            if (texel_program(mat.prog, 2, uv0, uv1, t3)) ks = t3[0];
            if (kSpecPow && texel_program(mat.prog, 3, uv0, uv1, t3)) sp = t3[0];
        }
        tc = texel(mat.color, uv0, uv1, 3);
        tkd = texel(mat.diffuse, uv0, uv1, 1);
        tks = texel(mat.specular, uv0, uv1, 1);
        if (kSpecPow) tsp = texel(mat.specular_power, uv0, uv1, 1);
    }
    // every lane loads (a lane without the texture reads a dummy word); Material::get's values
    // are selected where the shading first needs them
    const bool has_c = tc, has_kd = tkd, has_ks = tks, has_sp = kSpecPow && tsp;
    const auto* tcg = as_global(tc ? tc : g_texel_dummy);
    const float vc0 = tcg[0], vc1 = tcg[1], vc2 = tcg[2];
    const float vkd = *as_global(tkd ? tkd : g_texel_dummy);
    const float vks = *as_global(tks ? tks : g_texel_dummy);
    const float vsp = kSpecPow ? *as_global(tsp ? tsp : g_texel_dummy) : 1.0f;
    bool resolved = false;
    auto material = [&]() {
        if (resolved) return;
        resolved = true;
        if (has_c) color = rgb{vc0, vc1, vc2};
        if (has_kd) kd = vkd;
        if (has_ks) ks = vks;
        if (has_sp) sp = vsp;
    };

    bool any = false;  // the lighting list as a running left fold (color.rs:82-87)
    rgb acc{0.0f, 0.0f, 0.0f};
    auto push = [&](rgb c) {
        if (any) {
            acc = cadd(acc, c);
        } else {
            acc = c;
            any = true;
        }
    };
    ERAY_TRACE_WAVE0(13);
    const HitBox hb = hit_box(have, P, N);  // (wave-uniform; shadow-ray face bounds)
    // Point lights first (engine.rs:130-135), 32 at a time: every light's shadow ray, then the
    // shading of the lights that reach the hit, in list order.  The texture loads above are
    // still in flight during the first shadow scan; the shading is their first use.
    for (uint32_t li0 = 0; li0 < p.nlights; li0 += 32) {
        const uint32_t li1 = min(p.nlights, li0 + 32);
        uint32_t lit = 0;  // bit li - li0: point light li reaches the lane's hit
        for (uint32_t li = li0; li < li1; ++li) {
            const LightDesc L = sc.light(li);
            ERAY_TRACE_WAVE0(18);
            if (L.variant == 1 || (!(kLdsTiles && coop) && !__any(have))) continue;  // (LDS tiles: barriers)
            const f3 Lp = mk3(L.pos[0], L.pos[1], L.pos[2]);
            // reaches_light(Ray::new(P + N * 0.1, Lp - P)) (engine.rs:136-142, 218-228)
            f3 S = mk3(0.0f, 0.0f, 0.0f);
            f3 sd = mk3(0.0f, 0.0f, 1.0f);
            float dist = 0.0f;
            bool reached = true, decided = false;
            bool ray = false;  // S, sd, dist computed
            auto shadow_ray = [&]() {
                if (ray) return;
                ray = true;
                if (have) {
                    S = add(P, mul(N, 0.1f));
                    sd = normalize(sub(Lp, P));
                    dist = len(sub(Lp, S));
                }
            };
            for (uint32_t oj = 0; oj < p.nobj; ++oj) {
                const ObjGeom ob = sc.geom(oj);
                ERAY_TRACE_WAVE0(19);
                // A point box (the loaded meshes'): when it certainly rejects every lane's shadow
                // ray (point_box_rejects), bbox_hit is false for all of them — no ray, no face
                // load (not where the LDS tiles' barriers need every wave)
                if (!(kLdsTiles && coop && ob.tri_count > kDirectMax) && point_box_xy(ob) &&
                    !__any(have && !decided && !point_box_rejects(ob, add(P, mul(N, 0.1f)), sub(Lp, P)))) {
                    ERAY_TRACE_VALUE(20, 1u + oj);  // (diagnostics: the skip fired for object oj)
                    continue;
                }
                ERAY_TRACE_VALUE(21, 1u + oj);  // (... the shadow scan of object oj ran)
                int f = -1;
                float u, v, t;
                if (!kLdsTiles || ob.tri_count <= kDirectMax) {
                    // faces some hit point's shadow ray may pass (box bounds, lane-parallel),
                    // then the exact tests in index order; the ray itself only when needed
                    int st = kDone;
                    bool opened = false;
                    for (uint32_t base = 0; base < ob.tri_count; base += 64) {
                        const uint32_t n = min(64u, ob.tri_count - base);
                        bool keep = lane < n;
                        if (keep && hb.ok) keep = shadow_box_may_hit(sc.hot_lane(ob.tri_begin + base + lane), Lp, hb);
                        const unsigned long long mask = __ballot(keep);
                        if (!mask) continue;
                        if (!opened) {
                            opened = true;
                            shadow_ray();
                            st = (have && !decided && bbox_hit(ob, S, sd)) ? kSearching : kDone;
                        }
                        if (!__any(st == kSearching)) break;
                        auto face = [&](uint32_t i) { return base + i; };
                        auto hot = [&](uint32_t i) { return sc.hot(ob.tri_begin + base + i); };
                        if (!test_candidates<kTestB>(mask, face, hot, st, S, sd, f, u, v, t)) break;
                    }
                } else if (!coop) {  // this wave alone (no barrier): faces its searching lanes may hit
                    shadow_ray();
                    int st = (have && !decided && bbox_hit(ob, S, sd)) ? kSearching : kDone;
                    auto never = []() { return false; };
                    first_hit<false, false, true, kTestB>(p, sc, ob.tri_begin, ob.tri_count, st, S, sd, bd, s_hot, s_cull,
                                                  never, f, u, v, t);
                } else {
                    shadow_ray();
                    int st = (have && !decided && bbox_hit(ob, S, sd)) ? kSearching : kDone;
                    auto never = []() { return false; };
                    first_hit<false, kLdsTiles, false, kTestB>(p, sc, ob.tri_begin, ob.tri_count, st, S, sd, bd, s_hot, s_cull,
                                                never, f, u, v, t);
                }
                if (f >= 0) {
                    const f3 hp = add(S, mul(sd, t));
                    reached = len(sub(hp, S)) > dist;
                    decided = true;
                }
            }
            if (have && reached) lit |= 1u << (li - li0);
        }
        ERAY_TRACE_WAVE0(14);
        if (!__any(lit != 0)) continue;
        material();
        for (uint32_t li = li0; li < li1; ++li) {
            const LightDesc L = sc.light(li);
            if (L.variant == 1 || !((lit >> (li - li0)) & 1u)) continue;  // engine.rs:143-178
            const f3 Lp = mk3(L.pos[0], L.pos[1], L.pos[2]);
            const f3 LmP = sub(Lp, P);
            float prod = rust_clamp(dot0(N, LmP), 0.0f, 1.0f);
            if (prod != prod) prod = 0.0f;
            const float falloff = 1.0f / len(LmP);
            const rgb lc{L.color[0], L.color[1], L.color[2]};
            const rgb diffusion =
                cmul(cmul(cmul(cmul(cmulc(color, lc), kd), prod), L.brightness), falloff);
            const f3 reflected = sub(d, mul(mul(N, 2.0f), dot0(d, N)));
            const float dotr = dot0(normalize(reflected), normalize(LmP));
            // specular_power defaults to 1 and powf(x, 1) == x; pow only when a
            // material has a specular-power output (kSpecPow)
            const float res =
                rust_clamp(ks * L.brightness * (kSpecPow ? powf_ref(dotr, sp) : dotr), 0.0f, 1.0f);
            const float sf = rust_clamp(kSpecPow ? powf_ref(falloff, sp) : falloff, 0.0f, 1.0f);
            const rgb specular{res * sf, res * sf, res * sf};
            push(cadd(diffusion, specular));
        }
    }
    if (have) {
        material();
        for (uint32_t li = 0; li < p.nlights; ++li) {  // ambient lights (engine.rs:197-209)
            const LightDesc L = sc.light(li);
            if (L.variant != 1) continue;
            const rgb m{rust_min(L.color[0], color.r), rust_min(L.color[1], color.g),
                        rust_min(L.color[2], color.b)};
            push(cmul(cmul(m, kd), L.brightness));
        }
    } else {
        push(rgb{0.1f, 0.1f, 0.2f});  // engine.rs:211-213
    }

    ERAY_TRACE_WAVE0(6);
    // ---- outputs: Image::set + Color::as_bytes, rows bottom-up (image.rs:41-74) ---
    const uint32_t b0 = sat_u8(acc.r * 255.0f), b1 = sat_u8(acc.g * 255.0f), b2 = sat_u8(acc.b * 255.0f);
    if (valid && fo.face) fo.face[(size_t)py * p.img_w + px] = have ? best_face : -1;
    // Frames into a ring beyond the Infinity Cache (non-temporal launches aside; dense builds
    // only: C2 in 16 slots is no faster staged) leave through the wave's LDS slice as
    // write-through 16-B row stores (3840x2160 / 70k in 4 slots 25.6 -> 24.8 us); elsewhere each lane stores its own pixel with plain (write-back) stores: C5 123.5 ->
    // 116, C2 40.6 -> 40.3 us (no LDS round trip and wave barriers in the chain).  Write-through
    // partial stores lose badly (C5 154 us).  Same-box A/B profiles/r05/ab/ab_r05ao.txt ..
    // ab_r05aq.txt
    const bool staged = kStaging && (p.launch_flags & kLaunchRingBeyondCache) && !fo.nt;
    if (staged && active && aligned && wx0 + kSubW <= p.cam_w && py0 + kBlkH <= p.rows) {
        // the wave's 16 x 4 pixels leave through its own LDS slice as 16-B row stores
        float* wrgb = reinterpret_cast<float*>(reinterpret_cast<char*>(s_rgb) + kSliceRgbBytes * wave);
        uint8_t* wppm = reinterpret_cast<uint8_t*>(s_ppm) + kSlicePpmBytes * wave;
        const uint32_t wl = lane % kSubW;
        float* srgb = wrgb + 3 * (ly * kSubW + wl);
        srgb[0] = acc.r;
        srgb[1] = acc.g;
        srgb[2] = acc.b;
        uint8_t* sppm = wppm + 3 * ((kBlkH - 1 - ly) * kSubW + wl);
        sppm[0] = (uint8_t)b0;
        sppm[1] = (uint8_t)b1;
        sppm[2] = (uint8_t)b2;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        store_slice(p, fo, wx0, py0, wrgb, wppm, lane);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // the slice is rewritten by the next block
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else if (valid) {
        const size_t idx = (size_t)py * p.img_w + px;
        if (fo.rgb) {
            float* o = fo.rgb + 3 * idx;
            o[0] = acc.r;
            o[1] = acc.g;
            o[2] = acc.b;
        }
        if (fo.ppm) {
            uint8_t* o = fo.ppm + 3 * ((size_t)(p.rows - 1 - py) * p.img_w + px);
            o[0] = (uint8_t)b0;
            o[1] = (uint8_t)b1;
            o[2] = (uint8_t)b2;
        }
    }
    ERAY_TRACE_WAVE0(7);
}

// detail rectangle k of the frame (kernel arguments, or the setup's CamState in device-camera
// mode; uniform index: scalar loads)
struct SubRect {  // sub-block coordinates (x in kSubW columns, y in kBlkH local rows), inclusive
    int32_t sx0, sx1, sy0, sy1;
};
template <bool kDev>
__device__ __forceinline__ SubRect frame_rect(const FrameParams& p, const CamState* cs, uint32_t k) {
    if (kDev) return load_const(reinterpret_cast<const SubRect*>(cs->rects), k);
    return SubRect{p.rects[k][0], p.rects[k][1], p.rects[k][2], p.rects[k][3]};
}
template <bool kDev>
__device__ __forceinline__ uint32_t frame_nrect(const FrameParams& p, const CamState* cs) {
    return kDev ? load_const(&cs->nrect, 0) : p.nrect;
}
__device__ __forceinline__ bool inside(const SubRect& r, int32_t sx, int32_t sy) {
    return sx >= r.sx0 && sx <= r.sx1 && sy >= r.sy0 && sy <= r.sy1;
}

// The background of the non-detail sub-blocks: fill workgroup f of nf strides over the 64 x 4
// blocks (shared by the frame kernel's fill roles and fill_kernel).
// s_waitcnt immediate (gfx9 encoding: vmcnt bits 3:0 and 15:14, expcnt 6:4, lgkmcnt 11:8) of the
// fill's per-block pacing: vmcnt(0), expcnt / lgkmcnt not waited for
constexpr int kFillPace = 0x0f70;
// cacheable stores: two operations may stay in flight (vmcnt(2) against (0): ns1 19.5 -> 19.4,
// C3 23.3 -> 22.7, C2 41.5 -> 41.0 us; (5) and (10) lose the pacing, profiles/r05/ab/ab_r05al.txt)
constexpr int kFillPaceCached = 0x0f72;
// ... cacheable stores into a ring beyond the Infinity Cache (the per-lane form): one operation in
// flight (3840x2160 / 70k in 4 slots: vmcnt(1) 23.42, (2) 23.65, (0) 23.75, (3) 24.1 us,
// profiles/r06/ab/ab_r06kk_pace_beyond.txt)
constexpr int kFillPaceBeyond = 0x0f71;
// kSgpr: block coordinates in SGPRs (the store offsets' block part a scalar); without it they are
// per-lane values and every store a full per-lane offset — faster for an unpaced fill into a ring
// beyond the Infinity Cache (3840x2160 in 4 slots 23.0 -> 19.8 us), slower elsewhere (C2's fill
// alone 34.7 -> 35.8 us, 3840x2160 / 70k 19.8 -> 20.1 us), same-box A/B profiles/r05/ab/ab_r05ah.txt
template <bool kDev, bool kNt, bool kPace, bool kSgpr = true>
__device__ __forceinline__ void fill_blocks(const FrameParams& p, const FrameOut& o, const CamState* cs,
                                            const uint8_t* detail_occ, uint32_t f, uint32_t nf, uint32_t wave,
                                            uint32_t lane, bool aligned) {
    constexpr uint32_t nwaves = kWG / 64;
    if constexpr (kSgpr) wave = __builtin_amdgcn_readfirstlane(wave);
    const uint32_t nblk = p.tiles_x * ((p.rows + kBlkH - 1) / kBlkH);
    const uint32_t fstride = nf * nwaves;
    constexpr bool kFast = kPace && !kNt && kSgpr;  // (below)
    BlockFill bf;
    if constexpr (kFast) bf = block_fill(p.img_w, lane);
    // blocks (bx, by) with bx < full_x and by < full_y are whole 64 x 4 blocks inside the frame
    const uint32_t full_x = aligned ? p.cam_w / kBlkW : 0u, full_y = p.rows / kBlkH;
    uint32_t occ = 0;  // detail list: lane i holds the occupancy of this wave's i-th next block
    uint32_t it = 0;
    const uint32_t nrect = detail_occ ? 0u : frame_nrect<kDev>(p, cs);
    // block coordinates advance incrementally (no integer division per block); the workgroup's
    // four waves take four neighbouring blocks, the workgroups consecutive runs of four
    const uint32_t first = f * nwaves + wave, step_y = fstride / p.tiles_x, step_x = fstride - step_y * p.tiles_x;
    uint32_t by = first / p.tiles_x, bx = first - by * p.tiles_x;
    for (uint32_t blk = first; blk < nblk; blk += fstride, ++it) {
        if (it) {
            bx += step_x;
            by += step_y;
            if (bx >= p.tiles_x) {
                bx -= p.tiles_x;
                ++by;
            }
        }
        uint32_t mask = 0;  // detail sub-blocks of this block
        if (detail_occ) {  // one load per 64 blocks, not a dependent load per block
            if ((it & 63u) == 0) {
                const uint32_t b = blk + lane * fstride;
                occ = b < nblk ? detail_occ[b] : 0u;
                asm volatile("" : "+v"(occ));  // (waited for here; the pacing below is explicit)
            }
            mask = (uint32_t)__builtin_amdgcn_readlane((int)occ, (int)(it & 63u));
        }
        for (uint32_t k = 0; k < nrect; ++k) {
            const SubRect r = frame_rect<kDev>(p, cs, k);
            if ((int32_t)by < r.sy0 || (int32_t)by > r.sy1) continue;
#pragma unroll
            for (int32_t i = 0; i < 4; ++i) {
                const int32_t sx = (int32_t)(4 * bx) + i;
                mask |= (sx >= r.sx0 && sx <= r.sx1) ? (1u << i) : 0u;
            }
        }
        // Pacing beside detail work: each block's stores wait until the wave's earlier stores are
        // acknowledged (vmcnt counts them).  Unpaced fill waves flood the memory system and
        // lengthen the detail waves' load chains — 3840x2160 / 70k 19.8 -> 24.6 us per frame, C3
        // 22.2 -> 27.2, C5 128 -> 141; C2 (8 frames) 40.9 -> 43.5 — and a looser bound (vmcnt(5)
        // or (10)) is no better; a fill with the GPU to itself is faster unpaced (3840x2160 18.3
        // vs 21.5 us), same-box A/B profiles/r05/ab/.
        if constexpr (kPace) __builtin_amdgcn_s_waitcnt(kNt ? kFillPace : kSgpr ? kFillPaceCached : kFillPaceBeyond);
        if (!mask) {
            // the hoisted-offset stores where the fill is paced and cached (C2 8 frames 52.8 ->
            // 41.2 us); unpaced or non-temporal, the per-block address form writes faster (fill
            // alone at 3840x2160 in 4 slots 23.3 -> 19.8 us, C5 130 -> 123 us), same-box A/B
            // profiles/r05/ab/
            if (kFast && bx < full_x && by < full_y)
                fill_block_fast<kNt>(p, o, bf, bx, by, lane);
            else
                fill_background<kBlkW, kNt>(p, o, bx * kBlkW, by * kBlkH, aligned, lane);
        } else if (mask != 0xfu) {
            for (uint32_t i = 0; i < 4; ++i)
                if (!((mask >> i) & 1u)) fill_background<kSubW, kNt>(p, o, bx * kBlkW + i * kSubW, by * kBlkH, aligned, lane);
        }
    }
}

// Fill role q of nf over the launch's frames: virtual roles v (more than nf only when nf < F),
// frame v % F, its (v / F)-th fill workgroup.
template <bool kDev>
__device__ __forceinline__ void fill_frames(const FrameParams& p, uint32_t q, uint32_t nf, uint32_t wave, uint32_t lane,
                                            bool aligned, bool pace) {
    const uint32_t F = p.nframes, roles = max(nf, F);
    for (uint32_t v = q; v < roles; v += nf) {
        const uint32_t fr = v % F, slot = p.dev_slots ? fr : 0u;
        const uint8_t* occ = p.detail_occ ? p.detail_occ + (size_t)slot * (p.dlist_stride / 4) : nullptr;
        const FrameOut o = frame_out(p, fr);
        const uint32_t g = v / F, ng = (roles - fr + F - 1) / F;
        const CamState* cs = p.cam_state + slot;
        // (separate loops: the unpaced fill, without the paced one's lane constants in its
        // registers, writes a 4-slot 3840x2160 frame in 19.8 instead of 22.3 us)
        if (o.nt && pace)
            fill_blocks<kDev, true, true>(p, o, cs, occ, g, ng, wave, lane, aligned);
        else if (o.nt)
            fill_blocks<kDev, true, false>(p, o, cs, occ, g, ng, wave, lane, aligned);
        else if (pace && (p.launch_flags & kLaunchRingBeyondCache))
            // paced into a ring beyond the Infinity Cache: per-lane block coordinates and per-block
            // addresses, as the unpaced form there (3840x2160 / 70k in 4 slots 24.06 -> 23.64 us;
            // C2, C3 and the 1-slot frame unchanged: same-box A/B profiles/r06/ab/ab_r06ii_paced_lane.txt)
            fill_blocks<kDev, false, true, false>(p, o, cs, occ, g, ng, wave, lane, aligned);
        else if (pace)
            fill_blocks<kDev, false, true>(p, o, cs, occ, g, ng, wave, lane, aligned);
        else if (p.launch_flags & kLaunchRingBeyondCache)
            fill_blocks<kDev, false, false, false>(p, o, cs, occ, g, ng, wave, lane, aligned);
        else
            fill_blocks<kDev, false, false>(p, o, cs, occ, g, ng, wave, lane, aligned);
    }
}

// kDense (large meshes only): 4 workgroups per CU instead of 2 (at most 128 VGPRs), for frames
// whose detail sub-blocks exceed one round of the 2-per-CU grid — there the detail waves are
// latency bound and more resident detail waves mean fewer rounds.  Round 5 (profiles/r05/ab/):
// the culled large-mesh path lost its 64-bit per-lane addresses (buffer loads of records and
// bin entries, scalar store offsets) and fits 4 per CU; with the fill at one workgroup per CU
// (launch_frame_kernel) 3840x2160 / 70k 22.2 -> 20.1 us, its moving camera 50.0 -> 46.7 us.
constexpr int kDenseWgs = 4;
template <bool kCull, bool kLdsTiles, int kMat, bool kLdsScene, bool kDense = false, bool kDev = false>
__global__ void __launch_bounds__(kWG, (kMat & kMatSpecPow) ? 1 : (kLdsTiles && !kDense) ? 1 : (kDense ? kDenseWgs : 3))  // 3 workgroups per CU where that fits
    frame_kernel(const ObjectDesc* h_objects, const LightDesc* h_lights, const TriCull* h_cull, const TriHot* h_tris,
                 const void* h_aux, uint32_t h_counts, uint32_t h_total_tris, uint32_t h_total_sub,
                 uint32_t h_roles, uint32_t h_band, FrameParams p) {
    // h_aux (preloaded): the TriShade array in the LDS-scene builds (the scene preload reads it
    // first), else the detail list (p.detail_list), whose first entry is each detail wave's first
    // load.  (gfx950 preloads 14 argument dwords — 16 user SGPRs less the argument pointer — so
    // h_band and everything after it are loads.)
    // h_roles (a preloaded argument, see frame_roles): the grid size, the detail workgroups and
    // the role flags, so the role decision — and the scene preload behind it — does not wait for
    // a kernel-argument load from memory
    const uint32_t grid = h_roles & 0xfffu;  // == gridDim.x, without the implicit-argument load
    uint32_t detail_wgs = (h_roles >> 12) & 0xfffu;
    bool fill_first = (h_roles >> 30) & 1u;
    const bool separate_fill = (h_roles >> 31) & 1u;
    // large objects: LDS tiles (shadow rays, brute force) and, aliased, the per-wave binned
    // primary search (first_hit ends its tile loop on a barrier, so the two never overlap)
    // (the culled large-mesh builds search bins wave by wave and scan shadow rays per wave: no
    // workgroup tiles)
    constexpr size_t kTileBytes = (kCull && kLdsTiles) ? 0 : kTriTile * sizeof(TriHot);
    constexpr size_t kBinBytes = (kCull && kLdsTiles) ? (kWG / 64) * kBinLdsBytes + 2 * (kWG / 64) * 4 : 0;
    __shared__ __attribute__((aligned(16))) char s_large[kLdsTiles ? (kTileBytes > kBinBytes ? kTileBytes : kBinBytes) : 16];
    TriHot* s_hot = reinterpret_cast<TriHot*>(s_large);
    TriCull* s_cull = nullptr;
    char* s_bins = s_large;
    __shared__ float4 s_rgb[kBlkW * kBlkH * 3 / 4];    // each wave's f32 RGB rows, staged
    __shared__ uint32_t s_ppm[kBlkW * kBlkH * 3 / 4];  // ... and its PPM byte rows
    extern __shared__ __attribute__((aligned(16))) char dyn[];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t nwaves = kWG / 64;
    const bool aligned = p.aligned != 0;  // (a kernel-argument read where it is used)
    // Frames in flight: the launch renders F independent frames; detail and fill workgroups are
    // dealt round-robin over them (frame v % F), so one frame's latency-bound detail chains
    // overlap the others' fill stores instead of ending the launch alone.
    const uint32_t F = ((h_roles >> 24) & 63u) + 1u;  // == p.nframes (the role decision needs no load)
    auto cam_state = [&](uint32_t fr) { return p.cam_state + (p.dev_slots ? fr : 0u); };
    // detail sub-blocks per frame (device-camera mode: counted by the setup kernels; the most of
    // any frame sizes the detail roles), and the small-scene fill reservation chosen from that
    // count as launch_frame_kernel does from the host's
    uint32_t total_max = h_total_sub;
    if (kDev) {
        total_max = 0;
        for (uint32_t fr = 0; fr < F; ++fr) total_max = max(total_max, load_const(&cam_state(fr)->total_sub, 0));
    }
    if (kDev && p.detail_wgs_alt && F * total_max > detail_wgs * nwaves) {
        detail_wgs = p.detail_wgs_alt;
        fill_first = true;
    }
    // workgroups [0, nd) render the detail sub-blocks (persistent: rounds of nd * 4 sub-blocks),
    // the others write the background at the same time; at most detail_wgs detail workgroups
    // (the launcher keeps a share of the grid for the fill, so a large detail area overlaps the
    // fill's HBM writes instead of preceding them); when every workgroup has detail work, all of
    // them fill afterwards
    const uint32_t nd = min(detail_wgs ? detail_wgs : grid, F * ((total_max + nwaves - 1) / nwaves));
    // the workgroup's role index: detail roles [0, nd), fill roles [nd, grid); with fill_first
    // the fill roles go to the first-dispatched (older, VALU-priority) workgroups
    const uint32_t bid = (fill_first && nd < grid) ? (blockIdx.x + nd) % grid : blockIdx.x;

    ERAY_TRACE_POINT(0);
    // ---- detail sub-blocks -------------------------------------------------------------------
    if (bid < nd) {
        // the ordered detail list's heavy count: the threshold of the cooperative (workgroup-shared)
        // sub-blocks in builds that keep those paths (brute-force large meshes; no count: every
        // iteration shares its work)
        const bool counted = kLdsTiles && !(p.launch_flags & kLaunchSharedDetail);
        const uint32_t heavy0 =
            (!kCull && counted && p.detail_heavy) ? load_const(p.detail_heavy, 0) : 0xffffffffu;
        // the detail list (preloaded in h_aux outside the LDS-scene builds, which have none)
        const uint32_t* list_base = kLdsScene ? p.detail_list : static_cast<const uint32_t*>(h_aux);
        // One camera (args mode): the wave's first list entry (role bid) depends on preloaded
        // arguments only, so it is loaded first, beside the kernel-argument loads that follow
        // (branch-free: without a list it reads a word of the descriptors, unused).
        uint32_t e_first = 0;
        if constexpr (!kDev && !kLdsScene) {
            const uint32_t c = (bid / F) * nwaves + wave;
            e_first = vload_u32(list_base ? list_base : reinterpret_cast<const uint32_t*>(h_objects),
                                list_base && c < h_total_sub ? c : 0u);
        }
        // snake order for the ordered (heavy-first) lists of binned meshes
        constexpr bool kSnake = kLdsTiles;
        const RowMap rm{p.row0, h_band & 31u, h_band >> 5};
        const uint32_t nobj = h_counts & 0xffffu;
        // virtual detail roles v (more than nd only when nd < F): frame v % F, its (v / F)-th
        // detail workgroup of nk
        const uint32_t roles = max(nd, F);
        for (uint32_t v = bid; v < roles; v += nd) {
            const uint32_t fr = v % F, kw = v / F, nk = (roles - fr + F - 1) / F;
            const uint32_t c0 = kw * nwaves;
            const CamState* cs = cam_state(fr);
            const uint32_t total = kDev ? load_const(&cs->total_sub, 0) : h_total_sub;
            // (per-frame setup slots exist only in device-camera mode)
            const uint32_t slot = (kDev && p.dev_slots) ? fr : 0u;
            const uint32_t* dlist = list_base ? (kDev ? list_base + (size_t)slot * p.dlist_stride : list_base) : nullptr;
            const FrameOut fo = frame_out(p, fr);
            const ObjectDesc* objs = h_objects + (size_t)slot * nobj;
            const TriCull* culls = h_cull ? h_cull + (size_t)slot * h_total_tris : nullptr;
            const uint32_t nrect = dlist ? 0u : frame_nrect<kDev>(p, cs);
            const CamDev cam = frame_camera<kDev>(p, cs);
            // a split list (camera paths): the frame's heavy sub-blocks from the front, the light
            // ones from the back (bins.hip detail_list_kernel) — list positions always follow the
            // setup's heavy count; `heavy` is the cooperative threshold (none without a count)
            const bool split = kDev && p.dlist_split && dlist;
            const uint32_t split_heavy = split ? load_const(&cs->heavy_sub, 0) : 0u;
            const uint32_t heavy = split ? (counted ? split_heavy : 0xffffffffu) : heavy0;
            auto lpos = [&](uint32_t j) {
                return split && j >= split_heavy ? p.dlist_split - 1u - (j - split_heavy) : j;
            };
            // detail sub-block j (enumeration order) -> sub-block coordinates
            auto locate = [&](uint32_t j, int32_t& sx, int32_t& sy, bool first = false) {
                if (dlist) {
                    const uint32_t e = __builtin_amdgcn_readfirstlane((!kDev && !kLdsScene && first && v == bid)
                                                                          ? e_first
                                                                          : vload_u32(dlist, lpos(j)));
                    sx = (int32_t)(e & 0xffffu);
                    sy = (int32_t)(e >> 16);
                    return;
                }
                for (uint32_t k = 0; k < nrect; ++k) {  // the rectangles are disjoint (setup): by area
                    const SubRect r = frame_rect<kDev>(p, cs, k);
                    const uint32_t w = (uint32_t)(r.sx1 - r.sx0 + 1);
                    const uint32_t a = w * (uint32_t)(r.sy1 - r.sy0 + 1);
                    if (j < a) {
                        sx = r.sx0 + (int32_t)(j % w);
                        sy = r.sy0 + (int32_t)(j / w);
                        return;
                    }
                    j -= a;
                }
            };
            // the wave's first sub-block and its camera rays, before the scene is in: the kernel
            // arguments' scalar loads and the ray arithmetic overlap the preload's round trip
            int32_t sx0 = 0, sy0 = 0;
            f3 d0;
            constexpr bool kGivenRay = true;
            auto first_rays = [&]() {
                if (c0 + wave < total) locate(c0 + wave, sx0, sy0, true);
                ERAY_TRACE_WAVE0(11);
                d0 = camera_dir(cam, p, (uint32_t)sx0 * kSubW + lane % kSubW, cam_row(rm, (uint32_t)sy0 * kBlkH + lane / kSubW));
                asm volatile("" : "+v"(d0.x), "+v"(d0.y), "+v"(d0.z));  // here, not after the barrier
            };
            auto detail = [&](const auto& sc, const uint32_t pobj, const uint32_t* pstart) {
                // Rounds of nk * 4 sub-blocks, dealt in snake order: in odd rounds the last
                // workgroup takes the first sub-blocks, so the waves whose first sub-block came
                // from the ordered list's heavy head (the longest chains) take the light tail
                // of the second round.  (A device-wide atomic work counter instead measured
                // 2.5x slower at 3840x2160 / 70k: one hot address under the frame's write stream.)
                const uint32_t round = nk * nwaves;
                auto job = [&](uint32_t r, bool& valid, bool& coop) {  // round r's sub-block of this wave
                    const bool odd = (r & 1u) && kSnake;
                    const uint32_t first = r * round + (odd ? round - nwaves - c0 : c0);
                    valid = first < total;
                    coop = first < heavy;
                    return odd ? first + (nwaves - 1 - wave) : first + wave;
                };
                // Binned meshes with a detail list: the wave's next sub-block — its list entry and
                // its bin range in the first binned object pobj (bin starts pstart) — is loaded
                // during the current one (vector loads, used one sub-block later), so a round
                // after the first starts with its search, not with two dependent round trips.
                uint32_t nx_e = 0, nx_lo = 0, nx_hi = 0;  // (VGPRs: the loads' results)
                bool nx_range = false;                    // nx_lo / nx_hi were issued
                for (uint32_t r = 0;; ++r) {  // workgroup-uniform
                    bool valid, coop;
                    const uint32_t j = job(r, valid, coop);
                    if (!valid) break;
                    const bool active = j < total;
                    int32_t sx = sx0, sy = sy0;
                    PreRange pre{0u, 0u, false};
                    const bool have_pre = pstart && r != 0 && nx_range;
                    if (r != 0 && active) {
                        if (pstart) {  // prefetched during the previous sub-block
                            const uint32_t e = __builtin_amdgcn_readfirstlane(nx_e);
                            sx = (int32_t)(e & 0xffffu);
                            sy = (int32_t)(e >> 16);
                        } else {
                            locate(j, sx, sy);
                        }
                    }
                    if (have_pre && active)
                        pre = PreRange{(uint32_t)__builtin_amdgcn_readfirstlane(nx_lo),
                                       (uint32_t)__builtin_amdgcn_readfirstlane(nx_hi), true};
                    // the next round's sub-block of this wave: its list entry now, its bin range
                    // once this sub-block's first hits are known (mid)
                    bool nvalid = false, ncoop = false;
                    const uint32_t jn = job(r + 1, nvalid, ncoop);
                    const bool nactive = nvalid && jn < total && pstart;
                    if (nactive) nx_e = vload_u32(dlist, lpos(jn));
                    nx_range = false;
                    auto mid = [&]() {
                        if (!nactive) return;
                        const uint32_t e = __builtin_amdgcn_readfirstlane(nx_e);
                        const uint32_t bin = ((cam_row(rm, (e >> 16) * kBlkH) + kBinH - p.bin_phase) / kBinH) * p.bins_x +
                                             (e & 0xffffu);
                        nx_lo = vload_u32(pstart, bin);
                        nx_hi = vload_u32(pstart, bin + 1);
                        nx_range = true;
                    };
                    // the ordered detail list's heavy sub-blocks (bins of several chunks) come
                    // first, so the longest chains start in the first round (coop: shared by the
                    // workgroup in builds that keep the cooperative paths, render_sub)
                    // (the first sub-block's rays by value: a pointer would keep them in scratch memory)
                    render_sub<kCull, kLdsTiles, kMat, kDense>(p, fo, cam, rm, sc, (uint32_t)sx * kSubW, (uint32_t)sy * kBlkH,
                                                       active, s_hot, s_cull, s_bins, s_rgb, s_ppm, aligned,
                                                       kGivenRay && r == 0, d0, coop, pre, pobj, mid);
                }
            };
            if constexpr (kLdsScene) {
                if (v != bid) __syncthreads();  // the previous frame's reads of the LDS scene are done
                const FrameHot hf{objs, h_lights, culls, h_tris, static_cast<const TriShade*>(h_aux), h_counts, h_total_tris,
                                  h_total_sub, grid};
                const SceneLds sc = preload_scene(hf, dyn, first_rays);
                __syncthreads();
                detail(sc, ~0u, nullptr);
            } else {
                const SceneGlobal sc{p, objs, culls};
                uint32_t pobj = ~0u;  // the first binned object (culled large-mesh builds with a list)
                const uint32_t* pstart = nullptr;
                if constexpr (kLdsTiles && kCull) {
                    // the first object's descriptor is loaded before the list entry is waited for:
                    // the first sub-block's two inputs in one round trip
                    const ObjGeom g0 = nobj ? sc.geom(0) : ObjGeom{};
                    // The scalar cache lines of what the shading reads after the search — the first
                    // object's MaterialDesc (its two 64-B lines) and the lights — touched now, in
                    // the same round trip: their first reads come after the search, each a scalar
                    // cache miss in a dependent chain otherwise
                    uint32_t warm = 0;
                    if (nobj) {
                        const uint32_t* od = reinterpret_cast<const uint32_t*>(objs);
                        warm = load_const(od + 16, 0) ^ load_const(od + 32, 0);
                    }
                    if (h_counts >> 16) warm ^= load_const(reinterpret_cast<const uint32_t*>(h_lights), 0);
                    if ((h_counts >> 16) > 2u) warm ^= load_const(reinterpret_cast<const uint32_t*>(h_lights + 2), 0);
                    first_rays();
                    asm volatile("" ::"s"(warm));
                    if (dlist)
                        for (uint32_t oi = 0; oi < nobj; ++oi) {
                            const ObjGeom g = oi == 0 ? g0 : sc.geom(oi);
                            if (g.bin_start) {
                                pobj = oi;
                                pstart = g.bin_start;
                                break;
                            }
                        }
                } else {
                    first_rays();
                }
                ERAY_TRACE_WAVE0(12);
                detail(sc, pobj, pstart);
            }
        }
        ERAY_TRACE_POINT(1);
        if (nd < grid) {
            return;
        }
    }

    // ---- background of the non-detail sub-blocks ---------------------------------------------
    if (separate_fill) return;  // fill_kernel writes the background beside this launch
    const uint32_t nf = min(nd < grid ? grid - nd : grid, p.fill_cap ? p.fill_cap : grid);  // filling workgroups
    const uint32_t f = nd < grid ? bid - nd : bid;
    if (f >= nf) return;
    ERAY_TRACE_POINT(2);
    // paced beside detail work — except small scenes whose ring of frames exceeds the Infinity Cache
    // (C2 in 16 slots: 55.7 paced, 51.7 us unpaced per 8 frames; the binned north-star frame in
    // 4 slots 25.1 paced, 29.7 unpaced), profiles/r05/ab/
    const bool pace = nd != 0 && (p.detail_occ || !(p.launch_flags & kLaunchRingBeyondCache));
    fill_frames<kDev>(p, f, nf, wave, lane, aligned, pace);
    ERAY_TRACE_POINT(3);
}

// The background alone, beside a detail-only frame kernel on another stream (FrameParams::
// separate_fill): small workgroups that hold few registers, so the fill waves do not take the
// register budget of the large-mesh detail build.  (A flat order — every output array as one
// byte range, one workgroup per CU, 6.9 TB/s alone at 7680x4320 in scripts/microbench/
// fill_pat.hip — wrote C5's background in 263 us beside the detail kernel against 151 us in
// blocks from two workgroups per CU: profiles/r04/ab/ab_flat_fill.txt, launch spans.)
template <bool kDev>
__global__ void __launch_bounds__(kWG) fill_kernel(FrameParams p) {
    fill_frames<kDev>(p, blockIdx.x, gridDim.x, threadIdx.x >> 6, threadIdx.x & 63, p.aligned != 0, true);
}

// Measurement only (eray_time_write_ceiling): the launch's frames' background bytes written by the
// plainest store stream there is — scripts/microbench/fill_pace.hip's `blk` pattern: one
// workgroup per CU, wave w of the grid's W takes 64 x 4 blocks w, w + W, ... over all the
// launch's frames, each block's 16-B write-through stores at per-lane offsets computed per block,
// no pacing, no role logic, no scene.  The same bytes as the frame kernel's background, into the
// same ring slots, so the frame kernel's fill floor can be compared with the chip's own write
// rate for that ring in the same process.  Whole blocks only (aligned frames, rows % 4 == 0).
__global__ void __launch_bounds__(kWG) ceiling_fill_kernel(FrameParams p) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t tiles_x = p.img_w / kBlkW, bands = p.rows / kBlkH, nblk = tiles_x * bands;
    const uint32_t nw = gridDim.x * (kWG / 64), w = blockIdx.x * (kWG / 64) + wave;
    for (uint32_t b = w; b < nblk * p.nframes; b += nw) {
        const uint32_t fr = b / nblk, k = b - fr * nblk, bx = k % tiles_x, by = k / tiles_x;
        const FrameOut o = frame_out(p, fr);
        if (o.rgb) {
#pragma unroll
            for (uint32_t i = lane; i < kBlkH * 48u; i += 64) {
                const uint32_t r = i / 48u, c = i % 48u;
                const float4 v = bg_rgb4(c % 3u);
                stream16_pol<false>(o.rgb, 12u * ((by * kBlkH + r) * p.img_w + bx * kBlkW) + 16u * c, 0u,
                                    make_uint4(__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z),
                                               __float_as_uint(v.w)));
            }
        }
        if (o.ppm && lane < 48u) {
            const uint32_t r = lane / 12u, c = lane % 12u;
            stream16_pol<false>(o.ppm, 3u * ((p.rows - kBlkH - by * kBlkH + r) * p.img_w + bx * kBlkW) + 16u * c, 0u,
                                bg_ppm16(c % 3u));
        }
        if (o.face) {
            const uint32_t r = lane / 16u, c = lane % 16u;
            stream16_pol<false>(o.face, 4u * ((by * kBlkH + r) * p.img_w + bx * kBlkW) + 16u * c, 0u,
                                make_uint4(~0u, ~0u, ~0u, ~0u));
        }
    }
}

// Image<Color>::save_as_ppm body: byte row k = image row h-1-k.
__global__ void __launch_bounds__(256) pack_ppm_kernel(const float* __restrict__ rgb, uint32_t w,
                                                       uint32_t h, uint8_t* __restrict__ out) {
    const size_t n = (size_t)w * h;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t y = (uint32_t)(i / w), x = (uint32_t)(i - (size_t)y * w);
        const float* c = rgb + 3 * i;
        uint8_t* o = out + 3 * ((size_t)(h - 1 - y) * w + x);
        o[0] = (uint8_t)sat_u8(c[0] * 255.0f);
        o[1] = (uint8_t)sat_u8(c[1] * 255.0f);
        o[2] = (uint8_t)sat_u8(c[2] * 255.0f);
    }
}

}  // namespace

hipError_t launch_tri_precompute(const float* pos, const float* nrm, const float* uv, uint32_t T,
                                 TriHot* hot, TriShade* shade, hipStream_t s) {
    if (!T) return hipSuccess;
    tri_precompute_kernel<<<(T + 255) / 256, 256, 0, s>>>(pos, nrm, uv, T, hot, shade);
    return hipGetLastError();
}

namespace {
// Persistent grid: as many workgroups as are resident at once (occupancy API), capped by the
// work (fill blocks or detail sub-blocks, whichever needs more workgroups).
// frame_kernel's h_roles (a preloaded dword): grid | detail_wgs << 12 | (frames - 1) << 24 |
// fill_first << 30 | separate_fill << 31 (grid <= kMaxFrameGrid, frames <= kMaxFramesPerLaunch)
constexpr uint32_t kMaxFrameGrid = 4095;
uint32_t frame_roles(uint32_t grid, const FrameParams& q) {
    return (grid & 0xfffu) | ((q.detail_wgs & 0xfffu) << 12) | (((q.nframes - 1u) & 63u) << 24) |
           ((q.fill_first ? 1u : 0u) << 30) |
           ((q.separate_fill ? 1u : 0u) << 31);
}

// frame_kernel's h_band: the band shift and stride of the row mapping in one dword
uint32_t band_word(const FrameParams& q) { return (q.band_shift & 31u) | (q.band_stride << 5); }
// frame_kernel's h_aux: TriShade records (LDS-scene builds) or the detail list
template <bool K>
const void* aux_arg(const FrameParams& q) {
    return K ? static_cast<const void*>(q.shade) : static_cast<const void*>(q.detail_list);
}

uint32_t device_cus() {
    static const uint32_t cus = [] {  // (thread-safe initialisation)
        int dev = 0, n = 0;
        return (hipGetDevice(&dev) == hipSuccess &&
                hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
                   ? (uint32_t)n
                   : 256u;
    }();
    return cus;
}

constexpr uint32_t kFillWgsPerCu = 1;

// A kernel launch, with its dispatch's own start / stop timestamps recorded into t[0] / t[1] when
// they are given (LaunchCtx: measurement only).
template <typename... KArgs, typename... Args>
hipError_t launch_k(void (*kernel)(KArgs...), uint32_t grid, size_t dyn, hipStream_t s, const hipEvent_t (&t)[2],
                    Args... args) {
    if (t[0])
        hipExtLaunchKernelGGL(kernel, dim3(grid), dim3(kWG), (uint32_t)dyn, s, t[0], t[1], 0u, (KArgs)args...);
    else
        kernel<<<grid, kWG, dyn, s>>>(args...);
    return hipGetLastError();
}

template <bool C, bool L, int M, bool K, bool D = false, bool V = false>
hipError_t launch_frame_kernel(const FrameParams& p, uint32_t want, size_t dyn, const LaunchCtx& lc, hipStream_t s) {
    static std::mutex mu;  // resident workgroups per CU of this build, per dynamic LDS size
    static int per_cu = -1;
    static size_t per_cu_dyn = 0;
    int wg_cu;
    {
        std::lock_guard<std::mutex> lock(mu);
        if (per_cu < 0 || per_cu_dyn != dyn) {
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, frame_kernel<C, L, M, K, D, V>, kWG, dyn) !=
                    hipSuccess ||
                per_cu <= 0)
                per_cu = 1;
            per_cu_dyn = dyn;
        }
        wg_cu = per_cu;
    }
    const uint32_t cus = device_cus();
    const uint32_t grid = min(min(want, (uint32_t)wg_cu * cus), kMaxFrameGrid);
    // Workgroups kept for the fill so that it overlaps a large detail area instead of following
    // it: one per 64 background blocks, at most 1/share of the grid.  Measured (graph-replayed
    // frames, profiles/ab/ab_knobs*.log): the fill needs enough store-issuing waves on every CU
    // (3840x2160 / 70k: 128 fill workgroups 52 us, 256 31 us, none 34 us) and the detail waves'
    // VALU issue; share 2 with the detail roles first is best for C2, C3 and 3840x2160 / 70k
    // (27.8 us; share 3 29.4-30.3, share 4 37), while a small-scene frame with more than one
    // round of detail sub-blocks (the cube at 3840x2160) wants one fill workgroup per CU
    // dispatched first (share 3, fill_first: 22.8 -> 20.4 us; at C2 fill_first costs 0.7 us).
    // blocks and detail sub-blocks of all the launch's frames (frames in flight)
    const uint32_t nblk = p.nframes * p.tiles_x * ((p.rows + kBlkH - 1) / kBlkH);
    const uint32_t total_sub = p.nframes * p.total_sub;
    auto detail_wgs = [&](float share) {
        return share >= 1.0f && grid >= 2 ? grid - max(min((uint32_t)((float)grid / share), (nblk + 63) / 64), 1u)
                                          : 0u;
    };
    FrameParams q = p;
    // (the dense large-mesh build, 4 workgroups per CU: one per CU fills, three do detail work —
    // the fill's store stream no longer needs the issue slots it did, round 5)
    q.detail_wgs = detail_wgs((L && D) ? 4.0f : 2.0f);
    q.fill_first = 0;
    q.detail_wgs_alt = 0;
    if (!L) {
        if (p.cam_state) {  // the count is on the device: frame_kernel picks the share
            q.detail_wgs_alt = detail_wgs(3.0f);
        } else if (total_sub > q.detail_wgs * (kWG / 64)) {
            q.detail_wgs = detail_wgs(3.0f);
            q.fill_first = 1;
        }
    }
    // large meshes: the fill roles take the first-dispatched workgroups — the 2-per-CU build (C3):
    // 13.0 -> 12.7-12.9 us; the dense build (3840x2160 / 70k, spill-free since round 3): 23.4 ->
    // 22.4 us (profiles/r03/ab/)
    if (L) q.fill_first = 1;
    q.separate_fill = 0;
    // Fill workgroups: one per CU writes the background where the fill has the GPU (nearly) to
    // itself — fewer concurrent write streams keep the HBM pages open (scripts/microbench/
    // fill_pat.hip: 3840x2160 beyond the cache 23-24 us with 2-4 per CU, 18.6 us with one; the
    // empty-scene floor 24.5 -> 21.3 us, C2's 37.2 -> 34.0 us per 8 frames) — but not beside
    // the binned meshes' detail waves, which take issue slots from fewer fill waves (3840x2160 /
    // 70k: 22.6 -> 28.2 us with one per CU), same-box A/B (profiles/r04/ab/ab_fill_cap.txt).
    q.fill_cap = L ? 0u : kFillWgsPerCu * cus;
    if constexpr (D) {
        // Separate fill: the dense build does detail work only, at most 2 workgroups per CU, and
        // fill_kernel's small workgroups (58 VGPRs) write the background beside it from a second
        // stream (fork / join by events, which a graph capture records as two parallel nodes).
        // Measured (profiles/ab/ab_sepfill.log): with many rounds of detail sub-blocks the detail
        // waves get the register budget the fill roles held (C5's frame 216 -> 190 us); with
        // ~2 rounds the single launch overlaps better (3840x2160 / 70k 27.9 vs 37.8 us).  Used
        // above 16 detail sub-blocks per CU (ERAY_RENDER_SEPARATE_FILL / _NO_SEPARATE_FILL force
        // it on / off).
        const bool separate = (p.launch_flags & kLaunchSeparateFill)     ? true
                              : (p.launch_flags & kLaunchNoSeparateFill) ? false
                                                                         : total_sub > 16u * cus;
        if (separate) {
            if (!lc.side || !lc.fork || !lc.join) return hipErrorInvalidValue;
            q.separate_fill = 1;
            q.detail_wgs = 0;
            q.fill_first = 0;
            const uint32_t dgrid = max(1u, min(min(grid, 2u * cus), (total_sub + kWG / 64 - 1) / (kWG / 64)));
            // (two per CU: beside the detail waves one per CU writes C5's background in 186 us
            // instead of 151, profiles/r04/ab/ab_fill_cap.txt launch spans)
            const uint32_t fgrid = max(1u, min(2u * cus, (nblk + 3) / 4));
            hipError_t e;
            if ((e = hipEventRecord(lc.fork, s)) != hipSuccess || (e = hipStreamWaitEvent(lc.side, lc.fork, 0)) != hipSuccess)
                return e;
            if ((e = launch_k(frame_kernel<C, L, M, K, D, V>, dgrid, dyn, s, lc.frame_t, q.objects, q.lights, q.cull,
                              q.tris, aux_arg<K>(q), q.nobj | (q.nlights << 16), q.total_tris, q.total_sub,
                              frame_roles(dgrid, q), band_word(q), q)) != hipSuccess)
                return e;
            if ((e = launch_k(fill_kernel<V>, fgrid, 0, lc.side, lc.fill_t, q)) != hipSuccess) return e;
            if (lc.fill_used) *lc.fill_used = 1u;
            if ((e = hipEventRecord(lc.join, lc.side)) != hipSuccess) return e;
            return hipStreamWaitEvent(s, lc.join, 0);
        }
    }
    return launch_k(frame_kernel<C, L, M, K, D, V>, grid, dyn, s, lc.frame_t, q.objects, q.lights, q.cull, q.tris,
                    aux_arg<K>(q), q.nobj | (q.nlights << 16), q.total_tris, q.total_sub, frame_roles(grid, q), band_word(q),
                    q);
}

template <bool C, int M, bool V>
hipError_t launch_frame_cs(const FrameParams& p, uint32_t want, const LaunchCtx& lc, hipStream_t s) {
    // small scenes are preloaded into LDS whole (no object then needs the LDS tiles); otherwise
    // everything is read from the device arrays
    if (p.lds_scene) {
        const size_t dyn = scene_lds_layout(p.nobj, p.nlights, p.total_tris, C).bytes;
        return launch_frame_kernel<C, false, M, true, false, V>(p, want, dyn, lc, s);
    }
    if (p.max_object_tris > kDirectMax) {
        if constexpr (!(M & kMatSpecPow)) {
            // more detail sub-blocks than the 2-per-CU grid's detail waves (half the grid, four
            // waves each: launch_frame_kernel) take in one round: the 3-per-CU build
            // (ERAY_RENDER_DENSE_DETAIL / _NO_DENSE_DETAIL force it on / off)
            const bool dense = (p.launch_flags & kLaunchDense)     ? true
                               : (p.launch_flags & kLaunchNoDense) ? false
                                                                   : p.nframes * p.total_sub > device_cus() * (kWG / 64);
            if (dense) return launch_frame_kernel<C, true, M, false, true, V>(p, want, 0, lc, s);
        }
        return launch_frame_kernel<C, true, M, false, false, V>(p, want, 0, lc, s);
    }
    return launch_frame_kernel<C, false, M, false, false, V>(p, want, 0, lc, s);
}
}  // namespace

hipError_t launch_render(const FrameParams& p_in, const LaunchCtx& lc, hipStream_t s) {
    FrameParams p = p_in;
    if (p.nframes < 1 || p.nframes > kMaxFramesPerLaunch || ((p.aa || p.bounces) && p.nframes != 1))
        return hipErrorInvalidValue;
    {  // the launch's output bytes against the Infinity Cache (FrameParams::store_nt)
        const uint64_t px = (uint64_t)p.nframes * p.rows * p.img_w;
        const uint64_t out = px * ((p.out_rgb ? 12u : 0u) + (p.out_ppm ? 3u : 0u) + (p.out_face ? 4u : 0u));
        p.store_nt = out > kInfinityCacheBytes ? 1u : 0u;
    }
    if (p.aa || p.bounces) return launch_trace(p, lc, s);
    const uint32_t by_n = (p.rows + kBlkH - 1) / kBlkH;
    const uint32_t nblk = p.tiles_x * by_n;
    if (!nblk) return hipSuccess;
    // enough workgroups for one fill block or one round of detail sub-blocks per wave (device-
    // camera mode: the detail count is not known here, so as many as fit)
    const uint32_t want = p.nframes * (p.cam_state ? max((nblk + 3) / 4, nblk) : max((nblk + 3) / 4, (p.total_sub + 3) / 4));
    const int mat = (p.spec_pow ? kMatSpecPow : 0) | (p.example_mat ? kMatExample : 0);
    // device-camera mode (the setup's CamState) is a separate build: args-mode frames carry no
    // branch or load for it
    if (p.cull && p.cam_state) {
        switch (mat) {
            case 0: return launch_frame_cs<true, 0, true>(p, want, lc, s);
            case kMatSpecPow: return launch_frame_cs<true, kMatSpecPow, true>(p, want, lc, s);
            case kMatExample: return launch_frame_cs<true, kMatExample, true>(p, want, lc, s);
            default: return launch_frame_cs<true, kMatSpecPow | kMatExample, true>(p, want, lc, s);
        }
    }
    if (p.cull) {
        switch (mat) {
            case 0: return launch_frame_cs<true, 0, false>(p, want, lc, s);
            case kMatSpecPow: return launch_frame_cs<true, kMatSpecPow, false>(p, want, lc, s);
            case kMatExample: return launch_frame_cs<true, kMatExample, false>(p, want, lc, s);
            default: return launch_frame_cs<true, kMatSpecPow | kMatExample, false>(p, want, lc, s);
        }
    }
    switch (mat) {
        case 0: return launch_frame_cs<false, 0, false>(p, want, lc, s);
        case kMatSpecPow: return launch_frame_cs<false, kMatSpecPow, false>(p, want, lc, s);
        case kMatExample: return launch_frame_cs<false, kMatExample, false>(p, want, lc, s);
        default: return launch_frame_cs<false, kMatSpecPow | kMatExample, false>(p, want, lc, s);
    }
}

hipError_t launch_write_ceiling(const FrameParams& p, uint32_t wgs_per_cu, const hipEvent_t (&t)[2], hipStream_t s) {
    if (!p.aligned || p.img_w % kBlkW || p.rows % kBlkH || p.nframes < 1 || !wgs_per_cu || wgs_per_cu > 8)
        return hipErrorInvalidValue;
    return launch_k(ceiling_fill_kernel, wgs_per_cu * device_cus(), 0, s, t, p);
}

hipError_t launch_pack_ppm(const float* rgb, uint32_t w, uint32_t h, uint8_t* out, hipStream_t s) {
    const size_t n = (size_t)w * h;
    if (!n) return hipSuccess;
    size_t blocks = (n + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    pack_ppm_kernel<<<(unsigned)blocks, 256, 0, s>>>(rgb, w, h, out);
    return hipGetLastError();
}

}  // namespace gpu
}  // namespace eray
