// setup.hip — per-camera setup of the frame kernel, entirely on the device.
//
// A camera change (Scene::set_camera, scene.rs:39-54, before Engine::render, engine.rs:46-81)
// needs, before its frame: every triangle's culling record for the new camera, the objects'
// pixel rectangles and the frame's merged detail rectangles.  One kernel does it all and leaves
// the results in device memory (CamState, the object descriptors): nothing is read back, so the
// frame kernel can follow at once and a sequence of cameras can be replayed from one HIP graph.
// The last workgroup to finish (a device-scope counter) reduces the per-object accumulators and
// resets them and the counter for the next setup.
#include "cull_record.hpp"
#include "device_math.hpp"
#include "face_rect.hpp"
#include "internal.hpp"

namespace eray {
namespace gpu {
namespace {

using namespace eray::dev;

constexpr int kSetupWG = 256;

// the object owning triangle i (objects are consecutive triangle ranges)
__device__ __forceinline__ uint32_t object_of(const uint32_t* begin, uint32_t nobj, uint32_t i) {
    if (nobj <= 1) return 0u;
    uint32_t lo = 0, hi = nobj;  // last object whose first triangle is <= i
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (begin[mid] <= i) lo = mid;
        else hi = mid;
    }
    return lo;
}

// rectangle accumulator words of one face rectangle: (~x0, x1 + 1, ~y0, y1 + 1), max-reduced
__device__ __forceinline__ void rect_words(const int32_t (&r)[4], uint32_t (&a)[4]) {
    a[0] = ~(uint32_t)r[0];
    a[1] = (uint32_t)r[1] + 1u;
    a[2] = ~(uint32_t)r[2];
    a[3] = (uint32_t)r[3] + 1u;
}

// Per-object unions without contended atomics: workgroup b owns the contiguous triangle chunk
// [b * chunk, (b + 1) * chunk), whose objects are a contiguous run [o_first, o_last].  It reduces
// its faces' rectangles per object in LDS; an object strictly inside the run belongs to this
// workgroup alone (its union is final and stored to acc), the run's two end objects may continue
// in the neighbours (stored as this workgroup's partials).  The last workgroup combines: a scene
// whose one object spans every workgroup costs one counter increment per workgroup, not four
// atomics per wave on the same four words (70k faces: 73 -> a few us).
constexpr uint32_t kSpan = kSetupWG;  // objects per workgroup reduced in LDS (more: global atomics)
constexpr uint32_t kTab = 2048;       // objects the last workgroup combines in LDS (more: in acc)
static_assert(kSetupBatchMaxObjects <= kSpan, "a batched setup keeps every object's union in LDS");

// exclusive scan of v over the workgroup (thread order); *total gets the sum.  s_w: 4 words of
// LDS, free on entry and on return.
__device__ __forceinline__ unsigned long long block_exclusive_scan(unsigned long long v, unsigned long long* s_w,
                                                                   unsigned long long* total) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    unsigned long long incl = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const unsigned long long y = __shfl_up(incl, off);
        if ((int)lane >= off) incl += y;
    }
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    unsigned long long before = 0, all = 0;
#pragma unroll
    for (uint32_t w = 0; w < kSetupWG / 64; ++w) {
        before += w < wave ? s_w[w] : 0ull;
        all += s_w[w];
    }
    *total = all;
    __syncthreads();
    return before + incl - v;
}

__device__ __forceinline__ void max4(uint32_t* dst, const uint32_t (&a)[4]) {
    for (int k = 0; k < 4; ++k) atomicMax(dst + k, a[k]);
}

// kMode 0: one workgroup does everything (small scenes); kMode 1: the chunks' workgroups reduce
// and publish (no finalisation); kMode 2: one workgroup combines the nparts workgroups' partials;
// kMode 3: workgroup k does kMode 0's work for camera k of a batch, into its own slots.
// (A last-workgroup finalisation inside kMode 1 cost every workgroup a device-scope fence — an
// L2 write-back on this multi-XCD part — and a contended counter: 59 us at 70k faces.)
template <int kMode>
__global__ void __launch_bounds__(kSetupWG) camera_setup_kernel(SetupParams sp, uint32_t nparts) {
    __shared__ double s_poly[16 * kSetupWG];  // face_rect's clip output, 128 B per thread
    __shared__ uint32_t s_acc[kSpan][4];      // this workgroup's objects (o - o_first)
    __shared__ uint32_t s_tab[kMode == 1 ? 1 : kTab][4];  // the combining workgroup's per-object unions
    __shared__ unsigned long long s_scan[kSetupWG / 64];
    if (kMode == 3) {  // camera blockIdx.x of the batch: its slots
        sp.cam += blockIdx.x;
        sp.cull += (size_t)blockIdx.x * sp.T;
        sp.objs += (size_t)blockIdx.x * sp.nobj;
        sp.state += blockIdx.x;
    }
    const CamDev cam = *sp.cam;
    const uint32_t tid = threadIdx.x;
    const uint32_t chunk = kMode == 3 ? sp.T : (sp.T + gridDim.x - 1) / gridDim.x;
    const uint32_t lo = kMode == 3 ? 0u : min(blockIdx.x * chunk, sp.T), hi = min(lo + chunk, sp.T);
    // several cameras at once (sp.ncam > 1, binned scenes' camera paths): face i is face i % T1 of
    // camera i / T1, object k * nobj1 + o of camera k is that camera's copy of object o (SetupParams)
    const bool multi = kMode != 3 && sp.ncam > 1;
    auto vobject = [&](uint32_t i) -> uint32_t {
        if (!multi) return object_of(sp.obj_begin, sp.nobj, i);
        const uint32_t k = i / sp.T1;
        return k * sp.nobj1 + object_of(sp.obj_begin, sp.nobj1, i - k * sp.T1);
    };
    const uint32_t o_first = lo < hi ? vobject(lo) : 0u;
    const uint32_t o_last = lo < hi ? vobject(hi - 1) : 0u;
    for (uint32_t j = tid; j < kSpan; j += kSetupWG)
        for (int k = 0; k < 4; ++k) s_acc[j][k] = 0u;
    __syncthreads();
    unsigned long long run = 0;  // binned faces: pairs of this chunk's faces so far
    CullCam cc{};
    uint32_t cc_k = ~0u;
    for (uint32_t i0 = lo; i0 < hi && kMode != 2; i0 += kSetupWG) {  // workgroup-uniform
        const uint32_t i = i0 + tid;
        unsigned long long ar = 0;
        if (i < hi) {
            // (keep_all: the general tracer's viewport, jittered rays reach -1/W and -1/H)
            const double xa = sp.keep_all ? -2.0 / (double)sp.W : 0.0, ya = sp.keep_all ? -2.0 / (double)sp.H : 0.0;
            const uint32_t kc = multi ? i / sp.T1 : 0u;  // (the face's camera)
            if (kc != cc_k) {  // the camera's part of the records: once per camera and thread
                cc = cull_cam(multi ? sp.cam[kc] : cam, xa, 1.0, ya, 1.0);
                cc_k = kc;
            }
            const TriCull c = cull_record(sp.hot[i - kc * sp.T1], cc);
            sp.cull[i] = c;
            const uint32_t obj = vobject(i);
            int32_t r[4];
            // a face none of whose rays can pass anywhere in the viewport (the frame kernel's own
            // f32 rectangle test, the viewport widened: about half of a closed mesh's faces, the
            // back-facing ones) needs no double-precision clip
            const bool none = cull_rejects(c, (float)xa - 1e-6f, 1.0f + 1e-6f, (float)ya - 1e-6f, 1.0f + 1e-6f);
            const bool any = !none && face_rect(c, sp.W, sp.H, r, s_poly + tid, kSetupWG, xa, ya);
            if (any) {
                uint32_t a[4];
                rect_words(r, a);
                if (obj - o_first < kSpan) max4(s_acc[obj - o_first], a);
                else max4(sp.acc + 4 * obj, a);  // (a workgroup spanning very many objects)
            }
            if (sp.range) {  // bins.hip: the face's bin rectangle, if its object is binned
                uint32_t k = sp.objkey[multi ? obj % sp.nobj1 : obj];  // (camera kc's copy: kc * nb1 + k)
                if (multi && k != ~0u) k += kc * sp.nb1;
                int4 g = make_int4(1, 0, 1, 0);
                if (k != ~0u && any) {
                    // bin row of camera row y: (y + kBinH - phase) / kBinH
                    g = make_int4(r[0] / (int32_t)kBinW, r[1] / (int32_t)kBinW,
                                  (r[2] + (int32_t)kBinH - (int32_t)sp.phase) / (int32_t)kBinH,
                                  (r[3] + (int32_t)kBinH - (int32_t)sp.phase) / (int32_t)kBinH);
                    ar = (unsigned long long)(g.w - g.z + 1) *  // (units: rows, or bins)
                         (bin_segments(sp) ? 1ull : (unsigned long long)(g.y - g.x + 1));
                }
                sp.range[i] = g;
                sp.area[i] = ar;
                sp.fkey[i] = k;
            }
        }
        if (sp.range) {  // the chunk's exclusive scan of the units, in face order
            unsigned long long all = 0;
            const unsigned long long ex = block_exclusive_scan(ar, s_scan, &all);
            if (i < hi) sp.first_local[i] = run + ex;
            run += all;
        }
    }
    if (kMode == 1 && sp.range && tid == 0) sp.boff[blockIdx.x] = run;  // the chunk's total
    if (kMode == 2 && sp.range) {  // chunk totals -> chunk offsets, and all pairs at [nparts]
        constexpr uint32_t kPer = kSetupMaxBlocks / kSetupWG;  // chunks per thread, consecutive
        unsigned long long v[kPer], sum = 0;
#pragma unroll
        for (uint32_t k = 0; k < kPer; ++k) {
            const uint32_t b = tid * kPer + k;
            v[k] = b < nparts ? sp.boff[b] : 0ull;
            sum += v[k];
        }
        unsigned long long all = 0;
        unsigned long long ex = block_exclusive_scan(sum, s_scan, &all);
#pragma unroll
        for (uint32_t k = 0; k < kPer; ++k) {
            const uint32_t b = tid * kPer + k;
            if (b < nparts) sp.boff[b] = ex;
            ex += v[k];
        }
        if (tid == 0) sp.boff[nparts] = all;
    }
    __syncthreads();
    constexpr bool single = kMode == 0 || kMode == 3;
    if (kMode == 1) {  // publish: inner objects' unions are final, the two end objects' are partial
        const uint32_t span = lo < hi ? min(o_last - o_first + 1, kSpan) : 0u;
        for (uint32_t j = tid; j < span; j += kSetupWG) {
            const uint32_t o = o_first + j;
            if (o == o_first || o == o_last) continue;
            for (int k = 0; k < 4; ++k) sp.acc[4 * o + k] = s_acc[j][k];
        }
        if (tid == 0) {
            uint32_t* pb = sp.part + 10 * blockIdx.x;
            pb[0] = lo < hi ? o_first : ~0u;
            pb[5] = lo < hi ? o_last : ~0u;
            for (int k = 0; k < 4; ++k) {
                pb[1 + k] = s_acc[0][k];
                pb[6 + k] = lo < hi && o_last - o_first < kSpan ? s_acc[o_last - o_first][k] : 0u;
            }
        }
        return;
    }
    // ---- one workgroup: every object's union
    const bool in_lds = sp.nobj <= kTab;
    if (single && sp.nobj <= kSpan) {
        for (uint32_t j = tid; j < sp.nobj; j += kSetupWG) {
            uint32_t w[4];
            for (int k = 0; k < 4; ++k) w[k] = s_acc[j][k];
            for (int k = 0; k < 4; ++k) s_tab[j][k] = w[k];
        }
    } else if (in_lds) {
        for (uint32_t j = tid; j < sp.nobj; j += kSetupWG)
            for (int k = 0; k < 4; ++k) {
                s_tab[j][k] = sp.acc[4 * j + k];
                sp.acc[4 * j + k] = 0u;  // zero for the next setup
            }
        __syncthreads();
        if (single) {  // more objects than kSpan: the first kSpan are still in s_acc
            for (uint32_t j = tid; j < min(sp.nobj, kSpan); j += kSetupWG)
                for (int k = 0; k < 4; ++k) s_tab[j][k] = max(s_tab[j][k], s_acc[j][k]);
        } else {
            for (uint32_t b = tid; b < nparts; b += kSetupWG) {
                const uint32_t* pb = sp.part + 10 * b;
                if (pb[0] != ~0u) {
                    uint32_t a[4] = {pb[1], pb[2], pb[3], pb[4]};
                    max4(s_tab[pb[0]], a);
                }
                if (pb[5] != ~0u) {
                    uint32_t a[4] = {pb[6], pb[7], pb[8], pb[9]};
                    max4(s_tab[pb[5]], a);
                }
            }
        }
    } else {  // very many objects: combine in the global accumulators
        if (single) {
            for (uint32_t j = tid; j < min(sp.nobj, kSpan); j += kSetupWG) {
                uint32_t a[4] = {s_acc[j][0], s_acc[j][1], s_acc[j][2], s_acc[j][3]};
                max4(sp.acc + 4 * j, a);
            }
        } else {
            for (uint32_t b = tid; b < nparts; b += kSetupWG) {
                const uint32_t* pb = sp.part + 10 * b;
                if (pb[0] != ~0u) {
                    uint32_t a[4] = {pb[1], pb[2], pb[3], pb[4]};
                    max4(sp.acc + 4 * pb[0], a);
                }
                if (pb[5] != ~0u) {
                    uint32_t a[4] = {pb[6], pb[7], pb[8], pb[9]};
                    max4(sp.acc + 4 * pb[5], a);
                }
            }
        }
        __threadfence();
    }
    __syncthreads();
    for (uint32_t j = tid; j < sp.nobj; j += kSetupWG) {
        uint32_t w[4];
        if (in_lds) {
            for (int k = 0; k < 4; ++k) w[k] = s_tab[j][k];
        } else {
            for (int k = 0; k < 4; ++k) w[k] = atomicExch(sp.acc + 4 * j + k, 0u);  // read and reset
        }
        int32_t r[4];
        if (w[1] == 0) {  // no face can be hit (or no faces)
            r[0] = r[2] = 1;
            r[1] = r[3] = 0;
        } else {
            r[0] = (int32_t)~w[0];
            r[1] = (int32_t)w[1] - 1;
            r[2] = (int32_t)~w[2];
            r[3] = (int32_t)w[3] - 1;
        }
        if (kMode == 3) sp.objs[j] = sp.objs_src[j];  // the slot's descriptor, then its rectangle
        for (int k = 0; k < 4; ++k) sp.objs[j].g.rect[k] = r[k];
        // a camera path's union (binned objects: bins.hip folds in their narrowed rectangles)
        if (sp.path_union && sp.objkey[multi ? j % sp.nobj1 : j] == ~0u)
            union_rect(sp.path_union, sp.union_nobj, j % sp.union_nobj, r);
        if (j < kTab)
            for (int k = 0; k < 4; ++k) s_tab[j][k] = (uint32_t)r[k];
    }
    __syncthreads();
    if (tid != 0) return;
    if (multi) {  // (binned scenes: bins.hip narrows the rectangles and lists the detail sub-blocks)
        for (uint32_t k = 0; k < sp.ncam; ++k) sp.state[k].cam = sp.cam[k];
        return;
    }
    CamState& st = *sp.state;
    st.cam = cam;
    if (sp.binned) return;  // bins.hip narrows the rectangles and lists the detail sub-blocks
    // detail rectangles in sub-block units (16 px x 4 rank-local rows), made disjoint by merging
    // overlapping ones into their bounding box; more than kMaxRects widen the last one
    int32_t rects[kMaxRects][4];
    uint32_t nrect = 0;
    const int32_t rows_i = (int32_t)sp.rows, w_i = (int32_t)sp.W;
    for (uint32_t j = 0; j < sp.nobj; ++j) {
        int32_t r[4];
        for (int k = 0; k < 4; ++k) r[k] = j < kTab ? (int32_t)s_tab[j][k] : sp.objs[j].g.rect[k];
        int32_t x0 = r[0], x1 = r[1], y0, y1;  // camera rows -> rank-local rows
        band_local_range(sp.row0, sp.band_shift, sp.band_stride, r[2], r[3], &y0, &y1);
        x1 = x1 < w_i - 1 ? x1 : w_i - 1;
        y0 = y0 > 0 ? y0 : 0;
        y1 = y1 < rows_i - 1 ? y1 : rows_i - 1;
        if (x0 > x1 || y0 > y1) continue;
        const int32_t q[4] = {x0 / 16, x1 / 16, y0 / 4, y1 / 4};
        if (nrect == (uint32_t)kMaxRects) {
            int32_t* l = rects[kMaxRects - 1];
            l[0] = min(l[0], q[0]);
            l[1] = max(l[1], q[1]);
            l[2] = min(l[2], q[2]);
            l[3] = max(l[3], q[3]);
            continue;
        }
        for (int k = 0; k < 4; ++k) rects[nrect][k] = q[k];
        ++nrect;
    }
    for (bool merged = true; merged;) {
        merged = false;
        for (uint32_t x = 0; x < nrect && !merged; ++x)
            for (uint32_t y = x + 1; y < nrect && !merged; ++y) {
                int32_t* ra = rects[x];
                const int32_t* rb = rects[y];
                if (ra[0] > rb[1] || rb[0] > ra[1] || ra[2] > rb[3] || rb[2] > ra[3]) continue;
                ra[0] = min(ra[0], rb[0]);
                ra[1] = max(ra[1], rb[1]);
                ra[2] = min(ra[2], rb[2]);
                ra[3] = max(ra[3], rb[3]);
                for (uint32_t z = y; z + 1 < nrect; ++z)
                    for (int k = 0; k < 4; ++k) rects[z][k] = rects[z + 1][k];
                --nrect;
                merged = true;
            }
    }
    uint32_t total = 0;
    for (uint32_t k = 0; k < nrect; ++k) {
        total += (uint32_t)(rects[k][1] - rects[k][0] + 1) * (uint32_t)(rects[k][3] - rects[k][2] + 1);
        for (int q = 0; q < 4; ++q) st.rects[k][q] = rects[k][q];
    }
    st.nrect = nrect;
    st.total_sub = total;
}

__global__ void set_camera_kernel(CamDev cam, CamDev* slot) {
    if (threadIdx.x == 0) *slot = cam;
}

__global__ void __launch_bounds__(256) union_flush_kernel(int32_t* __restrict__ acc, uint32_t nobj,
                                                          int32_t* __restrict__ host) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < 4 * nobj; i += gridDim.x * 256u) {
        if (host) host[i] = acc[i];
        acc[i] = i < 2 * nobj ? 0x7fffffff : (int32_t)0x80000000;
    }
}

}  // namespace

hipError_t launch_camera_setup(const SetupParams& sp, hipStream_t s) {
    const uint32_t blocks = setup_blocks(sp.T);
    if (blocks == 1 && !sp.range) {  // (binned faces' pair offsets come from the two-kernel form)
        camera_setup_kernel<0><<<1, kSetupWG, 0, s>>>(sp, 1u);
        return hipGetLastError();
    }
    camera_setup_kernel<1><<<blocks, kSetupWG, 0, s>>>(sp, blocks);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    camera_setup_kernel<2><<<1, kSetupWG, 0, s>>>(sp, blocks);
    return hipGetLastError();
}

hipError_t launch_camera_setup_batch(const SetupParams& sp, uint32_t ncam, hipStream_t s) {
    if (sp.binned || sp.nobj > kSetupBatchMaxObjects) return hipErrorInvalidValue;
    if (!ncam) return hipSuccess;
    camera_setup_kernel<3><<<ncam, kSetupWG, 0, s>>>(sp, 1u);
    return hipGetLastError();
}

hipError_t launch_union_flush(int32_t* acc, uint32_t nobj, int32_t* host, hipStream_t s) {
    if (!nobj) return hipSuccess;
    union_flush_kernel<<<(4 * nobj + 255) / 256 < 64 ? (4 * nobj + 255) / 256 : 64, 256, 0, s>>>(acc, nobj, host);
    return hipGetLastError();
}

hipError_t launch_set_camera(const CamDev& cam, CamDev* slot, hipStream_t s) {
    set_camera_kernel<<<1, 64, 0, s>>>(cam, slot);
    return hipGetLastError();
}

}  // namespace gpu
}  // namespace eray
