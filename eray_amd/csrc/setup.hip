// setup.hip — per-camera setup of the frame kernel, entirely on the device.
//
// A camera change (Scene::set_camera, scene.rs:39-54, before Engine::render, engine.rs:46-81)
// needs, before its frame: every triangle's culling record for the new camera, the objects'
// pixel rectangles and the frame's merged detail rectangles.  One kernel does it all and leaves
// the results in device memory (CamState, the object descriptors): nothing is read back, so the
// frame kernel can follow at once and a sequence of cameras can be replayed from one HIP graph.
// The last workgroup to finish (a device-scope counter) reduces the per-object accumulators and
// resets them and the counter for the next setup.
#include "device_math.hpp"
#include "face_rect.hpp"
#include "internal.hpp"

namespace eray {
namespace gpu {
namespace {

using namespace eray::dev;

constexpr int kSetupWG = 256;

// --------------------------------------------------------------------- culling record ------
// Derivation (u = 2^-24, all norms are 1-norms of the float inputs; d = normalised direction).
// The reference computes, in f32 from ao = C - a (C the camera centre),
//   det = -(d.n),  a_u = e2.(ao x d),  a_v = -(e1.(ao x d)),  u = a_u/det, v = a_v/det,
//   t = (ao.n)/det,  hit iff det >= 1e-6, t >= 0, u >= 0, v >= 0, u + v <= 1.
// In real arithmetic on the same float inputs these are linear in d:
//   det = d.(-n), a_u = d.w_u (w_u = e2 x ao), a_v = d.w_v (w_v = ao x e1), and
//   det - a_u - a_v = d.w_w (w_w = -(n + w_u + w_v)).
// Float evaluation errors (|d_i| <= 1 + 4u): |det_f - det| <= E_n = 4u|n|,
// |a_u_f - a_u| <= 8u|e2||ao|, |a_v_f - a_v| <= 8u|e1||ao|; an a_u within 2^-149|n| of 0 can
// still round u to -0 (accepted), hence the 2^-149|n| floors.  A hit needs u+v <= 1 after
// rounding, which implies d.w_w >= -(E_u + E_v + 1.01 E_n + 3.2u|n|).  So condition k certainly
// fails for direction d when d.w_k < -E_k.
// The camera's unnormalised direction is D(x', y') = (bl - C) + (vw x', 2y', 0) with bl, vw the
// reference's float viewport corner and width (camera.rs:57-76), so D.w_k = K + A x' + B y' is
// affine and its maximum over a pixel rectangle sits at a corner.  The reference's float
// direction differs from D/|D| by at most 4u S (S = |bl| + vw + 2 + |C|) before and 4u after
// normalisation, so condition k fails for every pixel of the rectangle when
//   max_rect (K + A x' + B y') < -T_k,
//   T_k = 2 * [ (E_k + 4u|w_k|) Dmax + 4u S |w_k| + 6u (|K| + |A| + |B|) ]
// (Dmax = largest |D| over the frame; factor 2 = safety).  t >= 0 does not depend on d: when
// ao.n < -2^-149 |n| (or |n|(1+8u) < 1e-6) no camera ray can hit the face and the whole
// record rejects.  Any non-finite input disables culling for the face (T = +inf).
__device__ TriCull cull_record(const TriHot& h, const CamDev& cam) {
    const double u = 0x1p-24;
    const float cx = cam.cx, cy = cam.cy, cz = cam.cz;
    const f3 e1f = mk3(h.q0.x, h.q0.y, h.q0.z), e2f = mk3(h.q0.w, h.q1.x, h.q1.y);
    const f3 nf = mk3(h.q1.z, h.q1.w, h.q2.x), af = mk3(h.q2.y, h.q2.z, h.q2.w);
    const f3 Cf = mk3(cx, cy, cz);
    const f3 aof = sub(Cf, af);        // exactly the reference's `*ray.start() - a`
    const float atf = dot0(aof, nf);   // exactly the reference's `ao.dot_product(&n)`
    // camera.rs:57-76 in f32, as the reference computes it
    const float vw = cam.ratio * 2.0f;
    const f3 bl = sub(sub(sub(Cf, divs(mk3(vw, 0.0f, 0.0f), 2.0f)), divs(mk3(0.0f, 2.0f, 0.0f), 2.0f)),
                      mk3(0.0f, 0.0f, cam.z_dist));
    // doubles from here on
    const double e1[3] = {e1f.x, e1f.y, e1f.z}, e2[3] = {e2f.x, e2f.y, e2f.z};
    const double n[3] = {nf.x, nf.y, nf.z}, ao[3] = {aof.x, aof.y, aof.z};
    const double blc[3] = {(double)bl.x - cx, (double)bl.y - cy, (double)bl.z - cz};
    auto n1 = [](const double* v) { return fabs(v[0]) + fabs(v[1]) + fabs(v[2]); };
    auto crs = [](const double* s, const double* o, double* r) {
        r[0] = s[1] * o[2] - s[2] * o[1];
        r[1] = s[2] * o[0] - s[0] * o[2];
        r[2] = s[0] * o[1] - s[1] * o[0];
    };
    double wu[3], wv[3], ww[3], wn[3];
    crs(e2, ao, wu);
    crs(ao, e1, wv);
    for (int k = 0; k < 3; ++k) {
        ww[k] = -(n[k] + wu[k] + wv[k]);
        wn[k] = -n[k];
    }
    const double nn = n1(n), ne1 = n1(e1), ne2 = n1(e2), nao = n1(ao);
    const double floor_n = nn * 0x1p-149;
    const double Eu = 8.0 * u * ne2 * nao + floor_n;
    const double Ev = 8.0 * u * ne1 * nao + floor_n;
    const double En = 4.0 * u * nn;
    const double Ew = (8.0 * u * ne2 * nao) + (8.0 * u * ne1 * nao) + 1.01 * En + 3.2 * u * nn + floor_n;
    // largest |D| over the frame (corners of x', y' in [0, 1]) and the magnitude scale S
    double dmax = 0.0;
    for (int cxr = 0; cxr < 2; ++cxr)
        for (int cyr = 0; cyr < 2; ++cyr) {
            double D0 = blc[0] + (double)vw * cxr, D1 = blc[1] + 2.0 * cyr, D2 = blc[2];
            double l = sqrt(D0 * D0 + D1 * D1 + D2 * D2);
            dmax = l > dmax ? l : dmax;
        }
    const double S = fabs((double)bl.x) + fabs((double)bl.y) + fabs((double)bl.z) + fabs((double)vw) + 2.0 +
                     fabs((double)cx) + fabs((double)cy) + fabs((double)cz);
    dmax = dmax * (1.0 + 1e-6) + 8.0 * u * S;
    const double* W[4] = {wu, wv, ww, wn};
    const double E[4] = {Eu, Ev, Ew, En};
    float A[4], B[4], K[4], Tt[4];
    bool finite = true;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const double* w = W[k];
        double Kd = blc[0] * w[0] + blc[1] * w[1] + blc[2] * w[2];
        double Ad = (double)vw * w[0];
        double Bd = 2.0 * w[1];
        double thr = 2.0 * ((E[k] + 4.0 * u * n1(w)) * dmax + 4.0 * u * S * n1(w) +
                            6.0 * u * (fabs(Kd) + fabs(Ad) + fabs(Bd)));
        thr = thr * (1.0 + 0x1p-20) + 0x1p-126;  // round the float threshold up
        A[k] = (float)Ad;
        B[k] = (float)Bd;
        K[k] = (float)Kd;
        Tt[k] = (float)thr;
        finite = finite && isfinite(A[k]) && isfinite(B[k]) && isfinite(K[k]) && isfinite(Tt[k]);
    }
    bool all_finite = finite && isfinite(atf) && isfinite(nn) && isfinite(nao) && isfinite(ne1) &&
                      isfinite(ne2) && isfinite(dmax);
    // t >= 0 fails for every camera ray / det >= 1e-6 is unreachable: reject the whole face
    bool reject_all = all_finite && (((double)atf < -floor_n * 2.0) || (nn * (1.0 + 8.0 * u) < 1e-6));
    if (!all_finite) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            A[k] = B[k] = K[k] = 0.0f;
            Tt[k] = __builtin_inff();
        }
    } else if (reject_all) {
        A[3] = B[3] = K[3] = 0.0f;
        Tt[3] = -__builtin_inff();
    }
    TriCull c;
    c.A = make_float4(A[0], A[1], A[2], A[3]);
    c.B = make_float4(B[0], B[1], B[2], B[3]);
    c.K = make_float4(K[0], K[1], K[2], K[3]);
    c.T = make_float4(Tt[0], Tt[1], Tt[2], Tt[3]);
    return c;
}

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
    const uint32_t o_first = lo < hi ? object_of(sp.obj_begin, sp.nobj, lo) : 0u;
    const uint32_t o_last = lo < hi ? object_of(sp.obj_begin, sp.nobj, hi - 1) : 0u;
    for (uint32_t j = tid; j < kSpan; j += kSetupWG)
        for (int k = 0; k < 4; ++k) s_acc[j][k] = 0u;
    __syncthreads();
    unsigned long long run = 0;  // binned faces: pairs of this chunk's faces so far
    for (uint32_t i0 = lo; i0 < hi && kMode != 2; i0 += kSetupWG) {  // workgroup-uniform
        const uint32_t i = i0 + tid;
        unsigned long long ar = 0;
        if (i < hi) {
            const TriCull c = cull_record(sp.hot[i], cam);
            sp.cull[i] = c;
            const uint32_t obj = object_of(sp.obj_begin, sp.nobj, i);
            int32_t r[4];
            const bool any = face_rect(c, sp.W, sp.H, r, s_poly + tid, kSetupWG);
            if (any) {
                uint32_t a[4];
                rect_words(r, a);
                if (obj - o_first < kSpan) max4(s_acc[obj - o_first], a);
                else max4(sp.acc + 4 * obj, a);  // (a workgroup spanning very many objects)
            }
            if (sp.range) {  // bins.hip: the face's bin rectangle, if its object is binned
                const uint32_t k = sp.objkey[obj];
                int4 g = make_int4(1, 0, 1, 0);
                if (k != ~0u && any) {
                    // bin row of camera row y: (y + kBinH - phase) / kBinH
                    g = make_int4(r[0] / (int32_t)kBinW, r[1] / (int32_t)kBinW,
                                  (r[2] + (int32_t)kBinH - (int32_t)sp.phase) / (int32_t)kBinH,
                                  (r[3] + (int32_t)kBinH - (int32_t)sp.phase) / (int32_t)kBinH);
                    ar = (unsigned long long)(g.y - g.x + 1) * (unsigned long long)(g.w - g.z + 1);
                }
                sp.range[i] = g;
                sp.area[i] = ar;
                sp.fkey[i] = k;
            }
        }
        if (sp.range) {  // the chunk's exclusive scan of the areas, in face order
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
        if (j < kTab)
            for (int k = 0; k < 4; ++k) s_tab[j][k] = (uint32_t)r[k];
    }
    __syncthreads();
    if (tid != 0) return;
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

hipError_t launch_set_camera(const CamDev& cam, CamDev* slot, hipStream_t s) {
    set_camera_kernel<<<1, 64, 0, s>>>(cam, slot);
    return hipGetLastError();
}

}  // namespace gpu
}  // namespace eray
