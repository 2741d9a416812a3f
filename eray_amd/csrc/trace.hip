// trace.hip — the general tracer on gfx950: Engine::render with anti-aliasing and reflection
// bounces (src/lib/engine.rs:46-81, 112-228).
//
// The frame kernel (render.hip) is specialised for what the reference's default engine does —
// one primary ray per pixel at the integer pixel corner, no recursion — and its culling
// records, pixel rectangles and screen bins all assume those rays.  Jittered anti-aliasing
// rays and reflected rays go anywhere, so this kernel is the plain form of the same semantics:
// one thread per pixel (a 256-thread workgroup owns a 64 x 4 pixel tile, each wave a 16 x 4
// sub-block), every ray finds each object's FIRST face whose Triangle::intersects passes
// (Object::intersects, object.rs:58-81: bbox test, then the faces in index order), with the
// triangle records read through L1/L2 (TriHot, 48 B) — camera rays from the faces their wave can
// reach (the background skip below), the others from every face.  It runs only when the caller asks for
// anti_aliasing > 0, or for bounces > 0 on a scene with a reflection output; the reference's
// default engine never takes it.
//
// Recursion.  cast_ray returns a Vec<Color> whose nested bounce lists are flattened into the
// parent's (`lighting.extend(cast_ray(..).map(|c| c * reflection))`, engine.rs:187-190) and
// the pixel value is the left fold of the flattened list (color.rs:82-87).  So the pixel is
// one running sum over a depth-first walk: an element produced at depth k is multiplied by the
// reflection factors of depths k-1, ..., 0, in that order, and added.  Only the closest
// object's elements survive a level (`lighting.clear()` on a closer hit, engine.rs:119-126),
// so each level first finds its closest hit, then emits.  The walk keeps one frame per depth
// (hit point, normal, ray direction, material, next light) — bounces <= kMaxBounces.
//
// Anti-aliasing.  engine.rs:62-69 draws two gen_range(-1.0..1.0) values per extra ray from
// rand::thread_rng (ChaCha12, OS-seeded: not reproducible).  Here the stream is Philox4x32-10
// keyed by the caller's seed with counter (x, y, sample, 0) — words 0 and 1 are the x and y
// draws — mapped to [-1, 1) exactly as rand 0.8's UniformFloat::sample_single does.  The
// oracle uses the same stream (oracle_render_aa), so results are comparable bit for bit.
#include "cull_record.hpp"
#include "device_math.hpp"
#include "glibc_cosf.hpp"
#include "hit.hpp"
#include "internal.hpp"

namespace eray {
namespace gpu {
namespace {

using namespace eray::dev;

// Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11; Random123's philox4x32 with 10 rounds).
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int round = 0; round < 10; ++round) {
        if (round) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
        const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
        c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
    }
    return c;
}

// rand 0.8 UniformFloat::<f32>::sample_single(-1.0, 1.0) from one 32-bit word: 23 bits as a
// float in [1, 2), minus 1, times the range (2), plus low (-1); never reaches high, so one draw.
__device__ __forceinline__ float jitter(uint32_t word) {
    const float value0_1 = __uint_as_float((word >> 9) | 0x3F800000u) - 1.0f;
    return value0_1 * 2.0f + -1.0f;
}

// Camera::pixel_to_ray(x', y').dir (camera.rs:57-76, Ray::new normalises)
__device__ __forceinline__ f3 camera_ray_dir(const FrameParams& p, float xf, float yf) {
    const f3 C = mk3(p.cx, p.cy, p.cz);
    const float vw = p.ratio * 2.0f;
    const f3 horizontal = mk3(vw, 0.0f, 0.0f), vertical = mk3(0.0f, 2.0f, 0.0f);
    const f3 botleft = sub(sub(sub(C, divs(horizontal, 2.0f)), divs(vertical, 2.0f)), mk3(0.0f, 0.0f, p.z_dist));
    return normalize(sub(add(add(botleft, mul(horizontal, xf)), mul(vertical, yf)), C));
}

// Object<Built>::intersects up to the face (object.rs:58-78): bbox, then the first face in
// index order; u, v, t of that face.
// `live` (camera rays of a scene of at most kSkipTris faces, else null): bit f of the
// wave-uniform mask is clear when face f's culling record rejects every camera ray of the wave —
// its exact test cannot pass, so skipping it leaves the first passing face unchanged.
__device__ __forceinline__ int first_face(const TriHot* tris, const ObjGeom& ob, f3 o, f3 d, float& u, float& v,
                                          float& t, const uint64_t* live) {
    if (!bbox_hit(ob, o, d)) return -1;
    const TriHot* r = tris + ob.tri_begin;
    if (live) {
        if (!ob.tri_count) return -1;
        const uint32_t b = ob.tri_begin, e = ob.tri_begin + ob.tri_count;
        for (uint32_t w = b >> 6; w <= (e - 1) >> 6; ++w) {
            uint64_t m = live[w];
            if (w == (b >> 6)) m &= ~0ull << (b & 63);
            if (w == ((e - 1) >> 6) && (e & 63)) m &= ~(~0ull << (e & 63));
            while (m) {
                const uint32_t f = w * 64 + (uint32_t)__builtin_ctzll(m) - b;
                m &= m - 1;
                if (exact_test(r[f], o, d, u, v, t)) return (int)f;
            }
        }
        return -1;
    }
    for (uint32_t f = 0; f < ob.tri_count; ++f)
        if (exact_test(r[f], o, d, u, v, t)) return (int)f;
    return -1;
}

// One level of cast_ray: the closest object's hit and the Material::get values at it.
struct Level {
    f3 P, N, d;  // hit point, interpolated normal, the (normalised) ray direction
    rgb color;
    float kd, ks, sp, refl;
    uint32_t li;  // next light of the per-light loop (engine.rs:130-192)
};

// A ray's closest object so far (engine.rs:116-126): the first object whose hit point is strictly
// closer to the camera (|P - C|²) than every earlier object's replaces it.
struct Hit {
    float dsq, u, v, t;
    int32_t f;    // face relative to the object's first, -1: no hit yet
    uint32_t o;
};
__device__ __forceinline__ void closer(Hit& h, uint32_t oi, int f, float u, float v, float t, f3 o, f3 d, f3 C) {
    if (f < 0) return;
    const float dsq = len_sq(sub(add(o, mul(d, t)), C));
    if (h.f < 0 || dsq < h.dsq) h = Hit{dsq, u, v, t, f, oi};
}

// The hit's Level: Triangle::intersects' P and N (primitives.rs:60-69), RaycastHit's UV and
// Material::get (object.rs:70-74, material.rs:56-94).
__device__ void fill_level(const FrameParams& p, f3 o, f3 d, const Hit& h, Level& L) {
    const float bu = h.u, bv = h.v, bt = h.t;
    const ObjectDesc& od = p.objects[h.o];
    const TriShade sh = p.shade[od.g.tri_begin + (uint32_t)h.f];
    L.P = add(o, mul(d, bt));
    const f3 na = mk3(sh.s0.x, sh.s0.y, sh.s0.z), nb = mk3(sh.s0.w, sh.s1.x, sh.s1.y);
    const f3 nc = mk3(sh.s1.z, sh.s1.w, sh.s2.x);
    L.N = normalize(add(add(mul(na, bu), mul(nb, bv)), mul(nc, bt)));  // (t, not w: primitives.rs:63)
    L.d = d;
    const float w = 1.0f - bu - bv;
    const float uv0 = ((sh.s2.y * w) + (sh.s2.w * bu)) + (sh.s3.y * bv);
    const float uv1 = ((sh.s2.z * w) + (sh.s3.x * bu)) + (sh.s3.z * bv);
    const MaterialDesc& mat = od.mat;
    // defaults at use (engine.rs:128,155,160,164,181)
    L.color = rgb{0.0f, 0.0f, 0.0f};
    L.kd = 0.5f;
    L.ks = 0.5f;
    L.sp = 1.0f;
    L.refl = 0.0f;
    if (mat.example) {  // main.rs's graph at the texel Material::get reads
        const uint32_t ix = mod_size(sat_u32(uv0 * (float)mat.ex_w), mat.ex_w);
        const uint32_t iy = mod_size(sat_u32(uv1 * (float)mat.ex_h), mat.ex_h);
        const float wv = __builtin_fabsf(libm::cosf_glibc(libm::div10_f32((float)ix * mat.ex_xf + (float)iy * mat.ex_yf)));
        const float omf = 1.0f - mat.ex_factor;
        L.color = rgb{wv * omf + mat.ex_r * mat.ex_factor, wv * omf + mat.ex_g * mat.ex_factor,
                      wv * omf + mat.ex_b * mat.ex_factor};
        L.kd = wv;
    }
    if (mat.prog) {  // a shader graph at the texel (its outputs have no texture)
        float t3[3];
        if (texel_program(mat.prog, 0, uv0, uv1, t3)) L.color = rgb{t3[0], t3[1], t3[2]};
        if (texel_program(mat.prog, 1, uv0, uv1, t3)) L.kd = t3[0];
        if (texel_program(mat.prog, 2, uv0, uv1, t3)) L.ks = t3[0];
        if (texel_program(mat.prog, 3, uv0, uv1, t3)) L.sp = t3[0];
        if (texel_program(mat.prog, 4, uv0, uv1, t3)) L.refl = t3[0];
    }
    if (const float* c = texel(mat.color, uv0, uv1, 3)) L.color = rgb{c[0], c[1], c[2]};
    if (const float* c = texel(mat.diffuse, uv0, uv1, 1)) L.kd = *c;
    if (const float* c = texel(mat.specular, uv0, uv1, 1)) L.ks = *c;
    if (const float* c = texel(mat.specular_power, uv0, uv1, 1)) L.sp = *c;
    if (const float* c = texel(mat.reflection, uv0, uv1, 1)) L.refl = *c;
    L.li = 0;
}

// The closest object's first hit along Ray(o, d) (engine.rs:116-126) and its Level; false on a
// miss.  Every face of every object (reflected rays; camera rays of small scenes via `live`).
__device__ bool surface(const FrameParams& p, f3 o, f3 d, Level& L, int32_t* face_out, const uint64_t* live) {
    const f3 C = mk3(p.cx, p.cy, p.cz);
    Hit h;
    h.f = -1;
    for (uint32_t oi = 0; oi < p.nobj; ++oi) {
        const ObjGeom ob = p.objects[oi].g;
        float u, v, t;
        const int f = first_face(p.tris, ob, o, d, u, v, t, live);
        closer(h, oi, f, u, v, t, o, d, C);
    }
    if (h.f < 0) return false;
    if (face_out) *face_out = h.f;
    fill_level(p, o, d, h, L);
    return true;
}

// Camera rays of one pixel, up to kRays at once (the corner ray and anti-aliasing rays), against
// every object: the closest hit of each (engine.rs:116-126).  Binned objects (p.trace_bins) are
// searched in one pass over the sub-block's screen bin `bin` (bins.hip, the tracer's setup) for all
// its rays together: a camera ray of the bin's pixels — the corner ray or a jittered one, whose
// viewport point stays inside [-1/W, 1] x [-1/H, 1] — can only hit faces whose entry marks its
// pixel (face_rect.hpp bin_pixels_jittered), and Object::intersects' first face (object.rs:63-78)
// is the smallest index that passes, whatever order the entries come in.
// A group of kW waves searches one sub-block (lane = pixel: bit row * 16 + column of a bin mask):
// each wave loads 64 entries at a time into its LDS chunk (one round trip), an entry marking at
// most kWide of the searching pixels is tested as (entry, pixel) pairs, compacted in LDS and dealt
// one per lane — a pole of the mesh, where hundreds of thin faces meet, puts a thousand entries
// into one bin, each covering a few pixels — and a wider one by the whole wave (lane = pixel).
// Each (ray, pixel) keeps its smallest passing face in LDS (atomicMin); wave 0 then re-tests its
// pixels' winners for u, v, t (the same f32 operations: the same values).  kW = 1: every wave its
// own sub-block; kW = 4: the workgroup on one heavy sub-block (trace_kernel).  Wave 0's lanes
// hold the pixels' rays `d` and receive the hits; every lane of the group must call (`valid`
// false: a lane off the frame, no rays).  Objects without bins: first_face per ray.
constexpr int kRays = 5;    // anti_aliasing = 4 in one pass
constexpr uint32_t kWide = 16;
struct BinRays {              // the sub-block's rays and results, shared by the group
    float dir[kRays][3][64];  // lane = pixel
    uint32_t best[kRays][64];  // smallest passing face per (ray, pixel), ~0u: none
    uint32_t in[64];           // bit r: ray r of the pixel passes the object's bounding box
    unsigned long long act;    // pixels with some ray in the box
    unsigned long long pad;
};
struct BinChunk {             // one wave's chunk of the bin's entries
    TriHot hot[64];
    unsigned long long mask[64];
    uint32_t tri[64];
    uint16_t pairs[64 * kWide];  // (entry << 6) | pixel
};
template <int kW>
struct BinGroup {
    BinRays R;
    BinChunk E[kW];
};

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
template <int kW>
__device__ __forceinline__ void group_sync() {
    if (kW == 1) wave_sync();
    else __syncthreads();
}
template <int kW>
__device__ void camera_hits(const FrameParams& p, f3 C, const f3 (&d)[kRays], uint32_t nr, bool valid, uint32_t bin,
                            BinGroup<kW>& G, Hit (&h)[kRays]) {
    const uint32_t lane = threadIdx.x & 63, wg = kW == 1 ? 0u : (threadIdx.x >> 6);
    BinRays& R = G.R;
    BinChunk& E = G.E[wg];
#pragma unroll
    for (int r = 0; r < kRays; ++r) {
        h[r].f = -1;
        if (wg == 0) {
            R.dir[r][0][lane] = d[r].x;
            R.dir[r][1][lane] = d[r].y;
            R.dir[r][2][lane] = d[r].z;
        }
    }
    for (uint32_t oi = 0; oi < p.nobj; ++oi) {
        const ObjGeom ob = load_const(&p.objects[oi].g, 0);
        if (!ob.bin_start) {
            if (wg == 0) {
#pragma unroll
                for (uint32_t r = 0; r < (uint32_t)kRays; ++r)
                    if (valid && r < nr) {
                        float u, v, t;
                        const int f = first_face(p.tris, ob, C, d[r], u, v, t, nullptr);
                        closer(h[r], oi, f, u, v, t, C, d[r], C);
                    }
            }
            continue;
        }
        if (wg == 0) {
            uint32_t inb = 0;
#pragma unroll
            for (int r = 0; r < kRays; ++r) {
                if (valid && (uint32_t)r < nr && bbox_hit(ob, C, d[r])) inb |= 1u << r;
                R.best[r][lane] = ~0u;
            }
            R.in[lane] = inb;
            const unsigned long long a = __ballot(inb != 0);
            if (lane == 0) R.act = a;
        }
        group_sync<kW>();
        const unsigned long long act = R.act;
        const uint32_t lo = act ? load_const(ob.bin_start, bin) : 0u, hi = act ? load_const(ob.bin_start, bin + 1) : 0u;
        for (uint32_t rb = lo; rb < hi; rb += 64 * kW) {
            const uint32_t j = rb + 64 * wg + lane;
            unsigned long long m = 0;
            if (j < hi) {
                const BinEntry x = ob.bin_ent[j];  // (one 64-B line per entry)
                m = x.mask & act;
                E.tri[lane] = x.tri;
                E.hot[lane] = x.hot;
            }
            const uint32_t pop = (uint32_t)__popcll(m);
            const bool narrow = pop && pop <= kWide;
            // the narrow entries' pairs: exclusive scan of their counts over the lanes
            uint32_t incl = narrow ? pop : 0u;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)incl, off);
                if ((int)lane >= off) incl += y;
            }
            const uint32_t npairs = (uint32_t)__shfl((int)incl, 63);
            if (narrow) {
                uint32_t at = incl - pop;
                unsigned long long mm = m;
                while (mm) {
                    E.pairs[at++] = (uint16_t)((lane << 6) | (uint32_t)__builtin_ctzll(mm));
                    mm &= mm - 1;
                }
            }
            unsigned long long wide = __ballot(pop > kWide);
            E.mask[lane] = m;
            wave_sync();
            for (uint32_t i = lane; i < npairs; i += 64) {  // one (entry, pixel) pair per lane
                const uint32_t pr = E.pairs[i], k = pr >> 6, q = pr & 63u;
                const uint32_t f = E.tri[k], bits = R.in[q];
                const TriHot hh = E.hot[k];
#pragma unroll
                for (uint32_t r = 0; r < (uint32_t)kRays; ++r) {
                    if (r >= nr) break;
                    if (!((bits >> r) & 1u) || f >= R.best[r][q]) continue;
                    float u, v, t;
                    const f3 dq = mk3(R.dir[r][0][q], R.dir[r][1][q], R.dir[r][2][q]);
                    if (exact_test_flat(hh, C, dq, u, v, t)) atomicMin(&R.best[r][q], f);
                }
            }
            const uint32_t bits = R.in[lane];
            while (wide) {  // a wide entry: every lane tests its own pixel's rays
                const uint32_t k = (uint32_t)__builtin_ctzll(wide);
                wide &= wide - 1;
                const uint32_t f = E.tri[k];
                if (!((E.mask[k] >> lane) & 1ull)) continue;
                const TriHot hh = E.hot[k];
#pragma unroll
                for (uint32_t r = 0; r < (uint32_t)kRays; ++r) {
                    if (r >= nr) break;
                    float u, v, t;
                    const f3 dq = mk3(R.dir[r][0][lane], R.dir[r][1][lane], R.dir[r][2][lane]);
                    if (((bits >> r) & 1u) && f < R.best[r][lane] && exact_test_flat(hh, C, dq, u, v, t))
                        atomicMin(&R.best[r][lane], f);
                }
            }
            wave_sync();  // (the next chunk rewrites the wave's slot)
        }
        group_sync<kW>();  // every wave's results are in
        if (wg == 0) {  // the winners' u, v, t: the exact test again on the winning face's record
#pragma unroll
            for (uint32_t r = 0; r < (uint32_t)kRays; ++r) {
                const uint32_t f = R.best[r][lane];
                if (r < nr && f != ~0u) {
                    float u, v, t;
                    exact_test_flat(p.tris[ob.tri_begin + f], C, d[r], u, v, t);
                    closer(h[r], oi, (int)f, u, v, t, C, d[r], C);
                }
            }
        }
        group_sync<kW>();  // (R is rewritten for the next object)
    }
}

// Engine::reaches_light (engine.rs:218-228): the FIRST object with any hit decides.
__device__ bool reaches_light(const FrameParams& p, f3 S, f3 sd, f3 Lp) {
    const float dist = len(sub(Lp, S));
    for (uint32_t oi = 0; oi < p.nobj; ++oi) {
        const ObjGeom ob = p.objects[oi].g;
        float u, v, t;
        if (first_face(p.tris, ob, S, sd, u, v, t, nullptr) >= 0) return len(sub(add(S, mul(sd, t)), S)) > dist;
    }
    return true;
}

// diffuse + specular of one point light that reaches the hit (engine.rs:143-176)
__device__ __forceinline__ rgb shade(const Level& L, const LightDesc& Ld) {
    const f3 Lp = mk3(Ld.pos[0], Ld.pos[1], Ld.pos[2]);
    const f3 LmP = sub(Lp, L.P);
    float prod = rust_clamp(dot0(L.N, LmP), 0.0f, 1.0f);
    if (prod != prod) prod = 0.0f;
    const float falloff = 1.0f / len(LmP);
    const rgb lc{Ld.color[0], Ld.color[1], Ld.color[2]};
    const rgb diffusion = cmul(cmul(cmul(cmul(cmulc(L.color, lc), L.kd), prod), Ld.brightness), falloff);
    const f3 reflected = sub(L.d, mul(mul(L.N, 2.0f), dot0(L.d, L.N)));
    const float res =
        rust_clamp(L.ks * Ld.brightness * powf_ref(dot0(normalize(reflected), normalize(LmP)), L.sp), 0.0f, 1.0f);
    const float sf = rust_clamp(powf_ref(falloff, L.sp), 0.0f, 1.0f);
    return cadd(diffusion, rgb{res * sf, res * sf, res * sf});
}

// Engine::cast_ray(ray, 0).sum() (engine.rs:112-216, color.rs:82-87) as a depth-first walk from
// the first level's hit `first`.  kBounce false: no reflection levels (bounces == 0), so the walk
// needs no per-depth frames.
template <bool kBounce>
__device__ rgb walk(const FrameParams& p, const Level& first) {
    Level st[kBounce ? kMaxBounces + 1 : 1];
    st[0] = first;
    bool any = false;
    rgb acc{0.0f, 0.0f, 0.0f};
    auto emit = [&](rgb c, int depth) {  // c * refl[depth-1] * ... * refl[0], then the fold
        if (kBounce)
            for (int j = depth - 1; j >= 0; --j) c = cmul(c, st[j].refl);
        acc = any ? cadd(acc, c) : c;
        any = true;
    };
    const rgb miss{0.1f, 0.1f, 0.2f};  // engine.rs:211-213
    int depth = 0;
    while (depth >= 0) {
        Level& L = st[kBounce ? depth : 0];
        if (L.li < p.nlights) {
            const LightDesc Ld = p.lights[L.li++];
            if (Ld.variant == 1) continue;  // ambient lights come after the loop
            const f3 Lp = mk3(Ld.pos[0], Ld.pos[1], Ld.pos[2]);
            const f3 S = add(L.P, mul(L.N, 0.1f));
            if (reaches_light(p, S, normalize(sub(Lp, L.P)), Lp)) emit(shade(L, Ld), depth);
            if (kBounce && (uint32_t)depth < p.bounces && L.refl != 0.0f) {  // engine.rs:181-191
                const f3 rd = normalize(sub(L.d, mul(mul(L.N, 2.0f), dot0(L.d, L.N))));
                if (surface(p, S, rd, st[depth + 1], nullptr, nullptr))
                    ++depth;
                else
                    emit(miss, depth + 1);
            }
        } else {
            for (uint32_t li = 0; li < p.nlights; ++li) {  // ambient lights (engine.rs:197-208)
                const LightDesc A = p.lights[li];
                if (A.variant != 1) continue;
                const rgb m{rust_min(A.color[0], L.color.r), rust_min(A.color[1], L.color.g),
                            rust_min(A.color[2], L.color.b)};
                emit(cmul(cmul(m, L.kd), A.brightness), depth);
            }
            --depth;
        }
    }
    return acc;
}

// The miss colour (engine.rs:211-213): a ray that hits nothing returns vec![it].
__device__ __forceinline__ rgb miss_color() { return rgb{0.1f, 0.1f, 0.2f}; }

// Engine::cast_ray(ray, 0).sum() of one ray.  `miss_known`: the caller knows the ray hits
// nothing (trace_kernel's background skip); `live`: the faces a camera ray of the wave can hit
// (first_face), for the first level only.
template <bool kBounce>
__device__ rgb cast_ray(const FrameParams& p, f3 o, f3 d, int32_t* face_out, bool miss_known, const uint64_t* live) {
    Level L;
    if (miss_known || !surface(p, o, d, L, face_out, live)) return miss_color();
    return walk<kBounce>(p, L);
}

// Element r of a per-ray array (r < kRays, run time) without a dynamically indexed private array
// (which would live in scratch memory).
template <typename T>
__device__ __forceinline__ T pick(const T (&a)[kRays], uint32_t r) {
    T out = a[0];
#pragma unroll
    for (uint32_t k = 1; k < (uint32_t)kRays; ++k)
        if (r == k) out = a[k];
    return out;
}

// Waves.  A 256-thread workgroup owns a 64 x 4 pixel block and each wave a 16 x 4 sub-block of
// it, lane = row * 16 + column: one screen bin (bins.hip), so a binned object's camera rays read
// the same entries in every lane.  (Interleaved bands are multiples of 4 rows: a sub-block's rows
// are consecutive camera rows.)
//
// Background skip.  Every ray a wave casts from the camera — its 64 primary rays and their
// jittered anti-aliasing rays — goes through the viewport rectangle [x0 - 1, x0 + 16] x [y0 - 1,
// y0 + 4] / (W, H) (jitter in [-1, 1), engine.rs:62-69).  A wave that can show that none of those
// rays reaches any face casts none: every one of its rays is the reference's miss
// (engine.rs:211-213) — cast_ray's own miss path, the same float sums — and the shadow and
// reflected rays, which start only at a hit, never exist.
//  * Scenes of at most kSkipTris triangles: trace_cull_kernel computes every triangle's culling
//    record for this camera (cull_record.hpp, the frame kernel's conservative bounds, with the
//    viewport range widened to the jittered rays') and each workgroup copies them into LDS; a wave
//    none of whose records survives its rectangle skips, the other waves keep the survivors' bits
//    (live_mask): their camera rays test only those faces, in index order.
//  * Scenes with binned objects (p.trace_bins): the tracer's per-camera setup works over the
//    viewport the jittered rays reach, [-1/W, 1] x [-1/H, 1]: a binned object's bin lists every
//    face any ray of the bin's pixels may hit (camera_hits), a small object's rectangle (the
//    union of face_rect.hpp's) holds every pixel one of whose rays may hit it.  A wave whose bin
//    is empty for every binned object and whose sub-block meets no small object's rectangle
//    skips; the others search their bin (camera_hits).
// Bit-identical to the brute-force scan (ERAY_RENDER_BRUTE_FORCE turns both off;
// tests/test_gpu_trace.py compares them).
constexpr uint32_t kSkipTris = kTraceSkipTris;

// The records, once per camera and scene (one workgroup; the host passes trace_cull only for
// scenes of at most kSkipTris faces, and launches it when the camera or the scene changed:
// capi.cpp prepare_render — not in every frame's graph, C2 with AA = 4: 56 -> 47 us per frame).
__global__ void __launch_bounds__(256) trace_cull_kernel(FrameParams p) {
    const uint32_t i = threadIdx.x;
    if (i >= p.total_tris) return;
    const CamDev cam{p.cx, p.cy, p.cz, p.ratio, p.z_dist, {0u, 0u, 0u}};
    const double xa = -2.0 / (double)p.cam_w, ya = -2.0 / (double)p.cam_h;  // (rays reach -1/W, -1/H)
    p.trace_cull[i] = cull_record(p.tris[i], cam, xa, 1.0, ya, 1.0);
}

__device__ __forceinline__ float widen_down(float v) { return v >= 0.0f ? v * (1.0f - 0x1p-20f) : v * (1.0f + 0x1p-20f); }
__device__ __forceinline__ float widen_up(float v) { return v >= 0.0f ? v * (1.0f + 0x1p-20f) : v * (1.0f - 0x1p-20f); }

// ray i of pixel (px, camera row y): 0 is cast_ray_from_camera(x as f32, y as f32) (engine.rs:60,
// 100-109), 1 + s the s-th anti-aliasing ray (engine.rs:62-69); the pixel sums them in that order
__device__ __forceinline__ f3 pixel_ray(const FrameParams& p, uint32_t px, uint32_t y, uint32_t i) {
    if (i == 0) return camera_ray_dir(p, (float)px / (float)p.cam_w, (float)y / (float)p.cam_h);
    const uint4 r = philox4x32_10(make_uint4(px, y, i - 1, 0u), p.seed_lo, p.seed_hi);
    const float xf = ((float)px + jitter(r.x)) / (float)p.cam_w;
    const float yf = ((float)y + jitter(r.y)) / (float)p.cam_h;
    return camera_ray_dir(p, xf, yf);
}

// (average / aa as f32).clamp() (engine.rs:71-73), then Image::set and the PPM bytes
// (Color::as_bytes, rows bottom-up: image.rs:48-74, color.rs:31-37) and the first ray's face
__device__ __forceinline__ void store_pixel(const FrameParams& p, uint32_t px, uint32_t py, rgb avg, int32_t face) {
    if (p.aa) {
        const float n = (float)p.aa;
        avg = rgb{rust_clamp(avg.r / n, 0.0f, 1.0f), rust_clamp(avg.g / n, 0.0f, 1.0f),
                  rust_clamp(avg.b / n, 0.0f, 1.0f)};
    }
    const size_t idx = (size_t)py * p.img_w + px;
    if (p.out_rgb) {
        float* o = p.out_rgb + 3 * idx;
        o[0] = avg.r;
        o[1] = avg.g;
        o[2] = avg.b;
    }
    if (p.out_ppm) {
        uint8_t* o = p.out_ppm + 3 * ((size_t)(p.rows - 1 - py) * p.img_w + px);
        o[0] = (uint8_t)sat_u8(avg.r * 255.0f);
        o[1] = (uint8_t)sat_u8(avg.g * 255.0f);
        o[2] = (uint8_t)sat_u8(avg.b * 255.0f);
    }
    if (p.out_face) p.out_face[idx] = face;
}

// The binned search of a sub-block's rays (camera_hits: the wave alone, or with `heavy` the
// workgroup's four waves together) and, in the pixel's lane of wave 0, the walks of their hits:
// the pixel's sum and first face.
template <bool kBounce, bool heavy>
__device__ void binned_pixel(const FrameParams& p, uint32_t px, uint32_t y, bool valid, uint32_t bin,
                             unsigned char* lds, rgb& avg, int32_t& face) {
    const bool lead = !heavy || (threadIdx.x >> 6) == 0;
    const f3 C = mk3(p.cx, p.cy, p.cz);
    const uint32_t n = 1 + p.aa;
    for (uint32_t i0 = 0; i0 < n; i0 += kRays) {  // (wave- / workgroup-uniform)
        const uint32_t nr = min((uint32_t)kRays, n - i0);
        f3 d[kRays];
#pragma unroll
        for (uint32_t r = 0; r < (uint32_t)kRays; ++r)
            d[r] = (lead && r < nr) ? pixel_ray(p, px, y, i0 + r) : mk3(0.0f, 0.0f, -1.0f);
        Hit h[kRays];
        if constexpr (heavy) camera_hits<4>(p, C, d, nr, valid && lead, bin, *reinterpret_cast<BinGroup<4>*>(lds), h);
        else camera_hits<1>(p, C, d, nr, valid, bin, *reinterpret_cast<BinGroup<1>*>(lds), h);
        if (!valid || !lead) continue;
        for (uint32_t r = 0; r < nr; ++r) {
            const Hit hr = pick(h, r);
            rgb c = miss_color();
            if (hr.f >= 0) {
                Level L;
                fill_level(p, C, pick(d, r), hr, L);
                c = walk<kBounce>(p, L);
            }
            if (i0 + r == 0) {
                avg = c;
                face = hr.f;
            } else {
                avg = cadd(avg, c);
            }
        }
    }
}


// Heavy sub-blocks (scenes with binned objects).  A bin of more than kTraceHeavyMin entries (the
// tracer setup's detail list puts those first, bins.hip) would keep its wave long after the
// others; trace_binned_kernel's first workgroups take them instead, the whole workgroup on one
// sub-block (camera_hits<4>).
template <bool kBounce>
__device__ void heavy_role(const FrameParams& p, unsigned char* s_raw, uint32_t first, uint32_t stride) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t nheavy = *p.detail_heavy;
    for (uint32_t hv = first; hv < nheavy; hv += stride) {
        const uint32_t sub = p.detail_list[hv], sx = sub & 0xffffu, sy = sub >> 16;
        const uint32_t px = sx * kBinW + (lane & 15), py = sy * kBinH + (lane >> 4);
        const uint32_t y0 = band_camera_row(p.row0, p.band_shift, p.band_mask, p.band_stride, sy * kBinH);
        const uint32_t y = y0 + (lane >> 4);
        const uint32_t bin = ((y0 + kBinH - p.bin_phase) / kBinH) * p.bins_x + sx;
        const bool valid = px < p.cam_w && py < p.rows;
        rgb avg{0.0f, 0.0f, 0.0f};
        int32_t face = -1;
        binned_pixel<kBounce, true>(p, px, y, valid, bin, s_raw, avg, face);
        if (wave == 0 && valid) store_pixel(p, px, py, avg, face);
        __syncthreads();  // (the next sub-block rewrites the group's LDS)
    }
}

template <bool kBounce>
__global__ void __launch_bounds__(256) trace_kernel(FrameParams p) {
    __shared__ TriCull s_cull[kSkipTris];  // the culling records (scenes of at most kSkipTris faces)
    __shared__ uint64_t s_live[4][kSkipTris / 64];  // each wave's live_mask (LDS: run-time indexed)
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t bx = blockIdx.x % p.tiles_x, by = blockIdx.x / p.tiles_x;
    const uint32_t x0 = bx * 64 + wave * 16;  // the wave's sub-block: columns x0 .. x0 + 15
    const uint32_t px = x0 + (lane & 15);
    const uint32_t py0 = by * 4, py = py0 + (lane >> 4);  // rank-local rows
    const uint32_t y0 = band_camera_row(p.row0, p.band_shift, p.band_mask, p.band_stride, py0);
    const uint32_t y = y0 + (lane >> 4);
    bool skip = false;
    uint64_t* live_mask = s_live[wave];
    const uint64_t* live = nullptr;
    if (p.trace_cull) {  // workgroup-uniform
        if (threadIdx.x < p.total_tris) s_cull[threadIdx.x] = p.trace_cull[threadIdx.x];
        __syncthreads();
        const float rw = 1.0f / (float)p.cam_w, rh = 1.0f / (float)p.cam_h;
        // (x' <= 1, y' <= 1: the rays reach at most x = W, y = H; the bounds assume |x'|, |y'| <= 1)
        const float xe = __builtin_fminf((float)x0 + 16.0f, (float)p.cam_w);
        const float ye = __builtin_fminf((float)y0 + 4.0f, (float)p.cam_h);
        const float xlo = widen_down(((float)x0 - 1.0f) * rw), xhi = widen_up(xe * rw);
        const float ylo = widen_down(((float)y0 - 1.0f) * rh), yhi = widen_up(ye * rh);
        uint64_t any = 0;
#pragma unroll
        for (uint32_t w = 0; w < kSkipTris / 64; ++w) {
            const uint64_t m = __ballot(w * 64 + lane < p.total_tris && !cull_rejects(s_cull[w * 64 + lane], xlo, xhi, ylo, yhi));
            if (lane == 0) live_mask[w] = m;
            any |= m;
        }
        skip = any == 0;
        live = live_mask;
    }
    const bool valid = px < p.cam_w && py < p.rows;
    const f3 C = mk3(p.cx, p.cy, p.cz);
    int32_t face = -1;
    rgb avg{0.0f, 0.0f, 0.0f};
    if (!valid) return;
    if (skip) {  // every camera ray misses (the jitter only moves a ray that misses anyway)
        avg = miss_color();
        for (uint32_t s = 0; s < p.aa; ++s) avg = cadd(avg, miss_color());
    } else {
        avg = cast_ray<kBounce>(p, C, pixel_ray(p, px, y, 0), &face, false, live);
        for (uint32_t s = 0; s < p.aa; ++s)
            avg = cadd(avg, cast_ray<kBounce>(p, C, pixel_ray(p, px, y, 1 + s), nullptr, false, live));
    }
    store_pixel(p, px, py, avg, face);
}


// The background colour of a pixel none of whose rays hits: (1 + aa) miss colours summed, then
// (average / aa).clamp() (engine.rs:59-77, 211-213).
__device__ __forceinline__ rgb background_color(const FrameParams& p) {
    rgb avg = miss_color();
    for (uint32_t s = 0; s < p.aa; ++s) avg = cadd(avg, miss_color());
    if (p.aa) {
        const float n = (float)p.aa;
        avg = rgb{rust_clamp(avg.r / n, 0.0f, 1.0f), rust_clamp(avg.g / n, 0.0f, 1.0f), rust_clamp(avg.b / n, 0.0f, 1.0f)};
    }
    return avg;
}

// Background of the pixels [x0, x0 + kW) x rows [py0, py0 + 4) (kW = 64 or 16), wave-wide: the
// colour `c` (bytes `b`) as 16-byte write-through row stores, the face -1 (engine.rs:211-213).
template <uint32_t kW>
__device__ void fill_color(const FrameParams& p, uint32_t x0, uint32_t py0, uint32_t lane, const float (&c)[3],
                           const uint8_t (&b)[3]) {
    if (p.aligned && x0 + kW <= p.cam_w && py0 + kBinH <= p.rows) {
        constexpr uint32_t kRow4 = kW * 3 / 4, kRow16 = kW * 3 / 16, kFace4 = kW / 4;
        if (p.out_rgb) {
#pragma unroll
            for (uint32_t i = lane; i < kBinH * kRow4; i += 64) {
                const uint32_t r = i / kRow4, q = i % kRow4, ph = q % 3;  // float offset 4q: component (4q) % 3
                const float4 w = make_float4(c[ph], c[(ph + 1) % 3], c[(ph + 2) % 3], c[ph]);
                stream16(p.out_rgb, reinterpret_cast<float4*>(p.out_rgb + 3 * ((size_t)(py0 + r) * p.img_w + x0)) + q, w);
            }
        }
        if (p.out_ppm && lane < kBinH * kRow16) {
            const uint32_t r = lane / kRow16, q = lane % kRow16;
            uint32_t w[4];
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) {  // byte 16q + 4k + j: component (q + 4k + j) % 3
                w[k] = 0;
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) w[k] |= (uint32_t)b[(q + 4 * k + j) % 3] << (8 * j);
            }
            const size_t row = (size_t)(p.rows - py0 - kBinH + r);  // file rows, bottom-up
            stream16(p.out_ppm, reinterpret_cast<uint4*>(p.out_ppm + 3 * (row * p.img_w + x0)) + q,
                     make_uint4(w[0], w[1], w[2], w[3]));
        }
        if (p.out_face && lane < kBinH * kFace4) {
            const uint32_t r = lane / kFace4, q = lane % kFace4;
            stream16(p.out_face, reinterpret_cast<int4*>(p.out_face + (size_t)(py0 + r) * p.img_w + x0) + q,
                     make_uint4(~0u, ~0u, ~0u, ~0u));
        }
        return;
    }
    for (uint32_t k = lane; k < kW * kBinH; k += 64) {  // image edge or unaligned output: per pixel
        const uint32_t px = x0 + k % kW, py = py0 + k / kW;
        if (px >= p.cam_w || py >= p.rows) continue;
        const size_t idx = (size_t)py * p.img_w + px;
        if (p.out_rgb) {
            float* o = p.out_rgb + 3 * idx;
            o[0] = c[0];
            o[1] = c[1];
            o[2] = c[2];
        }
        if (p.out_ppm) {
            uint8_t* o = p.out_ppm + 3 * ((size_t)(p.rows - 1 - py) * p.img_w + px);
            o[0] = b[0];
            o[1] = b[1];
            o[2] = b[2];
        }
        if (p.out_face) p.out_face[idx] = -1;
    }
}

// Scenes with binned objects (p.trace_bins): the tracer's setup lists the sub-blocks some ray of
// which may hit a face (bins.hip: non-empty bins, small objects' rectangles — the same
// conditions as trace_kernel's background skip), the heavy ones first, with an occupancy byte per
// 64 x 4 block.  The grid's first trace_heavy_wgs workgroups take the heavy sub-blocks
// (heavy_role), the next trace_fill_wgs write the background of the unlisted sub-blocks, the
// others take the light listed sub-blocks, one per wave (camera_hits<1>).
// Three workgroups per CU (168 VGPRs, a few spilled; LDS 45 KB each): 3840x2160 / 70k with
// AA = 4 178 -> 130 us per frame against two per CU (178 VGPRs), same-box A/B
// (profiles/r04/ab/ab_r04f.txt).
template <bool kBounce>
__global__ void __launch_bounds__(256, 3) trace_binned_kernel(FrameParams p) {
    constexpr size_t kLds = 4 * sizeof(BinGroup<1>) > sizeof(BinGroup<4>) ? 4 * sizeof(BinGroup<1>) : sizeof(BinGroup<4>);
    __shared__ __attribute__((aligned(16))) unsigned char s_raw[kLds];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t nheavy_wgs = p.trace_heavy_wgs, nfill = p.trace_fill_wgs;
    if (blockIdx.x < nheavy_wgs) {  // workgroup-uniform: the heavy sub-blocks, a workgroup each
        heavy_role<kBounce>(p, s_raw, blockIdx.x, nheavy_wgs);
        return;
    }
    const uint32_t wg = blockIdx.x - nheavy_wgs;
    if (wg < nfill) {  // workgroup-uniform: background
        const rgb bg = background_color(p);
        const float c[3] = {bg.r, bg.g, bg.b};
        const uint8_t b[3] = {(uint8_t)sat_u8(bg.r * 255.0f), (uint8_t)sat_u8(bg.g * 255.0f), (uint8_t)sat_u8(bg.b * 255.0f)};
        const uint32_t nblk = p.tiles_x * ((p.rows + kBinH - 1) / kBinH), stride = nfill * 4;
        uint32_t occ = 0, it = 0;  // lane i: the occupancy of this wave's i-th next block
        for (uint32_t blk = wave * nfill + wg; blk < nblk; blk += stride, ++it) {
            if ((it & 63u) == 0) {  // one load per 64 blocks, not a dependent load per block
                const uint32_t bl = blk + lane * stride;
                occ = bl < nblk ? p.detail_occ[bl] : 0u;
            }
            const uint32_t mask = (uint32_t)__builtin_amdgcn_readlane((int)occ, (int)(it & 63u));  // listed sub-blocks
            const uint32_t bx = blk % p.tiles_x, by = blk / p.tiles_x;
            if (!mask) {
                fill_color<64>(p, bx * 64, by * kBinH, lane, c, b);
            } else if (mask != 0xfu) {
                for (uint32_t i = 0; i < 4; ++i)
                    if (!((mask >> i) & 1u)) fill_color<16>(p, bx * 64 + i * 16, by * kBinH, lane, c, b);
            }
        }
        return;
    }
    const uint32_t heavy = p.detail_heavy[0], nl = p.detail_heavy[1];
    const uint32_t stride = (gridDim.x - nheavy_wgs - nfill) * 4;
    for (uint32_t j = (wg - nfill) * 4 + wave; j < nl; j += stride) {  // (wave-uniform)
        const uint32_t sub = p.detail_list[heavy + j], sx = sub & 0xffffu, sy = sub >> 16;
        const uint32_t px = sx * kBinW + (lane & 15), py = sy * kBinH + (lane >> 4);
        const uint32_t y0 = band_camera_row(p.row0, p.band_shift, p.band_mask, p.band_stride, sy * kBinH);
        const uint32_t y = y0 + (lane >> 4);
        const uint32_t bin = ((y0 + kBinH - p.bin_phase) / kBinH) * p.bins_x + sx;
        const bool valid = px < p.cam_w && py < p.rows;
        rgb avg{0.0f, 0.0f, 0.0f};
        int32_t face = -1;
        binned_pixel<kBounce, false>(p, px, y, valid, bin, s_raw + wave * sizeof(BinGroup<1>), avg, face);
        if (valid) store_pixel(p, px, py, avg, face);
    }
}

}  // namespace

// The culling records of p's camera into p.trace_cull.
hipError_t launch_trace_cull(const FrameParams& p, hipStream_t s) {
    if (!p.trace_cull || p.total_tris > kSkipTris) return hipErrorInvalidValue;
    hipLaunchKernelGGL(trace_cull_kernel, dim3(1), dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_trace(const FrameParams& p0, const LaunchCtx&, hipStream_t s) {
    FrameParams p = p0;
    if (p.trace_bins) {  // listed sub-blocks: heavy, light and background roles
        if (!p.detail_list || !p.detail_heavy || !p.detail_occ) return hipErrorInvalidValue;
        static const uint32_t cus = [] {
            int dev = 0, n = 0;
            return (hipGetDevice(&dev) == hipSuccess &&
                    hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
                       ? (uint32_t)n
                       : 256u;
        }();
        p.trace_heavy_wgs = cus / 4;  // (heavy sub-blocks are few: poles, dense folds; dispatched first)
        p.trace_fill_wgs = cus;       // one per CU: the background is a write stream
        // light sub-blocks: one per wave where the list allows (the workgroups past its end return
        // at once, and the dispatcher hands the freed slots to the next ones: 3840x2160 / 70k with
        // AA = 4 129 -> 111 us against two per CU, profiles/r04/ab/ab_r04k.txt)
        p.trace_light_wgs = 8 * cus;
        const dim3 grid(p.trace_heavy_wgs + p.trace_fill_wgs + p.trace_light_wgs);
        if (p.bounces) hipLaunchKernelGGL(trace_binned_kernel<true>, grid, dim3(256), 0, s, p);
        else hipLaunchKernelGGL(trace_binned_kernel<false>, grid, dim3(256), 0, s, p);
        return hipGetLastError();
    }
    if (p.trace_cull && p.total_tris > kSkipTris) return hipErrorInvalidValue;
    const dim3 grid(((p.cam_w + 63) / 64) * ((p.rows + 3) / 4));
    if (p.bounces) hipLaunchKernelGGL(trace_kernel<true>, grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL(trace_kernel<false>, grid, dim3(256), 0, s, p);
    return hipGetLastError();
}

}  // namespace gpu
}  // namespace eray
