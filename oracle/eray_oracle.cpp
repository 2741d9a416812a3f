// eray_oracle.cpp — CPU ORACLE for the eray per-pixel ray-tracing hot path.
//
// TEST INFRASTRUCTURE ONLY.  A literal, single-threaded restatement of HoloTheDrunk/eray
// (reference @ 2024-11-15, Rust) used as the checker for the MI355X product path.  Only
// tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the product
// (eray_amd/) never links, calls or falls back to it.
//
// Parity status: PARTIALLY PINNED.  The reference is Rust and cannot be compiled here (no
// rustc/cargo, crates not vendored), so there is no oracle/_ref build.
// This restatement is pinned by every known answer the reference's own tests hold
// (vector.rs:253-299 dot/cross/angle, primitives.rs:88-112 projection, image.rs:201-213
// mod_get) plus derived known answers (the centre pixel, texel (0,0)); the triangle, shading,
// shaderlib and PPM arithmetic beyond those is restated from the source, not pinned by a
// reference-produced vector.
//
// Float semantics: Rust on x86-64 evaluates f32 with scalar SSE, no FMA contraction, IEEE
// division and sqrt.  Build with `-O2 -ffp-contract=off` (no -ffast-math, no -march=native)
// to get the same.  Every expression below keeps the reference's operation order; `0.0f + x`
// terms reproduce the fold-from-zero of Vector::dot_product (vector.rs:188-193).
//
// Third-party arithmetic on the path: Rust's f32::cos / f32::powf lower to the platform
// libm (glibc 2.35 here): oracle_cosf / oracle_powf call it directly.

#include "eray_oracle.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

// ---------------------------------------------------------------- vector.rs ---------------
struct V3 {
    float v[3];
};
struct V2 {
    float v[2];
};

inline V3 mk(float x, float y, float z) { return V3{{x, y, z}}; }
// impl_vec_vec_op Add/Sub (vector.rs:73-97): element-wise
inline V3 add(V3 a, V3 b) { return mk(a.v[0] + b.v[0], a.v[1] + b.v[1], a.v[2] + b.v[2]); }
inline V3 sub(V3 a, V3 b) { return mk(a.v[0] - b.v[0], a.v[1] - b.v[1], a.v[2] - b.v[2]); }
// impl_vec_type_op Mul/Div (vector.rs:99-125): element-wise with a scalar
inline V3 mul(V3 a, float s) { return mk(a.v[0] * s, a.v[1] * s, a.v[2] * s); }
inline V3 dvs(V3 a, float s) { return mk(a.v[0] / s, a.v[1] / s, a.v[2] / s); }
inline V2 add2(V2 a, V2 b) { return V2{{a.v[0] + b.v[0], a.v[1] + b.v[1]}}; }
inline V2 mul2(V2 a, float s) { return V2{{a.v[0] * s, a.v[1] * s}}; }
// dot_product: fold starting at TYPE::default() (vector.rs:188-193)
inline float dot(V3 a, V3 b) {
    float acc = 0.0f;
    acc = acc + a.v[0] * b.v[0];
    acc = acc + a.v[1] * b.v[1];
    acc = acc + a.v[2] * b.v[2];
    return acc;
}
inline float len_sq(V3 a) { return dot(a, a); }                // vector.rs:183-185
inline float len(V3 a) { return std::sqrt(len_sq(a)); }         // vector.rs:150-152
inline V3 normalize(V3 a) { return dvs(a, len(a)); }           // vector.rs:156-158
// cross_product(self, other) (vector.rs:198-206)
inline V3 cross(V3 s, V3 o) {
    return mk(o.v[2] * s.v[1] - s.v[2] * o.v[1], o.v[0] * s.v[2] - s.v[0] * o.v[2],
              o.v[1] * s.v[0] - s.v[1] * o.v[0]);
}
// div_under(above): above / v element-wise (vector.rs:169-175)
inline V3 div_under(V3 a, float above) { return mk(above / a.v[0], above / a.v[1], above / a.v[2]); }

// ---------------------------------------------------------------- color.rs ----------------
struct Color {
    float r, g, b;
};
inline Color cadd(Color a, Color b) { return Color{a.r + b.r, a.g + b.g, a.b + b.b}; }  // derive_more Add
inline Color cmul(Color a, float s) { return Color{a.r * s, a.g * s, a.b * s}; }          // color.rs:58-68
inline Color cmulc(Color a, Color b) { return Color{a.r * b.r, a.g * b.g, a.b * b.b}; }   // color.rs:70-80

// Rust f32::min lowers to llvm.minnum; x86-64 codegen: isnan(a) ? b : (b < a ? b : a).
inline float rust_min(float a, float b) {
    if (std::isnan(a)) return b;
    return (b < a) ? b : a;
}
// Rust f32::clamp: NaN propagates (core::f32::clamp).
inline float rust_clamp(float x, float lo, float hi) {
    if (x < lo) x = lo;
    if (x > hi) x = hi;
    return x;
}
inline Color cmin(Color a, Color b) {  // color.rs:49-55
    return Color{rust_min(a.r, b.r), rust_min(a.g, b.g), rust_min(a.b, b.b)};
}
// `f as u32` / `f as u8`: saturating, NaN -> 0, truncation toward zero.
inline uint32_t sat_u32(float f) {
    if (!(f > 0.0f)) return 0u;              // NaN, negatives, zeros
    if (f >= 4294967296.0f) return 0xffffffffu;
    return (uint32_t)f;
}
inline uint8_t sat_u8(float f) {
    if (!(f > 0.0f)) return 0;
    if (f >= 255.0f) return 255;
    return (uint8_t)f;
}

// ---------------------------------------------------------------- raycasting.rs -----------
struct Ray {
    V3 start, dir;
};
inline Ray ray_new(V3 start, V3 dir) { return Ray{start, normalize(dir)}; }  // raycasting.rs:16-21

// ---------------------------------------------------------------- camera.rs ---------------
struct Camera {
    V3 center;
    float fov0, fov1;
    uint32_t width;
    float z_dist;
};
inline float fov_ratio(const Camera& c) { return c.fov0 / c.fov1; }  // camera.rs:10-12
inline void camera_size(const Camera& c, uint32_t* w, uint32_t* h) {  // camera.rs:36-38
    *w = c.width;
    *h = sat_u32((float)c.width / fov_ratio(c));
}
Ray pixel_to_ray(const Camera& c, float x, float y) {  // camera.rs:57-76
    float aspect_ratio = fov_ratio(c);
    float viewport_height = 2.0f;
    float viewport_width = aspect_ratio * viewport_height;
    float focal_length = c.z_dist;
    V3 horizontal = mk(viewport_width, 0.0f, 0.0f);
    V3 vertical = mk(0.0f, viewport_height, 0.0f);
    V3 botleft = sub(sub(sub(c.center, dvs(horizontal, 2.0f)), dvs(vertical, 2.0f)),
                     mk(0.0f, 0.0f, focal_length));
    V3 dir = sub(add(add(botleft, mul(horizontal, x)), mul(vertical, y)), c.center);
    return ray_new(c.center, dir);
}

// ---------------------------------------------------------------- image.rs ----------------
struct ImgRef {
    const float* data;
    uint32_t w, h;
    int channels;
};
// mod_get (image.rs:36-38) with u32 arithmetic
inline size_t mod_index(const ImgRef& im, uint32_t x, uint32_t y) {
    return (size_t)((y % im.h) * im.w + x % im.w);
}

// ---------------------------------------------------------------- material.rs -------------
struct Bundle {  // MaterialOutputBundle (material.rs:120-131)
    bool has_color;
    Color color;
    bool has_diffuse, has_specular, has_sp, has_refl;
    float diffuse, specular, sp, refl;
};
struct Material {
    ImgRef color, diffuse, specular, sp, refl;  // data == nullptr: None
};
inline bool sample_value(const ImgRef& im, float x, float y, float* out) {
    if (!im.data) return false;
    uint32_t ix = sat_u32(x * (float)im.w);
    uint32_t iy = sat_u32(y * (float)im.h);
    *out = im.data[mod_index(im, ix, iy)];
    return true;
}
Bundle material_get(const Material& m, float x, float y) {  // material.rs:56-94
    Bundle b{};
    if (m.color.data) {
        uint32_t ix = sat_u32(x * (float)m.color.w);
        uint32_t iy = sat_u32(y * (float)m.color.h);
        const float* p = m.color.data + 3 * mod_index(m.color, ix, iy);
        b.has_color = true;
        b.color = Color{p[0], p[1], p[2]};
    }
    b.has_diffuse = sample_value(m.diffuse, x, y, &b.diffuse);
    b.has_specular = sample_value(m.specular, x, y, &b.specular);
    b.has_sp = sample_value(m.sp, x, y, &b.sp);
    b.has_refl = sample_value(m.refl, x, y, &b.refl);
    return b;
}

// ---------------------------------------------------------------- primitives.rs -----------
struct Vertex {
    V3 position, normal;
    V2 uv;
};
struct Triangle {
    Vertex a, b, c;
    V3 normal;
};
Triangle triangle_new(Vertex a, Vertex b, Vertex c) {  // primitives.rs:33-36
    Triangle t{a, b, c, cross(sub(b.position, a.position), sub(c.position, a.position))};
    return t;
}
// Triangle::intersects (primitives.rs:41-72)
bool triangle_intersects(const Triangle& tri, const Ray& ray, V3* pos, V3* nrm, V3* bary) {
    V3 a = tri.a.position, b = tri.b.position, c = tri.c.position;
    V3 e1 = sub(b, a);
    V3 e2 = sub(c, a);
    V3 n = cross(e1, e2);
    if (dot(n, ray.dir) > 0.0f) return false;  // backface culling
    float det = -dot(ray.dir, n);
    float invdet = 1.0f / det;
    V3 ao = sub(ray.start, a);
    V3 dao = cross(ao, ray.dir);
    float u = dot(e2, dao) * invdet;
    float v = -dot(e1, dao) * invdet;
    float t = dot(ao, n) * invdet;
    if (det >= 1e-6f && t >= 0.0f && u >= 0.0f && v >= 0.0f && (u + v) <= 1.0f) {
        *pos = add(ray.start, mul(ray.dir, t));
        *nrm = normalize(add(add(mul(tri.a.normal, u), mul(tri.b.normal, v)), mul(tri.c.normal, t)));
        *bary = mk(u, v, 1.0f - u - v);
        return true;
    }
    return false;
}
V3 triangle_project(const Triangle& tri, V3 point) {  // primitives.rs:75-81
    V3 v = sub(point, tri.a.position);
    float dist = dot(v, tri.normal);
    return sub(point, mul(tri.normal, dist));
}

// ---------------------------------------------------------------- object.rs ---------------
struct BBox {
    V3 lo, hi;
};
// BoundingBox::intersects (object.rs:327-379)
bool bbox_intersects(const BBox& bb, const Ray& ray) {
    V3 start = ray.start;
    V3 invdir = div_under(ray.dir, 1.0f);
    float signs[3];
    for (int i = 0; i < 3; ++i) signs[i] = (float)(uint32_t)(invdir.v[i] < 0.0f);
    V3 bounds[2] = {bb.lo, bb.hi};
    size_t s0 = (size_t)signs[0], s1 = (size_t)signs[1], s2 = (size_t)signs[2];
    float txmin = (bounds[s0].v[0] - start.v[0]) * invdir.v[0];
    float txmax = (bounds[1 - s0].v[0] - start.v[0]) * invdir.v[0];
    float tymin = (bounds[s1].v[1] - start.v[1]) * invdir.v[1];
    float tymax = (bounds[1 - s1].v[1] - start.v[1]) * invdir.v[1];
    if ((txmin > tymax) || (tymin > txmax)) return false;
    if (tymin > txmin) txmin = tymin;
    if (tymax < txmax) txmax = tymax;
    float tzmin = (bounds[s2].v[2] - start.v[2]) * invdir.v[2];
    float tzmax = (bounds[1 - s2].v[2] - start.v[2]) * invdir.v[2];
    if (tzmin > txmin) txmin = tzmin;
    if (tzmax < txmax) txmax = tzmax;
    float t = txmin;
    if (t < 0.0f) {
        t = txmax;
        if (t < 0.0f) return false;
    }
    return true;
}

struct Object {
    std::vector<Triangle> faces;
    BBox bbox;
    Material material;
};
struct Hit {  // RaycastHit (raycasting.rs:43-54)
    size_t face_index;
    V3 position, normal;
    Bundle material;
};
// Object<Built>::intersects (object.rs:58-81)
bool object_intersects(const Object& obj, const Ray& ray, Hit* hit, uint64_t* tests) {
    if (!bbox_intersects(obj.bbox, ray)) return false;
    for (size_t i = 0; i < obj.faces.size(); ++i) {
        const Triangle& f = obj.faces[i];
        V3 pos, nrm, bary;
        ++*tests;
        if (triangle_intersects(f, ray, &pos, &nrm, &bary)) {
            hit->face_index = i;
            hit->position = pos;
            hit->normal = nrm;
            V2 uv = add2(add2(mul2(f.a.uv, bary.v[2]), mul2(f.b.uv, bary.v[0])), mul2(f.c.uv, bary.v[1]));
            hit->material = material_get(obj.material, uv.v[0], uv.v[1]);
            return true;
        }
    }
    return false;
}

// ---------------------------------------------------------------- light.rs / engine.rs ----
struct Light {
    V3 position;
    int variant;  // 0 point, 1 ambient
    Color color;
    float brightness;
};

struct Engine {
    std::vector<Object> objects;
    std::vector<Light> lights;
    Camera camera;
    uint32_t bounces;
    oracle_stats stats;

    // Engine::reaches_light (engine.rs:218-228)
    bool reaches_light(const Ray& ray, const Light& light) {
        float dist = len(sub(light.position, ray.start));
        for (const Object& o : objects) {
            Hit h;
            if (object_intersects(o, ray, &h, &stats.shadow_tests))
                return len(sub(h.position, ray.start)) > dist;
        }
        return true;
    }

    // Engine::cast_ray (engine.rs:112-216); returns the `lighting` list.
    void cast_ray(const Ray& ray, uint32_t bounce_depth, std::vector<Color>& lighting,
                  int32_t* face_out, int32_t* obj_out) {
        lighting.clear();
        bool have_closest = false;
        float closest = 0.0f;
        for (size_t oi = 0; oi < objects.size(); ++oi) {
            const Object& object = objects[oi];
            Hit hit;
            if (!object_intersects(object, ray, &hit, &stats.primary_tests)) continue;
            V3 position = hit.position, normal = hit.normal;
            const Bundle& material = hit.material;
            float dist_sq = len_sq(sub(position, camera.center));
            if (!have_closest || dist_sq < closest) {
                have_closest = true;
                closest = dist_sq;
                lighting.clear();
                if (face_out) *face_out = (int32_t)hit.face_index;
                if (obj_out) *obj_out = (int32_t)oi;
            } else {
                continue;
            }
            Color color = material.has_color ? material.color : Color{0.0f, 0.0f, 0.0f};
            for (const Light& light : lights) {
                if (light.variant == 1) continue;  // non-ambient lights first
                if (reaches_light(ray_new(add(position, mul(normal, 0.1f)), sub(light.position, position)),
                                  light)) {
                    float prod = rust_clamp(dot(normal, sub(light.position, position)), 0.0f, 1.0f);
                    if (std::isnan(prod)) prod = 0.0f;
                    float falloff = 1.0f / len(sub(light.position, position));
                    Color diffusion = cmul(cmul(cmul(cmul(cmulc(color, light.color),
                                                          material.has_diffuse ? material.diffuse : 0.5f),
                                                     prod),
                                                light.brightness),
                                           falloff);
                    float specular_power = material.has_sp ? material.sp : 1.0f;
                    V3 reflected = sub(ray.dir, mul(mul(normal, 2.0f), dot(ray.dir, normal)));
                    float res = rust_clamp(
                        (material.has_specular ? material.specular : 0.5f) * light.brightness *
                            oracle_powf(dot(normalize(reflected), normalize(sub(light.position, position))),
                                        specular_power),
                        0.0f, 1.0f);
                    Color specular = cmul(Color{res, res, res},
                                          rust_clamp(oracle_powf(falloff, specular_power), 0.0f, 1.0f));
                    lighting.push_back(cadd(diffusion, specular));
                }
                float reflection = material.has_refl ? material.refl : 0.0f;
                if (bounce_depth < bounces && reflection != 0.0f) {  // engine.rs:181-191
                    V3 start = add(position, mul(normal, 0.1f));
                    V3 dir = sub(ray.dir, mul(mul(normal, 2.0f), dot(ray.dir, normal)));
                    std::vector<Color> sub_lighting;
                    cast_ray(ray_new(start, dir), bounce_depth + 1, sub_lighting, nullptr, nullptr);
                    for (const Color& c : sub_lighting) lighting.push_back(cmul(c, reflection));
                }
            }
            for (const Light& ambient : lights) {
                if (ambient.variant != 1) continue;
                lighting.push_back(cmul(cmul(cmin(ambient.color, color),
                                             material.has_diffuse ? material.diffuse : 0.5f),
                                        ambient.brightness));
            }
        }
        if (!have_closest) lighting.push_back(Color{0.1f, 0.1f, 0.2f});
    }
};

// impl Sum for Color: reduce(|acc, cur| acc + cur).unwrap_or_default() (color.rs:82-87)
inline Color color_sum(const std::vector<Color>& items) {
    if (items.empty()) return Color{0.0f, 0.0f, 0.0f};
    Color acc = items[0];
    for (size_t i = 1; i < items.size(); ++i) acc = cadd(acc, items[i]);
    return acc;
}

Camera to_camera(const oracle_camera* c) {
    Camera cam;
    cam.center = mk(c->center[0], c->center[1], c->center[2]);
    cam.fov0 = c->fov0;
    cam.fov1 = c->fov1;
    cam.width = c->width;
    cam.z_dist = c->z_dist;
    return cam;
}
ImgRef to_img(oracle_image im, int ch) { return ImgRef{im.data, im.width, im.height, ch}; }

Triangle tri_from(const float* p, const float* n, const float* uv) {
    Vertex v[3];
    for (int k = 0; k < 3; ++k) {
        v[k].position = mk(p[3 * k], p[3 * k + 1], p[3 * k + 2]);
        v[k].normal = mk(n[3 * k], n[3 * k + 1], n[3 * k + 2]);
        v[k].uv = V2{{uv[2 * k], uv[2 * k + 1]}};
    }
    return triangle_new(v[0], v[1], v[2]);
}

bool img_ok(oracle_image im) { return !im.data || (im.width > 0 && im.height > 0); }

}  // namespace

extern "C" {

void oracle_vec_dot(const float a[3], const float b[3], float* out) {
    *out = dot(mk(a[0], a[1], a[2]), mk(b[0], b[1], b[2]));
}
void oracle_vec_cross(const float a[3], const float b[3], float out[3]) {
    V3 r = cross(mk(a[0], a[1], a[2]), mk(b[0], b[1], b[2]));
    std::memcpy(out, r.v, sizeof r.v);
}
void oracle_vec_angle(const float a[3], const float b[3], float* out) {  // vector.rs:161-165
    V3 x = mk(a[0], a[1], a[2]), y = mk(b[0], b[1], b[2]);
    float d = dot(x, y);
    float res = d / (len(x) * len(y));
    *out = std::acos(res);
}
void oracle_triangle_project(const float tri_pos[9], const float point[3], float out[3]) {
    float zeros[9] = {0}, uv[6] = {0};
    Triangle t = tri_from(tri_pos, zeros, uv);
    V3 r = triangle_project(t, mk(point[0], point[1], point[2]));
    std::memcpy(out, r.v, sizeof r.v);
}
int oracle_triangle_intersects(const float pos[9], const float nrm[9], const float start[3],
                               const float dir[3], float out_pos[3], float out_normal[3],
                               float out_bary[3]) {
    float uv[6] = {0};
    Triangle t = tri_from(pos, nrm, uv);
    Ray r = ray_new(mk(start[0], start[1], start[2]), mk(dir[0], dir[1], dir[2]));
    V3 p, n, b;
    if (!triangle_intersects(t, r, &p, &n, &b)) return 0;
    std::memcpy(out_pos, p.v, sizeof p.v);
    std::memcpy(out_normal, n.v, sizeof n.v);
    std::memcpy(out_bary, b.v, sizeof b.v);
    return 1;
}
void oracle_camera_size(const oracle_camera* c, uint32_t* w, uint32_t* h) {
    camera_size(to_camera(c), w, h);
}
void oracle_pixel_to_ray(const oracle_camera* c, float x, float y, float start[3], float dir[3]) {
    Ray r = pixel_to_ray(to_camera(c), x, y);
    std::memcpy(start, r.start.v, sizeof r.start.v);
    std::memcpy(dir, r.dir.v, sizeof r.dir.v);
}

float oracle_cosf(float x) { return cosf(x); }
float oracle_powf(float x, float y) { return powf(x, y); }

// wave.rs:100-137
int oracle_node_wave(uint32_t w, uint32_t h, float x_fac, float y_fac, float* out) {
    for (uint32_t y = 0; y < h; ++y)
        for (uint32_t x = 0; x < w; ++x) {
            float value = std::fabs(oracle_cosf(((float)x * x_fac + (float)y * y_fac) / 10.0f));
            out[(size_t)y * w + x] = value;
        }
    return ORACLE_OK;
}
// rgb.rs:64-103: pixels[index] of each input with the OUTPUT's index (panics past the end)
int oracle_node_rgb(uint32_t w, uint32_t h, oracle_image r, oracle_image g, oracle_image b,
                    float* out) {
    size_t n = (size_t)w * h;
    if (!r.data || !g.data || !b.data) return ORACLE_E_ARG;
    if ((size_t)r.width * r.height < n || (size_t)g.width * g.height < n ||
        (size_t)b.width * b.height < n)
        return ORACLE_E_OOB;
    for (uint32_t y = 0; y < h; ++y)
        for (uint32_t x = 0; x < w; ++x) {
            size_t index = (size_t)y * w + x;
            out[3 * index + 0] = r.data[index];
            out[3 * index + 1] = g.data[index];
            out[3 * index + 2] = b.data[index];
        }
    return ORACLE_OK;
}
// flat_color.rs:65-95
int oracle_node_flat_color(uint32_t w, uint32_t h, float r, float g, float b, float* out) {
    size_t n = (size_t)w * h;
    for (size_t i = 0; i < n; ++i) {
        out[3 * i + 0] = r;
        out[3 * i + 1] = g;
        out[3 * i + 2] = b;
    }
    return ORACLE_OK;
}
// mix_color.rs:57-102
int oracle_node_mix_color(uint32_t w, uint32_t h, oracle_image left, oracle_image right,
                          float factor, float* out) {
    if (!left.data || !right.data) return ORACLE_E_ARG;
    if ((w > 0 && h > 0) && (!left.width || !left.height || !right.width || !right.height))
        return ORACLE_E_OOB;  // `% 0` panics
    ImgRef L = to_img(left, 3), R = to_img(right, 3);
    for (uint32_t y = 0; y < h; ++y)
        for (uint32_t x = 0; x < w; ++x) {
            size_t index = (size_t)y * w + x;
            const float* l = L.data + 3 * mod_index(L, x, y);
            const float* r = R.data + 3 * mod_index(R, x, y);
            for (int c = 0; c < 3; ++c) out[3 * index + c] = l[c] * (1.0f - factor) + r[c] * factor;
        }
    return ORACLE_OK;
}
// main.rs:80-144: the example material graph evaluated node by node, as Graph::run does.
int oracle_example_material(uint32_t w, uint32_t h, float x_fac, float y_fac, float r, float g,
                            float b, float factor, float* out_color, float* out_diffuse) {
    size_t n = (size_t)w * h;
    std::vector<float> wave(n), rgb(3 * n), flat(3 * n);
    oracle_node_wave(w, h, x_fac, y_fac, wave.data());
    oracle_image wi{wave.data(), w, h};
    int st = oracle_node_rgb(w, h, wi, wi, wi, rgb.data());
    if (st) return st;
    oracle_node_flat_color(w, h, r, g, b, flat.data());
    st = oracle_node_mix_color(w, h, oracle_image{rgb.data(), w, h}, oracle_image{flat.data(), w, h},
                               factor, out_color);
    if (st) return st;
    std::memcpy(out_diffuse, wave.data(), n * sizeof(float));
    return ORACLE_OK;
}

void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]};
    uint32_t k0 = key[0], k1 = key[1];
    for (int round = 0; round < 10; ++round) {
        if (round) {
            k0 += 0x9E3779B9u;  // Weyl key schedule
            k1 += 0xBB67AE85u;
        }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0;
        c[1] = lo1;
        c[2] = n2;
        c[3] = lo0;
    }
    std::memcpy(out, c, sizeof c);
}

float oracle_jitter(uint32_t word) {
    // rand 0.8 UniformFloat::<f32>::sample_single(-1.0, 1.0): 23 random bits as a float in
    // [1, 2), minus 1, times the range, plus low (value0_1 * scale + low, unfused)
    uint32_t bits = (word >> 9) | 0x3F800000u;
    float value1_2;
    std::memcpy(&value1_2, &bits, sizeof bits);
    const float value0_1 = value1_2 - 1.0f;
    return value0_1 * 2.0f + -1.0f;
}

int oracle_render(const oracle_object* objects, uint32_t object_count, const oracle_light* lights,
                  uint32_t light_count, const oracle_camera* cam, uint32_t image_width,
                  uint32_t image_height, uint32_t row0, uint32_t rows, uint32_t bounces,
                  float* out_rgb, int32_t* out_face, int32_t* out_object, oracle_stats* stats) {
    return oracle_render_aa(objects, object_count, lights, light_count, cam, image_width, image_height,
                            row0, rows, bounces, 0, 0, out_rgb, out_face, out_object, stats);
}

// Engine::render restricted to the camera pixels [x0, x0 + cols) x rows [row0, row0 + rows):
// the same per-pixel loop body (engine.rs:52-78), output pixel (x, y) at (y - row0) * stride +
// (x - x0).  The whole-frame entry points pass x0 = 0, cols = camera width, stride = image width.
static int render_region(const oracle_object* objects, uint32_t object_count, const oracle_light* lights,
                         uint32_t light_count, const oracle_camera* cam, uint32_t image_width,
                         uint32_t image_height, uint32_t row0, uint32_t rows, uint32_t x0, uint32_t cols,
                         uint32_t stride, uint32_t bounces, uint32_t anti_aliasing, uint64_t seed, float* out_rgb,
                         int32_t* out_face, int32_t* out_object, oracle_stats* stats) {
    Engine e;
    e.camera = to_camera(cam);
    e.bounces = bounces;
    e.stats = oracle_stats{0, 0, 0};
    for (uint32_t i = 0; i < object_count; ++i) {
        const oracle_object& o = objects[i];
        Object obj;
        obj.faces.reserve(o.triangle_count);
        for (uint32_t t = 0; t < o.triangle_count; ++t)
            obj.faces.push_back(tri_from(o.positions + 9 * (size_t)t, o.normals + 9 * (size_t)t,
                                         o.uvs + 6 * (size_t)t));
        obj.bbox = BBox{mk(o.bbox_min[0], o.bbox_min[1], o.bbox_min[2]),
                        mk(o.bbox_max[0], o.bbox_max[1], o.bbox_max[2])};
        const oracle_material& m = o.material;
        if (!img_ok(m.color) || !img_ok(m.diffuse) || !img_ok(m.specular) || !img_ok(m.specular_power) ||
            !img_ok(m.reflection))
            return ORACLE_E_OOB;
        obj.material = Material{to_img(m.color, 3), to_img(m.diffuse, 1), to_img(m.specular, 1),
                                to_img(m.specular_power, 1), to_img(m.reflection, 1)};
        e.objects.push_back(std::move(obj));
    }
    for (uint32_t i = 0; i < light_count; ++i) {
        const oracle_light& l = lights[i];
        e.lights.push_back(Light{mk(l.position[0], l.position[1], l.position[2]), l.variant,
                                 Color{l.color[0], l.color[1], l.color[2]}, l.brightness});
    }
    uint32_t width, height;
    camera_size(e.camera, &width, &height);
    if (row0 + rows > height) return ORACLE_E_ARG;
    // Image::set (image.rs:41-43) indexes with the ENGINE image width; it panics past the end.
    if (width > 0 && height > 0 &&
        ((uint64_t)(height - 1) * image_width + (width - 1)) >= (uint64_t)image_width * image_height)
        return ORACLE_E_OOB;
    if (cols == UINT32_MAX) cols = width;
    if ((uint64_t)x0 + cols > width) return ORACLE_E_ARG;
    if (stride == UINT32_MAX) stride = image_width;
    std::vector<Color> lighting;
    for (uint32_t y = row0; y < row0 + rows; ++y) {
        for (uint32_t x = x0; x < x0 + cols; ++x) {
            Ray ray = pixel_to_ray(e.camera, (float)x / (float)width, (float)y / (float)height);
            int32_t face = -1, obj = -1;
            e.cast_ray(ray, 0, lighting, &face, &obj);
            if (face >= 0) ++e.stats.hit_pixels;
            Color average = color_sum(lighting);
            // engine.rs:62-69: anti_aliasing more rays at (x + jx, y + jy), jx and jy drawn
            // from gen_range(-1.0..1.0) in that order.  thread_rng (ChaCha12, OS-seeded) is
            // replaced by Philox4x32-10 keyed by `seed`, counter (x, y, sample, 0): words 0
            // and 1 are the two draws.
            for (uint32_t s = 0; s < anti_aliasing; ++s) {
                const uint32_t ctr[4] = {x, y, s, 0u};
                const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
                uint32_t r[4];
                oracle_philox4x32_10(ctr, key, r);
                const float jx = oracle_jitter(r[0]), jy = oracle_jitter(r[1]);
                Ray aa_ray = pixel_to_ray(e.camera, ((float)x + jx) / (float)width, ((float)y + jy) / (float)height);
                e.cast_ray(aa_ray, 0, lighting, nullptr, nullptr);
                average = cadd(average, color_sum(lighting));  // AddAssign (color.rs:12)
            }
            if (anti_aliasing > 0) {  // (average / aa as f32).clamp() (engine.rs:71-73); else raw
                const float n = (float)anti_aliasing;
                average = Color{rust_clamp(average.r / n, 0.0f, 1.0f), rust_clamp(average.g / n, 0.0f, 1.0f),
                                rust_clamp(average.b / n, 0.0f, 1.0f)};
            }
            size_t idx = (size_t)(y - row0) * stride + (x - x0);
            out_rgb[3 * idx + 0] = average.r;
            out_rgb[3 * idx + 1] = average.g;
            out_rgb[3 * idx + 2] = average.b;
            if (out_face) out_face[idx] = face;
            if (out_object) out_object[idx] = obj;
        }
    }
    if (stats) *stats = e.stats;
    return ORACLE_OK;
}

int oracle_render_aa(const oracle_object* objects, uint32_t object_count, const oracle_light* lights,
                     uint32_t light_count, const oracle_camera* cam, uint32_t image_width,
                     uint32_t image_height, uint32_t row0, uint32_t rows, uint32_t bounces,
                     uint32_t anti_aliasing, uint64_t seed, float* out_rgb, int32_t* out_face,
                     int32_t* out_object, oracle_stats* stats) {
    return render_region(objects, object_count, lights, light_count, cam, image_width, image_height, row0, rows, 0,
                         UINT32_MAX, UINT32_MAX, bounces, anti_aliasing, seed, out_rgb, out_face, out_object, stats);
}

int oracle_render_span(const oracle_object* objects, uint32_t object_count, const oracle_light* lights,
                       uint32_t light_count, const oracle_camera* cam, uint32_t row0, uint32_t rows, uint32_t x0,
                       uint32_t cols, float* out_rgb, int32_t* out_face, oracle_stats* stats) {
    uint32_t width, height;
    camera_size(to_camera(cam), &width, &height);
    return render_region(objects, object_count, lights, light_count, cam, width, height, row0, rows, x0, cols, cols,
                         0, 0, 0, out_rgb, out_face, nullptr, stats);
}

int oracle_ppm_bytes(const float* rgb, uint32_t width, uint32_t height, uint8_t* out) {
    size_t o = 0;
    for (uint32_t yy = 0; yy < height; ++yy) {
        uint32_t y = height - 1 - yy;  // windows(w).step_by(w).rev()
        for (uint32_t x = 0; x < width; ++x) {
            const float* p = rgb + 3 * ((size_t)y * width + x);
            out[o++] = sat_u8(p[0] * 255.0f);  // Color::as_bytes (color.rs:31-37)
            out[o++] = sat_u8(p[1] * 255.0f);
            out[o++] = sat_u8(p[2] * 255.0f);
        }
    }
    return ORACLE_OK;
}
size_t oracle_ppm_header(uint32_t width, uint32_t height, char* buf, size_t cap) {
    int n = std::snprintf(buf, cap, "P6 %u %u %u\n", width, height, 255u);
    return n < 0 ? 0 : (size_t)n;
}

// ------------------------------------------------------------ Object::load_obj --------------
namespace {
bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v'; }
std::vector<std::string> split_ws(const std::string& s) {
    std::vector<std::string> out;
    size_t i = 0;
    while (i < s.size()) {
        while (i < s.size() && is_ws(s[i])) ++i;
        size_t j = i;
        while (j < s.size() && !is_ws(s[j])) ++j;
        if (j > i) out.push_back(s.substr(i, j - i));
        i = j;
    }
    return out;
}
// str::parse::<f32>: decimal literals, inf/infinity/nan; no hex, no surrounding whitespace.
bool parse_f32(const std::string& tok, float* out) {
    if (tok.empty()) return false;
    for (char c : tok)
        if (c == 'x' || c == 'X' || c == 'p' || c == 'P') return false;
    char* end = nullptr;
    *out = std::strtof(tok.c_str(), &end);
    return end == tok.c_str() + tok.size();
}
// str::parse::<usize>: optional '+', decimal digits only.
bool parse_usize(const std::string& tok, size_t* out) {
    size_t i = 0;
    if (!tok.empty() && tok[0] == '+') i = 1;
    if (i >= tok.size()) return false;
    size_t v = 0;
    for (; i < tok.size(); ++i) {
        if (tok[i] < '0' || tok[i] > '9') return false;
        v = v * 10 + (size_t)(tok[i] - '0');
    }
    *out = v;
    return true;
}
}  // namespace

int oracle_load_obj(const char* text, size_t len, float** positions, float** normals, float** uvs,
                    uint32_t* triangle_count, char* err, size_t err_cap) {
    auto fail = [&](int code, const std::string& msg) {
        if (err && err_cap) std::snprintf(err, err_cap, "%s", msg.c_str());
        return code;
    };
    std::vector<V3> verts, norms;
    std::vector<V2> tex;
    std::vector<float> P, N, U;
    std::string content(text, len);
    size_t pos = 0;
    size_t line_no = 0;
    while (pos < content.size()) {  // str::lines(): split on '\n', strip one trailing '\r'
        size_t nl = content.find('\n', pos);
        std::string line = content.substr(pos, nl == std::string::npos ? std::string::npos : nl - pos);
        pos = (nl == std::string::npos) ? content.size() : nl + 1;
        if (!line.empty() && line.back() == '\r') line.pop_back();
        size_t ln = line_no++;
        if (line.empty() || line[0] == '#') continue;
        std::vector<std::string> tok = split_ws(line);
        if (tok.empty()) return fail(ORACLE_E_PARSE, "line " + std::to_string(ln) + ": no marker");
        const std::string& marker = tok[0];
        if (marker == "o" || marker == "g") {
            if (tok.size() < 2) return fail(ORACLE_E_PARSE, "missing name");
        } else if (marker == "s") {
            if (tok.size() < 2) return fail(ORACLE_E_PARSE, "missing smooth setting");
            const std::string& v = tok[1];
            if (!(v == "1" || v == "on" || v == "0" || v == "off"))
                return fail(ORACLE_E_PARSE, "Unhandled smooth shading setting `" + v + "`");
        } else if (marker == "v" || marker == "vn" || marker == "vt") {
            std::vector<float> coords;
            for (size_t i = 1; i < tok.size(); ++i) {
                float f;
                if (!parse_f32(tok[i], &f)) return fail(ORACLE_E_PARSE, "Failed to parse coords: " + tok[i]);
                coords.push_back(f);
            }
            if (!(coords.size() >= 2 && coords.size() < 4))
                return fail(ORACLE_E_PARSE, "Invalid coordinate count at line " + std::to_string(ln));
            if (marker == "vt") {
                tex.push_back(V2{{coords[0], coords[1]}});
            } else {
                if (coords.size() < 3) return fail(ORACLE_E_PARSE, "coords[0..=2] out of range");
                (marker == "v" ? verts : norms).push_back(mk(coords[0], coords[1], coords[2]));
            }
        } else if (marker == "f") {
            std::vector<Vertex> vs;
            for (size_t i = 1; i < tok.size(); ++i) {
                std::vector<std::string> parts;
                size_t s = 0;
                const std::string& t = tok[i];
                while (true) {
                    size_t sl = t.find('/', s);
                    parts.push_back(t.substr(s, sl == std::string::npos ? std::string::npos : sl - s));
                    if (sl == std::string::npos) break;
                    s = sl + 1;
                }
                size_t idx[3];
                bool ok[3];
                for (int k = 0; k < 3; ++k) ok[k] = k < (int)parts.size() && parse_usize(parts[k], &idx[k]);
                // Vertex { position: vertices[i0-1], uv: uvs[i1-1], normal: normals[i2-1] }
                if ((int)parts.size() < 1 || !ok[0] || idx[0] == 0 || idx[0] > verts.size())
                    return fail(ORACLE_E_PARSE, "bad vertex index at line " + std::to_string(ln));
                if ((int)parts.size() < 2 || !ok[1] || idx[1] == 0 || idx[1] > tex.size())
                    return fail(ORACLE_E_PARSE, "bad uv index at line " + std::to_string(ln));
                if ((int)parts.size() < 3 || !ok[2] || idx[2] == 0 || idx[2] > norms.size())
                    return fail(ORACLE_E_PARSE, "bad normal index at line " + std::to_string(ln));
                vs.push_back(Vertex{verts[idx[0] - 1], norms[idx[2] - 1], tex[idx[1] - 1]});
            }
            if (vs.size() != 3)
                return fail(ORACLE_E_PARSE, "Invalid vertex count for face at line " + std::to_string(ln));
            for (int k = 0; k < 3; ++k) {
                P.insert(P.end(), vs[k].position.v, vs[k].position.v + 3);
                N.insert(N.end(), vs[k].normal.v, vs[k].normal.v + 3);
                U.insert(U.end(), vs[k].uv.v, vs[k].uv.v + 2);
            }
        } else {
            return fail(ORACLE_E_PARSE, "Unhandled marker " + marker);
        }
    }
    if (verts.empty()) return fail(ORACLE_E_BUILD, "Missing vertices");  // Object::build
    if (norms.empty()) return fail(ORACLE_E_BUILD, "Missing normals");
    size_t T = P.size() / 9;
    *positions = (float*)std::malloc(sizeof(float) * (P.size() ? P.size() : 1));
    *normals = (float*)std::malloc(sizeof(float) * (N.size() ? N.size() : 1));
    *uvs = (float*)std::malloc(sizeof(float) * (U.size() ? U.size() : 1));
    if (!P.empty()) std::memcpy(*positions, P.data(), P.size() * sizeof(float));
    if (!N.empty()) std::memcpy(*normals, N.data(), N.size() * sizeof(float));
    if (!U.empty()) std::memcpy(*uvs, U.data(), U.size() * sizeof(float));
    *triangle_count = (uint32_t)T;
    return ORACLE_OK;
}
void oracle_free(void* p) { std::free(p); }

}  // extern "C"
