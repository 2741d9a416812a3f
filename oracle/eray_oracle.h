/*
 * eray_oracle.h — C interface of the CPU ORACLE (test infrastructure only).
 *
 * This header and the library built from oracle/eray_oracle.cpp are the CHECKER for the
 * MI355X product path.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it.  It is never linked into eray_amd/ and the product never falls back to it.
 *
 * The structs here are deliberately independent of include/eray_hip.h (the product's C-ABI):
 * the oracle is a second, literal implementation of the reference semantics, so the two must
 * not share code.
 */
#ifndef ERAY_ORACLE_H
#define ERAY_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* An image socket value (graph.rs:160-169 IValue / IColor). data == NULL means "absent"
 * (the Option is None or the selected output is missing / of the wrong type). */
typedef struct {
    const float* data;      /* IValue: 1 float per pixel, IColor: 3 floats (r,g,b) per pixel */
    uint32_t width, height;
} oracle_image;

/* Material::get inputs (material.rs:56-94): the selected standard outputs. */
typedef struct {
    oracle_image color;          /* IColor */
    oracle_image diffuse;        /* IValue */
    oracle_image specular;       /* IValue */
    oracle_image specular_power; /* IValue */
    oracle_image reflection;     /* IValue */
} oracle_material;

/* Object<Built> (object.rs:30-52): faces in file order as per-face vertex copies. */
typedef struct {
    const float* positions;  /* T x 9 : a.xyz b.xyz c.xyz */
    const float* normals;    /* T x 9 */
    const float* uvs;        /* T x 6 */
    uint32_t triangle_count;
    float bbox_min[3];       /* BoundingBox ranges' starts (object.rs:306-324) */
    float bbox_max[3];       /* ... and ends */
    oracle_material material;
} oracle_object;

typedef struct {
    float center[3];
    float fov0, fov1;        /* Fov(f32, f32) (camera.rs:7-12) */
    uint32_t width;
    float z_dist;
} oracle_camera;

typedef struct {
    float position[3];       /* Transform::translation() (matrix.rs:45-47) */
    int32_t variant;         /* 0 = Point, 1 = Ambient (light.rs:20-25) */
    float color[3];
    float brightness;
} oracle_light;

typedef struct {
    uint64_t primary_tests;  /* Triangle::intersects calls made for camera / bounce rays */
    uint64_t shadow_tests;   /* ... made inside reaches_light */
    uint64_t hit_pixels;     /* pixels whose camera ray hit some object */
} oracle_stats;

/* Status codes: 0 ok, <0 error (the reference panics in those cases). */
#define ORACLE_OK 0
#define ORACLE_E_ARG (-1)
#define ORACLE_E_OOB (-2)      /* index out of bounds: the reference panics */
#define ORACLE_E_PARSE (-3)    /* load_obj panics (object.rs:101-186, 396-421) */
#define ORACLE_E_BUILD (-4)    /* Object::build Err (object.rs:213-218) */
#define ORACLE_E_IO (-5)

/* --- vector.rs known answers (vector.rs:243-299) --------------------------------------- */
void oracle_vec_dot(const float a[3], const float b[3], float* out);
void oracle_vec_cross(const float a[3], const float b[3], float out[3]);
void oracle_vec_angle(const float a[3], const float b[3], float* out);
void oracle_triangle_project(const float tri_pos[9], const float point[3], float out[3]);
/* Triangle::intersects on one ray; returns 1 on hit and fills pos/normal/bary. */
int oracle_triangle_intersects(const float pos[9], const float nrm[9], const float start[3],
                               const float dir_unnormalized[3], float out_pos[3],
                               float out_normal[3], float out_bary[3]);
/* Camera::size and Camera::pixel_to_ray (already normalised by Ray::new). */
void oracle_camera_size(const oracle_camera* cam, uint32_t* w, uint32_t* h);
void oracle_pixel_to_ray(const oracle_camera* cam, float x, float y, float start[3], float dir[3]);

/* --- math dependencies of the path (Rust std -> glibc libm) ----------------------------- */
float oracle_cosf(float x);              /* f32::cos  (wave.rs:127) */
float oracle_powf(float x, float y);     /* f32::powf (engine.rs:171,174) */

/* --- shaderlib nodes (src/shaderlib/{wave,rgb,flat_color,mix_color}.rs); outputs allocated by the caller -------------- */
int oracle_node_wave(uint32_t w, uint32_t h, float x_fac, float y_fac, float* out);
int oracle_node_rgb(uint32_t w, uint32_t h, oracle_image r, oracle_image g, oracle_image b,
                    float* out_rgb);
int oracle_node_flat_color(uint32_t w, uint32_t h, float r, float g, float b, float* out_rgb);
int oracle_node_mix_color(uint32_t w, uint32_t h, oracle_image left, oracle_image right,
                          float factor, float* out_rgb);
/* main.rs:80-144's graph: color = mix(rgb(wave,wave,wave), flat(r,g,b), factor), diffuse = wave */
int oracle_example_material(uint32_t w, uint32_t h, float x_fac, float y_fac, float r, float g,
                            float b, float factor, float* out_color, float* out_diffuse);

/* --- Engine::render (engine.rs:46-81) over camera rows [row0, row0+rows) ---------------- *
 * out_rgb: rows x image_width x 3 floats, pixel (x, row0 + j) at [(j*image_width + x)*3].
 * Pixels outside the camera's x-range are left untouched.  out_face (optional): the face
 * index of the closest object's hit, or -1 (object index in out_object, optional).          */
int oracle_render(const oracle_object* objects, uint32_t object_count,
                  const oracle_light* lights, uint32_t light_count, const oracle_camera* cam,
                  uint32_t image_width, uint32_t image_height, uint32_t row0, uint32_t rows,
                  uint32_t bounces, float* out_rgb, int32_t* out_face, int32_t* out_object,
                  oracle_stats* stats);

/* The same with Engine::anti_aliasing = `anti_aliasing` (engine.rs:59-77): the reference's
 * OS-seeded thread_rng is replaced by Philox4x32-10 (key = seed, counter = (x, y, sample, 0));
 * each draw maps a 32-bit word to [-1, 1) as rand 0.8's gen_range(-1.0..1.0) does.           */
int oracle_render_aa(const oracle_object* objects, uint32_t object_count,
                     const oracle_light* lights, uint32_t light_count, const oracle_camera* cam,
                     uint32_t image_width, uint32_t image_height, uint32_t row0, uint32_t rows,
                     uint32_t bounces, uint32_t anti_aliasing, uint64_t seed, float* out_rgb,
                     int32_t* out_face, int32_t* out_object, oracle_stats* stats);
/* Engine::render's loop body over the pixel span [x0, x0+cols) x camera rows [row0, row0+rows)
 * (AA = 0, no bounces): out_rgb is rows x cols x 3 floats, out_face (optional) rows x cols.
 * Lets a test check a few pixels of a frame whose full oracle render would take minutes. */
int oracle_render_span(const oracle_object* objects, uint32_t object_count,
                       const oracle_light* lights, uint32_t light_count, const oracle_camera* cam,
                       uint32_t row0, uint32_t rows, uint32_t x0, uint32_t cols, float* out_rgb,
                       int32_t* out_face, oracle_stats* stats);
/* Philox4x32-10 (Salmon et al., SC'11; Random123's philox4x32 with 10 rounds) and the
 * gen_range(-1.0..1.0) mapping of one of its words. */
void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
float oracle_jitter(uint32_t word);

/* Image<Color>::save_as_ppm body bytes (image.rs:48-74): rows bottom-up, sat-u8 bytes. */
int oracle_ppm_bytes(const float* rgb, uint32_t width, uint32_t height, uint8_t* out);
/* "P6 {w} {h} 255\n" (image.rs:56); returns header length. */
size_t oracle_ppm_header(uint32_t width, uint32_t height, char* buf, size_t cap);

/* --- Object::load_obj + build (object.rs:101-230), panics reported as errors ------------ *
 * Parses `text`; on success allocates positions, normals and uvs (free them with oracle_free). */
int oracle_load_obj(const char* text, size_t len, float** positions, float** normals,
                    float** uvs, uint32_t* triangle_count, char* err, size_t err_cap);
void oracle_free(void* p);

#ifdef __cplusplus
}
#endif
#endif
