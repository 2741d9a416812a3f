// shaderlib.hip — gfx950 kernels for the four shaderlib node operators (src/shaderlib/*.rs)
// and the fused evaluation of main.rs's material graph.
//
// All of them are streaming, HBM-write-bound kernels (0 reads for wave/flat, 12 B/texel of
// reads for rgb, 24 for mix).  rgb, flat and mix produce kVec consecutive texels per thread so
// that every store is a 16-B-per-lane (dwordx4) store when the row is aligned, with a scalar
// tail; wave and the fused material kernel one texel per thread (below).  Grids stride over the
// image.
#include "device_math.hpp"
#include "glibc_cosf.hpp"
#include "int_div.hpp"
#include "internal.hpp"

namespace eray {
namespace gpu {
namespace {

constexpr int kBlock = 256;
constexpr int kVec = 4;

inline unsigned grid_for1(size_t items) {
    size_t blocks = (items + kBlock - 1) / kBlock;
    if (blocks > 8192) blocks = 8192;
    return blocks ? (unsigned)blocks : 1u;
}

inline unsigned grid_for(size_t items) {
    size_t blocks = (items + (size_t)kBlock * kVec - 1) / ((size_t)kBlock * kVec);
    if (blocks > 2048) blocks = 2048;
    return blocks ? (unsigned)blocks : 1u;
}

// wave.rs:127 — |cos((x as f32 * x_fac + y as f32 * y_fac) / 10.)|
__device__ __forceinline__ float wave_value(uint32_t x, uint32_t y, float xf, float yf) {
    const float arg = libm::div10_f32((float)x * xf + (float)y * yf);
    return __builtin_fabsf(libm::cosf_glibc(arg));
}

// One texel per thread: the restated cosf is a chain of dependent double-precision steps, so
// its latency is hidden by resident waves (measured faster than four texels per thread with 16-B
// stores: 6.9 vs 10.1 us per 1024 x 1024 material update, profiles/r05/ab/).  Below 2^32 texels
// (and 4 GB of output) the texel's row is a multiply-high by the launch's invariant divisor
// (int_div.hpp) and the stores buffer stores with 32-bit offsets: the index arithmetic is a few
// of the ~110 VALU instructions per texel the cosf leaves (profiles/r05/material_pmc.json).
struct TexelIndex {
    uint32_t w;
    DivU32 dw;  // texel index / w
};
__device__ __forceinline__ void texel_xy(uint32_t i, const TexelIndex& t, uint32_t& x, uint32_t& y) {
    y = div_u32(i, t.dw);
    x = i - y * t.w;
}
__device__ __forceinline__ void store_f32(float* base, uint32_t byte_off, float v) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, -1, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, byte_off, 0, 0);
}

template <bool kWide>  // kWide: 64-bit indices (2^32 texels or more)
__global__ void __launch_bounds__(kBlock) wave_kernel(TexelIndex t, uint32_t h, float xf, float yf,
                                                      float* __restrict__ out) {
    if constexpr (kWide) {
        const size_t n = (size_t)t.w * h, stride = (size_t)gridDim.x * kBlock;
        for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
            const uint32_t y = (uint32_t)(i / t.w), x = (uint32_t)(i - (size_t)y * t.w);
            out[i] = wave_value(x, y, xf, yf);
        }
    } else {
        const uint32_t n = t.w * h, stride = gridDim.x * kBlock;
        for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
            uint32_t x, y;
            texel_xy(i, t, x, y);
            store_f32(out, 4u * i, wave_value(x, y, xf, yf));
        }
    }
}

__device__ __forceinline__ void store_rgb4(float* __restrict__ out, size_t i0, size_t n,
                                           const float (&c)[kVec][3]) {
    float* p = out + 3 * i0;
    if (i0 + kVec <= n && ((reinterpret_cast<uintptr_t>(p) & 15) == 0)) {
        float4* q = reinterpret_cast<float4*>(p);
        q[0] = make_float4(c[0][0], c[0][1], c[0][2], c[1][0]);
        q[1] = make_float4(c[1][1], c[1][2], c[2][0], c[2][1]);
        q[2] = make_float4(c[2][2], c[3][0], c[3][1], c[3][2]);
    } else {
        for (int k = 0; k < kVec && i0 + k < n; ++k) {
            p[3 * k + 0] = c[k][0];
            p[3 * k + 1] = c[k][1];
            p[3 * k + 2] = c[k][2];
        }
    }
}

// rgb.rs:89-95 — Color::new(red.pixels[i], green.pixels[i], blue.pixels[i])
__global__ void __launch_bounds__(kBlock) rgb_kernel(size_t n, const float* __restrict__ r,
                                                     const float* __restrict__ g,
                                                     const float* __restrict__ b,
                                                     float* __restrict__ out) {
    const size_t stride = (size_t)gridDim.x * kBlock * kVec;
    for (size_t i0 = ((size_t)blockIdx.x * kBlock + threadIdx.x) * kVec; i0 < n; i0 += stride) {
        float c[kVec][3];
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
            size_t i = i0 + k < n ? i0 + k : n - 1;
            c[k][0] = r[i];
            c[k][1] = g[i];
            c[k][2] = b[i];
        }
        store_rgb4(out, i0, n, c);
    }
}

// flat_color.rs:88 — Image::new(w, h, Color::new(r, g, b))
__global__ void __launch_bounds__(kBlock) flat_kernel(size_t n, float r, float g, float b,
                                                      float* __restrict__ out) {
    const size_t stride = (size_t)gridDim.x * kBlock * kVec;
    for (size_t i0 = ((size_t)blockIdx.x * kBlock + threadIdx.x) * kVec; i0 < n; i0 += stride) {
        float c[kVec][3];
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
            c[k][0] = r;
            c[k][1] = g;
            c[k][2] = b;
        }
        store_rgb4(out, i0, n, c);
    }
}

// mix_color.rs:84-91 — interp(l, r) = l * (1. - factor) + r * factor on mod_get'd texels
__global__ void __launch_bounds__(kBlock) mix_kernel(uint32_t w, uint32_t h, TexView left,
                                                     TexView right, float factor,
                                                     float* __restrict__ out) {
    const size_t n = (size_t)w * h;
    const float omf = 1.0f - factor;
    const size_t stride = (size_t)gridDim.x * kBlock * kVec;
    for (size_t i0 = ((size_t)blockIdx.x * kBlock + threadIdx.x) * kVec; i0 < n; i0 += stride) {
        float c[kVec][3];
        uint32_t y = (uint32_t)(i0 / w), x = (uint32_t)(i0 - (size_t)y * w);
#pragma unroll
        for (int k = 0; k < kVec; ++k) {
            uint32_t yy = y < h ? y : h - 1;
            const float* l = left.data + 3 * (size_t)((yy % left.h) * left.w + x % left.w);
            const float* rr = right.data + 3 * (size_t)((yy % right.h) * right.w + x % right.w);
            c[k][0] = l[0] * omf + rr[0] * factor;
            c[k][1] = l[1] * omf + rr[1] * factor;
            c[k][2] = l[2] * omf + rr[2] * factor;
            if (++x == w) { x = 0; ++y; }
        }
        store_rgb4(out, i0, n, c);
    }
}

// main.rs:80-144 fused: wave -> rgb(wave, wave, wave) -> mix(.., flat(r, g, b), factor);
// diffuse = wave.  Every node's image has the graph's width x height, so mix's mod_get is the
// identity and the chain reduces to per-texel arithmetic in the nodes' own operation order
// (r * factor is the same product per texel, so it is formed once).
// kTexels > 1: each thread evaluates texels i, i + stride, ... (stride = the grid's threads)
// together, so their independent cosf chains interleave (ILP) over a grid that many times smaller.
template <bool kWide, int kTexels = 1>
__global__ void __launch_bounds__(kBlock) material_example_kernel(
    TexelIndex t, uint32_t h, float xf, float yf, float r, float g, float b, float factor,
    float* __restrict__ color, float* __restrict__ diffuse) {
    const float omf = 1.0f - factor, rf = r * factor, gf = g * factor, bf = b * factor;
    if constexpr (kWide) {
        const size_t n = (size_t)t.w * h, stride = (size_t)gridDim.x * kBlock;
        for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
            const uint32_t y = (uint32_t)(i / t.w), x = (uint32_t)(i - (size_t)y * t.w);
            const float v = wave_value(x, y, xf, yf), m = v * omf;
            if (color) {
                float* c = color + 3 * i;
                c[0] = m + rf;
                c[1] = m + gf;
                c[2] = m + bf;
            }
            if (diffuse) diffuse[i] = v;
        }
    } else {
        const uint32_t n = t.w * h, stride = gridDim.x * kBlock;
        for (uint32_t i0 = blockIdx.x * kBlock + threadIdx.x; i0 < n; i0 += kTexels * stride) {
            float v[kTexels];
#pragma unroll
            for (int k = 0; k < kTexels; ++k) {
                uint32_t x, y;
                texel_xy(min(i0 + (uint32_t)k * stride, n - 1u), t, x, y);
                v[k] = wave_value(x, y, xf, yf);
            }
#pragma unroll
            for (int k = 0; k < kTexels; ++k) {
                const uint32_t i = i0 + (uint32_t)k * stride;
                if (i >= n) break;
                const float m = v[k] * omf;
                if (color) {
                    store_f32(color, 12u * i, m + rf);
                    store_f32(color, 12u * i + 4u, m + gf);
                    store_f32(color, 12u * i + 8u, m + bf);
                }
                if (diffuse) store_f32(diffuse, 4u * i, v[k]);
            }
        }
    }
}
// texels per thread of the fused material kernel (narrow launches)
constexpr int kMatTexels = 2;

}  // namespace

// 32-bit texel indices and byte offsets while the largest output (12 B per texel) stays below 4 GB
inline bool narrow_texels(size_t n) { return n * 12 <= UINT32_MAX; }

hipError_t launch_wave(uint32_t w, uint32_t h, float xf, float yf, float* out, hipStream_t s) {
    size_t n = (size_t)w * h;
    if (!n) return hipSuccess;
    const TexelIndex t{w, make_div_u32(w)};
    if (narrow_texels(n))
        wave_kernel<false><<<grid_for1(n), kBlock, 0, s>>>(t, h, xf, yf, out);
    else
        wave_kernel<true><<<grid_for1(n), kBlock, 0, s>>>(t, h, xf, yf, out);
    return hipGetLastError();
}
hipError_t launch_rgb(uint32_t w, uint32_t h, const float* r, const float* g, const float* b,
                      float* out, hipStream_t s) {
    size_t n = (size_t)w * h;
    if (!n) return hipSuccess;
    rgb_kernel<<<grid_for(n), kBlock, 0, s>>>(n, r, g, b, out);
    return hipGetLastError();
}
hipError_t launch_flat(uint32_t w, uint32_t h, float r, float g, float b, float* out,
                       hipStream_t s) {
    size_t n = (size_t)w * h;
    if (!n) return hipSuccess;
    flat_kernel<<<grid_for(n), kBlock, 0, s>>>(n, r, g, b, out);
    return hipGetLastError();
}
hipError_t launch_mix(uint32_t w, uint32_t h, TexView left, TexView right, float factor,
                      float* out, hipStream_t s) {
    size_t n = (size_t)w * h;
    if (!n) return hipSuccess;
    mix_kernel<<<grid_for(n), kBlock, 0, s>>>(w, h, left, right, factor, out);
    return hipGetLastError();
}
hipError_t launch_material_example(uint32_t w, uint32_t h, float xf, float yf, float r, float g,
                                   float b, float factor, float* color, float* diffuse,
                                   hipStream_t s) {
    size_t n = (size_t)w * h;
    if (!n) return hipSuccess;
    const TexelIndex t{w, make_div_u32(w)};
    if (narrow_texels(n))
        material_example_kernel<false, kMatTexels><<<grid_for1((n + kMatTexels - 1) / kMatTexels), kBlock, 0, s>>>(
            t, h, xf, yf, r, g, b, factor, color, diffuse);
    else
        material_example_kernel<true><<<grid_for1(n), kBlock, 0, s>>>(t, h, xf, yf, r, g, b, factor, color, diffuse);
    return hipGetLastError();
}

}  // namespace gpu
}  // namespace eray
