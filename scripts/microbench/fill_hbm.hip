// Microbenchmark (diagnostic, not product): the background write stream into rings beyond the
// Infinity Cache — which store order and cache policy writes 3840x2160 frames into 4 ring slots
// (and C2's 8-frame launches into 16 slots) fastest.  Patterns alternate round by round on one box.
//   blk      render.hip's fill / ceiling_fill_kernel: wave w takes 64x4 blocks w, w + nw, ...
//   flat     each array as one byte range, grid-stride 16 B per lane (the grid writes 4 KB per
//            workgroup of one contiguous region per step), RGB then PPM
//   chunk    each workgroup its own contiguous 1/grid of each array, 4 KB per step
//   rows     flat, but per step the grid takes whole camera rows: RGB row and its PPM row together
//   *nt      the same with non-temporal stores (sc1 nt)
//   hipcc -O3 --offload-arch=gfx950 fill_hbm.hip -o fill_hbm && ./fill_hbm
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <cstdio>

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
template <bool kNt>
__device__ __forceinline__ void st16(void* base, uint32_t off, uint4 v) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, -1, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{v.x, v.y, v.z, v.w}, r, off, 0, kNt ? 18 : 16);
}
__device__ __forceinline__ uint4 pat(uint32_t ph) {
    const uint32_t a = 0x3dcccccdu, b = 0x3e4ccccdu;
    return ph == 0 ? make_uint4(a, a, b, a) : ph == 1 ? make_uint4(a, b, a, a) : make_uint4(b, a, a, b);
}
struct Frames {
    float* rgb;
    uint8_t* ppm;
    uint32_t W, H, F;
    uint64_t stride;  // bytes between frames of the RGB array (PPM: stride / 4)
};

template <int P, bool kNt>
__global__ void __launch_bounds__(256) fill(Frames fr) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t tiles_x = fr.W / 64, bands = fr.H / 4, nblk = tiles_x * bands;
    for (uint32_t f = 0; f < fr.F; ++f) {
        char* rgb = reinterpret_cast<char*>(fr.rgb) + f * fr.stride;
        uint8_t* ppm = fr.ppm + f * (fr.stride / 4);
        const uint32_t nrgb = fr.W * fr.H * 12 / 16, nppm = fr.W * fr.H * 3 / 16;  // 16-B words
        if (P == 0) {
            const uint32_t nw = gridDim.x * 4, w0 = blockIdx.x * 4 + wave;
            // (frames in turn: a launch's frames one after another, as the frame kernel's F frames)
            for (uint32_t b = w0; b < nblk; b += nw) {
                const uint32_t bx = b % tiles_x, by = b / tiles_x;
#pragma unroll
                for (uint32_t i = lane; i < 4 * 48; i += 64) {
                    const uint32_t r = i / 48, c = i % 48;
                    st16<kNt>(rgb, 12u * ((by * 4 + r) * fr.W + bx * 64) + 16u * c, pat(c % 3));
                }
                if (lane < 48) {
                    const uint32_t r = lane / 12, c = lane % 12;
                    st16<kNt>(ppm, 3u * ((fr.H - 4 - by * 4 + r) * fr.W + bx * 64) + 16u * c, pat(c % 3));
                }
            }
        } else if (P == 1) {
            const uint32_t stride = gridDim.x * 256, i0 = blockIdx.x * 256 + threadIdx.x;
            for (uint32_t i = i0; i < nrgb; i += stride) st16<kNt>(rgb, 16u * i, pat(i % 3));
            for (uint32_t i = i0; i < nppm; i += stride) st16<kNt>(ppm, 16u * i, pat(i % 3));
        } else if (P == 2) {
            const uint32_t cr = (nrgb + gridDim.x - 1) / gridDim.x, cp = (nppm + gridDim.x - 1) / gridDim.x;
            const uint32_t r0 = blockIdx.x * cr, r1 = min(r0 + cr, nrgb), p0 = blockIdx.x * cp, p1 = min(p0 + cp, nppm);
            for (uint32_t i = r0 + threadIdx.x; i < r1; i += 256) st16<kNt>(rgb, 16u * i, pat(i % 3));
            for (uint32_t i = p0 + threadIdx.x; i < p1; i += 256) st16<kNt>(ppm, 16u * i, pat(i % 3));
        } else {
            // rows: step s covers camera rows; RGB row y = W*12 B, PPM file row H-1-y = W*3 B
            const uint32_t wr = fr.W * 12 / 16, wp = fr.W * 3 / 16, per = wr + wp;  // words per row pair
            const uint32_t stride = gridDim.x * 256;
            for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < per * fr.H; i += stride) {
                const uint32_t y = i / per, k = i - y * per;
                if (k < wr)
                    st16<kNt>(rgb, 16u * (y * wr + k), pat(k % 3));
                else
                    st16<kNt>(ppm, 16u * ((fr.H - 1 - y) * wp + (k - wr)), pat((k - wr) % 3));
            }
        }
    }
}

int main() {
    struct Shape {
        uint32_t W, H, F, slots;
    };
    const Shape shapes[] = {{3840, 2160, 1, 4}, {1920, 1080, 8, 16}, {3840, 2160, 1, 1}};
    const int R = 32;
    hipEvent_t ev[2 * R];
    for (auto& e : ev) (void)hipEventCreate(&e);
    for (const Shape& sh : shapes) {
        const size_t frame = (size_t)sh.W * sh.H;
        float* rgb;
        uint8_t* ppm;
        (void)hipMalloc(&rgb, frame * 12 * sh.slots);
        (void)hipMalloc(&ppm, frame * 3 * sh.slots);
        const double bytes = (double)frame * 15 * sh.F;
        auto run = [&](const char* name, int g, auto k) {
            auto at = [&](int i) {
                const uint32_t s0 = (uint32_t)(i * sh.F) % sh.slots;
                return Frames{rgb + frame * 3 * s0, ppm + frame * 3 * s0, sh.W, sh.H, sh.F, frame * 12};
            };
            for (int i = 0; i < 4; ++i) k<<<g, 256>>>(at(i));
            for (int i = 0; i < R; ++i)
                (void)hipExtLaunchKernelGGL(k, dim3(g), dim3(256), 0, nullptr, ev[2 * i], ev[2 * i + 1], 0, at(i));
            (void)hipDeviceSynchronize();
            float sum = 0.0f, lo = 1e9f;
            for (int i = 0; i < R; ++i) {
                float ms;
                (void)hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]);
                sum += ms;
                lo = ms < lo ? ms : lo;
            }
            printf("%ux%u F%u slots %2u %-8s grid %4d: %8.2f us mean %8.2f min  %.2f TB/s\n", sh.W, sh.H, sh.F, sh.slots,
                   name, g, sum * 1e3 / R, lo * 1e3, bytes / (sum * 1e-3 / R) / 1e12);
            fflush(stdout);
        };
        for (int round = 0; round < 3; ++round)
            for (int g : {256, 512}) {
                run("blk", g, fill<0, false>);
                run("blknt", g, fill<0, true>);
                run("flat", g, fill<1, false>);
                run("flatnt", g, fill<1, true>);
                run("chunk", g, fill<2, false>);
                run("chunknt", g, fill<2, true>);
                run("rows", g, fill<3, false>);
                run("rowsnt", g, fill<3, true>);
            }
        (void)hipFree(rgb);
        (void)hipFree(ppm);
    }
    return 0;
}
