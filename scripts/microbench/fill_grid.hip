// Microbenchmark (diagnostic, not product): does the frame kernel's launch shape slow its fill?
// The background fill's 64x4-block store pattern (fill_pat.hip `blk`: wave w takes blocks
// w, w + nw, ...; f32 RGB + PPM rows, 16-B sc1 buffer stores) written by g workgroups, launched as
//   exact  a grid of exactly g workgroups
//   first  a grid of 3g workgroups of which the first g write and the rest return at once
//          (frame_kernel: 768 resident workgroups, the fill roles the first dispatched)
//   third  a grid of 3g workgroups of which every third writes
//   fast   exact, with the per-lane store offsets and words hoisted out of the block loop and the
//          block base as the stores' scalar offset (render.hip fill_block_fast)
//   slow   fast with an s_sleep 1 after each block (fewer stores in flight per wave)
// on 3840x2160 frames in 1 and 4 ring slots (one frame per launch) and C2's 8 frames into 8 slots.
//   hipcc -O3 --offload-arch=gfx950 fill_grid.hip -o fill_grid && ./fill_grid
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <cstdio>

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st16(void* base, uint32_t voff, uint32_t soff, uint4 v) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, -1, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{v.x, v.y, v.z, v.w}, r, voff, soff, 16);
}
__device__ __forceinline__ uint4 pat(uint32_t ph) {
    const uint32_t a = 0x3dcccccdu, b = 0x3e4ccccdu;
    return ph == 0 ? make_uint4(a, a, b, a) : ph == 1 ? make_uint4(a, b, a, a) : make_uint4(b, a, a, b);
}

struct Frames {
    float* rgb;  // frame f at rgb + f * W * H * 3
    uint8_t* ppm;
    uint32_t W, H, F, g;
};

// mode 0 exact, 1 first, 2 third, 3 fast, 4 slow
template <int M>
__global__ void __launch_bounds__(256) fill(Frames fr) {
    uint32_t wg = blockIdx.x;
    if (M == 1) {
        if (wg >= fr.g) return;
    } else if (M == 2) {
        if (wg % 3) return;
        wg /= 3;
    }
    const uint32_t lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t tiles_x = fr.W / 64, bands = fr.H / 4, nblk = tiles_x * bands;
    const uint32_t nw = fr.g * 4, w = wg * 4 + wave;
    uint32_t roff[3], poff = 0;
    uint4 rv[3], pv = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) {
        const uint32_t i = lane + 64 * k, r = i / 48, c = i % 48;
        roff[k] = r * fr.W * 12 + c * 16;
        rv[k] = pat(c % 3);
    }
    {
        const uint32_t r = lane / 12, c = lane % 12;
        poff = r * fr.W * 3 + c * 16;
        pv = pat(c % 3);
    }
    for (uint32_t b = w; b < nblk * fr.F; b += nw) {
        const uint32_t f = b / nblk, k = b % nblk, bx = k % tiles_x, by = k / tiles_x;
        float* rgb = fr.rgb + (size_t)f * fr.W * fr.H * 3;
        uint8_t* ppm = fr.ppm + (size_t)f * fr.W * fr.H * 3;
        if (M >= 3) {
            const uint32_t base = (by * 4 * fr.W + bx * 64) * 12;
#pragma unroll
            for (uint32_t q = 0; q < 3; ++q) st16(rgb, roff[q], base, rv[q]);
            if (lane < 48) st16(ppm, poff, ((fr.H - 4 - by * 4) * fr.W + bx * 64) * 3, pv);
            if (M == 4) __builtin_amdgcn_s_sleep(1);
        } else {
#pragma unroll
            for (uint32_t i = lane; i < 4 * 48; i += 64) {
                const uint32_t r = i / 48, c = i % 48;
                st16(rgb, 12u * ((by * 4 + r) * fr.W + bx * 64) + 16u * c, 0, pat(c % 3));
            }
            if (lane < 48) {
                const uint32_t r = lane / 12, c = lane % 12;
                st16(ppm, 3u * ((fr.H - 4 - by * 4 + r) * fr.W + bx * 64) + 16u * c, 0, pat(c % 3));
            }
        }
    }
}

int main() {
    struct Shape {
        uint32_t W, H, F, slots;
    };
    const Shape shapes[] = {{3840, 2160, 1, 1}, {3840, 2160, 1, 4}, {1920, 1080, 8, 8}};
    const int R = 24;
    hipEvent_t ev[2 * R];
    for (auto& e : ev) (void)hipEventCreate(&e);
    for (const Shape& sh : shapes) {
        const size_t frame = (size_t)sh.W * sh.H;
        float* rgb;
        uint8_t* ppm;
        (void)hipMalloc(&rgb, frame * 12 * sh.slots);
        (void)hipMalloc(&ppm, frame * 3 * sh.slots);
        const double bytes = (double)frame * 15 * sh.F;
        for (uint32_t g : {256u, 384u, 512u}) {
            auto run = [&](const char* name, int grid, auto k) {
                auto at = [&](int i) {
                    const uint32_t s0 = (uint32_t)(i * sh.F) % sh.slots;
                    return Frames{rgb + frame * 3 * s0, ppm + frame * 3 * s0, sh.W, sh.H, sh.F, g};
                };
                for (int i = 0; i < 4; ++i) k<<<grid, 256>>>(at(i));
                for (int i = 0; i < R; ++i)
                    (void)hipExtLaunchKernelGGL(k, dim3(grid), dim3(256), 0, nullptr, ev[2 * i], ev[2 * i + 1], 0, at(i));
                (void)hipDeviceSynchronize();
                float sum = 0.0f, lo = 1e9f;
                for (int i = 0; i < R; ++i) {
                    float ms;
                    (void)hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]);
                    sum += ms;
                    lo = ms < lo ? ms : lo;
                }
                printf("%ux%u F%u slots %u %-5s g %4u grid %5d: %8.2f us mean %8.2f min  %.2f TB/s\n", sh.W, sh.H, sh.F,
                       sh.slots, name, g, grid, sum * 1e3 / R, lo * 1e3, bytes / (sum * 1e-3 / R) / 1e12);
                fflush(stdout);
            };
            run("exact", g, fill<0>);
            run("first", 3 * g, fill<1>);
            run("third", 3 * g, fill<2>);
            run("fast", g, fill<3>);
            run("slow", g, fill<4>);
        }
        (void)hipFree(rgb);
        (void)hipFree(ppm);
    }
    return 0;
}
