// Microbenchmark (diagnostic, not product): the background fill's store pattern, per dispatch
// (hipExtLaunchKernelGGL start / stop events), on the bench's frame shapes — C2's ring (1920x1080,
// 8 frames per launch into 8 slots), 3840x2160 in 1 and 4 slots (one frame per launch), 7680x4320.
// f32 RGB (12 B/px) + PPM (3 B/px, rows bottom-up) with 16-B sc1 buffer stores, as render.hip.
//   blk    render.hip's fill_blocks: wave w takes 64x4 blocks w, w + nw, ... (4 rows x 768 B)
//   strip  a wave takes a 256x4 strip (4 blocks): each row's 3 KB of RGB in 3 contiguous 1-KB
//          stores, its 768 B of PPM in one
//   band   a workgroup takes a 4-row band of blocks, wave r its row r, left to right in 256-px
//          steps (the same 3 KB + 768 B stores); workgroups stride over the bands
//   flat   the RGB then the PPM array as flat byte ranges, 16 B per lane, grid-stride
//   blkup  blk with the PPM rows top-down (the RGB rows' direction) instead of the file's bottom-up
//   blk2   blk in two passes: every block's RGB, then every block's PPM
//   flatil flat with each step's RGB and PPM chunks together (4 RGB chunks per PPM chunk)
//   hipcc -O3 --offload-arch=gfx950 fill_pat.hip -o fill_pat && ./fill_pat
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <cstdio>

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st16(void* base, size_t off, uint4 v) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, -1, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{v.x, v.y, v.z, v.w}, r, (uint32_t)off, 0, 16);
}
__device__ __forceinline__ uint4 pat(uint32_t ph) {
    const uint32_t a = 0x3dcccccdu, b = 0x3e4ccccdu;
    return ph == 0 ? make_uint4(a, a, b, a) : ph == 1 ? make_uint4(a, b, a, a) : make_uint4(b, a, a, b);
}

struct Frames {
    float* rgb;  // frame f at rgb + f * W * H * 3
    uint8_t* ppm;
    uint32_t W, H, F;
};

// 64 x 4 block (bx, by) of frame f (parts: 1 RGB, 2 PPM; up: PPM rows top-down)
__device__ __forceinline__ void block(const Frames& fr, uint32_t f, uint32_t bx, uint32_t by, uint32_t lane,
                                      uint32_t parts = 3, bool up = false) {
    float* rgb = fr.rgb + (size_t)f * fr.W * fr.H * 3;
    uint8_t* ppm = fr.ppm + (size_t)f * fr.W * fr.H * 3;
    if (parts & 1) {
#pragma unroll
        for (uint32_t i = lane; i < 4 * 48; i += 64) {
            const uint32_t r = i / 48, c = i % 48;
            st16(rgb, 12ull * ((size_t)(by * 4 + r) * fr.W + bx * 64) + 16ull * c, pat(c % 3));
        }
    }
    if ((parts & 2) && lane < 48) {
        const uint32_t r = lane / 12, c = lane % 12;
        const size_t row = up ? by * 4 + r : fr.H - 4 - by * 4 + r;
        st16(ppm, 3ull * (row * fr.W + bx * 64) + 16ull * c, pat(c % 3));
    }
}
// row r (0..3) of the 256 x 4 strip at block (bx, by): 3 KB RGB + 768 B PPM
__device__ __forceinline__ void strip_row(const Frames& fr, uint32_t f, uint32_t bx, uint32_t by, uint32_t r, uint32_t lane) {
    float* rgb = fr.rgb + (size_t)f * fr.W * fr.H * 3;
    uint8_t* ppm = fr.ppm + (size_t)f * fr.W * fr.H * 3;
    const size_t row = 12ull * ((size_t)(by * 4 + r) * fr.W + bx * 64);
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) st16(rgb, row + 16ull * (64 * k + lane), pat((64 * k + lane) % 3));
    if (lane < 48) st16(ppm, 3ull * ((size_t)(fr.H - 4 - by * 4 + r) * fr.W + bx * 64) + 16ull * lane, pat(lane % 3));
}

template <int P>
__global__ void __launch_bounds__(256) fill(Frames fr) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t tiles_x = fr.W / 64, bands = fr.H / 4, nblk = tiles_x * bands;
    const uint32_t nw = gridDim.x * 4, w = blockIdx.x * 4 + wave;
    if (P == 0) {
        for (uint32_t b = w; b < nblk * fr.F; b += nw) {
            const uint32_t f = b / nblk, k = b % nblk;
            block(fr, f, k % tiles_x, k / tiles_x, lane);
        }
    } else if (P == 1) {
        const uint32_t sx = tiles_x / 4, nstrip = sx * bands;
        for (uint32_t s = w; s < nstrip * fr.F; s += nw) {
            const uint32_t f = s / nstrip, k = s % nstrip;
            for (uint32_t r = 0; r < 4; ++r) strip_row(fr, f, (k % sx) * 4, k / sx, r, lane);
        }
    } else if (P == 2) {
        const uint32_t sx = tiles_x / 4;
        for (uint32_t b = blockIdx.x; b < bands * fr.F; b += gridDim.x) {
            const uint32_t f = b / bands, by = b % bands;
            for (uint32_t s = 0; s < sx; ++s) strip_row(fr, f, s * 4, by, wave, lane);
        }
    } else if (P == 3) {
        const size_t n = (size_t)fr.W * fr.H * 12 / 16 * fr.F, m = (size_t)fr.W * fr.H * 3 / 16 * fr.F;
        const size_t stride = (size_t)gridDim.x * 256, i0 = (size_t)blockIdx.x * 256 + threadIdx.x;
        for (size_t i = i0; i < n; i += stride) st16(fr.rgb, 16 * i, pat(i % 3));
        for (size_t i = i0; i < m; i += stride) st16(fr.ppm, 16 * i, pat(i % 3));
    } else if (P == 4) {
        for (uint32_t b = w; b < nblk * fr.F; b += nw) {
            const uint32_t f = b / nblk, k = b % nblk;
            block(fr, f, k % tiles_x, k / tiles_x, lane, 3, true);
        }
    } else if (P == 5) {
        for (uint32_t part = 1; part <= 2; ++part)
            for (uint32_t b = w; b < nblk * fr.F; b += nw) {
                const uint32_t f = b / nblk, k = b % nblk;
                block(fr, f, k % tiles_x, k / tiles_x, lane, part);
            }
    } else {
        const size_t m = (size_t)fr.W * fr.H * 3 / 16 * fr.F;  // PPM chunks; RGB = 4 m
        const size_t stride = (size_t)gridDim.x * 256, i0 = (size_t)blockIdx.x * 256 + threadIdx.x;
        for (size_t i = i0; i < m; i += stride) {
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) st16(fr.rgb, 16 * (4 * (i - threadIdx.x) + k * 256 + threadIdx.x), pat(k % 3));
            st16(fr.ppm, 16 * i, pat(i % 3));
        }
    }
}

int main() {
    struct Shape {
        uint32_t W, H, F, slots;
    };
    const Shape shapes[] = {{1920, 1080, 8, 8}, {3840, 2160, 1, 1}, {3840, 2160, 1, 4}, {7680, 4320, 1, 1}};
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
        auto run = [&](const char* name, int g, auto k) {
            auto at = [&](int i) {  // launch i's frames: slots (i * F) % slots ..
                const uint32_t s0 = (uint32_t)(i * sh.F) % sh.slots;
                return Frames{rgb + frame * 3 * s0, ppm + frame * 3 * s0, sh.W, sh.H, sh.F};
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
            printf("%ux%u F%u slots %u %-5s grid %5d: %8.2f us mean %8.2f min  %.2f TB/s\n", sh.W, sh.H, sh.F, sh.slots,
                   name, g, sum * 1e3 / R, lo * 1e3, bytes / (sum * 1e-3 / R) / 1e12);
            fflush(stdout);
        };
        for (int g : {256, 512}) {
            run("blk", g, fill<0>);
            run("flat", g, fill<3>);
            run("blkup", g, fill<4>);
            run("blk2", g, fill<5>);
            run("flatil", g, fill<6>);
        }
        (void)hipFree(rgb);
        (void)hipFree(ppm);
    }
    return 0;
}
