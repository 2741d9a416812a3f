// Microbenchmark (diagnostic, not product): the background fill's store patterns with and without
// the frame kernel's per-unit pacing (render.hip fill_blocks: s_waitcnt vmcnt(0) before each
// unit's stores), one workgroup per CU, on C2's ring (1920x1080, 8 frames into 8 slots) and
// 3840x2160 in 1 and 4 slots.  Patterns (fill_pat.hip): blk (64x4 blocks), strip (a wave's 256x4
// strip, row by row: 3 contiguous 1-KB RGB stores + 768 B PPM), band (a workgroup's 4-row band,
// wave r its row r).
//   hipcc -O3 --offload-arch=gfx950 fill_pace.hip -o fill_pace && ./fill_pace
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <cstdio>

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st16(void* base, uint32_t off, uint4 v) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, -1, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{v.x, v.y, v.z, v.w}, r, off, 0, 16);
}
__device__ __forceinline__ uint4 pat(uint32_t ph) {
    const uint32_t a = 0x3dcccccdu, b = 0x3e4ccccdu;
    return ph == 0 ? make_uint4(a, a, b, a) : ph == 1 ? make_uint4(a, b, a, a) : make_uint4(b, a, a, b);
}
struct Frames {
    float* rgb;
    uint8_t* ppm;
    uint32_t W, H, F;
};
__device__ __forceinline__ void block(const Frames& fr, uint32_t f, uint32_t bx, uint32_t by, uint32_t lane) {
    float* rgb = fr.rgb + (size_t)f * fr.W * fr.H * 3;
    uint8_t* ppm = fr.ppm + (size_t)f * fr.W * fr.H * 3;
#pragma unroll
    for (uint32_t i = lane; i < 4 * 48; i += 64) {
        const uint32_t r = i / 48, c = i % 48;
        st16(rgb, 12u * ((by * 4 + r) * fr.W + bx * 64) + 16u * c, pat(c % 3));
    }
    if (lane < 48) {
        const uint32_t r = lane / 12, c = lane % 12;
        st16(ppm, 3u * ((fr.H - 4 - by * 4 + r) * fr.W + bx * 64) + 16u * c, pat(c % 3));
    }
}
__device__ __forceinline__ void strip_row(const Frames& fr, uint32_t f, uint32_t bx, uint32_t by, uint32_t r, uint32_t lane) {
    float* rgb = fr.rgb + (size_t)f * fr.W * fr.H * 3;
    uint8_t* ppm = fr.ppm + (size_t)f * fr.W * fr.H * 3;
    const uint32_t row = 12u * ((by * 4 + r) * fr.W + bx * 64);
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) st16(rgb, row + 16u * (64 * k + lane), pat((64 * k + lane) % 3));
    if (lane < 48) st16(ppm, 3u * ((fr.H - 4 - by * 4 + r) * fr.W + bx * 64) + 16u * lane, pat(lane % 3));
}
constexpr int kPace = 0x0f70;  // s_waitcnt vmcnt(0)

template <int P, bool kPaced>
__global__ void __launch_bounds__(256) fill(Frames fr) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t tiles_x = fr.W / 64, bands = fr.H / 4, nblk = tiles_x * bands;
    const uint32_t nw = gridDim.x * 4, w = blockIdx.x * 4 + wave;
    if (P == 0) {
        for (uint32_t b = w; b < nblk * fr.F; b += nw) {
            if (kPaced) __builtin_amdgcn_s_waitcnt(kPace);
            const uint32_t f = b / nblk, k = b % nblk;
            block(fr, f, k % tiles_x, k / tiles_x, lane);
        }
    } else if (P == 1) {
        const uint32_t sx = tiles_x / 4, nstrip = sx * bands;
        for (uint32_t s = w; s < nstrip * fr.F; s += nw) {
            const uint32_t f = s / nstrip, k = s % nstrip;
            for (uint32_t r = 0; r < 4; ++r) {
                if (kPaced) __builtin_amdgcn_s_waitcnt(kPace);
                strip_row(fr, f, (k % sx) * 4, k / sx, r, lane);
            }
        }
    } else {
        const uint32_t sx = tiles_x / 4;
        for (uint32_t b = blockIdx.x; b < bands * fr.F; b += gridDim.x) {
            const uint32_t f = b / bands, by = b % bands;
            for (uint32_t s = 0; s < sx; ++s) {
                if (kPaced) __builtin_amdgcn_s_waitcnt(kPace);
                strip_row(fr, f, s * 4, by, wave, lane);
            }
        }
    }
}

int main() {
    struct Shape {
        uint32_t W, H, F, slots;
    };
    const Shape shapes[] = {{1920, 1080, 8, 8}, {3840, 2160, 1, 1}, {3840, 2160, 1, 4}};
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
            auto at = [&](int i) {
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
            printf("%ux%u F%u slots %u %-10s grid %4d: %8.2f us mean %8.2f min  %.2f TB/s\n", sh.W, sh.H, sh.F, sh.slots,
                   name, g, sum * 1e3 / R, lo * 1e3, bytes / (sum * 1e-3 / R) / 1e12);
            fflush(stdout);
        };
        for (int g : {256, 512}) {
            run("blk", g, fill<0, false>);
            run("blk-paced", g, fill<0, true>);
            run("strip", g, fill<1, false>);
            run("strip-pace", g, fill<1, true>);
            run("band", g, fill<2, false>);
            run("band-paced", g, fill<2, true>);
        }
        (void)hipFree(rgb);
        (void)hipFree(ppm);
    }
    return 0;
}
