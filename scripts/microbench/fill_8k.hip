// Microbenchmark (diagnostic, not product): the background fill's write rate at 7680x4320 (C5's
// frame, 498 MB of f32 RGB + PPM: twice the 256 MB MALL) by store pattern and grid, per dispatch
// (hipExtLaunchKernelGGL start/stop events).  Patterns:
//   blk   render.hip's fill_blocks order: wave w takes 64x4 blocks w, w + nw, ... (4 rows x 768 B)
//   blk4  four horizontally consecutive blocks per wave per step (a 256x4 strip)
//   row   wave w takes whole 64-pixel row segments (1 row x 768 B, consecutive in the row)
//   flat  the RGB and PPM arrays as flat byte ranges, 16 B per lane, grid-stride (the ideal)
//   hipcc -O3 --offload-arch=gfx950 fill_8k.hip -o fill_8k && ./fill_8k
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

__device__ __forceinline__ void block(float* rgb, uint8_t* ppm, uint32_t W, uint32_t H, uint32_t bx, uint32_t by,
                                      uint32_t lane) {
#pragma unroll
    for (uint32_t i = lane; i < 4 * 48; i += 64) {  // 4 rows x 48 float4
        const uint32_t r = i / 48, c = i % 48;
        st16(rgb, 12ull * ((size_t)(by * 4 + r) * W + bx * 64) + 16ull * c, pat(c % 3));
    }
    if (lane < 48) {
        const uint32_t r = lane / 12, c = lane % 12;
        st16(ppm, 3ull * ((size_t)(H - 4 - by * 4 + r) * W + bx * 64) + 16ull * c, pat(c % 3));
    }
}

template <int P>
__global__ void __launch_bounds__(256) fill(float* rgb, uint8_t* ppm, uint32_t W, uint32_t H) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t tiles_x = W / 64, nblk = tiles_x * (H / 4);
    const uint32_t nw = gridDim.x * 4, w = blockIdx.x * 4 + wave;
    if (P == 0) {
        for (uint32_t b = w; b < nblk; b += nw) block(rgb, ppm, W, H, b % tiles_x, b / tiles_x, lane);
    } else if (P == 1) {
        for (uint32_t b = 4 * w; b < nblk; b += 4 * nw)
            for (uint32_t u = 0; u < 4 && b + u < nblk; ++u) block(rgb, ppm, W, H, (b + u) % tiles_x, (b + u) / tiles_x, lane);
    } else if (P == 2) {  // row segments: 64 px x 1 row = 768 B RGB (48 lanes) + 192 B PPM (12 lanes)
        const uint32_t nseg = tiles_x * H;
        for (uint32_t s = w; s < nseg; s += nw) {
            const uint32_t y = s / tiles_x, x = s % tiles_x;
            if (lane < 48) st16(rgb, 12ull * ((size_t)y * W + x * 64) + 16ull * lane, pat(lane % 3));
            else if (lane < 60) st16(ppm, 3ull * ((size_t)(H - 1 - y) * W + x * 64) + 16ull * (lane - 48), pat(lane % 3));
        }
    } else {  // flat
        const size_t n_rgb = (size_t)W * H * 12 / 16, n_ppm = (size_t)W * H * 3 / 16;
        const size_t stride = (size_t)gridDim.x * 256, i0 = (size_t)blockIdx.x * 256 + threadIdx.x;
        for (size_t i = i0; i < n_rgb; i += stride) st16(rgb, 16 * i, pat(i % 3));
        for (size_t i = i0; i < n_ppm; i += stride) st16(ppm, 16 * i, pat(i % 3));
    }
}

int main() {
    const uint32_t W = 7680, H = 4320;
    const size_t bytes = (size_t)W * H * 15;
    float* rgb;
    uint8_t* ppm;
    (void)hipMalloc(&rgb, (size_t)W * H * 12);
    (void)hipMalloc(&ppm, (size_t)W * H * 3);
    const int R = 24;
    hipEvent_t ev[2 * R];
    for (auto& e : ev) (void)hipEventCreate(&e);
    auto run = [&](const char* name, int g, auto k) {
        for (int i = 0; i < 4; ++i) k<<<g, 256>>>(rgb, ppm, W, H);
        for (int i = 0; i < R; ++i)
            (void)hipExtLaunchKernelGGL(k, dim3(g), dim3(256), 0, nullptr, ev[2 * i], ev[2 * i + 1], 0, rgb, ppm, W, H);
        (void)hipDeviceSynchronize();
        float sum = 0.0f, lo = 1e9f;
        for (int i = 0; i < R; ++i) {
            float ms;
            (void)hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]);
            sum += ms;
            lo = ms < lo ? ms : lo;
        }
        printf("7680x4320 %-4s grid %5d: %7.2f us mean %7.2f min  %.2f TB/s\n", name, g, sum * 1e3 / R, lo * 1e3,
               bytes / (sum * 1e-3 / R) / 1e12);
        fflush(stdout);
    };
    for (int g : {256, 512, 768, 1024, 2048, 4096}) {
        run("blk", g, fill<0>);
        run("blk4", g, fill<1>);
        run("row", g, fill<2>);
        run("flat", g, fill<3>);
    }
    return 0;
}
