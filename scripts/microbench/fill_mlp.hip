// Microbenchmark (diagnostic, not product): how many waves the background fill needs to reach the
// HBM write rate, and whether unrolling more 64x4 blocks per loop iteration (more stores in flight
// per wave) lets fewer waves do it.  Writes f32 RGB (12 B/px) + PPM (3 B/px) of a W x H frame with
// 16-B sc1 buffer stores as render.hip's fill does; `slots` frames round-robin (1: the same
// buffer every launch, MALL-resident for small frames; 8: a ring far larger than the 256 MB MALL).
//   hipcc -O3 --offload-arch=gfx950 fill_mlp.hip -o fill_mlp && ./fill_mlp
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

template <int U>
__global__ void __launch_bounds__(256) fill(float* rgb, uint8_t* ppm, uint32_t W, uint32_t H) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t tiles_x = W / 64, nblk = tiles_x * (H / 4);
    const uint32_t nw = gridDim.x * 4, w = blockIdx.x * 4 + wave;
    for (uint32_t b0 = w * U; b0 < nblk; b0 += nw * U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t blk = b0 + u;
            if (blk >= nblk) break;
            const uint32_t by = blk / tiles_x, bx = blk - by * tiles_x;
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
    }
}

int main() {
    for (int sz = 0; sz < 2; ++sz) {
        const uint32_t W = sz ? 3840 : 1920, H = sz ? 2160 : 1080;
        const size_t bytes = (size_t)W * H * 15;
        for (int slots : {1, 8}) {
            float* rgb;
            uint8_t* ppm;
            (void)hipMalloc(&rgb, (size_t)W * H * 12 * slots);
            (void)hipMalloc(&ppm, (size_t)W * H * 3 * slots);
            hipEvent_t a, b;
            (void)hipEventCreate(&a);
            (void)hipEventCreate(&b);
            auto run = [&](const char* name, int g, auto k) {
                const int R = 64;
                for (int i = 0; i < 16; ++i)
                    k<<<g, 256>>>(rgb + (size_t)W * H * 3 * (i % slots), ppm + (size_t)W * H * 3 * (i % slots), W, H);
                (void)hipEventRecord(a);
                for (int i = 0; i < R; ++i)
                    k<<<g, 256>>>(rgb + (size_t)W * H * 3 * (i % slots), ppm + (size_t)W * H * 3 * (i % slots), W, H);
                (void)hipEventRecord(b);
                (void)hipEventSynchronize(b);
                float ms;
                (void)hipEventElapsedTime(&ms, a, b);
                printf("%ux%u slots %d %-4s grid %5d: %7.2f us/frame  %.2f TB/s\n", W, H, slots, name, g, ms * 1e3 / R,
                       bytes / (ms * 1e-3 / R) / 1e12);
            };
            for (int g : {128, 256, 384, 512, 768, 1024, 2048}) {
                run("U1", g, fill<1>);
                run("U2", g, fill<2>);
                run("U4", g, fill<4>);
            }
            (void)hipFree(rgb);
            (void)hipFree(ppm);
        }
    }
    return 0;
}
