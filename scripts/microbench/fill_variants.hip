// Microbenchmark (diagnostic, not product): how the 31.1 MB frame fill behaves under different
// work decompositions.  Each variant writes f32 RGB (12 B/px) + PPM bytes (3 B/px) of 1920x1080.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int W = 1920, H = 1080;
__device__ __forceinline__ float4 pat(int ph) {
  return ph == 0 ? make_float4(.1f, .1f, .2f, .1f) : ph == 1 ? make_float4(.1f, .2f, .1f, .1f) : make_float4(.2f, .1f, .1f, .2f);
}
__device__ __forceinline__ uint4 patb(int ph) {
  const uint32_t a = 0x19331919u, b = 0x19193319u, c = 0x33191933u;
  return ph == 0 ? make_uint4(a, b, c, a) : ph == 1 ? make_uint4(b, c, a, b) : make_uint4(c, a, b, c);
}
// sub-block of SW x 4 px per wave; rows of SW*12 B rgb / SW*3 B ppm
template <int SW>
__device__ __forceinline__ void store_sub(float* rgb, uint8_t* ppm, int x0, int y0, int lane) {
  constexpr int R4 = SW * 3 / 4, P16 = SW * 3 / 16;
  for (int i = lane; i < 4 * R4; i += 64) {
    int r = i / R4, c = i % R4;
    reinterpret_cast<float4*>(rgb + 3 * ((size_t)(y0 + r) * W + x0))[c] = pat(c % 3);
  }
  for (int i = lane; i < 4 * P16; i += 64) {
    int r = i / P16, c = i % P16;
    reinterpret_cast<uint4*>(ppm + 3 * ((size_t)(H - 1 - y0 - 3 + r) * W + x0))[c] = patb(c % 3);
  }
}
// (A) one wave per SW x 4 sub-block, non-persistent
template <int SW>
__global__ void __launch_bounds__(256) fill_sub(float* rgb, uint8_t* ppm) {
  int wave = (blockIdx.x * 256 + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  const int sx = W / SW;
  if (wave >= sx * (H / 4)) return;
  store_sub<SW>(rgb, ppm, (wave % sx) * SW, (wave / sx) * 4, lane);
}
// (B) persistent: `grid` workgroups stride over SW x 4 sub-blocks
template <int SW>
__global__ void __launch_bounds__(256) fill_sub_persist(float* rgb, uint8_t* ppm) {
  int lane = threadIdx.x & 63;
  const int sx = W / SW, n = sx * (H / 4);
  for (int s = blockIdx.x * 4 + (threadIdx.x >> 6); s < n; s += gridDim.x * 4)
    store_sub<SW>(rgb, ppm, (s % sx) * SW, (s / sx) * 4, lane);
}
// (C) like B but VGPR-heavy (forces low occupancy): dummy register pressure via launch bounds
template <int SW>
__global__ void __launch_bounds__(256, 1) fill_sub_persist_lowocc(float* rgb, uint8_t* ppm, int pad) {
  __shared__ float big[40000];  // ~156 KB LDS: 1 workgroup per CU
  if (pad) big[threadIdx.x] = 1;
  int lane = threadIdx.x & 63;
  const int sx = W / SW, n = sx * (H / 4);
  for (int s = blockIdx.x * 4 + (threadIdx.x >> 6); s < n; s += gridDim.x * 4)
    store_sub<SW>(rgb, ppm, (s % sx) * SW, (s / sx) * 4, lane);
  if (pad) rgb[0] = big[threadIdx.x + 1];
}

int main() {
  float* rgb; uint8_t* ppm;
  (void)hipMalloc(&rgb, (size_t)W * H * 12); (void)hipMalloc(&ppm, (size_t)W * H * 3);
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  auto time = [&](const char* name, auto launch) {
    for (int i = 0; i < 20; ++i) launch();
    (void)hipDeviceSynchronize();
    float best = 1e9, sum = 0; const int R = 100;
    for (int i = 0; i < R; ++i) { (void)hipEventRecord(a); launch(); (void)hipEventRecord(b); (void)hipEventSynchronize(b); float ms; (void)hipEventElapsedTime(&ms, a, b); best = ms < best ? ms : best; sum += ms; }
    printf("%-34s mean %6.2f us  best %6.2f us  (%.2f TB/s)\n", name, sum / R * 1e3, best * 1e3, (double)W * H * 15 / (best * 1e-3) / 1e12);
  };
  const int n16 = (W / 16) * (H / 4), n64 = (W / 64) * (H / 4);
  time("sub16 one wave each", [&] { fill_sub<16><<<(n16 + 3) / 4, 256>>>(rgb, ppm); });
  time("sub64 one wave each", [&] { fill_sub<64><<<(n64 + 3) / 4, 256>>>(rgb, ppm); });
  for (int g : {256, 512, 768, 1024, 2048}) {
    char name[64]; snprintf(name, 64, "sub16 persistent grid %d", g);
    time(name, [&] { fill_sub_persist<16><<<g, 256>>>(rgb, ppm); });
    snprintf(name, 64, "sub64 persistent grid %d", g);
    time(name, [&] { fill_sub_persist<64><<<g, 256>>>(rgb, ppm); });
  }
  time("sub64 persistent 1 WG/CU (256)", [&] { fill_sub_persist_lowocc<64><<<256, 256>>>(rgb, ppm, 0); });
  time("sub16 persistent 1 WG/CU (256)", [&] { fill_sub_persist_lowocc<16><<<256, 256>>>(rgb, ppm, 0); });
  return 0;
}
