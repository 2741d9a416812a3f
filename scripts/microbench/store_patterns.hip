// Microbenchmark (diagnostic, not product): write a 1920x1080 f32-RGB + PPM-byte frame
// (31.1 MB) with different per-wave store patterns and time each with HIP events.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int W = 1920, H = 1080;

// (a) lane owns 4 adjacent pixels: 3 x 16 B at a 48-byte lane stride (current cull_fill)
__global__ void fill_lane48(float* rgb, uint8_t* ppm) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;  // one lane per 4 pixels
  if (t >= W * H / 4) return;
  float4* o = reinterpret_cast<float4*>(rgb) + 3 * t;
  o[0] = make_float4(.1f, .1f, .2f, .1f); o[1] = make_float4(.1f, .2f, .1f, .1f); o[2] = make_float4(.2f, .1f, .1f, .2f);
  uint32_t* q = reinterpret_cast<uint32_t*>(ppm) + 3 * t;
  q[0] = 0x19331919u; q[1] = 0x19193319u; q[2] = 0x33191933u;
}
// (b) contiguous: consecutive lanes write consecutive 16-byte words (1 KB per wave instruction)
__global__ void fill_contig(float* rgb, uint8_t* ppm) {
  const int nrgb = W * H * 3 / 4, nppm = W * H * 3 / 16;
  int stride = gridDim.x * blockDim.x;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nrgb; i += stride) {
    int ph = i % 3;
    reinterpret_cast<float4*>(rgb)[i] = ph == 0 ? make_float4(.1f,.1f,.2f,.1f) : ph == 1 ? make_float4(.1f,.2f,.1f,.1f) : make_float4(.2f,.1f,.1f,.2f);
  }
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nppm; i += stride)
    reinterpret_cast<uint4*>(ppm)[i] = make_uint4(0x19331919u, 0x19193319u, 0x33191933u, 0x19331919u);
}
// (c) contiguous, one pass per block of 3 instructions: lane l of wave w writes words w*192 + j*64 + l
__global__ void fill_wave3(float* rgb, uint8_t* ppm) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  const int base = wave * 192;  // float4 words of 256 pixels
  if (base >= W * H * 3 / 4) return;
  for (int j = 0; j < 3; ++j) {
    int i = base + j * 64 + lane; int ph = i % 3;
    reinterpret_cast<float4*>(rgb)[i] = ph == 0 ? make_float4(.1f,.1f,.2f,.1f) : ph == 1 ? make_float4(.1f,.2f,.1f,.1f) : make_float4(.2f,.1f,.1f,.2f);
  }
  if (lane < 48) reinterpret_cast<uint4*>(ppm)[wave * 48 + lane] = make_uint4(0x19331919u, 0x19193319u, 0x33191933u, 0x19331919u);
}
// (d) rgb only contiguous (no ppm) to see the f32 part alone
__global__ void fill_rgb_only(float* rgb) {
  const int nrgb = W * H * 3 / 4; int stride = gridDim.x * blockDim.x;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nrgb; i += stride)
    reinterpret_cast<float4*>(rgb)[i] = make_float4(.1f,.1f,.2f,.1f);
}

int main() {
  float* rgb; uint8_t* ppm;
  hipMalloc(&rgb, (size_t)W * H * 12); hipMalloc(&ppm, (size_t)W * H * 3);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  auto time = [&](const char* name, auto launch) {
    for (int i = 0; i < 20; ++i) launch();
    hipDeviceSynchronize();
    float best = 1e9, sum = 0; const int R = 100;
    for (int i = 0; i < R; ++i) { hipEventRecord(a); launch(); hipEventRecord(b); hipEventSynchronize(b); float ms; hipEventElapsedTime(&ms, a, b); best = ms < best ? ms : best; sum += ms; }
    double bytes = (double)W * H * 15;
    printf("%-14s mean %.2f us  best %.2f us  -> %.2f TB/s (best)\n", name, sum / R * 1e3, best * 1e3, bytes / (best * 1e-3) / 1e12);
  };
  const int n4 = W * H / 4;
  time("lane48", [&] { fill_lane48<<<(n4 + 255) / 256, 256>>>(rgb, ppm); });
  time("contig_2048", [&] { fill_contig<<<2048, 256>>>(rgb, ppm); });
  time("contig_8192", [&] { fill_contig<<<8192, 256>>>(rgb, ppm); });
  time("wave3", [&] { fill_wave3<<<(n4 + 255) / 256, 256>>>(rgb, ppm); });
  time("rgb_only", [&] { fill_rgb_only<<<4096, 256>>>(rgb); });
  hipFree(rgb); hipFree(ppm);
  return 0;
}
