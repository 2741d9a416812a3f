// Diagnostics build of render.hip (not the product): every frame_kernel workgroup records
// s_memrealtime (100 MHz) at its start (0), the end of its detail work (1), and the start (2) and
// end (3) of its background fill, and wave 0 the phases of its latest sub-block; eray_debug_read_trace copies the records of the last frame out.
// Built by scripts/build_trace.sh into eray_amd/lib/liberay_hip_trace.so (ERAY_LIB selects it).
#include <hip/hip_runtime.h>
#include <cstdint>

__device__ unsigned long long g_eray_trace[8192 * 16];

#define ERAY_TRACE_POINT(k)                                                                   \
    do {                                                                                      \
        __syncthreads();                                                                      \
        if (threadIdx.x == 0 && blockIdx.x < 8192)                                            \
            g_eray_trace[blockIdx.x * 16 + (k)] = __builtin_amdgcn_s_memrealtime();            \
    } while (0)

// wave 0's phases of its latest sub-block: start (4), first hits known (5), shaded (6), outputs
// stored (7); inside: bin range + rays (8), first barrier (9), chunks done (10), last barrier (11),
// winner re-tested (12), hit records + texel addresses (13), shadow rays (14)
#define ERAY_TRACE_WAVE0(k)                                                                   \
    do {                                                                                      \
        if (threadIdx.x == 0 && blockIdx.x < 8192)                                            \
            g_eray_trace[blockIdx.x * 16 + (k)] = __builtin_amdgcn_s_memrealtime();            \
    } while (0)

#include "../../eray_amd/csrc/render.hip"

extern "C" int eray_debug_read_trace(unsigned long long* out, size_t n) {
    if (n > 8192 * 16) n = 8192 * 16;
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_eray_trace), n * sizeof(unsigned long long), 0,
                                    hipMemcpyDeviceToHost);
}
extern "C" int eray_debug_clear_trace() {
    static unsigned long long zero[8192 * 16];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_eray_trace), zero, sizeof(zero), 0, hipMemcpyHostToDevice);
}
