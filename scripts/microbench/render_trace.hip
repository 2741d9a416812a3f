// Diagnostics build of render.hip (not the product): every frame_kernel workgroup records
// s_memrealtime (100 MHz) at its start (0), the end of its detail work (1), and the start (2) and
// end (3) of its background fill; wave 0 records the phases of its first sub-block (slots
// 32 + k) and of its latest one (slots k); eray_debug_read_trace copies the records of the last
// frame out.
// Built by scripts/build_trace.sh into eray_amd/lib/liberay_hip_trace.so (ERAY_LIB selects it).
#include <hip/hip_runtime.h>
#include <cstdint>

constexpr int kTraceSlots = 64;
__device__ unsigned long long g_eray_trace[8192 * kTraceSlots];
// wave 0's phase k already recorded once by this workgroup (first sub-block: slot 32 + k)
__shared__ unsigned int eray_trace_seen[32];

#define ERAY_TRACE_POINT(k)                                                                   \
    do {                                                                                      \
        if ((k) == 0 && threadIdx.x < 32) eray_trace_seen[threadIdx.x] = 0u;                  \
        __syncthreads();                                                                      \
        if (threadIdx.x == 0 && blockIdx.x < 8192)                                            \
            g_eray_trace[blockIdx.x * kTraceSlots + (k)] = __builtin_amdgcn_s_memrealtime();   \
    } while (0)

// wave 0's phases of a sub-block: start (4), first hits known (5), shaded (6), outputs stored
// (7); the per-wave bin search: rays + bbox with the first chunk load in flight (8), first chunk
// entries in registers (9), chunks done (10); hit records + texel addresses (13), shadow rays
// (14); value 15: the bin's chunks; the first role's list entry + camera rays (11), its binned
// object found (12); the first object's ObjGeom (16), the hit object's MaterialDesc (17); in the
// shadow loop: a light's descriptor read (18), an object's ObjGeom read (19); values: 1 + the object
// whose shadow scan the point-box test skipped (20) or ran (21)
#define ERAY_TRACE_RECORD(k, v)                                                               \
    do {                                                                                      \
        if (threadIdx.x == 0 && blockIdx.x < 8192) {                                          \
            const unsigned int seen = eray_trace_seen[k];                                     \
            g_eray_trace[blockIdx.x * kTraceSlots + (k) + (seen ? 0 : 32)] = (v);             \
            if (!seen) eray_trace_seen[k] = 1u;                                               \
        }                                                                                     \
    } while (0)
#define ERAY_TRACE_WAVE0(k) ERAY_TRACE_RECORD(k, __builtin_amdgcn_s_memrealtime())
#define ERAY_TRACE_VALUE(k, v) ERAY_TRACE_RECORD(k, (unsigned long long)(v))

#include "../../eray_amd/csrc/render.hip"

extern "C" int eray_debug_read_trace(unsigned long long* out, size_t n) {
    if (n > 8192 * kTraceSlots) n = 8192 * kTraceSlots;
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_eray_trace), n * sizeof(unsigned long long), 0,
                                    hipMemcpyDeviceToHost);
}
extern "C" int eray_debug_clear_trace() {
    static unsigned long long zero[8192 * kTraceSlots];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_eray_trace), zero, sizeof(zero), 0, hipMemcpyHostToDevice);
}
