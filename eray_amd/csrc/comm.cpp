// comm.cpp — the multi-GPU frame gather of the C-ABI, over RCCL.
//
// Every pixel is independent (engine.rs:52-78), so a frame shards by row tiles across the GPUs of
// a node, one process (one eray context) per GPU: rank r renders the r-th block of PPM file rows
// (camera rows [H - (r+1) h, H - r h); eray_render's fused out_ppm writes them in file order), and
// one gather concatenates the blocks on rank 0 in rank order — the PPM body Image::save_as_ppm
// writes (image.rs:48-74).  One collective per frame, over xGMI: u8 rows, 4x fewer bytes than f32.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstring>

#include "../../include/eray_hip.h"

static_assert(ERAY_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");

// capi.cpp's error reporting and the context's gather staging buffer
int eray_internal_error(eray_ctx* ctx, int code, const char* msg);
void* eray_internal_staging(eray_ctx* ctx, size_t bytes);

namespace {
// camera rows of `rank` in the interleaved band split (eray_band_rows)
__host__ __device__ uint32_t band_rows_of(uint32_t height, uint32_t band_rows, uint32_t nranks, uint32_t rank) {
    if (!band_rows || !nranks || rank >= nranks) return 0;
    const uint32_t bands = height / band_rows, tail = height % band_rows;  // the last band may be short
    uint32_t rows = (bands / nranks + (rank < bands % nranks ? 1u : 0u)) * band_rows;
    if (tail && bands % nranks == rank) rows += tail;  // the short band, band index `bands`
    return rows;
}

// Banded gather, on rank 0: file row F of the frame (camera row Y = H - 1 - F) comes from rank
// r = (Y / B) % N, local row j = (Y / (N B)) B + Y % B, which that rank's fused PPM output holds at
// block row rows_r - 1 - j (local file order); the blocks sit at staging + r * block.
__global__ void __launch_bounds__(256) unband_rows_kernel(const uint8_t* __restrict__ staging, uint8_t* __restrict__ frame,
                                                          uint32_t H, uint32_t row_bytes, uint32_t B, uint32_t N,
                                                          uint32_t rows_max) {
    const uint32_t F = blockIdx.x;
    const uint32_t Y = H - 1 - F;
    const uint32_t r = (Y / B) % N;
    const uint32_t j = (Y / (N * B)) * B + Y % B;
    const uint32_t rows_r = band_rows_of(H, B, N, r);
    const uint8_t* src = staging + ((size_t)r * rows_max + (rows_r - 1 - j)) * row_bytes;
    uint8_t* dst = frame + (size_t)F * row_bytes;
    if ((row_bytes % 16) == 0 && ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0) {
        for (uint32_t k = threadIdx.x; k < row_bytes / 16; k += blockDim.x)
            reinterpret_cast<uint4*>(dst)[k] = reinterpret_cast<const uint4*>(src)[k];
    } else {
        for (uint32_t k = threadIdx.x; k < row_bytes; k += blockDim.x) dst[k] = src[k];
    }
}


int nccl_error(eray_ctx* ctx, const char* what, ncclResult_t r) {
    char buf[256];
    std::snprintf(buf, sizeof buf, "%s: %s", what, ncclGetErrorString(r));
    return eray_internal_error(ctx, ERAY_E_HIP, buf);
}
}  // namespace

extern "C" {

int eray_comm_unique_id(uint8_t* id) {
    if (!id) return eray_internal_error(nullptr, ERAY_E_INVALID_ARGUMENT, "id is null");
    ncclUniqueId u;
    const ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return nccl_error(nullptr, "ncclGetUniqueId", r);
    std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    return ERAY_OK;
}

int eray_comm_init(eray_ctx* ctx, int nranks, int rank, const uint8_t* id, void** nccl_comm) {
    if (!ctx || !id || !nccl_comm || nranks < 1 || rank < 0 || rank >= nranks)
        return eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT, "comm_init: bad arguments");
    *nccl_comm = nullptr;
    if (int st = eray_synchronize(ctx)) return st;  // selects the context's device
    ncclUniqueId u;
    std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    ncclComm_t c = nullptr;
    const ncclResult_t r = ncclCommInitRank(&c, nranks, u, rank);
    if (r != ncclSuccess) return nccl_error(ctx, "ncclCommInitRank", r);
    *nccl_comm = c;
    return ERAY_OK;
}

int eray_comm_destroy(void* nccl_comm) {
    if (!nccl_comm) return ERAY_OK;
    const ncclResult_t r = ncclCommDestroy((ncclComm_t)nccl_comm);
    return r == ncclSuccess ? ERAY_OK : nccl_error(nullptr, "ncclCommDestroy", r);
}

uint32_t eray_band_rows(uint32_t height, uint32_t band_rows, uint32_t nranks, uint32_t rank) {
    return band_rows_of(height, band_rows, nranks, rank);
}

int eray_gather_rows(eray_ctx* ctx, void* nccl_comm, const uint8_t* local, uint8_t* frame, uint32_t height,
                     uint32_t width, uint32_t band_rows) {
    if (!ctx || !nccl_comm) return eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT, "gather: null context or comm");
    ncclComm_t c = (ncclComm_t)nccl_comm;
    int nranks = 0, rank = 0;
    ncclResult_t r = ncclCommCount(c, &nranks);
    if (r == ncclSuccess) r = ncclCommUserRank(c, &rank);
    if (r != ncclSuccess) return nccl_error(ctx, "gather: communicator", r);
    if (band_rows % 4) return eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT, "gather: band_rows must be a multiple of 4");
    if (!band_rows && height % (uint32_t)nranks)
        return eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT, "gather: height does not split into equal blocks");
    const size_t row_bytes = (size_t)width * 3u;
    const uint32_t rows = band_rows ? band_rows_of(height, band_rows, (uint32_t)nranks, 0) : height / (uint32_t)nranks;
    const size_t bytes = (size_t)rows * row_bytes;
    if (bytes && !local) return eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT, "gather: local rows are null");
    if (bytes && rank == 0 && !frame) return eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT, "gather: frame is null");
    if (!bytes) return ERAY_OK;
    hipStream_t s = (hipStream_t)eray_get_stream(ctx);
    if (!band_rows) {
        // rank order = PPM file order: rank r's block lands at frame + r * bytes on rank 0 (in place
        // when rank 0's local rows already sit at frame + 0)
        r = ncclGather(local, rank == 0 ? frame : nullptr, bytes, ncclUint8, 0, c, s);
        if (r != ncclSuccess) return nccl_error(ctx, "ncclGather", r);
        return ERAY_OK;
    }
    // bands: every rank sends rows_max rows (rank 0's count; the others' buffers are padded), rank
    // 0 gathers them into its staging buffer and puts each row at its file row
    uint8_t* staging = nullptr;
    if (rank == 0) {
        staging = static_cast<uint8_t*>(eray_internal_staging(ctx, bytes * (size_t)nranks));
        if (!staging) return eray_internal_error(ctx, ERAY_E_OUT_OF_MEMORY, "gather: staging buffer");
    }
    r = ncclGather(local, staging, bytes, ncclUint8, 0, c, s);
    if (r != ncclSuccess) return nccl_error(ctx, "ncclGather", r);
    if (rank == 0) {
        unband_rows_kernel<<<height, 256, 0, s>>>(staging, frame, height, (uint32_t)row_bytes, band_rows, (uint32_t)nranks,
                                                   rows);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return eray_internal_error(ctx, ERAY_E_HIP, hipGetErrorString(e));
    }
    return ERAY_OK;
}

// Diagnostics (tests): rank 0's reordering step of the banded gather alone — staging holds the N
// ranks' padded local PPM blocks as the collective would leave them.
int eray_debug_unband(eray_ctx* ctx, const uint8_t* staging, uint8_t* frame, uint32_t height, uint32_t width,
                      uint32_t band_rows, uint32_t nranks) {
    if (!ctx || !staging || !frame || !band_rows || band_rows % 4 || !nranks)
        return eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT, "unband: bad arguments");
    if (!height) return ERAY_OK;
    hipStream_t s = (hipStream_t)eray_get_stream(ctx);
    unband_rows_kernel<<<height, 256, 0, s>>>(staging, frame, height, width * 3u, band_rows, nranks,
                                               band_rows_of(height, band_rows, nranks, 0));
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? ERAY_OK : eray_internal_error(ctx, ERAY_E_HIP, hipGetErrorString(e));
}

}  // extern "C"
