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

// capi.cpp's error reporting and stream access for a context
int eray_internal_error(eray_ctx* ctx, int code, const char* msg);

namespace {
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

int eray_gather_rows(eray_ctx* ctx, void* nccl_comm, const uint8_t* local, uint8_t* frame, uint32_t rows,
                     uint32_t width) {
    if (!ctx || !nccl_comm) return eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT, "gather: null context or comm");
    ncclComm_t c = (ncclComm_t)nccl_comm;
    int nranks = 0, rank = 0;
    ncclResult_t r = ncclCommCount(c, &nranks);
    if (r == ncclSuccess) r = ncclCommUserRank(c, &rank);
    if (r != ncclSuccess) return nccl_error(ctx, "gather: communicator", r);
    const size_t bytes = (size_t)rows * width * 3u;
    if (bytes && !local) return eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT, "gather: local rows are null");
    if (bytes && rank == 0 && !frame) return eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT, "gather: frame is null");
    if (!bytes) return ERAY_OK;
    hipStream_t s = (hipStream_t)eray_get_stream(ctx);
    // rank order = PPM file order: rank r's block lands at frame + r * bytes on rank 0 (in place
    // when rank 0's local rows already sit at frame + 0)
    r = ncclGather(local, rank == 0 ? frame : nullptr, bytes, ncclUint8, 0, c, s);
    if (r != ncclSuccess) return nccl_error(ctx, "ncclGather", r);
    return ERAY_OK;
}

}  // extern "C"
