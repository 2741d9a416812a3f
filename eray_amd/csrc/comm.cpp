// comm.cpp — the multi-GPU frame gather of the C-ABI, over RCCL.
//
// Every pixel is independent (engine.rs:52-78), so a frame shards by row tiles across the GPUs of
// a node, one process (one eray context) per GPU: rank r renders the r-th block of PPM file rows
// (camera rows [H - (r+1) h, H - r h); eray_render's fused out_ppm writes them in file order), and
// one gather concatenates the blocks on rank 0 in rank order — the PPM body Image::save_as_ppm
// writes (image.rs:48-74).  u8 rows, 4x fewer bytes than f32.  With interleaved bands (equal work
// per rank) the rows travel coded (uniform 64-pixel segments as one word) by point-to-point
// transfers into rank 0, which writes each file row from them.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/eray_hip.h"
#include "internal.hpp"

static_assert(ERAY_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");

// capi.cpp's error reporting, the context's gather staging buffer, the scene camera's setup and
// the context's slot for this file's gather plan
int eray_internal_error(eray_ctx* ctx, int code, const char* msg);
void* eray_internal_staging(eray_ctx* ctx, size_t bytes);
int eray_internal_frame_source(eray_ctx* ctx, const uint8_t* local, uint64_t stride, uint32_t n,
                               eray::gpu::FrameSource* out);
int eray_internal_source_layout(eray_ctx* ctx, const eray::gpu::FrameSource& src, eray::gpu::SceneLayout* out);
int eray_internal_scene_setup_source(eray_ctx* ctx, eray::gpu::FrameSource* out);
void** eray_internal_gather_plan(eray_ctx* ctx, void (*free_fn)(void*));
int eray_internal_use_device(eray_ctx* ctx);
void eray_internal_untag(eray_ctx* ctx, const void* p, size_t bytes);
void eray_internal_gather_source(const eray_ctx* ctx, eray::gpu::FrameSource* out);
uint8_t* eray_internal_coll_scratch(eray_ctx* ctx);

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

// ---- coded transport of the banded gather -------------------------------------------------
// A frame is mostly rows of the same colour (engine.rs:212's miss colour, wherever no face is
// hit), so each rank sends its rows as 64-pixel segments: a uniform segment as one code word
// (flag bit + its pixel's 3 bytes), any other as its 192 bytes, packed.  Rank 0 receives every
// rank's code words (4 B per segment) and packed segments and writes each file row from them.
// At C2's pixel pitch about 1 segment in 30 is not uniform: 6.2 MB of rows per rank become
// ~0.2 MB, and the gather into rank 0 is no longer bound by its xGMI links.
constexpr uint32_t kSegPx = 64, kSegBytes = 3 * kSegPx;
constexpr uint32_t kUniform = 0x80000000u;
constexpr int kMaxCodedRanks = eray::gpu::kMaxGatherRanks;
constexpr uint32_t kCountFailed = 0xffffffffu;  // a rank's count word when it cannot take part
struct RankOffsets {
    uint32_t v[kMaxCodedRanks];  // first packed segment of each rank in rank 0's staging
};

// segment g = q * S + s: block row q of the rank's local rows (rows_r valid of rows_max), pixels
// [64 s, min(64 s + 64, W)).  Its code word: kUniform | b0 | b1 << 8 | b2 << 16 when all its pixels
// equal the first, else the index of its slot in `packed`, where its bytes are copied (slots
// taken with one counter atomic per workgroup: in no particular order, the code word says where).
// *count ends as the number of packed segments (zero on entry).
// Rows of 16-byte multiples (W % 16 == 0) on 16-byte aligned buffers: 16 lanes per segment, each
// comparing one 16-byte word with the first pixel's repeating pattern (coalesced, a ballot per
// segment), then copying the words of the workgroup's non-uniform segments to their slots;
// otherwise one lane per segment, byte by byte.
__device__ __forceinline__ void pattern_words(uint32_t c, uint32_t (&d)[3]) {  // the 12-byte period
    const uint32_t b0 = c & 0xffu, b1 = (c >> 8) & 0xffu, b2 = (c >> 16) & 0xffu;
    d[0] = b0 | (b1 << 8) | (b2 << 16) | (b0 << 24);
    d[1] = b1 | (b2 << 8) | (b0 << 16) | (b1 << 24);
    d[2] = b2 | (b0 << 8) | (b1 << 16) | (b2 << 24);
}
// one slot per set bit of `want` (lanes of the wave), from the shared counter
__device__ __forceinline__ uint32_t wave_slot(unsigned long long want, uint32_t lane, uint32_t* count) {
    if (!want) return 0u;
    const uint32_t first = (uint32_t)(__ffsll(want) - 1);
    uint32_t base = 0;
    if (lane == first) base = atomicAdd(count, (uint32_t)__popcll(want));
    base = (uint32_t)__shfl((int)base, (int)first);
    return base + (uint32_t)__popcll(want & ((1ull << lane) - 1ull));
}
constexpr uint32_t kBlkSegs = 64;  // segments per workgroup of the wide encoder: one slot atomic each
__global__ void __launch_bounds__(256) seg_encode_wide_kernel(const uint8_t* __restrict__ local, uint32_t rows_r,
                                                              uint32_t rows_max, uint32_t W, uint32_t S,
                                                              uint32_t* __restrict__ code, uint8_t* __restrict__ packed,
                                                              uint32_t* __restrict__ count) {
    __shared__ uint32_t s_code[kBlkSegs];  // uniform code, or ~0u for a segment to pack
    __shared__ uint32_t s_slot[kBlkSegs];
    const uint32_t G = rows_max * S;
    const uint32_t k = threadIdx.x & 15u, lane = threadIdx.x & 63u;
    // pass 1: 16 lanes per segment compare its 16-byte words with the first pixel's pattern
    for (uint32_t it = 0; it < kBlkSegs / 16; ++it) {
        const uint32_t i = it * 16 + (threadIdx.x >> 4), g = blockIdx.x * kBlkSegs + i;
        const bool in = g < G;
        const uint32_t q = in ? g / S : 0u, s = in ? g - q * S : 0u;
        const bool live = in && q < rows_r;  // (padding rows of a rank with fewer bands: never decoded)
        const uint32_t words = live ? min(kSegPx, W - s * kSegPx) * 3u / 16u : 0u;
        const uint4* seg = reinterpret_cast<const uint4*>(local + (size_t)q * W * 3u + (size_t)s * kSegBytes);
        uint32_t c = 0;
        bool bad = false;
        if (live) {
            c = reinterpret_cast<const uint32_t*>(seg)[0] & 0xffffffu;
            if (k < words) {
                uint32_t d[3];
                pattern_words(c, d);
                const uint4 v = seg[k];  // dword 4k + j of the segment is period word (k + j) % 3
                bad = v.x != d[k % 3] || v.y != d[(k + 1) % 3] || v.z != d[(k + 2) % 3] || v.w != d[k % 3];
            }
        }
        const unsigned long long m = __ballot(bad);
        if (k == 0) s_code[i] = ((m >> (lane & ~15u)) & 0xffffull) ? ~0u : (kUniform | c);
    }
    __syncthreads();
    // one slot atomic for the workgroup's packed segments
    if (threadIdx.x < kBlkSegs) {
        const bool want = s_code[threadIdx.x] == ~0u;
        const unsigned long long bal = __ballot(want);
        uint32_t base = 0;
        if (threadIdx.x == 0 && bal) base = atomicAdd(count, (uint32_t)__popcll(bal));
        base = (uint32_t)__shfl((int)base, 0);
        s_slot[threadIdx.x] = base + (uint32_t)__popcll(bal & ((1ull << threadIdx.x) - 1ull));
    }
    __syncthreads();
    // pass 2: the code words, and the packed segments' bytes (L2-resident since pass 1)
    for (uint32_t it = 0; it < kBlkSegs / 16; ++it) {
        const uint32_t i = it * 16 + (threadIdx.x >> 4), g = blockIdx.x * kBlkSegs + i;
        if (g >= G) continue;
        const uint32_t cw = s_code[i];
        if (cw != ~0u) {
            if (k == 0) code[g] = cw;
            continue;
        }
        const uint32_t q = g / S, s = g - q * S;
        const uint32_t words = min(kSegPx, W - s * kSegPx) * 3u / 16u;
        const uint32_t slot = s_slot[i];
        if (k == 0) code[g] = slot;
        if (k < words)
            reinterpret_cast<uint4*>(packed + (size_t)slot * kSegBytes)[k] =
                reinterpret_cast<const uint4*>(local + (size_t)q * W * 3u + (size_t)s * kSegBytes)[k];
    }
}
__global__ void __launch_bounds__(256) seg_encode_kernel(const uint8_t* __restrict__ local, uint32_t rows_r,
                                                         uint32_t rows_max, uint32_t W, uint32_t S,
                                                         uint32_t* __restrict__ code, uint8_t* __restrict__ packed,
                                                         uint32_t* __restrict__ count) {
    const uint32_t g = blockIdx.x * 256u + threadIdx.x, lane = threadIdx.x & 63u;
    const bool in = g < rows_max * S;
    const uint32_t q = in ? g / S : 0u, s = in ? g - q * S : 0u;
    const bool live = in && q < rows_r;
    const uint8_t* p = local + (size_t)q * W * 3u + (size_t)s * kSegBytes;
    const uint32_t n = live ? min(kSegPx, W - s * kSegPx) * 3u : 0u;
    uint32_t b0 = 0, b1 = 0, b2 = 0;
    bool uniform = true;
    if (live) {
        b0 = p[0];
        b1 = p[1];
        b2 = p[2];
        for (uint32_t k = 3; k < n; k += 3) uniform &= p[k] == b0 && p[k + 1] == b1 && p[k + 2] == b2;
    }
    const uint32_t slot = wave_slot(__ballot(live && !uniform), lane, count);
    if (!in) return;
    if (live && !uniform) {
        uint8_t* dst = packed + (size_t)slot * kSegBytes;
        for (uint32_t k = 0; k < n; ++k) dst[k] = p[k];
        code[g] = slot;
    } else {
        code[g] = kUniform | b0 | (b1 << 8) | (b2 << 16);
    }
}

// Rank 0: file row F of the frame (camera row Y = H - 1 - F) from rank r = (Y / B) % N, local row
// j = (Y / (N B)) B + Y % B at that rank's block row rows_r - 1 - j (as unband_rows_kernel), each
// segment from its code word: the colour repeated, or the packed bytes.
__device__ __forceinline__ uint8_t code_byte(uint32_t c, uint32_t i) { return (uint8_t)(c >> (8u * (i % 3u))); }
__global__ void __launch_bounds__(256) seg_decode_kernel(const uint32_t* __restrict__ codes,
                                                         const uint8_t* __restrict__ packed, RankOffsets off,
                                                         uint8_t* __restrict__ frame, uint32_t H, uint32_t W,
                                                         uint32_t S, uint32_t B, uint32_t N, uint32_t rows_max) {
    const uint32_t F = blockIdx.x;
    const uint32_t Y = H - 1 - F;
    const uint32_t r = (Y / B) % N;
    const uint32_t j = (Y / (N * B)) * B + Y % B;
    const uint32_t q = band_rows_of(H, B, N, r) - 1 - j;
    const uint32_t* cr = codes + ((size_t)r * rows_max + q) * S;
    const uint8_t* pr = packed + (size_t)off.v[r] * kSegBytes;
    const uint32_t row_bytes = W * 3u;
    uint8_t* dst = frame + (size_t)F * row_bytes;
    if ((row_bytes % 16) == 0 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0 &&
        (reinterpret_cast<uintptr_t>(packed) & 15) == 0) {
        for (uint32_t k = threadIdx.x; k < row_bytes / 16; k += blockDim.x) {
            const uint32_t s = k / (kSegBytes / 16), w = k - s * (kSegBytes / 16);
            const uint32_t c = cr[s];
            uint4 v;
            if (c & kUniform) {  // dword 4w + t of the segment is period word (w + t) % 3
                uint32_t d[3];
                pattern_words(c, d);
                const uint32_t ph = w % 3u;
                v = make_uint4(d[ph], d[(ph + 1) % 3u], d[(ph + 2) % 3u], d[ph]);
            } else {
                v = reinterpret_cast<const uint4*>(pr + (size_t)c * kSegBytes)[w];
            }
            reinterpret_cast<uint4*>(dst)[k] = v;
        }
    } else {
        for (uint32_t k = threadIdx.x; k < row_bytes; k += blockDim.x) {
            const uint32_t s = k / kSegBytes, i = k - s * kSegBytes;
            const uint32_t c = cr[s];
            dst[k] = (c & kUniform) ? code_byte(c, i) : pr[(size_t)c * kSegBytes + i];
        }
    }
}

// Device buffers of one rank's coded gather: the code words and packed segments carved from one
// staging allocation (rank 0: a code block and packed room for every rank); the packed count and
// the all-gathered counts in the context's collective scratch (no allocation can keep a rank out
// of the count exchange).
struct CodedBufs {
    uint32_t *code = nullptr, *count = nullptr, *counts = nullptr;
    uint8_t* packed = nullptr;
};
bool coded_bufs(eray_ctx* ctx, uint32_t G, uint32_t slots, CodedBufs* b) {
    auto up = [](size_t x) { return (x + 255) / 256 * 256; };
    const size_t n_code = up((size_t)slots * G * 4);
    const size_t n_packed = (size_t)slots * G * kSegBytes;
    uint8_t* base = static_cast<uint8_t*>(eray_internal_staging(ctx, n_code + n_packed));
    if (!base) return false;
    b->code = reinterpret_cast<uint32_t*>(base);
    b->packed = base + n_code;
    return true;
}

// Encodes `rows_r` local block rows (of rows_max) into code (G words) and packed; the count of
// packed segments into *b.count.
hipError_t encode_rows(const uint8_t* local, uint32_t rows_r, uint32_t rows_max, uint32_t W, uint32_t S,
                       uint32_t* code, uint8_t* packed, const CodedBufs& b, hipStream_t s) {
    const uint32_t G = rows_max * S;
    hipError_t e = hipMemsetAsync(b.count, 0, 4, s);
    if (e != hipSuccess) return e;
    const bool wide = (W % 16u) == 0 && ((reinterpret_cast<uintptr_t>(local) | reinterpret_cast<uintptr_t>(packed)) & 15) == 0;
    if (wide)
        seg_encode_wide_kernel<<<(G + kBlkSegs - 1) / kBlkSegs, 256, 0, s>>>(local, rows_r, rows_max, W, S, code, packed,
                                                                             b.count);
    else
        seg_encode_kernel<<<(G + 255) / 256, 256, 0, s>>>(local, rows_r, rows_max, W, S, code, packed, b.count);
    return hipGetLastError();
}

// ---- scene-camera gather: only the objects' pixel rectangles travel --------------------------
// The frame kernel writes engine.rs:212's miss colour at every pixel outside the objects' pixel
// rectangles (ObjGeom::rect: no primary ray there can hit any face, the same conservative bounds
// the kernel culls with).  So when every rank's local rows are its renders of the scene camera,
// the frame on rank 0 is the miss colour except inside those rectangles, and only their bytes need
// to cross xGMI.  The rectangles are fixed per camera: each rank states its own (rank-local rows,
// 16-pixel column groups) once, one all-gather exchanges them (the only host synchronisation),
// and every later gather enqueues a pack kernel, fixed-size point-to-point transfers and, on rank
// 0, one assembly kernel — no host round trip, so a serving loop can capture it in a graph.
constexpr int kPlanRects = 8;
struct GatherRect {        // one rectangle of a rank's rows, 32 B
    int32_t l0, l1;        // local rows (inclusive)
    int32_t c0, c1;        // 16-pixel column groups (inclusive)
    uint32_t off;          // byte offset of its first row in the rank's per-frame pack
    uint32_t row_bytes;    // 48 * (c1 - c0 + 1)
    uint32_t first;        // its first packed row among the rank's (pack kernel)
    uint32_t pad;
};
struct RankLayout {        // a rank's rectangles and its share of rank 0's receive buffer
    GatherRect r[kPlanRects];
    uint32_t nrect, bytes;  // bytes per frame (a multiple of 48)
    uint64_t off;           // per-frame offset of the rank's block (prefix sum of bytes)
    uint32_t rows, packed_rows;
    uint32_t pad[2];
};
// Which rank assembles frame k of a batch of B: rank 0, or (ERAY_GATHER_ROTATE_ROOT) rank k % n,
// which spreads the assembly's frame writes and the inbound xGMI bytes of a stream of frames over
// every GPU instead of piling them on rank 0.  A rank's pack of the batch holds its frames grouped
// by root (one transfer per rank pair moves each group); the frames it assembles itself are packed
// straight into its receive area.
struct Roots {
    uint32_t B, n;  // n == 0: every frame's root is rank 0
    __host__ __device__ uint32_t root(uint32_t k) const { return n ? k % n : 0u; }
    __host__ __device__ uint32_t index(uint32_t k) const { return n ? k / n : k; }  // among its root's frames
    __host__ __device__ uint32_t count(uint32_t r) const {
        return n ? (r < B ? (B - 1u - r) / n + 1u : 0u) : (r ? 0u : B);
    }
    __host__ __device__ uint32_t before(uint32_t r) const {  // frames whose root is below r
        return n ? (B / n) * r + (B % n < r ? B % n : r) : 0u;
    }
    // frame k's slot in rank `me`'s send area (frames of other roots, grouped by root)
    __host__ __device__ uint32_t send_slot(uint32_t k, uint32_t me) const {
        const uint32_t r = root(k);
        return before(r) - (r > me ? count(me) : 0u) + index(k);
    }
    // roots with frames (0 .. roots() - 1), and root r's group among me's send groups
    __host__ __device__ uint32_t roots() const { return n ? (B < n ? B : n) : 1u; }
    __host__ __device__ uint32_t group(uint32_t r, uint32_t me) const {
        const uint32_t R = roots();
        return (r < R ? r : R) - (me < r && me < R ? 1u : 0u);
    }
};

// Every transfer of the scene-camera gather ends with its sender's header: the sender's verdict
// on its own arguments and the source (kind, key) of the frames it packed.  A root assembles its
// frames only when every header it uses says ERAY_OK and the plan's source; otherwise it writes
// none of them and raises the plan's fault word, which the context's next eray_gather_frames
// reports — a rank that could not use its arguments still takes part in the transfers, and its
// stale bytes never become a frame.
struct XferHeader {
    int32_t status;
    uint32_t kind, key_lo, key_hi;
};
constexpr size_t kHdr = sizeof(XferHeader);
static_assert(kHdr == 16, "one 16-B word");
__host__ __device__ inline bool header_ok(const XferHeader& h, uint32_t kind, uint64_t key) {
    return h.status == 0 && h.kind == kind && h.key_lo == (uint32_t)key && h.key_hi == (uint32_t)(key >> 32);
}
// Rank q's block in a receive area of `mine` frames: its packs (mine x bytes), then its header.
__host__ __device__ inline uint64_t recv_block(const RankLayout& L, uint32_t q, uint32_t mine) {
    return (uint64_t)mine * L.off + kHdr * q;
}

// A rank's record in the plan exchange: [status, source kind, key low, key high | nrect, then
// nrect x (l0, l1, c0, c1)] — every rank learns every rank's status and source, so all of them
// accept the plan or all fail together.
constexpr int kXchgHead = 4;
constexpr int kXchgInts = kXchgHead + 1 + 4 * kPlanRects;

// The context's collective scratch (eray_internal_coll_scratch, allocated with the context):
// status and count words at kScrWords, the plan exchange's records at kScrXchg, the plan's rank
// table (the assembly kernels' RankLayout array) at kScrRanks.
constexpr size_t kScrWords = 0, kScrXchg = 1024, kScrRanks = kScrXchg + 12288;
static_assert(4 * (kMaxCodedRanks + 2) <= kScrXchg, "status words");
static_assert(kScrXchg + sizeof(int32_t) * kXchgInts * (kMaxCodedRanks + 1) <= kScrRanks, "plan records");
static_assert(kScrRanks + sizeof(RankLayout) * kMaxCodedRanks <= eray::gpu::kCollScratchBytes, "rank table");

struct GatherPlan {
    void* comm = nullptr;
    int32_t* fault = nullptr;      // mapped host word: a root met a failed or foreign header
    int32_t* d_fault = nullptr;    // (its device address)
    hipEvent_t asm_ev = nullptr;   // after the last assembly enqueued outside a graph capture
    bool asm_pending = false;      // ... whose fault word has not been read yet
    uint32_t kind = 0;
    uint64_t key = 0;
    uint32_t H = 0, W = 0, band = 0, nranks = 0, rank = 0;
    bool valid = false;
    std::vector<RankLayout> ranks;
    uint64_t total = 0;            // every rank's bytes per frame
    RankLayout* d_ranks = nullptr; // the assembly's table (every rank: any may be a root), in the scratch
    uint8_t* buf = nullptr;        // [receive area: its frames x every rank's packs | send area: its packs]
    size_t buf_cap = 0;
    // batch sizes whose transfer buffers every rank has confirmed since the plan was made (a new
    // size's first call agrees on that before any transfer)
    std::vector<uint32_t> batches;
};
void plan_release(GatherPlan& P) {
    if (P.buf) (void)hipFree(P.buf);
    if (P.fault) (void)hipHostFree(P.fault);
    if (P.asm_ev) (void)hipEventDestroy(P.asm_ev);
    P.d_ranks = nullptr;
    P.buf = nullptr;
    P.fault = P.d_fault = nullptr;
    P.asm_ev = nullptr;
    P.asm_pending = false;
}
void plan_free(void* v) {
    auto* P = static_cast<GatherPlan*>(v);
    if (!P) return;
    plan_release(*P);
    delete P;
}

// The local rows of rank `rank` (rows, camera row of local row j): interleaved bands (band > 0)
// or the rank's block of PPM file rows (camera rows [H - (rank+1) h, H - rank h)).
struct RankRows {
    uint32_t row0, rows, shift, stride;
};
RankRows rank_rows(uint32_t H, uint32_t band, uint32_t N, uint32_t rank) {
    if (!band) {
        const uint32_t h = H / N;
        return RankRows{H - (rank + 1) * h, h, 31u, 0u};
    }
    uint32_t shift = 0;
    while ((1u << shift) < band) ++shift;
    return RankRows{rank * band, band_rows_of(H, band, N, rank), shift, N * band};
}

// This rank's rectangles: the objects' pixel rectangles in its local rows and 16-pixel column
// groups, overlapping ones merged (as camera_setup_kernel merges the detail rectangles), more than
// kPlanRects merged into the last.
std::vector<std::array<int32_t, 4>> my_rects(const std::vector<std::array<int32_t, 4>>& rects, const RankRows& rr,
                                             uint32_t W) {
    std::vector<std::array<int32_t, 4>> out;
    for (const auto& q : rects) {
        int32_t x0 = std::max(q[0], 0), x1 = std::min(q[1], (int32_t)W - 1), l0, l1;
        if (x0 > x1 || q[2] > q[3]) continue;
        eray::gpu::band_local_range(rr.row0, rr.shift, rr.stride, q[2], q[3], &l0, &l1);
        l0 = std::max(l0, 0);
        l1 = std::min(l1, (int32_t)rr.rows - 1);
        if (l0 > l1) continue;
        std::array<int32_t, 4> r{l0, l1, x0 / 16, x1 / 16};
        if (out.size() == (size_t)kPlanRects) {
            auto& z = out.back();
            z = {std::min(z[0], r[0]), std::max(z[1], r[1]), std::min(z[2], r[2]), std::max(z[3], r[3])};
        } else {
            out.push_back(r);
        }
    }
    for (bool merged = true; merged;) {
        merged = false;
        for (size_t a = 0; a < out.size() && !merged; ++a)
            for (size_t b = a + 1; b < out.size() && !merged; ++b) {
                auto &x = out[a], &y = out[b];
                if (x[0] > y[1] || y[0] > x[1] || x[2] > y[3] || y[2] > x[3]) continue;
                x = {std::min(x[0], y[0]), std::max(x[1], y[1]), std::min(x[2], y[2]), std::max(x[3], y[3])};
                out.erase(out.begin() + (std::ptrdiff_t)b);
                merged = true;
            }
    }
    return out;
}

// The rectangle part of an exchange record (nrect, then the rectangles).
void write_rects(const std::vector<std::array<int32_t, 4>>& mine, int32_t* rec) {
    rec[0] = (int32_t)mine.size();
    for (size_t i = 0; i < mine.size(); ++i)
        for (int q = 0; q < 4; ++q) rec[1 + 4 * i + q] = mine[i][q];
}

RankLayout layout_of(const int32_t* rec, uint32_t rows) {
    RankLayout R{};
    R.nrect = (uint32_t)std::min(std::max(rec[0], 0), kPlanRects);
    R.rows = rows;
    uint32_t off = 0, first = 0;
    for (uint32_t i = 0; i < R.nrect; ++i) {
        GatherRect& g = R.r[i];
        g.l0 = rec[1 + 4 * i];
        g.l1 = rec[2 + 4 * i];
        g.c0 = rec[3 + 4 * i];
        g.c1 = rec[4 + 4 * i];
        g.off = off;
        g.row_bytes = 48u * (uint32_t)(g.c1 - g.c0 + 1);
        g.first = first;
        first += (uint32_t)(g.l1 - g.l0 + 1);
        off += g.row_bytes * (uint32_t)(g.l1 - g.l0 + 1);
    }
    R.bytes = off;
    R.packed_rows = first;
    return R;
}

// Rank `me`'s rows of frame blockIdx.y, rectangle by rectangle (16-B words: rows of W % 16 == 0
// pixels on 16-B aligned buffers, column groups of 48 B), into its slot: own + index * bytes when
// `me` assembles the frame, else send + send_slot * bytes.
__global__ void __launch_bounds__(256) gather_pack_kernel(const uint8_t* __restrict__ local, uint64_t local_stride,
                                                          uint8_t* __restrict__ send, uint8_t* __restrict__ own,
                                                          RankLayout L, uint32_t W, Roots R, uint32_t me) {
    const uint32_t q = blockIdx.x, k = blockIdx.y;
    const uint32_t rk = R.root(k);
    uint8_t* out = rk == me ? own + (size_t)R.index(k) * L.bytes
                            : send + (size_t)R.send_slot(k, me) * L.bytes + kHdr * R.group(rk, me);
    uint32_t i = 0;
    while (i + 1 < L.nrect && q >= L.r[i + 1].first) ++i;
    const GatherRect& g = L.r[i];
    const uint32_t j = (uint32_t)g.l0 + (q - g.first);
    const uint4* src = reinterpret_cast<const uint4*>(local + k * local_stride + (size_t)(L.rows - 1 - j) * W * 3u +
                                                      48u * (uint32_t)g.c0);
    uint4* dst = reinterpret_cast<uint4*>(out + g.off + (size_t)(q - g.first) * g.row_bytes);
    for (uint32_t w = threadIdx.x; w < g.row_bytes / 16u; w += blockDim.x) dst[w] = src[w];
}

// A root: file row blockIdx.x of its frame blockIdx.y (of B) — the miss colour, except inside the
// owning rank's rectangles, whose bytes come from that rank's block of the receive area.
__global__ void __launch_bounds__(256) gather_assemble_kernel(const uint8_t* __restrict__ recv,
                                                              const RankLayout* __restrict__ lay, uint32_t B,
                                                              uint8_t* __restrict__ frames, uint64_t frame_stride,
                                                              uint32_t H, uint32_t W, uint32_t band, uint32_t N,
                                                              uint32_t kind, uint64_t key, int32_t* fault) {
    __shared__ RankLayout s_L;
    // every sender's header (and this root's own): all ERAY_OK and the plan's source, or no frame
    bool bad = false;
    if (threadIdx.x < N) {
        const RankLayout& Lq = lay[threadIdx.x];
        if (Lq.bytes) {
            const XferHeader h = *reinterpret_cast<const XferHeader*>(recv + recv_block(Lq, threadIdx.x, B) +
                                                                      (size_t)B * Lq.bytes);
            bad = !header_ok(h, kind, key);
        }
    }
    if (__syncthreads_or(bad)) {
        if (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0) __hip_atomic_store(fault, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    const uint32_t F = blockIdx.x, k = blockIdx.y;
    const uint32_t Y = H - 1 - F;  // camera row
    uint32_t r, j;
    if (band) {
        r = (Y / band) % N;
        j = (Y / (N * band)) * band + Y % band;
    } else {
        const uint32_t h = H / N;
        r = (H - 1 - Y) / h;
        j = Y - (H - (r + 1) * h);
    }
    if (threadIdx.x < sizeof(RankLayout) / 4)
        reinterpret_cast<uint32_t*>(&s_L)[threadIdx.x] = reinterpret_cast<const uint32_t*>(lay + r)[threadIdx.x];
    __syncthreads();
    uint32_t bg[3];
    pattern_words(25u | (25u << 8) | (51u << 16), bg);  // sat_u8(0.1 * 255), sat_u8(0.2 * 255)
    const uint8_t* base = recv + recv_block(s_L, r, B) + (size_t)k * s_L.bytes;
    uint4* dst = reinterpret_cast<uint4*>(frames + k * frame_stride + (size_t)F * W * 3u);
    for (uint32_t w = threadIdx.x; w < W * 3u / 16u; w += blockDim.x) {
        const uint32_t c = w / 3u;  // 16-pixel column group (48 B = 3 words)
        uint4 v;
        const uint32_t ph = w % 3u;
        v = make_uint4(bg[ph], bg[(ph + 1) % 3u], bg[(ph + 2) % 3u], bg[ph]);
        for (uint32_t i = 0; i < s_L.nrect; ++i) {
            const GatherRect& g = s_L.r[i];
            if ((int32_t)j >= g.l0 && (int32_t)j <= g.l1 && (int32_t)c >= g.c0 && (int32_t)c <= g.c1) {
                v = reinterpret_cast<const uint4*>(base + g.off + (size_t)((int32_t)j - g.l0) * g.row_bytes)
                    [w - 3u * (uint32_t)g.c0];
                break;
            }
        }
        dst[w] = v;
    }
}

// The headers a rank writes into its buffer: one after each send group, one after its own packs.
struct HeaderSpots {
    uint64_t off[kMaxCodedRanks + 1];
    uint32_t n;
};
__global__ void gather_header_kernel(uint8_t* __restrict__ buf, HeaderSpots at, XferHeader h) {
    if (threadIdx.x < at.n) *reinterpret_cast<XferHeader*>(buf + at.off[threadIdx.x]) = h;
}

int nccl_error(eray_ctx* ctx, const char* what, ncclResult_t r) {
    char buf[256];
    std::snprintf(buf, sizeof buf, "%s: %s", what, ncclGetErrorString(r));
    return eray_internal_error(ctx, ERAY_E_HIP, buf);
}

// Every rank's status word, all-gathered through the collective scratch (one stream
// synchronisation): this rank's own failure, else the first failing rank's, else ERAY_OK — the
// same outcome on every rank, so they all go on to the next collective or all return.
int agree(eray_ctx* ctx, ncclComm_t c, int nranks, int status, const char* what) {
    hipStream_t s = (hipStream_t)eray_get_stream(ctx);
    int32_t* words = reinterpret_cast<int32_t*>(eray_internal_coll_scratch(ctx) + kScrWords);
    const int32_t mine = status;
    std::vector<int32_t> all((size_t)nranks);
    hipError_t he;
    if ((he = hipMemcpyAsync(words, &mine, 4, hipMemcpyHostToDevice, s)) != hipSuccess)
        return eray_internal_error(ctx, ERAY_E_HIP, hipGetErrorString(he));
    const ncclResult_t r = ncclAllGather(words, words + 1, 1, ncclInt32, c, s);
    if (r != ncclSuccess) return nccl_error(ctx, what, r);
    if ((he = hipMemcpyAsync(all.data(), words + 1, 4u * (size_t)nranks, hipMemcpyDeviceToHost, s)) != hipSuccess ||
        (he = hipStreamSynchronize(s)) != hipSuccess)
        return eray_internal_error(ctx, ERAY_E_HIP, hipGetErrorString(he));
    if (status != ERAY_OK) return status;
    for (int q = 0; q < nranks; ++q)
        if (all[(size_t)q] != ERAY_OK) {
            char msg[128];
            std::snprintf(msg, sizeof msg, "%s: rank %d could not take part (status %d)", what, q, all[(size_t)q]);
            return eray_internal_error(ctx, all[(size_t)q], msg);
        }
    return ERAY_OK;
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
    if (band_rows && (band_rows < 4 || (band_rows & (band_rows - 1))))  // as eray_render's bands (capi.cpp)
        return eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT, "gather: band_rows must be a power of two >= 4");
    if (!band_rows && height % (uint32_t)nranks)
        return eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT, "gather: height does not split into equal blocks");
    if (nranks > kMaxCodedRanks)  // (shared arguments: every rank returns here)
        return eray_internal_error(ctx, ERAY_E_UNSUPPORTED, "gather: more than 64 ranks");
    const size_t row_bytes = (size_t)width * 3u;
    const uint32_t rows = band_rows ? band_rows_of(height, band_rows, (uint32_t)nranks, 0) : height / (uint32_t)nranks;
    const size_t bytes = (size_t)rows * row_bytes;
    if (!bytes) return ERAY_OK;  // (shared arguments: every rank returns here)
    // this rank's verdict on its own buffers: a failing rank still takes part in the status
    // exchange below, and every rank returns an error before any rows move
    int status = ERAY_OK;
    if (!local) status = eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT, "gather: local rows are null");
    else if (rank == 0 && !frame) status = eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT, "gather: frame is null");
    hipStream_t s = (hipStream_t)eray_get_stream(ctx);
    hipError_t he;
    if (!band_rows) {
        // every rank's status (one word each, all-gathered, one stream synchronisation), then the
        // rows: rank order = PPM file order, rank r's block lands at frame + r * bytes on rank 0 (in
        // place when rank 0's local rows already sit at frame + 0)
        if (int st = agree(ctx, c, nranks, status, "gather")) return st;
        r = ncclGather(local, rank == 0 ? frame : nullptr, bytes, ncclUint8, 0, c, s);
        if (r != ncclSuccess) return nccl_error(ctx, "ncclGather", r);
        return ERAY_OK;
    }
    {
        // bands, coded (see seg_classify_kernel): every rank encodes its rows; the packed counts
        // reach every host (one all-gather of a word each, then a stream synchronisation: the
        // point-to-point sizes must be known to post them); rank 0 receives every rank's code
        // words and packed segments and decodes the frame
        const uint32_t S = (width + kSegPx - 1) / kSegPx, G = rows * S;
        const uint32_t mine = band_rows_of(height, band_rows, (uint32_t)nranks, (uint32_t)rank);
        CodedBufs b;
        b.count = reinterpret_cast<uint32_t*>(eray_internal_coll_scratch(ctx) + kScrWords);
        b.counts = b.count + 1;
        if (status == ERAY_OK && !coded_bufs(ctx, G, rank == 0 ? (uint32_t)nranks : 1u, &b))
            status = eray_internal_error(ctx, ERAY_E_OUT_OF_MEMORY, "gather: staging buffer");
        // the packed-segment counts carry the ranks' verdicts: a rank that cannot use its buffers
        // (or allocate its staging) sends kCountFailed, and every rank returns an error before the
        // transfers
        if (status == ERAY_OK) {
            he = encode_rows(local, mine, rows, width, S, b.code, b.packed, b, s);
            if (he != hipSuccess) status = eray_internal_error(ctx, ERAY_E_HIP, hipGetErrorString(he));
        }
        if (status != ERAY_OK && (he = hipMemsetAsync(b.count, 0xff, 4, s)) != hipSuccess)
            return eray_internal_error(ctx, ERAY_E_HIP, hipGetErrorString(he));
        r = ncclAllGather(b.count, b.counts, 1, ncclUint32, c, s);
        if (r != ncclSuccess) return nccl_error(ctx, "ncclAllGather", r);
        std::vector<uint32_t> counts((size_t)nranks);
        if ((he = hipMemcpyAsync(counts.data(), b.counts, 4u * (size_t)nranks, hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (he = hipStreamSynchronize(s)) != hipSuccess)
            return eray_internal_error(ctx, ERAY_E_HIP, hipGetErrorString(he));
        if (status != ERAY_OK) return status;
        for (int q = 0; q < nranks; ++q)
            if (counts[(size_t)q] == kCountFailed) {
                char msg[80];
                std::snprintf(msg, sizeof msg, "gather: rank %d could not use its buffers", q);
                return eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT, msg);
            }
        RankOffsets off{};
        for (int k = 1; k < nranks; ++k) off.v[k] = off.v[k - 1] + counts[(size_t)k - 1];
        if (nranks > 1) {
            if ((r = ncclGroupStart()) != ncclSuccess) return nccl_error(ctx, "ncclGroupStart", r);
            if (rank == 0) {
                for (int k = 1; k < nranks && r == ncclSuccess; ++k) {
                    r = ncclRecv(b.code + (size_t)k * G, G, ncclUint32, k, c, s);
                    if (r == ncclSuccess && counts[(size_t)k])
                        r = ncclRecv(b.packed + (size_t)off.v[k] * kSegBytes, (size_t)counts[(size_t)k] * kSegBytes,
                                     ncclUint8, k, c, s);
                }
            } else {
                r = ncclSend(b.code, G, ncclUint32, 0, c, s);
                if (r == ncclSuccess && counts[(size_t)rank])
                    r = ncclSend(b.packed, (size_t)counts[(size_t)rank] * kSegBytes, ncclUint8, 0, c, s);
            }
            const ncclResult_t r2 = ncclGroupEnd();
            if (r != ncclSuccess) return nccl_error(ctx, "ncclSend/ncclRecv", r);
            if (r2 != ncclSuccess) return nccl_error(ctx, "ncclGroupEnd", r2);
        }
        if (rank == 0) {
            seg_decode_kernel<<<height, 256, 0, s>>>(b.code, b.packed, off, frame, height, width, S, band_rows,
                                                     (uint32_t)nranks, rows);
            if ((he = hipGetLastError()) != hipSuccess) return eray_internal_error(ctx, ERAY_E_HIP, hipGetErrorString(he));
        }
        return ERAY_OK;
    }
}

}  // extern "C"

namespace {
// Every rank's verdict on a plan exchange from the same records (so all accept the plan or all
// fail together): the first rank's failure, or a source other than this rank's.  status: this
// rank's own verdict (its message already set).
int plan_verdict(eray_ctx* ctx, const int32_t* all, int nranks, int status, const int32_t* mine) {
    for (int q = 0; q < nranks; ++q) {
        const int32_t* o = all + (size_t)q * kXchgInts;
        if (o[0] != ERAY_OK) {
            if (status != ERAY_OK) return status;
            char msg[128];
            std::snprintf(msg, sizeof msg, "scene-camera gather: rank %d could not use its frames (status %d)", q, o[0]);
            return eray_internal_error(ctx, o[0], msg);
        }
    }
    if (status != ERAY_OK) return status;
    for (int q = 0; q < nranks; ++q) {
        const int32_t* o = all + (size_t)q * kXchgInts;
        if (o[1] != mine[1] || o[2] != mine[2] || o[3] != mine[3])
            return eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT,
                                       "scene-camera gather: the ranks' frames come from different cameras or paths");
    }
    return ERAY_OK;
}

// Exchanges the ranks' records for a new plan (a collective: every rank calls it at the same
// point, one stream synchronisation).  `status` is this rank's verdict (ERAY_OK, or the error it
// met looking up its frames' source and rectangles); on success every rank holds every rank's
// layout, otherwise every rank returns an error.
int exchange_plan(eray_ctx* ctx, ncclComm_t c, int nranks, int rank, uint32_t H, uint32_t W, uint32_t band,
                  const eray::gpu::FrameSource& src, int status, const std::vector<std::array<int32_t, 4>>& rects,
                  GatherPlan* P) {
    P->valid = false;
    P->batches.clear();
    hipStream_t s = (hipStream_t)eray_get_stream(ctx);
    hipError_t he;
    // (the records travel through the context's collective scratch: nothing to allocate before
    // the all-gather, so this rank always takes part)
    int32_t* xchg = reinterpret_cast<int32_t*>(eray_internal_coll_scratch(ctx) + kScrXchg);
    if (status == ERAY_OK && !P->fault) {  // the roots' fault word (a failure here is this rank's verdict)
        if (hipHostMalloc((void**)&P->fault, sizeof(int32_t), hipHostMallocMapped) != hipSuccess ||
            hipHostGetDevicePointer((void**)&P->d_fault, P->fault, 0) != hipSuccess) {
            if (P->fault) (void)hipHostFree(P->fault);
            P->fault = P->d_fault = nullptr;
            status = eray_internal_error(ctx, ERAY_E_OUT_OF_MEMORY, "gather plan: fault word");
        } else {
            *P->fault = 0;
        }
    }
    if (status == ERAY_OK && !P->asm_ev && hipEventCreateWithFlags(&P->asm_ev, hipEventDisableTiming) != hipSuccess) {
        P->asm_ev = nullptr;
        status = eray_internal_error(ctx, ERAY_E_HIP, "gather plan: assembly event");
    }
    int32_t rec[kXchgInts] = {};
    rec[0] = status;
    rec[1] = (int32_t)src.kind;
    rec[2] = (int32_t)(uint32_t)src.key;
    rec[3] = (int32_t)(uint32_t)(src.key >> 32);
    if (status == ERAY_OK) write_rects(my_rects(rects, rank_rows(H, band, (uint32_t)nranks, (uint32_t)rank), W), rec + kXchgHead);
    std::vector<int32_t> all((size_t)kXchgInts * (size_t)nranks);
    if ((he = hipMemcpyAsync(xchg, rec, sizeof rec, hipMemcpyHostToDevice, s)) != hipSuccess)
        return eray_internal_error(ctx, ERAY_E_HIP, hipGetErrorString(he));
    const ncclResult_t r = ncclAllGather(xchg, xchg + kXchgInts, kXchgInts, ncclInt32, c, s);
    if (r != ncclSuccess) return nccl_error(ctx, "ncclAllGather (gather plan)", r);
    if ((he = hipMemcpyAsync(all.data(), xchg + kXchgInts, sizeof(int32_t) * all.size(), hipMemcpyDeviceToHost, s)) !=
            hipSuccess ||
        (he = hipStreamSynchronize(s)) != hipSuccess)
        return eray_internal_error(ctx, ERAY_E_HIP, hipGetErrorString(he));
    if (int st = plan_verdict(ctx, all.data(), nranks, status, rec)) return st;
    P->ranks.assign((size_t)nranks, RankLayout{});
    P->total = 0;
    for (int q = 0; q < nranks; ++q) {
        RankLayout R = layout_of(all.data() + (size_t)q * kXchgInts + kXchgHead,
                                 rank_rows(H, band, (uint32_t)nranks, (uint32_t)q).rows);
        R.off = P->total;
        P->total += R.bytes;
        P->ranks[(size_t)q] = R;
    }
    // the rank table lives in the scratch: the previous plan's assemblies (on any stream) read it
    // until they finish, so the device drains first (a re-plan is once per camera)
    P->d_ranks = reinterpret_cast<RankLayout*>(eray_internal_coll_scratch(ctx) + kScrRanks);
    if ((he = hipDeviceSynchronize()) != hipSuccess ||
        (he = hipMemcpy(P->d_ranks, P->ranks.data(), sizeof(RankLayout) * (size_t)nranks, hipMemcpyHostToDevice)) !=
            hipSuccess)
        return eray_internal_error(ctx, ERAY_E_HIP, hipGetErrorString(he));
    P->comm = (void*)c;
    P->kind = src.kind;
    P->key = src.key;
    P->H = H;
    P->W = W;
    P->band = band;
    P->nranks = (uint32_t)nranks;
    P->rank = (uint32_t)rank;
    P->valid = true;
    return ERAY_OK;
}

// The plan's transfer buffer grown to `bytes` (the first call of a batch size): the new buffer is
// allocated before the old one is released, so a failure leaves the plan as it was.
int grow(eray_ctx* ctx, GatherPlan* P, size_t bytes) {
    if (bytes <= P->buf_cap && P->buf) return ERAY_OK;
    hipStream_t s = (hipStream_t)eray_get_stream(ctx);
    uint8_t* nb = nullptr;
    hipError_t he = hipDeviceSynchronize();  // (the old buffer's transfers are done, on whichever stream)
    if (he == hipSuccess) he = hipMalloc((void**)&nb, std::max<size_t>(bytes, 256));
    if (he != hipSuccess) return eray_internal_error(ctx, ERAY_E_OUT_OF_MEMORY, hipGetErrorString(he));
    if (P->buf) (void)hipFree(P->buf);
    P->buf = nb;
    P->buf_cap = std::max<size_t>(bytes, 256);
    return ERAY_OK;
}

// One rank's part of a batch of B frames: where its packs go in its buffer, how much buffer it
// needs, and its point-to-point transfers (offsets into the buffer).  Its receive area holds, for
// each of the `mine` frames it assembles, every rank's pack and then that rank's header (rank q's
// block at recv_block: mine * off_q + 16 q, frame j at + j * bytes_q, the layout
// gather_assemble_kernel reads); its send area the frames of the other roots, grouped by root,
// each group followed by this rank's header, so each (rank, root) pair is one transfer.
struct Xfer {
    uint32_t peer;
    bool send;
    size_t off, bytes;
};
struct Schedule {
    Roots R;
    uint32_t mine;             // frames this rank assembles
    size_t send_base, own;     // its send area; its own packs' block in the receive area
    size_t need;               // buffer bytes
    std::vector<Xfer> ops;
    HeaderSpots hdr;           // where this rank writes its header (after each send group, after its own packs)
    std::vector<uint64_t> peer_hdr;  // per rank: its header in this rank's receive area (~0: not used)
};
Schedule schedule(const std::vector<RankLayout>& ranks, uint64_t total, uint32_t rank, uint32_t B, bool rotate) {
    Schedule S;
    const uint32_t N = (uint32_t)ranks.size();
    S.R = Roots{B, rotate ? N : 0u};
    S.mine = S.R.count(rank);
    const RankLayout& me = ranks[rank];
    S.send_base = (size_t)S.mine * total + kHdr * N;
    S.own = recv_block(me, rank, S.mine);
    S.hdr.n = 0;
    S.peer_hdr.assign(N, ~0ull);
    size_t groups = 0;
    for (uint32_t q = 0; q < N; ++q) {
        if (q != rank && S.R.count(q) && me.bytes) {
            const size_t off = S.send_base + (size_t)(S.R.before(q) - (q > rank ? S.mine : 0u)) * me.bytes +
                               kHdr * S.R.group(q, rank);
            const size_t bytes = (size_t)S.R.count(q) * me.bytes;
            S.ops.push_back({q, true, off, bytes + kHdr});
            S.hdr.off[S.hdr.n++] = off + bytes;
            ++groups;
        }
        if (S.mine && ranks[q].bytes) {
            const size_t off = recv_block(ranks[q], q, S.mine), bytes = (size_t)S.mine * ranks[q].bytes;
            if (q != rank) S.ops.push_back({q, false, off, bytes + kHdr});
            S.peer_hdr[q] = off + bytes;
        }
    }
    if (S.mine) S.hdr.off[S.hdr.n++] = S.own + (size_t)S.mine * me.bytes;
    S.need = S.send_base + (size_t)(B - S.mine) * me.bytes + kHdr * groups;
    return S;
}

// Pack (every rank), transfer, assemble (each frame's root) `B` frames with plan P.  status != OK
// (this rank's own arguments are unusable): its headers carry the status and it runs only the
// plan's transfers, so the other ranks' matching sends and receives complete and their roots
// refuse the batch — no kernel touches the caller's buffers.
int scene_gather(eray_ctx* ctx, ncclComm_t c, GatherPlan& P, const Schedule& S, const uint8_t* local,
                 uint64_t local_stride, uint8_t* frames, uint64_t frame_stride, uint32_t B, int status = ERAY_OK) {
    hipStream_t s = (hipStream_t)eray_get_stream(ctx);
    const RankLayout& me = P.ranks[P.rank];
    const bool fail_safe = status != ERAY_OK;
    hipError_t he;
    if (S.hdr.n) {
        const XferHeader h{status, P.kind, (uint32_t)P.key, (uint32_t)(P.key >> 32)};
        gather_header_kernel<<<1, 64, 0, s>>>(P.buf, S.hdr, h);
        if ((he = hipGetLastError()) != hipSuccess) return eray_internal_error(ctx, ERAY_E_HIP, hipGetErrorString(he));
    }
    if (me.bytes && !fail_safe) {
        gather_pack_kernel<<<dim3(me.packed_rows, B), 256, 0, s>>>(local, local_stride, P.buf + S.send_base,
                                                                   P.buf + S.own, me, P.W, S.R, P.rank);
        if ((he = hipGetLastError()) != hipSuccess) return eray_internal_error(ctx, ERAY_E_HIP, hipGetErrorString(he));
    }
    if (!S.ops.empty()) {
        ncclResult_t r = ncclGroupStart();
        if (r != ncclSuccess) return nccl_error(ctx, "ncclGroupStart", r);
        for (size_t i = 0; i < S.ops.size() && r == ncclSuccess; ++i) {
            const Xfer& x = S.ops[i];
            r = x.send ? ncclSend(P.buf + x.off, x.bytes, ncclUint8, (int)x.peer, c, s)
                       : ncclRecv(P.buf + x.off, x.bytes, ncclUint8, (int)x.peer, c, s);
        }
        const ncclResult_t r2 = ncclGroupEnd();
        if (r != ncclSuccess) return nccl_error(ctx, "ncclSend/ncclRecv", r);
        if (r2 != ncclSuccess) return nccl_error(ctx, "ncclGroupEnd", r2);
    }
    if (S.mine && !fail_safe) {
        gather_assemble_kernel<<<dim3(P.H, S.mine), 256, 0, s>>>(P.buf, P.d_ranks, S.mine, frames, frame_stride, P.H, P.W,
                                                                 P.band, P.nranks, P.kind, P.key, P.d_fault);
        if ((he = hipGetLastError()) != hipSuccess) return eray_internal_error(ctx, ERAY_E_HIP, hipGetErrorString(he));
        // the next call reads the fault word once this assembly is done (not under a graph capture,
        // whose replays' refusals the first call after them reads)
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(s, &cap) == hipSuccess && cap == hipStreamCaptureStatusNone &&
            hipEventRecord(P.asm_ev, s) == hipSuccess)
            P.asm_pending = true;
    }
    return ERAY_OK;
}

// The re-plan decision of eray_gather_frames' scene-camera transport.  Its inputs are the state
// every rank holds alike when the ranks make the same calls (SPMD): the shared arguments, whether
// the cached plan was made for them (by an exchange whose verdict every rank shares), and the
// context's latest scene-camera or camera-path render — never this rank's own buffers or their
// tags, so a rank whose `local` is unusable enters the same collectives as its peers.
bool gather_replan(bool cached, uint32_t plan_kind, uint64_t plan_key, uint32_t cur_kind, uint64_t cur_key) {
    return !cached || plan_kind != cur_kind || plan_key != cur_key;
}
}  // namespace

extern "C" {

int eray_gather_frames(eray_ctx* ctx, void* nccl_comm, const uint8_t* local, uint64_t local_stride, uint8_t* frames,
                       uint64_t frame_stride, uint32_t nframes, uint32_t height, uint32_t width, uint32_t band_rows,
                       uint32_t flags) {
    if (!ctx || !nccl_comm) return eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT, "gather: null context or comm");
    if (flags & ~(uint32_t)(ERAY_GATHER_SCENE_CAMERA | ERAY_GATHER_ROTATE_ROOT))
        return eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT, "gather: unknown flags");
    const bool rotate = (flags & ERAY_GATHER_ROTATE_ROOT) != 0;
    if (rotate && !(flags & ERAY_GATHER_SCENE_CAMERA))
        return eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT, "gather: rotating roots need ERAY_GATHER_SCENE_CAMERA");
    if (int st = eray_internal_use_device(ctx)) return st;
    ncclComm_t c = (ncclComm_t)nccl_comm;
    int nranks = 0, rank = 0;
    ncclResult_t r = ncclCommCount(c, &nranks);
    if (r == ncclSuccess) r = ncclCommUserRank(c, &rank);
    if (r != ncclSuccess) return nccl_error(ctx, "gather: communicator", r);
    if (!nframes || !height || !width) return ERAY_OK;
    const bool rows_ok = band_rows ? band_rows >= 4 && !(band_rows & (band_rows - 1)) : height % (uint32_t)nranks == 0;
    if (flags & ERAY_GATHER_SCENE_CAMERA) {
        // The transport is chosen from arguments every rank shares (flags, the frame size, the
        // split), never from this rank's own pointers or state, so all ranks take the same path.
        if (width % 16 || !rows_ok)
            return eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT,
                                       "scene-camera gather: width must be a multiple of 16 and the rows a valid split");
        if (nranks > kMaxCodedRanks)
            return eray_internal_error(ctx, ERAY_E_UNSUPPORTED, "scene-camera gather: more than 64 ranks");
        // This rank's verdict on its own arguments and frames.  Whatever it is, the rank takes
        // part in the same collectives as the others (chosen from the shared arguments and the
        // shared render history, gather_replan), then returns its error.
        const bool assembles = rotate ? (uint32_t)rank < nframes : rank == 0;
        const bool aligned = ((reinterpret_cast<uintptr_t>(local) | local_stride) & 15) == 0 &&
                             (!assembles || ((reinterpret_cast<uintptr_t>(frames) | frame_stride) & 15) == 0);
        int status = ERAY_OK;
        if (!local || (assembles && !frames) || !aligned)
            status = eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT,
                                         "scene-camera gather: null or unaligned (16 B) buffers or strides");
        // what the plan is for: the context's latest render of the scene camera or of a camera path
        eray::gpu::FrameSource cur;
        eray_internal_gather_source(ctx, &cur);
        if (status == ERAY_OK && cur.kind != eray::gpu::kSrcScene && cur.kind != eray::gpu::kSrcPath)
            status = eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT,
                                         "scene-camera gather: this context has rendered neither its scene camera nor a "
                                         "camera path");
        // this rank's frames must be frames of that render, over this rank's share
        eray::gpu::FrameSource src;
        if (status == ERAY_OK) status = eray_internal_frame_source(ctx, local, local_stride, nframes, &src);
        if (status == ERAY_OK && (src.kind != cur.kind || src.key != cur.key))
            status = eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT,
                                         "scene-camera gather: the frames are not of this context's latest scene-camera "
                                         "or camera-path render");
        const RankRows rr = rank_rows(height, band_rows, (uint32_t)nranks, (uint32_t)rank);
        if (status == ERAY_OK && (src.W != width || src.H != height || src.row0 != rr.row0 || src.rows != rr.rows ||
                                  src.band_shift != rr.shift || (band_rows && src.band_stride != rr.stride)))
            status = eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT,
                                         "scene-camera gather: the frames cover other rows or another frame size than "
                                         "this rank's share");
        GatherPlan*& P = *reinterpret_cast<GatherPlan**>(eray_internal_gather_plan(ctx, plan_free));
        if (!P) P = new (std::nothrow) GatherPlan();
        if (!P) {  // no plan object: this rank still takes part in the (first) exchange, with its error
            GatherPlan tmp;
            eray_internal_error(ctx, ERAY_E_OUT_OF_MEMORY, "gather plan");
            const int st = exchange_plan(ctx, c, nranks, rank, height, width, band_rows, cur, ERAY_E_OUT_OF_MEMORY, {}, &tmp);
            plan_release(tmp);
            return st ? st : ERAY_E_OUT_OF_MEMORY;
        }
        hipStream_t s = (hipStream_t)eray_get_stream(ctx);
        // a failed or foreign batch met by one of this context's earlier assemblies: read once that
        // assembly is done (reported after this call's own collectives)
        bool faulted = false;
        if (P->fault) {
            hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
            const bool capturing = hipStreamIsCapturing(s, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone;
            if (P->asm_pending && !capturing) {
                const hipError_t he = hipEventSynchronize(P->asm_ev);
                if (he != hipSuccess && status == ERAY_OK)
                    status = eray_internal_error(ctx, ERAY_E_HIP, hipGetErrorString(he));
                P->asm_pending = false;
            }
            if (!P->asm_pending) faulted = __atomic_exchange_n(P->fault, 0, __ATOMIC_RELAXED) != 0;
        }
        const bool cached = P->valid && P->comm == (void*)c && P->H == height && P->W == width &&
                            P->band == band_rows && P->nranks == (uint32_t)nranks && P->rank == (uint32_t)rank;
        if (gather_replan(cached, P->kind, P->key, cur.kind, cur.key)) {  // a new plan: every rank exchanges
            eray::gpu::SceneLayout L;
            if (status == ERAY_OK) status = eray_internal_source_layout(ctx, src, &L);
            if (int st = exchange_plan(ctx, c, nranks, rank, height, width, band_rows, cur, status, L.rects, P)) return st;
        }
        const Schedule S = schedule(P->ranks, P->total, (uint32_t)rank, nframes, rotate);
        if (std::find(P->batches.begin(), P->batches.end(), nframes) == P->batches.end()) {
            // a batch size's first call: every rank's transfer buffer for it, agreed on before any
            // transfer (a rank that cannot allocate makes every rank return instead of leaving its
            // peers' sends and receives waiting)
            std::string keep = status != ERAY_OK ? eray_last_error(ctx) : std::string();
            const int gst = grow(ctx, P, S.need);
            if (status != ERAY_OK) eray_internal_error(ctx, status, keep.c_str());  // (the first failure's message)
            if (int st = agree(ctx, c, nranks, gst, "scene-camera gather: transfer buffer")) return status ? status : st;
            P->batches.push_back(nframes);
        }
        std::string msg = status != ERAY_OK ? eray_last_error(ctx) : std::string();
        const int st = scene_gather(ctx, c, *P, S, local, local_stride, frames, frame_stride, nframes, status);
        if (status != ERAY_OK) return eray_internal_error(ctx, status, msg.c_str());
        if (st) return st;
        if (S.mine) eray_internal_untag(ctx, frames, (size_t)(S.mine - 1) * frame_stride + (size_t)height * width * 3u);
        if (faulted)
            return eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT,
                                       "scene-camera gather: an earlier batch assembled here had a rank that could not "
                                       "use its frames; its frames were left unwritten");
        return ERAY_OK;
    }
    for (uint32_t k = 0; k < nframes; ++k)  // one frame at a time through eray_gather_rows
        if (int st = eray_gather_rows(ctx, nccl_comm, local ? local + k * local_stride : nullptr,
                                      frames ? frames + k * frame_stride : nullptr, height, width, band_rows))
            return st;
    return ERAY_OK;
}

// Diagnostics (tests, host only): rank `rank`'s share of the scene-camera gather of `nranks` ranks
// for objects whose pixel rectangles are `rects` (n x (x0, x1, y0, y1), camera rows) — the layout
// exchange_plan builds from that rank's record.  out (4 + 8 * 8 words): rows, nrect, bytes per
// frame, packed rows, then per rectangle l0, l1, c0, c1 (local rows, 16-pixel column groups), its
// byte offset in the rank's per-frame pack, its row bytes, its first packed row, 0.
int eray_debug_gather_layout(const int32_t* rects, uint32_t n, uint32_t height, uint32_t width, uint32_t band_rows,
                             uint32_t nranks, uint32_t rank, uint32_t* out) {
    if ((n && !rects) || !out || !nranks || rank >= nranks || width % 16 ||
        (band_rows && (band_rows < 4 || (band_rows & (band_rows - 1)))) || (!band_rows && height % nranks))
        return eray_internal_error(nullptr, ERAY_E_INVALID_ARGUMENT, "gather layout: bad arguments");
    std::vector<std::array<int32_t, 4>> rs;
    for (uint32_t i = 0; i < n; ++i) rs.push_back({rects[4 * i], rects[4 * i + 1], rects[4 * i + 2], rects[4 * i + 3]});
    const RankRows rr = rank_rows(height, band_rows, nranks, rank);
    int32_t rec[kXchgInts - kXchgHead] = {};
    write_rects(my_rects(rs, rr, width), rec);
    const RankLayout R = layout_of(rec, rr.rows);
    std::memset(out, 0, sizeof(uint32_t) * (4 + 8 * kPlanRects));
    out[0] = R.rows;
    out[1] = R.nrect;
    out[2] = R.bytes;
    out[3] = R.packed_rows;
    for (uint32_t i = 0; i < R.nrect; ++i) {
        const GatherRect& g = R.r[i];
        const uint32_t v[8] = {(uint32_t)g.l0, (uint32_t)g.l1, (uint32_t)g.c0, (uint32_t)g.c1, g.off, g.row_bytes, g.first, 0u};
        std::memcpy(out + 4 + 8 * i, v, sizeof v);
    }
    return ERAY_OK;
}

}  // extern "C"

namespace {
// The schedule of eray_debug_gather_* for packs of rank_bytes[q] bytes per frame (no plan).
Schedule debug_schedule(const uint32_t* rank_bytes, uint32_t nranks, uint32_t rank, uint32_t nframes, uint32_t rotate,
                        std::vector<RankLayout>* ranks_out = nullptr) {
    std::vector<RankLayout> ranks(nranks, RankLayout{});
    uint64_t total = 0;
    for (uint32_t q = 0; q < nranks; ++q) {
        ranks[q].bytes = rank_bytes[q];
        ranks[q].off = total;
        total += rank_bytes[q];
    }
    if (ranks_out) *ranks_out = ranks;
    return schedule(ranks, total, rank, nframes, rotate != 0);
}
bool debug_schedule_args(const uint32_t* rank_bytes, uint32_t nranks, uint32_t rank) {
    return rank_bytes && nranks && nranks <= (uint32_t)kMaxCodedRanks && rank < nranks;
}
}  // namespace

extern "C" {

// Diagnostics (tests, host only): rank `rank`'s schedule for a batch of `nframes` frames when the
// ranks' packs are rank_bytes[q] bytes per frame (rank order = receive-area order) — what
// eray_gather_frames' pack kernel and point-to-point transfers do.  out (u64): buffer bytes,
// frames this rank assembles, number of transfers T; then per frame k its pack's offset in the
// buffer; then per rank q where q's packs of this rank's frames start (frame j: + j * bytes_q);
// then per transfer: peer, 1 = send / 0 = receive, offset, bytes (each transfer ends with its
// sender's 16-B header); then the number of headers this rank writes and their offsets (T + 1
// slots); then per rank q the offset of q's header in this rank's receive area (~0: unused).
int eray_debug_gather_schedule(const uint32_t* rank_bytes, uint32_t nranks, uint32_t rank, uint32_t nframes,
                               uint32_t rotate, uint64_t* out, uint32_t cap) {
    if (!debug_schedule_args(rank_bytes, nranks, rank) || !out || cap < 5u + nframes + 12u * nranks)
        return eray_internal_error(nullptr, ERAY_E_INVALID_ARGUMENT, "gather schedule: bad arguments");
    std::vector<RankLayout> ranks;
    const Schedule S = debug_schedule(rank_bytes, nranks, rank, nframes, rotate, &ranks);
    const uint64_t bytes = rank_bytes[rank];
    out[0] = S.need;
    out[1] = S.mine;
    out[2] = S.ops.size();
    for (uint32_t k = 0; k < nframes; ++k) {
        const uint32_t r = S.R.root(k);
        out[3 + k] = r == rank ? S.own + S.R.index(k) * bytes
                               : S.send_base + S.R.send_slot(k, rank) * bytes + (bytes ? kHdr * S.R.group(r, rank) : 0);
    }
    for (uint32_t q = 0; q < nranks; ++q) out[3 + nframes + q] = recv_block(ranks[q], q, S.mine);
    uint64_t* o = out + 3 + nframes + nranks;
    for (const Xfer& x : S.ops) {
        o[0] = x.peer;
        o[1] = x.send ? 1u : 0u;
        o[2] = x.off;
        o[3] = x.bytes;
        o += 4;
    }
    *o++ = S.hdr.n;
    for (uint32_t i = 0; i < S.hdr.n; ++i) *o++ = S.hdr.off[i];
    for (uint32_t q = 0; q < nranks; ++q) *o++ = S.peer_hdr[q];
    return ERAY_OK;
}

// Diagnostics (tests, host only): the headers rank `rank` writes into its transfer buffer `buf`
// (host memory of the schedule's size) — its verdict `status` and its frames' source (kind, key).
int eray_debug_gather_write_headers(const uint32_t* rank_bytes, uint32_t nranks, uint32_t rank, uint32_t nframes,
                                    uint32_t rotate, int32_t status, uint32_t kind, uint64_t key, uint8_t* buf) {
    if (!debug_schedule_args(rank_bytes, nranks, rank) || !buf)
        return eray_internal_error(nullptr, ERAY_E_INVALID_ARGUMENT, "gather headers: bad arguments");
    const Schedule S = debug_schedule(rank_bytes, nranks, rank, nframes, rotate);
    const XferHeader h{status, kind, (uint32_t)key, (uint32_t)(key >> 32)};
    for (uint32_t i = 0; i < S.hdr.n; ++i) std::memcpy(buf + S.hdr.off[i], &h, kHdr);
    return ERAY_OK;
}

// Diagnostics (tests, host only): a root's verdict on its received batch (gather_assemble_kernel's
// check, on a host copy of its buffer): ERAY_OK when every header it uses says ERAY_OK and the
// plan's source (kind, key), else ERAY_E_INVALID_ARGUMENT (the root writes none of the frames).
int eray_debug_gather_check(const uint32_t* rank_bytes, uint32_t nranks, uint32_t rank, uint32_t nframes,
                            uint32_t rotate, uint32_t kind, uint64_t key, const uint8_t* buf) {
    if (!debug_schedule_args(rank_bytes, nranks, rank) || !buf)
        return eray_internal_error(nullptr, ERAY_E_INVALID_ARGUMENT, "gather check: bad arguments");
    const Schedule S = debug_schedule(rank_bytes, nranks, rank, nframes, rotate);
    for (uint32_t q = 0; q < nranks; ++q) {
        if (S.peer_hdr[q] == ~0ull) continue;
        XferHeader h;
        std::memcpy(&h, buf + S.peer_hdr[q], kHdr);
        if (!header_ok(h, kind, key))
            return eray_internal_error(nullptr, ERAY_E_INVALID_ARGUMENT, "gather: a rank could not use its frames");
    }
    return ERAY_OK;
}

// Diagnostics (tests, host only): a new plan's verdict on this rank (exchange_plan's): records
// holds every rank's (status, kind, key low, key high), `rank`'s own among them.
// Diagnostics (tests, host only): eray_gather_frames' re-plan decision (gather_replan) — from the
// cached plan's state and the context's latest render, the only inputs it has.
int eray_debug_gather_replan(uint32_t cached, uint32_t plan_kind, uint64_t plan_key, uint32_t cur_kind, uint64_t cur_key) {
    return gather_replan(cached != 0, plan_kind, plan_key, cur_kind, cur_key) ? 1 : 0;
}

int eray_debug_plan_verdict(const int32_t* records, uint32_t nranks, uint32_t rank) {
    if (!records || !nranks || nranks > (uint32_t)kMaxCodedRanks || rank >= nranks)
        return eray_internal_error(nullptr, ERAY_E_INVALID_ARGUMENT, "plan verdict: bad arguments");
    std::vector<int32_t> all((size_t)kXchgInts * nranks, 0);
    for (uint32_t q = 0; q < nranks; ++q) std::memcpy(all.data() + (size_t)q * kXchgInts, records + 4 * q, 4 * sizeof(int32_t));
    const int32_t* mine = all.data() + (size_t)rank * kXchgInts;
    if (mine[0] != ERAY_OK) eray_internal_error(nullptr, mine[0], "plan verdict: this rank's own failure");
    return plan_verdict(nullptr, all.data(), (int)nranks, mine[0], mine);
}

// Diagnostics (tests): the scene-camera gather of a batch of `nframes` frames by N ranks,
// simulated on one GPU with the real pack and assembly kernels and each rank's schedule (its
// point-to-point transfers as device copies between the ranks' buffers).  The context has
// rendered the scene camera's whole frame (its setup's rectangles stand for every rank's);
// staging holds frame k of rank q's padded local PPM block at (k * N + q) * rows_max rows
// (rows_max = rank 0's rows; band_rows > 0: bands, 0: blocks).  Root r's assembled frames land at
// frames + (frames of roots below r + j) * H W 3 — in batch order unless `rotate`.
int eray_debug_scene_gather_batch(eray_ctx* ctx, const uint8_t* staging, uint8_t* frames, uint32_t nframes,
                                  uint32_t height, uint32_t width, uint32_t band_rows, uint32_t nranks, uint32_t rotate) {
    if (!ctx || !staging || !frames || !nframes || !nranks || nranks > (uint32_t)kMaxCodedRanks || width % 16 ||
        (band_rows && (band_rows < 4 || (band_rows & (band_rows - 1)))) || (!band_rows && height % nranks))
        return eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT, "scene gather: bad arguments");
    eray::gpu::FrameSource src;
    eray::gpu::SceneLayout L;
    if (int st = eray_internal_scene_setup_source(ctx, &src)) return st;
    if (int st = eray_internal_source_layout(ctx, src, &L)) return st;
    if (src.W != width || src.H != height || src.row0 != 0 || src.rows != height || src.band_shift != 31u)
        return eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT, "scene gather: render the whole scene-camera frame first");
    GatherPlan P;
    P.H = height;
    P.W = width;
    P.band = band_rows;
    P.nranks = nranks;
    P.rank = 0;
    P.kind = src.kind;
    P.key = src.key;
    const uint32_t rows_max = rank_rows(height, band_rows, nranks, 0).rows;
    for (uint32_t q = 0; q < nranks; ++q) {
        const RankRows rr = rank_rows(height, band_rows, nranks, q);
        int32_t rec[kXchgInts - kXchgHead] = {};
        write_rects(my_rects(L.rects, rr, width), rec);
        RankLayout R = layout_of(rec, rr.rows);
        R.off = P.total;
        P.total += R.bytes;
        P.ranks.push_back(R);
    }
    std::vector<Schedule> S;
    std::vector<size_t> base;  // rank q's buffer inside P.buf
    size_t all = 0;
    for (uint32_t q = 0; q < nranks; ++q) {
        S.push_back(schedule(P.ranks, P.total, q, nframes, rotate != 0));
        base.push_back(all);
        all += (S.back().need + 255) & ~(size_t)255;
    }
    const size_t block = (size_t)rows_max * width * 3u, frame_bytes = (size_t)height * width * 3u;
    hipStream_t s = (hipStream_t)eray_get_stream(ctx);
    hipError_t he = hipMalloc((void**)&P.d_ranks, sizeof(RankLayout) * nranks);
    if (he == hipSuccess) he = hipMalloc((void**)&P.buf, std::max<size_t>(all, 256));
    if (he == hipSuccess) he = hipMalloc((void**)&P.d_fault, sizeof(int32_t));
    if (he == hipSuccess) he = hipMemsetAsync(P.d_fault, 0, sizeof(int32_t), s);
    const XferHeader hdr{ERAY_OK, P.kind, (uint32_t)P.key, (uint32_t)(P.key >> 32)};
    for (uint32_t q = 0; q < nranks && he == hipSuccess; ++q) {  // every rank's headers
        if (!S[q].hdr.n) continue;
        gather_header_kernel<<<1, 64, 0, s>>>(P.buf + base[q], S[q].hdr, hdr);
        he = hipGetLastError();
    }
    if (he == hipSuccess)
        he = hipMemcpyAsync(P.d_ranks, P.ranks.data(), sizeof(RankLayout) * nranks, hipMemcpyHostToDevice, s);
    for (uint32_t q = 0; q < nranks && he == hipSuccess; ++q) {  // every rank packs its frames
        const RankLayout& R = P.ranks[q];
        if (!R.bytes) continue;
        gather_pack_kernel<<<dim3(R.packed_rows, nframes), 256, 0, s>>>(staging + q * block, nranks * block,
                                                                        P.buf + base[q] + S[q].send_base,
                                                                        P.buf + base[q] + S[q].own, R, width, S[q].R, q);
        he = hipGetLastError();
    }
    for (uint32_t q = 0; q < nranks && he == hipSuccess; ++q)  // each send meets its peer's receive
        for (const Xfer& x : S[q].ops) {
            if (!x.send) continue;
            const Xfer* m = nullptr;
            for (const Xfer& y : S[x.peer].ops)
                if (!y.send && y.peer == q) m = &y;
            if (!m || m->bytes != x.bytes) {
                he = hipErrorInvalidValue;
                break;
            }
            he = hipMemcpyAsync(P.buf + base[x.peer] + m->off, P.buf + base[q] + x.off, x.bytes, hipMemcpyDeviceToDevice, s);
            if (he != hipSuccess) break;
        }
    for (uint32_t r = 0; r < nranks && he == hipSuccess; ++r) {  // every root assembles its frames
        if (!S[r].mine) continue;
        gather_assemble_kernel<<<dim3(height, S[r].mine), 256, 0, s>>>(P.buf + base[r], P.d_ranks, S[r].mine,
                                                                       frames + S[r].R.before(r) * frame_bytes,
                                                                       frame_bytes, height, width, band_rows, nranks,
                                                                       P.kind, P.key, P.d_fault);
        he = hipGetLastError();
    }
    int32_t fault = 0;
    if (he == hipSuccess) he = hipMemcpyAsync(&fault, P.d_fault, sizeof fault, hipMemcpyDeviceToHost, s);
    if (he == hipSuccess) he = hipStreamSynchronize(s);
    if (P.d_fault) (void)hipFree(P.d_fault);
    P.d_fault = nullptr;  // (not the mapped word plan_release frees)
    if (P.d_ranks) (void)hipFree(P.d_ranks);  // (this plan's own table, not the context's scratch)
    plan_release(P);
    if (he != hipSuccess) return eray_internal_error(ctx, ERAY_E_HIP, hipGetErrorString(he));
    return fault ? eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT, "scene gather: a root refused its batch") : ERAY_OK;
}

// One frame of eray_debug_scene_gather_batch (staging: the N ranks' blocks; frame: rank 0's).
int eray_debug_scene_gather(eray_ctx* ctx, const uint8_t* staging, uint8_t* frame, uint32_t height, uint32_t width,
                            uint32_t band_rows, uint32_t nranks) {
    return eray_debug_scene_gather_batch(ctx, staging, frame, 1, height, width, band_rows, nranks, 0);
}

}  // extern "C"

extern "C" {

// Diagnostics (tests): the coded banded gather of N ranks on one GPU — staging holds the N ranks'
// padded local PPM blocks; each is encoded into rank 0's code / packed layout as the point-to-
// point transfers would leave it, then decoded into frame.
int eray_debug_coded_unband(eray_ctx* ctx, const uint8_t* staging, uint8_t* frame, uint32_t height, uint32_t width,
                            uint32_t band_rows, uint32_t nranks) {
    if (!ctx || !staging || !frame || !band_rows || band_rows % 4 || !nranks || nranks > (uint32_t)kMaxCodedRanks)
        return eray_internal_error(ctx, ERAY_E_INVALID_ARGUMENT, "coded unband: bad arguments");
    if (!height || !width) return ERAY_OK;
    hipStream_t s = (hipStream_t)eray_get_stream(ctx);
    const uint32_t rows = band_rows_of(height, band_rows, nranks, 0);
    const uint32_t S = (width + kSegPx - 1) / kSegPx, G = rows * S;
    CodedBufs b;
    b.count = reinterpret_cast<uint32_t*>(eray_internal_coll_scratch(ctx) + kScrWords);
    if (!coded_bufs(ctx, G, nranks, &b))
        return eray_internal_error(ctx, ERAY_E_OUT_OF_MEMORY, "coded unband: staging buffer");
    RankOffsets off{};
    std::vector<uint32_t> counts(nranks);
    for (uint32_t k = 0; k < nranks; ++k) {
        if (k) off.v[k] = off.v[k - 1] + counts[k - 1];
        const uint8_t* local = staging + (size_t)k * rows * width * 3u;
        hipError_t e = encode_rows(local, band_rows_of(height, band_rows, nranks, k), rows, width, S,
                                   b.code + (size_t)k * G, b.packed + (size_t)off.v[k] * kSegBytes, b, s);
        if (e == hipSuccess) e = hipMemcpyAsync(&counts[k], b.count, 4, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return eray_internal_error(ctx, ERAY_E_HIP, hipGetErrorString(e));
    }
    seg_decode_kernel<<<height, 256, 0, s>>>(b.code, b.packed, off, frame, height, width, S, band_rows, nranks, rows);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? ERAY_OK : eray_internal_error(ctx, ERAY_E_HIP, hipGetErrorString(e));
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
