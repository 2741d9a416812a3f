// bins.hip — screen bins of a large object's faces for the frame kernel's primary-ray scan.
// A bin is one 16 x 4 pixel sub-block: exactly one wave's pixels.
//
// The per-face pixel rectangles (face_rect.hpp) say which pixel bins a face can be hit
// in.  For objects too large to scan per wave (> kDirectMax faces) the frame kernel reads, for
// its sub-block's bin, the list of those faces in INCREASING FACE INDEX (the reference's
// first-hit order, object.rs:63-78) and runs the exact culling + tests on that list only: a face
// outside the list cannot be hit by any ray of the bin, so the first hit is the reference's.
//
// Each entry also carries the bin's pixels the face may cover (bin_pixels: the four culling
// bounds solved per pixel row), so the frame kernel only tests (face, pixel) pairs that can hit.
//
// Built once per camera / geometry change (and per row phase of the rendered rows):
// each face's bin rectangle -> exclusive scan of the rectangles' areas (the (face, bin) pairs,
// face-major) -> pixel masks of all pairs, one thread per pair (balanced: a near-silhouette
// face's rectangle can span the frame's width, thousands of bins that one thread per face
// walked alone) -> the non-empty pairs compacted in pair order, i.e. (bin, position) in face
// order -> stable radix sort by bin (LSD: keeps face order within a bin) -> bin start offsets ->
// faces, pixel masks and intersection records gathered in bin order.
#include <algorithm>
#include <cstdlib>

#include <hipcub/hipcub.hpp>

#include "face_rect.hpp"
#include "internal.hpp"

namespace eray {
namespace gpu {
namespace {

// per face: its bin rectangle (face_rect; empty: x0 > x1) and the rectangle's number of bins
__global__ void __launch_bounds__(256) bin_range_kernel(const TriCull* __restrict__ cull, uint32_t T, uint32_t W,
                                                        uint32_t H, uint32_t phase, int4* __restrict__ range,
                                                        unsigned long long* __restrict__ area) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= T) return;
    int32_t r[4];
    int4 g = make_int4(1, 0, 1, 0);
    unsigned long long a = 0;
    if (face_rect(cull[i], W, H, r)) {
        // bin row of camera row y: (y + kBinH - phase) / kBinH
        g = make_int4(r[0] / (int32_t)kBinW, r[1] / (int32_t)kBinW,
                      (r[2] + (int32_t)kBinH - (int32_t)phase) / (int32_t)kBinH,
                      (r[3] + (int32_t)kBinH - (int32_t)phase) / (int32_t)kBinH);
        a = (unsigned long long)(g.y - g.x + 1) * (unsigned long long)(g.w - g.z + 1);
    }
    range[i] = g;
    area[i] = a;
}

// Pair j of [j0, j0 + len) (face-major, each face's bins row-major): its face (the last face
// whose first pair is <= j), bin and pixel mask.  emit == false: only the number of non-empty
// pairs, added to *nonempty; emit == true: the pair's mask, bin key and face, and a 0/1 flag.
template <bool emit>
__global__ void __launch_bounds__(256) bin_pairs_kernel(const TriCull* __restrict__ cull, const int4* __restrict__ range,
                                                        const unsigned long long* __restrict__ first, uint32_t T,
                                                        unsigned long long j0, uint32_t len, uint32_t W, uint32_t H,
                                                        uint32_t phase, uint32_t bins_x,
                                                        unsigned long long* __restrict__ nonempty,
                                                        unsigned long long* __restrict__ pmask,
                                                        uint32_t* __restrict__ pkey, uint32_t* __restrict__ pface,
                                                        uint32_t* __restrict__ pflag) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long m = 0;
    uint32_t key = 0, i = 0;
    if (k < len) {
        const unsigned long long j = j0 + k;
        uint32_t lo = 0, hi = T;  // first face whose first pair is > j
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (first[mid] <= j) lo = mid + 1;
            else hi = mid;
        }
        i = lo - 1;
        const int4 g = range[i];
        const uint32_t w = (uint32_t)(g.y - g.x + 1);
        const uint32_t c = (uint32_t)(j - first[i]);
        const uint32_t tx = (uint32_t)g.x + c % w, ty = (uint32_t)g.z + c / w;
        m = bin_pixels(cull[i], W, H, phase, tx, ty);
        key = ty * bins_x + tx;
    }
    if constexpr (emit) {
        if (k < len) {
            pmask[k] = m;
            pkey[k] = key;
            pface[k] = i;
            pflag[k] = m != 0;
        }
    } else {
        const unsigned long long b = __ballot(m != 0);
        if ((threadIdx.x & 63) == 0 && b) atomicAdd(nonempty, (unsigned long long)__popcll(b));
    }
}

// the non-empty pairs of a chunk at their compacted positions base + pos (pair order = face order)
__global__ void __launch_bounds__(256) bin_emit_kernel(const unsigned long long* __restrict__ pmask,
                                                       const uint32_t* __restrict__ pkey,
                                                       const uint32_t* __restrict__ pface,
                                                       const uint32_t* __restrict__ pflag,
                                                       const uint32_t* __restrict__ pos, uint32_t len, uint32_t base,
                                                       uint32_t* __restrict__ keys, uint32_t* __restrict__ order,
                                                       uint32_t* __restrict__ tri, unsigned long long* __restrict__ mask) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= len || !pflag[k]) return;
    const uint32_t o = base + pos[k];
    keys[o] = pkey[k];
    order[o] = o;  // emit positions increase with the face index
    tri[o] = pface[k];
    mask[o] = pmask[k];
}

// entries in bin order: face, pixel mask and intersection record
__global__ void __launch_bounds__(256) bin_gather_kernel(const uint32_t* __restrict__ order,
                                                         const uint32_t* __restrict__ tri_in,
                                                         const unsigned long long* __restrict__ mask_in,
                                                         const TriHot* __restrict__ hot, size_t n,
                                                         uint32_t* __restrict__ tri_out,
                                                         unsigned long long* __restrict__ mask_out,
                                                         TriHot* __restrict__ hot_out) {
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t pos = order[j];
    const uint32_t f = tri_in[pos];
    tri_out[j] = f;
    mask_out[j] = mask_in[pos];
    hot_out[j] = hot[f];
}

// start[t] = first position of bin t in the sorted keys (start[nbins] = n): one thread per bin,
// a lower bound over the keys (a thread per key filling the gap to the next key left the last
// thread walking every bin after the last non-empty one: 0.85 ms at 3840x2160)
__global__ void __launch_bounds__(256) bin_start_kernel(const uint32_t* __restrict__ keys, uint32_t n,
                                                        uint32_t nbins, uint32_t* __restrict__ start) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t > nbins) return;
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (keys[mid] < t) lo = mid + 1;
        else hi = mid;
    }
    start[t] = lo;
}

// The pixel rectangle of the non-empty bins (camera pixels), accumulated as tri_rect_kernel's:
// (~x0, x1 + 1, ~y0, y1 + 1) by atomicMax into zeroed words.
__global__ void __launch_bounds__(256) bins_rect_kernel(const uint32_t* __restrict__ start, uint32_t bins_x,
                                                        uint32_t nbins, uint32_t W, uint32_t H, uint32_t phase,
                                                        uint32_t* __restrict__ acc) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t a[4] = {0u, 0u, 0u, 0u};
    if (b < nbins && start[b + 1] > start[b]) {
        const uint32_t bx = b % bins_x, by = b / bins_x;
        const int32_t y0 = (int32_t)(by * kBinH + phase) - (int32_t)kBinH;
        const uint32_t x0 = bx * kBinW, x1 = min(x0 + kBinW, W) - 1;
        const uint32_t r0 = (uint32_t)max(y0, 0), r1 = (uint32_t)min(y0 + (int32_t)kBinH, (int32_t)H) - 1;
        a[0] = ~x0;
        a[1] = x1 + 1u;
        a[2] = ~r0;
        a[3] = r1 + 1u;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
        for (int off = 32; off > 0; off >>= 1) a[k] = max(a[k], (uint32_t)__shfl_xor((int)a[k], off));
    // one set of atomics per workgroup (per wave they serialised on the same four words)
    __shared__ uint32_t s_a[4][4];
    const uint32_t wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < 4; ++k) s_a[wave][k] = a[k];
    __syncthreads();
    if (threadIdx.x < 4) {  // (launched with 256 threads: four waves)
        uint32_t m = 0, any = 0;
        for (uint32_t w = 0; w < 4; ++w) {
            m = max(m, s_a[w][threadIdx.x]);
            any |= s_a[w][1];  // some bin of the workgroup is non-empty
        }
        if (any) atomicMax(acc + threadIdx.x, m);
    }
}

template <typename T>
hipError_t grow(T** p, size_t* cap, size_t need) {
    if (*p && *cap >= need) return hipSuccess;
    if (*p) {
        hipError_t e = hipFree(*p);
        if (e != hipSuccess) return e;
        *p = nullptr;
    }
    *cap = 0;
    hipError_t e = hipMalloc((void**)p, (need ? need : 1) * sizeof(T));
    if (e == hipSuccess) *cap = need ? need : 1;
    return e;
}

// Sub-block s = sy * (4 * tiles_x) + sx (padded rows: a 64 x 4 block's four sub-blocks are four
// consecutive threads): listed when some object can be hit there (see build_detail_list).
__global__ void __launch_bounds__(256) detail_flags_kernel(const ObjectDesc* __restrict__ objs, uint32_t nobj,
                                                           uint32_t cam_w, uint32_t row0, uint32_t rows,
                                                           uint32_t bins_x, uint32_t phase, uint32_t tiles_x,
                                                           uint32_t n, uint8_t* __restrict__ flags,
                                                           uint32_t* __restrict__ packed, uint8_t* __restrict__ occ) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t row_subs = 4 * tiles_x;
    const uint32_t sx = s % row_subs, sy = s / row_subs;
    bool hit = false;
    if (s < n && sx * kBinW < cam_w) {
        const int32_t x0 = (int32_t)(sx * kBinW), x1 = x0 + (int32_t)kBinW - 1;
        const int32_t y0 = (int32_t)(row0 + sy * kBinH), y1 = min(y0 + (int32_t)kBinH, (int32_t)(row0 + rows)) - 1;
        for (uint32_t oi = 0; oi < nobj && !hit; ++oi) {
            const ObjGeom& g = objs[oi].g;
            if (!g.tri_count) continue;
            if (g.bin_start) {  // the frame kernel's bin of this sub-block (first_hit_binned)
                const uint32_t bin = ((row0 + sy * kBinH + kBinH - phase) / kBinH) * bins_x + sx;
                hit = g.bin_start[bin + 1] > g.bin_start[bin];
            } else {
                hit = x0 <= g.rect[1] && x1 >= g.rect[0] && y0 <= g.rect[3] && y1 >= g.rect[2];
            }
        }
    }
    if (s < n) {
        flags[s] = hit ? 1 : 0;
        packed[s] = (sy << 16) | sx;
    }
    // the block's four flags: lanes 4b .. 4b + 3 of the wave (row_subs is a multiple of 4)
    const unsigned long long bal = __ballot(hit);
    if (s < n && (threadIdx.x & 3) == 0) occ[s / 4] = (uint8_t)((bal >> (threadIdx.x & 63)) & 0xfu);
}

}  // namespace

hipError_t build_detail_list(const ObjectDesc* objs, uint32_t nobj, uint32_t cam_w, uint32_t row0, uint32_t rows,
                             uint32_t bins_x, uint32_t phase, uint32_t tiles_x, uint32_t* list, uint8_t* occ,
                             uint32_t* count, hipStream_t s) {
    const uint32_t subs_y = (rows + kBinH - 1) / kBinH;
    const uint32_t n = 4 * tiles_x * subs_y;
    *count = 0;
    if (!n) return hipSuccess;
    uint8_t* flags = nullptr;
    uint32_t *packed = nullptr, *d_count = nullptr;
    void* temp = nullptr;
    auto done = [&](hipError_t err) {
        for (void* q : {(void*)flags, (void*)packed, (void*)d_count, temp})
            if (q) hipFree(q);
        return err;
    };
    hipError_t e;
    if ((e = hipMalloc((void**)&flags, n)) != hipSuccess) return done(e);
    if ((e = hipMalloc((void**)&packed, sizeof(uint32_t) * n)) != hipSuccess) return done(e);
    if ((e = hipMalloc((void**)&d_count, sizeof(uint32_t))) != hipSuccess) return done(e);
    detail_flags_kernel<<<(n + 255) / 256, 256, 0, s>>>(objs, nobj, cam_w, row0, rows, bins_x, phase, tiles_x, n,
                                                        flags, packed, occ);
    if ((e = hipGetLastError()) != hipSuccess) return done(e);
    size_t temp_bytes = 0;
    if ((e = hipcub::DeviceSelect::Flagged(nullptr, temp_bytes, packed, flags, list, d_count, (int)n, s)) !=
        hipSuccess)
        return done(e);
    if ((e = hipMalloc(&temp, temp_bytes ? temp_bytes : 1)) != hipSuccess) return done(e);
    if ((e = hipcub::DeviceSelect::Flagged(temp, temp_bytes, packed, flags, list, d_count, (int)n, s)) != hipSuccess)
        return done(e);
    if ((e = hipMemcpyAsync(count, d_count, sizeof(uint32_t), hipMemcpyDeviceToHost, s)) != hipSuccess ||
        (e = hipStreamSynchronize(s)) != hipSuccess)
        return done(e);
    return done(hipSuccess);
}

hipError_t launch_bins_rect(const uint32_t* start, uint32_t bins_x, uint32_t bins_y, uint32_t W, uint32_t H,
                            uint32_t phase, uint32_t* acc, hipStream_t s) {
    const uint32_t nbins = bins_x * bins_y;
    if (!nbins) return hipSuccess;
    bins_rect_kernel<<<(nbins + 255) / 256, 256, 0, s>>>(start, bins_x, nbins, W, H, phase, acc);
    return hipGetLastError();
}

hipError_t build_bins(const TriCull* cull, const TriHot* hot, uint32_t T, uint32_t W, uint32_t H, uint32_t phase,
                      uint32_t bins_x, uint32_t bins_y, ObjBins* out, hipStream_t s) {
    const uint32_t nbins = bins_x * bins_y;
    hipError_t e = grow(&out->start, &out->start_cap, (size_t)nbins + 1);
    if (e != hipSuccess) return e;
    uint32_t *keys = nullptr, *keys2 = nullptr, *order = nullptr, *order2 = nullptr, *tri = nullptr;
    uint32_t *pkey = nullptr, *pface = nullptr, *pflag = nullptr, *pos = nullptr;
    unsigned long long *mask = nullptr, *area = nullptr, *first = nullptr, *d_n = nullptr, *pmask = nullptr;
    int4* range = nullptr;
    void* temp = nullptr;
    size_t n = 0;
    unsigned long long pairs = 0;  // (face, bin) pairs of the faces' bin rectangles
    auto done = [&](hipError_t err) {
        for (void* q : {(void*)keys, (void*)keys2, (void*)order, (void*)order2, (void*)tri, (void*)pkey,
                        (void*)pface, (void*)pflag, (void*)pos, (void*)mask, (void*)area, (void*)first, (void*)d_n,
                        (void*)pmask, (void*)range, temp})
            if (q) hipFree(q);
        return err;
    };
    // scratch scans: one temp buffer, grown to the largest request
    size_t temp_cap = 0;
    auto temp_for = [&](size_t bytes) -> hipError_t {
        if (temp && temp_cap >= bytes) return hipSuccess;
        if (temp) hipFree(temp);
        temp = nullptr;
        temp_cap = 0;
        const hipError_t err = hipMalloc(&temp, bytes ? bytes : 1);
        if (err == hipSuccess) temp_cap = bytes;
        return err;
    };
    // pairs per pass (24 B of scratch each); tests shrink it (ERAY_BIN_PAIR_CHUNK) to cover the
    // multi-pass compaction
    const char* e_chunk = getenv("ERAY_BIN_PAIR_CHUNK");
    const unsigned long long kPairChunk = e_chunk && atoll(e_chunk) > 0 ? (unsigned long long)atoll(e_chunk) : 1ull << 24;
    if (T) {
        if ((e = hipMalloc((void**)&range, sizeof(int4) * T)) != hipSuccess) return done(e);
        if ((e = hipMalloc((void**)&area, sizeof(unsigned long long) * T)) != hipSuccess) return done(e);
        if ((e = hipMalloc((void**)&first, sizeof(unsigned long long) * T)) != hipSuccess) return done(e);
        if ((e = hipMalloc((void**)&d_n, sizeof(unsigned long long))) != hipSuccess) return done(e);
        bin_range_kernel<<<(T + 255) / 256, 256, 0, s>>>(cull, T, W, H, phase, range, area);
        if ((e = hipGetLastError()) != hipSuccess) return done(e);
        size_t temp_bytes = 0;
        if ((e = hipcub::DeviceScan::ExclusiveSum(nullptr, temp_bytes, area, first, T, s)) != hipSuccess ||
            (e = temp_for(temp_bytes)) != hipSuccess ||
            (e = hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, area, first, T, s)) != hipSuccess)
            return done(e);
        unsigned long long last[2];
        if ((e = hipMemcpyAsync(&last[0], first + T - 1, 8, hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipMemcpyAsync(&last[1], area + T - 1, 8, hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipMemsetAsync(d_n, 0, sizeof(unsigned long long), s)) != hipSuccess ||
            (e = hipStreamSynchronize(s)) != hipSuccess)
            return done(e);
        pairs = last[0] + last[1];
        // the non-empty pairs (count only)
        for (unsigned long long j0 = 0; j0 < pairs; j0 += kPairChunk) {
            const uint32_t len = (uint32_t)std::min(kPairChunk, pairs - j0);
            bin_pairs_kernel<false><<<(len + 255) / 256, 256, 0, s>>>(cull, range, first, T, j0, len, W, H, phase,
                                                                      bins_x, d_n, nullptr, nullptr, nullptr, nullptr);
            if ((e = hipGetLastError()) != hipSuccess) return done(e);
        }
        unsigned long long nn = 0;
        if ((e = hipMemcpyAsync(&nn, d_n, 8, hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipStreamSynchronize(s)) != hipSuccess)
            return done(e);
        if (nn >= (1ull << 31)) return done(hipErrorOutOfMemory);  // entries are indexed by int (radix sort)
        n = (size_t)nn;
    }
    if ((e = grow(&out->tri, &out->tri_cap, n)) != hipSuccess) return done(e);
    if ((e = grow(&out->mask, &out->mask_cap, n)) != hipSuccess) return done(e);
    if ((e = grow(&out->hot, &out->hot_cap, n)) != hipSuccess) return done(e);
    out->n = n;
    if (n) {
        for (uint32_t** q : {&keys, &keys2, &order, &order2, &tri})
            if ((e = hipMalloc((void**)q, sizeof(uint32_t) * n)) != hipSuccess) return done(e);
        if ((e = hipMalloc((void**)&mask, sizeof(unsigned long long) * n)) != hipSuccess) return done(e);
        const size_t chunk = (size_t)std::min(kPairChunk, pairs);
        if ((e = hipMalloc((void**)&pmask, sizeof(unsigned long long) * chunk)) != hipSuccess) return done(e);
        for (uint32_t** q : {&pkey, &pface, &pflag, &pos})
            if ((e = hipMalloc((void**)q, sizeof(uint32_t) * chunk)) != hipSuccess) return done(e);
        // the pairs again, now written out, and compacted in pair order (= face order)
        uint32_t base = 0;
        for (unsigned long long j0 = 0; j0 < pairs; j0 += kPairChunk) {
            const uint32_t len = (uint32_t)std::min(kPairChunk, pairs - j0);
            bin_pairs_kernel<true><<<(len + 255) / 256, 256, 0, s>>>(cull, range, first, T, j0, len, W, H, phase,
                                                                     bins_x, nullptr, pmask, pkey, pface, pflag);
            if ((e = hipGetLastError()) != hipSuccess) return done(e);
            size_t temp_bytes = 0;
            if ((e = hipcub::DeviceScan::ExclusiveSum(nullptr, temp_bytes, pflag, pos, len, s)) != hipSuccess ||
                (e = temp_for(temp_bytes)) != hipSuccess ||
                (e = hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, pflag, pos, len, s)) != hipSuccess)
                return done(e);
            bin_emit_kernel<<<(len + 255) / 256, 256, 0, s>>>(pmask, pkey, pface, pflag, pos, len, base, keys, order,
                                                              tri, mask);
            if ((e = hipGetLastError()) != hipSuccess) return done(e);
            if (j0 + len < pairs) {  // the next chunk's base
                uint32_t last[2];
                if ((e = hipMemcpyAsync(&last[0], pos + len - 1, 4, hipMemcpyDeviceToHost, s)) != hipSuccess ||
                    (e = hipMemcpyAsync(&last[1], pflag + len - 1, 4, hipMemcpyDeviceToHost, s)) != hipSuccess ||
                    (e = hipStreamSynchronize(s)) != hipSuccess)
                    return done(e);
                base += last[0] + last[1];
            }
        }
        if ((e = hipGetLastError()) != hipSuccess) return done(e);
        int end_bit = 1;
        while (end_bit < 32 && (1ull << end_bit) < (unsigned long long)nbins) ++end_bit;
        hipcub::DoubleBuffer<uint32_t> kb(keys, keys2), vb(order, order2);
        size_t temp_bytes = 0;
        if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, kb, vb, (int)n, 0, end_bit, s)) !=
                hipSuccess ||
            (e = temp_for(temp_bytes)) != hipSuccess)
            return done(e);
        if ((e = hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, kb, vb, (int)n, 0, end_bit, s)) != hipSuccess)
            return done(e);
        bin_start_kernel<<<(nbins + 1 + 255) / 256, 256, 0, s>>>(kb.Current(), (uint32_t)n, nbins, out->start);
        if ((e = hipGetLastError()) != hipSuccess) return done(e);
        bin_gather_kernel<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(vb.Current(), tri, mask, hot, n, out->tri,
                                                                       out->mask, out->hot);
    } else {
        bin_start_kernel<<<(nbins + 1 + 255) / 256, 256, 0, s>>>(nullptr, 0, nbins, out->start);
    }
    if ((e = hipGetLastError()) != hipSuccess) return done(e);
    e = hipStreamSynchronize(s);  // the scratch buffers are freed below
    return done(e);
}

}  // namespace gpu
}  // namespace eray
