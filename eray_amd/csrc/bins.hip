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
// count covered bins per face -> exclusive scan -> emit (bin, position) pairs in face order ->
// stable radix sort by bin (LSD: keeps face order within a bin) -> bin start offsets -> faces,
// pixel masks and intersection records gathered in bin order.
#include <hipcub/hipcub.hpp>

#include "face_rect.hpp"
#include "internal.hpp"

namespace eray {
namespace gpu {
namespace {

// per face: its bins (face_rect) and how many of them it may actually cover (bin_pixels != 0)
__global__ void __launch_bounds__(256) bin_count_kernel(const TriCull* __restrict__ cull, uint32_t T, uint32_t W,
                                                        uint32_t H, uint32_t phase, uint32_t* __restrict__ count,
                                                        int4* __restrict__ range) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= T) return;
    const TriCull c = cull[i];
    int32_t r[4];
    uint32_t n = 0;
    int4 g = make_int4(1, 0, 1, 0);
    if (face_rect(c, W, H, r)) {
        // bin row of camera row y: (y + kBinH - phase) / kBinH
        g = make_int4(r[0] / (int32_t)kBinW, r[1] / (int32_t)kBinW,
                      (r[2] + (int32_t)kBinH - (int32_t)phase) / (int32_t)kBinH,
                      (r[3] + (int32_t)kBinH - (int32_t)phase) / (int32_t)kBinH);
        for (int32_t ty = g.z; ty <= g.w; ++ty)
            for (int32_t tx = g.x; tx <= g.y; ++tx) n += bin_pixels(c, W, H, phase, (uint32_t)tx, (uint32_t)ty) != 0;
    }
    count[i] = n;
    range[i] = g;
}

__global__ void __launch_bounds__(256) bin_emit_kernel(const TriCull* __restrict__ cull,
                                                       const uint32_t* __restrict__ offset,
                                                       const uint32_t* __restrict__ count,
                                                       const int4* __restrict__ range, uint32_t T, uint32_t W,
                                                       uint32_t H, uint32_t phase, uint32_t bins_x,
                                                       uint32_t* __restrict__ keys, uint32_t* __restrict__ order,
                                                       uint32_t* __restrict__ tri, unsigned long long* __restrict__ mask) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= T || !count[i]) return;
    const TriCull c = cull[i];
    uint32_t o = offset[i];
    const int4 g = range[i];
    for (int32_t ty = g.z; ty <= g.w; ++ty)
        for (int32_t tx = g.x; tx <= g.y; ++tx) {
            const unsigned long long m = bin_pixels(c, W, H, phase, (uint32_t)tx, (uint32_t)ty);
            if (!m) continue;
            keys[o] = (uint32_t)ty * bins_x + (uint32_t)tx;
            order[o] = o;  // emit positions increase with the face index
            tri[o] = i;
            mask[o] = m;
            ++o;
        }
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

// start[t] = first position of bin t in the sorted keys (start[nbins] = n)
__global__ void __launch_bounds__(256) bin_start_kernel(const uint32_t* __restrict__ keys, uint32_t n,
                                                        uint32_t nbins, uint32_t* __restrict__ start) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    const uint32_t lo = i == 0 ? 0u : keys[i - 1] + 1u;
    const uint32_t hi = i == n ? nbins : keys[i];
    for (uint32_t t = lo; t <= hi && t <= nbins; ++t) start[t] = i;
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
    if ((threadIdx.x & 63) == 0 && a[1])
        for (int k = 0; k < 4; ++k) atomicMax(acc + k, a[k]);
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
    uint32_t *count = nullptr, *offset = nullptr, *keys = nullptr, *keys2 = nullptr, *order = nullptr,
             *order2 = nullptr, *tri = nullptr;
    unsigned long long* mask = nullptr;
    int4* range = nullptr;
    void* temp = nullptr;
    size_t n = 0;
    auto done = [&](hipError_t err) {
        for (void* q : {(void*)count, (void*)offset, (void*)keys, (void*)keys2, (void*)order, (void*)order2,
                        (void*)tri, (void*)mask, (void*)range, temp})
            if (q) hipFree(q);
        return err;
    };
    if (T) {
        if ((e = hipMalloc((void**)&count, sizeof(uint32_t) * T)) != hipSuccess) return done(e);
        if ((e = hipMalloc((void**)&offset, sizeof(uint32_t) * T)) != hipSuccess) return done(e);
        if ((e = hipMalloc((void**)&range, sizeof(int4) * T)) != hipSuccess) return done(e);
        bin_count_kernel<<<(T + 255) / 256, 256, 0, s>>>(cull, T, W, H, phase, count, range);
        if ((e = hipGetLastError()) != hipSuccess) return done(e);
        size_t temp_bytes = 0;
        if ((e = hipcub::DeviceScan::ExclusiveSum(nullptr, temp_bytes, count, offset, T, s)) != hipSuccess)
            return done(e);
        if ((e = hipMalloc(&temp, temp_bytes ? temp_bytes : 1)) != hipSuccess) return done(e);
        if ((e = hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, count, offset, T, s)) != hipSuccess)
            return done(e);
        uint32_t last[2];
        if ((e = hipMemcpyAsync(&last[0], offset + T - 1, 4, hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipMemcpyAsync(&last[1], count + T - 1, 4, hipMemcpyDeviceToHost, s)) != hipSuccess ||
            (e = hipStreamSynchronize(s)) != hipSuccess)
            return done(e);
        n = (size_t)last[0] + last[1];
        hipFree(temp);
        temp = nullptr;
    }
    if ((e = grow(&out->tri, &out->tri_cap, n)) != hipSuccess) return done(e);
    if ((e = grow(&out->mask, &out->mask_cap, n)) != hipSuccess) return done(e);
    if ((e = grow(&out->hot, &out->hot_cap, n)) != hipSuccess) return done(e);
    out->n = n;
    if (n) {
        for (uint32_t** q : {&keys, &keys2, &order, &order2, &tri})
            if ((e = hipMalloc((void**)q, sizeof(uint32_t) * n)) != hipSuccess) return done(e);
        if ((e = hipMalloc((void**)&mask, sizeof(unsigned long long) * n)) != hipSuccess) return done(e);
        bin_emit_kernel<<<(T + 255) / 256, 256, 0, s>>>(cull, offset, count, range, T, W, H, phase, bins_x, keys,
                                                        order, tri, mask);
        if ((e = hipGetLastError()) != hipSuccess) return done(e);
        int end_bit = 1;
        while (end_bit < 32 && (1ull << end_bit) < (unsigned long long)nbins) ++end_bit;
        hipcub::DoubleBuffer<uint32_t> kb(keys, keys2), vb(order, order2);
        size_t temp_bytes = 0;
        if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, kb, vb, (int)n, 0, end_bit, s)) !=
            hipSuccess)
            return done(e);
        if ((e = hipMalloc(&temp, temp_bytes ? temp_bytes : 1)) != hipSuccess) return done(e);
        if ((e = hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, kb, vb, (int)n, 0, end_bit, s)) != hipSuccess)
            return done(e);
        bin_start_kernel<<<(uint32_t)((n + 1 + 255) / 256), 256, 0, s>>>(kb.Current(), (uint32_t)n, nbins,
                                                                          out->start);
        if ((e = hipGetLastError()) != hipSuccess) return done(e);
        bin_gather_kernel<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(vb.Current(), tri, mask, hot, n, out->tri,
                                                                       out->mask, out->hot);
    } else {
        bin_start_kernel<<<1, 256, 0, s>>>(nullptr, 0, nbins, out->start);
    }
    if ((e = hipGetLastError()) != hipSuccess) return done(e);
    e = hipStreamSynchronize(s);  // the scratch buffers are freed below
    return done(e);
}

}  // namespace gpu
}  // namespace eray
