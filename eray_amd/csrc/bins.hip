// bins.hip — screen bins of the large objects' faces for the frame kernel's primary-ray scan,
// rebuilt per camera entirely on the device.  A bin is one 16 x 4 pixel sub-block: exactly one
// wave's pixels.
//
// The per-face pixel rectangles (face_rect.hpp, setup.hip) say which bins a face can be hit in.
// For objects too large to scan per wave (> kDirectMax faces) the frame kernel reads, for its
// sub-block's bin, the faces that can be hit there and runs the exact tests on those only: a face
// outside the bin's list cannot be hit by any ray of the bin.  The list need not be in index
// order: the frame kernel keeps, per pixel, the smallest face index whose Triangle::intersects
// passes, which is the reference's first hit (object.rs:63-78).
//
// Each entry also carries the bin's pixels the face may cover (bin_pixels: the four culling
// bounds solved per pixel row), so the frame kernel only tests (face, pixel) pairs that can hit.
// The general tracer's setup (SetupParams::keep_all) masks the pixels any of whose jittered
// anti-aliasing rays may pass instead (bin_pixels_jittered; trace.hip).
//
// Per camera, after camera_setup_kernel (each binned face's bin rectangle and its number of units,
// bin rows or bins): exclusive scan of the units -> the pair pass (bin_segments_kernel /
// bin_pairs_kernel below) computes the (face, bin) pairs' pixel masks and appends the non-empty
// pairs (wave-aggregated slot counter) with a per-bin count -> exclusive scan of the counts ->
// each entry scattered to its bin (one 64-B BinEntry line: record, mask, face) -> the counts
// zeroed for the next camera, the binned objects' rectangles narrowed to their non-empty bins,
// their bin views in the descriptors -> the detail sub-block list.
// Buffers are preallocated (bins_alloc); if the pairs exceed the capacity the bins are dropped
// for that camera (the frame kernel scans those objects through LDS tiles instead, still exact)
// and CamState reports the count, so the host can grow the capacity.
#include <algorithm>
#include <mutex>

#include <hipcub/hipcub.hpp>

#include "cull_record.hpp"
#include "face_rect.hpp"
#include "internal.hpp"

namespace eray {
namespace gpu {
namespace {

constexpr int kBinWG = 256;
constexpr uint32_t kPairGrid = 2048;  // workgroups of the grid-stride pair and scatter loops

// The entry list's slot counter is sharded: device-scope atomics execute at the memory side, and
// one word (or one 64-B line) takes about 88 returning atomics per microsecond (MI355X_MICROARCH.md
// dequeue row), so one counter bumped once per 256 pairs serialised the pair pass (C5's four-camera
// build: ~115k bumps, 1.3-1.8 ms).  Workgroup b appends to shard b % kShards, which owns entries
// [s * region, (s + 1) * region) (region = cap / kShards); its counter sits kShardStride words
// from the next one (a line of its own).  Pairs are dealt to the workgroups in 256-pair chunks
// round-robin, so the shards fill evenly.
constexpr uint32_t kShards = 32, kShardStride = 32;
// binned object k's rectangle accumulator: acc + kAccStride * k (a line per object: the
// finaliser's per-workgroup atomics on different objects do not share a line)
constexpr uint32_t kAccStride = 16;


// Inclusive prefix max over the wave's lanes (DPP row shifts, then the row broadcasts; an invalid
// source lane reads 0, the identity).  Every lane of the wave calls.
template <int kCtrl, int kRowMask>
__device__ __forceinline__ uint32_t dpp_max_step(uint32_t v) {
    return max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, kRowMask, 0xf, false));
}
__device__ __forceinline__ uint32_t wave_prefix_max(uint32_t v) {
    v = dpp_max_step<0x111, 0xf>(v);  // row_shr:1
    v = dpp_max_step<0x112, 0xf>(v);  // row_shr:2
    v = dpp_max_step<0x114, 0xf>(v);  // row_shr:4
    v = dpp_max_step<0x118, 0xf>(v);  // row_shr:8: each row's inclusive prefix
    v = dpp_max_step<0x142, 0xa>(v);  // row_bcast:15 (rows 1 and 3)
    return dpp_max_step<0x143, 0xc>(v);  // row_bcast:31 (rows 2 and 3)
}

// The setup enumerates units of every binned face — the (face, bin) pairs of its bin rectangle,
// or the rectangle's bin rows (segments, below) — in face order, with face i's first unit at
// boff[i / chunk] + first_local[i] (its setup chunk's offset + its place in the chunk's own scan)
// and all P units at boff[nparts].  Every wave walks its own contiguous range of units, 64 at a
// time: one search for the face of its first unit, after which each slice starts from the face of
// the previous slice's last unit (the next slice's face ranges loaded ahead).  (A grid-stride
// loop searched anew for every slice — ~12 dependent global loads per 64 units, the pass's
// critical path: C5's four-camera build 1.3-1.8 ms.)  body(j, valid, face) runs once per slice
// with every lane of the wave (lane = unit j; `valid`: j is one of the wave's units).
struct UnitWalk {
    const unsigned long long* s_boff;  // (LDS) boff
    const unsigned long long* first_local;
    uint32_t nparts, chunk, T;
    uint32_t* s_face;  // (LDS) kBinWG words: the faces starting at each lane's unit
};
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
template <typename Body>
__device__ __forceinline__ void walk_units(const UnitWalk& u, Body&& body) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned long long P = u.s_boff[u.nparts];
    auto first = [&](uint32_t i) { return u.s_boff[i / u.chunk] + u.first_local[i]; };
    auto face_of = [&](unsigned long long j) -> uint32_t {
        // the chunk: the last one starting at or before j (in LDS; an empty chunk never is, the next
        // one starts at the same unit) ...
        uint32_t cb = 0, ce = u.nparts;
        while (ce - cb > 1) {
            const uint32_t mid = (cb + ce) >> 1;
            if (u.s_boff[mid] <= j) cb = mid;
            else ce = mid;
        }
        // ... then, inside it, the last face whose first unit is <= j
        const unsigned long long jl = j - u.s_boff[cb];
        uint32_t lo = cb * u.chunk, hi = min(lo + u.chunk, u.T);
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (u.first_local[mid] <= jl) lo = mid + 1;
            else hi = mid;
        }
        return lo - 1;
    };
    const unsigned long long slices = (unsigned long long)gridDim.x * (kBinWG / 64) * 64ull;
    const unsigned long long per = (P + slices - 1) / slices * 64ull;  // units per wave (multiple of 64)
    const unsigned long long w_lo = ((unsigned long long)blockIdx.x * (kBinWG / 64) + wave) * per;
    const unsigned long long w_hi = min(w_lo + per, P);
    uint32_t fb = w_lo < P ? face_of(w_lo) : 0u;
    // face fi's units [a, b) for the 64 faces from fb on (P past the last face)
    auto face_units = [&](uint32_t fb0, unsigned long long& a, unsigned long long& b) {
        const uint32_t fi = fb0 + lane;
        a = P;
        b = P;
        if (fi < u.T) {
            a = first(fi);
            b = fi + 1 < u.T ? first(fi + 1) : P;
        }
    };
    unsigned long long pa, pb;  // the next slice's first 64 faces' units, loaded ahead
    face_units(fb, pa, pb);
    for (unsigned long long j0 = w_lo; j0 < w_hi; j0 += 64) {  // wave-uniform
        const unsigned long long jend = min(j0 + 64ull, w_hi), j = j0 + lane;
        // The wave's 64 consecutive units belong to a run of consecutive faces from fb on: each
        // non-empty face starting inside the slice writes its index at its first unit's slot (no
        // two do: the ranges are contiguous), then a prefix max over the lanes gives every slot
        // the last face starting at or before it — its owner; slot 0's owner may start earlier,
        // and is then fb, the previous slice's last face (a face starting at j0 overrides it).
        u.s_face[threadIdx.x] = lane ? 0u : fb;
        wave_sync();
        bool ahead = true;  // the first 64 faces were loaded ahead
        for (unsigned long long covered = j0; covered < jend; fb += 64, ahead = false) {  // wave-uniform
            unsigned long long a = pa, b = pb;
            if (!ahead) face_units(fb, a, b);
            if (a < b && a >= j0 && a < jend) u.s_face[64 * wave + (uint32_t)(a - j0)] = fb + lane;
            covered = (unsigned long long)__shfl((long long)b, 63);
        }
        wave_sync();
        const uint32_t owner = wave_prefix_max(u.s_face[threadIdx.x]);
        fb = (uint32_t)__builtin_amdgcn_readlane((int)owner, (int)(jend - 1 - j0));  // the next slice starts in this face or later
        if (jend < w_hi) face_units(fb, pa, pb);  // in flight while this slice's units are processed
        body(j, j < jend, owner, j < jend ? j - first(owner) : 0ull);
    }
}

// Entries appended to the shard's region of the entry list (one counter atomic per wave and
// call), each with its rank in its bin from the bin's count atomic (the scatter then needs no
// atomics: a returning atomic per entry there cost as much as this pass).  Every lane calls; m == 0:
// no entry.
struct EntryOut {
    uint32_t *n, *count, *ekey, *eface, *erank;
    unsigned long long* emask;
    uint32_t shard, region;
};
__device__ __forceinline__ void append_entries(const EntryOut& o, unsigned long long m, uint32_t key, uint32_t face) {
    const uint32_t lane = threadIdx.x & 63;
    const unsigned long long bal = __ballot(m != 0);
    if (!bal) return;
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(o.n + o.shard * kShardStride, (uint32_t)__popcll(bal));
    base = (uint32_t)__shfl((int)base, 0);
    if (m) {
        const uint32_t local = base + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
        if (local < o.region) {
            const uint32_t slot = o.shard * o.region + local;
            o.erank[slot] = atomicAdd(o.count + key, 1u);
            o.ekey[slot] = key;
            o.eface[slot] = face;
            o.emask[slot] = m;
        }
    }
}

// (face, bin) pairs of the binned faces' bin rectangles (face-major, each rectangle row-major):
// the non-empty ones appended to the entry list, counted per bin key.  The general tracer's setup
// (kJitter, SetupParams::keep_all: bin_pixels_jittered's masks) and frames wider than 65535
// pixels; otherwise bin_segments_kernel.
// waves per SIMD the pair pass is built for: 6 (80 VGPRs, a few spills in the mask path) over
// 5 (88 VGPRs): C5's moving-camera frame 491 -> 476 us; 8 (64 VGPRs, 22 spills) 525 us
constexpr int kPairsWaves = 6;
template <bool kJitter>
__global__ void __launch_bounds__(kBinWG, kPairsWaves) bin_pairs_kernel(const TriCull* __restrict__ cull,
                                                           const int4* __restrict__ range,
                                                           const unsigned long long* __restrict__ first_local,
                                                           const unsigned long long* __restrict__ boff,
                                                           uint32_t nparts, uint32_t chunk,
                                                           const uint32_t* __restrict__ fkey, uint32_t T, uint32_t W,
                                                           uint32_t H, uint32_t phase, uint32_t bins_x, uint32_t nbins,
                                                           uint32_t cap, uint32_t* __restrict__ n,
                                                           uint32_t* __restrict__ count, uint32_t* __restrict__ ekey,
                                                           uint32_t* __restrict__ eface,
                                                           unsigned long long* __restrict__ emask,
                                                           uint32_t* __restrict__ erank) {
    // face i's first pair: its setup chunk's offset + its place in the chunk's own scan
    __shared__ unsigned long long s_boff[kSetupMaxBlocks + 1];
    __shared__ double s_poly[kJitter ? 16 * kBinWG : 1];  // clip_box's workspace
    for (uint32_t b = threadIdx.x; b <= nparts; b += kBinWG) s_boff[b] = boff[b];
    __syncthreads();
    auto first = [&](uint32_t i) { return s_boff[i / chunk] + first_local[i]; };
    const unsigned long long P = s_boff[nparts];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned long long lt = (1ull << lane) - 1ull;
    // each wave appends to shard (global wave index) % kShards, one counter atomic per 64 kept pairs
    const uint32_t shard = (blockIdx.x * (kBinWG / 64) + wave) % kShards, region = cap / kShards;
    __shared__ uint32_t s_face[kBinWG];  // the faces starting at each lane's pair (then the prefix max)
    // each wave's queue of pairs that survive the bin-rectangle test: face, bin (tx | ty << 16), key
    __shared__ uint32_t s_qf[kBinWG / 64][128], s_qt[kBinWG / 64][128], s_qk[kBinWG / 64][128];
    auto face_of = [&](unsigned long long j) -> uint32_t {
        // the chunk: the last one starting at or before j (in LDS; an empty chunk never is, the next
        // one starts at the same pair) ...
        uint32_t cb = 0, ce = nparts;
        while (ce - cb > 1) {
            const uint32_t mid = (cb + ce) >> 1;
            if (s_boff[mid] <= j) cb = mid;
            else ce = mid;
        }
        // ... then, inside it, the last face whose first pair is <= j
        const unsigned long long jl = j - s_boff[cb];
        uint32_t lo = cb * chunk, hi = min(lo + chunk, T);
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (first_local[mid] <= jl) lo = mid + 1;
            else hi = mid;
        }
        return lo - 1;
    };
    // the queue's first cnt (<= 64) pairs: pixel masks (double precision), the non-empty ones
    // appended to the entry list (wave-uniform)
    auto emit = [&](uint32_t cnt) {
        unsigned long long m = 0;
        uint32_t key = 0, i = 0;
        if (lane < cnt) {
            i = s_qf[wave][lane];
            const uint32_t t = s_qt[wave][lane];
            key = s_qk[wave][lane];
            if constexpr (kJitter) m = bin_pixels_jittered(cull[i], W, H, phase, t & 0xffffu, t >> 16, s_poly + threadIdx.x, kBinWG);
            else m = bin_pixels(cull[i], W, H, phase, t & 0xffffu, t >> 16);
        }
        const unsigned long long bal = __ballot(m != 0);
        if (!bal) return;
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(n + shard * kShardStride, (uint32_t)__popcll(bal));
        base = (uint32_t)__shfl((int)base, 0);
        if (m) {
            const uint32_t local = base + (uint32_t)__popcll(bal & lt);
            if (local < region) {
                const uint32_t slot = shard * region + local;
                // the entry's rank in its bin comes back with the count: the scatter needs no
                // atomics (a returning atomic per entry there cost as much as this pass)
                erank[slot] = atomicAdd(count + key, 1u);
                ekey[slot] = key;
                eface[slot] = i;
                emask[slot] = m;
            }
        }
    };
    // Every wave walks its own contiguous range of pairs, 64 at a time: one search for the face
    // of its first pair, after which each slice starts from the face of the previous slice's last
    // pair.  (A grid-stride loop searched anew for every slice — ~12 dependent global loads per
    // 64 pairs, the pass's critical path: C5's four-camera build 1.3-1.8 ms.)  Most pairs of a
    // face's bin rectangle are empty (C5: 7.1M pairs, 0.47M entries per camera), so each pair is
    // first tested against the bin's whole pixel rectangle with the frame kernel's own f32 culling
    // test (cull_rejects over the rectangle of the bin's corner rays, widened as make_bundle does:
    // a rejected bin has no pixel whose ray can hit the face); the survivors queue in LDS and go
    // through the per-row double-precision masks 64 at a time.
    const unsigned long long slices = (unsigned long long)gridDim.x * (kBinWG / 64) * 64ull;
    const unsigned long long per = (P + slices - 1) / slices * 64ull;  // pairs per wave (multiple of 64)
    const unsigned long long w_lo = ((unsigned long long)blockIdx.x * (kBinWG / 64) + wave) * per;
    const unsigned long long w_hi = min(w_lo + per, P);
    const float rw = __builtin_amdgcn_rcpf((float)W), rh = __builtin_amdgcn_rcpf((float)H);
    const float wlo = 1.0f - 0x1p-20f, whi = 1.0f + 0x1p-20f;
    uint32_t fb = w_lo < P ? face_of(w_lo) : 0u;
    // face fi's pairs [a, b) for the 64 faces from fb on (P past the last face)
    auto face_pairs = [&](uint32_t fb0, unsigned long long& a, unsigned long long& b) {
        const uint32_t fi = fb0 + lane;
        a = P;
        b = P;
        if (fi < T) {
            a = first(fi);
            b = fi + 1 < T ? first(fi + 1) : P;
        }
    };
    unsigned long long pa, pb;  // the next slice's first 64 faces' pairs, loaded ahead
    face_pairs(fb, pa, pb);
    uint32_t qn = 0;  // queued pairs (wave-uniform)
    for (unsigned long long j0 = w_lo; j0 < w_hi; j0 += 64) {  // wave-uniform
        const unsigned long long jend = min(j0 + 64ull, w_hi), j = j0 + lane;
        // The wave's 64 consecutive pairs belong to a run of consecutive faces from fb on: each
        // non-empty face starting inside the slice writes its index at its first pair's slot (no
        // two do: the ranges are contiguous), then a prefix max over the lanes gives every slot
        // the last face starting at or before it — its owner; slot 0's owner may start earlier,
        // and is then fb, the previous slice's last face (a face starting at j0 overrides it).
        s_face[threadIdx.x] = lane ? 0u : fb;
        wave_sync();
        bool ahead = true;  // the first 64 faces were loaded ahead
        for (unsigned long long covered = j0; covered < jend; fb += 64, ahead = false) {  // wave-uniform
            unsigned long long a = pa, b = pb;
            if (!ahead) face_pairs(fb, a, b);
            if (a < b && a >= j0 && a < jend) s_face[64 * wave + (uint32_t)(a - j0)] = fb + lane;
            covered = (unsigned long long)__shfl((long long)b, 63);
        }
        wave_sync();
        const uint32_t owner = wave_prefix_max(s_face[threadIdx.x]);
        fb = (uint32_t)__builtin_amdgcn_readlane((int)owner, (int)(jend - 1 - j0));  // the next slice starts in this face or later
        if (jend < w_hi) face_pairs(fb, pa, pb);  // in flight while this slice's pairs are tested
        bool keep = false;
        uint32_t i = 0, tx = 0, ty = 0, key = 0;
        if (j < jend) {
            i = owner;
            key = fkey[i];  // (in the same round trip as the face's records)
            const int4 g = range[i];
            const uint32_t w = (uint32_t)(g.y - g.x + 1);
            const uint32_t c = (uint32_t)(j - first(i));
            // c / w and c % w (c < 2^24: exact in f32) by a float quotient, corrected by one
            uint32_t qy = (uint32_t)((float)c / (float)w);
            int32_t rx = (int32_t)(c - qy * w);
            if (rx < 0) {
                --qy;
                rx += (int32_t)w;
            } else if (rx >= (int32_t)w) {
                ++qy;
                rx -= (int32_t)w;
            }
            tx = (uint32_t)g.x + (uint32_t)rx;
            ty = (uint32_t)g.z + qy;
            keep = true;
            if constexpr (!kJitter) {
                const int32_t x0 = (int32_t)(tx * kBinW), x1 = min(x0 + (int32_t)kBinW, (int32_t)W) - 1;
                const int32_t yb = (int32_t)(ty * kBinH + phase) - (int32_t)kBinH;
                const int32_t y0 = max(yb, 0), y1 = min(yb + (int32_t)kBinH, (int32_t)H) - 1;
                keep = y0 <= y1 && !cull_rejects(cull[i], ((float)x0 * rw) * wlo, ((float)x1 * rw) * whi,
                                                 ((float)y0 * rh) * wlo, ((float)y1 * rh) * whi);
            }
        }
        const unsigned long long kb = __ballot(keep);
        if (keep) {
            const uint32_t pos = qn + (uint32_t)__popcll(kb & lt);
            s_qf[wave][pos] = i;
            s_qt[wave][pos] = tx | (ty << 16);
            s_qk[wave][pos] = key * nbins + ty * bins_x + tx;
        }
        qn += (uint32_t)__popcll(kb);
        wave_sync();
        if (qn >= 64) {
            emit(64);
            const uint32_t rest = qn - 64;  // the queue's tail to its front
            uint32_t f2 = 0, t2 = 0, k2 = 0;
            if (lane < rest) {
                f2 = s_qf[wave][64 + lane];
                t2 = s_qt[wave][64 + lane];
                k2 = s_qk[wave][64 + lane];
            }
            wave_sync();
            if (lane < rest) {
                s_qf[wave][lane] = f2;
                s_qt[wave][lane] = t2;
                s_qk[wave][lane] = k2;
            }
            wave_sync();
            qn = rest;
        }
    }
    if (qn) emit(qn);
}

// Segments (frame setups): the units are the bin rows of each binned face's bin rectangle.  A
// segment's four camera rows each get the pixel range where all four culling conditions of the
// face can pass — bin_pixels' own double-precision lines (face_rect.hpp row_range), over the
// rectangle's columns instead of one bin's 16: the same values, so a bin's bin_pixels mask is
// exactly those ranges cut to its columns — and only the bins the ranges reach become pairs,
// dealt over the wave's lanes (lane = pair) so that one long segment (a sliver across the frame)
// does not serialise its wave.  Every pair bin_pixels would mark non-empty is appended, with the
// same mask, so the entries are the rectangle form's (which also drops pairs its f32 pre-test
// rejects: the frame kernel's exact tests decide either way).  C5: 7.06M rectangle pairs per
// camera for 0.47M entries — the rectangle form spent its time walking the empty ones.
__global__ void __launch_bounds__(kBinWG, kPairsWaves) bin_segments_kernel(const TriCull* __restrict__ cull,
                                                              const int4* __restrict__ range,
                                                              const unsigned long long* __restrict__ first_local,
                                                              const unsigned long long* __restrict__ boff,
                                                              uint32_t nparts, uint32_t chunk,
                                                              const uint32_t* __restrict__ fkey, uint32_t T, uint32_t W,
                                                              uint32_t H, uint32_t phase, uint32_t bins_x,
                                                              uint32_t nbins, uint32_t cap, uint32_t* __restrict__ n,
                                                              uint32_t* __restrict__ count, uint32_t* __restrict__ ekey,
                                                              uint32_t* __restrict__ eface,
                                                              unsigned long long* __restrict__ emask,
                                                              uint32_t* __restrict__ erank) {
    __shared__ unsigned long long s_boff[kSetupMaxBlocks + 1];
    __shared__ uint32_t s_face[kBinWG];
    __shared__ uint32_t s_own[kBinWG];  // the lanes whose segment's pairs start at each slot
    for (uint32_t b = threadIdx.x; b <= nparts; b += kBinWG) s_boff[b] = boff[b];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const EntryOut out{n, count, ekey, eface, erank, emask, (blockIdx.x * (kBinWG / 64) + wave) % kShards, cap / kShards};
    const UnitWalk u{s_boff, first_local, nparts, chunk, T, s_face};
    walk_units(u, [&](unsigned long long, bool valid, uint32_t i, unsigned long long c) {
        // the lane's segment: face i, bin row ty, its rows' pixel ranges packed lo | hi << 16 (lo >
        // hi: none) and its bins [bx0, bx0 + width)
        uint32_t ty = 0, key = 0, bx0 = 0, width = 0;
        uint32_t rr[kBinH] = {1u, 1u, 1u, 1u};
        if (valid) {
            const int4 g = range[i];
            key = fkey[i];
            ty = (uint32_t)g.z + (uint32_t)c;
            const int32_t xa = g.x * (int32_t)kBinW, xb = min((g.y + 1) * (int32_t)kBinW, (int32_t)W) - 1;
            int32_t lo = INT32_MAX, hi = INT32_MIN;
            row_ranges(cull[i], W, H, phase, ty, xa, xb, rr, lo, hi);
            if (lo <= hi) {
                bx0 = (uint32_t)lo / kBinW;
                width = (uint32_t)hi / kBinW - bx0 + 1;
            }
        }
        // the wave's pairs: lane l's segment owns [start_l, start_l + width_l)
        uint32_t incl = width;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)incl, off);
            if ((int)lane >= off) incl += y;
        }
        const uint32_t total = (uint32_t)__shfl((int)incl, 63), start = incl - width;
        uint32_t cur = 0;  // the lane owning the pair before the window
        for (uint32_t t0 = 0; t0 < total; t0 += 64) {  // (wave-uniform)
            s_own[threadIdx.x] = lane ? 0u : cur;
            wave_sync();
            if (width && start >= t0 && start < t0 + 64) s_own[64 * wave + (start - t0)] = lane;
            wave_sync();
            const uint32_t o = wave_prefix_max(s_own[threadIdx.x]);  // (lanes in segment order)
            cur = (uint32_t)__builtin_amdgcn_readlane((int)o, 63);
            const uint32_t t = t0 + lane;
            // the owner's segment
            const uint32_t oi = (uint32_t)__shfl((int)i, (int)o), oty = (uint32_t)__shfl((int)ty, (int)o);
            const uint32_t okey = (uint32_t)__shfl((int)key, (int)o), obx0 = (uint32_t)__shfl((int)bx0, (int)o);
            const uint32_t ostart = (uint32_t)__shfl((int)start, (int)o);
            uint32_t orr[kBinH];
#pragma unroll
            for (uint32_t r = 0; r < kBinH; ++r) orr[r] = (uint32_t)__shfl((int)rr[r], (int)o);
            unsigned long long m = 0;
            const uint32_t bx = obx0 + (t - ostart);
            if (t < total) m = bin_mask_of_rows(orr, bx);
            append_entries(out, m, okey * nbins + oty * bins_x + bx, oi);
            wave_sync();  // (s_own is rewritten by the next window)
        }
    });
}

// every stored entry to its bin: start[key] + its rank, as one 64-B line (BinEntry: the face's
// intersection record, its pixel mask and its index in the object); the finaliser zeroes the
// counts for the next camera (coalesced over the keys, not a scattered word per entry).  The
// shards' entries are one index space (each workgroup prefix-sums the 32 shard counts in LDS), so
// every thread of the grid takes a share: a loop over the shards gave each shard's entries to the
// grid's first threads only, which then walked 32 dependent gather-and-store chains one after the
// other (16 cameras at 3840x2160 / 70k: 114 us).
__global__ void __launch_bounds__(kBinWG) bin_scatter_kernel(const uint32_t* __restrict__ n, uint32_t cap,
                                                             const uint32_t* __restrict__ ekey,
                                                             const uint32_t* __restrict__ eface,
                                                             const unsigned long long* __restrict__ emask,
                                                             const uint32_t* __restrict__ erank,
                                                             const uint32_t* __restrict__ start,
                                                             const uint32_t* __restrict__ kbegin, uint32_t nbins,
                                                             const TriHot* __restrict__ hot, uint32_t T1,
                                                             BinEntry* __restrict__ ent) {
    static_assert(kShards <= 64, "one wave scans the shard counts");
    __shared__ uint32_t s_pre[kShards + 1];  // each shard's first index in the joint space, and the total
    const uint32_t region = cap / kShards;
    if (threadIdx.x < 64) {
        const uint32_t lane = threadIdx.x;
        const uint32_t c = lane < kShards ? min(n[lane * kShardStride], region) : 0u;
        uint32_t incl = c;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off);
            if ((int)lane >= off) incl += y;
        }
        if (lane < kShards) s_pre[lane] = incl - c;
        if (lane == kShards - 1) s_pre[kShards] = incl;
    }
    __syncthreads();
    const uint32_t total = s_pre[kShards];
    for (uint32_t g = blockIdx.x * kBinWG + threadIdx.x; g < total; g += gridDim.x * kBinWG) {
        uint32_t lo = 0, hi = kShards;  // the shard holding g: the last one starting at or before it
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_pre[mid] <= g) lo = mid;
            else hi = mid;
        }
        const uint32_t e = lo * region + (g - s_pre[lo]);
        const uint32_t key = ekey[e], f = eface[e];
        BinEntry x;
        x.hot = hot[T1 ? f % T1 : f];  // (several cameras: face f is face f % T1 of camera f / T1)
        x.mask = emask[e];
        x.tri = f - kbegin[key / nbins];
        x.pad = 0u;
        ent[start[key] + erank[e]] = x;
    }
}

// The binned objects' non-empty bins -> their pixel rectangles ((~x0, x1 + 1, ~y0, y1 + 1),
// max-reduced); the last workgroup narrows each binned object's rectangle to them, publishes its
// bin views (none on overflow) and resets the counters.  Keys are object-major, so a workgroup's
// 256 keys belong to a run of binned objects [k_first, k_last]: reduced in LDS, then atomically
// max-merged into the objects' accumulators by the workgroups that found a non-empty bin.
constexpr uint32_t kFinSpan = 8;    // binned objects per workgroup reduced in LDS (more: atomics)
constexpr uint32_t kFinTab = 1024;  // binned objects the last workgroup combines in LDS
constexpr uint32_t kFinGrid = 512;  // workgroups of the per-key pass

__device__ __forceinline__ void max4(uint32_t* dst, const uint32_t (&a)[4]) {
    for (int q = 0; q < 4; ++q) atomicMax(dst + q, a[q]);
}

// The scatter leaves a bin's entries in no particular order.  The frame kernel's result does not
// depend on it (each pixel keeps its smallest hitting face), but its work does: a bin is searched
// in chunks of 64 entries, and a chunk whose faces all come after every live pixel's best hit so
// far is skipped — in face order, the later chunks of a dense bin mostly are.  So each bin with
// more than one chunk (and at most kSortMax entries; longer ones stay as they are) is sorted by
// face index: bins of up to kSortWave entries one wave each, longer ones (the poles of the 1M-face
// stand-in put 300-700 entries into a few bins) one workgroup each.  The frame kernel relies on
// it: in a bin of 65 to kBinSortMax entries the position order is the face order
// (render.hip first_hit_binned / first_hit_binned_wave), and chunk c's first two entries carry the
// union of the masks of chunks c + 1 .. (BinEntry::pad): pixels outside it cannot be hit by
// anything later in the bin.
constexpr uint32_t kSortMax = kBinSortMax;
constexpr uint32_t kSortWave = 256;            // bins sorted by one wave (whole bin in its LDS slice)
constexpr uint32_t kSortPer = kSortWave / 64;  // entries per lane
constexpr uint32_t kSortChunks = kSortMax / 64;
constexpr uint32_t kSortGrid = 1024;  // workgroups of the sort kernel's grid-stride loops
static_assert(kSortMax == (kBinWG / 64) * kSortWave, "a workgroup's sort LDS holds one longest bin");

// The bins to sort, appended to a work list (one counter atomic per wave and kind), so that the
// sort kernel spreads them over all its waves: the dense bins sit next to each other on the
// screen.  Wave-sorted bins go to the front of sortq (count nsort[0]), workgroup-sorted ones to
// the back (sortq[keys - 1 - i], count nsort[1]); together they are at most `keys`.
__device__ __forceinline__ void queue_sort(const uint32_t* __restrict__ start, uint32_t b, uint32_t keys,
                                           uint32_t* __restrict__ sortq, uint32_t* __restrict__ nsort) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t cnt = b < keys ? start[b + 1] - start[b] : 0u;
#pragma unroll
    for (uint32_t big = 0; big < 2; ++big) {
        const bool want = cnt > (big ? kSortWave : 64u) && cnt <= (big ? kSortMax : kSortWave);
        const unsigned long long bal = __ballot(want);
        if (!bal) continue;
        const uint32_t first = (uint32_t)(__ffsll(bal) - 1);
        uint32_t base = 0;
        if (lane == first) base = atomicAdd(nsort + big, (uint32_t)__popcll(bal));
        base = (uint32_t)__shfl((int)base, (int)first);
        const uint32_t at = base + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
        if (want) sortq[big ? keys - 1u - at : at] = b;
    }
}

// A sorted entry's pad word: chunk c's first two entries (rank 64 c, 64 c + 1) get the low and
// high halves of sfx[c + 1], the union of the masks of chunks c + 1 .. (sfx[nch] = 0).
__device__ __forceinline__ uint32_t sorted_pad(uint32_t rank, uint32_t nch, const unsigned long long* sfx) {
    const uint32_t c = rank >> 6, k = rank & 63u;
    if (k > 1u || c + 1u >= nch) return 0u;
    const unsigned long long u = sfx[c + 1u];
    return k ? (uint32_t)(u >> 32) : (uint32_t)u;
}

// Each queued bin: its entries staged in LDS, each entry's rank = the number of the bin's faces
// below its own (a face appears at most once per bin), the chunks' mask unions OR-ed by rank and
// suffix-combined, each entry written back at its rank.
__global__ void __launch_bounds__(kBinWG) bin_sort_kernel(const uint32_t* __restrict__ sortq,
                                                          const uint32_t* __restrict__ nsort,
                                                          const uint32_t* __restrict__ start,
                                                          BinEntry* __restrict__ ent, uint32_t keys) {
    __shared__ BinEntry s_ent[kBinWG / 64][kSortWave];  // a wave's bin; the workgroup's: all of it
    __shared__ unsigned long long s_cu[kBinWG / 64][kSortChunks];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // ---- bins of 65..kSortWave entries: one wave each
    {
        const uint32_t items = nsort[0];
        BinEntry* se = s_ent[wave];
        unsigned long long* cu = s_cu[wave];
        for (uint32_t it = blockIdx.x * (kBinWG / 64) + wave; it < items; it += gridDim.x * (kBinWG / 64)) {
            const uint32_t key = sortq[it];  // wave-uniform
            const uint32_t s0 = start[key], n = start[key + 1] - s0, nch = (n + 63) / 64;
            uint32_t v[kSortPer], r[kSortPer];
#pragma unroll
            for (uint32_t q = 0; q < kSortPer; ++q) {
                const uint32_t e = lane + 64 * q;
                v[q] = 0xffffffffu;
                r[q] = 0;
                if (e < n) {
                    se[e] = ent[s0 + e];
                    v[q] = se[e].tri;
                }
            }
            if (lane < kSortPer) cu[lane] = 0ull;
            wave_sync();
            for (uint32_t j = 0; j < n; ++j) {
                const uint32_t f = se[j].tri;
#pragma unroll
                for (uint32_t q = 0; q < kSortPer; ++q) r[q] += f < v[q] ? 1u : 0u;
            }
#pragma unroll
            for (uint32_t q = 0; q < kSortPer; ++q)
                if (lane + 64 * q < n) atomicOr(&cu[r[q] >> 6], se[lane + 64 * q].mask);
            wave_sync();
            if (lane == 0)
                for (uint32_t c = nch - 1; c-- > 0;) cu[c] |= cu[c + 1];
            wave_sync();
#pragma unroll
            for (uint32_t q = 0; q < kSortPer; ++q) {
                const uint32_t e = lane + 64 * q;
                if (e < n) {
                    BinEntry x = se[e];
                    x.pad = sorted_pad(r[q], nch, cu);
                    ent[s0 + r[q]] = x;
                }
            }
            wave_sync();  // the LDS is rewritten by the next bin
        }
    }
    __syncthreads();  // (the workgroup's bins below use every wave's slice)
    // ---- bins of kSortWave + 1..kSortMax entries: one workgroup each
    const uint32_t nbig = nsort[1];
    BinEntry* se = &s_ent[0][0];
    unsigned long long* cu = s_cu[0];
    constexpr uint32_t kPer = kSortMax / kBinWG;
    for (uint32_t it = blockIdx.x; it < nbig; it += gridDim.x) {  // workgroup-uniform
        const uint32_t key = sortq[keys - 1u - it];
        const uint32_t s0 = start[key], n = start[key + 1] - s0, nch = (n + 63) / 64;
        uint32_t v[kPer], r[kPer];
#pragma unroll
        for (uint32_t q = 0; q < kPer; ++q) {
            const uint32_t e = threadIdx.x + kBinWG * q;
            v[q] = 0xffffffffu;
            r[q] = 0;
            if (e < n) {
                se[e] = ent[s0 + e];
                v[q] = se[e].tri;
            }
        }
        if (threadIdx.x < kSortChunks) cu[threadIdx.x] = 0ull;
        __syncthreads();
        for (uint32_t j = 0; j < n; ++j) {
            const uint32_t f = se[j].tri;
#pragma unroll
            for (uint32_t q = 0; q < kPer; ++q) r[q] += f < v[q] ? 1u : 0u;
        }
#pragma unroll
        for (uint32_t q = 0; q < kPer; ++q)
            if (threadIdx.x + kBinWG * q < n) atomicOr(&cu[r[q] >> 6], se[threadIdx.x + kBinWG * q].mask);
        __syncthreads();
        if (threadIdx.x == 0)
            for (uint32_t c = nch - 1; c-- > 0;) cu[c] |= cu[c + 1];
        __syncthreads();
#pragma unroll
        for (uint32_t q = 0; q < kPer; ++q) {
            const uint32_t e = threadIdx.x + kBinWG * q;
            if (e < n) {
                BinEntry x = se[e];
                x.pad = sorted_pad(r[q], nch, cu);
                ent[s0 + r[q]] = x;
            }
        }
        __syncthreads();  // the LDS is rewritten by the next bin
    }
}

// kFinal false: each workgroup reduces its `per` consecutive keys (a multiple of kBinWG: each
// thread keeps a running union while its keys stay in one object) and publishes; true: one
// workgroup combines.  (One workgroup per 256 keys put ~8k atomics of C5's four-camera build on
// one line: 330 us.)
template <bool kFinal>
__global__ void __launch_bounds__(kBinWG) bins_finalize_kernel(uint32_t per, const uint32_t* __restrict__ start, uint32_t nb,
                                                               uint32_t bins_x, uint32_t nbins, uint32_t W, uint32_t H,
                                                               uint32_t phase, uint32_t* __restrict__ acc,
                                                               uint32_t* __restrict__ part,
                                                               uint32_t* __restrict__ done, uint32_t* __restrict__ n,
                                                               uint32_t cap, const uint32_t* __restrict__ kobj,
                                                               ObjectDesc* __restrict__ objs, const BinEntry* ent,
                                                               uint32_t* __restrict__ count,
                                                               uint32_t* __restrict__ sortq, uint32_t* __restrict__ nsort,
                                                               CamState* __restrict__ st, uint32_t ncam,
                                                               int32_t* __restrict__ path_union, uint32_t union_nobj) {
    __shared__ uint32_t s_acc[kFinSpan][4];
    __shared__ uint32_t s_tab[kFinal ? kFinTab : 1][4];
    const uint32_t keys = nb * nbins;
    const uint32_t b0 = kFinal ? 0u : blockIdx.x * per, b1 = kFinal ? 0u : min(b0 + per, keys);
    const uint32_t k_first = b0 < b1 ? b0 / nbins : 0u, k_last = b0 < b1 ? (b1 - 1) / nbins : 0u;
    if (threadIdx.x < kFinSpan * 4) s_acc[threadIdx.x / 4][threadIdx.x % 4] = 0u;
    __syncthreads();
    if constexpr (!kFinal) {
        uint32_t kc = ~0u, a[4] = {0u, 0u, 0u, 0u};  // this thread's union of object kc's bins so far
        auto flush = [&]() {
            if (kc == ~0u) return;
            if (kc - k_first < kFinSpan) max4(s_acc[kc - k_first], a);
            else max4(acc + kAccStride * kc, a);
        };
        for (uint32_t b = b0 + threadIdx.x; b < b0 + per; b += kBinWG) {  // workgroup-uniform trip count
            if (b < b1) count[b] = 0u;  // (the scatter has read the ranks: zero for the next camera)
            if (b < b1 && start[b + 1] > start[b]) {
                const uint32_t k = b / nbins;
                const uint32_t lb = b - k * nbins;
                const uint32_t bx = lb % bins_x, by = lb / bins_x;
                const int32_t y0 = (int32_t)(by * kBinH + phase) - (int32_t)kBinH;
                const uint32_t x0 = bx * kBinW, x1 = min(x0 + kBinW, W) - 1;
                const uint32_t r0 = (uint32_t)max(y0, 0), r1 = (uint32_t)min(y0 + (int32_t)kBinH, (int32_t)H) - 1;
                const uint32_t w[4] = {~x0, x1 + 1u, ~r0, r1 + 1u};
                if (k != kc) {
                    flush();
                    kc = k;
                    for (int q = 0; q < 4; ++q) a[q] = 0u;
                }
                for (int q = 0; q < 4; ++q) a[q] = max(a[q], w[q]);
            }
            queue_sort(start, b, keys, sortq, nsort);
        }
        flush();
    }
    __syncthreads();
    // this workgroup's objects' unions into the accumulators: only workgroups with a non-empty
    // bin, four atomics per object (a single combining workgroup reading every workgroup's
    // partials took 28 us at 16 cameras x 32k bins)
    const uint32_t span = !kFinal && b0 < b1 ? min(k_last - k_first + 1, kFinSpan) : 0u;
    if (threadIdx.x < span && s_acc[threadIdx.x][1] != 0u) {
        const uint32_t a[4] = {s_acc[threadIdx.x][0], s_acc[threadIdx.x][1], s_acc[threadIdx.x][2], s_acc[threadIdx.x][3]};
        max4(acc + kAccStride * (k_first + threadIdx.x), a);
    }
    if (!kFinal) return;
    const bool in_lds = nb <= kFinTab;
    if (in_lds) {
        for (uint32_t j = threadIdx.x; j < nb; j += kBinWG)
            for (int q = 0; q < 4; ++q) {
                s_tab[j][q] = acc[kAccStride * j + q];
                acc[kAccStride * j + q] = 0u;
            }
        __syncthreads();
    }
    __syncthreads();
    // the shards' counts: an overflow if any shard outgrew its region; the entries needed for the
    // capacity are the fullest shard's times kShards
    uint32_t found = 0, fullest = 0;
    for (uint32_t sh = 0; sh < kShards; ++sh) {
        const uint32_t c = n[sh * kShardStride];
        found += c;
        fullest = max(fullest, c);
    }
    const bool overflow = fullest > cap / kShards;
    const uint32_t need = max(found, fullest * kShards);
    for (uint32_t j = threadIdx.x; j < nb; j += kBinWG) {
        uint32_t w[4];
        for (int q = 0; q < 4; ++q) w[q] = in_lds ? s_tab[j][q] : atomicExch(acc + kAccStride * j + q, 0u);
        ObjGeom& g = objs[kobj[j]].g;
        if (overflow) {  // keep the face rectangles; the frame kernel scans through LDS tiles
            g.bin_start = nullptr;
            g.bin_ent = nullptr;
            if (path_union) union_rect(path_union, union_nobj, kobj[j] % union_nobj, g.rect);
            continue;
        }
        // a pixel of an empty bin has no face whose culling bounds can pass there (bin_pixels),
        // so no primary ray hits the object: its rectangle narrows to the non-empty bins
        int32_t* r = g.rect;
        if (w[1] == 0) {
            r[0] = r[2] = 1;
            r[1] = r[3] = 0;
        } else {
            r[0] = max(r[0], (int32_t)~w[0]);
            r[1] = min(r[1], (int32_t)w[1] - 1);
            r[2] = max(r[2], (int32_t)~w[2]);
            r[3] = min(r[3], (int32_t)w[3] - 1);
        }
        if (path_union) union_rect(path_union, union_nobj, kobj[j] % union_nobj, r);
        g.bin_start = start + (size_t)j * nbins;
        g.bin_ent = ent;
    }
    __syncthreads();  // (every thread has read the counts)
    if (threadIdx.x < kShards) n[threadIdx.x * kShardStride] = 0u;
    if (threadIdx.x == 0) {
        nsort[0] = nsort[1] = 0u;  // (bin_sort_kernel has run)
        // the most entries any setup needed since the buffers were allocated (the host grows the
        // capacity from it), and whether any overflowed
        for (uint32_t k = 0; k < ncam; ++k) {  // (several cameras: every camera's state)
            st[k].bin_entries = max(st[k].bin_entries, need);
            st[k].bin_overflow |= overflow ? 1u : 0u;
            st[k].nrect = 0u;
            st[k].total_sub = 0u;  // counted by detail_list_kernel
            st[k].heavy_sub = 0u;
            st[k].light_sub = 0u;
        }
    }
}

// Sub-block s = sy * (4 * tiles_x) + sx (padded rows: a 64 x 4 block's four sub-blocks are four
// consecutive threads): listed when some object can be hit there — a binned object's bin is
// non-empty (the frame kernel's bin of the sub-block, first_hit_binned) or another object's pixel
// rectangle reaches it.  Ordered form (one-camera setups): flags, then device-wide compactions in
// raster order — first the heavy sub-blocks (a bin of more than one 64-entry chunk), then the
// others.  The frame kernel deals the list out in rounds of one sub-block per detail wave, so the
// heavy ones go in the first round and the last round holds only one-chunk sub-blocks
// (3840x2160 / 70k: two rounds, and the second one's slowest workgroups set the frame's end,
// profiles/r02/trace/).  Any order gives the same image.
__global__ void __launch_bounds__(kBinWG) detail_flags_kernel(const ObjectDesc* __restrict__ objs, uint32_t nobj,
                                                              uint32_t cam_w, uint32_t row0, uint32_t rows,
                                                              uint32_t band_shift, uint32_t band_mask,
                                                              uint32_t band_stride,
                                                              uint32_t bins_x, uint32_t phase, uint32_t tiles_x,
                                                              uint32_t n, uint32_t heavy_min, uint8_t* __restrict__ flags,
                                                              uint8_t* __restrict__ flags_light,
                                                              uint32_t* __restrict__ packed, uint8_t* __restrict__ occ) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t row_subs = 4 * tiles_x;
    const uint32_t sx = s % row_subs, sy = s / row_subs;
    bool hit = false, heavy = false;
    if (s < n && sx * kBinW < cam_w) {
        const int32_t x0 = (int32_t)(sx * kBinW), x1 = x0 + (int32_t)kBinW - 1;
        // the sub-block's camera rows (one band: bands are multiples of kBinH rows)
        const int32_t y0 = (int32_t)band_camera_row(row0, band_shift, band_mask, band_stride, sy * kBinH);
        const int32_t y1 = y0 + (int32_t)min(kBinH, rows - sy * kBinH) - 1;
        for (uint32_t oi = 0; oi < nobj && !hit; ++oi) {
            const ObjGeom& g = objs[oi].g;
            if (!g.tri_count) continue;
            if (g.bin_start) {
                const uint32_t bin = (((uint32_t)y0 + kBinH - phase) / kBinH) * bins_x + sx;
                hit = g.bin_start[bin + 1] > g.bin_start[bin];
                heavy = g.bin_start[bin + 1] - g.bin_start[bin] > heavy_min;
            } else {
                hit = x0 <= g.rect[1] && x1 >= g.rect[0] && y0 <= g.rect[3] && y1 >= g.rect[2];
            }
        }
    }
    if (s < n) {
        flags[s] = (hit && heavy) ? 1 : 0;
        flags_light[s] = (hit && !heavy) ? 1 : 0;
        packed[s] = (sy << 16) | sx;
    }
    // the block's four flags: lanes 4b .. 4b + 3 of the wave (row_subs is a multiple of 4)
    const unsigned long long bal = __ballot(hit);
    if (s < n && (threadIdx.x & 3) == 0) occ[s / 4] = (uint8_t)((bal >> (threadIdx.x & 63)) & 0xfu);
}

// Appended form (camera paths: one launch instead of four): the same flags, the listed sub-blocks
// appended with one counter atomic per workgroup and kind — heavy ones (a bin of more than one
// 64-entry chunk) from the front of the camera's list, light ones from its back — so the frame
// kernel still deals the heavy sub-blocks first and searches the light ones one wave each
// (FrameParams::dlist_split; unordered, every sub-block was shared by a workgroup: the moving
// 3840x2160 / 70k frame kernel ran 40 us against 22.6 static).  The counts land in CamState
// (total_sub, heavy_sub, light_sub; zeroed by the finaliser).  (Carrying the bin range in the
// entry, one scalar load fewer per sub-block, measured slower: C3 +0.3 us, 3840x2160 / 70k +1 us.)
__global__ void __launch_bounds__(kBinWG) detail_list_kernel(const ObjectDesc* __restrict__ objs, uint32_t nobj,
                                                             uint32_t cam_w, uint32_t row0, uint32_t rows,
                                                             uint32_t band_shift, uint32_t band_mask,
                                                             uint32_t band_stride, uint32_t bins_x, uint32_t phase,
                                                             uint32_t tiles_x, uint32_t n,
                                                             uint32_t* __restrict__ list, uint8_t* __restrict__ occ,
                                                             CamState* __restrict__ st) {
    __shared__ uint32_t s_cnt[2][kBinWG / 64];
    __shared__ uint32_t s_base[2];
    // camera blockIdx.y of a multi-camera setup: its descriptors, list, occupancy and counts
    objs += (size_t)blockIdx.y * nobj;
    list += (size_t)blockIdx.y * n;
    occ += (size_t)blockIdx.y * (n / 4);
    CamState& cs = st[blockIdx.y];
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t row_subs = 4 * tiles_x;
    const uint32_t sx = s % row_subs, sy = s / row_subs;
    bool hit = false, heavy = false;
    if (s < n && sx * kBinW < cam_w) {
        const int32_t x0 = (int32_t)(sx * kBinW), x1 = x0 + (int32_t)kBinW - 1;
        // the sub-block's camera rows (one band: bands are multiples of kBinH rows)
        const int32_t y0 = (int32_t)band_camera_row(row0, band_shift, band_mask, band_stride, sy * kBinH);
        const int32_t y1 = y0 + (int32_t)min(kBinH, rows - sy * kBinH) - 1;
        for (uint32_t oi = 0; oi < nobj; ++oi) {
            const ObjGeom& g = objs[oi].g;
            if (!g.tri_count) continue;
            if (g.bin_start) {
                const uint32_t bin = (((uint32_t)y0 + kBinH - phase) / kBinH) * bins_x + sx;
                const uint32_t cnt = g.bin_start[bin + 1] - g.bin_start[bin];
                hit |= cnt != 0;
                heavy |= cnt > 64;
            } else {
                hit |= x0 <= g.rect[1] && x1 >= g.rect[0] && y0 <= g.rect[3] && y1 >= g.rect[2];
            }
        }
    }
    // the block's four flags: lanes 4b .. 4b + 3 of the wave (row_subs is a multiple of 4)
    const unsigned long long bal = __ballot(hit), bh = __ballot(hit && heavy), bl = bal & ~bh;
    if (s < n && (threadIdx.x & 3) == 0) occ[s / 4] = (uint8_t)((bal >> (threadIdx.x & 63)) & 0xfu);
    if (lane == 0) {
        s_cnt[0][wave] = (uint32_t)__popcll(bh);
        s_cnt[1][wave] = (uint32_t)__popcll(bl);
    }
    __syncthreads();
    uint32_t before[2] = {0u, 0u}, all[2] = {0u, 0u};
#pragma unroll
    for (uint32_t w = 0; w < kBinWG / 64; ++w)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            before[k] += w < wave ? s_cnt[k][w] : 0u;
            all[k] += s_cnt[k][w];
        }
    if (threadIdx.x == 0) {
        s_base[0] = all[0] ? atomicAdd(&cs.heavy_sub, all[0]) : 0u;
        s_base[1] = all[1] ? atomicAdd(&cs.light_sub, all[1]) : 0u;
        if (all[0] + all[1]) atomicAdd(&cs.total_sub, all[0] + all[1]);
    }
    __syncthreads();
    const uint32_t e = (sy << 16) | sx;
    const unsigned long long lt = (1ull << lane) - 1ull;
    if (hit && heavy) list[s_base[0] + before[0] + (uint32_t)__popcll(bh & lt)] = e;
    else if (hit) list[n - 1 - (s_base[1] + before[1] + (uint32_t)__popcll(bl & lt))] = e;
}

// The light sub-blocks after the heavy ones (ordered detail list); the list's length into CamState.
__global__ void __launch_bounds__(kBinWG) detail_append_kernel(const uint32_t* __restrict__ light,
                                                               const uint32_t* __restrict__ counts,
                                                               uint32_t* __restrict__ list, CamState* st) {
    const uint32_t heavy = counts[0], nl = counts[1];
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nl; i += gridDim.x * blockDim.x)
        list[heavy + i] = light[i];
    if (blockIdx.x == 0 && threadIdx.x == 0) st->total_sub = heavy + nl;
}

// Workgroups of kBinWG threads of kernel `k` resident at once on the device (occupancy API, per
// kernel slot), kPairGrid if unknown.
uint32_t resident_grid(const void* k, int slot) {
    static std::mutex mu;
    static int per_cu[3] = {-1, -1, -1}, cus = -1;
    std::lock_guard<std::mutex> lock(mu);
    if (cus < 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 0;
    }
    if (per_cu[slot] < 0 && hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu[slot], k, kBinWG, 0) != hipSuccess)
        per_cu[slot] = 0;
    return cus > 0 && per_cu[slot] > 0 ? (uint32_t)(cus * per_cu[slot]) : kPairGrid;
}

template <typename T>
hipError_t grow(T** p, size_t need) {
    if (*p) {
        hipError_t e = hipFree(*p);
        if (e != hipSuccess) return e;
        *p = nullptr;
    }
    return hipMalloc((void**)p, (need ? need : 1) * sizeof(T));
}

}  // namespace

void bins_free(BinBuffers& b) {
    void* ptrs[] = {b.first, b.boff, b.count,  b.start,  b.kbegin, b.kobj,   b.n,       b.done,    b.acc,   b.part, b.ekey,
                    b.eface, b.emask,  b.erank,  b.ent,    b.dflags,  b.dpacked, b.dlist, b.docc,
                    b.sortq, b.nsort,  b.temp,   b.dflags_light, b.dlight, b.dcount};
    for (void* p : ptrs)
        if (p) hipFree(p);
    b = BinBuffers{};
}

hipError_t bins_alloc(BinBuffers& b, uint32_t T, uint32_t nb, const uint32_t* kbegin, const uint32_t* kobj, uint32_t W,
                      uint32_t H, uint32_t phase, uint32_t tiles_x, uint32_t rows, size_t cap, hipStream_t s,
                      uint32_t ncam) {
    hipError_t e = hipStreamSynchronize(s);  // the buffers may be in use by enqueued work
    if (e != hipSuccess) return e;
    bins_free(b);
    b.nb = nb;
    b.T = T;
    b.bins_x = (W + kBinW - 1) / kBinW;
    b.bins_y = H ? (H - 1 + kBinH - phase) / kBinH + 1 : 1;
    b.nbins = b.bins_x * b.bins_y;
    b.phase = phase;
    b.cap = cap;
    const size_t keys = (size_t)nb * b.nbins;
    const uint32_t subs_y = (rows + kBinH - 1) / kBinH;
    b.nsub = 4 * (size_t)tiles_x * subs_y;
    if ((e = grow(&b.first, T)) != hipSuccess || (e = grow(&b.boff, kSetupMaxBlocks + 1)) != hipSuccess || (e = grow(&b.count, keys + 1)) != hipSuccess ||
        (e = grow(&b.start, keys + 1)) != hipSuccess || (e = grow(&b.kbegin, nb)) != hipSuccess ||
        (e = grow(&b.kobj, nb)) != hipSuccess || (e = grow(&b.n, kShards * kShardStride)) != hipSuccess ||
        (e = grow(&b.done, 1)) != hipSuccess || (e = grow(&b.acc, kAccStride * (size_t)nb)) != hipSuccess ||
        (e = grow(&b.part, 10 * std::max<size_t>((keys + kBinWG - 1) / kBinWG, 1))) != hipSuccess ||
        (e = grow(&b.ekey, cap)) != hipSuccess || (e = grow(&b.eface, cap)) != hipSuccess ||
        (e = grow(&b.emask, cap)) != hipSuccess || (e = grow(&b.erank, cap)) != hipSuccess || (e = grow(&b.ent, cap)) != hipSuccess ||
        (e = grow(&b.dflags, b.nsub)) != hipSuccess || (e = grow(&b.dpacked, b.nsub)) != hipSuccess ||
        (e = grow(&b.dflags_light, b.nsub)) != hipSuccess || (e = grow(&b.dlight, b.nsub)) != hipSuccess ||
        (e = grow(&b.dcount, 2)) != hipSuccess ||
        (e = grow(&b.dlist, b.nsub * ncam)) != hipSuccess ||
        (e = grow(&b.docc, (size_t)tiles_x * subs_y * ncam)) != hipSuccess ||
        (e = grow(&b.sortq, std::max<size_t>(keys, 1))) != hipSuccess || (e = grow(&b.nsort, 2)) != hipSuccess)
        return e;
    // counters zero between builds (each build leaves them so)
    if ((e = hipMemsetAsync(b.count, 0, sizeof(uint32_t) * (keys + 1), s)) != hipSuccess ||
        (e = hipMemsetAsync(b.n, 0, sizeof(uint32_t) * kShards * kShardStride, s)) != hipSuccess ||
        (e = hipMemsetAsync(b.nsort, 0, 2 * sizeof(uint32_t), s)) != hipSuccess ||
        (e = hipMemsetAsync(b.done, 0, sizeof(uint32_t), s)) != hipSuccess ||
        (e = hipMemsetAsync(b.acc, 0, sizeof(uint32_t) * kAccStride * nb, s)) != hipSuccess ||
        (e = hipMemcpyAsync(b.kbegin, kbegin, sizeof(uint32_t) * nb, hipMemcpyHostToDevice, s)) != hipSuccess ||
        (e = hipMemcpyAsync(b.kobj, kobj, sizeof(uint32_t) * nb, hipMemcpyHostToDevice, s)) != hipSuccess)
        return e;
    // hipcub scratch: the larger of the two device-wide passes
    size_t t1 = 0, t2 = 0, t3 = 0;
    if ((e = hipcub::DeviceScan::ExclusiveSum(nullptr, t2, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)(keys + 1), s)) !=
            hipSuccess ||
        (e = hipcub::DeviceSelect::Flagged(nullptr, t3, (uint32_t*)nullptr, (uint8_t*)nullptr, (uint32_t*)nullptr,
                                           (uint32_t*)nullptr, (int)std::max<size_t>(b.nsub, 1), s)) != hipSuccess)
        return e;
    b.temp_bytes = std::max(std::max(t1, t2), t3);
    if ((e = hipMalloc(&b.temp, b.temp_bytes ? b.temp_bytes : 1)) != hipSuccess) return e;
    return hipStreamSynchronize(s);  // the host arrays above are the caller's
}

hipError_t launch_bins_build(const SetupParams& sp, BinBuffers& b, uint32_t tiles_x, bool ordered, hipStream_t s) {
    hipError_t e;
    const size_t keys = (size_t)b.nb * b.nbins;
    size_t tb = b.temp_bytes;
    const bool multi = sp.ncam > 1;
    const uint32_t ncam = multi ? sp.ncam : 1u;
    if (sp.T) {  // (a multi-camera build may set up fewer cameras than the buffers hold)
        const uint32_t nparts = setup_blocks(sp.T), chunk = (sp.T + nparts - 1) / nparts;  // as camera_setup_kernel
        auto* k = bin_segments(sp) ? bin_segments_kernel : sp.keep_all ? bin_pairs_kernel<true> : bin_pairs_kernel<false>;
        // exactly the resident workgroups (each wave walks a fixed share of the units: a second
        // round of workgroups would double the pass)
        const uint32_t pgrid = resident_grid(reinterpret_cast<const void*>(k), bin_segments(sp) ? 2 : sp.keep_all ? 1 : 0);
        k<<<pgrid, kBinWG, 0, s>>>(sp.cull, sp.range, b.first, b.boff, nparts, chunk, sp.fkey, sp.T, sp.W, sp.H, sp.phase,
                                       b.bins_x, b.nbins, (uint32_t)b.cap, b.n, b.count, b.ekey, b.eface, b.emask, b.erank);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    tb = b.temp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(b.temp, tb, b.count, b.start, (int)(keys + 1), s)) != hipSuccess) return e;
    bin_scatter_kernel<<<kPairGrid, kBinWG, 0, s>>>(b.n, (uint32_t)b.cap, b.ekey, b.eface, b.emask, b.erank, b.start,
                                                    b.kbegin, b.nbins, sp.hot, multi ? sp.T1 : 0u, b.ent);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // at most kFinGrid workgroups, each over `per` consecutive keys
    const uint32_t per = (uint32_t)std::max<size_t>(kBinWG, (keys + (size_t)kFinGrid * kBinWG - 1) / ((size_t)kFinGrid * kBinWG) * kBinWG);
    const uint32_t fgrid = (uint32_t)std::max<size_t>((keys + per - 1) / per, 1);
    bins_finalize_kernel<false><<<fgrid, kBinWG, 0, s>>>(per, b.start, b.nb, b.bins_x, b.nbins, sp.W, sp.H, b.phase,
                                                         b.acc, b.part, b.done, b.n, (uint32_t)b.cap, b.kobj, sp.objs,
                                                         b.ent, b.count, b.sortq, b.nsort, sp.state, ncam, nullptr, 1u);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    bin_sort_kernel<<<kSortGrid, kBinWG, 0, s>>>(b.sortq, b.nsort, b.start, b.ent, (uint32_t)keys);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    bins_finalize_kernel<true><<<1, kBinWG, 0, s>>>(per, b.start, b.nb, b.bins_x, b.nbins, sp.W, sp.H, b.phase, b.acc,
                                                    b.part, b.done, b.n, (uint32_t)b.cap, b.kobj, sp.objs, b.ent, b.count,
                                                    b.sortq, b.nsort, sp.state, ncam, sp.path_union,
                                                    sp.union_nobj ? sp.union_nobj : 1u);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (!b.nsub) return hipSuccess;
    const uint32_t n = (uint32_t)b.nsub;
    if (ordered) {
        detail_flags_kernel<<<(n + kBinWG - 1) / kBinWG, kBinWG, 0, s>>>(sp.objs, sp.nobj, sp.W, sp.row0, sp.rows,
                                                                        sp.band_shift, sp.band_mask, sp.band_stride,
                                                                        b.bins_x, b.phase, tiles_x, n, sp.keep_all ? kTraceHeavyMin : 64u, b.dflags,
                                                                        b.dflags_light, b.dpacked, b.docc);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        tb = b.temp_bytes;
        if ((e = hipcub::DeviceSelect::Flagged(b.temp, tb, b.dpacked, b.dflags, b.dlist, b.dcount, (int)n, s)) !=
            hipSuccess)
            return e;
        tb = b.temp_bytes;
        if ((e = hipcub::DeviceSelect::Flagged(b.temp, tb, b.dpacked, b.dflags_light, b.dlight, b.dcount + 1, (int)n,
                                               s)) != hipSuccess)
            return e;
        detail_append_kernel<<<std::max<uint32_t>(1u, std::min<uint32_t>(1024u, (n + kBinWG - 1) / kBinWG)), kBinWG, 0,
                               s>>>(b.dlight, b.dcount, b.dlist, sp.state);
        return hipGetLastError();
    }
    detail_list_kernel<<<dim3((n + kBinWG - 1) / kBinWG, ncam), kBinWG, 0, s>>>(
        sp.objs, multi ? sp.nobj1 : sp.nobj, sp.W, sp.row0, sp.rows, sp.band_shift, sp.band_mask, sp.band_stride, b.bins_x,
        b.phase, tiles_x, n, b.dlist, b.docc, sp.state);
    return hipGetLastError();
}

}  // namespace gpu
}  // namespace eray
