// face_rect.hpp — conservative pixel rectangle of a face from its culling record (device).
#pragma once

#include "internal.hpp"

namespace eray {
namespace gpu {

// The culling records also bound where a face can be hit at all: condition k can only pass at
// viewport points with K_k + A_k x' + B_k y' >= -T_k (x' = x / W, y' = y / H, camera_dir).
// Clipping the viewport square by the four half-planes (double precision; each relaxed by 1e-9
// of its magnitude, far above the clip's rounding, so the computed polygon contains the exact
// one) and widening its bounding box by 1 pixel (x' is the reference's f32 x/W, within a relative
// 2^-24 of x/W: far less than a pixel) gives a conservative pixel rectangle per face.  The
// object's rectangle is the union: no primary ray outside it can hit the object, so those pixels
// need no test for it.
// The polygon (at most 8 vertices: 4 + one per clip) is held in registers (fully unrolled, so
// every vertex index is a compile-time constant); only a clip's output, whose positions depend on
// the data, goes through the caller's LDS workspace `ws` (2 arrays of 8 doubles, element k of
// array a at ws[(a * 8 + k) * stride]) and is read back in one round trip per clip.  (As private
// arrays with run-time indices the polygon lived in scratch memory, and as an LDS polygon read
// vertex by vertex each clip was a chain of LDS round trips.)
// The bounding box [xmin, xmax] x [ymin, ymax] of the viewport points of the box [bx0, bx1] x
// [by0, by1] where every condition of record c can pass; false when there are none.
// Fast path (a face whose relaxed edge half-planes meet in a triangle inside the box and inside
// the det half-plane — every face of a mesh in view but the ones crossing the frame's edge or
// grazing the view): conditions 0..2 (u >= 0, v >= 0, u + v <= 1) are the face's edges, so the
// three pairwise intersections of their relaxed lines are the polygon's vertices when each lies on
// the inner side of the third line (then the three inward normals span the plane: the region is
// that bounded triangle), inside the box and in condition 3's half-plane (convexity: the whole
// triangle is).  The clip would return the same polygon; its box comes from three 2 x 2 solves
// instead of four clips (camera_setup_kernel is VALU bound on them: ~1250 instructions per face).
// Vertices computed within ~1e-15 of the relaxed ones stay far inside the 1e-9 relaxation; a
// vertex whose check fails by rounding only sends the face to the clip (and a vertex rounded into
// the box or condition 3's half-plane only widens the box: bbox(triangle) contains the clip's).
__device__ inline bool tri_box(const double (&a)[4], const double (&b)[4], const double (&cc)[4], double bx0, double bx1,
                               double by0, double by1, double& xmin, double& xmax, double& ymin, double& ymax) {
    double vx[3], vy[3];
#pragma unroll
    for (int e = 0; e < 3; ++e) {  // vertex e: lines e and e + 1 (mod 3); the third line is e + 2
        const int i = e, j = (e + 1) % 3, k = (e + 2) % 3;
        const double det = a[i] * b[j] - a[j] * b[i];
        if (!(fabs(det) > 1e-12 * (fabs(a[i] * b[j]) + fabs(a[j] * b[i])))) return false;  // (near-)parallel
        const double x = (b[i] * cc[j] - b[j] * cc[i]) / det, y = (a[j] * cc[i] - a[i] * cc[j]) / det;
        // strictly inside the third line, beyond rounding (three nearly concurrent lines, whose
        // signs rounding could flip, leave for the clip: their region may be an unbounded wedge)
        const double fk = a[k] * x + b[k] * y + cc[k];
        if (!(fk > 1e-12 * (fabs(a[k] * x) + fabs(b[k] * y) + fabs(cc[k])))) return false;
        if (!(a[3] * x + b[3] * y + cc[3] >= 0.0)) return false;
        if (!(x >= bx0 && x <= bx1 && y >= by0 && y <= by1)) return false;
        vx[e] = x;
        vy[e] = y;
    }
    xmin = fmin(fmin(vx[0], vx[1]), vx[2]);
    xmax = fmax(fmax(vx[0], vx[1]), vx[2]);
    ymin = fmin(fmin(vy[0], vy[1]), vy[2]);
    ymax = fmax(fmax(vy[0], vy[1]), vy[2]);
    return true;
}

// (try_tri: the fast path first — for boxes that usually hold whole faces, the viewport)
__device__ inline bool clip_box(const TriCull& c, double bx0, double bx1, double by0, double by1, double* ws,
                                uint32_t stride, double& xmin, double& xmax, double& ymin, double& ymax,
                                bool try_tri = false) {
    constexpr int kMax = 8;
    const float A[4] = {c.A.x, c.A.y, c.A.z, c.A.w}, B[4] = {c.B.x, c.B.y, c.B.z, c.B.w};
    const float K[4] = {c.K.x, c.K.y, c.K.z, c.K.w}, T[4] = {c.T.x, c.T.y, c.T.z, c.T.w};
    if (try_tri) {
        bool finite = true;
        double fa[4], fb[4], fc[4];  // the clip's relaxed lines, as below
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            finite = finite && T[k] < __builtin_inff() && T[k] > -__builtin_inff();
            fa[k] = A[k];
            fb[k] = B[k];
            const double mag = fabs((double)K[k]) + fabs(fa[k]) + fabs(fb[k]) + fabs((double)T[k]);
            fc[k] = (double)K[k] + (double)T[k] + 1e-9 * mag + 1e-300;
        }
        if (finite && tri_box(fa, fb, fc, bx0, bx1, by0, by1, xmin, xmax, ymin, ymax)) return true;
    }
    double* qx = ws;
    double* qy = ws + kMax * stride;
    double px[kMax] = {bx0, bx1, bx1, bx0, 0.0, 0.0, 0.0, 0.0};
    double py[kMax] = {by0, by0, by1, by1, 0.0, 0.0, 0.0, 0.0};
    int n = 4;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (T[k] == __builtin_inff()) continue;  // condition disabled (non-finite record)
        if (!(T[k] > -__builtin_inff())) return false;  // the face rejects every camera ray
        const double a = A[k], b = B[k];
        const double mag = fabs((double)K[k]) + fabs(a) + fabs(b) + fabs((double)T[k]);
        const double cc = (double)K[k] + (double)T[k] + 1e-9 * mag + 1e-300;
        double f[kMax];
#pragma unroll
        for (int i = 0; i < kMax; ++i) f[i] = a * px[i] + b * py[i] + cc;
        int m = 0;
#pragma unroll
        for (int i = 0; i < kMax; ++i) {
            if (i >= n) break;
            const bool last = i + 1 == n;  // edge i -> i + 1 (the last edge closes the polygon)
            const double xj = last ? px[0] : px[(i + 1) % kMax], yj = last ? py[0] : py[(i + 1) % kMax];
            const double fi = f[i], fj = last ? f[0] : f[(i + 1) % kMax];
            if (fi >= 0.0) {
                qx[m * stride] = px[i];
                qy[m * stride] = py[i];
                ++m;
            }
            if ((fi >= 0.0) != (fj >= 0.0)) {
                double t = fi / (fi - fj);
                t = t < 0.0 ? 0.0 : (t > 1.0 ? 1.0 : t);
                qx[m * stride] = px[i] + t * (xj - px[i]);
                qy[m * stride] = py[i] + t * (yj - py[i]);
                ++m;
            }
        }
        n = m;
        if (!n) return false;
#pragma unroll
        for (int i = 0; i < kMax; ++i)
            if (i < n) {
                px[i] = qx[i * stride];
                py[i] = qy[i * stride];
            }
    }
    xmin = px[0];
    xmax = px[0];
    ymin = py[0];
    ymax = py[0];
#pragma unroll
    for (int i = 1; i < kMax; ++i)
        if (i < n) {
            xmin = fmin(xmin, px[i]);
            xmax = fmax(xmax, px[i]);
            ymin = fmin(ymin, py[i]);
            ymax = fmax(ymax, py[i]);
        }
    return true;
}

// (xa, ya): the viewport's lower corner — (0, 0) for the camera rays of the pixel corners; the
// general tracer's jittered rays reach x' = -1/W, y' = -1/H in column and row 0 (its setup passes
// (-2/W, -2/H) and records computed for that range, cull_record.hpp).
__device__ inline bool face_rect(const TriCull& c, uint32_t W, uint32_t H, int32_t (&r)[4], double* ws,
                                 uint32_t stride, double xa = 0.0, double ya = 0.0) {
    double xmin, xmax, ymin, ymax;
    if (!clip_box(c, xa, 1.0, ya, 1.0, ws, stride, xmin, xmax, ymin, ymax, true)) return false;
    r[0] = max((int32_t)floor(xmin * W) - 1, 0);
    r[1] = min((int32_t)ceil(xmax * W) + 1, (int32_t)W - 1);
    r[2] = max((int32_t)floor(ymin * H) - 1, 0);
    r[3] = min((int32_t)ceil(ymax * H) + 1, (int32_t)H - 1);
    return r[0] <= r[1] && r[2] <= r[3];
}

// Where condition k of a culling record can pass along a camera row, in pixels: from
// K + A xf + B yf >= -T (the culling bound at the pixel's own f32 viewport coordinates), solved
// for xf in double: x >= c0 - c1 yf (A > 0) or x <= c0 - c1 yf (A < 0), widened by `tol` pixels:
// the f32 xf = x/W is within a relative 2^-24 of x/W (at most W * 2^-24 < 1e-3 pixel for any
// W < 16.7M) and the double solve is within ~1e-15 (|c0| + |c1|) pixels, so 1e-3 + 1e-12 (|c0| +
// |c1|) contains every pixel whose bound can pass, without the whole-pixel widening that would
// add false (face, pixel) pairs around every small face.  A condition nearly independent of x is
// decided per row from its x-free part (kind 3); a disabled one (T = +inf) does not narrow the
// interval (kind 0).
struct CondLine {
    double c0, c1, tol;
    int kind;  // 0 none, 1 lower bound x >= c0 - c1 yf, 2 upper bound, 3 flat: fails if c0 - c1 yf > tol
};
__device__ inline CondLine cond_line(float A, float B, float K, float T, uint32_t W) {
    CondLine l{0.0, 0.0, 0.0, 0};
    if (!(T < __builtin_inff())) return l;
    const double mag = fabs((double)K) + fabs((double)T) + fabs((double)B) + 1e-300;
    if (fabs((double)A) <= 1e-9 * mag) {
        // A xf >= R(yf) with |A xf| <= 1e-9 mag: the row fails only when R exceeds that
        l.c0 = -((double)K + (double)T);
        l.c1 = (double)B;
        l.tol = 2e-9 * mag;
        l.kind = 3;
        return l;
    }
    const double inv = (double)W / (double)A;
    l.c0 = -((double)K + (double)T) * inv;
    l.c1 = (double)B * inv;
    l.tol = 1e-3 + 1e-12 * (fabs(l.c0) + fabs(l.c1));
    l.kind = A > 0.0f ? 1 : 2;
    return l;
}
// Row r of bin row `by` (camera row y = by * kBinH + phase + r - kBinH; yf the reference's f32
// y / H, camera_dir): the columns [xl, xr] of [x_lo, x_hi] where all four lines can pass; false
// when there are none.  (apply_line's cases as selects: lanes hold pairs of different faces,
// whose condition kinds differ — branches diverged 3 ways per condition and row.)
__device__ inline bool row_span(const CondLine (&l)[4], uint32_t H, uint32_t phase, uint32_t by, uint32_t r,
                                int32_t x_lo, int32_t x_hi, int32_t& xl_out, int32_t& xr_out) {
    const int32_t y = (int32_t)(by * kBinH + phase + r) - (int32_t)kBinH;
    const double yf = (double)((float)(uint32_t)y / (float)H);
    double xl = (double)x_lo, xr = (double)x_hi;
    bool fail = y < 0 || y >= (int32_t)H;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const double q = l[k].c0 - l[k].c1 * yf;
        const double lo = ceil(q - l[k].tol), hi = floor(q + l[k].tol);
        xl = (l[k].kind == 1 && lo > xl) ? lo : xl;
        xr = (l[k].kind == 2 && hi < xr) ? hi : xr;
        fail |= l[k].kind == 3 && q > l[k].tol;
    }
    if (fail || !(xl <= xr)) return false;  // (xl >= x_lo, xr <= x_hi)
    xl_out = (int32_t)xl;
    xr_out = (int32_t)xr;
    return true;
}
__device__ inline void cond_lines(const TriCull& c, uint32_t W, CondLine (&l)[4]) {
    l[0] = cond_line(c.A.x, c.B.x, c.K.x, c.T.x, W);
    l[1] = cond_line(c.A.y, c.B.y, c.K.y, c.T.y, W);
    l[2] = cond_line(c.A.z, c.B.z, c.K.z, c.T.z, W);
    l[3] = cond_line(c.A.w, c.B.w, c.K.w, c.T.w, W);
}
// bits [xl, xr] of a bin starting at column x_lo, in its row r (bit r * kBinW + column)
__device__ __forceinline__ unsigned long long row_bits(int32_t xl, int32_t xr, int32_t x_lo, uint32_t r) {
    const uint32_t n = (uint32_t)(xr - xl + 1), s = (uint32_t)(xl - x_lo);
    return (unsigned long long)((((n >= 32 ? 0xffffffffu : ((1u << n) - 1u)) << s) & 0xffffu)) << (kBinW * r);
}

// Pixels of the kBinW x kBinH bin at (bx, by) (camera columns bx*kBinW.., rows y0..y0+3 with
// y0 = by*kBinH + phase - kBinH) where all four conditions of record c can pass: bit
// r * kBinW + col.
__device__ inline unsigned long long bin_pixels(const TriCull& c, uint32_t W, uint32_t H, uint32_t phase,
                                                uint32_t bx, uint32_t by) {
    CondLine l[4];
    cond_lines(c, W, l);
    const int32_t x_lo = (int32_t)(bx * kBinW), x_hi = min((int32_t)((bx + 1) * kBinW), (int32_t)W) - 1;
    unsigned long long pix = 0;
#pragma unroll
    for (uint32_t r = 0; r < kBinH; ++r) {
        int32_t xl, xr;
        if (row_span(l, H, phase, by, r, x_lo, x_hi, xl, xr)) pix |= row_bits(xl, xr, x_lo, r);
    }
    return pix;
}

// The same rows over the columns [xa, xb] of a face's bin rectangle (bins.hip
// bin_segments_kernel): rr[r] = xl | xr << 16 (1: no column; columns < 65536), [lo, hi] the rows'
// extent (lo > hi: none).  A bin's bin_pixels mask is these ranges cut to its 16 columns
// (bin_mask_of_rows): the lines and each row's bounds are the same double values, and a bin's
// range is max / min of them with its own first / last column.
__device__ inline void row_ranges(const TriCull& c, uint32_t W, uint32_t H, uint32_t phase, uint32_t by, int32_t xa,
                                  int32_t xb, uint32_t (&rr)[kBinH], int32_t& lo, int32_t& hi) {
    CondLine l[4];
    cond_lines(c, W, l);
#pragma unroll
    for (uint32_t r = 0; r < kBinH; ++r) {
        int32_t xl, xr;
        rr[r] = 1u;
        if (row_span(l, H, phase, by, r, xa, xb, xl, xr)) {
            rr[r] = (uint32_t)xl | ((uint32_t)xr << 16);
            lo = min(lo, xl);
            hi = max(hi, xr);
        }
    }
}
__device__ __forceinline__ unsigned long long bin_mask_of_rows(const uint32_t (&rr)[kBinH], uint32_t bx) {
    const int32_t x_lo = (int32_t)(bx * kBinW), x_hi = x_lo + (int32_t)kBinW - 1;
    unsigned long long pix = 0;
#pragma unroll
    for (uint32_t r = 0; r < kBinH; ++r) {
        const int32_t xl = max((int32_t)(rr[r] & 0xffffu), x_lo), xr = min((int32_t)(rr[r] >> 16), x_hi);
        if (xl <= xr) pix |= row_bits(xl, xr, x_lo, r);
    }
    return pix;
}

// The same for the general tracer's rays (trace.hip): pixel (x, y) casts its corner ray and
// jittered ones through viewport points x' = fl(fl(x + jx) / W), y' likewise, jx, jy in [-1, 1):
// x' W within [x - 1, x + 1] up to e = 1e-3 + 2.4e-7 W pixels of rounding.  So pixel x of row y
// can have a ray whose conditions all pass only if the polygon where they can pass (clip_box,
// over the row's band [y - 1, y + 1] / H and the bin's columns widened by 1 + e) reaches x - 1 - e
// .. x + 1 + e: the pixels from ceil(xmin W - 1 - e) to floor(xmax W + 1 + e).  `ws`: clip_box's
// LDS workspace.
__device__ inline unsigned long long bin_pixels_jittered(const TriCull& c, uint32_t W, uint32_t H, uint32_t phase,
                                                         uint32_t bx, uint32_t by, double* ws, uint32_t stride) {
    const int32_t x_lo = (int32_t)(bx * kBinW), x_hi = min((int32_t)((bx + 1) * kBinW), (int32_t)W) - 1;
    const double e = 1e-3 + 2.4e-7 * (double)W, dW = (double)W, dH = (double)H;
    unsigned long long pix = 0;
    for (uint32_t r = 0; r < kBinH; ++r) {
        const int32_t y = (int32_t)(by * kBinH + phase + r) - (int32_t)kBinH;
        if (y < 0 || y >= (int32_t)H) continue;
        double xmin, xmax, ymin, ymax;
        if (!clip_box(c, ((double)x_lo - 1.0 - e) / dW, ((double)x_hi + 1.0 + e) / dW, ((double)y - 1.0) / dH - 3e-7,
                      ((double)y + 1.0) / dH + 3e-7, ws, stride, xmin, xmax, ymin, ymax))
            continue;
        const double lo = ceil(xmin * dW - 1.0 - e), hi = floor(xmax * dW + 1.0 + e);
        const int32_t xl = max(x_lo, (int32_t)fmax(lo, -1.0)), xr = min(x_hi, (int32_t)fmin(hi, 2e9));
        if (xl <= xr) {
            const uint32_t n = (uint32_t)(xr - xl + 1), s = (uint32_t)(xl - x_lo);
            pix |= (unsigned long long)((((n >= 32 ? 0xffffffffu : ((1u << n) - 1u)) << s) & 0xffffu)) << (kBinW * r);
        }
    }
    return pix;
}

}  // namespace gpu
}  // namespace eray
