// cull_record.hpp — per-camera culling record of one triangle (the frame kernel's exact wave
// culling, render.hip; the general tracer's background skip, trace.hip).
#pragma once
#include "device_math.hpp"
#include "internal.hpp"

namespace eray {
namespace gpu {

using namespace eray::dev;

// --------------------------------------------------------------------- culling record ------
// Derivation (u = 2^-24, all norms are 1-norms of the float inputs; d = normalised direction).
// The reference computes, in f32 from ao = C - a (C the camera centre),
//   det = -(d.n),  a_u = e2.(ao x d),  a_v = -(e1.(ao x d)),  u = a_u/det, v = a_v/det,
//   t = (ao.n)/det,  hit iff det >= 1e-6, t >= 0, u >= 0, v >= 0, u + v <= 1.
// In real arithmetic on the same float inputs these are linear in d:
//   det = d.(-n), a_u = d.w_u (w_u = e2 x ao), a_v = d.w_v (w_v = ao x e1), and
//   det - a_u - a_v = d.w_w (w_w = -(n + w_u + w_v)).
// Float evaluation errors (|d_i| <= 1 + 4u): |det_f - det| <= E_n = 4u|n|,
// |a_u_f - a_u| <= 8u|e2||ao|, |a_v_f - a_v| <= 8u|e1||ao|; an a_u within 2^-149|n| of 0 can
// still round u to -0 (accepted), hence the 2^-149|n| floors.  A hit needs u+v <= 1 after
// rounding, which implies d.w_w >= -(E_u + E_v + 1.01 E_n + 3.2u|n|).  So condition k certainly
// fails for direction d when d.w_k < -E_k.
// The camera's unnormalised direction is D(x', y') = (bl - C) + (vw x', 2y', 0) with bl, vw the
// reference's float viewport corner and width (camera.rs:57-76), so D.w_k = K + A x' + B y' is
// affine and its maximum over a pixel rectangle sits at a corner.  The reference's float
// direction differs from D/|D| by at most 4u S (S = |bl| + vw + 2 + |C|) before and 4u after
// normalisation, so condition k fails for every pixel of the rectangle when
//   max_rect (K + A x' + B y') < -T_k,
//   T_k = 2 * [ (E_k + 4u|w_k|) Dmax + 4u S |w_k| + 6u (|K| + |A| + |B|) ]
// (Dmax = largest |D| over the frame; factor 2 = safety).  For det the bound is tightened to the
// reference's own threshold: |D| det_f <= D.w_n + T_n / 2 and |D| >= |D_z| = |bl.z - C.z| (the
// z component of D is the same for every pixel), so det_f < 1e-6 for every pixel when
//   max_rect (K_n + A x' + B y') < 1e-6 |bl.z - C.z| - T_n
// — the faces that graze the view (det below 1e-6 but above 0: on the 1M-face stand-in, |n| ~ 2e-5,
// the band within ~3 degrees of edge-on) leave the bins and their pixel masks.  t >= 0 does not depend on d: when
// ao.n < -2^-149 |n| (or |n|(1+8u) < 1e-6) no camera ray can hit the face and the whole
// record rejects.  Any non-finite input disables culling for the face (T = +inf).
// `xa`..`yb`: the viewport coordinates the rays can take (the frame kernel's camera rays: x', y'
// in [0, 1]; trace.hip's jittered anti-aliasing rays reach -1/W and -1/H) — only Dmax depends on
// them, and |x'|, |y'| <= 1 is kept for the S and evaluation terms.
// The camera's part of the record (the same for every face): the reference's f32 viewport corner
// and width, the corner relative to the centre, the largest |D| over the x', y' range and the
// magnitude scale S.  (Per face it cost four double square roots.)
struct CullCam {
    float cx, cy, cz, vw;
    f3 bl;
    double blc[3];
    double dmax, S;
};
__device__ inline CullCam cull_cam(const CamDev& cam, double xa = 0.0, double xb = 1.0, double ya = 0.0,
                                   double yb = 1.0) {
    const double u = 0x1p-24;
    CullCam c;
    c.cx = cam.cx;
    c.cy = cam.cy;
    c.cz = cam.cz;
    const f3 Cf = mk3(c.cx, c.cy, c.cz);
    // camera.rs:57-76 in f32, as the reference computes it
    c.vw = cam.ratio * 2.0f;
    c.bl = sub(sub(sub(Cf, divs(mk3(c.vw, 0.0f, 0.0f), 2.0f)), divs(mk3(0.0f, 2.0f, 0.0f), 2.0f)),
               mk3(0.0f, 0.0f, cam.z_dist));
    c.blc[0] = (double)c.bl.x - c.cx;
    c.blc[1] = (double)c.bl.y - c.cy;
    c.blc[2] = (double)c.bl.z - c.cz;
    // largest |D| over the frame (corners of the x', y' range) and the magnitude scale S
    double dmax = 0.0;
    for (int cxr = 0; cxr < 2; ++cxr)
        for (int cyr = 0; cyr < 2; ++cyr) {
            const double xc = cxr ? xb : xa, yc = cyr ? yb : ya;
            double D0 = c.blc[0] + (double)c.vw * xc, D1 = c.blc[1] + 2.0 * yc, D2 = c.blc[2];
            double l = sqrt(D0 * D0 + D1 * D1 + D2 * D2);
            dmax = l > dmax ? l : dmax;
        }
    c.S = fabs((double)c.bl.x) + fabs((double)c.bl.y) + fabs((double)c.bl.z) + fabs((double)c.vw) + 2.0 +
          fabs((double)c.cx) + fabs((double)c.cy) + fabs((double)c.cz);
    c.dmax = dmax * (1.0 + 1e-6) + 8.0 * u * c.S;
    return c;
}

__device__ inline TriCull cull_record(const TriHot& h, const CullCam& cc) {
    const double u = 0x1p-24;
    const float cx = cc.cx, cy = cc.cy, cz = cc.cz;
    const f3 e1f = mk3(h.q0.x, h.q0.y, h.q0.z), e2f = mk3(h.q0.w, h.q1.x, h.q1.y);
    const f3 nf = mk3(h.q1.z, h.q1.w, h.q2.x), af = mk3(h.q2.y, h.q2.z, h.q2.w);
    const f3 Cf = mk3(cx, cy, cz);
    const f3 aof = sub(Cf, af);        // exactly the reference's `*ray.start() - a`
    const float atf = dot0(aof, nf);   // exactly the reference's `ao.dot_product(&n)`
    const float vw = cc.vw;
    const double* blc = cc.blc;
    const double dmax = cc.dmax, S = cc.S;
    // doubles from here on
    const double e1[3] = {e1f.x, e1f.y, e1f.z}, e2[3] = {e2f.x, e2f.y, e2f.z};
    const double n[3] = {nf.x, nf.y, nf.z}, ao[3] = {aof.x, aof.y, aof.z};
    auto n1 = [](const double* v) { return fabs(v[0]) + fabs(v[1]) + fabs(v[2]); };
    auto crs = [](const double* s, const double* o, double* r) {
        r[0] = s[1] * o[2] - s[2] * o[1];
        r[1] = s[2] * o[0] - s[0] * o[2];
        r[2] = s[0] * o[1] - s[1] * o[0];
    };
    double wu[3], wv[3], ww[3], wn[3];
    crs(e2, ao, wu);
    crs(ao, e1, wv);
    for (int k = 0; k < 3; ++k) {
        ww[k] = -(n[k] + wu[k] + wv[k]);
        wn[k] = -n[k];
    }
    const double nn = n1(n), ne1 = n1(e1), ne2 = n1(e2), nao = n1(ao);
    const double floor_n = nn * 0x1p-149;
    const double Eu = 8.0 * u * ne2 * nao + floor_n;
    const double Ev = 8.0 * u * ne1 * nao + floor_n;
    const double En = 4.0 * u * nn;
    const double Ew = (8.0 * u * ne2 * nao) + (8.0 * u * ne1 * nao) + 1.01 * En + 3.2 * u * nn + floor_n;
    const double* W[4] = {wu, wv, ww, wn};
    const double E[4] = {Eu, Ev, Ew, En};
    float A[4], B[4], K[4], Tt[4];
    bool finite = true;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const double* w = W[k];
        double Kd = blc[0] * w[0] + blc[1] * w[1] + blc[2] * w[2];
        // det's threshold (primitives.rs:47-66, 1e-6 in f32), scaled by the smallest |D|, rounded down
        if (k == 3) Kd -= (double)1e-6f * fabs(blc[2]) * (1.0 - 0x1p-20);
        double Ad = (double)vw * w[0];
        double Bd = 2.0 * w[1];
        double thr = 2.0 * ((E[k] + 4.0 * u * n1(w)) * dmax + 4.0 * u * S * n1(w) +
                            6.0 * u * (fabs(Kd) + fabs(Ad) + fabs(Bd)));
        thr = thr * (1.0 + 0x1p-20) + 0x1p-126;  // round the float threshold up
        A[k] = (float)Ad;
        B[k] = (float)Bd;
        K[k] = (float)Kd;
        Tt[k] = (float)thr;
        finite = finite && isfinite(A[k]) && isfinite(B[k]) && isfinite(K[k]) && isfinite(Tt[k]);
    }
    bool all_finite = finite && isfinite(atf) && isfinite(nn) && isfinite(nao) && isfinite(ne1) &&
                      isfinite(ne2) && isfinite(dmax);
    // t >= 0 fails for every camera ray / det >= 1e-6 is unreachable: reject the whole face
    bool reject_all = all_finite && (((double)atf < -floor_n * 2.0) || (nn * (1.0 + 8.0 * u) < 1e-6));
    if (!all_finite) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            A[k] = B[k] = K[k] = 0.0f;
            Tt[k] = __builtin_inff();
        }
    } else if (reject_all) {
        A[3] = B[3] = K[3] = 0.0f;
        Tt[3] = -__builtin_inff();
    }
    TriCull c;
    c.A = make_float4(A[0], A[1], A[2], A[3]);
    c.B = make_float4(B[0], B[1], B[2], B[3]);
    c.K = make_float4(K[0], K[1], K[2], K[3]);
    c.T = make_float4(Tt[0], Tt[1], Tt[2], Tt[3]);
    return c;
}
__device__ inline TriCull cull_record(const TriHot& h, const CamDev& cam, double xa = 0.0, double xb = 1.0,
                                      double ya = 0.0, double yb = 1.0) {
    return cull_record(h, cull_cam(cam, xa, xb, ya, yb));
}

// true when condition k fails for every pixel of [xlo,xhi] x [ylo,yhi]
__device__ __forceinline__ bool cull_one(float A, float B, float K, float T, float xlo, float xhi,
                                         float ylo, float yhi) {
    float ax = __builtin_fmaxf(A * xlo, A * xhi);
    float by = __builtin_fmaxf(B * ylo, B * yhi);
    float fmax = (K + ax) + by;
    return fmax < -T;
}
__device__ __forceinline__ bool cull_rejects(const TriCull c, float xlo, float xhi, float ylo,
                                             float yhi) {
    // all four conditions, no short-circuit: the record is one 64-byte load
    return ((int)cull_one(c.A.x, c.B.x, c.K.x, c.T.x, xlo, xhi, ylo, yhi) |
            (int)cull_one(c.A.y, c.B.y, c.K.y, c.T.y, xlo, xhi, ylo, yhi) |
            (int)cull_one(c.A.z, c.B.z, c.K.z, c.T.z, xlo, xhi, ylo, yhi) |
            (int)cull_one(c.A.w, c.B.w, c.K.w, c.T.w, xlo, xhi, ylo, yhi)) != 0;
}

}  // namespace gpu
}  // namespace eray
