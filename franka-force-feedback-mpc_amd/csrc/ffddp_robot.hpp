// ffddp_robot.hpp — world-frame rigid-body pass for the serial 7-DoF arm.
//
// One forward sweep over the joints computes, generic over T in {double, Dual}:
//   * joint frames (forwardKinematics) and the EE frame placement
//     (updateFramePlacements, crocoddyl_classical.py:201-202),
//   * the EE LOCAL_WORLD_ALIGNED velocity and classical acceleration
//     (ResidualModelFrameVelocity, ContactModel1D/3D drift),
//   * joint torques by recursive Newton-Euler with an external contact force
//     at the EE origin (pinocchio::rnea with fext, computeRNEADerivatives),
//   * optionally (T = double) the joint-space inertia by the composite
//     rigid-body algorithm (pinocchio::crba inside computeAllTerms).
// Spatial convention: motion = (v_O, w), force = (f, n about the world origin),
// everything in the world frame (Pinocchio's oMi/ov/oa/of quantities).
#pragma once

#include "../../include/ffddp.h"
#include "ffddp_math.hpp"

namespace ffddp {

template <class T> struct RBOut {
  T tau[FFDDP_NQ];
  V3<T> z[FFDDP_NQ];  // joint axes (world)
  V3<T> o[FFDDP_NQ];  // joint origins (world)
  M3<T> Ree;
  V3<T> pee;
  V3<T> vp, w;  // EE origin velocity, angular velocity (LWA)
  V3<T> ap;     // EE origin classical acceleration at the given qdd (gravity free)
};

// a: joint acceleration (fixed, no tangent);  lam_w: world-aligned linear
// contact force on the robot at the EE origin (or nullptr);  M: 28 packed
// lower-triangular entries (only when WITH_M).
template <class T, bool WITH_TAU, bool WITH_M>
FFD_HD void rb_pass(const ffddp_robot& rb, const T* q, const T* v, const double* a, const double* lam_w,
                    RBOut<T>& out, double* M) {
  M3<T> Rprev = m3eye<T>();
  V3<T> oprev = v3zero<T>();
  V3<T> vO = v3zero<T>(), w = v3zero<T>(), aO = v3zero<T>(), al = v3zero<T>();
  // Torques without keeping per-link forces live: tau_i = S_i . (F_tot - P_i)
  // with P_i = sum_{k<i} f_k; the S_i . P_i part is accumulated on the way out.
  V3<T> Pl = v3zero<T>(), Pa = v3zero<T>();
  V3<T> Sv_[FFDDP_NQ];
  // composite-inertia tuples (m, h = m c, I_O) for CRBA (double only)
  double cm[FFDDP_NQ], ch[FFDDP_NQ][3], cI[FFDDP_NQ][6];
  const V3<T> g = v3c<T>(rb.gravity);
#pragma unroll
  for (int i = 0; i < FFDDP_NQ; ++i) {
    const V3<T> o = oprev + mulc_v(Rprev, rb.joint_p[i]);
    const M3<T> Rp = mulc(Rprev, rb.joint_R[i]);
    T s, c;
    sincos_(q[i], s, c);
    M3<T> R;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      R.m[3 * r + 0] = c * Rp.m[3 * r + 0] + s * Rp.m[3 * r + 1];
      R.m[3 * r + 1] = c * Rp.m[3 * r + 1] - s * Rp.m[3 * r + 0];
      R.m[3 * r + 2] = Rp.m[3 * r + 2];
    }
    const V3<T> z = {R.m[2], R.m[5], R.m[8]};
    const V3<T> Sv = cross(o, z);
    const V3<T> Svq = v[i] * Sv, zq = v[i] * z;
    vO = vO + Svq;
    w = w + zq;
    // oa_i = oa_{i-1} + S_i qdd_i + ov_i x (S_i qd_i)
    aO = aO + scale(Sv, a[i]) + (cross(w, Svq) + cross(vO, zq));
    al = al + scale(z, a[i]) + cross(w, zq);
    out.z[i] = z;
    out.o[i] = o;
    if (WITH_TAU || WITH_M) {
      const double m = rb.mass[i];
      const V3<T> cw = o + mulc_v(R, rb.com[i]);
      if (WITH_TAU) {
        // Icw x = R (Ic (R^T x))
        const V3<T> Iw = mul(R, cmul(rb.inertia[i], mulT(R, w)));
        const V3<T> Ial = mul(R, cmul(rb.inertia[i], mulT(R, al)));
        const V3<T> hl = scale(vO - cross(cw, w), m);
        const V3<T> ha = cross(cw, hl) + Iw;
        const V3<T> ag = aO - g;
        const V3<T> f1 = scale(ag - cross(cw, al), m);
        const V3<T> n1 = cross(cw, f1) + Ial;
        const V3<T> fli = f1 + cross(w, hl);
        const V3<T> fai = n1 + cross(w, ha) + cross(vO, hl);
        out.tau[i] = -(dot(Sv, Pl) + dot(z, Pa));
        Pl = Pl + fli;
        Pa = Pa + fai;
        Sv_[i] = Sv;
      }
      if (WITH_M) {
        // tuple in world: m, h = m c, I_O = Ic_w + m (|c|^2 I - c c^T)   (T = double)
        const double cx = val(cw.x), cy = val(cw.y), cz = val(cw.z);
        double Rd[9];
        for (int k = 0; k < 9; ++k) Rd[k] = val(R.m[k]);
        double IcR[9];  // Ic R^T
        for (int r = 0; r < 3; ++r)
          for (int cc = 0; cc < 3; ++cc)
            IcR[3 * r + cc] = rb.inertia[i][3 * r + 0] * Rd[3 * cc + 0] + rb.inertia[i][3 * r + 1] * Rd[3 * cc + 1] +
                              rb.inertia[i][3 * r + 2] * Rd[3 * cc + 2];
        double Iw[9];
        for (int r = 0; r < 3; ++r)
          for (int cc = 0; cc < 3; ++cc)
            Iw[3 * r + cc] = Rd[3 * r + 0] * IcR[0 * 3 + cc] + Rd[3 * r + 1] * IcR[1 * 3 + cc] + Rd[3 * r + 2] * IcR[2 * 3 + cc];
        const double c2 = cx * cx + cy * cy + cz * cz;
        cm[i] = m;
        ch[i][0] = m * cx;
        ch[i][1] = m * cy;
        ch[i][2] = m * cz;
        cI[i][0] = Iw[0] + m * (c2 - cx * cx);  // xx
        cI[i][1] = Iw[1] - m * cx * cy;         // xy
        cI[i][2] = Iw[2] - m * cx * cz;         // xz
        cI[i][3] = Iw[4] + m * (c2 - cy * cy);  // yy
        cI[i][4] = Iw[5] - m * cy * cz;         // yz
        cI[i][5] = Iw[8] + m * (c2 - cz * cz);  // zz
      }
    }
    Rprev = R;
    oprev = o;
  }
  // EE frame
  out.pee = oprev + mulc_v(Rprev, rb.ee_p);
  out.Ree = mulc(Rprev, rb.ee_R);
  out.w = w;
  out.vp = vO + cross(w, out.pee);
  out.ap = aO + cross(al, out.pee) + cross(w, out.vp);
  if (WITH_TAU) {
    if (lam_w != nullptr) {
      // external force acts on the last link only: subtract it from every F_i
      // (P_i never contains it, F_tot does)
      const V3<T> lw = v3c<T>(lam_w);
      Pl = Pl - lw;
      Pa = Pa - cross(out.pee, lw);
    }
#pragma unroll
    for (int i = 0; i < FFDDP_NQ; ++i) out.tau[i] = out.tau[i] + (dot(Sv_[i], Pl) + dot(out.z[i], Pa));
  }
  if (WITH_M) {
    double m = 0, hx = 0, hy = 0, hz = 0, I0 = 0, I1 = 0, I2 = 0, I3 = 0, I4 = 0, I5 = 0;
#pragma unroll
    for (int j = FFDDP_NQ - 1; j >= 0; --j) {
      m += cm[j];
      hx += ch[j][0];
      hy += ch[j][1];
      hz += ch[j][2];
      I0 += cI[j][0];
      I1 += cI[j][1];
      I2 += cI[j][2];
      I3 += cI[j][3];
      I4 += cI[j][4];
      I5 += cI[j][5];
      // F = Ic S_j: f = m Sv - h x Sw ; n = h x Sv + I_O Sw
      const double zx = val(out.z[j].x), zy = val(out.z[j].y), zz = val(out.z[j].z);
      const double ox = val(out.o[j].x), oy = val(out.o[j].y), oz = val(out.o[j].z);
      const double svx = oy * zz - oz * zy, svy = oz * zx - ox * zz, svz = ox * zy - oy * zx;
      const double flx = m * svx - (hy * zz - hz * zy);
      const double fly = m * svy - (hz * zx - hx * zz);
      const double flz = m * svz - (hx * zy - hy * zx);
      const double nax = (hy * svz - hz * svy) + I0 * zx + I1 * zy + I2 * zz;
      const double nay = (hz * svx - hx * svz) + I1 * zx + I3 * zy + I4 * zz;
      const double naz = (hx * svy - hy * svx) + I2 * zx + I4 * zy + I5 * zz;
#pragma unroll
      for (int i = 0; i <= j; ++i) {
        const double wx = val(out.z[i].x), wy = val(out.z[i].y), wz = val(out.z[i].z);
        const double px = val(out.o[i].x), py = val(out.o[i].y), pz = val(out.o[i].z);
        const double sx = py * wz - pz * wy, sy = pz * wx - px * wz, sz = px * wy - py * wx;
        M[tri(j, i)] = sx * flx + sy * fly + sz * flz + wx * nax + wy * nay + wz * naz;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Per-link world-frame data at (q, v, qdd = a) for the closed-form tangents
// of the calcDiff kernel (layout LK_*; double only).  Per link k:
//   S = (o x z, z), o, V = (vO, w), A = (aO, al) (qdd = a), F = I (A - G) +
//   V x* (I V) (link force, no contact), H = I V, tuple (m, h = m c, I_O);
// then the EE: p, v_p (LWA), w, classical acceleration a_p (qdd = a).
// ---------------------------------------------------------------------------
constexpr int LK_SV = 0, LK_Z = 3, LK_O = 6, LK_VO = 9, LK_W = 12, LK_AO = 15, LK_AL = 18, LK_F = 21, LK_N = 24,
              LK_HL = 27, LK_HA = 30, LK_M = 33, LK_H = 34, LK_IO = 37, LK_STRIDE = 43;
constexpr int LK_EE = FFDDP_NQ * LK_STRIDE;  // pee(3) vp(3) w(3) ap(3)
constexpr int LK_WORDS = LK_EE + 12;         // 313
constexpr int LK_ALLOC = 320;

FFD_HD void rb_links(const ffddp_robot& rb, const double* q, const double* v, const double* a, double* lk) {
  M3<double> Rprev = m3eye<double>();
  V3<double> oprev = v3zero<double>();
  V3<double> vO = v3zero<double>(), w = v3zero<double>(), aO = v3zero<double>(), al = v3zero<double>();
  const V3<double> g = v3c<double>(rb.gravity);
#pragma unroll
  for (int i = 0; i < FFDDP_NQ; ++i) {
    double* L = lk + i * LK_STRIDE;
    const V3<double> o = oprev + mulc_v(Rprev, rb.joint_p[i]);
    const M3<double> Rp = mulc(Rprev, rb.joint_R[i]);
    double s, c;
    sincos_(q[i], s, c);
    M3<double> R;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      R.m[3 * r + 0] = c * Rp.m[3 * r + 0] + s * Rp.m[3 * r + 1];
      R.m[3 * r + 1] = c * Rp.m[3 * r + 1] - s * Rp.m[3 * r + 0];
      R.m[3 * r + 2] = Rp.m[3 * r + 2];
    }
    const V3<double> z = {R.m[2], R.m[5], R.m[8]};
    const V3<double> Sv = cross(o, z);
    const V3<double> Svq = v[i] * Sv, zq = v[i] * z;
    vO = vO + Svq;
    w = w + zq;
    aO = aO + scale(Sv, a[i]) + (cross(w, Svq) + cross(vO, zq));
    al = al + scale(z, a[i]) + cross(w, zq);
    // inertia tuple about the world origin
    const double m = rb.mass[i];
    const V3<double> cw = o + mulc_v(R, rb.com[i]);
    double IcR[9], Iw[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int cc = 0; cc < 3; ++cc)
        IcR[3 * r + cc] = rb.inertia[i][3 * r + 0] * R.m[3 * cc + 0] + rb.inertia[i][3 * r + 1] * R.m[3 * cc + 1] +
                          rb.inertia[i][3 * r + 2] * R.m[3 * cc + 2];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int cc = 0; cc < 3; ++cc)
        Iw[3 * r + cc] = R.m[3 * r + 0] * IcR[0 * 3 + cc] + R.m[3 * r + 1] * IcR[1 * 3 + cc] + R.m[3 * r + 2] * IcR[2 * 3 + cc];
    const double c2 = dot(cw, cw);
    const V3<double> h = scale(cw, m);
    const double IO[6] = {Iw[0] + m * (c2 - cw.x * cw.x), Iw[1] - m * cw.x * cw.y, Iw[2] - m * cw.x * cw.z,
                          Iw[4] + m * (c2 - cw.y * cw.y), Iw[5] - m * cw.y * cw.z, Iw[8] + m * (c2 - cw.z * cw.z)};
    auto IOmul = [&](V3<double> x) -> V3<double> {
      return {IO[0] * x.x + IO[1] * x.y + IO[2] * x.z, IO[1] * x.x + IO[3] * x.y + IO[4] * x.z,
              IO[2] * x.x + IO[4] * x.y + IO[5] * x.z};
    };
    // H = I V ; F = I (A - G) + V x* H
    const V3<double> hl = scale(vO, m) - cross(h, w);
    const V3<double> ha = cross(h, vO) + IOmul(w);
    const V3<double> ag = aO - g;
    const V3<double> f1 = scale(ag, m) - cross(h, al);
    const V3<double> n1 = cross(h, ag) + IOmul(al);
    const V3<double> f = f1 + cross(w, hl);
    const V3<double> n = n1 + cross(w, ha) + cross(vO, hl);
    const V3<double> vals[11] = {Sv, z, o, vO, w, aO, al, f, n, hl, ha};
#pragma unroll
    for (int e = 0; e < 11; ++e) {
      L[3 * e + 0] = vals[e].x;
      L[3 * e + 1] = vals[e].y;
      L[3 * e + 2] = vals[e].z;
    }
    L[LK_M] = m;
    L[LK_H + 0] = h.x;
    L[LK_H + 1] = h.y;
    L[LK_H + 2] = h.z;
#pragma unroll
    for (int e = 0; e < 6; ++e) L[LK_IO + e] = IO[e];
    Rprev = R;
    oprev = o;
  }
  const V3<double> pee = oprev + mulc_v(Rprev, rb.ee_p);
  const V3<double> vp = vO + cross(w, pee);
  const V3<double> ap = aO + cross(al, pee) + cross(w, vp);
  const V3<double> ee[4] = {pee, vp, w, ap};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    lk[LK_EE + 3 * e + 0] = ee[e].x;
    lk[LK_EE + 3 * e + 1] = ee[e].y;
    lk[LK_EE + 3 * e + 2] = ee[e].z;
  }
}

// gravity torque rnea(q, 0, 0) (crocoddyl_classical.py:447-451)
FFD_HD void gravity_torque(const ffddp_robot& rb, const double* q, double* tau) {
  double zero[FFDDP_NQ] = {0, 0, 0, 0, 0, 0, 0};
  RBOut<double> o;
  rb_pass<double, true, false>(rb, q, zero, zero, nullptr, o, nullptr);
  for (int i = 0; i < FFDDP_NQ; ++i) tau[i] = o.tau[i];
}

}  // namespace ffddp
