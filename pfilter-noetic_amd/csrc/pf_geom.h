// Per-element geometry of the odometry path, evaluated inside the kernels (double precision,
// compiled with -ffp-contract=off so every product and sum rounds exactly as written).
//
//   qrot / qmul / q2m / m2q      Eigen 3.3 quaternion formulas used by pointAssociateToMap
//                                (src/odomEstimationClass.cpp:162-174), updatePointsToMap
//                                (:239, :278-280) and the cost functions.
//   se3_exp / se3_plus           getTransformFromSe3 / PoseSE3Parameterization::Plus
//                                (src/lidarOptimization.cpp:80-143)
//   edge_eval / surf_eval        Edge/SurfNormAnalyticCostFunction::Evaluate (:12-78)
//   eig3                         SelfAdjointEigenSolver<Matrix3d> contract (ascending; cyclic Jacobi)
//   plane5                       ColPivHouseholderQR<Matrix<double,5,3>>::solve of A n = -1 (:461)
#pragma once
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>

#define PF_HD __host__ __device__ __forceinline__

namespace pf {

struct d3 { double x, y, z; };
PF_HD d3 mk3(double x, double y, double z) { return d3{x, y, z}; }
PF_HD d3 add3(d3 a, d3 b) { return d3{a.x + b.x, a.y + b.y, a.z + b.z}; }
PF_HD d3 sub3(d3 a, d3 b) { return d3{a.x - b.x, a.y - b.y, a.z - b.z}; }
PF_HD d3 cross3(d3 a, d3 b) { return d3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
PF_HD double dot3(d3 a, d3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
PF_HD double nrm3(d3 a) { return sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }

struct qd { double x, y, z, w; };

// Eigen _transformVector: uv = 2 (q.vec x v); v + w uv + q.vec x uv
PF_HD d3 qrot(const qd& q, d3 v) {
    d3 qv{q.x, q.y, q.z};
    d3 uv = cross3(qv, v);
    uv = add3(uv, uv);
    d3 c = cross3(qv, uv);
    return d3{v.x + q.w * uv.x + c.x, v.y + q.w * uv.y + c.y, v.z + q.w * uv.z + c.z};
}
PF_HD qd qmul(const qd& a, const qd& b) {
    qd r;
    r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
    r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
    r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
    r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
    return r;
}

struct m3 { double m[3][3]; };
PF_HD m3 m3_eye() {
    m3 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r.m[i][j] = (i == j) ? 1.0 : 0.0;
    return r;
}
PF_HD m3 m3_mul(const m3& a, const m3& b) {
    m3 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            r.m[i][j] = a.m[i][0] * b.m[0][j] + a.m[i][1] * b.m[1][j] + a.m[i][2] * b.m[2][j];
    return r;
}
PF_HD d3 m3_vec(const m3& a, d3 v) {
    return d3{a.m[0][0] * v.x + a.m[0][1] * v.y + a.m[0][2] * v.z, a.m[1][0] * v.x + a.m[1][1] * v.y + a.m[1][2] * v.z,
              a.m[2][0] * v.x + a.m[2][1] * v.y + a.m[2][2] * v.z};
}
PF_HD m3 m3_t(const m3& a) {
    m3 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r.m[i][j] = a.m[j][i];
    return r;
}
PF_HD m3 q2m(const qd& q) {
    const double tx = 2.0 * q.x, ty = 2.0 * q.y, tz = 2.0 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    m3 r;
    r.m[0][0] = 1.0 - (tyy + tzz); r.m[0][1] = txy - twz;         r.m[0][2] = txz + twy;
    r.m[1][0] = txy + twz;         r.m[1][1] = 1.0 - (txx + tzz); r.m[1][2] = tyz - twx;
    r.m[2][0] = txz - twy;         r.m[2][1] = tyz + twx;         r.m[2][2] = 1.0 - (txx + tyy);
    return r;
}
template <int I>
PF_HD void m2q_branch(const m3& a, double* c) {
    constexpr int J = (I + 1) % 3, K = (J + 1) % 3;
    double t = sqrt(a.m[I][I] - a.m[J][J] - a.m[K][K] + 1.0);
    c[I] = 0.5 * t;
    t = 0.5 / t;
    c[3] = (a.m[K][J] - a.m[J][K]) * t;
    c[J] = (a.m[J][I] + a.m[I][J]) * t;
    c[K] = (a.m[K][I] + a.m[I][K]) * t;
}
PF_HD qd m2q(const m3& a) {
    double c[4];
    double t = a.m[0][0] + a.m[1][1] + a.m[2][2];
    if (t > 0.0) {
        t = sqrt(t + 1.0);
        c[3] = 0.5 * t;
        t = 0.5 / t;
        c[0] = (a.m[2][1] - a.m[1][2]) * t;
        c[1] = (a.m[0][2] - a.m[2][0]) * t;
        c[2] = (a.m[1][0] - a.m[0][1]) * t;
    } else {
        int i = 0;
        if (a.m[1][1] > a.m[0][0]) i = 1;
        if (a.m[2][2] > (i == 0 ? a.m[0][0] : a.m[1][1])) i = 2;     // a.m[i][i], statically indexed
        if (i == 0) m2q_branch<0>(a, c);             // static indices: no scratch arrays
        else if (i == 1) m2q_branch<1>(a, c);
        else m2q_branch<2>(a, c);
    }
    return qd{c[0], c[1], c[2], c[3]};
}

// Transform<double,3,Isometry>::rotation() in Eigen 3.3 (the ROS Noetic / Ubuntu 20.04 Eigen) is
// NOT linear(): it is the orthogonal polar factor computeRotationScaling() takes from a
// JacobiSVD<Matrix3d>(ComputeFullU|ComputeFullV). That re-orthonormalisation is what keeps |q|
// at 1 through the constant-velocity prediction (src/odomEstimationClass.cpp:235-239); without
// it the norm error is tripled every frame once the heading passes ~90 degrees.
// Two-sided Jacobi sweep exactly as JacobiSVD::compute (square input: no QR preconditioner).
struct jrot { double c, s; };
// rows p,q of A (applyOnTheLeft); x' = c x + s y, y' = -s x + c y
PF_HD void rot_rows(double A[3][3], int p, int q, jrot j) {
    if (j.c == 1.0 && j.s == 0.0) return;
    for (int k = 0; k < 3; ++k) {
        const double x = A[p][k], y = A[q][k];
        A[p][k] = j.c * x + j.s * y;
        A[q][k] = -j.s * x + j.c * y;
    }
}
// columns p,q of A rotated by j (apply_rotation_in_the_plane on two columns)
PF_HD void rot_cols(double A[3][3], int p, int q, jrot j) {
    if (j.c == 1.0 && j.s == 0.0) return;
    for (int k = 0; k < 3; ++k) {
        const double x = A[k][p], y = A[k][q];
        A[k][p] = j.c * x + j.s * y;
        A[k][q] = -j.s * x + j.c * y;
    }
}
PF_HD jrot make_jacobi(double x, double y, double z) {   // JacobiRotation::makeJacobi (real)
    const double deno = 2.0 * fabs(y);
    if (deno < DBL_MIN) return jrot{1.0, 0.0};
    const double tau = (x - z) / deno;
    const double w = sqrt(tau * tau + 1.0);
    const double t = tau > 0.0 ? 1.0 / (tau + w) : 1.0 / (tau - w);
    const double sign_t = t > 0.0 ? 1.0 : -1.0;
    const double n = 1.0 / sqrt(t * t + 1.0);
    return jrot{n, -sign_t * (y / fabs(y)) * fabs(t) * n};
}
PF_HD m3 polar_rotation(const m3& a) {
    double W[3][3], U[3][3], V[3][3];
    double scale = 0.0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) scale = fmax(scale, fabs(a.m[i][j]));
    if (scale == 0.0) scale = 1.0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            W[i][j] = a.m[i][j] / scale;
            U[i][j] = V[i][j] = (i == j) ? 1.0 : 0.0;
        }
    const double precision = 2.0 * DBL_EPSILON;
    double maxdiag = fmax(fmax(fabs(W[0][0]), fabs(W[1][1])), fabs(W[2][2]));
    bool finished = false;
    for (int sweep = 0; !finished && sweep < 64; ++sweep) {
        finished = true;
        for (int p = 1; p < 3; ++p)
            for (int q = 0; q < p; ++q) {
                const double thr = fmax(DBL_MIN, precision * maxdiag);
                if (!(fabs(W[p][q]) > thr || fabs(W[q][p]) > thr)) continue;
                finished = false;
                // real_2x2_jacobi_svd on the (p,q) block
                double m00 = W[p][p], m01 = W[p][q], m10 = W[q][p], m11 = W[q][q];
                jrot r1{1.0, 0.0};
                const double t = m00 + m11, d = m10 - m01;
                if (fabs(d) >= DBL_MIN) {
                    const double u = t / d;
                    const double tmp = sqrt(1.0 + u * u);
                    r1 = jrot{u / tmp, 1.0 / tmp};
                }
                if (!(r1.c == 1.0 && r1.s == 0.0)) {
                    const double a0 = m00, a1 = m01, b0 = m10, b1 = m11;
                    m00 = r1.c * a0 + r1.s * b0; m01 = r1.c * a1 + r1.s * b1;
                    m10 = -r1.s * a0 + r1.c * b0; m11 = -r1.s * a1 + r1.c * b1;
                }
                const jrot jr = make_jacobi(m00, m01, m11);
                // j_left = rot1 * j_right.transpose()
                const jrot jl{r1.c * jr.c - r1.s * (-jr.s), r1.c * (-jr.s) + r1.s * jr.c};
                rot_rows(W, p, q, jl);                   // W.applyOnTheLeft(p,q,j_left)
                rot_cols(U, p, q, jl);                   // U.applyOnTheRight(p,q,j_left.transpose())
                rot_cols(W, p, q, jrot{jr.c, -jr.s});    // W.applyOnTheRight(p,q,j_right)
                rot_cols(V, p, q, jrot{jr.c, -jr.s});    // V.applyOnTheRight(p,q,j_right)
                maxdiag = fmax(maxdiag, fmax(fabs(W[p][p]), fabs(W[q][q])));
            }
    }
    double sv[3];
    for (int i = 0; i < 3; ++i) {
        sv[i] = fabs(W[i][i]);
        if (W[i][i] < 0.0)
            for (int k = 0; k < 3; ++k) U[k][i] = -U[k][i];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {                        // descending order, first max wins
        int pos = i;
        double best = sv[i];
#pragma unroll
        for (int k = i + 1; k < 3; ++k)
            if (sv[k] > best) { best = sv[k]; pos = k; }
#pragma unroll
        for (int pk = i + 1; pk < 3; ++pk) {             // swap with column pos (static indices)
            if (pk != pos) continue;
            const double ts = sv[i]; sv[i] = sv[pk]; sv[pk] = ts;
            for (int k = 0; k < 3; ++k) {
                double tu = U[k][i]; U[k][i] = U[k][pk]; U[k][pk] = tu;
                double tv = V[k][i]; V[k][i] = V[k][pk]; V[k][pk] = tv;
            }
        }
    }
    m3 uvt;                                              // U * V^T
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            uvt.m[i][j] = U[i][0] * V[j][0] + (U[i][1] * V[j][1] + U[i][2] * V[j][2]);
    const double (*M)[3] = uvt.m;
    const double x = M[0][0] * (M[1][1] * M[2][2] - M[1][2] * M[2][1])   // bruteforce_det3_helper
                   - M[0][1] * (M[1][0] * M[2][2] - M[1][2] * M[2][0])
                   + M[0][2] * (M[1][0] * M[2][1] - M[1][1] * M[2][0]);
    for (int k = 0; k < 3; ++k) U[k][0] /= x;
    m3 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            r.m[i][j] = U[i][0] * V[j][0] + (U[i][1] * V[j][1] + U[i][2] * V[j][2]);
    return r;
}

struct iso { m3 R; d3 t; };
PF_HD iso iso_mul(const iso& a, const iso& b) {
    d3 rt = m3_vec(a.R, b.t);
    return iso{m3_mul(a.R, b.R), add3(rt, a.t)};
}
PF_HD iso iso_inv(const iso& a) {
    m3 rt = m3_t(a.R);
    d3 tt = m3_vec(rt, a.t);
    return iso{rt, d3{-tt.x, -tt.y, -tt.z}};
}

PF_HD m3 skew(d3 v) {
    m3 s;
    s.m[0][0] = 0.0; s.m[0][1] = -v.z; s.m[0][2] = v.y;
    s.m[1][0] = v.z; s.m[1][1] = 0.0;  s.m[1][2] = -v.x;
    s.m[2][0] = -v.y; s.m[2][1] = v.x; s.m[2][2] = 0.0;
    return s;
}

// sin and cos of x from + - * and rint only (no libm, no FMA under -ffp-contract=off), so the host
// and gfx950 produce the same bits: the oracle's GPU_EQUIV mode restates this function and follows
// the device's SE(3) updates bit for bit over a whole sequence (libm's and the device library's
// sin/cos differ in the last ulp now and then, and an ulp in the pose moves f32 map points).
// Cody-Waite reduction by pi/2 in two 33-bit parts (exact products for |k| < 2^20), then the
// classic fdlibm minimax kernels on [-pi/4, pi/4]; error <= 1 ulp there. Arguments beyond 2^19 pi
// still give deterministic (if inexact) values; NaN and inf give NaN.
PF_HD void det_sincos(double x, double* sn, double* cs) {
    const double invpio2 = 6.36619772367581382433e-01;
    const double pio2_1 = 1.57079632673412561417e+00;    // first 33 bits of pi/2
    const double pio2_1t = 6.07710050650619224932e-11;   // pi/2 - pio2_1
    const double k = rint(x * invpio2);
    const double r = (x - k * pio2_1) - k * pio2_1t;
    const double z = r * r;
    const double v = z * r;
    const double ps = 8.33333333332248946124e-03 +
                      z * (-1.98412698298579493134e-04 +
                           z * (2.75573137070700676789e-06 + z * (-2.50507602534068634195e-08 + z * 1.58969099521155010221e-10)));
    const double s = r + v * (-1.66666666666666324348e-01 + z * ps);
    const double pc = z * (4.16666666666666019037e-02 +
                           z * (-1.38888888888741095749e-03 +
                                z * (2.48015872894767294178e-05 +
                                     z * (-2.75573143513906633035e-07 +
                                          z * (2.08757232129817482790e-09 + z * -1.13596475577881948265e-11)))));
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    const double c = w + (((1.0 - w) - hz) + z * pc);
    const long long n = (k == k && fabs(k) < 9.0e15) ? (long long)k : 0;
    switch ((int)(n & 3)) {
        case 0: *sn = s; *cs = c; break;
        case 1: *sn = c; *cs = -s; break;
        case 2: *sn = -s; *cs = -c; break;
        default: *sn = -c; *cs = s; break;
    }
}

// getTransformFromSe3 (src/lidarOptimization.cpp:106-143) in the source's own form: the quaternion
// from sin / cos of theta / 2, the translation Jacobian from (1 - cos(theta)) / theta^2 and
// (theta - sin(theta)) / theta^3 of the full angle, both sincos from det_sincos and theta^3 as a product
// where the source calls pow (an ulp now and then). Round 3 took the half-angle identities
// 1 - cos(theta) = 2 sin^2(theta / 2) and sin(theta) = 2 s c instead: more accurate for small theta,
// where 1 - cos(theta) cancels, but not the source's arithmetic, and that systematic difference (up to
// ~1e-8 relative in the two coefficients) is what an ill-conditioned stretch of the S64T town
// sequence amplified into a count flip at frame 338 (tools/drift_probe.py: the oracle's device-LM
// restatement separates from the faithful oracle there with the half-angle form and tracks it with
// this one; neither the LM's normal equations nor libm's last bit do it).
PF_HD void se3_exp(const double* se3, qd& q, d3& t) {
    d3 omega{se3[0], se3[1], se3[2]};
    d3 upsilon{se3[3], se3[4], se3[5]};
    m3 Om = skew(omega);
    const double theta = nrm3(omega);
    const double half_theta = 0.5 * theta;
    double s_h, c_h;
    det_sincos(half_theta, &s_h, &c_h);
    double imag_factor;
    const double real_factor = c_h;
    if (theta < 1e-10) {
        const double theta_sq = theta * theta;
        const double theta_po4 = theta_sq * theta_sq;
        imag_factor = 0.5 - 0.0208333 * theta_sq + 0.000260417 * theta_po4;
    } else {
        imag_factor = s_h / theta;
    }
    q = qd{imag_factor * omega.x, imag_factor * omega.y, imag_factor * omega.z, real_factor};
    m3 J;
    if (theta < 1e-10) {
        J = q2m(q);
    } else {
        m3 Om2 = m3_mul(Om, Om);
        double s_t, c_t;
        det_sincos(theta, &s_t, &c_t);
        const double a = (1.0 - c_t) / (theta * theta);
        const double b = (theta - s_t) / (theta * theta * theta);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) J.m[i][j] = (i == j ? 1.0 : 0.0) + a * Om.m[i][j] + b * Om2.m[i][j];
    }
    t = m3_vec(J, upsilon);
}

PF_HD void se3_plus(const double* x, const double* delta, double* out) {
    d3 trans{x[4], x[5], x[6]};
    qd dq;
    d3 dt;
    se3_exp(delta, dq, dt);
    qd quater{x[0], x[1], x[2], x[3]};
    qd qp = qmul(dq, quater);
    d3 tp = add3(qrot(dq, trans), dt);
    out[0] = qp.x; out[1] = qp.y; out[2] = qp.z; out[3] = qp.w;
    out[4] = tp.x; out[5] = tp.y; out[6] = tp.z;
}

// edge residual (weight applied to r only when w is exactly 1, 2 or 12) and J[0..5]
PF_HD double edge_eval(const double* x, d3 cur, d3 a, d3 b, double w, double* J) {
    qd q{x[0], x[1], x[2], x[3]};
    d3 lp = add3(qrot(q, cur), d3{x[4], x[5], x[6]});
    d3 nu = cross3(sub3(lp, a), sub3(lp, b));
    d3 de = sub3(a, b);
    const double de_norm = nrm3(de);
    const double nn = nrm3(nu);
    double r = nn / de_norm;
    if (w == 1 || w == 2) r = w * r;
    else if (w == 12) r = w * r;
    if (J) {
        m3 sl = skew(lp);
        m3 sd = skew(de);
        const double v1[3] = {-nu.x / nn, -nu.y / nn, -nu.z / nn};
        double v2[3];
        for (int j = 0; j < 3; ++j) v2[j] = v1[0] * sd.m[0][j] + v1[1] * sd.m[1][j] + v1[2] * sd.m[2][j];
        for (int j = 0; j < 3; ++j)
            J[j] = (v2[0] * -sl.m[0][j] + v2[1] * -sl.m[1][j] + v2[2] * -sl.m[2][j]) / de_norm;
        for (int j = 0; j < 3; ++j) {
            // dp_by_se3 right block is the identity
            const double e0 = (j == 0) ? 1.0 : 0.0, e1 = (j == 1) ? 1.0 : 0.0, e2 = (j == 2) ? 1.0 : 0.0;
            J[3 + j] = (v2[0] * e0 + v2[1] * e1 + v2[2] * e2) / de_norm;
        }
    }
    return r;
}

PF_HD double surf_eval(const double* x, d3 cur, d3 n, double d, double w, double* J) {
    qd q{x[0], x[1], x[2], x[3]};
    d3 pw = add3(qrot(q, cur), d3{x[4], x[5], x[6]});
    double r = dot3(n, pw) + d;
    if (w != 0) r = w * r;
    if (J) {
        m3 sp = skew(pw);
        for (int j = 0; j < 3; ++j) J[j] = n.x * -sp.m[0][j] + n.y * -sp.m[1][j] + n.z * -sp.m[2][j];
        for (int j = 0; j < 3; ++j) {
            const double e0 = (j == 0) ? 1.0 : 0.0, e1 = (j == 1) ? 1.0 : 0.0, e2 = (j == 2) ? 1.0 : 0.0;
            J[3 + j] = n.x * e0 + n.y * e1 + n.z * e2;
        }
    }
    return r;
}

// symmetric 3x3 eigen-decomposition (cyclic Jacobi), eigenvalues ascending, eigenvector columns
PF_HD void eig3(double a[3][3], double ev[3], double V[3][3]) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) V[i][j] = (i == j) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 50; ++sweep) {
        const double off = a[0][1] * a[0][1] + a[0][2] * a[0][2] + a[1][2] * a[1][2];
        const double diag = a[0][0] * a[0][0] + a[1][1] * a[1][1] + a[2][2] * a[2][2];
        if (off <= 1e-36 * diag || off == 0.0) break;
        for (int p = 0; p < 2; ++p) {
            for (int q = p + 1; q < 3; ++q) {
                const double apq = a[p][q];
                if (apq == 0.0) continue;
                const double theta = (a[q][q] - a[p][p]) / (2.0 * apq);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0);
                const double s = t * c;
                for (int k = 0; k < 3; ++k) {
                    const double akp = a[k][p], akq = a[k][q];
                    a[k][p] = c * akp - s * akq;
                    a[k][q] = s * akp + c * akq;
                }
                for (int k = 0; k < 3; ++k) {
                    const double apk = a[p][k], aqk = a[q][k];
                    a[p][k] = c * apk - s * aqk;
                    a[q][k] = s * apk + c * aqk;
                }
                for (int k = 0; k < 3; ++k) {
                    const double vkp = V[k][p], vkq = V[k][q];
                    V[k][p] = c * vkp - s * vkq;
                    V[k][q] = s * vkp + c * vkq;
                }
            }
        }
    }
    double d[3] = {a[0][0], a[1][1], a[2][2]};
    int o[3] = {0, 1, 2};
    // ascending, ties by index (3-element sorting network on (value, index), columns moved along)
#define PF_SWP(i, j)                                                                   \
    if (d[j] < d[i] || (d[j] == d[i] && o[j] < o[i])) {                                \
        const double td = d[i]; d[i] = d[j]; d[j] = td;                                \
        const int tt = o[i]; o[i] = o[j]; o[j] = tt;                                   \
        for (int r = 0; r < 3; ++r) { const double tv = V[r][i]; V[r][i] = V[r][j]; V[r][j] = tv; } \
    }
    PF_SWP(0, 1) PF_SWP(1, 2) PF_SWP(0, 1)
#undef PF_SWP
    for (int c = 0; c < 3; ++c) ev[c] = d[c];
}

PF_HD void householder(const double* x, int n, double* ess, double& tau, double& beta) {
    double tail = 0.0;
    for (int i = 1; i < n; ++i) tail += x[i] * x[i];
    const double c0 = x[0];
    if (tail <= DBL_MIN) {
        tau = 0.0;
        beta = c0;
        for (int i = 1; i < n; ++i) ess[i] = 0.0;
    } else {
        beta = sqrt(c0 * c0 + tail);
        if (c0 >= 0.0) beta = -beta;
        for (int i = 1; i < n; ++i) ess[i] = x[i] / (c0 - beta);
        tau = (beta - c0) / beta;
    }
}

// least-squares plane normal n with A n = -1, column-pivoting Householder QR (Eigen order)
PF_HD d3 plane5(const double Ain[5][3]) {
    // every loop has constant bounds and every pivot swap is written with static indices, so the
    // arrays stay in registers (no scratch); the arithmetic and its order are Eigen's
    const int R = 5, C = 3;
    double A[5][3];
    for (int i = 0; i < R; ++i)
        for (int j = 0; j < C; ++j) A[i][j] = Ain[i][j];
    double b[5] = {-1, -1, -1, -1, -1};
    int perm[3] = {0, 1, 2};
    double hc[3] = {0, 0, 0};
    double cn[3], cu[3];
    const double eps = DBL_EPSILON;
    double maxnorm = 0.0;
#pragma unroll
    for (int j = 0; j < C; ++j) {
        double s = 0;
        for (int i = 0; i < R; ++i) s += A[i][j] * A[i][j];
        cn[j] = sqrt(s);
        cu[j] = cn[j];
        if (j == 0 || cn[j] > maxnorm) maxnorm = cn[j];
    }
    const double thr_helper = (maxnorm * eps) * (maxnorm * eps) / (double)R;
    const double downdate_thr = sqrt(eps);
    int nonzero = C;
#pragma unroll
    for (int k = 0; k < C; ++k) {
        int best = k;
        double bn = cu[k];
#pragma unroll
        for (int j = k + 1; j < C; ++j)
            if (cu[j] > bn) { bn = cu[j]; best = j; }
        if (nonzero == C && bn * bn < thr_helper * (double)(R - k)) nonzero = k;
#pragma unroll
        for (int jb = k + 1; jb < C; ++jb) {
            if (jb != best) continue;
            for (int i = 0; i < R; ++i) { double t = A[i][k]; A[i][k] = A[i][jb]; A[i][jb] = t; }
            int tp = perm[k]; perm[k] = perm[jb]; perm[jb] = tp;
            double t1 = cn[k]; cn[k] = cn[jb]; cn[jb] = t1;
            double t2 = cu[k]; cu[k] = cu[jb]; cu[jb] = t2;
        }
        double x[5], ess[5];
        const int n = R - k;
        for (int i = 0; i < n; ++i) x[i] = A[k + i][k];
        double tau, beta;
        householder(x, n, ess, tau, beta);
        A[k][k] = beta;
        for (int i = 1; i < n; ++i) A[k + i][k] = ess[i];
        hc[k] = tau;
        if (tau != 0.0 && n > 1) {
#pragma unroll
            for (int j = k + 1; j < C; ++j) {
                double tmp = 0.0;
                for (int i = 1; i < n; ++i) tmp += ess[i] * A[k + i][j];
                tmp += A[k][j];
                A[k][j] -= tau * tmp;
                for (int i = 1; i < n; ++i) A[k + i][j] -= tau * ess[i] * tmp;
            }
        }
#pragma unroll
        for (int j = k + 1; j < C; ++j) {
            if (cu[j] != 0.0) {
                double temp = fabs(A[k][j]) / cu[j];
                temp = (1.0 + temp) * (1.0 - temp);
                temp = temp < 0.0 ? 0.0 : temp;
                const double rr = cu[j] / cn[j];
                const double temp2 = temp * (rr * rr);
                if (temp2 <= downdate_thr) {
                    double s = 0;
                    for (int i = k + 1; i < R; ++i) s += A[i][j] * A[i][j];
                    cn[j] = sqrt(s);
                    cu[j] = cn[j];
                } else {
                    cu[j] *= sqrt(temp);
                }
            }
        }
    }
    if (nonzero == 0) return d3{0, 0, 0};
#pragma unroll
    for (int k = 0; k < C; ++k) {
        const int n = R - k;
        if (k >= nonzero || hc[k] == 0.0 || n < 2) continue;
        double tmp = 0.0;
        for (int i = 1; i < n; ++i) tmp += A[k + i][k] * b[k + i];
        tmp += b[k];
        b[k] -= hc[k] * tmp;
        for (int i = 1; i < n; ++i) b[k + i] -= hc[k] * A[k + i][k] * tmp;
    }
#pragma unroll
    for (int i = C - 1; i >= 0; --i) {
        if (i >= nonzero) continue;
        b[i] /= A[i][i];
        for (int s = 0; s < i; ++s) b[s] -= b[i] * A[s][i];
    }
    double out[3] = {0, 0, 0};
#pragma unroll
    for (int k = 0; k < C; ++k) {
        if (k >= nonzero) continue;
#pragma unroll
        for (int j = 0; j < C; ++j)
            if (perm[k] == j) out[j] = b[k];
    }
    return d3{out[0], out[1], out[2]};
}

}  // namespace pf
