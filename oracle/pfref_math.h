// pfref math: restatement of the Eigen 3.3 formulas and the reference's cost functions.
// TEST INFRASTRUCTURE (oracle) — see pfref.h header.
#pragma once
#include <cmath>
#include <cstring>
#include <algorithm>
#include <limits>

namespace pfref {

struct V3 { double x, y, z; };
inline V3 v3(double x, double y, double z) { return {x, y, z}; }
inline V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 scl(double s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
// Eigen cross (Geometry/OrthoMethods.h): (a1 b2 - a2 b1, a2 b0 - a0 b2, a0 b1 - a1 b0)
inline V3 cross(V3 a, V3 b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
inline double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline double sqnorm(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
inline double norm(V3 a) { return std::sqrt(sqnorm(a)); }

struct Quat { double x, y, z, w; };  // Eigen coeffs order (x, y, z, w)

// Eigen QuaternionBase::_transformVector: uv = vec x v; uv += uv; v + w*uv + vec x uv
inline V3 qrot(const Quat& q, V3 v) {
    V3 qv{q.x, q.y, q.z};
    V3 uv = cross(qv, v);
    uv = add(uv, uv);
    V3 c = cross(qv, uv);
    return {v.x + q.w * uv.x + c.x, v.y + q.w * uv.y + c.y, v.z + q.w * uv.z + c.z};
}
// Eigen quat_product (generic path)
inline Quat qmul(const Quat& a, const Quat& b) {
    Quat r;
    r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
    r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
    r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
    r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
    return r;
}

struct M3 { double m[3][3]; };
inline M3 m3_identity() { M3 r{}; r.m[0][0] = r.m[1][1] = r.m[2][2] = 1.0; return r; }
inline M3 mmul(const M3& a, const M3& b) {
    M3 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            r.m[i][j] = a.m[i][0] * b.m[0][j] + a.m[i][1] * b.m[1][j] + a.m[i][2] * b.m[2][j];
    return r;
}
inline V3 mvec(const M3& a, V3 v) {
    return {a.m[0][0] * v.x + a.m[0][1] * v.y + a.m[0][2] * v.z,
            a.m[1][0] * v.x + a.m[1][1] * v.y + a.m[1][2] * v.z,
            a.m[2][0] * v.x + a.m[2][1] * v.y + a.m[2][2] * v.z};
}
inline M3 mtrans(const M3& a) {
    M3 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r.m[i][j] = a.m[j][i];
    return r;
}
// Eigen QuaternionBase::toRotationMatrix
inline M3 q2m(const Quat& q) {
    const double tx = 2.0 * q.x, ty = 2.0 * q.y, tz = 2.0 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    M3 r;
    r.m[0][0] = 1.0 - (tyy + tzz); r.m[0][1] = txy - twz;         r.m[0][2] = txz + twy;
    r.m[1][0] = txy + twz;         r.m[1][1] = 1.0 - (txx + tzz); r.m[1][2] = tyz - twx;
    r.m[2][0] = txz - twy;         r.m[2][1] = tyz + twx;         r.m[2][2] = 1.0 - (txx + tyy);
    return r;
}
// Eigen quaternionbase_assign_impl<Matrix3> (Quaterniond(const Matrix3d&))
inline Quat m2q(const M3& a) {
    double c[4];  // x, y, z, w
    double t = a.m[0][0] + a.m[1][1] + a.m[2][2];
    if (t > 0.0) {
        t = std::sqrt(t + 1.0);
        c[3] = 0.5 * t;
        t = 0.5 / t;
        c[0] = (a.m[2][1] - a.m[1][2]) * t;
        c[1] = (a.m[0][2] - a.m[2][0]) * t;
        c[2] = (a.m[1][0] - a.m[0][1]) * t;
    } else {
        int i = 0;
        if (a.m[1][1] > a.m[0][0]) i = 1;
        if (a.m[2][2] > a.m[i][i]) i = 2;
        int j = (i + 1) % 3, k = (j + 1) % 3;
        t = std::sqrt(a.m[i][i] - a.m[j][j] - a.m[k][k] + 1.0);
        c[i] = 0.5 * t;
        t = 0.5 / t;
        c[3] = (a.m[k][j] - a.m[j][k]) * t;
        c[j] = (a.m[j][i] + a.m[i][j]) * t;
        c[k] = (a.m[k][i] + a.m[i][k]) * t;
    }
    return {c[0], c[1], c[2], c[3]};
}

// Eigen 3.3 Transform::rotation(): computeRotationScaling() -> JacobiSVD<Matrix3d>(FullU|FullV),
// rotation = U' V^T with U'.col(0) /= det(U V^T) (Eigen/src/Geometry/Transform.h, 3.3.7; the
// Isometry shortcut returning linear() only appeared in Eigen 3.4). Restated step by step from
// JacobiSVD::compute, real_2x2_jacobi_svd and JacobiRotation::makeJacobi.
struct JRot { double c, s; };
inline void jrot_pair(double& x, double& y, const JRot& j) {   // apply_rotation_in_the_plane
    const double xi = x, yi = y;
    x = j.c * xi + j.s * yi;
    y = -j.s * xi + j.c * yi;
}
inline JRot jrot_transpose(const JRot& j) { return {j.c, -j.s}; }
inline JRot jrot_product(const JRot& a, const JRot& b) { return {a.c * b.c - a.s * b.s, a.c * b.s + a.s * b.c}; }
inline JRot jrot_make_jacobi(double x, double y, double z) {
    const double deno = 2.0 * std::fabs(y);
    if (deno < std::numeric_limits<double>::min()) return {1.0, 0.0};
    const double tau = (x - z) / deno;
    const double w = std::sqrt(tau * tau + 1.0);
    double t;
    if (tau > 0.0) t = 1.0 / (tau + w);
    else t = 1.0 / (tau - w);
    const double sign_t = t > 0.0 ? 1.0 : -1.0;
    const double n = 1.0 / std::sqrt(t * t + 1.0);
    return {n, -sign_t * (y / std::fabs(y)) * std::fabs(t) * n};
}
inline void left_rot(double A[3][3], int p, int q, const JRot& j) {     // A.applyOnTheLeft(p,q,j)
    if (j.c == 1.0 && j.s == 0.0) return;
    for (int k = 0; k < 3; ++k) jrot_pair(A[p][k], A[q][k], j);
}
inline void right_rot(double A[3][3], int p, int q, const JRot& j) {    // A.applyOnTheRight(p,q,j)
    const JRot jt = jrot_transpose(j);
    if (jt.c == 1.0 && jt.s == 0.0) return;
    for (int k = 0; k < 3; ++k) jrot_pair(A[k][p], A[k][q], jt);
}
inline double dot3_eigen(double a0, double a1, double a2, double b0, double b1, double b2) {
    return a0 * b0 + (a1 * b1 + a2 * b2);     // 3-term redux unrolled as x0 + (x1 + x2)
}
inline M3 rotation_polar(const M3& in) {
    double W[3][3], U[3][3], V[3][3];
    double scale = 0.0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) scale = std::max(scale, std::fabs(in.m[i][j]));
    if (scale == 0.0) scale = 1.0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            W[i][j] = in.m[i][j] / scale;
            U[i][j] = (i == j) ? 1.0 : 0.0;
            V[i][j] = (i == j) ? 1.0 : 0.0;
        }
    const double precision = 2.0 * std::numeric_limits<double>::epsilon();
    const double tiny = std::numeric_limits<double>::min();
    double max_diag = std::max(std::fabs(W[0][0]), std::max(std::fabs(W[1][1]), std::fabs(W[2][2])));
    bool finished = false;
    while (!finished) {
        finished = true;
        for (int p = 1; p < 3; ++p) {
            for (int q = 0; q < p; ++q) {
                const double threshold = std::max(tiny, precision * max_diag);
                if (std::fabs(W[p][q]) > threshold || std::fabs(W[q][p]) > threshold) {
                    finished = false;
                    // real_2x2_jacobi_svd(W, p, q)
                    double m[2][2] = {{W[p][p], W[p][q]}, {W[q][p], W[q][q]}};
                    JRot rot1;
                    const double t = m[0][0] + m[1][1];
                    const double d = m[1][0] - m[0][1];
                    if (std::fabs(d) < tiny) {
                        rot1 = {1.0, 0.0};
                    } else {
                        const double u = t / d;
                        const double tmp = std::sqrt(1.0 + u * u);
                        rot1 = {u / tmp, 1.0 / tmp};
                    }
                    if (!(rot1.c == 1.0 && rot1.s == 0.0))
                        for (int k = 0; k < 2; ++k) jrot_pair(m[0][k], m[1][k], rot1);
                    const JRot j_right = jrot_make_jacobi(m[0][0], m[0][1], m[1][1]);
                    const JRot j_left = jrot_product(rot1, jrot_transpose(j_right));
                    left_rot(W, p, q, j_left);
                    right_rot(U, p, q, jrot_transpose(j_left));
                    right_rot(W, p, q, j_right);
                    right_rot(V, p, q, j_right);
                    max_diag = std::max(max_diag, std::max(std::fabs(W[p][p]), std::fabs(W[q][q])));
                }
            }
        }
    }
    double sv[3];
    for (int i = 0; i < 3; ++i) {
        const double a = W[i][i];
        sv[i] = std::fabs(a);
        if (a < 0.0)
            for (int k = 0; k < 3; ++k) U[k][i] = -U[k][i];
    }
    for (int i = 0; i < 3; ++i) {
        int pos = i;
        for (int k = i + 1; k < 3; ++k)
            if (sv[k] > sv[pos]) pos = k;
        if (pos != i) {
            std::swap(sv[i], sv[pos]);
            for (int k = 0; k < 3; ++k) {
                std::swap(U[k][i], U[k][pos]);
                std::swap(V[k][i], V[k][pos]);
            }
        }
    }
    double P[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) P[i][j] = dot3_eigen(U[i][0], U[i][1], U[i][2], V[j][0], V[j][1], V[j][2]);
    const double det = P[0][0] * (P[1][1] * P[2][2] - P[1][2] * P[2][1]) -
                       P[0][1] * (P[1][0] * P[2][2] - P[1][2] * P[2][0]) +
                       P[0][2] * (P[1][0] * P[2][1] - P[1][1] * P[2][0]);
    for (int k = 0; k < 3; ++k) U[k][0] /= det;
    M3 r;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r.m[i][j] = dot3_eigen(U[i][0], U[i][1], U[i][2], V[j][0], V[j][1], V[j][2]);
    return r;
}

struct Iso { M3 R; V3 t; };  // Eigen::Isometry3d
inline Iso iso_identity() { return {m3_identity(), {0, 0, 0}}; }
inline Iso iso_mul(const Iso& a, const Iso& b) {   // Transform * Transform
    V3 rt = mvec(a.R, b.t);
    return {mmul(a.R, b.R), add(rt, a.t)};
}
inline Iso iso_inv(const Iso& a) {                 // Isometry inverse: (R^T, -R^T t)
    M3 rt = mtrans(a.R);
    V3 tt = mvec(rt, a.t);
    return {rt, {-tt.x, -tt.y, -tt.z}};
}

// skew (src/lidarOptimization.cpp:145-155)
inline M3 skew(V3 v) {
    M3 s{};
    s.m[0][1] = -v.z; s.m[0][2] = v.y; s.m[1][2] = -v.x;
    s.m[1][0] = v.z;  s.m[2][0] = -v.y; s.m[2][1] = v.x;
    return s;
}

// getTransformFromSe3 (src/lidarOptimization.cpp:106-143)
void trig_dump(double v);   // development: PFREF_TRIG_DUMP (pfref_odom.cpp)
extern thread_local bool g_ld_trig;   // PFREF_LD_TRIG for the solve in progress
extern thread_local bool g_qr_rev;    // PFREF_QR_REVSUM for the solve in progress
extern thread_local bool g_dev_half;  // PFREF_DEV_HALFANGLE for the solve in progress
inline double lsin(double x) { return g_ld_trig ? (double)sinl((long double)x) : std::sin(x); }
inline double lcos(double x) { return g_ld_trig ? (double)cosl((long double)x) : std::cos(x); }
inline double lcube(double x) {
    return g_ld_trig ? (double)((long double)x * (long double)x * (long double)x) : std::pow(x, 3);
}
inline void se3_exp(const double se3[6], Quat& q, V3& t) {
    V3 omega{se3[0], se3[1], se3[2]};
    V3 upsilon{se3[3], se3[4], se3[5]};
    M3 Omega = skew(omega);
    double theta = norm(omega);
    trig_dump(theta);
    double half_theta = 0.5 * theta;
    double imag_factor;
    double real_factor = lcos(half_theta);
    if (theta < 1e-10) {
        double theta_sq = theta * theta;
        double theta_po4 = theta_sq * theta_sq;
        imag_factor = 0.5 - 0.0208333 * theta_sq + 0.000260417 * theta_po4;
    } else {
        double sin_half_theta = lsin(half_theta);
        imag_factor = sin_half_theta / theta;
    }
    q = {imag_factor * omega.x, imag_factor * omega.y, imag_factor * omega.z, real_factor};
    M3 J;
    if (theta < 1e-10) {
        J = q2m(q);
    } else {
        M3 Omega2 = mmul(Omega, Omega);
        double a = (1.0 - lcos(theta)) / (theta * theta);
        double b = (theta - lsin(theta)) / lcube(theta);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                J.m[i][j] = (i == j ? 1.0 : 0.0) + a * Omega.m[i][j] + b * Omega2.m[i][j];
    }
    t = mvec(J, upsilon);
}

// PoseSE3Parameterization::Plus (src/lidarOptimization.cpp:80-95)
inline void se3_plus(const double* x, const double* delta, double* out) {
    V3 trans{x[4], x[5], x[6]};
    Quat dq; V3 dt;
    se3_exp(delta, dq, dt);
    Quat quater{x[0], x[1], x[2], x[3]};
    Quat qp = qmul(dq, quater);
    V3 tp = add(qrot(dq, trans), dt);
    out[0] = qp.x; out[1] = qp.y; out[2] = qp.z; out[3] = qp.w;
    out[4] = tp.x; out[5] = tp.y; out[6] = tp.z;
}

// --- GPU_EQUIV (PFREF_LM_NORMAL_EQ) SE(3) update -----------------------------------------
// The device evaluates getTransformFromSe3 with ONE sincos of theta/2 and the half-angle identities
// sin(theta) = 2 s c, 1 - cos(theta) = 2 s^2, theta^3 as a product, and takes that sincos from a
// routine built from + - * and rint only, so the host and gfx950 agree to the bit (libm's and the
// device library's sin/cos differ in the last ulp now and then). Both are restated here; each
// value is within ~1 ulp of se3_exp above (tests/test_oracle_units.py bounds the difference).
// Cody-Waite reduction by pi/2 (two 33-bit parts), fdlibm's minimax sin/cos kernels on [-pi/4, pi/4].
inline void det_sincos(double x, double* sn, double* cs) {
    const double invpio2 = 6.36619772367581382433e-01;
    const double pio2_1 = 1.57079632673412561417e+00;
    const double pio2_1t = 6.07710050650619224932e-11;
    const double k = std::rint(x * invpio2);
    const double r = (x - k * pio2_1) - k * pio2_1t;
    const double z = r * r;
    const double v = z * r;
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double s = r + v * (S1 + z * (S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)))));
    const double pc = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    const double c = w + (((1.0 - w) - hz) + z * pc);
    const long long n = (k == k && std::fabs(k) < 9.0e15) ? (long long)k : 0;
    switch ((int)(n & 3)) {
        case 0: *sn = s; *cs = c; break;
        case 1: *sn = c; *cs = -s; break;
        case 2: *sn = -s; *cs = -c; break;
        default: *sn = -c; *cs = s; break;
    }
}
inline void se3_exp_half(const double se3[6], Quat& q, V3& t) {
    V3 omega{se3[0], se3[1], se3[2]};
    V3 upsilon{se3[3], se3[4], se3[5]};
    M3 Omega = skew(omega);
    const double theta = norm(omega);
    const double half_theta = 0.5 * theta;
    double s_h, c_h;
    det_sincos(half_theta, &s_h, &c_h);
    double imag_factor;
    if (theta < 1e-10) {
        const double theta_sq = theta * theta;
        const double theta_po4 = theta_sq * theta_sq;
        imag_factor = 0.5 - 0.0208333 * theta_sq + 0.000260417 * theta_po4;
    } else {
        imag_factor = s_h / theta;
    }
    q = {imag_factor * omega.x, imag_factor * omega.y, imag_factor * omega.z, c_h};
    M3 J;
    if (theta < 1e-10) {
        J = q2m(q);
    } else {
        M3 Omega2 = mmul(Omega, Omega);
        double a, b;
        if (!g_dev_half) {                               // the reference's own form, full-angle sincos
            double s_t, c_t;
            det_sincos(theta, &s_t, &c_t);
            a = (1.0 - c_t) / (theta * theta);
            b = (theta - s_t) / (theta * theta * theta);
        } else {                                         // round 3's half-angle identities (experiment)
            a = (2.0 * (s_h * s_h)) / (theta * theta);
            b = (theta - 2.0 * (s_h * c_h)) / (theta * theta * theta);
        }
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) J.m[i][j] = (i == j ? 1.0 : 0.0) + a * Omega.m[i][j] + b * Omega2.m[i][j];
    }
    t = mvec(J, upsilon);
}
inline void se3_plus_half(const double* x, const double* delta, double* out) {
    V3 trans{x[4], x[5], x[6]};
    Quat dq; V3 dt;
    se3_exp_half(delta, dq, dt);
    Quat quater{x[0], x[1], x[2], x[3]};
    Quat qp = qmul(dq, quater);
    V3 tp = add(qrot(dq, trans), dt);
    out[0] = qp.x; out[1] = qp.y; out[2] = qp.z; out[3] = qp.w;
    out[4] = tp.x; out[5] = tp.y; out[6] = tp.z;
}

// EdgeAnalyticCostFunction::Evaluate (src/lidarOptimization.cpp:12-46); J has 7 entries, J[6]=0
inline double edge_eval(const double* x, V3 cur, V3 a, V3 b, double w, double* J) {
    Quat q{x[0], x[1], x[2], x[3]};
    V3 lp = add(qrot(q, cur), V3{x[4], x[5], x[6]});
    V3 nu = cross(sub(lp, a), sub(lp, b));
    V3 de = sub(a, b);
    double de_norm = norm(de);
    double r = norm(nu) / de_norm;
    if (w == 1 || w == 2) r = w * r;
    else if (w == 12) r = w * r;
    if (J) {
        M3 sl = skew(lp);
        double dp[3][6];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) { dp[i][j] = -sl.m[i][j]; dp[i][3 + j] = (i == j) ? 1.0 : 0.0; }
        M3 sd = skew(de);
        double nn = norm(nu);
        double v1[3] = {-nu.x / nn, -nu.y / nn, -nu.z / nn};
        double v2[3];
        for (int j = 0; j < 3; ++j) v2[j] = v1[0] * sd.m[0][j] + v1[1] * sd.m[1][j] + v1[2] * sd.m[2][j];
        for (int j = 0; j < 6; ++j) J[j] = (v2[0] * dp[0][j] + v2[1] * dp[1][j] + v2[2] * dp[2][j]) / de_norm;
        J[6] = 0.0;
    }
    return r;
}

// SurfNormAnalyticCostFunction::Evaluate (src/lidarOptimization.cpp:56-78)
inline double surf_eval(const double* x, V3 cur, V3 n, double d, double w, double* J) {
    Quat q{x[0], x[1], x[2], x[3]};
    V3 pw = add(qrot(q, cur), V3{x[4], x[5], x[6]});
    double r = dot(n, pw) + d;
    if (w != 0) r = w * r;
    if (J) {
        M3 sp = skew(pw);
        double dp[3][6];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) { dp[i][j] = -sp.m[i][j]; dp[i][3 + j] = (i == j) ? 1.0 : 0.0; }
        for (int j = 0; j < 6; ++j) J[j] = n.x * dp[0][j] + n.y * dp[1][j] + n.z * dp[2][j];
        J[6] = 0.0;
    }
    return r;
}

// Symmetric 3x3 eigen-decomposition by cyclic Jacobi rotations, eigenvalues ascending,
// eigenvectors as columns (restates Eigen::SelfAdjointEigenSolver<Matrix3d>'s contract;
// its tridiagonal-QL rounding is not reproduced: parity unpinned).
inline void eigen_sym3(const double in[3][3], double ev[3], double V[3][3]) {
    double a[3][3];
    std::memcpy(a, in, sizeof(a));
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) V[i][j] = (i == j) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 50; ++sweep) {
        double off = a[0][1] * a[0][1] + a[0][2] * a[0][2] + a[1][2] * a[1][2];
        double diag = a[0][0] * a[0][0] + a[1][1] * a[1][1] + a[2][2] * a[2][2];
        if (off <= 1e-36 * diag || off == 0.0) break;
        for (int p = 0; p < 2; ++p) {
            for (int q = p + 1; q < 3; ++q) {
                double apq = a[p][q];
                if (apq == 0.0) continue;
                double theta = (a[q][q] - a[p][p]) / (2.0 * apq);
                double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
                double c = 1.0 / std::sqrt(t * t + 1.0);
                double s = t * c;
                for (int k = 0; k < 3; ++k) {   // A <- A J (columns p, q)
                    double akp = a[k][p], akq = a[k][q];
                    a[k][p] = c * akp - s * akq;
                    a[k][q] = s * akp + c * akq;
                }
                for (int k = 0; k < 3; ++k) {   // A <- J^T A (rows p, q)
                    double apk = a[p][k], aqk = a[q][k];
                    a[p][k] = c * apk - s * aqk;
                    a[q][k] = s * apk + c * aqk;
                }
                for (int k = 0; k < 3; ++k) {
                    double vkp = V[k][p], vkq = V[k][q];
                    V[k][p] = c * vkp - s * vkq;
                    V[k][q] = s * vkp + c * vkq;
                }
            }
        }
    }
    double d[3] = {a[0][0], a[1][1], a[2][2]};
    int order[3] = {0, 1, 2};
    std::sort(order, order + 3, [&](int i, int j) { return d[i] < d[j] || (d[i] == d[j] && i < j); });
    double Vs[3][3];
    for (int c = 0; c < 3; ++c) {
        ev[c] = d[order[c]];
        for (int r = 0; r < 3; ++r) Vs[r][c] = V[r][order[c]];
    }
    std::memcpy(V, Vs, sizeof(Vs));
}

// Eigen makeHouseholder on x[0..n): returns tau, beta; essential part in ess[1..n)
inline void make_householder(const double* x, int n, double* ess, double& tau, double& beta) {
    double tail = 0.0;
    if (g_qr_rev)
        for (int i = n - 1; i >= 1; --i) tail += x[i] * x[i];
    else
        for (int i = 1; i < n; ++i) tail += x[i] * x[i];
    double c0 = x[0];
    const double tol = std::numeric_limits<double>::min();
    if (tail <= tol) {
        tau = 0.0; beta = c0;
        for (int i = 1; i < n; ++i) ess[i] = 0.0;
    } else {
        beta = std::sqrt(c0 * c0 + tail);
        if (c0 >= 0.0) beta = -beta;
        for (int i = 1; i < n; ++i) ess[i] = x[i] / (c0 - beta);
        tau = (beta - c0) / beta;
    }
}

// ColPivHouseholderQR<Matrix<double,5,3>>::solve(-1 vector) (src/odomEstimationClass.cpp:449-461),
// restating Eigen 3.3.9 ColPivHouseholderQR::computeInPlace + _solve_impl operation order.
inline V3 plane_fit5(const double A_in[5][3]) {
    const int R = 5, C = 3;
    double A[5][3];
    std::memcpy(A, A_in, sizeof(A));
    double b[5] = {-1, -1, -1, -1, -1};
    int perm[3] = {0, 1, 2};
    double hc[3];
    double colnorm[3], colnorm_upd[3];
    const double eps = std::numeric_limits<double>::epsilon();
    double maxnorm = 0.0;
    for (int j = 0; j < C; ++j) {
        double s = 0; for (int i = 0; i < R; ++i) s += A[i][j] * A[i][j];
        colnorm[j] = std::sqrt(s); colnorm_upd[j] = colnorm[j];
        if (j == 0 || colnorm[j] > maxnorm) maxnorm = colnorm[j];
    }
    const double thr_helper = (maxnorm * eps) * (maxnorm * eps) / (double)R;
    const double downdate_thr = std::sqrt(eps);
    int nonzero = C;
    for (int k = 0; k < C; ++k) {
        int best = k;
        double bn = colnorm_upd[k];
        for (int j = k + 1; j < C; ++j)
            if (colnorm_upd[j] > bn) { bn = colnorm_upd[j]; best = j; }
        double bsq = bn * bn;
        if (nonzero == C && bsq < thr_helper * (double)(R - k)) nonzero = k;
        if (best != k) {
            for (int i = 0; i < R; ++i) std::swap(A[i][k], A[i][best]);
            std::swap(perm[k], perm[best]);
            std::swap(colnorm[k], colnorm[best]);
            std::swap(colnorm_upd[k], colnorm_upd[best]);
        }
        double x[5] = {0, 0, 0, 0, 0}, ess[5] = {0, 0, 0, 0, 0};
        int n = R - k;
        for (int i = 0; i < n; ++i) x[i] = A[k + i][k];
        double tau, beta;
        make_householder(x, n, ess, tau, beta);
        A[k][k] = beta;
        for (int i = 1; i < n; ++i) A[k + i][k] = ess[i];
        hc[k] = tau;
        if (tau != 0.0 && n > 1) {           // applyHouseholderOnTheLeft
            for (int j = k + 1; j < C; ++j) {
                double tmp = 0.0;
                for (int i = 1; i < n; ++i) tmp += ess[i] * A[k + i][j];
                tmp += A[k][j];
                A[k][j] -= tau * tmp;
                for (int i = 1; i < n; ++i) A[k + i][j] -= tau * ess[i] * tmp;
            }
        }
        for (int j = k + 1; j < C; ++j) {    // stable column-norm downdate (LAPACK xGEQPF)
            if (colnorm_upd[j] != 0.0) {
                double temp = std::fabs(A[k][j]) / colnorm_upd[j];
                temp = (1.0 + temp) * (1.0 - temp);
                temp = temp < 0.0 ? 0.0 : temp;
                double rr = colnorm_upd[j] / colnorm[j];
                double temp2 = temp * (rr * rr);
                if (temp2 <= downdate_thr) {
                    double s = 0; for (int i = k + 1; i < R; ++i) s += A[i][j] * A[i][j];
                    colnorm[j] = std::sqrt(s); colnorm_upd[j] = colnorm[j];
                } else {
                    colnorm_upd[j] *= std::sqrt(temp);
                }
            }
        }
    }
    double out[3] = {0, 0, 0};
    if (nonzero == 0) return {0, 0, 0};
    for (int k = 0; k < nonzero; ++k) {      // c = Q^T b (householder sequence, length nonzero)
        int n = R - k;
        if (hc[k] == 0.0 || n < 2) continue;
        double tmp = 0.0;
        for (int i = 1; i < n; ++i) tmp += A[k + i][k] * b[k + i];
        tmp += b[k];
        b[k] -= hc[k] * tmp;
        for (int i = 1; i < n; ++i) b[k + i] -= hc[k] * A[k + i][k] * tmp;
    }
    for (int i = nonzero - 1; i >= 0; --i) { // upper-triangular solve, column oriented
        b[i] /= A[i][i];
        for (int s = 0; s < i; ++s) b[s] -= b[i] * A[s][i];
    }
    for (int k = 0; k < nonzero; ++k) out[perm[k]] = b[k];
    return {out[0], out[1], out[2]};
}

}  // namespace pfref
