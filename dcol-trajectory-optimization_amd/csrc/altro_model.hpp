// altro_model.hpp -- continuous dynamics and RK4 step of the three reference systems,
// shared by the host library (altro_host.cpp, g++) and the device Jacobian kernel
// (altro_device.hip, hipcc).  Both translation units compile it WITHOUT floating-point
// contraction (-ffp-contract=off) and with IEEE division and square root, so a knot's
// Jacobian is bitwise the same on either side (tests/test_altro_device.py).
#pragma once
#include <math.h>

#include "../../include/dcol_altro.h"

#if defined(__HIPCC__)
#define DCOL_AHD __host__ __device__ inline
#else
#define DCOL_AHD inline
#endif

namespace dcol_altro {

constexpr int MX = DCOL_ALTRO_MAX_NX;
constexpr int MU = DCOL_ALTRO_MAX_NU;

// ------------------------------------------------------------------------ small algebra
DCOL_AHD void skew(const double* p, double S[9]) {
    S[0] = 0;     S[1] = -p[2]; S[2] = p[1];
    S[3] = p[2];  S[4] = 0;     S[5] = -p[0];
    S[6] = -p[1]; S[7] = p[0];  S[8] = 0;
}

DCOL_AHD void mat3_mul(const double* A, const double* B, double* C) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

DCOL_AHD void mat3_vec(const double* A, const double* x, double* y) {
    for (int i = 0; i < 3; ++i) y[i] = A[3 * i] * x[0] + A[3 * i + 1] * x[1] + A[3 * i + 2] * x[2];
}

DCOL_AHD void cross(const double* a, const double* b, double* c) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

// x = J^{-1} b by Gaussian elimination with partial pivoting (LAPACK dgesv semantics).
DCOL_AHD void solve3(const double* Jm, const double* b, double* x) {
    double a[9], r[3];
    for (int i = 0; i < 9; ++i) a[i] = Jm[i];
    for (int i = 0; i < 3; ++i) r[i] = b[i];
    for (int c = 0; c < 3; ++c) {
        int piv = c;
        for (int i = c + 1; i < 3; ++i)
            if (fabs(a[3 * i + c]) > fabs(a[3 * piv + c])) piv = i;
        if (piv != c) {
            for (int j = 0; j < 3; ++j) {
                const double t = a[3 * c + j];
                a[3 * c + j] = a[3 * piv + j];
                a[3 * piv + j] = t;
            }
            const double t = r[c];
            r[c] = r[piv];
            r[piv] = t;
        }
        for (int i = c + 1; i < 3; ++i) {
            const double l = a[3 * i + c] / a[3 * c + c];
            for (int j = c; j < 3; ++j) a[3 * i + j] -= l * a[3 * c + j];
            r[i] -= l * r[c];
        }
    }
    for (int i = 2; i >= 0; --i) {
        double s = r[i];
        for (int j = i + 1; j < 3; ++j) s -= a[3 * i + j] * x[j];
        x[i] = s / a[3 * i + i];
    }
}

// Rotation matrix of MRP p, expanded like primitives/problem_matrices.py dcm_from_mrp.
DCOL_AHD void dcm_from_mrp(const double* p, double Q[9]) {
    const double q1 = p[0] * p[0], q2 = p[1] * p[1], q3 = p[2] * p[2];
    const double s = q1 + q2 + q3 + 1, den = s * s;
    const double a = 4 * q1 + 4 * q2 + 4 * q3 - 4;
    auto dg = [den](double u, double v) { return -((8 * u + 8 * v) / den - 1) * den; };
    const double M[9] = {dg(q2, q3),
                         8 * p[0] * p[1] + p[2] * a,
                         8 * p[0] * p[2] - p[1] * a,
                         8 * p[0] * p[1] - p[2] * a,
                         dg(q1, q3),
                         8 * p[1] * p[2] + p[0] * a,
                         8 * p[0] * p[2] + p[1] * a,
                         8 * p[1] * p[2] - p[0] * a,
                         dg(q1, q2)};
    const double iden = 1.0 / den;
    for (int i = 0; i < 9; ++i) Q[i] = M[i] * iden;
}

// --------------------------------------------------------------------- continuous models
// piano_mover.py:7-25: x = [rx ry vx vy theta omega], u = [ax ay tau].
DCOL_AHD void f_piano(const dcol_altro_model& m, const double* x, const double* u, double* xd) {
    xd[0] = x[2];
    xd[1] = x[3];
    xd[2] = u[0];
    xd[3] = u[1];
    xd[4] = x[5];
    xd[5] = u[2] / m.u_scale;
}

// MRP kinematics factor (I + 2(S^2 + S)/(1+|p|^2)) shared by both 3-D models.
DCOL_AHD void mrp_kin(const double* p, double n2, double M[9]) {
    double S[9], SS[9];
    skew(p, S);
    mat3_mul(S, S, SS);
    const double inv = 1.0 / (1 + n2);
    for (int i = 0; i < 9; ++i) M[i] = ((i % 4 == 0) ? 1.0 : 0.0) + 2 * (SS[i] + S[i]) * inv;
}

DCOL_AHD void euler_rate(const dcol_altro_model& m, const double* w, const double* tau, double* wd) {
    double Jw[3], c[3], rhs[3];
    mat3_vec(m.inertia, w, Jw);
    cross(w, Jw, c);
    for (int i = 0; i < 3; ++i) rhs[i] = tau[i] - c[i];
    solve3(m.inertia, rhs, wd);
}

// cluttered_hallway_quadrotor.py:19-84 (constants carried in the model struct).
DCOL_AHD void f_quad(const dcol_altro_model& m, const double* x, const double* u, double* xd) {
    const double* p = x + 6;
    const double* w = x + 9;
    double Q[9];
    dcm_from_mrp(p, Q);
    double F[4], Mt[4];
    for (int i = 0; i < 4; ++i) {
        F[i] = fmax(0.0, m.kf * u[i]);
        Mt[i] = m.km * u[i];
    }
    const double Fz = F[0] + F[1] + F[2] + F[3];
    const double tau[3] = {m.arm * (F[1] - F[3]), m.arm * (F[2] - F[0]), Mt[0] - Mt[1] + Mt[2] - Mt[3]};
    for (int i = 0; i < 3; ++i) {
        xd[i] = x[3 + i];
        xd[3 + i] = (m.mass * m.gravity[i] + Q[3 * i + 2] * Fz) / m.mass;
    }
    const double n2 = p[0] * p[0] + p[1] * p[1] + p[2] * p[2];
    double K[9];
    mrp_kin(p, n2, K);
    const double c = (1 + n2) / 4;
    for (int i = 0; i < 9; ++i) K[i] = c * K[i];
    mat3_vec(K, w, xd + 6);
    euler_rate(m, w, tau, xd + 9);
}

// cone_through_wall.py:19-52: force/torque-actuated rigid body, x = [r v p w], u = [f tau].
DCOL_AHD void f_rigid(const dcol_altro_model& m, const double* x, const double* u, double* xd) {
    const double* p = x + 6;
    const double* w = x + 9;
    for (int i = 0; i < 3; ++i) {
        xd[i] = x[3 + i];
        xd[3 + i] = u[i] / m.mass;
    }
    const double np_ = sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]);
    const double n2 = np_ * np_;
    double K[9], pd[3];
    mrp_kin(p, n2, K);
    mat3_vec(K, w, pd);
    const double c = (1 + n2) / 4;
    for (int i = 0; i < 3; ++i) xd[6 + i] = c * pd[i];
    euler_rate(m, w, u + 3, xd + 9);
}

DCOL_AHD void f_model(const dcol_altro_model& m, const double* x, const double* u, double* xd) {
    switch (m.system) {
        case DCOL_SYS_PIANO: f_piano(m, x, u, xd); break;
        case DCOL_SYS_QUADROTOR: f_quad(m, x, u, xd); break;
        default: f_rigid(m, x, u, xd); break;
    }
}

// RK4 step (piano_mover.py:28-47 and the identical discrete_dynamics of the 3-D systems).
DCOL_AHD void rk4(const dcol_altro_model& m, const double* x, const double* u, double* xn) {
    const int nx = m.nx;
    double k1[MX] = {}, k2[MX] = {}, k3[MX] = {}, k4[MX] = {}, t[MX] = {};
    f_model(m, x, u, k1);
    for (int i = 0; i < nx; ++i) k1[i] = m.dt * k1[i];
    for (int i = 0; i < nx; ++i) t[i] = x[i] + 0.5 * k1[i];
    f_model(m, t, u, k2);
    for (int i = 0; i < nx; ++i) k2[i] = m.dt * k2[i];
    for (int i = 0; i < nx; ++i) t[i] = x[i] + 0.5 * k2[i];
    f_model(m, t, u, k3);
    for (int i = 0; i < nx; ++i) k3[i] = m.dt * k3[i];
    for (int i = 0; i < nx; ++i) t[i] = x[i] + k3[i];
    f_model(m, t, u, k4);
    for (int i = 0; i < nx; ++i) k4[i] = m.dt * k4[i];
    const double sixth = 1.0 / 6.0;
    for (int i = 0; i < nx; ++i) xn[i] = x[i] + sixth * (k1[i] + 2 * k2[i] + 2 * k3[i] + k4[i]);
}

bool model_ok(const dcol_altro_model* m) {
    if (!m || m->nx <= 0 || m->nx > MX || m->nu <= 0 || m->nu > MU) return false;
    switch (m->system) {
        case DCOL_SYS_PIANO: return m->nx == 6 && m->nu == 3 && m->u_scale != 0;
        case DCOL_SYS_QUADROTOR: return m->nx == 12 && m->nu == 4 && m->mass != 0;
        case DCOL_SYS_RIGID: return m->nx == 12 && m->nu == 6 && m->mass != 0;
        default: return false;
    }
}

}  // namespace dcol_altro
