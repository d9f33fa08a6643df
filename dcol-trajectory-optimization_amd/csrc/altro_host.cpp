// Native host kernels of the batched ALTRO driver (include/dcol_altro.h).
//
// These are the knot-sequential pieces of the AL-iLQR loop that stay on the CPU: at the
// reference's sizes (N = 60..100 knots, nx <= 12, nu <= 6) one backward or forward sweep
// is a few microseconds of scalar FP64 here, while a GPU launch alone costs more — the
// knot-parallel work (all N x n_obs proximity solves of a phase) goes to the device
// through dcol.h instead.
//
// Arithmetic follows the reference's expression order (numpy evaluates left to right,
// no contraction: this file is compiled with -ffp-contract=off) so results agree with it
// to rounding; 3-term dot products inside BLAS may differ in the last bit.
#include "../../include/dcol_altro.h"

#include <cmath>
#include <cstring>

namespace {

constexpr int MX = DCOL_ALTRO_MAX_NX;
constexpr int MU = DCOL_ALTRO_MAX_NU;

// ------------------------------------------------------------------------ small algebra
inline void skew(const double* p, double S[9]) {
    S[0] = 0;     S[1] = -p[2]; S[2] = p[1];
    S[3] = p[2];  S[4] = 0;     S[5] = -p[0];
    S[6] = -p[1]; S[7] = p[0];  S[8] = 0;
}

inline void mat3_mul(const double* A, const double* B, double* C) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

inline void mat3_vec(const double* A, const double* x, double* y) {
    for (int i = 0; i < 3; ++i) y[i] = A[3 * i] * x[0] + A[3 * i + 1] * x[1] + A[3 * i + 2] * x[2];
}

inline void cross(const double* a, const double* b, double* c) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

// x = J^{-1} b by Gaussian elimination with partial pivoting (LAPACK dgesv semantics).
inline void solve3(const double* Jm, const double* b, double* x) {
    double a[9], r[3];
    std::memcpy(a, Jm, sizeof(a));
    std::memcpy(r, b, sizeof(r));
    for (int c = 0; c < 3; ++c) {
        int piv = c;
        for (int i = c + 1; i < 3; ++i)
            if (std::fabs(a[3 * i + c]) > std::fabs(a[3 * piv + c])) piv = i;
        if (piv != c) {
            for (int j = 0; j < 3; ++j) std::swap(a[3 * c + j], a[3 * piv + j]);
            std::swap(r[c], r[piv]);
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
inline void dcm_from_mrp(const double* p, double Q[9]) {
    const double q1 = p[0] * p[0], q2 = p[1] * p[1], q3 = p[2] * p[2];
    const double s = q1 + q2 + q3 + 1, den = s * s;
    const double a = 4 * q1 + 4 * q2 + 4 * q3 - 4;
    auto dg = [&](double u, double v) { return -((8 * u + 8 * v) / den - 1) * den; };
    const double M[9] = {dg(q2, q3),
                         8 * p[0] * p[1] + p[2] * a,
                         8 * p[0] * p[2] - p[1] * a,
                         8 * p[0] * p[1] - p[2] * a,
                         dg(q1, q3),
                         8 * p[1] * p[2] + p[0] * a,
                         8 * p[0] * p[2] + p[1] * a,
                         8 * p[1] * p[2] - p[0] * a,
                         dg(q1, q2)};
    for (int i = 0; i < 9; ++i) Q[i] = M[i] / den;
}

// --------------------------------------------------------------------- continuous models
// piano_mover.py:7-25: x = [rx ry vx vy theta omega], u = [ax ay tau].
inline void f_piano(const dcol_altro_model& m, const double* x, const double* u, double* xd) {
    xd[0] = x[2];
    xd[1] = x[3];
    xd[2] = u[0];
    xd[3] = u[1];
    xd[4] = x[5];
    xd[5] = u[2] / m.u_scale;
}

// MRP kinematics factor (I + 2(S^2 + S)/(1+|p|^2)) shared by both 3-D models.
inline void mrp_kin(const double* p, double n2, double M[9]) {
    double S[9], SS[9];
    skew(p, S);
    mat3_mul(S, S, SS);
    for (int i = 0; i < 9; ++i) M[i] = ((i % 4 == 0) ? 1.0 : 0.0) + 2 * (SS[i] + S[i]) / (1 + n2);
}

inline void euler_rate(const dcol_altro_model& m, const double* w, const double* tau, double* wd) {
    double Jw[3], c[3], rhs[3];
    mat3_vec(m.inertia, w, Jw);
    cross(w, Jw, c);
    for (int i = 0; i < 3; ++i) rhs[i] = tau[i] - c[i];
    solve3(m.inertia, rhs, wd);
}

// cluttered_hallway_quadrotor.py:19-84 (constants carried in the model struct).
inline void f_quad(const dcol_altro_model& m, const double* x, const double* u, double* xd) {
    const double* p = x + 6;
    const double* w = x + 9;
    double Q[9];
    dcm_from_mrp(p, Q);
    double F[4], Mt[4];
    for (int i = 0; i < 4; ++i) {
        F[i] = std::fmax(0.0, m.kf * u[i]);
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
inline void f_rigid(const dcol_altro_model& m, const double* x, const double* u, double* xd) {
    const double* p = x + 6;
    const double* w = x + 9;
    for (int i = 0; i < 3; ++i) {
        xd[i] = x[3 + i];
        xd[3 + i] = u[i] / m.mass;
    }
    const double np_ = std::sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]);
    const double n2 = np_ * np_;
    double K[9], pd[3];
    mrp_kin(p, n2, K);
    mat3_vec(K, w, pd);
    const double c = (1 + n2) / 4;
    for (int i = 0; i < 3; ++i) xd[6 + i] = c * pd[i];
    euler_rate(m, w, u + 3, xd + 9);
}

inline void f_model(const dcol_altro_model& m, const double* x, const double* u, double* xd) {
    switch (m.system) {
        case DCOL_SYS_PIANO: f_piano(m, x, u, xd); break;
        case DCOL_SYS_QUADROTOR: f_quad(m, x, u, xd); break;
        default: f_rigid(m, x, u, xd); break;
    }
}

// RK4 step (piano_mover.py:28-47 and the identical discrete_dynamics of the 3-D systems).
inline void rk4(const dcol_altro_model& m, const double* x, const double* u, double* xn) {
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

// In-place lower Cholesky of the n x n SPD matrix a (row-major); false if not PD.
bool cholesky(double* a, int n) {
    for (int j = 0; j < n; ++j) {
        double d = a[j * n + j];
        for (int k = 0; k < j; ++k) d -= a[j * n + k] * a[j * n + k];
        if (!(d > 0)) return false;
        const double l = std::sqrt(d);
        a[j * n + j] = l;
        for (int i = j + 1; i < n; ++i) {
            double s = a[i * n + j];
            for (int k = 0; k < j; ++k) s -= a[i * n + k] * a[j * n + k];
            a[i * n + j] = s / l;
        }
    }
    return true;
}

// Solve (L L') x = b in place for one right-hand side.
void chol_solve(const double* L, int n, double* b) {
    for (int i = 0; i < n; ++i) {
        double s = b[i];
        for (int k = 0; k < i; ++k) s -= L[i * n + k] * b[k];
        b[i] = s / L[i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
        double s = b[i];
        for (int k = i + 1; k < n; ++k) s -= L[k * n + i] * b[k];
        b[i] = s / L[i * n + i];
    }
}

}  // namespace

extern "C" {

int32_t dcol_altro_abi_version(void) { return DCOL_ALTRO_ABI_VERSION; }

int dcol_altro_dynamics(const dcol_altro_model* m, int64_t M, const double* X, const double* U, double* Xn) {
    if (!model_ok(m) || M < 0 || (M > 0 && (!X || !U || !Xn))) return DCOL_ALTRO_ERR_ARG;
    for (int64_t i = 0; i < M; ++i) rk4(*m, X + i * m->nx, U + i * m->nu, Xn + i * m->nx);
    return DCOL_ALTRO_OK;
}

int dcol_altro_jacobians(const dcol_altro_model* m, int64_t T, const double* X, const double* U, double delta,
                         double* A, double* B) {
    if (!model_ok(m) || T < 0 || (T > 0 && (!X || !U || !A || !B)) || !(delta != 0)) return DCOL_ALTRO_ERR_ARG;
    const int nx = m->nx, nu = m->nu;
    // knots are independent: spread them over the host cores for the larger problems
#pragma omp parallel for schedule(static) if (T * (nx + nu) >= 512)
    for (int64_t t = 0; t < T; ++t) {
        double f0[MX], f1[MX], xp[MX], up[MU];
        const double* x = X + t * nx;
        const double* u = U + t * nu;
        double* At = A + t * nx * nx;
        double* Bt = B + t * nx * nu;
        rk4(*m, x, u, f0);
        for (int j = 0; j < nx; ++j) {
            std::memcpy(xp, x, sizeof(double) * nx);
            xp[j] += delta;
            rk4(*m, xp, u, f1);
            for (int i = 0; i < nx; ++i) At[i * nx + j] = (f1[i] - f0[i]) / delta;
        }
        for (int j = 0; j < nu; ++j) {
            std::memcpy(up, u, sizeof(double) * nu);
            up[j] += delta;
            rk4(*m, x, up, f1);
            for (int i = 0; i < nx; ++i) Bt[i * nu + j] = (f1[i] - f0[i]) / delta;
        }
    }
    return DCOL_ALTRO_OK;
}

int dcol_altro_backward(int64_t T, int32_t nx, int32_t nu, const double* A, const double* B, const double* lx,
                        const double* lu, const double* lxx, const double* luu, const double* VxT,
                        const double* VxxT, double reg, double* K, double* k, double* dJ, int64_t* fail_knot) {
    if (T < 0 || nx <= 0 || nx > MX || nu <= 0 || nu > MU || !VxT || !VxxT || !dJ) return DCOL_ALTRO_ERR_ARG;
    if (T > 0 && (!A || !B || !lx || !lu || !lxx || !luu || !K || !k)) return DCOL_ALTRO_ERR_ARG;
    double Vx[MX], Vxx[MX * MX], P[MX * MX];
    double PB[MX * MU], PA[MX * MX], Qu[MU], Quu[MU * MU], Qux[MU * MX], L[MU * MU];
    double Acl[MX * MX], VA[MX * MX], LK[MU * MX], t1[MX], t2[MX], nVx[MX], nVxx[MX * MX];
    std::memcpy(Vx, VxT, sizeof(double) * nx);
    std::memcpy(Vxx, VxxT, sizeof(double) * nx * nx);
    double acc = 0;
    for (int64_t t = T - 1; t >= 0; --t) {
        const double* At = A + t * nx * nx;
        const double* Bt = B + t * nx * nu;
        const double* lxt = lx + t * nx;
        const double* lut = lu + t * nu;
        const double* lxxt = lxx + t * nx * nx;
        const double* luut = luu + t * nu * nu;
        double* Kt = K + t * nu * nx;
        double* kt = k + t * nu;
        // P = Vxx' + reg I ; PB = P B ; PA = P A
        for (int i = 0; i < nx; ++i)
            for (int j = 0; j < nx; ++j) P[i * nx + j] = Vxx[i * nx + j] + (i == j ? reg : 0.0);
        for (int i = 0; i < nx; ++i) {
            for (int j = 0; j < nu; ++j) {
                double s = 0;
                for (int q = 0; q < nx; ++q) s += P[i * nx + q] * Bt[q * nu + j];
                PB[i * nu + j] = s;
            }
            for (int j = 0; j < nx; ++j) {
                double s = 0;
                for (int q = 0; q < nx; ++q) s += P[i * nx + q] * At[q * nx + j];
                PA[i * nx + j] = s;
            }
        }
        // Qu = lu + B'Vx' ; Quu = luu + B'PB ; Qux = B'PA
        for (int i = 0; i < nu; ++i) {
            double s = 0;
            for (int q = 0; q < nx; ++q) s += Bt[q * nu + i] * Vx[q];
            Qu[i] = lut[i] + s;
            for (int j = 0; j < nu; ++j) {
                double r = 0;
                for (int q = 0; q < nx; ++q) r += Bt[q * nu + i] * PB[q * nu + j];
                Quu[i * nu + j] = luut[i * nu + j] + r;
            }
            for (int j = 0; j < nx; ++j) {
                double r = 0;
                for (int q = 0; q < nx; ++q) r += Bt[q * nu + i] * PA[q * nx + j];
                Qux[i * nx + j] = r;
            }
        }
        std::memcpy(L, Quu, sizeof(double) * nu * nu);
        if (!cholesky(L, nu)) {
            if (fail_knot) *fail_knot = t;
            return DCOL_ALTRO_ERR_NOT_PD;
        }
        for (int i = 0; i < nu; ++i) kt[i] = Qu[i];
        chol_solve(L, nu, kt);
        for (int j = 0; j < nx; ++j) {
            double col[MU];
            for (int i = 0; i < nu; ++i) col[i] = Qux[i * nx + j];
            chol_solve(L, nu, col);
            for (int i = 0; i < nu; ++i) Kt[i * nx + j] = col[i];
        }
        // Acl = A - B K
        for (int i = 0; i < nx; ++i)
            for (int j = 0; j < nx; ++j) {
                double s = 0;
                for (int q = 0; q < nu; ++q) s += Bt[i * nu + q] * Kt[q * nx + j];
                Acl[i * nx + j] = At[i * nx + j] - s;
            }
        // Vxx = lxx + K' luu K + Acl' Vxx' Acl
        for (int i = 0; i < nu; ++i)
            for (int j = 0; j < nx; ++j) {
                double s = 0;
                for (int q = 0; q < nu; ++q) s += luut[i * nu + q] * Kt[q * nx + j];
                LK[i * nx + j] = s;
            }
        for (int i = 0; i < nx; ++i)
            for (int j = 0; j < nx; ++j) {
                double s = 0;
                for (int q = 0; q < nx; ++q) s += Vxx[i * nx + q] * Acl[q * nx + j];
                VA[i * nx + j] = s;
            }
        for (int i = 0; i < nx; ++i)
            for (int j = 0; j < nx; ++j) {
                double a = 0, b = 0;
                for (int q = 0; q < nu; ++q) a += Kt[q * nx + i] * LK[q * nx + j];
                for (int q = 0; q < nx; ++q) b += Acl[q * nx + i] * VA[q * nx + j];
                nVxx[i * nx + j] = lxxt[i * nx + j] + a + b;
            }
        // Vx = lx - K' lu + K' luu k + Acl' (Vx' - Vxx' B k)
        for (int i = 0; i < nx; ++i) {
            double s = 0;
            for (int q = 0; q < nu; ++q) s += Bt[i * nu + q] * kt[q];
            t1[i] = s;   // B k
        }
        for (int i = 0; i < nx; ++i) {
            double s = 0;
            for (int q = 0; q < nx; ++q) s += Vxx[i * nx + q] * t1[q];
            t2[i] = Vx[i] - s;
        }
        double luk[MU];
        for (int i = 0; i < nu; ++i) {
            double s = 0;
            for (int q = 0; q < nu; ++q) s += luut[i * nu + q] * kt[q];
            luk[i] = s;
        }
        for (int i = 0; i < nx; ++i) {
            double a = 0, b = 0, c = 0;
            for (int q = 0; q < nu; ++q) {
                a += Kt[q * nx + i] * lut[q];
                b += Kt[q * nx + i] * luk[q];
            }
            for (int q = 0; q < nx; ++q) c += Acl[q * nx + i] * t2[q];
            nVx[i] = lxt[i] - a + b + c;
        }
        double d = 0;
        for (int i = 0; i < nu; ++i) d += Qu[i] * kt[i];
        acc += d;
        std::memcpy(Vx, nVx, sizeof(double) * nx);
        std::memcpy(Vxx, nVxx, sizeof(double) * nx * nx);
    }
    *dJ = acc;
    return DCOL_ALTRO_OK;
}

int dcol_altro_rollout(const dcol_altro_model* m, int64_t T, const double* X, const double* U, const double* K,
                       const double* k, double a, double* Xn, double* Un) {
    if (!model_ok(m) || T < 0 || !X || !Xn || (T > 0 && (!U || !K || !k || !Un))) return DCOL_ALTRO_ERR_ARG;
    const int nx = m->nx, nu = m->nu;
    std::memcpy(Xn, X, sizeof(double) * nx);
    double dx[MX];
    for (int64_t t = 0; t < T; ++t) {
        const double* xt = X + t * nx;
        double* xn = Xn + t * nx;
        double* un = Un + t * nu;
        for (int i = 0; i < nx; ++i) dx[i] = xn[i] - xt[i];
        for (int i = 0; i < nu; ++i) {
            double s = 0;
            for (int j = 0; j < nx; ++j) s += K[(t * nu + i) * nx + j] * dx[j];
            un[i] = U[t * nu + i] - s - a * k[t * nu + i];
        }
        rk4(*m, xn, un, xn + nx);
    }
    return DCOL_ALTRO_OK;
}

}  // extern "C"
