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
// to rounding; the Riccati sweep's matrix products (mm / mtm) use explicit fused
// multiply-adds, as the BLAS kernels behind numpy's matmul do.
#include "../../include/dcol_altro.h"
#include "altro_model.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

namespace {

using namespace dcol_altro;

// In-place lower Cholesky of the n x n SPD matrix a (row-major); false if not PD.
__attribute__((always_inline)) inline bool cholesky(double* a, int n) {
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
__attribute__((always_inline)) inline void chol_solve(const double* L, int n, double* b) {
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

// C[m x n] = A[m x p] B[p x n]; i-q-j order so the inner loop runs over contiguous
// output columns (vectorises without reassociating any sum)
__attribute__((always_inline)) inline void mm(int m, int p, int n, const double* A, const double* B, double* C) {
    for (int i = 0; i < m; ++i) {
        double* c = C + i * n;
        for (int j = 0; j < n; ++j) c[j] = 0.0;
        for (int q = 0; q < p; ++q) {
            const double a = A[i * p + q];
            const double* b = B + q * n;
            for (int j = 0; j < n; ++j) c[j] = std::fma(a, b[j], c[j]);
        }
    }
}

// C[m x n] = A' B with A [p x m], B [p x n]
__attribute__((always_inline)) inline void mtm(int p, int m, int n, const double* A, const double* B, double* C) {
    for (int i = 0; i < m * n; ++i) C[i] = 0.0;
    for (int q = 0; q < p; ++q) {
        const double* b = B + q * n;
        for (int i = 0; i < m; ++i) {
            const double a = A[q * m + i];
            double* c = C + i * n;
            for (int j = 0; j < n; ++j) c[j] = std::fma(a, b[j], c[j]);
        }
    }
}

// Riccati recursion; NX/NU > 0 fix the sizes at compile time (fully unrolled small loops
// for the three reference systems), 0 = runtime sizes.
template <int NX, int NU>
int backward_impl(int64_t T, int nx_, int nu_, const double* A, const double* B, const double* lx, const double* lu,
                  const double* lxx, const double* luu, const double* VxT, const double* VxxT, double reg, double* K,
                  double* k, double* dJ, int64_t* fail_knot) {
    const int nx = NX > 0 ? NX : nx_;
    const int nu = NU > 0 ? NU : nu_;
    // Per knot (Vx', Vxx' = next knot's cost-to-go, P = Vxx' + reg I):
    //   VB = Vxx' B, VA = Vxx' A;  Qu = lu + B'Vx';  Quu = luu + B'(VB + reg B);
    //   Qux = B'(VA + reg A);  k = Quu^-1 Qu, K = Quu^-1 Qux;  Acl = A - B K;
    //   Vxx = lxx + K' luu K + Acl' (VA - VB K);   (VA - VB K = Vxx' Acl)
    //   Vx  = lx - K' lu + K' luu k + Acl' (Vx' - VB k)
    double Vx[MX], Vxx[MX * MX], VA[MX * MX], VB[MX * MU], Qu[MU], Quu[MU * MU], Qux[MU * MX], L[MU * MU];
    double Acl[MX * MX], Wm[MX * MX], LK[MU * MX], tmp[MX * MX], v1[MX], luk[MU];
    std::memcpy(Vx, VxT, sizeof(double) * nx);
    std::memcpy(Vxx, VxxT, sizeof(double) * nx * nx);
    double acc = 0;
    for (int64_t t = T - 1; t >= 0; --t) {
        const double* At = A + t * nx * nx;
        const double* Bt = B + t * nx * nu;
        const double* luut = luu + t * nu * nu;
        double* Kt = K + t * nu * nx;
        double* kt = k + t * nu;
        mm(nx, nx, nu, Vxx, Bt, VB);
        mm(nx, nx, nx, Vxx, At, VA);
        for (int i = 0; i < nx * nu; ++i) tmp[i] = VB[i] + reg * Bt[i];
        mtm(nx, nu, nu, Bt, tmp, Quu);
        for (int i = 0; i < nu * nu; ++i) Quu[i] += luut[i];
        for (int i = 0; i < nx * nx; ++i) tmp[i] = VA[i] + reg * At[i];
        mtm(nx, nu, nx, Bt, tmp, Qux);
        mtm(nx, nu, 1, Bt, Vx, Qu);
        for (int i = 0; i < nu; ++i) Qu[i] += lu[t * nu + i];
        std::memcpy(L, Quu, sizeof(double) * nu * nu);
        if (!cholesky(L, nu)) {
            if (fail_knot) *fail_knot = t;
            return DCOL_ALTRO_ERR_NOT_PD;
        }
        for (int i = 0; i < nu; ++i) kt[i] = Qu[i];
        chol_solve(L, nu, kt);
        // K = Quu^-1 Qux: the nx right-hand sides side by side (row-major, the same
        // per-column operation order as chol_solve, vectorised over the columns)
        std::memcpy(Kt, Qux, sizeof(double) * nu * nx);
        for (int i = 0; i < nu; ++i) {
            double* ki = Kt + i * nx;
            for (int q = 0; q < i; ++q) {
                const double l = L[i * nu + q];
                const double* kq = Kt + q * nx;
                for (int j = 0; j < nx; ++j) ki[j] -= l * kq[j];
            }
            const double d = L[i * nu + i];
            for (int j = 0; j < nx; ++j) ki[j] = ki[j] / d;
        }
        for (int i = nu - 1; i >= 0; --i) {
            double* ki = Kt + i * nx;
            for (int q = i + 1; q < nu; ++q) {
                const double l = L[q * nu + i];
                const double* kq = Kt + q * nx;
                for (int j = 0; j < nx; ++j) ki[j] -= l * kq[j];
            }
            const double d = L[i * nu + i];
            for (int j = 0; j < nx; ++j) ki[j] = ki[j] / d;
        }
        mm(nx, nu, nx, Bt, Kt, tmp);                       // B K
        for (int i = 0; i < nx * nx; ++i) Acl[i] = At[i] - tmp[i];
        mm(nx, nu, nx, VB, Kt, tmp);                       // VB K
        for (int i = 0; i < nx * nx; ++i) Wm[i] = VA[i] - tmp[i];
        mm(nu, nu, nx, luut, Kt, LK);                      // luu K
        mtm(nu, nx, nx, Kt, LK, tmp);                      // K' luu K
        mtm(nx, nx, nx, Acl, Wm, Vxx);                     // Acl' Vxx' Acl
        for (int i = 0; i < nx * nx; ++i) Vxx[i] = lxx[t * nx * nx + i] + tmp[i] + Vxx[i];
        mm(nx, nu, 1, VB, kt, v1);                         // VB k
        for (int i = 0; i < nx; ++i) v1[i] = Vx[i] - v1[i];
        mm(nu, nu, 1, luut, kt, luk);
        double a[MX], b[MX], c[MX];
        mtm(nu, nx, 1, Kt, lu + t * nu, a);
        mtm(nu, nx, 1, Kt, luk, b);
        mtm(nx, nx, 1, Acl, v1, c);
        for (int i = 0; i < nx; ++i) Vx[i] = lx[t * nx + i] - a[i] + b[i] + c[i];
        double d = 0;
        for (int i = 0; i < nu; ++i) d += Qu[i] * kt[i];
        acc += d;
    }
    *dJ = acc;
    return DCOL_ALTRO_OK;
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
    if (nx == 6 && nu == 3) return backward_impl<6, 3>(T, nx, nu, A, B, lx, lu, lxx, luu, VxT, VxxT, reg, K, k, dJ, fail_knot);
    if (nx == 12 && nu == 4) return backward_impl<12, 4>(T, nx, nu, A, B, lx, lu, lxx, luu, VxT, VxxT, reg, K, k, dJ, fail_knot);
    if (nx == 12 && nu == 6) return backward_impl<12, 6>(T, nx, nu, A, B, lx, lu, lxx, luu, VxT, VxxT, reg, K, k, dJ, fail_knot);
    return backward_impl<0, 0>(T, nx, nu, A, B, lx, lu, lxx, luu, VxT, VxxT, reg, K, k, dJ, fail_knot);
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

int dcol_altro_rollouts(const dcol_altro_model* m, int64_t T, const double* X, const double* U, const double* K,
                        const double* k, const double* a, int32_t na, double* Xn, double* Un) {
    if (!model_ok(m) || T < 0 || na < 0 || (na > 0 && (!a || !X || !Xn || (T > 0 && (!U || !K || !k || !Un)))))
        return DCOL_ALTRO_ERR_ARG;
    const int64_t sx = (T + 1) * m->nx, su = T * m->nu;
    int rc = DCOL_ALTRO_OK;
#pragma omp parallel for schedule(static) if (na > 1) reduction(min : rc)
    for (int32_t j = 0; j < na; ++j) rc = std::min(rc, dcol_altro_rollout(m, T, X, U, K, k, a[j], Xn + j * sx, Un + j * su));
    return rc;
}

}  // extern "C"

// ---------------------------------------------------------------- AL objective pieces
namespace {

bool problem_ok(const dcol_altro_problem* p) {
    return p && p->N >= 2 && p->nx > 0 && p->nx <= MX && p->nu > 0 && p->nu <= MU && p->ncx >= 0 && p->Q && p->R &&
           p->Qf && p->Xref && p->Uref && p->u_min && p->u_max;
}

// x' M x for a row-major n x n M
inline double quad(const double* M, const double* x, int n) {
    double acc = 0.0;
    for (int i = 0; i < n; ++i) {
        double r = 0.0;
        for (int j = 0; j < n; ++j) r += M[i * n + j] * x[j];
        acc += x[i] * r;
    }
    return acc;
}

// AL term of one constraint block: dual . h + rho/2 sum_{active} h^2, active = dual > 0 or h > 0
inline double al_term(const double* dual, const double* h, int n, double rho) {
    double d = 0.0, q = 0.0;
    for (int i = 0; i < n; ++i) {
        d += dual[i] * h[i];
        if (dual[i] > 0 || h[i] > 0) q += h[i] * h[i];
    }
    return d + 0.5 * rho * q;
}

inline void control_h(const dcol_altro_problem* p, const double* u, double* h) {
    for (int i = 0; i < p->nu; ++i) {
        h[i] = u[i] - p->u_max[i];
        h[p->nu + i] = -u[i] + p->u_min[i];
    }
}

}  // namespace

extern "C" {

int dcol_altro_cost(const dcol_altro_problem* p, const double* X, const double* U, const double* hx, const double* mu,
                    const double* mux, const double* lam, double rho, double* J) {
    if (!problem_ok(p) || !X || !U || !mu || !mux || !lam || !J || (p->ncx > 0 && !hx)) return DCOL_ALTRO_ERR_ARG;
    const int N = p->N, nx = p->nx, nu = p->nu, nc = p->ncx;
    double cost = 0.0, dx[MX], du[MU], hu[2 * MU];
    for (int t = 0; t < N - 1; ++t) {
        for (int i = 0; i < nx; ++i) dx[i] = X[t * nx + i] - p->Xref[t * nx + i];
        for (int i = 0; i < nu; ++i) du[i] = U[t * nu + i] - p->Uref[t * nu + i];
        cost += 0.5 * quad(p->Q, dx, nx) + 0.5 * quad(p->R, du, nu);
        control_h(p, U + t * nu, hu);
        cost += al_term(mu + t * 2 * nu, hu, 2 * nu, rho);
        cost += al_term(mux + t * nc, hx + t * nc, nc, rho);
    }
    const double* xN = X + (N - 1) * nx;
    const double* rN = p->Xref + (N - 1) * nx;
    for (int i = 0; i < nx; ++i) dx[i] = xN[i] - rN[i];
    cost += 0.5 * quad(p->Qf, dx, nx);
    cost += al_term(mux + (N - 1) * nc, hx + (N - 1) * nc, nc, rho);
    double lg = 0.0, gg = 0.0;
    for (int i = 0; i < nx; ++i) {
        lg += lam[i] * dx[i];
        gg += dx[i] * dx[i];
    }
    cost += lg + 0.5 * rho * gg;
    *J = cost;
    return DCOL_ALTRO_OK;
}

int dcol_altro_stage_terms(const dcol_altro_problem* p, const double* X, const double* U, const double* hx,
                           const double* Gx, const double* mu, const double* mux, const double* lam, double rho,
                           double* lx, double* lu, double* lxx, double* luu, double* VxT, double* VxxT) {
    if (!problem_ok(p) || !X || !U || !mu || !mux || !lam || !lx || !lu || !lxx || !luu || !VxT || !VxxT ||
        (p->ncx > 0 && (!hx || !Gx)))
        return DCOL_ALTRO_ERR_ARG;
    const int N = p->N, nx = p->nx, nu = p->nu, nc = p->ncx;
    double hu[2 * MU], w[64], mk[64];
    if (nc > 64) return DCOL_ALTRO_ERR_ARG;
    // collision terms of knot t into (gx, gxx): gx += Gx' (mux + rho m h), gxx += rho Gx' diag(m) Gx
    auto collision = [&](int t, double* gx, double* gxx) {
        const double* h = hx + t * nc;
        const double* d = mux + t * nc;
        const double* G = Gx + (int64_t)t * nc * nx;
        for (int c = 0; c < nc; ++c) {
            mk[c] = (d[c] > 0 || h[c] > 0) ? 1.0 : 0.0;
            w[c] = d[c] + rho * (mk[c] * h[c]);
        }
        for (int c = 0; c < nc; ++c) {
            const double* g = G + c * nx;
            for (int i = 0; i < nx; ++i) gx[i] += g[i] * w[c];
            if (mk[c] != 0.0) {
                const double rm = rho * mk[c];
                for (int i = 0; i < nx; ++i) {
                    const double gi = rm * g[i];
                    for (int j = 0; j < nx; ++j) gxx[i * nx + j] += gi * g[j];
                }
            }
        }
    };
    for (int t = 0; t < N - 1; ++t) {
        double* lxt = lx + t * nx;
        double* lut = lu + t * nu;
        double* lxxt = lxx + (int64_t)t * nx * nx;
        double* luut = luu + (int64_t)t * nu * nu;
        for (int i = 0; i < nx; ++i) {
            double r = 0.0;
            for (int j = 0; j < nx; ++j) r += p->Q[i * nx + j] * (X[t * nx + j] - p->Xref[t * nx + j]);
            lxt[i] = r;
        }
        for (int i = 0; i < nx * nx; ++i) lxxt[i] = p->Q[i];
        collision(t, lxt, lxxt);
        for (int i = 0; i < nu; ++i) {
            double r = 0.0;
            for (int j = 0; j < nu; ++j) r += p->R[i * nu + j] * (U[t * nu + j] - p->Uref[t * nu + j]);
            lut[i] = r;
        }
        for (int i = 0; i < nu * nu; ++i) luut[i] = p->R[i];
        control_h(p, U + t * nu, hu);
        const double* mt = mu + t * 2 * nu;
        for (int i = 0; i < nu; ++i) {                  // Gu = [I; -I]
            const double m1 = (mt[i] > 0 || hu[i] > 0) ? 1.0 : 0.0;
            const double m2 = (mt[nu + i] > 0 || hu[nu + i] > 0) ? 1.0 : 0.0;
            lut[i] += (mt[i] + rho * (m1 * hu[i])) - (mt[nu + i] + rho * (m2 * hu[nu + i]));
            luut[i * nu + i] += rho * (m1 + m2);
        }
    }
    const int T = N - 1;
    const double* xN = X + T * nx;
    const double* rN = p->Xref + T * nx;
    for (int i = 0; i < nx; ++i) {
        double r = 0.0;
        for (int j = 0; j < nx; ++j) r += p->Qf[i * nx + j] * (xN[j] - rN[j]);
        VxT[i] = r;
    }
    for (int i = 0; i < nx * nx; ++i) VxxT[i] = p->Qf[i];
    collision(T, VxT, VxxT);
    for (int i = 0; i < nx; ++i) {
        VxT[i] += lam[i] + rho * (xN[i] - rN[i]);
        VxxT[i * nx + i] += rho;
    }
    return DCOL_ALTRO_OK;
}

int dcol_altro_victim_poses(const dcol_altro_model* m, int64_t N, const double* X, double* poses) {
    if (!model_ok(m) || N < 0 || (N > 0 && (!X || !poses))) return DCOL_ALTRO_ERR_ARG;
    const int nx = m->nx;
    for (int64_t t = 0; t < N; ++t) {
        const double* x = X + t * nx;
        double* q = poses + 6 * t;
        if (m->system == DCOL_SYS_PIANO) {      // r = (x0, x1, 0), p = (0, 0, 1) tan(theta / 4)
            const double tq = std::tan(x[4] / 4);
            q[0] = x[0]; q[1] = x[1]; q[2] = 0.0;
            q[3] = 0.0 * tq; q[4] = 0.0 * tq; q[5] = tq;
        } else {                                // r = x[0:3], p = x[6:9]
            for (int i = 0; i < 3; ++i) {
                q[i] = x[i];
                q[3 + i] = x[6 + i];
            }
        }
    }
    return DCOL_ALTRO_OK;
}

namespace {
// element (pair i = t ncx + k, component c) of dalpha at dalpha[i s_pair + c s_comp]
int constraint_jacobian_strided(const dcol_altro_model* m, int64_t N, int32_t ncx, const double* X,
                                const double* dalpha, int64_t s_pair, int64_t s_comp, double* Gx) {
    const int nx = m->nx;
    for (int64_t t = 0; t < N; ++t) {
        const double* x = X + t * nx;
        double c = 0.0;
        if (m->system == DCOL_SYS_PIANO) {      // dp/dtheta = (0, 0, 1) / (4 cos^2(theta / 4))
            const double cs = std::cos(x[4] / 4);
            c = 1 / (4 * (cs * cs));
        }
        for (int k = 0; k < ncx; ++k) {
            const double* Jp = dalpha + (t * ncx + k) * s_pair;
            double J[6];   // d alpha / d (r1, p1): the victim's pose
            for (int i = 0; i < 6; ++i) J[i] = Jp[i * s_comp];
            double* g = Gx + (t * ncx + k) * nx;
            for (int i = 0; i < nx; ++i) g[i] = 0.0;
            if (m->system == DCOL_SYS_PIANO) {
                g[0] = -J[0];
                g[1] = -J[1];
                g[4] = -(J[3] * 0.0 + J[4] * 0.0 + J[5] * c);
            } else {
                for (int i = 0; i < 3; ++i) {
                    g[i] = -J[i];
                    g[6 + i] = -J[3 + i];
                }
            }
        }
    }
    return DCOL_ALTRO_OK;
}
}  // namespace

extern "C" int dcol_altro_constraint_jacobian(const dcol_altro_model* m, int64_t N, int32_t ncx, const double* X,
                                              const double* dalpha, double* Gx) {
    if (!model_ok(m) || N < 0 || ncx < 0 || (N > 0 && ncx > 0 && (!X || !dalpha || !Gx))) return DCOL_ALTRO_ERR_ARG;
    return constraint_jacobian_strided(m, N, ncx, X, dalpha, 12, 1, Gx);
}

// ---------------------------------------------------------------- fused driver steps
// One call per optimizer phase instead of one per piece (the per-call cost of the Python
// binding exceeded the work of the small pieces); each equals the calls it replaces.
int dcol_altro_backward_pass(const dcol_altro_model* m, const dcol_altro_problem* p, const double* X,
                             const double* U, const double* alpha, const double* dalpha, int64_t dalpha_comp_stride,
                             const double* A, const double* B, const double* mu, const double* mux, const double* lam,
                             double rho, double reg, double* K, double* k, double* dJ, double* J, int64_t* fail_knot) {
    if (!model_ok(m) || !problem_ok(p) || m->nx != p->nx || m->nu != p->nu || !X || !U || !A || !B || !K || !k ||
        !dJ || !J || (p->ncx > 0 && (!alpha || !dalpha)) || dalpha_comp_stride < 0)
        return DCOL_ALTRO_ERR_ARG;
    const int N = p->N, nx = p->nx, nu = p->nu, nc = p->ncx;
    thread_local std::vector<double> ws;
    const size_t need = (size_t)N * nc * (1 + nx) + (size_t)(N - 1) * (nx + nu + nx * nx + nu * nu) + nx + nx * nx;
    if (ws.size() < need) ws.resize(need);
    double* hx = ws.data();
    double* Gx = hx + (size_t)N * nc;
    double* lx = Gx + (size_t)N * nc * nx;
    double* lu = lx + (size_t)(N - 1) * nx;
    double* lxx = lu + (size_t)(N - 1) * nu;
    double* luu = lxx + (size_t)(N - 1) * nx * nx;
    double* VxT = luu + (size_t)(N - 1) * nu * nu;
    double* VxxT = VxT + nx;
    for (size_t i = 0; i < (size_t)N * nc; ++i) hx[i] = 1 - alpha[i];
    int rc = dalpha_comp_stride ? constraint_jacobian_strided(m, N, nc, X, dalpha, 1, dalpha_comp_stride, Gx)
                                : constraint_jacobian_strided(m, N, nc, X, dalpha, 12, 1, Gx);
    if (rc == DCOL_ALTRO_OK) rc = dcol_altro_stage_terms(p, X, U, hx, Gx, mu, mux, lam, rho, lx, lu, lxx, luu, VxT, VxxT);
    if (rc == DCOL_ALTRO_OK)
        rc = dcol_altro_backward(N - 1, nx, nu, A, B, lx, lu, lxx, luu, VxT, VxxT, reg, K, k, dJ, fail_knot);
    if (rc == DCOL_ALTRO_OK) rc = dcol_altro_cost(p, X, U, hx, mu, mux, lam, rho, J);
    return rc;
}

int dcol_altro_trial(const dcol_altro_model* m, int64_t T, const double* X, const double* U, const double* K,
                     const double* k, double a, double* Xn, double* Un, double* poses) {
    int rc = dcol_altro_rollout(m, T, X, U, K, k, a, Xn, Un);
    if (rc == DCOL_ALTRO_OK) rc = dcol_altro_victim_poses(m, T + 1, Xn, poses);
    return rc;
}

}  // extern "C"
