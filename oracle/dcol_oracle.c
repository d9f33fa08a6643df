/*
 * dcol_oracle.c -- plain-C restatement of the reference DCOL proximity path.
 * TEST INFRASTRUCTURE ONLY: used by tests/ (full-size parity checks on the GPU box) and by
 * bench.py's cpu_baseline leg.  Never linked into, or called by, the product library.
 *
 * Follows the reference op-for-op in reference row order, like oracle/dcol_oracle.py:
 *   dcm_from_mrp ............. primitives/problem_matrices.py:213-251
 *   primitive blocks ......... primitives/problem_matrices.py:4-209 (dispatch :255-364)
 *   combine .................. primitives/combine_problem_matrices.py:3-70 (case 4 -> status 2)
 *   initialize ............... proximity/pdip.py:291-332 (quirks Q1, Q2)
 *   solve_lp_pdip ............ proximity/pdip.py:373-470 (50-iteration cap, mu-only exit)
 *   NT scaling ............... proximity/NT/NT_scaling.py:340-463 (SOC W solved by Cholesky
 *                              of W, as cho_factor/cho_solve do)
 *   FD gradient .............. proximity/proximity_gradient.py:8-138 + scipy approx_fprime
 * Parity: pinned against the reference's golden vectors (tests/test_c_oracle.py).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#define MMAX 136   /* 128 orthant rows (the engine's pair capacity) + two 4-row SOC blocks */
#define FMAX 128   /* faces / edges per primitive */
#define NMAX 8

enum { POLYTOPE = 0, SPHERE = 1, CONE = 2, CAPSULE = 3, CYLINDER = 4, POLYGON = 5 };
enum { ST_OK = 0, ST_MAXITER = 1, ST_UNSUPPORTED = 2, ST_NOT_PD = 3, ST_NONFINITE = 4, ST_TOO_LARGE = 5 };

typedef struct {
    int type, nh;
    const double *A, *b;   /* A rows of 3 doubles in the pool (polygon uses the first 2) */
    double R, L, H, beta;
    double roff[3], Qoff[9];
} Shape;

typedef struct {           /* one primitive's conic blocks */
    int no, ns, nc;        /* orthant rows, SOC rows, columns */
    double Go[FMAX][NMAX], ho[FMAX];
    double Gs[4][NMAX], hs[4];
} Blocks;

typedef struct {           /* the combined problem */
    int m, n, no, n1, n2;
    double G[MMAX][NMAX], h[MMAX], c[NMAX];
} Prob;

static void dcm_from_mrp(const double p[3], double Q[9]) {
    const double p1 = p[0], p2 = p[1], p3 = p[2];
    const double s = p1 * p1 + p2 * p2 + p3 * p3 + 1;
    const double den = s * s;
    const double a = (4 * (p1 * p1) + 4 * (p2 * p2) + 4 * (p3 * p3) - 4);
    Q[0] = -((8 * (p2 * p2) + 8 * (p3 * p3)) / den - 1) * den / den;
    Q[1] = (8 * p1 * p2 + p3 * a) / den;
    Q[2] = (8 * p1 * p3 - p2 * a) / den;
    Q[3] = (8 * p1 * p2 - p3 * a) / den;
    Q[4] = -((8 * (p1 * p1) + 8 * (p3 * p3)) / den - 1) * den / den;
    Q[5] = (8 * p2 * p3 + p1 * a) / den;
    Q[6] = (8 * p1 * p3 + p2 * a) / den;
    Q[7] = (8 * p2 * p3 - p1 * a) / den;
    Q[8] = -((8 * (p1 * p1) + 8 * (p2 * p2)) / den - 1) * den / den;
}

static void mat3(const double* A, const double* B, double* C) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

/* problem_matrices(shape, r, p) */
static int blocks(const Shape* sh, const double r[3], const double p[3], Blocks* b) {
    double Q[9], Qe[9], re[3];
    dcm_from_mrp(p, Q);
    for (int k = 0; k < 3; ++k) re[k] = r[k] + (Q[3 * k] * sh->roff[0] + Q[3 * k + 1] * sh->roff[1] + Q[3 * k + 2] * sh->roff[2]);
    mat3(Q, sh->Qoff, Qe);
    memset(b, 0, sizeof(*b));
    switch (sh->type) {
        case POLYTOPE:
            if (sh->nh > FMAX) return -1;
            b->no = sh->nh; b->ns = 0; b->nc = 4;
            for (int j = 0; j < sh->nh; ++j) {
                const double* a = sh->A + 3 * j;
                double u[3];
                for (int l = 0; l < 3; ++l) u[l] = a[0] * Qe[3 * l] + a[1] * Qe[3 * l + 1] + a[2] * Qe[3 * l + 2];
                b->Go[j][0] = u[0]; b->Go[j][1] = u[1]; b->Go[j][2] = u[2]; b->Go[j][3] = -sh->b[j];
                b->ho[j] = u[0] * re[0] + u[1] * re[1] + u[2] * re[2];
            }
            return 0;
        case SPHERE:
            b->no = 0; b->ns = 4; b->nc = 4;
            b->Gs[0][3] = -sh->R;
            for (int k = 0; k < 3; ++k) { b->Gs[k + 1][k] = -1; b->hs[k + 1] = -re[k]; }
            return 0;
        case CONE: {
            const double tb = tan(sh->beta);
            b->no = 1; b->ns = 3; b->nc = 4;
            b->Go[0][0] = Qe[0]; b->Go[0][1] = Qe[3]; b->Go[0][2] = Qe[6]; b->Go[0][3] = -sh->H / 4;
            b->ho[0] = Qe[0] * re[0] + Qe[3] * re[1] + Qe[6] * re[2];
            for (int k = 0; k < 3; ++k) {
                const double e = k == 0 ? tb : 1.0;
                double u[3];
                for (int l = 0; l < 3; ++l) u[l] = -(e * Qe[3 * l + k]);
                b->Gs[k][0] = u[0]; b->Gs[k][1] = u[1]; b->Gs[k][2] = u[2];
                b->Gs[k][3] = k == 0 ? -(tb * 3 * sh->H / 4) : 0.0;
                b->hs[k] = u[0] * re[0] + u[1] * re[1] + u[2] * re[2];
            }
            return 0;
        }
        case CAPSULE:
        case CYLINDER: {
            const double bx[3] = {Qe[0], Qe[3], Qe[6]};
            b->ns = 4; b->nc = 5;
            b->Gs[0][3] = -sh->R;
            for (int k = 0; k < 3; ++k) { b->Gs[k + 1][k] = -1; b->Gs[k + 1][4] = bx[k]; b->hs[k + 1] = -re[k]; }
            b->Go[0][3] = -sh->L / 2; b->Go[0][4] = 1;
            b->Go[1][3] = -sh->L / 2; b->Go[1][4] = -1;
            b->no = 2;
            if (sh->type == CYLINDER) {
                const double d = bx[0] * re[0] + bx[1] * re[1] + bx[2] * re[2];
                for (int l = 0; l < 3; ++l) { b->Go[2][l] = -bx[l]; b->Go[3][l] = bx[l]; }
                b->Go[2][3] = -sh->L / 2; b->Go[3][3] = -sh->L / 2;
                b->ho[2] = -d; b->ho[3] = d;
                b->no = 4;
            }
            return 0;
        }
        case POLYGON:
            if (sh->nh > FMAX) return -1;
            b->no = sh->nh; b->ns = 4; b->nc = 6;
            for (int j = 0; j < sh->nh; ++j) {
                b->Go[j][3] = -sh->b[j];
                b->Go[j][4] = sh->A[3 * j];
                b->Go[j][5] = sh->A[3 * j + 1];
            }
            b->Gs[0][3] = -sh->R;
            for (int k = 0; k < 3; ++k) {
                b->Gs[k + 1][k] = -1; b->Gs[k + 1][4] = Qe[3 * k]; b->Gs[k + 1][5] = Qe[3 * k + 1];
                b->hs[k + 1] = -re[k];
            }
            return 0;
    }
    return -1;
}

/* combine_problem_matrices: rows [ort1; ort2; soc1; soc2], narrower side zero-padded */
static int combine(const Blocks* a, const Blocks* b, Prob* P) {
    if (a->nc > 4 && b->nc > 4) return ST_UNSUPPORTED;   /* case 4 */
    const int n = a->nc > b->nc ? a->nc : b->nc;
    const int m = a->no + b->no + a->ns + b->ns;
    if (m > MMAX) return ST_TOO_LARGE;
    memset(P, 0, sizeof(*P));
    P->n = n; P->m = m; P->no = a->no + b->no; P->n1 = a->ns; P->n2 = b->ns;
    P->c[3] = 1.0;
    int row = 0;
    for (int i = 0; i < a->no; ++i, ++row) { memcpy(P->G[row], a->Go[i], sizeof(double) * a->nc); P->h[row] = a->ho[i]; }
    for (int i = 0; i < b->no; ++i, ++row) { memcpy(P->G[row], b->Go[i], sizeof(double) * b->nc); P->h[row] = b->ho[i]; }
    for (int i = 0; i < a->ns; ++i, ++row) { memcpy(P->G[row], a->Gs[i], sizeof(double) * a->nc); P->h[row] = a->hs[i]; }
    for (int i = 0; i < b->ns; ++i, ++row) { memcpy(P->G[row], b->Gs[i], sizeof(double) * b->nc); P->h[row] = b->hs[i]; }
    return ST_OK;
}

/* ------------------------------------------------------------------ small dense algebra */
/* lower Cholesky A = L L' (LAPACK dpotrf semantics: fail on a pivot <= 0 or NaN) */
static int chol_lower(int n, const double A[NMAX][NMAX], double L[NMAX][NMAX]) {
    memset(L, 0, sizeof(double) * NMAX * NMAX);
    for (int j = 0; j < n; ++j) {
        double d = A[j][j];
        for (int k = 0; k < j; ++k) d -= L[j][k] * L[j][k];
        if (!(d > 0)) return 0;
        L[j][j] = sqrt(d);
        for (int i = j + 1; i < n; ++i) {
            double t = A[i][j];
            for (int k = 0; k < j; ++k) t -= L[i][k] * L[j][k];
            L[i][j] = t / L[j][j];
        }
    }
    return 1;
}
static void fwd(int n, const double L[NMAX][NMAX], const double* b, double* y) {   /* L y = b */
    for (int i = 0; i < n; ++i) {
        double t = b[i];
        for (int k = 0; k < i; ++k) t -= L[i][k] * y[k];
        y[i] = t / L[i][i];
    }
}
static void bwd(int n, const double L[NMAX][NMAX], const double* y, double* x) {   /* L' x = y */
    for (int i = n - 1; i >= 0; --i) {
        double t = y[i];
        for (int k = i + 1; k < n; ++k) t -= L[k][i] * x[k];
        x[i] = t / L[i][i];
    }
}

/* ------------------------------------------------------------------ cones */
typedef struct {
    int no, n1, n2, m, deg;
    double ort[MMAX];                /* orthant NT scaling */
    double W1[4][4], W2[4][4];       /* SOC NT scalings */
    double L1[NMAX][NMAX], L2[NMAX][NMAX];   /* their Cholesky factors */
} NT;

static double socJ(const double* v, int q) {
    double t = 0;
    for (int k = 1; k < q; ++k) t += v[k] * v[k];
    return v[0] * v[0] - t;
}

static int soc_nt(const double* s, const double* z, int q, double W[4][4], double L[NMAX][NMAX]) {
    double zb[4], sb[4];
    const double jz = sqrt(socJ(z, q)), js = sqrt(socJ(s, q));
    for (int k = 0; k < q; ++k) { zb[k] = z[k] / jz; sb[k] = s[k] / js; }
    double dot = 0;
    for (int k = 0; k < q; ++k) dot += zb[k] * sb[k];
    const double g = sqrt((1.0 + dot) / 2.0);
    double w[4];
    w[0] = (sb[0] + zb[0]) / (2 * g);
    for (int k = 1; k < q; ++k) w[k] = (sb[k] - zb[k]) / (2 * g);
    const double bb = 1.0 / (w[0] + 1.0);
    const double Jz = socJ(z, q);
    const double eta = Jz != 0 ? pow(socJ(s, q) / Jz, 0.25) : 1.0;
    double A[NMAX][NMAX];
    for (int i = 0; i < q; ++i)
        for (int j = 0; j < q; ++j) {
            double v;
            if (i == 0) v = w[j];
            else if (j == 0) v = w[i];
            else v = (i == j ? 1.0 : 0.0) + bb * w[i] * w[j];
            W[i][j] = eta * v;
            A[i][j] = W[i][j];
        }
    for (int i = 0; i < q * q; ++i)
        if (!isfinite(W[i / q][i % q])) return ST_NONFINITE;   /* cho_factor check_finite */
    if (!chol_lower(q, (const double(*)[NMAX])A, L)) return ST_NOT_PD;
    return ST_OK;
}

static int nt_init(NT* W, const double* s, const double* z) {
    for (int i = 0; i < W->no; ++i) W->ort[i] = sqrt(s[i] / z[i]);
    int st = ST_OK;
    if (W->n1) st = soc_nt(s + W->no, z + W->no, W->n1, W->W1, W->L1);
    if (st == ST_OK && W->n2) st = soc_nt(s + W->no + W->n1, z + W->no + W->n1, W->n2, W->W2, W->L2);
    return st;
}
static void nt_mul(const NT* W, const double* g, double* out) {
    for (int i = 0; i < W->no; ++i) out[i] = g[i] * W->ort[i];
    for (int blk = 0; blk < 2; ++blk) {
        const int q = blk ? W->n2 : W->n1, o = W->no + (blk ? W->n1 : 0);
        for (int i = 0; i < q; ++i) {
            double t = 0;
            for (int j = 0; j < q; ++j) t += (blk ? W->W2 : W->W1)[i][j] * g[o + j];
            out[o + i] = t;
        }
    }
}
static void nt_solve(const NT* W, const double* g, double* out) {
    for (int i = 0; i < W->no; ++i) out[i] = g[i] / W->ort[i];
    for (int blk = 0; blk < 2; ++blk) {
        const int q = blk ? W->n2 : W->n1, o = W->no + (blk ? W->n1 : 0);
        if (!q) continue;
        double y[NMAX];
        fwd(q, blk ? W->L2 : W->L1, g + o, y);
        bwd(q, blk ? W->L2 : W->L1, y, out + o);
    }
}
static void cone_prod(const NT* W, const double* u, const double* v, double* out) {
    for (int i = 0; i < W->no; ++i) out[i] = u[i] * v[i];
    for (int blk = 0; blk < 2; ++blk) {
        const int q = blk ? W->n2 : W->n1, o = W->no + (blk ? W->n1 : 0);
        if (!q) continue;
        double d = 0;
        for (int k = 0; k < q; ++k) d += u[o + k] * v[o + k];
        for (int k = 1; k < q; ++k) out[o + k] = u[o] * v[o + k] + v[o] * u[o + k];
        out[o] = d;
    }
}
static void inv_cone_prod(const NT* W, const double* u, const double* w, double* out) {
    for (int i = 0; i < W->no; ++i) out[i] = w[i] / u[i];
    for (int blk = 0; blk < 2; ++blk) {
        const int q = blk ? W->n2 : W->n1, o = W->no + (blk ? W->n1 : 0);
        if (!q) continue;
        double rho = u[o] * u[o], nu = 0, t = 0;
        for (int k = 1; k < q; ++k) { t += u[o + k] * u[o + k]; nu += u[o + k] * w[o + k]; }
        rho -= t;
        const double c1 = nu / u[o] - w[o], c2 = rho / u[o];
        out[o] = (1.0 / rho) * (u[o] * w[o] - nu);
        for (int k = 1; k < q; ++k) out[o + k] = (1.0 / rho) * (c1 * u[o + k] + c2 * w[o + k]);
    }
}
static double ls_soc(const double* y, const double* d, int q) {
    double yy = 0, yd = 0;
    for (int k = 1; k < q; ++k) { yy += y[k] * y[k]; yd += y[k] * d[k]; }
    double nu = y[0] * y[0] - yy;
    if (nu < 1e-25) nu = 1e-25;
    const double zeta = y[0] * d[0] - yd;
    const double sn = sqrt(nu);
    const double rho0 = zeta / nu;
    const double coef = (zeta / sn + d[0]) / (y[0] / sn + 1);
    double n2 = 0;
    for (int k = 1; k < q; ++k) {
        const double r = d[k] / sn - coef * (y[k] / nu);
        n2 += r * r;
    }
    const double n1 = sqrt(n2);
    if (n1 > rho0) { const double a = 1 / (n1 - rho0); return a < 1.0 ? a : 1.0; }
    return 1.0;
}
static double linesearch(const NT* W, const double* x, const double* dx) {
    double a = 1.0;
    for (int i = 0; i < W->no; ++i)
        if (dx[i] < 0) { const double t = -x[i] / dx[i]; if (t < a) a = t; }
    if (W->n1) { const double t = ls_soc(x + W->no, dx + W->no, W->n1); if (t < a) a = t; }
    if (W->n2) { const double t = ls_soc(x + W->no + W->n1, dx + W->no + W->n1, W->n2); if (t < a) a = t; }
    return a;
}
static void bring2cone(const NT* W, double* r) {
    double a = -1;
    int any = 0;
    double mn = INFINITY;
    for (int i = 0; i < W->no; ++i) { if (r[i] <= 0) any = 1; if (r[i] < mn) mn = r[i]; }
    if (any) a = -mn;
    for (int blk = 0; blk < 2; ++blk) {
        const int q = blk ? W->n2 : W->n1, o = W->no + (blk ? W->n1 : 0);
        if (!q) continue;
        double t = 0;
        for (int k = 1; k < q; ++k) t += r[o + k] * r[o + k];
        const double res = r[o] - sqrt(t);
        if (res <= 0 && -res > a) a = -res;
    }
    if (a < 0) return;
    for (int i = 0; i < W->no; ++i) r[i] += 1 + a;
    if (W->n1) r[W->no] += 1 + a;
    if (W->n2) r[W->no + W->n1] += 1 + a;
}

/* solve_lp_pdip; returns status, *iters = Newton steps */
static int pdip(const Prob* P, double tol, double* x, double* s, double* z, int* iters) {
    const int m = P->m, n = P->n;
    NT W;
    memset(&W, 0, sizeof(W));
    W.no = P->no; W.n1 = P->n1; W.n2 = P->n2; W.m = m;
    W.deg = P->no + (P->n1 > 0) + (P->n2 > 0);
    double e[MMAX] = {0};
    for (int i = 0; i < P->no; ++i) e[i] = 1;
    if (P->n1) e[P->no] = 1;
    if (P->n2) e[P->no + P->n1] = 1;
    /* initialize */
    double A[NMAX][NMAX], L[NMAX][NMAX], gth[NMAX] = {0}, y[NMAX];
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double t = 0;
            for (int k = 0; k < m; ++k) t += P->G[k][i] * P->G[k][j];
            A[i][j] = t;
        }
    if (!chol_lower(n, (const double(*)[NMAX])A, L)) return ST_NOT_PD;
    for (int j = 0; j < n; ++j)
        for (int k = 0; k < m; ++k) gth[j] += P->G[k][j] * P->h[k];
    fwd(n, L, gth, y);
    bwd(n, L, y, x);
    for (int k = 0; k < m; ++k) {
        double t = 0;
        for (int j = 0; j < n; ++j) t += P->G[k][j] * x[j];
        s[k] = t - P->h[k];
    }
    bring2cone(&W, s);
    double yx[NMAX] = {0}, xz[NMAX];
    for (int j = 0; j < n; ++j) yx[j] = -P->c[j] / L[j][j];   /* quirk Q1 */
    bwd(n, L, yx, xz);
    for (int k = 0; k < m; ++k) {
        double t = 0;
        for (int j = 0; j < n; ++j) t += P->G[k][j] * xz[j];
        z[k] = t;
    }
    bring2cone(&W, z);
    for (int it = 0; it < 50; ++it) {
        int st = nt_init(&W, s, z);
        if (st != ST_OK) { *iters = it; return st; }
        double lam[MMAX], ll[MMAX], rx[NMAX], rz[MMAX], mu = 0;
        nt_mul(&W, z, lam);
        cone_prod(&W, lam, lam, ll);
        for (int j = 0; j < n; ++j) {
            double t = 0;
            for (int k = 0; k < m; ++k) t += P->G[k][j] * z[k];
            rx[j] = t + P->c[j];
        }
        for (int k = 0; k < m; ++k) {
            double t = 0;
            for (int j = 0; j < n; ++j) t += P->G[k][j] * x[j];
            rz[k] = s[k] + t - P->h[k];
        }
        for (int k = 0; k < m; ++k) mu += s[k] * z[k];
        const double sz = mu;
        mu /= W.deg;
        if (mu < tol) { *iters = it; return ST_OK; }
        double Gt[MMAX][NMAX], col[MMAX], res[MMAX], Hm[NMAX][NMAX], F[NMAX][NMAX];
        for (int j = 0; j < n; ++j) {
            for (int k = 0; k < m; ++k) col[k] = P->G[k][j];
            nt_solve(&W, col, res);
            for (int k = 0; k < m; ++k) Gt[k][j] = res[k];
        }
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) {
                double t = 0;
                for (int k = 0; k < m; ++k) t += Gt[k][i] * Gt[k][j];
                Hm[i][j] = t;
                if (!isfinite(t)) { *iters = it; return ST_NONFINITE; }
            }
        if (!chol_lower(n, (const double(*)[NMAX])Hm, F)) { *iters = it; return ST_NOT_PD; }
        double lds[MMAX], tmp[MMAX], bzt[MMAX], rhs[NMAX], dxv[NMAX], dz[MMAX], ds[MMAX], v[MMAX];
        for (int pass = 0; pass < 2; ++pass) {
            double alpha_pass;
            if (pass == 0) {
                for (int k = 0; k < m; ++k) tmp[k] = -ll[k];
                inv_cone_prod(&W, lam, tmp, lds);
            }
            nt_mul(&W, lds, tmp);
            for (int k = 0; k < m; ++k) tmp[k] = -rz[k] - tmp[k];
            nt_solve(&W, tmp, bzt);
            for (int j = 0; j < n; ++j) {
                double t = 0;
                for (int k = 0; k < m; ++k) t += Gt[k][j] * bzt[k];
                rhs[j] = -rx[j] + t;
            }
            double yy[NMAX];
            fwd(n, F, rhs, yy);
            bwd(n, F, yy, dxv);
            for (int k = 0; k < m; ++k) {
                double t = 0;
                for (int j = 0; j < n; ++j) t += Gt[k][j] * dxv[j];
                v[k] = t - bzt[k];
            }
            nt_solve(&W, v, dz);
            nt_mul(&W, dz, tmp);
            for (int k = 0; k < m; ++k) tmp[k] = lds[k] - tmp[k];
            nt_mul(&W, tmp, ds);
            const double ls1 = linesearch(&W, s, ds), ls2 = linesearch(&W, z, dz);
            const double mn = ls1 < ls2 ? ls1 : ls2;
            if (pass == 0) {
                alpha_pass = mn;
                double rho = 0;
                for (int k = 0; k < m; ++k) rho += (s[k] + alpha_pass * ds[k]) * (z[k] + alpha_pass * dz[k]);
                rho /= sz;
                double sig = rho < 0 ? 0 : (rho > 1 ? 1 : rho);
                sig = sig * sig * sig;
                double t1[MMAX], t2[MMAX], cp[MMAX];
                nt_solve(&W, ds, t1);
                nt_mul(&W, dz, t2);
                cone_prod(&W, t1, t2, cp);
                for (int k = 0; k < m; ++k) tmp[k] = -ll[k] - cp[k] + sig * mu * e[k];
                inv_cone_prod(&W, lam, tmp, lds);
            } else {
                alpha_pass = 0.99 * mn;
                if (alpha_pass > 1) alpha_pass = 1;
                for (int j = 0; j < n; ++j) x[j] += alpha_pass * dxv[j];
                for (int k = 0; k < m; ++k) { s[k] += alpha_pass * ds[k]; z[k] += alpha_pass * dz[k]; }
            }
        }
    }
    *iters = 50;
    return ST_MAXITER;
}

static int assemble(const Shape* a, const double* th1, const Shape* b, const double* th2, Prob* P) {
    Blocks B1, B2;
    if (blocks(a, th1, th1 + 3, &B1) || blocks(b, th2, th2 + 3, &B2)) return ST_TOO_LARGE;
    return combine(&B1, &B2, P);
}

static double lag_con(const Shape* a, const Shape* b, const double* x, const double* z, const double* th) {
    Prob P;
    assemble(a, th, b, th + 6, &P);
    double f = 0;
    for (int k = 0; k < P.m; ++k) {
        double t = 0;
        for (int j = 0; j < P.n; ++j) t += P.G[k][j] * x[j];
        f += z[k] * (t - P.h[k]);
    }
    return f;
}

static void load_shape(int k, const int32_t* type, const int32_t* nh, const int32_t* A_off, const double* A_pool,
                       const double* b_pool, const double* params, const double* roff, const double* Qoff, Shape* s) {
    s->type = type[k];
    s->nh = nh[k];
    s->A = A_pool + 3 * (int64_t)A_off[k];
    s->b = b_pool + A_off[k];
    s->R = params[4 * k]; s->L = params[4 * k + 1]; s->H = params[4 * k + 2]; s->beta = params[4 * k + 3];
    for (int i = 0; i < 3; ++i) s->roff[i] = roff[3 * k + i];
    for (int i = 0; i < 9; ++i) s->Qoff[i] = Qoff[9 * k + i];
}

int dcol_oracle_batch(int32_t n_shapes, const int32_t* type, const int32_t* nh, const int32_t* A_off,
                      const double* A_pool, const double* b_pool, const double* params, const double* roff,
                      const double* Qoff, int64_t B, const int32_t* s1, const int32_t* s2, const double* pose1,
                      const double* pose2, double tol, int32_t want_grad, int32_t nthreads, double* alpha,
                      double* contact, double* grad, int32_t* iters, int32_t* status) {
    (void)n_shapes;
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads > 0 ? nthreads : 1)
    for (int64_t i = 0; i < B; ++i) {
        Shape a, b;
        load_shape(s1[i], type, nh, A_off, A_pool, b_pool, params, roff, Qoff, &a);
        load_shape(s2[i], type, nh, A_off, A_pool, b_pool, params, roff, Qoff, &b);
        Prob P;
        double x[NMAX], s[MMAX], z[MMAX];
        int it = 0;
        int st = assemble(&a, pose1 + 6 * i, &b, pose2 + 6 * i, &P);
        if (st == ST_OK) st = pdip(&P, tol, x, s, z, &it);
        status[i] = st;
        iters[i] = it;
        alpha[i] = st == ST_OK ? x[3] : NAN;
        for (int k = 0; k < 3; ++k) contact[3 * i + k] = st == ST_OK ? x[k] : NAN;
        for (int k = 0; k < 12; ++k) grad[12 * i + k] = NAN;
        if (st == ST_OK && want_grad) {
            double th[12], th1[12];
            for (int k = 0; k < 6; ++k) { th[k] = pose1[6 * i + k]; th[6 + k] = pose2[6 * i + k]; }
            const double hstep = 1.4901161193847656e-08;
            const double f0 = lag_con(&a, &b, x, z, th);
            memcpy(th1, th, sizeof(th));
            for (int k = 0; k < 12; ++k) {
                double h = hstep;
                if ((th[k] + h) - th[k] == 0) h = hstep * (th[k] >= 0 ? 1.0 : -1.0) * fmax(1.0, fabs(th[k]));
                th1[k] += h;
                const double dx = th1[k] - th[k];
                grad[12 * i + k] = (lag_con(&a, &b, x, z, th1) - f0) / dx;
                th1[k] = th[k];
            }
        }
    }
    return 0;
}
