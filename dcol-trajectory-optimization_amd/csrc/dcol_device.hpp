// dcol_device.hpp — device-side DCOL proximity solver for gfx950 (MI355X / CDNA4).
//
// Execution model: ONE LANE OWNS ONE (knot x primitive-pair) problem.  The per-pair conic
// programs are tiny (m <= 40 rows, n <= 6 columns), independent and FP64: there is no
// contraction worth an MFMA and no cross-lane data dependence, so the wave64 is used as 64
// independent solvers.  Every per-pair quantity lives in VGPRs; the kernel is specialised at
// compile time on (N = primal dimension, NSOC = number of second-order-cone blocks,
// OMAX = orthant-row capacity) so all row/column loops are fully unrolled and register
// indices are static.  Pairs are bucketed by variant on the host (dcol_plan), so a wave
// never diverges on structure; lanes only diverge on the Newton iteration count.
//
// Algorithm (reference file:line):
//   assembly  ............ primitives/problem_matrices.py:4-364, combine_problem_matrices.py:3-70
//   PDIP init ............ proximity/pdip.py:291-332 (quirks Q1, Q2, Q11)
//   PDIP loop ............ proximity/pdip.py:373-470 (quirks Q3-Q8, Q10)
//   NT scaling ........... proximity/NT/NT_scaling.py:340-463 (quirk Q9)
//   FD gradient .......... proximity/proximity_gradient.py:8-138 + scipy approx_fprime
//
// Rounding-level (not algorithmic) departures, all measured harmless for the iterate
// sequence (SURVEY.md §7 "Hard parts"): FMA contraction; the SOC scaling is applied in
// closed form W^-1 = eta^-1 J Wbar J instead of cho_factor/cho_solve; G~ = W^-1 G is never
// materialised (G~'G~ and G~'v are accumulated as G'(W^-1 ...) ); the FD numerator is
// formed from the perturbed primitive's own rows only.
//
// Row layout inside a lane (compile-time positions):
//   rows [0, OMAX)                orthant rows; the first o1 belong to prim 1, the next
//                                 o2 to prim 2 (reference order [ort1; ort2]); rows >= o
//                                 are inert padding (G = 0, s = z = 1, masked everywhere)
//   rows [OMAX + 4b, OMAX + 4b+4) SOC block b (b = 0: first primitive that has one).
//                                 3-dim cone SOCs are padded with an identically-zero 4th
//                                 coordinate, which is exact: it stays +-0 through every
//                                 operation of the method.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Device functions are also host-callable so that tests/emul can compile the exact same
// solver for x86 and check it against the golden vectors without a GPU (test-only; the
// product library never runs them on the host).
#define DCOL_HD __host__ __device__ __forceinline__

namespace dcol {

enum : int32_t { ST_OK = 0, ST_MAXITER = 1, ST_UNSUPPORTED = 2, ST_NOT_PD = 3, ST_NONFINITE = 4, ST_TOO_LARGE = 5 };
enum : int32_t { SOC_NONE = 0, SOC_BALL = 1, SOC_CONE = 2 };
enum : int32_t { F_GRAD_FD = 1, F_GRAD_ENV = 2, F_CONTACT = 4 };

// One primitive, pre-digested on the host (dcol_capi.cpp: digest_shape()).
struct DevShape {
    int32_t type;      // dcol_shape_type
    int32_t n_ort;     // orthant rows contributed
    int32_t row_off;   // first row in the row pool
    int32_t soc_kind;  // SOC_NONE / SOC_BALL / SOC_CONE
    int32_t n_extra;   // extra primal columns (capsule/cylinder 1, polygon 2)
    int32_t pad0, pad1, pad2;
    double R;          // ball SOC radius (sphere/capsule/cylinder/polygon)
    double cone_c;     // cone SOC row 0, column 3: -(tan(beta) * 3 * H / 4)
    double tanb;       // cone: tan(beta)  (E = diag(tanb, 1, 1))
    double pad3;
    double r_off[4];   // body-frame position offset (+pad)
    double Q_off[9];   // row-major orientation offset
    double pad4[3];
};
static_assert(sizeof(DevShape) == 192, "DevShape layout");

// Orthant row descriptor: G row = [Qe * a, g3, ex0, ex1], h = (Qe * a) . r_eff
// (every orthant row of every primitive has this form; see digest_shape()).
struct DevRow {
    double a[3];
    double g3;
    double ex[2];
    double pad[2];
};
static_assert(sizeof(DevRow) == 64, "DevRow layout");

struct KArgs {
    const DevShape* __restrict__ shapes;
    const DevRow* __restrict__ rows;
    const int32_t* __restrict__ s1;
    const int32_t* __restrict__ s2;
    const double* __restrict__ pose1;   // [6][B]
    const double* __restrict__ pose2;   // [6][B]
    const int32_t* __restrict__ perm;   // slot -> pair index, or nullptr (identity)
    int64_t B;
    int64_t slot0;                      // this launch covers slots [slot0, slot0 + n)
    int64_t n;
    double tol;
    int32_t max_iter;
    int32_t flags;
    double* __restrict__ alpha;         // [B]
    double* __restrict__ contact;       // [3][B]
    double* __restrict__ grad;          // [12][B]
    int32_t* __restrict__ iters;        // [B]
    int32_t* __restrict__ status;       // [B]
};

// ------------------------------------------------------------------------------------
// primitive frames
// ------------------------------------------------------------------------------------
struct Frame {
    double Qe[9];  // Q(p) * Q_offset
    double re[3];  // r + Q(p) * r_offset
};

// dcm_from_mrp, problem_matrices.py:213-251 (same expanded expression)
DCOL_HD void dcm_from_mrp(double p1, double p2, double p3, double Q[9]) {
    const double s = p1 * p1 + p2 * p2 + p3 * p3 + 1.0;
    const double den = s * s;
    const double a = 4.0 * (p1 * p1) + 4.0 * (p2 * p2) + 4.0 * (p3 * p3) - 4.0;
    const double iden = 1.0 / den;
    Q[0] = (-((8.0 * (p2 * p2) + 8.0 * (p3 * p3)) * iden - 1.0) * den) * iden;
    Q[1] = (8.0 * p1 * p2 + p3 * a) * iden;
    Q[2] = (8.0 * p1 * p3 - p2 * a) * iden;
    Q[3] = (8.0 * p1 * p2 - p3 * a) * iden;
    Q[4] = (-((8.0 * (p1 * p1) + 8.0 * (p3 * p3)) * iden - 1.0) * den) * iden;
    Q[5] = (8.0 * p2 * p3 + p1 * a) * iden;
    Q[6] = (8.0 * p1 * p3 + p2 * a) * iden;
    Q[7] = (8.0 * p2 * p3 - p1 * a) * iden;
    Q[8] = (-((8.0 * (p1 * p1) + 8.0 * (p2 * p2)) * iden - 1.0) * den) * iden;
}

// problem_matrices.py:275-282 (r_eff = r + Q r_offset; Q_eff = Q Q_offset)
DCOL_HD void make_frame(const DevShape& S, const double th[6], Frame& F) {
    double Q[9];
    dcm_from_mrp(th[3], th[4], th[5], Q);
    const double o0 = S.r_off[0], o1 = S.r_off[1], o2 = S.r_off[2];
#pragma unroll
    for (int k = 0; k < 3; ++k) F.re[k] = th[k] + (Q[3 * k] * o0 + Q[3 * k + 1] * o1 + Q[3 * k + 2] * o2);
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c)
            F.Qe[3 * r + c] = Q[3 * r] * S.Q_off[c] + Q[3 * r + 1] * S.Q_off[3 + c] + Q[3 * r + 2] * S.Q_off[6 + c];
}

// ------------------------------------------------------------------------------------
// closed-form envelope gradient
// ------------------------------------------------------------------------------------
// d/dp_j of the reference DCM (problem_matrices.py:213-251), written Q = I + Nm/den with
// Nm = 8(p p' - S I) + a K, a = 4S - 4, den = (1+S)^2, S = p'p and
// K = [[0, p3, -p2], [-p3, 0, p1], [p2, -p1, 0]]:
//   dQ/dp_j = [8(e_j p' + p e_j' - 2 p_j I) + 8 p_j K + a K_j - 4 p_j Nm / (1+S)] / den
DCOL_HD void dcm_jacobian(const double p[3], double dQ[3][9]) {
    const double S = p[0] * p[0] + p[1] * p[1] + p[2] * p[2];
    const double s1 = 1.0 + S;
    const double iden = 1.0 / (s1 * s1);
    const double a = 4.0 * S - 4.0;
    const double K[9] = {0.0, p[2], -p[1], -p[2], 0.0, p[0], p[1], -p[0], 0.0};
    double Nm[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) Nm[3 * r + c] = 8.0 * (p[r] * p[c] - (r == c ? S : 0.0)) + a * K[3 * r + c];
    // K_j = dK/dp_j
    const double Kj[3][9] = {{0, 0, 0, 0, 0, 1, 0, -1, 0}, {0, 0, -1, 0, 0, 0, 1, 0, 0}, {0, 1, 0, -1, 0, 0, 0, 0, 0}};
    const double is1 = 1.0 / s1;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const double sym = (r == j ? p[c] : 0.0) + (c == j ? p[r] : 0.0) - (r == c ? 2.0 * p[j] : 0.0);
                const double v = 8.0 * sym + 8.0 * p[j] * K[3 * r + c] + a * Kj[j][3 * r + c] - 4.0 * p[j] * Nm[3 * r + c] * is1;
                dQ[j][3 * r + c] = v * iden;
            }
    }
}

// ------------------------------------------------------------------------------------
// second-order cone helpers (4-vectors)
// ------------------------------------------------------------------------------------
struct SocNT {
    double w0, w1[3], bf, eta, ieta;
};

// soc_NT_scaling, NT_scaling.py:340-405; W = eta * Wbar,
// Wbar = [[w0, w1'], [w1, I + bf w1 w1']], bf = 1/(w0+1), eta = (J(s)/J(z))^(1/4)
DCOL_HD void soc_nt(const double* s, const double* z, SocNT& W) {
    const double Jz = z[0] * z[0] - (z[1] * z[1] + z[2] * z[2] + z[3] * z[3]);
    const double Js = s[0] * s[0] - (s[1] * s[1] + s[2] * s[2] + s[3] * s[3]);
    const double iz = 1.0 / sqrt(Jz);
    const double is = 1.0 / sqrt(Js);
    double zb[4], sb[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        zb[k] = z[k] * iz;
        sb[k] = s[k] * is;
    }
    const double dot = zb[0] * sb[0] + zb[1] * sb[1] + zb[2] * sb[2] + zb[3] * sb[3];
    const double gamma = sqrt((1.0 + dot) * 0.5);
    const double i2g = 1.0 / (2.0 * gamma);
    W.w0 = (sb[0] + zb[0]) * i2g;
#pragma unroll
    for (int k = 0; k < 3; ++k) W.w1[k] = (sb[k + 1] - zb[k + 1]) * i2g;
    W.bf = 1.0 / (W.w0 + 1.0);
    W.eta = (Jz != 0.0) ? sqrt(sqrt(Js / Jz)) : 1.0;   // quirk Q9
    W.ieta = 1.0 / W.eta;
}

// out = W v
DCOL_HD void soc_mul(const SocNT& W, const double* v, double* out) {
    const double d = W.w1[0] * v[1] + W.w1[1] * v[2] + W.w1[2] * v[3];
    out[0] = W.eta * (W.w0 * v[0] + d);
    const double c = W.bf * d;
#pragma unroll
    for (int k = 0; k < 3; ++k) out[k + 1] = W.eta * (v[0] * W.w1[k] + v[k + 1] + c * W.w1[k]);
}

// out = W^-1 v = eta^-1 J Wbar J v   (closed form; replaces cho_solve, NT_scaling.py:109)
DCOL_HD void soc_solve(const SocNT& W, const double* v, double* out) {
    const double d = W.w1[0] * v[1] + W.w1[1] * v[2] + W.w1[2] * v[3];
    out[0] = W.ieta * (W.w0 * v[0] - d);
    const double c = W.bf * d;
#pragma unroll
    for (int k = 0; k < 3; ++k) out[k + 1] = W.ieta * (v[k + 1] - v[0] * W.w1[k] + c * W.w1[k]);
}

// soc_cone_product(u, v), pdip.py:165-200
DCOL_HD void soc_prod(const double* u, const double* v, double* out) {
    const double s = u[0] * v[0] + u[1] * v[1] + u[2] * v[2] + u[3] * v[3];
    out[1] = u[0] * v[1] + v[0] * u[1];
    out[2] = u[0] * v[2] + v[0] * u[2];
    out[3] = u[0] * v[3] + v[0] * u[3];
    out[0] = s;
}

// inverse_soc_cone_product(u, w), pdip.py:88-122
DCOL_HD void soc_iprod(const double* u, const double* w, double* out) {
    const double rho = u[0] * u[0] - (u[1] * u[1] + u[2] * u[2] + u[3] * u[3]);
    const double nu = u[1] * w[1] + u[2] * w[2] + u[3] * w[3];
    const double irho = 1.0 / rho;
    const double iu0 = 1.0 / u[0];
    const double c1 = nu * iu0 - w[0];
    const double c2 = rho * iu0;
    out[0] = irho * (u[0] * w[0] - nu);
#pragma unroll
    for (int k = 1; k < 4; ++k) out[k] = irho * (c1 * u[k] + c2 * w[k]);
}

// soc_linesearch, pdip.py:25-52 (quirk Q10: nu floored at 1e-25)
DCOL_HD double soc_ls(const double* y, const double* d) {
    const double nu = fmax(y[0] * y[0] - (y[1] * y[1] + y[2] * y[2] + y[3] * y[3]), 1e-25);
    const double zeta = y[0] * d[0] - (y[1] * d[1] + y[2] * d[2] + y[3] * d[3]);
    const double sn = sqrt(nu);
    const double isn = 1.0 / sn;
    const double inu = 1.0 / nu;
    const double rho0 = zeta * inu;
    const double coef = (zeta * isn + d[0]) / (y[0] * isn + 1.0);
    double n2 = 0.0;
#pragma unroll
    for (int k = 1; k < 4; ++k) {
        const double r = d[k] * isn - coef * (y[k] * inu);
        n2 += r * r;
    }
    const double n1 = sqrt(n2);
    return (n1 > rho0) ? fmin(1.0, 1.0 / (n1 - rho0)) : 1.0;
}

// ------------------------------------------------------------------------------------
// the per-pair solver
// ------------------------------------------------------------------------------------
template <int N, int NSOC, int OMAX>
struct Solver {
    static constexpr int M = OMAX + 4 * NSOC;
    static constexpr int NH = N * (N + 1) / 2;

    // state
    double G[M][N];
    double h[M];
    double x[N], s[M], z[M];
    int o1, o;

    DCOL_HD static bool valid(int i, int o_) { return i >= OMAX || i < o_; }

    // -------- assembly (problem_matrices.py + combine_problem_matrices.py) --------------
    DCOL_HD void assemble(const KArgs& A, const DevShape& S1, const DevShape& S2,
                                             const Frame& F1, const Frame& F2, int slot_owner[2]) {
        o1 = S1.n_ort;
        o = o1 + S2.n_ort;
        const double* __restrict__ rows = reinterpret_cast<const double*>(A.rows);
#pragma unroll
        for (int i = 0; i < OMAX; ++i) {
            const bool v = i < o;
            const bool p2 = i >= o1;
            double a0 = 0, a1 = 0, a2 = 0, g3 = 0, e0 = 0, e1 = 0;
            if (v) {
                const int ri = p2 ? (S2.row_off + (i - o1)) : (S1.row_off + i);
                const double2* rw = reinterpret_cast<const double2*>(rows + 8 * (int64_t)ri);
                const double2 q0 = rw[0], q1 = rw[1], q2 = rw[2];
                a0 = q0.x; a1 = q0.y; a2 = q1.x; g3 = q1.y; e0 = q2.x; e1 = q2.y;
            }
            double Qe[9], re[3];
#pragma unroll
            for (int k = 0; k < 9; ++k) Qe[k] = p2 ? F2.Qe[k] : F1.Qe[k];
#pragma unroll
            for (int k = 0; k < 3; ++k) re[k] = p2 ? F2.re[k] : F1.re[k];
            const double u0 = Qe[0] * a0 + Qe[1] * a1 + Qe[2] * a2;
            const double u1 = Qe[3] * a0 + Qe[4] * a1 + Qe[5] * a2;
            const double u2 = Qe[6] * a0 + Qe[7] * a1 + Qe[8] * a2;
            G[i][0] = u0; G[i][1] = u1; G[i][2] = u2; G[i][3] = g3;
            if constexpr (N > 4) G[i][4] = e0;
            if constexpr (N > 5) G[i][5] = e1;
            h[i] = u0 * re[0] + u1 * re[1] + u2 * re[2];
        }
        // SOC blocks: slot 0 = first primitive with a SOC, slot 1 = prim 2 when both have one
        slot_owner[0] = S1.soc_kind != SOC_NONE ? 0 : 1;
        slot_owner[1] = 1;
#pragma unroll
        for (int b = 0; b < NSOC; ++b) {
            const bool p2 = slot_owner[b] == 1;
            const int kind = p2 ? S2.soc_kind : S1.soc_kind;
            const double R = p2 ? S2.R : S1.R;
            const double cc = p2 ? S2.cone_c : S1.cone_c;
            const double tb = p2 ? S2.tanb : S1.tanb;
            const int nx = p2 ? S2.n_extra : S1.n_extra;
            double Qe[9], re[3];
#pragma unroll
            for (int k = 0; k < 9; ++k) Qe[k] = p2 ? F2.Qe[k] : F1.Qe[k];
#pragma unroll
            for (int k = 0; k < 3; ++k) re[k] = p2 ? F2.re[k] : F1.re[k];
            soc_rows(kind, R, cc, tb, nx, Qe, re, &G[OMAX + 4 * b], &h[OMAX + 4 * b]);
        }
    }

    // The 4 rows of one SOC block.  Ball (sphere/capsule/cylinder/polygon):
    //   [0 0 0 -R | 0..], h 0;  [-e_k | 0 | Qe[k][0..nx)], h -re[k]     (problem_matrices.py:21-28, 66-76, 112-119, 165-176)
    // Cone: [-E Qe' | -(tanb 3H/4) e_0], h = -E Qe' re; 4th row zero     (problem_matrices.py:138-145)
    DCOL_HD static void soc_rows(int kind, double R, double cc, double tb, int nx,
                                                    const double* Qe, const double* re, double (*Gb)[N], double* hb) {
        if (kind == SOC_CONE) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const double e = (k == 0) ? tb : 1.0;
                const double u0 = -(e * Qe[0 + k]);
                const double u1 = -(e * Qe[3 + k]);
                const double u2 = -(e * Qe[6 + k]);
                Gb[k][0] = u0; Gb[k][1] = u1; Gb[k][2] = u2;
                Gb[k][3] = (k == 0) ? cc : 0.0;
#pragma unroll
                for (int j = 4; j < N; ++j) Gb[k][j] = 0.0;
                hb[k] = u0 * re[0] + u1 * re[1] + u2 * re[2];
            }
#pragma unroll
            for (int j = 0; j < N; ++j) Gb[3][j] = 0.0;
            hb[3] = 0.0;
        } else {
            Gb[0][0] = 0.0; Gb[0][1] = 0.0; Gb[0][2] = 0.0; Gb[0][3] = -R;
#pragma unroll
            for (int j = 4; j < N; ++j) Gb[0][j] = 0.0;
            hb[0] = 0.0;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
#pragma unroll
                for (int j = 0; j < 3; ++j) Gb[k + 1][j] = (j == k) ? -1.0 : 0.0;
                Gb[k + 1][3] = 0.0;
                if constexpr (N > 4) Gb[k + 1][4] = (nx >= 1) ? Qe[3 * k] : 0.0;
                if constexpr (N > 5) Gb[k + 1][5] = (nx >= 2) ? Qe[3 * k + 1] : 0.0;
                hb[k + 1] = -re[k];
            }
        }
    }

    // -------- small dense helpers ------------------------------------------------------
    // y = G x - h (per row, pads -> 0 since G = h = 0)
    DCOL_HD void Gx(const double* v, double* out) const {
#pragma unroll
        for (int i = 0; i < M; ++i) {
            double acc = G[i][0] * v[0];
#pragma unroll
            for (int j = 1; j < N; ++j) acc += G[i][j] * v[j];
            out[i] = acc;
        }
    }
    // out = G' w   (pads contribute 0 * w = 0: w is finite on pads)
    DCOL_HD void GTx(const double* w, double* out) const {
#pragma unroll
        for (int j = 0; j < N; ++j) out[j] = 0.0;
#pragma unroll
        for (int i = 0; i < M; ++i)
#pragma unroll
            for (int j = 0; j < N; ++j) out[j] += G[i][j] * w[i];
    }

    // upper Cholesky H = F'F on packed upper triangle (scipy.linalg.cholesky semantics);
    // returns false if a pivot is <= 0 or NaN (LAPACK dpotrf info > 0)
    DCOL_HD static bool chol(double (&H)[N][N], double (&F)[N][N], double (&idg)[N]) {
        bool ok = true;
#pragma unroll
        for (int j = 0; j < N; ++j) {
            double d = H[j][j];
#pragma unroll
            for (int k = 0; k < j; ++k) d -= F[k][j] * F[k][j];
            ok = ok && (d > 0.0);
            const double fjj = sqrt(d);
            F[j][j] = fjj;
            idg[j] = 1.0 / fjj;
#pragma unroll
            for (int c = j + 1; c < N; ++c) {
                double t = H[j][c];
#pragma unroll
                for (int k = 0; k < j; ++k) t -= F[k][j] * F[k][c];
                F[j][c] = t * idg[j];
            }
        }
        return ok;
    }
    // solve F'F x = b  (cho_solve((F, False), b))
    DCOL_HD static void chol_solve(const double (&F)[N][N], const double (&idg)[N], const double* b, double* out) {
        double y[N];
#pragma unroll
        for (int j = 0; j < N; ++j) {
            double t = b[j];
#pragma unroll
            for (int k = 0; k < j; ++k) t -= F[k][j] * y[k];
            y[j] = t * idg[j];
        }
#pragma unroll
        for (int j = N - 1; j >= 0; --j) {
            double t = y[j];
#pragma unroll
            for (int k = j + 1; k < N; ++k) t -= F[j][k] * out[k];
            out[j] = t * idg[j];
        }
    }

    // bring2cone, pdip.py:237-287 (quirk Q11)
    DCOL_HD void bring2cone(double* r) const {
        double a = -1.0;
        bool any = false;
        double mn = 0.0;
#pragma unroll
        for (int i = 0; i < OMAX; ++i) {
            if (i < o) {
                if (r[i] <= 0.0) any = true;
                mn = (i == 0) ? r[i] : fmin(mn, r[i]);
            }
        }
        if (any) a = -mn;
#pragma unroll
        for (int b = 0; b < NSOC; ++b) {
            const double* q = r + OMAX + 4 * b;
            const double res = q[0] - sqrt(q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
            if (res <= 0.0) a = fmax(a, -res);
        }
        if (a >= 0.0) {
            const double sh = 1.0 + a;
#pragma unroll
            for (int i = 0; i < OMAX; ++i)
                if (i < o) r[i] += sh;
#pragma unroll
            for (int b = 0; b < NSOC; ++b) r[OMAX + 4 * b] += sh;
        }
    }

    // -------- initialize, pdip.py:291-332 ------------------------------------------------
    DCOL_HD bool initialize() {
        double H[N][N], F[N][N], idg[N];
#pragma unroll
        for (int j = 0; j < N; ++j)
#pragma unroll
            for (int c = j; c < N; ++c) {
                double acc = 0.0;
#pragma unroll
                for (int i = 0; i < M; ++i) acc += G[i][j] * G[i][c];
                H[j][c] = acc;
            }
        const bool ok = chol(H, F, idg);   // F' = np.linalg.cholesky(G'G) (lower L = F')
        double gth[N], xh[N];
        GTx(h, gth);
        chol_solve(F, idg, gth, xh);        // x_hat = L^-T L^-1 G'h
        double r[M];
        Gx(xh, r);
#pragma unroll
        for (int i = 0; i < M; ++i) r[i] -= h[i];   // quirk Q2: G x_hat - h
        bring2cone(r);
        // quirk Q1: y = solve_triangular(L, -c) with lower=False reads diag(L) only:
        // y = -c / diag(L) = -e_3 / L_33;  then x = L^-T y (proper back substitution)
        double yv[N], xz[N];
#pragma unroll
        for (int j = 0; j < N; ++j) yv[j] = (j == 3) ? -idg[3] : 0.0;
#pragma unroll
        for (int j = N - 1; j >= 0; --j) {
            double t = yv[j];
#pragma unroll
            for (int k = j + 1; k < N; ++k) t -= F[j][k] * xz[k];
            xz[j] = t * idg[j];
        }
        double zt[M];
        Gx(xz, zt);
        bring2cone(zt);
#pragma unroll
        for (int j = 0; j < N; ++j) x[j] = xh[j];
#pragma unroll
        for (int i = 0; i < M; ++i) {
            const bool v = valid(i, o);
            s[i] = v ? r[i] : 1.0;
            z[i] = v ? zt[i] : 1.0;
        }
        return ok;
    }

    // -------- NT scaling application ---------------------------------------------------
    struct Scaling {
        double w[OMAX], wi[OMAX];
        SocNT soc[NSOC > 0 ? NSOC : 1];
    };
    DCOL_HD static void mulW(const Scaling& W, const double* v, double* out) {
#pragma unroll
        for (int i = 0; i < OMAX; ++i) out[i] = v[i] * W.w[i];
#pragma unroll
        for (int b = 0; b < NSOC; ++b) soc_mul(W.soc[b], v + OMAX + 4 * b, out + OMAX + 4 * b);
    }
    DCOL_HD static void solveW(const Scaling& W, const double* v, double* out) {
#pragma unroll
        for (int i = 0; i < OMAX; ++i) out[i] = v[i] * W.wi[i];
#pragma unroll
        for (int b = 0; b < NSOC; ++b) soc_solve(W.soc[b], v + OMAX + 4 * b, out + OMAX + 4 * b);
    }
    DCOL_HD static void cone_prod(const double* u, const double* v, double* out) {
#pragma unroll
        for (int i = 0; i < OMAX; ++i) out[i] = u[i] * v[i];
#pragma unroll
        for (int b = 0; b < NSOC; ++b) soc_prod(u + OMAX + 4 * b, v + OMAX + 4 * b, out + OMAX + 4 * b);
    }
    DCOL_HD static void cone_iprod(const double* lam, const double* v, double* out) {
#pragma unroll
        for (int i = 0; i < OMAX; ++i) out[i] = v[i] / lam[i];
#pragma unroll
        for (int b = 0; b < NSOC; ++b) soc_iprod(lam + OMAX + 4 * b, v + OMAX + 4 * b, out + OMAX + 4 * b);
    }
    // linesearch, pdip.py:55-85
    DCOL_HD double linesearch(const double* v, const double* d) const {
        double a = 1.0;
#pragma unroll
        for (int i = 0; i < OMAX; ++i)
            if (i < o && d[i] < 0.0) a = fmin(a, -v[i] / d[i]);
#pragma unroll
        for (int b = 0; b < NSOC; ++b) a = fmin(a, soc_ls(v + OMAX + 4 * b, d + OMAX + 4 * b));
        return a;
    }
    DCOL_HD double dotm(const double* u, const double* v) const {
        double acc = 0.0;
#pragma unroll
        for (int i = 0; i < M; ++i)
            if (valid(i, o)) acc += u[i] * v[i];
        return acc;
    }

    // Newton direction for a given lambda\ds:  b~z = W^-1(-rz - W lds);
    // dx = (G~'G~)^-1 (-rx + G~' b~z); dz = W^-1(G~ dx - b~z); ds = W(lds - W dz)
    DCOL_HD void direction(const Scaling& W, const double (&F)[N][N], const double (&idg)[N],
                                              const double* rx, const double* rz, const double* lds,
                                              double* dx, double* dz, double* ds) const {
        double t[M], bzt[M];
        mulW(W, lds, t);
#pragma unroll
        for (int i = 0; i < M; ++i) t[i] = -rz[i] - t[i];
        solveW(W, t, bzt);
        solveW(W, bzt, t);                       // t = W^-1 b~z  (G~'b~z = G' W^-1 b~z)
        double rhs[N];
        GTx(t, rhs);
#pragma unroll
        for (int j = 0; j < N; ++j) rhs[j] -= rx[j];
        chol_solve(F, idg, rhs, dx);
        double u[M];
        Gx(dx, u);
        solveW(W, u, t);                         // G~ dx = W^-1 G dx
#pragma unroll
        for (int i = 0; i < M; ++i) t[i] -= bzt[i];
        solveW(W, t, dz);
        mulW(W, dz, t);
#pragma unroll
        for (int i = 0; i < M; ++i) t[i] = lds[i] - t[i];
        mulW(W, t, ds);
    }

    // -------- solve_lp_pdip, pdip.py:373-470 -------------------------------------------
    // returns status; *it = Newton steps taken
    DCOL_HD int32_t pdip(double tol, int max_iter, int* it_out) {
        const int deg = o + NSOC;                       // quirk Q7
        int it = 0;
        int32_t st = ST_MAXITER;
        for (it = 0; it < max_iter; ++it) {
            Scaling W;
#pragma unroll
            for (int i = 0; i < OMAX; ++i) {
                const double wv = sqrt(s[i] / z[i]);
                W.w[i] = wv;
                W.wi[i] = 1.0 / wv;
            }
#pragma unroll
            for (int b = 0; b < NSOC; ++b) soc_nt(s + OMAX + 4 * b, z + OMAX + 4 * b, W.soc[b]);
            double lam[M], ll[M];
            mulW(W, z, lam);
            cone_prod(lam, lam, ll);
            double rx[N], rz[M];
            GTx(z, rx);
            rx[3] += 1.0;                               // + c (c = e_3)
            Gx(x, rz);
#pragma unroll
            for (int i = 0; i < M; ++i) rz[i] = s[i] + rz[i] - h[i];
            const double sz = dotm(s, z);
            const double mu = sz / (double)deg;
            if (mu < tol) {                             // quirk Q3
                st = ST_OK;
                break;
            }
            // normal matrix G~'G~, G~ = W^-1 G  (pdip.py:429-434)
            double Hm[N][N];
#pragma unroll
            for (int j = 0; j < N; ++j)
#pragma unroll
                for (int c = j; c < N; ++c) Hm[j][c] = 0.0;
#pragma unroll
            for (int i = 0; i < OMAX; ++i) {
                double g[N];
#pragma unroll
                for (int j = 0; j < N; ++j) g[j] = G[i][j] * W.wi[i];
#pragma unroll
                for (int j = 0; j < N; ++j)
#pragma unroll
                    for (int c = j; c < N; ++c) Hm[j][c] += g[j] * g[c];
            }
#pragma unroll
            for (int b = 0; b < NSOC; ++b) {
                double gt[4][N];
#pragma unroll
                for (int j = 0; j < N; ++j) {
                    double col[4], res[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k) col[k] = G[OMAX + 4 * b + k][j];
                    soc_solve(W.soc[b], col, res);
#pragma unroll
                    for (int k = 0; k < 4; ++k) gt[k][j] = res[k];
                }
#pragma unroll
                for (int k = 0; k < 4; ++k)
#pragma unroll
                    for (int j = 0; j < N; ++j)
#pragma unroll
                        for (int c = j; c < N; ++c) Hm[j][c] += gt[k][j] * gt[k][c];
            }
            bool finite = true;
#pragma unroll
            for (int j = 0; j < N; ++j)
#pragma unroll
                for (int c = j; c < N; ++c) finite = finite && __builtin_isfinite(Hm[j][c]);
            if (!finite) { st = ST_NONFINITE; break; }  // scipy check_finite -> ValueError
            double F[N][N], idg[N];
            if (!chol(Hm, F, idg)) { st = ST_NOT_PD; break; }

            // predictor (affine) step
            double neg[M], lds[M], dx[N], dz[M], ds[M];
#pragma unroll
            for (int i = 0; i < M; ++i) neg[i] = -ll[i];
            cone_iprod(lam, neg, lds);
            direction(W, F, idg, rx, rz, lds, dx, dz, ds);
            const double aa = fmin(linesearch(s, ds), linesearch(z, dz));   // quirk Q5
            double sp[M], zp[M];
#pragma unroll
            for (int i = 0; i < M; ++i) {
                sp[i] = s[i] + aa * ds[i];
                zp[i] = z[i] + aa * dz[i];
            }
            const double rho = dotm(sp, zp) / sz;
            const double sc = fmax(0.0, fmin(1.0, rho));
            const double sigma = sc * sc * sc;         // quirk Q6

            // corrector (combined) step
            double t1[M], t2[M], cp[M];
            solveW(W, ds, t1);
            mulW(W, dz, t2);
            cone_prod(t1, t2, cp);
            const double smu = sigma * mu;
#pragma unroll
            for (int i = 0; i < M; ++i) neg[i] = -ll[i] - cp[i];
#pragma unroll
            for (int i = 0; i < OMAX; ++i) neg[i] += smu;
#pragma unroll
            for (int b = 0; b < NSOC; ++b) neg[OMAX + 4 * b] += smu;
            cone_iprod(lam, neg, lds);
            direction(W, F, idg, rx, rz, lds, dx, dz, ds);
            const double a = fmin(1.0, 0.99 * fmin(linesearch(s, ds), linesearch(z, dz)));
#pragma unroll
            for (int j = 0; j < N; ++j) x[j] += a * dx[j];
#pragma unroll
            for (int i = 0; i < M; ++i) {
                if (valid(i, o)) {
                    s[i] += a * ds[i];
                    z[i] += a * dz[i];
                }
            }
        }
        *it_out = it;
        return st;
    }

    // -------- FD envelope gradient, proximity_gradient.py:8-88 -------------------------
    // f_k(theta_k) = sum over rows of primitive k of z_i (G_i(theta_k) x - h_i(theta_k))
    DCOL_HD double lag_part(const KArgs& A, const DevShape& S, int k, int slot, const double th[6]) const {
        Frame Fr;
        make_frame(S, th, Fr);
        const double* __restrict__ rows = reinterpret_cast<const double*>(A.rows);
        double acc = 0.0;
#pragma unroll
        for (int i = 0; i < OMAX; ++i) {
            const bool own = (k == 0) ? (i < o1) : (i >= o1 && i < o);
            if (own) {
                const int ri = S.row_off + ((k == 0) ? i : (i - o1));
                const double2* rw = reinterpret_cast<const double2*>(rows + 8 * (int64_t)ri);
                const double2 q0 = rw[0], q1 = rw[1], q2 = rw[2];
                const double u0 = Fr.Qe[0] * q0.x + Fr.Qe[1] * q0.y + Fr.Qe[2] * q1.x;
                const double u1 = Fr.Qe[3] * q0.x + Fr.Qe[4] * q0.y + Fr.Qe[5] * q1.x;
                const double u2 = Fr.Qe[6] * q0.x + Fr.Qe[7] * q0.y + Fr.Qe[8] * q1.x;
                double gx = u0 * x[0] + u1 * x[1] + u2 * x[2] + q1.y * x[3];
                if constexpr (N > 4) gx += q2.x * x[4];
                if constexpr (N > 5) gx += q2.y * x[5];
                const double hh = u0 * Fr.re[0] + u1 * Fr.re[1] + u2 * Fr.re[2];
                acc += z[i] * (gx - hh);
            }
        }
#pragma unroll
        for (int b = 0; b < NSOC; ++b) {
            if (b == slot) {
                double Gb[4][N], hb[4];
                soc_rows(S.soc_kind, S.R, S.cone_c, S.tanb, S.n_extra, Fr.Qe, Fr.re, Gb, hb);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    double gx = Gb[r][0] * x[0];
#pragma unroll
                    for (int j = 1; j < N; ++j) gx += Gb[r][j] * x[j];
                    acc += z[OMAX + 4 * b + r] * (gx - hb[r]);
                }
            }
        }
        return acc;
    }

    // scipy approx_fprime(theta, f, sqrt(eps)) restricted to primitive k's 6 coordinates
    DCOL_HD void fd_grad_prim(const KArgs& A, const DevShape& S, int k, int slot,
                                                 const double th0[6], double* g) const {
        const double hstep = 1.4901161193847656e-08;   // sqrt(finfo(float).eps)
        const double f0 = lag_part(A, S, k, slot, th0);
#pragma unroll 1
        for (int j = 0; j < 6; ++j) {
            double th[6];
#pragma unroll
            for (int q = 0; q < 6; ++q) th[q] = th0[q];
            double hj = hstep;
            if ((th0[j] + hstep) - th0[j] == 0.0)       // _numdiff: fall back to a relative step
                hj = hstep * (th0[j] >= 0.0 ? 1.0 : -1.0) * fmax(1.0, fabs(th0[j]));
            th[j] = th0[j] + hj;
            const double dxj = th[j] - th0[j];
            g[j] = (lag_part(A, S, k, slot, th) - f0) / dxj;
        }
    }

    // d/dtheta_k of z'(G(theta)x - h(theta)) in closed form.  Every row of primitive k reads
    // value_i = u_i.(x[0:3] - r_eff) + (theta-free terms) + ex_i(Qe).x[4:], with u_i = Qe a_i
    // (rotated rows: polytope/cone/cylinder orthant rows, cone SOC rows) or u = -e_k
    // (ball SOC rows).  With w = sum z_i a_i (rotated rows, body frame), zeta = z of the ball
    // SOC rows 1..3, xi = (x4, x5, 0) restricted to the extra columns:
    //   d/dr   = zeta - Qe w
    //   d/dp_j = d' Q_j (Qoff w) - (Qe w - zeta)' Q_j r_off + zeta' Q_j (Qoff xi)
    DCOL_HD void env_grad_prim(const KArgs& A, const DevShape& S, int k, int slot,
                                                  const double th[6], double* g) const {
        Frame Fr;
        make_frame(S, th, Fr);
        const double* __restrict__ rows = reinterpret_cast<const double*>(A.rows);
        double w[3] = {0.0, 0.0, 0.0};
#pragma unroll
        for (int i = 0; i < OMAX; ++i) {
            const bool own = (k == 0) ? (i < o1) : (i >= o1 && i < o);
            if (own) {
                const int ri = S.row_off + ((k == 0) ? i : (i - o1));
                const double2* rw = reinterpret_cast<const double2*>(rows + 8 * (int64_t)ri);
                const double2 q0 = rw[0], q1 = rw[1];
                w[0] += z[i] * q0.x;
                w[1] += z[i] * q0.y;
                w[2] += z[i] * q1.x;
            }
        }
        double zeta[3] = {0.0, 0.0, 0.0};
        double xi[3] = {0.0, 0.0, 0.0};
#pragma unroll
        for (int b = 0; b < NSOC; ++b) {
            if (b == slot) {
                const double* zb = z + OMAX + 4 * b;
                if (S.soc_kind == SOC_CONE) {
                    w[0] -= zb[0] * S.tanb;     // a_k = -E_kk e_k
                    w[1] -= zb[1];
                    w[2] -= zb[2];
                } else {
                    zeta[0] = zb[1]; zeta[1] = zb[2]; zeta[2] = zb[3];
                    if constexpr (N > 4) xi[0] = (S.n_extra >= 1) ? x[4] : 0.0;
                    if constexpr (N > 5) xi[1] = (S.n_extra >= 2) ? x[5] : 0.0;
                }
            }
        }
        double e[3], d[3], c1[3], c2[3];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const double qw = Fr.Qe[3 * r] * w[0] + Fr.Qe[3 * r + 1] * w[1] + Fr.Qe[3 * r + 2] * w[2];
            e[r] = qw - zeta[r];
            g[r] = -e[r];
            d[r] = x[r] - Fr.re[r];
            c1[r] = S.Q_off[3 * r] * w[0] + S.Q_off[3 * r + 1] * w[1] + S.Q_off[3 * r + 2] * w[2];
            c2[r] = S.Q_off[3 * r] * xi[0] + S.Q_off[3 * r + 1] * xi[1] + S.Q_off[3 * r + 2] * xi[2];
        }
        double dQ[3][9];
        dcm_jacobian(th + 3, dQ);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            double acc = 0.0;
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                const double* q = &dQ[j][3 * r];
                const double m1 = q[0] * c1[0] + q[1] * c1[1] + q[2] * c1[2];
                const double m2 = q[0] * S.r_off[0] + q[1] * S.r_off[1] + q[2] * S.r_off[2];
                const double m3 = q[0] * c2[0] + q[1] * c2[1] + q[2] * c2[2];
                acc += d[r] * m1 - e[r] * m2 + zeta[r] * m3;
            }
            g[3 + j] = acc;
        }
    }
};

// ------------------------------------------------------------------------------------
// kernel
// ------------------------------------------------------------------------------------
template <int N, int NSOC, int OMAX>
DCOL_HD void solve_one(const KArgs& A, int64_t pi) {
    const int64_t B = A.B;
    const int k1 = A.s1[pi], k2 = A.s2[pi];
    const DevShape& S1 = A.shapes[k1];
    const DevShape& S2 = A.shapes[k2];
    double th1[6], th2[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) {
        th1[q] = A.pose1[q * B + pi];
        th2[q] = A.pose2[q * B + pi];
    }
    Frame F1, F2;
    make_frame(S1, th1, F1);
    make_frame(S2, th2, F2);

    Solver<N, NSOC, OMAX> P;
    int slot_owner[2];
    P.assemble(A, S1, S2, F1, F2, slot_owner);
    int it = 0;
    int32_t st;
    if (!P.initialize()) st = ST_NOT_PD;
    else st = P.pdip(A.tol, A.max_iter, &it);

    const double nan = __builtin_nan("");
    const bool ok = st == ST_OK;
    A.alpha[pi] = ok ? P.x[3] : nan;
    if (A.iters) A.iters[pi] = it;
    if (A.status) A.status[pi] = st;
    if ((A.flags & F_CONTACT) && A.contact) {
#pragma unroll
        for (int q = 0; q < 3; ++q) A.contact[q * B + pi] = ok ? P.x[q] : nan;
    }
    if ((A.flags & (F_GRAD_FD | F_GRAD_ENV)) && A.grad) {
        double g[12];
        if (ok) {
            const int slot1 = (S1.soc_kind != SOC_NONE) ? 0 : -1;
            const int slot2 = (S2.soc_kind != SOC_NONE) ? ((S1.soc_kind != SOC_NONE) ? 1 : 0) : -1;
            if (A.flags & F_GRAD_ENV) {
                P.env_grad_prim(A, S1, 0, slot1, th1, g);
                P.env_grad_prim(A, S2, 1, slot2, th2, g + 6);
            } else {
                P.fd_grad_prim(A, S1, 0, slot1, th1, g);
                P.fd_grad_prim(A, S2, 1, slot2, th2, g + 6);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 12; ++q) g[q] = nan;
        }
#pragma unroll
        for (int q = 0; q < 12; ++q) A.grad[q * B + pi] = g[q];
    }
}

// One lane per pair.  Slots [slot0, slot0+n) of the plan's permutation (or identity).
template <int N, int NSOC, int OMAX>
__global__ void __launch_bounds__(256) prox_kernel(KArgs A) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= A.n) return;
    const int64_t pi = A.perm ? (int64_t)A.perm[A.slot0 + t] : (A.slot0 + t);
    solve_one<N, NSOC, OMAX>(A, pi);
}

}  // namespace dcol
