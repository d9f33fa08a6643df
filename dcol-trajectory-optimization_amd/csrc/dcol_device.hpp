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

// Fast reciprocal / reciprocal square root: the hardware estimate (v_rcp_f64 / v_rsq_f64,
// measured up to 2.5e8 ulp = 2^-24.5 relative) refined by Newton steps.  Measured on MI355X
// over 4.2M inputs spanning 2^-60..2^60 (tools/rcp_ulp.hip, profiles/r02_altro/rcp_ulp.log):
// frcp (two steps) correctly rounded on every input; frcp1 (one step) <= 11 ulp, mean 0.59,
// 59 % correctly rounded; frsqrt <= 2 ulp, mean 0.2.  frcp1 serves the per-iteration
// reciprocals (rows' 1/(s z), step lengths, rho, SOC NT scalars, soc_iprod): their
// operands carry far more than 11 ulp of rounding from the sums and cancellations that
// form them, and the iterate sequence stays equal to the reference's on every golden
// vector (GPU tests); the host build used by tests/emul keeps IEEE division.
DCOL_HD double frcp(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    double y = __builtin_amdgcn_rcp(x);
    double e = __builtin_fma(-x, y, 1.0);
    y = __builtin_fma(y, e, y);
    e = __builtin_fma(-x, y, 1.0);
    return __builtin_fma(y, e, y);
#else
    return 1.0 / x;
#endif
}
DCOL_HD double frcp1(double x) {   // v_rcp_f64 + one Newton step (<= 11 ulp measured)
#if defined(__HIP_DEVICE_COMPILE__)
    double y = __builtin_amdgcn_rcp(x);
    const double e = __builtin_fma(-x, y, 1.0);
    return __builtin_fma(y, e, y);
#else
    return 1.0 / x;
#endif
}
DCOL_HD double frsqrt(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = 0.5 * y;               // g ~ sqrt(x), h ~ 1/(2 sqrt(x))
    double r = __builtin_fma(-g, h, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    r = __builtin_fma(-g, h, 0.5);
    h = __builtin_fma(h, r, h);
    return h + h;
#else
    return 1.0 / sqrt(x);
#endif
}

// x > 0 and finite (one v_cmp_class on the GPU: +subnormal | +normal)
DCOL_HD bool pos_finite(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_class(x, 0x180);
#else
    return x > 0.0 && x < __builtin_inf();
#endif
}

enum : int32_t { ST_OK = 0, ST_MAXITER = 1, ST_UNSUPPORTED = 2, ST_NOT_PD = 3, ST_NONFINITE = 4, ST_TOO_LARGE = 5 };
constexpr int32_t ST_SUSPENDED = 100;   // internal: handed to the resume launch (never reported)
enum : int32_t { SOC_NONE = 0, SOC_BALL = 1, SOC_CONE = 2 };
enum : int32_t { F_GRAD_FD = 1, F_GRAD_ENV = 2, F_CONTACT = 4, F_GRAD_IMP = 16 };

// One primitive, pre-digested on the host (dcol_capi.cpp: digest_shape()).
struct DevShape {
    int32_t type;      // dcol_shape_type
    int32_t n_ort;     // orthant rows contributed
    int32_t row_off;   // first row in the row pool
    int32_t soc_kind;  // SOC_NONE / SOC_BALL / SOC_CONE
    int32_t n_extra;   // extra primal columns (capsule/cylinder 1, polygon 2)
    int32_t plain;     // r_off == 0 and Q_off == I (make_frame skips the offset products)
    int32_t n_p;       // orthant rows of the pose form [Qe a, g3, 0..] (polytope faces, cone base,
                       // cylinder caps); the other n_ort - n_p rows have the extra-column form
                       // [0 0 0, g3, ex] (capsule / cylinder segment rows, polygon edges).  In the
                       // row pool the extra-column rows come first, then the pose rows.
    int32_t boxp;      // polytope of 6 rows whose rows 3..5 are the exact negatives of rows 0..2
                       // (rect prisms: create_rect_prism) -- the BOX kernels (Solver)
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

constexpr int kRec = 14;   // doubles per packed record (include/dcol.h DCOL_REC)

// the record's last slot: (int32 status, int32 iters) in one 8-byte word (status low)
DCOL_HD double rec_ints(int32_t status, int32_t iters) {
    const unsigned long long w = ((unsigned long long)(unsigned)iters << 32) | (unsigned long long)(unsigned)status;
#if defined(__HIP_DEVICE_COMPILE__)
    return __longlong_as_double((long long)w);
#else
    double d;
    __builtin_memcpy(&d, &w, sizeof d);
    return d;
#endif
}

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
    // [B][kRec] packed per-pair records (include/dcol.h DCOL_REC: alpha, grad(12), the int32
    // pair (status, iters) in the last slot), written straight from the solver's epilogue by
    // dcol_prox_batch_multi_gpu's in-place path; nullptr: none.  With rec set, alpha / grad /
    // iters / status may be nullptr (record-only).
    double* __restrict__ rec = nullptr;
    // Suspend / resume (variants with FL bit 4; dcol_capi.cpp): in the main launch, a wave
    // whose still-iterating pairs drop to susp_t or fewer, at iteration susp_min or later,
    // hands those pairs -- their iterate (x, s, z, r) and iteration count -- to the resume
    // launch, which reassembles their rows and continues the same iteration sequence.  One
    // entry per suspended pair; at most susp_t per wave, so susp_cap = waves * susp_t suffices.
    int32_t susp_t;                     // 0: never suspend
    int32_t susp_min;
    int32_t* susp_count;                // entries appended (zeroed before the main launch)
    int32_t* susp_pi;                   // [susp_cap] pair index (slot index into perm space)
    double* susp_state;                 // [fields][susp_cap]: it, x[N], then (s, z, r) per lane row
    int64_t susp_cap;
#ifdef DCOL_STAMPS
    unsigned long long* stamps = nullptr;   // diagnostic build only (tools/stamp_probe.hip, the pair
                                            // server of lib_stamps): [B][16]; nullptr: none
#endif
};

#if defined(DCOL_STAMPS) && defined(__HIP_DEVICE_COMPILE__)
#define DCOL_STAMP(A, pi, q, k)                                                         \
    do {                                                                                \
        __builtin_amdgcn_sched_barrier(0);                                              \
        unsigned long long t_;                                                          \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");      \
        __builtin_amdgcn_sched_barrier(0);                                              \
        if ((q) == 0 && (A).stamps) (A).stamps[16 * (pi) + (k)] = t_;                   \
    } while (0)
// sub-phases of PDIP iteration 2 into stamps[16 * pi + 8 + k] (Solver::dbg); with
// DCOL_STAMPS_INIT the sub-phases of initialize() instead (DCOL_NSTAMP)
#ifdef DCOL_STAMPS_INIT
#define DCOL_ISTAMP(it, k) \
    do {                   \
    } while (0)
#define DCOL_NSTAMP(k) DCOL_ISTAMP_(2, k)
#else
#define DCOL_ISTAMP(it, k) DCOL_ISTAMP_(it, k)
#define DCOL_NSTAMP(k) \
    do {               \
    } while (0)
#endif
#define DCOL_ISTAMP_(it, k)                                                             \
    do {                                                                                \
        if ((it) == 2 && dbg) {                                                         \
            __builtin_amdgcn_sched_barrier(0);                                          \
            unsigned long long t_;                                                      \
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");  \
            __builtin_amdgcn_sched_barrier(0);                                          \
            dbg[k] = t_;                                                                \
        }                                                                               \
    } while (0)
#else
#define DCOL_STAMP(A, pi, q, k) \
    do {                        \
    } while (0)
#define DCOL_ISTAMP(it, k) \
    do {                   \
    } while (0)
#define DCOL_NSTAMP(k) \
    do {               \
    } while (0)
#endif

// ------------------------------------------------------------------------------------
// primitive frames
// ------------------------------------------------------------------------------------
struct Frame {
    double Qe[9];  // Q(p) * Q_offset
    double re[3];  // r + Q(p) * r_offset
    double qro[3]; // Q(p) * r_offset
};

// dcm_from_mrp, problem_matrices.py:213-251 (same expanded expression)
DCOL_HD void dcm_from_mrp(double p1, double p2, double p3, double Q[9]) {
    const double s = p1 * p1 + p2 * p2 + p3 * p3 + 1.0;
    const double den = s * s;
    const double a = 4.0 * (p1 * p1) + 4.0 * (p2 * p2) + 4.0 * (p3 * p3) - 4.0;
    const double iden = frcp(den);
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

// problem_matrices.py:275-282 (r_eff = r + Q r_offset; Q_eff = Q Q_offset).  With
// identity offsets (S.plain) the products are exact no-ops (q*1 + q'*0 + q''*0 == q,
// r + (+-0) == r) and are skipped: same bits, ~36 fewer instructions per frame.
// plain: S.plain, passed in by a caller that loaded it early (see solve_one)
DCOL_HD void make_frame(const DevShape& S, const double th[6], Frame& F, int32_t plain) {
    double Q[9];
    dcm_from_mrp(th[3], th[4], th[5], Q);
    double qe[9], qr[3];
    if (plain) {
#pragma unroll
        for (int k = 0; k < 9; ++k) qe[k] = Q[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) qr[k] = 0.0;
    } else {
        const double o0 = S.r_off[0], o1 = S.r_off[1], o2 = S.r_off[2];
#pragma unroll
        for (int k = 0; k < 3; ++k) qr[k] = Q[3 * k] * o0 + Q[3 * k + 1] * o1 + Q[3 * k + 2] * o2;
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c)
                qe[3 * r + c] = Q[3 * r] * S.Q_off[c] + Q[3 * r + 1] * S.Q_off[3 + c] + Q[3 * r + 2] * S.Q_off[6 + c];
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) F.Qe[k] = qe[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        F.qro[k] = qr[k];
        F.re[k] = th[k] + qr[k];
    }
}
DCOL_HD void make_frame(const DevShape& S, const double th[6], Frame& F) { make_frame(S, th, F, S.plain); }

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
    const double iden = frcp(s1 * s1);
    const double a = 4.0 * S - 4.0;
    const double K[9] = {0.0, p[2], -p[1], -p[2], 0.0, p[0], p[1], -p[0], 0.0};
    double Nm[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) Nm[3 * r + c] = 8.0 * (p[r] * p[c] - (r == c ? S : 0.0)) + a * K[3 * r + c];
    // K_j = dK/dp_j
    const double Kj[3][9] = {{0, 0, 0, 0, 0, 1, 0, -1, 0}, {0, 0, -1, 0, 0, 0, 1, 0, 0}, {0, 1, 0, -1, 0, 0, 0, 0, 0}};
    const double is1 = frcp(s1);
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
// second-order cone helpers (D-vectors: D = 4 for ball blocks and the padded dense layout,
// D = 3 for cone blocks in the CONE kernels -- the cone's own dimension, no zero padding)
// ------------------------------------------------------------------------------------
// v[1:] . w[1:] and v . w, written as the sums of the D = 4 originals
template <int D>
DCOL_HD double tail_dot(const double* v, const double* w) {
    if constexpr (D == 4) return v[1] * w[1] + v[2] * w[2] + v[3] * w[3];
    else if constexpr (D == 2) return v[1] * w[1];   // (a SPLIT lane's half: the caller completes the sum)
    else return v[1] * w[1] + v[2] * w[2];
}
template <int D>
DCOL_HD double full_dot(const double* v, const double* w) {
    if constexpr (D == 4) return v[0] * w[0] + v[1] * w[1] + v[2] * w[2] + v[3] * w[3];
    else if constexpr (D == 2) return v[0] * w[0] + v[1] * w[1];
    else return v[0] * w[0] + v[1] * w[1] + v[2] * w[2];
}

struct SocNT {
    double w0, w1[3], bf, eta, ieta;
    // soc_linesearch inputs that depend only on the current s (index 0) / z (index 1), shared
    // by the predictor's and the corrector's line search: 1/sqrt(max(J, 1e-25)) and
    // 1/(y_0 / sqrt(nu) + 1)
    double lis[2], lrc[2];
};

// soc_NT_scaling, NT_scaling.py:340-405; W = eta * Wbar,
// Wbar = [[w0, w1'], [w1, I + bf w1 w1']], bf = 1/(w0+1), eta = (J(s)/J(z))^(1/4)
template <int D = 4>
DCOL_HD void soc_nt(const double* s, const double* z, SocNT& W) {
    const double Jz = z[0] * z[0] - tail_dot<D>(z, z);
    const double Js = s[0] * s[0] - tail_dot<D>(s, s);
    const double iz = frsqrt(Jz);
    const double is = frsqrt(Js);
    double zb[D], sb[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
        zb[k] = z[k] * iz;
        sb[k] = s[k] * is;
    }
    const double dot = full_dot<D>(zb, sb);
    const double i2g = 0.5 * frsqrt((1.0 + dot) * 0.5);   // 1/(2 gamma)
    W.w0 = (sb[0] + zb[0]) * i2g;
#pragma unroll
    for (int k = 0; k < 3; ++k) W.w1[k] = (k < D - 1) ? (sb[k + 1] - zb[k + 1]) * i2g : 0.0;
    W.bf = frcp1(W.w0 + 1.0);
#if defined(__HIP_DEVICE_COMPILE__)
    // line-search scalars from the normalisation rsqrts (same J expressions as soc_ls_inv);
    // J below the reference's 1e-25 floor (or NaN) takes 1/sqrt(1e-25)
    W.lis[0] = (Js >= 1e-25) ? is : 3162277660168.3794;
    W.lis[1] = (Jz >= 1e-25) ? iz : 3162277660168.3794;
#else
    W.lis[0] = frsqrt(fmax(Js, 1e-25));
    W.lis[1] = frsqrt(fmax(Jz, 1e-25));
#endif
    W.lrc[0] = frcp1(fma(s[0], W.lis[0], 1.0));
    W.lrc[1] = frcp1(fma(z[0], W.lis[1], 1.0));
#if defined(__HIP_DEVICE_COMPILE__)
    // eta = (J(s)/J(z))^(1/4) = sqrt(u), u = sqrt(J(s)) / sqrt(J(z)) = J(s) is iz from the
    // normalisations above: one reciprocal square root instead of two sqrt sequences and two
    // reciprocals (rounding-level)
    const double u = (Js * is) * iz;
    const double ie = frsqrt(u);
    W.eta = (Jz != 0.0) ? u * ie : 1.0;                     // quirk Q9
    W.ieta = (Jz != 0.0) ? ie : 1.0;
#else
    W.eta = (Jz != 0.0) ? sqrt(sqrt(Js * frcp1(Jz))) : 1.0;   // quirk Q9
    W.ieta = frcp1(W.eta);
#endif
}

// out = W v
template <int D = 4>
DCOL_HD void soc_mul(const SocNT& W, const double* v, double* out) {
    const double d = (D == 4) ? W.w1[0] * v[1] + W.w1[1] * v[2] + W.w1[2] * v[3] : W.w1[0] * v[1] + W.w1[1] * v[2];
    out[0] = W.eta * (W.w0 * v[0] + d);
    const double c = W.bf * d;
#pragma unroll
    for (int k = 0; k < D - 1; ++k) out[k + 1] = W.eta * (v[0] * W.w1[k] + v[k + 1] + c * W.w1[k]);
}

// out = W^-1 v = eta^-1 J Wbar J v   (closed form; replaces cho_solve, NT_scaling.py:109)
template <int D = 4>
DCOL_HD void soc_solve(const SocNT& W, const double* v, double* out) {
    const double d = (D == 4) ? W.w1[0] * v[1] + W.w1[1] * v[2] + W.w1[2] * v[3] : W.w1[0] * v[1] + W.w1[1] * v[2];
    out[0] = W.ieta * (W.w0 * v[0] - d);
    const double c = W.bf * d;
#pragma unroll
    for (int k = 0; k < D - 1; ++k) out[k + 1] = W.ieta * (v[k + 1] - v[0] * W.w1[k] + c * W.w1[k]);
}

// out = W^-2 v = eta^-2 J Wbar^2 J v with Wbar^2 = [[2 w0^2 - 1, 2 w0 w1'], [2 w0 w1, I + 2 w1 w1']]
// (uses w0^2 - |w1|^2 = 1 of the NT point; one pass instead of two soc_solve)
template <int D = 4>
DCOL_HD void soc_w2inv(const SocNT& W, const double* v, double* out) {
    const double d = (D == 4) ? W.w1[0] * v[1] + W.w1[1] * v[2] + W.w1[2] * v[3] : W.w1[0] * v[1] + W.w1[1] * v[2];
    const double e2 = W.ieta * W.ieta;
    const double tw = 2.0 * W.w0;
    out[0] = e2 * ((tw * W.w0 - 1.0) * v[0] - tw * d);
    const double c = 2.0 * d - tw * v[0];
#pragma unroll
    for (int k = 0; k < D - 1; ++k) out[k + 1] = e2 * (v[k + 1] + c * W.w1[k]);
}

// soc_cone_product(u, v), pdip.py:165-200
template <int D = 4>
DCOL_HD void soc_prod(const double* u, const double* v, double* out) {
    const double s = full_dot<D>(u, v);
#pragma unroll
    for (int k = 1; k < D; ++k) out[k] = u[0] * v[k] + v[0] * u[k];
    out[0] = s;
}

// inverse_soc_cone_product(u, w), pdip.py:88-122
template <int D = 4>
DCOL_HD void soc_iprod(const double* u, const double* w, double* out) {
    const double rho = u[0] * u[0] - tail_dot<D>(u, u);
    const double nu = tail_dot<D>(u, w);
    const double irho = frcp1(rho);
    const double iu0 = frcp1(u[0]);
    const double c1 = nu * iu0 - w[0];
    const double c2 = rho * iu0;
    out[0] = irho * (u[0] * w[0] - nu);
#pragma unroll
    for (int k = 1; k < D; ++k) out[k] = irho * (c1 * u[k] + c2 * w[k]);
}

// soc_linesearch, pdip.py:25-52 (quirk Q10: nu floored at 1e-25), in inverse form: returns
// 1 / step bound = max(1, |rho_1| - rho_0) (the reference's min(1, 1/(|rho_1| - rho_0)) if
// |rho_1| > rho_0, else 1), so the caller takes one reciprocal of the combined orthant /
// SOC maximum (bound_inv) instead of one per cone.
// isn = 1/sqrt(nu), rc = 1/(y_0 isn + 1) come precomputed from soc_nt (SocNT::lis, lrc).
template <int D = 4>
DCOL_HD double soc_ls_inv(const double* y, const double* d, double isn, double rc) {
    const double zeta = y[0] * d[0] - tail_dot<D>(y, d);
    const double inu = isn * isn;
    const double rho0 = zeta * inu;
    const double coef = (zeta * isn + d[0]) * rc;
    double n2 = 0.0;
#pragma unroll
    for (int k = 1; k < D; ++k) {
        const double r = d[k] * isn - coef * (y[k] * inu);
        n2 += r * r;
    }
#if defined(__HIP_DEVICE_COMPILE__)
    const double n1 = n2 > 0.0 ? n2 * frsqrt(n2) : 0.0;   // |rho_1| without the sqrt sequence
#else
    const double n1 = sqrt(n2);
#endif
    return fmax(1.0, n1 - rho0);                          // NaN -> 1, as the reference's test
}

// ------------------------------------------------------------------------------------
// lane-group reductions (one pair = LPP consecutive lanes; DPP quad permutations)
// ------------------------------------------------------------------------------------
// Butterflies with commutative adds: every lane of a group ends with the bitwise same
// value, so the replicated scalar part of the method (Cholesky, mu, sigma, step) takes
// identical decisions in every lane of the pair.
#ifdef DCOL_CHECK_EXEC
// Diagnostic build (make check-exec, lib_check/): every DPP read whose source lane is
// inactive is counted -- the only way a reduction could read a register the program never
// wrote ("Codegen invariance").  A counter, not a trap: a trapping
// kernel can take the whole GPU down.
// one counter per translation unit (no relocatable device code): dcol_launch.hpp
// DCOL_EXEC_READER reads it back
static __device__ unsigned long long dcol_exec_violations;
#endif
#if defined(__HIP_DEVICE_COMPILE__)
#ifdef DCOL_CHECK_EXEC
template <int CTRL>
__device__ __forceinline__ void dpp_check() {
    const unsigned lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    unsigned src;
    if (CTRL == 0xB1) src = lane ^ 1u;
    else if (CTRL == 0x4E) src = lane ^ 2u;
    else if (CTRL == 0xA0) src = lane & ~1u;
    else if (CTRL == 0xF5) src = lane | 1u;
    else if (CTRL == 0x141) src = (lane & ~7u) | (7u - (lane & 7u));
    else src = (lane & ~15u) | (15u - (lane & 15u));
    const unsigned long long exec = __builtin_amdgcn_read_exec();
    if (!((exec >> src) & 1ull)) atomicAdd(&dcol_exec_violations, 1ull);
}
#endif
// bound_ctrl = true: a lane whose source lane is out of range or disabled reads 0 instead of
// keeping the destination register's previous (undefined) content, so no schedule can feed
// an unwritten register into a sum.  Every reduction's group is all-active (a pair's lanes
// take identical branches), which the DCOL_CHECK_EXEC build verifies, so the results are the
// same bits either way.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
#ifdef DCOL_CHECK_EXEC
    dpp_check<CTRL>();
#endif
    const long long b = __double_as_longlong(v);
    int lo = (int)(b & 0xffffffffLL), hi = (int)(b >> 32);
    lo = __builtin_amdgcn_mov_dpp(lo, CTRL, 0xF, 0xF, true);
    hi = __builtin_amdgcn_mov_dpp(hi, CTRL, 0xF, 0xF, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
#define DCOL_XOR1(v) dpp_d<0xB1>(v)   // quad_perm [1,0,3,2]
#define DCOL_XOR2(v) dpp_d<0x4E>(v)   // quad_perm [2,3,0,1]
#define DCOL_HMIR(v) dpp_d<0x141>(v)  // row_half_mirror: lane i <-> 7-i within 8 lanes
#define DCOL_RMIR(v) dpp_d<0x140>(v)  // row_mirror: lane i <-> 15-i within 16 lanes
#define DCOL_BC0(v) dpp_d<0xA0>(v)    // quad_perm [0,0,2,2]: a lane pair's first lane to both
#define DCOL_BC1(v) dpp_d<0xF5>(v)    // quad_perm [1,1,3,3]: its second lane to both
#else
#define DCOL_XOR1(v) (__builtin_trap(), (v))   // multi-lane groups run on the GPU only
#define DCOL_XOR2(v) (__builtin_trap(), (v))
#define DCOL_HMIR(v) (__builtin_trap(), (v))
#define DCOL_RMIR(v) (__builtin_trap(), (v))
#define DCOL_BC0(v) (__builtin_trap(), (v))
#define DCOL_BC1(v) (__builtin_trap(), (v))
#endif

template <int LPP>
struct Grp;
template <>
struct Grp<1> {
    DCOL_HD static double sum(double v) { return v; }
    DCOL_HD static double min(double v) { return v; }
    DCOL_HD static double max(double v) { return v; }
};
template <>
struct Grp<2> {
    DCOL_HD static double sum(double v) { return v + DCOL_XOR1(v); }
    DCOL_HD static double min(double v) { return fmin(v, DCOL_XOR1(v)); }
    DCOL_HD static double max(double v) { return fmax(v, DCOL_XOR1(v)); }
};
template <>
struct Grp<8> {
    // after the two quad steps every lane holds its quad's value; the half-row mirror pairs
    // each lane with one of the other quad
    DCOL_HD static double sum(double v) {
        v = v + DCOL_XOR1(v);
        v = v + DCOL_XOR2(v);
        return v + DCOL_HMIR(v);
    }
    DCOL_HD static double min(double v) {
        v = fmin(v, DCOL_XOR1(v));
        v = fmin(v, DCOL_XOR2(v));
        return fmin(v, DCOL_HMIR(v));
    }
    DCOL_HD static double max(double v) {
        v = fmax(v, DCOL_XOR1(v));
        v = fmax(v, DCOL_XOR2(v));
        return fmax(v, DCOL_HMIR(v));
    }
};
template <>
struct Grp<16> {
    // 8-lane sums as Grp<8>, then the row mirror pairs each lane with one of the other half
    // (the 48-128-row buckets: polytopes / polygons with many faces)
    DCOL_HD static double sum(double v) {
        v = v + DCOL_XOR1(v);
        v = v + DCOL_XOR2(v);
        v = v + DCOL_HMIR(v);
        return v + DCOL_RMIR(v);
    }
    DCOL_HD static double min(double v) {
        v = fmin(v, DCOL_XOR1(v));
        v = fmin(v, DCOL_XOR2(v));
        v = fmin(v, DCOL_HMIR(v));
        return fmin(v, DCOL_RMIR(v));
    }
    DCOL_HD static double max(double v) {
        v = fmax(v, DCOL_XOR1(v));
        v = fmax(v, DCOL_XOR2(v));
        v = fmax(v, DCOL_HMIR(v));
        return fmax(v, DCOL_RMIR(v));
    }
};
template <>
struct Grp<4> {
    DCOL_HD static double sum(double v) {
        v = v + DCOL_XOR1(v);
        return v + DCOL_XOR2(v);
    }
    DCOL_HD static double min(double v) {
        v = fmin(v, DCOL_XOR1(v));
        return fmin(v, DCOL_XOR2(v));
    }
    DCOL_HD static double max(double v) {
        v = fmax(v, DCOL_XOR1(v));
        return fmax(v, DCOL_XOR2(v));
    }
};

// ------------------------------------------------------------------------------------
// the per-pair solver
// ------------------------------------------------------------------------------------
// A pair's rows are spread over LPP lanes: orthant row i lives in lane i % LPP, slot
// i / LPP; SOC block b lives in lane b % LPP, SOC slot b / LPP.  Per-row work is lane
// local; sums over rows are group all-reduces; the n x n part (normal matrix Cholesky and
// triangular solves, step lengths) is replicated in every lane of the group.
//
// Rounding-level reformulations relative to the reference (none changes the algorithm):
//  * orthant NT scaling from lambda = sqrt(s z): w = s/lambda, w^-1 = z/lambda and
//    lambda\v = v/lambda share ONE reciprocal per row per iteration;
//    lambda o lambda = s z;
//  * the primal residual r = G x - h is carried incrementally (r += a G dx);
//  * orthant ratio tests as a running max of -d/x through the row reciprocals (bound_inv);
//  * G~ = W^-1 G is never formed: G~'G~ and G~'v accumulate G'(W^-1 ...).
//
// BALL: every SOC block of the launch is a ball block (sphere / capsule / cylinder /
// polygon; no cone -- the host buckets such pairs separately).  A ball block's rows are
// [0 0 0 -R | 0] and [-e_k | 0 | X_k] (k = 0..2, X = the primitive's extra columns
// Qe[:, 0..nx)), problem_matrices.py:21-28, 66-76, 112-119, 165-176, so only (R, X) are
// held -- scaled by sv = 1 (real block) / 0 (inert slot) -- and every product with the
// block is written out with its zeros dropped (same nonzero terms in the same order as the
// dense rows).  Frees 4N doubles of registers per SOC slot.
//
// Row partition (OE > 0, "PART" kernels; N = 5 / 6 pairs of combine cases 1-3, where exactly
// one primitive has extra columns): every orthant row is either a pose row [Qe a, g3, 0..]
// (polytope faces, the cone base, cylinder caps) or an extra-column row [0 0 0, g3, ex]
// (capsule / cylinder segment rows, polygon edges), problem_matrices.py:4-120, :181-209.
// The lane's first PL = (OMAX - OE) / LPP slots hold pose rows (both primitives', prim 1's
// first), the last EL = OE / LPP slots the extra-column rows, so each slot's column pattern
// is known at compile time and every product skips the structural zeros: a row's normal-
// matrix update is 10 (pose) or 6 (extra) FMAs instead of 21 for N = 6, its G'v / G v terms
// 4 or 3 instead of 6, and it holds 4 or 3 doubles of G instead of 6.  The rows' reference
// order within a pair changes, i.e. the lane sums add the same terms in another order
// (rounding level); parity is pinned by iteration-count equality on every golden vector.
// SPLIT (round 6): the one ball SOC block of an NSOC = 1 pair at LPP 2
// split over the pair's two lanes -- lane q holds the block's coordinates 2q, 2q + 1 (its s,
// z, r and every per-coordinate product), instead of the whole block in lane 0 while lane 1
// idles through the SOC work.  The block's scalars (J(s), J(z), w'v, the line-search sums)
// are partial sums over a lane's coordinates completed by one DPP exchange (R::sum); the
// head coordinate's value reaches lane 1 by one more (bc0); the NT point w is held whole in
// both lanes.  The structured ball rows (R, X) are replicated; the block's share of the
// normal matrix and of G'G in initialize() is taken in lane 0 (lane 1 adds zeros), G_b'v per
// coordinate in its own lane (the group sum adds them).  Rounding-level against the one-lane
// block (sums in another order); pinned by iteration-count equality against the C oracle.
template <int N, int NSOC, int OMAX, int LPP, bool BALL = false, bool CONE = false, int OE = 0, bool GLDS = false,
          bool BOX = false, bool SPLIT = false>
struct Solver {
    static_assert(!SPLIT || (BALL && NSOC == 1 && LPP == 2 && !GLDS && !BOX), "SPLIT: one ball block over two lanes");
    static_assert(OMAX % LPP == 0, "OMAX must be a multiple of LPP");
    static_assert(!(BALL && CONE) && (!CONE || N == 4), "CONE: cone-only SOC blocks of N = 4 pairs");
    static_assert(OE % LPP == 0 && OE <= OMAX && (OE == 0 || (N == 5 || N == 6)), "PART: N = 5 / 6, OE % LPP == 0");
    static constexpr bool PART = OE > 0;
    // BOX: both primitives are boxes (DevShape::boxp) and every slot holds a row (FULL).  A
    // lane's slots hold whole AXIS PAIRS: slots 2m, 2m + 1 = rows a, a + 3 of one primitive,
    // G = [u, g3] and [-u, g3'] with u = Qe a_a, so the pair's products share u: the normal
    // matrix takes (d + d') u u' + (d g3 - d' g3') u + (d g3^2 + d' g3'^2) e3 e3' instead of two
    // rank-one updates, G'v takes (t - t') u, a row product u.v is formed once for both rows,
    // and -u is never stored.  Axis pair t = m * LPP + q: t < 3 primitive 1's axis t, else
    // primitive 2's axis t - 3.  The reassociated sums are rounding-level (parity: iteration
    // counts and values against the oracle on every golden and every pair of the 100k set).
    static_assert(!BOX || (N == 4 && NSOC == 0 && !PART && (OMAX / LPP) % 2 == 0 && OMAX == 12),
                  "BOX: box x box pairs, whole axis pairs per lane");
    static constexpr int OR = OMAX / LPP;              // orthant slots per lane
    static constexpr int EL = OE / LPP;                // PART: extra-column slots per lane (the last EL)
    static constexpr int PL = OR - EL;                 // PART: pose slots per lane (the first PL)
    static constexpr int SS = (NSOC + LPP - 1) / LPP;  // SOC slots per lane
    static constexpr int SD = CONE ? 3 : (SPLIT ? 2 : 4);   // rows per SOC slot (cones unpadded in CONE;
                                                            // SPLIT: this lane's half of the block)
    static constexpr int M = OR + SD * SS;             // lane-local rows
    static constexpr int SSA = SS > 0 ? SS : 1;
    static constexpr int MG = (BALL || CONE) ? OR : M; // rows held densely in G
    static constexpr int NX = N - 4;                   // extra primal columns
    static constexpr int NXA = NX > 0 ? NX : 1;
    using R = Grp<LPP>;

    // GLDS ("LDS rows", variants.py): G and the CONE rows live in this lane's column of a
    // per-workgroup LDS array instead of registers -- they are constant through the PDIP loop
    // and read a few times per iteration -- so the kernel fits fewer VGPRs (no AGPR parking,
    // two waves per SIMD for the one-lane cone x polytope kernel).  Compact layout (gidx):
    // a PART pose slot stores columns 0..3, an extra-column slot columns 3..N-1, any other row
    // all N; the CONE rows follow (10 per slot).  The LDS pointer is laundered at the PDIP
    // phase boundaries (grefresh), so no load is hoisted out of its phase and held in
    // registers across the loop (which would undo the point).  Same arithmetic in the same
    // order as the register form: bitwise equal results (the codegen-invariance twin is built
    // without LDS rows, tests/test_gpu_fullsize.py).
#if defined(__HIP_DEVICE_COMPILE__)
    using lds_d = __attribute__((address_space(3))) double;
#else
    using lds_d = double;
#endif
    DCOL_HD static constexpr int gidx(int k, int j) {
        if constexpr (PART) {
            if (k < PL) return 4 * k + j;
            if (k < OR) return 4 * PL + (N - 3) * (k - PL) + (j - 3);
            return 4 * PL + (N - 3) * EL + N * (k - OR) + j;
        }
        return N * k + j;
    }
    static constexpr int GW = PART ? 4 * PL + (N - 3) * EL + N * (MG - OR) : MG * N;   // doubles of G
    static constexpr int LDSW = GW + (CONE ? 10 * SSA : 0);   // doubles per lane in LDS (GLDS)
    static constexpr int kLdsStride = 64;                     // lanes per workgroup (kSolveBlock)
    double G[GLDS ? 1 : MG][N];
    double sv[SSA], sR[SSA], sX[SSA][3][NXA];   // BALL: structured SOC rows (see above)
    double cq[GLDS ? 1 : SSA][3][3], cc0[GLDS ? 1 : SSA];   // CONE: row e of slot b = [cq[b][e] | e == 0 ? cc0[b] : 0]
    mutable lds_d* gb = nullptr;                // GLDS: this lane's first element
    DCOL_HD decltype(auto) gx(int k, int j) const {
        if constexpr (GLDS) return (gb[gidx(k, j) * kLdsStride]);
        else return (G[k][j]);
    }
    DCOL_HD decltype(auto) gx(int k, int j) {
        if constexpr (GLDS) return (gb[gidx(k, j) * kLdsStride]);
        else return (G[k][j]);
    }
    DCOL_HD decltype(auto) cqx(int b, int e, int c) const {
        if constexpr (GLDS) return (gb[(GW + 10 * b + 3 * e + c) * kLdsStride]);
        else return (cq[b][e][c]);
    }
    DCOL_HD decltype(auto) cqx(int b, int e, int c) {
        if constexpr (GLDS) return (gb[(GW + 10 * b + 3 * e + c) * kLdsStride]);
        else return (cq[b][e][c]);
    }
    DCOL_HD decltype(auto) ccx(int b) const {
        if constexpr (GLDS) return (gb[(GW + 10 * b + 9) * kLdsStride]);
        else return (cc0[b]);
    }
    DCOL_HD decltype(auto) ccx(int b) {
        if constexpr (GLDS) return (gb[(GW + 10 * b + 9) * kLdsStride]);
        else return (cc0[b]);
    }
    DCOL_HD void grefresh() const {
#if defined(__HIP_DEVICE_COMPILE__)
        if constexpr (GLDS) asm volatile("" : "+v"(gb));
#endif
    }
    // G entry (k, j) by value: BOX slot 2m + 1 holds only column 3 (its columns 0..2 are the
    // exact negatives of slot 2m's)
    DCOL_HD double gr(int k, int j) const {
        if constexpr (BOX) {
            if ((k & 1) && j < 3) return -static_cast<double>(gx(k - 1, j));
        }
        return gx(k, j);
    }
    // BOX: u.v of axis pair m (the same expression for both rows: one evaluation after CSE)
    DCOL_HD double qdot(int m, const double* v) const {
        double acc = gr(2 * m, 0) * v[0];
        acc += gr(2 * m, 1) * v[1];
        acc += gr(2 * m, 2) * v[2];
        return acc;
    }
    DCOL_HD int box_prim(int m) const { return m * LPP + q >= 3 ? 1 : 0; }   // BOX: primitive of axis pair m
    double s[M], z[M], r[M];   // slack, dual, primal residual G x - h
    double x[N];
    double vimp[N];            // implicit-gradient mode: H^-1 e3 at the returned iterate
    int q, o1, o, deg;
    int op1, op, oe;           // PART: pose rows of prim 1 / of the pair, extra-column rows
    int xo2;                   // first extra column of primitive 2 minus 4: S1.n_extra for a
                               // case-4 pair (both primitives have extras; opt-in extension),
                               // else 0 (combine_problem_matrices.py cases 1-3)
    bool vs[SSA];              // SOC slot holds a real block
#ifdef DCOL_STAMPS
    unsigned long long* dbg = nullptr;
#endif
    int soc_owner[SSA];        // primitive (0/1) owning the block in SOC slot b

    DCOL_HD bool vort(int k) const {
        if constexpr (PART) return k < PL ? (k * LPP + q < op) : ((k - PL) * LPP + q < oe);
        return k * LPP + q < o;
    }
    // column j of lane row k can be nonzero (compile-time after unrolling): the PART slots'
    // column patterns; every column of every other row
    DCOL_HD static constexpr bool nz(int k, int j) {
        return !PART || k >= OR || (k < PL ? j < 4 : j >= 3);
    }
    // column offset of a primitive's extra columns (static 0 unless N >= 6 can be case 4)
    DCOL_HD int xoff(bool p2) const { return (N >= 6 && p2) ? xo2 : 0; }
    // value of column j >= 4 of a row whose primitive puts (e0, e1) at columns 4+off, 5+off
    DCOL_HD static double excol(int j, int off, double e0, double e1) {
        const int t = j - 4 - off;
        return t == 0 ? e0 : (t == 1 ? e1 : 0.0);
    }
    DCOL_HD bool vrow(int k) const { return k < OR ? vort(k) : vs[(k - OR) / SD]; }

    // -------- assembly (problem_matrices.py + combine_problem_matrices.py) --------------
    // One orthant slot: row i = k * LPP + q of primitive p2 (frame F) -> G[k], h in r[k].
    // A slot without a row (v false) reads the pool's zero row 0 (dcol_host.hpp
    // init_row_pool) instead of skipping its loads: a load under a per-slot branch waits for
    // its data before the branch joins, which serialised the slots' L2 round trips.
    DCOL_HD void orth_row(const double* __restrict__ rows, int k, bool v, bool p2, int ri, const Frame& F) {
        const double2* rw = reinterpret_cast<const double2*>(rows + 8 * (int64_t)(v ? ri : 0));
        const double2 q0 = rw[0], q1 = rw[1], q2 = rw[2];
        const double a0 = q0.x, a1 = q0.y, a2 = q1.x, g3 = q1.y, e0 = q2.x, e1 = q2.y;
        const double u0 = F.Qe[0] * a0 + F.Qe[1] * a1 + F.Qe[2] * a2;
        const double u1 = F.Qe[3] * a0 + F.Qe[4] * a1 + F.Qe[5] * a2;
        const double u2 = F.Qe[6] * a0 + F.Qe[7] * a1 + F.Qe[8] * a2;
        gx(k, 0) = u0; gx(k, 1) = u1; gx(k, 2) = u2; gx(k, 3) = g3;
        const int off = xoff(p2);
#pragma unroll
        for (int j = 4; j < N; ++j)
            if (nz(k, j)) gx(k, j) = excol(j, off, e0, e1);
        r[k] = u0 * F.re[0] + u1 * F.re[1] + u2 * F.re[2];
    }
    // PART: one extra-column slot (pose-independent row [0 0 0, g3, ex], h = 0)
    DCOL_HD void ext_row(const double* __restrict__ rows, int k, bool v, int ri) {
        const double2* rw = reinterpret_cast<const double2*>(rows + 8 * (int64_t)(v ? ri : 0));
        const double2 q1 = rw[1], q2 = rw[2];
        const double g3 = q1.y, e0 = q2.x, e1 = q2.y;
        gx(k, 3) = g3;
#pragma unroll
        for (int j = 4; j < N; ++j) gx(k, j) = excol(j, 0, e0, e1);
        r[k] = 0.0;
    }
    // leaves h in r[] (init turns it into G x_hat - h)
    DCOL_HD void assemble(const KArgs& A, const DevShape& S1, const DevShape& S2, const Frame& F1, const Frame& F2) {
        o1 = S1.n_ort;
        o = o1 + S2.n_ort;
        xo2 = (N >= 6 && S1.n_extra > 0 && S2.n_extra > 0) ? S1.n_extra : 0;
        deg = o + NSOC;                                   // quirk Q7
        const double* __restrict__ rows = reinterpret_cast<const double*>(A.rows);
        if constexpr (PART) {
            // pose rows of prim 1 then prim 2 in the pose slots (each primitive's pose rows
            // follow its extra-column rows in the pool); the extra-column rows of the one
            // primitive that has them in the extra slots
            op1 = S1.n_p;
            op = op1 + S2.n_p;
            oe = o - op;
            const int eb = S2.n_extra > 0 ? S2.row_off : S1.row_off;
#pragma unroll
            for (int k = 0; k < PL; ++k) {
                const int i = k * LPP + q;
                const bool p2 = i >= op1;
                Frame F;
#pragma unroll
                for (int c = 0; c < 9; ++c) F.Qe[c] = p2 ? F2.Qe[c] : F1.Qe[c];
#pragma unroll
                for (int c = 0; c < 3; ++c) F.re[c] = p2 ? F2.re[c] : F1.re[c];
                const int ri = p2 ? (S2.row_off + (S2.n_ort - S2.n_p) + (i - op1)) : (S1.row_off + (S1.n_ort - S1.n_p) + i);
                orth_row(rows, k, i < op, p2, ri, F);
            }
#pragma unroll
            for (int k = PL; k < OR; ++k) {
                const int i = (k - PL) * LPP + q;
                ext_row(rows, k, i < oe, eb + i);
            }
        } else if constexpr (BOX) {
            // axis pair m of this lane: rows a, a + 3 of one primitive (see BOX above); the
            // second row's u and h are the exact negatives of the first's, only its g3 is loaded
#pragma unroll
            for (int m = 0; m < OR / 2; ++m) {
                const int t = m * LPP + q;
                const bool p2 = t >= 3;
                const int a = p2 ? t - 3 : t;
                Frame F;
#pragma unroll
                for (int c = 0; c < 9; ++c) F.Qe[c] = p2 ? F2.Qe[c] : F1.Qe[c];
#pragma unroll
                for (int c = 0; c < 3; ++c) F.re[c] = p2 ? F2.re[c] : F1.re[c];
                const int ri = (p2 ? S2.row_off : S1.row_off) + a;
                orth_row(rows, 2 * m, true, p2, ri, F);
                gx(2 * m + 1, 3) = rows[8 * (int64_t)(ri + 3) + 3];   // DevRow g3
                r[2 * m + 1] = -r[2 * m];
            }
        } else {
#pragma unroll
            for (int k = 0; k < OR; ++k) {
                const int i = k * LPP + q;
                const bool v = i < o;
                const bool p2 = i >= o1;
                Frame F;   // element-wise select of the row's frame
#pragma unroll
                for (int c = 0; c < 9; ++c) F.Qe[c] = p2 ? F2.Qe[c] : F1.Qe[c];
#pragma unroll
                for (int c = 0; c < 3; ++c) F.re[c] = p2 ? F2.re[c] : F1.re[c];
                orth_row(rows, k, v, p2, p2 ? (S2.row_off + (i - o1)) : (S1.row_off + i), F);
            }
        }
        // global SOC block 0 = first primitive with a SOC, block 1 = prim 2 when both have one
        const int own0 = S1.soc_kind != SOC_NONE ? 0 : 1;
#pragma unroll
        for (int b = 0; b < SS; ++b) {
            const int gb = SPLIT ? 0 : b * LPP + q;   // SPLIT: both lanes hold (half of) block 0
            vs[b] = gb < NSOC;
            const bool p2 = (gb == 0) ? (own0 == 1) : true;
            soc_owner[b] = p2 ? 1 : 0;
            double Qe[9], re[3];
#pragma unroll
            for (int c = 0; c < 9; ++c) Qe[c] = p2 ? F2.Qe[c] : F1.Qe[c];
#pragma unroll
            for (int c = 0; c < 3; ++c) re[c] = p2 ? F2.re[c] : F1.re[c];
            const int kind = vs[b] ? (p2 ? S2.soc_kind : S1.soc_kind) : SOC_NONE;
            if constexpr (BALL) {
                const double one = vs[b] ? 1.0 : 0.0;
                const int nx = p2 ? S2.n_extra : S1.n_extra;
                const int off = xoff(p2);
                sv[b] = one;
                sR[b] = vs[b] ? (p2 ? S2.R : S1.R) : 0.0;
                if constexpr (!SPLIT) r[OR + SD * b] = 0.0;
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const double c0 = (nx >= 1) ? Qe[3 * k] : 0.0, c1 = (nx >= 2) ? Qe[3 * k + 1] : 0.0;
#pragma unroll
                    for (int j = 4; j < N; ++j) sX[b][k][j - 4] = one * excol(j, off, c0, c1);
                    if constexpr (!SPLIT) r[OR + SD * b + 1 + k] = vs[b] ? -re[k] : 0.0;
                }
                if constexpr (SPLIT) {   // h of this lane's coordinates: 0 for the head, -re[c - 1]
                    r[OR] = q ? -re[1] : 0.0;
                    r[OR + 1] = q ? -re[2] : -re[0];
                }
            } else if constexpr (CONE) {
                // cone block, problem_matrices.py:138-145: rows -E Qe' (E = diag(tanb, 1, 1)),
                // row 0 column 3 cc = -(tanb 3H/4), h = -E Qe' re; the same products as
                // soc_rows; an inert slot holds zero rows
                const double tb = p2 ? S2.tanb : S1.tanb;
                ccx(b) = vs[b] ? (p2 ? S2.cone_c : S1.cone_c) : 0.0;
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const double e = (k == 0) ? tb : 1.0;
                    const double u0 = -(e * Qe[0 + k]);
                    const double u1 = -(e * Qe[3 + k]);
                    const double u2 = -(e * Qe[6 + k]);
                    cqx(b, k, 0) = vs[b] ? u0 : 0.0;
                    cqx(b, k, 1) = vs[b] ? u1 : 0.0;
                    cqx(b, k, 2) = vs[b] ? u2 : 0.0;
                    r[OR + SD * b + k] = vs[b] ? u0 * re[0] + u1 * re[1] + u2 * re[2] : 0.0;
                }
                (void)kind;
            } else {
                double Gb[4][N];
                soc_rows(kind, p2 ? S2.R : S1.R, p2 ? S2.cone_c : S1.cone_c, p2 ? S2.tanb : S1.tanb,
                         p2 ? S2.n_extra : S1.n_extra, xoff(p2), Qe, re, Gb, &r[OR + SD * b]);
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int j = 0; j < N; ++j) gx(OR + SD * b + e, j) = Gb[e][j];
            }
        }
    }

    // The 4 rows of one SOC block (kind SOC_NONE -> inert zero block).  Ball (sphere/
    // capsule/cylinder/polygon): [0 0 0 -R | 0..], h 0;  [-e_k | 0 | Qe[k][0..nx)], h -re[k]
    //   (problem_matrices.py:21-28, 66-76, 112-119, 165-176)
    // Cone: [-E Qe' | -(tanb 3H/4) e_0], h = -E Qe' re; 4th row zero  (problem_matrices.py:138-145)
    DCOL_HD static void soc_rows(int kind, double R, double cc, double tb, int nx, int off, const double* Qe,
                                 const double* re, double (*Gb)[N], double* hb) {
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
        } else if (kind == SOC_BALL) {
            Gb[0][0] = 0.0; Gb[0][1] = 0.0; Gb[0][2] = 0.0; Gb[0][3] = -R;
#pragma unroll
            for (int j = 4; j < N; ++j) Gb[0][j] = 0.0;
            hb[0] = 0.0;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
#pragma unroll
                for (int j = 0; j < 3; ++j) Gb[k + 1][j] = (j == k) ? -1.0 : 0.0;
                Gb[k + 1][3] = 0.0;
                const double c0 = (nx >= 1) ? Qe[3 * k] : 0.0, c1 = (nx >= 2) ? Qe[3 * k + 1] : 0.0;
#pragma unroll
                for (int j = 4; j < N; ++j) Gb[k + 1][j] = excol(j, off, c0, c1);
                hb[k + 1] = -re[k];
            }
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
#pragma unroll
                for (int j = 0; j < N; ++j) Gb[k][j] = 0.0;
                hb[k] = 0.0;
            }
        }
    }

    // -------- SOC block arithmetic (NT_scaling.py:340-463, pdip.py:25-200): the SD-row
    // templates, or under SPLIT this lane's two coordinates c = 2q, 2q + 1 of the one block --
    // lane 0's value of x in both lanes (the head coordinate: lane 0's local slot 0)
    DCOL_HD double bc0(double x) const {
        if constexpr (LPP == 2) return DCOL_BC0(x);
        return x;
    }
    // sums over the block of v_c w_c: the tail (c >= 1) / every coordinate
    DCOL_HD double sp_tail(const double* v, const double* w) const {
        return R::sum(q ? fma(v[0], w[0], v[1] * w[1]) : v[1] * w[1]);
    }
    DCOL_HD double sp_full(const double* v, const double* w) const { return R::sum(fma(v[0], w[0], v[1] * w[1])); }
    // w1 at this lane's local slot e (W whole in both lanes; slot 0 of lane 0 is the head)
    DCOL_HD double wloc(const SocNT& W, int e) const {
        return e == 0 ? (q ? W.w1[1] : W.w0) : (q ? W.w1[2] : W.w1[0]);
    }
    DCOL_HD double wtail(const SocNT& W, const double* v) const {   // w1'v1 over the block
        return R::sum(q ? fma(W.w1[1], v[0], W.w1[2] * v[1]) : W.w1[0] * v[1]);
    }
    DCOL_HD void nt(const double* sl, const double* zl, SocNT& W) const {
        if constexpr (!SPLIT) {
            soc_nt<SD>(sl, zl, W);
        } else {
            const double z0 = bc0(zl[0]), s0 = bc0(sl[0]);
            const double Jz = z0 * z0 - sp_tail(zl, zl);
            const double Js = s0 * s0 - sp_tail(sl, sl);
            const double iz = frsqrt(Jz);
            const double is = frsqrt(Js);
            double zb[2], sb[2];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                zb[k] = zl[k] * iz;
                sb[k] = sl[k] * is;
            }
            const double dot = sp_full(zb, sb);
            const double i2g = 0.5 * frsqrt((1.0 + dot) * 0.5);   // 1/(2 gamma)
            const double wl0 = (q ? sb[0] - zb[0] : sb[0] + zb[0]) * i2g, wl1 = (sb[1] - zb[1]) * i2g;
            W.w0 = DCOL_BC0(wl0);   // w whole in both lanes: coordinates 0, 1 from lane 0, 2, 3 from lane 1
            W.w1[0] = DCOL_BC0(wl1);
            W.w1[1] = DCOL_BC1(wl0);
            W.w1[2] = DCOL_BC1(wl1);
            W.bf = frcp1(W.w0 + 1.0);
#if defined(__HIP_DEVICE_COMPILE__)
            W.lis[0] = (Js >= 1e-25) ? is : 3162277660168.3794;
            W.lis[1] = (Jz >= 1e-25) ? iz : 3162277660168.3794;
            const double u = (Js * is) * iz;
            const double ie = frsqrt(u);
            W.eta = (Jz != 0.0) ? u * ie : 1.0;                     // quirk Q9
            W.ieta = (Jz != 0.0) ? ie : 1.0;
#else
            W.lis[0] = frsqrt(fmax(Js, 1e-25));
            W.lis[1] = frsqrt(fmax(Jz, 1e-25));
            W.eta = (Jz != 0.0) ? sqrt(sqrt(Js * frcp1(Jz))) : 1.0;
            W.ieta = frcp1(W.eta);
#endif
            W.lrc[0] = frcp1(fma(s0, W.lis[0], 1.0));
            W.lrc[1] = frcp1(fma(z0, W.lis[1], 1.0));
        }
    }
    DCOL_HD void wmul(const SocNT& W, const double* v, double* out) const {   // W v
        if constexpr (!SPLIT) {
            soc_mul<SD>(W, v, out);
        } else {
            const double d = wtail(W, v), v0 = bc0(v[0]);
            const double c = W.bf * d;
            const double w = wloc(W, 0), w1 = wloc(W, 1);
            out[0] = q ? W.eta * (v0 * w + v[0] + c * w) : W.eta * (W.w0 * v0 + d);
            out[1] = W.eta * (v0 * w1 + v[1] + c * w1);
        }
    }
    DCOL_HD void wsolve(const SocNT& W, const double* v, double* out) const {   // W^-1 v
        if constexpr (!SPLIT) {
            soc_solve<SD>(W, v, out);
        } else {
            const double d = wtail(W, v), v0 = bc0(v[0]);
            const double c = W.bf * d;
            const double w = wloc(W, 0), w1 = wloc(W, 1);
            out[0] = q ? W.ieta * (v[0] - v0 * w + c * w) : W.ieta * (W.w0 * v0 - d);
            out[1] = W.ieta * (v[1] - v0 * w1 + c * w1);
        }
    }
    DCOL_HD void w2inv(const SocNT& W, const double* v, double* out) const {   // W^-2 v
        if constexpr (!SPLIT) {
            soc_w2inv<SD>(W, v, out);
        } else {
            const double d = wtail(W, v), v0 = bc0(v[0]);
            const double e2 = W.ieta * W.ieta;
            const double tw = 2.0 * W.w0;
            const double c = 2.0 * d - tw * v0;
            out[0] = q ? e2 * (v[0] + c * wloc(W, 0)) : e2 * ((tw * W.w0 - 1.0) * v0 - tw * d);
            out[1] = e2 * (v[1] + c * wloc(W, 1));
        }
    }
    DCOL_HD void cprod(const double* u, const double* v, double* out) const {   // u o v
        if constexpr (!SPLIT) {
            soc_prod<SD>(u, v, out);
        } else {
            const double sd = sp_full(u, v), u0 = bc0(u[0]), v0 = bc0(v[0]);
            out[0] = q ? u0 * v[0] + v0 * u[0] : sd;
            out[1] = u0 * v[1] + v0 * u[1];
        }
    }
    DCOL_HD void ciprod(const double* u, const double* w, double* out) const {   // u \ w
        if constexpr (!SPLIT) {
            soc_iprod<SD>(u, w, out);
        } else {
            const double u0 = bc0(u[0]), w0 = bc0(w[0]);
            const double rho = u0 * u0 - sp_tail(u, u);
            const double nu = sp_tail(u, w);
            const double irho = frcp1(rho);
            const double iu0 = frcp1(u0);
            const double c1 = nu * iu0 - w0;
            const double c2 = rho * iu0;
            out[0] = q ? irho * (c1 * u[0] + c2 * w[0]) : irho * (u0 * w0 - nu);
            out[1] = irho * (c1 * u[1] + c2 * w[1]);
        }
    }
    DCOL_HD double lsinv(const double* y, const double* d, double isn, double rc) const {   // soc_ls_inv
        if constexpr (!SPLIT) {
            return soc_ls_inv<SD>(y, d, isn, rc);
        } else {
            const double y0 = bc0(y[0]), d0 = bc0(d[0]);
            const double zeta = y0 * d0 - sp_tail(y, d);
            const double inu = isn * isn;
            const double rho0 = zeta * inu;
            const double coef = (zeta * isn + d0) * rc;
            const double r0 = d[0] * isn - coef * (y[0] * inu);
            const double r1 = d[1] * isn - coef * (y[1] * inu);
            const double n2 = R::sum(q ? fma(r0, r0, r1 * r1) : r1 * r1);
#if defined(__HIP_DEVICE_COMPILE__)
            const double n1 = n2 > 0.0 ? n2 * frsqrt(n2) : 0.0;
#else
            const double n1 = sqrt(n2);
#endif
            return fmax(1.0, n1 - rho0);
        }
    }

    // -------- small dense helpers ------------------------------------------------------
    DCOL_HD double rowdot(int k, const double* v) const {
        if constexpr (BOX)
            if (k < OR) {   // u.v shared by the pair's two rows (CSE)
                const double uv = qdot(k / 2, v);
                return fma(gr(k, 3), v[3], (k & 1) ? -uv : uv);
            }
        if constexpr (BALL)
            if (k >= OR) return ball_row(k, v);
        if constexpr (CONE)
            if (k >= OR) return cone_row(k, v);
        if constexpr (PART)
            if (k < OR) {   // the slot's structural nonzeros only
                const int j0 = k < PL ? 0 : 3, j1 = k < PL ? 4 : N;
                double acc = gr(k, j0) * v[j0];
#pragma unroll
                for (int j = j0 + 1; j < j1; ++j) acc += gr(k, j) * v[j];
                return acc;
            }
        double acc = gr(k, 0) * v[0];
#pragma unroll
        for (int j = 1; j < N; ++j) acc += gr(k, j) * v[j];
        return acc;
    }
    // BALL: row e of SOC slot b times v
    DCOL_HD double ball_row(int k, const double* v) const {
        if constexpr (SPLIT) {   // this lane's coordinate c = 2q + e: c = 0 the head row, else [-e_(c-1) | 0 | X_(c-1)]
            const int e = k - OR;
            if (e == 0) {
                const double a = q ? v[1] : v[3];
                double acc = fma(q ? -sv[0] : -sR[0], a, 0.0);
#pragma unroll
                for (int i = 0; i < NX; ++i) acc = fma(q ? sX[0][1][i] : 0.0, v[4 + i], acc);
                return acc;
            }
            double acc = -sv[0] * (q ? v[2] : v[0]);
#pragma unroll
            for (int i = 0; i < NX; ++i) acc = fma(q ? sX[0][2][i] : sX[0][0][i], v[4 + i], acc);
            return acc;
        }
        const int b = (k - OR) / 4, e = (k - OR) % 4;
        // an fma (as the dense row's last term), not a bare product the optimiser could
        // contract into a consumer differently in different kernels (fused == split bitwise)
        if (e == 0) return fma(-sR[b], v[3], 0.0);
        double acc = -sv[b] * v[e - 1];
#pragma unroll
        for (int i = 0; i < NX; ++i) acc = fma(sX[b][e - 1][i], v[4 + i], acc);
        return acc;
    }
    // CONE: row e of SOC slot b times v (the dense row's nonzero terms, same order)
    DCOL_HD double cone_row(int k, const double* v) const {
        const int b = (k - OR) / SD, e = (k - OR) % SD;
        double acc = cqx(b, e, 0) * v[0];
        acc += cqx(b, e, 1) * v[1];
        acc += cqx(b, e, 2) * v[2];
        if (e == 0) acc += ccx(b) * v[3];
        return acc;
    }
    // out += G_b' v over the rows of SOC slot b (dense or structured)
    DCOL_HD void soc_gtv(int b, const double* v, double* out) const {
        const int k0 = OR + SD * b;
        if constexpr (CONE) {
#pragma unroll
            for (int e = 0; e < 3; ++e) {
#pragma unroll
                for (int j = 0; j < 3; ++j) out[j] += cqx(b, e, j) * v[e];
                if (e == 0) out[3] += ccx(b) * v[0];
            }
        } else if constexpr (SPLIT) {   // this lane's coordinates (c = 2q, 2q + 1); the group sum adds the other's
            const double t0 = v[0], t1 = v[1];
            out[0] = fma(q ? 0.0 : -sv[0], t1, out[0]);
            out[1] = fma(q ? -sv[0] : 0.0, t0, out[1]);
            out[2] = fma(q ? -sv[0] : 0.0, t1, out[2]);
            out[3] = fma(q ? 0.0 : -sR[0], t0, out[3]);
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                out[4 + i] = fma(q ? sX[0][1][i] : 0.0, t0, out[4 + i]);
                out[4 + i] = fma(q ? sX[0][2][i] : sX[0][0][i], t1, out[4 + i]);
            }
        } else if constexpr (BALL) {
#pragma unroll
            for (int j = 0; j < 3; ++j) out[j] = fma(-sv[b], v[j + 1], out[j]);
            out[3] = fma(-sR[b], v[0], out[3]);
#pragma unroll
            for (int i = 0; i < NX; ++i)
#pragma unroll
                for (int k = 0; k < 3; ++k) out[4 + i] = fma(sX[b][k][i], v[k + 1], out[4 + i]);
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int j = 0; j < N; ++j) out[j] += gr(k0 + e, j) * v[e];
        }
    }
    // gt = W^-1 G_b (SD x N), the SOC block of G~ (NT_scaling.py:164-202)
    DCOL_HD void soc_gtilde(int b, const SocNT& W, double (&gt)[SD][N]) const {
        const int k0 = OR + SD * b;
        if constexpr (CONE) {
#pragma unroll
            for (int j = 0; j < N; ++j) {
                double col[3], res[3];
#pragma unroll
                for (int e = 0; e < 3; ++e) col[e] = (j < 3) ? cqx(b, e, j) : (e == 0 ? ccx(b) : 0.0);
                soc_solve<3>(W, col, res);
#pragma unroll
                for (int e = 0; e < 3; ++e) gt[e][j] = res[e];
            }
        } else if constexpr (BALL) {
            // columns 0..2: W^-1 (-e_{j+1}); column 3: W^-1 (-R e_0); extras: W^-1 (0, X_i)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const double d = -(sv[b] * W.w1[j]);
                const double c = W.bf * d;
                gt[0][j] = W.ieta * (-d);
#pragma unroll
                for (int k = 0; k < 3; ++k) gt[k + 1][j] = W.ieta * fma(c, W.w1[k], (k == j) ? -sv[b] : 0.0);
            }
            gt[0][3] = W.ieta * (W.w0 * -sR[b]);
#pragma unroll
            for (int k = 0; k < 3; ++k) gt[k + 1][3] = W.ieta * (sR[b] * W.w1[k]);
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                const double d = W.w1[0] * sX[b][0][i] + W.w1[1] * sX[b][1][i] + W.w1[2] * sX[b][2][i];
                const double c = W.bf * d;
                gt[0][4 + i] = W.ieta * (-d);
#pragma unroll
                for (int k = 0; k < 3; ++k) gt[k + 1][4 + i] = W.ieta * fma(c, W.w1[k], sX[b][k][i]);
            }
        } else {
#pragma unroll
            for (int j = 0; j < N; ++j) {
                double col[4], res[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) col[e] = gr(k0 + e, j);
                soc_solve(W, col, res);
#pragma unroll
                for (int e = 0; e < 4; ++e) gt[e][j] = res[e];
            }
        }
    }
    // Hm += G_b' W^-2 G_b, the SOC block's share of the normal matrix G~'G~ (pdip.py:434).
    // Dense / CONE rows: through G~_b = W^-1 G_b (soc_gtilde).  BALL rows [0 0 0 -R | 0],
    // [-e_k | 0 | X_k]: straight from the entries of M = W^-2 = eta^-2 J Wbar^2 J
    // (M00 = e2 (2 w0^2 - 1), M0k = -2 e2 w0 w1_k, Mkl = e2 (d_kl + 2 w1_k w1_l)), so
    //   H[j][c] = M(j+1,c+1), H[j][3] = R M(0,j+1), H[3][3] = R^2 M00 (j, c < 3),
    //   H[j][4+i] = -(M' X)(j,i), H[3][4+i] = -R (M0' X)(i), H[4+i][4+i2] = X_i' M' X_i2
    // with M' = M(1:,1:) -- the same matrix by fewer products (rounding-level).  An inert slot
    // (sv = R = X = 0) adds zeros.
    DCOL_HD void soc_hadd(int b, const SocNT& W, double (&Hm)[N][N]) const {
        if constexpr (BALL) {
            const double e2 = W.ieta * W.ieta;
            const double tw = 2.0 * W.w0;
            const double m00 = e2 * fma(tw, W.w0, -1.0);
            const double et = e2 * tw;
            double m0[3], mm[3][3];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                m0[k] = -(et * W.w1[k]);
#pragma unroll
                for (int l = k; l < 3; ++l) {
                    mm[k][l] = e2 * fma(2.0 * W.w1[k], W.w1[l], k == l ? 1.0 : 0.0);
                    mm[l][k] = mm[k][l];
                }
            }
            // (SPLIT: the whole block's share in lane 0, zeros from lane 1 -- W is whole in both)
            const double own = (!SPLIT || q == 0) ? 1.0 : 0.0;
            const double v = sv[b] * own, R = sR[b] * own;
#pragma unroll
            for (int j = 0; j < 3; ++j) {
#pragma unroll
                for (int c = j; c < 3; ++c) Hm[j][c] = fma(v, mm[j][c], Hm[j][c]);
                Hm[j][3] = fma(v * R, m0[j], Hm[j][3]);
            }
            Hm[3][3] = fma(R * R, m00, Hm[3][3]);
            if constexpr (NX > 0) {
                double mx[3][NXA], m0x[NXA], X[3][NXA];
#pragma unroll
                for (int k = 0; k < 3; ++k)
#pragma unroll
                    for (int i = 0; i < NX; ++i) X[k][i] = SPLIT ? sX[b][k][i] * own : sX[b][k][i];
#pragma unroll
                for (int i = 0; i < NX; ++i) {
                    m0x[i] = m0[0] * X[0][i] + m0[1] * X[1][i] + m0[2] * X[2][i];
#pragma unroll
                    for (int k = 0; k < 3; ++k)
                        mx[k][i] = mm[k][0] * X[0][i] + mm[k][1] * X[1][i] + mm[k][2] * X[2][i];
                }
#pragma unroll
                for (int i = 0; i < NX; ++i) {
#pragma unroll
                    for (int j = 0; j < 3; ++j) Hm[j][4 + i] = fma(-v, mx[j][i], Hm[j][4 + i]);
                    Hm[3][4 + i] = fma(-R, m0x[i], Hm[3][4 + i]);
#pragma unroll
                    for (int i2 = i; i2 < NX; ++i2)
                        Hm[4 + i][4 + i2] += X[0][i] * mx[0][i2] + X[1][i] * mx[1][i2] + X[2][i] * mx[2][i2];
                }
            }
        } else {
            double gt[SD][N];
            soc_gtilde(b, W, gt);
#pragma unroll
            for (int e = 0; e < SD; ++e)
#pragma unroll
                for (int j = 0; j < N; ++j)
#pragma unroll
                    for (int c = j; c < N; ++c) Hm[j][c] += gt[e][j] * gt[e][c];
        }
    }
    // Factorisation of the normal matrix (scipy.linalg.cholesky / cho_solve, pdip.py:434-436),
    // in one of two forms with the same interface (F: strict upper triangle, idg: per-pivot
    // scale), chosen per kernel at compile time (LDL):
    //  * upper Cholesky H = F_c' F_c: F = F_c, idg = 1 / diag(F_c) (v_rsq_f64 + refinement);
    //  * square-root-free H = U' D U (U unit upper, D = diag(d), d_j = F_c[j][j]^2 -- the
    //    same pivots): F = U, idg = 1 / d.  The pivots sit on the replicated critical path of
    //    every PDIP iteration and of initialize(); without the square-root refinement the
    //    poly x poly loop is 646 -> 614 instructions and its Cholesky section 590 -> 476
    //    cycles.  Used by every N = 4 kernel (polytope, sphere and cone pairs).  The pivot
    //    reciprocal is v_rcp_f64 + one Newton step in the polytope x polytope kernels and the
    //    correctly rounded two-step frcp in the SOC ones: with the one-step reciprocal there,
    //    one polytope x cone pair of the 1M mixed set (its exit test decided at
    //    mu = tol (1 - 1e-7) in the oracle) took one more iteration than the oracle.  The
    //    N = 5 / 6 kernels keep the square-root form: the factorisation's extra row block (E
    //    below) pushed the one-wave PART kernels into in-loop scratch (polygon x polytope
    //    -13 %).  -DDCOL_CHOL_SQRT: the square-root form everywhere (A/B runs).
    // False if a pivot is <= 0, infinite or NaN.  Any non-finite entry of H's upper triangle
    // makes some pivot non-finite (a diagonal entry directly, an off-diagonal one through the
    // products that update later pivots), so a non-finite H always fails here and the caller
    // only classifies failures.
#ifdef DCOL_CHOL_SQRT
    static constexpr bool LDL = false;
#else
    static constexpr bool LDL = N == 4;
#endif
    DCOL_HD static bool chol(const double (&H)[N][N], double (&F)[N][N], double (&idg)[N]) {
        bool ok = true;
        double E[LDL ? N : 1][N];   // LDL: E[k][c] = d_k U[k][c], the rows before their pivot's scaling
#pragma unroll
        for (int j = 0; j < N; ++j) {
            double d = H[j][j];
#pragma unroll
            for (int k = 0; k < j; ++k) d -= (LDL ? E[LDL ? k : 0][j] : F[k][j]) * F[k][j];
            ok = ok && pos_finite(d);
            idg[j] = !LDL ? frsqrt(d) : (NSOC == 0 ? frcp1(d) : frcp(d));
#pragma unroll
            for (int c = j + 1; c < N; ++c) {
                double t = H[j][c];
#pragma unroll
                for (int k = 0; k < j; ++k) t -= (LDL ? E[LDL ? k : 0][j] : F[k][j]) * F[k][c];
                if constexpr (LDL) E[j][c] = t;
                F[j][c] = t * idg[j];
            }
        }
        return ok;
    }
    // solve H x = b: Cholesky F_c' F_c x = b (cho_solve((F, False), b)); LDL forward U' y = b,
    // w = y / d, backward U x = w
    DCOL_HD static void chol_solve(const double (&F)[N][N], const double (&idg)[N], const double* b, double* out) {
        double y[N];
#pragma unroll
        for (int j = 0; j < N; ++j) {
            double t = b[j];
#pragma unroll
            for (int k = 0; k < j; ++k) t -= F[k][j] * y[k];
            y[j] = LDL ? t : t * idg[j];
        }
#pragma unroll
        for (int j = N - 1; j >= 0; --j) {
            double t = LDL ? y[j] * idg[j] : y[j];
#pragma unroll
            for (int k = j + 1; k < N; ++k) t -= F[j][k] * out[k];
            out[j] = LDL ? t : t * idg[j];
        }
    }
    // quirk Q1 (pdip.py:313-318): y = solve_triangular(L, -c) with lower=False reads diag(L)
    // only: y = -e_3 / L_33; then x = L^-T y, i.e. F_c x = y (LDL: U x = D^(-1/2) y = -e_3 / d_3)
    DCOL_HD static void q1_solve(const double (&F)[N][N], const double (&idg)[N], double* out) {
#pragma unroll
        for (int j = N - 1; j >= 0; --j) {
            double acc = (j == 3) ? -idg[3] : 0.0;
#pragma unroll
            for (int k = j + 1; k < N; ++k) acc -= F[j][k] * out[k];
            out[j] = LDL ? acc : acc * idg[j];
        }
    }
    // group all-reduce of the packed upper triangle / of an N-vector
    DCOL_HD static void allsum_sym(double (&H)[N][N]) {
#pragma unroll
        for (int j = 0; j < N; ++j)
#pragma unroll
            for (int c = j; c < N; ++c) H[j][c] = R::sum(H[j][c]);
    }
    DCOL_HD static void allsum_vec(double* v) {
#pragma unroll
        for (int j = 0; j < N; ++j) v[j] = R::sum(v[j]);
    }

    // bring2cone, pdip.py:237-287 (quirk Q11), group-wide.  FULL: every orthant slot holds a
    // row (the padding masks fold away, as in the PDIP loop)
    template <bool FULL>
    DCOL_HD void bring2cone(double* v) const {
        double any = 0.0, mn = __builtin_inf(), socv = -__builtin_inf();
#pragma unroll
        for (int k = 0; k < OR; ++k) {
            const bool vk = live<FULL>(k);
            any = (vk & (v[k] <= 0.0)) ? 1.0 : any;
            mn = vk ? fmin(mn, v[k]) : mn;
        }
#pragma unroll
        for (int b = 0; b < SS; ++b) {
            const double* p = v + OR + SD * b;
            const double res = SPLIT ? bc0(p[0]) - sqrt(R::sum(q ? fma(p[0], p[0], p[1] * p[1]) : p[1] * p[1]))
                                     : p[0] - sqrt(tail_dot<SD>(p, p));
            socv = (vs[b] & (res <= 0.0)) ? fmax(socv, -res) : socv;
        }
        any = R::max(any);
        mn = R::min(mn);
        socv = R::max(socv);
        double a = -1.0;
        if (any > 0.0) a = -mn;
        a = fmax(a, socv);
        if (a >= 0.0) {
            const double sh = 1.0 + a;
#pragma unroll
            for (int k = 0; k < OR; ++k) v[k] = live<FULL>(k) ? v[k] + sh : v[k];
#pragma unroll
            for (int b = 0; b < SS; ++b)   // (the head coordinate: lane 0's under SPLIT)
                v[OR + SD * b] = (vs[b] && (!SPLIT || q == 0)) ? v[OR + SD * b] + sh : v[OR + SD * b];
        }
    }

    // -------- initialize, pdip.py:291-332 ------------------------------------------------
    template <bool FULL>
    DCOL_HD bool initialize() {
        DCOL_NSTAMP(0);
        double H[N][N], F[N][N], idg[N], gth[N];
#pragma unroll
        for (int j = 0; j < N; ++j) {
            gth[j] = 0.0;
#pragma unroll
            for (int c = j; c < N; ++c) H[j][c] = 0.0;
        }
        if constexpr (BOX) {                       // axis pairs: G'G = 2 u u' + ..., G'h = (h - h') u + ...
#pragma unroll
            for (int m = 0; m < OR / 2; ++m) {
                const int k = 2 * m;
                const double ge = gr(k, 3), go = gr(k + 1, 3);
                const double dh = r[k] - r[k + 1];
                const double cg = ge - go;
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    const double uj = gr(k, j);
                    gth[j] = fma(uj, dh, gth[j]);
                    const double u2 = 2.0 * uj;
#pragma unroll
                    for (int c = j; c < 3; ++c) H[j][c] = fma(u2, gr(k, c), H[j][c]);
                    H[j][3] = fma(uj, cg, H[j][3]);
                }
                gth[3] = fma(ge, r[k], fma(go, r[k + 1], gth[3]));
                H[3][3] = fma(ge, ge, fma(go, go, H[3][3]));
            }
        } else {
#pragma unroll
        for (int k = 0; k < MG; ++k) {
#pragma unroll
            for (int j = 0; j < N; ++j) {
                if (!nz(k, j)) continue;
                gth[j] += gr(k, j) * r[k];          // r holds h here
#pragma unroll
                for (int c = j; c < N; ++c)
                    if (nz(k, c)) H[j][c] += gr(k, j) * gr(k, c);
            }
        }
        }
        if constexpr (BALL) {                      // the ball rows' products, zeros dropped
#pragma unroll
            for (int b = 0; b < SS; ++b) {
                const int k0 = OR + SD * b;
                soc_gtv(b, r + k0, gth);
                // (SPLIT: G_b'G_b from lane 0 only; G_b'h per coordinate above)
                const double own = (!SPLIT || q == 0) ? 1.0 : 0.0;
                const double sRb = sR[b] * own, svb = sv[b] * own;
                H[3][3] = fma(sRb, sRb, H[3][3]);
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    H[j][j] = fma(svb, svb, H[j][j]);
#pragma unroll
                    for (int i = 0; i < NX; ++i) H[j][4 + i] = fma(-svb, sX[b][j][i], H[j][4 + i]);
                }
#pragma unroll
                for (int i = 0; i < NX; ++i)
#pragma unroll
                    for (int i2 = i; i2 < NX; ++i2)
#pragma unroll
                        for (int k = 0; k < 3; ++k)
                            H[4 + i][4 + i2] = fma(sX[b][k][i] * own, sX[b][k][i2], H[4 + i][4 + i2]);
            }
        }
        if constexpr (CONE) {                      // the cone rows, same order as dense rows
#pragma unroll
            for (int b = 0; b < SS; ++b)
#pragma unroll
                for (int e = 0; e < 3; ++e) {
                    const int k = OR + SD * b + e;
                    double g[4] = {cqx(b, e, 0), cqx(b, e, 1), cqx(b, e, 2), (e == 0) ? ccx(b) : 0.0};
#pragma unroll
                    for (int j = 0; j < N; ++j) {
                        if (j == 3 && e != 0) continue;
                        gth[j] += g[j] * r[k];
#pragma unroll
                        for (int c = j; c < N; ++c)
                            if (!(c == 3 && e != 0)) H[j][c] += g[j] * g[c];
                    }
                }
        }
        allsum_sym(H);
        allsum_vec(gth);
        DCOL_NSTAMP(1);
        const bool ok = chol(H, F, idg);             // F' = np.linalg.cholesky(G'G)
        chol_solve(F, idg, gth, x);                  // x_hat = L^-T L^-1 G'h
        DCOL_NSTAMP(2);
        double t[M];
#pragma unroll
        for (int k = 0; k < M; ++k) {
            r[k] = rowdot(k, x) - r[k];              // r = G x_hat - h  (quirk Q2: s~ = G x_hat - h)
            t[k] = r[k];
        }
        DCOL_NSTAMP(3);
        bring2cone<FULL>(t);
        DCOL_NSTAMP(4);
        // quirk Q1: y = solve_triangular(L, -c) with lower=False reads diag(L) only:
        // y = -e_3 / L_33, then x = L^-T y
        double xz[N];
        q1_solve(F, idg, xz);
        double zt[M];
#pragma unroll
        for (int k = 0; k < M; ++k) zt[k] = rowdot(k, xz);
        DCOL_NSTAMP(5);
        bring2cone<FULL>(zt);
        DCOL_NSTAMP(6);
#pragma unroll
        for (int k = 0; k < M; ++k) {
            const bool v = k < OR ? live<FULL>(k) : vrow(k);
            const double one = (k < OR || (((k - OR) % SD) == 0 && (!SPLIT || q == 0))) ? 1.0 : 0.0;   // inert: e
            s[k] = v ? t[k] : one;
            z[k] = v ? zt[k] : one;
        }
        DCOL_NSTAMP(7);
        return ok;
    }

    // Ratio tests in reciprocal form: the orthant step bound min(1, min_{d<0} x/(-d))
    // (pdip.py:7-22) is 1 / max(1, max_i (-d_i / x_i)), accumulated as a running max of
    // -d_i * (1/x_i) -- a multiply and a max per row bound instead of a compare-and-select
    // argmin (the reciprocal 1/s is already at hand for every row).  Rows with d >= 0 give
    // a candidate <= 0 and never win; inert padding rows (s = z = 1, G = 0, r = 0) give
    // candidates -d <= 1 in both directions (ds = -1, dz = 0 or sigma mu), so no mask is
    // needed.  Rounding-level only: the bound differs from the reference's quotient by a
    // few ulp.
    DCOL_HD static double bound_inv(double cmax, double d, double ix) { return fmax(cmax, -d * ix); }

    struct SocState {
        SocNT W;
        double lam[SD];
        double ll[SD];
    };

    // -------- solve_lp_pdip, pdip.py:373-470 -------------------------------------------
    // FULL: every orthant slot holds a real row (o == OMAX for the whole launch), so the
    // padding masks of the loop fold away at compile time.
    template <bool FULL>
    DCOL_HD bool live(int k) const { return FULL || vort(k); }

    // it0: first iteration (a resumed pair continues its count); susp_t > 0: suspension
    // check (SUSP main launch) -- see KArgs
    template <bool FULL, bool SUSP = false>
    DCOL_HD int32_t pdip(double tol, int max_iter, int* it_out, int it0 = 0, int susp_t = 0, int susp_min = 0) {
        int it = 0;
        int32_t st = ST_MAXITER;
        // mu = s'z / deg as a multiply by the correctly rounded 1/deg plus one FMA remainder
        // correction (Markstein): the correctly rounded quotient, without a division sequence
        // per iteration
        const double degd = FULL ? (double)(OMAX + NSOC) : (double)deg;
        const double rdeg = 1.0 / degd;
        for (it = it0; it < max_iter; ++it) {
            DCOL_ISTAMP(it, 0);
            // ---- mu = s'z / deg and the exit test first (pdip.py:410-422, quirk Q3): the
            // iteration that returns does not build the normal matrix
            double isz[OR > 0 ? OR : 1];   // orthant rows: 1 / (s z); 1 / s = z / (s z) is formed at
                                           // each use (ilv): one multiply instead of a register
                                           // array live across the whole iteration
            double sz = 0.0;
#pragma unroll
            for (int k = 0; k < OR; ++k) {
                // one reciprocal for both (one Newton step: the iterate sequence is unchanged on
                // every golden vector, -12 VALU instructions per iteration)
                const double rsz = frcp1(s[k] * z[k]);
                isz[k] = rsz;
                sz = fma(live<FULL>(k) ? s[k] : 0.0, z[k], sz);
            }
#pragma unroll
            for (int b = 0; b < SS; ++b) {
                const int k0 = OR + SD * b;
                const double szb = full_dot<SD>(s + k0, z + k0);
                sz = vs[b] ? sz + szb : sz;
            }
            sz = R::sum(sz);
            const double mq = sz * rdeg;
            const double mu = fma(fma(-mq, degd, sz), rdeg, mq);
            if (mu < tol) {
                st = ST_OK;
                break;
            }
#if defined(__HIP_DEVICE_COMPILE__)
            if constexpr (SUSP) {
                // the lanes still in the loop (every lane of a live pair; the decision is
                // wave-uniform, so a pair's lanes suspend together)
                if (it >= susp_min && susp_t > 0 &&
                    __builtin_popcountll(__builtin_amdgcn_ballot_w64(true)) <= susp_t * LPP) {
                    st = ST_SUSPENDED;
                    break;
                }
            }
#endif
            grefresh();
            // ---- NT scalings, residuals, normal matrix (pdip.py:410-434)
            SocState so[SSA];
            double Hm[N][N];
#pragma unroll
            for (int j = 0; j < N; ++j)
#pragma unroll
                for (int c = j; c < N; ++c) Hm[j][c] = 0.0;
            if constexpr (BOX) {
                // axis pair (rows [u, ge], [-u, go], W^-2 = d, d'): (d + d') u u' in the 3 x 3
                // block, (d ge - d' go) u in column 3, d ge^2 + d' go^2 at (3, 3)
#pragma unroll
                for (int m = 0; m < OR / 2; ++m) {
                    const int k = 2 * m;
                    const double de = z[k] * ilv(k, isz), dO = z[k + 1] * ilv(k + 1, isz);
                    const double ge = gr(k, 3), go = gr(k + 1, 3);
                    const double ue = de * ge, uo = dO * go;
                    const double sd = de + dO, cg = ue - uo;
#pragma unroll
                    for (int j = 0; j < 3; ++j) {
                        const double uj = gr(k, j);
                        const double su = sd * uj;
#pragma unroll
                        for (int c = j; c < 3; ++c) Hm[j][c] = fma(su, gr(k, c), Hm[j][c]);
                        Hm[j][3] = fma(cg, uj, Hm[j][3]);
                    }
                    Hm[3][3] = fma(ue, ge, fma(uo, go, Hm[3][3]));
                }
            } else {
#pragma unroll
            for (int k = 0; k < OR; ++k) {
                const double zk = z[k];
                const double d = zk * ilv(k, isz);        // W^-2 = z / s on the orthant
                double g[N];
#pragma unroll
                for (int j = 0; j < N; ++j)
                    if (nz(k, j)) g[j] = gr(k, j) * d;
#pragma unroll
                for (int j = 0; j < N; ++j)
#pragma unroll
                    for (int c = j; c < N; ++c)
                        if (nz(k, j) && nz(k, c)) Hm[j][c] += g[j] * gr(k, c);
            }
            }
#pragma unroll
            for (int b = 0; b < SS; ++b) {
                const int k0 = OR + SD * b;
                nt(s + k0, z + k0, so[b].W);
                wmul(so[b].W, z + k0, so[b].lam);
                cprod(so[b].lam, so[b].lam, so[b].ll);
            }
            // SOC part of the normal matrix
#pragma unroll
            for (int b = 0; b < SS; ++b) soc_hadd(b, so[b].W, Hm);
            allsum_sym(Hm);
            DCOL_ISTAMP(it, 1);
            double F[N][N], idg[N];
            if (!chol(Hm, F, idg)) {                        // scipy check_finite -> ValueError,
                bool finite = true;                         // else LinAlgError (not PD)
#pragma unroll
                for (int j = 0; j < N; ++j)
#pragma unroll
                    for (int c = j; c < N; ++c) finite = finite && __builtin_isfinite(Hm[j][c]);
                st = finite ? ST_NOT_PD : ST_NONFINITE;
                break;
            }
            DCOL_ISTAMP(it, 2);

            // ---- predictor (affine) direction
            double cp[M];                                // (W^-1 ds_a) o (W dz_a)
            double dsS[SSA * SD], dzS[SSA * SD];         // SOC rows of the affine step
            double dx[N];
            double cmax = 1.0, p1 = 0.0, p2 = 0.0;
            grefresh();
            predictor<FULL>(so, isz, F, idg, dx, cp, dsS, dzS, cmax, p1, p2);
            soc_bound(so, dsS, dzS, cmax);
            const double aa = frcp1(R::max(cmax));                   // quirk Q5 (no 0.99)
            DCOL_ISTAMP(it, 3);
            // rho = (s + aa ds)'(z + aa dz) / s'z, expanded as
            // s'z + aa (s'dz + z'ds) + aa^2 ds'dz (orthant sums accumulated by predictor())
#pragma unroll
            for (int b = 0; b < SS; ++b)
#pragma unroll
                for (int e = 0; e < SD; ++e) {
                    const int k = OR + SD * b + e;
                    const double dsk = dsS[SD * b + e], dzk = dzS[SD * b + e];
                    p1 = vs[b] ? fma(s[k], dzk, fma(z[k], dsk, p1)) : p1;
                    p2 = vs[b] ? fma(dsk, dzk, p2) : p2;
                }
            const double rho = (sz + R::sum(fma(aa, p1, (aa * aa) * p2))) * frcp1(sz);
            const double sc = fmax(0.0, fmin(1.0, rho));
            const double sigma = sc * sc * sc;                      // quirk Q6
#pragma unroll
            for (int b = 0; b < SS; ++b) {
                const int k0 = OR + SD * b;
                double t1[SD], t2[SD];
                wsolve(so[b].W, dsS + SD * b, t1);
                wmul(so[b].W, dzS + SD * b, t2);
                cprod(t1, t2, cp + k0);
            }

            // ---- corrector (combined) direction; orthant G dx and dz are kept for the
            // update, ds (two adds) is recomputed there.
            const double smu = sigma * mu;
            double sbzt[SSA][SD], slds[SSA][SD];
            DCOL_ISTAMP(it, 4);
            grefresh();
            rhs_solve(so, isz, F, idg, cp, smu, dx, sbzt, slds);
            DCOL_ISTAMP(it, 5);
            grefresh();
            cmax = 1.0;
            double cu[OR > 0 ? OR : 1], cdz[OR > 0 ? OR : 1];   // G dx and dz, kept for the update
#pragma unroll
            for (int k = 0; k < OR; ++k) {
                double dsk, num;
                orth_step(k, isz, cp, smu, dx, cu[k], cdz[k], dsk, num);
                cmax = bound_inv(cmax, dsk, ilv(k, isz));
                cmax = bound_inv(cmax, num, isz[k]);       // -dz / z = -num / (s z)
            }
            double sdz[SSA][SD], sds[SSA][SD], su[SSA][SD];
#pragma unroll
            for (int b = 0; b < SS; ++b) {
                soc_step(so[b], OR + SD * b, sbzt[b], slds[b], dx, su[b], sdz[b], sds[b]);
                cmax = soc_bound1(so[b].W, b, sds[b], sdz[b], cmax);
            }
            const double a = fmin(1.0, 0.99 * frcp1(R::max(cmax)));
            DCOL_ISTAMP(it, 6);
#pragma unroll
            for (int j = 0; j < N; ++j) x[j] += a * dx[j];
#pragma unroll
            for (int k = 0; k < OR; ++k) {
                const double dsk = -(s[k] + r[k]) - cu[k];
                r[k] += a * cu[k];
                // padding rows / inert SOC slots keep s = z = e: a zero step (their ds, dz
                // are finite), one select per row instead of one per updated value
                const double ak = live<FULL>(k) ? a : 0.0;
                s[k] += ak * dsk;
                z[k] += ak * cdz[k];
            }
#pragma unroll
            for (int b = 0; b < SS; ++b) {
                const int k0 = OR + SD * b;
                const double ab = vs[b] ? a : 0.0;
#pragma unroll
                for (int e = 0; e < SD; ++e) {
                    r[k0 + e] += a * su[b][e];
                    s[k0 + e] += ab * sds[b][e];
                    z[k0 + e] += ab * sdz[b][e];
                }
            }
            DCOL_ISTAMP(it, 7);
        }
        *it_out = it;
        return st;
    }

    // Newton direction.  Predictor (cp == nullptr): lambda\ds = lambda\(-lambda o lambda).
    // Corrector: lambda\ds = lambda\(-lambda o lambda - cp + smu e).  Then
    // b~z = W^-1(-rz - W lds); dx = (G~'G~)^-1(-rx + G' W^-1 b~z);
    // dz = W^-1(W^-1 G dx - b~z); ds = W(lds - W dz)          (pdip.py:424-460)
    // rx = G'z + c is folded into the same row sums: -rx + G'(W^-1 b~z) = G'(W^-1 b~z - z) - c,
    // and on an orthant row (W^-1 b~z)_k - z_k = -(z (s + r) + smu - cp) / s  (one G'v pass
    // per right-hand side, no separate G'z accumulation).
    // 1 / s of orthant row k from 1 / (s z) (the iteration's one reciprocal per row)
    DCOL_HD double ilv(int k, const double* isz) const { return z[k] * isz[k]; }
    DCOL_HD void rhs_solve(const SocState* so, const double* isz, const double (&F)[N][N], const double (&idg)[N],
                           const double* cp, double smu, double* dx, double (*sbzt)[SD], double (*slds)[SD]) const {
        double rhs[N];
#pragma unroll
        for (int j = 0; j < N; ++j) rhs[j] = 0.0;
        const auto tk = [&](int k) {
            // (W^-1 b~z)_k - z_k; the predictor's -(z (s + r)) / s reuses W^-2 = z / s of the
            // normal matrix (dd)
            return !cp ? -((z[k] * ilv(k, isz)) * (s[k] + r[k])) : -orth_num(k, cp, smu, s[k] + r[k]) * ilv(k, isz);
        };
        if constexpr (BOX) {   // axis pair: (t - t') u, ge t + go t'
#pragma unroll
            for (int m = 0; m < OR / 2; ++m) {
                const int k = 2 * m;
                const double te = tk(k), to = tk(k + 1);
                const double dt = te - to;
#pragma unroll
                for (int j = 0; j < 3; ++j) rhs[j] = fma(gr(k, j), dt, rhs[j]);
                rhs[3] = fma(gr(k, 3), te, fma(gr(k + 1, 3), to, rhs[3]));
            }
        } else {
#pragma unroll
        for (int k = 0; k < OR; ++k) {
            const double t = tk(k);
#pragma unroll
            for (int j = 0; j < N; ++j)
                if (nz(k, j)) rhs[j] += gr(k, j) * t;
        }
        }
#pragma unroll
        for (int b = 0; b < SS; ++b) {
            const int k0 = OR + SD * b;
            // W^-1 b~z = W^-1 W^-1 (-rz - W lds) = -W^-2 (s + r) - W^-1 lds   (rz = s + G x - h)
            double sr[SD], q[SD], bz[SD];
#pragma unroll
            for (int e = 0; e < SD; ++e) sr[e] = s[k0 + e] + r[k0 + e];
            w2inv(so[b].W, sr, q);
            if (!cp) {
                // predictor: lambda \ ds = -lambda, so W^-1 lds = -W^-1 W z = -z exactly:
                // W^-1 b~z = z - W^-2 (s + r) and (W^-1 b~z) - z = -W^-2 (s + r) (no soc_solve)
#pragma unroll
                for (int e = 0; e < SD; ++e) {
                    slds[b][e] = -so[b].lam[e];
                    sbzt[b][e] = z[k0 + e] - q[e];
                    bz[e] = -q[e];
                }
            } else {
                soc_lds(so[b], cp + k0, smu, slds[b]);
                double m[SD];
                wsolve(so[b].W, slds[b], m);
#pragma unroll
                for (int e = 0; e < SD; ++e) sbzt[b][e] = -q[e] - m[e];
#pragma unroll
                for (int e = 0; e < SD; ++e) bz[e] = sbzt[b][e] - z[k0 + e];
            }
            soc_gtv(b, bz, rhs);
        }
        allsum_vec(rhs);
        rhs[3] -= 1.0;                                   // - c (c = e_3)
        chol_solve(F, idg, rhs, dx);
    }
    // One orthant row of the step.  With W = diag(sqrt(s/z)) and lambda = W z the
    // reference's dz = W^-1(W^-1 u - b~z), ds = W(lds - W dz) reduce exactly to
    //   dz = (z (u + r) + smu - cp) / s,   ds = -(s + r) - u   (u = G_k dx, r = G_k x - h_k),
    // i.e. the primal and complementarity rows of the same Newton system, in fewer operations.
    DCOL_HD void orth_step(int k, const double* isz, const double* cp, double smu, const double* dx, double& u,
                           double& dz, double& ds, double& num) const {
        u = rowdot(k, dx);
        num = orth_num(k, cp, smu, u + r[k]);
        dz = num * ilv(k, isz);
        ds = -(s[k] + r[k]) - u;
    }
    // one SOC block of the step: dz = W^-1(W^-1 u - b~z) = W^-2 u - W^-1 b~z (wbz), and
    // ds = W(lds - W dz) = -(s + r) - u (the primal row of the Newton system)
    DCOL_HD void soc_step(const SocState& S, int k0, const double* wbz, const double* lds, const double* dx, double* u,
                          double* dz, double* ds) const {
        double t[SD];
#pragma unroll
        for (int e = 0; e < SD; ++e) u[e] = rowdot(k0 + e, dx);
        w2inv(S.W, u, t);
#pragma unroll
        for (int e = 0; e < SD; ++e) {
            dz[e] = t[e] - wbz[e];
            ds[e] = -(s[k0 + e] + r[k0 + e]) - u[e];
        }
        (void)lds;
    }
    // predictor (affine) direction and the orthant part of its step bound.  Orthant rows:
    // dz = z t with t = (u + r) / s, so the z-row bound candidate -dz/z is -t itself; their
    // ds/dz are not kept -- only cp = ds o dz (the corrector's cross term) and the sums
    // p1 = s'dz + z'ds, p2 = ds'dz that rho needs.  SOC rows keep ds/dz (dsS, dzS).
    template <bool FULL>
    DCOL_HD void predictor(const SocState* so, const double* isz, const double (&F)[N][N], const double (&idg)[N],
                           double* dx, double* cp, double* dsS, double* dzS, double& cmax,
                           double& p1, double& p2) const {
        double sbzt[SSA][SD], slds[SSA][SD];
        rhs_solve(so, isz, F, idg, nullptr, 0.0, dx, sbzt, slds);
        grefresh();
#pragma unroll
        for (int k = 0; k < OR; ++k) {
            const double u = rowdot(k, dx);
            const double t = (u + r[k]) * ilv(k, isz);
            const double dz = z[k] * t;
            const double ds = -(s[k] + r[k]) - u;
            cmax = bound_inv(cmax, ds, ilv(k, isz));
            cmax = fmax(cmax, -t);
            const double c = ds * dz;
            cp[k] = c;
            const bool v = live<FULL>(k);
            p1 = v ? fma(s[k], dz, fma(z[k], ds, p1)) : p1;
            p2 = v ? p2 + c : p2;
        }
#pragma unroll
        for (int b = 0; b < SS; ++b) {
            double u[SD];
            soc_step(so[b], OR + SD * b, sbzt[b], slds[b], dx, u, dzS + SD * b, dsS + SD * b);
        }
    }
    // z v + (smu - cp) on the corrector, z v on the predictor
    DCOL_HD double orth_num(int k, const double* cp, double smu, double v) const {
        return cp ? fma(z[k], v, smu - cp[k]) : z[k] * v;
    }
    DCOL_HD void soc_lds(const SocState& S, const double* cp, double smu, double* out) const {
        if (!cp) {                               // lambda \ (-lambda o lambda) = -lambda
#pragma unroll
            for (int e = 0; e < SD; ++e) out[e] = -S.lam[e];
            return;
        }
        double v[SD];
#pragma unroll
        for (int e = 0; e < SD; ++e) v[e] = -S.ll[e] - (cp ? cp[e] : 0.0);
        if (cp && (!SPLIT || q == 0)) v[0] += smu;   // + smu e (the head coordinate)
        ciprod(S.lam, v, out);
    }
    // SOC part of the step bound (soc_linesearch over the lane's blocks; ds/dz hold the
    // SOC rows only), as a running max of inverse bounds like the orthant's cmax
    DCOL_HD void soc_bound(const SocState* so, const double* ds, const double* dz, double& cmax) const {
#pragma unroll
        for (int b = 0; b < SS; ++b) cmax = soc_bound1(so[b].W, b, ds + SD * b, dz + SD * b, cmax);
    }
    DCOL_HD double soc_bound1(const SocNT& W, int b, const double* ds, const double* dz, double cmax) const {
        const int k0 = OR + SD * b;
        const double ib = fmax(lsinv(s + k0, ds, W.lis[0], W.lrc[0]), lsinv(z + k0, dz, W.lis[1], W.lrc[1]));
        return vs[b] ? fmax(cmax, ib) : cmax;
    }

    // -------- suspend / resume (KArgs susp_*) --------------------------------------------
    // fields of a suspended pair's entry: it, x[N], then (s, z, r) of every lane row
    static constexpr int SUSP_FIELDS = 1 + N + 3 * M * LPP;
    DCOL_HD static int64_t sfield(int k, int q, int c) { return 1 + N + ((int64_t)(k * LPP + q) * 3 + c); }
    // Main launch, after pdip: the pairs that returned ST_SUSPENDED take consecutive entries
    // (one atomic per wave); true for their lanes, which then return.  Every lane of the wave
    // runs this (wave-level ballot).
    DCOL_HD bool suspend(const KArgs& A, int64_t pi, int32_t st, int it) const {
#if defined(__HIP_DEVICE_COMPILE__)
        const bool me = st == ST_SUSPENDED;
        const unsigned long long m = __builtin_amdgcn_ballot_w64(me);
        if (m == 0ull) return false;
        constexpr unsigned long long lead_pat = LPP == 1 ? ~0ull : LPP == 2 ? 0x5555555555555555ull
                                              : LPP == 4 ? 0x1111111111111111ull : LPP == 8 ? 0x0101010101010101ull
                                                                                 : 0x0001000100010001ull;
        const unsigned long long lead = m & lead_pat;
        const unsigned lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        const int first = __builtin_ctzll(m);
        int base = 0;
        if ((int)lane == first) base = atomicAdd(A.susp_count, __builtin_popcountll(lead));
        base = __builtin_amdgcn_readlane(base, first);
        if (!me) return false;
        const unsigned l0 = lane - (unsigned)q;   // the pair's first lane
        const int64_t ci = base + __builtin_popcountll(lead & ((1ull << l0) - 1ull));
        const int64_t cap = A.susp_cap;
        double* __restrict__ o = A.susp_state;
        if (q == 0) {
            A.susp_pi[ci] = (int32_t)pi;
            o[ci] = (double)it;
#pragma unroll
            for (int j = 0; j < N; ++j) o[(1 + j) * cap + ci] = x[j];
        }
#pragma unroll
        for (int k = 0; k < M; ++k) {
            o[sfield(k, q, 0) * cap + ci] = s[k];
            o[sfield(k, q, 1) * cap + ci] = z[k];
            o[sfield(k, q, 2) * cap + ci] = r[k];
        }
        return true;
#else
        (void)A; (void)pi; (void)st; (void)it;
        return false;
#endif
    }
    // Resume launch: the entry's iterate in place of initialize(); returns its iteration count
    DCOL_HD int load_state(const KArgs& A, int64_t ci) {
        const int64_t cap = A.susp_cap;
        const double* __restrict__ o = A.susp_state;
#pragma unroll
        for (int j = 0; j < N; ++j) x[j] = o[(1 + j) * cap + ci];
#pragma unroll
        for (int k = 0; k < M; ++k) {
            s[k] = o[sfield(k, q, 0) * cap + ci];
            z[k] = o[sfield(k, q, 1) * cap + ci];
            r[k] = o[sfield(k, q, 2) * cap + ci];
        }
        return (int)o[ci];
    }

    // -------- gradient helpers ---------------------------------------------------------
    // orthant slot k holds a row of primitive prim that enters the pose aggregate (PART: the
    // pose slots; the extra-column rows have no pose columns)
    DCOL_HD bool owns_row(int k, int prim) const {
        if constexpr (BOX) return box_prim(k / 2) == prim;
        if constexpr (PART) {
            if (k >= PL) return false;
            const int i = k * LPP + q;
            return prim == 0 ? (i < op1) : (i >= op1 && i < op);
        }
        const int i = k * LPP + q;
        return prim == 0 ? (i < o1) : (i >= o1 && i < o);
    }

    // Pose-dependent part of f_k(theta_k) = z'(G(theta_k) x - h(theta_k)) over the rows of
    // primitive k.  Every row of every primitive is linear in (Qe, re): orthant rows
    // z_i((Qe a_i).(x - re) + g3_i x3 + ex_i.xe) sum to (Qe w).(x - re) + const with
    // w = sum z_i a_i; a ball SOC block adds z_1..3 . (re + Qe[:, extras] xe) + const; a cone
    // SOC block's rows are Qe(-E e_k) rows of the same form (w gains -E z_0..2).  The
    // constants are pose-independent and cancel exactly in a forward difference, so they are
    // never formed.  w is taken from the assembled rows in registers rather than the row
    // table: u = sum z_i G_i[0:3] = Qe w (world frame), w = Qe' u (Qe orthogonal; the same w
    // enters every evaluation of the difference, so its rounding is not amplified by 1/h).
    struct LagAgg {
        double u[3];     // sum of z_i G_i[0:3] over the primitive's orthant and cone rows, group-summed
        double zs[4];    // the primitive's SOC block duals (zero if none), group-summed
        int kind;        // SOC kind of the primitive's block
    };
    // wt: per-row weights replacing z (the implicit mode's -W^-2 G v), nullptr = z
    DCOL_HD LagAgg lag_aggregate(const DevShape& S, int prim, const double* wt = nullptr) const {
        LagAgg g;
        g.u[0] = g.u[1] = g.u[2] = 0.0;
        g.zs[0] = g.zs[1] = g.zs[2] = g.zs[3] = 0.0;
        g.kind = NSOC > 0 ? S.soc_kind : SOC_NONE;   // polytope pairs: no record read
        if constexpr (BOX) {   // axis pair: (z - z') u
#pragma unroll
            for (int m = 0; m < OR / 2; ++m) {
                const int k = 2 * m;
                const double zd = owns_row(k, prim) ? (wt ? wt[k] - wt[k + 1] : z[k] - z[k + 1]) : 0.0;
#pragma unroll
                for (int c = 0; c < 3; ++c) g.u[c] = fma(zd, gr(k, c), g.u[c]);
            }
        } else {
#pragma unroll
        for (int k = 0; k < OR; ++k) {
            if (PART && k >= PL) continue;   // extra-column rows: G[k][0:3] = 0
            const double zk = owns_row(k, prim) ? (wt ? wt[k] : z[k]) : 0.0;
#pragma unroll
            for (int c = 0; c < 3; ++c) g.u[c] = fma(zk, gr(k, c), g.u[c]);
        }
        }
        if constexpr (SPLIT) {   // lane q holds coordinates 2q, 2q + 1 of the block
            const bool own = vs[0] && soc_owner[0] == prim;
            const double z0 = own ? (wt ? wt[OR] : z[OR]) : 0.0, z1 = own ? (wt ? wt[OR + 1] : z[OR + 1]) : 0.0;
            g.zs[0] = q ? 0.0 : z0;
            g.zs[1] = q ? 0.0 : z1;
            g.zs[2] = q ? z0 : 0.0;
            g.zs[3] = q ? z1 : 0.0;
        } else
#pragma unroll
        for (int b = 0; b < SS; ++b) {
            const bool own = vs[b] && soc_owner[b] == prim;
#pragma unroll
            for (int e = 0; e < SD; ++e) {
                const double ze = own ? (wt ? wt[OR + SD * b + e] : z[OR + SD * b + e]) : 0.0;
                g.zs[e] = own ? ze : g.zs[e];
                if constexpr (CONE) {
                    if (e < 3) {                                          // cone rows: Qe(-E e_k)
#pragma unroll
                        for (int c = 0; c < 3; ++c) g.u[c] = fma(ze, cqx(b, e, c), g.u[c]);
                    }
                } else if constexpr (!BALL) {
                    const double zc = (g.kind == SOC_CONE) ? ze : 0.0;   // cone rows: Qe(-E e_k)
#pragma unroll
                    for (int c = 0; c < 3; ++c) g.u[c] = fma(zc, gr(OR + SD * b + e, c), g.u[c]);
                }
            }
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) g.u[c] = R::sum(g.u[c]);
#pragma unroll
        for (int e = 0; e < 4; ++e) g.zs[e] = R::sum(g.zs[e]);
        return g;
    }
    // body-frame w = Qe' u
    DCOL_HD static void body_w(const LagAgg& g, const Frame& Fr, double* w) {
#pragma unroll
        for (int c = 0; c < 3; ++c) w[c] = Fr.Qe[c] * g.u[0] + Fr.Qe[3 + c] * g.u[1] + Fr.Qe[6 + c] * g.u[2];
    }
    // y'Q(p) b for the reference's DCM (problem_matrices.py:213-251) without forming it:
    // Q(p) = I + (8 (p p' - S I) + al K) / den with S = p'p, al = 4 S - 4, den = (1 + S)^2 and
    // K b = b x p (dcm_jacobian's Nm), so
    //   y'Q b = y.b + (8 (y.p)(p.b) - 8 S (y.b) + al p.(y x b)) / den.
    // The p-independent y.b is left out (returned: the p-dependent correction only) -- it
    // cancels in a forward difference, and leaving it out keeps its rounding out of the
    // difference.  yb = y.b and c = y x b are the caller's (p-independent).
    DCOL_HD static double qcorr(const double* y, const double* b, double yb, const double* c, const double* p,
                                double S, double al, double iden) {
        const double yp = y[0] * p[0] + y[1] * p[1] + y[2] * p[2];
        const double pb = p[0] * b[0] + p[1] * b[1] + p[2] * b[2];
        const double pc = p[0] * c[0] + p[1] * c[1] + p[2] * c[2];
        const double t = fma(-S, yb, yp * pb);
        return fma(al, pc, 8.0 * t) * iden;
    }
    DCOL_HD static void cross3(const double* a, const double* b, double* c) {
        c[0] = a[1] * b[2] - a[2] * b[1];
        c[1] = a[2] * b[0] - a[0] * b[2];
        c[2] = a[0] * b[1] - a[1] * b[0];
    }

    // scipy approx_fprime(theta, f, sqrt(eps)) restricted to primitive prim's 6 coordinates
    // (proximity_gradient.py:50-88) for f_k(theta) = z'(G(theta) x - h(theta)) over the rows
    // of primitive k, on its aggregate ag (lag_aggregate: u = sum of z_i G_i[0:3] in the world
    // frame, the SOC duals zs; group sums already taken).  Every row is linear in the frame
    // (Qe, r_eff) (see LagAgg), so with Q = Q(p), Qe = Q Q_off, r_eff = r + Q r_off:
    //   f(r, p) = (Q w').(x - r) - w'.r_off + zs.r + zs.(Q y) + const,
    //   w' = Q(p0)' u (= Q_off w, w = Qe(p0)' u the body-frame aggregate; Q_off a rotation),
    //   y = r_off + Q_off (xe0, xe1, 0) (xe: the primitive's extra columns of x),
    // zs the ball SOC duals 1..3 (zero for other primitives).
    //  * translations: f is affine in r, so its forward difference is (zs - u)_j whatever the
    //    step (exact in exact arithmetic; taken in closed form).
    //  * rotations: forward differences with the reference's step rule of f in closed form
    //    (qcorr: no DCM is formed), the quotient through the reciprocal of the exact step.
    // Rounding-level against re-assembling the rows at each perturbed pose (the reference),
    // which the parity tests bound (1e-5 of max(|g|, 0.01) against the reference's own FD).
    DCOL_HD void fd_grad_prim(const LagAgg& ag, const DevShape& S, int prim, const double th0[6], double* g) const {
        const double hstep = 1.4901161193847656e-08;   // sqrt(finfo(float).eps)
        double zs[3] = {0.0, 0.0, 0.0};
        if (ag.kind == SOC_BALL) {
            zs[0] = ag.zs[1]; zs[1] = ag.zs[2]; zs[2] = ag.zs[3];
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) g[j] = zs[j] - ag.u[j];
        const double* p0 = th0 + 3;
        // w' = Q(p0)' u = Q(-p0) u:  u + (8 p (p.u) - 8 S u - al (u x p)) / den
        const double S0 = p0[0] * p0[0] + p0[1] * p0[1] + p0[2] * p0[2];
        const double s10 = 1.0 + S0;
        const double iden0 = frcp(s10 * s10);
        const double al0 = 4.0 * S0 - 4.0;
        double wq[3], up[3];
        cross3(ag.u, p0, up);
        const double pu = p0[0] * ag.u[0] + p0[1] * ag.u[1] + p0[2] * ag.u[2];
#pragma unroll
        for (int k = 0; k < 3; ++k) wq[k] = fma(fma(8.0 * p0[k], pu, -8.0 * S0 * ag.u[k]) - al0 * up[k], iden0, ag.u[k]);
        double d[3], cd[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) d[k] = x[k] - th0[k];
        cross3(d, wq, cd);
        const double dw = d[0] * wq[0] + d[1] * wq[1] + d[2] * wq[2];
        // ball primitives: zs.(Q y)
        double y[3] = {0.0, 0.0, 0.0}, cz[3] = {0.0, 0.0, 0.0}, zy = 0.0;
        if constexpr (NSOC > 0) {
            const int off = xoff(prim == 1);
            double xe0 = 0.0, xe1 = 0.0;
#pragma unroll
            for (int j = 4; j < N; ++j) {
                if (S.n_extra >= 1 && j == 4 + off) xe0 = x[j];
                if (S.n_extra >= 2 && j == 5 + off) xe1 = x[j];
            }
#pragma unroll
            for (int k = 0; k < 3; ++k) y[k] = S.r_off[k] + S.Q_off[3 * k] * xe0 + S.Q_off[3 * k + 1] * xe1;
            cross3(zs, y, cz);
            zy = zs[0] * y[0] + zs[1] * y[1] + zs[2] * y[2];
        }
        // f(p) - (p-independent terms), at p0 and at the three perturbed rotations
        auto fr = [&](const double* p) {
            const double Sp = p[0] * p[0] + p[1] * p[1] + p[2] * p[2];
            const double s1 = 1.0 + Sp;
            const double iden = frcp(s1 * s1);
            const double al = 4.0 * Sp - 4.0;
            double f = qcorr(d, wq, dw, cd, p, Sp, al, iden);
            if constexpr (NSOC > 0) f += qcorr(zs, y, zy, cz, p, Sp, al, iden);
            return f;
        };
        const double f0 = fr(p0);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const double t0 = p0[j];
            double hj = hstep;
            if ((t0 + hstep) - t0 == 0.0)       // _numdiff: fall back to a relative step
                hj = hstep * (t0 >= 0.0 ? 1.0 : -1.0) * fmax(1.0, fabs(t0));
            const double tj = t0 + hj;
            double p[3] = {p0[0], p0[1], p0[2]};
            p[j] = tj;
            g[3 + j] = (fr(p) - f0) * frcp(tj - t0);
        }
    }

    // closed-form d/dtheta_k of z'(G(theta)x - h(theta)) (see DESIGN.md "gradient modes"):
    //   d/dr = zeta - Qe w;  d/dp_j = d' Q_j (Qoff w) - (Qe w - zeta)' Q_j r_off + zeta' Q_j (Qoff xi)
    // w = sum z_i a_i over rotated rows (body frame), zeta = z of the ball SOC rows 1..3,
    // xi = (x4, x5, 0) on the extra columns, d = x[0:3] - r_eff
    DCOL_HD void env_grad_prim(const LagAgg& ag, const DevShape& S, int prim, const double th[6], double* g) const {
        Frame Fr;
        make_frame(S, th, Fr);
        double w[3], zeta[3] = {0.0, 0.0, 0.0};
        body_w(ag, Fr, w);                  // includes the cone rows' -E z_0..2
        if (ag.kind == SOC_BALL) {
            zeta[0] = ag.zs[1]; zeta[1] = ag.zs[2]; zeta[2] = ag.zs[3];
        }
        double xi[3] = {0.0, 0.0, 0.0};
        if (S.soc_kind == SOC_BALL) {
            const int off = xoff(prim == 1);
#pragma unroll
            for (int j = 4; j < N; ++j) {
                if (S.n_extra >= 1 && j == 4 + off) xi[0] = x[j];
                if (S.n_extra >= 2 && j == 5 + off) xi[1] = x[j];
            }
        }
        double e[3], d[3], c1[3], c2[3];
#pragma unroll
        for (int rr = 0; rr < 3; ++rr) {
            const double qw = Fr.Qe[3 * rr] * w[0] + Fr.Qe[3 * rr + 1] * w[1] + Fr.Qe[3 * rr + 2] * w[2];
            e[rr] = qw - zeta[rr];
            g[rr] = -e[rr];
            d[rr] = x[rr] - Fr.re[rr];
            c1[rr] = S.Q_off[3 * rr] * w[0] + S.Q_off[3 * rr + 1] * w[1] + S.Q_off[3 * rr + 2] * w[2];
            c2[rr] = S.Q_off[3 * rr] * xi[0] + S.Q_off[3 * rr + 1] * xi[1] + S.Q_off[3 * rr + 2] * xi[2];
        }
        double dQ[3][9];
        dcm_jacobian(th + 3, dQ);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            double acc = 0.0;
#pragma unroll
            for (int rr = 0; rr < 3; ++rr) {
                const double* qq = &dQ[j][3 * rr];
                const double m1 = qq[0] * c1[0] + qq[1] * c1[1] + qq[2] * c1[2];
                const double m2 = qq[0] * S.r_off[0] + qq[1] * S.r_off[1] + qq[2] * S.r_off[2];
                const double m3 = qq[0] * c2[0] + qq[1] * c2[1] + qq[2] * c2[2];
                acc += d[rr] * m1 - e[rr] * m2 + zeta[rr] * m3;
            }
            g[3 + j] = acc;
        }
    }

    // -------- implicit-function gradient (DCOL_GRAD_IMPLICIT) --------------------------
    // The KKT system at the returned iterate, G'z + c = 0, G x + s = h, s o z = mu e,
    // linearised in the pose with the NT scaling (ds = -W^2 dz, the PDIP's own Newton
    // linearisation, pdip.py:424-460): H dx = -dG'z - G'W^-2 (dG x - dh), H = G'W^-2 G (the
    // normal matrix G~'G~ of pdip.py:434), so with v = H^-1 e3
    //   d alpha = e3'dx = sum_i a_i (dG_i x - dh_i) - z_i (dG_i v),   a = -W^-2 G v.
    // Returns the per-row weights a (lane rows, like z) and v in vimp; false if the normal
    // matrix at this iterate does not factor (the caller then uses the envelope form).
    DCOL_HD bool implicit_weights(double* wts) {
        double Hm[N][N], dd[OR > 0 ? OR : 1];
#pragma unroll
        for (int j = 0; j < N; ++j)
#pragma unroll
            for (int c = j; c < N; ++c) Hm[j][c] = 0.0;
#pragma unroll
        for (int k = 0; k < OR; ++k) {
            const double rsz = frcp1(s[k] * z[k]);
            dd[k] = z[k] * (z[k] * rsz);                      // W^-2 = z / s
            double g[N];
#pragma unroll
            for (int j = 0; j < N; ++j)
                if (nz(k, j)) g[j] = gr(k, j) * dd[k];
#pragma unroll
            for (int j = 0; j < N; ++j)
#pragma unroll
                for (int c = j; c < N; ++c)
                    if (nz(k, j) && nz(k, c)) Hm[j][c] += g[j] * gr(k, c);
        }
        SocNT W[SSA];
#pragma unroll
        for (int b = 0; b < SS; ++b) {
            nt(s + OR + SD * b, z + OR + SD * b, W[b]);
            soc_hadd(b, W[b], Hm);
        }
        allsum_sym(Hm);
        double F[N][N], idg[N], e3[N];
        const bool fine = chol(Hm, F, idg);
#pragma unroll
        for (int j = 0; j < N; ++j) e3[j] = (j == 3) ? 1.0 : 0.0;
        chol_solve(F, idg, e3, vimp);
#pragma unroll
        for (int k = 0; k < OR; ++k) wts[k] = -(dd[k] * rowdot(k, vimp));
#pragma unroll
        for (int b = 0; b < SS; ++b) {
            const int k0 = OR + SD * b;
            double u[SD], t[SD];
#pragma unroll
            for (int e = 0; e < SD; ++e) u[e] = rowdot(k0 + e, vimp);
            w2inv(W[b], u, t);
#pragma unroll
            for (int e = 0; e < SD; ++e) wts[k0 + e] = vs[b] ? -t[e] : 0.0;
        }
        return fine;
    }
    // d alpha / d theta_prim = E(agA; x) - E_G(agZ; v): E the envelope form of
    // env_grad_prim with the weights a, E_G(z; v) = sum_i z_i dG_i v (dG only: no h term;
    // zero for translations, v3' Q_j (Q_off w_z) + zeta_z' Q_j (Q_off xi_v) for rotations)
    DCOL_HD void imp_grad_prim(const LagAgg& agA, const LagAgg& agZ, const DevShape& S, int prim, const double th[6],
                               double* g) const {
        env_grad_prim(agA, S, prim, th, g);
        Frame Fr;
        make_frame(S, th, Fr);
        double w[3], zeta[3] = {0.0, 0.0, 0.0}, xi[3] = {0.0, 0.0, 0.0};
        body_w(agZ, Fr, w);
        if (agZ.kind == SOC_BALL) {
            zeta[0] = agZ.zs[1]; zeta[1] = agZ.zs[2]; zeta[2] = agZ.zs[3];
        }
        if (S.soc_kind == SOC_BALL) {
            const int off = xoff(prim == 1);
#pragma unroll
            for (int j = 4; j < N; ++j) {
                if (S.n_extra >= 1 && j == 4 + off) xi[0] = vimp[j];
                if (S.n_extra >= 2 && j == 5 + off) xi[1] = vimp[j];
            }
        }
        double c1[3], c2[3];
#pragma unroll
        for (int rr = 0; rr < 3; ++rr) {
            c1[rr] = S.Q_off[3 * rr] * w[0] + S.Q_off[3 * rr + 1] * w[1] + S.Q_off[3 * rr + 2] * w[2];
            c2[rr] = S.Q_off[3 * rr] * xi[0] + S.Q_off[3 * rr + 1] * xi[1] + S.Q_off[3 * rr + 2] * xi[2];
        }
        double dQ[3][9];
        dcm_jacobian(th + 3, dQ);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            double acc = 0.0;
#pragma unroll
            for (int rr = 0; rr < 3; ++rr) {
                const double* qq = &dQ[j][3 * rr];
                const double m1 = qq[0] * c1[0] + qq[1] * c1[1] + qq[2] * c1[2];
                const double m3 = qq[0] * c2[0] + qq[1] * c2[1] + qq[2] * c2[2];
                acc += vimp[rr] * m1 + zeta[rr] * m3;
            }
            g[3 + j] -= acc;
        }
    }
};

// ------------------------------------------------------------------------------------
// kernel
// ------------------------------------------------------------------------------------
#ifndef DCOL_BLOCK
#define DCOL_BLOCK 64
#endif
constexpr int kLdsLanes = DCOL_BLOCK;   // GLDS: lanes per workgroup sharing the LDS row array
// Hide a pointer's provenance from the optimiser (forces fresh loads through it).
template <typename P>
DCOL_HD void launder(P& p) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+s"(p));
#else
    asm volatile("" : "+r"(p));
#endif
}

// FULL: every pair of the launch has o == OMAX (no padding rows); BALL: every SOC block of
// the launch is a ball block (Solver).  The host picks the variant per launch
// (dcol_capi.cpp: bucket_pairs).
// MODE 0: one launch; 1: main launch of a suspend / resume pair (KArgs susp_*); 2: the
// resume launch, for continuation entry ci (pi = its pair)
// GLDS: G rows in LDS (Solver; the one-wave-per-workgroup solve kernels only)
// FDONLY: the copy built for the reference's FD gradient mode alone (launched only for runs
// without DCOL_GRAD_ENVELOPE / DCOL_GRAD_IMPLICIT): the envelope and implicit code is not
// compiled in, so its register pressure never shapes the FD path (variants.py BOX_FD)
template <int N, int NSOC, int OMAX, int LPP, bool FULL = false, bool BALL = false, bool CONE = false, int OE = 0,
          int MODE = 0, bool GLDS = false, bool BOX = false, bool FDONLY = false, bool SPLIT = false>
DCOL_HD void solve_one(const KArgs& A, int64_t pi, int q, int64_t ci = -1, int k1o = -1, int k2o = -1) {
    DCOL_STAMP(A, pi, q, 0);
    const int64_t B = A.B;
    // k1o / k2o >= 0: the shape ids given (the one-pair server reads them with its request)
    const int k1 = k1o >= 0 ? k1o : A.s1[pi], k2 = k2o >= 0 ? k2o : A.s2[pi];
    const DevShape& S1 = A.shapes[k1];
    const DevShape& S2 = A.shapes[k2];
    double th1[6], th2[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        th1[c] = A.pose1[c * B + pi];
        th2[c] = A.pose2[c * B + pi];
    }
    Frame F1, F2;
    // both records' plain flags read before either frame: their loads issue together (read
    // inside make_frame, the second record's load waited for the first frame's branch)
    const int32_t plain1 = S1.plain, plain2 = S2.plain;
    make_frame(S1, th1, F1, plain1);
    make_frame(S2, th2, F2, plain2);
    DCOL_STAMP(A, pi, q, 1);

    static_assert(!BOX || FULL, "BOX kernels are padding-free");
    using Slv = Solver<N, NSOC, OMAX, LPP, BALL, CONE, OE, GLDS, BOX, SPLIT>;
    Slv P;
    P.q = q;
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (GLDS) {
        static_assert(kLdsLanes == 64, "GLDS: one wave per workgroup");
        __shared__ double rows_lds[Slv::LDSW * 64];
        P.gb = (typename Slv::lds_d*)&rows_lds[threadIdx.x & 63];
    }
#endif
#ifdef DCOL_STAMPS
    P.dbg = (q == 0 && A.stamps) ? A.stamps + 16 * pi + 8 : nullptr;
#endif
    P.assemble(A, S1, S2, F1, F2);
    DCOL_STAMP(A, pi, q, 2);
    int it = 0;
    int32_t st;
    if constexpr (MODE == 2) {   // continue the suspended iteration sequence
        const int it0 = P.load_state(A, ci);
        st = P.template pdip<FULL>(A.tol, A.max_iter, &it, it0);
    } else {
        const bool init_ok = P.template initialize<FULL>();
        DCOL_STAMP(A, pi, q, 3);
        if (!init_ok) st = ST_NOT_PD;
        else st = P.template pdip<FULL, MODE == 1>(A.tol, A.max_iter, &it, 0, A.susp_t, A.susp_min);
    }
    DCOL_STAMP(A, pi, q, 4);
    if constexpr (MODE == 1) {
        if (P.suspend(A, pi, st, it)) return;   // the resume launch finishes this pair
    }

    const double nan = __builtin_nan("");
    const bool ok = st == ST_OK;
    double g[12];
    const bool want_grad = (A.flags & (F_GRAD_FD | F_GRAD_ENV | F_GRAD_IMP)) && (A.grad || A.rec);
    if (want_grad) {
        // Phase boundary: make the gradient re-read poses, shape records and row descriptors
        // instead of keeping the assembly-phase copies live across the whole PDIP loop
        // (register pressure: ~150 -> ~300 VGPRs without this).
        asm volatile("" ::: "memory");
        KArgs L = A;   // laundered copies of the table pointers: no load CSE across the loop
        launder(L.shapes);
        launder(L.rows);
        launder(L.pose1);
        launder(L.pose2);
        const DevShape& T1 = L.shapes[k1];
        const DevShape& T2 = L.shapes[k2];
        if (ok) {
            using Agg = typename Slv::LagAgg;
            // implicit mode first: its weights a = -W^-2 G v at this iterate, aggregated like
            // z -- so that nothing of the other modes (the z aggregates, the poses) is live
            // across implicit_weights' normal matrix and Cholesky factor (held across it, they
            // spilled to scratch in every mode: 124 B per lane in the three-wave BOX kernel)
            const bool imp = !FDONLY && (A.flags & F_GRAD_IMP) != 0;
            Agg agA0, agA1;
            bool imp_ok = false;
            if (imp) {
                double wts[Slv::M];
                imp_ok = P.implicit_weights(wts);
                agA0 = P.lag_aggregate(T1, 0, wts);
                agA1 = P.lag_aggregate(T2, 1, wts);
            }
            // group sums for both primitives first (every lane of the group), then each
            // lane differentiates one primitive: lane q takes primitive q & 1, so a 2+-lane
            // group does the two 6-coordinate gradients side by side instead of both in
            // every lane (a 1-lane group does both in turn)
            const Agg ag0 = P.lag_aggregate(T1, 0);
            const Agg ag1 = P.lag_aggregate(T2, 1);
#pragma unroll
            for (int c = 0; c < 6; ++c) {
                th1[c] = L.pose1[c * B + pi];
                th2[c] = L.pose2[c * B + pi];
            }
            constexpr int NP = LPP >= 2 ? 1 : 2;
#pragma unroll
            for (int pp = 0; pp < NP; ++pp) {
                const int prim = LPP >= 2 ? (q & 1) : pp;
                const DevShape& T = prim ? T2 : T1;
                Agg ag;   // element-wise select (a reference select would put both on the stack)
#pragma unroll
                for (int c = 0; c < 3; ++c) ag.u[c] = prim ? ag1.u[c] : ag0.u[c];
#pragma unroll
                for (int c = 0; c < 4; ++c) ag.zs[c] = prim ? ag1.zs[c] : ag0.zs[c];
                ag.kind = prim ? ag1.kind : ag0.kind;
                double th[6];
#pragma unroll
                for (int c = 0; c < 6; ++c) th[c] = prim ? th2[c] : th1[c];
                double* gp = g + 6 * pp;
                if (imp && imp_ok) {
                    Agg agA;
#pragma unroll
                    for (int c = 0; c < 3; ++c) agA.u[c] = prim ? agA1.u[c] : agA0.u[c];
#pragma unroll
                    for (int c = 0; c < 4; ++c) agA.zs[c] = prim ? agA1.zs[c] : agA0.zs[c];
                    agA.kind = ag.kind;
                    P.imp_grad_prim(agA, ag, T, prim, th, gp);
                } else if (!FDONLY && (A.flags & (F_GRAD_ENV | F_GRAD_IMP))) {
                    P.env_grad_prim(ag, T, prim, th, gp);
                } else {
                    P.fd_grad_prim(ag, T, prim, th, gp);
                }
            }
        } else {
#pragma unroll
            for (int c = 0; c < 12; ++c) g[c] = nan;
        }
    }
    DCOL_STAMP(A, pi, q, 5);
    double* const rec = A.rec ? A.rec + (int64_t)kRec * pi : nullptr;
    if (want_grad) {
        if (LPP >= 2) {   // lane 1 of the group holds primitive 2's block (see above)
            if (q == 1) {
#pragma unroll
                for (int c = 0; c < 6; ++c) {
                    const double v = ok ? g[c] : nan;
                    if (A.grad) A.grad[(6 + c) * B + pi] = v;
                    if (rec) rec[7 + c] = v;
                }
            }
        } else {
#pragma unroll
            for (int c = 6; c < 12; ++c) {
                if (A.grad) A.grad[c * B + pi] = g[c];
                if (rec) rec[1 + c] = g[c];
            }
        }
    }
    if (q != 0) return;
    const double al = ok ? P.x[3] : nan;
    if (A.alpha) A.alpha[pi] = al;
    if (A.iters) A.iters[pi] = it;
    if (A.status) A.status[pi] = st;
    if ((A.flags & F_CONTACT) && A.contact) {
#pragma unroll
        for (int c = 0; c < 3; ++c) A.contact[c * B + pi] = ok ? P.x[c] : nan;
    }
    if (want_grad && A.grad) {
#pragma unroll
        for (int c = 0; c < 6; ++c) A.grad[c * B + pi] = g[c];
    }
    if (rec) {   // the record's alpha, primitive 1's gradient (all 12 NaN without one), ints
        rec[0] = al;
#pragma unroll
        for (int c = 0; c < 6; ++c) rec[1 + c] = want_grad ? g[c] : nan;
        if (!want_grad) {
#pragma unroll
            for (int c = 6; c < 12; ++c) rec[1 + c] = nan;
        }
        rec[13] = rec_ints(st, it);
    }
}

// LPP lanes per pair; slots [slot0, slot0+n) of the plan's permutation (or identity).
// The n*LPP threads of a launch are contiguous, so a group never straddles the tail.
// WPS = minimum waves per SIMD requested from the register allocator (variants.py).
#ifndef DCOL_BLOCK
#define DCOL_BLOCK 64
#endif
constexpr int kSolveBlock = DCOL_BLOCK;
static_assert(kSolveBlock % 64 == 0, "one or more whole waves per workgroup");

// FL: variant flags, bit 0 FULL, bit 1 BALL, bit 2 CONE, bit 3 BOX, bit 5 SPLIT ball block, bit 6 FD-only
// gradient (variants.py)
// OE > 0: the row-partitioned (PART) copy with OE extra-column row slots (Solver).
// FL bit 4 (16): the main launch of a suspend / resume pair (solve_one MODE 1)
// WPS >= 10: the LDS-rows copy (Solver GLDS) at WPS - 10 waves per SIMD (variants.py);
// DCOL_NO_GLDS builds every copy with register rows (the codegen-invariance twin, A/B)
#ifdef DCOL_NO_GLDS
constexpr bool kGlds = false;
#else
constexpr bool kGlds = true;
#endif
template <int N, int NSOC, int OMAX, int LPP, int WPS, int FL, int OE = 0>
__global__ void __launch_bounds__(kSolveBlock, WPS % 10) prox_kernel(KArgs A) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t slot = t / LPP;
    const int q = (int)(t % LPP);
    if (slot >= A.n) return;
    const int64_t pi = A.perm ? (int64_t)A.perm[A.slot0 + slot] : (A.slot0 + slot);
    solve_one<N, NSOC, OMAX, LPP, (FL & 1) != 0, (FL & 2) != 0, (FL & 4) != 0, OE, (FL & 16) ? 1 : 0,
              kGlds && WPS >= 10, (FL & 8) != 0, (FL & 64) != 0, (FL & 32) != 0>(A, pi, q);
}

// The resume launch of a suspend / resume pair: one lane group per continuation entry;
// entries past the count the main launch appended exit at once.
template <int N, int NSOC, int OMAX, int LPP, int WPS, int FL, int OE = 0>
__global__ void __launch_bounds__(kSolveBlock, WPS % 10) prox_resume_kernel(KArgs A) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t ci = t / LPP;
    const int q = (int)(t % LPP);
    if (ci >= A.susp_cap || ci >= (int64_t)*A.susp_count) return;
    const int64_t pi = A.susp_pi[ci];
    solve_one<N, NSOC, OMAX, LPP, (FL & 1) != 0, (FL & 2) != 0, (FL & 4) != 0, OE, 2, false, (FL & 8) != 0>(A, pi, q, ci);
}

}  // namespace dcol
