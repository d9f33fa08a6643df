/*
 * dcol_oracle_opcount.cpp -- op-counting build of the C restatement ("the
 * C++ restatement should carry an op-counter mode that emits exact per-class counts").
 * TEST / MEASUREMENT INFRASTRUCTURE ONLY: never linked into the product library.
 *
 * dcol_oracle.c is compiled unchanged as C++ with `double` replaced by a counted scalar:
 * every FP64 +, -, *, / and sqrt the restatement executes (which follows the reference
 * op-for-op) adds one to a per-thread counter; comparisons, fabs / fmax, negation and copies
 * are free (the hand model's convention).  dcol_opcount_batch() solves a
 * batch like dcol_oracle_batch() and returns, per pair, the ops of each phase: assembly
 * (problem matrices + combine), PDIP (initialize + every iteration incl. the exit one) and
 * the FD gradient (13 Lagrangian evaluations + the 12 quotients), plus the iteration count.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

namespace dcol_oc {
inline thread_local long long ops = 0;

struct CD {
    double v;
    CD() = default;
    template <typename T>
    CD(T x) : v((double)x) {}
};
inline CD operator+(CD a, CD b) { ++ops; return CD(a.v + b.v); }
inline CD operator-(CD a, CD b) { ++ops; return CD(a.v - b.v); }
inline CD operator*(CD a, CD b) { ++ops; return CD(a.v * b.v); }
inline CD operator/(CD a, CD b) { ++ops; return CD(a.v / b.v); }
inline CD operator-(CD a) { return CD(-a.v); }
inline CD operator+(CD a) { return a; }
inline CD& operator+=(CD& a, CD b) { a = a + b; return a; }
inline CD& operator-=(CD& a, CD b) { a = a - b; return a; }
inline CD& operator*=(CD& a, CD b) { a = a * b; return a; }
inline CD& operator/=(CD& a, CD b) { a = a / b; return a; }
inline bool operator<(CD a, CD b) { return a.v < b.v; }
inline bool operator>(CD a, CD b) { return a.v > b.v; }
inline bool operator<=(CD a, CD b) { return a.v <= b.v; }
inline bool operator>=(CD a, CD b) { return a.v >= b.v; }
inline bool operator==(CD a, CD b) { return a.v == b.v; }
inline bool operator!=(CD a, CD b) { return a.v != b.v; }
inline CD sqrt(CD a) { ++ops; return CD(::sqrt(a.v)); }
inline CD fabs(CD a) { return CD(::fabs(a.v)); }
inline CD fmax(CD a, CD b) { return CD(::fmax(a.v, b.v)); }
inline CD tan(CD a) { ++ops; return CD(::tan(a.v)); }
inline CD pow(CD a, CD b) { ++ops; return CD(::pow(a.v, b.v)); }
inline bool isfinite(CD a) { return ::isfinite(a.v); }
}  // namespace dcol_oc

using dcol_oc::CD;
using dcol_oc::fabs;
using dcol_oc::fmax;
using dcol_oc::pow;
using dcol_oc::sqrt;
using dcol_oc::tan;
#undef isfinite
using dcol_oc::isfinite;

#pragma GCC diagnostic ignored "-Wclass-memaccess"
#define double CD
#include "dcol_oracle.c"
#undef double

static_assert(sizeof(CD) == sizeof(double), "CD must be layout-compatible with double");

extern "C" int dcol_opcount_batch(const int32_t* type, const int32_t* nh, const int32_t* A_off,
                                  const double* A_pool, const double* b_pool, const double* params,
                                  const double* roff, const double* Qoff, int64_t B, const int32_t* s1,
                                  const int32_t* s2, const double* pose1, const double* pose2, double tol,
                                  int64_t* ops_assembly, int64_t* ops_pdip, int64_t* ops_grad, int32_t* iters,
                                  int32_t* status) {
    auto C = [](const double* p) { return reinterpret_cast<const CD*>(p); };
    for (int64_t i = 0; i < B; ++i) {
        Shape a, b;
        load_shape(s1[i], type, nh, A_off, C(A_pool), C(b_pool), C(params), C(roff), C(Qoff), &a);
        load_shape(s2[i], type, nh, A_off, C(A_pool), C(b_pool), C(params), C(roff), C(Qoff), &b);
        Prob P;
        CD x[NMAX], s[MMAX], z[MMAX];
        int it = 0;
        dcol_oc::ops = 0;
        int st = assemble(&a, C(pose1) + 6 * i, &b, C(pose2) + 6 * i, &P);
        ops_assembly[i] = dcol_oc::ops;
        dcol_oc::ops = 0;
        if (st == ST_OK) st = pdip(&P, CD(tol), x, s, z, &it);
        ops_pdip[i] = dcol_oc::ops;
        dcol_oc::ops = 0;
        if (st == ST_OK) {   // proximity_gradient.py:50-88 with approx_fprime's step rule
            CD th[12], th1[12];
            for (int k = 0; k < 6; ++k) { th[k] = C(pose1)[6 * i + k]; th[6 + k] = C(pose2)[6 * i + k]; }
            const CD hstep = 1.4901161193847656e-08;
            const CD f0 = lag_con(&a, &b, x, z, th);
            memcpy(th1, th, sizeof(th));
            for (int k = 0; k < 12; ++k) {
                CD h = hstep;
                if ((th[k] + h) - th[k] == 0) h = hstep * (th[k] >= 0 ? 1.0 : -1.0) * fmax(1.0, fabs(th[k]));
                th1[k] += h;
                const CD dx = th1[k] - th[k];
                (void)((lag_con(&a, &b, x, z, th1) - f0) / dx);
                th1[k] = th[k];
            }
        }
        ops_grad[i] = dcol_oc::ops;
        iters[i] = it;
        status[i] = st;
    }
    return 0;
}
