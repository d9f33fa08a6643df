// dcol_host.hpp — host-side digest of primitives and pair classification, shared by the
// C-ABI (dcol_capi.cpp) and the test-only x86 emulator (tests/emul).
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/dcol.h"
#include "dcol_device.hpp"
#include "dcol_variants.inc"

namespace dcol_host {
using namespace dcol;

inline std::string& last_error() {
    thread_local std::string e;
    return e;
}

inline int fail(int code, const std::string& msg) {
    last_error() = msg;
    return code;
}

// sorted OMAX buckets per (N, NSOC), from the compiled variant list
inline const std::map<std::pair<int, int>, std::vector<int>>& buckets() {
    static const std::map<std::pair<int, int>, std::vector<int>> m = [] {
        std::map<std::pair<int, int>, std::vector<int>> r;
#define DCOL_ADD(NN, NS, OM) r[{NN, NS}].push_back(OM);
        DCOL_SHAPES(DCOL_ADD)
#undef DCOL_ADD
        for (auto& kv : r) std::sort(kv.second.begin(), kv.second.end());
        return r;
    }();
    return m;
}

// Compiled (LPP, WPS) list of a kernel shape in one flavour: fl 2 the ball-SOC copies, 4 the
// structured-cone copies, else the dense kernels (variants.py CONFIG / CONFIG_FL); the
// first entry is the throughput choice.
#define DCOL_FOR_FLAVOUR(fl, X)          \
    do {                                 \
        if ((fl) == 2) {                 \
            DCOL_BALL_VARIANTS(X)        \
        } else if ((fl) == 4) {          \
            DCOL_CONE_VARIANTS(X)        \
        } else {                         \
            DCOL_VARIANTS(X)             \
        }                                \
    } while (0)

// largest compiled LPP for a kernel shape (latency choice for launches that leave the GPU
// mostly idle)
inline int max_lpp(int N, int nsoc, int omax, int fl = 0) {
    int best = 0;
#define DCOL_MAXL(NN, NS, OM, LP, WP, FL) \
    if (NN == N && NS == nsoc && OM == omax && LP > best) best = LP;
    DCOL_FOR_FLAVOUR(fl, DCOL_MAXL);
#undef DCOL_MAXL
    return (best == 0 && fl != 0) ? max_lpp(N, nsoc, omax, 0) : best;   // no copies of the flavour: dense
}
inline bool lpp_forced() { return std::getenv("DCOL_LPP") != nullptr; }
// lanes per pair for a kernel shape: the first compiled LPP of the flavour, or DCOL_LPP=<n>
// if that alternative is compiled (A/B experiments)
inline int choose_lpp(int N, int nsoc, int omax, int fl = 0) {
    static const int forced = [] {
        const char* e = std::getenv("DCOL_LPP");
        return e ? std::atoi(e) : 0;
    }();
    int first = 0;
#define DCOL_PICK(NN, NS, OM, LP, WP, FL)                          \
    if (NN == N && NS == nsoc && OM == omax) {                     \
        if (first == 0) first = LP;                                \
        if (forced == LP) return LP;                               \
    }
    DCOL_FOR_FLAVOUR(fl, DCOL_PICK);
#undef DCOL_PICK
    return (first == 0 && fl != 0) ? choose_lpp(N, nsoc, omax, 0) : first;   // no copies of the flavour: dense
}

// A row pool starts with one zero row (index 0; every shape's rows follow): a lane slot
// without a row of its pair loads that row instead of branching around its loads (the
// kernels' orth_row / ext_row), so all slots' loads issue back to back.
inline void init_row_pool(std::vector<DevRow>& rows) { rows.assign(1, DevRow{}); }

// Static digest of one primitive (misc_primitive_constructor.py:4-88 ->
// problem_matrices.py:4-209).  Every orthant row is [Qe a, g3, ex0, ex1] with
// h = (Qe a) . r_eff; the SOC block is generated in-kernel from (kind, R, cone_c, tanb).
inline int digest_shape(const dcol_shape_desc& d, int32_t idx, DevShape& S, std::vector<DevRow>& rows) {
    std::memset(&S, 0, sizeof(S));
    S.type = d.type;
    S.row_off = (int32_t)rows.size();
    for (int k = 0; k < 3; ++k) S.r_off[k] = d.r_offset[k];
    for (int k = 0; k < 9; ++k) S.Q_off[k] = d.Q_offset[k];
    {   // identity offsets: make_frame's products with them are exact no-ops and are skipped
        bool plain = true;
        for (int k = 0; k < 3; ++k) plain = plain && S.r_off[k] == 0.0;
        for (int k = 0; k < 9; ++k) plain = plain && S.Q_off[k] == ((k % 4 == 0) ? 1.0 : 0.0);
        S.plain = plain ? 1 : 0;
    }
    auto add = [&](double a0, double a1, double a2, double g3, double e0, double e1) {
        DevRow r;
        std::memset(&r, 0, sizeof(r));
        r.a[0] = a0; r.a[1] = a1; r.a[2] = a2; r.g3 = g3; r.ex[0] = e0; r.ex[1] = e1;
        rows.push_back(r);
    };
    switch (d.type) {
        case DCOL_POLYTOPE:   // G_ort = [A Qe', -b], h = A Qe' r   (:181-209)
            if (d.nh < 1 || !d.A || !d.b) return fail(DCOL_ERR_ARG, "shape " + std::to_string(idx) + ": polytope needs nh >= 1, A, b");
            for (int j = 0; j < d.nh; ++j) add(d.A[3 * j], d.A[3 * j + 1], d.A[3 * j + 2], -d.b[j], 0, 0);
            S.n_ort = d.nh;
            S.n_p = d.nh;
            S.soc_kind = SOC_NONE;
            if (d.nh == 6) {   // axis pairs: rows 3..5 the exact negatives of rows 0..2 (BOX kernels)
                bool bp = true;
                for (int j = 0; j < 3; ++j)
                    for (int c = 0; c < 3; ++c) bp = bp && d.A[3 * (j + 3) + c] == -d.A[3 * j + c];
                S.boxp = bp ? 1 : 0;
            }
            break;
        case DCOL_SPHERE:     // SOC only   (:151-178)
            S.n_ort = 0;
            S.soc_kind = SOC_BALL;
            S.R = d.R;
            break;
        case DCOL_CONE: {     // G_ort = [bx', -H/4], h = bx'r; SOC [-E Qe', -(tanb 3H/4) e0]   (:125-148)
            const double tb = std::tan(d.beta);
            add(1.0, 0.0, 0.0, -d.H / 4, 0, 0);
            S.n_ort = 1;
            S.n_p = 1;
            S.soc_kind = SOC_CONE;
            S.tanb = tb;
            S.cone_c = -(tb * 3 * d.H / 4);
            break;
        }
        case DCOL_CAPSULE:    // G_ort = [0 0 0 -L/2 +-1]   (:4-44)
            add(0, 0, 0, -d.L / 2, 1.0, 0);
            add(0, 0, 0, -d.L / 2, -1.0, 0);
            S.n_ort = 2;
            S.soc_kind = SOC_BALL;
            S.R = d.R;
            S.n_extra = 1;
            break;
        case DCOL_CYLINDER:   // capsule rows + [-+bx', -L/2, 0], h = -+bx'r   (:47-87)
            add(0, 0, 0, -d.L / 2, 1.0, 0);
            add(0, 0, 0, -d.L / 2, -1.0, 0);
            add(-1.0, 0, 0, -d.L / 2, 0, 0);
            add(1.0, 0, 0, -d.L / 2, 0, 0);
            S.n_ort = 4;
            S.n_p = 2;        // the two caps (extra-column rows first, as n_p requires)
            S.soc_kind = SOC_BALL;
            S.R = d.R;
            S.n_extra = 1;
            break;
        case DCOL_POLYGON:    // G_ort = [0 0 0 -b A], h = 0; SOC with Qe[:, :2]   (:90-120)
            if (d.nh < 1 || !d.A || !d.b) return fail(DCOL_ERR_ARG, "shape " + std::to_string(idx) + ": polygon needs nh >= 1, A, b");
            for (int j = 0; j < d.nh; ++j) add(0, 0, 0, -d.b[j], d.A[2 * j], d.A[2 * j + 1]);
            S.n_ort = d.nh;
            S.soc_kind = SOC_BALL;
            S.R = d.R;
            S.n_extra = 2;
            break;
        default:
            return fail(DCOL_ERR_ARG, "shape " + std::to_string(idx) + ": unknown type " + std::to_string(d.type));
    }
    return DCOL_SUCCESS;
}

struct PairClass {
    int32_t status;   // OK / UNSUPPORTED / TOO_LARGE
    int N, nsoc, o, omax, lpp;
    int oe = 0;       // row-partitioned bucket: extra-row slots (0: dense-row kernels)
};

// DCOL_NO_PART=1: no row-partitioned kernels (A/B runs, tests)
inline bool part_disabled() {
    static const bool off = std::getenv("DCOL_NO_PART") != nullptr;
    return off;
}

// DCOL_SPLIT=1: {capsule, cylinder} x polytope PART buckets with a split-SOC copy
// (variants.py SPLIT) run it, at two lanes per pair (opt-in A/B; off by default)
inline bool split_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("DCOL_SPLIT");
        return e && std::atoi(e) != 0;
    }();
    return on;
}
inline bool split_built(int N, int nsoc, int omax, int oe) {
    bool built = false;
#define DCOL_SPB(NN, NS, OM, LP, WP, FL, OEE) \
    if (NN == N && NS == nsoc && OM == omax && OEE == oe) built = true;
    DCOL_SPLIT_VARIANTS(DCOL_SPB)
#undef DCOL_SPB
    return built;
}

// Compiled LPP of a PART bucket: the first listed (throughput choice), DCOL_LPP=<n> if that
// one is compiled, or with latency = true the largest; 0 if the bucket has none (or not the
// forced one)
inline int part_lpp(int N, int nsoc, int omax, int oe, bool latency = false) {
    static const int forced = [] {
        const char* e = std::getenv("DCOL_LPP");
        return e ? std::atoi(e) : 0;
    }();
    int first = 0, best = 0, hit = 0;
#define DCOL_PL(NN, NS, OM, LP, WP, FL, OEE)                   \
    if (NN == N && NS == nsoc && OM == omax && OEE == oe) {    \
        if (first == 0) first = LP;                            \
        if (LP > best) best = LP;                              \
        if (forced == LP) hit = LP;                            \
    }
    DCOL_PART_VARIANTS(DCOL_PL)
#undef DCOL_PL
    if (latency) return best;
    if (forced) return hit;
    if (split_enabled() && split_built(N, nsoc, omax, oe)) return 2;
    return first;
}

// A PART kernel of the bucket at lpp whose SOC flavour a launch may use: ball rows (FL bit 1)
// only when every SOC block of the pair is a ball block (ball), else the dense SOC rows
inline bool part_flavour_built(int N, int nsoc, int omax, int oe, int lpp, bool ball) {
    bool built = false;
#define DCOL_PFB(NN, NS, OM, LP, WP, FL, OEE) \
    if (NN == N && NS == nsoc && OM == omax && OEE == oe && LP == lpp && (ball || (FL & 2) == 0)) built = true;
    DCOL_PART_VARIANTS(DCOL_PFB)
#undef DCOL_PFB
    return built;
}

// Row-partitioned bucket of a pair with op pose rows and oe extra-column rows (N = 5 / 6,
// one primitive with extra columns): the smallest (omax, oe) holding both, fewest slots
// first, then fewest extra slots (DCOL_PART_SHAPES is sorted that way per (N, NSOC));
// false if none fits.
inline bool part_bucket(int N, int nsoc, int op, int oe, PairClass& c) {
    bool found = false;
#define DCOL_PB(NN, NS, OM, OEE)                                                           \
    if (!found && NN == N && NS == nsoc && OM - OEE >= op && OEE >= oe && OEE > 0) {       \
        const int l = part_lpp(N, nsoc, OM, OEE);                                          \
        if (l > 0) {                                                                       \
            c.omax = OM;                                                                   \
            c.oe = OEE;                                                                    \
            c.lpp = l;                                                                     \
            found = true;                                                                  \
        }                                                                                  \
    }
    DCOL_PART_SHAPES(DCOL_PB)
#undef DCOL_PB
    return found;
}

// case4: DCOL_PLAN_CASE4 extension (both primitives with extra columns: n = 4 + e1 + e2);
// part: row-partitioned buckets allowed (DCOL_NO_PART unset)
inline PairClass classify(const DevShape& a, const DevShape& b, bool case4 = false, bool part = !part_disabled()) {
    PairClass c{DCOL_OK, 4, 0, 0, 0, 0};
    if (a.n_extra > 0 && b.n_extra > 0 && !case4) {   // combine_problem_matrices.py:58-67 (case 4)
        c.status = DCOL_UNSUPPORTED;
        return c;
    }
    c.N = 4 + a.n_extra + b.n_extra;
    c.nsoc = (a.soc_kind != SOC_NONE) + (b.soc_kind != SOC_NONE);
    c.o = a.n_ort + b.n_ort;
    if ((a.n_extra > 0) != (b.n_extra > 0) && part) {   // cases 1-3 with extra columns
        const int op = a.n_p + b.n_p;
        if (part_bucket(c.N, c.nsoc, op, c.o - op, c)) return c;
    }
    auto it = buckets().find({c.N, c.nsoc});
    if (it == buckets().end()) {
        c.status = DCOL_TOO_LARGE;
        return c;
    }
    for (int om : it->second)
        if (om >= std::max(c.o, 1)) {
            c.omax = om;
            c.lpp = choose_lpp(c.N, c.nsoc, om);
            return c;
        }
    c.status = DCOL_TOO_LARGE;
    return c;
}

}  // namespace dcol_host
