// TEST-ONLY (tests/emul): per-pair dispatch of the x86 solver build, one translation unit
// per primal dimension N (emul_n<N>.hip) so the variants compile in parallel.
#pragma once
#include "../../dcol-trajectory-optimization_amd/csrc/dcol_host.hpp"

namespace emul {
using namespace dcol;
using namespace dcol_host;

// Solves pair i of A with the variant the GPU plan would pick for class c (LPP = 1);
// false if no compiled shape matches.  One instantiation per (N, NSOC) and row form
// (emul_inst.hip, built once per combination by the Makefile, in parallel).
template <int X, int XS>
bool solve_n(const PairClass& c, bool full, bool ball, bool cone, bool box, const KArgs& A, int64_t i) {
#define DCOL_EMUL(NN, NS, OM)                                                      \
    if constexpr (NN == X && NS == XS) {                                           \
        if (c.omax == OM) {                                                        \
            if constexpr (NN == 4 && NS == 0 && OM == 12) {   /* variants.py BOX */ \
                if (full && box) {                                                 \
                    solve_one<NN, NS, OM, 1, true, false, false, 0, 0, false, true>(A, i, 0); \
                    return true;                                                   \
                }                                                                  \
            }                                                                      \
            if constexpr (NN == 4 && NS == 0) {   /* variants.py FULL shapes */    \
                if (full) {                                                        \
                    solve_one<NN, NS, OM, 1, true>(A, i, 0);                       \
                    return true;                                                   \
                }                                                                  \
            }                                                                      \
            if constexpr (NS > 0 && NN <= 6) {    /* variants.py ball() */         \
                if (ball) {                                                        \
                    solve_one<NN, NS, OM, 1, false, true>(A, i, 0);                \
                    return true;                                                   \
                }                                                                  \
            }                                                                      \
            if constexpr (NS > 0 && NN == 4 && OM <= 32) {   /* variants.py cone() */ \
                if (cone) {                                                        \
                    solve_one<NN, NS, OM, 1, false, false, true>(A, i, 0);         \
                    return true;                                                   \
                }                                                                  \
            }                                                                      \
            solve_one<NN, NS, OM, 1, false>(A, i, 0);                              \
            return true;                                                           \
        }                                                                          \
    }
    DCOL_SHAPES(DCOL_EMUL)
#undef DCOL_EMUL
    (void)c; (void)full; (void)ball; (void)cone; (void)box; (void)A; (void)i;
    return false;
}

// row-partitioned buckets (variants.py PART): BALL or dense SOC rows, FULL or padded
template <int X, int XS>
bool solve_part(const PairClass& c, bool full, bool ball, const KArgs& A, int64_t i) {
#define DCOL_EMUL_PART(NN, NS, OM, OEE)                                                        \
    if constexpr (NN == X && NS == XS) {                                                     \
        if (c.oe == OEE && c.omax == OM) {                                                   \
            if (ball) {                                                                      \
                if (full) solve_one<NN, NS, OM, 1, true, true, false, OEE>(A, i, 0);         \
                else solve_one<NN, NS, OM, 1, false, true, false, OEE>(A, i, 0);             \
            } else {                                                                         \
                if (full) solve_one<NN, NS, OM, 1, true, false, false, OEE>(A, i, 0);        \
                else solve_one<NN, NS, OM, 1, false, false, false, OEE>(A, i, 0);            \
            }                                                                                \
            return true;                                                                     \
        }                                                                                    \
    }
    DCOL_PART_SHAPES(DCOL_EMUL_PART)
#undef DCOL_EMUL_PART
    (void)c; (void)full; (void)ball; (void)A; (void)i;
    return false;
}

#define EMUL_SOLVE_DECL(X, XS)                                                                              \
    extern template bool solve_n<X, XS>(const PairClass&, bool, bool, bool, bool, const KArgs&, int64_t);        \
    extern template bool solve_part<X, XS>(const PairClass&, bool, bool, const KArgs&, int64_t);
EMUL_SOLVE_DECL(4, 0) EMUL_SOLVE_DECL(4, 1) EMUL_SOLVE_DECL(4, 2) EMUL_SOLVE_DECL(5, 1) EMUL_SOLVE_DECL(5, 2)
EMUL_SOLVE_DECL(6, 1) EMUL_SOLVE_DECL(6, 2) EMUL_SOLVE_DECL(7, 2) EMUL_SOLVE_DECL(8, 2)
#undef EMUL_SOLVE_DECL
}  // namespace emul
