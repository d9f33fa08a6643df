// TEST-ONLY (tests/emul): per-pair dispatch of the x86 solver build, one translation unit
// per primal dimension N (emul_n<N>.hip) so the variants compile in parallel.
#pragma once
#include "../../dcol-trajectory-optimization_amd/csrc/dcol_host.hpp"

namespace emul {
using namespace dcol;
using namespace dcol_host;

// Solves pair i of A with the variant the GPU plan would pick for class c (LPP = 1);
// false if no compiled shape matches.
template <int X>
bool solve_n(const PairClass& c, bool full, bool ball, bool cone, const KArgs& A, int64_t i) {
#define DCOL_EMUL(NN, NS, OM)                                                      \
    if constexpr (NN == X) {                                                       \
        if (c.nsoc == NS && c.omax == OM) {                                        \
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
    (void)c; (void)full; (void)ball; (void)cone; (void)A; (void)i;
    return false;
}

extern template bool solve_n<4>(const PairClass&, bool, bool, bool, const KArgs&, int64_t);
extern template bool solve_n<5>(const PairClass&, bool, bool, bool, const KArgs&, int64_t);
extern template bool solve_n<6>(const PairClass&, bool, bool, bool, const KArgs&, int64_t);
extern template bool solve_n<7>(const PairClass&, bool, bool, bool, const KArgs&, int64_t);
extern template bool solve_n<8>(const PairClass&, bool, bool, bool, const KArgs&, int64_t);
}  // namespace emul
