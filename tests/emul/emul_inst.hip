// TEST-ONLY (tests/emul): one (N, NSOC) instantiation of the x86 solver dispatch, built by
// the Makefile once per combination with -DEMUL_N=.. -DEMUL_NS=..; -DEMUL_PART=1 builds the
// row-partitioned buckets' dispatch instead (its own object, compiled in parallel), and
// -DEMUL_NO_PART_SHAPES=1 adds the (empty) one of a combination without PART buckets.
#include "emul_solve.hpp"

#if EMUL_PART
template bool emul::solve_part<EMUL_N, EMUL_NS>(const dcol_host::PairClass&, bool, bool, const dcol::KArgs&, int64_t);
#else
template bool emul::solve_n<EMUL_N, EMUL_NS>(const dcol_host::PairClass&, bool, bool, bool, bool, const dcol::KArgs&, int64_t);
#if EMUL_NO_PART_SHAPES
template bool emul::solve_part<EMUL_N, EMUL_NS>(const dcol_host::PairClass&, bool, bool, const dcol::KArgs&, int64_t);
#endif
#endif
