// TEST-ONLY (tests/emul): x86 solver variants with N = 7
#include "emul_solve.hpp"

template bool emul::solve_n<7>(const dcol_host::PairClass&, bool, bool, bool, const dcol::KArgs&, int64_t);
