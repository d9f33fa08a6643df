// TEST-ONLY (tests/emul): x86 solver variants with N = 8
#include "emul_solve.hpp"

template bool emul::solve_n<8>(const dcol_host::PairClass&, bool, bool, bool, const dcol::KArgs&, int64_t);
