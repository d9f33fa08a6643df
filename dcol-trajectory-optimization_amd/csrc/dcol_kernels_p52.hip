// Row-partitioned kernels, N = 5, NSOC = 2 (dcol_kernels_part.inc).
#define DCOL_TU_N 5
#define DCOL_TU_NS 2
#define DCOL_TU_TAG p52
#define DCOL_TU_FN launch_part_n5s2
#include "dcol_kernels_part.inc"
