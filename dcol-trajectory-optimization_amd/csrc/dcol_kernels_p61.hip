// Row-partitioned kernels, N = 6, NSOC = 1 (dcol_kernels_part.inc).
#define DCOL_TU_N 6
#define DCOL_TU_NS 1
#define DCOL_TU_TAG p61
#define DCOL_TU_FN launch_part_n6s1
#include "dcol_kernels_part.inc"
