// Row-partitioned kernels, N = 5, NSOC = 1 (dcol_kernels_part.inc).
#define DCOL_TU_N 5
#define DCOL_TU_NS 1
#define DCOL_TU_TAG p51
#define DCOL_TU_FN launch_part_n5s1
#include "dcol_kernels_part.inc"
