// Row-partitioned kernels, N = 6, NSOC = 2, ball-row copies (dcol_kernels_part.inc); the
// dense-row copies (cone partners) are dcol_kernels_p62d.hip.
#define DCOL_TU_N 6
#define DCOL_TU_FLOK(FL) (((FL) & 2) != 0)
#define DCOL_TU_NS 2
#define DCOL_TU_TAG p62
#define DCOL_TU_FN launch_part_n6s2
#include "dcol_kernels_part.inc"
