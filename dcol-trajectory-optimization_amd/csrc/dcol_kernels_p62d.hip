// Row-partitioned kernels, N = 6, NSOC = 2, dense-SOC-row copies (cone x polygon / polygon x
// cone; dcol_kernels_part.inc), apart from the ball-row copies (dcol_kernels_p62.hip) so that
// each runs under its faster machine schedule (Makefile SCHED_XPOLY)
#define DCOL_TU_N 6
#define DCOL_TU_NS 2
#define DCOL_TU_FLOK(FL) (((FL) & 2) == 0)
#define DCOL_TU_TAG p62d
#define DCOL_TU_FN launch_part_n6s2_dense
#include "dcol_kernels_part.inc"
