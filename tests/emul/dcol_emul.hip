// TEST-ONLY x86 build of the device solver (csrc/dcol_device.hpp: dcol::solve_one) so the
// kernel's arithmetic can be checked against the golden vectors in a container without a
// GPU.  Built by tests/emul/Makefile into tests/emul/libdcol_emul.so; loaded only by
// tests/test_emul_golden.py.  The product library (lib/libdcol.so) never runs this path.
#include <vector>

#include "emul_solve.hpp"

using namespace dcol;
using namespace dcol_host;

extern "C" int dcol_emul_batch(const dcol_shape_desc* shapes, int32_t n, int64_t B, const int32_t* s1,
                               const int32_t* s2, const double* pose1, const double* pose2, double tol,
                               int32_t max_iter, int32_t flags, double* alpha, double* contact, double* grad,
                               int32_t* iters, int32_t* status) {
    std::vector<DevShape> sh(n);
    std::vector<DevRow> rows;
    init_row_pool(rows);
    for (int32_t i = 0; i < n; ++i) {
        int rc = digest_shape(shapes[i], i, sh[i], rows);
        if (rc) return rc;
    }
    std::vector<double> p1(6 * B), p2(6 * B), ct(3 * B), gr(12 * B);
    for (int64_t i = 0; i < B; ++i)
        for (int q = 0; q < 6; ++q) {
            p1[q * B + i] = pose1[6 * i + q];
            p2[q * B + i] = pose2[6 * i + q];
        }
    KArgs A;
    A.shapes = sh.data();
    A.rows = rows.data();
    A.s1 = s1;
    A.s2 = s2;
    A.pose1 = p1.data();
    A.pose2 = p2.data();
    A.perm = nullptr;
    A.B = B;
    A.slot0 = 0;
    A.n = B;
    A.tol = tol;
    A.max_iter = max_iter;
    A.flags = flags;
    A.alpha = alpha;
    A.contact = ct.data();
    A.grad = gr.data();
    A.iters = iters;
    A.status = status;
    const bool no_ball = std::getenv("DCOL_NO_BALL") != nullptr;
    const bool no_cone = std::getenv("DCOL_NO_CONE") != nullptr;
    const bool part = std::getenv("DCOL_NO_PART") == nullptr;   // read per call (tests toggle it)
    const bool no_box = std::getenv("DCOL_NO_BOX") != nullptr;
    for (int64_t i = 0; i < B; ++i) {
        PairClass c = classify(sh[s1[i]], sh[s2[i]], false, part);
        if (c.status != DCOL_OK) {
            alpha[i] = __builtin_nan("");
            iters[i] = 0;
            status[i] = c.status;
            for (int q = 0; q < 3; ++q) ct[q * B + i] = __builtin_nan("");
            for (int q = 0; q < 12; ++q) gr[q * B + i] = __builtin_nan("");
            continue;
        }
        const bool full = c.o == c.omax;   // both loop specialisations, as the GPU launches pick them
                                           // (row-partitioned buckets: both slot kinds full)
        // ball-SOC specialisation as the GPU plans pick it (DCOL_NO_BALL: the dense rows)
        const bool ball = c.nsoc > 0 && sh[s1[i]].soc_kind != SOC_CONE && sh[s2[i]].soc_kind != SOC_CONE && !no_ball;
        // structured-cone specialisation (N = 4, every SOC block a cone; DCOL_NO_CONE: dense)
        const bool cone = c.nsoc > 0 && c.N == 4 && sh[s1[i]].soc_kind != SOC_BALL && sh[s2[i]].soc_kind != SOC_BALL &&
                          !no_cone;
        // box x box axis-pair rows (Solver<..., BOX>) as the GPU plans pick them (DCOL_NO_BOX:
        // the padding-free dense rows)
        const bool box = c.N == 4 && c.nsoc == 0 && c.omax == 12 && c.o == 12 && sh[s1[i]].boxp && sh[s2[i]].boxp &&
                         !no_box;
        bool done = false;
#define EMUL_CASE(NN, NS)                                                                     \
        if (c.N == NN && c.nsoc == NS)                                                        \
            done = c.oe > 0 ? emul::solve_part<NN, NS>(c, full, ball, A, i) : emul::solve_n<NN, NS>(c, full, ball, cone, box, A, i);
        EMUL_CASE(4, 0) EMUL_CASE(4, 1) EMUL_CASE(4, 2) EMUL_CASE(5, 1) EMUL_CASE(5, 2)
        EMUL_CASE(6, 1) EMUL_CASE(6, 2) EMUL_CASE(7, 2) EMUL_CASE(8, 2)
#undef EMUL_CASE
        if (done) continue;
        return fail(DCOL_ERR_ARG, "no variant");
    }
    for (int64_t i = 0; i < B; ++i) {
        for (int q = 0; q < 3; ++q) contact[3 * i + q] = ct[q * B + i];
        for (int q = 0; q < 12; ++q) grad[12 * i + q] = gr[q * B + i];
    }
    return DCOL_SUCCESS;
}
