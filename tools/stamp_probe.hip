// Diagnostic build of the solver kernel with s_memtime stamps at phase boundaries
// (compiled with -DDCOL_STAMPS; never part of the library).  Workload = bench.py's config
// (random rect-prism pairs from a 64-shape table, r ~ U(-3,3)^3, p ~ U(-1,1)^3), own RNG.
//   hipcc -DDCOL_STAMPS --offload-arch=gfx950 -O3 -std=c++17 \
//         -I dcol-trajectory-optimization_amd/csrc tools/stamp_probe.hip -o /tmp/stamp_probe
//   /tmp/stamp_probe [pairs=100000] [flags=1 (FD) | 2 (envelope)]
// (-DDCOL_STAMPS_INIT: sub-phases of initialize() in place of PDIP iteration 2's)
// Prints mean cycles per phase (per pair group, lane 0's s_memtime) and the per-wave
// (32 pairs) critical phase lengths.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "dcol_host.hpp"

#ifndef DCOL_PROBE_FL
#define DCOL_PROBE_FL 1   // variants.py FL of the probed copy (1: FULL, as the library launches box x box)
#endif

using namespace dcol;
using namespace dcol_host;

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e = (x);                                                   \
        if (e != hipSuccess) {                                                \
            std::printf("%s: %s\n", #x, hipGetErrorString(e));                \
            std::exit(1);                                                     \
        }                                                                     \
    } while (0)

int main(int argc, char** argv) {
    const int64_t B = argc > 1 ? std::atoll(argv[1]) : 100000;
    const int flags = argc > 2 ? std::atoi(argv[2]) : 1;
    constexpr int NS = 64;
    std::mt19937_64 rng(0);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    std::vector<double> A(NS * 18), b(NS * 6);
    std::vector<dcol_shape_desc> descs(NS);
    for (int k = 0; k < NS; ++k) {
        const double d[3] = {0.2 + 1.8 * U(rng), 0.2 + 1.8 * U(rng), 0.2 + 1.8 * U(rng)};
        const double nrm[6][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {-1, 0, 0}, {0, -1, 0}, {0, 0, -1}};
        for (int j = 0; j < 6; ++j) {
            for (int c = 0; c < 3; ++c) A[k * 18 + 3 * j + c] = nrm[j][c];
            b[k * 6 + j] = d[j % 3] / 2;
        }
        dcol_shape_desc& s = descs[k];
        std::memset(&s, 0, sizeof(s));
        s.type = DCOL_POLYTOPE;
        s.nh = 6;
        s.A = &A[k * 18];
        s.b = &b[k * 6];
        s.Q_offset[0] = s.Q_offset[4] = s.Q_offset[8] = 1.0;
    }
    std::vector<DevShape> sh(NS);
    std::vector<DevRow> rows;
    init_row_pool(rows);
    for (int k = 0; k < NS; ++k) digest_shape(descs[k], k, sh[k], rows);
    std::vector<int32_t> s1(B), s2(B);
    std::vector<double> p1(6 * B), p2(6 * B);
    for (int64_t i = 0; i < B; ++i) {
        s1[i] = (int32_t)(U(rng) * NS);
        s2[i] = (int32_t)(U(rng) * NS);
        for (int c = 0; c < 6; ++c) {
            p1[c * B + i] = c < 3 ? -3 + 6 * U(rng) : -1 + 2 * U(rng);
            p2[c * B + i] = c < 3 ? -3 + 6 * U(rng) : -1 + 2 * U(rng);
        }
    }
    DevShape* dsh;
    DevRow* drw;
    int32_t *ds1, *ds2, *dit, *dst;
    double *dp1, *dp2, *dal, *dgr;
    unsigned long long* dstamp;
    CK(hipMalloc(&dsh, sizeof(DevShape) * NS));
    CK(hipMalloc(&drw, sizeof(DevRow) * rows.size()));
    CK(hipMalloc(&ds1, 4 * B));
    CK(hipMalloc(&ds2, 4 * B));
    CK(hipMalloc(&dit, 4 * B));
    CK(hipMalloc(&dst, 4 * B));
    CK(hipMalloc(&dp1, 48 * B));
    CK(hipMalloc(&dp2, 48 * B));
    CK(hipMalloc(&dal, 8 * B));
    CK(hipMalloc(&dgr, 96 * B));
    CK(hipMalloc(&dstamp, 128 * B));
    CK(hipMemcpy(dsh, sh.data(), sizeof(DevShape) * NS, hipMemcpyHostToDevice));
    CK(hipMemcpy(drw, rows.data(), sizeof(DevRow) * rows.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(ds1, s1.data(), 4 * B, hipMemcpyHostToDevice));
    CK(hipMemcpy(ds2, s2.data(), 4 * B, hipMemcpyHostToDevice));
    CK(hipMemcpy(dp1, p1.data(), 48 * B, hipMemcpyHostToDevice));
    CK(hipMemcpy(dp2, p2.data(), 48 * B, hipMemcpyHostToDevice));
    CK(hipMemset(dstamp, 0, 128 * B));
    KArgs a;
    std::memset(&a, 0, sizeof(a));
    a.shapes = dsh; a.rows = drw; a.s1 = ds1; a.s2 = ds2; a.pose1 = dp1; a.pose2 = dp2; a.perm = nullptr;
    a.B = B; a.slot0 = 0; a.n = B; a.tol = 1e-6; a.max_iter = 50; a.flags = flags;
    a.alpha = dal; a.contact = nullptr; a.grad = dgr; a.iters = dit; a.status = dst; a.stamps = dstamp;
    constexpr int LPP = 2;
    const int64_t grid = (B * LPP + kSolveBlock - 1) / kSolveBlock;
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL((prox_kernel<4, 0, 12, LPP, 2, DCOL_PROBE_FL>), dim3(grid), dim3(kSolveBlock), 0, 0, a);
        CK(hipDeviceSynchronize());
    }
    std::vector<unsigned long long> st(16 * B);
    std::vector<int32_t> it(B), stat(B);
    CK(hipMemcpy(st.data(), dstamp, 128 * B, hipMemcpyDeviceToHost));
    CK(hipMemcpy(it.data(), dit, 4 * B, hipMemcpyDeviceToHost));
    CK(hipMemcpy(stat.data(), dst, 4 * B, hipMemcpyDeviceToHost));
    const char* names[5] = {"loads+frames", "assembly", "initialize", "pdip loop", "gradient"};
    double sum[5] = {0}, wmax[5] = {0};
    const int PW = 64 / LPP;   // pairs per wave
    double it_mean = 0, it_wmax = 0;
    unsigned long long t_first = ~0ull, t_last = 0;
    for (int64_t i = 0; i < B; ++i) {
        for (int k = 0; k < 5; ++k) sum[k] += (double)(st[16 * i + k + 1] - st[16 * i + k]);
        it_mean += it[i];
        t_first = std::min(t_first, st[16 * i]);
        t_last = std::max(t_last, st[16 * i + 5]);
    }
    for (int64_t w = 0; w * PW < B; ++w) {
        double m[5] = {0};
        int im = 0;
        for (int64_t i = w * PW; i < std::min<int64_t>(B, (w + 1) * PW); ++i) {
            for (int k = 0; k < 5; ++k) m[k] = std::max(m[k], (double)(st[16 * i + k + 1] - st[16 * i + k]));
            im = std::max(im, it[i]);
        }
        for (int k = 0; k < 5; ++k) wmax[k] += m[k];
        it_wmax += im;
    }
    const double nw = (double)((B + PW - 1) / PW);
    std::printf("pairs %lld flags %d  mean iters %.3f  mean per-wave max iters %.3f\n", (long long)B, flags, it_mean / B,
                it_wmax / nw);
    for (int k = 0; k < 5; ++k)
        std::printf("  %-14s mean %9.0f cyc/pair   per-wave max %9.0f cyc\n", names[k], sum[k] / B, wmax[k] / nw);
    // sub-phases of PDIP iteration 2 (pairs that reached it), or with -DDCOL_STAMPS_INIT of
    // initialize()
#ifdef DCOL_STAMPS_INIT
    const char* sub[7] = {"G'G, G'h + sums", "chol + solve", "r = G x - h", "bring2cone(s)",
                          "L^-T y, G x_z", "bring2cone(z)", "s, z select"};
#else
    const char* sub[7] = {"NT + normal matrix", "Cholesky", "predictor + bound", "rho, sigma, cp",
                          "corrector rhs", "corrector bound", "update"};
#endif
    double ss[7] = {0};
    int64_t cnt = 0;
    for (int64_t i = 0; i < B; ++i) {
        const unsigned long long* t = &st[16 * i + 8];
        if (t[0] == 0 || t[7] == 0) continue;
        ++cnt;
        for (int k = 0; k < 7; ++k) ss[k] += (double)(t[k + 1] - t[k]);
    }
#ifdef DCOL_STAMPS_INIT
    std::printf("  initialize (%lld pairs):\n", (long long)cnt);
#else
    std::printf("  iteration 2 (%lld pairs):\n", (long long)cnt);
#endif
    for (int k = 0; k < 7; ++k) std::printf("    %-20s %8.0f cyc\n", sub[k], cnt ? ss[k] / cnt : 0.0);
    return 0;
}
