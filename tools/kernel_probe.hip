// Headline solve kernel timed on its own (no library, no torch): prox_kernel<4, 0, 12, 2, 2, 1>
// on bench.py's configs[3] distribution (random rect-prism pairs from a 64-shape table, own
// RNG), HIP events around back-to-back launches on one stream after a warm-up -- for A/B
// builds of dcol_device.hpp variants (-I <dir with the variant header>) in seconds.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=on \
//         -I dcol-trajectory-optimization_amd/csrc tools/kernel_probe.hip -o tools/bin/kernel_probe
//   tools/bin/kernel_probe [pairs=100000] [launches=500] [warmup=200]
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
    CK(hipMemcpy(dsh, sh.data(), sizeof(DevShape) * NS, hipMemcpyHostToDevice));
    CK(hipMemcpy(drw, rows.data(), sizeof(DevRow) * rows.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(ds1, s1.data(), 4 * B, hipMemcpyHostToDevice));
    CK(hipMemcpy(ds2, s2.data(), 4 * B, hipMemcpyHostToDevice));
    CK(hipMemcpy(dp1, p1.data(), 48 * B, hipMemcpyHostToDevice));
    CK(hipMemcpy(dp2, p2.data(), 48 * B, hipMemcpyHostToDevice));
    KArgs a;
    std::memset(&a, 0, sizeof(a));
    a.shapes = dsh; a.rows = drw; a.s1 = ds1; a.s2 = ds2; a.pose1 = dp1; a.pose2 = dp2; a.perm = nullptr;
    a.B = B; a.slot0 = 0; a.n = B; a.tol = 1e-6; a.max_iter = 50; a.flags = flags;
    a.alpha = dal; a.contact = nullptr; a.grad = dgr; a.iters = dit; a.status = dst;
    constexpr int LPP = 2;
    const int64_t grid = (B * LPP + kSolveBlock - 1) / kSolveBlock;
    const int launches = argc > 2 ? std::atoi(argv[2]) : 500;
    const int warm = argc > 3 ? std::atoi(argv[3]) : 200;
    for (int rep = 0; rep < warm; ++rep)
        hipLaunchKernelGGL((prox_kernel<4, 0, 12, LPP, 2, DCOL_PROBE_FL>), dim3(grid), dim3(kSolveBlock), 0, 0, a);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ms(launches);
    for (int rep = 0; rep < launches; ++rep) {
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL((prox_kernel<4, 0, 12, LPP, 2, DCOL_PROBE_FL>), dim3(grid), dim3(kSolveBlock), 0, 0, a);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms[rep], e0, e1));
    }
    std::vector<int32_t> it(B);
    CK(hipMemcpy(it.data(), dit, 4 * B, hipMemcpyDeviceToHost));
    double isum = 0;
    for (int64_t i = 0; i < B; ++i) isum += it[i];
    std::sort(ms.begin(), ms.end());
    double mean = 0;
    for (float v : ms) mean += v;
    mean /= launches;
    std::printf("pairs %lld launches %d  kernel us: mean %.2f  median %.2f  min %.2f  (mean iters %.3f)\n", (long long)B,
                launches, 1e3 * mean, 1e3 * ms[launches / 2], 1e3 * ms[0], isum / B);
    return 0;
}
