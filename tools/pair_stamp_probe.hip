// Diagnostic (never part of the library): per-phase cycles of ONE pair solved alone -- the
// drop-in's single-pair latency (dcol_prox_pair) -- for the quadrotor hallway's pair kinds
// at their latency configurations, with s_memtime stamps at the phase boundaries
// (-DDCOL_STAMPS, dcol_device.hpp DCOL_STAMP).
//   hipcc -DDCOL_STAMPS --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=on \
//         -I dcol-trajectory-optimization_amd/csrc tools/pair_stamp_probe.hip -o tools/bin/pair_stamp_probe
//   tools/bin/pair_stamp_probe [reps=200]
// Prints, per kind and per flags (contact only = proximity_mrp, FD gradient =
// proximity_gradient), the median cycles of each phase over `reps` one-pair launches.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "dcol_host.hpp"

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

struct Dev {
    DevShape* sh;
    DevRow* rw;
    int32_t *s1, *s2, *it, *st;
    double *p1, *p2, *al, *ct, *gr;
    unsigned long long* stamp;
};

template <int N, int NS, int OM, int LP, int WP, int FL>
void probe(const char* name, const Dev& d, int reps) {
    const char* names[5] = {"loads+frames", "assembly", "initialize", "pdip loop", "gradient"};
    for (const int flags : {4 /* contact */, 1 /* FD gradient */}) {
        KArgs a;
        std::memset(&a, 0, sizeof(a));
        a.shapes = d.sh; a.rows = d.rw; a.s1 = d.s1; a.s2 = d.s2; a.pose1 = d.p1; a.pose2 = d.p2;
        a.B = 1; a.slot0 = 0; a.n = 1; a.tol = 1e-6; a.max_iter = 50; a.flags = flags;
        a.alpha = d.al; a.contact = d.ct; a.grad = d.gr; a.iters = d.it; a.status = d.st; a.stamps = d.stamp;
        std::vector<std::vector<double>> ph(6), sub(7);
        int iters = 0, status = 0;
        for (int r = 0; r < reps; ++r) {
            CK(hipMemset(d.stamp, 0, 128));   // (16 stamps: phases 0-5, iteration-2 sub-phases 8-15)
            hipLaunchKernelGGL((prox_kernel<N, NS, OM, LP, WP, FL>), dim3(1), dim3(kSolveBlock), 0, 0, a);
            CK(hipDeviceSynchronize());
            unsigned long long s[16];
            CK(hipMemcpy(s, d.stamp, 128, hipMemcpyDeviceToHost));
            for (int k = 0; k < 5; ++k) ph[k].push_back((double)(s[k + 1] - s[k]));
            ph[5].push_back((double)(s[5] - s[0]));
            if (s[8] && s[15])
                for (int k = 0; k < 7; ++k) sub[k].push_back((double)(s[9 + k] - s[8 + k]));
            CK(hipMemcpy(&iters, d.it, 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(&status, d.st, 4, hipMemcpyDeviceToHost));
        }
        std::printf("%-16s <%d,%d,%d,LPP %d,FL %d> %s  iters %d status %d\n", name, N, NS, OM, LP, FL,
                    flags == 1 ? "FD gradient" : "contact    ", iters, status);
        for (int k = 0; k < 6; ++k) {
            std::sort(ph[k].begin(), ph[k].end());
            std::printf("    %-14s %8.0f cyc\n", k < 5 ? names[k] : "total", ph[k][ph[k].size() / 2]);
        }
        const char* subn[7] = {"NT + normal matrix", "Cholesky", "predictor + bound", "rho, sigma, cp",
                               "corrector rhs", "corrector bound", "update"};
        for (int k = 0; k < 7 && !sub[k].empty(); ++k) {
            std::sort(sub[k].begin(), sub[k].end());
            std::printf("      it2 %-18s %6.0f cyc\n", subn[k], sub[k][sub[k].size() / 2]);
        }
    }
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 200;
    // shapes: 0 sphere R 0.25 (the quadrotor's victim), 1 box 1 x 2 x 0.5, 2 sphere R 0.6
    std::vector<dcol_shape_desc> descs(3);
    for (auto& s : descs) {
        std::memset(&s, 0, sizeof(s));
        s.Q_offset[0] = s.Q_offset[4] = s.Q_offset[8] = 1.0;
    }
    descs[0].type = DCOL_SPHERE;
    descs[0].R = 0.25;
    double A[18], b[6];
    const double nrm[6][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {-1, 0, 0}, {0, -1, 0}, {0, 0, -1}};
    const double hd[3] = {0.5, 1.0, 0.25};
    for (int j = 0; j < 6; ++j) {
        for (int c = 0; c < 3; ++c) A[3 * j + c] = nrm[j][c];
        b[j] = hd[j % 3];
    }
    descs[1].type = DCOL_POLYTOPE;
    descs[1].nh = 6;
    descs[1].A = A;
    descs[1].b = b;
    descs[2].type = DCOL_SPHERE;
    descs[2].R = 0.6;
    std::vector<DevShape> sh(3);
    std::vector<DevRow> rows;
    init_row_pool(rows);
    for (int k = 0; k < 3; ++k) digest_shape(descs[k], k, sh[k], rows);
    Dev d;
    CK(hipMalloc(&d.sh, sizeof(DevShape) * 3));
    CK(hipMalloc(&d.rw, sizeof(DevRow) * rows.size()));
    CK(hipMalloc(&d.s1, 4));
    CK(hipMalloc(&d.s2, 4));
    CK(hipMalloc(&d.it, 4));
    CK(hipMalloc(&d.st, 4));
    CK(hipMalloc(&d.p1, 48));
    CK(hipMalloc(&d.p2, 48));
    CK(hipMalloc(&d.al, 8));
    CK(hipMalloc(&d.ct, 24));
    CK(hipMalloc(&d.gr, 96));
    CK(hipMalloc(&d.stamp, 128));
    CK(hipMemcpy(d.sh, sh.data(), sizeof(DevShape) * 3, hipMemcpyHostToDevice));
    CK(hipMemcpy(d.rw, rows.data(), sizeof(DevRow) * rows.size(), hipMemcpyHostToDevice));
    const double p1[6] = {1.3, 0.4, 0.9, 0.05, -0.1, 0.2}, p2[6] = {0.0, 0.0, 0.0, 0.1, 0.2, -0.15};
    CK(hipMemcpy(d.p1, p1, 48, hipMemcpyHostToDevice));
    CK(hipMemcpy(d.p2, p2, 48, hipMemcpyHostToDevice));
    int32_t k1 = 0, k2 = 1;
    CK(hipMemcpy(d.s1, &k1, 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d.s2, &k2, 4, hipMemcpyHostToDevice));
    probe<4, 1, 8, 8, 2, 2>("sphere x box", d, reps);      // the latency configuration (8-row bucket, 8 lanes)
    probe<4, 1, 8, 2, 1, 2>("sphere x box", d, reps);
    probe<4, 1, 6, 2, 2, 2>("sphere x box", d, reps);
    probe<4, 1, 6, 1, 1, 2>("sphere x box", d, reps);
    k2 = 2;
    CK(hipMemcpy(d.s2, &k2, 4, hipMemcpyHostToDevice));
    probe<4, 2, 2, 2, 2, 2>("sphere x sphere", d, reps);
    return 0;
}
