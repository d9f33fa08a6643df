// Accuracy of the kernel's reciprocal / reciprocal-square-root sequences on the GPU
// (dcol_device.hpp: frcp = v_rcp_f64 + 2 Newton steps, frcp1 = + 1 step, frsqrt =
// v_rsq_f64 + Goldschmidt/Newton refinement), against the correctly rounded values computed
// on the host (IEEE 1.0 / x; 1 / sqrt in long double, rounded).  Also the raw hardware
// estimates.  Inputs: 2^22 values log-uniform over [2^-60, 2^60] plus mantissa sweeps.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=on -I<csrc> rcp_ulp.hip -o rcp_ulp
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "dcol_device.hpp"

__global__ void probe(const double* x, double* out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double v = x[i];
    out[6 * i + 0] = __builtin_amdgcn_rcp(v);
    out[6 * i + 1] = dcol::frcp1(v);
    out[6 * i + 2] = dcol::frcp(v);
    out[6 * i + 3] = __builtin_amdgcn_rsq(v);
    out[6 * i + 4] = dcol::frsqrt(v);
    out[6 * i + 5] = v * dcol::frsqrt(v);   // sqrt as used by chol (d * idg)
}

static double ulp_of(double v) { return std::nextafter(std::fabs(v), INFINITY) - std::fabs(v); }

int main() {
    const int64_t n = 1 << 22;
    std::vector<double> x(n);
    std::mt19937_64 rng(42);
    std::uniform_real_distribution<double> e(-60.0, 60.0), m(1.0, 2.0);
    for (int64_t i = 0; i < n; ++i) x[i] = (i & 1) ? std::exp2(e(rng)) : std::ldexp(m(rng), (int)(i % 41) - 20);
    double *dx, *dout;
    if (hipMalloc(&dx, n * sizeof(double)) != hipSuccess || hipMalloc(&dout, 6 * n * sizeof(double)) != hipSuccess) return 1;
    hipMemcpy(dx, x.data(), n * sizeof(double), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3((n + 255) / 256), dim3(256), 0, 0, dx, dout, n);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::vector<double> out(6 * n);
    hipMemcpy(out.data(), dout, 6 * n * sizeof(double), hipMemcpyDeviceToHost);
    const char* names[6] = {"v_rcp_f64 (raw)", "frcp1 (rcp + 1 Newton)", "frcp (rcp + 2 Newton)",
                            "v_rsq_f64 (raw)", "frsqrt", "x * frsqrt(x) (sqrt)"};
    double maxe[6] = {0}, sume[6] = {0};
    int64_t exact[6] = {0};
    for (int64_t i = 0; i < n; ++i) {
        const double v = x[i];
        const double r = 1.0 / v;
        const long double rl = 1.0L / std::sqrt((long double)v);
        const double rs = (double)rl;
        const double sq = std::sqrt(v);
        const double ref[6] = {r, r, r, rs, rs, sq};
        for (int k = 0; k < 6; ++k) {
            const double err = std::fabs(out[6 * i + k] - ref[k]) / ulp_of(ref[k]);
            maxe[k] = std::fmax(maxe[k], err);
            sume[k] += err;
            exact[k] += out[6 * i + k] == ref[k];
        }
    }
    for (int k = 0; k < 6; ++k)
        std::printf("{\"op\": \"%s\", \"max_ulp\": %.4g, \"mean_ulp\": %.4g, \"correctly_rounded_frac\": %.6f, \"n\": %lld}\n",
                    names[k], maxe[k], sume[k] / n, (double)exact[k] / n, (long long)n);
    hipFree(dx);
    hipFree(dout);
    return 0;
}
