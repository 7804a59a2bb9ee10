// Micro-benchmark of the suffstats kernel on synthetic sorted labels (development tool).
#include "../noparama_amd/csrc/np8_kernels.hip"

#include <cstdio>
#include <vector>

__global__ void just_read(const double *X, const int32_t *z, int64_t n, double *out) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    double s = z[p];
    for (int a = 0; a < 8; ++a) s += X[a * n + p];
    if (s == 12345.678) out[0] = s;
}

int main(int argc, char **argv) {
    const int64_t n = 1000000;
    const int D = 8, K = 64, W = D + D * (D + 1) / 2;
    const int mode = argc > 1 ? atoi(argv[1]) : 0;  // 0 sorted, 1 random labels, 2 sorted + 1% movers
    std::vector<double> X(n * D);
    std::vector<int32_t> z(n);
    for (int64_t i = 0; i < n; ++i) {
        z[i] = mode == 1 ? (int32_t)((i * 2654435761ull) % K) : (int32_t)(i * K / n);
        if (mode == 2 && i % 97 == 0) z[i] = (z[i] + 1) % K;
        for (int a = 0; a < D; ++a) X[a * n + i] = z[i] + 0.01 * ((i * 31 + a) % 100);
    }
    double *dX, *dacc, *dmu, *dout;
    int32_t *dz, *dcnt;
    Ctl *ctl;
    hipMalloc(&dX, n * D * 8);
    hipMalloc(&dz, n * 4);
    hipMalloc(&dacc, K * W * 8);
    hipMalloc(&dmu, K * D * 8);
    hipMalloc(&dout, 8);
    hipMalloc(&dcnt, K * 4);
    hipMalloc(&ctl, sizeof(Ctl));
    hipMemset(ctl, 0, sizeof(Ctl));
    hipMemset(dmu, 0, K * D * 8);
    hipMemcpy(dX, X.data(), n * D * 8, hipMemcpyHostToDevice);
    hipMemcpy(dz, z.data(), n * 4, hipMemcpyHostToDevice);
    ParamArgs A{};
    A.X = dX;
    A.z = dz;
    A.sorted = 0;
    A.n_loc = n;
    A.kcap = K;
    A.D = D;
    A.acc = dacc;
    A.slot_mu = dmu;
    A.ctl = ctl;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 3; ++rep) {
        hipMemset(dacc, 0, K * W * 8);
        hipEventRecord(e0);
        for (int it = 0; it < 20; ++it) np8_launch_suffstats(A, 0);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        hipEventRecord(e0);
        for (int it = 0; it < 20; ++it) hipLaunchKernelGGL(just_read, dim3((n + 255) / 256), dim3(256), 0, 0, dX, dz, n, dout);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms2;
        hipEventElapsedTime(&ms2, e0, e1);
        printf("mode %d: suffstats %.2f us/launch, plain read %.2f us/launch\n", mode, ms * 50, ms2 * 50);
    }
    std::vector<double> acc(K * W);
    hipMemcpy(acc.data(), dacc, K * W * 8, hipMemcpyDeviceToHost);
    printf("acc[0]=%g (expect %g)\n", acc[0] / 20, 0.0);
    return 0;
}
