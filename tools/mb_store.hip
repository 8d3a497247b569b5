// mb_store.hip -- store-bandwidth ceilings for the k_eval write pattern on MI355X.
// Same bytes as one B = 512 evaluation of the 50x4x13 racetrack (~252 MB of writes).
//   A: one-wave workgroups (8 x 701 grid), 88 row stores of 512 B each (8 B / lane)
//   B: same grid, 44 stores of 1 KB (16 B / lane: two rows per instruction)
//   C: 256-thread workgroups, grid-stride 16 B / lane streaming stores (reference)
//   D: A plus 55 coalesced 512-B loads per wave from a 21 MB buffer (k_eval's read volume)
//   F, G: A and D with nontemporal stores
// Build: hipcc -O3 --offload-arch=gfx950 -o mb_store tools/mb_store.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

constexpr int B = 512, UNITS = 701, ROWS = 88;

__global__ __launch_bounds__(64) void kA(double* J, double v) {
    const long base = (long)blockIdx.y * ROWS * B + blockIdx.x * 64 + threadIdx.x;
#pragma unroll 8
    for (int i = 0; i < ROWS; ++i) J[base + (long)i * B] = v + i;
}

__global__ __launch_bounds__(64) void kB(double* J, double v) {
    const int l = threadIdx.x;
    const long base = (long)blockIdx.y * ROWS * B + blockIdx.x * 64 + (l >= 32 ? B : 0) + 2 * (l & 31);
#pragma unroll 8
    for (int i = 0; i < ROWS; i += 2) {
        double2 t = {v + i, v + i + 1};
        *reinterpret_cast<double2*>(J + base + (long)i * B) = t;
    }
}

__global__ __launch_bounds__(256) void kC(double2* J, long n2, double v) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n2; i += (long)gridDim.x * 256) J[i] = {v, v};
}

__global__ __launch_bounds__(64) void kD(double* J, const double* w, double v) {
    const long base = (long)blockIdx.y * ROWS * B + blockIdx.x * 64 + threadIdx.x;
    const long rb = (long)(blockIdx.y % 50) * 106 * B + blockIdx.x * 64 + threadIdx.x;
    double acc = v;
#pragma unroll 11
    for (int i = 0; i < 55; ++i) acc += w[rb + (long)i * B];
#pragma unroll 8
    for (int i = 0; i < ROWS; ++i) J[base + (long)i * B] = acc + i;
}

// F: A with nontemporal (streaming) stores; G: D with nontemporal stores
__global__ __launch_bounds__(64) void kF(double* J, double v) {
    const long base = (long)blockIdx.y * ROWS * B + blockIdx.x * 64 + threadIdx.x;
#pragma unroll 8
    for (int i = 0; i < ROWS; ++i) __builtin_nontemporal_store(v + i, J + base + (long)i * B);
}

__global__ __launch_bounds__(64) void kG(double* J, const double* w, double v) {
    const long base = (long)blockIdx.y * ROWS * B + blockIdx.x * 64 + threadIdx.x;
    const long rb = (long)(blockIdx.y % 50) * 106 * B + blockIdx.x * 64 + threadIdx.x;
    double acc = v;
#pragma unroll 11
    for (int i = 0; i < 55; ++i) acc += w[rb + (long)i * B];
#pragma unroll 8
    for (int i = 0; i < ROWS; ++i) __builtin_nontemporal_store(acc + i, J + base + (long)i * B);
}

// E: read 64 MiB once, 8 B / lane coalesced (FETCH_SIZE calibration for k_eval's load width)
__global__ __launch_bounds__(256) void kE(const double* x, long n, double* out) {
    double acc = 0;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) acc += x[i];
    if (acc == 1234.5) out[0] = acc;
}

int main() {
    const long n = (long)UNITS * ROWS * B * 8;   // doubles for 8 chunks
    const long nw = 5300L * B;
    double *J, *w;
    CHECK(hipMalloc(&J, n * sizeof(double) / 8 * 8));
    CHECK(hipMalloc(&w, nw * sizeof(double)));
    CHECK(hipMemset(w, 0, nw * sizeof(double)));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const double bytes = (double)UNITS * ROWS * 512.0 * 8;
    auto run = [&](const char* name, auto launch) {
        for (int i = 0; i < 5; ++i) launch();
        hipDeviceSynchronize();
        hipEventRecord(a);
        const int reps = 50;
        for (int i = 0; i < reps; ++i) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        const double us = ms * 1e3 / reps;
        printf("%-44s %8.1f us  %6.2f TB/s\n", name, us, bytes / (us * 1e-6) / 1e12);
    };
    dim3 g(8, UNITS);
    run("A one-wave WG, 8B/lane row stores", [&] { kA<<<g, 64>>>(J, 1.0); });
    run("B one-wave WG, 16B/lane paired stores", [&] { kB<<<g, 64>>>(J, 1.0); });
    run("C 256-thr grid-stride 16B/lane (2048 WG)", [&] { kC<<<2048, 256>>>((double2*)J, (long)(bytes / 16), 1.0); });
    run("D = A + 55 coalesced loads per wave", [&] { kD<<<g, 64>>>(J, w, 1.0); });
    run("F = A, nontemporal stores", [&] { kF<<<g, 64>>>(J, 1.0); });
    run("G = D, nontemporal stores", [&] { kG<<<g, 64>>>(J, w, 1.0); });
    double* big;
    const long nbig = 8L << 20;   // 64 MiB of doubles
    CHECK(hipMalloc(&big, nbig * sizeof(double)));
    CHECK(hipMemset(big, 0, nbig * sizeof(double)));
    hipEventRecord(a);
    kE<<<2048, 256>>>(big, nbig, J);
    hipEventRecord(b);
    hipEventSynchronize(b);
    printf("E read 64 MiB (8 B/lane) once: %ld bytes\n", nbig * 8);
    return 0;
}
