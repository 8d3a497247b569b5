// mb_store_scale.hip -- HBM store bandwidth against the written volume on MI355X: does the k_eval
// write stream (252 MB per launch at B = 512, 2.2 GB at B = 4096) run at the same rate once it no
// longer fits the 256 MB MALL? Streaming 16-byte stores (grid-stride, 256-thread workgroups) and the
// k_eval pattern (one-wave workgroups, 88 rows of 8 B per lane, [row][B] interleaved) over B.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/mb_store_scale tools/mb_store_scale.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

__global__ __launch_bounds__(256) void k_stream(double2* J, long n2, double v) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n2; i += (long)gridDim.x * 256) J[i] = {v, v};
}

constexpr int ROWS = 88, UNITS = 701;

__global__ __launch_bounds__(64) void k_rows(double* J, int B, double v) {
    const long base = (long)blockIdx.y * ROWS * B + blockIdx.x * 64 + threadIdx.x;
#pragma unroll 8
    for (int i = 0; i < ROWS; ++i) J[base + (long)i * B] = v + i;
}

int main() {
    const size_t max_bytes = (size_t)4 << 30;
    double* J;
    CHECK(hipMalloc((void**)&J, max_bytes));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const size_t sizes_mb[] = {128, 256, 512, 1024, 2200, 4096};
    for (size_t mb : sizes_mb) {
        const size_t bytes = mb << 20;
        const long n2 = (long)(bytes / 16);
        float best = 1e30f;
        for (int r = 0; r < 6; ++r) {
            CHECK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_stream, dim3(256 * 64), dim3(256), 0, 0, (double2*)J, n2, 1.0 + r);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (r > 0 && ms < best) best = ms;
        }
        printf("{\"kernel\": \"stream16\", \"MB\": %zu, \"ms\": %.4f, \"TBps\": %.3f}\n", mb, best, bytes / (best * 1e-3) / 1e12);
    }
    const int batches[] = {512, 1024, 2048, 4096, 8192};
    for (int B : batches) {
        const size_t bytes = (size_t)UNITS * ROWS * B * 8;
        if (bytes > max_bytes) break;
        float best = 1e30f;
        for (int r = 0; r < 6; ++r) {
            CHECK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_rows, dim3(B / 64, UNITS), dim3(64), 0, 0, J, B, 1.0 + r);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (r > 0 && ms < best) best = ms;
        }
        printf("{\"kernel\": \"rows8\", \"B\": %d, \"MB\": %.1f, \"ms\": %.4f, \"TBps\": %.3f}\n", B, bytes / 1048576.0, best,
               bytes / (best * 1e-3) / 1e12);
    }
    CHECK(hipFree(J));
    return 0;
}
