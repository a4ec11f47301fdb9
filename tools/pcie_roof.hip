// pcie_roof.hip -- host<->device copy ceilings for the end-to-end path (DESIGN.md,
// end-to-end section): page-locked H2D and D2H alone, both directions at once on two
// streams, in 16 MiB pieces as the pipelined rewrite issues them.  Diagnostic tool.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

static double ms_between(hipEvent_t a, hipEvent_t b) {
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    const size_t total = 80u << 20, piece = 16u << 20;
    void *h_in, *h_out, *d_in, *d_out;
    if (hipHostMalloc(&h_in, total, 0) != hipSuccess || hipHostMalloc(&h_out, total, 0) != hipSuccess ||
        hipMalloc(&d_in, total) != hipSuccess || hipMalloc(&d_out, total) != hipSuccess)
        return 1;
    memset(h_in, 1, total);
    memset(h_out, 2, total);
    hipStream_t s1, s2;
    hipStreamCreate(&s1);
    hipStreamCreate(&s2);
    hipEvent_t e0, e1, e2;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventCreate(&e2);
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0, s1);
        for (size_t o = 0; o < total; o += piece)
            hipMemcpyAsync((char *)d_in + o, (char *)h_in + o, piece, hipMemcpyHostToDevice, s1);
        hipEventRecord(e1, s1);
        hipEventSynchronize(e1);
        const double h2d = ms_between(e0, e1);
        hipEventRecord(e0, s1);
        for (size_t o = 0; o < total; o += piece)
            hipMemcpyAsync((char *)h_out + o, (char *)d_out + o, piece, hipMemcpyDeviceToHost, s1);
        hipEventRecord(e1, s1);
        hipEventSynchronize(e1);
        const double d2h = ms_between(e0, e1);
        // both directions at once: H2D on s1, D2H on s2
        hipEventRecord(e0, s1);
        hipStreamWaitEvent(s2, e0, 0);
        for (size_t o = 0; o < total; o += piece) {
            hipMemcpyAsync((char *)d_in + o, (char *)h_in + o, piece, hipMemcpyHostToDevice, s1);
            hipMemcpyAsync((char *)h_out + o, (char *)d_out + o, piece, hipMemcpyDeviceToHost, s2);
        }
        hipEventRecord(e1, s1);
        hipEventRecord(e2, s2);
        hipEventSynchronize(e1);
        hipEventSynchronize(e2);
        const double both = ms_between(e0, e1) > ms_between(e0, e2) ? ms_between(e0, e1) : ms_between(e0, e2);
        printf("pcie 80 MiB in 16 MiB pieces: H2D %.3f ms (%.1f GB/s)  D2H %.3f ms (%.1f GB/s)  "
               "both at once %.3f ms (%.1f GB/s each way)\n",
               h2d, total / h2d / 1e6, d2h, total / d2h / 1e6, both, total / both / 1e6);
    }
    return 0;
}
