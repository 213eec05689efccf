// Microbenchmark: HBM write rate of 8-byte-per-lane (512 B per wave) stores
// under two item orders of the voting_for_hypothesis byte mask:
//   A: wave = one window, loops over 64 rows 2.15 MB apart (current kernel)
//   B: neighbouring waves take neighbouring windows of the same rows
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_store(uint8_t *out, int64_t rstep, int nwin, int nrows, int order, int items_per_wave) {
    const int wave = blockIdx.x * 4 + threadIdx.x / 64, lane = threadIdx.x & 63;
    const int nitems = 72 * nwin;   // (v, c) pairs x windows, 64 rows each
    for (int it = 0; it < items_per_wave; ++it) {
        int item = wave * items_per_wave + it;
        if (order == 1) item = it * (gridDim.x * 4) + wave;
        if (item >= nitems) return;
        int w = item % nwin, vc = item / nwin;
        uint8_t *p = out + (int64_t)vc * 29861 + (int64_t)w * 512 + lane * 8;
        for (int i = 0; i < nrows; ++i) *(uint2 *)(p + rstep * i) = make_uint2(i, i);
    }
}

int main() {
    const int64_t tn = 29861, vn = 9, hn = 512;
    const int64_t bytes = hn * vn * tn + 4096;
    uint8_t *out;
    if (hipMalloc(&out, bytes) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int nwin = (int)((tn + 7 + 511) / 512);
    const int64_t rstep = 8 * vn * tn;
    const int nitems = 72 * nwin;
    for (int order = 0; order < 2; ++order) {
        for (int ipw = 1; ipw <= 2; ++ipw) {
            int waves = (nitems + ipw - 1) / ipw;
            int blocks = (waves + 3) / 4;
            k_store<<<blocks, 256>>>(out, rstep, nwin, 64, order, ipw);
            (void)hipEventRecord(e0);
            for (int r = 0; r < 10; ++r) k_store<<<blocks, 256>>>(out, rstep, nwin, 64, order, ipw);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            double b = (double)nitems * 64 * 512;
            printf("order %c items/wave %d: %.1f us  %.0f GB/s\n", order ? 'B' : 'A', ipw, ms * 100, b / (ms / 10) / 1e6);
        }
    }
    return 0;
}
