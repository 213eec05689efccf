// Microbenchmark: HBM write rate of the voting_for_hypothesis byte mask
// (512 hyp x 9 kp rows of 29,861 bytes) with 8-byte vs 16-byte stores per
// lane: wave = one window of 64 rows, window = 64 lanes x W bytes.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int W, bool NT>
__global__ void k_store(uint8_t *out, int64_t rstep, int nwin, int nrows) {
    const int wave = blockIdx.x * 4 + threadIdx.x / 64, lane = threadIdx.x & 63;
    const int split = 64 / nrows;
    const int nitems = 72 * nwin * split;
    if (wave >= nitems) return;
    const int part = wave % split, it = wave / split;
    const int w = it % nwin, vc = it / nwin;
    uint8_t *p = out + (int64_t)vc * 29861 + (int64_t)w * (64 * W) + lane * W + rstep * (int64_t)(part * nrows);
    for (int i = 0; i < nrows; ++i) {
        if (NT) {
            if (W == 8) __builtin_nontemporal_store((unsigned long long)i * 0x100000001ull, (unsigned long long *)(p + rstep * i));
            else {
                typedef unsigned int v4u __attribute__((ext_vector_type(4)));
                v4u x = {(unsigned)i, (unsigned)i, (unsigned)i, (unsigned)i};
                __builtin_nontemporal_store(x, (v4u *)(p + rstep * i));
            }
        } else {
            if (W == 8) *(uint2 *)(p + rstep * i) = make_uint2(i, i);
            else *(uint4 *)(p + rstep * i) = make_uint4(i, i, i, i);
        }
    }
}

int main() {
    const int64_t tn = 29861, vn = 9, hn = 512;
    uint8_t *out;
    if (hipMalloc(&out, hn * vn * tn + 65536) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int64_t rstep = 8 * vn * tn;
    for (int cfg = 0; cfg < 12; ++cfg) {
        const int W = (cfg % 6) < 3 ? 8 : 16, nrows = 64 >> (cfg % 3);
        const bool nt = cfg >= 6;
        const int nwin = (int)((tn + 15 + 64 * W - 1) / (64 * W));
        const int waves = 72 * nwin * (64 / nrows), blocks = (waves + 3) / 4;
        auto go = [&]() {
            if (nt) {
                if (W == 8) k_store<8, true><<<blocks, 256>>>(out, rstep, nwin, nrows);
                else k_store<16, true><<<blocks, 256>>>(out, rstep, nwin, nrows);
            } else {
                if (W == 8) k_store<8, false><<<blocks, 256>>>(out, rstep, nwin, nrows);
                else k_store<16, false><<<blocks, 256>>>(out, rstep, nwin, nrows);
            }
        };
        go();
        (void)hipEventRecord(e0);
        for (int r = 0; r < 10; ++r) go();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        double b = (double)waves * 64 * nrows * W;
        printf("nt=%d W=%d rows/wave=%d: %d waves, %.1f us  %.0f GB/s\n", (int)nt, W, nrows, waves, ms * 100, b / (ms / 10) / 1e6);
    }
    return 0;
}
