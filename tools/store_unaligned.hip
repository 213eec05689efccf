// Microbenchmark: the voting_for_hypothesis byte mask written with 8-byte
// stores at each row's own (unaligned) offset: wave = (keypoint v, 512-pixel
// window, 64 consecutive hypotheses); vs the class-aligned pattern.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef unsigned long long u64a1 __attribute__((aligned(1)));

__global__ void k_unaligned(uint8_t *out, int tn, int vn, int hn, int nwin, int rows_per_wave) {
    const int wave = blockIdx.x * 4 + threadIdx.x / 64, lane = threadIdx.x & 63;
    const int hgroups = hn / rows_per_wave;
    const int nitems = vn * nwin * hgroups;
    if (wave >= nitems) return;
    const int hg = wave % hgroups, rest = wave / hgroups;
    const int w = rest % nwin, v = rest / nwin;
    const int t = 512 * w + 8 * lane;
    if (t + 8 > tn) return;   // (the tail would use byte stores)
    for (int i = 0; i < rows_per_wave; ++i) {
        const int h = hg * rows_per_wave + i;
        const int64_t R = ((int64_t)h * vn + v) * tn;
        *(u64a1 *)(out + R + t) = 0x0101010101010101ull * (i & 1);
    }
}

int main() {
    const int tn = 29861, vn = 9, hn = 512;
    uint8_t *out;
    if (hipMalloc(&out, (size_t)hn * vn * tn + 4096) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int nwin = (tn + 511) / 512;
    for (int rpw : {64, 32, 16}) {
        const int waves = vn * nwin * (hn / rpw), blocks = (waves + 3) / 4;
        k_unaligned<<<blocks, 256>>>(out, tn, vn, hn, nwin, rpw);
        (void)hipEventRecord(e0);
        for (int r = 0; r < 10; ++r) k_unaligned<<<blocks, 256>>>(out, tn, vn, hn, nwin, rpw);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double b = (double)hn * vn * tn;
        printf("unaligned rows/wave=%d: %d waves, %.1f us  %.0f GB/s\n", rpw, waves, ms * 100, b / (ms / 10) / 1e6);
    }
    return 0;
}
