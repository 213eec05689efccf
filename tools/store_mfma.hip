// Microbenchmark: HBM write rate of the voting_for_hypothesis byte mask
// (512 hyp x 9 kp rows of 29,861 bytes, rows at any byte) under the store
// patterns a matrix-core vote kernel could use:
//   P1: a store = 64 lanes x 8 B of one row (512 B), a wave loops over rows
//       (the current k_vote_bytes pattern, also what an LDS transpose gives)
//   P2: a store = 32 rows x 16 B (the 32x32 MFMA output: lane = hypothesis
//       column, lane halves = 8 + 8 pixels), a wave loops over 16-pixel batches
//   P3: P2 through an LDS transpose (32 rows x 512 B tile), then P1 stores
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

constexpr int TN = 29861, VN = 9, HN = 512, NWIN = (TN + 511) / 512;
typedef uint64_t u64a1 __attribute__((aligned(1)));

__global__ __launch_bounds__(256) void k_p1(uint8_t *out) {
    const int wave = blockIdx.x * 4 + threadIdx.x / 64, lane = threadIdx.x & 63;
    const int items = VN * NWIN * (HN / 64);
    if (wave >= items) return;
    const int g = wave % (HN / 64), r = wave / (HN / 64), v = r % VN, w = r / VN;
    const int t = w * 512 + lane * 8;
    for (int i = 0; i < 64; ++i) {
        const int h = g * 64 + i;
        uint8_t *p = out + ((int64_t)h * VN + v) * TN + t;
        if (t + 8 <= TN) *(u64a1 *)p = 0x0101010101010101ull * (uint64_t)(i & 1);
    }
}

__global__ __launch_bounds__(256) void k_p2(uint8_t *out) {
    const int wave = blockIdx.x * 4 + threadIdx.x / 64, lane = threadIdx.x & 63;
    const int items = VN * NWIN * (HN / 64);
    if (wave >= items) return;
    const int g = wave % (HN / 64), r = wave / (HN / 64), v = r % VN, w = r / VN;
    const int col = lane & 31, half = lane >> 5;
    for (int s = 0; s < 2; ++s) {
        const int h = g * 64 + s * 32 + col;
        uint8_t *p = out + ((int64_t)h * VN + v) * TN + w * 512 + 8 * half;
        for (int b = 0; b < 32; ++b) {
            const int t = w * 512 + 16 * b + 8 * half;
            if (t + 8 <= TN) *(u64a1 *)(p + 16 * b) = 0x0101010101010101ull * (uint64_t)(b & 1);
        }
    }
}

__global__ __launch_bounds__(256) void k_p3(uint8_t *out) {
    __shared__ uint64_t tile[4][32 * 65];
    const int wave = blockIdx.x * 4 + threadIdx.x / 64, lane = threadIdx.x & 63, wid = threadIdx.x / 64;
    const int items = VN * NWIN * (HN / 64);
    if (wave >= items) return;
    const int g = wave % (HN / 64), r = wave / (HN / 64), v = r % VN, w = r / VN;
    const int col = lane & 31, half = lane >> 5;
    uint64_t *T = tile[wid];
    for (int s = 0; s < 2; ++s) {
        for (int b = 0; b < 32; ++b) T[col * 65 + 2 * b + half] = 0x0101010101010101ull * (uint64_t)(b & 1);
        __builtin_amdgcn_wave_barrier();
        const int t = w * 512 + lane * 8;
        for (int i = 0; i < 32; ++i) {
            const int h = g * 64 + s * 32 + i;
            uint8_t *p = out + ((int64_t)h * VN + v) * TN + t;
            const uint64_t x = T[i * 65 + lane];
            if (t + 8 <= TN) *(u64a1 *)p = x;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

int main() {
    uint8_t *out;
    const size_t n = (size_t)HN * VN * TN;
    hipMalloc(&out, n);
    const int items = VN * NWIN * (HN / 64), grid = (items + 3) / 4;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int k = 0; k < 4; ++k) {
        for (int rep = 0; rep < 3; ++rep) {
            const int R = 50;
            hipEventRecord(a);
            for (int i = 0; i < R; ++i) {
                if (k == 0) k_p1<<<grid, 256>>>(out);
                else if (k == 1) k_p2<<<grid, 256>>>(out);
                else if (k == 2) k_p3<<<grid, 256>>>(out);
                else hipMemsetAsync(out, 1, n);
            }
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            const char *nm[] = {"P1 row x 512B", "P2 32 rows x 16B", "P3 LDS transpose", "memset"};
            printf("%-18s %7.2f us  %6.0f GB/s\n", nm[k], ms * 1e3 / R, n / (ms * 1e-3 / R) / 1e9);
        }
    }
    return 0;
}
