// Throughput of single VALU instructions on gfx950 (wave64): 8 independent
// chains per wave, 1 or 4 waves per SIMD.  Cycles per instruction per SIMD at
// the measured kernel duration and an assumed 2.4 GHz clock.
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_rates tools/valu_rates.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define OP2(name, str)                                                                      \
    __global__ __launch_bounds__(256) void name(float *out, int iters, float a, float b) {  \
        float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, \
              x7 = x0 + 7;                                                                  \
        for (int i = 0; i < iters; ++i) {                                                   \
            _Pragma("unroll") for (int k = 0; k < 8; ++k) {                                 \
                asm volatile(str : "+v"(x0) : "v"(a), "v"(b));                              \
                asm volatile(str : "+v"(x1) : "v"(a), "v"(b));                              \
                asm volatile(str : "+v"(x2) : "v"(a), "v"(b));                              \
                asm volatile(str : "+v"(x3) : "v"(a), "v"(b));                              \
                asm volatile(str : "+v"(x4) : "v"(a), "v"(b));                              \
                asm volatile(str : "+v"(x5) : "v"(a), "v"(b));                              \
                asm volatile(str : "+v"(x6) : "v"(a), "v"(b));                              \
                asm volatile(str : "+v"(x7) : "v"(a), "v"(b));                              \
            }                                                                               \
        }                                                                                   \
        out[blockIdx.x * 256 + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;       \
    }

OP2(k_fma, "v_fma_f32 %0, %0, %1, %2")
OP2(k_add, "v_add_f32 %0, %0, %1")
OP2(k_mul, "v_mul_f32 %0, %0, %1")
OP2(k_min, "v_min_f32 %0, %0, %1")
OP2(k_min3, "v_min3_f32 %0, %0, %1, %2")
OP2(k_minimum3, "v_minimum3_f32 %0, %0, %1, %2")
OP2(k_minimum3abs, "v_minimum3_f32 %0, %0, |%1|, |%2|")
OP2(k_perm, "v_perm_b32 %0, %0, %1, %2")
OP2(k_sad, "v_sad_u8 %0, %1, %2, %0")
OP2(k_or, "v_or_b32 %0, %0, %1")
OP2(k_or3, "v_or3_b32 %0, %0, %1, %2")
OP2(k_addu, "v_add_u32 %0, %0, %1")
OP2(k_lshr, "v_lshrrev_b32 %0, %1, %0")
OP2(k_bfe, "v_bfe_u32 %0, %0, %1, %2")
OP2(k_med3, "v_med3_f32 %0, %0, %1, %2")
OP2(k_cnd, "v_cndmask_b32 %0, %0, %1, vcc")
OP2(k_and_or, "v_and_or_b32 %0, %0, %1, %2")
OP2(k_xad, "v_xad_u32 %0, %0, %1, %2")
OP2(k_maxi, "v_max_i32 %0, %0, %1")
OP2(k_cvtf16, "v_cvt_pk_f16_f32 %0, %0, %1")
OP2(k_mov, "v_mov_b32 %0, %1")

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float *out;
    hipMalloc(&out, (size_t)cus * 8 * 256 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 4000;
    struct K { const char *n; void (*f)(float *, int, float, float); };
    K ks[] = {{"v_fma_f32", k_fma}, {"v_add_f32", k_add}, {"v_mul_f32", k_mul}, {"v_min_f32", k_min},
              {"v_min3_f32", k_min3}, {"v_minimum3_f32", k_minimum3}, {"v_minimum3_f32 |abs|", k_minimum3abs},
              {"v_perm_b32", k_perm}, {"v_sad_u8", k_sad}, {"v_or_b32", k_or}, {"v_or3_b32", k_or3},
              {"v_add_u32", k_addu}, {"v_lshrrev_b32", k_lshr}, {"v_bfe_u32", k_bfe}, {"v_med3_f32", k_med3},
              {"v_cndmask_b32", k_cnd}, {"v_and_or_b32", k_and_or}, {"v_xad_u32", k_xad}, {"v_max_i32", k_maxi},
              {"v_cvt_pk_f16_f32", k_cvtf16}, {"v_mov_b32", k_mov}};
    for (auto &k : ks) {
        for (int wps : {1, 4}) {
            hipLaunchKernelGGL(k.f, dim3(cus * wps), dim3(256), 0, 0, out, 10, 1.0001f, 0.5f);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k.f, dim3(cus * wps), dim3(256), 0, 0, out, iters, 1.0001f, 0.5f);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double ops_per_simd = (double)wps * iters * 64;
            printf("%-24s %d waves/SIMD: %.2f cyc per instruction per SIMD\n", k.n, wps, ms * 1e-3 * 2.4e9 / ops_per_simd);
        }
    }
    return 0;
}
