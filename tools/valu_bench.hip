// Microbenchmark: issue rate of v_fma_f32 vs v_pk_fma_f32 (wave64) on gfx950.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ __launch_bounds__(256) void k_fma(float *out, int iters, float a, float b) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x0) : "v"(a), "v"(b));
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x1) : "v"(a), "v"(b));
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x2) : "v"(a), "v"(b));
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x3) : "v"(a), "v"(b));
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x4) : "v"(a), "v"(b));
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x5) : "v"(a), "v"(b));
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x6) : "v"(a), "v"(b));
            asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x7) : "v"(a), "v"(b));
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

typedef float f2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_pkfma(float *out, int iters, float a, float b) {
    f2 x0 = {(float)threadIdx.x, 1.f}, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6,
       x7 = x0 + 7;
    f2 A = {a, a}, B = {b, b};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x0) : "v"(A), "v"(B));
            asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x1) : "v"(A), "v"(B));
            asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x2) : "v"(A), "v"(B));
            asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x3) : "v"(A), "v"(B));
            asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x4) : "v"(A), "v"(B));
            asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x5) : "v"(A), "v"(B));
            asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x6) : "v"(A), "v"(B));
            asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x7) : "v"(A), "v"(B));
        }
    }
    f2 s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
    out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y;
}

// v_cmp + v_addc (count idiom) mixed with fma
__global__ __launch_bounds__(256) void k_cmpcnt(float *out, int iters, float a, float b) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
    int c = 0;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            x0 = fmaf(x0, a, b); x1 = fmaf(x1, a, b); x2 = fmaf(x2, a, b); x3 = fmaf(x3, a, b);
            c += x0 > 0.5f; c += x1 > 0.5f; c += x2 > 0.5f; c += x3 > 0.5f;
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = x0 + x1 + x2 + x3 + c;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float *out;
    hipMalloc(&out, 1 << 26);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 2000;
    for (int wps = 1; wps <= 8; wps *= 2) {   // waves per SIMD
        int blocks = cus * wps;            // 256 threads = 4 waves = 1 per SIMD
        for (int kind = 0; kind < 3; ++kind) {
            auto launch = [&]() {
                if (kind == 0) k_fma<<<blocks, 256>>>(out, iters, 0.999f, 0.001f);
                else if (kind == 1) k_pkfma<<<blocks, 256>>>(out, iters, 0.999f, 0.001f);
                else k_cmpcnt<<<blocks, 256>>>(out, iters, 0.999f, 0.001f);
            };
            launch();
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            double instr = (double)blocks * 4 * iters * (kind == 2 ? 16 * 8 : 64);   // wave-instructions
            double per_simd = instr / (cus * 4.0);
            double cyc = ms * 1e-3 * 2.4e9 / per_simd;
            double flops = (double)blocks * 256 * iters * 64 * 2 * (kind == 1 ? 2 : 1);
            printf("waves/SIMD %d %-7s %8.3f ms  %.2f cycles per wave-instr per SIMD  %.1f TFLOP/s\n", wps,
                   kind == 0 ? "fma" : kind == 1 ? "pk_fma" : "cmpcnt", ms, cyc, kind == 2 ? 0.0 : flops / ms / 1e9);
        }
    }
    return 0;
}
