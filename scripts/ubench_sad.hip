// Issue-rate microbenchmark of the SAD instructions on gfx950 (MI355X):
// v_qsad_pk_u16_u8, v_sad_u8 and v_add_u32 (reference), 8 independent chains
// per lane, every CU fully occupied. Prints wave-instructions per clock per CU
// and absdiff/s for the whole chip (scripts/gpu_ubench.sh; DESIGN.md roofline).
#include <hip/hip_runtime.h>
#include <stdio.h>

#define ITERS 4096

__global__ void __launch_bounds__(256) k_qsad(unsigned long long *out, uint32_t seed) {
    unsigned long long a[8];
    uint32_t s = seed ^ threadIdx.x;
    unsigned long long r = ((unsigned long long)(s * 2654435761u) << 32) | (s * 40503u);
    for (int k = 0; k < 8; k++) a[k] = k;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) a[k] = __builtin_amdgcn_qsad_pk_u16_u8(r, s + k, a[k]);
    }
    unsigned long long t = 0;
    for (int k = 0; k < 8; k++) t ^= a[k];
    if (t == 0x123456789ull) out[0] = t;
}

__global__ void __launch_bounds__(256) k_sad(unsigned long long *out, uint32_t seed) {
    uint32_t a[8];
    uint32_t s = seed ^ threadIdx.x, r = s * 2654435761u;
    for (int k = 0; k < 8; k++) a[k] = k;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) a[k] = __builtin_amdgcn_sad_u8(r, s + k, a[k]);
    }
    uint32_t t = 0;
    for (int k = 0; k < 8; k++) t ^= a[k];
    if (t == 0x12345678u) out[0] = t;
}

__global__ void __launch_bounds__(256) k_add(unsigned long long *out, uint32_t seed) {
    uint32_t a[8];
    uint32_t s = seed ^ threadIdx.x;
    for (int k = 0; k < 8; k++) a[k] = k * s;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) a[k] = a[k] + (s ^ k);
    }
    uint32_t t = 0;
    for (int k = 0; k < 8; k++) t ^= a[k];
    if (t == 0x12345678u) out[0] = t;
}

template <typename K>
static double run(K kern, unsigned long long *d, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, 1u);
    hipEventRecord(a, 0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, (uint32_t)r);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / 5;
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const double clk = p.clockRate * 1e3; // Hz
    unsigned long long *d;
    hipMalloc(&d, 64);
    const int blocks = cus * 8; // 32 waves per CU
    const double waves = blocks * 4.0, instr = waves * ITERS * 8.0;
    struct {
        const char *name;
        double ms;
        int absdiff;
    } r[3] = {{"v_qsad_pk_u16_u8", run(k_qsad, d, blocks), 16},
              {"v_sad_u8", run(k_sad, d, blocks), 4},
              {"v_add_u32", run(k_add, d, blocks), 0}};
    printf("{\"cus\": %d, \"clock_mhz\": %.0f", cus, clk / 1e6);
    for (auto &x : r) {
        const double per_cu_clk = instr / (x.ms * 1e-3) / cus / clk;
        printf(", \"%s\": {\"ms\": %.4f, \"wave_instr_per_clk_per_cu\": %.3f, \"T_absdiff_s\": %.1f}", x.name, x.ms,
               per_cu_clk, instr * 64.0 * x.absdiff / (x.ms * 1e-3) / 1e12);
    }
    printf("}\n");
    hipFree(d);
    return 0;
}
