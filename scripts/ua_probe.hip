// Probe: 16-byte buffer / global loads at byte (unaligned) offsets return the
// bytes at those offsets (ROCm compute queues run in unaligned mode on gfx9+).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef uint32_t u4a1 __attribute__((ext_vector_type(4), aligned(1)));
__global__ void k(const uint8_t *a, uint32_t *o) {
    const int t = threadIdx.x; // byte offset 0..63
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)a, 0, (int)0xFFFFFFFF, 0x00020000);
    const u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, t, 3, 0); // byte offset t + 3
    const u4a1 g = *(const __attribute__((address_space(1))) u4a1 *)(uintptr_t)(a + t + 5);
    o[t * 8 + 0] = v[0], o[t * 8 + 1] = v[1], o[t * 8 + 2] = v[2], o[t * 8 + 3] = v[3];
    o[t * 8 + 4] = g[0], o[t * 8 + 5] = g[1], o[t * 8 + 6] = g[2], o[t * 8 + 7] = g[3];
}
int main() {
    uint8_t h[256];
    for (int i = 0; i < 256; i++) h[i] = (uint8_t)(i * 7 + 1);
    uint8_t *d;
    uint32_t *o, ho[64 * 8];
    hipMalloc(&d, 256);
    hipMalloc(&o, sizeof(ho));
    hipMemcpy(d, h, 256, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o);
    if (hipMemcpy(ho, o, sizeof(ho), hipMemcpyDeviceToHost) != hipSuccess) { printf("copy failed\n"); return 2; }
    int bad = 0;
    for (int t = 0; t < 64; t++)
        for (int w = 0; w < 4; w++) {
            uint32_t eb = 0, eg = 0;
            for (int b = 0; b < 4; b++) {
                eb |= (uint32_t)h[t + 3 + 4 * w + b] << (8 * b);
                eg |= (uint32_t)h[t + 5 + 4 * w + b] << (8 * b);
            }
            bad += ho[t * 8 + w] != eb;
            bad += ho[t * 8 + 4 + w] != eg;
        }
    printf("unaligned loads: %s (%d mismatches)\n", bad ? "WRONG" : "ok", bad);
    return bad ? 1 : 0;
}
