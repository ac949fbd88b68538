// Diagnostic hooks of k_hme (NOT part of the product library).
//
// scripts/build_diag_lib.sh compiles svtme_stages.hip with
// `-include csrc/diag/svtme_diag.h` and one of the defines below into a
// separate libsvtme_<name>.so; the product build never includes this file, so
// its HME_STAMP / HME_STOP hooks are empty there.
//
//   -DSVTME_STAMPS        thread 0 of every k_hme workgroup records the shader
//                         clock at each phase boundary (scripts/hme_stamps.py)
//   -DSVTME_STOP_AFTER=K  k_hme ends after phase K (scripts/gpu_phase_cost.sh)
//   -DSVTME_CLOCKBINS     shader cycles / real-time ticks per workgroup binned by
//                         start time: the clock over time (scripts/clock_probe.py)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifdef SVTME_STAMPS
__device__ unsigned long long g_hme_stamps[1 << 17][32];
// slots 0-7 shader clock per phase; 8 / 9 the 100 MHz real-time clock at the
// first / latest stamp; 10 XCC_ID, 11 HW_ID (CU, SE) register values; 12-15
// HW_ID of waves 0-3; 16 shader clock after the final search centre (HME_STOP(55))
#define HME_STAMP(k)                                                                                                   \
    do {                                                                                                               \
        if (threadIdx.x == 0 && blockIdx.x < (1u << 17)) {                                                             \
            g_hme_stamps[blockIdx.x][k] = __builtin_readcyclecounter();                                                \
            g_hme_stamps[blockIdx.x][(k) == 0 ? 8 : 9] = __builtin_amdgcn_s_memrealtime();                             \
            if ((k) == 0) {                                                                                            \
                g_hme_stamps[blockIdx.x][10] = (unsigned)__builtin_amdgcn_s_getreg(20 | (31 << 11));                   \
                g_hme_stamps[blockIdx.x][11] = (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));                    \
            }                                                                                                          \
        }                                                                                                              \
        if ((k) == 0 && (threadIdx.x & 63) == 0 && blockIdx.x < (1u << 17))                                            \
            g_hme_stamps[blockIdx.x][12 + (threadIdx.x >> 6)] = (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));   \
    } while (0)
#define HME_STOP(k)                                                                                                    \
    do {                                                                                                               \
        if ((k) == 55 && threadIdx.x == 0 && blockIdx.x < (1u << 17))                                                  \
            g_hme_stamps[blockIdx.x][16] = __builtin_readcyclecounter();                                               \
    } while (0)
// stage E's sub-phases (stage_c_tail): 17 after me_prune_ref, 18 after the records, 19 after the image zeroing,
// 20 after the candidate arrays (finish_sb's barrier), 21 at the end of wave 0's SB results
// 22 / 23 in fp_slot: after the search area (and its probe), after the search
// HME_WAVE(k): lane 0 of every wavefront w stamps slot 24 + 4 k + w (k 0: its phase-0 work done,
// k 1: its full-pel records done), before the barrier that ends the phase
#define HME_WAVE(k)                                                                                                    \
    do {                                                                                                               \
        if ((threadIdx.x & 63) == 0 && blockIdx.x < (1u << 17))                                                        \
            g_hme_stamps[blockIdx.x][24 + 4 * (k) + (threadIdx.x >> 6)] = __builtin_readcyclecounter();                 \
    } while (0)
#define HME_SUB(k)                                                                                                     \
    do {                                                                                                               \
        if (threadIdx.x == 0 && blockIdx.x < (1u << 17))                                                               \
            g_hme_stamps[blockIdx.x][k] = __builtin_readcyclecounter();                                                \
    } while (0)
extern "C" int svtme_debug_hme_stamps(unsigned long long *out, uint32_t nblocks) {
    if (nblocks > (1u << 17))
        nblocks = 1u << 17;
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_hme_stamps), (size_t)nblocks * 32 * sizeof(unsigned long long));
}
#elif defined(SVTME_STOP_AFTER)
#define HME_STAMP(k)                                                                                                   \
    do {                                                                                                               \
        if ((k) == SVTME_STOP_AFTER)                                                                                   \
            return;                                                                                                    \
    } while (0)
// extra stop points (no stamp slot)
#define HME_STOP(k) HME_STAMP(k)
#elif defined(SVTME_CLOCKBINS)
// thread 0 of every k_hme workgroup adds its shader cycles (s_memtime) and its
// 100 MHz real-time ticks (s_memrealtime) from start to end into the bin of its
// start time (2^13 ticks = 81.92 us per bin, 4096 bins = 335 ms before wrapping):
// cycles / ticks x 100 MHz is the clock the workgroups ran at in that bin
__device__ unsigned long long g_clock_bins[4096][3];
__device__ unsigned long long g_clock_start[1 << 17][2]; // per workgroup: cycles, ticks at phase 0
#define HME_STAMP(k)                                                                                                   \
    do {                                                                                                               \
        if (threadIdx.x == 0) {                                                                                        \
            unsigned long long *st = g_clock_start[blockIdx.x & ((1u << 17) - 1)];                                     \
            if ((k) == 0) {                                                                                            \
                st[0] = __builtin_readcyclecounter();                                                                  \
                st[1] = __builtin_amdgcn_s_memrealtime();                                                              \
            } else if ((k) == 7) {                                                                                     \
                const unsigned long long c1 = __builtin_readcyclecounter(), r1 = __builtin_amdgcn_s_memrealtime();     \
                const unsigned long long c0 = st[0], r0 = st[1];                                                       \
                const int bin = (int)((r0 >> 13) & 4095);                                                              \
                atomicAdd(&g_clock_bins[bin][0], c1 - c0);                                                             \
                atomicAdd(&g_clock_bins[bin][1], r1 - r0);                                                             \
                atomicAdd(&g_clock_bins[bin][2], 1ull);                                                                \
            }                                                                                                          \
        }                                                                                                              \
    } while (0)
extern "C" int svtme_debug_clock_bins(unsigned long long *out) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_clock_bins), sizeof(g_clock_bins));
}
#endif
