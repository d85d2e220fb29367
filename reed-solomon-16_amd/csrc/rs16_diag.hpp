// rs16_diag.hpp -- diagnostics hooks of the kernels (not product code).
//
// Phase timelines for scripts/stamps.py: a library built with
// -DRS16_STAMPS=1 (never the shipped one) makes thread 0 of every workgroup
// store s_memtime at phase i to stamps[block * 16 + i] of the launch
// arguments' `stamps` buffer (rs16_engine_set_stamps); slot 14 / 15 hold
// s_memrealtime at the start / end (for the clock), 12 / 13 the HW_ID and
// XCC_ID registers.  In every other build the hooks are empty macros, so the
// shipped kernels contain no trace of them.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef RS16_STAMPS
#define RS16_STAMPS 0
#endif

#if RS16_STAMPS
namespace rs16 {
template <class Args>
__device__ __forceinline__ void diag_stamp(const Args& a, int i) {
    if (a.stamps && threadIdx.x == 0) {
        uint64_t* p = a.stamps + blockIdx.x * 16;
        p[i] = __builtin_amdgcn_s_memtime();
        if (i == 0) {
            p[14] = __builtin_amdgcn_s_memrealtime();
            p[12] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
            p[13] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
        }
        if (i == 11) p[15] = __builtin_amdgcn_s_memrealtime();
    }
}
}  // namespace rs16
// phase i reached
#define RS16_STAMP(args, i) ::rs16::diag_stamp((args), (i))
// the workgroup's stores have completed (phase 11)
#define RS16_STAMP_END(args)                \
    do {                                    \
        __builtin_amdgcn_s_waitcnt(0);      \
        ::rs16::diag_stamp((args), 11);     \
    } while (0)
#else
#define RS16_STAMP(args, i) ((void)0)
#define RS16_STAMP_END(args) ((void)0)
#endif
