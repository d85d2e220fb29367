// Microbenchmark: the cost of a hand-rolled grid-wide dependency wait on
// MI355X (the mechanism a pass-pipelined persistent kernel would use, DESIGN
// 8 item 1).  A grid of G workgroups x 256 threads, all resident, does K
// rounds of: (optionally) store 32 KiB per workgroup, wave stores done,
// workgroup barrier, thread 0 adds 1 to a device counter with an agent-scope
// release, spins (bounded) on an agent-scope acquire load until the counter
// reaches the round's target, workgroup barrier.  RELAXED_POLL (default):
// relaxed polling loads and one acquire fence after the wait; 0: every
// polling load an acquire (a cache invalidate per poll).  Reported: us per round,
// against K rounds of the same work without the wait.
#include <hip/hip_runtime.h>
#include <cstdio>
#ifndef RELAXED_POLL
#define RELAXED_POLL 1  // poll with relaxed loads, one acquire fence after the wait
#endif

template <bool WAIT, bool STORE>
__global__ void __launch_bounds__(256) sync_k(unsigned* cnt, uint4* buf, int rounds, unsigned nwg) {
    uint4 v = make_uint4(threadIdx.x, blockIdx.x, 1, 2);
    for (int r = 0; r < rounds; r++) {
        if (STORE) {
            uint4* p = buf + (size_t)blockIdx.x * 2048;  // 32 KiB per workgroup
#pragma unroll
            for (int i = 0; i < 8; i++) p[threadIdx.x + 256 * i] = v;
            v.x += 1;
        }
        if (WAIT) {
            __builtin_amdgcn_s_waitcnt(0);
            __syncthreads();
            if (threadIdx.x == 0) {
                __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned target = (unsigned)(r + 1) * nwg;
                for (unsigned i = 0; i < (1u << 22); i++) {
                    if (__hip_atomic_load(cnt, RELAXED_POLL ? __ATOMIC_RELAXED : __ATOMIC_ACQUIRE,
                                          __HIP_MEMORY_SCOPE_AGENT) >= target)
                        break;
                    __builtin_amdgcn_s_sleep(1);
                }
                if (RELAXED_POLL) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            }
            __syncthreads();
        }
    }
}

static float run(void (*k)(unsigned*, uint4*, int, unsigned), unsigned nwg, int rounds, unsigned* cnt, uint4* buf) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
        hipMemset(cnt, 0, 4);
        hipEventRecord(a);
        hipLaunchKernelGGL(k, dim3(nwg), dim3(256), 0, 0, cnt, buf, rounds, nwg);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    return best * 1e3f;
}

int main() {
    unsigned* cnt;
    uint4* buf;
    hipMalloc(&cnt, 256);
    hipMalloc(&buf, (size_t)1024 * 32768);
    for (unsigned nwg : {256u, 512u, 1024u}) {
        const int R = 50;
        const float w0 = run(sync_k<false, false>, nwg, R, cnt, buf), w1 = run(sync_k<true, false>, nwg, R, cnt, buf);
        const float s0 = run(sync_k<false, true>, nwg, R, cnt, buf), s1 = run(sync_k<true, true>, nwg, R, cnt, buf);
        printf("workgroups %4u: wait-only %.2f us per round (%.1f / %.1f us for %d rounds); with 32 KiB stores per "
               "workgroup %.2f us per round (%.1f / %.1f us)\n",
               nwg, (w1 - w0) / R, w0, w1, R, (s1 - s0) / R, s0, s1);
    }
    return 0;
}
